#!/bin/bash
# Round-4 probe: chainNet -rescore teardown on C5 -- the nets' arenas freed on
# 16 threads with MADV_DONTNEED first and the chain arrays dropped (default),
# or munmap on 8 threads (round 3).
set -o pipefail
tag=${1:-r04free}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
d=/tmp/c5
P=genomealignmenttools_amd
timeout -k 10 200 $P/libexec/gac_synth c5 $d -seed=1234 -chains=5000000 -sizesDir=$P/data -threads=16 || exit $?
run() {
  local name=$1; shift
  rm -f $d/o.t.net $d/o.q.net
  s=$(date +%s.%N)
  env "$@" GAC_TIMING=1 timeout -k 10 120 $P/bin/chainNet $d/in.chain $d/t.sizes $d/q.sizes $d/o.t.net $d/o.q.net \
      -rescore -tNibDir=$d/t.2bit -qNibDir=$d/q.2bit -linearGap=loose 2> $out/$name.err || return $?
  e=$(date +%s.%N)
  python3 -c "print('$name wall', round($e - $s, 3))" >> $out/times.txt
}
for i in 1 2 3; do
  run default_$i GAC_X=1 || exit $?
  run nomadv_$i GAC_FREE_MADV=0 GAC_FREE_THREADS=8 || exit $?
done
sha256sum $d/o.t.net $d/o.q.net >> $out/times.txt
echo ok
