#!/bin/bash
# Round-4: C5 chainNet -rescore host stage breakdown (GAC_TIMING) on the box.
set -o pipefail
tag=${1:-r04net}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
(while sleep 50; do date +%T >> $out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
d=/tmp/c5
P=genomealignmenttools_amd
timeout -k 10 200 $P/libexec/gac_synth c5 $d -seed=1234 -chains=5000000 -sizesDir=$P/data -threads=16 || exit $?
for i in 1 2 3; do
  rm -f $d/o.t.net $d/o.q.net
  s=$(date +%s.%N)
  GAC_TIMING=1 timeout -k 10 120 $P/bin/chainNet $d/in.chain $d/t.sizes $d/q.sizes $d/o.t.net $d/o.q.net \
      -rescore -tNibDir=$d/t.2bit -qNibDir=$d/q.2bit -linearGap=loose 2> $out/c5_net_$i.err || exit $?
  e=$(date +%s.%N)
  python3 -c "print('run $i wall', $e - $s)" >> $out/c5_times.txt
done
sha256sum $d/o.t.net $d/o.q.net >> $out/c5_times.txt
echo ok
