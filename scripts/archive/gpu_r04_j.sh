#!/bin/bash
# Round-4: C5 chainNet -rescore (3 runs) and C4 axtChain (2 runs) timings with
# GAC_TIMING on the box, output sha256 each.
set -o pipefail
tag=${1:-r04j}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
(while sleep 50; do date +%T >> $out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
P=genomealignmenttools_amd
d=/tmp/c5
timeout -k 10 200 $P/libexec/gac_synth c5 $d -seed=1234 -chains=5000000 -sizesDir=$P/data -threads=16 || exit $?
for i in 1 2 3; do
  rm -f $d/o.t.net $d/o.q.net
  s=$(date +%s.%N)
  GAC_TIMING=1 timeout -k 10 120 $P/bin/chainNet $d/in.chain $d/t.sizes $d/q.sizes $d/o.t.net $d/o.q.net \
      -rescore -tNibDir=$d/t.2bit -qNibDir=$d/q.2bit -linearGap=loose 2> $out/c5_net_$i.err || exit $?
  e=$(date +%s.%N)
  python3 -c "print('c5 run $i wall', round($e - $s, 3))" >> $out/times.txt
done
sha256sum $d/o.t.net $d/o.q.net >> $out/times.txt
rm -rf $d
c=/tmp/c4_50m
timeout -k 10 120 $P/libexec/gac_synth c4 $c -blocks=50000000 -threads=16 || exit $?
for i in 1 2; do
  rm -f $c/ours.chain
  s=$(date +%s.%N)
  GAC_TIMING=1 timeout -k 10 300 $P/bin/axtChain -linearGap=loose -verbose=2 -psl \
      $c/in.psl $c/t.2bit $c/q.2bit $c/ours.chain 2> $out/c4_$i.err || exit $?
  e=$(date +%s.%N)
  python3 -c "print('c4 run $i wall', round($e - $s, 3))" >> $out/times.txt
done
sha256sum $c/ours.chain >> $out/times.txt
echo ok
