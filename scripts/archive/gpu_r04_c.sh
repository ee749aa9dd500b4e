#!/bin/bash
# Round-4: axtChain C4 (50 M blocks) team-DP timings on the box: lag 32
# (default) and 16.
set -o pipefail
tag=${1:-r04c}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
(while sleep 50; do date +%T >> $out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
d=/tmp/c4_50m
timeout -k 10 120 genomealignmenttools_amd/libexec/gac_synth c4 $d -blocks=50000000 -threads=16 || exit $?
for lag in 32 16; do
  rm -f $d/ours.chain
  s=$(date +%s.%N)
  GAC_DP_LAG=$lag GAC_TIMING=1 timeout -k 10 300 genomealignmenttools_amd/bin/axtChain -linearGap=loose -verbose=2 -psl \
      $d/in.psl $d/t.2bit $d/q.2bit $d/ours.chain 2> $out/c4_lag$lag.err || exit $?
  e=$(date +%s.%N)
  python3 -c "print('lag $lag wall', $e - $s)" >> $out/c4_times.txt
  sha256sum $d/ours.chain >> $out/c4_times.txt
done
echo ok
