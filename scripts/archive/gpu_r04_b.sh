#!/bin/bash
# Round-4: the exact fast / team kd-tree DP on the box -- axtChain GPU tests
# (goldens, KATs, C4 shape, full-scale C4 sha) and C4 timings; the gather
# ceiling probe.
set -o pipefail
tag=${1:-r04b}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
(while sleep 50; do date +%T >> $out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 120 genomealignmenttools_amd/libexec/gac_gather_ceiling 2048 > $out/gather_ceiling.json 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -k "axtchain or c4" \
    tests/test_gpu_tools.py tests/test_gpu_configs.py --durations=10 > $out/gpu_tests.txt 2>&1 || exit $?
d=/tmp/c4_50m
timeout -k 10 120 genomealignmenttools_amd/libexec/gac_synth c4 $d -blocks=50000000 -threads=16 || exit $?
for i in 1 2; do
  rm -f $d/ours.chain
  s=$(date +%s.%N)
  GAC_TIMING=1 timeout -k 10 300 genomealignmenttools_amd/bin/axtChain -linearGap=loose -verbose=2 -psl \
      $d/in.psl $d/t.2bit $d/q.2bit $d/ours.chain 2> $out/c4_ours_$i.err || exit $?
  e=$(date +%s.%N)
  python3 -c "print('run $i wall', $e - $s)" >> $out/c4_times.txt
done
sha256sum $d/ours.chain >> $out/c4_times.txt
echo ok
