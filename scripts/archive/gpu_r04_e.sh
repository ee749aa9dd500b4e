#!/bin/bash
# Round-4: the full -m gpu suite and smoke on the flat upload kernels, then
# axtChain C4 (50 M blocks) with the applier thread (default) and without.
set -o pipefail
tag=${1:-r04e}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
(while sleep 50; do date +%T >> $out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests \
    --durations=25 > $out/gpu_tests.txt 2>&1 || exit $?
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || exit $?
d=/tmp/c4_50m
timeout -k 10 120 genomealignmenttools_amd/libexec/gac_synth c4 $d -blocks=50000000 -threads=16 || exit $?
for ap in 1 0; do
  rm -f $d/ours.chain
  s=$(date +%s.%N)
  GAC_DP_APPLY=$ap GAC_TIMING=1 timeout -k 10 300 genomealignmenttools_amd/bin/axtChain -linearGap=loose -verbose=2 -psl \
      $d/in.psl $d/t.2bit $d/q.2bit $d/ours.chain 2> $out/c4_apply$ap.err || exit $?
  e=$(date +%s.%N)
  python3 -c "print('apply $ap wall', $e - $s)" >> $out/c4_times.txt
  sha256sum $d/ours.chain >> $out/c4_times.txt
done
echo ok
