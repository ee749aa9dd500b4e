#!/bin/bash
# Round-4: axtChain-side change check -- the tool and config GPU tests, then
# C4 (50 M PSL blocks) twice with GAC_TIMING, output sha256.
set -o pipefail
tag=${1:-r04k}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
(while sleep 50; do date +%T >> $out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
P=genomealignmenttools_amd
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_tools.py tests/test_gpu_configs.py > $out/gpu_tests.txt 2>&1 || exit $?
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
