#!/bin/bash
# Round 6: the kd-tree DP's inputs built on the device (gac_chain_dp_blocks):
# the axtChain GPU tests (every GAC_AXT_DP=gpu run takes the device build),
# then C4 at 50 M blocks with the hybrid's device share at several caps.
set -o pipefail
out=gpurun_out/${1:-r06dt}
mkdir -p $out
export TMPDIR=/tmp
( while sleep 30; do date +%T >> $out/heartbeat.txt; done ) &
hb=$!
trap "kill $hb" EXIT
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread \
    tests/test_gpu_configs.py tests/test_gpu_tools.py -k "axtchain or device_dp" > $out/tests.txt 2>&1
rc=$?
tail -5 $out/tests.txt
[ $rc -eq 0 ] || exit $rc
REPS=${REPS:-1} MODES=${MODES:-"host 50000 200000 us7_400000 dt0_200000"} bash scripts/gpu_r06_c4split.sh ${1:-r06dt}/split
