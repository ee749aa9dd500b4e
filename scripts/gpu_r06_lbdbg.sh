#!/bin/bash
# k_plan_lb debug: the scoring tests with -s and the launch check's print,
# then the k_plan_lb A/B (scripts/gpu_r06_lb.sh)
set -o pipefail
out=gpurun_out/${1:-r06lbdbg}
mkdir -p $out
export TMPDIR=/tmp
GAC_DEBUG_LAUNCH=1 timeout -k 10 400 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread \
    tests/test_gpu_scoring.py > $out/tests_s.txt 2>&1 || { tail -30 $out/tests_s.txt; exit 1; }
grep -B3 "k_plan_lb\]" $out/tests_s.txt | head -40
bash scripts/gpu_r06_lb.sh r06lb
