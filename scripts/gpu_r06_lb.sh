#!/bin/bash
# Round 6: the single-pass fills planning (k_plan_lb) -- the scoring tests,
# then the bench's kernel legs with it (default) and without (GAC_PLAN_LB=0),
# then rocprofv3 kernel stats of the kernel legs with it.
set -o pipefail
out=gpurun_out/${1:-r06lb}
mkdir -p $out
export TMPDIR=/tmp
( while sleep 30; do date +%T >> $out/heartbeat.txt; done ) &
hb=$!
trap "kill $hb" EXIT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_scoring.py \
    > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
tail -3 $out/tests.txt
K="--steps 1 --warmup 0 --kernel-steps 20 --no-c2 --no-cpu-baseline --no-c4 --no-c3"
GAC_PLAN_LB=1 timeout -k 10 400 python -u bench.py $K --no-pmc > $out/bench_lb1.json 2> $out/bench_lb1.err || exit $?
GAC_PLAN_LB=0 timeout -k 10 400 python -u bench.py $K --no-pmc > $out/bench_lb0.json 2> $out/bench_lb0.err || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof \
    -o run -- python3 $GRAFT_REPO_ROOT/bench.py $K --no-pmc > $GRAFT_REPO_ROOT/$out/prof_bench.json \
    2> $GRAFT_REPO_ROOT/$out/prof_bench.err || exit $?
echo ok
