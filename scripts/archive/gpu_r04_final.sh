#!/bin/bash
# Round-4 bench evidence: bench.py as the driver runs it (defaults: C5
# headline with full-scale parity, C2 leg, kernel legs with in-run PMC
# traffic and the gather ceiling, C4 axtChain leg, cpu baseline); then
# rocprofv3 --kernel-trace --stats over a short kernel-leg run; then the
# N = 2 path rehearsed on this one-GPU box.  Each GPU step time-limited.
set -o pipefail
tag=${1:-r04final}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
(while sleep 50; do date +%T >> $out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err || exit $?
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof \
    -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --kernel-steps 10 --no-c2 \
    --no-cpu-baseline --no-pmc --no-c4 > $GRAFT_REPO_ROOT/$out/prof_bench.json \
    2> $GRAFT_REPO_ROOT/$out/prof_bench.err || exit $?
cd $GRAFT_REPO_ROOT
GAC_BENCH_ONE_GPU=1 GAC_THREADS=8 timeout -k 10 500 python bench.py --gpus 2 --steps 2 --warmup 1 \
    --no-kernel > $out/bench_n2.json 2> $out/bench_n2.err || exit $?
echo ok
