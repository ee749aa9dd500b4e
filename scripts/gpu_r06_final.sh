#!/bin/bash
# Round-6 closing evidence, in two calls (the box's 20-minute limit):
#   tests: the whole -m gpu suite and smoke()
#   bench: bench.py as the driver runs it, then rocprofv3 kernel stats over
#          the kernel legs (upload kernels included)
set -o pipefail
part=${1:-tests}
tag=${2:-r06final}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
(while sleep 50; do date +%T >> $out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
if [ "$part" = tests ]; then
    timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests \
        --durations=30 > $out/gpu_tests.txt 2>&1 || exit $?
    timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || exit $?
else
    timeout -k 10 600 python -u bench.py > $out/bench.json 2> $out/bench.err || exit $?
    cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof \
        -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --kernel-steps 10 --no-c2 \
        --no-cpu-baseline --no-pmc --no-c4 --no-c3 > $GRAFT_REPO_ROOT/$out/prof_bench.json \
        2> $GRAFT_REPO_ROOT/$out/prof_bench.err || exit $?
fi
echo ok
