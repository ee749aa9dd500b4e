#!/bin/bash
# GPU-box check: parity tests, bench, rocprofv3 kernel stats.  Every GPU step
# has its own time limit and the chain stops at the first failure.
# usage: bash scripts/gpu_check.sh TAG [bench args...]
set -o pipefail
TAG=${1:-run}; shift
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
make -j16 all oracle > "$OUT/build.log" 2>&1 || { echo "build failed"; exit 1; }
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 900 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?
echo "pytest rc=$rc" >> "$OUT/tests.log"
tail -3 "$OUT/tests.log"
# 0 = pass, 1 = a test failed; anything else (abort, fault, time limit): stop here
[ $rc -le 1 ] || exit $rc
timeout -k 10 900 python bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --steps 10 --warmup 2 "$@" > "$GRAFT_REPO_ROOT/$OUT/prof.log" 2>&1
echo "prof rc=$?"
