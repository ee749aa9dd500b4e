#!/bin/bash
# GPU parity tests, then end-to-end tool timings (scripts/archive/gpu_tool_bench.sh).
# usage: bash scripts/archive/gpu_tests_tools.sh TAG tool...
set -o pipefail
TAG=${1:-t}; shift
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1
rc=$?
tail -3 gpurun_out/$TAG/tests.log
[ $rc -eq 0 ] || exit $rc
bash scripts/archive/gpu_tool_bench.sh "$@"
