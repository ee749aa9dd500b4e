#!/bin/bash
# Device kd-tree DP (GAC_AXT_DP=gpu, rows A13/A14): parity tests, then the
# C4-like axtChain timed with the DP on host threads and on the device, and a
# rocprofv3 kernel trace of the device run.
# usage: bash scripts/archive/gpu_dp_probe.sh TAG BLOCKS
set -o pipefail
TAG=${1:-dp}; BLOCKS=${2:-2000000}
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
make -j16 all oracle > "$OUT/build.log" 2>&1 || { echo "build failed"; exit 1; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_tools.py tests/test_gpu_configs.py -x -v -m gpu -k "axtchain" --timeout 600 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?
tail -3 "$OUT/tests.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/bench_tools.py axtchain --blocks $BLOCKS --dp host > "$OUT/host.json" 2> "$OUT/host.err" || { echo "host run failed"; tail -5 "$OUT/host.err"; exit 1; }
cat "$OUT/host.json"
timeout -k 10 900 python scripts/bench_tools.py axtchain --blocks $BLOCKS --dp gpu --no-ref > "$OUT/gpu.json" 2> "$OUT/gpu.err" || { echo "gpu run failed"; tail -5 "$OUT/gpu.err"; exit 1; }
cat "$OUT/gpu.json"
D=/tmp/c4_$BLOCKS
cmp "$D/ours.chain" "$D/ref.chain" && echo "device DP output identical to the reference"
cd /tmp
GAC_PROFILE_EXIT=1 GAC_AXT_DP=gpu timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run -- "$GRAFT_REPO_ROOT/genomealignmenttools_amd/libexec/axtChain" -linearGap=loose -verbose=0 -psl $D/in.psl $D/t.2bit $D/q.2bit /tmp/prof.chain > "$GRAFT_REPO_ROOT/$OUT/prof.log" 2>&1
echo "prof rc=$?"
cmp /tmp/prof.chain $D/ref.chain && echo "profiled run identical"
