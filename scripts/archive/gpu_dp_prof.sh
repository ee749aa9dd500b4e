#!/bin/bash
# The device kd-tree DP (GAC_AXT_DP=gpu) on the C4-like axtChain input:
# one timed run checked against the reference's output, then a rocprofv3
# kernel trace (k_dp / k_xover durations) of the same command.
# usage: bash scripts/archive/gpu_dp_prof.sh TAG BLOCKS
set -o pipefail
TAG=${1:-dpprof}; BLOCKS=${2:-2000000}
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python scripts/bench_tools.py axtchain --blocks $BLOCKS --dp gpu > "$OUT/gpu.json" 2> "$OUT/gpu.err" || { echo "gpu run failed"; tail -5 "$OUT/gpu.err"; exit 1; }
cat "$OUT/gpu.json"
D=/tmp/c4_$BLOCKS
cd /tmp
GAC_PROFILE_EXIT=1 GAC_AXT_DP=gpu timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run -- "$GRAFT_REPO_ROOT/genomealignmenttools_amd/libexec/axtChain" -linearGap=loose -verbose=0 -psl $D/in.psl $D/t.2bit $D/q.2bit /tmp/prof.chain > "$GRAFT_REPO_ROOT/$OUT/prof.log" 2>&1
echo "prof rc=$?"
cmp /tmp/prof.chain $D/ref.chain && echo "profiled run identical"
find "$GRAFT_REPO_ROOT/$OUT/prof" -name "*stats*" | head
