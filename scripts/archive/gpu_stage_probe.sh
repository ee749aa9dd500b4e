#!/bin/bash
# Per-stage timings of bin/chainNet -rescore on C2 (GAC_TIMING=1: device
# open laps, genome upload, netting phases) under several environments.
# usage: bash scripts/archive/gpu_stage_probe.sh TAG
set -o pipefail
TAG=${1:-probe}; shift
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -c "
import sys; sys.path.insert(0, '.')
import bench
a = bench.parse(); print(bench.c2_files(a)[0])" --tmp /tmp > "$OUT/dir.txt" 2> "$OUT/gen.log" || exit 1
D=$(cat "$OUT/dir.txt")
run() { # name env...
  local name=$1; shift
  for i in 1 2 3; do
    local t0=$(date +%s%N)
    env GAC_TIMING=1 "$@" timeout -k 10 120 genomealignmenttools_amd/bin/chainNet $D/in.chain $D/t.sizes $D/q.sizes /tmp/o.t.net /tmp/o.q.net \
      -rescore -tNibDir=$D/t.2bit -qNibDir=$D/q.2bit -linearGap=loose -verbose=2 > "$OUT/$name.$i.log" 2>&1 || return 1
    local t1=$(date +%s%N)
    echo "$name run $i wall_ms $(( (t1 - t0) / 1000000 ))" >> "$OUT/wall.log"
  done
}
run base || exit 1
run nodefer HIP_ENABLE_DEFERRED_LOADING=0 || exit 1
run defer HIP_ENABLE_DEFERRED_LOADING=1 || exit 1
run hwq1 GPU_MAX_HW_QUEUES=1 || exit 1
run nullstream GAC_STREAM=null || exit 1
cat "$OUT/wall.log"
grep -h 'gac_open\]\|overlapped\|fill list' "$OUT"/*.3.log
