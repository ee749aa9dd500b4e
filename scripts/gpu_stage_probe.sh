#!/bin/bash
# Per-stage timings of bin/chainNet -rescore on C2 (GAC_TIMING=1: device
# open laps, genome upload, netting phases), three runs.
# usage: bash scripts/gpu_stage_probe.sh TAG [extra env assignments...]
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
for i in 1 2 3; do
  env GAC_TIMING=1 "$@" timeout -k 10 120 genomealignmenttools_amd/bin/chainNet $D/in.chain $D/t.sizes $D/q.sizes /tmp/o.t.net /tmp/o.q.net \
    -rescore -tNibDir=$D/t.2bit -qNibDir=$D/q.2bit -linearGap=loose -verbose=2 > "$OUT/run$i.log" 2>&1 || exit 1
  /usr/bin/time -f "wall %e" timeout -k 10 120 genomealignmenttools_amd/bin/chainNet $D/in.chain $D/t.sizes $D/q.sizes /tmp/o.t.net /tmp/o.q.net \
    -rescore -tNibDir=$D/t.2bit -qNibDir=$D/q.2bit -linearGap=loose >> "$OUT/wall.log" 2>&1 || exit 1
done
cat "$OUT/run3.log"; cat "$OUT/wall.log"
