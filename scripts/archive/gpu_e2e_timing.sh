#!/bin/bash
# bin/chainNet -rescore on C2 with every timing lap (GAC_TIMING=1), 3 runs,
# wall clock per run; the last run's log is printed.
# usage: bash scripts/archive/gpu_e2e_timing.sh TAG [ENV=VAL ...]
set -o pipefail
TAG=${1:-e2e}; shift
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -c "
import sys; sys.path.insert(0, '.')
import bench
a = bench.parse(); print(bench.c2_files(a)[0])" --tmp /tmp > "$OUT/dir.txt" 2> "$OUT/gen.log" || exit 1
D=$(cat "$OUT/dir.txt")
for i in 1 2 3 4; do
  t0=$(date +%s%N)
  env GAC_TIMING=1 "$@" timeout -k 10 120 genomealignmenttools_amd/bin/chainNet $D/in.chain $D/t.sizes $D/q.sizes /tmp/o.t.net /tmp/o.q.net \
    -rescore -tNibDir=$D/t.2bit -qNibDir=$D/q.2bit -linearGap=loose -verbose=2 > "$OUT/run$i.log" 2>&1 || { echo "run $i failed"; tail "$OUT/run$i.log"; exit 1; }
  t1=$(date +%s%N)
  echo "run $i wall_ms $(( (t1 - t0) / 1000000 ))" | tee -a "$OUT/wall.log"
done
cat "$OUT/run4.log"
