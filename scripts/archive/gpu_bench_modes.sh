#!/bin/bash
# Bench under each event-timing mode (how much the HIP event markers cost).
# usage: bash scripts/archive/gpu_bench_modes.sh TAG [bench args...]
set -o pipefail
TAG=${1:-modes}; shift
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
make -j16 all oracle > "$OUT/build.log" 2>&1 || { echo "build failed"; exit 1; }
for m in none tile all; do
  timeout -k 10 600 python bench.py --no-cpu-baseline --prof $m "$@" > "$OUT/bench_$m.json" 2> "$OUT/bench_$m.err" || { echo "bench $m failed"; tail -5 "$OUT/bench_$m.err"; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/bench_$m.json')); print('$m', round(d['value'],1), round(d['ms_per_step']*1e3,1), {k: round(v*1e3,1) for k,v in d['kernel_ms_per_step'].items()})"
done
