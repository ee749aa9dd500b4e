#!/bin/bash
# k_tile experiments on the kernel leg (rescore fills): each argument is
# "NAME:ENV=VAL,ENV=VAL:MAKEVARS" -- rebuild with MAKEVARS (e.g.
# HIPEXTRA=-DGAC_VARIANT=1) when given, then time the kernel leg with ENV set.
# usage: bash scripts/archive/gpu_tile_probe.sh TAG SPEC...
set -o pipefail
TAG=${1:-tile}; shift
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; envs=${rest%%:*}; mk=${rest#*:}
  [ "$mk" = "$rest" ] && mk=""
  if [ -n "$mk" ]; then
    make -B -j16 all $mk > "$OUT/build_$name.log" 2>&1 || { echo "build $name failed"; exit 1; }
  fi
  envcmd=$(echo "$envs" | tr ',' ' ')
  env $envcmd timeout -k 10 300 python bench.py --workload rescore --no-cpu-baseline --prof tile --kernel-steps 30 > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "bench $name failed"; tail -5 "$OUT/$name.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$name.json')); k=d['kernel']; r=d['roofline']; print('$name', 'step_us', round(k['ms_per_step']*1e3,1), 'tile_us', round(r['kernel_avg_ms']*1e3,2), 'frac', round(r['frac'],3))"
done
