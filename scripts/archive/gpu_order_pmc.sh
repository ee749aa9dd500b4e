#!/bin/bash
# Kernel leg (rescore fills) under several range orders: per-kernel times and
# memory-side read requests / L2 hits of each kernel (one --pmc pass per
# counter group, --kernel-trace only).
# usage: bash scripts/archive/gpu_order_pmc.sh TAG "order1 order2 ..." [bench args...]
set -o pipefail
TAG=${1:-ordpmc}; shift
ORDERS=${1:-"net chain"}; shift
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for o in $ORDERS; do
  timeout -k 10 300 python bench.py --workload rescore --no-cpu-baseline --prof all --order $o "$@" > "$OUT/$o.json" 2> "$OUT/$o.err" || { echo "bench $o failed"; tail -5 "$OUT/$o.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$o.json')); k=d['kernel']; print('$o', round(k['value'],1), round(k['ms_per_step']*1e3,1), {a: round(b*1e3,1) for a,b in k['kernel_ms'].items()}, 'tile frac', round(d['roofline']['frac'],3))"
done
cd /tmp
for o in $ORDERS; do
  i=0
  for set in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$OUT/pmc_$o/pmc$i" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload rescore --no-cpu-baseline --order $o --kernel-steps 3 "$@" > "$OUT/pmc_${o}_$i.log" 2>&1
    rc=$?
    [ $rc -eq 0 ] || { echo "pmc $o $i rc=$rc"; exit $rc; }
  done
  python3 "$GRAFT_REPO_ROOT/scripts/pmc_summary.py" "$OUT/pmc_$o" > "$OUT/pmc_$o.json"
  python3 -c "
import json; d=json.load(open('$OUT/pmc_$o.json'))
for k,v in d.items():
    if 'hbm_read_bytes' in v: print('$o', k, 'MB', round(v['hbm_read_bytes']/1e6,1), 'hit', round(v.get('TCC_HIT_sum',0)/max(1,v.get('TCC_HIT_sum',0)+v.get('TCC_MISS_sum',0)),3))"
done
