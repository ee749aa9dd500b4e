#!/bin/bash
# PMC counter passes for the bench's kernels (separate rocprofv3 runs, each
# with --kernel-trace only; never combined with sys/runtime traces).
# usage: bash scripts/archive/gpu_counters.sh TAG [bench args...]
set -o pipefail
TAG=${1:-ctr}; shift
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" \
           "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$OUT/pmc$i" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --steps 3 --warmup 1 "$@" > "$OUT/pmc$i.log" 2>&1
  rc=$?
  echo "pmc pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
