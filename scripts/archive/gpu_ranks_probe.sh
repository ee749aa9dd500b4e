#!/bin/bash
# chainNet -rescore -nranks=N on the replicated-C2 input (bench.py's N>1
# workload), all ranks on this box's one GPU: wall time per step and the
# per-rank stage times.  GAC_THREADS per rank = 16/N (the box's CPU share).
# usage: bash scripts/archive/gpu_ranks_probe.sh TAG "1 2 4"
set -o pipefail
TAG=${1:-ranks}; NS=${2:-"1 2 4"}
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for n in $NS; do
  timeout -k 10 300 python bench.py --gen-only --replicas $n --tmp /tmp > $OUT/gen$n.log 2>&1 || { echo "gen $n failed"; exit 1; }
  D=/tmp/gac_bench_c2_200000_42; [ $n -gt 1 ] && D=${D}_x$n
  th=$((16 / n))
  for step in 1 2 3; do
    rm -f /tmp/o$n.*
    t0=$(date +%s%N)
    pids=""
    for r in $(seq 0 $((n-1))); do
      extra=""; [ $n -gt 1 ] && extra="-nranks=$n -rank=$r -gpu=0"
      GAC_THREADS=$th GAC_TIMING=1 timeout -k 10 120 genomealignmenttools_amd/bin/chainNet $D/in.chain $D/t.sizes $D/q.sizes /tmp/o$n.t.net /tmp/o$n.q.net \
        -rescore -tNibDir=$D/t.2bit -qNibDir=$D/q.2bit -linearGap=loose -verbose=2 $extra > $OUT/n$n.s$step.r$r.log 2>&1 &
      pids="$pids $!"
    done
    for p in $pids; do wait $p || { echo "rank failed (n=$n)"; exit 1; }; done
    t1=$(date +%s%N)
    echo "n=$n step $step wall_ms $(( (t1 - t0) / 1000000 ))" | tee -a $OUT/wall.log
  done
  grep -h "stage\]" $OUT/n$n.s3.r0.log | tr -s ' ' | sed "s/^/n=$n r0 /"
done
