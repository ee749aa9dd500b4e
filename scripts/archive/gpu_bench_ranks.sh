#!/bin/bash
# bench.py's N>1 path rehearsed on this one-GPU box (GAC_BENCH_ONE_GPU: all
# ranks on device 0, gloo for the clock) with torchrun, N = 2 and 4; then
# the nets of the last step checked against a single-process run of the tool
# on the same replicated input.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/benchranks; mkdir -p $OUT
export TMPDIR=/tmp
for n in 2 4; do
  GAC_BENCH_ONE_GPU=1 GAC_THREADS=$((16 / n)) timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 3 --warmup 1 --no-kernel \
    > $OUT/bench$n.json 2> $OUT/bench$n.err || { echo "bench n=$n failed"; tail -20 $OUT/bench$n.err; exit 1; }
  cat $OUT/bench$n.json
  D=/tmp/gac_bench_c2_200000_42_x$n
  timeout -k 10 120 genomealignmenttools_amd/bin/chainNet $D/in.chain $D/t.sizes $D/q.sizes /tmp/one.t.net /tmp/one.q.net \
    -rescore -tNibDir=$D/t.2bit -qNibDir=$D/q.2bit -linearGap=loose > $OUT/one$n.log 2>&1 || { echo "single run failed"; exit 1; }
  cmp /tmp/one.t.net $D/ours.r$n.t.net && cmp /tmp/one.q.net $D/ours.r$n.q.net && echo "n=$n nets identical to the single-process run"
done
