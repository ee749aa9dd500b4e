#!/bin/bash
# bench.py's N>1 path on this one-GPU box (GAC_BENCH_ONE_GPU), N = 4, with the
# sparse genome upload on and off, alternating (3 rounds).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-ranksab}; mkdir -p $OUT
export TMPDIR=/tmp
n=4
for round in 1 2 3; do
  for sp in 1 0; do
    GAC_NET_SPARSE=$sp GAC_BENCH_ONE_GPU=1 GAC_THREADS=4 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29500 + round * 2 + sp)) bench.py --gpus $n --steps 5 --warmup 1 --no-kernel \
      > $OUT/b.$sp.$round.json 2> $OUT/b.$sp.$round.err || { echo "bench sparse=$sp failed"; tail -20 $OUT/b.$sp.$round.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('sparse=$sp', round(d['ms_per_step'],1), 'ms', round(d['value'],3))" $OUT/b.$sp.$round.json
  done
done
