#!/bin/bash
# Round-3 final evidence, part B: rocprofv3 --kernel-trace --stats over a short
# bench run (kernel legs), then bench.py's N = 2 strong-scaling path rehearsed
# on this one-GPU box (GAC_BENCH_ONE_GPU: both ranks on device 0, gloo clock).
set -o pipefail
tag=${1:-r03f}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
bash scripts/archive/gpu_r03_prof.sh $tag || exit $?
GAC_BENCH_ONE_GPU=1 GAC_THREADS=8 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 2 \
    --warmup 1 --no-kernel > $out/bench_n2.json 2> $out/bench_n2.err
rc=$?
echo "n2 rc=$rc"; tail -3 $out/bench_n2.err
exit $rc
