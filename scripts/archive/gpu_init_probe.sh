#!/bin/bash
# HIP bring-up cost under several environments (scripts/probes/hip_init_probe.c)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/init; mkdir -p $OUT
gcc -O2 scripts/probes/hip_init_probe.c -o $OUT/hip_init_probe -ldl || exit 1
for e in "X=0" "HSA_ENABLE_SDMA=0" "HIP_ENABLE_DEFERRED_LOADING=0" "GPU_MAX_HW_QUEUES=1" "ROCR_VISIBLE_DEVICES=0" "AMD_DIRECT_DISPATCH=0" "HSA_ENABLE_INTERRUPT=0"; do
  for i in 1 2 3; do
    echo -n "$e: "; env $e timeout -k 5 60 $OUT/hip_init_probe || exit 1
  done
done 2>&1 | tee $OUT/init.log
