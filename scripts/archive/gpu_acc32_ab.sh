#!/bin/bash
# k_tile int32 LDS block accumulators (GAC_ACC32) A/B on the kernel leg,
# GPU parity tests of the variant, then the default build's full check.
# usage: bash scripts/archive/gpu_acc32_ab.sh TAG
set -o pipefail
TAG=${1:-acc32}
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
bash scripts/archive/gpu_tile_probe.sh $TAG base::HIPEXTRA= acc32::HIPEXTRA=-DGAC_ACC32=1 \
  base2::HIPEXTRA= acc32b::HIPEXTRA=-DGAC_ACC32=1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_scoring.py tests/test_gpu_tools.py -x -q -m gpu \
  --timeout 300 --timeout-method thread > "$OUT/acc32_tests.log" 2>&1
rc=$?; tail -2 "$OUT/acc32_tests.log"; [ $rc -le 1 ] || exit $rc
make -B -j16 all HIPEXTRA= > "$OUT/rebuild.log" 2>&1 || exit 1
bash scripts/gpu_check.sh ${TAG}_check
