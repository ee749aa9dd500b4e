#!/bin/bash
# chainNet -rescore with the sparse genome upload: the chainNet GPU parity
# tests, then C2 end to end with sparse vs whole-genome uploads (A/B).
# usage: bash scripts/archive/gpu_sparse_check.sh TAG
set -o pipefail
TAG=${1:-sparse}
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_tools.py tests/test_gpu_configs.py -x -v -m gpu -k "chainnet" --timeout 600 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?
tail -3 "$OUT/tests.log"
[ $rc -eq 0 ] || exit $rc
bash scripts/archive/gpu_e2e_ab.sh "$TAG/ab" "sparse:GAC_NET_SPARSE=1" "whole:GAC_NET_SPARSE=0"
