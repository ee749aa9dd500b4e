#!/bin/bash
# Device bring-up phases (gac_open, GAC_TIMING) of one small scoreChain run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/open
G=tests/golden/synth11
for k in 1 2; do
  GAC_TIMING=1 timeout -k 10 60 genomealignmenttools_amd/bin/scoreChain $G/in.chain $G/t.2bit $G/q.2bit \
    gpurun_out/open/out.chain -linearGap=loose -verbose=2 2>&1 | grep -E "gac_open|stage" | tee gpurun_out/open/run$k.txt
done
