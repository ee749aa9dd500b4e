#!/bin/bash
# Round 6: rocprofv3 kernel statistics of the kd-tree DP on the C4-shaped
# 1 M-block set, every pair on the device (GAC_AXT_DP=gpu): k_dp_spec (16
# waves per pair, the default) and k_dp_fast (GAC_DP_WAVES=1); the device
# build kernels (k_dt_*) in the same trace.
set -o pipefail
out=gpurun_out/${1:-r06dpprof}
mkdir -p $out
export TMPDIR=/tmp
S=genomealignmenttools_amd/libexec/gac_synth
X=$GRAFT_REPO_ROOT/genomealignmenttools_amd/libexec/axtChain
d=/tmp/c4p
$S c4 $d -seed=7 -blocks=1000000 -threads=16 > /dev/null || exit 1
cd $d
for w in 16 1; do
  GAC_AXT_DP=gpu GAC_DP_WAVES=$w GAC_TIMING=1 GAC_PROFILE_EXIT=1 HSA_ENABLE_SDMA=0 timeout -k 10 300 \
    rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/w$w -o run -- \
    $X -linearGap=loose -psl in.psl t.2bit q.2bit w$w.chain > $GRAFT_REPO_ROOT/$out/w$w.err 2>&1 || exit $?
done
cmp w16.chain w1.chain && echo "w16 = w1 chains" | tee -a $GRAFT_REPO_ROOT/$out/summary.txt
cd $GRAFT_REPO_ROOT
find $out -name "*kernel_stats.csv" | while read f; do echo "== $f"; head -12 "$f"; done | tee -a $out/summary.txt
