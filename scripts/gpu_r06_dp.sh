#!/bin/bash
# k_dp_fast on a C4-shaped set (GAC_AXT_DP=gpu, every pair on the device) with
# GAC_DP_PROF's per-phase cycle counters, against the host DP's output.
set -o pipefail
out=gpurun_out/${1:-r06dp}
mkdir -p $out
export TMPDIR=/tmp
S=genomealignmenttools_amd/libexec/gac_synth
B=$GRAFT_REPO_ROOT/genomealignmenttools_amd/bin
d=/tmp/c4dp
$S c4 $d -seed=7 -blocks=${BLOCKS:-1000000} -threads=16 > /dev/null || exit 1
( cd $d && GAC_AXT_DP=host timeout -k 10 200 $B/axtChain -linearGap=loose -psl in.psl t.2bit q.2bit h.chain ) \
    > $out/host.err 2>&1 || exit $?
for i in $(seq 1 ${REPS:-2}); do
  # run 1: plain; runs 2..: with GAC_DP_PROF's counters
  prof=$([ $i -gt 1 ] && echo 1 || echo "")
  ( cd $d && GAC_AXT_DP=gpu GAC_DP_PROF=$prof GAC_TIMING=1 GAC_DP_WALK=${WALK:-} timeout -k 10 300 $B/axtChain -linearGap=loose -psl in.psl \
      t.2bit q.2bit g.chain ) > $out/gpu_$i.err 2>&1 || exit $?
  cmp $d/h.chain $d/g.chain && echo "same $i" >> $out/gpu_$i.err || { echo DIFF >> $out/gpu_$i.err; exit 1; }
done
if [ -n "$AB" ]; then  # the other walk, plain
  ( cd $d && GAC_AXT_DP=gpu GAC_TIMING=1 GAC_DP_WALK=$AB timeout -k 10 300 $B/axtChain -linearGap=loose -psl in.psl \
      t.2bit q.2bit a.chain ) > $out/ab.err 2>&1 || exit $?
  cmp $d/h.chain $d/a.chain || exit 1
fi
grep -h "k_dp_fast\|device DP" $out/*.err
rm -rf $d
echo ok
