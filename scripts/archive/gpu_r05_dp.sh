#!/bin/bash
# Round-5: the exact fast device DP (k_dp_fast) -- axtChain GPU tests under
# GAC_AXT_DP=gpu, then C4 sets of 1 M and 5 M PSL blocks chained by the host
# DP and by the device DP (GAC_TIMING stage laps), outputs compared.
set -o pipefail
tag=${1:-r05dp}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
(while sleep 50; do date +%T >> $out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
    tests/test_gpu_tools.py -k axtchain tests/test_gpu_configs.py::test_c4_shaped_axtchain \
    > $out/gpu_tests.txt 2>&1 || exit $?
S=genomealignmenttools_amd/libexec/gac_synth
A=genomealignmenttools_amd/bin/axtChain
for nb in ${DP_SIZES:-1000000 5000000}; do
  d=/tmp/c4_$nb
  $S c4 $d -seed=7 -blocks=$nb -threads=16 > /dev/null || exit 1
  ( cd $d && GAC_TIMING=1 timeout -k 10 300 $GRAFT_REPO_ROOT/$A -linearGap=loose -verbose=0 -psl in.psl t.2bit q.2bit host.chain ) \
      > $out/c4_${nb}_host.err 2>&1 || exit $?
  ( cd $d && GAC_AXT_DP=gpu GAC_TIMING=1 timeout -k 10 600 $GRAFT_REPO_ROOT/$A -linearGap=loose -verbose=0 -psl in.psl t.2bit q.2bit dev.chain ) \
      > $out/c4_${nb}_dev.err 2>&1 || exit $?
  cmp $d/host.chain $d/dev.chain > $out/c4_${nb}_cmp.txt 2>&1 && echo same >> $out/c4_${nb}_cmp.txt
  rm -rf $d
done
echo ok
