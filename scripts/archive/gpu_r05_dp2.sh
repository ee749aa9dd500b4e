#!/bin/bash
# Round-5: the hybrid DP -- k_dp_fast with LDS/arithmetic gap costs: device
# tests, the device's per-leaf rate (C4 1 M, all pairs on the device), then
# C4 at 50 M blocks: host DP only vs the hybrid default, sha256 of each run
# against the reference golden.
set -o pipefail
tag=${1:-r05dp2}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
(while sleep 50; do date +%T >> $out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_tools.py -k axtchain tests/test_gpu_configs.py::test_c4_shaped_axtchain \
    > $out/gpu_tests.txt 2>&1 || exit $?
S=genomealignmenttools_amd/libexec/gac_synth
A=$GRAFT_REPO_ROOT/genomealignmenttools_amd/bin/axtChain
d=/tmp/c4_1m
$S c4 $d -seed=7 -blocks=1000000 -threads=16 > /dev/null || exit 1
( cd $d && GAC_AXT_DP=gpu GAC_TIMING=1 timeout -k 10 300 $A -linearGap=loose -verbose=0 -psl in.psl t.2bit q.2bit dev.chain \
  && GAC_AXT_DP=host timeout -k 10 300 $A -linearGap=loose -verbose=0 -psl in.psl t.2bit q.2bit host.chain \
  && cmp dev.chain host.chain && echo same ) > $out/c4_1m.txt 2>&1 || exit $?
rm -rf $d
d=/tmp/c4_50m
$S c4 $d -seed=7 -blocks=50000000 -threads=16 > /dev/null || exit 1
for mode in host hybrid hybrid10 host hybrid; do
  case $mode in
    host) env="GAC_AXT_DP=host";; hybrid) env="GAC_DP_DEV_US=20";; hybrid10) env="GAC_DP_DEV_US=10";;
  esac
  t0=$(date +%s%N)
  ( cd $d && env $env GAC_TIMING=1 timeout -k 10 300 $A -linearGap=loose -verbose=0 -psl in.psl t.2bit q.2bit $mode.chain ) \
      >> $out/c4_50m_$mode.txt 2>&1 || exit $?
  echo "wall $(( ($(date +%s%N) - t0) / 1000000 )) ms" >> $out/c4_50m_$mode.txt
  sha256sum $d/$mode.chain >> $out/c4_50m_$mode.txt && rm -f $d/$mode.chain
done
rm -rf $d
echo ok
