#!/bin/bash
# Round 6: k_dp_spec (W waves per pair, in-order commits) vs k_dp_fast on a
# C4-shaped set with every pair on the device (GAC_AXT_DP=gpu), outputs
# compared with the host DP's; then C4 at 50 M blocks with the hybrid.
set -o pipefail
out=gpurun_out/${1:-r06spec}
mkdir -p $out
export TMPDIR=/tmp
S=genomealignmenttools_amd/libexec/gac_synth
B=$GRAFT_REPO_ROOT/genomealignmenttools_amd/bin
d=/tmp/c4w
$S c4 $d -seed=7 -blocks=${BLOCKS:-1000000} -threads=16 > /dev/null || exit 1
args="-linearGap=loose -psl in.psl t.2bit q.2bit"
( cd $d && GAC_AXT_DP=host timeout -k 10 300 $B/axtChain $args host.chain ) > $out/host.err 2>&1 || exit 1
for w in ${WAVES:-1 4 8 16}; do
  ( cd $d && GAC_AXT_DP=gpu GAC_DP_WAVES=$w GAC_DP_PROF=1 GAC_TIMING=1 timeout -k 10 200 $B/axtChain $args w$w.chain ) > $out/w$w.err 2>&1
  rc=$?
  same=$(cmp -s $d/host.chain $d/w$w.chain && echo same || echo DIFF)
  echo "waves $w rc $rc $same $(grep -o 'k_dp_[a-z]* [0-9.]* s, [0-9]* pairs, [0-9]* leaves, [0-9]* fallbacks' $out/w$w.err) $(grep -o 'k_dp[_a-z]* [0-9.]* s, results' $out/w$w.err)" | tee -a $out/summary.txt
  [ $rc -eq 0 ] || exit $rc
done
rm -rf $d
echo ok
