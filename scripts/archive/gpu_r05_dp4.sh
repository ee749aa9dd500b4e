#!/bin/bash
# Round-5: C4 at 50 M blocks, host DP only vs hybrid variants (device share
# by GAC_DP_DEV_US, pool threads GAC_DP_POOL, the device side's host threads
# GAC_DP_DEV_THREADS), alternating; sha256 of every output.
set -o pipefail
tag=${1:-r05dp4}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
(while sleep 50; do date +%T >> $out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
S=genomealignmenttools_amd/libexec/gac_synth
A=$GRAFT_REPO_ROOT/genomealignmenttools_amd/bin/axtChain
d=/tmp/c4_50m
$S c4 $d -seed=7 -blocks=50000000 -threads=16 > /dev/null || exit 1
run() {  # tag env...
  local t=$1; shift
  local t0=$(date +%s%N)
  ( cd $d && env "$@" GAC_TIMING=1 timeout -k 10 300 $A -linearGap=loose -verbose=0 -psl in.psl t.2bit q.2bit $t.chain ) \
      >> $out/c4_$t.txt 2>&1 || return 1
  echo "wall $(( ($(date +%s%N) - t0) / 1000000 )) ms" >> $out/c4_$t.txt
  sha256sum $d/$t.chain >> $out/c4_$t.txt && rm -f $d/$t.chain
}
for i in ${REPS:-1 2}; do
  for v in ${VARIANTS:-host:GAC_AXT_DP=host h20:GAC_DP_DEV_US=20 h30:GAC_DP_DEV_US=30}; do
    t=${v%%:*}; e=${v#*:}
    run $t $(echo $e | tr ',' ' ') || exit 1
  done
done
rm -rf $d
echo ok
