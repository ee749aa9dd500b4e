#!/bin/bash
# C4 (axtChain, 50 M blocks, default hybrid): rocprofv3 kernel trace of one
# run (the tool's binary under the profiler, exit(0) so it writes its data)
set -o pipefail
out=gpurun_out/${1:-r06c4prof}
mkdir -p $out
export TMPDIR=/tmp
S=genomealignmenttools_amd/libexec/gac_synth
X=$GRAFT_REPO_ROOT/genomealignmenttools_amd/libexec/axtChain
d=/tmp/c4p
$S c4 $d -seed=7 -blocks=50000000 -threads=16 > /dev/null || exit 1
cd $d
GAC_TIMING=1 GAC_PROFILE_EXIT=1 HSA_ENABLE_SDMA=0 timeout -k 10 300 \
  rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof -o run -- \
  $X -linearGap=loose -psl in.psl t.2bit q.2bit o.chain > $GRAFT_REPO_ROOT/$out/run.err 2>&1 || exit $?
sha256sum o.chain | cut -c1-16 > $GRAFT_REPO_ROOT/$out/sha.txt
echo ok
