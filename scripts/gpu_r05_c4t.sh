#!/bin/bash
# C4 (axtChain -psl, 50 M blocks) with GAC_TIMING: its stage laps, REPS runs.
set -o pipefail
out=gpurun_out/${1:-r05c4t}
mkdir -p $out
export TMPDIR=/tmp
S=genomealignmenttools_amd/libexec/gac_synth
B=$GRAFT_REPO_ROOT/genomealignmenttools_amd/bin
d=/tmp/c4t
$S c4 $d -seed=7 -blocks=50000000 -threads=16 > /dev/null || exit 1
for i in $(seq 1 ${REPS:-2}); do
  t0=$(date +%s%N)
  ( cd $d && GAC_TIMING=1 timeout -k 10 200 $B/axtChain -linearGap=loose -verbose=${VERB:-0} -psl in.psl \
      t.2bit q.2bit o.chain ) > $out/c4_$i.err 2>&1 || exit $?
  echo "wall $(( ($(date +%s%N) - t0) / 1000000 )) ms" >> $out/c4_$i.err
  sha256sum $d/o.chain >> $out/c4_$i.err
  rm -f $d/o.chain
done
rm -rf $d
echo ok
