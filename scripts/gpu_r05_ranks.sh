#!/bin/bash
# Round-5: DESIGN §6's per-rank tables -- every rank of chainNet -nranks=N
# (C5, the headline) and axtChain -nranks=N (C4 50 M) run ALONE
# (GAC_RANK_SOLO=1: no rank waits for another, as on a node where each rank
# has its own GPU and host cores) with 16 host threads, one after another:
# its wall time, stage laps and work (GAC_TIMING).  The predicted N-GPU step
# is the slowest rank's solo time plus the part placement.
set -o pipefail
tag=${1:-r05ranks}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
(while sleep 50; do date +%T >> $out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
S=genomealignmenttools_amd/libexec/gac_synth
B=$GRAFT_REPO_ROOT/genomealignmenttools_amd/bin
d=/tmp/c5r
$S c5 $d -seed=1234 -chains=5000000 -sizesDir=genomealignmenttools_amd/data -threads=16 > /dev/null || exit 1
for n in ${NS:-1 2 4 8}; do
  for r in $(seq 0 $((n - 1))); do
    t0=$(date +%s%N)
    ( cd $d && GAC_RANK_SOLO=1 GAC_RANK_TOKEN=solo$n GAC_THREADS=16 GAC_TIMING=1 timeout -k 10 120 \
        $B/chainNet in.chain t.sizes q.sizes o.t.net o.q.net -rescore -tNibDir=t.2bit -qNibDir=q.2bit \
        -linearGap=loose $( [ $n -gt 1 ] && echo "-nranks=$n -rank=$r -gpu=0" ) ) \
        > $out/c5_n${n}_r${r}.err 2>&1 || exit $?
    echo "wall $(( ($(date +%s%N) - t0) / 1000000 )) ms" >> $out/c5_n${n}_r${r}.err
    rm -f $d/o.*
  done
done
rm -rf $d
[ "$NS4" = skip ] && echo ok && exit 0
d=/tmp/c4r
$S c4 $d -seed=7 -blocks=50000000 -threads=16 > /dev/null || exit 1
for n in ${NS4:-1 8}; do
  for r in $(seq 0 $((n - 1))); do
    t0=$(date +%s%N)
    ( cd $d && GAC_RANK_SOLO=1 GAC_RANK_TOKEN=solo$n GAC_THREADS=16 GAC_TIMING=1 timeout -k 10 200 \
        $B/axtChain -linearGap=loose -verbose=0 -psl in.psl t.2bit q.2bit o.chain \
        $( [ $n -gt 1 ] && echo "-nranks=$n -rank=$r -gpu=0" ) ) > $out/c4_n${n}_r${r}.err 2>&1 || exit $?
    echo "wall $(( ($(date +%s%N) - t0) / 1000000 )) ms" >> $out/c4_n${n}_r${r}.err
    rm -f $d/o.chain*
  done
done
rm -rf $d
echo ok
