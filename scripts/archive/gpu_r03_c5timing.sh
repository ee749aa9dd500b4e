#!/bin/bash
# Probe: full stage/sub-stage timing (GAC_TIMING) of bin/chainNet -rescore on
# C5 (gac_synth, seed 1234), twice, stderr kept whole.
set -o pipefail
tag=${1:-r03d}
out=$PWD/gpurun_out/$tag
mkdir -p $out
P=$PWD/genomealignmenttools_amd
D=${TMPDIR:-/tmp}/c5probe
mkdir -p $D
[ -f $D/info.json ] || timeout -k 10 120 $P/libexec/gac_synth c5 $D -seed=1234 -threads=16 \
    -sizesDir=$P/data > $out/synth.txt 2>&1 || exit $?
cd $D
for i in 1 2; do
    rm -f o.t.net o.q.net
    GAC_TIMING=1 timeout -k 10 120 $P/bin/chainNet -verbose=2 -rescore -tNibDir=t.2bit \
        -qNibDir=q.2bit -linearGap=loose in.chain t.sizes q.sizes o.t.net o.q.net \
        > $out/c5_timing_$i.txt 2>&1 || exit $?
done
echo "c5 timing ok"
