#!/bin/bash
# axtChain host-DP A/B on the C4-like set (GPU box host): environment
# variants interleaved, 3 rounds; DP stage lines and outputs compared.
# usage: bash scripts/archive/gpu_dp_ab.sh TAG BLOCKS "NAME:ENV=V,ENV=V" ...
set -o pipefail
TAG=${1:-dpab}; BLOCKS=${2:-2000000}; shift 2
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python scripts/bench_tools.py axtchain --blocks $BLOCKS --no-ref > $OUT/gen.json 2> $OUT/gen.err || { echo gen failed; tail $OUT/gen.err; exit 1; }
D=/tmp/c4_$BLOCKS
for round in 1 2 3; do
  for spec in "$@"; do
    name=${spec%%:*}; envs=$(echo "${spec#*:}" | tr ',' ' ')
    t0=$(date +%s%N)
    env GAC_TIMING=1 GAC_DP_STATS=1 $envs timeout -k 10 600 genomealignmenttools_amd/bin/axtChain -linearGap=loose -verbose=0 -psl $D/in.psl $D/t.2bit $D/q.2bit /tmp/ab.$name.chain > $OUT/$name.$round.log 2>&1 || { echo "$name failed"; tail $OUT/$name.$round.log; exit 1; }
    t1=$(date +%s%N)
    echo "$name $round $(( (t1 - t0) / 1000000 )) ms $(grep -h 'largest' $OUT/$name.$round.log | sed 's/.*largest/largest/')" | tee -a $OUT/wall.txt
  done
done
for spec in "$@"; do name=${spec%%:*}; cmp /tmp/ab.$name.chain $D/ours.chain && echo "$name identical to the first run"; done
grep -h "\[dp\]" $OUT/*.1.log | sort | uniq | tail -4
