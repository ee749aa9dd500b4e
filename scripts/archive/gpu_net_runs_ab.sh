#!/bin/bash
# Net writer run size A/B (GAC_NET_RUN_FILLS) on C5 at --chains: chainNet
# -rescore, variants interleaved, 2 rounds; write-nets stage and wall time.
set -o pipefail
TAG=${1:-netruns}; CH=${2:-1000000}; shift 2
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
(while sleep 50; do date +%T >> $OUT/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 900 python scripts/bench_tools.py c5 --chains $CH --seed 1234 --no-ref > $OUT/gen.json 2> $OUT/gen.err || { echo gen failed; exit 1; }
D=/tmp/c5_${CH}_1234
for round in 1 2; do
  for v in "$@"; do
    t0=$(date +%s%N)
    GAC_NET_RUN_FILLS=$v GAC_TIMING=1 timeout -k 10 300 genomealignmenttools_amd/bin/chainNet $D/in.chain $D/t.sizes $D/q.sizes /tmp/n.$v.t.net /tmp/n.$v.q.net -rescore -tNibDir=$D/t.2bit -qNibDir=$D/q.2bit -linearGap=loose > $OUT/n.$v.$round.log 2>&1 || { echo "run $v failed"; exit 1; }
    t1=$(date +%s%N)
    echo "fills/run $v round $round wall $(( (t1 - t0) / 1000000 )) ms $(grep -h 'write nets' $OUT/n.$v.$round.log)" | tee -a $OUT/wall.txt
  done
done
for v in "$@"; do cmp /tmp/n.$v.t.net $D/ours.t.net && cmp /tmp/n.$v.q.net $D/ours.q.net && echo "$v identical"; done
