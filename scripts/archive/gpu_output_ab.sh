#!/bin/bash
# Large-output A/B: scoreChain and chainNet -rescore on C5 at --chains
# (default 1e6) with gac_par_output's mapped path on (default threshold) and
# off (GAC_OUTPUT_MMAP_MIN=-1), interleaved, 3 rounds; outputs compared.
set -o pipefail
TAG=${1:-outab}; CH=${2:-1000000}
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
(while sleep 50; do date +%T >> $OUT/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 600 python scripts/bench_tools.py c5 --chains $CH --seed 1234 --no-ref > $OUT/gen.json 2> $OUT/gen.err || { echo gen failed; tail $OUT/gen.err; exit 1; }
D=/tmp/c5_${CH}_1234
for round in 1 2 3; do
  for m in on off; do
    if [ $m = on ]; then E=""; else E="GAC_OUTPUT_MMAP_MIN=-1"; fi
    t0=$(date +%s%N)
    env GAC_TIMING=1 $E timeout -k 10 300 genomealignmenttools_amd/bin/scoreChain $D/in.chain $D/t.2bit $D/q.2bit /tmp/sc.$m.chain -linearGap=loose > $OUT/sc.$m.$round.log 2>&1 || { echo sc failed; exit 1; }
    t1=$(date +%s%N)
    env GAC_TIMING=1 $E timeout -k 10 300 genomealignmenttools_amd/bin/chainNet $D/in.chain $D/t.sizes $D/q.sizes /tmp/cn.$m.t.net /tmp/cn.$m.q.net -rescore -tNibDir=$D/t.2bit -qNibDir=$D/q.2bit -linearGap=loose > $OUT/cn.$m.$round.log 2>&1 || { echo cn failed; exit 1; }
    t2=$(date +%s%N)
    echo "$m $round scoreChain $(( (t1 - t0) / 1000000 )) chainNet $(( (t2 - t1) / 1000000 ))" | tee -a $OUT/wall.txt
  done
done
cmp /tmp/sc.on.chain /tmp/sc.off.chain && cmp /tmp/cn.on.t.net /tmp/cn.off.t.net && cmp /tmp/cn.on.q.net /tmp/cn.off.q.net && echo "outputs identical"
ls -la /tmp/sc.on.chain /tmp/cn.on.t.net /tmp/cn.on.q.net
df -T /tmp | tail -1
grep -h "par_output\|write" $OUT/*.on.3.log $OUT/*.off.3.log
