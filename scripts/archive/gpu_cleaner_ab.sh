#!/bin/bash
# chainCleaner at 20k planted loci, alternating the small-batch scoring path
# (k_small, default) and the tile pipeline for every call (GAC_SMALL_MAX=0).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/clab
mkdir -p $OUT
timeout -k 10 600 python scripts/bench_tools.py cleaner --loci 20000 --no-ref > $OUT/gen.json 2> $OUT/gen.log || exit 1
D=/tmp/c3_20000
for k in 1 2 3; do
  for m in 256 0; do
    s=$(date +%s.%N)
    ( cd $D && GAC_SMALL_MAX=$m GAC_TIMING=1 timeout -k 10 120 "$GRAFT_REPO_ROOT/genomealignmenttools_amd/bin/chainCleaner" in.chain t.2bit q.2bit ab.chain ab.bed \
        -tSizes=t.sizes -qSizes=q.sizes -linearGap=loose -verbose=1 ) > $OUT/run_${m}_$k.log 2>&1 || exit 1
    e=$(date +%s.%N)
    cmp -s $D/ab.chain $D/ours.chain && cmp -s $D/ab.bed $D/ours.bed && same=same || same=DIFF
    echo "small_max=$m run $k wall $(python3 -c "print(round($e-$s,3))") $same $(grep '^GPU:' $OUT/run_${m}_$k.log)" | tee -a $OUT/summary.txt
  done
done
