#!/bin/bash
# Run the chainCleaner drop-in on every golden case (tests/golden/cleaner),
# keep the outputs under gpurun_out/cc/<case>/ and diff them against the
# reference's.  Usage (GPU box): bash scripts/archive/gpu_cleaner_probe.sh
set -u
G=tests/golden/cleaner
BIN=genomealignmenttools_amd/bin/chainCleaner
OUT=gpurun_out/cc
rm -rf $OUT && mkdir -p $OUT
for c in default pairs lowfold filters sdata debug; do
  mkdir -p $OUT/$c
  opts=$(python3 -c "import json;print(' '.join(json.load(open('$G/cases.json'))['cases']['$c']))")
  ( cd $OUT/$c && timeout -k 10 300 ../../../$BIN ../../../$G/in.chain ../../../$G/t.2bit \
      ../../../$G/q.2bit out.chain out.bed -net=../../../$G/in.net $opts -verbose=2 \
      > log.txt 2>&1 ); rc=$?
  echo "case $c rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $OUT/$c/log.txt; [ $rc -ge 124 ] && exit $rc; continue; }
  for f in $(ls $G/$c); do
    cmp -s $OUT/$c/$f $G/$c/$f && echo "  $f same" || echo "  $f DIFF"
  done
done
mkdir -p $OUT/nonet
( cd $OUT/nonet && timeout -k 10 300 ../../../$BIN ../../../$G/in.chain ../../../$G/t.2bit \
    ../../../$G/q.2bit out.chain out.bed -tSizes=../../../$G/t.sizes \
    -qSizes=../../../$G/q.sizes -linearGap=loose > log.txt 2>&1 ) ; echo "nonet rc=$?"
for f in out.chain out.bed; do
  cmp -s $OUT/nonet/$f $G/default/$f && echo "  nonet $f same" || echo "  nonet $f DIFF"
done
