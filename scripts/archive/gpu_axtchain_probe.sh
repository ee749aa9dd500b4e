#!/bin/bash
# Run the axtChain drop-in on the golden cases; keep outputs under
# gpurun_out/ax/ and compare with the reference's (tests/golden).
set -u
G=$PWD/tests/golden
BIN=$PWD/genomealignmenttools_amd/bin/axtChain
OUT=gpurun_out/ax
rm -rf $OUT && mkdir -p $OUT
for c in newStyleLastz oldStyleBlastz; do
  timeout -k 10 120 $BIN -psl $G/chrM/$c.psl -minScore=3000 -linearGap=loose $G/chrM/hg19.chrM.2bit \
    -scoreScheme=$G/chrM/$c.Q.txt $G/chrM/susScr3.chrM.2bit $OUT/$c.chain 2> $OUT/$c.log; rc=$?
  echo "kat $c rc=$rc"; [ $rc -ge 124 ] && exit $rc
  cmp -s $OUT/$c.chain $G/chrM/$c.chain && echo "  same" || echo "  DIFF"
done
for s in 5 6; do
  for c in loose medium0 hoxd axt; do
    mkdir -p $OUT/s$s/$c
    opts=$(python3 -c "import json;print(' '.join(json.load(open('$G/axtchain/cases.json'))['$c']).replace('../../chrM','$G/chrM'))")
    inp=in.psl; [ $c = axt ] && inp=in.axt.gz
    ( cd $OUT/s$s/$c && timeout -k 10 120 $BIN $opts $G/axtchain/s$s/$inp $G/axtchain/s$s/t.2bit \
        $G/axtchain/s$s/q.2bit out.chain > log.txt 2>&1 ); rc=$?
    echo "s$s $c rc=$rc"; [ $rc -ge 124 ] && exit $rc
    cmp -s $OUT/s$s/$c/out.chain $G/axtchain/s$s/$c.chain && echo "  chain same" || echo "  chain DIFF"
    [ $c = hoxd ] && { cmp -s $OUT/s$s/$c/hoxd.details $G/axtchain/s$s/hoxd.details && echo "  details same" || echo "  details DIFF"; }
  done
done
exit 0
