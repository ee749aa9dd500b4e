#!/bin/bash
# A/B of scoreChain's chain upload on C5 (GAC_TIMING laps), the current
# library vs lib/variants/old (the chain records zero-filled on one thread),
# alternating, three runs each.
set -o pipefail
tag=${1:-r03ua}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --gen-only > $out/gen.log 2>&1 || exit $?
D=$(ls -d /tmp/gac_bench_c5_5000000_1234)
L=genomealignmenttools_amd/lib
cp $L/libgachain.so $L/variants/new.so
for r in 1 2 3; do
  for v in new old; do
    cp $L/variants/$( [ $v = new ] && echo new.so || echo old/libgachain.so ) $L/libgachain.so
    /usr/bin/env GAC_TIMING=1 timeout -k 10 120 genomealignmenttools_amd/bin/scoreChain $D/in.chain $D/t.2bit $D/q.2bit /tmp/sc.out -linearGap=loose > /dev/null 2> $out/sc_${v}_$r.err || exit $?
    rm -f /tmp/sc.out
    echo "$v $r: $(grep -E 'chain records|allocations|chains to HBM' $out/sc_${v}_$r.err | tr -s ' ' | tr '\n' ';')" | tee -a $out/summary.txt
  done
done
cp $L/variants/new.so $L/libgachain.so
