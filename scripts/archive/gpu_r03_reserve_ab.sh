#!/bin/bash
# The -m gpu suite, then scoreChain on C5 end to end with and without the
# chain set reserved during the parse (GAC_NO_RESERVE=1), alternating, 3 each.
set -o pipefail
tag=${1:-r03rs}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 1200 --timeout-method thread \
    > $out/gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/gpu_tests.txt; tail -2 $out/gpu_tests.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --gen-only > $out/gen.log 2>&1 || exit $?
D=/tmp/gac_bench_c5_5000000_1234
for r in 1 2 3; do
  for v in reserve noreserve; do
    E=""; [ $v = noreserve ] && E="GAC_NO_RESERVE=1"
    t0=$(date +%s.%N)
    /usr/bin/env $E GAC_TIMING=1 timeout -k 10 120 genomealignmenttools_amd/bin/scoreChain $D/in.chain $D/t.2bit $D/q.2bit /tmp/sc.out -linearGap=loose > /dev/null 2> $out/sc_${v}_$r.err || exit $?
    t1=$(date +%s.%N)
    rm -f /tmp/sc.out
    echo "$v $r: wall $(echo "$t1 - $t0" | bc) s; $(grep -E 'chain records|allocations|chains to HBM|read chains' $out/sc_${v}_$r.err | tr -s ' ' | tr '\n' ';')" | tee -a $out/summary.txt
  done
done
