#!/bin/bash
# Chain-text writer throughput on the GPU box's host (no GPU work): the C2
# chain file rewritten by gt_par_write at several thread counts and run
# sizes, to /tmp and to /dev/null.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-wprobe}; mkdir -p $OUT
export TMPDIR=/tmp
gcc -O2 -std=gnu11 -Iinclude -Igenomealignmenttools_amd/csrc -Igenomealignmenttools_amd/csrc/tools/lib scripts/probes/chain_write_probe.c build/obj/tools/lib/*.o -o /tmp/wprobe -Lgenomealignmenttools_amd/lib -lgachain -Wl,-rpath,$GRAFT_REPO_ROOT/genomealignmenttools_amd/lib -lz -lm -lpthread || exit 1
timeout -k 10 300 python bench.py --gen-only > $OUT/gen.log 2>&1 || exit 1
D=/tmp/gac_bench_c2_200000_42
for t in 1 16; do
  for items in default 50 1000 10000; do
    E=""; [ $items = default ] || E="GAC_RUN_ITEMS=$items"
    echo "threads $t items $items tmp: $(env $E GAC_THREADS=$t timeout 120 /tmp/wprobe $D/in.chain /tmp/w.chain | tr '\n' ' ')"
    echo "threads $t items $items null: $(env $E GAC_THREADS=$t timeout 120 /tmp/wprobe $D/in.chain /dev/null | tr '\n' ' ')"
  done
done | tee $OUT/probe.txt
cmp /tmp/w.chain $D/in.chain && echo "round trip identical"
