#!/bin/bash
# Round-3 probes: random-load request sizes (default vs non-temporal) and
# where the end-to-end tool's exit time goes.  Each GPU step has its own
# time limit; a failure ends the script.
set -o pipefail
out=gpurun_out/${1:-r03b}
mkdir -p $out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 90 $R/scripts/probes/ld_granularity > $out/ld.txt 2>&1 || exit $?
cat $out/ld.txt
(cd /tmp && timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_32B_sum \
    TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --output-format csv -d /tmp/pmc_ld -o run \
    -- $R/scripts/probes/ld_granularity > /dev/null 2>&1) || exit $?
python3 - <<'PY' > $out/ld_pmc.txt
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for p in glob.glob('/tmp/pmc_ld/**/*counter_collection.csv', recursive=True):
    for row in csv.DictReader(open(p)):
        agg[row['Kernel_Name'][:40]][row['Counter_Name']].append(float(row['Counter_Value']))
for k, v in agg.items():
    print(k, {c: sum(x) / len(x) for c, x in v.items()})
PY
cat $out/ld_pmc.txt
d=/tmp/gac_bench_c5_5000000_1234
[ -e $d/info.json ] || timeout -k 10 120 $R/genomealignmenttools_amd/libexec/gac_synth c5 $d \
    -chains=5000000 -sizesDir=$R/genomealignmenttools_amd/data -threads=16 || exit $?
P=$R/scripts/probes/exit_probe
CN=$R/genomealignmenttools_amd/bin/chainNet
timeout -k 10 400 python3 $R/scripts/exit_probe.py 3 -- \
    $P open ";;" $P alloc 6 ";;" $P keep 6 ";;" $P host 8 ";;" $P host 24 ";;" \
    $CN $d/in.chain $d/t.sizes $d/q.sizes /tmp/a.t.net /tmp/a.q.net -verbose=2 ";;" \
    $CN $d/in.chain $d/t.sizes $d/q.sizes /tmp/b.t.net /tmp/b.q.net -rescore \
        -tNibDir=$d/t.2bit -qNibDir=$d/q.2bit -linearGap=loose -verbose=2 \
    > $out/exit.txt 2>&1 || exit $?
cat $out/exit.txt
