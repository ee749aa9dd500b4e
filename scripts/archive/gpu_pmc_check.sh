#!/bin/bash
# The bench's counter-pass child under rocprofv3: kernel trace alone, then
# the two --pmc passes bench.py makes; k_tile durations and counters side by
# side (checks that the in-run traffic figure measures the bench's call).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-pmcchk}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --gen-only > $OUT/gen.log 2>&1 || exit 1
cd /tmp
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 $GRAFT_REPO_ROOT/bench.py --pmc-child > $OUT/kt.log 2>&1 || { echo "kt failed"; tail $OUT/kt.log; exit 1; }
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum --output-format csv -d $OUT/p1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --pmc-child > $OUT/p1.log 2>&1 || { echo "p1 failed"; tail $OUT/p1.log; exit 1; }
grep -h "k_tile" $OUT/kt/*kernel_stats.csv | cut -c1-200
python3 - $OUT <<'PY'
import csv, glob, sys, collections
root = sys.argv[1]
for path in glob.glob(root + "/p1/**/*counter_collection.csv", recursive=True):
    rows = list(csv.DictReader(open(path)))
    print(path, len(rows), "rows; columns:", list(rows[0].keys()))
    per = collections.defaultdict(float); cnt = collections.Counter()
    for r in rows:
        if "k_tile" in r["Kernel_Name"]:
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
            cnt[(r["Dispatch_Id"], r["Counter_Name"])] += 1
    for k in sorted(per, key=lambda k: (int(k[0]), k[1])):
        print(k, per[k], "rows", cnt[k])
for path in glob.glob(root + "/p1/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(path)):
        if "k_tile" in r["Kernel_Name"]:
            print("dispatch", r.get("Dispatch_Id"), "dur_us", (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
PY
