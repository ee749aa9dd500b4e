#!/bin/bash
# debug: the device-built DP inputs (GAC_DT_DUMP) against the CPU stand-in's
# on one C4-shaped set; first mismatch per array
set -o pipefail
out=gpurun_out/${1:-r06dd}
mkdir -p $out
export TMPDIR=/tmp
d=/tmp/dd
mkdir -p $d/gpu $d/cpu
genomealignmenttools_amd/libexec/gac_synth c4 $d -blocks=${BLOCKS:-300000} -nt=6 -nq=5 -tsize=4000000 -qsize=3000000 -threads=4 > /dev/null || exit 1
args="-linearGap=loose -psl in.psl t.2bit q.2bit"
( cd $d && GAC_AXT_DP=gpu GAC_DT_DUMP=$d/gpu timeout -k 10 300 $GRAFT_REPO_ROOT/genomealignmenttools_amd/bin/axtChain $args gpu.chain ) > $out/gpu.err 2>&1
echo "gpu rc $?" | tee -a $out/summary.txt
( cd $d && GAC_AXT_DP=gpu GAC_DT_DUMP=$d/cpu timeout -k 10 600 $GRAFT_REPO_ROOT/oracle/_build/axtChain_cpu $args cpu.chain ) > $out/cpu.err 2>&1
echo "cpu rc $?" | tee -a $out/summary.txt
cmp $d/gpu.chain $d/cpu.chain >> $out/summary.txt 2>&1
python3 - $d >> $out/summary.txt 2>&1 <<'PY'
import sys, numpy as np
d = sys.argv[1]
kinds = {"leaf_off": (np.int64, 1), "lf": (np.int32, 4), "lnode": (np.int32, 1), "na": (np.int32, 4),
         "nb": (np.int32, 2), "poff": (np.int64, 1), "path": (np.int32, 1), "ooff": (np.int64, 1),
         "ov": (np.int32, 1), "lf_total": (np.int64, 1), "lf_pred": (np.int32, 1)}
lo = np.fromfile(f"{d}/cpu/leaf_off", np.int64)
for k, (t, w) in kinds.items():
    try:
        a = np.fromfile(f"{d}/gpu/{k}", t); b = np.fromfile(f"{d}/cpu/{k}", t)
    except FileNotFoundError as e:
        print(k, "missing", e); continue
    if a.shape != b.shape:
        print(k, "shape", a.shape, b.shape); continue
    bad = np.nonzero(a != b)[0]
    print(k, "n", a.size, "mismatches", bad.size, "first", bad[:8].tolist(),
          "gpu", a[bad[:4]].tolist(), "cpu", b[bad[:4]].tolist())
PY
cat $out/summary.txt
