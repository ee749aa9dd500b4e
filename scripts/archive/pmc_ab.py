#!/usr/bin/env python3
"""Probe (measurement only): PMC counters of k_tile for one bench leg
(fills | scorechain) under a few env settings, one rocprofv3 --kernel-trace
--pmc pass per counter group (no other trace domains), averaged over the
k_tile dispatches.  Usage: pmc_ab.py OUTDIR LEG NAME=ENV[,ENV...] ...
e.g. pmc_ab.py gpurun_out/x scorechain target=GAC_WHOLE_ORDER=target set=GAC_WHOLE_ORDER=set
Writes OUTDIR/pmc_<LEG>.json.  Needs the C5 files (bench.py --gen-only)."""
import csv
import glob
import json
import os
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PASSES = (
    "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum",
    "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum",
    "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT",
    "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU "
    "SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES",
    "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES",
)
# PMC_SET=mem: the memory pipeline (address translation, L1 -> L2 latency,
# TA/TD/TCP stalls, DRAM credit stalls)
MEM_PASSES = (
    "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum "
    "TCP_UTCL1_STALL_MULTI_MISS_sum",
    "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum "
    "TCP_PENDING_STALL_CYCLES_sum",
    "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TC_STALL_sum TD_TD_BUSY_sum "
    "TCP_TCR_TCP_STALL_CYCLES_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum "
    "TCP_UTCL1_THRASHING_STALL_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum",
    "TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum GRBM_GUI_ACTIVE",
)
if os.environ.get("PMC_SET") == "mem":
    PASSES = MEM_PASSES


def one(leg, env_extra, out):
    child = [sys.executable, os.path.join(REPO, "bench.py"), "--pmc-child", leg]
    env = dict(os.environ, TMPDIR="/tmp", **env_extra)
    vals, durs = {}, []
    for i, counters in enumerate(PASSES):
        d = os.path.join(out, f"p{i}")
        cmd = ["timeout", "-s", "KILL", "240", "rocprofv3", "--kernel-trace", "--pmc",
               *counters.split(), "--output-format", "csv", "-d", d, "-o", "run", "--", *child]
        r = subprocess.run(cmd, capture_output=True, text=True, cwd="/tmp", env=env, timeout=300)
        if r.returncode != 0:
            vals[f"pass{i}_error"] = r.stderr[-600:]
            print(f"pass {i} rc={r.returncode}", r.stderr[-600:], flush=True)
            continue
        per = {}
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(path) as f:
                for row in csv.DictReader(f):
                    if "k_tile<" not in row["Kernel_Name"]:
                        continue
                    key = (row["Dispatch_Id"], row["Counter_Name"])
                    per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
        by = {}
        for (_, c), v in per.items():
            by.setdefault(c, []).append(v)
        vals.update({c: sum(v) / len(v) for c, v in by.items()})
        for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            with open(path) as f:
                for row in csv.DictReader(f):
                    if "k_tile<" in row["Kernel_Name"]:
                        durs.append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
        shutil.rmtree(d, ignore_errors=True)
        print(f"pass {i} ok", flush=True)
    vals["avg_ms"] = sum(durs) / len(durs) / 1e6 if durs else None
    try:
        vals["read_bytes"] = (32 * vals["TCC_EA0_RDREQ_32B_sum"] + 64 * vals["TCC_EA0_RDREQ_64B_sum"]
                              + 128 * vals["TCC_EA0_RDREQ_128B_sum"])
        w64 = vals["TCC_EA0_WRREQ_64B_sum"]
        vals["write_bytes"] = 64 * w64 + 32 * (vals["TCC_EA0_WRREQ_sum"] - w64)
        vals["l2_hit"] = vals["TCC_HIT_sum"] / (vals["TCC_HIT_sum"] + vals["TCC_MISS_sum"])
    except KeyError:
        pass
    return vals


def main():
    out, leg = sys.argv[1], sys.argv[2]
    os.makedirs(out, exist_ok=True)
    res = {}
    for spec in sys.argv[3:]:
        name, _, envs = spec.partition("=")
        env = dict(e.split("=", 1) for e in envs.split(",") if e)
        tmp = tempfile.mkdtemp(prefix="pmcab_", dir="/tmp")
        res[name] = {"env": env, **one(leg, env, tmp)}
        print(name, json.dumps(res[name]), flush=True)
        with open(os.path.join(out, f"pmc_{leg}.json"), "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
