"""Upload-kernel timing probe (GPU box only): the C5 chain set uploaded three
times with the scoring set first (k_chain_prep, k_tile_chain,
k_build_flat<true>), no scoring call.  Run under rocprofv3 --kernel-trace
--stats; GAC_LIB_VARIANT picks a probe build (GAC_UP_PROBE bits)."""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.getcwd()))
sys.argv = ["bench.py"]
import bench  # noqa: E402
from genomealignmenttools_amd.gachain import GAC_Q, GAC_T, Engine, GapCosts  # noqa: E402

args = bench.parse()
d, _ = bench.c5_files(args)
ch = bench.load_chains_bin(d)
e = Engine(0)
e.load_2bit(GAC_T, os.path.join(d, "t.2bit"))
e.load_2bit(GAC_Q, os.path.join(d, "q.2bit"))
e.set_scoring(bench.BLASTZ, GapCosts("loose"))
names = lambda path: [ln.split()[0] for ln in open(path) if ln.strip()]
tmap = bench.np.array([e.seq_index(GAC_T, x) for x in names(os.path.join(d, "t.sizes"))], "int32")
qmap = bench.np.array([e.seq_index(GAC_Q, x) for x in names(os.path.join(d, "q.sizes"))], "int32")
for _ in range(3):
    cs = e.upload_chain_arrays(tmap[ch["tseq"]], qmap[ch["qseq"]], ch["strand"], ch["off"], ch["bt"],
                               ch["bq"], ch["bs"])
print("ok", ch["n"], ch["nb"])
