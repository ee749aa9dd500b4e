#!/bin/bash
# rocprofv3 --kernel-trace --stats over a short bench.py run (kernel legs
# in-process; the headline's chainNet children traced too).
set -o pipefail
tag=${1:-r03e}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 ${PROF_LIMIT:-400} rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof \
    -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --kernel-steps 10 --no-c2 \
    --no-cpu-baseline --no-pmc > $GRAFT_REPO_ROOT/$out/prof_bench.json 2> $GRAFT_REPO_ROOT/$out/prof_bench.err
rc=$?
echo "prof rc=$rc"
exit $rc
