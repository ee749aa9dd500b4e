#!/bin/bash
# TD/TA throughput probe (scripts/probes/td_rate.hip, built in-tree by
# hipcc into genomealignmenttools_amd/lib/probes/td_rate): timings, then one
# counter pass over the same run.
set -o pipefail
out=gpurun_out/${1:-r03t}
mkdir -p $out
bin=$GRAFT_REPO_ROOT/genomealignmenttools_amd/lib/probes/td_rate
timeout -k 10 120 $bin 64 > $out/td_rate.jsonl 2>&1 || exit $?
cat $out/td_rate.jsonl
cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TD_TD_BUSY_sum TA_TA_BUSY_sum \
    TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum --output-format csv \
    -d $GRAFT_REPO_ROOT/$out/pmc -o run -- $bin 16 > $GRAFT_REPO_ROOT/$out/pmc.log 2>&1 || exit $?
