#!/bin/bash
# Round-4: upload-kernel A/B (lib variants: blocks per lane kUpPer 2 / 4 / 1),
# rocprofv3 --kernel-trace --stats over a short kernel-leg bench run each.
set -o pipefail
tag=${1:-r04upab}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
(while sleep 50; do date +%T >> $out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for v in base up4 up1; do
  if [ $v = base ]; then unset GAC_LIB_VARIANT; else export GAC_LIB_VARIANT=$v; fi
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof_$v \
      -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --kernel-steps 2 --no-c2 \
      --no-cpu-baseline --no-pmc --no-c4 > $GRAFT_REPO_ROOT/$out/bench_$v.json \
      2> $GRAFT_REPO_ROOT/$out/bench_$v.err) || exit $?
done
echo ok
