#!/bin/bash
# SURVEY §8(d) sizes on one MI355X: C5 at 5e6 chains (scoreChain + chainNet
# -rescore) or C4 at 5e7 PSL blocks (axtChain), ours vs the reference
# binaries on this host, outputs compared byte for byte.  A heartbeat file
# marks progress while the single-threaded reference runs.
# usage: bash scripts/archive/gpu_big_configs.sh TAG c5|c4
set -o pipefail
TAG=${1:-big}; WHAT=${2:-c5}
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
(while sleep 50; do date +%T >> $OUT/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
if [ "$WHAT" = c5 ]; then
  timeout -k 10 1100 python scripts/bench_tools.py c5 --chains 5000000 --seed 1234 > $OUT/c5.json 2> $OUT/c5.err
else
  timeout -k 10 1100 python scripts/bench_tools.py axtchain --blocks 50000000 --seed 7 > $OUT/c4.json 2> $OUT/c4.err
fi
rc=$?
echo "rc=$rc"
tail -5 $OUT/*.err
cat $OUT/*.json
exit $rc
