#!/bin/bash
# C5 at --chains (default 5e6): ours only (scoreChain + chainNet -rescore),
# twice, with the per-stage times; the reference side is in
# scripts/archive/gpu_big_configs.sh (its outputs' checksums are compared here
# against the committed reference-checked run when given).
set -o pipefail
TAG=${1:-c5ours}; CH=${2:-5000000}
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
(while sleep 50; do date +%T >> $OUT/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for i in 1 2; do
  timeout -k 10 900 python scripts/bench_tools.py c5 --chains $CH --seed 1234 --no-ref > $OUT/c5.$i.json 2> $OUT/c5.$i.err || { echo failed; tail $OUT/c5.$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print({k: d[k] for k in ('ours_scorechain_s','ours_chainnet_s','ours_s')})" $OUT/c5.$i.json
done
D=/tmp/c5_${CH}_1234
sha256sum $D/ours.sc.chain $D/ours.t.net $D/ours.q.net | tee $OUT/sha.txt
