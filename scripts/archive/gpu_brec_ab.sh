#!/bin/bash
# Planner bucket records (BucketRec) on/off: scoring parity tests, then the
# kernel leg (bench.py --workload rescore) alternated, 3 rounds, with k_plan
# timed by HIP events (--prof all).
set -o pipefail
TAG=${1:-brec}
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_scoring.py tests/test_gpu_tools.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2 3; do
  for m in on off; do
    if [ $m = on ]; then E=""; else E="GAC_BREC_MAX_MB=0"; fi
    env $E timeout -k 10 300 python bench.py --workload rescore --kernel-steps 50 --no-cpu-baseline --no-pmc --prof all > $OUT/k.$m.$round.json 2> $OUT/k.$m.$round.err || { echo "bench $m failed"; tail $OUT/k.$m.$round.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernel']; print('$m', $round, round(k['ms_per_step']*1e3,1), 'us/step', {a: round(b*1e3,1) for a,b in k['kernel_ms'].items()})" $OUT/k.$m.$round.json
  done
done
