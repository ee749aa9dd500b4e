#!/bin/bash
# Round-3 GPU check: the -m gpu suite, then a short bench.py run.  Each GPU
# step has its own time limit; a fault/abort/timeout stops the script.
set -o pipefail
tag=${1:-r03a}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 ${TEST_LIMIT:-660} python -u -m pytest tests -m gpu -x -v --timeout 900 \
    --timeout-method thread ${TEST_K:+-k "$TEST_K"} > $out/gpu_tests.txt 2>&1
rc=$?
echo "pytest rc=$rc" >> $out/gpu_tests.txt
tail -3 $out/gpu_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
[ -n "$NO_BENCH" ] && exit $rc
timeout -k 10 ${BENCH_LIMIT:-480} python -u bench.py --steps ${STEPS:-3} --warmup 1 \
    --kernel-steps 10 $BENCH_ARGS > $out/bench.json 2> $out/bench.err
brc=$?
echo "bench rc=$brc"
tail -5 $out/bench.err
exit $(( rc > brc ? rc : brc ))
