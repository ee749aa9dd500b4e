set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_gpu_scoring.py -x -q -m gpu > gpurun_out/gpu2_tests.log 2>&1
echo "pytest rc=$?" >> gpurun_out/gpu2_tests.log
timeout -k 10 500 python bench.py --workload scorechain --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/gpu2_bench.json 2> gpurun_out/gpu2_bench.err || exit 1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload scorechain --steps 5 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/gpu2_prof.log 2>&1
echo "prof rc=$?" >> $GRAFT_REPO_ROOT/gpurun_out/gpu2_prof.log
