cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/gr && timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py -x -v -m gpu -k "ranks" --timeout 600 --timeout-method thread > gpurun_out/gr/tests.log 2>&1; rc=$?; tail -4 gpurun_out/gr/tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/archive/gpu_bench_ranks.sh && bash scripts/archive/gpu_ranks_probe.sh ranks2 "1 2 4 8"
