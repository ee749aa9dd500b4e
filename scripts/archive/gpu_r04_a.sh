#!/bin/bash
# Round-4 box check: the bench launcher tests, the kent rebind case, the
# host-range validation, axtChain -nranks, the full-scale C5 / C4 goldens,
# smoke; then axtChain on C4 with stage timings.
set -o pipefail
tag=${1:-r04a}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
(while sleep 50; do date +%T >> $out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
nproc > $out/host.txt; grep -m1 "model name" /proc/cpuinfo >> $out/host.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_bench.py \
    "tests/test_gpu_scoring.py::test_kent_shims_vs_reference" \
    "tests/test_gpu_scoring.py::test_host_ranges_and_reupload" \
    "tests/test_gpu_tools.py::test_axtchain_synth_ranks" \
    "tests/test_gpu_configs.py::test_c5_fullscale_vs_reference_sha" \
    "tests/test_gpu_configs.py::test_c4_fullscale_axtchain_vs_reference_sha" \
    --durations=20 > $out/gpu_tests.txt 2>&1 || exit $?
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || exit $?
d=/tmp/c4_50m
timeout -k 10 120 genomealignmenttools_amd/libexec/gac_synth c4 $d -blocks=50000000 -threads=16 || exit $?
GAC_TIMING=1 timeout -k 10 300 genomealignmenttools_amd/bin/axtChain -linearGap=loose -verbose=2 -psl \
    $d/in.psl $d/t.2bit $d/q.2bit $d/ours.chain 2> $out/c4_ours.err || exit $?
echo ok
