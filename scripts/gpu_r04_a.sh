#!/bin/bash
# Round-4 first box check: the bench launcher tests, smoke, and axtChain on
# the C4 shape of SURVEY §8(d) (gac_synth c4: 24 x 21 pairs x 2 strands,
# 50 M PSL blocks) with stage timings and the output's sha256.
set -o pipefail
tag=${1:-r04a}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
(while sleep 50; do date +%T >> $out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_bench.py "tests/test_gpu_scoring.py::test_kent_shims_vs_reference" \
    > $out/gpu_bench_tests.txt 2>&1 || exit $?
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || exit $?
d=/tmp/c4_50m
timeout -k 10 120 genomealignmenttools_amd/libexec/gac_synth c4 $d -blocks=50000000 -threads=16 || exit $?
cat $d/info.json > $out/c4_info.json
nproc > $out/host.txt; grep -m1 "model name" /proc/cpuinfo >> $out/host.txt
for i in 1 2; do
  rm -f $d/ours.chain
  s=$(date +%s.%N)
  GAC_TIMING=1 timeout -k 10 300 genomealignmenttools_amd/bin/axtChain -linearGap=loose -verbose=0 -psl \
      $d/in.psl $d/t.2bit $d/q.2bit $d/ours.chain 2> $out/c4_ours_$i.err || exit $?
  e=$(date +%s.%N)
  python3 -c "print('run $i wall', $e - $s)" >> $out/c4_times.txt
done
sha256sum $d/ours.chain $d/in.psl > $out/c4_sha.txt
echo ok
