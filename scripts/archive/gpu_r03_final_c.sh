#!/bin/bash
# Round-3 closing check on the committed tree: the whole -m gpu suite, then
# __graft_entry__.smoke() as the driver calls it.
set -o pipefail
tag=${1:-r03fc}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 1200 --timeout-method thread \
    > $out/gpu_tests.txt 2>&1
rc=$?
echo "pytest rc=$rc" >> $out/gpu_tests.txt
tail -2 $out/gpu_tests.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > $out/smoke.txt 2>&1
rc=$?
cat $out/smoke.txt | tail -3
exit $rc
