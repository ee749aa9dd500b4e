#!/bin/bash
# Round-4: k_build_flat cost breakdown -- the upload probe under rocprofv3
# --kernel-trace --stats with the default build and the GAC_UP_PROBE variants.
set -o pipefail
tag=${1:-r04upprobe}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
(while sleep 50; do date +%T >> $out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for v in base p1 p2 p4 p7; do
  if [ $v = base ]; then unset GAC_LIB_VARIANT; else export GAC_LIB_VARIANT=$v; fi
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof_$v \
      -o run -- python3 $GRAFT_REPO_ROOT/scripts/probes/upload_probe.py \
      > $GRAFT_REPO_ROOT/$out/probe_$v.txt 2>&1) || exit $?
done
echo ok
