#!/bin/bash
# Round-4: axtChain C4 (50 M blocks) team-DP variants on the box: default
# teams pinned to an L3 domain or not, applier on or off.
set -o pipefail
tag=${1:-r04g}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
(while sleep 50; do date +%T >> $out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
d=/tmp/c4_50m
timeout -k 10 120 genomealignmenttools_amd/libexec/gac_synth c4 $d -blocks=50000000 -threads=16 || exit $?
run() {
  local name=$1; shift
  rm -f $d/ours.chain
  s=$(date +%s.%N)
  env "$@" GAC_TIMING=1 timeout -k 10 300 genomealignmenttools_amd/bin/axtChain -linearGap=loose -verbose=2 -psl \
      $d/in.psl $d/t.2bit $d/q.2bit $d/ours.chain 2> $out/c4_$name.err || return $?
  e=$(date +%s.%N)
  python3 -c "print('$name wall', $e - $s)" >> $out/c4_times.txt
  sha256sum $d/ours.chain >> $out/c4_times.txt
}
run pin_apply GAC_X=1 || exit $?
run pin_noapply GAC_DP_APPLY=0 || exit $?
run nopin_apply GAC_DP_PIN=0 || exit $?
run nopin_noapply GAC_DP_PIN=0 GAC_DP_APPLY=0 || exit $?
run pin_apply2 GAC_X=1 || exit $?
run pin_noapply2 GAC_DP_APPLY=0 || exit $?
echo ok
