#!/bin/bash
# Round-4 probe: C4 axtChain with the largest team at 8 (default split), 9
# and 10 threads (the second team and the pool take the rest).
set -o pipefail
tag=${1:-r04k}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
(while sleep 50; do date +%T >> $out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
P=genomealignmenttools_amd
c=/tmp/c4_50m
timeout -k 10 120 $P/libexec/gac_synth c4 $c -blocks=50000000 -threads=16 || exit $?
run() {
  local name=$1; shift
  rm -f $c/ours.chain
  s=$(date +%s.%N)
  env "$@" GAC_TIMING=1 timeout -k 10 300 $P/bin/axtChain -linearGap=loose -verbose=2 -psl \
      $c/in.psl $c/t.2bit $c/q.2bit $c/ours.chain 2> $out/c4_$name.err || return $?
  e=$(date +%s.%N)
  python3 -c "print('$name wall', round($e - $s, 3))" >> $out/times.txt
  sha256sum $c/ours.chain >> $out/times.txt
}
for i in 1 2; do
  run default_$i GAC_X=1 || exit $?
  run t9_$i GAC_DP_TEAM0=9 || exit $?
  run t10_$i GAC_DP_TEAM0=10 || exit $?
done
echo ok
