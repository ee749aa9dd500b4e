#!/bin/bash
# bin/chainNet -rescore on C2 under several environments, interleaved (one
# run of each per round, 6 rounds): wall time per run and the device laps.
# usage: bash scripts/archive/gpu_e2e_ab.sh TAG "NAME:ENV=V,ENV=V" ...
set -o pipefail
TAG=${1:-ab}; shift
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --gen-only --tmp /tmp > $OUT/gen.log 2>&1 || exit 1
D=/tmp/gac_bench_c2_200000_42
for round in $(seq 1 ${ROUNDS:-6}); do
  for spec in "$@"; do
    name=${spec%%:*}; envs=$(echo "${spec#*:}" | tr ',' ' ')
    t0=$(date +%s%N)
    env GAC_TIMING=1 $envs timeout -k 10 120 genomealignmenttools_amd/bin/chainNet $D/in.chain $D/t.sizes $D/q.sizes /tmp/ab.t.net /tmp/ab.q.net \
      -rescore -tNibDir=$D/t.2bit -qNibDir=$D/q.2bit -linearGap=loose -verbose=2 > $OUT/$name.$round.log 2>&1 || { echo "$name failed"; tail $OUT/$name.$round.log; exit 1; }
    t1=$(date +%s%N)
    echo "$name $round $(( (t1 - t0) / 1000000 ))" >> $OUT/wall.txt
  done
done
python3 - "$OUT" <<'PY'
import collections, sys, statistics
w = collections.defaultdict(list)
for line in open(sys.argv[1] + "/wall.txt"):
    n, _, ms = line.split(); w[n].append(int(ms))
for n, v in w.items():
    print(f"{n}: median {statistics.median(v)} ms  runs {v}")
PY
grep -h "overlapped\|fill list" $OUT/*.2.log
