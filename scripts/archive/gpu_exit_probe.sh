#!/bin/bash
# Wall time of chainNet on C5 against the sum of its stage timers (the
# difference is process exit), with -rescore (HIP used) and without (host
# only).  r01: 0.26-0.28 s with HIP, 0.00-0.19 s without; a hipDeviceReset at
# context close did not change it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/exitp
: > gpurun_out/exitp/summary.txt
timeout -k 10 300 python scripts/bench_tools.py c5 --chains 1000000 --no-ref > gpurun_out/exitp/gen.json 2> gpurun_out/exitp/gen.log || exit 1
D=/tmp/c5_1000000_1234
for k in 1 2; do
  for v in rescore plain; do
    case $v in
      plain) E=""; R="";;
      rescore) E=""; R="-rescore -tNibDir=$D/t.2bit -qNibDir=$D/q.2bit -linearGap=loose";;
    esac
    rm -f /tmp/t.net /tmp/q.net
    s=$(date +%s.%N)
    env $E timeout -k 10 120 genomealignmenttools_amd/bin/chainNet $D/in.chain $D/t.sizes $D/q.sizes /tmp/t.net /tmp/q.net \
      $R -verbose=2 2> gpurun_out/exitp/$v$k.err || exit 1
    e=$(date +%s.%N)
    python3 -c "
s=sum(float(l.split()[-2]) for l in open('gpurun_out/exitp/$v$k.err') if '[stage]' in l and 'overlapped' not in l)
print('$v run $k wall %.3f stages %.3f gap %.3f' % ($e-$s, s, $e-$s-s))" | tee -a gpurun_out/exitp/summary.txt
  done
done
