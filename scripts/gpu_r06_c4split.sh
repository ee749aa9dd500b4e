#!/bin/bash
# C4 (axtChain -psl, 50 M blocks): the hybrid DP's device share A/B --
# host only, the default cap, and larger caps -- alternating, REPS rounds;
# wall time, the split line and the output's sha256 per run.
set -o pipefail
out=gpurun_out/${1:-r06split}
mkdir -p $out
export TMPDIR=/tmp
S=genomealignmenttools_amd/libexec/gac_synth
B=$GRAFT_REPO_ROOT/genomealignmenttools_amd/bin
d=/tmp/c4s
$S c4 $d -seed=7 -blocks=50000000 -threads=16 > /dev/null || exit 1
for i in $(seq 1 ${REPS:-2}); do
  for mode in ${MODES:-host default 50000 200000}; do
    case $mode in
      host) env="GAC_AXT_DP=host" ;;
      default) env="" ;;
      gpu) env="GAC_AXT_DP=gpu" ;;
      tt0) env="GAC_DP_TEAMTREE=0" ;;
      early0) env="GAC_AXT_SCORE_EARLY=0" ;;
      hosttt) env="GAC_DP_GPU_MAX=0" ;;
      dt0_*) env="GAC_DP_DEVTREE=0 GAC_DP_GPU_MAX=${mode#dt0_}" ;;
      us*_*) u=${mode%%_*}; env="GAC_DP_DEV_US=${u#us} GAC_DP_GPU_MAX=${mode#*_}" ;;
      *) env="GAC_DP_GPU_MAX=$mode" ;;
    esac
    t0=$(date +%s%N)
    ( cd $d && env $env GAC_TIMING=1 timeout -k 10 200 $B/axtChain -linearGap=loose -psl in.psl \
        t.2bit q.2bit o.chain ) > $out/${mode}_$i.err 2>&1 || exit $?
    ms=$(( ($(date +%s%N) - t0) / 1000000 ))
    sha=$(sha256sum $d/o.chain | cut -c1-16)
    split=$(grep -o "hybrid DP: [^)]*)" $out/${mode}_$i.err | head -1)
    dev=$(grep -o "device's [0-9]* pairs took [0-9.]* s" $out/${mode}_$i.err | head -1)
    split="$split $dev"
    echo "$mode rep $i: wall $ms ms sha $sha $split" | tee -a $out/summary.txt
    rm -f $d/o.chain
  done
done
rm -rf $d
echo ok
