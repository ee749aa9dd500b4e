#!/bin/bash
# Box CPU topology for thread placement: the allowed CPUs, their L3 domains.
set -o pipefail
out=gpurun_out/${1:-r04topo}
mkdir -p $out
{
  nproc; lscpu 2>/dev/null | head -30
  python3 -c "import os; a=sorted(os.sched_getaffinity(0)); print('affinity', len(a), a)"
  for c in $(python3 -c "import os; print(' '.join(map(str, sorted(os.sched_getaffinity(0)))))"); do
    echo "cpu$c l3 $(cat /sys/devices/system/cpu/cpu$c/cache/index3/shared_cpu_list 2>/dev/null) core $(cat /sys/devices/system/cpu/cpu$c/topology/core_id 2>/dev/null) sib $(cat /sys/devices/system/cpu/cpu$c/topology/thread_siblings_list 2>/dev/null) node $(ls -d /sys/devices/system/cpu/cpu$c/node* 2>/dev/null | xargs -n1 basename)"
  done
  cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null
  env | grep -E "OMP|MAX_JOBS|THREADS" 
} > $out/topo.txt 2>&1
echo ok
