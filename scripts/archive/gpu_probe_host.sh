#!/bin/bash
# Host topology of the GPU box: CPU model, cores, NUMA nodes, the GPU's NUMA node, shared memory, memory.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/probe
mkdir -p $O
{
  echo "== nproc"; nproc
  echo "== lscpu"; lscpu
  echo "== numa nodes"; ls /sys/devices/system/node/ | grep node
  for n in /sys/devices/system/node/node*; do echo "$n cpus=$(cat $n/cpulist) mem=$(grep MemTotal $n/meminfo)"; done
  echo "== gpu pci numa"
  for d in /sys/class/drm/card*/device; do echo "$d $(cat $d/numa_node 2>/dev/null) $(basename $(readlink -f $d))"; done
  echo "== affinity"; taskset -p $$ || true
  echo "== shm"; df -h /dev/shm
  echo "== mem"; free -g
  echo "== ulimit"; ulimit -a
  echo "== cgroup"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /sys/fs/cgroup/memory.max 2>/dev/null
  echo "== zlib"; ls /usr/lib/x86_64-linux-gnu/libz* /usr/include/zlib.h 2>&1
  echo "== numactl"; which numactl; ls /usr/include/numa.h /usr/lib/x86_64-linux-gnu/libnuma* 2>&1
  echo "== gcc native"; gcc -march=native -Q --help=target 2>/dev/null | grep -E "march=|mavx512f|msse4.2|mpclmul|mvpclmul" | head
} > $O/host.txt 2>&1
cat $O/host.txt | head -120
