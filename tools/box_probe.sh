set -o pipefail
echo "nproc=$(nproc)"; python3 -c 'import os;print("affinity",len(os.sched_getaffinity(0)))'
cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /proc/self/status | grep -i cpus_allowed_list
lscpu | grep -E "Model name|Socket|Thread|Core" 
