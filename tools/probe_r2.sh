set -o pipefail
mkdir -p gpurun_out/probe
{ nproc; python3 -c 'import os;print("affinity",len(os.sched_getaffinity(0)),"cpu_count",os.cpu_count())'; cat /sys/fs/cgroup/cpu.max 2>/dev/null || echo nocpumax; lscpu | grep -E "Model name|^CPU\(s\)|Socket|Thread" ; env | grep -E "OMP|MAX_JOBS" ; } > gpurun_out/probe/sys.txt 2>&1
timeout -k 10 120 python3 bench.py --steps 10 --warmup 3 --no-cpu --streams 1 > gpurun_out/probe/b_s1.json 2> gpurun_out/probe/b_s1.err &&
timeout -k 10 120 python3 bench.py --steps 10 --warmup 3 --no-cpu --streams 2 > gpurun_out/probe/b_s2.json 2> gpurun_out/probe/b_s2.err
