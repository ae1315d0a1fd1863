cd $GRAFT_REPO_ROOT
for t in 8 16; do FPM_HOST_THREADS=$t timeout -k 5 60 ./build/pool_probe; FPM_HOST_THREADS=$t POOL_PROBE_HIP=1 timeout -k 5 60 ./build/pool_probe; done
nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null
