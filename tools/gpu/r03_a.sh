#!/bin/bash
# round 3, first GPU pass: host facts, the whole -m gpu suite, the default bench line
set -eo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
{ echo "nproc $(nproc)"; python3 -c 'import os; print("affinity", len(os.sched_getaffinity(0)))';
  cat /proc/self/cgroup; cat /sys/fs/cgroup/cpu.max 2>/dev/null || true;
  cat /sys/fs/cgroup$(cut -d: -f3 /proc/self/cgroup | head -1)/cpu.max 2>/dev/null || true; } > gpurun_out/r03_host.txt 2>&1
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03_gpu_tests.log 2>&1
timeout -k 10 900 python3 bench.py > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err
