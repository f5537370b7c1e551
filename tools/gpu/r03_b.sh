#!/bin/bash
# round 3: host facts, the whole -m gpu suite, then the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
{ echo "nproc $(nproc)"; python3 -c 'import os; print("affinity", len(os.sched_getaffinity(0)))';
  cat /proc/self/cgroup; cat /sys/fs/cgroup$(cut -d: -f3 /proc/self/cgroup | head -1)/cpu.max 2>/dev/null; } > gpurun_out/r03_host.txt 2>&1
timeout -k 10 700 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r03_gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r03_gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 420 python3 bench.py > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err
