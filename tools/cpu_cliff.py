#!/usr/bin/env python3
"""Why the CPU baseline collapses above the box's CPU share.

Prints the box's CPU allotment as every interface shows it (affinity mask, cgroup v1 / v2 CPU quota, the
environment the pool sets) and times one 2^18-row FibCpu oracle proof at several OpenMP thread counts, each in
a fresh process (so OMP_WAIT_POLICY, read once by libgomp at start-up, takes effect), with the default
(spinning) wait policy and with PASSIVE.  CPU-only; run on the GPU box, where the share is enforced.
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def read(path):
    try:
        return open(path).read().strip()
    except OSError:
        return None


def allotment():
    cg = read("/proc/self/cgroup") or ""
    out = {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)), "proc_self_cgroup": cg.splitlines()[:6],
           "env": {k: os.environ.get(k) for k in ("OMP_NUM_THREADS", "MAX_JOBS", "CMAKE_BUILD_PARALLEL_LEVEL")}}
    for line in cg.splitlines():
        parts = line.split(":", 2)
        if len(parts) == 3:
            ctrl, path = parts[1], parts[2]
            if ctrl == "":  # v2
                out["v2_cpu.max"] = read(f"/sys/fs/cgroup{path}/cpu.max")
                out["v2_cpu.stat"] = (read(f"/sys/fs/cgroup{path}/cpu.stat") or "").splitlines()[:6]
            if "cpu" in ctrl.split(","):
                for base in ("/sys/fs/cgroup/cpu,cpuacct", "/sys/fs/cgroup/cpu"):
                    q = read(f"{base}{path}/cpu.cfs_quota_us")
                    if q is not None:
                        out["v1_cfs_quota_us"] = q
                        out["v1_cfs_period_us"] = read(f"{base}{path}/cpu.cfs_period_us")
                        out["v1_cpu.stat"] = (read(f"{base}{path}/cpu.stat") or "").splitlines()
                        break
    out["root_cpu.max"] = read("/sys/fs/cgroup/cpu.max")
    return out


CHILD = r"""
import sys, time
sys.path.insert(0, %r)
from tests import _oracle as O
from zkmips_amd import workloads as W
m, prep, tr, pv = W.fib_shard(1 << 18, seed=2)
pr = O.OracleProver(m, prep, num_queries=84)
pr.prove(tr, pv)
t = time.time()
rc, _ = pr.prove(tr, pv)
assert rc == 0
print(time.time() - t)
"""


def run(threads, policy):
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    if policy:
        env["OMP_WAIT_POLICY"] = policy
    t0 = time.time()
    try:
        r = subprocess.run([sys.executable, "-c", CHILD % ROOT], env=env, capture_output=True, text=True, timeout=150)
        return round(float(r.stdout.strip().splitlines()[-1]), 3) if r.returncode == 0 else f"rc {r.returncode}"
    except subprocess.TimeoutExpired:
        return f"> 150 s (wall {time.time() - t0:.0f})"


def main():
    print(json.dumps({"allotment": allotment()}, indent=1), flush=True)
    for policy in ("", "PASSIVE"):
        for th in (8, 16, 32, 64, 128):
            print(json.dumps({"policy": policy or "default(active spin)", "threads": th, "prove_2e18_s": run(th, policy)}),
                  flush=True)


if __name__ == "__main__":
    main()
