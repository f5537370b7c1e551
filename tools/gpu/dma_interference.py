"""Does a concurrent PCIe H2D stream slow the prover's kernels?  Single-shard resident proofs
timed alone, then with a background thread copying 1.1 GB pinned host buffers to HBM nonstop."""
import os, sys, threading, time
import numpy as np
import torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import bench
from zkmips_amd import workloads as W
from zkmips_amd._lib import Device
from zkmips_amd.prover import HipProver

m, prep, tr, pv = W.fib_shard(1 << 22, 1000)
dev = Device(0)
pr = HipProver(dev, m, prep, num_queries=84)
dt = {k: torch.from_numpy(v.view(np.int32)).cuda() for k, v in tr.items()}
host = torch.empty((1 << 22) * 67, dtype=torch.int32, pin_memory=True)
dst = torch.empty_like(host, device="cuda")
stop = False
ncopies = [0]
def bg():
    s = torch.cuda.Stream()
    while not stop:
        with torch.cuda.stream(s):
            dst.copy_(host, non_blocking=True)
        s.synchronize()
        ncopies[0] += 1
for _ in range(2):
    bench.prove_resident(pr, dt, pv)
def timeit(n=6):
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(n):
        bench.prove_resident(pr, dt, pv)
    torch.cuda.synchronize(); return (time.perf_counter() - t) / n * 1e3
a = timeit()
th = threading.Thread(target=bg); th.start(); time.sleep(0.2)
t0 = time.perf_counter(); c0 = ncopies[0]
b = timeit()
rate = (ncopies[0] - c0) * host.numel() * 4 / (time.perf_counter() - t0) / 1e9
stop = True; th.join()
print(f"serial resident proof: {a:.2f} ms alone, {b:.2f} ms with background H2D ({rate:.1f} GB/s achieved meanwhile)")
