"""Throughput of K concurrent shard proofs (one host thread and HIP stream each) vs sequential."""
import sys, time, threading, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np
import torch
import bench
from zkmips_amd import workloads as W
from zkmips_amd._lib import Device
from zkmips_amd.prover import HipProver

n = 1 << 22
K = int(sys.argv[1]) if len(sys.argv) > 1 else 2
dev = Device(0)
shards = []
for k in range(K):
    m, prep, traces, pvs = W.fib_shard(n, seed=1000 + k)
    shards.append(({kk: torch.from_numpy(v.view(np.int32)).cuda() for kk, v in traces.items()}, pvs))
prover = HipProver(dev, m, prep, num_queries=84)
torch.cuda.synchronize()
ref = [bench.prove_resident(prover, t, p) for t, p in shards]
t0 = time.perf_counter()
for _ in range(3):
    for t, p in shards:
        bench.prove_resident(prover, t, p)
seq = (time.perf_counter() - t0) / (3 * K)
out = [None] * K
def work(k):
    for _ in range(3):
        out[k] = bench.prove_resident(prover, *shards[k])
t0 = time.perf_counter()
th = [threading.Thread(target=work, args=(k,)) for k in range(K)]
[t.start() for t in th]
[t.join() for t in th]
par = (time.perf_counter() - t0) / (3 * K)
print(f"K={K}: sequential {seq*1e3:.2f} ms/shard, concurrent {par*1e3:.2f} ms/shard, identical={out == ref}")
