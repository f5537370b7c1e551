"""Serial FibCpu 2^22 shard proofs (one in flight) for kernel timelines: python3 tools/gpu/prove_serial.py [n_proofs]"""
import sys
import time

sys.path.insert(0, __import__("os").environ.get("GRAFT_REPO_ROOT", "."))
from zkmips_amd import workloads as W  # noqa: E402
from zkmips_amd._lib import Device  # noqa: E402
from zkmips_amd.prover import HipProver  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
dev = Device(0)
m, prep, traces, pvs = W.fib_shard(1 << 22)
gpu = HipProver(dev, m, prep, num_queries=84)
for i in range(n):
    t = time.time()
    proof = gpu.prove_shard(traces, pvs)
    print(f"proof {i}: {len(proof)} bytes, {1e3 * (time.time() - t):.1f} ms host wall", flush=True)
