"""Experiment: does the destination memory type of a concurrent H2D stream change how much it slows the
prover?  Serial resident FibCpu 2^22 proofs alone, then with a background thread copying a 1.1 GB
pinned host buffer nonstop into (a) ordinary device memory, (b) hipDeviceMallocUncached memory,
(c) hipDeviceMallocFinegrained memory.  Hypothesis: PCIe writes streaming through the Infinity Cache
evict the LDE's column batches (they rely on staying MALL-resident between passes)."""
import ctypes as C
import os
import sys
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import bench  # noqa: E402
from zkmips_amd import workloads as W  # noqa: E402
from zkmips_amd._lib import Device  # noqa: E402
from zkmips_amd.prover import HipProver  # noqa: E402

hip = C.CDLL("libamdhip64.so")
hip.hipExtMallocWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
hip.hipStreamSynchronize.argtypes = [C.c_void_p]
hip.hipFree.argtypes = [C.c_void_p]

m, prep, tr, pv = W.fib_shard(1 << 22, 1000)
dev = Device(0)
pr = HipProver(dev, m, prep, num_queries=84)
dt = {k: torch.from_numpy(v.view(np.int32)).cuda() for k, v in tr.items()}
nbytes = (1 << 22) * 67 * 4
host = torch.empty(nbytes // 4, dtype=torch.int32, pin_memory=True)
host.numpy()[...] = 1


def timeit(n=6):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        bench.prove_resident(pr, dt, pv)
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


for _ in range(2):
    bench.prove_resident(pr, dt, pv)
print(f"alone: {timeit():.2f} ms", flush=True)
for name, flags in (("default", None), ("uncached", 0x3), ("finegrained", 0x1)):
    if flags is None:
        buf = torch.empty_like(host, device="cuda")
        dst = buf.data_ptr()
    else:
        p = C.c_void_p()
        rc = hip.hipExtMallocWithFlags(C.byref(p), nbytes, flags)
        if rc != 0:
            print(f"{name}: hipExtMallocWithFlags failed ({rc})", flush=True)
            continue
        dst = p.value
    stop = [False]
    ncopies = [0]

    def bg():
        s = torch.cuda.Stream()
        while not stop[0]:
            hip.hipMemcpyAsync(dst, host.data_ptr(), nbytes, 1, s.cuda_stream)
            hip.hipStreamSynchronize(s.cuda_stream)
            ncopies[0] += 1
    th = threading.Thread(target=bg)
    th.start()
    time.sleep(0.3)
    t0, c0 = time.perf_counter(), ncopies[0]
    b = timeit()
    rate = (ncopies[0] - c0) * nbytes / (time.perf_counter() - t0) / 1e9
    stop[0] = True
    th.join()
    print(f"{name}: {b:.2f} ms with background H2D ({rate:.1f} GB/s)", flush=True)
    if flags is not None:
        hip.hipFree(dst)
