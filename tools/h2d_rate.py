"""H2D ceiling of the host-trace mode: page-locked host -> HBM copy rate of one FibCpu 2^22 shard's trace bytes
(1.127 GB), with no proving, as (a) one copy on one stream, (b) the shard's per-chip copies, (c) the bytes split
over 2 and 3 streams, (d) 3 slots each copying a whole shard at once (the pipelined bench's worst case).
python tools/h2d_rate.py [total_MB]"""
import sys
import time

import torch


def rate(fn, nbytes, reps=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return nbytes * reps / (time.perf_counter() - t) / 1e9


def main():
    total = int(float(sys.argv[1]) * (1 << 20)) if len(sys.argv) > 1 else 1127219200
    n = total // 4
    host = torch.empty(n, dtype=torch.int32, pin_memory=True)
    host.fill_(7)
    dev = torch.empty(n, dtype=torch.int32, device="cuda")
    streams = [torch.cuda.Stream() for _ in range(3)]
    print(f"bytes {total}", flush=True)

    def one():
        with torch.cuda.stream(streams[0]):
            dev.copy_(host, non_blocking=True)
    print(f"one copy, one stream      {rate(one, total):7.2f} GB/s", flush=True)

    for k in (2, 3):
        parts = [(i * n // k, (i + 1) * n // k) for i in range(k)]

        def split():
            for s, (a, b) in zip(streams, parts):
                with torch.cuda.stream(s):
                    dev[a:b].copy_(host[a:b], non_blocking=True)
        print(f"split over {k} streams      {rate(split, total):7.2f} GB/s", flush=True)

    chunks = [(i * n // 16, (i + 1) * n // 16) for i in range(16)]

    def chunked():
        with torch.cuda.stream(streams[0]):
            for a, b in chunks:
                dev[a:b].copy_(host[a:b], non_blocking=True)
    print(f"16 chunks, one stream     {rate(chunked, total):7.2f} GB/s", flush=True)

    hosts = [host] + [torch.empty(n, dtype=torch.int32, pin_memory=True) for _ in range(2)]
    devs = [dev] + [torch.empty(n, dtype=torch.int32, device="cuda") for _ in range(2)]

    def slots():
        for s, h, d in zip(streams, hosts, devs):
            with torch.cuda.stream(s):
                d.copy_(h, non_blocking=True)
    print(f"3 slots x one shard       {rate(slots, 3 * total, reps=3):7.2f} GB/s", flush=True)

    # while kernels keep the GPU busy: a device-side stream of HBM traffic on the default stream
    big = torch.empty(1 << 29, dtype=torch.int32, device="cuda")
    big2 = torch.empty_like(big)

    def busy_copy():
        for _ in range(6):
            big2.copy_(big)
        with torch.cuda.stream(streams[0]):
            dev.copy_(host, non_blocking=True)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(3):
        busy_copy()
    torch.cuda.synchronize()
    el = time.perf_counter() - t
    t = time.perf_counter()
    for _ in range(3):
        for _ in range(6):
            big2.copy_(big)
    torch.cuda.synchronize()
    el_k = time.perf_counter() - t
    print(f"D2D traffic alone {el_k * 1e3 / 3:.1f} ms per round, with the H2D beside it {el * 1e3 / 3:.1f} ms "
          f"(the H2D alone takes {total / rate(one, total, 2) / 1e6:.1f} ms)", flush=True)


if __name__ == "__main__":
    main()
