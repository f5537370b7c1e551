"""H2D attribution: run the headline ShardBench in ONE mode (pipelined = host traces with the look-ahead
DMA, resident = traces in HBM) for a few steps, so that a rocprofv3 kernel trace of each mode can be
compared kernel by kernel (tools/kdelta.py).
python tools/h2d_attrib.py {pipelined|resident|per_call} [steps] [log_n] [in_flight]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    mode = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    log_n = int(sys.argv[3]) if len(sys.argv) > 3 else 22
    k = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    args = argparse.Namespace(gpus=None, queries=84, h2d_dst="torch", inflight=k)
    rk = bench.Ranks(args)
    sb = bench.ShardBench(args, rk, "fib", 1 << log_n, k)
    sb.run_steps(1, mode)
    _, el = sb.timed(steps, mode)
    waits = {k: [round(1e3 * w, 1) for w in v] for k, v in sorted(sb.slot_waits.items())}
    calls = [t for (m, _), v in sb.slot_proof_s.items() if m == mode for t in v]
    if calls:
        print(f"{mode}: zkm_prove_shard calls {1e3 * sum(calls) / len(calls):.2f} ms mean, "
              f"{1e3 * min(calls):.2f} min, {1e3 * max(calls):.2f} max", flush=True)
    print(f"{mode}: {1e3 * el / (k * steps):.3f} ms per shard ({steps} steps x {k} in flight)"
          + (f"; copy waits per slot and step (ms): {waits}" if mode == "pipelined" else ""), flush=True)
    time.sleep(0.1)


if __name__ == "__main__":
    main()
