"""Order / pause sensitivity of the host-trace measurement (why bench.py's pipelined run, right after the
resident one, is slower than the same mode in a fresh process): runs the headline ShardBench timed regions
in the given order, optionally pausing between them, and prints ms per shard and the mean proof-call time.
python tools/h2d_order.py <mode,mode,...> [pause_s] [steps] [warm-up modes, default resident,pipelined]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    modes = sys.argv[1].split(",")
    pause = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    warm = sys.argv[4].split(",") if len(sys.argv) > 4 else ["resident", "pipelined"]
    args = argparse.Namespace(gpus=None, queries=84, h2d_dst="torch", inflight=3)
    rk = bench.Ranks(args)
    sb = bench.ShardBench(args, rk, "fib", 1 << 22, 3)
    for m in warm:
        sb.run_steps(2 if m == "resident" else 1, m)
    for i, m in enumerate(modes):
        if i and pause:
            time.sleep(pause)
        _, el = sb.timed(steps, m)
        calls = [t for (mm, _), v in sb.slot_proof_s.items() if mm == m for t in v]
        print(f"{m}: {1e3 * el / (3 * steps):.3f} ms per shard, proof calls {1e3 * sum(calls) / len(calls):.2f} ms "
              f"mean (pause {pause} s before; warm-up {warm})", flush=True)


if __name__ == "__main__":
    main()
