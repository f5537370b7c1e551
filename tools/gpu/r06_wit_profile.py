"""Where a compress node's witness time goes (config 5's critical path): cProfile of node_witness for a layer-1
node (two MIPS leaves) and a layer-2 node (two compress proofs), each on a warm template, plus the shared-memory
hand-over.  python tools/gpu/r06_wit_profile.py [leaf_log]"""
import cProfile
import io
import os
import pstats
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def prof(label, fn):
    pr = cProfile.Profile()
    t = time.perf_counter()
    pr.enable()
    out = fn()
    pr.disable()
    dt = time.perf_counter() - t
    s = io.StringIO()
    st = pstats.Stats(pr, stream=s)
    st.sort_stats("cumulative").print_stats(28)
    st.sort_stats("tottime").print_stats(22)
    print(f"==== {label}: {dt:.3f} s (times {out[4] if isinstance(out, tuple) and len(out) == 5 else ''})")
    print(s.getvalue(), flush=True)
    return out


def main():
    leaf_log = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    import bench
    from zkmips_amd import compress_tree as CT
    d = tempfile.mkdtemp(prefix="zkm_wp_", dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
    try:
        meta, info, gen_s = bench._compress_leaves_job(d, 8, 22 - leaf_log)
        run = bench._load_tendermint(d, meta)
    finally:
        shutil.rmtree(d, ignore_errors=True)
    print(f"leaves generated in {gen_s:.1f} s", flush=True)
    import torch
    torch.cuda.init()  # torch's HIP context before the prover library's (as bench.py orders them)
    from zkmips_amd._lib import Device
    dev = Device(0)
    leaves, _ = bench.mips_leaves(dev, 84, run, info)
    provers, stats = CT.GpuProvers(dev), CT.TreeStats()

    def witness(ch, **fl):
        return CT.node_witness(ch, True, True, True, False, **fl)

    def prove(w):
        pr = provers.get(w[0], stats)
        return CT.compress_child_vk(pr.vk_commit, w[3]), pr.prove_shard(CT.materialize(w[1]), w[2])

    t = time.perf_counter()
    w0 = witness(leaves[0:2], is_first=True)
    print(f"layer 1 first node (template build): {time.perf_counter() - t:.3f} s {w0[4]}", flush=True)
    w1 = prof("layer 1 node on the template", lambda: witness(leaves[2:4]))
    t = time.perf_counter()
    packed = CT.shm_pack(w1)
    t1 = time.perf_counter()
    CT.register_prep(CT.shm_unpack(packed))
    print(f"shm_pack {t1 - t:.3f} s, unpack + register {time.perf_counter() - t1:.3f} s", flush=True)
    n = [prove(w0), prove(w1), prove(witness(leaves[4:6])), prove(witness(leaves[6:8]))]
    t = time.perf_counter()
    w = witness(n[0:2], is_first=True)
    print(f"layer 2 first node (template build): {time.perf_counter() - t:.3f} s {w[4]}", flush=True)
    prof("layer 2 node on the template", lambda: witness(n[2:4]))
    prof("layer 2 node on the template (again)", lambda: witness(n[2:4]))


if __name__ == "__main__":
    main()
