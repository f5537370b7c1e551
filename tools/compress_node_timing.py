"""Serial timing of one compress-node proof over two MIPS leaves (config 5's layer-1 node): host traces vs
the Poseidon2WideDeg3 trace built on the device, with the per-stage profile of the device form.
python tools/compress_node_timing.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from zkmips_amd import compress_tree as CT
    from zkmips_amd._lib import Device
    dev = Device(0)
    leaves, info = bench.mips_leaves(dev, 84, n_leaves=2, distinct=2)
    import pickle
    for p2dev, compact in ((False, False), (True, False), (True, True)):
        t = time.perf_counter()
        wit = CT.node_witness(leaves, True, p2dev, compact, False)
        wit_s = time.perf_counter() - t
        prep, tr, pv, shape, times = wit
        mb = len(pickle.dumps(wit, protocol=pickle.HIGHEST_PROTOCOL)) / 1e6
        provers = CT.GpuProvers(dev)
        pr = provers.get(prep, CT.TreeStats())
        for _ in range(2):
            pr.prove_shard(CT.materialize(tr), pv)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(5):
            proof = pr.prove_shard(CT.materialize(tr), pv)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) / 5 * 1e3
        print(f"p2_on_device={p2dev} compact={compact}: witness {wit_s:.2f} s ({times}), {mb:.1f} MB pickled, "
              f"proof {ms:.2f} ms serial, "
              f"{len(proof)} bytes, max rows {max(v.shape[0] for v in CT.materialize(tr).values())}", flush=True)
    dt = CT.materialize(tr)  # the compact witness: every trace built on the device
    # the node program: a full build vs node_flat's template (verify_shard against a hint tape only)
    from zkmips_amd import recursion as R
    from zkmips_amd import recursion_verifier as RV
    children = [(CT.resolve_vk(vk), p) for vk, p in leaves]
    t = time.perf_counter()
    R.flatten(RV.compress_node_program(children))
    full_s = time.perf_counter() - t
    RV._TEMPLATES.clear()
    t = time.perf_counter()
    RV.node_flat(children)
    first_s = time.perf_counter() - t
    t = time.perf_counter()
    RV.node_flat(children)
    tpl_s = time.perf_counter() - t
    print(f"node program: full build + flatten {full_s:.3f} s, node_flat first {first_s:.3f} s, "
          f"node_flat from the template {tpl_s:.3f} s", flush=True)
    prof, serial_ms, text = bench.profile_proofs(pr, dt, pv, 3)
    print(f"all traces resident: {serial_ms:.2f} ms serial")
    for k, v in sorted(prof.items(), key=lambda kv: -kv[1][1]):
        if not k.endswith(("_perms", "_gfops")):
            print(f"   {k:24s} {v[1] / 3:8.3f} ms")


if __name__ == "__main__":
    main()
