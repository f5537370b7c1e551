#!/usr/bin/env python3
"""Benchmark: shard trace rows proved per second (BASELINE.json `metric`).

Workload (N = 1 unless --gpus): the S-SHARD synthetic shard of SURVEY.md §8d at 2^22 rows —
FibCpu (main 67 columns, 20 local lookups -> 11 EF LogUp columns, quotient degree 2, shaped like
the reference's Cpu chip) plus the preprocessed FibTable chip — proven end to end exactly as the
reference's CpuProver::commit + CpuProver::open would (LDE, Poseidon2 MMCS, LogUp trace, quotient,
openings, FRI with 84 queries and 16 PoW bits).  One step = one shard proof with the traces
already resident in HBM; for N > 1 every rank proves its own shard (shards are independent,
prove.rs:208-209) and the proof bytes are gathered over RCCL inside the timed region.

Also reported: the roofline of the dominant stage (HIP events on the launching stream over the
timed region), the PCIe-inclusive rate (host traces), and the CPU oracle on a bounded sample.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse_profile(text):
    out = {}
    for line in text.strip().splitlines():
        name, cnt, ms, units = line.split()
        out[name] = (int(cnt), float(ms), float(units))
    return out


def device_matrix(tensor, name, keep):
    from zkmips_amd._lib import Matrix, ZKM_REPR_CANONICAL
    nm = name.encode()
    keep.append(nm)
    return Matrix(nm, tensor.data_ptr(), tensor.shape[0], tensor.shape[1], ZKM_REPR_CANONICAL | 0x100)


def prove_resident(prover, dev_traces, pvs):
    """zkm_prove_shard over device-resident row-major traces (ZKM_MEM_DEVICE)."""
    from zkmips_amd._lib import Matrix, check, lib
    keep = []
    arr = (Matrix * len(dev_traces))(*[device_matrix(t, n, keep) for n, t in dev_traces.items()])
    base = prover.base_challenger()
    out = C.POINTER(C.c_uint8)()
    n = C.c_uint64()
    check(lib().zkm_prove_shard(prover.dev.h, prover.pk, arr, len(dev_traces), pvs.ctypes.data, pvs.size,
                                C.byref(base), C.byref(out), C.byref(n)), "zkm_prove_shard")
    b = C.string_at(out, n.value)
    lib().zkm_free_bytes(out)
    return b


STAGE_KERNEL = {"merkle_leaves": "k_hash_leaves", "merkle_nodes": "k_compress_level", "quotient": "zkm_quot_jit",
                "fri_reduce": "k_fri_reduce", "perm_trace": "zkm_perm_jit", "open_eval": "k_open_dot"}


def pmc_traffic(stage):
    """HBM bytes per launch of the stage's kernel from the newest committed rocprofv3 PMC summary
    (profiles/rNN_pmc_summary.json: 2 x FETCH_SIZE + WRITE_SIZE, gfx950 correction, tools/pmc_summary.py)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_summary.json")))
    k = STAGE_KERNEL.get(stage)
    if not files or not k:
        return None, None
    d = json.load(open(files[-1]))["kernels"].get(k, {})
    if "hbm_bytes_per_launch" not in d:
        return None, None
    return round(d["hbm_bytes_per_launch"]), os.path.basename(files[-1])


def measured_hbm(match):
    """HBM-bandwidth utilisation of a kernel family (BASELINE north star: NTT and quotient achieved
    HBM GB/s): PMC bytes (2 x FETCH_SIZE + WRITE_SIZE per launch, the gfx950 correction of
    tools/pmc_summary.py) over the kernels' measured durations, summed over every kernel whose name
    satisfies `match` in the committed rocprofv3 profile."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_summary.json")))
    if not files:
        return None
    byts = ms = 0.0
    for k, v in json.load(open(files[-1]))["kernels"].items():
        if match(k) and "hbm_bytes_per_launch" in v and "avg_ms" in v:
            byts += v["hbm_bytes_per_launch"] * v["calls"]
            ms += v["avg_ms"] * v["calls"]
    if not ms:
        return None
    gbps = byts / (ms / 1e3) / 1e9
    return {"GBps": round(gbps, 1), "frac": round(gbps / HBM_PEAK_GBS, 4), "source": os.path.basename(files[-1])}


def lde_measured_hbm():
    return measured_hbm(lambda k: "ntt" in k or "lde" in k)


VALU_PEAK_TSLOTS = 256 * 4 * 32 * 2.4e9 / 1e12  # CUs x SIMDs x SIMD-32 lanes x 2.4 GHz (MI355X_MICROARCH.md)


def valu_roofline(perms, ms):
    """Poseidon2 leaf hashing is integer-VALU bound: issue slots per permutation (static ISA count of
    the permutation weighted by the measured issue cost of each instruction class,
    profiles/rNN_isa_p2.json from tools/isa_slots.py) x permutations / measured stage time, against
    the architectural VALU issue rate."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_isa_p2.json")))
    if not files:
        return None
    slots = json.load(open(files[-1]))["issue_slots"]
    pps = perms / (ms / 1e3)
    achieved = pps * slots / 1e12
    return {"bound": "valu", "achieved": round(achieved, 2), "peak": round(VALU_PEAK_TSLOTS, 2),
            "unit": "T VALU issue slots/s", "frac": round(achieved / VALU_PEAK_TSLOTS, 4),
            "permutations_per_s": round(pps), "slots_per_permutation": slots,
            "source": os.path.basename(files[-1])}


def cpu_baseline(log_n, queries):
    """The CPU oracle (a C/OpenMP restatement, not the reference binary) on one bounded shard."""
    from tests import _oracle as O
    from zkmips_amd import workloads as W
    n = 1 << log_n
    m, prep, traces, pvs = W.fib_shard(n, seed=1)
    pr = O.OracleProver(m, prep, num_queries=queries)
    t0 = time.time()
    rc, proof = pr.prove(traces, pvs)
    dt = time.time() - t0
    assert rc == 0
    cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    return {"value": n / dt, "unit": "rows/s", "cores": cores, "kind": "port",
            "sample": f"one S-SHARD FibCpu 2^{log_n}-row shard (+FibTable), full commit+open, {queries} queries, "
                      f"{dt:.2f} s wall on {cores} OpenMP threads"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--log-n", type=int, default=22)
    ap.add_argument("--workload", choices=["fib", "alu", "core"], default="fib",
                    help="fib: S-SHARD FibCpu (the headline config); alu: MIPS ALU slice (AddSub, Bitwise, Lt, "
                         "ShiftLeft, ShiftRight, CloClz, Byte restated from the reference AIRs + CPU stand-in, "
                         "zkmips_amd/mips_alu.py), 2^(log-n) "
                         "instructions per shard; core: Cpu + Program + Mul + DivRem + Branch + Jump + MovCond + MemoryInstrs + MiscInstrs chips over the ALU slice "
                         "(zkmips_amd/mips_core.py) running a counted loop, Cpu 2^(log-n) rows")
    ap.add_argument("--queries", type=int, default=84)
    ap.add_argument("--cpu-log-n", type=int, default=18)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--profile-out", default="")
    ap.add_argument("--profile-steps", type=int, default=3, help="single-shard proofs in the profiled region")
    ap.add_argument("--inflight", type=int, default=3,
                    help="shards proven concurrently per GPU (one host thread + HIP stream each), as the "
                         "reference's prove_with_context runs commit/open for all shards of a batch at once")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    # ZKM_BENCH_REHEARSE=1: rehearse the N-rank flow on a box with fewer GPUs (ranks share the
    # cards, gloo instead of RCCL); never set by the driver, so the N-GPU bench is always RCCL
    rehearse = os.environ.get("ZKM_BENCH_REHEARSE") == "1"
    if rehearse:
        local_rank = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_rank)
    coll_dev = "cpu" if rehearse else "cuda"
    if world > 1:
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    from zkmips_amd import workloads as W
    from zkmips_amd._lib import Device, lib
    from zkmips_amd.prover import HipProver

    n = 1 << args.log_n
    K = max(1, args.inflight)
    shards = []
    core = None
    if args.workload == "core":  # one program (one proving key); its trace is generated once and proven K times
        from zkmips_amd import mips_core as MC
        core = MC.loop_shard(60, (3 * n // 4) // 104, seed=1)  # ~98 instructions per iteration
    for k in range(K):
        if core is not None:
            m, prep, traces_k, pvs_k = core
        elif args.workload == "alu":
            from zkmips_amd import mips_alu as A
            m, prep, traces_k, pvs_k = A.alu_shard(n // 4, n // 4, seed=1000 + rank * K + k, n_lt=n // 4,
                                                   n_sll=n // 8, n_sr=n // 16, n_clz=n // 16)
        else:
            m, prep, traces_k, pvs_k = W.fib_shard(n, seed=1000 + rank * K + k)
        shards.append(({kk: torch.from_numpy(v.view(np.int32)).cuda() for kk, v in traces_k.items()}, pvs_k, traces_k))
    dev = Device(local_rank)
    prover = HipProver(dev, m, prep, num_queries=args.queries)
    dev_traces, pvs, traces = shards[0]
    torch.cuda.synchronize()
    rows_per_shard = max(v.shape[0] for v in traces.values())

    def run_steps(nsteps):
        """nsteps shard proofs per in-flight slot; returns the last proof of slot 0."""
        if K == 1:
            proof = b""
            for _ in range(nsteps):
                proof = prove_resident(prover, dev_traces, pvs)
                gather(proof)
            return proof
        import threading
        out = [b""] * K
        def slot(k):
            for _ in range(nsteps):
                out[k] = prove_resident(prover, shards[k][0], shards[k][1])
        th = [threading.Thread(target=slot, args=(k,)) for k in range(K)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        gather(out[0])
        return out[0]

    def gather(proof):
        """MachineProof aggregation: all ranks' shard proofs over RCCL (zkmips_amd/dist.py)."""
        if world == 1:
            return {0: proof}
        from zkmips_amd.dist import gather_proofs
        return gather_proofs({rank: proof}, device=coll_dev)

    if args.warmup:
        run_steps(args.warmup)

    # timed region: `steps` batches of K concurrent shard proofs
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    proof = run_steps(args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    # profiled region: single-shard latency with per-stage HIP events on the launching stream
    # (one shard in flight, so a stage's events bracket only its own kernels); the roofline and
    # the stage table come from here, the throughput `value` from the timed region above
    nprof = max(1, args.profile_steps)
    lib().zkm_profile_reset()
    lib().zkm_profile_enable(1)
    torch.cuda.synchronize()
    ts = time.perf_counter()
    for _ in range(nprof):
        prove_resident(prover, dev_traces, pvs)
    torch.cuda.synchronize()
    serial_ms = (time.perf_counter() - ts) / nprof * 1e3
    lib().zkm_profile_enable(0)
    need = lib().zkm_profile_dump(None, 0)
    buf = C.create_string_buffer(need)
    lib().zkm_profile_dump(buf, need)
    prof = parse_profile(buf.value.decode())

    # PCIe-inclusive rate (host traces, same prover): one extra untimed-by-value pass
    tp = time.perf_counter()
    prover.prove_shard(traces, pvs)
    pcie_s = time.perf_counter() - tp

    kernel_stages = ["lde", "merkle_leaves", "merkle_nodes", "quotient", "perm_trace", "open_eval", "fri_reduce"]
    dom = max((s for s in kernel_stages if s in prof), key=lambda s: prof[s][1])
    cnt, ms, units = prof[dom]
    achieved = units / (ms / 1e3) / 1e9  # GB/s, algorithmic bytes / measured stage time
    traffic, tsrc = pmc_traffic(dom)
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": dom,
                "launches": cnt, "avg_ms": round(ms / cnt, 4),
                "algorithmic_bytes_per_launch": round(units / cnt), "traffic_source": tsrc}
    if dom == "merkle_leaves" and "merkle_leaves_perms" in prof:
        roofline["valu"] = valu_roofline(prof["merkle_leaves_perms"][2], ms)
    ntt = None
    if "lde" in prof and "lde_gfops" in prof:
        # NTT GF-ops/s (BASELINE metric) against the HBM roofline of the same work: 12 B of HBM
        # traffic per input element (4 B read, 8 B written) at 8 TB/s, i.e. (8e12 / 12) x ops/elem
        lcnt, lms, lbytes = prof["lde"]
        gfops = prof["lde_gfops"][2]
        rate = gfops / (lms / 1e3)
        roof = HBM_PEAK_GBS * 1e9 / lbytes * gfops
        ntt = {"gf_ops_per_s": float(f"{rate:.4g}"), "hbm_roofline_gf_ops_per_s": float(f"{roof:.4g}"),
               "frac": round(rate / roof, 4), "algorithmic_GBps": round(lbytes / (lms / 1e3) / 1e9, 1),
               "launches": lcnt, "stage_ms_per_shard": round(lms / nprof, 3)}
        meas = lde_measured_hbm()
        if meas:
            ntt["hbm_measured"] = meas
    hbm_kernels = {name: measured_hbm(lambda k, p=pat: k == p)
                   for name, pat in (("quotient", "zkm_quot_jit"), ("logup_trace", "zkm_perm_jit"),
                                     ("fri_reduce", "k_fri_reduce"), ("openings", "k_open_dot"))}
    stages = {k: {"count": v[0], "ms_per_shard": round(v[1] / nprof, 3)}
              for k, v in sorted(prof.items()) if not k.endswith("_perms") and not k.endswith("_gfops")}

    value = world * K * rows_per_shard * args.steps / elapsed
    line = {
        "metric": "shard trace rows proved/sec at 2^22 rows",
        "value": round(value, 1),
        "unit": "rows/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "ms_per_shard": round(1e3 * elapsed / (args.steps * K), 3),
        "serial_ms_per_shard": round(serial_ms, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32 (KoalaBear mod p, EF = F[X]/(X^4-3))",
        "data": "synthetic (seeded S-SHARD traces, SURVEY.md §8d)",
        "config": {"workload": (f"S-SHARD FibCpu 2^{args.log_n} rows (main 67, LogUp 11 EF, quotient 2) + FibTable "
                                f"2^{W.fib_table_height(n).bit_length() - 1} (prep 2): full commit+open per shard")
                   if args.workload == "fib" else
                   (f"MIPS core shard: a counted loop (60-instruction body of ALU and load/store ops, forward branches, jal/jalr calls "
                    f"of a subroutine, bal) "
                    f"executed to {int(traces['Cpu'][:, 65].sum())} instructions: Cpu 2^{args.log_n} (main 67, "
                    f"LogUp 11 EF) + Program (prep 14) + DivRem, AddSub, Bitwise, Mul, Lt, ShiftLeft, ShiftRight, CloClz, MovCond, MemoryInstrs, MiscInstrs, "
                    f"Branch, Jump + Byte 2^16 (prep 12) + RegisterState: full commit+open per shard")
                   if args.workload == "core" else
                   (f"MIPS ALU slice: InstrSource 2^{args.log_n} + AddSub, Bitwise, Lt 2^{args.log_n - 2} + ShiftLeft, "
                    f"ShiftRight (CPU + CloClz SRLs) 2^{args.log_n - 3} + CloClz 2^{args.log_n - 4} + Byte 2^16 "
                    f"(prep 12): full commit+open per shard"),
                   "rows_per_shard": rows_per_shard, "fri_queries": args.queries, "pow_bits": 16, "log_blowup": 1,
                   "shards_per_gpu_per_step": K, "parallelism": f"shard-parallel x{world}, {K} in flight per GPU",
                   "proof_bytes": len(proof)},
        "pcie_inclusive_rows_per_s": round(rows_per_shard / pcie_s, 1),
        "roofline": roofline,
        "ntt": ntt,
        "hbm_measured": {k: v for k, v in hbm_kernels.items() if v},
        "stages_ms_per_shard": stages,
        "profiled_region": f"{nprof} single-shard proofs after the timed region (stages, roofline, ntt, serial_ms_per_shard)",
    }
    if not args.no_cpu_baseline and world == 1:
        line["cpu_baseline"] = cpu_baseline(args.cpu_log_n, args.queries)
    if args.profile_out:
        with open(args.profile_out, "w") as f:
            f.write(buf.value.decode())
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
