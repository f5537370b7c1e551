#!/usr/bin/env python3
"""Benchmark: shard trace rows proved per second (BASELINE.json `metric`).

Workload (N = 1 unless --gpus): the S-SHARD synthetic shard of SURVEY.md §8d at 2^22 rows —
FibCpu (main 67 columns, 20 local lookups -> 11 EF LogUp columns, quotient degree 2, shaped like
the reference's Cpu chip) plus the preprocessed FibTable chip — proven end to end exactly as the
reference's CpuProver::commit + CpuProver::open would (LDE, Poseidon2 MMCS, LogUp trace, quotient,
openings, FRI with 84 queries and 16 PoW bits).

One step = one batch of --inflight concurrent shard proofs per GPU.  `value` is the throughput with
the traces already resident in HBM when the timed region starts (the benchmark contract: inputs in
HBM; the proof's D2H is inside the span).  The PCIe-inclusive rate is reported beside it as
`host_traces`: the traces sit in page-locked host memory and each in-flight slot runs the
reference's pipeline shape (prove.rs:162-526: the next shard's traces travel while the current one
proves) — the H2D DMA of shard j+1 into one of two HBM buffers is issued before shard j is proven
from the other, so PCIe (≈57 GB/s, 1.13 GB per 2^22 shard) overlaps the kernels.  For N > 1 every
rank proves its own shards (shards are independent, prove.rs:208-209) and the proofs are gathered
to rank 0 over RCCL inside the timed region.

Also reported: `host_per_call` (each zkm_prove_shard call copies its own pinned host traces, no
look-ahead), `sizes` (the same resident measurement at 2^20, 2^21 and 2^23 rows; 2^24 has no LDE
domain), the roofline of the dominant stage (HIP events on the launching stream, PMC traffic from
rocprofv3 passes in this run) and the CPU baseline on a bounded sample.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))

# Hardware queues per process (read by the HIP runtime at initialisation).  HIP's default of 4 is fewer than
# the streams of the host-trace mode (3 prover slots, the copy stream, torch's own): the copy stream then
# shares a queue with a prover stream, whose kernels wait behind each 19.6 ms copy (34 ms per shard instead
# of 27.5; profiles/r04_hw_queues.txt).  8 gives every stream its own queue; the resident rate is unchanged.
# Forced, not a default: the GPU box exports GPU_MAX_HW_QUEUES=4, which a setdefault left in place (round 4's
# bench line ran its host-trace mode with 4 queues: 1.27x resident, against 1.03-1.04x with 8 in the
# controlled runs).  ZKM_BENCH_HW_QUEUES overrides (A/B only).
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("ZKM_BENCH_HW_QUEUES", "8")
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


class RawDev:
    """A device buffer from hipExtMallocWithFlags, shaped like the trace it receives (bench --h2d-dst)."""
    _hip = None

    def __init__(self, shape, flags):
        if RawDev._hip is None:
            h = C.CDLL("libamdhip64.so")
            h.hipExtMallocWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
            h.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
            RawDev._hip = h
        self.shape = tuple(shape)
        self.nbytes = int(np.prod(shape)) * 4
        p = C.c_void_p()
        if RawDev._hip.hipExtMallocWithFlags(C.byref(p), max(self.nbytes, 4), flags) != 0:
            raise RuntimeError("hipExtMallocWithFlags failed")
        self.ptr = p.value

    def data_ptr(self):
        return self.ptr

    def copy_from_host(self, host_tensor, stream):
        RawDev._hip.hipMemcpyAsync(self.ptr, host_tensor.data_ptr(), self.nbytes, 1, stream.cuda_stream)


H2D_FLAGS = {"uncached": 0x3, "finegrained": 0x1}


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


STAGE_KERNELS = {  # profiled stage -> the kernels it brackets (kernel-name prefixes)
    "merkle_leaves": ("k_hash_leaves",), "merkle_nodes": ("k_compress", "k_tree_top"),
    "quotient": ("zkm_quot", "k_quotient"), "fri_reduce": ("k_fri_reduce",),
    "perm_trace": ("zkm_perm", "k_perm", "k_ef_scan", "k_scan"), "open_eval": ("k_open_dot", "k_inv_points"),
    "lde": ("k_lde", "k_ntt", "k_twist", "k_bitrev"),
}


def _counter_rows(d, counter=None):
    """(dispatch id, kernel short name, counter value) of every row of a rocprofv3 counter CSV under d
    (only the rows of `counter` when a pass collected several)."""
    import csv
    import glob
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if counter and r.get("Counter_Name") != counter:
                continue
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("zkm::", "")
            rows.append((int(r["Dispatch_Id"]), k, float(r["Counter_Value"])))
    rows.sort()
    return rows


def _last_proof(rows):
    """The child proves the same shard twice after setup: the dispatch sequence ends with two equal
    runs of L kernels; return the last run (one proof's dispatches)."""
    names = [k for _, k, _ in rows]
    for L in range(len(names) // 2, 0, -1):
        if names[-L:] == names[-2 * L:-L]:
            return rows[-L:]
    return []


def pmc_in_run(args, timeout_s=240):
    """HBM bytes per kernel for one shard proof, measured now on this box: two rocprofv3 counter passes
    (FETCH_SIZE, then WRITE_SIZE: they do not fit one pass) over `bench.py --pmc-child`, kernel dispatch
    counters only.  Bytes = 2 x FETCH_SIZE + WRITE_SIZE (KB -> B), the gfx950 correction of
    MI355X_MICROARCH.md §HBM (FETCH_SIZE reports half of a coalesced streaming read).
    Returns {kernel: [bytes per proof, launches per proof]} or None when rocprofv3 is unavailable."""
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3")
    if not prof:
        return None
    out = {}
    base = tempfile.mkdtemp(prefix="zkm_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    child = [sys.executable, os.path.join(ROOT, "bench.py"), "--pmc-child", "--workload", args.workload,
             "--log-n", str(args.log_n), "--queries", str(args.queries)]
    sq = {}
    for ctr, mult in (("FETCH_SIZE", 2.0), ("WRITE_SIZE", 1.0), (" ".join(SQ_COUNTERS), None)):
        progress(f"counter pass {ctr.split()[0]}")
        d = os.path.join(base, ctr.split()[0])
        cmd = ["timeout", "-s", "KILL", str(timeout_s), prof, "--pmc"] + ctr.split() + [
            "--output-format", "csv", "-d", d, "-o", "run", "--"] + child
        r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, cwd=base)
        if r.returncode != 0:
            sys.stderr.write(f"pmc pass {ctr} failed ({r.returncode}): {r.stderr.decode()[-400:]}\n")
            if mult is None:
                break  # the SQ pass is optional: keep the HBM bytes
            return None
        if mult is None:  # SQ / GRBM counters per kernel per proof
            for c in SQ_COUNTERS:
                for _, k, v in _last_proof(_counter_rows(d, c)):
                    sq.setdefault(k, {}).setdefault(c, 0.0)
                    sq[k][c] += v
            continue
        for _, k, v in _last_proof(_counter_rows(d)):
            e = out.setdefault(k, [0.0, 0, 0.0])
            e[0] += mult * v * 1024.0
            if ctr == "FETCH_SIZE":
                e[1] += 1
            e[2] += v * 1024.0 if ctr == "FETCH_SIZE" else 0.0
    shutil.rmtree(base, ignore_errors=True)
    return {k: {"bytes_per_proof": v[0], "launches_per_proof": v[1], "fetch_raw_per_proof": v[2],
                "sq": sq.get(k)} for k, v in out.items()}


# one rocprofv3 pass (at most 8 SQ + 2 GRBM counters): VALU instructions and waves summed over the
# dispatch, and the GPU-busy cycles summed over the 8 XCDs (MI355X_MICROARCH.md)
SQ_COUNTERS = ("SQ_INSTS_VALU", "SQ_WAVES", "GRBM_GUI_ACTIVE", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT",
               "SQ_LDS_IDX_ACTIVE")
P2_KERNELS = ("k_hash_leaves", "k_compress_level", "k_subtree16", "k_compress_inject")


def lds_counters(pmc):
    """LDS use of the Poseidon2 kernels over one proof (the same SQ pass): LDS instructions per wave and the
    bank-conflict cycles per LDS-active cycle (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE; 0 = every LDS
    access served conflict-free).  The throughput kernels hold the permutation state in registers (one
    lane per state), so their LDS use is the row staging of the leaf loads and the subtree levels."""
    if not pmc:
        return None
    out = {}
    for k, v in pmc.items():
        c = v.get("sq") or {}
        if not k.startswith(P2_KERNELS) or not c.get("SQ_WAVES") or "SQ_INSTS_LDS" not in c:
            continue
        name = next(p for p in P2_KERNELS if k.startswith(p))
        e = out.setdefault(name, {"SQ_WAVES": 0.0, "SQ_INSTS_LDS": 0.0, "SQ_LDS_BANK_CONFLICT": 0.0,
                                  "SQ_LDS_IDX_ACTIVE": 0.0})
        for f in e:
            e[f] += c.get(f, 0.0)
    res = {}
    for name, e in out.items():
        res[name] = {"lds_insts_per_wave": round(e["SQ_INSTS_LDS"] / e["SQ_WAVES"], 2) if e["SQ_WAVES"] else None,
                     "bank_conflict_per_active_cycle": (round(e["SQ_LDS_BANK_CONFLICT"] / e["SQ_LDS_IDX_ACTIVE"], 4)
                                                        if e["SQ_LDS_IDX_ACTIVE"] else 0.0)}
    return res or None


def valu_counters(pmc, ms_per_proof, kernel="k_hash_leaves"):
    """Counter-derived VALU figures of a kernel over one proof (its PMC child run): VALU instructions per
    wave (SQ_INSTS_VALU / SQ_WAVES), busy cycles per XCD (GRBM_GUI_ACTIVE / 8), the effective clock
    (those cycles over the kernel's time in this run's profiled region) and the issue fraction
    SQ_INSTS_VALU x 2 cycles (wave64 on SIMD-32) x the mean issue cost per instruction of the
    permutation's ISA / (1024 SIMDs x busy cycles): how full the VALU issue ports were at the clock the
    chip actually ran."""
    if not pmc or kernel not in pmc or not pmc[kernel].get("sq"):
        return None
    c = pmc[kernel]["sq"]
    cyc = c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
    if not cyc or not c.get("SQ_WAVES"):
        return None
    out = {"source": "rocprofv3 --pmc " + " ".join(SQ_COUNTERS) + " in this run",
           "valu_insts_per_wave": round(c["SQ_INSTS_VALU"] / c["SQ_WAVES"], 1),
           "busy_cycles_per_xcd": round(cyc),
           "effective_clock_ghz": round(cyc / (ms_per_proof / 1e3) / 1e9, 3) if ms_per_proof else None}
    f = os.path.join(ROOT, "zkmips_amd", "isa_p2.json")
    if os.path.exists(f):
        j = json.load(open(f))
        if j.get("valu_instructions"):
            w = j["issue_slots"] / j["valu_instructions"]
            out["issue_frac"] = round(c["SQ_INSTS_VALU"] * 2.0 * w / (1024.0 * cyc), 4)
            out["mean_issue_cost"] = round(w, 3)
    return out


def stage_traffic(pmc, stage):
    """(HBM bytes per proof, launches per proof) of the kernels a profiled stage brackets."""
    if not pmc:
        return None, 0
    pre = STAGE_KERNELS.get(stage, ())
    b = n = 0
    for k, v in pmc.items():
        if k.startswith(pre):
            b += v["bytes_per_proof"]
            n += v["launches_per_proof"]
    return (b, n) if n else (None, 0)


VALU_PEAK_TSLOTS = 256 * 4 * 32 * 2.4e9 / 1e12  # CUs x SIMDs x SIMD-32 lanes x 2.4 GHz (MI355X_MICROARCH.md)


def valu_roofline(perms, ms):
    """Poseidon2 leaf hashing is integer-VALU bound: issue slots per permutation (static ISA count of
    the permutation weighted by the measured issue cost of each instruction class,
    profiles/rNN_isa_p2.json from tools/isa_slots.py) x permutations / measured stage time, against
    the architectural VALU issue rate."""
    f = os.path.join(ROOT, "zkmips_amd", "isa_p2.json")
    if not os.path.exists(f):
        return None
    slots = json.load(open(f))["issue_slots"]
    pps = perms / (ms / 1e3)
    achieved = pps * slots / 1e12
    return {"bound": "valu", "achieved": round(achieved, 2), "peak": round(VALU_PEAK_TSLOTS, 2),
            "unit": "T VALU issue slots/s", "frac": round(achieved / VALU_PEAK_TSLOTS, 4),
            "permutations_per_s": round(pps), "slots_per_permutation": slots,
            "source": "zkmips_amd/isa_p2.json (tools/isa_slots.py)"}


def host_info():
    """CPU model, logical CPUs and RAM of the box (BASELINE.md §3 asks for them beside the CPU number)."""
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
        mem = next(int(l.split()[1]) for l in open("/proc/meminfo") if l.startswith("MemTotal"))
    except (OSError, StopIteration):
        mem = 0
    return {"cpu_model": model, "nproc": os.cpu_count(), "mem_gib": round(mem / 2**20, 1),
            "omp_threads": os.environ.get("OMP_NUM_THREADS")}


def cgroup_cpu_limit(proc_cgroup="/proc/self/cgroup", mount="/sys/fs/cgroup"):
    """The cgroup v2 CPU quota of this process in CPUs, or None if unlimited: the tightest cpu.max ("quota
    period") on the path from the process's cgroup up to the mount root.  On the GPU box the process's own
    cgroup has no cpu.max and the quota (1600000 100000 = 16 CPUs) sits on /sys/fs/cgroup itself
    (profiles/r05_cpu_cliff.txt), so reading only the leaf misses it."""
    try:
        cg = open(proc_cgroup).read().strip().split("\n")[0].split(":", 2)[2]
    except (OSError, IndexError):
        cg = "/"
    best = None
    path = cg.rstrip("/")
    while True:
        try:
            q, p = open(f"{mount}{path}/cpu.max").read().split()
            if q != "max":
                c = int(q) / int(p)
                best = c if best is None else min(best, c)
        except (OSError, ValueError):
            pass
        if not path:
            break
        path = path.rsplit("/", 1)[0]
    return None if best is None else round(best, 2)


def _omp(threads=None) -> int:
    gomp = C.CDLL("libgomp.so.1")  # the oracle's OpenMP runtime (same soname, same instance)
    if threads:
        gomp.omp_set_num_threads(int(threads))
    return gomp.omp_get_max_threads()


def cpu_threads() -> int:
    return _omp()


def calibrate_cpu_threads(log_n=18, queries=84):
    """How many OpenMP threads the oracle actually profits from on this box: one 2^log_n FibCpu proof at
    each candidate count up to the CPUs the job is allotted (the affinity mask, capped by the cgroup's CFS
    quota), fastest wins.  (The GPU box shows 256 CPUs with a 16-CPU quota: there 128 threads ran a proof
    ~100x slower than 16, spin-waiting against the throttle; profiles/r05_cpu_cliff.txt.)"""
    from tests import _oracle as O
    from zkmips_amd import workloads as W
    cpus = len(os.sched_getaffinity(0))
    quota = cgroup_cpu_limit()
    allot = {int(quota)} if quota and quota >= 1 else set()
    # counts up to the CPUs the job may use: the affinity mask, capped by the CFS quota when there is one (above
    # the quota the spinning OpenMP barriers are throttled, profiles/r05_cpu_cliff.txt)
    cap = min(cpus, int(quota)) if allot else cpus
    m, prep, traces, pvs = W.fib_shard(1 << log_n, seed=2)
    pr = O.OracleProver(m, prep, num_queries=queries)
    table = {}
    for c in sorted({c for c in {8, 16, 24, 32, 48, 64, 128, cpus} | allot if c <= cap}):
        _omp(c)
        t = time.time()
        rc, _ = pr.prove(traces, pvs)
        assert rc == 0
        table[c] = round(time.time() - t, 3)
    best = min(table, key=table.get)
    _omp(best)
    return best, table


def cpu_baseline(log_n, queries):
    """The CPU oracle (a C/OpenMP restatement, not the reference binary; AVX-512 Poseidon2 and LDE, batch
    inversions, oracle/p2x16.c, oracle/lde_x16.c) on one shard of the headline size, with the OpenMP
    thread count that is fastest on this box (calibrated over every count up to the whole affinity
    mask, whatever OMP_NUM_THREADS the environment set)."""
    from tests import _oracle as O
    from zkmips_amd import workloads as W
    best, table = calibrate_cpu_threads(queries=queries)
    n = 1 << log_n
    m, prep, traces, pvs = W.fib_shard(n, seed=1)
    pr = O.OracleProver(m, prep, num_queries=queries)
    threads = _omp(best)
    t0 = time.time()
    rc, proof = pr.prove(traces, pvs)
    dt = time.time() - t0
    assert rc == 0
    cpus = len(os.sched_getaffinity(0))
    quota = cgroup_cpu_limit()
    return {"value": n / dt, "unit": "rows/s", "cores": threads, "kind": "port",
            "cpus_allotted": quota if quota is not None else cpus,
            "host": dict(host_info(), cpus_allowed=cpus, cgroup_cpu_quota=quota),
            "thread_calibration_s": {str(k): v for k, v in table.items()},
            "sample": f"one S-SHARD FibCpu 2^{log_n}-row shard (+FibTable), full commit+open, {queries} queries, "
                      f"{dt:.2f} s wall on {threads} OpenMP threads, the fastest count for this box among "
                      f"{sorted(table)} (2^18-row calibration proofs; {cpus} CPUs in the affinity mask, "
                      f"CFS quota {quota} CPUs: more threads than the quota spin-wait against the throttle, "
                      "DESIGN.md §7) (AVX-512 Poseidon2/LDE)"}


def profile_proofs(prover, dev_traces, pvs, nprof):
    """nprof single-shard resident proofs with the per-stage HIP events on: (stage table, ms per proof)."""
    import torch
    from zkmips_amd._lib import lib
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
    return parse_profile(buf.value.decode()), serial_ms, buf.value.decode()


def size_series(args, prover0, K, logs=(20, 21, 23)):
    """north_star's 2^20..2^24 sweep beside the 2^22 headline: for each size one FibCpu shard resident in
    HBM, K concurrent slots proving it `steps` times (timed like `value`), then single-shard proofs with
    the stage events (LDE stage time and its NTT GF-ops/s).  2^24 rows need a 2^25-point LDE domain,
    beyond KoalaBear's two-adicity 24: not provable by the reference either."""
    import threading
    import torch
    from zkmips_amd import workloads as W
    from zkmips_amd.prover import HipProver
    out = {}
    for lg in logs:
        n = 1 << lg
        m, prep, tr, pvs = W.fib_shard(n, seed=1)
        dev = {k: torch.from_numpy(v.view(np.int32)).cuda() for k, v in tr.items()}
        pr = HipProver(prover0.dev, m, prep, num_queries=args.queries)
        steps = max(2, args.steps // (2 if lg > 22 else 1))
        proofs = [b""] * K
        prove_resident(pr, dev, pvs)  # warm (allocator pool at this size)

        def slot(k):
            for _ in range(steps):
                proofs[k] = prove_resident(pr, dev, pvs)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        th = [threading.Thread(target=slot, args=(k,)) for k in range(K)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        assert all(p == proofs[0] for p in proofs), "size series: slots' proofs differ"
        prof, serial_ms, _ = profile_proofs(pr, dev, pvs, 2)
        e = {"value": round(K * n * steps / el, 1), "unit": "rows/s", "ms_per_shard": round(1e3 * el / (K * steps), 3),
             "serial_ms_per_shard": round(serial_ms, 3), "steps": steps, "in_flight": K, "proof_bytes": len(proofs[0])}
        if "lde" in prof and "lde_gfops" in prof:
            lcnt, lms, lbytes = prof["lde"]
            e["lde_ms_per_shard"] = round(lms / 2, 3)
            e["ntt_gf_ops_per_s"] = float(f"{prof['lde_gfops'][2] / (lms / 1e3):.4g}")
            e["lde_algorithmic_GBps"] = round(lbytes / (lms / 1e3) / 1e9, 1)
        out[f"2^{lg}"] = e
        del pr, dev
        torch.cuda.synchronize()
    out["2^24"] = "N/A: a 2^24-row trace needs a 2^25-point coset LDE (blowup 2); KoalaBear's two-adicity is 24"
    return out


def maxshape_leg(args, rk, n, K):
    """Secondary field of the default line (BASELINE config 3's shape): the reference's maximal 2^22 MIPS shard
    shape (maximal_shapes.json["22"][2], zkmips_amd/shapes.py: 17 chips, 557M main cells, 2.23 GB of traces).
    `value`: the executor's event records (1.09 GB) in page-locked host memory, their H2D inside the span and
    pipelined like the headline's, each shard's traces built on the device from them and proven (the trait's
    generate_traces + commit + open, prover.rs:70-108,111-137); beside it the same steps from page-locked host
    traces (2.23 GB of H2D per shard) and from traces resident in HBM."""
    sb = ShardBench(args, rk, "maxshape", n, K, records=True)
    sb.run_steps(1, "records")
    sb.run_steps(1, "pipelined")
    steps = max(1, args.maxshape_steps)
    p0, el_rec = sb.timed(steps, "records")
    rec_waits = {k: list(v) for k, v in sb.slot_waits.items()}
    p1, el = sb.timed(steps, "pipelined")
    p2, el_res = sb.timed(steps, "resident")
    assert p0 == p1 == p2, "maxshape: records / host-trace / resident proofs differ"
    tr = sb.shards[0][2]
    rows = sb.rows_per_shard
    rec_bytes = int(sum(int(t.numel()) for t in sb.records["pinned"].values()))
    out = {"workload": "MIPS shard in the reference maximal shape maximal_shapes.json[\"22\"][2]: "
                       + ", ".join(f"{k} 2^{int(np.log2(len(tr[k])))}" for k in sorted(tr, key=lambda c: -len(tr[c]))),
           "rows_per_shard": rows, "main_cells": int(sum(v.size for v in tr.values())), "steps": steps, "in_flight": K,
           "value": round(K * rows * steps / el_rec, 1), "unit": "rows/s",
           "ms_per_shard": round(1e3 * el_rec / (steps * K), 3),
           "value_basis": "event records in page-locked host memory, H2D of the records + device trace generation + "
                          "commit + open + proof D2H inside the span",
           "h2d_bytes_per_shard": rec_bytes,
           "vs_resident": round(el_rec / el_res, 3),
           "records_copy_wait_ms": [round(1e3 * sum(v), 2) for _, v in sorted(rec_waits.items())],
           "call_ms_mean": {m_: round(1e3 * float(np.mean([t for (mm, _), v in sb.slot_proof_s.items() if mm == m_
                                                           for t in v])), 3)
                            for m_ in ("records", "pipelined", "resident")},
           "tracegen_ms_mean_per_step": round(1e3 * float(np.mean([t for v in sb.slot_tracegen_s.values() for t in v])), 3),
           "host_traces": {"value": round(K * rows * steps / el, 1), "ms_per_shard": round(1e3 * el / (steps * K), 3),
                           "h2d_bytes_per_shard": int(sum(v.nbytes for v in tr.values())),
                           "vs_resident": round(el / el_res, 3)},
           "resident": {"value": round(K * rows * steps / el_res, 1), "ms_per_shard": round(1e3 * el_res / (steps * K), 3)},
           "proof_bytes": len(p1), "trace_generation_s": round(sb.gen_s, 1)}
    out["from_device_traces"] = maxshape_from_records(sb, steps)
    del sb
    return out


_CAPTURE = {}


def maxshape_from_records(sb, steps):
    """The maximal-shape shard's traces built on the device from the executor's records (every chip at the
    shape's height, Byte and Program multiplicities included), then proven from them: device trace time
    (records already in HBM; their H2D timed apart), per-shard proof time from the device traces, and the
    proof bytes checked against the host-trace proof."""
    import torch
    from zkmips_amd import mips_alu as A
    from zkmips_amd import tracegen as TG
    cap = _CAPTURE.get("maxshape")
    if not cap:
        return None
    dev_t, pv = sb.shards[0][0], sb.shards[0][1]
    heights = {k: int(v.shape[0]) for k, v in dev_t.items() if k not in ("Byte", "Program")}
    t0 = time.perf_counter()
    recs = TG.shard_records_to_device(cap)
    torch.cuda.synchronize()
    h2d_s = time.perf_counter() - t0
    rec_bytes = sum(int(v.numel()) for k, v in recs.items() if k != "_n")
    bm = torch.zeros((A.BYTE_ROWS, A.BYTE_MULT_WIDTH), dtype=torch.int32, device="cuda")
    TG.shard_traces(cap, byte_mult=bm, heights=heights, records=recs)  # warm (JIT of nothing; allocator)
    reps = 3
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        bm.zero_()
        tr = TG.shard_traces(cap, byte_mult=bm, heights=heights, records=recs)
    e1.record()
    torch.cuda.synchronize()
    gen_ms = e0.elapsed_time(e1) / reps
    tr["Byte"] = bm
    tr = {k: v for k, v in tr.items() if k in dev_t}
    ref = sb.prover.prove_shard(dev_t, pv)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        p = sb.prover.prove_shard(tr, pv)
    torch.cuda.synchronize()
    ms = 1e3 * (time.perf_counter() - t0) / steps
    assert p == ref, "maxshape: device-trace proof differs from the host-trace proof"
    trace_bytes = sum(int(v.numel()) * 4 for v in tr.values())
    return {"device_tracegen_ms": round(gen_ms, 3), "records_bytes": rec_bytes,
            "records_convert_and_upload_s": round(h2d_s, 3),  # Python executor tuples -> structs, then H2D
            "trace_bytes": trace_bytes, "serial_ms_per_shard_from_device_traces": round(ms, 3),
            "proof_bytes_equal_host_trace_proof": True,
            "what": "every chip of the shard built on the device from the executor's event records at the shape's "
                    "heights (zkmips_amd/tracegen.shard_traces), then one shard proof at a time from them"}


def make_shard(workload, n, seed):
    from zkmips_amd import workloads as W
    if workload == "core":
        from zkmips_amd import mips_core as MC
        return MC.loop_shard(60, (3 * n // 4) // 104, seed=1)  # ~98 instructions per iteration
    if workload == "maxshape":  # the reference's 2^22 maximal shape, scaled to 2^log_n Cpu rows
        from zkmips_amd import shapes as SH
        _CAPTURE["maxshape"] = cap = {}  # the executor's records, for the device-trace sub-leg
        return SH.shape_shard(SH.MAXIMAL_22, seed=1, down=22 - (n.bit_length() - 1), capture=cap)
    if workload == "alu":
        from zkmips_amd import mips_alu as A
        return A.alu_shard(n // 4, n // 4, seed=seed, n_lt=n // 4, n_sll=n // 8, n_sr=n // 16, n_clz=n // 16)
    return W.fib_shard(n, seed=seed)


class Ranks:
    """This process's place in the job: RANK / LOCAL_RANK / WORLD_SIZE from the launcher (the driver's
    torch.distributed.run, or `launch_ranks` below), the GPU it binds, and the process group (RCCL over
    xGMI; gloo when rehearsing N ranks on fewer GPUs, ZKM_BENCH_REHEARSE=1).  `--gpus` must equal the
    live world size."""

    def __init__(self, args, bind=True):
        import torch.distributed as dist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        if args.gpus is not None and args.gpus != self.world:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={self.world}")
        # ZKM_BENCH_REHEARSE=1: rehearse the N-rank flow on a box with fewer GPUs (ranks share the cards,
        # gloo instead of RCCL); never set by the driver, so the N-GPU bench is always RCCL.
        self.rehearse = os.environ.get("ZKM_BENCH_REHEARSE") == "1"
        # ZKM_BENCH_REPLAY=<dir> (rehearsal only, CPU tests of the launch/deal/gather plumbing): shard
        # proofs are read from <dir>/shard_<i>.bin instead of proven; no GPU is touched.
        self.replay = os.environ.get("ZKM_BENCH_REPLAY") if self.rehearse else None
        self.coll_dev = "cpu" if self.rehearse else "cuda"
        self.numa = None
        if not self.replay:
            import torch
            if self.rehearse:
                self.local_rank %= max(1, torch.cuda.device_count())
            torch.cuda.set_device(self.local_rank)
            if bind and os.environ.get("ZKM_NO_NUMA_BIND") != "1":
                self.numa = bind_near_gpu(self.local_rank)
        if self.world > 1:
            if self.rehearse:
                dist.init_process_group("gloo")
            else:
                import torch
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.local_rank))
            self.world = dist.get_world_size()
            assert self.world == (args.gpus or self.world), "process group size differs from --gpus"

    def sync(self):
        if not self.replay:
            import torch
            torch.cuda.synchronize()

    def barrier(self):
        if self.world > 1:
            import torch.distributed as dist
            dist.barrier()
        self.sync()

    def max_over_ranks(self, el):
        if self.world == 1:
            return el
        import torch
        import torch.distributed as dist
        t = torch.tensor([el], dtype=torch.float64, device=self.coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def close(self):
        if self.world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()


def _tendermint_job(outdir: str):
    """Pool worker (no GPU): the tendermint guest on the reference's blocks executed and traced
    (zkmips_amd/tendermint.tendermint_shards), the traces written as .npy files under outdir (a
    /dev/shm directory the bench process memory-maps).  Returns (chip names per shard, info, seconds)."""
    from zkmips_amd import tendermint as T
    t0 = time.perf_counter()
    shards, info = T.tendermint_shards()
    gen_s = time.perf_counter() - t0
    meta = []
    for i, (_, prep, tr, pv) in enumerate(shards):
        for k, v in tr.items():
            np.save(os.path.join(outdir, f"s{i}_{k}.npy"), v)
        np.save(os.path.join(outdir, f"s{i}__pv.npy"), pv)
        meta.append(sorted(tr))
    for k, v in shards[0][1].items():
        if v is not None:
            np.save(os.path.join(outdir, f"prep_{k}.npy"), v)
    info = {k: (v.hex() if isinstance(v, bytes) else v) for k, v in info.items()}
    return meta, info, gen_s


def _compress_leaves_job(outdir: str, n_leaves: int, down: int):
    """Pool worker (no GPU): config 5's leaves -- ONE execution of a loop in the reference's maximal 2^22 shape
    scaled to Cpu 2^(22-down), cut into n_leaves - 1 consecutive CPU shards (each padded to the scaled shape)
    plus the memory shard that closes it (zkmips_amd/shapes.shape_execution), so the compress nodes' chaining
    checks (shard numbers, pcs, address bits, global sums) hold and the root is a complete proof.  Traces as
    .npy files under outdir, as _tendermint_job."""
    from zkmips_amd import shapes as SH
    t0 = time.perf_counter()
    shards = SH.shape_execution(SH.MAXIMAL_22, n_leaves - 1, down=down)
    gen_s = time.perf_counter() - t0
    meta = []
    for i, (_, prep, tr, pv) in enumerate(shards):
        for k, v in tr.items():
            np.save(os.path.join(outdir, f"s{i}_{k}.npy"), v)
        np.save(os.path.join(outdir, f"s{i}__pv.npy"), pv)
        meta.append(sorted(tr))
    for k, v in shards[0][1].items():
        if v is not None:
            np.save(os.path.join(outdir, f"prep_{k}.npy"), v)
    return meta, {"cpu_shards": n_leaves - 1, "leaf_shape": {k: int(v.shape[0]) for k, v in shards[0][2].items()}}, gen_s


def _load_tendermint(outdir: str, meta):
    from zkmips_amd import mips_core as MC
    m = MC.core_machine()
    prep = {c.name: np.load(os.path.join(outdir, f"prep_{c.name}.npy"))
            for c in m.chips if os.path.exists(os.path.join(outdir, f"prep_{c.name}.npy"))}
    run = [(m, prep, {k: np.load(os.path.join(outdir, f"s{i}_{k}.npy")) for k in names},
            np.load(os.path.join(outdir, f"s{i}__pv.npy"))) for i, names in enumerate(meta)]
    return run


def prove_execution(args, rk, run, steps: int, warmup: int):
    """Configs 3/4: every shard of one execution proven (traces resident in HBM, `--inflight` shards at once
    per GPU, largest first); with N ranks the shards are dealt by cost (dist.deal_by_cost), the proofs
    gathered to rank 0 and the machine-level global cumulative sum checked there (machine.rs:639-654).
    Returns (seconds per execution, proofs on rank 0, rows per shard, shard kinds, the deal)."""
    import threading
    from zkmips_amd.dist import deal_by_cost, prove_shards_distributed, shard_cost
    from zkmips_amd.proof import machine_global_sum_is_zero
    world, rank = rk.world, rk.rank
    costs = [shard_cost(tr) for _, _, tr, _ in run]
    deal = deal_by_cost(costs, world)
    mine = deal[rank]
    if rk.replay:
        prove_one = lambda i: open(os.path.join(rk.replay, f"shard_{i}.bin"), "rb").read()
    else:
        import torch
        from zkmips_amd._lib import Device
        from zkmips_amd.prover import HipProver
        m, prep, _, _ = run[0]
        prep = {k: v for k, v in prep.items() if v is not None}
        prover = HipProver(Device(rk.local_rank), m, prep, num_queries=args.queries)
        dev = {i: ({k: torch.from_numpy(np.ascontiguousarray(v).view(np.int32)).cuda() for k, v in run[i][2].items()},
                   run[i][3]) for i in mine}
        prove_one = lambda i: prove_resident(prover, dev[i][0], dev[i][1])
    rows = [max(v.shape[0] for v in tr.values()) for _, _, tr, _ in run]
    kinds = ["cpu" if "Cpu" in tr else "memory" if "MemoryGlobalInit" in tr else "sha_extend" if "ShaExtend" in tr
             else "sha_compress" if "ShaCompress" in tr else "ed_add" if "EdAddAssign" in tr
             else "ed_decompress" if "EdDecompress" in tr else "uint256_mul" if "Uint256MulMod" in tr
             else "precompile" for _, _, tr, _ in run]
    rk.sync()

    def prove_local():
        idx = sorted(mine, key=lambda i: (-costs[i], i))  # largest first within the rank too
        out = {}
        nxt = [0]
        lock = threading.Lock()

        def worker():
            while True:
                with lock:
                    k = nxt[0]
                    nxt[0] += 1
                if k >= len(idx):
                    return
                i = idx[k]
                out[i] = prove_one(i)
        th = [threading.Thread(target=worker) for _ in range(max(1, args.inflight))]
        for t in th:
            t.start()
        for t in th:
            t.join()
        return out

    def prove_all():
        if world == 1:
            out = prove_local()
            proofs = [out[i] for i in range(len(run))]
            assert machine_global_sum_is_zero(proofs), "the execution's global cumulative sums do not add to zero"
            return proofs
        local = prove_local()
        return prove_shards_distributed(lambda i: local[i], len(run), device=rk.coll_dev, check_global_sum=True,
                                        costs=costs)

    for _ in range(max(1, warmup)):
        proofs = prove_all()
    rk.barrier()
    t1 = time.time()
    for _ in range(steps):
        proofs = prove_all()
    rk.barrier()
    el = rk.max_over_ranks(time.time() - t1)
    return el / steps, proofs, rows, kinds, deal


def tendermint_leg(args, pool_result, outdir, rk):
    """Config 4 as a field of the default line: the tendermint guest on examples/tendermint's two blocks
    (traces generated in the witness pool while the GPU legs ran), every shard proven, global sum checked."""
    meta, info, gen_s = pool_result
    run = _load_tendermint(outdir, meta)
    sec, proofs, rows, kinds, _ = prove_execution(args, rk, run, 1, 1)
    return {"metric": "shard trace rows proved/sec (tendermint light-client execution on the reference's blocks, "
                      "BASELINE config 4)",
            "value": round(sum(rows) / sec, 1), "unit": "rows/s", "ms_per_execution": round(1e3 * sec, 3),
            "shards": len(run), "shard_rows": [f"{k} 2^{r.bit_length() - 1}" for k, r in zip(kinds, rows)],
            "rows_per_execution": sum(rows), "proof_bytes": sum(len(p) for p in proofs),
            "global_sum_checked": True, "exit_code": info["exit_code"],
            "public_values_digest_matches_host": info["pv_digest"] == info["expected_digest"],
            "votes_verified": info["votes"], "trace_generation_s": round(gen_s, 1),
            "workload": "examples/tendermint guest restated (zkmips_amd/tendermint.py) on block_2279100.json -> "
                        "block_2279130.json: both header hashes (SHA-256 Merkle), three validator-set hashes, "
                        "100 vote signatures (SHA-512 in MIPS, ED_DECOMPRESS/ED_ADD, k mod L by UINT256_MUL), "
                        "voting-power thresholds, public-values digest committed"}


def execution_bench(args):
    """BASELINE configs 3/4 as their own bench line: a whole execution proven shard by shard.  `sha2`: the
    guest (mips_core.sha_program) hashes `--sha-blocks` 64-byte blocks with SHA_EXTEND + SHA_COMPRESS;
    `tendermint`: the light-client check of examples/tendermint on the reference's two block fixtures
    (zkmips_amd/tendermint.py).  See prove_execution."""
    from zkmips_amd import mips_core as MC
    rk = Ranks(args, bind=False)
    world, rank = rk.world, rk.rank
    t0 = time.time()
    info = None
    if args.workload == "tendermint":
        from zkmips_amd import tendermint as T
        run, info = T.tendermint_shards()
    else:
        max_steps = min((1 << args.log_n) * 4 // 5, (1 << 24) // 5 - 1)
        prog = MC.sha_program(args.sha_blocks, seed=1)
        run = MC.program_shards(prog, seed=1, shard_size=max_steps, precompile_events_per_shard=args.sha_events_per_shard)
    gen_s = time.time() - t0
    print(f"{args.workload}: {len(run)} shards generated in {gen_s:.1f} s", file=sys.stderr, flush=True)
    sec, proofs, rows, kinds, deal = prove_execution(args, rk, run, args.steps, args.warmup)
    what = ("tendermint light-client check on the reference's blocks 2279100 -> 2279130 (100 vote signatures)"
            if args.workload == "tendermint" else f"sha2-precompile execution: {args.sha_blocks} blocks")
    line = {
        "metric": ("shard trace rows proved/sec (whole tendermint execution, BASELINE config 4)"
                   if args.workload == "tendermint" else
                   "shard trace rows proved/sec (whole sha2-precompile execution, BASELINE config 3)"),
        "value": round(sum(rows) / sec, 1), "unit": "rows/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1e3 * sec, 3), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u32 (KoalaBear mod p, EF = F[X]/(X^4-3))",
        "data": ("examples/tendermint/host/files block fixtures (zkmips_amd/tendermint.py)"
                 if args.workload == "tendermint" else "synthetic sha2 guest (mips_core.sha_program)")
                + ", traces resident in HBM"
                + (" (REPLAYED proofs: launch/deal/gather rehearsal, nothing proven)" if rk.replay else ""),
        "config": {"workload": f"{what}, {len(run)} shards "
                               f"({', '.join(f'{k} 2^{r.bit_length() - 1}' for k, r in zip(kinds, rows))}), "
                               f"all MIPS + syscall + precompile + memory chips, full commit+open per shard",
                   "shards": len(run), "rows_per_execution": sum(rows), "fri_queries": args.queries,
                   "proof_bytes": sum(len(p) for p in proofs) if rank == 0 else None,
                   "parallelism": f"{args.inflight} shards in flight" + (
                       f" per rank, shards dealt by cost (LPT) over {world} ranks {deal}, proofs gathered to rank 0 "
                       "(global sum checked there)" if world > 1 else ""),
                   "trace_generation_s": round(gen_s, 1), "global_sum_checked": True},
    }
    if info:
        line["config"]["exit_code"] = info["exit_code"]
        line["config"]["public_values_digest"] = info["pv_digest"].hex()
    if rank == 0:
        print(json.dumps(line), flush=True)
    rk.close()


def tracegen_bench(args):
    """Device trace generation (include/zkm_tracegen.h, §8f row 2): the Cpu chip's trace of a
    2^log_n-row shard (the largest chip of a MIPS shard, 67 columns) from CpuEventFfi records resident
    in HBM, Byte and Program multiplicities included; plus AddSub (19 columns) and MemoryLocal.  The
    records are a real execution (mips_core.loop_program, 2^14 instructions) tiled to 2^log_n rows.
    HBM-bound: per Cpu row 280 B of record read + 268 B of trace written (+ the program fetch and the
    multiplicity atomics, served by L2).  Global: 2^log_n random messages lifted onto the septic curve
    and scanned (compute-bound; the host restatement takes ≈18 s for 2^22 on 8 cores)."""
    import torch
    from zkmips_amd import mips_core as MC
    from zkmips_amd import tracegen as TG
    torch.cuda.set_device(0)
    n = 1 << args.log_n
    cap = {}
    MC.program_shard(MC.loop_program(24, (1 << 14) // 28, seed=3), seed=3, shard=1, capture=cap)
    base = TG.cpu_events(cap["steps"], 1)
    tile = lambda r: r[np.arange(n) % len(r)]  # (np.resize would repack the padded record dtype)
    ev = tile(base)
    prog = TG.program_ffi(cap["prog"])
    adds = tile(TG.add_sub_records(cap["alu"]))
    ml = tile(TG.memory_local_events(cap["entries"]))
    d_ev, d_prog, d_add, d_ml = (TG.to_device(x) for x in (ev, prog, adds, ml))
    bm = torch.zeros((65536, 10), dtype=torch.int32, device="cuda")
    pm = torch.zeros((len(prog), 1), dtype=torch.int32, device="cuda")
    rng = np.random.default_rng(5)
    gmsg = rng.integers(0, 256, (n, 7)).astype(np.uint32)
    gmsg[:, 0], gmsg[:, 1], gmsg[:, 2] = 1, rng.integers(0, 1 << 24, n), rng.integers(0, 1 << 30, n)
    d_glob = TG.to_device(TG.global_events(gmsg, rng.integers(0, 2, n), np.ones(n)))
    d_p2 = torch.from_numpy(rng.integers(0, 0x7F000001, (n // 4) * 32).astype(np.int32)).cuda()
    chips = {
        "Cpu": (lambda: TG.cpu_trace(d_ev, n, 1, d_prog, len(prog), height=n, byte_mult=bm, program_mult=pm),
                280 + 4 * TG.CPU_WIDTH),
        "Global": (lambda: TG.global_trace(d_glob, n, height=n, byte_mult=bm), 32 + 4 * TG.GLOBAL_WIDTH),
        "AddSub": (lambda: TG.add_sub_trace(d_add, n, height=n, byte_mult=bm), 28 + 4 * TG.ADD_SUB_WIDTH),
        "MemoryLocal": (lambda: TG.memory_local_trace(d_ml, n, height=n // 4), 28 + 4 * 14),
        # recursion machine: a permutation per row (compute-bound); n // 4 rows
        "Poseidon2WideDeg3": (lambda: TG.poseidon2_wide_trace(d_p2, n // 4, height=n // 4), 64 + 4 * 313, n // 4),
    }
    # the other core chips at their heights in the reference's maximal 2^22 shape (maximal_shapes.json["22"][2],
    # relative to Cpu 2^22): records of the same execution (plus random ALU events for the shifts) tiled
    ev_alu = MC.A.alu_events(0, 1 << 12, seed=9, n_lt=1 << 12, n_sll=1 << 12, n_sr=1 << 12)
    for kind, (_, chip, width), lg in (("bit", TG.ALU_CHIPS["bit"], 2), ("lt", TG.ALU_CHIPS["lt"], 2),
                                       ("sll", TG.ALU_CHIPS["sll"], 4), ("sr", TG.ALU_CHIPS["sr"], 3)):
        m_ = n >> lg
        op, a, b, c, pc = ev_alu[kind]
        d = TG.to_device(tile(TG.alu_events(op, a, b, c, pc))[:m_])
        chips[chip] = ((lambda k=kind, d=d, m_=m_: TG.alu_trace(k, d, m_, height=m_, byte_mult=bm)), 28 + 4 * width, m_)
    d_br = TG.to_device(tile(TG.branch_records(cap["branches"]))[:n >> 3])
    chips["Branch"] = (lambda: TG.branch_trace(d_br, n >> 3, height=n >> 3, byte_mult=bm), 28 + 4 * TG.BRANCH_WIDTH,
                       n >> 3)
    d_mi = TG.to_device(tile(TG.mem_instr_records(cap["mevs"], 1))[:n >> 2])
    chips["MemoryInstrs"] = (lambda: TG.memory_instrs_trace(d_mi, n >> 2, height=n >> 2, byte_mult=bm),
                             84 + 4 * TG.MEMORY_INSTRS_WIDTH, n >> 2)
    # the SHA precompile chips at a 2^20-row precompile shard (config 3): a sha2 guest's calls tiled
    from zkmips_amd import mips_syscall as SY
    st = MC.fresh_state()
    MC.program_shard(MC.sha_program(4, seed=5), 5, 1, 1 << 14, state=st, regs=MC.initial_registers(5))
    ext = [e for code, _, e in st["precompile"] if code == SY.SHA_EXTEND]
    cmp_ = [e for code, _, e in st["precompile"] if code == SY.SHA_COMPRESS]
    n_ext, n_cmp = (n >> 2) // 48, (n >> 2) // 80
    se_rows = TG.sha_extend_records(ext)
    d_se = TG.to_device(se_rows[np.arange(48 * n_ext) % len(se_rows)])
    d_sc = TG.to_device(TG.sha_compress_records(cmp_)[np.arange(n_cmp) % len(cmp_)])
    chips["ShaExtend"] = (lambda: TG.sha_extend_trace(d_se, 48 * n_ext, height=n >> 2, byte_mult=bm),
                          116 + 4 * TG.SHA_EXTEND_WIDTH, 48 * n_ext)
    chips["ShaCompress"] = (lambda: TG.sha_compress_trace(d_sc, n_cmp, height=n >> 2, byte_mult=bm),
                            1648 / 80 + 4 * TG.SHA_COMPRESS_WIDTH, 80 * n_cmp)
    # every other precompile chip (one thread per row; the emulated-field chips compute their witnesses):
    # the calls of the all-precompile guest, a Keccak guest and an Ed25519 guest, each chip's records tiled
    # to n >> 6 rows (KeccakSponge: 24 rows per absorbed block)
    import collections
    from zkmips_amd import mips_ec as EC
    from zkmips_amd import mips_edwards as ED
    from zkmips_amd import mips_keccak as KS
    calls = collections.defaultdict(list)
    for gprog, seed in ((EC.ec_program(1, reps=1), 1), (KS.keccak_program([bytes(range(256)) * 2, b"abc" * 100]), 1),
                        (ED.ed25519_program(1, seed=3, scalar_bits=6), 3)):
        st = MC.fresh_state()  # (gprog: the Cpu lambda above reads prog when it runs)
        MC._execute(gprog, MC.initial_registers(seed), 1, 1 << 22, st)
        for code, _, e in st["precompile"]:
            calls[code].append(e)
    for code, evs in calls.items():
        name, rec, fn = TG.precompile_chip(code, evs)
        per = 24 if name == "KeccakSponge" else 1
        m_ = max(1, (n >> 6) // per)
        d = TG.to_device(rec[np.arange(m_) % len(rec)])
        width = fn(d, m_, byte_mult=bm).shape[1]
        chips[name] = ((lambda fn=fn, d=d, m_=m_: fn(d, m_, byte_mult=bm)), rec.dtype.itemsize / per + 4 * width,
                       m_ * per)
    res = {}
    for name, spec in chips.items():
        fn, bytes_per_row = spec[0], spec[1]
        rows_n = spec[2] if len(spec) > 2 else n
        for _ in range(max(1, args.warmup)):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.steps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.steps
        gbs = rows_n * bytes_per_row / ms / 1e6
        res[name] = {"ms": round(ms, 4), "rows": rows_n, "rows_per_s": round(rows_n / ms * 1e3, 1),
                     "algorithmic_bytes_per_row": bytes_per_row,
                     "GBps": round(gbs, 1), "frac_of_hbm_peak": round(gbs / (HBM_PEAK_GBS), 3)}
    cpu = res["Cpu"]
    line = {
        "metric": "Cpu trace rows generated/sec (device trace generation, zkm_cpu_events_to_trace)",
        "value": cpu["rows_per_s"], "unit": "rows/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": cpu["ms"], "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "data": "CpuEventFfi records of a real execution (loop_program, 2^14 instructions) tiled, resident in HBM",
        "config": {"workload": f"tracegen: Cpu 2^{args.log_n} rows (67 columns) + Byte/Program multiplicities"},
        "roofline": {"bound": "hbm", "achieved": cpu["GBps"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": cpu["frac_of_hbm_peak"], "traffic": None},
        "chips": res,
    }
    print(json.dumps(line), flush=True)


def start_witness_pool(n: int):
    """The compress witness-generation process pool, its workers spawned NOW (before anything in this
    process touches the GPU: they are started as fresh interpreters, never forked from a GPU process)."""
    from zkmips_amd.compress_tree import AffinityPool
    return AffinityPool(n).warm()


def mips_leaves(dev, queries: int, run, info: dict):
    """Config 5's leaves: the core shard proofs of one execution (_compress_leaves_job's shards, in shard
    order), proven on this GPU before the timed region with one proving key."""
    from zkmips_amd import recursion_verifier as RV
    from zkmips_amd.prover import HipProver
    m, prep = run[0][0], run[0][1]
    hp = HipProver(dev, m, prep, num_queries=queries)
    vk = RV.ChildVk.of(m, prep, hp.vk_commit, num_queries=queries)
    proofs = [hp.prove_shard(tr, pv) for _, _, tr, pv in run]
    from zkmips_amd.proof import machine_global_sum_is_zero
    assert machine_global_sum_is_zero(proofs), "compress leaves: the execution's global sums do not add to zero"
    info = dict(info, leaves=len(proofs), leaf_queries=queries, leaf_proof_bytes=len(proofs[0]),
                memory_shard_chips=sorted(run[-1][2]))
    return [(vk, p) for p in proofs], info


def _union_s(intervals) -> float:
    """Length of the union of (start, end) intervals: the time at least one proof was on the GPU."""
    tot, cur_s, cur_e = 0.0, None, None
    for s_, e_ in sorted(intervals):
        if cur_e is None or s_ > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s_, e_
        else:
            cur_e = max(cur_e, e_)
    return tot + (cur_e - cur_s if cur_e is not None else 0.0)


def _by_layer(times: dict) -> dict:
    """Reducer.times (node -> submit / witness / proved) grouped by the node's layer (complete entries only)."""
    out = {}
    for (layer, _), v in times.items():
        if len(v) == 3:
            out.setdefault(layer, []).append(v)
    return out


def compress_tree_run(pool, dev, leaves, inflight: int, distributed: bool = False):
    """One 64-leaf compress tree, dependency-driven (zkmips_amd/compress_tree.py): witness generation in
    the pool overlapping GPU proving.  Returns (root (vk, proof), result dict)."""
    import threading
    from zkmips_amd import compress_tree as CT
    provers = CT.GpuProvers(dev)
    stats = CT.TreeStats()
    lock = threading.Lock()
    spans = []
    shapes = {}

    def prove(wit):
        prep, traces, pvs, shape, times = wit
        pr = provers.get(prep, stats)
        t = time.perf_counter()
        traces = CT.materialize(traces)  # the Poseidon2 trace built on the device from its inputs
        proof = pr.prove_shard(traces, pvs)
        e = time.perf_counter()
        with lock:
            spans.append((t, e))
            stats.prove_s += e - t
            stats.proofs += 1
            stats.build_s += times["build_s"]
            stats.execute_s += times["execute_and_traces_s"]
            k = ",".join(f"{c}:{shape[c]}" for c in sorted(shape))
            shapes[k] = shapes.get(k, 0) + 1
            shapes.setdefault("_rows", {})[k] = max(int(v.shape[0]) for v in traces.values())
        return CT.compress_child_vk(pr.vk_commit, shape), proof

    # compact witnesses: main traces as event rows laid out on the device, prep traces once per program
    # (children's verifying keys by reference: each worker loads a key's file once)
    # (a node's job preferably to a worker holding its program's template: CT.AffinityPool)
    reducer = CT.Reducer(lambda ch, fl: pool.submit(CT.node_witness_shm, CT.by_ref(ch), True, True, True, **fl,
                                                    tag=CT.node_tag(ch)), prove, inflight)
    t0 = time.perf_counter()
    root = CT.reduce_distributed(leaves, reducer) if distributed else CT.reduce_serial(leaves, reducer)
    wall = time.perf_counter() - t0
    tl = [v for v in reducer.times.values() if len(v) == 3]
    timeline = None
    if tl:
        # per node: submit -> witness back (worker queue + build + execute + transfer), witness -> proof
        # (GPU queue + materialise + prove); and the depth of the tree's last node
        timeline = {"witness_latency_s_mean": round(float(np.mean([v["witness"] - v["submit"] for v in tl])), 3),
                    "prove_latency_s_mean": round(float(np.mean([v["proved"] - v["witness"] for v in tl])), 3),
                    "first_witness_back_s": round(min(v["witness"] for v in tl) - t0, 3),
                    "last_layer_submit_s": round(max(v["submit"] for v in tl) - t0, 3),
                    # per layer, seconds from the tree's start: the first node ready to build (children proven),
                    # the last witness back, the last proof done
                    "layers": [{"layer": L, "nodes": len(vs),
                                "first_ready_s": round(min(v["submit"] for v in vs) - t0, 3),
                                "last_witness_s": round(max(v["witness"] for v in vs) - t0, 3),
                                "last_proved_s": round(max(v["proved"] for v in vs) - t0, 3)}
                               for L, vs in sorted(_by_layer(reducer.times).items())]}
    rows = shapes.pop("_rows")
    from zkmips_amd import recursion as R
    names = {",".join(f"{c}:{sh[c]}" for c in sorted(sh)): i for i, sh in enumerate(R.RECURSION_SHAPES)}
    res = {"wall_s": wall, "gpu_busy_s": _union_s(spans), "proofs": stats.proofs, "timeline": timeline,
           "witness_build_s": stats.build_s, "witness_execute_and_traces_s": stats.execute_s,
           "setups": stats.setups, "setup_s": stats.setup_s, "lookups": stats.lookups,
           "shapes": {f"RecursionShapeConfig[{names.get(k, '?')}]" + (" (fastest)" if names.get(k) == 0 else ""):
                      {"nodes": v, "max_rows": rows[k], "log_heights": dict(kv.split(":") for kv in k.split(","))}
                      for k, v in shapes.items()}}
    return root, res


def compress_leg(args, pool, dev, world: int = 1, rank: int = 0, inflight: int = 3, leaves_job=None,
                 n_leaves: int = 64, leaf_log: int = None):
    """BASELINE config 5 as a field of a bench line: 64 MIPS leaf proofs reduced by the compress tree.
    Node programs verify their children in full (transcript, PoW, Merkle paths, FRI, and the out-of-domain
    constraint check, zkmips_amd/recursion_verifier.py), are padded to the first fitting
    RecursionShapeConfig shape, and are set up (proving key by preprocessed-trace digest, zkm_setup when
    new) and proven on the GPU as soon as their witness exists.  `value` is end to end (witness generation
    overlapped with proving, every setup inside), `prove_only` counts the time a proof was on the GPU."""
    from zkmips_amd import compress_tree as CT
    from zkmips_amd import recursion_verifier as RV
    import shutil
    import tempfile
    leaf_log = leaf_log or args.leaf_log
    if leaves_job is None:  # generated here (the default line submits it to the pool earlier)
        d = tempfile.mkdtemp(prefix="zkm_cl_", dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
        leaves_job = (pool.submit(_compress_leaves_job, d, n_leaves, 22 - leaf_log), d)
    fut, d = leaves_job
    try:
        meta, info, gen_s = fut.result()
        run = _load_tendermint(d, meta)
    finally:
        shutil.rmtree(d, ignore_errors=True)
    leaves, info = mips_leaves(dev, args.queries, run, dict(info, leaf_generation_s=round(gen_s, 1)))
    # warm-up (untimed): node witnesses and proofs of the first leaves (JIT modules, allocator pools; the keys are
    # dropped), and in every witness worker the program templates of the tree's first layers and of its right
    # spine, built from real chaining children (CT.prebuild_template) -- the reference holds its recursion programs
    # ready per shape (prover/src/lib.rs:366-410: join programs precomputed, core programs in an LRU by shape)
    warm, wst = CT.GpuProvers(dev), CT.TreeStats()

    def wprove(children, **fl):
        w = CT.node_witness(children, True, True, True, False, **fl)
        pr = warm.get(w[0], wst)
        return CT.compress_child_vk(pr.vk_commit, w[3]), pr.prove_shard(CT.materialize(w[1]), w[2])
    cur = list(leaves[:8])
    for depth in range(3):
        if len(cur) < 2:
            break
        if hasattr(pool, "run_all"):
            pool.run_all(CT.prebuild_template, CT.by_ref(cur[:2]), is_first=depth == 0)
        if depth == 2 or len(cur) < 4:
            break
        cur = [wprove(cur[i:i + 2], is_first=depth == 0 and i == 0) for i in range(0, len(cur) - 1, 2)]
    # the execution's last leaf is its memory shard, another proof shape: the programs of the tree's right spine
    # (its layer-1 node, and the layer-2 node over it) are other structures, known from the shard shapes as well
    if len(leaves) >= 4 and hasattr(pool, "run_all"):
        pool.run_all(CT.prebuild_template, CT.by_ref(leaves[-2:]))
        if len(leaves) >= 8:
            pool.run_all(CT.prebuild_template, CT.by_ref([wprove(leaves[-4:-2]), wprove(leaves[-2:])]))
    del warm, cur
    (rvk, rproof), r = compress_tree_run(pool, dev, leaves, inflight, distributed=world > 1)
    n = r["proofs"]
    nodes = len(leaves) - 1  # a binary tree over the leaves (odd nodes carried up) has leaves - 1 nodes
    out = {"metric": f"compress proofs/sec, end to end ({len(leaves)}-leaf compress tree = {nodes} recursion-machine "
                     f"proofs, BASELINE config 5), leaves of Cpu 2^{leaf_log} rows",
           "value": round(nodes / r["wall_s"], 3), "unit": "proofs/s", "tree_wall_s": round(r["wall_s"], 3),
           "prove_only": {"value": round(nodes / r["gpu_busy_s"], 3), "unit": "proofs/s",
                          "gpu_busy_s": round(r["gpu_busy_s"], 3),
                          "what": f"{nodes} proofs over the time at least one node proof was on the GPU"},
           "witness_generation": {"build_s_per_node": round(r["witness_build_s"] / max(1, n), 3),
                                  "execute_and_traces_s_per_node": round(r["witness_execute_and_traces_s"] / max(1, n), 3),
                                  "workers": args.node_workers,
                                  "what": "host: node program (verifying both children) + recursion runtime + traces, "
                                          "in a process pool, overlapped with proving"},
           "timeline": r["timeline"],
           "setups": r["setups"], "setup_ms_total": round(1e3 * r["setup_s"], 3), "setup_lookups": r["lookups"],
           "node_shapes": r["shapes"], "root_proof_bytes": len(rproof), "proofs_this_rank": n,
           "leaves": info, "in_flight": inflight,
           "node_program": "verifies each child: transcript replay, PoW, query bits, Merkle paths of every opening, "
                           "FRI reduced openings and folds, out-of-domain constraint check of every chip against the "
                           "quotient, local cumulative sum; then the reference's public-value checks (core.rs over "
                           "shard leaves: shard / execution-shard / pc chaining, address bits, digests, exit code, "
                           "first-shard conditions; compress.rs over node children: vk membership in the dummy vk "
                           "Merkle tree, child digests, chaining) and the septic-curve sum of the global sums; "
                           "assert_complete at the root; RecursionShapeConfig::fix_shape padding",
           "root_is_complete": bool(int(RV.parse_shard_proof(rproof).pv[220]))}
    return out, (rvk, rproof)


def compress_bench(args):
    """BASELINE config 5 as its own bench line (`--workload compress`): compress_leg on N ranks (the tree
    dealt by leaf blocks, zkmips_amd/compress_tree.reduce_distributed), plus the CPU oracle on one node
    proof (the CPU baseline, byte-identical to the GPU's)."""
    pool = start_witness_pool(max(1, min(args.node_workers, 32)))
    import torch
    from zkmips_amd import compress_tree as CT
    from zkmips_amd._lib import Device
    rk = Ranks(args, bind=False)
    dev = Device(rk.local_rank)
    rk.barrier()
    res, root = compress_leg(args, pool, dev, rk.world, rk.rank, args.inflight)
    res["ms_per_proof"] = round(1e3 * res["tree_wall_s"] / 63, 3)
    rk.barrier()
    wall = rk.max_over_ranks(res["tree_wall_s"])
    line = {"metric": res.pop("metric"), "value": round(63 / wall, 3), "unit": "proofs/s", "n_gpus": rk.world,
            "steps": 1, "warmup": 1, "ms_per_step": round(1e3 * wall, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "u32 (KoalaBear mod p, EF = F[X]/(X^4-3))",
            "data": "64 real MIPS leaf proofs (reference maximal shape scaled to Cpu 2^16, 84 queries)",
            "config": {"workload": "compress tree: 63 compress-machine shards verifying two child proofs each, "
                                   "blowup 4, 42 queries", "parallelism": f"tree dealt by leaf blocks over {rk.world} ranks"}}
    line.update({k: v for k, v in res.items() if k != "value"})
    cpu = None
    if not args.no_cpu_baseline and rk.rank == 0 and rk.world == 1:
        from tests import _oracle as O
        wit = CT.node_witness([root, root])
        cm = CT.GpuProvers(dev)
        gpu = cm.get(wit[0], CT.TreeStats()).prove_shard(wit[1], wit[2])
        o = O.OracleProver(cm.machine, wit[0], **cm.kw)
        tc = time.time()
        rc, ref = o.prove(wit[1], wit[2])
        dt = time.time() - tc
        assert rc == 0 and ref == gpu, "GPU compress proof differs from the CPU oracle"
        cpu = {"value": round(1.0 / dt, 4), "unit": "compress proofs/s", "cores": cpu_threads(), "kind": "port",
               "host": host_info(), "sample": f"one layer-7 compress-node proof (verifying the root twice; blowup 4, "
                                               f"42 queries), {dt:.2f} s wall; byte-identical to the GPU proof"}
    line["cpu_baseline"] = cpu
    pool.shutdown()
    if rk.rank == 0:
        print(json.dumps(line), flush=True)
    rk.close()


def pmc_child(args):
    """Runs under rocprofv3 counter passes (pmc_in_run): setup, then the same shard proven twice."""
    from zkmips_amd._lib import Device
    from zkmips_amd.prover import HipProver
    m, prep, traces, pvs = make_shard(args.workload, 1 << args.log_n, 1000)
    prover = HipProver(Device(0), m, prep, num_queries=args.queries)
    a = prover.prove_shard(traces, pvs)
    b = prover.prove_shard(traces, pvs)
    assert a == b


def bind_near_gpu(device: int):
    """Pin this rank's host threads to the CPUs of its GPU's NUMA node (sysfs local_cpulist of the GPU's
    PCI function), intersected with the CPUs this process may use, so the page-locked trace buffers it
    then allocates (first touch) and the DMA reads of them stay on the GPU's socket.  Best effort:
    returns the CPU list used, or None when the topology is not visible."""
    try:
        hip = C.CDLL("libamdhip64.so")
        buf = C.create_string_buffer(64)
        if hip.hipDeviceGetPCIBusId(buf, 64, device) != 0:
            return None
        bus = buf.value.decode().lower()
        with open(f"/sys/bus/pci/devices/{bus}/local_cpulist") as f:
            spec = f.read().strip()
        cpus = set()
        for part in spec.split(","):
            a, _, b = part.partition("-")
            cpus.update(range(int(a), int(b or a) + 1))
        cpus &= os.sched_getaffinity(0)
        if not cpus:
            return None
        os.sched_setaffinity(0, cpus)
        return f"{bus}: {len(cpus)} CPUs ({spec})"
    except (OSError, ValueError, AttributeError):
        return None


def launch_ranks(n: int, argv) -> int:
    """`bench.py --gpus N` with no external launcher: start N rank processes of this script (RANK =
    LOCAL_RANK = r, WORLD_SIZE = N, rendezvous on 127.0.0.1) before anything touches a GPU, wait for
    them, and return the worst exit code.  If a rank fails, the others are stopped (by their PIDs), so
    a failed rank cannot leave the rest waiting in a collective."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0:
                rc = rc or code
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc if rc >= 0 else 128 - rc


class ShardBench:
    """`K` in-flight slots proving shards of one workload on this rank's GPU, in four modes:
    "pipelined" (the headline: page-locked host traces, the H2D DMA of steps j+1..j+depth on the copy
    stream while step j proves from another HBM buffer), "records" (maximal shape: the executor's event
    records are what crosses PCIe, pipelined the same way, and each step builds its traces on the device
    from them -- the trait's own generate_traces, prover.rs:70-108 -- before proving), "per_call"
    (zkm_prove_shard copies the pinned host traces itself) and "resident" (traces already in HBM)."""

    def __init__(self, args, rk, workload, n, K, records: bool = False):
        import torch
        from zkmips_amd._lib import Device
        from zkmips_amd.prover import HipProver
        self.args, self.rk, self.K = args, rk, K
        self.shards = []
        one = None
        if workload in ("core", "maxshape"):  # one program (one proving key), generated once, proven K times
            t0 = time.time()
            one = make_shard(workload, n, 1)
            self.gen_s = time.time() - t0
        self.depth = max(1, getattr(args, "h2d_depth", 2))  # copies in flight ahead of the proving step
        nbuf = self.depth + 1
        self.records = None
        if records:
            # the executor's records as the header's structs (converted once, outside any timed region: the
            # reference's executor hands its event vectors as they lie), page-locked
            from zkmips_amd import tracegen as TG
            host = TG.shard_records(_CAPTURE[workload])
            self.records = {"_n": {kk: len(v) for kk, v in host.items()}, "pinned": {}}
            for kk, v in host.items():
                raw = np.ascontiguousarray(v).view(np.uint8).reshape(-1)
                t = torch.empty(max(1, raw.size), dtype=torch.uint8, pin_memory=True)
                t.numpy()[:raw.size] = raw
                self.records["pinned"][kk] = t
        for k in range(K):
            m, prep, traces_k, pvs_k = one if one is not None else make_shard(workload, n, 1000 + rk.rank * K + k)
            pinned = {}
            for kk, v in traces_k.items():
                pinned[kk] = torch.empty(v.shape, dtype=torch.int32, pin_memory=True)
                pinned[kk].numpy()[...] = v.view(np.int32)
            self.shards.append(({kk: torch.from_numpy(v.view(np.int32)).cuda() for kk, v in traces_k.items()}, pvs_k,
                                {kk: t.numpy().view(np.uint32) for kk, t in pinned.items()}, pinned,
                                [{kk: (torch.empty_like(t, device="cuda") if args.h2d_dst == "torch" else
                                       RawDev(t.shape, H2D_FLAGS[args.h2d_dst])) for kk, t in pinned.items()}
                                 for _ in range(nbuf)],
                                torch.cuda.Stream(),
                                # the records mode's HBM buffers (one set per step in flight)
                                [{kk: torch.empty_like(t, device="cuda") for kk, t in self.records["pinned"].items()}
                                 for _ in range(nbuf)] if records else None))
        if records:
            from zkmips_amd import mips_alu as A
            self.heights = {kk: int(v.shape[0]) for kk, v in self.shards[0][0].items() if kk not in ("Byte", "Program")}
            self.byte_mult = [torch.zeros((A.BYTE_ROWS, A.BYTE_MULT_WIDTH), dtype=torch.int32, device="cuda")
                              for _ in range(K)]
        self.m = m
        self.prover = HipProver(Device(rk.local_rank), m, prep, num_queries=args.queries)
        torch.cuda.synchronize()
        self.rows_per_shard = max(v.shape[0] for v in self.shards[0][2].values())
        self.stagger = None
        self.slot_waits = {}
        self.slot_proof_s = {}  # (mode, slot) -> host seconds of each zkm_prove_shard call
        self.slot_tracegen_s = {}  # slot -> host seconds of each records-mode trace build (waited for)
        import threading
        self.copy_lock = threading.Lock()
        self.copy_stream = torch.cuda.Stream() if os.environ.get("ZKM_BENCH_COPY_STREAMS") != "slot" else None

    def slot_steps(self, k, nsteps, mode):
        """nsteps shard proofs of in-flight slot k; returns the last proof."""
        import torch
        prover = self.prover
        dev_t, pv, host_np, host_t, bufs, cs, rbufs = self.shards[k]
        if mode == "records":
            bufs = rbufs
        if mode == "resident":
            pr = b""
            ts = []
            for _ in range(nsteps):
                t = time.perf_counter()
                pr = prove_resident(prover, dev_t, pv)
                ts.append(time.perf_counter() - t)
            self.slot_proof_s[(mode, k)] = ts
            return pr
        if mode == "per_call":
            pr = b""
            for _ in range(nsteps):
                pr = prover.prove_shard(host_np, pv)
            return pr

        # one copy stream for all slots (ZKM_BENCH_COPY_STREAMS=slot: one per slot): copies run FIFO at the full
        # PCIe rate in the order the slots issue them, instead of sharing the link and all landing late
        slot_stream = cs
        cs = self.copy_stream if self.copy_stream is not None else cs
        nbuf = len(bufs)
        src_t = self.records["pinned"] if mode == "records" else host_t

        def issue(j):
            b = bufs[j % nbuf]
            # one slot's copies go into the shared stream together (FIFO per slot, not interleaved per trace)
            with self.copy_lock, torch.cuda.stream(cs):
                for kk, t in src_t.items():
                    if isinstance(b[kk], RawDev):
                        b[kk].copy_from_host(t, cs)
                    else:
                        b[kk].copy_(t, non_blocking=True)
                e = torch.cuda.Event()
                e.record(cs)
            return e
        # per-slot copy streams: the slots' first copies go one after another (slot k starts when slot k-1's
        # has landed), so slot 0 proves after one copy time instead of all slots waiting for K copies sharing
        # PCIe (the shared FIFO stream orders them by itself)
        stagger = self.stagger if self.copy_stream is None else None
        if stagger is not None and k > 0:
            stagger[k - 1].wait(60)  # bounded: a failing slot must not hang the others
        evs = {0: issue(0)}  # step -> its copies' event; the look-ahead copies are issued once step 0's landed
        pr = b""
        waits, ts = [], []
        for j in range(nsteps):
            t = time.perf_counter()
            evs.pop(j).synchronize()
            waits.append(time.perf_counter() - t)
            if j == 0 and stagger is not None:
                stagger[k].set()
            for jj in range(j + 1, min(nsteps, j + 1 + self.depth)):
                if jj not in evs:  # buffer jj % nbuf last served step jj - nbuf <= j - 1: proven already
                    evs[jj] = issue(jj)
            # ZKM_BENCH_DMA_PROBE=1 (experiment only): the same copies, proofs from the resident traces
            src = dev_t if os.environ.get("ZKM_BENCH_DMA_PROBE") == "1" else bufs[j % nbuf]
            t = time.perf_counter()
            if mode == "records":
                src = self.traces_from_records(k, src, slot_stream)
                self.slot_tracegen_s.setdefault(k, []).append(time.perf_counter() - t)
            pr = prove_resident(prover, src, pv)
            ts.append(time.perf_counter() - t)
        self.slot_waits[k] = waits  # host seconds each step waited for its traces' copy
        self.slot_proof_s[(mode, k)] = ts
        return pr

    def traces_from_records(self, k, recs, stream):
        """Slot k's shard traces built on the device (zkmips_amd/tracegen.shard_traces, every chip at the
        shape's height, Byte and Program multiplicities included) from its records in HBM, on its stream,
        waited for."""
        import torch
        from zkmips_amd import tracegen as TG
        bm = self.byte_mult[k]
        with torch.cuda.stream(stream):
            bm.zero_()
            tr = TG.shard_traces(_CAPTURE["maxshape"], byte_mult=bm, heights=self.heights,
                                 records=dict(recs, _n=self.records["_n"]))
            tr["Byte"] = bm
            stream.synchronize()
        return {kk: tr[kk] for kk in self.shards[k][0]}  # the shard's chips, in the host-trace order

    def run_steps(self, nsteps, mode="pipelined"):
        """nsteps shard proofs per in-flight slot; returns the last proof of slot 0, after gathering
        every rank's to rank 0 (the MachineProof aggregation, RCCL over xGMI)."""
        import threading
        K = self.K
        if K == 1:
            proof = self.slot_steps(0, nsteps, mode)
        else:
            self.stagger = ([threading.Event() for _ in range(K)]
                            if mode == "pipelined" and os.environ.get("ZKM_NO_STAGGER") != "1" else None)
            out = [b""] * K

            def slot(k):
                out[k] = self.slot_steps(k, nsteps, mode)
            th = [threading.Thread(target=slot, args=(k,)) for k in range(K)]
            for t in th:
                t.start()
            for t in th:
                t.join()
            proof = out[0]
        if self.rk.world > 1:
            from zkmips_amd.dist import gather_proofs_to_root
            got = gather_proofs_to_root({self.rk.rank: proof}, device=self.rk.coll_dev)
            assert self.rk.rank != 0 or sorted(got) == list(range(self.rk.world)), "a rank's proof is missing"
        return proof

    def timed(self, nsteps, mode):
        """`nsteps` batches of K concurrent shard proofs, barrier + sync on both sides, max over ranks."""
        self.rk.barrier()
        t0 = time.perf_counter()
        pr = self.run_steps(nsteps, mode)
        self.rk.barrier()
        return pr, self.rk.max_over_ranks(time.perf_counter() - t0)


_T0 = time.time()


def progress(msg: str):
    """A progress line on stderr (rank 0): the one JSON line stays alone on stdout, and a long default run
    keeps writing while it works."""
    if os.environ.get("RANK", "0") == "0":
        sys.stderr.write(f"[bench {time.time() - _T0:7.1f} s] {msg}\n")
        sys.stderr.flush()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); without an external launcher bench.py starts them itself")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--log-n", type=int, default=22)
    ap.add_argument("--sha-blocks", type=int, default=16384, help="sha2 workload: 64-byte blocks hashed")
    ap.add_argument("--h2d-dst", choices=["torch", "uncached", "finegrained"], default="torch",
                    help="memory type of the HBM buffers the pipelined H2D copies land in")
    ap.add_argument("--h2d-depth", type=int, default=2,
                    help="host-trace / records modes: steps whose copies are issued ahead of the proving step")
    ap.add_argument("--sha-events-per-shard", type=int, default=16384,
                    help="sha2 workload: precompile calls per precompile shard")
    ap.add_argument("--workload", choices=["fib", "alu", "core", "maxshape", "sha2", "tendermint", "tracegen", "compress"],
                    default="fib",
                    help="fib: S-SHARD FibCpu (the headline config); alu: MIPS ALU slice (AddSub, Bitwise, Lt, "
                         "ShiftLeft, ShiftRight, CloClz, Byte restated from the reference AIRs + CPU stand-in, "
                         "zkmips_amd/mips_alu.py), 2^(log-n) "
                         "instructions per shard; core: Cpu + Program + Mul + DivRem + Branch + Jump + MovCond + MemoryInstrs + MiscInstrs chips over the ALU slice "
                         "(zkmips_amd/mips_core.py) running a counted loop, Cpu 2^(log-n) rows; maxshape: a MIPS shard "
                         "padded to the reference's maximal_shapes.json[\"22\"][2] (zkmips_amd/shapes.py)")
    ap.add_argument("--queries", type=int, default=84)
    ap.add_argument("--cpu-log-n", type=int, default=22)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-maxshape", action="store_true",
                    help="skip the default line's secondary leg: the reference's maximal 2^22 MIPS shard shape")
    ap.add_argument("--maxshape-steps", type=int, default=8)
    ap.add_argument("--no-compress", action="store_true",
                    help="skip the default line's compress leg (config 5: 64 MIPS leaves, 63 node proofs)")
    ap.add_argument("--no-tendermint", action="store_true",
                    help="skip the default line's config-4 leg (the tendermint guest on the reference's blocks)")
    ap.add_argument("--no-sizes", action="store_true",
                    help="skip the default line's size series (resident rows/s and LDE time at 2^20, 2^21, 2^23)")
    ap.add_argument("--no-leaf21", dest="leaf21", action="store_false",
                    help="skip the default line's compress_2e21 leg (a 4-leaf tree of 2^21-row MIPS shards)")
    ap.add_argument("--leaf-log", type=int, default=16, help="compress leg: MIPS leaf shards in the maximal shape scaled to Cpu 2^leaf_log rows")
    ap.add_argument("--node-workers", type=int, default=12,
                    help="compress workload: processes generating node witnesses (the box allots 16 CPUs per GPU)")
    ap.add_argument("--no-pmc", action="store_true", help="skip the in-run rocprofv3 HBM counter passes")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--profile-out", default="")
    ap.add_argument("--profile-steps", type=int, default=3, help="single-shard proofs in the profiled region")
    ap.add_argument("--inflight", type=int, default=3,
                    help="shards proven concurrently per GPU (one host thread + HIP stream each), as the "
                         "reference's prove_with_context runs commit/open for all shards of a batch at once")
    args = ap.parse_args()
    if args.gpus is not None and args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if args.pmc_child:
        return pmc_child(args)
    if args.workload in ("sha2", "tendermint"):
        return execution_bench(args)
    if args.workload == "tracegen":
        return tracegen_bench(args)
    if args.workload == "compress":
        return compress_bench(args)
    # the default line's compress leg (config 5): its witness pool starts before the GPU is touched
    pool = tm_future = tm_dir = None
    if (not (args.no_compress and args.no_tendermint) and args.workload == "fib"
            and int(os.environ.get("WORLD_SIZE", "1")) == 1 and not args.pmc_child):
        pool = start_witness_pool(max(1, min(args.node_workers, 32)))
    leaves_job = leaves21_job = None

    import torch
    rk = Ranks(args)
    world, rank, local_rank, numa = rk.world, rk.rank, rk.local_rank, rk.numa

    from zkmips_amd import workloads as W
    from zkmips_amd._lib import lib

    n = 1 << args.log_n
    K = max(1, args.inflight)
    progress(f"{args.workload} 2^{args.log_n}: generating the shard, setting up")
    sb = ShardBench(args, rk, args.workload, n, K)
    prover, m = sb.prover, sb.m
    dev_traces, pvs, traces = sb.shards[0][0], sb.shards[0][1], sb.shards[0][2]
    rows_per_shard = sb.rows_per_shard
    if args.warmup:
        sb.run_steps(args.warmup, "pipelined")
        sb.run_steps(1, "resident")
        sb.run_steps(1, "per_call")
    # timed region (the headline `value`): traces in page-locked host memory, their H2D
    # inside the span (pipelined: the next shards' copies overlap the current proof), commit + open + D2H of
    # the proof
    progress("timed regions: host traces (headline), resident, per-call copies")
    proof, elapsed = sb.timed(args.steps, "pipelined")
    copy_waits = {k: list(v) for k, v in sb.slot_waits.items()}
    # secondary: the same steps with the traces already in HBM, and with per-call host copies
    proof_res, elapsed_res = sb.timed(args.steps, "resident")
    proof_ms = {m: round(1e3 * float(np.mean([t for (mm, _), v in sb.slot_proof_s.items() if mm == m for t in v])), 3)
                for m in ("resident", "pipelined")}
    proof_pc, elapsed_pc = sb.timed(args.steps, "per_call")
    assert proof_res == proof == proof_pc, "resident / host-trace proofs differ"
    if pool is not None and not args.no_tendermint and rank == 0:
        # config 4's traces are generated on the host (a pool worker) while the later GPU legs run -- after
        # the timed regions above, so that they measure the prover alone
        import tempfile
        tm_dir = tempfile.mkdtemp(prefix="zkm_tm_", dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
        tm_future = pool.submit(_tendermint_job, tm_dir)
    if pool is not None and not args.no_compress and rank == 0:
        # config 5's leaf execution is traced on the host in a pool worker while the later GPU legs run
        import tempfile
        d = tempfile.mkdtemp(prefix="zkm_cl_", dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
        leaves_job = (pool.submit(_compress_leaves_job, d, 64, 22 - args.leaf_log), d)
        if args.leaf21:
            d21 = tempfile.mkdtemp(prefix="zkm_cl21_", dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
            leaves21_job = (pool.submit(_compress_leaves_job, d21, 4, 1), d21)

    if rank != 0:
        rk.close()
        return

    # profiled region: single-shard latency with per-stage HIP events on the launching stream
    # (one shard in flight, so a stage's events bracket only its own kernels); the roofline and
    # the stage table come from here, the throughput `value` from the timed region above
    nprof = max(1, args.profile_steps)
    progress("profiled region")
    prof, serial_ms, prof_text = profile_proofs(prover, dev_traces, pvs, nprof)

    # the PCIe ceiling of the host-trace mode: one shard's page-locked traces copied alone
    import torch
    h2d_s = []
    for _ in range(3):
        _, _, _, host_t, bufs, cs, _ = sb.shards[0]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(cs):
            for kk, t in host_t.items():
                b = bufs[0][kk]
                b.copy_from_host(t, cs) if isinstance(b, RawDev) else b.copy_(t, non_blocking=True)
        cs.synchronize()
        h2d_s.append(time.perf_counter() - t0)
    h2d_alone_s = min(h2d_s)

    # single-shard latency from pageable host memory (the runtime stages the copy)
    tp = time.perf_counter()
    prover.prove_shard({kk: np.array(v) for kk, v in traces.items()}, pvs)
    pageable_s = time.perf_counter() - tp

    # HBM bytes per kernel of one shard proof, measured on this box now (rank 0, N = 1 only)
    if not (args.no_pmc or world > 1 or args.workload == "maxshape"):
        progress("rocprofv3 counter passes")
    pmc = None if (args.no_pmc or world > 1 or args.workload == "maxshape") else pmc_in_run(args)
    kernel_stages = ["lde", "merkle_leaves", "merkle_nodes", "quotient", "perm_trace", "open_eval", "fri_reduce"]
    dom = max((s for s in kernel_stages if s in prof), key=lambda s: prof[s][1])
    cnt, ms, units = prof[dom]
    achieved = units / (ms / 1e3) / 1e9  # GB/s, algorithmic bytes / measured stage time
    tb, tn = stage_traffic(pmc, dom)
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                # PMC bytes per proof over the stage's launches per proof (the stage brackets every kernel
                # it runs, e.g. a commit's leaf hashing plus its injected shorter matrices), the same
                # denominator as algorithmic_bytes_per_launch
                "traffic": round(tb / (cnt / nprof)) if tb else None, "kernel": dom,
                "launches": cnt, "avg_ms": round(ms / cnt, 4),
                "algorithmic_bytes_per_launch": round(units / cnt),
                "traffic_source": "rocprofv3 FETCH_SIZE/WRITE_SIZE passes in this run (2xFETCH+WRITE)" if tb else None}
    if dom == "merkle_leaves" and "merkle_leaves_perms" in prof:
        roofline["valu"] = valu_roofline(prof["merkle_leaves_perms"][2], ms)
        vc = valu_counters(pmc, ms / nprof)
        if roofline["valu"] is not None and vc:
            roofline["valu"]["counters"] = vc
        lds = lds_counters(pmc)
        if roofline["valu"] is not None and lds:
            roofline["valu"]["lds"] = lds

    def measured(stage):
        """HBM utilisation of a stage's kernels: PMC bytes per proof over the stage's HIP-event time."""
        b_, n_ = stage_traffic(pmc, stage)
        if not b_ or stage not in prof:
            return None
        sms = prof[stage][1] / nprof
        gbps = b_ / (sms / 1e3) / 1e9
        out = {"GBps": round(gbps, 1), "frac": round(gbps / HBM_PEAK_GBS, 4), "bytes_per_shard": round(b_),
               "algorithmic_bytes_per_shard": round(prof[stage][2] / nprof),
               "counter_ratio": round(b_ / (prof[stage][2] / nprof), 3), "launches": n_,
               "stage_ms_per_shard": round(sms, 3)}
        # the same kernels' VALU side from the SQ pass: VALU instructions x 2 cycles (wave64 on SIMD-32) over
        # the 1024 SIMDs x busy cycles -- a lower bound on the issue fraction (half-rate 64-bit products
        # count once)
        pre = STAGE_KERNELS.get(stage, ())
        vi = cy = 0.0
        for k, v in (pmc or {}).items():
            c = v.get("sq") or {}
            if k.startswith(pre) and c.get("GRBM_GUI_ACTIVE"):
                vi += c.get("SQ_INSTS_VALU", 0.0)
                cy += c["GRBM_GUI_ACTIVE"] / 8.0
        if cy:
            out["valu_issue_lower_bound"] = round(vi * 2.0 / (1024.0 * cy), 4)
        return out

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
        meas = measured("lde")
        if meas:
            ntt["hbm_measured"] = meas
    hbm_kernels = {name: measured(st) for name, st in (("quotient", "quotient"), ("logup_trace", "perm_trace"),
                                                       ("fri_reduce", "fri_reduce"), ("openings", "open_eval"),
                                                       ("merkle_leaves", "merkle_leaves"))}
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
        "data": ("synthetic (seeded S-SHARD traces, SURVEY.md §8d) in page-locked host memory: their H2D and the "
                 "proof's D2H inside the timed span"),
        "config": {"workload": (f"S-SHARD FibCpu 2^{args.log_n} rows (main 67, LogUp 11 EF, quotient 2) + FibTable "
                                f"2^{W.fib_table_height(n).bit_length() - 1} (prep 2): full commit+open per shard")
                   if args.workload == "fib" else
                   (f"MIPS core shard: a counted loop (60-instruction body of ALU and load/store ops, forward branches, jal/jalr calls "
                    f"of a subroutine, bal) "
                    f"executed to {int(traces['Cpu'][:, 65].sum())} instructions: Cpu 2^{args.log_n} (main 67, "
                    f"LogUp 11 EF) + Program (prep 14) + DivRem, AddSub, Bitwise, Mul, Lt, ShiftLeft, ShiftRight, CloClz, MovCond, MemoryInstrs, MiscInstrs, "
                    f"Branch, Jump, MemoryLocal, Global (septic-curve digest) + Byte 2^16 (prep 12): full commit+open per shard")
                   if args.workload == "core" else
                   (f"MIPS shard in the reference maximal shape maximal_shapes.json[\"22\"][2] scaled to Cpu 2^{args.log_n}: "
                    + ", ".join(f"{k} 2^{int(np.log2(len(traces[k])))}" for k in sorted(traces, key=lambda c: -len(traces[c])))
                    + f"; {int(traces['Cpu'][:, 65].sum())} instructions (loop of ALU, load/store, branch, conditional-move "
                      f"ops, HALT): full commit+open per shard")
                   if args.workload == "maxshape" else
                   (f"MIPS ALU slice: InstrSource 2^{args.log_n} + AddSub, Bitwise, Lt 2^{args.log_n - 2} + ShiftLeft, "
                    f"ShiftRight (CPU + CloClz SRLs) 2^{args.log_n - 3} + CloClz 2^{args.log_n - 4} + Byte 2^16 "
                    f"(prep 12): full commit+open per shard"),
                   "rows_per_shard": rows_per_shard, "fri_queries": args.queries, "pow_bits": 16, "log_blowup": 1,
                   "shards_per_gpu_per_step": K, "parallelism": f"shard-parallel x{world}, {K} in flight per GPU",
                   "proof_bytes": len(proof)},
        "host_per_call": {"value": round(world * K * rows_per_shard * args.steps / elapsed_pc, 1), "unit": "rows/s",
                          "ms_per_shard": round(1e3 * elapsed_pc / (args.steps * K), 3),
                          "what": "same steps, each zkm_prove_shard copies its pinned host traces itself (no look-ahead)"},
        "value_basis": ("SURVEY.md section 8d: traces in page-locked host memory when the timed region starts, "
                        "every H2D copy and each proof's D2H inside it (copies of the next shards overlap the "
                        "current proofs); the same steps from traces already in HBM are `resident`"),
        "resident": {"value": round(world * K * rows_per_shard * args.steps / elapsed_res, 1), "unit": "rows/s",
                     "ms_per_shard": round(1e3 * elapsed_res / (args.steps * K), 3),
                     "ms_per_step": round(1e3 * elapsed_res / args.steps, 3)},
        "host_traces": {"value": round(world * K * rows_per_shard * args.steps / elapsed, 1), "unit": "rows/s",
                        "ms_per_shard": round(1e3 * elapsed / (args.steps * K), 3),
                        "vs_resident": round(elapsed / elapsed_res, 3),
                        "copies_ahead": sb.depth,
                        "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                        "h2d_alone_ms_per_shard": round(h2d_alone_s * 1e3, 3),
                        "h2d_GBps": round(sum(v.nbytes for v in traces.values()) / h2d_alone_s / 1e9, 2),
                        "copy_wait_ms": {"first_step_per_slot": [round(1e3 * v[0], 2) for _, v in sorted(copy_waits.items())],
                                         "later_steps_per_slot": [round(1e3 * sum(v[1:]), 2)
                                                                  for _, v in sorted(copy_waits.items())]},
                        "copy_streams": "one FIFO stream for all slots" if sb.copy_stream is not None else "one per slot",
                        "proof_call_ms_mean": proof_ms,
                        "what": "same steps from page-locked host traces: the H2D DMA of each slot's next shard "
                                "overlaps the current proof, every copy inside the timed span; copy_wait_ms = host "
                                "time each slot waited for its traces (the first step's copies cannot overlap a "
                                "proof), h2d_alone_ms_per_shard = one shard's copy with nothing else running"},
        "h2d_bytes_per_shard": int(sum(v.nbytes for v in traces.values())),
        "host_threads_bound_to": numa,
        "pageable_single_shard_ms": round(pageable_s * 1e3, 3),
        "roofline": roofline,
        "ntt": ntt,
        "hbm_measured": {k: v for k, v in hbm_kernels.items() if v},
        "stages_ms_per_shard": stages,
        "profiled_region": f"{nprof} single-shard proofs after the timed region (stages, roofline, ntt, serial_ms_per_shard)",
    }
    def leg(name, fn):
        """A secondary leg: its failure is recorded in the line (and on stderr), not fatal to the headline."""
        progress(f"{name} leg")
        try:
            line[name] = fn()
        except Exception as e:  # noqa: BLE001 -- reported, the headline stands
            import traceback
            traceback.print_exc()
            line[name] = {"error": f"{type(e).__name__}: {e}"}
    if not args.no_sizes and world == 1 and args.workload == "fib":
        leg("sizes", lambda: size_series(args, prover, K))
    if not args.no_maxshape and world == 1 and args.workload == "fib":
        leg("maxshape", lambda: maxshape_leg(args, rk, n, K))
    if pool is not None and not args.no_compress:
        leg("compress", lambda: compress_leg(args, pool, prover.dev, leaves_job=leaves_job)[0])
    if pool is not None and not args.no_compress and args.leaf21:
        # the reference's default shard size (2^21 Cpu rows, crates/stark/src/opts.rs:6): a 4-leaf tree (3 CPU
        # shards + the memory shard of one execution), so the node programs verify 2^21-row leaves
        leg("compress_2e21", lambda: compress_leg(args, pool, prover.dev, leaves_job=leaves21_job, n_leaves=4,
                                                  leaf_log=21)[0])
    if tm_future is not None:
        import shutil
        try:
            leg("tendermint", lambda: tendermint_leg(args, tm_future.result(), tm_dir, rk))
        finally:
            shutil.rmtree(tm_dir, ignore_errors=True)
    if pool is not None:
        pool.shutdown()
    if not args.no_cpu_baseline and world == 1:
        leg("cpu_baseline", lambda: cpu_baseline(args.cpu_log_n, args.queries))
    if args.profile_out:
        with open(args.profile_out, "w") as f:
            f.write(prof_text)
    print(json.dumps(line), flush=True)
    rk.close()


if __name__ == "__main__":
    main()
