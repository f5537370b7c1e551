"""Syscalls and the SHA-256 precompiles across shards: SyscallInstrs / SyscallCore in the CPU shards,
SyscallPrecompile + ShaExtend in the precompile shard, the syscall's memory accesses closed through
MemoryLocal on both sides, COMMIT / HALT against the public values, and the machine-level global sum.

The SHA-256 schedule the precompile computes is pinned to hashlib: a SHA-256 compression built on
`sha256_extend_ref` (FIPS 180-4 §6.2.2) reproduces hashlib's digests."""
import hashlib
import struct

import numpy as np
import pytest

from tests import _air_check
from tests import _oracle as O
from zkmips_amd import mips_core as C
from zkmips_amd import mips_memory as MM
from zkmips_amd import mips_syscall as SY
from zkmips_amd import septic as S
from zkmips_amd.proof import machine_global_sum_is_zero

_K = [0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
      0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
      0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
      0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
      0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
      0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
      0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
      0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2]
_H0 = [0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19]


def _compress(h, w):
    rot = lambda x, s: ((x >> s) | (x << (32 - s))) & 0xFFFFFFFF
    a, b, c, d, e, f, g, hh = h
    for i in range(64):
        s1 = rot(e, 6) ^ rot(e, 11) ^ rot(e, 25)
        ch = (e & f) ^ (~e & g)
        t1 = (hh + s1 + ch + _K[i] + w[i]) & 0xFFFFFFFF
        s0 = rot(a, 2) ^ rot(a, 13) ^ rot(a, 22)
        maj = (a & b) ^ (a & c) ^ (b & c)
        t2 = (s0 + maj) & 0xFFFFFFFF
        a, b, c, d, e, f, g, hh = (t1 + t2) & 0xFFFFFFFF, a, b, c, (d + t1) & 0xFFFFFFFF, e, f, g
    return [(x + y) & 0xFFFFFFFF for x, y in zip(h, [a, b, c, d, e, f, g, hh])]


def _sha256(msg: bytes) -> bytes:
    ml = len(msg) * 8
    msg = msg + b"\x80" + b"\0" * ((55 - len(msg)) % 64) + struct.pack(">Q", ml)
    h = list(_H0)
    for k in range(0, len(msg), 64):
        h = _compress(h, SY.sha256_extend_ref(struct.unpack(">16I", msg[k:k + 64])))
    return struct.pack(">8I", *h)


@pytest.mark.parametrize("msg", [b"", b"abc", bytes(range(200))])
def test_schedule_pinned_to_hashlib(msg):
    assert _sha256(msg) == hashlib.sha256(msg).digest()


def _execute(prog, seed=1):
    state, regs = C.fresh_state(), C.initial_registers(seed)
    C.program_shard(prog, seed, 1, 1 << 20, state=state, regs=regs)
    return state, regs


def test_sha_syscalls_compute_sha256():
    """SHA_EXTEND leaves the FIPS schedule of the buffer's first 16 words in it; SHA_COMPRESS folds it
    into the state at SHA_H_PTR, which after the guest's blocks equals the SHA-256 chaining value of
    those blocks (the compression pinned to hashlib above); V0 keeps the syscall code; HALT stops the
    program with exit code A0."""
    prog = C.sha_program(3, seed=4)
    state, regs = _execute(prog, seed=4)
    assert state["exit_code"] == 0 and state["pc"] == 0
    codes = [ev[0] for ev in state["precompile"]]
    assert codes == [SY.SHA_EXTEND, SY.SHA_COMPRESS] * 3
    h = list(C.SHA_H0)
    for code, (shard, clk, sid, arg1, arg2), ev in state["precompile"]:
        if code == SY.SHA_EXTEND:
            assert sid == 5 and arg2 == 0
            w16 = [r[0] for r in ev["r16"][:16]]  # reads of w[0..15]
            w = SY.sha256_extend_ref(w16)
            assert [wr[1] for wr in ev["wr"]] == w[16:]
        else:
            assert sid == 6 and (arg1, arg2) == (ev["w_ptr"], C.SHA_H_PTR)
            assert [r[0] for r in ev["wr"]] == w
            h = _compress(h, w)
            assert [x[1] for x in ev["hw"]] == h
    assert [state["mem"][C.SHA_H_PTR + 4 * i] for i in range(8)] == h
    assert regs[SY.REG_V0] == SY.HALT


@pytest.fixture(scope="module")
def run():
    return C.program_shards(C.sha_program(5, seed=2), seed=2, shard_size=150)


def test_syscall_shards_satisfy_air(run):
    kinds = [("Cpu" in tr, "ShaExtend" in tr, "ShaCompress" in tr, "MemoryGlobalInit" in tr) for _, _, tr, _ in run]
    assert kinds[-3:] == [(False, True, False, False), (False, False, True, False), (False, False, False, True)]
    assert all(k == (True, False, False, False) for k in kinds[:-3])
    for m, prep, tr, pv in run:
        assert _air_check.check(m, {k: v for k, v in prep.items() if v is not None}, tr, pv) == ([], [])
    cpu = [tr for _, _, tr, _ in run if "Cpu" in tr]
    assert sum(int(t["SyscallInstrs"][:, SY.SI_REAL].sum()) for t in cpu if "SyscallInstrs" in t) == 12
    assert sum(int(t["SyscallCore"][:, SY.SC_REAL].sum()) for t in cpu if "SyscallCore" in t) == 10
    ext, cmp_ = run[-3][2], run[-2][2]
    assert int(ext["SyscallPrecompile"][:, SY.SC_REAL].sum()) == 5
    assert int(ext["ShaExtend"][:, SY.SE_REAL].sum()) == 5 * 48
    assert int(cmp_["SyscallPrecompile"][:, SY.SC_REAL].sum()) == 5
    assert int(cmp_["ShaCompress"][:, SY.SC2_REAL].sum()) == 5 * 80


def test_closing_shards_keep_the_last_execution_shard(run):
    """The precompile and memory shards of a finished execution carry the last CPU shard's execution_shard
    (crates/core/machine/src/utils/prove.rs:308-311: no increment on the `done` path)."""
    cpu = [pv for _, _, tr, pv in run if "Cpu" in tr]
    rest = [pv for _, _, tr, pv in run if "Cpu" not in tr]
    assert len(rest) == 3 and [int(pv[C.PV_EXECUTION_SHARD]) for pv in cpu] == list(range(1, len(cpu) + 1))
    assert all(int(pv[C.PV_EXECUTION_SHARD]) == len(cpu) for pv in rest)


def test_halt_and_commit_public_values(run):
    _, _, tr, pv = [r for r in run if "Cpu" in r[2]][-1]
    assert pv[C.PV_NEXT_PC] == 0 and pv[SY.PV_EXIT_CODE] == 0
    si = tr["SyscallInstrs"]
    commit = si[(si[:, SY.SI_REAL] == 1) & (si[:, SY.SI_PREV_A] == SY.COMMIT)]
    assert len(commit) == 1
    assert list(pv[12:16]) == list(commit[0, SY.SI_C:SY.SI_C + 4])  # digest word 3


def test_cpu_memory_entries_split_at_syscalls():
    """A buffer word written by the CPU, read by SHA_EXTEND, then written again by the CPU in the same
    shard has two MemoryLocal entries there: the syscall's access closes the first
    (SyscallContext::postprocess)."""
    run = C.program_shards(C.sha_program(3, seed=3, compress=False), seed=3, shard_size=1 << 12)
    tr = run[0][2]
    ent = MM.local_entries(tr["MemoryLocal"])
    w0 = C.DATA_BASE + 0x400
    rows = ent[ent[:, 0] == w0]
    assert len(rows) == 2
    first, second = sorted(rows.tolist(), key=lambda e: e[2])
    pre = [e for e in MM.local_entries(run[1][2]["MemoryLocal"]).tolist() if e[0] == w0]
    # the syscall's entry continues the CPU's first one and hands over to the CPU's second one
    assert pre[0][1:4] == first[4:7] and pre[0][4:7] == second[1:4]


def test_global_sum_over_shards_is_zero(run):
    digs = np.asarray([C.shard_global_digest(tr) for _, _, tr, _ in run])
    assert np.array_equal(S.digest_sum(digs), S.CURVE_CUMULATIVE_SUM_START)
    without_pre = np.concatenate([digs[:-3], digs[-2:]])
    assert not np.array_equal(S.digest_sum(without_pre), S.CURVE_CUMULATIVE_SUM_START)


@pytest.mark.parametrize("what", ["schedule_word", "syscall_arg", "commit_pv", "rotate_carry", "round_state",
                                  "digest_write"])
def test_tamper_rejected(run, what):
    if what == "commit_pv":
        k = max(i for i, r in enumerate(run) if "Cpu" in r[2])
    elif what == "syscall_arg":
        k = 0
    elif what in ("round_state", "digest_write"):
        k = len(run) - 2
    else:
        k = len(run) - 3
    m, prep, tr, pv = run[k]
    bad = {n: v.copy() for n, v in tr.items()}
    pv = pv.copy()
    if what == "schedule_word":
        bad["ShaExtend"][5, SY.SE_WI + 4] ^= 1
    elif what == "syscall_arg":
        t = bad["SyscallCore"]
        t[0, SY.SC_ARG1] += 4
    elif what == "commit_pv":
        pv[12] ^= 1
    elif what == "rotate_carry":
        bad["ShaExtend"][7, SY.SE_RR7 + 8] ^= 1
    elif what == "round_state":  # a round's e word
        bad["ShaCompress"][30, SY.SC2_A + 16] ^= 1
    else:  # a finalize row's written digest word
        bad["ShaCompress"][75, SY.SC2_MEM + 4] ^= 1
    prep = {n: v for n, v in prep.items() if v is not None}
    assert _air_check.check(m, prep, bad, pv) != ([], [])
    pr = O.OracleProver(m, prep, num_queries=4)
    rc, p = pr.prove(bad, pv)
    assert pr.verify(p) != 0


def test_oracle_proofs_verify_and_sum_to_zero(run):
    m, prep, _, _ = run[0]
    pr = O.OracleProver(m, {k: v for k, v in prep.items() if v is not None}, num_queries=4)
    proofs = []
    for _, _, tr, pv in run:
        rc, p = pr.prove(tr, pv)
        assert rc == 0 and pr.verify(p) == 0
        proofs.append(p)
    assert machine_global_sum_is_zero(proofs)
    assert not machine_global_sum_is_zero(proofs[:-2] + proofs[-1:])  # the compress shard dropped


@pytest.mark.gpu
def test_syscall_gpu_proofs_identical(run):
    """Every shard (CPU shards with SyscallInstrs/SyscallCore, the SHA_EXTEND precompile shard, the memory
    shard) proves on the GPU byte-identical to the oracle; the GPU proofs' global sums add up to zero."""
    from zkmips_amd._lib import Device
    from zkmips_amd.prover import HipProver
    m, prep, _, _ = run[0]
    prep = {k: v for k, v in prep.items() if v is not None}
    gpu = HipProver(Device(0), m, prep, num_queries=16)
    cpu = O.OracleProver(m, prep, num_queries=16)
    proofs = []
    for _, _, tr, pv in run:
        p = gpu.prove_shard(tr, pv)
        rc, ref = cpu.prove(tr, pv)
        assert rc == 0 and p == ref
        proofs.append(p)
    assert machine_global_sum_is_zero(proofs)


# sys_linux_tests::sys_linux_program (crates/core/machine/src/syscall/precompiles/sys_linux/mod.rs:22-179),
# as (opcode, op_a, op_b, op_c, imm_b, imm_c) rows: 64 stores, then every Linux syscall the SysLinux
# table covers (mmap/mmap2 with and without a hint, brk, clone, fcntl over its fd/cmd cases, the
# no-op syscalls, read, write), then exit_group
def _sys_linux_program():
    ADD, SW = 0, C.OP_SW
    w_ptr, h_ptr = 100, 1000
    prog = [(ADD, 29, 0, 5, 0, 1)]
    for i in range(64):
        prog += [(ADD, 30, 0, w_ptr + 4 * i, 0, 1), (SW, 29, 30, 0, 0, 1)]
    calls = [(SY.SYS_MMAP, w_ptr, h_ptr), (SY.SYS_MMAP, 0, h_ptr), (SY.SYS_MMAP2, w_ptr, h_ptr),
             (SY.SYS_MMAP2, 0, h_ptr), (SY.SYS_BRK, 0, h_ptr), (SY.SYS_CLONE, 0, h_ptr)]
    calls += [(SY.SYS_FCNTL, a0, a1) for a1 in (3, 1) for a0 in (0, 1, 2, 0xff)] + [(SY.SYS_FCNTL, 1, 0x33)]
    calls += [(code, 1, 1) for code in (4263, 4005, 4288, 4006, 4194, 4195, 4206, 4215, 4218, 4222, 4240, 4338)]
    calls += [(SY.SYS_READ, 0, 0x33), (SY.SYS_READ, 1, 0x33)]
    for code, a0, a1 in calls:
        prog += [(ADD, 2, 0, code, 0, 1), (ADD, 4, 0, a0, 0, 1), (ADD, 5, 0, a1, 0, 1), (SY.OP_SYSCALL, 2, 4, 5, 0, 0)]
    for a1 in (0x33, 0x11):
        prog += [(ADD, 2, 0, SY.SYS_WRITE, 0, 1), (ADD, 4, 0, 0, 0, 1), (ADD, 5, 0, a1, 0, 1), (ADD, 6, 0, 0x100, 0, 1),
                 (SY.OP_SYSCALL, 2, 4, 5, 0, 0)]
    prog += [(ADD, 2, 0, SY.SYS_EXT_GROUP, 0, 1), (ADD, 4, 0, 0, 0, 1), (SY.OP_SYSCALL, 2, 4, 5, 0, 0)]
    return prog


@pytest.fixture(scope="module")
def linux_run():
    return C.program_shards(_sys_linux_program(), seed=5, shard_size=100)


def test_sys_linux_program_results():
    state, regs = _execute(_sys_linux_program(), seed=5)
    assert state["exit_code"] == 0 and state["pc"] == 0
    evs = [e for k, _, e in state["precompile"]]
    assert all(k == SY.SYS_LINUX for k, _, _ in state["precompile"]) and len(evs) == 32
    heap0 = C.initial_registers(5)[C.REG_HEAP]
    mm = [e for e in evs if e["code"] in (SY.SYS_MMAP, SY.SYS_MMAP2)]
    assert [e["v0"] for e in mm] == [100, heap0, 100, (heap0 + 0x1000) & 0xFFFFFFFF]  # 1000 rounds up to a page
    fc = [(e["a0"], e["a1"], e["v0"], e["writes"][0][1]) for e in evs if e["code"] == SY.SYS_FCNTL]
    assert fc[:4] == [(0, 3, 0, 0), (1, 3, 1, 0), (2, 3, 1, 0), (0xff, 3, 0xFFFFFFFF, 9)]
    assert fc[4:] == [(0, 1, 0, 0), (1, 1, 1, 0), (2, 1, 2, 0), (0xff, 1, 0xFFFFFFFF, 9), (1, 0x33, 0xFFFFFFFF, 9)]
    wr = [e for e in evs if e["code"] == SY.SYS_WRITE]
    assert [e["v0"] for e in wr] == [0x100, 0x100]
    assert regs[SY.REG_A3] == 0


def test_sys_linux_shards_satisfy_air(linux_run):
    assert "SysLinux" in linux_run[-2][2] and int(linux_run[-2][2]["SysLinux"][:, SY.SL_REAL].sum()) == 32
    for m, prep, tr, pv in linux_run:
        assert _air_check.check(m, {k: v for k, v in prep.items() if v is not None}, tr, pv) == ([], [])
    digs = np.asarray([C.shard_global_digest(tr) for _, _, tr, _ in linux_run])
    assert np.array_equal(S.digest_sum(digs), S.CURVE_CUMULATIVE_SUM_START)
    last_cpu = [pv for _, _, tr, pv in linux_run if "Cpu" in tr][-1]
    assert last_cpu[C.PV_NEXT_PC] == 0 and last_cpu[SY.PV_EXIT_CODE] == 0


@pytest.mark.parametrize("what", ["brk_result", "fcntl_errno", "mmap_heap"])
def test_sys_linux_tamper_rejected(linux_run, what):
    m, prep, tr, pv = linux_run[-2]
    t = tr["SysLinux"]
    codes = t[:, SY.SL_ID]
    bad = {n: v.copy() for n, v in tr.items()}
    if what == "brk_result":
        k = int(np.nonzero(codes == SY.SYS_BRK)[0][0])
        bad["SysLinux"][k, SY.SL_RES] ^= 1
    elif what == "fcntl_errno":
        k = int(np.nonzero((codes == SY.SYS_FCNTL) & (t[:, SY.SL_A0] == 0xff))[0][0])
        bad["SysLinux"][k, SY.SL_OUT + 4] = 0
    else:
        k = int(np.nonzero((codes == SY.SYS_MMAP) & (t[:, SY.SL_MMAP_A0_0] == 1))[0][0])
        bad["SysLinux"][k, SY.SL_IO + 4] ^= 4
    prep = {n: v for n, v in prep.items() if v is not None}
    assert _air_check.check(m, prep, bad, pv) != ([], [])


def test_sys_linux_oracle_proofs_verify(linux_run):
    m, prep, _, _ = linux_run[0]
    pr = O.OracleProver(m, {k: v for k, v in prep.items() if v is not None}, num_queries=4)
    proofs = []
    for _, _, tr, pv in linux_run:
        rc, p = pr.prove(tr, pv)
        assert rc == 0 and pr.verify(p) == 0
        proofs.append(p)
    assert machine_global_sum_is_zero(proofs)


@pytest.mark.gpu
def test_sys_linux_gpu_proofs_identical(linux_run):
    from zkmips_amd._lib import Device
    from zkmips_amd.prover import HipProver
    m, prep, _, _ = linux_run[0]
    prep = {k: v for k, v in prep.items() if v is not None}
    gpu = HipProver(Device(0), m, prep, num_queries=16)
    cpu = O.OracleProver(m, prep, num_queries=16)
    for _, _, tr, pv in linux_run:
        p = gpu.prove_shard(tr, pv)
        rc, ref = cpu.prove(tr, pv)
        assert rc == 0 and p == ref


def _two_rank_worker(rank, world, port, out_q):
    import os
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from zkmips_amd.dist import prove_shards_distributed
    run = C.program_shards(C.sha_program(3, seed=7), seed=7, shard_size=90)
    m, prep, _, _ = run[0]
    pr = O.OracleProver(m, {k: v for k, v in prep.items() if v is not None}, num_queries=4)

    def prove_one(i):
        rc, p = pr.prove(run[i][2], run[i][3])
        assert rc == 0
        return p

    proofs = prove_shards_distributed(prove_one, len(run), check_global_sum=True)
    if rank == 0:
        out_q.put((len(run), len(proofs), [i for i, (_, _, tr, _) in enumerate(run) if "Cpu" not in tr]))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_sha2_execution():
    """The CPU, SHA_EXTEND, SHA_COMPRESS and memory shards of one execution dealt to two gloo ranks; rank 0
    gathers the proofs and the machine-level global sum (syscall and memory messages) checks out."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_two_rank_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    n, got, non_cpu = q.get(timeout=600)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert got == n and len(non_cpu) == 3  # extend shard, compress shard, memory shard


@pytest.mark.gpu
def test_sha_compress_shard_full_global_height():
    """BASELINE config 3 at size: a SHA_COMPRESS precompile shard whose Global chip reaches
    its full 2^22 rows (14,600 compressions: ~145 global messages each -- the syscall plus the initial
    and final record of every word the call touched) and ShaCompress 2^21 rows proves on the GPU to
    the oracle's bytes (16 queries keep the oracle's run to tens of seconds)."""
    from zkmips_amd._lib import Device
    from zkmips_amd.prover import HipProver
    calls = 14600
    run = C.program_shards(C.sha_program(calls, seed=3, loads=0), seed=3, shard_size=1 << 21,
                           precompile_events_per_shard=calls)
    m, prep, tr, pv = next(r for r in run if "ShaCompress" in r[2])
    assert tr["Global"].shape[0] == 1 << 22 and tr["ShaCompress"].shape[0] == 1 << 21
    prep = {k: v for k, v in prep.items() if v is not None}
    gpu = HipProver(Device(0), m, prep, num_queries=16).prove_shard(tr, pv)
    rc, ref = O.OracleProver(m, prep, num_queries=16).prove(tr, pv)
    assert rc == 0 and gpu == ref
