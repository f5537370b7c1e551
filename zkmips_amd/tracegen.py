"""Device trace generation (include/zkm_tracegen.h).

The reference fills trace rows through a native per-row ABI (crates/core/machine/src/sys.rs:14-42 ->
cpp/extern.cpp:6-37) from its executor's event records.  Here the same records — numpy structured
arrays with the reference's #[repr(C)] layouts, byte for byte — go to the GPU and one launch per
chip fills the whole padded trace in HBM, plus the Byte and Program chips' multiplicities.  The
converters below build those records from this repository's executor (mips_core._execute via
program_shard(capture=...)); a Rust caller hands its own `Vec<CpuEvent>` (as CpuEventFfi) etc.

No fallback: every call goes to libzkm_hip.so and raises if it is missing.
"""
from __future__ import annotations

import ctypes as C
import functools
import os

import numpy as np

from . import _lib
from . import mips_alu as A
from . import mips_core as MC

u1, u4 = np.uint8, np.uint32

# OptionMemoryRecordEnum (events/cpu.rs:100-139): tag u8, MemoryReadRecord at 4, MemoryWriteRecord at 24
RECORD = np.dtype({"names": ["tag", "read", "write"], "formats": [u1, (u4, 5), (u4, 6)], "offsets": [0, 4, 24],
                   "itemsize": 48})
REC_READ, REC_WRITE, REC_NONE = 0, 1, 2
# CpuEventFfi (events/cpu.rs:46-75)
CPU_EVENT = np.dtype({
    "names": ["clk", "pc", "next_pc", "next_next_pc", "a", "a_record", "b", "b_record", "c", "c_record", "hi_tag",
              "hi", "hi_record", "memory_record", "exit_code"],
    "formats": [u4, u4, u4, u4, u4, RECORD, u4, RECORD, u4, RECORD, u1, u4, RECORD, RECORD, u4],
    "offsets": [0, 4, 8, 12, 16, 20, 68, 72, 120, 124, 172, 176, 180, 228, 276], "itemsize": 280})
# InstructionFfi (instruction.rs:29-45): opcode u8, op_a u8, op_b, op_c, imm_b, imm_c, raw: OptionU32
INSTRUCTION = np.dtype({"names": ["opcode", "op_a", "op_b", "op_c", "imm_b", "imm_c", "raw_tag", "raw"],
                        "formats": [u1, u1, u4, u4, u1, u1, u1, u4], "offsets": [0, 1, 4, 8, 12, 13, 16, 20],
                        "itemsize": 24})
# AluEvent (events/instr.rs:10-27)
ALU_EVENT = np.dtype({"names": ["pc", "next_pc", "opcode", "hi", "a", "b", "c"],
                      "formats": [u4, u4, u1, u4, u4, u4, u4], "offsets": [0, 4, 8, 12, 16, 20, 24], "itemsize": 28})
# MemoryLocalEvent (events/memory.rs:225-236): addr, initial (shard, timestamp, value), final (...)
MEMORY_LOCAL_EVENT = np.dtype({"names": ["addr", "initial", "final"], "formats": [u4, (u4, 3), (u4, 3)],
                               "offsets": [0, 4, 16], "itemsize": 28})
# MemoryInitializeFinalizeEvent (events/memory.rs:135-148)
MEMORY_INIT_FINAL_EVENT = np.dtype({"names": ["addr", "value", "shard", "timestamp"], "formats": [u4] * 4,
                                    "offsets": [0, 4, 8, 12], "itemsize": 16})
# SyscallEvent (events/syscall.rs:8-29)
SYSCALL_EVENT = np.dtype({"names": ["pc", "next_pc", "shard", "clk", "a_record", "a_record_is_real", "syscall_id",
                                    "arg1", "arg2"],
                          "formats": [u4, u4, u4, u4, (u4, 6), u1, u4, u4, u4],
                          "offsets": [0, 4, 8, 12, 16, 40, 44, 48, 52], "itemsize": 56})

# GlobalLookupEvent (events/global.rs:6-15): message[7], is_receive, kind
GLOBAL_EVENT = np.dtype({"names": ["message", "is_receive", "kind"], "formats": [(u4, 7), u1, u1],
                         "offsets": [0, 28, 29], "itemsize": 32})

# BranchEvent (events/instr.rs:159-177): pc, next_pc, next_next_pc, opcode, a, b, c
BRANCH_EVENT = np.dtype({"names": ["pc", "next_pc", "next_next_pc", "opcode", "a", "b", "c"],
                         "formats": [u4, u4, u4, u1, u4, u4, u4], "offsets": [0, 4, 8, 12, 16, 20, 24], "itemsize": 28})
# MemInstrEvent (events/instr.rs:112-135), mem_access as an OptionMemoryRecordEnum (zkm_tracegen.h)
MEM_INSTR_EVENT = np.dtype({"names": ["shard", "clk", "pc", "next_pc", "opcode", "a", "b", "c", "mem_access",
                                      "prev_a_val"],
                            "formats": [u4, u4, u4, u4, u1, u4, u4, u4, RECORD, u4],
                            "offsets": [0, 4, 8, 12, 16, 20, 24, 28, 32, 80], "itemsize": 84})

# JumpEvent (events/instr.rs:198-216) = BranchEvent's layout; MovCondEvent (:283-301)
JUMP_EVENT = BRANCH_EVENT
MOVCOND_EVENT = np.dtype({"names": ["pc", "next_pc", "opcode", "a", "b", "c", "prev_a"],
                          "formats": [u4, u4, u1, u4, u4, u4, u4], "offsets": [0, 4, 8, 12, 16, 20, 24], "itemsize": 28})
# CompAluEvent (events/instr.rs:44-72) with C layout (zkm_tracegen.h)
COMP_ALU_EVENT = np.dtype({"names": ["shard", "clk", "pc", "next_pc", "opcode", "hi", "a", "b", "c", "hi_record",
                                     "hi_record_is_real"],
                           "formats": [u4, u4, u4, u4, u1, u4, u4, u4, u4, (u4, 6), u1],
                           "offsets": [0, 4, 8, 12, 16, 20, 24, 28, 32, 36, 60], "itemsize": 64})

CPU_WIDTH, ADD_SUB_WIDTH, MEMORY_LOCAL_WIDTH, MEMORY_GLOBAL_WIDTH, SYSCALL_WIDTH = 67, 19, 56, 111, 6
BRANCH_WIDTH, MEMORY_INSTRS_WIDTH, JUMP_WIDTH, MOVCOND_WIDTH, MUL_WIDTH = 62, 79, 66, 32, 58
DIVREM_WIDTH, CLO_CLZ_WIDTH, SYSCALL_INSTRS_WIDTH, MISC_INSTRS_WIDTH = 106, 22, 64, 72
# the flattened ShaExtendEvent row (zkm_tracegen.h): shard, clk, w_ptr, four MemoryReadRecords, a MemoryWriteRecord
SHA_EXTEND_ROW = np.dtype({"names": ["shard", "clk", "w_ptr", "r15", "r2", "r16", "r7", "w"],
                           "formats": [u4, u4, u4, (u4, 5), (u4, 5), (u4, 5), (u4, 5), (u4, 6)],
                           "offsets": [0, 4, 8, 12, 32, 52, 72, 92], "itemsize": 116})
SHA_EXTEND_WIDTH = 176
# the ShaCompress call record (zkm_tracegen.h): shard, clk, w_ptr, h_ptr, 8 h reads, 64 w reads, 8 h writes
SHA_COMPRESS_EVENT = np.dtype({"names": ["shard", "clk", "w_ptr", "h_ptr", "h_read", "w_read", "h_write"],
                               "formats": [u4, u4, u4, u4, (u4, (8, 5)), (u4, (64, 5)), (u4, (8, 6))],
                               "offsets": [0, 4, 8, 12, 16, 176, 1456], "itemsize": 1648})
SHA_COMPRESS_WIDTH = 262
# MiscEvent (events/instr.rs:236-260)
MISC_EVENT = np.dtype({"names": ["shard", "clk", "pc", "next_pc", "opcode", "a", "b", "c", "prev_a", "hi_record"],
                       "formats": [u4, u4, u4, u4, u1, u4, u4, u4, u4, (u4, 6)],
                       "offsets": [0, 4, 8, 12, 16, 20, 24, 28, 32, 36], "itemsize": 60})
GLOBAL_WIDTH = 99


# ---------------------------------------------------------------- records from this repository's executor
PYCONV_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libzkm_pyconv.so")


@functools.lru_cache(maxsize=None)
def _pyconv():
    """libzkm_pyconv.so (csrc/host/pyconv.cpp): the executor's tuples walked natively.  PyDLL keeps the GIL
    held through each call and turns an error set there into a Python exception."""
    if not os.path.exists(PYCONV_PATH):
        raise RuntimeError(f"{PYCONV_PATH} is not built (make -C zkmips_amd/csrc, or __graft_entry__.build())")
    L = C.PyDLL(PYCONV_PATH)
    L.zkm_py_flatten_i64.argtypes = [C.py_object, C.c_int64, C.c_int64, C.c_void_p, C.c_int64]
    L.zkm_py_flatten_i64.restype = C.c_int64
    L.zkm_py_cpu_events.argtypes = [C.py_object] + [C.c_uint32] * 5 + [C.c_void_p, C.c_int64]
    L.zkm_py_cpu_events.restype = C.c_int64
    return L


def _rows(x, width: int, none_w: int = 0) -> np.ndarray:
    """An (n, width) int64 array of the executor's record tuples (or an array already), flattened natively
    (nested tuples allowed; None stands for none_w zeros)."""
    if isinstance(x, np.ndarray):
        return x.astype(np.int64, copy=False).reshape(-1, width)
    if not isinstance(x, (list, tuple)):
        x = list(x)
    out = np.empty((len(x), width), np.int64)
    if len(x):
        _pyconv().zkm_py_flatten_i64(x, width, none_w, out.ctypes.data, len(x))
    return out


def program_ffi(prog) -> np.ndarray:
    """Program::instructions as InstructionFfi (prog rows: opcode, op_a, op_b, op_c, imm_b, imm_c)."""
    P_ = _rows(prog, 6)
    out = np.zeros(len(P_), INSTRUCTION)
    out["opcode"], out["op_a"] = P_[:, 0], P_[:, 1]
    out["op_b"], out["op_c"] = P_[:, 2] & 0xFFFFFFFF, P_[:, 3] & 0xFFFFFFFF
    out["imm_b"], out["imm_c"] = P_[:, 4], P_[:, 5]
    out["raw_tag"] = 1  # None
    return out


def cpu_events(steps, shard: int) -> np.ndarray:
    """CpuEvent records (events/cpu.rs:8-44 as CpuEventFfi) of the executor's steps: the op_a access a
    write (a read when the value is unchanged), op_b / op_c reads unless immediate (executor.rs
    rr/rw at MemoryAccessPosition A = 3, B = 2, C = 1).  Written natively (zkm_py_cpu_events), struct by
    struct; cpu_events_numpy is the same conversion in numpy (the tests compare the bytes)."""
    n = len(steps)
    e = np.empty(n, CPU_EVENT)  # every byte written by the converter
    if n:
        _pyconv().zkm_py_cpu_events(steps if isinstance(steps, (list, tuple)) else list(steps), shard, MC.PC_BASE,
                                    MC.POS_A, MC.POS_B, MC.POS_C, e.ctypes.data, n)
    return e


def cpu_events_numpy(steps, shard: int) -> np.ndarray:
    """cpu_events in numpy (the reference for the native converter's bytes)."""
    n = len(steps)
    e = np.zeros(n, CPU_EVENT)
    if not n:
        return e
    # one flat pass over the step tuples per field group (np.fromiter over chained item getters: ~4x faster
    # than np.asarray of per-step lists)
    from itertools import chain
    from operator import itemgetter
    S = np.fromiter(chain.from_iterable(map(itemgetter(*range(11), 12, 13), steps)), np.int64,
                    count=13 * n).reshape(n, 13)
    ks, av, bv, cv, prev_a, written = S[:, 0], S[:, 2], S[:, 3], S[:, 4], S[:, 5], S[:, 6]
    immb, immc = S[:, 9].astype(bool), S[:, 10].astype(bool)
    clk, his = S[:, 12], S[:, 11]
    Z = (0, 0)
    prev = np.fromiter(chain.from_iterable(x or Z for x in chain.from_iterable(map(itemgetter(11), steps))),
                       np.int64, count=6 * n).reshape(n, 3, 2)  # c, b, a
    e["clk"], e["pc"] = clk, MC.PC_BASE + 4 * ks
    e["next_pc"], e["next_next_pc"] = S[:, 7], S[:, 8]
    e["a"], e["b"], e["c"] = av, bv, cv
    is_write = written != prev_a
    ar = e["a_record"]
    ar["tag"] = np.where(is_write, REC_WRITE, REC_READ)
    w = np.stack([written, np.full(n, shard), clk + MC.POS_A, prev_a, prev[:, 2, 0], prev[:, 2, 1]], axis=1)
    ar["write"] = np.where(is_write[:, None], w, 0)
    ar["read"] = np.where(is_write[:, None], 0, w[:, [0, 1, 2, 4, 5]])
    for field, val, pos, j, imm in (("b_record", bv, MC.POS_B, 1, immb), ("c_record", cv, MC.POS_C, 0, immc)):
        r = e[field]
        r["tag"] = np.where(imm, REC_NONE, REC_READ)
        rd = np.stack([val, np.full(n, shard), clk + pos, prev[:, j, 0], prev[:, j, 1]], axis=1)
        r["read"] = np.where(imm[:, None], 0, rd)
    e["hi_tag"] = np.where(his != 0, 0, 1)
    e["hi"] = his
    e["hi_record"]["tag"] = REC_NONE
    e["memory_record"]["tag"] = REC_NONE
    return e


def alu_events(op, a, b, c, pc, npc=None) -> np.ndarray:
    """AluEvent records (events/instr.rs:10-27)."""
    n = len(op)
    e = np.zeros(n, ALU_EVENT)
    e["pc"], e["opcode"], e["a"], e["b"], e["c"] = pc, op, a, b, c
    e["next_pc"] = np.asarray(pc, np.int64) + 4 if npc is None else npc
    return e


def memory_local_events(entries) -> np.ndarray:
    """MemoryLocalEvent records of (addr, initial shard, clk, value, final shard, clk, value) rows."""
    E = _rows(entries, 7)
    e = np.zeros(len(E), MEMORY_LOCAL_EVENT)
    e["addr"] = E[:, 0]
    e["initial"] = E[:, 1:4]
    e["final"] = E[:, 4:7]
    return e


def memory_init_final_events(events) -> np.ndarray:
    """MemoryInitializeFinalizeEvent records of (addr, value, shard, timestamp) rows, sorted by addr
    (MemoryGlobalChip::generate_trace sorts them, memory/global.rs:117-121)."""
    E = np.asarray(events, np.int64).reshape(-1, 4)
    E = E[np.argsort(E[:, 0], kind="stable")]
    e = np.zeros(len(E), MEMORY_INIT_FINAL_EVENT)
    e["addr"], e["value"], e["shard"], e["timestamp"] = E[:, 0], E[:, 1], E[:, 2], E[:, 3]
    return e


def syscall_events(syscalls) -> np.ndarray:
    """SyscallEvent records of the executor's syscall tuples (pc, next_pc, shard, clk, a, b, c, prev_a, id)."""
    S = _rows(syscalls, 9)
    e = np.zeros(len(S), SYSCALL_EVENT)
    e["pc"], e["next_pc"], e["shard"], e["clk"] = S[:, 0], S[:, 1], S[:, 2], S[:, 3]
    e["a_record"] = np.stack([S[:, 4], S[:, 2], S[:, 3] + MC.POS_A, S[:, 7], np.zeros(len(S)), np.zeros(len(S))],
                             axis=1)
    e["a_record_is_real"] = 1
    e["syscall_id"], e["arg1"], e["arg2"] = S[:, 8], S[:, 5], S[:, 6]
    return e


def global_events(messages, is_receive, kinds) -> np.ndarray:
    """GlobalLookupEvent records (the Global chip's input, global/mod.rs:77-108)."""
    M = np.asarray(messages, np.int64).reshape(-1, 7)
    e = np.zeros(len(M), GLOBAL_EVENT)
    e["message"] = M
    e["is_receive"] = np.asarray(is_receive, np.int64)
    e["kind"] = np.asarray(kinds, np.int64)
    return e


def shard_global_events(capture: dict) -> np.ndarray:
    """The Global chip's records of a CPU shard, in chip order: SyscallCore's sends, then MemoryLocal's
    receive/send pairs (program_shard)."""
    from . import mips_memory as MM
    from . import mips_syscall as SY
    core_sc = capture["core_syscalls"]
    core = core_sc[:, [2, 3, 8, 5, 6]] if len(core_sc) else np.zeros((0, 5), np.int64)
    smsg = SY.syscall_global_messages(core)
    gmsg, grec = MM.memory_local_global_events(_rows(capture["entries"], 7))
    return global_events(np.concatenate([smsg, gmsg]), np.concatenate([np.zeros(len(smsg), np.uint8), grec]),
                         np.concatenate([np.full(len(smsg), SY.KIND_SYSCALL), np.full(len(gmsg), MC.KIND_MEMORY)]))


def add_sub_records(alu) -> np.ndarray:
    """The AddSub chip's AluEvents from the executor's ALU event lists (kind "add")."""
    return alu_records(alu, "add")


def branch_records(branches) -> np.ndarray:
    """BranchEvents of the executor's branch tuples (pc, op, a, b, c, next_pc, next_next_pc, taken)."""
    B = _rows(branches, 8)
    e = np.zeros(len(B), BRANCH_EVENT)
    e["pc"], e["opcode"], e["a"], e["b"], e["c"] = B[:, 0], B[:, 1], B[:, 2], B[:, 3], B[:, 4]
    e["next_pc"], e["next_next_pc"] = B[:, 5], B[:, 6]
    return e


def mem_instr_records(mevs, shard: int) -> np.ndarray:
    """MemInstrEvents of the executor's memory-instruction tuples (pc, npc, op, a, b, c, prev_a, clk, addr,
    prev_mem, mem, mem_prev_shard, mem_prev_clk): loads carry a Read record, stores a Write record."""
    E = _rows(mevs, 13)
    n = len(E)
    assert np.array_equal(E[:, 8], (E[:, 4] + E[:, 5]) & 0xFFFFFFFF), "address = b + c"
    e = np.zeros(n, MEM_INSTR_EVENT)
    e["shard"], e["clk"], e["pc"], e["next_pc"], e["opcode"] = shard, E[:, 7], E[:, 0], E[:, 1], E[:, 2]
    e["a"], e["b"], e["c"], e["prev_a_val"] = E[:, 3], E[:, 4], E[:, 5], E[:, 6]
    load = np.isin(E[:, 2], MC.LOAD_OPS)
    m = e["mem_access"]
    m["tag"] = np.where(load, REC_READ, REC_WRITE)
    m["read"] = np.where(load[:, None], np.stack([E[:, 10], np.full(n, shard), E[:, 7], E[:, 11], E[:, 12]], 1), 0)
    m["write"] = np.where(load[:, None], 0, np.stack([E[:, 10], np.full(n, shard), E[:, 7], E[:, 9], E[:, 11], E[:, 12]], 1))
    e["mem_access"] = m
    return e


def jump_records(jumps) -> np.ndarray:
    """JumpEvents of the executor's jump tuples (pc, op, a, b, c, next_pc, next_next_pc)."""
    J = _rows(jumps, 7)
    e = np.zeros(len(J), JUMP_EVENT)
    e["pc"], e["opcode"], e["a"], e["b"], e["c"] = J[:, 0], J[:, 1], J[:, 2], J[:, 3], J[:, 4]
    e["next_pc"], e["next_next_pc"] = J[:, 5], J[:, 6]
    return e


def movcond_records(movs) -> np.ndarray:
    """MovCondEvents of the executor's tuples (pc, next_pc, op, a, b, c, prev_a)."""
    E = _rows(movs, 7)
    e = np.zeros(len(E), MOVCOND_EVENT)
    for j, f in enumerate(("pc", "next_pc", "opcode", "a", "b", "c", "prev_a")):
        e[f] = E[:, j]
    return e


def mul_records(muls, shard: int) -> np.ndarray:
    """CompAluEvents of the executor's Mul tuples (op, a, b, c, pc, npc, hi, clk, prev_hi, prev_shard, prev_clk;
    clk < 0: no HI write): the HI record written at clk + POS_HI."""
    E = _rows(muls, 11)
    n = len(E)
    e = np.zeros(n, COMP_ALU_EVENT)
    hrr = E[:, 7] >= 0
    e["opcode"], e["a"], e["b"], e["c"], e["pc"], e["next_pc"], e["hi"] = (E[:, j] for j in range(7))
    e["shard"] = np.where(hrr, shard, 0)
    e["clk"] = np.where(hrr, E[:, 7], 0)
    e["hi_record"] = np.where(hrr[:, None], np.stack([E[:, 6], np.full(n, shard), E[:, 7] + MC.POS_HI, E[:, 8], E[:, 9],
                                                      E[:, 10]], 1), 0)
    e["hi_record_is_real"] = hrr
    return e


def divrem_records(divs, shard: int) -> np.ndarray:
    """CompAluEvents of the executor's DivRem tuples (op, b, c, pc, npc, clk, prev_hi, prev_shard, prev_clk;
    clk < 0: no HI write): a = quotient, hi = remainder, the HI record (the remainder) written at clk + POS_HI."""
    E = _rows(divs, 9)
    n = len(E)
    qr = np.asarray([MC._qr(int(o), int(x), int(y)) for o, x, y in zip(E[:, 0], E[:, 1], E[:, 2])],
                    np.int64).reshape(n, 2)
    e = np.zeros(n, COMP_ALU_EVENT)
    hrr = E[:, 5] >= 0
    e["opcode"], e["b"], e["c"], e["pc"], e["next_pc"] = E[:, 0], E[:, 1], E[:, 2], E[:, 3], E[:, 4]
    e["a"], e["hi"] = qr[:, 0], qr[:, 1]
    e["shard"] = np.where(hrr, shard, 0)
    e["clk"] = np.where(hrr, E[:, 5], 0)
    e["hi_record"] = np.where(hrr[:, None], np.stack([qr[:, 1], np.full(n, shard), E[:, 5] + MC.POS_HI, E[:, 6],
                                                      E[:, 7], E[:, 8]], 1), 0)
    e["hi_record_is_real"] = hrr
    return e


def misc_records(misc, shard: int) -> np.ndarray:
    """MiscEvents of the executor's tuples (op, a, b, c, prev_a, pc, npc, clk, hi_prev, hi_new, hi_prev_shard,
    hi_prev_clk): MADDU / MSUBU / MADD / MSUB carry the HI write at clk + POS_HI."""
    E = _rows(misc, 12)
    n = len(E)
    e = np.zeros(n, MISC_EVENT)
    md = np.isin(E[:, 0], MC.MADDSUB_OPS)
    e["opcode"], e["a"], e["b"], e["c"], e["prev_a"], e["pc"], e["next_pc"] = (E[:, j] for j in range(7))
    e["shard"] = np.where(md, shard, 0)
    e["clk"] = E[:, 7]
    e["hi_record"] = np.where(md[:, None], np.stack([E[:, 9], np.full(n, shard), E[:, 7] + MC.POS_HI, E[:, 8],
                                                     E[:, 10], E[:, 11]], 1), 0)
    return e


def sha_extend_records(events) -> np.ndarray:
    """The ShaExtend rows of the executor's SHA_EXTEND events (mips_syscall.exec_sha_extend), 48 per call."""
    out = np.zeros(48 * len(events), SHA_EXTEND_ROW)
    for k, ev in enumerate(events):
        rows = out[48 * k:48 * (k + 1)]
        ts = ev["clk"] + np.arange(48)
        rows["shard"], rows["clk"], rows["w_ptr"] = ev["shard"], ev["clk"], ev["w_ptr"]
        for key in ("r15", "r2", "r16", "r7"):
            rd = np.asarray(ev[key], np.int64).reshape(48, 3)  # value, prev_shard, prev_clk
            rows[key] = np.stack([rd[:, 0], np.full(48, ev["shard"]), ts, rd[:, 1], rd[:, 2]], 1)
        wr = np.asarray(ev["wr"], np.int64).reshape(48, 4)  # prev_value, value, prev_shard, prev_clk
        rows["w"] = np.stack([wr[:, 1], np.full(48, ev["shard"]), ts, wr[:, 0], wr[:, 2], wr[:, 3]], 1)
        out[48 * k:48 * (k + 1)] = rows
    return out


UINT256_MUL_EVENT = np.dtype({"names": ["shard", "clk", "x_ptr", "y_ptr", "y", "modulus", "x"],
                              "formats": [u4, u4, u4, u4, (u4, (8, 5)), (u4, (8, 5)), (u4, (8, 6))],
                              "offsets": [0, 4, 8, 12, 16, 176, 336], "itemsize": 528})
UINT256_MUL_WIDTH = 480  # ZKM_UINT256_MUL_WIDTH


def uint256_mul_records(events) -> np.ndarray:
    """zkm_uint256_mul_event records of the executor's UINT256_MUL events (mips_ec.exec_uint256_mul): y and
    the modulus read at clk, x written at clk + 1."""
    out = np.zeros(len(events), UINT256_MUL_EVENT)
    for k, e in enumerate(events):
        sh, clk = e["shard"], e["clk"]
        r = out[k]
        r["shard"], r["clk"], r["x_ptr"], r["y_ptr"] = sh, clk, e["x_ptr"], e["y_ptr"]
        for key, name in (("y", "y"), ("m", "modulus")):
            rd = np.asarray(e[key], np.int64).reshape(8, 3)  # value, prev_shard, prev_clk
            r[name] = np.stack([rd[:, 0], np.full(8, sh), np.full(8, clk), rd[:, 1], rd[:, 2]], 1)
        wr = np.asarray(e["xw"], np.int64).reshape(8, 4)  # prev_value, value, prev_shard, prev_clk
        r["x"] = np.stack([wr[:, 1], np.full(8, sh), np.full(8, clk + 1), wr[:, 0], wr[:, 2], wr[:, 3]], 1)
    return out


def uint256_mul_trace(events_dev, n: int, height: int = None, byte_mult=None):
    """Uint256MulMod main trace (height x 480 int32, on the GPU) from n zkm_uint256_mul_event records; the
    Byte lookups added into byte_mult (nullable)."""
    height = height or _pow2(n)
    t = _trace(height, UINT256_MUL_WIDTH)
    what = "zkm_uint256_mul_events_to_trace"
    _lib.check(_bind().zkm_uint256_mul_events_to_trace(_records(events_dev, n, UINT256_MUL_EVENT, what), n,
                                                       t.data_ptr(), height, _words(byte_mult, 65536 * 10, what),
                                                       _stream()), what)
    return t


U256X2048_MUL_EVENT = np.dtype({"names": ["shard", "clk", "a_ptr", "b_ptr", "lo_ptr", "hi_ptr", "lo_ptr_reg", "hi_ptr_reg",
                                         "a", "b", "lo", "hi"],
                                "formats": [u4] * 6 + [(u4, 5), (u4, 5), (u4, (8, 5)), (u4, (64, 5)), (u4, (64, 6)),
                                                       (u4, (8, 6))],
                                "offsets": [0, 4, 8, 12, 16, 20, 24, 44, 64, 224, 1504, 3040], "itemsize": 3232})
U256X2048_MUL_WIDTH = 3129  # ZKM_U256XU2048_MUL_WIDTH


def u256x2048_mul_records(events) -> np.ndarray:
    """zkm_u256x2048_mul_event records of the executor's U256XU2048_MUL events (mips_ec.exec_u256x2048_mul):
    the registers, a and b read at clk, lo and hi written at clk + 1."""
    out = np.zeros(len(events), U256X2048_MUL_EVENT)

    def reads(recs, sh, clk):
        rd = np.asarray(recs, np.int64).reshape(-1, 3)  # value, prev_shard, prev_clk
        return np.stack([rd[:, 0], np.full(len(rd), sh), np.full(len(rd), clk), rd[:, 1], rd[:, 2]], 1)

    def writes(recs, sh, clk):
        wr = np.asarray(recs, np.int64).reshape(-1, 4)  # prev_value, value, prev_shard, prev_clk
        return np.stack([wr[:, 1], np.full(len(wr), sh), np.full(len(wr), clk), wr[:, 0], wr[:, 2], wr[:, 3]], 1)
    for k, e in enumerate(events):
        sh, clk = e["shard"], e["clk"]
        r = out[k]
        for f in ("shard", "clk", "a_ptr", "b_ptr", "lo_ptr", "hi_ptr"):
            r[f] = e[f]
        r["lo_ptr_reg"], r["hi_ptr_reg"] = reads([e["lo_reg"]], sh, clk)[0], reads([e["hi_reg"]], sh, clk)[0]
        r["a"], r["b"] = reads(e["a"], sh, clk), reads(e["b"], sh, clk)
        r["lo"], r["hi"] = writes(e["lo"], sh, clk + 1), writes(e["hi"], sh, clk + 1)
    return out


def u256x2048_mul_trace(events_dev, n: int, height: int = None, byte_mult=None):
    """U256XU2048Mul main trace (height x 3129 int32, on the GPU) from n zkm_u256x2048_mul_event records; the
    Byte lookups added into byte_mult (nullable)."""
    height = height or _pow2(n)
    t = _trace(height, U256X2048_MUL_WIDTH)
    what = "zkm_u256x2048_mul_events_to_trace"
    _lib.check(_bind().zkm_u256x2048_mul_events_to_trace(_records(events_dev, n, U256X2048_MUL_EVENT, what), n,
                                                         t.data_ptr(), height, _words(byte_mult, 65536 * 10, what),
                                                         _stream()), what)
    return t


FP_OP_EVENT = np.dtype({"names": ["shard", "clk", "x_ptr", "y_ptr", "op", "y", "x"],
                        "formats": [u4, u4, u4, u4, u4, (u4, (12, 5)), (u4, (12, 6))],
                        "offsets": [0, 4, 8, 12, 16, 20, 260], "itemsize": 548})
FP_OP_FIELDS = {"Bn254": (0, 372), "Bls12381": (1, 556)}  # ZKM_FIELD_*, ZKM_FP_OP_WIDTH_*
_FP_OP_CODE = {"add": 0, "sub": 1, "mul": 2}


def fp_op_records(events) -> np.ndarray:
    """zkm_fp_op_event records of the executor's FpOp events (mips_ec.exec_fp_op): y read at clk, x written at
    clk + 1 (8 or 12 words, in slots of 12)."""
    out = np.zeros(len(events), FP_OP_EVENT)
    for k, e in enumerate(events):
        sh, clk = e["shard"], e["clk"]
        r = out[k]
        r["shard"], r["clk"], r["x_ptr"], r["y_ptr"], r["op"] = sh, clk, e["x_ptr"], e["y_ptr"], _FP_OP_CODE[e["op"]]
        rd = np.asarray(e["y"], np.int64).reshape(-1, 3)
        wr = np.asarray(e["xw"], np.int64).reshape(-1, 4)
        w = len(rd)
        r["y"][:w] = np.stack([rd[:, 0], np.full(w, sh), np.full(w, clk), rd[:, 1], rd[:, 2]], 1)
        r["x"][:w] = np.stack([wr[:, 1], np.full(w, sh), np.full(w, clk + 1), wr[:, 0], wr[:, 2], wr[:, 3]], 1)
    return out


def fp_op_trace(field: str, events_dev, n: int, height: int = None, byte_mult=None):
    """FpOpAssign main trace of the bn254 / bls12-381 base field (height x 372 / 556 int32, on the GPU) from n
    zkm_fp_op_event records; the Byte lookups added into byte_mult (nullable)."""
    code, width = FP_OP_FIELDS[field]
    height = height or _pow2(n)
    t = _trace(height, width)
    what = "zkm_fp_op_events_to_trace"
    _lib.check(_bind().zkm_fp_op_events_to_trace(code, _records(events_dev, n, FP_OP_EVENT, what), n, t.data_ptr(),
                                                 height, _words(byte_mult, 65536 * 10, what), _stream()), what)
    return t


FP2_EVENT = np.dtype({"names": ["shard", "clk", "x_ptr", "y_ptr", "op", "y", "x"],
                      "formats": [u4, u4, u4, u4, u4, (u4, (24, 5)), (u4, (24, 6))],
                      "offsets": [0, 4, 8, 12, 16, 20, 500], "itemsize": 1076})
FP2_WIDTHS = {("Bn254", False): 734, ("Bls12381", False): 1102, ("Bn254", True): 1485, ("Bls12381", True): 2237}


def fp2_records(events) -> np.ndarray:
    """zkm_fp2_event records of the executor's Fp2AddSub / Fp2Mul events (mips_ec.exec_fp2_addsub /
    exec_fp2_mul): y read at clk, x written at clk + 1 (16 or 24 words, in slots of 24)."""
    out = np.zeros(len(events), FP2_EVENT)
    for k, e in enumerate(events):
        sh, clk = e["shard"], e["clk"]
        r = out[k]
        r["shard"], r["clk"], r["x_ptr"], r["y_ptr"] = sh, clk, e["x_ptr"], e["y_ptr"]
        r["op"] = _FP_OP_CODE.get(e.get("op", "add"), 0)
        rd = np.asarray(e["y"], np.int64).reshape(-1, 3)
        wr = np.asarray(e["xw"], np.int64).reshape(-1, 4)
        w = len(rd)
        r["y"][:w] = np.stack([rd[:, 0], np.full(w, sh), np.full(w, clk), rd[:, 1], rd[:, 2]], 1)
        r["x"][:w] = np.stack([wr[:, 1], np.full(w, sh), np.full(w, clk + 1), wr[:, 0], wr[:, 2], wr[:, 3]], 1)
    return out


def fp2_trace(field: str, mul: bool, events_dev, n: int, height: int = None, byte_mult=None):
    """Fp2AddSubAssign (mul False) or Fp2MulAssign main trace of the bn254 / bls12-381 extension (on the GPU)
    from n zkm_fp2_event records; the Byte lookups added into byte_mult (nullable)."""
    code = FP_OP_FIELDS[field][0]
    height = height or _pow2(n)
    t = _trace(height, FP2_WIDTHS[(field, bool(mul))])
    what = "zkm_fp2_events_to_trace"
    _lib.check(_bind().zkm_fp2_events_to_trace(code, int(bool(mul)), _records(events_dev, n, FP2_EVENT, what), n,
                                               t.data_ptr(), height, _words(byte_mult, 65536 * 10, what), _stream()),
               what)
    return t


EC_ADD_EVENT = np.dtype({"names": ["shard", "clk", "p_ptr", "q_ptr", "q", "p"],
                         "formats": [u4, u4, u4, u4, (u4, (24, 5)), (u4, (24, 6))],
                         "offsets": [0, 4, 8, 12, 16, 496], "itemsize": 1072})
EC_CURVES = {"Secp256k1": 0, "Secp256r1": 1, "Bn254": 2, "Bls12381": 3}  # ZKM_CURVE_*


def ec_add_records(events) -> np.ndarray:
    """zkm_ec_add_event records of the executor's EC add events (mips_ec.exec_ec_add): q read at clk, p written
    at clk + 1 (16 or 24 words, in slots of 24)."""
    out = np.zeros(len(events), EC_ADD_EVENT)
    for k, e in enumerate(events):
        sh, clk = e["shard"], e["clk"]
        r = out[k]
        r["shard"], r["clk"], r["p_ptr"], r["q_ptr"] = sh, clk, e["p_ptr"], e["q_ptr"]
        rd = np.asarray(e["q"], np.int64).reshape(-1, 3)
        wr = np.asarray(e["pw"], np.int64).reshape(-1, 4)
        w = len(rd)
        r["q"][:w] = np.stack([rd[:, 0], np.full(w, sh), np.full(w, clk), rd[:, 1], rd[:, 2]], 1)
        r["p"][:w] = np.stack([wr[:, 1], np.full(w, sh), np.full(w, clk + 1), wr[:, 0], wr[:, 2], wr[:, 3]], 1)
    return out


def ec_add_trace(curve: str, events_dev, n: int, height: int = None, byte_mult=None):
    """WeierstrassAddAssign main trace of a curve (on the GPU) from n zkm_ec_add_event records; the Byte
    lookups added into byte_mult (nullable)."""
    from . import mips_ec as EC
    height = height or _pow2(n)
    t = _trace(height, EC.AddLayout(EC.FIELDS[curve]).WIDTH)
    what = "zkm_ec_add_events_to_trace"
    _lib.check(_bind().zkm_ec_add_events_to_trace(EC_CURVES[curve], _records(events_dev, n, EC_ADD_EVENT, what), n,
                                                  t.data_ptr(), height, _words(byte_mult, 65536 * 10, what),
                                                  _stream()), what)
    return t


EC_DOUBLE_EVENT = np.dtype({"names": ["shard", "clk", "p_ptr", "p"], "formats": [u4, u4, u4, (u4, (24, 6))],
                            "offsets": [0, 4, 8, 12], "itemsize": 588})


def ec_double_records(events) -> np.ndarray:
    """zkm_ec_double_event records of the executor's EC double events (mips_ec.exec_ec_double): p written at
    clk (16 or 24 words, in slots of 24)."""
    out = np.zeros(len(events), EC_DOUBLE_EVENT)
    for k, e in enumerate(events):
        sh, clk = e["shard"], e["clk"]
        r = out[k]
        r["shard"], r["clk"], r["p_ptr"] = sh, clk, e["p_ptr"]
        wr = np.asarray(e["pw"], np.int64).reshape(-1, 4)
        w = len(wr)
        r["p"][:w] = np.stack([wr[:, 1], np.full(w, sh), np.full(w, clk), wr[:, 0], wr[:, 2], wr[:, 3]], 1)
    return out


def ec_double_trace(curve: str, events_dev, n: int, height: int = None, byte_mult=None):
    """WeierstrassDoubleAssign main trace of a curve (on the GPU) from n zkm_ec_double_event records; the Byte
    lookups added into byte_mult (nullable)."""
    from . import mips_ec as EC
    height = height or _pow2(n)
    t = _trace(height, EC.DoubleLayout(EC.FIELDS[curve]).WIDTH)
    what = "zkm_ec_double_events_to_trace"
    _lib.check(_bind().zkm_ec_double_events_to_trace(EC_CURVES[curve], _records(events_dev, n, EC_DOUBLE_EVENT, what),
                                                     n, t.data_ptr(), height, _words(byte_mult, 65536 * 10, what),
                                                     _stream()), what)
    return t


EC_DECOMPRESS_EVENT = np.dtype({"names": ["shard", "clk", "ptr", "sign", "x", "y"],
                                "formats": [u4, u4, u4, u4, (u4, (12, 5)), (u4, (12, 6))],
                                "offsets": [0, 4, 8, 12, 16, 256], "itemsize": 544})


def ec_decompress_records(events) -> np.ndarray:
    """zkm_ec_decompress_event records of the executor's decompress events (mips_ec.exec_ec_decompress): x read
    and y written at clk (8 or 12 words, in slots of 12)."""
    out = np.zeros(len(events), EC_DECOMPRESS_EVENT)
    for k, e in enumerate(events):
        sh, clk = e["shard"], e["clk"]
        r = out[k]
        r["shard"], r["clk"], r["ptr"], r["sign"] = sh, clk, e["ptr"], e["sign"]
        rd = np.asarray(e["x"], np.int64).reshape(-1, 3)
        wr = np.asarray(e["y"], np.int64).reshape(-1, 4)
        w = len(rd)
        r["x"][:w] = np.stack([rd[:, 0], np.full(w, sh), np.full(w, clk), rd[:, 1], rd[:, 2]], 1)
        r["y"][:w] = np.stack([wr[:, 1], np.full(w, sh), np.full(w, clk), wr[:, 0], wr[:, 2], wr[:, 3]], 1)
    return out


def ec_decompress_trace(curve: str, events_dev, n: int, height: int = None, byte_mult=None):
    """WeierstrassDecompress main trace of secp256k1 / secp256r1 / bls12-381 (on the GPU) from n
    zkm_ec_decompress_event records; the Byte lookups added into byte_mult (nullable)."""
    from . import mips_ec as EC
    height = height or _pow2(n)
    t = _trace(height, EC.DecompressLayout(EC.FIELDS[curve], EC.LEXICOGRAPHIC[curve]).WIDTH)
    what = "zkm_ec_decompress_events_to_trace"
    _lib.check(_bind().zkm_ec_decompress_events_to_trace(EC_CURVES[curve],
                                                         _records(events_dev, n, EC_DECOMPRESS_EVENT, what), n,
                                                         t.data_ptr(), height, _words(byte_mult, 65536 * 10, what),
                                                         _stream()), what)
    return t


ED_ADD_EVENT = np.dtype({"names": ["shard", "clk", "p_ptr", "q_ptr", "q", "p"],
                         "formats": [u4, u4, u4, u4, (u4, (16, 5)), (u4, (16, 6))],
                         "offsets": [0, 4, 8, 12, 16, 336], "itemsize": 720})
ED_ADD_WIDTH = 1861  # ZKM_ED_ADD_WIDTH


def ed_add_records(events) -> np.ndarray:
    """zkm_ed_add_event records of the executor's ED_ADD events (mips_edwards.exec_ed_add): q read at clk, p
    written at clk + 1."""
    out = np.zeros(len(events), ED_ADD_EVENT)
    for k, e in enumerate(events):
        sh, clk = e["shard"], e["clk"]
        r = out[k]
        r["shard"], r["clk"], r["p_ptr"], r["q_ptr"] = sh, clk, e["p_ptr"], e["q_ptr"]
        rd = np.asarray(e["q"], np.int64).reshape(16, 3)
        wr = np.asarray(e["pw"], np.int64).reshape(16, 4)
        r["q"] = np.stack([rd[:, 0], np.full(16, sh), np.full(16, clk), rd[:, 1], rd[:, 2]], 1)
        r["p"] = np.stack([wr[:, 1], np.full(16, sh), np.full(16, clk + 1), wr[:, 0], wr[:, 2], wr[:, 3]], 1)
    return out


def ed_add_trace(events_dev, n: int, height: int = None, byte_mult=None):
    """EdAddAssign main trace (height x 1861 int32, on the GPU) from n zkm_ed_add_event records; the Byte
    lookups added into byte_mult (nullable)."""
    height = height or _pow2(n)
    t = _trace(height, ED_ADD_WIDTH)
    what = "zkm_ed_add_events_to_trace"
    _lib.check(_bind().zkm_ed_add_events_to_trace(_records(events_dev, n, ED_ADD_EVENT, what), n, t.data_ptr(), height,
                                                  _words(byte_mult, 65536 * 10, what), _stream()), what)
    return t


ED_DECOMPRESS_EVENT = np.dtype({"names": ["shard", "clk", "ptr", "sign", "y", "x"],
                                "formats": [u4, u4, u4, u4, (u4, (8, 5)), (u4, (8, 6))],
                                "offsets": [0, 4, 8, 12, 16, 176], "itemsize": 368})
ED_DECOMPRESS_WIDTH = 1566  # ZKM_ED_DECOMPRESS_WIDTH


def ed_decompress_records(events) -> np.ndarray:
    """zkm_ed_decompress_event records of the executor's ED_DECOMPRESS events (mips_edwards.exec_ed_decompress):
    y read and x written at clk."""
    out = np.zeros(len(events), ED_DECOMPRESS_EVENT)
    for k, e in enumerate(events):
        sh, clk = e["shard"], e["clk"]
        r = out[k]
        r["shard"], r["clk"], r["ptr"], r["sign"] = sh, clk, e["ptr"], e["sign"]
        rd = np.asarray(e["y"], np.int64).reshape(8, 3)
        wr = np.asarray(e["x"], np.int64).reshape(8, 4)
        r["y"] = np.stack([rd[:, 0], np.full(8, sh), np.full(8, clk), rd[:, 1], rd[:, 2]], 1)
        r["x"] = np.stack([wr[:, 1], np.full(8, sh), np.full(8, clk), wr[:, 0], wr[:, 2], wr[:, 3]], 1)
    return out


def ed_decompress_trace(events_dev, n: int, height: int = None, byte_mult=None):
    """EdDecompress main trace (height x 1566 int32, on the GPU) from n zkm_ed_decompress_event records; the
    Byte lookups added into byte_mult (nullable)."""
    height = height or _pow2(n)
    t = _trace(height, ED_DECOMPRESS_WIDTH)
    what = "zkm_ed_decompress_events_to_trace"
    _lib.check(_bind().zkm_ed_decompress_events_to_trace(_records(events_dev, n, ED_DECOMPRESS_EVENT, what), n,
                                                         t.data_ptr(), height, _words(byte_mult, 65536 * 10, what),
                                                         _stream()), what)
    return t


KECCAK_BLOCK = np.dtype({"names": ["shard", "clk", "in_ptr", "out_ptr", "in_len", "block", "nblocks", "xored",
                                   "prev_xored", "in", "len", "out"],
                         "formats": [u4] * 7 + [(u4, 50), (u4, 50), (u4, (36, 5)), (u4, 5), (u4, (16, 6))],
                         "offsets": [0, 4, 8, 12, 16, 20, 24, 28, 228, 428, 1148, 1168], "itemsize": 1552})
KECCAK_SPONGE_WIDTH = 3531  # ZKM_KECCAK_SPONGE_WIDTH


def keccak_blocks(events) -> np.ndarray:
    """zkm_keccak_block records (one per absorbed block) of the executor's KECCAK_SPONGE events
    (mips_keccak.exec_keccak_sponge): input and length read at clk, output written at clk + 1."""
    def lanes(st):
        v = np.asarray(st, np.uint64)
        return np.stack([v & np.uint64(0xFFFFFFFF), v >> np.uint64(32)], 1).reshape(-1).astype(np.uint32)
    rows = []
    for e in events:
        sh, clk, nb = e["shard"], e["clk"], len(e["xored"])
        rd = np.asarray(e["in"], np.int64).reshape(-1, 3)
        ln = e["len"]
        wr = np.asarray(e["w"], np.int64).reshape(16, 4)
        out = np.stack([wr[:, 1], np.full(16, sh), np.full(16, clk + 1), wr[:, 0], wr[:, 2], wr[:, 3]], 1)
        for k in range(nb):
            r = np.zeros(1, KECCAK_BLOCK)[0]
            r["shard"], r["clk"], r["in_ptr"], r["out_ptr"] = sh, clk, e["in_ptr"] + 144 * k, e["out_ptr"]
            r["in_len"], r["block"], r["nblocks"] = len(e["in"]), k, nb
            r["xored"] = lanes(e["xored"][k])
            if k:
                r["prev_xored"] = lanes(e["xored"][k - 1])
            b = rd[36 * k:36 * (k + 1)]
            r["in"] = np.stack([b[:, 0], np.full(36, sh), np.full(36, clk), b[:, 1], b[:, 2]], 1)
            r["len"] = [ln[0], sh, clk, ln[1], ln[2]]
            r["out"] = out
            rows.append(r)
    return np.array(rows, KECCAK_BLOCK) if rows else np.zeros(0, KECCAK_BLOCK)


def keccak_sponge_trace(blocks_dev, n: int, height: int = None, byte_mult=None):
    """KeccakSponge main trace (height x 3531 int32, on the GPU) from n zkm_keccak_block records (24 rows
    each); the Byte lookups added into byte_mult (nullable)."""
    height = height or _pow2(24 * n)
    t = _trace(height, KECCAK_SPONGE_WIDTH)
    what = "zkm_keccak_sponge_events_to_trace"
    _lib.check(_bind().zkm_keccak_sponge_events_to_trace(_records(blocks_dev, n, KECCAK_BLOCK, what), n, t.data_ptr(),
                                                         height, _words(byte_mult, 65536 * 10, what), _stream()), what)
    return t


SYS_LINUX_EVENT = np.dtype({"names": ["shard", "clk", "code", "a0", "a1", "result", "a3", "io"],
                            "formats": [u4, u4, u4, u4, u4, u4, (u4, 6), (u4, 6)],
                            "offsets": [0, 4, 8, 12, 16, 20, 24, 48], "itemsize": 72})
SYS_LINUX_WIDTH = 69  # ZKM_SYS_LINUX_WIDTH


def sys_linux_records(events) -> np.ndarray:
    """zkm_sys_linux_event records of the executor's Linux syscall events (mips_syscall.exec_sys_linux):
    the A3 write and the io access (BRK / WRITE: the register read, MMAP(2) with a0 = 0: the heap write)."""
    from . import mips_syscall as SY
    out = np.zeros(len(events), SYS_LINUX_EVENT)
    for k, e in enumerate(events):
        sh, clk, code = e["shard"], e["clk"], e["code"]
        r = out[k]
        r["shard"], r["clk"], r["code"], r["a0"], r["a1"], r["result"] = sh, clk, code, e["a0"], e["a1"], e["v0"]
        prev, val, ps, pc = e["writes"][0]
        r["a3"] = [val, sh, clk, prev, ps, pc]
        if code in (SY.SYS_BRK, SY.SYS_WRITE):
            val, ps, pc = e["reads"][0]
            r["io"] = [val, sh, clk, val, ps, pc]
        elif code in (SY.SYS_MMAP, SY.SYS_MMAP2) and e["a0"] == 0:
            prev, val, ps, pc = e["writes"][1]
            r["io"] = [val, sh, clk, prev, ps, pc]
    return out


def sys_linux_trace(events_dev, n: int, height: int = None, byte_mult=None):
    """SysLinux main trace (height x 69 int32, on the GPU) from n zkm_sys_linux_event records; the Byte
    lookups added into byte_mult (nullable)."""
    height = height or _pow2(n)
    t = _trace(height, SYS_LINUX_WIDTH)
    what = "zkm_sys_linux_events_to_trace"
    _lib.check(_bind().zkm_sys_linux_events_to_trace(_records(events_dev, n, SYS_LINUX_EVENT, what), n, t.data_ptr(),
                                                     height, _words(byte_mult, 65536 * 10, what), _stream()), what)
    return t


POSEIDON2_PERMUTE_EVENT = np.dtype({"names": ["shard", "clk", "ptr", "state"], "formats": [u4, u4, u4, (u4, (16, 6))],
                                    "offsets": [0, 4, 8, 12], "itemsize": 396})
POSEIDON2_PERMUTE_WIDTH = 973  # ZKM_POSEIDON2_PERMUTE_WIDTH


def poseidon2_permute_records(events) -> np.ndarray:
    """zkm_poseidon2_permute_event records of the executor's POSEIDON2_PERMUTE events
    (mips_p2permute.exec_poseidon2_permute): the 16 state words written at the call's clk."""
    out = np.zeros(len(events), POSEIDON2_PERMUTE_EVENT)
    for k, ev in enumerate(events):
        w = np.asarray(ev["w"], np.int64).reshape(16, 4)  # prev_value, value, prev_shard, prev_clk
        out[k]["shard"], out[k]["clk"], out[k]["ptr"] = ev["shard"], ev["clk"], ev["ptr"]
        out[k]["state"] = np.stack([w[:, 1], np.full(16, ev["shard"]), np.full(16, ev["clk"]), w[:, 0], w[:, 2],
                                    w[:, 3]], 1)
    return out


def poseidon2_permute_trace(events_dev, n: int, height: int = None, byte_mult=None):
    """Poseidon2Permute main trace (height x 973 int32, on the GPU) from n zkm_poseidon2_permute_event
    records; its accesses' Byte lookups added into byte_mult (nullable)."""
    height = height or _pow2(n)
    t = _trace(height, POSEIDON2_PERMUTE_WIDTH)
    what = "zkm_poseidon2_permute_events_to_trace"
    _lib.check(_bind().zkm_poseidon2_permute_events_to_trace(_records(events_dev, n, POSEIDON2_PERMUTE_EVENT, what), n,
                                                             t.data_ptr(), height, _words(byte_mult, 65536 * 10, what),
                                                             _stream()), what)
    return t


def sha_extend_trace(rows_dev, n: int, height: int = None, byte_mult=None):
    """ShaExtend main trace (height x 176 int32 on the GPU) from n flattened rows (n a multiple of 48)."""
    height = height or max(16, 1 << max(2, (n - 1).bit_length()))
    t = _trace(height, SHA_EXTEND_WIDTH)
    what = "zkm_sha_extend_events_to_trace"
    _lib.check(_bind().zkm_sha_extend_events_to_trace(_records(rows_dev, n, SHA_EXTEND_ROW, what), n, t.data_ptr(),
                                                       height, _words(byte_mult, 65536 * 10, what), _stream()), what)
    return t


def sha_compress_records(events) -> np.ndarray:
    """ShaCompress call records of the executor's SHA_COMPRESS events (mips_syscall.exec_sha_compress): h and
    w read at clk, h written at clk + 1."""
    out = np.zeros(len(events), SHA_COMPRESS_EVENT)
    for k, ev in enumerate(events):
        sh, clk = ev["shard"], ev["clk"]
        hr = np.asarray(ev["hr"], np.int64).reshape(8, 3)
        wr = np.asarray(ev["wr"], np.int64).reshape(64, 3)
        hw = np.asarray(ev["hw"], np.int64).reshape(8, 4)  # prev_value, value, prev_shard, prev_clk
        out[k]["shard"], out[k]["clk"], out[k]["w_ptr"], out[k]["h_ptr"] = sh, clk, ev["w_ptr"], ev["h_ptr"]
        out[k]["h_read"] = np.stack([hr[:, 0], np.full(8, sh), np.full(8, clk), hr[:, 1], hr[:, 2]], 1)
        out[k]["w_read"] = np.stack([wr[:, 0], np.full(64, sh), np.full(64, clk), wr[:, 1], wr[:, 2]], 1)
        out[k]["h_write"] = np.stack([hw[:, 1], np.full(8, sh), np.full(8, clk + 1), hw[:, 0], hw[:, 2], hw[:, 3]], 1)
    return out


def sha_compress_trace(events_dev, n: int, height: int = None, byte_mult=None):
    """ShaCompress main trace (height x 262 int32 on the GPU) from n call records (80 rows each)."""
    height = height or _pow2(80 * n)
    t = _trace(height, SHA_COMPRESS_WIDTH)
    what = "zkm_sha_compress_events_to_trace"
    _lib.check(_bind().zkm_sha_compress_events_to_trace(_records(events_dev, n, SHA_COMPRESS_EVENT, what), n,
                                                         t.data_ptr(), height, _words(byte_mult, 65536 * 10, what),
                                                         _stream()), what)
    return t


def alu_records(alu, kind: str) -> np.ndarray:
    """The AluEvents of one ALU chip (kind "add", "bit", "lt", "sll" or "sr") from the executor's event
    lists; ShiftRight's include the SRL dependencies of the CLZ / CLO events."""
    def cols(lst):
        R = _rows(lst, 6).astype(np.uint32)
        return tuple(R[:, i] for i in range(6))
    ev = alu.get(kind, [])
    arrs = cols(ev) if len(ev) else tuple(np.zeros(0, np.uint32) for _ in range(6))
    if kind == "sr" and len(alu.get("clz", [])):
        op, a, b = cols(alu["clz"])[:3]
        dep = A.clz_dependencies(op, a, b)
        arrs = tuple(np.concatenate([x, d]).astype(np.uint32) for x, d in zip(arrs, dep))
    op, a, b, c, pc, npc = arrs
    return alu_events(op, a, b, c, pc, npc)


# ---------------------------------------------------------------- device entry points
def _bind():
    L = _lib.lib()
    if not getattr(L, "_tracegen_bound", False):
        vp, u64 = C.c_void_p, C.c_uint64
        L.zkm_cpu_events_to_trace.argtypes = [vp, u64, C.c_uint32, vp, u64, C.c_uint32, vp, u64, vp, vp, vp]
        L.zkm_add_sub_events_to_trace.argtypes = [vp, u64, vp, u64, vp, vp]
        for f in ALU_CHIPS.values():
            getattr(L, f[0]).argtypes = [vp, u64, vp, u64, vp, vp]
        L.zkm_branch_events_to_trace.argtypes = [vp, u64, vp, u64, vp, vp]
        L.zkm_jump_events_to_trace.argtypes = [vp, u64, vp, u64, vp]
        L.zkm_movcond_events_to_trace.argtypes = [vp, u64, vp, u64, vp]
        L.zkm_mul_events_to_trace.argtypes = [vp, u64, vp, u64, vp, vp]
        L.zkm_divrem_events_to_trace.argtypes = [vp, u64, vp, u64, vp, vp]
        L.zkm_clo_clz_events_to_trace.argtypes = [vp, u64, vp, u64, vp, vp]
        L.zkm_syscall_instrs_events_to_trace.argtypes = [vp, u64, vp, u64, vp]
        L.zkm_misc_instrs_events_to_trace.argtypes = [vp, u64, vp, u64, vp, vp]
        L.zkm_sha_extend_events_to_trace.argtypes = [vp, u64, vp, u64, vp, vp]
        L.zkm_sha_compress_events_to_trace.argtypes = [vp, u64, vp, u64, vp, vp]
        L.zkm_poseidon2_permute_events_to_trace.argtypes = [vp, u64, vp, u64, vp, vp]
        L.zkm_sys_linux_events_to_trace.argtypes = [vp, u64, vp, u64, vp, vp]
        L.zkm_uint256_mul_events_to_trace.argtypes = [vp, u64, vp, u64, vp, vp]
        L.zkm_u256x2048_mul_events_to_trace.argtypes = [vp, u64, vp, u64, vp, vp]
        L.zkm_fp_op_events_to_trace.argtypes = [C.c_int, vp, u64, vp, u64, vp, vp]
        L.zkm_fp2_events_to_trace.argtypes = [C.c_int, C.c_int, vp, u64, vp, u64, vp, vp]
        L.zkm_ec_add_events_to_trace.argtypes = [C.c_int, vp, u64, vp, u64, vp, vp]
        L.zkm_ec_double_events_to_trace.argtypes = [C.c_int, vp, u64, vp, u64, vp, vp]
        L.zkm_ec_decompress_events_to_trace.argtypes = [C.c_int, vp, u64, vp, u64, vp, vp]
        L.zkm_ed_add_events_to_trace.argtypes = [vp, u64, vp, u64, vp, vp]
        L.zkm_ed_decompress_events_to_trace.argtypes = [vp, u64, vp, u64, vp, vp]
        L.zkm_keccak_sponge_events_to_trace.argtypes = [vp, u64, vp, u64, vp, vp]
        L.zkm_memory_instrs_events_to_trace.argtypes = [vp, u64, vp, u64, vp, vp]
        L.zkm_memory_local_events_to_trace.argtypes = [vp, u64, vp, u64, vp]
        L.zkm_memory_global_events_to_trace.argtypes = [vp, u64, C.c_int, C.c_uint32, vp, u64, vp]
        L.zkm_syscall_events_to_trace.argtypes = [vp, u64, C.c_int, vp, u64, vp]
        L.zkm_global_events_to_trace.argtypes = [vp, u64, vp, u64, vp, vp, vp]
        L.zkm_poseidon2_wide_events_to_trace.argtypes = [vp, u64, C.c_uint32, vp, u64, vp]
        L.zkm_exp_reverse_bits_events_to_trace.argtypes = [vp, vp, vp, u64, C.c_uint32, vp, u64, vp]
        L.zkm_recursion_events_to_trace.argtypes = [C.c_uint32, vp, u64, C.c_uint32, vp, u64, vp]
        L.zkm_recursion_instrs_to_trace.argtypes = [C.c_uint32, vp, u64, C.c_uint32, vp, u64, vp]
        L._tracegen_bound = True
    return L


def _torch():
    import torch
    return torch


def to_device(records: np.ndarray):
    """A structured record array as a uint8 torch tensor on the current GPU (the record dtypes above:
    numpy operations that repack a padded dtype, e.g. np.resize, must not have touched it)."""
    torch = _torch()
    if records.dtype not in (CPU_EVENT, INSTRUCTION, ALU_EVENT, MEMORY_LOCAL_EVENT, MEMORY_INIT_FINAL_EVENT,
                             SYSCALL_EVENT, GLOBAL_EVENT, BRANCH_EVENT, MEM_INSTR_EVENT, MOVCOND_EVENT,
                             COMP_ALU_EVENT, MISC_EVENT, SHA_EXTEND_ROW, SHA_COMPRESS_EVENT, POSEIDON2_PERMUTE_EVENT,
                             SYS_LINUX_EVENT, UINT256_MUL_EVENT, U256X2048_MUL_EVENT, FP_OP_EVENT,
                             FP2_EVENT, EC_ADD_EVENT, EC_DOUBLE_EVENT, EC_DECOMPRESS_EVENT,
                             ED_ADD_EVENT, ED_DECOMPRESS_EVENT, KECCAK_BLOCK):
        raise ValueError(f"not a record array of zkm_tracegen.h: {records.dtype}")
    raw = np.ascontiguousarray(records).view(np.uint8).reshape(-1)
    return torch.from_numpy(raw.copy()).cuda() if raw.size else torch.zeros(1, dtype=torch.uint8, device="cuda")


def _ptr(t):
    return None if t is None else t.data_ptr()


def _records(t, n: int, dtype: np.dtype, what: str):
    """The device pointer of n records of `dtype` in tensor t, after checking t holds them (the ABI
    takes bare pointers: a short buffer would be read past its end)."""
    if n and (t is None or not t.is_cuda or t.numel() * t.element_size() < n * dtype.itemsize):
        raise ValueError(f"{what}: need {n} records of {dtype.itemsize} bytes on the GPU")
    return _ptr(t)


def _words(t, n: int, what: str):
    if t is not None and (not t.is_cuda or not t.is_contiguous() or t.element_size() != 4 or t.numel() < n):
        raise ValueError(f"{what}: need a contiguous 32-bit GPU tensor of at least {n} values")
    return _ptr(t)


def _stream():
    return _torch().cuda.current_stream().cuda_stream


def _pow2(n: int) -> int:
    return max(16, 1 << max(0, (n - 1).bit_length()))


def _trace(height: int, width: int):
    torch = _torch()
    return torch.empty((height, width), dtype=torch.int32, device="cuda")


def cpu_trace(events_dev, n: int, shard: int, program_dev, program_len: int, height: int = None, byte_mult=None,
              program_mult=None, pc_base: int = MC.PC_BASE):
    """Cpu main trace (height x 67 int32 on the GPU) from n CpuEventFfi records on the GPU."""
    height = height or _pow2(n)
    t = _trace(height, CPU_WIDTH)
    what = "zkm_cpu_events_to_trace"
    _lib.check(_bind().zkm_cpu_events_to_trace(_records(events_dev, n, CPU_EVENT, what), n, shard,
                                                _records(program_dev, program_len, INSTRUCTION, what), program_len,
                                                pc_base, t.data_ptr(), height, _words(byte_mult, 65536 * 10, what),
                                                _words(program_mult, program_len, what), _stream()), what)
    return t


def add_sub_trace(events_dev, n: int, height: int = None, byte_mult=None):
    height = height or _pow2(n)
    t = _trace(height, ADD_SUB_WIDTH)
    what = "zkm_add_sub_events_to_trace"
    _lib.check(_bind().zkm_add_sub_events_to_trace(_records(events_dev, n, ALU_EVENT, what), n, t.data_ptr(), height,
                                                    _words(byte_mult, 65536 * 10, what), _stream()), what)
    return t


# ALU chips on the AluEvent ABI beside AddSub: executor kind -> (entry point, chip, width)
ALU_CHIPS = {"bit": ("zkm_bitwise_events_to_trace", "Bitwise", 18), "lt": ("zkm_lt_events_to_trace", "Lt", 36),
             "sll": ("zkm_shift_left_events_to_trace", "ShiftLeft", 44),
             "sr": ("zkm_shift_right_events_to_trace", "ShiftRight", 71)}


def alu_trace(kind: str, events_dev, n: int, height: int = None, byte_mult=None):
    """Bitwise / Lt / ShiftLeft / ShiftRight main trace (height x width int32 on the GPU) from n AluEvents."""
    fn, _, width = ALU_CHIPS[kind]
    height = height or _pow2(n)
    t = _trace(height, width)
    _lib.check(getattr(_bind(), fn)(_records(events_dev, n, ALU_EVENT, fn), n, t.data_ptr(), height,
                                    _words(byte_mult, 65536 * 10, fn), _stream()), fn)
    return t


def branch_trace(events_dev, n: int, height: int = None, byte_mult=None):
    height = height or _pow2(n)
    t = _trace(height, BRANCH_WIDTH)
    what = "zkm_branch_events_to_trace"
    _lib.check(_bind().zkm_branch_events_to_trace(_records(events_dev, n, BRANCH_EVENT, what), n, t.data_ptr(), height,
                                                   _words(byte_mult, 65536 * 10, what), _stream()), what)
    return t


def memory_instrs_trace(events_dev, n: int, height: int = None, byte_mult=None):
    height = height or _pow2(n)
    t = _trace(height, MEMORY_INSTRS_WIDTH)
    what = "zkm_memory_instrs_events_to_trace"
    _lib.check(_bind().zkm_memory_instrs_events_to_trace(_records(events_dev, n, MEM_INSTR_EVENT, what), n,
                                                          t.data_ptr(), height, _words(byte_mult, 65536 * 10, what),
                                                          _stream()), what)
    return t


def jump_trace(events_dev, n: int, height: int = None):
    height = height or _pow2(n)
    t = _trace(height, JUMP_WIDTH)
    what = "zkm_jump_events_to_trace"
    _lib.check(_bind().zkm_jump_events_to_trace(_records(events_dev, n, JUMP_EVENT, what), n, t.data_ptr(), height,
                                                 _stream()), what)
    return t


def movcond_trace(events_dev, n: int, height: int = None):
    height = height or _pow2(n)
    t = _trace(height, MOVCOND_WIDTH)
    what = "zkm_movcond_events_to_trace"
    _lib.check(_bind().zkm_movcond_events_to_trace(_records(events_dev, n, MOVCOND_EVENT, what), n, t.data_ptr(),
                                                    height, _stream()), what)
    return t


def mul_trace(events_dev, n: int, height: int = None, byte_mult=None):
    height = height or _pow2(n)
    t = _trace(height, MUL_WIDTH)
    what = "zkm_mul_events_to_trace"
    _lib.check(_bind().zkm_mul_events_to_trace(_records(events_dev, n, COMP_ALU_EVENT, what), n, t.data_ptr(), height,
                                                _words(byte_mult, 65536 * 10, what), _stream()), what)
    return t


def divrem_trace(events_dev, n: int, height: int = None, byte_mult=None):
    height = height or _pow2(n)
    t = _trace(height, DIVREM_WIDTH)
    what = "zkm_divrem_events_to_trace"
    _lib.check(_bind().zkm_divrem_events_to_trace(_records(events_dev, n, COMP_ALU_EVENT, what), n, t.data_ptr(),
                                                   height, _words(byte_mult, 65536 * 10, what), _stream()), what)
    return t


def clo_clz_trace(events_dev, n: int, height: int = None, byte_mult=None):
    height = height or _pow2(n)
    t = _trace(height, CLO_CLZ_WIDTH)
    what = "zkm_clo_clz_events_to_trace"
    _lib.check(_bind().zkm_clo_clz_events_to_trace(_records(events_dev, n, ALU_EVENT, what), n, t.data_ptr(), height,
                                                    _words(byte_mult, 65536 * 10, what), _stream()), what)
    return t


def syscall_instrs_trace(events_dev, n: int, height: int = None):
    height = height or _pow2(n)
    t = _trace(height, SYSCALL_INSTRS_WIDTH)
    what = "zkm_syscall_instrs_events_to_trace"
    _lib.check(_bind().zkm_syscall_instrs_events_to_trace(_records(events_dev, n, SYSCALL_EVENT, what), n,
                                                           t.data_ptr(), height, _stream()), what)
    return t


def misc_instrs_trace(events_dev, n: int, height: int = None, byte_mult=None):
    height = height or _pow2(n)
    t = _trace(height, MISC_INSTRS_WIDTH)
    what = "zkm_misc_instrs_events_to_trace"
    _lib.check(_bind().zkm_misc_instrs_events_to_trace(_records(events_dev, n, MISC_EVENT, what), n, t.data_ptr(),
                                                        height, _words(byte_mult, 65536 * 10, what), _stream()), what)
    return t


def memory_local_trace(events_dev, n: int, height: int = None):
    height = height or _pow2((n + 3) // 4)
    t = _trace(height, MEMORY_LOCAL_WIDTH)
    what = "zkm_memory_local_events_to_trace"
    _lib.check(_bind().zkm_memory_local_events_to_trace(_records(events_dev, n, MEMORY_LOCAL_EVENT, what), n,
                                                         t.data_ptr(), height, _stream()), what)
    return t


def memory_global_trace(events_dev, n: int, initialize: bool, prev_addr: int = 0, height: int = None):
    height = height or _pow2(n)
    t = _trace(height, MEMORY_GLOBAL_WIDTH)
    what = "zkm_memory_global_events_to_trace"
    _lib.check(_bind().zkm_memory_global_events_to_trace(_records(events_dev, n, MEMORY_INIT_FINAL_EVENT, what), n,
                                                          0 if initialize else 1, prev_addr, t.data_ptr(), height,
                                                          _stream()), what)
    return t


def syscall_trace(events_dev, n: int, height: int = None):
    height = height or _pow2(n)
    t = _trace(height, SYSCALL_WIDTH)
    what = "zkm_syscall_events_to_trace"
    _lib.check(_bind().zkm_syscall_events_to_trace(_records(events_dev, n, SYSCALL_EVENT, what), n, 0, t.data_ptr(),
                                                    height, _stream()), what)
    return t


def global_trace(events_dev, n: int, height: int = None, byte_mult=None):
    """Global main trace (height x 99 int32 on the GPU) and the shard's global cumulative sum (14
    canonical words, numpy) from n GlobalLookupEvent records on the GPU."""
    torch = _torch()
    height = height or _pow2(n)
    t = _trace(height, GLOBAL_WIDTH)
    fin = torch.zeros(14, dtype=torch.int32, device="cuda")
    what = "zkm_global_events_to_trace"
    _lib.check(_bind().zkm_global_events_to_trace(_records(events_dev, n, GLOBAL_EVENT, what), n, t.data_ptr(),
                                                   height, _words(byte_mult, 65536 * 10, what), fin.data_ptr(),
                                                   _stream()), what)
    return t, fin.cpu().numpy().view(np.uint32)


def shard_records(capture: dict) -> dict:
    """The event records of one executed shard (program_shard(..., capture=c)) by chip, as the header's
    structs (numpy): what a host hands the device before its traces are built."""
    shard = capture["shard"]
    r = {"Cpu": cpu_events(capture["steps"], shard), "Program": program_ffi(capture["prog"]),
         "AddSub": add_sub_records(capture["alu"])}
    for kind, (_, chip, _) in ALU_CHIPS.items():
        r[chip] = alu_records(capture["alu"], kind)
    r["CloClz"] = alu_records(capture["alu"], "clz")
    r["Branch"] = branch_records(capture.get("branches", []))
    r["MemoryInstrs"] = mem_instr_records(capture.get("mevs", []), shard)
    r["Jump"] = jump_records(capture.get("jumps", []))
    r["MovCond"] = movcond_records(capture.get("movs", []))
    r["Mul"] = mul_records(capture.get("muls", []), shard)
    r["DivRem"] = divrem_records(capture.get("divs", []), shard)
    r["MiscInstrs"] = misc_records(capture.get("misc", []), shard)
    r["MemoryLocal"] = memory_local_events(capture["entries"])
    r["SyscallCore"] = syscall_events(capture["core_syscalls"]) if len(capture["core_syscalls"]) else \
        np.zeros(0, SYSCALL_EVENT)
    r["SyscallInstrs"] = syscall_events(capture["syscalls"]) if len(capture["syscalls"]) else np.zeros(0, SYSCALL_EVENT)
    r["Global"] = shard_global_events(capture)
    return r


def shard_traces(capture: dict, byte_mult=None, heights: dict = None, records: dict = None):
    """Device traces of one executed shard (program_shard(..., capture=c)): the chips of the reference's
    row ABI — Cpu (+ Program multiplicities), AddSub, MemoryLocal, SyscallCore — and beyond it Bitwise,
    Lt, ShiftLeft, ShiftRight, CloClz, Branch, MemoryInstrs, Jump, MovCond, Mul, DivRem, MiscInstrs,
    SyscallInstrs and the Global chip (septic-curve lift and running sum), with their Byte lookups added
    into `byte_mult` (65536 x 10 int32 on the GPU) if given.  heights: chip -> trace height (e.g. a
    reference shard shape; default the next power of two); records: the shard_records already on the GPU
    (uploaded here otherwise).  Chips with no events are left out unless heights names them.  Returns
    {chip name: GPU tensor}."""
    torch = _torch()
    heights = heights or {}
    host = shard_records(capture) if records is None else None
    nrec = {k: len(v) for k, v in (host or {}).items()}
    if records is None:
        records = {k: to_device(v) for k, v in host.items()}
    else:
        nrec = records.get("_n", nrec)
    n = lambda k: nrec[k] if nrec else 0
    h = lambda k, default: heights.get(k, default)
    want = lambda k: n(k) > 0 or k in heights
    shard = capture["shard"]
    npf = n("Program")
    pm = torch.zeros((h("Program", _pow2(npf)), 1), dtype=torch.int32, device="cuda")
    out = {"Cpu": cpu_trace(records["Cpu"], n("Cpu"), shard, records["Program"], npf, height=h("Cpu", None),
                            byte_mult=byte_mult, program_mult=pm),
           "Program": pm}
    if want("AddSub"):
        out["AddSub"] = add_sub_trace(records["AddSub"], n("AddSub"), height=h("AddSub", None), byte_mult=byte_mult)
    for kind, (_, chip, _) in ALU_CHIPS.items():
        if want(chip):
            out[chip] = alu_trace(kind, records[chip], n(chip), height=h(chip, None), byte_mult=byte_mult)
    simple = (("Branch", branch_trace, True), ("MemoryInstrs", memory_instrs_trace, True), ("Jump", jump_trace, False),
              ("MovCond", movcond_trace, False), ("Mul", mul_trace, True), ("DivRem", divrem_trace, True),
              ("MiscInstrs", misc_instrs_trace, True), ("CloClz", clo_clz_trace, True))
    for chip, fn, bytes_ in simple:
        if want(chip):
            kw = {"byte_mult": byte_mult} if bytes_ else {}
            out[chip] = fn(records[chip], n(chip), height=h(chip, None), **kw)
    out["MemoryLocal"] = memory_local_trace(records["MemoryLocal"], n("MemoryLocal"), height=h("MemoryLocal", None))
    if want("SyscallCore"):
        out["SyscallCore"] = syscall_trace(records["SyscallCore"], n("SyscallCore"), height=h("SyscallCore", None))
    if want("SyscallInstrs"):
        out["SyscallInstrs"] = syscall_instrs_trace(records["SyscallInstrs"], n("SyscallInstrs"),
                                                    height=h("SyscallInstrs", None))
    out["Global"], _ = global_trace(records["Global"], n("Global"), height=h("Global", None), byte_mult=byte_mult)
    return out


def shard_records_to_device(capture: dict) -> dict:
    """shard_records uploaded (the `records` argument of shard_traces), with their counts under "_n"."""
    host = shard_records(capture)
    d = {k: to_device(v) for k, v in host.items()}
    d["_n"] = {k: len(v) for k, v in host.items()}
    return d


POSEIDON2_WIDE_WIDTH = 313  # ZKM_POSEIDON2_WIDE_DEG3_WIDTH


def poseidon2_wide_trace(events_dev, n: int, height: int = None, montgomery: bool = False):
    """Poseidon2WideDeg3 main trace (height x 313 int32, canonical, on the GPU) from n Poseidon2Io
    records (32 words: input[16], output[16]) in a uint32/int32 GPU tensor; rows >= n are the
    permutation of zero (recursion/core/src/chips/poseidon2_wide/trace.rs)."""
    height = height or _pow2(n)
    t = _trace(height, POSEIDON2_WIDE_WIDTH)
    what = "zkm_poseidon2_wide_events_to_trace"
    _lib.check(_bind().zkm_poseidon2_wide_events_to_trace(_words(events_dev, 32 * n, what) if n else None, n,
                                                          1 if montgomery else 0, t.data_ptr(), height, _stream()), what)
    return t


EXP_REVERSE_BITS_LEN_WIDTH = 7  # ZKM_EXP_REVERSE_BITS_LEN_WIDTH


def exp_reverse_bits_trace(base_dev, bits_dev, offsets_dev, n: int, height: int, montgomery: bool = False):
    """ExpReverseBitsLen main trace (height x 7 int32, canonical, on the GPU): event e's bits are
    bits[offsets[e]:offsets[e+1]] (int64 offsets, n + 1 of them, on the GPU)."""
    t = _trace(height, EXP_REVERSE_BITS_LEN_WIDTH)
    what = "zkm_exp_reverse_bits_events_to_trace"
    if offsets_dev is None or not offsets_dev.is_cuda or offsets_dev.element_size() != 8 or offsets_dev.numel() < n + 1:
        raise ValueError(f"{what}: need n + 1 int64 offsets on the GPU")
    _lib.check(_bind().zkm_exp_reverse_bits_events_to_trace(_words(base_dev, n, what) if n else None,
                                                            _words(bits_dev, 0, what) if n else None, _ptr(offsets_dev),
                                                            n, 1 if montgomery else 0, t.data_ptr(), height, _stream()),
               what)
    return t


# zkm_recursion_events_to_trace chips: name -> (ZKM_REC_CHIP_*, words per event, events per row)
RECURSION_EVENT_CHIPS = {"BaseAlu": (0, 3, 4), "ExtAlu": (1, 12, 4), "BatchFRI": (2, 13, 1), "Select": (3, 5, 1),
                         "FriFold": (4, 33, 1), "PublicValues": (5, 1, 1), "MemoryVar": (6, 4, 2),
                         "MemoryConst": (7, 1, 0)}


def recursion_events_trace(chip: str, events_dev, n: int, height: int, montgomery: bool = False):
    """Main trace (height x width int32, canonical, on the GPU) of a recursion chip whose rows are its events
    (RECURSION_EVENT_CHIPS): n events of the chip's width back to back in a 32-bit GPU tensor."""
    code, w, k = RECURSION_EVENT_CHIPS[chip]
    t = _trace(height, w * k if k else 1)
    what = "zkm_recursion_events_to_trace"
    _lib.check(_bind().zkm_recursion_events_to_trace(code, _words(events_dev, n * w, what) if n else None, n,
                                                     1 if montgomery else 0, t.data_ptr(), height, _stream()), what)
    return t


# zkm_recursion_instrs_to_trace chips: name -> (ZKM_REC_CHIP_*, words per record, preprocessed width, the
# record words that are plain integers rather than field elements)
RECURSION_INSTR_CHIPS = {"BaseAlu": (0, 5, 32, (3,)), "ExtAlu": (1, 5, 32, (3,)), "BatchFRI": (2, 5, 6, (4,)),
                         "Select": (3, 7, 8, ()), "FriFold": (4, 12, 20, (11,)), "PublicValues": (5, 1, 10, ()),
                         "MemoryVar": (6, 2, 4, ()), "MemoryConst": (7, 6, 12, ()),
                         "ExpReverseBitsLen": (8, 6, 10, (4, 5)), "Poseidon2WideDeg3": (9, 48, 49, ())}


def recursion_instrs_trace(chip: str, records_dev, n: int, height: int, montgomery: bool = False):
    """Preprocessed trace (height x width int32, canonical, on the GPU) of a recursion chip from n instruction
    records (RECURSION_INSTR_CHIPS; recursion.prep_records builds them) in a 32-bit GPU tensor."""
    code, w, width, _ = RECURSION_INSTR_CHIPS[chip]
    t = _trace(height, width)
    what = "zkm_recursion_instrs_to_trace"
    _lib.check(_bind().zkm_recursion_instrs_to_trace(code, _words(records_dev, n * w, what) if n else None, n,
                                                     1 if montgomery else 0, t.data_ptr(), height, _stream()), what)
    return t


def precompile_chip(code: int, pevs):
    """The precompile chip of a syscall code: (chip name, its zkm_tracegen.h records of the calls pevs, the
    trace builder fn(records_dev, n, height=None, byte_mult=None))."""
    from . import mips_ec as EC
    from . import mips_keccak as KS
    from . import mips_p2permute as P2P
    from . import mips_syscall as SY
    if code == SY.SHA_EXTEND:
        rows = sha_extend_records(pevs)
        return "ShaExtend", rows, sha_extend_trace
    elif code == SY.SHA_COMPRESS:
        rec = sha_compress_records(pevs)
        return "ShaCompress", rec, sha_compress_trace
    elif code == EC.UINT256_MUL:
        rec = uint256_mul_records(pevs)
        return "Uint256MulMod", rec, uint256_mul_trace
    elif code == EC.U256XU2048_MUL:
        rec = u256x2048_mul_records(pevs)
        return "U256XU2048Mul", rec, u256x2048_mul_trace
    elif any(code == EC.FP_OPS[f][0] for f in FP_OP_FIELDS):
        field = next(f for f in FP_OP_FIELDS if code == EC.FP_OPS[f][0])
        rec = fp_op_records(pevs)
        return EC.FP_NAME[field], rec, functools.partial(fp_op_trace, field)
    elif any(code in (EC.FP2_ADDSUB[f][0], EC.FP2_MUL[f]) for f in FP_OP_FIELDS):
        field = next(f for f in FP_OP_FIELDS if code in (EC.FP2_ADDSUB[f][0], EC.FP2_MUL[f]))
        mul = code == EC.FP2_MUL[field]
        rec = fp2_records(pevs)
        name = EC.FP2_MUL_NAME[field] if mul else EC.FP2_ADDSUB_NAME[field]
        return name, rec, functools.partial(fp2_trace, field, mul)
    elif any(code == EC.EC_ADD[c] for c in EC_CURVES):
        curve = next(c for c in EC_CURVES if code == EC.EC_ADD[c])
        rec = ec_add_records(pevs)
        return f"{curve}AddAssign", rec, functools.partial(ec_add_trace, curve)
    elif any(code == EC.EC_DOUBLE[c] for c in EC_CURVES):
        curve = next(c for c in EC_CURVES if code == EC.EC_DOUBLE[c])
        rec = ec_double_records(pevs)
        return f"{curve}DoubleAssign", rec, functools.partial(ec_double_trace, curve)
    elif any(code == EC.EC_DECOMPRESS[c] for c in EC.EC_DECOMPRESS):
        curve = next(c for c in EC.EC_DECOMPRESS if code == EC.EC_DECOMPRESS[c])
        rec = ec_decompress_records(pevs)
        return f"{curve}Decompress", rec, functools.partial(ec_decompress_trace, curve)
    elif code == SY.ED_ADD:
        rec = ed_add_records(pevs)
        return "EdAddAssign", rec, ed_add_trace
    elif code == SY.ED_DECOMPRESS:
        rec = ed_decompress_records(pevs)
        return "EdDecompress", rec, ed_decompress_trace
    elif code == KS.KECCAK_SPONGE:
        rec = keccak_blocks(pevs)
        return "KeccakSponge", rec, keccak_sponge_trace
    elif code == SY.SYS_LINUX:
        rec = sys_linux_records(pevs)
        return "SysLinux", rec, sys_linux_trace
    elif code == P2P.POSEIDON2_PERMUTE:
        rec = poseidon2_permute_records(pevs)
        return "Poseidon2Permute", rec, poseidon2_permute_trace
    else:
        raise ValueError(f"no device trace for precompile {code:#x}")


def precompile_shard_traces(code: int, events, byte_mult=None):
    """Device traces of a SHA, Poseidon2, 256-bit multiplication, base-field (FpOp) or Linux-syscall
    precompile shard (mips_core.precompile_shard's chips for SHA_EXTEND / SHA_COMPRESS / POSEIDON2_PERMUTE /
    UINT256_MUL / U256XU2048_MUL / the bn254 and bls12-381 FP, FP2 add/sub and FP2 mul ops / the Weierstrass
    additions, doublings and decompressions / the Ed25519 addition and decompression / the Keccak sponge / the Linux syscalls): the precompile chip, SyscallPrecompile (one row per call), MemoryLocal (the calls' local
    memory accesses) and the Global chip (the syscall receives and the memory messages), with their Byte
    lookups added into byte_mult.  events: the shard's (code, syscall tuple, event) list."""
    from . import mips_memory as MM
    from . import mips_syscall as SY
    pevs = [e for _, _, e in events]
    sev = np.asarray([s_ for _, s_, _ in events], np.int64).reshape(-1, 5)  # shard, clk, id, arg1, arg2
    out = {}
    name, rec, fn = precompile_chip(code, pevs)
    out[name] = fn(to_device(rec), len(rec), byte_mult=byte_mult)
    sc = np.zeros(len(sev), SYSCALL_EVENT)
    sc["shard"], sc["clk"], sc["syscall_id"], sc["arg1"], sc["arg2"] = (sev[:, j] for j in range(5))
    out["SyscallPrecompile"] = syscall_trace(to_device(sc), len(sc))
    ent = np.asarray([x for e in pevs for x in e["local"]], np.int64).reshape(-1, 7)
    ml = memory_local_events(ent)
    out["MemoryLocal"] = memory_local_trace(to_device(ml), len(ml))
    gmsg, grec = MM.memory_local_global_events(ent)
    smsg = SY.syscall_global_messages(sev)
    ge = global_events(np.concatenate([smsg, gmsg]), np.concatenate([np.ones(len(smsg), np.uint8), grec]),
                       np.concatenate([np.full(len(smsg), SY.KIND_SYSCALL), np.full(len(gmsg), MC.KIND_MEMORY)]))
    out["Global"], _ = global_trace(to_device(ge), len(ge), byte_mult=byte_mult)
    return out
