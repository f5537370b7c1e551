"""Device trace generation (include/zkm_tracegen.h): the reference's per-row trace ABI
(crates/core/machine/src/sys.rs:14-42, include/{cpu,add_sub,memory_local,memory_global,syscall}.hpp)
as whole-trace HIP kernels.

Modelled on the reference's own FFI tests, which fill a trace through the C++ event_to_row and
assert it equals the Rust generate_trace (cpu/trace.rs:279-314 `test_generate_cpu_trace_ffi_eq_rust`,
alu/add_sub/mod.rs:340-380, memory/local.rs:400-460): here the device traces must equal the host
trace builders of this repository (program_shard, mips_memory) bit for bit, the Byte and Program
multiplicities included, and a shard proven from device traces must produce the same proof bytes.

CPU tests: the record layouts equal the header's C structs (gcc offsetof), and a numpy restatement
of cpu.hpp's event_to_row over the converted records reproduces the host Cpu trace (so the records
carry everything the row needs)."""
import os
import subprocess

import numpy as np
import pytest

from zkmips_amd import mips_alu as A
from zkmips_amd import mips_core as MC
from zkmips_amd import mips_memory as MM
from zkmips_amd import mips_syscall as SY
from zkmips_amd import tracegen as TG

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

LAYOUTS = {
    "zkm_option_memory_record": (TG.RECORD, {"tag": "tag", "read": "read", "write": "write"}),
    "zkm_cpu_event_ffi": (TG.CPU_EVENT, {f: f for f in TG.CPU_EVENT.names if f not in ("hi_tag",)} | {"hi": "hi"}),
    "zkm_instruction_ffi": (TG.INSTRUCTION, {f: f for f in ("opcode", "op_a", "op_b", "op_c", "imm_b", "imm_c")}),
    "zkm_alu_event": (TG.ALU_EVENT, {f: f for f in TG.ALU_EVENT.names}),
    "zkm_memory_local_event": (TG.MEMORY_LOCAL_EVENT, {"addr": "addr", "initial": "initial_mem_access",
                                                      "final": "final_mem_access"}),
    "zkm_memory_init_final_event": (TG.MEMORY_INIT_FINAL_EVENT, {f: f for f in TG.MEMORY_INIT_FINAL_EVENT.names}),
    "zkm_syscall_event": (TG.SYSCALL_EVENT, {f: f for f in TG.SYSCALL_EVENT.names}),
    "zkm_global_lookup_event": (TG.GLOBAL_EVENT, {f: f for f in TG.GLOBAL_EVENT.names}),
    "zkm_branch_event": (TG.BRANCH_EVENT, {f: f for f in TG.BRANCH_EVENT.names}),
    "zkm_mem_instr_event": (TG.MEM_INSTR_EVENT, {f: f for f in TG.MEM_INSTR_EVENT.names}),
    "zkm_jump_event": (TG.JUMP_EVENT, {f: f for f in TG.JUMP_EVENT.names}),
    "zkm_movcond_event": (TG.MOVCOND_EVENT, {f: f for f in TG.MOVCOND_EVENT.names}),
    "zkm_comp_alu_event": (TG.COMP_ALU_EVENT, {f: f for f in TG.COMP_ALU_EVENT.names}),
    "zkm_misc_event": (TG.MISC_EVENT, {f: f for f in TG.MISC_EVENT.names}),
    "zkm_sha_extend_row": (TG.SHA_EXTEND_ROW, {"shard": "shard", "clk": "clk", "w_ptr": "w_ptr", "r15": "w_i_minus_15",
                                               "r2": "w_i_minus_2", "r16": "w_i_minus_16", "r7": "w_i_minus_7",
                                               "w": "w_i"}),
    "zkm_sha_compress_event": (TG.SHA_COMPRESS_EVENT, {"shard": "shard", "clk": "clk", "w_ptr": "w_ptr", "h_ptr": "h_ptr",
                                                       "h_read": "h_read_records", "w_read": "w_i_read_records",
                                                       "h_write": "h_write_records"}),
}


def test_record_layouts_match_header(tmp_path):
    """numpy record dtypes == the C structs of include/zkm_tracegen.h (sizes and field offsets)."""
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "zkm_tracegen.h"', "int main(void) {"]
    for st, (_, fields) in LAYOUTS.items():
        lines.append(f'printf("{st} size %zu\\n", sizeof({st}));')
        for np_name, c_name in fields.items():
            # OptionU32 `hi` is {tag, value}: the record keeps the tag at the struct's offset
            expr = f"offsetof({st}, {c_name})" + (" + 4" if (st, c_name) == ("zkm_cpu_event_ffi", "hi") else "")
            lines.append(f'printf("{st} {np_name} %zu\\n", (size_t)({expr}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    got = {}
    for ln in out:
        if ln:
            st, f, v = ln.split()
            got[(st, f)] = int(v)
    for st, (dt, fields) in LAYOUTS.items():
        assert got[(st, "size")] == dt.itemsize, st
        for np_name in fields:
            assert got[(st, np_name)] == dt.fields[np_name][1], (st, np_name)
    assert TG.CPU_EVENT.fields["hi_tag"][1] == 172


# ---------------------------------------------------------------- numpy restatement of cpu.hpp (test-only)
def _bytes(x):
    return A._bytes(np.asarray(x, np.uint64).astype(np.uint32))


def _access(rec):
    """populate_read / populate_read_write (include/memory.hpp) over an OptionMemoryRecordEnum column."""
    tag = rec["tag"].astype(np.int64)
    rd, wr = rec["read"].astype(np.int64), rec["write"].astype(np.int64)
    is_w = tag == TG.REC_WRITE
    on = tag != TG.REC_NONE
    value = np.where(is_w, wr[:, 0], rd[:, 0])
    shard, ts = np.where(is_w, wr[:, 1], rd[:, 1]), np.where(is_w, wr[:, 2], rd[:, 2])
    prev_value = np.where(is_w, wr[:, 3], rd[:, 0])
    ps, pt = np.where(is_w, wr[:, 4], rd[:, 3]), np.where(is_w, wr[:, 5], rd[:, 4])
    cmp_ = ps == shard
    d = (np.where(cmp_, ts, shard) - np.where(cmp_, pt, ps) - 1) & 0xFFFFFFFF
    return on, value, prev_value, ps, pt, cmp_, d & 0xFFFF, (d >> 16) & 0xFF


def cpu_rows(ev, prog_ffi, shard, height):
    n = len(ev)
    t = np.zeros((height, MC.CPU_WIDTH), np.uint32)
    t[n:, MC.C_IMMB] = t[n:, MC.C_IMMC] = t[n:, MC.C_RW_A] = 1
    ins = prog_ffi[(ev["pc"].astype(np.int64) - MC.PC_BASE) >> 2]
    op = ins["opcode"].astype(np.int64)
    clk = ev["clk"].astype(np.int64)
    t[:n, MC.C_SHARD] = shard
    t[:n, MC.C_CLK16], t[:n, MC.C_CLK8] = clk & 0xFFFF, (clk >> 16) & 0xFF
    t[:n, MC.C_PC], t[:n, MC.C_NPC], t[:n, MC.C_NNPC] = ev["pc"], ev["next_pc"], ev["next_next_pc"]
    t[:n, MC.C_OPCODE], t[:n, MC.C_OPA] = op, ins["op_a"]
    t[:n, MC.C_OPB:MC.C_OPB + 4], t[:n, MC.C_OPC:MC.C_OPC + 4] = _bytes(ins["op_b"]), _bytes(ins["op_c"])
    t[:n, MC.C_OPA0] = ins["op_a"] == 0
    t[:n, MC.C_IMMB], t[:n, MC.C_IMMC] = ins["imm_b"], ins["imm_c"]
    branch = np.isin(op, MC.BRANCH_OPS)
    t[:n, MC.C_A_IMM] = branch | np.isin(op, (MC.OP_SB, MC.OP_SH, MC.OP_SW, MC.OP_SWL, MC.OP_SWR))
    t[:n, MC.C_RW_A] = np.isin(op, (30, MC.OP_INS, MC.OP_MEQ, MC.OP_MNE) + MC.MADDSUB_OPS + MC.MEM_OPS)
    check = np.isin(op, MC.MULT_DIV + (30,) + MC.MADDSUB_OPS + MC.MEM_OPS)
    t[:n, MC.C_CHECK_MEM] = check
    t[:n, MC.C_A_VAL:MC.C_A_VAL + 4] = _bytes(ev["a"])
    hi_some = ev["hi_tag"] == 0
    t[:n, MC.C_HI_PREV_A:MC.C_HI_PREV_A + 4] = np.where(hi_some[:, None], _bytes(ev["hi"]), 0)
    t[:n, MC.C_SHARD_SEND] = np.where(check, shard, 0)
    t[:n, MC.C_CLK_SEND] = np.where(check, clk, 0)
    for base, val, rec in ((MC.C_A_ACC + 4, "a", "a_record"), (MC.C_B_ACC, "b", "b_record"),
                           (MC.C_C_ACC, "c", "c_record")):
        on, value, prev_value, ps, pt, cmp_, d16, d8 = _access(ev[rec])
        t[:n, base:base + 4] = _bytes(np.where(on, value, ev[val]))
        t[:n, base + MC.ACC_PREV_SHARD] = np.where(on, ps, 0)
        t[:n, base + MC.ACC_PREV_CLK] = np.where(on, pt, 0)
        t[:n, base + MC.ACC_COMPARE] = on & cmp_
        t[:n, base + MC.ACC_D16] = np.where(on, d16, 0)
        t[:n, base + MC.ACC_D8] = np.where(on, d8, 0)
        if rec == "a_record":
            t[:n, MC.C_A_ACC:MC.C_A_ACC + 4] = np.where(on[:, None], _bytes(prev_value), 0)
    sys_ = op == 30
    pa = t[:n, MC.C_A_ACC:MC.C_A_ACC + 4].astype(np.int64)
    halt = sys_ & (((pa[:, 0] == 0) & (pa[:, 1] == 0)) | ((pa[:, 0] == 0x96) & (pa[:, 1] == 0x10)))
    t[:n, MC.C_HALT] = halt
    t[:n, MC.C_EXTRA] = np.where(sys_, pa[:, 3], 0)
    t[:n, MC.C_SEQ] = ~(halt | branch | np.isin(op, MC.JUMP_OPS))
    t[:n, MC.C_REAL] = 1
    return t


def expected_byte_mult(cpu, shard, add_sub=None, glob=None):
    """The Byte lookups program_shard makes for the Cpu rows (mips_core.py program_shard),
    alu_traces for AddSub and global_trace for Global, recomputed from the traces' columns."""
    mult = np.zeros((A.BYTE_ROWS, A.BYTE_MULT_WIDTH), np.uint64)
    look = A.byte_lookup_into(mult)
    if glob is not None:
        m0 = glob[glob[:, MM.G_REAL] == 1, MM.G_MSG].astype(np.int64)
        look(A.B_U16RANGE, m0 >> 8, m0 & 0xFF)
    t = cpu[cpu[:, MC.C_REAL] == 1].astype(np.int64)
    n = len(t)
    look(A.B_U16RANGE, np.full(n, shard >> 8), np.full(n, shard & 0xFF))
    look(A.B_U16RANGE, t[:, MC.C_CLK16] >> 8, t[:, MC.C_CLK16] & 0xFF)
    look(A.B_U8RANGE, np.zeros(n, np.int64), t[:, MC.C_CLK8])
    for base, sel in ((MC.C_C_ACC, t[:, MC.C_IMMC] == 0), (MC.C_B_ACC, t[:, MC.C_IMMB] == 0),
                      (MC.C_A_ACC + 4, np.ones(n, bool))):
        d16, d8 = t[sel, base + MC.ACC_D16], t[sel, base + MC.ACC_D8]
        look(A.B_U16RANGE, d16 >> 8, d16 & 0xFF)
        look(A.B_U8RANGE, np.zeros(len(d8), np.int64), d8)
    wb = t[:, MC.C_A_ACC + 4:MC.C_A_ACC + 8]
    look(A.B_U8RANGE, wb[:, 0], wb[:, 1])
    look(A.B_U8RANGE, wb[:, 2], wb[:, 3])
    if add_sub is not None:
        s = add_sub[(add_sub[:, A.AS_ADD] + add_sub[:, A.AS_SUB]) == 1].astype(np.int64)
        for b in (A.AS_OP1, A.AS_OP2, A.AS_VAL):
            look(A.B_U8RANGE, s[:, b], s[:, b + 1])
            look(A.B_U8RANGE, s[:, b + 2], s[:, b + 3])
    return mult


def _sys_linux_program():
    from tests.test_syscall import _sys_linux_program as f
    return f()


PROGRAMS = {
    "loop": lambda: MC.loop_program(24, 40, seed=3),
    "random": lambda: MC.random_program(600, seed=4),
    "sha_syscalls": lambda: MC.sha_program(3, seed=2),
    "sys_linux": _sys_linux_program,
}


def _capture(name):
    prog = PROGRAMS[name]()
    cap = {}
    m, prep, tr, pv = MC.program_shard(prog, seed=7, shard=3, capture=cap)
    return cap, tr, pv, m, prep


@pytest.mark.parametrize("name", sorted(PROGRAMS))
def test_cpu_records_reproduce_host_trace(name):
    """cpu.hpp's event_to_row (numpy restatement) over the converted CpuEventFfi records equals the
    host Cpu trace, and the restated lookups account for the shard's byte multiplicities."""
    cap, tr, _, _, _ = _capture(name)
    ev = TG.cpu_events(cap["steps"], cap["shard"])
    got = cpu_rows(ev, TG.program_ffi(cap["prog"]), cap["shard"], len(tr["Cpu"]))
    assert np.array_equal(got, tr["Cpu"])
    mult = expected_byte_mult(tr["Cpu"], cap["shard"], tr.get("AddSub"))
    assert (mult <= tr["Byte"]).all()  # a part of the shard's lookups


def alu_chip_byte_mult(cap):
    """The Byte lookups of the shard's Bitwise, Lt, ShiftLeft, ShiftRight, Branch and MemoryInstrs rows (the
    host builders over the same events the device gets; CloClz's own lookups excluded)."""
    mult = np.zeros((A.BYTE_ROWS, A.BYTE_MULT_WIDTH), np.uint64)
    ev = {"add": tuple(np.zeros(0, np.uint32) for _ in range(6))}
    for kind in list(TG.ALU_CHIPS) + ["clz"]:  # ShiftRight's CLZ dependencies come from the "clz" events
        r = TG.alu_events(*MC._ev_arrays(cap["alu"][kind])[:5]) if len(cap["alu"].get(kind, [])) else \
            np.zeros(0, TG.ALU_EVENT)
        ev[kind] = (r["opcode"].astype(np.uint32), r["a"], r["b"], r["c"], r["pc"], r["next_pc"])
    A.alu_traces(ev, mult)
    look = A.byte_lookup_into(mult)  # Branch and MemoryInstrs (host builders)
    if len(cap.get("branches", [])):
        MC._branch_trace(cap["branches"], look)
    if len(cap.get("mevs", [])):
        MC._mem_instr_trace(cap["mevs"], cap["shard"], look)
    if len(cap.get("muls", [])):
        MC._mul_trace(cap["muls"], cap["shard"], look)
    if len(cap.get("divs", [])):
        MC._divrem_trace(cap["divs"], cap["shard"], look)
    if len(cap.get("misc", [])):
        MC._misc_trace(cap["misc"], cap["shard"], look)
    return mult


def test_records_reproduce_executor_tuples():
    """Branch / MemInstr records round-trip the executor's tuples (decision and address recomputable)."""
    cap, tr, _, _, _ = _capture("loop")
    br = TG.branch_records(cap["branches"])
    assert len(br) == len(cap["branches"]) and len(br)
    taken = [MC._taken(int(o), int(a), int(b)) for o, a, b in zip(br["opcode"], br["a"], br["b"])]
    assert taken == [bool(t[7]) for t in cap["branches"]]
    mi = TG.mem_instr_records(cap["mevs"], cap["shard"])
    assert len(mi) == len(cap["mevs"]) and len(mi)
    load = np.isin(mi["opcode"], MC.LOAD_OPS)
    assert (mi["mem_access"]["tag"][load] == TG.REC_READ).all() and (mi["mem_access"]["tag"][~load] == TG.REC_WRITE).all()


@pytest.mark.parametrize("name", sorted(PROGRAMS))
def test_native_record_conversion_is_the_numpy_one(name):
    """libzkm_pyconv.so (csrc/host/pyconv.cpp) writes the same CpuEventFfi bytes as the numpy conversion, and
    its generic flattener the same rows as numpy's; malformed rows raise instead of being read."""
    cap, _, _, _, _ = _capture(name)
    a = TG.cpu_events(cap["steps"], cap["shard"])
    b = TG.cpu_events_numpy(cap["steps"], cap["shard"])
    assert len(a) == len(cap["steps"]) and a.tobytes() == b.tobytes()
    for key, w in (("branches", 8), ("mevs", 13), ("jumps", 7), ("movs", 7), ("muls", 11), ("divs", 9),
                   ("misc", 12)):
        lst = cap.get(key, [])
        if len(lst):
            assert np.array_equal(TG._rows(lst, w), np.asarray(lst, np.int64).reshape(-1, w)), key
    assert np.array_equal(TG._rows(cap["entries"], 7), np.asarray(cap["entries"], np.int64).reshape(-1, 7))
    assert np.array_equal(TG._rows([(1, (2, 3), None), [4, [5, 6], (7, 8)]], 5, none_w=2),
                          [[1, 2, 3, 0, 0], [4, 5, 6, 7, 8]])
    assert TG._rows([], 4).shape == (0, 4)
    with pytest.raises(ValueError):
        TG._rows([(1, 2), (3,)], 2)
    with pytest.raises(TypeError):
        TG._rows([(1, "x")], 2)
    with pytest.raises(OverflowError):
        TG._rows([(1, 1 << 70)], 2)
    with pytest.raises(ValueError):
        TG.cpu_events([(1, 2, 3)], 1)


def test_alu_records_carry_the_clz_dependencies():
    """ShiftRight's records = the CPU's SRL/SRA/ROR events then the CLZ/CLO dependencies (as its host trace)."""
    cap, tr, _, _, _ = _capture("random")
    rec = TG.alu_records(cap["alu"], "sr")
    assert len(rec) == int(tr["ShiftRight"][:, A.SR_REAL].sum())
    assert np.array_equal(rec["pc"], tr["ShiftRight"][:len(rec), A.SR_PC])


# ---------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(PROGRAMS))
def test_device_shard_traces_match_host(name):
    import torch
    cap, tr, _, _, _ = _capture(name)
    bm = torch.zeros((A.BYTE_ROWS, A.BYTE_MULT_WIDTH), dtype=torch.int32, device="cuda")
    dev = TG.shard_traces(cap, byte_mult=bm)
    torch.cuda.synchronize()
    for chip, t in dev.items():
        host = tr[chip]
        assert np.array_equal(t.cpu().numpy().view(np.uint32), host), chip
    assert set(dev) >= {"Cpu", "Program", "MemoryLocal", "Global"}
    want = expected_byte_mult(tr["Cpu"], cap["shard"], tr.get("AddSub"), tr["Global"]) + alu_chip_byte_mult(cap)
    assert np.array_equal(bm.cpu().numpy().astype(np.uint64), want)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 127, 129, 5000])
def test_device_alu_chips_match_host(n):
    """Bitwise, Lt, ShiftLeft and ShiftRight from AluEvents (every opcode, every shift amount and
    comparison-byte position; empty and ragged inputs) == the host builders, Byte lookups included."""
    import torch
    ev = A.alu_events(0, n, seed=n + 1, n_lt=n, n_sll=n, n_sr=n)
    for kind, (_, chip, width) in TG.ALU_CHIPS.items():
        op, a, b, c, pc = ev[kind]
        mult = np.zeros((A.BYTE_ROWS, A.BYTE_MULT_WIDTH), np.uint64)
        host = A.alu_traces({k: ev[k] if k == kind else tuple(np.zeros(0, np.uint32) for _ in range(5))
                             for k in ("add", "bit", "lt", "sll", "sr")}, mult).get(chip)
        h = max(16, 1 << max(0, (n - 1).bit_length()))
        bm = torch.zeros((A.BYTE_ROWS, A.BYTE_MULT_WIDTH), dtype=torch.int32, device="cuda")
        rec = TG.alu_events(op, a, b, c, pc)
        dev = TG.alu_trace(kind, TG.to_device(rec), n, height=h, byte_mult=bm).cpu().numpy().view(np.uint32)
        if n:
            assert np.array_equal(dev, host), chip
        else:
            assert dev.shape == (16, width)
        assert np.array_equal(bm.cpu().numpy().astype(np.uint64), mult), chip


@pytest.mark.gpu
@pytest.mark.parametrize("n,prev_addr,initialize", [(0, 0, True), (1, 0, True), (37, 0, False), (300, 0x1234, True),
                                                   (1000, 0xFFFF0, False), (16, 8, False)])
def test_device_memory_global_matches_host(n, prev_addr, initialize):
    import torch
    rng = np.random.default_rng(n + prev_addr)
    addr = np.sort(rng.choice(np.arange(prev_addr + 1, prev_addr + 1 + 50 * max(n, 1), dtype=np.int64), n,
                              replace=False))
    if n > 2:
        addr[-1] = 0x7EFFFFFF - 4  # the top of the KoalaBear range (and_most_sig_byte columns)
        addr = np.sort(addr)
    ev = np.stack([addr, rng.integers(0, 1 << 32, n), rng.integers(0, 5, n), rng.integers(0, 1 << 24, n)], axis=1)
    host, _, _ = MM.memory_global_trace(ev, initialize, prev_addr)
    rec = TG.memory_init_final_events(ev)
    dev = TG.memory_global_trace(TG.to_device(rec), n, initialize, prev_addr, height=len(host))
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy().view(np.uint32), host)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 100, 2048, 2049, 5000])
def test_device_global_matches_host(n):
    """Global: septic-curve lift + running sum (a multi-level scan past 2048 points) == the host's
    lift and sequential fold, trace, final digest and U16 lookups."""
    import torch
    rng = np.random.default_rng(11 + n)
    msg = rng.integers(0, 256, (n, 7)).astype(np.uint32)
    msg[:, 0] = rng.integers(0, 4, n)       # shard
    msg[:, 1] = rng.integers(0, 1 << 24, n)  # clk
    msg[:, 2] = rng.integers(0, 1 << 30, n)  # address
    rec = rng.integers(0, 2, n).astype(np.uint8)
    kinds = rng.integers(1, 3, n).astype(np.uint32)
    mult = np.zeros((A.BYTE_ROWS, A.BYTE_MULT_WIDTH), np.uint64)
    host, fin = MM.global_trace(msg, rec, kinds, A.byte_lookup_into(mult))
    bm = torch.zeros((A.BYTE_ROWS, A.BYTE_MULT_WIDTH), dtype=torch.int32, device="cuda")
    dev, dfin = TG.global_trace(TG.to_device(TG.global_events(msg, rec, kinds)), n, height=len(host), byte_mult=bm)
    assert np.array_equal(dev.cpu().numpy().view(np.uint32), host)
    assert np.array_equal(dfin, fin)
    assert np.array_equal(bm.cpu().numpy().astype(np.uint64), mult)


@pytest.mark.gpu
def test_device_traces_empty_and_ragged():
    """n = 0 gives padding rows only; n one short of / one past a block boundary fills exactly n rows."""
    import torch
    prog = TG.program_ffi(MC.random_program(50, seed=1))
    for n in (0, 127, 129):
        cap = {}
        if n:
            MC.program_shard(MC.random_program(n, seed=5), seed=5, capture=cap)
            steps = cap["steps"][:n]
            ev, p = TG.cpu_events(steps, 1), TG.program_ffi(cap["prog"])
        else:
            ev, p = TG.cpu_events([], 1), prog
        h = max(16, 1 << max(0, (len(ev) - 1).bit_length()))
        t = TG.cpu_trace(TG.to_device(ev), len(ev), 1, TG.to_device(p), len(p), height=h).cpu().numpy()
        want = cpu_rows(ev, p, 1, h)
        assert np.array_equal(t.view(np.uint32), want)
    e = TG.add_sub_trace(TG.to_device(np.zeros(0, TG.ALU_EVENT)), 0).cpu().numpy()
    assert e.shape == (16, TG.ADD_SUB_WIDTH) and not e.any()
    torch.cuda.synchronize()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["sha_syscalls", "loop", "random"])
def test_device_traces_prove_identically(name):
    """A shard proven from device-generated traces (ZKM_MEM_DEVICE) gives the host traces' proof bytes."""
    import torch
    from zkmips_amd._lib import Device
    from zkmips_amd.prover import HipProver
    cap, tr, pv, m, prep = _capture(name)
    bm = torch.zeros((A.BYTE_ROWS, A.BYTE_MULT_WIDTH), dtype=torch.int32, device="cuda")
    dev = TG.shard_traces(cap, byte_mult=bm)
    rest = tr["Byte"].astype(np.int64) - (expected_byte_mult(tr["Cpu"], cap["shard"], tr.get("AddSub"), tr["Global"])
                                          + alu_chip_byte_mult(cap)).astype(np.int64)
    bm += torch.from_numpy(rest.astype(np.int32)).cuda()  # the other chips' lookups, from the host builders
    traces = {k: v for k, v in tr.items() if k not in dev}
    if name in ("loop", "random"):  # every main trace and every Byte lookup of these shards came from the device
        assert not rest.any() and set(traces) == {"Byte"}, sorted(traces)
    traces.update(dev)
    traces["Byte"] = bm
    prover = HipProver(Device(0), m, prep, num_queries=16)
    assert prover.prove_shard(traces, pv) == prover.prove_shard(tr, pv)


def test_repacked_records_are_refused():
    """np.resize repacks a padded record dtype (280 -> 262 bytes): such arrays must not reach the ABI,
    which takes bare pointers and would read past the buffer."""
    ev = np.zeros(3, TG.CPU_EVENT)
    assert ev[np.arange(10) % 3].dtype == TG.CPU_EVENT
    with pytest.raises(ValueError):
        TG.to_device(np.resize(ev, 10))


def _sha_extend_events(calls):
    prog = MC.sha_program(calls, seed=4, compress=False)
    state = MC.fresh_state()
    regs = MC.initial_registers(1)
    MC.program_shard(prog, 1, 1, 1 << 14, state=state, regs=regs)
    return [e for code, _, e in state["precompile"] if code == SY.SHA_EXTEND]


@pytest.mark.gpu
@pytest.mark.parametrize("calls", [1, 3, 7])
def test_device_sha_extend_matches_host(calls):
    """ShaExtend rows from the executor's SHA_EXTEND events == the host builder (flags of the padding rows,
    access columns, rotate / shift carries, XORs, Add4), Byte lookups included."""
    import torch
    evs = _sha_extend_events(calls)
    assert len(evs) == calls
    mult = np.zeros((A.BYTE_ROWS, A.BYTE_MULT_WIDTH), np.uint64)
    host = SY.sha_extend_trace(evs, A.byte_lookup_into(mult))
    rows = TG.sha_extend_records(evs)
    bm = torch.zeros((A.BYTE_ROWS, A.BYTE_MULT_WIDTH), dtype=torch.int32, device="cuda")
    dev = TG.sha_extend_trace(TG.to_device(rows), len(rows), height=len(host), byte_mult=bm)
    assert np.array_equal(dev.cpu().numpy().view(np.uint32), host)
    assert np.array_equal(bm.cpu().numpy().astype(np.uint64), mult)


@pytest.mark.gpu
@pytest.mark.parametrize("calls", [1, 2, 5])
def test_device_sha_compress_matches_host(calls):
    """ShaCompress rows (round state expanded on the device) == the host builder, Byte lookups included."""
    import torch
    prog = MC.sha_program(calls, seed=6)
    state = MC.fresh_state()
    MC.program_shard(prog, 1, 1, 1 << 14, state=state, regs=MC.initial_registers(1))
    evs = [e for code, _, e in state["precompile"] if code == SY.SHA_COMPRESS]
    assert len(evs) == calls
    mult = np.zeros((A.BYTE_ROWS, A.BYTE_MULT_WIDTH), np.uint64)
    host = SY.sha_compress_trace(evs, A.byte_lookup_into(mult))
    rec = TG.sha_compress_records(evs)
    bm = torch.zeros((A.BYTE_ROWS, A.BYTE_MULT_WIDTH), dtype=torch.int32, device="cuda")
    dev = TG.sha_compress_trace(TG.to_device(rec), len(rec), height=len(host), byte_mult=bm)
    assert np.array_equal(dev.cpu().numpy().view(np.uint32), host)
    assert np.array_equal(bm.cpu().numpy().astype(np.uint64), mult)


@pytest.mark.gpu
def test_sha_precompile_shards_from_device_traces_prove_identically():
    """The SHA_EXTEND and SHA_COMPRESS precompile shards of a sha2 guest, every main trace and Byte lookup
    generated on the device (precompile chip, SyscallPrecompile, MemoryLocal, Global), prove to the host
    traces' bytes."""
    import torch
    from zkmips_amd._lib import Device
    from zkmips_amd.prover import HipProver
    prog = MC.sha_program(3, seed=2)
    run = MC.program_shards(prog, seed=2, shard_size=1 << 12, precompile_events_per_shard=2)
    state = MC.fresh_state()
    regs = MC.initial_registers(2)
    while MC.PC_BASE <= state["pc"] < MC.PC_BASE + 4 * len(prog) and state["exit_code"] is None:
        MC.program_shard(prog, 2, 1, 1 << 12, state=state, regs=regs)
    by_code = {}
    for ev in state["precompile"]:
        by_code.setdefault(ev[0], []).append(ev)
    m, prep, _, _ = run[0]
    prep = {k: v for k, v in prep.items() if v is not None}
    prover = HipProver(Device(0), m, prep, num_queries=16)
    checked = 0
    for code in (SY.SHA_EXTEND, SY.SHA_COMPRESS):
        chip = "ShaExtend" if code == SY.SHA_EXTEND else "ShaCompress"
        shards = [r for r in run if chip in r[2]]
        evs = by_code[code]
        for k, (_, _, tr, pv) in enumerate(shards):
            bm = torch.zeros((A.BYTE_ROWS, A.BYTE_MULT_WIDTH), dtype=torch.int32, device="cuda")
            dev = TG.precompile_shard_traces(code, evs[2 * k:2 * k + 2], byte_mult=bm)
            torch.cuda.synchronize()
            for name, t in dev.items():
                assert np.array_equal(t.cpu().numpy().view(np.uint32), tr[name]), name
            assert np.array_equal(bm.cpu().numpy().view(np.uint32), tr["Byte"])
            traces = {k_: v for k_, v in tr.items() if k_ not in dev}
            assert set(traces) <= {"Byte", "Program"}, sorted(traces)
            traces.update(dev)
            traces["Byte"] = bm
            assert prover.prove_shard(traces, pv) == prover.prove_shard(tr, pv)
            checked += 1
    assert checked >= 2


def _p2permute_events(n: int = 37, seed: int = 5):
    """POSEIDON2_PERMUTE calls through the executor's syscall memory (mips_p2permute.exec_poseidon2_permute):
    states at five reused addresses over several shards, so the accesses' previous records are of the same
    shard (compare) and of earlier ones."""
    from zkmips_amd import mips_p2permute as P2
    mem, mem_init, mem_last = {}, {}, {}
    evs = []
    for k in range(n):
        shard, clk, ptr = 1 + k // 10, 100 + 7 * k, 0x1000 + 64 * (k % 5)
        pm = SY.PrecompileMemory(mem, mem_init, mem_last, {}, [], shard, lambda a: (a * 2654435761 + seed) % MC.P)
        evs.append((P2.POSEIDON2_PERMUTE, (shard, clk, SY.syscall_id(P2.POSEIDON2_PERMUTE), ptr, 0),
                    P2.exec_poseidon2_permute(pm, shard, clk, ptr, 0)))
    return evs


def test_poseidon2_permute_records_layout():
    """zkm_poseidon2_permute_event records: shard, clk, ptr, then each state word's MemoryWriteRecord
    (value = the permuted word, prev_value = the word before)."""
    evs = _p2permute_events(3)
    rec = TG.poseidon2_permute_records([e for _, _, e in evs])
    raw = rec.view(np.uint32).reshape(3, 99)
    for k, (_, _, e) in enumerate(evs):
        assert list(raw[k, :3]) == [e["shard"], e["clk"], e["ptr"]]
        st = raw[k, 3:].reshape(16, 6)
        assert list(st[:, 0]) == e["post"] and list(st[:, 3]) == e["pre"]
        assert (st[:, 1] == e["shard"]).all() and (st[:, 2] == e["clk"]).all()


@pytest.mark.gpu
def test_poseidon2_permute_shard_from_device_traces():
    """A POSEIDON2_PERMUTE precompile shard with every main trace and Byte lookup built on the device
    (Poseidon2Permute, SyscallPrecompile, MemoryLocal, Global) equals the host builders' traces and
    multiplicities and proves to the same bytes."""
    import torch
    from zkmips_amd import mips_p2permute as P2
    from zkmips_amd._lib import Device
    from zkmips_amd.prover import HipProver
    evs = _p2permute_events()
    m, prep, tr, pv = MC.precompile_shard(P2.POSEIDON2_PERMUTE, evs, shard=5)
    bm = torch.zeros((A.BYTE_ROWS, A.BYTE_MULT_WIDTH), dtype=torch.int32, device="cuda")
    dev = TG.precompile_shard_traces(P2.POSEIDON2_PERMUTE, evs, byte_mult=bm)
    torch.cuda.synchronize()
    assert "Poseidon2Permute" in dev
    for name, t in dev.items():
        assert np.array_equal(t.cpu().numpy().view(np.uint32), tr[name]), name
    assert np.array_equal(bm.cpu().numpy().view(np.uint32), tr["Byte"])
    traces = {k: v for k, v in tr.items() if k not in dev}
    assert set(traces) <= {"Byte", "Program"}, sorted(traces)
    traces.update(dev)
    traces["Byte"] = bm
    prover = HipProver(Device(0), m, _core_prep(), num_queries=16)
    assert prover.prove_shard(traces, pv) == prover.prove_shard(tr, pv)


def _core_prep():
    """The core machine's preprocessed traces of a small program (the Program chip's rows), the proving key
    the precompile shards above are proven under."""
    _, prep, _, _ = MC.program_shards(MC.sha_program(1, seed=1), seed=1, shard_size=1 << 12)[0]
    return {k: v for k, v in prep.items() if v is not None}


def _uint256_events(seed: int = 11):
    """UINT256_MUL calls through the executor (mips_ec.exec_uint256_mul): full-width, one-limb and
    two-limb moduli, the zero modulus (2^256), operands below the modulus, over two shards."""
    from zkmips_amd import emulated_field as EF
    from zkmips_amd import mips_ec as EC
    rng = np.random.default_rng(seed)
    words = {}
    mem, mem_init, mem_last = {}, {}, {}
    evs = []
    mods = [int.from_bytes(rng.bytes(32), "little") | (1 << 255) | 1 for _ in range(6)]
    mods += [0, 0, 0xFFFFFFFB, 7, (1 << 40) + 3, int.from_bytes(rng.bytes(20), "little") | 1, 1 << 255]
    for k, m in enumerate(mods * 2):
        bound = m if m else 1 << 256
        x, y = (int.from_bytes(rng.bytes(32), "little") % bound for _ in range(2))
        xp, yp = 0x4000 + 0x100 * k, 0x8000 + 0x100 * k
        for i, w in enumerate(EF.int_to_words(x, 8)):
            words[xp + 4 * i] = w
        for i, w in enumerate(EF.int_to_words(y, 8) + EF.int_to_words(m, 8)):
            words[yp + 4 * i] = w
        shard, clk = 3 + k // 10, 50 + 8 * k
        pm = SY.PrecompileMemory(mem, mem_init, mem_last, {}, [], shard, lambda a: words.get(a, 0))
        evs.append((EC.UINT256_MUL, (shard, clk, SY.syscall_id(EC.UINT256_MUL), xp, yp),
                    EC.exec_uint256_mul(pm, shard, clk, xp, yp)))
    return evs


def test_uint256_mul_records_layout():
    """zkm_uint256_mul_event records: y and the modulus read at clk, x written at clk + 1."""
    evs = _uint256_events()
    rec = TG.uint256_mul_records([e for _, _, e in evs])
    assert rec.dtype.itemsize == 528
    for r, (_, _, e) in zip(rec, evs):
        assert list(r["y"][:, 0]) == [v[0] for v in e["y"]] and list(r["modulus"][:, 0]) == [v[0] for v in e["m"]]
        assert list(r["x"][:, 3]) == e["x"] and (r["x"][:, 2] == e["clk"] + 1).all()


@pytest.mark.gpu
def test_uint256_mul_shard_from_device_traces():
    """A UINT256_MUL precompile shard with every main trace and Byte lookup built on the device (the
    product divided by the modulus on the device, the vanishing polynomial's witness) equals the host
    builders' traces and multiplicities and proves to the same bytes."""
    import torch
    from zkmips_amd import mips_ec as EC
    from zkmips_amd._lib import Device
    from zkmips_amd.prover import HipProver
    evs = _uint256_events()
    m, prep, tr, pv = MC.precompile_shard(EC.UINT256_MUL, evs, shard=5)
    bm = torch.zeros((A.BYTE_ROWS, A.BYTE_MULT_WIDTH), dtype=torch.int32, device="cuda")
    dev = TG.precompile_shard_traces(EC.UINT256_MUL, evs, byte_mult=bm)
    torch.cuda.synchronize()
    assert "Uint256MulMod" in dev
    for name, t in dev.items():
        got = t.cpu().numpy().view(np.uint32)
        bad = np.argwhere(got != tr[name])
        assert not len(bad), (name, bad[:8].tolist())
    assert np.array_equal(bm.cpu().numpy().view(np.uint32), tr["Byte"])
    traces = {k: v for k, v in tr.items() if k not in dev}
    traces.update(dev)
    traces["Byte"] = bm
    prover = HipProver(Device(0), m, _core_prep(), num_queries=16)
    assert prover.prove_shard(traces, pv) == prover.prove_shard(tr, pv)


def _u256x2048_events(seed: int = 13):
    """U256XU2048_MUL calls through the executor (mips_ec.exec_u256x2048_mul): random a and b, all-ones
    operands (every carry at its largest), zeros, over two shards."""
    from zkmips_amd import emulated_field as EF
    from zkmips_amd import mips_ec as EC
    rng = np.random.default_rng(seed)
    words = {}
    regs = [0] * MC.NUM_REGS
    last = [(1, r) for r in range(MC.NUM_REGS)]
    reg_start, reg_done = [(last[r], regs[r]) for r in range(MC.NUM_REGS)], []
    mem, mem_init, mem_last = {}, {}, {}
    ops = [(int.from_bytes(rng.bytes(32), "little"), int.from_bytes(rng.bytes(256), "little")) for _ in range(7)]
    ops += [((1 << 256) - 1, (1 << 2048) - 1), (0, 0), (1, (1 << 2048) - 1)]
    evs = []
    for k, (a, b) in enumerate(ops * 2):
        ap, bp, lo, hi = 0x10000 + 0x1000 * k, 0x10100 + 0x1000 * k, 0x10200 + 0x1000 * k, 0x10400 + 0x1000 * k
        for i, w in enumerate(EF.int_to_words(a, 8)):
            words[ap + 4 * i] = w
        for i, w in enumerate(EF.int_to_words(b, 64)):
            words[bp + 4 * i] = w
        regs[SY.REG_A2], regs[SY.REG_A3] = lo, hi
        shard, clk = 3 + k // 10, 60 + 8 * k
        pm = SY.PrecompileMemory(mem, mem_init, mem_last, {}, [], shard, lambda x: words.get(x, 0), regs, last,
                                 reg_start, reg_done)
        evs.append((EC.U256XU2048_MUL, (shard, clk, SY.syscall_id(EC.U256XU2048_MUL), ap, bp),
                    EC.exec_u256x2048_mul(pm, shard, clk, ap, bp)))
    return evs


def test_u256x2048_mul_records_layout():
    """zkm_u256x2048_mul_event records: registers, a, b read at clk, lo and hi written at clk + 1."""
    evs = _u256x2048_events()
    rec = TG.u256x2048_mul_records([e for _, _, e in evs])
    assert rec.dtype.itemsize == 3232
    for r, (_, _, e) in zip(rec, evs):
        assert r["lo_ptr_reg"][0] == e["lo_ptr"] and r["hi_ptr_reg"][0] == e["hi_ptr"]
        assert list(r["b"][:, 0]) == [v[0] for v in e["b"]] and list(r["hi"][:, 0]) == [v[1] for v in e["hi"]]
        assert (r["lo"][:, 2] == e["clk"] + 1).all()


@pytest.mark.gpu
def test_u256x2048_mul_shard_from_device_traces():
    """A U256XU2048_MUL precompile shard built on the device (the eight chained mul-and-carry field ops)
    equals the host builders' traces and multiplicities and proves to the same bytes."""
    import torch
    from zkmips_amd import mips_ec as EC
    from zkmips_amd._lib import Device
    from zkmips_amd.prover import HipProver
    evs = _u256x2048_events()
    m, prep, tr, pv = MC.precompile_shard(EC.U256XU2048_MUL, evs, shard=5)
    bm = torch.zeros((A.BYTE_ROWS, A.BYTE_MULT_WIDTH), dtype=torch.int32, device="cuda")
    dev = TG.precompile_shard_traces(EC.U256XU2048_MUL, evs, byte_mult=bm)
    torch.cuda.synchronize()
    assert "U256XU2048Mul" in dev
    for name, t in dev.items():
        got = t.cpu().numpy().view(np.uint32)
        bad = np.argwhere(got != tr[name])
        assert not len(bad), (name, bad[:8].tolist())
    assert np.array_equal(bm.cpu().numpy().view(np.uint32), tr["Byte"])
    traces = {k: v for k, v in tr.items() if k not in dev}
    traces.update(dev)
    traces["Byte"] = bm
    prover = HipProver(Device(0), m, _core_prep(), num_queries=16)
    assert prover.prove_shard(traces, pv) == prover.prove_shard(tr, pv)


def _fp_op_events(field: str, seed: int = 17):
    """FpOp calls of one field through the executor (mips_ec.exec_fp_op): add, sub, mul on random words
    (operands at or above the modulus included, reduced by the call), zeros and p - 1."""
    from zkmips_amd import emulated_field as EF
    from zkmips_amd import mips_ec as EC
    rng = np.random.default_rng(seed)
    fp = EC.FIELDS[field]
    words = {}
    mem, mem_init, mem_last = {}, {}, {}
    vals = [int.from_bytes(rng.bytes(fp.nl), "little") for _ in range(10)] + [0, fp.modulus - 1, fp.modulus]
    evs = []
    for k in range(2 * len(vals)):
        op = ("add", "sub", "mul")[k % 3]
        x, y = vals[k % len(vals)], vals[(3 * k + 1) % len(vals)]
        xp, yp = 0x20000 + 0x100 * k, 0x30000 + 0x100 * k
        for i, w in enumerate(EF.int_to_words(x, fp.words)):
            words[xp + 4 * i] = w
        for i, w in enumerate(EF.int_to_words(y, fp.words)):
            words[yp + 4 * i] = w
        shard, clk = 3 + k // 12, 70 + 8 * k
        pm = SY.PrecompileMemory(mem, mem_init, mem_last, {}, [], shard, lambda a: words.get(a, 0))
        code = EC.FP_OPS[field][("add", "sub", "mul").index(op)]
        evs.append((EC.FP_OPS[field][0], (shard, clk, SY.syscall_id(code), xp, yp),
                    EC.exec_fp_op(field, op, pm, shard, clk, xp, yp)))
    return evs


@pytest.mark.parametrize("field", ["Bn254", "Bls12381"])
def test_fp_op_records_layout(field):
    """zkm_fp_op_event records: the op code, y read at clk, x written at clk + 1, in slots of 12 words."""
    evs = _fp_op_events(field)
    rec = TG.fp_op_records([e for _, _, e in evs])
    assert rec.dtype.itemsize == 548
    w = 8 if field == "Bn254" else 12
    for r, (_, _, e) in zip(rec, evs):
        assert r["op"] == ("add", "sub", "mul").index(e["op"])
        assert list(r["x"][:w, 3]) == e["x"] and (r["x"][:w, 2] == e["clk"] + 1).all() and not r["x"][w:].any()


@pytest.mark.gpu
@pytest.mark.parametrize("field", ["Bn254", "Bls12381"])
def test_fp_op_shard_from_device_traces(field):
    """A base-field FpOp precompile shard built on the device (operands reduced, the sum / difference /
    product divided by the modulus, the field op's witness) equals the host builders' traces and
    multiplicities and proves to the same bytes."""
    import torch
    from zkmips_amd import mips_ec as EC
    from zkmips_amd._lib import Device
    from zkmips_amd.prover import HipProver
    evs = _fp_op_events(field)
    key = EC.FP_OPS[field][0]
    m, prep, tr, pv = MC.precompile_shard(key, evs, shard=5)
    bm = torch.zeros((A.BYTE_ROWS, A.BYTE_MULT_WIDTH), dtype=torch.int32, device="cuda")
    dev = TG.precompile_shard_traces(key, evs, byte_mult=bm)
    torch.cuda.synchronize()
    assert EC.FP_NAME[field] in dev
    for name, t in dev.items():
        got = t.cpu().numpy().view(np.uint32)
        bad = np.argwhere(got != tr[name])
        assert not len(bad), (name, bad[:8].tolist())
    assert np.array_equal(bm.cpu().numpy().view(np.uint32), tr["Byte"])
    traces = {k: v for k, v in tr.items() if k not in dev}
    traces.update(dev)
    traces["Byte"] = bm
    prover = HipProver(Device(0), m, _core_prep(), num_queries=16)
    assert prover.prove_shard(traces, pv) == prover.prove_shard(tr, pv)


def _fp2_events(field: str, mul: bool, seed: int = 19):
    """Fp2AddSub (add and sub) or Fp2Mul calls of one field through the executor (mips_ec.exec_fp2_addsub /
    exec_fp2_mul): random coordinates (some at or above the modulus), zeros and p - 1."""
    from zkmips_amd import emulated_field as EF
    from zkmips_amd import mips_ec as EC
    rng = np.random.default_rng(seed)
    fp = EC.FIELDS[field]
    words = {}
    mem, mem_init, mem_last = {}, {}, {}
    vals = [int.from_bytes(rng.bytes(fp.nl), "little") for _ in range(8)] + [0, fp.modulus - 1, fp.modulus]
    evs = []
    for k in range(22):
        op = "mul" if mul else ("add", "sub")[k % 2]
        x = [vals[(k + j) % len(vals)] for j in (0, 3)]
        y = [vals[(5 * k + j) % len(vals)] for j in (1, 7)]
        xp, yp = 0x40000 + 0x200 * k, 0x50000 + 0x200 * k
        for i, w in enumerate(EF.int_to_words(x[0], fp.words) + EF.int_to_words(x[1], fp.words)):
            words[xp + 4 * i] = w
        for i, w in enumerate(EF.int_to_words(y[0], fp.words) + EF.int_to_words(y[1], fp.words)):
            words[yp + 4 * i] = w
        shard, clk = 3 + k // 12, 90 + 8 * k
        pm = SY.PrecompileMemory(mem, mem_init, mem_last, {}, [], shard, lambda a: words.get(a, 0))
        if mul:
            key = code = EC.FP2_MUL[field]
            ev = EC.exec_fp2_mul(field, pm, shard, clk, xp, yp)
        else:
            key, code = EC.FP2_ADDSUB[field][0], EC.FP2_ADDSUB[field][k % 2]
            ev = EC.exec_fp2_addsub(field, op, pm, shard, clk, xp, yp)
        evs.append((key, (shard, clk, SY.syscall_id(code), xp, yp), ev))
    return evs


@pytest.mark.gpu
@pytest.mark.parametrize("field", ["Bn254", "Bls12381"])
@pytest.mark.parametrize("mul", [False, True])
def test_fp2_shard_from_device_traces(field, mul):
    """Fp2AddSub / Fp2Mul precompile shards built on the device (two / six chained base-field ops per row)
    equal the host builders' traces and multiplicities and prove to the same bytes."""
    import torch
    from zkmips_amd import mips_ec as EC
    from zkmips_amd._lib import Device
    from zkmips_amd.prover import HipProver
    evs = _fp2_events(field, mul)
    key = evs[0][0]
    m, prep, tr, pv = MC.precompile_shard(key, evs, shard=5)
    bm = torch.zeros((A.BYTE_ROWS, A.BYTE_MULT_WIDTH), dtype=torch.int32, device="cuda")
    dev = TG.precompile_shard_traces(key, evs, byte_mult=bm)
    torch.cuda.synchronize()
    assert (EC.FP2_MUL_NAME if mul else EC.FP2_ADDSUB_NAME)[field] in dev
    for name, t in dev.items():
        got = t.cpu().numpy().view(np.uint32)
        bad = np.argwhere(got != tr[name])
        assert not len(bad), (name, bad[:8].tolist())
    assert np.array_equal(bm.cpu().numpy().view(np.uint32), tr["Byte"])
    traces = {k: v for k, v in tr.items() if k not in dev}
    traces.update(dev)
    traces["Byte"] = bm
    prover = HipProver(Device(0), m, _core_prep(), num_queries=16)
    assert prover.prove_shard(traces, pv) == prover.prove_shard(tr, pv)


def _ec_add_events(curve: str, seed: int = 23):
    """Weierstrass additions of random points through the executor (mips_ec.exec_ec_add)."""
    from zkmips_amd import mips_ec as EC
    rng = np.random.default_rng(seed)
    words = {}
    mem, mem_init, mem_last = {}, {}, {}
    evs = []
    for k in range(20):
        p, q = EC.random_point(curve, rng), EC.random_point(curve, rng)
        pp, qp = 0x60000 + 0x200 * k, 0x70000 + 0x200 * k
        for i, w in enumerate(EC.point_words(curve, p)):
            words[pp + 4 * i] = w
        for i, w in enumerate(EC.point_words(curve, q)):
            words[qp + 4 * i] = w
        shard, clk = 3 + k // 12, 110 + 8 * k
        pm = SY.PrecompileMemory(mem, mem_init, mem_last, {}, [], shard, lambda a: words.get(a, 0))
        evs.append((EC.EC_ADD[curve], (shard, clk, SY.syscall_id(EC.EC_ADD[curve]), pp, qp),
                    EC.exec_ec_add(curve, pm, shard, clk, pp, qp)))
    return evs


@pytest.mark.gpu
@pytest.mark.parametrize("curve", ["Secp256k1", "Secp256r1", "Bn254", "Bls12381"])
def test_ec_add_shard_from_device_traces(curve):
    """Weierstrass addition shards built on the device (nine chained field ops, the slope through a modular
    inverse) equal the host builders' traces and multiplicities and prove to the same bytes."""
    import torch
    from zkmips_amd import mips_ec as EC
    from zkmips_amd._lib import Device
    from zkmips_amd.prover import HipProver
    evs = _ec_add_events(curve)
    key = evs[0][0]
    m, prep, tr, pv = MC.precompile_shard(key, evs, shard=5)
    bm = torch.zeros((A.BYTE_ROWS, A.BYTE_MULT_WIDTH), dtype=torch.int32, device="cuda")
    dev = TG.precompile_shard_traces(key, evs, byte_mult=bm)
    torch.cuda.synchronize()
    assert f"{curve}AddAssign" in dev
    for name, t in dev.items():
        got = t.cpu().numpy().view(np.uint32)
        bad = np.argwhere(got != tr[name])
        assert not len(bad), (name, bad[:8].tolist())
    assert np.array_equal(bm.cpu().numpy().view(np.uint32), tr["Byte"])
    traces = {k: v for k, v in tr.items() if k not in dev}
    traces.update(dev)
    traces["Byte"] = bm
    prover = HipProver(Device(0), m, _core_prep(), num_queries=16)
    assert prover.prove_shard(traces, pv) == prover.prove_shard(tr, pv)


def _ec_double_events(curve: str, seed: int = 29):
    """Weierstrass doublings of random points through the executor (mips_ec.exec_ec_double)."""
    from zkmips_amd import mips_ec as EC
    rng = np.random.default_rng(seed)
    words = {}
    mem, mem_init, mem_last = {}, {}, {}
    evs = []
    for k in range(20):
        pp = 0x80000 + 0x200 * k
        for i, w in enumerate(EC.point_words(curve, EC.random_point(curve, rng))):
            words[pp + 4 * i] = w
        shard, clk = 3 + k // 12, 130 + 8 * k
        pm = SY.PrecompileMemory(mem, mem_init, mem_last, {}, [], shard, lambda a: words.get(a, 0))
        evs.append((EC.EC_DOUBLE[curve], (shard, clk, SY.syscall_id(EC.EC_DOUBLE[curve]), pp, 0),
                    EC.exec_ec_double(curve, pm, shard, clk, pp, 0)))
    return evs


@pytest.mark.gpu
@pytest.mark.parametrize("curve", ["Secp256k1", "Secp256r1", "Bn254", "Bls12381"])
def test_ec_double_shard_from_device_traces(curve):
    """Weierstrass doubling shards built on the device (eleven chained field ops; padding rows double
    (0, 1) with the dummy y record) equal the host builders' traces and multiplicities and prove to the same
    bytes."""
    import torch
    from zkmips_amd._lib import Device
    from zkmips_amd.prover import HipProver
    evs = _ec_double_events(curve)
    key = evs[0][0]
    m, prep, tr, pv = MC.precompile_shard(key, evs, shard=5)
    bm = torch.zeros((A.BYTE_ROWS, A.BYTE_MULT_WIDTH), dtype=torch.int32, device="cuda")
    dev = TG.precompile_shard_traces(key, evs, byte_mult=bm)
    torch.cuda.synchronize()
    assert f"{curve}DoubleAssign" in dev
    for name, t in dev.items():
        got = t.cpu().numpy().view(np.uint32)
        bad = np.argwhere(got != tr[name])
        assert not len(bad), (name, bad[:8].tolist())
    assert np.array_equal(bm.cpu().numpy().view(np.uint32), tr["Byte"])
    traces = {k: v for k, v in tr.items() if k not in dev}
    traces.update(dev)
    traces["Byte"] = bm
    prover = HipProver(Device(0), m, _core_prep(), num_queries=16)
    assert prover.prove_shard(traces, pv) == prover.prove_shard(tr, pv)


def _ec_decompress_events(curve: str, seed: int = 31):
    """Weierstrass decompressions through the executor (mips_ec.exec_ec_decompress): random points' x with
    both signs."""
    from zkmips_amd import emulated_field as EF
    from zkmips_amd import mips_ec as EC
    rng = np.random.default_rng(seed)
    fp = EC.FIELDS[curve]
    words = {}
    mem, mem_init, mem_last = {}, {}, {}
    evs = []
    for k in range(20):
        ptr = 0x90000 + 0x200 * k
        for i, w in enumerate(EF.int_to_words(EC.random_point(curve, rng)[0], fp.words)):
            words[ptr + fp.nl + 4 * i] = w
        shard, clk = 3 + k // 12, 150 + 8 * k
        pm = SY.PrecompileMemory(mem, mem_init, mem_last, {}, [], shard, lambda a: words.get(a, 0))
        evs.append((EC.EC_DECOMPRESS[curve], (shard, clk, SY.syscall_id(EC.EC_DECOMPRESS[curve]), ptr, k % 2),
                    EC.exec_ec_decompress(curve, pm, shard, clk, ptr, k % 2)))
    return evs


@pytest.mark.gpu
@pytest.mark.parametrize("curve", ["Secp256k1", "Secp256r1", "Bls12381"])
def test_ec_decompress_shard_from_device_traces(curve):
    """Weierstrass decompression shards built on the device (the square root by exponentiation, the inner
    product a x + b, bls12-381's lexicographic choice) equal the host builders' traces and multiplicities
    and prove to the same bytes."""
    import torch
    from zkmips_amd._lib import Device
    from zkmips_amd.prover import HipProver
    evs = _ec_decompress_events(curve)
    key = evs[0][0]
    m, prep, tr, pv = MC.precompile_shard(key, evs, shard=5)
    bm = torch.zeros((A.BYTE_ROWS, A.BYTE_MULT_WIDTH), dtype=torch.int32, device="cuda")
    dev = TG.precompile_shard_traces(key, evs, byte_mult=bm)
    torch.cuda.synchronize()
    assert f"{curve}Decompress" in dev
    for name, t in dev.items():
        got = t.cpu().numpy().view(np.uint32)
        bad = np.argwhere(got != tr[name])
        assert not len(bad), (name, bad[:8].tolist())
    assert np.array_equal(bm.cpu().numpy().view(np.uint32), tr["Byte"])
    traces = {k: v for k, v in tr.items() if k not in dev}
    traces.update(dev)
    traces["Byte"] = bm
    prover = HipProver(Device(0), m, _core_prep(), num_queries=16)
    assert prover.prove_shard(traces, pv) == prover.prove_shard(tr, pv)


def _ed_add_events(seed: int = 37):
    """Ed25519 additions through the executor (mips_edwards.exec_ed_add): multiples of the base point,
    a point added to itself, the identity."""
    from zkmips_amd import mips_edwards as ED
    rng = np.random.default_rng(seed)
    words = {}
    mem, mem_init, mem_last = {}, {}, {}
    pts = [ED._scalar_mul(int(rng.integers(1, 1 << 62)), (ED.BASE_X, ED.BASE_Y)) for _ in range(8)] + [(0, 1)]
    evs = []
    for k in range(20):
        p, q = pts[k % len(pts)], pts[(k * 5 + 2) % len(pts)]
        pp, qp = 0xA0000 + 0x200 * k, 0xB0000 + 0x200 * k
        for i, w in enumerate(ED._point_words(*p)):
            words[pp + 4 * i] = w
        for i, w in enumerate(ED._point_words(*q)):
            words[qp + 4 * i] = w
        shard, clk = 3 + k // 12, 170 + 8 * k
        pm = SY.PrecompileMemory(mem, mem_init, mem_last, {}, [], shard, lambda a: words.get(a, 0))
        evs.append((SY.ED_ADD, (shard, clk, SY.syscall_id(SY.ED_ADD), pp, qp), ED.exec_ed_add(pm, shard, clk, pp, qp)))
    return evs


@pytest.mark.gpu
def test_ed_add_shard_from_device_traces():
    """An ED_ADD precompile shard built on the device (inner products, products, the two denominators'
    inverses) equals the host builders' traces and multiplicities and proves to the same bytes."""
    import torch
    from zkmips_amd._lib import Device
    from zkmips_amd.prover import HipProver
    evs = _ed_add_events()
    m, prep, tr, pv = MC.precompile_shard(SY.ED_ADD, evs, shard=5)
    bm = torch.zeros((A.BYTE_ROWS, A.BYTE_MULT_WIDTH), dtype=torch.int32, device="cuda")
    dev = TG.precompile_shard_traces(SY.ED_ADD, evs, byte_mult=bm)
    torch.cuda.synchronize()
    assert "EdAddAssign" in dev
    for name, t in dev.items():
        got = t.cpu().numpy().view(np.uint32)
        bad = np.argwhere(got != tr[name])
        assert not len(bad), (name, bad[:8].tolist())
    assert np.array_equal(bm.cpu().numpy().view(np.uint32), tr["Byte"])
    traces = {k: v for k, v in tr.items() if k not in dev}
    traces.update(dev)
    traces["Byte"] = bm
    prover = HipProver(Device(0), m, _core_prep(), num_queries=16)
    assert prover.prove_shard(traces, pv) == prover.prove_shard(tr, pv)


def _ed_decompress_events(seed: int = 41):
    """Ed25519 decompressions through the executor (mips_edwards.exec_ed_decompress): y of multiples of the
    base point with both signs."""
    from zkmips_amd import mips_edwards as ED
    rng = np.random.default_rng(seed)
    words = {}
    mem, mem_init, mem_last = {}, {}, {}
    evs = []
    for k in range(20):
        _, y = ED._scalar_mul(int(rng.integers(1, 1 << 62)), (ED.BASE_X, ED.BASE_Y))
        ptr = 0xC0000 + 0x200 * k
        for i, w in enumerate(ED._point_words(0, y)[8:]):
            words[ptr + 32 + 4 * i] = w
        shard, clk = 3 + k // 12, 190 + 8 * k
        pm = SY.PrecompileMemory(mem, mem_init, mem_last, {}, [], shard, lambda a: words.get(a, 0))
        evs.append((SY.ED_DECOMPRESS, (shard, clk, SY.syscall_id(SY.ED_DECOMPRESS), ptr, k % 2),
                    ED.exec_ed_decompress(pm, shard, clk, ptr, k % 2)))
    return evs


@pytest.mark.gpu
def test_ed_decompress_shard_from_device_traces():
    """An ED_DECOMPRESS precompile shard built on the device (the square root with lsb 0, its FieldSqrtCols)
    equals the host builders' traces and multiplicities and proves to the same bytes."""
    import torch
    from zkmips_amd._lib import Device
    from zkmips_amd.prover import HipProver
    evs = _ed_decompress_events()
    m, prep, tr, pv = MC.precompile_shard(SY.ED_DECOMPRESS, evs, shard=5)
    bm = torch.zeros((A.BYTE_ROWS, A.BYTE_MULT_WIDTH), dtype=torch.int32, device="cuda")
    dev = TG.precompile_shard_traces(SY.ED_DECOMPRESS, evs, byte_mult=bm)
    torch.cuda.synchronize()
    assert "EdDecompress" in dev
    for name, t in dev.items():
        got = t.cpu().numpy().view(np.uint32)
        bad = np.argwhere(got != tr[name])
        assert not len(bad), (name, bad[:8].tolist())
    assert np.array_equal(bm.cpu().numpy().view(np.uint32), tr["Byte"])
    traces = {k: v for k, v in tr.items() if k not in dev}
    traces.update(dev)
    traces["Byte"] = bm
    prover = HipProver(Device(0), m, _core_prep(), num_queries=16)
    assert prover.prove_shard(traces, pv) == prover.prove_shard(tr, pv)


def _keccak_events(seed: int = 43):
    """KECCAK_SPONGE calls through the executor (mips_keccak.exec_keccak_sponge): one, two and three
    absorbed blocks, repeated over two shards."""
    from zkmips_amd import mips_keccak as KS
    rng = np.random.default_rng(seed)
    words = {}
    mem, mem_init, mem_last = {}, {}, {}
    evs = []
    for k, nb in enumerate([1, 2, 3, 1, 2]):
        ip, op = 0xD0000 + 0x1000 * k, 0xE0000 + 0x1000 * k
        for i in range(36 * nb):
            words[ip + 4 * i] = int(rng.integers(0, 1 << 32))
        words[op + 64] = 36 * nb
        shard, clk = 3 + k // 3, 210 + 8 * k
        pm = SY.PrecompileMemory(mem, mem_init, mem_last, {}, [], shard, lambda a: words.get(a, 0))
        evs.append((KS.KECCAK_SPONGE, (shard, clk, SY.syscall_id(KS.KECCAK_SPONGE), ip, op),
                    KS.exec_keccak_sponge(pm, shard, clk, ip, op)))
    return evs


def test_keccak_block_records():
    """zkm_keccak_block records: one per absorbed block, the previous block's xored state, the block's reads."""
    evs = _keccak_events()
    rec = TG.keccak_blocks([e for _, _, e in evs])
    assert rec.dtype.itemsize == 1552 and len(rec) == 9
    assert list(rec["block"]) == [0, 0, 1, 0, 1, 2, 0, 0, 1] and list(rec["nblocks"]) == [1, 2, 2, 3, 3, 3, 1, 2, 2]
    assert (rec["prev_xored"][rec["block"] == 0] == 0).all()
    assert np.array_equal(rec["prev_xored"][2], rec["xored"][1])


@pytest.mark.gpu
def test_keccak_sponge_shard_from_device_traces():
    """A KECCAK_SPONGE precompile shard built on the device (the rounds recomputed per row, the sponge
    columns, the XOR and access lookups) equals the host builders' traces and multiplicities and proves to
    the same bytes."""
    import torch
    from zkmips_amd import mips_keccak as KS
    from zkmips_amd._lib import Device
    from zkmips_amd.prover import HipProver
    evs = _keccak_events()
    m, prep, tr, pv = MC.precompile_shard(KS.KECCAK_SPONGE, evs, shard=5)
    bm = torch.zeros((A.BYTE_ROWS, A.BYTE_MULT_WIDTH), dtype=torch.int32, device="cuda")
    dev = TG.precompile_shard_traces(KS.KECCAK_SPONGE, evs, byte_mult=bm)
    torch.cuda.synchronize()
    assert "KeccakSponge" in dev
    for name, t in dev.items():
        got = t.cpu().numpy().view(np.uint32)
        bad = np.argwhere(got != tr[name])
        assert not len(bad), (name, bad[:8].tolist())
    assert np.array_equal(bm.cpu().numpy().view(np.uint32), tr["Byte"])
    traces = {k: v for k, v in tr.items() if k not in dev}
    traces.update(dev)
    traces["Byte"] = bm
    prover = HipProver(Device(0), m, _core_prep(), num_queries=16)
    assert prover.prove_shard(traces, pv) == prover.prove_shard(tr, pv)


def _sys_linux_events():
    """Linux syscalls through the executor (mips_syscall.exec_sys_linux): BRK above and below the break,
    MMAP / MMAP2 with a0 = 0 (aligned and unaligned sizes) and a0 != 0, CLONE, EXIT_GROUP, FCNTL (a1 = 1, 3,
    other; good and bad fds), READ (stdin, other fd), WRITE and a no-op syscall, over two shards."""
    regs = [(0x1000 * r + 7) % (1 << 32) for r in range(MC.NUM_REGS)]
    regs[MC.REG_BRK], regs[MC.REG_HEAP] = 0x10000000, 0x20000000
    last = [(1, r) for r in range(MC.NUM_REGS)]
    reg_start, reg_done = [(last[r], regs[r]) for r in range(MC.NUM_REGS)], []
    mem, mem_init, mem_last = {}, {}, {}
    calls = [(SY.SYS_BRK, 0x10001000, 0), (SY.SYS_BRK, 0x0FFF0000, 0), (SY.SYS_MMAP, 0, 0x3000),
             (SY.SYS_MMAP, 0, 0x2801), (SY.SYS_MMAP2, 0x4000, 0x1000), (SY.SYS_MMAP2, 0, 0x10), (SY.SYS_CLONE, 0, 0),
             (SY.SYS_FCNTL, 1, 3), (SY.SYS_FCNTL, 2, 1), (SY.SYS_FCNTL, 7, 3), (SY.SYS_FCNTL, 0, 4), (SY.SYS_READ, 0, 0),
             (SY.SYS_READ, 3, 0), (SY.SYS_WRITE, 1, 0), (SY.SYS_NOPS[0], 5, 6), (SY.SYS_EXT_GROUP, 0, 0)]
    evs = []
    for k, (code, a0, a1) in enumerate(calls * 2):
        shard, clk = 2 + k // 20, 40 + 8 * k
        pm = SY.PrecompileMemory(mem, mem_init, mem_last, {}, [], shard, lambda a: 0, regs, last, reg_start,
                                 reg_done)
        _, ev = SY.exec_sys_linux(pm, shard, clk, code, a0, a1)
        evs.append((SY.SYS_LINUX, (shard, clk, SY.syscall_id(code), a0, a1), ev))
    return evs


def test_sys_linux_records_layout():
    """zkm_sys_linux_event records: the call, the A3 write, the io access of BRK / WRITE / MMAP with a0 = 0."""
    evs = _sys_linux_events()
    rec = TG.sys_linux_records([e for _, _, e in evs])
    assert rec.dtype.itemsize == 72
    for r, (_, _, e) in zip(rec, evs):
        assert (r["code"], r["a0"], r["a1"], r["result"]) == (e["code"], e["a0"], e["a1"], e["v0"])
        assert r["a3"][3] == e["writes"][0][0] and r["a3"][0] == e["writes"][0][1]
        if e["code"] == SY.SYS_BRK:
            assert r["io"][0] == r["io"][3] == e["reads"][0][0]
        elif e["code"] in (SY.SYS_MMAP, SY.SYS_MMAP2) and e["a0"] == 0:
            assert list(r["io"][[3, 0]]) == list(e["writes"][1][:2])
        elif e["code"] != SY.SYS_WRITE:
            assert not r["io"].any()


@pytest.mark.gpu
def test_sys_linux_shard_from_device_traces():
    """A Linux-syscall precompile shard with every main trace and Byte lookup built on the device equals the
    host builders' traces and multiplicities and proves to the same bytes."""
    import torch
    from zkmips_amd._lib import Device
    from zkmips_amd.prover import HipProver
    evs = _sys_linux_events()
    m, prep, tr, pv = MC.precompile_shard(SY.SYS_LINUX, evs, shard=5)
    bm = torch.zeros((A.BYTE_ROWS, A.BYTE_MULT_WIDTH), dtype=torch.int32, device="cuda")
    dev = TG.precompile_shard_traces(SY.SYS_LINUX, evs, byte_mult=bm)
    torch.cuda.synchronize()
    assert "SysLinux" in dev
    for name, t in dev.items():
        assert np.array_equal(t.cpu().numpy().view(np.uint32), tr[name]), name
    assert np.array_equal(bm.cpu().numpy().view(np.uint32), tr["Byte"])
    traces = {k: v for k, v in tr.items() if k not in dev}
    traces.update(dev)
    traces["Byte"] = bm
    prover = HipProver(Device(0), m, _core_prep(), num_queries=16)
    assert prover.prove_shard(traces, pv) == prover.prove_shard(tr, pv)


@pytest.mark.gpu
def test_maxshape_shard_from_device_traces():
    """The reference's maximal 2^22 shard shape (scaled to Cpu 2^16): every chip's trace built on the device
    at the shape's height from the executor's records equals the host trace padded to the shape, the Byte
    multiplicities equal, and the proof bytes are identical."""
    import torch
    from zkmips_amd import shapes as SH
    from zkmips_amd._lib import Device
    from zkmips_amd.prover import HipProver
    cap = {}
    m, prep, tr, pv = SH.shape_shard(SH.MAXIMAL_22, seed=3, down=6, capture=cap)
    heights = {k: len(v) for k, v in tr.items() if k not in ("Byte", "Program")}
    bm = torch.zeros((A.BYTE_ROWS, A.BYTE_MULT_WIDTH), dtype=torch.int32, device="cuda")
    dev = TG.shard_traces(cap, byte_mult=bm, heights=heights)
    torch.cuda.synchronize()
    for name, t in dev.items():
        assert np.array_equal(t.cpu().numpy().view(np.uint32), tr[name]), name
    assert set(dev) >= set(heights), sorted(set(heights) - set(dev))
    assert np.array_equal(bm.cpu().numpy().view(np.uint32), tr["Byte"])
    traces = dict(dev)
    traces["Byte"] = bm
    prover = HipProver(Device(0), m, {k: v for k, v in prep.items() if v is not None}, num_queries=16)
    assert prover.prove_shard({k: v for k, v in traces.items() if k in tr}, pv) == prover.prove_shard(tr, pv)


def test_every_precompile_has_a_device_chip():
    """tracegen.precompile_chip maps every precompile the all-precompile, Keccak, Ed25519 and sha2 guests
    call to its chip, records of the header's layout and a trace builder (no chip left host-built)."""
    import collections
    from zkmips_amd import mips_ec as EC
    from zkmips_amd import mips_edwards as ED
    from zkmips_amd import mips_keccak as KS
    calls = collections.defaultdict(list)
    for prog, seed in ((EC.ec_program(1, reps=1), 1), (KS.keccak_program([b"abc" * 50]), 1),
                       (ED.ed25519_program(1, seed=3, scalar_bits=6), 3), (MC.sha_program(1, seed=5), 5)):
        st = MC.fresh_state()
        MC._execute(prog, MC.initial_registers(seed), 1, 1 << 22, st)
        for code, _, e in st["precompile"]:
            calls[code].append(e)
    names = set()
    for code, evs in calls.items():
        name, rec, fn = TG.precompile_chip(code, evs)
        assert callable(fn) and len(rec) >= len(evs) and rec.dtype.itemsize % 4 == 0
        names.add(name)
    assert len(names) == 25 and {"KeccakSponge", "EdAddAssign", "Bls12381Decompress", "ShaCompress"} <= names
