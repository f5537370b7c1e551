"""MIPS core shard: the reference's CPU and Program chips restated as machine-blob AIRs on top of the
ALU slice.

* ``Program`` crates/core/machine/src/program/mod.rs:31-41, :66-181 — preprocessed (pc, instruction)
  table receiving the CPU's program lookups, one multiplicity column.
* ``Cpu``     crates/core/machine/src/cpu/{columns,air/mod.rs:26-215,air/register.rs:13-75,trace.rs} —
  the 67-column CPU AIR: program and instruction lookups, register reads/writes through the memory
  argument (`eval_memory_access`, crates/core/machine/src/air/memory.rs:18-173, with the 24-bit
  timestamp range checks), shard/clk/pc/is_real constraints against the public values.
* the ALU chips and the Byte table of `mips_alu` receive the CPU's instructions and byte lookups.

Stand-in: in a real shard the register accesses' memory lookups are closed by MemoryLocal (and its
global interactions with the Global chip's septic-curve digest).  ``RegisterState`` stands in for
that: one row per register receiving its value at the shard's start and sending its value at the
end, so the memory argument balances inside the shard.  The program is straight-line MIPS ALU code
(no branches: the Branch/Jump chips are not restated), executed once per shard.
"""
from __future__ import annotations

import numpy as np

from . import mips_alu as A
from .machine import (ChipDesc, IS_FIRST, IS_LAST, IS_TRANSITION, KIND_BYTE, KIND_INSTRUCTION, KIND_MEMORY,
                      KIND_PROGRAM, Lookup, MachineDesc, P, VirtualPairCol as V, main, main_next, pv)
from .workloads import NUM_PV_ELTS, PROOF_MAX_NUM_PVS, splitmix64

_m = A._m
ZERO = A.ZERO
_assert_bool = A._assert_bool

# PublicValues (crates/stark/src/air/public_values.rs:18-32): 8 digest words (32), 8 deferred, then
PV_START_PC, PV_NEXT_PC, PV_EXIT_CODE, PV_SHARD, PV_EXECUTION_SHARD = 40, 41, 42, 43, 44
POS_C, POS_B, POS_A = 1, 2, 3  # MemoryAccessPosition (core/executor/src/events/memory.rs:29-40)
PC_BASE = 0x00400000

# ---------------------------------------------------------------- Cpu columns (cpu/columns/mod.rs)
C_SHARD, C_CLK16, C_CLK8, C_SHARD_SEND, C_CLK_SEND, C_PC, C_NPC, C_NNPC = range(8)
C_OPCODE, C_OPA, C_OPB, C_OPC, C_OPA0, C_IMMB, C_IMMC = 8, 9, 10, 14, 18, 19, 20  # InstructionCols
C_EXTRA, C_RW_A, C_CHECK_MEM, C_HALT, C_SEQ = 21, 22, 23, 24, 25
C_A_VAL, C_HI_PREV_A = 26, 30
C_A_ACC, C_B_ACC, C_C_ACC = 34, 47, 56  # MemoryReadWriteCols (prev_value + access), MemoryReadCols x2
C_REAL, C_A_IMM = 65, 66
CPU_WIDTH = 67
# MemoryAccessCols offsets (memory/consistency/columns.rs:29-50)
ACC_VALUE, ACC_PREV_SHARD, ACC_PREV_CLK, ACC_COMPARE, ACC_D16, ACC_D8 = 0, 4, 5, 6, 7, 8


def _word(base):
    return [main(base + i) for i in range(4)]


def _vword(base):
    return [_m(base + i) for i in range(4)]


def _eval_memory_access(ch, acc, prev_value_base, clk_pos, addr_col, do_check_expr, do_check_vpc):
    """MemoryAirBuilder::eval_memory_access + eval_memory_access_timestamp + eval_range_check_24bits
    (air/memory.rs:18-62, :90-173) for one register access of the CPU row."""
    M = main
    shard = M(C_SHARD)
    clk = M(C_CLK8) * 65536 + M(C_CLK16) + clk_pos
    compare = M(acc + ACC_COMPARE)
    _assert_bool(ch, do_check_expr)
    _assert_bool(ch, compare, do_check_expr)
    ch.assert_zero(do_check_expr * compare * (shard - M(acc + ACC_PREV_SHARD)))
    prev_comp = compare * M(acc + ACC_PREV_CLK) + (1 - compare) * M(acc + ACC_PREV_SHARD)
    cur_comp = compare * clk + (1 - compare) * shard
    diff_minus_one = cur_comp - prev_comp - 1
    ch.assert_zero(do_check_expr * (diff_minus_one - (M(acc + ACC_D16) + M(acc + ACC_D8) * 65536)))
    ch.sends.append(Lookup([V.const(A.B_U16RANGE), _m(acc + ACC_D16), ZERO, ZERO, ZERO], do_check_vpc, KIND_BYTE))
    ch.sends.append(Lookup([V.const(A.B_U8RANGE), ZERO, ZERO, ZERO, _m(acc + ACC_D8)], do_check_vpc, KIND_BYTE))
    prev_vals = [_m(acc + ACC_PREV_SHARD), _m(acc + ACC_PREV_CLK), _m(addr_col)] + _vword(prev_value_base)
    cur_vals = [_m(C_SHARD), V([("main", C_CLK8, 65536), ("main", C_CLK16, 1)], clk_pos), _m(addr_col)]
    cur_vals += _vword(acc + ACC_VALUE)
    ch.sends.append(Lookup(prev_vals, do_check_vpc, KIND_MEMORY))
    ch.receives.append(Lookup(cur_vals, do_check_vpc, KIND_MEMORY))


def cpu_chip() -> ChipDesc:
    """CpuChip::eval (cpu/air/mod.rs:26-102) with eval_registers, eval_shard_clk, eval_pc and
    eval_is_real in the reference's order."""
    ch = ChipDesc("Cpu", prep_width=0, main_width=CPU_WIDTH)
    M = main
    real = M(C_REAL)
    clk = M(C_CLK8) * 65536 + M(C_CLK16)
    instr = [_m(C_OPCODE), _m(C_OPA)] + _vword(C_OPB) + _vword(C_OPC) + [_m(C_OPA0), _m(C_IMMB), _m(C_IMMC)]
    ch.sends.append(Lookup([_m(C_PC)] + instr, _m(C_REAL), KIND_PROGRAM))  # send_program (air/program.rs:14-26)
    # eval_registers (cpu/air/register.rs:13-75)
    b_val, c_val = C_B_ACC + ACC_VALUE, C_C_ACC + ACC_VALUE
    for i in range(4):
        ch.assert_zero(M(C_IMMB) * (M(b_val + i) - M(C_OPB + i)))
    for i in range(4):
        ch.assert_zero(M(C_IMMC) * (M(c_val + i) - M(C_OPC + i)))
    _eval_memory_access(ch, C_B_ACC, b_val, POS_B, C_OPB, 1 - M(C_IMMB), V([("main", C_IMMB, P - 1)], 1))
    _eval_memory_access(ch, C_C_ACC, c_val, POS_C, C_OPC, 1 - M(C_IMMC), V([("main", C_IMMC, P - 1)], 1))
    a_val = C_A_ACC + 4 + ACC_VALUE
    for i in range(4):
        ch.assert_zero(M(C_OPA0) * M(a_val + i))
    for i in range(4):
        ch.assert_zero((1 - M(C_OPA0)) * (M(C_A_VAL + i) - M(a_val + i)))
    for i in range(4):
        ch.assert_zero(M(C_RW_A) * (M(C_HI_PREV_A + i) - M(C_A_ACC + i)))
    _eval_memory_access(ch, C_A_ACC + 4, C_A_ACC, POS_A, C_OPA, real, _m(C_REAL))
    for k in (0, 2):
        ch.sends.append(Lookup([V.const(A.B_U8RANGE), ZERO, ZERO, _m(a_val + k), _m(a_val + k + 1)], _m(C_REAL),
                               KIND_BYTE))
    for i in range(4):
        ch.assert_zero(M(C_A_IMM) * (M(a_val + i) - M(C_A_ACC + i)))
    # shard / clk to send (cpu/air/mod.rs:52-61)
    ch.assert_zero(real * (M(C_SHARD_SEND) - (M(C_CHECK_MEM) * M(C_SHARD) + (1 - M(C_CHECK_MEM)) * 0)))
    ch.assert_zero(real * (M(C_CLK_SEND) - (M(C_CHECK_MEM) * clk + (1 - M(C_CHECK_MEM)) * 0)))
    ins = [_m(C_SHARD_SEND), _m(C_CLK_SEND), _m(C_PC), _m(C_NPC), _m(C_NNPC), _m(C_EXTRA), _m(C_OPCODE)]
    ins += _vword(C_A_VAL) + _vword(b_val) + _vword(c_val) + _vword(C_HI_PREV_A)
    ins += [_m(C_A_IMM), _m(C_RW_A), _m(C_CHECK_MEM), _m(C_HALT), _m(C_SEQ)]
    ch.sends.append(Lookup(ins, _m(C_REAL), KIND_INSTRUCTION))  # send_instruction
    # eval_shard_clk (:113-156)
    next_real = main_next(C_REAL)
    ch.assert_zero(IS_TRANSITION * next_real * (M(C_SHARD) - main_next(C_SHARD)))
    ch.sends.append(Lookup([V.const(A.B_U16RANGE), _m(C_SHARD), ZERO, ZERO, ZERO], _m(C_REAL), KIND_BYTE))
    ch.assert_zero(IS_FIRST * clk)
    next_clk = main_next(C_CLK8) * 65536 + main_next(C_CLK16)
    ch.assert_zero(IS_TRANSITION * next_real * (clk + 5 + M(C_EXTRA) - next_clk))
    ch.assert_zero(real * (clk - (M(C_CLK16) + M(C_CLK8) * 65536)))  # eval_range_check_24bits
    ch.sends.append(Lookup([V.const(A.B_U16RANGE), _m(C_CLK16), ZERO, ZERO, ZERO], _m(C_REAL), KIND_BYTE))
    ch.sends.append(Lookup([V.const(A.B_U8RANGE), ZERO, ZERO, ZERO, _m(C_CLK8)], _m(C_REAL), KIND_BYTE))
    # eval_pc (:159-200)
    ch.assert_zero(real * (pv(PV_EXECUTION_SHARD) - M(C_SHARD)))
    ch.assert_zero(IS_FIRST * (pv(PV_START_PC) - M(C_PC)))
    ch.assert_zero(IS_FIRST * (1 - M(C_HALT)) * (M(C_PC) + 4 - M(C_NPC)))
    ch.assert_zero(IS_TRANSITION * next_real * (M(C_NPC) - main_next(C_PC)))
    ch.assert_zero(IS_TRANSITION * next_real * (1 - main_next(C_HALT)) * (M(C_NNPC) - main_next(C_NPC)))
    ch.assert_zero(IS_TRANSITION * real * M(C_SEQ) * (M(C_NNPC) - (M(C_NPC) + 4)))
    ch.assert_zero(IS_TRANSITION * (real - next_real) * (pv(PV_NEXT_PC) - M(C_NPC)))
    ch.assert_zero(IS_LAST * real * (pv(PV_NEXT_PC) - M(C_NPC)))
    # eval_is_real (:206-215)
    _assert_bool(ch, real)
    ch.assert_zero(IS_FIRST * (real - 1))
    ch.assert_zero(IS_TRANSITION * (1 - real) * next_real)
    ch.assert_zero(IS_TRANSITION * M(C_HALT) * next_real)
    # padding rows (:95-99)
    for col in (C_IMMB, C_IMMC, C_RW_A):
        ch.assert_zero((1 - real) * (1 - M(col)))
    return ch


# ---------------------------------------------------------------- Program (program/mod.rs)
PROG_PREP_WIDTH, PROG_MAIN_WIDTH = 14, 1


def program_chip() -> ChipDesc:
    ch = ChipDesc("Program", prep_width=PROG_PREP_WIDTH, main_width=PROG_MAIN_WIDTH)
    ch.receives.append(Lookup([V.single_prep(i) for i in range(PROG_PREP_WIDTH)], _m(0), KIND_PROGRAM))
    return ch


# ---------------------------------------------------------------- register-state stand-in
RS_ADDR, RS_INIT_SHARD, RS_INIT_CLK, RS_INIT_VAL, RS_FIN_SHARD, RS_FIN_CLK, RS_FIN_VAL, RS_REAL = 0, 1, 2, 3, 7, 8, 9, 13
RS_WIDTH = 14


def register_state_chip() -> ChipDesc:
    """Closes the register chain of the memory argument inside the shard (stand-in for MemoryLocal)."""
    ch = ChipDesc("RegisterState", prep_width=0, main_width=RS_WIDTH, local_only=True)
    ch.receives.append(Lookup([_m(RS_INIT_SHARD), _m(RS_INIT_CLK), _m(RS_ADDR)] + _vword(RS_INIT_VAL),
                              _m(RS_REAL), KIND_MEMORY))
    ch.sends.append(Lookup([_m(RS_FIN_SHARD), _m(RS_FIN_CLK), _m(RS_ADDR)] + _vword(RS_FIN_VAL), _m(RS_REAL),
                           KIND_MEMORY))
    _assert_bool(ch, main(RS_REAL))
    return ch


def core_machine() -> MachineDesc:
    # MipsAir::chips order (crates/core/machine/src/mips/mod.rs): Program, Cpu, ALUs, ..., Byte, memory
    return MachineDesc([program_chip(), cpu_chip(), A.add_sub_chip(), A.bitwise_chip(), A.lt_chip(),
                        A.shift_left_chip(), A.shift_right_chip(), A.clo_clz_chip(), A.byte_chip(),
                        register_state_chip()], NUM_PV_ELTS)


# ---------------------------------------------------------------- program + execution
# (opcode, uses immediate c) mix of straight-line ALU code
_MIX = [(A.OP_ADD, 0), (A.OP_ADD, 1), (A.OP_SUB, 0), (A.OP_AND, 0), (A.OP_AND, 1), (A.OP_OR, 0), (A.OP_OR, 1),
        (A.OP_XOR, 0), (A.OP_XOR, 1), (A.OP_NOR, 0), (A.OP_SLT, 0), (A.OP_SLT, 1), (A.OP_SLTU, 0),
        (A.OP_SLL, 1), (A.OP_SRL, 1), (A.OP_SRA, 1), (A.OP_ROR, 1), (A.OP_SRL, 0), (A.OP_CLZ, 1), (A.OP_CLO, 1)]
_KIND = {A.OP_ADD: "add", A.OP_SUB: "add", A.OP_AND: "bit", A.OP_OR: "bit", A.OP_XOR: "bit", A.OP_NOR: "bit",
         A.OP_SLT: "lt", A.OP_SLTU: "lt", A.OP_SLL: "sll", A.OP_SRL: "sr", A.OP_SRA: "sr", A.OP_ROR: "sr",
         A.OP_CLZ: "clz", A.OP_CLO: "clz"}
M32 = 0xFFFFFFFF


def _alu(op, b, c):
    if op == A.OP_ADD:
        return (b + c) & M32
    if op == A.OP_SUB:
        return (b - c) & M32
    if op == A.OP_AND:
        return b & c
    if op == A.OP_OR:
        return b | c
    if op == A.OP_XOR:
        return b ^ c
    if op == A.OP_NOR:
        return ~(b | c) & M32
    if op == A.OP_SLT:
        return int((b - (1 << 32) if b >> 31 else b) < (c - (1 << 32) if c >> 31 else c))
    if op == A.OP_SLTU:
        return int(b < c)
    s = c & 31
    if op == A.OP_SLL:
        return (b << s) & M32
    if op == A.OP_SRL:
        return b >> s
    if op == A.OP_SRA:
        return ((b - (1 << 32) if b >> 31 else b) >> s) & M32
    if op == A.OP_ROR:
        return ((b >> s) | (b << (32 - s))) & M32 if s else b
    x = b if op == A.OP_CLZ else ~b & M32
    return 32 - x.bit_length()


def random_program(n: int, seed: int = 1):
    """n straight-line ALU instructions: (opcode, op_a, op_b, op_c, imm_c); register 0 is written now and
    then (the write is dropped, op_a_0)."""
    r = splitmix64(0xC0DE000 + seed, 5 * n + 5)
    prog = []
    for i in range(n):
        op, imm = _MIX[int(r[5 * i] % len(_MIX))]
        ra = int(r[5 * i + 1] % 32) if r[5 * i + 4] % 16 == 0 else 1 + int(r[5 * i + 1] % 31)
        rb = int(r[5 * i + 2] % 32)
        if op in (A.OP_CLZ, A.OP_CLO):
            c = 0
        elif imm and op in (A.OP_SLL, A.OP_SRL, A.OP_SRA, A.OP_ROR):
            c = int(r[5 * i + 3] % 32)
        elif imm:
            c = int(r[5 * i + 3] & np.uint64(M32))
        else:
            c = int(r[5 * i + 3] % 32)
        prog.append((op, ra, rb, c, imm))
    return prog


def core_shard(n: int, seed: int = 1, shard: int = 1):
    """(machine, prep_traces, traces, public_values) of one shard executing an n-instruction
    straight-line program once (n < 2^24 / 5: the CPU clk is range-checked to 24 bits)."""
    assert 0 < n and 5 * n + 5 < (1 << 24)
    prog = random_program(n, seed)
    init = splitmix64(0x5EED000 + seed, 32) & np.uint64(M32)
    regs = [0] + [int(x) for x in init[1:]]
    init_vals = list(regs)
    last = [(0, 0)] * 32  # (shard, timestamp) of each register's previous access
    height = max(16, 1 << (n - 1).bit_length())
    t = np.zeros((height, CPU_WIDTH), np.uint32)
    t[n:, C_IMMB] = 1
    t[n:, C_IMMC] = 1
    t[n:, C_RW_A] = 1
    rows = {k: [] for k in ("op", "a", "b", "c", "pc")}
    acc = np.zeros((n, 3, 4), np.int64)  # per access (C, B, A): prev_shard, prev_clk, compare, diff
    vals = np.zeros((n, 6), np.int64)  # a, b, c, prev_a, written a, executed? (unused)
    for i, (op, ra, rb, c, imm) in enumerate(prog):
        clk = 5 * i
        if not imm:
            ps, pc_ = last[c]
            acc[i, 0] = (ps, pc_, ps == shard, 0)
            last[c] = (shard, clk + POS_C)
            cv = regs[c]
        else:
            cv = c
        ps, pc_ = last[rb]
        acc[i, 1] = (ps, pc_, ps == shard, 0)
        last[rb] = (shard, clk + POS_B)
        bv = regs[rb]
        av = _alu(op, bv, cv)
        ps, pc_ = last[ra]
        acc[i, 2] = (ps, pc_, ps == shard, 0)
        last[ra] = (shard, clk + POS_A)
        prev_a = regs[ra]
        written = av if ra else 0
        if ra:
            regs[ra] = av
        vals[i] = (av, bv, cv, prev_a, written, 0)
        rows["op"].append(op)
        rows["pc"].append(PC_BASE + 4 * i)
    ops = np.asarray(rows["op"], np.uint32)
    pcs = np.asarray(rows["pc"], np.uint32)
    av, bv, cv, prev_a, written = (vals[:, j].astype(np.uint32) for j in range(5))
    clk = 5 * np.arange(n, dtype=np.int64)
    immc = np.asarray([p[4] for p in prog], np.uint32)
    opa = np.asarray([p[1] for p in prog], np.uint32)
    opb = np.asarray([p[2] for p in prog], np.uint32)
    opc = np.asarray([p[3] for p in prog], np.uint32)

    mult = np.zeros((A.BYTE_ROWS, A.BYTE_MULT_WIDTH), np.uint64)
    byte_lookup = A.byte_lookup_into(mult)
    t[:n, C_SHARD] = shard
    t[:n, C_CLK16] = clk & 0xFFFF
    t[:n, C_CLK8] = (clk >> 16) & 0xFF
    t[:n, C_PC] = pcs
    t[:n, C_NPC] = pcs + 4
    t[:n, C_NNPC] = pcs + 8
    t[:n, C_OPCODE] = ops
    t[:n, C_OPA] = opa
    t[:n, C_OPB:C_OPB + 4] = A._bytes(opb)
    t[:n, C_OPC:C_OPC + 4] = A._bytes(opc)
    t[:n, C_OPA0] = opa == 0
    t[:n, C_IMMB] = 0
    t[:n, C_IMMC] = immc
    t[:n, C_RW_A] = 0
    t[:n, C_SEQ] = 1
    t[:n, C_A_VAL:C_A_VAL + 4] = A._bytes(av)
    t[:n, C_REAL] = 1
    byte_lookup(A.B_U16RANGE, np.full(n, shard >> 8), np.full(n, shard & 0xFF))  # U16Range(shard): row a1
    byte_lookup(A.B_U16RANGE, (clk & 0xFFFF) >> 8, clk & 0xFF)
    byte_lookup(A.B_U8RANGE, np.zeros(n, np.int64), (clk >> 16) & 0xFF)
    for j, (base, value, pos, mask) in enumerate(((C_C_ACC, cv, POS_C, immc == 0), (C_B_ACC, bv, POS_B, None),
                                                   (C_A_ACC + 4, written, POS_A, None))):
        sel = np.ones(n, bool) if mask is None else mask
        t[:n, base + ACC_VALUE:base + ACC_VALUE + 4] = A._bytes(value)  # value always (cpu/trace.rs:151-152)
        t[:n, base + ACC_PREV_SHARD] = np.where(sel, acc[:, j, 0], 0)
        t[:n, base + ACC_PREV_CLK] = np.where(sel, acc[:, j, 1], 0)
        comp = acc[:, j, 2].astype(bool)
        t[:n, base + ACC_COMPARE] = sel & comp
        cur = np.where(comp, clk + pos, shard)
        prev = np.where(comp, acc[:, j, 1], acc[:, j, 0])
        d = (cur - prev - 1).astype(np.int64)
        assert (d[sel] >= 0).all() and (d[sel] < (1 << 24)).all()
        d = np.where(sel, d, 0)
        t[:n, base + ACC_D16] = d & 0xFFFF
        t[:n, base + ACC_D8] = d >> 16
        byte_lookup(A.B_U16RANGE, (d[sel] & 0xFFFF) >> 8, d[sel] & 0xFF)
        byte_lookup(A.B_U8RANGE, np.zeros(int(sel.sum()), np.int64), d[sel] >> 16)
    t[:n, C_A_ACC:C_A_ACC + 4] = A._bytes(prev_a)  # op_a_access.prev_value
    wb = A._bytes(written)
    byte_lookup(A.B_U8RANGE, wb[:, 0], wb[:, 1])
    byte_lookup(A.B_U8RANGE, wb[:, 2], wb[:, 3])

    # ALU chips from the executed instructions (the CPU sends them, the ALU chips receive them)
    ev = {}
    kind_of = np.asarray([_KIND.get(o, "") for o in range(max(_KIND) + 1)])[ops]
    for kind in ("add", "bit", "lt", "sll", "sr", "clz"):
        s = kind_of == kind
        ev[kind] = (ops[s], av[s], bv[s], cv[s], pcs[s])
    traces = {"Cpu": t}
    traces.update(A.alu_traces(ev, mult))

    # Program: one row per instruction, executed once
    ph = max(16, 1 << (n - 1).bit_length())
    prep = np.zeros((ph, PROG_PREP_WIDTH), np.uint32)
    prep[:n, 0] = pcs
    prep[:n, 1:PROG_PREP_WIDTH] = t[:n, C_OPCODE:C_IMMC + 1]
    pm = np.zeros((ph, 1), np.uint32)
    pm[:n, 0] = 1
    traces["Program"] = pm

    rs = np.zeros((32, RS_WIDTH), np.uint32)
    rs[:, RS_ADDR] = np.arange(32)
    rs[:, RS_INIT_VAL:RS_INIT_VAL + 4] = A._bytes(np.asarray(init_vals, np.uint32))
    rs[:, RS_FIN_SHARD] = [s_ for s_, _ in last]
    rs[:, RS_FIN_CLK] = [c_ for _, c_ in last]
    rs[:, RS_FIN_VAL:RS_FIN_VAL + 4] = A._bytes(np.asarray(regs, np.uint32))
    rs[:, RS_REAL] = 1
    traces["RegisterState"] = rs

    assert mult.max() < P
    traces["Byte"] = mult.astype(np.uint32)
    pvs = (splitmix64(0xC0DE100 + seed, PROOF_MAX_NUM_PVS) % np.uint64(P)).astype(np.uint32)
    pvs[PV_START_PC] = PC_BASE
    pvs[PV_NEXT_PC] = PC_BASE + 4 * n
    pvs[PV_EXECUTION_SHARD] = shard
    prep_traces = {"Program": prep, "Byte": A.byte_prep_trace()}
    return core_machine(), prep_traces, traces, pvs
