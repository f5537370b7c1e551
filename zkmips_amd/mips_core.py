"""MIPS core shard: the reference's CPU and Program chips restated as machine-blob AIRs on top of the
ALU slice.

* ``Program`` crates/core/machine/src/program/mod.rs:31-41, :66-181 — preprocessed (pc, instruction)
  table receiving the CPU's program lookups, one multiplicity column.
* ``Cpu``     crates/core/machine/src/cpu/{columns,air/mod.rs:26-215,air/register.rs:13-75,trace.rs} —
  the 67-column CPU AIR: program and instruction lookups, register reads/writes through the memory
  argument (`eval_memory_access`, crates/core/machine/src/air/memory.rs:18-173, with the 24-bit
  timestamp range checks), shard/clk/pc/is_real constraints against the public values.
* the ALU chips and the Byte table of `mips_alu` receive the CPU's instructions and byte lookups.

The memory argument of a shard closes through MemoryLocal (every register and data word the shard
touched: its value at the shard's start received, its value at the end sent) and the Global chip,
which lifts MemoryLocal's global messages onto the septic curve and accumulates them into the shard's
global cumulative sum (zkmips_amd/mips_memory.py).
"""
from __future__ import annotations

import numpy as np

from . import mips_alu as A
from . import mips_memory as MM
from . import mips_syscall as SY
from .machine import (ChipDesc, Expr, IS_FIRST, IS_LAST, IS_TRANSITION, KIND_BYTE, KIND_INSTRUCTION, KIND_MEMORY,
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


CPU_CLK = ((C_CLK8, 65536), (C_CLK16, 1))  # clk = clk_8bit_limb * 2^16 + clk_16bit_limb


def _eval_memory_access(ch, acc, prev_value_base, clk_pos, addr, do_check_expr, do_check_vpc, shard_col=C_SHARD,
                        clk_terms=CPU_CLK):
    """MemoryAirBuilder::eval_memory_access + eval_memory_access_timestamp + eval_range_check_24bits
    (air/memory.rs:18-62, :90-173) for one register access at timestamp clk + clk_pos; `addr` is the
    register-number column or a constant (VirtualPairCol)."""
    M = main
    shard = M(shard_col)
    clk = sum((M(c) * w for c, w in clk_terms[1:]), M(clk_terms[0][0]) * clk_terms[0][1]) + clk_pos
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
    addr_v = addr if isinstance(addr, V) else _m(addr)
    prev_vals = [_m(acc + ACC_PREV_SHARD), _m(acc + ACC_PREV_CLK), addr_v] + _vword(prev_value_base)
    cur_vals = [_m(shard_col), V([("main", c, w) for c, w in clk_terms], clk_pos), addr_v]
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


# ---------------------------------------------------------------- Branch (control_flow/branch)
OP_BEQ, OP_BGEZ, OP_BGTZ, OP_BLEZ, OP_BLTZ, OP_BNE = 21, 22, 23, 24, 25, 26  # executor/src/opcode.rs:39-44
BRANCH_OPS = (OP_BEQ, OP_BGEZ, OP_BGTZ, OP_BLEZ, OP_BLTZ, OP_BNE)
# BranchColumns (control_flow/branch/columns.rs:11-61); a KoalaBearWordRangeChecker is 8 bits of the
# top byte + 6 running products (operations/koala_bear_word.rs:11-31)
RC_WIDTH = 14
BR_PC, BR_NPC, BR_NPC_RC, BR_TGT, BR_NNPC, BR_NNPC_RC = 0, 1, 5, 19, 23, 27
BR_A, BR_B, BR_C = 41, 45, 49
BR_BEQ, BR_BNE, BR_BLTZ, BR_BLEZ, BR_BGTZ, BR_BGEZ = range(53, 59)
BR_BRANCHING, BR_GT, BR_LT = 59, 60, 61
BR_WIDTH = 62


def _word_range_check(ch, value, rc, is_real):
    """KoalaBearWordRangeChecker::range_check (operations/koala_bear_word.rs:54-115): the word is a
    canonical field element (top byte < 0x7F, or == 0x7F with zero lower bytes)."""
    M = main
    bits = [M(rc + i) for i in range(8)]
    rec = Expr.lift(0)
    for i, b in enumerate(bits):
        _assert_bool(ch, b, is_real)
        rec = rec + (1 << i) * b
    ch.assert_zero(is_real * (rec - M(value + 3)))
    ch.assert_zero(is_real * bits[7])
    ch.assert_zero(is_real * (M(rc + 8) - bits[0] * bits[1]))
    for k in range(1, 6):
        ch.assert_zero(is_real * (M(rc + 8 + k) - M(rc + 7 + k) * bits[k + 1]))
    ch.assert_zero(is_real * M(rc + 13) * (M(value) + M(value + 1) + M(value + 2)))


def _send_alu(ch, opcode, a, b, c, mult):
    """send_alu (stark/src/air/builder.rs:282-323): an Instruction lookup at UNUSED_PC."""
    vals = [ZERO, ZERO, V.const(A.UNUSED_PC), V.const(A.UNUSED_PC + A.DEFAULT_PC_INC),
            V.const(A.UNUSED_PC + 2 * A.DEFAULT_PC_INC), ZERO, V.const(opcode)]
    vals += list(a) + list(b) + list(c) + [ZERO] * 4 + [ZERO, ZERO, ZERO, ZERO, V.const(1)]
    ch.sends.append(Lookup(vals, mult, KIND_INSTRUCTION))


def branch_chip() -> ChipDesc:
    """BranchChip::eval (control_flow/branch/air.rs:27-210), constraints and lookups in its order."""
    ch = ChipDesc("Branch", prep_width=0, main_width=BR_WIDTH, local_only=True)
    M = main
    order = (BR_BEQ, BR_BNE, BR_BLTZ, BR_BGEZ, BR_BLEZ, BR_BGTZ)
    for col in order:
        _assert_bool(ch, M(col))
    is_real = M(BR_BEQ) + M(BR_BNE) + M(BR_BLTZ) + M(BR_BGEZ) + M(BR_BLEZ) + M(BR_BGTZ)
    _assert_bool(ch, is_real)
    real_v = V([("main", col, 1) for col in order])
    opcode = V([("main", BR_BEQ, OP_BEQ), ("main", BR_BNE, OP_BNE), ("main", BR_BLTZ, OP_BLTZ),
                ("main", BR_BGEZ, OP_BGEZ), ("main", BR_BLEZ, OP_BLEZ), ("main", BR_BGTZ, OP_BGTZ)])
    red_v = lambda base: V([("main", base + i, 1 << (8 * i)) for i in range(4)])
    red = lambda base: sum((M(base + i) * (1 << (8 * i)) for i in range(1, 4)), M(base))
    ins = [ZERO, ZERO, _m(BR_PC), red_v(BR_NPC), red_v(BR_NNPC), ZERO, opcode]
    ins += _vword(BR_A) + _vword(BR_B) + _vword(BR_C) + [ZERO] * 4 + [V.const(1), ZERO, ZERO, ZERO, ZERO]
    ch.receives.append(Lookup(ins, real_v, KIND_INSTRUCTION))
    _word_range_check(ch, BR_NPC, BR_NPC_RC, is_real)
    _word_range_check(ch, BR_NNPC, BR_NNPC_RC, is_real)
    br = M(BR_BRANCHING)
    _send_alu(ch, A.OP_ADD, _vword(BR_TGT), _vword(BR_NPC), _vword(BR_C), _m(BR_BRANCHING))
    ch.assert_zero(is_real * (1 - br) * (red(BR_NPC) + 4 - red(BR_NNPC)))
    not_br = V([("main", col, 1) for col in order] + [("main", BR_BRANCHING, P - 1)])
    for base in (BR_NPC, BR_NNPC):
        for k in (0, 2):
            ch.sends.append(Lookup([V.const(A.B_U8RANGE), ZERO, ZERO, _m(base + k), _m(base + k + 1)], not_br,
                                   KIND_BYTE))
    for i in range(4):
        ch.assert_zero(is_real * br * (M(BR_TGT + i) - M(BR_NNPC + i)))
    ch.assert_zero((1 - is_real) * br)
    _assert_bool(ch, br, is_real)
    gt, lt = M(BR_GT), M(BR_LT)
    beq, bne, bltz, blez, bgtz, bgez = (M(c) for c in (BR_BEQ, BR_BNE, BR_BLTZ, BR_BLEZ, BR_BGTZ, BR_BGEZ))
    ch.assert_zero(beq * br * (gt + lt))
    ch.assert_zero(beq * (1 - br) * (gt + lt - 1))
    ch.assert_zero(bne * br * (gt + lt - 1))
    ch.assert_zero(bne * (1 - br) * (gt + lt))
    ch.assert_zero(bltz * br * (lt - 1))
    ch.assert_zero(bltz * (1 - br) * lt)
    ch.assert_zero(blez * br * gt)
    ch.assert_zero(blez * (1 - br) * (gt - 1))
    ch.assert_zero(bgtz * br * (gt - 1))
    ch.assert_zero(bgtz * (1 - br) * gt)
    ch.assert_zero(bgez * br * lt)
    ch.assert_zero(bgez * (1 - br) * (lt - 1))
    _send_alu(ch, A.OP_SLT, [_m(BR_LT), ZERO, ZERO, ZERO], _vword(BR_A), _vword(BR_B), real_v)
    _send_alu(ch, A.OP_SLT, [_m(BR_GT), ZERO, ZERO, ZERO], _vword(BR_B), _vword(BR_A), real_v)
    return ch


def _range_checker_cols(v: np.ndarray) -> np.ndarray:
    """KoalaBearWordRangeChecker::populate (operations/koala_bear_word.rs:34-52)."""
    bits = ((v[:, None].astype(np.uint64) >> (24 + np.arange(8, dtype=np.uint64))) & 1).astype(np.uint32)
    out = np.zeros((len(v), RC_WIDTH), np.uint32)
    out[:, :8] = bits
    acc = bits[:, 0] * bits[:, 1]
    out[:, 8] = acc
    for k in range(1, 6):
        acc = acc * bits[:, k + 1]
        out[:, 8 + k] = acc
    return out


# ---------------------------------------------------------------- Mul (alu/mul)
OP_MUL, OP_MULT, OP_MULTU = 2, 3, 4  # executor/src/opcode.rs:18-20
MUL_OPS = (OP_MUL, OP_MULT, OP_MULTU)
REG_LO, REG_HI = 32, 33  # Register::LO / HI; MULT/MULTU write LO via op_a, HI at position HI
REG_BRK, REG_HEAP, NUM_REGS = 34, 35, 36  # executor/src/register.rs:3-42
POS_HI = 4
# MulCols (alu/mul/mod.rs:35-105); op_hi_access is MemoryReadWriteCols (prev_value + access)
MU_PC, MU_NPC, MU_HI, MU_A, MU_B, MU_C, MU_CARRY, MU_PROD = 0, 1, 2, 6, 10, 14, 18, 26
MU_BMSB, MU_CMSB, MU_BSE, MU_CSE, MU_MUL, MU_MULT, MU_MULTU, MU_REAL = range(34, 42)
MU_HI_ACC, MU_HRR, MU_SHARD, MU_CLK = 42, 55, 56, 57
MU_WIDTH = 58


def mul_chip() -> ChipDesc:
    """MulChip::eval (alu/mul/mod.rs:335-506), constraints and lookups in its order."""
    ch = ChipDesc("Mul", prep_width=0, main_width=MU_WIDTH, local_only=True)
    M = main
    real = _m(MU_REAL)
    for msb, byte in ((MU_BMSB, MU_B + 3), (MU_CMSB, MU_C + 3)):
        ch.sends.append(Lookup([V.const(A.B_MSB), _m(msb), ZERO, _m(byte), ZERO], real, KIND_BYTE))
    ch.assert_zero(M(MU_BSE) - M(MU_MULT) * M(MU_BMSB))
    ch.assert_zero(M(MU_CSE) - M(MU_MULT) * M(MU_CMSB))
    b = [M(MU_B + i) for i in range(4)] + [M(MU_BSE) * 255] * 4
    c = [M(MU_C + i) for i in range(4)] + [M(MU_CSE) * 255] * 4
    m = [None] * 8
    for i in range(8):
        for j in range(8):
            if i + j < 8:
                t = b[i] * c[j]
                m[i + j] = t if m[i + j] is None else m[i + j] + t
    carry = [M(MU_CARRY + i) for i in range(8)]
    prod = [M(MU_PROD + i) for i in range(8)]
    for i in range(8):
        rhs = m[i] - carry[i] * 256 if i == 0 else m[i] + carry[i - 1] - carry[i] * 256
        ch.assert_zero(prod[i] - rhs)
    has_hi = M(MU_MULT) + M(MU_MULTU)
    for i in range(4):
        ch.assert_zero(prod[i] - M(MU_A + i))
        ch.assert_zero(has_hi * (prod[i + 4] - M(MU_HI + i)))
    for col in (MU_BMSB, MU_CMSB, MU_BSE, MU_CSE, MU_MUL, MU_MULT, MU_MULTU, MU_REAL, MU_HRR):
        _assert_bool(ch, M(col))
    ch.assert_zero(M(MU_BSE) * (M(MU_BMSB) - 1))
    ch.assert_zero(M(MU_CSE) * (M(MU_CMSB) - 1))
    ch.assert_zero(M(MU_REAL) * (M(MU_MUL) + M(MU_MULT) + M(MU_MULTU) - 1))
    for i in range(8):  # slice_range_check_u16(carry)
        ch.sends.append(Lookup([V.const(A.B_U16RANGE), _m(MU_CARRY + i), ZERO, ZERO, ZERO], real, KIND_BYTE))
    for k in range(0, 8, 2):  # slice_range_check_u8(product)
        ch.sends.append(Lookup([V.const(A.B_U8RANGE), ZERO, ZERO, _m(MU_PROD + k), _m(MU_PROD + k + 1)], real,
                               KIND_BYTE))
    opcode = V([("main", MU_MUL, OP_MUL), ("main", MU_MULT, OP_MULT), ("main", MU_MULTU, OP_MULTU)])
    ins = [_m(MU_SHARD), _m(MU_CLK), _m(MU_PC), _m(MU_NPC), V([("main", MU_NPC, 1)], 4), ZERO, opcode]
    ins += _vword(MU_A) + _vword(MU_B) + _vword(MU_C) + _vword(MU_HI) + [ZERO, ZERO, _m(MU_HRR), ZERO, V.const(1)]
    ch.receives.append(Lookup(ins, real, KIND_INSTRUCTION))
    _eval_memory_access(ch, MU_HI_ACC + 4, MU_HI_ACC, POS_HI, V.const(REG_HI), M(MU_HRR), _m(MU_HRR),
                        shard_col=MU_SHARD, clk_terms=((MU_CLK, 1),))
    ch.assert_zero(M(MU_HRR) * (M(MU_MULT) + M(MU_MULTU) - 1))
    for i in range(4):
        ch.assert_zero(M(MU_HRR) * (M(MU_HI + i) - M(MU_HI_ACC + 4 + ACC_VALUE + i)))
    ch.assert_zero((1 - M(MU_HRR)) * M(MU_CLK))
    ch.assert_zero((1 - M(MU_HRR)) * M(MU_SHARD))
    return ch


def _access_cols(t, rows, base, value, prev, shard, clk, sel, byte_lookup):
    """MemoryAccessCols::populate_access (memory/consistency/trace.rs:36-100) for rows `rows` (value,
    previous (shard, timestamp), compare flag, 16+8-bit limbs of the timestamp difference - 1) and the
    Byte lookups of its range checks; `sel` masks the accesses that happened."""
    t[rows, base + ACC_VALUE:base + ACC_VALUE + 4] = A._bytes(value)
    t[rows, base + ACC_PREV_SHARD] = np.where(sel, prev[:, 0], 0)
    t[rows, base + ACC_PREV_CLK] = np.where(sel, prev[:, 1], 0)
    comp = prev[:, 0] == shard
    t[rows, base + ACC_COMPARE] = sel & comp
    cur = np.where(comp, clk, shard)
    d = cur - np.where(comp, prev[:, 1], prev[:, 0]) - 1
    assert (d[sel] >= 0).all() and (d[sel] < (1 << 24)).all()
    d = np.where(sel, d, 0)
    t[rows, base + ACC_D16] = d & 0xFFFF
    t[rows, base + ACC_D8] = d >> 16
    byte_lookup(A.B_U16RANGE, (d[sel] & 0xFFFF) >> 8, d[sel] & 0xFF)
    byte_lookup(A.B_U8RANGE, np.zeros(int(sel.sum()), np.int64), d[sel] >> 16)


def _mul_trace(muls, shard, byte_lookup):
    """MulChip::event_to_row (alu/mul/mod.rs:218-318).  muls: (op, a, b, c, pc, npc, hi, clk, prev_hi,
    prev_shard, prev_clk) in execution order; clk < 0 for MUL (no HI record)."""
    E = np.asarray(muls, np.int64).reshape(-1, 11)
    n = len(E)
    t = np.zeros((A._pow2(n), MU_WIDTH), np.uint32)
    op, a, b, c, pc, npc, hi, clk = (E[:, j] for j in range(8))
    t[:n, MU_PC], t[:n, MU_NPC] = pc, npc
    for base, v in ((MU_HI, hi), (MU_A, a), (MU_B, b), (MU_C, c)):
        t[:n, base:base + 4] = A._bytes(v.astype(np.uint32))
    bw, cw = A._bytes(b.astype(np.uint32)).astype(np.int64), A._bytes(c.astype(np.uint32)).astype(np.int64)
    bmsb, cmsb = bw[:, 3] >> 7, cw[:, 3] >> 7
    bse, cse = (op == OP_MULT) & (bmsb == 1), (op == OP_MULT) & (cmsb == 1)
    t[:n, MU_BMSB], t[:n, MU_CMSB], t[:n, MU_BSE], t[:n, MU_CSE] = bmsb, cmsb, bse, cse
    b8 = np.concatenate([bw, np.where(bse, 255, 0)[:, None].repeat(4, 1)], axis=1)
    c8 = np.concatenate([cw, np.where(cse, 255, 0)[:, None].repeat(4, 1)], axis=1)
    prod = np.zeros((n, 8), np.int64)
    for i in range(8):
        for j in range(8 - i):
            prod[:, i + j] += b8[:, i] * c8[:, j]
    carry = np.zeros((n, 8), np.int64)
    for i in range(8):
        carry[:, i] = prod[:, i] >> 8
        prod[:, i] &= 0xFF
        if i + 1 < 8:
            prod[:, i + 1] += carry[:, i]
    t[:n, MU_CARRY:MU_CARRY + 8] = carry
    t[:n, MU_PROD:MU_PROD + 8] = prod
    t[:n, MU_MUL], t[:n, MU_MULT], t[:n, MU_MULTU] = op == OP_MUL, op == OP_MULT, op == OP_MULTU
    t[:n, MU_REAL] = 1
    byte_lookup(A.B_MSB, bw[:, 3], np.zeros(n, np.int64))
    byte_lookup(A.B_MSB, cw[:, 3], np.zeros(n, np.int64))
    for i in range(8):
        byte_lookup(A.B_U16RANGE, carry[:, i] >> 8, carry[:, i] & 0xFF)
    for k in range(0, 8, 2):
        byte_lookup(A.B_U8RANGE, prod[:, k], prod[:, k + 1])
    hrr = clk >= 0
    rows = np.arange(n)
    t[:n, MU_HRR] = hrr
    t[:n, MU_SHARD] = np.where(hrr, shard, 0)
    t[:n, MU_CLK] = np.where(hrr, clk, 0)
    t[:n, MU_HI_ACC:MU_HI_ACC + 4] = np.where(hrr[:, None], A._bytes(E[:, 8].astype(np.uint32)), 0)
    _access_cols(t, rows, MU_HI_ACC + 4, np.where(hrr, hi, 0).astype(np.uint32), E[:, 9:11], shard,
                 np.where(hrr, clk + POS_HI, 0), hrr, byte_lookup)
    return t


# ---------------------------------------------------------------- DivRem (alu/divrem)
OP_DIV, OP_DIVU, OP_MOD, OP_MODU = 5, 6, 7, 8  # executor/src/opcode.rs:21-24
DIV_OPS = (OP_DIV, OP_DIVU, OP_MOD, OP_MODU)
MULT_DIV = (OP_MULT, OP_MULTU, OP_DIV, OP_DIVU)  # Instruction::is_mult_div_instruction (instruction.rs:302)
# DivRemCols (alu/divrem/mod.rs); IsZeroWordOperation = 4 x (inverse, result) + lower, upper, result
DV_PC, DV_NPC, DV_B, DV_C, DV_Q, DV_R, DV_ABS_R, DV_ABS_C, DV_MAXC = 0, 1, 2, 6, 10, 14, 18, 22, 26
DV_CTQ, DV_CARRY, DV_IS_C0 = 30, 38, 46
DV_DIV, DV_DIVU, DV_MOD, DV_MODU, DV_OVF, DV_OVF_B, DV_OVF_C = 57, 58, 59, 60, 61, 62, 73
DV_BMSB, DV_RMSB, DV_CMSB, DV_BNEG, DV_RNEG, DV_CNEG, DV_RCM = range(84, 91)
DV_HI_ACC, DV_SHARD, DV_CLK = 91, 104, 105
DV_WIDTH = 106
IZW_WIDTH = 11


def _is_zero_word(ch, a, base, is_real):
    """IsZeroWordOperation::eval (operations/is_zero_word.rs:49-92) with IsZeroOperation per byte
    (operations/is_zero.rs:47-66)."""
    M = main
    for i in range(4):
        inv, res = M(base + 2 * i), M(base + 2 * i + 1)
        ch.assert_zero(is_real * ((1 - inv * a[i]) - res))
        _assert_bool(ch, res, is_real)
        ch.assert_zero(is_real * res * a[i])
    _assert_bool(ch, is_real)
    lower, upper, result = M(base + 8), M(base + 9), M(base + 10)
    for x in (lower, upper, result):
        _assert_bool(ch, x, is_real)
    ch.assert_zero(is_real * (lower - M(base + 1) * M(base + 3)))
    ch.assert_zero(is_real * (upper - M(base + 5) * M(base + 7)))
    ch.assert_zero(is_real * (result - lower * upper))


def _is_equal_word(ch, a, b, base, is_real):
    """IsEqualWordOperation::eval (operations/is_equal_word.rs:38-58)."""
    _assert_bool(ch, is_real)
    _is_zero_word(ch, [a[i] - b[i] for i in range(4)], base, is_real)


def divrem_chip() -> ChipDesc:
    """DivRemChip::eval (alu/divrem/mod.rs), constraints and lookups in its order."""
    ch = ChipDesc("DivRem", prep_width=0, main_width=DV_WIDTH, local_only=True)
    M = main
    w = lambda base: [M(base + i) for i in range(4)]
    div, divu, mod_, modu = M(DV_DIV), M(DV_DIVU), M(DV_MOD), M(DV_MODU)
    is_real = div + divu + mod_ + modu
    real_v = V([("main", c, 1) for c in (DV_DIV, DV_DIVU, DV_MOD, DV_MODU)])
    for msb, neg in ((DV_BMSB, DV_BNEG), (DV_RMSB, DV_RNEG), (DV_CMSB, DV_CNEG)):
        ch.assert_zero(M(msb) * (div + mod_) - M(neg))
    mul_op = V([("main", DV_DIV, OP_MULT), ("main", DV_MOD, OP_MULT), ("main", DV_DIVU, OP_MULTU),
                ("main", DV_MODU, OP_MULTU)])
    ctq = [_m(DV_CTQ + i) for i in range(8)]
    vals = [ZERO, ZERO, V.const(A.UNUSED_PC), V.const(A.UNUSED_PC + 4), V.const(A.UNUSED_PC + 8), ZERO, mul_op]
    vals += ctq[:4] + _vword(DV_Q) + _vword(DV_C) + ctq[4:] + [ZERO, ZERO, ZERO, ZERO, V.const(1)]
    ch.sends.append(Lookup(vals, real_v, KIND_INSTRUCTION))  # send_alu_with_hi(MULT/MULTU, ...)
    _is_equal_word(ch, w(DV_B), [0, 0, 0, 0x80], DV_OVF_B, is_real)
    _is_equal_word(ch, w(DV_C), [0xFF] * 4, DV_OVF_C, is_real)
    ch.assert_zero(M(DV_OVF) - M(DV_OVF_B + 10) * M(DV_OVF_C + 10) * (div + mod_))
    carry = [M(DV_CARRY + i) for i in range(8)]
    e = []
    for i in range(8):
        x = M(DV_CTQ + i) + (M(DV_R + i) if i < 4 else M(DV_RNEG) * 255) - carry[i] * 256
        e.append(x + carry[i - 1] if i > 0 else x)
    ovf, bneg = M(DV_OVF), M(DV_BNEG)
    for i in range(8):
        if i < 4:
            ch.assert_zero(M(DV_B + i) - e[i])
        else:
            ch.assert_zero((1 - ovf) * bneg * (e[i] - 255))
            ch.assert_zero((1 - ovf) * (1 - bneg) * e[i])
            ch.assert_zero(ovf * e[i])
    rneg, cneg = M(DV_RNEG), M(DV_CNEG)
    rem_sum = M(DV_R) + M(DV_R + 1) + M(DV_R + 2) + M(DV_R + 3)
    ch.assert_zero(rneg * (bneg - 1))
    ch.assert_zero(rem_sum * (1 - rneg) * bneg)
    _is_zero_word(ch, w(DV_C), DV_IS_C0, is_real)
    c0 = M(DV_IS_C0 + 10)
    for i in range(4):
        ch.assert_zero(c0 * (M(DV_Q + i) - 255))
    for i in range(4):
        ch.assert_zero((1 - cneg) * (M(DV_C + i) - M(DV_ABS_C + i)))
        ch.assert_zero((1 - rneg) * (M(DV_R + i) - M(DV_ABS_R + i)))
    _send_alu(ch, A.OP_ADD, [ZERO] * 4, _vword(DV_C), _vword(DV_ABS_C), _m(DV_CNEG))
    _send_alu(ch, A.OP_ADD, [ZERO] * 4, _vword(DV_R), _vword(DV_ABS_R), _m(DV_RNEG))
    mx = [c0 * 1 + (1 - c0) * M(DV_ABS_C)] + [(1 - c0) * M(DV_ABS_C + i) for i in (1, 2, 3)]
    for i in range(4):
        ch.assert_zero(is_real * (M(DV_MAXC + i) - mx[i]))
    ch.assert_zero((1 - c0) * is_real - M(DV_RCM))
    _send_alu(ch, A.OP_SLTU, [V.const(1), ZERO, ZERO, ZERO], _vword(DV_ABS_R), _vword(DV_MAXC), _m(DV_RCM))
    for msb, byte in ((DV_BMSB, DV_B + 3), (DV_CMSB, DV_C + 3), (DV_RMSB, DV_R + 3)):
        ch.sends.append(Lookup([V.const(A.B_MSB), _m(msb), ZERO, _m(byte), ZERO], real_v, KIND_BYTE))
    for base in (DV_Q, DV_R):
        for k in (0, 2):
            ch.sends.append(Lookup([V.const(A.B_U8RANGE), ZERO, ZERO, _m(base + k), _m(base + k + 1)], real_v,
                                   KIND_BYTE))
    for i in range(8):
        _assert_bool(ch, carry[i])
    for k in range(0, 8, 2):
        ch.sends.append(Lookup([V.const(A.B_U8RANGE), ZERO, ZERO, _m(DV_CTQ + k), _m(DV_CTQ + k + 1)], real_v,
                               KIND_BYTE))
    for col in (DV_DIV, DV_DIVU, DV_MOD, DV_MODU, DV_OVF, DV_BMSB, DV_RMSB, DV_CMSB, DV_BNEG, DV_RNEG, DV_CNEG):
        _assert_bool(ch, M(col))
    ch.assert_zero(is_real * (1 - (divu + div + mod_ + modu)))
    opcode = V([("main", DV_DIVU, OP_DIVU), ("main", DV_DIV, OP_DIV), ("main", DV_MOD, OP_MOD),
                ("main", DV_MODU, OP_MODU)])
    npc4 = V([("main", DV_NPC, 1)], 4)
    ins = [_m(DV_SHARD), _m(DV_CLK), _m(DV_PC), _m(DV_NPC), npc4, ZERO, opcode] + _vword(DV_Q) + _vword(DV_B)
    ins += _vword(DV_C) + _vword(DV_R) + [ZERO, ZERO, V.const(1), ZERO, V.const(1)]
    ch.receives.append(Lookup(ins, V([("main", DV_DIV, 1), ("main", DV_DIVU, 1)]), KIND_INSTRUCTION))
    ins = [ZERO, ZERO, _m(DV_PC), _m(DV_NPC), npc4, ZERO, opcode] + _vword(DV_R) + _vword(DV_B) + _vword(DV_C)
    ins += [ZERO] * 4 + [ZERO, ZERO, ZERO, ZERO, V.const(1)]
    ch.receives.append(Lookup(ins, V([("main", DV_MOD, 1), ("main", DV_MODU, 1)]), KIND_INSTRUCTION))
    _eval_memory_access(ch, DV_HI_ACC + 4, DV_HI_ACC, POS_HI, V.const(REG_HI), div + divu,
                        V([("main", DV_DIV, 1), ("main", DV_DIVU, 1)]), shard_col=DV_SHARD,
                        clk_terms=((DV_CLK, 1),))
    for i in range(4):
        ch.assert_zero((div + divu) * (M(DV_R + i) - M(DV_HI_ACC + 4 + ACC_VALUE + i)))
    return ch


def _izw_cols(words: np.ndarray) -> np.ndarray:
    """IsZeroWordOperation::populate_from_field_element over rows of 4 field elements."""
    n = len(words)
    out = np.zeros((n, IZW_WIDTH), np.uint32)
    x = words.astype(np.int64) % P
    inv = A.inv_mod_p(x).reshape(n, 4)
    z = (x == 0).astype(np.uint32)
    out[:, 0:8:2] = inv
    out[:, 1:8:2] = z
    out[:, 8] = z[:, 0] * z[:, 1]
    out[:, 9] = z[:, 2] * z[:, 3]
    out[:, 10] = out[:, 8] * out[:, 9]
    return out


def _qr(op, b, c):
    """get_quotient_and_remainder (executor/src/utils.rs:33-43)."""
    if c == 0:
        return M32, b
    if op in (OP_DIV, OP_MOD):
        sb, sc = _s32(b), _s32(c)
        if sb == -(1 << 31) and sc == -1:
            return b, 0  # wrapping_div / wrapping_rem
        q = abs(sb) // abs(sc) * (1 if (sb < 0) == (sc < 0) else -1)
        return q & M32, (sb - q * sc) & M32
    return b // c, b % c


def _divrem_trace(divs, shard, byte_lookup):
    """DivRemChip::generate_trace (alu/divrem/mod.rs).  divs: (op, b, c, pc, npc, clk, prev_hi, prev_shard,
    prev_clk) in execution order; clk < 0 for MOD/MODU (no HI record)."""
    E = np.asarray(divs, np.int64).reshape(-1, 9)
    n = len(E)
    t = np.zeros((A._pow2(n), DV_WIDTH), np.uint32)
    op, b, c, pc, npc, clk = (E[:, j] for j in range(6))
    qr = np.asarray([_qr(int(o), int(x), int(y)) for o, x, y in zip(op, b, c)], np.int64).reshape(n, 2)
    q, r = qr[:, 0], qr[:, 1]
    signed = np.isin(op, (OP_DIV, OP_MOD))
    u = lambda v: v.astype(np.uint32)
    t[:n, DV_PC], t[:n, DV_NPC] = pc, npc
    for base, v in ((DV_B, b), (DV_C, c), (DV_Q, q), (DV_R, r)):
        t[:n, base:base + 4] = A._bytes(u(v))
    for col, code in ((DV_DIV, OP_DIV), (DV_DIVU, OP_DIVU), (DV_MOD, OP_MOD), (DV_MODU, OP_MODU)):
        t[:n, col] = op == code
    t[:n, DV_IS_C0:DV_IS_C0 + IZW_WIDTH] = _izw_cols(A._bytes(u(c)))
    diff = lambda x, k: A._bytes(u(x)).astype(np.int64) - np.asarray(list(k), np.int64)[None, :]
    t[:n, DV_OVF_B:DV_OVF_B + IZW_WIDTH] = _izw_cols(diff(b, (0, 0, 0, 0x80)))
    t[:n, DV_OVF_C:DV_OVF_C + IZW_WIDTH] = _izw_cols(diff(c, (255, 255, 255, 255)))
    bmsb, cmsb, rmsb = b >> 31, c >> 31, r >> 31
    t[:n, DV_BMSB], t[:n, DV_CMSB], t[:n, DV_RMSB] = bmsb, cmsb, rmsb
    t[:n, DV_BNEG], t[:n, DV_CNEG], t[:n, DV_RNEG] = bmsb & signed, cmsb & signed, rmsb & signed
    t[:n, DV_OVF] = signed & (b == 0x80000000) & (c == M32)
    sabs = lambda v: np.abs(u(v).view(np.int32).astype(np.int64))
    abs_r = np.where(signed, sabs(r), r)
    abs_c = np.where(signed, sabs(c), c)
    t[:n, DV_ABS_R:DV_ABS_R + 4] = A._bytes(u(abs_r))
    t[:n, DV_ABS_C:DV_ABS_C + 4] = A._bytes(u(abs_c))
    t[:n, DV_MAXC:DV_MAXC + 4] = A._bytes(u(np.maximum(1, abs_c)))
    t[:n, DV_RCM] = c != 0
    s32 = lambda v: u(v).view(np.int32).astype(object)
    ctq = np.asarray([(int(qq) * int(cc)) & ((1 << 64) - 1) for qq, cc in
                      zip(np.where(signed, s32(q), q.astype(object)), np.where(signed, s32(c), c.astype(object)))],
                     np.uint64)
    ctq_b = np.stack([(ctq >> np.uint64(8 * i)) & np.uint64(0xFF) for i in range(8)], axis=1).astype(np.int64)
    r64 = np.where(signed, r | np.where(rmsb == 1, 0xFFFFFFFF00000000, 0), r).astype(np.uint64)
    r_b = np.stack([(r64 >> np.uint64(8 * i)) & np.uint64(0xFF) for i in range(8)], axis=1).astype(np.int64)
    carry = np.zeros((n, 8), np.int64)
    for i in range(8):
        x = ctq_b[:, i] + r_b[:, i] + (carry[:, i - 1] if i else 0)
        carry[:, i] = x >> 8
    t[:n, DV_CTQ:DV_CTQ + 8] = ctq_b
    t[:n, DV_CARRY:DV_CARRY + 8] = carry
    hrr = clk >= 0
    t[:n, DV_SHARD] = np.where(hrr, shard, 0)
    t[:n, DV_CLK] = np.where(hrr, clk, 0)
    t[:n, DV_HI_ACC:DV_HI_ACC + 4] = np.where(hrr[:, None], A._bytes(u(E[:, 6])), 0)
    _access_cols(t, np.arange(n), DV_HI_ACC + 4, u(np.where(hrr, r, 0)), E[:, 7:9], shard,
                 np.where(hrr, clk + POS_HI, 0), hrr, byte_lookup)
    for v in (b, c, r):
        byte_lookup(A.B_MSB, A._bytes(u(v))[:, 3], np.zeros(n, np.int64))
    for v in (q, r):
        wb = A._bytes(u(v))
        byte_lookup(A.B_U8RANGE, wb[:, 0], wb[:, 1])
        byte_lookup(A.B_U8RANGE, wb[:, 2], wb[:, 3])
    for k in range(0, 8, 2):
        byte_lookup(A.B_U8RANGE, ctq_b[:, k], ctq_b[:, k + 1])
    return t, q, r, abs_c, abs_r, ctq


# ---------------------------------------------------------------- MovCond (misc/mov_cond)
OP_MEQ, OP_MNE, OP_WSBH = 50, 51, 52  # MOVZ, MOVN, WSBH (executor/src/opcode.rs:70-72)
MOVCOND_OPS = (OP_MEQ, OP_MNE, OP_WSBH)
# MovCondCols (misc/mov_cond/mod.rs)
MC_PC, MC_NPC, MC_A, MC_PREV_A, MC_B, MC_C, MC_C0, MC_MNE, MC_MEQ, MC_WSBH = 0, 1, 2, 6, 10, 14, 18, 29, 30, 31
MC_WIDTH = 32


def movcond_chip() -> ChipDesc:
    """MovCondChip::eval + eval_wsbh (misc/mov_cond/mod.rs), constraints and lookups in its order."""
    ch = ChipDesc("MovCond", prep_width=0, main_width=MC_WIDTH, local_only=True)
    M = main
    mne, meq, wsbh = M(MC_MNE), M(MC_MEQ), M(MC_WSBH)
    is_real = mne + meq + wsbh
    opcode = V([("main", MC_WSBH, OP_WSBH), ("main", MC_MEQ, OP_MEQ), ("main", MC_MNE, OP_MNE)])
    ins = [ZERO, ZERO, _m(MC_PC), _m(MC_NPC), V([("main", MC_NPC, 1)], 4), ZERO, opcode]
    ins += _vword(MC_A) + _vword(MC_B) + _vword(MC_C) + _vword(MC_PREV_A)
    ins += [ZERO, V([("main", MC_MNE, 1), ("main", MC_MEQ, 1)]), ZERO, ZERO, V.const(1)]
    ch.receives.append(Lookup(ins, V([("main", c, 1) for c in (MC_MNE, MC_MEQ, MC_WSBH)]), KIND_INSTRUCTION))
    _is_zero_word(ch, [M(MC_C + i) for i in range(4)], MC_C0, is_real)
    r = M(MC_C0 + 10)
    for cond, src in ((meq * r, MC_B), (meq * (1 - r), MC_PREV_A), (mne * (1 - r), MC_B), (mne * r, MC_PREV_A)):
        for i in range(4):
            ch.assert_zero(cond * (M(MC_A + i) - M(src + i)))
    for i, j in ((0, 1), (1, 0), (2, 3), (3, 2)):
        ch.assert_zero(wsbh * (M(MC_A + i) - M(MC_B + j)))
    for x in (mne, meq, wsbh, is_real):
        _assert_bool(ch, x)
    return ch


def _movcond_trace(movs):
    """MovCondChip::event_to_row (misc/mov_cond/mod.rs): (pc, npc, op, a, b, c, prev_a)."""
    E = np.asarray(movs, np.int64).reshape(-1, 7)
    n = len(E)
    t = np.zeros((A._pow2(n), MC_WIDTH), np.uint32)
    t[:n, MC_PC], t[:n, MC_NPC] = E[:, 0], E[:, 1]
    for base, j in ((MC_A, 3), (MC_B, 4), (MC_C, 5), (MC_PREV_A, 6)):
        t[:n, base:base + 4] = A._bytes(E[:, j].astype(np.uint32))
    t[:n, MC_C0:MC_C0 + IZW_WIDTH] = _izw_cols(A._bytes(E[:, 5].astype(np.uint32)))
    t[:n, MC_MEQ], t[:n, MC_MNE], t[:n, MC_WSBH] = E[:, 2] == OP_MEQ, E[:, 2] == OP_MNE, E[:, 2] == OP_WSBH
    return t


# ---------------------------------------------------------------- MemoryInstrs (memory/instructions)
OP_LB, OP_LBU, OP_LH, OP_LHU, OP_LW, OP_LWL, OP_LWR, OP_LL = range(31, 39)  # executor/src/opcode.rs:50-63
OP_SB, OP_SH, OP_SW, OP_SWL, OP_SWR, OP_SC = range(39, 45)
LOAD_OPS, STORE_OPS = tuple(range(31, 39)), tuple(range(39, 45))
MEM_OPS = LOAD_OPS + STORE_OPS
REF_NUM_REGISTERS = 36  # executor/src/register.rs:3: data addresses start above the register file
DATA_BASE = 0x00010000
# MemoryInstructionsColumns (memory/instructions/columns.rs:15-103); selectors in opcode order
MI_PC, MI_NPC, MI_SHARD, MI_CLK, MI_A, MI_B, MI_C, MI_SEL = 0, 1, 2, 3, 4, 8, 12, 16
MI_ADDR, MI_ALIGNED, MI_LS2, MI_L1, MI_L2, MI_L3, MI_ADDR_RC, MI_ACC = 30, 34, 35, 36, 37, 38, 39, 53
MI_PREV_A, MI_UMV, MI_MSBIT, MI_MSBYTE, MI_NEG, MI_MSBZ = 66, 70, 74, 75, 76, 77
MI_WIDTH = 79


def memory_instructions_chip() -> ChipDesc:
    """MemoryInstructionsChip::eval (memory/instructions/air.rs:23-519): address = b + c through the ADD
    table, word range and register-file checks, offset flags, the memory access at the aligned address,
    load extraction (LB/LBU/LH/LHU/LW/LWL/LWR/LL with the SUB that sign-extends) and store merging
    (SB/SH/SW/SWL/SWR/SC), constraints and lookups in the reference's order."""
    ch = ChipDesc("MemoryInstrs", prep_width=0, main_width=MI_WIDTH, local_only=True)
    M = main
    sel = [M(MI_SEL + k) for k in range(14)]
    lb, lbu, lh, lhu, lw, lwl, lwr, ll, sb, sh, sw, swl, swr, sc = sel
    is_real = sum(sel[1:], sel[0])
    real_v = V([("main", MI_SEL + k, 1) for k in range(14)])
    for x in sel:
        _assert_bool(ch, x)
    _assert_bool(ch, is_real)
    # eval_memory_address_and_access (:129-225)
    _send_alu(ch, A.OP_ADD, _vword(MI_ADDR), _vword(MI_B), _vword(MI_C), real_v)
    _word_range_check(ch, MI_ADDR, MI_ADDR_RC, is_real)
    ch.sends.append(Lookup([V.const(A.B_U8RANGE), ZERO, ZERO, _m(MI_ADDR + 1), _m(MI_ADDR + 2)], real_v, KIND_BYTE))
    ch.sends.append(Lookup([V.const(A.B_LTU), V.const(1), ZERO, V.const(REF_NUM_REGISTERS - 1), _m(MI_ADDR)],
                           _m(MI_MSBZ + 1), KIND_BYTE))
    res = M(MI_MSBZ + 1)
    ch.assert_zero(res * (is_real - 1))
    x = M(MI_ADDR + 1) + M(MI_ADDR + 2) + M(MI_ADDR + 3)
    ch.assert_zero(is_real * ((1 - M(MI_MSBZ) * x) - res))  # IsZeroOperation (operations/is_zero.rs:47-66)
    _assert_bool(ch, res, is_real)
    ch.assert_zero(is_real * res * x)
    l1, l2, l3, two = M(MI_L1), M(MI_L2), M(MI_L3), M(MI_LS2)
    oz = 1 - l1 - l2 - l3
    for f in (l1, l2, l3, oz):  # eval_offset_value_flags (:496-519)
        _assert_bool(ch, f)
    ch.assert_zero(oz * two)
    ch.assert_zero(l1 * (two - 1))
    ch.assert_zero(l2 * (two - 2))
    ch.assert_zero(l3 * (two - 3))
    red = sum((M(MI_ADDR + i) * (1 << (8 * i)) for i in range(1, 4)), M(MI_ADDR))
    ch.assert_zero(is_real * ((M(MI_ALIGNED) + two) - red))
    ch.sends.append(Lookup([V.const(A.B_AND), _m(MI_LS2), ZERO, _m(MI_ADDR), V.const(3)], real_v, KIND_BYTE))
    _eval_memory_access(ch, MI_ACC + 4, MI_ACC, 0, _m(MI_ALIGNED), is_real, real_v, shard_col=MI_SHARD,
                        clk_terms=((MI_CLK, 1),))
    mem = [M(MI_ACC + 4 + i) for i in range(4)]
    pm = [M(MI_ACC + i) for i in range(4)]
    loads = lb + lbu + lh + lhu + lw + lwl + lwr + ll
    for i in range(4):
        ch.assert_zero(loads * (mem[i] - pm[i]))
    # eval_memory_load / eval_unsigned_mem_value (:228-284, :402-493)
    umv = [M(MI_UMV + i) for i in range(4)]
    pa = [M(MI_PREV_A + i) for i in range(4)]
    a = [M(MI_A + i) for i in range(4)]
    byte_value = [mem[0] * oz + mem[1] * l1 + mem[2] * l2 + mem[3] * l3, 0, 0, 0]
    for i in range(4):
        ch.assert_zero((lb + lbu) * (byte_value[i] - umv[i]))
    ch.assert_zero((lh + lhu) * (l1 + l3))
    ch.assert_zero(lw * (oz - 1))
    half = [oz * mem[0] + l2 * mem[2], oz * mem[1] + l2 * mem[3], 0, 0]
    for i in range(4):
        ch.assert_zero((lh + lhu) * (half[i] - umv[i]))
    for i in range(4):
        ch.assert_zero(lw * (mem[i] - umv[i]))
    lwr_v = [mem[0] * oz + mem[1] * l1 + mem[2] * l2 + mem[3] * l3,
             mem[1] * oz + mem[2] * l1 + mem[3] * l2 + pa[1] * l3,
             mem[2] * oz + mem[3] * l1 + pa[2] * (1 - l1 - oz),
             mem[3] * oz + pa[3] * (1 - oz)]
    for i in range(4):
        ch.assert_zero(lwr * (umv[i] - lwr_v[i]))
    lwl_v = [mem[0] * l3 + pa[0] * (1 - l3),
             mem[1] * l3 + mem[0] * l2 + pa[1] * l1 + pa[1] * oz,
             mem[2] * l3 + mem[1] * l2 + mem[0] * l1 + pa[2] * oz,
             mem[3] * l3 + mem[2] * l2 + mem[1] * l1 + mem[0] * oz]
    for i in range(4):
        ch.assert_zero(lwl * (umv[i] - lwl_v[i]))
    for i in range(4):
        ch.assert_zero(ll * (umv[i] - mem[i]))
    ch.assert_zero(ll * (oz - 1))
    neg = M(MI_NEG)
    ch.assert_zero(neg - (lb + lh) * M(MI_MSBIT))
    ch.sends.append(Lookup([V.const(A.B_MSB), _m(MI_MSBIT), ZERO, _m(MI_MSBYTE), ZERO],
                           V([("main", MI_SEL + 0, 1), ("main", MI_SEL + 2, 1)]), KIND_BYTE))
    ch.assert_zero(M(MI_MSBYTE) - (lb * umv[0] + lh * umv[1]))
    _send_alu(ch, A.OP_SUB, _vword(MI_A), _vword(MI_UMV), [ZERO, _m(MI_SEL + 0), _m(MI_SEL + 2), ZERO], _m(MI_NEG))
    pos = (lb + lh - neg) + lbu + lhu + lw + ll + lwl + lwr
    for i in range(4):
        ch.assert_zero(pos * (umv[i] - a[i]))
    # eval_memory_store (:287-398)
    sb_v = [a[0] * oz + (1 - oz) * pm[0], a[0] * l1 + (1 - l1) * pm[1], a[0] * l2 + (1 - l2) * pm[2],
            a[0] * l3 + (1 - l3) * pm[3]]
    for i in range(4):
        ch.assert_zero(sb * (mem[i] - sb_v[i]))
    ch.assert_zero(sh * (l1 + l3))
    ch.assert_zero(sw * (oz - 1))
    sh_v = [a[0] * oz + (1 - oz) * pm[0], a[1] * oz + (1 - oz) * pm[1], a[0] * l2 + (1 - l2) * pm[2],
            a[1] * l2 + (1 - l2) * pm[3]]
    for i in range(4):
        ch.assert_zero(sh * (mem[i] - sh_v[i]))
    for i in range(4):
        ch.assert_zero(sw * (mem[i] - a[i]))
    swl_v = [a[3] * oz + a[2] * l1 + a[1] * l2 + a[0] * l3,
             pm[1] * oz + a[3] * l1 + a[2] * l2 + a[1] * l3,
             pm[2] * (oz + l1) + a[3] * l2 + a[2] * l3,
             pm[3] * (1 - l3) + a[3] * l3]
    for i in range(4):
        ch.assert_zero(swl * (mem[i] - swl_v[i]))
    swr_v = [a[0] * oz + pm[0] * (1 - oz),
             a[1] * oz + a[0] * l1 + pm[1] * (l2 + l3),
             a[2] * oz + a[1] * l1 + a[0] * l2 + pm[2] * l3,
             a[3] * oz + a[2] * l1 + a[1] * l2 + a[0] * l3]
    for i in range(4):
        ch.assert_zero(swr * (mem[i] - swr_v[i]))
    ch.assert_zero(sc * (oz - 1))
    for i in range(4):
        ch.assert_zero(sc * (pa[i] - mem[i]))
    ch.assert_zero(sc * (a[0] - 1))
    for i in (1, 2, 3):
        ch.assert_zero(sc * a[i])
    opcode = V([("main", MI_SEL + k, 31 + k) for k in range(14)])
    ins = [_m(MI_SHARD), _m(MI_CLK), _m(MI_PC), _m(MI_NPC), V([("main", MI_NPC, 1)], 4), ZERO, opcode]
    ins += _vword(MI_A) + _vword(MI_B) + _vword(MI_C) + _vword(MI_PREV_A)
    ins += [V([("main", MI_SEL + k, 1) for k in range(8, 13)]), V.const(1), V.const(1), ZERO, V.const(1)]
    ch.receives.append(Lookup(ins, real_v, KIND_INSTRUCTION))
    return ch


def _load_value(op, mem, two, rt):
    """execute_load's value (executor/src/executor.rs:1953-2005); `two` = addr & 3."""
    if op in (OP_LB, OP_LBU):
        v = (mem >> (8 * two)) & 0xFF
        return (v - 256) & M32 if op == OP_LB and v >> 7 else v
    if op in (OP_LH, OP_LHU):
        v = (mem >> (8 * (two & 2))) & 0xFFFF
        return (v - 65536) & M32 if op == OP_LH and v >> 15 else v
    if op == OP_LWL:
        sh = 24 - 8 * two
        return (rt & ~((M32 << sh) & M32) & M32) | ((mem << sh) & M32)
    if op == OP_LWR:
        sh = 8 * two
        return (rt & ~(M32 >> sh) & M32) | (mem >> sh)
    return mem  # LW, LL


def _store_value(op, mem, two, rt):
    """execute_store's merged word (executor/src/executor.rs:2029-2079)."""
    if op == OP_SB:
        return (mem & (M32 ^ (0xFF << (8 * two)))) | ((rt & 0xFF) << (8 * two))
    if op == OP_SH:
        s = 8 * (two & 2)
        return (mem & (M32 ^ (0xFFFF << s))) | ((rt & 0xFFFF) << s)
    if op == OP_SWL:
        sh = 24 - 8 * two
        return (mem & ~(M32 >> sh) & M32) | (rt >> sh)
    if op == OP_SWR:
        sh = 8 * two
        return (mem & ~((M32 << sh) & M32) & M32) | ((rt << sh) & M32)
    return rt  # SW, SC


def _mem_instr_trace(mevs, shard, byte_lookup):
    """MemoryInstructionsChip::event_to_row (memory/instructions/trace.rs:88-251).  mevs: (pc, npc, op, a,
    b, c, prev_a, clk, addr, prev_mem, mem, mem_prev_shard, mem_prev_clk)."""
    E = np.asarray(mevs, np.int64).reshape(-1, 13)
    n = len(E)
    t = np.zeros((A._pow2(n), MI_WIDTH), np.uint32)
    u = lambda v: v.astype(np.uint32)
    pc, npc, op, a, b, c, prev_a, clk, addr, pmem, nmem = (E[:, j] for j in range(11))
    t[:n, MI_PC], t[:n, MI_NPC], t[:n, MI_SHARD], t[:n, MI_CLK] = pc, npc, shard, clk
    for base, v in ((MI_A, a), (MI_B, b), (MI_C, c), (MI_PREV_A, prev_a), (MI_ADDR, addr), (MI_ACC, pmem)):
        t[:n, base:base + 4] = A._bytes(u(v))
    for k in range(14):
        t[:n, MI_SEL + k] = op == 31 + k
    two = addr & 3
    t[:n, MI_ALIGNED] = addr - two
    t[:n, MI_LS2] = two
    t[:n, MI_L1], t[:n, MI_L2], t[:n, MI_L3] = two == 1, two == 2, two == 3
    t[:n, MI_ADDR_RC:MI_ADDR_RC + RC_WIDTH] = _range_checker_cols(u(addr))
    _access_cols(t, np.arange(n), MI_ACC + 4, u(nmem), E[:, 11:13], shard, clk, np.ones(n, bool), byte_lookup)
    ab = A._bytes(u(addr)).astype(np.int64)
    byte_lookup(A.B_AND, ab[:, 0], np.full(n, 3))
    ld = np.isin(op, LOAD_OPS)
    mb = A._bytes(u(pmem)).astype(np.int64)
    byte_ = mb[np.arange(n), two]
    half = np.where((two >> 1) & 1, pmem >> 16, pmem & 0xFFFF)
    umv = np.select([np.isin(op, (OP_LB, OP_LBU)), np.isin(op, (OP_LH, OP_LHU)), np.isin(op, (OP_LWL, OP_LWR))],
                    [byte_, half, a], pmem)
    umv = np.where(ld, umv, 0)
    t[:n, MI_UMV:MI_UMV + 4] = A._bytes(u(umv))
    signed = np.isin(op, (OP_LB, OP_LH))
    msbyte = np.where(op == OP_LB, umv & 0xFF, (umv >> 8) & 0xFF)
    msbit = msbyte >> 7
    t[:n, MI_MSBYTE] = np.where(signed, msbyte, 0)
    t[:n, MI_MSBIT] = np.where(signed, msbit, 0)
    t[:n, MI_NEG] = signed & (msbit == 1)
    byte_lookup(A.B_MSB, msbyte[signed], np.zeros(int(signed.sum()), np.int64))
    byte_lookup(A.B_U8RANGE, ab[:, 1], ab[:, 2])
    s = ab[:, 1] + ab[:, 2] + ab[:, 3]
    t[:n, MI_MSBZ] = A.inv_mod_p(s)
    t[:n, MI_MSBZ + 1] = s == 0
    z = s == 0
    byte_lookup(A.B_LTU, np.full(int(z.sum()), REF_NUM_REGISTERS - 1), ab[z, 0])
    return t


# ---------------------------------------------------------------- MiscInstrs (misc/others)
OP_INS, OP_MADDU, OP_MSUBU, OP_MADD, OP_MSUB = 45, 46, 47, 48, 49  # executor/src/opcode.rs:65-75
OP_EXT, OP_TEQ, OP_SEXT = 53, 54, 55
MISC_OPS = (OP_SEXT, OP_INS, OP_EXT, OP_MADDU, OP_MSUBU, OP_MADD, OP_MSUB, OP_TEQ)  # column order
MADDSUB_OPS = (OP_MADDU, OP_MSUBU, OP_MADD, OP_MSUB)
# MiscInstrColumns (misc/others/columns/mod.rs); misc_specific_columns is a union whose widest view is
# MaddsubCols: mul_lo, mul_hi, AddDoubleOperation (value, value_hi, carry[7]), src2_hi, src2_lo, op_hi_access
MS_SHARD, MS_CLK, MS_PC, MS_NPC, MS_A, MS_PREV_A, MS_B, MS_C, MS_SPEC = 0, 1, 2, 3, 4, 8, 12, 16, 20
MS_SEL = 64  # is_sext, is_ins, is_ext, is_maddu, is_msubu, is_madd, is_msub, is_teq
MS_WIDTH = 72
_MD_LO, _MD_HI, _MD_VAL, _MD_VALHI, _MD_CARRY, _MD_S2HI, _MD_S2LO, _MD_HIACC = 0, 4, 8, 12, 16, 23, 27, 31


def _add_double(ch, a, a_hi, b, b_hi, val, val_hi, carry, is_real, real_v, byte_words):
    """AddDoubleOperation::eval (operations/add_double.rs): 64-bit byte-wise add with 7 carries."""
    M = main
    ov = [a[0] + b[0] - val[0]] + [a[j] + b[j] - val[j] + carry[j - 1] for j in (1, 2, 3)]
    for j in range(4):
        ch.assert_zero(is_real * (ov[j] * (ov[j] - 256)))
    for j in range(4):
        ch.assert_zero(is_real * (carry[j] * (ov[j] - 256)))
    for j in range(4):
        ch.assert_zero(is_real * ((carry[j] - 1) * ov[j]))
    ovh = [a_hi[j] + b_hi[j] - val_hi[j] + carry[3 + j] for j in range(4)]
    for j in range(4):
        ch.assert_zero(is_real * (ovh[j] * (ovh[j] - 256)))
    for j in range(3):
        ch.assert_zero(is_real * (carry[4 + j] * (ovh[j] - 256)))
    for j in range(3):
        ch.assert_zero(is_real * ((carry[4 + j] - 1) * ovh[j]))
    for j in range(7):
        _assert_bool(ch, carry[j], is_real)
    _assert_bool(ch, is_real, is_real)
    for base in byte_words:  # slice_range_check_u8 of a, a_hi, b, b_hi, value, value_hi
        for k in (0, 2):
            ch.sends.append(Lookup([V.const(A.B_U8RANGE), ZERO, ZERO, _m(base + k), _m(base + k + 1)], real_v,
                                   KIND_BYTE))


def _shift_word(*terms):
    """Word([const + sum(weight * col), 0, 0, 0]) as VirtualPairCols: terms = (const, [(col, weight)])."""
    const, cols = terms
    return [V([("main", c, w % P) for c, w in cols], const), ZERO, ZERO, ZERO]


def misc_instructions_chip() -> ChipDesc:
    """MiscInstrsChip::eval with eval_ext / eval_ins / eval_maddsub / eval_sext (misc/others/air.rs:24-418):
    SEXT (SEB/SEH), EXT, INS, MADDU/MSUBU/MADD/MSUB and TEQ, constraints and lookups in its order."""
    ch = ChipDesc("MiscInstrs", prep_width=0, main_width=MS_WIDTH)
    M = main
    sext, ins, ext, maddu, msubu, madd, msub, teq = (M(MS_SEL + k) for k in range(8))
    is_real = sext + ins + ext + maddu + msubu + madd + msub + teq
    for k in range(8):
        _assert_bool(ch, M(MS_SEL + k))
    _assert_bool(ch, is_real)
    sel = lambda *ks, const=0: V([("main", MS_SEL + k, 1) for k in ks], const)
    opcode = V([("main", MS_SEL + k, op) for k, op in enumerate(MISC_OPS)])
    npc4 = V([("main", MS_NPC, 1)], 4)
    body = [opcode] + _vword(MS_A) + _vword(MS_B) + _vword(MS_C) + _vword(MS_PREV_A)
    ch.receives.append(Lookup([_m(MS_SHARD), _m(MS_CLK), _m(MS_PC), _m(MS_NPC), npc4, ZERO] + body +
                              [ZERO, sel(3, 4, 5, 6, 1), sel(3, 4, 5, 6), ZERO, V.const(1)], sel(3, 4, 5, 6),
                              KIND_INSTRUCTION))
    ch.receives.append(Lookup([ZERO, ZERO, _m(MS_PC), _m(MS_NPC), npc4, ZERO] + body +
                              [ZERO, sel(3, 4, 5, 6, 1), ZERO, ZERO, V.const(1)], sel(0, 7, 2, 1), KIND_INSTRUCTION))
    S = MS_SPEC
    red = lambda base: sum((M(base + i) * (1 << (8 * i)) for i in range(1, 4)), M(base))
    # eval_ext: ext view = lsb, msbd, sll_val
    lsb, msbd = S, S + 1
    _send_alu(ch, A.OP_SLL, _vword(S + 2), _vword(MS_B), _shift_word(31, [(lsb, -1), (msbd, -1)]), _m(MS_SEL + 2))
    _send_alu(ch, A.OP_SRL, _vword(MS_A), _vword(S + 2), _shift_word(31, [(msbd, -1)]), _m(MS_SEL + 2))
    ch.assert_zero(ext * (red(MS_C) - (M(lsb) + M(msbd) * 32)))
    ch.sends.append(Lookup([V.const(A.B_U8RANGE), ZERO, ZERO, _m(lsb), _m(msbd)], _m(MS_SEL + 2), KIND_BYTE))
    ch.sends.append(Lookup([V.const(A.B_LTU), V.const(1), ZERO, V([("main", lsb, 1), ("main", msbd, 1)]),
                            V.const(32)], _m(MS_SEL + 2), KIND_BYTE))
    # eval_ins: ins view = lsb, msb, ror_val, srl_val, sll_val, add_val
    lsb, msb, ror, srl, sll, add = S, S + 1, S + 2, S + 6, S + 10, S + 14
    isv = _m(MS_SEL + 1)
    _send_alu(ch, A.OP_ROR, _vword(ror), _vword(MS_PREV_A), _shift_word(0, [(lsb, 1)]), isv)
    _send_alu(ch, A.OP_SRL, _vword(srl), _vword(ror), _shift_word(1, [(msb, 1), (lsb, -1)]), isv)
    _send_alu(ch, A.OP_SLL, _vword(sll), _vword(MS_B), _shift_word(31, [(msb, -1), (lsb, 1)]), isv)
    _send_alu(ch, A.OP_ADD, _vword(add), _vword(srl), _vword(sll), isv)
    _send_alu(ch, A.OP_ROR, _vword(MS_A), _vword(add), _shift_word(31, [(msb, -1)]), isv)
    ch.assert_zero(ins * (red(MS_C) - (M(lsb) + M(msb) * 32)))
    ch.sends.append(Lookup([V.const(A.B_U8RANGE), ZERO, ZERO, _m(lsb), _m(msb)], isv, KIND_BYTE))
    ch.sends.append(Lookup([V.const(A.B_LTU), V.const(1), ZERO, _m(lsb), V([("main", msb, 1)], 1)], isv, KIND_BYTE))
    ch.sends.append(Lookup([V.const(A.B_LTU), V.const(1), ZERO, _m(msb), V.const(32)], isv, KIND_BYTE))
    # eval_maddsub
    md_real = maddu + msubu + madd + msub
    md_v = sel(3, 4, 5, 6)
    is_add, is_sub = maddu + madd, msubu + msub
    mul_op = V([("main", MS_SEL + 5, OP_MULT), ("main", MS_SEL + 6, OP_MULT), ("main", MS_SEL + 3, OP_MULTU),
                ("main", MS_SEL + 4, OP_MULTU)])
    vals = [ZERO, ZERO, V.const(A.UNUSED_PC), V.const(A.UNUSED_PC + 4), V.const(A.UNUSED_PC + 8), ZERO, mul_op]
    vals += _vword(S + _MD_LO) + _vword(MS_B) + _vword(MS_C) + _vword(S + _MD_HI) + [ZERO, ZERO, ZERO, ZERO,
                                                                                       V.const(1)]
    ch.sends.append(Lookup(vals, md_v, KIND_INSTRUCTION))  # send_alu_with_hi(MULT/MULTU, ...)
    hacc = S + _MD_HIACC
    for i in range(4):
        ch.assert_zero(md_real * (M(S + _MD_S2HI + i) - (M(hacc + i) * is_add + M(hacc + 4 + ACC_VALUE + i) * is_sub)))
        ch.assert_zero(md_real * (M(S + _MD_S2LO + i) - (M(MS_PREV_A + i) * is_add + M(MS_A + i) * is_sub)))
    w = lambda base: [M(base + i) for i in range(4)]
    _add_double(ch, w(S + _MD_LO), w(S + _MD_HI), w(S + _MD_S2LO), w(S + _MD_S2HI), w(S + _MD_VAL), w(S + _MD_VALHI),
                [M(S + _MD_CARRY + j) for j in range(7)], md_real, md_v,
                (S + _MD_LO, S + _MD_HI, S + _MD_S2LO, S + _MD_S2HI, S + _MD_VAL, S + _MD_VALHI))
    for i in range(4):
        ch.assert_zero(is_add * (M(MS_A + i) - M(S + _MD_VAL + i)))
    for i in range(4):
        ch.assert_zero(is_add * (M(hacc + 4 + ACC_VALUE + i) - M(S + _MD_VALHI + i)))
    for i in range(4):
        ch.assert_zero(is_sub * (M(MS_PREV_A + i) - M(S + _MD_VAL + i)))
    for i in range(4):
        ch.assert_zero(is_sub * (M(hacc + i) - M(S + _MD_VALHI + i)))
    _eval_memory_access(ch, hacc + 4, hacc, POS_HI, V.const(REG_HI), md_real, md_v, shard_col=MS_SHARD,
                        clk_terms=((MS_CLK, 1),))
    # eval_sext: sext view = most_sig_bit, sig_byte, a_eq_b, is_seb, is_seh
    msbit, sbyte, aeqb, seb, seh = (M(S + k) for k in range(5))
    for i in range(4):
        ch.assert_zero(teq * aeqb * (M(MS_A + i) - M(MS_B + i)))
    ch.assert_zero(teq * aeqb)
    ch.sends.append(Lookup([V.const(A.B_MSB), _m(S), ZERO, _m(S + 1), ZERO], _m(MS_SEL + 0), KIND_BYTE))
    c0 = M(MS_C)
    ch.assert_zero(sext * (c0 * (c0 - 1)))
    ch.assert_zero(sext * seb * c0)
    ch.assert_zero(sext * seh * (c0 - 1))
    ch.assert_zero(sext * seb * (M(MS_B) - sbyte))
    ch.assert_zero(sext * seh * (M(MS_B + 1) - sbyte))
    sign = msbit * 255
    ch.assert_zero(sext * (M(MS_A) - M(MS_B)))
    ch.assert_zero(sext * seb * (M(MS_A + 1) - sign))
    ch.assert_zero(sext * seh * (M(MS_A + 1) - M(MS_B + 1)))
    ch.assert_zero(sext * (M(MS_A + 2) - sign))
    ch.assert_zero(sext * (M(MS_A + 3) - sign))
    ch.assert_zero((ins + ext) * M(MS_C + 2))
    ch.assert_zero((ins + ext) * M(MS_C + 3))
    return ch


def _misc_trace(misc, shard, byte_lookup):
    """MiscInstrsChip::event_to_row + populate_* (misc/others/trace.rs:81-262), vectorised over the rows of
    each opcode group.  misc: (op, a, b, c, prev_a, pc, npc, clk, hi_prev, hi_new, hi_prev_shard, hi_prev_clk)."""
    E = np.asarray(misc, np.int64).reshape(-1, 12)
    n = len(E)
    t = np.zeros((A._pow2(n), MS_WIDTH), np.uint32)
    u64 = lambda v: np.asarray(v, np.int64).astype(np.uint64)
    wb = lambda v: A._bytes(u64(v) & np.uint64(M32))
    S = MS_SPEC
    op, a, b, c, pa = (E[:, j] for j in range(5))
    t[:n, MS_PC], t[:n, MS_NPC] = E[:, 5], E[:, 6]
    for base, v in ((MS_A, a), (MS_B, b), (MS_C, c), (MS_PREV_A, pa)):
        t[:n, base:base + 4] = wb(v)
    col = np.full(64, -1, np.int64)
    col[list(MISC_OPS)] = np.arange(len(MISC_OPS))
    t[np.arange(n), MS_SEL + col[op]] = 1
    # SEXT / TEQ: sext view (most_sig_bit, sig_byte, a_eq_b, is_seb, is_seh)
    r = np.nonzero((op == OP_SEXT) | (op == OP_TEQ))[0]
    if len(r):
        bb, half = b[r], c[r] > 0
        bit = np.where(half, (bb & 0xFFFF) >> 15, (bb & 0xFF) >> 7)
        byte = np.where(half, (bb >> 8) & 0xFF, bb & 0xFF)
        t[r, S], t[r, S + 1], t[r, S + 2] = bit, byte, a[r] == bb
        t[r, S + 3], t[r, S + 4] = ~half, half
        sx = op[r] == OP_SEXT
        byte_lookup(A.B_MSB, byte[sx], np.zeros(int(sx.sum()), np.int64))
    # EXT: ext view (lsb, msbd, sll_val)
    r = np.nonzero(op == OP_EXT)[0]
    if len(r):
        lsb, msbd = c[r] & 31, c[r] >> 5
        t[r, S], t[r, S + 1] = lsb, msbd
        t[r, S + 2:S + 6] = wb(u64(b[r]) << u64(31 - lsb - msbd))
        byte_lookup(A.B_U8RANGE, lsb, msbd)
        byte_lookup(A.B_LTU, lsb + msbd, np.full(len(r), 32))
    # INS: ins view (lsb, msb, ror_val, srl_val, sll_val, add_val); the SRL shift is the field width, which
    # the generator keeps below 32 (a full-width INS cannot satisfy eval_ins: see _execute)
    r = np.nonzero(op == OP_INS)[0]
    if len(r):
        lsb, msb = c[r] & 31, c[r] >> 5
        p = u64(pa[r])
        ror = ((p >> u64(lsb)) | (p << u64(32 - lsb))) & np.uint64(M32)
        srl = ror >> u64(msb - lsb + 1)
        sll = (u64(b[r]) << u64(31 - msb + lsb)) & np.uint64(M32)
        t[r, S], t[r, S + 1] = lsb, msb
        for off, v in ((2, ror), (6, srl), (10, sll), (14, srl + sll)):
            t[r, S + off:S + off + 4] = wb(v)
        byte_lookup(A.B_U8RANGE, lsb, msb)
        byte_lookup(A.B_LTU, lsb, msb + 1)
        byte_lookup(A.B_LTU, msb, np.full(len(r), 32))
    # MADDU / MSUBU / MADD / MSUB: maddsub view (product, 64-bit AddDouble with its 7 carries, HI access)
    r = np.nonzero(np.isin(op, MADDSUB_OPS))[0]
    if len(r):
        o = op[r]
        t[r, MS_SHARD], t[r, MS_CLK] = shard, E[r, 7]
        signed = (o == OP_MADD) | (o == OP_MSUB)
        sb = np.where(b[r] >> 31, b[r] - (1 << 32), b[r])
        sc = np.where(c[r] >> 31, c[r] - (1 << 32), c[r])
        prod = np.where(signed, (sb * sc).astype(np.uint64), u64(b[r]) * u64(c[r]))
        is_add = (o == OP_MADDU) | (o == OP_MADD)
        s2lo = np.where(is_add, pa[r], a[r])
        s2hi = np.where(is_add, E[r, 8], E[r, 9])
        addend = (u64(s2hi) << np.uint64(32)) | u64(s2lo)
        tot = prod + addend  # wraps mod 2^64
        pb = prod[:, None] >> (np.uint64(8) * np.arange(8, dtype=np.uint64))[None, :] & np.uint64(0xFF)
        qb = addend[:, None] >> (np.uint64(8) * np.arange(8, dtype=np.uint64))[None, :] & np.uint64(0xFF)
        cy = np.zeros(len(r), np.uint64)
        for j in range(7):
            cy = ((pb[:, j] + qb[:, j] + cy) > 255).astype(np.uint64)
            t[r, S + _MD_CARRY + j] = cy
        lo32 = lambda v: v & np.uint64(M32)
        hi32 = lambda v: v >> np.uint64(32)
        for off, v in ((_MD_LO, lo32(prod)), (_MD_HI, hi32(prod)), (_MD_VAL, lo32(tot)), (_MD_VALHI, hi32(tot)),
                       (_MD_S2HI, u64(s2hi)), (_MD_S2LO, u64(s2lo)), (_MD_HIACC, u64(E[r, 8]))):
            t[r, S + off:S + off + 4] = wb(v)
        for v in (lo32(prod), hi32(prod), u64(s2lo), u64(s2hi), lo32(tot), hi32(tot)):
            w = wb(v)
            byte_lookup(A.B_U8RANGE, w[:, 0], w[:, 1])
            byte_lookup(A.B_U8RANGE, w[:, 2], w[:, 3])
    md = np.isin(E[:, 0], MADDSUB_OPS)
    if md.any():
        rows = np.nonzero(md)[0]
        _access_cols(t, rows, S + _MD_HIACC + 4, E[rows, 9].astype(np.uint32), E[rows][:, 10:12], shard, E[rows, 7] + POS_HI,
                     np.ones(len(rows), bool), byte_lookup)
    return t


# ---------------------------------------------------------------- Jump (control_flow/jump)
OP_JUMP, OP_JUMPI, OP_JUMPDIRECT = 27, 28, 29  # JR/JALR, J/JAL, BAL (executor/src/opcode.rs:45-47)
JUMP_OPS = (OP_JUMP, OP_JUMPI, OP_JUMPDIRECT)
# JumpColumns (control_flow/jump/columns.rs:9-37)
J_PC, J_NPC, J_NPC_RC, J_NNPC, J_NNPC_RC, J_A, J_B, J_C = 0, 1, 5, 19, 23, 37, 41, 45
J_JUMP, J_JUMPI, J_JDIRECT, J_A_RC = 49, 50, 51, 52
J_WIDTH = 66


def jump_chip() -> ChipDesc:
    """JumpChip::eval (control_flow/jump/air.rs:19-115), constraints and lookups in its order."""
    ch = ChipDesc("Jump", prep_width=0, main_width=J_WIDTH, local_only=True)
    M = main
    for col in (J_JUMP, J_JUMPI, J_JDIRECT):
        _assert_bool(ch, M(col))
    is_real = M(J_JUMP) + M(J_JUMPI) + M(J_JDIRECT)
    _assert_bool(ch, is_real)
    real_v = V([("main", J_JUMP, 1), ("main", J_JUMPI, 1), ("main", J_JDIRECT, 1)])
    opcode = V([("main", J_JUMP, OP_JUMP), ("main", J_JUMPI, OP_JUMPI), ("main", J_JDIRECT, OP_JUMPDIRECT)])
    red_v = lambda base: V([("main", base + i, 1 << (8 * i)) for i in range(4)])
    red = lambda base: sum((M(base + i) * (1 << (8 * i)) for i in range(1, 4)), M(base))
    ins = [ZERO, ZERO, _m(J_PC), red_v(J_NPC), red_v(J_NNPC), ZERO, opcode]
    ins += _vword(J_A) + _vword(J_B) + _vword(J_C) + [ZERO] * 4 + [ZERO, ZERO, ZERO, ZERO, ZERO]
    ch.receives.append(Lookup(ins, real_v, KIND_INSTRUCTION))
    ch.assert_zero(is_real * (red(J_A) - (red(J_NPC) + 4)))
    _word_range_check(ch, J_A, J_A_RC, is_real)
    _word_range_check(ch, J_NPC, J_NPC_RC, is_real)
    _word_range_check(ch, J_NNPC, J_NNPC_RC, is_real)
    for i in range(4):
        ch.assert_zero((M(J_JUMP) + M(J_JUMPI)) * (M(J_NNPC + i) - M(J_B + i)))
    _send_alu(ch, A.OP_ADD, _vword(J_NNPC), _vword(J_NPC), _vword(J_B), _m(J_JDIRECT))
    return ch


def _jump_trace(jumps):
    """JumpChip::event_to_row (control_flow/jump/trace.rs:83-102); no byte lookups."""
    J = np.asarray(jumps, np.int64).reshape(-1, 7)
    nj = len(J)
    t = np.zeros((A._pow2(nj), J_WIDTH), np.uint32)
    op = J[:, 1]
    t[:nj, J_PC] = J[:, 0]
    t[:nj, J_JUMP] = op == OP_JUMP
    t[:nj, J_JUMPI] = op == OP_JUMPI
    t[:nj, J_JDIRECT] = op == OP_JUMPDIRECT
    for base, j in ((J_A, 2), (J_B, 3), (J_C, 4), (J_NPC, 5), (J_NNPC, 6)):
        t[:nj, base:base + 4] = A._bytes(J[:, j].astype(np.uint32))
    t[:nj, J_A_RC:J_A_RC + RC_WIDTH] = _range_checker_cols(J[:, 2].astype(np.uint32))
    t[:nj, J_NPC_RC:J_NPC_RC + RC_WIDTH] = _range_checker_cols(J[:, 5].astype(np.uint32))
    t[:nj, J_NNPC_RC:J_NNPC_RC + RC_WIDTH] = _range_checker_cols(J[:, 6].astype(np.uint32))
    return t


_CORE_MACHINE = []


def core_machine() -> MachineDesc:
    """The MIPS machine (its chip descriptions are built once per process: the precompile AIRs take seconds
    to assemble; callers get their own chip list)."""
    if not _CORE_MACHINE:
        _CORE_MACHINE.append(_build_core_machine())
    m = _CORE_MACHINE[0]
    return MachineDesc(list(m.chips), m.num_pv)


def _build_core_machine() -> MachineDesc:
    # MipsAir::get_airs_and_costs order (crates/core/machine/src/mips/mod.rs:207-437): Cpu, Program, the
    # precompiles, SyscallCore/Precompile, the ALUs, Branch, Jump, SyscallInstrs, MemoryInstrs, MiscInstrs,
    # the memory chips, Global, Byte, (SysLinux,) MovCond
    from . import mips_ec as EC
    from . import mips_edwards as ED
    return MachineDesc([cpu_chip(), program_chip(), SY.sha_extend_chip(), SY.sha_compress_chip(), ED.ed_add_chip(),
                        ED.ed_decompress_chip()] + EC.chips_in_machine_order() + [SY.syscall_chip(True),
                        SY.syscall_chip(False), divrem_chip(), A.add_sub_chip(), A.bitwise_chip(), mul_chip(),
                        A.shift_right_chip(), A.shift_left_chip(), A.lt_chip(), A.clo_clz_chip(), branch_chip(),
                        jump_chip(), SY.syscall_instrs_chip(), memory_instructions_chip(), misc_instructions_chip(),
                        MM.memory_global_chip(True), MM.memory_global_chip(False), MM.memory_local_chip(),
                        MM.global_chip(), A.byte_chip(), SY.sys_linux_chip(), movcond_chip()], NUM_PV_ELTS)


# ---------------------------------------------------------------- program + execution
# An instruction is (opcode, op_a, op_b, op_c, imm_b, imm_c) at pc = PC_BASE + 4 * index
# (Instruction::new, executor/src/instruction.rs; branches: op_a = rs, op_b = rt or immediate 0,
# op_c = sign-extended offset << 2, instruction.rs:405-475).
_MIX = [(A.OP_ADD, 0), (A.OP_ADD, 1), (A.OP_SUB, 0), (A.OP_AND, 0), (A.OP_AND, 1), (A.OP_OR, 0), (A.OP_OR, 1),
        (A.OP_XOR, 0), (A.OP_XOR, 1), (A.OP_NOR, 0), (A.OP_SLT, 0), (A.OP_SLT, 1), (A.OP_SLTU, 0),
        (A.OP_SLL, 1), (A.OP_SRL, 1), (A.OP_SRA, 1), (A.OP_ROR, 1), (A.OP_SRL, 0), (A.OP_CLZ, 1), (A.OP_CLO, 1),
        (OP_MUL, 0), (OP_MULT, 0), (OP_MULTU, 0), (OP_DIV, 0), (OP_DIVU, 0), (OP_MOD, 0), (OP_MODU, 0),
        ("MFLO", 0), ("MFHI", 0), ("MTLO", 0), ("MTHI", 0), (OP_MEQ, 0), (OP_MNE, 0), (OP_WSBH, 1)]
_MIX += [(op, 1) for op in MEM_OPS]
_MIX += [(OP_SEXT, 1), (OP_EXT, 1), (OP_INS, 1), (OP_MADDU, 0), (OP_MSUBU, 0), (OP_MADD, 0), (OP_MSUB, 0)]
_KIND = {A.OP_ADD: "add", A.OP_SUB: "add", A.OP_AND: "bit", A.OP_OR: "bit", A.OP_XOR: "bit", A.OP_NOR: "bit",
         A.OP_SLT: "lt", A.OP_SLTU: "lt", A.OP_SLL: "sll", A.OP_SRL: "sr", A.OP_SRA: "sr", A.OP_ROR: "sr",
         A.OP_CLZ: "clz", A.OP_CLO: "clz"}
M32 = 0xFFFFFFFF


def _s32(x):
    return x - (1 << 32) if x >> 31 else x


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
        return int(_s32(b) < _s32(c))
    if op == A.OP_SLTU:
        return int(b < c)
    s = c & 31
    if op == A.OP_SLL:
        return (b << s) & M32
    if op == A.OP_SRL:
        return b >> s
    if op == A.OP_SRA:
        return (_s32(b) >> s) & M32
    if op == A.OP_ROR:
        return ((b >> s) | (b << (32 - s))) & M32 if s else b
    if op == OP_MUL:
        return (b * c) & M32
    if op in (OP_MULT, OP_MULTU):  # (lo, hi), executor.rs:1900-1907
        prod = (_s32(b) * _s32(c)) & ((1 << 64) - 1) if op == OP_MULT else b * c
        return prod & M32, prod >> 32
    x = b if op == A.OP_CLZ else ~b & M32
    return 32 - x.bit_length()


def _taken(op, a, b):
    """Executor::execute_branch (executor/src/executor.rs:2098-2120)."""
    if op == OP_BEQ:
        return a == b
    if op == OP_BNE:
        return a != b
    sa = _s32(a)
    return {OP_BGEZ: sa >= 0, OP_BLEZ: sa <= 0, OP_BGTZ: sa > 0, OP_BLTZ: sa < 0}[op]


_REGS_AVOID = {}


def _random_alu(r, avoid=()):
    """One random ALU instruction from 5 random words (destination never in `avoid`)."""
    op, imm = _MIX[int(r[0] % len(_MIX))]
    regs = _REGS_AVOID.get(avoid)
    if regs is None:
        regs = _REGS_AVOID[avoid] = [x for x in range(32) if x not in avoid]
    ra = 0 if (r[4] % 16 == 0 and 0 not in avoid) else regs[1 + int(r[1] % (len(regs) - 1))]
    rb = int(r[2] % 32)
    if isinstance(op, str):  # MFLO/MFHI rd = lo/hi; MTLO/MTHI lo/hi = rs: ADDs with register 32/33 (instruction.rs:387-394)
        reg = REG_LO if op.endswith("LO") else REG_HI
        return (A.OP_ADD, ra, reg, 0, 0, 1) if op.startswith("MF") else (A.OP_ADD, reg, rb, 0, 0, 1)
    if op in (OP_SEXT, OP_EXT, OP_INS):  # SEB/SEH; EXT/INS fields (msbd/msb << 5 | lsb), INS narrower than 32
        lsb = int(r[3] % 32)
        hi5 = int((r[3] >> np.uint64(8)) % (32 - lsb))
        if op == OP_INS and lsb == 0 and hi5 == 31:
            hi5 = 30
        c = int(r[3] % 2) if op == OP_SEXT else ((hi5 + (lsb if op == OP_INS else 0)) << 5) | lsb
        return (op, ra, rb, c, 0, 1)
    if op in MADDSUB_OPS:
        return (op, REG_LO, rb, int(r[3] % 32), 0, 0)
    if op in MEM_OPS:  # base r0 + offset into a 256-byte data window, so words are re-read and re-written
        sub = int((r[3] >> np.uint64(8)) % 4)
        if op in (OP_LW, OP_LL, OP_SW, OP_SC):
            sub = 0
        elif op in (OP_LH, OP_LHU, OP_SH):
            sub &= 2
        if op in STORE_OPS and op != OP_SC:
            ra = int(r[1] % 32)  # the stored register is only read
        return (op, ra, 0, DATA_BASE + 4 * int(r[3] % 64) + sub, 0, 1)
    if op in (OP_MULT, OP_MULTU, OP_DIV, OP_DIVU):  # MULT/DIV rs, rt: op_a = LO (instruction.rs:368-384)
        ra = REG_LO
    if op in (A.OP_CLZ, A.OP_CLO, OP_WSBH):
        c = 0
    elif imm and op in (A.OP_SLL, A.OP_SRL, A.OP_SRA, A.OP_ROR):
        c = int(r[3] % 32)
    elif imm:
        c = int(r[3] & np.uint64(M32))
    else:
        c = int(r[3] % 32)
    return (op, ra, rb, c, 0, imm)


def random_program(n: int, seed: int = 1):
    """n straight-line ALU instructions; register 0 is written now and then (the write is dropped,
    op_a_0)."""
    r = splitmix64(0xC0DE000 + seed, 5 * n + 5)
    return [_random_alu(r[5 * i:5 * i + 5]) for i in range(n)]


COUNTER, TARGET, LINK = 3, 30, 31  # loop counter, call-target and link registers of loop_program
_AVOID = (COUNTER, TARGET, LINK)
SUB_LEN = 5  # subroutine: 3 ALU instructions, jr r31, delay slot


def loop_program(body: int, iters: int, seed: int = 1):
    """A counted loop (the shape of examples/fibonacci's guest loop) calling a subroutine:

        r3 = r0 + iters
        r30 = r0 + S
      L: <body: random ALU instructions, forward branches of all six kinds (BEQ/BNE/BLTZ/BLEZ/BGTZ/BGEZ),
          calls `jal S` / `jalr r31, r30`, and forward `bal` (link in r31)>
        r3 = r3 + (-1)
        bne r3, r0, L
        <delay slot>
        j END
        <delay slot>
      S: <3 ALU instructions>
        jr r31
        <delay slot>
      END:

    Forward branches skip 0..2 instructions past their delay slot and never leave the body; no
    branch or jump sits in a delay slot; ALU instructions never write r3, r30, r31."""
    assert body >= 4 and 0 < iters < (1 << 31)
    r = splitmix64(0xB0D1000 + seed, 6 * body + 64)
    n_total = 2 + body + 5 + SUB_LEN
    sub_pc = PC_BASE + 4 * (2 + body + 5)
    prog = [(A.OP_ADD, COUNTER, 0, iters, 0, 1), (A.OP_ADD, TARGET, 0, sub_pc, 0, 1)]
    k = 0
    alu = lambda w: _random_alu(w, avoid=_AVOID)
    while k < body:
        w = r[6 * k:6 * k + 6]
        j = len(prog)  # index of this instruction; the body ends at 2 + body
        room = (2 + body) - (j + 2)  # instructions after the delay slot left in the body
        kind = int(w[5] % 10)
        if kind < 2 and room >= 0 and k + 1 < body:  # forward branch
            op = BRANCH_OPS[int(w[0] % 6)]
            skip = int(w[3] % 3) if room >= 2 else int(w[3] % (room + 1))
            rs = int(w[1] % 32)
            off = 4 * (skip + 1)  # target = next_pc + off: `skip` instructions past the delay slot
            if op in (OP_BEQ, OP_BNE):
                prog.append((op, rs, int(w[2] % 8), off, 0, 1))  # low registers: equal now and then
            else:
                prog.append((op, rs, 0, off, 1, 1))
            k += 1
        elif kind == 2 and room >= 0 and k + 1 < body:  # bal: forward jump-and-link
            skip = int(w[3] % 3) if room >= 2 else int(w[3] % (room + 1))
            prog.append((OP_JUMPDIRECT, LINK, 4 * (skip + 1), 0, 1, 1))
            k += 1
        elif kind == 3 and k + 1 < body:  # jal S
            prog.append((OP_JUMPI, LINK, sub_pc, 0, 1, 1))
            k += 1
        elif kind == 4 and k + 1 < body:  # jalr r31, r30
            prog.append((OP_JUMP, LINK, TARGET, 0, 0, 1))
            k += 1
        else:
            prog.append(alu(w[:5]))
            k += 1
            continue
        prog.append(alu(r[6 * k:6 * k + 5]))  # delay slot
        k += 1
    assert len(prog) == 2 + body
    prog.append((A.OP_ADD, COUNTER, COUNTER, M32, 0, 1))
    back = (2 - (len(prog) + 1)) * 4  # target = pc(L) = next_pc + c, next_pc = pc of the delay slot
    prog.append((OP_BNE, COUNTER, 0, back & M32, 0, 1))
    w = r[6 * body:]
    prog.append(alu(w[0:5]))
    prog.append((OP_JUMPI, 0, PC_BASE + 4 * n_total, 0, 1, 1))  # j END
    prog.append(alu(w[5:10]))
    prog += [alu(w[10:15]), alu(w[15:20]), alu(w[20:25]), (OP_JUMP, 0, LINK, 0, 0, 1), alu(w[25:30])]
    assert len(prog) == n_total
    return prog


def fresh_state():
    """Machine state before the first instruction: each register's / data word's last access
    (shard, timestamp), the data words' values, and (pc, next_pc)."""
    return {"last": [(0, 0)] * NUM_REGS, "pc": PC_BASE, "npc": PC_BASE + 4, "mem": {}, "mem_init": {},
            "mem_last": {}, "precompile": [], "exit_code": None}


def _execute(prog, regs, shard, max_steps, state=None):
    """Runs `prog` from the state's pc until pc leaves it (delay slots: pc <- next_pc, next_pc <-
    next_next_pc).  Returns the per-step records, the ALU/Branch events in execution order (the
    instruction's own event, then the dependencies emit_branch_dependencies adds,
    executor/src/dependencies.rs:175-224), and each register's last (shard, timestamp).
    With a `state` (continuation), the shard ends after max_steps instructions at the first point
    where the next instruction is not a delay slot (a shard's first row has next_pc = pc + 4,
    cpu/air/mod.rs eval_pc), and `state`/`regs` carry over to the next shard."""
    split = state is not None
    if state is None:
        state = fresh_state()
    end = PC_BASE + 4 * len(prog)
    last = state["last"]
    pc, npc = state["pc"], state["npc"]
    steps = []
    ev = {k: [] for k in ("add", "bit", "lt", "sll", "sr", "clz")}
    branches, jumps, muls, divs, movs, mevs, misc = [], [], [], [], [], [], []
    mem, mem_init, mem_last = state["mem"], state["mem_init"], state["mem_last"]
    # the CPU's own MemoryLocal entries for data words: (shard, clk, value) before its first access in the
    # shard; entries a syscall closed early (SyscallContext::postprocess) go to cpu_done
    cpu_first, cpu_done = {}, []
    # the CPU's register entries likewise: the record each register's open entry starts from
    reg_start, reg_done = [(last[r], regs[r]) for r in range(NUM_REGS)], []
    syscalls, commits = [], {}
    U = A.UNUSED_PC
    clk = 0
    while PC_BASE <= pc < end and state.get("exit_code") is None:  # the program halts when pc leaves it
        # a continuation shard also ends before its 24-bit clk could overflow (a syscall adds <= 255 cycles)
        if split and (len(steps) >= max_steps or clk > (1 << 24) - 1024) and npc == pc + 4:
            break
        assert len(steps) < max_steps or (split and len(steps) < max_steps + 2)
        k = (pc - PC_BASE) >> 2
        op, ra, rb, c, immb, immc = prog[k]
        extra = 0
        acc = []
        if immc:
            cv = c
            acc.append(None)
        else:
            acc.append(last[c])
            last[c] = (shard, clk + POS_C)
            cv = regs[c]
        if immb:
            bv = rb
            acc.append(None)
        else:
            acc.append(last[rb])
            last[rb] = (shard, clk + POS_B)
            bv = regs[rb]
        prev_a = regs[ra]
        if op in BRANCH_OPS:
            av = written = prev_a
            taken = _taken(op, prev_a, bv)
            nnpc = (npc + cv) & M32 if taken else npc + 4
            branches.append((pc, op, av, bv, cv, npc, nnpc, taken))
            ev["lt"].append((A.OP_SLT, int(_s32(av) < _s32(bv)), av, bv, U, U + 4))
            ev["lt"].append((A.OP_SLT, int(_s32(av) > _s32(bv)), bv, av, U, U + 4))
            if taken:
                ev["add"].append((A.OP_ADD, nnpc, npc, cv, U, U + 4))
        elif op in JUMP_OPS:
            # execute_jump / execute_jumpi / execute_jump_direct (executor.rs:2122-2154): link = next_pc + 4
            av = (npc + 4) & M32
            written = av if ra else 0
            if ra:
                regs[ra] = av
            nnpc = (npc + bv) & M32 if op == OP_JUMPDIRECT else bv
            jumps.append((pc, op, av, bv, cv, npc, nnpc))
            if op == OP_JUMPDIRECT:  # emit_jump_dependencies (dependencies.rs:230-248)
                ev["add"].append((A.OP_ADD, nnpc, npc, bv, U, U + 4))
        elif op in MUL_OPS:  # the Mul chip; MULT/MULTU also write HI at position HI (alu_rw, executor.rs:1430-1449)
            hi = 0
            if op == OP_MUL:
                av = _alu(op, bv, cv)
                muls.append((op, av, bv, cv, pc, npc, 0, -1, 0, 0, 0))
            else:
                av, hi = _alu(op, bv, cv)
                ps, pcl = last[REG_HI]
                muls.append((op, av, bv, cv, pc, npc, hi, clk, regs[REG_HI], ps, pcl))
            written = av if ra else 0
            if ra:
                regs[ra] = av
            nnpc = npc + 4
        elif op in MEM_OPS:  # execute_load / execute_store (executor.rs:1932-2096)
            addr = (bv + cv) & M32
            two = addr & 3
            aligned = addr - two
            if aligned not in mem:
                mem[aligned] = mem_init[aligned] = _mem_word(aligned)
            pmem = mem[aligned]
            mps, mpc = mem_last.get(aligned, (0, 0))
            if aligned not in cpu_first:
                cpu_first[aligned] = (mps, mpc, pmem)
            hi = prev_a  # hi_or_prev_a = the register's previous value
            if op in LOAD_OPS:
                av = nmem = None
                av = _load_value(op, pmem, two, prev_a)
                nmem = pmem
                written = av if ra else 0
                if ra:
                    regs[ra] = av
            else:
                nmem = _store_value(op, pmem, two, prev_a)
                mem[aligned] = nmem
                if op == OP_SC:  # SC writes 1 to rt
                    av = 1
                    written = 1 if ra else 0
                    if ra:
                        regs[ra] = 1
                else:  # op_a is read, not written
                    av = written = prev_a
            mem_last[aligned] = (shard, clk)
            mevs.append((pc, npc, op, av, bv, cv, prev_a, clk, addr, pmem, nmem, mps, mpc))
            # emit_memory_dependencies (dependencies.rs:125-180): the address ADD, the sign-extending SUB
            ev["add"].append((A.OP_ADD, addr, bv, cv, U, U + 4))
            if op in (OP_LB, OP_LH):
                um = (pmem >> (8 * two)) & 0xFF if op == OP_LB else (pmem >> (8 * (two & 2))) & 0xFFFF
                if um >> (7 if op == OP_LB else 15):
                    ev["add"].append((A.OP_SUB, av, um, 256 if op == OP_LB else 65536, U, U + 4))
            nnpc = npc + 4
        elif op in MISC_OPS:  # executor.rs:1692-1834; dependencies: emit_misc_dependencies (dependencies.rs:251-376)
            hi = ev_prev = 0
            if op == OP_SEXT:
                v, bits = (bv & 0xFFFF, 16) if cv else (bv & 0xFF, 8)
                av = (v - (1 << bits) if v >> (bits - 1) else v) & M32
            elif op == OP_EXT:
                lsb, msbd = cv & 31, cv >> 5
                av = (bv & (M32 if msbd + lsb == 31 else (1 << (msbd + lsb + 1)) - 1)) >> lsb
                sll = (bv << (31 - lsb - msbd)) & M32
                ev["sll"].append((A.OP_SLL, sll, bv, 31 - lsb - msbd, U, U + 4))
                ev["sr"].append((A.OP_SRL, av, sll, 31 - msbd, U, U + 4))
            elif op == OP_INS:
                lsb, msb = cv & 31, cv >> 5
                width = msb - lsb + 1
                # A full-width INS (width 32) has no satisfying MiscInstrs row: eval_ins proves
                # a = ror(srl + sll, 31 - msb) with srl looked up as SRL(ror, 32), which the ShiftRight chip
                # evaluates with the shift masked to 0 (srl = ror, so a = prev_a + b), while the reference's
                # dependency event says srl = 0 (dependencies.rs:328-329).  The reference cannot prove it
                # either; such programs are rejected here rather than producing an unprovable shard.
                assert width < 32, "full-width INS is not provable by the MiscInstrs AIR"
                field = (((1 << width) - 1) << lsb) & M32
                av = (prev_a & ~field & M32) | ((bv << lsb) & field)
                hi = ev_prev = prev_a
                ror = ((prev_a >> lsb) | (prev_a << (32 - lsb))) & M32 if lsb else prev_a
                srl = ror >> width
                sll = (bv << (31 - msb + lsb)) & M32
                add = (srl + sll) & M32
                ev["sr"].append((A.OP_ROR, ror, prev_a, lsb, U, U + 4))
                ev["sr"].append((A.OP_SRL, srl, ror, width, U, U + 4))
                ev["sll"].append((A.OP_SLL, sll, bv, 31 - msb + lsb, U, U + 4))
                ev["add"].append((A.OP_ADD, add, srl, sll, U, U + 4))
                ev["sr"].append((A.OP_ROR, av, add, 31 - msb, U, U + 4))
            elif op == OP_TEQ:  # traps when equal (execute_teq); only non-trapping TEQs reach a trace
                av = prev_a
                assert av != bv, "TEQ trap"
            if op in MADDSUB_OPS:  # (HI, LO) +/-= b * c; LO through op_a, HI at position HI
                signed = op in (OP_MADD, OP_MSUB)
                prod = ((_s32(bv) * _s32(cv)) if signed else bv * cv) & ((1 << 64) - 1)
                addend = (regs[REG_HI] << 32) | prev_a
                out = (addend + prod if op in (OP_MADDU, OP_MADD) else addend - prod) & ((1 << 64) - 1)
                av, hn = out & M32, out >> 32
                hi = ev_prev = prev_a
                hps, hpc = last[REG_HI]
                misc.append((op, av, bv, cv, ev_prev, pc, npc, clk, regs[REG_HI], hn, hps, hpc))
                last[REG_HI] = (shard, clk + POS_HI)
                regs[REG_HI] = hn
                muls.append((OP_MULT if signed else OP_MULTU, prod & M32, bv, cv, U, U + 4, prod >> 32, -1, 0, 0, 0))
            else:
                misc.append((op, av, bv, cv, ev_prev, pc, npc, 0, 0, 0, 0, 0))
            written = av if ra else 0
            if ra:
                regs[ra] = av
            nnpc = npc + 4
        elif op in MOVCOND_OPS:  # execute_condmov / execute_wsbh (executor.rs:1782-1857)
            if op == OP_WSBH:
                av = (((bv >> 16) & 0xFF) << 24) | (((bv >> 24) & 0xFF) << 16) | ((bv & 0xFF) << 8) | ((bv >> 8) & 0xFF)
                hi = 0
            else:
                av = bv if (cv == 0) == (op == OP_MEQ) else prev_a
                hi = prev_a  # hi_or_prev_a
            movs.append((pc, npc, op, av, bv, cv, hi))
            written = av if ra else 0
            if ra:
                regs[ra] = av
            nnpc = npc + 4
        elif op in DIV_OPS:  # the DivRem chip; the reference executor traps on c = 0, the AIR covers it
            q, r = _qr(op, bv, cv)
            if op in (OP_DIV, OP_DIVU):  # (LO, HI) = (quotient, remainder)
                av, hi = q, r
                ps, pcl = last[REG_HI]
                divs.append((op, bv, cv, pc, npc, clk, regs[REG_HI], ps, pcl))
            else:
                av, hi = r, 0
                divs.append((op, bv, cv, pc, npc, -1, 0, 0, 0))
            # emit_divrem_dependencies (dependencies.rs:12-102)
            signed = op in (OP_DIV, OP_MOD)
            abs_c = abs(_s32(cv)) if signed else cv
            abs_r = abs(_s32(r)) if signed else r
            if signed and cv >> 31:
                ev["add"].append((A.OP_ADD, 0, cv, abs_c & M32, U, U + 4))
            if signed and r >> 31:
                ev["add"].append((A.OP_ADD, 0, r, abs_r & M32, U, U + 4))
            ctq = ((_s32(q) * _s32(cv)) if signed else q * cv) & ((1 << 64) - 1)
            muls.append((OP_MULT if signed else OP_MULTU, ctq & M32, q, cv, U, U + 4, ctq >> 32, -1, 0, 0, 0))
            if cv:
                ev["lt"].append((A.OP_SLTU, 1, abs_r & M32, max(1, abs_c) & M32, U, U + 4))
            written = av if ra else 0
            if ra:
                regs[ra] = av
            nnpc = npc + 4
        elif op == SY.OP_SYSCALL:  # executor.rs:1570-1652: V0 holds the code, A0/A1 the arguments
            code = prev_a
            sid = SY.syscall_id(code)
            extra = code >> 24
            av = hi = code  # the syscalls here return None: V0 keeps the code
            npc = pc + 4  # SyscallContext::new: next_pc = pc + 4 (HALT sets 0)
            if sid == SY.syscall_id(SY.HALT):
                npc = 0
                state["exit_code"] = bv
            elif sid == SY.COMMIT:
                commits[bv] = cv
            elif sid == SY.COMMIT_DEFERRED_PROOFS:  # syscalls/commit.rs: deferred_proofs_digest[idx]
                commits[("deferred", bv)] = cv
            elif code in SY.PRECOMPILES or SY.is_linux(code):
                pm = SY.PrecompileMemory(mem, mem_init, mem_last, cpu_first, cpu_done, shard, _mem_word,
                                         regs, last, reg_start, reg_done)
                if SY.is_linux(code):  # syscalls/precompiles/sys_linux/*.rs: V0 <- v0 unless None
                    ret, pev = SY.exec_sys_linux(pm, shard, clk, code, bv, cv)
                    if sid == SY.SYS_EXT_GROUP:
                        npc = 0
                        state["exit_code"] = bv
                    if ret is not None:
                        av = ret
                    key = SY.SYS_LINUX
                else:
                    pev = SY.PRECOMPILES[code](pm, shard, clk, bv, cv)
                    key = SY.PRECOMPILE_KEY.get(code, code)  # the fp ops share one chip per field
                state["precompile"].append((key, (shard, clk, sid, bv, cv), pev))
            else:
                raise NotImplementedError(f"syscall {code:#x}")
            syscalls.append((pc, npc, shard, clk, av, bv, cv, prev_a, sid))
            written = av
            regs[ra] = av
            nnpc = npc + 4
        else:
            av = _alu(op, bv, cv)
            written = av if ra else 0
            if ra:
                regs[ra] = av
            nnpc = npc + 4
            ev[_KIND[op]].append((op, av, bv, cv, pc, npc))
        acc.append(last[ra])
        last[ra] = (shard, clk + POS_A)
        if op in MULT_DIV:
            last[REG_HI] = (shard, clk + POS_HI)
            regs[REG_HI] = hi
        steps.append((k, op, av, bv, cv, prev_a, written, npc, nnpc, immb, immc, acc,
                      hi if op in MUL_OPS + DIV_OPS + MOVCOND_OPS + MEM_OPS + MISC_OPS + (SY.OP_SYSCALL,) else 0,
                      clk, extra))
        clk += 5 + extra
        assert clk < (1 << 24), "the shard's clk must stay within 24 bits"
        pc, npc = npc, nnpc
    state["pc"], state["npc"] = pc, npc
    mem_entries = cpu_done + [(x, *cpu_first[x], *mem_last[x], mem[x]) for x in sorted(cpu_first)]
    reg_entries = reg_done + [(r, *reg_start[r][0], reg_start[r][1], *last[r], regs[r]) for r in range(NUM_REGS)
                              if last[r] != reg_start[r][0]]
    sysinfo = {"syscalls": syscalls, "commits": commits, "mem_entries": mem_entries, "reg_entries": reg_entries}
    return steps, ev, branches, jumps, muls, divs, movs, last, (mevs, mem_init, mem, mem_last), misc, sysinfo


def _commit_pvs(pvs, commits: dict):
    """committed_value_digest / deferred_proofs_digest words from COMMIT / COMMIT_DEFERRED_PROOFS calls."""
    for idx, word in commits.items():  # COMMIT: committed_value_digest[idx] (syscalls/commit.rs)
        if isinstance(idx, tuple):  # COMMIT_DEFERRED_PROOFS: deferred_proofs_digest[idx]
            pvs[SY.PV_DEFERRED + idx[1]] = word
        else:
            pvs[4 * idx:4 * idx + 4] = A._bytes(np.asarray([word], np.uint32))[0]


def _deferred_shard_pvs(state, shard: int) -> np.ndarray:
    """A shard without CPU (precompile or memory shard, prove.rs:300-320): the running state -- its pc where
    the execution stopped (start_pc = next_pc), the digests and exit code so far -- and its shard number.
    program_shards emits these shards after the execution has finished, i.e. on the reference's `done` path,
    which skips `state.execution_shard += 1` (prove.rs:308-311): they keep the last CPU shard's
    execution_shard."""
    pvs = np.zeros(PROOF_MAX_NUM_PVS, np.uint32)
    st = state or {}
    pc = 0 if st.get("exit_code") is not None else int(st.get("pc", 0))
    pvs[PV_START_PC] = pvs[PV_NEXT_PC] = pc
    pvs[PV_EXIT_CODE] = int(st.get("exit_code") or 0)
    pvs[PV_SHARD] = shard
    pvs[PV_EXECUTION_SHARD] = int(st.get("cpu_shards", 0))
    _commit_pvs(pvs, st.get("commits", {}))
    return pvs


def _mem_word(addr):
    """Initial content of a data word (synthetic, deterministic in the address)."""
    return (addr * 0x9E3779B1 + 0x7F4A7C15) & M32


def _ev_arrays(lst):
    from itertools import chain
    arr = np.fromiter(chain.from_iterable(lst), np.int64, count=6 * len(lst)).reshape(-1, 6)
    return tuple(arr[:, i].astype(np.uint32) for i in range(6))


def initial_registers(seed: int):
    init = splitmix64(0x5EED000 + seed, NUM_REGS) & np.uint64(M32)
    return [0] + [int(x) for x in init[1:]]


def program_shard(prog, seed: int = 1, shard: int = 1, max_steps: int = (1 << 24) // 5 - 1, state=None, regs=None,
                  capture: dict = None):
    """(machine, prep_traces, traces, public_values) of one shard executing `prog` from PC_BASE to its end
    (at most max_steps instructions: the CPU clk is range-checked to 24 bits).  With `state` and `regs`
    (program_shards), the shard continues a longer execution and stops after about max_steps.  With
    `capture` (a dict), the executor's records are left there for zkmips_amd.tracegen (device traces)."""
    if state is None:
        regs = initial_registers(seed)
    start_pc = state["pc"] if state else PC_BASE
    steps, ev, branches, jumps, muls, divs, movs, last, (mevs, mem_init, mem, mem_last), misc, sysinfo = \
        _execute(prog, regs, shard, max_steps, state)
    n = len(steps)
    assert n > 0
    height = max(16, 1 << (n - 1).bit_length())
    t = np.zeros((height, CPU_WIDTH), np.uint32)
    t[n:, C_IMMB] = 1
    t[n:, C_IMMC] = 1
    t[n:, C_RW_A] = 1
    S = np.asarray([s_[:11] for s_ in steps], np.int64)
    ks, ops = S[:, 0], S[:, 1].astype(np.uint32)
    av, bv, cv, prev_a, written = (S[:, j].astype(np.uint32) for j in range(2, 7))
    npc, nnpc, immb, immc = S[:, 7], S[:, 8], S[:, 9].astype(bool), S[:, 10].astype(bool)
    P_ = np.asarray(prog, np.int64).reshape(-1, 6)
    pcs = (PC_BASE + 4 * ks).astype(np.uint32)
    clk = np.asarray([s_[13] for s_ in steps], np.int64)
    extra = np.asarray([s_[14] for s_ in steps], np.int64)
    is_branch = np.isin(ops, BRANCH_OPS)
    is_syscall = ops == SY.OP_SYSCALL
    # cpu/trace.rs:179-195: HALT / SYS_EXT_GROUP syscalls halt
    halt = is_syscall & np.isin(prev_a & 0xFFFF, (SY.syscall_id(SY.HALT), SY.SYS_EXT_GROUP))
    is_seq = ~(is_branch | np.isin(ops, JUMP_OPS) | halt)

    mult = np.zeros((A.BYTE_ROWS, A.BYTE_MULT_WIDTH), np.uint64)
    byte_lookup = A.byte_lookup_into(mult)
    instr_cols = np.zeros((len(prog), C_IMMC + 1 - C_OPCODE), np.uint32)  # InstructionCols
    instr_cols[:, 0] = P_[:, 0]
    instr_cols[:, C_OPA - C_OPCODE] = P_[:, 1]
    instr_cols[:, C_OPB - C_OPCODE:C_OPB - C_OPCODE + 4] = A._bytes(P_[:, 2].astype(np.uint32))
    instr_cols[:, C_OPC - C_OPCODE:C_OPC - C_OPCODE + 4] = A._bytes(P_[:, 3].astype(np.uint32))
    instr_cols[:, C_OPA0 - C_OPCODE] = P_[:, 1] == 0
    instr_cols[:, C_IMMB - C_OPCODE] = P_[:, 4]
    instr_cols[:, C_IMMC - C_OPCODE] = P_[:, 5]
    t[:n, C_SHARD] = shard
    t[:n, C_CLK16] = clk & 0xFFFF
    t[:n, C_CLK8] = (clk >> 16) & 0xFF
    t[:n, C_PC] = pcs
    t[:n, C_NPC] = npc
    t[:n, C_NNPC] = nnpc
    t[:n, C_OPCODE:C_IMMC + 1] = instr_cols[ks]
    t[:n, C_RW_A] = np.isin(ops, (OP_MEQ, OP_MNE, OP_INS, SY.OP_SYSCALL) + MEM_OPS + MADDSUB_OPS)  # instruction.rs:180-205
    t[:n, C_SEQ] = is_seq
    t[:n, C_HALT] = halt
    t[:n, C_EXTRA] = extra
    his = np.asarray([s_[12] for s_ in steps], np.int64)
    # is_mult_div_instruction || is_check_memory_instruction: the row sends its shard and clk
    mult_div = np.isin(ops, MULT_DIV + MEM_OPS + MADDSUB_OPS + (SY.OP_SYSCALL,))
    t[:n, C_HI_PREV_A:C_HI_PREV_A + 4] = A._bytes(his.astype(np.uint32))
    t[:n, C_CHECK_MEM] = mult_div
    t[:n, C_SHARD_SEND] = np.where(mult_div, shard, 0)
    t[:n, C_CLK_SEND] = np.where(mult_div, clk, 0)
    t[:n, C_A_IMM] = is_branch | np.isin(ops, (OP_SB, OP_SH, OP_SW, OP_SWL, OP_SWR))  # cpu/trace.rs:135-138
    t[:n, C_A_VAL:C_A_VAL + 4] = A._bytes(av)
    t[:n, C_REAL] = 1
    byte_lookup(A.B_U16RANGE, np.full(n, shard >> 8), np.full(n, shard & 0xFF))  # U16Range(shard): row a1
    byte_lookup(A.B_U16RANGE, (clk & 0xFFFF) >> 8, clk & 0xFF)
    byte_lookup(A.B_U8RANGE, np.zeros(n, np.int64), (clk >> 16) & 0xFF)
    for j, (base, value, pos, sel) in enumerate(((C_C_ACC, cv, POS_C, ~immc), (C_B_ACC, bv, POS_B, ~immb),
                                                 (C_A_ACC + 4, written, POS_A, np.ones(n, bool)))):
        prev = np.asarray([a_[11][j] if a_[11][j] is not None else (0, 0) for a_ in steps], np.int64).reshape(-1, 2)
        t[:n, base + ACC_VALUE:base + ACC_VALUE + 4] = A._bytes(value)  # value always (cpu/trace.rs:151-152)
        t[:n, base + ACC_PREV_SHARD] = np.where(sel, prev[:, 0], 0)
        t[:n, base + ACC_PREV_CLK] = np.where(sel, prev[:, 1], 0)
        comp = prev[:, 0] == shard
        t[:n, base + ACC_COMPARE] = sel & comp
        cur = np.where(comp, clk + pos, shard)
        d = cur - np.where(comp, prev[:, 1], prev[:, 0]) - 1
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

    traces = {"Cpu": t}
    traces.update(A.alu_traces({k: _ev_arrays(v) for k, v in ev.items()}, mult))
    if branches:
        traces["Branch"] = _branch_trace(branches, byte_lookup)
    if jumps:
        traces["Jump"] = _jump_trace(jumps)
    if movs:
        traces["MovCond"] = _movcond_trace(movs)
    if divs:
        traces["DivRem"] = _divrem_trace(divs, shard, byte_lookup)[0]
    if muls:
        traces["Mul"] = _mul_trace(muls, shard, byte_lookup)
    if mevs:
        traces["MemoryInstrs"] = _mem_instr_trace(mevs, shard, byte_lookup)
    if misc:
        traces["MiscInstrs"] = _misc_trace(misc, shard, byte_lookup)
    sc = np.asarray(sysinfo["syscalls"], np.int64).reshape(-1, 9)
    core_sc = np.zeros((0, 5), np.int64)
    if len(sc):
        traces["SyscallInstrs"] = SY.syscall_instrs_trace(sc)
        # SyscallChip(Core) rows: codes with a table (byte 2) or Linux syscalls (chip.rs:157-166)
        tab = ((sc[:, 7] >> 16) & 0xFF == 1) | ((sc[:, 7] >> 8) & 0xFF != 0)
        core_sc = sc[tab][:, [2, 3, 8, 5, 6]]
        traces["SyscallCore"] = SY.syscall_trace(core_sc)

    # Program: one row per instruction, multiplicity = executions
    ph = max(16, 1 << (len(prog) - 1).bit_length())
    prep = np.zeros((ph, PROG_PREP_WIDTH), np.uint32)
    prep[:len(prog), 0] = PC_BASE + 4 * np.arange(len(prog))
    prep[:len(prog), 1:PROG_PREP_WIDTH] = instr_cols
    pm = np.zeros((ph, 1), np.uint32)
    pm[:len(prog), 0] = np.bincount(ks, minlength=len(prog))
    traces["Program"] = pm

    # MemoryLocal: every register the shard accessed, then every data word it touched, by address (the
    # reference collects them from a hash map; the order is free), with the access record before the
    # shard (shard, clk, value) and after it
    ent = sysinfo["reg_entries"] + sysinfo["mem_entries"]
    ent = np.asarray(ent, np.int64).reshape(-1, 7)
    traces["MemoryLocal"] = MM.memory_local_trace(ent)
    gmsg, grec = MM.memory_local_global_events(ent)
    # Global messages in chip order: SyscallCore's sends, then MemoryLocal's
    smsg = SY.syscall_global_messages(core_sc)
    msg = np.concatenate([smsg, gmsg])
    rec = np.concatenate([np.zeros(len(smsg), np.uint8), grec])
    kinds = np.concatenate([np.full(len(smsg), SY.KIND_SYSCALL, np.uint32), np.full(len(gmsg), KIND_MEMORY, np.uint32)])
    traces["Global"], _ = MM.global_trace(msg, rec, kinds, byte_lookup)
    if capture is not None:
        capture.update(steps=steps, alu=ev, syscalls=sc, core_syscalls=sc[tab] if len(sc) else sc, entries=ent,
                       shard=shard, prog=prog, branches=branches, mevs=mevs, jumps=jumps, movs=movs,
                       muls=muls, divs=divs, misc=misc)

    assert mult.max() < P
    traces["Byte"] = mult.astype(np.uint32)
    # The public values as the reference's prover state gives them to a CPU shard (prove.rs:266-280): the
    # running shard and execution-shard numbers, the shard's pcs, the digests committed so far (carried from
    # shard to shard: once committed, every later shard holds them), the exit code; no MemoryInit/Finalize
    # in a CPU shard, so its address bits stay zero.
    pvs = np.zeros(PROOF_MAX_NUM_PVS, np.uint32)
    pvs[PV_START_PC] = start_pc
    pvs[PV_NEXT_PC] = int(npc[-1])  # where the program left off (its end, a jump out of it, or 0 on HALT)
    pvs[PV_SHARD] = shard
    pvs[PV_EXECUTION_SHARD] = shard
    commits = state.setdefault("commits", {}) if state is not None else {}
    commits.update(sysinfo["commits"])
    _commit_pvs(pvs, commits)
    if halt.any():
        pvs[PV_EXIT_CODE] = int(bv[halt][0])
    prep_traces = {"Program": prep, "Byte": A.byte_prep_trace()}
    return core_machine(), prep_traces, traces, pvs


def _branch_trace(branches, byte_lookup):
    """BranchChip::event_to_row (control_flow/branch/trace.rs:85-130)."""
    B = np.asarray(branches, np.int64).reshape(-1, 8)
    nb = len(B)
    t = np.zeros((A._pow2(nb), BR_WIDTH), np.uint32)
    op, a, b, c, npc, nnpc, taken = (B[:, j] for j in range(1, 8))
    t[:nb, BR_PC] = B[:, 0]
    for col, code in ((BR_BEQ, OP_BEQ), (BR_BNE, OP_BNE), (BR_BLTZ, OP_BLTZ), (BR_BGTZ, OP_BGTZ),
                      (BR_BLEZ, OP_BLEZ), (BR_BGEZ, OP_BGEZ)):
        t[:nb, col] = op == code
    t[:nb, BR_A:BR_A + 4] = A._bytes(a.astype(np.uint32))
    t[:nb, BR_B:BR_B + 4] = A._bytes(b.astype(np.uint32))
    t[:nb, BR_C:BR_C + 4] = A._bytes(c.astype(np.uint32))
    sa, sb = a.astype(np.uint32).view(np.int32), b.astype(np.uint32).view(np.int32)
    t[:nb, BR_LT] = sa < sb
    t[:nb, BR_GT] = sa > sb
    t[:nb, BR_NPC:BR_NPC + 4] = A._bytes(npc.astype(np.uint32))
    t[:nb, BR_TGT:BR_TGT + 4] = A._bytes(((npc + c) & M32).astype(np.uint32))
    t[:nb, BR_NNPC:BR_NNPC + 4] = A._bytes(nnpc.astype(np.uint32))
    t[:nb, BR_NPC_RC:BR_NPC_RC + RC_WIDTH] = _range_checker_cols(npc.astype(np.uint32))
    t[:nb, BR_NNPC_RC:BR_NNPC_RC + RC_WIDTH] = _range_checker_cols(nnpc.astype(np.uint32))
    t[:nb, BR_BRANCHING] = taken
    nt = taken == 0
    for v in (npc[nt], nnpc[nt]):
        w = A._bytes(v.astype(np.uint32))
        byte_lookup(A.B_U8RANGE, w[:, 0], w[:, 1])
        byte_lookup(A.B_U8RANGE, w[:, 2], w[:, 3])
    return t


def memory_shard(state, regs, init_regs, shard: int, seed: int = 1):
    """The shard that initialises and finalises the memory image of a whole execution (the executor's
    postprocess, executor.rs:2538-2596): address 0 first, then every accessed register, then every touched
    data word; MemoryGlobalInit sends each address's initial value, MemoryGlobalFinalize receives its
    final access record, the Global chip accumulates both.  Public values chain the address ranges
    (previous_*_addr_bits = 0: this is the only memory shard)."""
    last, mem, mem_init, mem_last = state["last"], state["mem"], state["mem_init"], state["mem_last"]
    rec0 = last[0] if last[0] != (0, 0) else (0, 1)
    init = [(0, 0, 1, 1)]
    fin = [(0, regs[0], rec0[0], rec0[1])]
    for r in range(1, NUM_REGS):
        if last[r] != (0, 0):
            init.append((r, init_regs[r], 1, 1))
            fin.append((r, regs[r], last[r][0], last[r][1]))
    for x in sorted(mem):
        init.append((x, mem_init[x], 1, 1))
        fin.append((x, mem[x], mem_last[x][0], mem_last[x][1]))
    mult = np.zeros((A.BYTE_ROWS, A.BYTE_MULT_WIDTH), np.uint64)
    byte_lookup = A.byte_lookup_into(mult)
    ti, mi, ri = MM.memory_global_trace(np.asarray(init, np.int64), True)
    tf, mf, rf = MM.memory_global_trace(np.asarray(fin, np.int64), False)
    msg, rec = np.concatenate([mi, mf]), np.concatenate([ri, rf])
    tg, _ = MM.global_trace(msg, rec, np.full(len(msg), KIND_MEMORY, np.uint32), byte_lookup)
    traces = {"MemoryGlobalInit": ti, "MemoryGlobalFinalize": tf, "Global": tg, "Byte": mult.astype(np.uint32)}
    pvs = _deferred_shard_pvs(state, shard)
    last_addr = max(a for a, *_ in init)
    pvs[MM.PV_PREV_INIT_BITS:MM.PV_PREV_INIT_BITS + 32] = 0
    pvs[MM.PV_PREV_FIN_BITS:MM.PV_PREV_FIN_BITS + 32] = 0
    pvs[MM.PV_LAST_INIT_BITS:MM.PV_LAST_INIT_BITS + 32] = MM._bits32(last_addr)
    pvs[MM.PV_LAST_FIN_BITS:MM.PV_LAST_FIN_BITS + 32] = MM._bits32(last_addr)
    pvs[PV_SHARD] = shard
    prep_traces = {"Program": None, "Byte": A.byte_prep_trace()}
    return core_machine(), prep_traces, traces, pvs


PRECOMPILE_CHIP = {SY.SHA_EXTEND: "ShaExtend", SY.SHA_COMPRESS: "ShaCompress", SY.ED_ADD: "EdAddAssign",
                   SY.ED_DECOMPRESS: "EdDecompress", SY.SYS_LINUX: "SysLinux"}


def _ec_keys():
    from . import mips_ec as EC
    keys = [EC.EC_ADD[c] for c in EC.FIELDS] + [EC.EC_DOUBLE[c] for c in EC.FIELDS] + [EC.UINT256_MUL]
    keys += list(EC.EC_DECOMPRESS.values()) + [0x00_01_00_30, 0x01_01_00_09, EC.U256XU2048_MUL]  # + POSEIDON2_PERMUTE, KECCAK_SPONGE
    for f in EC.FP_OPS:
        keys += [EC.FP_OPS[f][0], EC.FP2_ADDSUB[f][0], EC.FP2_MUL[f]]
    return {k: EC.chip_for_key(k) for k in keys}


PRECOMPILE_CHIP.update(_ec_keys())  # Weierstrass curves, field towers, Uint256MulMod (mips_ec.py)


def precompile_shard(code: int, events, shard: int, seed: int = 1, state=None):
    """A precompile shard (ExecutionRecord::split, executor/src/record.rs:130-193): the syscall events of one
    precompile, its chip's rows, SyscallPrecompile (one row per call), the calls' local memory accesses in
    MemoryLocal and the Global chip accumulating the syscall receives and the memory messages."""
    mult = np.zeros((A.BYTE_ROWS, A.BYTE_MULT_WIDTH), np.uint64)
    byte_lookup = A.byte_lookup_into(mult)
    pevs = [e for _, _, e in events]
    sev = np.asarray([s_ for _, s_, _ in events], np.int64).reshape(-1, 5)
    traces = {}
    if code == SY.SHA_EXTEND:
        traces["ShaExtend"] = SY.sha_extend_trace(pevs, byte_lookup)
    elif code == SY.SHA_COMPRESS:
        traces["ShaCompress"] = SY.sha_compress_trace(pevs, byte_lookup)
    elif code == SY.ED_ADD:
        from . import mips_edwards as ED
        traces["EdAddAssign"] = ED.ed_add_trace(pevs, byte_lookup)
    elif code == SY.ED_DECOMPRESS:
        from . import mips_edwards as ED
        traces["EdDecompress"] = ED.ed_decompress_trace(pevs, byte_lookup)
    elif code == SY.SYS_LINUX:
        traces["SysLinux"] = SY.sys_linux_trace(pevs, byte_lookup)
    else:
        from . import mips_ec as EC
        traces[EC.chip_for_key(code)] = EC.trace_for_key(code, pevs, byte_lookup)
    traces["SyscallPrecompile"] = SY.syscall_trace(sev)
    ent = np.asarray([x for e in pevs for x in e["local"]], np.int64).reshape(-1, 7)
    traces["MemoryLocal"] = MM.memory_local_trace(ent)
    gmsg, grec = MM.memory_local_global_events(ent)
    smsg = SY.syscall_global_messages(sev)
    msg = np.concatenate([smsg, gmsg])
    rec = np.concatenate([np.ones(len(smsg), np.uint8), grec])
    kinds = np.concatenate([np.full(len(smsg), SY.KIND_SYSCALL, np.uint32), np.full(len(gmsg), KIND_MEMORY, np.uint32)])
    traces["Global"], _ = MM.global_trace(msg, rec, kinds, byte_lookup)
    assert mult.max() < P
    traces["Byte"] = mult.astype(np.uint32)
    pvs = _deferred_shard_pvs(state, shard)
    return core_machine(), {"Program": None, "Byte": A.byte_prep_trace()}, traces, pvs


def program_shards(prog, seed: int = 1, shard_size: int = 1 << 12, precompile_events_per_shard: int = 1 << 10):
    """A whole execution of `prog` as the reference's continuation shards (prove_with_context): CPU shards of
    about shard_size instructions (the register/memory state carries over, each shard's MemoryLocal
    closes its accesses through the Global chip), then the precompile shards (each precompile's calls in
    chunks, ExecutionRecord::split), then the memory shard.  Returns the list of
    (machine, prep_traces, traces, public_values)."""
    regs = initial_registers(seed)
    init_regs = list(regs)
    state = fresh_state()
    end = PC_BASE + 4 * len(prog)
    out, shard = [], 1
    while PC_BASE <= state["pc"] < end and state["exit_code"] is None:
        out.append(program_shard(prog, seed, shard, shard_size, state=state, regs=regs))
        state["cpu_shards"] = shard
        shard += 1
    by_code = {}
    for ev in state["precompile"]:
        by_code.setdefault(ev[0], []).append(ev)
    for code in sorted(by_code, key=lambda c: list(PRECOMPILE_CHIP).index(c)):
        evs = by_code[code]
        for k in range(0, len(evs), precompile_events_per_shard):
            out.append(precompile_shard(code, evs[k:k + precompile_events_per_shard], shard, seed, state=state))
            shard += 1
    out.append(memory_shard(state, regs, init_regs, shard, seed))
    # every shard holds the preprocessed chips (the verifier opens each vk chip in every shard,
    # verifier.rs:123-138): the Program chip with zero multiplicities in the non-CPU shards
    prog_prep = out[0][1]["Program"]
    for m, prep, traces, pvs in out:
        if "Program" not in traces:
            prep["Program"] = prog_prep
            traces["Program"] = np.zeros((prog_prep.shape[0], PROG_MAIN_WIDTH), np.uint32)
    return out


SHA_H_PTR = DATA_BASE + 0x300
SHA_H0 = [0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19]


def sha_program(calls: int, seed: int = 1, loads: int = 4, commit: bool = True, halt: bool = True,
                compress: bool = True):
    """A guest hashing `calls` random 64-byte blocks the way the reference's sha2 guests do: per block it
    stores 16 words, calls SHA_EXTEND on them (two buffers used in turn, so a word's CPU MemoryLocal
    entry is split by the syscall), then SHA_COMPRESS into the state at SHA_H_PTR (initialised to the
    SHA-256 IV), reads some words back and sums them; then COMMITs the sum and HALTs."""
    r = splitmix64(0x5A5A000 + seed, 16 * calls + 8)
    prog = []
    acc, tmp = 10, 9
    if compress:
        for i, hv in enumerate(SHA_H0):
            prog += [(A.OP_ADD, 8, 0, hv, 0, 1), (OP_SW, 8, 0, SHA_H_PTR + 4 * i, 0, 1)]
    for k in range(calls):
        w_ptr = DATA_BASE + 0x400 + 0x100 * (k % 2)
        for i in range(16):
            prog.append((A.OP_ADD, 8, 0, int(r[16 * k + i] & np.uint64(M32)), 0, 1))
            prog.append((OP_SW, 8, 0, w_ptr + 4 * i, 0, 1))
        prog += [(A.OP_ADD, SY.REG_V0, 0, SY.SHA_EXTEND, 0, 1), (A.OP_ADD, SY.REG_A0, 0, w_ptr, 0, 1),
                 (A.OP_ADD, SY.REG_A1, 0, 0, 0, 1), (SY.OP_SYSCALL, SY.REG_V0, SY.REG_A0, SY.REG_A1, 0, 0)]
        if compress:
            prog += [(A.OP_ADD, SY.REG_V0, 0, SY.SHA_COMPRESS, 0, 1), (A.OP_ADD, SY.REG_A1, 0, SHA_H_PTR, 0, 1),
                     (SY.OP_SYSCALL, SY.REG_V0, SY.REG_A0, SY.REG_A1, 0, 0),
                     (OP_LW, tmp, 0, SHA_H_PTR + 4 * (k % 8), 0, 1), (A.OP_ADD, acc, acc, tmp, 0, 0)]
        for j in range(loads):
            prog.append((OP_LW, tmp, 0, w_ptr + 4 * (16 + (7 * j + k) % 48), 0, 1))
            prog.append((A.OP_ADD, acc, acc, tmp, 0, 0))
    if commit:
        prog += [(A.OP_ADD, SY.REG_V0, 0, SY.COMMIT, 0, 1), (A.OP_ADD, SY.REG_A0, 0, 3, 0, 1),
                 (A.OP_ADD, SY.REG_A1, acc, 0, 0, 1), (SY.OP_SYSCALL, SY.REG_V0, SY.REG_A0, SY.REG_A1, 0, 0)]
    if halt:
        prog += [(A.OP_ADD, SY.REG_V0, 0, SY.HALT, 0, 1), (A.OP_ADD, SY.REG_A0, 0, 0, 0, 1),
                 (SY.OP_SYSCALL, SY.REG_V0, SY.REG_A0, SY.REG_A1, 0, 0)]
    return prog


def deferred_commit_program(words, body: int = 8, iters: int = 30, seed: int = 9):
    """A guest that runs a counted loop (loop_program), commits `words` as its deferred_proofs_digest
    (COMMIT_DEFERRED_PROOFS word by word, syscalls/commit.rs) and halts: the public values of a guest that
    verified deferred proofs, whose Compress request then carries those proofs (node_pv.deferred_node)."""
    prog = list(loop_program(body, iters, seed))  # its END is the instruction after it
    for i, w in enumerate(words):
        prog += [(A.OP_ADD, SY.REG_V0, 0, SY.COMMIT_DEFERRED_PROOFS, 0, 1), (A.OP_ADD, SY.REG_A0, 0, i, 0, 1),
                 (A.OP_ADD, SY.REG_A1, 0, int(w) % P, 0, 1), (SY.OP_SYSCALL, SY.REG_V0, SY.REG_A0, SY.REG_A1, 0, 0)]
    prog += [(A.OP_ADD, SY.REG_V0, 0, SY.HALT, 0, 1), (A.OP_ADD, SY.REG_A0, 0, 0, 0, 1),
             (SY.OP_SYSCALL, SY.REG_V0, SY.REG_A0, SY.REG_A1, 0, 0)]
    return prog


def shard_global_digest(traces) -> np.ndarray:
    """ShardProof::global_cumulative_sum of a shard: the Global chip's last-row cumulative sum."""
    return traces["Global"][-1, MM.G_CUM_X:MM.G_CUM_X + 14].copy()


def core_shard(n: int, seed: int = 1, shard: int = 1):
    """One shard executing an n-instruction straight-line program once (n < 2^24 / 5)."""
    assert 0 < n and 5 * n + 5 < (1 << 24)
    return program_shard(random_program(n, seed), seed, shard)


def loop_shard(body: int, iters: int, seed: int = 1, shard: int = 1):
    """One shard executing loop_program(body, iters): iters * (body + 3) + 1 instructions plus the
    forward branches' skips."""
    return program_shard(loop_program(body, iters, seed), seed, shard)
