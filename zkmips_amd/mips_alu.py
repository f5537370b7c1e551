"""MIPS ALU slice: real Ziren chips restated as machine-blob AIRs (first step).

The reference describes each chip's AIR in Rust; with no Rust toolchain here the constraint DAG
cannot be exported, so the chips below are restated by hand from the reference source, constraint
for constraint and lookup for lookup in the order their `eval` emits them (that order fixes the
alpha powers of the quotient fold and the LogUp column layout):

* ``AddSub``  crates/core/machine/src/alu/add_sub/mod.rs:180-226 (+ AddOperation,
  crates/core/machine/src/operations/add.rs:55-99); trace: event_to_row :149-163.
* ``Bitwise`` crates/core/machine/src/alu/bitwise/mod.rs:184-234; columns :33-59.
* ``Lt``      crates/core/machine/src/alu/lt/mod.rs:277-466 (SLT/SLTU); trace: event_to_row :179-263.
* ``ShiftLeft`` crates/core/machine/src/alu/sll/mod.rs:273-406 (SLL); trace :200-260, padding :142-155.
* ``ShiftRight`` crates/core/machine/src/alu/sr/mod.rs:338-536 (SRL, SRA, ROR); trace :220-325.
* ``CloClz``  crates/core/machine/src/alu/clo_clz/mod.rs:181-271 (CLZ/CLO); it sends an SRL to
  ShiftRight like the executor's dependency event (executor/src/dependencies.rs:107-122).
* ``Byte``    crates/core/machine/src/bytes/{air.rs:24-74, columns.rs, mod.rs:50-120, trace.rs:40-70}:
  the preprocessed 2^16-row table of all byte operations and its 10 multiplicity columns.

The chip that *sends* these instructions in the reference is the CPU chip (`send_instruction`,
crates/stark/src/air/builder.rs:191-235), a ~100-column AIR over the whole execution.  It is not
restated here; ``InstrSource`` stands in for it: one row per ALU instruction holding exactly the
tuple the CPU would send (pc, next_pc, opcode, a, b, c), so the shard's Instruction lookups balance
the way they do in a real MIPS shard.  Its only constraint is ``is_real`` booleanity.  Everything
else (byte range checks, carries, bitwise tables, the Byte chip's multiplicities) is the reference
AIR.
"""
from __future__ import annotations

import numpy as np

from .machine import (ChipDesc, Expr, KIND_BYTE, KIND_INSTRUCTION, Lookup, MachineDesc, P, VirtualPairCol,
                      main, prep)
from .workloads import NUM_PV_ELTS, PROOF_MAX_NUM_PVS, splitmix64

# crates/core/executor/src/opcode.rs:15-78 (Opcode), :184-205 (ByteOpcode)
OP_ADD, OP_SUB, OP_AND, OP_OR, OP_XOR, OP_NOR = 0, 1, 15, 16, 17, 18
B_AND, B_OR, B_XOR, B_SLL, B_U8RANGE, B_SHRCARRY, B_LTU, B_MSB, B_U16RANGE, B_NOR = range(10)
BYTE_ALL = [B_AND, B_OR, B_XOR, B_SLL, B_U8RANGE, B_SHRCARRY, B_LTU, B_MSB, B_U16RANGE, B_NOR]  # byte.rs:165-180

V = VirtualPairCol
ZERO = V.const(0)


def _m(c: int) -> V:
    return V.single_main(c)


def _assert_bool(chip: ChipDesc, x: Expr, when: Expr = None):
    e = x * (x - 1)
    chip.assert_zero(e if when is None else when * e)


def _instruction(pc: int, next_pc: int, opcode: V, a, b, c) -> list:
    """The Instruction lookup tuple of send/receive_instruction (builder.rs:191-283) for an ALU op:
    shard 0, clk 0, pc, next_pc, next_pc + 4, extra cycles 0, opcode, a, b, c, hi = 0, then
    op_a_immutable 0, is_rw_a 0, is_check_memory 0, is_halt 0, is_sequential 1."""
    vals = [ZERO, ZERO, _m(pc), _m(next_pc), V([("main", next_pc, 1)], 4), ZERO, opcode]
    vals += list(a) + list(b) + list(c) + [ZERO] * 4 + [ZERO, ZERO, ZERO, ZERO, V.const(1)]
    return vals


# ---------------------------------------------------------------- AddSub
# AddSubCols (add_sub/mod.rs:43-63): pc, next_pc, add_operation{value[4], carry[3]}, operand_1[4],
# operand_2[4], is_add, is_sub
AS_PC, AS_NPC, AS_VAL, AS_CARRY, AS_OP1, AS_OP2, AS_ADD, AS_SUB = 0, 1, 2, 6, 9, 13, 17, 18
AS_WIDTH = 19


def add_sub_chip() -> ChipDesc:
    ch = ChipDesc("AddSub", prep_width=0, main_width=AS_WIDTH, local_only=True)
    a = [main(AS_OP1 + i) for i in range(4)]
    b = [main(AS_OP2 + i) for i in range(4)]
    val = [main(AS_VAL + i) for i in range(4)]
    carry = [main(AS_CARRY + i) for i in range(3)]
    is_add, is_sub = main(AS_ADD), main(AS_SUB)
    is_real = is_add + is_sub
    # AddOperation::eval (operations/add.rs:55-99), every assertion under when(is_real)
    ov = [a[0] + b[0] - val[0]] + [a[i] + b[i] - val[i] + carry[i - 1] for i in (1, 2, 3)]
    ch.assert_zero(is_real * (ov[3] * (ov[3] - 256)))
    for i in range(3):
        ch.assert_zero(is_real * (carry[i] * (ov[i] - 256)))
    for i in range(3):
        ch.assert_zero(is_real * ((carry[i] - 1) * ov[i]))
    for i in range(3):
        _assert_bool(ch, carry[i], is_real)
    _assert_bool(ch, is_real, is_real)
    # slice_range_check_u8 of a, b, value (air/word.rs:55-80): U8Range sends in byte pairs
    mult = V([("main", AS_ADD, 1), ("main", AS_SUB, 1)])
    for base in (AS_OP1, AS_OP2, AS_VAL):
        for k in (0, 2):
            ch.sends.append(Lookup([V.const(B_U8RANGE), ZERO, ZERO, _m(base + k), _m(base + k + 1)], mult, KIND_BYTE))
    w = lambda base: [_m(base + i) for i in range(4)]
    ch.receives.append(Lookup(_instruction(AS_PC, AS_NPC, V.const(OP_ADD), w(AS_VAL), w(AS_OP1), w(AS_OP2)),
                              _m(AS_ADD), KIND_INSTRUCTION))
    ch.receives.append(Lookup(_instruction(AS_PC, AS_NPC, V.const(OP_SUB), w(AS_OP1), w(AS_VAL), w(AS_OP2)),
                              _m(AS_SUB), KIND_INSTRUCTION))
    _assert_bool(ch, is_add)
    _assert_bool(ch, is_sub)
    _assert_bool(ch, is_real)
    return ch


# ---------------------------------------------------------------- Bitwise
# BitwiseCols (bitwise/mod.rs:33-59): pc, next_pc, a[4], b[4], c[4], is_nor, is_xor, is_or, is_and
BW_PC, BW_NPC, BW_A, BW_B, BW_C, BW_NOR, BW_XOR, BW_OR, BW_AND = 0, 1, 2, 6, 10, 14, 15, 16, 17
BW_WIDTH = 18


def bitwise_chip() -> ChipDesc:
    ch = ChipDesc("Bitwise", prep_width=0, main_width=BW_WIDTH, local_only=True)
    flags = [(BW_XOR, B_XOR, OP_XOR), (BW_OR, B_OR, OP_OR), (BW_AND, B_AND, OP_AND), (BW_NOR, B_NOR, OP_NOR)]
    byte_op = V([("main", col, bop) for col, bop, _ in flags if bop])  # AND = 0 drops out
    mult = V([("main", col, 1) for col, _, _ in flags])
    for i in range(4):
        ch.sends.append(Lookup([byte_op, _m(BW_A + i), ZERO, _m(BW_B + i), _m(BW_C + i)], mult, KIND_BYTE))
    cpu_op = V([("main", col, op) for col, _, op in flags])
    w = lambda base: [_m(base + i) for i in range(4)]
    ch.receives.append(Lookup(_instruction(BW_PC, BW_NPC, cpu_op, w(BW_A), w(BW_B), w(BW_C)), mult, KIND_INSTRUCTION))
    is_real = main(BW_XOR) + main(BW_OR) + main(BW_AND) + main(BW_NOR)
    for col in (BW_XOR, BW_OR, BW_AND, BW_XOR):  # as in the reference: is_xor twice, is_nor unchecked
        _assert_bool(ch, main(col))
    _assert_bool(ch, is_real)
    return ch


# ---------------------------------------------------------------- Byte
# BytePreprocessedCols (bytes/columns.rs:14-49) and ByteMultCols (:54-57)
BP_B, BP_C, BP_AND, BP_OR, BP_XOR, BP_NOR, BP_SLL, BP_SHR, BP_SHR_CARRY, BP_LTU, BP_MSB, BP_U16 = range(12)
BYTE_PREP_WIDTH, BYTE_MULT_WIDTH, BYTE_ROWS = 12, 10, 1 << 16


def byte_chip() -> ChipDesc:
    ch = ChipDesc("Byte", prep_width=BYTE_PREP_WIDTH, main_width=BYTE_MULT_WIDTH)
    p = V.single_prep
    for op in BYTE_ALL:  # bytes/air.rs:31-72
        mult = _m(op)
        if op == B_U8RANGE:
            vals = [V.const(op), ZERO, ZERO, p(BP_B), p(BP_C)]
        elif op == B_SHRCARRY:
            vals = [V.const(op), p(BP_SHR), p(BP_SHR_CARRY), p(BP_B), p(BP_C)]
        elif op == B_MSB:
            vals = [V.const(op), p(BP_MSB), ZERO, p(BP_B), ZERO]
        elif op == B_U16RANGE:
            vals = [V.const(op), p(BP_U16), ZERO, ZERO, ZERO]
        else:
            res = {B_AND: BP_AND, B_OR: BP_OR, B_XOR: BP_XOR, B_NOR: BP_NOR, B_SLL: BP_SLL, B_LTU: BP_LTU}[op]
            vals = [V.const(op), p(res), ZERO, p(BP_B), p(BP_C)]
        ch.receives.append(Lookup(vals, mult, KIND_BYTE))
    return ch


def byte_prep_trace() -> np.ndarray:
    """ByteChip::trace (bytes/mod.rs:50-120): row b * 256 + c."""
    b = np.repeat(np.arange(256, dtype=np.uint32), 256)
    c = np.tile(np.arange(256, dtype=np.uint32), 256)
    sh = c & 7
    shr = b >> sh
    carry = np.where(sh != 0, (b & ((1 << sh) - 1)), 0).astype(np.uint32)
    cols = [b, c, b & c, b | c, b ^ c, (~(b | c)) & 0xFF, (b << sh) & 0xFF, shr, carry,
            (b < c).astype(np.uint32), (b >> 7) & 1, (b << 8) + c]
    return np.ascontiguousarray(np.stack(cols, axis=1).astype(np.uint32))


# ---------------------------------------------------------------- instruction source (CPU stand-in)
IS_PC, IS_NPC, IS_OP, IS_A, IS_B, IS_C, IS_REAL = 0, 1, 2, 3, 7, 11, 15
IS_WIDTH = 16


def instr_source_chip() -> ChipDesc:
    ch = ChipDesc("InstrSource", prep_width=0, main_width=IS_WIDTH, local_only=True)
    w = lambda base: [_m(base + i) for i in range(4)]
    ch.sends.append(Lookup(_instruction(IS_PC, IS_NPC, _m(IS_OP), w(IS_A), w(IS_B), w(IS_C)), _m(IS_REAL),
                           KIND_INSTRUCTION))
    _assert_bool(ch, main(IS_REAL))
    return ch


# ---------------------------------------------------------------- Lt
# LtCols (alu/lt/mod.rs:37-86)
(LT_PC, LT_NPC, LT_SLT, LT_SLTU, LT_A, LT_B, LT_C, LT_FLAGS, LT_BM, LT_CM, LT_INV, LT_MSB_B, LT_MSB_C, LT_BIT_B,
 LT_BIT_C, LT_SLTU_R, LT_COMP_EQ, LT_SIGN_EQ, LT_CMP, LT_BEQ) = (0, 1, 2, 3, 4, 8, 12, 16, 20, 21, 22, 23, 24, 25,
                                                                 26, 27, 28, 29, 30, 32)
LT_WIDTH = 36
OP_SLT, OP_SLTU, OP_SLL = 13, 14, 9
INV_128 = pow(128, P - 2, P)


def lt_chip() -> ChipDesc:
    """LtChip::eval, alu/lt/mod.rs:277-466."""
    ch = ChipDesc("Lt", prep_width=0, main_width=LT_WIDTH, local_only=True)
    M = main
    is_slt, is_sltu = M(LT_SLT), M(LT_SLTU)
    is_real = is_slt + is_sltu
    mult = V([("main", LT_SLT, 1), ("main", LT_SLTU, 1)])
    b = [M(LT_B + i) for i in range(4)]
    c = [M(LT_C + i) for i in range(4)]
    b_comp, c_comp = list(b), list(c)
    b_comp[3] = b[3] * is_sltu + M(LT_BM) * is_slt
    c_comp[3] = c[3] * is_sltu + M(LT_CM) * is_slt
    ch.sends.append(Lookup([V.const(B_AND), _m(LT_BM), ZERO, _m(LT_B + 3), V.const(0x7F)], mult, KIND_BYTE))
    ch.sends.append(Lookup([V.const(B_AND), _m(LT_CM), ZERO, _m(LT_C + 3), V.const(0x7F)], mult, KIND_BYTE))
    ch.assert_zero(M(LT_BIT_B) - M(LT_MSB_B) * is_slt)
    ch.assert_zero(M(LT_BIT_C) - M(LT_MSB_C) * is_slt)
    ch.assert_zero(M(LT_MSB_B) - (b[3] - M(LT_BM)) * INV_128)
    ch.assert_zero(M(LT_MSB_C) - (c[3] - M(LT_CM)) * INV_128)
    _assert_bool(ch, M(LT_SIGN_EQ))
    ch.assert_zero(M(LT_SIGN_EQ) * (M(LT_BIT_B) - M(LT_BIT_C)))
    ch.assert_zero(is_real * (1 - M(LT_SIGN_EQ)) * (M(LT_BIT_B) + M(LT_BIT_C) - 1))
    ch.assert_zero(M(LT_A) - (M(LT_BIT_B) * (1 - M(LT_BIT_C)) + M(LT_SIGN_EQ) * M(LT_SLTU_R)))
    for i in (1, 2, 3):
        ch.assert_zero(M(LT_A + i))
    flags = [M(LT_FLAGS + i) for i in range(4)]
    sum_flags = flags[0] + flags[1] + flags[2] + flags[3]
    for f in flags:
        _assert_bool(ch, f)
    _assert_bool(ch, sum_flags)
    ch.assert_zero(is_real * ((1 - M(LT_COMP_EQ)) - sum_flags))
    _assert_bool(ch, M(LT_COMP_EQ))
    visited, bcb, ccb = Expr.lift(0), Expr.lift(0), Expr.lift(0)
    for i in (3, 2, 1, 0):
        visited = visited + flags[i]
        bcb = bcb + b_comp[i] * flags[i]
        ccb = ccb + c_comp[i] * flags[i]
        ch.assert_zero((1 - visited) * (b_comp[i] - c_comp[i]))
        ch.assert_zero(M(LT_COMP_EQ) * visited)
    ch.assert_zero(M(LT_CMP) - bcb)
    ch.assert_zero(M(LT_CMP + 1) - ccb)
    ch.assert_zero((1 - M(LT_COMP_EQ)) * (M(LT_INV) * (M(LT_CMP) - M(LT_CMP + 1)) - is_real))
    ch.sends.append(Lookup([V.const(B_LTU), _m(LT_SLTU_R), ZERO, _m(LT_CMP), _m(LT_CMP + 1)], mult, KIND_BYTE))
    _assert_bool(ch, is_slt)
    _assert_bool(ch, is_sltu)
    _assert_bool(ch, is_real)
    w = lambda base: [_m(base + i) for i in range(4)]
    op = V([("main", LT_SLT, OP_SLT), ("main", LT_SLTU, OP_SLTU)])
    ch.receives.append(Lookup(_instruction(LT_PC, LT_NPC, op, w(LT_A), w(LT_B), w(LT_C)), mult, KIND_INSTRUCTION))
    return ch


# ---------------------------------------------------------------- ShiftLeft
# ShiftLeftCols (alu/sll/mod.rs:64-98)
SL_PC, SL_NPC, SL_A, SL_B, SL_C, SL_CBITS, SL_NBITS, SL_MULT, SL_RES, SL_CARRY, SL_NBYTES, SL_REAL = (
    0, 1, 2, 6, 10, 14, 22, 30, 31, 35, 39, 43)
SL_WIDTH = 44


def shift_left_chip() -> ChipDesc:
    """ShiftLeft::eval, alu/sll/mod.rs:273-406."""
    ch = ChipDesc("ShiftLeft", prep_width=0, main_width=SL_WIDTH, local_only=True)
    M = main
    cb = [M(SL_CBITS + i) for i in range(8)]
    ch.assert_zero(sum((cb[i] * (1 << i) for i in range(1, 8)), cb[0]) - M(SL_C))
    nbits = cb[0] + cb[1] * 2 + cb[2] * 4
    for i in range(8):
        ch.assert_zero(M(SL_NBITS + i) * (nbits - i))
    for i in range(8):
        ch.assert_zero(M(SL_NBITS + i) * (M(SL_MULT) - (1 << i)))
    for i in range(4):
        v = M(SL_B + i) * M(SL_MULT) - M(SL_CARRY + i) * 256
        if i > 0:
            v = v + M(SL_CARRY + i - 1)
        ch.assert_zero(M(SL_RES + i) - v)
    nbytes = cb[3] + cb[4] * 2
    for i in range(4):
        ch.assert_zero(M(SL_NBYTES + i) * (nbytes - i))
    for nb in range(4):
        for i in range(4):
            rhs = Expr.lift(0) if i < nb else M(SL_RES + i - nb)
            ch.assert_zero(M(SL_NBYTES + nb) * (M(SL_A + i) - rhs))
    for i in range(8):
        _assert_bool(ch, cb[i])
    for i in range(8):
        _assert_bool(ch, M(SL_NBITS + i))
    ch.assert_zero(sum((M(SL_NBITS + i) for i in range(1, 8)), M(SL_NBITS)) - 1)
    for base in (SL_RES, SL_CARRY):
        for k in (0, 2):
            ch.sends.append(Lookup([V.const(B_U8RANGE), ZERO, ZERO, _m(base + k), _m(base + k + 1)], _m(SL_REAL),
                                   KIND_BYTE))
    for i in range(4):
        _assert_bool(ch, M(SL_NBYTES + i))
    ch.assert_zero(sum((M(SL_NBYTES + i) for i in range(1, 4)), M(SL_NBYTES)) - 1)
    _assert_bool(ch, M(SL_REAL))
    w = lambda base: [_m(base + i) for i in range(4)]
    ch.receives.append(Lookup(_instruction(SL_PC, SL_NPC, V.const(OP_SLL), w(SL_A), w(SL_B), w(SL_C)), _m(SL_REAL),
                              KIND_INSTRUCTION))
    return ch


# ---------------------------------------------------------------- ShiftRight
# ShiftRightCols (alu/sr/mod.rs:88-137)
(SR_PC, SR_NPC, SR_A, SR_B, SR_C, SR_NBITS, SR_NBYTES, SR_BYTE_RES, SR_BIT_RES, SR_CARRY, SR_SHIFTED, SR_MSB,
 SR_CBITS, SR_SRL, SR_ROR, SR_SRA, SR_REAL) = (0, 1, 2, 6, 10, 14, 22, 26, 34, 42, 50, 58, 59, 67, 68, 69, 70)
SR_WIDTH = 71
OP_SRL, OP_SRA, OP_ROR = 10, 11, 12


def shift_right_chip() -> ChipDesc:
    """ShiftRightChip::eval, alu/sr/mod.rs:338-536 (SRL, SRA, ROR)."""
    ch = ChipDesc("ShiftRight", prep_width=0, main_width=SR_WIDTH)
    M = main
    real = _m(SR_REAL)
    ch.sends.append(Lookup([V.const(B_MSB), _m(SR_MSB), ZERO, _m(SR_B + 3), ZERO], real, KIND_BYTE))
    cb = [M(SR_CBITS + i) for i in range(8)]
    ch.assert_zero(sum((cb[i] * (1 << i) for i in range(1, 8)), cb[0]) - M(SR_C))
    nbits = cb[0] + cb[1] * 2 + cb[2] * 4
    for i in range(8):
        ch.assert_zero(M(SR_NBITS + i) * (nbits - i))
    ch.assert_zero(sum((M(SR_NBITS + i) for i in range(1, 8)), M(SR_NBITS)) - 1)
    nbytes = cb[3] + cb[4] * 2
    for i in range(4):
        ch.assert_zero(M(SR_NBYTES + i) * (nbytes - i))
    ch.assert_zero(sum((M(SR_NBYTES + i) for i in range(1, 4)), M(SR_NBYTES)) - 1)
    sext = [M(SR_B + i) for i in range(4)]
    sext += [M(SR_SRA) * M(SR_MSB) * 0xFF + M(SR_ROR) * M(SR_B + i) for i in range(4)]
    for nb in range(4):
        for i in range(8 - nb):
            ch.assert_zero(M(SR_NBYTES + nb) * (M(SR_BYTE_RES + i) - sext[i + nb]))
    carry_mult = sum((M(SR_NBITS + i) * (1 << (8 - i)) for i in range(1, 8)), M(SR_NBITS) * 256)
    nbits_vpc = V([("main", SR_CBITS, 1), ("main", SR_CBITS + 1, 2), ("main", SR_CBITS + 2, 4)])
    for i in range(7, -1, -1):
        ch.sends.append(Lookup([V.const(B_SHRCARRY), _m(SR_SHIFTED + i), _m(SR_CARRY + i), _m(SR_BYTE_RES + i),
                                nbits_vpc], real, KIND_BYTE))
    for i in range(7, -1, -1):
        v = M(SR_SHIFTED + i)
        if i + 1 < 8:
            v = v + M(SR_CARRY + i + 1) * carry_mult
        ch.assert_zero(v - M(SR_BIT_RES + i))
    for i in range(4):
        ch.assert_zero(M(SR_A + i) - M(SR_BIT_RES + i))
    for col in (SR_SRL, SR_SRA, SR_ROR, SR_REAL, SR_MSB):
        _assert_bool(ch, M(col))
    for i in range(4):
        _assert_bool(ch, M(SR_NBYTES + i))
    for i in range(8):
        _assert_bool(ch, M(SR_NBITS + i))
    for i in range(8):
        _assert_bool(ch, cb[i])
    for base in (SR_BYTE_RES, SR_BIT_RES, SR_CARRY, SR_SHIFTED):
        for k in (0, 2, 4, 6):
            ch.sends.append(Lookup([V.const(B_U8RANGE), ZERO, ZERO, _m(base + k), _m(base + k + 1)], real, KIND_BYTE))
    for col in (SR_SRL, SR_SRA, SR_ROR, SR_REAL):
        _assert_bool(ch, M(col))
    ch.assert_zero(M(SR_SRL) + M(SR_SRA) + M(SR_ROR) - M(SR_REAL))
    w = lambda base: [_m(base + i) for i in range(4)]
    op = V([("main", SR_SRL, OP_SRL), ("main", SR_SRA, OP_SRA), ("main", SR_ROR, OP_ROR)])
    ch.receives.append(Lookup(_instruction(SR_PC, SR_NPC, op, w(SR_A), w(SR_B), w(SR_C)), real, KIND_INSTRUCTION))
    return ch


# ---------------------------------------------------------------- CloClz
# CloClzCols (alu/clo_clz/mod.rs:44-73)
CZ_PC, CZ_NPC, CZ_A, CZ_B, CZ_BB, CZ_BB_ZERO, CZ_SR1, CZ_CLZ, CZ_CLO, CZ_REAL = 0, 1, 2, 6, 10, 14, 15, 19, 20, 21
CZ_WIDTH = 22
OP_CLZ, OP_CLO = 19, 20
UNUSED_PC, DEFAULT_PC_INC = 1, 4  # crates/stark/src/air/builder.rs:19-22


def clo_clz_chip() -> ChipDesc:
    """CloClzChip::eval, alu/clo_clz/mod.rs:181-271.  It sends an SRL to the ShiftRight chip
    (send_alu, builder.rs:283-322) to prove that bit 31 - a of bb is its leading one."""
    ch = ChipDesc("CloClz", prep_width=0, main_width=CZ_WIDTH)
    M = main
    for i in range(4):
        ch.assert_zero(M(CZ_CLO) * (M(CZ_B + i) + M(CZ_BB + i) - 255))
        ch.assert_zero(M(CZ_CLZ) * (M(CZ_B + i) - M(CZ_BB + i)))
    real = _m(CZ_REAL)
    for k in (0, 2):
        ch.sends.append(Lookup([V.const(B_U8RANGE), ZERO, ZERO, _m(CZ_BB + k), _m(CZ_BB + k + 1)], real, KIND_BYTE))
    ch.sends.append(Lookup([V.const(B_LTU), V.const(1), ZERO, _m(CZ_A), V.const(33)], real, KIND_BYTE))
    for i in (1, 2, 3):
        ch.assert_zero(M(CZ_REAL) * M(CZ_A + i))
    w = lambda base: [_m(base + i) for i in range(4)]
    op = V([("main", CZ_CLO, OP_CLO), ("main", CZ_CLZ, OP_CLZ)])
    ch.receives.append(Lookup(_instruction(CZ_PC, CZ_NPC, op, w(CZ_A), w(CZ_B), [ZERO] * 4), real, KIND_INSTRUCTION))
    zero_bb = M(CZ_BB_ZERO)
    _assert_bool(ch, zero_bb)
    ch.assert_zero(zero_bb * sum((M(CZ_BB + i) * (1 << (8 * i)) for i in range(1, 4)), M(CZ_BB)))
    ch.assert_zero(zero_bb * M(CZ_BB + 3))
    ch.assert_zero(zero_bb * (M(CZ_A) - 32))
    srl = [ZERO, ZERO, V.const(UNUSED_PC), V.const(UNUSED_PC + DEFAULT_PC_INC),
           V.const(UNUSED_PC + 2 * DEFAULT_PC_INC), ZERO, V.const(OP_SRL)]
    srl += w(CZ_SR1) + w(CZ_BB) + [V([("main", CZ_A, P - 1)], 31), ZERO, ZERO, ZERO] + [ZERO] * 4
    srl += [ZERO, ZERO, ZERO, ZERO, V.const(1)]
    ch.sends.append(Lookup(srl, V([("main", CZ_BB_ZERO, P - 1)], 1), KIND_INSTRUCTION))
    ch.assert_zero((1 - zero_bb) * (sum((M(CZ_SR1 + i) * (1 << (8 * i)) for i in range(1, 4)), M(CZ_SR1)) - 1))
    ch.assert_zero((1 - zero_bb) * M(CZ_SR1 + 3))
    _assert_bool(ch, M(CZ_CLO))
    _assert_bool(ch, M(CZ_CLZ))
    ch.assert_zero(M(CZ_CLO) + M(CZ_CLZ) - 1)
    return ch


def alu_machine() -> MachineDesc:
    # chip order as in MipsAir::chips (crates/core/machine/src/mips/mod.rs): Cpu first, ALUs, Byte
    return MachineDesc([instr_source_chip(), add_sub_chip(), bitwise_chip(), lt_chip(), shift_left_chip(),
                        shift_right_chip(), clo_clz_chip(), byte_chip()], NUM_PV_ELTS)


# ---------------------------------------------------------------- trace generation
def _bytes(x: np.ndarray) -> np.ndarray:
    return np.stack([(x >> (8 * i)) & 0xFF for i in range(4)], axis=1).astype(np.uint32)


def _pow2(n: int) -> int:
    return max(16, 1 << max(0, (n - 1).bit_length()))


def alu_events(n_add: int, n_bit: int, seed: int = 3, n_lt: int = 0, n_sll: int = 0, n_sr: int = 0,
               n_clz: int = 0):
    """Synthetic ALU events per chip: (opcode, a, b, c, pc) with a = op(b, c) as the executor computes
    it; ADD/SUB, the four bitwise ops and SLT/SLTU alternate; operands uniform u32 (SplitMix64),
    Lt operands share their top bytes half of the time so every comparison-byte position occurs."""
    n = n_add + n_bit + n_lt + n_sll + n_sr + n_clz
    r = splitmix64(0xA1B0000 + seed, 2 * n + 2)
    b = (r[0::2] & np.uint64(0xFFFFFFFF)).astype(np.uint32)[:n]
    c = (r[1::2] & np.uint64(0xFFFFFFFF)).astype(np.uint32)[:n]
    pc = (0x00400000 + 4 * np.arange(n, dtype=np.uint64)).astype(np.uint32)
    out, o = {}, 0
    ba, ca = b[o:o + n_add].astype(np.uint64), c[o:o + n_add].astype(np.uint64)
    is_sub = (np.arange(n_add) % 2 == 1)
    a_add = np.where(is_sub, (ba - ca) & np.uint64(0xFFFFFFFF), (ba + ca) & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    out["add"] = (np.where(is_sub, OP_SUB, OP_ADD).astype(np.uint32), a_add, b[o:o + n_add], c[o:o + n_add],
                  pc[o:o + n_add])
    o += n_add
    bb, cb = b[o:o + n_bit], c[o:o + n_bit]
    kind = np.arange(n_bit) % 4
    ops = np.asarray([OP_AND, OP_OR, OP_XOR, OP_NOR], np.uint32)[kind]
    a_bit = np.select([kind == 0, kind == 1, kind == 2], [bb & cb, bb | cb, bb ^ cb], ~(bb | cb)).astype(np.uint32)
    out["bit"] = (ops, a_bit, bb, cb, pc[o:o + n_bit])
    o += n_bit
    bl, cl = b[o:o + n_lt].copy(), c[o:o + n_lt].copy()
    k = np.arange(n_lt)
    keep = (k % 8).astype(np.uint32)  # 0..3 top bytes shared (0 = independent), 4 = equal, 5..7 independent
    for nb in (1, 2, 3):
        m = np.uint32(((1 << (8 * nb)) - 1) << (8 * (4 - nb)))
        sel = keep == nb
        cl[sel] = (cl[sel] & ~m) | (bl[sel] & m)
    cl[keep == 4] = bl[keep == 4]
    slt = k % 2 == 0
    lt_s = bl.view(np.int32) < cl.view(np.int32)
    out["lt"] = (np.where(slt, OP_SLT, OP_SLTU).astype(np.uint32), np.where(slt, lt_s, bl < cl).astype(np.uint32),
                 bl, cl, pc[o:o + n_lt])
    o += n_lt
    bs, cs = b[o:o + n_sll], c[o:o + n_sll]
    out["sll"] = (np.full(n_sll, OP_SLL, np.uint32), (bs << (cs & np.uint32(31))).astype(np.uint32), bs, cs,
                  pc[o:o + n_sll])
    o += n_sll
    br, cr = b[o:o + n_sr], c[o:o + n_sr]
    kind = np.arange(n_sr) % 3
    sh = (cr & np.uint32(31)).astype(np.uint64)
    b64 = br.astype(np.uint64)
    srl = b64 >> sh
    sra = (br.view(np.int32).astype(np.int64) >> sh.astype(np.int64)).astype(np.uint64)
    ror = ((b64 | (b64 << np.uint64(32))) >> sh)
    a_sr = (np.select([kind == 0, kind == 1], [srl, sra], ror) & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    out["sr"] = (np.asarray([OP_SRL, OP_SRA, OP_ROR], np.uint32)[kind], a_sr, br, cr, pc[o:o + n_sr])
    o += n_sr
    bz = b[o:o + n_clz] >> (c[o:o + n_clz] & np.uint32(31))  # every leading-zero count occurs
    k = np.arange(n_clz)
    clo = k % 2 == 1
    bz = np.where(clo, ~bz, bz).astype(np.uint32)
    bz[k % 16 == 14] = 0
    bz[k % 16 == 15] = 0xFFFFFFFF
    out["clz"] = (np.where(clo, OP_CLO, OP_CLZ).astype(np.uint32), _count_leading(bz, clo), bz,
                  np.zeros(n_clz, np.uint32), pc[o:o + n_clz])
    return out


def _count_leading(b: np.ndarray, ones: np.ndarray) -> np.ndarray:
    x = np.where(ones, ~b, b).astype(np.uint32)
    n = np.full(len(x), 32, np.uint32)
    for s_ in range(31, -1, -1):
        n = np.where((x >> s_) & 1, np.minimum(n, 31 - s_), n)
    return n.astype(np.uint32)


def events_from_list(add_events, bit_events, lt_events=(), sll_events=(), sr_events=(), clz_events=()):
    """Events given as the reference's AluEvent::new(pc, opcode, a, b, c) tuples (next_pc = pc + 4,
    crates/core/executor/src/events/instr.rs:31-33)."""
    def cols(evs):
        arr = np.asarray([(op, a, b, c, pc) for pc, op, a, b, c in evs], np.uint64).reshape(-1, 5)
        return tuple(arr[:, i].astype(np.uint32) for i in range(5))
    return {"add": cols(add_events), "bit": cols(bit_events), "lt": cols(lt_events), "sll": cols(sll_events),
            "sr": cols(sr_events), "clz": cols(clz_events)}


def alu_shard(n_add: int, n_bit: int, seed: int = 3, n_lt: int = 0, n_sll: int = 0, n_sr: int = 0,
              n_clz: int = 0):
    """(machine, prep_traces, traces, public_values) of one ALU-slice shard of random events."""
    return alu_shard_from(alu_events(n_add, n_bit, seed, n_lt, n_sll, n_sr, n_clz), seed)


def inv_mod_p(x) -> np.ndarray:
    """Element-wise x^-1 mod p (0 for x = 0), by square-and-multiply over the whole array."""
    x = np.asarray(x, np.int64) % P
    b = x.astype(np.uint64)
    r = np.ones_like(b)
    e = P - 2
    while e:
        if e & 1:
            r = r * b % np.uint64(P)
        b = b * b % np.uint64(P)
        e >>= 1
    r[x == 0] = 0
    return r.astype(np.int64)


def _inv_table():
    """(x mod p)^-1 for x = b - c, b, c bytes (index x + 255)."""
    return np.asarray([pow(x % P, P - 2, P) if x else 0 for x in range(-255, 256)], np.uint64)


def byte_lookup_into(mult: np.ndarray):
    """Accumulator of Byte-chip multiplicities (bytes/trace.rs:40-70: row b * 256 + c, U16Range at a1)."""
    def byte_lookup(op, b, c, m=1):
        idx = ((np.asarray(b).astype(np.int64) << 8) + np.asarray(c).astype(np.int64)).ravel()
        if np.ndim(m) == 0:
            mult[:, op] += np.bincount(idx, minlength=BYTE_ROWS).astype(np.uint64) * np.uint64(m)
        else:
            w = np.broadcast_to(np.asarray(m, np.int64), np.shape(idx))
            mult[:, op] += np.bincount(idx, weights=w, minlength=BYTE_ROWS).astype(np.uint64)
    return byte_lookup


def alu_shard_from(ev, seed: int = 3):
    mult = np.zeros((BYTE_ROWS, BYTE_MULT_WIDTH), np.uint64)
    traces = alu_traces(ev, mult)

    # instruction source: the CPU's send_instruction tuple of every ALU event
    kinds = [ev[k] for k in ("add", "bit", "lt", "sll", "sr", "clz") if k in ev]
    n = sum(len(e[0]) for e in kinds)
    t = np.zeros((_pow2(n), IS_WIDTH), np.uint32)
    t[:n, IS_PC] = np.concatenate([e[4] for e in kinds])
    t[:n, IS_NPC] = t[:n, IS_PC] + 4
    t[:n, IS_OP] = np.concatenate([e[0] for e in kinds])
    for base, j in ((IS_A, 1), (IS_B, 2), (IS_C, 3)):
        t[:n, base:base + 4] = _bytes(np.concatenate([e[j] for e in kinds]))
    t[:n, IS_REAL] = 1
    traces = {"InstrSource": t, **traces}

    assert mult.max() < P
    traces["Byte"] = mult.astype(np.uint32)
    pvs = (splitmix64(0xA1B1000 + seed, PROOF_MAX_NUM_PVS) % np.uint64(P)).astype(np.uint32)
    return alu_machine(), {"Byte": byte_prep_trace()}, traces, pvs


def clz_dependencies(op, a, b):
    """The SRL events a CLZ / CLO event adds for ShiftRight (executor/src/dependencies.rs:107-122):
    bb >> (31 - a) for a nonzero operand bb (b, or ~b for CLO), pc = UNUSED_PC."""
    bbv = np.where(op == OP_CLO, ~b, b).astype(np.uint32)
    nz = bbv != 0
    sh = np.where(nz, 31 - a.astype(np.int64), 0).astype(np.uint32)
    sr1 = np.where(nz, bbv >> sh, 0).astype(np.uint32)
    nd = int(nz.sum())
    return (np.full(nd, OP_SRL, np.uint32), sr1[nz], bbv[nz], sh[nz], np.full(nd, UNUSED_PC, np.uint32),
            np.full(nd, UNUSED_PC + DEFAULT_PC_INC, np.uint32))


def alu_traces(ev, mult: np.ndarray) -> dict:
    """Traces of the ALU chips that have events in `ev` ({kind: (opcode, a, b, c, pc[, next_pc])}); their Byte
    lookups are added to `mult`."""
    byte_lookup = byte_lookup_into(mult)
    # events may carry their next_pc (AluEvent::next_pc: a delay-slot instruction after a taken branch
    # continues at the target); without it next_pc = pc + 4
    ev = {k: tuple(e[:5]) + ((e[5] if len(e) > 5 else (np.asarray(e[4]) + 4).astype(np.uint32)),)
          for k, e in ev.items()}
    traces = {}
    # AddSub (event_to_row, add_sub/mod.rs:149-163; AddOperation::populate, add.rs:21-52)
    op, a, b, c, pc, npc = ev["add"]
    n_add = len(op)
    if n_add:
        sub = op == OP_SUB
        op1 = np.where(sub, a, b)
        val = ((op1.astype(np.uint64) + c) & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        t = np.zeros((_pow2(n_add), AS_WIDTH), np.uint32)
        t[:n_add, AS_PC] = pc
        t[:n_add, AS_NPC] = npc
        t[:n_add, AS_VAL:AS_VAL + 4] = _bytes(val)
        x, y = _bytes(op1), _bytes(c)
        prev = np.zeros(n_add, np.uint32)
        for k in range(3):
            prev = ((x[:, k] + y[:, k] + prev) > 255).astype(np.uint32)
            t[:n_add, AS_CARRY + k] = prev
        t[:n_add, AS_OP1:AS_OP1 + 4] = x
        t[:n_add, AS_OP2:AS_OP2 + 4] = y
        t[:n_add, AS_ADD] = ~sub
        t[:n_add, AS_SUB] = sub
        for word in (x, y, _bytes(val)):
            byte_lookup(B_U8RANGE, word[:, 0], word[:, 1])
            byte_lookup(B_U8RANGE, word[:, 2], word[:, 3])
        traces["AddSub"] = t

    # Bitwise (bitwise/mod.rs:140-171): one byte lookup per limb
    op, a, b, c, pc, npc = ev["bit"]
    n_bit = len(op)
    if n_bit:
        t = np.zeros((_pow2(n_bit), BW_WIDTH), np.uint32)
        t[:n_bit, BW_PC] = pc
        t[:n_bit, BW_NPC] = npc
        ab, bb, cb = _bytes(a), _bytes(b), _bytes(c)
        t[:n_bit, BW_A:BW_A + 4] = ab
        t[:n_bit, BW_B:BW_B + 4] = bb
        t[:n_bit, BW_C:BW_C + 4] = cb
        for col, o in ((BW_NOR, OP_NOR), (BW_XOR, OP_XOR), (BW_OR, OP_OR), (BW_AND, OP_AND)):
            t[:n_bit, col] = op == o
        bop = np.select([op == OP_AND, op == OP_OR, op == OP_XOR], [B_AND, B_OR, B_XOR], B_NOR)
        for k in range(4):
            for o in (B_AND, B_OR, B_XOR, B_NOR):
                s_ = bop == o
                byte_lookup(o, bb[s_, k], cb[s_, k])
        traces["Bitwise"] = t

    # Lt (alu/lt/mod.rs:179-263)
    op, a, b, c, pc, npc = ev["lt"]
    n_lt = len(op)
    if n_lt:
        t = np.zeros((_pow2(n_lt), LT_WIDTH), np.uint32)
        ab, bb, cb = _bytes(a), _bytes(b), _bytes(c)
        slt = op == OP_SLT
        t[:n_lt, LT_PC] = pc
        t[:n_lt, LT_NPC] = npc
        t[:n_lt, LT_A:LT_A + 4] = ab
        t[:n_lt, LT_B:LT_B + 4] = bb
        t[:n_lt, LT_C:LT_C + 4] = cb
        bm, cm = bb[:, 3] & 0x7F, cb[:, 3] & 0x7F
        t[:n_lt, LT_BM], t[:n_lt, LT_CM] = bm, cm
        byte_lookup(B_AND, bb[:, 3], np.full(n_lt, 0x7F))
        byte_lookup(B_AND, cb[:, 3], np.full(n_lt, 0x7F))
        bc, cc = bb.copy(), cb.copy()
        bc[slt, 3], cc[slt, 3] = bm[slt], cm[slt]
        diff = bc != cc
        first = np.full(n_lt, -1)
        for i in (0, 1, 2, 3):  # the most significant differing byte wins
            first = np.where(diff[:, i], i, first)
        has = first >= 0
        fi = np.where(has, first, 0)
        rows = np.arange(n_lt)
        bcb = np.where(has, bc[rows, fi], 0).astype(np.int64)
        ccb = np.where(has, cc[rows, fi], 0).astype(np.int64)
        sltu = (bcb < ccb).astype(np.uint32)
        for i in range(4):
            t[:n_lt, LT_FLAGS + i] = has & (first == i)
        t[:n_lt, LT_INV] = _inv_table()[bcb - ccb + 255].astype(np.uint32)
        t[:n_lt, LT_CMP], t[:n_lt, LT_CMP + 1] = bcb, ccb
        t[:n_lt, LT_SLTU_R] = sltu
        t[:n_lt, LT_COMP_EQ] = ~has
        msb_b, msb_c = bb[:, 3] >> 7, cb[:, 3] >> 7
        t[:n_lt, LT_MSB_B], t[:n_lt, LT_MSB_C] = msb_b, msb_c
        t[:n_lt, LT_SIGN_EQ] = np.where(slt, msb_b == msb_c, True)
        t[:n_lt, LT_SLT], t[:n_lt, LT_SLTU] = slt, ~slt
        t[:n_lt, LT_BIT_B], t[:n_lt, LT_BIT_C] = msb_b * slt, msb_c * slt
        assert np.array_equal(ab[:, 0], (msb_b * slt) * (1 - msb_c * slt) + t[:n_lt, LT_SIGN_EQ] * sltu)
        byte_lookup(B_LTU, bcb, ccb)
        traces["Lt"] = t

    # ShiftLeft (alu/sll/mod.rs:200-260); padded rows: shift_by_n_bits[0] = shift_by_n_bytes[0] =
    # bit_shift_multiplier = 1 (:142-155)
    op, a, b, c, pc, npc = ev["sll"]
    n_sll = len(op)
    if n_sll:
        t = np.zeros((_pow2(n_sll), SL_WIDTH), np.uint32)
        t[:, SL_NBITS] = 1
        t[:, SL_NBYTES] = 1
        t[:, SL_MULT] = 1
        bb = _bytes(b)
        t[:n_sll, SL_PC] = pc
        t[:n_sll, SL_NPC] = npc
        t[:n_sll, SL_A:SL_A + 4] = _bytes(a)
        t[:n_sll, SL_B:SL_B + 4] = bb
        t[:n_sll, SL_C:SL_C + 4] = _bytes(c)
        for i in range(8):
            t[:n_sll, SL_CBITS + i] = (c >> i) & 1
        nb = c % 8
        t[:n_sll, SL_NBITS] = 0
        for i in range(8):
            t[:n_sll, SL_NBITS + i] = nb == i
        mul = (np.uint32(1) << nb).astype(np.uint32)
        t[:n_sll, SL_MULT] = mul
        carry = np.zeros(n_sll, np.uint32)
        res = np.zeros((n_sll, 4), np.uint32)
        cry = np.zeros((n_sll, 4), np.uint32)
        for i in range(4):
            v = bb[:, i] * mul + carry
            carry = v >> 8
            res[:, i], cry[:, i] = v & 0xFF, carry
        t[:n_sll, SL_RES:SL_RES + 4] = res
        t[:n_sll, SL_CARRY:SL_CARRY + 4] = cry
        nbyte = (c & 31) // 8
        t[:n_sll, SL_NBYTES] = 0
        for i in range(4):
            t[:n_sll, SL_NBYTES + i] = nbyte == i
        t[:n_sll, SL_REAL] = 1
        for word in (res, cry):
            byte_lookup(B_U8RANGE, word[:, 0], word[:, 1])
            byte_lookup(B_U8RANGE, word[:, 2], word[:, 3])
        traces["ShiftLeft"] = t

    # CloClz (alu/clo_clz/mod.rs:85-160); its SRL dependencies (executor/src/dependencies.rs:107-122)
    # join the ShiftRight events with pc = UNUSED_PC
    none = (np.zeros(0, np.uint32),) * 6
    op, a, b, c, pc, npc = ev.get("clz", none)
    n_cz = len(op)
    dep = none
    if n_cz:
        t = np.zeros((_pow2(n_cz), CZ_WIDTH), np.uint32)
        t[:, CZ_A] = 32  # padding rows: clz(0) = 32
        t[:, CZ_CLZ] = 1
        t[:, CZ_BB_ZERO] = 1
        clo = op == OP_CLO
        bbv = np.where(clo, ~b, b).astype(np.uint32)
        t[:n_cz, CZ_PC] = pc
        t[:n_cz, CZ_NPC] = npc
        t[:n_cz, CZ_A:CZ_A + 4] = _bytes(a)
        t[:n_cz, CZ_B:CZ_B + 4] = _bytes(b)
        t[:n_cz, CZ_BB:CZ_BB + 4] = _bytes(bbv)
        nz = bbv != 0
        t[:n_cz, CZ_BB_ZERO] = ~nz
        sh = np.where(nz, 31 - a.astype(np.int64), 0).astype(np.uint32)
        sr1 = np.where(nz, bbv >> sh, 0).astype(np.uint32)
        t[:n_cz, CZ_SR1:CZ_SR1 + 4] = _bytes(sr1)
        t[:n_cz, CZ_CLZ], t[:n_cz, CZ_CLO] = ~clo, clo
        t[:n_cz, CZ_REAL] = 1
        bbb = _bytes(bbv)
        byte_lookup(B_U8RANGE, bbb[:, 0], bbb[:, 1])
        byte_lookup(B_U8RANGE, bbb[:, 2], bbb[:, 3])
        byte_lookup(B_LTU, a, np.full(n_cz, 33))
        traces["CloClz"] = t
        dep = clz_dependencies(op, a, b)

    # ShiftRight (alu/sr/mod.rs:220-325); padded rows: shift_by_n_bits[0] = shift_by_n_bytes[0] = 1
    cpu_sr = ev.get("sr", none)
    op, a, b, c, pc, npc = (np.concatenate([cpu_sr[j], dep[j]]).astype(np.uint32) for j in range(6))
    n_sr = len(op)
    if n_sr:
        t = np.zeros((_pow2(n_sr), SR_WIDTH), np.uint32)
        t[:, SR_NBITS] = 1
        t[:, SR_NBYTES] = 1
        t[:n_sr, SR_PC] = pc
        t[:n_sr, SR_NPC] = npc
        t[:n_sr, SR_A:SR_A + 4] = _bytes(a)
        bb = _bytes(b)
        t[:n_sr, SR_B:SR_B + 4] = bb
        t[:n_sr, SR_C:SR_C + 4] = _bytes(c)
        msb = (b >> 31) & 1
        t[:n_sr, SR_MSB] = msb
        byte_lookup(B_MSB, bb[:, 3], np.zeros(n_sr, np.uint32))
        for i in range(8):
            t[:n_sr, SR_CBITS + i] = (c >> i) & 1
        t[:n_sr, SR_SRL], t[:n_sr, SR_SRA], t[:n_sr, SR_ROR] = op == OP_SRL, op == OP_SRA, op == OP_ROR
        t[:n_sr, SR_REAL] = 1
        nbyte = ((c & 31) // 8).astype(np.uint64)
        nbit = ((c & 31) % 8).astype(np.uint32)
        b64 = b.astype(np.uint64)
        sext = np.where(op == OP_SRA, (b.view(np.int32).astype(np.int64)).astype(np.uint64),
                        np.where(op == OP_ROR, b64 | (b64 << np.uint64(32)), b64))
        bsr = sext >> (np.uint64(8) * nbyte)
        byte_res = np.stack([((bsr >> np.uint64(8 * i)) & np.uint64(0xFF)).astype(np.uint32) for i in range(8)], 1)
        t[:n_sr, SR_NBYTES] = 0
        for i in range(4):
            t[:n_sr, SR_NBYTES + i] = nbyte == i
        t[:n_sr, SR_NBITS] = 0
        for i in range(8):
            t[:n_sr, SR_NBITS + i] = nbit == i
        shifted = byte_res >> nbit[:, None]
        carry = byte_res & ((np.uint32(1) << nbit) - 1)[:, None]
        bit_res = shifted.copy()
        bit_res[:, :7] = (shifted[:, :7] + (carry[:, 1:] << (8 - nbit)[:, None])) & 0xFF
        t[:n_sr, SR_BYTE_RES:SR_BYTE_RES + 8] = byte_res
        t[:n_sr, SR_BIT_RES:SR_BIT_RES + 8] = bit_res
        t[:n_sr, SR_CARRY:SR_CARRY + 8] = carry
        t[:n_sr, SR_SHIFTED:SR_SHIFTED + 8] = shifted
        assert np.array_equal(bit_res[:, :4], t[:n_sr, SR_A:SR_A + 4])
        for i in range(8):
            byte_lookup(B_SHRCARRY, byte_res[:, i], nbit)
        for word in (byte_res, bit_res, carry, shifted):
            for k in (0, 2, 4, 6):
                byte_lookup(B_U8RANGE, word[:, k], word[:, k + 1])
        traces["ShiftRight"] = t

    return traces
