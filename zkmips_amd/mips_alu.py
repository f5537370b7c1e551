"""MIPS ALU slice: real Ziren chips restated as machine-blob AIRs (first step).

The reference describes each chip's AIR in Rust; with no Rust toolchain here the constraint DAG
cannot be exported, so the chips below are restated by hand from the reference source, constraint
for constraint and lookup for lookup in the order their `eval` emits them (that order fixes the
alpha powers of the quotient fold and the LogUp column layout):

* ``AddSub``  crates/core/machine/src/alu/add_sub/mod.rs:180-226 (+ AddOperation,
  crates/core/machine/src/operations/add.rs:55-99); trace: event_to_row :149-163.
* ``Bitwise`` crates/core/machine/src/alu/bitwise/mod.rs:184-234; columns :33-59.
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


def alu_machine() -> MachineDesc:
    # chip order as in MipsAir::chips (crates/core/machine/src/mips/mod.rs): Cpu first, ALUs, Byte
    return MachineDesc([instr_source_chip(), add_sub_chip(), bitwise_chip(), byte_chip()], NUM_PV_ELTS)


# ---------------------------------------------------------------- trace generation
def _bytes(x: np.ndarray) -> np.ndarray:
    return np.stack([(x >> (8 * i)) & 0xFF for i in range(4)], axis=1).astype(np.uint32)


def _pow2(n: int) -> int:
    return max(16, 1 << max(0, (n - 1).bit_length()))


def alu_events(n_add: int, n_bit: int, seed: int = 3):
    """Synthetic ALU events: (opcode, a, b, c, pc) with a = op(b, c), half ADD/SUB, the four bitwise
    ops in turn; operands uniform u32 (SplitMix64)."""
    r = splitmix64(0xA1B0000 + seed, 2 * (n_add + n_bit) + 2)
    b = (r[0::2] & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    c = (r[1::2] & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    i = np.arange(n_add + n_bit, dtype=np.uint32)
    pc = (0x00400000 + 4 * i).astype(np.uint32)
    ba, ca = b[:n_add].astype(np.uint64), c[:n_add].astype(np.uint64)
    is_sub = (np.arange(n_add) % 2 == 1)
    a_add = np.where(is_sub, (ba - ca) & np.uint64(0xFFFFFFFF), (ba + ca) & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    op_add = np.where(is_sub, OP_SUB, OP_ADD).astype(np.uint32)
    bb, cb = b[n_add:n_add + n_bit], c[n_add:n_add + n_bit]
    kind = np.arange(n_bit) % 4
    ops = np.asarray([OP_AND, OP_OR, OP_XOR, OP_NOR], np.uint32)[kind]
    a_bit = np.select([kind == 0, kind == 1, kind == 2], [bb & cb, bb | cb, bb ^ cb], ~(bb | cb)).astype(np.uint32)
    return {"add": (op_add, a_add, b[:n_add], c[:n_add], pc[:n_add]),
            "bit": (ops, a_bit, bb, cb, pc[n_add:n_add + n_bit])}


def events_from_list(add_events, bit_events):
    """Events given as the reference's AluEvent::new(pc, opcode, a, b, c) tuples (next_pc = pc + 4,
    crates/core/executor/src/events/instr.rs:31-33)."""
    def cols(evs):
        arr = np.asarray([(op, a, b, c, pc) for pc, op, a, b, c in evs], np.uint64).reshape(-1, 5)
        return tuple(arr[:, i].astype(np.uint32) for i in range(5))
    return {"add": cols(add_events), "bit": cols(bit_events)}


def alu_shard(n_add: int, n_bit: int, seed: int = 3):
    """(machine, prep_traces, traces, public_values) of one ALU-slice shard of random events."""
    return alu_shard_from(alu_events(n_add, n_bit, seed), seed)


def alu_shard_from(ev, seed: int = 3):
    n_add, n_bit = len(ev["add"][0]), len(ev["bit"][0])
    mult = np.zeros((BYTE_ROWS, BYTE_MULT_WIDTH), np.uint64)

    def byte_lookup(op, b, c, m=1):
        np.add.at(mult[:, op], (b.astype(np.int64) << 8) + c.astype(np.int64), m)

    # AddSub (event_to_row, add_sub/mod.rs:149-163; AddOperation::populate, add.rs:21-52)
    op, a, b, c, pc = ev["add"]
    sub = op == OP_SUB
    op1 = np.where(sub, a, b)
    val = (op1.astype(np.uint64) + c) & np.uint64(0xFFFFFFFF)
    t_as = np.zeros((_pow2(n_add), AS_WIDTH), np.uint32)
    t_as[:n_add, AS_PC] = pc
    t_as[:n_add, AS_NPC] = pc + 4
    t_as[:n_add, AS_VAL:AS_VAL + 4] = _bytes(val.astype(np.uint32))
    x, y = _bytes(op1), _bytes(c)
    cy = np.zeros((n_add, 3), np.uint32)
    prev = np.zeros(n_add, np.uint32)
    for k in range(3):
        prev = ((x[:, k] + y[:, k] + prev) > 255).astype(np.uint32)
        cy[:, k] = prev
    t_as[:n_add, AS_CARRY:AS_CARRY + 3] = cy
    t_as[:n_add, AS_OP1:AS_OP1 + 4] = x
    t_as[:n_add, AS_OP2:AS_OP2 + 4] = y
    t_as[:n_add, AS_ADD] = ~sub
    t_as[:n_add, AS_SUB] = sub
    for word in (x, y, _bytes(val.astype(np.uint32))):
        byte_lookup(B_U8RANGE, word[:, 0], word[:, 1])
        byte_lookup(B_U8RANGE, word[:, 2], word[:, 3])

    # Bitwise (bitwise/mod.rs event_to_row): one byte lookup per limb
    op, a, b, c, pc2 = ev["bit"]
    t_bw = np.zeros((_pow2(n_bit), BW_WIDTH), np.uint32)
    t_bw[:n_bit, BW_PC] = pc2
    t_bw[:n_bit, BW_NPC] = pc2 + 4
    ab, bb, cb = _bytes(a), _bytes(b), _bytes(c)
    t_bw[:n_bit, BW_A:BW_A + 4] = ab
    t_bw[:n_bit, BW_B:BW_B + 4] = bb
    t_bw[:n_bit, BW_C:BW_C + 4] = cb
    for col, o in ((BW_NOR, OP_NOR), (BW_XOR, OP_XOR), (BW_OR, OP_OR), (BW_AND, OP_AND)):
        t_bw[:n_bit, col] = op == o
    bop = np.select([op == OP_AND, op == OP_OR, op == OP_XOR], [B_AND, B_OR, B_XOR], B_NOR)
    for k in range(4):
        for o in (B_AND, B_OR, B_XOR, B_NOR):
            s = bop == o
            byte_lookup(o, bb[s, k], cb[s, k])

    # instruction source: the CPU's send_instruction tuple of every ALU event
    n = n_add + n_bit
    t_is = np.zeros((_pow2(n), IS_WIDTH), np.uint32)
    ops = np.concatenate([ev["add"][0], ev["bit"][0]])
    t_is[:n, IS_PC] = np.concatenate([ev["add"][4], ev["bit"][4]])
    t_is[:n, IS_NPC] = t_is[:n, IS_PC] + 4
    t_is[:n, IS_OP] = ops
    for base, j in ((IS_A, 1), (IS_B, 2), (IS_C, 3)):
        t_is[:n, base:base + 4] = _bytes(np.concatenate([ev["add"][j], ev["bit"][j]]))
    t_is[:n, IS_REAL] = 1

    assert mult.max() < P
    traces = {"InstrSource": t_is, "AddSub": t_as, "Bitwise": t_bw, "Byte": mult.astype(np.uint32)}
    pvs = (splitmix64(0xA1B1000 + seed, PROOF_MAX_NUM_PVS) % np.uint64(P)).astype(np.uint32)
    return alu_machine(), {"Byte": byte_prep_trace()}, traces, pvs
