"""Syscalls and the SHA-256 precompiles restated as machine-blob AIRs.

* ``SyscallInstrs``  crates/core/machine/src/syscall/instructions/{air.rs:22-425, columns.rs, trace.rs:81-162}:
  receives the CPU's SYSCALL instruction, decodes the syscall code in the previous value of V0
  (byte 0-1 id, byte 2 "has its own table", byte 3 extra cycles), sends the syscall to SyscallCore,
  and checks HALT / COMMIT / COMMIT_DEFERRED_PROOFS against the public values.
* ``SyscallCore`` / ``SyscallPrecompile``  crates/core/machine/src/syscall/chip.rs:78-295: one row per
  syscall that has a table; the core variant receives it in the CPU shard and sends it to the Global
  chip, the precompile variant sends it to the precompile chip in the precompile shard and receives it
  from the Global chip.
* ``ShaExtend``  crates/core/machine/src/syscall/precompiles/sha256/extend/{air.rs:25-221, flags.rs,
  columns.rs, trace.rs:98-150}: 48 rows per SHA_EXTEND call, row j computing w[16 + j] from four memory
  reads and one write at timestamp clk + j.
* ``ShaCompress``  .../sha256/compress/{air.rs, columns.rs, trace.rs}: see sha_compress_chip.

Execution side (executor/src/executor.rs:1570-1652, syscalls/context.rs, syscalls/precompiles/sha256/*.rs):
the syscall's memory accesses are made at (shard, clk + k) and recorded in the precompile's own
local-memory map; a word the CPU touched earlier in the shard has its CPU MemoryLocal entry closed at
that point (SyscallContext::postprocess, context.rs:128-147), so both shards' memory arguments close.
"""
from __future__ import annotations

import numpy as np

from . import mips_alu as A
from .machine import (ChipDesc, Expr, IS_FIRST, IS_LAST, IS_TRANSITION, KIND_BYTE, KIND_GLOBAL, KIND_INSTRUCTION,
                      KIND_SYSCALL, Lookup, P, VirtualPairCol as V, main, main_next, pv)

_m = A._m
ZERO = A.ZERO
_assert_bool = A._assert_bool
M32 = 0xFFFFFFFF

OP_SYSCALL = 30  # executor/src/opcode.rs:48
REG_V0, REG_A0, REG_A1 = 2, 4, 5  # Instruction::new(SYSCALL, 2, 4, 5, false, false), instruction.rs:552

# SyscallCode (executor/src/syscalls/code.rs:27-186): id (bytes 0-1), has-table (byte 2), extra cycles (byte 3)
HALT, COMMIT, COMMIT_DEFERRED_PROOFS = 0x00_00_00_00, 0x00_00_00_10, 0x00_00_00_1A
ENTER_UNCONSTRAINED, EXIT_UNCONSTRAINED, HINT_LEN = 0x03, 0x04, 0xF0
SHA_EXTEND, SHA_COMPRESS = 0x30_01_00_05, 0x01_01_00_06
SYS_EXT_GROUP = 4246
# Linux syscalls (code.rs:143-183), handled by the SysLinux precompile table (byte 1 != 0)
SYS_LINUX, SYS_READ, SYS_WRITE, SYS_BRK, SYS_FCNTL, SYS_MMAP2, SYS_CLONE, SYS_MMAP = 4000, 4003, 4004, 4045, 4055, 4090, 4120, 4210
SYS_NOPS = (4005, 4006, 4091, 4194, 4195, 4206, 4215, 4218, 4222, 4240, 4263, 4288, 4338)  # open .. prlimit64
REG_A2, REG_A3, REG_BRK, REG_HEAP = 6, 7, 34, 35
MIPS_EBADF, PAGE_SIZE = 9, 0x1000
PV_DIGEST_WORDS = 8
PV_DEFERRED = 32  # deferred_proofs_digest follows the 8 committed-value digest words
PV_EXIT_CODE = 42


def syscall_id(code: int) -> int:
    return code & 0xFFFF


def is_linux(code: int) -> bool:
    return code in (SYS_READ, SYS_WRITE, SYS_BRK, SYS_FCNTL, SYS_MMAP2, SYS_CLONE, SYS_MMAP, SYS_EXT_GROUP) + SYS_NOPS


def _w(base):
    return [main(base + i) for i in range(4)]


def _vw(base):
    return [_m(base + i) for i in range(4)]


def _reduce(base) -> Expr:
    """Word::reduce: sum byte_i * 256^i."""
    return sum((main(base + i) * (1 << (8 * i)) for i in range(1, 4)), main(base))


def _reduce_v(base) -> V:
    return V([("main", base + i, 1 << (8 * i)) for i in range(4)])


def _is_zero_op(ch: ChipDesc, a: Expr, base: int, is_real):
    """IsZeroOperation::eval (operations/is_zero.rs): cols (inverse, result) at base, base + 1."""
    inv, res = main(base), main(base + 1)
    ch.assert_zero(is_real * ((1 - inv * a) - res))
    ch.assert_zero(is_real * (res * (res - 1)))
    ch.assert_zero(is_real * res * a)


def _is_zero_cols(a: np.ndarray):
    """IsZeroOperation::populate_from_field_element over a column of field elements."""
    a = np.asarray(a, np.int64) % P
    return A.inv_mod_p(a).astype(np.uint32), (a == 0).astype(np.uint32)


# ---------------------------------------------------------------- SyscallInstrs
# SyscallInstrColumns (syscall/instructions/columns.rs:11-77)
SI_PC, SI_NPC, SI_SHARD, SI_CLK, SI_EXTRA, SI_HALT, SI_LINUX, SI_ID = range(8)
SI_A, SI_B, SI_C, SI_PREV_A = 8, 12, 16, 20
SI_IZ_EU, SI_IZ_HL, SI_IZ_HALT, SI_IZ_EG, SI_IZ_COMMIT, SI_IZ_CDP = 24, 26, 28, 30, 32, 34
SI_BITMAP, SI_RC_BITS, SI_RC_AND, SI_OPERAND, SI_RCOP, SI_REAL = 36, 44, 52, 58, 62, 63
SI_WIDTH = 64


def _kb_word_range_check(ch, value_base, bits_base, and_base, is_real):
    """KoalaBearWordRangeChecker::range_check (operations/koala_bear_word.rs): the most significant byte's
    bits; value < p."""
    M = main
    bits = [M(bits_base + i) for i in range(8)]
    rec = Expr.lift(0)
    for i, b in enumerate(bits):
        _assert_bool(ch, b, is_real)
        rec = rec + (1 << i) * b
    ch.assert_zero(is_real * (rec - M(value_base + 3)))
    ch.assert_zero(is_real * bits[7])
    ch.assert_zero(is_real * (M(and_base) - bits[0] * bits[1]))
    for k in range(1, 6):
        ch.assert_zero(is_real * (M(and_base + k) - M(and_base + k - 1) * bits[k + 1]))
    ch.assert_zero(is_real * M(and_base + 5) * (M(value_base) + M(value_base + 1) + M(value_base + 2)))


def syscall_instrs_chip() -> ChipDesc:
    """SyscallInstrsChip::eval (syscall/instructions/air.rs:28-95) with eval_is_halt_syscall, eval_syscall,
    eval_commit and eval_halt_unimpl in the reference's order."""
    ch = ChipDesc("SyscallInstrs", prep_width=0, main_width=SI_WIDTH)
    M = main
    real = M(SI_REAL)
    prev = _w(SI_PREV_A)
    sid = prev[0] + prev[1] * 256
    _assert_bool(ch, real)
    # eval_is_halt_syscall (:339-375)
    _is_zero_op(ch, sid - syscall_id(HALT), SI_IZ_HALT, real)
    _is_zero_op(ch, sid - SYS_EXT_GROUP, SI_IZ_EG, real)
    ch.assert_zero(M(SI_HALT) - (M(SI_IZ_HALT + 1) + M(SI_IZ_EG + 1)) * real)
    # receive_instruction (:56-74): op_a_immutable 0, is_rw_a 1, is_check_memory 1, is_sequential 1 - is_halt
    ins = [_m(SI_SHARD), _m(SI_CLK), _m(SI_PC), _m(SI_NPC), V([("main", SI_NPC, 1)], 4), _m(SI_EXTRA),
           V.const(OP_SYSCALL)] + _vw(SI_A) + _vw(SI_B) + _vw(SI_C) + _vw(SI_PREV_A)
    ins += [ZERO, V.const(1), V.const(1), _m(SI_HALT), V([("main", SI_HALT, P - 1)], 1)]
    ch.receives.append(Lookup(ins, _m(SI_REAL), KIND_INSTRUCTION))
    ch.assert_zero(M(SI_EXTRA) - prev[3] * real)
    # eval_syscall (:134-243)
    linux = M(SI_LINUX)
    send_table = linux + prev[2]
    _assert_bool(ch, prev[2])
    _assert_bool(ch, linux)
    _assert_bool(ch, send_table)
    ch.assert_zero((1 - real) * send_table)
    ch.sends.append(Lookup([_m(SI_SHARD), _m(SI_CLK), V([("main", SI_PREV_A, 1), ("main", SI_PREV_A + 1, 256)]),
                            _reduce_v(SI_B), _reduce_v(SI_C)],
                           V([("main", SI_LINUX, 1), ("main", SI_PREV_A + 2, 1)]), KIND_SYSCALL))
    _is_zero_op(ch, sid - ENTER_UNCONSTRAINED, SI_IZ_EU, real)
    eu = M(SI_IZ_EU + 1)
    ch.assert_zero(real * (1 - eu) * (M(SI_ID) - sid))
    ch.assert_zero(real * eu * (M(SI_ID) - EXIT_UNCONSTRAINED))
    _is_zero_op(ch, sid - HINT_LEN, SI_IZ_HL, real)
    hl = M(SI_IZ_HL + 1)
    for i in range(4):
        ch.assert_zero(real * eu * M(SI_A + i))
    for i in range(4):
        ch.assert_zero(real * (1 - (eu + hl + linux)) * (M(SI_A + i) - prev[i]))
    ch.assert_zero(real * (1 - linux) * prev[1])
    ch.assert_zero(M(SI_RCOP) - real * (M(SI_IZ_HALT + 1) + M(SI_IZ_EG + 1) + M(SI_IZ_CDP + 1)))
    _kb_word_range_check(ch, SI_OPERAND, SI_RC_BITS, SI_RC_AND, M(SI_RCOP))
    # eval_commit (:246-317)
    _is_zero_op(ch, sid - COMMIT, SI_IZ_COMMIT, real)
    _is_zero_op(ch, sid - COMMIT_DEFERRED_PROOFS, SI_IZ_CDP, real)
    ic, icdp = M(SI_IZ_COMMIT + 1), M(SI_IZ_CDP + 1)
    bits = [M(SI_BITMAP + i) for i in range(PV_DIGEST_WORDS)]
    bsum = sum(bits[1:], bits[0])
    for b in bits:
        _assert_bool(ch, b, real)
    ch.assert_zero(real * (ic + icdp) * (bsum - 1))
    ch.assert_zero(real * (1 - (ic + icdp)) * bsum)
    for i, b in enumerate(bits):
        ch.assert_zero(real * b * (M(SI_B) - i))
    for i in range(3):
        ch.assert_zero(real * (ic + icdp) * M(SI_B + i + 1))
    for j in range(4):  # index_word_array(committed_value_digest, bitmap) == op_c
        exp = sum((pv(4 * k + j) * bits[k] for k in range(1, PV_DIGEST_WORDS)), pv(j) * bits[0])
        ch.assert_zero(real * ic * (exp - M(SI_C + j)))
    for j in range(4):
        ch.assert_zero(real * icdp * (M(SI_C + j) - M(SI_OPERAND + j)))
    exp_d = sum((pv(PV_DEFERRED + k) * bits[k] for k in range(1, PV_DIGEST_WORDS)), pv(PV_DEFERRED) * bits[0])
    ch.assert_zero(real * icdp * (exp_d - _reduce(SI_C)))
    # eval_halt_unimpl (:320-336)
    halt = M(SI_HALT)
    ch.assert_zero(halt * M(SI_NPC))
    for j in range(4):
        ch.assert_zero(halt * (M(SI_B + j) - M(SI_OPERAND + j)))
    ch.assert_zero(halt * (_reduce(SI_B) - pv(PV_EXIT_CODE)))
    return ch


def syscall_instrs_trace(ev: np.ndarray) -> np.ndarray:
    """SyscallInstrsChip::event_to_row (trace.rs:82-162).  ev: n x 9 = (pc, next_pc, shard, clk, a, b, c,
    prev_a, syscall_id); no byte lookups."""
    E = np.asarray(ev, np.int64).reshape(-1, 9)
    n = len(E)
    t = np.zeros((A._pow2(n), SI_WIDTH), np.uint32)
    if n == 0:
        return t
    pc, npc, shard, clk, a, b, c, prev, sidc = (E[:, j] for j in range(9))
    sid = prev & 0xFFFF
    t[:n, SI_PC], t[:n, SI_NPC], t[:n, SI_SHARD], t[:n, SI_CLK] = pc, npc, shard, clk
    for base, v in ((SI_A, a), (SI_B, b), (SI_C, c), (SI_PREV_A, prev)):
        t[:n, base:base + 4] = A._bytes(v.astype(np.uint32))
    t[:n, SI_ID] = sidc
    t[:n, SI_EXTRA] = prev >> 24
    halt = (sid == syscall_id(HALT)) | (sid == SYS_EXT_GROUP)
    t[:n, SI_HALT] = halt
    t[:n, SI_LINUX] = (prev & 0xFF00) != 0
    for base, code in ((SI_IZ_EU, ENTER_UNCONSTRAINED), (SI_IZ_HL, HINT_LEN), (SI_IZ_HALT, HALT),
                       (SI_IZ_EG, SYS_EXT_GROUP), (SI_IZ_COMMIT, COMMIT), (SI_IZ_CDP, COMMIT_DEFERRED_PROOFS)):
        t[:n, base], t[:n, base + 1] = _is_zero_cols(sid - syscall_id(code))
    commit = (sid == COMMIT) | (sid == COMMIT_DEFERRED_PROOFS)
    rows = np.nonzero(commit)[0]
    t[rows, SI_BITMAP + b[rows]] = 1
    cdp = sid == COMMIT_DEFERRED_PROOFS
    operand = np.where(halt, b, np.where(cdp, c, 0))
    chk = halt | cdp
    ow = A._bytes(operand.astype(np.uint32))
    t[:n, SI_OPERAND:SI_OPERAND + 4] = np.where(chk[:, None], ow, 0)
    msb = ow[:, 3].astype(np.int64)
    bits = (msb[:, None] >> np.arange(8)) & 1
    ands = np.cumprod(bits[:, :7], axis=1)[:, 1:]  # b0*b1, .., b0*..*b6
    t[:n, SI_RC_BITS:SI_RC_BITS + 8] = np.where(chk[:, None], bits, 0)
    t[:n, SI_RC_AND:SI_RC_AND + 6] = np.where(chk[:, None], ands, 0)
    t[:n, SI_RCOP] = chk
    t[:n, SI_REAL] = 1
    return t


# ---------------------------------------------------------------- SyscallCore / SyscallPrecompile
SC_SHARD, SC_CLK, SC_ID, SC_ARG1, SC_ARG2, SC_REAL = range(6)
SC_WIDTH = 6


def syscall_chip(core: bool) -> ChipDesc:
    """SyscallChip::eval (syscall/chip.rs:221-294)."""
    ch = ChipDesc("SyscallCore" if core else "SyscallPrecompile", prep_width=0, main_width=SC_WIDTH)
    _assert_bool(ch, main(SC_REAL))
    vals = [_m(SC_SHARD), _m(SC_CLK), _m(SC_ID), _m(SC_ARG1), _m(SC_ARG2)]
    real = _m(SC_REAL)
    (ch.receives if core else ch.sends).append(Lookup(vals, real, KIND_SYSCALL))
    flags = [real, ZERO] if core else [ZERO, real]  # (is_send, is_receive) of the Global message
    ch.sends.append(Lookup(vals + [ZERO, ZERO] + flags + [V.const(KIND_SYSCALL)], real, KIND_GLOBAL))
    return ch


def syscall_trace(ev: np.ndarray) -> np.ndarray:
    """SyscallChip::generate_trace (chip.rs:138-183).  ev: n x 5 = (shard, clk, syscall_id, arg1, arg2)."""
    E = np.asarray(ev, np.int64).reshape(-1, 5)
    n = len(E)
    t = np.zeros((A._pow2(n), SC_WIDTH), np.uint32)
    t[:n, :5] = E
    t[:n, SC_REAL] = 1
    return t


def syscall_global_messages(ev: np.ndarray):
    """SyscallChip::generate_dependencies (chip.rs:89-121): messages [shard, clk, id, arg1, arg2, 0, 0]."""
    E = np.asarray(ev, np.int64).reshape(-1, 5)
    msg = np.zeros((len(E), 7), np.uint32)
    msg[:, :5] = E
    return msg


# ---------------------------------------------------------------- word operations shared by the SHA chips
def _eval_shr_carry_op(ch, src, rotation, base, is_real_v, rotate: bool):
    """FixedRotateRightOperation / FixedShiftRightOperation::eval: cols value[4], shift[4], carry[4]."""
    nbytes, nbits = rotation // 8, rotation % 8
    mult = 1 << (8 - nbits)
    val, shift, carry = base, base + 4, base + 8
    if rotate:
        rot = [src[(i + nbytes) % 4] for i in range(4)]
    else:
        rot = [src[i + nbytes] if i + nbytes < 4 else None for i in range(4)]
    last_carry = None
    first_shift = None
    for i in range(3, -1, -1):
        b = rot[i] if rot[i] is not None else ZERO
        ch.sends.append(Lookup([V.const(A.B_SHRCARRY), _m(shift + i), _m(carry + i), b, V.const(nbits)], is_real_v,
                               KIND_BYTE))
        if i == 3:
            first_shift = main(shift + i)
        else:
            ch.assert_zero(main(val + i) - (main(shift + i) + last_carry * mult))
        last_carry = main(carry + i)
    if rotate:
        ch.assert_zero(main(val + 3) - (first_shift + last_carry * mult))
    else:
        ch.assert_zero(main(val + 3) - first_shift)


def _shr_carry_cols(x: np.ndarray, rotation: int, rotate: bool, byte_lookup):
    """populate of the fixed rotate/shift: (value, shift, carry) n x 4 each, with the ShrCarry lookups."""
    nbytes, nbits = rotation // 8, rotation % 8
    mult = 1 << (8 - nbits)
    xb = A._bytes(x.astype(np.uint32)).astype(np.int64)
    n = len(xb)
    if rotate:
        rb = xb[:, [(i + nbytes) % 4 for i in range(4)]]
    else:
        rb = np.zeros_like(xb)
        rb[:, :4 - nbytes] = xb[:, nbytes:]
    shift = rb >> nbits
    carry = rb & ((1 << nbits) - 1)
    value = np.zeros_like(xb)
    value[:, :3] = shift[:, :3] + carry[:, 1:] * mult
    value[:, 3] = shift[:, 3] + (carry[:, 0] * mult if rotate else 0)
    for i in range(4):
        byte_lookup(A.B_SHRCARRY, rb[:, i], np.full(n, nbits))
    return value, shift, carry


def _eval_xor(ch, a, b, base, is_real_v):
    """XorOperation::eval: value[4] at base."""
    for i in range(4):
        ch.sends.append(Lookup([V.const(A.B_XOR), _m(base + i), ZERO, a[i], b[i]], is_real_v, KIND_BYTE))


def _xor_cols(a: np.ndarray, b: np.ndarray, byte_lookup):
    ab, bb = A._bytes(a.astype(np.uint32)), A._bytes(b.astype(np.uint32))
    for i in range(4):
        byte_lookup(A.B_XOR, ab[:, i], bb[:, i])
    return ab ^ bb


def _u8_pairs(ch, cols, is_real_v):
    """slice_range_check_u8 (air/word.rs): U8Range lookups on byte pairs."""
    for k in range(0, len(cols), 2):
        ch.sends.append(Lookup([V.const(A.B_U8RANGE), ZERO, ZERO, cols[k], cols[k + 1]], is_real_v, KIND_BYTE))


def _u8_pairs_lookup(words_bytes, byte_lookup):
    for wb in words_bytes:
        byte_lookup(A.B_U8RANGE, wb[:, 0], wb[:, 1])
        byte_lookup(A.B_U8RANGE, wb[:, 2], wb[:, 3])


def _add_n_cols(words, byte_lookup):
    """Add4/Add5 populate: (value bytes, is_carry one-hot n x nin x 4, carry) with the U8 range lookups."""
    nin = len(words)
    wb = [A._bytes(w.astype(np.uint32)).astype(np.int64) for w in words]
    n = len(wb[0])
    value = np.zeros((n, 4), np.int64)
    carry = np.zeros((n, 4), np.int64)
    for i in range(4):
        s = sum(w[:, i] for w in wb) + (carry[:, i - 1] if i else 0)
        value[:, i], carry[:, i] = s & 0xFF, s >> 8
    onehot = np.zeros((n, nin, 4), np.int64)
    for k in range(nin):
        onehot[:, k, :] = carry == k
    _u8_pairs_lookup(wb + [value], byte_lookup)
    return value, onehot, carry


def _eval_and(ch, a, b, base, is_real_v):
    """AndOperation::eval: AND byte lookups, value[4] at base."""
    for i in range(4):
        ch.sends.append(Lookup([V.const(A.B_AND), _m(base + i), ZERO, a[i], b[i]], is_real_v, KIND_BYTE))


def _and_cols(a, b, byte_lookup):
    ab, bb = A._bytes(a.astype(np.uint32)), A._bytes(b.astype(np.uint32))
    for i in range(4):
        byte_lookup(A.B_AND, ab[:, i], bb[:, i])
    return ab & bb


# ---------------------------------------------------------------- ShaExtend
# ShaExtendCols (sha256/extend/columns.rs:17-75)
SE_SHARD, SE_CLK, SE_WPTR, SE_I, SE_C16, SE_C16S, SE_C16E, SE_C48, SE_C48S, SE_C48E = 0, 1, 2, 3, 4, 5, 7, 9, 12, 13
SE_W15, SE_RR7, SE_RR18, SE_RS3, SE_S0I, SE_S0 = 14, 23, 35, 47, 59, 63
SE_W2, SE_RR17, SE_RR19, SE_RS10, SE_S1I, SE_S1 = 67, 76, 88, 100, 112, 116
SE_W16, SE_W7, SE_S2, SE_WI, SE_REAL = 120, 129, 138, 162, 175
SE_WIDTH = 176
G16 = 148625052  # KoalaBear::two_adic_generator(4) = 3^((p-1)/16), order 16


def sha_extend_chip() -> ChipDesc:
    """ShaExtendChip::eval (extend/air.rs:29-221) with eval_flags (flags.rs:38-116)."""
    from .mips_core import ACC_VALUE, _eval_memory_access
    ch = ChipDesc("ShaExtend", prep_width=0, main_width=SE_WIDTH)
    M, N = main, main_next
    real = M(SE_REAL)
    real_v = _m(SE_REAL)
    # eval_flags
    ch.assert_zero(IS_FIRST * (M(SE_C16) - G16))
    ch.assert_zero(IS_FIRST * (M(SE_I) - 16))
    ch.assert_zero(IS_TRANSITION * (M(SE_C16) * G16 - N(SE_C16)))
    one = Expr.lift(1)
    _is_zero_op(ch, M(SE_C16) - G16, SE_C16S, one)
    _is_zero_op(ch, M(SE_C16) - 1, SE_C16E, one)
    c48 = [M(SE_C48 + i) for i in range(3)]
    ch.assert_zero(IS_FIRST * (c48[0] - 1))
    ch.assert_zero(IS_FIRST * c48[1])
    ch.assert_zero(IS_FIRST * c48[2])
    end16 = M(SE_C16E + 1)
    for i in range(3):
        ch.assert_zero(IS_TRANSITION * end16 * (c48[i] - N(SE_C48 + (i + 1) % 3)))
        ch.assert_zero(IS_TRANSITION * (1 - end16) * (c48[i] - N(SE_C48 + i)))
        _assert_bool(ch, c48[i])
    ch.assert_zero(M(SE_C16S + 1) * c48[0] * real - M(SE_C48S))
    ch.assert_zero(end16 * c48[2] * real - M(SE_C48E))
    ch.assert_zero(IS_TRANSITION * (end16 * c48[2]) * (N(SE_I) - 16))
    ch.assert_zero(IS_TRANSITION * (1 - end16 * c48[2]) * (M(SE_I) + 1 - N(SE_I)))
    # inputs carried through the 48-row cycle
    for col in (SE_SHARD, SE_CLK, SE_WPTR):
        ch.assert_zero(IS_TRANSITION * (1 - end16 * c48[2]) * (M(col) - N(col)))
    clk_terms = ((SE_CLK, 1), (SE_I, 1))
    for acc, off in ((SE_W15, 15), (SE_W2, 2), (SE_W16, 16), (SE_W7, 7)):
        addr = V([("main", SE_WPTR, 1), ("main", SE_I, 4)], -4 * off)
        _eval_memory_access(ch, acc, acc + ACC_VALUE, -16, addr, real, real_v, shard_col=SE_SHARD,
                            clk_terms=clk_terms)
    w15, w2 = _vw(SE_W15 + ACC_VALUE), _vw(SE_W2 + ACC_VALUE)
    _eval_shr_carry_op(ch, w15, 7, SE_RR7, real_v, True)
    _eval_shr_carry_op(ch, w15, 18, SE_RR18, real_v, True)
    _eval_shr_carry_op(ch, w15, 3, SE_RS3, real_v, False)
    _eval_xor(ch, _vw(SE_RR7), _vw(SE_RR18), SE_S0I, real_v)
    _eval_xor(ch, _vw(SE_S0I), _vw(SE_RS3), SE_S0, real_v)
    _eval_shr_carry_op(ch, w2, 17, SE_RR17, real_v, True)
    _eval_shr_carry_op(ch, w2, 19, SE_RR19, real_v, True)
    _eval_shr_carry_op(ch, w2, 10, SE_RS10, real_v, False)
    _eval_xor(ch, _vw(SE_RR17), _vw(SE_RR19), SE_S1I, real_v)
    _eval_xor(ch, _vw(SE_S1I), _vw(SE_RS10), SE_S1, real_v)
    ins = [_vw(SE_W16 + ACC_VALUE), _vw(SE_S0), _vw(SE_W7 + ACC_VALUE), _vw(SE_S1)]
    _add_n_eval_exprs(ch, ins, SE_S2, real, real_v)
    _eval_memory_access(ch, SE_WI + 4, SE_WI, -16, V([("main", SE_WPTR, 1), ("main", SE_I, 4)]), real, real_v,
                        shard_col=SE_SHARD, clk_terms=clk_terms)
    for i in range(4):
        ch.assert_zero(M(SE_WI + 4 + ACC_VALUE + i) - M(SE_S2 + i))
    ch.receives.append(Lookup([_m(SE_SHARD), _m(SE_CLK), V.const(syscall_id(SHA_EXTEND)), _m(SE_WPTR), ZERO],
                              _m(SE_C48S), KIND_SYSCALL))
    _assert_bool(ch, real)
    ch.assert_zero(IS_TRANSITION * (1 - M(SE_C48E)) * (real - N(SE_REAL)))
    ch.assert_zero(IS_LAST * real)
    return ch


def _add_n_eval_exprs(ch, ins_v, base, is_real, is_real_v):
    """_eval_add_n over words given as VirtualPairCols (lookups) with matching Exprs (constraints)."""
    ins_e = [[_v_expr(v) for v in w] for w in ins_v]
    nin = len(ins_v)
    for w in ins_v:
        _u8_pairs(ch, w, is_real_v)
    _u8_pairs(ch, [_m(base + i) for i in range(4)], is_real_v)
    M = main
    _assert_bool(ch, is_real)
    isc = lambda k, i: M(base + 4 + 4 * k + i)
    carry = lambda i: M(base + 4 + 4 * nin + i)
    for i in range(4):
        for k in range(nin):
            _assert_bool(ch, isc(k, i), is_real)
        ch.assert_zero(is_real * (sum((isc(k, i) for k in range(1, nin)), isc(0, i)) - 1))
    for i in range(4):
        ch.assert_zero(is_real * (carry(i) - sum((isc(k, i) * k for k in range(2, nin)), isc(1, i))))
    for i in range(4):
        over = sum((w[i] for w in ins_e[1:]), ins_e[0][i]) - M(base + i)
        if i > 0:
            over = over + carry(i - 1)
        ch.assert_zero(is_real * (carry(i) * 256 - over))


def _v_expr(v: V) -> Expr:
    """A single-column VirtualPairCol as an Expr."""
    assert len(v.terms) == 1 and v.terms[0][0] == "main" and v.terms[0][2] == 1 and v.constant == 0
    return main(v.terms[0][1])


def _flags_16_48(rows: np.ndarray, real: np.ndarray):
    """ShaExtendCols::populate_flags(i) for row indices i (flags.rs:13-34)."""
    i = np.asarray(rows, np.int64)
    g = np.ones(16, np.int64)
    for k in range(1, 16):
        g[k] = g[k - 1] * G16 % P
    c16 = g[(i + 1) % 16]
    s_inv, s_res = _is_zero_cols(c16 - G16)
    e_inv, e_res = _is_zero_cols(c16 - 1)
    j = 16 + i % 48
    c48 = np.stack([(j >= 16) & (j < 32), (j >= 32) & (j < 48), (j >= 48) & (j < 64)], axis=1).astype(np.int64)
    return c16, (s_inv, s_res), (e_inv, e_res), j, c48, c48[:, 0] * s_res * real, c48[:, 2] * e_res * real


def sha_extend_trace(events, byte_lookup) -> np.ndarray:
    """ShaExtendChip::generate_trace + event_to_rows (extend/trace.rs:29-150).  events: list of dicts with
    shard, clk, w_ptr and, per row j < 48, the four reads (value, prev_shard, prev_clk) 'r15', 'r2', 'r16',
    'r7' (48 x 3 each) and the write (prev_value, value, prev_shard, prev_clk) 'wr' (48 x 4)."""
    from .mips_core import ACC_VALUE, _access_cols
    ne = len(events)
    n = 48 * ne
    h = 1 << max(2, (n - 1).bit_length()) if n else 4
    h = max(h, 16)
    t = np.zeros((h, SE_WIDTH), np.uint32)
    rows = np.arange(h)
    real = (rows < n).astype(np.int64)
    c16, (si, sr), (ei, er), j, c48, c48s, c48e = _flags_16_48(rows, real)
    t[:, SE_I], t[:, SE_C16] = j, c16
    t[:, SE_C16S], t[:, SE_C16S + 1], t[:, SE_C16E], t[:, SE_C16E + 1] = si, sr, ei, er
    t[:, SE_C48:SE_C48 + 3] = c48
    t[:, SE_C48S], t[:, SE_C48E] = c48s, c48e
    if ne == 0:
        return t
    cat = lambda k: np.concatenate([np.asarray(e[k], np.int64).reshape(48, -1) for e in events])
    shard = np.repeat([e["shard"] for e in events], 48).astype(np.int64)
    clk0 = np.repeat([e["clk"] for e in events], 48).astype(np.int64)
    clk = clk0 + np.tile(np.arange(48), ne)
    r = np.arange(n)
    t[:n, SE_SHARD], t[:n, SE_CLK] = shard, clk0
    t[:n, SE_WPTR] = np.repeat([e["w_ptr"] for e in events], 48)
    sel = np.ones(n, bool)
    vals = {}
    for key, acc in (("r15", SE_W15), ("r2", SE_W2), ("r16", SE_W16), ("r7", SE_W7)):
        rd = cat(key)
        vals[key] = rd[:, 0].astype(np.uint32)
        _access_cols(t, r, acc + ACC_VALUE, vals[key], rd[:, 1:3], shard, clk, sel, byte_lookup)
    w15, w2 = vals["r15"], vals["r2"]
    rr = lambda x, s: ((x >> np.uint32(s)) | (x << np.uint32(32 - s))).astype(np.uint32)
    s0 = rr(w15, 7) ^ rr(w15, 18) ^ (w15 >> np.uint32(3))
    s1 = rr(w2, 17) ^ rr(w2, 19) ^ (w2 >> np.uint32(10))
    parts = {}
    for key, base, x, rot, is_rot in (("rr7", SE_RR7, w15, 7, True), ("rr18", SE_RR18, w15, 18, True),
                                      ("rs3", SE_RS3, w15, 3, False)):
        v, sh, ca = _shr_carry_cols(x, rot, is_rot, byte_lookup)
        t[:n, base:base + 4], t[:n, base + 4:base + 8], t[:n, base + 8:base + 12] = v, sh, ca
        parts[key] = _word_of(v)
    t[:n, SE_S0I:SE_S0I + 4] = _xor_cols(parts["rr7"], parts["rr18"], byte_lookup)
    t[:n, SE_S0:SE_S0 + 4] = _xor_cols(parts["rr7"] ^ parts["rr18"], parts["rs3"], byte_lookup)
    for key, base, x, rot, is_rot in (("rr17", SE_RR17, w2, 17, True), ("rr19", SE_RR19, w2, 19, True),
                                      ("rs10", SE_RS10, w2, 10, False)):
        v, sh, ca = _shr_carry_cols(x, rot, is_rot, byte_lookup)
        t[:n, base:base + 4], t[:n, base + 4:base + 8], t[:n, base + 8:base + 12] = v, sh, ca
        parts[key] = _word_of(v)
    t[:n, SE_S1I:SE_S1I + 4] = _xor_cols(parts["rr17"], parts["rr19"], byte_lookup)
    t[:n, SE_S1:SE_S1 + 4] = _xor_cols(parts["rr17"] ^ parts["rr19"], parts["rs10"], byte_lookup)
    assert np.array_equal(parts["rr7"] ^ parts["rr18"] ^ parts["rs3"], s0)
    assert np.array_equal(parts["rr17"] ^ parts["rr19"] ^ parts["rs10"], s1)
    value, onehot, carry = _add_n_cols([vals["r16"], s0, vals["r7"], s1], byte_lookup)
    t[:n, SE_S2:SE_S2 + 4] = value
    t[:n, SE_S2 + 4:SE_S2 + 20] = onehot.reshape(n, 16)
    t[:n, SE_S2 + 20:SE_S2 + 24] = carry
    wr = cat("wr")
    assert np.array_equal(_word_of(value), wr[:, 1].astype(np.uint32))
    t[:n, SE_WI:SE_WI + 4] = A._bytes(wr[:, 0].astype(np.uint32))
    _access_cols(t, r, SE_WI + 4 + ACC_VALUE, wr[:, 1].astype(np.uint32), wr[:, 2:4], shard, clk, sel, byte_lookup)
    t[:n, SE_REAL] = 1
    return t


def _word_of(b: np.ndarray) -> np.ndarray:
    b = np.asarray(b, np.uint32)
    return (b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16) | (b[:, 3] << 24)).astype(np.uint32)


# ---------------------------------------------------------------- ShaCompress
# ShaCompressCols (sha256/compress/columns.rs:25-110)
SC2_SHARD, SC2_CLK, SC2_WPTR, SC2_HPTR, SC2_START, SC2_OCTET, SC2_OCTNUM = 0, 1, 2, 3, 4, 5, 13
SC2_MEM, SC2_ADDR = 23, 36  # MemoryReadWriteCols: prev_value[4], then the access (value[4], ...)
SC2_A, SC2_K = 37, 69  # a..h: 37, 41, .., 65
SC2_ERR6, SC2_ERR11, SC2_ERR25, SC2_S1I, SC2_S1 = 73, 85, 97, 109, 113
SC2_EANDF, SC2_ENOT, SC2_ENOTG, SC2_CH, SC2_TEMP1 = 117, 121, 125, 129, 133
SC2_ARR2, SC2_ARR13, SC2_ARR22, SC2_S0I, SC2_S0 = 161, 173, 185, 197, 201
SC2_AANDB, SC2_AANDC, SC2_BANDC, SC2_MAJI, SC2_MAJ = 205, 209, 213, 217, 221
SC2_TEMP2, SC2_DT1, SC2_T1T2, SC2_FOP, SC2_FADD = 225, 232, 239, 246, 250
SC2_INIT, SC2_COMP, SC2_FIN, SC2_LAST, SC2_REAL = 257, 258, 259, 260, 261
SC2_WIDTH = 262
SHA_K = [0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
         0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
         0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
         0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
         0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
         0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
         0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
         0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2]


def _eval_add(ch, a_base, b_base, base, is_real, is_real_v):
    """AddOperation::eval (operations/add.rs): value[4], carry[3] at base."""
    M = main
    a, b = _w(a_base), _w(b_base)
    val, carry = _w(base), [M(base + 4 + i) for i in range(3)]
    ov = [a[0] + b[0] - val[0]] + [a[i] + b[i] - val[i] + carry[i - 1] for i in (1, 2, 3)]
    ch.assert_zero(is_real * (ov[3] * (ov[3] - 256)))
    for i in range(3):
        ch.assert_zero(is_real * (carry[i] * (ov[i] - 256)))
    for i in range(3):
        ch.assert_zero(is_real * ((carry[i] - 1) * ov[i]))
    for i in range(3):
        _assert_bool(ch, carry[i], is_real)
    _assert_bool(ch, is_real, is_real)
    for w in (a_base, b_base, base):
        _u8_pairs(ch, _vw(w), is_real_v)


def _add_cols(a, b, byte_lookup):
    """AddOperation::populate: (value bytes, carry n x 3) and the U8 range lookups of a, b, value."""
    ab, bb = A._bytes(a.astype(np.uint32)).astype(np.int64), A._bytes(b.astype(np.uint32)).astype(np.int64)
    val = A._bytes(((a.astype(np.uint64) + b.astype(np.uint64)) & M32).astype(np.uint32)).astype(np.int64)
    carry = np.zeros((len(ab), 3), np.int64)
    c = np.zeros(len(ab), np.int64)
    for i in range(3):
        c = (ab[:, i] + bb[:, i] + c) >> 8
        carry[:, i] = c
    _u8_pairs_lookup([ab, bb, val], byte_lookup)
    return val, carry


def sha_compress_chip() -> ChipDesc:
    """ShaCompressChip::eval (compress/air.rs:36-507): eval_control_flow_flags, eval_memory,
    eval_compression_ops, eval_finalize_ops, then the start flag and the syscall receive."""
    from .mips_core import ACC_VALUE, _eval_memory_access
    ch = ChipDesc("ShaCompress", prep_width=0, main_width=SC2_WIDTH)
    M, N = main, main_next
    octet = [M(SC2_OCTET + i) for i in range(8)]
    onum = [M(SC2_OCTNUM + i) for i in range(10)]
    nocte = lambda i: N(SC2_OCTET + i)
    nonum = lambda i: N(SC2_OCTNUM + i)
    real, init, comp, fin, last = M(SC2_REAL), M(SC2_INIT), M(SC2_COMP), M(SC2_FIN), M(SC2_LAST)
    var = lambda i: _w(SC2_A + 4 * i)
    nvar = lambda i: [N(SC2_A + 4 * i + j) for j in range(4)]
    mem_prev = _w(SC2_MEM)
    mem_val = _w(SC2_MEM + 4 + ACC_VALUE)
    # eval_control_flow_flags
    for x in octet:
        _assert_bool(ch, x)
    ch.assert_zero(sum(octet[1:], octet[0]) - 1)
    ch.assert_zero(IS_FIRST * (octet[0] - 1))
    for i in range(8):
        ch.assert_zero(IS_TRANSITION * octet[i] * (nocte((i + 1) % 8) - 1))
    for x in onum:
        _assert_bool(ch, x)
    ch.assert_zero(sum(onum[1:], onum[0]) - 1)
    ch.assert_zero(IS_FIRST * (onum[0] - 1))
    for i in range(10):
        ch.assert_zero(IS_TRANSITION * (1 - octet[7]) * (onum[i] - nonum(i)))
    for i in range(10):
        ch.assert_zero(IS_TRANSITION * octet[7] * (onum[i] - nonum((i + 1) % 10)))
    for i in range(8):
        for j in range(4):
            ch.assert_zero(IS_TRANSITION * (onum[0] + onum[9] * (1 - octet[7])) * (var(i)[j] - nvar(i)[j]))
        for j in range(4):
            ch.assert_zero(IS_TRANSITION * (onum[0] * octet[i]) * (var(i)[j] - mem_val[j]))
    ch.assert_zero(init - onum[0] * real)
    ch.assert_zero(comp - sum(onum[2:9], onum[1]) * real)
    ch.assert_zero(fin - onum[9] * real)
    ch.assert_zero(last - octet[7] * onum[9])
    for col in (SC2_SHARD, SC2_CLK, SC2_WPTR, SC2_HPTR):
        ch.assert_zero(IS_TRANSITION * real * (1 - last) * (M(col) - N(col)))
    _assert_bool(ch, real)
    ch.assert_zero(IS_TRANSITION * real * (1 - last) * (N(SC2_REAL) - 1))
    ch.assert_zero(IS_TRANSITION * (1 - real) * N(SC2_REAL))
    ch.assert_zero(IS_LAST * real)
    # eval_memory
    do_check_v = V([("main", SC2_INIT, 1), ("main", SC2_COMP, 1), ("main", SC2_FIN, 1)])
    _eval_memory_access(ch, SC2_MEM + 4, SC2_MEM, 0, SC2_ADDR, init + comp + fin, do_check_v, shard_col=SC2_SHARD,
                        clk_terms=((SC2_CLK, 1), (SC2_FIN, 1)))
    cycle_num = sum((onum[i] * i for i in range(2, 10)), onum[1])
    cycle_step = sum((octet[i] * i for i in range(2, 8)), octet[1])
    ch.assert_zero(init * (M(SC2_ADDR) - (M(SC2_HPTR) + cycle_step * 4)))
    ch.assert_zero(comp * (M(SC2_ADDR) - (M(SC2_WPTR) + ((cycle_num - 1) * 8 + cycle_step) * 4)))
    ch.assert_zero(fin * (M(SC2_ADDR) - (M(SC2_HPTR) + cycle_step * 4)))
    for i in range(8):
        for j in range(4):
            ch.assert_zero(init * octet[i] * (var(i)[j] - mem_prev[j]))
        for j in range(4):
            ch.assert_zero(init * octet[i] * (var(i)[j] - mem_val[j]))
    for j in range(4):
        ch.assert_zero(comp * (mem_prev[j] - mem_val[j]))
    for j in range(4):
        ch.assert_zero(fin * (mem_val[j] - M(SC2_FADD + j)))
    # eval_compression_ops
    for i in range(64):
        sel = onum[i // 8 + 1] * octet[i % 8]
        for j in range(4):
            ch.assert_zero(sel * (M(SC2_K + j) - ((SHA_K[i] >> (8 * j)) & 0xFF)))
    comp_v = _m(SC2_COMP)
    e_v, a_v = _vw(SC2_A + 16), _vw(SC2_A)
    for rot, base in ((6, SC2_ERR6), (11, SC2_ERR11), (25, SC2_ERR25)):
        _eval_shr_carry_op(ch, e_v, rot, base, comp_v, True)
    _eval_xor(ch, _vw(SC2_ERR6), _vw(SC2_ERR11), SC2_S1I, comp_v)
    _eval_xor(ch, _vw(SC2_S1I), _vw(SC2_ERR25), SC2_S1, comp_v)
    _eval_and(ch, e_v, _vw(SC2_A + 20), SC2_EANDF, comp_v)
    _u8_pairs(ch, e_v, comp_v)  # NotOperation::eval
    for i in range(4):
        ch.assert_zero(comp * (M(SC2_ENOT + i) + M(SC2_A + 16 + i) - 255))
    _eval_and(ch, _vw(SC2_ENOT), _vw(SC2_A + 24), SC2_ENOTG, comp_v)
    _eval_xor(ch, _vw(SC2_EANDF), _vw(SC2_ENOTG), SC2_CH, comp_v)
    _add_n_eval_exprs(ch, [_vw(SC2_A + 28), _vw(SC2_S1), _vw(SC2_CH), _vw(SC2_K), _vw(SC2_MEM + 4 + ACC_VALUE)],
                      SC2_TEMP1, comp, comp_v)
    for rot, base in ((2, SC2_ARR2), (13, SC2_ARR13), (22, SC2_ARR22)):
        _eval_shr_carry_op(ch, a_v, rot, base, comp_v, True)
    _eval_xor(ch, _vw(SC2_ARR2), _vw(SC2_ARR13), SC2_S0I, comp_v)
    _eval_xor(ch, _vw(SC2_S0I), _vw(SC2_ARR22), SC2_S0, comp_v)
    _eval_and(ch, a_v, _vw(SC2_A + 4), SC2_AANDB, comp_v)
    _eval_and(ch, a_v, _vw(SC2_A + 8), SC2_AANDC, comp_v)
    _eval_and(ch, _vw(SC2_A + 4), _vw(SC2_A + 8), SC2_BANDC, comp_v)
    _eval_xor(ch, _vw(SC2_AANDB), _vw(SC2_AANDC), SC2_MAJI, comp_v)
    _eval_xor(ch, _vw(SC2_MAJI), _vw(SC2_BANDC), SC2_MAJ, comp_v)
    _eval_add(ch, SC2_S0, SC2_MAJ, SC2_TEMP2, comp, comp_v)
    _eval_add(ch, SC2_A + 12, SC2_TEMP1, SC2_DT1, comp, comp_v)
    _eval_add(ch, SC2_TEMP1, SC2_TEMP2, SC2_T1T2, comp, comp_v)
    # h := g, g := f, f := e, e := d + temp1, d := c, c := b, b := a, a := temp1 + temp2
    for dst, src in ((7, SC2_A + 24), (6, SC2_A + 20), (5, SC2_A + 16), (4, SC2_DT1), (3, SC2_A + 8), (2, SC2_A + 4),
                     (1, SC2_A), (0, SC2_T1T2)):
        for j in range(4):
            ch.assert_zero(IS_TRANSITION * comp * (nvar(dst)[j] - M(src + j)))
    # eval_finalize_ops
    for j in range(4):
        filt = sum((octet[i] * var(i)[j] for i in range(1, 8)), octet[0] * var(0)[j])
        ch.assert_zero(fin * (filt - M(SC2_FOP + j)))
    _eval_add(ch, SC2_MEM, SC2_FOP, SC2_FADD, fin, _m(SC2_FIN))
    ch.assert_zero(M(SC2_START) - real * octet[0] * onum[0])
    ch.receives.append(Lookup([_m(SC2_SHARD), _m(SC2_CLK), V.const(syscall_id(SHA_COMPRESS)), _m(SC2_WPTR),
                               _m(SC2_HPTR)], _m(SC2_START), KIND_SYSCALL))
    return ch


def sha_compress_trace(events, byte_lookup) -> np.ndarray:
    """ShaCompressChip::generate_trace + event_to_rows (compress/trace.rs:32-305).  events: dicts with
    shard, clk, w_ptr, h_ptr, 'hr' (8 x 3 reads of h: value, prev_shard, prev_clk), 'wr' (64 x 3 reads of w),
    'hw' (8 x 4 writes: prev_value, value, prev_shard, prev_clk)."""
    from .mips_core import ACC_VALUE, _access_cols
    ne = len(events)
    n = 80 * ne
    h = max(16, 1 << max(0, (n - 1).bit_length())) if n else 16
    t = np.zeros((h, SC2_WIDTH), np.uint32)
    rows = np.arange(h)
    # octet / octet_num for every row (real rows restart per event, padding continues from 0)
    pos = np.where(rows < n, rows % 80, (rows - n) % 80)
    oc, on = pos % 8, pos // 8
    t[rows, SC2_OCTET + oc] = 1
    t[rows, SC2_OCTNUM + on] = 1
    compr = (on >= 1) & (on <= 8)
    kidx = np.where(compr, (on - 1) * 8 + oc, 0)
    kw = np.asarray(SHA_K, np.uint32)[kidx]
    t[compr, SC2_K:SC2_K + 4] = A._bytes(kw[compr])
    t[:, SC2_LAST] = (oc == 7) & (on == 9)
    if ne == 0:
        return t
    real = rows < n
    t[real, SC2_REAL] = 1
    t[real & (on == 0), SC2_INIT] = 1
    t[real & compr, SC2_COMP] = 1
    t[real & (on == 9), SC2_FIN] = 1
    t[real & (on == 0) & (oc == 0), SC2_START] = 1
    rep = lambda key: np.repeat(np.asarray([e[key] for e in events], np.int64), 80)
    shard, clk0 = rep("shard"), rep("clk")
    t[:n, SC2_SHARD], t[:n, SC2_CLK], t[:n, SC2_WPTR], t[:n, SC2_HPTR] = shard, clk0, rep("w_ptr"), rep("h_ptr")
    hr = np.asarray([e["hr"] for e in events], np.int64)  # E x 8 x 3
    wr = np.asarray([e["wr"] for e in events], np.int64)  # E x 64 x 3
    hw = np.asarray([e["hw"] for e in events], np.int64)  # E x 8 x 4
    # the memory access of each row: init reads h[j], compression reads w[j], finalize writes h[j]
    acc_val = np.concatenate([hr[:, :, 0], wr[:, :, 0], hw[:, :, 1]], axis=1).reshape(-1)
    acc_prevval = np.concatenate([hr[:, :, 0], wr[:, :, 0], hw[:, :, 0]], axis=1).reshape(-1)
    acc_prev = np.concatenate([hr[:, :, 1:3], wr[:, :, 1:3], hw[:, :, 2:4]], axis=1).reshape(-1, 2)
    fin_r = (on[:n] == 9)
    clk = clk0 + fin_r
    t[:n, SC2_MEM:SC2_MEM + 4] = A._bytes(acc_prevval.astype(np.uint32))
    _access_cols(t, np.arange(n), SC2_MEM + 4 + ACC_VALUE, acc_val.astype(np.uint32), acc_prev, shard, clk,
                 np.ones(n, bool), byte_lookup)
    hp, wp = rep("h_ptr"), rep("w_ptr")
    pe = pos[:n]
    t[:n, SC2_ADDR] = np.where(pe < 8, hp + 4 * pe, np.where(pe < 72, wp + 4 * (pe - 8), hp + 4 * (pe - 72)))
    # a..h per row: the state before each round (init rows hold the initial state, finalize rows the last)
    st = np.zeros((ne, 80, 8), np.int64)
    cur = hr[:, :, 0].copy()
    st[:, :8, :] = cur[:, None, :]
    E = np.arange(ne)
    comp_rows = np.arange(8, 72)
    wv = wr[:, :, 0]
    ops = {k: [] for k in ("e", "f", "g", "h", "a", "b", "c", "d", "w")}
    for j in range(64):
        st[:, 8 + j, :] = cur
        a, b, c, d, e, f, g, hh = (cur[:, i] for i in range(8))
        s1 = _rotr_np(e, 6) ^ _rotr_np(e, 11) ^ _rotr_np(e, 25)
        chv = (e & f) ^ (~e & g & M32)
        t1 = (hh + s1 + chv + SHA_K[j] + wv[:, j]) & M32
        s0 = _rotr_np(a, 2) ^ _rotr_np(a, 13) ^ _rotr_np(a, 22)
        maj = (a & b) ^ (a & c) ^ (b & c)
        t2 = (s0 + maj) & M32
        cur = np.stack([(t1 + t2) & M32, a, b, c, (d + t1) & M32, e, f, g], axis=1)
    st[:, 72:, :] = cur[:, None, :]
    assert np.array_equal((hr[:, :, 0] + cur) & M32, hw[:, :, 1])
    stf = st.reshape(n, 8)
    for i in range(8):
        t[:n, SC2_A + 4 * i:SC2_A + 4 * i + 4] = A._bytes(stf[:, i].astype(np.uint32))
    # compression-row operations
    cr = (np.arange(ne)[:, None] * 80 + comp_rows[None, :]).reshape(-1)
    sc = stf[cr]
    a, b, c, d, e, f, g, hh = (sc[:, i].astype(np.uint32) for i in range(8))
    w_j = wv.reshape(-1).astype(np.uint32)
    kj = np.tile(np.asarray(SHA_K, np.uint32), ne)
    put = lambda base, v: t.__setitem__((cr, slice(base, base + v.shape[1])), v)
    parts = {}
    for key, base, x, rot in (("e6", SC2_ERR6, e, 6), ("e11", SC2_ERR11, e, 11), ("e25", SC2_ERR25, e, 25),
                              ("a2", SC2_ARR2, a, 2), ("a13", SC2_ARR13, a, 13), ("a22", SC2_ARR22, a, 22)):
        v, sh, ca = _shr_carry_cols(x, rot, True, byte_lookup)
        put(base, v), put(base + 4, sh), put(base + 8, ca)
        parts[key] = _word_of(v)
    put(SC2_S1I, _xor_cols(parts["e6"], parts["e11"], byte_lookup))
    s1 = parts["e6"] ^ parts["e11"] ^ parts["e25"]
    put(SC2_S1, _xor_cols(parts["e6"] ^ parts["e11"], parts["e25"], byte_lookup))
    eandf = e & f
    put(SC2_EANDF, _and_cols(e, f, byte_lookup))
    enot = (~e).astype(np.uint32)
    put(SC2_ENOT, A._bytes(enot))
    _u8_pairs_lookup([A._bytes(e).astype(np.int64)], byte_lookup)
    enotg = enot & g
    put(SC2_ENOTG, _and_cols(enot, g, byte_lookup))
    chv = eandf ^ enotg
    put(SC2_CH, _xor_cols(eandf, enotg, byte_lookup))
    val, onehot, carry = _add_n_cols([hh, s1, chv, kj, w_j], byte_lookup)
    put(SC2_TEMP1, val), put(SC2_TEMP1 + 4, onehot.reshape(-1, 20)), put(SC2_TEMP1 + 24, carry)
    t1 = _word_of(val)
    put(SC2_S0I, _xor_cols(parts["a2"], parts["a13"], byte_lookup))
    s0 = parts["a2"] ^ parts["a13"] ^ parts["a22"]
    put(SC2_S0, _xor_cols(parts["a2"] ^ parts["a13"], parts["a22"], byte_lookup))
    put(SC2_AANDB, _and_cols(a, b, byte_lookup))
    put(SC2_AANDC, _and_cols(a, c, byte_lookup))
    put(SC2_BANDC, _and_cols(b, c, byte_lookup))
    put(SC2_MAJI, _xor_cols(a & b, a & c, byte_lookup))
    maj = (a & b) ^ (a & c) ^ (b & c)
    put(SC2_MAJ, _xor_cols((a & b) ^ (a & c), b & c, byte_lookup))
    v2, c2 = _add_cols(s0, maj, byte_lookup)
    put(SC2_TEMP2, v2), put(SC2_TEMP2 + 4, c2)
    t2 = _word_of(v2)
    v3, c3 = _add_cols(d, t1, byte_lookup)
    put(SC2_DT1, v3), put(SC2_DT1 + 4, c3)
    v4, c4 = _add_cols(t1, t2, byte_lookup)
    put(SC2_T1T2, v4), put(SC2_T1T2 + 4, c4)
    # finalize rows: finalized operand = state word j, finalize_add = h[j] + operand
    fr = (np.arange(ne)[:, None] * 80 + 72 + np.arange(8)[None, :]).reshape(-1)
    opnd = cur.reshape(-1).astype(np.uint32)
    t[fr, SC2_FOP:SC2_FOP + 4] = A._bytes(opnd)
    v5, c5 = _add_cols(hr[:, :, 0].reshape(-1).astype(np.uint32), opnd, byte_lookup)
    t[fr, SC2_FADD:SC2_FADD + 4] = v5
    t[fr, SC2_FADD + 4:SC2_FADD + 7] = c5
    return t


def _rotr_np(x, s):
    x = np.asarray(x, np.int64)
    return ((x >> s) | (x << (32 - s))) & M32


# ---------------------------------------------------------------- SysLinux
# SysLinuxCols (sys_linux/columns.rs:12-62)
SL_SHARD, SL_CLK, SL_ID, SL_A0, SL_A1, SL_RES, SL_IO, SL_OUT = 0, 1, 2, 3, 7, 11, 15, 28
SL_A0_0, SL_A0_1, SL_A0_2, SL_MMAP, SL_MMAP2, SL_MMAP_A0_0, SL_PAGE_OFF, SL_OFF_0, SL_UPPER = range(41, 50)
SL_CLONE, SL_EXIT, SL_BRK, SL_GT = 50, 51, 52, 53  # GtColsBytes: byte_flags[4], a_cmp, b_cmp, result
SL_FCNTL, SL_A1_1, SL_A1_3, SL_F_A1_1, SL_F_A1_3, SL_READ, SL_WRITE, SL_NOP, SL_REAL = range(60, 69)
SL_WIDTH = 69


def _eval_gt_bytes(ch, a_base, b_base, base, is_real, is_real_v):
    """GtColsBytes::eval (operations/cmp.rs:74-137): a > b over little-endian bytes."""
    M = main
    _u8_pairs(ch, _vw(a_base), is_real_v)
    _u8_pairs(ch, _vw(b_base), is_real_v)
    flags = [M(base + i) for i in range(4)]
    for f in flags:
        _assert_bool(ch, f, is_real)
    _assert_bool(ch, sum(flags[1:], flags[0]), is_real)
    visited = Expr.lift(0)
    first_gt = Expr.lift(0)
    b_cmp = Expr.lift(0)
    for i in range(3, -1, -1):
        visited = visited + flags[i]
        first_gt = first_gt + M(a_base + i) * flags[i]
        b_cmp = b_cmp + M(b_base + i) * flags[i]
        ch.assert_zero((1 - visited) * is_real * (M(a_base + i) - M(b_base + i)))
    ch.assert_zero(is_real * (M(base + 4) - first_gt))
    ch.assert_zero(is_real * (M(base + 5) - b_cmp))
    ch.sends.append(Lookup([V.const(A.B_LTU), _m(base + 6), ZERO, _m(base + 5), _m(base + 4)], is_real_v, KIND_BYTE))


def sys_linux_chip() -> ChipDesc:
    """SysLinuxChip::eval (sys_linux/air.rs:33-323): eval_brk, eval_clone, eval_exit_group, eval_fnctl,
    eval_read, eval_write, eval_mmap, eval_nop, the A3 write, flag checks, the syscall receive."""
    from .mips_core import ACC_VALUE, _eval_memory_access
    ch = ChipDesc("SysLinux", prep_width=0, main_width=SL_WIDTH)
    M = main
    f = lambda c: M(c)
    a0, a1, res = _w(SL_A0), _w(SL_A1), _w(SL_RES)
    io_prev, io_val = _w(SL_IO), _w(SL_IO + 4 + ACC_VALUE)
    out = _w(SL_OUT + 4 + ACC_VALUE)
    mem = lambda acc, reg, chk, chk_v: _eval_memory_access(ch, acc + 4, acc, 0, V.const(reg), chk, chk_v,
                                                           shard_col=SL_SHARD, clk_terms=((SL_CLK, 1),))
    word_is = lambda when, w, k: [ch.assert_zero(when * (w[j] - ((k >> (8 * j)) & 0xFF))) for j in range(4)]
    a0s = f(SL_A0_0) + f(SL_A0_1) + f(SL_A0_2)
    # eval_brk
    mem(SL_IO, REG_BRK, f(SL_BRK), _m(SL_BRK))
    _eval_gt_bytes(ch, SL_A0, SL_IO + 4 + ACC_VALUE, SL_GT, f(SL_BRK), _m(SL_BRK))
    gt = f(SL_GT + 6)
    for j in range(4):
        ch.assert_zero(f(SL_BRK) * gt * (res[j] - a0[j]))
    for j in range(4):
        ch.assert_zero(f(SL_BRK) * (1 - gt) * (res[j] - io_prev[j]))
    word_is(f(SL_BRK), out, 0)
    # eval_clone
    word_is(f(SL_CLONE), out, 0)
    word_is(f(SL_CLONE), res, 1)
    # eval_exit_group
    word_is(f(SL_EXIT), out, 0)
    # eval_fnctl
    fc = f(SL_FCNTL)
    ch.assert_zero(fc * f(SL_A1_1) * (a1[0] - 1))
    ch.assert_zero(fc * f(SL_A1_3) * (a1[0] - 3))
    for j in (1, 2, 3):
        ch.assert_zero(fc * (f(SL_A1_1) + f(SL_A1_3)) * a1[j])
    ch.assert_zero(f(SL_F_A1_3) * (f(SL_A1_3) * fc - 1))
    ch.assert_zero(f(SL_F_A1_1) * (f(SL_A1_1) * fc - 1))
    word_is(f(SL_F_A1_3) * f(SL_A0_0), res, 0)
    word_is(f(SL_F_A1_3) * (f(SL_A0_1) + f(SL_A0_2)), res, 1)
    word_is(f(SL_F_A1_3) * (1 - a0s), res, M32)
    word_is(fc * (1 - (f(SL_A1_3) + f(SL_A1_1))), res, M32)
    word_is((f(SL_F_A1_3) + f(SL_F_A1_1)) * a0s, out, 0)
    word_is((f(SL_F_A1_3) + f(SL_F_A1_1)) * (1 - a0s), out, MIPS_EBADF)
    word_is(fc * (1 - (f(SL_A1_3) + f(SL_A1_1))), out, MIPS_EBADF)
    # eval_read
    word_is(f(SL_READ) * f(SL_A0_0), res, 0)
    word_is(f(SL_READ) * f(SL_A0_0), out, 0)
    word_is(f(SL_READ) * (1 - f(SL_A0_0)), res, M32)
    word_is(f(SL_READ) * (1 - f(SL_A0_0)), out, MIPS_EBADF)
    # eval_write
    mem(SL_IO, REG_A2, f(SL_WRITE), _m(SL_WRITE))
    for j in range(4):
        ch.assert_zero(f(SL_WRITE) * (res[j] - io_val[j]))
    word_is(f(SL_WRITE), out, 0)
    # eval_mmap
    mm = f(SL_MMAP)
    ch.assert_zero(mm * f(SL_OFF_0) * f(SL_PAGE_OFF))
    ch.assert_zero(mm * (f(SL_PAGE_OFF) + f(SL_UPPER) - _reduce(SL_A1)))
    size = f(SL_UPPER) + PAGE_SIZE * (1 - f(SL_OFF_0))
    ch.assert_zero(mm * f(SL_A0_0) * (_reduce(SL_IO + 4 + ACC_VALUE) - (size + _reduce(SL_IO))))
    ch.assert_zero(f(SL_MMAP_A0_0) * (mm * f(SL_A0_0) - 1))
    for j in range(4):
        ch.assert_zero(f(SL_MMAP_A0_0) * f(SL_A0_0) * (io_prev[j] - res[j]))
    mem(SL_IO, REG_HEAP, f(SL_MMAP_A0_0), _m(SL_MMAP_A0_0))
    for j in range(4):
        ch.assert_zero(mm * (1 - f(SL_A0_0)) * (a0[j] - res[j]))
    # eval_nop
    word_is(f(SL_NOP), out, 0)
    word_is(f(SL_NOP), res, 0)
    # the A3 write
    mem(SL_OUT, REG_A3, f(SL_REAL), _m(SL_REAL))
    for c in (SL_A0_0, SL_A0_1, SL_A0_2, SL_MMAP, SL_MMAP2, SL_MMAP_A0_0, SL_OFF_0, SL_CLONE, SL_EXIT, SL_BRK,
              SL_FCNTL, SL_A1_1, SL_A1_3, SL_F_A1_1, SL_F_A1_3, SL_READ, SL_WRITE, SL_NOP, SL_REAL):
        _assert_bool(ch, f(c))
    real = f(SL_REAL)
    ch.assert_zero(real * f(SL_A0_0) * a0[0])
    ch.assert_zero(real * f(SL_A0_1) * (a0[0] - 1))
    ch.assert_zero(real * f(SL_A0_2) * (a0[0] - 2))
    for j in (1, 2, 3):
        ch.assert_zero(real * a0s * a0[j])
    sid = f(SL_ID)
    ch.assert_zero(mm * (1 - f(SL_MMAP2)) * (sid - SYS_MMAP))
    ch.assert_zero(f(SL_MMAP2) * (sid - SYS_MMAP2))
    ch.assert_zero(f(SL_MMAP2) * (mm - 1))
    for col, code in ((SL_CLONE, SYS_CLONE), (SL_EXIT, SYS_EXT_GROUP), (SL_BRK, SYS_BRK), (SL_FCNTL, SYS_FCNTL),
                      (SL_READ, SYS_READ), (SL_WRITE, SYS_WRITE)):
        ch.assert_zero(f(col) * (sid - code))
    kinds = [f(c) for c in (SL_CLONE, SL_EXIT, SL_BRK, SL_FCNTL, SL_READ, SL_WRITE, SL_NOP)]
    ch.assert_zero(real * (sum(kinds, mm) - 1))
    ch.receives.append(Lookup([_m(SL_SHARD), _m(SL_CLK), _m(SL_ID), _reduce_v(SL_A0), _reduce_v(SL_A1)],
                              _m(SL_REAL), KIND_SYSCALL))
    return ch


def sys_linux_trace(events, byte_lookup) -> np.ndarray:
    """SysLinuxChip::event_to_row (sys_linux/trace.rs:106-167), one row per Linux syscall."""
    from .mips_core import ACC_VALUE, _access_cols
    n = len(events)
    t = np.zeros((max(16, 1 << max(0, (n - 1).bit_length())), SL_WIDTH), np.uint32)
    for k, e in enumerate(events):
        code, a0, a1 = e["code"], e["a0"], e["a1"]
        r = np.asarray([k])
        row = t[k]
        row[SL_SHARD], row[SL_CLK], row[SL_ID], row[SL_REAL] = e["shard"], e["clk"], code, 1
        row[SL_A0:SL_A0 + 4] = A._bytes(np.asarray([a0], np.uint32))[0]
        row[SL_A1:SL_A1 + 4] = A._bytes(np.asarray([a1], np.uint32))[0]
        row[SL_RES:SL_RES + 4] = A._bytes(np.asarray([e["v0"]], np.uint32))[0]
        row[SL_A0_0], row[SL_A0_1], row[SL_A0_2] = a0 == 0, a0 == 1, a0 == 2
        shard, clk = np.asarray([e["shard"]]), np.asarray([e["clk"]])
        one = np.ones(1, bool)

        def write(acc, rec):
            prev, val, ps, pc_ = rec
            t[k, acc:acc + 4] = A._bytes(np.asarray([prev], np.uint32))[0]
            _access_cols(t, r, acc + 4 + ACC_VALUE, np.asarray([val], np.uint32), np.asarray([[ps, pc_]]), shard, clk,
                         one, byte_lookup)

        def read(acc, rec):
            write(acc, (rec[0], rec[0], rec[1], rec[2]))

        write(SL_OUT, e["writes"][0])
        if code == SYS_BRK:
            row[SL_BRK] = 1
            brk = e["reads"][0][0]
            ab, bb = [(a0 >> (8 * j)) & 0xFF for j in range(4)], [(brk >> (8 * j)) & 0xFF for j in range(4)]
            res, ac, bc = 0, 0, 0
            for j in range(3, -1, -1):  # GtColsBytes::populate: the most significant differing byte
                if ab[j] != bb[j]:
                    row[SL_GT + j] = 1
                    ac, bc, res = ab[j], bb[j], int(ab[j] > bb[j])
                    break
            row[SL_GT + 4], row[SL_GT + 5], row[SL_GT + 6] = ac, bc, res
            byte_lookup(A.B_LTU, np.asarray([bc]), np.asarray([ac]))
            _u8_pairs_lookup([np.asarray([ab]), np.asarray([bb])], byte_lookup)
            read(SL_IO, e["reads"][0])
        elif code == SYS_CLONE:
            row[SL_CLONE] = 1
        elif code == SYS_EXT_GROUP:
            row[SL_EXIT] = 1
        elif code == SYS_FCNTL:
            row[SL_FCNTL] = 1
            row[SL_A1_1], row[SL_A1_3] = a1 == 1, a1 == 3
            row[SL_F_A1_1], row[SL_F_A1_3] = a1 == 1, a1 == 3
        elif code in (SYS_MMAP, SYS_MMAP2):
            row[SL_MMAP], row[SL_MMAP2], row[SL_MMAP_A0_0] = 1, code == SYS_MMAP2, a0 == 0
            row[SL_PAGE_OFF], row[SL_OFF_0], row[SL_UPPER] = a1 & 0xFFF, (a1 & 0xFFF) == 0, (a1 >> 12) << 12
            if a0 == 0:
                write(SL_IO, e["writes"][1])
        elif code == SYS_READ:
            row[SL_READ] = 1
        elif code == SYS_WRITE:
            read(SL_IO, e["reads"][0])
            row[SL_WRITE] = 1
        else:
            row[SL_NOP] = 1
    return t


# ---------------------------------------------------------------- execution of the precompiles
class PrecompileMemory:
    """The memory view of one syscall (SyscallContext::mr / mw, context.rs:63-100): every access at
    (shard, clk) updates the shared memory image; the first access to a word closes the CPU's open
    MemoryLocal entry for it and opens the syscall's own (initial = the previous record, final = the last)."""

    def __init__(self, mem, mem_init, mem_last, cpu_first, cpu_done, shard, init_word, regs=None, last=None,
                 reg_start=None, reg_done=None):
        self.mem, self.mem_init, self.mem_last = mem, mem_init, mem_last
        self.cpu_first, self.cpu_done = cpu_first, cpu_done
        self.shard, self.init_word = shard, init_word
        self.regs, self.last, self.reg_start, self.reg_done = regs, last, reg_start, reg_done
        self.local = {}
        self.reg_local = {}

    def peek(self, addr):
        """The current word without an access record (SyscallContext::slice_unsafe, ec.rs:113)."""
        return self.mem[addr] if addr in self.mem else self.init_word(addr)

    def _touch_reg(self, r):
        if self.last[r] != self.reg_start[r][0]:  # the CPU's open entry for r ends here
            s0, v0 = self.reg_start[r]
            self.reg_done.append((r, *s0, v0, *self.last[r], self.regs[r]))
        if r not in self.reg_local:
            self.reg_local[r] = (*self.last[r], self.regs[r])

    def reg_read(self, r, clk):
        """rr_traced (context.rs:102-111) -> (value, prev_shard, prev_clk)"""
        self._touch_reg(r)
        ps, pc_ = self.last[r]
        self.last[r] = (self.shard, clk)
        self.reg_start[r] = (self.last[r], self.regs[r])
        return self.regs[r], ps, pc_

    def reg_write(self, r, value, clk):
        """rw_traced (context.rs:113-123) -> (prev_value, value, prev_shard, prev_clk)"""
        self._touch_reg(r)
        ps, pc_ = self.last[r]
        prev = self.regs[r]
        self.regs[r] = value & M32
        self.last[r] = (self.shard, clk)
        self.reg_start[r] = (self.last[r], self.regs[r])
        return prev, value & M32, ps, pc_

    def _touch(self, addr):
        if addr not in self.mem:
            self.mem[addr] = self.mem_init[addr] = self.init_word(addr)
        if addr in self.cpu_first:  # SyscallContext::postprocess: the CPU's entry ends here
            s, c, v = self.cpu_first.pop(addr)
            fs, fc = self.mem_last[addr]
            self.cpu_done.append((addr, s, c, v, fs, fc, self.mem[addr]))
        if addr not in self.local:
            ps, pc_ = self.mem_last.get(addr, (0, 0))
            self.local[addr] = (ps, pc_, self.mem[addr])

    def read(self, addr, clk):
        """-> (value, prev_shard, prev_clk)"""
        assert addr % 4 == 0
        self._touch(addr)
        ps, pc_ = self.mem_last.get(addr, (0, 0))
        self.mem_last[addr] = (self.shard, clk)
        return self.mem[addr], ps, pc_

    def write(self, addr, value, clk):
        """-> (prev_value, value, prev_shard, prev_clk)"""
        assert addr % 4 == 0
        self._touch(addr)
        ps, pc_ = self.mem_last.get(addr, (0, 0))
        prev = self.mem[addr]
        self.mem[addr] = value & M32
        self.mem_last[addr] = (self.shard, clk)
        return prev, value & M32, ps, pc_

    def local_entries(self):
        """The syscall's MemoryLocal entries (addr, initial shard/clk/value, final shard/clk/value)."""
        ent = [(r, s, c, v, *self.last[r], self.regs[r]) for r, (s, c, v) in self.reg_local.items()]
        return ent + [(a, s, c, v, *self.mem_last[a], self.mem[a]) for a, (s, c, v) in self.local.items()]


def _rotr(x, s):
    return ((x >> s) | (x << (32 - s))) & M32


def exec_sha_extend(pm: PrecompileMemory, shard: int, clk: int, w_ptr: int, arg2: int):
    """Sha256ExtendSyscall::execute (syscalls/precompiles/sha256/extend.rs:14-81)."""
    assert arg2 == 0, "arg2 must be 0"
    ev = {"shard": shard, "clk": clk, "w_ptr": w_ptr, "r15": [], "r2": [], "r16": [], "r7": [], "wr": []}
    for i in range(16, 64):
        c = clk + i - 16
        r15 = pm.read(w_ptr + (i - 15) * 4, c)
        s0 = _rotr(r15[0], 7) ^ _rotr(r15[0], 18) ^ (r15[0] >> 3)
        r2 = pm.read(w_ptr + (i - 2) * 4, c)
        s1 = _rotr(r2[0], 17) ^ _rotr(r2[0], 19) ^ (r2[0] >> 10)
        r16 = pm.read(w_ptr + (i - 16) * 4, c)
        r7 = pm.read(w_ptr + (i - 7) * 4, c)
        w_i = (s1 + r16[0] + s0 + r7[0]) & M32
        ev["wr"].append(pm.write(w_ptr + i * 4, w_i, c))
        for k, rec in (("r15", r15), ("r2", r2), ("r16", r16), ("r7", r7)):
            ev[k].append(rec)
    ev["local"] = pm.local_entries()
    return ev


def exec_sha_compress(pm: PrecompileMemory, shard: int, clk: int, w_ptr: int, h_ptr: int):
    """Sha256CompressSyscall::execute (syscalls/precompiles/sha256/compress.rs:24-116): h and w read at clk,
    the new h written at clk + 1."""
    assert w_ptr != h_ptr
    ev = {"shard": shard, "clk": clk, "w_ptr": w_ptr, "h_ptr": h_ptr}
    ev["hr"] = [pm.read(h_ptr + 4 * i, clk) for i in range(8)]
    hx = [r[0] for r in ev["hr"]]
    a, b, c, d, e, f, g, h = hx
    ev["wr"] = []
    for i in range(64):
        s1 = _rotr(e, 6) ^ _rotr(e, 11) ^ _rotr(e, 25)
        chv = (e & f) ^ (~e & g & M32)
        rec = pm.read(w_ptr + 4 * i, clk)
        ev["wr"].append(rec)
        t1 = (h + s1 + chv + SHA_K[i] + rec[0]) & M32
        s0 = _rotr(a, 2) ^ _rotr(a, 13) ^ _rotr(a, 22)
        maj = (a & b) ^ (a & c) ^ (b & c)
        t2 = (s0 + maj) & M32
        h, g, f, e, d, c, b, a = g, f, e, (d + t1) & M32, c, b, a, (t1 + t2) & M32
    v = [a, b, c, d, e, f, g, h]
    ev["hw"] = [pm.write(h_ptr + 4 * i, hx[i] + v[i], clk + 1) for i in range(8)]
    ev["local"] = pm.local_entries()
    return ev


def exec_sys_linux(pm: PrecompileMemory, shard: int, clk: int, code: int, a0: int, a1: int):
    """The Linux syscalls (executor/src/syscalls/precompiles/sys_linux/*.rs): returns (value for V0 or None,
    LinuxEvent as a dict: read records (value, prev_shard, prev_clk), write records (prev, value, prev_shard,
    prev_clk))."""
    reads, writes, ret = [], [], 0
    if code == SYS_BRK:  # sysbrk.rs
        rec = pm.reg_read(REG_BRK, clk)
        reads.append(rec)
        ret = a0 if a0 > rec[0] else rec[0]
        writes.append(pm.reg_write(REG_A3, 0, clk))
    elif code in (SYS_MMAP, SYS_MMAP2):  # sysmmap.rs
        size = a1
        if size & (PAGE_SIZE - 1):
            size = (size + PAGE_SIZE - (size & (PAGE_SIZE - 1))) & M32
        writes.append(pm.reg_write(REG_A3, 0, clk))
        if a0 == 0:
            ret = pm.regs[REG_HEAP]
            writes.append(pm.reg_write(REG_HEAP, ret + size, clk))
        else:
            ret = a0
    elif code == SYS_CLONE:
        ret = 1
        writes.append(pm.reg_write(REG_A3, 0, clk))
    elif code == SYS_EXT_GROUP:
        ret = None
        writes.append(pm.reg_write(REG_A3, 0, clk))
    elif code == SYS_FCNTL:  # sysfcntl.rs
        if a1 == 3 and a0 in (0, 1, 2):
            ret, err = (0 if a0 == 0 else 1), 0
        elif a1 == 1 and a0 in (0, 1, 2):
            ret, err = a0, 0
        else:
            ret, err = M32, MIPS_EBADF
        writes.append(pm.reg_write(REG_A3, err, clk))
    elif code == SYS_READ:  # sysread.rs: only stdin
        ret, err = (0, 0) if a0 == 0 else (M32, MIPS_EBADF)
        writes.append(pm.reg_write(REG_A3, err, clk))
    elif code == SYS_WRITE:  # syswrite.rs: returns A2 (the byte count); the bytes go to the host fd
        rec = pm.reg_read(REG_A2, clk)
        reads.append(rec)
        ret = rec[0]
        writes.append(pm.reg_write(REG_A3, 0, clk))
    else:  # sysnop.rs
        ret = 0
        writes.append(pm.reg_write(REG_A3, 0, clk))
    ev = {"shard": shard, "clk": clk, "a0": a0, "a1": a1, "v0": 0 if ret is None else ret, "code": code,
          "reads": reads, "writes": writes, "local": pm.local_entries()}
    return ret, ev


def sha256_extend_ref(w16):
    """Plain SHA-256 message schedule (FIPS 180-4 §6.2.2 step 1) for tests."""
    w = list(w16) + [0] * 48
    for i in range(16, 64):
        s0 = _rotr(w[i - 15], 7) ^ _rotr(w[i - 15], 18) ^ (w[i - 15] >> 3)
        s1 = _rotr(w[i - 2], 17) ^ _rotr(w[i - 2], 19) ^ (w[i - 2] >> 10)
        w[i] = (w[i - 16] + s0 + w[i - 7] + s1) & M32
    return w


def _exec_ed_add(pm, shard, clk, a0, a1):
    from .mips_edwards import exec_ed_add
    return exec_ed_add(pm, shard, clk, a0, a1)


def _exec_ed_decompress(pm, shard, clk, a0, a1):
    from .mips_edwards import exec_ed_decompress
    return exec_ed_decompress(pm, shard, clk, a0, a1)


ED_ADD, ED_DECOMPRESS = 0x01_01_00_07, 0x00_01_00_08  # executor/src/syscalls/code.rs:50-54
PRECOMPILES = {SHA_EXTEND: exec_sha_extend, SHA_COMPRESS: exec_sha_compress, ED_ADD: _exec_ed_add,
               ED_DECOMPRESS: _exec_ed_decompress}


def _ec_precompiles():
    from . import mips_ec as EC
    return EC.precompile_table(), EC.PRECOMPILE_KEY


_EC_TABLE, PRECOMPILE_KEY = _ec_precompiles()  # Weierstrass curves, field towers, Uint256MulMod (mips_ec.py)
PRECOMPILES.update(_EC_TABLE)
