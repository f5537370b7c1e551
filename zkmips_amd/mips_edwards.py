"""Ed25519 precompiles: EdAddAssign and EdDecompress (MipsAir::Ed25519Add / Ed25519Decompress,
crates/core/machine/src/mips/mod.rs:129-131), the chips BASELINE config 4's tendermint guest verifies
its ed25519 signatures through (the patched curve25519-dalek, /root/reference/Cargo.toml:75).

Restated from:
* syscall/precompiles/edwards/ed_add.rs (EdAddAssignCols, eval :248-326, populate_field_ops :72-99),
  syscall/precompiles/edwards/ed_decompress.rs (EdDecompressCols, eval :104-190, populate :62-101);
* the emulated-field gadgets they use, operations/field/: field_op.rs (FieldOpCols: result, carry,
  witness_low, witness_high; eval_with_modulus / populate_with_modulus), field_inner_product.rs,
  field_den.rs, field_sqrt.rs, range.rs (FieldLtCols), util_air.rs (eval_field_operation: the
  vanishing polynomial equals witness(x) * (x - 2^8), coefficient by coefficient) and util.rs
  (compute_root_quotient_and_shift, split_u16_limbs_to_u8_limbs);
* the field parameters of crates/curves/src/edwards/ed25519.rs: p = 2^255 - 19 in 32 byte limbs,
  62 witness limbs, WITNESS_OFFSET = 2^14, d, ed25519_sqrt (lsb-0 root), decompress;
* the executor syscalls, crates/core/executor/src/syscalls/precompiles/edwards/{add,decompress}.rs and
  events/precompiles/ec.rs:96-139 (create_ec_add_event: p peeked, q read at clk, p written at clk + 1).

Column layouts follow the #[repr(C)] structs (MemoryWriteCols = prev_value[4] + MemoryAccessCols[9],
MemoryReadCols = MemoryAccessCols[9]); constraint and lookup order is the eval order, which fixes the
alpha folding and the LogUp column layout.  Costs equal mips_costs.json (EdAddAssign 3637 = 1861 main +
4 x 442 LogUp + 4 x 2; EdDecompress 3062 = 1566 + 4 x 372 + 4 x 2).
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np

from . import emulated_field as EF
from . import mips_alu as A
from .machine import ChipDesc, Expr, KIND_BYTE, KIND_SYSCALL, Lookup, P, main
from .machine import VirtualPairCol as V
from .mips_alu import ZERO, _assert_bool, _m

ED_P = (1 << 255) - 19
ED_D = int.from_bytes(bytes([163, 120, 89, 19, 202, 77, 235, 117, 171, 216, 65, 65, 77, 10, 112, 0, 152, 232, 121, 119,
                             121, 64, 199, 140, 115, 254, 111, 43, 238, 108, 3, 82]), "little")
SQRT_M1 = 19681161376707505956807079304988542015446066515923890162744021073123829784752
BASE_X = 15112221349535400772501151409588531511454012693041857206046113283949847762202
BASE_Y = 46316835694926478169428394003475163141307993866256225615783033603165251855960
NL, NWIT = 32, 62  # NumLimbs for Ed25519BaseField: Limbs = U32, Witness = U62
WITNESS_OFFSET = 1 << 14
FOP_W = 2 * NL + 2 * NWIT  # FieldOpCols / FieldInnerProductCols / FieldDenCols width (188)
LT_W = NL + 2  # FieldLtCols: byte_flags[32], lhs_comparison_byte, rhs_comparison_byte
MOD_LIMBS = list(ED_P.to_bytes(32, "little"))
D_LIMBS = list(ED_D.to_bytes(32, "little"))

ED_ADD, ED_DECOMPRESS = 0x01_01_00_07, 0x00_01_00_08  # SyscallCode (executor/src/syscalls/code.rs:50-54)
WR_W, RD_W = 13, 9  # MemoryWriteCols, MemoryReadCols
ACC_VALUE = 0

# ---------------------------------------------------------------- EdAddAssignCols (ed_add.rs:41-58)
EA_REAL, EA_SHARD, EA_CLK, EA_PPTR, EA_QPTR = 0, 1, 2, 3, 4
EA_P = 5                      # p_access: 16 x MemoryWriteCols
EA_Q = EA_P + 16 * WR_W       # q_access: 16 x MemoryReadCols
EA_X3N = EA_Q + 16 * RD_W     # x3_numerator
EA_Y3N, EA_X1Y1, EA_X2Y2, EA_F, EA_DF, EA_X3, EA_Y3 = (EA_X3N + FOP_W * k for k in range(1, 8))
EA_WIDTH = EA_X3N + 8 * FOP_W  # 1861

# ---------------------------------------------------------------- EdDecompressCols (ed_decompress.rs:45-62)
ED_REAL, ED_SHARD, ED_CLK, ED_PTR, ED_SIGN = 0, 1, 2, 3, 4
ED_X = 5                        # x_access: 8 x MemoryWriteCols
ED_Y = ED_X + 8 * WR_W          # y_access: 8 x MemoryReadCols
ED_YRANGE = ED_Y + 8 * RD_W     # FieldLtCols
ED_YY = ED_YRANGE + LT_W
ED_U, ED_DYY, ED_V, ED_UDV = (ED_YY + FOP_W * k for k in range(1, 5))
ED_SQRT = ED_YY + 5 * FOP_W     # FieldSqrtCols: multiplication (FieldOpCols), range (FieldLtCols), lsb
ED_SQRT_RANGE = ED_SQRT + FOP_W
ED_SQRT_LSB = ED_SQRT_RANGE + LT_W
ED_NEGX = ED_SQRT_LSB + 1
ED_WIDTH = ED_NEGX + FOP_W      # 1566


# ---------------------------------------------------------------- emulated-field gadgets (emulated_field.py)
ED_FP = EF.FieldParams("Ed25519BaseField", ED_P, NL, NWIT, WITNESS_OFFSET)
p_add, p_sub, p_mul = EF.p_add, EF.p_sub, EF.p_mul


def _cols(base: int, n: int = NL) -> List[Expr]:
    return EF.cols(base, n)


def _write_prev_limbs(base: int, words: int) -> List[Expr]:
    """limbs_from_prev_access over MemoryWriteCols: the prev_value bytes (utils/mod.rs:42-49)."""
    return [main(base + WR_W * w + i) for w in range(words) for i in range(4)]


def _write_value_limbs(base: int, words: int) -> List[Expr]:
    """limbs_from_access / value_as_limbs over MemoryWriteCols: the written value bytes."""
    return [main(base + WR_W * w + 4 + ACC_VALUE + i) for w in range(words) for i in range(4)]


def _read_limbs(base: int, words: int) -> List[Expr]:
    return [main(base + RD_W * w + ACC_VALUE + i) for w in range(words) for i in range(4)]


_u8_range, _vcols = EF.u8_range, EF.vcols


def eval_field_op(ch: ChipDesc, base: int, a, b, op: str, mult: V, result=None, result_cols=None):
    EF.eval_field_op(ch, base, a, b, op, mult, ED_FP, result=result, result_cols=result_cols)


def eval_inner_product(ch: ChipDesc, base: int, a_vec, b_vec, mult: V):
    EF.eval_inner_product(ch, base, a_vec, b_vec, mult, ED_FP)


def eval_den(ch: ChipDesc, base: int, a, b, sign: bool, mult: V):
    EF.eval_den(ch, base, a, b, sign, mult, ED_FP)


def eval_field_lt(ch: ChipDesc, base: int, lhs: Sequence, rhs: Sequence, is_real: Expr, mult: V):
    EF.eval_field_lt(ch, base, lhs, rhs, is_real, mult, ED_FP)


def _eval_access_slice(ch: ChipDesc, base: int, words: int, write: bool, ptr_col: int, addr_off: int, clk_pos: int,
                       is_real: Expr, mult: V):
    """eval_memory_access_slice (air/memory.rs:65-82): word i at ptr + addr_off + 4 i, timestamp clk + clk_pos."""
    from .mips_core import _eval_memory_access
    w = WR_W if write else RD_W
    for i in range(words):
        acc = base + w * i + (4 if write else 0)
        prev = base + w * i if write else acc + ACC_VALUE
        addr = V([("main", ptr_col, 1)], addr_off + 4 * i)
        _eval_memory_access(ch, acc, prev, clk_pos, addr, is_real, mult, shard_col=1, clk_terms=((2, 1),))


def ed_add_chip() -> ChipDesc:
    """EdAddAssignChip::eval (ed_add.rs:248-326)."""
    ch = ChipDesc("EdAddAssign", prep_width=0, main_width=EA_WIDTH, local_only=True)
    real, rv = main(EA_REAL), _m(EA_REAL)
    x1, y1 = _write_prev_limbs(EA_P, 8), _write_prev_limbs(EA_P + 8 * WR_W, 8)
    x2, y2 = _read_limbs(EA_Q, 8), _read_limbs(EA_Q + 8 * RD_W, 8)
    eval_inner_product(ch, EA_X3N, [x1, x2], [y2, y1], rv)
    eval_inner_product(ch, EA_Y3N, [y1, x1], [y2, x2], rv)
    eval_field_op(ch, EA_X1Y1, x1, y1, "mul", rv)
    eval_field_op(ch, EA_X2Y2, x2, y2, "mul", rv)
    eval_field_op(ch, EA_F, _cols(EA_X1Y1), _cols(EA_X2Y2), "mul", rv)
    eval_field_op(ch, EA_DF, _cols(EA_F), D_LIMBS, "mul", rv)
    eval_den(ch, EA_X3, _cols(EA_X3N), _cols(EA_DF), True, rv)
    eval_den(ch, EA_Y3, _cols(EA_Y3N), _cols(EA_DF), False, rv)
    pv = _write_value_limbs(EA_P, 16)
    for a, b in zip(_cols(EA_X3), pv[:NL]):
        ch.assert_zero(real * (a - b))
    for a, b in zip(_cols(EA_Y3), pv[NL:]):
        ch.assert_zero(real * (a - b))
    _eval_access_slice(ch, EA_Q, 16, False, EA_QPTR, 0, 0, real, rv)
    _eval_access_slice(ch, EA_P, 16, True, EA_PPTR, 0, 1, real, rv)
    ch.receives.append(Lookup([_m(EA_SHARD), _m(EA_CLK), V.const(ED_ADD & 0xFFFF), _m(EA_PPTR), _m(EA_QPTR)], rv,
                              KIND_SYSCALL))
    return ch


def ed_decompress_chip() -> ChipDesc:
    """EdDecompressChip::eval -> EdDecompressCols::eval (ed_decompress.rs:104-190)."""
    ch = ChipDesc("EdDecompress", prep_width=0, main_width=ED_WIDTH, local_only=True)
    real, rv = main(ED_REAL), _m(ED_REAL)
    sign = main(ED_SIGN)
    _assert_bool(ch, sign)
    y = _read_limbs(ED_Y, 8)
    eval_field_lt(ch, ED_YRANGE, y, MOD_LIMBS, real, rv)
    eval_field_op(ch, ED_YY, y, y, "mul", rv)
    eval_field_op(ch, ED_U, _cols(ED_YY), [1], "sub", rv)
    eval_field_op(ch, ED_DYY, D_LIMBS, _cols(ED_YY), "mul", rv)
    eval_field_op(ch, ED_V, [1], _cols(ED_DYY), "add", rv)
    eval_field_op(ch, ED_UDV, _cols(ED_U), _cols(ED_V), "div", rv)
    # FieldSqrtCols::eval (field_sqrt.rs:113-158): sqrt stored in multiplication.result; the product is
    # checked against the input a (= u / v), whose limbs the multiplication's range check covers
    sqrt = _cols(ED_SQRT)
    eval_field_op(ch, ED_SQRT, sqrt, sqrt, "mul", rv, result=_cols(ED_UDV), result_cols=_vcols(ED_UDV, NL))
    eval_field_lt(ch, ED_SQRT_RANGE, sqrt, MOD_LIMBS, real, rv)
    _u8_range(ch, _vcols(ED_SQRT, NL), rv)
    lsb = main(ED_SQRT_LSB)
    _assert_bool(ch, lsb)
    ch.assert_zero(real * (lsb - 0))  # is_odd = 0: the nonnegative root
    ch.sends.append(Lookup([V.const(A.B_AND), _m(ED_SQRT_LSB), ZERO, _m(ED_SQRT), V.const(1)], rv, KIND_BYTE))
    eval_field_op(ch, ED_NEGX, [0], sqrt, "sub", rv)
    _eval_access_slice(ch, ED_X, 8, True, ED_PTR, 0, 0, real, rv)
    _eval_access_slice(ch, ED_Y, 8, False, ED_PTR, 32, 0, real, rv)
    xv = _write_value_limbs(ED_X, 8)
    for a, b in zip(_cols(ED_NEGX), xv):
        ch.assert_zero(real * sign * (a - b))
    for a, b in zip(sqrt, xv):
        ch.assert_zero(real * (1 - sign) * (a - b))
    ch.receives.append(Lookup([_m(ED_SHARD), _m(ED_CLK), V.const(ED_DECOMPRESS & 0xFFFF), _m(ED_PTR), _m(ED_SIGN)],
                              rv, KIND_SYSCALL))
    return ch


# ---------------------------------------------------------------- field arithmetic (trace side)
def ed25519_sqrt(a: int) -> int:
    """ed25519.rs:75-113: the square root with least significant bit 0."""
    beta = pow(a, (ED_P + 3) // 8, ED_P)
    bsq = beta * beta % ED_P
    if bsq == (ED_P - a) % ED_P:
        beta = beta * SQRT_M1 % ED_P
    if bsq != a % ED_P and bsq != (ED_P - a) % ED_P:
        raise ValueError("not a square")
    if beta & 1:
        beta = (ED_P - beta) % ED_P
    return beta


def ed_add_points(p, q):
    """AffinePoint::ed_add (curves/src/edwards/mod.rs:111-129), a = -1."""
    (x1, y1), (x2, y2) = p, q
    x3n = (x1 * y2 + y1 * x2) % ED_P
    y3n = (y1 * y2 + x1 * x2) % ED_P
    dxy = ED_D * (x1 * y1 % ED_P * x2 % ED_P * y2) % ED_P
    return (x3n * pow((1 + dxy) % ED_P, -1, ED_P) % ED_P, y3n * pow((1 - dxy) % ED_P, -1, ED_P) % ED_P)


def ed_decompress_point(y: int, sign: int):
    """curves/src/edwards/ed25519.rs decompress: x from y and the sign bit."""
    yy = y * y % ED_P
    u = (yy - 1) % ED_P
    v = (yy * ED_D + 1) % ED_P
    x = ed25519_sqrt(u * pow(v, -1, ED_P) % ED_P)
    return ((ED_P - x) % ED_P if sign else x), y


def _limbs(xs: Sequence[int], n: int = NL) -> np.ndarray:
    return EF.limbs(xs, n)


_Rec = EF.Rec


def pop_field_op(a: Sequence[int], b: Sequence[int], op: str):
    return EF.pop_field_op(a, b, op, ED_FP)


def pop_inner_product(a_vec, b_vec):
    return EF.pop_inner_product(a_vec, b_vec, ED_FP)


def pop_den(a: Sequence[int], b: Sequence[int], sign: bool):
    return EF.pop_den(a, b, sign, ED_FP)


def pop_field_lt(lhs: Sequence[int], rec, real: np.ndarray) -> np.ndarray:
    return EF.pop_field_lt(lhs, rec, real, ED_FP)


# ---------------------------------------------------------------- traces
def _access_block(t, rows, base, recs, write: bool, shard, clk, byte_lookup):
    """MemoryReadCols / MemoryWriteCols populate for word records at timestamp clk (per row)."""
    from .mips_core import _access_cols
    w = WR_W if write else RD_W
    for i in range(len(recs[0])):
        r = np.asarray([x[i] for x in recs], np.int64)  # read: (value, prev_shard, prev_clk); write: (prev, value, ps, pc)
        acc = base + w * i + (4 if write else 0)
        if write:
            t[rows, base + w * i:base + w * i + 4] = A._bytes(r[:, 0].astype(np.uint32))
            value, prev = r[:, 1], r[:, 2:4]
        else:
            value, prev = r[:, 0], r[:, 1:3]
        _access_cols(t, rows, acc, value.astype(np.uint32), prev, shard, clk, np.ones(len(rows), bool), byte_lookup)


_words_to_int = EF.words_to_int


def ed_add_trace(events, byte_lookup) -> np.ndarray:
    """EdAddAssignChip::generate_trace + event_to_row (ed_add.rs:111-238); padding rows hold the field
    operations on zero inputs (pad_rows_fixed)."""
    ne = len(events)
    h = max(16, 1 << max(0, (ne - 1).bit_length()))
    t = np.zeros((h, EA_WIDTH), np.int64)
    rec = _Rec(byte_lookup)
    real = np.zeros(h, bool)
    real[:ne] = True
    px = [0] * h
    py = [0] * h
    qx = [0] * h
    qy = [0] * h
    for i, e in enumerate(events):
        px[i], py[i] = _words_to_int(e["p"][:8]), _words_to_int(e["p"][8:])
        qv = [r[0] for r in e["q"]]
        qx[i], qy[i] = _words_to_int(qv[:8]), _words_to_int(qv[8:])
    x3n, t[:, EA_X3N:EA_X3N + FOP_W] = pop_inner_product([px, qx], [qy, py])
    y3n, t[:, EA_Y3N:EA_Y3N + FOP_W] = pop_inner_product([py, px], [qy, qx])
    x1y1, t[:, EA_X1Y1:EA_X1Y1 + FOP_W] = pop_field_op(px, py, "mul")
    x2y2, t[:, EA_X2Y2:EA_X2Y2 + FOP_W] = pop_field_op(qx, qy, "mul")
    f, t[:, EA_F:EA_F + FOP_W] = pop_field_op(x1y1, x2y2, "mul")
    df, t[:, EA_DF:EA_DF + FOP_W] = pop_field_op(f, [ED_D] * h, "mul")
    x3, t[:, EA_X3:EA_X3 + FOP_W] = pop_den(x3n, df, True)
    y3, t[:, EA_Y3:EA_Y3 + FOP_W] = pop_den(y3n, df, False)
    for base in (EA_X3N, EA_Y3N, EA_X1Y1, EA_X2Y2, EA_F, EA_DF, EA_X3, EA_Y3):
        rec.u8(t[real, base:base + FOP_W])
    if ne:
        rows = np.arange(ne)
        t[rows, EA_REAL] = 1
        shard = np.array([e["shard"] for e in events], np.int64)
        clk = np.array([e["clk"] for e in events], np.int64)
        t[rows, EA_SHARD], t[rows, EA_CLK] = shard, clk
        t[rows, EA_PPTR] = [e["p_ptr"] for e in events]
        t[rows, EA_QPTR] = [e["q_ptr"] for e in events]
        for i, e in enumerate(events):
            assert (x3[i], y3[i]) == ed_add_points((px[i], py[i]), (qx[i], qy[i]))
        _access_block(t, rows, EA_Q, [e["q"] for e in events], False, shard, clk, byte_lookup)
        _access_block(t, rows, EA_P, [e["pw"] for e in events], True, shard, clk + 1, byte_lookup)
    return (t % P).astype(np.uint32)


def ed_decompress_trace(events, byte_lookup) -> np.ndarray:
    """EdDecompressChip::generate_trace + EdDecompressCols::populate (ed_decompress.rs:64-101, :214-247);
    padding rows hold the field operations of y = 0."""
    ne = len(events)
    h = max(16, 1 << max(0, (ne - 1).bit_length()))
    t = np.zeros((h, ED_WIDTH), np.int64)
    rec = _Rec(byte_lookup)
    real = np.zeros(h, bool)
    real[:ne] = True
    y = [0] * h
    for i, e in enumerate(events):
        y[i] = _words_to_int([r[0] for r in e["y"]])
    t[:, ED_YRANGE:ED_YRANGE + LT_W] = pop_field_lt(y, rec, real)
    yy, t[:, ED_YY:ED_YY + FOP_W] = pop_field_op(y, y, "mul")
    u, t[:, ED_U:ED_U + FOP_W] = pop_field_op(yy, [1] * h, "sub")
    dyy, t[:, ED_DYY:ED_DYY + FOP_W] = pop_field_op([ED_D] * h, yy, "mul")
    v, t[:, ED_V:ED_V + FOP_W] = pop_field_op([1] * h, dyy, "add")
    udv, t[:, ED_UDV:ED_UDV + FOP_W] = pop_field_op(u, v, "div")
    sq = [ed25519_sqrt(x) for x in udv]
    sq2, cols = pop_field_op(sq, sq, "mul")
    assert sq2 == udv
    cols[:, :NL] = _limbs(sq)  # FieldSqrtCols stores the root in multiplication.result
    t[:, ED_SQRT:ED_SQRT + FOP_W] = cols
    t[:, ED_SQRT_RANGE:ED_SQRT_RANGE + LT_W] = pop_field_lt(sq, rec, real)
    t[:, ED_SQRT_LSB] = _limbs(sq)[:, 0] & 1
    negx, t[:, ED_NEGX:ED_NEGX + FOP_W] = pop_field_op([0] * h, sq, "sub")
    # byte lookups in populate order (the Byte chip only counts them)
    for base in (ED_YY, ED_U, ED_DYY, ED_V, ED_UDV):
        rec.u8(t[real, base:base + FOP_W])
    sqc = t[real, ED_SQRT:ED_SQRT + FOP_W].copy()
    sqc[:, :NL] = t[real, ED_UDV:ED_UDV + NL]  # the multiplication's populate range-checks sqrt^2 = u / v
    rec.u8(sqc)
    if real.any():
        byte_lookup(A.B_AND, t[real, ED_SQRT], np.ones(int(real.sum()), np.int64))
    rec.u8(t[real, ED_SQRT:ED_SQRT + NL])
    rec.u8(t[real, ED_NEGX:ED_NEGX + FOP_W])
    if ne:
        rows = np.arange(ne)
        t[rows, ED_REAL] = 1
        shard = np.array([e["shard"] for e in events], np.int64)
        clk = np.array([e["clk"] for e in events], np.int64)
        t[rows, ED_SHARD], t[rows, ED_CLK] = shard, clk
        t[rows, ED_PTR] = [e["ptr"] for e in events]
        t[rows, ED_SIGN] = [e["sign"] for e in events]
        for i, e in enumerate(events):
            want = negx[i] if e["sign"] else sq[i]
            assert want == _words_to_int([r[1] for r in e["x"]]), "decompressed x differs from the executor's"
        _access_block(t, rows, ED_X, [e["x"] for e in events], True, shard, clk, byte_lookup)
        _access_block(t, rows, ED_Y, [e["y"] for e in events], False, shard, clk, byte_lookup)
    return (t % P).astype(np.uint32)


# ---------------------------------------------------------------- executor (syscalls)
def _point_words(x: int, y: int) -> List[int]:
    b = x.to_bytes(32, "little") + y.to_bytes(32, "little")
    return [int.from_bytes(b[4 * i:4 * i + 4], "little") for i in range(16)]


def exec_ed_add(pm, shard: int, clk: int, p_ptr: int, q_ptr: int):
    """EdwardsAddAssignSyscall::execute -> create_ec_add_event (events/precompiles/ec.rs:96-139): p is read
    without a record, q read at clk, p + q written to p at clk + 1 (p and q may be the same)."""
    assert p_ptr % 4 == 0 and q_ptr % 4 == 0
    p = [pm.peek(p_ptr + 4 * i) for i in range(16)]
    q = [pm.read(q_ptr + 4 * i, clk) for i in range(16)]
    pt = (_words_to_int(p[:8]), _words_to_int(p[8:]))
    qt = (_words_to_int([r[0] for r in q[:8]]), _words_to_int([r[0] for r in q[8:]]))
    res = _point_words(*ed_add_points(pt, qt))
    pw = [pm.write(p_ptr + 4 * i, res[i], clk + 1) for i in range(16)]
    return {"shard": shard, "clk": clk, "p_ptr": p_ptr, "q_ptr": q_ptr, "p": p, "q": q, "pw": pw,
            "local": pm.local_entries()}


def exec_ed_decompress(pm, shard: int, clk: int, ptr: int, sign: int):
    """EdwardsDecompressSyscall::execute (syscalls/precompiles/edwards/decompress.rs): y read from
    ptr + 32 at clk, the decompressed x written to ptr at clk."""
    assert ptr % 4 == 0 and sign <= 1
    yr = [pm.read(ptr + 32 + 4 * i, clk) for i in range(8)]
    y = _words_to_int([r[0] for r in yr])
    assert y < ED_P, "y must be reduced (the sign bit is passed separately)"
    x, _ = ed_decompress_point(y, sign)
    xw = _point_words(x, 0)[:8]
    xr = [pm.write(ptr + 4 * i, xw[i], clk) for i in range(8)]
    return {"shard": shard, "clk": clk, "ptr": ptr, "sign": sign, "y": yr, "x": xr, "local": pm.local_entries()}


# ---------------------------------------------------------------- ed25519 signatures (RFC 8032) + the guest
ED_L = (1 << 252) + 27742317777372353535851937790883648493  # prime group order


def _scalar_mul(k: int, pt):
    acc = (0, 1)
    for bit in bin(k)[2:]:
        acc = ed_add_points(acc, acc)
        if bit == "1":
            acc = ed_add_points(acc, pt)
    return acc


def _encode(pt) -> bytes:
    x, y = pt
    return (y | ((x & 1) << 255)).to_bytes(32, "little")


def ed25519_keypair_sign(seed: bytes, msg: bytes):
    """RFC 8032 Ed25519 (the scheme tendermint's validators sign with): returns (A, R, S, k) with A the
    public point, (R, S) the signature of msg and k = H(R || A || M) mod L, so [S]B = R + [k]A."""
    import hashlib
    h = hashlib.sha512(seed).digest()
    a = int.from_bytes(h[:32], "little")
    a = (a & ~7 & ((1 << 254) - 1)) | (1 << 254)
    B = (BASE_X, BASE_Y)
    A = _scalar_mul(a, B)
    r = int.from_bytes(hashlib.sha512(h[32:] + msg).digest(), "little") % ED_L
    R = _scalar_mul(r, B)
    k = int.from_bytes(hashlib.sha512(_encode(R) + _encode(A) + msg).digest(), "little") % ED_L
    S = (r + k * a) % ED_L
    return A, R, S, k


def ed25519_program(n_sigs: int, seed: int = 1, scalar_bits: int = 253, sha_blocks: int = 0, halt: bool = True):
    """A guest with the shape of the tendermint light-client check (BASELINE config 4): n_sigs ed25519
    signature verifications through the precompiles -- per signature the public key A and the
    commitment R are decompressed from their 32-byte encodings (ED_DECOMPRESS), [S]B and R + [k]A are
    computed by double-and-add (ED_ADD on points in memory, p = q for the doublings) and compared word by
    word (the XOR of the two results is folded into a register that must end at 0) -- plus `sha_blocks`
    SHA-256 compressions (the header hashing, SHA_EXTEND + SHA_COMPRESS), then COMMIT and HALT.
    scalar_bits < 253 keeps only the low bits of S and k (small test guests; the check then no longer
    holds and the register is only committed)."""
    from . import mips_core as MC
    from . import mips_syscall as SY
    rng = np.random.default_rng(seed)
    prog = []
    base = MC.DATA_BASE + 0x2000
    b_ptr = base  # the base point B (x, y)
    acc, tmp = 10, 9

    def li(reg, v):
        prog.append((A.OP_ADD, reg, 0, int(v) & 0xFFFFFFFF, 0, 1))

    def store_point(ptr, pt):
        for i, w in enumerate(_point_words(*pt)):
            li(8, w)
            prog.append((MC.OP_SW, 8, 0, ptr + 4 * i, 0, 1))

    def syscall(code, a0, a1):
        li(SY.REG_V0, code)
        li(SY.REG_A0, a0)
        li(SY.REG_A1, a1)
        prog.append((SY.OP_SYSCALL, SY.REG_V0, SY.REG_A0, SY.REG_A1, 0, 0))

    def scalar_mul(dst, pt_ptr, k):
        store_point(dst, (0, 1))
        for bit in bin(k)[2:] if k else "":
            syscall(ED_ADD, dst, dst)
            if bit == "1":
                syscall(ED_ADD, dst, pt_ptr)

    li(acc, 0)
    store_point(b_ptr, (BASE_X, BASE_Y))
    mask = (1 << scalar_bits) - 1
    for s in range(n_sigs):
        slot = base + 0x100 + 0x200 * s
        a_ptr, r_ptr, acc1, acc2 = slot, slot + 0x40, slot + 0x80, slot + 0xC0
        msg = bytes(rng.integers(0, 256, 64, dtype=np.uint8))
        A_, R_, S_, k_ = ed25519_keypair_sign(bytes(rng.integers(0, 256, 32, dtype=np.uint8)), msg)
        for ptr, pt in ((a_ptr, A_), (r_ptr, R_)):  # the compressed encodings: y words, sign = x & 1
            for i, w in enumerate(_point_words(0, pt[1])[8:]):
                li(8, w)
                prog.append((MC.OP_SW, 8, 0, ptr + 32 + 4 * i, 0, 1))
            syscall(ED_DECOMPRESS, ptr, pt[0] & 1)
        scalar_mul(acc1, b_ptr, S_ & mask)
        scalar_mul(acc2, a_ptr, k_ & mask)
        syscall(ED_ADD, acc2, r_ptr)
        for i in range(16):  # acc |= [S]B xor (R + [k]A), word by word
            prog.append((MC.OP_LW, tmp, 0, acc1 + 4 * i, 0, 1))
            prog.append((MC.OP_LW, 8, 0, acc2 + 4 * i, 0, 1))
            prog.append((A.OP_XOR, tmp, tmp, 8, 0, 0))
            prog.append((A.OP_OR, acc, acc, tmp, 0, 0))
    if sha_blocks:
        prog += MC.sha_program(sha_blocks, seed=seed, commit=False, halt=False)
    prog += [(A.OP_ADD, SY.REG_V0, 0, SY.COMMIT, 0, 1), (A.OP_ADD, SY.REG_A0, 0, 0, 0, 1),
             (A.OP_ADD, SY.REG_A1, acc, 0, 0, 1), (SY.OP_SYSCALL, SY.REG_V0, SY.REG_A0, SY.REG_A1, 0, 0)]
    if halt:
        prog += [(A.OP_ADD, SY.REG_V0, 0, SY.HALT, 0, 1), (A.OP_ADD, SY.REG_A0, 0, 0, 0, 1),
                 (SY.OP_SYSCALL, SY.REG_V0, SY.REG_A0, SY.REG_A1, 0, 0)]
    return prog
