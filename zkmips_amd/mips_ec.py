"""Weierstrass-curve, field-tower and 256-bit precompiles: the chips of MipsAir (crates/core/machine/src/
mips/mod.rs:133-173) built on the emulated-field gadgets (emulated_field.py):

* WeierstrassAddAssignChip<E> / WeierstrassDoubleAssignChip<E> (syscall/precompiles/weierstrass/
  weierstrass_add.rs, weierstrass_double.rs) for secp256k1, secp256r1, bn254 and bls12-381 (field
  parameters crates/curves/src/weierstrass/*.rs; the affine slope formulas of sw_add / sw_double,
  crates/curves/src/weierstrass/mod.rs:175-240);
* FpOpChip<P>, Fp2AddSubAssignChip<P>, Fp2MulAssignChip<P> (syscall/precompiles/fptower/) over the bn254
  and bls12-381 base fields;
* Uint256MulChip (syscall/precompiles/uint256/air.rs): x <- x * y mod m, m = 2^256 when the modulus
  words are zero (U256Field: 32 limbs, 63 witness limbs, crates/curves/src/uint256.rs).

Column layouts follow the #[repr(C)] structs; constraint and lookup order is each chip's eval order
(that order fixes the alpha folding and the LogUp columns).  Costs equal mips_costs.json.  The executor
side follows crates/core/executor/src/syscalls/precompiles/{weierstrass,fptower,uint256.rs} and
events/precompiles/ec.rs (create_ec_add_event / create_ec_double_event): the point / x operand is read
without a record, the other operand read at clk, the result written at clk + 1 (add, field ops) or at
clk (double).
"""
from __future__ import annotations

from typing import Dict, List, Sequence

import numpy as np

from . import emulated_field as EF
from .emulated_field import FieldParams
from .machine import ChipDesc, Expr, KIND_SYSCALL, Lookup, P, main
from .machine import VirtualPairCol as V
from .mips_alu import _assert_bool, _m

WR_W, RD_W, ACC_VALUE = 13, 9, 0  # MemoryWriteCols, MemoryReadCols, value offset in MemoryAccessCols
WIDTH_P2 = 16

# ---------------------------------------------------------------- field and curve parameters
SECP256K1_P = (1 << 256) - (1 << 32) - 977
SECP256R1_P = (1 << 256) - (1 << 224) + (1 << 192) + (1 << 96) - 1
BN254_P = 21888242871839275222246405745257275088696311157297823662689037894645226208583
BLS12381_P = int("1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab", 16)

FIELDS: Dict[str, FieldParams] = {
    "Secp256k1": FieldParams("Secp256k1BaseField", SECP256K1_P, 32, 62, 1 << 14),
    "Secp256r1": FieldParams("Secp256r1BaseField", SECP256R1_P, 32, 62, 1 << 14),
    "Bn254": FieldParams("Bn254BaseField", BN254_P, 32, 62, 1 << 14),
    "Bls12381": FieldParams("Bls12381BaseField", BLS12381_P, 48, 94, 1 << 15),
}
U256 = FieldParams("U256Field", 1 << 256, 32, 63, 1 << 14)

# y^2 = x^3 + a x + b (a_int / b_int of each WeierstrassParameters)
CURVE_A = {"Secp256k1": 0, "Secp256r1": SECP256R1_P - 3, "Bn254": 0, "Bls12381": 0}
CURVE_B = {"Secp256k1": 7,
           "Secp256r1": 0x5AC635D8AA3A93E7B3EBBD55769886BC651D06B0CC53B0F63BCE3C3E27D2604B,
           "Bn254": 3, "Bls12381": 4}

# the generators' abscissae (padding rows of the decompress chips decompress E::generator().0)
GEN_X = {"Secp256k1": 0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798,
         "Secp256r1": 0x6B17D1F2E12C4247F8BCE6E563A440F277037D812DEB33A0F4A13945D898C296,
         "Bls12381": int("17f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00"
                         "adb22c6bb", 16)}

# SyscallCode (crates/core/executor/src/syscalls/code.rs:60-141)
SECP256K1_ADD, SECP256K1_DOUBLE = 0x01_01_00_0A, 0x00_01_00_0B
BN254_ADD, BN254_DOUBLE = 0x01_01_00_0E, 0x00_01_00_0F
UINT256_MUL = 0x01_01_00_1D
BLS12381_ADD, BLS12381_DOUBLE = 0x01_01_00_1E, 0x00_01_00_1F
BLS12381_FP_ADD, BLS12381_FP_SUB, BLS12381_FP_MUL = 0x01_01_00_20, 0x01_01_00_21, 0x01_01_00_22
BLS12381_FP2_ADD, BLS12381_FP2_SUB, BLS12381_FP2_MUL = 0x01_01_00_23, 0x01_01_00_24, 0x01_01_00_25
BN254_FP_ADD, BN254_FP_SUB, BN254_FP_MUL = 0x01_01_00_26, 0x01_01_00_27, 0x01_01_00_28
BN254_FP2_ADD, BN254_FP2_SUB, BN254_FP2_MUL = 0x01_01_00_29, 0x01_01_00_2A, 0x01_01_00_2B
SECP256R1_ADD, SECP256R1_DOUBLE = 0x01_01_00_2C, 0x00_01_00_2D
SECP256K1_DECOMPRESS, SECP256R1_DECOMPRESS, BLS12381_DECOMPRESS = 0x00_01_00_0C, 0x00_01_00_2E, 0x00_01_00_1C
EC_DECOMPRESS = {"Secp256k1": SECP256K1_DECOMPRESS, "Secp256r1": SECP256R1_DECOMPRESS,
                 "Bls12381": BLS12381_DECOMPRESS}
# SignChoiceRule (weierstrass_decompress.rs:82-112): the k256 / p256 chips take y's parity, bls12-381
# the lexicographic order of y and -y
LEXICOGRAPHIC = {"Secp256k1": False, "Secp256r1": False, "Bls12381": True}

EC_ADD = {"Secp256k1": SECP256K1_ADD, "Secp256r1": SECP256R1_ADD, "Bn254": BN254_ADD, "Bls12381": BLS12381_ADD}
EC_DOUBLE = {"Secp256k1": SECP256K1_DOUBLE, "Secp256r1": SECP256R1_DOUBLE, "Bn254": BN254_DOUBLE,
             "Bls12381": BLS12381_DOUBLE}
FP_OPS = {"Bn254": (BN254_FP_ADD, BN254_FP_SUB, BN254_FP_MUL),
          "Bls12381": (BLS12381_FP_ADD, BLS12381_FP_SUB, BLS12381_FP_MUL)}
FP2_ADDSUB = {"Bn254": (BN254_FP2_ADD, BN254_FP2_SUB), "Bls12381": (BLS12381_FP2_ADD, BLS12381_FP2_SUB)}
FP2_MUL = {"Bn254": BN254_FP2_MUL, "Bls12381": BLS12381_FP2_MUL}

# chip names (the reference's `name()`, typos included)
FP_NAME = {"Bn254": "Bn254FpOpAssign", "Bls12381": "Bls12381FpOpAssign"}
FP2_ADDSUB_NAME = {"Bn254": "Bn254Fp2AddSubAssign", "Bls12381": "Bls12831Fp2AddSubAssign"}
FP2_MUL_NAME = {"Bn254": "Bn254Fp2MulAssign", "Bls12381": "Bls12831Fp2MulAssign"}


def sid(code: int) -> int:
    return code & 0xFFFF


# precompile events are grouped per chip (rt.add_precompile_event keys: the fp ops under their ADD code)
PRECOMPILE_KEY = {}
for _c in FP_OPS.values():
    PRECOMPILE_KEY.update({k: _c[0] for k in _c})
for _c in FP2_ADDSUB.values():
    PRECOMPILE_KEY.update({k: _c[0] for k in _c})


# ---------------------------------------------------------------- AIR helpers
def _write_prev_limbs(base: int, words: int) -> List[Expr]:
    """limbs_from_prev_access over MemoryWriteCols: the prev_value bytes (utils/mod.rs:42-49)."""
    return [main(base + WR_W * w + i) for w in range(words) for i in range(4)]


def _write_value_limbs(base: int, words: int) -> List[Expr]:
    """value_as_limbs over MemoryWriteCols: the written value bytes."""
    return [main(base + WR_W * w + 4 + ACC_VALUE + i) for w in range(words) for i in range(4)]


def _read_limbs(base: int, words: int) -> List[Expr]:
    return [main(base + RD_W * w + ACC_VALUE + i) for w in range(words) for i in range(4)]


def _eval_access_slice(ch: ChipDesc, base: int, words: int, write: bool, ptr_col: int, clk_pos: int,
                       is_real: Expr, mult: V, shard_col: int, clk_col: int, addr_off: int = 0):
    """eval_memory_access_slice (air/memory.rs:65-82): word i at ptr + addr_off + 4 i, timestamp clk + clk_pos."""
    from .mips_core import _eval_memory_access
    w = WR_W if write else RD_W
    for i in range(words):
        acc = base + w * i + (4 if write else 0)
        prev = base + w * i if write else acc + ACC_VALUE
        addr = V([("main", ptr_col, 1)], addr_off + 4 * i)
        _eval_memory_access(ch, acc, prev, clk_pos, addr, is_real, mult, shard_col=shard_col,
                            clk_terms=((clk_col, 1),))


def _eval_variable(ch: ChipDesc, base: int, a, b, modulus, is_add, is_sub, is_mul, mult: V, fp: FieldParams):
    """FieldOpCols::eval_variable (field_op.rs:244-280) with is_div = 0: one constraint system for
    add / sub / mul selected by the flag columns."""
    res = EF.cols(base, fp.nl)
    p_result = EF.p_add(EF.p_scale(res, is_add + is_mul), EF.p_scale(a, is_sub))
    p_op = EF.p_add(EF.p_add(EF.p_scale(EF.p_add(a, b), is_add), EF.p_scale(EF.p_add(res, b), is_sub)),
                    EF.p_scale(EF.p_mul(a, b), is_mul))
    carry = EF.cols(base + fp.nl, fp.nl)
    vanishing = EF.p_sub(EF.p_sub(p_op, p_result), EF.p_mul(carry, modulus))
    EF.eval_field_operation(ch, vanishing, base, fp)
    EF.field_range_checks(ch, base, mult, fp)


# ---------------------------------------------------------------- Weierstrass add / double
class AddLayout:
    """WeierstrassAddAssignCols (weierstrass_add.rs:46-61)."""

    def __init__(self, fp: FieldParams):
        w = fp.words
        self.REAL, self.SHARD, self.CLK, self.PPTR, self.QPTR = range(5)
        self.P = 5
        self.Q = self.P + 2 * w * WR_W
        base = self.Q + 2 * w * RD_W
        names = ["slope_denominator", "slope_numerator", "slope", "slope_squared", "p_x_plus_q_x", "x3_ins",
                 "p_x_minus_x", "y3_ins", "slope_times_p_x_minus_x"]
        self.F = {n: base + k * fp.fop_w for k, n in enumerate(names)}
        self.WIDTH = base + len(names) * fp.fop_w


class DoubleLayout:
    """WeierstrassDoubleAssignCols (weierstrass_double.rs:45-62)."""

    def __init__(self, fp: FieldParams):
        w = fp.words
        self.REAL, self.SHARD, self.CLK, self.PPTR = range(4)
        self.P = 4
        base = self.P + 2 * w * WR_W
        names = ["slope_denominator", "slope_numerator", "slope", "p_x_squared", "p_x_squared_times_3",
                 "slope_squared", "p_x_plus_p_x", "x3_ins", "p_x_minus_x", "y3_ins", "slope_times_p_x_minus_x"]
        self.F = {n: base + k * fp.fop_w for k, n in enumerate(names)}
        self.WIDTH = base + len(names) * fp.fop_w


def _result_eq(ch: ChipDesc, real: Expr, x3: Sequence, y3: Sequence, pv: Sequence, nl: int):
    """x3_ins / y3_ins results equal the written point, limb by limb (x and y interleaved)."""
    for i in range(nl):
        ch.assert_zero(real * (x3[i] - pv[i]))
        ch.assert_zero(real * (y3[i] - pv[nl + i]))


def weierstrass_add_chip(curve: str) -> ChipDesc:
    """WeierstrassAddAssignChip::eval (weierstrass_add.rs:262-381)."""
    fp = FIELDS[curve]
    L = AddLayout(fp)
    nl, w = fp.nl, fp.words
    ch = ChipDesc(f"{curve}AddAssign", prep_width=0, main_width=L.WIDTH, local_only=True)
    real, rv = main(L.REAL), _m(L.REAL)
    px, py = _write_prev_limbs(L.P, w), _write_prev_limbs(L.P + w * WR_W, w)
    qx, qy = _read_limbs(L.Q, w), _read_limbs(L.Q + w * RD_W, w)
    F, c = L.F, lambda n: EF.cols(L.F[n], nl)
    EF.eval_field_op(ch, F["slope_numerator"], qy, py, "sub", rv, fp)
    EF.eval_field_op(ch, F["slope_denominator"], qx, px, "sub", rv, fp)
    EF.eval_field_op(ch, F["slope"], c("slope_numerator"), c("slope_denominator"), "div", rv, fp)
    slope = c("slope")
    EF.eval_field_op(ch, F["slope_squared"], slope, slope, "mul", rv, fp)
    EF.eval_field_op(ch, F["p_x_plus_q_x"], px, qx, "add", rv, fp)
    EF.eval_field_op(ch, F["x3_ins"], c("slope_squared"), c("p_x_plus_q_x"), "sub", rv, fp)
    EF.eval_field_op(ch, F["p_x_minus_x"], px, c("x3_ins"), "sub", rv, fp)
    EF.eval_field_op(ch, F["slope_times_p_x_minus_x"], slope, c("p_x_minus_x"), "mul", rv, fp)
    EF.eval_field_op(ch, F["y3_ins"], c("slope_times_p_x_minus_x"), py, "sub", rv, fp)
    _result_eq(ch, real, c("x3_ins"), c("y3_ins"), _write_value_limbs(L.P, 2 * w), nl)
    _eval_access_slice(ch, L.Q, 2 * w, False, L.QPTR, 0, real, rv, L.SHARD, L.CLK)
    _eval_access_slice(ch, L.P, 2 * w, True, L.PPTR, 1, real, rv, L.SHARD, L.CLK)
    ch.receives.append(Lookup([_m(L.SHARD), _m(L.CLK), V.const(sid(EC_ADD[curve])), _m(L.PPTR), _m(L.QPTR)], rv,
                              KIND_SYSCALL))
    return ch


def weierstrass_double_chip(curve: str) -> ChipDesc:
    """WeierstrassDoubleAssignChip::eval (weierstrass_double.rs:277-408)."""
    fp = FIELDS[curve]
    L = DoubleLayout(fp)
    nl, w = fp.nl, fp.words
    ch = ChipDesc(f"{curve}DoubleAssign", prep_width=0, main_width=L.WIDTH, local_only=True)
    real, rv = main(L.REAL), _m(L.REAL)
    px, py = _write_prev_limbs(L.P, w), _write_prev_limbs(L.P + w * WR_W, w)
    F, c = L.F, lambda n: EF.cols(L.F[n], nl)
    EF.eval_field_op(ch, F["p_x_squared"], px, px, "mul", rv, fp)
    EF.eval_field_op(ch, F["p_x_squared_times_3"], c("p_x_squared"), EF.const_limbs(3, fp), "mul", rv, fp)
    EF.eval_field_op(ch, F["slope_numerator"], EF.const_limbs(CURVE_A[curve], fp), c("p_x_squared_times_3"), "add",
                     rv, fp)
    EF.eval_field_op(ch, F["slope_denominator"], EF.const_limbs(2, fp), py, "mul", rv, fp)
    EF.eval_field_op(ch, F["slope"], c("slope_numerator"), c("slope_denominator"), "div", rv, fp)
    slope = c("slope")
    EF.eval_field_op(ch, F["slope_squared"], slope, slope, "mul", rv, fp)
    EF.eval_field_op(ch, F["p_x_plus_p_x"], px, px, "add", rv, fp)
    EF.eval_field_op(ch, F["x3_ins"], c("slope_squared"), c("p_x_plus_p_x"), "sub", rv, fp)
    EF.eval_field_op(ch, F["p_x_minus_x"], px, c("x3_ins"), "sub", rv, fp)
    EF.eval_field_op(ch, F["slope_times_p_x_minus_x"], slope, c("p_x_minus_x"), "mul", rv, fp)
    EF.eval_field_op(ch, F["y3_ins"], c("slope_times_p_x_minus_x"), py, "sub", rv, fp)
    _result_eq(ch, real, c("x3_ins"), c("y3_ins"), _write_value_limbs(L.P, 2 * w), nl)
    _eval_access_slice(ch, L.P, 2 * w, True, L.PPTR, 0, real, rv, L.SHARD, L.CLK)
    ch.receives.append(Lookup([_m(L.SHARD), _m(L.CLK), V.const(sid(EC_DOUBLE[curve])), _m(L.PPTR), V.const(0)], rv,
                              KIND_SYSCALL))
    return ch


# ---------------------------------------------------------------- field towers
class FpLayout:
    """FpOpCols (fptower/fp.rs:38-51)."""

    def __init__(self, fp: FieldParams):
        (self.REAL, self.SHARD, self.CLK, self.IS_ADD, self.IS_SUB, self.IS_MUL, self.XPTR,
         self.YPTR) = range(8)
        self.X = 8
        self.Y = self.X + fp.words * WR_W
        self.OUT = self.Y + fp.words * RD_W
        self.WIDTH = self.OUT + fp.fop_w


def fp_op_chip(field: str) -> ChipDesc:
    """FpOpChip::eval (fptower/fp.rs:191-269)."""
    fp = FIELDS[field]
    L = FpLayout(fp)
    ch = ChipDesc(FP_NAME[field], prep_width=0, main_width=L.WIDTH, local_only=True)
    real, rv = main(L.REAL), _m(L.REAL)
    ia, isb, im = main(L.IS_ADD), main(L.IS_SUB), main(L.IS_MUL)
    for f in (ia, isb, im):
        _assert_bool(ch, f)
    ch.assert_zero(ia + isb + im - 1)
    p = _write_prev_limbs(L.X, fp.words)
    q = _read_limbs(L.Y, fp.words)
    _eval_variable(ch, L.OUT, p, q, fp.mod_limbs, ia, isb, im, rv, fp)
    for a, b in zip(EF.cols(L.OUT, fp.nl), _write_value_limbs(L.X, fp.words)):
        ch.assert_zero(real * (a - b))
    _eval_access_slice(ch, L.Y, fp.words, False, L.YPTR, 0, real, rv, L.SHARD, L.CLK)
    _eval_access_slice(ch, L.X, fp.words, True, L.XPTR, 1, real, rv, L.SHARD, L.CLK)
    add, sub, mul = (sid(c) for c in FP_OPS[field])
    ident = V([("main", L.IS_ADD, add), ("main", L.IS_SUB, sub), ("main", L.IS_MUL, mul)], 0)
    ch.receives.append(Lookup([_m(L.SHARD), _m(L.CLK), ident, _m(L.XPTR), _m(L.YPTR)], rv, KIND_SYSCALL))
    return ch


class Fp2AddSubLayout:
    """Fp2AddSubAssignCols (fptower/fp2_addsub.rs:40-51)."""

    def __init__(self, fp: FieldParams):
        self.REAL, self.SHARD, self.CLK, self.IS_ADD, self.XPTR, self.YPTR = range(6)
        self.X = 6
        self.Y = self.X + 2 * fp.words * WR_W
        self.C0 = self.Y + 2 * fp.words * RD_W
        self.C1 = self.C0 + fp.fop_w
        self.WIDTH = self.C1 + fp.fop_w


def fp2_addsub_chip(field: str) -> ChipDesc:
    """Fp2AddSubAssignChip::eval (fptower/fp2_addsub.rs:199-282)."""
    fp = FIELDS[field]
    L = Fp2AddSubLayout(fp)
    w = fp.words
    ch = ChipDesc(FP2_ADDSUB_NAME[field], prep_width=0, main_width=L.WIDTH, local_only=True)
    real, rv = main(L.REAL), _m(L.REAL)
    ia = main(L.IS_ADD)
    _assert_bool(ch, ia)
    px, py = _write_prev_limbs(L.X, w), _write_prev_limbs(L.X + w * WR_W, w)
    qx, qy = _read_limbs(L.Y, w), _read_limbs(L.Y + w * RD_W, w)
    _eval_variable(ch, L.C0, px, qx, fp.mod_limbs, ia, 1 - ia, 0, rv, fp)
    _eval_variable(ch, L.C1, py, qy, fp.mod_limbs, ia, 1 - ia, 0, rv, fp)
    xv = _write_value_limbs(L.X, 2 * w)
    for a, b in zip(EF.cols(L.C0, fp.nl), xv[:fp.nl]):
        ch.assert_zero(real * (a - b))
    for a, b in zip(EF.cols(L.C1, fp.nl), xv[fp.nl:]):
        ch.assert_zero(real * (a - b))
    _eval_access_slice(ch, L.Y, 2 * w, False, L.YPTR, 0, real, rv, L.SHARD, L.CLK)
    _eval_access_slice(ch, L.X, 2 * w, True, L.XPTR, 1, real, rv, L.SHARD, L.CLK)
    add, sub = (sid(c) for c in FP2_ADDSUB[field])
    ident = V([("main", L.IS_ADD, (add - sub) % P)], sub)
    ch.receives.append(Lookup([_m(L.SHARD), _m(L.CLK), ident, _m(L.XPTR), _m(L.YPTR)], rv, KIND_SYSCALL))
    return ch


class Fp2MulLayout:
    """Fp2MulAssignCols (fptower/fp2_mul.rs:40-55)."""

    def __init__(self, fp: FieldParams):
        self.REAL, self.SHARD, self.CLK, self.XPTR, self.YPTR = range(5)
        self.X = 5
        self.Y = self.X + 2 * fp.words * WR_W
        base = self.Y + 2 * fp.words * RD_W
        names = ["a0_mul_b0", "a1_mul_b1", "a0_mul_b1", "a1_mul_b0", "c0", "c1"]
        self.F = {n: base + k * fp.fop_w for k, n in enumerate(names)}
        self.WIDTH = base + len(names) * fp.fop_w


def fp2_mul_chip(field: str) -> ChipDesc:
    """Fp2MulAssignChip::eval (fptower/fp2_mul.rs:225-331)."""
    fp = FIELDS[field]
    L = Fp2MulLayout(fp)
    w, nl = fp.words, fp.nl
    ch = ChipDesc(FP2_MUL_NAME[field], prep_width=0, main_width=L.WIDTH, local_only=True)
    real, rv = main(L.REAL), _m(L.REAL)
    px, py = _write_prev_limbs(L.X, w), _write_prev_limbs(L.X + w * WR_W, w)
    qx, qy = _read_limbs(L.Y, w), _read_limbs(L.Y + w * RD_W, w)
    F, c = L.F, lambda n: EF.cols(L.F[n], nl)
    EF.eval_field_op(ch, F["a0_mul_b0"], px, qx, "mul", rv, fp)
    EF.eval_field_op(ch, F["a1_mul_b1"], py, qy, "mul", rv, fp)
    EF.eval_field_op(ch, F["c0"], c("a0_mul_b0"), c("a1_mul_b1"), "sub", rv, fp)
    EF.eval_field_op(ch, F["a0_mul_b1"], px, qy, "mul", rv, fp)
    EF.eval_field_op(ch, F["a1_mul_b0"], py, qx, "mul", rv, fp)
    EF.eval_field_op(ch, F["c1"], c("a0_mul_b1"), c("a1_mul_b0"), "add", rv, fp)
    xv = _write_value_limbs(L.X, 2 * w)
    for a, b in zip(c("c0"), xv[:nl]):
        ch.assert_zero(real * (a - b))
    for a, b in zip(c("c1"), xv[nl:]):
        ch.assert_zero(real * (a - b))
    _eval_access_slice(ch, L.Y, 2 * w, False, L.YPTR, 0, real, rv, L.SHARD, L.CLK)
    _eval_access_slice(ch, L.X, 2 * w, True, L.XPTR, 1, real, rv, L.SHARD, L.CLK)
    ch.receives.append(Lookup([_m(L.SHARD), _m(L.CLK), V.const(sid(FP2_MUL[field])), _m(L.XPTR), _m(L.YPTR)], rv,
                              KIND_SYSCALL))
    return ch


# ---------------------------------------------------------------- Uint256MulMod
class U256Layout:
    """Uint256MulCols (uint256/air.rs:37-67)."""

    def __init__(self):
        self.SHARD, self.CLK, self.XPTR, self.YPTR = range(4)
        self.X = 4
        self.Y = self.X + 8 * WR_W
        self.M = self.Y + 8 * RD_W
        self.IZ_INV = self.M + 8 * RD_W          # modulus_is_zero: IsZeroOperation (inverse, result)
        self.IZ_RES = self.IZ_INV + 1
        self.NOT_ZERO = self.IZ_RES + 1          # modulus_is_not_zero
        self.OUT = self.NOT_ZERO + 1             # FieldOpCols<U256Field>
        self.LT = self.OUT + U256.fop_w          # FieldLtCols<U256Field>
        self.REAL = self.LT + U256.lt_w
        self.WIDTH = self.REAL + 1


U256L = U256Layout()


def uint256_mul_chip() -> ChipDesc:
    """Uint256MulChip::eval (uint256/air.rs:189-281)."""
    L = U256L
    ch = ChipDesc("Uint256MulMod", prep_width=0, main_width=L.WIDTH, local_only=True)
    real, rv = main(L.REAL), _m(L.REAL)
    x = _write_prev_limbs(L.X, 8)
    y = _read_limbs(L.Y, 8)
    m = _read_limbs(L.M, 8)
    # IsZeroOperation::eval on the modulus byte sum (operations/is_zero.rs)
    s = Expr.lift(0)
    for b in m:
        s = s + b
    iz = main(L.IZ_RES)
    ch.assert_zero(real * ((1 - main(L.IZ_INV) * s) - iz))
    _assert_bool(ch, iz, real)
    ch.assert_zero(real * iz * s)
    # p_modulus = m (1 - is_zero) + x^32 is_zero
    p_mod = EF.p_add(EF.p_scale(m, 1 - iz), [0] * 32 + [iz])
    EF.eval_field_op(ch, L.OUT, x, y, "mul", rv, U256, modulus=p_mod)
    EF.eval_field_lt(ch, L.LT, EF.cols(L.OUT, 32), m, main(L.NOT_ZERO), _m(L.NOT_ZERO), U256)
    ch.assert_zero(main(L.NOT_ZERO) - real * (1 - iz))
    for a, b in zip(EF.cols(L.OUT, 32), _write_value_limbs(L.X, 8)):
        ch.assert_zero(real * (a - b))
    _eval_access_slice(ch, L.X, 8, True, L.XPTR, 1, real, rv, L.SHARD, L.CLK)
    _eval_access_slice(ch, L.Y, 16, False, L.YPTR, 0, real, rv, L.SHARD, L.CLK)
    ch.receives.append(Lookup([_m(L.SHARD), _m(L.CLK), V.const(sid(UINT256_MUL)), _m(L.XPTR), _m(L.YPTR)], rv,
                              KIND_SYSCALL))
    _assert_bool(ch, real)
    return ch


# ---------------------------------------------------------------- curve arithmetic (trace / executor side)
def sw_add(curve: str, p, q):
    """AffinePoint::sw_add (weierstrass/mod.rs:175-202); p != q."""
    m = FIELDS[curve].modulus
    (x1, y1), (x2, y2) = p, q
    assert (x1, y1) != (x2, y2), "points are the same: use sw_double"
    s = (y2 - y1) % m * pow((x2 - x1) % m, -1, m) % m
    x3 = (s * s - x1 - x2) % m
    return x3, (s * (x1 - x3) - y1) % m


def sw_double(curve: str, p):
    """AffinePoint::sw_double (weierstrass/mod.rs:204-240)."""
    m = FIELDS[curve].modulus
    x1, y1 = p
    s = (CURVE_A[curve] + 3 * x1 * x1) % m * pow(2 * y1 % m, -1, m) % m
    x3 = (s * s - 2 * x1) % m
    return x3, (s * (x1 - x3) - y1) % m


def point_from_x(curve: str, x: int):
    """A curve point with abscissa x, or None (every base field here has p = 3 mod 4)."""
    m = FIELDS[curve].modulus
    assert m % 4 == 3
    rhs = (x * x * x + CURVE_A[curve] * x + CURVE_B[curve]) % m
    y = pow(rhs, (m + 1) // 4, m)
    return (x, y) if y * y % m == rhs else None


def random_point(curve: str, rng):
    m = FIELDS[curve].modulus
    while True:
        x = int.from_bytes(rng.bytes(FIELDS[curve].nl), "little") % m
        pt = point_from_x(curve, x)
        if pt is not None:
            return pt


def point_words(curve: str, pt) -> List[int]:
    w = FIELDS[curve].words
    return EF.int_to_words(pt[0], w) + EF.int_to_words(pt[1], w)


# ---------------------------------------------------------------- executor (syscalls)
def exec_ec_add(curve: str, pm, shard: int, clk: int, p_ptr: int, q_ptr: int):
    """create_ec_add_event (events/precompiles/ec.rs:96-139)."""
    nw = 2 * FIELDS[curve].words
    assert p_ptr % 4 == 0 and q_ptr % 4 == 0
    p = [pm.peek(p_ptr + 4 * i) for i in range(nw)]
    q = [pm.read(q_ptr + 4 * i, clk) for i in range(nw)]
    h = nw // 2
    pt = (EF.words_to_int(p[:h]), EF.words_to_int(p[h:]))
    qt = (EF.words_to_int([r[0] for r in q[:h]]), EF.words_to_int([r[0] for r in q[h:]]))
    res = point_words(curve, sw_add(curve, pt, qt))
    pw = [pm.write(p_ptr + 4 * i, res[i], clk + 1) for i in range(nw)]
    return {"shard": shard, "clk": clk, "p_ptr": p_ptr, "q_ptr": q_ptr, "p": p, "q": q, "pw": pw,
            "local": pm.local_entries()}


def exec_ec_double(curve: str, pm, shard: int, clk: int, p_ptr: int, _a1: int):
    """create_ec_double_event (events/precompiles/ec.rs:141-173): p written at clk."""
    nw = 2 * FIELDS[curve].words
    assert p_ptr % 4 == 0
    p = [pm.peek(p_ptr + 4 * i) for i in range(nw)]
    h = nw // 2
    res = point_words(curve, sw_double(curve, (EF.words_to_int(p[:h]), EF.words_to_int(p[h:]))))
    pw = [pm.write(p_ptr + 4 * i, res[i], clk) for i in range(nw)]
    return {"shard": shard, "clk": clk, "p_ptr": p_ptr, "p": p, "pw": pw, "local": pm.local_entries()}


def exec_fp_op(field: str, op: str, pm, shard: int, clk: int, x_ptr: int, y_ptr: int):
    """FpOpSyscall::execute (executor/src/syscalls/precompiles/fptower/fp.rs)."""
    fp = FIELDS[field]
    m, nw = fp.modulus, fp.words
    assert x_ptr % 4 == 0 and y_ptr % 4 == 0
    x = [pm.peek(x_ptr + 4 * i) for i in range(nw)]
    yr = [pm.read(y_ptr + 4 * i, clk) for i in range(nw)]
    a, b = EF.words_to_int(x) % m, EF.words_to_int([r[0] for r in yr]) % m
    r = {"add": (a + b) % m, "sub": (a + m - b) % m, "mul": a * b % m}[op]
    res = EF.int_to_words(r, nw)
    xw = [pm.write(x_ptr + 4 * i, res[i], clk + 1) for i in range(nw)]
    return {"shard": shard, "clk": clk, "x_ptr": x_ptr, "y_ptr": y_ptr, "op": op, "x": x, "y": yr, "xw": xw,
            "local": pm.local_entries()}


def exec_fp2_addsub(field: str, op: str, pm, shard: int, clk: int, x_ptr: int, y_ptr: int):
    """Fp2AddSubSyscall::execute (executor/src/syscalls/precompiles/fptower/fp2_addsub.rs)."""
    fp = FIELDS[field]
    m, nw = fp.modulus, 2 * fp.words
    x = [pm.peek(x_ptr + 4 * i) for i in range(nw)]
    yr = [pm.read(y_ptr + 4 * i, clk) for i in range(nw)]
    h = nw // 2
    ac0, ac1 = EF.words_to_int(x[:h]) % m, EF.words_to_int(x[h:]) % m
    bc0, bc1 = EF.words_to_int([r[0] for r in yr[:h]]) % m, EF.words_to_int([r[0] for r in yr[h:]]) % m
    if op == "add":
        c0, c1 = (ac0 + bc0) % m, (ac1 + bc1) % m
    else:
        c0, c1 = (ac0 + m - bc0) % m, (ac1 + m - bc1) % m
    res = EF.int_to_words(c0, h) + EF.int_to_words(c1, h)
    xw = [pm.write(x_ptr + 4 * i, res[i], clk + 1) for i in range(nw)]
    return {"shard": shard, "clk": clk, "x_ptr": x_ptr, "y_ptr": y_ptr, "op": op, "x": x, "y": yr, "xw": xw,
            "local": pm.local_entries()}


def exec_fp2_mul(field: str, pm, shard: int, clk: int, x_ptr: int, y_ptr: int):
    """Fp2MulSyscall::execute (executor/src/syscalls/precompiles/fptower/fp2_mul.rs): (a0 + a1 u)(b0 + b1 u)
    with u^2 = -1."""
    fp = FIELDS[field]
    m, nw = fp.modulus, 2 * fp.words
    x = [pm.peek(x_ptr + 4 * i) for i in range(nw)]
    yr = [pm.read(y_ptr + 4 * i, clk) for i in range(nw)]
    h = nw // 2
    a0, a1 = EF.words_to_int(x[:h]) % m, EF.words_to_int(x[h:]) % m
    b0, b1 = EF.words_to_int([r[0] for r in yr[:h]]) % m, EF.words_to_int([r[0] for r in yr[h:]]) % m
    c0 = (a0 * b0 % m + m - a1 * b1 % m) % m
    c1 = (a0 * b1 % m + a1 * b0 % m) % m
    res = EF.int_to_words(c0, h) + EF.int_to_words(c1, h)
    xw = [pm.write(x_ptr + 4 * i, res[i], clk + 1) for i in range(nw)]
    return {"shard": shard, "clk": clk, "x_ptr": x_ptr, "y_ptr": y_ptr, "x": x, "y": yr, "xw": xw,
            "local": pm.local_entries()}


def exec_uint256_mul(pm, shard: int, clk: int, x_ptr: int, y_ptr: int):
    """Uint256MulSyscall::execute (executor/src/syscalls/precompiles/uint256.rs)."""
    assert x_ptr % 4 == 0 and y_ptr % 4 == 0
    x = [pm.peek(x_ptr + 4 * i) for i in range(8)]
    yr = [pm.read(y_ptr + 4 * i, clk) for i in range(8)]
    mr = [pm.read(y_ptr + 32 + 4 * i, clk) for i in range(8)]
    a, b = EF.words_to_int(x), EF.words_to_int([r[0] for r in yr])
    m = EF.words_to_int([r[0] for r in mr])
    res = EF.int_to_words(a * b % (m if m else 1 << 256), 8)
    xw = [pm.write(x_ptr + 4 * i, res[i], clk + 1) for i in range(8)]
    return {"shard": shard, "clk": clk, "x_ptr": x_ptr, "y_ptr": y_ptr, "x": x, "y": yr, "m": mr, "xw": xw,
            "local": pm.local_entries()}


def _bind(fn, *args):
    return lambda pm, shard, clk, a0, a1: fn(*args, pm, shard, clk, a0, a1)


def precompile_table():
    """syscall code -> executor, for mips_syscall.PRECOMPILES."""
    t = {}
    for curve in FIELDS:
        t[EC_ADD[curve]] = _bind(exec_ec_add, curve)
        t[EC_DOUBLE[curve]] = _bind(exec_ec_double, curve)
    for field in FP_OPS:
        for code, op in zip(FP_OPS[field], ("add", "sub", "mul")):
            t[code] = _bind(exec_fp_op, field, op)
        for code, op in zip(FP2_ADDSUB[field], ("add", "sub")):
            t[code] = _bind(exec_fp2_addsub, field, op)
        t[FP2_MUL[field]] = _bind(exec_fp2_mul, field)
    t[UINT256_MUL] = exec_uint256_mul
    for curve in EC_DECOMPRESS:
        t[EC_DECOMPRESS[curve]] = _bind(exec_ec_decompress, curve)
    t[_p2().POSEIDON2_PERMUTE] = _p2().exec_poseidon2_permute
    t[_keccak().KECCAK_SPONGE] = _keccak().exec_keccak_sponge
    t[U256XU2048_MUL] = exec_u256x2048_mul
    return t


# ---------------------------------------------------------------- traces
def _access_block(t, rows, base, recs, write: bool, shard, clk, byte_lookup):
    """MemoryReadCols / MemoryWriteCols populate for word records at timestamp clk (per row)."""
    from .mips_edwards import _access_block as ab
    ab(t, rows, base, recs, write, shard, clk, byte_lookup)


def _height(n: int) -> int:
    return max(16, 1 << max(0, (n - 1).bit_length()))


def _fill(t, base, fp, res_cols):
    t[:, base:base + fp.fop_w] = res_cols


def weierstrass_add_trace(curve: str, events, byte_lookup) -> np.ndarray:
    """WeierstrassAddAssignChip::generate_trace + populate_row (weierstrass_add.rs:192-252, :384-420):
    padding rows hold the field operations on zero inputs."""
    fp = FIELDS[curve]
    L = AddLayout(fp)
    ne, h, hw = len(events), _height(len(events)), fp.words
    t = np.zeros((h, L.WIDTH), np.int64)
    rec = EF.Rec(byte_lookup)
    px, py, qx, qy = [0] * h, [0] * h, [0] * h, [0] * h
    for i, e in enumerate(events):
        px[i], py[i] = EF.words_to_int(e["p"][:hw]), EF.words_to_int(e["p"][hw:])
        qv = [r[0] for r in e["q"]]
        qx[i], qy[i] = EF.words_to_int(qv[:hw]), EF.words_to_int(qv[hw:])
    F = L.F
    num, t[:, F["slope_numerator"]:F["slope_numerator"] + fp.fop_w] = EF.pop_field_op(qy, py, "sub", fp)
    den, t[:, F["slope_denominator"]:F["slope_denominator"] + fp.fop_w] = EF.pop_field_op(qx, px, "sub", fp)
    slope, t[:, F["slope"]:F["slope"] + fp.fop_w] = EF.pop_field_op(num, den, "div", fp)
    s2, t[:, F["slope_squared"]:F["slope_squared"] + fp.fop_w] = EF.pop_field_op(slope, slope, "mul", fp)
    pq, t[:, F["p_x_plus_q_x"]:F["p_x_plus_q_x"] + fp.fop_w] = EF.pop_field_op(px, qx, "add", fp)
    x3, t[:, F["x3_ins"]:F["x3_ins"] + fp.fop_w] = EF.pop_field_op(s2, pq, "sub", fp)
    pmx, t[:, F["p_x_minus_x"]:F["p_x_minus_x"] + fp.fop_w] = EF.pop_field_op(px, x3, "sub", fp)
    stp, t[:, F["slope_times_p_x_minus_x"]:F["slope_times_p_x_minus_x"] + fp.fop_w] = EF.pop_field_op(
        slope, pmx, "mul", fp)
    y3, t[:, F["y3_ins"]:F["y3_ins"] + fp.fop_w] = EF.pop_field_op(stp, py, "sub", fp)
    for base in F.values():
        rec.fop(t[:ne, base:base + fp.fop_w], fp)
    if ne:
        rows = np.arange(ne)
        t[rows, L.REAL] = 1
        shard = np.array([e["shard"] for e in events], np.int64)
        clk = np.array([e["clk"] for e in events], np.int64)
        t[rows, L.SHARD], t[rows, L.CLK] = shard, clk
        t[rows, L.PPTR] = [e["p_ptr"] for e in events]
        t[rows, L.QPTR] = [e["q_ptr"] for e in events]
        for i in range(ne):
            assert (x3[i], y3[i]) == sw_add(curve, (px[i], py[i]), (qx[i], qy[i]))
        _access_block(t, rows, L.Q, [e["q"] for e in events], False, shard, clk, byte_lookup)
        _access_block(t, rows, L.P, [e["pw"] for e in events], True, shard, clk + 1, byte_lookup)
    return (t % P).astype(np.uint32)


def weierstrass_double_trace(curve: str, events, byte_lookup) -> np.ndarray:
    """WeierstrassDoubleAssignChip::generate_trace + populate_row (weierstrass_double.rs:201-270,
    :411-440); padding rows: the field operations of p = (0, 1), whose y comes from a dummy write record
    (value 1, timestamp 1, previous value 1) in the first y word."""
    fp = FIELDS[curve]
    L = DoubleLayout(fp)
    ne, h, hw = len(events), _height(len(events)), fp.words
    t = np.zeros((h, L.WIDTH), np.int64)
    rec = EF.Rec(byte_lookup)
    px, py = [0] * h, [1] * h
    for i, e in enumerate(events):
        px[i], py[i] = EF.words_to_int(e["p"][:hw]), EF.words_to_int(e["p"][hw:])
    F = L.F
    a = CURVE_A[curve]
    x2, t[:, F["p_x_squared"]:F["p_x_squared"] + fp.fop_w] = EF.pop_field_op(px, px, "mul", fp)
    x23, t[:, F["p_x_squared_times_3"]:F["p_x_squared_times_3"] + fp.fop_w] = EF.pop_field_op(x2, [3] * h, "mul",
                                                                                                 fp)
    num, t[:, F["slope_numerator"]:F["slope_numerator"] + fp.fop_w] = EF.pop_field_op([a] * h, x23, "add", fp)
    den, t[:, F["slope_denominator"]:F["slope_denominator"] + fp.fop_w] = EF.pop_field_op([2] * h, py, "mul", fp)
    slope, t[:, F["slope"]:F["slope"] + fp.fop_w] = EF.pop_field_op(num, den, "div", fp)
    s2, t[:, F["slope_squared"]:F["slope_squared"] + fp.fop_w] = EF.pop_field_op(slope, slope, "mul", fp)
    pp, t[:, F["p_x_plus_p_x"]:F["p_x_plus_p_x"] + fp.fop_w] = EF.pop_field_op(px, px, "add", fp)
    x3, t[:, F["x3_ins"]:F["x3_ins"] + fp.fop_w] = EF.pop_field_op(s2, pp, "sub", fp)
    pmx, t[:, F["p_x_minus_x"]:F["p_x_minus_x"] + fp.fop_w] = EF.pop_field_op(px, x3, "sub", fp)
    stp, t[:, F["slope_times_p_x_minus_x"]:F["slope_times_p_x_minus_x"] + fp.fop_w] = EF.pop_field_op(
        slope, pmx, "mul", fp)
    y3, t[:, F["y3_ins"]:F["y3_ins"] + fp.fop_w] = EF.pop_field_op(stp, py, "sub", fp)
    for base in F.values():
        rec.fop(t[:ne, base:base + fp.fop_w], fp)
    # the dummy write record of the padding rows: y word 0, prev_value 1, value 1, compare 1 (same
    # shard 0), timestamp difference 1 - 0 - 1 = 0
    from .mips_core import ACC_COMPARE
    y0 = L.P + hw * WR_W
    t[ne:, y0] = 1
    t[ne:, y0 + 4 + ACC_VALUE] = 1
    t[ne:, y0 + 4 + ACC_COMPARE] = 1
    if ne:
        rows = np.arange(ne)
        t[rows, L.REAL] = 1
        shard = np.array([e["shard"] for e in events], np.int64)
        clk = np.array([e["clk"] for e in events], np.int64)
        t[rows, L.SHARD], t[rows, L.CLK] = shard, clk
        t[rows, L.PPTR] = [e["p_ptr"] for e in events]
        for i in range(ne):
            assert (x3[i], y3[i]) == sw_double(curve, (px[i], py[i]))
        _access_block(t, rows, L.P, [e["pw"] for e in events], True, shard, clk, byte_lookup)
    return (t % P).astype(np.uint32)


def fp_op_trace(field: str, events, byte_lookup) -> np.ndarray:
    """FpOpChip::generate_trace (fptower/fp.rs:90-160): padding rows are the addition 0 + 0 (is_add = 1)."""
    fp = FIELDS[field]
    L = FpLayout(fp)
    ne, h, m = len(events), _height(len(events)), fp.modulus
    t = np.zeros((h, L.WIDTH), np.int64)
    rec = EF.Rec(byte_lookup)
    ops = [e["op"] for e in events] + ["add"] * (h - ne)
    a = [EF.words_to_int(e["x"]) % m for e in events] + [0] * (h - ne)
    b = [EF.words_to_int([r[0] for r in e["y"]]) % m for e in events] + [0] * (h - ne)
    for op in ("add", "sub", "mul"):
        idx = [i for i in range(h) if ops[i] == op]
        if idx:
            _, c = EF.pop_field_op([a[i] for i in idx], [b[i] for i in idx], op, fp)
            t[idx, L.OUT:L.OUT + fp.fop_w] = c
    t[:, L.IS_ADD] = [o == "add" for o in ops]
    t[:, L.IS_SUB] = [o == "sub" for o in ops]
    t[:, L.IS_MUL] = [o == "mul" for o in ops]
    rec.fop(t[:ne, L.OUT:L.OUT + fp.fop_w], fp)
    if ne:
        rows = np.arange(ne)
        t[rows, L.REAL] = 1
        shard = np.array([e["shard"] for e in events], np.int64)
        clk = np.array([e["clk"] for e in events], np.int64)
        t[rows, L.SHARD], t[rows, L.CLK] = shard, clk
        t[rows, L.XPTR] = [e["x_ptr"] for e in events]
        t[rows, L.YPTR] = [e["y_ptr"] for e in events]
        _access_block(t, rows, L.Y, [e["y"] for e in events], False, shard, clk, byte_lookup)
        _access_block(t, rows, L.X, [e["xw"] for e in events], True, shard, clk + 1, byte_lookup)
    return (t % P).astype(np.uint32)


def fp2_addsub_trace(field: str, events, byte_lookup) -> np.ndarray:
    """Fp2AddSubAssignChip::generate_trace (fptower/fp2_addsub.rs:93-183): padding rows add zeros."""
    fp = FIELDS[field]
    L = Fp2AddSubLayout(fp)
    ne, h, m, hw = len(events), _height(len(events)), fp.modulus, fp.words
    t = np.zeros((h, L.WIDTH), np.int64)
    rec = EF.Rec(byte_lookup)
    ops = [e["op"] for e in events] + ["add"] * (h - ne)
    xs = [(EF.words_to_int(e["x"][:hw]) % m, EF.words_to_int(e["x"][hw:]) % m) for e in events]
    ys = [(EF.words_to_int([r[0] for r in e["y"][:hw]]) % m, EF.words_to_int([r[0] for r in e["y"][hw:]]) % m)
          for e in events]
    xs += [(0, 0)] * (h - ne)
    ys += [(0, 0)] * (h - ne)
    for op in ("add", "sub"):
        idx = [i for i in range(h) if ops[i] == op]
        if idx:
            for k, base in ((0, L.C0), (1, L.C1)):
                _, c = EF.pop_field_op([xs[i][k] for i in idx], [ys[i][k] for i in idx], op, fp)
                t[idx, base:base + fp.fop_w] = c
    t[:, L.IS_ADD] = [o == "add" for o in ops]
    rec.fop(t[:ne, L.C0:L.C0 + fp.fop_w], fp)
    rec.fop(t[:ne, L.C1:L.C1 + fp.fop_w], fp)
    if ne:
        rows = np.arange(ne)
        t[rows, L.REAL] = 1
        shard = np.array([e["shard"] for e in events], np.int64)
        clk = np.array([e["clk"] for e in events], np.int64)
        t[rows, L.SHARD], t[rows, L.CLK] = shard, clk
        t[rows, L.XPTR] = [e["x_ptr"] for e in events]
        t[rows, L.YPTR] = [e["y_ptr"] for e in events]
        _access_block(t, rows, L.Y, [e["y"] for e in events], False, shard, clk, byte_lookup)
        _access_block(t, rows, L.X, [e["xw"] for e in events], True, shard, clk + 1, byte_lookup)
    return (t % P).astype(np.uint32)


def fp2_mul_trace(field: str, events, byte_lookup) -> np.ndarray:
    """Fp2MulAssignChip::generate_trace (fptower/fp2_mul.rs:122-210): padding rows multiply zeros."""
    fp = FIELDS[field]
    L = Fp2MulLayout(fp)
    ne, h, m, hw = len(events), _height(len(events)), fp.modulus, fp.words
    t = np.zeros((h, L.WIDTH), np.int64)
    rec = EF.Rec(byte_lookup)
    a0 = [EF.words_to_int(e["x"][:hw]) % m for e in events] + [0] * (h - ne)
    a1 = [EF.words_to_int(e["x"][hw:]) % m for e in events] + [0] * (h - ne)
    b0 = [EF.words_to_int([r[0] for r in e["y"][:hw]]) % m for e in events] + [0] * (h - ne)
    b1 = [EF.words_to_int([r[0] for r in e["y"][hw:]]) % m for e in events] + [0] * (h - ne)
    F = L.F
    r00, t[:, F["a0_mul_b0"]:F["a0_mul_b0"] + fp.fop_w] = EF.pop_field_op(a0, b0, "mul", fp)
    r11, t[:, F["a1_mul_b1"]:F["a1_mul_b1"] + fp.fop_w] = EF.pop_field_op(a1, b1, "mul", fp)
    r01, t[:, F["a0_mul_b1"]:F["a0_mul_b1"] + fp.fop_w] = EF.pop_field_op(a0, b1, "mul", fp)
    r10, t[:, F["a1_mul_b0"]:F["a1_mul_b0"] + fp.fop_w] = EF.pop_field_op(a1, b0, "mul", fp)
    _, t[:, F["c0"]:F["c0"] + fp.fop_w] = EF.pop_field_op(r00, r11, "sub", fp)
    _, t[:, F["c1"]:F["c1"] + fp.fop_w] = EF.pop_field_op(r01, r10, "add", fp)
    for base in F.values():
        rec.fop(t[:ne, base:base + fp.fop_w], fp)
    if ne:
        rows = np.arange(ne)
        t[rows, L.REAL] = 1
        shard = np.array([e["shard"] for e in events], np.int64)
        clk = np.array([e["clk"] for e in events], np.int64)
        t[rows, L.SHARD], t[rows, L.CLK] = shard, clk
        t[rows, L.XPTR] = [e["x_ptr"] for e in events]
        t[rows, L.YPTR] = [e["y_ptr"] for e in events]
        _access_block(t, rows, L.Y, [e["y"] for e in events], False, shard, clk, byte_lookup)
        _access_block(t, rows, L.X, [e["xw"] for e in events], True, shard, clk + 1, byte_lookup)
    return (t % P).astype(np.uint32)


def uint256_mul_trace(events, byte_lookup) -> np.ndarray:
    """Uint256MulChip::generate_trace (uint256/air.rs:103-186): the product mod m (2^256 when m = 0);
    the range check result < m only when m != 0; padding rows multiply zeros modulo 2^256."""
    L = U256L
    ne, h = len(events), _height(len(events))
    t = np.zeros((h, L.WIDTH), np.int64)
    rec = EF.Rec(byte_lookup)
    x = [EF.words_to_int(e["x"]) for e in events] + [0] * (h - ne)
    y = [EF.words_to_int([r[0] for r in e["y"]]) for e in events] + [0] * (h - ne)
    m = [EF.words_to_int([r[0] for r in e["m"]]) for e in events] + [0] * (h - ne)
    eff = [mm if mm else 1 << 256 for mm in m]
    res, c = EF.pop_field_op(x, y, "mul", U256, modulus=eff)
    t[:, L.OUT:L.OUT + U256.fop_w] = c
    rec.fop(t[:ne, L.OUT:L.OUT + U256.fop_w], U256)
    real = np.zeros(h, bool)
    real[:ne] = True
    nz = real & np.array([mm != 0 for mm in m])
    t[:, L.LT:L.LT + U256.lt_w] = EF.pop_field_lt(res, rec, nz, U256, rhs=[mm if mm else 0 for mm in m], fill=nz)
    if ne:
        rows = np.arange(ne)
        t[rows, L.REAL] = 1
        shard = np.array([e["shard"] for e in events], np.int64)
        clk = np.array([e["clk"] for e in events], np.int64)
        t[rows, L.SHARD], t[rows, L.CLK] = shard, clk
        t[rows, L.XPTR] = [e["x_ptr"] for e in events]
        t[rows, L.YPTR] = [e["y_ptr"] for e in events]
        bsum = np.array([sum(int.to_bytes(mm, 32, "little")) for mm in m[:ne]], np.int64)
        t[rows, L.IZ_RES] = bsum == 0
        t[rows, L.IZ_INV] = [pow(int(s), P - 2, P) if s else 0 for s in bsum]
        t[rows, L.NOT_ZERO] = bsum != 0
        for i, e in enumerate(events):
            assert EF.words_to_int([r[1] for r in e["xw"]]) == res[i]
        _access_block(t, rows, L.X, [e["xw"] for e in events], True, shard, clk + 1, byte_lookup)
        _access_block(t, rows, L.Y, [e["y"] for e in events], False, shard, clk, byte_lookup)
        _access_block(t, rows, L.M, [e["m"] for e in events], False, shard, clk, byte_lookup)
    return (t % P).astype(np.uint32)


# ---------------------------------------------------------------- chip registry
def chips_in_machine_order() -> List[ChipDesc]:
    """The chips of this module in MipsAir order (mips/mod.rs:223-318): secp256k1 decompress/add/double,
    secp256r1 decompress/add/double, bn254 add/double, bls12-381 add/double, Uint256MulMod, the bls12-381
    towers, the bn254 towers, bls12-381 decompress; Poseidon2Permute (mips_p2permute.py) sits after the
    secp256r1 chips as in the reference, KeccakSponge (mips_keccak.py) after it."""
    return [weierstrass_decompress_chip("Secp256k1"), weierstrass_add_chip("Secp256k1"),
            weierstrass_double_chip("Secp256k1"), weierstrass_decompress_chip("Secp256r1"),
            weierstrass_add_chip("Secp256r1"), weierstrass_double_chip("Secp256r1"),
            _p2().poseidon2_permute_chip(), _keccak().keccak_sponge_chip(),
            weierstrass_add_chip("Bn254"), weierstrass_double_chip("Bn254"),
            weierstrass_add_chip("Bls12381"), weierstrass_double_chip("Bls12381"),
            uint256_mul_chip(), u256x2048_mul_chip(),
            fp_op_chip("Bls12381"), fp2_addsub_chip("Bls12381"), fp2_mul_chip("Bls12381"),
            fp_op_chip("Bn254"), fp2_addsub_chip("Bn254"), fp2_mul_chip("Bn254"),
            weierstrass_decompress_chip("Bls12381")]


def _p2():
    from . import mips_p2permute as P2
    return P2


def _keccak():
    from . import mips_keccak as K
    return K


def chip_for_key(key: int) -> str:
    """Chip name of a precompile event key."""
    if key == _p2().POSEIDON2_PERMUTE:
        return "Poseidon2Permute"
    if key == _keccak().KECCAK_SPONGE:
        return "KeccakSponge"
    if key == U256XU2048_MUL:
        return "U256XU2048Mul"
    for curve in EC_DECOMPRESS:
        if key == EC_DECOMPRESS[curve]:
            return f"{curve}Decompress"
    for curve in FIELDS:
        if key == EC_ADD[curve]:
            return f"{curve}AddAssign"
        if key == EC_DOUBLE[curve]:
            return f"{curve}DoubleAssign"
    for field in FP_OPS:
        if key == FP_OPS[field][0]:
            return FP_NAME[field]
        if key == FP2_ADDSUB[field][0]:
            return FP2_ADDSUB_NAME[field]
        if key == FP2_MUL[field]:
            return FP2_MUL_NAME[field]
    if key == UINT256_MUL:
        return "Uint256MulMod"
    raise KeyError(hex(key))


def trace_for_key(key: int, events, byte_lookup) -> np.ndarray:
    if key == _p2().POSEIDON2_PERMUTE:
        return _p2().poseidon2_permute_trace(events, byte_lookup)
    if key == _keccak().KECCAK_SPONGE:
        return _keccak().keccak_sponge_trace(events, byte_lookup)
    if key == U256XU2048_MUL:
        return u256x2048_mul_trace(events, byte_lookup)
    for curve in EC_DECOMPRESS:
        if key == EC_DECOMPRESS[curve]:
            return weierstrass_decompress_trace(curve, events, byte_lookup)
    for curve in FIELDS:
        if key == EC_ADD[curve]:
            return weierstrass_add_trace(curve, events, byte_lookup)
        if key == EC_DOUBLE[curve]:
            return weierstrass_double_trace(curve, events, byte_lookup)
    for field in FP_OPS:
        if key == FP_OPS[field][0]:
            return fp_op_trace(field, events, byte_lookup)
        if key == FP2_ADDSUB[field][0]:
            return fp2_addsub_trace(field, events, byte_lookup)
        if key == FP2_MUL[field]:
            return fp2_mul_trace(field, events, byte_lookup)
    if key == UINT256_MUL:
        return uint256_mul_trace(events, byte_lookup)
    raise KeyError(hex(key))


# ---------------------------------------------------------------- a guest exercising every syscall here
def ec_program(seed: int = 1, reps: int = 2, halt: bool = True):
    """A guest that calls every precompile of this module `reps` times: per curve P <- P + Q and
    Q <- 2 Q on random points; per tower field x <- x op y for op in add, sub, mul (Fp) and add, sub, mul
    (Fp2); Uint256MulMod with a random modulus and with modulus 0 (2^256).  The result words are read
    back and folded into a register that is committed, then HALT."""
    from . import mips_alu as A
    from . import mips_core as MC
    from . import mips_syscall as SY
    rng = np.random.default_rng(seed)
    prog = []
    acc, tmp = 10, 9
    slot = [MC.DATA_BASE + 0x4000]

    def alloc(nbytes):
        p = slot[0]
        slot[0] += (nbytes + 63) // 64 * 64
        return p

    def li(reg, v):
        prog.append((A.OP_ADD, reg, 0, int(v) & 0xFFFFFFFF, 0, 1))

    def store(ptr, words):
        for i, w in enumerate(words):
            li(8, w)
            prog.append((MC.OP_SW, 8, 0, ptr + 4 * i, 0, 1))

    def syscall(code, a0, a1):
        li(SY.REG_V0, code)
        li(SY.REG_A0, a0)
        li(SY.REG_A1, a1)
        prog.append((SY.OP_SYSCALL, SY.REG_V0, SY.REG_A0, SY.REG_A1, 0, 0))

    def fold(ptr, n):
        for i in range(n):
            prog.append((MC.OP_LW, tmp, 0, ptr + 4 * i, 0, 1))
            prog.append((A.OP_XOR, acc, acc, tmp, 0, 0))

    li(acc, 0)
    for curve in FIELDS:
        nw = 2 * FIELDS[curve].words
        pp, qp = alloc(4 * nw), alloc(4 * nw)
        store(pp, point_words(curve, random_point(curve, rng)))
        store(qp, point_words(curve, random_point(curve, rng)))
        for _ in range(reps):
            syscall(EC_ADD[curve], pp, qp)
            syscall(EC_DOUBLE[curve], qp, 0)
        fold(pp, nw)
        fold(qp, nw)
        if curve in EC_DECOMPRESS:  # decompress a fresh point's x with either sign: y lands at the slot's start
            w = FIELDS[curve].words
            for sign in (0, 1):
                dp = alloc(8 * w)
                store(dp + 4 * w, EF.int_to_words(random_point(curve, rng)[0], w))
                syscall(EC_DECOMPRESS[curve], dp, sign)
                fold(dp, w)
    for field in FP_OPS:
        fp = FIELDS[field]
        w = fp.words
        xp, yp = alloc(4 * w), alloc(4 * w)
        store(xp, EF.int_to_words(int.from_bytes(rng.bytes(fp.nl), "little") % fp.modulus, w))
        store(yp, EF.int_to_words(int.from_bytes(rng.bytes(fp.nl), "little") % fp.modulus, w))
        for _ in range(reps):
            for code in FP_OPS[field]:
                syscall(code, xp, yp)
        fold(xp, w)
        x2, y2 = alloc(8 * w), alloc(8 * w)
        store(x2, EF.int_to_words(int.from_bytes(rng.bytes(fp.nl), "little") % fp.modulus, w)
              + EF.int_to_words(int.from_bytes(rng.bytes(fp.nl), "little") % fp.modulus, w))
        store(y2, EF.int_to_words(int.from_bytes(rng.bytes(fp.nl), "little") % fp.modulus, w)
              + EF.int_to_words(int.from_bytes(rng.bytes(fp.nl), "little") % fp.modulus, w))
        for _ in range(reps):
            for code in FP2_ADDSUB[field] + (FP2_MUL[field],):
                syscall(code, x2, y2)
        fold(x2, 2 * w)
    sp = alloc(64)  # Poseidon2Permute: 16 canonical words permuted in place
    store(sp, [int(v) for v in rng.integers(0, P, WIDTH_P2)])
    for _ in range(reps):
        syscall(_p2().POSEIDON2_PERMUTE, sp, 0)
    fold(sp, WIDTH_P2)
    for zero_mod in (False, True):
        # operands below the modulus (the carry has 32 limbs: x y / m < 2^256)
        xp, yp = alloc(32), alloc(64)
        m = 0 if zero_mod else int.from_bytes(rng.bytes(32), "little") | (1 << 255) | 1
        bound = m if m else 1 << 256
        store(xp, EF.int_to_words(int.from_bytes(rng.bytes(32), "little") % bound, 8))
        store(yp, EF.int_to_words(int.from_bytes(rng.bytes(32), "little") % bound, 8) + EF.int_to_words(m, 8))
        for _ in range(reps):
            syscall(UINT256_MUL, xp, yp)
        fold(xp, 8)
    for _ in range(reps):  # U256XU2048_MUL: lo / hi pointers in A2 / A3
        ap, bp, lop, hip = alloc(32), alloc(256), alloc(256), alloc(32)
        store(ap, EF.int_to_words(int.from_bytes(rng.bytes(32), "little"), 8))
        store(bp, EF.int_to_words(int.from_bytes(rng.bytes(256), "little"), 64))
        li(SY.REG_A2, lop)
        li(SY.REG_A3, hip)
        syscall(U256XU2048_MUL, ap, bp)
        fold(lop, 64)
        fold(hip, 8)
    prog += [(A.OP_ADD, SY.REG_V0, 0, SY.COMMIT, 0, 1), (A.OP_ADD, SY.REG_A0, 0, 0, 0, 1),
             (A.OP_ADD, SY.REG_A1, acc, 0, 0, 1), (SY.OP_SYSCALL, SY.REG_V0, SY.REG_A0, SY.REG_A1, 0, 0)]
    if halt:
        prog += [(A.OP_ADD, SY.REG_V0, 0, SY.HALT, 0, 1), (A.OP_ADD, SY.REG_A0, 0, 0, 0, 1),
                 (SY.OP_SYSCALL, SY.REG_V0, SY.REG_A0, SY.REG_A1, 0, 0)]
    return prog


# ---------------------------------------------------------------- Weierstrass decompress
class DecompressLayout:
    """WeierstrassDecompressCols (weierstrass_decompress.rs:49-65) + LexicographicChoiceCols (:67-80)."""

    def __init__(self, fp: FieldParams, lex: bool):
        w = fp.words
        self.REAL, self.SHARD, self.CLK, self.PTR, self.SIGN = range(5)
        self.X = 5                                   # x_access: MemoryReadCols
        self.Y = self.X + w * RD_W                   # y_access: MemoryReadWriteCols (prev_value + access)
        self.RANGE_X = self.Y + w * WR_W
        self.X2 = self.RANGE_X + fp.lt_w
        self.X3 = self.X2 + fp.fop_w
        self.AXB = self.X3 + fp.fop_w                # FieldInnerProductCols
        self.X3AXB = self.AXB + fp.fop_w
        self.SQRT = self.X3AXB + fp.fop_w            # FieldSqrtCols: multiplication, range, lsb
        self.SQRT_RANGE = self.SQRT + fp.fop_w
        self.SQRT_LSB = self.SQRT_RANGE + fp.lt_w
        self.NEGY = self.SQRT_LSB + 1
        self.WIDTH = self.NEGY + fp.fop_w
        if lex:
            self.CMP = self.WIDTH                    # comparison_lt_cols
            self.NEGY_RANGE = self.CMP + fp.lt_w     # neg_y_range_check
            self.IS_Y_EQ = self.NEGY_RANGE + fp.lt_w
            self.WHEN_SQRT_LT = self.IS_Y_EQ + 1
            self.WHEN_NEG_LT = self.WHEN_SQRT_LT + 1
            self.WIDTH = self.WHEN_NEG_LT + 1


def weierstrass_decompress_chip(curve: str) -> ChipDesc:
    """WeierstrassDecompressChip::eval (weierstrass_decompress.rs:327-492)."""
    from . import mips_alu as A
    from .machine import KIND_BYTE
    from .mips_alu import ZERO
    fp, lex = FIELDS[curve], LEXICOGRAPHIC[curve]
    L = DecompressLayout(fp, lex)
    nl, w = fp.nl, fp.words
    ch = ChipDesc(f"{curve}Decompress", prep_width=0, main_width=L.WIDTH, local_only=True)
    real, rv = main(L.REAL), _m(L.REAL)
    sign = main(L.SIGN)
    _assert_bool(ch, sign)
    x = _read_limbs(L.X, w)
    EF.eval_field_lt(ch, L.RANGE_X, x, fp.mod_limbs, real, rv, fp)
    EF.eval_field_op(ch, L.X2, x, x, "mul", rv, fp)
    EF.eval_field_op(ch, L.X3, EF.cols(L.X2, nl), x, "mul", rv, fp)
    EF.eval_inner_product(ch, L.AXB, [EF.const_limbs(CURVE_A[curve], fp), EF.const_limbs(CURVE_B[curve], fp)],
                          [x, EF.const_limbs(1, fp)], rv, fp)
    EF.eval_field_op(ch, L.X3AXB, EF.cols(L.X3, nl), EF.cols(L.AXB, nl), "add", rv, fp)
    sqrt = EF.cols(L.SQRT, nl)
    EF.eval_field_op(ch, L.NEGY, [0], sqrt, "sub", rv, fp)
    # FieldSqrtCols::eval (field_sqrt.rs:100-145) with is_odd = its own lsb column
    EF.eval_field_op(ch, L.SQRT, sqrt, sqrt, "mul", rv, fp, result=EF.cols(L.X3AXB, nl),
                     result_cols=EF.vcols(L.X3AXB, nl))
    EF.eval_field_lt(ch, L.SQRT_RANGE, sqrt, fp.mod_limbs, real, rv, fp)
    EF.u8_range(ch, EF.vcols(L.SQRT, nl), rv)
    lsb = main(L.SQRT_LSB)
    _assert_bool(ch, lsb)
    ch.assert_zero(real * (lsb - lsb))
    ch.sends.append(Lookup([V.const(A.B_AND), _m(L.SQRT_LSB), ZERO, _m(L.SQRT), V.const(1)], rv, KIND_BYTE))
    y = _write_value_limbs(L.Y, w)
    negy = EF.cols(L.NEGY, nl)
    if not lex:
        # when(is_real).when_ne(lsb, 1 - sign): y = sqrt; when_ne(lsb, sign): y = -sqrt
        for a, b in zip(sqrt, y):
            ch.assert_zero(real * (lsb - (1 - sign)) * (a - b))
        for a, b in zip(negy, y):
            ch.assert_zero(real * (lsb - sign) * (a - b))
    else:
        eq, wsq, wng = main(L.IS_Y_EQ), main(L.WHEN_SQRT_LT), main(L.WHEN_NEG_LT)
        EF.eval_field_lt(ch, L.NEGY_RANGE, negy, fp.mod_limbs, real, rv, fp)
        for f in (eq, wsq, wng):
            _assert_bool(ch, f)
        ch.assert_zero(real * (wsq + wng - 1))
        for a, b in zip(sqrt, y):
            ch.assert_zero(real * eq * (a - b))
        for a, b in zip(negy, y):
            ch.assert_zero(real * (1 - eq) * (a - b))
        ch.assert_zero((1 - real) * wsq)
        ch.assert_zero((1 - real) * wng)
        ch.assert_zero(real * sign * (eq - wng))
        ch.assert_zero(real * (1 - sign) * (eq - wsq))
        EF.eval_field_lt(ch, L.CMP, sqrt, negy, wsq, _m(L.WHEN_SQRT_LT), fp)
        EF.eval_field_lt(ch, L.CMP, negy, sqrt, wng, _m(L.WHEN_NEG_LT), fp)
    # x words at ptr + nl, y words at ptr, both at clk
    _eval_access_slice(ch, L.X, w, False, L.PTR, 0, real, rv, L.SHARD, L.CLK, addr_off=nl)
    _eval_access_slice(ch, L.Y, w, True, L.PTR, 0, real, rv, L.SHARD, L.CLK)
    ch.receives.append(Lookup([_m(L.SHARD), _m(L.CLK), V.const(sid(EC_DECOMPRESS[curve])), _m(L.PTR), _m(L.SIGN)],
                              rv, KIND_SYSCALL))
    return ch


def field_sqrt(curve: str, a: int) -> int:
    """secp256k1_sqrt / secp256r1_sqrt / bls12381_sqrt (crates/curves/src/weierstrass/*.rs, through the
    k256 / p256 / miracl field types): a^((p+1)/4), every field here having p = 3 mod 4."""
    m = FIELDS[curve].modulus
    r = pow(a, (m + 1) // 4, m)
    if r * r % m != a % m:
        raise ValueError("no square root")
    return r


def decompress_y(curve: str, x: int, sign: int) -> int:
    """secp256k1_decompress / secp256r1_decompress (y with parity `sign`) and bls12381_decompress (the
    lexicographically larger of y, -y when `sign`)."""
    m = FIELDS[curve].modulus
    y = field_sqrt(curve, (x * x * x + CURVE_A[curve] * x + CURVE_B[curve]) % m)
    neg = (m - y) % m
    if LEXICOGRAPHIC[curve]:
        return max(y, neg) if sign else min(y, neg)
    return y if (y & 1) == sign else neg


def exec_ec_decompress(curve: str, pm, shard: int, clk: int, ptr: int, sign: int):
    """create_ec_decompress_event (events/precompiles/ec.rs:175-220): x read from ptr + nl at clk, the
    decompressed y written to ptr at clk."""
    fp = FIELDS[curve]
    assert ptr % 4 == 0 and sign <= 1
    xr = [pm.read(ptr + fp.nl + 4 * i, clk) for i in range(fp.words)]
    x = EF.words_to_int([r[0] for r in xr])
    yw = EF.int_to_words(decompress_y(curve, x, sign), fp.words)
    yr = [pm.write(ptr + 4 * i, yw[i], clk) for i in range(fp.words)]
    return {"shard": shard, "clk": clk, "ptr": ptr, "sign": sign, "x": xr, "y": yr, "local": pm.local_entries()}


def weierstrass_decompress_trace(curve: str, events, byte_lookup) -> np.ndarray:
    """WeierstrassDecompressChip::generate_trace (weierstrass_decompress.rs:161-303): padding rows
    decompress the generator's abscissa (value words only in x_access, no choice columns)."""
    from . import mips_alu as A
    fp, lex = FIELDS[curve], LEXICOGRAPHIC[curve]
    L = DecompressLayout(fp, lex)
    ne, h, m, nl = len(events), _height(len(events)), fp.modulus, fp.nl
    t = np.zeros((h, L.WIDTH), np.int64)
    rec = EF.Rec(byte_lookup)
    real = np.zeros(h, bool)
    real[:ne] = True
    xs = [EF.words_to_int([r[0] for r in e["x"]]) for e in events] + [GEN_X[curve]] * (h - ne)
    t[:, L.RANGE_X:L.RANGE_X + fp.lt_w] = EF.pop_field_lt(xs, rec, real, fp)
    x2, t[:, L.X2:L.X2 + fp.fop_w] = EF.pop_field_op(xs, xs, "mul", fp)
    x3, t[:, L.X3:L.X3 + fp.fop_w] = EF.pop_field_op(x2, xs, "mul", fp)
    axb, t[:, L.AXB:L.AXB + fp.fop_w] = EF.pop_inner_product([[CURVE_A[curve]] * h, [CURVE_B[curve]] * h],
                                                             [xs, [1] * h], fp)
    rhs, t[:, L.X3AXB:L.X3AXB + fp.fop_w] = EF.pop_field_op(x3, axb, "add", fp)
    sq = [field_sqrt(curve, v) for v in rhs]
    sq2, cols = EF.pop_field_op(sq, sq, "mul", fp)
    assert sq2 == rhs
    cols[:, :nl] = EF.limbs(sq, nl)  # FieldSqrtCols stores the root in multiplication.result
    t[:, L.SQRT:L.SQRT + fp.fop_w] = cols
    t[:, L.SQRT_RANGE:L.SQRT_RANGE + fp.lt_w] = EF.pop_field_lt(sq, rec, real, fp)
    t[:, L.SQRT_LSB] = EF.limbs(sq, nl)[:, 0] & 1
    negy, t[:, L.NEGY:L.NEGY + fp.fop_w] = EF.pop_field_op([0] * h, sq, "sub", fp)
    # padding rows: the generator's x as the value of the x reads (x_access[i].access.value)
    gx = EF.limbs([GEN_X[curve]], nl)[0]
    for i in range(fp.words):
        t[ne:, L.X + RD_W * i + ACC_VALUE:L.X + RD_W * i + ACC_VALUE + 4] = gx[4 * i:4 * i + 4]
    # byte lookups of the real rows (populate order does not matter to the counts)
    for base in (L.X2, L.X3, L.AXB, L.X3AXB, L.NEGY):
        rec.fop(t[:ne, base:base + fp.fop_w], fp)
    sqc = t[:ne, L.SQRT:L.SQRT + fp.fop_w].copy()
    sqc[:, :nl] = t[:ne, L.X3AXB:L.X3AXB + nl]  # the multiplication's range check covers its result a
    rec.fop(sqc, fp)
    if ne:
        byte_lookup(A.B_AND, t[:ne, L.SQRT], np.ones(ne, np.int64))
    rec.u8(t[:ne, L.SQRT:L.SQRT + nl])
    if ne:
        rows = np.arange(ne)
        t[rows, L.REAL] = 1
        shard = np.array([e["shard"] for e in events], np.int64)
        clk = np.array([e["clk"] for e in events], np.int64)
        t[rows, L.SHARD], t[rows, L.CLK] = shard, clk
        t[rows, L.PTR] = [e["ptr"] for e in events]
        t[rows, L.SIGN] = [e["sign"] for e in events]
        ys = [EF.words_to_int([r[1] for r in e["y"]]) for e in events]
        if lex:
            eq = np.array([(ys[i] & 1) == (sq[i] & 1) for i in range(ne)])
            t[rows, L.IS_Y_EQ] = eq
            sg = np.array([e["sign"] for e in events], bool)
            t[rows, L.WHEN_SQRT_LT] = np.where(sg, ~eq, eq)
            t[rows, L.WHEN_NEG_LT] = np.where(sg, eq, ~eq)
            t[rows, L.NEGY_RANGE:L.NEGY_RANGE + fp.lt_w] = EF.pop_field_lt(
                [negy[i] for i in range(ne)], rec, np.ones(ne, bool), fp)
            for i in range(ne):
                neg = (m - ys[i]) % m
                lhs, rhs_ = (neg, ys[i]) if events[i]["sign"] else (ys[i], neg)
                assert lhs < rhs_
                t[i, L.CMP:L.CMP + fp.lt_w] = EF.pop_field_lt([lhs], rec, np.ones(1, bool), fp, rhs=[rhs_])[0]
        for i, e in enumerate(events):
            assert ys[i] == decompress_y(curve, xs[i], e["sign"])
        _access_block(t, rows, L.X, [e["x"] for e in events], False, shard, clk, byte_lookup)
        _access_block(t, rows, L.Y, [e["y"] for e in events], True, shard, clk, byte_lookup)
    return (t % P).astype(np.uint32)


# ---------------------------------------------------------------- U256x2048Mul
U256XU2048_MUL = 0x01_01_00_2F


class U2048Layout:
    """U256x2048MulCols (u256x2048_mul/air.rs:51-77)."""

    def __init__(self):
        self.SHARD, self.CLK, self.APTR, self.BPTR, self.LOPTR, self.HIPTR = range(6)
        self.LOPTR_MEM = 6                       # MemoryReadCols of register A2
        self.HIPTR_MEM = self.LOPTR_MEM + RD_W   # register A3
        self.A = self.HIPTR_MEM + RD_W           # 8 x MemoryReadCols
        self.B = self.A + 8 * RD_W               # 64 x MemoryReadCols
        self.LO = self.B + 64 * RD_W             # 64 x MemoryWriteCols
        self.HI = self.LO + 64 * WR_W            # 8 x MemoryWriteCols
        self.OUT = [self.HI + 8 * WR_W + k * U256.fop_w for k in range(8)]  # a_mul_b1, ab2_plus_carry, ...
        self.REAL = self.OUT[-1] + U256.fop_w
        self.WIDTH = self.REAL + 1


U2048L = U2048Layout()
_MOD_2_256 = [0] * 32 + [1]


def u256x2048_mul_chip() -> ChipDesc:
    """U256x2048MulChip::eval (u256x2048_mul/air.rs:266-385): (lo, hi) = a * b over 2048 + 256 bits, the
    eight 256-bit limbs of b multiplied in a chain whose carries feed the next."""
    from .mips_core import _eval_memory_access
    from .mips_syscall import REG_A2, REG_A3
    L = U2048L
    ch = ChipDesc("U256XU2048Mul", prep_width=0, main_width=L.WIDTH)
    real, rv = main(L.REAL), _m(L.REAL)
    _assert_bool(ch, real)
    ch.receives.append(Lookup([_m(L.SHARD), _m(L.CLK), V.const(sid(U256XU2048_MUL)), _m(L.APTR), _m(L.BPTR)], rv,
                              KIND_SYSCALL))
    for reg, base in ((REG_A2, L.LOPTR_MEM), (REG_A3, L.HIPTR_MEM)):
        _eval_memory_access(ch, base, base + ACC_VALUE, 0, V.const(reg), real, rv, shard_col=L.SHARD,
                            clk_terms=((L.CLK, 1),))
    _eval_access_slice(ch, L.A, 8, False, L.APTR, 0, real, rv, L.SHARD, L.CLK)
    _eval_access_slice(ch, L.B, 64, False, L.BPTR, 0, real, rv, L.SHARD, L.CLK)
    _eval_access_slice(ch, L.LO, 64, True, L.LOPTR, 1, real, rv, L.SHARD, L.CLK)
    _eval_access_slice(ch, L.HI, 8, True, L.HIPTR, 1, real, rv, L.SHARD, L.CLK)
    a = _read_limbs(L.A, 8)
    prev = [0]
    for k in range(8):
        EF.eval_mul_and_carry(ch, L.OUT[k], a, _read_limbs(L.B + 8 * k * RD_W, 8), prev, _MOD_2_256, rv, U256)
        prev = EF.cols(L.OUT[k] + 32, 32)
    for x, y in zip(prev, _write_value_limbs(L.HI, 8)):
        ch.assert_zero(real * (x - y))
    for k in range(8):
        for x, y in zip(EF.cols(L.OUT[k], 32), _write_value_limbs(L.LO + 8 * k * WR_W, 8)):
            ch.assert_zero(real * (x - y))
    for ptr, base in ((L.LOPTR, L.LOPTR_MEM), (L.HIPTR, L.HIPTR_MEM)):
        word = sum((main(base + ACC_VALUE + j) * (1 << (8 * j)) for j in range(1, 4)), main(base + ACC_VALUE))
        ch.assert_zero(real * (main(ptr) - word))
    return ch


def exec_u256x2048_mul(pm, shard: int, clk: int, a_ptr: int, b_ptr: int):
    """U256xU2048MulSyscall::execute (executor/src/syscalls/precompiles/u256x2048_mul.rs): lo_ptr / hi_ptr
    from registers A2 / A3, a and b read at clk, lo and hi written at clk + 1."""
    from .mips_syscall import REG_A2, REG_A3
    lo_reg, hi_reg = pm.reg_read(REG_A2, clk), pm.reg_read(REG_A3, clk)
    lo_ptr, hi_ptr = lo_reg[0], hi_reg[0]
    ar = [pm.read(a_ptr + 4 * i, clk) for i in range(8)]
    br = [pm.read(b_ptr + 4 * i, clk) for i in range(64)]
    prod = EF.words_to_int([r[0] for r in ar]) * EF.words_to_int([r[0] for r in br])
    lo_w, hi_w = EF.int_to_words(prod % (1 << 2048), 64), EF.int_to_words(prod >> 2048, 8)
    lw = [pm.write(lo_ptr + 4 * i, lo_w[i], clk + 1) for i in range(64)]
    hw = [pm.write(hi_ptr + 4 * i, hi_w[i], clk + 1) for i in range(8)]
    return {"shard": shard, "clk": clk, "a_ptr": a_ptr, "b_ptr": b_ptr, "lo_ptr": lo_ptr, "hi_ptr": hi_ptr,
            "lo_reg": lo_reg, "hi_reg": hi_reg, "a": ar, "b": br, "lo": lw, "hi": hw, "local": pm.local_entries()}


def u256x2048_mul_trace(events, byte_lookup) -> np.ndarray:
    """U256x2048MulChip::generate_trace (u256x2048_mul/air.rs:109-213): padding rows hold the eight
    mul-and-carry operations of zeros."""
    L = U2048L
    ne, h = len(events), _height(len(events))
    t = np.zeros((h, L.WIDTH), np.int64)
    rec = EF.Rec(byte_lookup)
    a = [EF.words_to_int([r[0] for r in e["a"]]) for e in events] + [0] * (h - ne)
    bs = [[EF.words_to_int([r[0] for r in e["b"][8 * k:8 * k + 8]]) for e in events] + [0] * (h - ne)
          for k in range(8)]
    carry = [0] * h
    for k in range(8):
        res, carry, c = EF.pop_mul_and_carry(a, bs[k], carry, 1 << 256, U256)
        t[:, L.OUT[k]:L.OUT[k] + U256.fop_w] = c
        rec.fop(t[:ne, L.OUT[k]:L.OUT[k] + U256.fop_w], U256)
    if ne:
        rows = np.arange(ne)
        t[rows, L.REAL] = 1
        shard = np.array([e["shard"] for e in events], np.int64)
        clk = np.array([e["clk"] for e in events], np.int64)
        t[rows, L.SHARD], t[rows, L.CLK] = shard, clk
        for col, key in ((L.APTR, "a_ptr"), (L.BPTR, "b_ptr"), (L.LOPTR, "lo_ptr"), (L.HIPTR, "hi_ptr")):
            t[rows, col] = [e[key] for e in events]
        for i, e in enumerate(events):
            assert EF.words_to_int([r[1] for r in e["hi"]]) == carry[i]
        _access_block(t, rows, L.LOPTR_MEM, [[e["lo_reg"]] for e in events], False, shard, clk, byte_lookup)
        _access_block(t, rows, L.HIPTR_MEM, [[e["hi_reg"]] for e in events], False, shard, clk, byte_lookup)
        _access_block(t, rows, L.A, [e["a"] for e in events], False, shard, clk, byte_lookup)
        _access_block(t, rows, L.B, [e["b"] for e in events], False, shard, clk, byte_lookup)
        _access_block(t, rows, L.LO, [e["lo"] for e in events], True, shard, clk + 1, byte_lookup)
        _access_block(t, rows, L.HI, [e["hi"] for e in events], True, shard, clk + 1, byte_lookup)
    return (t % P).astype(np.uint32)
