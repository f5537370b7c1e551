"""Emulated (non-native) field arithmetic gadgets shared by the precompile chips: the reference's
crates/core/machine/src/operations/field/ over any FieldParameters (crates/curves/src/params.rs):

* FieldOpCols (field_op.rs: result, carry, witness_low, witness_high; eval_with_modulus /
  eval_with_polynomials :304-357, populate_with_modulus :193-266), FieldInnerProductCols
  (field_inner_product.rs), FieldDenCols (field_den.rs), FieldLtCols (range.rs);
* eval_field_operation (util_air.rs): with w(x) = witness_low(x) + 2^8 witness_high(x) - OFFSET, every
  coefficient of vanishing(x) - w(x) (x - 2^8) is zero;
* compute_root_quotient_and_shift / split (util.rs) on the trace side.

A field element is `nl` byte limbs (NB_BITS_PER_LIMB = 8); the witness has `nwit` limbs.  Both the AIR
side (constraints over Expr polynomials) and the trace side (numpy over a batch of rows) take the
parameters explicitly, so one implementation serves Ed25519, the Weierstrass curves' base fields
(secp256k1, secp256r1, bn254, bls12-381), the fp towers and Uint256MulMod's variable modulus.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Sequence

import numpy as np

from . import mips_alu as A
from .machine import ChipDesc, Expr, KIND_BYTE, Lookup, P, main
from .machine import VirtualPairCol as V
from .mips_alu import ZERO, _assert_bool, _m


@dataclass(frozen=True)
class FieldParams:
    """FieldParameters + NumLimbs of a base field (crates/curves/src/params.rs)."""
    name: str
    modulus: int
    nl: int          # Limbs (bytes per element)
    nwit: int        # Witness limbs
    offset: int      # WITNESS_OFFSET

    @property
    def mod_limbs(self) -> List[int]:
        return list(self.modulus.to_bytes(self.nl, "little"))

    @property
    def fop_w(self) -> int:
        """FieldOpCols / FieldInnerProductCols / FieldDenCols width: result, carry, witness low / high."""
        return 2 * self.nl + 2 * self.nwit

    @property
    def lt_w(self) -> int:
        """FieldLtCols: byte_flags[nl], lhs_comparison_byte, rhs_comparison_byte."""
        return self.nl + 2

    @property
    def words(self) -> int:
        return self.nl // 4


# ---------------------------------------------------------------- polynomials over limbs (AIR side)
# A polynomial is a list of coefficients, each an int (a constant) or an Expr.
def _add(a, b):
    if isinstance(a, int) and isinstance(b, int):
        return (a + b) % P
    if isinstance(a, int) and a % P == 0:
        return b
    if isinstance(b, int) and b % P == 0:
        return a
    return a + b


def _mulc(a, b):
    if isinstance(a, int) and isinstance(b, int):
        return a * b % P
    if isinstance(a, int):
        a, b = b, a
    if isinstance(b, int):
        if b % P == 0:
            return 0
        if b % P == 1:
            return a
    return a * b


def p_add(a: Sequence, b: Sequence) -> List:
    return [_add(a[i] if i < len(a) else 0, b[i] if i < len(b) else 0) for i in range(max(len(a), len(b)))]


def p_neg(a: Sequence) -> List:
    return [(-x) % P if isinstance(x, int) else -x for x in a]


def p_sub(a: Sequence, b: Sequence) -> List:
    return p_add(a, p_neg(b))


def p_mul(a: Sequence, b: Sequence) -> List:
    """Polynomial::mul (zkm_stark air/polynomial.rs): coefficient k = sum_{i + j = k} a_i b_j."""
    out = [0] * (len(a) + len(b) - 1)
    for i, x in enumerate(a):
        for j, y in enumerate(b):
            out[i + j] = _add(out[i + j], _mulc(x, y))
    return out


def p_scale(a: Sequence, s) -> List:
    return [_mulc(x, s) for x in a]


def const_limbs(x: int, fp: FieldParams) -> List[int]:
    """FieldParameters::to_limbs_field of a constant."""
    return list(int(x).to_bytes(fp.nl, "little"))


def cols(base: int, n: int) -> List[Expr]:
    return [main(base + i) for i in range(n)]


def vcols(base: int, n: int) -> List[V]:
    return [_m(base + i) for i in range(n)]


def u8_range(ch: ChipDesc, cs: Sequence[V], mult: V):
    """slice_range_check_u8 (air/word.rs:55-80): U8Range byte lookups on pairs (a trailing single with 0)."""
    for k in range(0, len(cs) - 1, 2):
        ch.sends.append(Lookup([V.const(A.B_U8RANGE), ZERO, ZERO, cs[k], cs[k + 1]], mult, KIND_BYTE))
    if len(cs) % 2:
        ch.sends.append(Lookup([V.const(A.B_U8RANGE), ZERO, ZERO, cs[-1], ZERO], mult, KIND_BYTE))


def eval_field_operation(ch: ChipDesc, vanishing: Sequence, base: int, fp: FieldParams):
    """util_air.rs eval_field_operation (nwit + 1 constraints)."""
    wlo, whi = base + 2 * fp.nl, base + 2 * fp.nl + fp.nwit
    w = [main(wlo + j) + main(whi + j) * 256 - fp.offset for j in range(fp.nwit)]
    # w(x) * (x - 256): coefficient k = w_{k-1} - 256 w_k
    prod = [0] * (fp.nwit + 1)
    for j in range(fp.nwit):
        prod[j] = _add(prod[j], w[j] * (P - 256))
        prod[j + 1] = _add(prod[j + 1], w[j])
    for c in p_sub(vanishing, prod):
        ch.assert_zero(Expr.lift(c))


def field_range_checks(ch: ChipDesc, base: int, mult: V, fp: FieldParams, result_cols: Sequence[V] = None):
    """The four slice_range_check_u8 of an emulated-field operation (result, carry, witness low/high)."""
    u8_range(ch, vcols(base, fp.nl) if result_cols is None else result_cols, mult)
    u8_range(ch, vcols(base + fp.nl, fp.nl), mult)
    u8_range(ch, vcols(base + 2 * fp.nl, fp.nwit), mult)
    u8_range(ch, vcols(base + 2 * fp.nl + fp.nwit, fp.nwit), mult)


def eval_field_op(ch: ChipDesc, base: int, a, b, op: str, mult: V, fp: FieldParams, result=None, result_cols=None,
                  modulus=None):
    """FieldOpCols::eval / eval_with_modulus (field_op.rs:304-373).  `result` overrides the result
    polynomial (FieldSqrtCols passes the input there); `modulus` a modulus polynomial (Uint256MulMod)."""
    res = cols(base, fp.nl) if result is None else result
    carry = cols(base + fp.nl, fp.nl)
    if op in ("add", "mul"):
        pa, pres = a, res
    else:  # sub / div: a = result op b
        pa, pres = res, a
    pop = p_add(pa, b) if op in ("add", "sub") else p_mul(pa, b)
    vanishing = p_sub(p_sub(pop, pres), p_mul(carry, fp.mod_limbs if modulus is None else modulus))
    eval_field_operation(ch, vanishing, base, fp)
    field_range_checks(ch, base, mult, fp, result_cols)


def eval_inner_product(ch: ChipDesc, base: int, a_vec, b_vec, mult: V, fp: FieldParams):
    """FieldInnerProductCols::eval (field_inner_product.rs:121-170)."""
    acc = [0]
    for pa, pb in zip(a_vec, b_vec):
        acc = p_add(acc, p_mul(pa, pb))
    vanishing = p_sub(p_sub(acc, cols(base, fp.nl)), p_mul(cols(base + fp.nl, fp.nl), fp.mod_limbs))
    eval_field_operation(ch, vanishing, base, fp)
    field_range_checks(ch, base, mult, fp)


def eval_den(ch: ChipDesc, base: int, a, b, sign: bool, mult: V, fp: FieldParams):
    """FieldDenCols::eval (field_den.rs:124-175): a / (1 + b) if sign else a / (1 - b)."""
    res, carry = cols(base, fp.nl), cols(base + fp.nl, fp.nl)
    br = p_mul(b, res)
    lhs = p_add(br, res) if sign else p_add(br, a)
    rhs = a if sign else res
    vanishing = p_sub(p_sub(lhs, rhs), p_mul(carry, fp.mod_limbs))
    eval_field_operation(ch, vanishing, base, fp)
    field_range_checks(ch, base, mult, fp)


def eval_field_lt(ch: ChipDesc, base: int, lhs: Sequence, rhs: Sequence, is_real: Expr, mult: V, fp: FieldParams):
    """FieldLtCols::eval (range.rs:62-141): exactly one byte flag, bytes equal above it, and the LTU byte
    lookup on the flagged pair."""
    flags = cols(base, fp.nl)
    total = Expr.lift(0)
    for f in flags:
        _assert_bool(ch, f, is_real)
        total = total + f
    ch.assert_zero(is_real * (total - 1))
    visited = Expr.lift(0)
    lcmp, rcmp = Expr.lift(0), Expr.lift(0)
    for lb, rb, f in zip(reversed(lhs), reversed(rhs), reversed(flags)):
        visited = visited + f
        lcmp = lcmp + Expr.lift(lb) * f
        rcmp = rcmp + f * Expr.lift(rb)
        ch.assert_zero(is_real * (1 - visited) * (Expr.lift(lb) - Expr.lift(rb)))
    ch.assert_zero(is_real * (main(base + fp.nl) - lcmp))
    ch.assert_zero(is_real * (main(base + fp.nl + 1) - rcmp))
    ch.sends.append(Lookup([V.const(A.B_LTU), V.const(1), ZERO, _m(base + fp.nl), _m(base + fp.nl + 1)], mult,
                           KIND_BYTE))


# ---------------------------------------------------------------- trace side (numpy over a batch)
def limbs(xs: Sequence[int], n: int) -> np.ndarray:
    return np.array([list(int(x).to_bytes(n, "little")) for x in xs], np.int64).reshape(len(xs), n)


def pmul_np(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    out = np.zeros((a.shape[0], a.shape[1] + b.shape[1] - 1), np.int64)
    for i in range(a.shape[1]):
        out[:, i:i + b.shape[1]] += a[:, i:i + 1] * b
    return out


def padd_np(*ps) -> np.ndarray:
    n = max(p.shape[1] for p in ps)
    out = np.zeros((ps[0].shape[0], n), np.int64)
    for p in ps:
        out[:, :p.shape[1]] += p
    return out


def witness(vanishing: np.ndarray, fp: FieldParams) -> np.ndarray:
    """compute_root_quotient_and_shift + split (util.rs:20-72): w(x) = vanishing(x) / (x - 256), shifted by
    the offset; returns (n, 2 nwit): the low bytes then the high bytes."""
    v = vanishing
    nw = fp.nwit
    # trailing zero coefficients beyond the witness length carry nothing
    assert v.shape[1] <= nw + 1 or not np.any(v[:, nw + 1:]), "vanishing polynomial longer than the witness"
    v = v[:, :nw + 1] if v.shape[1] > nw + 1 else np.pad(v, ((0, 0), (0, nw + 1 - v.shape[1])))
    q = np.zeros((v.shape[0], nw), np.int64)
    q[:, nw - 1] = v[:, nw]
    for k in range(nw - 1, 0, -1):
        q[:, k - 1] = v[:, k] + 256 * q[:, k]
    assert np.all(v[:, 0] == -256 * q[:, 0]), "the vanishing polynomial has no root at 2^8"
    q = q + fp.offset
    assert np.all((q >= 0) & (q < (1 << 16)))
    return np.concatenate([q & 0xFF, q >> 8], axis=1)


class Rec:
    """Byte lookups of one trace, recorded through `byte_lookup(opcode, b, c)` (added to the Byte chip's
    multiplicities only for the rows passed)."""

    def __init__(self, byte_lookup):
        self.bl = byte_lookup

    def u8(self, x: np.ndarray):
        """add_u8_range_checks_field on the columns x (n, k): pairs (and a trailing single with 0)."""
        k = x.shape[1]
        for j in range(0, k - 1, 2):
            self.bl(A.B_U8RANGE, x[:, j], x[:, j + 1])
        if k % 2:
            self.bl(A.B_U8RANGE, x[:, k - 1], np.zeros(len(x), np.int64))

    def fop(self, x: np.ndarray, fp: FieldParams):
        """The four add_u8_range_checks_field of a FieldOpCols block (result, carry, witness low, witness
        high), each paired on its own (they differ from one slice when nwit is odd)."""
        nl, nw = fp.nl, fp.nwit
        for a, b in ((0, nl), (nl, 2 * nl), (2 * nl, 2 * nl + nw), (2 * nl + nw, 2 * nl + 2 * nw)):
            self.u8(x[:, a:b])


def fop_cols(res: np.ndarray, carry: np.ndarray, vanishing: np.ndarray, fp: FieldParams) -> np.ndarray:
    return np.concatenate([res, carry, witness(vanishing, fp)], axis=1)


def pop_field_op(a: Sequence[int], b: Sequence[int], op: str, fp: FieldParams, modulus: Sequence[int] = None):
    """FieldOpCols::populate_with_modulus (field_op.rs:193-266) over a batch: returns (result ints,
    (n, fop_w) columns).  sub / div populate as (result + b) / (result * b).  `modulus` gives a modulus
    per row (Uint256MulMod; it may be 2^256, whose limb polynomial has nl + 1 coefficients)."""
    mods = [fp.modulus] * len(a) if modulus is None else list(modulus)
    if op == "sub":
        r = [(m + x - y) % m for x, y, m in zip(a, b, mods)]
        lhs, rhs, mode = r, b, "add"
    elif op == "div":
        assert all(y or not x for x, y in zip(a, b)), "division by zero is allowed only when dividing zero"
        r = [x * pow(y, -1, m) % m if y else 0 for x, y, m in zip(a, b, mods)]
        lhs, rhs, mode = r, b, "mul"
    else:
        lhs, rhs, mode = a, b, op
        r = [((x + y) if op == "add" else (x * y)) % m for x, y, m in zip(a, b, mods)]
    full = [(x + y) if mode == "add" else (x * y) for x, y in zip(lhs, rhs)]
    mres = [f % m for f, m in zip(full, mods)]
    carry = [(f - mr) // m for f, mr, m in zip(full, mres, mods)]
    la, lb = limbs(lhs, fp.nl), limbs(rhs, fp.nl)
    pop = (la + lb) if mode == "add" else pmul_np(la, lb)
    ml = limbs(mods, fp.nl + 1)  # 2^256 needs the extra coefficient
    van = padd_np(pop, -limbs(mres, fp.nl), -pmul_np(limbs(carry, fp.nl), ml))
    return r, fop_cols(limbs(r, fp.nl), limbs(carry, fp.nl), van, fp)


def pop_inner_product(a_vec, b_vec, fp: FieldParams):
    """FieldInnerProductCols::populate (field_inner_product.rs:33-94)."""
    n = len(a_vec[0])
    ip = [sum(a[i] * b[i] for a, b in zip(a_vec, b_vec)) for i in range(n)]
    r = [x % fp.modulus for x in ip]
    carry = [(x - y) // fp.modulus for x, y in zip(ip, r)]
    acc = padd_np(*[pmul_np(limbs(a, fp.nl), limbs(b, fp.nl)) for a, b in zip(a_vec, b_vec)])
    van = padd_np(acc, -limbs(r, fp.nl), -pmul_np(limbs(carry, fp.nl), np.array(fp.mod_limbs, np.int64)[None, :]))
    return r, fop_cols(limbs(r, fp.nl), limbs(carry, fp.nl), van, fp)


def pop_den(a: Sequence[int], b: Sequence[int], sign: bool, fp: FieldParams):
    """FieldDenCols::populate (field_den.rs:33-94)."""
    p = fp.modulus
    r, carry = [], []
    for x, y in zip(a, b):
        den = ((y if sign else p - y) + 1) % p
        res = x * pow(den, -1, p) % p
        lhs = y * res + res if sign else y * res + x
        rhs = x if sign else res
        r.append(res)
        carry.append((lhs - rhs) // p)
    lr, lb, la = limbs(r, fp.nl), limbs(b, fp.nl), limbs(a, fp.nl)
    br = pmul_np(lb, lr)
    lhs = padd_np(br, lr) if sign else padd_np(br, la)
    rhs = la if sign else lr
    van = padd_np(lhs, -rhs, -pmul_np(limbs(carry, fp.nl), np.array(fp.mod_limbs, np.int64)[None, :]))
    return r, fop_cols(lr, limbs(carry, fp.nl), van, fp)


def pop_field_lt(lhs: Sequence[int], rec: Rec, real: np.ndarray, fp: FieldParams,
                 rhs: Sequence[int] = None, fill: np.ndarray = None) -> np.ndarray:
    """FieldLtCols::populate (range.rs:27-58): rhs = the modulus unless given per row; rows in `fill`
    (default: all, padding rows included) are populated, the LTU lookup is recorded for the rows in `real`."""
    L = limbs(lhs, fp.nl)
    R = np.array([fp.mod_limbs] * len(lhs), np.int64) if rhs is None else limbs(rhs, fp.nl)
    out = np.zeros((len(lhs), fp.lt_w), np.int64)
    for i in range(len(lhs)):
        if fill is not None and not fill[i]:
            continue
        for k in range(fp.nl - 1, -1, -1):
            if L[i, k] < R[i, k]:
                out[i, k] = 1
                out[i, fp.nl], out[i, fp.nl + 1] = L[i, k], R[i, k]
                break
            assert L[i, k] == R[i, k], "FieldLtCols: lhs is not below rhs"
    if real.any():
        rec.bl(A.B_LTU, out[real, fp.nl], out[real, fp.nl + 1])
    return out


def words_to_int(ws) -> int:
    return int.from_bytes(b"".join(int(w).to_bytes(4, "little") for w in ws), "little")


def int_to_words(x: int, n_words: int) -> List[int]:
    b = int(x).to_bytes(4 * n_words, "little")
    return [int.from_bytes(b[4 * i:4 * i + 4], "little") for i in range(n_words)]


def eval_mul_and_carry(ch: ChipDesc, base: int, a, b, c, modulus, mult: V, fp: FieldParams):
    """FieldOpCols::eval_mul_and_carry (field_op.rs:281-303): a b + c = result + carry modulus."""
    res, carry = cols(base, fp.nl), cols(base + fp.nl, fp.nl)
    vanishing = p_sub(p_sub(p_add(p_mul(a, b), c), res), p_mul(carry, modulus))
    eval_field_operation(ch, vanishing, base, fp)
    field_range_checks(ch, base, mult, fp)


def pop_mul_and_carry(a: Sequence[int], b: Sequence[int], c: Sequence[int], modulus: int, fp: FieldParams):
    """FieldOpCols::populate_mul_and_carry (field_op.rs:47-101) over a batch: returns (result, carry,
    (n, fop_w) columns)."""
    full = [x * y + z for x, y, z in zip(a, b, c)]
    res = [f % modulus for f in full]
    carry = [f // modulus for f in full]
    mlimbs = np.array(list(modulus.to_bytes((modulus.bit_length() + 7) // 8, "little")), np.int64)[None, :]
    van = padd_np(pmul_np(limbs(a, fp.nl), limbs(b, fp.nl)), limbs(c, fp.nl), -limbs(res, fp.nl),
                  -pmul_np(limbs(carry, fp.nl), mlimbs))
    return res, carry, fop_cols(limbs(res, fp.nl), limbs(carry, fp.nl), van, fp)
