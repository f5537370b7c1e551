"""The memory argument's shard-level chips restated from the reference AIRs:

* ``MemoryLocal`` crates/core/machine/src/memory/local.rs:26-271 — four entries per row, each receiving
  the address's value at the shard's start and sending it at the shard's end (Memory lookups, local),
  and sending both as Global-kind lookups to the Global chip.
* ``Global``      crates/core/machine/src/global/mod.rs:53-273 with GlobalLookupOperation
  (operations/global_lookup.rs:14-155) and GlobalAccumulationOperation (operations/global_accumulation.rs:
  18-224) — every global message lifted to a point of the septic curve y^2 = x^3 + 3z x - 3 over
  F_p[z]/(z^7 + 2z - 8) (crates/stark/src/septic_curve.rs) and accumulated from the zero digest; the last
  row's cumulative sum (the chip's last 14 columns) is the shard's global cumulative sum
  (commit scope Global, prover.rs:352-361).

Constraint and lookup order follow each `eval` (that order fixes the alpha-power folding and the LogUp
columns).  The septic-curve arithmetic of the trace (square roots, additions) runs in the host C++
helper zkmips_amd/csrc/host/septic.cpp.
"""
from __future__ import annotations

import numpy as np

from . import mips_alu as A
from . import septic as S
from .machine import (ChipDesc, Expr, IS_FIRST, IS_TRANSITION, KIND_BYTE, KIND_GLOBAL, KIND_MEMORY, Lookup, P,
                      VirtualPairCol as V, main, main_next)

_m = A._m
ZERO = A.ZERO
_assert_bool = A._assert_bool

# ---------------------------------------------------------------- septic arithmetic over Expr
# An element of F_p[z]/(z^7 + 2z - 8) is a list of 7 coefficients, each an int (constant) or an Expr.


def _is_zero(t) -> bool:
    return isinstance(t, int) and t % P == 0


def _add(a, b):
    if _is_zero(a):
        return b
    if _is_zero(b):
        return a
    if isinstance(a, int) and isinstance(b, int):
        return (a + b) % P
    return a + b


def _mul(a, b):
    if _is_zero(a) or _is_zero(b):
        return 0
    if isinstance(a, int) and isinstance(b, int):
        return a * b % P
    if isinstance(a, int) and a % P == 1:
        return b
    if isinstance(b, int) and b % P == 1:
        return a
    return a * b


def _neg(a):
    return (-a) % P if isinstance(a, int) else -a


def s_add(a, b):
    return [_add(x, y) for x, y in zip(a, b)]


def s_sub(a, b):
    return [_add(x, _neg(y)) for x, y in zip(a, b)]


def _shared(t):
    return t.share() if isinstance(t, Expr) else t


def s_mul(a, b):
    """SepticExtension::mul (septic_extension.rs:300-316): schoolbook, then z^7 = 8 - 2z.  Operands and
    results are shared nodes (the reference clones Rc'd symbolic expressions into the 49 products, so
    its DAG holds each coefficient once)."""
    a = [_shared(x) for x in a]
    b = a if b is a else [_shared(x) for x in b]
    res = [0] * 13
    for i in range(7):
        for j in range(7):
            res[i + j] = _add(res[i + j], _mul(a[i], b[j]))
    ret = res[:7]
    for i in range(7, 13):
        ret[i - 7] = _add(ret[i - 7], _mul(8, res[i]))
        ret[i - 6] = _add(ret[i - 6], _mul(P - 2, res[i]))
    return [_shared(x) for x in ret]


def s_square(a):
    a = [_shared(x) for x in a]
    return s_mul(a, a)


def curve_formula(x):
    """SepticCurve::curve_formula (septic_curve.rs:101-122): x^3 + 3z x - 3."""
    return s_sub(s_add(s_mul(s_square(x), x), s_mul(x, [0, 3, 0, 0, 0, 0, 0])), [3, 0, 0, 0, 0, 0, 0])


def sum_checker_x(p1, p2, p3):
    """(x1 + x2 + x3)(x2 - x1)^2 - (y2 - y1)^2 (septic_curve.rs:159-166)."""
    (x1, y1), (x2, y2), (x3, _) = p1, p2, p3
    return s_sub(s_mul(s_add(s_add(x1, x2), x3), s_square(s_sub(x2, x1))), s_square(s_sub(y2, y1)))


def sum_checker_y(p1, p2, p3):
    """(y1 + y3)(x2 - x1) - (y2 - y1)(x1 - x3) (septic_curve.rs:169-176)."""
    (x1, y1), (x2, y2), (x3, y3) = p1, p2, p3
    return s_sub(s_mul(s_add(y1, y3), s_sub(x2, x1)), s_mul(s_sub(y2, y1), s_sub(x1, x3)))


def _assert_septic_eq(ch, a, b, when=None):
    for x, y in zip(a, b):
        e = Expr.lift(_add(x, _neg(y)))
        ch.assert_zero(e if when is None else when * e)


def _cols(base, n=7):
    return [main(base + i) for i in range(n)]


def _next_cols(base, n=7):
    return [main_next(base + i) for i in range(n)]


# ---------------------------------------------------------------- MemoryLocal (memory/local.rs)
ML_ENTRIES = 4  # NUM_LOCAL_MEMORY_ENTRIES_PER_ROW
# SingleMemoryLocal: addr, initial_shard, final_shard, initial_clk, final_clk, initial_value[4], final_value[4], is_real
ML_ADDR, ML_ISHARD, ML_FSHARD, ML_ICLK, ML_FCLK, ML_IVAL, ML_FVAL, ML_REAL = 0, 1, 2, 3, 4, 5, 9, 13
ML_ENTRY_WIDTH = 14
ML_WIDTH = ML_ENTRIES * ML_ENTRY_WIDTH  # 56


def memory_local_chip() -> ChipDesc:
    """MemoryLocalChip::eval (memory/local.rs:204-270)."""
    ch = ChipDesc("MemoryLocal", prep_width=0, main_width=ML_WIDTH)
    for k in range(ML_ENTRIES):
        b = k * ML_ENTRY_WIDTH
        real = _m(b + ML_REAL)
        _assert_bool(ch, main(b + ML_REAL))
        ch.receives.append(Lookup([_m(b + ML_ISHARD), _m(b + ML_ICLK), _m(b + ML_ADDR)] +
                                  [_m(b + ML_IVAL + i) for i in range(4)], real, KIND_MEMORY))
        ch.sends.append(Lookup([_m(b + ML_ISHARD), _m(b + ML_ICLK), _m(b + ML_ADDR)] +
                               [_m(b + ML_IVAL + i) for i in range(4)] + [ZERO, real, V.const(KIND_MEMORY)],
                               real, KIND_GLOBAL))
        ch.sends.append(Lookup([_m(b + ML_FSHARD), _m(b + ML_FCLK), _m(b + ML_ADDR)] +
                               [_m(b + ML_FVAL + i) for i in range(4)] + [real, ZERO, V.const(KIND_MEMORY)],
                               real, KIND_GLOBAL))
        ch.sends.append(Lookup([_m(b + ML_FSHARD), _m(b + ML_FCLK), _m(b + ML_ADDR)] +
                               [_m(b + ML_FVAL + i) for i in range(4)], real, KIND_MEMORY))
    return ch


def memory_local_trace(entries: np.ndarray) -> np.ndarray:
    """MemoryLocalChip::generate_trace (memory/local.rs:144-185).  entries: n x 11 =
    (addr, initial shard, initial clk, initial value, final shard, final clk, final value)."""
    e = np.asarray(entries, np.int64).reshape(-1, 7)
    n = len(e)
    rows = (n + ML_ENTRIES - 1) // ML_ENTRIES
    t = np.zeros((A._pow2(rows) * ML_ENTRIES, ML_ENTRY_WIDTH), np.uint32)
    t[:n, ML_ADDR] = e[:, 0]
    t[:n, ML_ISHARD], t[:n, ML_ICLK] = e[:, 1], e[:, 2]
    t[:n, ML_IVAL:ML_IVAL + 4] = A._bytes(e[:, 3].astype(np.uint32))
    t[:n, ML_FSHARD], t[:n, ML_FCLK] = e[:, 4], e[:, 5]
    t[:n, ML_FVAL:ML_FVAL + 4] = A._bytes(e[:, 6].astype(np.uint32))
    t[:n, ML_REAL] = 1
    return t.reshape(-1, ML_WIDTH)


def local_entries(trace: np.ndarray) -> np.ndarray:
    """The real entries of a MemoryLocal trace as rows (addr, initial shard, initial clk, initial value,
    final shard, final clk, final value) -- the inverse of memory_local_trace."""
    t = np.asarray(trace).reshape(-1, ML_ENTRY_WIDTH).astype(np.int64)
    t = t[t[:, ML_REAL] == 1]
    word = lambda b: t[:, b] | (t[:, b + 1] << 8) | (t[:, b + 2] << 16) | (t[:, b + 3] << 24)
    return np.stack([t[:, ML_ADDR], t[:, ML_ISHARD], t[:, ML_ICLK], word(ML_IVAL), t[:, ML_FSHARD], t[:, ML_FCLK],
                     word(ML_FVAL)], axis=1)


def memory_local_global_events(entries: np.ndarray):
    """MemoryLocalChip::generate_dependencies (memory/local.rs:97-135): per entry, the initial access as
    a global receive, then the final access as a global send.  Returns (messages n x 7, is_receive)."""
    e = np.asarray(entries, np.int64).reshape(-1, 7)
    msg = np.zeros((2 * len(e), 7), np.uint32)
    iv, fv = A._bytes(e[:, 3].astype(np.uint32)), A._bytes(e[:, 6].astype(np.uint32))
    msg[0::2, 0], msg[0::2, 1], msg[0::2, 2], msg[0::2, 3:7] = e[:, 1], e[:, 2], e[:, 0], iv
    msg[1::2, 0], msg[1::2, 1], msg[1::2, 2], msg[1::2, 3:7] = e[:, 4], e[:, 5], e[:, 0], fv
    rec = np.zeros(2 * len(e), np.uint8)
    rec[0::2] = 1
    return msg, rec


# ---------------------------------------------------------------- Global (global/mod.rs)
G_MSG, G_KIND = 0, 7
G_OFFSET, G_X, G_Y, G_Y6BITS, G_RCW = 8, 16, 23, 30, 60  # GlobalLookupOperation
G_IS_RECEIVE, G_IS_SEND, G_REAL = 61, 62, 63
G_INIT_X, G_INIT_Y, G_SUMCHK, G_CUM_X, G_CUM_Y = 64, 71, 78, 85, 92  # GlobalAccumulationOperation<_, 1>
G_WIDTH = 99
HALF_P_PLUS = (1 << 30) - (1 << 23) + 1  # (p + 1) / 2


def global_chip() -> ChipDesc:
    """GlobalChip::eval (global/mod.rs:213-273): the Global-kind receive, eval_single_digest
    (global_lookup.rs:92-154) and eval_accumulation (global_accumulation.rs:113-223), N = 1."""
    ch = ChipDesc("Global", prep_width=0, main_width=G_WIDTH, commit_scope=1)
    M = main
    real, is_recv, is_send = M(G_REAL), M(G_IS_RECEIVE), M(G_IS_SEND)
    ch.receives.append(Lookup([_m(G_MSG + i) for i in range(7)] + [_m(G_IS_SEND), _m(G_IS_RECEIVE), _m(G_KIND)],
                              _m(G_REAL), KIND_GLOBAL))
    # eval_single_digest
    _assert_bool(ch, real)
    for i in range(8):
        _assert_bool(ch, M(G_OFFSET + i))
    ch.sends.append(Lookup([V.const(A.B_U16RANGE), _m(G_MSG), ZERO, ZERO, ZERO], _m(G_REAL), KIND_BYTE))
    x, y = _cols(G_X), _cols(G_Y)
    _assert_septic_eq(ch, s_square(y), curve_formula(x))
    y6_value = Expr.lift(0)
    top7 = Expr.lift(0)
    for i in range(30):
        b = M(G_Y6BITS + i)
        _assert_bool(ch, b)
        y6_value = y6_value + b * (1 << i)
        if i >= 23:
            top7 = top7 + b
    ch.assert_zero(real * (M(G_RCW) * (top7 - 7) - 1))
    ch.assert_zero(is_recv * (y[6] - (1 + y6_value)))
    ch.assert_zero(is_send * (y[6] - (HALF_P_PLUS + y6_value)))
    # eval_accumulation
    _assert_bool(ch, real)
    ch.assert_zero(IS_TRANSITION * (1 - real) * main_next(G_REAL))
    init = (_cols(G_INIT_X), _cols(G_INIT_Y))
    zero = S.CURVE_CUMULATIVE_SUM_START.astype(int).tolist()
    _assert_septic_eq(ch, init[0], zero[:7], IS_FIRST)
    _assert_septic_eq(ch, init[1], zero[7:], IS_FIRST)
    point = (x, y)
    nxt = (_cols(G_CUM_X), _cols(G_CUM_Y))
    witnessed = _cols(G_SUMCHK)
    _assert_septic_eq(ch, sum_checker_x(init, point, nxt), witnessed)
    _assert_septic_eq(ch, witnessed, [0] * 7, real)
    _assert_septic_eq(ch, sum_checker_y(init, point, nxt), [0] * 7, real)
    _assert_septic_eq(ch, init[0], nxt[0], 1 - real)
    _assert_septic_eq(ch, init[1], nxt[1], 1 - real)
    _assert_septic_eq(ch, nxt[0], _next_cols(G_INIT_X), IS_TRANSITION)
    _assert_septic_eq(ch, nxt[1], _next_cols(G_INIT_Y), IS_TRANSITION)
    return ch


def _inv(x: int) -> int:
    return pow(int(x) % P, P - 2, P)


def global_trace(messages: np.ndarray, is_receive: np.ndarray, kinds: np.ndarray, byte_lookup):
    """GlobalChip::generate_dependencies + generate_trace (global/mod.rs:77-196): one row per global
    message, its curve point, the running sum from the zero digest; padding rows repeat the final
    digest with the dummy point.  Returns (trace, final digest 14 words)."""
    msg = np.asarray(messages, np.uint32).reshape(-1, 7)
    rec = np.asarray(is_receive, np.uint8)
    kinds = np.asarray(kinds, np.uint32)
    n = len(msg)
    t = np.zeros((A._pow2(n), G_WIDTH), np.uint32)
    byte_lookup(A.B_U16RANGE, msg[:, 0].astype(np.int64) >> 8, msg[:, 0].astype(np.int64) & 0xFF)
    pts, off = S.lift(msg, kinds, rec)
    sums = S.cumsum(pts)
    assert not sums[:, 14].any(), "the running global sum hit the point at infinity"
    final = sums[-1, :14] if n else S.CURVE_WITNESS_DUMMY_POINT
    dummy = S.CURVE_WITNESS_DUMMY_POINT
    final_chk = S.sum_checker_x(final, dummy, final)
    if n:
        t[:n, G_MSG:G_MSG + 7] = msg
        t[:n, G_KIND] = kinds
        t[:n, G_OFFSET:G_OFFSET + 8] = (off[:, None] >> np.arange(8, dtype=np.uint32)) & 1
        t[:n, G_X:G_X + 7], t[:n, G_Y:G_Y + 7] = pts[:, :7], pts[:, 7:]
        y6 = pts[:, 13].astype(np.int64)
        rcv = np.where(rec == 1, y6 - 1, y6 - (P + 1) // 2)
        bits = (rcv[:, None] >> np.arange(30, dtype=np.int64)) & 1
        t[:n, G_Y6BITS:G_Y6BITS + 30] = bits
        top = bits[:, 23:].sum(axis=1)
        t[:n, G_RCW] = A.inv_mod_p((top - 7) % P)
        t[:n, G_REAL] = 1
        t[:n, G_IS_RECEIVE] = rec
        t[:n, G_IS_SEND] = 1 - rec
        t[:n, G_INIT_X:G_INIT_X + 14] = sums[:n, :14]
        t[:n, G_CUM_X:G_CUM_X + 14] = sums[1:, :14]
    if len(t) > n:
        t[n:, G_X:G_X + 7], t[n:, G_Y:G_Y + 7] = dummy[:7], dummy[7:]
        t[n:, G_INIT_X:G_INIT_X + 14] = final
        t[n:, G_SUMCHK:G_SUMCHK + 7] = final_chk
        t[n:, G_CUM_X:G_CUM_X + 14] = final
    return t, np.asarray(final, np.uint32)


# ---------------------------------------------------------------- MemoryGlobalInit / Finalize (memory/global.rs)
# MemoryInitCols (memory/global.rs:206-241)
MG_SHARD, MG_TS, MG_ADDR, MG_LT = 0, 1, 2, 3                     # lt_cols: AssertLtColsBits<_, 32>
MG_BITS = 35                                                     # addr_bits: KoalaBearBitDecomposition
MG_AND = 67                                                      #   and_most_sig_byte_decomp_0_to_{2..7}
MG_VALUE, MG_REAL, MG_NEXT_COMP = 73, 105, 106
MG_IZ_INV, MG_IZ_RES, MG_FIRST_COMP, MG_LAST_ADDR = 107, 108, 109, 110
MG_WIDTH = 111
# PublicValues (crates/stark/src/air/public_values.rs:22-60)
PV_PREV_INIT_BITS, PV_LAST_INIT_BITS, PV_PREV_FIN_BITS, PV_LAST_FIN_BITS = 45, 77, 109, 141


def _koala_bear_range_check(ch, value, bits_base, and_base, is_real):
    """KoalaBearBitDecomposition::range_check (operations/koala_bear_range.rs:51-120)."""
    M = main
    bits = [M(bits_base + i) for i in range(32)]
    rec = Expr.lift(0)
    for i, b in enumerate(bits):
        _assert_bool(ch, b, is_real)
        rec = rec + ((1 << i) % P) * b
    ch.assert_zero(is_real * (rec - M(value)))
    msb = bits[24:32]
    ch.assert_zero(is_real * msb[7])
    ch.assert_zero(is_real * (M(and_base) - msb[0] * msb[1]))
    for k in range(1, 6):
        ch.assert_zero(is_real * (M(and_base + k) - M(and_base + k - 1) * msb[k + 1]))
    lower = Expr.lift(0)
    for b in bits[:24]:
        lower = lower + b
    ch.assert_zero(is_real * M(and_base + 5) * lower)


def _assert_lt_bits(ch, flags_base, a, b, is_real, flags_next=False):
    """AssertLtColsBits<_, 32>::eval (operations/cmp.rs:289-354): a < b as 32-bit little-endian bit
    vectors; the flag marks the most significant differing bit."""
    col = main_next if flags_next else main
    flags = [col(flags_base + i) for i in range(32)]
    s = Expr.lift(0)
    for f in flags:
        _assert_bool(ch, f)
        s = s + f
    ch.assert_zero(is_real * (s - 1))
    visited, acmp, bcmp = Expr.lift(0), Expr.lift(0), Expr.lift(0)
    for i in range(31, -1, -1):
        visited = visited + flags[i]
        acmp = acmp + a[i] * flags[i]
        bcmp = bcmp + b[i] * flags[i]
        ch.assert_zero(is_real * (1 - visited) * (a[i] - b[i]))
    ch.assert_zero(is_real * acmp)
    ch.assert_zero(is_real * (bcmp - 1))


def memory_global_chip(initialize: bool) -> ChipDesc:
    """MemoryGlobalChip::eval (memory/global.rs:245-442) for MemoryGlobalInit / MemoryGlobalFinalize."""
    from .machine import IS_LAST, pv
    ch = ChipDesc("MemoryGlobalInit" if initialize else "MemoryGlobalFinalize", prep_width=0, main_width=MG_WIDTH)
    M, N = main, main_next
    real = M(MG_REAL)
    _assert_bool(ch, real)
    for i in range(32):
        _assert_bool(ch, M(MG_VALUE + i))
    byte = [V([("main", MG_VALUE + 8 * k + i, 1 << i) for i in range(8)]) for k in range(4)]
    if initialize:
        vals = [ZERO, ZERO, _m(MG_ADDR)] + byte + [_m(MG_REAL), ZERO, V.const(KIND_MEMORY)]
    else:
        vals = [_m(MG_SHARD), _m(MG_TS), _m(MG_ADDR)] + byte + [ZERO, _m(MG_REAL), V.const(KIND_MEMORY)]
    ch.sends.append(Lookup(vals, _m(MG_REAL), KIND_GLOBAL))
    _koala_bear_range_check(ch, MG_ADDR, MG_BITS, MG_AND, real)
    ch.assert_zero(IS_TRANSITION * (N(MG_NEXT_COMP) - N(MG_REAL)))
    _assert_lt_bits(ch, MG_LT, [M(MG_BITS + i) for i in range(32)], [N(MG_BITS + i) for i in range(32)],
                    N(MG_NEXT_COMP), flags_next=True)
    ch.assert_zero(IS_TRANSITION * (1 - real) * N(MG_REAL))
    prev_base = PV_PREV_INIT_BITS if initialize else PV_PREV_FIN_BITS
    last_base = PV_LAST_INIT_BITS if initialize else PV_LAST_FIN_BITS
    prev_bits = [pv(prev_base + i) for i in range(32)]
    prev_addr = Expr.lift(0)
    for i in range(32):
        prev_addr = prev_addr + prev_bits[i] * ((1 << i) % P)
    # IsZeroOperation::eval(prev_addr, is_prev_addr_zero, is_first_row) (operations/is_zero.rs:42-66)
    res = M(MG_IZ_RES)
    ch.assert_zero(IS_FIRST * ((1 - M(MG_IZ_INV) * prev_addr) - res))
    ch.assert_zero(IS_FIRST * (res * (res - 1)))
    ch.assert_zero(IS_FIRST * res * prev_addr)
    _assert_bool(ch, M(MG_FIRST_COMP))
    ch.assert_zero(IS_FIRST * (M(MG_FIRST_COMP) - (1 - res)))
    ch.assert_zero(IS_FIRST * (real - 1))
    _assert_lt_bits(ch, MG_LT, prev_bits, [M(MG_BITS + i) for i in range(32)], M(MG_FIRST_COMP))
    ch.assert_zero(IS_FIRST * res * M(MG_ADDR))
    ch.assert_zero(IS_FIRST * res * (N(MG_REAL) - 1))
    ch.assert_zero(IS_FIRST * res * (N(MG_NEXT_COMP) - 1))
    if initialize:
        ch.assert_zero(real * (M(MG_TS) - 1))
    for i in range(32):
        ch.assert_zero(IS_FIRST * (1 - M(MG_FIRST_COMP)) * M(MG_VALUE + i))
    ch.assert_zero(IS_TRANSITION * (M(MG_LAST_ADDR) - real * (1 - N(MG_REAL))))
    for i in range(32):
        bit = M(MG_BITS + i) - pv(last_base + i)
        ch.assert_zero(IS_LAST * real * bit)
        ch.assert_zero(IS_TRANSITION * M(MG_LAST_ADDR) * bit)
    return ch


def _bits32(x: int):
    return [(int(x) >> i) & 1 for i in range(32)]


def memory_global_trace(events: np.ndarray, initialize: bool, prev_addr: int = 0):
    """MemoryGlobalChip::generate_dependencies + generate_trace (memory/global.rs:62-188).  events: n x 4
    (addr, value, shard, timestamp).  Returns (trace, global messages n x 7, is_receive n)."""
    ev = np.asarray(events, np.int64).reshape(-1, 4)
    ev = ev[np.argsort(ev[:, 0], kind="stable")]
    n = len(ev)
    t = np.zeros((A._pow2(n), MG_WIDTH), np.uint32)
    addr = ev[:, 0]
    t[:n, MG_ADDR], t[:n, MG_SHARD], t[:n, MG_TS] = addr, ev[:, 2], ev[:, 3]
    bits = (addr[:, None] >> np.arange(32, dtype=np.int64)) & 1
    t[:n, MG_BITS:MG_BITS + 32] = bits
    msb = bits[:, 24:32]
    acc = msb[:, 0] * msb[:, 1]
    t[:n, MG_AND] = acc
    for k in range(1, 6):
        acc = acc * msb[:, k + 1]
        t[:n, MG_AND + k] = acc
    t[:n, MG_VALUE:MG_VALUE + 32] = (ev[:, 1:2] >> np.arange(32, dtype=np.int64)) & 1
    t[:n, MG_REAL] = 1

    def lt_flags(a: int, b: int):
        x = a ^ b
        f = [0] * 32
        if x:
            f[x.bit_length() - 1] = 1
        return f

    if n:
        t[0, MG_IZ_INV] = _inv(prev_addr) if prev_addr else 0
        t[0, MG_IZ_RES] = 1 if prev_addr == 0 else 0
        t[0, MG_FIRST_COMP] = 1 if prev_addr != 0 else 0
        if prev_addr != 0:
            assert prev_addr < addr[0]
            t[0, MG_LT:MG_LT + 32] = lt_flags(prev_addr, int(addr[0]))
        for i in range(1, n):
            assert addr[i - 1] < addr[i]
            t[i, MG_NEXT_COMP] = 1
            t[i, MG_LT:MG_LT + 32] = lt_flags(int(addr[i - 1]), int(addr[i]))
        t[n - 1, MG_LAST_ADDR] = 1
    else:
        t[0, MG_IZ_RES] = 1 if prev_addr == 0 else 0
    msg = np.zeros((n, 7), np.uint32)
    if not initialize:
        msg[:, 0], msg[:, 1] = ev[:, 2], ev[:, 3]
    msg[:, 2] = addr
    msg[:, 3:7] = A._bytes(ev[:, 1].astype(np.uint32))
    rec = np.full(n, 0 if initialize else 1, np.uint8)
    return t, msg, rec
