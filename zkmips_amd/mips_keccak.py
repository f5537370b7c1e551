"""KeccakSponge precompile (MipsAir::KeccakSponge, crates/core/machine/src/mips/mod.rs:277-279): the
KECCAK_SPONGE syscall absorbs a message of 36-word (1088-bit) blocks into a Keccak-f[1600] state and
writes the first 16 words of the squeezed state.

Restated from crates/core/machine/src/syscall/precompiles/keccak_sponge/ (columns.rs KeccakSpongeCols,
air.rs eval / eval_flags / eval_memory_access / eval_state_keccakf, trace.rs event_to_rows /
generate_trace) and the executor's syscalls/precompiles/keccak/sponge.rs.  The permutation columns are
Plonky3's `p3-keccak-air` (ProjectZKM/Plonky3 @ faa24ca, Cargo.lock; a git dependency that is not
vendored in /root/reference), restated from its published algorithm: KeccakCols (step_flags, export,
preimage, a, c, c', a', a'', the bits of a''[0][0], a'''[0][0]), `eval_round_flags`, `KeccakAir::eval`
and `generate_trace_rows` (one row per round: C, C' = C ^ C[x-1] ^ rot(C[x+1], 1), A' = A ^ C ^ C',
B = rho/pi of A', A'' = chi(B), A'''[0][0] = A''[0][0] ^ RC[round]).  The permutation itself is pinned
to hashlib's SHA3 (same Keccak-f[1600], tests/test_keccak.py).  Cost 24 x 4259 = 102216 = mips_costs.json.
"""
from __future__ import annotations

from typing import List

import numpy as np

from . import mips_alu as A
from .machine import ChipDesc, Expr, IS_FIRST, IS_LAST, IS_TRANSITION, KIND_SYSCALL, Lookup, P, main, main_next
from .machine import VirtualPairCol as V
from .mips_alu import _assert_bool, _m

KECCAK_SPONGE = 0x01_01_00_09  # SyscallCode (executor/src/syscalls/code.rs:57)
RATE_U32S, STATE_U32S, OUT_U32S = 36, 50, 16  # keccak_sponge/mod.rs:10-12
NUM_ROUNDS, U64_LIMBS, BITS_PER_LIMB = 24, 4, 16
RD_W, WR_W = 9, 13  # MemoryReadCols / MemoryWriteCols

# Keccak-f[1600] round constants and rho offsets R[x][y] (the Keccak reference; p3-keccak-air constants.rs)
RC = [0x0000000000000001, 0x0000000000008082, 0x800000000000808A, 0x8000000080008000, 0x000000000000808B,
      0x0000000080000001, 0x8000000080008081, 0x8000000000008009, 0x000000000000008A, 0x0000000000000088,
      0x0000000080008009, 0x000000008000000A, 0x000000008000808B, 0x800000000000008B, 0x8000000000008089,
      0x8000000000008003, 0x8000000000008002, 0x8000000000000080, 0x000000000000800A, 0x800000008000000A,
      0x8000000080008081, 0x8000000000008080, 0x0000000080000001, 0x8000000080008008]
R = [[0, 36, 3, 41, 18], [1, 44, 10, 45, 2], [62, 6, 43, 15, 61], [28, 55, 25, 21, 56], [27, 20, 39, 8, 14]]

# KeccakCols (p3-keccak-air columns.rs); a[y][x][limb], c[x][z], a'[y][x][z]
K_STEP = 0
K_EXPORT = K_STEP + NUM_ROUNDS
K_PRE = K_EXPORT + 1
K_A = K_PRE + 100
K_C = K_A + 100
K_CP = K_C + 320
K_AP = K_CP + 320
K_APP = K_AP + 1600
K_APP00_BITS = K_APP + 100
K_APPP00 = K_APP00_BITS + 64
NUM_KECCAK_COLS = K_APPP00 + U64_LIMBS  # 2633

# KeccakSpongeCols (keccak_sponge/columns.rs:16-38)
BLOCK_MEM = NUM_KECCAK_COLS               # 36 x MemoryReadCols
SHARD = BLOCK_MEM + RATE_U32S * RD_W
CLK, REAL, READ_BLOCK, IN_ADDR, OUT_ADDR, IN_LEN, ABSORBED_U32S, IS_ABSORBED, RECV, WRITE_OUT, FIRST_BLK, FINAL_BLK = \
    range(SHARD + 1, SHARD + 13)
ORIG = FINAL_BLK + 1                      # original_state: 50 words
XORED = ORIG + 4 * STATE_U32S             # xored_general_rate: 36 x XorOperation (a word)
IN_LEN_MEM = XORED + 4 * RATE_U32S        # MemoryReadCols
OUT_MEM = IN_LEN_MEM + RD_W               # 16 x MemoryWriteCols
WIDTH = OUT_MEM + OUT_U32S * WR_W         # 3531


def _a(y, x, limb):
    return K_A + (5 * y + x) * U64_LIMBS + limb


def _pre(y, x, limb):
    return K_PRE + (5 * y + x) * U64_LIMBS + limb


def _app(y, x, limb):
    return K_APP + (5 * y + x) * U64_LIMBS + limb


def _c(x, z):
    return K_C + 64 * x + z


def _cp(x, z):
    return K_CP + 64 * x + z


def _ap(y, x, z):
    return K_AP + (5 * y + x) * 64 + z


def _b(x, y, z):
    """KeccakCols::b: B[x, y] = ROT(A'[(x + 3y) % 5, x], R[(x + 3y) % 5][x]) as an alias of an A' column."""
    a = (x + 3 * y) % 5
    return _ap(x, a, (z + 64 - R[a][x]) % 64)


def _appp(y, x, limb):
    """KeccakCols::a_prime_prime_prime."""
    return K_APPP00 + limb if (x, y) == (0, 0) else _app(y, x, limb)


def _rc_bit(r, z):
    return (RC[r] >> z) & 1


def _xor(x: Expr, y: Expr) -> Expr:
    return x + y - x * (y * 2)  # xor_gen


def _xor3(x, y, z):
    return _xor(x, _xor(y, z))


def _andn(x, y):
    return (1 - x) * y


def _bits_to_limb(bits) -> Expr:
    """The fold `(limb*16..limb*16+16).rev().fold(0, |acc, z| acc.double() + bit(z))` (doubling as a
    product by the constant 2, which is the same value)."""
    acc = Expr.lift(0)
    for b in reversed(bits):
        acc = acc * 2 + b
    return acc


def eval_keccak_air(ch: ChipDesc):
    """KeccakAir::eval with eval_round_flags (p3-keccak-air air.rs, round_flags.rs) over columns
    0..NUM_KECCAK_COLS of the chip (SubAirBuilder)."""
    M, N = main, main_next
    for i in range(NUM_ROUNDS):  # eval_round_flags
        ch.assert_zero(IS_FIRST * (M(K_STEP + i) - (1 if i == 0 else 0)))
    for i in range(NUM_ROUNDS):
        ch.assert_zero(IS_TRANSITION * (N(K_STEP + (i + 1) % NUM_ROUNDS) - M(K_STEP + i)))
    first_step, final_step = M(K_STEP), M(K_STEP + NUM_ROUNDS - 1)
    not_final_step = 1 - final_step
    for y in range(5):
        for x in range(5):
            for limb in range(U64_LIMBS):
                ch.assert_zero(first_step * (M(_pre(y, x, limb)) - M(_a(y, x, limb))))
    _assert_bool(ch, M(K_EXPORT))
    ch.assert_zero(not_final_step * M(K_EXPORT))
    for y in range(5):
        for x in range(5):
            for limb in range(U64_LIMBS):
                ch.assert_zero(not_final_step * IS_TRANSITION * (M(_pre(y, x, limb)) - N(_pre(y, x, limb))))
    for x in range(5):  # C'[x, z] = xor(C[x, z], C[x - 1, z], C[x + 1, z - 1])
        for z in range(64):
            _assert_bool(ch, M(_c(x, z)))
            ch.assert_zero(M(_cp(x, z)) - _xor3(M(_c(x, z)), M(_c((x + 4) % 5, z)), M(_c((x + 1) % 5, (z + 63) % 64))))
    for y in range(5):  # A[x, y, z] = xor(A'[x, y, z], C[x, z], C'[x, z])
        for x in range(5):
            for limb in range(U64_LIMBS):
                zs = range(limb * BITS_PER_LIMB, (limb + 1) * BITS_PER_LIMB)
                for z in reversed(zs):
                    _assert_bool(ch, M(_ap(y, x, z)))
                bits = [_xor3(M(_ap(y, x, z)), M(_c(x, z)), M(_cp(x, z))) for z in zs]
                ch.assert_zero(_bits_to_limb(bits) - M(_a(y, x, limb)))
    for x in range(5):  # xor_y A'[x, y, z] = C'[x, z]: diff (diff - 2) (diff - 4) = 0
        for z in range(64):
            s = M(_ap(0, x, z))
            for y in range(1, 5):
                s = s + M(_ap(y, x, z))
            diff = (s - M(_cp(x, z))).share()
            ch.assert_zero(diff * (diff - 2) * (diff - 4))
    for y in range(5):  # A''[x, y] = xor(B[x, y], andn(B[x + 1, y], B[x + 2, y]))
        for x in range(5):
            for limb in range(U64_LIMBS):
                zs = range(limb * BITS_PER_LIMB, (limb + 1) * BITS_PER_LIMB)
                bits = [_xor(M(_b(x, y, z)), _andn(M(_b((x + 1) % 5, y, z)), M(_b((x + 2) % 5, y, z)))) for z in zs]
                ch.assert_zero(_bits_to_limb(bits) - M(_app(y, x, limb)))
    for limb in range(U64_LIMBS):  # the bits of A''[0, 0]
        zs = range(limb * BITS_PER_LIMB, (limb + 1) * BITS_PER_LIMB)
        for z in reversed(zs):
            _assert_bool(ch, M(K_APP00_BITS + z))
        ch.assert_zero(_bits_to_limb([M(K_APP00_BITS + z) for z in zs]) - M(_app(0, 0, limb)))
    for limb in range(U64_LIMBS):  # A'''[0, 0] = A''[0, 0] ^ RC (the round's constant bit from the step flags)
        bits = []
        for z in range(limb * BITS_PER_LIMB, (limb + 1) * BITS_PER_LIMB):
            rc = Expr.lift(0)
            for r in range(NUM_ROUNDS):
                rc = rc + M(K_STEP + r) * _rc_bit(r, z)
            bits.append(_xor(M(K_APP00_BITS + z), rc))
        ch.assert_zero(_bits_to_limb(bits) - M(K_APPP00 + limb))
    for x in range(5):  # this round's output is the next round's input
        for y in range(5):
            for limb in range(U64_LIMBS):
                ch.assert_zero(IS_TRANSITION * not_final_step * (M(_appp(y, x, limb)) - N(_a(y, x, limb))))


def _limbs_of_words(lo: int, hi: int, nxt=False):
    """Two u32 memory words (byte columns) as four u16 limbs."""
    f = main_next if nxt else main
    return [f(lo) + f(lo + 1) * 256, f(lo + 2) + f(lo + 3) * 256, f(hi) + f(hi + 1) * 256, f(hi + 2) + f(hi + 3) * 256]


def keccak_sponge_chip() -> ChipDesc:
    """KeccakSpongeChip::eval (keccak_sponge/air.rs:27-119) in the reference's order."""
    from .mips_core import _eval_memory_access
    from .mips_syscall import _eval_xor
    M, N = main, main_next
    ch = ChipDesc("KeccakSponge", prep_width=0, main_width=WIDTH)
    real, first_step, final_step = M(REAL), M(K_STEP), M(K_STEP + NUM_ROUNDS - 1)
    not_final_step = 1 - final_step
    not_final_sponge = 1 - M(WRITE_OUT)
    # eval_flags (:121-141)
    ch.assert_zero(M(FIRST_BLK) * first_step * real - M(RECV))
    ch.assert_zero(M(FINAL_BLK) * final_step * real - M(WRITE_OUT))
    ch.assert_zero(M(IS_ABSORBED) - final_step * (1 - M(FINAL_BLK)) * real)
    # eval_memory_access (:143-188): the input length at output_address + 64, the block, the output at clk + 1
    clk_terms = ((CLK, 1),)
    _eval_memory_access(ch, IN_LEN_MEM, IN_LEN_MEM, 0, V([("main", OUT_ADDR, 1)], 64), M(RECV), _m(RECV),
                        shard_col=SHARD, clk_terms=clk_terms)
    for j in range(4):
        ch.assert_zero(real * (M(IN_LEN_MEM + j) - M(IN_LEN_MEM + j)))
    for i in range(RATE_U32S):
        acc = BLOCK_MEM + RD_W * i
        _eval_memory_access(ch, acc, acc, 0, V([("main", IN_ADDR, 1)], 4 * i), M(READ_BLOCK), _m(READ_BLOCK),
                            shard_col=SHARD, clk_terms=clk_terms)
    for i in range(RATE_U32S):
        acc = BLOCK_MEM + RD_W * i
        for j in range(4):
            ch.assert_zero(real * (M(acc + j) - M(acc + j)))
    for i in range(OUT_U32S):
        base = OUT_MEM + WR_W * i
        _eval_memory_access(ch, base + 4, base, 1, V([("main", OUT_ADDR, 1)], 4 * i), M(WRITE_OUT), _m(WRITE_OUT),
                            shard_col=SHARD, clk_terms=clk_terms)
    # eval_state_keccakf (:189-284)
    for i in range(STATE_U32S // 2):
        y, x = divmod(i, 5)
        src = XORED if i < RATE_U32S // 2 else ORIG
        cur = _limbs_of_words(src + 8 * i, src + 8 * i + 4)
        for j in range(U64_LIMBS):
            ch.assert_zero(first_step * real * (cur[j] - M(_a(y, x, j))))
        nxt = _limbs_of_words(ORIG + 8 * i, ORIG + 8 * i + 4, nxt=True)
        for j in range(U64_LIMBS):
            ch.assert_zero(M(IS_ABSORBED) * (nxt[j] - M(_appp(y, x, j))))
    for i in range(OUT_U32S // 2):
        y, x = divmod(i, 5)
        out = _limbs_of_words(OUT_MEM + WR_W * 2 * i + 4, OUT_MEM + WR_W * (2 * i + 1) + 4)
        for j in range(U64_LIMBS):
            ch.assert_zero(M(WRITE_OUT) * (out[j] - M(_appp(y, x, j))))
    ch.receives.append(Lookup([_m(SHARD), _m(CLK), V.const(KECCAK_SPONGE & 0xFFFF), _m(IN_ADDR), _m(OUT_ADDR)],
                              _m(RECV), KIND_SYSCALL))
    for c in (SHARD, CLK, REAL, IN_LEN, OUT_ADDR):  # the inputs stay the same through a call's rows
        ch.assert_zero(IS_TRANSITION * not_final_sponge * (M(c) - N(c)))
    ch.assert_zero(IS_LAST * real)
    for i in range(RATE_U32S):  # xored_general_rate = original_state ^ block
        _eval_xor(ch, [_m(ORIG + 4 * i + j) for j in range(4)], [_m(BLOCK_MEM + RD_W * i + j) for j in range(4)],
                  XORED + 4 * i, _m(READ_BLOCK))
    ch.assert_zero(IS_TRANSITION * not_final_step * (M(ABSORBED_U32S) - N(ABSORBED_U32S)))
    ch.assert_zero(M(FIRST_BLK) * (M(ABSORBED_U32S) - 0))
    ch.assert_zero(M(FINAL_BLK) * (M(ABSORBED_U32S) - (M(IN_LEN) - RATE_U32S)))
    ch.assert_zero(M(IS_ABSORBED) * (M(ABSORBED_U32S) - (N(ABSORBED_U32S) - RATE_U32S)))
    ch.assert_zero(M(IS_ABSORBED) * (M(IN_ADDR) - (N(IN_ADDR) - 4 * RATE_U32S)))
    eval_keccak_air(ch)
    return ch


# ---------------------------------------------------------------- the permutation and its rows
_M64 = (1 << 64) - 1


def _rotl(v: np.ndarray, s: int) -> np.ndarray:
    s %= 64
    if s == 0:
        return v.copy()
    return (v << np.uint64(s)) | (v >> np.uint64(64 - s))


def keccakf(state: np.ndarray) -> np.ndarray:
    """Keccak-f[1600] over (n, 25) uint64 lanes (lane index 5y + x), as tiny_keccak::keccakf."""
    a = np.array(state, np.uint64).reshape(-1, 25).copy()
    for r in range(NUM_ROUNDS):
        a = _round(a, r)[-1]
    return a


def _round(a: np.ndarray, r: int):
    """One round: returns (C, C', A', A'', A''') with A''' the next round's A."""
    c = np.stack([a[:, x] ^ a[:, 5 + x] ^ a[:, 10 + x] ^ a[:, 15 + x] ^ a[:, 20 + x] for x in range(5)], 1)
    cp = np.stack([c[:, x] ^ c[:, (x + 4) % 5] ^ _rotl(c[:, (x + 1) % 5], 1) for x in range(5)], 1)
    ap = np.empty_like(a)
    for y in range(5):
        for x in range(5):
            ap[:, 5 * y + x] = a[:, 5 * y + x] ^ c[:, x] ^ cp[:, x]
    b = np.empty_like(a)  # b[5y + x] = B[x, y]
    for y in range(5):
        for x in range(5):
            s = (x + 3 * y) % 5
            b[:, 5 * y + x] = _rotl(ap[:, 5 * x + s], R[s][x])
    app = np.empty_like(a)
    for y in range(5):
        for x in range(5):
            app[:, 5 * y + x] = b[:, 5 * y + x] ^ (~b[:, 5 * y + (x + 1) % 5] & b[:, 5 * y + (x + 2) % 5])
    appp = app.copy()
    appp[:, 0] ^= np.uint64(RC[r])
    return c, cp, ap, app, appp


def _limb_cols(lanes: np.ndarray) -> np.ndarray:
    """(n, k) uint64 lanes -> (n, 4k) u16 limbs, lane-major."""
    sh = np.arange(U64_LIMBS, dtype=np.uint64) * np.uint64(16)
    return ((lanes[:, :, None] >> sh) & np.uint64(0xFFFF)).reshape(len(lanes), -1)


def _bit_cols(lanes: np.ndarray) -> np.ndarray:
    """(n, k) uint64 lanes -> (n, 64k) bits, lane-major."""
    sh = np.arange(64, dtype=np.uint64)
    return ((lanes[:, :, None] >> sh) & np.uint64(1)).reshape(len(lanes), -1)


def keccak_rows(inputs: np.ndarray) -> np.ndarray:
    """generate_trace_rows restricted to the 24 rows of each input: (n, 25) u64 -> (24 n, NUM_KECCAK_COLS),
    the rows of permutation k at 24 k .. 24 k + 23."""
    inp = np.asarray(inputs, np.uint64).reshape(-1, 25)
    n = len(inp)
    t = np.zeros((n, NUM_ROUNDS, NUM_KECCAK_COLS), np.int64)
    pre = _limb_cols(inp)
    a = inp.copy()
    for r in range(NUM_ROUNDS):
        c, cp, ap, app, appp = _round(a, r)
        row = t[:, r]
        row[:, K_STEP + r] = 1
        row[:, K_PRE:K_PRE + 100] = pre
        row[:, K_A:K_A + 100] = _limb_cols(a)
        row[:, K_C:K_C + 320] = _bit_cols(c)
        row[:, K_CP:K_CP + 320] = _bit_cols(cp)
        row[:, K_AP:K_AP + 1600] = _bit_cols(ap)
        row[:, K_APP:K_APP + 100] = _limb_cols(app)
        row[:, K_APP00_BITS:K_APP00_BITS + 64] = _bit_cols(app[:, :1])
        row[:, K_APPP00:K_APPP00 + 4] = _limb_cols(appp[:, :1])
        a = appp
    return t.reshape(n * NUM_ROUNDS, NUM_KECCAK_COLS)


# ---------------------------------------------------------------- execution
def _u64s(words: List[int]) -> List[int]:
    return [words[2 * i] | (words[2 * i + 1] << 32) for i in range(len(words) // 2)]


def exec_keccak_sponge(pm, shard: int, clk: int, input_ptr: int, result_ptr: int):
    """KeccakSpongeSyscall::execute (executor/src/syscalls/precompiles/keccak/sponge.rs:21-96): the input
    length (in words) is read from result_ptr + 64, the input and its length at clk, the 16 output words
    written at clk + 1."""
    len_rec = pm.read(result_ptr + 16 * 4, clk)
    n = len_rec[0]
    assert n % RATE_U32S == 0 and n > 0, "the input length must be a positive multiple of 36 words"
    in_recs = [pm.read(input_ptr + 4 * i, clk) for i in range(n)]
    words = [r[0] for r in in_recs]
    state = np.zeros((1, 25), np.uint64)
    xored = []
    for blk in range(n // RATE_U32S):
        for i, v in enumerate(_u64s(words[blk * RATE_U32S:(blk + 1) * RATE_U32S])):
            state[0, i] ^= np.uint64(v)
        xored.append([int(v) for v in state[0]])
        state = keccakf(state)
    out = []
    for i in range(OUT_U32S // 2):
        v = int(state[0, i])
        out += [v & 0xFFFFFFFF, v >> 32]
    w_recs = [pm.write(result_ptr + 4 * i, out[i], clk + 1) for i in range(OUT_U32S)]
    return {"shard": shard, "clk": clk, "in_ptr": input_ptr, "out_ptr": result_ptr, "len": len_rec, "in": in_recs,
            "xored": xored, "out": out, "w": w_recs, "local": pm.local_entries()}


# ---------------------------------------------------------------- trace
def keccak_sponge_trace(events, byte_lookup) -> np.ndarray:
    """KeccakSpongeChip::generate_trace + event_to_rows (keccak_sponge/trace.rs:62-196): 24 rows per
    absorbed block, padding rows repeat the zero-input permutation's rows (row i holds round i % 24)."""
    from .mips_core import _access_cols
    from .mips_syscall import _xor_cols
    blocks = [(e, k) for e in events for k in range(len(e["xored"]))]
    nreal = NUM_ROUNDS * len(blocks)
    h = max(16, 1 << max(0, (nreal - 1).bit_length()))
    t = np.zeros((h, WIDTH), np.int64)
    if blocks:
        t[:nreal, :NUM_KECCAK_COLS] = keccak_rows(np.array([e["xored"][k] for e, k in blocks], np.uint64))
    npad = h - nreal
    if npad:
        dummy = keccak_rows(np.zeros((1, 25), np.uint64))
        t[nreal:, :NUM_KECCAK_COLS] = dummy[np.arange(nreal, h) % NUM_ROUNDS]
    if not blocks:
        return (t % P).astype(np.uint32)
    nb = len(blocks)
    base = np.arange(nb) * NUM_ROUNDS
    r0, r23 = base, base + NUM_ROUNDS - 1
    rows = np.arange(nreal)
    blk_of_row = rows // NUM_ROUNDS
    ev = [e for e, _ in blocks]
    k_of = np.array([k for _, k in blocks])
    nblk = np.array([len(e["xored"]) for e in ev])
    first, final = k_of == 0, k_of == nblk - 1
    shard = np.array([e["shard"] for e in ev], np.int64)
    clk = np.array([e["clk"] for e in ev], np.int64)
    t[rows, SHARD] = shard[blk_of_row]
    t[rows, CLK] = clk[blk_of_row]
    t[rows, REAL] = 1
    t[rows, IN_LEN] = np.array([len(e["in"]) for e in ev])[blk_of_row]
    t[rows, ABSORBED_U32S] = (k_of * RATE_U32S)[blk_of_row]
    t[r23[~final], IS_ABSORBED] = 1
    t[rows, FIRST_BLK] = first[blk_of_row]
    t[rows, FINAL_BLK] = final[blk_of_row]
    t[r0, READ_BLOCK] = 1
    t[r0[first], RECV] = 1
    t[r23[final], WRITE_OUT] = 1
    t[rows, OUT_ADDR] = np.array([e["out_ptr"] for e in ev], np.int64)[blk_of_row]
    t[rows, IN_ADDR] = (np.array([e["in_ptr"] for e in ev], np.int64) + k_of * 4 * RATE_U32S)[blk_of_row]
    # original_state: the state before the block's absorption (keccakf of the previous xored state)
    orig = np.zeros((nb, 25), np.uint64)
    for j, (e, k) in enumerate(blocks):
        if k:
            orig[j] = keccakf(np.array([e["xored"][k - 1]], np.uint64))[0]
    orig_words = np.stack([orig & np.uint64(0xFFFFFFFF), orig >> np.uint64(32)], 2).reshape(nb, STATE_U32S)
    t[rows, ORIG:ORIG + 4 * STATE_U32S] = A._bytes(orig_words.astype(np.uint32).reshape(-1)).reshape(nb, -1)[blk_of_row]
    # round 0 of every block: the block reads and the xor with the rate words
    in_recs = np.array([e["in"][k * RATE_U32S:(k + 1) * RATE_U32S] for e, k in blocks], np.int64)  # (nb, 36, 3)
    for i in range(RATE_U32S):
        _access_cols(t, r0, BLOCK_MEM + RD_W * i, in_recs[:, i, 0].astype(np.uint32), in_recs[:, i, 1:3], shard, clk,
                     np.ones(nb, bool), byte_lookup)
    for i in range(RATE_U32S):
        xo = _xor_cols(orig_words[:, i].astype(np.uint32), in_recs[:, i, 0].astype(np.uint32), byte_lookup)
        t[r0, XORED + 4 * i:XORED + 4 * i + 4] = xo
    # the first row of a call reads the input length, its last row writes the output
    fi = np.nonzero(first)[0]
    lrec = np.array([ev[j]["len"] for j in fi], np.int64)
    _access_cols(t, r0[fi], IN_LEN_MEM, lrec[:, 0].astype(np.uint32), lrec[:, 1:3], shard[fi], clk[fi],
                 np.ones(len(fi), bool), byte_lookup)
    li = np.nonzero(final)[0]
    wrec = np.array([ev[j]["w"] for j in li], np.int64)  # (calls, 16, 4): prev, value, prev_shard, prev_clk
    for i in range(OUT_U32S):
        base_c = OUT_MEM + WR_W * i
        t[r23[li], base_c:base_c + 4] = A._bytes(wrec[:, i, 0].astype(np.uint32))
        _access_cols(t, r23[li], base_c + 4, wrec[:, i, 1].astype(np.uint32), wrec[:, i, 2:4], shard[li], clk[li] + 1,
                     np.ones(len(li), bool), byte_lookup)
    return (t % P).astype(np.uint32)


# ---------------------------------------------------------------- a guest
def sha3_pad(msg: bytes, rate: int = 4 * RATE_U32S) -> bytes:
    """SHA-3 padding (0x06 ... 0x80) to a multiple of the 144-byte rate the syscall absorbs."""
    m = bytearray(msg) + b"\x06"
    m += bytes(-len(m) % rate)
    m[-1] |= 0x80
    return bytes(m)


def keccak_program(messages: List[bytes], halt: bool = True):
    """A guest that hashes each message with KECCAK_SPONGE (padded by the guest as SHA3-224 pads; the first
    28 output bytes are then hashlib.sha3_224(message)): it stores the padded message and its length in
    words at result + 64, calls the syscall, reads the 16 output words back and folds them into a
    register that is committed, then HALT."""
    from . import mips_core as MC
    from . import mips_syscall as SY
    prog = []
    acc, tmp = 10, 9
    slot = [MC.DATA_BASE + 0x8000]

    def alloc(nbytes):
        p_ = slot[0]
        slot[0] += (nbytes + 63) // 64 * 64
        return p_

    def li(reg, v):
        prog.append((A.OP_ADD, reg, 0, int(v) & 0xFFFFFFFF, 0, 1))

    li(acc, 0)
    for msg in messages:
        padded = sha3_pad(msg)
        words = np.frombuffer(padded, "<u4")
        ip, rp = alloc(len(padded)), alloc(4 * (OUT_U32S + 1))
        for i, w in enumerate(list(words) + [len(words)]):
            li(8, int(w))
            prog.append((MC.OP_SW, 8, 0, (ip + 4 * i) if i < len(words) else rp + 64, 0, 1))
        li(SY.REG_V0, KECCAK_SPONGE)
        li(SY.REG_A0, ip)
        li(SY.REG_A1, rp)
        prog.append((SY.OP_SYSCALL, SY.REG_V0, SY.REG_A0, SY.REG_A1, 0, 0))
        for i in range(OUT_U32S):
            prog.append((MC.OP_LW, tmp, 0, rp + 4 * i, 0, 1))
            prog.append((A.OP_XOR, acc, acc, tmp, 0, 0))
    prog += [(A.OP_ADD, SY.REG_V0, 0, SY.COMMIT, 0, 1), (A.OP_ADD, SY.REG_A0, 0, 0, 0, 1),
             (A.OP_ADD, SY.REG_A1, acc, 0, 0, 1), (SY.OP_SYSCALL, SY.REG_V0, SY.REG_A0, SY.REG_A1, 0, 0)]
    if halt:
        prog += [(A.OP_ADD, SY.REG_V0, 0, SY.HALT, 0, 1), (A.OP_ADD, SY.REG_A0, 0, 0, 0, 1),
                 (SY.OP_SYSCALL, SY.REG_V0, SY.REG_A0, SY.REG_A1, 0, 0)]
    return prog
