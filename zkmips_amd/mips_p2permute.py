"""Poseidon2Permute precompile (MipsAir::Poseidon2Permute, crates/core/machine/src/mips/mod.rs:145):
POSEIDON2_PERMUTE replaces 16 KoalaBear words in memory by their Poseidon2-16 permutation.

Restated from crates/core/machine/src/syscall/precompiles/poseidon2/ (columns.rs Poseidon2MemCols, air.rs
eval, trace.rs event_to_row / generate_trace) over operations/poseidon2/ (Poseidon2Degree3Cols: the
external / internal round states, the s0 ghost columns, the output and the degree-3 S-box columns;
eval_external_round / eval_internal_rounds), and the executor's permute.rs (the state read without a
record and written at clk).  The round expressions reuse the recursion chip's shared-subexpression
forms (recursion.py: the same permutation with the same column layout).  Cost 1117 = mips_costs.json.
"""
from __future__ import annotations

from typing import List

import numpy as np

from . import mips_alu as A
from . import recursion as R
from .machine import ChipDesc, KIND_SYSCALL, Lookup, P, main
from .machine import VirtualPairCol as V
from .mips_alu import _assert_bool, _m

WIDTH, NE, NI = R.WIDTH, R.NUM_EXTERNAL_ROUNDS, R.NUM_INTERNAL_ROUNDS
POSEIDON2_PERMUTE = 0x00_01_00_30  # SyscallCode (executor/src/syscalls/code.rs:181)
WR_W = 13

# Poseidon2MemCols (poseidon2/columns.rs:9-20)
PERM = 0                       # Poseidon2Degree3Cols (313)
SHARD = PERM + R.P2_COLS
CLK = SHARD + 1
ADDR = CLK + 1
MEM = ADDR + 1                 # state_mem: 16 x MemoryWriteCols
PRE_RC = MEM + WIDTH * WR_W    # pre_state_range_check_cols: 16 x KoalaBearWordRangeChecker
RC_WIDTH = 14                  # KoalaBearWordRangeChecker (= mips_core.RC_WIDTH)
POST_RC = PRE_RC + WIDTH * RC_WIDTH
REAL = POST_RC + WIDTH * RC_WIDTH
WIDTH_COLS = REAL + 1


def _word_expr(base: int):
    return sum((main(base + j) * (1 << (8 * j)) for j in range(1, 4)), main(base))


def poseidon2_permute_chip() -> ChipDesc:
    """Poseidon2PermuteChip::eval (poseidon2/air.rs:31-97)."""
    from .mips_core import RC_WIDTH as RCW, _eval_memory_access, _word_range_check
    assert RCW == RC_WIDTH
    ch = ChipDesc("Poseidon2Permute", prep_width=0, main_width=WIDTH_COLS)
    real, rv = main(REAL), _m(REAL)
    _assert_bool(ch, real)
    for i in range(WIDTH):  # the pre-state: canonical words equal to the first external round's input
        _word_range_check(ch, MEM + WR_W * i, PRE_RC + RC_WIDTH * i, real)
        ch.assert_zero(real * (main(PERM + R.P2_EXT + i) - _word_expr(MEM + WR_W * i)))
    for r in range(NE):  # eval_external_round (operations/poseidon2/air.rs:84-132)
        st = [main(PERM + R.P2_EXT + r * WIDTH + i) for i in range(WIDTH)]
        if r == 0:
            st = R._external_layer_expr(st)
        rnd = r if r < NE // 2 else r + NI
        sb = []
        for i in range(WIDTH):
            a = (st[i] + R.RC[rnd][i]).share()
            col = PERM + R.P2_ESBOX + r * WIDTH + i
            ch.assert_zero(main(col) - a * a * a)
            sb.append(main(col))
        st = R._external_layer_expr(sb)
        if r == NE // 2 - 1:
            nxt = [PERM + R.P2_INT + i for i in range(WIDTH)]
        elif r == NE - 1:
            nxt = [PERM + R.P2_OUT + i for i in range(WIDTH)]
        else:
            nxt = [PERM + R.P2_EXT + (r + 1) * WIDTH + i for i in range(WIDTH)]
        for i in range(WIDTH):
            ch.assert_zero(main(nxt[i]) - st[i])
    st = [main(PERM + R.P2_INT + i) for i in range(WIDTH)]  # eval_internal_rounds (:134-170)
    for r in range(NI):
        base = st[0] if r == 0 else main(PERM + R.P2_S0 + r - 1)
        a = (base + R.RC[r + NE // 2][0]).share()
        ch.assert_zero(main(PERM + R.P2_ISBOX + r) - a * a * a)
        st = R._internal_layer_expr([main(PERM + R.P2_ISBOX + r)] + st[1:])
        if r < NI - 1:
            ch.assert_zero(main(PERM + R.P2_S0 + r) - st[0])
    for i in range(WIDTH):
        ch.assert_zero(main(PERM + R.P2_EXT + (NE // 2) * WIDTH + i) - st[i])
    for i in range(WIDTH):  # the post-state: canonical words equal to the permutation's output
        acc = MEM + WR_W * i + 4
        _word_range_check(ch, acc, POST_RC + RC_WIDTH * i, real)
        ch.assert_zero(real * (main(PERM + R.P2_OUT + i) - _word_expr(acc)))
    for i in range(WIDTH):  # eval_memory_access_slice at clk
        addr = V([("main", ADDR, 1)], 4 * i)
        _eval_memory_access(ch, MEM + WR_W * i + 4, MEM + WR_W * i, 0, addr, real, rv, shard_col=SHARD,
                            clk_terms=((CLK, 1),))
    ch.receives.append(Lookup([_m(SHARD), _m(CLK), V.const(POSEIDON2_PERMUTE & 0xFFFF), _m(ADDR), V.const(0)], rv,
                              KIND_SYSCALL))
    return ch


def permute(state: List[int]) -> List[int]:
    """Poseidon2-16 over KoalaBear (the permutation poseidon2_init() builds, executor permute.rs), from
    the round columns of R.poseidon2_rows (the recursion chip's trace, same permutation)."""
    rows = R.poseidon2_rows(np.asarray([state], np.uint32))
    return [int(x) for x in rows[0, R.P2_OUT:R.P2_OUT + WIDTH]]


def exec_poseidon2_permute(pm, shard: int, clk: int, ptr: int, a1: int):
    """Poseidon2PermuteSyscall::execute (executor/src/syscalls/precompiles/poseidon2/permute.rs)."""
    assert a1 == 0 and ptr % 4 == 0
    pre = [pm.peek(ptr + 4 * i) for i in range(WIDTH)]
    assert all(w < P for w in pre), "the state words must be canonical KoalaBear elements"
    post = permute(pre)
    rec = [pm.write(ptr + 4 * i, post[i], clk) for i in range(WIDTH)]
    return {"shard": shard, "clk": clk, "ptr": ptr, "pre": pre, "post": post, "w": rec, "local": pm.local_entries()}


def poseidon2_permute_trace(events, byte_lookup) -> np.ndarray:
    """Poseidon2PermuteChip::generate_trace + event_to_row (poseidon2/trace.rs): padding rows hold the
    permutation of zeros."""
    from .mips_core import _range_checker_cols
    from .mips_edwards import _access_block
    ne = len(events)
    h = max(16, 1 << max(0, (ne - 1).bit_length()))
    t = np.zeros((h, WIDTH_COLS), np.int64)
    ins = np.zeros((h, WIDTH), np.uint32)
    for i, e in enumerate(events):
        ins[i] = e["pre"]
    t[:, PERM:PERM + R.P2_COLS] = R.poseidon2_rows(ins)
    if ne:
        rows = np.arange(ne)
        t[rows, REAL] = 1
        shard = np.array([e["shard"] for e in events], np.int64)
        clk = np.array([e["clk"] for e in events], np.int64)
        t[rows, SHARD], t[rows, CLK], t[rows, ADDR] = shard, clk, [e["ptr"] for e in events]
        for i, e in enumerate(events):
            assert list(t[i, PERM + R.P2_OUT:PERM + R.P2_OUT + WIDTH]) == e["post"]
        for k in range(WIDTH):
            t[rows, PRE_RC + RC_WIDTH * k:PRE_RC + RC_WIDTH * (k + 1)] = _range_checker_cols(
                np.array([e["pre"][k] for e in events], np.uint32))
            t[rows, POST_RC + RC_WIDTH * k:POST_RC + RC_WIDTH * (k + 1)] = _range_checker_cols(
                np.array([e["post"][k] for e in events], np.uint32))
        _access_block(t, rows, MEM, [e["w"] for e in events], True, shard, clk, byte_lookup)
    return (t % P).astype(np.uint32)
