"""Debug aid: evaluate a machine blob's constraints and lookups directly on the traces (no STARK).

For each chip, runs the postfix constraint program (zkmips_amd/machine.py) over every row with the
selectors of the trace domain (is_first = row 0, is_last = row N-1, is_transition = row != N-1)
and reports constraints that are non-zero; then sums every lookup tuple's multiplicity per kind
(sends +, receives -) across chips and reports tuples that do not balance.  Test/debug only.

    python -m tests._air_check [n]       # checks mips_core.core_shard(n)
"""
from __future__ import annotations

import collections
import sys

import numpy as np

from zkmips_amd import machine as M

P = M.P


def _eval(code, main, prep, pvs, n, memo=None):
    """Value of a builder expression's code on every row; shared definitions (OP_REF) are evaluated
    once per `memo` (one chip)."""
    memo = {} if memo is None else memo
    st = []
    i = 0
    nxt = lambda a: np.roll(a, -1, axis=0)
    rows = np.arange(n)
    while i < len(code):
        op = code[i]
        i += 1
        if op in (M.OP_MAIN_L, M.OP_MAIN_N, M.OP_PREP_L, M.OP_PREP_N):
            c = code[i]
            i += 1
            src = main if op in (M.OP_MAIN_L, M.OP_MAIN_N) else prep
            col = src[:, c].astype(np.int64)
            st.append(nxt(col) if op in (M.OP_MAIN_N, M.OP_PREP_N) else col)
        elif op == M.OP_CONST:
            st.append(np.full(n, code[i], np.int64))
            i += 1
        elif op == M.OP_PV:
            st.append(np.full(n, int(pvs[code[i]]) % P, np.int64))
            i += 1
        elif op == M.OP_IS_FIRST:
            st.append((rows == 0).astype(np.int64))
        elif op == M.OP_IS_LAST:
            st.append((rows == n - 1).astype(np.int64))
        elif op == M.OP_IS_TRANS:
            st.append((rows != n - 1).astype(np.int64))
        elif op in (M.OP_ADD, M.OP_SUB, M.OP_MUL):
            b, a = st.pop(), st.pop()
            st.append((a + b) % P if op == M.OP_ADD else (a - b) % P if op == M.OP_SUB else (a * b) % P)
        elif op == M.OP_NEG:
            st.append((-st.pop()) % P)
        elif op == M.OP_REF:
            g = code[i]
            i += 1
            if g not in memo:
                memo[g] = _eval(M._SHARED[g], main, prep, pvs, n, memo)
            st.append(memo[g])
        else:
            raise ValueError(op)
    assert len(st) == 1
    return st[0]


def _vpc(v, main, prep, n):
    out = np.full(n, v.constant % P, np.int64)
    for kind, idx, w in v.terms:
        col = (main if kind == "main" else prep)[:, idx].astype(np.int64)
        out = (out + col * (w % P)) % P
    return out


def check(machine, prep_traces, traces, pvs, max_report=5):
    bad = []
    balance = collections.defaultdict(int)
    for ch in machine.chips:
        if ch.name not in traces:
            continue
        main = traces[ch.name]
        n = main.shape[0]
        prep = prep_traces.get(ch.name, np.zeros((n, 0), np.uint32))
        memo = {}
        for k, c in enumerate(ch.constraints):
            r = _eval(c.code, main, prep, pvs, n, memo)
            nz = np.nonzero(r)[0]
            if len(nz):
                bad.append((ch.name, k, nz[:max_report].tolist(), len(nz)))
        for sign, lks in ((1, ch.sends), (-1, ch.receives)):
            for lk in lks:
                if lk.scope != M.LOOKUP_LOCAL:
                    continue
                m = _vpc(lk.multiplicity, main, prep, n)
                vals = np.stack([_vpc(v, main, prep, n) for v in lk.values], axis=1)
                for r in np.nonzero(m)[0]:
                    balance[(lk.kind,) + tuple(vals[r].tolist())] += sign * int(m[r])
    unbalanced = [(k, v) for k, v in balance.items() if v % P]
    return bad, unbalanced


if __name__ == "__main__":
    from zkmips_amd import mips_core as C
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    bad, unb = check(*C.core_shard(n, seed=3))
    for b in bad:
        print("constraint", b)
    for k, v in sorted(unb)[:40]:
        print("unbalanced", k, v)
    print(len(bad), "failing constraints,", len(unb), "unbalanced tuples")
