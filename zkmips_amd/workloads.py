"""Synthetic shard workloads — deterministic, seeded, host-side numpy.

* ``fib_machine()``: the S-SHARD machine.  Chip ``FibCpu`` is shaped like the reference's Cpu
  chip (main width 67, 20 local lookups -> 11 EF LogUp columns, quotient degree 2;
  cost 119 as in executor/src/artifacts/mips_costs.json "Cpu"): 33 Fibonacci pairs seeded from
  public values plus an ``is_real`` column.  Chip ``FibTable`` carries a preprocessed table
  (so the preprocessed round of `open` is exercised, like Program/Byte in the real machine), is
  ``local_only`` and has a smaller height (so MMCS height injection and mixed-height FRI
  reductions are exercised).
* ``random_matrix()``: S-NTT / S-COMMIT uniform field matrices.

Trace generation is outside the timed span of the reference pipeline (prove.rs:426-497), so this
module is plain numpy.
"""
from __future__ import annotations

import numpy as np

from .machine import (ChipDesc, IS_FIRST, IS_TRANSITION, KIND_BYTE, Lookup, MachineDesc, P,
                      VirtualPairCol, main, main_next, prep, pv)

NUM_PV_ELTS = 176      # ZKM_PROOF_NUM_PV_ELTS (observed), crates/stark/src/air/public_values.rs:11
PROOF_MAX_NUM_PVS = 231  # length of the public value vector, crates/stark/src/types.rs:73
FIB_PAIRS = 33
FIB_WIDTH = 2 * FIB_PAIRS + 1  # 67
FIB_LOOKUPS = 10               # sends; the same tuples are received -> 20 local lookups


def splitmix64(seed: int, n: int) -> np.ndarray:
    """n outputs of SplitMix64 starting at `seed` (uint64)."""
    with np.errstate(over="ignore"):
        x = (np.uint64(seed) + np.arange(1, n + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15))
        z = x
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def random_matrix(height: int, width: int, seed: int = 42) -> np.ndarray:
    """Row-major height x width matrix, column c from SplitMix64(0x5A4B4D00 + c, mixed with seed)."""
    cols = [(splitmix64((0x5A4B4D00 + c) ^ (seed * 0x100000001B3), height) % np.uint64(P)).astype(np.uint32)
            for c in range(width)]
    return np.ascontiguousarray(np.stack(cols, axis=1)) if width else np.zeros((height, 0), np.uint32)


def fib_machine() -> MachineDesc:
    cpu = ChipDesc("FibCpu", prep_width=0, main_width=FIB_WIDTH)
    real = main(FIB_WIDTH - 1)
    for p in range(FIB_PAIRS):
        a, b = main(2 * p), main(2 * p + 1)
        cpu.assert_zero(IS_FIRST * (a - pv(2 * p)))
        cpu.assert_zero(IS_FIRST * (b - pv(2 * p + 1)))
    for p in range(FIB_PAIRS):
        a, b = main(2 * p), main(2 * p + 1)
        cpu.assert_zero(IS_TRANSITION * real * (main_next(2 * p) - b))
        cpu.assert_zero(IS_TRANSITION * real * (main_next(2 * p + 1) - a - b))
    cpu.assert_zero(real * (real - 1))
    cpu.assert_zero(IS_TRANSITION * main_next(FIB_WIDTH - 1) * (1 - real))
    mult = VirtualPairCol.single_main(FIB_WIDTH - 1)
    for j in range(FIB_LOOKUPS):
        vals = [VirtualPairCol.single_main(2 * j), VirtualPairCol.single_main(2 * j + 1),
                VirtualPairCol([("main", 2 * (j + 10), 1), ("main", 2 * (j + 10) + 1, 2)], 7),
                VirtualPairCol.single_main(2 * ((j + 5) % FIB_PAIRS) + 1)]
        if j % 2:
            vals.append(VirtualPairCol.single_main(2 * ((j + 20) % FIB_PAIRS)))
        if j % 3 == 0:
            vals.append(VirtualPairCol.const(j + 1))
        kind = (j % 7) + 1
        cpu.sends.append(Lookup(vals, mult, kind))
        cpu.receives.append(Lookup(list(vals), mult, kind))

    table = ChipDesc("FibTable", prep_width=2, main_width=3, local_only=True)
    table.assert_zero(main(0) - prep(0))
    table.assert_zero(main(1) - prep(1))
    tm = VirtualPairCol.single_main(2)
    table.sends.append(Lookup([VirtualPairCol.single_main(0), VirtualPairCol.single_main(1)], tm, KIND_BYTE))
    table.receives.append(Lookup([VirtualPairCol.single_prep(0), VirtualPairCol.single_prep(1)], tm, KIND_BYTE))
    return MachineDesc([cpu, table], NUM_PV_ELTS)


def _fib_mod_p(n: int) -> np.ndarray:
    """F_{-1}, F_0, ..., F_{n} mod p as uint64 (length n + 2)."""
    B = 4096
    small = [1, 0]  # F_{-1}, F_0
    for _ in range(B + 1):
        small.append((small[-1] + small[-2]) % P)
    fsmall = np.asarray(small, dtype=np.uint64)  # index j+1 -> F_j, j in [-1, B+1]
    out = np.empty(n + 2, dtype=np.uint64)
    # F_{kB + j} = F_{kB} F_{j+1} + F_{kB-1} F_j
    fk, fkm1 = 0, 1  # F_0, F_{-1}
    k = 0
    jj = np.arange(0, B, dtype=np.int64)
    while k * B <= n + 1:
        idx = k * B + jj  # target indices i (F_i), i >= 0
        sel = idx <= n
        i = idx[sel]
        j = jj[sel]
        vals = (np.uint64(fk) * fsmall[j + 2] + np.uint64(fkm1) * fsmall[j + 1]) % np.uint64(P)
        out[i + 1] = vals
        # advance to F_{(k+1)B}, F_{(k+1)B - 1}
        nfk = (fk * int(fsmall[B + 2]) + fkm1 * int(fsmall[B + 1])) % P
        nfkm1 = (fk * int(fsmall[B + 1]) + fkm1 * int(fsmall[B])) % P
        fk, fkm1 = nfk, nfkm1
        k += 1
    out[0] = 1
    return out


def fib_public_values(seed: int = 7) -> np.ndarray:
    return (splitmix64(0xF1B0000 + seed, PROOF_MAX_NUM_PVS) % np.uint64(P)).astype(np.uint32)


def fib_cpu_trace(n: int, pvs: np.ndarray) -> np.ndarray:
    f = _fib_mod_p(n + 1)  # f[i+1] = F_i
    i = np.arange(n)
    fm1, f0, f1 = f[i], f[i + 1], f[i + 2]  # F_{i-1}, F_i, F_{i+1}
    t = np.empty((n, FIB_WIDTH), dtype=np.uint32)
    for p_ in range(FIB_PAIRS):
        a0, b0 = np.uint64(pvs[2 * p_]), np.uint64(pvs[2 * p_ + 1])
        t[:, 2 * p_] = ((fm1 * a0) % np.uint64(P) + (f0 * b0) % np.uint64(P)) % np.uint64(P)
        t[:, 2 * p_ + 1] = ((f0 * a0) % np.uint64(P) + (f1 * b0) % np.uint64(P)) % np.uint64(P)
    real_rows = n - max(1, n // 8)
    t[:, FIB_WIDTH - 1] = (i < real_rows).astype(np.uint32)
    return t


def fib_table_height(n: int) -> int:
    return max(16, n >> 4)


def fib_table_prep(m: int) -> np.ndarray:
    x = np.arange(m, dtype=np.uint64)
    return np.ascontiguousarray(np.stack([x, (x * x) % np.uint64(P)], axis=1).astype(np.uint32))


def fib_table_trace(m: int) -> np.ndarray:
    x = np.arange(m, dtype=np.uint64)
    return np.ascontiguousarray(np.stack([x, (x * x) % np.uint64(P), (x % np.uint64(3))], axis=1).astype(np.uint32))


def fib_shard(n: int, seed: int = 7):
    """(machine, prep_traces_by_chip, shard_traces_by_chip, public_values)."""
    m = fib_machine()
    pvs = fib_public_values(seed)
    th = fib_table_height(n)
    prep_traces = {"FibTable": fib_table_prep(th)}
    traces = {"FibCpu": fib_cpu_trace(n, pvs), "FibTable": fib_table_trace(th)}
    return m, prep_traces, traces, pvs


def deg5_shard(n: int, seed: int = 7):
    """fib_shard plus a degree-5 chip (log_quotient_degree 2, which needs blowup 4): ``Pow5`` proves
    y = x^5 on every row and sends/receives (x, y) as a balanced local lookup; its height is n / 2, so
    the shard mixes quotient degrees 2 and 4 and three trace heights (compressed_fri_config's
    shape of problem, crates/stark/src/kb31_poseidon2.rs:217-227; COMPRESS_DEGREE, prover/src/lib.rs:106)."""
    from .machine import ChipDesc, Lookup, VirtualPairCol, main
    m, prep, traces, pvs = fib_shard(n, seed)
    ch = ChipDesc("Pow5", prep_width=0, main_width=3)
    x, y, real = main(0), main(1), main(2)
    ch.assert_zero(y - x * x * x * x * x)
    ch.assert_zero(real * (real - 1))
    vals = [VirtualPairCol.single_main(0), VirtualPairCol.single_main(1)]
    ch.sends.append(Lookup(vals, VirtualPairCol.single_main(2), 5))
    ch.receives.append(Lookup(list(vals), VirtualPairCol.single_main(2), 5))
    m.chips.append(ch)
    h = max(16, n // 2)
    xs = splitmix64(0xDE65000 + seed, h) % np.uint64(P)
    t = np.zeros((h, 3), np.uint32)
    t[:, 0] = xs
    x2 = xs * xs % np.uint64(P)
    t[:, 1] = x2 * x2 % np.uint64(P) * xs % np.uint64(P)
    t[:, 2] = (np.arange(h) % 4 != 3)
    traces["Pow5"] = t
    return m, prep, traces, pvs
