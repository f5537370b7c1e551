"""Shared subexpressions in the machine blob (OP_LET / OP_GET, include/zkm_hip.h): a chip's constraint
program stays linear in the size of its symbolic DAG, as the reference's get_symbolic_constraints
output is a DAG of Rc-shared SymbolicExpression nodes (machine.rs:357-362).

* Poseidon2WideDeg3 written with chained round layers (no hand-folded linear forms) and the Global
  chip's septic arithmetic both lower to blobs smaller than before (21,864 -> ~11k and 20,384 -> ~6k
  words);
* the shared program evaluates to the same constraint values as the expanded one;
* proofs through the oracle (CPU) and, on the GPU, through the JIT and through the interpreter kernel
  (ZKM_NO_JIT=1, slots in global scratch) are byte-identical to the oracle's."""
import numpy as np
import pytest

from tests import _air_check as AC
from tests import _oracle as O
from zkmips_amd import machine as M
from zkmips_amd import mips_memory as MM
from zkmips_amd import recursion as R


def _expand(code):
    """The builder code with every shared reference replaced by its definition (no sharing)."""
    out, i = [], 0
    while i < len(code):
        op = code[i]
        if op == M.OP_REF:
            out += _expand(M._SHARED[code[i + 1]])
            i += 2
        elif op in M._OPERAND_OPS:
            out += code[i:i + 2]
            i += 2
        else:
            out.append(op)
            i += 1
    return out


def _expanded_len(code, memo):
    """len(_expand(code)), counted without building it (the expansion is exponential in depth)."""
    n, i = 0, 0
    while i < len(code):
        op = code[i]
        if op == M.OP_REF:
            g = code[i + 1]
            if g not in memo:
                memo[g] = _expanded_len(M._SHARED[g], memo)
            n += memo[g]
            i += 2
        elif op in M._OPERAND_OPS:
            n += 2
            i += 2
        else:
            n += 1
            i += 1
    return n


def test_program_defines_slots_in_order():
    c = M.ChipDesc("T", 0, 3)
    a = (M.main(0) + M.main(1)).share()
    b = (a * a + M.main(2)).share()
    c.assert_zero(b * a - M.main(2))
    c.assert_zero(b - 5)
    p = c.program()
    lets = [p[i + 1] for i in range(len(p) - 1) if p[i] == M.OP_LET]
    assert lets == [0, 1]
    # leaves are not shared
    assert M.main(4).share().code == M.main(4).code
    # the values equal the expanded expressions
    rng = np.random.default_rng(1)
    tr = rng.integers(0, M.P, (16, 3)).astype(np.uint32)
    for con in c.constraints:
        v1 = AC._eval(con.code, tr, np.zeros((16, 0), np.uint32), np.zeros(4, np.uint32), 16)
        v2 = AC._eval(_expand(con.code), tr, np.zeros((16, 0), np.uint32), np.zeros(4, np.uint32), 16)
        assert np.array_equal(v1, v2)


def test_dag_chips_are_compact():
    p2 = R.poseidon2_wide_chip()
    assert len(p2.words()) < 12000
    assert sum(1 for i in range(len(p2.program()) - 1) if p2.program()[i] == M.OP_LET) > 500
    g = MM.global_chip()
    assert len(g.words()) < 6500
    # the expansion of the chained layers is far larger: the blob would not be linear without sharing
    memo = {}
    assert sum(_expanded_len(c.code, memo) for c in p2.constraints) > 5 * len(p2.words())


def test_poseidon2_chained_layers_satisfied_by_trace():
    """The chained-layer constraints vanish on real permutation rows (and fail on a corrupted one)."""
    rng = np.random.default_rng(5)
    rows = R.poseidon2_rows(rng.integers(0, M.P, (16, 16)).astype(np.uint32))
    ch = R.poseidon2_wide_chip()
    prep = np.zeros((16, ch.prep_width), np.uint32)
    pv = np.zeros(R.PROOF_MAX_NUM_PVS if hasattr(R, "PROOF_MAX_NUM_PVS") else 231, np.uint32)
    memo = {}
    for con in ch.constraints:
        assert not np.any(AC._eval(con.code, rows, prep, pv, 16, memo))
    bad = rows.copy()
    bad[3, R.P2_ESBOX + 5] = (int(bad[3, R.P2_ESBOX + 5]) + 1) % M.P
    memo = {}
    assert any(np.any(AC._eval(con.code, bad, prep, pv, 16, memo)) for con in ch.constraints)


@pytest.mark.gpu
@pytest.mark.parametrize("no_jit", ["0", "1"])
def test_gpu_shared_programs_identical(no_jit, monkeypatch):
    """A compress shard (Poseidon2 chained layers) and a MIPS core shard (Global septic DAG) prove to the
    oracle's bytes through the JIT and through the interpreter (slots in global scratch)."""
    from zkmips_amd import mips_core as MC
    from zkmips_amd._lib import Device
    from zkmips_amd.prover import HipProver
    monkeypatch.setenv("ZKM_NO_JIT", no_jit)
    dev = Device(0)
    m, prep, tr, pv = R.shard(R.program_merkle_openings(6, 21, 8)[0])
    kw = dict(num_queries=R.COMPRESS_NUM_QUERIES, log_blowup=R.COMPRESS_LOG_BLOWUP)
    gpu = HipProver(dev, m, prep, **kw).prove_shard(tr, pv)
    rc, ref = O.OracleProver(m, prep, **kw).prove(tr, pv)
    assert rc == 0 and gpu == ref
    m, prep, tr, pv = MC.core_shard(200, seed=2)
    gpu = HipProver(dev, m, prep, num_queries=16).prove_shard(tr, pv)
    rc, ref = O.OracleProver(m, prep, num_queries=16).prove(tr, pv)
    assert rc == 0 and gpu == ref
