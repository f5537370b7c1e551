"""GPU kernel parity (through the C ABI) against the CPU oracle: bit-exact.

Poseidon2 batch vs the reference KATs, coset LDE vs the oracle's textbook DFT (every height the
multi-pass NTT plans differently), PCS commit roots (LDE + MMCS, mixed heights = injection) vs the
oracle.  Full-size properties: LDE linearity, the LDE restricted to even rows re-interpolates to
the same polynomial (low-degree check).
"""
import json
import os

import numpy as np
import pytest

from tests import _oracle as O
from zkmips_amd import workloads as W
from zkmips_amd.machine import P

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(__file__)


@pytest.fixture(scope="module")
def dev():
    from zkmips_amd._lib import Device
    d = Device(0)
    yield d
    d.close()


def test_poseidon2_batch_kat(dev):
    kat = json.load(open(os.path.join(HERE, "golden", "poseidon2_kat.json")))
    ins = np.asarray([v["input"] for v in kat.values()], np.uint32)
    outs = dev.poseidon2_permute(ins)
    assert outs.tolist() == [v["output"] for v in kat.values()]


def test_poseidon2_batch_vs_oracle(dev):
    st = W.random_matrix(4096, 16, seed=11)
    out = dev.poseidon2_permute(st)
    for i in [0, 1, 2, 777, 4095]:
        assert np.array_equal(out[i], O.permute(st[i]))


@pytest.mark.parametrize("logn", [1, 2, 4, 7, 11, 12, 13, 14, 15, 16, 17, 18, 19])
def test_coset_lde_vs_oracle(dev, logn):
    n = 1 << logn
    w = 3 if logn < 16 else 2
    m = W.random_matrix(n, w, seed=logn)
    got = dev.coset_lde(m, 3)
    exp = O.lde(m, 1, 3)
    assert np.array_equal(got, exp)


@pytest.mark.parametrize("logn,w", [(20, 2), (21, 2), (22, 1), (22, 3), (23, 1), (23, 2)])
def test_coset_lde_large_vs_oracle(dev, logn, w):
    m = W.random_matrix(1 << logn, w, seed=logn)
    assert np.array_equal(dev.coset_lde(m, 3), O.lde(m, 1, 3))


@pytest.mark.parametrize("logn", [3, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 23])
def test_coset_lde_bitrev_input(dev, logn):
    """The quotient-chunk pipeline: evaluations handed over in bit-reversed row order."""
    n = 1 << logn
    m = W.random_matrix(n, 3, seed=100 + logn)
    idx = np.asarray([int(format(i, f"0{logn}b")[::-1], 2) for i in range(n)]) if logn <= 14 else None
    if idx is None:
        r = np.arange(n, dtype=np.uint64)
        idx = np.zeros(n, np.uint64)
        for b in range(logn):
            idx |= ((r >> np.uint64(b)) & np.uint64(1)) << np.uint64(logn - 1 - b)
    shift = pow(3, (P - 1) >> (logn + 1), P)
    got = dev.coset_lde(m[idx], shift, bitrev_in=True)
    assert np.array_equal(got, O.lde(m, 1, shift))


def test_coset_lde_other_shift(dev):
    m = W.random_matrix(1 << 13, 4, seed=5)
    shift = pow(3, (P - 1) >> 14, P)  # quotient-chunk style shift w_2N^-1 analogue
    assert np.array_equal(dev.coset_lde(m, shift), O.lde(m, 1, shift))


def test_coset_lde_linearity_large(dev):
    n = 1 << 20
    a = W.random_matrix(n, 1, seed=1)
    b = W.random_matrix(n, 1, seed=2)
    s = ((a.astype(np.uint64) + b) % P).astype(np.uint32)
    la, lb, ls = dev.coset_lde(a), dev.coset_lde(b), dev.coset_lde(s)
    assert np.array_equal(ls, ((la.astype(np.uint64) + lb) % P).astype(np.uint32))
    # low coset (first n bit-reversed rows) re-interpolates: the LDE of a constant column is constant
    c = np.full((n, 1), 12345, np.uint32)
    assert np.all(dev.coset_lde(c) == 12345)


@pytest.mark.parametrize("logn,w", [(4, 67), (10, 67), (14, 9), (20, 67)])
def test_pcs_commit_root_vs_oracle(dev, logn, w):
    """(20, 67) is BASELINE configuration 2 (S-COMMIT: a 2^20 x 67 trace, LDE + Poseidon2 MMCS root)."""
    m = W.random_matrix(1 << logn, w, seed=logn + w)
    assert np.array_equal(dev.pcs_commit_root([m]), O.commit_root([m]))


def test_pcs_commit_mixed_heights(dev):
    mats = [W.random_matrix(1 << 10, 5, 1), W.random_matrix(1 << 6, 9, 2), W.random_matrix(1 << 10, 3, 3),
            W.random_matrix(1 << 4, 1, 4), W.random_matrix(1 << 6, 0, 5)]
    assert np.array_equal(dev.pcs_commit_root(mats), O.commit_root(mats))
