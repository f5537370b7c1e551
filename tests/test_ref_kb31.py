"""The reference's own KoalaBear host type (crates/core/machine/include/kb31_t.hpp, compiled from the
reference's source into oracle/_ref/libkb31_ref.so by `make -C oracle ref`) pins:

* the field: add / sub / mul / reciprocal / x^(2^k) over p = 2^31 - 2^24 + 1 equal plain modular
  arithmetic (which is what the oracle and the GPU kernels restate);
* the Montgomery encoding of the reference's in-memory values (R = 2^32): the form that
  `RowMajorMatrix<KoalaBear>` traces cross the C ABI in (ZKM_REPR_MONTGOMERY, core/machine/cpp/
  extern.cpp:6-37); on the GPU, traces encoded by the reference's own conversion prove to the same
  bytes as the canonical traces.

Skipped when the library is absent (it is built only where /root/reference exists; the .so travels
to the GPU box prebuilt)."""
import ctypes as C
import os

import numpy as np
import pytest

P = 0x7F000001
LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref", "libkb31_ref.so")
pytestmark = pytest.mark.skipif(not os.path.exists(LIB), reason="oracle/_ref/libkb31_ref.so not built")


def _lib():
    L = C.CDLL(LIB)
    u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
    L.ref_kb31_to_monty.argtypes = [u32p, u32p, C.c_uint64]
    L.ref_kb31_from_monty.argtypes = [u32p, u32p, C.c_uint64]
    L.ref_kb31_binop.argtypes = [C.c_int, u32p, u32p, u32p, C.c_uint64]
    return L


def ref_to_monty(x):
    x = np.ascontiguousarray(x, np.uint32)
    out = np.empty_like(x)
    _lib().ref_kb31_to_monty(x.reshape(-1), out.reshape(-1), x.size)
    return out


def _binop(op, a, b):
    out = np.empty_like(a)
    _lib().ref_kb31_binop(op, a, b, out, a.size)
    return out


def test_field_ops_equal_modular_arithmetic():
    rng = np.random.default_rng(3)
    a = rng.integers(0, P, 4096, dtype=np.uint64)
    b = rng.integers(0, P, 4096, dtype=np.uint64)
    a[:6] = [0, 1, P - 1, 2, P - 2, 1 << 30]
    b[:6] = [0, P - 1, P - 1, 1, 3, 1 << 24]
    a32, b32 = a.astype(np.uint32), b.astype(np.uint32)
    assert np.array_equal(_binop(0, a32, b32), ((a + b) % P).astype(np.uint32))
    assert np.array_equal(_binop(1, a32, b32), ((a + P - b) % P).astype(np.uint32))
    assert np.array_equal(_binop(2, a32, b32), ((a * b) % P).astype(np.uint32))
    nz = a32[a32 != 0]
    inv = _binop(3, nz, nz)
    assert np.all((inv.astype(np.uint64) * nz.astype(np.uint64)) % P == 1)
    k = (b32 % 40).astype(np.uint32)
    want = np.array([pow(int(x), 1 << int(e), P) for x, e in zip(a32[:512], k[:512])], np.uint32)
    assert np.array_equal(_binop(4, a32[:512], k[:512]), want)


def test_montgomery_encoding_is_r_2_32():
    rng = np.random.default_rng(4)
    x = rng.integers(0, P, 4096, dtype=np.uint64)
    x[:3] = [0, 1, P - 1]
    m = ref_to_monty(x.astype(np.uint32))
    assert np.array_equal(m, ((x << np.uint64(32)) % P).astype(np.uint32))
    back = np.empty_like(m)
    _lib().ref_kb31_from_monty(m, back, m.size)
    assert np.array_equal(back, x.astype(np.uint32))
    # the reference's ONE constant (kb31_t.hpp:29) is R mod p
    assert int(ref_to_monty(np.array([1], np.uint32))[0]) == 0x1FFFFFE


@pytest.mark.gpu
def test_reference_montgomery_traces_prove_identically():
    """A shard handed over in the reference's in-memory form (converted by its own kb31_t) proves to the
    same bytes as the canonical shard, and equals the oracle's."""
    from tests import _oracle as O
    from zkmips_amd import workloads as W
    from zkmips_amd._lib import Device
    from zkmips_amd.prover import HipProver
    m, prep, tr, pv = W.fib_shard(1 << 12, 5)
    hp = HipProver(Device(0), m, prep, num_queries=16)
    canon = hp.prove_shard(tr, pv)
    ch = hp.base_challenger()
    data = hp.commit({k: ref_to_monty(v) for k, v in tr.items()}, pv, montgomery_input=True)
    mont = hp.open(data, ch)
    rc, ref = O.OracleProver(m, prep, num_queries=16).prove(tr, pv)
    assert rc == 0 and canon == mont == ref
