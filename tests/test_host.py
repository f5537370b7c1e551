"""Host-side checks that need no GPU: the C-ABI library loads and exports every symbol
include/*.h declare (no compute calls), the machine blob round-trips through an independent
parser (the oracle's), and the synthetic workloads satisfy their own AIR."""
import ctypes
import os
import re

import numpy as np
import pytest

from zkmips_amd import workloads as W
from zkmips_amd.machine import P

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    syms = set()
    for h in sorted(os.listdir(os.path.join(ROOT, "include"))):
        if h.endswith(".h"):
            src = open(os.path.join(ROOT, "include", h)).read()
            src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
            syms |= set(re.findall(r"\b(zkm_[a-z0-9_]+)\s*\(", src))
    return sorted(syms)


def test_library_exports_every_declared_symbol():
    path = os.path.join(ROOT, "zkmips_amd", "libzkm_hip.so")
    if not os.path.exists(path):
        pytest.skip("library not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(path)
    syms = declared_symbols()
    assert len(syms) >= 20 and "zkm_cpu_events_to_trace" in syms
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_product_binding_loads():
    from zkmips_amd import _lib
    L = _lib.lib()
    assert L.zkm_setup and L.zkm_open and L.zkm_commit


def test_machine_blob_independent_parse():
    from tests import _oracle as O
    m = W.fib_machine()
    blob = m.blob()
    h = O.lib().orc_api_machine_new(blob, blob.size)
    assert h
    info = np.zeros(7, np.int32)
    for i, c in enumerate(m.chips):
        assert O.lib().orc_api_machine_info(h, i, info) == 0
        assert list(info[:5]) == [c.prep_width, c.main_width, c.perm_width_ef, c.log_quotient_degree,
                                  c.num_constraints]
    cpu = m.chips[0]
    assert cpu.perm_width_ef == 11 and cpu.log_quotient_degree == 1
    # cost 119 = main 67 + 44 perm + 8 quotient, like the reference's Cpu chip (chip.rs:154-163)
    assert cpu.main_width + 4 * cpu.perm_width_ef + 4 * (1 << cpu.log_quotient_degree) == 119
    O.lib().orc_api_machine_free(h)


def test_fib_trace_satisfies_air():
    n = 1 << 12
    pvs = W.fib_public_values(3)
    t = W.fib_cpu_trace(n, pvs).astype(np.int64)
    real = t[:, -1]
    assert real[0] == 1 and real[-1] == 0
    for p_ in range(W.FIB_PAIRS):
        a, b = t[:, 2 * p_], t[:, 2 * p_ + 1]
        assert a[0] == pvs[2 * p_] and b[0] == pvs[2 * p_ + 1]
        assert np.all(((a[1:] - b[:-1]) % P)[real[:-1] == 1] == 0)
        assert np.all(((b[1:] - a[:-1] - b[:-1]) % P)[real[:-1] == 1] == 0)


def test_bench_profile_parser():
    import bench
    d = bench.parse_profile("lde 4 1.5 120.0\nquotient 2 3.0 8.0\n")
    assert d["lde"] == (4, 1.5, 120.0)


def test_quotient_jit_codegen_compiles_for_gfx950():
    """The per-chip quotient kernels zkm_setup JIT-compiles (hiprtc) build without a device."""
    path = os.path.join(ROOT, "zkmips_amd", "libzkm_hip.so")
    if not os.path.exists(path):
        pytest.skip("library not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(path)
    blob = np.frombuffer(W.fib_machine().blob(), np.uint32)
    n = ctypes.c_uint64()
    rc = lib.zkm_quotient_jit_compile(blob.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(blob.size), ctypes.byref(n))
    assert rc == 0 and n.value > 1000
    # a malformed blob is rejected as an argument error, not a crash
    bad = blob.copy()
    bad[1] = 99
    assert lib.zkm_quotient_jit_compile(bad.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(bad.size),
                                        ctypes.byref(n)) == -1


def test_product_poseidon2_host_matches_oracle(tmp_path):
    """The product permutation (p2.cuh: scaled state, 64-bit linear layers, lazy reductions) compiled
    for the host agrees with the oracle's on KAT-style edge states and random states."""
    exe = tmp_path / "p2chk"
    orc = tmp_path / "orc_p2.o"
    import subprocess
    subprocess.check_call(["gcc", "-O2", "-c", os.path.join(ROOT, "oracle", "poseidon2.c"), "-o", str(orc)])
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "--offload-arch=gfx950", "-x", "hip",
                           os.path.join(ROOT, "tools", "check", "p2_host_check.cpp"), "-x", "none", str(orc),
                           "-o", str(exe)])
    out = subprocess.run([str(exe), "40000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "0 mismatches" in out.stdout


def test_host_poseidon2_batch_matches_oracle():
    """libzkm_trace.so's batch permutation (sixteen states per AVX-512 pass, csrc/host/p2_simd.cpp, and the
    one-state code for short tails) against the oracle's permutation, state by state: random states, all-zero
    and all-(P-1) states, counts that are not multiples of 16, and in place."""
    import ctypes
    import numpy as np
    from tests import _oracle as O
    lib = ctypes.CDLL(os.path.join(ROOT, "zkmips_amd", "libzkm_trace.so"))
    f = lib.zkm_host_poseidon2_permute
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
    orc = O.lib()
    P = 0x7f000001
    rng = np.random.default_rng(5)
    a = rng.integers(0, P, size=(16 * 64 + 7, 16), dtype=np.uint32)
    a[0] = 0
    a[1] = P - 1
    a[17] = np.arange(16)
    out = np.empty_like(a)
    f(a.ctypes.data, out.ctypes.data, len(a))
    for i in range(len(a)):
        st = (ctypes.c_uint32 * 16)(*[int(x) for x in a[i]])
        orc.orc_p2_permute(st)
        assert list(st) == [int(x) for x in out[i]], i
    for n in (50, 3):  # a short tail (one-state code after the batches), and no full batch at all
        o2 = np.empty((n, 16), np.uint32)
        f(np.ascontiguousarray(a[:n]).ctypes.data, o2.ctypes.data, n)
        assert np.array_equal(o2, out[:n]), n
    b = a.copy()
    f(b.ctypes.data, b.ctypes.data, len(b))
    assert np.array_equal(b, out)
