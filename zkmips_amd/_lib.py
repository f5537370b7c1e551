"""ctypes binding of libzkm_hip.so (include/zkm_hip.h).

The product path has no fallback: if the HIP library is missing or cannot initialise a gfx950
device, every call raises.  Build it with ``python -c "import __graft_entry__ as g; g.build()"``.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ZKM_LIB") or os.path.join(HERE, "libzkm_hip.so")  # ZKM_LIB: A/B of a second build

ZKM_OK = 0
ZKM_REPR_CANONICAL, ZKM_REPR_MONTGOMERY = 0, 1
ZKM_MEM_DEVICE = 0x100  # zkm_matrix_t.repr flag: data is GPU-resident


class ZkmError(RuntimeError):
    pass


class Matrix(C.Structure):
    _fields_ = [("name", C.c_char_p), ("data", C.c_void_p), ("height", C.c_uint64), ("width", C.c_uint64),
                ("repr", C.c_uint32)]


class Config(C.Structure):
    _fields_ = [("num_queries", C.c_uint32), ("pow_bits", C.c_uint32), ("log_blowup", C.c_uint32),
                ("proof_montgomery", C.c_uint32)]


class ChallengerState(C.Structure):
    _fields_ = [("sponge_state", C.c_uint32 * 16), ("num_inputs", C.c_uint32), ("input_buffer", C.c_uint32 * 8),
                ("num_outputs", C.c_uint32), ("output_buffer", C.c_uint32 * 8)]

    def to_words(self) -> np.ndarray:
        return np.frombuffer(bytes(self), dtype=np.uint32).copy()

    @staticmethod
    def from_words(w) -> "ChallengerState":
        return ChallengerState.from_buffer_copy(np.ascontiguousarray(w, dtype=np.uint32).tobytes())


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ZkmError(f"{LIB_PATH} not built: run __graft_entry__.build()")
    L = C.CDLL(LIB_PATH)
    vp, u32p = C.c_void_p, C.POINTER(C.c_uint32)
    L.zkm_last_error.restype = C.c_char_p
    L.zkm_init.argtypes = [C.c_int, C.POINTER(vp)]
    L.zkm_destroy.argtypes = [vp]
    L.zkm_device_count.restype = C.c_int
    L.zkm_coset_lde.argtypes = [vp, C.POINTER(Matrix), C.c_uint32, vp]
    L.zkm_coset_lde_ex.argtypes = [vp, C.POINTER(Matrix), C.c_uint32, C.c_int, vp]
    L.zkm_poseidon2_permute.argtypes = [vp, vp, C.c_uint64]
    L.zkm_pcs_commit_root.argtypes = [vp, C.POINTER(Matrix), C.c_uint32, vp]
    L.zkm_bench_lde.argtypes = [vp, C.c_uint64, C.c_uint64, C.c_int, C.POINTER(C.c_double)]
    L.zkm_host_alloc.argtypes = [C.c_size_t, C.POINTER(vp)]
    L.zkm_host_free.argtypes = [vp]
    if hasattr(L, "zkm_setup"):
        L.zkm_setup.argtypes = [vp, vp, C.c_size_t, C.POINTER(Config), C.POINTER(Matrix), C.c_uint32, C.c_uint32,
                                vp, C.POINTER(vp), vp]
        L.zkm_pk_free.argtypes = [vp]
        L.zkm_pk_observe.argtypes = [vp, C.POINTER(ChallengerState)]
        L.zkm_commit.argtypes = [vp, vp, C.POINTER(Matrix), C.c_uint32, vp, C.c_uint32, C.POINTER(vp), vp]
        L.zkm_main_free.argtypes = [vp]
        L.zkm_machine_new.argtypes = [vp, C.c_size_t, C.POINTER(Config), C.POINTER(vp)]
        L.zkm_machine_free.argtypes = [vp]
        L.zkm_commit_machine.argtypes = [vp, vp, C.POINTER(Matrix), C.c_uint32, vp, C.c_uint32, C.POINTER(vp), vp]
        L.zkm_open.argtypes = [vp, vp, vp, C.POINTER(ChallengerState), C.POINTER(C.POINTER(C.c_uint8)),
                               C.POINTER(C.c_uint64)]
        L.zkm_prove_shard.argtypes = [vp, vp, C.POINTER(Matrix), C.c_uint32, vp, C.c_uint32,
                                      C.POINTER(ChallengerState), C.POINTER(C.POINTER(C.c_uint8)),
                                      C.POINTER(C.c_uint64)]
        L.zkm_free_bytes.argtypes = [C.POINTER(C.c_uint8)]
    _lib = L
    return L


def check(rc: int, what: str):
    if rc != ZKM_OK:
        msg = lib().zkm_last_error()
        raise ZkmError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


def as_u32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.uint32)


def matrix(arr: np.ndarray, name: str = "", montgomery: bool = False, keep: list = None) -> Matrix:
    a = as_u32(arr)
    if a.ndim == 1:
        a = a.reshape(-1, 1)
    if keep is not None:
        keep.append(a)
    nm = name.encode()
    if keep is not None:
        keep.append(nm)
    return Matrix(nm, a.ctypes.data if a.size else None, a.shape[0], a.shape[1],
                  ZKM_REPR_MONTGOMERY if montgomery else ZKM_REPR_CANONICAL)


class PinnedArray:
    """A numpy u32 array in page-locked host memory (zkm_host_alloc): traces written here cross PCIe
    by asynchronous DMA, overlapped with kernels.  Keep the object alive while the array is used."""

    def __init__(self, shape):
        n = int(np.prod(shape))
        self.p = C.c_void_p()
        check(lib().zkm_host_alloc(max(4, n * 4), C.byref(self.p)), "zkm_host_alloc")
        self.array = np.ctypeslib.as_array(C.cast(self.p, C.POINTER(C.c_uint32)), shape=(max(1, n),))[:n].reshape(shape)

    def __del__(self):
        if getattr(self, "p", None):
            self.array = None
            lib().zkm_host_free(self.p)
            self.p = None


def pinned_copy(a: np.ndarray) -> PinnedArray:
    b = PinnedArray(a.shape)
    np.copyto(b.array, as_u32(a))
    return b


class Device:
    """One zkm_ctx (a GPU).  Mirrors the reference's per-GPU prover context."""

    def __init__(self, device: int = 0):
        self.h = C.c_void_p()
        check(lib().zkm_init(device, C.byref(self.h)), f"zkm_init({device})")
        self.device = device

    def close(self):
        if self.h:
            lib().zkm_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- kernel-level helpers ----
    def coset_lde(self, m: np.ndarray, shift: int = 3, bitrev_in: bool = False) -> np.ndarray:
        keep = []
        mm = matrix(m, keep=keep)
        out = np.zeros((2 * mm.height, mm.width), np.uint32)
        check(lib().zkm_coset_lde_ex(self.h, C.byref(mm), shift, int(bitrev_in), out.ctypes.data), "zkm_coset_lde")
        return out

    def poseidon2_permute(self, states: np.ndarray) -> np.ndarray:
        s = as_u32(states).reshape(-1, 16).copy()
        check(lib().zkm_poseidon2_permute(self.h, s.ctypes.data, s.shape[0]), "zkm_poseidon2_permute")
        return s

    def pcs_commit_root(self, mats) -> np.ndarray:
        keep = []
        arr = (Matrix * len(mats))(*[matrix(m, keep=keep) for m in mats])
        out = np.zeros(8, np.uint32)
        check(lib().zkm_pcs_commit_root(self.h, arr, len(mats), out.ctypes.data), "zkm_pcs_commit_root")
        return out

    def bench_lde(self, h: int, w: int, iters: int = 5) -> float:
        ms = C.c_double()
        check(lib().zkm_bench_lde(self.h, h, w, iters, C.byref(ms)), "zkm_bench_lde")
        return ms.value


def _compile_blob(blob) -> int:
    """Worker of prefill_jit_cache: compile one single-chip machine blob into the code-object cache."""
    n = C.c_uint64(0)
    blob = np.ascontiguousarray(blob, np.uint32)
    rc = lib().zkm_quotient_jit_compile(blob.ctypes.data_as(C.c_void_p), C.c_size_t(blob.size), C.byref(n))
    if rc != 0:
        raise ZkmError(f"quotient JIT compile failed ({rc}): {lib().zkm_last_error().decode()}")
    return n.value


def prefill_jit_cache(machines, prune: bool = False, workers: int = None) -> int:
    """Compile every chip's quotient/permutation kernels of `machines` for gfx950 into the JIT's on-disk
    code-object cache (zkmips_amd/jit_cache, see csrc/jit.cpp); no device needed.  hiprtc serialises
    compiles inside one process, so the distinct chips (one single-chip machine blob each, largest first)
    compile in a pool of processes.  With `prune` (opt-in: only the build step, which prefills every
    shipped machine while nothing else runs, passes it), code objects of the default cache directory that
    none of these machines uses (older kernel sources, other machines) are deleted.  Returns code bytes."""
    import concurrent.futures as cf
    import multiprocessing as mp
    import time
    from .machine import MAGIC, VERSION
    blobs, seen = [], set()
    for m in machines:
        for c in m.chips:
            w = c.words()
            key = (c.name, m.num_pv, hash(tuple(w)))
            if key not in seen:
                seen.add(key)
                blobs.append(np.asarray([MAGIC, VERSION, m.num_pv, 1] + list(w), np.uint32))
    blobs.sort(key=lambda b: -b.size)
    cache = os.path.join(os.path.dirname(os.path.abspath(__file__)), "jit_cache")
    prune = prune and "ZKM_JIT_CACHE" not in os.environ and os.path.isdir(cache)
    t0 = time.time() - 1.0
    if prune:
        os.environ["ZKM_JIT_TOUCH"] = "1"  # cache hits refresh their file's mtime (the workers inherit it)
    try:
        n = workers or max(1, min(len(blobs), os.cpu_count() or 1, 16))
        with cf.ProcessPoolExecutor(n, mp_context=mp.get_context("spawn")) as ex:
            total = sum(ex.map(_compile_blob, blobs))
    finally:
        if prune:
            del os.environ["ZKM_JIT_TOUCH"]
    if prune:
        for f in os.listdir(cache):
            path = os.path.join(cache, f)
            if f.endswith(".co") and os.path.getmtime(path) < t0:
                os.remove(path)
    return total

