"""ctypes wrapper for the CPU oracle (oracle/liboracle.so) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "oracle", "liboracle.so")
CHAL_WORDS = 34

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        L = C.CDLL(LIB_PATH)
        u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
        L.orc_api_p2_permute.argtypes = [u32p]
        L.orc_api_hash.argtypes = [u32p, C.c_uint64, u32p]
        L.orc_api_compress.argtypes = [u32p, u32p, u32p]
        L.orc_api_lde.argtypes = [u32p, C.c_uint64, C.c_uint64, C.c_int, C.c_uint32, u32p]
        L.orc_api_dft.argtypes = [u32p, C.c_int, C.c_int]
        L.orc_api_merkle_root.argtypes = [C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), u32p]
        L.orc_api_commit_root.argtypes = [C.c_int, C.POINTER(C.c_void_p), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), u32p]
        L.orc_api_chal_observe.argtypes = [u32p, u32p, C.c_uint64]
        L.orc_api_chal_sample.argtypes = [u32p, u32p, C.c_uint64]
        L.orc_api_chal_grind.argtypes = [u32p, C.c_int]
        L.orc_api_chal_grind.restype = C.c_uint32
        L.orc_api_machine_new.argtypes = [u32p, C.c_uint64]
        L.orc_api_machine_new.restype = C.c_void_p
        L.orc_api_machine_free.argtypes = [C.c_void_p]
        L.orc_api_machine_info.argtypes = [C.c_void_p, C.c_int, np.ctypeslib.ndpointer(np.int32)]
        L.orc_api_setup.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p),
                                    C.POINTER(C.c_uint64), C.c_uint32, u32p, u32p, C.c_int]
        L.orc_api_setup.restype = C.c_void_p
        L.orc_api_pk_free.argtypes = [C.c_void_p]
        L.orc_api_pk_observe.argtypes = [C.c_void_p, u32p]
        L.orc_api_prove.argtypes = [C.c_void_p, C.c_int, np.ctypeslib.ndpointer(np.int32), C.POINTER(C.c_void_p),
                                    C.POINTER(C.c_uint64), u32p, C.c_int, u32p,
                                    C.POINTER(C.POINTER(C.c_uint8)), C.POINTER(C.c_uint64)]
        L.orc_api_verify.argtypes = [C.c_void_p, C.c_char_p, C.c_uint64, u32p]
        L.orc_api_free_bytes.argtypes = [C.POINTER(C.c_uint8)]
        L.orc_serialize_digest_map.argtypes = [u32p, np.ctypeslib.ndpointer(np.uint64), C.c_uint64, C.c_int,
                                               C.POINTER(C.POINTER(C.c_uint8))]
        L.orc_serialize_digest_map.restype = C.c_size_t
        _lib = L
    return _lib


def _u32(a):
    return np.ascontiguousarray(a, dtype=np.uint32)


def permute(state):
    s = _u32(state).copy()
    lib().orc_api_p2_permute(s)
    return s


def hash_(values):
    out = np.zeros(8, np.uint32)
    v = _u32(values)
    lib().orc_api_hash(v if v.size else np.zeros(1, np.uint32), v.size, out)
    return out


def compress(l, r):
    out = np.zeros(8, np.uint32)
    lib().orc_api_compress(_u32(l), _u32(r), out)
    return out


def dft(a, inverse=False):
    x = _u32(a).copy()
    lib().orc_api_dft(x, int(np.log2(x.size)), int(inverse))
    return x


def lde(evals, log_blowup=1, shift=3):
    e = _u32(evals)
    h, w = e.shape
    out = np.zeros((h << log_blowup, w), np.uint32)
    lib().orc_api_lde(e, h, w, log_blowup, shift, out)
    return out


def _ptrs(mats):
    arr = (C.c_void_p * len(mats))(*[m.ctypes.data for m in mats])
    return arr


def merkle_root(mats):
    mats = [_u32(m) for m in mats]
    hs = (C.c_uint64 * len(mats))(*[m.shape[0] for m in mats])
    ws = (C.c_uint64 * len(mats))(*[m.shape[1] for m in mats])
    out = np.zeros(8, np.uint32)
    lib().orc_api_merkle_root(len(mats), _ptrs(mats), hs, ws, out)
    return out


def commit_root(mats):
    """LDE (blowup 2, shift 3) + bit-reverse + MMCS root: TwoAdicFriPcs::commit for trace domains."""
    mats = [_u32(m) for m in mats]
    hs = (C.c_uint64 * len(mats))(*[m.shape[0] for m in mats])
    ws = (C.c_uint64 * len(mats))(*[m.shape[1] for m in mats])
    out = np.zeros(8, np.uint32)
    lib().orc_api_commit_root(len(mats), _ptrs(mats), hs, ws, out)
    return out


def serialize_digest_map(keys, vals, montgomery=False) -> bytes:
    """bincode of BTreeMap<[F;8], usize> with the proof serializer's conventions (oracle/serialize.c)."""
    k = _u32(keys).reshape(-1, 8)
    v = np.ascontiguousarray(vals, dtype=np.uint64)
    out = C.POINTER(C.c_uint8)()
    n = lib().orc_serialize_digest_map(k if k.size else np.zeros(8, np.uint32), v if v.size else np.zeros(1, np.uint64),
                                       k.shape[0], int(montgomery), C.byref(out))
    data = bytes(C.string_at(out, n))
    lib().orc_api_free_bytes(out)
    return data


class Challenger:
    def __init__(self, state=None):
        self.s = np.zeros(CHAL_WORDS, np.uint32) if state is None else _u32(state).copy()

    def observe(self, vals):
        v = _u32(np.atleast_1d(vals))
        lib().orc_api_chal_observe(self.s, v, v.size)

    def sample(self, n=1):
        out = np.zeros(n, np.uint32)
        lib().orc_api_chal_sample(self.s, out, n)
        return out

    def grind(self, bits):
        return lib().orc_api_chal_grind(self.s, bits)

    def copy(self):
        return Challenger(self.s)


class OracleProver:
    """CPU restatement of CpuProver (setup + commit/open) and the shard verifier."""

    def __init__(self, machine, prep_traces, num_queries=84, pow_bits=16, montgomery=False,
                 pc_start=None, gcs=None, log_blowup=1):
        from zkmips_amd.machine import P  # noqa
        self.machine = machine
        self.blob = machine.blob()
        self.mh = lib().orc_api_machine_new(self.blob, self.blob.size)
        assert self.mh, "machine parse failed"
        self._keep = []
        ptrs = (C.c_void_p * len(machine.chips))()
        hs = (C.c_uint64 * len(machine.chips))()
        for i, c in enumerate(machine.chips):
            if c.name in prep_traces:
                t = _u32(prep_traces[c.name])
                self._keep.append(t)
                ptrs[i] = t.ctypes.data
                hs[i] = t.shape[0]
        if gcs is None:
            gcs = np.asarray([637514027, 1595065213, 1998064738, 72333738, 1211544370, 822986770, 1518535784,
                              1604177449, 90440090, 259343427, 140470264, 1162099742, 941559812, 1064053343], np.uint32)
        self.commit = np.zeros(8, np.uint32)
        if pc_start is None:  # the machine's programs' entry (MachineDesc.pc_start)
            pc_start = getattr(machine, "pc_start", 0x00400000)
        self.pk = lib().orc_api_setup(self.mh, num_queries, pow_bits, int(montgomery), ptrs, hs, pc_start, _u32(gcs),
                                      self.commit, log_blowup)
        assert self.pk, "setup failed"

    def base_challenger(self):
        ch = Challenger()
        lib().orc_api_pk_observe(self.pk, ch.s)
        return ch

    def prove(self, traces: dict, public_values, challenger=None):
        ch = challenger or self.base_challenger()
        names = list(traces)
        idx = np.asarray([self.machine.chip_index(n) for n in names], np.int32)
        mats = [_u32(traces[n]) for n in names]
        hs = (C.c_uint64 * len(mats))(*[m.shape[0] for m in mats])
        out = C.POINTER(C.c_uint8)()
        ln = C.c_uint64()
        pvs = _u32(public_values)
        rc = lib().orc_api_prove(self.pk, len(mats), idx, _ptrs(mats), hs, pvs, pvs.size, ch.s, C.byref(out), C.byref(ln))
        data = bytes(C.string_at(out, ln.value)) if ln.value else b""
        if ln.value:
            lib().orc_api_free_bytes(out)
        return rc, data

    def verify(self, proof: bytes, challenger=None):
        ch = challenger or self.base_challenger()
        return lib().orc_api_verify(self.pk, proof, len(proof), ch.s)

    def __del__(self):
        try:
            lib().orc_api_pk_free(self.pk)
            lib().orc_api_machine_free(self.mh)
        except Exception:
            pass
