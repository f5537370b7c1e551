"""Septic-curve helpers for the Global chip's trace (ctypes over libzkm_trace.so, host C++:
zkmips_amd/csrc/host/septic.cpp).

The curve is y^2 = x^3 + 3z x - 3 over F_{p^7} = F_p[z]/(z^7 + 2z - 8) (crates/stark/src/septic_curve.rs,
septic_extension.rs); points are 14 canonical words (x[7], y[7]).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libzkm_trace.so")

# crates/stark/src/septic_digest.rs:8-22, septic_curve.rs:17-24
CURVE_CUMULATIVE_SUM_START = np.asarray([637514027, 1595065213, 1998064738, 72333738, 1211544370, 822986770,
                                         1518535784, 1604177449, 90440090, 259343427, 140470264, 1162099742,
                                         941559812, 1064053343], np.uint32)
DIGEST_SUM_START = np.asarray([1656788302, 897965284, 874620737, 1581672598, 655804282, 1962911564, 80580607,
                               1024875409, 218609128, 1856341123, 583920580, 1274441611, 118766316, 81843042],
                              np.uint32)
CURVE_WITNESS_DUMMY_POINT = np.asarray([1706420302, 1319108093, 148224806, 26874985, 1766171812, 1645633948,
                                        2028659224, 942390502, 1239997438, 458866455, 1843332012, 1309764648,
                                        572807436, 74267719], np.uint32)

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} not built: run __graft_entry__.build()")
        L = C.CDLL(LIB_PATH)
        u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
        u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
        L.zkm_septic_lift.argtypes = [u32p, u32p, u8p, C.c_uint64, u32p, u32p]
        L.zkm_septic_cumsum.argtypes = [u32p, u32p, C.c_uint64, u32p]
        L.zkm_septic_mul.argtypes = [u32p, u32p, u32p]
        L.zkm_septic_frobenius_col.argtypes = [C.c_int, u32p]
        L.zkm_septic_on_curve.argtypes = [u32p]
        L.zkm_septic_sum_checker_x.argtypes = [u32p, u32p, u32p, u32p]
        L.zkm_septic_digest_sum.argtypes = [u32p, C.c_uint64, u32p, u32p, u32p]
        _lib = L
    return _lib


def _u32(a):
    return np.ascontiguousarray(a, dtype=np.uint32)


def lift(messages: np.ndarray, kinds: np.ndarray, is_receive: np.ndarray):
    """GlobalLookupOperation::get_digest per message (global_lookup.rs:26-38): (points n x 14, offsets n)."""
    m = _u32(messages).reshape(-1, 7)
    n = m.shape[0]
    xy = np.zeros((max(n, 1), 14), np.uint32)
    off = np.zeros(max(n, 1), np.uint32)
    if n:
        rc = lib().zkm_septic_lift(m, _u32(kinds), np.ascontiguousarray(is_receive, np.uint8), n, xy, off)
        if rc:
            raise RuntimeError("a message has no curve lift within 256 offsets")
    return xy[:n], off[:n]


def cumsum(points: np.ndarray, start=CURVE_CUMULATIVE_SUM_START):
    """start, start + P0, start + P0 + P1, ... with complete addition: (n + 1) x 15 (x, y, is_infinity)."""
    p = _u32(points).reshape(-1, 14)
    out = np.zeros((p.shape[0] + 1, 15), np.uint32)
    lib().zkm_septic_cumsum(_u32(start), p if p.size else np.zeros(14, np.uint32), p.shape[0], out)
    return out


def mul(a, b):
    out = np.zeros(7, np.uint32)
    lib().zkm_septic_mul(_u32(a), _u32(b), out)
    return out


def frobenius_col(i: int):
    out = np.zeros(7, np.uint32)
    lib().zkm_septic_frobenius_col(i, out)
    return out


def on_curve(xy) -> bool:
    return bool(lib().zkm_septic_on_curve(_u32(xy)))


def sum_checker_x(p1, p2, p3):
    out = np.zeros(7, np.uint32)
    lib().zkm_septic_sum_checker_x(_u32(p1), _u32(p2), _u32(p3), out)
    return out


def digest_sum(digests):
    """Sum of SepticDigests (septic_digest.rs:57-73); zero = CURVE_CUMULATIVE_SUM_START."""
    d = _u32(digests).reshape(-1, 14)
    out = np.zeros(14, np.uint32)
    lib().zkm_septic_digest_sum(d if d.size else np.zeros(14, np.uint32), d.shape[0],
                                CURVE_CUMULATIVE_SUM_START, DIGEST_SUM_START, out)
    return out
