// Executor records -> the zkm_tracegen.h structs, natively (libzkm_pyconv.so, loaded with ctypes.PyDLL so
// every call holds the GIL and a Python error raised here surfaces as an exception).
//
// This repository's executor (zkmips_amd/mips_core.py _execute) leaves its events as Python tuples; the
// reference's executor hands its Rust event vectors to the row ABI as they lie (CpuEvent -> CpuEventFfi,
// crates/core/executor/src/events/cpu.rs:46-75).  Converting 3-4 M step tuples through numpy took ~9 s per
// maximal 2^22 shard; walking them here with the CPython API and writing the structs
// directly takes a fraction of a second.
//
//   zkm_py_flatten_i64: rows of ints (nested tuples / lists allowed; None = none_w zeros) -> int64[n][width]
//   zkm_py_cpu_events:  the executor's step tuples -> zkm_cpu_event_ffi[n] (tracegen.cpu_events, same bytes)
#include <Python.h>

#include <cstdint>
#include <cstring>

#include "../../../include/zkm_tracegen.h"

static_assert(sizeof(zkm_option_memory_record) == 48, "OptionMemoryRecordEnum layout");
static_assert(sizeof(zkm_cpu_event_ffi) == 280, "CpuEventFfi layout");

namespace {

constexpr uint8_t REC_READ = 0, REC_WRITE = 1, REC_NONE = 2;

inline bool as_i64(PyObject *o, int64_t *v) {
    long long x = PyLong_AsLongLong(o);
    if (x == -1 && PyErr_Occurred()) return false;
    *v = (int64_t)x;
    return true;
}

// depth-first over ints / tuples / lists / None; writes at most cap values, counts them all in *k
bool flat(PyObject *o, int64_t *out, int64_t cap, int64_t *k, int64_t none_w, int depth) {
    if (o == Py_None) {
        for (int64_t i = 0; i < none_w; i++, (*k)++)
            if (*k < cap) out[*k] = 0;
        return true;
    }
    if (PyLong_Check(o)) {
        int64_t v;
        if (!as_i64(o, &v)) return false;
        if (*k < cap) out[*k] = v;
        (*k)++;
        return true;
    }
    if (depth > 8) {
        PyErr_SetString(PyExc_ValueError, "zkm_py_flatten_i64: rows nested too deep");
        return false;
    }
    if (PyTuple_Check(o)) {
        const Py_ssize_t n = PyTuple_GET_SIZE(o);
        for (Py_ssize_t i = 0; i < n; i++)
            if (!flat(PyTuple_GET_ITEM(o, i), out, cap, k, none_w, depth + 1)) return false;
        return true;
    }
    if (PyList_Check(o)) {
        const Py_ssize_t n = PyList_GET_SIZE(o);
        for (Py_ssize_t i = 0; i < n; i++)
            if (!flat(PyList_GET_ITEM(o, i), out, cap, k, none_w, depth + 1)) return false;
        return true;
    }
    if (PyIndex_Check(o)) {  // numpy integer scalars
        PyObject *x = PyNumber_Index(o);
        if (!x) return false;
        int64_t v;
        const bool ok = as_i64(x, &v);
        Py_DECREF(x);
        if (!ok) return false;
        if (*k < cap) out[*k] = v;
        (*k)++;
        return true;
    }
    PyErr_Format(PyExc_TypeError, "zkm_py_flatten_i64: unexpected %s in a record", Py_TYPE(o)->tp_name);
    return false;
}

// (shard, clk) of a previous access, or (0, 0) for a falsy entry (None, ())
bool prev_pair(PyObject *o, uint32_t *s, uint32_t *c) {
    *s = *c = 0;
    if (o == Py_None) return true;
    if (!PyTuple_Check(o) && !PyList_Check(o)) {
        PyErr_SetString(PyExc_TypeError, "zkm_py_cpu_events: previous access is not a pair");
        return false;
    }
    PyObject *seq = o;
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
    if (n == 0) return true;
    if (n != 2) {
        PyErr_SetString(PyExc_ValueError, "zkm_py_cpu_events: previous access is not a pair");
        return false;
    }
    int64_t a, b;
    if (!as_i64(PySequence_Fast_GET_ITEM(seq, 0), &a) || !as_i64(PySequence_Fast_GET_ITEM(seq, 1), &b)) return false;
    *s = (uint32_t)a;
    *c = (uint32_t)b;
    return true;
}

}  // namespace

extern "C" {

// rows: a list / tuple of n rows; each row must flatten to exactly `width` int64 values.  Returns n.
int64_t zkm_py_flatten_i64(PyObject *rows, int64_t width, int64_t none_w, int64_t *out, int64_t n_expect) {
    PyObject *seq = PySequence_Fast(rows, "zkm_py_flatten_i64: rows must be a sequence");
    if (!seq) return -1;
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
    if (n != n_expect) {
        Py_DECREF(seq);
        PyErr_Format(PyExc_ValueError, "zkm_py_flatten_i64: %zd rows, buffer for %lld", n, (long long)n_expect);
        return -1;
    }
    PyObject **items = PySequence_Fast_ITEMS(seq);
    for (Py_ssize_t r = 0; r < n; r++) {
        int64_t k = 0;
        if (!flat(items[r], out + r * width, width, &k, none_w, 0)) {
            Py_DECREF(seq);
            return -1;
        }
        if (k != width) {
            Py_DECREF(seq);
            PyErr_Format(PyExc_ValueError, "zkm_py_flatten_i64: row %zd has %lld values, want %lld", r, (long long)k,
                         (long long)width);
            return -1;
        }
    }
    Py_DECREF(seq);
    return n;
}

// steps: the executor's step tuples (k, op, a, b, c, prev_a, written, next_pc, next_next_pc, imm_b, imm_c,
// [prev c, prev b, prev a access], hi, clk, ...) -- the fields tracegen.cpu_events reads, with its meaning:
// op_a's access is a write when the register changed (a read otherwise), op_b / op_c reads unless immediate
// (executor.rs rr / rw at MemoryAccessPosition A / B / C).  out: n zkm_cpu_event_ffi.  Returns n.
int64_t zkm_py_cpu_events(PyObject *steps, uint32_t shard, uint32_t pc_base, uint32_t pos_a, uint32_t pos_b,
                          uint32_t pos_c, zkm_cpu_event_ffi *out, int64_t n_expect) {
    PyObject *seq = PySequence_Fast(steps, "zkm_py_cpu_events: steps must be a sequence");
    if (!seq) return -1;
    const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
    if (n != n_expect) {
        Py_DECREF(seq);
        PyErr_Format(PyExc_ValueError, "zkm_py_cpu_events: %zd steps, buffer for %lld", n, (long long)n_expect);
        return -1;
    }
    PyObject **items = PySequence_Fast_ITEMS(seq);
    std::memset(out, 0, sizeof(zkm_cpu_event_ffi) * (size_t)n);
    for (Py_ssize_t r = 0; r < n; r++) {
        PyObject *st = items[r];
        if (!PyTuple_Check(st) || PyTuple_GET_SIZE(st) < 14) {
            Py_DECREF(seq);
            PyErr_Format(PyExc_ValueError, "zkm_py_cpu_events: step %zd is not an executor step tuple", r);
            return -1;
        }
        int64_t f[14];
        for (int i = 0; i < 14; i++) {
            if (i == 11) continue;
            if (!as_i64(PyTuple_GET_ITEM(st, i), &f[i])) {
                Py_DECREF(seq);
                return -1;
            }
        }
        PyObject *acc = PyTuple_GET_ITEM(st, 11);  // previous accesses of op_c, op_b, op_a
        uint32_t ps[3] = {0, 0, 0}, pc[3] = {0, 0, 0};
        if (acc != Py_None) {
            if ((!PyList_Check(acc) && !PyTuple_Check(acc)) || PySequence_Fast_GET_SIZE(acc) != 3) {
                Py_DECREF(seq);
                PyErr_Format(PyExc_ValueError, "zkm_py_cpu_events: step %zd: want three previous accesses", r);
                return -1;
            }
            for (int j = 0; j < 3; j++)
                if (!prev_pair(PySequence_Fast_GET_ITEM(acc, j), &ps[j], &pc[j])) {
                    Py_DECREF(seq);
                    return -1;
                }
        }
        const int64_t k = f[0], av = f[2], bv = f[3], cv = f[4], prev_a = f[5], written = f[6];
        const uint32_t clk = (uint32_t)f[13];
        zkm_cpu_event_ffi &e = out[r];
        e.clk = clk;
        e.pc = pc_base + 4u * (uint32_t)k;
        e.next_pc = (uint32_t)f[7];
        e.next_next_pc = (uint32_t)f[8];
        e.a = (uint32_t)av;
        e.b = (uint32_t)bv;
        e.c = (uint32_t)cv;
        if (written != prev_a) {
            e.a_record.tag = REC_WRITE;
            e.a_record.write = {(uint32_t)written, shard, clk + pos_a, (uint32_t)prev_a, ps[2], pc[2]};
        } else {
            e.a_record.tag = REC_READ;
            e.a_record.read = {(uint32_t)written, shard, clk + pos_a, ps[2], pc[2]};
        }
        if (f[9]) {
            e.b_record.tag = REC_NONE;
        } else {
            e.b_record.tag = REC_READ;
            e.b_record.read = {(uint32_t)bv, shard, clk + pos_b, ps[1], pc[1]};
        }
        if (f[10]) {
            e.c_record.tag = REC_NONE;
        } else {
            e.c_record.tag = REC_READ;
            e.c_record.read = {(uint32_t)cv, shard, clk + pos_c, ps[0], pc[0]};
        }
        e.hi.tag = f[12] != 0 ? 0 : 1;  // OptionU32: 0 Some, 1 None
        e.hi.value = (uint32_t)f[12];
        e.hi_record.tag = REC_NONE;
        e.memory_record.tag = REC_NONE;
    }
    Py_DECREF(seq);
    return n;
}

}  // extern "C"
