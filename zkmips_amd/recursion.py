"""The recursion machine's compress AIR (BASELINE config 5), restated from the
reference, and the recursion runtime that produces its traces.

The compress stage proves recursion programs with the same STARK hot path as the core shards, under
``compressed_fri_config`` (log_blowup 2, 42 queries, 16 PoW bits; crates/stark/src/kb31_poseidon2.rs:
217-227) and ``RecursionAir<F, COMPRESS_DEGREE = 3>::compress_machine`` (crates/prover/src/lib.rs:106,121;
crates/recursion/core/src/machine.rs:112-128).  Its chips, in machine order:

=====================  =========================================================  ====  =====
chip                   reference                                                  prep  main
=====================  =========================================================  ====  =====
MemoryConst            recursion/core/src/chips/mem/constant.rs:17-155             12     1
MemoryVar              chips/mem/variable.rs:18-160                                  4     8
BaseAlu                chips/alu_base.rs:21-301                                     32    12
ExtAlu                 chips/alu_ext.rs:18-303                                      32    48
Poseidon2WideDeg3      chips/poseidon2_wide/{air.rs,trace.rs,columns/*}             49   313
BatchFRI               chips/batch_fri.rs:30-361                                     6    13
Select                 chips/select.rs:21-251                                        8     5
ExpReverseBitsLen      chips/exp_reverse_bits.rs:28-452                             10     7
PublicValues           chips/public_values.rs:24-310                                10     1
=====================  =========================================================  ====  =====

All chips talk through one bus: ``send_block`` / ``receive_block`` of (address, 4-word block) as Memory
lookups (recursion/core/src/builder.rs:18-72); a write sends with multiplicity = number of reads, a
read receives (or sends with a negative multiplicity).  Every chip's constraints and lookups are emitted
in the order its ``eval`` emits them, which fixes the alpha folding and the LogUp columns.

The runtime (``execute``) follows recursion/core/src/runtime/mod.rs:336-625 instruction by instruction
semantics, but executes a program as *blocks* of same-kind, mutually independent instructions
(numpy-vectorised): chip rows come out in program order, as the reference's trace generators emit them.
Write multiplicities are counted from the program's reads (the recursion compiler's job in the
reference), unless an instruction states one.
"""
from __future__ import annotations

import os
import re
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .machine import (ChipDesc, Expr, IS_FIRST, IS_TRANSITION, KIND_MEMORY, Lookup, MachineDesc, P,
                      VirtualPairCol as V, main, main_next, prep, prep_next, pv)

D = 4                      # extension degree, runtime/mod.rs (D)
W_EXT = 3                  # EF = F[x]/(x^4 - 3)
WIDTH = 16                 # Poseidon2 width
NUM_EXTERNAL_ROUNDS = 8    # poseidon2_wide/mod.rs:22-24
NUM_INTERNAL_ROUNDS = 13
PROOF_MAX_NUM_PVS = 231    # crates/stark/src/types.rs:73 (= RECURSIVE_PROOF_NUM_PV_ELTS)
PV_DIGEST_START = 223      # RecursionPublicValues.digest (air/public_values.rs:79-145): 32+8+6+128+16+8+8+14+3
DIGEST_SIZE = 8
PUB_VALUES_LOG_HEIGHT = 4  # chips/public_values.rs:30
COMPRESS_LOG_BLOWUP = 2    # kb31_poseidon2.rs:217-227
COMPRESS_NUM_QUERIES = 42
U = np.uint64
PU = U(P)

OP_ADD, OP_SUB, OP_MUL, OP_DIV = 0, 1, 2, 3

# Poseidon2 internal diagonal, poseidon2_wide/mod.rs:85-102 (canonical values)
DIAG = [P - 2, 1, 2, (P + 1) >> 1, 3, 4, (P - 1) >> 1, P - 3, P - 4, P - ((P - 1) >> 8), P - ((P - 1) >> 3),
        P - 127, (P - 1) >> 8, (P - 1) >> 3, (P - 1) >> 4, 127]


def _load_rc() -> List[List[int]]:
    """RC_16_30 (crates/primitives/src/lib.rs:19), from the generated table the HIP library is built with."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc", "p2_rc.inc")
    with open(path) as f:
        nums = [int(x, 16) for x in re.findall(r"0x([0-9a-fA-F]+)u", f.read())]
    assert len(nums) == 30 * 16
    return [nums[i * 16:(i + 1) * 16] for i in range(30)]


RC = _load_rc()


# ------------------------------------------------------------------ field helpers (numpy, canonical u64)

def _m(a, b):
    return (a * b) % PU


_HOST = {}


def _host(name: str):
    """A batch helper of libzkm_trace.so (zkmips_amd/csrc/host/ef_host.cpp, p2_host.cpp)."""
    f = _HOST.get(name)
    if f is None:
        import ctypes as C
        from . import septic
        f = getattr(septic.lib(), name)
        u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
        # (the per-call helpers take raw pointers: callers pass C-contiguous uint32 arrays' .ctypes.data, which
        # costs a fraction of ndpointer's checks on the replay's thousands of small calls)
        vp = C.c_void_p
        f.argtypes = {"zkm_host_ef_mul": [vp, vp, vp, C.c_uint64],
                      "zkm_host_batch_fri": [u32p, u32p, u32p, C.c_uint64, C.c_uint64, u32p],
                      "zkm_host_poseidon2_permute": [vp, vp, C.c_uint64],
                      "zkm_host_recursion_execute": [C.c_uint64, C.c_uint64,
                                                     np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS"),
                                                     C.c_void_p, C.c_char_p, C.c_uint64]}[name]
        if name == "zkm_host_recursion_execute":
            f.restype = C.c_int
        _HOST[name] = f
    return f


def ext_mul(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """(n,4) x (n,4) over F[x]/(x^4 - 3)."""
    if a.shape == b.shape and a.ndim == 2 and a.shape[0] >= 1:  # host C++ (ef_host.cpp): one ctypes call
        x = np.ascontiguousarray(a, dtype=np.uint32)
        y = np.ascontiguousarray(b, dtype=np.uint32)
        out = np.empty_like(x)
        _host("zkm_host_ef_mul")(x.ctypes.data, y.ctypes.data, out.ctypes.data, len(x))
        return out.astype(U)
    r = np.zeros(np.broadcast(a, b).shape, dtype=U)
    for i in range(D):
        for j in range(D):
            t = _m(a[..., i], b[..., j])
            if i + j >= D:
                r[..., i + j - D] = (r[..., i + j - D] + _m(t, U(W_EXT))) % PU
            else:
                r[..., i + j] = (r[..., i + j] + t) % PU
    return r


def _pow(x: np.ndarray, e: int) -> np.ndarray:
    r = np.ones_like(x)
    b = x.copy()
    while e:
        if e & 1:
            r = _m(r, b)
        b = _m(b, b)
        e >>= 1
    return r


def _pow_vec(x: np.ndarray, e: np.ndarray) -> np.ndarray:
    """x ** e elementwise (per-element exponents)."""
    r = np.ones_like(x)
    b = x.copy()
    e = np.asarray(e, np.int64).copy()
    while (e > 0).any():
        r = np.where(e & 1, _m(r, b), r)
        b = _m(b, b)
        e >>= 1
    return r


def ext_inv(a: np.ndarray) -> np.ndarray:
    """a^-1 via a(x) a(-x) = b0 + b2 x^2 and (b0 + b2 y)(b0 - b2 y) = b0^2 - 3 b2^2 in F."""
    conj = a.copy()
    conj[..., 1] = (PU - a[..., 1]) % PU
    conj[..., 3] = (PU - a[..., 3]) % PU
    b = ext_mul(a, conj)               # b1 = b3 = 0
    n = (_m(b[..., 0], b[..., 0]) + PU - _m(U(W_EXT), _m(b[..., 2], b[..., 2]))) % PU
    ninv = _pow(n, P - 2)
    c = np.zeros_like(a)
    c[..., 0] = b[..., 0]
    c[..., 2] = (PU - b[..., 2]) % PU
    r = ext_mul(conj, c)
    return _m(r, ninv[..., None])


# ------------------------------------------------------------------ Poseidon2 (for the trace)

def _m4(x):
    t01 = (x[0] + x[1]) % PU
    t23 = (x[2] + x[3]) % PU
    t0123 = (t01 + t23) % PU
    t01123 = (t0123 + x[1]) % PU
    t01233 = (t0123 + x[3]) % PU
    y3 = (t01233 + 2 * x[0]) % PU
    y1 = (t01123 + 2 * x[2]) % PU
    y0 = (t01123 + t01) % PU
    y2 = (t01233 + t23) % PU
    return [y0, y1, y2, y3]


def external_linear_layer(s: List[np.ndarray]) -> List[np.ndarray]:
    """poseidon2_wide/mod.rs:56-82: M4 per 4-block, then add the column sums."""
    out = []
    for j in range(0, WIDTH, 4):
        out += _m4(s[j:j + 4])
    sums = [(out[k] + out[4 + k] + out[8 + k] + out[12 + k]) % PU for k in range(4)]
    return [(out[j] + sums[j % 4]) % PU for j in range(WIDTH)]


def internal_linear_layer(s: List[np.ndarray]) -> List[np.ndarray]:
    """p3_poseidon2::matmul_internal with the diagonal above: s_i <- d_i s_i + sum."""
    tot = s[0]
    for j in range(1, WIDTH):
        tot = (tot + s[j]) % PU
    return [(_m(s[i], U(DIAG[i])) + tot) % PU for i in range(WIDTH)]


# Poseidon2WideDeg3 main columns (PermutationSBox, columns/permutation.rs:20-72)
P2_EXT = 0                                   # external_rounds_state [8][16]
P2_INT = P2_EXT + NUM_EXTERNAL_ROUNDS * WIDTH  # internal_rounds_state [16]
P2_S0 = P2_INT + WIDTH                       # internal_rounds_s0 [12]
P2_OUT = P2_S0 + NUM_INTERNAL_ROUNDS - 1     # output_state [16]
P2_ESBOX = P2_OUT + WIDTH                    # external_rounds_sbox_state [8][16]
P2_ISBOX = P2_ESBOX + NUM_EXTERNAL_ROUNDS * WIDTH  # internal_rounds_sbox_state [13]
P2_COLS = P2_ISBOX + NUM_INTERNAL_ROUNDS     # 313 = NUM_POSEIDON2_DEGREE3_COLS


def poseidon2_rows(inputs: np.ndarray) -> np.ndarray:
    """(n,16) canonical inputs -> (n,313) Poseidon2WideDeg3 rows (trace.rs populate_perm): the
    permutation's round states, s-box cubes and output."""
    n = inputs.shape[0]
    t = np.zeros((n, P2_COLS), dtype=U)
    ext = [inputs[:, i].astype(U) % PU for i in range(WIDTH)]
    t[:, P2_EXT:P2_EXT + WIDTH] = np.stack(ext, 1)

    def external_round(state, r):
        if r == 0:
            state = external_linear_layer(state)
        rnd = r if r < NUM_EXTERNAL_ROUNDS // 2 else r + NUM_INTERNAL_ROUNDS
        sb = []
        for i in range(WIDTH):
            a = (state[i] + U(RC[rnd][i])) % PU
            sb.append(_m(_m(a, a), a))
        t[:, P2_ESBOX + r * WIDTH:P2_ESBOX + (r + 1) * WIDTH] = np.stack(sb, 1)
        return external_linear_layer(sb)

    state = ext
    for r in range(NUM_EXTERNAL_ROUNDS // 2):
        state = external_round(state, r)
        if r == NUM_EXTERNAL_ROUNDS // 2 - 1:
            t[:, P2_INT:P2_INT + WIDTH] = np.stack(state, 1)
        else:
            t[:, P2_EXT + (r + 1) * WIDTH:P2_EXT + (r + 2) * WIDTH] = np.stack(state, 1)
    for r in range(NUM_INTERNAL_ROUNDS):
        a = (state[0] + U(RC[r + NUM_EXTERNAL_ROUNDS // 2][0])) % PU
        sb = _m(_m(a, a), a)
        t[:, P2_ISBOX + r] = sb
        state = internal_linear_layer([sb] + state[1:])
        if r < NUM_INTERNAL_ROUNDS - 1:
            t[:, P2_S0 + r] = state[0]
    r4 = NUM_EXTERNAL_ROUNDS // 2
    t[:, P2_EXT + r4 * WIDTH:P2_EXT + (r4 + 1) * WIDTH] = np.stack(state, 1)
    for r in range(r4, NUM_EXTERNAL_ROUNDS):
        state = external_round(state, r)
        if r == NUM_EXTERNAL_ROUNDS - 1:
            t[:, P2_OUT:P2_OUT + WIDTH] = np.stack(state, 1)
        else:
            t[:, P2_EXT + (r + 1) * WIDTH:P2_EXT + (r + 2) * WIDTH] = np.stack(state, 1)
    return t


def p2_inputs(rec: ExecutionRecord) -> np.ndarray:
    """The program's Poseidon2 inputs in instruction order (n x 16 canonical): the Poseidon2WideDeg3 events."""
    return np.ascontiguousarray(rec.ev["p2"][:, :WIDTH])


def poseidon2_permute_host(inputs: np.ndarray) -> np.ndarray:
    """Poseidon2-16 of every row (canonical): the product permutation (p2.cuh) compiled for the host,
    zkm_host_poseidon2_permute in libzkm_trace.so -- the runtime's Poseidon2 instruction."""
    x = np.ascontiguousarray(inputs, dtype=np.uint32).reshape(-1, WIDTH)
    out = np.empty_like(x)
    if len(x):
        _host("zkm_host_poseidon2_permute")(x.ctypes.data, out.ctypes.data, len(x))
    return out.astype(U)


def poseidon2_permute(inputs: np.ndarray) -> np.ndarray:
    return poseidon2_rows(np.atleast_2d(inputs))[:, P2_OUT:P2_OUT + WIDTH]


# ------------------------------------------------------------------ program (blocks of instructions)

@dataclass
class Block:
    """A run of same-kind instructions that read only what earlier blocks wrote."""
    kind: str
    a: Dict[str, np.ndarray] = field(default_factory=dict)

    def __len__(self):
        return len(next(iter(self.a.values())))


@dataclass
class RecursionProgram:
    blocks: List[Block] = field(default_factory=list)
    num_addrs: int = 0

    # --- builders (runtime/instruction.rs helpers, vectorised) ---
    def alloc(self, n: int) -> np.ndarray:
        a = np.arange(self.num_addrs, self.num_addrs + n, dtype=np.int64)
        self.num_addrs += n
        return a

    def _add(self, kind, **arrays):
        self.blocks.append(Block(kind, {k: np.asarray(v) for k, v in arrays.items()}))

    def mem_write(self, addr, vals, mult=None):
        """Instruction::Mem Write (constant memory): vals (n,4)."""
        addr = np.atleast_1d(np.asarray(addr, np.int64))
        vals = np.asarray(vals, dtype=U).reshape(len(addr), D) % PU
        self._add("mem", addr=addr, vals=vals, write=np.ones(len(addr), bool), mult=_mults(mult, len(addr)))

    def mem_read(self, addr, vals, mult=1):
        addr = np.atleast_1d(np.asarray(addr, np.int64))
        vals = np.asarray(vals, dtype=U).reshape(len(addr), D) % PU
        m = np.broadcast_to(np.asarray(mult, np.int64), (len(addr),)).copy()
        self._add("mem", addr=addr, vals=vals, write=np.zeros(len(addr), bool), mult=m)

    def hint(self, addr, vals, mult=None):
        """Instruction::Hint: witness blocks written to variable memory (MemoryVar)."""
        addr = np.atleast_1d(np.asarray(addr, np.int64))
        vals = np.asarray(vals, dtype=U).reshape(len(addr), D) % PU
        self._add("hint", addr=addr, vals=vals, mult=_mults(mult, len(addr)))

    def base_alu(self, op, out, in1, in2, mult=None):
        out = np.atleast_1d(np.asarray(out, np.int64))
        n = len(out)
        self._add("base", op=_vec(op, n), out=out, in1=_vec(in1, n), in2=_vec(in2, n), mult=_mults(mult, n))

    def ext_alu(self, op, out, in1, in2, mult=None):
        out = np.atleast_1d(np.asarray(out, np.int64))
        n = len(out)
        self._add("ext", op=_vec(op, n), out=out, in1=_vec(in1, n), in2=_vec(in2, n), mult=_mults(mult, n))

    def poseidon2(self, outs, ins, mults=None):
        outs = np.asarray(outs, np.int64).reshape(-1, WIDTH)
        ins = np.asarray(ins, np.int64).reshape(-1, WIDTH)
        m = None if mults is None else np.asarray(mults, np.int64).reshape(-1, WIDTH)
        self._add("p2", out=outs, inp=ins, mult=_mults(m, outs.shape))

    def select(self, bit, out1, out2, in1, in2, mult1=None, mult2=None):
        bit = np.atleast_1d(np.asarray(bit, np.int64))
        n = len(bit)
        self._add("select", bit=bit, out1=np.asarray(out1, np.int64).reshape(n), out2=np.asarray(out2, np.int64).reshape(n),
                  in1=np.asarray(in1, np.int64).reshape(n), in2=np.asarray(in2, np.int64).reshape(n),
                  mult1=_mults(mult1, n), mult2=_mults(mult2, n))

    def exp_reverse_bits(self, base, exps, result, mult=None):
        """Instruction::ExpReverseBitsLen; exps (n, L) bit addresses (one length per block)."""
        base = np.atleast_1d(np.asarray(base, np.int64))
        exps = np.asarray(exps, np.int64).reshape(len(base), -1)
        self._add("exprev", base=base, exps=exps, result=np.asarray(result, np.int64).reshape(len(base)),
                  mult=_mults(mult, len(base)))

    def batch_fri(self, acc, alpha_pow, p_at_z, p_at_x):
        """Instruction::BatchFRI: acc = sum_i alpha_pow_i (p_at_z_i - p_at_x_i); (n, L) address arrays."""
        acc = np.atleast_1d(np.asarray(acc, np.int64))
        n = len(acc)
        self._add("batchfri", acc=acc, alpha_pow=np.asarray(alpha_pow, np.int64).reshape(n, -1),
                  p_at_z=np.asarray(p_at_z, np.int64).reshape(n, -1), p_at_x=np.asarray(p_at_x, np.int64).reshape(n, -1),
                  mult=np.ones(n, np.int64))

    def fri_fold(self, x, z, alpha, p_at_x, p_at_z, alpha_pow_in, ro_in, alpha_pow_out, ro_out,
                 alpha_pow_mults=None, ro_mults=None):
        """Instruction::FriFold (runtime/mod.rs:461-535): one instruction, m = len(p_at_z) entries;
        ro_out = ro_in + alpha_pow_in (p_at_x - p_at_z) / (x - z), alpha_pow_out = alpha_pow_in alpha."""
        v = lambda a: np.asarray(a, np.int64).reshape(1, -1)
        m = v(p_at_z).shape[1]
        self._add("frifold", x=np.asarray([x], np.int64), z=np.asarray([z], np.int64), alpha=np.asarray([alpha], np.int64),
                  p_at_x=v(p_at_x), p_at_z=v(p_at_z), alpha_pow_in=v(alpha_pow_in), ro_in=v(ro_in),
                  alpha_pow_out=v(alpha_pow_out), ro_out=v(ro_out),
                  apm=_mults(None if alpha_pow_mults is None else v(alpha_pow_mults), (1, m)),
                  rom=_mults(None if ro_mults is None else v(ro_mults), (1, m)))

    def commit_public_values(self, pv_addrs):
        pv_addrs = np.asarray(pv_addrs, np.int64).reshape(PROOF_MAX_NUM_PVS)
        self._add("commit", pv=pv_addrs[None, :])


def _vec(x, n: int) -> np.ndarray:
    """x as an int64 vector of n entries (address arrays are never modified after a block is added, so an
    array of the right shape is kept as it is)."""
    a = np.asarray(x, np.int64)
    return a if a.shape == (n,) else np.broadcast_to(a, (n,)).copy()


def _mults(m, shape):
    """-1 marks 'count the reads' (filled in by ``execute``)."""
    if m is None:
        return np.full(shape, -1, np.int64)
    return np.broadcast_to(np.asarray(m, np.int64), shape).copy()


# reads of each block kind: (array name, per-element multiplicity) -- runtime/mod.rs mr() calls that the
# AIR matches with a receive
def _reads(b: Block):
    a = b.a
    if b.kind == "mem":
        return [(a["addr"][~a["write"]], a["mult"][~a["write"]])]
    if b.kind in ("base", "ext"):
        return [(a["in1"], 1), (a["in2"], 1)]
    if b.kind == "p2":
        return [(a["inp"].ravel(), 1)]
    if b.kind == "select":
        return [(a["bit"], 1), (a["in1"], 1), (a["in2"], 1)]
    if b.kind == "exprev":
        return [(a["base"], 1), (a["exps"].ravel(), 1)]
    if b.kind == "batchfri":
        return [(a["alpha_pow"].ravel(), 1), (a["p_at_z"].ravel(), 1), (a["p_at_x"].ravel(), 1)]
    if b.kind == "commit":
        return [(a["pv"][0, PV_DIGEST_START:PV_DIGEST_START + DIGEST_SIZE], 1)]
    if b.kind == "frifold":
        return [(a["x"], 1), (a["z"], 1), (a["alpha"], 1), (a["p_at_x"].ravel(), 1), (a["p_at_z"].ravel(), 1),
                (a["alpha_pow_in"].ravel(), 1), (a["ro_in"].ravel(), 1)]
    return []


def _writes(b: Block):
    a = b.a
    if b.kind == "mem":
        return [("addr", "mult", a["write"])]
    if b.kind in ("hint", "base", "ext"):
        return [("out" if b.kind != "hint" else "addr", "mult", None)]
    if b.kind == "p2":
        return [("out", "mult", None)]
    if b.kind == "select":
        return [("out1", "mult1", None), ("out2", "mult2", None)]
    if b.kind in ("exprev",):
        return [("result", "mult", None)]
    if b.kind == "batchfri":
        return [("acc", "mult", None)]
    if b.kind == "frifold":
        return [("alpha_pow_out", "apm", None), ("ro_out", "rom", None)]
    return []


def resolve_mults(prog: RecursionProgram) -> None:
    """Fill every '-1' write multiplicity with the number of reads of that address."""
    cnt = np.zeros(prog.num_addrs, np.int64)
    for b in prog.blocks:
        for addrs, m in _reads(b):
            np.add.at(cnt, addrs, m)
    for b in prog.blocks:
        for an, mn, sel in _writes(b):
            m = b.a[mn]
            auto = m < 0
            if sel is not None:
                auto &= sel
            m[auto] = cnt[b.a[an][auto]]


# ------------------------------------------------------------------ runtime

KINDS = ("mem", "hint", "base", "ext", "p2", "select", "exprev", "batchfri", "frifold", "commit")
_KIND_CODE = {k: i for i, k in enumerate(KINDS)}
# zkm_host_recursion_execute's pointer slots (csrc/host/rec_exec.cpp enum Slot), in order
_RX_SLOTS = ("mem.addr", "mem.vals", "mem.write", "hint.addr", "hint.vals",
             "base.op", "base.out", "base.in1", "base.in2", "ev.base",
             "ext.op", "ext.out", "ext.in1", "ext.in2", "ev.ext",
             "p2.out", "p2.inp", "ev.p2",
             "select.bit", "select.out1", "select.out2", "select.in1", "select.in2", "ev.select",
             "exprev.base", "exprev.result", "exprev.exps", "ev.exprev",
             "batchfri.acc", "batchfri.alpha_pow", "batchfri.p_at_z", "batchfri.p_at_x", "ev.batchfri",
             "frifold.x", "frifold.z", "frifold.alpha", "frifold.p_at_x", "frifold.p_at_z", "frifold.alpha_pow_in",
             "frifold.ro_in", "frifold.alpha_pow_out", "frifold.ro_out", "ev.frifold",
             "commit.pv", "ev.commit", "mem_image")
# event row widths (the chips' main-trace rows; p2: input[16] + output[16]; commit: all public values)
EV_WIDTH = {"base": 3, "ext": 3 * D, "p2": 2 * WIDTH, "select": 5, "exprev": 7, "batchfri": 13, "frifold": 33,
            "commit": PROOF_MAX_NUM_PVS}


@dataclass
class FlatProgram:
    """A program flattened by instruction kind: every kind's operand arrays concatenated in program order
    (`a[kind][name]`), and a block table (nblocks x 5 int64: kind code, first entry, entries, row length L,
    first flat row) -- the form the native runtime and the vectorised trace builders take.  Entries of
    exprev / batchfri have L rows each (their address matrices are flattened to rows); a frifold block is
    one entry of L rows; `mult` arrays are resolved (no -1 left)."""
    num_addrs: int
    table: np.ndarray
    a: Dict[str, Dict[str, np.ndarray]]
    n: Dict[str, int]       # entries per kind
    rows: Dict[str, int]    # flat rows per kind (exprev, batchfri, frifold)


_FLAT_FIELDS = {
    "mem": (("addr", np.int64), ("vals", np.uint32), ("write", np.uint8), ("mult", np.int64)),
    "hint": (("addr", np.int64), ("vals", np.uint32), ("mult", np.int64)),
    "base": (("op", np.int64), ("out", np.int64), ("in1", np.int64), ("in2", np.int64), ("mult", np.int64)),
    "ext": (("op", np.int64), ("out", np.int64), ("in1", np.int64), ("in2", np.int64), ("mult", np.int64)),
    "p2": (("out", np.int64), ("inp", np.int64), ("mult", np.int64)),
    "select": (("bit", np.int64), ("out1", np.int64), ("out2", np.int64), ("in1", np.int64), ("in2", np.int64),
               ("mult1", np.int64), ("mult2", np.int64)),
    "exprev": (("base", np.int64), ("result", np.int64), ("mult", np.int64)),
    "batchfri": (("acc", np.int64), ("mult", np.int64)),
    "frifold": (("x", np.int64), ("z", np.int64), ("alpha", np.int64)),
    "commit": (("pv", np.int64),),
}
_FLAT_ROWS = {"exprev": ("exps",), "batchfri": ("alpha_pow", "p_at_z", "p_at_x"),
              "frifold": ("p_at_x", "p_at_z", "alpha_pow_in", "ro_in", "alpha_pow_out", "ro_out", "apm", "rom")}
_FLAT_TAIL = {("mem", "vals"): (D,), ("hint", "vals"): (D,), ("p2", "out"): (WIDTH,), ("p2", "inp"): (WIDTH,),
              ("p2", "mult"): (WIDTH,), ("commit", "pv"): (PROOF_MAX_NUM_PVS,)}


def flatten(prog: RecursionProgram) -> FlatProgram:
    """The program's FlatProgram, with the write multiplicities resolved (recursion compiler's job in the
    reference): -1 becomes the number of reads of the address."""
    parts = {k: {nm: [] for nm, _ in _FLAT_FIELDS[k]} for k in KINDS}
    rparts = {k: {nm: [] for nm in v} for k, v in _FLAT_ROWS.items()}
    lens = {k: [] for k in _FLAT_ROWS}
    table = np.zeros((len(prog.blocks), 5), np.int64)
    n = {k: 0 for k in KINDS}
    rows = {k: 0 for k in _FLAT_ROWS}
    for bi, b in enumerate(prog.blocks):
        k, a = b.kind, b.a
        if k == "frifold":
            cnt, L = 1, a["p_at_z"].shape[1]
        elif k in ("exprev", "batchfri"):
            key = "exps" if k == "exprev" else "p_at_x"
            cnt, L = a[key].shape
        elif k == "commit":
            cnt, L = 1, 0
        else:
            cnt, L = len(next(iter(a.values()))), 0
        table[bi] = (_KIND_CODE[k], n[k], cnt, L, rows.get(k, 0))
        for nm, _ in _FLAT_FIELDS[k]:
            parts[k][nm].append(a[nm])
        if k in _FLAT_ROWS:
            for nm in _FLAT_ROWS[k]:
                rparts[k][nm].append(a[nm].reshape(-1))
            lens[k].append(np.full(cnt, L, np.int64))
            rows[k] += cnt * L
        n[k] += cnt
    out = {}
    for k in KINDS:
        d = {}
        for nm, dt in _FLAT_FIELDS[k]:
            xs = parts[k][nm]
            tail = _FLAT_TAIL.get((k, nm), ())
            if k in ("frifold",) or k == "commit":
                xs = [np.asarray(x).reshape((-1,) + tail) for x in xs]
            d[nm] = (np.ascontiguousarray(np.concatenate(xs).astype(dt, copy=False)) if xs
                     else np.zeros((0,) + tail, dt))
        if k in _FLAT_ROWS:
            for nm in _FLAT_ROWS[k]:
                xs = rparts[k][nm]
                d[nm] = np.ascontiguousarray(np.concatenate(xs).astype(np.int64)) if xs else np.zeros(0, np.int64)
            d["L"] = np.concatenate(lens[k]) if lens[k] else np.zeros(0, np.int64)
        out[k] = d
    fp = FlatProgram(prog.num_addrs, table, out, n, rows)
    _resolve_mults_flat(fp)
    return fp


def _resolve_mults_flat(fp: FlatProgram) -> None:
    """resolve_mults on the flat arrays, vectorised: one count of every read (runtime/mod.rs mr() calls the
    AIR matches with a receive), then every '-1' write multiplicity set to its address's count."""
    a = fp.a
    na = fp.num_addrs
    reads = [a["base"]["in1"], a["base"]["in2"], a["ext"]["in1"], a["ext"]["in2"], a["p2"]["inp"].ravel(),
             a["select"]["bit"], a["select"]["in1"], a["select"]["in2"], a["exprev"]["base"], a["exprev"]["exps"],
             a["batchfri"]["alpha_pow"], a["batchfri"]["p_at_z"], a["batchfri"]["p_at_x"],
             a["commit"]["pv"][:, PV_DIGEST_START:PV_DIGEST_START + DIGEST_SIZE].ravel(),
             a["frifold"]["x"], a["frifold"]["z"], a["frifold"]["alpha"], a["frifold"]["p_at_x"],
             a["frifold"]["p_at_z"], a["frifold"]["alpha_pow_in"], a["frifold"]["ro_in"]]
    cnt = np.bincount(np.concatenate(reads).astype(np.int64), minlength=na).astype(np.int64)
    rd = a["mem"]["write"] == 0
    if rd.any():
        np.add.at(cnt, a["mem"]["addr"][rd], a["mem"]["mult"][rd])
    for k, an, mn, sel in (("mem", "addr", "mult", "write"), ("hint", "addr", "mult", None),
                           ("base", "out", "mult", None), ("ext", "out", "mult", None), ("p2", "out", "mult", None),
                           ("select", "out1", "mult1", None), ("select", "out2", "mult2", None),
                           ("exprev", "result", "mult", None), ("batchfri", "acc", "mult", None),
                           ("frifold", "alpha_pow_out", "apm", None), ("frifold", "ro_out", "rom", None)):
        m = a[k][mn]
        auto = m < 0
        if sel is not None:
            auto &= a[k][sel].astype(bool)
        if auto.any():
            m[auto] = cnt[a[k][an][auto]]


class ExecutionRecord:
    """A program's execution: its FlatProgram, the events per kind (`ev`: the chips' main-trace rows,
    uint32 canonical, concatenated in program order; EV_WIDTH columns) and the committed public values.
    `events` gives the per-block view (lists of dicts, as the numpy runtime produced them)."""

    def __init__(self, program, flat, ev, public_values, events=None):
        self.program, self.flat, self.ev, self.public_values = program, flat, ev, public_values
        self._events = events

    @property
    def events(self) -> Dict[str, List[Dict[str, np.ndarray]]]:
        if self._events is None:
            self._events = _legacy_events(self)
        return self._events


def _legacy_events(rec: ExecutionRecord):
    ev, out = rec.ev, {k: [] for k in KINDS}
    for kc, s, n, L, fs in rec.flat.table:
        k = KINDS[kc]
        e = ev.get(k)
        if k == "mem":
            out[k].append({})
        elif k == "hint":
            out[k].append({"vals": rec.flat.a["hint"]["vals"][s:s + n].astype(U)})
        elif k == "base":
            x = e[s:s + n].astype(U)
            out[k].append({"out": x[:, 0], "in1": x[:, 1], "in2": x[:, 2]})
        elif k == "ext":
            x = e[s:s + n].astype(U)
            out[k].append({"out": x[:, 0:4], "in1": x[:, 4:8], "in2": x[:, 8:12]})
        elif k == "p2":
            x = e[s:s + n].astype(U)
            out[k].append({"inputs": x[:, :WIDTH], "outputs": x[:, WIDTH:]})
        elif k == "select":
            x = e[s:s + n].astype(U)
            out[k].append({nm: x[:, j] for j, nm in enumerate(("bit", "out1", "out2", "in1", "in2"))})
        elif k in ("exprev", "batchfri"):
            out[k].append({"rows": e[fs:fs + n * L].astype(U), "L": int(L), "n": int(n)})
        elif k == "frifold":
            out[k].append({"rows": e[fs:fs + L].astype(U)})
        elif k == "commit":
            out[k].append({"pv": e[s].astype(U)})
    return out


def _ev_from_legacy(fp: FlatProgram, events) -> Dict[str, np.ndarray]:
    ev = {}
    for k in ("base", "ext", "p2", "select", "exprev", "batchfri", "frifold", "commit"):
        w = EV_WIDTH[k]
        es = events[k]
        if k == "base":
            xs = [np.stack([e["out"], e["in1"], e["in2"]], 1) for e in es]
        elif k == "ext":
            xs = [np.concatenate([e["out"], e["in1"], e["in2"]], 1) for e in es]
        elif k == "p2":
            xs = [np.concatenate([e["inputs"], e["outputs"]], 1) for e in es]
        elif k == "select":
            xs = [np.stack([e[nm] for nm in ("bit", "out1", "out2", "in1", "in2")], 1) for e in es]
        elif k == "commit":
            xs = [e["pv"][None, :] for e in es]
        else:
            xs = [e["rows"] for e in es]
        ev[k] = (np.ascontiguousarray(np.concatenate(xs).astype(np.uint32)) if xs else np.zeros((0, w), np.uint32))
    return ev


def execute(prog, mem_out: Optional[dict] = None) -> ExecutionRecord:
    """Run the program (runtime/mod.rs:336-625) in the native runtime (csrc/host/rec_exec.cpp,
    libzkm_trace.so): memory is write-once, every value read must have been written by an earlier
    block, constant-memory reads must match; a violation is a RuntimeError naming the block.  `prog` is a
    RecursionProgram or an already flattened FlatProgram (then the record's `program` is None)."""
    import ctypes as C
    flat_in = isinstance(prog, FlatProgram)
    fp = prog if flat_in else flatten(prog)
    a = fp.a
    ev = {k: np.zeros((fp.rows[k] if k in fp.rows else fp.n[k], EV_WIDTH[k]), np.uint32) for k in EV_WIDTH}
    img = np.zeros((fp.num_addrs, D), np.uint32) if mem_out is not None else None
    ptrs = (C.c_void_p * len(_RX_SLOTS))()
    for i, nm in enumerate(_RX_SLOTS):
        if nm == "mem_image":
            arr = img
        elif nm.startswith("ev."):
            arr = ev[nm[3:]]
        else:
            k, f = nm.split(".")
            arr = a[k][f]
        ptrs[i] = None if arr is None or arr.size == 0 else arr.ctypes.data
    err = C.create_string_buffer(256)
    f = _host("zkm_host_recursion_execute")
    rc = f(fp.num_addrs, len(fp.table), np.ascontiguousarray(fp.table), C.cast(ptrs, C.c_void_p), err, 256)
    if mem_out is not None:
        mem_out["mem"] = img.astype(U)
    if rc != 0:
        raise RuntimeError(err.value.decode())
    pvs = ev["commit"][-1].copy() if len(ev["commit"]) else np.zeros(PROOF_MAX_NUM_PVS, np.uint32)
    return ExecutionRecord(None if flat_in else prog, fp, ev, pvs)


def execute_numpy(prog: RecursionProgram, mem_out: Optional[dict] = None) -> ExecutionRecord:
    """The same runtime as numpy blocks (the native runtime's cross-check in tests/test_recursion.py):
    returns per-kind event lists in program order."""
    resolve_mults(prog)
    mem = np.zeros((prog.num_addrs, D), U)
    written = np.zeros(prog.num_addrs, bool)
    if mem_out is not None:  # diagnostics: the memory image (also after a failed check)
        mem_out["mem"] = mem
    ev: Dict[str, List[Dict[str, np.ndarray]]] = {k: [] for k in
                                                 ("mem", "hint", "base", "ext", "p2", "select", "exprev", "batchfri", "commit",
                                                  "frifold")}
    pvs = np.zeros(PROOF_MAX_NUM_PVS, np.uint32)

    def rd(addr):
        addr = np.asarray(addr)
        if addr.size and (addr.min() < 0 or addr.max() >= prog.num_addrs or not written[addr].all()):
            raise RuntimeError("read of an unassigned address")
        return mem[addr]

    def wr(addr, vals):
        if written[addr].any() or len(np.unique(addr)) != len(addr):
            raise RuntimeError("write to an assigned address")
        mem[addr] = vals
        written[addr] = True

    for bi, b in enumerate(prog.blocks):
        a = b.a
        k = b.kind
        if k == "mem":
            w = a["write"]
            if (~w).any():
                if not np.array_equal(rd(a["addr"][~w]), a["vals"][~w]):
                    raise RuntimeError(f"stored memory value should be the specified value (block {bi})")
            wr(a["addr"][w], a["vals"][w])
            ev["mem"].append({})
        elif k == "hint":
            wr(a["addr"], a["vals"])
            ev["hint"].append({"vals": a["vals"]})
        elif k == "base":
            x, y = rd(a["in1"])[:, 0], rd(a["in2"])[:, 0]
            op = a["op"]
            out = np.where(op == OP_ADD, (x + y) % PU, np.where(op == OP_SUB, (x + PU - y) % PU, _m(x, y)))
            if (op == OP_DIV).any():
                d = op == OP_DIV
                out[d] = _m(x[d], _pow(y[d], P - 2))
            blk = np.zeros((len(out), D), U)
            blk[:, 0] = out
            wr(a["out"], blk)
            ev["base"].append({"out": out, "in1": x, "in2": y})
        elif k == "ext":
            x, y = rd(a["in1"]), rd(a["in2"])
            op = a["op"][:, None]
            out = np.where(op == OP_ADD, (x + y) % PU, np.where(op == OP_SUB, (x + PU - y) % PU, ext_mul(x, y)))
            d = a["op"] == OP_DIV
            if d.any():
                out[d] = ext_mul(x[d], ext_inv(y[d]))
            wr(a["out"], out)
            ev["ext"].append({"out": out, "in1": x, "in2": y})
        elif k == "p2":
            x = rd(a["inp"].ravel())[:, 0].reshape(-1, WIDTH)
            out = poseidon2_permute_host(x)
            blk = np.zeros((x.size, D), U)
            blk[:, 0] = out.ravel()
            wr(a["out"].ravel(), blk)
            ev["p2"].append({"inputs": x, "outputs": out})  # the trace rows are built with the traces
        elif k == "select":
            bit, x, y = rd(a["bit"])[:, 0], rd(a["in1"])[:, 0], rd(a["in2"])[:, 0]
            nb = (PU + 1 - bit) % PU
            o1 = (_m(bit, y) + _m(nb, x)) % PU
            o2 = (_m(bit, x) + _m(nb, y)) % PU
            for nm, v in (("out1", o1), ("out2", o2)):
                blk = np.zeros((len(v), D), U)
                blk[:, 0] = v
                wr(a[nm], blk)
            ev["select"].append({"bit": bit, "out1": o1, "out2": o2, "in1": x, "in2": y})
        elif k == "exprev":
            base = rd(a["base"])[:, 0]
            n, L = a["exps"].shape
            bits = rd(a["exps"].ravel())[:, 0].reshape(n, L)
            acc = np.ones(n, U)
            cols = np.zeros((n, L, 7), U)
            for i in range(L):
                prev = acc
                mult = np.where(bits[:, i] == 1, base, U(1))
                psq = _m(prev, prev)
                acc = _m(psq, mult)
                cols[:, i] = np.stack([base, bits[:, i], psq, _m(psq, mult), acc, _m(acc, acc), mult], 1)
            blk = np.zeros((n, D), U)
            blk[:, 0] = acc
            wr(a["result"], blk)
            ev["exprev"].append({"rows": cols.reshape(n * L, 7), "L": L, "n": n})
        elif k == "batchfri":
            n, L = a["p_at_x"].shape
            px = rd(a["p_at_x"].ravel())[:, 0].reshape(n, L)
            pz = rd(a["p_at_z"].ravel()).reshape(n, L, D)
            al = rd(a["alpha_pow"].ravel()).reshape(n, L, D)
            runs = np.empty((n, L, D), np.uint32)
            _host("zkm_host_batch_fri")(np.ascontiguousarray(al, dtype=np.uint32), np.ascontiguousarray(pz, dtype=np.uint32),
                                        np.ascontiguousarray(px, dtype=np.uint32), n, L, runs)
            rows = np.zeros((n, L, 13), U)
            rows[:, :, 0:4] = runs
            rows[:, :, 4:8] = al
            rows[:, :, 8:12] = pz
            rows[:, :, 12] = px
            acc = rows[:, L - 1, 0:4].copy() if L else np.zeros((n, D), U)
            wr(a["acc"], acc)
            ev["batchfri"].append({"rows": rows.reshape(n * L, 13), "L": L, "n": n})
        elif k == "frifold":
            x = rd(a["x"])[0, 0]
            z, alpha = rd(a["z"])[0], rd(a["alpha"])[0]
            px, pz = rd(a["p_at_x"][0]), rd(a["p_at_z"][0])
            ap, ro = rd(a["alpha_pow_in"][0]), rd(a["ro_in"][0])
            xz = (PU - z) % PU
            xz[0] = (xz[0] + x) % PU                       # x - z
            q = ext_mul((px + PU - pz) % PU, ext_inv(np.broadcast_to(xz, px.shape).copy()))
            new_ro = (ro + ext_mul(ap, q)) % PU
            new_ap = ext_mul(ap, np.broadcast_to(alpha, ap.shape))
            wr(a["ro_out"][0], new_ro)
            wr(a["alpha_pow_out"][0], new_ap)
            mm = px.shape[0]
            rows = np.zeros((mm, 33), U)
            rows[:, 0:4], rows[:, 4:8], rows[:, 8] = z, alpha, x
            rows[:, 9:13], rows[:, 13:17], rows[:, 17:21], rows[:, 21:25] = px, pz, ap, ro
            rows[:, 25:29], rows[:, 29:33] = new_ap, new_ro
            ev["frifold"].append({"rows": rows})
        elif k == "commit":
            vals = rd(a["pv"][0])[:, 0]
            pvs = vals.astype(np.uint32)
            ev["commit"].append({"pv": vals})
        else:
            raise ValueError(k)
    fp = flatten(prog)
    return ExecutionRecord(prog, fp, _ev_from_legacy(fp, ev), pvs, ev)


# ------------------------------------------------------------------ chips (AIR restatement)

def _ext_expr_mul(a, b):
    """BinomialExtension::mul (crates/stark/src/air/extension.rs:55-75) over Expr components."""
    r = [None] * D
    for i in range(D):
        for j in range(D):
            t = a[i] * b[j]
            if i + j >= D:
                t = W_EXT * t
                k = i + j - D
            else:
                k = i + j
            r[k] = t if r[k] is None else r[k] + t
    return r


def _blk(kind, c0):
    f = main if kind == "main" else prep
    return [f(c0 + k) for k in range(D)]


def _vblk(kind, c0):
    f = V.single_main if kind == "main" else V.single_prep
    return [f(c0 + k) for k in range(D)]


def _single(vcol):
    return [vcol, V.const(0), V.const(0), V.const(0)]


def _mem(addr: V, vals: List[V], mult: V) -> Lookup:
    return Lookup([addr] + vals, mult, KIND_MEMORY)


def mem_const_chip() -> ChipDesc:
    """MemoryConst (mem/constant.rs:142-155): prep = 2 x (value[4], addr, mult); send_block each."""
    c = ChipDesc("MemoryConst", prep_width=12, main_width=1, local_only=True)
    for e in range(2):
        b = 6 * e
        c.sends.append(_mem(V.single_prep(b + 4), _vblk("prep", b), V.single_prep(b + 5)))
    return c


def mem_var_chip() -> ChipDesc:
    """MemoryVar (mem/variable.rs:144-160): prep = 2 x (addr, mult), main = 2 x value[4]."""
    c = ChipDesc("MemoryVar", prep_width=4, main_width=8, local_only=True)
    for e in range(2):
        c.sends.append(_mem(V.single_prep(2 * e), _vblk("main", 4 * e), V.single_prep(2 * e + 1)))
    return c


def _alu_chip(name: str, ext: bool) -> ChipDesc:
    """BaseAlu (alu_base.rs:268-301) / ExtAlu (alu_ext.rs:264-303): 4 entries per row; main entry =
    (out, in1, in2) as felts or blocks; prep entry = (addr out, in1, in2, is_add, is_sub, is_mul, is_div,
    mult)."""
    w = D if ext else 1
    c = ChipDesc(name, prep_width=32, main_width=12 * w, local_only=True)
    for e in range(4):
        mb, pb = 3 * w * e, 8 * e
        out, in1, in2 = ([main(mb + k * w + j) for j in range(w)] for k in range(3))
        is_add, is_sub, is_mul, is_div, mult = (prep(pb + 3 + j) for j in range(5))
        is_real = is_add + is_sub + is_mul + is_div
        c.assert_zero(is_real * (is_real - 1))
        if ext:
            s = [in1[j] + in2[j] for j in range(D)]
            for j in range(D):
                c.assert_zero(is_add * (s[j] - out[j]))
            s = [in2[j] + out[j] for j in range(D)]
            for j in range(D):
                c.assert_zero(is_sub * (in1[j] - s[j]))
            pr = _ext_expr_mul(in1, in2)
            for j in range(D):
                c.assert_zero(is_mul * (pr[j] - out[j]))
            pr = _ext_expr_mul(in2, out)
            for j in range(D):
                c.assert_zero(is_div * (in1[j] - pr[j]))
        else:
            c.assert_zero(is_add * ((in1[0] + in2[0]) - out[0]))
            c.assert_zero(is_sub * (in1[0] - (in2[0] + out[0])))
            c.assert_zero(is_mul * (out[0] - in1[0] * in2[0]))
            c.assert_zero(is_div * (in2[0] * out[0] - in1[0]))
        real = V([("prep", pb + 3 + j, 1) for j in range(4)], 0)
        vals = lambda k: (_vblk("main", mb + k * w) if ext else _single(V.single_main(mb + k)))
        c.receives.append(_mem(V.single_prep(pb + 1), vals(1), real))
        c.receives.append(_mem(V.single_prep(pb + 2), vals(2), real))
        c.sends.append(_mem(V.single_prep(pb + 0), vals(0), V.single_prep(pb + 7)))
    return c


def _m4_expr(x):
    """Poseidon2's M4 block (the x[0..4] -> 4 outputs of apply_m_4, air.rs:31-56), intermediates shared."""
    t01 = (x[0] + x[1]).share()
    t23 = (x[2] + x[3]).share()
    t0123 = (t01 + t23).share()
    t01123 = (t0123 + x[1]).share()
    t01233 = (t0123 + x[3]).share()
    return [t01123 + t01, t01123 + 2 * x[2], t01233 + t23, t01233 + 2 * x[0]]


def _external_layer_expr(s):
    """external_linear_layer: M4 on each 4-block, then every element plus its column's sum over the blocks.
    Each output is a shared node, so the next round reads it once per use (the chained symbolic state
    of air.rs:84-132, shared as Plonky3 shares Rc'd SymbolicExpression nodes)."""
    out = []
    for j in range(0, WIDTH, 4):
        out += [e.share() for e in _m4_expr(s[j:j + 4])]
    sums = [(out[k] + out[4 + k] + out[8 + k] + out[12 + k]).share() for k in range(4)]
    return [(out[j] + sums[j % 4]).share() for j in range(WIDTH)]


def _internal_layer_expr(s):
    """internal_linear_layer: s_i <- d_i s_i + sum(s) with the diagonal DIAG (air.rs:12-29)."""
    tot = s[0]
    for j in range(1, WIDTH):
        tot = tot + s[j]
    tot = tot.share()
    return [(DIAG[i] * s[i] + tot).share() for i in range(WIDTH)]


def poseidon2_wide_chip() -> ChipDesc:
    """Poseidon2WideDeg3 (poseidon2_wide/air.rs:39-179): prep = input addrs[16], (output addr, mult)[16],
    is_real_neg; main = PermutationSBox (313 columns).  The round states are chained symbolic
    expressions as in the reference's eval (external rounds air.rs:84-132, internal rounds :134-170),
    each state element a shared subexpression (OP_LET/OP_GET), so the 13 chained internal layers cost
    one node per element instead of an exponentially growing expression."""
    c = ChipDesc("Poseidon2WideDeg3", prep_width=49, main_width=P2_COLS, local_only=True)
    x = main(P2_EXT)
    c.assert_zero(x * x * x - x * x * x)  # dummy constraint normalising the degree to 3
    for i in range(WIDTH):
        c.sends.append(_mem(V.single_prep(i), _single(V.single_main(P2_EXT + i)), V.single_prep(48)))
    for i in range(WIDTH):
        c.sends.append(_mem(V.single_prep(16 + 2 * i), _single(V.single_main(P2_OUT + i)), V.single_prep(17 + 2 * i)))

    for r in range(NUM_EXTERNAL_ROUNDS):
        st = [main(P2_EXT + r * WIDTH + i) for i in range(WIDTH)]
        if r == 0:
            st = _external_layer_expr(st)
        rnd = r if r < NUM_EXTERNAL_ROUNDS // 2 else r + NUM_INTERNAL_ROUNDS
        sb = []
        for i in range(WIDTH):
            a = (st[i] + RC[rnd][i]).share()
            col = P2_ESBOX + r * WIDTH + i
            c.assert_zero(main(col) - a * a * a)
            sb.append(main(col))
        st = _external_layer_expr(sb)
        if r == NUM_EXTERNAL_ROUNDS // 2 - 1:
            nxt = [P2_INT + i for i in range(WIDTH)]
        elif r == NUM_EXTERNAL_ROUNDS - 1:
            nxt = [P2_OUT + i for i in range(WIDTH)]
        else:
            nxt = [P2_EXT + (r + 1) * WIDTH + i for i in range(WIDTH)]
        for i in range(WIDTH):
            c.assert_zero(main(nxt[i]) - st[i])
    st = [main(P2_INT + i) for i in range(WIDTH)]
    for r in range(NUM_INTERNAL_ROUNDS):
        base = st[0] if r == 0 else main(P2_S0 + r - 1)
        a = (base + RC[r + NUM_EXTERNAL_ROUNDS // 2][0]).share()
        c.assert_zero(main(P2_ISBOX + r) - a * a * a)
        st = _internal_layer_expr([main(P2_ISBOX + r)] + st[1:])
        if r < NUM_INTERNAL_ROUNDS - 1:
            c.assert_zero(main(P2_S0 + r) - st[0])
    r4 = NUM_EXTERNAL_ROUNDS // 2
    for i in range(WIDTH):
        c.assert_zero(main(P2_EXT + r4 * WIDTH + i) - st[i])
    return c


def batch_fri_chip() -> ChipDesc:
    """BatchFRI (batch_fri.rs:292-361): prep = (is_real, is_end, acc, alpha_pow, p_at_z, p_at_x addrs);
    main = (acc[4], alpha_pow[4], p_at_z[4], p_at_x)."""
    c = ChipDesc("BatchFRI", prep_width=6, main_width=13)
    is_real, is_end = prep(0), prep(1)
    c.assert_zero(is_real * is_real * is_real - is_real * is_real * is_real)
    rv = V.single_prep(0)
    c.receives.append(_mem(V.single_prep(3), _vblk("main", 4), rv))
    c.receives.append(_mem(V.single_prep(4), _vblk("main", 8), rv))
    c.receives.append(_mem(V.single_prep(5), _single(V.single_main(12)), rv))
    c.sends.append(_mem(V.single_prep(2), _vblk("main", 0), V.single_prep(1)))

    def term(f):  # alpha_pow * (p_at_z - from_base(p_at_x))
        al = [f(4 + k) for k in range(D)]
        z = [f(8 + k) for k in range(D)]
        z[0] = z[0] - f(12)
        return _ext_expr_mul(al, z)

    t = term(main)
    for k in range(D):
        c.assert_zero(IS_FIRST * (main(k) - t[k]))
    t = term(main_next)
    for k in range(D):
        c.assert_zero(IS_TRANSITION * is_end * (main_next(k) - t[k]))
    for k in range(D):
        c.assert_zero(IS_TRANSITION * (1 - is_end) * (main_next(k) - (main(k) + t[k])))
    return c


def fri_fold_chip() -> ChipDesc:
    """FriFold (fri_fold.rs:371-490): prep = is_first, (addr, mult) of z, alpha, x, alpha_pow_input,
    ro_input, p_at_x, p_at_z, ro_output, alpha_pow_output, is_real; main = z[4], alpha[4], x,
    p_at_x[4], p_at_z[4], alpha_pow_input[4], ro_input[4], alpha_pow_output[4], ro_output[4]."""
    c = ChipDesc("FriFold", prep_width=20, main_width=33)
    is_real = prep(19)
    c.assert_zero(is_real * is_real * is_real - is_real * is_real * is_real)
    keep = lambda: IS_TRANSITION * prep_next(19) * (1 - prep_next(0))
    c.sends.append(_mem(V.single_prep(5), _single(V.single_main(8)), V.single_prep(6)))
    c.assert_zero(keep() * (main(8) - main_next(8)))
    c.sends.append(_mem(V.single_prep(1), _vblk("main", 0), V.single_prep(2)))
    for k in range(D):
        c.assert_zero(keep() * (main(k) - main_next(k)))
    c.sends.append(_mem(V.single_prep(3), _vblk("main", 4), V.single_prep(4)))
    for k in range(D):
        c.assert_zero(keep() * (main(4 + k) - main_next(4 + k)))
    for addr, val in ((7, 17), (9, 21), (13, 13), (11, 9), (17, 25), (15, 29)):
        c.sends.append(_mem(V.single_prep(addr), _vblk("main", val), V.single_prep(addr + 1)))
    alpha, old_ap, new_ap = _blk("main", 4), _blk("main", 17), _blk("main", 25)
    t = _ext_expr_mul(old_ap, alpha)
    for k in range(D):
        c.assert_zero(t[k] - new_ap[k])
    z, px, pz, old_ro, new_ro = _blk("main", 0), _blk("main", 9), _blk("main", 13), _blk("main", 21), _blk("main", 29)
    xz = [main(8) - z[0]] + [0 - z[k] for k in range(1, D)]
    lhs = _ext_expr_mul([new_ro[k] - old_ro[k] for k in range(D)], xz)
    rhs = _ext_expr_mul([px[k] - pz[k] for k in range(D)], old_ap)
    for k in range(D):
        c.assert_zero(lhs[k] - rhs[k])
    return c


def select_chip() -> ChipDesc:
    """Select (select.rs:229-251): prep = (is_real, bit, out1, out2, in1, in2 addrs, mult1, mult2);
    main = (bit, out1, out2, in1, in2)."""
    c = ChipDesc("Select", prep_width=8, main_width=5, local_only=True)
    rv = V.single_prep(0)
    c.receives.append(_mem(V.single_prep(1), _single(V.single_main(0)), rv))
    c.receives.append(_mem(V.single_prep(4), _single(V.single_main(3)), rv))
    c.receives.append(_mem(V.single_prep(5), _single(V.single_main(4)), rv))
    c.sends.append(_mem(V.single_prep(2), _single(V.single_main(1)), V.single_prep(6)))
    c.sends.append(_mem(V.single_prep(3), _single(V.single_main(2)), V.single_prep(7)))
    bit, o1, o2, i1, i2 = (main(j) for j in range(5))
    c.assert_zero(o1 - (bit * i2 + (1 - bit) * i1))
    c.assert_zero(o2 - (bit * i1 + (1 - bit) * i2))
    return c


def exp_reverse_bits_chip() -> ChipDesc:
    """ExpReverseBitsLen (exp_reverse_bits.rs:355-452): prep = (x, exponent, result) (addr, mult),
    iteration_num, is_first, is_last, is_real; main = (x, current_bit, prev_accum_squared,
    prev_accum_squared_times_multiplier, accum, accum_squared, multiplier)."""
    c = ChipDesc("ExpReverseBitsLen", prep_width=10, main_width=7)
    x, bit, psq, psqm, acc, accsq, mult = (main(j) for j in range(7))
    is_first, is_last, is_real = prep(7), prep(8), prep(9)
    c.sends.append(_mem(V.single_prep(0), _single(V.single_main(0)), V.single_prep(1)))
    c.assert_zero(IS_TRANSITION * prep_next(9) * (1 - is_last) * (x - main_next(0)))
    c.sends.append(_mem(V.single_prep(2), _single(V.single_main(1)), V.single_prep(3)))
    c.assert_zero(is_first * (acc - mult))
    c.assert_zero(is_real * bit * (mult - x))
    c.assert_zero(is_real * (1 - bit) * (mult - 1))
    c.assert_zero(is_real * (psqm - psq * mult))
    c.assert_zero(is_real * (1 - is_first) * (acc - psqm))
    c.assert_zero(is_real * (accsq - acc * acc))
    c.assert_zero(IS_TRANSITION * prep_next(9) * (1 - is_last) * (main_next(2) - accsq))
    c.sends.append(_mem(V.single_prep(4), _single(V.single_main(4)), V.single_prep(5)))
    return c


def public_values_chip() -> ChipDesc:
    """PublicValues (public_values.rs:289-310): prep = (pv_idx[8], pv_mem addr, mult); main = pv_element."""
    c = ChipDesc("PublicValues", prep_width=10, main_width=1)
    c.sends.append(_mem(V.single_prep(8), _single(V.single_main(0)), V.single_prep(9)))
    for i in range(DIGEST_SIZE):
        c.assert_zero(prep(i) * (pv(PV_DIGEST_START + i) - main(0)))
    return c


def compress_machine() -> MachineDesc:
    """RecursionAir::<F, 3>::compress_machine (machine.rs:112-128), observing all 231 public values."""
    return MachineDesc([mem_const_chip(), mem_var_chip(), _alu_chip("BaseAlu", False), _alu_chip("ExtAlu", True),
                        poseidon2_wide_chip(), batch_fri_chip(), select_chip(), exp_reverse_bits_chip(),
                        public_values_chip()], PROOF_MAX_NUM_PVS, pc_start=0)


def wide_machine() -> MachineDesc:
    """RecursionAir::<F, 3>::machine_wide_with_all_chips (machine.rs:68-87): the compress chips plus FriFold."""
    return MachineDesc([mem_const_chip(), mem_var_chip(), _alu_chip("BaseAlu", False), _alu_chip("ExtAlu", True),
                        poseidon2_wide_chip(), fri_fold_chip(), batch_fri_chip(), select_chip(), exp_reverse_bits_chip(),
                        public_values_chip()], PROOF_MAX_NUM_PVS, pc_start=0)


# ------------------------------------------------------------------ traces

def _pow2(n: int, fixed: Optional[int] = None) -> int:
    """core/machine/src/utils/mod.rs:99-121 next_power_of_two (>= 16) or the shape's fixed height."""
    if fixed is not None:
        if n > (1 << fixed):
            raise ValueError(f"fixed log2 rows is too small: got {n}, expected {1 << fixed}")
        return 1 << fixed
    return max(16, 1 << max(0, (n - 1).bit_length()))


def _neg(m):
    return (P - np.asarray(m, np.int64) % P) % P


def _cat(xs, shape_tail, dtype=U):
    return np.concatenate(xs) if xs else np.zeros((0,) + shape_tail, dtype)


# main-trace layouts of the chips whose rows are their events (event_to_row of alu_base.hpp, alu_ext.hpp,
# batch_fri.hpp, select.hpp, fri_fold.hpp, exp_reverse_bits.hpp, public_values.hpp, mem/variable.rs):
# chip -> (event kind, entries per row); a row is its entries' event rows side by side, padding rows zero
MAIN_LAYOUT = {"MemoryVar": ("hint", 2), "BaseAlu": ("base", 4), "ExtAlu": ("ext", 4), "BatchFRI": ("batchfri", 1),
               "Select": ("select", 1), "ExpReverseBitsLen": ("exprev", 1), "FriFold": ("frifold", 1),
               "PublicValues": ("commit", 1)}


def _heights(rec: ExecutionRecord, shape: Dict[str, int]) -> Dict[str, int]:
    n, rows = rec.flat.n, rec.flat.rows
    need = {"MemoryConst": (n["mem"] + 1) // 2, "MemoryVar": (n["hint"] + 1) // 2, "BaseAlu": (n["base"] + 3) // 4,
            "ExtAlu": (n["ext"] + 3) // 4, "Poseidon2WideDeg3": n["p2"], "BatchFRI": rows["batchfri"],
            "FriFold": rows["frifold"], "Select": n["select"], "ExpReverseBitsLen": rows["exprev"],
            "PublicValues": 1 << PUB_VALUES_LOG_HEIGHT}
    return {k: _pow2(v, shape.get(k)) for k, v in need.items()}


def main_events(rec: ExecutionRecord, name: str) -> np.ndarray:
    """The event rows (entries x width, uint32 canonical) chip `name`'s main trace lays out (MAIN_LAYOUT)."""
    kind, _ = MAIN_LAYOUT[name]
    if kind == "hint":
        return rec.flat.a["hint"]["vals"]
    if kind == "commit":
        e = rec.ev["commit"]
        return (e[0, PV_DIGEST_START:PV_DIGEST_START + DIGEST_SIZE][:, None] if len(e)
                else np.zeros((0, 1), np.uint32))
    return rec.ev[kind]


def _lay_out(entries: np.ndarray, epr: int, h: int) -> np.ndarray:
    t = np.zeros((h, epr * entries.shape[1]), np.uint32)
    t.reshape(-1)[:entries.size] = entries.reshape(-1)
    return t


def _mod(m):
    return (np.asarray(m, np.int64) % P).astype(np.uint32)


def prep_traces(rec: ExecutionRecord, shape: Optional[Dict[str, int]] = None) -> Dict[str, np.ndarray]:
    """The preprocessed traces (instr_to_row of the reference's include/*.hpp, mem/{constant,variable}.rs),
    row-major uint32 canonical, padded to the shape's heights (zero rows)."""
    shape = shape or {}
    a, h = rec.flat.a, _heights(rec, shape)
    out = {}
    m = a["mem"]
    mm = np.where(m["write"].astype(bool), _mod(m["mult"]), _mod(-np.asarray(m["mult"], np.int64)))
    ent = np.concatenate([m["vals"], m["addr"][:, None].astype(np.uint32), mm[:, None]], 1) if len(mm) else \
        np.zeros((0, 6), np.uint32)
    out["MemoryConst"] = _lay_out(ent, 2, h["MemoryConst"])
    hn = a["hint"]
    out["MemoryVar"] = _lay_out(np.stack([hn["addr"].astype(np.uint32), _mod(hn["mult"])], 1).reshape(-1, 2), 2,
                                h["MemoryVar"])
    for kind, name in (("base", "BaseAlu"), ("ext", "ExtAlu")):
        x = a[kind]
        k = len(x["out"])
        e = np.zeros((k, 8), np.uint32)
        e[:, 0], e[:, 1], e[:, 2] = x["out"], x["in1"], x["in2"]
        e[np.arange(k), 3 + x["op"]] = 1
        e[:, 7] = _mod(x["mult"])
        out[name] = _lay_out(e, 4, h[name])
    x = a["p2"]
    k = len(x["out"])
    e = np.zeros((k, 49), np.uint32)
    e[:, 0:16] = x["inp"]
    e[:, 16:48:2] = x["out"]
    e[:, 17:48:2] = _mod(x["mult"])
    e[:, 48] = P - 1
    out["Poseidon2WideDeg3"] = _lay_out(e, 1, h["Poseidon2WideDeg3"])
    # BatchFRI / ExpReverseBitsLen: entry q spans L_q rows; i = row within the entry
    for kind, name in (("batchfri", "BatchFRI"), ("exprev", "ExpReverseBitsLen")):
        x = a[kind]
        L = x["L"]
        q = np.repeat(np.arange(len(L)), L)
        i = np.arange(len(q)) - np.repeat(np.cumsum(L) - L, L)
        first, last = i == 0, i == L[q] - 1
        if kind == "batchfri":
            e = np.zeros((len(q), 6), np.uint32)
            e[:, 0] = 1
            e[:, 1] = last
            e[:, 2] = x["acc"][q]
            e[:, 3], e[:, 4], e[:, 5] = x["alpha_pow"], x["p_at_z"], x["p_at_x"]
        else:
            e = np.zeros((len(q), 10), np.uint32)
            e[:, 0] = x["base"][q]
            e[:, 1] = np.where(first, P - 1, 0)
            e[:, 2] = x["exps"]
            e[:, 3] = P - 1
            e[:, 4] = x["result"][q]
            e[:, 5] = np.where(last, _mod(x["mult"])[q], 0)
            e[:, 6] = i
            e[:, 7], e[:, 8], e[:, 9] = first, last, 1
        out[name] = _lay_out(e, 1, h[name])
    x = a["frifold"]
    L = x["L"]
    q = np.repeat(np.arange(len(L)), L)
    first = (np.arange(len(q)) - np.repeat(np.cumsum(L) - L, L)) == 0
    e = np.zeros((len(q), 20), np.uint32)
    fm = np.where(first, P - 1, 0)
    e[:, 0] = first
    e[:, 1], e[:, 2] = x["z"][q], fm
    e[:, 3], e[:, 4] = x["alpha"][q], fm
    e[:, 5], e[:, 6] = x["x"][q], fm
    for c, nm in ((7, "alpha_pow_in"), (9, "ro_in"), (11, "p_at_x"), (13, "p_at_z")):
        e[:, c], e[:, c + 1] = x[nm], P - 1
    e[:, 15], e[:, 16] = x["ro_out"], _mod(x["rom"])
    e[:, 17], e[:, 18] = x["alpha_pow_out"], _mod(x["apm"])
    e[:, 19] = 1
    out["FriFold"] = _lay_out(e, 1, h["FriFold"])
    x = a["select"]
    e = np.stack([np.ones(len(x["bit"]), np.int64), x["bit"], x["out1"], x["out2"], x["in1"], x["in2"],
                  np.asarray(x["mult1"]) % P, np.asarray(x["mult2"]) % P], 1).astype(np.uint32).reshape(-1, 8)
    out["Select"] = _lay_out(e, 1, h["Select"])
    e = np.zeros((0, 10), np.uint32)
    if len(a["commit"]["pv"]):
        e = np.zeros((DIGEST_SIZE, 10), np.uint32)
        e[np.arange(DIGEST_SIZE), np.arange(DIGEST_SIZE)] = 1
        e[:, 8] = a["commit"]["pv"][0, PV_DIGEST_START:PV_DIGEST_START + DIGEST_SIZE]
        e[:, 9] = P - 1
    out["PublicValues"] = _lay_out(e, 1, h["PublicValues"])
    return out


# the FlatProgram arrays prep_traces reads (everything but the hinted values): with the heights they fix
# the preprocessed traces, so nodes with equal keys share one proving key
_PREP_INPUTS = {"mem": ("addr", "vals", "write", "mult"), "hint": ("addr", "mult"),
                "base": ("op", "out", "in1", "in2", "mult"), "ext": ("op", "out", "in1", "in2", "mult"),
                "p2": ("inp", "out", "mult"), "batchfri": ("acc", "alpha_pow", "p_at_z", "p_at_x", "L"),
                "exprev": ("base", "exps", "result", "mult", "L"),
                "frifold": ("x", "z", "alpha", "p_at_x", "p_at_z", "alpha_pow_in", "ro_in", "alpha_pow_out", "ro_out",
                            "apm", "rom", "L"),
                "select": ("bit", "out1", "out2", "in1", "in2", "mult1", "mult2"), "commit": ("pv",)}


def prep_key(rec: ExecutionRecord, shape: Optional[Dict[str, int]] = None) -> bytes:
    """Identity of the program's preprocessed traces without building them: xxh3-128 over the heights and
    every array prep_traces reads (tests/test_recursion.py checks equal keys give equal traces)."""
    import xxhash
    h = xxhash.xxh3_128()
    h.update(repr(sorted(_heights(rec, shape or {}).items())).encode())
    for k in sorted(_PREP_INPUTS):
        for nm in _PREP_INPUTS[k]:
            v = np.ascontiguousarray(rec.flat.a[k][nm])
            h.update(f"{k}.{nm}{v.shape}{v.dtype}".encode())
            h.update(_array_digest(v))
    return h.digest()


_DIGESTS: "OrderedDict[int, tuple]" = OrderedDict()  # id -> (array, xxh3-128 of its bytes): large arrays


def _array_digest(v: np.ndarray) -> bytes:
    """xxh3-128 of an array's bytes, memoised for large arrays by identity (a node on a program template shares
    the template's instruction arrays, recursion_verifier.node_flat, which nothing writes to; the entry holds
    the array, so its id is not reused while the entry lives)."""
    import xxhash
    if v.size < (1 << 15):
        return xxhash.xxh3_128(v.view(np.uint8).data).digest()
    e = _DIGESTS.get(id(v))
    if e is not None and e[0] is v:
        _DIGESTS.move_to_end(id(v))
        return e[1]
    d = xxhash.xxh3_128(v.view(np.uint8).data).digest()
    _DIGESTS[id(v)] = (v, d)
    while len(_DIGESTS) > 256:
        _DIGESTS.popitem(last=False)
    return d


def prep_records(rec: ExecutionRecord, shape: Optional[Dict[str, int]] = None) -> Dict[str, tuple]:
    """The preprocessed traces as instruction records for the device (tracegen.recursion_instrs_trace,
    zkm_recursion_instrs_to_trace): chip -> (records n x words uint32, height).  Laid out by the kernel they
    are prep_traces (tests/test_recursion.py checks it on the GPU)."""
    shape = shape or {}
    a, h = rec.flat.a, _heights(rec, shape)
    u = lambda x: np.asarray(x, np.int64).astype(np.uint32)
    out = {}
    m = a["mem"]
    mm = np.where(m["write"].astype(bool), _mod(m["mult"]), _mod(-np.asarray(m["mult"], np.int64)))
    out["MemoryConst"] = np.concatenate([m["vals"].astype(np.uint32).reshape(-1, 4), u(m["addr"])[:, None],
                                         mm[:, None]], 1)
    out["MemoryVar"] = np.stack([u(a["hint"]["addr"]), _mod(a["hint"]["mult"])], 1)
    for kind, name in (("base", "BaseAlu"), ("ext", "ExtAlu")):
        x = a[kind]
        out[name] = np.stack([u(x["out"]), u(x["in1"]), u(x["in2"]), u(x["op"]), _mod(x["mult"])], 1)
    x = a["p2"]
    out["Poseidon2WideDeg3"] = np.concatenate([u(x["inp"]).reshape(-1, WIDTH), u(x["out"]).reshape(-1, WIDTH),
                                               _mod(x["mult"]).reshape(-1, WIDTH)], 1)
    for kind, name in (("batchfri", "BatchFRI"), ("exprev", "ExpReverseBitsLen")):
        x = a[kind]
        L = x["L"]
        q = np.repeat(np.arange(len(L)), L)
        i = np.arange(len(q)) - np.repeat(np.cumsum(L) - L, L)
        if kind == "batchfri":
            out[name] = np.stack([u(x["acc"][q]), u(x["alpha_pow"]), u(x["p_at_z"]), u(x["p_at_x"]),
                                  (i == L[q] - 1).astype(np.uint32)], 1)
        else:
            out[name] = np.stack([u(x["base"][q]), u(x["exps"]), u(x["result"][q]), _mod(x["mult"])[q],
                                  i.astype(np.uint32), L[q].astype(np.uint32)], 1)
    x = a["frifold"]
    L = x["L"]
    q = np.repeat(np.arange(len(L)), L)
    first = (np.arange(len(q)) - np.repeat(np.cumsum(L) - L, L)) == 0
    out["FriFold"] = np.stack([u(x["z"][q]), u(x["alpha"][q]), u(x["x"][q]), u(x["alpha_pow_in"]), u(x["ro_in"]),
                               u(x["p_at_x"]), u(x["p_at_z"]), u(x["ro_out"]), _mod(x["rom"]), u(x["alpha_pow_out"]),
                               _mod(x["apm"]), first.astype(np.uint32)], 1)
    pv = a["commit"]["pv"]
    out["Select"] = np.stack([u(a["select"][f]) for f in ("bit", "out1", "out2", "in1", "in2")]
                             + [_mod(a["select"]["mult1"]), _mod(a["select"]["mult2"])], 1)
    out["PublicValues"] = (u(pv[0, PV_DIGEST_START:PV_DIGEST_START + DIGEST_SIZE])[:, None] if len(pv)
                           else np.zeros((0, 1), np.uint32))
    from .tracegen import RECURSION_INSTR_CHIPS as RIC
    return {k: (np.ascontiguousarray(v.reshape(len(v), RIC[k][1]).astype(np.uint32)), h[k]) for k, v in out.items()}


def main_traces(rec: ExecutionRecord, shape: Optional[Dict[str, int]] = None, p2_main: bool = True):
    """The main traces on the host (event_to_row layouts, padding rows zero; Poseidon2WideDeg3's padding
    rows are the permutation of zero, trace.rs), row-major uint32 canonical."""
    shape = shape or {}
    h = _heights(rec, shape)
    out = {"MemoryConst": np.zeros((h["MemoryConst"], 1), np.uint32)}
    for name, (_, epr) in MAIN_LAYOUT.items():
        out[name] = _lay_out(main_events(rec, name), epr, h[name])
    if p2_main:
        hp = h["Poseidon2WideDeg3"]
        mn = np.zeros((hp, P2_COLS), np.uint32)
        ins = rec.ev["p2"][:, :WIDTH]
        mn[:len(ins)] = poseidon2_rows(ins.astype(U)).astype(np.uint32)
        mn[len(ins):] = poseidon2_rows(np.zeros((1, WIDTH), U)).astype(np.uint32)
        out["Poseidon2WideDeg3"] = mn
    return out


def generate_traces(rec: ExecutionRecord, shape: Optional[Dict[str, int]] = None, p2_main: bool = True):
    """(prep_traces, main_traces) by chip name, row-major uint32 canonical.  p2_main=False leaves out the
    Poseidon2WideDeg3 main trace (313 columns, the largest) for the caller to build on the device from the
    permutation inputs (`p2_inputs`, tracegen.poseidon2_wide_trace)."""
    return prep_traces(rec, shape), main_traces(rec, shape, p2_main)


# RecursionShapeConfig::default (crates/recursion/core/src/shape.rs:115-170): the compress programs'
# allowed shapes (log2 heights), fastest first
RECURSION_SHAPES = [
    {"MemoryVar": 18, "Select": 18, "MemoryConst": 16, "BatchFRI": 17, "BaseAlu": 15, "ExtAlu": 15,
     "ExpReverseBitsLen": 17, "Poseidon2WideDeg3": 16, "PublicValues": PUB_VALUES_LOG_HEIGHT},
    {"MemoryVar": 19, "Select": 19, "MemoryConst": 17, "BatchFRI": 19, "BaseAlu": 16, "ExtAlu": 16,
     "ExpReverseBitsLen": 18, "Poseidon2WideDeg3": 17, "PublicValues": PUB_VALUES_LOG_HEIGHT},
    {"MemoryVar": 20, "Select": 20, "MemoryConst": 18, "BatchFRI": 21, "BaseAlu": 16, "ExtAlu": 19,
     "ExpReverseBitsLen": 18, "Poseidon2WideDeg3": 18, "PublicValues": PUB_VALUES_LOG_HEIGHT},
]


def program_heights(prog: RecursionProgram) -> Dict[str, int]:
    """RecursionAir::heights (crates/recursion/core/src/machine.rs): the rows each compress-machine chip
    needs for the program's instructions, before padding."""
    n = {k: 0 for k in ("mem", "hint", "base", "ext", "p2", "batchfri", "select", "exprev")}
    if isinstance(prog, FlatProgram):
        n.update({k: prog.n[k] for k in ("mem", "hint", "base", "ext", "p2", "select")})
        n.update({k: prog.rows[k] for k in ("batchfri", "exprev")})
    for b in ([] if isinstance(prog, FlatProgram) else prog.blocks):
        a = b.a
        if b.kind == "mem":
            n["mem"] += len(a["addr"])
        elif b.kind in ("hint", "base", "ext", "select"):
            n[b.kind] += len(next(iter(a.values())))
        elif b.kind == "p2":
            n["p2"] += a["out"].shape[0]
        elif b.kind == "batchfri":
            n["batchfri"] += a["p_at_x"].size
        elif b.kind == "exprev":
            n["exprev"] += a["exps"].size
    return {"MemoryConst": (n["mem"] + 1) // 2, "MemoryVar": (n["hint"] + 1) // 2, "BaseAlu": (n["base"] + 3) // 4,
            "ExtAlu": (n["ext"] + 3) // 4, "Poseidon2WideDeg3": n["p2"], "BatchFRI": n["batchfri"],
            "Select": n["select"], "ExpReverseBitsLen": n["exprev"], "PublicValues": 1 << PUB_VALUES_LOG_HEIGHT}


def fix_shape(prog: RecursionProgram, shapes=None) -> Dict[str, int]:
    """RecursionShapeConfig::fix_shape (shape.rs:50-75): the first allowed shape every chip's height fits;
    an error (the reference panics) when none does."""
    heights = program_heights(prog)
    for sh in (shapes or RECURSION_SHAPES):
        if all(h <= (1 << sh[k]) for k, h in heights.items()):
            return dict(sh)
    raise ValueError(f"no recursion shape found for heights: {heights}")


def shard_parts(prog: RecursionProgram, shape: Optional[Dict[str, int]] = None):
    """A compress-machine shard whose Poseidon2WideDeg3 main trace is left for the device: (machine,
    prep_traces, traces without that chip, public values, the permutation inputs (n x 16), its height)."""
    rec = execute(prog)
    pr, tr = generate_traces(rec, shape, p2_main=False)
    m = compress_machine()
    if rec.flat.n["frifold"]:
        raise ValueError("FriFold instructions need the wide machine")
    pr = {c.name: pr[c.name] for c in m.chips if c.prep_width}
    tr.pop("FriFold", None)
    return m, pr, tr, rec.public_values, p2_inputs(rec), pr["Poseidon2WideDeg3"].shape[0]


def shard(prog: RecursionProgram, shape: Optional[Dict[str, int]] = None, wide: bool = False):
    """(machine, prep_traces, traces, public_values) of one compress-machine shard of ``prog`` (or of the
    wide machine with FriFold, ``wide=True``)."""
    rec = execute(prog)
    pr, tr = generate_traces(rec, shape)
    m = wide_machine() if wide else compress_machine()
    if not wide:
        if rec.flat.n["frifold"]:
            raise ValueError("FriFold instructions need the wide machine")
        pr.pop("FriFold", None)
        tr.pop("FriFold", None)
    pr = {c.name: pr[c.name] for c in m.chips if c.prep_width}
    return m, pr, tr, rec.public_values


# ------------------------------------------------------------------ programs

def _rand(rng, shape):
    return rng.integers(0, P, size=shape, dtype=np.int64).astype(U)


def _rand_ext_nonzero(rng, n):
    x = _rand(rng, (n, D))
    x[:, 0] |= U(1)
    return x


def program_basic_mem() -> RecursionProgram:
    """mem/constant.rs:212-221 prove_basic_mem: Write 2 at 1 (mult 1), Read it once."""
    p = RecursionProgram(num_addrs=2)
    p.mem_write([1], [[2, 0, 0, 0]], mult=1)
    p.mem_read([1], [[2, 0, 0, 0]], mult=1)
    return p


def program_base_four_ops(n: int = 1000, seed: int = 0xDEADBEEF) -> RecursionProgram:
    """alu_base.rs:332-366 four_ops: per round write in1 = in2*quot, in2 (mult 4), then Add/Sub/Mul/Div
    and read each result back."""
    rng = np.random.default_rng(seed)
    quot, in2 = _rand(rng, n), _rand(rng, n) | U(1)
    in1 = _m(in2, quot)
    p = RecursionProgram()
    a = p.alloc(6 * n).reshape(n, 6)
    blk = lambda v: np.stack([v, v * 0, v * 0, v * 0], 1)
    p.mem_write(a[:, 0], blk(in1), mult=4)
    p.mem_write(a[:, 1], blk(in2), mult=4)
    ops = [(OP_ADD, (in1 + in2) % PU), (OP_SUB, (in1 + PU - in2) % PU), (OP_MUL, _m(in1, in2)), (OP_DIV, quot)]
    for j, (op, res) in enumerate(ops):
        p.base_alu(op, a[:, 2 + j], a[:, 0], a[:, 1], mult=1)
        p.mem_read(a[:, 2 + j], blk(res), 1)
    return p


def program_ext_four_ops(n: int = 1000, seed: int = 0xDEADBEEF) -> RecursionProgram:
    """alu_ext.rs:339-376 four_ops over the extension field."""
    rng = np.random.default_rng(seed)
    quot, in2 = _rand(rng, (n, D)), _rand_ext_nonzero(rng, n)
    in1 = ext_mul(in2, quot)
    p = RecursionProgram()
    a = p.alloc(6 * n).reshape(n, 6)
    p.mem_write(a[:, 0], in1, mult=4)
    p.mem_write(a[:, 1], in2, mult=4)
    ops = [(OP_ADD, (in1 + in2) % PU), (OP_SUB, (in1 + PU - in2) % PU), (OP_MUL, ext_mul(in1, in2)), (OP_DIV, quot)]
    for j, (op, res) in enumerate(ops):
        p.ext_alu(op, a[:, 2 + j], a[:, 0], a[:, 1], mult=1)
        p.mem_read(a[:, 2 + j], res, 1)
    return p


def program_select(n: int = 1000, seed: int = 0xDEADBEEF) -> RecursionProgram:
    """select.rs:297-330 prove_select."""
    rng = np.random.default_rng(seed)
    in1, in2 = _rand(rng, n), _rand(rng, n)
    bit = rng.integers(0, 2, n).astype(U)
    o1 = np.where(bit == 1, in2, in1)
    o2 = np.where(bit == 1, in1, in2)
    p = RecursionProgram()
    a = p.alloc(5 * n).reshape(n, 5)
    blk = lambda v: np.stack([v, v * 0, v * 0, v * 0], 1)
    p.mem_write(a[:, 0], blk(bit), 1)
    p.mem_write(a[:, 3], blk(in1), 1)
    p.mem_write(a[:, 4], blk(in2), 1)
    p.select(a[:, 0], a[:, 1], a[:, 2], a[:, 3], a[:, 4], 1, 1)
    p.mem_read(a[:, 1], blk(o1), 1)
    p.mem_read(a[:, 2], blk(o2), 1)
    return p


def program_poseidon2(seed: int = 1) -> RecursionProgram:
    """poseidon2_wide/mod.rs:135-202 test_poseidon2: perm([1;16]) and perm(random), outputs read back."""
    rng = np.random.default_rng(seed)
    inputs = np.stack([np.ones(WIDTH, U), _rand(rng, WIDTH)])
    outs = poseidon2_permute(inputs)
    p = RecursionProgram(num_addrs=4 * WIDTH)
    for k in range(2):
        ia = np.arange(2 * k * WIDTH, (2 * k + 1) * WIDTH)
        oa = ia + WIDTH
        p.mem_write(ia, np.stack([inputs[k], *(inputs[k] * 0,) * 3], 1), 1)
        p.poseidon2(oa, ia, np.ones(WIDTH))
        p.mem_read(oa, np.stack([outs[k], *(outs[k] * 0,) * 3], 1), 1)
    return p


def program_exp_reverse_bits(n: int = 100, bits: int = 16, seed: int = 7) -> RecursionProgram:
    """exp_reverse_bits.rs tests: x^{rev_len(e)} from hinted bits, result read back."""
    rng = np.random.default_rng(seed)
    x = _rand(rng, n)
    e = rng.integers(0, 1 << bits, n)
    p = RecursionProgram()
    xa, ea, ra = p.alloc(n), p.alloc(n * bits).reshape(n, bits), p.alloc(n)
    blk = lambda v: np.stack([v, v * 0, v * 0, v * 0], 1)
    p.mem_write(xa, blk(x))
    bitv = ((e[:, None] >> np.arange(bits)[None, :]) & 1).astype(U)
    p.hint(ea.ravel(), blk(bitv.ravel()))
    p.exp_reverse_bits(xa, ea, ra, mult=1)
    rev = np.array([int(format(int(v), f"0{bits}b")[::-1], 2) for v in e])
    res = np.array([pow(int(xi), int(r), P) for xi, r in zip(x, rev)], U)
    p.mem_read(ra, blk(res), 1)
    return p


def program_batch_fri(n: int = 20, length: int = 7, seed: int = 3) -> RecursionProgram:
    """BatchFRI instances (runtime/mod.rs:535-576) over hinted alpha powers, p(z) and p(x)."""
    rng = np.random.default_rng(seed)
    p = RecursionProgram()
    al, pz, px, acc = (p.alloc(n * length).reshape(n, length), p.alloc(n * length).reshape(n, length),
                       p.alloc(n * length).reshape(n, length), p.alloc(n))
    alv, pzv = _rand(rng, (n * length, D)), _rand(rng, (n * length, D))
    pxv = _rand(rng, n * length)
    p.hint(al.ravel(), alv)
    p.hint(pz.ravel(), pzv)
    p.mem_write(px.ravel(), np.stack([pxv, pxv * 0, pxv * 0, pxv * 0], 1))
    p.batch_fri(acc, al, pz, px)
    diff = pzv.copy()
    diff[:, 0] = (diff[:, 0] + PU - pxv) % PU
    terms = ext_mul(alv, diff).reshape(n, length, D)
    want = terms.sum(1) % PU
    p.mem_read(acc, want, 1)
    return p


def program_public_values(seed: int = 5) -> RecursionProgram:
    """public_values.rs tests: hint 231 values and commit them; the chip checks the digest."""
    rng = np.random.default_rng(seed)
    p = RecursionProgram()
    a = p.alloc(PROOF_MAX_NUM_PVS)
    v = _rand(rng, PROOF_MAX_NUM_PVS)
    p.hint(a, np.stack([v, v * 0, v * 0, v * 0], 1))
    p.commit_public_values(a)
    return p


def merkle_layers(matrix: np.ndarray) -> List[np.ndarray]:
    """MerkleTreeMmcs over one matrix (kb31_poseidon2.rs:176-177): leaf i = PaddingFreeSponge<16,8,8>
    of row i (state zeroed, each 8-chunk overwrites lanes [0, len), permute; out = lanes 0..8), node =
    TruncatedPermutation(left || right)[0..8].  Layers from the leaves (h x 8) to the root (1 x 8)."""
    M = np.asarray(matrix, U) % PU
    h, w = M.shape
    st = np.zeros((h, WIDTH), U)
    for c in range(0, w, 8):
        chunk = M[:, c:c + 8]
        st[:, :chunk.shape[1]] = chunk
        st = poseidon2_permute(st)
    layers = [st[:, :8].copy()]
    while layers[-1].shape[0] > 1:
        x = layers[-1]
        layers.append(poseidon2_permute(np.concatenate([x[0::2], x[1::2]], 1))[:, :8].copy())
    return layers


def merkle_openings(prog: RecursionProgram, matrix: np.ndarray, indices: Sequence[int], layers=None) -> None:
    """Append the verification of `matrix`'s rows at `indices` against its MMCS root, as the recursion
    verifier does it (recursion/circuit/src/merkle_tree.rs, hash.rs:40-50, builder.rs:167-177): the
    opened rows and the sibling paths are hinted (MemoryVar), the index bits hinted as HintBits
    outputs, each row is absorbed by Poseidon2 permutations, each level orders (node, sibling) by the
    index bit with two Select lanes per digest word and compresses, and the root is read back as a
    constant (MemoryConst): the memory bus only balances if every recomputed root equals it."""
    layers = merkle_layers(matrix) if layers is None else layers
    M = np.asarray(matrix, U) % PU
    h, w = M.shape
    depth = len(layers) - 1
    idx = np.asarray(indices, np.int64)
    q = len(idx)
    blk = lambda v: np.stack([v, v * 0, v * 0, v * 0], -1).reshape(-1, D)
    zero = prog.alloc(1)
    prog.mem_write(zero, blk(np.zeros(1, U)))
    rows = prog.alloc(q * w).reshape(q, w)
    prog.hint(rows.ravel(), blk(M[idx].ravel()))
    state = np.full((q, WIDTH), zero[0], np.int64)
    for c in range(0, w, 8):
        k = min(8, w - c)
        inp = state.copy()
        inp[:, :k] = rows[:, c:c + k]
        out = prog.alloc(q * WIDTH).reshape(q, WIDTH)
        prog.poseidon2(out, inp)
        state = out
    node = state[:, :8]
    if depth:
        bits = prog.alloc(q * depth).reshape(q, depth)
        prog.hint(bits.ravel(), blk(((idx[:, None] >> np.arange(depth)[None, :]) & 1).astype(U).ravel()))
        sib = prog.alloc(q * depth * 8).reshape(q, depth, 8)
        sv = np.stack([layers[l][(idx >> l) ^ 1] for l in range(depth)], 1)
        prog.hint(sib.ravel(), blk(sv.ravel()))
        for l in range(depth):
            left, right = prog.alloc(q * 8).reshape(q, 8), prog.alloc(q * 8).reshape(q, 8)
            prog.select(np.repeat(bits[:, l], 8), left.ravel(), right.ravel(), node.ravel(), sib[:, l].ravel())
            out = prog.alloc(q * WIDTH).reshape(q, WIDTH)
            prog.poseidon2(out, np.concatenate([left, right], 1))
            node = out[:, :8]
    root = layers[-1][0]
    prog.mem_read(node.ravel(), blk(np.tile(root, q)), 1)


def program_merkle_openings(log_h: int = 8, width: int = 21, queries: int = 16, seed: int = 9):
    """Merkle openings of a random log_h x width matrix at `queries` random rows (``merkle_openings``);
    returns (program, matrix) so tests can pin the root to the MMCS."""
    rng = np.random.default_rng(seed)
    mat = _rand(rng, (1 << log_h, width))
    p = RecursionProgram()
    merkle_openings(p, mat, rng.integers(0, 1 << log_h, queries))
    return p, mat


def program_fri_fold(n: int = 8, m: int = 5, seed: int = 4) -> RecursionProgram:
    """FriFold instructions (fri_fold.rs tests): n folds of m entries each over hinted z, alpha, x,
    openings and running (alpha_pow, ro), the outputs read back."""
    rng = np.random.default_rng(seed)
    p = RecursionProgram()
    for _ in range(n):
        x_a, z_a, al_a = p.alloc(1), p.alloc(1), p.alloc(1)
        ins = [p.alloc(m) for _ in range(4)]
        outs = [p.alloc(m) for _ in range(2)]
        xv = _rand(rng, 1)
        p.hint(x_a, np.stack([xv, xv * 0, xv * 0, xv * 0], 1))
        zv, alv = _rand(rng, (1, D)), _rand(rng, (1, D))
        p.hint(z_a, zv)
        p.hint(al_a, alv)
        vals = [_rand(rng, (m, D)) for _ in range(4)]
        for a_, v_ in zip(ins, vals):
            p.hint(a_, v_)
        p.fri_fold(x_a[0], z_a[0], al_a[0], ins[0], ins[1], ins[2], ins[3], outs[0], outs[1],
                   alpha_pow_mults=np.ones(m), ro_mults=np.ones(m))
        px, pz, ap, ro = vals
        xz = (PU - zv) % PU
        xz[0, 0] = (xz[0, 0] + xv[0]) % PU
        q = ext_mul((px + PU - pz) % PU, ext_inv(np.repeat(xz, m, 0)))
        p.mem_read(outs[1], (ro + ext_mul(ap, q)) % PU, 1)
        p.mem_read(outs[0], ext_mul(ap, np.repeat(alv, m, 0)), 1)
    return p


# The reference's fixed shape of the shrink/compress machine (machine.rs:155-171 shrink_shape)
SHRINK_SHAPE = {"MemoryVar": 18, "Select": 18, "MemoryConst": 17, "BatchFRI": 17, "BaseAlu": 17, "ExtAlu": 15,
                "ExpReverseBitsLen": 17, "Poseidon2WideDeg3": 16, "PublicValues": PUB_VALUES_LOG_HEIGHT}


def program_verifier_shaped(shape: Dict[str, int] = SHRINK_SHAPE, fill: float = 0.9, seed: int = 11) -> RecursionProgram:
    """A recursion program with the instruction mix of a verifier program that fills each chip of
    ``shape`` to ``fill``: Merkle openings of a committed matrix verified against its root
    (``merkle_openings``: hinted rows and paths, Poseidon2 sponge and compressions, Select ordering by the
    index bits), more hinted proof data (MemoryVar) and Poseidon2 sponge chains over it (the
    transcript), the index bits of the queries (ExpReverseBitsLen), selects (Select),
    FRI reduced openings (BatchFRI), base/extension arithmetic (BaseAlu / ExtAlu) and constants
    (MemoryConst), ending with CommitPublicValues.  Every value is produced by the runtime."""
    rng = np.random.default_rng(seed)
    cap = lambda name, per_row=1: int(fill * (1 << shape[name])) * per_row
    p = RecursionProgram()
    blk = lambda v: np.stack([v, v * 0, v * 0, v * 0], 1)

    n_p2 = cap("Poseidon2WideDeg3")
    n_ext = cap("ExtAlu", 4)
    n_base = cap("BaseAlu", 4)
    n_sel = cap("Select")
    erb_len = 22
    n_erb = cap("ExpReverseBitsLen") // erb_len
    fri_len = 64
    n_fri = cap("BatchFRI") // fri_len
    n_var = cap("MemoryVar", 2)
    n_const = cap("MemoryConst", 2)

    # Merkle openings of a committed matrix (the inner proofs' query openings): a 2^mlog-row, 16-column
    # matrix, rows at random indices verified against its root; they take the Select budget (8 lanes per
    # level) and part of the Poseidon2 budget
    mlog = max(4, min(16, shape["Poseidon2WideDeg3"] - 2))
    per_q = 2 + mlog
    spare_var = n_var - 2 * n_fri * fri_len - n_erb * erb_len - PROOF_MAX_NUM_PVS  # after the other hints
    n_q = max(1, min(n_sel // (8 * mlog), n_p2 // (2 * per_q), (spare_var // 2) // (16 + 9 * mlog)))
    mat = _rand(rng, (1 << mlog, 16))
    merkle_openings(p, mat, rng.integers(0, 1 << mlog, n_q))
    n_sel = max(1, n_sel - n_q * 8 * mlog)
    n_p2 = max(64, n_p2 - n_q * per_q)
    n_var = max(0, n_var - n_q * (16 + 9 * mlog))  # rows, index bits, sibling digests
    n_const = max(32, n_const - 1 - 8 * n_q)  # the zero constant, the roots read back

    # hinted proof data: ext blocks (alpha powers, p(z)) and felts (p(x), sponge input, bits)
    n_hint_ext = 2 * n_fri * fri_len
    n_bits = n_erb * erb_len
    n_hint_felt = max(0, n_var - n_hint_ext - n_bits - PROOF_MAX_NUM_PVS)
    ext_a = p.alloc(n_hint_ext)
    p.hint(ext_a, _rand(rng, (n_hint_ext, D)))
    bits_a = p.alloc(n_bits)
    p.hint(bits_a, blk(rng.integers(0, 2, n_bits).astype(U)))
    felt_a = p.alloc(n_hint_felt)
    p.hint(felt_a, blk(_rand(rng, n_hint_felt)))

    # constants (MemoryConst writes, read by the ALUs); the rest of MemoryConst: read-backs below
    n_cw = max(16, n_const // 2)
    const_a = p.alloc(n_cw)
    p.mem_write(const_a, blk(_rand(rng, n_cw) | U(1)))

    # Poseidon2 sponge: chains of permutations absorbing hinted felts; 8 lanes of capacity carried
    chains = 64
    per = n_p2 // chains
    state = np.stack([felt_a[(np.arange(chains) * 16 + i) % max(1, n_hint_felt)] for i in range(WIDTH)], 1)
    absorb = 0
    p2_outs = []
    for r in range(per):
        out = p.alloc(chains * WIDTH).reshape(chains, WIDTH)
        p.poseidon2(out, state)
        p2_outs.append(out)
        nxt = out.copy()
        idx = (chains * 8 * r + np.arange(chains * 8) + absorb) % max(1, n_hint_felt)
        nxt[:, :8] = felt_a[idx].reshape(chains, 8)
        state = nxt
    p2_last = p2_outs[-1] if p2_outs else const_a[:chains * WIDTH].reshape(-1, WIDTH)

    # base ALU: mix hinted felts with constants and permutation outputs (4 ops, no division by unknowns)
    src = np.concatenate([felt_a, p2_last.ravel()]) if n_hint_felt else p2_last.ravel()
    out_b = p.alloc(n_base)
    ops = rng.integers(0, 3, n_base)
    div_every = 16
    ops[::div_every] = OP_DIV  # division by a (non-zero) constant
    in1 = src[rng.integers(0, len(src), n_base)]
    in2 = np.where(ops == OP_DIV, const_a[rng.integers(0, n_cw, n_base)], src[rng.integers(0, len(src), n_base)])
    p.base_alu(ops, out_b, in1, in2, mult=None)

    # selects on hinted bits (Merkle path ordering)
    sbit = bits_a[np.arange(n_sel) % max(1, n_bits)] if n_bits else const_a[:n_sel]
    s_in1, s_in2 = out_b[rng.integers(0, n_base, n_sel)], src[rng.integers(0, len(src), n_sel)]
    so1, so2 = p.alloc(n_sel), p.alloc(n_sel)
    p.select(sbit, so1, so2, s_in1, s_in2)

    # exp reverse bits: query index powers of a generator-like base from the sponge
    erb_base = src[rng.integers(0, len(src), n_erb)]
    erb_res = p.alloc(n_erb)
    p.exp_reverse_bits(erb_base, bits_a.reshape(n_erb, erb_len), erb_res)

    # batch FRI: reduced openings over hinted alpha powers / p(z) and felt p(x)
    fri_acc = p.alloc(n_fri)
    px = np.concatenate([so1, so2, out_b])[:n_fri * fri_len]
    if len(px) < n_fri * fri_len:
        px = np.resize(px, n_fri * fri_len)
    p.batch_fri(fri_acc, ext_a[:n_fri * fri_len].reshape(n_fri, fri_len),
                ext_a[n_fri * fri_len:].reshape(n_fri, fri_len), px.reshape(n_fri, fri_len))

    # extension ALU: each reduced opening is consumed once (BatchFRI writes acc with multiplicity 1,
    # batch_fri.rs:113), then arithmetic over those sums and the hinted ext values
    out_f = p.alloc(n_fri)
    p.ext_alu(OP_ADD, out_f, fri_acc, ext_a[:n_fri])
    ext_src = np.concatenate([out_f, ext_a])
    n_e = max(0, n_ext - n_fri)
    out_e = p.alloc(n_e)
    eops = rng.integers(0, 3, n_e)
    p.ext_alu(eops, out_e, ext_src[rng.integers(0, len(ext_src), n_e)], ext_src[rng.integers(0, len(ext_src), n_e)])

    # public values: hinted, the digest is the first 8 words of a permutation output
    pv_a = p.alloc(PROOF_MAX_NUM_PVS)
    p.hint(pv_a, blk(_rand(rng, PROOF_MAX_NUM_PVS)))
    pv_addrs = pv_a.copy()
    pv_addrs[PV_DIGEST_START:PV_DIGEST_START + DIGEST_SIZE] = p2_last[0, :DIGEST_SIZE]
    p.commit_public_values(pv_addrs)

    # MemoryConst read-backs of computed values (the verifier's assertions)
    n_rb = max(0, n_const - n_cw)
    if n_rb:
        rec = execute(_copy_program(p))
        pool = np.concatenate([out_b, so1, so2])[:n_rb]
        p.mem_read(pool, rec_mem(rec, pool), 1)
    return p


def _copy_program(p: RecursionProgram) -> RecursionProgram:
    return RecursionProgram([Block(b.kind, {k: v.copy() for k, v in b.a.items()}) for b in p.blocks], p.num_addrs)


def rec_mem(rec: ExecutionRecord, addrs: np.ndarray) -> np.ndarray:
    """Values at ``addrs`` after executing ``rec``'s program (re-derived from its events)."""
    mem = np.zeros((rec.program.num_addrs, D), U)
    bl = rec.program.blocks
    ev_iter = {k: iter(v) for k, v in rec.events.items()}
    for b in bl:
        a, k = b.a, b.kind
        e = next(ev_iter[k]) if k in ev_iter else None
        if k == "mem":
            mem[a["addr"][a["write"]]] = a["vals"][a["write"]]
        elif k == "hint":
            mem[a["addr"]] = a["vals"]
        elif k == "base":
            mem[a["out"], 0] = e["out"]
        elif k == "ext":
            mem[a["out"]] = e["out"]
        elif k == "p2":
            mem[a["out"].ravel(), 0] = e["outputs"].ravel()
        elif k == "select":
            mem[a["out1"], 0] = e["out1"]
            mem[a["out2"], 0] = e["out2"]
        elif k == "exprev":
            mem[a["result"], 0] = e["rows"].reshape(e["n"], e["L"], 7)[:, -1, 4]
        elif k == "batchfri":
            mem[a["acc"]] = e["rows"].reshape(e["n"], e["L"], 13)[:, -1, 0:4]
    return mem[addrs]
