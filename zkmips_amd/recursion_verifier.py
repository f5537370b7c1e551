"""Compress-node programs that verify their child proofs (BASELINE config 5: "batch inner-proof
verification").

The reference's compress node runs the recursion verifier program over its children's ShardProofs
(crates/prover/src/lib.rs:614-954; the program compiled from crates/recursion/circuit/src/stark.rs:246-432,
fri.rs, merkle_tree.rs, challenger.rs).  `verify_shard` appends that verification for one child proof
to a RecursionProgram, with the proof's data as hints (MemoryVar) and the child's verifying key as
constants (MemoryConst):

* the Fiat-Shamir transcript (DuplexChallenger, challenger.rs:60-233) replayed in the program: every
  observed value (public values, the three commitments, the chips' cumulative sums, the FRI commitments,
  the final polynomial, the PoW witness) enters Poseidon2 permutations in the duplexing pattern, and
  the challenges (zeta, the FRI alpha and betas, the query indices) are read from their outputs;
* the proof of work: the low pow_bits bits of the sample after the witness are zero;
* the query indices: HintBits decompositions of the sampled elements, checked by recomposition and
  canonical (< p);
* every query's input openings: the opened rows of the preprocessed, main, permutation and quotient
  batches re-hashed (PaddingFreeSponge) and walked up their Merkle paths with height injection
  (MerkleTreeMmcs verify_batch, fri.rs:363-400) to the committed roots;
* the FRI reduced openings (fri.rs:155-203): per row x = 3 w^rev(i) (ExpReverseBitsLen), BatchFRI
  accumulations sum alpha^k (p(z) - p(x)) over the opened values, divided by (z - x), per height;
* the FRI commit phase (fri.rs:247-361): per round the pair (folded, sibling) ordered by the index bit,
  its leaf hashed and walked to the round's commitment, and the fold
  e0 + (beta - x0)(e1 - e0)/(x1 - x0) + beta^2 ro[h - 1]; the last folded value equals the final
  polynomial, and ro[log_blowup] = 0.

Not in the program (documented in DESIGN.md): the OOD evaluation of every chip's constraints at zeta
against the quotient (verifier.rs:316-397, constraints.rs) and the shape checks the reference's
verifier does before the transcript.  A program built from a proof executes only if every check above
holds: a changed byte of the child proof changes a hinted value, and the runtime's memory reads
(`mem_read` of the expected 0) fail.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import recursion as R
from .machine import P
from .septic import CURVE_CUMULATIVE_SUM_START as S_CURVE_START

U, PU, D = R.U, R.PU, R.D
GENERATOR = 3
W_EXT = 3  # EF = F[X]/(X^4 - 3)


def two_adic_gen(bits: int) -> int:
    return pow(3, (P - 1) >> bits, P)


# ---------------------------------------------------------------- EF arithmetic on ints (host replay)
def ef_mul(a, b):
    r = [0] * 7
    for i in range(4):
        for j in range(4):
            r[i + j] += a[i] * b[j]
    return [(r[k] + (W_EXT * r[k + 4] if k + 4 < 7 else 0)) % P for k in range(4)]


def ef_add(a, b):
    return [(x + y) % P for x, y in zip(a, b)]


def ef_sub(a, b):
    return [(x - y) % P for x, y in zip(a, b)]


def ef_inv(a):
    return [int(v) for v in R.ext_inv(np.asarray([a], U))[0]]


def ef_base(x):
    return [x % P, 0, 0, 0]


# ---------------------------------------------------------------- the proof (bincode ShardProof)
@dataclass
class ChipOpened:
    prep_l: np.ndarray
    prep_n: np.ndarray
    main_l: np.ndarray
    main_n: np.ndarray
    perm_l: np.ndarray
    perm_n: np.ndarray
    quot: np.ndarray  # (chunks, 4, 4): chunk j, column e, EF
    gcs: np.ndarray
    lcs: np.ndarray
    log_degree: int


@dataclass
class ShardProofData:
    main_c: np.ndarray
    perm_c: np.ndarray
    quot_c: np.ndarray
    chips: List[ChipOpened]
    fri_commits: np.ndarray           # (rounds, 8)
    queries: list                     # [(input: [(rows: [np.ndarray], path: (L, 8))] x 4, steps: [(sib EF, path)])]
    final_poly: np.ndarray
    pow_witness: int
    names: List[str]
    pv: np.ndarray
    # the queries' sections stacked over the queries (what the verifier consumes): per input round t the
    # opened rows of matrix k (nq, width) and the Merkle paths (nq, L, 8); per commit-phase step the
    # siblings (nq, 4) and paths (nq, L, 8)
    q_rows: list = None
    q_paths: list = None
    q_sib: list = None
    q_fpath: list = None


def parse_shard_proof(b: bytes) -> ShardProofData:
    """The bincode-1 layout zkm_open writes (zkmips_amd/csrc/prover.cpp `serialize`, crates/stark/src/
    types.rs:77-83): canonical field elements, u64 lengths."""
    p, end = parse_shard_proof_at(b, 0)
    if end != len(b):
        raise ValueError("trailing bytes in the shard proof")
    return p


def parse_shard_proof_at(b: bytes, start: int):
    """One ShardProof starting at byte `start` of b (e.g. inside a Vec<ShardProof>): (data, end offset)."""
    pos = [start]

    def u64():
        v = int.from_bytes(b[pos[0]:pos[0] + 8], "little")
        pos[0] += 8
        return v

    def u32s(n):
        v = np.frombuffer(b, np.uint32, n, pos[0]).astype(np.int64)
        pos[0] += 4 * n
        return v

    def efv():
        n = u64()
        return u32s(4 * n).reshape(n, 4)

    def digests():
        n = u64()
        return u32s(8 * n).reshape(n, 8)

    main_c, perm_c, quot_c = u32s(8), u32s(8), u32s(8)
    chips = []
    for _ in range(u64()):
        pl, pn, ml, mn, rl, rn = (efv() for _ in range(6))
        nq = u64()
        quot = np.stack([efv() for _ in range(nq)]) if nq else np.zeros((0, 4, 4), np.int64)
        gcs, lcs = u32s(14), u32s(4)
        chips.append(ChipOpened(pl, pn, ml, mn, rl, rn, quot, gcs, lcs, u64()))
    fri_commits = digests()
    queries, stacked = _parse_queries(b, pos, u64, u32s, digests)
    final_poly, pow_w = u32s(4), int(u32s(1)[0])
    names = [None] * 0
    order = []
    for _ in range(u64()):
        n = u64()
        nm = b[pos[0]:pos[0] + n].decode()
        pos[0] += n
        order.append((u64(), nm))
    names = [nm for _, nm in sorted(order)]
    pv = u32s(u64())
    return ShardProofData(main_c, perm_c, quot_c, chips, fri_commits, queries, final_poly, pow_w, names, pv,
                          *stacked), pos[0]


def _parse_queries(b: bytes, pos: list, u64, u32s, digests):
    """The query proofs: (per-query list, (q_rows, q_paths, q_sib, q_fpath)).  Query 0 is parsed field by
    field, recording each field's word offset; when every query repeats its layout (all length prefixes
    equal -- a proof of one shape) the rest are read as one (nq, words) matrix and sliced per field."""
    nq = u64()
    if nq == 0:
        return [], ([], [], [], [])
    q0 = pos[0]
    prefixes, fields = [], []  # word offsets (from q0) of the u64 length prefixes; (kind, t, off, count)

    def pre():
        prefixes.append((pos[0] - q0) // 4)
        return u64()

    def take(kind, t, n_words):
        fields.append((kind, t, (pos[0] - q0) // 4, n_words))
        pos[0] += 4 * n_words

    for t in range(pre()):
        for _ in range(pre()):
            take("row", t, pre())
        take("path", t, 8 * pre())
    for s_ in range(pre()):
        take("sib", s_, 4)
        take("fpath", s_, 8 * pre())
    qw = (pos[0] - q0) // 4
    if q0 + 4 * nq * qw > len(b):
        raise ValueError("truncated query proofs")
    M = np.frombuffer(b, np.uint32, nq * qw, q0).reshape(nq, qw)
    pcols = np.asarray(sorted(set(prefixes) | {o + 1 for o in prefixes}), np.int64)
    if not (M[:, pcols] == M[0, pcols]).all():
        # queries of different shapes (a malformed proof): field by field, check_shape rejects it
        pos[0] = q0
        queries = []
        for _ in range(nq):
            inputs = []
            for _ in range(u64()):
                rows = [u32s(u64()) for _ in range(u64())]
                inputs.append((rows, digests()))
            steps = []
            for _ in range(u64()):
                sib = u32s(4)
                steps.append((sib, digests()))
            queries.append((inputs, steps))
        return queries, (None, None, None, None)
    pos[0] = q0 + 4 * nq * qw
    M = M.astype(np.int64)
    q_rows, q_paths, q_sib, q_fpath = [], [], [], []
    for kind, t, off, n in fields:
        blk = M[:, off:off + n]
        if kind == "row":
            while len(q_rows) <= t:
                q_rows.append([])
            q_rows[t].append(blk)
        elif kind == "path":
            q_paths.append(blk.reshape(nq, n // 8, 8))
        elif kind == "sib":
            q_sib.append(blk)
        else:
            q_fpath.append(blk.reshape(nq, n // 8, 8))
    for t in range(len(q_paths)):
        while len(q_rows) <= t:
            q_rows.append([])
    queries = [([([r[q] for r in q_rows[t]], q_paths[t][q]) for t in range(len(q_paths))],
                [(q_sib[s_][q], q_fpath[s_][q]) for s_ in range(len(q_sib))]) for q in range(nq)]
    return queries, (q_rows, q_paths, q_sib, q_fpath)


# ---------------------------------------------------------------- the child's verifying key
@dataclass(frozen=True)
class LookupVk:
    """A local lookup as the constraint folder sees it (permutation.rs:205-347): the kind, the value
    VirtualPairCols and the multiplicity, each (terms ((is_main, col, weight), ...), constant)."""
    kind: int
    values: tuple
    mult: tuple
    is_send: bool


def _vpc(v) -> tuple:
    return (tuple((k == "main", int(c), int(w) % P) for k, c, w in v.terms), int(v.constant) % P)


@dataclass(frozen=True)
class ChipShape:
    """What the verifier needs of a chip (a picklable summary of a ChipDesc): its shape, and for the
    out-of-domain check its constraint program (the blob's postfix code, machine.py) and local lookups."""
    name: str
    prep_width: int
    main_width: int
    perm_width_ef: int
    log_quotient_degree: int
    local_only: bool
    code: tuple = ()
    lookups: tuple = ()
    num_constraints: int = 0
    commit_scope: int = 0

    @staticmethod
    def of(c) -> "ChipShape":
        from .machine import LOOKUP_LOCAL
        lks = tuple(LookupVk(int(l.kind), tuple(_vpc(v) for v in l.values), _vpc(l.multiplicity), i < len(c.sends))
                    for i, l in enumerate(c.sends + c.receives) if l.scope == LOOKUP_LOCAL)
        return ChipShape(c.name, c.prep_width, c.main_width, c.perm_width_ef, c.log_quotient_degree,
                         bool(c.local_only), tuple(int(x) for x in c.program()), lks, c.num_constraints,
                         int(c.commit_scope))


@dataclass
class ChildVk:
    """What a compress program knows of its child's machine: chip shapes (from the machine blob), the
    preprocessed commitment and heights, pc_start, the initial global cumulative sum, FRI parameters."""
    chips: Dict[str, ChipShape]
    num_pv: int
    commit: np.ndarray                # vk.commit, 8 canonical words
    prep_order: List[str]             # preprocessed chips sorted by (height desc, name) (machine.rs:383-384)
    prep_heights: Dict[str, int]
    pc_start: int = 0x00400000
    gcs: np.ndarray = None
    log_blowup: int = 1
    num_queries: int = 84
    pow_bits: int = 16

    @staticmethod
    def of(machine, prep_traces: Dict[str, np.ndarray], commit, log_blowup=1, num_queries=84, pow_bits=16,
           pc_start=None, gcs=None):
        from . import septic as S
        prep = {k: v for k, v in prep_traces.items() if v is not None}
        order = sorted(prep, key=lambda k: (-prep[k].shape[0], k))
        shapes = {c.name: ChipShape.of(c) for c in machine.chips}
        return ChildVk(shapes, machine.num_pv, np.asarray(commit, np.int64), order,
                       {k: prep[k].shape[0] for k in prep},
                       getattr(machine, "pc_start", 0x00400000) if pc_start is None else pc_start,
                       np.asarray(S.CURVE_CUMULATIVE_SUM_START if gcs is None else gcs, np.int64), log_blowup,
                       num_queries, pow_bits)


# ---------------------------------------------------------------- host transcript replay
class HostChallenger:
    """DuplexChallenger<F, Poseidon2, 16, 8> (challenger.rs:60-233) on canonical ints."""

    def __init__(self):
        self.st = [0] * 16
        self.inp: List[int] = []
        self.out: List[int] = []

    def duplex(self):
        for i, v in enumerate(self.inp):
            self.st[i] = v
        self.inp = []
        self.st = [int(x) for x in R.poseidon2_permute_host(np.asarray([self.st], U))[0]]
        self.out = self.st[:8]

    def observe(self, v):
        self.out = []
        self.inp.append(int(v) % P)
        if len(self.inp) == 8:
            self.duplex()

    def sample(self):
        if self.inp or not self.out:
            self.duplex()
        return self.out.pop()

    def sample_ef(self):
        return [self.sample() for _ in range(4)]


@dataclass
class Replay:
    zeta: list
    fri_alpha: list
    betas: list
    pow_sample: int
    index_samples: List[int]
    log_max: int


def replay(vk: ChildVk, p: ShardProofData) -> Replay:
    """The verifier's transcript (machine.rs:77-85 observe_into, then verifier.rs / the PCS)."""
    ch = HostChallenger()
    for v in list(vk.commit) + [vk.pc_start] + list(vk.gcs) + [0]:
        ch.observe(v)
    for v in p.pv[:vk.num_pv]:
        ch.observe(v)
    for v in p.main_c:
        ch.observe(v)
    ch.sample_ef(), ch.sample_ef()
    for v in p.perm_c:
        ch.observe(v)
    for c in p.chips:
        for v in list(c.lcs) + list(c.gcs):
            ch.observe(v)
    ch.sample_ef()
    for v in p.quot_c:
        ch.observe(v)
    zeta = ch.sample_ef()
    fa = ch.sample_ef()
    betas = []
    for r in p.fri_commits:
        for v in r:
            ch.observe(v)
        betas.append(ch.sample_ef())
    for v in p.final_poly:
        ch.observe(v)
    ch.observe(p.pow_witness)
    pw = ch.sample()
    idx = [ch.sample() for _ in range(vk.num_queries)]
    return Replay(zeta, fa, betas, pw, idx, len(p.fri_commits) + vk.log_blowup)


# ---------------------------------------------------------------- the program builder
def _blk(vals) -> np.ndarray:
    """Base values as memory blocks [v, 0, 0, 0]."""
    v = np.asarray(vals, U).reshape(-1) % PU
    out = np.zeros((len(v), D), U)
    out[:, 0] = v
    return out


class Builder:
    """A RecursionProgram with constants, hinted values and the arithmetic the verifier needs, address
    arrays vectorised over the queries."""

    def __init__(self, prog: R.RecursionProgram):
        self.p = prog
        self._tape = isinstance(prog, _HintTape)  # addresses only: no operand arrays to build
        self._consts: Dict[tuple, int] = {}
        self.labels: Dict[int, str] = {}  # block index of each check -> what it checks (diagnostics)

    def const(self, v) -> int:
        """Address of a constant block (MemoryConst); v an int or 4 ints."""
        key = tuple(int(x) % P for x in (v if isinstance(v, (list, tuple, np.ndarray)) else [v, 0, 0, 0]))
        if key not in self._consts:
            a = self.p.alloc(1)
            self.p.mem_write(a, np.asarray([key], U))
            self._consts[key] = int(a[0])
        return self._consts[key]

    def const_fresh(self, vals) -> np.ndarray:
        """Addresses of a new constant block per call holding `vals` (base values), never shared with an
        equal constant: node_flat's templates take its values like hints (the child vk's commitment)."""
        blk = _blk(vals)
        a = self.p.alloc(len(blk))
        if isinstance(self.p, _HintTape):
            self.p.fresh.append(blk)
        else:
            self.p.__dict__.setdefault("fresh_blocks", []).append(len(self.p.blocks))
        self.p.mem_write(a, blk)
        return a

    def hint_base(self, vals) -> np.ndarray:
        v = np.asarray(vals, np.int64)
        a = self.p.alloc(v.size).reshape(v.shape)
        if v.size:
            if self._tape:  # the tape's value blocks directly (_blk, as uint32)
                blk = np.zeros((v.size, D), np.uint32)
                blk[:, 0] = np.asarray(v, U).reshape(-1) % PU
                self.p.vals.append(blk)
            else:
                self.p.hint(a.ravel(), _blk(v.ravel()))
        return a

    def hint_ext(self, vals) -> np.ndarray:
        v = np.asarray(vals, np.int64).reshape(-1, 4)
        a = self.p.alloc(len(v))
        if len(v):
            if self._tape:
                self.p.vals.append((v.astype(U) % PU).astype(np.uint32))
            else:
                self.p.hint(a, v.astype(U) % PU)
        return a

    def _out(self, x, y) -> np.ndarray:
        sx, sy = np.shape(x), np.shape(y)
        shp = sx if sx == sy or not sy else sy if not sx else np.broadcast_shapes(sx, sy)
        return self.p.alloc(math.prod(shp)).reshape(shp)

    def base(self, op, x, y) -> np.ndarray:
        if self._tape:
            return self._out(x, y)
        x, y = np.broadcast_arrays(np.asarray(x, np.int64), np.asarray(y, np.int64))
        out = self.p.alloc(x.size).reshape(x.shape)
        if x.size:
            self.p.base_alu(op, out.ravel(), x.ravel(), y.ravel())
        return out

    def ext(self, op, x, y) -> np.ndarray:
        if self._tape:
            return self._out(x, y)
        x, y = np.broadcast_arrays(np.asarray(x, np.int64), np.asarray(y, np.int64))
        out = self.p.alloc(x.size).reshape(x.shape)
        if x.size:
            self.p.ext_alu(op, out.ravel(), x.ravel(), y.ravel())
        return out

    def assert_zero_base(self, addrs, label: str = ""):
        a = np.asarray(addrs, np.int64).ravel()
        if a.size:
            self.labels[len(self.p.blocks)] = label
            self.p.mem_read(a, np.zeros((a.size, D), U), 1)

    def assert_eq_base(self, x, y, label: str = ""):
        self.assert_zero_base(self.base(R.OP_SUB, x, y), label)

    def assert_eq_ext(self, x, y, label: str = ""):
        d = self.ext(R.OP_SUB, x, y)
        self.labels[len(self.p.blocks)] = label
        self.p.mem_read(np.asarray(d, np.int64).ravel(), np.zeros((np.asarray(d).size, D), U), 1)

    def p2(self, inp: np.ndarray) -> np.ndarray:
        """Poseidon2 permutations of (n, 16) input address rows -> (n, 16) output addresses."""
        if self._tape:
            return self.p.alloc(np.size(inp)).reshape(-1, R.WIDTH)
        inp = np.asarray(inp, np.int64).reshape(-1, R.WIDTH)
        out = self.p.alloc(inp.size).reshape(inp.shape)
        self.p.poseidon2(out, inp)
        return out

    def sponge(self, cols: np.ndarray) -> np.ndarray:
        """PaddingFreeSponge<P, 16, 8, 8> (hash.rs:40-50) of (n, w) base addresses -> (n, 8)."""
        n, w = cols.shape
        zero = self.const(0)
        state = np.full((n, R.WIDTH), zero, np.int64)
        for c in range(0, w, 8):
            k = min(8, w - c)
            inp = state.copy()
            inp[:, :k] = cols[:, c:c + k]
            state = self.p2(inp)
        return state[:, :8]

    def compress(self, left: np.ndarray, right: np.ndarray) -> np.ndarray:
        return self.p2(np.concatenate([left, right], 1))[:, :8]

    def select(self, bits, x, y):
        """(bit ? y : x, bit ? x : y) per element: Select (select.rs)."""
        if self._tape:
            shp = np.broadcast_shapes(np.shape(bits), np.shape(x), np.shape(y))
            return self.p.alloc(math.prod(shp)).reshape(shp), self.p.alloc(math.prod(shp)).reshape(shp)
        bits, x, y = np.broadcast_arrays(*(np.asarray(v, np.int64) for v in (bits, x, y)))
        o1, o2 = self.p.alloc(x.size).reshape(x.shape), self.p.alloc(x.size).reshape(x.shape)
        if x.size:
            self.p.select(bits.ravel(), o1.ravel(), o2.ravel(), x.ravel(), y.ravel())
        return o1, o2

    def bits_of(self, samples: np.ndarray, values: Sequence[int]) -> np.ndarray:
        """HintBits: the 31 bits of each sampled element (lsb first), checked boolean, recomposed to the
        sample, and canonical (not the bits of x + p): returns (n, 31) bit addresses."""
        v = np.asarray(values, np.int64)
        bits = self.hint_base(((v[:, None] >> np.arange(31)[None, :]) & 1))
        if self._tape:  # (the checks below add no hints)
            return bits
        sq = self.base(R.OP_MUL, bits, bits)
        self.assert_eq_base(sq, bits, "bits boolean")
        acc = bits[:, 0]
        for i in range(1, 31):
            acc = self.base(R.OP_ADD, acc, self.base(R.OP_MUL, bits[:, i], self.const(1 << i)))
        self.assert_eq_base(acc, samples, "bits recompose the sample")
        # x >= p iff bits 24..30 are all one and the low 24 bits are not all zero
        top = bits[:, 24]
        for i in range(25, 31):
            top = self.base(R.OP_MUL, top, bits[:, i])
        low = bits[:, 0]
        for i in range(1, 24):
            low = self.base(R.OP_ADD, low, bits[:, i])
        self.assert_zero_base(self.base(R.OP_MUL, top, low), "bits canonical")
        return bits

    def ef_from_base4(self, words: np.ndarray) -> np.ndarray:
        """(n, 4) base addresses -> EF addresses sum_k w_k X^k."""
        x = self.const([0, 1, 0, 0])
        acc = words[:, 3]
        for k in (2, 1, 0):
            acc = self.ext(R.OP_ADD, self.ext(R.OP_MUL, acc, x), words[:, k])
        return acc


class ProgChallenger:
    """The DuplexChallenger inside the program: inputs overwrite the state's first lanes, permutations are
    Poseidon2 instructions, samples are permutation output addresses."""

    def __init__(self, b: Builder):
        self.b = b
        z = b.const(0)
        self.st = np.full(R.WIDTH, z, np.int64)
        self.inp: List[int] = []
        self.out: List[int] = []

    def duplex(self):
        x = self.st.copy()
        x[:len(self.inp)] = self.inp
        self.inp = []
        self.st = self.b.p2(x[None, :])[0]
        self.out = list(self.st[:8])

    def observe(self, addrs):
        for a in np.asarray(addrs, np.int64).ravel():
            self.out = []
            self.inp.append(int(a))
            if len(self.inp) == 8:
                self.duplex()

    def sample(self) -> int:
        if self.inp or not self.out:
            self.duplex()
        return self.out.pop()

    def sample_ef(self) -> int:
        w = np.asarray([[self.sample() for _ in range(4)]], np.int64)
        return int(self.b.ef_from_base4(w)[0])


class ExtDag:
    """Extension-field arithmetic recorded as a DAG and emitted level by level: every node of one depth
    is one ExtAlu block (the runtime runs a block as one vectorised step), so the thousands of
    operations of a machine's constraint programs cost as many blocks as the DAG is deep."""

    def __init__(self, b: Builder):
        self.b = b
        self.op: List[int] = []
        self.x: List[int] = []
        self.y: List[int] = []
        self.lvl: List[int] = []
        self.addr: List[int] = []
        self._leaf: Dict[int, int] = {}
        self._const: Dict[tuple, int] = {}

    def leaf(self, addr: int) -> int:
        a = int(addr)
        n = self._leaf.get(a)
        if n is None:
            n = len(self.op)
            self.op.append(-1), self.x.append(-1), self.y.append(-1), self.lvl.append(0), self.addr.append(a)
            self._leaf[a] = n
        return n

    def const(self, v) -> int:
        return self.leaf(self.b.const(v))

    def _node(self, op, x, y) -> int:
        n = len(self.op)
        self.op.append(op), self.x.append(x), self.y.append(y)
        self.lvl.append(max(self.lvl[x], self.lvl[y]) + 1)
        self.addr.append(-1)
        return n

    def add(self, x, y):
        return self._node(R.OP_ADD, x, y)

    def sub(self, x, y):
        return self._node(R.OP_SUB, x, y)

    def mul(self, x, y):
        return self._node(R.OP_MUL, x, y)

    def div(self, x, y):
        return self._node(R.OP_DIV, x, y)

    def sum(self, xs: List[int]) -> int:
        xs = list(xs)
        if not xs:
            return self.const([0, 0, 0, 0])
        while len(xs) > 1:  # balanced: depth log2(n)
            nxt = [self.add(xs[i], xs[i + 1]) for i in range(0, len(xs) - 1, 2)]
            if len(xs) & 1:
                nxt.append(xs[-1])
            xs = nxt
        return xs[0]

    def prod(self, xs: List[int]) -> int:
        xs = list(xs)
        if not xs:
            return self.const([1, 0, 0, 0])
        while len(xs) > 1:
            nxt = [self.mul(xs[i], xs[i + 1]) for i in range(0, len(xs) - 1, 2)]
            if len(xs) & 1:
                nxt.append(xs[-1])
            xs = nxt
        return xs[0]

    def powers(self, base: int, n: int) -> List[int]:
        """base^0 .. base^(n-1) at depth ~ 64 + n / 64 (two chains and one product level)."""
        one = self.const([1, 0, 0, 0])
        lo = [one]
        for _ in range(1, min(n, 64)):
            lo.append(self.mul(lo[-1], base))
        if n <= 64:
            return lo[:n]
        b64 = self.mul(lo[63], base)
        hi = [one, b64]
        while len(hi) * 64 < n:
            hi.append(self.mul(hi[-1], b64))
        return [lo[k] if k < 64 else self.mul(hi[k >> 6], lo[k & 63]) for k in range(n)]

    def emit(self):
        """Allocate and append every not-yet-emitted node, one ExtAlu block per depth."""
        pend = [i for i, a in enumerate(self.addr) if a < 0]
        if not pend:
            return
        by = {}
        for i in pend:
            by.setdefault(self.lvl[i], []).append(i)
        for lv in sorted(by):
            ids = by[lv]
            out = self.b.p.alloc(len(ids))
            for i, a in zip(ids, out):
                self.addr[i] = int(a)
            self.b.p.ext_alu(np.asarray([self.op[i] for i in ids], np.int64), out,
                             np.asarray([self.addr[self.x[i]] for i in ids], np.int64),
                             np.asarray([self.addr[self.y[i]] for i in ids], np.int64))

    def address(self, n: int) -> int:
        assert self.addr[n] >= 0, "node not emitted"
        return self.addr[n]


def _chip_constraints(dag: ExtDag, c: ChipShape, prep_l, prep_n, main_l, main_n, perm_l, perm_n, is_first,
                      is_last, is_trans, pv, alpha_perm, beta_pows, lcs, gcs) -> List[int]:
    """The chip's constraint values at zeta in folding order (air_eval of the oracle; crates/stark/src/
    folder.rs:79-102 for the AIR, permutation.rs:205-347 for LogUp, the Global-scope digest rows last)."""
    out: List[int] = []
    st: List[int] = []
    slots: Dict[int, int] = {}
    code = c.code
    pc = 0
    from . import machine as M
    while pc < len(code):
        op = code[pc]
        pc += 1
        if op == M.OP_MAIN_L:
            st.append(main_l[code[pc]]); pc += 1
        elif op == M.OP_MAIN_N:
            st.append(main_n[code[pc]]); pc += 1
        elif op == M.OP_PREP_L:
            st.append(prep_l[code[pc]]); pc += 1
        elif op == M.OP_PREP_N:
            st.append(prep_n[code[pc]]); pc += 1
        elif op == M.OP_CONST:
            st.append(dag.const(code[pc] % P)); pc += 1
        elif op == M.OP_PV:
            st.append(pv[code[pc]]); pc += 1
        elif op == M.OP_IS_FIRST:
            st.append(is_first)
        elif op == M.OP_IS_LAST:
            st.append(is_last)
        elif op == M.OP_IS_TRANS:
            st.append(is_trans)
        elif op in (M.OP_ADD, M.OP_SUB, M.OP_MUL):
            y = st.pop()
            x = st.pop()
            st.append(dag.add(x, y) if op == M.OP_ADD else dag.sub(x, y) if op == M.OP_SUB else dag.mul(x, y))
        elif op == M.OP_NEG:
            st.append(dag.sub(dag.const(0), st.pop()))
        elif op == M.OP_EMIT:
            out.append(st.pop())
        elif op == M.OP_LET:
            slots[code[pc]] = st.pop(); pc += 1
        elif op == M.OP_GET:
            st.append(slots[code[pc]]); pc += 1
        else:
            raise ValueError(f"bad opcode {op} in the constraint program of {c.name}")
    if c.lookups:
        def vpc(v):
            terms, k = v
            acc = [dag.const(k)] if k else []
            for is_main, col, w in terms:
                x = main_l[col] if is_main else prep_l[col]
                acc.append(x if w == 1 else dag.mul(x, dag.const(w)))
            return dag.sum(acc) if acc else dag.const(0)
        batch = 1 << c.log_quotient_degree
        nb = c.perm_width_ef - 1
        for bi in range(nb):
            rlcs, ms = [], []
            for lk in c.lookups[bi * batch:(bi + 1) * batch]:
                terms = [dag.add(alpha_perm, dag.const(lk.kind))]
                for v, val in enumerate(lk.values):
                    terms.append(dag.mul(beta_pows[v], vpc(val)))
                rlcs.append(dag.sum(terms))
                m = vpc(lk.mult)
                ms.append(m if lk.is_send else dag.sub(dag.const(0), m))
            prod = dag.prod(rlcs)
            num = dag.sum([dag.mul(dag.prod([r for j, r in enumerate(rlcs) if j != i]), ms[i]) for i in range(len(rlcs))])
            out.append(dag.sub(dag.mul(prod, perm_l[bi]), num))
        sum_l, sum_n = dag.sum(perm_l[:nb]), dag.sum(perm_n[:nb])
        phi_l, phi_n = perm_l[nb], perm_n[nb]
        out.append(dag.mul(dag.sub(phi_l, sum_l), is_first))
        out.append(dag.mul(dag.sub(dag.sub(phi_n, phi_l), sum_n), is_trans))
        out.append(dag.mul(dag.sub(phi_l, lcs), is_last))
    if c.commit_scope == 1:
        w = c.main_width
        for i in range(7):
            out.append(dag.mul(dag.sub(main_l[w - 14 + i], gcs[i]), is_last))
            out.append(dag.mul(dag.sub(main_l[w - 7 + i], gcs[7 + i]), is_last))
    if len(out) != c.num_constraints:
        raise ValueError(f"{c.name}: {len(out)} constraint values, the vk says {c.num_constraints}")
    return out


def _zp_base(log_n: int, shift: int, x: int) -> int:
    """Z of the coset shift * H_(2^log_n) at a base-field point: (x / shift)^(2^log_n) - 1."""
    return (pow(x * pow(shift, P - 2, P) % P, 1 << log_n, P) - 1) % P


def verify_constraints(b: Builder, vk: ChildVk, p: ShardProofData, chips: List[ChipShape], opened, zeta: int,
                       alpha: int, perm_ch, pv, lcs_words, gcs_words):
    """The out-of-domain check (crates/stark/src/verifier.rs:316-397; recursion/circuit/src/stark.rs:
    246-432 / constraints.rs:39-196 in the reference's recursion program): for every chip, its folded
    constraints at zeta times 1/Z_H(zeta) equal the quotient recombined from the opened chunks, and the
    chips' local cumulative sums add to zero.  `opened[name]` holds the hinted EF addresses of the
    chip's opened values: prep/main/perm at zeta and at g*zeta, and the quotient chunks."""
    dag = ExtDag(b)
    zl = dag.leaf(zeta)
    al = dag.leaf(alpha)
    ap, bp = dag.leaf(perm_ch[0]), dag.leaf(perm_ch[1])
    max_ln = max(o.log_degree for o in p.chips)
    zsq = [zl]  # zeta^(2^k)
    for _ in range(max_ln):
        zsq.append(dag.mul(zsq[-1], zsq[-1]))
    one = dag.const([1, 0, 0, 0])
    mono = [dag.const([1 if e == k else 0 for e in range(4)]) for k in range(4)]
    max_nc = max((c.num_constraints for c in chips), default=1)
    apows = dag.powers(al, max(1, max_nc))
    max_vals = max((len(lk.values) for c in chips for lk in c.lookups), default=0)
    bpows = dag.powers(bp, max_vals + 1)[1:] if max_vals else []
    pv_n = [dag.leaf(a) for a in pv]
    checks = []
    lcs_all = []
    for i, (c, o) in enumerate(zip(chips, p.chips)):
        ln = o.log_degree
        op = opened[c.name]
        prep_l = [dag.leaf(a) for a in op["prep_l"]]
        prep_n = [dag.leaf(a) for a in op["prep_n"]]
        main_l = [dag.leaf(a) for a in op["main_l"]]
        main_n = [dag.leaf(a) for a in op["main_n"]]
        pl_w = [dag.leaf(a) for a in op["perm_l"]]
        pn_w = [dag.leaf(a) for a in op["perm_n"]]
        perm_l = [dag.sum([dag.mul(mono[e], pl_w[4 * k + e]) for e in range(4)]) for k in range(c.perm_width_ef)]
        perm_n = [dag.sum([dag.mul(mono[e], pn_w[4 * k + e]) for e in range(4)]) for k in range(c.perm_width_ef)]
        lw = [dag.leaf(a) for a in lcs_words[i]]
        lcs = dag.sum([dag.mul(mono[e], lw[e]) for e in range(4)])
        lcs_all.append(lcs)
        gcs = [dag.leaf(a) for a in gcs_words[i]]
        ginv = pow(two_adic_gen(ln), P - 2, P)
        zh = dag.sub(zsq[ln], one)
        is_first = dag.div(zh, dag.sub(zl, one))
        is_last = dag.div(zh, dag.sub(zl, dag.const(ginv)))
        is_trans = dag.sub(zl, dag.const(ginv))
        vals = _chip_constraints(dag, c, prep_l, prep_n, main_l, main_n, perm_l, perm_n, is_first, is_last, is_trans,
                                 pv_n, ap, bpows, lcs, gcs)
        nc = len(vals)
        folded = dag.sum([dag.mul(apows[nc - 1 - k], v) for k, v in enumerate(vals)])
        # recompute_quotient (verifier.rs:400-436): chunk a's domain is the coset g_a H_n, g_a = 3 w_Q^a
        nq = 1 << c.log_quotient_degree
        wq = two_adic_gen(ln + c.log_quotient_degree)
        shifts = [GENERATOR * pow(wq, a, P) % P for a in range(nq)]
        chunks = []
        for a in range(nq):
            fac = []
            for bb in range(nq):
                if bb == a:
                    continue
                # zp_b(zeta) = zeta^n * shift_b^-n - 1, divided by zp_b(shift_a) (a base constant)
                sbn = pow(pow(shifts[bb], P - 2, P), 1 << ln, P)
                num = dag.sub(dag.mul(zsq[ln], dag.const(sbn)), one)
                fac.append(dag.mul(num, dag.const(pow(_zp_base(ln, shifts[bb], shifts[a]), P - 2, P))))
            qw = [dag.leaf(x) for x in op["quot"][a]]
            chunk = dag.sum([dag.mul(mono[e], qw[e]) for e in range(4)])
            chunks.append(dag.mul(dag.prod(fac), chunk) if fac else chunk)
        quotient = dag.sum(chunks)
        checks.append((c.name, dag.div(folded, zh), quotient))
    total_lcs = dag.sum(lcs_all)
    dag.emit()
    for name, lhs, rhs in checks:
        b.assert_eq_ext([dag.address(lhs)], [dag.address(rhs)], f"ood evaluation {name}")
    b.assert_eq_ext([dag.address(total_lcs)], [int(b.const([0, 0, 0, 0]))], "local cumulative sum")


def _verify_batch(b: Builder, root, mats: List[dict], ridx: np.ndarray, ridx_bits: np.ndarray, paths: np.ndarray):
    """MerkleTreeMmcs::verify_batch (fri.rs:363-400) for every query: mats = [{height, rows (q, w) addrs}] in
    commit order; ridx_bits (q, L) the row index bits; paths (q, L, 8) sibling addresses; root 8 addresses."""
    order = sorted(range(len(mats)), key=lambda k: -mats[k]["height"])
    cur = mats[order[0]]["height"]
    pos = 0
    cols = []
    while pos < len(order) and mats[order[pos]]["height"] == cur:
        cols.append(mats[order[pos]]["rows"])
        pos += 1
    node = b.sponge(np.concatenate(cols, 1))
    for lvl in range(paths.shape[1]):
        bit = ridx_bits[:, lvl]
        left, right = b.select(np.repeat(bit[:, None], 8, 1), node, paths[:, lvl])
        node = b.compress(left, right)
        cur >>= 1
        cols = []
        while pos < len(order) and mats[order[pos]]["height"] == cur:
            cols.append(mats[order[pos]]["rows"])
            pos += 1
        if cols:
            node = b.compress(node, b.sponge(np.concatenate(cols, 1)))
    assert pos == len(order)
    b.assert_eq_base(node, np.broadcast_to(np.asarray(root, np.int64), node.shape), "merkle root")


def check_shape(vk: ChildVk, p: ShardProofData):
    """verify_opening_shape and the proof-shape checks the reference's verifier makes before the transcript
    (verifier.rs:248-312, fri.rs): the chip set and widths against the vk, preprocessed heights, query and
    FRI round counts, Merkle path lengths.  Raises ValueError (the program's structure is derived from the
    proof, so a malformed proof must be rejected here, not turned into a different program)."""
    if len(p.chips) != len(p.names) or len(set(p.names)) != len(p.names):
        raise ValueError("chip ordering does not match the opened values")
    for name, o in zip(p.names, p.chips):
        c = vk.chips.get(name)
        if c is None:
            raise ValueError(f"chip {name} is not in the verifying key")
        if (o.prep_l.shape[0] != c.prep_width or o.main_l.shape[0] != c.main_width
                or o.perm_l.shape[0] != 4 * c.perm_width_ef or o.quot.shape[0] != 1 << c.log_quotient_degree
                or not 0 <= o.log_degree <= 24):
            raise ValueError(f"{name}: opening shape")
        if name in vk.prep_heights and (1 << o.log_degree) != vk.prep_heights[name]:
            raise ValueError(f"{name}: height differs from its preprocessed trace")
        if (not c.local_only and (o.main_n.shape[0] != c.main_width or o.prep_n.shape[0] != c.prep_width)):
            raise ValueError(f"{name}: next-row opening shape")
    for name in vk.prep_order:
        if name not in p.names:
            raise ValueError(f"preprocessed chip {name} missing from the shard")
    if len(p.queries) != vk.num_queries:
        raise ValueError("query count")
    log_max = len(p.fri_commits) + vk.log_blowup
    if log_max > 25 or max(o.log_degree for o in p.chips) + vk.log_blowup != log_max:
        raise ValueError("FRI round count does not match the tallest trace")
    for inputs, steps in p.queries:
        if len(inputs) != 4 or len(steps) != len(p.fri_commits):
            raise ValueError("query proof shape")
        for off, (_, path) in enumerate(steps):
            if path.shape[0] != log_max - 1 - off:
                raise ValueError("FRI commit-phase path length")
        for rows, path in inputs:
            if path.shape[0] > log_max:
                raise ValueError("input opening path length")


def verify_shard(prog: R.RecursionProgram, vk: ChildVk, proof: bytes, b: Optional[Builder] = None,
                 ood: bool = True):
    """Append the verification of one child ShardProof (module docstring).  Returns what the node's
    public-value checks read of the child (zkmips_amd/node_pv.ChildVars: its hinted public values, the vk
    commitment's addresses, chip names and heights, the Global-scope chips' cumulative sums)."""
    from .node_pv import V, ChildVars
    b = b or Builder(prog)
    p = parse_shard_proof(proof)
    check_shape(vk, p)
    if isinstance(prog, _HintTape):  # the chip order and heights: part of a template's key (node_flat)
        prog.shapes.append((tuple(p.names), tuple(int(o.log_degree) for o in p.chips)))
    rp = replay(vk, p)
    lb, nq = vk.log_blowup, vk.num_queries
    chips = [vk.chips[n] for n in p.names]
    ch = ProgChallenger(b)
    # observe_into: vk commit, pc_start, initial global sum, 0 -- constants of the program (the commit's own
    # constant block, not shared with equal values: the program's structure does not depend on it)
    vkc = [int(a) for a in b.const_fresh(vk.commit)]
    ch.observe(vkc + [b.const(int(v)) for v in [vk.pc_start] + list(vk.gcs) + [0]])
    pv = b.hint_base(p.pv)
    ch.observe(pv[:vk.num_pv])
    cvars = ChildVars(V(np.asarray(pv, np.int64), np.asarray(p.pv, np.int64) % P), np.asarray(vkc, np.int64),
                      list(p.names), [int(o.log_degree) for o in p.chips])
    main_c, perm_c, quot_c = b.hint_base(p.main_c), b.hint_base(p.perm_c), b.hint_base(p.quot_c)
    ch.observe(main_c)
    perm_ch = (ch.sample_ef(), ch.sample_ef())
    ch.observe(perm_c)
    lcs_words, gcs_words = [], []
    start = [int(b.const(int(v))) for v in S_CURVE_START]
    for c, cs in zip(p.chips, chips):
        sums = b.hint_base(np.concatenate([c.lcs, c.gcs]))
        ch.observe(sums)
        lcs_words.append(sums[:4])
        gcs_words.append(sums[4:])
        if cs.commit_scope != 0:  # a Global-scope chip's cumulative sum joins the node's sum (core.rs:543-547)
            cvars.global_sums.append(V(np.asarray(sums[4:], np.int64), np.asarray(c.gcs, np.int64) % P))
        if cs.commit_scope == 0:  # verifier.rs: a Local-scope chip's global sum is the zero digest
            b.assert_eq_base(sums[4:], np.asarray(start, np.int64), f"{cs.name} global sum")
        if not cs.lookups:  # no local lookups: no local sum
            b.assert_zero_base(sums[:4], f"{cs.name} local sum")
    alpha = ch.sample_ef()
    ch.observe(quot_c)
    zeta = ch.sample_ef()
    fa = ch.sample_ef()
    fri_c = b.hint_base(p.fri_commits)
    betas = []
    for r in range(len(p.fri_commits)):
        ch.observe(fri_c[r])
        betas.append(ch.sample_ef())
    final = b.hint_ext(p.final_poly)[0]
    fp_words = b.hint_base(p.final_poly)
    b.assert_eq_ext(b.ef_from_base4(fp_words[None, :]), final, "final poly words")
    ch.observe(fp_words)
    pow_w = b.hint_base([p.pow_witness])
    ch.observe(pow_w)
    pow_s = ch.sample()
    if vk.pow_bits:
        pbits = b.bits_of(np.asarray([pow_s]), [rp.pow_sample])
        b.assert_zero_base(pbits[0, :vk.pow_bits], "proof of work")
    samples = np.asarray([ch.sample() for _ in range(nq)], np.int64)
    ibits = b.bits_of(samples, rp.index_samples)  # (nq, 31)
    log_max = rp.log_max
    index = np.asarray(rp.index_samples, np.int64) & ((1 << log_max) - 1)

    # ---- the four input rounds (verifier.rs:124-205): matrices, heights, opening points, values ----
    g_zeta = {}

    def zeta_next(log_n):
        if log_n not in g_zeta:
            g_zeta[log_n] = int(b.ext(R.OP_MUL, zeta, b.const(two_adic_gen(log_n))))
        return g_zeta[log_n]
    rounds = []
    mats = []
    for name in vk.prep_order:  # round 0: the vk's preprocessed traces
        i = p.names.index(name)
        c, o = vk.chips[name], p.chips[i]
        pts = [(zeta, o.prep_l)] + ([] if c.local_only else [(zeta_next(o.log_degree), o.prep_n)])
        mats.append({"log_n": int(np.log2(vk.prep_heights[name])), "width": c.prep_width, "pts": pts})
    rounds.append((vkc, mats))
    mats = []
    for c, o in zip(chips, p.chips):  # round 1: main
        pts = [(zeta, o.main_l)] + ([] if c.local_only else [(zeta_next(o.log_degree), o.main_n)])
        mats.append({"log_n": o.log_degree, "width": c.main_width, "pts": pts})
    rounds.append((main_c, mats))
    mats = [{"log_n": o.log_degree, "width": 4 * c.perm_width_ef,
             "pts": [(zeta, o.perm_l), (zeta_next(o.log_degree), o.perm_n)]} for c, o in zip(chips, p.chips)]
    rounds.append((perm_c, mats))
    mats = []
    for c, o in zip(chips, p.chips):  # round 3: quotient chunks
        for j in range(1 << c.log_quotient_degree):
            mats.append({"log_n": o.log_degree, "width": 4, "pts": [(zeta, o.quot[j])]})
    rounds.append((quot_c, mats))
    # host mirror of the rounds (z values as ints) for the FRI leaf words
    zeta_h = rp.zeta
    zn_h: Dict[int, list] = {}  # per height: zeta times the subgroup generator
    rounds_host = []
    for _, ms in rounds:
        hm = []
        for m in ms:
            pts = []
            for z, vals in m["pts"]:
                if z != zeta and m["log_n"] not in zn_h:
                    zn_h[m["log_n"]] = ef_mul(zeta_h, ef_base(two_adic_gen(m["log_n"])))
                zh = zeta_h if z == zeta else zn_h[m["log_n"]]
                pts.append((zh, np.asarray(vals, np.int64).reshape(-1, 4)))
            hm.append((m["log_n"], m["width"], pts))
        rounds_host.append(hm)
    fri_pairs = host_fri_pairs(vk, p, rp, rounds_host)
    # hinted opened values at the points (shared by the queries and the out-of-domain check)
    for _, ms in rounds:
        for m in ms:
            m["pts"] = [(z, b.hint_ext(np.asarray(vals, np.int64).reshape(-1, 4))) for z, vals in m["pts"]]
    tape = isinstance(prog, _HintTape)
    if tape:  # the rest adds hints only for the query rows, Merkle paths and the FRI steps: those alone
        for t, (_, ms) in enumerate(rounds):
            for k, m in enumerate(ms):
                if m["width"]:
                    b.hint_base(_q_rows(p, t, k))
            b.hint_base(p.q_paths[t] if p.q_paths is not None else np.stack([qq[0][t][1] for qq in p.queries]))
        for off in range(len(p.fri_commits)):
            b.hint_ext(p.q_sib[off] if p.q_sib is not None else np.stack([qq[1][off][0] for qq in p.queries]))
            b.hint_base(fri_pairs[off].astype(np.int64))
            b.hint_base(p.q_fpath[off] if p.q_fpath is not None else np.stack([qq[1][off][1] for qq in p.queries]))
        return cvars
    if ood:  # (no hints in the constraint check)
        none = np.zeros(0, np.int64)
        opened = {c.name: {"prep_l": none, "prep_n": none, "quot": []} for c in chips}
        for name, m in zip(vk.prep_order, rounds[0][1]):
            opened[name]["prep_l"] = m["pts"][0][1]
            opened[name]["prep_n"] = m["pts"][1][1] if len(m["pts"]) > 1 else none
        for c, mm, pm in zip(chips, rounds[1][1], rounds[2][1]):
            d = opened[c.name]
            d["main_l"], d["main_n"] = mm["pts"][0][1], (mm["pts"][1][1] if len(mm["pts"]) > 1 else none)
            d["perm_l"], d["perm_n"] = pm["pts"][0][1], pm["pts"][1][1]
        qi = 0
        for c in chips:
            for _ in range(1 << c.log_quotient_degree):
                opened[c.name]["quot"].append(rounds[3][1][qi]["pts"][0][1])
                qi += 1
        verify_constraints(b, vk, p, chips, opened, zeta, alpha, perm_ch, pv, lcs_words, gcs_words)
    # alpha powers per height (counter per log height, fri.rs:155-203)
    counts: Dict[int, int] = {}
    for _, ms in rounds:
        for m in ms:
            lh = m["log_n"] + lb
            counts[lh] = counts.get(lh, 0) + m["width"] * len(m["pts"])
    apow = [b.const([1, 0, 0, 0])]
    for _ in range(max(counts.values())):
        apow.append(int(b.ext(R.OP_MUL, apow[-1], fa)))
    # ---- queries, vectorised ----
    ro = {}
    lhp: Dict[int, int] = {}  # alpha-power counter per log height, across the rounds
    zero_ef = b.const([0, 0, 0, 0])
    for t, (root, ms) in enumerate(rounds):
        lbm = max(m["log_n"] for m in ms) + lb
        rows = []
        for k, m in enumerate(ms):
            vals = _q_rows(p, t, k)  # (nq, width)
            rows.append({"height": 1 << (m["log_n"] + lb), "rows": b.hint_base(vals) if m["width"] else
                         np.zeros((nq, 0), np.int64)})
        paths = b.hint_base(p.q_paths[t] if p.q_paths is not None else
                            np.stack([qq[0][t][1] for qq in p.queries]))  # (nq, L, 8)
        shift = log_max - lbm
        _verify_batch(b, root, rows, index >> shift, ibits[:, shift:shift + lbm], paths)
        for k, m in enumerate(ms):
            lh = m["log_n"] + lb
            s = log_max - lh
            # x = 3 w_lh^rev(row): ExpReverseBitsLen over the row's bits (lsb first)
            xr = prog.alloc(nq)
            prog.exp_reverse_bits(np.full(nq, b.const(two_adic_gen(lh)), np.int64), ibits[:, s:s + lh], xr)
            x = b.base(R.OP_MUL, xr, b.const(GENERATOR))
            for z, pz in m["pts"]:
                w = m["width"]
                al = np.asarray(apow[lhp.get(lh, 0):lhp.get(lh, 0) + w], np.int64)
                lhp[lh] = lhp.get(lh, 0) + w
                if w:
                    acc = prog.alloc(nq)
                    prog.batch_fri(acc, np.broadcast_to(al, (nq, w)), np.broadcast_to(pz, (nq, w)), rows[k]["rows"])
                else:
                    acc = np.full(nq, zero_ef, np.int64)
                zx = b.ext(R.OP_SUB, np.full(nq, z, np.int64), x)
                term = b.ext(R.OP_DIV, acc, zx)
                ro[lh] = term if lh not in ro else b.ext(R.OP_ADD, ro[lh], term)
    if lb in ro:
        b.assert_eq_ext(ro[lb], np.full(nq, zero_ef, np.int64), "ro[log_blowup] = 0")
    # ---- FRI commit phase (fri.rs:247-361) ----
    folded = ro[log_max]
    xr = prog.alloc(nq)
    prog.exp_reverse_bits(np.full(nq, b.const(two_adic_gen(log_max)), np.int64), ibits[:, :log_max], xr)
    x = xr
    zero = b.const(0)
    for off in range(len(p.fri_commits)):
        lfh = log_max - 1 - off
        bit = ibits[:, off]
        sib = b.hint_ext(p.q_sib[off] if p.q_sib is not None else np.stack([qq[1][off][0] for qq in p.queries]))
        d = b.ext(R.OP_SUB, sib, folded)
        e0 = b.ext(R.OP_ADD, folded, b.ext(R.OP_MUL, bit, d))      # bit ? sib : folded
        e1 = b.ext(R.OP_SUB, b.ext(R.OP_ADD, folded, sib), e0)
        # the leaf (e0 || e1) as 8 base words: hinted, recomposed to e0 and e1
        words = b.hint_base(fri_pairs[off].astype(np.int64))
        b.assert_eq_ext(b.ef_from_base4(words[:, :4]), e0, f"fri leaf e0 round {off}")
        b.assert_eq_ext(b.ef_from_base4(words[:, 4:]), e1, f"fri leaf e1 round {off}")
        fpaths = b.hint_base(p.q_fpath[off] if p.q_fpath is not None else
                             np.stack([qq[1][off][1] for qq in p.queries]))
        _verify_batch(b, fri_c[off], [{"height": 1 << lfh, "rows": words}], index >> (off + 1),
                      ibits[:, off + 1:off + 1 + lfh], fpaths)
        xn = b.base(R.OP_SUB, zero, x)
        x0, x1 = b.select(bit, x, xn)
        inv = b.base(R.OP_DIV, b.const(1), b.base(R.OP_SUB, x1, x0))
        t = b.ext(R.OP_MUL, b.ext(R.OP_SUB, np.full(nq, betas[off], np.int64), x0),
                  b.ext(R.OP_MUL, b.ext(R.OP_SUB, e1, e0), inv))
        folded = b.ext(R.OP_ADD, e0, t)
        if lfh in ro:
            bsq = b.ext(R.OP_MUL, betas[off], betas[off])
            folded = b.ext(R.OP_ADD, folded, b.ext(R.OP_MUL, np.full(nq, bsq, np.int64), ro[lfh]))
        x = b.base(R.OP_MUL, x, x)
    b.assert_eq_ext(folded, np.full(nq, final, np.int64), "final fold = final poly")
    return cvars


def _bitrev_arr(v: np.ndarray, bits: int) -> np.ndarray:
    r = np.zeros_like(v)
    for i in range(bits):
        r |= ((v >> i) & 1) << (bits - 1 - i)
    return r


def _base_dot_ef(rows: np.ndarray, ef: np.ndarray) -> np.ndarray:
    """sum_c rows[q, c] * ef[c] mod p for every q: (nq, w) canonical base values x (w, 4) EF -> (nq, 4).
    The EF words are split into 16-bit halves so that a uint64 matmul cannot overflow (w < 2^15)."""
    rows = np.asarray(rows, U)
    lo, hi = ef & U(0xFFFF), ef >> U(16)
    a = (rows @ lo) % PU
    b = (rows @ hi) % PU
    return (a + _m_u(b, U(1 << 16))) % PU


def _m_u(a, b):
    return (a * b) % PU


def _q_rows(p: ShardProofData, t: int, k: int) -> np.ndarray:
    """The queries' opened rows of matrix k of input round t, (nq, width) int64."""
    if p.q_rows is not None:
        return p.q_rows[t][k]
    return np.stack([np.asarray(qq[0][t][0][k], np.int64) for qq in p.queries])


def host_fri_pairs(vk: ChildVk, p: ShardProofData, rp: Replay, rounds_host) -> List[np.ndarray]:
    """The verifier's reduced openings and folds on the host (fri.rs:155-203, :247-361), per commit-phase
    round the queries' (e0 || e1) leaf pairs as an (nq, 8) word array: the pair the program hashes (as hinted base words)
    and recomposes against its own in-program fold.  Vectorised over the queries: per matrix and point
    the reduced opening is A - B[q] with A = sum_c alpha^c p_c(z) (query-independent) and
    B[q] = sum_c alpha^c p_c(x_q) (a base x EF dot product), divided by (z - x_q)."""
    lb, log_max = vk.log_blowup, rp.log_max
    nq = len(p.queries)
    fa = np.asarray(rp.fri_alpha, U)
    idx = np.asarray(rp.index_samples, np.int64) & ((1 << log_max) - 1)
    total = {}
    for ms in rounds_host:
        for log_n, width, pts in ms:
            total[log_n + lb] = total.get(log_n + lb, 0) + width * len(pts)
    npow = max(total.values()) if total else 0
    apow, step = np.asarray([[1, 0, 0, 0]], U), fa[None, :]
    while len(apow) < npow:  # doubling: [a^0..a^(k-1)] then a^k times them, one native EF product per step
        apow = np.concatenate([apow, R.ext_mul(apow, np.broadcast_to(step, apow.shape))])
        step = R.ext_mul(step, step)
    apow = apow[:max(npow, 1)]
    ro: Dict[int, np.ndarray] = {}
    lhp: Dict[int, int] = {}
    xs: Dict[int, np.ndarray] = {}        # per LDE height: the queries' points x_q (one per height)
    # every (matrix, point) term is (A - B[q]) / (z - x_q), and the divisor depends on (z, height) only: the
    # matrices sharing one are summed first -- their columns side by side, one dot product and one division
    groups: Dict[tuple, list] = {}  # (z, height) -> [alpha powers, opened values at z, query rows] per matrix
    for t, ms in enumerate(rounds_host):
        for k, (log_n, width, pts) in enumerate(ms):
            lh = log_n + lb
            rows = _q_rows(p, t, k) if width else None
            for z, vals in pts:
                pw = lhp.get(lh, 0)
                lhp[lh] = pw + width
                g = groups.setdefault((tuple(int(v) for v in z), lh), [[], [], []])
                if width:
                    g[0].append(apow[pw:pw + width])
                    g[1].append(np.asarray(vals, U) % PU)
                    g[2].append(np.asarray(rows, U))
    for (z, lh), (als, vals, rows) in groups.items():
        x = xs.get(lh)
        if x is None:
            row = (idx >> (log_max - lh)) & ((1 << lh) - 1)
            g = np.full(nq, two_adic_gen(lh), U)
            x = _m_u(R._pow_vec(g, _bitrev_arr(row, lh)), U(GENERATOR)) if lh else np.full(nq, GENERATOR, U)
            xs[lh] = x
        if als:
            al = np.concatenate(als)
            A = R.ext_mul(al, np.concatenate(vals)).sum(axis=0) % PU
            acc = (A[None, :] + PU - _base_dot_ef(np.concatenate(rows, 1), al)) % PU
        else:
            acc = np.zeros((nq, 4), U)
        zx = np.broadcast_to(np.asarray(z, U) % PU, (nq, 4)).copy()
        zx[:, 0] = (zx[:, 0] + PU - x) % PU
        term = R.ext_mul(acc, R.ext_inv(zx))
        ro[lh] = term if lh not in ro else (ro[lh] + term) % PU
    folded = ro[log_max]
    x = R._pow_vec(np.full(nq, two_adic_gen(log_max), U), _bitrev_arr(idx, log_max))
    # 1 / (x1 - x0) = +-1 / (2 x), and the next round's x is x^2: one inversion for all rounds
    half_inv_x = _m_u(R._pow(x, P - 2), U(pow(2, P - 2, P)))
    pairs = []
    for off, _ in enumerate(p.queries[0][1]):
        bit = ((idx >> off) & 1).astype(bool)
        sib = (p.q_sib[off] if p.q_sib is not None else np.stack([p.queries[qn][1][off][0] for qn in range(nq)])).astype(U)
        e0 = np.where(bit[:, None], sib, folded)
        e1 = np.where(bit[:, None], folded, sib)
        pairs.append(np.concatenate([e0, e1], 1))
        xn = (PU - x) % PU
        x0 = np.where(bit, xn, x)
        inv = np.where(bit, half_inv_x, (PU - half_inv_x) % PU)  # bit: x1 - x0 = 2x, else -2x
        beta = np.asarray(rp.betas[off], U)
        bx = np.broadcast_to(beta, (nq, 4)).copy()
        bx[:, 0] = (bx[:, 0] + PU - x0) % PU
        d = (e1 + PU - e0) % PU
        t_ = R.ext_mul(bx, _m_u(d, inv[:, None]))
        folded = (e0 + t_) % PU
        lfh = log_max - 1 - off
        if lfh in ro:
            b2 = R.ext_mul(beta[None, :], beta[None, :])
            folded = (folded + R.ext_mul(np.broadcast_to(b2, (nq, 4)), ro[lfh])) % PU
        x = _m_u(x, x)
        half_inv_x = _m_u(_m_u(half_inv_x, half_inv_x), U(2))  # 1 / (2 x^2) = 2 (1 / (2x))^2
    fp = np.asarray(p.final_poly, U)
    bad = np.nonzero((folded != fp[None, :]).any(axis=1))[0]
    if len(bad):
        raise ValueError(f"FRI query {int(bad[0])}: the folds do not reach the final polynomial (invalid child proof)")
    return pairs


def _build_node(prog, b, children: Sequence[tuple], ood: bool, is_first: bool, is_complete: bool, deferred=None):
    from .node_pv import node_public_values
    if not children:
        raise ValueError("a compress node needs at least one child")
    cvs = [verify_shard(prog, vk, proof, b, ood=ood) for vk, proof in children]
    pv = node_public_values(b, children, cvs, is_first=is_first, is_complete=is_complete, deferred=deferred)
    prog.commit_public_values(np.asarray(pv.a, np.int64))
    return pv


def compress_node_program(children: Sequence[tuple], ood: bool = True, is_first: bool = False,
                          is_complete: bool = False, deferred=None) -> R.RecursionProgram:
    """A compress node (prover/src/lib.rs:614-954): verify every child (ChildVk, proof bytes), check their
    public values the way the reference's core / compress recursion programs do, and commit the node's
    RecursionPublicValues (zkmips_amd/node_pv.py).  is_first: the node's first child is the execution's first
    batch (core.rs `is_first_shard`); is_complete: the node is the root of the whole execution; deferred
    (node_pv.DeferredHints): the deferred program over complete compress proofs (machine/deferred.rs)."""
    prog = R.RecursionProgram()
    b = Builder(prog)
    _build_node(prog, b, children, ood, is_first, is_complete, deferred)
    return prog


class _HintTape(R.RecursionProgram):
    """A RecursionProgram that keeps only its hints' values, in program order: verify_shard run against it
    yields a node's witness without building the instructions (node_flat).  The out-of-domain check, which
    adds no hints, is skipped."""

    def __init__(self):
        super().__init__()
        self.vals: List[np.ndarray] = []
        self.fresh: List[np.ndarray] = []  # const_fresh blocks
        self.shapes: List[tuple] = []

    def hint(self, addr, vals, mult=None):  # (RecursionProgram.hint's values, no block)
        self.vals.append((np.asarray(vals, dtype=U).reshape(-1, D) % PU).astype(np.uint32))

    def _add(self, kind, **arrays):
        if kind == "hint":
            self.vals.append(np.asarray(arrays["vals"], np.uint32))

    def _skip(self, *args, **kwargs):
        pass

    mem_write = mem_read = base_alu = ext_alu = poseidon2 = select = exp_reverse_bits = batch_fri = _skip
    fri_fold = commit_public_values = _skip


def _vk_key(vk: ChildVk) -> bytes:
    """Digest of everything in a ChildVk but its commitment (memoised on the object), which the program
    holds in a const_fresh block: with the hint sizes it keys node_flat's program templates."""
    k = vk.__dict__.get("_struct_key")
    if k is None:
        import hashlib
        chips = sorted((n, repr(c)) for n, c in vk.chips.items())
        k = hashlib.blake2b(repr((chips, vk.num_pv, list(vk.prep_order),
                                  sorted(vk.prep_heights.items()), vk.pc_start, np.asarray(vk.gcs).tolist(),
                                  vk.log_blowup, vk.num_queries, vk.pow_bits)).encode(), digest_size=16).digest()
        vk.__dict__["_struct_key"] = k
    return k


_TEMPLATES: Dict[tuple, tuple] = {}  # per process: structure key -> (FlatProgram, const_fresh mem rows)


def node_flat(children: Sequence[tuple], ood: bool = True, is_first: bool = False,
              is_complete: bool = False, deferred=None) -> "R.FlatProgram":
    """compress_node_program(children) flattened, built once per program structure.  The verifier program
    depends on the children's vks and proof shapes only; the proofs themselves enter as hints.  So the
    first node of a structure is built in full and its FlatProgram kept; a later node with the same vks and
    the same hint sizes (which fix the proof shape: chips, heights, FRI rounds, path lengths) runs
    verify_shard against a _HintTape and gets the template with its hint values replaced.  The result is
    the FlatProgram of compress_node_program(children) (tests/test_compress_verify.py)."""
    tape = _HintTape()
    b = Builder(tape)
    _build_node(tape, b, children, ood, is_first, is_complete, deferred)
    sizes = tuple(len(v) for v in tape.vals)
    key = (deferred is not None, tuple(_vk_key(vk) for vk, _ in children), tuple(tape.shapes), bool(ood), sizes,
           tuple(len(v) for v in tape.fresh))
    hit = _TEMPLATES.get(key)
    if hit is None:
        prog = compress_node_program(children, ood=ood, is_first=is_first, is_complete=is_complete, deferred=deferred)
        tpl = R.flatten(prog)
        hint_rows = tuple(int(n) for kc, _, n, _, _ in tpl.table if R.KINDS[kc] == "hint")
        fresh = [(int(tpl.table[bi][1]), int(tpl.table[bi][2])) for bi in prog.__dict__.get("fresh_blocks", [])]
        if hint_rows != sizes or [n for _, n in fresh] != [len(v) for v in tape.fresh]:
            raise AssertionError("hint tape and program disagree")
        _TEMPLATES[key] = (tpl, fresh)
        return tpl
    tpl, fresh = hit
    a = dict(tpl.a)
    a["hint"] = dict(a["hint"], vals=np.concatenate(tape.vals) if tape.vals else a["hint"]["vals"])
    if fresh:
        mv = a["mem"]["vals"].copy()
        for (s0, n), v in zip(fresh, tape.fresh):
            mv[s0:s0 + n] = v
        a["mem"] = dict(a["mem"], vals=mv)
    return R.FlatProgram(tpl.num_addrs, tpl.table, a, tpl.n, tpl.rows)


def compress_vk(machine, prep_traces, commit, num_queries: int = None) -> ChildVk:
    """The ChildVk of a compress-machine proof (compressed_fri_config: blowup 4, 42 queries) of the program
    whose preprocessed traces are `prep_traces` and whose setup gave `commit`."""
    return ChildVk.of(machine, prep_traces, commit, log_blowup=R.COMPRESS_LOG_BLOWUP,
                      num_queries=num_queries or R.COMPRESS_NUM_QUERIES)
