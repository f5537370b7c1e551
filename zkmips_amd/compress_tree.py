"""The compress stage as a dependency-driven tree (BASELINE config 5; crates/prover/src/lib.rs:614-954).

The reference reduces shard proofs two at a time (REDUCE_BATCH_SIZE = 2, lib.rs:111): trace workers build
and execute each node's recursion program and generate its traces (lib.rs:718-790), prover workers set up
the program and prove it (`compress_prover.setup(&program)`, `commit`, `open`, lib.rs:806-829), and a node
enters the queue as soon as its two children exist.  Here:

* witness generation (the node program verifying its children, zkmips_amd/recursion_verifier.py; its
  execution, RecursionShapeConfig::fix_shape and the traces, zkmips_amd/recursion.py) runs in a process
  pool, `node_witness`;
* proving runs on the GPU in `inflight` host threads, each node as soon as its witness lands;
* a node's witness job is submitted the moment its second child's proof exists, so witness generation of
  one part of the tree overlaps proving of another (no per-layer barrier).

Across ranks (`reduce_distributed`) node (L, j) belongs to the rank owning its leftmost leaf (leaves are
dealt in contiguous blocks), so every subtree inside one block is reduced locally with no communication;
only a node whose right child lives on another rank receives that child's proof, point to point.  The tree
(which children pair up) is the serial tree's, so the root is the same proof on any number of ranks.
"""
from __future__ import annotations

import pickle
import queue
import threading
import time
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

Node = Tuple[int, int]  # (layer, index); leaves are layer 0


@dataclass
class DeviceP2:
    """A Poseidon2WideDeg3 main trace to be built on the GPU (tracegen.poseidon2_wide_trace) from the
    program's permutation inputs: 8 MB of inputs instead of a 160 MB host trace per node."""
    inputs: np.ndarray   # n x 16 canonical
    height: int


@dataclass
class DeviceRows:
    """A recursion chip's main trace laid out on the GPU from its event rows (tracegen.recursion_events_trace,
    zkm_recursion_events_to_trace): n x width canonical words, no padding rows."""
    chip: str
    events: np.ndarray
    height: int


@dataclass
class DeviceExpRev:
    """ExpReverseBitsLen's main trace built on the GPU (tracegen.exp_reverse_bits_trace): each event's base,
    its exponent bits and the events' row offsets."""
    base: np.ndarray
    bits: np.ndarray
    offsets: np.ndarray
    height: int


@dataclass
class Prep:
    """A node program's proving-key identity (recursion.prep_key) and its preprocessed traces as instruction
    records ({chip: (records, height)}, recursion.prep_records; laid out on the GPU at setup by
    tracegen.recursion_instrs_trace) -- None when the worker that built this witness already sent them with
    an earlier one (register_prep keeps them)."""
    key: bytes
    traces: Optional[dict]
    session: object = None  # node_witness's dedup session: register_prep pins `key` for it (release_session)


@dataclass(frozen=True)
class VkRef:
    """A ChildVk passed to a witness worker by reference: its pickle is written once to a file (a few MB
    for a MIPS child: every chip's constraint program and lookups) and each worker process loads it once,
    instead of the submitting process pickling it into every witness job."""
    digest: bytes
    path: str


_VK_DIR: List[str] = []
# Both bounded (a long-running service sees an unbounded stream of programs): least recently used out.
_VK_REFS: "OrderedDict[int, tuple]" = OrderedDict()    # id(vk) -> (vk, VkRef), submitting side (keeps vk alive)
_VK_CACHE: "OrderedDict[bytes, object]" = OrderedDict()  # digest -> ChildVk on the loading side
_VK_LOCK = threading.Lock()
CACHE_ENTRIES = 64


def _lru_put(d: OrderedDict, k, v, cap: int = CACHE_ENTRIES):
    d[k] = v
    d.move_to_end(k)
    while len(d) > cap:
        d.popitem(last=False)


def _vk_dir() -> str:
    if not _VK_DIR:
        import atexit
        import os
        import shutil
        import tempfile
        d = tempfile.mkdtemp(prefix="zkm_vk_", dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
        atexit.register(shutil.rmtree, d, True)
        _VK_DIR.append(d)
    return _VK_DIR[0]


def vk_ref(vk) -> VkRef:
    """The VkRef of vk (its file written on first use)."""
    with _VK_LOCK:
        hit = _VK_REFS.get(id(vk))
        if hit is not None and hit[0] is vk:
            _VK_REFS.move_to_end(id(vk))
            return hit[1]
    import os
    import xxhash
    data = pickle.dumps(vk, protocol=pickle.HIGHEST_PROTOCOL)
    digest = xxhash.xxh3_128(data).digest()
    path = os.path.join(_vk_dir(), digest.hex() + ".pkl")
    if not os.path.exists(path):
        tmp = f"{path}.{os.getpid()}.{threading.get_ident()}"
        with open(tmp, "wb") as f:
            f.write(data)
        os.replace(tmp, path)
    ref = VkRef(digest, path)
    with _VK_LOCK:
        _lru_put(_VK_REFS, id(vk), (vk, ref))
        if digest not in _VK_CACHE:
            _lru_put(_VK_CACHE, digest, vk)
    return ref


def resolve_vk(v):
    """A ChildVk from a VkRef (loaded once per process; the file is this run's own, written by vk_ref) or
    the ChildVk itself."""
    if not isinstance(v, VkRef):
        return v
    with _VK_LOCK:
        vk = _VK_CACHE.get(v.digest)
    if vk is None:
        with open(v.path, "rb") as f:
            vk = pickle.loads(f.read())
        with _VK_LOCK:
            _lru_put(_VK_CACHE, v.digest, vk)
    return vk


def by_ref(children: Sequence[tuple]) -> List[tuple]:
    """Children with their verifying keys passed by reference (see VkRef)."""
    return [(vk_ref(vk), proof) for vk, proof in children]


# Worker side: per session (one tree / one Compress request), the keys whose traces this process already
# returned.  A session's consumer registers its witnesses in arrival order (Reducer.on_witness), so within
# a session "sent once" is safe; a new session (a new request, or a retry after a failed tree whose
# in-flight witnesses were dropped) starts empty, so it never depends on traces another session consumed.
_SENT_KEYS: "OrderedDict[object, set]" = OrderedDict()
_PREP_STORE: "OrderedDict[bytes, dict]" = OrderedDict()  # consumer side: traces by key (content-addressed)
# consumer side: session -> the keys its witnesses named.  A pinned key is never evicted from _PREP_STORE: a
# worker sends a program's traces once per session, so a later node of that session may need them however
# many other programs went through the store meanwhile.  release_session unpins (the end of a tree); the
# session None (callers without sessions: a worker's dedup set lives as long as the worker) is never released.
_PINS: Dict[object, set] = {}
_STORE_LOCK = threading.Lock()
SESSIONS_KEPT = 16


def new_session() -> str:
    """A fresh dedup session id for node_witness (one per tree)."""
    import uuid
    return uuid.uuid4().hex


def _sent_keys(session) -> set:
    got = _SENT_KEYS.get(session)
    if got is None:
        got = set()
        _lru_put(_SENT_KEYS, session, got, SESSIONS_KEPT)
    return got


@dataclass
class Packed:
    """A witness handed over through shared memory: the pickle of its small parts (`head`) and one
    /dev/shm file holding every array buffer (pickle protocol 5, out of band) at `spans` (offset, bytes)."""
    head: bytes
    path: str
    spans: list


_SHM_DIR = "/dev/shm"
_SHM_PREFIX = "zkm_wit_"
_shm_count = [0]


def shm_pack(obj, min_bytes: int = 1 << 20):
    """obj as a Packed (its arrays copied once into a new /dev/shm file named after the consuming process,
    this worker's parent), or obj itself when its arrays are smaller than min_bytes.  A process pool's pipe
    moves a 90 MB witness in ~0.35 s (pickle, pipe, unpickle in the consumer under its GIL); this is one
    copy here and none there (shm_unpack maps the file)."""
    import os
    bufs = []
    head = pickle.dumps(obj, protocol=5, buffer_callback=bufs.append)
    raws = [b.raw() for b in bufs]
    total = sum(r.nbytes for r in raws)
    if total < min_bytes:
        return obj
    _shm_count[0] += 1
    path = f"{_SHM_DIR}/{_SHM_PREFIX}{os.getppid()}_{os.getpid()}_{_shm_count[0]}"
    fd = os.open(path, os.O_CREAT | os.O_EXCL | os.O_RDWR, 0o600)
    try:
        # write(2) into the tmpfs file: ~2x faster than stores through a fresh mapping, which fault page by page
        spans, off = [], 0
        for r in raws:
            mv = memoryview(r).cast("B")
            done = 0
            while done < mv.nbytes:
                done += os.write(fd, mv[done:])
            spans.append((off, mv.nbytes))
            off += mv.nbytes
    except BaseException:
        os.unlink(path)
        raise
    finally:
        os.close(fd)
    return Packed(head, path, spans)


def shm_unpack(x):
    """The object shm_pack made: its arrays map the file privately (copy on write), the file is unlinked at
    once (the mapping lives as long as the arrays)."""
    if not isinstance(x, Packed):
        return x
    import mmap
    import os
    fd = os.open(x.path, os.O_RDONLY)
    try:
        mm = mmap.mmap(fd, os.fstat(fd).st_size, flags=mmap.MAP_PRIVATE, prot=mmap.PROT_READ | mmap.PROT_WRITE)
    finally:
        os.close(fd)
        os.unlink(x.path)
    mv = memoryview(mm)
    return pickle.loads(x.head, buffers=[mv[o:o + n] for o, n in x.spans])


def shm_cleanup():
    """Remove /dev/shm witness files addressed to this process that were never unpacked (a tree that
    failed part-way)."""
    import glob
    import os
    for f in glob.glob(f"{_SHM_DIR}/{_SHM_PREFIX}{os.getpid()}_*"):
        try:
            os.unlink(f)
        except OSError:
            pass


def _store_put(key: bytes, traces: dict):
    """_PREP_STORE[key] = traces, then least recently used unpinned keys out down to CACHE_ENTRIES (pinned
    keys stay, beyond the bound if need be).  Caller holds _STORE_LOCK."""
    _PREP_STORE[key] = traces
    _PREP_STORE.move_to_end(key)
    excess = len(_PREP_STORE) - CACHE_ENTRIES
    if excess > 0:
        pinned = set().union(*_PINS.values()) if _PINS else set()
        for k in [k for k in _PREP_STORE if k not in pinned][:excess]:
            del _PREP_STORE[k]


def register_prep(wit):
    """Record a compact witness's preprocessed traces on the consuming side (called in arrival order, before
    any witness of the same worker that omits them is proven) and pin its key for the witness's session.  A
    Packed witness is unpacked first."""
    wit = shm_unpack(wit)
    p = wit[0]
    if isinstance(p, Prep):
        with _STORE_LOCK:
            _PINS.setdefault(p.session, set()).add(p.key)
            if p.traces is not None:
                _store_put(p.key, p.traces)
    return wit


def release_session(session):
    """Unpin the keys of a finished session (Reducer.run does this for the sessions of its witnesses)."""
    if session is None:
        return
    with _STORE_LOCK:
        _PINS.pop(session, None)


def _prep_traces_of(p: "Prep") -> dict:
    if p.traces is not None:
        return p.traces
    with _STORE_LOCK:
        t = _PREP_STORE.get(p.key)
    if t is None:
        raise RuntimeError("compress node: preprocessed traces of this program were never received")
    return t


def device_prep(records: dict) -> dict:
    """A program's preprocessed traces laid out on the current GPU from its instruction records
    (zkm_recursion_instrs_to_trace), waited for."""
    import torch
    from . import tracegen as TG
    out = {}
    for name, (recs, h) in records.items():
        r = np.ascontiguousarray(recs, np.uint32)
        t = torch.from_numpy(r.reshape(-1).view(np.int32) if r.size else np.zeros(1, np.int32)).cuda()
        out[name] = TG.recursion_instrs_trace(name, t, len(r), h)
    torch.cuda.current_stream().synchronize()
    return out


def compact_traces(rec, shape) -> dict:
    """The node's main traces as device work items: the event-row chips (DeviceRows), ExpReverseBitsLen
    (DeviceExpRev) and Poseidon2WideDeg3 (DeviceP2) -- the events only, no padding rows."""
    from . import recursion as R
    h = R._heights(rec, shape)
    out = {"MemoryConst": DeviceRows("MemoryConst", np.zeros((0, 1), np.uint32), h["MemoryConst"])}
    for name in ("MemoryVar", "BaseAlu", "ExtAlu", "BatchFRI", "Select", "PublicValues"):
        out[name] = DeviceRows(name, np.ascontiguousarray(R.main_events(rec, name)), h[name])
    er = rec.ev["exprev"]
    L = rec.flat.a["exprev"]["L"]
    off = np.concatenate([[0], np.cumsum(L)]).astype(np.int64)
    out["ExpReverseBitsLen"] = DeviceExpRev(np.ascontiguousarray(er[off[:-1], 0]), np.ascontiguousarray(er[:, 1]), off,
                                            h["ExpReverseBitsLen"])
    out["Poseidon2WideDeg3"] = DeviceP2(R.p2_inputs(rec), h["Poseidon2WideDeg3"])
    return out


def node_witness(children: Sequence[tuple], fix: bool = True, p2_on_device: bool = False, compact: bool = False,
                 dedup: bool = True, session=None, is_first: bool = False, is_complete: bool = False, deferred=None):
    """Worker body (no GPU): the compress node's program from its (ChildVk, proof) children, executed,
    padded to the first allowed recursion shape (fix=False: natural power-of-two heights, for small
    tests), as a compress-machine shard.  Returns (prep traces, main traces, public values, shape,
    seconds); with p2_on_device the Poseidon2WideDeg3 entry is a DeviceP2 (see materialize).  compact:
    every main trace is a device work item (compact_traces) and the prep traces a Prep, sent once per
    program structure, worker process and `session` (dedup; a consumer must pass the witnesses of one worker
    through register_prep in the order they were made, as Reducer does; one session per tree) -- a fraction
    of the bytes through the pool's pipe.  is_first / is_complete: the node covers the execution's first
    shard / is the root of the whole tree (node_flags).  deferred (node_pv.DeferredHints): the children are the
    request's deferred proofs and the node is their deferred program (machine/deferred.rs)."""
    from . import recursion as R
    from . import recursion_verifier as RV
    t0 = time.perf_counter()
    children = [(resolve_vk(vk), proof) for vk, proof in children]
    # a FlatProgram: built once per program structure, then hints only
    prog = RV.node_flat(children, is_first=is_first, is_complete=is_complete, deferred=deferred)
    t1 = time.perf_counter()
    shape = R.fix_shape(prog) if fix else {k: max(4, (h - 1).bit_length()) for k, h in R.program_heights(prog).items()}
    if compact:
        rec = R.execute(prog)
        if rec.flat.n["frifold"]:
            raise ValueError("FriFold instructions need the wide machine")
        key = R.prep_key(rec, shape)
        prep = None
        sent = _sent_keys(session) if dedup else set()
        if key not in sent:
            pr = R.prep_records(rec, shape)
            prep = {c.name: pr[c.name] for c in R.compress_machine().chips if c.prep_width}
            sent.add(key)
        traces = compact_traces(rec, shape)
        t2 = time.perf_counter()
        return Prep(key, prep, session), traces, rec.public_values, shape, {"build_s": t1 - t0, "execute_and_traces_s": t2 - t1}
    if p2_on_device:
        _, prep, traces, pvs, p2in, p2h = R.shard_parts(prog, shape)
        traces["Poseidon2WideDeg3"] = DeviceP2(p2in, p2h)
    else:
        _, prep, traces, pvs = R.shard(prog, shape)
    t2 = time.perf_counter()
    return prep, traces, pvs, shape, {"build_s": t1 - t0, "execute_and_traces_s": t2 - t1}


def warm_worker() -> int:
    """A witness worker's one-time start-up, outside any timed region: the verifier / runtime modules and the
    native host library (libzkm_trace.so) loaded, as the first node job would otherwise do."""
    import os
    from . import recursion as R
    from . import recursion_verifier as RV  # noqa: F401
    for name in ("zkm_host_recursion_execute", "zkm_host_poseidon2_permute", "zkm_host_ef_mul"):
        R._host(name)
    return os.getpid()


def prebuild_template(children: Sequence[tuple], is_first: bool = False) -> int:
    """Build (and keep, in this process) the node program template of `children`'s structure
    (recursion_verifier.node_flat) without executing it: later nodes of the same structure -- any children with the
    same vks up to their commitment and the same proof shapes -- only replace hint values.  The reference keeps
    its programs ready the same way: the compress (join) programs precomputed per shape when the prover is built
    (prover/src/lib.rs:398-410 `join_programs_map`), the core programs in an LRU cache by shape (:366-396).  The
    children are real proofs that chain (every check applies); returns the number of templates held."""
    from . import recursion_verifier as RV
    RV.node_flat([(resolve_vk(vk), p) for vk, p in children], is_first=is_first)
    return len(RV._TEMPLATES)


def node_witness_shm(*args, **kwargs):
    """node_witness through shared memory (shm_pack): the pool's job for a consumer whose Reducer unpacks
    (register_prep)."""
    return shm_pack(node_witness(*args, **kwargs))


def materialize(traces: dict) -> dict:
    """Build every device work item's trace on the current GPU (DeviceP2: rows past the inputs the
    permutation of zero; DeviceRows / DeviceExpRev: zero padding rows) and wait for them; other entries
    pass through."""
    out = dict(traces)
    todo = [(k, v) for k, v in traces.items() if isinstance(v, (DeviceP2, DeviceRows, DeviceExpRev))]
    if not todo:
        return out
    import torch
    from . import tracegen as TG

    def up(a, dtype=np.int32):
        a = np.ascontiguousarray(a)
        return torch.from_numpy(a.view(dtype).reshape(-1) if a.size else np.zeros(1, dtype)).cuda()
    for k, v in todo:
        if isinstance(v, DeviceP2):
            n = len(v.inputs)
            ev = np.zeros((max(n, 1), 32), np.uint32)
            ev[:n, :16] = v.inputs
            out[k] = TG.poseidon2_wide_trace(up(ev), n, v.height)
        elif isinstance(v, DeviceRows):
            out[k] = TG.recursion_events_trace(v.chip, up(v.events), len(v.events), v.height)
        else:
            out[k] = TG.exp_reverse_bits_trace(up(v.base), up(v.bits), up(v.offsets, np.int64), len(v.base), v.height)
    torch.cuda.current_stream().synchronize()
    return out


_CVK_LOCK = threading.Lock()
_CVK_CHIPS: Dict[object, object] = {}  # 0 -> the compress machine's chip shapes; (commit, shape, nq) -> ChildVk
# (insertion-ordered; bounded to CACHE_ENTRIES child keys, oldest out)


def compress_child_vk(commit, shape: Dict[str, int], num_queries: int = None):
    """The ChildVk of a compress-machine proof from what a parent needs to know of it: the program's
    preprocessed commitment and its recursion shape (every preprocessed height is 2^shape).  The chip
    descriptions are the compress machine's (built once per process)."""
    from . import recursion as R
    from . import recursion_verifier as RV
    with _CVK_LOCK:
        chips = _CVK_CHIPS.get(0)
        if chips is None:
            m = R.compress_machine()
            chips = {"shapes": {c.name: RV.ChipShape.of(c) for c in m.chips}, "num_pv": m.num_pv,
                     "prep": [c.name for c in m.chips if c.prep_width], "pc_start": m.pc_start}
            _CVK_CHIPS[0] = chips
        # one object per (program, shape): parents pass it by reference (vk_ref) without re-pickling it
        key = (tuple(int(x) for x in commit), tuple(sorted(shape.items())), num_queries)
        vk = _CVK_CHIPS.get(key)
        if vk is not None:
            return vk
    heights = {k: 1 << shape[k] for k in chips["prep"]}
    order = sorted(heights, key=lambda k: (-heights[k], k))
    from .septic import CURVE_CUMULATIVE_SUM_START
    vk = RV.ChildVk(chips["shapes"], chips["num_pv"], np.asarray(commit, np.int64), order, heights,
                    pc_start=chips["pc_start"], gcs=np.asarray(CURVE_CUMULATIVE_SUM_START, np.int64),
                    log_blowup=R.COMPRESS_LOG_BLOWUP, num_queries=num_queries or R.COMPRESS_NUM_QUERIES)
    with _CVK_LOCK:
        got = _CVK_CHIPS.get(key)
        if got is not None:
            return got
        _CVK_CHIPS[key] = vk
        while len(_CVK_CHIPS) > CACHE_ENTRIES + 1:  # entry 0 (the chip shapes) is kept
            _CVK_CHIPS.pop(next(k for k in _CVK_CHIPS if k != 0))
        return vk


@dataclass
class TreeStats:
    witness_s: float = 0.0            # summed worker seconds (program build + execution + traces)
    build_s: float = 0.0
    execute_s: float = 0.0
    prove_s: float = 0.0              # summed GPU-thread seconds inside prove_shard
    setup_s: float = 0.0              # zkm_setup of new programs
    setups: int = 0
    lookups: int = 0
    proofs: int = 0
    shapes: Dict[str, int] = field(default_factory=dict)  # chosen shape -> nodes


class GpuProvers:
    """Proving keys of node programs, looked up by a digest of the preprocessed traces (programs with the
    same structure share one zkm_setup), as `compress_prover.setup(&program)` (lib.rs:807) would compute
    the same key for them."""

    def __init__(self, dev, num_queries=None, max_provers: int = 16):
        from . import recursion as R
        self.dev = dev
        self.machine = R.compress_machine()
        self.kw = dict(num_queries=num_queries or R.COMPRESS_NUM_QUERIES, log_blowup=R.COMPRESS_LOG_BLOWUP)
        # least recently used out: each prover holds its program's preprocessed LDE and tree on the GPU,
        # and a long-running service sees a new program for every distinct core program (its vk commit
        # is in MemoryConst)
        self.cache: "OrderedDict[bytes, object]" = OrderedDict()
        self.max_provers = max(1, max_provers)
        self.lock = threading.Lock()

    def get(self, prep, stats: TreeStats):
        """The prover of a node's program: prep is its preprocessed traces, or a Prep (compact witness)."""
        from .prover import HipProver
        if isinstance(prep, Prep):
            register_prep((prep,))
            key = prep.key
        else:
            key = prep_digest(prep)
        with self.lock:
            stats.lookups += 1
            pr = self.cache.get(key)
            if pr is None:
                t = time.perf_counter()
                pt = device_prep(_prep_traces_of(prep)) if isinstance(prep, Prep) else prep
                pr = HipProver(self.dev, self.machine, pt, **self.kw)
                stats.setup_s += time.perf_counter() - t
                stats.setups += 1
                _lru_put(self.cache, key, pr, self.max_provers)  # an evicted prover in use stays alive
            else:
                self.cache.move_to_end(key)
        return pr


def prep_digest(prep) -> bytes:
    """Identity of a program's proving key: xxh3-128 over its preprocessed traces (name, shape, words)."""
    try:
        import xxhash
        h = xxhash.xxh3_128()
    except ImportError:  # pragma: no cover
        import hashlib
        h = hashlib.sha256()
    for k in sorted(prep):
        v = prep[k]
        if v is None:
            continue
        h.update(k.encode() + np.asarray(v.shape, np.int64).tobytes())
        h.update(np.ascontiguousarray(v).view(np.uint8).data)
    return h.digest()


def tree_nodes(n_leaves: int) -> List[List[Node]]:
    """The serial tree's layers: layer L has ceil(n_{L-1} / 2) nodes; node (L, j) has children
    (L-1, 2j) and (L-1, 2j + 1) when the latter exists (a last odd node has one child)."""
    layers, n, L = [], n_leaves, 0
    while n > 1:
        L += 1
        n = (n + 1) // 2
        layers.append([(L, j) for j in range(n)])
    return layers


def children_of(node: Node, width_below: int) -> List[Node]:
    L, j = node
    return [(L - 1, c) for c in (2 * j, 2 * j + 1) if c < width_below]


def node_tag(children) -> tuple:
    """A cheap stand-in for a node's program structure (node_flat's template key), for AffinityPool: the
    number of children and their proofs' lengths (a proof's length is fixed by its shape)."""
    return (len(children),) + tuple(len(p) for _, p in children)


class AffinityPool:
    """The witness workers as single-process executors (spawned: fresh interpreters, safe beside a GPU
    process), so a node's job can go to a worker that already holds its program's template
    (recursion_verifier.node_flat, built once per structure and process): submit(fn, *args, tag=t) takes
    the least loaded worker, among those preferring one that has run tag t.  Otherwise the surface of a
    ProcessPoolExecutor (submit / shutdown)."""

    def __init__(self, n: int):
        import multiprocessing as mpc
        from concurrent.futures import ProcessPoolExecutor
        ctx = mpc.get_context("spawn")
        self._ex = [ProcessPoolExecutor(1, mp_context=ctx) for _ in range(max(1, n))]
        self._load = [0] * len(self._ex)
        self._tags = [set() for _ in self._ex]
        self._lock = threading.Lock()

    def submit(self, fn, *args, tag=None, **kwargs):
        with self._lock:
            i = min(range(len(self._ex)),
                    key=lambda k: (self._load[k], 0 if tag is not None and tag in self._tags[k] else 1, k))
            self._load[i] += 1
            if tag is not None:
                self._tags[i].add(tag)
        fut = self._ex[i].submit(fn, *args, **kwargs)
        fut.add_done_callback(lambda f, k=i: self._release(k))
        return fut

    def warm(self):
        """warm_worker on every worker (each its own executor), waited for."""
        self.run_all(warm_worker)
        return self

    def run_all(self, fn, *args, **kwargs) -> list:
        """fn(*args, **kwargs) on every worker, waited for: their results in worker order."""
        return [f.result() for f in [e.submit(fn, *args, **kwargs) for e in self._ex]]

    def _release(self, k: int):
        with self._lock:
            self._load[k] -= 1

    def shutdown(self, wait: bool = True):
        for e in self._ex:
            e.shutdown(wait=wait)
        shm_cleanup()


def node_flags(node: Node, root: Node, complete: bool = True) -> dict:
    """node_witness's flags for node (L, j): its first leaf is the execution's first shard (core.rs
    `is_first_shard`, lib.rs:543 batch_idx == 0) and it is the tree's root (is_complete, lib.rs:901-909).
    complete=False: the root is not asserted complete either (trees of leaves that are not a whole MIPS
    execution, e.g. synthetic test machines, whose root assert_complete would reject)."""
    return {"is_first": node[1] == 0, "is_complete": complete and node == root}


class Reducer:
    """The event-driven reduction of one rank's part of the tree.

    witness(children, flags) -> concurrent.futures.Future of node_witness's result (flags: node_flags);
    prove(witness) -> (child vk, proof bytes) for the parent (GPU, called from `inflight` threads).
    complete: the root is asserted complete (node_flags).  The dedup sessions named by the witnesses'
    Prep are released when run() ends."""

    def __init__(self, submit_witness: Callable, prove: Callable, inflight: int = 3,
                 on_witness: Callable = register_prep, complete: bool = True):
        self.submit_witness = submit_witness
        self.prove = prove
        self.on_witness = on_witness  # called on each witness in arrival order, before it is queued
        self.complete = complete
        self.sessions: set = set()
        self.times: Dict[Node, Dict[str, float]] = {}  # node -> perf_counter of submit / witness / proved
        self.inflight = max(1, inflight)
        self.events: "queue.Queue" = queue.Queue()
        self.gpu_q: "queue.Queue" = queue.Queue()

    def _gpu_worker(self):
        while True:
            item = self.gpu_q.get()
            if item is None:
                return
            node, wit = item
            try:
                self.events.put(("proof", node, self.prove(wit)))
            except BaseException as e:  # surfaced by the event loop
                self.events.put(("error", node, e))

    def run(self, done: Dict[Node, tuple], mine: Sequence[Node], widths: Dict[int, int],
            remote: Optional[Callable] = None, on_done: Optional[Callable] = None) -> Dict[Node, tuple]:
        """Prove every node in `mine` (a set closed under 'left child'), given `done` (leaves and anything
        already known).  remote(poll) -> [(node, (vk, proof))] delivers children other ranks prove;
        on_done(node, result) is called for every node proven here."""
        pending = set(mine)
        submitted = set()
        top = max(widths)
        root = (top, 0)
        futs: Dict[Node, object] = {}  # witness jobs whose result has not been taken yet
        threads = [threading.Thread(target=self._gpu_worker, daemon=True) for _ in range(self.inflight)]
        for t in threads:
            t.start()

        def ready(node):
            ch = children_of(node, widths[node[0] - 1])
            return all(c in done for c in ch), ch

        def try_submit():
            for node in sorted(pending - submitted):
                ok, ch = ready(node)
                if ok:
                    submitted.add(node)
                    self.times.setdefault(node, {})["submit"] = time.perf_counter()
                    fut = self.submit_witness([done[c] for c in ch], node_flags(node, root, self.complete))
                    futs[node] = fut
                    fut.add_done_callback(lambda f, n=node: self.events.put(("witness", n, f)))
        ok = False
        try:
            try_submit()
            while pending:
                if remote is not None:
                    got = remote()
                    for node, res in got:
                        done[node] = res
                    if got:
                        try_submit()
                try:
                    kind, node, val = self.events.get(timeout=0.005 if remote is not None else 60.0)
                except queue.Empty:
                    continue
                if kind == "witness":
                    futs.pop(node, None)
                    self.times.setdefault(node, {})["witness"] = time.perf_counter()
                    wit = self.on_witness(val.result())
                    if isinstance(wit, tuple) and wit and isinstance(wit[0], Prep) and wit[0].session is not None:
                        self.sessions.add(wit[0].session)
                    self.gpu_q.put((node, wit))
                elif kind == "proof":
                    self.times.setdefault(node, {})["proved"] = time.perf_counter()
                    done[node] = val
                    pending.discard(node)
                    if on_done:
                        on_done(node, val)
                    try_submit()
                else:
                    raise val
            ok = True
        finally:
            if not ok:  # a failed tree: its in-flight witnesses are discarded when they land
                for f in futs.values():
                    f.cancel()
                    f.add_done_callback(_discard_witness)
            for _ in threads:
                self.gpu_q.put(None)
            for t in threads:
                t.join(timeout=60)
            for sid in self.sessions:  # every node of the sessions has been proven (or the tree failed)
                release_session(sid)
            self.sessions.clear()
        return done


def _discard_witness(f):
    """Drop a witness nobody will prove: unlink its /dev/shm file (a Packed one)."""
    if f.cancelled() or f.exception() is not None:
        return
    x = f.result()
    if isinstance(x, Packed):
        import os
        try:
            os.unlink(x.path)
        except OSError:
            pass


def owner(node: Node, n_leaves: int, world: int) -> int:
    """The rank that proves node (L, j): the owner of its leftmost leaf j * 2^L, leaves dealt to ranks in
    contiguous blocks."""
    L, j = node
    return min(world - 1, ((j << L) * world) // n_leaves)


def reduce_serial(leaves: Sequence[tuple], reducer: Reducer) -> tuple:
    """The whole tree on one GPU: returns the root's (vk, proof) (a single leaf is its own root)."""
    layers = tree_nodes(len(leaves))
    if not layers:
        return leaves[0]
    widths = {0: len(leaves)}
    widths.update({i + 1: len(l) for i, l in enumerate(layers)})
    done = {(0, i): leaves[i] for i in range(len(leaves))}
    mine = [n for l in layers for n in l]
    reducer.run(done, mine, widths)
    return done[layers[-1][0]]


def reduce_with_deferred(leaves: Sequence[tuple], deferred: Sequence[tuple], submit_witness: Callable,
                         prove: Callable, inflight: int = 3) -> tuple:
    """A Compress request with deferred proofs (prover/src/lib.rs:614-954 over get_first_layer_inputs, :599-612):
    the execution's shard leaves reduce to a root that is not complete; every deferred proof (ChildVk, complete
    compress proof) gets its own deferred node (first_layer_batch_size 1) whose reconstruct-deferred chain starts
    where the previous one ended (hash_deferred_proofs) and whose other values come from the last shard
    (get_recursion_deferred_inputs, :551-593); then [execution root, deferred nodes...] in that order reduce to
    the complete root, whose end digest must be the execution's committed deferred_proofs_digest
    (assert_complete).  submit_witness / prove as for Reducer; returns the root's (vk, proof)."""
    from . import node_pv as NP
    from . import recursion_verifier as RV
    if not leaves or not deferred:
        raise ValueError("reduce_with_deferred: shard leaves and deferred proofs")
    if len(leaves) == 1:
        core = prove(register_prep(submit_witness(list(leaves), {"is_first": True, "is_complete": False}).result()))
    else:
        core = reduce_serial(leaves, Reducer(submit_witness, prove, inflight, complete=False))
    core_vk = resolve_vk(leaves[0][0])
    last_pv = RV.parse_shard_proof(leaves[-1][1]).pv
    digest = np.zeros(8, np.int64)
    futs = []
    for vk, p in deferred:
        h = NP.DeferredHints.of(core_vk, last_pv, digest)
        futs.append(submit_witness([(vk, p)], {"is_first": False, "is_complete": False, "deferred": h}))
        digest = NP.hash_deferred_proofs(digest, [RV.parse_shard_proof(p).pv])
    nodes = [prove(register_prep(f.result())) for f in futs]
    return reduce_serial([core] + nodes, Reducer(submit_witness, prove, inflight, complete=True))


MSG_BYTES = 8 << 20  # fixed point-to-point message: a pickled (vk, proof) of a node (KB-MB)


def _pack(obj) -> np.ndarray:
    raw = pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL)
    if len(raw) + 8 > MSG_BYTES:
        raise ValueError(f"compress node message of {len(raw)} bytes exceeds {MSG_BYTES}")
    buf = np.zeros(MSG_BYTES, np.uint8)
    buf[:8] = np.frombuffer(len(raw).to_bytes(8, "little"), np.uint8)
    buf[8:8 + len(raw)] = np.frombuffer(raw, np.uint8)
    return buf


def _unpack(buf: np.ndarray):
    n = int.from_bytes(buf[:8].tobytes(), "little")
    return pickle.loads(buf[8:8 + n].tobytes())


_GLOO = {}


def _exchange_group():
    """Proof messages go over gloo (host memory, KB-MB each): a gloo subgroup when the default group is
    RCCL, whose p2p receives would otherwise sit on the GPU waiting for the sender."""
    import torch.distributed as dist
    if dist.get_backend() == "gloo":
        return None
    if "g" not in _GLOO:
        _GLOO["g"] = dist.new_group(backend="gloo")
    return _GLOO["g"]


def reduce_distributed(leaves: Sequence[tuple], reducer: Reducer, broadcast_root: bool = True):
    """The tree across the ranks of the default process group (module docstring).  Every rank passes the
    same leaves; returns the root's (vk, proof) on every rank (broadcast from the rank that proves it), or
    on the root's owner only with broadcast_root=False (None elsewhere)."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(), dist.get_rank()
    grp = _exchange_group()
    n = len(leaves)
    layers = tree_nodes(n)
    if not layers:
        return leaves[0]
    widths = {0: n}
    widths.update({i + 1: len(l) for i, l in enumerate(layers)})
    nodes = [nd for l in layers for nd in l]
    mine = [nd for nd in nodes if owner(nd, n, world) == rank]
    # children proven elsewhere that my nodes need, and my nodes others need
    need = [(c, owner(c, n, world)) for nd in mine for c in children_of(nd, widths[nd[0] - 1])
            if c[0] > 0 and owner(c, n, world) != rank]
    give = {nd: owner((nd[0] + 1, nd[1] // 2), n, world) for nd in mine
            if nd[0] < len(layers) and owner((nd[0] + 1, nd[1] // 2), n, world) != rank}
    done = {(0, i): leaves[i] for i in range(n)}
    arrived: "queue.Queue" = queue.Queue()

    def receiver(buf, work):
        work.wait()
        # the message names its node: one sender may send two nodes to this rank, completed in either
        # order, and untagged receives from one source match in posting order, not by node
        arrived.put(_unpack(buf.numpy()))
    rthreads = []
    for c, src in need:  # one message per (sender, receiver) pair and node: posted up front, waited in threads
        buf = torch.empty(MSG_BYTES, dtype=torch.uint8)
        t = threading.Thread(target=receiver, args=(buf, dist.irecv(buf, src=src, group=grp)), daemon=True)
        t.start()
        rthreads.append(t)
    sends = []

    def remote():
        got = []
        while True:
            try:
                got.append(arrived.get_nowait())
            except queue.Empty:
                return got

    def on_done(node, res):
        if node in give:
            t = torch.from_numpy(_pack((node, res)))
            sends.append((t, dist.isend(t, dst=give[node], group=grp)))

    reducer.run(done, mine, widths, remote=remote if need else None, on_done=on_done)
    for t, w in sends:
        w.wait()
    for t in rthreads:
        t.join(timeout=60)
    root = layers[-1][0]
    ro = owner(root, n, world)
    if not broadcast_root:
        return done[root] if rank == ro else None
    obj = [done[root] if rank == ro else None]
    dist.broadcast_object_list(obj, src=ro, group=grp)
    return obj[0]
