"""Config 5's compress tree (zkmips_amd/compress_tree.py): RecursionShapeConfig::fix_shape
(crates/recursion/core/src/shape.rs:50-75,115-170), the dependency-driven reduction with witness
generation in a process pool, and — on the GPU — a node verifying two real MIPS-shard leaves, padded to
a reference recursion shape, proven byte-identically to the oracle."""
import multiprocessing as mpc
from concurrent.futures import Future, ProcessPoolExecutor

import numpy as np
import pytest

from tests import _oracle as O
from zkmips_amd import compress_tree as CT
from zkmips_amd import recursion as R
from zkmips_amd import recursion_verifier as RV
from zkmips_amd import workloads as W

NQ = 8


def test_shapes_are_the_references():
    # shape.rs:126-166, fastest first; every compress chip named, PublicValues at PUB_VALUES_LOG_HEIGHT
    names = {c.name for c in R.compress_machine().chips}
    assert [sorted(s) for s in R.RECURSION_SHAPES] == [sorted(names)] * 3
    assert R.RECURSION_SHAPES[0]["MemoryVar"] == 18 and R.RECURSION_SHAPES[1]["BatchFRI"] == 19
    assert R.RECURSION_SHAPES[2]["ExtAlu"] == 19 and all(s["PublicValues"] == 4 for s in R.RECURSION_SHAPES)


def test_fix_shape_first_fit():
    prog = R.program_ext_four_ops(100)
    h = R.program_heights(prog)
    assert R.fix_shape(prog) == R.RECURSION_SHAPES[0]
    # the heights are what generate_traces pads: natural traces have next_pow2 of them
    _, _, tr, _ = R.shard(prog)
    for k, v in tr.items():
        assert v.shape[0] == max(16, 1 << max(0, (h[k] - 1).bit_length())), k
    # a program needing ExtAlu 2^16 rows skips the fastest shape; 2^20 fits none
    assert R.fix_shape(prog, [dict(R.RECURSION_SHAPES[0], ExtAlu=4)] + R.RECURSION_SHAPES[1:]) == R.RECURSION_SHAPES[1]
    with pytest.raises(ValueError):
        R.fix_shape(prog, [dict(s, ExtAlu=4) for s in R.RECURSION_SHAPES])
    # padding to the shape keeps the program's proof valid
    m, prep, tr, pv = R.shard(prog, R.RECURSION_SHAPES[0])
    assert tr["ExtAlu"].shape[0] == 1 << 15 and tr["MemoryVar"].shape[0] == 1 << 18


@pytest.fixture(scope="module")
def fib_leaves():
    m, prep, _, _ = W.fib_shard(256, seed=3)
    pr = O.OracleProver(m, prep, num_queries=NQ)
    vk = RV.ChildVk.of(m, prep, pr.commit, num_queries=NQ)
    out = []
    for s in range(4):
        _, _, tr, pv = W.fib_shard(256, seed=10 + s)
        rc, p = pr.prove(tr, pv)
        assert rc == 0
        out.append((vk, p))
    return out


def _oracle_prove_factory(nq):
    cm = R.compress_machine()
    kw = dict(num_queries=nq, log_blowup=R.COMPRESS_LOG_BLOWUP)

    def prove(wit):
        prep, traces, pvs, shape, _ = wit
        pr = O.OracleProver(cm, prep, **kw)
        rc, p = pr.prove(traces, pvs)
        assert rc == 0 and pr.verify(p) == 0
        return CT.compress_child_vk(pr.commit, shape, num_queries=nq), p
    return prove


def _witness_small(children, **flags):
    return CT.node_witness(children, fix=False, **flags)


def test_tree_with_witness_pool_matches_serial(fib_leaves):
    """4 leaves -> 3 node proofs: the event-driven reduction (witnesses in a spawn process pool, proofs in
    2 threads) gives the same root as proving the layers one after another."""
    prove = _oracle_prove_factory(4)
    with ProcessPoolExecutor(2, mp_context=mpc.get_context("spawn")) as pool:
        # verifying keys by reference (VkRef: written once, loaded once per worker)
        # (Fibonacci leaves are no MIPS execution: the root is not asserted complete)
        red = CT.Reducer(lambda ch, fl: pool.submit(_witness_small, CT.by_ref(ch), **fl), prove, inflight=2,
                         complete=False)
        root = CT.reduce_serial(fib_leaves, red)
    a = prove(_witness_small(fib_leaves[:2]))
    b = prove(_witness_small(fib_leaves[2:]))
    want = prove(_witness_small([a, b]))
    assert root[1] == want[1]
    assert np.array_equal(root[0].commit, want[0].commit)
    # a complete root needs an execution shard (assert_complete): over these children it is refused
    with pytest.raises(ValueError, match="execution shard"):
        _witness_small([a, b], is_complete=True)


def test_tree_with_affinity_pool_matches_serial(fib_leaves):
    """The same tree through CT.AffinityPool (single-process workers, jobs routed by node_tag to a worker
    that has built the structure's program template): the same root."""
    prove = _oracle_prove_factory(4)
    pool = CT.AffinityPool(2)
    try:
        red = CT.Reducer(lambda ch, fl: pool.submit(_witness_small, CT.by_ref(ch), **fl, tag=CT.node_tag(ch)), prove,
                         inflight=2, complete=False)
        root = CT.reduce_serial(fib_leaves, red)
    finally:
        pool.shutdown()
    a = prove(_witness_small(fib_leaves[:2]))
    b = prove(_witness_small(fib_leaves[2:]))
    assert root[1] == prove(_witness_small([a, b]))[1]


def _packed_job(n):
    arrs = {"a": np.arange(n, dtype=np.uint32), "b": np.arange(2 * n, dtype=np.int64).reshape(2, n)[:, ::2]}
    return CT.shm_pack((CT.Prep(b"k", arrs), "small", 3))


def test_witness_through_shared_memory():
    """shm_pack in a worker / shm_unpack here: the same arrays (non-contiguous ones too), writable, the
    /dev/shm file gone once mapped; small objects go through the pipe as themselves."""
    import glob
    import os
    pool = CT.AffinityPool(1)
    try:
        x = pool.submit(_packed_job, 1 << 19).result()
        assert isinstance(x, CT.Packed) and os.path.exists(x.path)
        wit = CT.register_prep(x)
        assert not os.path.exists(x.path)
        n = 1 << 19
        assert np.array_equal(wit[0].traces["a"], np.arange(n, dtype=np.uint32)) and wit[1:] == ("small", 3)
        assert np.array_equal(wit[0].traces["b"], np.arange(2 * n, dtype=np.int64).reshape(2, n)[:, ::2])
        wit[0].traces["a"][0] = 7  # copy on write
        assert not isinstance(pool.submit(_packed_job, 16).result(), CT.Packed)
        y = pool.submit(_packed_job, 1 << 19).result()  # never unpacked: removed at shutdown
    finally:
        pool.shutdown()
    assert not os.path.exists(y.path)
    assert not glob.glob(f"/dev/shm/zkm_wit_{os.getpid()}_*")


def test_affinity_pool_routing():
    """Least loaded first; among equally loaded workers, one that has run the tag."""
    import os
    import time
    pool = CT.AffinityPool(2)
    try:
        p0 = pool.submit(os.getpid, tag="a").result()
        busy = pool.submit(time.sleep, 1.0, tag="a")      # worker 0 (has "a") busy
        p1 = pool.submit(os.getpid, tag="x").result()     # -> the idle worker 1
        busy.result()
        assert p1 != p0
        assert pool.submit(os.getpid, tag="x").result() == p1  # both idle: the one that ran "x"
        assert pool.submit(os.getpid, tag="a").result() == p0
    finally:
        pool.shutdown()


def _host_layout(v):
    """A compact witness's device work item laid out on the host (what the kernels must produce)."""
    if isinstance(v, CT.DeviceRows):
        from zkmips_amd import tracegen as TG
        _, w, k = TG.RECURSION_EVENT_CHIPS[v.chip]
        return R._lay_out(v.events, max(k, 1), v.height) if k else np.zeros((v.height, 1), np.uint32)
    if isinstance(v, CT.DeviceP2):
        t = np.zeros((v.height, R.P2_COLS), np.uint32)
        t[:len(v.inputs)] = R.poseidon2_rows(v.inputs.astype(np.uint64)).astype(np.uint32)
        t[len(v.inputs):] = R.poseidon2_rows(np.zeros((1, R.WIDTH), np.uint64)).astype(np.uint32)
        return t
    assert isinstance(v, CT.DeviceExpRev)
    t = np.zeros((v.height, 7), np.uint32)
    for e in range(len(v.base)):
        acc = 1
        x = int(v.base[e])
        for r in range(v.offsets[e], v.offsets[e + 1]):
            b = int(v.bits[r])
            mult = x if b == 1 else 1
            psq = acc * acc % R.P
            acc = psq * mult % R.P
            t[r] = [x, b, psq, acc, acc, acc * acc % R.P, mult]
    return t


def test_compact_witness_is_the_full_witness(fib_leaves):
    """node_witness(compact=True): its device work items laid out as the kernels lay them out are the host
    main traces, its Prep carries the host prep traces, and a second node of the same structure from the
    same worker omits them (same prep_key), to be filled in by register_prep."""
    CT._SENT_KEYS.clear()
    full = CT.node_witness(fib_leaves[:2], fix=False)
    comp = CT.node_witness(fib_leaves[:2], fix=False, compact=True)
    assert isinstance(comp[0], CT.Prep) and comp[0].traces is not None
    from tests import _rec_model as RM
    prep = RM.prep_from_records(comp[0].traces)  # the device layout's host model
    assert set(prep) == set(full[0]) and all(np.array_equal(prep[k], full[0][k]) for k in full[0])
    assert set(comp[1]) == set(full[1])
    for k, v in comp[1].items():
        assert np.array_equal(_host_layout(v), full[1][k]), k
    assert np.array_equal(comp[2], full[2]) and comp[3] == full[3]
    # the other two leaves: a different witness, the same program structure -> same key, prep omitted
    other = CT.node_witness(fib_leaves[2:], fix=False, compact=True)
    assert other[0].key == comp[0].key and other[0].traces is None
    assert not np.array_equal(_host_layout(other[1]["MemoryVar"]), _host_layout(comp[1]["MemoryVar"]))
    CT.register_prep(comp)
    assert CT._prep_traces_of(other[0]) is comp[0].traces
    # dedup off: always sent
    assert CT.node_witness(fib_leaves[2:], fix=False, compact=True, dedup=False)[0].traces is not None
    # a new session (another tree / Compress request) gets the traces again, once
    sid = CT.new_session()
    assert CT.node_witness(fib_leaves[2:], fix=False, compact=True, session=sid)[0].traces is not None
    assert CT.node_witness(fib_leaves[:2], fix=False, compact=True, session=sid)[0].traces is None


def test_prep_store_keeps_live_sessions_keys():
    """More than CACHE_ENTRIES programs through the consumer's store across interleaved sessions: a key a live
    session received (its traces sent once per session) survives every eviction until the session ends;
    afterwards it is evicted like any other."""
    CT._PREP_STORE.clear()
    CT._PINS.clear()
    a, b = CT.new_session(), CT.new_session()
    t0 = {"MemoryConst": np.arange(4, dtype=np.uint32)}
    CT.register_prep((CT.Prep(b"k0", t0, a), None))
    for i in range(CT.CACHE_ENTRIES + 10):  # session b: many programs, each sent with its traces
        CT.register_prep((CT.Prep(b"b%d" % i, {"x": np.zeros(1, np.uint32)}, b), None))
        if i % 7 == 0:  # session a's later nodes of k0 arrive in between, traces omitted
            CT.register_prep((CT.Prep(b"k0", None, a), None))
    assert CT._prep_traces_of(CT.Prep(b"k0", None, a)) is t0
    # b's keys are pinned too (b is live): the store grew past the bound instead of dropping them
    assert all(CT._prep_traces_of(CT.Prep(b"b%d" % i, None, b)) is not None for i in range(CT.CACHE_ENTRIES + 10))
    # a Reducer over witnesses of session a releases it when its tree ends
    red = CT.Reducer(lambda ch, fl: _done_future((CT.Prep(b"k0", None, a), ch)), lambda w: ("vk", b"p"),
                     inflight=1, complete=False)
    CT.reduce_serial([("vk", b"l0"), ("vk", b"l1")], red)
    assert a not in CT._PINS and b in CT._PINS
    CT.release_session(b)
    for i in range(CT.CACHE_ENTRIES + 1):
        CT.register_prep((CT.Prep(b"c%d" % i, {"x": np.zeros(1, np.uint32)}, None), None))
    assert b"k0" not in CT._PREP_STORE and len(CT._PREP_STORE) <= CT.CACHE_ENTRIES + 1  # (session None: pinned)
    CT._PREP_STORE.clear()
    CT._PINS.clear()


def _done_future(v):
    f = Future()
    f.set_result(v)
    return f


def test_failed_tree_discards_in_flight_witnesses(tmp_path):
    """A tree whose proving fails drops the witnesses still in flight: their /dev/shm files are unlinked
    when they land, and nothing else is proven."""
    import threading
    from concurrent.futures import Future
    gate = threading.Event()
    files = []

    def submit(ch, flags):
        f = Future()
        f.set_running_or_notify_cancel()  # as an executor's job that has started: cannot be cancelled
        path = tmp_path / f"w{len(files)}"
        path.write_bytes(b"x")
        files.append(path)

        def land():
            if len(files) > 1:
                gate.wait(10)  # the second witness lands after the first proof failed
            f.set_result(CT.Packed(b"", str(path), []))
        threading.Thread(target=land, daemon=True).start()
        return f

    def prove(w):
        raise RuntimeError("device failure")
    red = CT.Reducer(submit, prove, inflight=1, on_witness=lambda w: w)
    with pytest.raises(RuntimeError):
        CT.reduce_serial([("vk", b"a"), ("vk", b"b"), ("vk", b"c"), ("vk", b"d")], red)
    gate.set()
    import time
    for _ in range(100):
        if not files[1].exists():
            break
        time.sleep(0.02)
    assert len(files) == 2 and not files[1].exists()


def test_prep_key_tracks_the_prep_traces(fib_leaves):
    """prep_key follows what the preprocessed traces are made of: a changed constant or shape changes the
    key, a changed hinted (witness) value does not."""
    prog = RV.compress_node_program(fib_leaves[:2])
    rec = R.execute(prog)
    h = {k: max(4, (v - 1).bit_length()) for k, v in R.program_heights(prog).items()}

    def key(p):  # the key of p's instructions (prep_key reads only the flattened program and heights)
        return R.prep_key(R.ExecutionRecord(p, R.flatten(p), rec.ev, rec.public_values), h)
    k0 = R.prep_key(rec, h)
    assert key(prog) == k0
    assert R.prep_key(rec, dict(h, MemoryVar=h["MemoryVar"] + 1)) != k0
    for kind, same in (("mem", False), ("hint", True)):
        p = R._copy_program(prog)
        b = next(b for b in p.blocks if b.kind == kind)
        b.a["vals"][0, 0] = (int(b.a["vals"][0, 0]) + 1) % R.P
        assert (key(p) == k0) == same, kind


def test_vk_by_reference(fib_leaves):
    """by_ref / resolve_vk: one file per distinct key, the same ChildVk back (a fresh process loads it)."""
    vk, proof = fib_leaves[0]
    refs = CT.by_ref(fib_leaves)
    assert len({r.digest for r, _ in refs}) == 1 and refs[0][1] == proof
    assert CT.resolve_vk(refs[0][0]) is vk and CT.resolve_vk(vk) is vk
    import pickle
    with open(refs[0][0].path, "rb") as f:
        again = pickle.loads(f.read())
    assert again.prep_heights == vk.prep_heights and np.array_equal(again.commit, vk.commit)
    assert CT.compress_child_vk(np.arange(8), R.RECURSION_SHAPES[0]) is CT.compress_child_vk(np.arange(8),
                                                                                              R.RECURSION_SHAPES[0])


def test_node_rejects_malformed_child(fib_leaves):
    """Shape checks before the program is built (verifier.rs:248-312): a proof with a dropped query, or
    claimed for a different verifying key, is a ValueError, not a different program."""
    vk, proof = fib_leaves[0]
    import dataclasses
    with pytest.raises(ValueError):
        RV.compress_node_program([(dataclasses.replace(vk, num_queries=NQ + 1), proof)])
    bad_heights = dict(vk.prep_heights)
    bad_heights["FibTable"] *= 2
    with pytest.raises(ValueError):
        RV.compress_node_program([(dataclasses.replace(vk, prep_heights=bad_heights), proof)])


def test_ood_check_binds_the_air(fib_leaves):
    """The out-of-domain check (verifier.rs:316-397): a node whose verifying key describes a different AIR
    (one constraint constant changed) no longer executes on a valid child proof."""
    import dataclasses
    from zkmips_amd import machine as M
    vk, proof = fib_leaves[0]
    R.execute(RV.compress_node_program([(vk, proof)]))
    c = vk.chips["FibCpu"]
    code = list(c.code)
    i = code.index(M.OP_CONST)
    code[i + 1] = (code[i + 1] + 1) % M.P
    vk2 = dataclasses.replace(vk, chips=dict(vk.chips, FibCpu=dataclasses.replace(c, code=tuple(code))))
    with pytest.raises(RuntimeError):
        R.execute(RV.compress_node_program([(vk2, proof)]))
    # and a node built without the check accepts it (the check is what binds the AIR)
    R.execute(RV.compress_node_program([(vk2, proof)], ood=False))


@pytest.mark.gpu
def test_gpu_mips_node_reference_shape():
    """One compress node over the first two shards of a real MIPS execution (the reference's maximal 2^22
    shape scaled to Cpu 2^16, 17 chips, 84 queries, proven on the GPU), with the reference's public-value
    checks (core.rs), its program padded to the first fitting RecursionShapeConfig shape: the GPU proof
    bytes equal the oracle's, and the oracle verifies them."""
    from zkmips_amd import shapes as SH
    from zkmips_amd._lib import Device
    from zkmips_amd.prover import HipProver
    dev = Device(0)
    sh = SH.shape_execution(SH.MAXIMAL_22, 2, down=6)[:2]
    m, prep = sh[0][0], sh[0][1]
    hp = HipProver(dev, m, prep, num_queries=84)
    vk = RV.ChildVk.of(m, prep, hp.vk_commit, num_queries=84)
    leaves = [(vk, hp.prove_shard(s[2], s[3])) for s in sh]
    with pytest.raises(ValueError):  # the shards out of order do not chain
        CT.node_witness(leaves[::-1], is_first=True)
    prep_c, tr, pv, shape, _ = CT.node_witness(leaves, is_first=True)
    assert shape in R.RECURSION_SHAPES
    for k, v in tr.items():
        assert v.shape[0] == 1 << shape[k], k
    cm = R.compress_machine()
    kw = dict(num_queries=R.COMPRESS_NUM_QUERIES, log_blowup=R.COMPRESS_LOG_BLOWUP)
    gpu = HipProver(dev, cm, prep_c, **kw).prove_shard(tr, pv)
    o = O.OracleProver(cm, prep_c, **kw)
    rc, ref = o.prove(tr, pv)
    assert rc == 0 and gpu == ref
    assert o.verify(gpu) == 0
    # the device-P2 form: the Poseidon2WideDeg3 trace built on the device from the permutation inputs
    prep_d, tr_d, pv_d, shape_d, _ = CT.node_witness(leaves, True, True, is_first=True)
    assert isinstance(tr_d["Poseidon2WideDeg3"], CT.DeviceP2) and shape_d == shape
    assert HipProver(dev, cm, prep_d, **kw).prove_shard(CT.materialize(tr_d), pv_d) == gpu
    # the bench's compact form: every main trace laid out on the device from its events, the proving key
    # found by prep_key (GpuProvers)
    wit = CT.node_witness(leaves, True, True, True, False, is_first=True)
    assert all(isinstance(v, (CT.DeviceRows, CT.DeviceExpRev, CT.DeviceP2)) for v in wit[1].values())
    dt = CT.materialize(wit[1])
    for k, v in dt.items():
        assert np.array_equal(v.cpu().numpy().view(np.uint32), tr[k]), k
    pr = CT.GpuProvers(dev).get(wit[0], CT.TreeStats())
    assert pr.prove_shard(dt, wit[2]) == gpu


@pytest.mark.gpu
def test_gpu_mips_node_2e21_leaves():
    """BASELINE config 5 at the reference's default shard size (2^21 Cpu rows, crates/stark/src/opts.rs:6): a
    node over the first two shards of one execution in the maximal shape scaled to Cpu 2^21.  The leaves are
    GPU proofs that the oracle's verifier accepts; the node's program (fix_shape picks its
    RecursionShapeConfig shape) proves to the oracle's bytes on the GPU."""
    from zkmips_amd import shapes as SH
    from zkmips_amd._lib import Device
    from zkmips_amd.prover import HipProver
    dev = Device(0)
    sh = SH.shape_execution(SH.MAXIMAL_22, 2, down=1)[:2]
    m, prep = sh[0][0], sh[0][1]
    assert sh[0][2]["Cpu"].shape[0] == 1 << 21
    hp = HipProver(dev, m, prep, num_queries=84)
    vk = RV.ChildVk.of(m, prep, hp.vk_commit, num_queries=84)
    leaves = [(vk, hp.prove_shard(s[2], s[3])) for s in sh]
    ov = O.OracleProver(m, prep, num_queries=84)
    assert all(ov.verify(p) == 0 for _, p in leaves)
    wit = CT.node_witness(leaves, True, True, True, False, is_first=True)
    print("2^21 leaves: node shape", wit[3], flush=True)
    assert wit[3] in R.RECURSION_SHAPES
    pr = CT.GpuProvers(dev).get(wit[0], CT.TreeStats())
    dt = CT.materialize(wit[1])
    gpu = pr.prove_shard(dt, wit[2])
    prep_c, tr, pv, shape, _ = CT.node_witness(leaves, is_first=True)
    assert shape == wit[3] and np.array_equal(pv, wit[2])
    cm = R.compress_machine()
    o = O.OracleProver(cm, prep_c, num_queries=R.COMPRESS_NUM_QUERIES, log_blowup=R.COMPRESS_LOG_BLOWUP)
    rc, ref = o.prove(tr, pv)
    assert rc == 0 and gpu == ref
    assert o.verify(gpu) == 0


@pytest.fixture(scope="module")
def mips_execution():
    """One MIPS execution in the maximal shape scaled to Cpu 2^10: three consecutive CPU shards and the
    memory shard, oracle-proven with one key (leaves whose public values chain)."""
    from zkmips_amd import shapes as SH
    sh = SH.shape_execution(SH.MAXIMAL_22, 3, down=12)
    m, prep = sh[0][0], sh[0][1]
    pr = O.OracleProver(m, prep, num_queries=NQ)
    proofs = []
    for _, _, tr, pv in sh:
        rc, p = pr.prove(tr, pv)
        assert rc == 0
        proofs.append(p)
    from zkmips_amd.proof import machine_global_sum_is_zero
    assert machine_global_sum_is_zero(proofs)
    return RV.ChildVk.of(m, prep, pr.commit, num_queries=NQ), proofs


def test_core_node_chaining(mips_execution):
    """A node over MIPS shard leaves checks what the reference's core recursion program checks
    (machine/core.rs): consecutive shards in order pass and commit the covered range; reordered, gapped or
    wrongly flagged batches are rejected; the whole execution in one node is complete."""
    from zkmips_amd import node_pv as NP
    vk, proofs = mips_execution
    ok = [([0, 1], True), ([1, 2], False), ([2, 3], False), ([0, 1, 2, 3], True)]
    for order, first in ok:
        complete = len(order) == len(proofs)
        rec = R.execute(RV.compress_node_program([(vk, proofs[i]) for i in order], is_first=first,
                                                 is_complete=complete))
        pv = rec.public_values.astype(np.int64)
        assert pv[NP.R_START_SHARD] == order[0] + 1 and pv[NP.R_NEXT_SHARD] == order[-1] + 2
        assert pv[NP.R_IS_COMPLETE] == int(complete) and pv[NP.R_CONTAINS_EXEC] == int(order[0] < 3)
        assert pv[NP.R_DIGEST:NP.R_DIGEST + 8].tolist() == NP.VT.hash_slice(pv[:NP.R_DIGEST]).tolist()
        assert pv[NP.R_VK_DIGEST:NP.R_VK_DIGEST + 8].tolist() == NP.VT.vk_digest(vk).tolist()
    bad = [([1, 0], True, False), ([0, 2], True, False), ([1, 2], True, False), ([0, 1], False, False),
           ([0, 1], True, True),  # not the whole execution: incomplete
           ([3, 2], False, False)]
    for order, first, complete in bad:
        with pytest.raises(ValueError):
            RV.compress_node_program([(vk, proofs[i]) for i in order], is_first=first, is_complete=complete)


def test_compress_node_chaining(mips_execution):
    """Nodes over node proofs (machine/compress.rs + vkey_proof.rs): two consecutive nodes reduce to a
    complete root whose global sum is the zero digest; the same nodes swapped do not chain; a child node
    vk's Merkle opening in the dummy vk tree is checked."""
    from zkmips_amd import node_pv as NP
    from zkmips_amd import vk_tree as VT
    vk, proofs = mips_execution
    prove = _oracle_prove_factory(4)
    a = prove(CT.node_witness([(vk, p) for p in proofs[:2]], fix=False, is_first=True))
    b = prove(CT.node_witness([(vk, p) for p in proofs[2:]], fix=False))
    rec = R.execute(RV.compress_node_program([a, b], is_complete=True))
    pv = rec.public_values.astype(np.int64)
    assert pv[NP.R_IS_COMPLETE] == 1 and pv[NP.R_START_SHARD] == 1 and pv[NP.R_NEXT_SHARD] == 5
    assert pv[NP.R_GCS:NP.R_GCS + 14].tolist() == NP.SP.CURVE_CUMULATIVE_SUM_START.astype(np.int64).tolist()
    assert pv[NP.R_VK_ROOT:NP.R_VK_ROOT + 8].tolist() == VT.dummy_tree().root.astype(np.int64).tolist()
    with pytest.raises(ValueError):
        RV.compress_node_program([b, a])
    # the template path (node_flat) gives the same program for the same children
    _flat = RV.node_flat([a, b], is_complete=True)
    assert np.array_equal(R.execute(_flat).public_values, rec.public_values)


def test_dummy_vk_tree():
    """The dummy vk map's tree (prover/src/lib.rs:223-233, merkle_tree.rs): 10000 leaves [i; 8] padded to
    2^14; open / verify agree for the first, last and a middle leaf; a wrong sibling fails.  The root itself
    and vk_digest are parity unpinned (the reference holds no vk_root / vk digest value; vk_tree.py)."""
    from zkmips_amd import vk_tree as VT
    t = VT.dummy_tree()
    assert t.height == 14
    for i in (0, 4321, 9999):
        v, path = t.open(i)
        assert np.all(v == i) and VT.MerkleTree.verify(i, v, path, t.root)
        path = path.copy()
        path[3, 0] ^= 1
        assert not VT.MerkleTree.verify(i, v, path, t.root)


@pytest.fixture(scope="module")
def deferred_setup(mips_execution):
    """Execution A's complete compress root (the deferred proof) and execution B, whose guest commits the
    deferred digest of A's root, oracle-proven: B's shard leaves and A's root."""
    from zkmips_amd import mips_core as MC
    from zkmips_amd import node_pv as NP
    prove = _oracle_prove_factory(4)
    vk, proofs = mips_execution
    root_a = prove(CT.node_witness([(vk, p) for p in proofs], fix=False, is_first=True, is_complete=True))
    pv_a = RV.parse_shard_proof(root_a[1]).pv
    assert int(pv_a[NP.R_IS_COMPLETE]) == 1
    d = NP.hash_deferred_proofs(np.zeros(8, np.int64), [pv_a])
    run = MC.program_shards(MC.deferred_commit_program(d), seed=9, shard_size=1 << 10)
    m, prep = run[0][0], run[0][1]
    pr = O.OracleProver(m, prep, num_queries=NQ)
    leaves = []
    vk_b = RV.ChildVk.of(m, prep, pr.commit, num_queries=NQ)
    for _, _, tr, pv in run:
        rc, p = pr.prove(tr, pv)
        assert rc == 0
        leaves.append((vk_b, p))
    assert [int(x) for x in run[-1][3][NP.C_DEFERRED:NP.C_DEFERRED + 8]] == [int(x) for x in d]
    return leaves, root_a, d, prove


def test_deferred_proof_chains_into_a_complete_root(deferred_setup):
    """A Compress request with one deferred proof (prover/src/lib.rs:551-612, machine/deferred.rs): execution B's
    shards reduce to a root that is not complete, A's complete root goes through a deferred node (its vk in the
    vk tree, its digest valid, is_complete 1) that extends the reconstruct-deferred chain from zero, and the two
    reduce to a complete root whose end digest is B's committed deferred_proofs_digest.  Without the deferred
    proof B cannot complete; a deferred node over an incomplete proof, or one starting its chain elsewhere, is
    refused."""
    from zkmips_amd import node_pv as NP
    leaves, root_a, d, prove = deferred_setup
    submit = lambda ch, fl: _done_future(CT.node_witness(ch, fix=False, **fl))
    root = CT.reduce_with_deferred(leaves, [root_a], submit, prove, inflight=1)
    pv = RV.parse_shard_proof(root[1]).pv
    assert int(pv[NP.R_IS_COMPLETE]) == 1 and int(pv[NP.R_CONTAINS_EXEC]) == 1
    assert [int(x) for x in pv[NP.R_END_RECON:NP.R_END_RECON + 8]] == [int(x) for x in d]
    assert not np.any(pv[NP.R_START_RECON:NP.R_START_RECON + 8])
    with pytest.raises(ValueError, match="deferred"):
        CT.node_witness(leaves, fix=False, is_first=True, is_complete=True)
    last = RV.parse_shard_proof(leaves[-1][1]).pv
    h = NP.DeferredHints.of(leaves[0][0], last, np.zeros(8, np.int64))
    w = CT.node_witness([root_a], fix=False, deferred=h)
    assert int(w[2][NP.R_CONTAINS_EXEC]) == 0 and int(w[2][NP.R_START_SHARD]) == int(last[NP.C_SHARD]) + 1
    core = prove(CT.node_witness(leaves, fix=False, is_first=True))
    with pytest.raises(ValueError, match="complete"):
        CT.node_witness([core], fix=False, deferred=h)  # not a complete proof
    bad = NP.DeferredHints.of(leaves[0][0], last, np.ones(8, np.int64))  # a chain that does not start at zero
    dn = prove(CT.node_witness([root_a], fix=False, deferred=bad))
    with pytest.raises(ValueError, match="deferred digest"):
        CT.node_witness([core, dn], fix=False, is_complete=True)


def test_prebuilt_template_serves_later_nodes(fib_leaves):
    """prebuild_template keeps a node structure's program template in the process (as the reference holds its
    recursion programs per shape); a later node of that structure is a template hit whose program executes to
    the full build's public values."""
    RV._TEMPLATES.clear()
    n = CT.prebuild_template(fib_leaves[:2])
    assert n == 1
    flat = RV.node_flat(fib_leaves[2:])
    assert len(RV._TEMPLATES) == 1
    full = R.flatten(RV.compress_node_program(fib_leaves[2:]))
    assert np.array_equal(R.execute(flat).public_values, R.execute(full).public_values)


def test_two_deferred_proofs_chain_in_order(deferred_setup, mips_execution):
    """Two deferred proofs: the second deferred node's chain starts where the first ended (hash_deferred_proofs
    over both), [execution root, deferred 1, deferred 2] reduce to a complete root whose end digest is the
    guest's committed digest of both."""
    from zkmips_amd import mips_core as MC
    from zkmips_amd import node_pv as NP
    _, root_a, d1, prove = deferred_setup
    pv_a = RV.parse_shard_proof(root_a[1]).pv
    d2 = NP.hash_deferred_proofs(np.zeros(8, np.int64), [pv_a, pv_a])
    assert [int(x) for x in NP.hash_deferred_proofs(d1, [pv_a])] == [int(x) for x in d2]
    run = MC.program_shards(MC.deferred_commit_program(d2), seed=9, shard_size=1 << 10)
    m, prep = run[0][0], run[0][1]
    pr = O.OracleProver(m, prep, num_queries=NQ)
    vk_b = RV.ChildVk.of(m, prep, pr.commit, num_queries=NQ)
    leaves = []
    for _, _, tr, pv in run:
        rc, p = pr.prove(tr, pv)
        assert rc == 0
        leaves.append((vk_b, p))
    submit = lambda ch, fl: _done_future(CT.node_witness(ch, fix=False, **fl))
    root = CT.reduce_with_deferred(leaves, [root_a, root_a], submit, prove, inflight=1)
    pv = RV.parse_shard_proof(root[1]).pv
    assert int(pv[NP.R_IS_COMPLETE]) == 1
    assert [int(x) for x in pv[NP.R_END_RECON:NP.R_END_RECON + 8]] == [int(x) for x in d2]
