"""The memory argument across shards: MemoryLocal, Global (septic-curve digests), MemoryGlobalInit /
MemoryGlobalFinalize, a continuation execution split into shards, and the machine-level check that the
shards' global cumulative sums add up to the zero digest (crates/stark/src/machine.rs:639-654)."""
import os
import socket

import numpy as np
import pytest

from tests import _air_check
from tests import _oracle as O
from zkmips_amd import mips_core as C
from zkmips_amd import mips_memory as MM
from zkmips_amd import septic as S
from zkmips_amd.proof import machine_global_sum_is_zero, shard_global_cumulative_sum

# SepticExtension::z_pow_p(1), z_pow_p(2) (crates/stark/src/septic_extension.rs:430-449)
Z_POW_P1 = [587483156, 843070426, 856916903, 802055410, 1274370027, 839777993, 1763169463]
Z_POW_P2 = [1211185764, 536911287, 1786731555, 1891857573, 591969516, 550155966, 706525029]


def test_septic_field_and_curve_constants():
    """The trace helper's Frobenius equals the reference's constants; the reference's three fixed points
    (septic_digest.rs test_const_points) are on the curve."""
    assert list(S.frobenius_col(1)) == Z_POW_P1 and list(S.frobenius_col(2)) == Z_POW_P2
    for pt in (S.CURVE_CUMULATIVE_SUM_START, S.DIGEST_SUM_START, S.CURVE_WITNESS_DUMMY_POINT):
        assert S.on_curve(pt)


def test_lift_is_normalised():
    """lift_x (septic_curve.rs:130-154) + get_digest (global_lookup.rs:26-38): x = message (+ kind << 16,
    last coefficient * 256 + offset), y on the curve with y_6 in [1, (p-1)/2] for receives, negated for
    sends."""
    rng = np.random.default_rng(5)
    msg = rng.integers(0, 1 << 16, (200, 7), dtype=np.uint32)
    rec = (np.arange(200) % 2).astype(np.uint8)
    kinds = np.full(200, 1, np.uint32)
    xy, off = S.lift(msg, kinds, rec)
    half = (MM.P - 1) // 2
    for k in range(200):
        assert S.on_curve(xy[k]) and off[k] < 256
        assert list(xy[k, 1:6]) == list(msg[k, 1:6]) and xy[k, 0] == (msg[k, 0] + (1 << 16)) % MM.P
        assert xy[k, 6] == (int(msg[k, 6]) * 256 + int(off[k])) % MM.P
        y6 = int(xy[k, 13])
        assert (1 <= y6 <= half) if rec[k] else (half < y6)


@pytest.fixture(scope="module")
def run():
    return C.program_shards(C.loop_program(20, 60, seed=5), seed=5, shard_size=400)


def test_continuation_shards_satisfy_air(run):
    """7 CPU shards and the memory shard: every constraint holds, every local lookup balances; the state
    carries across shards (each shard's first pc is the previous shard's next pc)."""
    assert len(run) == 8
    for m, prep, tr, pv in run:
        assert _air_check.check(m, {k: v for k, v in prep.items() if v is not None}, tr, pv) == ([], [])
    for (_, _, _, a), (_, _, _, b) in zip(run[:-2], run[1:-1]):
        assert a[C.PV_NEXT_PC] == b[C.PV_START_PC]
    assert set(run[-1][2]) == {"MemoryGlobalInit", "MemoryGlobalFinalize", "Global", "Byte", "Program"}


def test_global_sum_over_shards_is_zero(run):
    digs = np.asarray([C.shard_global_digest(tr) for _, _, tr, _ in run])
    assert np.array_equal(S.digest_sum(digs), S.CURVE_CUMULATIVE_SUM_START)
    assert not np.array_equal(S.digest_sum(digs[:-1]), S.CURVE_CUMULATIVE_SUM_START)  # without the memory shard


def test_global_sum_from_proofs(run):
    """Proved by the oracle: the global cumulative sums read back from the proof bytes add up to zero,
    and a shard missing from the MachineProof breaks the sum."""
    m, prep, _, _ = run[0]
    pr = O.OracleProver(m, {k: v for k, v in prep.items() if v is not None}, num_queries=4)
    proofs = []
    for _, _, tr, pv in run:
        rc, p = pr.prove(tr, pv)
        assert rc == 0 and pr.verify(p) == 0
        assert np.array_equal(shard_global_cumulative_sum(p), S.digest_sum([C.shard_global_digest(tr)]))
        proofs.append(p)
    assert machine_global_sum_is_zero(proofs)
    assert not machine_global_sum_is_zero(proofs[:3] + proofs[4:])


@pytest.mark.parametrize("what", ["addr_order", "init_timestamp", "final_value", "last_addr_pv"])
def test_memory_shard_tamper_rejected(run, what):
    m, prep, tr, pv = run[-1]
    bad = {k: v.copy() for k, v in tr.items()}
    pv = pv.copy()
    if what == "addr_order":  # two initialised addresses swapped: no longer increasing
        t = bad["MemoryGlobalInit"]
        t[[2, 3]] = t[[3, 2]]
    elif what == "init_timestamp":
        bad["MemoryGlobalInit"][1, MM.MG_TS] = 2
    elif what == "final_value":
        bad["MemoryGlobalFinalize"][3, MM.MG_VALUE] ^= 1
    else:
        pv[MM.PV_LAST_FIN_BITS] ^= 1
    prep = {k: v for k, v in prep.items() if v is not None}
    assert _air_check.check(m, prep, bad, pv) != ([], [])
    pr = O.OracleProver(m, prep, num_queries=4)
    rc, p = pr.prove(bad, pv)
    assert pr.verify(p) != 0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_q, drop):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from zkmips_amd.dist import prove_shards_distributed
    run = C.program_shards(C.loop_program(12, 30, seed=2), seed=2, shard_size=200)
    if drop:
        run = run[1:]
    m, prep, _, _ = run[-1]
    pr = O.OracleProver(m, {k: v for k, v in prep.items() if v is not None}, num_queries=4)

    def prove_one(i):
        rc, p = pr.prove(run[i][2], run[i][3])
        assert rc == 0
        return p

    try:
        proofs = prove_shards_distributed(prove_one, len(run), check_global_sum=True)
        res = ("ok", len(proofs))
    except ValueError:
        res = ("nonzero", 0)
    if rank == 0:
        out_q.put(res)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("drop", [False, True])
def test_two_rank_multishard_global_sum(drop):
    """Shards of one execution dealt to 2 gloo ranks, proofs gathered to rank 0, which checks the
    global cumulative sum; dropping a shard makes rank 0 reject the MachineProof."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, drop)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=600)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert got[0] == ("nonzero" if drop else "ok")


@pytest.mark.gpu
def test_continuation_gpu_proofs_identical(run):
    """Every shard of the continuation (CPU shards with MemoryLocal/Global, the memory shard with
    MemoryGlobalInit/Finalize) proves on the GPU byte-identical to the oracle, and the GPU proofs'
    global cumulative sums add up to zero."""
    from zkmips_amd._lib import Device
    from zkmips_amd.prover import HipProver
    m, prep, _, _ = run[0]
    prep = {k: v for k, v in prep.items() if v is not None}
    dev = Device(0)
    gpu = HipProver(dev, m, prep, num_queries=16)
    cpu = O.OracleProver(m, prep, num_queries=16)
    proofs = []
    for _, _, tr, pv in run:
        p = gpu.prove_shard(tr, pv)
        rc, ref = cpu.prove(tr, pv)
        assert rc == 0 and p == ref
        proofs.append(p)
    assert machine_global_sum_is_zero(proofs)
