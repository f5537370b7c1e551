"""Ed25519 precompiles (EdAddAssign, EdDecompress; zkmips_amd/mips_edwards.py) and a tendermint-shaped
execution (BASELINE config 4: signature verifications through the precompiles + SHA-256 blocks).

Pins: the curve arithmetic reproduces the RFC 8032 Ed25519 test vector 1 (public key and signature,
an external published vector); chip shapes and costs equal mips_costs.json (tests/test_chip_table.py);
decompression inverts compression; the traces satisfy every constraint and balance every lookup; the
oracle proves and verifies every shard with the machine-level global sum at zero; tampering is rejected.
On the GPU every shard's proof bytes equal the oracle's."""
import os
import socket

import numpy as np
import pytest

from tests import _air_check as AC
from tests import _oracle as O
from zkmips_amd import mips_core as MC
from zkmips_amd import mips_edwards as ED
from zkmips_amd.proof import machine_global_sum_is_zero


def test_rfc8032_vector_1():
    sk = bytes.fromhex("9d61b19deffd5a60ba844af492ec2cc44449c5697b326919703bac031cae7f60")
    A, R, S, k = ED.ed25519_keypair_sign(sk, b"")
    assert ED._encode(A).hex() == "d75a980182b10ab7d54bfed3c964073a0ee172f3daa62325af021a68f707511a"
    sig = ED._encode(R) + S.to_bytes(32, "little")
    assert sig.hex() == ("e5564300c360ac729086e2cc806e828a84877f1eb8e5d974d873e065224901555fb8821590a33bacc61e3970"
                         "1cf9b46bd25bf5f0595bbe24655141438e7a100b")
    B = (ED.BASE_X, ED.BASE_Y)
    assert ED._scalar_mul(S, B) == ED.ed_add_points(R, ED._scalar_mul(k, A))


def test_decompress_inverts_compress():
    rng = np.random.default_rng(2)
    pt = (ED.BASE_X, ED.BASE_Y)
    for _ in range(8):
        pt = ED._scalar_mul(int(rng.integers(1, 1 << 62)), pt)
        assert ED.ed_decompress_point(pt[1], pt[0] & 1) == pt
        assert ED.ed25519_sqrt(pt[0] * pt[0] % ED.ED_P) % 2 == 0


@pytest.fixture(scope="module")
def run():
    return MC.program_shards(ED.ed25519_program(1, seed=3, scalar_bits=6), seed=1, shard_size=400,
                             precompile_events_per_shard=64)


def test_execution_satisfies_air(run):
    kinds = [sorted(k for k in tr if k.startswith("Ed")) for _, _, tr, _ in run]
    assert ["EdAddAssign"] in kinds and ["EdDecompress"] in kinds
    for m, prep, tr, pv in run:
        bad, unb = AC.check(m, {k: v for k, v in prep.items() if v is not None}, tr, pv)
        assert not bad and not unb


def test_tampered_result_is_rejected(run):
    m, prep, tr, pv = next(r for r in run if "EdAddAssign" in r[2])
    bad_tr = dict(tr)
    t = tr["EdAddAssign"].copy()
    t[0, ED.EA_X3] = (int(t[0, ED.EA_X3]) + 1) % ED.P  # x3 limb 0 of the first addition
    bad_tr["EdAddAssign"] = t
    bad, _ = AC.check(m, {k: v for k, v in prep.items() if v is not None}, bad_tr, pv)
    assert bad
    pr = O.OracleProver(m, {k: v for k, v in prep.items() if v is not None}, num_queries=4)
    rc, proof = pr.prove(bad_tr, pv)
    assert rc != 0 or pr.verify(proof) != 0  # refused, or the proof of an unsatisfied trace fails to verify


def test_oracle_proves_execution(run):
    m, prep, _, _ = run[0]
    pr = O.OracleProver(m, {k: v for k, v in prep.items() if v is not None}, num_queries=4)
    proofs = []
    for _, _, tr, pv in run:
        rc, p = pr.prove(tr, pv)
        assert rc == 0 and pr.verify(p) == 0
        proofs.append(p)
    assert machine_global_sum_is_zero(proofs)
    assert not machine_global_sum_is_zero(proofs[:-1])  # a dropped shard breaks the sum


def test_full_verification_guest_checks():
    """With full 253-bit scalars the guest's check [S]B == R + [k]A holds: its accumulator commits 0."""
    prog = ED.ed25519_program(1, seed=5)
    regs = MC.initial_registers(5)
    st = MC.fresh_state()
    MC._execute(prog, regs, 1, 1 << 22, st)
    assert st["exit_code"] == 0
    assert regs[10] == 0
    n_add = sum(1 for e in st["precompile"] if e[0] == ED.ED_ADD)
    assert n_add > 500


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _two_rank_worker(rank, world, port, out_q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from zkmips_amd.dist import deal_by_cost, prove_shards_distributed, shard_cost
    run = MC.program_shards(ED.ed25519_program(1, seed=3, scalar_bits=6), seed=1, shard_size=400,
                            precompile_events_per_shard=64)
    m, prep, _, _ = run[0]
    pr = O.OracleProver(m, {k: v for k, v in prep.items() if v is not None}, num_queries=4)
    costs = [shard_cost(tr) for _, _, tr, _ in run]
    mine = deal_by_cost(costs, world)[rank]

    def prove_one(i):
        assert i in mine
        rc, p = pr.prove(run[i][2], run[i][3])
        assert rc == 0
        return p
    proofs = prove_shards_distributed(prove_one, len(run), check_global_sum=True, costs=costs)
    if rank == 0:
        out_q.put((len(proofs), len(run)))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_ed25519_execution():
    """The execution's CPU, EdAddAssign, EdDecompress and memory shards dealt (by cost) to two gloo ranks;
    rank 0 gathers them and the machine-level global sum checks out."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_two_rank_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = q.get(timeout=600)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert got[0] == got[1] >= 4


@pytest.mark.gpu
def test_gpu_ed25519_execution_bytes_identical(run):
    """Every shard of the ed25519 execution proves on the GPU to the oracle's bytes; the global sum is
    zero over the GPU proofs."""
    from zkmips_amd._lib import Device
    from zkmips_amd.prover import HipProver
    m, prep, _, _ = run[0]
    prep = {k: v for k, v in prep.items() if v is not None}
    gpu = HipProver(Device(0), m, prep, num_queries=16)
    cpu = O.OracleProver(m, prep, num_queries=16)
    proofs = []
    for _, _, tr, pv in run:
        p = gpu.prove_shard(tr, pv)
        rc, ref = cpu.prove(tr, pv)
        assert rc == 0 and p == ref
        proofs.append(p)
    assert machine_global_sum_is_zero(proofs)
