"""BASELINE config 4 on the reference's own data (zkmips_amd/tendermint.py): the light-client check of
examples/tendermint (guest/src/main.rs:34-65) over examples/tendermint/host/files/block_2279100.json ->
block_2279130.json (copied to tests/golden/tendermint/).

The fixtures pin the host-side encodings: each header's Merkle hash is its commit's block_id.hash, each
validator set hashes to the value its header carries, and every vote signature verifies over the
canonical-vote sign bytes.  The guest performs the same computation in MIPS (SHA-256 precompiles,
SHA-512 in software, ED_DECOMPRESS / ED_ADD, UINT256_MUL) and halts with exit code 0 only if every check
holds; on the GPU every shard of its execution proves byte-identically to the oracle and the shards'
global cumulative sums add to zero."""
import hashlib

import numpy as np
import pytest

from zkmips_amd import mips_core as MC
from zkmips_amd import tendermint as T


@pytest.fixture(scope="module")
def blocks():
    return T.load_block(2279100), T.load_block(2279130)


def test_header_hashes_are_the_block_ids(blocks):
    for b in blocks:
        assert T.header_hash(b).hex().upper() == b["signed_header"]["commit"]["block_id"]["hash"]


def test_validator_set_hashes(blocks):
    b1, b2 = blocks
    assert T.validators_hash(b1["next_validator_set"]).hex().upper() == b1["signed_header"]["header"]["next_validators_hash"]
    assert T.validators_hash(b2["validator_set"]).hex().upper() == b2["signed_header"]["header"]["validators_hash"]
    assert T.validators_hash(b2["next_validator_set"]).hex().upper() == b2["signed_header"]["header"]["next_validators_hash"]


def test_vote_signatures_verify(blocks):
    votes = T.signed_votes(blocks[1])
    assert len(votes) == 100 and sum(v["commit"] for v in votes) == 99  # 99 commits, 1 nil vote
    for v in votes[:8] + votes[-2:]:  # the nil vote is last
        assert T.ed25519_verify(v["pub"], v["msg"], v["sig"])
    bad = bytearray(votes[0]["msg"])
    bad[20] ^= 1
    assert not T.ed25519_verify(votes[0]["pub"], bytes(bad), votes[0]["sig"])


def _run(prog):
    state = MC.fresh_state()
    MC._execute(prog, MC.initial_registers(1), 1, 1 << 24, state=state)
    return state


def test_sha512_in_mips():
    for n in (0, 111, 112, 174, 300):
        msg = bytes((7 * i + n) & 0xFF for i in range(n))
        a = T.Asm(MC.DATA_BASE)
        sha = T.Sha512(a)
        words = T._sha512_padded_words(msg)
        mp = a.alloc(len(words), 8)
        a.store_words(mp, words)
        sha.hash(mp, len(words) // 32)
        mem = _run(a.program())["mem"]
        got = b"".join(mem[sha.h_ptr + 4 * i].to_bytes(4, "big") for i in range(16))
        assert got == hashlib.sha512(msg).digest(), n


def test_guest_subset_and_tamper(blocks):
    """Three votes verified in the guest (headers and validator sets too): exit code 0; one signature bit
    flipped: nonzero exit code."""
    prog, exp = T.tendermint_program(*blocks, votes=slice(97, 100))
    st = _run(prog)
    assert st["exit_code"] == 0
    prog, _ = T.tendermint_program(*blocks, votes=slice(97, 100), tamper=1)
    assert _run(prog)["exit_code"] != 0


@pytest.fixture(scope="module")
def tm_proofs():
    """The whole execution (100 votes; exit code 0 and the committed public-values digest equal the host's,
    checked by tendermint_shards), every shard proven on the GPU."""
    from zkmips_amd._lib import Device
    from zkmips_amd.prover import HipProver
    shards, info = T.tendermint_shards()
    assert info["exit_code"] == 0 and info["pv_digest"] == hashlib.sha256(info["public_values"]).digest()
    m, prep = shards[0][0], {k: v for k, v in shards[0][1].items() if v is not None}
    hp = HipProver(Device(0), m, prep, num_queries=84)
    return shards, prep, [hp.prove_shard(tr, pv) for _, _, tr, pv in shards]


@pytest.mark.gpu
def test_gpu_tendermint_global_sum(tm_proofs):
    """The shards' global cumulative sums add to zero (machine.rs:639-654)."""
    from zkmips_amd.proof import machine_global_sum_is_zero
    shards, _, proofs = tm_proofs
    assert len(proofs) == len(shards) >= 8
    assert machine_global_sum_is_zero(proofs)


@pytest.mark.gpu
@pytest.mark.parametrize("part", [0, 1, 2])
def test_gpu_tendermint_bytes(tm_proofs, part):
    """Every shard's GPU proof bytes equal the oracle's (the shards in three groups, one test each)."""
    from tests import _oracle as O
    shards, prep, proofs = tm_proofs
    o = O.OracleProver(shards[0][0], prep, num_queries=84)
    for i in range(part, len(shards), 3):
        _, _, tr, pv = shards[i]
        rc, ref = o.prove(tr, pv)
        assert rc == 0 and ref == proofs[i], f"shard {i}"


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _two_rank_worker(rank, world, port, out_q):
    import os
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tests import _oracle as O
    from zkmips_amd.dist import deal_by_cost, prove_shards_distributed, shard_cost
    prog, _ = T.tendermint_program(T.load_block(2279100), T.load_block(2279130), votes=slice(99, 100))
    run = MC.program_shards(prog, seed=1, shard_size=1 << 16, precompile_events_per_shard=512)
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
        out_q.put((len(proofs), len(run), sorted(set(k for _, _, tr, _ in run for k in tr))))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_tendermint_execution():
    """A tendermint execution on the reference's blocks (headers and validator sets hashed, the nil vote's
    signature verified) split into CPU, SHA_EXTEND, SHA_COMPRESS, ED_ADD, ED_DECOMPRESS, UINT256_MUL and
    memory shards, dealt by cost to two gloo ranks; rank 0 gathers every proof and the machine-level global
    cumulative sum checks out (machine.rs:639-654)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_two_rank_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = q.get(timeout=900)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert got[0] == got[1] >= 7
    assert {"ShaExtend", "ShaCompress", "EdAddAssign", "EdDecompress", "Uint256MulMod"} <= set(got[2])
