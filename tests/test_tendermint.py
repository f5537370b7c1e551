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
