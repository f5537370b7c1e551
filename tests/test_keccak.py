"""KeccakSponge precompile (zkmips_amd/mips_keccak.py; reference keccak_sponge/{air,trace,columns}.rs and
the executor's keccak/sponge.rs, over Plonky3's p3-keccak-air restated).

Pins: Keccak-f[1600] through hashlib's SHA3-224 (same permutation; the syscall's 144-byte rate is
SHA3-224's), the chip's shape and cost (24 x 4259 = mips_costs.json, tests/test_chip_table.py).  A guest
hashing messages of one, two and three blocks executes into CPU, KECCAK_SPONGE and memory shards whose
traces satisfy every constraint and balance every lookup; the output words are the SHA3-224 digests;
the oracle proves and verifies every shard with the global sum at zero; forged permutation bits,
absorbed state words and output words are rejected.  On the GPU every shard's proof bytes equal the
oracle's."""
import hashlib

import numpy as np
import pytest

from tests import _air_check as AC
from tests import _oracle as O
from zkmips_amd import mips_core as MC
from zkmips_amd import mips_keccak as K
from zkmips_amd.proof import machine_global_sum_is_zero

MSGS = [b"", b"abc", bytes(range(200)), bytes(i * 7 % 256 for i in range(300))]


def _sponge_sha3_224(msg):
    st = np.zeros((1, 25), np.uint64)
    m = K.sha3_pad(msg)
    for b in range(0, len(m), 144):
        st[0, :18] ^= np.frombuffer(m[b:b + 144], "<u8")
        st = K.keccakf(st)
    return st[0].astype("<u8").tobytes()[:28]


@pytest.mark.parametrize("n", [0, 1, 135, 143, 144, 145, 287, 288, 1000])
def test_keccakf_pinned_to_sha3(n):
    msg = bytes((i * 31 + 7) % 256 for i in range(n))
    assert _sponge_sha3_224(msg) == hashlib.sha3_224(msg).digest()


def test_rows_follow_the_rounds():
    """Row r of a permutation holds round r's input in `a` and the next row's `a` is this row's a'''."""
    inp = np.random.default_rng(3).integers(0, 2**63, (2, 25), dtype=np.uint64)
    t = K.keccak_rows(inp)
    for p in range(2):
        a = inp[p:p + 1].copy()
        for r in range(K.NUM_ROUNDS):
            row = t[24 * p + r]
            assert row[K.K_STEP + r] == 1 and row[K.K_STEP:K.K_STEP + 24].sum() == 1
            assert np.array_equal(row[K.K_A:K.K_A + 100], K._limb_cols(a)[0])
            a = K._round(a, r)[-1]
        assert np.array_equal(a, K.keccakf(inp[p:p + 1]))


@pytest.fixture(scope="module")
def run():
    return MC.program_shards(K.keccak_program(MSGS), seed=1, shard_size=2000, precompile_events_per_shard=2)


def test_sponge_outputs_are_sha3_224(run):
    ks = [tr for _, _, tr, _ in run if "KeccakSponge" in tr]
    assert len(ks) == 2  # 4 calls, 2 per precompile shard
    state = MC.fresh_state()
    prog = K.keccak_program(MSGS)
    # re-execute to read the output words back from the events
    evs = []
    regs = MC.initial_registers(1)
    while MC.PC_BASE <= state["pc"] < MC.PC_BASE + 4 * len(prog) and state["exit_code"] is None:
        MC.program_shard(prog, 1, len(evs) + 1, 2000, state=state, regs=regs)
        evs.append(1)
    calls = [e for code, _, e in state["precompile"] if code == K.KECCAK_SPONGE]
    assert len(calls) == len(MSGS)
    for msg, e in zip(MSGS, calls):
        out = np.asarray(e["out"], "<u4").tobytes()
        assert out[:28] == hashlib.sha3_224(msg).digest()


def test_execution_satisfies_air(run):
    for m, prep, tr, pv in run:
        bad, unb = AC.check(m, {k: v for k, v in prep.items() if v is not None}, tr, pv)
        assert not bad and not unb, sorted(tr)


@pytest.mark.parametrize("col", [K._ap(2, 3, 17), K.ORIG + 4 * 30 + 1, K.OUT_MEM + 4 + 2, K.K_APPP00 + 1, K._c(4, 63)])
def test_forged_cell_is_rejected(run, col):
    m, prep, tr, pv = next(r for r in run if "KeccakSponge" in r[2])
    t = tr["KeccakSponge"].copy()
    rows = {K.OUT_MEM + 4 + 2: np.nonzero(t[:, K.WRITE_OUT])[0][0], K.ORIG + 4 * 30 + 1: 24}
    r = rows.get(col, 30)
    t[r, col] = (int(t[r, col]) + 1) % K.P
    bad, unb = AC.check(m, {k: v for k, v in prep.items() if v is not None}, dict(tr, KeccakSponge=t), pv)
    assert bad or unb


def test_oracle_proves_execution(run):
    m, prep, _, _ = run[0]
    pr = O.OracleProver(m, {k: v for k, v in prep.items() if v is not None}, num_queries=4)
    proofs = []
    for _, _, tr, pv in run:
        rc, p = pr.prove(tr, pv)
        assert rc == 0 and pr.verify(p) == 0, sorted(tr)
        proofs.append(p)
    assert machine_global_sum_is_zero(proofs)


@pytest.mark.gpu
def test_gpu_keccak_execution_bytes_identical(run):
    """Every shard (the KeccakSponge shards among them) proves on the GPU to the oracle's bytes."""
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
        assert rc == 0 and p == ref, sorted(tr)
        proofs.append(p)
    assert machine_global_sum_is_zero(proofs)
