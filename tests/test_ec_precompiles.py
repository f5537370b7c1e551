"""Weierstrass-curve, field-tower and Uint256MulMod precompiles (zkmips_amd/mips_ec.py on the shared
emulated-field gadgets of zkmips_amd/emulated_field.py).

Pins: every base field's modulus, witness offset, limb / witness sizes and the curves' a / b equal the
reference's FieldParameters / WeierstrassParameters (tests/golden/curve_params.json, extracted by
tests/golden/make_ref_fixtures.py); chip shapes and costs equal mips_costs.json
(tests/test_chip_table.py); the affine formulas agree with an independent projective check (the
results lie on the curve and P + Q - Q = P).  A guest calling every syscall (Poseidon2Permute included) executes into CPU,
precompile and memory shards whose traces satisfy every constraint and balance every lookup; the
oracle proves and verifies every shard with the machine-level global sum at zero; forged results are
rejected.  On the GPU every shard's proof bytes equal the oracle's."""
import json
import os

import numpy as np
import pytest

from tests import _air_check as AC
from tests import _oracle as O
from zkmips_amd import emulated_field as EF
from zkmips_amd import mips_core as MC
from zkmips_amd import mips_ec as EC
from zkmips_amd.proof import machine_global_sum_is_zero

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _le(words, bits=32):
    return sum(int(w) << (bits * i) for i, w in enumerate(words))


def test_field_params_equal_reference():
    ref = json.load(open(os.path.join(GOLDEN, "curve_params.json")))
    for name, fp in list(EC.FIELDS.items()) + [("U256", EC.U256)]:
        r = ref[name]
        assert _le(r["modulus_le"], 8) == fp.modulus, name
        assert (r["limbs"], r["witness"], 1 << r["witness_offset_log2"]) == (fp.nl, fp.nwit, fp.offset), name
        if name != "U256":
            assert _le(r.get("a_int_u32_le", [0])) == EC.CURVE_A[name], name
            assert _le(r["b_int_u32_le"]) == EC.CURVE_B[name], name
        if name in EC.GEN_X:
            gx, gy = (int(v) for v in r["generator"])
            assert gx == EC.GEN_X[name], name
            assert EC.point_from_x(name, gx)[1] in (gy, fp.modulus - gy), name


@pytest.mark.parametrize("curve", sorted(EC.FIELDS))
def test_curve_arithmetic(curve):
    rng = np.random.default_rng(5)
    m, a, b = EC.FIELDS[curve].modulus, EC.CURVE_A[curve], EC.CURVE_B[curve]
    on = lambda pt: (pt[1] * pt[1] - pt[0] ** 3 - a * pt[0] - b) % m == 0  # noqa: E731
    p, q = EC.random_point(curve, rng), EC.random_point(curve, rng)
    s, d = EC.sw_add(curve, p, q), EC.sw_double(curve, p)
    assert on(p) and on(q) and on(s) and on(d)
    assert EC.sw_add(curve, s, (q[0], (m - q[1]) % m)) == p  # (P + Q) - Q
    assert EC.sw_add(curve, d, (p[0], (m - p[1]) % m)) == p  # 2P - P


@pytest.mark.parametrize("curve", sorted(EC.EC_DECOMPRESS))
def test_decompress_sign_rule(curve):
    rng = np.random.default_rng(7)
    m = EC.FIELDS[curve].modulus
    for _ in range(4):
        x, y = EC.random_point(curve, rng)
        for sign in (0, 1):
            yy = EC.decompress_y(curve, x, sign)
            assert yy in (y, m - y)
            if EC.LEXICOGRAPHIC[curve]:
                assert (yy > m - yy) == bool(sign)
            else:
                assert yy & 1 == sign


@pytest.fixture(scope="module")
def run():
    return MC.program_shards(EC.ec_program(1, reps=2), seed=1, shard_size=2000, precompile_events_per_shard=64)


def test_every_precompile_chip_gets_a_shard(run):
    names = {k for _, _, tr, _ in run for k in tr}
    for ch in EC.chips_in_machine_order():
        if ch.name == "KeccakSponge":  # its own guest: tests/test_keccak.py
            continue
        assert ch.name in names, ch.name


def test_execution_satisfies_air(run):
    for m, prep, tr, pv in run:
        bad, unb = AC.check(m, {k: v for k, v in prep.items() if v is not None}, tr, pv)
        assert not bad and not unb, sorted(tr)


@pytest.mark.parametrize("chip,col", [("Secp256k1AddAssign", lambda: EC.AddLayout(EC.FIELDS["Secp256k1"]).F["x3_ins"]),
                                      ("Bls12381DoubleAssign",
                                       lambda: EC.DoubleLayout(EC.FIELDS["Bls12381"]).F["y3_ins"]),
                                      ("Bn254Fp2MulAssign", lambda: EC.Fp2MulLayout(EC.FIELDS["Bn254"]).F["c1"]),
                                      ("Uint256MulMod", lambda: EC.U256L.OUT),
                                      ("U256XU2048Mul", lambda: EC.U2048L.OUT[3]),
                                      ("Bls12381Decompress",
                                       lambda: EC.DecompressLayout(EC.FIELDS["Bls12381"], True).SQRT),
                                      ("Secp256k1Decompress",
                                       lambda: EC.DecompressLayout(EC.FIELDS["Secp256k1"], False).NEGY)])
def test_forged_result_is_rejected(run, chip, col):
    m, prep, tr, pv = next(r for r in run if chip in r[2])
    bad_tr = dict(tr)
    t = tr[chip].copy()
    c = col()
    t[0, c] = (int(t[0, c]) + 1) % EC.P
    bad_tr[chip] = t
    bad, _ = AC.check(m, {k: v for k, v in prep.items() if v is not None}, bad_tr, pv)
    assert bad


def test_uint256_zero_modulus_is_2_256(run):
    """Modulus 0 means 2^256 (no range check); a nonzero modulus range-checks the result below it."""
    m, prep, tr, pv = next(r for r in run if "Uint256MulMod" in r[2])
    t = tr["Uint256MulMod"]
    L = EC.U256L
    real = t[:, L.REAL] == 1
    assert set(t[real, L.IZ_RES].tolist()) == {0, 1}
    assert np.all(t[real, L.NOT_ZERO] == 1 - t[real, L.IZ_RES])


def test_oracle_proves_execution(run):
    m, prep, _, _ = run[0]
    pr = O.OracleProver(m, {k: v for k, v in prep.items() if v is not None}, num_queries=4)
    proofs = []
    for _, _, tr, pv in run:
        rc, p = pr.prove(tr, pv)
        assert rc == 0 and pr.verify(p) == 0, sorted(tr)
        proofs.append(p)
    assert machine_global_sum_is_zero(proofs)
    assert not machine_global_sum_is_zero(proofs[:-1])


@pytest.mark.gpu
def test_gpu_ec_execution_bytes_identical(run):
    """Every shard (the 15 precompile chips' shards among them) proves on the GPU to the oracle's bytes;
    the global sum is zero over the GPU proofs."""
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


def test_emulated_field_witness_roundtrip():
    """The witness of a random product satisfies vanishing(x) = w(x) (x - 256) for every field here."""
    rng = np.random.default_rng(3)
    for fp in list(EC.FIELDS.values()) + [EC.U256]:
        a = [int.from_bytes(rng.bytes(fp.nl), "little") % fp.modulus for _ in range(4)]
        b = [int.from_bytes(rng.bytes(fp.nl), "little") % fp.modulus for _ in range(4)]
        r, cols = EF.pop_field_op(a, b, "mul", fp)
        assert r == [x * y % fp.modulus for x, y in zip(a, b)]
        assert cols.shape == (4, fp.fop_w) and cols.min() >= 0 and cols.max() < 256


def test_poseidon2_permute_matches_kat():
    """POSEIDON2_PERMUTE computes the pinned Poseidon2-16 permutation (tests/golden/poseidon2_kat.json)."""
    from zkmips_amd import mips_p2permute as P2
    kat = json.load(open(os.path.join(GOLDEN, "poseidon2_kat.json")))
    for v in kat.values():
        assert P2.permute([int(x) for x in v["input"]]) == [int(x) for x in v["output"]]
