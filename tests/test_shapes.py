"""A MIPS core shard in a reference 2^22 maximal shape (maximal_shapes.json["22"][2]): every chip padded to
the shape's height, at reduced scale on the CPU, byte parity on the GPU at Cpu 2^18, and the full-size
shard proved on the GPU and accepted by the oracle verifier."""
import json
import os

import numpy as np
import pytest

from tests import _air_check
from tests import _oracle as O
from zkmips_amd import shapes as SH

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_maximal_shape_is_the_reference_entry():
    shapes = json.load(open(os.path.join(GOLDEN, "maximal_shapes_22.json")))
    assert shapes[2] == SH.MAXIMAL_22


@pytest.fixture(scope="module")
def small():
    return SH.shape_shard(SH.MAXIMAL_22, seed=3, down=6)


def test_shape_shard_heights_and_air(small):
    m, prep, tr, pv = small
    want = SH.scaled(SH.MAXIMAL_22, 6)
    assert {k: int(np.log2(len(tr[k]))) for k in want} == want
    assert set(tr) - set(want) == {"Program", "Byte"}
    # the chips are mostly full, not padding
    for chip, col in (("Cpu", 65), ("AddSub", None)):
        if col is not None:
            assert tr[chip][:, col].sum() > 0.6 * len(tr[chip])
    assert _air_check.check(m, {k: v for k, v in prep.items() if v is not None}, tr, pv) == ([], [])


def test_shape_shard_oracle_proof_verifies(small):
    m, prep, tr, pv = small
    pr = O.OracleProver(m, prep, num_queries=8)
    rc, p = pr.prove(tr, pv)
    assert rc == 0 and pr.verify(p) == 0


def test_too_many_events_rejected():
    with pytest.raises(ValueError):
        SH.pad_to_shape(SH.shape_shard(SH.MAXIMAL_22, seed=3, down=6)[0],
                        {"Cpu": np.zeros((1 << 17, 67), np.uint32)}, SH.scaled(SH.MAXIMAL_22, 6))


@pytest.mark.gpu
def test_shape_shard_gpu_proof_bytes_identical():
    from zkmips_amd._lib import Device
    from zkmips_amd.prover import HipProver
    m, prep, tr, pv = SH.shape_shard(SH.MAXIMAL_22, seed=4, down=4)
    gpu = HipProver(Device(0), m, prep, num_queries=84)
    cpu = O.OracleProver(m, prep, num_queries=84)
    p = gpu.prove_shard(tr, pv)
    rc, ref = cpu.prove(tr, pv)
    assert rc == 0 and p == ref


@pytest.mark.gpu
def test_shape_shard_full_size_gpu_proof_verifies():
    """The full maximal 2^22 shape: GPU proof bytes == the oracle's, accepted; a tampered trace is rejected."""
    from zkmips_amd._lib import Device
    from zkmips_amd.prover import HipProver
    m, prep, tr, pv = SH.shape_shard(SH.MAXIMAL_22, seed=5, down=0)
    assert len(tr["Cpu"]) == 1 << 22 and len(tr["AddSub"]) == 1 << 21
    gpu = HipProver(Device(0), m, prep, num_queries=84)
    p = gpu.prove_shard(tr, pv)
    cpu = O.OracleProver(m, prep, num_queries=84)
    assert cpu.verify(p) == 0
    rc, ref = cpu.prove(tr, pv)  # the reference's maximal 2^22 shape, byte for byte (BASELINE config 3's size)
    assert rc == 0 and p == ref
    bad = dict(tr)
    bad["Bitwise"] = tr["Bitwise"].copy()
    bad["Bitwise"][12345, 3] ^= 1
    assert cpu.verify(gpu.prove_shard(bad, pv)) != 0
