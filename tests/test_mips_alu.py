"""MIPS ALU slice (AddSub, Bitwise, Lt, ShiftLeft, ShiftRight, CloClz, Byte restated from the reference AIRs; zkmips_amd/mips_alu.py).

CPU part: the trace generators reproduce the reference's own fixtures and table semantics, the
oracle proves and its verifier accepts a multi-chip shard whose Byte / Instruction lookups balance
across chips, and it rejects broken carries, forged bitwise results and wrong multiplicities.
GPU part: the HIP prover's proofs are byte-identical to the oracle's, and at the bench size
(InstrSource 2^22 rows) the oracle verifier accepts them."""
import numpy as np
import pytest

from tests import _oracle as O
from zkmips_amd import mips_alu as A


def test_byte_table_semantics():
    t = A.byte_prep_trace()
    assert t.shape == (1 << 16, 12)
    for b, c in [(0, 0), (10, 19), (255, 1), (200, 7), (3, 255), (128, 9)]:
        r = t[b * 256 + c]
        sh = c & 7
        assert list(r[:2]) == [b, c]
        assert r[A.BP_AND] == b & c and r[A.BP_OR] == b | c and r[A.BP_XOR] == b ^ c
        assert r[A.BP_NOR] == (~(b | c)) & 0xFF and r[A.BP_SLL] == (b << sh) & 0xFF
        assert r[A.BP_SHR] == b >> sh and r[A.BP_SHR_CARRY] == (b & ((1 << sh) - 1) if sh else 0)
        assert r[A.BP_LTU] == int(b < c) and r[A.BP_MSB] == b >> 7 and r[A.BP_U16] == (b << 8) + c


def test_reference_fixture_events():
    """The events of the reference's own generate_trace tests (bitwise/mod.rs:253-258,
    add_sub/mod.rs:296) land in the documented columns and prove."""
    ev = A.events_from_list([(0, A.OP_ADD, 14, 8, 6)],
                            [(0, A.OP_XOR, 25, 10, 19), (0, A.OP_OR, 27, 10, 19), (0, A.OP_AND, 2, 10, 19),
                             (0, A.OP_NOR, 228 + (0xFFFFFF << 8), 10, 19)])
    m, prep, tr, pv = A.alu_shard_from(ev)
    asub = tr["AddSub"][0]
    assert list(asub[A.AS_VAL:A.AS_VAL + 4]) == [14, 0, 0, 0]
    assert list(asub[A.AS_OP1:A.AS_OP1 + 4]) == [8, 0, 0, 0] and asub[A.AS_ADD] == 1 and asub[A.AS_NPC] == 4
    bw = tr["Bitwise"]
    assert [bw[i, A.BW_A] for i in range(4)] == [25, 27, 2, 228]
    assert bw[0, A.BW_XOR] == 1 and bw[1, A.BW_OR] == 1 and bw[2, A.BW_AND] == 1 and bw[3, A.BW_NOR] == 1
    mult = tr["Byte"]
    assert mult[10 * 256 + 19, A.B_XOR] == 1 and mult[10 * 256 + 19, A.B_NOR] == 1
    assert mult[0, A.B_NOR] == 3  # upper NOR limbs: NOR(0, 0) = 255
    cpu = O.OracleProver(m, prep, num_queries=8)
    rc, proof = cpu.prove(tr, pv)
    assert rc == 0 and cpu.verify(proof) == 0


@pytest.fixture(scope="module")
def shard():
    return A.alu_shard(300, 200, seed=5, n_lt=250, n_sll=100, n_sr=120, n_clz=40)


@pytest.fixture(scope="module")
def oracle(shard):
    m, prep, _, _ = shard
    return O.OracleProver(m, prep, num_queries=16)


def test_alu_shard_proves_and_verifies(shard, oracle):
    m, _, tr, pv = shard
    heights = {k: v.shape[0] for k, v in tr.items()}
    assert heights == {"InstrSource": 1024, "AddSub": 512, "Bitwise": 256, "Lt": 256, "ShiftLeft": 128,
                       "ShiftRight": 256, "CloClz": 64, "Byte": 65536}
    assert [c.name for c in m.chips] == ["InstrSource", "AddSub", "Bitwise", "Lt", "ShiftLeft", "ShiftRight",
                                         "CloClz", "Byte"]
    assert [c.perm_width_ef for c in m.chips] == [2, 5, 4, 3, 4, 14, 4, 6]
    rc, proof = oracle.prove(tr, pv)
    assert rc == 0 and oracle.verify(proof) == 0


def test_shard_without_some_chips(oracle):
    """A shard includes only the chips that have events (MachineAir::included)."""
    m, prep, tr, pv = A.alu_shard(64, 32, seed=8)
    assert sorted(tr) == ["AddSub", "Bitwise", "Byte", "InstrSource"]
    rc, proof = oracle.prove(tr, pv)
    assert rc == 0 and oracle.verify(proof) == 0


def test_cloclz_reference_fixture():
    """The events of the reference's CloClz generate_trace test (alu/clo_clz/mod.rs:289-296); every
    non-zero operand makes the chip send an SRL that the ShiftRight chip receives."""
    ev = A.events_from_list([], [], clz_events=[(0, A.OP_CLZ, 32, 0, 0), (0, A.OP_CLZ, 8, 0x00800000, 0),
                                                (0, A.OP_CLZ, 0, 0xFFFFFFFF, 0), (0, A.OP_CLO, 32, 0xFFFFFFFF, 0),
                                                (0, A.OP_CLO, 8, 0xFF7FFFFF, 0), (0, A.OP_CLO, 0, 0, 0)])
    m, prep, tr, pv = A.alu_shard_from(ev)
    cz, sr = tr["CloClz"], tr["ShiftRight"]
    assert list(cz[:6, A.CZ_BB_ZERO]) == [1, 0, 0, 1, 0, 0]
    assert list(sr[:4, A.SR_PC]) == [A.UNUSED_PC] * 4 and sr[:4, A.SR_SRL].all()
    assert list(cz[10, [A.CZ_A, A.CZ_CLZ, A.CZ_BB_ZERO, A.CZ_REAL]]) == [32, 1, 1, 0]  # padding row
    cpu = O.OracleProver(m, prep, num_queries=8)
    rc, proof = cpu.prove(tr, pv)
    assert rc == 0 and cpu.verify(proof) == 0


def test_shift_right_semantics():
    """SRL/SRA/ROR by every shift amount, including negative operands for SRA."""
    b = 0x8123F567
    evs = []
    for i in range(40):
        s = i & 31
        evs += [(12 * i, A.OP_SRL, b >> s, b, i), (12 * i + 4, A.OP_SRA, ((b - (1 << 32)) >> s) & 0xFFFFFFFF, b, i),
                (12 * i + 8, A.OP_ROR, ((b >> s) | (b << (32 - s))) & 0xFFFFFFFF, b, i)]
    m, prep, tr, pv = A.alu_shard_from(A.events_from_list([], [], sr_events=evs))
    sr = tr["ShiftRight"]
    assert sr.shape[0] == 128 and sr[127, A.SR_NBITS] == 1 and sr[127, A.SR_NBYTES] == 1  # padding rows
    cpu = O.OracleProver(m, prep, num_queries=8)
    rc, proof = cpu.prove(tr, pv)
    assert rc == 0 and cpu.verify(proof) == 0


def test_lt_sll_semantics():
    """SLT/SLTU over equal, sign-differing and shared-prefix operands; SLL by every shift amount."""
    ev = A.events_from_list([], [], [(0, A.OP_SLT, 1, 0xFFFFFFFF, 0), (4, A.OP_SLTU, 0, 0xFFFFFFFF, 0),
                                     (8, A.OP_SLT, 0, 7, 7), (12, A.OP_SLTU, 1, 0x12345600, 0x12345700),
                                     (16, A.OP_SLT, 0, 0x7FFFFFFF, 0x80000000)],
                            [(4 * i, A.OP_SLL, (0x81234567 << (i & 31)) & 0xFFFFFFFF, 0x81234567, i) for i in range(40)])
    m, prep, tr, pv = A.alu_shard_from(ev)
    lt = tr["Lt"]
    assert list(lt[:5, A.LT_COMP_EQ]) == [0, 0, 1, 0, 0]
    assert list(lt[3, A.LT_FLAGS:A.LT_FLAGS + 4]) == [0, 1, 0, 0]  # first differing byte from the top
    sl = tr["ShiftLeft"]
    assert all(sl[i, A.SL_NBYTES + ((i & 31) // 8)] == 1 for i in range(40))
    assert list(sl[50, A.SL_NBITS:A.SL_NBITS + 2]) == [1, 0] and sl[50, A.SL_MULT] == 1  # padding row
    cpu = O.OracleProver(m, prep, num_queries=8)
    rc, proof = cpu.prove(tr, pv)
    assert rc == 0 and cpu.verify(proof) == 0


@pytest.mark.parametrize("what", ["carry", "bitwise_result", "byte_mult", "dropped_instruction", "lt_result",
                                  "sll_carry", "sr_sign", "clz_count"])
def test_alu_tamper_rejected(shard, oracle, what):
    _, _, tr, pv = shard
    bad = {k: v.copy() for k, v in tr.items()}
    if what == "carry":  # a carry that does not match the limb sums breaks AddOperation
        bad["AddSub"][7, A.AS_CARRY] ^= 1
    elif what == "bitwise_result":  # a forged result byte: the Byte lookup no longer balances
        bad["Bitwise"][3, A.BW_A] = (int(bad["Bitwise"][3, A.BW_A]) + 1) % 256
    elif what == "byte_mult":
        bad["Byte"][1234, A.B_U8RANGE] += 1
    elif what == "lt_result":  # SLT result flipped together with the intermediate sltu
        bad["Lt"][9, A.LT_A] ^= 1
        bad["Lt"][9, A.LT_SLTU_R] ^= 1
    elif what == "sll_carry":
        bad["ShiftLeft"][4, A.SL_CARRY] += 1
    elif what == "clz_count":  # a wrong leading-zero count: the SRL it sends has no receiver
        bad["CloClz"][3, A.CZ_A] += 1
    elif what == "sr_sign":  # an SRA/ROR row whose sign bit disagrees with b's top byte
        bad["ShiftRight"][5, A.SR_MSB] ^= 1
    else:  # the CPU stand-in claims an instruction no ALU chip executes
        bad["InstrSource"][1020, A.IS_REAL] = 1  # a padding row (1010 events)
    rc, proof = oracle.prove(bad, pv)
    assert rc == 0
    assert oracle.verify(proof) != 0


# ---------------------------------------------------------------- GPU parity
@pytest.fixture(scope="module")
def dev():
    from zkmips_amd._lib import Device
    d = Device(0)
    yield d
    d.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n_add,n_bit,n_lt,n_sll,n_sr,n_clz", [(300, 200, 0, 0, 0, 0), (300, 200, 250, 100, 120, 40),
                                                              (1 << 13, 5000, 3000, 1 << 12, 7000, 3000),
                                                              (1 << 15, 1 << 15, 1 << 15, 1 << 14, 1 << 13, 1 << 13)])
def test_alu_gpu_proof_bytes_identical(dev, n_add, n_bit, n_lt, n_sll, n_sr, n_clz):
    from zkmips_amd.prover import HipProver
    m, prep, tr, pv = A.alu_shard(n_add, n_bit, seed=n_add, n_lt=n_lt, n_sll=n_sll, n_sr=n_sr, n_clz=n_clz)
    gpu = HipProver(dev, m, prep, num_queries=16)
    cpu = O.OracleProver(m, prep, num_queries=16)
    assert np.array_equal(gpu.vk_commit, cpu.commit)
    proof = gpu.prove_shard(tr, pv)
    rc, ref = cpu.prove(tr, pv)
    assert rc == 0 and proof == ref
    assert cpu.verify(proof) == 0


@pytest.mark.gpu
def test_alu_gpu_full_size_verifies(dev):
    from zkmips_amd.prover import HipProver
    m, prep, tr, pv = A.alu_shard(1 << 20, 1 << 20, seed=9, n_lt=1 << 20, n_sll=1 << 19, n_sr=1 << 18,
                                  n_clz=1 << 18)
    assert tr["InstrSource"].shape[0] == 1 << 22
    gpu = HipProver(dev, m, prep, num_queries=84)
    cpu = O.OracleProver(m, prep, num_queries=84)
    proof = gpu.prove_shard(tr, pv)
    assert cpu.verify(proof) == 0
    bad = {k: v.copy() for k, v in tr.items()}
    bad["AddSub"][12345, A.AS_CARRY + 1] ^= 1
    assert cpu.verify(gpu.prove_shard(bad, pv)) != 0
