"""The recursion machine's compress AIR (BASELINE config 5; zkmips_amd/recursion.py) under
compressed_fri_config (log_blowup 2, 42 queries; crates/stark/src/kb31_poseidon2.rs:217-227).

CPU: chip shapes against the reference's column structs, the Poseidon2 trace rows against the KATs, the
reference's own recursion test programs (mem/constant.rs:212-257, alu_base.rs:332-366,
alu_ext.rs:339-376, select.rs:297-330, poseidon2_wide/mod.rs:135-202) satisfy every constraint and
lookup, prove and verify at blowup 4; the reference's should_panic cases fail here too.
GPU: proof bytes equal the oracle's for every program and a verifier-shaped shard; the reference's
shrink shape (machine.rs:155-171) proves and verifies at full size.
The reference tests draw their values from StdRng; ours come from numpy's seeded generator (same
program structure, different field values)."""
import json
import os

import numpy as np
import pytest

from tests import _air_check as AC
from tests import _oracle as O
from tests import _rec_model as _RM
from zkmips_amd import recursion as R

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
LB, NQ = R.COMPRESS_LOG_BLOWUP, R.COMPRESS_NUM_QUERIES

# name: (prep, main, perm EF columns, log_qd, local_only, reference column structs / local_only override)
CHIPS = {
    "MemoryConst": (12, 1, 2, 1, True, "mem/constant.rs:24-38, :137-139"),
    "MemoryVar": (4, 8, 2, 1, True, "mem/variable.rs:25-38, :139-141"),
    "BaseAlu": (32, 12, 7, 1, True, "alu_base.rs:28-62, :263-265"),
    "ExtAlu": (32, 48, 7, 1, True, "alu_ext.rs:25-57, :259-261"),
    "Poseidon2WideDeg3": (49, 313, 17, 1, True, "poseidon2_wide/columns/permutation.rs:20-72, preprocessed.rs, trace.rs:170"),
    "BatchFRI": (6, 13, 3, 1, False, "batch_fri.rs:35-56"),
    "Select": (8, 5, 4, 1, True, "select.rs:25-40, :220-222"),
    "ExpReverseBitsLen": (10, 7, 3, 1, False, "exp_reverse_bits.rs:33-55"),
    "PublicValues": (10, 1, 2, 1, False, "public_values.rs:33-44"),
}


def test_compress_machine_chip_table():
    m = R.compress_machine()
    assert [c.name for c in m.chips] == list(CHIPS)  # machine.rs:112-128 order
    assert m.num_pv == 231
    for c in m.chips:
        prep, main, perm, lqd, lo, _ = CHIPS[c.name]
        assert (c.prep_width, c.main_width, c.perm_width_ef, c.log_quotient_degree, c.local_only) == \
            (prep, main, perm, lqd, lo), c.name
        assert c.log_quotient_degree <= LB


def test_wide_machine_chip_table():
    """machine_wide_with_all_chips (machine.rs:68-87): the compress chips with FriFold after
    Poseidon2WideDeg3; FriFold's columns are fri_fold.rs:40-78 and it opens at zeta and g*zeta."""
    m = R.wide_machine()
    names = [c.name for c in m.chips]
    assert names == ["MemoryConst", "MemoryVar", "BaseAlu", "ExtAlu", "Poseidon2WideDeg3", "FriFold", "BatchFRI",
                     "Select", "ExpReverseBitsLen", "PublicValues"]
    c = m.chips[m.chip_index("FriFold")]
    assert (c.prep_width, c.main_width, c.perm_width_ef, c.log_quotient_degree, c.local_only) == (20, 33, 6, 1, False)


def test_fri_fold_program():
    """FriFold instructions prove on the wide machine; a forged running reduced opening is rejected; the
    compress machine refuses them (it has no FriFold chip)."""
    m, pr, tr, pvs = R.shard(R.program_fri_fold(), wide=True)
    assert not any(AC.check(m, pr, tr, pvs))
    o = O.OracleProver(m, pr, num_queries=NQ, log_blowup=LB)
    rc, proof = o.prove(tr, pvs)
    assert rc == 0 and o.verify(proof) == 0
    bad = {k: v.copy() for k, v in tr.items()}
    bad["FriFold"][2, 30] = (int(bad["FriFold"][2, 30]) + 1) % R.P  # ro_output word 1 of row 2
    assert any(AC.check(m, pr, bad, pvs))
    with pytest.raises(ValueError):
        R.shard(R.program_fri_fold())


def test_poseidon2_rows_match_kats():
    kat = json.load(open(os.path.join(GOLDEN, "poseidon2_kat.json")))
    for v in kat.values():
        out = R.poseidon2_permute(np.asarray(v["input"], np.uint64))[0]
        assert [int(x) for x in out] == v["output"]


def test_ext_inverse():
    rng = np.random.default_rng(1)
    a = rng.integers(1, R.P, size=(64, 4)).astype(np.uint64)
    one = R.ext_mul(a, R.ext_inv(a))
    assert (one[:, 0] == 1).all() and (one[:, 1:] == 0).all()


PROGRAMS = {
    "empty": R.RecursionProgram,  # every chip present, all padding (height 16)
    "basic_mem": R.program_basic_mem,
    "base_four_ops": lambda: R.program_base_four_ops(1000),
    "ext_four_ops": lambda: R.program_ext_four_ops(1000),
    "select": lambda: R.program_select(1000),
    "poseidon2": R.program_poseidon2,
    "exp_reverse_bits": lambda: R.program_exp_reverse_bits(100, 16),
    "batch_fri": lambda: R.program_batch_fri(20, 7),
    "public_values": R.program_public_values,
    "merkle_openings": lambda: R.program_merkle_openings()[0],
}

SMALL_SHAPE = {k: (v - 7 if k != "PublicValues" else v) for k, v in R.SHRINK_SHAPE.items()}


@pytest.mark.parametrize("name", list(PROGRAMS))
def test_program_air_holds(name):
    m, pr, tr, pvs = R.shard(PROGRAMS[name]())
    bad_c, bad_l = AC.check(m, pr, tr, pvs)
    assert not bad_c and not bad_l


@pytest.mark.parametrize("name", ["basic_mem", "ext_four_ops", "poseidon2", "exp_reverse_bits", "batch_fri",
                                  "public_values"])
def test_program_oracle_proves_and_verifies(name):
    m, pr, tr, pvs = R.shard(PROGRAMS[name]())
    o = O.OracleProver(m, pr, num_queries=NQ, log_blowup=LB)
    rc, proof = o.prove(tr, pvs)
    assert rc == 0 and o.verify(proof) == 0


@pytest.mark.parametrize("name", list(PROGRAMS) + ["fri_fold", "verifier_shaped"])
def test_native_runtime_equals_numpy_runtime(name):
    """The native runtime (csrc/host/rec_exec.cpp) against the numpy one: the same event rows, resolved
    multiplicities and public values, so the same traces."""
    make = {"fri_fold": R.program_fri_fold, "verifier_shaped": lambda: R.program_verifier_shaped(SMALL_SHAPE)}
    prog = make[name]() if name in make else PROGRAMS[name]()
    a = R.execute(prog)
    b = R.execute_numpy(R._copy_program(prog))
    for k in b.ev:
        assert a.ev[k].shape == b.ev[k].shape and np.array_equal(a.ev[k], b.ev[k]), k
    for k in b.flat.a:
        for nm, v in b.flat.a[k].items():
            assert np.array_equal(a.flat.a[k][nm], v), (k, nm)
    assert np.array_equal(a.public_values, b.public_values)
    for x, y in zip(R.generate_traces(a), R.generate_traces(b)):
        assert set(x) == set(y) and all(np.array_equal(x[k], y[k]) for k in x)
    # the per-block event view of the native record is the numpy runtime's
    for k, evs in b.events.items():
        for e, f in zip(a.events[k], evs):
            assert set(e) == set(f) and all(np.array_equal(e[nm], f[nm]) for nm in e), k


def test_native_runtime_rejects_what_the_numpy_one_rejects():
    """Write-once memory: a second write, a read of an unwritten address, a read inside the block that
    writes it, and a constant-memory read of a different value are RuntimeErrors naming the block."""
    def prog(build):
        p = R.RecursionProgram(num_addrs=8)
        p.mem_write([0, 1], [[2, 0, 0, 0], [3, 0, 0, 0]])
        build(p)
        return p
    bad = [lambda p: p.base_alu(R.OP_ADD, [0], [0], [1]),                  # writes address 0 again
           lambda p: p.base_alu(R.OP_MUL, [2], [5], [1]),                  # reads unwritten address 5
           lambda p: p.base_alu(R.OP_ADD, [2, 3], [0, 2], [1, 1]),         # reads 2 in the block writing it
           lambda p: p.mem_read([1], [[4, 0, 0, 0]]),                      # constant read of a wrong value
           lambda p: p.select([0], [2], [2], [0], [1])]                    # both outputs to one address
    for f in bad:
        with pytest.raises(RuntimeError, match="block 1"):
            R.execute(prog(f))
        with pytest.raises(RuntimeError):
            R.execute_numpy(prog(f))
    R.execute(prog(lambda p: p.base_alu(R.OP_DIV, [2], [0], [1])))


def test_verifier_shaped_program():
    prog = R.program_verifier_shaped(SMALL_SHAPE)
    m, pr, tr, pvs = R.shard(prog, SMALL_SHAPE)
    for name, lg in SMALL_SHAPE.items():
        assert tr[name].shape[0] == 1 << lg
    assert not any(AC.check(m, pr, tr, pvs))
    o = O.OracleProver(m, pr, num_queries=NQ, log_blowup=LB)
    rc, proof = o.prove(tr, pvs)
    assert rc == 0 and o.verify(proof) == 0


def test_merkle_layers_root_is_the_mmcs_root():
    """The recursion program's hashing (sponge of a row, TruncatedPermutation of two digests) is the
    MerkleTreeMmcs of the core prover: its root equals the oracle's MMCS root of the same matrix."""
    for h, w in ((16, 8), (64, 21), (256, 67)):
        m = np.random.default_rng(h).integers(0, R.P, (h, w)).astype(np.uint32)
        assert np.array_equal(R.merkle_layers(m)[-1][0].astype(np.uint32), O.merkle_root([m]))


def test_merkle_openings_reject_a_wrong_path():
    """A forged sibling digest (or opened value) recomputes a different root: the runtime's read-back of
    the root fails, and a trace built anyway leaves the memory bus unbalanced."""
    p, mat = R.program_merkle_openings(6, 9, 4, seed=2)
    hint = next(b for b in p.blocks if b.kind == "hint" and len(b) == 4 * 6 * 8)  # the sibling digests
    hint.a["vals"][5, 0] = (hint.a["vals"][5, 0] + 1) % R.P
    with pytest.raises(RuntimeError):
        R.shard(p)
    p2, _ = R.program_merkle_openings(6, 9, 4, seed=2)
    rows = next(b for b in p2.blocks if b.kind == "hint" and len(b) == 4 * 9)  # the opened rows
    rows.a["vals"][3, 0] = (rows.a["vals"][3, 0] + 1) % R.P
    with pytest.raises(RuntimeError):
        R.shard(p2)


def test_reference_should_panic_cases():
    """mem/constant.rs:222-257 / mem/variable.rs:201-242: a read of 999 copies, of address 999 and of
    the value 999 after writing 2 at address 1 (mult 1)."""
    p = R.RecursionProgram(num_addrs=2)
    p.mem_write([1], [[2, 0, 0, 0]], mult=1)
    p.mem_read([1], [[2, 0, 0, 0]], mult=999)
    m, pr, tr, pvs = R.shard(p)
    assert AC.check(m, pr, tr, pvs)[1], "bad mult must unbalance the memory bus"
    o = O.OracleProver(m, pr, num_queries=8, log_blowup=LB)
    rc, proof = o.prove(tr, pvs)
    assert rc != 0 or o.verify(proof) != 0
    for addr, val in ((999, 2), (1, 999)):
        p = R.RecursionProgram(num_addrs=2)
        p.mem_write([1], [[2, 0, 0, 0]], mult=1)
        p.mem_read([addr], [[val, 0, 0, 0]], mult=1)
        with pytest.raises((RuntimeError, IndexError)):
            R.shard(p)


@pytest.mark.parametrize("chip,row,col", [("BaseAlu", 3, 0), ("ExtAlu", 5, 13), ("Poseidon2WideDeg3", 1, 200),
                                          ("ExpReverseBitsLen", 4, 4), ("BatchFRI", 2, 1), ("Select", 0, 1)])
def test_tampered_traces_rejected(chip, row, col):
    prog = R.program_verifier_shaped(SMALL_SHAPE)
    m, pr, tr, pvs = R.shard(prog, SMALL_SHAPE)
    tr[chip][row, col] = (int(tr[chip][row, col]) + 1) % R.P
    assert any(AC.check(m, pr, tr, pvs))
    o = O.OracleProver(m, pr, num_queries=8, log_blowup=LB)
    rc, proof = o.prove(tr, pvs)
    assert rc != 0 or o.verify(proof) != 0


def test_public_values_digest_bound():
    m, pr, tr, pvs = R.shard(R.program_public_values())
    bad = pvs.copy()
    bad[R.PV_DIGEST_START + 3] ^= 1
    assert AC.check(m, pr, tr, bad)[0]
    bad = pvs.copy()
    bad[5] ^= 1  # outside the digest: not constrained by the PublicValues chip
    assert not any(AC.check(m, pr, tr, bad))


@pytest.fixture(scope="module")
def dev():
    from zkmips_amd._lib import Device
    d = Device(0)
    yield d
    d.close()


@pytest.mark.gpu
def test_gpu_recursion_programs_proof_bytes_identical(dev):
    from zkmips_amd.prover import HipProver
    for name, mk in PROGRAMS.items():
        m, pr, tr, pvs = R.shard(mk())
        gpu = HipProver(dev, m, pr, num_queries=NQ, log_blowup=LB)
        cpu = O.OracleProver(m, pr, num_queries=NQ, log_blowup=LB)
        assert np.array_equal(gpu.vk_commit, cpu.commit), name
        proof = gpu.prove_shard(tr, pvs)
        rc, ref = cpu.prove(tr, pvs)
        assert rc == 0 and proof == ref, name
        assert cpu.verify(proof) == 0, name


@pytest.mark.gpu
def test_gpu_wide_machine_fri_fold_bytes_identical(dev):
    from zkmips_amd.prover import HipProver
    m, pr, tr, pvs = R.shard(R.program_fri_fold(64, 7), wide=True)
    gpu = HipProver(dev, m, pr, num_queries=NQ, log_blowup=LB)
    cpu = O.OracleProver(m, pr, num_queries=NQ, log_blowup=LB)
    proof = gpu.prove_shard(tr, pvs)
    rc, ref = cpu.prove(tr, pvs)
    assert rc == 0 and proof == ref and cpu.verify(proof) == 0


@pytest.mark.gpu
def test_gpu_verifier_shaped_proof_bytes_identical(dev):
    from zkmips_amd.prover import HipProver
    shape = {k: (v - 4 if k != "PublicValues" else v) for k, v in R.SHRINK_SHAPE.items()}
    m, pr, tr, pvs = R.shard(R.program_verifier_shaped(shape), shape)
    gpu = HipProver(dev, m, pr, num_queries=NQ, log_blowup=LB)
    cpu = O.OracleProver(m, pr, num_queries=NQ, log_blowup=LB)
    assert np.array_equal(gpu.vk_commit, cpu.commit)
    proof = gpu.prove_shard(tr, pvs)
    rc, ref = cpu.prove(tr, pvs)
    assert rc == 0 and proof == ref and cpu.verify(proof) == 0


@pytest.mark.gpu
def test_gpu_shrink_shape_full_size_verifies(dev):
    """The reference's shrink shape (MemoryVar/Select 2^18, ..., Poseidon2WideDeg3 2^16) at full size:
    GPU proof bytes == the oracle's; the oracle verifier accepts the GPU proof and rejects a flipped byte."""
    from zkmips_amd.prover import HipProver
    m, pr, tr, pvs = R.shard(R.program_verifier_shaped(), R.SHRINK_SHAPE)
    gpu = HipProver(dev, m, pr, num_queries=NQ, log_blowup=LB)
    cpu = O.OracleProver(m, pr, num_queries=NQ, log_blowup=LB)
    proof = gpu.prove_shard(tr, pvs)
    assert cpu.verify(proof) == 0
    rc, ref = cpu.prove(tr, pvs)
    assert rc == 0 and proof == ref  # byte for byte at the reference's shrink shape
    bad = bytearray(proof)
    bad[len(bad) // 2] ^= 1
    assert cpu.verify(bytes(bad)) != 0


def _p2_records(rec):
    """Poseidon2Io records (input[16], output[16]) of a run's Poseidon2 events, canonical."""
    ins = np.concatenate([e["inputs"] for e in rec.events["p2"]])
    outs = np.concatenate([e["outputs"] for e in rec.events["p2"]])
    return np.ascontiguousarray(np.concatenate([ins, outs], 1).astype(np.uint32))


def test_poseidon2_wide_trace_abi_declared():
    hdr = open(os.path.join(os.path.dirname(GOLDEN), "..", "include", "zkm_tracegen.h")).read()
    assert "#define ZKM_POSEIDON2_WIDE_DEG3_WIDTH 313" in hdr and "zkm_poseidon2_wide_events_to_trace" in hdr


@pytest.mark.gpu
@pytest.mark.parametrize("montgomery", [False, True])
def test_gpu_poseidon2_wide_device_trace_equals_host(dev, montgomery):
    """zkm_poseidon2_wide_events_to_trace == the host trace builder, padding rows included, for the
    shrink-shape program's 59k permutations (height 2^16) and a ragged small case; Montgomery input
    (a Rust Vec<Poseidon2Event<KoalaBear>> as it lies in memory) gives the same canonical trace."""
    import torch
    from zkmips_amd import tracegen as TG
    for prog, shape in ((R.program_poseidon2(), None), (R.program_verifier_shaped(), R.SHRINK_SHAPE)):
        rec = R.execute(prog)
        _, tr = R.generate_traces(rec, shape)
        want = tr["Poseidon2WideDeg3"]
        recs = _p2_records(rec)
        if montgomery:
            recs = ((recs.astype(np.uint64) << np.uint64(32)) % np.uint64(R.P)).astype(np.uint32)
        d = torch.from_numpy(recs.view(np.int32).reshape(-1).copy()).cuda()
        got = TG.poseidon2_wide_trace(d, len(recs), height=want.shape[0], montgomery=montgomery)
        torch.cuda.synchronize()
        assert np.array_equal(got.cpu().numpy().view(np.uint32), want)


@pytest.mark.gpu
def test_gpu_device_poseidon2_trace_proves_identically(dev):
    """A compress shard whose Poseidon2WideDeg3 trace comes from the device proves to the host traces'
    proof bytes."""
    import torch
    from zkmips_amd import tracegen as TG
    from zkmips_amd.prover import HipProver
    shape = {k: (v - 4 if k != "PublicValues" else v) for k, v in R.SHRINK_SHAPE.items()}
    prog = R.program_verifier_shaped(shape)
    m, pr, tr, pvs = R.shard(prog, shape)
    rec = R.execute(R.program_verifier_shaped(shape))
    recs = _p2_records(rec)
    d = torch.from_numpy(recs.view(np.int32).reshape(-1).copy()).cuda()
    dev_tr = dict(tr)
    dev_tr["Poseidon2WideDeg3"] = TG.poseidon2_wide_trace(d, len(recs), height=tr["Poseidon2WideDeg3"].shape[0]) \
        .cpu().numpy().view(np.uint32)
    gpu = HipProver(dev, m, pr, num_queries=NQ, log_blowup=LB)
    assert gpu.prove_shard(dev_tr, pvs) == gpu.prove_shard(tr, pvs)


_PREP_PROGRAMS = [(R.program_fri_fold, None), (R.program_batch_fri, None), (lambda: R.program_select(100), None),
                  (lambda: R.program_exp_reverse_bits(20, 8), None), (R.program_poseidon2, None),
                  (R.RecursionProgram, None), (R.program_public_values, None), (R.program_basic_mem, None),
                  (lambda: R.program_ext_four_ops(50), None), (lambda: R.program_base_four_ops(50), None)]


def test_prep_records_lay_out_to_prep_traces():
    """recursion.prep_records, laid out as zkm_recursion_instrs_to_trace lays them out (a numpy model of
    the kernel), are the preprocessed traces, padding rows included."""
    for make, shape in _PREP_PROGRAMS:
        rec = R.execute(make())
        want = R.prep_traces(rec, shape)
        for chip, (recs, h) in R.prep_records(rec, shape).items():
            assert np.array_equal(_RM.instr_rows_model(chip, recs, h), want[chip]), chip


@pytest.mark.gpu
@pytest.mark.parametrize("montgomery", [False, True])
def test_gpu_recursion_instr_rows_equal_host(dev, montgomery):
    """zkm_recursion_instrs_to_trace (instr_to_row of every compress / wide-machine chip) == the host
    preprocessed traces, for the test programs and the verifier-shaped program at its shape; Montgomery
    field words as the Rust records hold them, integer words plain."""
    import torch
    from zkmips_amd import tracegen as TG
    for make, shape in _PREP_PROGRAMS + [(lambda: R.program_verifier_shaped(SMALL_SHAPE), SMALL_SHAPE)]:
        rec = R.execute(make())
        want = R.prep_traces(rec, shape)
        for chip, (recs, h) in R.prep_records(rec, shape).items():
            words = recs.copy()
            if montgomery:
                ints = TG.RECURSION_INSTR_CHIPS[chip][3]
                fw = [c for c in range(words.shape[1]) if c not in ints]
                words[:, fw] = ((words[:, fw].astype(np.uint64) << np.uint64(32)) % np.uint64(R.P)).astype(np.uint32)
            t = torch.from_numpy(words.reshape(-1).view(np.int32).copy() if words.size else np.zeros(1, np.int32)).cuda()
            got = TG.recursion_instrs_trace(chip, t, len(recs), h, montgomery=montgomery)
            torch.cuda.synchronize()
            assert np.array_equal(got.cpu().numpy().view(np.uint32), want[chip]), chip


@pytest.mark.gpu
@pytest.mark.parametrize("montgomery", [False, True])
def test_gpu_recursion_event_rows_equal_host(dev, montgomery):
    """zkm_recursion_events_to_trace (BaseAlu, ExtAlu, BatchFRI, Select, FriFold, PublicValues, MemoryVar,
    MemoryConst) == the host main traces, padding rows included, for the wide machine's programs and the
    verifier-shaped program at its shape; canonical and Montgomery event words."""
    import torch
    from zkmips_amd import tracegen as TG
    for prog, shape in ((R.program_fri_fold(), None), (R.program_batch_fri(), None), (R.program_select(300), None),
                        (R.program_verifier_shaped(SMALL_SHAPE), SMALL_SHAPE), (R.RecursionProgram(), None)):
        rec = R.execute(prog)
        want = R.main_traces(rec, shape, p2_main=False)
        h = R._heights(rec, shape or {})
        for chip in TG.RECURSION_EVENT_CHIPS:
            ev = (np.zeros((0, 1), np.uint32) if chip == "MemoryConst" else np.ascontiguousarray(R.main_events(rec, chip)))
            words = ev if not montgomery else ((ev.astype(np.uint64) << np.uint64(32)) % np.uint64(R.P)).astype(np.uint32)
            t = torch.from_numpy(words.reshape(-1).view(np.int32).copy() if words.size else np.zeros(1, np.int32)).cuda()
            got = TG.recursion_events_trace(chip, t, len(ev), h[chip], montgomery=montgomery)
            torch.cuda.synchronize()
            assert np.array_equal(got.cpu().numpy().view(np.uint32), want[chip]), chip
    with pytest.raises(Exception):
        TG.recursion_events_trace("BaseAlu", torch.zeros(3 * 65, dtype=torch.int32, device="cuda"), 65, 16)


@pytest.mark.gpu
def test_gpu_exp_reverse_bits_device_trace_equals_host(dev):
    """zkm_exp_reverse_bits_events_to_trace == the host ExpReverseBitsLen trace (the reference test
    program and the shrink-shape program's 5362 events), canonical and Montgomery records."""
    import torch
    from zkmips_amd import tracegen as TG
    for prog, shape in ((R.program_exp_reverse_bits(100, 16), None), (R.program_verifier_shaped(), R.SHRINK_SHAPE)):
        rec = R.execute(prog)
        _, tr = R.generate_traces(rec, shape)
        want = tr["ExpReverseBitsLen"]
        ev = rec.events["exprev"]
        rows = np.concatenate([e["rows"] for e in ev])
        lens = np.concatenate([np.full(e["n"], e["L"]) for e in ev])
        offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        base = rows[offs[:-1], 0].astype(np.uint32)
        bits = rows[:, 1].astype(np.uint32)
        for mont in (False, True):
            b_, x_ = (bits, base) if not mont else tuple(
                ((v.astype(np.uint64) << np.uint64(32)) % np.uint64(R.P)).astype(np.uint32) for v in (bits, base))
            got = TG.exp_reverse_bits_trace(torch.from_numpy(x_.view(np.int32).copy()).cuda(),
                                            torch.from_numpy(b_.view(np.int32).copy()).cuda(),
                                            torch.from_numpy(offs).cuda(), len(base), want.shape[0], montgomery=mont)
            torch.cuda.synchronize()
            assert np.array_equal(got.cpu().numpy().view(np.uint32), want)
