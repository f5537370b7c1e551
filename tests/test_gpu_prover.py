"""Shard proofs from the MI355X path vs the CPU oracle: byte-identical proofs and identical
Fiat-Shamir transcripts (challenger state after `open`), plus acceptance by the oracle's
restated verifier.  This is the parity gate for MachineProver::commit/open."""
import numpy as np
import pytest

from tests import _oracle as O
from zkmips_amd import workloads as W
from zkmips_amd.machine import P

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    from zkmips_amd._lib import Device
    d = Device(0)
    yield d
    d.close()


def same_challenger(a, b):
    """sponge state, pending inputs and unread outputs (stale buffer slots are not state)."""
    a, b = np.asarray(a), np.asarray(b)
    nin, nout = int(a[16]), int(a[25])
    return (np.array_equal(a[:17], b[:17]) and np.array_equal(a[17:17 + nin], b[17:17 + nin])
            and a[25] == b[25] and np.array_equal(a[26:26 + nout], b[26:26 + nout]))


def provers(dev, n, nq=16, seed=7, montgomery=False):
    from zkmips_amd.prover import HipProver
    m, prep, traces, pvs = W.fib_shard(n, seed)
    gpu = HipProver(dev, m, prep, num_queries=nq, proof_montgomery=montgomery)
    cpu = O.OracleProver(m, prep, num_queries=nq, montgomery=montgomery)
    return gpu, cpu, traces, pvs


def test_setup_commitment_matches(dev):
    gpu, cpu, _, _ = provers(dev, 64)
    assert np.array_equal(gpu.vk_commit, cpu.commit)


@pytest.mark.parametrize("n", [16, 64, 1024, 1 << 13, 1 << 16])
def test_shard_proof_bytes_identical(dev, n):
    gpu, cpu, traces, pvs = provers(dev, n)
    ch = gpu.base_challenger()
    data = gpu.commit(traces, pvs)
    proof = gpu.open(data, ch)
    och = cpu.base_challenger()
    rc, ref = cpu.prove(traces, pvs, och)
    assert rc == 0
    assert len(proof) == len(ref)
    assert proof == ref
    # transcripts: the challenger ends in the same state
    assert same_challenger(ch.to_words(), och.s)
    assert cpu.verify(proof) == 0


def test_montgomery_proof_bytes(dev):
    gpu, cpu, traces, pvs = provers(dev, 64, nq=8, montgomery=True)
    proof = gpu.prove_shard(traces, pvs)
    rc, ref = cpu.prove(traces, pvs)
    assert rc == 0 and proof == ref and cpu.verify(proof) == 0


def test_montgomery_trace_input(dev):
    """Traces handed over in Montgomery form (the in-memory form of p3 MontyField31)."""
    gpu, cpu, traces, pvs = provers(dev, 256, nq=8)
    mont = {k: ((v.astype(np.uint64) << np.uint64(32)) % np.uint64(P)).astype(np.uint32) for k, v in traces.items()}
    ch = gpu.base_challenger()
    data = gpu.commit(mont, pvs, montgomery_input=True)
    proof = gpu.open(data, ch)
    rc, ref = cpu.prove(traces, pvs)
    assert proof == ref


def test_unsatisfied_trace_is_rejected(dev):
    """Like the reference, the prover emits a proof for a trace that breaks a constraint (all
    committed LDEs are low-degree by construction); the verifier's OOD check rejects it."""
    gpu, cpu, traces, pvs = provers(dev, 256, nq=8)
    bad = dict(traces)
    t = traces["FibCpu"].copy()
    t[100, 7] = (int(t[100, 7]) + 5) % P
    bad["FibCpu"] = t
    proof = gpu.prove_shard(bad, pvs)
    rc, ref = cpu.prove(bad, pvs)
    assert proof == ref
    assert cpu.verify(proof) != 0


def test_multi_shard_prove(dev):
    """MachineProver::prove: shards share the pk-observed challenger, each opens on a clone."""
    gpu, cpu, _, _ = provers(dev, 128, nq=8)
    shards, pvss = [], []
    for seed in (1, 2, 3):
        _, _, tr, pv = W.fib_shard(128, seed)
        shards.append(tr)
        pvss.append(pv)
    proofs = gpu.prove(shards, pvss)
    for tr, pv, pf in zip(shards, pvss, proofs):
        rc, ref = cpu.prove(tr, pv)
        assert rc == 0 and pf == ref


def test_concurrent_shards_from_threads(dev):
    """prove_with_context calls commit/open for all shards of a batch from rayon workers at once
    (crates/core/machine/src/utils/prove.rs:487-521): concurrent calls (one stream each) must give
    exactly the proofs of sequential calls."""
    import threading
    gpu, cpu, _, _ = provers(dev, 1 << 12, nq=8)
    work = [W.fib_shard(1 << 12, seed)[2:] for seed in (11, 12, 13, 14)]
    seq = [gpu.prove_shard(tr, pv) for tr, pv in work]
    out = [None] * len(work)

    def run(i):
        for _ in range(2):
            out[i] = gpu.prove_shard(*work[i])

    th = [threading.Thread(target=run, args=(i,)) for i in range(len(work))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert out == seq
    rc, ref = cpu.prove(*work[0])
    assert rc == 0 and seq[0] == ref


def test_shard_proof_bytes_identical_2e18(dev):
    """Byte parity at the largest size the oracle proves in seconds (84 queries, as the bench)."""
    gpu, cpu, traces, pvs = provers(dev, 1 << 18, nq=84)
    proof = gpu.prove_shard(traces, pvs)
    rc, ref = cpu.prove(traces, pvs)
    assert rc == 0 and proof == ref


def test_shard_proof_bytes_identical_2e22(dev):
    """Byte parity at the headline configuration itself: a 2^22-row FibCpu shard, 84 queries, the
    proof the bench times (the oracle needs ~1 min of its OpenMP threads for it)."""
    gpu, cpu, traces, pvs = provers(dev, 1 << 22, nq=84, seed=1000)
    ch = gpu.base_challenger()
    proof = gpu.open(gpu.commit(traces, pvs), ch)
    och = cpu.base_challenger()
    rc, ref = cpu.prove(traces, pvs, och)
    assert rc == 0 and proof == ref
    assert same_challenger(ch.to_words(), och.s)


@pytest.mark.parametrize("logn", [20, 22, 23])
def test_full_size_proof_verifies(dev, logn):
    """BASELINE sizes (2^20 .. 2^23 rows; 2^23 is the largest the two-adicity allows at blowup 2):
    size-independent properties where the oracle prover would take minutes -- the oracle's
    restated verifier accepts the GPU proof, proving twice is deterministic, and a flipped
    proof byte is rejected."""
    gpu, cpu, traces, pvs = provers(dev, 1 << logn, nq=84)
    proof = gpu.prove_shard(traces, pvs)
    assert cpu.verify(proof) == 0
    assert gpu.prove_shard(traces, pvs) == proof
    bad = bytearray(proof)
    bad[len(bad) // 2] ^= 1
    assert cpu.verify(bytes(bad)) != 0


def test_two_adicity_limit_is_an_error(dev):
    """A 2^24-row trace would need a 2^25-point LDE, beyond KoalaBear's two-adicity (24): the C ABI
    returns an error status instead of faulting."""
    from zkmips_amd._lib import ZkmError
    with pytest.raises(ZkmError):
        dev.bench_lde(1 << 24, 1, 1)


@pytest.mark.parametrize("zero_copy", ["0", "1"])
def test_pinned_host_traces(dev, zero_copy, monkeypatch):
    """Traces in page-locked host memory (zkm_host_alloc): copied by the DMA engine, or (ZKM_ZERO_COPY=1)
    read over PCIe by the transpose kernel itself; the proof equals the oracle's either way, for a main
    trace and a narrow table, with the CPU-side buffers released only after the call returns."""
    from zkmips_amd._lib import pinned_copy
    monkeypatch.setenv("ZKM_ZERO_COPY", zero_copy)
    gpu, cpu, traces, pvs = provers(dev, 1 << 14, seed=11)
    held = {k: pinned_copy(v) for k, v in traces.items()}
    p = gpu.prove_shard({k: h.array for k, h in held.items()}, pvs)
    rc, ref = cpu.prove(traces, pvs)
    assert rc == 0 and p == ref


def test_commit_through_machine_handle(dev):
    """zkm_commit_machine (no proving key) + zkm_open(key) gives the key-committed bytes; a shard
    committed under another machine is refused by open (ZKM_ERR_ARG), not proven against the key."""
    from zkmips_amd import mips_alu as A
    from zkmips_amd.prover import MachineHandle
    gpu, cpu, traces, pvs = provers(dev, 1 << 10, seed=9)
    mh = MachineHandle(gpu.machine, num_queries=16)
    data = mh.commit(dev, traces, pvs)
    proof = gpu.open(data, gpu.base_challenger())
    assert proof == gpu.prove_shard(traces, pvs)
    other = MachineHandle(A.alu_machine(), num_queries=16)
    am, aprep, atr, apv = A.alu_shard(64, 64, seed=1)
    bad = other.commit(dev, atr, apv)
    from zkmips_amd._lib import ZkmError
    with pytest.raises(ZkmError, match="different machine"):
        gpu.open(bad, gpu.base_challenger())
