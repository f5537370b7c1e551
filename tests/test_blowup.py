"""log_blowup 2 (blowup 4), the recursion/compress configuration (compressed_fri_config: log_blowup 2,
crates/stark/src/kb31_poseidon2.rs:217-227), with a degree-5 chip whose log_quotient_degree 2 equals it.
Bit-reversed LDE rows on 3 H_{4N} are the blowup-2 LDE (shift 3) followed by the blowup-2 LDE with
shift 3 w_{4N}; the quotient domain (2^log_qd N points) is the first rows of it."""
import numpy as np
import pytest

from tests import _oracle as O
from zkmips_amd import workloads as W


def test_deg5_chip_quotient_degree():
    m, _, _, _ = W.deg5_shard(64)
    assert m.chips[m.chip_index("Pow5")].log_quotient_degree == 2
    assert m.chips[m.chip_index("FibCpu")].log_quotient_degree == 1


@pytest.mark.parametrize("shard", ["fib", "deg5"])
def test_oracle_blowup4_proves_and_verifies(shard):
    m, prep, tr, pv = (W.fib_shard if shard == "fib" else W.deg5_shard)(1 << 9, 3)
    pr = O.OracleProver(m, prep, num_queries=8, log_blowup=2)
    rc, proof = pr.prove(tr, pv)
    assert rc == 0 and pr.verify(proof) == 0
    bad = {k: v.copy() for k, v in tr.items()}
    k = "Pow5" if shard == "deg5" else "FibCpu"
    bad[k][5, 1] = (int(bad[k][5, 1]) + 1) % W.P
    rc, proof = pr.prove(bad, pv)
    assert pr.verify(proof) != 0


def test_oracle_rejects_quotient_degree_above_blowup():
    m, prep, tr, pv = W.deg5_shard(1 << 6, 3)
    pr = O.OracleProver(m, prep, num_queries=8, log_blowup=1)
    rc, _ = pr.prove(tr, pv)
    assert rc != 0


@pytest.fixture(scope="module")
def dev():
    from zkmips_amd._lib import Device
    d = Device(0)
    yield d
    d.close()


@pytest.mark.gpu
@pytest.mark.parametrize("shard,n", [("fib", 16), ("fib", 1 << 12), ("deg5", 64), ("deg5", 1 << 14)])
def test_gpu_blowup4_proof_bytes_identical(dev, shard, n):
    from zkmips_amd.prover import HipProver
    m, prep, tr, pv = (W.fib_shard if shard == "fib" else W.deg5_shard)(n, 5)
    gpu = HipProver(dev, m, prep, num_queries=42, log_blowup=2)
    cpu = O.OracleProver(m, prep, num_queries=42, log_blowup=2)
    assert np.array_equal(gpu.vk_commit, cpu.commit)
    proof = gpu.prove_shard(tr, pv)
    rc, ref = cpu.prove(tr, pv)
    assert rc == 0 and proof == ref and cpu.verify(proof) == 0


@pytest.mark.gpu
def test_gpu_blowup4_large_verifies(dev):
    """2^20 rows at blowup 4 (a 2^22-point LDE): the oracle verifier accepts, a flipped byte is rejected."""
    from zkmips_amd.prover import HipProver
    m, prep, tr, pv = W.deg5_shard(1 << 20, 9)
    gpu = HipProver(dev, m, prep, num_queries=42, log_blowup=2)
    cpu = O.OracleProver(m, prep, num_queries=42, log_blowup=2)
    proof = gpu.prove_shard(tr, pv)
    assert cpu.verify(proof) == 0
    bad = bytearray(proof)
    bad[len(bad) // 3] ^= 1
    assert cpu.verify(bytes(bad)) != 0


@pytest.mark.gpu
def test_gpu_rejects_quotient_degree_above_blowup(dev):
    from zkmips_amd._lib import ZkmError
    from zkmips_amd.prover import HipProver
    m, prep, tr, pv = W.deg5_shard(64, 5)
    gpu = HipProver(dev, m, prep, num_queries=8, log_blowup=1)
    with pytest.raises(ZkmError):
        gpu.prove_shard(tr, pv)


_BATCHED = r"""
import hashlib, sys
from zkmips_amd import workloads as W
from zkmips_amd._lib import Device
from zkmips_amd.prover import HipProver
m, prep, tr, pv = W.deg5_shard(1 << 14, 5)
d = Device(0)
print(hashlib.sha256(HipProver(d, m, prep, num_queries=42, log_blowup=2).prove_shard(tr, pv)).hexdigest())
d.close()
"""


@pytest.mark.gpu
@pytest.mark.parametrize("env", [{"ZKM_LDE_CB": "3"}, {"ZKM_LDE_CB": "3", "ZKM_LDE4_SHARED": "0"}])
def test_gpu_blowup4_column_batches(env):
    """The natural-order LDE in batches of 3 columns (several batches per trace, the shared inverse
    transform's buffer reused across them), and the unshared two-pass form: bytes equal the oracle's.
    Both switches are read once per process, hence the child process."""
    import hashlib, os, subprocess, sys
    m, prep, tr, pv = W.deg5_shard(1 << 14, 5)
    rc, ref = O.OracleProver(m, prep, num_queries=42, log_blowup=2).prove(tr, pv)
    assert rc == 0
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", _BATCHED], cwd=root, env={**os.environ, **env},
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    assert out.stdout.split()[-1] == hashlib.sha256(ref).hexdigest()
