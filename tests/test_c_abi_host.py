"""A native (non-Python) host drives the C ABI: examples/prove_shard.c reads a machine blob and raw
u32 traces from files and calls zkm_init / zkm_setup / zkm_pk_observe / zkm_prove_shard, as a Rust
shim would.  Its proof must equal the Python binding's and the oracle's."""
import os
import subprocess

import numpy as np
import pytest

from tests import _oracle as O
from zkmips_amd import mips_alu as A
from zkmips_amd import workloads as W

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "examples", "prove_shard")


def write_manifest(tmp, m, prep, traces, pvs, queries):
    lines = []
    blob = tmp / "machine.u32"
    m.blob().astype("<u4").tofile(blob)
    lines.append(f"blob {blob}")
    lines.append(f"queries {queries}")
    for kind, mats in (("prep", prep), ("trace", traces)):
        for name, t in mats.items():
            p = tmp / f"{kind}_{name}.u32"
            np.ascontiguousarray(t, dtype="<u4").tofile(p)
            lines.append(f"{kind} {name} {t.shape[0]} {t.shape[1]} {p}")
    pv = tmp / "pv.u32"
    np.asarray(pvs, dtype="<u4").tofile(pv)
    lines.append(f"pv {len(pvs)} {pv}")
    out = tmp / "proof.bin"
    lines.append(f"out {out}")
    man = tmp / "manifest.txt"
    man.write_text("\n".join(lines) + "\n")
    return man, out


def test_native_host_builds_and_rejects_bad_usage(tmp_path):
    assert os.access(EXE, os.X_OK), "examples/prove_shard not built (__graft_entry__.build)"
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "usage" in r.stderr
    bad = tmp_path / "m.txt"
    bad.write_text("nonsense 1\n")
    r = subprocess.run([EXE, str(bad)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "unknown manifest key" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("workload", ["fib", "alu"])
def test_native_host_proof_matches(tmp_path, workload):
    from zkmips_amd._lib import Device
    from zkmips_amd.prover import HipProver
    if workload == "fib":
        m, prep, traces, pvs = W.fib_shard(1 << 10, 3)
    else:
        m, prep, traces, pvs = A.alu_shard(300, 200, seed=4, n_lt=100, n_sll=50, n_sr=60, n_clz=30)
    man, out = write_manifest(tmp_path, m, prep, traces, pvs, 16)
    r = subprocess.run([EXE, str(man)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    native = out.read_bytes()
    dev = Device(0)
    py = HipProver(dev, m, prep, num_queries=16).prove_shard(traces, pvs)
    cpu = O.OracleProver(m, prep, num_queries=16)
    rc, ref = cpu.prove(traces, pvs)
    assert rc == 0 and native == py == ref
    assert cpu.verify(native) == 0
