"""Twirp ProverService (zkmips_amd/service.py; the reference's api.proto:5-13 and its client,
crates/cuda/src/lib.rs:157-206): protobuf / JSON transport, Twirp routes and errors, the Ready poll
the client runs, and (GPU) a shard proven through the service equal to the direct prover's bytes."""
import base64
import http.client
import json
import threading

import numpy as np
import pytest

from zkmips_amd import service as SV
from zkmips_amd import workloads as W


@pytest.fixture
def server():
    def start(device_factory=None):
        svc = SV.ProverService(device_factory=device_factory)
        srv = SV.serve("127.0.0.1", 0, service=svc)
        th = threading.Thread(target=srv.serve_forever, daemon=True)
        th.start()
        started.append(srv)
        return srv.server_address[1]
    started = []
    yield start
    for s in started:
        s.shutdown()
        s.server_close()


def post(port, method, body, ctype="application/protobuf"):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=120)
    c.request("POST", SV.PREFIX + method, body=body, headers={"Content-Type": ctype})
    r = c.getresponse()
    out = r.status, r.getheader("Content-Type"), r.read()
    c.close()
    return out


def test_protobuf_wire_format_roundtrip():
    for data in (b"", b"x", bytes(range(256)) * 3, b"\0" * 300):
        enc = SV.encode_bytes_field(1, data)
        assert SV.decode_fields(enc).get(1, b"") == data
    assert SV.encode_bool_field(1, True) == b"\x08\x01" and SV.encode_bool_field(1, False) == b""
    assert SV.decode_fields(b"\x08\x01") == {1: 1}
    with pytest.raises(ValueError):
        SV.decode_fields(b"\x0a\x05ab")  # truncated bytes field


def test_ready_and_routes(server):
    port = server(device_factory=lambda i: object())
    st, ct, body = post(port, "Ready", b"")
    assert st == 200 and ct == "application/protobuf" and SV.decode_fields(body) == {1: 1}
    st, ct, body = post(port, "Ready", b"{}", "application/json")
    assert st == 200 and json.loads(body) == {"ready": True}
    for m in ("Setup", "ProveCore", "ProveCoreStateless", "Shrink", "Wrap"):
        st, ct, body = post(port, m, SV.encode_bytes_field(1, b"payload"))
        assert st == 501 and json.loads(body)["code"] == "unimplemented", m
    st, ct, body = post(port, "Compress", SV.encode_bytes_field(1, b"payload"))  # not a bincode payload
    assert st == 400 and json.loads(body)["code"] == "invalid_argument"
    st, _, body = post(port, "NoSuchMethod", b"")
    assert st == 404 and json.loads(body)["code"] == "bad_route"
    st, _, body = post(port, "Ready", b"", "text/plain")
    assert st == 404 and json.loads(body)["code"] == "bad_route"
    st, _, body = post(port, "ProveShard", SV.encode_bytes_field(1, b"not an npz"))
    assert st == 400 and json.loads(body)["code"] == "invalid_argument"


def test_not_ready_without_device(server):
    def no_device(i):
        raise RuntimeError("no gfx950 device")
    port = server(device_factory=no_device)
    st, _, body = post(port, "Ready", b"")
    assert st == 200 and SV.decode_fields(body) == {}  # ready = false is the proto3 default: omitted


def test_shard_payload_roundtrip():
    m, prep, tr, pv = W.fib_shard(1 << 6, 3)
    data = SV.pack_shard(m.blob(), prep, tr, pv, num_queries=16)
    blob, p2, t2, pv2, nq, lb, pc = SV.unpack_shard(data)
    assert np.array_equal(blob, m.blob()) and np.array_equal(pv2, pv) and nq == 16 and lb == 1 and pc == m.pc_start
    assert set(t2) == set(tr) and all(np.array_equal(t2[k], tr[k]) for k in tr)
    assert set(p2) == {k for k, v in prep.items() if v is not None}


@pytest.mark.gpu
def test_prove_shard_through_service(server):
    from zkmips_amd._lib import Device
    from zkmips_amd.prover import HipProver
    port = server()
    st, _, body = post(port, "Ready", b"")
    assert st == 200 and SV.decode_fields(body) == {1: 1}
    m, prep, tr, pv = W.fib_shard(1 << 10, 3)
    direct = HipProver(Device(0), m, prep, num_queries=16).prove_shard(tr, pv)
    data = SV.pack_shard(m.blob(), prep, tr, pv, num_queries=16)
    st, ct, body = post(port, "ProveShard", SV.encode_bytes_field(1, data))
    assert st == 200 and SV.decode_fields(body)[1] == direct
    st, ct, body = post(port, "ProveShard", json.dumps({"data": base64.b64encode(data).decode()}).encode(),
                        "application/json")
    assert st == 200 and base64.b64decode(json.loads(body)["result"]) == direct


@pytest.mark.gpu
def test_prove_compress_shard_through_service(server):
    """A recursion-machine (compress) shard at blowup 4 / 42 queries through ProveShard equals the
    direct prover's bytes and the CPU oracle's."""
    from tests import _oracle as O
    from zkmips_amd import recursion as R
    port = server()
    m, prep, tr, pv = R.shard(R.program_merkle_openings(6, 21, 8)[0])
    data = SV.pack_shard(m.blob(), prep, tr, pv, num_queries=R.COMPRESS_NUM_QUERIES, log_blowup=R.COMPRESS_LOG_BLOWUP,
                         pc_start=m.pc_start)
    st, ct, body = post(port, "ProveShard", SV.encode_bytes_field(1, data))
    assert st == 200
    rc, ref = O.OracleProver(m, prep, num_queries=R.COMPRESS_NUM_QUERIES, log_blowup=R.COMPRESS_LOG_BLOWUP).prove(tr, pv)
    assert rc == 0 and SV.decode_fields(body)[1] == ref


class _FakeProver:
    def __init__(self, blob, prep, nq, lb):
        self.key = SV.prover_key(blob, prep, nq, lb)

    def prove_shard(self, traces, pv):
        return self.key


def test_prover_cache_keyed_on_preprocessed_traces():
    """Two programs of one machine (same blob, different preprocessed traces) get two proving keys;
    the same program is set up once; the cache is LRU-bounded; a failed setup is not cached."""
    svc = SV.ProverService(device_factory=lambda i: object(), max_provers=2,
                           prover_factory=lambda d, b, p, nq, lb: _FakeProver(b, p, nq, lb))
    m, prep, tr, pv = W.fib_shard(1 << 6, 3)
    prep2 = {k: (None if v is None else (v + 1) % 0x7F000001) for k, v in prep.items()}
    a = svc.prove_shard(SV.pack_shard(m.blob(), prep, tr, pv, num_queries=16))
    b = svc.prove_shard(SV.pack_shard(m.blob(), prep2, tr, pv, num_queries=16))
    assert a != b and svc.setups == 2
    assert svc.prove_shard(SV.pack_shard(m.blob(), prep, tr, pv, num_queries=16)) == a and svc.setups == 2
    c = svc.prove_shard(SV.pack_shard(m.blob(), prep, tr, pv, num_queries=8))  # FRI parameters are in the key
    assert c not in (a, b) and svc.setups == 3 and len(svc._provers) == 2
    svc.prove_shard(SV.pack_shard(m.blob(), prep2, tr, pv, num_queries=16))  # evicted (LRU) -> set up again
    assert svc.setups == 4

    def boom(*_):
        raise RuntimeError("setup failed")
    bad = SV.ProverService(device_factory=lambda i: object(), prover_factory=boom)
    with pytest.raises(RuntimeError):
        bad.prove_shard(SV.pack_shard(m.blob(), prep, tr, pv, num_queries=16))
    assert bad.setups == 0 and not bad._pending


def test_ready_not_blocked_by_a_setup(server):
    """A slow setup (e.g. first-time hiprtc compilation) does not block the client's Ready polls."""
    gate = threading.Event()

    def slow(d, b, p, nq, lb):
        gate.wait(30)
        return _FakeProver(b, p, nq, lb)
    svc = SV.ProverService(device_factory=lambda i: object(), prover_factory=slow)
    srv = SV.serve("127.0.0.1", 0, service=svc)
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    port = srv.server_address[1]
    try:
        m, prep, tr, pv = W.fib_shard(1 << 6, 3)
        data = SV.pack_shard(m.blob(), prep, tr, pv, num_queries=16)
        res = {}
        t = threading.Thread(target=lambda: res.setdefault("r", post(port, "ProveShard", SV.encode_bytes_field(1, data))))
        t.start()
        st, _, body = post(port, "Ready", b"")
        assert st == 200 and SV.decode_fields(body) == {1: 1} and not gate.is_set()
        gate.set()
        t.join(60)
        assert res["r"][0] == 200
    finally:
        gate.set()
        srv.shutdown()
        srv.server_close()


@pytest.mark.gpu
def test_two_compress_programs_through_one_server(server):
    """two recursion programs of the same machine sent to one server each prove against
    their own preprocessed commitment (equal to a direct HipProver's bytes and the oracle's)."""
    from tests import _oracle as O
    from zkmips_amd import recursion as R
    from zkmips_amd._lib import Device
    from zkmips_amd.prover import HipProver
    port = server()
    blobs = []
    for seed in (21, 22):
        m, prep, tr, pv = R.shard(R.program_merkle_openings(6, 21, 8, seed=seed)[0])
        blobs.append(m.blob().tobytes())
        data = SV.pack_shard(m.blob(), prep, tr, pv, num_queries=R.COMPRESS_NUM_QUERIES,
                             log_blowup=R.COMPRESS_LOG_BLOWUP, pc_start=m.pc_start)
        st, _, body = post(port, "ProveShard", SV.encode_bytes_field(1, data))
        assert st == 200, body
        direct = HipProver(Device(0), m, prep, num_queries=R.COMPRESS_NUM_QUERIES,
                           log_blowup=R.COMPRESS_LOG_BLOWUP).prove_shard(tr, pv)
        rc, ref = O.OracleProver(m, prep, num_queries=R.COMPRESS_NUM_QUERIES,
                                 log_blowup=R.COMPRESS_LOG_BLOWUP).prove(tr, pv)
        assert rc == 0 and SV.decode_fields(body)[1] == direct == ref
    assert blobs[0] == blobs[1]  # one machine, two programs


@pytest.mark.gpu
def test_compress_two_mips_shards_through_service(server):
    """Compress (lib.rs:92-102): the two shard proofs of a whole MIPS execution (a CPU shard in the reference's
    2^22 shape scaled to Cpu 2^16 and the memory shard, 84 queries) sent as a bincode CompressRequestPayload
    come back as a ZKMReduceProof whose proof is the complete root node proof a direct HipProver makes from the
    same children, the oracle verifies it, and its vk is that node program's StarkVerifyingKey."""
    from tests import _oracle as O
    from zkmips_amd import bincode as B
    from zkmips_amd import compress_tree as CT
    from zkmips_amd import recursion as R
    from zkmips_amd import recursion_verifier as RV
    from zkmips_amd import shapes as SH
    from zkmips_amd._lib import Device
    from zkmips_amd.prover import HipProver
    from zkmips_amd.septic import CURVE_CUMULATIVE_SUM_START as GCS
    dev = Device(0)
    sh = SH.shape_execution(SH.MAXIMAL_22, 1, down=6)
    assert len(sh) == 2
    m, prep = sh[0][0], sh[0][1]
    hp = HipProver(dev, m, prep, num_queries=84)
    proofs = [hp.prove_shard(s[2], s[3]) for s in sh]
    req = B.write_compress_request(B.StarkVk.of_program(m, prep, hp.vk_commit, 0x00400000, GCS), proofs)
    port = server()
    st, _, body = post(port, "Compress", SV.encode_bytes_field(1, req))
    assert st == 200, body
    rvk, rproof = B.read_reduce_proof(SV.decode_fields(body)[1])
    vk = RV.ChildVk.of(m, prep, hp.vk_commit, num_queries=84)
    cprep, tr, pv, shape, _ = CT.node_witness([(vk, p) for p in proofs], is_first=True, is_complete=True)
    assert int(pv[220]) == 1  # RecursionPublicValues.is_complete
    cm = R.compress_machine()
    kw = dict(num_queries=R.COMPRESS_NUM_QUERIES, log_blowup=R.COMPRESS_LOG_BLOWUP)
    direct = HipProver(dev, cm, cprep, **kw)
    assert rproof == direct.prove_shard(tr, pv)
    assert O.OracleProver(cm, cprep, **kw).verify(rproof) == 0
    assert rvk.commit == [int(x) for x in direct.vk_commit]
    assert {c[0]: c[1] for c in rvk.chips} == {k: shape[k] for k in rvk.ordering}


@pytest.mark.gpu
def test_compress_with_a_deferred_proof_through_service(server):
    """Compress with `deferred_proofs` (crates/cuda/src/lib.rs:98-106, prover/src/lib.rs:551-612): execution A
    compressed through the service is the deferred proof of execution B, whose guest committed A's deferred
    digest.  The request comes back as a complete root whose end reconstruct-deferred digest is that digest; the
    deferred node (machine/deferred.rs) at its RecursionShapeConfig shape proves to the oracle's bytes on the GPU
    and the oracle verifies it; a request whose deferred proof is not the committed one is refused."""
    from tests import _oracle as O
    from zkmips_amd import bincode as B
    from zkmips_amd import compress_tree as CT
    from zkmips_amd import mips_core as MC
    from zkmips_amd import node_pv as NP
    from zkmips_amd import recursion as R
    from zkmips_amd import recursion_verifier as RV
    from zkmips_amd import shapes as SH
    from zkmips_amd._lib import Device
    from zkmips_amd.prover import HipProver
    from zkmips_amd.septic import CURVE_CUMULATIVE_SUM_START as GCS
    dev = Device(0)
    port = server()
    sh = SH.shape_execution(SH.MAXIMAL_22, 1, down=6)
    m, prep = sh[0][0], sh[0][1]
    hp = HipProver(dev, m, prep, num_queries=84)
    proofs = [hp.prove_shard(s[2], s[3]) for s in sh]
    st, _, body = post(port, "Compress", SV.encode_bytes_field(1, B.write_compress_request(
        B.StarkVk.of_program(m, prep, hp.vk_commit, MC.PC_BASE, GCS), proofs)))
    assert st == 200, body
    a_vk, a_proof = B.read_reduce_proof(SV.decode_fields(body)[1])
    pv_a = RV.parse_shard_proof(a_proof).pv
    d = NP.hash_deferred_proofs(np.zeros(8, np.int64), [pv_a])
    run = MC.program_shards(MC.deferred_commit_program(d), seed=9, shard_size=1 << 10)
    mb, prepb = run[0][0], run[0][1]
    hb = HipProver(dev, mb, prepb, num_queries=84)
    proofs_b = [hb.prove_shard(s[2], s[3]) for s in run]
    svk_b = B.StarkVk.of_program(mb, prepb, hb.vk_commit, MC.PC_BASE, GCS)
    req = B.write_compress_request(svk_b, proofs_b, deferred=[(a_vk, a_proof)])
    assert B.read_compress_request(req, with_deferred=True)[2] == [(a_vk, a_proof)]
    st, _, body = post(port, "Compress", SV.encode_bytes_field(1, req))
    assert st == 200, body
    rvk, rproof = B.read_reduce_proof(SV.decode_fields(body)[1])
    pv = RV.parse_shard_proof(rproof).pv
    assert int(pv[NP.R_IS_COMPLETE]) == 1 and int(pv[NP.R_CONTAINS_EXEC]) == 1
    assert [int(x) for x in pv[NP.R_END_RECON:NP.R_END_RECON + 8]] == [int(x) for x in d]
    # the deferred node at its reference shape: GPU bytes == oracle bytes, verified
    vk_b = SV.core_child_vk(svk_b)
    h = NP.DeferredHints.of(vk_b, RV.parse_shard_proof(proofs_b[-1]).pv, np.zeros(8, np.int64))
    cprep, tr, dpv, shape, _ = CT.node_witness([(SV.deferred_child_vk(a_vk), a_proof)], deferred=h)
    assert shape in R.RECURSION_SHAPES and int(dpv[NP.R_CONTAINS_EXEC]) == 0
    cm = R.compress_machine()
    kw = dict(num_queries=R.COMPRESS_NUM_QUERIES, log_blowup=R.COMPRESS_LOG_BLOWUP)
    got = HipProver(dev, cm, cprep, **kw).prove_shard(tr, dpv)
    ov = O.OracleProver(cm, cprep, **kw)
    rc, ref = ov.prove(tr, dpv)
    assert rc == 0 and got == ref and ov.verify(got) == 0
    # B's guest committed A's digest: another deferred proof (B's own root would be incomplete; use A twice)
    bad = B.write_compress_request(svk_b, proofs_b, deferred=[(a_vk, a_proof), (a_vk, a_proof)])
    st, _, body = post(port, "Compress", SV.encode_bytes_field(1, bad))
    assert st == 400 and json.loads(body)["code"] == "invalid_argument"
