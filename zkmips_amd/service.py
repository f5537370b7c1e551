"""Twirp `ProverService` server: the out-of-process GPU seam of the reference.

The reference's `CudaProver` talks Twirp to a closed GPU server image (crates/cuda/proto/api.proto:5-13,
client crates/cuda/src/lib.rs:157-206; endpoint `CUDA_ENDPOINT`, default
http://localhost:3000/twirp/).  This is that server's transport on MI355X: Twirp over HTTP/1.1
(`POST /twirp/api.ProverService/<Method>`, protobuf or JSON bodies, Twirp JSON errors), the message
types of api.proto (every request/response is one `bytes` field, or `bool ready`), and the methods:

* ``Ready``    — ready = the HIP library loaded and a gfx950 device initialised (the client polls this
                 for up to 300 s, lib.rs:183-205).
* ``ProveShard`` (an extension, not in api.proto) — one shard through zkm_prove_shard: `data` is an
                 .npz archive (numpy, no pickles) with `machine_blob`, `public_values`, `num_queries`,
                 optional `log_blowup`, and `prep/<chip>` / `trace/<chip>` arrays; `result` is the
                 serialized ShardProof.  A prover per (machine blob, FRI parameters, preprocessed
                 traces) is kept, LRU-bounded (setup once per program).
* ``Compress`` — `data` is a bincode CompressRequestPayload (lib.rs:92-102: the core verifying key, the
                 ZKMCoreProof's shard proofs, deferred proofs), `result` a bincode ZKMReduceProof (the
                 root compress proof and its StarkVerifyingKey, zkmips_amd/bincode.py).  The shard
                 proofs are the leaves of the compress tree (zkmips_amd/compress_tree.py): node
                 programs verifying their children in full, padded to a RecursionShapeConfig shape,
                 set up and proven on the GPU; a single shard is still wrapped by one node.  Deferred
                 proofs are `unimplemented`.
* ``Setup``, ``ProveCore``, ``ProveCoreStateless``, ``Shrink``, ``Wrap`` — Twirp `unimplemented`: their
                 payloads are bincode `ZKMStdin` / ELF (lib.rs:57-90) or the shrink / BN254 wrap
                 stages (lib.rs:104-116), outside the §8 rows.

Run: ``python -m zkmips_amd.service --port 3000`` (then CUDA_ENDPOINT=http://<host>:3000/twirp/).
"""
from __future__ import annotations

import argparse
import io
import json
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Callable, Dict, Optional, Tuple

import numpy as np

PREFIX = "/twirp/api.ProverService/"
ALL_METHODS = ("Setup", "Ready", "ProveCore", "ProveCoreStateless", "Compress", "Shrink", "Wrap", "ProveShard")
UNIMPLEMENTED = {
    "Setup": "needs the ELF loader and executor (SetupRequestPayload { elf }, crates/cuda/src/lib.rs:60-71)",
    "ProveCore": "needs the MIPS executor to turn ZKMStdin into shard records (lib.rs:73-79)",
    "ProveCoreStateless": "needs the MIPS executor to turn ZKMStdin into shard records (lib.rs:81-90)",
    "Shrink": "recursion shrink is outside this server (lib.rs:104-109)",
    "Wrap": "the BN254 wrap is outside this server (lib.rs:111-116)",
}


# ---------------------------------------------------------------- protobuf wire format (api.proto)
def _varint(n: int) -> bytes:
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        out.append(b | (0x80 if n else 0))
        if not n:
            return bytes(out)


def _read_varint(buf: bytes, i: int) -> Tuple[int, int]:
    n = shift = 0
    while True:
        if i >= len(buf):
            raise ValueError("truncated varint")
        b = buf[i]
        i += 1
        n |= (b & 0x7F) << shift
        shift += 7
        if not b & 0x80:
            return n, i
        if shift > 63:
            raise ValueError("varint too long")


def decode_fields(buf: bytes) -> Dict[int, object]:
    """Field number -> value (bytes for length-delimited, int for varint); unknown fields kept."""
    out: Dict[int, object] = {}
    i = 0
    while i < len(buf):
        key, i = _read_varint(buf, i)
        field, wire = key >> 3, key & 7
        if wire == 0:
            out[field], i = _read_varint(buf, i)
        elif wire == 2:
            n, i = _read_varint(buf, i)
            if i + n > len(buf):
                raise ValueError("truncated field")
            out[field] = buf[i:i + n]
            i += n
        elif wire == 1:
            out[field] = buf[i:i + 8]
            i += 8
        elif wire == 5:
            out[field] = buf[i:i + 4]
            i += 4
        else:
            raise ValueError(f"unsupported wire type {wire}")
    return out


def encode_bytes_field(field: int, data: bytes) -> bytes:
    return _varint((field << 3) | 2) + _varint(len(data)) + data if data else b""


def encode_bool_field(field: int, v: bool) -> bytes:
    return _varint(field << 3) + _varint(1) if v else b""  # proto3: default values are omitted


# ---------------------------------------------------------------- shard payloads (ProveShard)
def pack_shard(machine_blob, prep: dict, traces: dict, public_values, num_queries: int = 84,
               log_blowup: int = 1, pc_start: int = 0x00400000) -> bytes:
    """A ProveShard payload (npz): the machine blob, FRI parameters, the programs' pc_start (MachineDesc.pc_start:
    0 for recursion programs), preprocessed and main traces, public values."""
    arrs = {"machine_blob": np.asarray(machine_blob, np.uint32), "public_values": np.asarray(public_values, np.uint32),
            "num_queries": np.asarray([num_queries], np.uint32), "log_blowup": np.asarray([log_blowup], np.uint32),
            "pc_start": np.asarray([pc_start], np.uint32)}
    for k, v in prep.items():
        if v is not None:
            arrs[f"prep/{k}"] = np.asarray(v, np.uint32)
    for k, v in traces.items():
        arrs[f"trace/{k}"] = np.asarray(v, np.uint32)
    b = io.BytesIO()
    np.savez(b, **arrs)
    return b.getvalue()


def unpack_shard(data: bytes):
    with np.load(io.BytesIO(data), allow_pickle=False) as z:
        files = {k: z[k] for k in z.files}
    blob = files.pop("machine_blob")
    pv = files.pop("public_values")
    nq = int(files.pop("num_queries")[0])
    lb = int(files.pop("log_blowup", np.asarray([1]))[0])
    pc = int(files.pop("pc_start", np.asarray([0x00400000]))[0])
    prep = {k[5:]: v for k, v in files.items() if k.startswith("prep/")}
    traces = {k[6:]: v for k, v in files.items() if k.startswith("trace/")}
    return blob, prep, traces, pv, nq, lb, pc


class TwirpError(Exception):
    STATUS = {"invalid_argument": 400, "malformed": 400, "not_found": 404, "bad_route": 404,
              "unimplemented": 501, "internal": 500, "unavailable": 503}

    def __init__(self, code: str, msg: str):
        super().__init__(msg)
        self.code, self.msg = code, msg


def prover_key(blob, prep: dict, num_queries: int, log_blowup: int, pc_start: int = 0x00400000) -> bytes:
    """Identity of a proving key: the machine blob, the FRI parameters AND the preprocessed traces.
    A recursion (compress) program lives in its chips' preprocessed columns, so two programs of one
    machine need two keys (the reference sets each compress program up anew, prover/src/lib.rs:807)."""
    import hashlib
    h = hashlib.sha256()
    h.update(np.asarray(blob, np.uint32).tobytes())
    h.update(np.asarray([num_queries, log_blowup] + ([pc_start] if pc_start != 0x00400000 else []),
                        np.uint64).tobytes())
    for name in sorted(k for k, v in prep.items() if v is not None):
        a = np.ascontiguousarray(np.asarray(prep[name], np.uint32))
        h.update(name.encode() + b"\0" + np.asarray(a.shape, np.uint64).tobytes())
        h.update(a.tobytes())
    return h.digest()


def core_child_vk(vk):
    """The ChildVk a compress node verifies a core shard proof against, from the request's
    StarkVerifyingKey<CoreSC>: the MIPS machine's chips (zkmips_amd/mips_core.py), the key's preprocessed
    commitment, heights, order, pc_start and initial global cumulative sum; core FRI parameters (84
    queries, blowup 2, 16 PoW bits).  A chip the MIPS machine does not preprocess, or a width that is not
    the chip's, is a ValueError."""
    from . import mips_core as MC
    from . import recursion_verifier as RV
    m = MC.core_machine()
    chips = {c.name: c for c in m.chips}
    heights = {}
    for name, log_n, shift, width, height in vk.chips:
        c = chips.get(name)
        if c is None or not c.prep_width:
            raise ValueError(f"chip {name!r} has no preprocessed trace in the MIPS machine")
        if width != c.prep_width or height != 1 << log_n or shift != 1:
            raise ValueError(f"chip {name!r}: preprocessed dimensions {width}x{height} (log_n {log_n}, "
                             f"shift {shift}) are not the machine's")
        heights[name] = height
    order = sorted(heights, key=lambda k: (-heights[k], k))
    if vk.ordering and sorted(vk.ordering, key=lambda k: vk.ordering[k]) != order:
        raise ValueError("chip_ordering is not the preprocessed order")
    return RV.ChildVk({k: RV.ChipShape.of(c) for k, c in chips.items()}, m.num_pv, np.asarray(vk.commit, np.int64),
                      order, heights, int(vk.pc_start), np.asarray(vk.gcs, np.int64))


def deferred_child_vk(vk):
    """The ChildVk of a deferred proof (ZKMReduceProof<InnerSC>.vk, a compress program's StarkVerifyingKey): the
    compress machine's chips, the key's commitment and preprocessed heights, compress FRI parameters.  A chip the
    compress machine does not preprocess, or a dimension that is not the chip's, is a ValueError."""
    from . import compress_tree as CT
    from . import recursion as R
    from .septic import CURVE_CUMULATIVE_SUM_START
    chips = {c.name: c for c in R.compress_machine().chips}
    shape = {}
    for name, log_n, shift, width, height in vk.chips:
        c = chips.get(name)
        if c is None or not c.prep_width:
            raise ValueError(f"deferred proof: chip {name!r} has no preprocessed trace in the compress machine")
        if width != c.prep_width or height != 1 << log_n or shift != 1:
            raise ValueError(f"deferred proof: chip {name!r} preprocessed dimensions are not the machine's")
        shape[name] = int(log_n)
    if sorted(shape) != sorted(k for k, c in chips.items() if c.prep_width):
        raise ValueError("deferred proof: not a compress program's verifying key")
    if int(vk.pc_start) != R.compress_machine().pc_start or \
            [int(x) for x in vk.gcs] != [int(x) for x in CURVE_CUMULATIVE_SUM_START]:
        raise ValueError("deferred proof: a compress vk has pc_start 0 and the zero initial global sum")
    return CT.compress_child_vk(vk.commit, shape)


def reduce_vk(cvk):
    """StarkVerifyingKey<InnerSC> of a compress proof's program (the vk field of ZKMReduceProof)."""
    from . import bincode as B
    from . import recursion as R
    widths = {c.name: c.prep_width for c in R.compress_machine().chips}
    chips = [(k, cvk.prep_heights[k].bit_length() - 1, 1, widths[k], cvk.prep_heights[k]) for k in cvk.prep_order]
    return B.StarkVk([int(x) for x in cvk.commit], int(cvk.pc_start), [int(x) for x in cvk.gcs], chips,
                     {k: i for i, k in enumerate(cvk.prep_order)})


class _Pending:
    """A proving key being set up: requests for the same key wait on it, others go ahead."""

    def __init__(self):
        self.done = threading.Event()
        self.prover = None
        self.error: Optional[BaseException] = None


class ProverService:
    """The method implementations; transport-independent (the HTTP handler below calls `call`).

    Proving keys are cached per `prover_key` (machine, FRI parameters, preprocessed traces), at most
    `max_provers` of them (least recently used evicted; each holds a device LDE + Merkle tree).  A key
    is built outside the cache lock, so `Ready` polls and requests for other keys are not serialised
    behind one setup (which may include minutes of first-time hiprtc compilation)."""

    def __init__(self, device: int = 0, device_factory: Optional[Callable] = None,
                 prover_factory: Optional[Callable] = None, max_provers: int = 8, compress_workers: int = 0,
                 compress_inflight: int = 2):
        from collections import OrderedDict
        self.device_index = device
        self._device_factory = device_factory
        self._prover_factory = prover_factory
        self.max_provers = max(1, max_provers)
        self._dev = None
        self._provers: "OrderedDict[bytes, object]" = OrderedDict()
        self._pending: Dict[bytes, _Pending] = {}
        self._dev_lock = threading.Lock()
        self._lock = threading.Lock()
        self.setups = 0  # proving keys built (tests check the cache behaviour)
        # compress: node witnesses in a spawn process pool started here, before this process touches the
        # GPU (0 workers: a thread pool), node proofs in `compress_inflight` threads
        self._pool = None
        if compress_workers > 0:
            from .compress_tree import AffinityPool
            self._pool = AffinityPool(compress_workers).warm()
        self.compress_inflight = compress_inflight
        self._compress_provers = None

    def _device(self):
        with self._dev_lock:
            if self._dev is None:
                if self._device_factory is not None:
                    self._dev = self._device_factory(self.device_index)
                else:
                    from ._lib import Device
                    self._dev = Device(self.device_index)
            return self._dev

    def _build(self, dev, blob, prep, nq, lb, pc_start=0x00400000):
        if self._prover_factory is not None:
            return self._prover_factory(dev, blob, prep, nq, lb)
        from .prover import HipProver
        return HipProver.from_blob(dev, blob, prep, num_queries=nq, log_blowup=lb, pc_start=pc_start)

    def get_prover(self, blob, prep: dict, nq: int, lb: int, pc_start: int = 0x00400000):
        """The cached prover of (blob, prep, nq, lb, pc_start), set up on first use."""
        key = prover_key(blob, prep, nq, lb, pc_start)
        dev = self._device()
        with self._lock:
            p = self._provers.get(key)
            if p is not None:
                self._provers.move_to_end(key)
                return p
            pend = self._pending.get(key)
            owner = pend is None
            if owner:
                pend = self._pending[key] = _Pending()
        if not owner:
            pend.done.wait()
            if pend.error is not None:
                raise pend.error
            return pend.prover
        try:
            pend.prover = self._build(dev, blob, prep, nq, lb, pc_start)
        except BaseException as e:
            pend.error = e
            raise
        finally:
            with self._lock:
                self._pending.pop(key, None)
                if pend.prover is not None:
                    self.setups += 1
                    self._provers[key] = pend.prover
                    while len(self._provers) > self.max_provers:
                        self._provers.popitem(last=False)
            pend.done.set()
        return pend.prover

    def ready(self) -> bool:
        try:
            self._device()
            return True
        except Exception:
            return False

    def prove_shard(self, data: bytes) -> bytes:
        try:
            blob, prep, traces, pv, nq, lb, pc = unpack_shard(data)
        except Exception as e:
            raise TwirpError("invalid_argument", f"ProveShard payload: {e}")
        return self.get_prover(blob, prep, nq, lb, pc).prove_shard(traces, pv)

    def compress(self, data: bytes) -> bytes:
        """CompressRequestPayload -> ZKMReduceProof (prover/src/lib.rs:614-954 on the GPU).  The shards must be
        one whole execution in order: the node programs check what the reference's recursion programs check
        (zkmips_amd/node_pv.py: consecutive shard numbers and pcs, address bits, digests, exit code, the
        first-shard conditions, the child vks' membership in the dummy vk tree) and the root asserts the
        proof complete (start shard 1, next_pc 0, global sum zero); a request that fails them answers
        invalid_argument before any GPU work.  Deferred proofs (complete compress proofs of other executions) are
        verified by deferred nodes chained after the execution's (CT.reduce_with_deferred, lib.rs:551-604).  Not
        supported: the real vk map (`vk_map.bin` is absent from the reference snapshot; the dummy map's tree is
        used, as VERIFY_VK=false does)."""
        from . import bincode as B
        from . import compress_tree as CT
        try:
            vk, shards, deferred = B.read_compress_request(data, with_deferred=True)
        except Exception as e:
            raise TwirpError("invalid_argument", f"Compress: payload: {e}")
        if not shards:
            raise TwirpError("invalid_argument", "Compress: the core proof has no shards")
        try:
            cvk = core_child_vk(vk)
            dleaves = [(deferred_child_vk(dvk), dp) for dvk, dp in deferred]
        except ValueError as e:
            raise TwirpError("invalid_argument", f"Compress: {e}")
        leaves = [(cvk, s) for s in shards]
        dev = self._device()
        with self._lock:
            if self._compress_provers is None:
                self._compress_provers = CT.GpuProvers(dev)
        provers, stats = self._compress_provers, CT.TreeStats()

        def prove(wit):
            prep, traces, pvs, shape, _ = wit
            pr = provers.get(prep, stats)
            proof = pr.prove_shard(CT.materialize(traces), pvs)
            return CT.compress_child_vk(pr.vk_commit, shape), proof

        if self._pool is not None:
            # one dedup session per request: a worker resends a program's prep traces to each request
            # (a failed or concurrent request never leaves another depending on traces it consumed)
            sid = CT.new_session()
            submit = lambda ch, fl: self._pool.submit(CT.node_witness_shm, CT.by_ref(ch), True, True, True,
                                                      session=sid, **fl, tag=CT.node_tag(ch))
        else:
            from concurrent.futures import ThreadPoolExecutor
            tp = ThreadPoolExecutor(2)
            # threads of this process: no once-per-program prep (arrival order is not completion order)
            submit = lambda ch, fl: tp.submit(CT.node_witness, ch, True, True, True, False, **fl)
        try:
            if dleaves:
                rvk, rproof = CT.reduce_with_deferred(leaves, dleaves, submit, prove, self.compress_inflight)
            elif len(leaves) == 1:  # one shard is still wrapped by a compress node
                rvk, rproof = prove(CT.register_prep(submit(leaves, {"is_first": True, "is_complete": True}).result()))
            else:
                rvk, rproof = CT.reduce_serial(leaves, CT.Reducer(submit, prove, self.compress_inflight))
        except ValueError as e:  # a child proof of the wrong shape for its verifying key
            raise TwirpError("invalid_argument", f"Compress: {e}")
        except RuntimeError as e:
            from ._lib import ZkmError
            if isinstance(e, ZkmError):  # the device side: Twirp internal
                raise
            # the node program's runtime check failed: a child proof that does not verify
            raise TwirpError("invalid_argument", f"Compress: a child proof does not verify ({e})")
        finally:
            if self._pool is None:
                tp.shutdown(wait=False)
            else:
                CT.release_session(sid)  # (the one-leaf path pins its program's key outside a Reducer)
        return B.write_reduce_proof(reduce_vk(rvk), rproof)

    def call(self, method: str, payload: Dict[int, object]) -> Dict[str, object]:
        if method == "Ready":
            return {"ready": self.ready()}
        if method == "ProveShard":
            data = payload.get(1, b"")
            return {"result": self.prove_shard(bytes(data))}
        if method == "Compress":
            return {"result": self.compress(bytes(payload.get(1, b"")))}
        if method in UNIMPLEMENTED:
            raise TwirpError("unimplemented", f"{method}: {UNIMPLEMENTED[method]}")
        raise TwirpError("bad_route", f"no such method: {method}")


def _handler(service: ProverService):
    class Handler(BaseHTTPRequestHandler):
        protocol_version = "HTTP/1.1"

        def log_message(self, fmt, *args):  # quiet
            pass

        def _send(self, status: int, ctype: str, body: bytes):
            self.send_response(status)
            self.send_header("Content-Type", ctype)
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def _error(self, e: TwirpError):
            self._send(TwirpError.STATUS.get(e.code, 500), "application/json",
                       json.dumps({"code": e.code, "msg": e.msg}).encode())

        def do_POST(self):
            n = int(self.headers.get("Content-Length") or 0)
            body = self.rfile.read(n) if n else b""
            if not self.path.startswith(PREFIX):
                return self._error(TwirpError("bad_route", f"no handler for path {self.path}"))
            method = self.path[len(PREFIX):]
            ctype = (self.headers.get("Content-Type") or "").split(";")[0].strip()
            try:
                if ctype == "application/protobuf":
                    payload = decode_fields(body)
                elif ctype == "application/json":
                    j = json.loads(body or b"{}")
                    payload = {1: __import__("base64").b64decode(j["data"])} if "data" in j else {}
                else:
                    raise TwirpError("bad_route", f"unexpected Content-Type: {ctype!r}")
            except TwirpError as e:
                return self._error(e)
            except Exception as e:
                return self._error(TwirpError("malformed", f"request body: {e}"))
            try:
                out = service.call(method, payload)
            except TwirpError as e:
                return self._error(e)
            except Exception as e:  # prover failure: Twirp internal with the library's message
                return self._error(TwirpError("internal", str(e)))
            if ctype == "application/protobuf":
                if "ready" in out:
                    resp = encode_bool_field(1, bool(out["ready"]))
                else:
                    resp = encode_bytes_field(1, out["result"])
                return self._send(200, "application/protobuf", resp)
            if "ready" in out:
                return self._send(200, "application/json", json.dumps({"ready": bool(out["ready"])}).encode())
            return self._send(200, "application/json", json.dumps(
                {"result": __import__("base64").b64encode(out["result"]).decode()}).encode())

        def do_GET(self):
            self._error(TwirpError("bad_route", "Twirp accepts POST only"))

    return Handler


def serve(host: str = "127.0.0.1", port: int = 3000, device: int = 0, service: ProverService = None):
    """A ThreadingHTTPServer for the service (caller runs serve_forever / shutdown)."""
    return ThreadingHTTPServer((host, port), _handler(service or ProverService(device)))


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=3000)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--compress-workers", type=int, default=8, help="witness processes of the Compress route")
    a = ap.parse_args()
    srv = serve(a.host, a.port, service=ProverService(a.device, compress_workers=a.compress_workers))
    print(f"ProverService on http://{a.host}:{a.port}/twirp/", flush=True)
    srv.serve_forever()


if __name__ == "__main__":
    main()
