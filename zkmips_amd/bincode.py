"""bincode-1 (fixint, little-endian) codecs of the reference's compress payloads, for the Twirp `Compress`
route (zkmips_amd/service.py; crates/cuda/src/lib.rs:92-102 CompressRequestPayload, the response a
ZKMReduceProof<InnerSC> crates/core/executor/src/reduce.rs:7-12).

Field elements are canonical u32 (the encoding that regenerates crates/prover/dummy_vk_map.bin, DESIGN.md
§3), usize / Vec / String lengths u64, fixed arrays without a length:

  StarkVerifyingKey (crates/stark/src/machine.rs:93-104)
      commit [F; 8], pc_start F, initial_global_cumulative_sum (x [F; 7], y [F; 7]),
      chip_information Vec<(String, TwoAdicMultiplicativeCoset { log_n usize, shift F },
                            Dimensions { width usize, height usize })>,
      chip_ordering HashMap<String, usize>
  ZKMCoreProof = ZKMProofWithMetadata<ZKMCoreProofData> (crates/prover/src/types.rs:114-140)
      proof Vec<ShardProof>, stdin ZKMStdin, public_values ZKMPublicValues, cycles u64
  CompressRequestPayload { vk ZKMVerifyingKey { vk StarkVerifyingKey }, proof ZKMCoreProof,
                           deferred_proofs Vec<ZKMReduceProof> }
  ZKMReduceProof { vk StarkVerifyingKey, proof ShardProof }
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import Dict, List, Sequence, Tuple

import numpy as np


class Reader:
    def __init__(self, b: bytes, pos: int = 0):
        self.b, self.pos = b, pos

    def u64(self) -> int:
        v = struct.unpack_from("<Q", self.b, self.pos)[0]
        self.pos += 8
        return v

    def u32(self) -> int:
        v = struct.unpack_from("<I", self.b, self.pos)[0]
        self.pos += 4
        return v

    def u32s(self, n: int) -> List[int]:
        v = list(struct.unpack_from(f"<{n}I", self.b, self.pos))
        self.pos += 4 * n
        return v

    def raw(self, n: int) -> bytes:
        if self.pos + n > len(self.b):
            raise ValueError("truncated bincode")
        v = self.b[self.pos:self.pos + n]
        self.pos += n
        return v

    def string(self) -> str:
        return self.raw(self.u64()).decode()


class Writer:
    def __init__(self):
        self.parts: List[bytes] = []

    def u64(self, v: int):
        self.parts.append(struct.pack("<Q", v))

    def u32s(self, vs):
        vs = [int(x) for x in vs]
        self.parts.append(struct.pack(f"<{len(vs)}I", *vs))

    def raw(self, b: bytes):
        self.parts.append(bytes(b))

    def string(self, s: str):
        e = s.encode()
        self.u64(len(e))
        self.raw(e)

    def bytes(self) -> bytes:
        return b"".join(self.parts)


@dataclass
class StarkVk:
    commit: List[int]
    pc_start: int
    gcs: List[int]                                   # 14 words: x then y
    chips: List[Tuple[str, int, int, int, int]]     # (name, log_n, shift, width, height)
    ordering: Dict[str, int] = field(default_factory=dict)

    @staticmethod
    def read(r: Reader) -> "StarkVk":
        commit, pc, gcs = r.u32s(8), r.u32(), r.u32s(14)
        chips = []
        for _ in range(r.u64()):
            name = r.string()
            log_n, shift = r.u64(), r.u32()
            width, height = r.u64(), r.u64()
            chips.append((name, log_n, shift, width, height))
        ordering = {}
        for _ in range(r.u64()):
            k = r.string()
            ordering[k] = r.u64()
        return StarkVk(commit, pc, gcs, chips, ordering)

    def write(self, w: Writer):
        w.u32s(self.commit)
        w.u32s([self.pc_start])
        w.u32s(self.gcs)
        w.u64(len(self.chips))
        for name, log_n, shift, width, height in self.chips:
            w.string(name)
            w.u64(log_n)
            w.u32s([shift])
            w.u64(width)
            w.u64(height)
        w.u64(len(self.ordering))
        for k in sorted(self.ordering, key=lambda k: self.ordering[k]):  # canonical: by index
            w.string(k)
            w.u64(self.ordering[k])

    @staticmethod
    def of_program(machine, prep: Dict[str, np.ndarray], commit, pc_start: int, gcs) -> "StarkVk":
        """StarkMachine::setup's vk (machine.rs:332-439): the preprocessed traces sorted by (height desc,
        name), each with its trace domain (shift 1) and dimensions."""
        pre = {c.name: prep[c.name] for c in machine.chips if prep.get(c.name) is not None}
        order = sorted(pre, key=lambda k: (-pre[k].shape[0], k))
        chips = [(k, int(pre[k].shape[0]).bit_length() - 1, 1, int(pre[k].shape[1]), int(pre[k].shape[0]))
                 for k in order]
        return StarkVk([int(x) for x in commit], int(pc_start), [int(x) for x in gcs], chips,
                       {k: i for i, k in enumerate(order)})


def shard_proof_end(b: bytes, pos: int) -> int:
    """Byte offset just past the ShardProof starting at `pos`."""
    from .recursion_verifier import parse_shard_proof_at
    return parse_shard_proof_at(b, pos)[1]


def read_compress_request(b: bytes, with_deferred: bool = False):
    """CompressRequestPayload (crates/cuda/src/lib.rs:98-106) -> (StarkVk of the core program, [ShardProof
    bytes], number of deferred proofs), or with_deferred: (StarkVk, [ShardProof bytes], [(StarkVk, ShardProof
    bytes)] of `deferred_proofs`).  The stdin (its buffers and the proofs the guest verifies, which the core
    proof already accounts for) and the public values that follow the shard proofs are skipped."""
    r = Reader(b)
    vk = StarkVk.read(r)
    shards = []
    for _ in range(r.u64()):
        start = r.pos
        r.pos = shard_proof_end(b, start)
        shards.append(bytes(b[start:r.pos]))
    # ZKMStdin { buffer: Vec<Vec<u8>>, ptr: usize, proofs: Vec<(ZKMReduceProof, StarkVerifyingKey)> }
    for _ in range(r.u64()):
        r.raw(r.u64())
    r.u64()
    n_stdin_proofs = r.u64()
    for _ in range(n_stdin_proofs):
        StarkVk.read(r)
        r.pos = shard_proof_end(b, r.pos)
        StarkVk.read(r)
    # ZKMPublicValues { buffer: Buffer { data: Vec<u8> } } -- Buffer.ptr is #[serde(skip)]
    # (crates/primitives/src/types.rs:13-18) -- then cycles u64
    r.raw(r.u64())
    r.u64()
    n_deferred = r.u64()
    if not with_deferred:
        return vk, shards, n_deferred + n_stdin_proofs
    deferred = []
    for _ in range(n_deferred):  # ZKMReduceProof { vk: StarkVerifyingKey, proof: ShardProof }
        dvk = StarkVk.read(r)
        start = r.pos
        r.pos = shard_proof_end(b, start)
        deferred.append((dvk, bytes(b[start:r.pos])))
    if r.pos != len(b):
        raise ValueError("trailing bytes after the deferred proofs")
    return vk, shards, deferred


def write_compress_request(vk: StarkVk, shards: List[bytes], stdin: List[bytes] = (), public_values: bytes = b"",
                           cycles: int = 0, deferred: Sequence[Tuple[StarkVk, bytes]] = ()) -> bytes:
    """The client side (crates/cuda/src/lib.rs:92-102), for tests and for a caller holding this
    repository's shard proofs."""
    w = Writer()
    vk.write(w)
    w.u64(len(shards))
    for s in shards:
        w.raw(s)
    w.u64(len(stdin))
    for x in stdin:
        w.u64(len(x))
        w.raw(x)
    w.u64(0)
    w.u64(0)
    w.u64(len(public_values))
    w.raw(public_values)  # Buffer.ptr is not serialized
    w.u64(cycles)
    w.u64(len(deferred))
    for dvk, dproof in deferred:  # ZKMReduceProof: vk then proof
        dvk.write(w)
        w.raw(dproof)
    return w.bytes()


def write_reduce_proof(vk: StarkVk, proof: bytes) -> bytes:
    w = Writer()
    vk.write(w)
    w.raw(proof)
    return w.bytes()


def read_reduce_proof(b: bytes) -> Tuple[StarkVk, bytes]:
    r = Reader(b)
    vk = StarkVk.read(r)
    start = r.pos
    end = shard_proof_end(b, start)
    if end != len(b):
        raise ValueError("trailing bytes after the reduce proof")
    return vk, bytes(b[start:end])
