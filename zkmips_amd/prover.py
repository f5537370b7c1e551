"""Host-side mirror of the reference's `MachineProver` surface over the HIP C ABI.

Reference: `MachineProver<SC, A>` / `CpuProver` (crates/stark/src/prover.rs:30-184, :210-694):
  setup(program) -> (pk, vk)         machine.rs:332-439
  pk_to_device(pk)                    prover.rs:250 (here: the preprocessed LDE + tree live on the GPU)
  commit(record, traces) -> ShardMainData   prover.rs:258-292
  open(pk, data, challenger) -> ShardProof   prover.rs:298-653
  prove(pk, records, challenger)       prover.rs:660-693 (per-shard challenger clones)
Every call goes through libzkm_hip.so; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import (ZKM_MEM_DEVICE, ZKM_REPR_CANONICAL, ChallengerState, Config, Device, Matrix, as_u32, check, lib,
                   matrix)
from .machine import MachineDesc

# CURVE_CUMULATIVE_SUM_START_{X,Y} (crates/stark/src/septic_digest.rs:9-14): SepticDigest::zero()
ZERO_DIGEST = np.asarray([637514027, 1595065213, 1998064738, 72333738, 1211544370, 822986770, 1518535784,
                          1604177449, 90440090, 259343427, 140470264, 1162099742, 941559812, 1064053343], np.uint32)


class ShardMainData:
    """Owns the device-side main LDE + Merkle tree of one shard (types.rs:16-22)."""

    def __init__(self, handle: C.c_void_p, commit: np.ndarray):
        self.h = handle
        self.main_commit = commit

    def __del__(self):
        if self.h:
            lib().zkm_main_free(self.h)
            self.h = None


def _device_matrix(tensor, name: str, keep: list) -> Matrix:
    """A row-major GPU tensor as a ZKM_MEM_DEVICE matrix; waits for the producing stream first (the
    prover's kernels run on streams of their own)."""
    import torch
    if not tensor.is_cuda or tensor.dim() != 2 or not tensor.is_contiguous() or tensor.element_size() != 4:
        raise ValueError(f"trace {name}: need a contiguous 2-D 32-bit tensor on the GPU")
    torch.cuda.current_stream(tensor.device).synchronize()
    nm = name.encode()
    keep.append(nm)
    keep.append(tensor)
    return Matrix(nm, tensor.data_ptr(), tensor.shape[0], tensor.shape[1], ZKM_REPR_CANONICAL | ZKM_MEM_DEVICE)


def blob_chip_names(blob: np.ndarray) -> List[str]:
    """The chip names of a machine blob, in machine order (format: include/zkm_hip.h)."""
    w = [int(x) for x in as_u32(blob)]
    if len(w) < 4 or w[0] != 0x4D4D4B5A:
        raise ValueError("not a machine blob")
    i, names = 4, []
    for _ in range(w[3]):
        n = w[i]
        nw = (n + 3) // 4
        names.append(b"".join(x.to_bytes(4, "little") for x in w[i + 1:i + 1 + nw])[:n].decode())
        i += 1 + nw + 6
        i += 1 + w[i]  # code
        nl = w[i] + w[i + 1]
        i += 2
        for _ in range(nl):
            nv = w[i + 2]
            i += 3
            for _ in range(nv + 1):
                i += 2 + 2 * w[i]
    if i != len(w):
        raise ValueError("malformed machine blob")
    return names


class _BlobMachine:
    """MachineDesc stand-in over a raw blob: chip names + the blob itself."""

    class _Chip:
        def __init__(self, name):
            self.name = name

    def __init__(self, blob: np.ndarray):
        self._blob = blob
        self.chips = [self._Chip(n) for n in blob_chip_names(blob)]

    def blob(self) -> np.ndarray:
        return self._blob


class MachineHandle:
    """A key-free machine layout for commit (zkm_machine_new / zkm_commit_machine): the reference's
    trait commit receives no proving key (prover.rs:111-115), and commit reads only chip names, main
    widths and the blowup.  zkm_open checks the shard against the key's machine."""

    def __init__(self, machine, log_blowup: int = 1, num_queries: int = 84, pow_bits: int = 16):
        self.blob = as_u32(machine.blob() if hasattr(machine, "blob") else machine)
        self.cfg = Config(num_queries, pow_bits, log_blowup, 0)
        self.h = C.c_void_p()
        check(lib().zkm_machine_new(self.blob.ctypes.data, self.blob.size, C.byref(self.cfg), C.byref(self.h)),
              "zkm_machine_new")

    def __del__(self):
        if getattr(self, "h", None):
            lib().zkm_machine_free(self.h)
            self.h = None

    def commit(self, device: Device, traces: Dict[str, np.ndarray], public_values: np.ndarray,
               montgomery_input: bool = False) -> "ShardMainData":
        keep: list = []
        arr = (Matrix * len(traces))(*[matrix(t, n, montgomery_input, keep) for n, t in traces.items()])
        pv = as_u32(public_values)
        h = C.c_void_p()
        root = np.zeros(8, np.uint32)
        check(lib().zkm_commit_machine(device.h, self.h, arr, len(traces), pv.ctypes.data, pv.size, C.byref(h),
                                       root.ctypes.data), "zkm_commit_machine")
        return ShardMainData(h, root)


class HipProver:
    """MI355X drop-in for CpuProver on one GPU."""

    def __init__(self, device: Device, machine: MachineDesc, prep_traces: Dict[str, np.ndarray],
                 num_queries: int = 84, pow_bits: int = 16, proof_montgomery: bool = False,
                 pc_start: Optional[int] = None, initial_global_cumulative_sum: Optional[np.ndarray] = None,
                 log_blowup: int = 1):
        self.dev = device
        self.machine = machine
        self.blob = machine.blob()
        self.cfg = Config(num_queries, pow_bits, log_blowup, int(proof_montgomery))
        keep: list = []
        mats = (Matrix * len(machine.chips))()
        for i, c in enumerate(machine.chips):
            if c.name in prep_traces:
                t = prep_traces[c.name]  # a host array, or a GPU-resident int32 tensor (ZKM_MEM_DEVICE)
                mats[i] = _device_matrix(t, c.name, keep) if hasattr(t, "data_ptr") else matrix(t, c.name, keep=keep)
            else:
                mats[i] = Matrix(c.name.encode(), None, 0, 0, 0)
        gcs = as_u32(ZERO_DIGEST if initial_global_cumulative_sum is None else initial_global_cumulative_sum)
        if pc_start is None:  # the machine's programs' entry (MachineDesc.pc_start)
            pc_start = getattr(machine, "pc_start", 0x00400000)
        self.pk = C.c_void_p()
        self.vk_commit = np.zeros(8, np.uint32)
        check(lib().zkm_setup(device.h, self.blob.ctypes.data, self.blob.size, C.byref(self.cfg), mats,
                              len(machine.chips), pc_start, gcs.ctypes.data, C.byref(self.pk),
                              self.vk_commit.ctypes.data), "zkm_setup")

    @classmethod
    def from_blob(cls, device: Device, blob: np.ndarray, prep_traces: Dict[str, np.ndarray], **kw) -> "HipProver":
        """A prover for a machine given only as its blob (e.g. received over the service)."""
        return cls(device, _BlobMachine(as_u32(blob)), prep_traces, **kw)

    def __del__(self):
        if getattr(self, "pk", None):
            lib().zkm_pk_free(self.pk)
            self.pk = None

    # ---- challenger helpers ----
    def base_challenger(self) -> ChallengerState:
        """A fresh DuplexChallenger that has observed the proving key (prove.rs:208-209)."""
        ch = ChallengerState()
        check(lib().zkm_pk_observe(self.pk, C.byref(ch)), "zkm_pk_observe")
        return ch

    # ---- MachineProver surface ----
    def commit(self, traces: Dict[str, np.ndarray], public_values: np.ndarray,
               montgomery_input: bool = False) -> ShardMainData:
        keep: list = []
        arr = (Matrix * len(traces))(*[matrix(t, n, montgomery_input, keep) for n, t in traces.items()])
        pv = as_u32(public_values)
        h = C.c_void_p()
        root = np.zeros(8, np.uint32)
        check(lib().zkm_commit(self.dev.h, self.pk, arr, len(traces), pv.ctypes.data, pv.size, C.byref(h),
                               root.ctypes.data), "zkm_commit")
        return ShardMainData(h, root)

    def open(self, data: ShardMainData, challenger: ChallengerState) -> bytes:
        out = C.POINTER(C.c_uint8)()
        n = C.c_uint64()
        h, data.h = data.h, None  # consumed by zkm_open
        check(lib().zkm_open(self.dev.h, self.pk, h, C.byref(challenger), C.byref(out), C.byref(n)), "zkm_open")
        b = C.string_at(out, n.value)
        lib().zkm_free_bytes(out)
        return b

    def prove_shard(self, traces: Dict[str, np.ndarray], public_values: np.ndarray,
                    challenger: Optional[ChallengerState] = None) -> bytes:
        """Traces are host arrays or GPU-resident int32 torch tensors (e.g. from zkmips_amd.tracegen),
        which cross the ABI as ZKM_MEM_DEVICE matrices."""
        base = challenger if challenger is not None else self.base_challenger()
        keep: list = []
        arr = (Matrix * len(traces))(*[_device_matrix(t, n, keep) if hasattr(t, "data_ptr") else
                                       matrix(t, n, False, keep) for n, t in traces.items()])
        pv = as_u32(public_values)
        out = C.POINTER(C.c_uint8)()
        n = C.c_uint64()
        check(lib().zkm_prove_shard(self.dev.h, self.pk, arr, len(traces), pv.ctypes.data, pv.size, C.byref(base),
                                    C.byref(out), C.byref(n)), "zkm_prove_shard")
        b = C.string_at(out, n.value)
        lib().zkm_free_bytes(out)
        return b

    def prove(self, shards: Sequence[Dict[str, np.ndarray]], public_values: Sequence[np.ndarray]) -> List[bytes]:
        """MachineProver::prove: observe pk once, then each shard opens on a clone (prover.rs:676-690)."""
        base = self.base_challenger()
        return [self.prove_shard(t, pv, ChallengerState.from_buffer_copy(bytes(base)))
                for t, pv in zip(shards, public_values)]
