"""Reading the fields of a serialized ShardProof the machine-level checks need.

Layout: bincode-1 of ShardProof (crates/stark/src/types.rs:77-83), as zkm_open writes it
(zkmips_amd/csrc/prover.cpp `serialize`): three commitments [F; 8]; Vec<ChipOpenedValues> with, per chip,
six Vec<EF> (preprocessed local/next, main local/next, permutation local/next), Vec<Vec<EF>> quotient
chunks, global_cumulative_sum [F; 14], local_cumulative_sum EF and log_degree u64; then the FRI proof,
chip_ordering and public values (not needed here).  u64 lengths, field elements as u32.
"""
from __future__ import annotations

from typing import List

import numpy as np

from .machine import P


class _Reader:
    def __init__(self, b: bytes):
        self.b, self.pos = b, 0

    def u64(self) -> int:
        v = int.from_bytes(self.b[self.pos:self.pos + 8], "little")
        self.pos += 8
        return v

    def u32s(self, n: int) -> np.ndarray:
        v = np.frombuffer(self.b, np.uint32, n, self.pos).copy()
        self.pos += 4 * n
        return v

    def skip(self, n: int):
        self.pos += n


def chip_global_sums(proof: bytes, montgomery: bool = False) -> List[np.ndarray]:
    """ChipOpenedValues::global_cumulative_sum of every chip of the shard proof (canonical words)."""
    r = _Reader(proof)
    r.skip(3 * 32)
    out = []
    for _ in range(r.u64()):
        for _ in range(6):
            r.skip(16 * r.u64())
        for _ in range(r.u64()):
            r.skip(16 * r.u64())
        g = r.u32s(14)
        if montgomery:  # x R -> x: multiply by R^-1 mod p
            rinv = pow(1 << 32, P - 2, P)
            g = (g.astype(np.uint64) * np.uint64(rinv) % np.uint64(P)).astype(np.uint32)
        out.append(g)
        r.skip(16 + 8)
    return out


def shard_global_cumulative_sum(proof: bytes, montgomery: bool = False) -> np.ndarray:
    """ShardProof::global_cumulative_sum (types.rs:105-107): the SepticDigest sum over its chips."""
    from . import septic as S
    return S.digest_sum(np.asarray(chip_global_sums(proof, montgomery)))


def machine_global_sum_is_zero(proofs, initial_global_cumulative_sum=None, montgomery: bool = False) -> bool:
    """The last step of StarkMachine::verify (crates/stark/src/machine.rs:639-654): the shards' global
    cumulative sums and the vk's initial one add up to the zero digest."""
    from . import septic as S
    init = S.CURVE_CUMULATIVE_SUM_START if initial_global_cumulative_sum is None else initial_global_cumulative_sum
    ds = [shard_global_cumulative_sum(p, montgomery) for p in proofs] + [np.asarray(init, np.uint32)]
    return bool(np.array_equal(S.digest_sum(np.asarray(ds)), S.CURVE_CUMULATIVE_SUM_START))
