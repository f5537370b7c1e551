"""Multi-GPU shard proving: one process per GPU, shards partitioned across ranks.

The reference proves all shards of a batch in parallel and independently: each shard opens on a
clone of a challenger that has only observed the proving key (crates/core/machine/src/utils/
prove.rs:208-209, :487-521; verifier mirrors it, crates/stark/src/machine.rs:620-624).  So the data
path needs no collective: shards are dealt to ranks and proved locally.  The shards of one execution
are very uneven (a CPU shard, precompile shards whose Global chip is 2^22 rows, a small memory shard),
so they are dealt by cost, largest first, each to the least-loaded rank (LPT), not i % N.  The only
exchange is the aggregation of finished proofs (KB-MB each) to rank 0, which assembles the
MachineProof in shard order and runs the machine-level check the reference's verifier ends with: the
shards' global cumulative sums add up to the zero digest (crates/stark/src/machine.rs:639-654) — one
gather over the process group (RCCL over xGMI with backend "nccl", gloo on CPU for tests).
"""
from __future__ import annotations

from typing import Callable, Dict, List, Sequence


def assign_shards(num_shards: int, world: int, rank: int) -> List[int]:
    """Round-robin shard indices for `rank` (shard i -> rank i % world): for shards of equal cost."""
    return [i for i in range(num_shards) if i % world == rank]


def deal_by_cost(costs: Sequence[float], world: int) -> List[List[int]]:
    """Longest-processing-time dealing: shards in descending cost (ties by index), each to the rank with
    the least cost so far (ties to the lowest rank).  Deterministic, so every rank computes the same
    deal without an exchange.  Returns the shard indices of every rank, each list in ascending order."""
    load = [0.0] * world
    out: List[List[int]] = [[] for _ in range(world)]
    for i in sorted(range(len(costs)), key=lambda i: (-costs[i], i)):
        r = min(range(world), key=lambda r: (load[r], r))
        load[r] += costs[i]
        out[r].append(i)
    return [sorted(x) for x in out]


def shard_cost(traces: Dict[str, object]) -> float:
    """Proving cost of a shard, in committed main-trace cells (rows x width summed over its chips): the
    LDE, the leaf hashing and the quotient all scale with it."""
    return float(sum(int(t.shape[0]) * int(t.shape[1]) for t in traces.values() if t is not None))


def _encode(local: Dict[int, bytes]) -> bytes:
    out = bytearray(len(local).to_bytes(8, "little"))
    for idx in sorted(local):
        b = local[idx]
        out += idx.to_bytes(8, "little") + len(b).to_bytes(8, "little") + b
    return bytes(out)


def _decode(buf: bytes) -> Dict[int, bytes]:
    n = int.from_bytes(buf[:8], "little")
    pos, res = 8, {}
    for _ in range(n):
        idx = int.from_bytes(buf[pos:pos + 8], "little")
        ln = int.from_bytes(buf[pos + 8:pos + 16], "little")
        res[idx] = bytes(buf[pos + 16:pos + 16 + ln])
        pos += 16 + ln
    return res


def gather_proofs(local: Dict[int, bytes], device="cpu") -> Dict[int, bytes]:
    """All-gather every rank's {shard index: proof bytes}; returns the union on every rank."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    payload = _encode(local)
    ln = torch.tensor([len(payload)], dtype=torch.int64, device=device)
    dist.all_reduce(ln, op=dist.ReduceOp.MAX)
    size = int(ln.item())
    buf = torch.zeros(size + 8, dtype=torch.uint8, device=device)
    buf[:8] = torch.tensor(list(len(payload).to_bytes(8, "little")), dtype=torch.uint8, device=device)
    if payload:
        buf[8:8 + len(payload)] = torch.frombuffer(bytearray(payload), dtype=torch.uint8).to(device)
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    out: Dict[int, bytes] = {}
    for p in parts:
        raw = p.cpu().numpy().tobytes()
        n = int.from_bytes(raw[:8], "little")
        out.update(_decode(raw[8:8 + n]))
    return out


def gather_proofs_to_root(local: Dict[int, bytes], device="cpu", root: int = 0) -> Dict[int, bytes]:
    """Gather every rank's {shard index: proof bytes} to `root` only (one padded gather; the padding is
    the largest rank payload, agreed by an 8-byte all_reduce).  Returns the union on root, {} elsewhere."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(), dist.get_rank()
    payload = _encode(local)
    ln = torch.tensor([len(payload)], dtype=torch.int64, device=device)
    dist.all_reduce(ln, op=dist.ReduceOp.MAX)
    size = int(ln.item())
    buf = torch.zeros(size + 8, dtype=torch.uint8, device=device)
    buf[:8] = torch.tensor(list(len(payload).to_bytes(8, "little")), dtype=torch.uint8, device=device)
    if payload:
        buf[8:8 + len(payload)] = torch.frombuffer(bytearray(payload), dtype=torch.uint8).to(device)
    parts = [torch.empty_like(buf) for _ in range(world)] if rank == root else None
    dist.gather(buf, parts, dst=root)
    out: Dict[int, bytes] = {}
    if rank == root:
        for p in parts:
            raw = p.cpu().numpy().tobytes()
            n = int.from_bytes(raw[:8], "little")
            out.update(_decode(raw[8:8 + n]))
    return out


def prove_shards_distributed(prove_one: Callable[[int], bytes], num_shards: int, device="cpu",
                             check_global_sum: bool = False, costs: Sequence[float] = None) -> List[bytes]:
    """MachineProver::prove across ranks: each rank proves its shards (dealt by `costs` when given,
    else round-robin); rank 0 receives every proof in shard order (other ranks get []), and with
    check_global_sum verifies that the shards' global cumulative sums add up to the zero digest
    (machine.rs:639-654)."""
    import torch.distributed as dist
    world, rank = dist.get_world_size(), dist.get_rank()
    mine = deal_by_cost(costs, world)[rank] if costs is not None else assign_shards(num_shards, world, rank)
    local = {i: prove_one(i) for i in mine}
    allp = gather_proofs_to_root(local, device)
    if rank != 0:
        return []
    proofs = [allp[i] for i in range(num_shards)]
    if check_global_sum:
        from .proof import machine_global_sum_is_zero
        if not machine_global_sum_is_zero(proofs):
            raise ValueError("the shards' global cumulative sums do not add up to zero")
    return proofs
