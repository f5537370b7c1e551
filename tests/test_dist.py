"""N > 1 path on CPU: world_size 2 with gloo.  Each rank proves its round-robin shards (with the
CPU oracle standing in for the GPU prover) and the gathered MachineProof equals the sequential
single-process proof list byte for byte."""
import os
import socket

import pytest
import torch.multiprocessing as mp

from zkmips_amd.dist import _decode, _encode, assign_shards


def test_assignment_partitions():
    for world in (1, 2, 3, 8):
        seen = sorted(i for r in range(world) for i in assign_shards(10, world, r))
        assert seen == list(range(10))


def test_encode_roundtrip():
    d = {3: b"abc", 0: b"", 7: bytes(range(256))}
    assert _decode(_encode(d)) == d


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tests import _oracle as O
    from zkmips_amd import workloads as W
    from zkmips_amd.dist import prove_shards_distributed
    m, prep, _, _ = W.fib_shard(32, 0)
    pr = O.OracleProver(m, prep, num_queries=4)

    def prove_one(i):
        _, _, tr, pv = W.fib_shard(32, seed=100 + i)
        rc, proof = pr.prove(tr, pv)
        assert rc == 0
        return proof

    proofs = prove_shards_distributed(prove_one, 5)
    if rank == 0:
        out_q.put([p.hex() for p in proofs])
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_matches_sequential():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    from tests import _oracle as O
    from zkmips_amd import workloads as W
    m, prep, _, _ = W.fib_shard(32, 0)
    pr = O.OracleProver(m, prep, num_queries=4)
    seq = []
    for i in range(5):
        _, _, tr, pv = W.fib_shard(32, seed=100 + i)
        seq.append(pr.prove(tr, pv)[1].hex())
    assert got == seq


def _tree_node(layer, j, children):
    import hashlib
    h = hashlib.sha256(f"{layer}:{j}:".encode())
    for c in children:
        h.update(len(c).to_bytes(8, "little") + c)
    return h.digest() * (1 + j % 3)  # ragged proof sizes


def _tree_serial(leaves):
    cur, layer = list(leaves), 0
    while len(cur) > 1:
        layer += 1
        cur = [_tree_node(layer, j, cur[2 * j:2 * j + 2]) for j in range((len(cur) + 1) // 2)]
    return cur[0]


def _tree_worker(rank, world, port, out_q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from zkmips_amd.dist import compress_tree_distributed
    calls = []

    def node(layer, j, children):
        calls.append((layer, j))
        return _tree_node(layer, j, children)

    for nleaves in (64, 5):
        leaves = [bytes([i]) * (i + 1) for i in range(nleaves)]
        root = compress_tree_distributed(node, leaves)
        out_q.put((rank, nleaves, root, list(calls)))
        calls.clear()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_compress_tree_distributed(world):
    """Config 5's layer-by-layer compress tree on `world` gloo ranks: every rank ends with the serial
    tree's root, each node is proved exactly once, on rank j % world."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_tree_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(2 * world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for nleaves in (64, 5):
        want = _tree_serial([bytes([i]) * (i + 1) for i in range(nleaves)])
        got = [r for r in res if r[1] == nleaves]
        assert all(r[2] == want for r in got)
        nodes = sorted(c for r in got for c in r[3])
        assert len(nodes) == len(set(nodes)) == (63 if nleaves == 64 else 6)
        for r in got:
            assert all(j % world == r[0] for _, j in r[3])
