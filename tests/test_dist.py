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


def _fake_reducer(calls, slow=None):
    """A Reducer whose witness step passes the children through (a thread pool stands in for the process
    pool) and whose prove step hashes them: the tree's shape decides the root.  slow: a first child's proof
    bytes whose node takes 3 s to prove (so nodes finish out of order)."""
    import hashlib
    import time
    from concurrent.futures import ThreadPoolExecutor
    from zkmips_amd.compress_tree import Reducer
    tp = ThreadPoolExecutor(4)

    def prove(children):
        if slow is not None and children[0][1] == slow:
            time.sleep(3.0)
        h = hashlib.sha256()
        for _, c in children:
            h.update(len(c).to_bytes(8, "little") + c)
        calls.append(1)
        d = h.digest()
        return ("vk", d * (1 + d[0] % 3))  # ragged proof sizes

    return Reducer(lambda ch, fl: tp.submit(lambda: ch), prove, inflight=2)


def _tree_worker(rank, world, port, out_q, sizes=(64, 5), slow=None):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from zkmips_amd.compress_tree import reduce_distributed
    for nleaves in sizes:
        calls = []
        leaves = [("vk", bytes([i]) * (i + 1)) for i in range(nleaves)]
        root = reduce_distributed(leaves, _fake_reducer(calls, slow))
        out_q.put((rank, nleaves, root, len(calls)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_compress_tree_distributed(world):
    """Config 5's dependency-driven compress tree on `world` gloo ranks: every rank ends with the serial
    tree's root, and each rank proves exactly the nodes it owns (the owner of a node's leftmost leaf), so
    every node is proven once."""
    from zkmips_amd.compress_tree import owner, reduce_serial, tree_nodes
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
        calls = []
        want = reduce_serial([("vk", bytes([i]) * (i + 1)) for i in range(nleaves)], _fake_reducer(calls))
        got = [r for r in res if r[1] == nleaves]
        assert all(r[2] == want for r in got)
        nodes = [nd for l in tree_nodes(nleaves) for nd in l]
        assert sum(r[3] for r in got) == len(nodes) == len(calls) == (63 if nleaves == 64 else 6)
        for r in got:
            assert r[3] == sum(1 for nd in nodes if owner(nd, nleaves, world) == r[0])


def test_compress_tree_distributed_out_of_order():
    """world 3, 16 leaves: rank 1 sends nodes (1,3) and (3,1) to rank 0, and (1,3) (leaves 6, 7) is made
    slow, so (3,1) arrives first; each message names its node, so rank 0 still pairs them correctly and
    every rank ends with the serial tree's root."""
    from zkmips_amd.compress_tree import owner, reduce_serial
    assert owner((1, 3), 16, 3) == owner((3, 1), 16, 3) == 1 and owner((2, 1), 16, 3) == owner((4, 0), 16, 3) == 0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    slow = bytes([6]) * 7
    ps = [ctx.Process(target=_tree_worker, args=(r, 3, port, q, (16,), slow)) for r in range(3)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(3)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = reduce_serial([("vk", bytes([i]) * (i + 1)) for i in range(16)], _fake_reducer([]))
    assert all(r[2] == want for r in res)
