"""`bench.py --gpus N` without an external launcher: bench.py starts its N
ranks itself, the live process group has N ranks, an execution's shards are dealt by cost (LPT), the
proofs are gathered to rank 0 and the machine-level global cumulative sum is checked there.

On CPU the ranks REPLAY proofs the oracle made beforehand (ZKM_BENCH_REPLAY, honoured only with
ZKM_BENCH_REHEARSE=1): the launch / deal / gather / check plumbing runs for real, nothing is proven.  The
GPU variant proves for real with two ranks sharing the box's one GPU."""
import json
import os
import subprocess
import sys

import pytest

from zkmips_amd import mips_core as MC
from zkmips_amd.dist import deal_by_cost, shard_cost

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")
ARGS = ["--workload", "sha2", "--log-n", "7", "--sha-blocks", "3", "--sha-events-per-shard", "1",
        "--steps", "1", "--warmup", "1", "--queries", "4", "--inflight", "2"]


def test_deal_by_cost_is_lpt():
    assert deal_by_cost([1, 1, 1, 1], 2) == [[0, 2], [1, 3]]
    assert deal_by_cost([10, 1, 1, 1, 1, 6], 2) == [[0], [1, 2, 3, 4, 5]]
    d = deal_by_cost([5, 3, 8, 2, 9, 1, 4], 3)
    assert sorted(i for r in d for i in r) == list(range(7))
    loads = [sum([5, 3, 8, 2, 9, 1, 4][i] for i in r) for r in d]
    assert max(loads) - min(loads) <= 2
    assert deal_by_cost([3.0], 4) == [[0], [], [], []]


def _run(env_extra, args, timeout=600):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra)
    r = subprocess.run([sys.executable, BENCH] + args, env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=timeout)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    return r, (json.loads(lines[-1]) if lines else None)


@pytest.fixture(scope="module")
def replay_dir(tmp_path_factory):
    from tests import _oracle as O
    run = MC.program_shards(MC.sha_program(3, seed=1), seed=1, shard_size=(1 << 7) * 4 // 5,
                            precompile_events_per_shard=1)
    m, prep, _, _ = run[0]
    pr = O.OracleProver(m, {k: v for k, v in prep.items() if v is not None}, num_queries=4)
    d = tmp_path_factory.mktemp("replay")
    for i, (_, _, tr, pv) in enumerate(run):
        rc, p = pr.prove(tr, pv)
        assert rc == 0
        (d / f"shard_{i}.bin").write_bytes(p)
    return d, run


def test_bench_launches_its_own_ranks(replay_dir):
    d, run = replay_dir
    r, line = _run({"ZKM_BENCH_REHEARSE": "1", "ZKM_BENCH_REPLAY": str(d)}, ["--gpus", "2"] + ARGS)
    assert r.returncode == 0, r.stderr[-2000:]
    assert line["n_gpus"] == 2 and line["config"]["global_sum_checked"]
    assert line["config"]["shards"] == len(run) >= 5
    assert line["config"]["proof_bytes"] == sum(os.path.getsize(d / f"shard_{i}.bin") for i in range(len(run)))
    deal = deal_by_cost([shard_cost(tr) for _, _, tr, _ in run], 2)
    assert str(deal) in line["config"]["parallelism"]
    # one rank: the same execution, same bytes
    r1, line1 = _run({"ZKM_BENCH_REHEARSE": "1", "ZKM_BENCH_REPLAY": str(d)}, ["--gpus", "1"] + ARGS)
    assert r1.returncode == 0 and line1["n_gpus"] == 1
    assert line1["config"]["proof_bytes"] == line["config"]["proof_bytes"]


def test_bench_rank_failure_propagates(replay_dir, tmp_path):
    """A wrong shard proof (the memory shard replaced by a CPU shard's) breaks the global sum on rank 0:
    the launcher returns non-zero and stops the other rank."""
    d, run = replay_dir
    for f in os.listdir(d):
        (tmp_path / f).write_bytes((d / f).read_bytes())
    (tmp_path / f"shard_{len(run) - 1}.bin").write_bytes((d / "shard_0.bin").read_bytes())
    r, line = _run({"ZKM_BENCH_REHEARSE": "1", "ZKM_BENCH_REPLAY": str(tmp_path)}, ["--gpus", "2"] + ARGS)
    assert r.returncode != 0 and line is None
    assert "global cumulative sums" in r.stderr


def test_gpus_must_match_world_size():
    r, line = _run({"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"}, ["--gpus", "3"] + ARGS, timeout=120)
    assert r.returncode != 0 and "--gpus 3 but WORLD_SIZE=2" in r.stderr


@pytest.mark.gpu
def test_bench_two_ranks_on_one_gpu():
    """Two real ranks (sharing the box's GPU, gloo) prove the headline shard: n_gpus 2 from the live group."""
    r, line = _run({"ZKM_BENCH_REHEARSE": "1"}, ["--gpus", "2", "--log-n", "16", "--steps", "1", "--warmup", "1",
                                                  "--inflight", "1", "--queries", "16", "--no-cpu-baseline",
                                                  "--no-pmc", "--no-maxshape", "--profile-steps", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert line["n_gpus"] == 2 and line["value"] > 0


def test_cgroup_cpu_limit_walks_up_to_the_root(tmp_path):
    """bench.cgroup_cpu_limit: the tightest cpu.max from the process's cgroup up to the mount root (the GPU box
    keeps its 16-CPU quota on the root cgroup, the process's own cgroup has no cpu.max)."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    mount = tmp_path / "cg"
    leaf = mount / "a" / "b"
    leaf.mkdir(parents=True)
    proc = tmp_path / "cgroup"
    proc.write_text("0::/a/b\n")
    assert bench.cgroup_cpu_limit(str(proc), str(mount)) is None  # no cpu.max anywhere
    (mount / "cpu.max").write_text("1600000 100000\n")
    assert bench.cgroup_cpu_limit(str(proc), str(mount)) == 16.0  # root only (the box)
    (mount / "a" / "cpu.max").write_text("max 100000\n")
    assert bench.cgroup_cpu_limit(str(proc), str(mount)) == 16.0  # "max" does not lift the root's quota
    (leaf / "cpu.max").write_text("400000 100000\n")
    assert bench.cgroup_cpu_limit(str(proc), str(mount)) == 4.0  # the tightest wins
