import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")
    config.addinivalue_line("markers", "slow: larger CPU sizes")


# The byte-parity tests of each BASELINE config run first, so that under `-x` a failure elsewhere
# cannot hide them: config 1/2 (FibCpu 2^22, 2^20x67 commit), config 3 (the maximal 2^22 shape),
# config 4 (the tendermint execution's shards), config 5 (a MIPS-leaf compress node at a reference
# recursion shape), then the device traces of every chip.
_PRIORITY = [
    "test_gpu_prover.py::test_shard_proof_bytes_identical_2e22",
    "test_gpu_kernels.py::test_pcs_commit_root_vs_oracle[20-67]",
    "test_shapes.py::test_shape_shard_full_size_gpu_proof_verifies",
    "test_shapes.py::test_shape_shard_gpu_proof_bytes_identical",
    "test_tendermint.py::test_gpu_tendermint",
    "test_compress_tree.py::test_gpu_mips_node",
    "test_service.py::test_compress_two_mips_shards",
    "test_tracegen.py::",
]


def _priority(item):
    nid = item.nodeid
    for k, key in enumerate(_PRIORITY):
        if key in nid:
            return k
    return len(_PRIORITY)


def pytest_collection_modifyitems(config, items):
    items.sort(key=_priority)  # stable: everything else keeps file order
    if os.environ.get("ZKM_FORCE_GPU_TESTS"):
        return
    try:
        import torch  # noqa: F401  (device discovery only)
        have = torch.cuda.is_available()
    except Exception:
        have = False
    if not have:
        skip = pytest.mark.skip(reason="no GPU visible")
        for it in items:
            if "gpu" in it.keywords:
                it.add_marker(skip)
