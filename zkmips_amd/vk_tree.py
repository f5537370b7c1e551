"""The recursion verifying-key Merkle tree (crates/recursion/circuit/src/merkle_tree.rs) and the vk digest
(`StarkVerifyingKey::hash_koalabear`, crates/prover/src/types.rs:80-98; in-program `VerifyingKeyVariable::hash`,
crates/recursion/circuit/src/types.rs:96-119).

A compress node proves that every child's verifying key belongs to the set of allowed recursion programs: the
child's vk digest is a leaf of a Merkle tree whose root (`vk_root`) every recursion proof carries in its public
values (`ZKMCompressWithVKeyVerifier`, machine/vkey_proof.rs:120-145).  The reference builds that set offline
(`vk_map.bin`, one key per recursion shape, "takes several days"; absent from the reference snapshot) and ships
`dummy_vk_map.bin` for `VERIFY_VK=false`: 10000 entries, entry i = key [i; 8] -> i (tests/golden pins it).  In
that mode (prover/src/lib.rs:1149-1188) the node opens the dummy tree at index = vk_digest[0] mod 10000 with the
value [index; 8], and the value is not asserted equal to the digest.  This module builds that tree; the node
program (recursion_verifier.compress_node_program) verifies the openings in-program.

Tree layout (MerkleTree::commit): leaves padded with [0; 8] to a power of two, stored bit-reversed, each layer
`constant_compress([l, r])` = Poseidon2(l || r)[0..8] (TruncatedPermutation); open(index) walks the bit-reversed
index; verify swaps the pair when the reversed index is odd.

Parity: the dummy map's keys are pinned by dummy_vk_map.bin, but the tree's root and the vk digest
(vk_digest) are **parity unpinned**: the reference holds no vk_root or hash_koalabear value to compare with
(no golden vector, no test literal), so the bit-reversed leaf order, the layer compression and the order of the
preprocessed domains in the digest rest on the restated code alone; the tests check open / verify against each
other and the node programs against this module.
"""
from __future__ import annotations

import functools
from typing import Tuple

import numpy as np

from . import recursion as R

P = 0x7F000001
DIGEST = 8
DUMMY_VK_ENTRIES = 10000  # crates/prover/dummy_vk_map.bin (tests/golden/dummy_vk_map.json)


def _rev(x: int, bits: int) -> int:
    return int(format(x, f"0{bits}b")[::-1], 2) if bits else 0


def compress(left: np.ndarray, right: np.ndarray) -> np.ndarray:
    """TruncatedPermutation<Perm, 2, 8, 16> of rows: Poseidon2(l || r)[0..8]."""
    x = np.concatenate([np.atleast_2d(left), np.atleast_2d(right)], axis=1).astype(np.uint32)
    return R.poseidon2_permute_host(x)[:, :DIGEST].astype(np.uint32)


def hash_slice(words) -> np.ndarray:
    """poseidon2_hash (PaddingFreeSponge<Perm, 16, 8, 8>, hash.rs:40-50) of a word slice."""
    w = [int(x) % P for x in words]
    st = np.zeros((1, 16), np.uint32)
    for c in range(0, len(w), 8):
        chunk = w[c:c + 8]
        st[0, :len(chunk)] = chunk
        st = R.poseidon2_permute_host(st).astype(np.uint32)
    return st[0, :DIGEST].copy()


class MerkleTree:
    """MerkleTree<KoalaBear, KoalaBearPoseidon2> (merkle_tree.rs:18-130)."""

    def __init__(self, leaves: np.ndarray):
        leaves = np.asarray(leaves, np.uint32).reshape(-1, DIGEST)
        if not len(leaves):
            raise ValueError("a vk tree needs at least one leaf")
        n = 1 << max(1, (len(leaves) - 1).bit_length())
        self.height = n.bit_length() - 1
        layer = np.zeros((n, DIGEST), np.uint32)
        layer[:len(leaves)] = leaves
        rev = np.asarray([_rev(i, self.height) for i in range(n)])
        layer = layer[np.argsort(rev)]  # position rev(i) holds leaf i
        self.layers = [layer]
        while len(layer) > 1:
            layer = compress(layer[0::2], layer[1::2])
            self.layers.append(layer)
        self.root = layer[0].copy()

    def open(self, index: int) -> Tuple[np.ndarray, np.ndarray]:
        """(value, path) of leaf `index` (MerkleTree::open)."""
        b = _rev(index, self.height)
        value = self.layers[0][b].copy()
        path = []
        for i in range(self.height):
            path.append(self.layers[i][b ^ 1])
            b >>= 1
        return value, np.asarray(path, np.uint32)

    @staticmethod
    def verify(index: int, value, path, root) -> bool:
        """MerkleTree::verify."""
        v = np.asarray(value, np.uint32)
        b = _rev(index, len(path))
        for sib in path:
            v = compress(v, sib)[0] if b % 2 == 0 else compress(sib, v)[0]
            b >>= 1
        return bool(np.array_equal(v, np.asarray(root, np.uint32)))


@functools.lru_cache(maxsize=1)
def dummy_tree() -> MerkleTree:
    """The tree of the reference's dummy_vk_map.bin (keys [i; 8], i < 10000, in BTreeMap order)."""
    keys = np.repeat(np.arange(DUMMY_VK_ENTRIES, dtype=np.uint32)[:, None], DIGEST, axis=1)
    return MerkleTree(keys)


def dummy_opening(vk_digest) -> Tuple[int, np.ndarray, np.ndarray]:
    """make_merkle_proofs with vk_verification = false (prover/src/lib.rs:1164-1173): index = digest[0] mod
    the map size, value [index; 8], and the tree's path for it."""
    t = dummy_tree()
    index = int(np.asarray(vk_digest)[0]) % DUMMY_VK_ENTRIES
    value, path = t.open(index)
    assert np.all(value == index)
    return index, value, path


def vk_hash_inputs(commit, pc_start: int, gcs, prep_log_heights) -> list:
    """The words StarkVerifyingKey::hash_koalabear absorbs: commit[0..8] || pc_start || initial global
    cumulative sum (x[7], y[7]) || per preprocessed domain in chip_information order (log_n, 2^log_n, shift = 1,
    two-adic generator of log_n)."""
    from .recursion_verifier import two_adic_gen
    out = [int(x) % P for x in commit] + [int(pc_start) % P] + [int(x) % P for x in gcs]
    for ln in prep_log_heights:
        out += [int(ln), (1 << int(ln)) % P, 1, two_adic_gen(int(ln))]
    return out


def vk_digest(vk) -> np.ndarray:
    """hash_koalabear of a ChildVk (its preprocessed chips in the vk's (height desc, name) order)."""
    logs = [int(vk.prep_heights[k]).bit_length() - 1 for k in vk.prep_order]
    return hash_slice(vk_hash_inputs(vk.commit, vk.pc_start, vk.gcs, logs))
