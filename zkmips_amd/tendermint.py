"""BASELINE config 4 on the reference's own data: the tendermint light-client check of
examples/tendermint (guest: examples/tendermint/guest/src/main.rs:34-65; fixtures
examples/tendermint/host/files/block_2279100.json and block_2279130.json).

The guest (tendermint-light-client-verifier 0.40.3, a crates.io dependency of the reference not vendored
in /root/reference; its published algorithm is restated here from the Tendermint specification):

1. hashes both headers: `Header::hash` = the simple Merkle tree (RFC 6962 style: leaf = SHA-256(0x00 || x),
   inner = SHA-256(0x01 || l || r), split at the largest power of two below n) of the header's 14 fields,
   each protobuf-encoded (version, chain_id, height, time, last_block_id, the eight hashes, proposer);
2. commits both header hashes;
3. checks `light_block_1.next_validators.hash() == next_validators_hash` (a validator set hash is the
   Merkle root of the validators' SimpleValidator {pub_key, voting_power} encodings);
4. `verify_update_header(untrusted = block 2279130, trusted = block 2279100)`: the untrusted header's
   validator sets hash to what the header says, then every non-absent commit vote is checked: its
   canonical-vote sign bytes (protobuf CanonicalVote, length-delimited) verified against the validator's
   Ed25519 key, and the committed voting power tallied — more than 2/3 of the untrusted validator set,
   and more than the trust threshold 1/3 of the trusted next validator set;
5. commits the CBOR-encoded verdict ("Success").

This module holds the host side: the encodings, hashes and signature checks in plain Python, pinned by the
fixtures themselves (the header hash of block 2279130 is its commit's block_id.hash in the JSON, and every
validator-set hash is in a header), and the guest generator (`tendermint_program`) that performs the same
computation in MIPS instructions and precompile calls: SHA-256 through SHA_EXTEND / SHA_COMPRESS, the
Ed25519 group law through ED_DECOMPRESS / ED_ADD, and SHA-512 (the Ed25519 challenge hash, software in the
reference's guest too: ed25519-consensus over sha2) as a MIPS loop with 64-bit arithmetic on register pairs.
"""
from __future__ import annotations

import base64
import calendar
import hashlib
import json
import os
from typing import Dict, List, Optional, Sequence, Tuple

FIXTURES = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "tendermint")


# ---------------------------------------------------------------- protobuf (proto3 wire format)
def varint(n: int) -> bytes:
    out = bytearray()
    n &= (1 << 64) - 1
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def f_varint(num: int, v: int) -> bytes:
    return b"" if v == 0 else varint(num << 3) + varint(v)


def f_bytes(num: int, b: bytes) -> bytes:
    return b"" if not b else varint((num << 3) | 2) + varint(len(b)) + b


def f_msg(num: int, b: bytes, always: bool = False) -> bytes:
    """An embedded message (omitted when empty unless `always`: gogoproto non-nullable fields)."""
    return (varint((num << 3) | 2) + varint(len(b)) + b) if (b or always) else b""


def f_sfixed64(num: int, v: int) -> bytes:
    return b"" if v == 0 else varint((num << 3) | 1) + (v & ((1 << 64) - 1)).to_bytes(8, "little")


def timestamp(s: str) -> Tuple[int, int]:
    """RFC 3339 (the fixtures' "2024-07-16T21:27:42.817717878Z") -> (seconds, nanos)."""
    assert s.endswith("Z")
    main, _, frac = s[:-1].partition(".")
    import datetime
    dt = datetime.datetime.strptime(main, "%Y-%m-%dT%H:%M:%S")
    return calendar.timegm(dt.timetuple()), int((frac + "000000000")[:9]) if frac else 0


def pb_timestamp(s: str) -> bytes:
    sec, ns = timestamp(s)
    return f_varint(1, sec) + f_varint(2, ns)


def pb_block_id(bid: dict) -> bytes:
    """tendermint.types.BlockID {hash (1), part_set_header (2) {total (1), hash (2)}}."""
    psh = f_varint(1, int(bid["parts"]["total"])) + f_bytes(2, bytes.fromhex(bid["parts"]["hash"]))
    return f_bytes(1, bytes.fromhex(bid["hash"])) + f_msg(2, psh, always=True)


# ---------------------------------------------------------------- simple Merkle tree (crypto/merkle)
def leaf_hash(x: bytes) -> bytes:
    return hashlib.sha256(b"\x00" + x).digest()


def inner_hash(l: bytes, r: bytes) -> bytes:
    return hashlib.sha256(b"\x01" + l + r).digest()


def split_point(n: int) -> int:
    """The largest power of two strictly below n (n >= 2)."""
    k = 1
    while k * 2 < n:
        k *= 2
    return k


def merkle_root(items: Sequence[bytes]) -> bytes:
    n = len(items)
    if n == 0:
        return hashlib.sha256(b"").digest()
    if n == 1:
        return leaf_hash(items[0])
    k = split_point(n)
    return inner_hash(merkle_root(items[:k]), merkle_root(items[k:]))


# ---------------------------------------------------------------- blocks
def load_block(height: int) -> dict:
    with open(os.path.join(FIXTURES, f"block_{height}.json")) as f:
        return json.load(f)


def header_fields(h: dict) -> List[bytes]:
    """The 14 leaves of Header::hash, each field encoded as the Go implementation's cdcEncode does
    (wrapper messages StringValue / Int64Value / BytesValue: field 1) or as its own proto message."""
    version = f_varint(1, int(h["version"]["block"])) + f_varint(2, int(h["version"]["app"]))
    hb = lambda k: f_bytes(1, bytes.fromhex(h[k]))
    return [version, f_bytes(1, h["chain_id"].encode()), f_varint(1, int(h["height"])), pb_timestamp(h["time"]),
            pb_block_id(h["last_block_id"]), hb("last_commit_hash"), hb("data_hash"), hb("validators_hash"),
            hb("next_validators_hash"), hb("consensus_hash"), hb("app_hash"), hb("last_results_hash"),
            hb("evidence_hash"), hb("proposer_address")]


def header_hash(block: dict) -> bytes:
    return merkle_root(header_fields(block["signed_header"]["header"]))


def validator_bytes(v: dict) -> bytes:
    """SimpleValidator {pub_key (1): PublicKey {ed25519 (1)}, voting_power (2)}."""
    assert v["pub_key"]["type"] == "tendermint/PubKeyEd25519"
    pk = f_bytes(1, base64.b64decode(v["pub_key"]["value"]))
    return f_msg(1, pk) + f_varint(2, int(v["power"]))


def validators_hash(vset: dict) -> bytes:
    return merkle_root([validator_bytes(v) for v in vset["validators"]])


def vote_sign_bytes(chain_id: str, commit: dict, sig: dict) -> bytes:
    """CanonicalVote {type (1) = PRECOMMIT, height (2) sfixed64, round (3) sfixed64, block_id (4)
    CanonicalBlockID (absent for a nil vote), timestamp (5), chain_id (6)}, length-delimited
    (types/vote.go VoteSignBytes)."""
    flag = int(sig["block_id_flag"])
    body = f_varint(1, 2) + f_sfixed64(2, int(commit["height"])) + f_sfixed64(3, int(commit["round"]))
    if flag == 2:  # BLOCK_ID_FLAG_COMMIT: the commit's block id; NIL: none
        bid = commit["block_id"]
        psh = f_varint(1, int(bid["parts"]["total"])) + f_bytes(2, bytes.fromhex(bid["parts"]["hash"]))
        body += f_msg(4, f_bytes(1, bytes.fromhex(bid["hash"])) + f_msg(2, psh, always=True))
    body += f_msg(5, pb_timestamp(sig["timestamp"]), always=True) + f_bytes(6, chain_id.encode())
    return varint(len(body)) + body


def signed_votes(block: dict) -> List[dict]:
    """The commit's non-absent votes with their validator (ValidatorSet lookup by address), sign bytes,
    key, signature and whether they count (block_id_flag COMMIT)."""
    sh = block["signed_header"]
    chain = sh["header"]["chain_id"]
    by_addr = {v["address"]: v for v in block["validator_set"]["validators"]}
    out = []
    for s in sh["commit"]["signatures"]:
        flag = int(s["block_id_flag"])
        if flag == 1:  # absent
            continue
        v = by_addr.get(s["validator_address"])
        if v is None:
            continue
        out.append({"address": s["validator_address"], "power": int(v["power"]),
                    "pub": base64.b64decode(v["pub_key"]["value"]), "sig": base64.b64decode(s["signature"]),
                    "msg": vote_sign_bytes(chain, sh["commit"], s), "commit": flag == 2})
    return out


# ---------------------------------------------------------------- Ed25519 (RFC 8032, cofactorless check)
def ed25519_challenge(R: bytes, A: bytes, msg: bytes) -> int:
    from .mips_edwards import ED_L
    return int.from_bytes(hashlib.sha512(R + A + msg).digest(), "little") % ED_L


def decode_point(b: bytes):
    from .mips_edwards import ED_P, ed_decompress_point
    y = int.from_bytes(b, "little") & ((1 << 255) - 1)
    if y >= ED_P:
        raise ValueError("non-canonical y")
    return ed_decompress_point(y, b[31] >> 7)


def ed25519_verify(pub: bytes, msg: bytes, sig: bytes) -> bool:
    """[S]B == R + [k]A with k = SHA-512(R || A || M) mod L (ed25519-consensus's check, without the
    cofactor: every honest signature satisfies it)."""
    from .mips_edwards import BASE_X, BASE_Y, ED_L, _scalar_mul, ed_add_points
    S = int.from_bytes(sig[32:], "little")
    if S >= ED_L:
        return False
    try:
        A, R = decode_point(pub), decode_point(sig[:32])
    except ValueError:
        return False
    k = ed25519_challenge(sig[:32], pub, msg)
    return _scalar_mul(S, (BASE_X, BASE_Y)) == ed_add_points(R, _scalar_mul(k, A))


def verify_update_header(untrusted: dict, trusted: dict) -> Tuple[bool, dict]:
    """The checks of verify_update_header that the guest performs: validator-set hashes of the untrusted
    block, every non-absent vote's signature, committed power > 2/3 of the untrusted set and > 1/3 of the
    trusted next validator set.  Returns (success, tallies)."""
    h = untrusted["signed_header"]["header"]
    ok = validators_hash(untrusted["validator_set"]).hex().upper() == h["validators_hash"]
    ok &= validators_hash(untrusted["next_validator_set"]).hex().upper() == h["next_validators_hash"]
    votes = signed_votes(untrusted)
    ok &= all(ed25519_verify(v["pub"], v["msg"], v["sig"]) for v in votes)
    total = sum(int(v["power"]) for v in untrusted["validator_set"]["validators"])
    tallied = sum(v["power"] for v in votes if v["commit"])
    trusted_pw = {v["address"]: int(v["power"]) for v in trusted["next_validator_set"]["validators"]}
    t_total = sum(trusted_pw.values())
    t_tallied = sum(trusted_pw.get(v["address"], 0) for v in votes if v["commit"])
    ok &= 3 * tallied > 2 * total and 3 * t_tallied > t_total
    return bool(ok), {"tallied": tallied, "total": total, "trusted_tallied": t_tallied, "trusted_total": t_total,
                      "votes": len(votes)}


VERDICT_SUCCESS_CBOR = b"\x67Success"  # serde_cbor of the unit variant Verdict::Success


# ---------------------------------------------------------------- the guest (MIPS instructions)
M32 = 0xFFFFFFFF
SHA512_K = [
    0x428a2f98d728ae22, 0x7137449123ef65cd, 0xb5c0fbcfec4d3b2f, 0xe9b5dba58189dbbc, 0x3956c25bf348b538,
    0x59f111f1b605d019, 0x923f82a4af194f9b, 0xab1c5ed5da6d8118, 0xd807aa98a3030242, 0x12835b0145706fbe,
    0x243185be4ee4b28c, 0x550c7dc3d5ffb4e2, 0x72be5d74f27b896f, 0x80deb1fe3b1696b1, 0x9bdc06a725c71235,
    0xc19bf174cf692694, 0xe49b69c19ef14ad2, 0xefbe4786384f25e3, 0x0fc19dc68b8cd5b5, 0x240ca1cc77ac9c65,
    0x2de92c6f592b0275, 0x4a7484aa6ea6e483, 0x5cb0a9dcbd41fbd4, 0x76f988da831153b5, 0x983e5152ee66dfab,
    0xa831c66d2db43210, 0xb00327c898fb213f, 0xbf597fc7beef0ee4, 0xc6e00bf33da88fc2, 0xd5a79147930aa725,
    0x06ca6351e003826f, 0x142929670a0e6e70, 0x27b70a8546d22ffc, 0x2e1b21385c26c926, 0x4d2c6dfc5ac42aed,
    0x53380d139d95b3df, 0x650a73548baf63de, 0x766a0abb3c77b2a8, 0x81c2c92e47edaee6, 0x92722c851482353b,
    0xa2bfe8a14cf10364, 0xa81a664bbc423001, 0xc24b8b70d0f89791, 0xc76c51a30654be30, 0xd192e819d6ef5218,
    0xd69906245565a910, 0xf40e35855771202a, 0x106aa07032bbd1b8, 0x19a4c116b8d2d0c8, 0x1e376c085141ab53,
    0x2748774cdf8eeb99, 0x34b0bcb5e19b48a8, 0x391c0cb3c5c95a63, 0x4ed8aa4ae3418acb, 0x5b9cca4f7763e373,
    0x682e6ff3d6b2b8a3, 0x748f82ee5defb2fc, 0x78a5636f43172f60, 0x84c87814a1f0ab72, 0x8cc702081a6439ec,
    0x90befffa23631e28, 0xa4506cebde82bde9, 0xbef9a3f7b2c67915, 0xc67178f2e372532b, 0xca273eceea26619c,
    0xd186b8c721c0c207, 0xeada7dd6cde0eb1e, 0xf57d4f7fee6ed178, 0x06f067aa72176fba, 0x0a637dc5a2c898a6,
    0x113f9804bef90dae, 0x1b710b35131c471b, 0x28db77f523047d84, 0x32caab7b40c72493, 0x3c9ebe0a15c9bebc,
    0x431d67c49c100d4c, 0x4cc5d4becb3e42b6, 0x597f299cfc657e2a, 0x5fcb6fab3ad6faec, 0x6c44198c4a475817]
SHA512_H0 = [0x6a09e667f3bcc908, 0xbb67ae8584caa73b, 0x3c6ef372fe94f82b, 0xa54ff53a5f1d36f1,
             0x510e527fade682d1, 0x9b05688c2b3e6c1f, 0x1f83d9abfb41bd6b, 0x5be0cd19137e2179]


def _le_words(b: bytes) -> List[int]:
    b = b + b"\0" * (-len(b) % 4)
    return [int.from_bytes(b[i:i + 4], "little") for i in range(0, len(b), 4)]


def _sha256_blocks(msg: bytes) -> List[List[int]]:
    """SHA-256 padding of msg as 64-byte blocks of big-endian u32 words (what SHA_EXTEND / SHA_COMPRESS
    take, as the guest's sha2 crate passes them)."""
    m = msg + b"\x80" + b"\0" * ((55 - len(msg)) % 64) + (8 * len(msg)).to_bytes(8, "big")
    return [[int.from_bytes(m[i + 4 * j:i + 4 * j + 4], "big") for j in range(16)] for i in range(0, len(m), 64)]


class Asm:
    """A small MIPS assembler over this repository's instruction tuples (op, a, b, c, imm_b, imm_c):
    labels, branches with their delay slots, and a bump allocator for data words."""

    def __init__(self, data_base: int):
        from . import mips_alu as A
        from . import mips_core as MC
        from . import mips_syscall as SY
        self.A, self.MC, self.SY = A, MC, SY
        self.p: List[tuple] = []
        self.labels: Dict[str, int] = {}
        self.fix: List[Tuple[int, str]] = []
        self.brk = data_base

    def alloc(self, words: int, align: int = 4) -> int:
        self.brk = (self.brk + align - 1) // align * align
        a = self.brk
        self.brk += 4 * words
        return a

    # --- ALU ---
    def e(self, *ins):
        self.p.append(tuple(ins))

    def li(self, r, v):
        self.e(self.A.OP_ADD, r, 0, int(v) & M32, 0, 1)

    def addi(self, rd, rs, imm):
        self.e(self.A.OP_ADD, rd, rs, int(imm) & M32, 0, 1)

    def rr(self, op, rd, rs, rt):
        self.e(op, rd, rs, rt, 0, 0)

    def add(self, rd, rs, rt):
        self.rr(self.A.OP_ADD, rd, rs, rt)

    def sub(self, rd, rs, rt):
        self.rr(self.A.OP_SUB, rd, rs, rt)

    def and_(self, rd, rs, rt):
        self.rr(self.A.OP_AND, rd, rs, rt)

    def or_(self, rd, rs, rt):
        self.rr(self.A.OP_OR, rd, rs, rt)

    def xor(self, rd, rs, rt):
        self.rr(self.A.OP_XOR, rd, rs, rt)

    def sltu(self, rd, rs, rt):
        self.rr(self.A.OP_SLTU, rd, rs, rt)

    def sll(self, rd, rs, sh):
        self.e(self.A.OP_SLL, rd, rs, sh, 0, 1)

    def srl(self, rd, rs, sh):
        self.e(self.A.OP_SRL, rd, rs, sh, 0, 1)

    def ror(self, rd, rs, sh):
        self.e(self.A.OP_ROR, rd, rs, sh, 0, 1)

    def bswap(self, rd, rs):  # WSBH + ROTR 16: the byte-reversed word (big-endian load)
        self.e(self.MC.OP_WSBH, rd, rs, 0, 0, 1)
        self.ror(rd, rd, 16)

    def movn(self, rd, rs, rt):  # rd = rs if rt != 0
        self.e(self.MC.OP_MNE, rd, rs, rt, 0, 0)

    def nop(self):
        self.sll(0, 0, 0)

    # --- memory ---
    def lw(self, rt, base, off):
        self.e(self.MC.OP_LW, rt, base, int(off) & M32, 0, 1)

    def sw(self, rt, base, off):
        self.e(self.MC.OP_SW, rt, base, int(off) & M32, 0, 1)

    def store_words(self, addr: int, words: Sequence[int], tmp: int = 8):
        """Input data: constant words written to memory (the guest's read of its input stream)."""
        for i, w in enumerate(words):
            self.li(tmp, w)
            self.sw(tmp, 0, addr + 4 * i)

    # --- control ---
    def label(self, name: str):
        self.labels[name] = len(self.p)

    def bne(self, rs, rt, name: str):
        """bne rs, rt, name; the caller emits the delay slot next."""
        self.fix.append((len(self.p), name))
        self.e(self.MC.OP_BNE, rs, rt, 0, 0, 1)

    def syscall(self, code: int, a0: Optional[int] = None, a1: Optional[int] = None, a0_reg=None, a1_reg=None):
        SY = self.SY
        self.li(SY.REG_V0, code)
        if a0_reg is not None:
            self.addi(SY.REG_A0, a0_reg, 0)
        elif a0 is not None:
            self.li(SY.REG_A0, a0)
        if a1_reg is not None:
            self.addi(SY.REG_A1, a1_reg, 0)
        elif a1 is not None:
            self.li(SY.REG_A1, a1)
        self.e(SY.OP_SYSCALL, SY.REG_V0, SY.REG_A0, SY.REG_A1, 0, 0)

    def program(self) -> List[tuple]:
        p = list(self.p)
        for at, name in self.fix:
            # target = next_pc + c, next_pc = pc + 4 (the delay slot)
            off = 4 * (self.labels[name] - (at + 1))
            op, a, b, _, ib, ic = p[at]
            p[at] = (op, a, b, off & M32, ib, ic)
        return p


# registers of the routines (r0 zero; r2/r4/r5 are the syscall's V0/A0/A1)
_T = [3, 24, 25, 26, 29, 6, 7, 2, 4, 5]  # temporaries
_ST = list(range(8, 24))                # SHA-512 working variables a..h as (hi, lo) pairs
R_PTR_K, R_PTR_W, R_CNT, R_ACC = 27, 28, 30, 31


def _add64(a: Asm, dh, dl, sh, sl, carry):
    """(dh, dl) += (sh, sl) (mod 2^64) with a carry temporary."""
    a.add(dl, dl, sl)
    a.sltu(carry, dl, sl)
    a.add(dh, dh, sh)
    a.add(dh, dh, carry)


def _rotr64(a: Asm, oh, ol, xh, xl, n, t):
    """(oh, ol) = rotr((xh, xl), n), 0 < n < 64, n != 32; one temporary t."""
    if n > 32:
        xh, xl, n = xl, xh, n - 32
    a.srl(oh, xh, n)
    a.sll(t, xl, 32 - n)
    a.or_(oh, oh, t)
    a.srl(ol, xl, n)
    a.sll(t, xh, 32 - n)
    a.or_(ol, ol, t)


def _shr64(a: Asm, oh, ol, xh, xl, n, t):
    a.srl(ol, xl, n)
    a.sll(t, xh, 32 - n)
    a.or_(ol, ol, t)
    a.srl(oh, xh, n)


def _sigma64(a: Asm, oh, ol, xh, xl, rots, shr, t):
    """xor of rotr(x, r) for r in rots (and shr(x, shr) when given) into (oh, ol); temporaries t[0..2]."""
    _rotr64(a, oh, ol, xh, xl, rots[0], t[0])
    for k, r in enumerate(list(rots[1:]) + ([None] if shr else [])):
        if r is None:
            _shr64(a, t[1], t[2], xh, xl, shr, t[0])
        else:
            _rotr64(a, t[1], t[2], xh, xl, r, t[0])
        a.xor(oh, oh, t[1])
        a.xor(ol, ol, t[2])


class Sha512:
    """SHA-512 (FIPS 180-4) in MIPS: the message schedule and the 80 rounds are loops (8 rounds unrolled
    per iteration, the working variables renamed instead of moved), 64-bit words as (hi, lo) register
    pairs.  Buffers: K (rodata), W (80 words), H (8 words) allocated once and reused."""

    def __init__(self, a: Asm):
        self.a = a
        self.k_ptr = a.alloc(160, 8)
        self.w_ptr = a.alloc(160, 8)
        self.h_ptr = a.alloc(16, 8)
        a.store_words(self.k_ptr, [w for k in SHA512_K for w in (k >> 32, k & M32)])
        self.n = 0

    def hash(self, msg_ptr: int, n_blocks: int):
        """H = SHA-512 of the padded message at msg_ptr (n_blocks x 32 little-endian words as in memory)."""
        a = self.a
        a.store_words(self.h_ptr, [w for h in SHA512_H0 for w in (h >> 32, h & M32)])
        for blk in range(n_blocks):
            self._block(msg_ptr + 128 * blk)

    def _block(self, src: int):
        a, t = self.a, _T
        tag = f"sha512_{self.n}"
        self.n += 1
        # W[0..15]: big-endian 64-bit words of the block
        for i in range(32):
            a.lw(t[0], 0, src + 4 * i)
            a.bswap(t[0], t[0])
            a.sw(t[0], 0, self.w_ptr + 4 * i)
        # W[16..79] = s1(W[t-2]) + W[t-7] + s0(W[t-15]) + W[t-16]
        a.li(R_PTR_W, self.w_ptr + 8 * 16)
        a.li(R_CNT, 64)
        a.label(tag + "_sched")
        h0, l0, h1, l1 = 8, 9, 10, 11
        a.lw(t[4], R_PTR_W, -16)
        a.lw(t[5], R_PTR_W, -12)
        _sigma64(a, h0, l0, t[4], t[5], (19, 61), 6, t[:3])
        a.lw(t[4], R_PTR_W, -120)
        a.lw(t[5], R_PTR_W, -116)
        _sigma64(a, h1, l1, t[4], t[5], (1, 8), 7, t[:3])
        _add64(a, h0, l0, h1, l1, t[0])
        a.lw(t[4], R_PTR_W, -56)
        a.lw(t[5], R_PTR_W, -52)
        _add64(a, h0, l0, t[4], t[5], t[0])
        a.lw(t[4], R_PTR_W, -128)
        a.lw(t[5], R_PTR_W, -124)
        _add64(a, h0, l0, t[4], t[5], t[0])
        a.sw(h0, R_PTR_W, 0)
        a.sw(l0, R_PTR_W, 4)
        a.addi(R_CNT, R_CNT, -1)
        a.bne(R_CNT, 0, tag + "_sched")
        a.addi(R_PTR_W, R_PTR_W, 8)  # delay slot
        # working variables from H
        for i in range(16):
            a.lw(_ST[i], 0, self.h_ptr + 4 * i)
        a.li(R_PTR_K, self.k_ptr)
        a.li(R_PTR_W, self.w_ptr)
        a.li(R_CNT, 10)
        a.label(tag + "_rounds")
        for r in range(8):
            v = [(_ST[2 * ((i - r) % 8)], _ST[2 * ((i - r) % 8) + 1]) for i in range(8)]  # a..h this round
            (ah, al), (bh, bl), (ch, cl), (dh, dl), (eh, el), (fh, fl), (gh, gl), (hh, hl) = v
            t1h, t1l = t[3], t[4]
            # T1 = h + S1(e) + Ch(e, f, g) + K[t] + W[t]
            _sigma64(a, t1h, t1l, eh, el, (14, 18, 41), None, t[:3])
            _add64(a, t1h, t1l, hh, hl, t[0])
            a.xor(t[1], fh, gh)
            a.xor(t[2], fl, gl)
            a.and_(t[1], t[1], eh)
            a.and_(t[2], t[2], el)
            a.xor(t[1], t[1], gh)
            a.xor(t[2], t[2], gl)
            _add64(a, t1h, t1l, t[1], t[2], t[0])
            a.lw(t[1], R_PTR_K, 8 * r)
            a.lw(t[2], R_PTR_K, 8 * r + 4)
            _add64(a, t1h, t1l, t[1], t[2], t[0])
            a.lw(t[1], R_PTR_W, 8 * r)
            a.lw(t[2], R_PTR_W, 8 * r + 4)
            _add64(a, t1h, t1l, t[1], t[2], t[0])
            # d += T1; h = T1 + S0(a) + Maj(a, b, c)
            _add64(a, dh, dl, t1h, t1l, t[0])
            _sigma64(a, t[5], t[6], ah, al, (28, 34, 39), None, t[:3])
            _add64(a, t1h, t1l, t[5], t[6], t[0])
            a.or_(t[1], ah, bh)
            a.or_(t[2], al, bl)
            a.and_(t[1], t[1], ch)
            a.and_(t[2], t[2], cl)
            a.and_(t[5], ah, bh)
            a.and_(t[6], al, bl)
            a.or_(t[1], t[1], t[5])
            a.or_(t[2], t[2], t[6])
            _add64(a, t1h, t1l, t[1], t[2], t[0])
            a.addi(hh, t1h, 0)
            a.addi(hl, t1l, 0)
        a.addi(R_PTR_K, R_PTR_K, 64)
        a.addi(R_CNT, R_CNT, -1)
        a.bne(R_CNT, 0, tag + "_rounds")
        a.addi(R_PTR_W, R_PTR_W, 64)  # delay slot
        # H += working variables
        for i in range(8):
            a.lw(t[1], 0, self.h_ptr + 8 * i)
            a.lw(t[2], 0, self.h_ptr + 8 * i + 4)
            _add64(a, t[1], t[2], _ST[2 * i], _ST[2 * i + 1], t[0])
            a.sw(t[1], 0, self.h_ptr + 8 * i)
            a.sw(t[2], 0, self.h_ptr + 8 * i + 4)


def _sha512_padded_words(msg: bytes) -> List[int]:
    m = msg + b"\x80" + b"\0" * ((111 - len(msg)) % 128) + (8 * len(msg)).to_bytes(16, "big")
    return _le_words(m)


class Sha256:
    """SHA-256 through the precompiles: the 16 message words of a block (big-endian u32 values, as the
    guest's sha2 crate hands them over) go into a 64-word W buffer, SHA_EXTEND fills W[16..64], and
    SHA_COMPRESS updates an 8-word state in memory, which is also where the digest stays."""

    def __init__(self, a: Asm):
        from . import mips_core as MC
        self.a, self.MC = a, MC
        self.w_ptr = a.alloc(64)

    def init(self) -> int:
        st = self.a.alloc(8)
        self.a.store_words(st, self.MC.SHA_H0)
        return st

    def block(self, st: int):
        """Extend + compress the block already in W[0..16]."""
        SY = self.a.SY
        self.a.syscall(SY.SHA_EXTEND, self.w_ptr, 0)
        self.a.syscall(SY.SHA_COMPRESS, self.w_ptr, st)

    def hash_le_bytes(self, msg_ptr: int, n_blocks: int) -> int:
        """Digest of a padded message lying in memory as bytes (little-endian words): each word loaded,
        byte-reversed into the big-endian word SHA-256 reads."""
        a, t = self.a, _T
        st = self.init()
        for b in range(n_blocks):
            for i in range(16):
                a.lw(t[0], 0, msg_ptr + 64 * b + 4 * i)
                a.bswap(t[0], t[0])
                a.sw(t[0], 0, self.w_ptr + 4 * i)
            self.block(st)
        return st

    def inner(self, l_ptr: int, r_ptr: int) -> int:
        """Merkle inner node SHA-256(0x01 || l || r) of two digests in memory (8 big-endian-valued words
        each): 65 bytes, so every word of the message straddles two digest words."""
        a, t = self.a, _T
        st = self.init()
        src = [("k", 0x01)] + [("l", i) for i in range(8)] + [("r", i) for i in range(8)]
        # the 65-byte message as 17 units; word j of block 1 = (u_j << 24) | (u_{j+1} >> 8) with u_0 the
        # prefix byte (shifted out entirely) -- i.e. (prev << 24) | (cur >> 8) over the digest words
        a.li(t[1], 0x01)  # prev = the prefix byte
        for j in range(16):
            kind, i = src[j + 1]
            a.lw(t[2], 0, (l_ptr if kind == "l" else r_ptr) + 4 * i)
            a.sll(t[3], t[1], 24)
            a.srl(t[4], t[2], 8)
            a.or_(t[3], t[3], t[4])
            a.sw(t[3], 0, self.w_ptr + 4 * j)
            a.addi(t[1], t[2], 0)
        self.block(st)
        a.sll(t[3], t[1], 24)  # block 2: r7's last byte, the 0x80 pad, zeros, the bit length 520
        a.li(t[4], 0x00800000)
        a.or_(t[3], t[3], t[4])
        a.sw(t[3], 0, self.w_ptr)
        for j in range(1, 15):
            a.sw(0, 0, self.w_ptr + 4 * j)
        a.li(t[3], 65 * 8)
        a.sw(t[3], 0, self.w_ptr + 60)
        self.block(st)
        return st

    def merkle(self, leaves: Sequence[int]) -> int:
        """crypto/merkle HashFromByteSlices over digests of already-hashed leaves (pointers)."""
        if len(leaves) == 1:
            return leaves[0]
        k = split_point(len(leaves))
        return self.inner(self.merkle(leaves[:k]), self.merkle(leaves[k:]))


def _store_le_message(a: Asm, msg: bytes, block: int) -> Tuple[int, int]:
    """Input bytes, padded (SHA-256 style when block == 64), stored as little-endian words."""
    m = msg + b"\x80" + b"\0" * ((block - 9 - len(msg)) % block) + (8 * len(msg)).to_bytes(8, "big")
    w = _le_words(m)
    ptr = a.alloc(len(w))
    a.store_words(ptr, w)
    return ptr, len(m) // block


def _xor_acc(a: Asm, x_ptr: int, y_words: Optional[Sequence[int]] = None, y_ptr: Optional[int] = None, n: int = 8,
             bswap_x: bool = False):
    """ACC |= x xor y over n words (y constants or memory): a failed check leaves ACC nonzero."""
    t = _T
    for i in range(n):
        a.lw(t[0], 0, x_ptr + 4 * i)
        if bswap_x:
            a.bswap(t[0], t[0])
        if y_ptr is not None:
            a.lw(t[1], 0, y_ptr + 4 * i)
        else:
            a.li(t[1], y_words[i])
        a.xor(t[0], t[0], t[1])
        a.or_(R_ACC, R_ACC, t[0])


def _be_words(b: bytes) -> List[int]:
    return [int.from_bytes(b[i:i + 4], "big") for i in range(0, len(b), 4)]


class Validators:
    """One validator set as the guest holds it: each validator's SimpleValidator leaf message (input bytes,
    0x00 prefix and padding included) in memory; the leaf digests; the Ed25519 key (32 bytes at offset 5 of
    the message, re-aligned by the guest) and the voting power (the varint at offset 38, decoded by the
    guest) pulled out of those same bytes."""

    def __init__(self, a: Asm, sha: Sha256, vset: dict, need_keys: bool, need_powers: bool):
        self.leaves, self.keys, self.power_regs = [], [], []
        self.powers_ptr = a.alloc(len(vset["validators"]))
        t = _T
        for i, v in enumerate(vset["validators"]):
            item = validator_bytes(v)
            assert item[:4] == b"\x0a\x22\x0a\x20", "SimpleValidator layout"
            msg = b"\x00" + item
            ptr, nb = _store_le_message(a, msg, 64)
            self.leaves.append(sha.hash_le_bytes(ptr, nb))
            if need_keys:  # bytes 5..36 of the message: word k = (m[1+k] >> 8) | (m[2+k] << 24)
                kp = a.alloc(8)
                for k in range(8):
                    a.lw(t[0], 0, ptr + 4 * (1 + k))
                    a.lw(t[1], 0, ptr + 4 * (2 + k))
                    a.srl(t[0], t[0], 8)
                    a.sll(t[1], t[1], 24)
                    a.or_(t[0], t[0], t[1])
                    a.sw(t[0], 0, kp + 4 * k)
                self.keys.append(kp)
            if need_powers:  # 0x10 at byte 37, the varint from byte 38
                n = len(item) - 37
                assert item[36] == 0x10 and 1 <= n <= 5
                a.li(t[2], 0)
                for j in range(n):
                    byte = 38 + j
                    a.lw(t[0], 0, ptr + 4 * (byte // 4))
                    a.srl(t[0], t[0], 8 * (byte % 4))
                    a.li(t[1], 0x7F)
                    a.and_(t[0], t[0], t[1])
                    a.sll(t[0], t[0], 7 * j)
                    a.or_(t[2], t[2], t[0])
                a.sw(t[2], 0, self.powers_ptr + 4 * i)
        self.root = sha.merkle(self.leaves)


# Ed25519 constants (the curve25519 field, the group order, 2^256 mod L)
def _ed_consts():
    from .mips_edwards import BASE_X, BASE_Y, ED_L, ED_P
    return ED_P, ED_L, BASE_X, BASE_Y


def _int_words(x: int, n: int = 8) -> List[int]:
    return [(x >> (32 * i)) & M32 for i in range(n)]


class Ed25519:
    """Signature check [S]B == R + [k]A (k = SHA-512(R || A || M) mod L) with the precompiles: A and R
    decompressed by ED_DECOMPRESS, the sum [S]B + [k](-A) by one double-and-add over both scalars
    (Shamir's trick: per bit one ED_ADD doubling and one ED_ADD of table[2 s_i + k_i] with table
    (O, -A, B, B - A), the identity included so the syscall sequence does not depend on the bits), k
    reduced mod L with UINT256_MUL."""

    def __init__(self, a: Asm, sha512: Sha512):
        from . import mips_ec as EC
        from . import mips_edwards as ED
        self.a, self.sha, self.EC, self.ED = a, sha512, EC, ED
        P, L, bx, by = _ed_consts()
        self.P, self.L = P, L
        self.table = a.alloc(64)          # 4 points x 16 words
        self.acc = a.alloc(16)
        self.pa = a.alloc(16)             # A: (x, y)
        self.pr = a.alloc(16)             # R: (x, y)
        self.msg = a.alloc(64, 8)         # the SHA-512 message: R || A || M || padding (2 blocks)
        self.x1, self.x2, self.x3 = a.alloc(8), a.alloc(8), a.alloc(8)
        self.y_c = a.alloc(16)            # (2^256 mod L, L)
        self.y_1 = a.alloc(16)            # (1, L)
        self.p_words = a.alloc(8)
        self.l_words = a.alloc(8)
        a.store_words(self.y_c, _int_words((1 << 256) % L) + _int_words(L))
        a.store_words(self.y_1, _int_words(1) + _int_words(L))
        a.store_words(self.p_words, _int_words(P))
        a.store_words(self.l_words, _int_words(L))
        a.store_words(self.table, [0] * 8 + _int_words(1) + [0] * 16 + _int_words(bx) + _int_words(by) + [0] * 16)
        self.n = 0

    def _decompress(self, dst: int, enc_ptr: int):
        """dst = (x, y) of a 32-byte encoding: y = enc with bit 255 cleared, sign = bit 255."""
        a, t = self.a, _T
        for k in range(8):
            a.lw(t[0], 0, enc_ptr + 4 * k)
            if k == 7:
                a.srl(t[5], t[0], 31)
                a.sll(t[0], t[0], 1)
                a.srl(t[0], t[0], 1)
            a.sw(t[0], 0, dst + 32 + 4 * k)
        a.syscall(self.ED.ED_DECOMPRESS, dst, a1_reg=t[5])

    def _sub_from(self, dst: int, m_ptr: int, x_ptr: int):
        """dst = m - x over 8 limbs (x <= m)."""
        a, t = self.a, _T
        a.li(t[3], 0)  # borrow
        for k in range(8):
            a.lw(t[0], 0, m_ptr + 4 * k)
            a.lw(t[1], 0, x_ptr + 4 * k)
            a.sub(t[2], t[0], t[1])
            a.sltu(t[4], t[0], t[1])
            a.sltu(t[6], t[2], t[3])
            a.sub(t[2], t[2], t[3])
            a.or_(t[3], t[4], t[6])
            a.sw(t[2], 0, dst + 4 * k)
        return t[3]

    def verify(self, a_ptr: int, sig_ptr: int, m_words: Sequence[int], hash_at: Optional[Tuple[int, int]] = None):
        """One signature: key words at a_ptr, signature (R || S) words at sig_ptr, the rest of the
        SHA-512 message (M and padding, from word 16 on) as input words; `hash_at` = (word offset in the
        message, digest pointer): those 8 message words are written from a digest the guest computed
        (the commit's block id = the header hash)."""
        a, t = self.a, _T
        tag = f"ed_{self.n}"
        self.n += 1
        # the SHA-512 message: R, A copied; M stored; the block id from the computed header hash
        for k in range(8):
            a.lw(t[0], 0, sig_ptr + 4 * k)
            a.sw(t[0], 0, self.msg + 4 * k)
            a.lw(t[0], 0, a_ptr + 4 * k)
            a.sw(t[0], 0, self.msg + 32 + 4 * k)
        a.store_words(self.msg + 64, m_words)
        if hash_at is not None:
            off, dptr = hash_at
            for k in range(8):
                a.lw(t[0], 0, dptr + 4 * k)
                a.bswap(t[0], t[0])
                a.sw(t[0], 0, self.msg + 4 * (off + k))
        self.sha.hash(self.msg, (64 + 4 * len(m_words)) // 128)
        # k = (k_hi (2^256 mod L) + k_lo) mod L over the little-endian digest
        h = self.sha.h_ptr
        for k in range(8):
            a.lw(t[0], 0, h + 4 * k)
            a.bswap(t[0], t[0])
            a.sw(t[0], 0, self.x2 + 4 * k)
            a.lw(t[0], 0, h + 32 + 4 * k)
            a.bswap(t[0], t[0])
            a.sw(t[0], 0, self.x1 + 4 * k)
        EC = self.EC
        a.syscall(EC.UINT256_MUL, self.x1, self.y_c)
        a.syscall(EC.UINT256_MUL, self.x2, self.y_1)
        a.li(t[3], 0)  # carry
        for k in range(8):
            a.lw(t[0], 0, self.x1 + 4 * k)
            a.lw(t[1], 0, self.x2 + 4 * k)
            a.add(t[2], t[0], t[1])
            a.sltu(t[4], t[2], t[0])
            a.add(t[2], t[2], t[3])
            a.sltu(t[6], t[2], t[3])
            a.or_(t[3], t[4], t[6])
            a.sw(t[2], 0, self.x3 + 4 * k)
        a.syscall(EC.UINT256_MUL, self.x3, self.y_1)
        # S < L (the canonical-scalar check): S - L must borrow
        borrow = self._sub_from(self.x1, sig_ptr + 32, self.l_words)
        a.li(t[0], 1)
        a.xor(t[0], t[0], borrow)
        a.or_(R_ACC, R_ACC, t[0])
        # table: (O, -A, B, B - A); acc = O
        self._decompress(self.pa, a_ptr)
        self._decompress(self.pr, sig_ptr)
        ta = self.table + 64
        self._sub_from(ta, self.p_words, self.pa)
        for k in range(8):
            a.lw(t[0], 0, self.pa + 32 + 4 * k)
            a.sw(t[0], 0, ta + 32 + 4 * k)
        for k in range(16):
            a.lw(t[0], 0, ta + 4 * k)
            a.sw(t[0], 0, self.table + 192 + 4 * k)
        a.syscall(self.ED.ED_ADD, self.table + 192, self.table + 128)
        for k in range(16):
            a.lw(t[0], 0, self.table + 4 * k)
            a.sw(t[0], 0, self.acc + 4 * k)
        # double-and-add over bits 252..0 of S (-> B) and k (-> -A), limb by limb from the top
        rs, rk, rb = 8, 9, 10
        a.li(rb, self.table)
        for limb in range(7, -1, -1):
            a.lw(rs, 0, sig_ptr + 32 + 4 * limb)
            a.lw(rk, 0, self.x3 + 4 * limb)
            nb = 29 if limb == 7 else 32
            if nb < 32:
                a.sll(rs, rs, 32 - nb)
                a.sll(rk, rk, 32 - nb)
            a.li(R_CNT, nb)
            a.label(f"{tag}_{limb}")
            a.syscall(self.ED.ED_ADD, self.acc, self.acc)
            a.srl(t[0], rs, 31)
            a.sll(t[0], t[0], 1)
            a.srl(t[1], rk, 31)
            a.or_(t[0], t[0], t[1])
            a.sll(t[0], t[0], 6)
            a.add(t[0], t[0], rb)
            a.syscall(self.ED.ED_ADD, self.acc, a1_reg=t[0])
            a.sll(rs, rs, 1)
            a.sll(rk, rk, 1)
            a.addi(R_CNT, R_CNT, -1)
            a.bne(R_CNT, 0, f"{tag}_{limb}")
            a.nop()
        _xor_acc(a, self.acc, y_ptr=self.pr, n=16)


def tendermint_program(trusted: dict, untrusted: dict, votes: Optional[slice] = None,
                       tamper: Optional[int] = None) -> Tuple[List[tuple], dict]:
    """The guest of examples/tendermint (module docstring) for the two light blocks: MIPS instructions for
    this repository's executor (mips_core).  ACC (r31) collects every failed comparison; the exit code is
    ACC, so a verifying execution halts with 0.  Returns (program, expected) with the public values the
    reference host expects (header hash 1 || header hash 2 || CBOR verdict) and their SHA-256 digest.
    Tests only: `votes` restricts the signature checks to a slice of the votes (the voting-power thresholds
    are then skipped), `tamper` flips a bit of that vote's signature."""
    from . import mips_core as MC
    from . import mips_syscall as SY
    a = Asm(MC.DATA_BASE + 0x1000)
    sha = Sha256(a)
    sha512 = Sha512(a)
    ed = Ed25519(a, sha512)
    t = _T
    a.li(R_ACC, 0)
    # 1. header hashes
    hh = []
    for blk in (trusted, untrusted):
        leaves = []
        for f in header_fields(blk["signed_header"]["header"]):
            ptr, nb = _store_le_message(a, b"\x00" + f, 64)
            leaves.append(sha.hash_le_bytes(ptr, nb))
        hh.append(sha.merkle(leaves))
    commit = untrusted["signed_header"]["commit"]
    _xor_acc(a, hh[1], _be_words(bytes.fromhex(commit["block_id"]["hash"])))  # commit.block_id = header hash
    # 2./3. validator sets: the trusted next set must hash to the trusted header's next_validators_hash;
    # the untrusted sets to what the untrusted header says
    tn = Validators(a, sha, trusted["next_validator_set"], True, True)
    uv = Validators(a, sha, untrusted["validator_set"], True, True)
    un = Validators(a, sha, untrusted["next_validator_set"], False, False)
    th, uh = trusted["signed_header"]["header"], untrusted["signed_header"]["header"]
    _xor_acc(a, tn.root, _be_words(bytes.fromhex(th["next_validators_hash"])))
    _xor_acc(a, uv.root, _be_words(bytes.fromhex(uh["validators_hash"])))
    _xor_acc(a, un.root, _be_words(bytes.fromhex(uh["next_validators_hash"])))
    # 4. the votes: each signature verified, committed power tallied (untrusted set, and the trusted next
    # set's power of the same validator: same key, checked)
    by_addr = {v["address"]: i for i, v in enumerate(untrusted["validator_set"]["validators"])}
    t_keys = [base64.b64decode(v["pub_key"]["value"]) for v in trusted["next_validator_set"]["validators"]]
    t_index = {k: i for i, k in enumerate(t_keys)}
    tal = a.alloc(2)  # the two tallies live in memory (SHA-512 uses every spare register)
    full = votes is None
    votes = signed_votes(untrusted)[votes if votes is not None else slice(None)]
    sig_bufs = []
    for n, v in enumerate(votes):
        sp = a.alloc(16)
        sig = bytearray(v["sig"])
        if tamper is not None and n == tamper:
            sig[33] ^= 0x10  # in S: R stays a curve point, [S]B no longer equals R + [k]A
        a.store_words(sp, _le_words(bytes(sig)))
        sig_bufs.append(sp)
    a.sw(0, 0, tal)
    a.sw(0, 0, tal + 4)
    for v, sp in zip(votes, sig_bufs):
        i = by_addr[v["address"]]
        m = v["msg"]
        mw = _le_words(_sha512_tail(v["sig"][:32] + v["pub"] + m)[64:])
        hash_at = (20, hh[1]) if v["commit"] else None
        if v["commit"]:
            assert m[14:16] == b"\x0a\x20" and m[16:48] == bytes.fromhex(commit["block_id"]["hash"])
        ed.verify(uv.keys[i], sp, mw, hash_at)  # the signature as input, R || S
        if v["commit"]:
            for k, (pw, idx) in enumerate(((uv.powers_ptr, i), (tn.powers_ptr, t_index.get(v["pub"])))):
                if idx is None:
                    continue
                if k == 1:  # the trusted next set's entry for this key: its key words equal uv's
                    _xor_acc(a, tn.keys[idx], y_ptr=uv.keys[i])
                a.lw(t[0], 0, pw + 4 * idx)
                a.lw(t[1], 0, tal + 4 * k)
                a.add(t[1], t[1], t[0])
                a.sw(t[1], 0, tal + 4 * k)
    # thresholds: 3 tallied > 2 total (untrusted), 3 trusted_tallied > trusted_total (trust level 1/3)
    for pw, n, k, num in ((uv.powers_ptr, len(untrusted["validator_set"]["validators"]), 0, 2),
                          (tn.powers_ptr, len(trusted["next_validator_set"]["validators"]), 1, 1)) if full else ():
        reg = t[7]
        a.lw(reg, 0, tal + 4 * k)
        a.li(t[2], 0)
        for i in range(n):
            a.lw(t[0], 0, pw + 4 * i)
            a.add(t[2], t[2], t[0])
        a.add(t[3], reg, reg)
        a.add(t[3], t[3], reg)      # 3 tallied
        a.addi(t[4], t[2], 0)
        if num == 2:
            a.add(t[4], t[4], t[2])  # 2 total
        a.sltu(t[5], t[4], t[3])
        a.li(t[6], 1)
        a.xor(t[5], t[5], t[6])
        a.or_(R_ACC, R_ACC, t[5])
    # 5. public values: hh1 || hh2 || cbor(Success); the digest committed word by word (halt.rs)
    pv = a.alloc(18)
    for k in range(2):
        for w in range(8):
            a.lw(t[0], 0, hh[k] + 4 * w)
            a.bswap(t[0], t[0])
            a.sw(t[0], 0, pv + 32 * k + 4 * w)
    a.store_words(pv + 64, _le_words(VERDICT_SUCCESS_CBOR))
    pv_bytes_len = 72
    # padded message: the 72 bytes, 0x80, zeros, length (2 blocks) -- assembled around the computed words
    tail = _le_words((b"\x80" + b"\0" * ((55 - pv_bytes_len) % 64) + (8 * pv_bytes_len).to_bytes(8, "big")))
    pmsg = a.alloc(32)
    for w in range(18):
        a.lw(t[0], 0, pv + 4 * w)
        a.sw(t[0], 0, pmsg + 4 * w)
    a.store_words(pmsg + 72, tail)
    dig = sha.hash_le_bytes(pmsg, 2)
    for w in range(8):
        a.lw(t[0], 0, dig + 4 * w)
        a.bswap(SY.REG_A1, t[0])
        a.li(SY.REG_A0, w)
        a.li(SY.REG_V0, SY.COMMIT)
        a.e(SY.OP_SYSCALL, SY.REG_V0, SY.REG_A0, SY.REG_A1, 0, 0)
    for w in range(8):
        a.syscall(SY.COMMIT_DEFERRED_PROOFS, w, 0)
    a.li(SY.REG_V0, SY.HALT)
    a.addi(SY.REG_A0, R_ACC, 0)
    a.e(SY.OP_SYSCALL, SY.REG_V0, SY.REG_A0, SY.REG_A1, 0, 0)
    assert a.brk < MC.PC_BASE, "guest data overlaps the program"
    pv_stream = header_hash(trusted) + header_hash(untrusted) + VERDICT_SUCCESS_CBOR
    expected = {"public_values": pv_stream, "digest": hashlib.sha256(pv_stream).digest(), "votes": len(votes),
                "data_bytes": a.brk - MC.DATA_BASE}
    return a.program(), expected


def _sha512_tail(msg: bytes) -> bytes:
    return msg + b"\x80" + b"\0" * ((111 - len(msg)) % 128) + (8 * len(msg)).to_bytes(16, "big")


def tendermint_shards(shard_size: int = 1 << 21, precompile_events_per_shard: int = 1 << 14, seed: int = 1):
    """The whole execution of the tendermint guest on the reference's two blocks as continuation shards
    (mips_core.program_shards: CPU shards, the SHA_EXTEND / SHA_COMPRESS / ED_ADD / ED_DECOMPRESS /
    UINT256_MUL precompile shards, the memory shard).  Returns (shards, info); info carries the expected
    public-values digest, which the last CPU shard's committed digest must equal (checked here), and the
    exit code (0: every check of the guest held)."""
    from . import mips_alu as A
    from . import mips_core as MC
    trusted, untrusted = load_block(2279100), load_block(2279130)
    prog, exp = tendermint_program(trusted, untrusted)
    shards = MC.program_shards(prog, seed=seed, shard_size=shard_size,
                               precompile_events_per_shard=precompile_events_per_shard)
    cpu = [s for s in shards if "Cpu" in s[2]]
    last = cpu[-1][3]
    words = [int.from_bytes(bytes(int(b) for b in last[4 * i:4 * i + 4]), "little") for i in range(8)]
    digest = b"".join(w.to_bytes(4, "little") for w in words)
    info = {"exit_code": int(last[MC.PV_EXIT_CODE]), "pv_digest": digest, "expected_digest": exp["digest"],
            "votes": exp["votes"], "public_values": exp["public_values"], "program_len": len(prog),
            "shards": len(shards)}
    if info["exit_code"] != 0 or digest != exp["digest"]:
        raise ValueError(f"tendermint guest failed: exit {info['exit_code']}, digest {digest.hex()} vs "
                         f"{exp['digest'].hex()}")
    del A
    return shards, info
