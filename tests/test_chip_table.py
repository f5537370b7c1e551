"""Every restated MIPS chip pinned to reference-held data (CPU only).

For each chip: its shape (prep, main, perm EF columns, log quotient degree, local_only) as the machine
blob describes it, the reference `MachineAir` impl it restates, and its per-row cost
prep + main + 4*perm_EF + 4*2^log_qd (crates/stark/src/chip.rs:154-163) against the reference's own
`crates/core/executor/src/artifacts/mips_costs.json` (copied to tests/golden/ by make_ref_fixtures.py;
the reference checks the same file in mips/mod.rs:720-727).

`local_only` decides whether a chip's main trace is opened at zeta only or at zeta and g*zeta
(crates/stark/src/prover.rs:519-532, 577-590).  The default is false (crates/stark/src/air/machine.rs:77-79);
the chips marked True override it in the reference (file:line below).
"""
import json
import os

import numpy as np
import pytest

from tests import _oracle as O
from zkmips_amd import mips_alu as A
from zkmips_amd import mips_core as MC
from zkmips_amd import mips_ec as EC
from zkmips_amd import mips_p2permute as P2
from zkmips_amd import mips_keccak as K
from zkmips_amd import mips_edwards as ED
from zkmips_amd import mips_memory as MM
from zkmips_amd import mips_syscall as SY
from zkmips_amd.machine import MachineDesc

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
COSTS = json.load(open(os.path.join(GOLDEN, "mips_costs.json")))

# name: (builder, prep, main, perm_ef, log_qd, local_only, reference MachineAir impl, local_only override)
CHIPS = {
    "Cpu": (MC.cpu_chip, 0, 67, 11, 1, False, "cpu/trace.rs:20", None),
    "Program": (MC.program_chip, 14, 1, 2, 1, False, "program/mod.rs:53", None),
    "Byte": (A.byte_chip, 12, 10, 6, 1, False, "bytes/trace.rs:17", None),
    "AddSub": (A.add_sub_chip, 0, 19, 5, 1, True, "alu/add_sub/mod.rs:65", "alu/add_sub/mod.rs:145"),
    "Bitwise": (A.bitwise_chip, 0, 18, 4, 1, True, "alu/bitwise/mod.rs:61", "alu/bitwise/mod.rs:133"),
    "Lt": (A.lt_chip, 0, 36, 3, 1, True, "alu/lt/mod.rs:96", "alu/lt/mod.rs:172"),
    "ShiftLeft": (A.shift_left_chip, 0, 44, 4, 1, True, "alu/sll/mod.rs:102", "alu/sll/mod.rs:193"),
    "ShiftRight": (A.shift_right_chip, 0, 71, 14, 1, False, "alu/sr/mod.rs:139", None),
    "CloClz": (A.clo_clz_chip, 0, 22, 4, 1, False, "alu/clo_clz/mod.rs:75", None),
    "Mul": (MC.mul_chip, 0, 58, 11, 1, True, "alu/mul/mod.rs:138", "alu/mul/mod.rs:214"),
    "DivRem": (MC.divrem_chip, 0, 106, 12, 1, True, "alu/divrem/mod.rs:199", "alu/divrem/mod.rs:360"),
    "Branch": (MC.branch_chip, 0, 62, 5, 1, True, "control_flow/branch/trace.rs:21", "control_flow/branch/trace.rs:76"),
    "Jump": (MC.jump_chip, 0, 66, 2, 1, True, "control_flow/jump/trace.rs:21", "control_flow/jump/trace.rs:76"),
    "MovCond": (MC.movcond_chip, 0, 32, 2, 1, True, "misc/mov_cond/mod.rs:64", "misc/mov_cond/mod.rs:119"),
    "MemoryInstrs": (MC.memory_instructions_chip, 0, 79, 7, 1, True, "memory/instructions/trace.rs:25",
                     "memory/instructions/trace.rs:82"),
    "MiscInstrs": (MC.misc_instructions_chip, 0, 72, 17, 1, False, "misc/others/trace.rs:24", None),
    "MemoryLocal": (MM.memory_local_chip, 0, 56, 9, 1, False, "memory/local.rs:86", None),
    "Global": (MM.global_chip, 0, 99, 2, 1, False, "global/mod.rs:65", None),
    "MemoryGlobalInit": (lambda: MM.memory_global_chip(True), 0, 111, 2, 1, False, "memory/global.rs:48", None),
    "MemoryGlobalFinalize": (lambda: MM.memory_global_chip(False), 0, 111, 2, 1, False, "memory/global.rs:48",
                             None),
    "SyscallInstrs": (SY.syscall_instrs_chip, 0, 64, 2, 1, False, "syscall/instructions/trace.rs:25", None),
    "SyscallCore": (lambda: SY.syscall_chip(True), 0, 6, 2, 1, False, "syscall/chip.rs:78", None),
    "SyscallPrecompile": (lambda: SY.syscall_chip(False), 0, 6, 2, 1, False, "syscall/chip.rs:78", None),
    "ShaExtend": (SY.sha_extend_chip, 0, 176, 37, 1, False, "sha256/extend/trace.rs:18", None),
    "ShaCompress": (SY.sha_compress_chip, 0, 262, 59, 1, False, "sha256/compress/trace.rs:21", None),
    "SysLinux": (SY.sys_linux_chip, 0, 69, 12, 1, False, "sys_linux/trace.rs:21", None),
    "EdAddAssign": (ED.ed_add_chip, 0, 1861, 442, 1, True, "syscall/precompiles/edwards/ed_add.rs:103",
                    "syscall/precompiles/edwards/ed_add.rs:200"),
    "EdDecompress": (ED.ed_decompress_chip, 0, 1566, 372, 1, True, "syscall/precompiles/edwards/ed_decompress.rs:202",
                     "syscall/precompiles/edwards/ed_decompress.rs:262"),
}
_PRE = "syscall/precompiles/"
for _curve in ("Secp256k1", "Secp256r1", "Bn254", "Bls12381"):
    _big = _curve == "Bls12381"
    CHIPS[f"{_curve}AddAssign"] = (lambda c=_curve: EC.weierstrass_add_chip(c), 0, 3089 if _big else 2049,
                                   737 if _big else 489, 1, True, _PRE + "weierstrass/weierstrass_add.rs:127",
                                   _PRE + "weierstrass/weierstrass_add.rs:263")
    CHIPS[f"{_curve}DoubleAssign"] = (lambda c=_curve: EC.weierstrass_double_chip(c), 0, 3440 if _big else 2280,
                                      831 if _big else 551, 1, True, _PRE + "weierstrass/weierstrass_double.rs:142",
                                      _PRE + "weierstrass/weierstrass_double.rs:288")
for _field, _shape in (("Bn254", ((372, 81), (734, 160), (1485, 348))),
                       ("Bls12381", ((556, 121), (1102, 240), (2237, 524)))):
    CHIPS[EC.FP_NAME[_field]] = (lambda f=_field: EC.fp_op_chip(f), 0, *_shape[0], 1, True,
                                 _PRE + "fptower/fp.rs:76", _PRE + "fptower/fp.rs:192")
    CHIPS[EC.FP2_ADDSUB_NAME[_field]] = (lambda f=_field: EC.fp2_addsub_chip(f), 0, *_shape[1], 1, True,
                                         _PRE + "fptower/fp2_addsub.rs:79", _PRE + "fptower/fp2_addsub.rs:210")
    CHIPS[EC.FP2_MUL_NAME[_field]] = (lambda f=_field: EC.fp2_mul_chip(f), 0, *_shape[2], 1, True,
                                      _PRE + "fptower/fp2_mul.rs:122", _PRE + "fptower/fp2_mul.rs:227")
for _curve, _w, _perm in (("Secp256k1", 1378, 325), ("Secp256r1", 1378, 325), ("Bls12381", 2177, 491)):
    CHIPS[f"{_curve}Decompress"] = (lambda c=_curve: EC.weierstrass_decompress_chip(c), 0, _w, _perm, 1, True,
                                    _PRE + "weierstrass/weierstrass_decompress.rs:145",
                                    _PRE + "weierstrass/weierstrass_decompress.rs:304")
CHIPS["Poseidon2Permute"] = (P2.poseidon2_permute_chip, 0, 973, 34, 1, False, _PRE + "poseidon2/trace.rs:21", None)
CHIPS["KeccakSponge"] = (K.keccak_sponge_chip, 0, 3531, 180, 1, False, _PRE + "keccak_sponge/trace.rs:23", None)
CHIPS["U256XU2048Mul"] = (EC.u256x2048_mul_chip, 0, 3129, 678, 1, False, _PRE + "u256x2048_mul/air.rs:90", None)
CHIPS["Uint256MulMod"] = (EC.uint256_mul_chip, 0, 480, 98, 1, True, _PRE + "uint256/air.rs:93",
                          _PRE + "uint256/air.rs:218")
# precompile chips are costed per call: rows per event x per-row cost (mips/mod.rs:216-222)
ROWS_PER_EVENT = {"ShaExtend": 48, "ShaCompress": 80, "KeccakSponge": 24}


def _cost(ch):
    return ch.prep_width + ch.main_width + 4 * ch.perm_width_ef + 4 * (1 << ch.log_quotient_degree)


@pytest.mark.parametrize("name", sorted(CHIPS))
def test_chip_shape_and_cost(name):
    build, prep, main, perm, lqd, local_only, _impl, _override = CHIPS[name]
    ch = build()
    assert ch.name == name
    assert (ch.prep_width, ch.main_width, ch.perm_width_ef, ch.log_quotient_degree) == (prep, main, perm, lqd)
    assert ch.local_only is local_only
    cost = ROWS_PER_EVENT.get(name, 1) * _cost(ch)
    assert cost == COSTS[name], f"{name}: cost {cost} != mips_costs.json {COSTS[name]}"


def test_local_only_reaches_the_blob():
    """The machine blob carries each chip's local_only to the prover (and the oracle)."""
    chips = [CHIPS[n][0]() for n in sorted(CHIPS)]
    m = MachineDesc(chips, 8)
    mh = O.lib().orc_api_machine_new(m.blob(), m.blob().size)
    try:
        for i, n in enumerate(sorted(CHIPS)):
            info = np.zeros(7, np.int32)
            assert O.lib().orc_api_machine_info(mh, i, info) == 0
            assert (info[0], info[1], info[2], info[3]) == CHIPS[n][1:5]
            assert bool(info[5]) is CHIPS[n][5]
    finally:
        O.lib().orc_api_machine_free(mh)


def test_every_restated_chip_is_a_reference_chip():
    """Chips the shard builders put in a machine are reference chips (plus the documented stand-ins)."""
    stand_ins = {"InstrSource"}
    names = {c.name for c in MC.core_machine().chips}
    assert names - stand_ins <= set(COSTS)
    assert names - stand_ins <= set(CHIPS)


def test_dummy_vk_map_bytes_reproduced():
    """crates/prover/dummy_vk_map.bin, regenerated from its decoded entries with the proof serializer's
    conventions (u64 fixint lengths, [F;8] with no length, canonical u32 field elements, usize as u64),
    hashes to the reference file's sha256.  Montgomery encoding does not."""
    import hashlib
    d = json.load(open(os.path.join(GOLDEN, "dummy_vk_map.json")))
    assert d["rule_holds"]
    n = d["entries"]
    keys = np.repeat(np.arange(n, dtype=np.uint32)[:, None], 8, axis=1)
    vals = np.arange(n, dtype=np.uint64)
    b = O.serialize_digest_map(keys, vals)
    assert len(b) == d["bytes"]
    assert hashlib.sha256(b).hexdigest() == d["sha256"]
    bm = O.serialize_digest_map(keys, vals, montgomery=True)
    assert hashlib.sha256(bm).hexdigest() != d["sha256"]
    rec = np.frombuffer(b[8:], np.uint8).reshape(n, 40)
    assert [int(x) for x in rec[1, :32].copy().view("<u4")] + [int(rec[1, 32:].copy().view("<u8")[0])] == d["first"][1]


def test_maximal_shapes_fixture():
    """The reference's 2^22 shard compositions name only chips of mips_costs.json; each holds a
    Cpu of at most 2^22 rows and no chip taller than 2^22."""
    shapes = json.load(open(os.path.join(GOLDEN, "maximal_shapes_22.json")))
    assert len(shapes) == 175
    for s in shapes:
        assert set(s) <= set(COSTS)
        assert s["Cpu"] <= 22 and max(s.values()) <= 22
