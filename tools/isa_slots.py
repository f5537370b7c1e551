"""Static VALU issue-slot count of one Poseidon2 permutation (the roofline model of bench.py).

Compiles zkmips_amd/csrc/merkle.hip for gfx950 (device only), disassembles k_p2_batch (one
permutation per thread, straight-line) and weights each VALU instruction by its measured issue cost
on MI355X (tools/probe/valu_probe.hip, profiles/r01_valu_probe.txt): v_add/v_sub/bitwise/v_mov run
at the full SIMD-32 rate (1 slot per wave64 instruction pair of cycles), everything else we use
(min/max, shifts, 32-bit multiplies, v_mad_u64_u32, v_lshl_add_u64, carry-out adds v_add_co/v_addc_co,
3-operand forms, DPP/SDWA forms) at half rate
(2 slots).  Writes profiles/<tag>_isa_p2.json and zkmips_amd/isa_p2.json.   python tools/isa_slots.py r01
"""
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "zkmips_amd", "csrc")
FULL = re.compile(r"^v_(add_u32|sub_u32|subrev_u32|and_b32|or_b32|xor_b32|mov_b32)(_e32|_e64)?$")


def main(tag):
    with tempfile.TemporaryDirectory() as td:
        obj = os.path.join(td, "m.o")
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-I",
                               os.path.join(CSRC, "build"), "-x", "hip", "--cuda-device-only",
                               "--no-gpu-bundle-output", "-c", os.path.join(CSRC, "merkle.hip"), "-o", obj])
        dis = subprocess.check_output(["/opt/rocm/lib/llvm/bin/llvm-objdump", "-d", obj], text=True)
    body, on = [], False
    for line in dis.splitlines():
        if re.match(r"^[0-9a-f]+ <", line):
            on = "k_p2_batchEPjm>" in line
            continue
        if on:
            m = re.match(r"^\s+([a-z0-9_]+)", line)
            if m:
                body.append(m.group(1))
    ops = collections.Counter(op for op in body if op.startswith("v_"))
    slots = sum(c * (1 if FULL.match(op) else 2) for op, c in ops.items())
    out = {"kernel": "k_p2_batch", "valu_instructions": sum(ops.values()), "issue_slots": slots,
           "full_rate_pattern": FULL.pattern, "by_op": dict(ops.most_common())}
    path = os.path.join(ROOT, "profiles", f"{tag}_isa_p2.json")
    json.dump(out, open(path, "w"), indent=1)
    # the copy bench.py reads on the GPU box (profiles/ does not travel there)
    json.dump(out, open(os.path.join(ROOT, "zkmips_amd", "isa_p2.json"), "w"), indent=1)
    print(path, out["valu_instructions"], slots)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
