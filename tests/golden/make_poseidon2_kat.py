"""Writes tests/golden/poseidon2_kat.json.

Provenance of the three vectors:
- ``perm_zeros`` (perm([0; 16])) is a literal in the reference itself: the expected output of the
  gnark Poseidon2-KoalaBear circuit test, crates/recursion/gnark-ffi/go/main.go:258-275
  (``expectedOutput`` of TestPoseidonKoalaBear2, main.go:237-275, input all zeros).  The strongest pin: reference-held
  data, independent of any build done here.
- ``perm_0_to_15`` and ``perm_ones`` are the values SURVEY.md §8c recorded from a build of the
  reference's C++ Poseidon2 (crates/recursion/core/include/poseidon2_wide.hpp populate_perm) in the
  survey container.  That build needed a stand-in for a cbindgen-generated header, so on its own it
  pins nothing; the vectors agree with an independent restatement from RC_16_30_U32
  (crates/primitives/src/lib.rs:563) and INTERNAL_DIAG_MONTY_16
  (crates/core/machine/src/operations/poseidon2/air.rs:12-29), and with perm_zeros through the same
  code.

The values are copied here verbatim; this script only re-serialises them.
"""
import json, os

KAT = {
    "perm_0_to_15": {"input": list(range(16)), "output": [1635930443, 1105042214, 1882043429, 1844048402, 1473750845, 312930215, 1730043656, 527466685, 315587567, 16091010, 1900299987, 511572576, 308360161, 643372060, 611592657, 1241962896]},
    "perm_ones": {"input": [1] * 16, "output": [1811698483, 1068710259, 1985337336, 805792844, 438157075, 1917939122, 931792294, 1736626050, 1759738447, 659850706, 260609625, 1946910843, 1635464896, 1262949863, 731049755, 611233391]},
    "perm_zeros": {"input": [0] * 16, "output": [1246627235, 628715430, 728127883, 1210800983, 1104325841, 123548278, 109211657, 1347389604, 350632487, 1919729472, 1334300527, 1417472912, 1710206249, 1032515169, 431466777, 1825850772]},
}
if __name__ == "__main__":
    with open(os.path.join(os.path.dirname(__file__), "poseidon2_kat.json"), "w") as f:
        json.dump(KAT, f, indent=1)
