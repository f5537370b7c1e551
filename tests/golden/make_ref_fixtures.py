"""Extract the reference-held data fixtures this repo pins against (run in the build container only,
where /root/reference exists; the outputs are committed, the GPU box never reads the reference).

* mips_costs.json      <- crates/core/executor/src/artifacts/mips_costs.json (verbatim data: the
                          per-row cost prep + main + 4*perm_EF + 4*2^log_qd of every MIPS chip,
                          crates/stark/src/chip.rs:154-163; checked by mips/mod.rs:720-727).
* maximal_shapes_22.json <- crates/core/machine/src/shape/maximal_shapes.json["22"] (the reference's
                          own 2^22 shard compositions: chip -> log2 height).
* dummy_vk_map.json    <- a description of crates/prover/dummy_vk_map.bin (bincode BTreeMap<[KoalaBear;8],
                          usize>, shapes.rs:370-379, loaded at prover/src/lib.rs:232): byte length,
                          sha256, entry count and the decoded first/last entries.  The file itself
                          is regenerated from its entries by the oracle's serializer in the test.
* curve_params.json    <- crates/curves/src/{weierstrass/*,uint256}.rs: each base field's MODULUS bytes,
                          WITNESS_OFFSET, Limbs / Witness sizes and, for the curves, a_int / b_int
                          (the FieldParameters / WeierstrassParameters the precompile chips use).
"""
import hashlib
import re
import json
import os

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    costs = json.load(open(os.path.join(REF, "crates/core/executor/src/artifacts/mips_costs.json")))
    json.dump(costs, open(os.path.join(HERE, "mips_costs.json"), "w"), indent=1, sort_keys=True)

    shapes = json.load(open(os.path.join(REF, "crates/core/machine/src/shape/maximal_shapes.json")))
    json.dump([s["inner"] for s in shapes["22"]], open(os.path.join(HERE, "maximal_shapes_22.json"), "w"))

    b = open(os.path.join(REF, "crates/prover/dummy_vk_map.bin"), "rb").read()
    n = int.from_bytes(b[:8], "little")
    rec = np.frombuffer(b[8:], dtype=np.uint8).reshape(n, 40)
    keys = rec[:, :32].copy().view("<u4")
    vals = rec[:, 32:].copy().view("<u8")[:, 0]
    desc = {
        "source": "crates/prover/dummy_vk_map.bin",
        "bytes": len(b),
        "sha256": hashlib.sha256(b).hexdigest(),
        "entries": n,
        "first": [[int(x) for x in keys[i]] + [int(vals[i])] for i in range(3)],
        "last": [int(x) for x in keys[-1]] + [int(vals[-1])],
        "rule": "entry i = key [i; 8] (canonical u32), value i",
        "rule_holds": bool(np.all(keys == np.arange(n)[:, None]) and np.all(vals == np.arange(n))),
    }
    json.dump(desc, open(os.path.join(HERE, "dummy_vk_map.json"), "w"), indent=1)

    params = {}
    for name, f in (("Secp256k1", "weierstrass/secp256k1.rs"), ("Secp256r1", "weierstrass/secp256r1.rs"),
                    ("Bn254", "weierstrass/bn254.rs"), ("Bls12381", "weierstrass/bls12_381.rs"),
                    ("U256", "uint256.rs")):
        src = open(os.path.join(REF, "crates/curves/src", f)).read()
        mod = re.search(r"const MODULUS: &'static \[u8\] = &\[(.*?)\];", src, re.S).group(1)
        e = {"modulus_le": [int(x, 0) for x in re.findall(r"0x[0-9a-fA-F]+|\d+", mod)],
             "witness_offset_log2": int(re.search(r"WITNESS_OFFSET: usize = 1usize << (\d+)", src).group(1)),
             "limbs": int(re.search(r"type Limbs = U(\d+)", src).group(1)),
             "witness": int(re.search(r"type Witness = U(\d+)", src).group(1))}
        for fn in ("a_int", "b_int"):
            m = re.search(r"fn " + fn + r"\(\) -> BigUint \{\s*BigUint::from_slice\(&\[(.*?)\]\)", src, re.S)
            if m:
                e[fn + "_u32_le"] = [int(x, 0) for x in re.findall(r"0x[0-9a-fA-F]+|\d+", m.group(1))]
            else:
                m = re.search(r"fn " + fn + r"\(\) -> BigUint \{\s*BigUint::from\((\d+)u32\)", src)
                if m:
                    e[fn + "_u32_le"] = [int(m.group(1))]
        g = re.search(r"fn generator\(\) -> \(BigUint, BigUint\) \{(.*?)\n    \}", src, re.S)
        if g:
            e["generator"] = [str(int(v)) for v in re.findall(r'"(\d+)"', g.group(1))]
        params[name] = e
    json.dump(params, open(os.path.join(HERE, "curve_params.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
