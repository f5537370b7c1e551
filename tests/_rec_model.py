"""A numpy model of zkm_recursion_instrs_to_trace (test infrastructure): the instr_to_row layouts of the
recursion chips' preprocessed traces, applied to recursion.prep_records."""
import numpy as np

from zkmips_amd import recursion as R


def instr_rows_model(chip, recs, h):
    """A numpy model of zkm_recursion_instrs_to_trace (the instr_to_row layouts it implements)."""
    from zkmips_amd import tracegen as TG
    P = R.P
    _, _, width, _ = TG.RECURSION_INSTR_CHIPS[chip]
    t = np.zeros((h, width), np.uint64)
    n = len(recs)
    for r in range(min(h, n)) if chip not in ("BaseAlu", "ExtAlu", "MemoryVar", "MemoryConst") else range(h):
        if chip in ("BaseAlu", "ExtAlu"):
            for e in range(4):
                if 4 * r + e < n:
                    q = recs[4 * r + e]
                    o = t[r, 8 * e:8 * e + 8]
                    o[0], o[1], o[2], o[7] = q[0], q[1], q[2], q[4]
                    o[3 + q[3]] = 1
        elif chip in ("MemoryVar", "MemoryConst"):
            w = 2 if chip == "MemoryVar" else 6
            for e in range(2):
                if 2 * r + e < n:
                    t[r, w * e:w * e + w] = recs[2 * r + e]
        elif chip == "BatchFRI":
            q = recs[r]
            t[r] = [1, 1 if q[4] else 0, q[0], q[1], q[2], q[3]]
        elif chip == "Select":
            t[r] = [1] + list(recs[r])
        elif chip == "FriFold":
            q = recs[r]
            f = 1 if q[11] else 0
            nf = P - 1 if f else 0
            t[r] = [f, q[0], nf, q[1], nf, q[2], nf, q[3], P - 1, q[4], P - 1, q[5], P - 1, q[6], P - 1, q[7], q[8],
                    q[9], q[10], 1]
        elif chip == "PublicValues":
            t[r, r], t[r, 8], t[r, 9] = 1, recs[r][0], P - 1
        elif chip == "ExpReverseBitsLen":
            q = recs[r]
            first, last = q[4] == 0, q[4] + 1 == q[5]
            t[r] = [q[0], P - 1 if first else 0, q[1], P - 1, q[2], q[3] if last else 0, q[4], first, last, 1]
        else:
            q = recs[r]
            t[r, 0:16], t[r, 16:48:2], t[r, 17:48:2], t[r, 48] = q[0:16], q[16:32], q[32:48], P - 1
    return t.astype(np.uint32)


def prep_from_records(records):
    """{chip: (records, height)} -> {chip: preprocessed trace} on the host."""
    return {k: instr_rows_model(k, r, h) for k, (r, h) in records.items()}
