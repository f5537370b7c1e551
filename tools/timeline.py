"""FRI commit-phase timeline from a rocprofv3 kernel trace (tools/gpu/fri_timeline.sh):
python3 tools/timeline.py gpurun_out/ktrace_<tag>.csv [proof_index]

The phase of a proof is the run of dispatches after its last `k_fri_reduce` up to its `k_pow`.  Prints
each dispatch (duration, idle gap before it) and the span / busy / idle totals, then busy time per
kernel name."""
import csv
import sys
from collections import defaultdict


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").replace("zkm::", "")


def main():
    rows = load(sys.argv[1])
    which = int(sys.argv[2]) if len(sys.argv) > 2 else -1
    pows = [i for i, r in enumerate(rows) if "k_pow" in r[2]]
    end = pows[which]
    start = end
    while start > 0 and "k_fri_reduce" not in rows[start - 1][2]:
        start -= 1
    ph = rows[start:end]
    busy = 0
    per = defaultdict(float)
    cnt = defaultdict(int)
    prev_end = rows[start - 1][1]
    gaps = 0
    for s, e, n in ph:
        gap = max(0, s - prev_end)
        gaps += gap
        busy += e - s
        per[short(n)] += e - s
        cnt[short(n)] += 1
        print(f"{short(n)[:40]:40s} {1e-3 * (e - s):9.1f} us  gap {1e-3 * gap:7.1f} us")
        prev_end = max(prev_end, e)
    span = ph[-1][1] - rows[start - 1][1]
    print(f"\nphase: {len(ph)} dispatches, span {1e-6 * span:.3f} ms, busy {1e-6 * busy:.3f} ms, idle {1e-6 * gaps:.3f} ms")
    for k, v in sorted(per.items(), key=lambda kv: -kv[1]):
        print(f"  {k[:40]:40s} {cnt[k]:4d} x  {1e-6 * v:.3f} ms")


if __name__ == "__main__":
    main()
