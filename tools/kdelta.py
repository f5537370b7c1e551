"""Per-kernel comparison of two rocprofv3 kernel_stats.csv files (same workload, two modes): calls, average
duration in each and the delta, sorted by the total-time delta.
python tools/kdelta.py A.csv B.csv [label_a label_b]"""
import csv
import sys


def load(p):
    out = {}
    for r in csv.DictReader(open(p)):
        k = r["Name"].split("(")[0].replace("void ", "").replace("zkm::", "")
        e = out.setdefault(k, [0, 0.0])
        e[0] += int(r["Calls"])
        e[1] += float(r["TotalDurationNs"])
    return out


a, b = load(sys.argv[1]), load(sys.argv[2])
la, lb = (sys.argv[3], sys.argv[4]) if len(sys.argv) > 4 else ("A", "B")
rows = []
for k in set(a) | set(b):
    ca, ta = a.get(k, (0, 0.0))
    cb, tb = b.get(k, (0, 0.0))
    avg_a = ta / ca / 1e3 if ca else 0.0
    avg_b = tb / cb / 1e3 if cb else 0.0
    rows.append((tb - ta, k, ca, cb, avg_a, avg_b, ta / 1e6, tb / 1e6))
rows.sort(reverse=True)
print(f"{'kernel':50s} {'calls ' + la:>12s} {'calls ' + lb:>12s} {'avg us ' + la:>14s} {'avg us ' + lb:>14s} "
      f"{'avg ratio':>9s} {'tot ms ' + la:>12s} {'tot ms ' + lb:>12s}")
for d, k, ca, cb, aa, ab, ta, tb in rows:
    r = ab / aa if aa else float("nan")
    print(f"{k[:50]:50s} {ca:12d} {cb:12d} {aa:14.1f} {ab:14.1f} {r:9.3f} {ta:12.2f} {tb:12.2f}")
print(f"{'TOTAL':50s} {'':12s} {'':12s} {'':14s} {'':14s} {'':9s} {sum(r[6] for r in rows):12.2f} "
      f"{sum(r[7] for r in rows):12.2f}")
