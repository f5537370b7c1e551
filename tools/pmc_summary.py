"""Summarise rocprofv3 runs into profiles/ (kernel stats + HBM traffic per launch).

Usage: python tools/pmc_summary.py <kernel_stats.csv> <fetch_counter.csv> <write_counter.csv> <out.json>

HBM traffic per launch = 2 * FETCH_SIZE + WRITE_SIZE (KB -> bytes).  The factor 2 on FETCH_SIZE is the
gfx950 correction of /opt/skills/guides/MI355X_MICROARCH.md §HBM (FETCH_SIZE reports half the bytes
of a coalesced streaming read; our leaf-hash and NTT loads are coalesced 256-B wave reads); WRITE_SIZE
is taken as is.  The correction was checked on k_hash_leaves (main tree): 2 x 1,098,110 KB = 2.249 GB
vs 2^23 rows x 67 columns x 4 B = 2.248 GB algorithmic.
"""
import collections
import csv
import json
import sys


def short(name):
    return name.split("(")[0].replace("void ", "").replace("zkm::", "")


def main(stats, fetch, write, out):
    res = {"kernels": {}}
    for r in csv.DictReader(open(stats)):
        res["kernels"].setdefault(short(r["Name"]), {}).update(
            {"calls": int(r["Calls"]), "total_ms": float(r["TotalDurationNs"]) / 1e6,
             "avg_ms": float(r["AverageNs"]) / 1e6, "pct": float(r["Percentage"])})
    traffic = collections.defaultdict(lambda: [0.0, 0.0, 0])
    for f, idx in ((fetch, 0), (write, 1)):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            traffic[k][idx] += float(r["Counter_Value"]) * 1024.0
            if idx == 0:
                traffic[k][2] += 1
    for k, (fb, wb, n) in traffic.items():
        d = res["kernels"].setdefault(k, {})
        d["pmc_launches"] = n
        d["hbm_bytes_per_launch"] = (2 * fb + wb) / max(n, 1)
        d["fetch_bytes_raw_per_launch"] = fb / max(n, 1)
        d["write_bytes_per_launch"] = wb / max(n, 1)
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main(*sys.argv[1:5])
