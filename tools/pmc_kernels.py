"""Sum rocprofv3 counter-collection CSVs per kernel (all dispatches) and print derived ratios.
python tools/pmc_kernels.py <dir> [<dir> ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(float))
calls = defaultdict(set)
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("zkm::", "")
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            calls[k].add((f, r["Dispatch_Id"]))
for k in sorted(acc, key=lambda k: -acc[k].get("SQ_WAVE_CYCLES", acc[k].get("GRBM_GUI_ACTIVE", 0))):
    c = acc[k]
    print(f"{k[:40]:40s} dispatches {len(calls[k])}")
    for n in sorted(c):
        print(f"    {n:28s} {c[n]:.4g}")
    w = c.get("SQ_WAVE_CYCLES")
    if w:
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
            if n in c:
                print(f"    {n + ' / WAVE_CYCLES':40s} {c[n] / w:.3f}")
