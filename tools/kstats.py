"""Per-proof kernel time summary of a rocprofv3 kernel_stats.csv (bench run: warmup + steps proofs).
python tools/kstats.py gpurun_out/kstats_<tag>.csv [proofs]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else None
if n is None:
    n = next((int(r["Calls"]) for r in rows if "k_pow" in r["Name"]), 1)
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:28]:
    print(f"{r['Name'][:60]:60s} {int(r['Calls'])//n:5d} {float(r['TotalDurationNs'])/1e6/n:8.3f} ms/proof "
          f"{float(r['AverageNs'])/1e3:9.1f} us avg")
print(f"total kernel time per proof: {tot/1e6/n:.2f} ms ({n} proofs)")
