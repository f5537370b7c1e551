"""Summarise rocprofv3 SQ counter CSVs per kernel: python tools/sq_summary.py <counter_collection.csv>..."""
import collections
import csv
import sys

agg = collections.defaultdict(collections.Counter)
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        agg[r['Kernel_Name'].split('(')[0][:44]][r['Counter_Name']] += float(r['Counter_Value'])
for n, c in sorted(agg.items(), key=lambda kv: -kv[1].get('SQ_BUSY_CYCLES', 0)):
    w = c.get('SQ_WAVES', 0) or 1
    wc = c.get('SQ_WAVE_CYCLES', 0) or 1
    line = f"{n:44s}"
    if 'SQ_WAVE_CYCLES' in c:
        line += (f" waves {w:8.0f} wait {100 * c['SQ_WAIT_ANY'] / wc:5.1f}% instst {100 * c['SQ_WAIT_INST_ANY'] / wc:5.1f}%"
                 f" active {100 * c['SQ_ACTIVE_INST_ANY'] / wc:5.1f}% valu {100 * c['SQ_ACTIVE_INST_VALU'] / wc:5.1f}%"
                 f" valuI/wave {c['SQ_INSTS_VALU'] / w:8.0f}")
    if 'SQ_LDS_IDX_ACTIVE' in c:
        line += (f" lds_conf {100 * c['SQ_LDS_BANK_CONFLICT'] / max(c['SQ_LDS_IDX_ACTIVE'], 1):5.1f}%"
                 f" ldsI {c['SQ_INSTS_LDS']:.0f} vmemI {c['SQ_INSTS_VMEM_RD']:.0f} waitlds {c['SQ_WAIT_INST_LDS']:.0f}")
    print(line)
