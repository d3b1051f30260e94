"""Per-kernel SQ counter averages from rocprofv3 --pmc runs (rocpd *.db or
counter_collection.csv), our kernels only:
    python tools/sq_summary.py DIR [DIR ...]"""
import csv
import os
import re
import sqlite3
import sys
from collections import defaultdict


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    return n[: n.find(">(") + 1] if ">(" in n else n.split("(")[0]


def rows(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        yield from c.execute("select kernel_name, counter_name, value, duration from counters_collection")
    else:
        for r in csv.DictReader(open(path)):
            yield r["Kernel_Name"], r["Counter_Name"], float(r["Counter_Value"]), 0


for d in sys.argv[1:]:
    agg = defaultdict(lambda: defaultdict(list))
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith(".db") or f.endswith("counter_collection.csv"):
                for name, cn, v, dur in rows(os.path.join(root, f)):
                    if re.search(r"at::|rocclr|distribution|elementwise|pack_weight", name):
                        continue
                    agg[short(name)][cn].append(v)
                    agg[short(name)]["_dur_ns"].append(dur)
    print("==", d)
    for k, cs in agg.items():
        print(" ", k[:90])
        for c, v in sorted(cs.items()):
            print(f"     {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
