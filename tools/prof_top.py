"""Top kernels of a rocprofv3 --stats run, per step: python tools/prof_top.py STATS.csv STEPS [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2])
n = int(sys.argv[3]) if len(sys.argv) > 3 else 30
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"kernel time per step {tot / steps / 1e6:.3f} ms, launches per step {sum(int(r['Calls']) for r in rows) / steps:.1f}")
for r in rows[:n]:
    t = float(r["TotalDurationNs"])
    print(f"{100 * t / tot:5.1f}% {t / steps / 1e3:8.1f} us/step  x{int(r['Calls']) / steps:5.1f}  "
          f"avg {float(r['AverageNs']) / 1e3:7.1f} us  {r['Name'][:95]}")
