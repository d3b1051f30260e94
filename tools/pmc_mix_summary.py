"""Per-kernel instruction mix from tools/pmc_mix.sh: VALU issue time (4 cycles per wave64
VALU instruction on each of the 1024 SIMDs, at 2.2 GHz) against the measured duration --
a ratio near or above ~0.5 marks a kernel whose vector ALU work, not HBM, sets its time.
Usage: python tools/pmc_mix_summary.py OUTDIR [top]"""
import collections
import glob
import sqlite3
import sys

db = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
c = sqlite3.connect(db)
per = collections.defaultdict(dict)
for did, kn, cn, v, dur in c.execute(
        "select dispatch_id, kernel_name, counter_name, value, duration from counters_collection"):
    d = per[did]
    d["k"] = kn
    d["dur"] = dur
    d[cn] = d.get(cn, 0) + v
agg = collections.defaultdict(lambda: collections.Counter())
for d in per.values():
    a = agg[d["k"]]
    a["n"] += 1
    for key in ("dur", "SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS", "SQ_INSTS_SALU",
                "SQ_WAVES"):
        a[key] += d.get(key, 0)
rows = sorted(agg.items(), key=lambda kv: -kv[1]["dur"])[:top]
print(f"{'kernel':60s} {'n':>4s} {'avg us':>8s} {'VALU/wave':>9s} {'VMEM/wave':>9s} {'LDS/wave':>8s} {'valu_us':>8s} {'ratio':>6s}")
for k, a in rows:
    n = a["n"]
    w = max(a["SQ_WAVES"], 1)
    dur = a["dur"] / n / 1e3
    valu_us = a["SQ_INSTS_VALU"] / n * 4 / 1024 / 2.2e9 * 1e6
    print(f"{k[:60]:60s} {n:4d} {dur:8.1f} {a['SQ_INSTS_VALU'] / w:9.0f} "
          f"{(a['SQ_INSTS_VMEM_RD'] + a['SQ_INSTS_VMEM_WR']) / w:9.1f} {a['SQ_INSTS_LDS'] / w:8.0f} "
          f"{valu_us:8.1f} {valu_us / max(dur, 1e-9):6.2f}")
