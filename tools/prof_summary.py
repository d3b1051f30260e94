"""Summarise a rocprofv3 rocpd database (``--kernel-trace`` output, *.db) into the
per-kernel table the profiles/ CSVs hold: calls, total ms, average us, share.

    python tools/prof_summary.py run_results.db [--steps N] [--csv out.csv]

--steps N divides totals by N to print per-step milliseconds."""
import argparse
import csv
import re
import sqlite3
from collections import defaultdict


def short(name):
    n = re.sub(r"\(anonymous namespace\)::", "", name)
    n = re.sub(r"^void ", "", n)
    return n.split("(")[0] if "<" not in n.split("(")[0] else n[: n.find(">(") + 1] if ">(" in n else n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--csv")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    agg = defaultdict(lambda: [0, 0])
    for name, dur in c.execute("select name, duration from kernels"):
        k = short(name)
        agg[k][0] += 1
        agg[k][1] += dur
    total = sum(v[1] for v in agg.values())
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
    out = []
    for k, (n, ns) in rows:
        out.append({"kernel": k, "calls": n, "total_ms": round(ns / 1e6, 3), "avg_us": round(ns / n / 1e3, 2),
                    "per_step_ms": round(ns / 1e6 / a.steps, 3), "pct": round(100.0 * ns / total, 2)})
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(out[0]))
            w.writeheader()
            w.writerows(out)
    print(f"total kernel time {total / 1e6:.2f} ms ({total / 1e6 / a.steps:.2f} ms/step over {a.steps})")
    for r in out[:40]:
        print(f"{r['pct']:6.2f}% {r['per_step_ms']:8.3f} ms/step {r['calls']:6d} calls {r['avg_us']:9.2f} us  {r['kernel'][:110]}")


if __name__ == "__main__":
    main()
