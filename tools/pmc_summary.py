"""Per-kernel HBM traffic from the two rocprofv3 PMC passes of tools/pmc_passes.sh.

    python tools/pmc_summary.py OUTDIR --workload NAME --json profiles/r01/pmc_traffic.json

Bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (both reported in KiB).  The factor 2:
on gfx950 FETCH_SIZE counts exactly half the bytes of wide (16 B/lane) coalesced
reads, global_load and buffer_load ... lds alike (MI355X_MICROARCH.md, 'HBM'); WRITE_SIZE
is exact for 16-B streaming stores.  Infinity-Cache hits are counted by these
memory-side counters, so this is L2->fabric traffic (an upper bound on HBM bytes).
"""
import argparse
import json
import os
import re
import sqlite3
from collections import defaultdict


def short(name):
    n = re.sub(r"\(anonymous namespace\)::", "", name)
    n = re.sub(r"^void ", "", n)
    return n.split("(")[0] if ">(" not in n else n[: n.find(">(") + 1]


def per_kernel(db, counter):
    c = sqlite3.connect(db)
    agg = defaultdict(lambda: [0, 0.0, 0])
    for name, val, dur in c.execute("select name, counter_value, duration from pmc_events where counter_name = ?",
                                    (counter,)):
        k = short(name)
        agg[k][0] += 1
        agg[k][1] += float(val)
        agg[k][2] += dur
    return agg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("outdir")
    ap.add_argument("--workload", required=True)
    ap.add_argument("--json", required=True)
    ap.add_argument("--command", default="")
    ap.add_argument("--batch", type=int, required=True)
    a = ap.parse_args()
    fetch = per_kernel(os.path.join(a.outdir, "FETCH_SIZE", "run_results.db"), "FETCH_SIZE")
    write = per_kernel(os.path.join(a.outdir, "WRITE_SIZE", "run_results.db"), "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) & set(write), key=lambda k: -fetch[k][1]):
        nf, kf, _ = fetch[k]
        nw, kw, _ = write[k]
        fb = 2.0 * kf * 1024 / nf
        wb = kw * 1024 / nw
        kernels[k] = {"launches": nf, "fetch_bytes_per_launch": round(fb), "write_bytes_per_launch": round(wb),
                      "hbm_bytes_per_launch": round(fb + wb)}
    res = {"workload": a.workload, "batch": a.batch, "command": a.command,
           "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes with --kernel-trace; "
                     "bytes = 2*FETCH_SIZE + WRITE_SIZE (KiB units, gfx950 wide-read correction)",
           "kernels": kernels}
    os.makedirs(os.path.dirname(a.json), exist_ok=True)
    with open(a.json, "w") as f:
        json.dump(res, f, indent=1)
    for k, v in list(kernels.items())[:15]:
        print(f"{v['hbm_bytes_per_launch'] / 1e6:10.1f} MB/launch  fetch {v['fetch_bytes_per_launch'] / 1e6:9.1f}  "
              f"write {v['write_bytes_per_launch'] / 1e6:9.1f}  x{v['launches']:5d}  {k}")


if __name__ == "__main__":
    main()
