"""Side-by-side per-kernel time of several rocprofv3 ``kernel_stats.csv`` files:

    python tools/prof_diff.py --steps N a_kernel_stats.csv b_kernel_stats.csv ..."""
import argparse
import csv
import re
from collections import defaultdict


def short(name):
    n = re.sub(r"\(anonymous namespace\)::", "", name).replace("void ", "")
    return n[: n.find(">(") + 1] if ">(" in n else n.split("(")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    tabs = []
    for f in a.files:
        t = defaultdict(float)
        for r in csv.DictReader(open(f)):
            t[short(r["Name"])] += float(r["TotalDurationNs"]) / 1e6 / a.steps
        tabs.append(t)
    keys = sorted(set().union(*tabs), key=lambda k: -max(t.get(k, 0) for t in tabs))
    print("  ".join(f"{'file%d' % i:>9}" for i in range(len(tabs))) + "   ms/step  kernel")
    for k in keys[: a.top]:
        print("  ".join(f"{t.get(k, 0):9.3f}" for t in tabs) + "   " + k[:100])
    print("  ".join(f"{sum(t.values()):9.3f}" for t in tabs) + "   TOTAL")


if __name__ == "__main__":
    main()
