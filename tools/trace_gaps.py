"""Busy/idle timeline of a rocprofv3 kernel trace over the last N steps: the union of
kernel intervals (all queues), idle gaps, per-queue busy time, and the kernels that
run while only one queue is busy (the critical path's exposed part).
    python tools/trace_gaps.py run_kernel_trace.csv [--anchor KERNEL] [--steps N]"""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
anchor = sys.argv[sys.argv.index("--anchor") + 1] if "--anchor" in sys.argv else "adamw_kernel"
nsteps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 3
rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Kernel_Name"])
        for r in csv.DictReader(open(path))]
rows.sort()
ends = [e for s, e, q, n in rows if anchor in n]            # one anchor kernel per step
t0, t1 = ends[-nsteps - 1], ends[-1]
win = [(max(s, t0), min(e, t1), q, n) for s, e, q, n in rows if e > t0 and s < t1]
busy, cur_s, cur_e = 0, None, None
gaps = []
for s, e, q, n in sorted(win):
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
            gaps.append(s - cur_e)
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = t1 - t0
perq = defaultdict(int)
for s, e, q, n in win:
    perq[q] += e - s
print(f"{nsteps} steps: span {span / 1e6 / nsteps:.3f} ms/step, GPU busy (union) {busy / 1e6 / nsteps:.3f} ms/step "
      f"({100 * busy / span:.1f} %), idle gaps {len(gaps) / nsteps:.0f}/step, "
      f"sum {sum(gaps) / 1e6 / nsteps:.3f} ms/step, >5us: {sum(g for g in gaps if g > 5000) / 1e6 / nsteps:.3f} ms/step")
for q, t in sorted(perq.items()):
    print(f"  queue {q}: kernel time {t / 1e6 / nsteps:.3f} ms/step")
if "--top" in sys.argv:
    k = int(sys.argv[sys.argv.index("--top") + 1])
    evs = sorted(win)
    lst, cur_e, prev = [], None, None
    for s, e, q, n in evs:
        if cur_e is not None and s > cur_e:
            lst.append((s - cur_e, prev, n))
        if cur_e is None or e > cur_e:
            cur_e, prev = e, n
    lst.sort(reverse=True)
    short = lambda x: x.replace("(anonymous namespace)::", "").replace("void ", "")[:70]
    for g, a, b in lst[:k]:
        print(f"  gap {g / 1e3:8.1f} us  after {short(a)}  before {short(b)}")
