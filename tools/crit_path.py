"""Critical-path view of a spin-first eager trace (tools/stf_trace_spin.sh): per step, the
window from the end of the spin kernel to the end of the optimizer kernel; per stream the
kernel time; on the main stream, the idle time (waiting for side streams) and which kernel
it waited before; the main-stream kernel time by kernel family.
    python tools/crit_path.py gpurun_out/stfspin/kernel_trace.csv.gz"""
import csv
import gzip
import sys
from collections import defaultdict

path = sys.argv[1]
f = gzip.open(path, "rt") if path.endswith(".gz") else open(path)
rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Kernel_Name"])
        for r in csv.DictReader(f)]
rows.sort()
short = lambda n: (n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0])[:70]
spins = [i for i, r in enumerate(rows) if "spin" in r[3].lower() or "sleep" in r[3].lower()]
if not spins:
    # plan-replayed steps (no spin kernel needed: the host is ahead): a step = from the end
    # of one optimizer kernel to the end of the next
    spins = [i for i, r in enumerate(rows) if "adamw" in r[3]]
    rows = rows[:spins[-1] + 1]     # the last full step ends with the last optimizer kernel
    spins = spins[:-1]
if not spins:
    sys.exit("no spin / optimizer kernel found")
steps = []
for k, i in enumerate(spins):
    j = spins[k + 1] if k + 1 < len(spins) else len(rows)
    steps.append(rows[i + 1:j])
last = steps[-1]
main = rows[spins[-1]][2]
t0 = rows[spins[-1]][1]
t1 = max(e for s, e, q, n in last)
print(f"step window {(t1 - t0) / 1e3:.1f} us, main stream {main}")
perq = defaultdict(int)
for s, e, q, n in last:
    perq[q] += e - s
for q, v in sorted(perq.items()):
    print(f"  stream {q}: kernel time {v / 1e3:8.1f} us")
fam = defaultdict(lambda: [0, 0])
idle = []
prev_end = t0
for s, e, q, n in last:
    if q != main:
        continue
    if s > prev_end:
        idle.append((s - prev_end, short(n)))
    prev_end = max(prev_end, e)
    fam[short(n)][0] += e - s
    fam[short(n)][1] += 1
tot_idle = sum(g for g, _ in idle)
print(f"main stream: kernels {sum(v[0] for v in fam.values()) / 1e3:.1f} us, idle {tot_idle / 1e3:.1f} us "
      f"in {len(idle)} gaps")
for g, n in sorted(idle, reverse=True)[:15]:
    print(f"   idle {g / 1e3:7.1f} us before {n}")
print("main-stream kernel time by kernel:")
for n, (t, c) in sorted(fam.items(), key=lambda kv: -kv[1][0])[:40]:
    print(f"  {t / 1e3:8.1f} us {c:4d}x  {n}")
