"""Summarize one training step of a rocprofv3 --kernel-trace CSV (the last step: between the
last two AdamW launches): step window vs summed kernel time, time per kernel family, and the
streaming BatchNorm launches in order (their bandwidth follows from the layer sizes).

  python tools/trace_summary.py gpurun_out/t17/run_kernel_trace.csv
"""
import argparse
import collections
import csv
import re


def family(name):
    n = re.sub(r"^(void )?\(anonymous namespace\)::", "", name)
    return n.split("(")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    args = ap.parse_args()
    rows = sorted(csv.DictReader(open(args.trace)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
    if len(idx) < 2:
        raise SystemExit("need two optimizer launches in the trace")
    step = rows[idx[-2] + 1: idx[-1] + 1]
    t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    busy = sum(dur(r) for r in step)
    print(f"step window {(t1 - t0) / 1e3:.1f} us, {len(step)} kernels, summed kernel time {busy:.1f} us")
    fam = collections.defaultdict(lambda: [0, 0.0])
    for r in step:
        f = fam[family(r["Kernel_Name"])]
        f[0] += 1
        f[1] += dur(r)
    print("\n  time us   share   n  kernel family")
    for k, (n, t) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
        print(f"{t:9.1f} {t / busy * 100:6.1f}% {n:3d}  {k}")
    print("\nstreaming BatchNorm launches in order (duration us):")
    for r in step:
        f = family(r["Kernel_Name"])
        if f.startswith(("bn_act", "bn_bwd_apply", "bn_bwd_reduce")):
            print(f"{dur(r):8.1f}  {f}")


if __name__ == "__main__":
    main()
