"""MFMA utilisation per kernel from the rocprofv3 pass of tools/pmc_mfma.sh.

    python tools/pmc_mfma_summary.py OUTDIR --workload NAME --json profiles/r02/pmc_mfma_unet256_b64.json

Per dispatch (counters summed over the chip by rocprofv3):
  * cycles     = GRBM_GUI_ACTIVE / 8          (the GRBM counter is reported summed over the 8 XCDs)
  * clock      = cycles / kernel duration      (the clock the chip held under this kernel)
  * mfma_util  = SQ_VALU_MFMA_BUSY_CYCLES / (cycles x 1024 SIMDs)   (rocprofv3's MfmaUtil formula)
  * mfma_flop  = SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512                 (rocprofv3's MfmaFlopsBF16)
  * util_flop  = mfma_flop / (cycles x 1024 SIMDs x 1024 FLOP/clk/SIMD): the dense-bf16 fraction at
                 the clock actually held (2.5 PF at 2.4 GHz = 1024 FLOP/clk per SIMD)
  * frac_2p5   = mfma_flop / duration / 2.5 PF: the same work against the datasheet peak
A dispatch's own quotient reads high on dispatches shorter than ~0.3 ms (MI355X_MICROARCH.md, DVFS
give-back), so the step clock -- sum of cycles / sum of durations over the run's dispatches of at least
0.3 ms -- is also reported, and every kernel's MFMA busy fraction is given at that clock too
(``mfma_busy_util_step_clock`` = busy cycles / (step clock x duration x 1024 SIMDs)): for the short
STF dispatches that is the number to read.
Profiled passes clock ~2-5 % below un-profiled runs (MI355X_MICROARCH.md, DVFS item 2), so the
absolute TF/s here read low; the utilisation ratios are per cycle and do not depend on it.
"""
import argparse
import json
import os
import re
import sqlite3
from collections import defaultdict

SIMDS = 256 * 4
FLOP_PER_CLK_SIMD = 2.5e15 / (2.4e9 * SIMDS)          # = 1017 (1024 nominal)
COUNTERS = ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_VALU_MFMA_MOPS_BF16", "GRBM_GUI_ACTIVE")

# UNet(in=8, base_c=64) forward 3x3 convs on the halo kernel, in launch order (cfg2):
# enc1.0 (8 input channels) and the 16x16 bottleneck run on the linear kernels
UNET_FWD_HALO = ["enc1.3", "enc2.0", "enc2.3", "enc3.0", "enc3.3", "enc4.0", "enc4.3",
                 "dec4.0", "dec4.3", "dec3.0", "dec3.3", "dec2.0", "dec2.3", "dec1.0", "dec1.3"]


def short(name):
    n = re.sub(r"\(anonymous namespace\)::", "", name)
    n = re.sub(r"^void ", "", n)
    return n.split("(")[0] if ">(" not in n else n[: n.find(">(") + 1]


def dispatches(db):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(pmc_events)")]
    key = next(k for k in ("dispatch_id", "correlation_id", "id") if k in cols)
    order = next((k for k in ("start", "start_timestamp", key) if k in cols), key)
    d = {}
    q = f"select {key}, name, counter_name, counter_value, duration, {order} from pmc_events"
    for k, name, cn, val, dur, o in c.execute(q):
        e = d.setdefault(k, {"name": short(name), "dur_ns": float(dur), "order": o})
        e[cn] = e.get(cn, 0.0) + float(val)
    return sorted(d.values(), key=lambda e: e["order"]), cols


def derive(e):
    cyc = e["GRBM_GUI_ACTIVE"] / 8.0
    flop = e["SQ_INSTS_VALU_MFMA_MOPS_BF16"] * 512.0
    return {"cycles": cyc, "clock_ghz": cyc / e["dur_ns"] if e["dur_ns"] else 0.0,
            "mfma_util": e["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * SIMDS) if cyc else 0.0,
            "mfma_flop": flop, "util_flop": flop / (cyc * SIMDS * FLOP_PER_CLK_SIMD) if cyc else 0.0,
            "tflops": flop / e["dur_ns"] / 1e3 if e["dur_ns"] else 0.0}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("outdir")
    ap.add_argument("--workload", required=True)
    ap.add_argument("--json", required=True)
    ap.add_argument("--command", default="")
    ap.add_argument("--unet-layers", action="store_true", help="label the forward halo convs (UNet cfg2)")
    a = ap.parse_args()
    ev, cols = dispatches(os.path.join(a.outdir, "MFMA", "run_results.db"))
    ev = [e for e in ev if all(c in e for c in COUNTERS)]
    agg = defaultdict(lambda: defaultdict(float))
    for e in ev:
        g = agg[e["name"]]
        g["launches"] += 1
        g["dur_ns"] += e["dur_ns"]
        for c in COUNTERS:
            g[c] += e[c]
    long_ = [e for e in ev if e["dur_ns"] >= 3e5]
    # cycles_i = clock x duration_i + c0 over every dispatch of the run (least squares): the slope
    # is the clock, the intercept the per-dispatch over-read that inflates short dispatches' quotient
    xs = [e["dur_ns"] for e in ev]
    ys = [e["GRBM_GUI_ACTIVE"] / 8.0 for e in ev]
    n = len(xs)
    mx, my = sum(xs) / n, sum(ys) / n
    sxx = sum((x - mx) ** 2 for x in xs)
    fit_clock = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sxx if sxx else 0.0
    fit_c0 = my - fit_clock * mx
    if len(long_) >= 10:
        step_clock = sum(e["GRBM_GUI_ACTIVE"] / 8.0 for e in long_) / sum(e["dur_ns"] for e in long_)
        clock_from = f"{len(long_)} dispatches of >= 0.3 ms (sum of GRBM_GUI_ACTIVE/8 / sum of durations)"
    else:
        step_clock = fit_clock
        clock_from = (f"slope of GRBM_GUI_ACTIVE/8 against duration over all {n} dispatches (fewer than 10 "
                      f"of >= 0.3 ms; intercept {fit_c0:.0f} cycles per dispatch)")
    kernels = {}
    for k, g in sorted(agg.items(), key=lambda kv: -kv[1]["dur_ns"]):
        d = derive(g)
        if d["mfma_flop"] <= 0:
            continue
        avg_ns = g["dur_ns"] / g["launches"]
        kernels[k] = {"launches": int(g["launches"]), "avg_us": round(avg_ns / 1e3, 2),
                      "clock_ghz": round(d["clock_ghz"], 3), "clock_reliable": avg_ns >= 3e5,
                      "mfma_busy_util_step_clock": round(g["SQ_VALU_MFMA_BUSY_CYCLES"] /
                                                        (step_clock * g["dur_ns"] * SIMDS), 4) if step_clock else None,
                      "mfma_busy_util": round(d["mfma_util"], 4),
                      "mfma_flop_util_at_clock": round(d["util_flop"], 4), "tflops": round(d["tflops"], 1),
                      "frac_of_2p5PF": round(d["tflops"] / 2500.0, 4)}
    res = {"workload": a.workload, "command": a.command,
           "method": "rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE "
                     "--kernel-trace (one pass); cycles = GRBM_GUI_ACTIVE/8; mfma_busy_util = MFMA busy "
                     "cycles / (cycles x 1024 SIMDs); mfma_flop_util_at_clock = MOPS_BF16*512 / (cycles x "
                     "1024 SIMDs x 1017 FLOP/clk); frac_of_2p5PF = MFMA FLOP / duration / 2.5 PF",
           "step_clock_ghz": round(step_clock, 3),
           "step_clock_from": clock_from,
           "fit_clock_ghz": round(fit_clock, 3), "fit_overread_cycles_per_dispatch": round(fit_c0),
           "kernels": kernels}
    if a.unet_layers:
        # (forward convs with BN statistics: the 64-channel halo kernel and, at >= 128 output
        # channels, the wide kernel since round 6)
        halo = [e for e in ev if e["name"].startswith(("conv3x3_halo_kernel<16, 32, 8, 2, 0, 2, false",
                                                       "conv3x3_wide_kernel<2"))]
        # per step: the 15 forward convs, then (since round 6) the 4 dgrads that write the concat
        # gradients with statistics rows (the ConvT bias gradients, stf_stat_sums) in the backward
        n = len(UNET_FWD_HALO)
        per_step = n + 4 if len(halo) % (n + 4) == 0 else n
        layers = defaultdict(list)
        for i, e in enumerate(halo[len(halo) - per_step:][:n]):   # the last profiled step's forward
            layers[UNET_FWD_HALO[i]].append(derive(e) | {"us": e["dur_ns"] / 1e3})
        res["forward_halo_layers_last_step"] = {
            k: {"us": round(v[0]["us"], 1), "clock_ghz": round(v[0]["clock_ghz"], 3),
                "mfma_busy_util": round(v[0]["mfma_util"], 4),
                "mfma_flop_util_at_clock": round(v[0]["util_flop"], 4), "tflops": round(v[0]["tflops"], 1)}
            for k, v in layers.items()}
    os.makedirs(os.path.dirname(os.path.abspath(a.json)), exist_ok=True)
    with open(a.json, "w") as f:
        json.dump(res, f, indent=1)
    print(f"step clock {step_clock:.3f} GHz from {clock_from}; fit over all dispatches: "
          f"{fit_clock:.3f} GHz + {fit_c0:.0f} cycles per dispatch")
    print(f"{'kernel':60s} {'n':>4s} {'avg us':>8s} {'GHz':>6s} {'busy':>6s} {'busy@step':>9s} {'flop@clk':>8s} "
          f"{'TF/s':>7s} {'/2.5PF':>6s}")
    for k, v in list(kernels.items())[:20]:
        bs = v["mfma_busy_util_step_clock"]
        print(f"{k[:60]:60s} {v['launches']:4d} {v['avg_us']:8.1f} {v['clock_ghz']:6.3f}{'' if v['clock_reliable'] else '*'}"
              f"{v['mfma_busy_util']:6.3f} {bs if bs is not None else float('nan'):9.3f} "
              f"{v['mfma_flop_util_at_clock']:8.3f} {v['tflops']:7.1f} {v['frac_of_2p5PF']:6.3f}")
    print("(* = average dispatch under 0.3 ms: its own clock reads high; use busy@step)")
    for k, v in res.get("forward_halo_layers_last_step", {}).items():
        print(f"  {k:8s} {v['us']:7.1f} us  {v['clock_ghz']:.3f} GHz  busy {v['mfma_busy_util']:.3f}  "
              f"flop@clk {v['mfma_flop_util_at_clock']:.3f}  {v['tflops']:.0f} TF/s")


if __name__ == "__main__":
    main()
