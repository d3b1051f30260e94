#!/usr/bin/env python3
"""Training-throughput benchmark (BASELINE.json metric) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--model unet|stf] ...

Default workload = BASELINE.json configs[1]: 2-D UNet(in=8, base_c=64), 256x256
DCE frames, batch 64 per GPU, bf16 compute (fp32 master weights / statistics),
one step = forward + CE+Dice criterion + backward (+ RCCL gradient all-reduce
when N > 1, or at N = 1 with --hook) + AdamW + LambdaLR step + the host's read of
the loss, exactly train_one_epoch's step (train_utils/train_and_eval.py:384-409:
``metric_logger.update(loss=loss.item(), ...)`` syncs the host once per step).  The
same K steps without the per-step loss read are timed as well and reported beside
the headline (``no_step_sync``).  Inputs are synthetic seeded DCE stacks
already resident in HBM.  For N > 1 the driver launches one process per GPU via
torch.distributed.run; every rank keeps its own batch (weak scaling) and the
timed region is bracketed by barrier + synchronize, max over ranks.

Prints ONE JSON line (rank 0) with the metric, the roofline of the dominant
kernel family (stf_igemm, timed with HIP events on its launch stream inside the
timed region) and the CPU baseline (the fp32 oracle restatement timed on this
host's cores on a bounded sample: the cpu_baseline leg is the only place bench.py
touches oracle/).
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
# STF_PKG_ROOT: import the package from another tree (same-box A/B of host-side changes)
sys.path.insert(0, os.environ.get("STF_PKG_ROOT", os.path.join(HERE, "stf-unet_amd")))
sys.path.insert(0, HERE)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

MFMA_BF16_PEAK_TFLOPS = 2500.0     # MI355X dense bf16 = fp16 (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)      # >= 50 timed after >= 10 warm-up
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", type=int, default=None, choices=[2, 3, 4, 5],
                    help="BASELINE.json configs[k-1] preset: 2 = UNet 256^2 B64 bf16 (the default workload), "
                         "3 = STF T8 256^2 B16 bf16, 4 = STF T16 256^2 B16 per GPU bf16 (the 8-GPU DDP config), "
                         "5 = STF T32+3 PK 512^2 fp16 + GradScaler, B4 per GPU")
    ap.add_argument("--model", default="unet", choices=["unet", "stf"],
                    help="unet = BASELINE configs[1] (default); stf = configs[2] (T=8, B=16)")
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (unet 64, stf 16)")
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--time-steps", type=int, default=8)
    ap.add_argument("--pk", action="store_true", help="STF with 3 PK-map channels (configs[4])")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16"],
                    help="16-bit activation storage; fp16 = the reference's --amp step (autocast float16 + "
                         "GradScaler, train_and_eval.py:389-404) on the fp16 library")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=3)
    ap.add_argument("--no-kernel-timer", action="store_true")
    ap.add_argument("--no-dice", action="store_true", help="skip the trained-weight Dice-vs-reference leg")
    ap.add_argument("--hook", action="store_true",
                    help="N = 1: form a world-1 RCCL group and attach the data-parallel gradient hook "
                         "(stfunet.ddp.GradAllReduce), i.e. time the per-GPU half of the DP step")
    ap.add_argument("--contend", default=None, metavar="BLOCKS,GBPS",
                    help="with --hook: after each bucket's collective, a proxy of what an 8-GPU RCCL "
                         "all-reduce does to the compute stream's CUs -- BLOCKS resident workgroups for "
                         "2*7/8*bytes/GBPS on the joiner stream (tools/contend); e.g. 32,300")
    a = ap.parse_args()
    presets = {2: dict(model="unet", batch=64, size=256, time_steps=8, pk=False, dtype="bf16"),
               3: dict(model="stf", batch=16, size=256, time_steps=8, pk=False, dtype="bf16"),
               4: dict(model="stf", batch=16, size=256, time_steps=16, pk=False, dtype="bf16"),
               5: dict(model="stf", batch=4, size=512, time_steps=32, pk=True, dtype="fp16")}
    if a.config is not None:
        for k, v in presets[a.config].items():
            if k != "batch" or a.batch is None:          # an explicit --batch wins
                setattr(a, k, v)
    return a


def workload_name(args):
    if args.model == "unet":
        cfg = "cfg2" if (args.size, args.time_steps) == (256, 8) else "custom"
        return f"{cfg} UNet(in={args.time_steps},base_c=64) {args.size}x{args.size} train step"
    cfg = {(256, 8, False): "cfg3", (256, 16, False): "cfg4 (per GPU)", (512, 32, True): "cfg5 (per GPU)"}.get(
        (args.size, args.time_steps, args.pk), "custom")
    return (f"{cfg} STFLSTMUNet(T={args.time_steps}{',PK' if args.pk else ''}) {args.size}x{args.size} "
            f"train step")


def pmc_traffic(kernel, workload, batch):
    """HBM bytes per launch of ``kernel`` from the committed PMC passes
    (tools/pmc_passes.sh + tools/pmc_summary.py: 2*FETCH_SIZE + WRITE_SIZE) of the
    same workload; None when no matching measurement is committed."""
    import glob
    for path in sorted(glob.glob(os.path.join(HERE, "profiles", "r*", "pmc_traffic*.json")), reverse=True):
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if d.get("workload") != workload or d.get("batch") != batch:
            continue
        k = d.get("kernels", {}).get(kernel)
        return (k["hbm_bytes_per_launch"], os.path.relpath(path, HERE)) if k else (None, None)
    return None, None


def pmc_mfma(kernel, workload):
    """MFMA busy fraction of ``kernel`` from the committed PMC pass of the same workload
    (tools/pmc_mfma.sh + tools/pmc_mfma_summary.py: SQ_VALU_MFMA_BUSY_CYCLES over
    GRBM_GUI_ACTIVE/8 x 1024 SIMDs, i.e. at the clock the chip held); None when absent."""
    import glob
    for path in sorted(glob.glob(os.path.join(HERE, "profiles", "r*", "pmc_mfma*.json")), reverse=True):
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if d.get("workload") != workload:
            continue
        k = d.get("kernels", {}).get(kernel)
        if not k:
            return None
        src = os.path.relpath(path, HERE)
        if k.get("clock_reliable") is False and "mfma_busy_util_step_clock" in k:
            # dispatches under ~0.3 ms read their own GRBM clock high (above the chip's 2.4 GHz):
            # the busy fraction at the step clock (slope of cycles against duration over the step)
            return {"mfma_busy_util": k["mfma_busy_util_step_clock"], "clock_ghz": d.get("step_clock_ghz"),
                    "clock_from": "step clock: " + str(d.get("step_clock_from", "")), "source": src}
        return {"mfma_busy_util": k["mfma_busy_util"], "clock_ghz": k["clock_ghz"], "source": src}
    return None


def roofline(kt, workload, batch, census):
    """Roofline of the dominant kernel (largest summed time in the census step;
    its every launch in the timed region bracketed by HIP events on its launch
    stream): algorithmic FLOPs per launch (2*M*N*K) over its average launch
    duration, against the dense bf16 MFMA peak."""
    if not kt:
        return None
    name = max(kt, key=lambda k: kt[k]["ms"])
    k = kt[name]
    traffic, src = pmc_traffic(name, workload, batch)
    gemm_ms = sum(v["ms"] for v in census.values())
    gemm_fl = sum(v["flops"] for v in census.values())
    return {"bound": "mfma", "kernel": name, "achieved": round(k["tflops"], 2), "peak": MFMA_BF16_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": round(k["tflops"] / MFMA_BF16_PEAK_TFLOPS, 4),
            "traffic": traffic, "traffic_unit": "HBM bytes per launch (PMC 2*FETCH_SIZE+WRITE_SIZE)",
            "traffic_source": src, "pmc_mfma": pmc_mfma(name, workload),
            "launches": k["launches"], "avg_launch_us": round(k["avg_us"], 2),
            "algorithmic_tflop_per_launch": round(k["flops"] / k["launches"] / 1e12, 6),
            "all_conv_gemm_kernels_census_step": {
                "ms": round(gemm_ms, 3), "tflops": round(gemm_fl / (gemm_ms * 1e-3) / 1e12, 2) if gemm_ms else 0.0}}


def doubleconv_report(blocks):
    """MFMA utilisation of each UNet DoubleConv in the census training step
    (north star: >= 70 % on DoubleConv at 256x256; SURVEY 8(d) names dec1
    (128->64, 64->64) as the fair target).  conv = its conv kernels only (fwd,
    dgrad, wgrad); block = everything the block launches (incl. BN/ReLU/pool
    passes) from the first to the last kernel of its forward / backward."""
    out = {}
    for name in sorted({t.rsplit(".", 1)[0] for t in blocks}):
        parts = [blocks[t] for t in (f"{name}.fwd", f"{name}.bwd") if t in blocks]
        fl = sum(p["flops"] for p in parts)
        cms = sum(p["conv_ms"] for p in parts)
        bms = sum(p["block_ms"] for p in parts)
        if cms <= 0 or bms <= 0:
            continue
        ct, bt = fl / (cms * 1e-3) / 1e12, fl / (bms * 1e-3) / 1e12
        out[name] = {"conv_tflops": round(ct, 1), "conv_mfma_frac": round(ct / MFMA_BF16_PEAK_TFLOPS, 3),
                     "block_tflops": round(bt, 1), "block_mfma_frac": round(bt / MFMA_BF16_PEAK_TFLOPS, 3),
                     "conv_ms": round(cms, 3), "block_ms": round(bms, 3)}
    return out


def dice_vs_reference(dev, dtype):
    """BASELINE metric's "Dice vs ref": the reference-trained UNet(in=8, base_c=8) of
    tests/golden/unet_trained.npz (make_golden_trained.py: trained by the reference's own
    train_one_epoch, parameters rounded to bf16, Dice from its own evaluate()) evaluated by
    engine.evaluate on this build's gfx950 path on the same 4 held-out batches (seeded
    splitmix DCE stacks, regenerated by stfunet.synthetic -- no oracle code).  The fixture
    is data (inputs' seeds, weights, the reference's Dice), not a CPU path."""
    import numpy as np
    from stfunet import UNet, engine
    from stfunet.synthetic import splitmix_dce_case
    z = np.load(os.path.join(HERE, "tests", "golden", "unet_trained.npz"))
    base_c, b, t, hw, _, _, n_eval = (int(v) for v in z["config"])
    model = UNet(in_channels=8, num_classes=2, base_c=base_c)
    sd = model.state_dict()
    for k, v in sd.items():
        if "bf16." + k in z.files:
            bits = z["bf16." + k].astype(np.uint32) << 16
            sd[k] = torch.from_numpy(bits.view(np.float32).reshape(v.shape).copy())
        else:
            sd[k] = torch.from_numpy(z["state." + k].copy()).reshape(v.shape)
    model.load_state_dict(sd)
    model.storage_dtype = torch.float16 if dtype == "fp16" else torch.bfloat16
    model = model.to(dev)
    data = [splitmix_dce_case(2000 + i, b, t, hw, hw) for i in range(n_eval)]
    import contextlib
    with contextlib.redirect_stdout(sys.stderr):          # evaluate()'s MetricLogger lines stay off stdout
        got = engine.evaluate(model, data, dev, num_classes=2)
    ref = float(z["dice"])
    return {"value": round(got["dice"], 7), "reference": round(ref, 7), "abs_diff": abs(got["dice"] - ref),
            "tolerance": 1e-4, "storage": dtype,
            "sample": f"reference-trained UNet(in=8, base_c={base_c}), eval mode, {n_eval} held-out batches "
                      f"[{b}, {t}, 1, {hw}, {hw}] (tests/golden/unet_trained.npz)"}


def dice_vs_reference_stf(dev, dtype):
    """STF "Dice vs ref": tests/golden/stf_trained.npz holds the Dice the reference's own
    train_one_epoch + evaluate reached training STFLSTMUNet(T=4) from the canonical init on seeded
    64^2 DCE stacks (make_golden_trained_stf.py; no weights: 27 M parameters), and of the same
    reference run at another CPU thread count.  Here the same training runs on the gfx950 path
    (engine.train_one_epoch, stfunet AdamW, same batches and schedule) and engine.evaluate scores
    it on the same held-out batches; the fixture is data (seeds, the reference's Dice)."""
    import contextlib
    import numpy as np
    from stfunet import STFLSTMUNet, engine
    from stfunet.optim import AdamW
    from stfunet.synthetic import canonical_state_dict, splitmix_dce_case
    z = np.load(os.path.join(HERE, "tests", "golden", "stf_trained.npz"))
    b, t, hw, epochs, steps, n_eval = (int(v) for v in z["config"])
    tgt = (hw // 2, hw // 2)
    m = STFLSTMUNet(in_channels=1, num_classes=2, time_steps=t)
    m.load_state_dict(canonical_state_dict(m.state_dict(), seed=0))
    m.storage_dtype = torch.float16 if dtype == "fp16" else torch.bfloat16
    m = m.to(dev)
    opt = AdamW([p for p in m.parameters() if p.requires_grad], lr=1e-3, betas=(0.9, 0.999), weight_decay=1e-4,
                eps=1e-8)
    sched = engine.create_lr_scheduler(opt, steps, epochs, warmup=True)
    t0 = time.perf_counter()
    with contextlib.redirect_stdout(sys.stderr):
        for ep in range(epochs):
            batches = [splitmix_dce_case(3000 + ep * steps + i, b, t, hw, hw, target_hw=tgt) for i in range(steps)]
            engine.train_one_epoch(m, opt, batches, dev, ep, 2, lr_scheduler=sched, print_freq=10 ** 6)
        ev = [splitmix_dce_case(4000 + i, b, t, hw, hw, target_hw=tgt) for i in range(n_eval)]
        got = engine.evaluate(m, ev, dev, num_classes=2)
    ref = float(z["dice"])
    band = z["band_dice"].astype(float)
    lo, hi = float(band.min()) - 1e-3, float(band.max()) + 1e-3
    return {"value": round(got["dice"], 6), "reference": round(ref, 6), "abs_diff": abs(got["dice"] - ref),
            "reference_band": [round(float(band.min()), 6), round(float(band.max()), 6)],
            "reference_band_runs": [str(n) for n in z["band_names"]],
            "accept": [round(lo, 6), round(hi, 6)], "within": bool(lo <= got["dice"] <= hi),
            "tolerance": "the reference's own run-to-run band (thread counts, bf16 autocast) widened by 1e-3, "
                         "as tests/test_dice_gpu.py",
            "storage": dtype, "train_s": round(time.perf_counter() - t0, 2),
            "sample": f"STFLSTMUNet(T={t}) trained {epochs}x{steps} steps from the canonical init on seeded "
                      f"[{b}, {t}, 1, {hw}, {hw}] stacks, then evaluate() on {n_eval} held-out batches "
                      f"(tests/golden/stf_trained.npz)"}


def cpu_baseline(args):
    """fp32 oracle (plain PyTorch CPU restatement of src/unet.py or
    src/stf_lstm_unet.py + criterion + AdamW) on a bounded sample: B=2 at the
    same frame size."""
    from oracle import loss as o_loss, optim as o_optim, stf as o_stf, unet as o_unet
    from oracle.init import canonical_state_dict
    # every core this job may use: the CPUs of its affinity mask, unless the host grants the job
    # a smaller share by OMP_NUM_THREADS (the GPU boxes do: 16 of a shared host's cores per GPU)
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    cores = max(1, min(avail, int(omp))) if omp.isdigit() and int(omp) > 0 else avail
    torch.set_num_threads(cores)
    b = 2 if args.size <= 256 else 1           # bounded sample (~10-30 s of CPU work)
    g = torch.Generator().manual_seed(1)
    if args.model == "unet":
        sd = canonical_state_dict(o_unet.template_state_dict(args.time_steps, 2, 64), seed=0)
        x = torch.randn(b, args.time_steps, args.size, args.size, generator=g)
        t = (torch.rand(b, args.size, args.size, generator=g) > 0.8).long()
        fwd = lambda p: o_unet.forward(p, x, training=True)  # noqa: E731
    else:
        sd = canonical_state_dict(o_stf.template_state_dict(use_pk_maps=args.pk), seed=0)
        x = torch.randn(b, args.time_steps + (3 if args.pk else 0), 1, args.size, args.size, generator=g)
        t = (torch.rand(b, args.size // 2, args.size // 2, generator=g) > 0.8).long()
        fwd = lambda p: o_stf.forward(p, x, training=True, use_pk_maps=args.pk)  # noqa: E731
    p = {k: v.clone().requires_grad_(v.is_floating_point() and "running" not in k) for k, v in sd.items()}
    names = [k for k in p if p[k].requires_grad]
    m = [torch.zeros_like(p[k]) for k in names]
    v = [torch.zeros_like(p[k]) for k in names]

    def step(i):
        for k in names:
            p[k].grad = None
        loss = o_loss.criterion(fwd(p)["out"], t)
        loss.backward()
        with torch.no_grad():
            o_optim.adamw_step([p[k] for k in names], [p[k].grad for k in names], m, v, i, lr=1e-3)

    step(1)
    t0 = time.perf_counter()
    for i in range(args.cpu_steps):
        step(i + 2)
    dt = (time.perf_counter() - t0) / args.cpu_steps
    what = (f"UNet(in={args.time_steps}, base_c=64)" if args.model == "unet" else
            f"STFLSTMUNet(T={args.time_steps}{', PK' if args.pk else ''})")
    return {"value": round(b / dt, 4), "unit": "samples/s", "cores": cores, "kind": "port",
            "sample": f"oracle fp32 {what} train step, batch {b}, {args.size}x{args.size}, "
                      f"{args.cpu_steps} timed steps after 1 warm-up, {dt:.3f} s/step; {cores} threads "
                      f"({avail} CPUs in the affinity mask, OMP_NUM_THREADS={omp or 'unset'})"}


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args):
    """``--gpus N`` without a launcher: start N ranks (one process per GPU) through
    torch.distributed.run as a CHILD process -- nothing here has touched the GPU yet --
    and return its exit code.  With a launcher (WORLD_SIZE set) --gpus must agree."""
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is not None:
        if int(world_env) != args.gpus:
            raise SystemExit(f"--gpus {args.gpus} but the launcher started WORLD_SIZE={world_env} ranks")
        return None
    if args.gpus <= 1:
        return None
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    args = parse()
    rc = launch_ranks(args)
    if rc is not None:
        sys.exit(rc)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # STF_DIST_BACKEND=gloo (+ ranks sharing one GPU, device = local rank mod
    # device count) rehearses the N > 1 path on a one-GPU box; the driver's
    # multi-GPU runs use RCCL ("nccl"), one GPU per rank.
    backend = os.environ.get("STF_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", local % max(ndev, 1))
    if world == 1 and args.hook:
        # a world-1 process group: the hook's bucketed all-reduces run through RCCL as at N > 1
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    dist_on = world > 1 or args.hook
    if dist_on:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(dev)
    if os.environ.get("STF_MAIN_PRIO") == "1":
        # A/B knob: the step's main stream at high priority (the side streams stay at 0)
        torch.cuda.set_stream(torch.cuda.Stream(device=dev, priority=-1))

    from stfunet import engine, nhwc, plan
    from stfunet.ddp import GradAllReduce, rccl_stream_note
    from stfunet.flops import stf_train_flops, unet_train_flops
    from stfunet.optim import AdamW
    from stfunet.synthetic import dce_batch
    from stfunet import STFLSTMUNet, UNet

    if args.batch is None:
        args.batch = 64 if args.model == "unet" else 16
    torch.manual_seed(1234)
    if args.model == "unet":
        model = UNet(in_channels=args.time_steps, num_classes=2, base_c=64).to(dev)
    else:
        model = STFLSTMUNet(in_channels=1, num_classes=2, time_steps=args.time_steps, use_pk_maps=args.pk).to(dev)
    model.train()
    fp16 = args.dtype == "fp16"
    model.storage_dtype = torch.float16 if fp16 else torch.bfloat16
    scaler = torch.amp.GradScaler("cuda") if fp16 else None
    opt = AdamW(model.parameters(), lr=1e-3, betas=(0.9, 0.999), weight_decay=1e-4, eps=1e-8)
    steps_total = args.warmup + args.steps
    sched = engine.create_lr_scheduler(opt, max(steps_total, 1), 10, warmup=True)
    ddp = GradAllReduce(model) if dist_on else None
    if args.contend and ddp is not None:
        ddp.after_launch = _contend_proxy(args.contend, dev)

    # synthetic batches resident in HBM before the timed region
    half = (args.size // 2, args.size // 2) if args.model == "stf" else None   # STF predicts at H/2
    batches = [dce_batch(args.batch, args.time_steps, args.size, args.size, seed=1000 * rank + i, device=dev,
                         pk_channels=3 if args.pk else 0, mask_hw=half) for i in range(2)]
    batches = [(engine.preprocess_input(x, model), t) for x, t in batches]

    def train_step(i):
        # train_one_epoch's step (train_and_eval.py:384-409); fp16 = its --amp branch
        x, t = batches[i % len(batches)]
        with torch.amp.autocast(device_type="cuda", enabled=fp16):
            loss = engine.criterion(model(x), t)
        opt.zero_grad()
        if scaler is not None:
            scaler.scale(loss).backward()
            if ddp is not None:
                ddp.finish()
            scaler.step(opt)
            scaler.update()
        else:
            loss.backward()
            if ddp is not None:
                ddp.finish()
            opt.step()
        sched.step()
        return loss

    # warmup; its last step is a census (every conv-GEMM launch timed) that picks
    # the dominant kernel, and only that kernel is instrumented in the timed
    # region (per-launch events on every kernel perturb a host-bound step)
    census, census_main, blocks = {}, {}, {}
    for i in range(args.warmup):
        if i == args.warmup - 1 and not args.no_kernel_timer:
            nhwc.TIMER = nhwc.KernelTimer()
        loss = train_step(i)
        if nhwc.TIMER is not None:
            census = nhwc.TIMER.summary()
            census_main = nhwc.TIMER.summary(main_only=True)
            blocks = nhwc.TIMER.tag_summary()
            nhwc.TIMER = None
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    # the dominant kernel's launches are bracketed by HIP events in the LAST timed step
    # only (every launch of that kernel in that step): timing events on every step
    # perturb a host-bound step (STF: 56 bracketed launches per step cost ~5 ms)
    dominant = None
    if not args.no_kernel_timer:
        dominant = max(census, key=lambda k: census[k]["ms"]) if census else None
    runtime = model.program.runtime

    def timed(sync_each, kernel_timer):
        """K steps bracketed by barrier + synchronize; sync_each: the host reads the loss after
        every step (train_one_epoch's loss.item()), else only the last one."""
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for i in range(args.steps):
            if kernel_timer and dominant is not None and i == args.steps - 1:
                if runtime.fwd is not None:       # native plan replays: events around that kernel's ranges
                    plan.TIMED = dominant
                    runtime.timing()              # drop anything timed before
                else:
                    nhwc.TIMER = nhwc.KernelTimer(only=dominant)
            loss = train_step(args.warmup + i)
            if sync_each:
                loss.item()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        if world > 1:
            e = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            el = float(e.item())
        return el, loss

    # the same K steps twice: without the per-step host read of the loss, then (the headline)
    # with it, as the reference's loop does
    elapsed_nosync, _ = timed(False, False)
    elapsed, loss = timed(True, True)
    kt = nhwc.TIMER.summary() if nhwc.TIMER is not None else {}
    nhwc.TIMER = None
    if plan.TIMED is not None:
        n, ms, fl = runtime.timing()
        plan.TIMED = None
        if n:
            kt = {dominant: dict(launches=n, ms=ms, flops=fl, avg_us=1e3 * ms / n,
                                 tflops=fl / (ms * 1e-3) / 1e12 if ms > 0 else 0.0)}
    last_loss = float(loss.item())

    samples = args.batch * world * args.steps
    value = samples / elapsed
    if rank == 0:
        if args.model == "unet":
            train_gflop = unet_train_flops(args.time_steps, 64, args.size, args.size) / 1e9
        else:
            train_gflop = stf_train_flops(args.time_steps, args.size, args.size, args.pk) / 1e9
        workload = workload_name(args)
        roof = roofline(kt, workload, args.batch, census)
        if roof is not None and census_main:
            # the compute stream's own dominant conv kernel in the census step: the critical path's
            # (STF's overall dominant kernel is the side stream's weight gradient, held to one
            # workgroup per CU so that it leaves the chip to the main chain)
            mk = max(census_main, key=lambda k: census_main[k]["ms"])
            m = census_main[mk]
            roof["main_stream_census"] = {
                "kernel": mk, "launches": m["launches"], "avg_launch_us": round(m["avg_us"], 2),
                "achieved": round(m["tflops"], 2), "frac": round(m["tflops"] / MFMA_BF16_PEAK_TFLOPS, 4),
                "main_stream_conv_ms": round(sum(v["ms"] for v in census_main.values()), 3),
                "note": "census step (last warm-up step, run eagerly: a short launch's events also "
                        "hold the host's launch gap), launches on the step's compute stream only"}
        res = {
            "metric": "training samples/sec (256x256 DCE-MRI frames)",
            "value": round(value, 3), "unit": "samples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
            "data": "synthetic (seeded DCE stacks: noise + wash-in discs), resident in HBM",
            "step": "train_one_epoch's step incl. the per-step host read loss.item() (train_and_eval.py:409)"
                    + (" + the data-parallel gradient hook (world-1 RCCL group)" if (args.hook and world == 1)
                       else (" + RCCL gradient all-reduce" if world > 1 else "")),
            "no_step_sync": {"value": round(samples / elapsed_nosync, 3),
                             "ms_per_step": round(1e3 * elapsed_nosync / args.steps, 3),
                             "note": "same steps, the host reads the loss only after the last one"},
            "execution": "native_plan" if runtime.fwd is not None else "eager",
            "config": {"workload": workload,
                       "model": "UNet" if args.model == "unet" else "STFLSTMUNet",
                       "global_batch": args.batch * world, "per_gpu_batch": args.batch,
                       "seq_len": args.time_steps, "image": [args.size, args.size],
                       "parallelism": f"dp{world}", "ddp_hook": bool(ddp is not None)},
            **({"rccl_stream": rccl_stream_note(), "contend": args.contend} if ddp is not None else {}),
            "train_gflop_per_sample": round(train_gflop, 2),
            "model_tflops_per_gpu": round(value / world * train_gflop / 1e3, 2),
            "model_mfu": round(value / world * train_gflop / 1e3 / MFMA_BF16_PEAK_TFLOPS, 4),
            "roofline": roof,
            "doubleconv": doubleconv_report(blocks),
            "kernels_census_step": {k: {kk: (round(vv, 3) if isinstance(vv, float) else vv) for kk, vv in d.items()}
                                    for k, d in census.items()},
            "last_loss": round(last_loss, 5),
            "build": _build_record(),
        }
        if not args.no_dice and world == 1:    # evaluate() all-reduces: rank 0 alone must not call it at N > 1
            res["dice_vs_ref"] = (dice_vs_reference(dev, args.dtype) if args.model == "unet"
                                  else dice_vs_reference_stf(dev, args.dtype))
        if not args.no_cpu_baseline and world == 1:      # reported baseline: rank 0 at N=1 only
            res["cpu_baseline"] = cpu_baseline(args)
        print(json.dumps(res), flush=True)
    # Explicit teardown, in dependency order, while the HIP runtime and the process group are
    # still up: the hook, the recorded step plans (their events, kernels' argument blocks and
    # private memory pools), the model's buffers, then the process group -- nothing of ours is
    # left for interpreter shutdown / __cxa_finalize to destroy after the runtime's own teardown
    # (a --hook run under rocprofv3 took SIGSEGV inside __cxa_finalize in round 5)
    torch.cuda.synchronize()
    prog = getattr(model, "_program", None)
    if prog is not None:
        prog.grad_ready_hook = None
        prog.runtime.close()
    del ddp, prog, runtime, model, opt, sched, batches, loss
    plan.drain_pools()
    import gc
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()


def _contend_proxy(spec, dev):
    """bench-only: tools/contend/libcontend.so's RCCL-shaped occupancy kernel, launched on the
    joiner stream right after each bucket's collective (see --contend)."""
    import ctypes
    blocks, gbps = (float(v) for v in spec.split(","))
    lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools", "contend", "libcontend.so"))
    lib.contend_launch.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_double, ctypes.c_void_p]
    scratch = {}

    def launch(t):
        nbytes = t.numel() * t.element_size()
        buf = scratch.get(nbytes)
        if buf is None:
            buf = scratch[nbytes] = torch.zeros(nbytes // 4, dtype=torch.float32, device=dev)
        usec = 2 * 7 / 8 * nbytes / (gbps * 1e9) * 1e6
        rc = lib.contend_launch(buf.data_ptr(), nbytes, int(blocks), usec,
                                torch.cuda.current_stream(dev).cuda_stream)
        assert rc == 0, rc
    return launch


def _build_record():
    """Which build ran: the loaded libraries' digests and the source digest they were built from
    (__graft_entry__.build() records it next to them)."""
    from stfunet import _lib
    if not hasattr(_lib, "build_info"):          # (an older package under STF_PKG_ROOT)
        return None
    i = _lib.build_info()
    return {"src": i["src_recorded"], "src_now": i["src_now"], "lib": i["lib"], "current": i["current"]}


if __name__ == "__main__":
    main()
