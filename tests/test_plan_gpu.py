"""Native step plans (stfunet/plan.py, csrc/plan.hip) against the eager schedule.

The plan records the training step's launches once and replays them from C++; a replayed
step must compute exactly what the eager Python schedule computes.  Checked bit for bit
over several optimizer steps (losses, every parameter, every BatchNorm buffer): UNet and
STFLSTMUNet (also with PK maps: the stem gather and PK-fusion paths with their row copies),
bf16 and fp16 storage (the --amp step with GradScaler), the data-parallel hook segments
(gradient snapshot at every hook), a re-record when the batch shape changes, and two
forwards before their backwards (the second must not overwrite the first's saved state).
"""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _make(which, pk=False, base_c=16):
    from stfunet import STFLSTMUNet, UNet
    torch.manual_seed(0)
    if which == "unet":
        return UNet(in_channels=8, num_classes=2, base_c=base_c).cuda().train()
    return STFLSTMUNet(in_channels=1, num_classes=2, time_steps=4, use_pk_maps=pk).cuda().train()


def _batches(which, n, pk=False, b=2, hw=128):
    from stfunet import engine
    from stfunet.synthetic import dce_batch
    out = []
    for i in range(n):
        if which == "unet":
            x, t = dce_batch(b, 8, hw, hw, seed=700 + i, device="cuda")
            out.append((x.flatten(1, 2), t))
        else:
            x, t = dce_batch(b, 4, hw, hw, seed=700 + i, device="cuda", pk_channels=3 if pk else 0,
                             mask_hw=(hw // 2, hw // 2))
            out.append((x, t))
    return out


def _train(which, plan_on, steps=5, pk=False, fp16=False, hook=False, batches=None):
    from stfunet import engine
    from stfunet.optim import AdamW
    os.environ["STF_PLAN"] = "1" if plan_on else "0"
    try:
        model = _make(which, pk)
        model.storage_dtype = torch.float16 if fp16 else torch.bfloat16
        opt = AdamW(model.parameters(), lr=1e-3, weight_decay=1e-4)
        scaler = torch.amp.GradScaler("cuda") if fp16 else None
        batches = batches or _batches(which, 3, pk)
        prog = model.program
        snaps = []
        if hook:
            def h(off, deps=()):
                cur = torch.cuda.current_stream()
                for st in deps:                 # gradients written on side streams
                    cur.wait_stream(st)
                snaps.append((off, prog.flat.grad[off:].clone()))
            prog.grad_ready_hook = h
        losses = []
        for i in range(steps):
            x, t = batches[i % len(batches)]
            with torch.amp.autocast("cuda", enabled=fp16):
                loss = engine.criterion(model(x), t)
            opt.zero_grad()
            if scaler is not None:
                scaler.scale(loss).backward()
                scaler.step(opt)
                scaler.update()
            else:
                loss.backward()
                opt.step()
            losses.append(loss.detach().clone())
        torch.cuda.synchronize()
        state = {k: v.detach().clone() for k, v in model.state_dict().items()}
        return dict(losses=torch.stack(losses), state=state, planned=prog.runtime.bwd is not None, snaps=snaps,
                    n_fwd=prog.runtime.fwd.n if prog.runtime.fwd is not None else 0)
    finally:
        os.environ.pop("STF_PLAN", None)


def _assert_same(a, b):
    assert b["planned"] and not a["planned"]
    assert torch.equal(a["losses"], b["losses"]), (a["losses"], b["losses"])
    for k in a["state"]:
        assert torch.equal(a["state"][k], b["state"][k]), k


@pytest.mark.parametrize("which", ["unet", "stf"])
def test_plan_replay_bitwise_vs_eager(which):
    eager = _train(which, False)
    planned = _train(which, True)
    _assert_same(eager, planned)
    assert planned["n_fwd"] > 20


def test_plan_replay_stf_pk_bitwise():
    _assert_same(_train("stf", False, steps=4, pk=True), _train("stf", True, steps=4, pk=True))


@pytest.mark.parametrize("which", ["unet", "stf"])
def test_plan_replay_fp16_gradscaler_bitwise(which):
    _assert_same(_train(which, False, steps=4, fp16=True), _train(which, True, steps=4, fp16=True))


@pytest.mark.parametrize("which", ["unet", "stf"])
def test_plan_hook_segments(which):
    """The data-parallel hook runs between replayed segments, at the same points and with the
    same finished gradient suffix as in the eager schedule."""
    eager = _train(which, False, steps=4, hook=True)
    planned = _train(which, True, steps=4, hook=True)
    _assert_same(eager, planned)
    assert len(eager["snaps"]) == len(planned["snaps"]) > 4
    for (oa, ga), (ob, gb) in zip(eager["snaps"], planned["snaps"]):
        assert oa == ob and torch.equal(ga, gb), oa


def test_plan_rerecords_on_shape_change():
    """A new batch shape is a new signature: eager warm-up, its own recording, then replays; the
    previous shape's plan stays cached (an epoch's smaller last batch must not cost the full batch
    its plan), and a replayed step's gradient equals an eager one."""
    from stfunet import engine
    os.environ["STF_PLAN"] = "1"
    try:
        model = _make("unet")
        small = _batches("unet", 2, b=2, hw=64)
        big = _batches("unet", 2, b=3, hw=64)
        rt = model.program.runtime
        plans = []
        for x, t in small * 2 + big * 2 + small * 2:
            for p in model.parameters():
                p.grad = None
            loss = engine.criterion(model(x), t)
            loss.backward()
            plans.append(rt.fwd)
        p_small, p_big = plans[1], plans[5]
        assert plans[0] is None and p_small is not None and plans[2] is p_small and plans[3] is p_small
        assert plans[4] is p_small                     # the big shape's eager warm-up step
        assert p_big is not None and p_big is not p_small and plans[6] is p_big and plans[7] is p_big
        assert plans[8] is p_small and plans[9] is p_small        # back to small: no re-recording
        assert len(rt.entries) == 2
        # the replayed small-batch gradient equals an eager one from the same weights
        g_plan = model.program.flat.grad.clone()
        os.environ["STF_PLAN"] = "0"
        x, t = small[1]
        model.program.flat.grad.zero_()
        for p in model.parameters():
            p.grad = None
        engine.criterion(model(x), t).backward()
        assert torch.equal(model.program.flat.grad, g_plan)
    finally:
        os.environ.pop("STF_PLAN", None)


def test_plan_two_forwards_before_backward():
    """forward A, forward B, backward A, backward B == the eager gradients: B must not replay
    over the static state A's backward still needs."""
    from stfunet import engine
    bs = _batches("stf", 2)

    def run(plan_on):
        os.environ["STF_PLAN"] = "1" if plan_on else "0"
        try:
            model = _make("stf")
            for i in range(3):                   # warm-up + record + one replay
                x, t = bs[i % 2]
                for p in model.parameters():
                    p.grad = None
                engine.criterion(model(x), t).backward()
            grads = []
            la = engine.criterion(model(bs[0][0]), bs[0][1])
            lb = engine.criterion(model(bs[1][0]), bs[1][1])
            for loss in (la, lb):
                model.program.flat.grad.zero_()
                for p in model.parameters():
                    p.grad = None
                loss.backward()
                grads.append(model.program.flat.grad.clone())
            return grads
        finally:
            os.environ.pop("STF_PLAN", None)

    ge, gp = run(False), run(True)
    assert torch.equal(ge[0], gp[0]) and torch.equal(ge[1], gp[1])


def test_plan_utility_ops():
    """stf_memset / stf_copy_rows / stf_i64_add_batch / stf_stream_wait."""
    import ctypes
    from stfunet import _lib, nhwc
    src = torch.randn(7, 33, device="cuda")
    dst = torch.full((7, 20), -1.0, device="cuda")
    nhwc.copy_rows(src, 33, dst, 20, 7, 19)
    assert torch.equal(dst[:, :19], src[:, :19]) and bool((dst[:, 19] == -1).all())
    z = torch.randn(1000, device="cuda")
    nhwc.memset0(z)
    assert bool((z == 0).all())
    cnt = [torch.tensor(5, dtype=torch.long, device="cuda") for _ in range(70)]
    arr = (ctypes.c_void_p * 70)(*[c.data_ptr() for c in cnt])
    _lib.call("stf_i64_add_batch", arr, 70, 3, _lib.stream())
    assert all(int(c) == 8 for c in cnt)
    side = torch.cuda.Stream()
    a = torch.zeros(1 << 22, device="cuda")
    a.add_(1.0)
    nhwc.wait(side, torch.cuda.current_stream())
    with torch.cuda.stream(side):
        b = a * 2
    nhwc.wait(torch.cuda.current_stream(), side)
    assert bool((b == 2).all())


_GC_SCRIPT = r"""
import contextlib, gc, sys, torch
sys.path.insert(0, "stf-unet_amd")
from stfunet import UNet, engine, plan
from stfunet.synthetic import dce_batch
plan._no_gc = contextlib.nullcontext          # the GC-off guard bypassed: the pool lifetime alone
gc.disable()                                 # collections only where this script asks for them
x, t = dce_batch(2, 8, 64, 64, seed=0, device="cuda")
x = x.flatten(1, 2)
def steps(m):
    for _ in range(3):
        engine.criterion(m(x), t).backward()
def pools(m):
    return sum(e.pool is not None for e in m.program.runtime.entries.values())
a = UNet(in_channels=8, num_classes=2, base_c=8).cuda().train()
steps(a)                                     # a's plans and private pool are recorded
c = UNet(in_channels=8, num_classes=2, base_c=8).cuda().train()
steps(c)
assert pools(a) == 1 and pools(c) == 1, (pools(a), pools(c))
import weakref
a.cycle = a                                  # only the cyclic collector can free a (and its pool) now
a_prog, a_rt = weakref.ref(a.program), weakref.ref(a.program.runtime)
a_pool = lambda: None                        # (weak references to a collected pool clear even if rescued)
del a
seen = []
ev0 = dict(plan.POOL_EVENTS)
def hook(rt, phase):                         # inside b's recording, its pool context open
    if seen:
        return
    c.program.runtime.close()                # drop the last reference to another live entry's pool
    after_close = len(plan._GRAVEYARD)
    n = gc.collect()                         # collect the dead program a, its entry and pool
    seen.append((phase, n, after_close, len(plan._GRAVEYARD), plan._POOL_ACTIVE,
                 a_prog() is None, a_rt() is None, a_pool() is None, dict(plan.POOL_EVENTS)))
plan.RECORD_HOOK = hook
b = UNet(in_channels=8, num_classes=2, base_c=8).cuda().train()
steps(b)                                     # b records: the hook runs inside the recording
plan.RECORD_HOOK = None
print(seen, plan.POOL_EVENTS)
phase, n, after_close, buried, active, prog_dead, rt_dead, pool_dead, ev = seen[0]
assert phase == "forward" and active == 1, seen
assert after_close >= 1, seen                # c's pool: deferred, not destroyed inside the context
assert prog_dead and rt_dead, seen           # the dead program was collected ...
assert ev["entry_del"] >= 1 and buried >= after_close + 1, seen   # ... its entry's pool buried, not freed
assert ev["destroyed"] == ev0["destroyed"], (seen, ev0)           # nothing destroyed inside the context
assert not plan._GRAVEYARD, len(plan._GRAVEYARD)   # destroyed at the recording's exit
assert plan.POOL_EVENTS["destroyed"] >= ev0["destroyed"] + 2, (plan.POOL_EVENTS, ev0)
steps(c)                                     # c records again from scratch
torch.cuda.synchronize()
print("ok")
"""


def test_plan_pool_lifetime_is_explicit():
    """A recorded entry's private MemPool is never destroyed while a recording's pool context
    is open (torch raises inside the pool's destructor then, which aborted the full GPU suite
    in round 3 during an STF forward recording, test_dice_gpu).  Deterministic (a child
    process, the GC-off guard bypassed): inside program b's forward recording a hook closes
    program c's runtime -- dropping the last reference to its pool -- and runs gc.collect()
    over a dead program a held only by a reference cycle.  Both pools must go to the graveyard
    (pool context count 1 at that moment, neither pool destroyed) and be destroyed once the
    recording's context exits; the process exits cleanly and c records again afterwards."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _GC_SCRIPT], cwd=root, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "ok" in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
