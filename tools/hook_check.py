"""World-1 check of the data-parallel gradient hook (stfunet.ddp.GradAllReduce): with one rank the
all-reduce is the identity, so the flat gradient after finish() must equal the hook-free step's bit
for bit -- in eager mode and through plan replays.  A bucket launched before its gradients were
final would copy stale values back.  python tools/hook_check.py [unet|stf] [gloo|nccl] [eager_join]"""
import os
import sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "stf-unet_amd")]
import torch
import torch.distributed as dist

which = sys.argv[1] if len(sys.argv) > 1 else "stf"
backend = sys.argv[2] if len(sys.argv) > 2 else "gloo"
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
torch.cuda.set_device(0)
dist.init_process_group(backend, rank=0, world_size=1)
from stfunet import STFLSTMUNet, UNet, engine  # noqa: E402
from stfunet.ddp import GradAllReduce  # noqa: E402
from stfunet.optim import AdamW  # noqa: E402
from stfunet.synthetic import dce_batch  # noqa: E402


def run(hook, plan_on, steps=4):
    os.environ["STF_PLAN"] = "1" if plan_on else "0"
    torch.manual_seed(0)
    if which == "unet":
        m = UNet(in_channels=8, num_classes=2, base_c=16).cuda().train()
        bs = [dce_batch(2, 8, 128, 128, seed=500 + i, device="cuda") for i in range(2)]
        bs = [(x.flatten(1, 2), t) for x, t in bs]
    else:
        m = STFLSTMUNet(in_channels=1, num_classes=2, time_steps=4).cuda().train()
        bs = [dce_batch(2, 4, 128, 128, seed=500 + i, device="cuda", mask_hw=(64, 64)) for i in range(2)]
    opt = AdamW(m.parameters(), lr=1e-3, weight_decay=1e-4)
    ddp = GradAllReduce(m, bucket_mb=0.5) if hook else None
    grads, losses = [], []
    for i in range(steps):
        x, t = bs[i % 2]
        loss = engine.criterion(m(x), t)
        opt.zero_grad()
        loss.backward()
        if ddp is not None:
            ddp.finish()
        grads.append(m.program.flat.grad.detach().clone())
        opt.step()
        losses.append(loss.detach().clone())
    torch.cuda.synchronize()
    m.program.grad_ready_hook = None
    return grads, torch.stack(losses)


base_e, le = run(False, False)
for hook, plan_on in ((True, False), (False, True), (True, True)):
    g, l = run(hook, plan_on)
    same = [bool(torch.equal(a, b)) for a, b in zip(base_e, g)]
    diff = [float((a - b).abs().max()) for a, b in zip(base_e, g)]
    print(f"{which} hook={hook} plan={plan_on}: grads equal per step {same} maxdiff {diff} "
          f"losses equal {bool(torch.equal(le, l))}", flush=True)
dist.destroy_process_group()
