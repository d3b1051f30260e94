"""Two ranks sharing one GPU over gloo (as tests/test_ddp_world2_gpu.py): per-step losses, gradient
sums and final parameter sums of the STF data-parallel step, three times eager and three times through
plans, to see where runs diverge (a missing cross-stream wait shows up as runs that differ; found the
encoder / LSTM side-stream race of round 5).
    W2_STEPS=8 [W2_NODDP=1: no all-reduce] [--sync: host sync every step] python tools/world2_debug.py"""
import os
import socket
import sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "stf-unet_amd")]
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
SYNC = "--sync" in sys.argv          # float() every step (hides a missing stream dependency)


def steps(rank, plan_on, n=int(os.environ.get("W2_STEPS", "4"))):
    from stfunet import STFLSTMUNet, engine
    from stfunet.ddp import GradAllReduce
    from stfunet.optim import AdamW
    from stfunet.synthetic import dce_batch
    os.environ["STF_PLAN"] = "1" if plan_on else "0"
    torch.manual_seed(0)
    m = STFLSTMUNet(in_channels=1, num_classes=2, time_steps=4).cuda().train()
    bs = [dce_batch(2, 4, 128, 128, seed=500 + r, device="cuda", mask_hw=(64, 64)) for r in range(2)]
    opt = AdamW(m.parameters(), lr=1e-3, weight_decay=1e-4)
    ddp = GradAllReduce(m, bucket_mb=0.5) if os.environ.get("W2_NODDP") != "1" else None
    out = []
    for i in range(n):
        x, t = bs[(rank + i) % 2]
        loss = engine.criterion(m(x), t)
        opt.zero_grad()
        loss.backward()
        if ddp is not None:
            ddp.finish()
        g = m.program.flat.grad.detach().double()
        opt.step()
        if SYNC:
            out.append((float(loss), float(g.abs().sum()), float((g * g).sum())))
        else:                  # as the test: no host sync inside the loop
            out.append((loss.detach().clone(), g.abs().sum(), (g * g).sum()))
    torch.cuda.synchronize()
    out = [tuple(float(v) for v in o) for o in out]
    out.append((float(m.program.flat.data.double().abs().sum()), 0.0, 0.0))
    m.program.grad_ready_hook = None
    return out


def worker(rank, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    res = {k: steps(rank, p) for k, p in (("eager1", False), ("eager2", False), ("eager3", False), ("plan1", True), ("plan2", True), ("plan3", True))}
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=240) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
    for rank in (0, 1):
        for k, v in out[rank].items():
            print(rank, k, " | ".join(f"{a:.9g} {b:.9g} {c:.9g}" for a, b, c in v))
