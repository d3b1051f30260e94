"""Where the fused-tap 3x3 weight gradient's time goes: per-wave cycle buckets from the DIAG=4
build of wgrad3x3_kernel (s_memtime around the next tile's global-load issue, the 18 MFMA steps,
the LDS store of the staged tile -- its wait for those loads included -- and the tile barrier),
summed over all waves of one launch (timing only: the slabs are overwritten).
    python tools/wgrad_timeline.py [H CIN COUT [B]]      (default: 256 64 64 64)"""
import ctypes
import os
import sys
NODIAG = "--nodiag" in sys.argv           # time the production kernel instead
if not NODIAG:
    os.environ["STF_WGRAD_DIAG"] = "4"
    os.environ["STF_ABLATION"] = "1"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "stf-unet_amd")]
import torch
from stfunet import nhwc
from stfunet import _lib
from stfunet._lib import ConvGeom, WgradArgs, call, stream

a = [int(v) for v in sys.argv[1:] if v.isdigit()]
H, ci, co, B = (a + [256, 64, 64, 64][len(a):])[:4]
dev = "cuda"
x = nhwc.new_feat(B, H, H, ci, dev)
x.buf.normal_()
dy = nhwc.new_feat(B, H, H, co, dev)
dy.buf.normal_()
g = ConvGeom(B, H, H, ci, ci, H, H, 3, 3, 1, 1, 0)
args = WgradArgs(g, dy.ptr(), co, co, x.ptr(), None, 0, 0)
splits, nbytes = ctypes.c_int(0), ctypes.c_size_t(0)
call("stf_wgrad_plan", ctypes.byref(args), ctypes.byref(splits), ctypes.byref(nbytes))
ws = torch.empty(nbytes.value // 4, dtype=torch.float32, device=dev)
args.ws, args.splits = ws.data_ptr(), splits.value
for rep in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    call("stf_wgrad", ctypes.byref(args), stream())
    e1.record()
    torch.cuda.synchronize()
name = _lib.load().stf_wgrad_kernel_name(ctypes.byref(args)).decode()
NB = 2 if name.endswith(", 2>") else 1
blocks = splits.value * (co // (64 * NB)) * (ci // 64)
print(f"{name}: splits {splits.value} ws {nbytes.value} B; last launch {e0.elapsed_time(e1):.3f} ms, "
      f"{2.0 * B * H * H * co * ci * 9 / e0.elapsed_time(e1) / 1e9:.0f} TF/s")
if NODIAG:
    sys.exit(0)
RSC = 9 * ci
rows = []
for z in range(ci // 64):
    for y in range(co // (64 * NB)):
        for sp in range(splits.value):
            off = (sp * co * RSC + y * 64 * NB * RSC + z * 64) // 2       # u64 index of the block's buckets
            rows.append(ws.view(torch.int64)[off: off + 16 * NB])
buf = torch.stack(rows).view(blocks, 4 * NB, 4).double()
tot = buf.sum((0, 1))
ms = e0.elapsed_time(e1)
names = ["load issue", "MFMA steps", "LDS store", "barrier"]
print(f"H={H} {ci}->{co} B={B}: {ms:.3f} ms (diag build), {blocks} blocks x {4 * NB} waves; cycles per wave "
      f"{buf.sum(2).mean().item():.0f}")
for n, v in zip(names, tot.tolist()):
    print(f"  {n:12s} {100.0 * v / tot.sum().item():6.2f} %   {v / (blocks * 4 * NB):12.0f} cycles/wave")
