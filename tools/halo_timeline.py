"""Where the halo conv kernel's time goes: cycle buckets per wave from the DIAG=4
build (s_memtime around the DMA wait, the stage barrier, the DMA issue, the nine
taps' MFMAs and the epilogue), summed over all waves of one launch.
    python tools/halo_timeline.py [H CIN COUT [B]]      (default: 256 64 64 64)"""
import os
import sys
os.environ["STF_HALO_DIAG"] = "4"
os.environ["STF_ABLATION"] = "1"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "stf-unet_amd")]
import torch
from stfunet import nhwc

a = [int(v) for v in sys.argv[1:]]
H, ci, co, B = (a + [256, 64, 64, 64][len(a):])[:4]
dev = "cuda"
x = nhwc.new_feat(B, H, H, ci, dev)
x.buf.normal_()
y = nhwc.new_feat(B, H, H, co, dev)
w = torch.randn(co, ci, 3, 3, device=dev) * 0.05
wp = nhwc.pack_weight(w, 0, ci)
for rep in range(3):
    stats, tiles = nhwc.igemm(x, wp, co, y, 3, 3, 1, 1, want_stats=True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    stats, tiles = nhwc.igemm(x, wp, co, y, 3, 3, 1, 1, want_stats=True)
    e1.record()
    torch.cuda.synchronize()
nw = 8
buf = stats.view(torch.int64)[: tiles * nw * 8].view(tiles, nw, 8)[:, :, :5].double()
tot = buf.sum((0, 1))
names = ["dma wait", "barrier", "dma issue", "taps (MFMA)", "epilogue"]
ms = e0.elapsed_time(e1)
per_wave = buf.sum(2)
print(f"H={H} {ci}->{co} B={B}: {ms:.3f} ms, {2.0 * B * H * H * co * 9 * ci / ms / 1e9:.0f} TF/s, "
      f"grid {tiles} x {nw} waves; cycles per wave (mean) {per_wave.mean().item():.0f} "
      f"(min {per_wave.min().item():.0f} max {per_wave.max().item():.0f})")
for n, v in zip(names, tot.tolist()):
    print(f"  {n:12s} {100.0 * v / tot.sum().item():6.2f} %   {v / (tiles * nw):12.0f} cycles/wave")
