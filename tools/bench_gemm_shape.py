"""Time one 1x1 stf_igemm shape (HIP events over R reps) under the current environment's tile /
split-K switches: python tools/bench_gemm_shape.py M N K [dst_cs] -- e.g. STF lstm4's per-step dh
GEMM 1024 512 2048 1024 (STF_IGEMM_CFG / STF_SPLITK select the variant; read once per process)."""
import os
import sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "stf-unet_amd")]
import torch
from stfunet import nhwc
from stfunet._lib import load

M, N, K = (int(v) for v in sys.argv[1:4])
dcs = int(sys.argv[4]) if len(sys.argv) > 4 else N
dev = "cuda"
src = nhwc.new_feat(M // 64, 8, 8, K, dev)
src.buf.normal_()
w = (torch.randn(N * K, device=dev) / K ** 0.5).to(nhwc.sdt())
full = nhwc.new_feat(M // 64, 8, 8, dcs, dev)
dst = full.slice(dcs - N, N) if dcs > N else full
for _ in range(3):
    nhwc.igemm(src, w, N, dst, 1, 1, 1, 0)
torch.cuda.synchronize()
R = 50
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(R):
    nhwc.igemm(src, w, N, dst, 1, 1, 1, 0)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / R * 1e3
tag = " ".join(f"{k}={os.environ[k]}" for k in ("STF_IGEMM_CFG", "STF_SPLITK") if k in os.environ)
print(f"M={M} N={N} K={K} dcs={dcs} {tag or 'default'}: {us:.1f} us  {2 * M * N * K / us / 1e6:.1f} TF/s")
