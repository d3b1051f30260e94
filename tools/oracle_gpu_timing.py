"""How long the fp32 oracle (functional torch) takes on the GPU at full spatial size:
forward / forward+backward per batch size (MIOpen kernel compilation shows in the first call)."""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "stf-unet_amd")]
import torch
from oracle import loss as o_loss, unet as o_unet
from oracle.init import canonical_state_dict
from stfunet import UNet
from stfunet.synthetic import dce_batch

torch.backends.cudnn.allow_tf32 = torch.backends.cuda.matmul.allow_tf32 = False
if os.environ.get("NO_MIOPEN") == "1":
    torch.backends.cudnn.enabled = False   # native im2col + rocBLAS convolutions: no kernel compilation
sd = {k: v.cuda() for k, v in canonical_state_dict(UNet(8, 2, 64).state_dict(), seed=0).items()}
for B in [int(b) for b in sys.argv[1:]] or [2, 2, 8, 64]:
    x, t = dce_batch(B, 8, 256, 256, seed=5, device="cuda")
    x = x.flatten(1, 2)
    p = {k: v.clone().requires_grad_(v.is_floating_point() and "running" not in k) for k, v in sd.items()}
    torch.cuda.synchronize(); t0 = time.time()
    out = o_unet.forward(p, x, training=True)["out"]
    torch.cuda.synchronize(); t1 = time.time()
    o_loss.criterion(out, t).backward()
    torch.cuda.synchronize(); t2 = time.time()
    print(f"B={B}: fwd {t1 - t0:.2f} s  bwd {t2 - t1:.2f} s", flush=True)
