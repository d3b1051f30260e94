"""Run one cfg2 conv layer repeatedly (for PMC counter passes).
    python tools/one_layer.py {fwd|dgrad|wgrad} H CIN COUT [REPS]"""
import os
import sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "stf-unet_amd")]
import torch
from stfunet import nhwc

what, H, ci, co = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 5
B, dev = 64, "cuda"
x = nhwc.new_feat(B, H, H, ci, dev)
x.buf.normal_()
y = nhwc.new_feat(B, H, H, co, dev)
y.buf.normal_()
w = torch.randn(co, ci, 3, 3, device=dev) * 0.05
wp = nhwc.pack_weight(w, 0, ci)
out = torch.empty(co * ci * 9, device=dev)
for _ in range(reps):
    if what == "fwd":
        nhwc.igemm(x, wp, co, y, 3, 3, 1, 1, want_stats=True)
    elif what == "dgrad":
        nhwc.conv_dgrad(y, w, x, 3, 3, 1, 1)
    else:
        nhwc.wgrad(y, x, 3, 3, 1, 1, out)
torch.cuda.synchronize()
print("ok")
