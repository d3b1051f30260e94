"""HBM rate of the BatchNorm elementwise kernels at the cfg2 256^2 x 64-channel shape
(batch 64): bn_act (+pool), bn_bwd_reduce (+pool routing), bn_bwd_apply.
    python tools/bn_bench.py [H C B]"""
import ctypes
import os
import sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "stf-unet_amd")]
import torch
from stfunet import nhwc
from stfunet._lib import call, stream
from stfunet.nhwc import _p

a = [int(v) for v in sys.argv[1:]]
H, C, B = (a + [256, 64, 64][len(a):])[:3]
dev = "cuda"
M = B * H * H
y = nhwc.new_feat(B, H, H, C, dev); y.buf.normal_()
dz = nhwc.new_feat(B, H, H, C, dev); dz.buf.normal_()
out = nhwc.new_feat(B, H, H, C, dev)
pooled = nhwc.new_feat(B, H // 2, H // 2, C, dev); pooled.buf.normal_()
st = nhwc.BNState(C, dev, M, 1)
st.scale.fill_(1.0); st.shift.fill_(0.1); st.mean.zero_(); st.invstd.fill_(1.0)
coef = torch.randn(3 * C, device=dev)
lib = __import__("stfunet._lib", fromlist=["load"]).load()


def timeit(fn, reps=10):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


E = M * C
tiles = lib.stf_bn_bwd_tiles(B, H, H, C, 1, 0)
ptiles = lib.stf_bn_bwd_tiles(B, H, H, C, 1, 1)
part = torch.empty(max(tiles, ptiles) * 2 * C, device=dev)
g = nhwc.new_feat(B, H, H, C, dev)
bpart = torch.empty(lib.stf_bn_bwd_apply_tiles(M, C) * C, device=dev)
dbias = torch.empty(C, device=dev)
rows = [
    ("bn_act", 4, lambda: call("stf_bn_act", y.ptr(), C, B, H, H, C, 1, _p(st.scale), _p(st.shift), 1, None, 0,
                                 None, None, out.ptr(), C, None, stream())),
    ("bn_act+pool", 4.5, lambda: call("stf_bn_act", y.ptr(), C, B, H, H, C, 1, _p(st.scale), _p(st.shift), 1, None,
                                        0, None, None, out.ptr(), C, pooled.ptr(), stream())),
    ("bwd_reduce relu", 4, lambda: call("stf_bn_bwd_reduce", dz.ptr(), C, None, y.ptr(), C, B, H, H, C, 1,
                                          _p(st.scale), _p(st.shift), _p(st.mean), _p(st.invstd), 1, None, 0, None,
                                          _p(part), stream())),
    ("bwd_reduce pool", 6.5, lambda: call("stf_bn_bwd_reduce", dz.ptr(), C, pooled.ptr(), y.ptr(), C, B, H, H, C, 1,
                                          _p(st.scale), _p(st.shift), _p(st.mean), _p(st.invstd), 1, None, 0, g.ptr(),
                                          _p(part), stream())),
    ("bwd_apply relu", 6, lambda: call("stf_bn_bwd_apply", dz.ptr(), C, y.ptr(), C, M, C, 1, _p(st.scale),
                                         _p(st.shift), _p(coef), out.ptr(), C, None, None, stream())),
    ("bwd_apply+dbias", 6, lambda: call("stf_bn_bwd_apply", g.ptr(), C, y.ptr(), C, M, C, 1, None, None, _p(coef),
                                          out.ptr(), C, _p(bpart), _p(dbias), stream())),
]
for name, bpe, fn in rows:
    us = timeit(fn)
    print(f"{name:18s} {us:8.1f} us  {bpe * E / us / 1e6:6.2f} TB/s  ({bpe} B/elem, {E / 1e6:.0f} M elems)")
