"""Per-scale timing of the LSTM step GEMMs (STF cfg3: T=8, B=16): forward step (cell
epilogue), backward recompute step (cell-backward epilogue), the d[x|h] GEMM, and the
same GEMM shape as a plain 1x1 conv (bf16 store, no epilogue) for reference.
    python tools/lstm_bench.py            (STF_LSTM_CFG=A|B|C|D forces the step tile)"""
import os
import sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "stf-unet_amd")]
import torch
from stfunet import nhwc
from stfunet._lib import LstmEpi
from stfunet.nhwc import _p

dev = "cuda"
R = 20


def timeit(fn):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(R):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / R * 1e3


B = 16
for h, C in ((64, 64), (32, 128), (16, 256), (8, 512)):
    P = B * h * h
    src = nhwc.new_feat(B, h, h, 2 * C, dev)
    src.buf.normal_()
    w = (torch.randn(4 * C * 2 * C, device=dev) * 0.05).to(torch.bfloat16)
    wt = (torch.randn(4 * C * 2 * C, device=dev) * 0.05).to(torch.bfloat16)
    bias = torch.randn(4 * C, device=dev)
    cp = torch.randn(P, C, device=dev)
    co = torch.empty(P, C, device=dev)
    hout = nhwc.new_feat(B, h, h, C, dev)
    dh = nhwc.new_feat(B, h, h, C, dev)
    dh.buf.normal_()
    dg = nhwc.new_feat(B, h, h, 4 * C, dev)
    dc = torch.randn(P, C, device=dev)
    d2 = nhwc.new_feat(B, h, h, 2 * C, dev)
    plain = nhwc.new_feat(B, h, h, 4 * C, dev)
    fl = 2.0 * P * 4 * C * 2 * C
    efw = LstmEpi(_p(cp), _p(co), hout.ptr(), hout.cs, None)
    ebw = LstmEpi(_p(cp), _p(co), None, 0, None, 1, dh.ptr(), dh.cs, _p(dc), _p(dc), dg.ptr())
    t_fw = timeit(lambda: nhwc.igemm(src, w, 4 * C, src, 1, 1, 1, 0, bias=bias, lstm=efw))
    t_bw = timeit(lambda: nhwc.igemm(src, w, 4 * C, src, 1, 1, 1, 0, bias=bias, lstm=ebw))
    t_dx = timeit(lambda: nhwc.igemm(dg, wt, 2 * C, d2, 1, 1, 1, 0))
    t_pl = timeit(lambda: nhwc.igemm(src, w, 4 * C, plain, 1, 1, 1, 0, bias=bias))
    print(f"C={C:4d} P={P:6d}  fwd {t_fw:7.1f} us  bwd-recompute {t_bw:7.1f} us  dxh {t_dx:7.1f} us  "
          f"plain-1x1 {t_pl:7.1f} us  ({fl/1e9:.2f} GF; plain {fl/t_pl/1e6:.0f} TF/s)", flush=True)
