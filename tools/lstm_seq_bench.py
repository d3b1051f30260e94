"""Whole-sequence LSTM forward / backward (stf_lstm_seq_fwd / _bwd) vs T per-step
launches, C = 64 at the STF scale-1 size (B=16 -> P = 65536 pixels per step), T = 8
and 32; compares the two paths' outputs.  python tools/lstm_seq_bench.py"""
import os
import sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "stf-unet_amd")]
import torch
from stfunet import nhwc
from stfunet.stf_lstm_unet import LSTMProgram

dev = "cuda"
for T in (8, 32):
    C, B, H = 64, 16, 64
    lstm = torch.nn.LSTM(C, C, batch_first=True).to(dev)
    lbuf = nhwc.zeros_feat(T * B, H, H, 2 * C, dev)
    lbuf.buf.view(T * B * H * H, 2 * C)[:, :C].normal_()
    prog = LSTMProgram(lstm)
    res = {}
    dhT = nhwc.new_feat(B, H, H, C, dev)
    dhT.buf.normal_()

    class _G:
        def __init__(self):
            self.g = {id(p): torch.zeros_like(p) for p in lstm.parameters()}

        def __call__(self, p):
            return self.g[id(p)]

    def timeit(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / 5 * 1e3
    for mode in ("0", "1"):
        os.environ["STF_LSTM_SEQ"] = mode
        hT = nhwc.new_feat(B, H, H, C, dev)
        st = prog.forward(lbuf, T, B, hT)
        gv = _G()
        dx = prog.backward(st, dhT, gv)
        torch.cuda.synchronize()
        res[mode] = (hT.buf.clone(), st.c.clone(), lbuf.buf.clone(), dx.dense().clone(),
                     *[gv(p).clone() for p in lstm.parameters()])
        tf = timeit(lambda: prog.forward(lbuf, T, B, hT))
        tb = timeit(lambda: prog.backward(st, dhT, gv))
        print(f"T={T} seq={mode}: forward {tf:8.1f} us, backward {tb:8.1f} us", flush=True)
    names = ["h_T", "c", "lbuf", "dx"] + [n for n, _ in lstm.named_parameters()]
    for n, a, b in zip(names, res["0"], res["1"]):
        a, b = a.double(), b.double()
        print(f"   {n:14s} equal={torch.equal(a, b)} rel={((a - b).norm() / b.norm().clamp_min(1e-30)).item():.2e}",
              flush=True)
