"""Per-layer timing of the UNet(in=8, base_c=64) convolutions at batch B, 256^2:
forward igemm, dgrad igemm and wgrad, each timed with HIP events over R reps.
Prints one line per layer with TF/s.  Usage: python tools/bench_layers.py [B]"""
import os
import sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "stf-unet_amd")]
import torch
from stfunet import nhwc

B = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 64
STF = "--stf" in sys.argv
R = 5
dev = "cuda"


def timeit(fn):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(R):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / R


if STF:
    # STF-LSTM-UNet encoder (T=8 x B=16 = 128 images): ResNet-34 layer convs + LSTM step GEMMs
    imgs = 128
    tot = {"fwd": [0, 0], "dgrad": [0, 0], "wgrad": [0, 0]}
    for name, h, ci, co, st in (("l1", 64, 64, 64, 1), ("l2.s2", 64, 64, 128, 2), ("l2", 32, 128, 128, 1),
                                ("l3.s2", 32, 128, 256, 2), ("l3", 16, 256, 256, 1), ("l4.s2", 16, 256, 512, 2),
                                ("l4", 8, 512, 512, 1)):
        ho = h // st
        x = nhwc.new_feat(imgs, h, h, ci, dev)
        x.buf.normal_()
        y = nhwc.new_feat(imgs, ho, ho, co, dev)
        y.buf.normal_()
        w = torch.randn(co, ci, 3, 3, device=dev) * 0.05
        wp = nhwc.pack_weight(w, 0, ci)
        flops = 2.0 * imgs * ho * ho * co * 9 * ci
        tf = timeit(lambda: nhwc.igemm(x, wp, co, y, 3, 3, st, 1, want_stats=True, groups=8))
        td = timeit(lambda: nhwc.conv_dgrad(y, w, x, 3, 3, st, 1))
        out = torch.empty(co * ci * 9, device=dev)
        tw = timeit(lambda: nhwc.wgrad(y, x, 3, 3, st, 1, out))
        for k, t in (("fwd", tf), ("dgrad", td), ("wgrad", tw)):
            tot[k][0] += t
            tot[k][1] += flops
        print(f"{name:8s} {ho:4d}^2 {ci:5d}->{co:5d}  GF {flops/1e9:8.1f}  fwd {tf:7.3f} ms {flops/tf/1e9:7.1f} TF"
              f"  dgrad {td:7.3f} ms {flops/td/1e9:7.1f} TF  wgrad {tw:7.3f} ms {flops/tw/1e9:7.1f} TF", flush=True)
    for k, (t, f) in tot.items():
        print(f"TOTAL {k}: {t:.2f} ms  {f/t/1e9:.1f} TF/s")
    sys.exit(0)

layers = []
H = 256
widths = [64, 128, 256, 512, 1024]
cin = 8
for i, c in enumerate(widths):
    h = H >> i
    layers += [(f"enc{i+1}.0" if i < 4 else "bott.0", h, cin, c), (f"enc{i+1}.3" if i < 4 else "bott.3", h, c, c)]
    cin = c
for i in range(4):
    c = widths[3 - i]
    h = H >> (3 - i)
    layers += [(f"dec{4-i}.0", h, 2 * c, c), (f"dec{4-i}.3", h, c, c)]
tot = {"fwd": [0, 0], "dgrad": [0, 0], "wgrad": [0, 0]}
for name, h, ci, co in layers:
    x = nhwc.new_feat(B, h, h, ci, dev)
    x.buf.normal_()
    y = nhwc.new_feat(B, h, h, co, dev)
    y.buf.normal_()
    w = torch.randn(co, ci, 3, 3, device=dev) * 0.05
    wp = nhwc.pack_weight(w, 0, ci)
    flops = 2.0 * B * h * h * co * 9 * ci
    tf = timeit(lambda: nhwc.igemm(x, wp, co, y, 3, 3, 1, 1, want_stats=True))
    td = timeit(lambda: nhwc.conv_dgrad(y, w, x, 3, 3, 1, 1)) if ci % 32 == 0 else float("nan")
    out = torch.empty(co * ci * 9, device=dev)
    tw = timeit(lambda: nhwc.wgrad(y, x, 3, 3, 1, 1, out))
    for k, t in (("fwd", tf), ("dgrad", td), ("wgrad", tw)):
        if t == t:
            tot[k][0] += t
            tot[k][1] += flops
    print(f"{name:8s} {h:4d}^2 {ci:5d}->{co:5d}  GF {flops/1e9:8.1f}  fwd {tf:7.3f} ms {flops/tf/1e9:7.1f} TF"
          f"  dgrad {td:7.3f} ms {flops/td/1e9:7.1f} TF  wgrad {tw:7.3f} ms {flops/tw/1e9:7.1f} TF", flush=True)
for k, (t, f) in tot.items():
    print(f"TOTAL {k}: {t:.2f} ms  {f/t/1e9:.1f} TF/s")

# ConvTranspose2d(k=2, s=2) of the decoder: forward (scatter epilogue into the concat
# half), input gradient (stride-2 2x2 gather) and weight gradient
tot = [0, 0, 0, 0]
for h, cin in ((16, 1024), (32, 512), (64, 256), (128, 128)):
    cout = cin // 2
    x = nhwc.new_feat(B, h, h, cin, dev)
    x.buf.normal_()
    cat = nhwc.new_feat(B, 2 * h, 2 * h, 2 * cout, dev)
    cat.buf.normal_()
    w = torch.randn(cin, cout, 2, 2, device=dev) * 0.05
    b = torch.randn(cout, device=dev)
    w2 = nhwc.pack_weight(w, 2)
    w3 = nhwc.pack_weight(w, 3)
    flops = 2.0 * B * h * h * cin * 4 * cout
    up = cat.slice(0, cout)
    tf = timeit(lambda: nhwc.igemm(x, w2, 4 * cout, up, 1, 1, 1, 0, bias=b, scatter2x2=True))
    dy = nhwc.new_feat(B, 2 * h, 2 * h, cout, dev)
    dy.buf.normal_()
    td = timeit(lambda: nhwc.igemm(dy, w3, cin, x, 2, 2, 2, 0))
    out = torch.empty(cin * cout * 4, device=dev)
    tw = timeit(lambda: nhwc.wgrad(x, dy, 2, 2, 2, 0, out))
    print(f"up{h:<5d} {h:4d}^2 {cin:5d}->{cout:5d}  GF {flops/1e9:8.1f}  fwd {tf:7.3f} ms {flops/tf/1e9:7.1f} TF"
          f"  dgrad {td:7.3f} ms {flops/td/1e9:7.1f} TF  wgrad {tw:7.3f} ms {flops/tw/1e9:7.1f} TF", flush=True)
    tot[0] += tf; tot[1] += td; tot[2] += tw; tot[3] += flops
print(f"TOTAL convT: fwd {tot[0]:.2f} ms dgrad {tot[1]:.2f} ms wgrad {tot[2]:.2f} ms")
