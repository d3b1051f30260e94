"""ConvTranspose2d(k=2, s=2) forward (scatter epilogue) and input-gradient igemm
timings of the UNet decoder shapes at batch B, under whatever STF_IGEMM_CFG the
environment forces (tools/ab_convt.sh sweeps it).  Usage: python tools/convt_cfg.py [B]"""
import os
import sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "stf-unet_amd")]
import torch
from stfunet import nhwc

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
R = 10


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


cfg = os.environ.get("STF_IGEMM_CFG", "auto")
tf_tot = td_tot = tw_tot = 0.0
for h, cin in ((16, 1024), (32, 512), (64, 256), (128, 128)):
    cout = cin // 2
    x = nhwc.new_feat(B, h, h, cin, "cuda")
    x.buf.normal_()
    cat = nhwc.new_feat(B, 2 * h, 2 * h, 2 * cout, "cuda")
    cat.buf.normal_()
    w = torch.randn(cin, cout, 2, 2, device="cuda") * 0.05
    b = torch.randn(cout, device="cuda")
    w2 = nhwc.pack_weight(w, 2)
    w3 = nhwc.pack_weight(w, 3)
    up = cat.slice(0, cout)
    tf = timeit(lambda: nhwc.igemm(x, w2, 4 * cout, up, 1, 1, 1, 0, bias=b, scatter2x2=True))
    dense = nhwc.new_feat(B, 2 * h, 2 * h, cout, "cuda")
    tfd = timeit(lambda: nhwc.igemm(x, w2, 4 * cout, dense, 1, 1, 1, 0, bias=b, scatter2x2=True))
    tz = timeit(lambda: dense.buf.zero_())
    dy = nhwc.new_feat(B, 2 * h, 2 * h, cout, "cuda")
    dy.buf.normal_()
    td = timeit(lambda: nhwc.igemm(dy, w3, cin, x, 2, 2, 2, 0))
    dw = torch.empty(cin * cout * 4, device="cuda")
    tw = timeit(lambda: nhwc.wgrad(x, dy, 2, 2, 2, 0, dw))
    mb = (B * h * h * cin * 2 + 4 * B * h * h * cout * 2) / 1e6
    print(f"cfg {cfg}  up{h:<4d} {cin:5d}->{cout:5d}  fwd {tf:7.1f} us ({mb / tf:5.2f} TB/s alg; dense dst {tfd:6.1f} us, its zero_ {tz:6.1f} us)  "
          f"dgrad {td:7.1f} us  wgrad {tw:7.1f} us", flush=True)
    tf_tot += tf
    td_tot += td
    tw_tot += tw
print(f"cfg {cfg}  TOTAL fwd {tf_tot:.1f} us  dgrad {td_tot:.1f} us  wgrad {tw_tot:.1f} us", flush=True)
