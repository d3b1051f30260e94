"""Per-launch time of the BatchNorm element-wise passes at the STF / UNet shapes.
    STF_BN_G=0|1 python tools/bench_bn.py      (group-major kernels off / on)"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "stf-unet_amd"))

import torch  # noqa: E402


def main():
    from stfunet import nhwc
    from stfunet.nhwc import BNState, new_feat
    from stfunet.plan import Plan
    dev = torch.device("cuda")
    # (N images, H, W, C, groups): STF cfg3 encoder levels (T*B = 128, 8 groups), UNet cfg2 levels
    shapes = [(128, 64, 64, 64, 8), (128, 32, 32, 128, 8), (128, 16, 16, 256, 8), (128, 8, 8, 512, 8),
              (16, 64, 64, 64, 1), (64, 256, 256, 64, 1), (64, 128, 128, 128, 1), (64, 32, 32, 512, 1)]
    torch.manual_seed(0)
    print(f"STF_BN_G={os.environ.get('STF_BN_G', '1')}")
    for N, H, W, C, G in shapes:
        y = new_feat(N, H, W, C, dev)
        y.buf.normal_()
        dz = new_feat(N, H, W, C, dev)
        dz.buf.normal_()
        out = new_feat(N, H, W, C, dev)
        st = BNState(C, dev, N * H * W, G)
        st.scale.uniform_(0.5, 1.5)
        st.shift.uniform_(-0.5, 0.5)
        st.mean.normal_()
        st.invstd.uniform_(0.5, 2)
        tiles = nhwc._lib.load().stf_bn_bwd_tiles(N, H, W, C, G, 0)
        part = torch.empty(G * tiles * 2 * C, device=dev)
        coef = torch.randn(G * 3 * C, device=dev)
        lib = nhwc._lib.load()
        s = nhwc.stream()
        runs = {
            "act": lambda: lib.stf_bn_act(y.ptr(), C, N, H, W, C, G, nhwc._p(st.scale), nhwc._p(st.shift), 1,
                                          None, 0, None, None, out.ptr(), C, None, s),
            "act_res": lambda: lib.stf_bn_act(y.ptr(), C, N, H, W, C, G, nhwc._p(st.scale), nhwc._p(st.shift), 1,
                                              dz.ptr(), C, None, None, out.ptr(), C, None, s),
            "reduce_m1": lambda: lib.stf_bn_bwd_reduce(dz.ptr(), C, None, y.ptr(), C, N, H, W, C, G,
                                                       nhwc._p(st.scale), nhwc._p(st.shift), nhwc._p(st.mean),
                                                       nhwc._p(st.invstd), 1, None, 0, None, nhwc._p(part), s),
            "reduce_m2g": lambda: lib.stf_bn_bwd_reduce(dz.ptr(), C, None, y.ptr(), C, N, H, W, C, G,
                                                        nhwc._p(st.scale), nhwc._p(st.shift), nhwc._p(st.mean),
                                                        nhwc._p(st.invstd), 2, out.ptr(), C, out.ptr(),
                                                        nhwc._p(part), s),
            "apply": lambda: lib.stf_bn_bwd_apply(dz.ptr(), C, y.ptr(), C, N * H * W, C, G, None, None,
                                                  nhwc._p(coef), out.ptr(), C, None, None, s),
            "apply_mask_inplace": lambda: lib.stf_bn_bwd_apply(out.ptr(), C, y.ptr(), C, N * H * W, C, G,
                                                               nhwc._p(st.scale), nhwc._p(st.shift), nhwc._p(coef),
                                                               out.ptr(), C, None, None, s),
        }
        mb = N * H * W * C * 2 / 1e6
        line = []
        for name, fn in runs.items():
            for _ in range(3):
                assert fn() == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 20
            pl = Plan()                       # replayed from C++: no host gaps between the launches
            pl.record(lambda: [fn() for _ in range(reps)])
            torch.cuda.synchronize()
            e0.record()
            pl.replay()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / reps
            line.append(f"{name} {us:6.1f}")
        print(f"  {N}x{H}x{W}x{C} G={G} ({mb:.1f} MB/tensor): " + "  ".join(line))


if __name__ == "__main__":
    main()
