"""Timing-only ablations of the UNet step (WRONG numerics; upper bounds of a fusion's gain).

    python tools/ablate_bench.py <ablation>[,<ablation>...] [bench.py args]

  bn1     every DoubleConv's first BN+ReLU pass is skipped (conv2 and its weight gradient read
          the raw conv1 output): the most that applying BN1+ReLU inside conv2's operand staging
          could save (VERDICT r02 "consumer-side BN fusion", forward half)
  bnapply the BatchNorm-backward apply passes are skipped (the statistics still finalized, the
          incoming gradient used as dy): the most that folding dy = A g + B y + C into the
          consumers' operand loads could save (the backward half)
  slab    every split of the fused 3x3 weight gradient writes the same slab (L2-resident) and
          the many-split reductions are skipped: the most an in-kernel split-K fold could save
  none    no ablation (the same process layout, for the A/B)
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "stf-unet_amd"))
sys.path.insert(0, ROOT)


def main():
    which = set(sys.argv[1].split(","))
    sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[2:]
    if "slab" in which:
        os.environ["STF_WGRAD_ONE_SLAB"] = "1"
        os.environ["STF_ABLATION"] = "1"
    import bench
    from stfunet import nhwc, unet

    if "bn1" in which:
        def _forward(self, src, training, need_bwd, out=None, pooled=None):
            conv1, bn1, conv2, bn2 = self.blk[0], self.blk[1], self.blk[3], self.blk[4]
            C, dev = self.cout, src.buf.device
            s = unet._Saved()
            s.src = src
            y1 = nhwc.new_feat(src.N, src.H, src.W, C, dev)
            st, tiles = nhwc.igemm(src, nhwc.pack_weight(conv1.weight, 0, src.C), C, y1, 3, 3, 1, 1,
                                   bias=conv1.bias.detach(), want_stats=training)
            s.bn1 = nhwc.bn_finalize(st, tiles, bn1, y1.M, training)
            a1 = y1                                           # ablated: no bn_act pass
            y2 = nhwc.new_feat(src.N, src.H, src.W, C, dev)
            st, tiles = nhwc.igemm(a1, nhwc.pack_weight(conv2.weight, 0, C), C, y2, 3, 3, 1, 1,
                                   bias=conv2.bias.detach(), want_stats=training)
            s.bn2 = nhwc.bn_finalize(st, tiles, bn2, y2.M, training)
            if out is not None:
                nhwc.bn_act(y2, s.bn2, out, pooled=pooled)
            s.y1, s.a1, s.y2 = y1, a1, y2
            return s if need_bwd else None
        unet.DoubleConvProgram._forward = _forward

    if "bnapply" in which:
        real_call = nhwc.call

        def call(name, *args):
            if name == "stf_bn_bwd_apply":
                return None
            return real_call(name, *args)
        orig = nhwc.bn_backward_from_partial

        def bn_backward_from_partial(g, y, st, bn, part, tiles, dgamma, dbeta, dbias=None, out=None,
                                     mask_relu=False):
            prev, nhwc.call = nhwc.call, call
            try:
                orig(g, y, st, bn, part, tiles, dgamma, dbeta, dbias, out=out, mask_relu=mask_relu)
            finally:
                nhwc.call = prev
            return g                                          # ablated: dy = the incoming gradient
        nhwc.bn_backward_from_partial = bn_backward_from_partial

    if "slab" in which:
        real_call2 = nhwc.call

        def call2(name, *args):
            if name == "stf_wgrad_reduce" and args[3] == 3 and args[4] == 3 and args[1] > 8:
                return None
            return real_call2(name, *args)
        nhwc.call = call2

    bench.main()


if __name__ == "__main__":
    main()
