// Paired training augmentation on the device:
// RandomResize -> flips -> RandomRotation -> RandomCrop -> ToTensor/Normalize of
// transforms.py:18-157 as get_transform composes them (train.py:51-73), bit-exact to the
// Pillow arithmetic the reference runs on the CPU (oracle/augment.py states it):
//
//   resize   Pillow ImagingResample, bilinear, 22-bit fixed-point taps, horizontal pass
//            then vertical, uint8 clip after each -- here one thread per resized pixel
//            recomputes its vertical taps' horizontal sums (identical integers, no
//            intermediate image)
//   flips    index mirroring, folded into the next stage's reads
//   rotate   Pillow ImagingGenericTransform bilinear: double coordinates and lerps
//            (contraction off: the CPU build has no FMA), uint8 truncation
//   crop     zero padding beyond the resized image, then the window
//   tensor   fp32 (v / 255 - mean) / std
//
// masks take the NEAREST branch in one kernel: pretabulated resize indices (Pillow's
// ImagingScaleAffine tables, built on the host the way Pillow builds them), 16.16
// fixed-point rotation (Pillow's affine fast path), crop, int64 store.
//
// All frames of a batch (T DCE frames + PK maps per sample, any source sizes) go
// through one launch per stage from a device array of stf_aug_frame descriptors;
// grid.y = descriptor.  Bytes per 224^2 output frame: ~50 KB source + ~50 KB resized
// (written, read back through L2) + 200 KB fp32 out -- HBM-trivial; the stages are
// latency/launch-bound at training batch sizes.
#include "common.h"
#include "../../include/stfunet.h"

namespace {

constexpr int AUG_NT = 256;
constexpr int PB = 22;

STF_DEV uint8_t clip8(int v) {
  if (v >= (1 << PB << 8)) return 255;
  if (v <= 0) return 0;
  return (uint8_t)(v >> PB);
}

// coefficient rows: [xmin, n, k_0 .. k_{ks-1}] per output index
__global__ __launch_bounds__(AUG_NT) void aug_resize_kernel(const uint8_t* __restrict__ src,
                                                             const stf_aug_frame* __restrict__ fr,
                                                             const int* __restrict__ coef,
                                                             uint8_t* __restrict__ scratch) {
  const stf_aug_frame d = fr[blockIdx.y];
  const int n_out = d.H2 * d.W2;
  const int i = blockIdx.x * AUG_NT + threadIdx.x;
  if (i >= n_out) return;
  const int yy = i / d.W2, xx = i - yy * d.W2;
  const int* cx = coef + d.cx + xx * (d.kx + 2);
  const int* cy = coef + d.cy + yy * (d.ky + 2);
  const int xmin = cx[0], xn = cx[1], ymin = cy[0], yn = cy[1];
  const uint8_t* s = src + d.src;
  int acc = 1 << (PB - 1);
  for (int y = 0; y < yn; ++y) {
    const uint8_t* row = s + (long)(ymin + y) * d.W + xmin;
    int h = 1 << (PB - 1);
    for (int x = 0; x < xn; ++x) h += (int)row[x] * cx[2 + x];
    acc += (int)clip8(h) * cy[2 + y];
  }
  scratch[d.rs + i] = clip8(acc);
}

#pragma clang fp contract(off)
// Pillow bilinear_filter8 at input position (xin, yin) of the (flipped) resized image
STF_DEV uint8_t rot_bilinear(const uint8_t* img, int H, int W, bool hf, bool vf, double xin, double yin,
                             bool& ok) {
  ok = !(xin < 0.0 || xin >= W || yin < 0.0 || yin >= H);
  if (!ok) return 0;
  xin -= 0.5;
  yin -= 0.5;
  const int x = (int)floor(xin), y = (int)floor(yin);
  const double dx = xin - x, dy = yin - y;
  auto at = [&](int r, int c) -> double {
    const int rr = vf ? H - 1 - r : r, cc = hf ? W - 1 - c : c;
    return (double)img[(long)rr * W + cc];
  };
  const int x0 = x < 0 ? 0 : (x < W ? x : W - 1);
  const int x1 = x + 1 < 0 ? 0 : (x + 1 < W ? x + 1 : W - 1);
  const int y0 = y < 0 ? 0 : (y < H ? y : H - 1);
  double v1 = at(y0, x0) + (at(y0, x1) - at(y0, x0)) * dx;
  double v2;
  if (y + 1 >= 0 && y + 1 < H) v2 = at(y + 1, x0) + (at(y + 1, x1) - at(y + 1, x0)) * dx;
  else v2 = v1;
  v1 = v1 + (v2 - v1) * dy;
  return (uint8_t)(int)v1;
}

__global__ __launch_bounds__(AUG_NT) void aug_finish_kernel(const uint8_t* __restrict__ scratch,
                                                             const stf_aug_frame* __restrict__ fr, float mean,
                                                             float stdv, float* __restrict__ out) {
  const stf_aug_frame d = fr[blockIdx.y];
  const int i = blockIdx.x * AUG_NT + threadIdx.x;
  if (i >= d.oh * d.ow) return;
  const int oy = i / d.ow, ox = i - oy * d.ow;
  const int y = oy + d.h0, x = ox + d.w0;                    // position in the padded image
  const bool hf = d.flags & STF_AUG_HFLIP, vf = d.flags & STF_AUG_VFLIP;
  const uint8_t* img = scratch + d.rs;
  uint8_t v = 0;
  if (y < d.H2 && x < d.W2) {
    if (d.flags & STF_AUG_ROTATE) {
      const double xi = x + 0.5, yi = y + 0.5;
      const double xs = d.m[0] * xi + d.m[1] * yi + d.m[2];
      const double ys = d.m[3] * xi + d.m[4] * yi + d.m[5];
      bool ok;
      v = rot_bilinear(img, d.H2, d.W2, hf, vf, xs, ys, ok);
    } else {
      const int r = vf ? d.H2 - 1 - y : y, c = hf ? d.W2 - 1 - x : x;
      v = img[(long)r * d.W2 + c];
    }
  }
  const float t = __fdiv_rn((float)v, 255.0f);
  out[d.out + i] = __fdiv_rn(t - mean, stdv);
}
#pragma clang fp contract(on)

// masks: NEAREST resize tables (cx: W2 source columns, cy: H2 source rows; -1 = outside)
__global__ __launch_bounds__(AUG_NT) void aug_mask_kernel(const uint8_t* __restrict__ src,
                                                           const stf_aug_frame* __restrict__ fr,
                                                           const int* __restrict__ tabs,
                                                           int64_t* __restrict__ out) {
  const stf_aug_frame d = fr[blockIdx.y];
  const int i = blockIdx.x * AUG_NT + threadIdx.x;
  if (i >= d.oh * d.ow) return;
  const int oy = i / d.ow, ox = i - oy * d.ow;
  int y = oy + d.h0, x = ox + d.w0;
  int64_t v = 0;
  if (y < d.H2 && x < d.W2) {
    bool ok = true;
    if (d.flags & STF_AUG_ROTATE) {                          // 16.16 fixed point, >> 16
      const int xi = (d.fx[4] + y * d.fx[1] + x * d.fx[0]) >> 16;
      const int yi = (d.fx[5] + y * d.fx[3] + x * d.fx[2]) >> 16;
      ok = xi >= 0 && xi < d.W2 && yi >= 0 && yi < d.H2;
      x = xi;
      y = yi;
    }
    if (ok) {
      const int r = (d.flags & STF_AUG_VFLIP) ? d.H2 - 1 - y : y;
      const int c = (d.flags & STF_AUG_HFLIP) ? d.W2 - 1 - x : x;
      const int sr = tabs[d.cy + r], sc = tabs[d.cx + c];
      if (sr >= 0 && sc >= 0) v = src[d.src + (long)sr * d.W + sc];
    }
  }
  out[d.out + i] = v;
}

bool aug_ok(int n, int max_px) { return n >= 0 && n <= 65535 && max_px >= 0; }

unsigned blocks_for(int px) { return (unsigned)((px + AUG_NT - 1) / AUG_NT); }

}  // namespace

extern "C" int stf_augment_frames(const uint8_t* src, const stf_aug_frame* frames, int n, const int* coef,
                                  uint8_t* scratch, int max_resized_px, int max_out_px, float mean, float stdv,
                                  float* out, stf_stream_t stream) {
  if (!aug_ok(n, max_resized_px) || max_out_px < 0) return STF_EINVAL;
  if (n == 0) return 0;
  if (max_resized_px > 0) {
    hipLaunchKernelGGL(aug_resize_kernel, dim3(blocks_for(max_resized_px), n), dim3(AUG_NT), 0,
                       (hipStream_t)stream, src, frames, coef, scratch);
    STF_CHECK_LAUNCH();
  }
  if (max_out_px > 0) {
    hipLaunchKernelGGL(aug_finish_kernel, dim3(blocks_for(max_out_px), n), dim3(AUG_NT), 0, (hipStream_t)stream,
                       scratch, frames, mean, stdv, out);
    STF_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int stf_augment_masks(const uint8_t* src, const stf_aug_frame* masks, int n, const int* tabs,
                                 int max_out_px, int64_t* out, stf_stream_t stream) {
  if (!aug_ok(n, max_out_px)) return STF_EINVAL;
  if (n == 0 || max_out_px == 0) return 0;
  hipLaunchKernelGGL(aug_mask_kernel, dim3(blocks_for(max_out_px), n), dim3(AUG_NT), 0, (hipStream_t)stream, src,
                     masks, tabs, out);
  STF_CHECK_LAUNCH();
  return 0;
}
