// Flat AdamW, layout packs (input NCHW fp32 -> NHWC bf16, fp32 weights -> bf16
// GEMM rows), per-channel column sums, and the error-string helper.
#include "common.h"
#include "../../include/stfunet.h"
#include "reduce.h"

__global__ void stf_tile_sum_kernel(const float* __restrict__ partial, int tiles, int C, float* __restrict__ out);

namespace {

constexpr int NT = 256;

// torch.optim.AdamW (decoupled weight decay), PyTorch evaluation order:
//   p *= 1 - lr*wd;  m = b1 m + (1-b1) g;  v = b2 v + (1-b2) g^2;
//   p -= (lr/bc1) * m / (sqrt(v)/sqrt(bc2) + eps)
__global__ void adamw_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                             float* __restrict__ v, long n, float lr, float b1, float b2, float eps, float wd,
                             float step_size, float inv_sqrt_bc2) {
  const long n4 = n / 4;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n4; i += (long)gridDim.x * NT) {
    float4 pv = reinterpret_cast<float4*>(p)[i];
    const float4 gv = reinterpret_cast<const float4*>(g)[i];
    float4 mv = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
    float* pp = &pv.x; const float* gg = &gv.x; float* mm = &mv.x; float* ww = &vv.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pp[j] *= 1.f - lr * wd;
      mm[j] = mm[j] + (1.f - b1) * (gg[j] - mm[j]);
      ww[j] = b2 * ww[j] + (1.f - b2) * gg[j] * gg[j];
      pp[j] -= step_size * mm[j] / (sqrtf(ww[j]) * inv_sqrt_bc2 + eps);
    }
    reinterpret_cast<float4*>(p)[i] = pv;
    reinterpret_cast<float4*>(m)[i] = mv;
    reinterpret_cast<float4*>(v)[i] = vv;
  }
  for (long i = n4 * 4 + blockIdx.x * (long)NT + threadIdx.x; i < n; i += (long)gridDim.x * NT) {
    float pp = p[i] * (1.f - lr * wd);
    const float gg = g[i];
    const float mm = m[i] + (1.f - b1) * (gg - m[i]);
    const float ww = b2 * v[i] + (1.f - b2) * gg * gg;
    pp -= step_size * mm / (sqrtf(ww) * inv_sqrt_bc2 + eps);
    p[i] = pp; m[i] = mm; v[i] = ww;
  }
}

__global__ void pack_input_kernel(const float* __restrict__ x, int N, int C, int H, int W, int Cpad,
                                  uint16_t* __restrict__ out) {
  // 32-bit index math (the host checks N*H*W*Cpad/8 < 2^31): three 64-bit divisions per unit
  // made this pass VALU-bound (3.3 TB/s on cfg2's 0.2 GB)
  const int HW = H * W, P = N * HW;
  const int CG = Cpad / 8;
  for (int u = blockIdx.x * NT + threadIdx.x; u < P * CG; u += gridDim.x * NT) {
    const int cg = u / P;
    const int pix = u - cg * P;        // consecutive threads -> consecutive pixels (coalesced reads)
    const int n = pix / HW, hw = pix - n * HW;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = cg * 8 + j;
      v[j] = c < C ? x[((size_t)n * C + c) * HW + hw] : 0.f;
    }
    *reinterpret_cast<uint4*>(out + (size_t)pix * Cpad + cg * 8) = pack8(v);
  }
}

// out element index -> source value, per mode (see include/stfunet.h).  32-bit
// index math (every packed weight is < 2^31 elements; stf_pack_weight(s) check).
STF_DEV float pack_src(const float* __restrict__ w, int d0, int d1, int R, int S, int mode, int cpad, int o) {
  const int RS = R * S;
  if (mode == 0) {              // Conv2d w[Co=d0][Ci=d1][R][S] -> [Co][R][S][cpad]
    const int t = o / cpad, c = o - t * cpad;
    const int co = t / RS, tap = t - co * RS;
    return c < d1 ? w[(co * d1 + c) * RS + tap] : 0.f;
  } else if (mode == 1) {       // Conv2d -> [Ci][R][S][Co]
    const int t = o / d0, co = o - t * d0;
    const int ci = t / RS, tap = t - ci * RS;
    return w[(co * d1 + ci) * RS + tap];
  } else if (mode == 2) {       // ConvT w[Ci=d0][Co=d1][R][S] -> [(tap)*Co + co][Ci]
    const int t = o / d0, ci = o - t * d0;
    const int tap = t / d1, co = t - tap * d1;
    return w[(ci * d1 + co) * RS + tap];
  } else if (mode == 3) {       // ConvT -> [Ci][R][S][Co]
    const int t = o / d1, co = o - t * d1;
    const int ci = t / RS, tap = t - ci * RS;
    return w[(ci * d1 + co) * RS + tap];
  } else if (mode == 5) {       // Conv2d -> [Ci][R-1-r][S-1-s][Co] (stride-1 dgrad as a forward gather)
    const int t = o / d0, co = o - t * d0;
    const int ci = t / RS, tap = t - ci * RS;
    const int r = tap / S, s_ = tap - r * S;
    return w[(co * d1 + ci) * RS + (R - 1 - r) * S + (S - 1 - s_)];
  }
  // mode 4: ConvT -> [Co][R][S][Ci]
  const int t = o / d0, ci = o - t * d0;
  const int co = t / RS, tap = t - co * RS;
  return w[(ci * d1 + co) * RS + tap];
}

STF_DEV long pack_total(int d0, int d1, int R, int S, int mode, int cpad) {
  return mode == 0 ? (long)d0 * R * S * cpad : (long)d0 * d1 * R * S;
}

__global__ void pack_weight_kernel(const float* __restrict__ w, int d0, int d1, int R, int S, int mode, int cpad,
                                   uint16_t* __restrict__ out) {
  const int total = (int)pack_total(d0, d1, R, S, mode, cpad);
  for (int o = blockIdx.x * NT + threadIdx.x; o < total; o += gridDim.x * NT)
    reinterpret_cast<e16*>(out)[o] = f2e(pack_src(w, d0, d1, R, S, mode, cpad, o));
}

// every descriptor of the list in one launch: blockIdx.y = descriptor
__global__ void pack_weights_kernel(const stf_pack_desc* __restrict__ descs) {
  const stf_pack_desc d = descs[blockIdx.y];
  const int total = (int)pack_total(d.d0, d.d1, d.R, d.S, d.mode, d.cpad);
  for (int o = blockIdx.x * NT + threadIdx.x; o < total; o += gridDim.x * NT)
    reinterpret_cast<e16*>(d.out)[o] = f2e(pack_src(d.w, d.d0, d.d1, d.R, d.S, d.mode, d.cpad, o));
}

// Tiled packing (every descriptor of the list in one launch; blockIdx.y = descriptor).
// Source w is [A = d0][Bc = d1][RS] fp32.  Modes whose rows run along A (1, 5: Conv
// dgrad rows [ci][tap][co]; 2, 4: ConvT rows over ci) transpose 32 (a) x 16 (b) x RS
// tiles through LDS; modes whose rows run along b (0: [co][tap][ci(pad)], 3: [ci][tap]
// [co]) transpose per-a [b][tap] blocks (4 a x 64 b).  Reads are whole source rows,
// writes are 16-B chunks of output rows (the element-wise gather above reads one
// scattered float per output: ~1.3 TB/s effective, 0.28 ms per cfg2 step).  32-row A tiles: 18.6 KB
// of LDS, 8 blocks per CU (64-row tiles, 37 KB, allowed 4: cfg2 167 -> 115 us per step, STF cfg3
// 127 -> 94 us; 16-row tiles 123 / 96 us).
constexpr int PK_TA = 32, PK_TB = 16, PK_IA = 4, PK_IB = 64, PK_MAXRS = 9;

STF_DEV bool pack_outer(int mode) { return mode == 1 || mode == 5 || mode == 2 || mode == 4; }

// output row (the index before the innermost a-run) of source element (b, tap) in the
// A-major modes
STF_DEV long pack_outer_row(int mode, int b, int tap, int d1, int RS) {
  if (mode == 1 || mode == 4) return (long)b * RS + tap;
  if (mode == 5) return (long)b * RS + (RS - 1 - tap);
  return (long)tap * d1 + b;                                   // mode 2: [(tap)*Co + co][Ci]
}

STF_DEV int pack_tiles(const stf_pack_desc& d) {
  const int bext = d.mode == 0 ? d.cpad : d.d1;
  return pack_outer(d.mode) ? ((d.d0 + PK_TA - 1) / PK_TA) * ((d.d1 + PK_TB - 1) / PK_TB)
                            : ((d.d0 + PK_IA - 1) / PK_IA) * ((bext + PK_IB - 1) / PK_IB);
}

constexpr int PK_UNR = 4;
__global__ __launch_bounds__(NT) void pack_tiled_kernel(const stf_pack_desc* __restrict__ descs) {
  __shared__ float tile[PK_TA * (PK_TB * PK_MAXRS + 1)];
  const stf_pack_desc d = descs[blockIdx.y];
  if ((int)blockIdx.x >= pack_tiles(d)) return;
  const int RS = d.R * d.S, tid = threadIdx.x;
  uint16_t* out = reinterpret_cast<uint16_t*>(d.out);
  if (pack_outer(d.mode)) {
    const int nbb = (d.d1 + PK_TB - 1) / PK_TB;
    const int a0 = (blockIdx.x / nbb) * PK_TA, b0 = (blockIdx.x % nbb) * PK_TB;
    const int na = min(PK_TA, d.d0 - a0), nb = min(PK_TB, d.d1 - b0), cols = nb * RS, LS = PK_TB * PK_MAXRS + 1;
    // whole source rows [a][b0..b0+nb)[tap]; PK_UNR independent loads in flight per thread (one
    // at a time, the loop waited on every load's latency: 1.6 TB/s)
    for (int e0 = tid; e0 < na * cols; e0 += PK_UNR * NT) {
      float v[PK_UNR];
      int at[PK_UNR];
#pragma unroll
      for (int k = 0; k < PK_UNR; ++k) {
        const int e = e0 + k * NT;
        at[k] = -1;
        if (e < na * cols) {
          const int a = e / cols, c = e - a * cols;
          v[k] = d.w[((long)(a0 + a) * d.d1 + b0) * RS + c];
          at[k] = a * LS + c;
        }
      }
#pragma unroll
      for (int k = 0; k < PK_UNR; ++k)
        if (at[k] >= 0) tile[at[k]] = v[k];
    }
    __syncthreads();
    const int qn = (na + 7) / 8;                               // 8-element chunks along a
    for (int e = tid; e < cols * qn; e += NT) {
      const int c = e / qn, q = e - c * qn, b = c / RS, tap = c - b * RS;
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (q * 8 + j < na) ? tile[(q * 8 + j) * LS + c] : 0.f;
      uint16_t* o = out + pack_outer_row(d.mode, b0 + b, tap, d.d1, RS) * d.d0 + a0 + q * 8;
      if (q * 8 + 8 <= na) *reinterpret_cast<uint4*>(o) = pack8(v);
      else
        for (int j = 0; j < na - q * 8; ++j) reinterpret_cast<e16*>(o)[j] = f2e(v[j]);
    }
  } else {
    const int bext = d.mode == 0 ? d.cpad : d.d1;              // mode 0 rows are cpad wide (zero pad)
    const int nbb = (bext + PK_IB - 1) / PK_IB;
    const int a0 = (blockIdx.x / nbb) * PK_IA, b0 = (blockIdx.x % nbb) * PK_IB;
    const int na = min(PK_IA, d.d0 - a0), nb = min(PK_IB, bext - b0), LS = PK_IB * PK_MAXRS + 1;
    const int nbs = max(0, min(nb, d.d1 - b0));                // source columns present
    for (int e0 = tid; e0 < na * nbs * RS; e0 += PK_UNR * NT) {
      float v[PK_UNR];
      int at[PK_UNR];
#pragma unroll
      for (int k = 0; k < PK_UNR; ++k) {
        const int e = e0 + k * NT;
        at[k] = -1;
        if (e < na * nbs * RS) {
          const int a = e / (nbs * RS), c = e - a * nbs * RS;
          v[k] = d.w[((long)(a0 + a) * d.d1 + b0) * RS + c];
          at[k] = a * LS + c;
        }
      }
#pragma unroll
      for (int k = 0; k < PK_UNR; ++k)
        if (at[k] >= 0) tile[at[k]] = v[k];
    }
    __syncthreads();
    const int qn = (nb + 7) / 8;
    for (int e = tid; e < na * RS * qn; e += NT) {
      const int a = e / (RS * qn), r = e - a * RS * qn, tap = r / qn, q = r - tap * qn;
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int b = q * 8 + j;
        v[j] = (b < nbs) ? tile[a * LS + b * RS + tap] : 0.f;
      }
      uint16_t* o = out + ((long)(a0 + a) * RS + tap) * bext + b0 + q * 8;
      if (q * 8 + 8 <= nb) *reinterpret_cast<uint4*>(o) = pack8(v);
      else
        for (int j = 0; j < nb - q * 8; ++j) reinterpret_cast<e16*>(o)[j] = f2e(v[j]);
    }
  }
}

__global__ void channel_sum_kernel(const uint16_t* __restrict__ x, int xcs, long M, int C,
                                   float* __restrict__ partial) {
  __shared__ float red[NT][9];
  const int CG = C / 8;
  const long gt = blockIdx.x * (long)NT + threadIdx.x;
  const int cg = (int)(gt % CG);
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (long u = gt; u < M * CG; u += (long)gridDim.x * NT) {
    const long pix = u / CG;
    float v[8];
    unpack8(*reinterpret_cast<const uint4*>(x + pix * xcs + cg * 8), v);
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] += v[j];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[threadIdx.x][j] = s[j];
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += NT) {
    const int g = c / 8, j = c - g * 8;
    float a = 0.f;
    for (int t = g; t < NT; t += CG) a += red[t][j];
    partial[(size_t)blockIdx.x * C + c] = a;
  }
}

long grid_for(long units, long cap) {
  long b = (units + NT - 1) / NT;
  return b < 1 ? 1 : (b > cap ? cap : b);
}

}  // namespace

// Graph-capturable variant: lr and the step count come from device memory (hyper[0] =
// lr, hyper[1] = step after this update's increment), so a captured training step can
// be replayed with the schedule's new lr (written between replays) and a step count
// that advances on the device.  Bias corrections in double, rounded to fp32 exactly as
// the host computes them for stf_adamw, so both paths produce the same bits.
// GradScaler (amp) variant: gradients arrive scaled by *gscale (NULL: already unscaled)
// and are multiplied by 1/*gscale in fp32 -- GradScaler.unscale_'s arithmetic, exact for
// its power-of-two scales; *finf != 0 (an inf/nan gradient) skips the whole update, like
// torch's fused AdamW under GradScaler, with no host synchronisation.
__global__ void adamw_dev_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                 float* __restrict__ v, long n, const float* __restrict__ hyper, float b1, float b2,
                                 float eps, float wd, const float* __restrict__ gscale,
                                 const float* __restrict__ finf) {
  if (finf && finf[0] != 0.f) return;
  const float inv = gscale ? 1.f / gscale[0] : 1.f;
  const float lr = hyper[0];
  const double step = hyper[1];
  const float bc1 = (float)(1.0 - pow((double)b1, step)), bc2 = (float)(1.0 - pow((double)b2, step));
  const float step_size = lr / bc1, inv_sqrt_bc2 = 1.f / sqrtf(bc2);
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < n; i += (long)gridDim.x * NT) {
    float pp = p[i] * (1.f - lr * wd);
    const float gg = gscale ? g[i] * inv : g[i];
    const float mm = m[i] + (1.f - b1) * (gg - m[i]);
    const float ww = b2 * v[i] + (1.f - b2) * gg * gg;
    pp -= step_size * mm / (sqrtf(ww) * inv_sqrt_bc2 + eps);
    p[i] = pp;
    m[i] = mm;
    v[i] = ww;
  }
}

// the device step count advances unless the update is skipped (one lane; vector stores)
__global__ void adamw_amp_step_kernel(float* __restrict__ hyper, const float* __restrict__ finf) {
  if (threadIdx.x == 0 && !(finf && finf[0] != 0.f)) hyper[1] += 1.f;
}

extern "C" int stf_adamw_dev(float* p, const float* g, float* m, float* v, int64_t n, const float* hyper, float beta1,
                             float beta2, float eps, float weight_decay, stf_stream_t stream) {
  if (n < 0 || !hyper) return STF_EINVAL;
  if (n == 0) return 0;
  hipLaunchKernelGGL(adamw_dev_kernel, dim3(grid_for(n, 4096)), dim3(NT), 0, (hipStream_t)stream, p, g, m, v, (long)n,
                     hyper, beta1, beta2, eps, weight_decay, nullptr, nullptr);
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_adamw_amp(float* p, const float* g, float* m, float* v, int64_t n, float* hyper,
                             const float* grad_scale, const float* found_inf, float beta1, float beta2, float eps,
                             float weight_decay, stf_stream_t stream) {
  if (n < 0 || !hyper || !found_inf) return STF_EINVAL;
  hipLaunchKernelGGL(adamw_amp_step_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, hyper, found_inf);
  STF_CHECK_LAUNCH();
  if (n == 0) return 0;
  hipLaunchKernelGGL(adamw_dev_kernel, dim3(grid_for(n, 4096)), dim3(NT), 0, (hipStream_t)stream, p, g, m, v, (long)n,
                     hyper, beta1, beta2, eps, weight_decay, grad_scale, found_inf);
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_adamw(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2,
                         float eps, float weight_decay, float bc1, float bc2, stf_stream_t stream) {
  if (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) return STF_EINVAL;
  const long blocks = grid_for(n / 4 + 1, 4096);
  hipLaunchKernelGGL(adamw_kernel, dim3(blocks), dim3(NT), 0, (hipStream_t)stream, p, g, m, v, (long)n, lr, beta1,
                     beta2, eps, weight_decay, lr / bc1, 1.f / sqrtf(bc2));
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_pack_input(const float* x, int N, int C, int H, int W, int Cpad, void* out, stf_stream_t stream) {
  if (Cpad % 8 || Cpad < C) return STF_EINVAL;
  const long units = (long)N * H * W * (Cpad / 8);
  if (units >= (1L << 31)) return STF_EINVAL;             // 32-bit index math in the kernel
  hipLaunchKernelGGL(pack_input_kernel, dim3(grid_for(units, 8192)), dim3(NT), 0, (hipStream_t)stream, x, N, C, H,
                     W, Cpad, (uint16_t*)out);
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_pack_weight(const float* w, int d0, int d1, int R, int S, int mode, int cpad, void* out,
                               stf_stream_t stream) {
  if (mode < 0 || mode > 5 || (mode == 0 && cpad < d1)) return STF_EINVAL;
  const long total = mode == 0 ? (long)d0 * R * S * cpad : (long)d0 * d1 * R * S;
  if (total >= (1L << 31) || (long)d0 * d1 * R * S >= (1L << 31)) return STF_EINVAL;
  hipLaunchKernelGGL(pack_weight_kernel, dim3(grid_for(total, 4096)), dim3(NT), 0, (hipStream_t)stream, w, d0, d1,
                     R, S, mode, cpad, (uint16_t*)out);
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_pack_tiles(int d0, int d1, int R, int S, int mode, int cpad) {
  // tiles of the tiled packing kernel for one descriptor, or -1 when it needs the
  // element-wise kernel (output rows not 8-aligned, RS > 9)
  const int RS = R * S;
  if (RS > PK_MAXRS || mode < 0 || mode > 5) return -1;
  const bool outer = mode == 1 || mode == 5 || mode == 2 || mode == 4;
  const int bext = mode == 0 ? cpad : d1;
  if (outer ? (d0 % 8) : (bext % 8)) return -1;
  return outer ? ((d0 + PK_TA - 1) / PK_TA) * ((d1 + PK_TB - 1) / PK_TB)
               : ((d0 + PK_IA - 1) / PK_IA) * ((bext + PK_IB - 1) / PK_IB);
}

extern "C" int stf_pack_weights_tiled(const stf_pack_desc* descs, int count, int max_tiles, stf_stream_t stream) {
  if (count <= 0) return 0;
  if (max_tiles <= 0 || count > 65535) return STF_EINVAL;
  hipLaunchKernelGGL(pack_tiled_kernel, dim3((unsigned)max_tiles, count), dim3(NT), 0, (hipStream_t)stream, descs);
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_pack_weights(const stf_pack_desc* descs, int count, int64_t max_elems, stf_stream_t stream) {
  if (count <= 0) return 0;
  if (count > 65535 || max_elems <= 0 || max_elems >= (1L << 31)) return STF_EINVAL;
  hipLaunchKernelGGL(pack_weights_kernel, dim3(grid_for(max_elems, 1024), count), dim3(NT), 0, (hipStream_t)stream,
                     descs);
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_channel_sum(const void* x, int x_cstride, int M, int C, float* partial, float* out,
                               stf_stream_t stream) {
  if (C % 8 || NT % (C / 8) || x_cstride % 8) return STF_EINVAL;
  const long tiles = grid_for((long)M * (C / 8), 1024);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(channel_sum_kernel, dim3(tiles), dim3(NT), 0, s, (const uint16_t*)x, x_cstride, (long)M, C,
                     partial);
  STF_CHECK_LAUNCH();
  const int S = stf::colsum_stage1(partial, tiles, C, s, 1, stf::FOLD16_ROWS);
  hipLaunchKernelGGL(stf_tile_sum_kernel, dim3((C + 15) / 16), dim3(stf::FOLD_NT), 0, s, partial, S, C, out);
  STF_CHECK_LAUNCH();
  return 0;
}

// out[c] = sum over the T rows of the statistics layout [T][2][Nout] of column c0 + c of the
// "sum" half (fixed order, as stf_tile_sum_kernel)
__global__ __launch_bounds__(stf::FOLD_NT) void stat_sums_kernel(const float* __restrict__ stats, int tiles, int Nout,
                                                                 int c0, int C, float* __restrict__ out) {
  __shared__ double red[stf::FOLD_NT];
  const int c = blockIdx.x * 16 + (threadIdx.x & 15);
  const bool cok = c < C;
  const double v = stf::fold16_finish(stf::fold16_partial(stats + c0, tiles, 2L * Nout, c, cok), red);
  if (cok && (threadIdx.x >> 4) == 0) out[c] = (float)v;
}

extern "C" int stf_stat_sums(const float* stats, int tiles, int Nout, int c0, int C, float* out,
                             stf_stream_t stream) {
  if (!stats || !out || tiles < 1 || C < 1 || c0 < 0 || c0 + C > Nout) return STF_EINVAL;
  hipLaunchKernelGGL(stat_sums_kernel, dim3((C + 15) / 16), dim3(stf::FOLD_NT), 0, (hipStream_t)stream, stats, tiles,
                     Nout, c0, C, out);
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" const char* stf_error_string(int code) {
  if (code == STF_EINVAL) return "stfunet: invalid argument (shape/alignment constraint violated)";
  return hipGetErrorString((hipError_t)code);
}

extern "C" int stf_abi_version(void) { return 17; }

extern "C" int stf_storage_type(void) {
#ifdef STF_FP16
  return STF_STORAGE_FP16;
#else
  return STF_STORAGE_BF16;
#endif
}
