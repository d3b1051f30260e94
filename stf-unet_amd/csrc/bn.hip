// Training-mode BatchNorm2d (+ReLU, +2x2 max pool) for NHWC bf16 activations.
//
// Forward: the producing conv's epilogue already wrote per-tile (sum, sum^2);
// stf_bn_finalize folds them (fp64) into mean/invstd, the affine (scale, shift)
// and the running-stat update; stf_bn_act applies y*scale+shift (+ReLU) while
// writing into a channel slice of the concat buffer and, optionally, the 2x2
// max-pooled tensor for the next encoder level -- one read of y, no separate
// pool or cat pass.
//
// Backward (per channel, M = N*H*W, xhat = (y-mean)*invstd, g = dL/d(BN out)):
//   dgamma = sum g*xhat, dbeta = sum g,
//   dy = gamma*invstd*(g - dbeta/M - xhat*dgamma/M) = A*g + B*y + C.
// stf_bn_bwd_reduce forms g (ReLU mask and max-pool routing recomputed from y,
// first maximum of each window in row-major order like torch's CPU kernel)
// and the two sums; stf_bn_bwd_apply evaluates the affine form in place.
#include "common.h"
#include "../../include/stfunet.h"
#include "reduce.h"

namespace {

constexpr int NT = 256;

STF_DEV void load_affine(const float* p, int c, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p + c);
  const float4 b = *reinterpret_cast<const float4*>(p + c + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

int tiles_for(long units) {
  long t = (units + NT - 1) / NT;
  return (int)(t < 1 ? 1 : (t > 1024 ? 1024 : t));
}

// ------------------------------------------------------------------ finalize
__global__ void bn_finalize_kernel(const float* __restrict__ stats, int tiles, int C, int M,
                                   const float* gamma, const float* beta, float mom, float eps,
                                   float* rm, float* rv, float* mean, float* invstd, float* scale,
                                   float* shift) {
  __shared__ double red[2][4][64];
  const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  double s1 = 0.0, s2 = 0.0;
  if (c < C && stats)
    for (int t = grp; t < tiles; t += 4) {
      s1 += stats[(size_t)t * 2 * C + c];
      s2 += stats[(size_t)t * 2 * C + C + c];
    }
  red[0][grp][cl] = s1;
  red[1][grp][cl] = s2;
  __syncthreads();
  if (grp != 0 || c >= C) return;
  double mu, var;
  if (!stats) {                       // eval mode: normalise with the running statistics
    mu = rm[c];
    var = rv[c];
  } else {
    for (int g = 1; g < 4; ++g) { s1 += red[0][g][cl]; s2 += red[1][g][cl]; }
    mu = s1 / M;
    var = s2 / M - mu * mu;
    if (var < 0) var = 0;
  }
  const float inv = (float)(1.0 / sqrt(var + (double)eps));
  const float sc = gamma[c] * inv;
  mean[c] = (float)mu;
  invstd[c] = inv;
  scale[c] = sc;
  shift[c] = beta[c] - (float)mu * sc;
  if (rm && stats) {
    rm[c] = (1.f - mom) * rm[c] + mom * (float)mu;
    const double unb = M > 1 ? var * M / (M - 1) : var;
    rv[c] = (1.f - mom) * rv[c] + mom * (float)unb;
  }
}

// ------------------------------------------------------------------ apply (+ pool)
template <bool POOL>
__global__ void bn_act_kernel(const uint16_t* __restrict__ y, int ycs, int N, int H, int W, int C,
                              const float* __restrict__ scale, const float* __restrict__ shift, int relu,
                              uint16_t* __restrict__ out, int ocs, uint16_t* __restrict__ pooled) {
  const int CG = C / 8;
  const long units = POOL ? (long)N * (H / 2) * (W / 2) * CG : (long)N * H * W * CG;
  for (long u = blockIdx.x * (long)NT + threadIdx.x; u < units; u += (long)gridDim.x * NT) {
    const int cg = (int)(u % CG);
    const long pix = u / CG;
    float sc[8], sh[8];
    load_affine(scale, cg * 8, sc);
    load_affine(shift, cg * 8, sh);
    if (!POOL) {
      float v[8];
      unpack8(*reinterpret_cast<const uint4*>(y + pix * ycs + cg * 8), v);
#pragma unroll
      for (int j = 0; j < 8; ++j) { v[j] = v[j] * sc[j] + sh[j]; if (relu) v[j] = fmaxf(v[j], 0.f); }
      *reinterpret_cast<uint4*>(out + pix * ocs + cg * 8) = pack8(v);
    } else {
      const int Wp = W / 2, Hp = H / 2;
      const int n = (int)(pix / ((long)Hp * Wp));
      const int rem = (int)(pix - (long)n * Hp * Wp);
      const int py = rem / Wp, px = rem - py * Wp;
      float mx[8];
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const long p = ((long)n * H + 2 * py + (d >> 1)) * W + 2 * px + (d & 1);
        float v[8];
        unpack8(*reinterpret_cast<const uint4*>(y + p * ycs + cg * 8), v);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          v[j] = v[j] * sc[j] + sh[j];
          if (relu) v[j] = fmaxf(v[j], 0.f);
          v[j] = round_bf(v[j]);
          mx[j] = d == 0 ? v[j] : fmaxf(mx[j], v[j]);
        }
        *reinterpret_cast<uint4*>(out + p * ocs + cg * 8) = pack8(v);
      }
      *reinterpret_cast<uint4*>(pooled + pix * C + cg * 8) = pack8(mx);
    }
  }
}

// ------------------------------------------------------------------ backward reduce
template <bool POOL>
__global__ void bn_bwd_reduce_kernel(const uint16_t* __restrict__ dz, int dzcs, const uint16_t* __restrict__ dpool,
                                     const uint16_t* __restrict__ y, int ycs, int N, int H, int W, int C,
                                     const float* __restrict__ scale, const float* __restrict__ shift,
                                     const float* __restrict__ mean, const float* __restrict__ invstd, int relu,
                                     uint16_t* __restrict__ g_out, float* __restrict__ partial) {
  __shared__ float red[NT][17];
  const int CG = C / 8;
  const long units = POOL ? (long)N * (H / 2) * (W / 2) * CG : (long)N * H * W * CG;
  const long gt = blockIdx.x * (long)NT + threadIdx.x;
  const int cg = (int)(gt % CG);                 // constant: total threads is a multiple of CG
  float sc[8], sh[8], mu[8], is[8];
  load_affine(scale, cg * 8, sc);
  load_affine(shift, cg * 8, sh);
  load_affine(mean, cg * 8, mu);
  load_affine(invstd, cg * 8, is);
  float sg[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sgx[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (long u = gt; u < units; u += (long)gridDim.x * NT) {
    const long pix = u / CG;
    if (!POOL) {
      float v[8], d[8];
      unpack8(*reinterpret_cast<const uint4*>(y + pix * ycs + cg * 8), v);
      unpack8(*reinterpret_cast<const uint4*>(dz + pix * dzcs + cg * 8), d);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float z = v[j] * sc[j] + sh[j];
        const float gj = (relu && !(z > 0.f)) ? 0.f : d[j];
        d[j] = gj;
        sg[j] += gj;
        sgx[j] += gj * (v[j] - mu[j]) * is[j];
      }
      *reinterpret_cast<uint4*>(g_out + pix * C + cg * 8) = pack8(d);
    } else {
      const int Wp = W / 2, Hp = H / 2;
      const int n = (int)(pix / ((long)Hp * Wp));
      const int rem = (int)(pix - (long)n * Hp * Wp);
      const int py = rem / Wp, px = rem - py * Wp;
      float v[4][8], a[4][8];
      long p[4];
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        p[d] = ((long)n * H + 2 * py + (d >> 1)) * W + 2 * px + (d & 1);
        unpack8(*reinterpret_cast<const uint4*>(y + p[d] * ycs + cg * 8), v[d]);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float t = v[d][j] * sc[j] + sh[j];
          if (relu) t = fmaxf(t, 0.f);
          a[d][j] = round_bf(t);
        }
      }
      float dp[8];
      unpack8(*reinterpret_cast<const uint4*>(dpool + pix * C + cg * 8), dp);
      int am[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        am[j] = 0;
        float best = a[0][j];
#pragma unroll
        for (int d = 1; d < 4; ++d) if (a[d][j] > best) { best = a[d][j]; am[j] = d; }
      }
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        float gd[8];
        if (dz) unpack8(*reinterpret_cast<const uint4*>(dz + p[d] * dzcs + cg * 8), gd);
        else {
#pragma unroll
          for (int j = 0; j < 8; ++j) gd[j] = 0.f;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float t = gd[j] + (am[j] == d ? dp[j] : 0.f);
          const float z = v[d][j] * sc[j] + sh[j];
          if (relu && !(z > 0.f)) t = 0.f;
          gd[j] = t;
          sg[j] += t;
          sgx[j] += t * (v[d][j] - mu[j]) * is[j];
        }
        *reinterpret_cast<uint4*>(g_out + p[d] * C + cg * 8) = pack8(gd);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) { red[threadIdx.x][j] = sg[j]; red[threadIdx.x][8 + j] = sgx[j]; }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += NT) {
    const int g = c / 8, j = c - g * 8;
    float a = 0.f, b = 0.f;
    for (int t = g; t < NT; t += CG) { a += red[t][j]; b += red[t][8 + j]; }
    partial[(size_t)blockIdx.x * 2 * C + c] = a;
    partial[(size_t)blockIdx.x * 2 * C + C + c] = b;
  }
}

__global__ void bn_bwd_finalize_kernel(const float* __restrict__ partial, int tiles, int C, int M,
                                       const float* gamma, const float* mean, const float* invstd,
                                       float* dgamma, float* dbeta, float* coef) {
  __shared__ double red[2][4][64];
  const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  double s1 = 0.0, s2 = 0.0;
  if (c < C)
    for (int t = grp; t < tiles; t += 4) {
      s1 += partial[(size_t)t * 2 * C + c];
      s2 += partial[(size_t)t * 2 * C + C + c];
    }
  red[0][grp][cl] = s1;
  red[1][grp][cl] = s2;
  __syncthreads();
  if (grp != 0 || c >= C) return;
  for (int g = 1; g < 4; ++g) { s1 += red[0][g][cl]; s2 += red[1][g][cl]; }
  if (dgamma) dgamma[c] = (float)s2;
  if (dbeta) dbeta[c] = (float)s1;
  const double A = (double)gamma[c] * invstd[c];
  const double B = -A * invstd[c] * s2 / M;
  const double Cc = -A * s1 / M + A * invstd[c] * mean[c] * s2 / M;
  coef[c] = (float)A;
  coef[C + c] = (float)B;
  coef[2 * C + c] = (float)Cc;
}

__global__ void bn_bwd_apply_kernel(const uint16_t* g, const uint16_t* __restrict__ y, int ycs,
                                    long M, int C, const float* __restrict__ coef, uint16_t* dy,
                                    float* __restrict__ bias_partial) {
  __shared__ float red[NT][9];
  const int CG = C / 8;
  const long units = M * CG;
  const long gt = blockIdx.x * (long)NT + threadIdx.x;
  const int cg = (int)(gt % CG);
  float A[8], B[8], Cc[8], sb[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  load_affine(coef, cg * 8, A);
  load_affine(coef + C, cg * 8, B);
  load_affine(coef + 2 * C, cg * 8, Cc);
  for (long u = gt; u < units; u += (long)gridDim.x * NT) {
    const long pix = u / CG;
    float gv[8], yv[8];
    unpack8(*reinterpret_cast<const uint4*>(g + pix * C + cg * 8), gv);
    unpack8(*reinterpret_cast<const uint4*>(y + pix * ycs + cg * 8), yv);
#pragma unroll
    for (int j = 0; j < 8; ++j) { gv[j] = A[j] * gv[j] + B[j] * yv[j] + Cc[j]; sb[j] += gv[j]; }
    *reinterpret_cast<uint4*>(dy + pix * C + cg * 8) = pack8(gv);
  }
  if (!bias_partial) return;
#pragma unroll
  for (int j = 0; j < 8; ++j) red[threadIdx.x][j] = sb[j];
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += NT) {
    const int gg = c / 8, j = c - gg * 8;
    float a = 0.f;
    for (int t = gg; t < NT; t += CG) a += red[t][j];
    bias_partial[(size_t)blockIdx.x * C + c] = a;
  }
}

}  // namespace

// sum over tiles of partial[t][C] -> out[C] (fixed order); shared with misc.hip
__global__ void stf_tile_sum_kernel(const float* __restrict__ partial, int tiles, int C, float* __restrict__ out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s = 0.0;
  for (int t = 0; t < tiles; ++t) s += partial[(size_t)t * C + c];
  out[c] = (float)s;
}

static bool cg_ok(int C) { return C % 8 == 0 && NT % (C / 8) == 0; }

extern "C" int stf_bn_finalize(float* stats, int tiles, int C, int M, const float* gamma, const float* beta,
                               float momentum, float eps, float* running_mean, float* running_var, float* mean,
                               float* invstd, float* scale, float* shift, stf_stream_t stream) {
  if (stats) tiles = stf::colsum_stage1(stats, tiles, 2L * C, (hipStream_t)stream);
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 63) / 64), dim3(256), 0, (hipStream_t)stream, stats, tiles,
                     C, M, gamma, beta, momentum, eps, running_mean, running_var, mean, invstd, scale, shift);
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_bn_act(const void* y, int y_cstride, int N, int H, int W, int C, const float* scale,
                          const float* shift, int relu, void* out, int out_cstride, void* pooled,
                          stf_stream_t stream) {
  if (C % 8 || y_cstride % 8 || out_cstride % 8 || (pooled && ((H | W) & 1))) return STF_EINVAL;
  const long units = pooled ? (long)N * (H / 2) * (W / 2) * (C / 8) : (long)N * H * W * (C / 8);
  long blocks = (units + NT - 1) / NT;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (pooled)
    hipLaunchKernelGGL(bn_act_kernel<true>, dim3(blocks), dim3(NT), 0, s, (const uint16_t*)y, y_cstride, N, H, W,
                       C, scale, shift, relu, (uint16_t*)out, out_cstride, (uint16_t*)pooled);
  else
    hipLaunchKernelGGL(bn_act_kernel<false>, dim3(blocks), dim3(NT), 0, s, (const uint16_t*)y, y_cstride, N, H,
                       W, C, scale, shift, relu, (uint16_t*)out, out_cstride, (uint16_t*)nullptr);
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_bn_bwd_tiles(int N, int H, int W, int C, int pooled) {
  const long units = pooled ? (long)N * (H / 2) * (W / 2) * (C / 8) : (long)N * H * W * (C / 8);
  return tiles_for(units);
}

extern "C" int stf_bn_bwd_reduce(const void* dz, int dz_cstride, const void* dpool, const void* y, int y_cstride,
                                 int N, int H, int W, int C, const float* scale, const float* shift,
                                 const float* mean, const float* invstd, int relu, void* g_out, float* partial,
                                 stf_stream_t stream) {
  if (!cg_ok(C) || y_cstride % 8 || (dz && dz_cstride % 8)) return STF_EINVAL;
  if (!dz && !dpool) return STF_EINVAL;
  if (dpool && ((H | W) & 1)) return STF_EINVAL;
  const int tiles = stf_bn_bwd_tiles(N, H, W, C, dpool != nullptr);
  hipStream_t s = (hipStream_t)stream;
  if (dpool)
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<true>, dim3(tiles), dim3(NT), 0, s, (const uint16_t*)dz, dz_cstride,
                       (const uint16_t*)dpool, (const uint16_t*)y, y_cstride, N, H, W, C, scale, shift, mean,
                       invstd, relu, (uint16_t*)g_out, partial);
  else
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<false>, dim3(tiles), dim3(NT), 0, s, (const uint16_t*)dz, dz_cstride,
                       (const uint16_t*)nullptr, (const uint16_t*)y, y_cstride, N, H, W, C, scale, shift, mean,
                       invstd, relu, (uint16_t*)g_out, partial);
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_bn_bwd_finalize(float* partial, int tiles, int C, int M, const float* gamma,
                                   const float* mean, const float* invstd, float* dgamma, float* dbeta, float* coef,
                                   stf_stream_t stream) {
  tiles = stf::colsum_stage1(partial, tiles, 2L * C, (hipStream_t)stream);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 63) / 64), dim3(256), 0, (hipStream_t)stream, partial,
                     tiles, C, M, gamma, mean, invstd, dgamma, dbeta, coef);
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_bn_bwd_apply(const void* g, const void* y, int y_cstride, int M, int C, const float* coef,
                                void* dy, float* bias_partial, float* dbias, stf_stream_t stream) {
  if (!cg_ok(C) || y_cstride % 8) return STF_EINVAL;
  const int tiles = tiles_for((long)M * (C / 8));
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(tiles), dim3(NT), 0, s, (const uint16_t*)g, (const uint16_t*)y,
                     y_cstride, (long)M, C, coef, (uint16_t*)dy, bias_partial);
  STF_CHECK_LAUNCH();
  if (bias_partial && dbias) {
    const int S = stf::colsum_stage1(bias_partial, tiles, C, s);
    hipLaunchKernelGGL(stf_tile_sum_kernel, dim3((C + 255) / 256), dim3(256), 0, s, bias_partial, S, C, dbias);
    STF_CHECK_LAUNCH();
  }
  return 0;
}
