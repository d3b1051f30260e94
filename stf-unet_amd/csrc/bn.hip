// Training-mode BatchNorm2d (+ReLU, +residual add, +2x2 max pool) for NHWC bf16
// activations, with optional statistic *groups* along the image axis.
//
// Groups: the STF encoder runs all T time steps as one batch of T*B images
// (t-major), but the reference normalises every time step with its own batch
// statistics and advances the running statistics once per step
// (src/stf_lstm_unet.py:168-186).  Group g = images [g*N/G, (g+1)*N/G) keeps its
// own mean/invstd/scale/shift; running stats are updated group by group in t
// order, exactly like T sequential BatchNorm calls.  UNet uses G = 1.
//
// Forward: the producing conv's epilogue wrote per-tile (sum, sum^2) for tiles
// aligned to groups ([G][tpg][2][C]); stf_bn_finalize folds them (fp64) and
// stf_bn_act applies  out = act(y*scale+shift [+ residual])  where the residual
// is another bf16 tensor (identity shortcut) or a second BN of a raw conv output
// (downsample shortcut: ResNet BasicBlock, ResidualConvBlock), optionally also
// writing the 2x2 max-pooled tensor (UNet Down, src/unet.py:25).
//
// Backward (per group and channel, xhat = (y-mean)*invstd):
//   g = dz [+ maxpool routing of dpool] masked by the ReLU (recomputed from y,
//       or read from the saved output when the ReLU followed a residual add),
//   dgamma = sum g*xhat, dbeta = sum g,  dy = A*g + B*y + C  (fp64 coefficients).
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

int tiles_per_group(long units_per_group, int groups) {
  long t = (units_per_group + NT - 1) / NT;
  const long cap = (1024 + groups - 1) / groups;    // <= FOLD16_ROWS partial rows per group
  if (t > cap) t = cap;
  if (t < 1) t = 1;
  return (int)t;
}

// ------------------------------------------------------------------ finalize
// stats: [G][T][2][C] with the first S rows of every group folded.  Grid =
// (channel chunks of 16) x G; block = 16 channels x 16 row-lanes folding ONE
// group.  With G > 1 the running statistics must see the G updates in order:
// each block parks (mean, biased var) in row 0 of its group (scratch) and
// bn_running_kernel applies them sequentially.
// the training-mode finalize of channel c of group g from its folded (sum, sum of squares)
STF_DEV void bn_fin_fwd_out(float* base, int g, int c, int G, int C, long Mg, double s1, double s2,
                            const float* gamma, const float* beta, float mom, float eps, float* rm, float* rv,
                            float* mean, float* invstd, float* scale, float* shift) {
  const double mu = s1 / Mg;
  double var = s2 / Mg - mu * mu;
  if (var < 0) var = 0;
  const float inv = (float)(1.0 / sqrt(var + (double)eps));
  const float sc = gamma[c] * inv;
  mean[g * C + c] = (float)mu;
  invstd[g * C + c] = inv;
  scale[g * C + c] = sc;
  shift[g * C + c] = beta[c] - (float)mu * sc;
  if (G == 1) {
    if (!rm) return;
    const double unb = Mg > 1 ? var * Mg / (Mg - 1) : var;
    rm[c] = (1.f - mom) * rm[c] + mom * (float)mu;
    rv[c] = (1.f - mom) * rv[c] + mom * (float)unb;
  } else {                               // parked for bn_running_kernel / stf_bn_running_batch
    base[c] = (float)mu;
    base[C + c] = (float)var;
  }
}

__global__ __launch_bounds__(stf::FOLD_NT) void bn_finalize_kernel(float* __restrict__ stats, int S, int T, int G, int C,
                                                        long Mg, const float* gamma, const float* beta, float mom,
                                                        float eps, float* rm, float* rv, float* mean, float* invstd,
                                                        float* scale, float* shift) {
  __shared__ double red[stf::FOLD_NT];
  const int g = blockIdx.y;
  const int c = blockIdx.x * 16 + (threadIdx.x & 15);
  const bool cok = c < C, lead = cok && (threadIdx.x >> 4) == 0;
  if (stats) {
    float* base = stats + (size_t)g * T * 2 * C;
    double s1, s2;
    stf::fold16_pair(base, S, 2L * C, C, c, cok, red, s1, s2);
    if (lead)
      bn_fin_fwd_out(base, g, c, G, C, Mg, s1, s2, gamma, beta, mom, eps, rm, rv, mean, invstd, scale, shift);
    return;
  }
  if (!lead) return;                     // eval mode: running statistics, no update
  const double mu = rm ? rm[c] : 0.f, var = rv ? rv[c] : 1.f;
  const float inv = (float)(1.0 / sqrt(var + (double)eps));
  const float sc = gamma[c] * inv;
  mean[g * C + c] = (float)mu;
  invstd[g * C + c] = inv;
  scale[g * C + c] = sc;
  shift[g * C + c] = beta[c] - (float)mu * sc;
}

__global__ void bn_running_kernel(const float* __restrict__ stats, int T, int G, int C, long Mg, float mom,
                                  float* rm, float* rv) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float run_m = rm[c], run_v = rv[c];
  for (int g = 0; g < G; ++g) {
    const float* base = stats + (size_t)g * T * 2 * C;
    const double var = base[C + c];
    const double unb = Mg > 1 ? var * Mg / (Mg - 1) : var;
    run_m = (1.f - mom) * run_m + mom * base[c];
    run_v = (1.f - mom) * run_v + mom * (float)unb;
  }
  rm[c] = run_m;
  rv[c] = run_v;
}

// dy = A g + B y + C coefficients of channel c of group g from its folded (sum g, sum g*xhat)
STF_DEV void bn_fin_bwd_out(float* base, int g, int c, int G, int C, long Mg, double s1, double s2,
                            const float* gamma, const float* mean, const float* invstd, float* dgamma, float* dbeta,
                            float* coef) {
  const double is = invstd[g * C + c];
  const double A = (double)gamma[c] * is;
  const double B = -A * is * s2 / Mg;
  const double Cc = -A * s1 / Mg + A * is * mean[g * C + c] * s2 / Mg;
  coef[(size_t)g * 3 * C + c] = (float)A;
  coef[(size_t)g * 3 * C + C + c] = (float)B;
  coef[(size_t)g * 3 * C + 2 * C + c] = (float)Cc;
  if (G == 1) {
    if (dgamma) dgamma[c] = (float)s2;
    if (dbeta) dbeta[c] = (float)s1;
  } else {
    base[c] = (float)s1;
    base[C + c] = (float)s2;
  }
}

// ------------------------------------------------------------------ apply
// res_mode 0: none, 1: + res tensor, 2: + (res*rscale[g] + rshift[g])
template <bool POOL>
__global__ void bn_act_kernel(const uint16_t* __restrict__ y, int ycs, long N, int H, int W, int C, long Mg,
                              const float* scale, const float* shift, int relu, int res_mode,
                              const uint16_t* __restrict__ res, int rcs, const float* __restrict__ rscale,
                              const float* __restrict__ rshift, uint16_t* __restrict__ out, int ocs,
                              uint16_t* __restrict__ pooled) {
  const int CG = C / 8;
  const long units = POOL ? N * (H / 2) * (W / 2) * CG : N * H * W * CG;
  for (long u = blockIdx.x * (long)NT + threadIdx.x; u < units; u += (long)gridDim.x * NT) {
    const int cg = (int)(u % CG);
    const long pix = u / CG;
    if (!POOL) {
      const int g = (int)(pix / Mg);
      float sc[8], sh[8], v[8];
      load_affine(scale + (size_t)g * C, cg * 8, sc);
      load_affine(shift + (size_t)g * C, cg * 8, sh);
      unpack8(*reinterpret_cast<const uint4*>(y + pix * ycs + cg * 8), v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = v[j] * sc[j] + sh[j];
      if (res_mode) {
        float r[8];
        unpack8(*reinterpret_cast<const uint4*>(res + pix * rcs + cg * 8), r);
        if (res_mode == 2) {
          float rs[8], rh[8];
          load_affine(rscale + (size_t)g * C, cg * 8, rs);
          load_affine(rshift + (size_t)g * C, cg * 8, rh);
#pragma unroll
          for (int j = 0; j < 8; ++j) r[j] = r[j] * rs[j] + rh[j];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += r[j];
      }
      if (relu) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = fmaxf(v[j], 0.f);
      }
      *reinterpret_cast<uint4*>(out + pix * ocs + cg * 8) = pack8(v);
    } else {
      const int Wp = W / 2, Hp = H / 2;
      const long n = pix / ((long)Hp * Wp);
      const int rem = (int)(pix - n * Hp * Wp);
      const int py = rem / Wp, px = rem - py * Wp;
      const int g = (int)(n * H * W / Mg);
      float sc[8], sh[8], mx[8];
      load_affine(scale + (size_t)g * C, cg * 8, sc);
      load_affine(shift + (size_t)g * C, cg * 8, sh);
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const long p = (n * H + 2 * py + (d >> 1)) * W + 2 * px + (d & 1);
        float v[8];
        unpack8(*reinterpret_cast<const uint4*>(y + p * ycs + cg * 8), v);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          v[j] = v[j] * sc[j] + sh[j];
          if (relu) v[j] = fmaxf(v[j], 0.f);
          v[j] = round_e(v[j]);
          mx[j] = d == 0 ? v[j] : fmaxf(mx[j], v[j]);
        }
        *reinterpret_cast<uint4*>(out + p * ocs + cg * 8) = pack8(v);
      }
      *reinterpret_cast<uint4*>(pooled + pix * C + cg * 8) = pack8(mx);
    }
  }
}

// ------------------------------------------------------------------ backward reduce
// mask_mode 0: none, 1: relu(y*scale+shift) > 0, 2: mask_src > 0
template <bool POOL>
__global__ void bn_bwd_reduce_kernel(const uint16_t* __restrict__ dz, int dzcs, const uint16_t* __restrict__ dpool,
                                     const uint16_t* __restrict__ y, int ycs, long N, int H, int W, int C, int G,
                                     int tpg, const float* __restrict__ scale, const float* __restrict__ shift,
                                     const float* __restrict__ mean, const float* __restrict__ invstd,
                                     int mask_mode, const uint16_t* __restrict__ msrc, int mcs,
                                     uint16_t* __restrict__ g_out, float* __restrict__ partial) {
  __shared__ float red[NT][17];
  const int CG = C / 8;
  const int g = blockIdx.x / tpg, tile = blockIdx.x - g * tpg;
  const long Ng = N / G;
  const long ppg = POOL ? Ng * (H / 2) * (W / 2) : Ng * H * W;            // pixels (or windows) per group
  const long upg = ppg * CG;
  const long gt = (long)tile * NT + threadIdx.x;
  const int cg = (int)(gt % CG);                 // constant: tpg*NT is a multiple of CG
  float sc[8], sh[8], mu[8], is[8];
  load_affine(scale + (size_t)g * C, cg * 8, sc);
  load_affine(shift + (size_t)g * C, cg * 8, sh);
  load_affine(mean + (size_t)g * C, cg * 8, mu);
  load_affine(invstd + (size_t)g * C, cg * 8, is);
  float sg[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sgx[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (long u = gt; u < upg; u += (long)tpg * NT) {
    const long pix = u / CG + g * ppg;
    if (!POOL) {
      float v[8], d[8];
      unpack8(*reinterpret_cast<const uint4*>(y + pix * ycs + cg * 8), v);
      unpack8(*reinterpret_cast<const uint4*>(dz + pix * dzcs + cg * 8), d);
      float mk[8];
      if (mask_mode == 2) unpack8(*reinterpret_cast<const uint4*>(msrc + pix * mcs + cg * 8), mk);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        bool keep = true;
        if (mask_mode == 1) keep = v[j] * sc[j] + sh[j] > 0.f;
        else if (mask_mode == 2) keep = mk[j] > 0.f;
        const float gj = keep ? d[j] : 0.f;
        d[j] = gj;
        sg[j] += gj;
        sgx[j] += gj * (v[j] - mu[j]) * is[j];
      }
      if (g_out) *reinterpret_cast<uint4*>(g_out + pix * C + cg * 8) = pack8(d);
    } else {
      const int Wp = W / 2, Hp = H / 2;
      const long n = pix / ((long)Hp * Wp);
      const int rem = (int)(pix - n * Hp * Wp);
      const int py = rem / Wp, px = rem - py * Wp;
      float v[4][8], a[4][8];
      long p[4];
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        p[d] = (n * H + 2 * py + (d >> 1)) * W + 2 * px + (d & 1);
        unpack8(*reinterpret_cast<const uint4*>(y + p[d] * ycs + cg * 8), v[d]);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float t = v[d][j] * sc[j] + sh[j];
          if (mask_mode == 1) t = fmaxf(t, 0.f);
          a[d][j] = round_e(t);
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
          if (mask_mode == 1 && !(v[d][j] * sc[j] + sh[j] > 0.f)) t = 0.f;
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
    const int gg = c / 8, j = c - gg * 8;
    float a = 0.f, b = 0.f;
    for (int t = gg; t < NT; t += CG) { a += red[t][j]; b += red[t][8 + j]; }
    partial[(size_t)blockIdx.x * 2 * C + c] = a;
    partial[(size_t)blockIdx.x * 2 * C + C + c] = b;
  }
}

// The pooled reduce with one lane per PIXEL (the 4 pixels of a 2x2 window in the 4
// lanes of a DPP quad, 8 channels each): the window's first maximum of relu(BN(y))
// (bf16-rounded, as the forward stored it) comes from two quad_perm DPP moves, so a
// lane holds 3 loads and a few dozen registers instead of a whole window (13 loads,
// ~150 registers: occupancy/latency bound at 3.4 TB/s).  Unit u: window pixel d =
// u & 3, channel chunk (u >> 2) % CG, window (u >> 2) / CG.  Needs 64 % (C / 8) == 0
// (the grid stride then keeps a thread's d and chunk fixed).
STF_DEV float quad_xor1(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));   // [1,0,3,2]
}
STF_DEV float quad_xor2(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));   // [2,3,0,1]
}

constexpr int PNT = 512;                      // 2x the waves of the other BN kernels: more loads in flight
__global__ __launch_bounds__(PNT) void bn_bwd_reduce_pool_kernel(const uint16_t* __restrict__ dz, int dzcs,
                                          const uint16_t* __restrict__ dpool, const uint16_t* __restrict__ y,
                                          int ycs, long N, int H, int W, int C, int G, int tpg,
                                          const float* __restrict__ scale, const float* __restrict__ shift,
                                          const float* __restrict__ mean, const float* __restrict__ invstd,
                                          int mask_mode, uint16_t* __restrict__ g_out,
                                          float* __restrict__ partial) {
  __shared__ float red[PNT][17];
  const int CG = C / 8;
  const int g = blockIdx.x / tpg, tile = blockIdx.x - g * tpg;
  const int Wp = W / 2, Hp = H / 2;
  const long wpg = (N / G) * Hp * Wp;                       // windows per group
  const long U = wpg * CG * 4;
  const long gt = (long)tile * PNT + threadIdx.x;
  const int d = (int)(gt & 3);
  const int cg = (int)((gt >> 2) % CG);
  float sc[8], sh[8], mu[8], is[8];
  load_affine(scale + (size_t)g * C, cg * 8, sc);
  load_affine(shift + (size_t)g * C, cg * 8, sh);
  load_affine(mean + (size_t)g * C, cg * 8, mu);
  load_affine(invstd + (size_t)g * C, cg * 8, is);
  const bool relu = mask_mode == 1;
  float sg[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sgx[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  // 32-bit index math (a 64-bit division is a long emulated sequence per unit): every
  // tensor here has < 2^31 windows and pixels (checked by the host)
  const int HpWp = Hp * Wp, cshift = __builtin_ctz(CG);   // CG is a power of two (64 % CG == 0)
  // two units per iteration, all six loads issued before either is used (more bytes in
  // flight per lane); the pair test is quad-uniform (U and the stride are multiples of 4)
  const long S = (long)tpg * PNT;
  auto pix = [&](long u, int& win) {
    win = (int)(u >> (2 + cshift)) + (int)(g * wpg);
    const int n = win / HpWp;
    const int rem = win - n * HpWp;
    const int py = rem / Wp, px = rem - py * Wp;
    return ((long)(n * H + 2 * py + (d >> 1))) * W + 2 * px + (d & 1);
  };
  auto unit = [&](long p, int win, const uint4& yv, const uint4& zv, const uint4& pv) {
    float v[8], gd[8], dp[8];
    unpack8(yv, v);
    if (dz) unpack8(zv, gd);
    else {
#pragma unroll
      for (int j = 0; j < 8; ++j) gd[j] = 0.f;
    }
    unpack8(pv, dp);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float t = v[j] * sc[j] + sh[j];
      const float a = round_e(relu ? fmaxf(t, 0.f) : t);
      float m = fmaxf(a, quad_xor1(a));
      m = fmaxf(m, quad_xor2(m));
      float c = a == m ? (float)d : 4.f;                       // first maximum of the window
      c = fminf(c, quad_xor1(c));
      c = fminf(c, quad_xor2(c));
      float gj = gd[j] + (c == (float)d ? dp[j] : 0.f);
      if (relu && !(t > 0.f)) gj = 0.f;
      gd[j] = gj;
      sg[j] += gj;
      sgx[j] += gj * (v[j] - mu[j]) * is[j];
    }
    *reinterpret_cast<uint4*>(g_out + p * C + cg * 8) = pack8(gd);
  };
  const uint4 zero4 = make_uint4(0, 0, 0, 0);
  for (long u = gt; u < U; u += 2 * S) {
    const bool two = u + S < U;
    int w0, w1 = 0;
    const long p0 = pix(u, w0);
    const long p1 = two ? pix(u + S, w1) : p0;
    const uint4 y0 = *reinterpret_cast<const uint4*>(y + p0 * ycs + cg * 8);
    const uint4 z0 = dz ? *reinterpret_cast<const uint4*>(dz + p0 * dzcs + cg * 8) : zero4;
    const uint4 q0 = *reinterpret_cast<const uint4*>(dpool + (long)w0 * C + cg * 8);
    uint4 y1 = zero4, z1 = zero4, q1 = zero4;
    if (two) {
      y1 = *reinterpret_cast<const uint4*>(y + p1 * ycs + cg * 8);
      if (dz) z1 = *reinterpret_cast<const uint4*>(dz + p1 * dzcs + cg * 8);
      q1 = *reinterpret_cast<const uint4*>(dpool + (long)w1 * C + cg * 8);
    }
    unit(p0, w0, y0, z0, q0);
    if (two) unit(p1, w1, y1, z1, q1);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) { red[threadIdx.x][j] = sg[j]; red[threadIdx.x][8 + j] = sgx[j]; }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += PNT) {
    const int gg = c / 8, j = c - gg * 8;
    float a = 0.f, b = 0.f;
    for (int t = 4 * gg; t < PNT; t += 4 * CG)               // threads holding chunk gg: (t >> 2) % CG == gg
      for (int q = 0; q < 4; ++q) { a += red[t + q][j]; b += red[t + q][8 + j]; }
    partial[(size_t)blockIdx.x * 2 * C + c] = a;
    partial[(size_t)blockIdx.x * 2 * C + C + c] = b;
  }
}

// partial: [G][T][2][C] (first S rows per group folded).  coef: [G][3][C].
// Grid = (channel chunks of 16) x G.  dgamma/dbeta are summed over the groups
// (one BatchNorm module, G calls): with G > 1 each block parks its group's sums
// in row 0 of the group and bn_bwd_groupsum_kernel adds them in order.
__global__ __launch_bounds__(stf::FOLD_NT) void bn_bwd_finalize_kernel(float* __restrict__ partial, int S, int T, int G,
                                                            int C, long Mg, const float* gamma, const float* mean,
                                                            const float* invstd, float* dgamma, float* dbeta,
                                                            float* coef) {
  __shared__ double red[stf::FOLD_NT];
  const int g = blockIdx.y;
  const int c = blockIdx.x * 16 + (threadIdx.x & 15);
  const bool cok = c < C, lead = cok && (threadIdx.x >> 4) == 0;
  float* base = partial + (size_t)g * T * 2 * C;
  double s1, s2;
  stf::fold16_pair(base, S, 2L * C, C, c, cok, red, s1, s2);
  if (lead) bn_fin_bwd_out(base, g, c, G, C, Mg, s1, s2, gamma, mean, invstd, dgamma, dbeta, coef);
}

// Deferred running-statistics updates of many grouped BatchNorms in one launch
// (blockIdx.y = descriptor; same arithmetic as bn_running_kernel).
constexpr int RUN_BATCH = 32;
struct RunBatch { stf_bn_run_desc d[RUN_BATCH]; };
__global__ void bn_running_batch_kernel(RunBatch b) {
  const stf_bn_run_desc& d = b.d[blockIdx.y];
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= d.C) return;
  float run_m = d.running_mean[c], run_v = d.running_var[c];
  const long Mg = (long)d.Mg;
  for (int g = 0; g < d.groups; ++g) {
    const float* base = d.stats + (size_t)g * d.tiles * 2 * d.C;
    const double var = base[d.C + c];
    const double unb = Mg > 1 ? var * Mg / (Mg - 1) : var;
    run_m = (1.f - d.momentum) * run_m + d.momentum * base[c];
    run_v = (1.f - d.momentum) * run_v + d.momentum * (float)unb;
  }
  d.running_mean[c] = run_m;
  d.running_var[c] = run_v;
}

// Deferred dgamma/dbeta sums of many grouped BatchNorm backwards in one launch
struct GsumBatch { stf_bn_gsum_desc d[RUN_BATCH]; };
__global__ void bn_groupsum_batch_kernel(GsumBatch b) {
  const stf_bn_gsum_desc& d = b.d[blockIdx.y];
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= d.C) return;
  double dg = 0.0, db = 0.0;
  for (int g = 0; g < d.groups; ++g) {
    const float* base = d.partial + (size_t)g * d.tiles * 2 * d.C;
    db += base[c];
    dg += base[d.C + c];
  }
  if (d.dgamma) d.dgamma[c] = (float)dg;
  if (d.dbeta) d.dbeta[c] = (float)db;
}

__global__ void bn_bwd_groupsum_kernel(const float* __restrict__ partial, int T, int G, int C, float* dgamma,
                                       float* dbeta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double dg = 0.0, db = 0.0;
  for (int g = 0; g < G; ++g) {
    const float* base = partial + (size_t)g * T * 2 * C;
    db += base[c];
    dg += base[C + c];
  }
  if (dgamma) dgamma[c] = (float)dg;
  if (dbeta) dbeta[c] = (float)db;
}

// dy = A*g' + B*y + C, g' = g (already masked) or, with mscale != NULL, the ReLU
// mask recomputed from y: g' = (y*mscale+mshift > 0) ? g : 0 (saves the masked copy)
__global__ void bn_bwd_apply_kernel(const uint16_t* g, int gcs, const uint16_t* __restrict__ y, int ycs, long M,
                                    int C, long Mg, const float* __restrict__ coef, const float* __restrict__ mscale,
                                    const float* __restrict__ mshift, uint16_t* dy, int dycs,
                                    float* __restrict__ bias_partial) {
  __shared__ float red[NT][9];
  const int CG = C / 8;
  const long units = M * CG;
  const long gt = blockIdx.x * (long)NT + threadIdx.x;
  const int cg = (int)(gt % CG);
  float sb[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int cur_g = -1;
  float A[8], B[8], Cc[8], ms[8], mh[8];
  for (long u = gt; u < units; u += (long)gridDim.x * NT) {
    const long pix = u / CG;
    const int grp = (int)(pix / Mg);
    if (grp != cur_g) {
      cur_g = grp;
      load_affine(coef + (size_t)grp * 3 * C, cg * 8, A);
      load_affine(coef + (size_t)grp * 3 * C + C, cg * 8, B);
      load_affine(coef + (size_t)grp * 3 * C + 2 * C, cg * 8, Cc);
      if (mscale) {
        load_affine(mscale + (size_t)grp * C, cg * 8, ms);
        load_affine(mshift + (size_t)grp * C, cg * 8, mh);
      }
    }
    float gv[8], yv[8];
    unpack8(*reinterpret_cast<const uint4*>(g + pix * gcs + cg * 8), gv);
    unpack8(*reinterpret_cast<const uint4*>(y + pix * ycs + cg * 8), yv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gj = (mscale && !(yv[j] * ms[j] + mh[j] > 0.f)) ? 0.f : gv[j];
      gv[j] = A[j] * gj + B[j] * yv[j] + Cc[j];
      sb[j] += gv[j];
    }
    *reinterpret_cast<uint4*>(dy + pix * dycs + cg * 8) = pack8(gv);
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

// ------------------------------------------------------------------ group-major streaming passes
// The same three element-wise passes with the grid split by statistics group (blockIdx.y = g):
// a thread's channel chunk and its group's affine / coefficient vectors are fixed, so the loop
// carries no per-unit division (the kernels above divide 64-bit unit and pixel indices by C/8
// and by the group size for every 16-B unit), and every thread issues the loads of UPT units
// (a block covers UPT x 256 consecutive units per iteration)
// before it uses any (UPT x 2-3 16-B loads in flight per lane: the STF encoder's 8-67 MB tensors
// are latency-bound at one unit per iteration).  Index math is 32-bit: units per group < 2^31
// (checked by the launchers).  Unit u of group g: pixel g * Mg + (u >> cgs), chunk u & (CG - 1).
constexpr int UPT = 4;

template <bool RES>
__global__ __launch_bounds__(NT) void bn_act_g_kernel(const uint16_t* __restrict__ y, int ycs, int Mg, int cgs,
                                                      const float* scale, const float* shift, int relu,
                                                      int res_mode, const uint16_t* __restrict__ res, int rcs,
                                                      const float* __restrict__ rscale,
                                                      const float* __restrict__ rshift, uint16_t* __restrict__ out,
                                                      int ocs) {
  const int g = blockIdx.y, C = 8 << cgs;
  const int upg = Mg << cgs, S = gridDim.x * NT * UPT;
  const int u0 = blockIdx.x * NT * UPT + threadIdx.x;
  const int cg = threadIdx.x & ((1 << cgs) - 1);
  float sc[8], sh[8], rs[8], rh[8];
  load_affine(scale + (size_t)g * C, cg * 8, sc);
  load_affine(shift + (size_t)g * C, cg * 8, sh);
  if (RES && res_mode == 2) {
    load_affine(rscale + (size_t)g * C, cg * 8, rs);
    load_affine(rshift + (size_t)g * C, cg * 8, rh);
  }
  const size_t p0 = (size_t)g * Mg;
  for (int u = u0; u < upg; u += S) {
    uint4 yv[UPT], rv[UPT];
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
      const int uk = u + k * NT;
      if (uk < upg) {
        const size_t p = p0 + (uk >> cgs);
        yv[k] = *reinterpret_cast<const uint4*>(y + p * ycs + cg * 8);
        if (RES) rv[k] = *reinterpret_cast<const uint4*>(res + p * rcs + cg * 8);
      }
    }
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
      const int uk = u + k * NT;
      if (uk >= upg) break;
      float v[8];
      unpack8(yv[k], v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = v[j] * sc[j] + sh[j];
      if (RES) {
        float r[8];
        unpack8(rv[k], r);
        if (res_mode == 2) {
#pragma unroll
          for (int j = 0; j < 8; ++j) r[j] = r[j] * rs[j] + rh[j];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += r[j];
      }
      if (relu) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = fmaxf(v[j], 0.f);
      }
      *reinterpret_cast<uint4*>(out + (p0 + (uk >> cgs)) * ocs + cg * 8) = pack8(v);
    }
  }
}

// mask_mode 0: none, 1: relu(y*scale+shift) > 0, 2: mask_src > 0; same sums as bn_bwd_reduce_kernel
template <int MASK>
__global__ __launch_bounds__(NT) void bn_bwd_reduce_g_kernel(const uint16_t* __restrict__ dz, int dzcs,
                                                             const uint16_t* __restrict__ y, int ycs, int Mg,
                                                             int cgs, const float* __restrict__ scale,
                                                             const float* __restrict__ shift,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ invstd,
                                                             const uint16_t* __restrict__ msrc, int mcs,
                                                             uint16_t* __restrict__ g_out, float* __restrict__ partial) {
  __shared__ float red[NT][17];
  const int g = blockIdx.y, CG = 1 << cgs, C = 8 << cgs;
  const int upg = Mg << cgs, S = gridDim.x * NT * UPT;
  const int u0 = blockIdx.x * NT * UPT + threadIdx.x;
  const int cg = threadIdx.x & (CG - 1);
  float sc[8], sh[8], mu[8], is[8];
  if (MASK == 1) {
    load_affine(scale + (size_t)g * C, cg * 8, sc);
    load_affine(shift + (size_t)g * C, cg * 8, sh);
  }
  load_affine(mean + (size_t)g * C, cg * 8, mu);
  load_affine(invstd + (size_t)g * C, cg * 8, is);
  float sg[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sgx[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const size_t p0 = (size_t)g * Mg;
  for (int u = u0; u < upg; u += S) {
    uint4 yv[UPT], zv[UPT], mv[UPT];
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
      const int uk = u + k * NT;
      if (uk < upg) {
        const size_t p = p0 + (uk >> cgs);
        yv[k] = *reinterpret_cast<const uint4*>(y + p * ycs + cg * 8);
        zv[k] = *reinterpret_cast<const uint4*>(dz + p * dzcs + cg * 8);
        if (MASK == 2) mv[k] = *reinterpret_cast<const uint4*>(msrc + p * mcs + cg * 8);
      }
    }
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
      const int uk = u + k * NT;
      if (uk >= upg) break;
      float v[8], d[8], mk[8];
      unpack8(yv[k], v);
      unpack8(zv[k], d);
      if (MASK == 2) unpack8(mv[k], mk);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        bool keep = true;
        if (MASK == 1) keep = v[j] * sc[j] + sh[j] > 0.f;
        else if (MASK == 2) keep = mk[j] > 0.f;
        const float gj = keep ? d[j] : 0.f;
        d[j] = gj;
        sg[j] += gj;
        sgx[j] += gj * (v[j] - mu[j]) * is[j];
      }
      if (g_out) *reinterpret_cast<uint4*>(g_out + (p0 + (uk >> cgs)) * C + cg * 8) = pack8(d);
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) { red[threadIdx.x][j] = sg[j]; red[threadIdx.x][8 + j] = sgx[j]; }
  __syncthreads();
  const size_t row = (size_t)g * gridDim.x + blockIdx.x;
  for (int c = threadIdx.x; c < C; c += NT) {
    const int gg = c >> 3, j = c & 7;
    float a = 0.f, b = 0.f;
    for (int t = gg; t < NT; t += CG) { a += red[t][j]; b += red[t][8 + j]; }
    partial[row * 2 * C + c] = a;
    partial[row * 2 * C + C + c] = b;
  }
}

// dy = A*g' + B*y + C (as bn_bwd_apply_kernel); bias_partial rows = g * gridDim.x + blockIdx.x
template <bool MASK>
__global__ __launch_bounds__(NT) void bn_bwd_apply_g_kernel(const uint16_t* g_in, int gcs,
                                                            const uint16_t* __restrict__ y, int ycs, int Mg, int cgs,
                                                            const float* coef, const float* __restrict__ mscale,
                                                            const float* __restrict__ mshift, uint16_t* dy,
                                                            int dycs, float* __restrict__ bias_partial) {
  __shared__ float red[NT][9];
  const int g = blockIdx.y, CG = 1 << cgs, C = 8 << cgs;
  const int upg = Mg << cgs, S = gridDim.x * NT * UPT;
  const int u0 = blockIdx.x * NT * UPT + threadIdx.x;
  const int cg = threadIdx.x & (CG - 1);
  float A[8], B[8], Cc[8], ms[8], mh[8];
  load_affine(coef + (size_t)g * 3 * C, cg * 8, A);
  load_affine(coef + (size_t)g * 3 * C + C, cg * 8, B);
  load_affine(coef + (size_t)g * 3 * C + 2 * C, cg * 8, Cc);
  if (MASK) {
    load_affine(mscale + (size_t)g * C, cg * 8, ms);
    load_affine(mshift + (size_t)g * C, cg * 8, mh);
  }
  float sb[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const size_t p0 = (size_t)g * Mg;
  for (int u = u0; u < upg; u += S) {
    uint4 gq[UPT], yq[UPT];
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
      const int uk = u + k * NT;
      if (uk < upg) {
        const size_t p = p0 + (uk >> cgs);
        gq[k] = *reinterpret_cast<const uint4*>(g_in + p * gcs + cg * 8);
        yq[k] = *reinterpret_cast<const uint4*>(y + p * ycs + cg * 8);
      }
    }
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
      const int uk = u + k * NT;
      if (uk >= upg) break;
      float gv[8], yv[8];
      unpack8(gq[k], gv);
      unpack8(yq[k], yv);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float gj = (MASK && !(yv[j] * ms[j] + mh[j] > 0.f)) ? 0.f : gv[j];
        gv[j] = A[j] * gj + B[j] * yv[j] + Cc[j];
        sb[j] += gv[j];
      }
      *reinterpret_cast<uint4*>(dy + (p0 + (uk >> cgs)) * dycs + cg * 8) = pack8(gv);
    }
  }
  if (!bias_partial) return;
#pragma unroll
  for (int j = 0; j < 8; ++j) red[threadIdx.x][j] = sb[j];
  __syncthreads();
  const size_t row = (size_t)g * gridDim.x + blockIdx.x;
  for (int c = threadIdx.x; c < C; c += NT) {
    const int gg = c >> 3, j = c & 7;
    float a = 0.f;
    for (int t = gg; t < NT; t += CG) a += red[t][j];
    bias_partial[row * C + c] = a;
  }
}

// ------------------------------------------------------------------ stem: BN backward through MaxPool(3,2,1)
// g of the stem's BatchNorm backward gathered straight from its max pool's backward: the sum of
// dout over the <= 4 windows whose recorded first maximum (argmax, index dy*3+dx) is this pixel,
// in the order stf_maxpool3s2_bwd adds them, rounded to the 16-bit storage -- so the values equal
// maxpool3s2_bwd + the mask-recomputing reduce / apply without writing or reading d a0.  A unit is
// a 2x2 block of input pixels (2by + a, 2bx + b): the windows (by + {0,1}, bx + {0,1}) cover all
// four, so each window's argmax and dout are loaded once per block (9 window reads for the four
// pixels in the per-pixel gather).
// APPLY = false: the (sum g, sum g*xhat) partials of bn_bwd_reduce_g_kernel<1>;
// APPLY = true: dy = A*g' + B*y + C with the ReLU mask recomputed (bn_bwd_apply_g_kernel<true>)
template <bool APPLY>
__global__ __launch_bounds__(NT) void bn_bwd_pool3_kernel(const uint8_t* __restrict__ argmax,
                                                          const uint16_t* __restrict__ dout,
                                                          const uint16_t* __restrict__ y, int H, int W, int Ho,
                                                          int Wo, int ipg, int cgs, const float* __restrict__ scale,
                                                          const float* __restrict__ shift,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ invstd,
                                                          const float* __restrict__ coef, uint16_t* __restrict__ dy,
                                                          float* __restrict__ partial) {
  __shared__ float red[APPLY ? 1 : NT][17];
  const int g = blockIdx.y, CG = 1 << cgs, C = 8 << cgs;
  const int H2 = (H + 1) >> 1, W2 = (W + 1) >> 1;
  const int bpi = H2 * W2;                               // 2x2 blocks per image
  const int upg = (ipg * bpi) << cgs, S = gridDim.x * NT;
  const int u0 = blockIdx.x * NT + threadIdx.x;
  const int cg = threadIdx.x & (CG - 1);
  float sc[8], sh[8], mu[8], is[8], A[8], B[8], Cc[8];
  load_affine(scale + (size_t)g * C, cg * 8, sc);
  load_affine(shift + (size_t)g * C, cg * 8, sh);
  if (APPLY) {
    load_affine(coef + (size_t)g * 3 * C, cg * 8, A);
    load_affine(coef + (size_t)g * 3 * C + C, cg * 8, B);
    load_affine(coef + (size_t)g * 3 * C + 2 * C, cg * 8, Cc);
  } else {
    load_affine(mean + (size_t)g * C, cg * 8, mu);
    load_affine(invstd + (size_t)g * C, cg * 8, is);
  }
  float sg[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sgx[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  // U units per iteration, all their loads issued before any use (the reduce runs <= 1024
  // blocks -- the finalize's row budget -- so it needs the memory-level parallelism per thread)
  constexpr int U = APPLY ? 1 : 2;
  for (int u = u0; u < upg; u += S * U) {
    uint2 am[U][2][2];
    uint4 dr[U][2][2], yr[U][2][2];
    int nn[U], bys[U], bxs[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int uk = u + k * S;
      const int b = uk >> cgs;
      const int n = g * ipg + b / bpi, rb = b - (b / bpi) * bpi;
      const int by = rb / W2, bx = rb - by * W2;
      nn[k] = uk < upg ? n : -1;
      bys[k] = by;
      bxs[k] = bx;
      // the four windows (by + wy, bx + wx): argmax (8 channel bytes) and dout (8 channels),
      // and the block's four pixels of y
#pragma unroll
      for (int wy = 0; wy < 2; ++wy)
#pragma unroll
        for (int wx = 0; wx < 2; ++wx) {
          const int oy = by + wy, ox = bx + wx;
          if (uk < upg && oy < Ho && ox < Wo) {
            const long wo = (((long)n * Ho + oy) * Wo + ox) * C + cg * 8;
            am[k][wy][wx] = *reinterpret_cast<const uint2*>(argmax + wo);
            dr[k][wy][wx] = *reinterpret_cast<const uint4*>(dout + wo);
          } else {
            am[k][wy][wx] = make_uint2(0xffffffffu, 0xffffffffu);    // matches no pixel
            dr[k][wy][wx] = make_uint4(0, 0, 0, 0);
          }
          const int iy = 2 * by + wy, ix = 2 * bx + wx;
          if (uk < upg && iy < H && ix < W)
            yr[k][wy][wx] = *reinterpret_cast<const uint4*>(y + (((size_t)n * H + iy) * W + ix) * C + cg * 8);
          else
            yr[k][wy][wx] = make_uint4(0, 0, 0, 0);
        }
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      if (nn[k] < 0) continue;
      const int n = nn[k], by = bys[k], bx = bxs[k];
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
          const int iy = 2 * by + a, ix = 2 * bx + bb;
          if (iy >= H || ix >= W) continue;
          float v[8], gq[8] = {0, 0, 0, 0, 0, 0, 0, 0};
          unpack8(yr[k][a][bb], v);
          // windows of pixel row iy: oy = by (always) and by + 1 (odd iy); same for x; ascending
#pragma unroll
          for (int wy = 0; wy < 2; ++wy) {
            if (wy > a) continue;
#pragma unroll
            for (int wx = 0; wx < 2; ++wx) {
              if (wx > bb) continue;
              const uint32_t me = (uint32_t)((iy - 2 * (by + wy) + 1) * 3 + (ix - 2 * (bx + wx) + 1));
              float d[8];
              unpack8(dr[k][wy][wx], d);
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                const uint32_t q = ((j < 4 ? am[k][wy][wx].x : am[k][wy][wx].y) >> (8 * (j & 3))) & 0xffu;
                if (q == me) gq[j] += d[j];
              }
            }
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float gr = round_e(gq[j]);
            const float gj = (v[j] * sc[j] + sh[j] > 0.f) ? gr : 0.f;
            if (APPLY) gq[j] = A[j] * gj + B[j] * v[j] + Cc[j];
            else {
              sg[j] += gj;
              sgx[j] += gj * (v[j] - mu[j]) * is[j];
            }
          }
          if (APPLY)
            *reinterpret_cast<uint4*>(dy + (((size_t)n * H + iy) * W + ix) * C + cg * 8) = pack8(gq);
        }
    }
  }
  if (APPLY) return;
#pragma unroll
  for (int j = 0; j < 8; ++j) { red[threadIdx.x][j] = sg[j]; red[threadIdx.x][8 + j] = sgx[j]; }
  __syncthreads();
  const size_t row = (size_t)g * gridDim.x + blockIdx.x;
  for (int c = threadIdx.x; c < C; c += NT) {
    const int gg = c >> 3, j = c & 7;
    float a = 0.f, b = 0.f;
    for (int t = gg; t < NT; t += CG) { a += red[t][j]; b += red[t][8 + j]; }
    partial[row * 2 * C + c] = a;
    partial[row * 2 * C + C + c] = b;
  }
}

}  // namespace

// the group-major kernels (STF_BN_G=0: the per-unit-division kernels, A/B); usable when C / 8 is
// a power of two dividing the block and a group's units fit 32-bit indices
static bool bn_g_ok(long Mg, int C) {
  static const bool on = stf::ab_switch("STF_BN_G", 1) != 0;
  const int CG = C / 8;
  return on && C % 8 == 0 && CG > 0 && (CG & (CG - 1)) == 0 && NT % CG == 0 && Mg * CG < (1L << 31);
}
static int log2i(int v) { return 31 - __builtin_clz(v); }
// blocks per group: about UPT units per thread, at least one, the whole grid <= cap blocks
static int g_tiles(long upg, int groups, long cap) {
  long t = (upg + (long)NT * UPT - 1) / ((long)NT * UPT);
  const long per = cap / groups > 0 ? cap / groups : 1;
  if (t > per) t = per;
  return (int)(t < 1 ? 1 : t);
}

// sum over tiles of partial[t][C] -> out[C] (fixed order); shared with misc.hip / loss.hip
// launch: grid ceil(C/16), 256 threads (16 channels x 16 row-lanes)
__global__ __launch_bounds__(stf::FOLD_NT) void stf_tile_sum_kernel(const float* __restrict__ partial, int tiles, int C,
                                                         float* __restrict__ out) {
  __shared__ double red[stf::FOLD_NT];
  const int c = blockIdx.x * 16 + (threadIdx.x & 15);
  const bool cok = c < C;
  const double s = stf::fold16_finish(stf::fold16_partial(partial, tiles, C, c, cok), red);
  if (cok && (threadIdx.x >> 4) == 0) out[c] = (float)s;
}

static bool cg_ok(int C) { return C % 8 == 0 && NT % (C / 8) == 0; }

extern "C" int stf_bn_finalize(float* stats, int tiles, int groups, int C, int64_t M, const float* gamma,
                               const float* beta, float momentum, float eps, float* running_mean,
                               float* running_var, float* mean, float* invstd, float* scale, float* shift,
                               stf_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  if (groups < 1 || M % groups) return STF_EINVAL;
  const int S = stats ? stf::colsum_stage1(stats, tiles, 2L * C, s, groups, stf::FOLD16_ROWS) : 0;
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 15) / 16, groups), dim3(stf::FOLD_NT), 0, s, stats, S, tiles, groups, C,
                     (long)(M / groups), gamma, beta, momentum, eps, running_mean, running_var, mean, invstd,
                     scale, shift);
  STF_CHECK_LAUNCH();
  if (stats && running_mean && groups > 1) {
    hipLaunchKernelGGL(bn_running_kernel, dim3((C + 255) / 256), dim3(256), 0, s, stats, tiles, groups, C,
                       (long)(M / groups), momentum, running_mean, running_var);
    STF_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int stf_bn_act(const void* y, int y_cstride, int N, int H, int W, int C, int groups,
                          const float* scale, const float* shift, int relu, const void* res, int res_cstride,
                          const float* res_scale, const float* res_shift, void* out, int out_cstride,
                          void* pooled, stf_stream_t stream) {
  if (C % 8 || y_cstride % 8 || out_cstride % 8 || (pooled && ((H | W) & 1)) || groups < 1 || N % groups)
    return STF_EINVAL;
  if (res && (res_cstride % 8 || pooled)) return STF_EINVAL;
  const int res_mode = res ? (res_scale ? 2 : 1) : 0;
  const long M = (long)N * H * W;
  const long units = pooled ? (long)N * (H / 2) * (W / 2) * (C / 8) : M * (C / 8);
  long blocks = (units + NT - 1) / NT;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) return 0;
  hipStream_t s = (hipStream_t)stream;
  const long Mg = M / groups;
  if (!pooled && bn_g_ok(Mg, C)) {
    const int cgs = log2i(C / 8);
    const dim3 grid(g_tiles(Mg * (C / 8), groups, 8192), groups);
    if (res)
      hipLaunchKernelGGL((bn_act_g_kernel<true>), grid, dim3(NT), 0, s, (const uint16_t*)y, y_cstride,
                         (int)Mg, cgs, scale, shift, relu, res_mode, (const uint16_t*)res, res_cstride, res_scale,
                         res_shift, (uint16_t*)out, out_cstride);
    else
      hipLaunchKernelGGL((bn_act_g_kernel<false>), grid, dim3(NT), 0, s, (const uint16_t*)y, y_cstride,
                         (int)Mg, cgs, scale, shift, relu, 0, (const uint16_t*)nullptr, 0, (const float*)nullptr,
                         (const float*)nullptr, (uint16_t*)out, out_cstride);
    STF_CHECK_LAUNCH();
    return 0;
  }
  if (pooled)
    hipLaunchKernelGGL((bn_act_kernel<true>), dim3(blocks), dim3(NT), 0, s, (const uint16_t*)y, y_cstride,
                       (long)N, H, W, C, Mg, scale, shift, relu, 0, (const uint16_t*)nullptr, 0,
                       (const float*)nullptr, (const float*)nullptr, (uint16_t*)out, out_cstride, (uint16_t*)pooled);
  else
    hipLaunchKernelGGL((bn_act_kernel<false>), dim3(blocks), dim3(NT), 0, s, (const uint16_t*)y, y_cstride,
                       (long)N, H, W, C, Mg, scale, shift, relu, res_mode, (const uint16_t*)res, res_cstride,
                       res_scale, res_shift, (uint16_t*)out, out_cstride, (uint16_t*)nullptr);
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_bn_bwd_tiles(int N, int H, int W, int C, int groups, int pooled) {
  const long Ng = (long)N / groups;
  const long upg = pooled ? Ng * (H / 2) * (W / 2) * (C / 8) : Ng * H * W * (C / 8);
  return tiles_per_group(upg, groups);
}

extern "C" int stf_bn_bwd_reduce(const void* dz, int dz_cstride, const void* dpool, const void* y, int y_cstride,
                                 int N, int H, int W, int C, int groups, const float* scale, const float* shift,
                                 const float* mean, const float* invstd, int mask_mode, const void* mask_src,
                                 int mask_cstride, void* g_out, float* partial, stf_stream_t stream) {
  if (!cg_ok(C) || y_cstride % 8 || (dz && dz_cstride % 8) || groups < 1 || N % groups) return STF_EINVAL;
  if (!dz && !dpool) return STF_EINVAL;
  if (!g_out && dpool) return STF_EINVAL;            // the pooled routing must be materialized
  if (dpool && (((H | W) & 1) || mask_mode == 2)) return STF_EINVAL;
  if (mask_mode == 2 && (!mask_src || mask_cstride % 8)) return STF_EINVAL;
  const int tpg = stf_bn_bwd_tiles(N, H, W, C, groups, dpool != nullptr);
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(tpg * groups);
  const long Mgp = (long)N * H * W / groups;
  if (!dpool && bn_g_ok(Mgp, C)) {
    const dim3 g2(tpg, groups);
    const int cgs = log2i(C / 8);
#define STF_RG(MM) hipLaunchKernelGGL(bn_bwd_reduce_g_kernel<MM>, g2, dim3(NT), 0, s, (const uint16_t*)dz, dz_cstride, \
                                      (const uint16_t*)y, y_cstride, (int)Mgp, cgs, scale, shift, mean, invstd,     \
                                      (const uint16_t*)mask_src, mask_cstride, (uint16_t*)g_out, partial)
    if (mask_mode == 1) STF_RG(1);
    else if (mask_mode == 2) STF_RG(2);
    else STF_RG(0);
#undef STF_RG
    STF_CHECK_LAUNCH();
    return 0;
  }
  static const bool lanes = stf::ab_switch("STF_POOL_LANES", 1) != 0;
  if (dpool && lanes && 64 % (C / 8) == 0 && mask_mode != 2 && (long)N * H * W < (1L << 31))
    hipLaunchKernelGGL(bn_bwd_reduce_pool_kernel, grid, dim3(PNT), 0, s, (const uint16_t*)dz, dz_cstride,
                       (const uint16_t*)dpool, (const uint16_t*)y, y_cstride, (long)N, H, W, C, groups, tpg, scale,
                       shift, mean, invstd, mask_mode, (uint16_t*)g_out, partial);
  else if (dpool)
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<true>, grid, dim3(NT), 0, s, (const uint16_t*)dz, dz_cstride,
                       (const uint16_t*)dpool, (const uint16_t*)y, y_cstride, (long)N, H, W, C, groups, tpg, scale,
                       shift, mean, invstd, mask_mode, (const uint16_t*)mask_src, mask_cstride, (uint16_t*)g_out,
                       partial);
  else
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<false>, grid, dim3(NT), 0, s, (const uint16_t*)dz, dz_cstride,
                       (const uint16_t*)nullptr, (const uint16_t*)y, y_cstride, (long)N, H, W, C, groups, tpg,
                       scale, shift, mean, invstd, mask_mode, (const uint16_t*)mask_src, mask_cstride,
                       (uint16_t*)g_out, partial);
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_bn_bwd_finalize(float* partial, int tiles, int groups, int C, int64_t M, const float* gamma,
                                   const float* mean, const float* invstd, float* dgamma, float* dbeta, float* coef,
                                   stf_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  if (groups < 1 || M % groups) return STF_EINVAL;
  const int S = stf::colsum_stage1(partial, tiles, 2L * C, s, groups, stf::FOLD16_ROWS);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 15) / 16, groups), dim3(stf::FOLD_NT), 0, s, partial, S, tiles, groups,
                     C, (long)(M / groups), gamma, mean, invstd, dgamma, dbeta, coef);
  STF_CHECK_LAUNCH();
  if (groups > 1 && (dgamma || dbeta)) {
    hipLaunchKernelGGL(bn_bwd_groupsum_kernel, dim3((C + 255) / 256), dim3(256), 0, s, partial, tiles, groups, C,
                       dgamma, dbeta);
    STF_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int stf_bn_running_batch(const stf_bn_run_desc* descs, int count, stf_stream_t stream) {
  for (int i = 0; i < count; ++i)
    if (!descs[i].stats || !descs[i].running_mean || !descs[i].running_var || descs[i].groups < 1 ||
        descs[i].C < 1 || descs[i].tiles < 1)
      return STF_EINVAL;
  for (int i0 = 0; i0 < count; i0 += RUN_BATCH) {
    const int n = count - i0 < RUN_BATCH ? count - i0 : RUN_BATCH;
    RunBatch b;
    int cmax = 0;
    for (int i = 0; i < n; ++i) { b.d[i] = descs[i0 + i]; cmax = cmax > b.d[i].C ? cmax : b.d[i].C; }
    hipLaunchKernelGGL(bn_running_batch_kernel, dim3((cmax + 255) / 256, n), dim3(256), 0, (hipStream_t)stream, b);
    STF_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int stf_bn_groupsum_batch(const stf_bn_gsum_desc* descs, int count, stf_stream_t stream) {
  for (int i = 0; i < count; ++i)
    if (!descs[i].partial || descs[i].groups < 1 || descs[i].C < 1 || descs[i].tiles < 1) return STF_EINVAL;
  for (int i0 = 0; i0 < count; i0 += RUN_BATCH) {
    const int n = count - i0 < RUN_BATCH ? count - i0 : RUN_BATCH;
    GsumBatch b;
    int cmax = 0;
    for (int i = 0; i < n; ++i) { b.d[i] = descs[i0 + i]; cmax = cmax > b.d[i].C ? cmax : b.d[i].C; }
    hipLaunchKernelGGL(bn_groupsum_batch_kernel, dim3((cmax + 255) / 256, n), dim3(256), 0, (hipStream_t)stream, b);
    STF_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int stf_bn_bwd_apply_tiles(int64_t M, int C) {
  long t = (M * (C / 8) + NT - 1) / NT;
  return (int)(t < 1 ? 1 : (t > 1024 ? 1024 : t));
}

extern "C" int stf_bn_bwd_apply(const void* g, int g_cstride, const void* y, int y_cstride, int64_t M, int C,
                                int groups, const float* mask_scale, const float* mask_shift, const float* coef,
                                void* dy, int dy_cstride, float* bias_partial, float* dbias, stf_stream_t stream) {
  if (!cg_ok(C) || y_cstride % 8 || dy_cstride % 8 || g_cstride % 8 || groups < 1 || M % groups) return STF_EINVAL;
  if ((mask_scale == nullptr) != (mask_shift == nullptr)) return STF_EINVAL;
  int tiles = stf_bn_bwd_apply_tiles(M, C);
  hipStream_t s = (hipStream_t)stream;
  const long Mg = M / groups;
  if (bn_g_ok(Mg, C)) {
    // bias_partial rows: groups x tpg <= stf_bn_bwd_apply_tiles (the caller's allocation)
    const int tpg = g_tiles(Mg * (C / 8), groups, bias_partial ? tiles : 8192);
    const dim3 grid(tpg, groups);
    const int cgs = log2i(C / 8);
    if (mask_scale)
      hipLaunchKernelGGL((bn_bwd_apply_g_kernel<true>), grid, dim3(NT), 0, s, (const uint16_t*)g, g_cstride,
                         (const uint16_t*)y, y_cstride, (int)Mg, cgs, coef, mask_scale, mask_shift, (uint16_t*)dy,
                         dy_cstride, bias_partial);
    else
      hipLaunchKernelGGL((bn_bwd_apply_g_kernel<false>), grid, dim3(NT), 0, s, (const uint16_t*)g, g_cstride,
                         (const uint16_t*)y, y_cstride, (int)Mg, cgs, coef, mask_scale, mask_shift, (uint16_t*)dy,
                         dy_cstride, bias_partial);
    tiles = tpg * groups;
  } else {
    hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(tiles), dim3(NT), 0, s, (const uint16_t*)g, g_cstride,
                       (const uint16_t*)y, y_cstride, (long)M, C, (long)(M / groups), coef, mask_scale, mask_shift,
                       (uint16_t*)dy, dy_cstride, bias_partial);
  }
  STF_CHECK_LAUNCH();
  if (bias_partial && dbias) {
    const int S = stf::colsum_stage1(bias_partial, tiles, C, s, 1, stf::FOLD16_ROWS);
    hipLaunchKernelGGL(stf_tile_sum_kernel, dim3((C + 15) / 16), dim3(stf::FOLD_NT), 0, s, bias_partial, S, C, dbias);
    STF_CHECK_LAUNCH();
  }
  return 0;
}

// BatchNorm backward of the STF stem through its MaxPool(3,2,1) (src/stf_lstm_unet.py:178-180):
// the incoming gradient is the pooled output's (dout [N][Ho][Wo][C]) routed by the forward's
// argmax (stf_bn_act_maxpool3s2 / stf_maxpool3s2_fwd), never materialized at full size.
// Partials as stf_bn_bwd_reduce (rows per group = stf_bn_bwd_tiles(N, H, W, C, groups, 0)).
extern "C" int stf_bn_bwd_reduce_pool3(const void* argmax, const void* dout, const void* y, int N, int H, int W,
                                       int C, int groups, const float* scale, const float* shift,
                                       const float* mean, const float* invstd, float* partial,
                                       stf_stream_t stream) {
  const long Mg = (long)N * H * W / (groups > 0 ? groups : 1);
  if (!argmax || !dout || !y || !partial || groups < 1 || N % groups || !bn_g_ok(Mg, C) ||
      (long)N * H * W >= (1L << 31))
    return STF_EINVAL;
  const int tpg = stf_bn_bwd_tiles(N, H, W, C, groups, 0);
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  hipLaunchKernelGGL(bn_bwd_pool3_kernel<false>, dim3(tpg, groups), dim3(NT), 0, (hipStream_t)stream,
                     (const uint8_t*)argmax, (const uint16_t*)dout, (const uint16_t*)y, H, W, Ho, Wo, N / groups,
                     log2i(C / 8), scale, shift, mean, invstd, (const float*)nullptr, (uint16_t*)nullptr, partial);
  STF_CHECK_LAUNCH();
  return 0;
}

// dy = A g' + B y + C (coef from stf_bn_bwd_finalize), g' = the routed gradient masked by the ReLU.
extern "C" int stf_bn_bwd_apply_pool3(const void* argmax, const void* dout, const void* y, int N, int H, int W,
                                      int C, int groups, const float* scale, const float* shift, const float* coef,
                                      void* dy, stf_stream_t stream) {
  const long Mg = (long)N * H * W / (groups > 0 ? groups : 1);
  if (!argmax || !dout || !y || !coef || !dy || groups < 1 || N % groups || !bn_g_ok(Mg, C) ||
      (long)N * H * W >= (1L << 31))
    return STF_EINVAL;
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  const long units = (long)(N / groups) * ((H + 1) / 2) * ((W + 1) / 2) * (C / 8);
  const dim3 grid(g_tiles(units, groups, 8192) * UPT, groups);
  hipLaunchKernelGGL(bn_bwd_pool3_kernel<true>, grid, dim3(NT), 0, (hipStream_t)stream, (const uint8_t*)argmax,
                     (const uint16_t*)dout, (const uint16_t*)y, H, W, Ho, Wo, N / groups, log2i(C / 8), scale, shift,
                     (const float*)nullptr, (const float*)nullptr, coef, (uint16_t*)dy, (float*)nullptr);
  STF_CHECK_LAUNCH();
  return 0;
}
