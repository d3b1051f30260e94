// PK-map generation: extended Tofts model and its per-pixel Adam fit (pk_fitting.py,
// SURVEY.md section 8(f) rank 3).
//
//   C(t_i) = vp Cp(t_i) + Ktrans dt sum_{tau_j < t_i} Cp(tau_j) exp(-Ktrans (t_i - tau_j) / ve)
//
// (pk_fitting.py:193-231; a time point with no tau_j < t_i stays 0).  The reference fits
// every tissue pixel by running its batched PyTorch model over batches of 1,024 pixels
// for 100 epochs (pk_fitting.py:233-420): ~25,600 Python-driven kernel sequences per
// 256x256 slice.  Every pixel's fit is independent -- the MSE of a batch splits into
// per-pixel terms scaled by 2 / (batch * T), and Adam is elementwise -- so here ONE
// launch runs the whole schedule, 16 lanes per pixel: the gradient when the pixel's own
// batch is stepped (the lanes split the convolution terms), a zero-gradient Adam step
// (the reference still moves those parameters through its momentum) for every other
// batch, the clamps after each step.  The tau grid and Cp(tau) sit in LDS; one expf
// per term.  VALU-bound (exp, the IEEE division kept from the reference's
// expression), no HBM traffic to speak of.
#include "common.h"
#include "../../include/stfunet.h"

namespace {

constexpr int PK_NT = 256;
constexpr int PK_MAXT = 32;

// S0 = sum_{j<n} Cp_j e_j, S1 = sum_{j<n} Cp_j e_j (t - tau_j), e_j = exp(-(k (t - tau_j)) / ve)
STF_DEV void tofts_sums(const float* tau, const float* cp, int n, float t, float k, float ve, double& s0,
                        double& s1) {
  double a0 = 0.0, a1 = 0.0;
  for (int j = 0; j < n; ++j) {
    const float d = t - tau[j];
    const float e = expf(-k * d / ve);
    const float ae = cp[j] * e;
    a0 += ae;
    a1 += (double)ae * d;
  }
  s0 = a0;
  s1 = a1;
}

__global__ __launch_bounds__(PK_NT) void tofts_forward_kernel(const float* __restrict__ kt,
                                                              const float* __restrict__ ve,
                                                              const float* __restrict__ vp, int P, int T,
                                                              const float* __restrict__ tp,
                                                              const float* __restrict__ cp_t,
                                                              const float* __restrict__ tau_g,
                                                              const float* __restrict__ cp_g,
                                                              const int* __restrict__ nv, int n_conv, float dt,
                                                              float* __restrict__ out) {
  extern __shared__ float sh[];
  float* tau = sh;
  float* cp = sh + n_conv;
  for (int j = threadIdx.x; j < n_conv; j += PK_NT) { tau[j] = tau_g[j]; cp[j] = cp_g[j]; }
  __syncthreads();
  const int q = blockIdx.x * PK_NT + threadIdx.x;
  if (q >= P) return;
  const float k = kt[q], v = ve[q], p = vp[q];
  for (int i = 0; i < T; ++i) {
    float c = 0.f;
    if (nv[i] > 0) {
      double s0, s1;
      tofts_sums(tau, cp, nv[i], tp[i], k, v, s0, s1);
      c = p * cp_t[i] + k * ((float)s0 * dt);
    }
    out[(size_t)q * T + i] = c;
  }
}

struct AdamCfg {
  float w1;        // 1 - beta1 (lerp weight)
  float b2, w2;    // beta2, 1 - beta2
  float eps;
  float lo[3], hi[3];
};

// PK_L lanes share one pixel: lane l sums the convolution terms j = l, l + PK_L, ... and
// the PK_L partial sums are combined with xor shuffles (every lane ends with the same
// totals, so all of them run the identical Adam step; lane 0 writes the result).  A
// 256x256 slice has ~40k tissue pixels: one thread per pixel would leave most SIMDs idle.
constexpr int PK_L = 16;

STF_DEV float lanes_sum(float v) {
#pragma unroll
  for (int o = PK_L / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, PK_L);
  return v;
}

__global__ __launch_bounds__(PK_NT) void tofts_fit_kernel(const float* __restrict__ curves, int P, int T,
                                                          const float* __restrict__ tp,
                                                          const float* __restrict__ cp_t,
                                                          const float* __restrict__ tau_g,
                                                          const float* __restrict__ cp_g,
                                                          const int* __restrict__ nv, int n_conv, float dt,
                                                          int batch, int epochs,
                                                          const float* __restrict__ sched, AdamCfg cfg,
                                                          float* __restrict__ params) {
  extern __shared__ float sh[];
  float* tau = sh;
  float* cp = sh + n_conv;
  for (int j = threadIdx.x; j < n_conv; j += PK_NT) { tau[j] = tau_g[j]; cp[j] = cp_g[j]; }
  __syncthreads();
  const int gq = (blockIdx.x * PK_NT + threadIdx.x) / PK_L, sl = threadIdx.x % PK_L;
  const bool live = gq < P;
  const int q = live ? gq : P - 1;                           // padding lanes shadow the last pixel
  const int nb = (P + batch - 1) / batch, myb = q / batch;
  const int bs = min(batch, P - myb * batch);
  const float norm = (float)(2.0 / ((double)bs * T));          // d mean((C - y)^2) / dC
  float p[3] = {params[q], params[P + q], params[2 * P + q]};
  float m[3] = {0.f, 0.f, 0.f}, v[3] = {0.f, 0.f, 0.f};
  const int steps = epochs * nb;
  for (int s = 0; s < steps; ++s) {
    float g[3] = {0.f, 0.f, 0.f};
    if (s % nb == myb) {
      const float k = p[0], e = p[1], vp = p[2];
      for (int i = 0; i < T; ++i) {
        const int n = nv[i];
        if (n == 0) continue;                                  // C(t_i) = 0, no parameter dependence
        const float ti = tp[i];
        float a0 = 0.f, a1 = 0.f;
        for (int j = sl; j < n; j += PK_L) {
          const float d = ti - tau[j];
          const float ae = cp[j] * expf(-k * d / e);
          a0 += ae;
          a1 += ae * d;
        }
        const float conv = lanes_sum(a0) * dt, sd = lanes_sum(a1) * dt;
        const float c = vp * cp_t[i] + k * conv;
        const float gl = norm * (c - curves[(size_t)q * T + i]);
        g[0] += gl * (conv - k * sd / e);
        g[1] += gl * (k * k * sd / (e * e));
        g[2] += gl * cp_t[i];
      }
    }
    // torch.optim.Adam single-tensor step (lerp, addcmul, addcdiv), then the clamps
    const float step_size = sched[2 * s], bc2 = sched[2 * s + 1];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      m[r] = m[r] + cfg.w1 * (g[r] - m[r]);
      v[r] = v[r] * cfg.b2 + cfg.w2 * g[r] * g[r];
      const float den = sqrtf(v[r]) / bc2 + cfg.eps;
      p[r] = p[r] + (-step_size) * m[r] / den;
      p[r] = fminf(fmaxf(p[r], cfg.lo[r]), cfg.hi[r]);
    }
  }
  if (live && sl == 0) {
    params[q] = p[0];
    params[P + q] = p[1];
    params[2 * P + q] = p[2];
  }
}

bool pk_args_ok(int P, int T, int n_conv, const int* nv) {
  return P >= 0 && T >= 1 && T <= PK_MAXT && n_conv >= 0 && n_conv <= 8192 && nv != nullptr;
}

}  // namespace

extern "C" int stf_tofts_forward(const float* ktrans, const float* ve, const float* vp, int P, int T,
                                 const float* time_points, const float* cp_t, const float* tau,
                                 const float* cp_tau, const int* n_valid, int n_conv, float dt, float* out,
                                 stf_stream_t stream) {
  if (!pk_args_ok(P, T, n_conv, n_valid)) return STF_EINVAL;
  if (P == 0) return 0;
  hipLaunchKernelGGL(tofts_forward_kernel, dim3((P + PK_NT - 1) / PK_NT), dim3(PK_NT), 2 * n_conv * sizeof(float),
                     (hipStream_t)stream, ktrans, ve, vp, P, T, time_points, cp_t, tau, cp_tau, n_valid, n_conv, dt,
                     out);
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_tofts_fit(const float* curves, int P, int T, const float* time_points, const float* cp_t,
                             const float* tau, const float* cp_tau, const int* n_valid, int n_conv, float dt,
                             int batch, int epochs, const float* adam_sched, float beta1, float beta2, float eps,
                             const float* bounds, float* params, stf_stream_t stream) {
  if (!pk_args_ok(P, T, n_conv, n_valid) || batch < 1 || epochs < 0 || !bounds) return STF_EINVAL;
  if (P == 0) return 0;
  AdamCfg cfg;
  cfg.w1 = (float)(1.0 - (double)beta1);
  cfg.b2 = beta2;
  cfg.w2 = (float)(1.0 - (double)beta2);
  cfg.eps = eps;
  for (int r = 0; r < 3; ++r) { cfg.lo[r] = bounds[2 * r]; cfg.hi[r] = bounds[2 * r + 1]; }
  const long threads = (long)P * PK_L;
  hipLaunchKernelGGL(tofts_fit_kernel, dim3((unsigned)((threads + PK_NT - 1) / PK_NT)), dim3(PK_NT),
                     2 * n_conv * sizeof(float),
                     (hipStream_t)stream, curves, P, T, time_points, cp_t, tau, cp_tau, n_valid, n_conv, dt, batch,
                     epochs, adam_sched, cfg, params);
  STF_CHECK_LAUNCH();
  return 0;
}
