// Segmentation head (1x1 OutConv fused with the last BN+ReLU) and the
// CE + multiclass-Dice criterion, forward and backward.
//
// Head: a = relu(y*scale + shift) is never materialised -- 8 lanes per pixel
// each take 8 channels, form partial logits and reduce them with xor shuffles.
// Loss (train_and_eval.py:299-313, dice_coefficient_loss.py:5-55), per image b
// and class k with p = softmax(logits), t = one_hot(target):
//   I = sum p t, S = sum p + sum t, D = (2I + eps)/(S + eps)  (S == 0 -> D = 1),
//   loss = mean CE + 1 - mean_k mean_b D.
// Backward: dz = go * [ (p - t)/Npix + p (G - sum_j p_j G_j) ],
//   G_k = -(1/(K*B)) dD/dp = -(1/(K*B)) (2 t/(S+eps) - (2I+eps)/(S+eps)^2).
#include "common.h"
#include "../../include/stfunet.h"
#include "reduce.h"

namespace {

constexpr int NT = 256;
constexpr int MAXK = 4;          // classes supported by the fused kernels
constexpr int LCHUNK = 64;       // loss partial chunks per image
constexpr float DICE_EPS = 1e-6f;

STF_DEV void load8f(const float* p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// sum over the CG adjacent lanes of a pixel (CG a power of two <= 64), every lane gets it: DPP
// inside a 16-lane row (quad swaps, half-row and row mirrors -- VALU, no LDS), ds_bpermute
// (__shfl_xor) only across rows.  (__shfl_xor for every step made head_fwd VALU/LDS-issue bound:
// 2 TB/s on a 0.29 GB pass.)
STF_DEV float lane_group_sum(float v, int CG) {
  if (CG >= 2) v += dpp_f<0xB1>(v);      // quad_perm [1,0,3,2]
  if (CG >= 4) v += dpp_f<0x4E>(v);      // quad_perm [2,3,0,1]
  if (CG >= 8) v += dpp_f<0x141>(v);     // row_half_mirror
  if (CG >= 16) v += dpp_f<0x140>(v);    // row_mirror
  for (int o = 16; o < CG; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

int head_tiles(long units) {
  long t = (units + NT - 1) / NT;
  return (int)(t < 1 ? 1 : (t > 1024 ? 1024 : t));
}

template <int K>
__global__ void head_fwd_kernel(const uint16_t* __restrict__ y, long P, int HW, int C,
                                const float* __restrict__ scale, const float* __restrict__ shift,
                                const float* __restrict__ w, const float* __restrict__ bias,
                                float* __restrict__ logits) {
  // CG lanes of one pixel are adjacent (NT and the grid stride are multiples of
  // CG, so a thread's channel group is fixed); 4 pixels per thread per round so
  // four 16-B loads are in flight before any arithmetic
  // 32-bit index math (the host checks P * CG < 2^31): 64-bit divisions cost ~40 instructions
  constexpr int U = 4;
  const int CG = C / 8, cgs = __builtin_ctz(CG);          // CG is a power of two (head_ok)
  const int units = (int)(P * CG);
  const int cg = (int)((blockIdx.x * NT + threadIdx.x) & (CG - 1));
  float sc[8], sh[8], wk[K][8], bk[K];
  load8f(scale + cg * 8, sc);
  load8f(shift + cg * 8, sh);
#pragma unroll
  for (int k = 0; k < K; ++k) { load8f(w + k * C + cg * 8, wk[k]); bk[k] = bias[k]; }
  const int stride = gridDim.x * NT;
  for (int u0 = blockIdx.x * NT; u0 < units; u0 += stride * U) {
    uint4 raw[U];
#pragma unroll
    for (int r = 0; r < U; ++r) {
      const int u = u0 + r * stride + threadIdx.x;
      raw[r] = u < units ? *reinterpret_cast<const uint4*>(y + (size_t)(u >> cgs) * C + cg * 8) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < U; ++r) {
      const int u = u0 + r * stride + threadIdx.x;
      float v[8], acc[K];
      unpack8(raw[r], v);
#pragma unroll
      for (int k = 0; k < K; ++k) acc[k] = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float a = fmaxf(v[j] * sc[j] + sh[j], 0.f);
#pragma unroll
        for (int k = 0; k < K; ++k) acc[k] += a * wk[k][j];
      }
#pragma unroll
      for (int k = 0; k < K; ++k) acc[k] = lane_group_sum(acc[k], CG);
      if (u < units && cg == 0) {
        const int pix = u >> cgs, n = pix / HW, hw = pix - n * HW;
#pragma unroll
        for (int k = 0; k < K; ++k) logits[(size_t)(n * K + k) * HW + hw] = acc[k] + bk[k];
      }
    }
  }
}

template <int K>
__global__ void head_bwd_kernel(const float* __restrict__ dlogits, const uint16_t* __restrict__ y, long P, int HW,
                                int C, const float* __restrict__ scale, const float* __restrict__ shift,
                                const float* __restrict__ mean, const float* __restrict__ invstd,
                                const float* __restrict__ w, uint16_t* __restrict__ g_out,
                                float* __restrict__ bn_partial, float* __restrict__ head_partial) {
  constexpr int NV = 16 + 8 * K + K;       // sg[8], sgx[8], dW[K][8], db[K]
  __shared__ float red[NT][NV + 1];
  const int CG = C / 8, cgs = __builtin_ctz(CG);          // CG is a power of two (head_ok)
  const int units = (int)(P * CG);                // < 2^31 (host check): 32-bit index math
  const int gt = blockIdx.x * NT + threadIdx.x;
  const int cg = gt & (CG - 1);
  float sc[8], sh[8], mu[8], is[8], wk[K][8];
  load8f(scale + cg * 8, sc);
  load8f(shift + cg * 8, sh);
  load8f(mean + cg * 8, mu);
  load8f(invstd + cg * 8, is);
#pragma unroll
  for (int k = 0; k < K; ++k) load8f(w + k * C + cg * 8, wk[k]);
  float sg[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sgx[8] = {0, 0, 0, 0, 0, 0, 0, 0}, dw[K][8], db[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    db[k] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) dw[k][j] = 0.f;
  }
  // one unit per iteration (two with the loads hoisted: 219 -> 245 us at cfg2, fewer waves)
  constexpr int U = 1;
  const int S = gridDim.x * NT;
  for (int u0 = gt; u0 < units; u0 += S * U) {
    float dlr[U][K];
    uint4 yr[U];
    int pixr[U];
#pragma unroll
    for (int r = 0; r < U; ++r) {
      const int u = u0 + r * S;
      const bool ok = u < units;
      const int pix = ok ? u >> cgs : 0, n = pix / HW, hw = pix - n * HW;
      pixr[r] = ok ? pix : -1;
#pragma unroll
      for (int k = 0; k < K; ++k) dlr[r][k] = ok ? dlogits[(size_t)(n * K + k) * HW + hw] : 0.f;
      yr[r] = ok ? *reinterpret_cast<const uint4*>(y + (size_t)pix * C + cg * 8) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < U; ++r) {
    if (pixr[r] < 0) continue;
    const int pix = pixr[r];
    const float* dl = dlr[r];
    float v[8], g[8];
    unpack8(yr[r], v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float z = v[j] * sc[j] + sh[j];
      const float a = fmaxf(z, 0.f);
      float da = 0.f;
#pragma unroll
      for (int k = 0; k < K; ++k) { da += dl[k] * wk[k][j]; dw[k][j] += dl[k] * a; }
      g[j] = z > 0.f ? da : 0.f;
      sg[j] += g[j];
      sgx[j] += g[j] * (v[j] - mu[j]) * is[j];
    }
    if (cg == 0) {
#pragma unroll
      for (int k = 0; k < K; ++k) db[k] += dl[k];
    }
    *reinterpret_cast<uint4*>(g_out + (size_t)pix * C + cg * 8) = pack8(g);
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) { red[threadIdx.x][j] = sg[j]; red[threadIdx.x][8 + j] = sgx[j]; }
#pragma unroll
  for (int k = 0; k < K; ++k) {
#pragma unroll
    for (int j = 0; j < 8; ++j) red[threadIdx.x][16 + k * 8 + j] = dw[k][j];
    red[threadIdx.x][16 + 8 * K + k] = db[k];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += NT) {
    const int gg = c / 8, j = c - gg * 8;
    float a = 0.f, b = 0.f;
    for (int t = gg; t < NT; t += CG) { a += red[t][j]; b += red[t][8 + j]; }
    bn_partial[(size_t)blockIdx.x * 2 * C + c] = a;
    bn_partial[(size_t)blockIdx.x * 2 * C + C + c] = b;
  }
  const int HC = K * (C + 1);
  for (int e = threadIdx.x; e < HC; e += NT) {
    float a = 0.f;
    if (e < K * C) {
      const int k = e / C, c = e - k * C, gg = c / 8, j = c - gg * 8;
      for (int t = gg; t < NT; t += CG) a += red[t][16 + k * 8 + j];
    } else {
      const int k = e - K * C;
      for (int t = 0; t < NT; t += CG) a += red[t][16 + 8 * K + k];
    }
    head_partial[(size_t)blockIdx.x * HC + e] = a;
  }
}

// ------------------------------------------------------------------ loss
template <int K>
__global__ void loss_fwd_kernel(const float* __restrict__ logits, const int64_t* __restrict__ target, int HW,
                                float* __restrict__ part) {
  // grid (LCHUNK, N): partial[n][chunk][3K + 1]
  constexpr int NV = 3 * K + 1;
  __shared__ float red[NT / 64][NV];
  const int n = blockIdx.y;
  float s[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) s[i] = 0.f;
  for (int hw = blockIdx.x * NT + threadIdx.x; hw < HW; hw += gridDim.x * NT) {
    float z[K], e[K], mx = -INFINITY;
#pragma unroll
    for (int k = 0; k < K; ++k) { z[k] = logits[((long)n * K + k) * HW + hw]; mx = fmaxf(mx, z[k]); }
    float se = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) { e[k] = expf(z[k] - mx); se += e[k]; }
    const int t = (int)target[(long)n * HW + hw];
    const float inv = 1.f / se, lse = logf(se);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const float p = e[k] * inv;
      const float tk = t == k ? 1.f : 0.f;
      s[3 * k] += p * tk;
      s[3 * k + 1] += p;
      s[3 * k + 2] += tk;
      if (t == k) s[3 * K] += lse - (z[k] - mx);   // -log_softmax, stable when p underflows
    }
  }
#pragma unroll
  for (int i = 0; i < NV; ++i) s[i] = wave_sum(s[i]);
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int i = 0; i < NV; ++i) red[threadIdx.x >> 6][i] = s[i];
  __syncthreads();
  if (threadIdx.x < NV) {
    float a = 0.f;
    for (int wv = 0; wv < NT / 64; ++wv) a += red[wv][threadIdx.x];
    part[((size_t)n * gridDim.x + blockIdx.x) * NV + threadIdx.x] = a;
  }
}

template <int K>
__global__ void loss_finalize_kernel(const float* __restrict__ part, int N, int HW, float* __restrict__ terms,
                                     float* __restrict__ loss) {
  constexpr int NV = 3 * K + 1;
  // one thread per (n, value), fixed summation order over chunks
  __shared__ double acc[64][NV];
  double ce = 0.0, dsum = 0.0;
  for (int base = 0; base < N; base += 64) {
    const int n = base + (int)threadIdx.x;
    if (threadIdx.x < 64) {
      for (int i = 0; i < NV; ++i) {
        double a = 0.0;
        if (n < N)
          for (int c = 0; c < LCHUNK; ++c) a += part[((size_t)n * LCHUNK + c) * NV + i];
        acc[threadIdx.x][i] = a;
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int r = 0; r < 64 && base + r < N; ++r) {
        for (int k = 0; k < K; ++k) {
          const double I = acc[r][3 * k], S = acc[r][3 * k + 1] + acc[r][3 * k + 2];
          const float If = (float)I, Sf = (float)S;
          const float setsum = Sf == 0.f ? 2.f * If : Sf;
          dsum += (double)((2.f * If + DICE_EPS) / (setsum + DICE_EPS));
          terms[((size_t)(base + r) * K + k) * 3 + 0] = If;
          terms[((size_t)(base + r) * K + k) * 3 + 1] = (float)acc[r][3 * k + 1];
          terms[((size_t)(base + r) * K + k) * 3 + 2] = (float)acc[r][3 * k + 2];
        }
        ce += acc[r][3 * K];
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    terms[(size_t)N * K * 3] = (float)ce;
    loss[0] = (float)(ce / ((double)N * HW) + 1.0 - dsum / ((double)N * K));
  }
}

template <int K>
__global__ void loss_bwd_kernel(const float* __restrict__ logits, const int64_t* __restrict__ target, int N, int HW,
                                const float* __restrict__ terms, const float* __restrict__ grad_out,
                                float* __restrict__ dlogits) {
  const long P = (long)N * HW;
  const float go = grad_out ? grad_out[0] : 1.f;
  const float inv_pix = 1.f / (float)P;
  const float dscale = -1.f / (float)(K * N);
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < P; i += (long)gridDim.x * NT) {
    const long n = i / HW, hw = i - n * HW;
    float z[K], mx = -INFINITY;
#pragma unroll
    for (int k = 0; k < K; ++k) { z[k] = logits[(n * K + k) * HW + hw]; mx = fmaxf(mx, z[k]); }
    float se = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) { z[k] = expf(z[k] - mx); se += z[k]; }
    const int t = (int)target[i];
    float p[K], G[K], pg = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      p[k] = z[k] / se;
      const float I = terms[(n * K + k) * 3], S = terms[(n * K + k) * 3 + 1] + terms[(n * K + k) * 3 + 2];
      const float tk = t == k ? 1.f : 0.f;
      float dd = 0.f;
      if (S != 0.f) {
        const float den = S + DICE_EPS;
        dd = 2.f * tk / den - (2.f * I + DICE_EPS) / (den * den);
      }
      G[k] = dscale * dd;
      pg += p[k] * G[k];
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const float tk = t == k ? 1.f : 0.f;
      dlogits[(n * K + k) * HW + hw] = go * ((p[k] - tk) * inv_pix + p[k] * (G[k] - pg));
    }
  }
}

// column sums of partial[tiles][C]: columns < split go to out[c], the rest to out2[c - split]
__global__ void sum_tiles_kernel(const float* __restrict__ partial, int tiles, int C, int split,
                                 float* __restrict__ out, float* __restrict__ out2) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s = 0.0;
  for (int t = 0; t < tiles; ++t) s += partial[(size_t)t * C + c];
  if (c < split) out[c] = (float)s;
  else out2[c - split] = (float)s;
}

bool head_ok(int C) { return C % 8 == 0 && C / 8 <= 64 && 64 % (C / 8) == 0; }

}  // namespace

#define STF_KDISPATCH(K_, EXPR)             \
  switch (K_) {                             \
    case 1: { constexpr int KK = 1; EXPR; } break; \
    case 2: { constexpr int KK = 2; EXPR; } break; \
    case 3: { constexpr int KK = 3; EXPR; } break; \
    case 4: { constexpr int KK = 4; EXPR; } break; \
    default: return STF_EINVAL;             \
  }

extern "C" int stf_head_tiles(int N, int H, int W, int C) { return head_tiles((long)N * H * W * (C / 8)); }

extern "C" int stf_head_fwd(const void* y, int N, int H, int W, int C, const float* scale, const float* shift,
                            const float* w, const float* bias, int classes, float* logits, stf_stream_t stream) {
  if (!head_ok(C)) return STF_EINVAL;
  const long P = (long)N * H * W, units = P * (C / 8);
  if (units >= (1L << 31)) return STF_EINVAL;
  long blocks = (units + NT - 1) / NT;
  if (blocks > 8192) blocks = 8192;
  hipStream_t s = (hipStream_t)stream;
  STF_KDISPATCH(classes, hipLaunchKernelGGL(head_fwd_kernel<KK>, dim3(blocks), dim3(NT), 0, s, (const uint16_t*)y,
                                            P, H * W, C, scale, shift, w, bias, logits));
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_head_bwd(const float* dlogits, const void* y, int N, int H, int W, int C, const float* scale,
                            const float* shift, const float* mean, const float* invstd, const float* w, int classes,
                            void* g_out, float* bn_partial, float* head_partial, float* dw, float* db,
                            stf_stream_t stream) {
  if (!head_ok(C) || (long)N * H * W * (C / 8) >= (1L << 31)) return STF_EINVAL;
  const long P = (long)N * H * W;
  const int tiles = stf_head_tiles(N, H, W, C);
  hipStream_t s = (hipStream_t)stream;
  STF_KDISPATCH(classes, hipLaunchKernelGGL(head_bwd_kernel<KK>, dim3(tiles), dim3(NT), 0, s, dlogits,
                                            (const uint16_t*)y, P, H * W, C, scale, shift, mean, invstd, w,
                                            (uint16_t*)g_out, bn_partial, head_partial));
  STF_CHECK_LAUNCH();
  const int HC = classes * (C + 1);
  // reduce [tiles][K*(C+1)] straight into dw[K*C] and db[K]
  const int S = stf::colsum_stage1(head_partial, tiles, HC, s);
  hipLaunchKernelGGL(sum_tiles_kernel, dim3((HC + 255) / 256), dim3(256), 0, s, head_partial, S, HC, classes * C,
                     dw, db);
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_loss_scratch_floats(int N, int classes) {
  return N * classes * 3 + 1 + N * LCHUNK * (3 * classes + 1);
}

extern "C" int stf_loss_fwd(const float* logits, const int64_t* target, int N, int H, int W, int classes,
                            float* terms, float* loss, stf_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  float* part = terms + N * classes * 3 + 1;
  STF_KDISPATCH(classes, {
    hipLaunchKernelGGL(loss_fwd_kernel<KK>, dim3(LCHUNK, N), dim3(NT), 0, s, logits, target, H * W, part);
    hipLaunchKernelGGL(loss_finalize_kernel<KK>, dim3(1), dim3(64), 0, s, part, N, H * W, terms, loss);
  });
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_loss_bwd(const float* logits, const int64_t* target, int N, int H, int W, int classes,
                            const float* terms, const float* grad_out, float* dlogits, stf_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  const long P = (long)N * H * W;
  long blocks = (P + NT - 1) / NT;
  if (blocks > 8192) blocks = 8192;
  STF_KDISPATCH(classes, hipLaunchKernelGGL(loss_bwd_kernel<KK>, dim3(blocks), dim3(NT), 0, s, logits, target, N,
                                            H * W, terms, grad_out, dlogits));
  STF_CHECK_LAUNCH();
  return 0;
}
