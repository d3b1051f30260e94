// Convolution weight gradient on MFMA (gfx950), split-K over pixels.
//
//   dW[n][r][s][c] = sum_m dy[m][n] * x[gather(m, r, s)][c]
//
// GEMM with M = dy channels (n), N = x channels of one tap (c), K = pixels.
// Both operands arrive NHWC (channel-contiguous), i.e. K-strided, so tiles are
// staged in LDS as [pixel][channel] rows and the MFMA fragments (8 consecutive
// pixels of one channel per lane) are read with ds_read_b64_tr_b16 (two 4-row
// transposed reads per fragment).  Rows are padded by 32 B so the eight rows a
// 32-lane half touches land on disjoint bank octets.
// Each block owns (n-tile, tap, c-tile, pixel split) and writes an fp32 partial
// slab; stf_wgrad_reduce sums the slabs in a fixed order (deterministic).
#include "common.h"
#include "../../include/stfunet.h"
#include "reduce.h"

namespace {

constexpr int NT = 256;
typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

struct WArgs {
  const uint16_t* dy; const uint16_t* x; float* ws;
  int N, Hs, Ws, Cs, xcs, Hd, Wd, R, S, st, pad, M, Nout, dycs, chunk;
};

template <int BM, int BN, int BKP, bool GENERAL>
__global__ __launch_bounds__(NT, 2) void wgrad_kernel(WArgs a) {
  constexpr int PAD = 16;                       // elements (32 B)
  constexpr int SA = BM + PAD, SB = BN + PAD;   // LDS row strides (elements)
  constexpr int WTM = BM / 2, WTN = BN / 2, TM = WTM / 16, TN = WTN / 16;
  constexpr int CPA = BM / 8, CPB = BN / 8;     // 16-B chunks per pixel row
  constexpr int CHA = BKP * CPA / NT, CHB = BKP * CPB / NT;
  static_assert(CHA >= 1 && CHB >= 1, "tile");
  __shared__ __attribute__((aligned(16))) uint16_t smem[2][BKP * (SA + SB)];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int split = blockIdx.x;
  const int n0 = blockIdx.y * BM;
  const int RSC = a.R * a.S * a.Cs;
  const int kb = blockIdx.z * BN;               // first column of this block in [0, RSC)
  // non-GENERAL (Cs % BN == 0): the whole column block lies inside one tap
  const int tap = kb / a.Cs, c0 = kb - tap * a.Cs;
  const int tr = tap / a.S, ts = tap - tr * a.S;
  const int p_begin = split * a.chunk;
  const int p_end = min(a.M, p_begin + a.chunk);
  const int hw = a.Hd * a.Wd;

  uint4 ra[CHA], rb[CHB];
  auto load = [&](int p0) {
#pragma unroll
    for (int i = 0; i < CHA; ++i) {
      const int e = tid + i * NT, row = e / CPA, ch = e - row * CPA;
      const int m = p0 + row;
      const int n = n0 + ch * 8;
      ra[i] = make_uint4(0, 0, 0, 0);
      if (m < p_end && n < a.Nout) ra[i] = *reinterpret_cast<const uint4*>(a.dy + (size_t)m * a.dycs + n);
    }
#pragma unroll
    for (int i = 0; i < CHB; ++i) {
      const int e = tid + i * NT, row = e / CPB, ch = e - row * CPB;
      const int m = p0 + row;
      int r_ = tr, s_ = ts, c_ = c0 + ch * 8;
      bool kok = true;
      if (GENERAL) {
        const int k = kb + ch * 8;
        kok = k < RSC;
        const int t = k / a.Cs;
        c_ = k - t * a.Cs; r_ = t / a.S; s_ = t - r_ * a.S;
      }
      rb[i] = make_uint4(0, 0, 0, 0);
      if (m < p_end && kok) {
        const int n = m / hw, rem = m - n * hw;
        const int yd = rem / a.Wd, xd = rem - yd * a.Wd;
        const int ys = yd * a.st - a.pad + r_, xs = xd * a.st - a.pad + s_;
        if (ys >= 0 && xs >= 0 && ys < a.Hs && xs < a.Ws)
          rb[i] = *reinterpret_cast<const uint4*>(a.x + (size_t)((n * a.Hs + ys) * a.Ws + xs) * a.xcs + c_);
      }
    }
  };
  auto store = [&](int buf) {
    uint16_t* sa = smem[buf];
    uint16_t* sb = sa + BKP * SA;
#pragma unroll
    for (int i = 0; i < CHA; ++i) {
      const int e = tid + i * NT, row = e / CPA, ch = e - row * CPA;
      *reinterpret_cast<uint4*>(sa + row * SA + ch * 8) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < CHB; ++i) {
      const int e = tid + i * NT, row = e / CPB, ch = e - row * CPB;
      *reinterpret_cast<uint4*>(sb + row * SB + ch * 8) = rb[i];
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transposed-read lane geometry: lane 4q+p of each 16-lane group addresses
  // row q (+4 for the second read) and columns 4p..4p+3 of the 16-column block.
  const int g = lane >> 4, q = (lane >> 2) & 3, p4 = (lane & 3) * 4;

  const int steps = (p_end - p_begin + BKP - 1) / BKP;
  if (steps > 0) { load(p_begin); store(0); }
  __syncthreads();
  for (int it = 0; it < steps; ++it) {
    const int cur = it & 1;
    if (it + 1 < steps) load(p_begin + (it + 1) * BKP);
    const uint16_t* sa = smem[cur];
    const uint16_t* sb = sa + BKP * SA;
#pragma unroll
    for (int kk = 0; kk < BKP; kk += 32) {
      bf16x8 af[TM], bfr[TN];
      const int krow = kk + 8 * g + q;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int col = wm * WTM + i * 16 + p4;
        v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(sa + krow * SA + col));
        v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(sa + (krow + 4) * SA + col));
        short s8[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[i] = __builtin_bit_cast(bf16x8, s8);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn * WTN + j * 16 + p4;
        v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(sb + krow * SB + col));
        v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(sb + (krow + 4) * SB + col));
        short s8[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bfr[j] = __builtin_bit_cast(bf16x8, s8);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (it + 1 < steps) store(cur ^ 1);
    __syncthreads();
  }

  // D[row = dy channel][col = x channel]: col = lane&15, rows (lane>>4)*4 + r
  float* out = a.ws + (size_t)split * a.Nout * RSC;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int k = kb + wn * WTN + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wm * WTM + i * 16 + (lane >> 4) * 4 + r;
        if (n < a.Nout && k < RSC) out[(size_t)n * RSC + k] = acc[i][j][r];
      }
    }
}

__global__ void wgrad_reduce_kernel(const float* __restrict__ ws, int splits, int Nout, int R, int S,
                                    int Cs, float* __restrict__ out) {
  const int RSC = R * S * Cs;
  const size_t total = (size_t)Nout * RSC;
  for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < total;
       idx += (size_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < splits; ++k) s += ws[(size_t)k * total + idx];
    const int n = idx / RSC, rem = idx - (size_t)n * RSC;
    const int tap = rem / Cs, c = rem - tap * Cs;
    out[((size_t)n * Cs + c) * (R * S) + tap] = s;
  }
}

bool big_tile(const stf_wgrad_args* a) { return a->Nout % 128 == 0 && a->g.Cs % 128 == 0; }

void plan(const stf_wgrad_args* a, int& splits, int& chunk) {
  const int M = a->g.N * a->g.Hd * a->g.Wd;
  const int bm = big_tile(a) ? 128 : 64, bkp = big_tile(a) ? 32 : 64;
  const long rsc = (long)a->g.R * a->g.S * a->g.Cs;
  const long tiles = (long)((a->Nout + bm - 1) / bm) * ((rsc + bm - 1) / bm);
  long want = (2048 + tiles - 1) / tiles;
  long maxs = (M + 4 * bkp - 1) / (4 * bkp);        // at least 4 K steps per split
  if (want > maxs) want = maxs;
  if (want < 1) want = 1;
  chunk = (int)(((M + want - 1) / want + bkp - 1) / bkp * bkp);
  splits = (M + chunk - 1) / chunk;
}

}  // namespace

extern "C" int stf_wgrad_plan(const stf_wgrad_args* a, int* splits, size_t* ws_bytes) {
  int s, chunk;
  plan(a, s, chunk);
  if (splits) *splits = s;
  if (ws_bytes) *ws_bytes = (size_t)s * a->Nout * a->g.R * a->g.S * a->g.Cs * sizeof(float);
  return 0;
}

extern "C" int stf_wgrad(const stf_wgrad_args* a, stf_stream_t stream) {
  const stf_conv_geom& c = a->g;
  if (c.transposed || a->Nout % 8 || c.Cs % 8 || a->dy_cstride % 8 || c.src_cstride % 8) return STF_EINVAL;
  if (((uintptr_t)a->dy & 15) || ((uintptr_t)a->x & 15)) return STF_EINVAL;
  int splits, chunk;
  plan(a, splits, chunk);
  if (a->splits != splits) return STF_EINVAL;
  WArgs w;
  w.dy = (const uint16_t*)a->dy; w.x = (const uint16_t*)a->x; w.ws = a->ws;
  w.N = c.N; w.Hs = c.Hs; w.Ws = c.Ws; w.Cs = c.Cs; w.xcs = c.src_cstride; w.Hd = c.Hd; w.Wd = c.Wd;
  w.R = c.R; w.S = c.S; w.st = c.stride; w.pad = c.pad; w.M = c.N * c.Hd * c.Wd; w.Nout = a->Nout;
  w.dycs = a->dy_cstride; w.chunk = chunk;
  hipStream_t s = (hipStream_t)stream;
  const int rsc = c.R * c.S * c.Cs;
  if (big_tile(a)) {
    dim3 grid(splits, a->Nout / 128, rsc / 128);
    hipLaunchKernelGGL((wgrad_kernel<128, 128, 32, false>), grid, dim3(NT), 0, s, w);
  } else if (c.Cs % 64 == 0) {
    dim3 grid(splits, (a->Nout + 63) / 64, rsc / 64);
    hipLaunchKernelGGL((wgrad_kernel<64, 64, 64, false>), grid, dim3(NT), 0, s, w);
  } else {
    dim3 grid(splits, (a->Nout + 63) / 64, (rsc + 63) / 64);
    hipLaunchKernelGGL((wgrad_kernel<64, 64, 64, true>), grid, dim3(NT), 0, s, w);
  }
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_wgrad_reduce(float* ws, int splits, int Nout, int R, int S, int Cs, float* out,
                                stf_stream_t stream) {
  const size_t total = (size_t)Nout * R * S * Cs;
  const int blocks = (int)std::min<size_t>((total + 255) / 256, 4096);
  const int rows = stf::colsum_stage1(ws, splits, (long)total, (hipStream_t)stream);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, ws, rows, Nout,
                     R, S, Cs, out);
  STF_CHECK_LAUNCH();
  return 0;
}
