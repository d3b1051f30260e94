// Whole-sequence nn.LSTM(C, C) over T steps for every pixel, one launch
// (src/stf_lstm_unet.py:124-127,214-242; gate order i, f, g, o; only h_T is used).
//
// The per-pixel LSTM is independent across pixels, so a workgroup can own 64 pixels
// for ALL T steps: the cell state c stays in registers, h_{t-1} in LDS, and the
// gate weights [W_ih | W_hh] (gate-interleaved rows, stf_lstm_pack) are loaded into
// registers once.  Per step only x_t comes in from HBM and c_t / h_t go out (for the
// backward's gate recompute), instead of one GEMM launch per step that also re-reads
// c_{t-1} and h_{t-1} (stf_igemm with the LSTM epilogue).  The step GEMM is the same
// MFMA sequence as that launch (weights as the A operand, K ascending, x then h), so
// c_t / h_t are bit-identical to the per-step path and the backward may recompute
// the gates with either.
//
// Layout: lbuf rows of step t = [x_t | h_{t-1}] (2C channels, P pixels per step, the
// encoder writes x_t; this kernel writes h_t into step t+1's h slot and h_{T-1}
// into hT); cst [T][P][C] fp32.  Workgroup = 4 waves; wave w owns gate rows
// [w C, (w+1) C) (hidden channels [w C/4, (w+1) C/4)) of all 64 pixels.
#include "common.h"
#include "../../include/stfunet.h"
#include <stdlib.h>

namespace {

constexpr int NT = 256, BM = 64;

template <int C, int OCC>
__global__ __launch_bounds__(NT, OCC) void lstm_seq_fwd_kernel(const uint16_t* __restrict__ wcat,
                                                            const float* __restrict__ bias, uint16_t* lbuf, int P,
                                                            int T, float* __restrict__ cst, uint16_t* hT, int hTcs) {
  constexpr int KS = 2 * C / 32;          // k-steps of 32 (x: the first C / 32)
  constexpr int NF = C / 16;              // n-fragments per wave (C gate rows)
  constexpr int MF = BM / 16;             // m-fragments (pixels)
  constexpr int CPR = C / 8;              // 16-B chunks per LDS row (C channels)
  constexpr int XCH = BM * CPR / NT;      // x chunks per thread per step
  static_assert(C % 32 == 0 && XCH >= 1 && BM * CPR % NT == 0, "shape");
  __shared__ __attribute__((aligned(16))) uint16_t xs[2][BM * C];
  __shared__ __attribute__((aligned(16))) uint16_t hs[2][BM * C];
  __shared__ __attribute__((aligned(16))) float cs[2][BM * C];   // c_t tile, leaves as whole rows

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fk = lane >> 4;
  const int m0 = blockIdx.x * BM;
  const int rows = min(BM, P - m0);
  const int lcs = 2 * C;
  const bool hvec = ((reinterpret_cast<uintptr_t>(hT) & 15) == 0) && (hTcs & 7) == 0;
  // LDS image: row r (pixel), 16-B chunk q at q ^ (r & 7) (conflict-free fragment reads)
  auto soff = [&](int r, int q) { return r * C + ((q ^ (r & 7)) << 3); };

  // weights (A operand) and bias, kept for all T steps
  e16x8 wf[NF][KS];
  float bv[NF][4];
#pragma unroll
  for (int nf = 0; nf < NF; ++nf) {
    const int n = wave * C + nf * 16 + fr;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      wf[nf][ks] = *reinterpret_cast<const e16x8*>(wcat + (size_t)n * lcs + ks * 32 + fk * 8);
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[nf][r] = bias[wave * C + nf * 16 + fk * 4 + r];
  }

  uint4 rx[XCH];
  auto load_x = [&](int t) {
#pragma unroll
    for (int i = 0; i < XCH; ++i) {
      const int e = tid + i * NT, r = e / CPR, q = e - r * CPR;
      rx[i] = r < rows ? *reinterpret_cast<const uint4*>(lbuf + ((size_t)t * P + m0 + r) * lcs + q * 8)
                       : make_uint4(0, 0, 0, 0);
    }
  };
  auto store_x = [&](int buf) {
#pragma unroll
    for (int i = 0; i < XCH; ++i) {
      const int e = tid + i * NT, r = e / CPR, q = e - r * CPR;
      *reinterpret_cast<uint4*>(&xs[buf][soff(r, q)]) = rx[i];
    }
  };
  for (int e = tid; e < BM * CPR; e += NT) {                  // h_{-1} = 0
    const int r = e / CPR, q = e - r * CPR;
    *reinterpret_cast<uint4*>(&hs[0][soff(r, q)]) = make_uint4(0, 0, 0, 0);
  }
  load_x(0);
  store_x(0);
  __syncthreads();

  float cc[MF][NF];                                             // cell state of this lane's cells
#pragma unroll
  for (int mf = 0; mf < MF; ++mf)
#pragma unroll
    for (int nf = 0; nf < NF; ++nf) cc[mf][nf] = 0.f;

  for (int t = 0; t < T; ++t) {
    const int cur = t & 1;
    if (t + 1 < T) load_x(t + 1);
    f32x4 acc[MF][NF];
#pragma unroll
    for (int mf = 0; mf < MF; ++mf)
#pragma unroll
      for (int nf = 0; nf < NF; ++nf) acc[mf][nf] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const bool isx = ks < KS / 2;
      const uint16_t* src = isx ? xs[cur] : hs[cur];
      const int q = (ks % (KS / 2)) * 4 + fk;                    // 16-B chunk of this lane's 8 k
      e16x8 bf[MF];
#pragma unroll
      for (int mf = 0; mf < MF; ++mf) {
        const int r = mf * 16 + fr;
        bf[mf] = *reinterpret_cast<const e16x8*>(src + soff(r, q));
      }
#pragma unroll
      for (int mf = 0; mf < MF; ++mf)
#pragma unroll
        for (int nf = 0; nf < NF; ++nf) acc[mf][nf] = mfma16x16x32(wf[nf][ks], bf[mf], acc[mf][nf]);
    }
    // cell update: lane holds the 4 gates of hidden channel ch of pixel r
#pragma unroll
    for (int mf = 0; mf < MF; ++mf) {
      const int r = mf * 16 + fr, m = m0 + r;
#pragma unroll
      for (int nf = 0; nf < NF; ++nf) {
        const int ch = wave * (C / 4) + nf * 4 + fk;
        float gi, gf, gg, go, c, hh;
        lstm_cell_fwd(acc[mf][nf][0] + bv[nf][0], acc[mf][nf][1] + bv[nf][1], acc[mf][nf][2] + bv[nf][2],
                      acc[mf][nf][3] + bv[nf][3], cc[mf][nf], gi, gf, gg, go, c, hh);
        cc[mf][nf] = c;
        reinterpret_cast<e16*>(hs[cur ^ 1])[soff(r, ch >> 3) + (ch & 7)] = f2e(hh);
        cs[cur][r * C + ((((ch >> 2) ^ (r & 7)) << 2) | (ch & 3))] = c;
      }
    }
    if (t + 1 < T) store_x(cur ^ 1);
    __syncthreads();
    // c_t and h_t leave as whole 16-B row chunks (the next step only reads hs / xs)
    const bool last = t + 1 == T;
    for (int e = tid; e < rows * (C / 4); e += NT) {
      const int r = e / (C / 4), q = e - r * (C / 4);
      *reinterpret_cast<float4*>(cst + ((size_t)t * P + m0 + r) * C + q * 4) =
          *reinterpret_cast<const float4*>(&cs[cur][r * C + ((q ^ (r & 7)) << 2)]);
    }
    for (int e = tid; e < rows * CPR; e += NT) {
      const int r = e / CPR, q = e - r * CPR;
      const uint4 v = *reinterpret_cast<const uint4*>(&hs[cur ^ 1][soff(r, q)]);
      uint16_t* dst = last ? hT + (size_t)(m0 + r) * hTcs + q * 8 : lbuf + ((size_t)(t + 1) * P + m0 + r) * lcs + C + q * 8;
      if (!last || hvec) *reinterpret_cast<uint4*>(dst) = v;
      else {
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        for (int k = 0; k < 8; ++k) dst[k] = (uint16_t)(w[k >> 1] >> ((k & 1) * 16));
      }
    }
  }
}

// Backward through all T steps (t = T-1 .. 0) for 64 pixels per workgroup, one launch:
//   1. the step's gate pre-activations are recomputed: [x_t | h_{t-1}] (lbuf rows t) x W
//      (weights in registers, the forward's MFMA sequence: bitwise the forward's gates);
//   2. cell backward (dc in registers): tc = tanh c_t, dc = dh o (1-tc^2) + dc,
//      pre-activation gradients (di, df, dg, do) -> 16-bit dgates (LDS + rows of dg for
//      the weight gradient afterwards), dc <- dc f;
//   3. [dx_t | dh_{t-1}] = dgates x W (W^T rows in registers as the A operand): dx_t
//      rows -> dxh (channels [0, C) of rows t), dh_{t-1} stays in LDS for step t-1.
// Same arithmetic and roundings as the per-step path (stf_igemm with the LSTM
// backward epilogue, then the dgates x W^T GEMM, which stores dh_{t-1} in 16 bits).
// One workgroup per CU (weights + transposed weights + two accumulator sets exceed a
// 2-wave register budget); the next step's [x | h] rows and c_{t-2} are prefetched
// into registers behind the step's MFMAs.
template <int C>
__global__ __launch_bounds__(NT, 1) void lstm_seq_bwd_kernel(const uint16_t* __restrict__ wcat,
                                                            const uint16_t* __restrict__ wcat_t,
                                                            const float* __restrict__ bias, const uint16_t* lbuf,
                                                            int P, int T, const float* __restrict__ cst,
                                                            const uint16_t* __restrict__ dhT, int dhcs,
                                                            uint16_t* __restrict__ dg, uint16_t* __restrict__ dxh,
                                                            int dxcs) {
  constexpr int K1 = 2 * C / 32, K2 = 4 * C / 32;   // k-steps of GEMM1 (x|h) and GEMM2 (gates)
  constexpr int NF1 = C / 16;                       // GEMM1 n-fragments per wave (C gate rows)
  constexpr int NF2 = 2 * C / 4 / 16;               // GEMM2 n-fragments per wave (2C/4 rows of [dx|dh])
  constexpr int MF = BM / 16;
  constexpr int R1 = 2 * C / 8, RC = C / 4, RG = 4 * C / 8, RH = C / 8;   // 16-B chunks per row
  constexpr int XCH = BM * R1 / NT, CCH = BM * RC / NT;
  static_assert(C == 64 && XCH >= 1 && CCH >= 1 && NF2 >= 1, "shape");
  __shared__ __attribute__((aligned(16))) uint16_t xh[2][BM * 2 * C];    // [x_t | h_{t-1}] rows
  __shared__ __attribute__((aligned(16))) float cb[3][BM * C];           // c tiles (rotating)
  __shared__ __attribute__((aligned(16))) uint16_t dhs[BM * C];          // dh_t
  __shared__ __attribute__((aligned(16))) uint16_t dgs[BM * 4 * C];      // dgates
  __shared__ __attribute__((aligned(16))) uint16_t dxs[BM * C];          // dx_t staging

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fk = lane >> 4;
  const int m0 = blockIdx.x * BM;
  const int rows = min(BM, P - m0);
  const int lcs = 2 * C;
  // 16-bit rows of W16 chunks: chunk q at q ^ (r & 15); fp32 c rows of RC chunks: q ^ (r & 7)
  auto o16 = [&](int r, int q, int w16) { return r * w16 * 8 + ((q ^ (r & 15)) << 3); };
  auto o32 = [&](int r, int q) { return r * C + ((q ^ (r & 7)) << 2); };

  e16x8 w1[NF1][K1], w2[NF2][K2];
  float bv[NF1][4];
#pragma unroll
  for (int nf = 0; nf < NF1; ++nf) {
    const int n = wave * C + nf * 16 + fr;
#pragma unroll
    for (int ks = 0; ks < K1; ++ks)
      w1[nf][ks] = *reinterpret_cast<const e16x8*>(wcat + (size_t)n * lcs + ks * 32 + fk * 8);
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[nf][r] = bias[wave * C + nf * 16 + fk * 4 + r];
  }
#pragma unroll
  for (int nf = 0; nf < NF2; ++nf) {
    const int o = wave * (2 * C / 4) + nf * 16 + fr;
#pragma unroll
    for (int ks = 0; ks < K2; ++ks)
      w2[nf][ks] = *reinterpret_cast<const e16x8*>(wcat_t + (size_t)o * 4 * C + ks * 32 + fk * 8);
  }

  uint4 rx[XCH];
  float4 rc[CCH];
  auto load_xh = [&](int t) {
#pragma unroll
    for (int i = 0; i < XCH; ++i) {
      const int e = tid + i * NT, r = e / R1, q = e - r * R1;
      rx[i] = r < rows ? *reinterpret_cast<const uint4*>(lbuf + ((size_t)t * P + m0 + r) * lcs + q * 8)
                       : make_uint4(0, 0, 0, 0);
    }
  };
  auto store_xh = [&](int buf) {
#pragma unroll
    for (int i = 0; i < XCH; ++i) {
      const int e = tid + i * NT, r = e / R1, q = e - r * R1;
      *reinterpret_cast<uint4*>(&xh[buf][o16(r, q, R1)]) = rx[i];
    }
  };
  auto load_c = [&](int t) {                          // t < 0: the zero initial state
#pragma unroll
    for (int i = 0; i < CCH; ++i) {
      const int e = tid + i * NT, r = e / RC, q = e - r * RC;
      rc[i] = (t >= 0 && r < rows) ? *reinterpret_cast<const float4*>(cst + ((size_t)t * P + m0 + r) * C + q * 4)
                                   : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store_c = [&](int buf) {
#pragma unroll
    for (int i = 0; i < CCH; ++i) {
      const int e = tid + i * NT, r = e / RC, q = e - r * RC;
      *reinterpret_cast<float4*>(&cb[buf][o32(r, q)]) = rc[i];
    }
  };

  // prologue: rows T-1, c_{T-1}, c_{T-2}, dh_{T-1} = dhT
  load_xh(T - 1);
  store_xh((T - 1) & 1);
  load_c(T - 1);
  store_c((T - 1) % 3);
  load_c(T - 2);
  store_c((T + 1) % 3);
  const bool dvec = ((reinterpret_cast<uintptr_t>(dhT) & 15) == 0) && (dhcs & 7) == 0;
  for (int e = tid; e < BM * RH; e += NT) {
    const int r = e / RH, q = e - r * RH;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r < rows) {
      const uint16_t* src = dhT + (size_t)(m0 + r) * dhcs + q * 8;
      if (dvec) v = *reinterpret_cast<const uint4*>(src);
      else
        v = make_uint4(src[0] | ((uint32_t)src[1] << 16), src[2] | ((uint32_t)src[3] << 16),
                       src[4] | ((uint32_t)src[5] << 16), src[6] | ((uint32_t)src[7] << 16));
    }
    *reinterpret_cast<uint4*>(&dhs[r * C + ((q ^ (r & 7)) << 3)]) = v;
  }
  __syncthreads();

  float dc[MF][NF1];
#pragma unroll
  for (int mf = 0; mf < MF; ++mf)
#pragma unroll
    for (int nf = 0; nf < NF1; ++nf) dc[mf][nf] = 0.f;

  for (int t = T - 1; t >= 0; --t) {
    const int xb = t & 1;
    const float* ct = cb[t % 3];
    const float* cp = cb[(t + 2) % 3];                 // c_{t-1} (zeros at t = 0)
    if (t > 0) { load_xh(t - 1); load_c(t - 2); }
    // 1. gates of step t
    f32x4 acc[MF][NF1];
#pragma unroll
    for (int mf = 0; mf < MF; ++mf)
#pragma unroll
      for (int nf = 0; nf < NF1; ++nf) acc[mf][nf] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < K1; ++ks) {
      e16x8 bf[MF];
#pragma unroll
      for (int mf = 0; mf < MF; ++mf)
        bf[mf] = *reinterpret_cast<const e16x8*>(&xh[xb][o16(mf * 16 + fr, ks * 4 + fk, R1)]);
#pragma unroll
      for (int mf = 0; mf < MF; ++mf)
#pragma unroll
        for (int nf = 0; nf < NF1; ++nf) acc[mf][nf] = mfma16x16x32(w1[nf][ks], bf[mf], acc[mf][nf]);
    }
    // 2. cell backward
#pragma unroll
    for (int mf = 0; mf < MF; ++mf) {
      const int r = mf * 16 + fr;
#pragma unroll
      for (int nf = 0; nf < NF1; ++nf) {
        const int ch = wave * (C / 4) + nf * 4 + fk;
        float gi, gf, gg, go, cx, hx;
        lstm_cell_fwd(acc[mf][nf][0] + bv[nf][0], acc[mf][nf][1] + bv[nf][1], acc[mf][nf][2] + bv[nf][2],
                      acc[mf][nf][3] + bv[nf][3], 0.f, gi, gf, gg, go, cx, hx);
        const int co = r * C + ((((ch >> 2) ^ (r & 7)) << 2) | (ch & 3));
        const float h = e2f(reinterpret_cast<const e16*>(dhs)[r * C + ((((ch >> 3) ^ (r & 7))) << 3) + (ch & 7)]);
        float d_i, d_f, d_g, d_o, dcp;
        lstm_cell_bwd(gi, gf, gg, go, ct[co], cp[co], h, dc[mf][nf], d_i, d_f, d_g, d_o, dcp);
        dc[mf][nf] = dcp;
        // gate row 4ch+q of pixel r: 16-B chunk (ch >> 1) of the 4C-wide row, slot (ch & 1) * 4
        *reinterpret_cast<uint2*>(&dgs[o16(r, ch >> 1, RG) + (ch & 1) * 4]) =
            make_uint2(pack2(d_i, d_f), pack2(d_g, d_o));
      }
    }
    __syncthreads();
    // dgates rows of step t -> dg (the weight gradient reads them afterwards)
    for (int e = tid; e < rows * RG; e += NT) {
      const int r = e / RG, q = e - r * RG;
      *reinterpret_cast<uint4*>(dg + ((size_t)t * P + m0 + r) * 4 * C + q * 8) =
          *reinterpret_cast<const uint4*>(&dgs[o16(r, q, RG)]);
    }
    // 3. [dx_t | dh_{t-1}] = dgates x W
    f32x4 a2[MF][NF2];
#pragma unroll
    for (int mf = 0; mf < MF; ++mf)
#pragma unroll
      for (int nf = 0; nf < NF2; ++nf) a2[mf][nf] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < K2; ++ks) {
      e16x8 bf[MF];
#pragma unroll
      for (int mf = 0; mf < MF; ++mf)
        bf[mf] = *reinterpret_cast<const e16x8*>(&dgs[o16(mf * 16 + fr, ks * 4 + fk, RG)]);
#pragma unroll
      for (int mf = 0; mf < MF; ++mf)
#pragma unroll
        for (int nf = 0; nf < NF2; ++nf) a2[mf][nf] = mfma16x16x32(w2[nf][ks], bf[mf], a2[mf][nf]);
    }
#pragma unroll
    for (int mf = 0; mf < MF; ++mf) {
      const int r = mf * 16 + fr;
#pragma unroll
      for (int nf = 0; nf < NF2; ++nf) {
        const int o = wave * (2 * C / 4) + nf * 16 + fk * 4;     // 4 consecutive output channels
        const uint2 v = make_uint2(pack2(a2[mf][nf][0], a2[mf][nf][1]), pack2(a2[mf][nf][2], a2[mf][nf][3]));
        const int oo = o < C ? o : o - C;
        uint16_t* buf = o < C ? dxs : dhs;
        *reinterpret_cast<uint2*>(&buf[r * C + ((((oo >> 3) ^ (r & 7))) << 3) + (oo & 7)]) = v;
      }
    }
    if (t > 0) { store_xh(xb ^ 1); store_c((t + 1) % 3); }
    __syncthreads();
    for (int e = tid; e < rows * RH; e += NT) {
      const int r = e / RH, q = e - r * RH;
      *reinterpret_cast<uint4*>(dxh + ((size_t)t * P + m0 + r) * dxcs + q * 8) =
          *reinterpret_cast<const uint4*>(&dxs[r * C + ((q ^ (r & 7)) << 3)]);
    }
  }
}

}  // namespace

extern "C" int stf_lstm_seq_bwd(const void* wcat, const void* wcat_t, const float* bias, const void* lbuf, int P,
                                int T, int C, const float* c_all, const void* dh_last, int dh_cstride, void* dgates,
                                void* dx, int dx_cstride, stf_stream_t stream) {
  if (P <= 0 || T <= 0) return 0;
  if (C != 64 || !wcat || !wcat_t || !bias || !lbuf || !c_all || !dh_last || !dgates || !dx || dh_cstride < C ||
      dx_cstride < C || dx_cstride % 8)
    return STF_EINVAL;
  if (((uintptr_t)wcat & 15) || ((uintptr_t)wcat_t & 15) || ((uintptr_t)lbuf & 15) || ((uintptr_t)dgates & 15) ||
      ((uintptr_t)dx & 15) || ((uintptr_t)c_all & 15))
    return STF_EINVAL;
  hipLaunchKernelGGL((lstm_seq_bwd_kernel<64>), dim3((P + BM - 1) / BM), dim3(NT), 0, (hipStream_t)stream,
                     (const uint16_t*)wcat, (const uint16_t*)wcat_t, bias, (const uint16_t*)lbuf, P, T, c_all,
                     (const uint16_t*)dh_last, dh_cstride, (uint16_t*)dgates, (uint16_t*)dx, dx_cstride);
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_lstm_seq_fwd(const void* wcat, const float* bias, void* lbuf, int P, int T, int C, float* c_out,
                                void* h_last, int h_cstride, stf_stream_t stream) {
  if (P <= 0 || T <= 0) return 0;
  if (C != 64 || !wcat || !bias || !lbuf || !c_out || !h_last || h_cstride < C) return STF_EINVAL;
  if (((uintptr_t)wcat & 15) || ((uintptr_t)lbuf & 15) || ((uintptr_t)c_out & 15)) return STF_EINVAL;
  const dim3 grid((P + BM - 1) / BM);
  hipLaunchKernelGGL((lstm_seq_fwd_kernel<64, 2>), grid, dim3(NT), 0, (hipStream_t)stream, (const uint16_t*)wcat,
                     bias, (uint16_t*)lbuf, P, T, c_out, (uint16_t*)h_last, h_cstride);
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_lstm_seq_supported(int C) { return C == 64; }
