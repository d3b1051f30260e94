// Implicit-GEMM convolution on MFMA (gfx950): forward / dgrad / transposed-conv.
//
// GEMM view: D[n][m] = sum_k W[n][k] * X[m][k]
//   m = destination pixel (N*Hd*Wd rows), n = output channel, k = (r, s, c) over
//   the gathered source tensor (stf_conv_geom in include/stfunet.h).
// The weight tile is the MFMA A operand and the im2col tile the B operand, so
// each lane ends with 4 consecutive *channels* of one pixel: the epilogue packs
// them into one 8-byte store (NHWC), adds bias, and reduces per-channel BatchNorm
// partial sums (sum, sum^2 of the bf16-rounded values) without another pass.
//
// Tiling: 256 threads = 4 waves, BK = 32 (= one v_mfma_f32_16x16x32_bf16 K),
// register-staged global->LDS double buffer, one barrier per K step.  LDS rows
// are 64 B; the 16-B chunk of row r is stored at chunk ^ ((-(r>>2)) & 3), which
// makes the ds_read_b128 fragment reads conflict-free for all four lane groups.
#include "common.h"
#include "../../include/stfunet.h"
#include <stdio.h>
#include <stdlib.h>

namespace {

constexpr int BK = 32;
constexpr int NT = 256;

struct Geo {
  const uint16_t* src; const uint16_t* wgt; uint16_t* dst;
  const float* bias; float* stats;
  int N, Hs, Ws, Cs, scs, Hd, Wd, R, S, st, pad, M, K, Nout, dcs;
  int Mg, tpg;          // rows per statistics group, M tiles per group
  int accumulate;
  // LSTM cell epilogue (Nout = 4*Ch, column 4c+q = gate q of hidden channel c)
  const float* c_prev; float* c_out; uint16_t* h_out; int hcs; float* gates;
  // LSTM cell backward epilogue (EPI 2, gates recomputed): c_out = c_t (read)
  const uint16_t* l_dh; int l_dhcs; const float* l_dcn; float* l_dcp; uint16_t* l_dg;
  // fused BN-backward reduction (stf_bnr_epi)
  const uint16_t* bnr_y; int bnr_ycs; const float *bnr_scale, *bnr_shift, *bnr_mean, *bnr_invstd;
  int bnr_relu; float* bnr_part;
  // stride-2 transposed gather with rows ordered by output parity class (see igemm_dma_kernel)
  int par;
  // split-K (plain DMA kernels): blockIdx.z = K slice, fp32 partials [ksplit][M][Nout] in ws,
  // folded by splitk_reduce_kernel (bias, bf16 store, BN statistics)
  int ksplit; float* ws;
  // halo kernel: keep a ring stage's weight rows across items when they are the rows
  // the next fill needs (same 64-channel output slice and source chunk)
  int wkeep;
  // halo direct epilogue: whole 128-B pixel rows per store instruction (lane exchange fr <-> fr ^ 8)
  int full;
};

STF_DEV int swz(int row, int kc) { return kc ^ ((-(row >> 2)) & 3); }



#ifndef STF_LSTM_STAGED
#define STF_LSTM_STAGED 1
#endif
STF_DEV constexpr bool lstm_staged() { return STF_LSTM_STAGED != 0; }

// Shared epilogue: acc[i][j][r] = pixel mrow[i] (this lane's GEMM row of
// fragment i, -1 = outside the image / tile), channel n0 + wn*WTN + j*16 +
// (lane>>4)*4 + r.  `tile` indexes the BatchNorm partial-statistics row.
template <int BM, int BN, int WM, int WN, bool SCATTER, int EPI, int NTH>
STF_DEV void igemm_epilogue(const Geo& a, f32x4 (&acc)[BM / WM / 16][BN / WN / 16], const int (&mrow)[BM / WM / 16],
                            int n0, int wm, int wn, int tid, char* smem, int tile) {
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  const int lane = tid & 63, fr = lane & 15, fk = lane >> 4;
  const int Cout = SCATTER ? a.Nout / 4 : a.Nout;
  float s1[TN][4], s2[TN][4];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int nb = n0 + wn * WTN + j * 16 + fk * 4;
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (a.bias && nb < a.Nout) {
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[r] = a.bias[SCATTER ? (nb + r) % Cout : nb + r];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) { s1[j][r] = 0.f; s2[j][r] = 0.f; }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = mrow[i];
      if (!(m >= 0 && nb < a.Nout)) continue;
      if (EPI == 1) {
        // LSTM cell (torch gate order i, f, g, o): c = f*c_prev + i*g, h = o*tanh(c)
        const int ch = nb >> 2, Ch = a.Nout >> 2;
        const float cp = a.c_prev ? a.c_prev[(size_t)m * Ch + ch] : 0.f;
        float gi, gf, gg, go, c, hh;
        lstm_cell_fwd(acc[i][j][0] + bv[0], acc[i][j][1] + bv[1], acc[i][j][2] + bv[2], acc[i][j][3] + bv[3], cp,
                      gi, gf, gg, go, c, hh);
        a.c_out[(size_t)m * Ch + ch] = c;
        reinterpret_cast<e16*>(a.h_out)[(size_t)m * a.hcs + ch] = f2e(hh);
        if (a.gates) *reinterpret_cast<float4*>(a.gates + (size_t)m * a.Nout + nb) = make_float4(gi, gf, gg, go);
        continue;
      }
      if (EPI == 2) {
        // LSTM cell backward on the recomputed gates (the forward's arithmetic, same GEMM):
        // dc = dh*o*(1-tanh(c)^2) + dc_next, dc_prev = dc*f, pre-activation gate gradients
        const int ch = nb >> 2, Ch = a.Nout >> 2;
        const size_t u = (size_t)m * Ch + ch;
        float gi, gf, gg, go, cx, hx;
        lstm_cell_fwd(acc[i][j][0] + bv[0], acc[i][j][1] + bv[1], acc[i][j][2] + bv[2], acc[i][j][3] + bv[3], 0.f,
                      gi, gf, gg, go, cx, hx);
        const float h = e2f(reinterpret_cast<const e16*>(a.l_dh)[(size_t)m * a.l_dhcs + ch]);
        const float cp = a.c_prev ? a.c_prev[u] : 0.f;
        float d_i, d_f, d_g, d_o, dcp;
        lstm_cell_bwd(gi, gf, gg, go, a.c_out[u], cp, h, a.l_dcn ? a.l_dcn[u] : 0.f, d_i, d_f, d_g, d_o, dcp);
        a.l_dcp[u] = dcp;
        *reinterpret_cast<uint2*>(a.l_dg + (size_t)m * a.Nout + nb) = make_uint2(pack2(d_i, d_f), pack2(d_g, d_o));
        continue;
      }
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] + bv[r];
      size_t off;
      if (SCATTER) {
        const int blk = nb / Cout, co = nb - blk * Cout;
        const int hw = a.Hd * a.Wd;
        const int n = m / hw, rem = m - n * hw;
        const int yd = rem / a.Wd, xd = rem - yd * a.Wd;
        const int yo = 2 * yd + (blk >> 1), xo = 2 * xd + (blk & 1);
        off = ((size_t)(n * 2 * a.Hd + yo) * (2 * a.Wd) + xo) * a.dcs + co;
      } else {
        off = (size_t)m * a.dcs + nb;
      }
      if (a.accumulate) {
        const uint2 old = *reinterpret_cast<const uint2*>(a.dst + off);
        v[0] += lo16(old.x);
        v[1] += hi16(old.x);
        v[2] += lo16(old.y);
        v[3] += hi16(old.y);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = round_e(v[r]);
      *reinterpret_cast<uint2*>(a.dst + off) = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
#pragma unroll
      for (int r = 0; r < 4; ++r) { s1[j][r] += v[r]; s2[j][r] += v[r] * v[r]; }
    }
  }
  if (EPI != 0 || a.stats == nullptr) return;
  // reduce over the 16 pixels held by lanes with equal fk, then over the WM waves
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        s1[j][r] += __shfl_xor(s1[j][r], o, 64);
        s2[j][r] += __shfl_xor(s2[j][r], o, 64);
      }
  float* red = reinterpret_cast<float*>(smem);     // [WM][2][BN]
  __syncthreads();
  if (fr == 0) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int col = wn * WTN + j * 16 + fk * 4 + r;
        red[(wm * 2 + 0) * BN + col] = s1[j][r];
        red[(wm * 2 + 1) * BN + col] = s2[j][r];
      }
  }
  __syncthreads();
  for (int col = tid; col < BN; col += NTH) {
    const int n = n0 + col;
    if (n >= a.Nout) continue;
    float t1 = 0.f, t2 = 0.f;
#pragma unroll
    for (int w = 0; w < WM; ++w) { t1 += red[(w * 2) * BN + col]; t2 += red[(w * 2 + 1) * BN + col]; }
    a.stats[(size_t)tile * 2 * a.Nout + n] = t1;
    a.stats[(size_t)tile * 2 * a.Nout + a.Nout + n] = t2;
  }
}


// LDS-staged epilogue of the linear DMA kernels (EPI 0): the BM x BN tile goes to
// LDS as bf16(acc + bias) (16-B chunk c of row r at c ^ (r & 7)), then every
// thread stores whole 16-B chunks of output rows (one fixed 8-channel chunk per
// thread: full 128-B+ row segments per wave instead of 8-B pieces of 16 rows),
// adds the old value when accumulating, and sums BN statistics of the stored
// values.  Needs BM*BN*2 + NW*2*BN*4 bytes of LDS (the drained ring).
template <int BM, int BN, int WM, int WN, bool SCATTER, int NTH>
STF_DEV void staged_epilogue(const Geo& a, f32x4 (&acc)[BM / WM / 16][BN / WN / 16], int m0, int m_end, int n0,
                             int wm, int wn, int tid, char* smem, int tile, int pcls = -1) {
  constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 16, TN = WTN / 16;
  constexpr int CPR = BN / 8, RPP = NTH / CPR, PASSES = BM / RPP, NW = WM * WN;
  static_assert(NTH % CPR == 0 && BM % RPP == 0, "epilogue mapping");
  const int lane = tid & 63, fr = lane & 15, fk = lane >> 4, wave = tid >> 6;
  const int Cout = SCATTER ? a.Nout / 4 : a.Nout;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int nl = wn * WTN + j * 16 + fk * 4;           // tile column of this lane's 4 channels
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (a.bias && n0 + nl < a.Nout) {
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[r] = a.bias[SCATTER ? (n0 + nl + r) % Cout : n0 + nl + r];
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = wm * WTM + i * 16 + fr;
      const uint2 v = make_uint2(pack2(acc[i][j][0] + bv[0], acc[i][j][1] + bv[1]),
                                 pack2(acc[i][j][2] + bv[2], acc[i][j][3] + bv[3]));
      *reinterpret_cast<uint2*>(smem + row * (BN * 2) + (((nl >> 3) ^ (row & 7)) << 4) + (nl & 7) * 2) = v;
    }
  }
  __syncthreads();
  const int c = tid % CPR, n = n0 + c * 8;
  const bool nok = n < a.Nout;
  const bool want = a.stats != nullptr;                 // uniform: no unpack / sums without statistics
  float s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
  // ConvT 2x2 scatter: the thread's pixel advances RPP rows a pass; its column x on the small
  // grid and its output offset are carried with adds (+2 dcs per pixel, +2 Wd dcs more per
  // small-grid row; image rows follow each other, so an image boundary needs nothing extra)
  // instead of per-pass divisions, which made the small-K launches VALU-bound (up128 2.9 TB/s)
  int sc_x = 0;
  size_t sc_off = 0;
  if (SCATTER) {
    const int blk = n / Cout, co = n - blk * Cout;
    const int m = m0 + tid / CPR, gy = m / a.Wd;      // global small-grid row (img * Hd + y)
    sc_x = m - gy * a.Wd;
    sc_off = ((size_t)(2 * gy + (blk >> 1)) * (2 * a.Wd) + 2 * sc_x + (blk & 1)) * a.dcs + co;
  }
#pragma unroll 4
  for (int ps = 0; ps < PASSES; ++ps) {
    const int row = tid / CPR + ps * RPP;
    const int m = m0 + row;
    if (nok && m < m_end) {
      uint4 u = *reinterpret_cast<const uint4*>(smem + row * (BN * 2) + ((c ^ (row & 7)) << 4));
      size_t off;
      if (SCATTER) {
        off = sc_off;
      } else if (pcls >= 0) {                        // parity-class row -> output pixel
        const int py = pcls >> 1, px = pcls & 1;
        const int Hc = (a.Hd - py + 1) >> 1, Wc = (a.Wd - px + 1) >> 1;
        const int img = m / (Hc * Wc), rem = m - img * (Hc * Wc), uu = rem / Wc, v = rem - uu * Wc;
        off = ((size_t)(img * a.Hd + 2 * uu + py) * a.Wd + 2 * v + px) * a.dcs + n;
      } else {
        off = (size_t)m * a.dcs + n;
      }
      if (a.accumulate || want) {
        float f[8];
        unpack8(u, f);
        if (a.accumulate) {
          float o[8];
          unpack8(*reinterpret_cast<const uint4*>(a.dst + off), o);
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] = round_e(f[e] + o[e]);
          u = pack8(f);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) { s1[e] += f[e]; s2[e] += f[e] * f[e]; }
      }
      *reinterpret_cast<uint4*>(a.dst + off) = u;
    }
    if (SCATTER) {
      sc_x += RPP;
      sc_off += (size_t)(2 * RPP) * a.dcs;
      while (sc_x >= a.Wd) {
        sc_x -= a.Wd;
        sc_off += (size_t)(2 * a.Wd) * a.dcs;
      }
    }
  }
  if (a.stats == nullptr) return;
  // threads with equal c: fold within the wave (lanes c, c+CPR, ...), then over waves
#pragma unroll
  for (int e = 0; e < 8; ++e)
#pragma unroll
    for (int o = CPR; o < 64; o <<= 1) {
      s1[e] += __shfl_xor(s1[e], o, 64);
      s2[e] += __shfl_xor(s2[e], o, 64);
    }
  float* red = reinterpret_cast<float*>(smem + BM * BN * 2);   // [NW][2][BN]
  constexpr int CW = CPR < 64 ? CPR : 64;                       // distinct chunks per wave
  if (lane < CW) {
    const int cc = (wave * 64 + lane) % CPR;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[(wave * 2 + 0) * BN + cc * 8 + e] = s1[e];
      red[(wave * 2 + 1) * BN + cc * 8 + e] = s2[e];
    }
  }
  __syncthreads();
  // chunk cc appears in the waves whose 64 lanes cover it
  for (int col = tid; col < 2 * BN; col += NTH) {
    const int q = col / BN, cl = col - q * BN, cc = cl >> 3;
    if (n0 + cl >= a.Nout) continue;
    float t = 0.f;
    for (int w = 0; w < NW; ++w) {
      const int first = (w * 64) % CPR;                         // chunks held by wave w: first .. first+CW-1 (mod CPR)
      if (((cc - first + CPR) % CPR) < CW) t += red[(w * 2 + q) * BN + cl];
    }
    a.stats[(size_t)tile * 2 * a.Nout + q * a.Nout + n0 + cl] = t;
  }
}

// LSTM cell epilogue of the DMA kernels, staged through LDS: the block's c_prev tile
// [BM pixels][BN/4 hidden channels] fp32 comes in as whole 16-B chunks of rows, the
// cell (gate order i, f, g, o: c = f c_prev + i g, h = o tanh c) runs on the MFMA
// layout (each lane holds the four gates of one hidden channel of one pixel), c and h go
// back to LDS and leave as whole row chunks (c: BN B per pixel row, h: BN/2 B) instead
// of one 4-B / 2-B store per lane for 16 scattered pixels.  The gates for the backward
// keep their direct float4 stores (64 contiguous B per pixel per instruction).
template <int BM, int BN, int WM, int WN, int NTH>
STF_DEV void lstm_staged_epilogue(const Geo& a, f32x4 (&acc)[BM / WM / 16][BN / WN / 16], int m0, int m_end,
                                  int n0, int wm, int wn, int tid, char* smem) {
  constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 16, TN = WTN / 16;
  constexpr int HC = BN / 4;                            // hidden channels per tile
  constexpr int PS = HC + 4;                            // fp32 row stride (16-B aligned, skewed)
  constexpr int CCH = HC / 4, HCH = HC / 8;             // 16-B chunks per c row / h row
  float* cs = reinterpret_cast<float*>(smem);           // [BM][PS] c_prev, then c
  e16* hs = reinterpret_cast<e16*>(smem + BM * PS * 4);   // [BM][HC + 8] h
  constexpr int HS = HC + 8;
  const int lane = tid & 63, fr = lane & 15, fk = lane >> 4;
  const int Ch = a.Nout >> 2, ch0 = n0 >> 2;
  const int hcn = min(HC, Ch - ch0);                    // hidden channels present in this tile
  // whole 16-B chunks need Ch % 4 (row alignment) and a chunk inside the tile's channels;
  // a tail chunk (hcn % 4, hcn % 8 for h) moves element by element
  const bool cvec = (Ch & 3) == 0;
  for (int e = tid; e < BM * CCH; e += NTH) {
    const int r = e / CCH, q = e - r * CCH, m = m0 + r;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (a.c_prev && m < m_end && q * 4 < hcn) {
      const float* src = a.c_prev + (size_t)m * Ch + ch0 + q * 4;
      if (cvec && q * 4 + 4 <= hcn) v = *reinterpret_cast<const float4*>(src);
      else {
        float t[4] = {0.f, 0.f, 0.f, 0.f};
        for (int k = 0; k < 4 && q * 4 + k < hcn; ++k) t[k] = src[k];
        v = make_float4(t[0], t[1], t[2], t[3]);
      }
    }
    *reinterpret_cast<float4*>(cs + r * PS + q * 4) = v;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int nl = wn * WTN + j * 16 + fk * 4, nb = n0 + nl, hl = nl >> 2;
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (a.bias && nb < a.Nout) {
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[r] = a.bias[nb + r];
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = wm * WTM + i * 16 + fr, m = m0 + row;
      if (!(m < m_end && nb < a.Nout)) continue;
      float gi, gf, gg, go, c, hh;
      lstm_cell_fwd(acc[i][j][0] + bv[0], acc[i][j][1] + bv[1], acc[i][j][2] + bv[2], acc[i][j][3] + bv[3],
                    cs[row * PS + hl], gi, gf, gg, go, c, hh);
      cs[row * PS + hl] = c;
      hs[row * HS + hl] = f2e(hh);
      if (a.gates) *reinterpret_cast<float4*>(a.gates + (size_t)m * a.Nout + nb) = make_float4(gi, gf, gg, go);
    }
  }
  __syncthreads();
  for (int e = tid; e < BM * CCH; e += NTH) {
    const int r = e / CCH, q = e - r * CCH, m = m0 + r;
    if (!(m < m_end && q * 4 < hcn)) continue;
    float* dst = a.c_out + (size_t)m * Ch + ch0 + q * 4;
    if (cvec && q * 4 + 4 <= hcn) *reinterpret_cast<float4*>(dst) = *reinterpret_cast<const float4*>(cs + r * PS + q * 4);
    else
      for (int k = 0; k < 4 && q * 4 + k < hcn; ++k) dst[k] = cs[r * PS + q * 4 + k];
  }
  const bool hvec = ((reinterpret_cast<uintptr_t>(a.h_out) & 15) == 0) && (a.hcs & 7) == 0;
  for (int e = tid; e < BM * HCH; e += NTH) {
    const int r = e / HCH, q = e - r * HCH, m = m0 + r;
    if (!(m < m_end && q * 8 < hcn)) continue;
    uint16_t* dst = a.h_out + (size_t)m * a.hcs + ch0 + q * 8;
    const e16* src = hs + r * HS + q * 8;
    if (hvec && q * 8 + 8 <= hcn) *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(src);
    else
      for (int k = 0; k < 8 && q * 8 + k < hcn; ++k) reinterpret_cast<e16*>(dst)[k] = src[k];
  }
}

// LSTM cell-backward epilogue (EPI 2), staged through LDS like the forward's: the
// block's c_t, c_{t-1}, dc_next (fp32) and dh (bf16) tiles come in as whole 16-B row
// chunks, the cell backward runs on the MFMA layout (a lane holds the four recomputed
// gate pre-activations of one hidden channel of one pixel), dc_prev goes back to LDS
// (over dc_next) and leaves as row chunks; the four bf16 gate gradients of a lane are
// one 8-B store (32 contiguous bytes per pixel per wave-instruction).
template <int BM, int BN>
constexpr int lstm_bwd_lds() { return 3 * BM * (BN / 4 + 4) * 4 + BM * (BN / 4 + 8) * 2; }

template <int BM, int BN, int WM, int WN, int NTH>
STF_DEV void lstm_bwd_staged_epilogue(const Geo& a, f32x4 (&acc)[BM / WM / 16][BN / WN / 16], int m0, int m_end,
                                      int n0, int wm, int wn, int tid, char* smem) {
  constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 16, TN = WTN / 16;
  constexpr int HC = BN / 4, PS = HC + 4, HS = HC + 8, CCH = HC / 4, HCH = HC / 8;
  float* cts = reinterpret_cast<float*>(smem);           // [BM][PS] c_t
  float* cps = cts + BM * PS;                            // [BM][PS] c_{t-1}
  float* dcs = cps + BM * PS;                            // [BM][PS] dc_next, then dc_prev
  e16* dhs = reinterpret_cast<e16*>(dcs + BM * PS);    // [BM][HS] dh
  const int lane = tid & 63, fr = lane & 15, fk = lane >> 4;
  const int Ch = a.Nout >> 2, ch0 = n0 >> 2;
  const int hcn = min(HC, Ch - ch0);
  const bool cvec = (Ch & 3) == 0;
  auto ld4 = [&](const float* base, int m, int q) {
    if (!base || m >= m_end || q * 4 >= hcn) return make_float4(0.f, 0.f, 0.f, 0.f);
    const float* src = base + (size_t)m * Ch + ch0 + q * 4;
    if (cvec && q * 4 + 4 <= hcn) return *reinterpret_cast<const float4*>(src);
    float t[4] = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < 4 && q * 4 + k < hcn; ++k) t[k] = src[k];
    return make_float4(t[0], t[1], t[2], t[3]);
  };
  for (int e = tid; e < BM * CCH; e += NTH) {
    const int r = e / CCH, q = e - r * CCH, m = m0 + r;
    *reinterpret_cast<float4*>(cts + r * PS + q * 4) = ld4(a.c_out, m, q);
    *reinterpret_cast<float4*>(cps + r * PS + q * 4) = ld4(a.c_prev, m, q);
    *reinterpret_cast<float4*>(dcs + r * PS + q * 4) = ld4(a.l_dcn, m, q);
  }
  const bool hvec = ((reinterpret_cast<uintptr_t>(a.l_dh) & 15) == 0) && (a.l_dhcs & 7) == 0;
  for (int e = tid; e < BM * HCH; e += NTH) {
    const int r = e / HCH, q = e - r * HCH, m = m0 + r;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (m < m_end && q * 8 < hcn) {
      const uint16_t* src = a.l_dh + (size_t)m * a.l_dhcs + ch0 + q * 8;
      if (hvec && q * 8 + 8 <= hcn) v = *reinterpret_cast<const uint4*>(src);
      else {
        uint16_t t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int k = 0; k < 8 && q * 8 + k < hcn; ++k) t[k] = src[k];
        v = make_uint4(t[0] | ((uint32_t)t[1] << 16), t[2] | ((uint32_t)t[3] << 16), t[4] | ((uint32_t)t[5] << 16),
                       t[6] | ((uint32_t)t[7] << 16));
      }
    }
    *reinterpret_cast<uint4*>(dhs + r * HS + q * 8) = v;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int nl = wn * WTN + j * 16 + fk * 4, nb = n0 + nl, hl = nl >> 2;
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (a.bias && nb < a.Nout) {
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[r] = a.bias[nb + r];
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = wm * WTM + i * 16 + fr, m = m0 + row;
      if (!(m < m_end && nb < a.Nout)) continue;
      float gi, gf, gg, go, cx, hx;
      lstm_cell_fwd(acc[i][j][0] + bv[0], acc[i][j][1] + bv[1], acc[i][j][2] + bv[2], acc[i][j][3] + bv[3], 0.f,
                    gi, gf, gg, go, cx, hx);
      float d_i, d_f, d_g, d_o, dcp;
      lstm_cell_bwd(gi, gf, gg, go, cts[row * PS + hl], cps[row * PS + hl], e2f(dhs[row * HS + hl]),
                    dcs[row * PS + hl], d_i, d_f, d_g, d_o, dcp);
      dcs[row * PS + hl] = dcp;
      *reinterpret_cast<uint2*>(a.l_dg + (size_t)m * a.Nout + nb) = make_uint2(pack2(d_i, d_f), pack2(d_g, d_o));
    }
  }
  __syncthreads();
  for (int e = tid; e < BM * CCH; e += NTH) {
    const int r = e / CCH, q = e - r * CCH, m = m0 + r;
    if (!(m < m_end && q * 4 < hcn)) continue;
    float* dst = a.l_dcp + (size_t)m * Ch + ch0 + q * 4;
    if (cvec && q * 4 + 4 <= hcn) *reinterpret_cast<float4*>(dst) = *reinterpret_cast<const float4*>(dcs + r * PS + q * 4);
    else
      for (int k = 0; k < 4 && q * 4 + k < hcn; ++k) dst[k] = dcs[r * PS + q * 4 + k];
  }
}

template <int BM, int BN, int WM, int WN, bool SMALLC, bool TRANS, bool SCATTER, int EPI>
__global__ __launch_bounds__(NT, 2) void igemm_kernel(Geo a) {
  constexpr int WTM = BM / WM, WTN = BN / WN;     // wave tile (pixels x channels)
  constexpr int TM = WTM / 16, TN = WTN / 16;     // 16x16 fragments per wave
  constexpr int CHA = BM * BK / 8 / NT;           // 16-B chunks per thread (im2col)
  constexpr int CHB = BN * BK / 8 / NT;           // 16-B chunks per thread (weights)
  static_assert(WM * WN == 4, "4 waves");
  static_assert(CHA >= 1 && CHB >= 1, "tile too small");
  constexpr int LDS_A = BM * BK * 2, LDS_B = BN * BK * 2;
  constexpr int LDS_MAIN = 2 * (LDS_A + LDS_B), LDS_RED = WM * 2 * BN * 4;
  __shared__ __attribute__((aligned(16))) char smem[LDS_MAIN > LDS_RED ? LDS_MAIN : LDS_RED];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  // M tiles never straddle a statistics group: block x = (group, tile within group)
  const int grp = blockIdx.x / a.tpg, gtile = blockIdx.x - grp * a.tpg;
  const int m0 = grp * a.Mg + gtile * BM, n0 = blockIdx.y * BN;
  const int m_end = min(m0 + BM, min((grp + 1) * a.Mg, a.M));
  const int kc = tid & 3;                 // this thread's 16-B chunk within a 64-B row

  // per-row gather state for the im2col rows this thread stages
  int rbase[CHA], ry[CHA], rx[CHA];
  bool rok[CHA];
#pragma unroll
  for (int i = 0; i < CHA; ++i) {
    const int m = m0 + (tid >> 2) + i * (NT / 4);
    rok[i] = m < m_end;
    const int mm = rok[i] ? m : 0;
    const int hw = a.Hd * a.Wd;
    const int n = mm / hw, rem = mm - n * hw;
    const int yd = rem / a.Wd, xd = rem - yd * a.Wd;
    rbase[i] = n * a.Hs * a.Ws;
    if (TRANS) { ry[i] = yd + a.pad; rx[i] = xd + a.pad; }
    else { ry[i] = yd * a.st - a.pad; rx[i] = xd * a.st - a.pad; }
  }

  uint4 ra[CHA], rb[CHB];
  int tr = 0, ts = 0, tc = 0;             // tap / channel cursor of the next K step (non-SMALLC)
  const int KT = (a.K + BK - 1) / BK;

  auto gather_src = [&](int i, int r, int s, int c, uint4& out) {
    int ys, xs; bool ok = rok[i];
    if (TRANS) {
      const int ty = ry[i] - r, tx = rx[i] - s;
      if (a.st == 2) { ok = ok && !(ty & 1) && !(tx & 1); ys = ty >> 1; xs = tx >> 1; }
      else { ys = ty; xs = tx; }
      ok = ok && ty >= 0 && tx >= 0;
    } else { ys = ry[i] + r; xs = rx[i] + s; ok = ok && ys >= 0 && xs >= 0; }
    ok = ok && ys < a.Hs && xs < a.Ws;
    out = make_uint4(0, 0, 0, 0);
    if (ok) out = *reinterpret_cast<const uint4*>(a.src + (size_t)(rbase[i] + ys * a.Ws + xs) * a.scs + c);
  };

  auto load_tiles = [&](int kt) {
    const int k0 = kt * BK;
    if (SMALLC) {
      const int k = k0 + kc * 8;
      const bool kok = k < a.K;
      const int tap = kok ? k / a.Cs : 0;
      const int c = k - tap * a.Cs;
      const int r = tap / a.S, s = tap - r * a.S;
#pragma unroll
      for (int i = 0; i < CHA; ++i) {
        if (kok) gather_src(i, r, s, c, ra[i]); else ra[i] = make_uint4(0, 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int i = 0; i < CHA; ++i) gather_src(i, tr, ts, tc + kc * 8, ra[i]);
      tc += BK;
      if (tc == a.Cs) { tc = 0; if (++ts == a.S) { ts = 0; ++tr; } }
    }
#pragma unroll
    for (int i = 0; i < CHB; ++i) {
      const int n = n0 + (tid >> 2) + i * (NT / 4);
      const int k = k0 + kc * 8;
      rb[i] = make_uint4(0, 0, 0, 0);
      if (n < a.Nout && k < a.K) rb[i] = *reinterpret_cast<const uint4*>(a.wgt + (size_t)n * a.K + k);
    }
  };

  auto store_tiles = [&](int buf) {
    char* sa = smem + buf * (LDS_A + LDS_B);
    char* sb = sa + LDS_A;
#pragma unroll
    for (int i = 0; i < CHA; ++i) {
      const int row = (tid >> 2) + i * (NT / 4);
      *reinterpret_cast<uint4*>(sa + row * 64 + swz(row, kc) * 16) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < CHB; ++i) {
      const int row = (tid >> 2) + i * (NT / 4);
      *reinterpret_cast<uint4*>(sb + row * 64 + swz(row, kc) * 16) = rb[i];
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  load_tiles(0);
  store_tiles(0);
  __syncthreads();

  const int fr = lane & 15, fk = lane >> 4;
  for (int kt = 0; kt < KT; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < KT) load_tiles(kt + 1);
    const char* sa = smem + cur * (LDS_A + LDS_B);
    const char* sb = sa + LDS_A;
    e16x8 xf[TM], wf[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = wm * WTM + i * 16 + fr;
      xf[i] = *reinterpret_cast<const e16x8*>(sa + row * 64 + swz(row, fk) * 16);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int row = wn * WTN + j * 16 + fr;
      wf[j] = *reinterpret_cast<const e16x8*>(sb + row * 64 + swz(row, fk) * 16);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = mfma16x16x32(wf[j], xf[i], acc[i][j]);
    if (kt + 1 < KT) store_tiles(cur ^ 1);
    __syncthreads();
  }

  int mrow[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + wm * WTM + i * 16 + (lane & 15);
    mrow[i] = m < m_end ? m : -1;
  }
  igemm_epilogue<BM, BN, WM, WN, SCATTER, EPI, NT>(a, acc, mrow, n0, wm, wn, tid, smem, blockIdx.x);
}

// ---------------------------------------------------------------------------
// LDS-DMA ring variant (Cs % BKK == 0): every 16-B chunk goes global -> LDS with
// buffer_load_dwordx4 ... lds (no VGPR staging, no ds_write).  The im2col halo
// and all tails are zero-filled by the buffer range check: an invalid lane gets
// voffset 0xFFFFFFF0 >= num_records.  One wave-instruction writes 1 KiB of rows
// linearly, so the chunk swizzle is applied on the SOURCE side (lane with LDS
// chunk slot p loads global chunk swz(row, p)); the fragment reads use the same
// involution.  STAGES-deep ring, STAGES-1 K steps in flight across the raw
// s_barrier; a counted vmcnt retires exactly the stage about to be read.
//   BKK = 32: 64-B rows, chunk ^ ((-(row>>2)) & 3)
//   BKK = 64: 128-B rows, chunk ^ ((row>>1) & 7)   (two MFMA k-halves per step)
// Both make each ds_read_b128 lane group (4 x 16 lanes) hit 16 distinct 16-B
// slots of the 256-B bank row.  Blocks are remapped so that consecutive tiles
// (shared halo rows) and all channel tiles of one pixel tile run on one XCD.
template <int BKK>
STF_DEV int swzk(int row, int kc) {
  if constexpr (BKK == 32) return kc ^ ((-(row >> 2)) & 3);
  else return kc ^ ((row >> 1) & 7);
}

// C8: 8-channel sources (network inputs): a 16-B chunk is one whole tap, so
// every lane gathers its own tap (k-step = 4 taps at BKK 32); K need not be a
// multiple of BKK (k >= K masked)
template <int BM, int BN, int WM, int WN, int BKK, int STAGES, bool TRANS, bool SCATTER, int EPI, bool C8 = false>
__global__ __launch_bounds__(64 * WM * WN, (WM * WN == 4 || (BM == 128 && BN == 256)) ? 2 : 1) void igemm_dma_kernel(
    Geo a, uint32_t src_bytes) {
  constexpr int NW = WM * WN, NTH = 64 * NW;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int ROWB = BKK * 2;                         // bytes per LDS row
  constexpr int CPR = BKK / 8;                          // 16-B chunks per row
  constexpr int RPI = 64 / CPR;                         // rows per DMA wave-instruction (1 KiB)
  constexpr int LA = BM / NW / RPI, LB = BN / NW / RPI; // DMA instructions per wave per K step
  constexpr int STAGE = (BM + BN) * ROWB;
  constexpr int LDS_MAIN = STAGES * STAGE;
  constexpr int LDS_RED = EPI == 0 ? BM * BN * 2 + NW * 2 * BN * 4 : (EPI == 2 ? lstm_bwd_lds<BM, BN>() : WM * 2 * BN * 4);
  static_assert(LA >= 1 && LB >= 1 && LA * RPI * NW == BM && LB * RPI * NW == BN, "tile");
  __shared__ __attribute__((aligned(16))) char smem[LDS_MAIN > LDS_RED ? LDS_MAIN : LDS_RED];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  // XCD-aware bijective remap of the linear block id (8 XCDs, round-robin dispatch)
  const int gx = gridDim.x, gy = gridDim.y, nwg = gx * gy;
  const int orig = blockIdx.y * gx + blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int bx = wid / gy, by = wid - bx * gy;
  const int grp = bx / a.tpg, gtile = bx - grp * a.tpg;
  int m0 = grp * a.Mg + gtile * BM, m_end = min(m0 + BM, min((grp + 1) * a.Mg, a.M));
  const int n0 = by * BN;
  const int sub = lane / CPR, slot = lane % CPR;
  // Parity mode (stride-2 transposed gather): output pixel (y, x) only receives the taps
  // r = y + pad (mod 2), s = x + pad (mod 2).  Rows are ordered by class (y & 1, x & 1),
  // each block lies in one class and walks only that class's taps (1/2/2/4 of the nine
  // for 3x3, none for the odd classes of 1x1) instead of masking 3/4 of the MFMAs to zero.
  // par == 2 (an accumulating launch): classes without taps (the odd ones of a 1x1 / stride-2
  // transposed gather) add nothing -- they get no blocks at all (stf_igemm counts the same way)
  int pcls = -1, py = 0, px = 0, Hc = 0, Wc = 0, r0 = 0, s0 = 0;
  if (TRANS && a.par) {
    int b = gtile;
#pragma unroll
    for (int ci = 0; ci < 4; ++ci) {
      const int c = 3 - ci;                         // (1,1) first: 4 taps, then 2, 2, 1 (shorter tail)
      const int hc = (a.Hd - (c >> 1) + 1) >> 1, wc = (a.Wd - (c & 1) + 1) >> 1;
      const int mc = a.N * hc * wc, nb = (mc + BM - 1) / BM;
      const int ntap = ((a.R - (((c >> 1) + a.pad) & 1) + 1) >> 1) * ((a.S - (((c & 1) + a.pad) & 1) + 1) >> 1);
      if (a.par == 2 && ntap == 0) continue;
      if (pcls < 0) {
        if (b < nb) { pcls = c; Hc = hc; Wc = wc; m0 = b * BM; m_end = min(m0 + BM, mc); }
        else b -= nb;
      }
    }
    py = pcls >> 1; px = pcls & 1;
    r0 = (py + a.pad) & 1; s0 = (px + a.pad) & 1;
  }

  const __amdgpu_buffer_rsrc_t rs_src = __builtin_amdgcn_make_buffer_rsrc((void*)a.src, 0, src_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_wgt =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.wgt, 0, (uint32_t)a.Nout * a.K * 2, 0x00020000);

  int rbase[LA], ry[LA], rx[LA], akc[LA];
  bool rok[LA];
#pragma unroll
  for (int i = 0; i < LA; ++i) {
    const int row = wave * (BM / NW) + i * RPI + sub;
    const int m = m0 + row;
    rok[i] = m < m_end;
    const int mm = rok[i] ? m : m0;
    int n, yd, xd;
    if (TRANS && a.par) {
      n = mm / (Hc * Wc);
      const int rem = mm - n * (Hc * Wc), u = rem / Wc;
      yd = 2 * u + py; xd = 2 * (rem - u * Wc) + px;
    } else {
      const int hw = a.Hd * a.Wd;
      n = mm / hw;
      const int rem = mm - n * hw;
      yd = rem / a.Wd; xd = rem - yd * a.Wd;
    }
    rbase[i] = n * a.Hs * a.Ws;
    if (TRANS) { ry[i] = yd + a.pad; rx[i] = xd + a.pad; }
    else { ry[i] = yd * a.st - a.pad; rx[i] = xd * a.st - a.pad; }
    akc[i] = swzk<BKK>(row, slot);
  }
  int bn_[LB], bkc[LB];
#pragma unroll
  for (int i = 0; i < LB; ++i) {
    const int row = wave * (BN / NW) + i * RPI + sub;
    bn_[i] = n0 + row;
    bkc[i] = swzk<BKK>(row, slot);
  }
  constexpr uint32_t BAD = 0xFFFFFFF0u;
  const int tstep = (TRANS && a.par) ? 2 : 1;          // tap stride of the cursor
  const int KTall = C8 ? (a.K + BKK - 1) / BKK
                       : ((TRANS && a.par) ? ((a.R - r0 + 1) >> 1) * ((a.S - s0 + 1) >> 1) * (a.Cs / BKK) : a.K / BKK);
  int tr = r0, ts = s0, tc = 0;                         // tap / channel cursor of the next K step to issue
  // split-K (plain gathers only, see ksplit_of): this block's slice of the K steps
  int KT = KTall;
  if (!C8 && !TRANS && !SCATTER && EPI == 0 && a.ksplit > 1) {
    const int kb = (int)((long)KTall * blockIdx.z / a.ksplit);
    KT = (int)((long)KTall * (blockIdx.z + 1) / a.ksplit) - kb;
    const int k0 = kb * BKK, tap = k0 / a.Cs;
    tc = k0 - tap * a.Cs; tr = tap / a.S; ts = tap - tr * a.S;
  }

  auto issue = [&](int kt) {
    char* st = smem + (kt % STAGES) * STAGE;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      int ys, xs;
      bool ok = rok[i];
      if (C8) {
        const int tap = (kt * BKK) / 8 + akc[i], r = tap / a.S, s_ = tap - r * a.S;
        ys = ry[i] + r;
        xs = rx[i] + s_;
        ok = ok && tap < a.R * a.S && ys >= 0 && xs >= 0 && ys < a.Hs && xs < a.Ws;
        const uint32_t off = ok ? (uint32_t)(((rbase[i] + ys * a.Ws + xs) * a.scs) * 2) : BAD;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rs_src, (__attribute__((address_space(3))) void*)(st + (wave * (BM / NW) + i * RPI) * ROWB), 16, off, 0,
            0, 0);
        continue;
      }
      if (TRANS) {
        const int ty = ry[i] - tr, tx = rx[i] - ts;
        if (a.st == 2) { ok = ok && !(ty & 1) && !(tx & 1); ys = ty >> 1; xs = tx >> 1; }
        else { ys = ty; xs = tx; }
        ok = ok && ty >= 0 && tx >= 0;
      } else { ys = ry[i] + tr; xs = rx[i] + ts; ok = ok && ys >= 0 && xs >= 0; }
      ok = ok && ys < a.Hs && xs < a.Ws;
      const uint32_t off = ok ? (uint32_t)(((rbase[i] + ys * a.Ws + xs) * a.scs + tc + akc[i] * 8) * 2) : BAD;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs_src, (__attribute__((address_space(3))) void*)(st + (wave * (BM / NW) + i * RPI) * ROWB), 16, off, 0, 0,
          0);
    }
    const int k0 = C8 ? kt * BKK : (tr * a.S + ts) * a.Cs + tc;
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const bool ok = bn_[i] < a.Nout && (!C8 || k0 + bkc[i] * 8 < a.K);
      const uint32_t off = ok ? (uint32_t)((bn_[i] * a.K + k0 + bkc[i] * 8) * 2) : BAD;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs_wgt, (__attribute__((address_space(3))) void*)(st + BM * ROWB + (wave * (BN / NW) + i * RPI) * ROWB),
          16, off, 0, 0, 0);
    }
    tc += BKK;
    if (tc == a.Cs) { tc = 0; ts += tstep; if (ts >= a.S) { ts = s0; tr += tstep; } }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  constexpr int D = STAGES - 1;                         // K steps in flight
  constexpr int L = LA + LB;                            // DMA ops per wave per K step
  for (int s = 0; s < D && s < KT; ++s) issue(s);
  const int fr = lane & 15, fk = lane >> 4;
  for (int kt = 0; kt < KT; ++kt) {
    // retire stage kt (this wave's DMAs), then the barrier makes every wave's visible
    if (kt + D <= KT) asm volatile("s_waitcnt vmcnt(%0)" :: "n"((D - 1) * L) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // the stage read at kt-1 is free for everyone now: refill it D steps ahead
    if (kt + D < KT) issue(kt + D);
    const char* sa = smem + (kt % STAGES) * STAGE;
    const char* sb = sa + BM * ROWB;
#pragma unroll
    for (int h = 0; h < BKK / 32; ++h) {
      e16x8 xf[TM], wf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WTM + i * 16 + fr;
        xf[i] = *reinterpret_cast<const e16x8*>(sa + row * ROWB + swzk<BKK>(row, fk + 4 * h) * 16);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * WTN + j * 16 + fr;
        wf[j] = *reinterpret_cast<const e16x8*>(sb + row * ROWB + swzk<BKK>(row, fk + 4 * h) * 16);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = mfma16x16x32(wf[j], xf[i], acc[i][j]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  if constexpr (!C8 && !TRANS && !SCATTER && EPI == 0) {
    if (a.ksplit > 1) {
      // raw fp32 partial of this K slice: lane holds 4 consecutive channels of one row
      float* wz = a.ws + (size_t)blockIdx.z * a.M * a.Nout;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = m0 + wm * WTM + i * 16 + fr;
        if (m >= m_end) continue;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int n = n0 + wn * WTN + j * 16 + fk * 4;
          if (n < a.Nout)
            *reinterpret_cast<float4*>(wz + (size_t)m * a.Nout + n) =
                make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
        }
      }
      return;
    }
  }
  __syncthreads();
  if constexpr (EPI == 0) {
    staged_epilogue<BM, BN, WM, WN, SCATTER, NTH>(a, acc, m0, m_end, n0, wm, wn, tid, smem, bx, pcls);
  } else if (EPI == 1 && lstm_staged()) {
    static_assert(EPI != 1 || LDS_MAIN >= BM * (BN / 4 + 4) * 4 + BM * (BN / 4 + 8) * 2, "LSTM staging");
    lstm_staged_epilogue<BM, BN, WM, WN, NTH>(a, acc, m0, m_end, n0, wm, wn, tid, smem);
  } else if (EPI == 2 && lstm_staged()) {
    lstm_bwd_staged_epilogue<BM, BN, WM, WN, NTH>(a, acc, m0, m_end, n0, wm, wn, tid, smem);
  } else {
    int mrow[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wm * WTM + i * 16 + fr;
      mrow[i] = m < m_end ? m : -1;
    }
    igemm_epilogue<BM, BN, WM, WN, SCATTER, EPI, NTH>(a, acc, mrow, n0, wm, wn, tid, smem, bx);
  }
}


// Split-K fold: dst = bf16(sum_z ws[z] + bias) (+ old dst), plus the BN partial
// statistics of the stored values per row tile (tiles aligned to the statistic
// groups: [G][tpg][2][Nout]).  Thread = 8 consecutive channels of SK_PASS rows
// (a tile = SK_PASS * 256 / (Nout / 8) rows); every slab's loads for the SK_PASS
// rows are issued together (the fold is latency-bound otherwise).
constexpr int SK_PASS = 4;
__host__ __device__ inline int sk_rows(int Nout) { return SK_PASS * (NT / (Nout / 8)); }
__global__ __launch_bounds__(NT) void splitk_reduce_kernel(Geo a, int tpg) {
  __shared__ float red[NT][17];
  const int CG = a.Nout / 8, RPP = NT / CG, RB = SK_PASS * RPP;
  const int grp = blockIdx.x / tpg, t = blockIdx.x - grp * tpg;
  const int r0 = grp * a.Mg + t * RB, r1 = min(r0 + RB, (grp + 1) * a.Mg);
  const int cg = threadIdx.x % CG, n = cg * 8, rr = threadIdx.x / CG;
  float f[SK_PASS][8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float bv = a.bias ? a.bias[n + e] : 0.f;
#pragma unroll
    for (int p = 0; p < SK_PASS; ++p) f[p][e] = bv;
  }
  const size_t slab = (size_t)a.M * a.Nout;
  for (int z = 0; z < a.ksplit; ++z) {
#pragma unroll
    for (int p = 0; p < SK_PASS; ++p) {
      const int m = r0 + rr + p * RPP;
      if (m >= r1) continue;
      const float* w = a.ws + z * slab + (size_t)m * a.Nout + n;
      const float4 lo = *reinterpret_cast<const float4*>(w);
      const float4 hi = *reinterpret_cast<const float4*>(w + 4);
      f[p][0] += lo.x; f[p][1] += lo.y; f[p][2] += lo.z; f[p][3] += lo.w;
      f[p][4] += hi.x; f[p][5] += hi.y; f[p][6] += hi.z; f[p][7] += hi.w;
    }
  }
  float s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int p = 0; p < SK_PASS; ++p) {
    const int m = r0 + rr + p * RPP;
    if (m >= r1) continue;
    uint16_t* d = a.dst + (size_t)m * a.dcs + n;
    if (a.accumulate) {
      float o[8];
      unpack8(*reinterpret_cast<const uint4*>(d), o);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[p][e] = round_e(f[p][e]) + o[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) f[p][e] = round_e(f[p][e]);
    *reinterpret_cast<uint4*>(d) = pack8(f[p]);
#pragma unroll
    for (int e = 0; e < 8; ++e) { s1[e] += f[p][e]; s2[e] += f[p][e] * f[p][e]; }
  }
  if (!a.stats) return;
#pragma unroll
  for (int e = 0; e < 8; ++e) { red[threadIdx.x][e] = s1[e]; red[threadIdx.x][8 + e] = s2[e]; }
  __syncthreads();
  for (int c = threadIdx.x; c < a.Nout; c += NT) {
    const int g8 = c / 8, e = c - g8 * 8;
    float u = 0.f, v = 0.f;
    for (int q = g8; q < NT; q += CG) { u += red[q][e]; v += red[q][8 + e]; }
    a.stats[(size_t)blockIdx.x * 2 * a.Nout + c] = u;
    a.stats[(size_t)blockIdx.x * 2 * a.Nout + a.Nout + c] = v;
  }
}

// ---------------------------------------------------------------------------
// Halo kernel: 3x3 / stride 1 / pad 1 convolution (forward, and the stride-1
// dgrad over flipped taps) as nine shifted views of one LDS halo.
//
// The linear kernels above gather the source rows of every tap separately, so
// each activation row crosses L2 -> LDS nine times; for the 64-channel
// full-resolution layers that re-read traffic (~26 GB/s per CU) is the bound.
// Here a workgroup owns a PH x PW pixel tile and a 64-channel output slice; per
// 32-channel source chunk one stage holds the (PH+2) x (PW+2) halo and the 64 x
// 9 weight rows of that chunk, and the nine taps are read from the halo at row
// offsets (r * (PW+2) + s).  Persistent: each workgroup walks a contiguous run
// of (tile, channel-slice) items through a 2-stage LDS-DMA ring, so the next
// stage streams in behind the MFMAs and the epilogue.  Rows are 64 B with the
// chunk swizzle kc ^ ((key >> 1) & 2): for weight rows key = row, for halo rows
// key = the halo COLUMN, so a tap's row shift dy leaves the swizzle unchanged (an
// immediate offset).  Both are conflict-free for every ds_read_b128 lane group at
// any tap shift (checked exhaustively over columns, shifts and row residues).
STF_DEV int swzh(int key, int kc) { return kc ^ ((key >> 1) & 2); }

// tap before which the first wave half issues the next stage's DMA share (-1: at the stage start;
// the second half issues at tap 4); a build-time A/B switch (-DHALO_ATAP=2)
#ifndef HALO_ATAP
#define HALO_ATAP -1
#endif

// output row (pixel index of the destination) of tile pixel p, or -1 outside the image
template <int PH, int PW, int IX>
STF_DEV int halo_pixel(int p, int img, int ty, int tx, int Hd, int Wd) {
  int y = ty * PH + p / PW, x = tx * PW + p % PW;
  if constexpr (IX > 1) {
    const int b = (p % PW) / (PW / IX);
    x = p % PW - b * (PW / IX);
    img += b;
  }
  return (y < Hd && x < Wd) ? (img * Hd + y) * Wd + x : -1;
}

// NW waves x 64 pixels = PH x PW tile; STAGES = 2: one 8-wave workgroup per CU
// with a 2-stage ring; STAGES = 1: two 4-wave workgroups per CU, single stage
// each, so one workgroup's DMA wait and epilogue overlap the other's MFMAs.
// DIRECT: weight rows are fetched in the permuted order
// row j*16 + fk*4 + r <- channel (j>>1)*32 + fk*8 + (j&1)*4 + r, so a lane's
// accumulators of fragments (0,1) and (2,3) are 8 consecutive channels each and
// the epilogue stores 16-B chunks straight from registers (no LDS staging).
//
// IX > 1 (multi-image tiles, conv3x3_halo2_kernel): the PH x PW tile is IX whole images of
// PH x (PW / IX) side by side (STF layer3: two 16 x 16 images in one 16 x 32 tile), so a
// small image fills the wide tile instead of half a 16 x 16 one: twice the pixels per stage
// for the same weight rows.  Neighbouring images share one zero column in the halo (image
// b's column x sits at halo column b * (IW + 1) + 1 + x), PW + IX + 1 columns in all.
// DEFER (8-wave, 2-stage direct epilogues): the second wave half (waves NW/2.., the SIMD
// partners of the first half) runs each item's epilogue after the next stage barrier, ahead of
// its next taps, so on every SIMD one wave's epilogue (VALU, stores) overlaps its partner's
// MFMAs instead of both idling the matrix pipe together; BatchNorm partials are then kept per
// wave (one statistics row per (group, workgroup, wave): no cross-wave LDS pass, no epilogue
// barrier) and the BN-backward y tile is loaded to registers.
template <int PH, int PW, int NW, int STAGES, int DIAG, int DIRECT, bool BNR, int IX, bool DEFER_T = false>
__device__ __forceinline__ void halo_body(Geo a, uint32_t src_bytes, int TY, int TX, int per, int rem) {
  constexpr int NTH = 64 * NW, BN = 64, RPI = 16;       // 64-B rows: 16 per 1-KiB DMA instruction
  constexpr int IW = PW / IX;                           // image width in a multi-image tile
  constexpr int HW = PW + IX + 1, HR = (PH + 2) * HW;   // halo rows
  // DMA instructions per stage, dealt to the waves as evenly as they go (wave w: hcnt(w) from
  // hbeg(w)); the ring holds exactly these rows, so the stages leave room for the affine area
  constexpr int HIN = (HR + RPI - 1) / RPI, WIN = 9 * BN / RPI;
  constexpr int HI = (HIN + NW - 1) / NW, WI = (WIN + NW - 1) / NW;   // per wave, at most
  constexpr int HROWS = HIN * RPI, WROWS = WIN * RPI;
  constexpr int STAGE = (HROWS + WROWS) * 64;
  constexpr int AFF = STAGES * STAGE;                 // BNR: per-wave BN affine [4][64] fp32 after the ring
  static_assert(9 * BN % RPI == 0, "weight rows");
  constexpr int PX = PH * PW, WTM = PX / NW, TM = WTM / 16, TN = BN / 16;
  constexpr int PPP = NTH / 8, NSTORE = PX / PPP;      // epilogue: pixels per pass, stores per lane
  // next stage's DMA (STAGES == 2): even waves at the stage start, odd waves after tap 4.
  // DIAG 4 cycle buckets (tools/halo_timeline.py, 256^2 64->64): with every wave issuing
  // at once a third of the wave time is spent stalled issuing LDS-DMA; staggered, one wave
  // of each SIMD computes while the other issues (-8 % cycles).  Spreading every wave's
  // instructions over the taps only moves the stall into the taps: the DMA path itself
  // is the limit, fewer bytes per FLOP is what would help.
  constexpr bool STAGGER = STAGES == 2 && NW == 8;
  constexpr bool DF = DEFER_T && DIRECT != 0 && STAGGER;   // the deferred epilogue (8-wave direct kernels)
  static_assert((WTM == 64 || WTM == 32) && PW % 16 == 0 && PX % PPP == 0, "tile");
  static_assert(PX * 128 + NW * 2 * 64 * 4 <= STAGE, "epilogue scratch");
  // per-wave epilogue scratch after the ring (BNR or DF): [scale | shift | mean | invstd][64] fp32 of
  // the current (group, slice) for the BN-backward reduction, or (DF forward) the slice's 64 biases
  constexpr int EPS = (BNR || DF) ? NW * 1024 : 0;
  static_assert((AFF + EPS) * (STAGES == 1 ? 2 : 1) <= 163840, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[STAGES * STAGE + EPS];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: scalar DMA addressing
  const int fr = lane & 15, fk = lane >> 4, sub = lane >> 2, slot = lane & 3;
  const bool late = DF ? wave >= NW / 2 : (wave & 1);   // issues its DMA share at tap 4
  const int NTn = a.Nout / BN, CC = a.Cs / 32, tpi = TY * TX;
  const int ntiles = (a.N / IX) * tpi;                  // items: channel slice major, pixel tile minor
  const int ipg = a.Mg / (a.Hd * a.Wd);                 // images per statistics group
  const int vb = blockIdx.x;
  const int cnt = per + (int)(vb < rem);
  const int it0 = vb * per + min(vb, rem);
  const int S = cnt * CC;
  if (S == 0) return;

  const __amdgpu_buffer_rsrc_t rs_src = __builtin_amdgcn_make_buffer_rsrc((void*)a.src, 0, src_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_wgt =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.wgt, 0, (uint32_t)a.Nout * a.K * 2, 0x00020000);
  constexpr uint32_t BAD = 0xFFFFFFF0u;
  // NULL bias -> zero-sized range: the loads return 0 without a branch
  const __amdgpu_buffer_rsrc_t rs_bias = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.bias, 0, a.bias ? (uint32_t)a.Nout * 4 : 0u, 0x00020000);

  // live = false: a dummy stage (all lanes out of range) so every iteration issues the same DMA count
  // DMA instructions k0 .. k1-1 of this wave's HI halo + WI weight instructions
  // weight rows held by each ring stage: key nt * CC + cc (wave-uniform, every wave tracks
  // the same sequence).  With an even chunk count a stage holds the same source chunk for
  // every item, so within one output slice its weight rows never change and the refill
  // of the stage only streams the halo (half the DMA instructions at 64 source channels).
  int wkey0 = -1, wkey1 = -1;
  auto issue_part = [&](int item, int cc, int buf, bool live, int k0, int k1, bool wload) {
    const int nt = item / ntiles, tile = item - nt * ntiles;
    const int tq = tile / tpi, t2 = tile - tq * tpi, ty = t2 / TX, tx = t2 - ty * TX, img = tq * IX;
    const int y0 = ty * PH - 1, x0 = tx * PW - 1;
    char* st = smem + buf * STAGE;
    const int hcnt = HIN / NW + (wave < HIN % NW), hbeg = wave * (HIN / NW) + min(wave, HIN % NW);
    const int wcnt = WIN / NW + (wave < WIN % NW), wbeg = wave * (WIN / NW) + min(wave, WIN % NW);
#pragma unroll
    for (int i = 0; i < HI; ++i) {
      if (i < k0 || i >= k1 || i >= hcnt) continue;
      const int hr = (hbeg + i) * RPI + sub;
      const int hy = hr / HW, hx = hr - hy * HW;
      int ys = y0 + hy, xs = x0 + hx, im = img;
      if constexpr (IX > 1) {                         // image b, column hx - b (IW + 1) - 1 (-1: a pad)
        const int b = min(hx / (IW + 1), IX - 1);
        xs = hx - b * (IW + 1) - 1;
        im = img + b;
      }
      const bool ok = live && hr < HR && ys >= 0 && xs >= 0 && ys < a.Hs && xs < (IX > 1 ? IW : a.Ws);
      const uint32_t off =
          ok ? (uint32_t)((((im * a.Hs + ys) * a.Ws + xs) * a.scs + cc * 32 + swzh(hx, slot) * 8) * 2) : BAD;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs_src, (__attribute__((address_space(3))) void*)(st + (hbeg + i) * RPI * 64), 16, off, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < WI; ++i) {
      if (HI + i < k0 || HI + i >= k1 || !wload || i >= wcnt) continue;
      const int wr = (wbeg + i) * RPI + sub;            // weight row = tap * 64 + n
      const int wrow = wr & 63;
      const int tap = wr >> 6,
                n = nt * BN + (DIRECT ? ((wrow >> 5) * 32 + ((wrow >> 2) & 3) * 8 + ((wrow >> 4) & 1) * 4 + (wrow & 3))
                                      : wrow);
      const bool ok = live && wr < 9 * BN;
      const uint32_t off = ok ? (uint32_t)(((size_t)n * a.K + tap * a.Cs + cc * 32 + swzh(wr, slot) * 8) * 2) : BAD;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs_wgt, (__attribute__((address_space(3))) void*)(st + (HROWS + (wbeg + i) * RPI) * 64), 16, off, 0,
          0, 0);
    }
  };
  auto issue = [&](int item, int cc, int buf, bool live, bool wload = true) {
    issue_part(item, cc, buf, live, 0, HI + WI, wload);
  };
  // does filling stage buf with (item, cc) need the weight DMA?  (and record what it holds)
  auto need_w = [&](int item, int cc, int buf, bool live) {
    if (STAGES != 2 || !a.wkeep || !live) return true;
    const int key = (item / ntiles) * CC + cc;
    int& held = buf ? wkey1 : wkey0;
    const bool need = held != key;
    held = key;
    return need;
  };

  // byte offset (within a stage) of this lane's halo read for fragment i at tap column dx,
  // tap row 0: the swizzle is keyed on the halo column, so the tap row dy only adds the
  // immediate dy * HW * 64 (12 address registers instead of one per (i, tap))
  int xb[TM][3];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int p = wave * WTM + i * 16 + fr;
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) {
      const int px = p % PW, hx = px + px / IW * (IX > 1 ? 1 : 0) + dx;   // + one shared pad per image
      xb[i][dx] = ((p / PW) * HW + hx) * 64 + swzh(hx, fk) * 16;
    }
  }
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (STAGES == 2) issue(it0, 0, 0, true, need_w(it0, 0, 0, true));
  int iit = it0, icc = 0;                               // issue cursor (last issued stage)
  int cit = it0, ccc = 0;                               // compute cursor
  // BN partial statistics, one row per (group, workgroup): stats [groups][gridDim][2][Nout].
  // Thread tid < 128 owns (sum | sum of squares, channel col) of the current (group, slice) and
  // zeroes its rows first (same thread, same addresses: ordered).  DF: the two wave halves finish
  // an item on opposite sides of a barrier, so there is no per-item cross-wave pass: every lane
  // keeps its wave's running partials of the last KMAX (group, slice) keys in registers (lane (fr,
  // fk), fragment half h: row half fr >> 3, channel h*32 + fk*8 + (fr & 7), where
  // row16_reduce_scatter leaves them; the host checks a workgroup's item run spans <= KMAX keys)
  // and the waves' partials are folded once, in wave order, after the loop.
  constexpr int KMAX = 2;
  const int q_st = tid >> 6, col_st = tid & 63;
  const int groups = a.M / a.Mg;
  int run_key = -1;
  float run = 0.f;
  float kr[KMAX][2];                                     // DF: running partials, newest key first
  int kv[KMAX], nk = 0;                                  // DF: their keys (wave-uniform)
#pragma unroll
  for (int k = 0; k < KMAX; ++k) { kr[k][0] = kr[k][1] = 0.f; kv[k] = -1; }
  // BNR: the same rows hold the fused BN-backward partials (sum g, sum g*xhat)
  float* const sbuf = BNR ? a.bnr_part : (DIRECT == 1 ? nullptr : a.stats);
  auto srow = [&](int g) { return (size_t)(g * gridDim.x + vb); };
  auto flush = [&]() {
    const int g = run_key / NTn, nt = run_key - g * NTn;
    sbuf[(srow(g) * 2 + q_st) * a.Nout + nt * BN + col_st] = run;
  };
  if (sbuf && tid < 128) {
    for (int g = 0; g < groups; ++g)
      for (int nt = 0; nt < NTn; ++nt) sbuf[(srow(g) * 2 + q_st) * a.Nout + nt * BN + col_st] = 0.f;
  }
  // BNR: this wave's copy of the BatchNorm affine of the current (group, slice) in LDS,
  // [scale | shift | mean | invstd][64 channels], reloaded when the key changes
  float* const aff = reinterpret_cast<float*>(smem + AFF) + wave * 256;
  int aff_key = -1, bias_key = -1;
  bool epi = false;                                      // previous stage ended with an epilogue (8 stores)
  bool wl_next = true;                                   // the next fill streams weight rows too
  bool pend = false;                                     // DF: this wave owes item pend_it's epilogue
  int pend_it = 0;
  f32x4 bv[TN];                                          // bias of the lane's 16 accumulator channels
#pragma unroll
  for (int j = 0; j < TN; ++j) bv[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // DIAG 4: per-wave cycle buckets (s_memtime) -- DMA wait, barrier, DMA issue, taps, epilogue
  uint64_t tb[5] = {0, 0, 0, 0, 0}, tprev = 0;
  auto stamp = [&](int k) {
    if constexpr (DIAG == 4) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      if (k >= 0) tb[k] += t - tprev;
      tprev = t;
    }
  };

  // ---- direct epilogue of item `item` from acc / bv: lane (fr, fk) holds pixel p's channels
  // 8fk..8fk+7 (fragments 0,1) and 32+8fk.. (2,3).  Order: pack the accumulators (64 fp32 -> 32
  // bf16x2 registers, the accumulators die), [BNR: the y tile], the dz stores, then the partial
  // sums from the packed (stored, rounded) values.  Every load precedes every store (vmcnt
  // retires in order: a later load would wait for the stores in front of it); invalid pixels get
  // an out-of-range offset, so every lane issues exactly NSTORE = 2 * TM stores.  Sums: DPP
  // reduce-scatter over the 16 pixels of a fragment row; without DF one LDS pass over the
  // waves (the stage just read is the scratch: `buf`).
  auto direct_epi = [&](int item, int buf) {
    const int nt = item / ntiles, tile = item - nt * ntiles;
    const int tq = tile / tpi, t2 = tile - tq * tpi, ty = t2 / TX, tx = t2 - ty * TX, img = tq * IX;
    const uint32_t dst_records = (uint32_t)((size_t)a.M * a.dcs * 2);
    const __amdgpu_buffer_rsrc_t rs_dst = __builtin_amdgcn_make_buffer_rsrc((void*)a.dst, 0, dst_records, 0x00020000);
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    uint4 uq[2][TM];
    int mq[TM];
    // bias of the lane's 16 accumulator channels: DF -- from the wave's LDS copy of the slice's
    // biases (no registers held across the stage), else the registers load_bias filled
    f32x4 be[TN];
    if constexpr (DF) {
#pragma unroll
      for (int j = 0; j < TN; ++j) be[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (!BNR && a.bias) {
        if (nt != bias_key) {                          // same-wave LDS write -> read: ordered
          bias_key = nt;
          aff[lane] = a.bias[nt * BN + lane];
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) be[j] = *reinterpret_cast<const f32x4*>(aff + (j >> 1) * 32 + fk * 8 + (j & 1) * 4);
      }
    } else {
#pragma unroll
      for (int j = 0; j < TN; ++j) be[j] = bv[j];
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int p = wave * WTM + i * 16 + fr;
      mq[i] = halo_pixel<PH, PW, IX>(p, img, ty, tx, a.Hd, a.Wd);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float f[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          f[r] = acc[i][2 * h][r] + be[2 * h][r];
          f[4 + r] = acc[i][2 * h + 1][r] + be[2 * h + 1][r];
        }
        if (a.accumulate && mq[i] >= 0) {
          float o[8];
          unpack8(*reinterpret_cast<const uint4*>(a.dst + (size_t)mq[i] * a.dcs + nt * BN + h * 32 + fk * 8), o);
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] += o[e];
        }
        uq[h][i] = pack8(f);
        acc[i][2 * h] = f32x4{0.f, 0.f, 0.f, 0.f};
        acc[i][2 * h + 1] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    const int key = (img / ipg) * NTn + nt;
    float* red = reinterpret_cast<float*>(smem + buf * STAGE);   // [NW][2][64]
    // BNR scratch without DF: y rows [WTM][128 B] per wave in the stage just read, after the
    // [NW][2][64] reduction rows (16-B chunk c of pixel row r at slot c ^ (r & 7): conflict-free)
    char* yl = smem + buf * STAGE + NW * 2 * 64 * 4 + wave * WTM * 128;
    uint4 yq[2][TM];
    if constexpr (BNR) {
      if (key != aff_key) {                             // this wave's affine of (group, slice)
        aff_key = key;
        const size_t o = (size_t)(img / ipg) * a.Nout + nt * BN + lane;
        const float v0 = a.bnr_scale[o], v1 = a.bnr_shift[o], v2 = a.bnr_mean[o], v3 = a.bnr_invstd[o];
        aff[lane] = v0; aff[64 + lane] = v1; aff[128 + lane] = v2; aff[192 + lane] = v3;
      }
      const __amdgpu_buffer_rsrc_t rs_y = __builtin_amdgcn_make_buffer_rsrc(
          (void*)a.bnr_y, 0, (uint32_t)((size_t)a.M * a.bnr_ycs * 2), 0x00020000);
      if constexpr (DF) {
        // y straight to registers (the accumulators are dead): lane (fr, fk) loads exactly the
        // 8 channels of pixel i*16+fr that it holds in uq[h][i]
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            const uint32_t off =
                mq[i] >= 0 ? (uint32_t)(((size_t)mq[i] * a.bnr_ycs + nt * BN + h * 32 + fk * 8) * 2) : 0xFFFFFFF0u;
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs_y, off, 0, 0);
            yq[h][i] = make_uint4(v.x, v.y, v.z, v.w);
          }
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();                   // every wave is done reading this stage
        (buf ? wkey1 : wkey0) = -1;                     // the y rows overwrite its weight rows
#pragma unroll
        for (int k = 0; k < WTM / 8; ++k) {
          const int r = k * 8 + (lane >> 3), p = wave * WTM + r;       // 8 pixel rows per instruction
          const int m = halo_pixel<PH, PW, IX>(p, img, ty, tx, a.Hd, a.Wd);
          const int c = (lane & 7) ^ (r & 7);
          const uint32_t off = m >= 0 ? (uint32_t)(((size_t)m * a.bnr_ycs + nt * BN + c * 8) * 2) : 0xFFFFFFF0u;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(
              rs_y, (__attribute__((address_space(3))) void*)(yl + k * 1024), 16, off, 0, 0, 0);
        }
      }
    }
    if (!BNR && IX == 1 && a.full) {
      // (not with the fused BN-backward reduction, nor in the multi-image kernels: their registers
      // leave no room -- they spilled)
      // lane (fr, fk) holds chunks fk (h = 0) and 4 + fk (h = 1) of pixel i*16 + fr: its h = 1 chunk
      // and pixel index go to lane fr ^ 8 (DPP row_ror:8), so each store writes 8 whole 128-B pixel
      // rows (pixels 0-7 of the group, then 8-15) instead of half of 16 -- as many stores
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const uint4 u1 = uq[1][i];
        const uint4 rcv = make_uint4(__builtin_amdgcn_update_dpp(0u, u1.x, 0x128, 0xF, 0xF, false),
                                     __builtin_amdgcn_update_dpp(0u, u1.y, 0x128, 0xF, 0xF, false),
                                     __builtin_amdgcn_update_dpp(0u, u1.z, 0x128, 0xF, 0xF, false),
                                     __builtin_amdgcn_update_dpp(0u, u1.w, 0x128, 0xF, 0xF, false));
        const int mx = __builtin_amdgcn_update_dpp(0, mq[i], 0x128, 0xF, 0xF, false);
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          const bool own = (half == 0) == (fr < 8);
          const uint4 v = own ? uq[0][i] : rcv;
          const int m = own ? mq[i] : mx;
          const int ch = (own ? 0 : 32) + fk * 8;
          const uint32_t off = m >= 0 ? (uint32_t)(((size_t)m * a.dcs + nt * BN + ch) * 2) : 0xFFFFFFF0u;
          __builtin_amdgcn_raw_buffer_store_b128(u32x4{v.x, v.y, v.z, v.w}, rs_dst, off, 0, 0);
        }
      }
    } else {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const uint4 u = uq[h][i];
          const uint32_t off =
              mq[i] >= 0 ? (uint32_t)(((size_t)mq[i] * a.dcs + nt * BN + h * 32 + fk * 8) * 2) : 0xFFFFFFF0u;
          __builtin_amdgcn_raw_buffer_store_b128(u32x4{u.x, u.y, u.z, u.w}, rs_dst, off, 0, 0);
        }
    }
    float res[2] = {0.f, 0.f};                           // row16_reduce_scatter results per half
    if constexpr (BNR) {
      // g = dz * [y*scale+shift > 0]; (sum g, sum g*xhat), like stf_bn_bwd_reduce
      // the y loads (issued before the stores) have landed; the stores stay in flight
      asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * TM) : "memory");
      auto aff8 = [&](int k, int c0, float* v) {
        const float4 lo = *reinterpret_cast<const float4*>(aff + k * 64 + c0);
        const float4 hi = *reinterpret_cast<const float4*>(aff + k * 64 + c0 + 4);
        v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w; v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
      };
      const bool norelu = !a.bnr_relu;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        // sum g*y per lane (TM pixels), turned into sum g*xhat = invstd*(sum g*y - mean*sum g)
        float q1[8], q2[8], sc[8], sh[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) { q1[e] = 0.f; q2[e] = 0.f; }
        aff8(0, h * 32 + fk * 8, sc);
        aff8(1, h * 32 + fk * 8, sh);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          float g[8], yv[8];
          unpack8(uq[h][i], g);
          const int r = i * 16 + fr;
          if constexpr (DF) unpack8(yq[h][i], yv);
          else unpack8(*reinterpret_cast<const uint4*>(yl + r * 128 + (((h * 4 + fk) ^ (r & 7)) << 4)), yv);
          const bool valid = mq[i] >= 0;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            // bitwise, not short-circuit: a select, no branch
            const bool keep = valid & (norelu | (yv[e] * sc[e] + sh[e] > 0.f));
            const float gg = keep ? g[e] : 0.f;
            q1[e] += gg;
            q2[e] += gg * yv[e];
          }
        }
        float mu[8], is[8], v[16];
        aff8(2, h * 32 + fk * 8, mu);
        aff8(3, h * 32 + fk * 8, is);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          v[e] = q1[e];
          v[8 + e] = is[e] * (q2[e] - mu[e] * q1[e]);
        }
        res[h] = row16_reduce_scatter(v, fr);
      }
    } else if constexpr (DIRECT == 2) {
      // BN statistics (sum, sum of squares) of the stored values
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float v[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) v[e] = 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          float g[8];
          unpack8(uq[h][i], g);
          const float w = mq[i] >= 0 ? 1.f : 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) { v[e] += w * g[e]; v[8 + e] += w * g[e] * g[e]; }
        }
        // lane fr ends with value fr: sum (fr < 8) or sum of squares of channel fr & 7
        res[h] = row16_reduce_scatter(v, fr);
      }
      if constexpr (!DF) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();                   // every wave is done reading this stage
      }
    }
    if (sbuf) {
      if constexpr (DF) {
        // this wave's running partials of the current (group, slice); a new key shifts them
        if (nk == 0 || key != kv[0]) {
#pragma unroll
          for (int k = KMAX - 1; k > 0; --k) { kr[k][0] = kr[k - 1][0]; kr[k][1] = kr[k - 1][1]; kv[k] = kv[k - 1]; }
          kr[0][0] = kr[0][1] = 0.f;
          kv[0] = key;
          ++nk;
        }
        kr[0][0] += res[0];
        kr[0][1] += res[1];
      } else {
#pragma unroll
        for (int h = 0; h < 2; ++h) red[(wave * 2 + (fr >> 3)) * 64 + h * 32 + fk * 8 + (fr & 7)] = res[h];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (tid < 128) {
          const int q = tid >> 6, col = tid & 63;
          float t = 0.f;
#pragma unroll
          for (int w = 0; w < NW; ++w) t += red[(w * 2 + q) * 64 + col];
          if (key != run_key) {
            if (run_key >= 0) flush();
            run_key = key;
            run = 0.f;
          }
          run += t;
        }
      }
    }
  };

  // DF: one more pass through the loop head after the last stage runs the last epilogue
  for (int s = 0; s < S + (DF ? 1 : 0); ++s) {
    const int buf = STAGES == 2 ? (s & 1) : 0;
    stamp(-1);
    auto load_bias = [&]() {
      // bias of this lane's 16 accumulator channels, loaded BEFORE the next DMA so
      // that waiting for it never waits for the DMA (BNR: a dgrad, no bias)
      if constexpr (BNR || (DF && DIRECT)) {           // (DF: direct_epi reads them from LDS)
#pragma unroll
        for (int j = 0; j < TN; ++j) bv[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      } else if (ccc == CC - 1) {
        const int nt = cit / ntiles;
#pragma unroll
        for (int j = 0; j < TN; ++j)
          bv[j] = __builtin_amdgcn_raw_buffer_load_b128(
            rs_bias, (nt * BN + (DIRECT ? (j >> 1) * 32 + fk * 8 + (j & 1) * 4 : j * 16 + fk * 4)) * 4, 0, 0);
      }
    };
    if constexpr (STAGES == 2) {
      // retire this stage's DMA; the previous epilogue's NSTORE buffer stores
      // (issued after it, stores and loads retire in order) may stay in flight
      if (epi) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NSTORE) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      stamp(0);
      epi = false;
      if constexpr (DF) {
        // the epilogue of the item that ended with the previous stage: the first wave half runs
        // it before this stage barrier, the second half (its SIMD partners) after it, ahead of
        // its taps -- one code site, the barrier instruction placed by wave half (s_barrier
        // counts arrivals, not program points; `late` is wave-uniform)
        if (late) __builtin_amdgcn_s_barrier();
        if (pend) { direct_epi(pend_it, buf ^ 1); pend = false; }
        if (!late) __builtin_amdgcn_s_barrier();
        if (s == S) break;
      } else {
        __builtin_amdgcn_s_barrier();
      }
      stamp(1);
      load_bias();
      const bool live = s + 1 < S;
      if (live && ++icc == CC) { icc = 0; ++iit; }
      wl_next = need_w(iit, icc, (s + 1) & 1, live && (DIAG != 2 || s < 1));
      // the first wave half issues the next stage's DMA now, the second (DF: its SIMD partners,
      // waves >= NW/2; else the odd waves) after tap 4: the address path takes ~300 cycles per 1-KiB
      // LDS-DMA instruction under load, and with all eight waves issuing at once both waves of a
      // SIMD stalled together (DIAG 4: a third of the time); staggered, one wave of each SIMD
      // computes while the other issues
      if (!STAGGER || (!late && HALO_ATAP < 0)) issue(iit, icc, (s + 1) & 1, live && (DIAG != 2 || s < 1), wl_next);
      stamp(2);
    } else {
      // single stage: every wave is done with the buffer, refill it, wait
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      load_bias();
      issue(cit, ccc, 0, DIAG != 2 || s < 1);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
    const char* hb = smem + buf * STAGE;
    if (DIAG == 3) { if (++ccc == CC) { ccc = 0; ++cit; } continue; }
    const char* wb = hb + HROWS * 64;
    // software-pipelined taps: tap t+1's fragments are read while tap t's TM x TN MFMAs
    // run (double-buffered registers).  The reads are inline-asm ds_read_b128 (kept in
    // issue order; the compiler otherwise sinks them next to their MFMAs and exposes the
    // LDS latency) and the wait is explicit: lgkmcnt(TM + TN) leaves exactly the tap-t+1
    // reads in flight, and it passes tap t's fragments through as operands so no MFMA
    // can be scheduled above it.  All reads have retired (lgkmcnt(0)) by the last tap.
    e16x8 xf[2][TM], wf[2][TN];
    const uint32_t hb32 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const char*)hb;
    const uint32_t wrow0 = (uint32_t)((HROWS + fr) * 64 + swzh(fr, fk) * 16);    // weight row j*16+fr of tap 0
    auto rd_tap = [&](int t, int b) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
        asm volatile("ds_read_b128 %0, %1 offset:%2"
                     : "=v"(xf[b][i]) : "v"(hb32 + xb[i][t % 3]), "i"((t / 3) * HW * 64));
#pragma unroll
      for (int j = 0; j < TN; ++j)                 // (row >> 1) & 2 of t*64 + j*16 + fr = that of fr
        asm volatile("ds_read_b128 %0, %1 offset:%2"
                     : "=v"(wf[b][j]) : "v"(hb32 + wrow0), "i"((t * BN + j * 16) * 64));
    };
    rd_tap(0, 0);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int b = t & 1;
      if constexpr (STAGGER) {
        if (t == (late ? 4 : HALO_ATAP)) issue(iit, icc, (s + 1) & 1, s + 1 < S && (DIAG != 2 || s < 1), wl_next);
      }
      if (t + 1 < 9) rd_tap(t + 1, b ^ 1);
      // wait for tap t's fragments (the TM + TN tap-t+1 reads may stay in flight)
      static_assert(TN == 4 && (TM == 4 || TM == 2), "fragment wait");
      if constexpr (TM == 4) {
        if (t + 1 < 9)
          asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(xf[b][0]), "+v"(xf[b][1]), "+v"(xf[b][2]), "+v"(xf[b][3]),
                       "+v"(wf[b][0]), "+v"(wf[b][1]), "+v"(wf[b][2]), "+v"(wf[b][3]));
        else
          asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(xf[b][0]), "+v"(xf[b][1]), "+v"(xf[b][2]), "+v"(xf[b][3]),
                       "+v"(wf[b][0]), "+v"(wf[b][1]), "+v"(wf[b][2]), "+v"(wf[b][3]));
      } else {
        if (t + 1 < 9)
          asm volatile("s_waitcnt lgkmcnt(6)" : "+v"(xf[b][0]), "+v"(xf[b][1]),
                       "+v"(wf[b][0]), "+v"(wf[b][1]), "+v"(wf[b][2]), "+v"(wf[b][3]));
        else
          asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(xf[b][0]), "+v"(xf[b][1]),
                       "+v"(wf[b][0]), "+v"(wf[b][1]), "+v"(wf[b][2]), "+v"(wf[b][3]));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = mfma16x16x32(wf[b][j], xf[b][i], acc[i][j]);
    }
    stamp(3);
    if (DIRECT && ccc + 1 == CC) {
      if constexpr (DF) {                              // at the next loop head
        pend = true;
        pend_it = cit;
      } else {
        direct_epi(cit, buf);
        epi = true;
      }
      stamp(4);
      ccc = 0;
      ++cit;
      continue;
    }
    if constexpr (DIRECT) {                            // (the last chunk took the branch above)
      ++ccc;
      continue;
    }
    if (++ccc == CC) {
      // ---- epilogue through LDS: the stage just read becomes the output tile
      // [PX][64] bf16 (128-B rows, 16-B chunk c at c ^ (p & 7)); full-row 16-B
      // buffer stores (invalid pixels get an out-of-range offset, so every lane
      // issues exactly NSTORE stores and the next stage can wait with vmcnt(NSTORE));
      // BN partial sums from the stored values; raw barriers only, so nothing
      // drains the stores or the DMA already in flight.
      const int nt = cit / ntiles, tile = cit - nt * ntiles;
      const int tq = tile / tpi, t2 = tile - tq * tpi, ty = t2 / TX, tx = t2 - ty * TX, img = tq * IX;
      char* ot = smem + buf * STAGE;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();                     // every wave is done reading this stage
      (buf ? wkey1 : wkey0) = -1;                       // the output tile overwrites its weight rows
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int p = wave * WTM + i * 16 + fr;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int ch = j * 16 + fk * 4, c16 = ch >> 3;
          const uint2 v = make_uint2(pack2(acc[i][j][0] + bv[j][0], acc[i][j][1] + bv[j][1]),
                                     pack2(acc[i][j][2] + bv[j][2], acc[i][j][3] + bv[j][3]));
          *reinterpret_cast<uint2*>(ot + p * 128 + ((c16 ^ (p & 7)) << 4) + (ch & 7) * 2) = v;
          acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      const int c16 = tid & 7;
      const uint32_t dst_records = (uint32_t)((size_t)a.M * a.dcs * 2);
      const __amdgpu_buffer_rsrc_t rs_dst = __builtin_amdgcn_make_buffer_rsrc((void*)a.dst, 0, dst_records, 0x00020000);
      float s1[8], s2[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
#pragma unroll
      for (int k = 0; k < NSTORE; ++k) {
        const int p = (tid >> 3) + PPP * k;
        const int mm = halo_pixel<PH, PW, IX>(p, img, ty, tx, a.Hd, a.Wd);
        const bool ok = mm >= 0;
        const int m = ok ? mm : 0;
        uint4 u = *reinterpret_cast<const uint4*>(ot + p * 128 + ((c16 ^ (p & 7)) << 4));
        const uint32_t off = ok ? (uint32_t)(((size_t)m * a.dcs + nt * BN + c16 * 8) * 2) : 0xFFFFFFF0u;
        float f[8];
        unpack8(u, f);
        if (a.accumulate && ok) {
          float o[8];
          unpack8(*reinterpret_cast<const uint4*>(a.dst + (size_t)m * a.dcs + nt * BN + c16 * 8), o);
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] = round_e(f[e] + o[e]);
          u = pack8(f);
        }
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{u.x, u.y, u.z, u.w}, rs_dst, off, 0, 0);
        if (ok) {
#pragma unroll
          for (int e = 0; e < 8; ++e) { s1[e] += f[e]; s2[e] += f[e] * f[e]; }
        }
      }
      if (a.stats) {
        // lanes with equal (lane & 7) hold the same 8 channels: fold 8 -> 1 per wave, then over waves
#pragma unroll
        for (int e = 0; e < 8; ++e)
#pragma unroll
          for (int o = 8; o < 64; o <<= 1) {
            s1[e] += __shfl_xor(s1[e], o, 64);
            s2[e] += __shfl_xor(s2[e], o, 64);
          }
        float* red = reinterpret_cast<float*>(ot + PX * 128);   // [NW][2][64]
        if (lane < 8) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            red[(wave * 2 + 0) * 64 + lane * 8 + e] = s1[e];
            red[(wave * 2 + 1) * 64 + lane * 8 + e] = s2[e];
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (tid < 128) {
          const int q = tid >> 6, col = tid & 63;
          float t = 0.f;
#pragma unroll
          for (int w = 0; w < NW; ++w) t += red[(w * 2 + q) * 64 + col];
          const int key = (img / ipg) * NTn + nt;
          if (key != run_key) {
            if (run_key >= 0) flush();
            run_key = key;
            run = 0.f;
          }
          run += t;
        }
      }
      ccc = 0;
      ++cit;
      epi = true;
    }
  }
  if constexpr (DF) {
    if (sbuf) {
      // every wave has left the loop (the second half after its last epilogue) and every DMA has
      // landed (the loop head's vmcnt(0)): the ring is free.  Partials [KMAX][NW][2][64] fp32,
      // folded in wave order by the threads that own the rows.
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      float* part = reinterpret_cast<float*>(smem);
      const int nkk = nk < KMAX ? nk : KMAX;
#pragma unroll
      for (int k = 0; k < KMAX; ++k)
        if (k < nkk)
#pragma unroll
          for (int h = 0; h < 2; ++h)
            part[((k * NW + wave) * 2 + (fr >> 3)) * 64 + h * 32 + fk * 8 + (fr & 7)] = kr[k][h];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (tid < 128) {
        for (int k = 0; k < nkk; ++k) {
          float t = 0.f;
#pragma unroll
          for (int w = 0; w < NW; ++w) t += part[((k * NW + w) * 2 + q_st) * 64 + col_st];
          run_key = kv[k];
          run = t;
          flush();
        }
      }
    }
  } else {
    if (sbuf && tid < 128 && run_key >= 0) flush();
  }
  if constexpr (DIAG == 4) {                           // a.stats doubles as the [grid][NW][8] u64 buffer
    if (lane == 0) {
      unsigned long long* d = reinterpret_cast<unsigned long long*>(a.stats) + (vb * NW + wave) * 8;
#pragma unroll
      for (int k = 0; k < 5; ++k) d[k] = tb[k];
    }
  }
}

template <int PH, int PW, int NW, int STAGES, int DIAG, int DIRECT = 0, bool BNR = false, bool DEFER = false>
__global__ __launch_bounds__(64 * NW, (STAGES == 1) ? 2 : 1) void conv3x3_halo_kernel(Geo a, uint32_t src_bytes,
                                                                                    int TY, int TX, int per, int rem) {
  halo_body<PH, PW, NW, STAGES, DIAG, DIRECT, BNR, 1, DEFER>(a, src_bytes, TY, TX, per, rem);
}

// two 16 x 16 images per 16 x 32 tile (IX = 2); TY = TX = 1
template <int DIRECT, bool BNR, bool DEFER = false>
__global__ __launch_bounds__(512, 1) void conv3x3_halo2_kernel(Geo a, uint32_t src_bytes, int TY, int TX, int per,
                                                               int rem) {
  halo_body<16, 32, 8, 2, 0, DIRECT, BNR, 2, DEFER>(a, src_bytes, TY, TX, per, rem);
}

// four 8 x 8 images per 8 x 32 tile (IX = 4; STF layer4), 4 waves, one stage, two workgroups per
// CU (61 KB of LDS each): one workgroup's DMA waits hide behind the other's MFMAs.  (A 2-stage
// ring at one workgroup per CU, for grids under 2 x CUs, was faster alone -- forward 64 -> 61 us,
// BN-backward dgrad 84 -> 66 us -- but its 123 KB of LDS kept the side streams' weight gradients
// and LSTMs off the CU: the STF step -0.5 % over five same-box repeats; removed in round 6.)
template <int DIRECT>
__global__ __launch_bounds__(256, 2) void conv3x3_halo4_kernel(Geo a, uint32_t src_bytes, int TY, int TX, int per,
                                                               int rem) {
  halo_body<8, 32, 4, 1, 0, DIRECT, false, 4>(a, src_bytes, TY, TX, per, rem);
}

// ---------------------------------------------------------------------------
// Wide halo kernel (round 6): the same 3x3 / stride 1 / pad 1 convolution as halo_body, for layers
// with >= 128 output channels, with a 16 x 32 pixel tile x 128-channel output slice per item
// (twice the outputs per workgroup: 128 accumulator registers per lane, wave tile 64 pixels x 128
// channels).  Per 32-channel source chunk (one "stage") the workgroup needs the (16+2) x (32+2)
// halo (39 KB, as halo_body) and 9 x 128 weight rows (74 KB): the same halo bytes for twice the
// MFMAs, 26 % fewer LDS-fill bytes per FLOP than the 64-channel slice.  Two whole stages do not
// fit in 160 KiB, so the weights are not double-buffered by stage: they live in two tap-group
// buffers (G0 = taps 0-4, G1 = taps 5-8), each refilled as soon as every wave has finished its taps
// -- G0 of the next chunk streams in while G1 of this chunk computes.  One barrier per group
// ("point"; a 3-group variant measured 1-2 % slower per layer):
//   P0(s): wait halo(s) + G0(s);  issue G1(s), halo(s+1)   [then taps 0-4 from G0]
//   P1(s): wait G1(s);            issue G0(s+1)            [taps 5-8 from G1]
// (the weights are L2-resident: 4-5 taps of MFMAs cover their fill; the halo has a whole stage).
// Every wave issues the same count at every point (4 + 5 and 5 DMA instructions, past the last
// stage with all lanes out of range), so the waits are fixed vmcnt values.  The first tap of G1
// reads its halo fragments before the P1 barrier.  Every wave issues its fills in one burst right
// after each barrier (measured against the alternatives: waves 4..7 after their first MFMA block
// -- WIDE_STAGGER, spills; the pieces spread through the taps; one wave per SIMD issuing for
// both -- all slower).  Direct epilogue (16-B stores of 8 consecutive
// channels, weight rows fetched in the permuted order of halo_body's DIRECT), BatchNorm partial
// statistics as halo_body's non-deferred path (one row per (group, workgroup)), the slice's biases
// by one LDS-DMA of wave 0 per item.  DIRECT: 2 = forward with statistics, 1 = no statistics (dgrad,
// eval forward); BNR (with 1): the BN-backward-fused dgrad.
#ifndef WIDE_ABL          // timing-only ablations (results wrong): 1 = half the B-fragment LDS reads,
#define WIDE_ABL 0        // 2 = no LDS-DMA fills after the first stage (3: no weight fills, 4: no halo fills,
                          // 5: every item's halo from tiles 0 / 1 (L2 hits))
#endif
#ifndef WIDE_STAGGER
#define WIDE_STAGGER 0
#endif
namespace wide {
constexpr int NW = 8, PH = 16, PW = 32, BN = 128, RPI = 16;
constexpr int HW = PW + 2, HR = (PH + 2) * HW;          // 612 halo rows
constexpr int HIN = 40, HPW = HIN / NW;                 // halo DMA instructions per stage: 5 per wave
constexpr int HSTAGE = HIN * RPI * 64;                  // 40960 B (rows >= 612 stay zero, never read)
// two weight groups per stage: G0 = taps 0-4 (640 rows, 5 DMA instructions per wave), G1 = taps 5-8
// (512 rows, 4 per wave)
constexpr int G1T = 5;                                  // first tap of G1
constexpr int GPW0 = G1T * BN / RPI / NW, GPW1 = (9 - G1T) * BN / RPI / NW;
constexpr int G0BYTES = G1T * BN * 64;                  // 40960 B
constexpr int WOFF = 2 * HSTAGE;                        // 81920: G0, then G1 at WOFF + G0BYTES
constexpr int BOFF = WOFF + 9 * BN * 64;                // 155648: the slice's 128 biases (1 KiB DMA target)
constexpr int ROFF = BOFF + 1024;                       // 156672: running statistics partials [2][128] fp32
constexpr int AOFF = ROFF + 1024;                       // 157696: BNR -- the item's BatchNorm affine
                                                        // [scale | shift | mean | invstd][128] fp32, 1 KiB DMA slot each
constexpr int LDS = AOFF + 4096;                        // 161792
constexpr int TM = 4, TN = 8, NST = 2 * TN;             // 16 epilogue stores per lane
static_assert(HIN * RPI >= HR && HIN % NW == 0 && G1T * BN % (RPI * NW) == 0 && (9 - G1T) * BN % (RPI * NW) == 0,
              "wide halo geometry");
static_assert(NW * 2 * BN * 4 <= (9 - G1T) * BN * 64, "statistics scratch in the G1 weight buffer");
}

// BNR (with DIRECT 1): the dgrad's output dz feeds the backward of ReLU(BN(y)); the epilogue also
// reduces the BatchNorm-backward partials (sum g, sum g*xhat), g = dz * [y*scale+shift > 0], as
// halo_body's BNR (same partial rows), y read per 32-channel block into registers
template <int DIRECT, bool BNR = false>
__global__ __launch_bounds__(512, 1) void conv3x3_wide_kernel(Geo a, uint32_t src_bytes, int TY, int TX, int per,
                                                              int rem) {
  using namespace wide;
  static_assert(!BNR || DIRECT == 1, "BNR: a dgrad, no statistics");
  __shared__ __attribute__((aligned(16))) char smem[LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fk = lane >> 4, sub = lane >> 2, slot = lane & 3;
  const int NTn = a.Nout / BN, CC = a.Cs / 32, tpi = TY * TX;
  const int ntiles = a.N * tpi;
  const int ipg = a.Mg / (a.Hd * a.Wd);
  const int vb = blockIdx.x;
  const int cnt = per + (int)(vb < rem);
  const int it0 = vb * per + min(vb, rem);
  const int S = cnt * CC;
  const bool has_bias = a.bias != nullptr;             // (eval-mode forwards run without statistics, with bias)
  const __amdgpu_buffer_rsrc_t rs_src = __builtin_amdgcn_make_buffer_rsrc((void*)a.src, 0, src_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_wgt =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.wgt, 0, (uint32_t)a.Nout * a.K * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_bias =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.bias, 0, a.bias ? (uint32_t)a.Nout * 4 : 0u, 0x00020000);
  constexpr uint32_t BAD = 0xFFFFFFF0u;
  typedef __attribute__((address_space(3))) void* lds_ptr;

  // stage s = (item it0 + s / CC, chunk s % CC); s >= S: not live (all lanes out of range)
  auto issue_halo = [&](int s) {
    const bool live = s < S;
    const int item = it0 + (live ? s / CC : 0), cc = live ? s % CC : 0;
    const int tile = WIDE_ABL == 5 ? item % 2 : item % ntiles;
    const int img = tile / tpi, t2 = tile - img * tpi, ty = t2 / TX, tx = t2 - ty * TX;
    const int y0 = ty * PH - 1, x0 = tx * PW - 1;
    char* st = smem + (s & 1) * HSTAGE;
    // the lane's row terms are recomputed at every issue (opaque copy): kept live across the taps
    // they would cost ~20 registers that the accumulators need
    int sb = sub;
    asm volatile("" : "+v"(sb));
#pragma unroll
    for (int i = 0; i < HPW; ++i) {
      const int hr = (wave * HPW + i) * RPI + sb;
      const int hy = hr / HW, hx = hr - hy * HW;
      const int ys = y0 + hy, xs = x0 + hx;
      const bool ok = live && hr < HR && ys >= 0 && xs >= 0 && ys < a.Hs && xs < a.Ws;
      const uint32_t off =
          ok ? (uint32_t)((((img * a.Hs + ys) * a.Ws + xs) * a.scs + cc * 32 + swzh(hx, slot) * 8) * 2) : BAD;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_src, (lds_ptr)(st + (wave * HPW + i) * RPI * 64), 16, off, 0, 0, 0);
    }
  };
  // weight rows of tap group g of stage s into its buffer: row (tap - first tap) * 128 + wrow
  auto issue_w = [&](int s, auto gc) {
    constexpr int g = decltype(gc)::value, GPW = g ? GPW1 : GPW0;
    const bool live = s < S;
    const int item = it0 + (live ? s / CC : 0), cc = live ? s % CC : 0;
    const int nt = item / ntiles;
    char* wb = smem + WOFF + g * G0BYTES;
    int sb = sub;
    asm volatile("" : "+v"(sb));
#pragma unroll
    for (int i = 0; i < GPW; ++i) {
      const int wr = (wave * GPW + i) * RPI + sb;
      const int wrow = wr & (BN - 1), tap = g * G1T + wr / BN;
      const int n = nt * BN + (wrow >> 5) * 32 + ((wrow >> 2) & 3) * 8 + ((wrow >> 4) & 1) * 4 + (wrow & 3);
      const uint32_t off = live ? (uint32_t)(((size_t)n * a.K + tap * a.Cs + cc * 32 + swzh(wr, slot) * 8) * 2) : BAD;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_wgt, (lds_ptr)(wb + (wave * GPW + i) * RPI * 64), 16, off, 0, 0, 0);
    }
  };
  // BNR, wave 0, first chunk of an item: the item's (group, slice) affine, four 512-B arrays, each by
  // one DMA instruction into its own 1 KiB slot (lanes 32..63 out of range write zeros after it)
  auto issue_aff = [&](int s) {
    const int item = it0 + s / CC;
    const int nt = item / ntiles, img = (item - nt * ntiles) / tpi;
    const uint32_t nbytes = (uint32_t)(a.M / a.Mg) * a.Nout * 4;
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const uint32_t off = ln < BN / 4 ? (uint32_t)(((img / ipg) * a.Nout + nt * BN + ln * 4) * 4) : BAD;
    const float* arr[4] = {a.bnr_scale, a.bnr_shift, a.bnr_mean, a.bnr_invstd};
#pragma unroll
    for (int k = 0; k < 4; ++k)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(__builtin_amdgcn_make_buffer_rsrc((void*)arr[k], 0, nbytes, 0x00020000),
                                               (lds_ptr)(smem + AOFF + k * 1024), 16, off, 0, 0, 0);
  };
  // wave 0, first chunk of an item: the slice's 128 biases (lanes 0..31 x 16 B) into BOFF
  auto issue_bias = [&](int s) {
    const int nt = (it0 + s / CC) / ntiles;
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const uint32_t off = ln < BN / 4 ? (uint32_t)((nt * BN + ln * 4) * 4) : BAD;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_bias, (lds_ptr)(smem + BOFF), 16, off, 0, 0, 0);
  };

  // this lane's halo read address for tap column dx (fragment 0, tap row 0, stage 0).  Fragment i
  // is pixel row 2*wave + (i >> 1), columns (i & 1) * 16 + fr: both shifts leave the column-keyed
  // swizzle unchanged (key hx + 16 flips no bit of (hx >> 1) & 2), so fragment, tap row and ring
  // stage are all immediate offsets -- three address registers in all
  const uint32_t s32 = (uint32_t)(uintptr_t)(lds_ptr)smem;
  uint32_t xa[3];
#pragma unroll
  for (int dx = 0; dx < 3; ++dx) {
    const int hx = fr + dx;
    xa[dx] = s32 + (uint32_t)(((2 * wave) * HW + hx) * 64 + swzh(hx, fk) * 16);
  }
  // weight rows: G0 from wb0, G1 from wb1 (immediate offsets < 40 KiB)
  const uint32_t wb0 = s32 + (uint32_t)(WOFF + fr * 64 + swzh(fr, fk) * 16);
  const uint32_t wb1 = wb0 + G0BYTES;

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // BatchNorm partial statistics rows [groups][gridDim][2][Nout], as halo_body (non-deferred): thread
  // tid < 256 owns (sum | sum of squares, channel) tid of the current (group, slice) key, its running
  // value in LDS (ROFF) and its row addresses recomputed when used (registers go to the accumulators).
  // BNR: the same rows hold (sum g, sum g*xhat)
  float* const sbuf = BNR ? a.bnr_part : (DIRECT == 2 ? a.stats : nullptr);
  float* const runl = reinterpret_cast<float*>(smem + ROFF);
  const int groups = a.M / a.Mg;
  auto srow_ptr = [&](int key) {                        // (group, slice) key -> this thread's element
    int t = tid;
    asm volatile("" : "+v"(t));
    const int g = key / NTn, nt = key - g * NTn;
    return sbuf + ((size_t)(g * gridDim.x + vb) * 2 + (t >> 7)) * a.Nout + nt * BN + (t & 127);
  };
  int run_key = -1;                                      // wave-uniform
  if (sbuf && tid < 256) {
    for (int k = 0; k < groups * NTn; ++k) *srow_ptr(k) = 0.f;
  }

  // prologue: the fills points P0(-1), P1(-1) would have issued
  issue_halo(0);
  issue_w(0, std::integral_constant<int, 0>());

  e16x8 xf[2][TM], wf[TN];
  auto rdA = [&](int t, int b, int ph) {                // ph: ring stage (compile-time)
#pragma unroll
    for (int i = 0; i < TM; ++i)
      asm volatile("ds_read_b128 %0, %1 offset:%2"
                   : "=v"(xf[b][i])
                   : "v"(xa[t % 3]), "i"(ph * HSTAGE + (t / 3 + (i >> 1)) * HW * 64 + (i & 1) * 16 * 64));
  };
  auto rdB = [&](int t, int half) {
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int j = half * 4 + jj;
      asm volatile("ds_read_b128 %0, %1 offset:%2"
                   : "=v"(wf[j]) : "v"(t >= G1T ? wb1 : wb0), "i"(((t >= G1T ? t - G1T : t) * BN + j * 16) * 64));
    }
  };
  bool epi = false;
  int cc = 0, item = it0;
  // two stages per iteration, so the ring stage of every LDS read is an immediate
  for (int s2 = 0; s2 < S; s2 += 2)
#pragma unroll
  for (int ph = 0; ph < 2; ++ph) {
    const int s = s2 + ph;
    if (s >= S) break;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const int t0 = g ? G1T : 0, t1 = g ? 9 : G1T;
      // ---- point P_g(s): this wave's fills for it have landed, then the barrier publishes everyone's
      // (and every wave has finished reading the buffer the point's fills overwrite)
      if (g == 0) {
        if (epi) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NST) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        epi = false;
      } else {
        asm volatile("s_waitcnt vmcnt(%0)" :: "n"(HPW) : "memory");   // (halo(s+1) may stay in flight)
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      auto issue_point = [&]() {
        if (WIDE_ABL == 2 && s >= 1) return;
        const bool wl = !(WIDE_ABL == 3 && s >= 1), hl = !(WIDE_ABL == 4 && s >= 1);
        if (g == 0) {
          if (has_bias && cc == 0 && wave == 0) issue_bias(s);
          if (BNR && cc == 0 && wave == 0) issue_aff(s);
          if (wl) issue_w(s, std::integral_constant<int, 1>());
          if (hl) issue_halo(s + 1);
        } else {
          if (wl) issue_w(s + 1, std::integral_constant<int, 0>());
        }
      };
      if (WIDE_STAGGER == 0 || wave < NW / 2) issue_point();   // (stagger: waves 4..7 after their first MFMA block)
      // ---- taps t0 .. t1-1, software-pipelined: A of tap t+1 (also across the group boundary: the
      // halo is the stage's) and each half of B of tap t+1 (within the group) are read while tap t's
      // MFMAs run
      if (g == 0) rdA(0, 0, ph);
      rdB(t0, 0);
      if (WIDE_ABL == 1) { wf[4] = wf[0]; wf[5] = wf[1]; wf[6] = wf[2]; wf[7] = wf[3]; }
      else rdB(t0, 1);
#pragma unroll
      for (int t = t0; t < t1; ++t) {
        const int b = t & 1;
        const bool nA = t + 1 < 9, nB = t + 1 < t1;
        if (nA) rdA(t + 1, b ^ 1, ph);
        if (nA)
          asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(xf[b][0]), "+v"(xf[b][1]), "+v"(xf[b][2]), "+v"(xf[b][3]),
                       "+v"(wf[0]), "+v"(wf[1]), "+v"(wf[2]), "+v"(wf[3]));
        else
          asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(xf[b][0]), "+v"(xf[b][1]), "+v"(xf[b][2]), "+v"(xf[b][3]),
                       "+v"(wf[0]), "+v"(wf[1]), "+v"(wf[2]), "+v"(wf[3]));
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
#pragma unroll
          for (int i = 0; i < TM; ++i) acc[i][jj] = mfma16x16x32(wf[jj], xf[b][i], acc[i][jj]);
        if (WIDE_STAGGER && t == t0 && wave >= NW / 2) issue_point();
        if (nB) {
          rdB(t + 1, 0);
          asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(wf[4]), "+v"(wf[5]), "+v"(wf[6]), "+v"(wf[7]));
        } else if (nA) {
          asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(wf[4]), "+v"(wf[5]), "+v"(wf[6]), "+v"(wf[7]));
        } else {
          asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(wf[4]), "+v"(wf[5]), "+v"(wf[6]), "+v"(wf[7]));
        }
#pragma unroll
        for (int jj = 4; jj < 8; ++jj)
#pragma unroll
          for (int i = 0; i < TM; ++i) acc[i][jj] = mfma16x16x32(wf[jj], xf[b][i], acc[i][jj]);
        if (nB) {
          if (WIDE_ABL == 1) { wf[4] = wf[0]; wf[5] = wf[1]; wf[6] = wf[2]; wf[7] = wf[3]; }
          else rdB(t + 1, 1);
        }
      }
    }
    if (++cc < CC) continue;
    // ---- direct epilogue of `item`: lane (fr, fk) holds pixel i*16+fr, channels h*32 + fk*8 + 0..7
    // in acc[i][2h], acc[i][2h+1]; every lane issues exactly NST stores (invalid pixels out of range)
    cc = 0;
    {
      const int nt = item / ntiles, tile = item - nt * ntiles;
      const int img = tile / tpi, t2 = tile - img * tpi, ty = t2 / TX, tx = t2 - ty * TX;
      const __amdgpu_buffer_rsrc_t rs_dst =
          __builtin_amdgcn_make_buffer_rsrc((void*)a.dst, 0, (uint32_t)((size_t)a.M * a.dcs * 2), 0x00020000);
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      int mq[TM];
      int fo = fr, ko = fk;                              // (opaque: recomputed per item, not kept live)
      asm volatile("" : "+v"(fo), "+v"(ko));
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int y = ty * PH + 2 * wave + (i >> 1), x = tx * PW + (i & 1) * 16 + fo;
        mq[i] = (y < a.Hd && x < a.Wd) ? (img * a.Hd + y) * a.Wd + x : -1;
      }
      float res[4] = {0.f, 0.f, 0.f, 0.f};
      const __amdgpu_buffer_rsrc_t rs_y = __builtin_amdgcn_make_buffer_rsrc(
          (void*)a.bnr_y, 0, BNR ? (uint32_t)((size_t)a.M * a.bnr_ycs * 2) : 0u, 0x00020000);
      // BNR: y of the lane's 8 channels of each pixel, one 32-channel block ahead (the MFMA operand
      // registers are free in the epilogue)
      uint4 yq[2][TM];
      auto load_y = [&](int h) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const uint32_t yo = mq[i] >= 0 ? (uint32_t)(((size_t)mq[i] * a.bnr_ycs + nt * BN + h * 32 + ko * 8) * 2) : BAD;
          const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs_y, yo, 0, 0);
          yq[h & 1][i] = make_uint4(v.x, v.y, v.z, v.w);
        }
      };
      if constexpr (BNR) load_y(0);
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        if constexpr (BNR)
          if (h < 3) load_y(h + 1);
        float bb[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (has_bias) {
          const float4 lo = *reinterpret_cast<const float4*>(smem + BOFF + (h * 32 + ko * 8) * 4);
          const float4 hi = *reinterpret_cast<const float4*>(smem + BOFF + (h * 32 + ko * 8 + 4) * 4);
          bb[0] = lo.x; bb[1] = lo.y; bb[2] = lo.z; bb[3] = lo.w; bb[4] = hi.x; bb[5] = hi.y; bb[6] = hi.z; bb[7] = hi.w;
        }
        float v[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) v[e] = 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          float f[8];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            f[r] = acc[i][2 * h][r] + bb[r];
            f[4 + r] = acc[i][2 * h + 1][r] + bb[4 + r];
          }
          const uint32_t off =
              mq[i] >= 0 ? (uint32_t)(((size_t)mq[i] * a.dcs + nt * BN + h * 32 + ko * 8) * 2) : BAD;
          if (a.accumulate) {                            // (out-of-range lanes read zeros)
            const u32x4 ov = __builtin_amdgcn_raw_buffer_load_b128(rs_dst, off, 0, 0);
            float o[8];
            unpack8(make_uint4(ov.x, ov.y, ov.z, ov.w), o);
#pragma unroll
            for (int e = 0; e < 8; ++e) f[e] += o[e];
          }
          const uint4 u = pack8(f);
          acc[i][2 * h] = f32x4{0.f, 0.f, 0.f, 0.f};
          acc[i][2 * h + 1] = f32x4{0.f, 0.f, 0.f, 0.f};
          __builtin_amdgcn_raw_buffer_store_b128(u32x4{u.x, u.y, u.z, u.w}, rs_dst, off, 0, 0);
          if constexpr (DIRECT == 2) {
            float gq[8];
            unpack8(u, gq);
            const float w = mq[i] >= 0 ? 1.f : 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) { v[e] += w * gq[e]; v[8 + e] += w * gq[e] * gq[e]; }
          }
          if constexpr (BNR) {
            // g = dz * [y*scale+shift > 0] (valid pixels); v: sum g, then sum g*y (-> g*xhat below)
            float gq[8], yv[8];
            unpack8(u, gq);
            unpack8(yq[h & 1][i], yv);
            const float* af = reinterpret_cast<const float*>(smem + AOFF) + h * 32 + ko * 8;
            const bool valid = mq[i] >= 0, norelu = !a.bnr_relu;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const bool keep = valid & (norelu | (yv[e] * af[e] + af[256 + e] > 0.f));
              const float gg = keep ? gq[e] : 0.f;
              v[e] += gg;
              v[8 + e] += gg * yv[e];
            }
          }
        }
        if constexpr (BNR) {
          const float* af = reinterpret_cast<const float*>(smem + AOFF) + h * 32 + ko * 8;
#pragma unroll
          for (int e = 0; e < 8; ++e) v[8 + e] = af[768 + e] * (v[8 + e] - af[512 + e] * v[e]);
        }
        if constexpr (DIRECT == 2 || BNR) res[h] = row16_reduce_scatter(v, fo);
      }
      epi = true;
      if (sbuf) {
        // every wave is done with the G1 buffer (its last taps): it holds the cross-wave partials
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        float* red = reinterpret_cast<float*>(smem + WOFF + G0BYTES);         // [NW][2][128]
#pragma unroll
        for (int h = 0; h < 4; ++h) red[(wave * 2 + (fo >> 3)) * BN + h * 32 + ko * 8 + (fo & 7)] = res[h];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        const int key = (img / ipg) * NTn + nt;
        int to = tid;
        asm volatile("" : "+v"(to));
        if (to < 256) {
          float t = 0.f;
#pragma unroll
          for (int w = 0; w < NW; ++w) t += red[w * 2 * BN + to];
          const float prev = runl[to];
          if (key != run_key && run_key >= 0) *srow_ptr(run_key) = prev;
          runl[to] = (key != run_key ? 0.f : prev) + t;
        }
        run_key = key;
      }
    }
    ++item;
  }
  if (sbuf && tid < 256 && run_key >= 0) *srow_ptr(run_key) = runl[tid];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");       // the trailing (not live) fills have landed
}

// ---------------------------------------------------------------------------
// 3x3 / stride 1 / pad 1 convolution of an 8-channel input (UNet's first layer: in_channels = 8,
// src/unet.py:12): K = 9 taps x 8 channels = 72, three 32-deep MFMA steps (taps 9-11 zero).  A
// workgroup walks 16 x 16 pixel tiles; per tile the 18 x 18 halo of 16-B rows (one pixel's 8
// channels) is staged in LDS once, and every MFMA B fragment -- 8 channels of one pixel at one tap
// -- is ONE ds_read_b128 of halo row (pixel + tap offset).  The 64 x 72 weights stay in registers
// for the whole launch.  (The linear kernel gathers the 16-B row of every tap with its own LDS-DMA
// instruction: ~9x the issue work for the same bytes.)  Weight rows are permuted as in the halo
// kernel's DIRECT epilogue, so each lane stores 16-B chunks of 8 consecutive channels straight
// from its accumulators; BN partial sums per (statistics group, workgroup) from the stored values.
constexpr int C8_T = 16, C8_HW = C8_T + 2, C8_HR = C8_HW * C8_HW;      // 324 halo rows per tile
__global__ __launch_bounds__(256, 2) void conv3x3_c8_kernel(Geo a, int TY, int TX, int per, int rem, int c8_full) {
  __shared__ __attribute__((aligned(16))) uint4 halo[2][C8_HR];
  __shared__ float red[4][2][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fk = lane >> 4;
  const int tpi = TY * TX;
  const int cnt = per + (int)(blockIdx.x < (unsigned)rem);
  const int t0 = blockIdx.x * per + min((int)blockIdx.x, rem);
  const int ipg = a.Mg / (a.Hd * a.Wd), groups = a.M / a.Mg;
  // weights: A row m of fragment j = output channel (j >> 1) * 32 + (m >> 2) * 8 + (j & 1) * 4 + (m & 3);
  // lane (fr, fk) of k-step ks holds tap ks * 4 + fk (8 channels)
  e16x8 wf[4][3];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = (j >> 1) * 32 + (fr >> 2) * 8 + (j & 1) * 4 + (fr & 3);
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) {
      const int t = ks * 4 + fk;
      wf[j][ks] = t < 9 ? *reinterpret_cast<const e16x8*>(a.wgt + (size_t)n * a.K + t * 8) : e16x8{};
    }
  }
  // this lane's 16 accumulator channels: h * 32 + fk * 8 + e (e = (j & 1) * 4 + r, h = j >> 1)
  float bv[2][8];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int e = 0; e < 8; ++e) bv[h][e] = a.bias ? a.bias[h * 32 + fk * 8 + e] : 0.f;
  if (a.stats && tid < 128) {           // this workgroup's rows of every group (the fold reads them all)
    for (int g = 0; g < groups; ++g) a.stats[((size_t)(g * gridDim.x + blockIdx.x) * 2 + (tid >> 6)) * 64 + (tid & 63)] = 0.f;
  }
  const __amdgpu_buffer_rsrc_t rs_dst =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.dst, 0, (uint32_t)((size_t)a.M * a.dcs * 2), 0x00020000);
  uint4 ld[2];
  auto load = [&](int tile) {
    const int img = tile / tpi, t2 = tile - img * tpi, ty = t2 / TX, tx = t2 - ty * TX;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int hr = tid + q * 256, hy = hr / C8_HW, hx = hr - hy * C8_HW;
      const int ys = ty * C8_T - 1 + hy, xs = tx * C8_T - 1 + hx;
      ld[q] = make_uint4(0, 0, 0, 0);
      if (hr < C8_HR && ys >= 0 && xs >= 0 && ys < a.Hs && xs < a.Ws)
        ld[q] = *reinterpret_cast<const uint4*>(a.src + ((size_t)(img * a.Hs + ys) * a.Ws + xs) * a.scs);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 2; ++q)
      if (tid + q * 256 < C8_HR) halo[buf][tid + q * 256] = ld[q];
  };
  float s1[2][8], s2[2][8];
  auto zero_sums = [&]() {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int e = 0; e < 8; ++e) { s1[h][e] = 0.f; s2[h][e] = 0.f; }
  };
  int run_key = -1;
  // the sums of the tiles since the last flush into this workgroup's row of group run_key
  auto flush = [&]() {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int e = 0; e < 8; ++e)
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          s1[h][e] += __shfl_xor(s1[h][e], o, 64);
          s2[h][e] += __shfl_xor(s2[h][e], o, 64);
        }
    if (fr == 0) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          red[wave][0][h * 32 + fk * 8 + e] = s1[h][e];
          red[wave][1][h * 32 + fk * 8 + e] = s2[h][e];
        }
    }
    __syncthreads();
    if (tid < 128) {
      const int q = tid >> 6, c = tid & 63;
      a.stats[((size_t)(run_key * gridDim.x + blockIdx.x) * 2 + q) * 64 + c] =
          red[0][q][c] + red[1][q][c] + red[2][q][c] + red[3][q][c];
    }
    __syncthreads();
    zero_sums();
  };
  zero_sums();
  load(t0);
  store(0);
  __syncthreads();
  for (int k = 0; k < cnt; ++k) {
    const int tile = t0 + k, buf = k & 1;
    const int img = tile / tpi, t2 = tile - img * tpi, ty = t2 / TX, tx = t2 - ty * TX;
    if (k + 1 < cnt) load(tile + 1);
    const int key = img / ipg;
    if (a.stats && key != run_key) {
      if (run_key >= 0) flush();
      run_key = key;
    }
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) {
      const int t = ks * 4 + fk, dy = t / 3, dx = t - dy * 3;
      e16x8 xf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint4 v = t < 9 ? halo[buf][(wave * 4 + i + dy) * C8_HW + fr + dx] : make_uint4(0, 0, 0, 0);
        xf[i] = __builtin_bit_cast(e16x8, v);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16x16x32(wf[j][ks], xf[i], acc[i][j]);
    }
    // epilogue: lane (fr, fk) holds chunks fk (h = 0) and 4 + fk (h = 1) of pixel (row wave * 4 + i,
    // column fr).  C8_FULL (default): the h = 1 chunk goes to lane fr ^ 8 (DPP row_ror:8) so that each
    // store instruction writes 8 whole 128-B pixel rows (pixels 0-7, then 8-15: lanes fr < 8 own
    // chunk fk, lanes fr >= 8 the partner's chunk 4 + fk) instead of half of 16 rows
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int y = ty * C8_T + wave * 4 + i, x = tx * C8_T + fr;
      const bool ok = y < a.Hd && x < a.Wd;
      const size_t m = ((size_t)img * a.Hd + y) * a.Wd + x;
      uint4 u[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float f[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          f[r] = round_e(acc[i][2 * h][r] + bv[h][r]);
          f[4 + r] = round_e(acc[i][2 * h + 1][r] + bv[h][4 + r]);
        }
        u[h] = pack8(f);
        if (ok) {
#pragma unroll
          for (int e = 0; e < 8; ++e) { s1[h][e] += f[e]; s2[h][e] += f[e] * f[e]; }
        }
      }
      if (c8_full) {
        const uint4 rcv = make_uint4(__builtin_amdgcn_update_dpp(0u, u[1].x, 0x128, 0xF, 0xF, false),
                                     __builtin_amdgcn_update_dpp(0u, u[1].y, 0x128, 0xF, 0xF, false),
                                     __builtin_amdgcn_update_dpp(0u, u[1].z, 0x128, 0xF, 0xF, false),
                                     __builtin_amdgcn_update_dpp(0u, u[1].w, 0x128, 0xF, 0xF, false));
        const bool lo = fr < 8;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          // half 0: pixels 0-7 of the tile row, half 1: pixels 8-15
          const uint4 v = (half == 0) == lo ? u[0] : rcv;
          const int px = (fr & 7) + half * 8, ch = ((half == 0) == lo ? 0 : 32) + fk * 8;
          const int xx = tx * C8_T + px;
          const size_t mm = ((size_t)img * a.Hd + y) * a.Wd + xx;
          const uint32_t off = (y < a.Hd && xx < a.Wd) ? (uint32_t)((mm * a.dcs + ch) * 2) : 0xFFFFFFF0u;
          __builtin_amdgcn_raw_buffer_store_b128(u32x4{v.x, v.y, v.z, v.w}, rs_dst, off, 0, 0);
        }
      } else {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const uint32_t off = ok ? (uint32_t)((m * a.dcs + h * 32 + fk * 8) * 2) : 0xFFFFFFF0u;
          __builtin_amdgcn_raw_buffer_store_b128(u32x4{u[h].x, u[h].y, u[h].z, u[h].w}, rs_dst, off, 0, 0);
        }
      }
    }
    if (k + 1 < cnt) store(buf ^ 1);
    __syncthreads();
  }
  if (a.stats && run_key >= 0) flush();
}

constexpr int HALO_PW = 32;
// 16 x 32 tile, 8 waves, 2-stage ring (1 WG/CU)
constexpr int HALO_PH = 16;
int halo_ph() { return HALO_PH; }
// tile width: 32 for W >= 32; 16x16 tiles (32 pixels per wave) for 16 <= W < 32
int halo_pw(const stf_conv_geom& c) { return c.Wd >= 32 ? HALO_PW : 16; }
// narrowest layer the halo kernel takes (measured in round 3: at 16 <= W < 32 the 16x16 tile
// wins up to 256 output channels, the 256x256 linear tile above that)
constexpr int HALO_MIN_W = 16;
// 8 x 8 layers through the halo kernel, four images per 8 x 32 tile (conv3x3_halo4_kernel;
// STF_HALO4=0: the linear split-K kernels, A/B)
bool halo8(const stf_igemm_args* a) {
  static const int mode = stf::ab_switch("STF_HALO4", 1);
  const stf_conv_geom& c = a->g;
  if (mode == 0 || (mode == 2 && a->bnr)) return false;
  if (c.Hd != 8 || c.Wd != 8 || c.N % 4 || a->Nout % 64 || c.Cs % 32) return false;
  const long M = (long)c.N * c.Hd * c.Wd;
  const long Mg = a->group_rows > 0 ? a->group_rows : M;
  return (Mg / (c.Hd * c.Wd)) % 4 == 0;
}

// 8-channel-input 3x3 layer through conv3x3_c8_kernel (STF_C8HALO=0: the linear 'e' kernel, A/B)
bool c8_halo(const stf_igemm_args* a) {
  static const bool on = stf::ab_switch("STF_C8HALO", 1) != 0;
  const stf_conv_geom& c = a->g;
  return on && !a->lstm && !a->scatter2x2 && !c.transposed && !a->bnr && !a->accumulate && c.Cs == 8 &&
         c.src_cstride % 8 == 0 && c.R == 3 && c.S == 3 && c.stride == 1 && c.pad == 1 && c.Hd == c.Hs &&
         c.Wd == c.Ws && a->Nout == 64 && a->dst_cstride % 8 == 0 && ((uintptr_t)a->dst & 15) == 0 &&
         (uint64_t)c.N * c.Hd * c.Wd * a->dst_cstride * 2 < 0xFFFFFF00ull;
}

// direct-store epilogue; STF_HALO_DIRECT=0 disables, =1 only without BN statistics (dgrad),
// =2 always (default: measured 1.7 % faster on the forward convs than the LDS-staged one)
bool halo_direct(const stf_igemm_args* a) {
  static const int mode = stf::ab_switch("STF_HALO_DIRECT", 2);
  return !halo8(a) && (mode == 2 || (mode == 1 && !a->stats));
}

// BN-backward reduction fused into the halo direct epilogue (STF_BNR_FUSED=0: separate
// stf_bn_bwd_reduce pass after the GEMM, for A/B measurements)
bool bnr_fused(const stf_igemm_args* a, char k) {
  static const bool on = stf::ab_switch("STF_BNR_FUSED", 1) != 0;
  return on && a->bnr && k == 'H' && halo_direct(a);
}

int halo_ix(const stf_igemm_args* a, bool with_stats);
int halo_grid(const stf_igemm_args* a, int ix);
void halo_tiles(const stf_conv_geom& c, int& ty, int& tx);

// the wide halo kernel (conv3x3_wide_kernel: 128-channel output slices) for 3x3 layers with >= 128
// output channels and W >= 32, forward, plain dgrad and BN-backward-fused dgrad (STF_WIDE_BNR=0: that one
// on the 64-channel kernel, A/B); STF_HALO_WIDE=0: the 64-channel halo kernel (A/B)
bool bnr_fused(const stf_igemm_args* a, char k);
bool halo_wide(const stf_igemm_args* a) {
  static const int on = stf::ab_switch("STF_HALO_WIDE", 1);
  static const int wbnr = stf::ab_switch("STF_WIDE_BNR", 1);
  const stf_conv_geom& c = a->g;
  if (a->bnr && !(wbnr && bnr_fused(a, 'H'))) return false;
  return on && !a->lstm && !a->scatter2x2 && !c.transposed && halo_direct(a) && a->Nout % 128 == 0 &&
         c.Wd >= 32 && c.Cs % 32 == 0 && halo_ix(a, a->stats != nullptr) == 1;
}

// deferred epilogue of the second wave half (halo_body DEFER; default on, STF_HALO_DEFER=0: off, A/B).  Its
// statistics fold keeps at most 2 (group, slice) keys per workgroup: the item run of a workgroup
// (items / grid + 1, slice-major, image-major within a slice) must not span more.
bool halo_defer(const stf_igemm_args* a) {
  static const int on = stf::ab_switch("STF_HALO_DEFER", 1);
  if (!(on && halo_direct(a) && !halo8(a)) || halo_wide(a)) return false;
  // (not the two-image 16 x 16 tiles: their deferred variants spill registers)
  const int ix = halo_ix(a, a->stats != nullptr);
  if (ix > 1) return false;
  if (!a->stats && !a->bnr) return true;                 // no statistics rows
  const stf_conv_geom& c = a->g;
  int ty, tx;
  halo_tiles(c, ty, tx);
  if (ix > 1) ty = tx = 1;
  const long M = (long)c.N * c.Hd * c.Wd;
  const long Mg = a->group_rows > 0 ? a->group_rows : M;
  const long run = (Mg / ((long)c.Hd * c.Wd) / ix) * ty * tx;   // items per (group, slice) key
  const long items = (long)(c.N / ix) * ty * tx * (a->Nout / 64);
  const long per = items / halo_grid(a, ix) + 1;
  return run > 0 && (per + run - 1) / run + 1 <= 2;
}

int num_cus() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return n;
}

int c8_tiles(const stf_conv_geom& c) { return c.N * ((c.Hd + C8_T - 1) / C8_T) * ((c.Wd + C8_T - 1) / C8_T); }
int c8_grid(const stf_igemm_args* a) { return std::min(c8_tiles(a->g), 2 * num_cus()); }

// Tile configurations of the DMA kernel.  'auto' picks per shape; the
// STF_IGEMM_CFG environment variable forces one (A/B measurements).
struct Cfg { int bm, bn, bkk; };
constexpr Cfg CFG_A{128, 128, 32};   // 4 waves (2x2), 4 stages, 2 blocks/CU
constexpr Cfg CFG_B{256, 128, 64};   // 8 waves (4x2), 3 stages
constexpr Cfg CFG_C{256, 256, 64};   // 8 waves (2x4), 2 stages
constexpr Cfg CFG_D{512, 64, 64};    // 8 waves (8x1), 2 stages
constexpr Cfg CFG_E{256, 64, 32};    // 4 waves (4x1), 4 stages, 2 blocks/CU
constexpr Cfg CFG_F{128, 256, 32};   // 8 waves (2x4), 2 stages, 2 blocks/CU (80 KiB each)

char forced_cfg() {
  static const char c = [] {
    const char e = stf::ab_letter("STF_IGEMM_CFG");
    return ((e >= 'A' && e <= 'F') || e == 'H' || e == 'L') ? e : '0';
  }();
  return c;
}

// STF_IGEMM_DMA=0 selects the register-staged kernel (A/B comparisons); read once.
bool dma_enabled() {
  static const bool on = stf::ab_switch("STF_IGEMM_DMA", 1) != 0;
  return on;
}

// which kernel runs: 'R' = register-staged (BM 256 for Nout <= 64, else 128), or a DMA config letter
char choose(const stf_igemm_args* a, bool dma_ok) {
  const stf_conv_geom& c = a->g;
  const bool plain = !a->lstm && !a->scatter2x2 && !c.transposed;
  if (c8_halo(a) && forced_cfg() == '0') return 'K';     // 8-channel network input, 3x3
  if (dma_enabled() && dma_ok && plain && c.Cs == 8 && forced_cfg() != 'R')   // 8-channel network inputs
    return a->Nout <= 64 ? 'e' : 'a';
  if (!dma_enabled() || !dma_ok || c.Cs % 32) return 'R';
  const char f = forced_cfg();
  const bool bk64 = c.Cs % 64 == 0;
  if (a->lstm) {
    // LSTM steps (1x1 GEMM, K = 2C): the 128 x 128 tile (any tile gives the same gates -- the
    // same MFMA sequence over ascending K -- so the backward recompute may run another tile)
    return 'A';
  }
  const bool halo_ok = plain && c.R == 3 && c.S == 3 && c.stride == 1 && c.pad == 1 && c.Hd == c.Hs &&
                       c.Wd == c.Ws && a->Nout % 64 == 0;
  if (f == 'H' && halo_ok) return 'H';
  // auto: the halo kernel for full-size 3x3 layers ('L' = auto over the linear kernels only)
  if (f == '0' && halo_ok && (c.Wd >= 32 || (c.Wd >= HALO_MIN_W && a->Nout <= 256))) return 'H';
  // 16 x 16 layers with more output channels (UNet's bottleneck): the two-image halo tiles
  if (f == '0' && halo_ok && a->Nout > 256 && halo_ix(a, a->stats != nullptr) == 2) return 'H';
  if (f == '0' && halo_ok && halo8(a)) return 'H';
  if (f != '0' && f != 'H' && f != 'L') {
    if (f == 'A' || f == 'E') return (f == 'E' && !(a->Nout <= 64 && !a->lstm)) ? 'A' : f;
    if ((plain || a->scatter2x2) && bk64 && !a->lstm && !c.transposed) return f;
  }
  if ((plain || (a->scatter2x2 && !c.transposed && !a->lstm)) && bk64) {
    // measured per layer (tools/bench_layers.py, cfg2 shapes): C where it fills the chip,
    // B for 128-multiples, D for 64 output channels
    const long M = (long)c.N * c.Hd * c.Wd;
    const long blocks_c = ((M + 255) / 256) * ((a->Nout + 255) / 256);
    if (a->Nout % 256 == 0 && blocks_c >= 240) return 'C';
    if (a->Nout % 128 == 0) return 'B';
    if (a->Nout == 64) return 'D';
  }
  if (a->Nout <= 64 && !a->lstm) return 'E';
  return 'A';
}

Cfg cfg_of(char k) {
  switch (k) {
    case 'a': return CFG_A;
    case 'e': return CFG_E;
    case 'B': return CFG_B;
    case 'C': return CFG_C;
    case 'D': return CFG_D;
    case 'E': return CFG_E;
    case 'F': return CFG_F;
    default: return CFG_A;
  }
}

template <int BM, int BN, int WM, int WN, int BKK, int STAGES>
void launch_dma(const Geo& g, bool trans, bool scatter, int lstm, bool c8, uint32_t src_bytes, hipStream_t s) {
  dim3 grid(g.tpg * ((g.M + g.Mg - 1) / g.Mg), (g.Nout + BN - 1) / BN, g.ksplit), block(64 * WM * WN);
#define STF_D(TR, SCA, E) \
  hipLaunchKernelGGL((igemm_dma_kernel<BM, BN, WM, WN, BKK, STAGES, TR, SCA, E>), grid, block, 0, s, g, src_bytes)
  if (c8)
    hipLaunchKernelGGL((igemm_dma_kernel<BM, BN, WM, WN, BKK, STAGES, false, false, 0, true>), grid, block, 0, s, g,
                       src_bytes);
  else if (lstm == 2) STF_D(false, false, 2);
  else if (lstm) STF_D(false, false, 1);
  else if (scatter) STF_D(false, true, 0);
  else if (trans) STF_D(true, false, 0);
  else STF_D(false, false, 0);
#undef STF_D
}

// plain forward gather (or its ConvT 2x2 scatter epilogue, or an LSTM step: lstm 1 =
// cell, 2 = cell backward) on the 8-wave tiles
template <int BM, int BN, int WM, int WN, int BKK, int STAGES>
void launch_dma_plain(const Geo& g, bool scatter, uint32_t src_bytes, hipStream_t s, int lstm = 0) {
  dim3 grid(g.tpg * ((g.M + g.Mg - 1) / g.Mg), (g.Nout + BN - 1) / BN, g.ksplit), block(64 * WM * WN);
  if constexpr (lstm_bwd_lds<BM, BN>() <= 163840) {
    if (lstm == 2) {
      hipLaunchKernelGGL((igemm_dma_kernel<BM, BN, WM, WN, BKK, STAGES, false, false, 2>), grid, block, 0, s, g,
                         src_bytes);
      return;
    }
  }
  if (lstm)
    hipLaunchKernelGGL((igemm_dma_kernel<BM, BN, WM, WN, BKK, STAGES, false, false, 1>), grid, block, 0, s, g,
                       src_bytes);
  else if (scatter)
    hipLaunchKernelGGL((igemm_dma_kernel<BM, BN, WM, WN, BKK, STAGES, false, true, 0>), grid, block, 0, s, g,
                       src_bytes);
  else
    hipLaunchKernelGGL((igemm_dma_kernel<BM, BN, WM, WN, BKK, STAGES, false, false, 0>), grid, block, 0, s, g,
                       src_bytes);
}

template <int BM, int BN, int WM, int WN>
int launch_reg(const Geo& g, bool smallc, bool trans, bool scatter, int lstm, hipStream_t s) {
  dim3 grid(g.tpg * ((g.M + g.Mg - 1) / g.Mg), (g.Nout + BN - 1) / BN), block(NT);
#define STF_L(SC, TR, SCA, E) hipLaunchKernelGGL((igemm_kernel<BM, BN, WM, WN, SC, TR, SCA, E>), grid, block, 0, s, g)
  if (lstm) {
    if (smallc) return STF_EINVAL;
    if (lstm == 2) STF_L(false, false, false, 2);
    else STF_L(false, false, false, 1);
  }
  else if (scatter) { if (smallc) STF_L(true, false, true, 0); else STF_L(false, false, true, 0); }
  else if (trans) { if (smallc) STF_L(true, true, false, 0); else STF_L(false, true, false, 0); }
  else { if (smallc) STF_L(true, false, false, 0); else STF_L(false, false, false, 0); }
#undef STF_L
  STF_CHECK_LAUNCH();
  return 0;
}

bool dma_fits(const stf_igemm_args* a) {
  const stf_conv_geom& c = a->g;
  const uint64_t src_bytes = (uint64_t)c.N * c.Hs * c.Ws * c.src_cstride * 2;
  const uint64_t wgt_bytes = (uint64_t)a->Nout * c.R * c.S * c.Cs * 2;
  return src_bytes < 0xFFFFFF00ull && wgt_bytes < 0xFFFFFF00ull;
}

int pick_mtile(const stf_igemm_args* a) {
  const char k = choose(a, dma_fits(a));
  if (k == 'R') return (a->Nout <= 64 && !a->lstm) ? 256 : 128;
  return cfg_of(k).bm;
}

void halo_tiles(const stf_conv_geom& c, int& ty, int& tx) {
  ty = (c.Hd + halo_ph() - 1) / halo_ph();
  tx = (c.Wd + halo_pw(c) - 1) / halo_pw(c);
}

// images per halo tile: 2 for 16 x 16 layers (conv3x3_halo2_kernel: two images side by side
// in one 16 x 32 tile) when the statistics groups hold an even number of images.
// STF_HALO2=0: one 16 x 16 image per tile; 1 (default): forward convs (with BN statistics)
// only -- the dgrads run beside the side-stream weight gradients, and the 160 KiB workgroup
// of the wide tile cannot share a CU with them (128 KiB for the 16 x 16 tile); 2: all
// with_stats: the launch writes BN statistics (the size queries pass what the launch will do:
// stf_igemm_stat_tiles is asked before the statistics buffer exists)
int halo_ix(const stf_igemm_args* a, bool with_stats) {
  static const int mode = stf::ab_switch("STF_HALO2", 1);
  const stf_conv_geom& c = a->g;
  if (halo8(a)) return 4;
  // (mode 1: two images per tile for the forward convs with statistics, and for every conv with more
  // than 256 output channels -- the UNet bottleneck, whose dgrads run 4-22 % faster on them than on
  // single-image tiles or the linear kernels, tools/bench_layers.py)
  if (mode == 0 || (mode == 1 && !with_stats && a->Nout <= 256)) return 1;
  if (c.Hd != 16 || c.Wd != 16 || c.N % 2) return 1;
  const long M = (long)c.N * c.Hd * c.Wd;
  const long Mg = a->group_rows > 0 ? a->group_rows : M;
  return ((Mg / (c.Hd * c.Wd)) % 2) ? 1 : 2;
}

long halo_items_ix(const stf_igemm_args* a, int ix) {
  int ty, tx;
  halo_tiles(a->g, ty, tx);
  if (ix > 1) ty = tx = 1;
  return (long)(a->g.N / ix) * ty * tx * (a->Nout / (ix == 1 && halo_wide(a) ? 128 : 64));
}

// persistent halo grid: one workgroup per CU (160 KiB LDS each; the single-stage 8 x 8 kernel two)
int halo_grid(const stf_igemm_args* a, int ix) {
  const long items = halo_items_ix(a, ix);
  return (int)std::min<long>(items, (long)num_cus() * (ix == 4 ? 2 : 1));
}

// Split-K factor for a plain gather on the linear DMA kernels that would leave the
// chip under-filled (small-M layers: STF layer4 at 8x8, LSTM backward GEMMs):
// K slices until ~256 workgroups, each keeping >= 8 K steps.  1 = no split.
// STF_SPLITK=0 disables it (A/B).
int ksplit_of(const stf_igemm_args* a) {
  static const bool on = stf::ab_switch("STF_SPLITK", 1) != 0;
  const stf_conv_geom& c = a->g;
  const char k = choose(a, dma_fits(a));
  if (!on || a->lstm || a->scatter2x2 || c.transposed || c.Cs == 8) return 1;
  if (!(k == 'A' || k == 'B' || k == 'C' || k == 'D' || k == 'E' || k == 'F')) return 1;
  if (a->Nout % 8 || NT % (a->Nout / 8) || a->dst_cstride % 8 || ((uintptr_t)a->dst & 15)) return 1;
  const Cfg f = cfg_of(k);
  const long M = (long)c.N * c.Hd * c.Wd;
  const long Mg = a->group_rows > 0 ? a->group_rows : M;
  const long blocks = (M / Mg) * ((Mg + f.bm - 1) / f.bm) * ((a->Nout + f.bn - 1) / f.bn);
  const long kt = (long)c.R * c.S * c.Cs / f.bkk;
  if (blocks >= 192 || kt < 16) return 1;
  long ks = (256 + blocks - 1) / blocks;
  if (ks > kt / 8) ks = kt / 8;
  if (ks > 8) ks = 8;
  return ks < 2 ? 1 : (int)ks;
}

// BatchNorm partial-statistics rows per group for the kernel that will run
int stat_tiles(const stf_igemm_args* a) {
  const stf_conv_geom& c = a->g;
  const long M = (long)c.N * c.Hd * c.Wd;
  const long Mg = a->group_rows > 0 ? a->group_rows : M;
  if (choose(a, dma_fits(a)) == 'H') return halo_grid(a, halo_ix(a, true));
  if (choose(a, dma_fits(a)) == 'K') return c8_grid(a);
  if (ksplit_of(a) > 1) return (int)((Mg + sk_rows(a->Nout) - 1) / sk_rows(a->Nout));
  const int bm = pick_mtile(a);
  return (int)((Mg + bm - 1) / bm);
}

}  // namespace

extern "C" int stf_igemm_stat_tiles(const stf_igemm_args* a) { return stat_tiles(a); }

extern "C" size_t stf_igemm_ws_bytes(const stf_igemm_args* a) {
  const int ks = ksplit_of(a);
  if (ks < 2) return 0;
  const stf_conv_geom& c = a->g;
  return (size_t)ks * c.N * c.Hd * c.Wd * a->Nout * sizeof(float);
}

extern "C" int stf_igemm_bnr_tiles(const stf_igemm_args* a) {
  const stf_conv_geom& c = a->g;
  const long M = (long)c.N * c.Hd * c.Wd;
  const int groups = a->group_rows > 0 ? (int)(M / a->group_rows) : 1;
  if (bnr_fused(a, choose(a, dma_fits(a)))) return halo_grid(a, halo_ix(a, false));
  return stf_bn_bwd_tiles(c.N, c.Hd, c.Wd, a->Nout, groups, 0);
}

// Name of the device kernel these args run (as rocprofv3 prints it), for timers
extern "C" const char* stf_igemm_kernel_name(const stf_igemm_args* a) {
  static thread_local char buf[128];
  const stf_conv_geom& c = a->g;
  const char k = choose(a, dma_fits(a));
  const int epi = a->lstm ? (a->lstm->backward ? 2 : 1) : 0;
  const char* tr = c.transposed ? "true" : "false";
  const char* sc = a->scatter2x2 ? "true" : "false";
  switch (k) {
    case 'K': snprintf(buf, sizeof buf, "conv3x3_c8_kernel"); break;
    case 'H':
      if (halo8(a))
        snprintf(buf, sizeof buf, "conv3x3_halo4_kernel<0>");
      else if (halo_wide(a))
        snprintf(buf, sizeof buf, "conv3x3_wide_kernel<%d, %s>", a->stats ? 2 : 1, a->bnr ? "true" : "false");
      else if (halo_ix(a, a->stats != nullptr) > 1)
        snprintf(buf, sizeof buf, "conv3x3_halo2_kernel<%d, %s, %s>", halo_direct(a) ? (a->stats ? 2 : 1) : 0,
                 bnr_fused(a, k) ? "true" : "false", halo_defer(a) ? "true" : "false");
      else
        snprintf(buf, sizeof buf, "conv3x3_halo_kernel<16, %d, 8, 2, 0, %d, %s, %s>", halo_pw(c),
                 halo_direct(a) ? (a->stats ? 2 : 1) : 0, bnr_fused(a, k) ? "true" : "false",
                 halo_defer(a) ? "true" : "false");
      break;
    case 'A': snprintf(buf, sizeof buf, "igemm_dma_kernel<128, 128, 2, 2, 32, 4, %s, %s, %d, false>", tr, sc, epi); break;
    case 'E': snprintf(buf, sizeof buf, "igemm_dma_kernel<256, 64, 4, 1, 32, 4, %s, %s, %d, false>", tr, sc, epi); break;
    case 'a': snprintf(buf, sizeof buf, "igemm_dma_kernel<128, 128, 2, 2, 32, 4, false, false, 0, true>"); break;
    case 'e': snprintf(buf, sizeof buf, "igemm_dma_kernel<256, 64, 4, 1, 32, 4, false, false, 0, true>"); break;
    case 'B': snprintf(buf, sizeof buf, "igemm_dma_kernel<256, 128, 4, 2, 64, 3, false, %s, %d, false>", sc, epi); break;
    case 'C': snprintf(buf, sizeof buf, "igemm_dma_kernel<256, 256, 2, 4, 64, 2, false, %s, %d, false>", sc, epi); break;
    case 'D': snprintf(buf, sizeof buf, "igemm_dma_kernel<512, 64, 8, 1, 64, 2, false, %s, %d, false>", sc, epi); break;
    case 'F': snprintf(buf, sizeof buf, "igemm_dma_kernel<128, 256, 2, 4, 32, 2, false, %s, 0, false>", sc); break;
    default: {
      const bool small = (a->Nout <= 64 && !a->lstm);
      snprintf(buf, sizeof buf, "igemm_kernel<%s, %s, %s, %s, %d>", small ? "256, 64, 4, 1" : "128, 128, 2, 2",
               (c.Cs % BK) ? "true" : "false", tr, sc, epi);
    }
  }
  return buf;
}

static int igemm_launch(const stf_igemm_args* a, stf_stream_t stream);

extern "C" int stf_igemm(const stf_igemm_args* a, stf_stream_t stream) {
  const int rc = igemm_launch(a, stream);
  if (rc || !a->bnr || bnr_fused(a, choose(a, dma_fits(a)))) return rc;
  // unfused: one stf_bn_bwd_reduce pass over the stored dz (same partial layout)
  const stf_conv_geom& c = a->g;
  const long M = (long)c.N * c.Hd * c.Wd;
  if (M <= 0) return 0;
  const int groups = a->group_rows > 0 ? (int)(M / a->group_rows) : 1;
  return stf_bn_bwd_reduce(a->dst, a->dst_cstride, nullptr, a->bnr->y, a->bnr->y_cstride, c.N, c.Hd, c.Wd, a->Nout,
                           groups, a->bnr->scale, a->bnr->shift, a->bnr->mean, a->bnr->invstd, a->bnr->relu ? 1 : 0,
                           nullptr, 0, nullptr, a->bnr->partial, stream);
}

static int igemm_launch(const stf_igemm_args* a, stf_stream_t stream) {
  const stf_conv_geom& c = a->g;
  if (a->Nout % 8 || c.Cs % 8 || c.src_cstride % 8 || a->dst_cstride % 4) return STF_EINVAL;
  if (c.transposed && !(c.stride == 1 || c.stride == 2)) return STF_EINVAL;
  if (a->scatter2x2 && (c.transposed || (a->Nout / 4) % 4)) return STF_EINVAL;
  if (((uintptr_t)a->src & 15) || ((uintptr_t)a->wgt & 15) || ((uintptr_t)a->dst & 7)) return STF_EINVAL;
  if (a->bnr && (a->stats || a->bias || a->lstm || a->scatter2x2 || !a->bnr->y || !a->bnr->partial || a->bnr->y_cstride % 8 ||
                 a->dst_cstride % 8 || ((uintptr_t)a->dst & 15) || ((uintptr_t)a->bnr->y & 15)))
    return STF_EINVAL;
  Geo g;
  g.src = (const uint16_t*)a->src; g.wgt = (const uint16_t*)a->wgt; g.dst = (uint16_t*)a->dst;
  g.bias = a->bias; g.stats = a->stats;
  g.N = c.N; g.Hs = c.Hs; g.Ws = c.Ws; g.Cs = c.Cs; g.scs = c.src_cstride;
  g.Hd = c.Hd; g.Wd = c.Wd; g.R = c.R; g.S = c.S; g.st = c.stride; g.pad = c.pad;
  g.M = c.N * c.Hd * c.Wd; g.K = c.R * c.S * c.Cs; g.Nout = a->Nout; g.dcs = a->dst_cstride;
  if (g.M <= 0) return 0;
  const int bm = pick_mtile(a);
  g.Mg = a->group_rows > 0 ? a->group_rows : g.M;
  if (g.M % g.Mg) return STF_EINVAL;
  g.tpg = (g.Mg + bm - 1) / bm;
  g.accumulate = a->accumulate;
  g.c_prev = nullptr; g.c_out = nullptr; g.h_out = nullptr; g.hcs = 0; g.gates = nullptr;
  g.bnr_y = nullptr; g.bnr_ycs = 0; g.bnr_scale = g.bnr_shift = g.bnr_mean = g.bnr_invstd = nullptr;
  g.bnr_relu = 0; g.bnr_part = nullptr;
  g.par = 0;
  g.ksplit = 1; g.ws = nullptr;
  static const int wkeep = stf::ab_switch("STF_HALO_WKEEP", 1);
  g.wkeep = wkeep;
  static const int full = stf::ab_switch("STF_HALO_FULL", 1);
  g.full = full;
  if (a->bnr) {
    g.bnr_y = (const uint16_t*)a->bnr->y; g.bnr_ycs = a->bnr->y_cstride;
    g.bnr_scale = a->bnr->scale; g.bnr_shift = a->bnr->shift; g.bnr_mean = a->bnr->mean;
    g.bnr_invstd = a->bnr->invstd; g.bnr_relu = a->bnr->relu; g.bnr_part = a->bnr->partial;
  }
  g.l_dh = nullptr; g.l_dhcs = 0; g.l_dcn = nullptr; g.l_dcp = nullptr; g.l_dg = nullptr;
  int lstm_epi = 0;
  if (a->lstm) {
    const stf_lstm_epi& l = *a->lstm;
    if (a->scatter2x2 || c.transposed || a->Nout % 4 || !l.c_out) return STF_EINVAL;
    if (l.backward) {
      if (!l.dh || !l.dc_prev || !l.dgates || ((uintptr_t)l.dgates & 7)) return STF_EINVAL;
      g.l_dh = (const uint16_t*)l.dh; g.l_dhcs = l.dh_cstride; g.l_dcn = l.dc_next; g.l_dcp = l.dc_prev;
      g.l_dg = (uint16_t*)l.dgates;
      lstm_epi = 2;
    } else {
      if (!l.h_out) return STF_EINVAL;
      lstm_epi = 1;
    }
    g.c_prev = l.c_prev; g.c_out = l.c_out; g.h_out = (uint16_t*)l.h_out;
    g.hcs = l.h_cstride; g.gates = l.gates;
  }
  const bool smallc = (c.Cs % BK) != 0;
  hipStream_t s = (hipStream_t)stream;
  const uint32_t src_bytes = (uint32_t)((uint64_t)c.N * c.Hs * c.Ws * c.src_cstride * 2);
  const char k = choose(a, dma_fits(a));
  if (k == 'K') {
    if ((g.Mg % (c.Hd * c.Wd)) != 0) return STF_EINVAL;
    const int TY = (c.Hd + C8_T - 1) / C8_T, TX = (c.Wd + C8_T - 1) / C8_T;
    const int tiles = c8_tiles(c), grid = c8_grid(a);
    // whole-pixel-row stores (STF_C8_FULL=0: the half-row stores, A/B)
    static const int c8_full = stf::ab_switch("STF_C8_FULL", 1) != 0;
    hipLaunchKernelGGL(conv3x3_c8_kernel, dim3(grid), dim3(256), 0, s, g, TY, TX, tiles / grid, tiles % grid,
                       c8_full);
    STF_CHECK_LAUNCH();
    return 0;
  }
  if (k == 'H') {
    if ((g.Mg % (c.Hd * c.Wd)) != 0) return STF_EINVAL;
    int ty, tx;
    halo_tiles(c, ty, tx);
    const int ix = halo_ix(a, a->stats != nullptr);
    if (ix > 1) ty = tx = 1;
    const long items = halo_items_ix(a, ix);
    const int grid = halo_grid(a, ix);
    static const int diag = stf::ablation_env("STF_HALO_DIAG");
#define STF_H(D) hipLaunchKernelGGL((conv3x3_halo_kernel<16, HALO_PW, 8, 2, D>), dim3(grid), dim3(512), 0, s, g, \
                                   src_bytes, ty, tx, (int)(items / grid), (int)(items % grid))
    const int d = halo_direct(a) ? (a->stats ? 2 : 1) : 0;
    const int per = (int)(items / grid), rem = (int)(items % grid);
    const bool dfr = halo_defer(a);
#define STF_HL(PWV, D, B) do {                                                                                      \
      if (dfr) hipLaunchKernelGGL((conv3x3_halo_kernel<16, PWV, 8, 2, 0, D, B, true>), dim3(grid), dim3(512), 0, s, g, \
                                  src_bytes, ty, tx, per, rem);                                                        \
      else hipLaunchKernelGGL((conv3x3_halo_kernel<16, PWV, 8, 2, 0, D, B>), dim3(grid), dim3(512), 0, s, g,          \
                              src_bytes, ty, tx, per, rem);                                                            \
    } while (0)
#define STF_H2(D, B) do {                                                                                           \
      if (dfr) hipLaunchKernelGGL((conv3x3_halo2_kernel<D, B, true>), dim3(grid), dim3(512), 0, s, g, src_bytes, ty,  \
                                  tx, per, rem);                                                                       \
      else hipLaunchKernelGGL((conv3x3_halo2_kernel<D, B>), dim3(grid), dim3(512), 0, s, g, src_bytes, ty, tx, per,   \
                              rem);                                                                                    \
    } while (0)
    if (ix == 1 && halo_wide(a)) {
      if (d == 2) hipLaunchKernelGGL((conv3x3_wide_kernel<2>), dim3(grid), dim3(512), 0, s, g, src_bytes, ty, tx, per, rem);
      else if (a->bnr) hipLaunchKernelGGL((conv3x3_wide_kernel<1, true>), dim3(grid), dim3(512), 0, s, g, src_bytes, ty, tx,
                                          per, rem);
      else hipLaunchKernelGGL((conv3x3_wide_kernel<1>), dim3(grid), dim3(512), 0, s, g, src_bytes, ty, tx, per, rem);
    } else if (ix == 4) {
      hipLaunchKernelGGL((conv3x3_halo4_kernel<0>), dim3(grid), dim3(256), 0, s, g, src_bytes, ty, tx, per, rem);
    } else if (ix > 1) {
      if (bnr_fused(a, k)) STF_H2(1, true);
      else if (d == 2) STF_H2(2, false);
      else if (d == 1) STF_H2(1, false);
      else STF_H2(0, false);
    } else if (bnr_fused(a, k)) {
      if (halo_pw(c) == 16) STF_HL(16, 1, true);
      else STF_HL(HALO_PW, 1, true);
    } else if (halo_pw(c) == 16) {
      if (d == 2) STF_HL(16, 2, false);
      else if (d == 1) STF_HL(16, 1, false);
      else STF_HL(16, 0, false);
    } else if (diag == 4) {                        // cycle buckets (tools/halo_timeline.py), no statistics
      hipLaunchKernelGGL((conv3x3_halo_kernel<16, HALO_PW, 8, 2, 4, 1, false>), dim3(grid), dim3(512), 0, s, g,
                         src_bytes, ty, tx, per, rem);
    } else if (diag == 2) {                        // ablation: no DMA reloads after the first stage
      if (d == 2) hipLaunchKernelGGL((conv3x3_halo_kernel<16, HALO_PW, 8, 2, 2, 2, false>), dim3(grid), dim3(512), 0,
                                     s, g, src_bytes, ty, tx, per, rem);
      else if (d == 1) hipLaunchKernelGGL((conv3x3_halo_kernel<16, HALO_PW, 8, 2, 2, 1, false>), dim3(grid), dim3(512),
                                          0, s, g, src_bytes, ty, tx, per, rem);
      else STF_H(2);
    } else if (d == 2) STF_HL(HALO_PW, 2, false);
    else if (d == 1) STF_HL(HALO_PW, 1, false);
    else STF_H(0);
#undef STF_H2
#undef STF_HL
#undef STF_H
    STF_CHECK_LAUNCH();
    return 0;
  }
  // stride-2 transposed gathers: rows by output parity class, only that class's taps
  // (STF_TRANS_PAR=0: all nine taps, 3/4 of them masked)
  static const bool par_on = stf::ab_switch("STF_TRANS_PAR", 1) != 0;
  if (par_on && c.transposed && c.stride == 2 && (k == 'A' || k == 'E') && g.Mg == g.M) {
    const int bmp = cfg_of(k).bm;
    // accumulating: tap-less classes add nothing, skip them (STF_TRANS_SKIP=0: launch them, A/B)
    static const bool skip_on = stf::ab_switch("STF_TRANS_SKIP", 1) != 0;
    // (only when the epilogue adds nothing of its own: no bias, statistics or fused BN reduce)
    const int par = a->accumulate && skip_on && !a->bias && !a->stats && !a->bnr ? 2 : 1;
    long blocks = 0;
    for (int cl = 0; cl < 4; ++cl) {
      const int ntap = ((c.R - (((cl >> 1) + c.pad) & 1) + 1) >> 1) * ((c.S - (((cl & 1) + c.pad) & 1) + 1) >> 1);
      if (par == 2 && ntap == 0) continue;
      blocks += ((long)c.N * ((c.Hd - (cl >> 1) + 1) >> 1) * ((c.Wd - (cl & 1) + 1) >> 1) + bmp - 1) / bmp;
    }
    g.par = par;
    g.tpg = (int)blocks;
  }
  const int ks = ksplit_of(a);
  if (ks > 1) {
    if (!a->ws || ((uintptr_t)a->ws & 15)) return STF_EINVAL;
    g.ksplit = ks; g.ws = a->ws;
  }
  switch (k) {
    case 'A': launch_dma<128, 128, 2, 2, 32, 4>(g, c.transposed, a->scatter2x2, lstm_epi, false, src_bytes, s); break;
    case 'E': launch_dma<256, 64, 4, 1, 32, 4>(g, c.transposed, a->scatter2x2, lstm_epi, false, src_bytes, s); break;
    case 'a': launch_dma<128, 128, 2, 2, 32, 4>(g, false, false, false, true, src_bytes, s); break;
    case 'e': launch_dma<256, 64, 4, 1, 32, 4>(g, false, false, false, true, src_bytes, s); break;
    case 'B': launch_dma_plain<256, 128, 4, 2, 64, 3>(g, a->scatter2x2, src_bytes, s, lstm_epi); break;
    case 'C': launch_dma_plain<256, 256, 2, 4, 64, 2>(g, a->scatter2x2, src_bytes, s, lstm_epi); break;
    case 'D': launch_dma_plain<512, 64, 8, 1, 64, 2>(g, a->scatter2x2, src_bytes, s, lstm_epi); break;
    case 'F': {                                    // plain gathers and the ConvT scatter only
      if (lstm_epi) return STF_EINVAL;
      dim3 grid(g.tpg * ((g.M + g.Mg - 1) / g.Mg), (g.Nout + 255) / 256, g.ksplit), block(512);
      if (a->scatter2x2)
        hipLaunchKernelGGL((igemm_dma_kernel<128, 256, 2, 4, 32, 2, false, true, 0>), grid, block, 0, s, g, src_bytes);
      else
        hipLaunchKernelGGL((igemm_dma_kernel<128, 256, 2, 4, 32, 2, false, false, 0>), grid, block, 0, s, g, src_bytes);
      break;
    }
    default:
      if (bm == 256) return launch_reg<256, 64, 4, 1>(g, smallc, c.transposed, a->scatter2x2, lstm_epi, s);
      return launch_reg<128, 128, 2, 2>(g, smallc, c.transposed, a->scatter2x2, lstm_epi, s);
  }
  STF_CHECK_LAUNCH();
  if (g.ksplit > 1) {
    const int tpg = (g.Mg + sk_rows(g.Nout) - 1) / sk_rows(g.Nout);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(tpg * (g.M / g.Mg)), dim3(NT), 0, s, g, tpg);
    STF_CHECK_LAUNCH();
  }
  return 0;
}
