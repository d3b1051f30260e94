// STF-LSTM-UNet specific kernels (src/stf_lstm_unet.py):
//   * input packing: [B, T(+P), C, H, W] fp32 -> t-major NHWC bf16 [T*B, H, W, Cpad]
//     with the PK maps appended as channels of every frame (:146-156,172-174)
//   * MaxPool2d(3, 2, 1) forward / backward (ResNet stem, :110,180)
//   * nn.LSTM weight packing into one gate-interleaved [W_ih | W_hh] GEMM operand,
//     the cell backward (BPTT) and the gradient unpacking (:124-127,214-236)
//   * bilinear (align_corners=True) resize of the PK maps into the PK-fusion
//     concat buffers (:189-200)
#include "common.h"
#include "../../include/stfunet.h"

namespace {

constexpr int NT = 256;

long grid_for(long units, long cap) {
  long b = (units + NT - 1) / NT;
  return b < 1 ? 1 : (b > cap ? cap : b);
}

// out[(t*B + b)][y][x][c]: c < C -> x[b][t][c], C <= c < C+P -> x[b][T + (c-C)][0], else 0
__global__ void pack_sequence_kernel(const float* __restrict__ x, int B, int Ttot, int C, int H, int W, int T, int P,
                                     int Cpad, uint16_t* __restrict__ out) {
  const long HW = (long)H * W, Pix = (long)T * B * HW;
  const int CG = Cpad / 8;
  for (long u = blockIdx.x * (long)NT + threadIdx.x; u < Pix * CG; u += (long)gridDim.x * NT) {
    const long pix = u % Pix;
    const int cg = (int)(u / Pix);
    const long img = pix / HW, hw = pix - img * HW;
    const int t = (int)(img / B), b = (int)(img - (long)t * B);
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = cg * 8 + j;
      float val = 0.f;
      if (c < C) val = x[(((long)b * Ttot + t) * C + c) * HW + hw];
      else if (c < C + P) val = x[(((long)b * Ttot + T + (c - C)) * C) * HW + hw];
      v[j] = val;
    }
    *reinterpret_cast<uint4*>(out + pix * Cpad + cg * 8) = pack8(v);
  }
}

// Stem im2col: cols[(t*B + b)][oy][ox][k], k = ci*KS*KS + r*KS + s (the PyTorch
// [Cout][Cin][KS][KS] weight order), value = input channel ci of frame t at
// (oy*st - pad + r, ox*st - pad + s), zero outside the image and for k >= Cin*KS*KS.
// Input channel ci < C is x[b][t][ci], C <= ci < C+P the PK map x[b][T+ci-C][0]
// (same channel order as pack_sequence).  One thread = 8 consecutive columns.
// One block per output row (image, oy): the KS input rows of every input channel it
// reads are staged in LDS with coalesced loads (zero padding written explicitly), then
// each thread assembles 16-B column chunks from LDS.  (A per-element gather from global
// memory put ~16 cache lines behind every 4-byte load instruction: 216 us vs ~60.)
constexpr int IM2COL_MAXC = 4, IM2COL_MAXW = 1024;
template <int KS>
__global__ __launch_bounds__(NT) void stem_im2col_kernel(const float* __restrict__ x, int B, int Ttot, int C, int H,
                                                         int W, int T, int P, int st, int pad, int Ho, int Wo,
                                                         int Kpad, uint16_t* __restrict__ out) {
  constexpr int KK = KS * KS;            // compile-time: the column -> (ci, r, s) split is multiplies
  extern __shared__ float rowbuf[];      // [Cin][KS][LW], column xx <-> input x = xx - pad
  const int Cin = C + P, LW = (Wo - 1) * st + KS;
  const int img = blockIdx.x / Ho, oy = blockIdx.x - img * Ho;
  const int t = img / B, b = img - t * B;
  for (int e = threadIdx.x; e < Cin * KS * LW; e += NT) {
    const int ci = e / (KS * LW), rem = e - ci * KS * LW, r = rem / LW, xx = rem - r * LW;
    const int iy = oy * st - pad + r, ix = xx - pad;
    float v = 0.f;
    if (iy >= 0 && iy < H && ix >= 0 && ix < W) {
      const long plane = ci < C ? ((long)b * Ttot + t) * C + ci : ((long)b * Ttot + T + (ci - C)) * C;
      v = x[(plane * H + iy) * (long)W + ix];
    }
    rowbuf[e] = v;
  }
  __syncthreads();
  const int CG = Kpad / 8, Kreal = Cin * KK;
  uint16_t* orow = out + ((long)img * Ho + oy) * Wo * (long)Kpad;
  if (NT % CG == 0) {
    // a thread's column group is fixed (NT is a multiple of CG): its 8 (ci, r, s) LDS offsets are
    // computed once, not per output pixel (the divisions made the kernel VALU-issue bound)
    const int cg = threadIdx.x % CG;
    int off[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = cg * 8 + j;
      const int ci = k / KK, rs = k - ci * KK, r = rs / KS, s = rs - r * KS;
      off[j] = k < Kreal ? (ci * KS + r) * LW + s : -1;
    }
    for (int ox = threadIdx.x / CG; ox < Wo; ox += NT / CG) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = off[j] >= 0 ? rowbuf[off[j] + ox * st] : 0.f;
      *reinterpret_cast<uint4*>(orow + (long)ox * Kpad + cg * 8) = pack8(v);
    }
    return;
  }
  for (int u = threadIdx.x; u < Wo * CG; u += NT) {
    const int ox = u / CG, cg = u - ox * CG;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = cg * 8 + j;
      float val = 0.f;
      if (k < Kreal) {
        const int ci = k / KK, rs = k - ci * KK, r = rs / KS, s = rs - r * KS;
        val = rowbuf[(ci * KS + r) * LW + ox * st + s];
      }
      v[j] = val;
    }
    *reinterpret_cast<uint4*>(orow + (long)ox * Kpad + cg * 8) = pack8(v);
  }
}

// MaxPool2d(k=3, s=2, p=1); first maximum in row-major window order (torch CPU)
__global__ void maxpool3_fwd_kernel(const uint16_t* __restrict__ x, int N, int H, int W, int C, int Ho, int Wo,
                                    uint16_t* __restrict__ out, uint8_t* __restrict__ argmax) {
  const int CG = C / 8;
  const long units = (long)N * Ho * Wo * CG;
  for (long u = blockIdx.x * (long)NT + threadIdx.x; u < units; u += (long)gridDim.x * NT) {
    const int cg = (int)(u % CG);
    const long p = u / CG;
    const int n = (int)(p / ((long)Ho * Wo));
    const int rem = (int)(p - (long)n * Ho * Wo);
    const int oy = rem / Wo, ox = rem - oy * Wo;
    // every valid tap's value is >= 0 (ReLU) > -inf, so the first valid tap always takes the
    // maximum and a strict '>' keeps the first maximum in row-major window order
    float mx[8];
    int am[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { mx[j] = -INFINITY; am[j] = 0; }
    for (int dy = 0; dy < 3; ++dy) {
      const int iy = 2 * oy - 1 + dy;
      if (iy < 0 || iy >= H) continue;
      for (int dx = 0; dx < 3; ++dx) {
        const int ix = 2 * ox - 1 + dx;
        if (ix < 0 || ix >= W) continue;
        float v[8];
        unpack8(*reinterpret_cast<const uint4*>(x + (((long)n * H + iy) * W + ix) * C + cg * 8), v);
#pragma unroll
        for (int j = 0; j < 8; ++j)          // first maximum in scan order (torch's index)
          if (v[j] > mx[j] || am[j] < 0) { mx[j] = v[j]; am[j] = dy * 3 + dx; }
      }
    }
    *reinterpret_cast<uint4*>(out + (size_t)p * C + cg * 8) = pack8(mx);
    if (argmax) {
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) { lo |= (uint32_t)am[j] << (8 * j); hi |= (uint32_t)am[4 + j] << (8 * j); }
      *reinterpret_cast<uint2*>(argmax + (size_t)p * C + cg * 8) = make_uint2(lo, hi);
    }
  }
}

// The stem's BatchNorm + ReLU fused into its max pool (src/stf_lstm_unet.py:178-180): each
// window tap is relu(y*scale[g]+shift[g]) rounded to the 16-bit storage -- exactly the value
// stf_bn_act would have stored in the activation a0 -- so the pooled output and the recorded
// argmax equal bn_act followed by maxpool3_fwd bit for bit, and a0 (4x the pooled bytes) is never
// written nor read back.  g = n / ipg (per-time-step statistics of the encoder).
__global__ void bn_act_maxpool3_kernel(const uint16_t* __restrict__ y, int N, int H, int W, int C, int Ho, int Wo,
                                       int ipg, const float* __restrict__ scale, const float* __restrict__ shift,
                                       uint16_t* __restrict__ out, uint8_t* __restrict__ argmax) {
  // 32-bit index math (the host checks units < 2^31; 64-bit divisions made this VALU-bound)
  const int CG = C / 8, HoWo = Ho * Wo;
  const int units = N * HoWo * CG;
  for (int u = blockIdx.x * NT + threadIdx.x; u < units; u += gridDim.x * NT) {
    const int p = u / CG, cg = u - p * CG;
    const int n = p / HoWo;
    const int rem = p - n * HoWo;
    const int oy = rem / Wo, ox = rem - oy * Wo;
    const int g = n / ipg;
    float sc[8], sh[8];
    {
      const float4 a = *reinterpret_cast<const float4*>(scale + (size_t)g * C + cg * 8);
      const float4 b = *reinterpret_cast<const float4*>(scale + (size_t)g * C + cg * 8 + 4);
      const float4 c = *reinterpret_cast<const float4*>(shift + (size_t)g * C + cg * 8);
      const float4 d = *reinterpret_cast<const float4*>(shift + (size_t)g * C + cg * 8 + 4);
      sc[0] = a.x; sc[1] = a.y; sc[2] = a.z; sc[3] = a.w; sc[4] = b.x; sc[5] = b.y; sc[6] = b.z; sc[7] = b.w;
      sh[0] = c.x; sh[1] = c.y; sh[2] = c.z; sh[3] = c.w; sh[4] = d.x; sh[5] = d.y; sh[6] = d.z; sh[7] = d.w;
    }
    // every valid tap's value is >= 0 (ReLU) > -inf, so the first valid tap always takes the
    // maximum and a strict '>' keeps the first maximum in row-major window order
    float mx[8];
    int am[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { mx[j] = -INFINITY; am[j] = 0; }
    for (int dy = 0; dy < 3; ++dy) {
      const int iy = 2 * oy - 1 + dy;
      if (iy < 0 || iy >= H) continue;
      for (int dx = 0; dx < 3; ++dx) {
        const int ix = 2 * ox - 1 + dx;
        if (ix < 0 || ix >= W) continue;
        float v[8];
        unpack8(*reinterpret_cast<const uint4*>(y + (((long)n * H + iy) * W + ix) * C + cg * 8), v);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float a = round_e(fmaxf(v[j] * sc[j] + sh[j], 0.f));     // bn_act's stored value
          if (a > mx[j]) { mx[j] = a; am[j] = dy * 3 + dx; }
        }
      }
    }
    const size_t o = (size_t)p * C + cg * 8;          // N*Ho*Wo*C may pass 2^31 (units < 2^31 only)
    *reinterpret_cast<uint4*>(out + o) = pack8(mx);
    if (argmax) {
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) { lo |= (uint32_t)am[j] << (8 * j); hi |= (uint32_t)am[4 + j] << (8 * j); }
      *reinterpret_cast<uint2*>(argmax + o) = make_uint2(lo, hi);
    }
  }
}

// gather form of the backward: every input pixel sums dout over the (<= 4)
// windows whose recorded first maximum is this pixel -- no atomics, fixed order
__global__ void maxpool3_bwd_kernel(const uint8_t* __restrict__ argmax, const uint16_t* __restrict__ dout, int N,
                                    int H, int W, int C, int Ho, int Wo, uint16_t* __restrict__ dx) {
  const int CG = C / 8;
  const long units = (long)N * H * W * CG;
  for (long u = blockIdx.x * (long)NT + threadIdx.x; u < units; u += (long)gridDim.x * NT) {
    const int cg = (int)(u % CG);
    const long p = u / CG;
    const int n = (int)(p / ((long)H * W));
    const int rem = (int)(p - (long)n * H * W);
    const int iy = rem / W, ix = rem - iy * W;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // windows containing iy: 2*oy-1 <= iy <= 2*oy+1  <=>  iy/2 <= oy <= (iy+1)/2
    for (int oy = iy / 2; oy <= min(Ho - 1, (iy + 1) / 2); ++oy) {
      for (int ox = ix / 2; ox <= min(Wo - 1, (ix + 1) / 2); ++ox) {
        const long wo = (((long)n * Ho + oy) * Wo + ox) * C + cg * 8;
        const uint2 am = *reinterpret_cast<const uint2*>(argmax + wo);
        const uint32_t me = (uint32_t)((iy - 2 * oy + 1) * 3 + (ix - 2 * ox + 1));
        float d[8];
        unpack8(*reinterpret_cast<const uint4*>(dout + wo), d);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t a = ((j < 4 ? am.x : am.y) >> (8 * (j & 3))) & 0xffu;
          if (a == me) acc[j] += d[j];
        }
      }
    }
    *reinterpret_cast<uint4*>(dx + p * C + cg * 8) = pack8(acc);
  }
}

// W_ih, W_hh [4C][C] (torch rows: gate q block q*C..) -> wcat [4C][2C] with row 4c+q,
// wcat_t [2C][4C] (its transpose, for the input gradient), bias[4c+q] = b_ih + b_hh
__global__ void lstm_pack_kernel(const float* __restrict__ wih, const float* __restrict__ whh,
                                 const float* __restrict__ bih, const float* __restrict__ bhh, int C,
                                 e16* __restrict__ wcat, e16* __restrict__ wcat_t, float* __restrict__ bias) {
  const long total = 8L * C * C;
  for (long o = blockIdx.x * (long)NT + threadIdx.x; o < total; o += (long)gridDim.x * NT) {
    const int row = (int)(o / (2 * C)), col = (int)(o - (long)row * 2 * C);   // row = 4c + q
    const int c = row >> 2, q = row & 3;
    const int src_row = q * C + c;
    const float v = col < C ? wih[(long)src_row * C + col] : whh[(long)src_row * C + col - C];
    wcat[o] = f2e(v);
    wcat_t[(long)col * 4 * C + row] = f2e(v);
    if (col == 0) bias[row] = (bih ? bih[src_row] : 0.f) + (bhh ? bhh[src_row] : 0.f);
  }
}

__global__ void lstm_unpack_grad_kernel(const float* __restrict__ dwcat, const float* __restrict__ dbias, int C,
                                        float* __restrict__ dwih, float* __restrict__ dwhh,
                                        float* __restrict__ dbih, float* __restrict__ dbhh) {
  const long total = 8L * C * C;
  for (long o = blockIdx.x * (long)NT + threadIdx.x; o < total; o += (long)gridDim.x * NT) {
    const int row = (int)(o / (2 * C)), col = (int)(o - (long)row * 2 * C);
    const int c = row >> 2, q = row & 3;
    const int dst_row = q * C + c;
    if (col < C) dwih[(long)dst_row * C + col] = dwcat[o];
    else dwhh[(long)dst_row * C + col - C] = dwcat[o];
    if (col == 0) {
      if (dbih) dbih[dst_row] = dbias[row];
      if (dbhh) dbhh[dst_row] = dbias[row];
    }
  }
}

// BPTT cell step for (m, c):  tc = tanh(c_t)
//   dc = dh*o*(1-tc^2) + dc_next;  do = dh*tc*o(1-o);  di = dc*g*i(1-i);
//   dg = dc*i*(1-g^2);  df = dc*c_prev*f(1-f);  dc_prev = dc*f
__global__ void lstm_cell_bwd_kernel(const float* __restrict__ gates, const float* __restrict__ cst,
                                     const float* __restrict__ cprev, const uint16_t* __restrict__ dh, int dhcs,
                                     const float* dc_in, float* dc_out, e16* __restrict__ dgates, long M, int C) {
  const long total = M * C;
  for (long u = blockIdx.x * (long)NT + threadIdx.x; u < total; u += (long)gridDim.x * NT) {
    const long m = u / C;
    const int c = (int)(u - m * C);
    const float4 gv = *reinterpret_cast<const float4*>(gates + m * 4 * C + 4 * c);
    const float h = e2f(reinterpret_cast<const e16*>(dh)[m * dhcs + c]);
    const float cp = cprev ? cprev[u] : 0.f;
    float d_i, d_f, d_g, d_o, dcp;
    lstm_cell_bwd(gv.x, gv.y, gv.z, gv.w, cst[u], cp, h, dc_in ? dc_in[u] : 0.f, d_i, d_f, d_g, d_o, dcp);
    dc_out[u] = dcp;
    const uint2 pk = make_uint2(pack2(d_i, d_f), pack2(d_g, d_o));
    *reinterpret_cast<uint2*>(dgates + m * 4 * C + 4 * c) = pk;
  }
}

// bilinear, align_corners=True (F.interpolate) of pk [B][P][H][W] to (h, w), written
// for every time step t into dst[(t*B + b)][y][x][coff + p] (bf16, stride dcs)
__global__ void pk_resize_kernel(const float* __restrict__ x, int B, int Ttot, int T, int P, int H, int W, int h,
                                 int w, uint16_t* __restrict__ dst, int dcs, int coff) {
  const long total = (long)T * B * h * w * P;
  for (long u = blockIdx.x * (long)NT + threadIdx.x; u < total; u += (long)gridDim.x * NT) {
    const int p = (int)(u % P);
    const long pix = u / P;
    const int xo = (int)(pix % w);
    const long r1 = pix / w;
    const int yo = (int)(r1 % h);
    const long img = r1 / h;
    const int b = (int)(img % B);
    const float sy = h > 1 ? (float)(H - 1) / (h - 1) : 0.f, sx = w > 1 ? (float)(W - 1) / (w - 1) : 0.f;
    const float fy = yo * sy, fx = xo * sx;
    const int y0 = min((int)fy, H - 1), x0 = min((int)fx, W - 1);
    const int y1 = min(y0 + 1, H - 1), x1 = min(x0 + 1, W - 1);
    const float ly = fy - y0, lx = fx - x0;
    const float* src = x + ((long)b * Ttot + T + p) * H * W;      // frame channel 0 of PK slot p
    const float v = (1.f - ly) * ((1.f - lx) * src[(long)y0 * W + x0] + lx * src[(long)y0 * W + x1]) +
                    ly * ((1.f - lx) * src[(long)y1 * W + x0] + lx * src[(long)y1 * W + x1]);
    reinterpret_cast<e16*>(dst)[pix * dcs + coff + p] = f2e(v);
  }
}

// ---------------------------------------------------------------------------
// The DecoderBlock's size fallback (src/stf_lstm_unet.py:56-57): when the transposed conv's
// 2h x 2w output differs from the skip's size (H or W not divisible by 32), the reference
// resizes it by F.interpolate(mode="bilinear", align_corners=True).  NHWC 16-bit, C % 8 == 0;
// PyTorch's arithmetic (upsample_bilinear2d): scale (in-1)/(out-1) in fp32, src = scale * dst,
// i0 = (int)src, i1 = i0 + (i0 < in-1), lambda = src - i0, fp32 blend, one 16-bit rounding.
STF_DEV void ac_coord(int o, float sc, int in, int& i0, int& i1, float& l1) {
  const float f = sc * (float)o;
  i0 = min((int)f, in - 1);
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l1 = f - (float)i0;
}

__global__ void bilinear_ac_fwd_kernel(const uint16_t* __restrict__ x, int N, int H, int W, int C, int xcs,
                                       uint16_t* __restrict__ y, int h, int w, int ycs) {
  const int CG = C / 8;
  const long units = (long)N * h * w * CG;
  const float sy = h > 1 ? (float)(H - 1) / (float)(h - 1) : 0.f;
  const float sx = w > 1 ? (float)(W - 1) / (float)(w - 1) : 0.f;
  for (long u = blockIdx.x * (long)NT + threadIdx.x; u < units; u += (long)gridDim.x * NT) {
    const int cg = (int)(u % CG);
    const long p = u / CG;
    const int ox = (int)(p % w);
    const long r = p / w;
    const int oy = (int)(r % h), n = (int)(r / h);
    int y0, y1, x0, x1;
    float ly, lx;
    ac_coord(oy, sy, H, y0, y1, ly);
    ac_coord(ox, sx, W, x0, x1, lx);
    const uint16_t* b = x + (long)n * H * W * xcs + cg * 8;
    float a00[8], a01[8], a10[8], a11[8], o[8];
    unpack8(*reinterpret_cast<const uint4*>(b + ((long)y0 * W + x0) * xcs), a00);
    unpack8(*reinterpret_cast<const uint4*>(b + ((long)y0 * W + x1) * xcs), a01);
    unpack8(*reinterpret_cast<const uint4*>(b + ((long)y1 * W + x0) * xcs), a10);
    unpack8(*reinterpret_cast<const uint4*>(b + ((long)y1 * W + x1) * xcs), a11);
    const float hy0 = 1.f - ly, wx0 = 1.f - lx;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = hy0 * (wx0 * a00[j] + lx * a01[j]) + ly * (wx0 * a10[j] + lx * a11[j]);
    *reinterpret_cast<uint4*>(y + p * ycs + cg * 8) = pack8(o);
  }
}

// backward as a gather (no atomics, fixed order): input pixel (iy, ix) sums w_y * w_x * dy over
// the output pixels whose interpolation reads it; the candidate rows / columns are a window
// around iy / scale, each checked with the forward's own coordinate arithmetic
__global__ void bilinear_ac_bwd_kernel(const uint16_t* __restrict__ dy, int N, int h, int w, int C, int dycs,
                                       uint16_t* __restrict__ dx, int H, int W, int dxcs) {
  const int CG = C / 8;
  const long units = (long)N * H * W * CG;
  const float sy = h > 1 ? (float)(H - 1) / (float)(h - 1) : 0.f;
  const float sx = w > 1 ? (float)(W - 1) / (float)(w - 1) : 0.f;
  for (long u = blockIdx.x * (long)NT + threadIdx.x; u < units; u += (long)gridDim.x * NT) {
    const int cg = (int)(u % CG);
    const long p = u / CG;
    const int ix = (int)(p % W);
    const long r = p / W;
    const int iy = (int)(r % H), n = (int)(r / H);
    const int oy0 = sy > 0.f ? max(0, (int)((float)(iy - 1) / sy) - 1) : 0;
    const int oy1 = sy > 0.f ? min(h - 1, (int)((float)(iy + 1) / sy) + 1) : h - 1;
    const int ox0 = sx > 0.f ? max(0, (int)((float)(ix - 1) / sx) - 1) : 0;
    const int ox1 = sx > 0.f ? min(w - 1, (int)((float)(ix + 1) / sx) + 1) : w - 1;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int oy = oy0; oy <= oy1; ++oy) {
      int y0, y1;
      float ly;
      ac_coord(oy, sy, H, y0, y1, ly);
      const float wy = (y0 == iy ? 1.f - ly : 0.f) + (y1 == iy ? ly : 0.f);
      if (wy == 0.f) continue;
      for (int ox = ox0; ox <= ox1; ++ox) {
        int x0, x1;
        float lx;
        ac_coord(ox, sx, W, x0, x1, lx);
        const float wx = (x0 == ix ? 1.f - lx : 0.f) + (x1 == ix ? lx : 0.f);
        if (wx == 0.f) continue;
        float g[8];
        unpack8(*reinterpret_cast<const uint4*>(dy + (((long)n * h + oy) * w + ox) * dycs + cg * 8), g);
        const float k = wy * wx;
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += k * g[j];
      }
    }
    *reinterpret_cast<uint4*>(dx + p * dxcs + cg * 8) = pack8(acc);
  }
}

// The same gather for the PK maps' input gradient (ABI v17): dy holds T frames of B images
// (t-major, [T*B][h][w], channels [0, 8) of stride dycs); the T frames are summed in fp32 at the
// low resolution (the resize is linear and the same for every frame) and the first P channels of
// the full-resolution sum are ADDED to out[b*obs + c*ocs + y*W + x] (fp32, the input's layout)
__global__ void bilinear_ac_bwd_tsum_kernel(const uint16_t* __restrict__ dy, int T, int B, int h, int w,
                                            int dycs, int P, float* __restrict__ out, long obs, long ocs, int H,
                                            int W) {
  const long units = (long)B * H * W;
  const float sy = h > 1 ? (float)(H - 1) / (float)(h - 1) : 0.f;
  const float sx = w > 1 ? (float)(W - 1) / (float)(w - 1) : 0.f;
  for (long p = blockIdx.x * (long)NT + threadIdx.x; p < units; p += (long)gridDim.x * NT) {
    const int ix = (int)(p % W);
    const long r = p / W;
    const int iy = (int)(r % H), b = (int)(r / H);
    const int oy0 = sy > 0.f ? max(0, (int)((float)(iy - 1) / sy) - 1) : 0;
    const int oy1 = sy > 0.f ? min(h - 1, (int)((float)(iy + 1) / sy) + 1) : h - 1;
    const int ox0 = sx > 0.f ? max(0, (int)((float)(ix - 1) / sx) - 1) : 0;
    const int ox1 = sx > 0.f ? min(w - 1, (int)((float)(ix + 1) / sx) + 1) : w - 1;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int oy = oy0; oy <= oy1; ++oy) {
      int y0, y1;
      float ly;
      ac_coord(oy, sy, H, y0, y1, ly);
      const float wy = (y0 == iy ? 1.f - ly : 0.f) + (y1 == iy ? ly : 0.f);
      if (wy == 0.f) continue;
      for (int ox = ox0; ox <= ox1; ++ox) {
        int x0, x1;
        float lx;
        ac_coord(ox, sx, W, x0, x1, lx);
        const float wx = (x0 == ix ? 1.f - lx : 0.f) + (x1 == ix ? lx : 0.f);
        if (wx == 0.f) continue;
        float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int t = 0; t < T; ++t) {
          float g[8];
          unpack8(*reinterpret_cast<const uint4*>(dy + ((((long)t * B + b) * h + oy) * w + ox) * dycs), g);
#pragma unroll
          for (int j = 0; j < 8; ++j) s[j] += g[j];
        }
        const float k = wy * wx;
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += k * s[j];
      }
    }
    float* o = out + (long)b * obs + (long)iy * W + ix;
    for (int c = 0; c < P; ++c) o[c * ocs] += acc[c];
  }
}


// Direct 7x7 / stride 2 / pad 3 stem convolution of a 1-channel frame sequence (ResNet-34 conv1,
// src/stf_lstm_unet.py:108,177) into NHWC bf16 [T*B][Ho][Wo][64], with the grouped BatchNorm
// statistics rows of its output -- the im2col + 1x1 GEMM path without the 268 MB im2col tensor
// written and read back (cfg3).  A persistent workgroup walks 16 x 16 output tiles; per tile the
// (2*16+5)^2 input patch (bf16, as the im2col rounds it) sits in LDS and every MFMA B fragment
// (8 k-slots = 8 taps of one output pixel) is gathered from it; the 64 x 64 weights (k = r*7 + s,
// zero past 49) stay in registers.  Same k order and MFMA sequence as the GEMM over the im2col
// columns; output, epilogue and statistics rows as conv3x3_c8_kernel.
constexpr int ST_T = 16, ST_P = 2 * ST_T + 5, ST_PR = ST_P * ST_P;   // 37 x 37 patch
constexpr int ST_LD = (ST_PR + 255) / 256;                             // patch values per thread
__global__ __launch_bounds__(256, 2) void stem7_conv_kernel(const float* __restrict__ x, int B, int Ttot, int H,
                                                            int W, int T, int Ho, int Wo,
                                                            const uint16_t* __restrict__ wgt,
                                                            uint16_t* __restrict__ y, float* __restrict__ stats,
                                                            int TY, int TX, int per, int rem) {
  __shared__ uint16_t patch[2][ST_PR];
  __shared__ float red[4][2][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fk = lane >> 4;
  const int tpi = TY * TX, N = T * B;
  const int cnt = per + (int)(blockIdx.x < (unsigned)rem);
  const int t0 = blockIdx.x * per + min((int)blockIdx.x, rem);
  e16x8 wf[4][2];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = (j >> 1) * 32 + (fr >> 2) * 8 + (j & 1) * 4 + (fr & 3);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) wf[j][ks] = *reinterpret_cast<const e16x8*>(wgt + (size_t)n * 64 + ks * 32 + fk * 8);
  }
  // this lane's 8 k-slots per k-step: tap offsets r * 37 + s in the patch (-1: zero column)
  int toff[2][8];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = ks * 32 + fk * 8 + e;
      toff[ks][e] = k < 49 ? (k / 7) * ST_P + k % 7 : -1;
    }
  if (stats && tid < 128) {
    for (int g = 0; g < T; ++g) stats[((size_t)(g * gridDim.x + blockIdx.x) * 2 + (tid >> 6)) * 64 + (tid & 63)] = 0.f;
  }
  const __amdgpu_buffer_rsrc_t rs_dst =
      __builtin_amdgcn_make_buffer_rsrc((void*)y, 0, (uint32_t)((size_t)N * Ho * Wo * 64 * 2), 0x00020000);
  float ld[ST_LD];
  auto load = [&](int tile) {
    const int img = tile / tpi, t2 = tile - img * tpi, ty = t2 / TX, tx = t2 - ty * TX;
    const int t = img / B, b = img - t * B;
    const float* plane = x + ((size_t)b * Ttot + t) * H * W;
#pragma unroll
    for (int q = 0; q < ST_LD; ++q) {
      const int e = tid + q * 256, py = e / ST_P, px = e - py * ST_P;
      const int iy = ty * 2 * ST_T - 3 + py, ix = tx * 2 * ST_T - 3 + px;
      ld[q] = (e < ST_PR && iy >= 0 && ix >= 0 && iy < H && ix < W) ? plane[(size_t)iy * W + ix] : 0.f;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int q = 0; q < ST_LD; ++q)
      if (tid + q * 256 < ST_PR) patch[buf][tid + q * 256] = __builtin_bit_cast(uint16_t, f2e(ld[q]));
  };
  float s1[2][8], s2[2][8];
  auto zero_sums = [&]() {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int e = 0; e < 8; ++e) { s1[h][e] = 0.f; s2[h][e] = 0.f; }
  };
  int run_key = -1;
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
      stats[((size_t)(run_key * gridDim.x + blockIdx.x) * 2 + q) * 64 + c] =
          red[0][q][c] + red[1][q][c] + red[2][q][c] + red[3][q][c];
    }
    __syncthreads();
    zero_sums();
  };
  zero_sums();
  if (cnt > 0) { load(t0); store(0); }
  __syncthreads();
  for (int kk = 0; kk < cnt; ++kk) {
    const int tile = t0 + kk, buf = kk & 1;
    const int img = tile / tpi, t2 = tile - img * tpi, ty = t2 / TX, tx = t2 - ty * TX;
    if (kk + 1 < cnt) load(tile + 1);
    const int key = img / B;                             // statistics group = time step
    if (stats && key != run_key) {
      if (run_key >= 0) flush();
      run_key = key;
    }
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      e16x8 xf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int base = 2 * (wave * 4 + i) * ST_P + 2 * fr;   // output pixel (row wave*4+i, column fr)
#pragma unroll
        for (int e = 0; e < 8; ++e)
          xf[i][e] = toff[ks][e] >= 0 ? __builtin_bit_cast(e16, patch[buf][base + toff[ks][e]]) : e16(0.f);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16x16x32(wf[j][ks], xf[i], acc[i][j]);
    }
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int oy = ty * ST_T + wave * 4 + i, ox = tx * ST_T + fr;
      const bool ok = oy < Ho && ox < Wo;
      const size_t m = ((size_t)img * Ho + oy) * Wo + ox;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float f[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          f[r] = round_e(acc[i][2 * h][r]);
          f[4 + r] = round_e(acc[i][2 * h + 1][r]);
        }
        const uint4 u = pack8(f);
        const uint32_t off = ok ? (uint32_t)((m * 64 + h * 32 + fk * 8) * 2) : 0xFFFFFFF0u;
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{u.x, u.y, u.z, u.w}, rs_dst, off, 0, 0);
        if (ok) {
#pragma unroll
          for (int e = 0; e < 8; ++e) { s1[h][e] += f[e]; s2[h][e] += f[e] * f[e]; }
        }
      }
    }
    if (kk + 1 < cnt) store(buf ^ 1);
    __syncthreads();
  }
  if (stats && run_key >= 0) flush();
}

// The stem's weight gradient without the im2col tensor: dW[n][k] = sum over output pixels of
// dy[px][n] * patch(px, tap k), per 16 x 16 output tile the dy tile [256 px][64] and the 37 x 37
// input patch in LDS, both MFMA operands gathered from them (k = pixel).  Wave w owns dy channels
// 16w..16w+15 x all 64 taps (49 real); every workgroup writes its fp32 partial [64][64] slab
// (ws[blockIdx.x]), stf_wgrad_reduce folds them in order.
__global__ __launch_bounds__(256, 2) void stem7_wgrad_kernel(const float* __restrict__ x, int B, int Ttot, int H,
                                                             int W, int T, int Ho, int Wo,
                                                             const uint16_t* __restrict__ dy, float* __restrict__ ws,
                                                             int TY, int TX, int per, int rem) {
  __shared__ uint16_t patch[2][ST_PR];
  __shared__ __attribute__((aligned(16))) uint16_t dyt[2][256 * 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fk = lane >> 4;
  const int tpi = TY * TX;
  const int cnt = per + (int)(blockIdx.x < (unsigned)rem);
  const int t0 = blockIdx.x * per + min((int)blockIdx.x, rem);
  int toff[4];                                           // this lane's tap (kb * 16 + fr) in the patch
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) {
    const int k = kb * 16 + fr;
    toff[kb] = k < 49 ? (k / 7) * ST_P + k % 7 : -1;
  }
  float ld[ST_LD];
  uint4 dv[8];
  auto load = [&](int tile) {
    const int img = tile / tpi, t2 = tile - img * tpi, ty = t2 / TX, tx = t2 - ty * TX;
    const int t = img / B, b = img - t * B;
    const float* plane = x + ((size_t)b * Ttot + t) * H * W;
#pragma unroll
    for (int q = 0; q < ST_LD; ++q) {
      const int e = tid + q * 256, py = e / ST_P, px = e - py * ST_P;
      const int iy = ty * 2 * ST_T - 3 + py, ix = tx * 2 * ST_T - 3 + px;
      ld[q] = (e < ST_PR && iy >= 0 && ix >= 0 && iy < H && ix < W) ? plane[(size_t)iy * W + ix] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = tid + q * 256, p = e >> 3, c8 = e & 7;
      const int oy = ty * ST_T + (p >> 4), ox = tx * ST_T + (p & 15);
      dv[q] = make_uint4(0, 0, 0, 0);
      if (oy < Ho && ox < Wo) dv[q] = *reinterpret_cast<const uint4*>(dy + (((size_t)img * Ho + oy) * Wo + ox) * 64 + c8 * 8);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int q = 0; q < ST_LD; ++q)
      if (tid + q * 256 < ST_PR) patch[buf][tid + q * 256] = __builtin_bit_cast(uint16_t, f2e(ld[q]));
#pragma unroll
    for (int q = 0; q < 8; ++q) *reinterpret_cast<uint4*>(&dyt[buf][(tid + q * 256) * 8]) = dv[q];
  };
  f32x4 acc[4];
#pragma unroll
  for (int kb = 0; kb < 4; ++kb) acc[kb] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (cnt > 0) { load(t0); store(0); }
  __syncthreads();
  for (int kk = 0; kk < cnt; ++kk) {
    const int buf = kk & 1;
    if (kk + 1 < cnt) load(t0 + kk + 1);
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      // k-slots fk*8+e = pixels ks*32 + fk*8 + e: one 8-pixel run of output row (ks*32 + fk*8) / 16
      const int p0 = ks * 32 + fk * 8;
      const int pb = 2 * (p0 >> 4) * ST_P + 2 * (p0 & 15);
      e16x8 a;
#pragma unroll
      for (int e = 0; e < 8; ++e) a[e] = __builtin_bit_cast(e16, dyt[buf][(p0 + e) * 64 + wave * 16 + fr]);
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        e16x8 bq;
#pragma unroll
        for (int e = 0; e < 8; ++e)
          bq[e] = toff[kb] >= 0 ? __builtin_bit_cast(e16, patch[buf][pb + 2 * e + toff[kb]]) : e16(0.f);
        acc[kb] = mfma16x16x32(a, bq, acc[kb]);
      }
    }
    if (kk + 1 < cnt) store(buf ^ 1);
    __syncthreads();
  }
  // lane (fr, fk), element r: dy channel wave*16 + 4*fk + r, tap kb*16 + fr
  float* slab = ws + (size_t)blockIdx.x * 64 * 64;
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int r = 0; r < 4; ++r) slab[(wave * 16 + 4 * fk + r) * 64 + kb * 16 + fr] = acc[kb][r];
}

int stem7_tiles(int N, int Ho, int Wo, int& TY, int& TX) {
  TY = (Ho + ST_T - 1) / ST_T;
  TX = (Wo + ST_T - 1) / ST_T;
  return N * TY * TX;
}

int stem7_cus() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return n;
}

}  // namespace

extern "C" int stf_bilinear_ac_fwd(const void* x, int N, int H, int W, int C, int x_cstride, void* y, int h, int w,
                                   int y_cstride, stf_stream_t stream) {
  if (!x || !y || N < 1 || H < 1 || W < 1 || h < 1 || w < 1 || C < 8 || C % 8 || x_cstride < C ||
      y_cstride < C || x_cstride % 8 || y_cstride % 8 || ((uintptr_t)x & 15) || ((uintptr_t)y & 15))
    return STF_EINVAL;
  const long units = (long)N * h * w * (C / 8);
  hipLaunchKernelGGL(bilinear_ac_fwd_kernel, dim3(grid_for(units, 8192)), dim3(NT), 0, (hipStream_t)stream,
                     (const uint16_t*)x, N, H, W, C, x_cstride, (uint16_t*)y, h, w, y_cstride);
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_bilinear_ac_bwd(const void* dy, int N, int h, int w, int C, int dy_cstride, void* dx, int H,
                                   int W, int dx_cstride, stf_stream_t stream) {
  if (!dy || !dx || N < 1 || H < 1 || W < 1 || h < 1 || w < 1 || C < 8 || C % 8 || dy_cstride < C ||
      dx_cstride < C || dy_cstride % 8 || dx_cstride % 8 || ((uintptr_t)dy & 15) || ((uintptr_t)dx & 15))
    return STF_EINVAL;
  const long units = (long)N * H * W * (C / 8);
  hipLaunchKernelGGL(bilinear_ac_bwd_kernel, dim3(grid_for(units, 8192)), dim3(NT), 0, (hipStream_t)stream,
                     (const uint16_t*)dy, N, h, w, C, dy_cstride, (uint16_t*)dx, H, W, dx_cstride);
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_bilinear_ac_bwd_tsum(const void* dy, int T, int B, int h, int w, int dy_cstride, int P,
                                        float* out, int64_t out_bstride, int64_t out_cstride, int H, int W,
                                        stf_stream_t stream) {
  if (!dy || !out || T < 1 || B < 1 || H < 1 || W < 1 || h < 1 || w < 1 || P < 1 || P > 8 || dy_cstride < 8 ||
      dy_cstride % 8 || ((uintptr_t)dy & 15) || out_bstride < 1 || out_cstride < 1)
    return STF_EINVAL;
  const long units = (long)B * H * W;
  hipLaunchKernelGGL(bilinear_ac_bwd_tsum_kernel, dim3(grid_for(units, 8192)), dim3(NT), 0, (hipStream_t)stream,
                     (const uint16_t*)dy, T, B, h, w, dy_cstride, P, out, (long)out_bstride, (long)out_cstride, H, W);
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_pack_sequence(const float* x, int B, int Ttot, int C, int H, int W, int T, int P, int Cpad,
                                 void* out, stf_stream_t stream) {
  if (Cpad % 8 || Cpad < C + P || Ttot < T + P || (P && C != 1)) return STF_EINVAL;
  const long units = (long)T * B * H * W * (Cpad / 8);
  hipLaunchKernelGGL(pack_sequence_kernel, dim3(grid_for(units, 8192)), dim3(NT), 0, (hipStream_t)stream, x, B,
                     Ttot, C, H, W, T, P, Cpad, (uint16_t*)out);
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_stem_im2col(const float* x, int B, int Ttot, int C, int H, int W, int T, int P, int KS,
                               int stride, int pad, int Kpad, void* out, stf_stream_t stream) {
  if (Kpad % 8 || Kpad < (C + P) * KS * KS || Ttot < T + P || (P && C != 1) || KS < 1 || stride < 1 || pad < 0)
    return STF_EINVAL;
  const int Ho = (H + 2 * pad - KS) / stride + 1, Wo = (W + 2 * pad - KS) / stride + 1;
  if (KS != 7) return STF_EINVAL;         // the ResNet stem (other sizes: add an instantiation)
  const int LW = (Wo - 1) * stride + KS;
  if (C + P > IM2COL_MAXC || LW > IM2COL_MAXW) return STF_EINVAL;
  const size_t lds = (size_t)(C + P) * KS * LW * sizeof(float);
  hipLaunchKernelGGL(stem_im2col_kernel<7>, dim3((unsigned)((long)T * B * Ho)), dim3(NT), lds, (hipStream_t)stream, x,
                     B, Ttot, C, H, W, T, P, stride, pad, Ho, Wo, Kpad, (uint16_t*)out);
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_maxpool3s2_fwd(const void* x, int N, int H, int W, int C, void* out, void* argmax,
                                  stf_stream_t stream) {
  if (C % 8) return STF_EINVAL;
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  const long units = (long)N * Ho * Wo * (C / 8);
  hipLaunchKernelGGL(maxpool3_fwd_kernel, dim3(grid_for(units, 8192)), dim3(NT), 0, (hipStream_t)stream,
                     (const uint16_t*)x, N, H, W, C, Ho, Wo, (uint16_t*)out, (uint8_t*)argmax);
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_bn_act_maxpool3s2(const void* y, int N, int H, int W, int C, int groups, const float* scale,
                                     const float* shift, void* out, void* argmax, stf_stream_t stream) {
  if (C % 8 || groups < 1 || N % groups || !y || !scale || !shift || !out) return STF_EINVAL;
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  const long units = (long)N * Ho * Wo * (C / 8);
  // 32-bit unit index incl. its grid stride (u + gridDim.x * NT must not wrap); byte offsets are 64-bit
  if (units >= (1L << 31) - 8192L * NT || (long)N * H * W * C >= (1L << 31) * 8L) return STF_EINVAL;
  hipLaunchKernelGGL(bn_act_maxpool3_kernel, dim3(grid_for(units, 8192)), dim3(NT), 0, (hipStream_t)stream,
                     (const uint16_t*)y, N, H, W, C, Ho, Wo, N / groups, scale, shift, (uint16_t*)out,
                     (uint8_t*)argmax);
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_maxpool3s2_bwd(const void* argmax, const void* dout, int N, int H, int W, int C, void* dx,
                                  stf_stream_t stream) {
  if (C % 8 || !argmax || !dout || !dx) return STF_EINVAL;     // the forward must have recorded the argmax
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  const long units = (long)N * H * W * (C / 8);
  hipLaunchKernelGGL(maxpool3_bwd_kernel, dim3(grid_for(units, 8192)), dim3(NT), 0, (hipStream_t)stream,
                     (const uint8_t*)argmax, (const uint16_t*)dout, N, H, W, C, Ho, Wo, (uint16_t*)dx);
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_lstm_pack(const float* w_ih, const float* w_hh, const float* b_ih, const float* b_hh, int C,
                             void* wcat, void* wcat_t, float* bias, stf_stream_t stream) {
  // the step GEMM's K = 2C rows stream in 32-channel steps (no masked K tail on the
  // LSTM epilogue path) and the bias gradient's channel sum wants 4C / 8 | 256:
  // hidden sizes 16, 32, ..., 512 (the reference's are 64..512)
  if (C < 16 || C % 16 || 512 % C) return STF_EINVAL;
  hipLaunchKernelGGL(lstm_pack_kernel, dim3(grid_for(8L * C * C, 4096)), dim3(NT), 0, (hipStream_t)stream, w_ih,
                     w_hh, b_ih, b_hh, C, (e16*)wcat, (e16*)wcat_t, bias);
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_lstm_unpack_grad(const float* dwcat, const float* dbias, int C, float* dw_ih, float* dw_hh,
                                    float* db_ih, float* db_hh, stf_stream_t stream) {
  hipLaunchKernelGGL(lstm_unpack_grad_kernel, dim3(grid_for(8L * C * C, 4096)), dim3(NT), 0, (hipStream_t)stream,
                     dwcat, dbias, C, dw_ih, dw_hh, db_ih, db_hh);
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_lstm_cell_bwd(const float* gates, const float* c_t, const float* c_prev, const void* dh,
                                 int dh_cstride, const float* dc_in, float* dc_out, void* dgates, int64_t M, int C,
                                 stf_stream_t stream) {
  if (C % 2) return STF_EINVAL;
  hipLaunchKernelGGL(lstm_cell_bwd_kernel, dim3(grid_for((long)M * C, 8192)), dim3(NT), 0, (hipStream_t)stream,
                     gates, c_t, c_prev, (const uint16_t*)dh, dh_cstride, dc_in, dc_out, (e16*)dgates, (long)M, C);
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_pk_resize(const float* x, int B, int Ttot, int T, int P, int H, int W, int h, int w, void* dst,
                             int dst_cstride, int coff, stf_stream_t stream) {
  const long total = (long)T * B * h * w * P;
  hipLaunchKernelGGL(pk_resize_kernel, dim3(grid_for(total, 8192)), dim3(NT), 0, (hipStream_t)stream, x, B, Ttot,
                     T, P, H, W, h, w, (uint16_t*)dst, dst_cstride, coff);
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_stem_conv7_grid(int B, int T, int H, int W) {
  if (B < 1 || T < 1 || H < 1 || W < 1) return 0;
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  int TY, TX;
  const int tiles = stem7_tiles(T * B, Ho, Wo, TY, TX);
  return std::min(tiles, 2 * stem7_cus());
}

extern "C" int stf_stem_conv7(const float* x, int B, int Ttot, int H, int W, int T, const void* wgt, void* y,
                              float* stats, stf_stream_t stream) {
  if (!x || !wgt || !y || B < 1 || T < 1 || Ttot < T || H < 1 || W < 1) return STF_EINVAL;
  if (((uintptr_t)wgt & 15) || ((uintptr_t)y & 15)) return STF_EINVAL;
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  if ((size_t)T * B * Ho * Wo * 64 * 2 >= 0xFFFFFF00ull) return STF_EINVAL;    // 32-bit store offsets
  int TY, TX;
  const int tiles = stem7_tiles(T * B, Ho, Wo, TY, TX);
  const int grid = stf_stem_conv7_grid(B, T, H, W);
  hipLaunchKernelGGL(stem7_conv_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, x, B, Ttot, H, W, T, Ho, Wo,
                     (const uint16_t*)wgt, (uint16_t*)y, stats, TY, TX, tiles / grid, tiles % grid);
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_stem_wgrad7(const float* x, int B, int Ttot, int H, int W, int T, const void* dy, float* ws,
                               stf_stream_t stream) {
  if (!x || !dy || !ws || B < 1 || T < 1 || Ttot < T || H < 1 || W < 1) return STF_EINVAL;
  if (((uintptr_t)dy & 15) || ((uintptr_t)ws & 15)) return STF_EINVAL;
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  int TY, TX;
  const int tiles = stem7_tiles(T * B, Ho, Wo, TY, TX);
  const int grid = stf_stem_conv7_grid(B, T, H, W);
  hipLaunchKernelGGL(stem7_wgrad_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, x, B, Ttot, H, W, T, Ho, Wo,
                     (const uint16_t*)dy, ws, TY, TX, tiles / grid, tiles % grid);
  STF_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------------------
// Input gradient of the stem conv 7x7 / stride 2 / pad 3 (ResNet-34 conv1, src/stf_lstm_unet.py:102;
// what autograd returns for the input sequence, :139-256): dx[b][t][c][y][x] = sum over the taps
// (r, s) with y + 3 - r and x + 3 - s even of dy[t*B + b][(y + 3 - r) / 2][(x + 3 - s) / 2][n] *
// w[n][c][r][s].  A workgroup owns ONE parity class (y & 1, x & 1) of a 32 x 32 input tile, so all
// of its lanes walk the same 3-4 x 3-4 taps and read the fp32 weights from LDS as broadcasts; each
// dy row (64 channels, 128 B) is read once per tap and dotted with up to 4 input channels' weights.
// fp32 accumulation, fp32 weights (the master copy), 16-bit dy as stored.  Not on the training
// path (train_one_epoch never asks for input gradients).
constexpr int SD_CC = 4;                                 // input channels per pass (LDS: 4 x 49 x 64 fp32)
__global__ __launch_bounds__(256) void stem7_dgrad_kernel(const uint16_t* __restrict__ dy, const float* __restrict__ w,
                                                         int B, int Ttot, int Cf, int H, int W, int Ho, int Wo,
                                                         int TY, int TX, float* __restrict__ dx) {
  __shared__ float wl[SD_CC][49][64];
  const int tid = threadIdx.x;
  int blk = blockIdx.x;
  const int cls = blk & 3;
  blk >>= 2;
  const int tx = blk % TX, ty = (blk / TX) % TY, img = blk / (TX * TY);
  const int t = img / B, b = img - t * B;
  const int cy = cls >> 1, cx = cls & 1;
  const int y = ty * 32 + 2 * (tid >> 4) + cy, x = tx * 32 + 2 * (tid & 15) + cx;
  const bool ok = y < H && x < W;
  const int r0 = (cy + 1) & 1, s0 = (cx + 1) & 1;       // first tap with y + 3 - r even
  for (int c0 = 0; c0 < Cf; c0 += SD_CC) {
    const int cc = min(SD_CC, Cf - c0);
    __syncthreads();
    for (int i = tid; i < SD_CC * 49 * 64; i += 256) {
      const int j = i / (49 * 64), k = (i / 64) % 49, n = i % 64;
      wl[j][k][n] = j < cc ? w[((size_t)n * Cf + c0 + j) * 49 + k] : 0.f;
    }
    __syncthreads();
    float acc[SD_CC] = {0.f, 0.f, 0.f, 0.f};
    for (int r = r0; r < 7; r += 2) {
      const int oy = (y + 3 - r) >> 1;
      for (int s = s0; s < 7; s += 2) {
        const int ox = (x + 3 - s) >> 1;
        if (!ok || oy < 0 || oy >= Ho || ox < 0 || ox >= Wo) continue;
        const uint4* row = reinterpret_cast<const uint4*>(dy + (((size_t)img * Ho + oy) * Wo + ox) * 64);
        const int k = r * 7 + s;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const uint4 u = row[q];
          const uint32_t v[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
          for (int h = 0; h < 4; ++h) {
            const float lo = e2f(__builtin_bit_cast(e16, (uint16_t)(v[h] & 0xFFFF)));
            const float hi = e2f(__builtin_bit_cast(e16, (uint16_t)(v[h] >> 16)));
            const int n = q * 8 + h * 2;
#pragma unroll
            for (int j = 0; j < SD_CC; ++j) acc[j] += lo * wl[j][k][n] + hi * wl[j][k][n + 1];
          }
        }
      }
    }
    if (ok)
      for (int j = 0; j < cc; ++j) dx[(((size_t)b * Ttot + t) * Cf + c0 + j) * H * W + (size_t)y * W + x] = acc[j];
  }
}

extern "C" int stf_stem_dgrad7(const void* dy, const float* w, int B, int Ttot, int Cf, int H, int W, int T,
                               float* dx, stf_stream_t stream) {
  if (!dy || !w || !dx || B < 1 || T < 1 || Ttot < T || Cf < 1 || H < 1 || W < 1) return STF_EINVAL;
  if ((uintptr_t)dy & 15) return STF_EINVAL;
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  const int TY = (H + 31) / 32, TX = (W + 31) / 32;
  const long blocks = (long)T * B * TY * TX * 4;
  if (blocks > 0x7FFFFFFFL) return STF_EINVAL;
  hipLaunchKernelGGL(stem7_dgrad_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                     (const uint16_t*)dy, w, B, Ttot, Cf, H, W, Ho, Wo, TY, TX, dx);
  STF_CHECK_LAUNCH();
  return 0;
}
