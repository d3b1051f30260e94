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
  int colmajor;         // fused 3x3: walk pixel tiles column-major (vertical neighbours in turn)
  int one_slab;         // timing-only ablation (STF_WGRAD_ONE_SLAB=1): every split writes slab 0
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
      e16x8 af[TM], bfr[TN];
      const int krow = kk + 8 * g + q;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int col = wm * WTM + i * 16 + p4;
        v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(sa + krow * SA + col));
        v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(sa + (krow + 4) * SA + col));
        short s8[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[i] = __builtin_bit_cast(e16x8, s8);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn * WTN + j * 16 + p4;
        v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(sb + krow * SB + col));
        v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(sb + (krow + 4) * SB + col));
        short s8[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bfr[j] = __builtin_bit_cast(e16x8, s8);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = mfma16x16x32(af[i], bfr[j], acc[i][j]);
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


// ---------------------------------------------------------------------------
// Fused-tap weight gradient for 3x3 / stride 1 / pad 1 convolutions.
//
// A block owns a 64 (dy channel) x 64 (x channel) tile for ALL nine taps and
// walks a run of 2-D pixel tiles (PH x PW = 64 output pixels).  Per pixel tile
// it stages the dy tile [64 px][64 n] and the x halo [(PH+2)(PW+2) px][64 c] in
// LDS; the nine taps are nine shifted views of the halo, so every dy / x
// element is read from HBM about once (the per-tap kernel above reads both 9x,
// which bounds it by HBM at C = 64).  MFMA k-slot -> pixel is permuted so the
// eight rows a 32-lane half reads with ds_read_b64_tr_b16 are eight consecutive
// pixels, i.e. eight consecutive LDS rows (160 B stride: disjoint bank octets).
// Waves: 1 (n) x 4 (c); each holds 64 n x 16 c x 9 taps = 36 accumulators.
template <int PW, int DIAG = 0>
__global__ __launch_bounds__(NT, 2) void wgrad3x3_kernel(WArgs a, int tiles_y, int tiles_x, int ntiles) {
  constexpr int PH = 64 / PW, HW = PW + 2, HR = (PH + 2) * HW;
  constexpr int SR = 64 + 16;                   // LDS row stride (elements), 160 B
  constexpr int A_EL = 64 * SR, B_EL = HR * SR;
  constexpr int CHA = 64 * 8 / NT;              // dy 16-B chunks per thread (2)
  constexpr int CHB = (HR * 8 + NT - 1) / NT;   // halo chunks per thread
  __shared__ __attribute__((aligned(16))) uint16_t smem[2][A_EL + B_EL];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // wave = 16-channel slice of x (TN = 1) x all 64 dy channels (TM = 4): the dy
  // fragments serve all nine taps, so fewer LDS reads per MFMA than 2 x 2 waves
  constexpr int TMW = 4, TNW = 1;
  const int wn = wave;
  const int split = blockIdx.x;
  const int n0 = blockIdx.y * 64, c0 = blockIdx.z * 64;
  const int t_begin = split * a.chunk, t_end = min(ntiles, t_begin + a.chunk);
  const int per_img = tiles_y * tiles_x;

  uint4 ra[CHA], rb[CHB];
  auto load = [&](int t) {
    const int img = t / per_img, rem = t - img * per_img;
    // column-major: the next tile is the one below, whose halo shares two of the (PH + 2)
    // rows just fetched (L2 hits) -- row-major neighbours share only two columns
    int ty, tx;
    if (a.colmajor) { tx = rem / tiles_y; ty = rem - tx * tiles_y; }
    else { ty = rem / tiles_x; tx = rem - ty * tiles_x; }
    const int y0 = ty * PH, x0 = tx * PW;
#pragma unroll
    for (int i = 0; i < CHA; ++i) {
      const int e = tid + i * NT, px = e >> 3, ch = e & 7;
      const int yd = y0 + px / PW, xd = x0 + px % PW;
      ra[i] = make_uint4(0, 0, 0, 0);
      if (yd < a.Hd && xd < a.Wd)
        ra[i] = *reinterpret_cast<const uint4*>(a.dy + (size_t)((img * a.Hd + yd) * a.Wd + xd) * a.dycs + n0 + ch * 8);
    }
#pragma unroll
    for (int i = 0; i < CHB; ++i) {
      const int e = tid + i * NT, hp = e >> 3, ch = e & 7;
      const int ys = y0 - 1 + hp / HW, xs = x0 - 1 + hp % HW;
      rb[i] = make_uint4(0, 0, 0, 0);
      if (hp < HR && ys >= 0 && xs >= 0 && ys < a.Hs && xs < a.Ws)
        rb[i] = *reinterpret_cast<const uint4*>(a.x + (size_t)((img * a.Hs + ys) * a.Ws + xs) * a.xcs + c0 + ch * 8);
    }
  };
  auto store = [&](int buf) {
    uint16_t* sa = smem[buf];
    uint16_t* sb = sa + A_EL;
#pragma unroll
    for (int i = 0; i < CHA; ++i) {
      const int e = tid + i * NT;
      *reinterpret_cast<uint4*>(sa + (e >> 3) * SR + (e & 7) * 8) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < CHB; ++i) {
      const int e = tid + i * NT;
      if (e < HR * 8) *reinterpret_cast<uint4*>(sb + (e >> 3) * SR + (e & 7) * 8) = rb[i];
    }
  };

  f32x4 acc[9][TMW][TNW];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < TMW; ++i)
#pragma unroll
      for (int j = 0; j < TNW; ++j) acc[t][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // lane (g, q, p4): k-slot 8g + 4h + q (h = lo/hi read) holds pixel
  // 16(g>>1) + 8h + 4(g&1) + q of the 32-pixel step.
  const int g = lane >> 4, q = (lane >> 2) & 3, p4 = (lane & 3) * 4;
  const int pl = 16 * (g >> 1) + 4 * (g & 1) + q;          // + 8h + kk
  int arow[2][2], brow[2][2];                                // [kk/32][h]
#pragma unroll
  for (int k2 = 0; k2 < 2; ++k2)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int px = 32 * k2 + 8 * h + pl;
      arow[k2][h] = px * SR;
      brow[k2][h] = ((px / PW) * HW + px % PW) * SR;
    }

  const int steps = t_end - t_begin;
  // DIAG 4 (timing only, the slabs are overwritten): per-wave cycle buckets (s_memtime) --
  // load issue, MFMA steps, LDS store (incl. the wait for the loads), barrier
  uint64_t tb[4] = {0, 0, 0, 0}, tprev = 0;
  auto stamp = [&](int k) {
    if constexpr (DIAG == 4) {
      const uint64_t tt = __builtin_amdgcn_s_memtime();
      if (k >= 0) tb[k] += tt - tprev;
      tprev = tt;
    }
  };
  if (steps > 0) { load(t_begin); store(0); }
  __syncthreads();
  for (int it = 0; it < steps; ++it) {
    const int cur = it & 1;
    stamp(-1);
    if (it + 1 < steps && (DIAG != 1 || it < 1)) load(t_begin + it + 1);
    stamp(0);
    const uint16_t* sa = smem[cur];
    const uint16_t* sb = sa + A_EL;
    if (DIAG == 2) { if (it + 1 < steps) store(cur ^ 1); __syncthreads(); continue; }
    // software-pipelined: the 18 (k-step, tap) steps in one flat sequence, B fragments
    // read two steps ahead (across the k-step boundary), the second k-step's A fragments
    // four steps before they are needed -- LDS latency hides behind the MFMAs
    auto readA = [&](int k2, int i) {
      const int col = i * 16 + p4;
      v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(sa + arow[k2][0] + col));
      v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(sa + arow[k2][1] + col));
      return __builtin_bit_cast(e16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    };
    auto readB = [&](int st) {
      const int k2 = st / 9, t = st % 9;
      const int toff = ((t / 3) * HW + t % 3) * SR;
      const int col = wn * 16 + p4;
      v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(sb + brow[k2][0] + toff + col));
      v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(sb + brow[k2][1] + toff + col));
      return __builtin_bit_cast(e16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    };
    e16x8 af[2][TMW], bq[18];
#pragma unroll
    for (int i = 0; i < TMW; ++i) af[0][i] = readA(0, i);
    bq[0] = readB(0);
    bq[1] = readB(1);
#pragma unroll
    for (int st = 0; st < 18; ++st) {
      if (st + 2 < 18) bq[st + 2] = readB(st + 2);
      if (st == 4) {
#pragma unroll
        for (int i = 0; i < TMW; ++i) af[1][i] = readA(1, i);
      }
      const int k2 = st / 9, t = st % 9;
#pragma unroll
      for (int i = 0; i < TMW; ++i)
        acc[t][i][0] = mfma16x16x32(af[k2][i], bq[st], acc[t][i][0]);
      __builtin_amdgcn_sched_barrier(0);        // keep the prefetch distance (no re-clustering)
    }
    stamp(1);
    if (it + 1 < steps) store(cur ^ 1);
    stamp(2);
    __syncthreads();
    stamp(3);
  }

  const int RSC = 9 * a.Cs;
  float* out = a.ws + (size_t)(a.one_slab ? 0 : split) * a.Nout * RSC;
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < TMW; ++i)
#pragma unroll
      for (int j = 0; j < TNW; ++j) {
        const int k = t * a.Cs + c0 + wn * 16 * TNW + j * 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = n0 + i * 16 + (lane >> 4) * 4 + r;
          out[(size_t)n * RSC + k] = acc[t][i][j][r];
        }
      }
  if constexpr (DIAG == 4) {
    // (after the real results, so the MFMA work is not dead code) the buckets overwrite the
    // first 32 floats of the block's tile: row n0, columns c0.. of tap 0
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (lane == 0) {
      unsigned long long* d = reinterpret_cast<unsigned long long*>(out + (size_t)n0 * RSC + c0) + wave * 4;
#pragma unroll
      for (int k = 0; k < 4; ++k) d[k] = tb[k];
    }
  }
}

// ---------------------------------------------------------------------------
// Fused-tap 3x3 weight gradient of the 8-channel-input layer (UNet's first conv, the input of
// conv3x3_c8_kernel; src/unet.py:10-18): dW[n][tap*8 + c] = sum over pixels of dy[px][n] *
// x[px + tap][c].  A persistent workgroup walks 16 x 16 pixel tiles with the dy tile [256 px][64]
// and the 18 x 18 halo of 16-B x rows in LDS (each dy and x element read from HBM about once --
// the generic kernel gathers x per tap); both MFMA operands are gathered from them (k = pixel).
// Wave w owns tile rows 4w..4w+3 (64 pixels of the K sum) x all 64 dy channels x the 72 columns
// (4 x 5 blocks of 16; the last block's upper half duplicates tap 8 and is dropped) -- splitting K
// instead of the channels keeps the x reads unshared.  Both operands come out of their row-major
// LDS images already K-major through ds_read_b64_tr_b16 (a 16-lane group reads 4 pixel rows x 16
// columns and lane i receives column i), two reads per 8-pixel fragment: 18 LDS reads per 32
// pixels where per-element gathers take 72.  The 4 wave partials are added through LDS at the end
// and every workgroup writes its fp32 slab [64][72] (split = blockIdx.x), stf_wgrad_reduce folds
// them.
constexpr int WC8_T = 16, WC8_HW = WC8_T + 2, WC8_HR = WC8_HW * WC8_HW;
// halo row stride 22 pixels: the taps 2 and 3 (read by one transposed read) then sit 20 rows =
// 4 (mod 8) bank slots apart, conflict-free with the neighbouring 8-pixel group
constexpr int WC8_HL = 22, WC8_HBYTES = WC8_HW * WC8_HL * 16;
constexpr int WC8_STAGE = WC8_HBYTES + 256 * 64 * 2;     // bytes: halo rows + dy tile
// dy tile: 32-B slot h of pixel p stored at slot h ^ wc8_swz(p), so that the 8 pixel rows one
// 32-lane half of a transposed read touches (p0 + 0..3, p0 + 8..11) cover all 64 banks once
__device__ __forceinline__ int wc8_swz(int p) { return ((p >> 1) & 1) | (((p >> 3) & 1) << 1); }
typedef short wc8_s4 __attribute__((ext_vector_type(4)));
typedef short wc8_s8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ e16x8 wc8_tr(const uint8_t* p, int second) {
  typedef __attribute__((address_space(3))) wc8_s4* lp;
  const wc8_s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(p));
  const wc8_s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(p + second));
  return __builtin_bit_cast(e16x8, (wc8_s8)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}
__global__ __launch_bounds__(NT, 2) void wgrad3x3_c8_kernel(WArgs a, int tiles_y, int tiles_x, int ntiles) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[2 * WC8_STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fk = lane >> 4, q = fr >> 2, pq = fr & 3;
  const int t_begin = blockIdx.x * a.chunk, t_end = min(ntiles, t_begin + a.chunk);
  const int per_img = tiles_y * tiles_x;
  const int cnt = t_end - t_begin;
  // transposed-read addresses (bytes from the stage base).  Lane 4q+pq of a 16-lane group supplies
  // row q's columns 4pq..4pq+3.  A (dy): rows = pixels p0+q, columns = channels nb*16 + 4pq.
  // B (x): rows = pixels p0+q shifted by a tap, columns = (tap pair of block kb)[pq>>1], channels
  // 4*(pq&1)..+3; block 4's second tap duplicates tap 8 (its columns are dropped).
  int aoff[2][4], boff[2][5];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const int p0 = wave * 64 + ks * 32 + fk * 8, px = p0 + q;
    const int hb = (p0 >> 4) * WC8_HL + (p0 & 15) + q;
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
      aoff[ks][nb] = WC8_HBYTES + px * 128 + (((nb ^ wc8_swz(px)) * 2 + (pq >> 1)) << 4) + (pq & 1) * 8;
#pragma unroll
    for (int kb = 0; kb < 5; ++kb) {
      const int t = kb == 4 ? 8 : 2 * kb + (pq >> 1);
      boff[ks][kb] = (hb + (t / 3) * WC8_HL + t % 3) * 16 + (pq & 1) * 8;
    }
  }
  uint4 hv[2], dv[8];
  auto load = [&](int t) {
    const int img = t / per_img, rem = t - img * per_img, ty = rem / tiles_x, tx = rem - ty * tiles_x;
#pragma unroll
    for (int q2 = 0; q2 < 2; ++q2) {
      const int hr = tid + q2 * 256, hy = hr / WC8_HW, hx = hr - hy * WC8_HW;
      const int ys = ty * WC8_T - 1 + hy, xs = tx * WC8_T - 1 + hx;
      hv[q2] = make_uint4(0, 0, 0, 0);
      if (hr < WC8_HR && ys >= 0 && xs >= 0 && ys < a.Hs && xs < a.Ws)
        hv[q2] = *reinterpret_cast<const uint4*>(a.x + ((size_t)(img * a.Hs + ys) * a.Ws + xs) * a.xcs);
    }
#pragma unroll
    for (int q2 = 0; q2 < 8; ++q2) {
      const int e = tid + q2 * 256, p = e >> 3, c8 = e & 7;
      const int oy = ty * WC8_T + (p >> 4), ox = tx * WC8_T + (p & 15);
      dv[q2] = make_uint4(0, 0, 0, 0);
      if (oy < a.Hd && ox < a.Wd)
        dv[q2] = *reinterpret_cast<const uint4*>(a.dy + ((size_t)(img * a.Hd + oy) * a.Wd + ox) * a.dycs + c8 * 8);
    }
  };
  auto store = [&](int buf) {
    uint4* h = reinterpret_cast<uint4*>(lds + buf * WC8_STAGE);
    uint4* d = reinterpret_cast<uint4*>(lds + buf * WC8_STAGE + WC8_HBYTES);
#pragma unroll
    for (int q2 = 0; q2 < 2; ++q2) {
      const int hr = tid + q2 * 256, hy = hr / WC8_HW;
      if (hr < WC8_HR) h[hy * WC8_HL + hr - hy * WC8_HW] = hv[q2];
    }
#pragma unroll
    for (int q2 = 0; q2 < 8; ++q2) {
      const int e = tid + q2 * 256, p = e >> 3, c8 = e & 7;
      d[p * 8 + ((((c8 >> 1) ^ wc8_swz(p)) << 1) | (c8 & 1))] = dv[q2];
    }
  };
  f32x4 acc[4][5];
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
#pragma unroll
    for (int kb = 0; kb < 5; ++kb) acc[nb][kb] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (cnt > 0) { load(t_begin); store(0); }
  __syncthreads();
  for (int kk = 0; kk < cnt; ++kk) {
    const int buf = kk & 1;
    if (kk + 1 < cnt) load(t_begin + kk + 1);
    const uint8_t* st = lds + buf * WC8_STAGE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      // k-slots fk*8 + 0..7 = pixels p0 + 0..7 (p0 = wave*64 + ks*32 + fk*8) in both operands
      e16x8 bq[5];
#pragma unroll
      for (int kb = 0; kb < 5; ++kb) bq[kb] = wc8_tr(st + boff[ks][kb], 4 * 16);
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const e16x8 av = wc8_tr(st + aoff[ks][nb], 4 * 128);
#pragma unroll
        for (int kb = 0; kb < 5; ++kb) acc[nb][kb] = mfma16x16x32(av, bq[kb], acc[nb][kb]);
      }
    }
    if (kk + 1 < cnt) store(buf ^ 1);
    __syncthreads();
  }
  // lane (fr, fk), element r: dy channel nb*16 + 4*fk + r; column fr of block kb = tap
  // (kb < 4 ? 2*kb + (fr >> 3) : 8), channel fr & 7 -> slab column tap*8 + channel (tap-major, as
  // the other fused kernels' slabs); the 4 wave partials [64][72] meet in LDS
  float* red = reinterpret_cast<float*>(lds);                  // [4][64][72] = 73.7 KB
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
#pragma unroll
    for (int kb = 0; kb < 5; ++kb)
      if (kb < 4 || fr < 8)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[(wave * 64 + nb * 16 + 4 * fk + r) * 72 + kb * 16 + fr] = acc[nb][kb][r];
  __syncthreads();
  float* slab = a.ws + (size_t)blockIdx.x * 64 * 72;
  for (int i = tid; i < 64 * 72; i += NT)
    slab[i] = (red[i] + red[64 * 72 + i]) + (red[2 * 64 * 72 + i] + red[3 * 64 * 72 + i]);
}


// ---------------------------------------------------------------------------
// ConvTranspose2d(k=2, s=2) weight gradient: one block per (64 dy-channel,
// 64 x-channel) tile covers all four taps.
//   dW[n][tap][c] = sum_p dy[p][n] * x[(2py + r, 2px + s)][c],  p over the small grid
// The taps read disjoint sub-pixels of x, staged as four sub-images of the pixel
// tile (LDS row = tap * 64 + p), so both operands cross HBM once (the per-tap
// kernel reads dy four times) and each tap's transposed reads hit consecutive
// rows.  Single LDS buffer (51 KB) -> 3 blocks per CU; the next tile's global
// loads are in flight (registers) during the MFMAs of the current one.
// NB = 2: a block covers 128 dy channels (two 64-channel LDS sub-tiles, 61 KB, 2 blocks
// per CU), so the 2x larger x tensor crosses HBM once per 128 dy channels, not per 64.
template <int PW, int NB>
__global__ __launch_bounds__(NT, NB == 1 ? 3 : 2) void wgrad2x2s2_kernel(WArgs a, int tiles_y, int tiles_x,
                                                                          int ntiles) {
  constexpr int PH = 64 / PW, SR = 64 + 16;
  constexpr int A_EL = NB * 64 * SR, B_EL = 4 * 64 * SR;
  constexpr int CHA = NB * 64 * 8 / NT, CHB = 4 * 64 * 8 / NT;
  __shared__ __attribute__((aligned(16))) uint16_t smem[A_EL + B_EL];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int TMW = 4 * NB;                   // all 64 NB dy channels per wave, 16 x channels (wave)
  const int split = blockIdx.x;
  const int n0 = blockIdx.y * 64 * NB, c0 = blockIdx.z * 64;
  const int t_begin = split * a.chunk, t_end = min(ntiles, t_begin + a.chunk);
  const int per_img = tiles_y * tiles_x;

  uint4 ra[CHA], rb[CHB];
  auto load = [&](int t) {
    const int img = t / per_img, rem = t - img * per_img;
    const int ty = rem / tiles_x, tx = rem - ty * tiles_x;
    const int y0 = ty * PH, x0 = tx * PW;
#pragma unroll
    for (int i = 0; i < CHA; ++i) {
      const int e = tid + i * NT, sub = e >> 9, px = (e >> 3) & 63, ch = e & 7;   // sub-tile, pixel, chunk
      const int yd = y0 + px / PW, xd = x0 + px % PW;
      ra[i] = make_uint4(0, 0, 0, 0);
      if (yd < a.Hd && xd < a.Wd)
        ra[i] = *reinterpret_cast<const uint4*>(a.dy + (size_t)((img * a.Hd + yd) * a.Wd + xd) * a.dycs + n0 +
                                                sub * 64 + ch * 8);
    }
#pragma unroll
    for (int i = 0; i < CHB; ++i) {
      const int e = tid + i * NT, row = e >> 3, ch = e & 7;
      const int tap = row >> 6, p = row & 63;
      const int yd = y0 + p / PW, xd = x0 + p % PW;
      const int ys = 2 * yd + (tap >> 1), xs = 2 * xd + (tap & 1);
      rb[i] = make_uint4(0, 0, 0, 0);
      if (yd < a.Hd && xd < a.Wd)
        rb[i] = *reinterpret_cast<const uint4*>(a.x + (size_t)((img * a.Hs + ys) * a.Ws + xs) * a.xcs + c0 + ch * 8);
    }
  };
  auto store = [&]() {
    uint16_t* sa = smem;
    uint16_t* sb = smem + A_EL;
#pragma unroll
    for (int i = 0; i < CHA; ++i) {
      const int e = tid + i * NT;                   // sub-tile e >> 9 starts at row 64 (e >> 9)
      *reinterpret_cast<uint4*>(sa + (e >> 3) * SR + (e & 7) * 8) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < CHB; ++i) {
      const int e = tid + i * NT;
      *reinterpret_cast<uint4*>(sb + (e >> 3) * SR + (e & 7) * 8) = rb[i];
    }
  };

  f32x4 acc[4][TMW];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int i = 0; i < TMW; ++i) acc[t][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transposed-read lane geometry and pixel permutation as in wgrad3x3_kernel
  const int g = lane >> 4, q = (lane >> 2) & 3, p4 = (lane & 3) * 4;
  const int pl = 16 * (g >> 1) + 4 * (g & 1) + q;
  int prow[2][2];
#pragma unroll
  for (int k2 = 0; k2 < 2; ++k2)
#pragma unroll
    for (int h = 0; h < 2; ++h) prow[k2][h] = (32 * k2 + 8 * h + pl) * SR;

  const int steps = t_end - t_begin;
  if (steps > 0) { load(t_begin); store(); }
  __syncthreads();
  for (int it = 0; it < steps; ++it) {
    if (it + 1 < steps) load(t_begin + it + 1);
    const uint16_t* sa = smem;
    const uint16_t* sb = smem + A_EL;
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) {
      e16x8 af[TMW];
#pragma unroll
      for (int i = 0; i < TMW; ++i) {
        const int col = (i >> 2) * 64 * SR + (i & 3) * 16 + p4;
        v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(sa + prow[k2][0] + col));
        v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(sa + prow[k2][1] + col));
        short s8[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[i] = __builtin_bit_cast(e16x8, s8);
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int col = wave * 16 + p4;
        const int toff = t * 64 * SR;
        v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(sb + toff + prow[k2][0] + col));
        v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(sb + toff + prow[k2][1] + col));
        short s8[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        const e16x8 bfr = __builtin_bit_cast(e16x8, s8);
#pragma unroll
        for (int i = 0; i < TMW; ++i)
          acc[t][i] = mfma16x16x32(af[i], bfr, acc[t][i]);
      }
    }
    if (it + 1 < steps) {
      __syncthreads();                          // every wave is done with this tile
      store();
      __syncthreads();
    }
  }

  const int RSC = 4 * a.Cs;
  float* out = a.ws + (size_t)split * a.Nout * RSC;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int i = 0; i < TMW; ++i) {
      const int k = t * a.Cs + c0 + wave * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + i * 16 + (lane >> 4) * 4 + r;
        out[(size_t)n * RSC + k] = acc[t][i][r];
      }
    }
}

// One launch, deterministic: a block owns 64 consecutive outputs; thread (r, c)
// (16 split-lanes r x 16 column threads c) sums slabs r, r+16, ... of outputs
// 4c..4c+3 with float4 loads (a wave reads 4 slabs x 256 contiguous bytes), the
// 16 lane totals are added in fixed order, and the result is written in the
// PyTorch [Nout][Cs][R][S] layout.  For plans with many splits (the high-resolution
// layers: 32-512 slabs of a small output).
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ ws, int splits, int Nout, int R,
                                                           int S, int Cs, float* __restrict__ out) {
  __shared__ double red[16][65];
  const int RSC = R * S * Cs;
  const long total = (long)Nout * RSC;                 // multiple of 8
  const int r = threadIdx.x >> 4, c = threadIdx.x & 15;
  const long e0 = blockIdx.x * 64L + c * 4;
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  if (e0 < total) {
    int k = r;
    for (; k + 16 < splits; k += 32) {                 // two slabs in flight
      const float4 u = *reinterpret_cast<const float4*>(ws + (long)k * total + e0);
      const float4 v = *reinterpret_cast<const float4*>(ws + (long)(k + 16) * total + e0);
      acc[0] += (double)u.x + v.x; acc[1] += (double)u.y + v.y;
      acc[2] += (double)u.z + v.z; acc[3] += (double)u.w + v.w;
    }
    for (; k < splits; k += 16) {
      const float4 u = *reinterpret_cast<const float4*>(ws + (long)k * total + e0);
      acc[0] += u.x; acc[1] += u.y; acc[2] += u.z; acc[3] += u.w;
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) red[r][c * 4 + j] = acc[j];
  __syncthreads();
  if (threadIdx.x < 64) {
    const long idx = blockIdx.x * 64L + threadIdx.x;
    if (idx < total) {
      double t = 0.0;
#pragma unroll
      for (int q = 0; q < 16; ++q) t += red[q][threadIdx.x];
      const int n = (int)(idx / RSC), rem = (int)(idx - (long)n * RSC);
      const int tap = rem / Cs, ch = rem - tap * Cs;
      out[((long)n * Cs + ch) * (R * S) + tap] = (float)t;
    }
  }
}

// Few-split plans (<= 8 slabs: the deep layers, whose slabs are a large output -- up to
// 1024 x 1024 x 9 -- rather than many partials of a small one; the transposed store above would
// scatter 4-B writes 36 B apart over tens of MB, 0.9-3.2 TB/s measured): a thread owns 4
// consecutive (n, c) columns of ONE tap and sums its float4 over every slab (fixed order,
// fp64, four slabs in flight); thread index = column-group * RS + tap, so a wave's scalar
// stores out[(col + j) * RS + tap] fill a contiguous run of the [Nout][Cs][R][S] output
// (tools/bench_wreduce.py: 2 x 1024 x 1024 x 9 slabs 82 -> 22 us, 4 x 1024 x 512 43 -> 18 us,
// 8 x 512 x 512 23 -> 17 us; from 14 slabs up the kernel above is faster).
template <int RS>
__global__ __launch_bounds__(256) void wgrad_reduce_tap_kernel(const float* __restrict__ ws, int splits, int Nout,
                                                               int Cs, float* __restrict__ out) {
  const long cols = (long)Nout * Cs;
  const long u = blockIdx.x * 256L + threadIdx.x;
  const long cg = u / RS;
  const int tap = (int)(u - cg * RS);
  const long col = cg * 4;
  if (col >= cols) return;
  const long total = cols * RS;
  const int n = (int)(col / Cs), ch = (int)(col - (long)n * Cs);
  const float* p = ws + (long)n * RS * Cs + tap * Cs + ch;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  int k = 0;
  for (; k + 3 < splits; k += 4) {
    const float4 u0 = *reinterpret_cast<const float4*>(p + (long)k * total);
    const float4 u1 = *reinterpret_cast<const float4*>(p + (long)(k + 1) * total);
    const float4 u2 = *reinterpret_cast<const float4*>(p + (long)(k + 2) * total);
    const float4 u3 = *reinterpret_cast<const float4*>(p + (long)(k + 3) * total);
    a0 += ((double)u0.x + u1.x) + ((double)u2.x + u3.x);
    a1 += ((double)u0.y + u1.y) + ((double)u2.y + u3.y);
    a2 += ((double)u0.z + u1.z) + ((double)u2.z + u3.z);
    a3 += ((double)u0.w + u1.w) + ((double)u2.w + u3.w);
  }
  for (; k < splits; ++k) {
    const float4 v = *reinterpret_cast<const float4*>(p + (long)k * total);
    a0 += v.x; a1 += v.y; a2 += v.z; a3 += v.w;
  }
  float* o = out + col * RS + tap;
  o[0] = (float)a0; o[RS] = (float)a1; o[2 * RS] = (float)a2; o[3 * RS] = (float)a3;
}

bool big_tile(const stf_wgrad_args* a) { return a->Nout % 128 == 0 && a->g.Cs % 128 == 0; }

// fused-tap kernel: 3x3, stride 1, pad 1, 64-multiples of channels, W >= 8
int fused_pw(const stf_wgrad_args* a) {
  static const bool enabled = stf::ab_switch("STF_WGRAD_FUSED", 1) != 0;
  const stf_conv_geom& c = a->g;
  if (!enabled) return 0;
  if (c.R != 3 || c.S != 3 || c.stride != 1 || c.pad != 1 || c.Hd != c.Hs || c.Wd != c.Ws) return 0;
  if (a->Nout % 64 || c.Cs % 64 || c.Wd < 8) return 0;
  return c.Wd >= 16 ? 16 : 8;
}

// ConvT 2x2 / stride 2 fused-tap kernel (x = the 2x larger gradient tensor)
int fused22_pw(const stf_wgrad_args* a) {
  static const bool enabled = stf::ab_switch("STF_WGRAD_FUSED", 1) != 0;
  const stf_conv_geom& c = a->g;
  if (!enabled || c.R != 2 || c.S != 2 || c.stride != 2 || c.pad != 0 || c.transposed) return 0;
  if (c.Hs != 2 * c.Hd || c.Ws != 2 * c.Wd || a->Nout % 64 || c.Cs % 64 || c.Wd < 8) return 0;
  return c.Wd >= 16 ? 16 : 8;
}

// dy channels per ConvT 2x2 block, in 64s: 2 from 256 dy channels up (measured, tools/ab_convt.sh,
// batch 64: up16/32/64 132/127/134 -> 104/99/107 us; at 128 channels the two 64-channel blocks
// of a pixel tile meet in L2 anyway and the 3-per-CU occupancy wins, 150 vs 172 us).
// STF_WGRAD22_NB=1: always 1 (A/B)
int fused22_nb(const stf_wgrad_args* a) {
  return (a->Nout % 128 == 0 && a->Nout >= 256) ? 2 : 1;
}

// the 8-channel-input 3x3 layer (conv3x3_c8_kernel's weight gradient; STF_WGRAD_C8=0: the
// generic wgrad_kernel<64, 96, 64, true>, A/B)
bool fused_c8(const stf_wgrad_args* a) {
  static const bool enabled = stf::ab_switch("STF_WGRAD_C8", 1) != 0;
  const stf_conv_geom& c = a->g;
  return enabled && c.R == 3 && c.S == 3 && c.stride == 1 && c.pad == 1 && c.Hd == c.Hs && c.Wd == c.Ws &&
         c.Cs == 8 && c.src_cstride == 8 && a->Nout == 64 && !c.transposed;
}

void c8_tiles(const stf_wgrad_args* a, int& ty, int& tx, int& nt) {
  ty = (a->g.Hd + WC8_T - 1) / WC8_T;
  tx = (a->g.Wd + WC8_T - 1) / WC8_T;
  nt = a->g.N * ty * tx;
}

void fused_tiles(const stf_wgrad_args* a, int pw, int& ty, int& tx, int& nt) {
  ty = (a->g.Hd + 64 / pw - 1) / (64 / pw);
  tx = (a->g.Wd + pw - 1) / pw;
  nt = a->g.N * ty * tx;
}

void plan(const stf_wgrad_args* a, int& splits, int& chunk) {
  if (fused_c8(a)) {                                 // persistent: two workgroups per CU
    int ty, tx, nt;
    c8_tiles(a, ty, tx, nt);
    const long want = std::min<long>(nt, a->grid_blocks > 0 ? a->grid_blocks : 512);
    chunk = (int)((nt + want - 1) / want);
    splits = (nt + chunk - 1) / chunk;
    return;
  }
  if (const int pw = fused_pw(a) ? fused_pw(a) : fused22_pw(a)) {
    int ty, tx, nt;
    fused_tiles(a, pw, ty, tx, nt);
    const long tiles = (long)(a->Nout / (fused_pw(a) ? 64 : 64 * fused22_nb(a))) * (a->g.Cs / 64);
    const long target = a->grid_blocks > 0 ? a->grid_blocks : 512;
    long want = (target + tiles - 1) / tiles;
    const long maxs = (nt + 3) / 4;                  // at least 4 pixel tiles per split
    if (want > maxs) want = maxs;
    if (want < 1) want = 1;
    chunk = (int)((nt + want - 1) / want);
    splits = (nt + chunk - 1) / chunk;
    return;
  }
  const int M = a->g.N * a->g.Hd * a->g.Wd;
  const int bm = big_tile(a) ? 128 : 64, bkp = big_tile(a) ? 32 : 64;
  const long rsc = (long)a->g.R * a->g.S * a->g.Cs;
  const long cblocks = (a->g.Cs % 64 && rsc > 64 && rsc <= 96) ? 1 : (rsc + bm - 1) / bm;
  const long tiles = (long)((a->Nout + bm - 1) / bm) * cblocks;
  // K splits until ~target workgroups: every split writes a [Nout][R*S*Cs] fp32 slab that the reduce
  // reads back, so the 128 x 128 tile (1x1 weight gradients of the STF LSTMs and downsamples: up to
  // 1024 splits of 134 MB slabs at 2048) aims at two workgroups per CU (STF cfg3 +2.6 % over 2048,
  // same box); the 64-wide tiles keep 2048 (UNet's first layer: 512 measured -0.5..-0.8 %)
  const long target = big_tile(a) ? 512 : 2048;
  long want = (target + tiles - 1) / tiles;
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

extern "C" const char* stf_wgrad_kernel_name(const stf_wgrad_args* a) {
  if (fused_c8(a)) return "wgrad3x3_c8_kernel";
  if (const int pw = fused_pw(a)) {
    return pw == 16 ? "wgrad3x3_kernel<16, 0>" : "wgrad3x3_kernel<8, 0>";
  }
  if (const int pw = fused22_pw(a)) {
    if (fused22_nb(a) == 2) return pw == 16 ? "wgrad2x2s2_kernel<16, 2>" : "wgrad2x2s2_kernel<8, 2>";
    return pw == 16 ? "wgrad2x2s2_kernel<16, 1>" : "wgrad2x2s2_kernel<8, 1>";
  }
  if (big_tile(a)) return "wgrad_kernel<128, 128, 32, false>";
  const int rsc = a->g.R * a->g.S * a->g.Cs;
  if (a->g.Cs % 64 == 0) return "wgrad_kernel<64, 64, 64, false>";
  return (rsc > 64 && rsc <= 96) ? "wgrad_kernel<64, 96, 64, true>" : "wgrad_kernel<64, 64, 64, true>";
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
  w.colmajor = 1;
  // timing-only ablation: the split-K slabs of the fused 3x3 kernel all land in slab 0 (L2-resident:
  // no slab traffic to HBM; the sums are wrong) -- the upper bound of folding the slabs in-kernel
  static const int one_slab = stf::ablation_env("STF_WGRAD_ONE_SLAB") == 1;
  w.one_slab = one_slab;
  hipStream_t s = (hipStream_t)stream;
  const int rsc = c.R * c.S * c.Cs;
  if (fused_c8(a)) {
    int ty, tx, nt;
    c8_tiles(a, ty, tx, nt);
    hipLaunchKernelGGL(wgrad3x3_c8_kernel, dim3(splits), dim3(NT), 0, s, w, ty, tx, nt);
    STF_CHECK_LAUNCH();
    return 0;
  }
  if (const int pw = fused_pw(a)) {
    int ty, tx, nt;
    fused_tiles(a, pw, ty, tx, nt);
    dim3 grid(splits, a->Nout / 64, c.Cs / 64);
    static const int diag = stf::ablation_env("STF_WGRAD_DIAG");
    if (pw == 16 && diag == 1)
      hipLaunchKernelGGL((wgrad3x3_kernel<16, 1>), grid, dim3(NT), 0, s, w, ty, tx, nt);
    else if (pw == 16 && diag == 2)
      hipLaunchKernelGGL((wgrad3x3_kernel<16, 2>), grid, dim3(NT), 0, s, w, ty, tx, nt);
    else if (pw == 16 && diag == 4)
      hipLaunchKernelGGL((wgrad3x3_kernel<16, 4>), grid, dim3(NT), 0, s, w, ty, tx, nt);
    else if (pw == 16)
      hipLaunchKernelGGL((wgrad3x3_kernel<16>), grid, dim3(NT), 0, s, w, ty, tx, nt);
    else
      hipLaunchKernelGGL((wgrad3x3_kernel<8>), grid, dim3(NT), 0, s, w, ty, tx, nt);
  } else if (const int pw22 = fused22_pw(a)) {
    int ty, tx, nt;
    fused_tiles(a, pw22, ty, tx, nt);
    const int nb = fused22_nb(a);
    dim3 grid(splits, a->Nout / (64 * nb), c.Cs / 64);
    if (nb == 2 && pw22 == 16) hipLaunchKernelGGL((wgrad2x2s2_kernel<16, 2>), grid, dim3(NT), 0, s, w, ty, tx, nt);
    else if (nb == 2) hipLaunchKernelGGL((wgrad2x2s2_kernel<8, 2>), grid, dim3(NT), 0, s, w, ty, tx, nt);
    else if (pw22 == 16) hipLaunchKernelGGL((wgrad2x2s2_kernel<16, 1>), grid, dim3(NT), 0, s, w, ty, tx, nt);
    else hipLaunchKernelGGL((wgrad2x2s2_kernel<8, 1>), grid, dim3(NT), 0, s, w, ty, tx, nt);
  } else if (big_tile(a)) {
    dim3 grid(splits, a->Nout / 128, rsc / 128);
    hipLaunchKernelGGL((wgrad_kernel<128, 128, 32, false>), grid, dim3(NT), 0, s, w);
  } else if (c.Cs % 64 == 0) {
    dim3 grid(splits, (a->Nout + 63) / 64, rsc / 64);
    hipLaunchKernelGGL((wgrad_kernel<64, 64, 64, false>), grid, dim3(NT), 0, s, w);
  } else if (rsc > 64 && rsc <= 96) {
    // 8-channel network input, 3x3 (72 columns): one 96-column block reads dy once
    // (two 64-column blocks would read the 64-channel dy twice)
    dim3 grid(splits, (a->Nout + 63) / 64, 1);
    hipLaunchKernelGGL((wgrad_kernel<64, 96, 64, true>), grid, dim3(NT), 0, s, w);
  } else {
    dim3 grid(splits, (a->Nout + 63) / 64, (rsc + 63) / 64);
    hipLaunchKernelGGL((wgrad_kernel<64, 64, 64, true>), grid, dim3(NT), 0, s, w);
  }
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_wgrad_reduce(float* ws, int splits, int Nout, int R, int S, int Cs, float* out,
                                stf_stream_t stream) {
  const long total = (long)Nout * R * S * Cs;
  if (total % 8 || ((uintptr_t)ws & 15)) return STF_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const int rs = R * S;
  const bool shape_ok = (rs == 9 || rs == 4 || rs == 1) && ((long)Nout * Cs) % 4 == 0;
  if (shape_ok && splits <= 8) {
    const unsigned blocks = (unsigned)(((long)Nout * Cs / 4 * rs + 255) / 256);
    if (rs == 9) hipLaunchKernelGGL(wgrad_reduce_tap_kernel<9>, dim3(blocks), dim3(256), 0, s, ws, splits, Nout, Cs, out);
    else if (rs == 4) hipLaunchKernelGGL(wgrad_reduce_tap_kernel<4>, dim3(blocks), dim3(256), 0, s, ws, splits, Nout, Cs, out);
    else hipLaunchKernelGGL(wgrad_reduce_tap_kernel<1>, dim3(blocks), dim3(256), 0, s, ws, splits, Nout, Cs, out);
  } else {
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((total + 63) / 64)), dim3(256), 0, s, ws, splits, Nout, R,
                       S, Cs, out);
  }
  STF_CHECK_LAUNCH();
  return 0;
}
