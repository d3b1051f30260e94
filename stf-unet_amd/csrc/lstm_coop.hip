// Whole-sequence nn.LSTM(C, C) for C = 128 / 256 / 512: one persistent launch per
// direction in which the workgroups of a pixel block share each time step
// (src/stf_lstm_unet.py:124-127,214-242; gate order i, f, g, o; only h_T is used).
//
// Why cooperative: at C >= 128 the [4C][2C] gate weights (256 KB - 4 MB in 16 bits) fit
// neither one workgroup's registers nor its LDS, and the per-step GEMM of the other path
// (one stf_igemm launch per step, M = pixels) is latency-bound at these sizes (~28 us per
// step for lstm4's 4.3 GFLOP at cfg3).  Here the 4C gate rows are cut into S = C/32 slices
// of 128 rows (32 hidden channels x 4 gates); workgroup (group, slice) keeps its slice of
// the weights in registers for the whole launch and, per 64-pixel block and time step,
// computes its 128 gate rows over the full [x_t | h_{t-1}] row (K = 2C), updates its 32
// cells (c in registers) and publishes h_t for its 32 channels.  The S workgroups of a
// pixel block hand h_t to each other through global memory inside the launch:
//   producer: h_t slice stored write-through (buffer store sc1), every wave
//             s_waitcnt vmcnt(0), barrier, one lane adds 1 to the (block, step) counter
//             (relaxed, agent scope);
//   consumer: one lane polls the counter of step t-1 until it reads S (relaxed, agent
//             scope, bounded spin), one agent-scope acquire (buffer_inv sc1), vmcnt(0),
//             barrier, then plain loads of the row
// (cdna_hip_programming.md section 6 Guideline 16).  The counters are zeroed by a
// hipMemsetAsync in front of every launch.  Progress needs only the S <= 16 workgroups of
// one group to be resident together (consecutive block ids; 1 workgroup per CU by LDS),
// so the launch drains even when other streams hold CUs; a spin that exceeds its bound
// (seconds) raises an error word instead of hanging.
//
// Numerics: the step GEMM is the per-step path's MFMA sequence (weights as the A operand,
// 16x16x32, K ascending, x then h, fp32 accumulation, bias added after), so c_t and h_t
// equal stf_igemm's LSTM epilogue bit for bit, and the per-step backward (which recomputes
// the gates with stf_igemm) sees exactly the forward's gates.
//
// Layout as stf_lstm_seq_fwd: lbuf rows of step t = [x_t | h_{t-1}] (2C channels, P pixels
// per step), h_t written into step t+1's h slot and h_{T-1} into hT; cst [T][P][C] fp32.
#include "common.h"
#include "../../include/stfunet.h"
#include <stdlib.h>

namespace {

constexpr int CNT = 256, CBM = 64, CR = 128;      // threads, pixels per block, gate rows per slice
constexpr unsigned SPIN_LIMIT = 1u << 25;          // ~4 s of s_sleep(2) polls (spin_limit = 0)

// consumer side of a hand-off (one lane): poll counter c until it reads S.  A poll count past
// `limit` sets the launch's error word and gives up; once the word is set anywhere in the
// launch every later wait gives up at once (a stalled launch drains in one timeout, not one
// per step and block).  The caller turns the word into a Python RuntimeError
// (stf_lstm_coop_error -> STFProgram.check_device_errors).
STF_DEV void coop_wait(unsigned* c, unsigned S, unsigned* err, unsigned limit) {
  if (limit == 0xFFFFFFFFu) {            // STF_COOP_FORCE_TIMEOUT: every hand-off "times out" (tests)
    __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  unsigned spins = 0;
  while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < S) {
    if ((spins & 255u) == 0 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
    __builtin_amdgcn_s_sleep(1);
    if (++spins > limit) { __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); break; }
  }
}

typedef __attribute__((address_space(1))) unsigned gu32;

// x / h tile row r (pixel, C channels), 16-B chunk q at q ^ (r & 7): conflict-free fragment reads
template <int C>
STF_DEV int so(int r, int q) { return r * C + ((q ^ (r & 7)) << 3); }

template <int C>
__global__ __launch_bounds__(CNT, 1) void lstm_coop_fwd_kernel(const uint16_t* __restrict__ wcat,
                                                               const float* __restrict__ bias, uint16_t* lbuf, int P,
                                                               int T, float* __restrict__ cst, uint16_t* hT, int hTcs,
                                                               float* __restrict__ gates, unsigned* cnt, unsigned* err,
                                                               unsigned limit) {
  constexpr int S = 4 * C / CR;            // slices (workgroups per pixel block)
  constexpr int KS = 2 * C / 32;           // k-steps: x (KS/2) then h (KS/2)
  constexpr int NF = 2;                    // 32 gate rows per wave
  constexpr int MF = CBM / 16;
  constexpr int NI = CBM * C * 2 / 1024;   // 1-KiB LDS-DMA instructions per x or h tile
  static_assert(C % 128 == 0 && NI % 4 == 0, "C");
  __shared__ __attribute__((aligned(16))) uint16_t xs[CBM * C];      // x_t rows
  __shared__ __attribute__((aligned(16))) uint16_t hin[CBM * C];     // h_{t-1} rows
  __shared__ __attribute__((aligned(16))) float cs[CBM * 32];        // c_t of this slice
  __shared__ __attribute__((aligned(16))) uint16_t hs[CBM * 32];     // h_t of this slice

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fk = lane >> 4;
  const int slice = blockIdx.x % S, group = blockIdx.x / S, groups = gridDim.x / S;
  const int npb = (P + CBM - 1) / CBM;
  const int lcs = 2 * C;
  const int row0 = slice * CR + wave * 32;              // this wave's first gate row
  const int ch0 = slice * 32;                           // this workgroup's first hidden channel

  e16x8 wf[NF][KS];
  float bv[NF][4];
#pragma unroll
  for (int nf = 0; nf < NF; ++nf) {
    const int n = row0 + nf * 16 + fr;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      wf[nf][ks] = *reinterpret_cast<const e16x8*>(wcat + (size_t)n * lcs + ks * 32 + fk * 8);
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[nf][r] = bias[row0 + nf * 16 + fk * 4 + r];
  }
  const uint32_t lbytes = (uint32_t)((size_t)T * P * lcs * 2);
  const __amdgpu_buffer_rsrc_t rs_l = __builtin_amdgcn_make_buffer_rsrc((void*)lbuf, 0, lbytes, 0x00020000);

  // the x (part 0) or h (part 1) half of the 64 rows of step t -> LDS by LDS-DMA (no registers,
  // every instruction in flight at once); rows past P and h_{-1} read as zeros
  auto dma = [&](uint16_t* dst, int t, int m0, int rows, int part) {
#pragma unroll
    for (int k = 0; k < NI / 4; ++k) {
      const int j = k * 4 + wave;
      const int pos = j * 1024 + lane * 16, r = pos / (2 * C), p = (pos - r * 2 * C) >> 4, q = p ^ (r & 7);
      const bool ok = r < rows && (part == 0 || t > 0);
      const uint32_t off = ok ? (uint32_t)((((size_t)t * P + m0 + r) * lcs + part * C + q * 8) * 2) : 0xFFFFFFF0u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_l, (__attribute__((address_space(3))) void*)(dst + j * 512), 16,
                                               off, 0, 0, 0);
    }
  };
  auto gemm = [&](const uint16_t* src, int k0, f32x4 (&acc)[MF][NF]) {
#pragma unroll
    for (int kk = 0; kk < KS / 2; ++kk) {
      e16x8 bf[MF];
#pragma unroll
      for (int mf = 0; mf < MF; ++mf) bf[mf] = *reinterpret_cast<const e16x8*>(&src[so<C>(mf * 16 + fr, kk * 4 + fk)]);
#pragma unroll
      for (int mf = 0; mf < MF; ++mf)
#pragma unroll
        for (int nf = 0; nf < NF; ++nf) acc[mf][nf] = mfma16x16x32(wf[nf][k0 + kk], bf[mf], acc[mf][nf]);
    }
  };

  for (int pb = group; pb < npb; pb += groups) {
    const int m0 = pb * CBM;
    const int rows = min(CBM, P - m0);
    float cc[MF][NF];
    f32x4 acc[MF][NF];
#pragma unroll
    for (int mf = 0; mf < MF; ++mf)
#pragma unroll
      for (int nf = 0; nf < NF; ++nf) { cc[mf][nf] = 0.f; acc[mf][nf] = f32x4{0.f, 0.f, 0.f, 0.f}; }
    dma(xs, 0, m0, rows, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    gemm(xs, 0, acc);                                     // x_0's half of step 0
    for (int t = 0; t < T; ++t) {
      if (t > 0) {
        // wait for the S slices of h_{t-1}, one agent-scope acquire, then its rows
        if (tid == 0) {
          coop_wait(&cnt[pb * T + t - 1], (unsigned)S, err, limit);
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        dma(hin, t, m0, rows, 1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        gemm(hin, KS / 2, acc);                           // h_{t-1}'s half (h_{-1} = 0: skipped)
      }
      // cell update: lane holds the 4 gates of local channel cl of pixel r
#pragma unroll
      for (int mf = 0; mf < MF; ++mf) {
        const int r = mf * 16 + fr;
#pragma unroll
        for (int nf = 0; nf < NF; ++nf) {
          const int cl = wave * 8 + nf * 4 + fk;
          float gi, gf, gg, go, c, hh;
          lstm_cell_fwd(acc[mf][nf][0] + bv[nf][0], acc[mf][nf][1] + bv[nf][1], acc[mf][nf][2] + bv[nf][2],
                        acc[mf][nf][3] + bv[nf][3], cc[mf][nf], gi, gf, gg, go, c, hh);
          cc[mf][nf] = c;
          reinterpret_cast<e16*>(hs)[r * 32 + cl] = f2e(hh);
          cs[r * 32 + cl] = c;
          acc[mf][nf] = f32x4{0.f, 0.f, 0.f, 0.f};
          if (gates && r < rows)            // activated gates for the cooperative backward
            *reinterpret_cast<float4*>(gates + ((size_t)t * P + m0 + r) * 4 * C + (ch0 + cl) * 4) =
                make_float4(gi, gf, gg, go);
        }
      }
      __syncthreads();
      // c_t (fp32, read by later launches) and h_t (write-through: read by the peers)
      for (int e = tid; e < rows * 8; e += CNT) {
        const int r = e >> 3, q = e & 7;
        *reinterpret_cast<float4*>(cst + ((size_t)t * P + m0 + r) * C + ch0 + q * 4) =
            *reinterpret_cast<const float4*>(&cs[r * 32 + q * 4]);
      }
      const bool last = t + 1 == T;
      for (int e = tid; e < rows * 4; e += CNT) {
        const int r = e >> 2, q = e & 3;
        const uint4 v = *reinterpret_cast<const uint4*>(&hs[r * 32 + q * 8]);
        if (last) {
          *reinterpret_cast<uint4*>(hT + (size_t)(m0 + r) * hTcs + ch0 + q * 8) = v;
        } else {
          const uint32_t off = (uint32_t)((((size_t)(t + 1) * P + m0 + r) * lcs + C + ch0 + q * 8) * 2);
          __builtin_amdgcn_raw_buffer_store_b128(u32x4v{v.x, v.y, v.z, v.w}, rs_l, off, 0, 16);
        }
      }
      if (!last) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_fetch_add(&cnt[pb * T + t], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // x_{t+1}'s half of step t+1 needs no hand-off: done while the peers finish step t
        dma(xs, t + 1, m0, rows, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        gemm(xs, 0, acc);
      } else {
        __syncthreads();             // hs / cs / xs are rewritten for the next pixel block
      }
    }
  }
}

// Backward through all T steps (t = T-1 .. 0), same workgroup grid.  Workgroup (group,
// slice s) owns hidden channels [32 s, 32 s + 32) for the cell backward (dc in registers,
// the forward's activated gates and c_t read back) and outputs [64 s, 64 s + 64) of
// [dx_t | dh_{t-1}] = dgates_t x W (K = 4C, its W^T rows in registers).  Two hand-offs
// per step inside the pixel block: dgates_t (every slice's 128 rows, write-through into
// dg, counter A) before the GEMM, and [dx_t | dh_{t-1}] (write-through into d2, counter
// B) before the next step's cell backward.  Same arithmetic as the per-step path (the
// cell backward of stf_igemm's LSTM epilogue on the same gates, then the dgates x W GEMM
// with K ascending), so equal to it bit for bit where that GEMM is not split over K.
template <int C>
__global__ __launch_bounds__(CNT, 1) void lstm_coop_bwd_kernel(const uint16_t* __restrict__ wcat_t,
                                                               const float* __restrict__ gates,
                                                               const float* __restrict__ cst, int P, int T,
                                                               const uint16_t* __restrict__ dhT, int dhcs,
                                                               uint16_t* dg, uint16_t* d2, int d2cs, unsigned* cnt,
                                                               unsigned* err, unsigned limit) {
  constexpr int S = 4 * C / CR;
  constexpr int K2 = 4 * C / 32;           // k-steps of the dgates x W GEMM
  constexpr int NF = 2, MF = CBM / 16;
  constexpr int PW = 4 * C < 1024 ? 4 * C : 1024;   // dgates columns staged per pass
  constexpr int NPASS = 4 * C / PW;
  constexpr int NI = CBM * PW * 2 / 1024;          // 1-KiB LDS-DMA instructions per pass
  static_assert(NI % 4 == 0, "C");
  __shared__ __attribute__((aligned(16))) uint16_t gl[CBM * PW];     // dgates rows (one pass)
  __shared__ __attribute__((aligned(16))) uint16_t go_[CBM * CR];    // this slice's dgates
  __shared__ __attribute__((aligned(16))) uint16_t ol[CBM * 64];     // this slice's [dx | dh] outputs

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fk = lane >> 4;
  const int slice = blockIdx.x % S, group = blockIdx.x / S, groups = gridDim.x / S;
  const int npb = (P + CBM - 1) / CBM;
  const int ch0 = slice * 32, o0 = slice * 64;
  unsigned* cntA = cnt;
  unsigned* cntB = cnt + (size_t)npb * T;

  e16x8 wt[K2];                            // W^T rows o0 + 16 wave + fr (A operand)
#pragma unroll
  for (int ks = 0; ks < K2; ++ks)
    wt[ks] = *reinterpret_cast<const e16x8*>(wcat_t + (size_t)(o0 + wave * 16 + fr) * 4 * C + ks * 32 + fk * 8);
  const uint32_t gbytes = (uint32_t)((size_t)T * P * 4 * C * 2);
  const __amdgpu_buffer_rsrc_t rs_g = __builtin_amdgcn_make_buffer_rsrc((void*)dg, 0, gbytes, 0x00020000);
  const uint32_t dbytes = (uint32_t)(((size_t)T * P - 1) * d2cs * 2 + 2 * C * 2);
  const __amdgpu_buffer_rsrc_t rs_d = __builtin_amdgcn_make_buffer_rsrc((void*)d2, 0, dbytes, 0x00020000);

  auto wait_for = [&](unsigned* c) {
    if (tid == 0) {
      coop_wait(c, (unsigned)S, err, limit);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
  };
  auto signal = [&](unsigned* c) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };

  for (int pb = group; pb < npb; pb += groups) {
    const int m0 = pb * CBM;
    const int rows = min(CBM, P - m0);
    float dc[MF][NF];
#pragma unroll
    for (int mf = 0; mf < MF; ++mf)
#pragma unroll
      for (int nf = 0; nf < NF; ++nf) dc[mf][nf] = 0.f;
    for (int t = T - 1; t >= 0; --t) {
      // the forward's gates and cell states of step t need no hand-off: all in flight before
      // the wait for dh_t (clamped addresses for rows past P: loaded, never used)
      float4 gt[MF][NF];
      float ct[MF][NF], c1[MF][NF];
#pragma unroll
      for (int mf = 0; mf < MF; ++mf) {
        const int r = min(mf * 16 + fr, rows - 1);
        const size_t m = (size_t)t * P + m0 + r;
#pragma unroll
        for (int nf = 0; nf < NF; ++nf) {
          const int ch = ch0 + wave * 8 + nf * 4 + fk;
          gt[mf][nf] = *reinterpret_cast<const float4*>(gates + m * 4 * C + ch * 4);
          ct[mf][nf] = cst[m * C + ch];
          c1[mf][nf] = t > 0 ? cst[(m - P) * C + ch] : 0.f;
        }
      }
      if (t < T - 1) wait_for(&cntB[pb * T + t + 1]);         // dh_t from step t+1's outputs
      float hv[MF][NF];
#pragma unroll
      for (int mf = 0; mf < MF; ++mf) {
        const int r = min(mf * 16 + fr, rows - 1);
        const size_t m = (size_t)t * P + m0 + r;
#pragma unroll
        for (int nf = 0; nf < NF; ++nf) {
          const int ch = ch0 + wave * 8 + nf * 4 + fk;
          hv[mf][nf] = t == T - 1 ? e2f(reinterpret_cast<const e16*>(dhT)[(size_t)(m0 + r) * dhcs + ch])
                                  : e2f(reinterpret_cast<const e16*>(d2)[(m + P) * d2cs + C + ch]);
        }
      }
      // 1. cell backward of this slice's 32 channels: lane = (pixel r, channel cl)
#pragma unroll
      for (int mf = 0; mf < MF; ++mf) {
        const int r = mf * 16 + fr;
#pragma unroll
        for (int nf = 0; nf < NF; ++nf) {
          const int cl = wave * 8 + nf * 4 + fk;
          float d_i, d_f, d_g, d_o, dcp;
          const float4 g4 = gt[mf][nf];
          lstm_cell_bwd(g4.x, g4.y, g4.z, g4.w, ct[mf][nf], c1[mf][nf], hv[mf][nf], dc[mf][nf], d_i, d_f, d_g, d_o,
                        dcp);
          dc[mf][nf] = dcp;
          *reinterpret_cast<uint2*>(&go_[r * CR + cl * 4]) = make_uint2(pack2(d_i, d_f), pack2(d_g, d_o));
        }
      }
      __syncthreads();
      // 2. this slice's dgates rows -> dg (write-through: the peers' GEMM reads them)
      for (int e = tid; e < rows * (CR / 8); e += CNT) {
        const int r = e / (CR / 8), q = e - r * (CR / 8);
        const uint4 v = *reinterpret_cast<const uint4*>(&go_[r * CR + q * 8]);
        const uint32_t off = (uint32_t)((((size_t)t * P + m0 + r) * 4 * C + slice * CR + q * 8) * 2);
        __builtin_amdgcn_raw_buffer_store_b128(u32x4v{v.x, v.y, v.z, v.w}, rs_g, off, 0, 16);
      }
      signal(&cntA[pb * T + t]);
      wait_for(&cntA[pb * T + t]);
      // 3. [dx_t | dh_{t-1}] outputs o0 .. o0+63 over all 4C dgates rows of the block
      f32x4 acc[MF];
#pragma unroll
      for (int mf = 0; mf < MF; ++mf) acc[mf] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ps = 0; ps < NPASS; ++ps) {
#pragma unroll
        for (int k = 0; k < NI / 4; ++k) {
          const int j = k * 4 + wave;
          const int pos = j * 1024 + lane * 16, r = pos / (2 * PW), p = (pos - r * 2 * PW) >> 4, q = p ^ (r & 7);
          const uint32_t off = r < rows ? (uint32_t)((((size_t)t * P + m0 + r) * 4 * C + ps * PW + q * 8) * 2)
                                        : 0xFFFFFFF0u;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rs_g, (__attribute__((address_space(3))) void*)(gl + j * 512), 16,
                                                   off, 0, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < PW / 32; ++kk) {
          e16x8 bf[MF];
#pragma unroll
          for (int mf = 0; mf < MF; ++mf) {
            const int r = mf * 16 + fr;
            bf[mf] = *reinterpret_cast<const e16x8*>(&gl[r * PW + (((kk * 4 + fk) ^ (r & 7)) << 3)]);
          }
#pragma unroll
          for (int mf = 0; mf < MF; ++mf) acc[mf] = mfma16x16x32(wt[ps * (PW / 32) + kk], bf[mf], acc[mf]);
        }
        __syncthreads();                 // gl is refilled by the next pass / step
      }
      // lane holds outputs o0 + 16 wave + 4 fk + (0..3) of pixel mf*16 + fr
#pragma unroll
      for (int mf = 0; mf < MF; ++mf) {
        const int r = mf * 16 + fr, oo = wave * 16 + fk * 4;
        *reinterpret_cast<uint2*>(&ol[r * 64 + oo]) =
            make_uint2(pack2(acc[mf][0], acc[mf][1]), pack2(acc[mf][2], acc[mf][3]));
      }
      __syncthreads();
      for (int e = tid; e < rows * 8; e += CNT) {
        const int r = e >> 3, q = e & 7;
        const uint4 v = *reinterpret_cast<const uint4*>(&ol[r * 64 + q * 8]);
        const uint32_t off = (uint32_t)((((size_t)t * P + m0 + r) * d2cs + o0 + q * 8) * 2);
        __builtin_amdgcn_raw_buffer_store_b128(u32x4v{v.x, v.y, v.z, v.w}, rs_d, off, 0, 16);
      }
      if (t > 0) signal(&cntB[pb * T + t]);
      else __syncthreads();
    }
  }
}

int num_cus() {
  static int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 0;
    return n;
  }();
  return cus;
}

template <int C>
int grid_of(int P, int max_wg) {
  constexpr int S = 4 * C / CR;
  const int npb = (P + CBM - 1) / CBM;
  const int budget = max_wg > 0 && max_wg < num_cus() ? max_wg : num_cus();
  int groups = budget / S;
  if (groups < 1) groups = 1;
  if (groups > npb) groups = npb;
  return groups * S;
}

template <int C>
int launch_fwd(const void* wcat, const float* bias, void* lbuf, int P, int T, float* c_out, void* h_last,
               int h_cstride, float* gates, unsigned* sync, int max_wg, unsigned limit, hipStream_t s) {
  if (num_cus() <= 0) return STF_EINVAL;
  const int npb = (P + CBM - 1) / CBM;
  const size_t words = 2 * (size_t)npb * T + 1;      // counters + the error word
  hipError_t e = stf::memset_async(sync, 0, ((words * 4 + 15) / 16) * 16, s);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL((lstm_coop_fwd_kernel<C>), dim3(grid_of<C>(P, max_wg)), dim3(CNT), 0, s, (const uint16_t*)wcat, bias,
                     (uint16_t*)lbuf, P, T, c_out, (uint16_t*)h_last, h_cstride, gates, sync,
                     sync + 2 * (size_t)npb * T, limit);
  STF_CHECK_LAUNCH();
  return 0;
}

template <int C>
int launch_bwd(const void* wcat_t, const float* gates, const float* c_all, int P, int T, const void* dh_last,
               int dh_cstride, void* dgates, void* dx, int dx_cstride, unsigned* sync, int max_wg, unsigned limit,
               hipStream_t s) {
  if (num_cus() <= 0) return STF_EINVAL;
  const int npb = (P + CBM - 1) / CBM;
  const size_t words = 2 * (size_t)npb * T + 1;
  hipError_t e = stf::memset_async(sync, 0, ((words * 4 + 15) / 16) * 16, s);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL((lstm_coop_bwd_kernel<C>), dim3(grid_of<C>(P, max_wg)), dim3(CNT), 0, s, (const uint16_t*)wcat_t, gates,
                     c_all, P, T, (const uint16_t*)dh_last, dh_cstride, (uint16_t*)dgates, (uint16_t*)dx, dx_cstride,
                     sync, sync + 2 * (size_t)npb * T, limit);
  STF_CHECK_LAUNCH();
  return 0;
}

}  // namespace

extern "C" size_t stf_lstm_coop_sync_bytes(int P, int T) {
  const size_t words = 2 * (size_t)((P + CBM - 1) / CBM) * T + 1;
  return ((words * 4 + 15) / 16) * 16;
}

extern "C" int stf_lstm_coop_supported(int C) { return C == 128 || C == 256 || C == 512; }

extern "C" int stf_lstm_coop_fwd(const void* wcat, const float* bias, void* lbuf, int P, int T, int C, float* c_out,
                                 void* h_last, int h_cstride, float* gates, unsigned* sync, int max_wg,
                                 unsigned spin_limit, stf_stream_t stream) {
  if (P <= 0 || T <= 0) return 0;
  if (!stf_lstm_coop_supported(C) || !wcat || !bias || !lbuf || !c_out || !h_last || !sync || h_cstride < C ||
      h_cstride % 8)
    return STF_EINVAL;
  if (((uintptr_t)wcat & 15) || ((uintptr_t)lbuf & 15) || ((uintptr_t)c_out & 15) || ((uintptr_t)h_last & 15) ||
      ((uintptr_t)sync & 15) || ((uintptr_t)gates & 15))
    return STF_EINVAL;
  if ((size_t)T * P * 2 * C * 2 >= 0xFFFFFF00ull) return STF_EINVAL;     // 32-bit buffer offsets
  hipStream_t s = (hipStream_t)stream;
  const unsigned lim = spin_limit ? spin_limit : SPIN_LIMIT;
  switch (C) {
    case 128: return launch_fwd<128>(wcat, bias, lbuf, P, T, c_out, h_last, h_cstride, gates, sync, max_wg, lim, s);
    case 256: return launch_fwd<256>(wcat, bias, lbuf, P, T, c_out, h_last, h_cstride, gates, sync, max_wg, lim, s);
    default: return launch_fwd<512>(wcat, bias, lbuf, P, T, c_out, h_last, h_cstride, gates, sync, max_wg, lim, s);
  }
}

extern "C" int stf_lstm_coop_bwd(const void* wcat_t, const float* gates, const float* c_all, int P, int T, int C,
                                 const void* dh_last, int dh_cstride, void* dgates, void* dx, int dx_cstride,
                                 unsigned* sync, int max_wg, unsigned spin_limit, stf_stream_t stream) {
  if (P <= 0 || T <= 0) return 0;
  if (!stf_lstm_coop_supported(C) || !wcat_t || !gates || !c_all || !dh_last || !dgates || !dx || !sync ||
      dh_cstride < C || dx_cstride < 2 * C || dx_cstride % 8)
    return STF_EINVAL;
  if (((uintptr_t)wcat_t & 15) || ((uintptr_t)gates & 15) || ((uintptr_t)dgates & 15) || ((uintptr_t)dx & 15) ||
      ((uintptr_t)sync & 15))
    return STF_EINVAL;
  if ((size_t)T * P * 4 * C * 2 >= 0xFFFFFF00ull || (size_t)T * P * dx_cstride * 2 >= 0xFFFFFF00ull)
    return STF_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const unsigned lim = spin_limit ? spin_limit : SPIN_LIMIT;
  switch (C) {
    case 128: return launch_bwd<128>(wcat_t, gates, c_all, P, T, dh_last, dh_cstride, dgates, dx, dx_cstride, sync, max_wg, lim, s);
    case 256: return launch_bwd<256>(wcat_t, gates, c_all, P, T, dh_last, dh_cstride, dgates, dx, dx_cstride, sync, max_wg, lim, s);
    default: return launch_bwd<512>(wcat_t, gates, c_all, P, T, dh_last, dh_cstride, dgates, dx, dx_cstride, sync, max_wg, lim, s);
  }
}

namespace {
__global__ void coop_error_or_kernel(const unsigned* __restrict__ word, unsigned* __restrict__ sticky) {
  if (threadIdx.x == 0 && *word) *sticky |= 1u;
}
}  // namespace

// sticky |= (the launch's error word), stream-ordered: a caller keeps one sticky word per program
// across steps and reads it back at a step boundary (no host sync on the step's path)
extern "C" int stf_lstm_coop_error(const unsigned* sync, int P, int T, unsigned* sticky, stf_stream_t stream) {
  if (!sync || !sticky || P <= 0 || T <= 0) return STF_EINVAL;
  const size_t npb = (size_t)(P + CBM - 1) / CBM;
  hipLaunchKernelGGL(coop_error_or_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, sync + 2 * npb * T, sticky);
  STF_CHECK_LAUNCH();
  return 0;
}
