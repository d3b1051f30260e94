// Deterministic column reductions over per-tile partial slabs [G][T][W] (fp32).
//
// Stage 1 (in place): block (x, s, g) sums rows s, s+S, s+2S, ... (< T) of group
// g, columns [256x, 256x+256), in fp64 and writes the result back into row s of
// that group -- only the thread that owns (g, s, j) ever touches element
// (g, s, j), so no workspace is needed and the summation order is fixed.
// Consumers then fold rows [g*T, g*T + S).  With S ~ T/64 every stage-1 thread
// sums ~64 independent, coalesced loads instead of one thread walking all T.
#pragma once
#include "common.h"

namespace stf {

static __global__ void colsum_inplace_kernel(float* __restrict__ buf, long T, long W, int S) {
  const long j = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const int s = blockIdx.y;
  if (j >= W) return;
  float* b = buf + (size_t)blockIdx.z * T * W;
  double acc = 0.0;
  for (long t = s; t < T; t += S) acc += b[t * W + j];
  b[(long)s * W + j] = (float)acc;
}

static inline int colsum_split(long T, long W, int G) {
  long s = T / 64;
  const long blocks_x = (W + 255) / 256;
  if (blocks_x * s * G < 512) s = T / 16;       // few columns: more parallel row groups
  if (s < 1) s = 1;
  if (s > 256) s = 256;
  if (s > T) s = (int)T;
  return (int)s;
}

// Fold each group's T rows to S rows in place; returns S (rows per group left,
// still at group stride T).
static inline int colsum_stage1(float* buf, long T, long W, hipStream_t st, int G = 1, long min_rows = 8) {
  if (T <= min_rows) return (int)T;
  const int S = colsum_split(T, W, G);
  if (S >= T) return (int)T;
  hipLaunchKernelGGL(colsum_inplace_kernel, dim3((W + 255) / 256, S, G), dim3(256), 0, st, buf, T, W, S);
  return S;
}

// Row folding inside one block: 16 columns x (blockDim / 16) row-lanes.  Column
// c = blockIdx.x * 16 + (tid & 15); lane r = tid >> 4 sums rows r, r+RL, ... < S
// (RL = blockDim / 16 row-lanes) of base[t * stride + c] (fp64); fold16_finish returns
// the total (fixed order) on lane 0 (threads 0..15).  The finalize kernels run 1024
// threads (64 row-lanes): their fold is a latency chain, ~4 dependent loads per lane
// instead of ~16 at 256 threads.  ``red`` holds blockDim doubles.
STF_DEV double fold16_partial(const float* base, int S, long stride, long c, bool cok) {
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;       // four chains: the loads pipeline
  if (cok) {
    const int RL = blockDim.x >> 4;
    int t = threadIdx.x >> 4;
    for (; t + 3 * RL < S; t += 4 * RL) {
      a0 += base[(long)t * stride + c];
      a1 += base[(long)(t + RL) * stride + c];
      a2 += base[(long)(t + 2 * RL) * stride + c];
      a3 += base[(long)(t + 3 * RL) * stride + c];
    }
    for (; t < S; t += RL) a0 += base[(long)t * stride + c];
  }
  return (a0 + a1) + (a2 + a3);
}

STF_DEV double fold16_finish(double v, double* red) {
  red[threadIdx.x] = v;
  __syncthreads();
  double tot = 0.0;
  const int RL = blockDim.x >> 4;
  if ((threadIdx.x >> 4) == 0)
    for (int r = 0; r < RL; ++r) tot += red[r * 16 + (threadIdx.x & 15)];
  __syncthreads();
  return tot;
}

// Both halves of a [rows][2][C] statistics slab at once (the BatchNorm finalize kernels: sum and
// sum of squares, or sum g and sum g*xhat): every lane issues the loads of both before adding,
// the four row-lanes a wave holds per column fold by shuffles, and the cross-wave fold is a
// 16-long chain per column instead of 64 (FOLD_NT / 16 row-lanes).  Fixed order: deterministic.
// Returns (on threads 0..15) the two totals; ``red`` holds 2 * (blockDim / 64) * 16 doubles.
STF_DEV void fold16_pair(const float* base, int S, long stride, long off2, long c, bool cok, double* red,
                         double& o1, double& o2) {
  double a0 = 0.0, a1 = 0.0, b0 = 0.0, b1 = 0.0;
  if (cok) {
    const int RL = blockDim.x >> 4;
    int t = threadIdx.x >> 4;
    for (; t + RL < S; t += 2 * RL) {
      const float x0 = base[(long)t * stride + c], y0 = base[(long)t * stride + off2 + c];
      const float x1 = base[(long)(t + RL) * stride + c], y1 = base[(long)(t + RL) * stride + off2 + c];
      a0 += x0; b0 += y0; a1 += x1; b1 += y1;
    }
    for (; t < S; t += RL) {
      a0 += base[(long)t * stride + c];
      b0 += base[(long)t * stride + off2 + c];
    }
  }
  double v1 = a0 + a1, v2 = b0 + b1;
  v1 += __shfl_xor(v1, 16, 64);
  v2 += __shfl_xor(v2, 16, 64);
  v1 += __shfl_xor(v1, 32, 64);
  v2 += __shfl_xor(v2, 32, 64);
  const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6, lane = threadIdx.x & 63;
  if (lane < 16) {
    red[wave * 16 + lane] = v1;
    red[(nw + wave) * 16 + lane] = v2;
  }
  __syncthreads();
  o1 = o2 = 0.0;
  if (threadIdx.x < 16)
    for (int w = 0; w < nw; ++w) {
      o1 += red[w * 16 + threadIdx.x];
      o2 += red[(nw + w) * 16 + threadIdx.x];
    }
}

constexpr int FOLD_NT = 1024;         // block size of the fold16 consumers (finalize kernels)

constexpr long FOLD16_ROWS = 1024;    // finalize kernels read up to this many rows directly

}  // namespace stf
