// Deterministic column reductions over per-tile partial slabs [T][W] (fp32).
//
// Stage 1 (in place): block (x, s) sums rows s, s+S, s+2S, ... of columns
// [256x, 256x+256) in fp64 and writes the result back into row s -- only the
// thread that owns (s, j) ever touches element (s, j), so no extra workspace is
// needed and the summation order is fixed.  Consumers then fold the first S
// rows.  With S ~ T/128 every stage-1 thread sums ~128 independent,
// coalesced loads instead of one thread walking all T tiles.
#pragma once
#include "common.h"

namespace stf {

static __global__ void colsum_inplace_kernel(float* __restrict__ buf, long T, long W, int S) {
  const long j = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const int s = blockIdx.y;
  if (j >= W) return;
  double acc = 0.0;
  for (long t = s; t < T; t += S) acc += buf[t * W + j];
  buf[(long)s * W + j] = (float)acc;
}

static inline int colsum_split(long T, long W) {
  long s = T / 64;
  const long blocks_x = (W + 255) / 256;
  if (blocks_x * s < 512) s = T / 16;            // few columns: more parallel row groups
  if (s < 1) s = 1;
  if (s > 256) s = 256;
  if (s > T) s = (int)T;
  return (int)s;
}

// Returns S (rows left to fold) and launches stage 1 when it helps.
static inline int colsum_stage1(float* buf, long T, long W, hipStream_t st) {
  if (T <= 8) return (int)T;
  const int S = colsum_split(T, W);
  if (S >= T) return (int)T;
  hipLaunchKernelGGL(colsum_inplace_kernel, dim3((W + 255) / 256, S), dim3(256), 0, st, buf, T, W, S);
  return S;
}

}  // namespace stf
