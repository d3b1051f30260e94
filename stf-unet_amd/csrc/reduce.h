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
static inline int colsum_stage1(float* buf, long T, long W, hipStream_t st, int G = 1) {
  if (T <= 8) return (int)T;
  const int S = colsum_split(T, W, G);
  if (S >= T) return (int)T;
  hipLaunchKernelGGL(colsum_inplace_kernel, dim3((W + 255) / 256, S, G), dim3(256), 0, st, buf, T, W, S);
  return S;
}

}  // namespace stf
