// Shared device helpers for the STF-Unet gfx950 kernels.
// Activations are NHWC bf16 (channel-contiguous, 16-B aligned channel groups);
// statistics, master weights and gradients are fp32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define STF_DEV __device__ __forceinline__

// ---------------------------------------------------------------- conversions
STF_DEV float bf2f(bf16 v) { return (float)v; }
STF_DEV bf16 f2bf(float v) { return (bf16)v; }   // v_cvt_pk_bf16_f32: RNE, NaN-preserving

STF_DEV void unpack8(const uint4& u, float (&f)[8]) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

STF_DEV uint32_t pack2(float a, float b) {
  bf16 x = f2bf(a), y = f2bf(b);
  return (uint32_t)__builtin_bit_cast(uint16_t, x) | ((uint32_t)__builtin_bit_cast(uint16_t, y) << 16);
}

STF_DEV uint4 pack8(const float (&f)[8]) {
  return make_uint4(pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7]));
}

STF_DEV float round_bf(float v) { return bf2f(f2bf(v)); }

// ---------------------------------------------------------------- reductions
STF_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

STF_DEV double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---------------------------------------------------------------- error plumbing
#define STF_CHECK_LAUNCH() do { hipError_t e__ = hipGetLastError(); if (e__ != hipSuccess) return (int)e__; } while (0)

// Argument-validation failures are reported as this code (outside hipError_t's range).
#define STF_EINVAL 100001
