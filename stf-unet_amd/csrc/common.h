// Shared device helpers for the STF-Unet gfx950 kernels.
// Activations are NHWC 16-bit (channel-contiguous, 16-B aligned channel groups);
// statistics, master weights and gradients are fp32.
//
// Storage type: every source is compiled twice (Makefile): bf16 storage
// (libstfunet_hip.so, the default) and, with -DSTF_FP16, fp16 storage
// (libstfunet_hip_f16.so: the reference's autocast(float16) + GradScaler numerics,
// train_and_eval.py:389, train.py:240).  Both are 16-bit with the same layouts, tiles and
// MFMA rate; only the element type, its conversions and the MFMA opcode differ.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <tuple>
#include <type_traits>
#include <utility>

#ifdef STF_FP16
typedef _Float16 e16;
#else
typedef __bf16 e16;
#endif
typedef e16 e16x8 __attribute__((ext_vector_type(8)));
typedef e16 e16x4 __attribute__((ext_vector_type(4)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));

#define STF_DEV __device__ __forceinline__

// ---------------------------------------------------------------- conversions
STF_DEV float e2f(e16 v) { return (float)v; }
// v_cvt_pk_bf16_f32 / v_cvt_f16_f32: round to nearest even, NaN-preserving
STF_DEV e16 f2e(float v) { return (e16)v; }

// D += A . B on one 16x16x32 MFMA of the storage type (fp32 accumulation)
STF_DEV f32x4 mfma16x16x32(e16x8 a, e16x8 b, f32x4 c) {
#ifdef STF_FP16
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
#else
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
#endif
}

STF_DEV float lo16(uint32_t w) {
#ifdef STF_FP16
  return (float)__builtin_bit_cast(_Float16, (uint16_t)(w & 0xffffu));
#else
  return __uint_as_float(w << 16);
#endif
}
STF_DEV float hi16(uint32_t w) {
#ifdef STF_FP16
  return (float)__builtin_bit_cast(_Float16, (uint16_t)(w >> 16));
#else
  return __uint_as_float(w & 0xffff0000u);
#endif
}

STF_DEV void unpack8(const uint4& u, float (&f)[8]) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = lo16(w[i]);
    f[2 * i + 1] = hi16(w[i]);
  }
}

STF_DEV uint32_t pack2(float a, float b) {
  e16 x = f2e(a), y = f2e(b);
  return (uint32_t)__builtin_bit_cast(uint16_t, x) | ((uint32_t)__builtin_bit_cast(uint16_t, y) << 16);
}

STF_DEV uint4 pack8(const float (&f)[8]) {
  return make_uint4(pack2(f[0], f[1]), pack2(f[2], f[3]), pack2(f[4], f[5]), pack2(f[6], f[7]));
}

STF_DEV float round_e(float v) { return e2f(f2e(v)); }

// LSTM activations on the hardware transcendental units (v_exp_f32, v_rcp_f32): ~1e-7
// absolute error, far below the bf16 storage of h.  The forward cell, the backward's
// gate recompute and the cell backward all use these, so the recomputed gates equal
// the forward's bit for bit.
STF_DEV float sigm(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
STF_DEV float tanh_f(float x) { return __builtin_fmaf(2.f, sigm(2.f * x), -1.f); }

// The LSTM cell, shared by every path that computes it (the per-step GEMM epilogues, the
// whole-sequence and the cooperative kernels, the standalone cell backward), with every
// contraction spelled out (contract(off) + explicit fma): left to the compiler, the same
// source expression fused differently in different kernels (register pressure decides) and
// the paths disagreed by an ulp.  Forward: gates from pre-activations (i, f, g, o),
// c = f c_prev + i g, h = o tanh(c).
STF_DEV void lstm_cell_fwd(float pi, float pf, float pg, float po, float cp, float& gi, float& gf, float& gg,
                           float& go, float& c, float& h) {
#pragma clang fp contract(off)
  gi = sigm(pi); gf = sigm(pf); gg = tanh_f(pg); go = sigm(po);
  c = __builtin_fmaf(gf, cp, gi * gg);
  h = go * tanh_f(c);
}
// Backward of one cell step: dct = dh o (1 - tanh^2 c) + dc_next; pre-activation gate
// gradients (di, df, dg, do) and dc_prev = dct f.
STF_DEV void lstm_cell_bwd(float gi, float gf, float gg, float go, float ct, float cp, float dh, float dcn,
                           float& d_i, float& d_f, float& d_g, float& d_o, float& dcp) {
#pragma clang fp contract(off)
  const float tc = tanh_f(ct);
  const float dct = __builtin_fmaf(dh * go, __builtin_fmaf(-tc, tc, 1.f), dcn);
  d_o = ((dh * tc) * go) * (1.f - go);
  d_i = ((dct * gg) * gi) * (1.f - gi);
  d_g = (dct * gi) * __builtin_fmaf(-gg, gg, 1.f);
  d_f = ((dct * cp) * gf) * (1.f - gf);
  dcp = dct * gf;
}

// ---------------------------------------------------------------- reductions
STF_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// DPP exchange inside a row of 16 lanes (VALU, no LDS traffic)
template <int CTRL>
STF_DEV float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}

// Reduce-scatter of 16 values over the 16 lanes of a DPP row: returns, on lane r of
// the row, the row sum of value r.  Hypercube over the lane masks 15, 7, 3, 1
// (row_mirror, row_half_mirror, quad_perm [3,2,1,0], quad_perm [1,0,3,2]); each
// step keeps the half of the values selected by the lane bit that mask flips last.
STF_DEV float row16_reduce_scatter(const float (&v)[16], int r) {
  float a[8], b[4], c[2];
  const bool h3 = r & 8, h2 = r & 4, h1 = r & 2, h0 = r & 1;
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] = (h3 ? v[k + 8] : v[k]) + dpp_f<0x140>(h3 ? v[k] : v[k + 8]);
#pragma unroll
  for (int k = 0; k < 4; ++k) b[k] = (h2 ? a[k + 4] : a[k]) + dpp_f<0x141>(h2 ? a[k] : a[k + 4]);
#pragma unroll
  for (int k = 0; k < 2; ++k) c[k] = (h1 ? b[k + 2] : b[k]) + dpp_f<0x1B>(h1 ? b[k] : b[k + 2]);
  return (h0 ? c[1] : c[0]) + dpp_f<0xB1>(h0 ? c[0] : c[1]);
}

STF_DEV double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---------------------------------------------------------------- launch plans
// Every launch of the library goes through stf::launch (hipLaunchKernelGGL is redefined
// below), and every async memset / copy through stf::memset_async / memcpy_async.  While a
// plan records on the calling thread (stf_plan_record, plan.hip), each one is executed AND
// appended to the plan with its final kernel arguments by value, so the whole step (the
// host-side tile choice, plans and size queries included) replays from C++ with one call
// per segment (stf_plan_replay): no Python, no ctypes, no re-planning.
namespace stf {
struct PlanOp {
  virtual ~PlanOp() {}
  virtual hipError_t run() const = 0;
};
bool plan_recording();              // a plan records on this thread
void plan_append(PlanOp* op, hipStream_t s);   // the recording plan takes ownership

template <class... A>
struct KernelOp final : PlanOp {
  const void* fn;
  dim3 grid, block;
  unsigned shmem;
  hipStream_t stream;
  std::tuple<A...> args;
  template <class... B>
  KernelOp(const void* f, dim3 g, dim3 b, unsigned sh, hipStream_t s, B&&... a)
      : fn(f), grid(g), block(b), shmem(sh), stream(s), args(std::forward<B>(a)...) {}
  hipError_t run() const override {
    return std::apply(
        [this](const A&... a) {
          void* p[sizeof...(A) + 1] = {const_cast<void*>(static_cast<const void*>(&a))...};
          return hipLaunchKernel(fn, grid, block, p, shmem, stream);
        },
        args);
  }
};

template <class... A, class... B>
inline void launch(void (*k)(A...), dim3 g, dim3 b, unsigned sh, hipStream_t s, B&&... args) {
  static_assert(sizeof...(A) == sizeof...(B), "kernel argument count");
  if (!plan_recording()) {
    // the kernel's own parameter types, converted exactly as a <<<>>> launch converts them
    std::tuple<std::decay_t<A>...> t(std::forward<B>(args)...);
    std::apply(
        [&](auto&... a) {
          void* p[sizeof...(A) + 1] = {static_cast<void*>(&a)...};
          (void)hipLaunchKernel((const void*)k, g, b, p, sh, s);
        },
        t);
    return;
  }
  auto* op = new KernelOp<std::decay_t<A>...>((const void*)k, g, b, sh, s, std::forward<B>(args)...);
  (void)op->run();
  plan_append(op, s);
}

hipError_t memset_async(void* p, int value, size_t bytes, hipStream_t s);
// Timing-only ablation knobs (results are WRONG while one is on: STF_HALO_DIAG, STF_WGRAD_DIAG,
// STF_WGRAD_ONE_SLAB) take effect only with STF_ABLATION=1 also set; otherwise a set knob is
// refused with one line on stderr and reads as 0.  Defined in plan.hip.
int ablation_env(const char* name);
// A/B switches (results stay valid; each is read once, at its first use).  The complete list, with
// defaults and what each compares, is DESIGN.md "A/B switches"; nothing else in the library reads
// the environment.
int ab_switch(const char* name, int dflt);
char ab_letter(const char* name);     // first character of the value, 0 when unset
hipError_t memcpy_async(void* dst, const void* src, size_t bytes, hipMemcpyKind kind, hipStream_t s);
}  // namespace stf

#undef hipLaunchKernelGGL
#define hipLaunchKernelGGL(K, G, B, SH, S, ...) ::stf::launch(K, G, B, SH, S, ##__VA_ARGS__)

// ---------------------------------------------------------------- error plumbing
#define STF_CHECK_LAUNCH() do { hipError_t e__ = hipGetLastError(); if (e__ != hipSuccess) return (int)e__; } while (0)

// Argument-validation failures are reported as this code (outside hipError_t's range).
#define STF_EINVAL 100001
