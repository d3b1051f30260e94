// Bench-only proxy for what RCCL's collective kernels do to the compute stream at N > 1
// (bench.py --hook --contend): on the DDP joiner stream, per gradient bucket, a kernel of
// RCCL-like shape -- `blocks` workgroups of 256 threads, resident for as long as an 8-GPU ring
// all-reduce of the bucket would take (2 (n-1)/n bytes / bus bandwidth), streaming over a
// scratch buffer of the bucket's size meanwhile.  Its workgroups hold their CUs exactly as the
// collective's would, so persistent kernels of the compute stream that launch during it see
// the same missing CUs.  Memory traffic: one read + write pass over the bucket-sized scratch
// (an all-reduce moves ~2x the bucket through local HBM), then the workgroups idle (s_sleep)
// until their time is up -- a proxy that streamed at full rate for the whole duration measured
// the HBM contention of a 1-2 TB/s copy, not what RCCL does.  Not part of the product library (include/stfunet.h): built by
// `make -C tools/contend` into tools/contend/libcontend.so and loaded by bench.py only.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ __launch_bounds__(256) void contend_kernel(float4* __restrict__ buf, long n4, long long ticks) {
  const long long t0 = __builtin_amdgcn_s_memrealtime();     // 100 MHz
  const long per = (n4 + gridDim.x - 1) / gridDim.x;
  const long lo = (long)blockIdx.x * per, hi = lo + per < n4 ? lo + per : n4;
  for (long i = lo + threadIdx.x; i < hi; i += 256) {
    float4 v = buf[i];
    v.x += 1.f;
    buf[i] = v;
  }
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

extern "C" int contend_launch(void* buf, long bytes, int blocks, double usec, hipStream_t stream) {
  if (!buf || bytes < 16 || blocks < 1) return 1;
  const long long ticks = (long long)(usec * 100.0);
  hipLaunchKernelGGL(contend_kernel, dim3(blocks), dim3(256), 0, stream, (float4*)buf, bytes / 16, ticks);
  return (int)hipGetLastError();
}
