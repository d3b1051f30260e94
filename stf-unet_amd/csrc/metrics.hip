// Evaluation counts: one pass over the logits of a batch gives
// the confusion-matrix increments and the per-class Dice counts that the reference's
// evaluate() builds with softmax + argmax + bincount + a per-class Python loop with a
// host synchronisation per class (train_utils/train_and_eval.py:30-39, 80-118, 316-336).
//
// Per pixel: pred = first argmax over the K logits; pd = first argmax over the K entries
// of probs (torch.softmax(logits, 1) for stf_eval_counts_sm, the reference's Dice path; the
// logits themselves for stf_eval_counts).
//   confusion:  target t in [0, K)  ->  confmat[t][pred] += 1
//   Dice:       with ignore_index >= 0 both pred and target are multiplied by
//               (t != ignore_index) (ignored pixels count as class 0 in both,
//               :87-90); counts[c] = (|P&T|, |P|, |T|) for c in [0, K)
// Block histograms in LDS (ds atomics), one 64-bit global atomic per counter per block.
#include "common.h"
#include "../../include/stfunet.h"

namespace {

constexpr int MT = 256;
constexpr int MAXK = 16;

__device__ __forceinline__ int first_argmax(const float* x, int K, long HW) {
  int pred = 0;
  float best = x[0];
  for (int k = 1; k < K; ++k) {
    const float v = x[k * HW];
    if (v > best || (v != v && best == best)) { best = v; pred = k; }   // first max; NaN wins (torch)
  }
  return pred;
}

__global__ __launch_bounds__(MT) void eval_counts_kernel(const float* __restrict__ logits,
                                                         const float* __restrict__ probs,
                                                         const int64_t* __restrict__ target, int B, int K,
                                                         long HW, long ignore, unsigned long long* confmat,
                                                         unsigned long long* counts) {
  __shared__ unsigned int hc[MAXK * MAXK], hd[MAXK * 3];
  for (int i = threadIdx.x; i < K * K; i += MT) hc[i] = 0;
  for (int i = threadIdx.x; i < K * 3; i += MT) hd[i] = 0;
  __syncthreads();
  const long total = (long)B * HW;
  for (long u = blockIdx.x * (long)MT + threadIdx.x; u < total; u += (long)gridDim.x * MT) {
    const long b = u / HW, hw = u - b * HW;
    const int pred = first_argmax(logits + b * K * HW + hw, K, HW);
    const int pdice = probs == logits ? pred : first_argmax(probs + b * K * HW + hw, K, HW);
    const long t = target[u];
    if (t >= 0 && t < K) atomicAdd(&hc[t * K + pred], 1u);
    const bool keep = ignore < 0 || t != ignore;
    const int pd = keep ? pdice : 0;
    const long tg = keep ? t : 0;
    atomicAdd(&hd[pd * 3 + 1], 1u);
    if (tg >= 0 && tg < K) {
      atomicAdd(&hd[tg * 3 + 2], 1u);
      if (tg == pd) atomicAdd(&hd[pd * 3 + 0], 1u);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < K * K; i += MT)
    if (hc[i]) atomicAdd(&confmat[i], (unsigned long long)hc[i]);
  for (int i = threadIdx.x; i < K * 3; i += MT)
    if (hd[i]) atomicAdd(&counts[i], (unsigned long long)hd[i]);
}

}  // namespace

extern "C" int stf_eval_counts_sm(const float* logits, const float* probs, const int64_t* target, int B, int K,
                                  int64_t HW, int64_t ignore_index, int64_t* confmat, int64_t* dice_counts,
                                  stf_stream_t stream) {
  if (B < 0 || K < 1 || K > MAXK || HW < 0 || !logits || !probs || !target || !confmat || !dice_counts)
    return STF_EINVAL;
  const long total = (long)B * HW;
  if (total == 0) return 0;
  long blocks = (total + MT - 1) / MT;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(eval_counts_kernel, dim3((unsigned)blocks), dim3(MT), 0, (hipStream_t)stream, logits, probs, target, B,
                     K, (long)HW, (long)ignore_index, (unsigned long long*)confmat, (unsigned long long*)dice_counts);
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_eval_counts(const float* logits, const int64_t* target, int B, int K, int64_t HW,
                               int64_t ignore_index, int64_t* confmat, int64_t* dice_counts, stf_stream_t stream) {
  return stf_eval_counts_sm(logits, logits, target, B, K, HW, ignore_index, confmat, dice_counts, stream);
}
