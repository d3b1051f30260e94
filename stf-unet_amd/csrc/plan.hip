// Launch plans: a training step's launch sequence recorded once and replayed from C++.
//
// The programs (stfunet/unet.py, stfunet/stf_lstm_unet.py) issue their step as ~500
// C-ABI calls from Python (STF: ~7 ms of host time per step around ~600 launches,
// DESIGN.md section 5).  While a plan records on the calling thread, every launch of
// this library (stf::launch, common.h), every async memset / copy and every cross-stream
// wait (stf_stream_wait) runs as usual AND is appended to the plan as a self-contained
// op: the kernel's final arguments by value (the host-side tile choice, split plans and
// size queries already resolved), its grid, block and stream.  stf_plan_replay then
// re-issues a range of ops from C++ -- the same kernels on the same streams in the same
// order, with the same cross-stream events -- so a replayed step computes bit for bit
// what the recorded (eager) step computed, for the buffers the plan was recorded on
// (the caller keeps them alive and at fixed addresses: stfunet/plan.py).
//
// Unlike a HIP graph, the replay keeps the eager multi-stream schedule: the runtime's
// own scheduling of a captured 600-node graph measured slower than eager (DESIGN.md
// section 5, r02).
#include "common.h"
#include "../../include/stfunet.h"

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace {

struct TagRange {
  int first, last;      // ops [first, last) belong to one tagged C-ABI call
  std::string name;
  double flops;
};

}  // namespace

struct stf_plan {
  std::vector<std::unique_ptr<stf::PlanOp>> ops;
  std::vector<hipStream_t> op_stream;      // stream of each op (timing events go there)
  std::vector<TagRange> tags;
  int open_tag = -1;                       // index into tags while a tagged call records
  // timing of tagged ranges during replays (stf_plan_replay with a tag name)
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
  std::vector<int> ev_range;               // range index of each used event pair
  size_t ev_used = 0;
  ~stf_plan() {
    for (auto& e : ev) {
      (void)hipEventDestroy(e.first);
      (void)hipEventDestroy(e.second);
    }
  }
};

namespace {

thread_local stf_plan* g_rec = nullptr;

struct MemsetOp final : stf::PlanOp {
  void* p;
  int value;
  size_t bytes;
  hipStream_t s;
  hipError_t run() const override { return hipMemsetAsync(p, value, bytes, s); }
};

struct MemcpyOp final : stf::PlanOp {
  void* dst;
  const void* src;
  size_t bytes;
  hipStream_t s;
  hipError_t run() const override { return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s); }
};

struct WaitOp final : stf::PlanOp {
  hipEvent_t ev = nullptr;                 // owned: one event per recorded wait
  hipStream_t waiter, waitee;
  ~WaitOp() override {
    if (ev) (void)hipEventDestroy(ev);
  }
  hipError_t run() const override {
    hipError_t e = hipEventRecord(ev, waitee);
    return e != hipSuccess ? e : hipStreamWaitEvent(waiter, ev, 0);
  }
};

void append(stf::PlanOp* op, hipStream_t s) {
  g_rec->ops.emplace_back(op);
  g_rec->op_stream.push_back(s);
}

// Eager cross-stream waits: a ring of events per device.  A wait enqueued on an event
// keeps waiting for the record it saw, so re-recording an event later is safe.
std::mutex g_pool_mu;
std::map<int, std::vector<hipEvent_t>> g_pool;
std::map<int, unsigned> g_pool_next;
constexpr int POOL = 64;

hipError_t pooled_event(hipEvent_t* out) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> g(g_pool_mu);
  auto& v = g_pool[dev];
  if (v.size() < POOL) {
    hipEvent_t ev;
    e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e != hipSuccess) return e;
    v.push_back(ev);
    *out = ev;
    return hipSuccess;
  }
  unsigned& i = g_pool_next[dev];
  *out = v[i++ % POOL];
  return hipSuccess;
}

// dst[r][c] = src[r][c] for r < rows, c < cols (fp32 rows of different lengths: a
// weight gradient computed over channel-padded columns copied into its parameter)
__global__ __launch_bounds__(256) void copy_rows_kernel(const float* __restrict__ src, int64_t src_ld,
                                                         float* __restrict__ dst, int64_t dst_ld, int rows,
                                                         int cols) {
  const int64_t n = (int64_t)rows * cols;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / cols, c = i - r * cols;
    dst[r * dst_ld + c] = src[r * src_ld + c];
  }
}

constexpr int I64_BATCH = 64;
struct I64Batch {
  int64_t* p[I64_BATCH];
};

__global__ void i64_add_kernel(I64Batch b, int n, int64_t inc) {
  if ((int)threadIdx.x < n) b.p[threadIdx.x][0] += inc;
}

}  // namespace

bool stf::plan_recording() { return g_rec != nullptr; }

void stf::plan_append(stf::PlanOp* op, hipStream_t s) { append(op, s); }

int stf::ablation_env(const char* name) {
  const char* e = getenv(name);
  if (!e || !e[0] || (e[0] == '0' && !e[1])) return 0;
  const char* ok = getenv("STF_ABLATION");
  if (ok && ok[0] == '1') {
    fprintf(stderr, "stfunet: timing-only ablation %s=%s is ON -- results are not valid\n", name, e);
    return atoi(e);
  }
  fprintf(stderr, "stfunet: %s=%s ignored (a timing-only ablation: set STF_ABLATION=1 as well)\n", name, e);
  return 0;
}

int stf::ab_switch(const char* name, int dflt) {
  const char* e = getenv(name);
  return (e && e[0]) ? atoi(e) : dflt;
}

char stf::ab_letter(const char* name) {
  const char* e = getenv(name);
  return e ? e[0] : 0;
}

hipError_t stf::memset_async(void* p, int value, size_t bytes, hipStream_t s) {
  if (!g_rec) return hipMemsetAsync(p, value, bytes, s);
  auto* op = new MemsetOp;
  op->p = p;
  op->value = value;
  op->bytes = bytes;
  op->s = s;
  hipError_t e = op->run();
  append(op, s);
  return e;
}

hipError_t stf::memcpy_async(void* dst, const void* src, size_t bytes, hipMemcpyKind kind, hipStream_t s) {
  if (!g_rec) return hipMemcpyAsync(dst, src, bytes, kind, s);
  // a recorded copy must not read host memory the caller frees after this call
  if (kind != hipMemcpyDeviceToDevice) return hipErrorInvalidValue;
  auto* op = new MemcpyOp;
  op->dst = dst;
  op->src = src;
  op->bytes = bytes;
  op->s = s;
  hipError_t e = op->run();
  append(op, s);
  return e;
}

// ---------------------------------------------------------------- C ABI
extern "C" stf_plan* stf_plan_create(void) { return new stf_plan; }

extern "C" void stf_plan_destroy(stf_plan* p) { delete p; }

extern "C" int stf_plan_record(stf_plan* p) {
  if (!p || g_rec) return STF_EINVAL;
  p->ops.clear();
  p->op_stream.clear();
  p->tags.clear();
  p->open_tag = -1;
  g_rec = p;
  return 0;
}

extern "C" int stf_plan_stop(void) {
  if (!g_rec) return STF_EINVAL;
  if (g_rec->open_tag >= 0) g_rec->tags[g_rec->open_tag].last = (int)g_rec->ops.size();
  g_rec->open_tag = -1;
  g_rec = nullptr;
  return 0;
}

extern "C" int stf_plan_size(const stf_plan* p) { return p ? (int)p->ops.size() : -1; }

extern "C" int stf_plan_tag(const char* name, double flops) {
  if (!g_rec || !name) return 0;       // tags only mean something while recording
  stf_plan* p = g_rec;
  if (p->open_tag >= 0) p->tags[p->open_tag].last = (int)p->ops.size();
  p->tags.push_back(TagRange{(int)p->ops.size(), -1, name, flops});
  p->open_tag = (int)p->tags.size() - 1;
  return 0;
}

extern "C" int stf_plan_tag_end(void) {
  if (!g_rec || g_rec->open_tag < 0) return 0;
  g_rec->tags[g_rec->open_tag].last = (int)g_rec->ops.size();
  g_rec->open_tag = -1;
  return 0;
}

extern "C" int stf_plan_replay(stf_plan* p, int first, int last, const char* timed_tag) {
  if (!p || g_rec == p || first < 0 || last > (int)p->ops.size() || first > last) return STF_EINVAL;
  if (!timed_tag) {
    for (int i = first; i < last; ++i) {
      hipError_t e = p->ops[i]->run();
      if (e != hipSuccess) return (int)e;
    }
    return 0;
  }
  // timed replay: events around every range tagged `timed_tag`, on the stream its first
  // launch was recorded on (one C-ABI call's launches share a stream)
  size_t r = 0;
  const size_t nr = p->tags.size();
  for (int i = first; i < last; ++i) {
    while (r < nr && (p->tags[r].first < i || p->tags[r].last <= p->tags[r].first)) ++r;
    const bool start = r < nr && p->tags[r].first == i && p->tags[r].last > i && p->tags[r].name == timed_tag;
    int stop_at = -1;
    hipStream_t ts = nullptr;
    if (start) {
      if (p->ev_used == p->ev.size()) {
        hipEvent_t a, b;
        hipError_t e = hipEventCreate(&a);
        if (e == hipSuccess) e = hipEventCreate(&b);
        if (e != hipSuccess) return (int)e;
        p->ev.emplace_back(a, b);
        p->ev_range.push_back(0);
      }
      p->ev_range[p->ev_used] = (int)r;
      ts = p->op_stream[i];
      hipError_t e = hipEventRecord(p->ev[p->ev_used].first, ts);
      if (e != hipSuccess) return (int)e;
      stop_at = p->tags[r].last;
    }
    if (start) {
      for (int j = i; j < stop_at && j < last; ++j) {
        hipError_t e = p->ops[j]->run();
        if (e != hipSuccess) return (int)e;
      }
      hipError_t e = hipEventRecord(p->ev[p->ev_used].second, ts);
      if (e != hipSuccess) return (int)e;
      ++p->ev_used;
      i = (stop_at < last ? stop_at : last) - 1;
      continue;
    }
    hipError_t e = p->ops[i]->run();
    if (e != hipSuccess) return (int)e;
  }
  return 0;
}

extern "C" int stf_plan_timing(stf_plan* p, int* launches, double* ms, double* flops) {
  // synchronizes on the events of the timed replays since the last call, then resets
  if (!p) return STF_EINVAL;
  double t = 0.0, f = 0.0;
  for (size_t k = 0; k < p->ev_used; ++k) {
    hipError_t e = hipEventSynchronize(p->ev[k].second);
    if (e != hipSuccess) return (int)e;
    float m = 0.f;
    e = hipEventElapsedTime(&m, p->ev[k].first, p->ev[k].second);
    if (e != hipSuccess) return (int)e;
    t += m;
    f += p->tags[p->ev_range[k]].flops;
  }
  *launches = (int)p->ev_used;
  *ms = t;
  *flops = f;
  p->ev_used = 0;
  return 0;
}

extern "C" int stf_stream_wait(stf_stream_t waiter, stf_stream_t waitee) {
  if (waiter == waitee) return 0;
  if (g_rec) {
    auto* op = new WaitOp;
    hipError_t e = hipEventCreateWithFlags(&op->ev, hipEventDisableTiming);
    if (e != hipSuccess) {
      op->ev = nullptr;
      delete op;
      return (int)e;
    }
    op->waiter = (hipStream_t)waiter;
    op->waitee = (hipStream_t)waitee;
    e = op->run();
    append(op, (hipStream_t)waiter);
    return (int)e;
  }
  hipEvent_t ev;
  hipError_t e = pooled_event(&ev);
  if (e == hipSuccess) e = hipEventRecord(ev, (hipStream_t)waitee);
  if (e == hipSuccess) e = hipStreamWaitEvent((hipStream_t)waiter, ev, 0);
  return (int)e;
}

extern "C" int stf_memset(void* p, int value, size_t bytes, stf_stream_t stream) {
  if (!p && bytes) return STF_EINVAL;
  if (!bytes) return 0;
  return (int)stf::memset_async(p, value, bytes, (hipStream_t)stream);
}

extern "C" int stf_copy_rows(const float* src, int64_t src_ld, float* dst, int64_t dst_ld, int rows, int cols,
                             stf_stream_t stream) {
  if (!src || !dst || rows < 0 || cols < 0 || src_ld < cols || dst_ld < cols) return STF_EINVAL;
  const int64_t n = (int64_t)rows * cols;
  if (!n) return 0;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(copy_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, src, src_ld, dst,
                     dst_ld, rows, cols);
  STF_CHECK_LAUNCH();
  return 0;
}

extern "C" int stf_i64_add_batch(int64_t* const* ptrs, int count, int64_t inc, stf_stream_t stream) {
  for (int i = 0; i < count; ++i)
    if (!ptrs[i] || ((uintptr_t)ptrs[i] & 7)) return STF_EINVAL;
  for (int i0 = 0; i0 < count; i0 += I64_BATCH) {
    const int n = count - i0 < I64_BATCH ? count - i0 : I64_BATCH;
    I64Batch b;
    for (int i = 0; i < I64_BATCH; ++i) b.p[i] = i < n ? ptrs[i0 + i] : nullptr;
    hipLaunchKernelGGL(i64_add_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, b, n, inc);
    STF_CHECK_LAUNCH();
  }
  return 0;
}
