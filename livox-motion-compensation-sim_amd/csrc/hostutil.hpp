// hostutil.hpp — host-side helpers shared by the C-ABI translation units (status codes,
// device allocation, staging buffer, timing events).
#pragma once
#include "../../include/mcdeskew.h"
#include "internal.hpp"

#include <vector>

using mcimpl::fail;
#define HIPCHK(expr)                                                                        \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess)                                                                   \
      return fail(e_ == hipErrorOutOfMemory ? MC_ERR_NOMEM : MC_ERR_HIP, "%s failed: %s", \
                  #expr, hipGetErrorString(e_));                                            \
  } while (0)

#define CHECK_ARG(cond, ...) \
  do {                       \
    if (!(cond)) return fail(MC_ERR_INVALID, __VA_ARGS__); \
  } while (0)

// ------------------------------------------------------------------------------------------------
// small device-buffer helpers
// ------------------------------------------------------------------------------------------------
template <typename T>
static inline int dev_alloc(T** p, size_t n) {
  *p = nullptr;
  if (n == 0) n = 1;
  HIPCHK(hipMalloc(reinterpret_cast<void**>(p), n * sizeof(T)));
  return MC_OK;
}
template <typename T>
static inline void dev_free(T*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}

static inline int ctx_stage(mc_ctx* c, size_t bytes, void** out) {
  if (bytes > c->stage_bytes) {
    if (c->d_stage) { (void)hipStreamSynchronize(c->stream); (void)hipFree(c->d_stage); c->d_stage = nullptr; }
    c->stage_bytes = 0;
    HIPCHK(hipMalloc(&c->d_stage, bytes));
    c->stage_bytes = bytes;
  }
  *out = c->d_stage;
  return MC_OK;
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    (void)hipGetDevice(&prev);
    if (prev != dev) (void)hipSetDevice(dev);
  }
};

// event timing around the hot kernels
static inline hipEvent_t ev_take(mc_ctx* c) {
  if (!c->ev_pool.empty()) { hipEvent_t e = c->ev_pool.back(); c->ev_pool.pop_back(); return e; }
  hipEvent_t e = nullptr;
  // timing-only events: no system-scope fence (no L2 writeback/invalidate between the kernels)
  if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) return nullptr;
  return e;
}
struct TimedRegion {
  mc_ctx* c; std::vector<std::pair<hipEvent_t, hipEvent_t>>* v; hipStream_t s; hipEvent_t e0 = nullptr;
  TimedRegion(mc_ctx* c_, std::vector<std::pair<hipEvent_t, hipEvent_t>>* v_, hipStream_t s_) : c(c_), v(v_), s(s_) {
    if (c->timing) { e0 = ev_take(c); if (e0) (void)hipEventRecord(e0, s); }
  }
  ~TimedRegion() {
    if (c->timing && e0) {
      hipEvent_t e1 = ev_take(c);
      if (e1) { (void)hipEventRecord(e1, s); v->emplace_back(e0, e1); }
      else c->ev_pool.push_back(e0);
    }
  }
};

// A pair of timing events for one kernel launched with hipExtLaunchKernel: the runtime stamps
// them from the dispatch itself, so timing adds no marker packets between the step's kernels.
struct LaunchEvents {
  hipEvent_t e0 = nullptr, e1 = nullptr;
  explicit LaunchEvents(mc_ctx* c) : LaunchEvents(c, c->timing) {}
  LaunchEvents(mc_ctx* c, bool on) {
    if (!on) return;
    e0 = ev_take(c);
    e1 = e0 ? ev_take(c) : nullptr;
    if (e0 && !e1) { c->ev_pool.push_back(e0); e0 = nullptr; }
  }
  void keep(std::vector<std::pair<hipEvent_t, hipEvent_t>>* v) {
    if (e0) v->emplace_back(e0, e1);
    e0 = e1 = nullptr;
  }
};

// both streams idle (before reallocating tables a pipelined prep may still read or write)
static inline int sync_all(mc_ctx* c) {
  HIPCHK(hipStreamSynchronize(c->side));
  HIPCHK(hipStreamSynchronize(c->stream));
  return MC_OK;
}

static inline int sum_events(mc_ctx* c, std::vector<std::pair<hipEvent_t, hipEvent_t>>& v, double* ms, int64_t* n) {
  double tot = 0.0;
  for (auto& p : v) {
    float m = 0.f;
    HIPCHK(hipEventElapsedTime(&m, p.first, p.second));
    tot += m;
  }
  if (ms) *ms = tot;
  if (n) *n = (int64_t)v.size();
  for (auto& p : v) { c->ev_pool.push_back(p.first); c->ev_pool.push_back(p.second); }
  v.clear();
  return MC_OK;
}
