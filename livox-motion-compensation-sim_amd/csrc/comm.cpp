// comm.cpp — multi-GPU merged-cloud gather over RCCL (xGMI), the only exchange step of the path.
//
// The reference concatenates the frame-ordered aligned clouds with np.vstack (LMC:887-889).
// Frames shard across ranks as contiguous, point-balanced ranges, so the merged cloud is the
// rank-ordered concatenation of every rank's blocked columns (frames start on 256-point block
// boundaries, so a rank's shard is one contiguous run of blocks): one ragged gather to root, one
// grouped ncclSend/ncclRecv per rank (no reduction collective is involved).  A shard whose
// column count differs from the merged batch's (t_ns carried on one side only) lands in a
// staging area and is re-pitched block by block with one 2-D copy.
// librccl is dlopen'ed on first use so the core library loads without it.
#include "../../include/mcdeskew.h"
#include "internal.hpp"
#include "gather.hpp"
#include "plan.hpp"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>
#include <vector>

using mcimpl::fail;

namespace {
struct Rccl {
  void* h = nullptr;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
};
Rccl g_rccl;
std::once_flag g_once;
std::string g_load_err;

void load_rccl() {
  const char* names[] = {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"};
  for (const char* n : names) {
    g_rccl.h = dlopen(n, RTLD_NOW | RTLD_LOCAL);
    if (g_rccl.h) break;
  }
  if (!g_rccl.h) { g_load_err = std::string("cannot dlopen librccl: ") + dlerror(); return; }
#define SYM(field, name)                                                             \
  g_rccl.field = reinterpret_cast<decltype(g_rccl.field)>(dlsym(g_rccl.h, name));     \
  if (!g_rccl.field) { g_load_err = "librccl lacks " name; g_rccl.h = nullptr; return; }
  SYM(GetUniqueId, "ncclGetUniqueId");
  SYM(CommInitRank, "ncclCommInitRank");
  SYM(CommDestroy, "ncclCommDestroy");
  SYM(Send, "ncclSend");
  SYM(Recv, "ncclRecv");
  SYM(AllGather, "ncclAllGather");
  SYM(AllReduce, "ncclAllReduce");
  SYM(GroupStart, "ncclGroupStart");
  SYM(GroupEnd, "ncclGroupEnd");
  SYM(GetErrorString, "ncclGetErrorString");
#undef SYM
}

int need_rccl() {
  std::call_once(g_once, load_rccl);
  if (!g_rccl.h) return fail(MC_ERR_COMM, "%s", g_load_err.c_str());
  return MC_OK;
}
}  // namespace

using mcgather::kPlanWords;

struct mc_comm {
  mc_ctx* ctx = nullptr;
  ncclComm_t comm = nullptr;
  int nranks = 0, rank = 0;
  int64_t* d_scratch = nullptr;  // kPlanWords (nranks + 1) int64: the per-rank plan allgather
  float* d_stage = nullptr;      // root: shards whose column count differs from the merged batch
  int64_t stage_cap = 0;
  double* d_red = nullptr;       // reduction buffer
  int64_t red_cap = 0;
};

namespace {
// grow-only device staging area for shards re-pitched on arrival
int ensure_stage(float** d, int64_t* cap, int64_t values) {
  if (values <= *cap) return MC_OK;
  if (*d) (void)hipFree(*d);
  *d = nullptr;
  *cap = 0;
  const hipError_t e = hipMalloc(d, (size_t)values * sizeof(float));
  if (e != hipSuccess) return fail(MC_ERR_NOMEM, "gather staging (%lld values): %s", (long long)values, hipGetErrorString(e));
  *cap = values;
  return MC_OK;
}
// plan.hpp's gather_finish with device copies on stream s (HIP status of the first failure)
hipError_t finish_on_device(const mcplan::GatherPlan& G, int nranks, int root, const int64_t* P, const int64_t* C,
                            mc_batch* merged, const float* root_src, const float* stage, hipStream_t s) {
  hipError_t err = hipSuccess;
  auto copy = [&](float* d, const float* src, int64_t n) {
    err = hipMemcpyAsync(d, src, (size_t)n * sizeof(float), hipMemcpyDeviceToDevice, s);
    return err == hipSuccess ? 0 : 1;
  };
  auto copy2d = [&](float* d, int64_t dp, const float* src, int64_t sp, int64_t w, int64_t rows) {
    err = hipMemcpy2DAsync(d, (size_t)dp * sizeof(float), src, (size_t)sp * sizeof(float), (size_t)w * sizeof(float),
                           (size_t)rows, hipMemcpyDeviceToDevice, s);
    return err == hipSuccess ? 0 : 1;
  };
  mcplan::gather_finish(G, nranks, root, P, C, merged->d_cols, merged->C, root_src, stage, copy, copy2d);
  return err;
}
}  // namespace

#define NCCLCHK(expr)                                                                     \
  do {                                                                                    \
    ncclResult_t r_ = (expr);                                                             \
    if (r_ != ncclSuccess) return fail(MC_ERR_COMM, "%s: %s", #expr, g_rccl.GetErrorString(r_)); \
  } while (0)
#define HIPCHK(expr)                                                                      \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess) return fail(MC_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

// mcgather::Transport over RCCL on the context stream: the plan words through one ncclAllGather of
// device scratch, shards as grouped ncclSend / ncclRecv, the finishing copies as HIP copies.
namespace {
struct RcclGather {
  mc_comm* c;
  hipStream_t s;
};
int rg_hip(hipError_t e, const char* what) {
  return e == hipSuccess ? MC_OK : fail(MC_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
}
int rg_nccl(ncclResult_t r, const char* what) {
  return r == ncclSuccess ? MC_OK : fail(MC_ERR_COMM, "%s: %s", what, g_rccl.GetErrorString(r));
}
mcgather::Transport rccl_transport(RcclGather* x) {
  mcgather::Transport T;
  T.self = x;
  T.nranks = x->c->nranks;
  T.rank = x->c->rank;
  T.allgather_i64 = [](void* p, const int64_t* mine, int n, int64_t* all) {
    RcclGather* g = static_cast<RcclGather*>(p);
    int64_t* d = g->c->d_scratch;   // [nranks * kPlanWords | own words]
    const int nr = g->c->nranks;
    if (int r = rg_hip(hipMemcpyAsync(d + (size_t)n * nr, mine, sizeof(int64_t) * n, hipMemcpyHostToDevice, g->s),
                       "plan upload")) return r;
    if (int r = rg_nccl(g_rccl.AllGather(d + (size_t)n * nr, d, (size_t)n, ncclInt64, g->c->comm, g->s),
                        "ncclAllGather")) return r;
    if (int r = rg_hip(hipMemcpyAsync(all, d, sizeof(int64_t) * n * nr, hipMemcpyDeviceToHost, g->s), "plan download"))
      return r;
    return rg_hip(hipStreamSynchronize(g->s), "plan sync");
  };
  T.group_start = [](void*) { return rg_nccl(g_rccl.GroupStart(), "ncclGroupStart"); };
  T.group_end = [](void*) { return rg_nccl(g_rccl.GroupEnd(), "ncclGroupEnd"); };
  T.send = [](void* p, const float* buf, int64_t n, int peer) {
    RcclGather* g = static_cast<RcclGather*>(p);
    return rg_nccl(g_rccl.Send(buf, (size_t)n, ncclFloat32, peer, g->c->comm, g->s), "ncclSend");
  };
  T.recv = [](void* p, float* buf, int64_t n, int peer) {
    RcclGather* g = static_cast<RcclGather*>(p);
    return rg_nccl(g_rccl.Recv(buf, (size_t)n, ncclFloat32, peer, g->c->comm, g->s), "ncclRecv");
  };
  T.stage = [](void* p, int64_t values, float** out) {
    RcclGather* g = static_cast<RcclGather*>(p);
    if (int r = ensure_stage(&g->c->d_stage, &g->c->stage_cap, values)) return r;
    *out = g->c->d_stage;
    return MC_OK;
  };
  T.copy = [](void* p, float* d, const float* src, int64_t n) {
    RcclGather* g = static_cast<RcclGather*>(p);
    return rg_hip(hipMemcpyAsync(d, src, (size_t)n * sizeof(float), hipMemcpyDeviceToDevice, g->s), "gather copy");
  };
  T.copy2d = [](void* p, float* d, int64_t dp, const float* src, int64_t sp, int64_t w, int64_t rows) {
    RcclGather* g = static_cast<RcclGather*>(p);
    return rg_hip(hipMemcpy2DAsync(d, (size_t)dp * sizeof(float), src, (size_t)sp * sizeof(float),
                                   (size_t)w * sizeof(float), (size_t)rows, hipMemcpyDeviceToDevice, g->s),
                  "gather re-pitch");
  };
  T.sync = [](void* p) { return rg_hip(hipStreamSynchronize(static_cast<RcclGather*>(p)->s), "gather sync"); };
  return T;
}
}  // namespace

extern "C" {

int mc_comm_unique_id(char id_out[128]) {
  if (!id_out) return fail(MC_ERR_INVALID, "id_out is NULL");
  if (int r = need_rccl()) return r;
  ncclUniqueId id;
  NCCLCHK(g_rccl.GetUniqueId(&id));
  std::memcpy(id_out, id.internal, NCCL_UNIQUE_ID_BYTES);
  return MC_OK;
}

int mc_comm_init(mc_ctx* ctx, int nranks, int rank, const char id_in[128], mc_comm** out) {
  if (!ctx || !id_in || !out) return fail(MC_ERR_INVALID, "NULL argument");
  *out = nullptr;
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail(MC_ERR_INVALID, "bad rank %d of %d", rank, nranks);
  if (int r = need_rccl()) return r;
  HIPCHK(hipSetDevice(ctx->device));
  ncclUniqueId id;
  std::memcpy(id.internal, id_in, NCCL_UNIQUE_ID_BYTES);
  mc_comm* c = new mc_comm();
  c->ctx = ctx;
  c->nranks = nranks;
  c->rank = rank;
  ncclResult_t r = g_rccl.CommInitRank(&c->comm, nranks, id, rank);
  if (r != ncclSuccess) { delete c; return fail(MC_ERR_COMM, "ncclCommInitRank: %s", g_rccl.GetErrorString(r)); }
  if (hipMalloc(&c->d_scratch, sizeof(int64_t) * kPlanWords * (nranks + 1)) != hipSuccess) {
    g_rccl.CommDestroy(c->comm);
    delete c;
    return fail(MC_ERR_NOMEM, "hipMalloc failed");
  }
  *out = c;
  return MC_OK;
}

int mc_comm_destroy(mc_comm* c) {
  if (!c) return MC_OK;
  (void)hipSetDevice(c->ctx->device);
  (void)hipStreamSynchronize(c->ctx->stream);
  if (c->comm) g_rccl.CommDestroy(c->comm);
  if (c->d_scratch) (void)hipFree(c->d_scratch);
  if (c->d_red) (void)hipFree(c->d_red);
  if (c->d_stage) (void)hipFree(c->d_stage);
  delete c;
  return MC_OK;
}

int mc_comm_gather_batch(mc_comm* c, const mc_batch* local, int root, mc_batch* merged) {
  if (!c || !local) return fail(MC_ERR_INVALID, "NULL argument");
  if (local->ctx != c->ctx) return fail(MC_ERR_INVALID, "batch belongs to another context");
  const bool is_root = c->rank == root;
  // a root whose merged batch is unusable still joins the plan all-gather as "no merged batch", so
  // every rank fails together instead of waiting on it
  const bool foreign = is_root && merged && merged->ctx != c->ctx;
  if (foreign) merged = nullptr;
  HIPCHK(hipSetDevice(c->ctx->device));
  RcclGather X{c, c->ctx->stream};
  const mcgather::Transport T = rccl_transport(&X);
  mcgather::Shard sh;
  sh.P = local->P; sh.C = local->C; sh.F = local->F; sh.counts = local->counts.data(); sh.cols = local->d_cols;
  mcgather::Merged mg;
  if (is_root && merged) {
    mg.P = merged->P; mg.C = merged->C; mg.F = merged->F; mg.counts = merged->counts.data(); mg.cols = merged->d_cols;
    merged->wrote(false);
  }
  std::string msg;
  const int r = mcgather::run(T, root, sh, is_root && merged ? &mg : nullptr, &msg);
  if (foreign) return fail(MC_ERR_INVALID, "merged batch belongs to another context");
  if (r == mcgather::kBadPlan) return fail(MC_ERR_INVALID, "%s", msg.c_str());
  if (r) return r;   // the primitive recorded its message (mc_last_error)
  if (is_root) merged->trange_valid = false;   // column 4 (t_ns) was written: its cached spans are stale
  return MC_OK;
}

int mc_comm_allreduce_max_f64(mc_comm* c, double* v, int64_t n) {
  if (!c || (!v && n > 0)) return fail(MC_ERR_INVALID, "NULL argument");
  if (n <= 0) return MC_OK;
  HIPCHK(hipSetDevice(c->ctx->device));
  hipStream_t s = c->ctx->stream;
  if (n > c->red_cap) {
    if (c->d_red) (void)hipFree(c->d_red);
    c->d_red = nullptr;
    c->red_cap = 0;
    HIPCHK(hipMalloc(&c->d_red, sizeof(double) * n));
    c->red_cap = n;
  }
  HIPCHK(hipMemcpyAsync(c->d_red, v, sizeof(double) * n, hipMemcpyHostToDevice, s));
  NCCLCHK(g_rccl.AllReduce(c->d_red, c->d_red, (size_t)n, ncclFloat64, ncclMax, c->comm, s));
  HIPCHK(hipMemcpyAsync(v, c->d_red, sizeof(double) * n, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  return MC_OK;
}

// Host-only: the plan of a merged-cloud gather (plan.hpp), for callers and tests to inspect.
int mc_gather_plan(int32_t nranks, int32_t root, const int64_t* padded, const int64_t* columns, int64_t merged_padded,
                   int32_t merged_columns, int64_t* offset_out, int64_t* stage_offset_out, int64_t* stage_values_out) {
  if (!padded || !columns) return fail(MC_ERR_INVALID, "NULL argument");
  mcplan::GatherPlan G;
  const std::string perr = mcplan::plan_gather(nranks, root, padded, columns, merged_padded, merged_columns, &G);
  if (!perr.empty()) return fail(MC_ERR_INVALID, "%s", perr.c_str());
  for (int32_t q = 0; q < nranks; ++q) {
    if (offset_out) offset_out[q] = G.off[q];
    if (stage_offset_out) stage_offset_out[q] = G.stage_off[q];
  }
  if (stage_values_out) *stage_values_out = G.stage_values;
  return MC_OK;
}

// One process, n shard batches of one context merged exactly as mc_comm_gather_batch merges n
// ranks' shards: the same plan, staging and re-pitch; device copies stand in for the RCCL
// receives (shard `root` is the root's own batch).
int mc_gather_batches(mc_ctx* ctx, int32_t n, const mc_batch* const* shards, int32_t root, mc_batch* merged) {
  if (!ctx || !shards || !merged || n < 1) return fail(MC_ERR_INVALID, "NULL argument");
  if (merged->ctx != ctx) return fail(MC_ERR_INVALID, "merged batch belongs to another context");
  std::vector<int64_t> P(n), C(n), F(n);
  std::vector<const int64_t*> counts(n);
  for (int32_t q = 0; q < n; ++q) {
    if (!shards[q] || shards[q]->ctx != ctx) return fail(MC_ERR_INVALID, "shard %d is NULL or of another context", q);
    if (shards[q] == merged) return fail(MC_ERR_INVALID, "shard %d is the merged batch (the copies would overlap)", q);
    P[q] = shards[q]->P;
    C[q] = shards[q]->C;
    F[q] = shards[q]->F;
    counts[q] = shards[q]->counts.data();
  }
  mcplan::GatherPlan G;
  std::string perr = mcplan::plan_gather(n, root, P.data(), C.data(), merged->P, merged->C, &G);
  if (perr.empty()) perr = mcplan::check_frame_concat(n, counts.data(), F.data(), merged->counts.data(), merged->F);
  if (!perr.empty()) return fail(MC_ERR_INVALID, "%s", perr.c_str());
  HIPCHK(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  float* stage = nullptr;
  if (G.stage_values > 0) HIPCHK(hipMalloc(&stage, (size_t)G.stage_values * sizeof(float)));
  merged->wrote(false);
  hipError_t e = hipSuccess;
  for (int32_t q = 0; q < n && e == hipSuccess; ++q) {
    if (q == root || P[q] == 0) continue;
    e = hipMemcpyAsync(mcplan::gather_dst(G, q, merged->d_cols, merged->C, stage), shards[q]->d_cols,
                       (size_t)(C[q] * P[q]) * sizeof(float), hipMemcpyDeviceToDevice, s);
  }
  if (e == hipSuccess) e = finish_on_device(G, n, root, P.data(), C.data(), merged, shards[root]->d_cols, stage, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (stage) (void)hipFree(stage);
  if (e != hipSuccess) return fail(MC_ERR_HIP, "gather_batches: %s", hipGetErrorString(e));
  merged->trange_valid = false;
  return MC_OK;
}

}  // extern "C"
