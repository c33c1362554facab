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

struct mc_comm {
  mc_ctx* ctx = nullptr;
  ncclComm_t comm = nullptr;
  int nranks = 0, rank = 0;
  int64_t* d_scratch = nullptr;  // 2 (nranks + 1) int64 for the (padded size, columns) allgather
  float* d_stage = nullptr;      // root: shards whose column count differs from the merged batch
  int64_t stage_cap = 0;
  double* d_red = nullptr;       // reduction buffer
  int64_t red_cap = 0;
};

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
  if (hipMalloc(&c->d_scratch, sizeof(int64_t) * 2 * (nranks + 1)) != hipSuccess) {
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
  if (root < 0 || root >= c->nranks) return fail(MC_ERR_INVALID, "bad root %d", root);
  if (local->ctx != c->ctx) return fail(MC_ERR_INVALID, "batch belongs to another context");
  HIPCHK(hipSetDevice(c->ctx->device));
  hipStream_t s = c->ctx->stream;
  // every rank's padded length and column count (the merged layout is the rank-ordered concatenation)
  const int64_t mine[2] = {local->P, local->C};
  HIPCHK(hipMemcpyAsync(c->d_scratch + 2 * c->nranks, mine, sizeof(mine), hipMemcpyHostToDevice, s));
  NCCLCHK(g_rccl.AllGather(c->d_scratch + 2 * c->nranks, c->d_scratch, 2, ncclInt64, c->comm, s));
  std::vector<int64_t> PC(2 * c->nranks);
  HIPCHK(hipMemcpyAsync(PC.data(), c->d_scratch, sizeof(int64_t) * 2 * c->nranks, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  auto P = [&](int q) { return PC[2 * q]; };
  auto C = [&](int q) { return PC[2 * q + 1]; };
  if (c->rank != root) {
    if (local->P > 0) {
      NCCLCHK(g_rccl.GroupStart());
      NCCLCHK(g_rccl.Send(local->d_cols, (size_t)(local->C * local->P), ncclFloat32, root, c->comm, s));
      NCCLCHK(g_rccl.GroupEnd());
    }
    HIPCHK(hipStreamSynchronize(s));
    return MC_OK;
  }
  if (!merged) return fail(MC_ERR_INVALID, "root needs a merged batch");
  int64_t tot = 0, staged = 0;
  for (int q = 0; q < c->nranks; ++q) {
    tot += P(q);
    if (q != root && C(q) != merged->C) staged += C(q) * P(q);
  }
  if (tot != merged->P)
    return fail(MC_ERR_INVALID, "merged batch holds %lld padded points, ranks sent %lld", (long long)merged->P,
                (long long)tot);
  if (staged > c->stage_cap) {
    if (c->d_stage) (void)hipFree(c->d_stage);
    c->d_stage = nullptr;
    c->stage_cap = 0;
    HIPCHK(hipMalloc(&c->d_stage, staged * sizeof(float)));
    c->stage_cap = staged;
  }
  // copy the first min(C) columns of every block of a shard into the merged batch at `off`
  auto repitch = [&](const float* src, int64_t cs, int64_t np, int64_t off) {
    const int64_t cm = merged->C, w = std::min(cs, cm);
    return hipMemcpy2DAsync(merged->d_cols + off * cm, (size_t)(cm * mcimpl::kBatchBlock * sizeof(float)), src,
                            (size_t)(cs * mcimpl::kBatchBlock * sizeof(float)), (size_t)(w * mcimpl::kBatchBlock * sizeof(float)),
                            (size_t)(np / mcimpl::kBatchBlock), hipMemcpyDeviceToDevice, s);
  };
  std::vector<int64_t> off(c->nranks), soff(c->nranks, -1);
  NCCLCHK(g_rccl.GroupStart());
  for (int64_t q = 0, o = 0, so = 0; q < c->nranks; o += P(q), ++q) {
    off[q] = o;
    if (q == root || P(q) == 0) continue;
    float* dst = merged->d_cols + o * merged->C;   // o is a multiple of kBatchBlock
    if (C(q) != merged->C) {
      dst = c->d_stage + so;
      soff[q] = so;
      so += C(q) * P(q);
    }
    NCCLCHK(g_rccl.Recv(dst, (size_t)(C(q) * P(q)), ncclFloat32, (int)q, c->comm, s));
  }
  NCCLCHK(g_rccl.GroupEnd());
  if (P(root) > 0) {
    if (local->C == merged->C)
      HIPCHK(hipMemcpyAsync(merged->d_cols + off[root] * merged->C, local->d_cols,
                            (size_t)(local->C * local->P) * sizeof(float), hipMemcpyDeviceToDevice, s));
    else
      HIPCHK(repitch(local->d_cols, local->C, local->P, off[root]));
  }
  for (int q = 0; q < c->nranks; ++q)
    if (soff[q] >= 0) HIPCHK(repitch(c->d_stage + soff[q], C(q), P(q), off[q]));
  HIPCHK(hipStreamSynchronize(s));
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

}  // extern "C"
