// comm.cpp — multi-GPU merged-cloud gather over RCCL (xGMI), the only exchange step of the path.
//
// The reference concatenates the frame-ordered aligned clouds with np.vstack (LMC:887-889).
// Frames shard across ranks as contiguous, point-balanced ranges, so the merged cloud is the
// rank-ordered concatenation of every rank's (padded-CSR) columns: one ragged gather to root,
// written as grouped ncclSend/ncclRecv per column (no reduction collective is involved).
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
  int64_t* d_scratch = nullptr;  // nranks int64 for the padded-size allgather
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
  if (hipMalloc(&c->d_scratch, sizeof(int64_t) * (nranks + 1)) != hipSuccess) {
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
  delete c;
  return MC_OK;
}

int mc_comm_gather_batch(mc_comm* c, const mc_batch* local, int root, mc_batch* merged) {
  if (!c || !local) return fail(MC_ERR_INVALID, "NULL argument");
  if (root < 0 || root >= c->nranks) return fail(MC_ERR_INVALID, "bad root %d", root);
  if (local->ctx != c->ctx) return fail(MC_ERR_INVALID, "batch belongs to another context");
  HIPCHK(hipSetDevice(c->ctx->device));
  hipStream_t s = c->ctx->stream;
  // every rank's padded length (the merged layout is the rank-ordered concatenation)
  int64_t mine = local->P;
  HIPCHK(hipMemcpyAsync(c->d_scratch + c->nranks, &mine, sizeof(int64_t), hipMemcpyHostToDevice, s));
  NCCLCHK(g_rccl.AllGather(c->d_scratch + c->nranks, c->d_scratch, 1, ncclInt64, c->comm, s));
  std::vector<int64_t> P(c->nranks);
  HIPCHK(hipMemcpyAsync(P.data(), c->d_scratch, sizeof(int64_t) * c->nranks, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (c->rank == root) {
    if (!merged) return fail(MC_ERR_INVALID, "root needs a merged batch");
    int64_t tot = 0;
    for (int64_t v : P) tot += v;
    if (tot != merged->P)
      return fail(MC_ERR_INVALID, "merged batch holds %lld padded points, ranks sent %lld", (long long)merged->P,
                  (long long)tot);
  }
  NCCLCHK(g_rccl.GroupStart());
  if (c->rank == root) {
    int64_t off = 0;
    for (int q = 0; q < c->nranks; ++q) {
      for (int col = 0; col < 4; ++col) {
        float* dst = merged->d_cols + col * merged->cap + off;
        if (P[q] == 0) continue;
        if (q == root) {
          if (hipMemcpyAsync(dst, local->d_cols + col * local->cap, P[q] * sizeof(float), hipMemcpyDeviceToDevice, s) !=
              hipSuccess) {
            g_rccl.GroupEnd();
            return fail(MC_ERR_HIP, "local copy failed");
          }
        } else {
          NCCLCHK(g_rccl.Recv(dst, (size_t)P[q], ncclFloat32, q, c->comm, s));
        }
      }
      off += P[q];
    }
  } else if (local->P > 0) {
    for (int col = 0; col < 4; ++col)
      NCCLCHK(g_rccl.Send(local->d_cols + col * local->cap, (size_t)local->P, ncclFloat32, root, c->comm, s));
  }
  NCCLCHK(g_rccl.GroupEnd());
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
