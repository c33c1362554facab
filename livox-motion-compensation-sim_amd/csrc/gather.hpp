// gather.hpp — the merged-cloud gather's call sequence (LMC:887-889 np.vstack of the frame-ordered
// shards), written once against a table of transport primitives.
//
// comm.cpp runs it over RCCL (device buffers, xGMI): mc_comm_gather_batch.  tests/host/gather_sockets.cpp
// runs the same code over host sockets between forked processes (worlds 2..8 on the CPU, under
// AddressSanitizer + UndefinedBehaviorSanitizer), so the sequence — plan all-gather, frame-hash
// check, grouped send / receive, finishing copies — has run with peers before any multi-GPU node.
// Plain C++ (no HIP).
#pragma once
#include <cstdint>
#include <string>

namespace mcgather {

// one rank's shard: P padded points of C columns per 256-point block (blocked CSR), F frames
struct Shard {
  int64_t P = 0, C = 4, F = 0;
  const int64_t* counts = nullptr;   // F frame sizes
  const float* cols = nullptr;       // C * P values
};
// the root's merged batch: its frames must be the rank-ordered concatenation of the shards' frames
struct Merged {
  int64_t P = 0, C = 4, F = 0;
  const int64_t* counts = nullptr;
  float* cols = nullptr;
};

// Transport primitives; each returns 0 or a status of its own (passed back unchanged by run).
// Buffers are the transport's memory (device memory for RCCL, host memory for sockets).
struct Transport {
  void* self = nullptr;
  int nranks = 1, rank = 0;
  // every rank's n words, rank-ordered into all (n * nranks); synchronous
  int (*allgather_i64)(void* self, const int64_t* mine, int n, int64_t* all) = nullptr;
  int (*group_start)(void* self) = nullptr;
  int (*group_end)(void* self) = nullptr;
  int (*send)(void* self, const float* buf, int64_t n, int peer) = nullptr;
  int (*recv)(void* self, float* buf, int64_t n, int peer) = nullptr;
  // a staging area of >= values floats (grow-only, owned by the transport)
  int (*stage)(void* self, int64_t values, float** out) = nullptr;
  int (*copy)(void* self, float* dst, const float* src, int64_t n) = nullptr;
  int (*copy2d)(void* self, float* dst, int64_t dpitch, const float* src, int64_t spitch, int64_t width,
                int64_t rows) = nullptr;
  int (*sync)(void* self) = nullptr;   // everything queued has completed
};

// words per rank in the plan all-gather: padded length, columns, merged padded length, merged
// columns (root), frames, frame-count hash, merged frames, merged frame-count hash (root)
constexpr int kPlanWords = 8;
constexpr int kBadPlan = -1;   // == MC_ERR_INVALID

// The gather to `root`: every rank calls it with its shard; the root also passes the merged batch
// (others nullptr).  All ranks agree on the plan before any data moves and reject a bad one
// together.  Returns 0, kBadPlan (msg set), or the first failing primitive's status.
int run(const Transport& T, int root, const Shard& local, const Merged* merged, std::string* msg);

}  // namespace mcgather
