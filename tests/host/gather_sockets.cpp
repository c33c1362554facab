// gather_sockets.cpp — mcgather::run (csrc/gather.cpp, the sequence behind mc_comm_gather_batch) over
// host memory and Unix sockets between forked rank processes (tests/test_dist.py).
//
//   gather_sockets <dir>
//
// <dir>/meta.txt:  "world root" / "merged P C F counts..." / one "P C F counts..." line per rank;
// <dir>/shard_<q>.bin: rank q's C * P float32 blocked columns.  Every rank runs the sequence with its
// shard; the root writes <dir>/merged.bin (the merged batch's C * P values).  Exit status: 0 when every
// rank returned 0; per rank one line "rank q status s" on stdout (s = run()'s status, -1 bad plan).
#include <signal.h>
#include <sys/socket.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "gather.hpp"

namespace {

struct Desc {
  int64_t P = 0, C = 4, F = 0;
  std::vector<int64_t> counts;
};

Desc read_desc(std::istream& in) {
  Desc d;
  in >> d.P >> d.C >> d.F;
  d.counts.resize((size_t)d.F);
  for (auto& c : d.counts) in >> c;
  return d;
}

constexpr int kIoErr = -6;   // == MC_ERR_COMM

int write_all(int fd, const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n > 0) {
    const ssize_t k = ::write(fd, c, n);
    if (k <= 0) return kIoErr;
    c += k;
    n -= (size_t)k;
  }
  return 0;
}
int read_all(int fd, void* p, size_t n) {
  char* c = static_cast<char*>(p);
  while (n > 0) {
    const ssize_t k = ::read(fd, c, n);
    if (k <= 0) return kIoErr;
    c += k;
    n -= (size_t)k;
  }
  return 0;
}

// host-memory transport: fd[q] is this rank's socket to rank q
struct Sockets {
  int rank = 0, nranks = 1;
  std::vector<int> fd;
  std::vector<float> stage;
  int groups_open = 0;
};

mcgather::Transport socket_transport(Sockets* s) {
  mcgather::Transport T;
  T.self = s;
  T.nranks = s->nranks;
  T.rank = s->rank;
  T.allgather_i64 = [](void* p, const int64_t* mine, int n, int64_t* all) {
    Sockets* k = static_cast<Sockets*>(p);
    // plan words are small: every rank writes to every peer first, then reads (socket buffers hold them)
    for (int q = 0; q < k->nranks; ++q)
      if (q != k->rank)
        if (int r = write_all(k->fd[q], mine, sizeof(int64_t) * n)) return r;
    std::memcpy(all + (size_t)n * k->rank, mine, sizeof(int64_t) * n);
    for (int q = 0; q < k->nranks; ++q)
      if (q != k->rank)
        if (int r = read_all(k->fd[q], all + (size_t)n * q, sizeof(int64_t) * n)) return r;
    return 0;
  };
  T.group_start = [](void* p) { ++static_cast<Sockets*>(p)->groups_open; return 0; };
  T.group_end = [](void* p) {
    Sockets* k = static_cast<Sockets*>(p);
    return --k->groups_open == 0 ? 0 : kIoErr;
  };
  // blocking: a non-root rank only sends to the root, and the root receives every peer in turn
  T.send = [](void* p, const float* buf, int64_t n, int peer) {
    Sockets* k = static_cast<Sockets*>(p);
    return k->groups_open ? write_all(k->fd[peer], buf, sizeof(float) * (size_t)n) : kIoErr;
  };
  T.recv = [](void* p, float* buf, int64_t n, int peer) {
    Sockets* k = static_cast<Sockets*>(p);
    return k->groups_open ? read_all(k->fd[peer], buf, sizeof(float) * (size_t)n) : kIoErr;
  };
  T.stage = [](void* p, int64_t values, float** out) {
    Sockets* k = static_cast<Sockets*>(p);
    if ((int64_t)k->stage.size() < values) k->stage.assign((size_t)values, -7.0f);
    *out = k->stage.data();
    return 0;
  };
  T.copy = [](void*, float* d, const float* src, int64_t n) {
    std::memcpy(d, src, sizeof(float) * (size_t)n);
    return 0;
  };
  T.copy2d = [](void*, float* d, int64_t dp, const float* src, int64_t sp, int64_t w, int64_t rows) {
    for (int64_t r = 0; r < rows; ++r) std::memcpy(d + r * dp, src + r * sp, sizeof(float) * (size_t)w);
    return 0;
  };
  T.sync = [](void*) { return 0; };
  return T;
}

int rank_main(const std::string& dir, int rank, int world, int root, const Desc& merged, const Desc& mine,
              std::vector<int> fds) {
  std::vector<float> cols((size_t)(mine.C * mine.P));
  {
    std::ifstream f(dir + "/shard_" + std::to_string(rank) + ".bin", std::ios::binary);
    f.read(reinterpret_cast<char*>(cols.data()), (std::streamsize)(cols.size() * sizeof(float)));
    if (!f) return 90;
  }
  Sockets S;
  S.rank = rank;
  S.nranks = world;
  S.fd = std::move(fds);
  const mcgather::Transport T = socket_transport(&S);
  mcgather::Shard sh;
  sh.P = mine.P; sh.C = mine.C; sh.F = mine.F; sh.counts = mine.counts.data(); sh.cols = cols.data();
  std::vector<float> out;
  mcgather::Merged mg;
  if (rank == root && merged.P >= 0) {
    out.assign((size_t)(merged.C * merged.P), -9.0f);   // every value must be overwritten
    mg.P = merged.P; mg.C = merged.C; mg.F = merged.F; mg.counts = merged.counts.data(); mg.cols = out.data();
  }
  std::string msg;   // (a merged line with P < 0: the root passes no merged batch)
  const int r = mcgather::run(T, root, sh, rank == root && merged.P >= 0 ? &mg : nullptr, &msg);
  std::printf("rank %d status %d %s\n", rank, r, msg.c_str());
  std::fflush(stdout);
  if (r == 0 && rank == root) {
    std::ofstream f(dir + "/merged.bin", std::ios::binary);
    f.write(reinterpret_cast<const char*>(out.data()), (std::streamsize)(out.size() * sizeof(float)));
    if (!f) return 91;
  }
  return r == 0 ? 0 : (r == mcgather::kBadPlan ? 3 : 4);
}

}  // namespace

int main(int argc, char** argv) {
  if (argc != 2) {
    std::fprintf(stderr, "usage: gather_sockets <dir>\n");
    return 2;
  }
  signal(SIGPIPE, SIG_IGN);
  const std::string dir = argv[1];
  std::ifstream meta(dir + "/meta.txt");
  int world = 0, root = 0;
  meta >> world >> root;
  if (!meta || world < 1 || world > 64) return 2;
  const Desc merged = read_desc(meta);
  std::vector<Desc> shard((size_t)world);
  for (auto& d : shard) d = read_desc(meta);
  if (!meta) return 2;
  // one socket pair per rank pair
  std::vector<std::vector<int>> fd((size_t)world, std::vector<int>((size_t)world, -1));
  for (int i = 0; i < world; ++i)
    for (int j = i + 1; j < world; ++j) {
      int sv[2];
      if (socketpair(AF_UNIX, SOCK_STREAM, 0, sv) != 0) return 2;
      fd[i][j] = sv[0];
      fd[j][i] = sv[1];
    }
  std::vector<pid_t> pids;
  for (int r = 0; r < world; ++r) {
    const pid_t pid = fork();
    if (pid < 0) return 2;
    if (pid == 0) {
      for (int i = 0; i < world; ++i)
        for (int j = 0; j < world; ++j)
          if (i != r && fd[i][j] >= 0) close(fd[i][j]);
      const int code = rank_main(dir, r, world, root, merged, shard[(size_t)r], fd[(size_t)r]);
      std::fflush(stdout);
      _exit(code);
    }
    pids.push_back(pid);
  }
  for (auto& row : fd)
    for (int f : row)
      if (f >= 0) close(f);
  int bad = 0;
  for (size_t r = 0; r < pids.size(); ++r) {
    int st = 0;
    waitpid(pids[r], &st, 0);
    const int code = WIFEXITED(st) ? WEXITSTATUS(st) : 128 + WTERMSIG(st);
    if (code) {
      std::printf("rank %zu exit %d\n", r, code);
      bad = bad ? bad : code;
    }
  }
  return bad;
}
