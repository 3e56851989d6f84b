// peer_algo.cc -- hydra::PeerAllreduce<T> (include/hydra/peer_allreduce.h) from C++: P
// processes (forked before any GPU call, all on device 0), rendezvous through the host
// runtime's FileStore + TCP full mesh, which also carries the IPC handle all-gather.  Each
// rank allreduces integer-valued buckets that change every iteration and checks every word
// exactly (small-integer sums are exact in any order), for fp32 (default geometry) and int32
// (maxSegmentSize 4096, ragged n, one-shot and two-shot).
//
// Usage: peer_algo P n store_dir   (exit 0 = every rank exact)
#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "hydra/peer_allreduce.h"

namespace {

// `dev` outlives every group that registers it: freeing a registered allocation and
// registering a new one in the same process intermittently gave a peer a mapping of the wrong
// memory on ROCm 7.2, so buckets are allocated once per process, as a
// framework's caching allocator keeps them.
template <typename T>
int check_type(const std::shared_ptr<hydra::Context>& ctx, void* dev, size_t n, int algo,
               size_t ms) {
  const int P = ctx->size, r = ctx->rank;

  int bad = 0;
  {
    hydra::PeerAllreduce<T> ar(ctx, static_cast<T*>(dev), n, nullptr, algo, ms);
    std::vector<T> h(n);
    for (int it = 0; it < 4; it++) {
      for (size_t i = 0; i < n; i++) h[i] = (T)((i % 1000) * (size_t)(r + 1) + it * (r + 2));
      hydra::gloo_compat::enforce(hydra_memcpy(dev, h.data(), n * sizeof(T)));
      ar.run();
      hydra::gloo_compat::enforce(hydra_memcpy(h.data(), dev, n * sizeof(T)));
      int b0 = 0;
      size_t first = n;
      for (size_t i = 0; i < n; i++) {
        const T want = (T)((i % 1000) * (size_t)(P * (P + 1) / 2) + it * (P * (P + 3) / 2));
        if (h[i] != want) {
          if (!b0) first = i;
          b0++;
        }
      }
      if (b0)
        std::printf("rank %d: %s n=%zu algo=%d it=%d: %d wrong, first at %zu (got %g want %g)\n",
                    r, sizeof(T) == 4 && (T)0.5 ? "f32" : "i32", n, algo, it, b0, first,
                    (double)h[first],
                    (double)(T)((first % 1000) * (size_t)(P * (P + 1) / 2) + it * (P * (P + 3) / 2)));
      bad += b0;
    }
  }
  return bad;
}

int run(int rank, int P, size_t n, const std::string& dir) {
  try {
    hydra::FileStore store(dir);
    auto ctx = std::make_shared<hydra::Context>(rank, P);
    ctx->connectFullMesh(store, "127.0.0.1");
    const size_t n2 = n / 3 + 7, n3 = 5003;
    void *d1 = nullptr, *d2 = nullptr, *d3 = nullptr;
    hydra::gloo_compat::enforce(hydra_malloc(0, n * sizeof(float), &d1));
    hydra::gloo_compat::enforce(hydra_malloc(0, n2 * sizeof(int32_t), &d2));
    hydra::gloo_compat::enforce(hydra_malloc(0, n3 * sizeof(int32_t), &d3));
    int bad = check_type<float>(ctx, d1, n, HYDRA_PEER_AUTO, 0);
    bad += check_type<int32_t>(ctx, d2, n2, HYDRA_PEER_TWO_SHOT, 4096);
    bad += check_type<int32_t>(ctx, d3, n3, HYDRA_PEER_ONE_SHOT, 4096);
    // ~PeerAllreduce was collective: no rank maps these any more
    hydra_free(d1);
    hydra_free(d2);
    hydra_free(d3);
    std::printf("rank %d: mismatches=%d\n", rank, bad);
    std::fflush(stdout);
    return bad ? 1 : 0;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "rank %d: %s\n", rank, e.what());
    return 2;
  }
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 4) return 2;
  const int P = std::atoi(argv[1]);
  const size_t n = (size_t)std::atoll(argv[2]);
  const std::string dir = argv[3];
  std::vector<pid_t> pids;
  for (int r = 0; r < P; r++) {
    pid_t pid = fork();
    if (pid < 0) return 2;
    if (pid == 0) _exit(run(r, P, n, dir));
    pids.push_back(pid);
  }
  int rc = 0;
  for (pid_t pid : pids) {
    int st = 0;
    waitpid(pid, &st, 0);
    if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) rc = 1;
  }
  std::printf("peer_algo P=%d n=%zu: %s\n", P, n, rc ? "FAIL" : "ok");
  return rc;
}
