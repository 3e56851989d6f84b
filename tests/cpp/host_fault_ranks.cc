// One rank of the host runtime's allreduce ring per PROCESS, looping until the transport fails:
// the process-per-rank fault tests of the reference (TransportMultiProcTest.IoErrors /
// IoTimeouts / UnboundIoErrors, gloo/gloo/test/transport_test.cc:44-240, on MultiProcTest,
// gloo/gloo/test/multiproc_test.{h,cc}) applied to the ring around the sum.  tests/test_fault.py
// starts P of these, lets them run, then SIGKILLs or SIGSTOPs rank 0 and checks how the others
// end: every survivor must leave with kExitWithIoException (10, multiproc_test.h:26), within
// half the timeout after a kill and at the timeout after a stop.
//
// Usage: host_fault_ranks RANK SIZE STORE_DIR N TIMEOUT_MS [bigsend | gpu]
// gpu (built with -DHYDRA_FAULT_GPU, tests/cpp/host_fault_ranks_gpu via hydra_amd/csrc/Makefile):
// the reducer is the gfx950 chunk-sum behind the drop-in Func (gloo_compat::hostSum<float>) and
// the ring's receive slots are pinned (gloo_compat::pinnedAlloc), the configuration the GPU host
// path runs in; a survivor must still leave with IoException, its GPU state released by exit.
// bigsend (SIZE 2): rank 0 never receives; rank 1 sends N floats to it, more than the socket
// buffers hold, so its writer blocks inside the write until rank 0 is killed -- the write then
// fails (EPIPE / ECONNRESET), which must surface as IoException, not as SIGPIPE.
// Rendezvous over a FileStore (processes) and a loopback TCP full mesh; a plain CPU sum is the
// reducer (the GPU reducer's failure paths are the GPU tests'); stdout "ready" after the first
// completed allreduce with the expected result.
#include <unistd.h>

#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "hydra/allreduce.h"
#ifdef HYDRA_FAULT_GPU
#include "hydra/gloo_reduce.h"
#endif

namespace {
constexpr int kExitWithIoException = 10;  // gloo/gloo/test/multiproc_test.h:26

void sum_f32(void* c, const void* a, const void* b, size_t n) {
  for (size_t i = 0; i < n; i++)
    static_cast<float*>(c)[i] = static_cast<const float*>(a)[i] + static_cast<const float*>(b)[i];
}
}  // namespace

int main(int argc, char** argv) {
  if (argc < 6) return 2;
  const int rank = std::atoi(argv[1]), size = std::atoi(argv[2]);
  const std::string dir = argv[3];
  const size_t n = (size_t)std::atoll(argv[4]);
  const long timeout_ms = std::atol(argv[5]);
  // SIGPIPE keeps its default action here: a write to a dead peer must come back as an error
  // from the library (MSG_NOSIGNAL), not kill this process.
  try {
    hydra::FileStore store(dir);
    auto ctx = std::make_shared<hydra::Context>(rank, size);
    ctx->setTimeout(std::chrono::milliseconds(timeout_ms));
    ctx->connectFullMesh(store, "127.0.0.1");
    const bool gpu = argc > 6 && std::string(argv[6]) == "gpu";
#ifdef HYDRA_FAULT_GPU
    if (gpu)
      ctx->setScratchAllocator({&hydra::gloo_compat::pinnedAlloc, &hydra::gloo_compat::pinnedFree});
#else
    if (gpu) {
      std::fprintf(stderr, "built without HYDRA_FAULT_GPU\n");
      return 2;
    }
#endif
    std::vector<float> buf(n);
    if (argc > 6 && std::string(argv[6]) == "bigsend") {
      std::printf("ready\n");
      std::fflush(stdout);
      if (rank == 0)
        for (;;) pause();  // holds its sockets open, reads nothing, until it is killed
      auto ub = ctx->createUnboundBuffer(buf.data(), n * sizeof(float));
      ub->send(0, 1, 0, n * sizeof(float));
      ub->waitSend(std::chrono::milliseconds(timeout_ms));
      std::fprintf(stderr, "rank %d: the send to a rank that reads nothing completed\n", rank);
      return 5;
    }
    for (long it = 0;; it++) {
      for (size_t i = 0; i < n; i++) buf[i] = (float)rank;
      hydra::AllreduceOptions opts(ctx);
      opts.setAlgorithm(hydra::AllreduceOptions::RING);
      opts.setOutput(buf.data(), n);
#ifdef HYDRA_FAULT_GPU
      if (gpu)
        opts.setReduceFunction(hydra::gloo_compat::hostSum<float>());
      else
#endif
        opts.setReduceFunction(&sum_f32);
      opts.setTag((uint32_t)(it & 0xffff));
      hydra::allreduce(opts);
      if (it == 0) {
        const float want = (float)(size * (size - 1) / 2);
        for (size_t i = 0; i < n; i++)
          if (buf[i] != want) {
            std::fprintf(stderr, "rank %d: wrong result %g at %zu (want %g)\n", rank, buf[i], i,
                         want);
            return 3;
          }
        std::printf("ready\n");
        std::fflush(stdout);
      }
    }
  } catch (const hydra::IoException& e) {
    std::fprintf(stderr, "rank %d: IoException: %s\n", rank, e.what());
    return kExitWithIoException;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "rank %d: %s\n", rank, e.what());
    return 4;
  }
}
