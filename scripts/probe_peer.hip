// probe_peer.hip -- de-risk probe for the peer-access allreduce on a one-GPU box.
// Two processes (forked before any HIP call) on device 0 share a data buffer and an uncached
// signal area by hipIpc handles, then run peer_barrier + a peer read in one kernel each.
// Checks: IPC open on the same device across processes, uncached-memory IPC, concurrent
// progress of two processes' spinning kernels, barrier round-trip latency.
// Build: hipcc --offload-arch=gfx950 -O3 -I../hydra_amd/csrc probe_peer.hip -o probe_peer
#include <hip/hip_runtime.h>
#include <sys/socket.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "peer_sync.h"

using namespace hydra;

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      fprintf(stderr, "rank %d: %s failed: %s\n", rank, #x, hipGetErrorString(e));  \
      return 2;                                                                       \
    }                                                                                 \
  } while (0)

__global__ void k_step(float* out, const float* mine, const float* peer, size_t n, PeerSigPtrs sig,
                       int P, int rank, uint32_t epoch, uint32_t* err) {
  if (!peer_barrier(sig, P, rank, epoch, 200000000ull, err, 1)) return;
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    out[i] = mine[i] + peer[i];
  peer_barrier(sig, P, rank, epoch + 1, 200000000ull, err, 2);
}

__global__ void k_bar(PeerSigPtrs sig, int P, int rank, uint32_t epoch0, int iters,
                      uint32_t* err) {
  for (int k = 0; k < iters; k++)
    if (!peer_barrier(sig, P, rank, epoch0 + k, 200000000ull, err, 3)) return;
}

__global__ void k_fill(float* p, size_t n, float v) {
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    p[i] = v;
}

static int xfer(int fd, void* buf, size_t len, bool send_) {
  char* b = (char*)buf;
  size_t done = 0;
  while (done < len) {
    ssize_t r = send_ ? write(fd, b + done, len - done) : read(fd, b + done, len - done);
    if (r <= 0) return -1;
    done += r;
  }
  return 0;
}

static int run(int rank, int fd) {
  const int P = 2;
  const size_t n = 4 << 20;
  CK(hipSetDevice(0));
  float *data, *out;
  PeerSignals* sig;
  uint32_t* err;
  CK(hipMalloc(&data, n * 4));
  CK(hipMalloc(&out, n * 4));
  CK(hipExtMallocWithFlags((void**)&sig, sizeof(PeerSignals), hipDeviceMallocUncached));
  CK(hipMemset(sig, 0, sizeof(PeerSignals)));
  CK(hipHostMalloc(&err, 4, hipHostMallocMapped | hipHostMallocCoherent));
  *err = 0;
  hipLaunchKernelGGL(k_fill, dim3(256), dim3(256), 0, 0, data, n, (float)(rank + 1));
  CK(hipDeviceSynchronize());
  hipIpcMemHandle_t hd, hs, pd, ps;
  CK(hipIpcGetMemHandle(&hd, data));
  CK(hipIpcGetMemHandle(&hs, sig));
  if (xfer(fd, &hd, sizeof hd, true) || xfer(fd, &hs, sizeof hs, true) ||
      xfer(fd, &pd, sizeof pd, false) || xfer(fd, &ps, sizeof ps, false)) {
    fprintf(stderr, "rank %d: handle exchange failed\n", rank);
    return 2;
  }
  void *peer_data, *peer_sig;
  CK(hipIpcOpenMemHandle(&peer_data, pd, hipIpcMemLazyEnablePeerAccess));
  CK(hipIpcOpenMemHandle(&peer_sig, ps, hipIpcMemLazyEnablePeerAccess));
  PeerSigPtrs sp{};
  sp.p[rank] = sig;
  sp.p[1 - rank] = (PeerSignals*)peer_sig;
  hipLaunchKernelGGL(k_step, dim3(16), dim3(256), 0, 0, out, data, (const float*)peer_data, n, sp,
                     P, rank, 1u, err);
  CK(hipDeviceSynchronize());
  std::vector<float> h(n);
  CK(hipMemcpy(h.data(), out, n * 4, hipMemcpyDeviceToHost));
  size_t bad = 0;
  for (size_t i = 0; i < n; i++) bad += h[i] != 3.0f;
  printf("rank %d: step err=%u mismatches=%zu\n", rank, *err, bad);
  // barrier latency: 2000 back-to-back barriers in one kernel, 1 and 16 workgroups
  for (int g : {1, 16}) {
    auto t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(k_bar, dim3(g), dim3(256), 0, 0, sp, P, rank, 10u + (g == 16 ? 5000u : 0u),
                       2000, err);
    CK(hipDeviceSynchronize());
    double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0)
                    .count();
    printf("rank %d: %d wg x 2000 barriers: %.2f us per barrier, err=%u\n", rank, g, us / 2000,
           *err);
  }
  CK(hipIpcCloseMemHandle(peer_data));
  CK(hipIpcCloseMemHandle(peer_sig));
  char c = 0;
  xfer(fd, &c, 1, true);  // keep own memory alive until the peer closed its mappings
  xfer(fd, &c, 1, false);
  return (bad || *err) ? 1 : 0;
}

int main() {
  int sv[2];
  if (socketpair(AF_UNIX, SOCK_STREAM, 0, sv)) return 2;
  pid_t pid = fork();
  if (pid < 0) return 2;
  if (pid == 0) {
    close(sv[0]);
    _exit(run(1, sv[1]));
  }
  close(sv[1]);
  int rc = run(0, sv[0]);
  int st = 0;
  waitpid(pid, &st, 0);
  int crc = WIFEXITED(st) ? WEXITSTATUS(st) : 100;
  printf("parent rc=%d child rc=%d\n", rc, crc);
  return rc || crc;
}
