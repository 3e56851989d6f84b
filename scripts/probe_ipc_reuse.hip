// probe_ipc_reuse.hip -- does an IPC import see the RIGHT memory when the exporter frees an
// allocation and gets a new one at the same address?  Two processes on device 0 (forked before
// any HIP call), handles over pipes.  Each round: A allocates, fills with round-specific bytes,
// exports; B opens, reads, checks, closes; A frees.  Prints whether handle bytes / addresses
// repeated and whether B ever read a previous round's bytes.
#include <hip/hip_runtime.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      _exit(3);                                                                 \
    }                                                                           \
  } while (0)

static void wr(int fd, const void* p, size_t n) {
  if (write(fd, p, n) != (ssize_t)n) _exit(4);
}
static void rd(int fd, void* p, size_t n) {
  size_t got = 0;
  while (got < n) {
    ssize_t k = read(fd, (char*)p + got, n - got);
    if (k <= 0) _exit(5);
    got += (size_t)k;
  }
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 8;
  const size_t bytes0 = argc > 2 ? (size_t)atoll(argv[2]) : (4u << 20);
  const int mode = argc > 3 ? atoi(argv[3]) : 0;  // 1: peer_algo's pattern (sizes cycle, + uncached sig)
  const size_t cyc[3] = {4000012, 1333364, 20012};
  auto size_of = [&](int r) { return mode ? cyc[r % 3] : bytes0; };
  const size_t sig_bytes = 8 * 1024 * 4 + 64;
  int a2b[2], b2a[2];
  if (pipe(a2b) || pipe(b2a)) return 2;
  pid_t pid = fork();
  if (pid == 0) {  // B: importer
    CK(hipSetDevice(0));
    std::vector<unsigned char> h(4u << 20);
    int stale = 0, wrong = 0;
    for (int r = 0; r < rounds; r++) {
      const size_t bytes = size_of(r);
      hipIpcMemHandle_t hd, hs;
      rd(a2b[0], &hd, sizeof(hd));
      rd(a2b[0], &hs, sizeof(hs));
      void* m = nullptr;
      void* ms = nullptr;
      if (mode) {
        hipError_t e = hipIpcOpenMemHandle(&ms, hs, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) std::printf("B round %d: sig open failed: %s\n", r, hipGetErrorString(e));
      }
      {
        hipError_t e = hipIpcOpenMemHandle(&m, hd, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) {
          std::printf("B round %d: bucket open failed: %s\n", r, hipGetErrorString(e));
          wrong++;
          if (ms) CK(hipIpcCloseMemHandle(ms));
          char ack = 1;
          wr(b2a[1], &ack, 1);
          continue;
        }
      }
      CK(hipMemcpy(h.data(), m, bytes, hipMemcpyDeviceToHost));
      int bad = 0, prev = 0;
      for (size_t i = 0; i < bytes; i += 4096) {
        if (h[i] != (unsigned char)(r + 1)) bad++;
        if (r > 0 && h[i] == (unsigned char)r) prev++;
      }
      std::printf("B round %d: %zu B mapped at %p, %d/%zu pages wrong (%d hold round %d's bytes)\n",
                  r, bytes, m, bad, (bytes + 4095) / 4096, prev, r - 1);
      wrong += bad != 0;
      stale += prev != 0;
      CK(hipIpcCloseMemHandle(m));
      if (ms) CK(hipIpcCloseMemHandle(ms));
      char ack = 1;
      wr(b2a[1], &ack, 1);
    }
    std::printf("B: %d of %d rounds read wrong bytes, %d saw the previous allocation\n", wrong,
                rounds, stale);
    fflush(stdout);
    _exit(wrong ? 1 : 0);
  }
  // A: exporter
  CK(hipSetDevice(0));
  hipIpcMemHandle_t prevh;
  void* prevp = nullptr;
  for (int r = 0; r < rounds; r++) {
    const size_t bytes = size_of(r);
    void* p = nullptr;
    void* sg = nullptr;
    if (mode) {
      CK(hipExtMallocWithFlags(&sg, sig_bytes, hipDeviceMallocUncached));
      CK(hipMemset(sg, 0, sig_bytes));
    }
    CK(hipMalloc(&p, bytes));
    CK(hipMemset(p, r + 1, bytes));
    CK(hipDeviceSynchronize());
    hipIpcMemHandle_t hd, hs{};
    // export through the allocation base the way hydra_peer_register does
    void* base = nullptr;
    size_t range = 0;
    CK(hipMemGetAddressRange(&base, &range, p));
    if (base != p || range < bytes)
      std::printf("A round %d: hipMemGetAddressRange(%p) = [%p, +%zu) for a %zu-byte allocation\n",
                  r, p, base, range, bytes);
    {
      hipError_t e = hipIpcGetMemHandle(&hd, base);
      if (e != hipSuccess) {
        std::printf("A round %d: hipIpcGetMemHandle(base) failed: %s; retry on p\n", r,
                    hipGetErrorString(e));
        CK(hipIpcGetMemHandle(&hd, p));
      }
    }
    if (mode) CK(hipIpcGetMemHandle(&hs, sg));
    std::printf("A round %d: alloc %p%s, handle %s\n", r, p, (r && p == prevp) ? " (same VA)" : "",
                (r && !std::memcmp(&hd, &prevh, sizeof(hd))) ? "IDENTICAL to previous" : "new");
    fflush(stdout);
    wr(a2b[1], &hd, sizeof(hd));
    wr(a2b[1], &hs, sizeof(hs));
    char ack;
    rd(b2a[0], &ack, 1);
    prevh = hd;
    prevp = p;
    CK(hipFree(p));
    if (sg) CK(hipFree(sg));
  }
  int st = 0;
  waitpid(pid, &st, 0);
  const int rc = WIFEXITED(st) ? WEXITSTATUS(st) : 9;
  std::printf("probe_ipc_reuse: %s\n", rc == 0 ? "ok" : "STALE/WRONG IMPORT");
  return rc;
}
