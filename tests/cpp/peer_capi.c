/* peer_capi.c -- the peer-access allreduce driven from plain C through include/hydra_hip.h only
 * (no HIP headers, no Python): P processes forked before any GPU call, handle blobs exchanged
 * over pipes -- the way a C/C++ caller such as the reference's benchmark would wire it up with
 * its own rendezvous channel.  Every rank checks its result against the
 * reference ring's value on integer-valued fp32 inputs (exact in any order): sum over ranks.
 *
 * Usage: peer_capi P n  (all ranks on device 0; exit 0 = every rank bit-exact) */
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <unistd.h>

#include "hydra_hip.h"

#define MAXP 8
static int up[MAXP][2], down[MAXP][2]; /* rank -> parent, parent -> rank */

static int xfer(int fd, void* buf, size_t len, int wr) {
  char* b = (char*)buf;
  while (len) {
    ssize_t r = wr ? write(fd, b, len) : read(fd, b, len);
    if (r <= 0) return -1;
    b += r;
    len -= (size_t)r;
  }
  return 0;
}

/* all-gather of one blob through the parent */
static int gather(int rank, const void* mine, void* all) {
  if (xfer(up[rank][1], (void*)mine, HYDRA_PEER_HANDLE_BYTES, 1)) return -1;
  return xfer(down[rank][0], all, (size_t)MAXP * HYDRA_PEER_HANDLE_BYTES, 0);
}

#define CK(x)                                                             \
  do {                                                                    \
    if ((x) != 0) {                                                       \
      fprintf(stderr, "rank %d: %s: %s\n", rank, #x, hydra_last_error()); \
      return 2;                                                           \
    }                                                                     \
  } while (0)

static int run(int rank, int P, size_t n) {
  char sig[HYDRA_PEER_HANDLE_BYTES], h[HYDRA_PEER_HANDLE_BYTES];
  char* all = calloc(MAXP, HYDRA_PEER_HANDLE_BYTES);
  float* host = malloc(n * sizeof(float));
  void* buf = NULL;
  hydra_peer_t peer = NULL;
  hydra_stream_t st = NULL;
  size_t i;
  int bad = 0, err = 0, it;
  for (i = 0; i < n; i++) host[i] = (float)((i % 1000) * (size_t)(rank + 1));
  CK(hydra_peer_create(P, rank, 0, &peer, sig));
  if (gather(rank, sig, all)) return 3;
  CK(hydra_peer_connect(peer, all));
  CK(hydra_malloc(0, n * sizeof(float), &buf));
  CK(hydra_stream_create(0, &st));
  CK(hydra_peer_register(peer, buf, n * sizeof(float), h));
  if (gather(rank, h, all)) return 3;
  CK(hydra_peer_open(peer, buf, n * sizeof(float), all));
  for (it = 0; it < 3; it++) {
    CK(hydra_memcpy(buf, host, n * sizeof(float)));
    CK(hydra_peer_allreduce(peer, it == 2 ? HYDRA_PEER_ONE_SHOT : HYDRA_PEER_TWO_SHOT, HYDRA_SUM,
                            HYDRA_FLOAT32, 0, buf, n, 0, st));
    CK(hydra_stream_synchronize(st));
  }
  CK(hydra_memcpy(host, buf, n * sizeof(float)));
  CK(hydra_peer_error(peer, &err));
  for (i = 0; i < n; i++)
    bad += host[i] != (float)((i % 1000) * (size_t)(P * (P + 1) / 2));
  /* collective teardown (hydra_hip.h): detach, barrier, then destroy and free */
  CK(hydra_peer_detach(peer));
  if (gather(rank, h, all)) return 3;
  CK(hydra_peer_destroy(peer));
  CK(hydra_free(buf));
  CK(hydra_stream_destroy(st));
  printf("rank %d: mismatches=%d err=%d\n", rank, bad, err);
  fflush(stdout);
  free(all);
  free(host);
  return (bad || err) ? 1 : 0;
}

int main(int argc, char** argv) {
  int P = argc > 1 ? atoi(argv[1]) : 2, r, rc = 0, round;
  size_t n = argc > 2 ? (size_t)atoll(argv[2]) : 1000003;
  pid_t pid[MAXP];
  if (P < 1 || P > MAXP) return 2;
  signal(SIGPIPE, SIG_IGN); /* a dead rank must not kill the relay */
  for (r = 0; r < P; r++)
    if (pipe(up[r]) || pipe(down[r])) return 2;
  for (r = 0; r < P; r++) {
    pid[r] = fork();
    if (pid[r] < 0) return 2;
    if (pid[r] == 0) {
      int s;
      for (s = 0; s < P; s++) { /* keep only this rank's two ends: a dead rank reads as EOF */
        close(up[s][0]);
        close(down[s][1]);
        if (s != r) {
          close(up[s][1]);
          close(down[s][0]);
        }
      }
      _exit(run(r, P, n));
    }
  }
  for (r = 0; r < P; r++) {
    close(up[r][1]);
    close(down[r][0]);
  }
  /* parent: relay three all-gathers (signal areas, bucket handles, final fence) */
  for (round = 0; round < 3; round++) {
    char* all = calloc(MAXP, HYDRA_PEER_HANDLE_BYTES);
    for (r = 0; r < P; r++)
      if (xfer(up[r][0], all + (size_t)r * HYDRA_PEER_HANDLE_BYTES, HYDRA_PEER_HANDLE_BYTES, 0))
        break;
    for (r = 0; r < P; r++) (void)xfer(down[r][1], all, (size_t)MAXP * HYDRA_PEER_HANDLE_BYTES, 1);
    free(all);
  }
  for (r = 0; r < P; r++) {
    int s = 0;
    waitpid(pid[r], &s, 0);
    if (!WIFEXITED(s) || WEXITSTATUS(s) != 0) rc = 1;
  }
  printf("peer_capi P=%d n=%zu: %s\n", P, n, rc ? "FAIL" : "ok");
  return rc;
}
