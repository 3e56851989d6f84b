/*
 * hydra_host.h -- C entry points of libhydra_host.so, the C++ host runtime (include/hydra/allreduce.h)
 * that mirrors hydra/Gloo's new_allreduce_ring and bew_allreduce_a over loopback TCP with the
 * per-segment reduction offloaded to the MI355X through include/hydra_hip.h.
 *
 * Ranks run as threads of the calling process, sharing an in-process store -- the reference's own
 * test harness (gloo/gloo/test/base_test.h:116-156).  Used by tests/ and bench.py.
 *
 * reducer: HYDRA_REDUCER_GPU  -> hydra_reduce_host (H2D -> gfx950 kernel -> D2H, synchronous)
 *          HYDRA_REDUCER_FN   -> the caller's function (CPU-side tests plug the oracle in here)
 *          HYDRA_REDUCER_GPU_PINNED -> GPU with pinned receive slots (Context scratch allocator);
 *                               with a pinned output every segment reduce is zero-copy
 *                               (hydra_host_bench allocates its output pinned itself)
 */
#ifndef HYDRA_HOST_H_
#define HYDRA_HOST_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void (*hydra_reduce_fn)(void* c, const void* a, const void* b, size_t n);
#define HYDRA_REDUCER_GPU 0
#define HYDRA_REDUCER_FN 1
#define HYDRA_REDUCER_GPU_PINNED 2
/* hydra_host_bench only: rank 0 reduces with HYDRA_REDUCER_GPU_PINNED, every other rank with
 * the caller's fn.  On a one-GPU box this gives rank 0 the PCIe link to itself, as BASELINE
 * config 3 (one MI355X per rank) would; rank 0's per-iteration times are the ones reported. */
#define HYDRA_REDUCER_GPU_PINNED_RANK0 3
#ifndef HYDRA_SPLIT_AA
#define HYDRA_SPLIT_AA 0 /* calculateElements_AA, pipeallreduce-a.h:296-376 (default) */
#define HYDRA_SPLIT_AG 1 /* calculateElements_AG, pipeallreduce-a.h:137-294 (ALLREDUCE_GLEX) */
#endif

/* gloo::allreduce on P thread-ranks.  in/out: P*nptr pointers [rank][ptr]; in == NULL is in
 * place (allreduce_test.cc:302-350).  algorithm: 0/1 RING, 2 BCUBE (AllreduceOptions::Algorithm).
 * timeout_ms <= 0: context default (30 s). */
int hydra_host_allreduce_threads(int P, int nptr, int op, int dtype, size_t n, void** in,
                                 void** out, size_t max_segment, int algorithm, int reducer,
                                 hydra_reduce_fn fn, long timeout_ms, char* err, size_t errlen);

/* gloo::apipe_allreduce (bew_allreduce_a) on P thread-ranks with two loopback rails each.
 * in/out: P pointers each. */
int hydra_host_apipe_threads(int P, int dtype, size_t n, void** in, void** out, int table,
                             int reducer, hydra_reduce_fn fn, char* err, size_t errlen);

/* The reference benchmark bodies on P thread-ranks: config 1 = NewAllreduceBenchmark
 * (benchmark/main.cc:321-358), config 3 = aAllreduceBenchmark (main.cc:629-664).  Rank 0's
 * per-iteration wall time in ns goes to samples_ns[iters]. */
int hydra_host_bench(int config, int P, size_t n, int warmup, int iters, int reducer,
                     hydra_reduce_fn fn, double* samples_ns, char* err, size_t errlen);

void hydra_host_calculate_elements(int table, int P, size_t n, size_t* e1, size_t* e2);

/* Old-style gloo::AllreduceRing<T>::run() (allreduce_ring.h:20-125) on P thread-ranks, in place
 * on bufs ([rank][ptr]).  fn, when reducer == HYDRA_REDUCER_FN, has the
 * ReductionFunction<T>::Function shape void(T* x, const T* y, size_t n). dtype: float32, int32,
 * float64 (GPU or custom reducer), float16 (custom reducer only). */
typedef void (*hydra_inplace_fn)(void* x, const void* y, size_t n);
int hydra_host_allreduce_ring_old_threads(int P, int nptr, int dtype, size_t n, void** bufs,
                                          int reducer, hydra_inplace_fn fn, char* err,
                                          size_t errlen);

/* hydra::HipAllreduceRing<T, W> (gloo::CudaAllreduceRing<T, W>, cuda_allreduce_ring.cc) on P
 * thread-ranks over loopback TCP; dev_bufs ([rank][ptr]) are device pointers, in place.
 * workspace: HYDRA_WORKSPACE_HOST / _DEVICE; user_streams: pass caller streams (outputs async).
 * dtype: float32, int32, float64, int64. */
#define HYDRA_WORKSPACE_HOST 0
#define HYDRA_WORKSPACE_DEVICE 1
int hydra_host_hip_ring_threads(int P, int nptr, int dtype, size_t n, void** dev_bufs,
                                int workspace, int user_streams, char* err, size_t errlen);

/* hydra::HipAllreduceRingChunked<T, W> (gloo::CudaAllreduceRingChunked<T, W>,
 * cuda_allreduce_ring_chunked.cc), same arguments as hydra_host_hip_ring_threads. */
int hydra_host_hip_ring_chunked_threads(int P, int nptr, int dtype, size_t n, void** dev_bufs,
                                        int workspace, int user_streams, char* err,
                                        size_t errlen);

/* gloo::AllreduceRingChunked<T>::run() (allreduce_ring_chunked.h:20-248), same arguments. */
int hydra_host_allreduce_ring_chunked_threads(int P, int nptr, int dtype, size_t n, void** bufs,
                                              int reducer, hydra_inplace_fn fn, char* err,
                                              size_t errlen);

/* gloo::reduce (reduce.cc:21-262) to `root` on P thread-ranks.  in/out: P pointers each
 * (in == NULL: in place on out, reduce_test.cc:27-33).  Every rank's out is left as the
 * reference's schedule leaves it; only the root's is the reduction. */
int hydra_host_reduce_threads(int P, int op, int dtype, size_t n, void** in, void** out,
                              int root, size_t max_segment, int reducer, hydra_reduce_fn fn,
                              long timeout_ms, char* err, size_t errlen);

/* ReduceTest.TestTimeout (reduce_test.cc:91-108): root 0 of 2 alone, IoException text. */
int hydra_host_reduce_timeout_probe(long timeout_ms, char* what, size_t len);

/* AllreduceNewTest.TestTimeout (allreduce_test.cc:381-397): rank 0 of 2 times out; returns 0 and
 * the IoException text if it was raised. */
int hydra_host_timeout_probe(long timeout_ms, char* what, size_t len);
/* Slow-peer timeout probe: rank 0 times out, rank 1 sends `delay_ms` later; *intact = 1 when
 * the late bytes did not land in rank 0's refilled bucket (its context was poisoned). */
int hydra_host_slow_peer_probe(long timeout_ms, long delay_ms, size_t n, char* what, size_t len,
                               int* intact);

#ifdef __cplusplus
}
#endif
#endif /* HYDRA_HOST_H_ */
