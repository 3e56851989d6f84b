/*
 * hydra_host_extra.h -- OUT OF SCOPE, opt-in: C drivers of the other old-style Algorithm-API
 * classes (include/hydra/allreduce_extra.h, include/hydra/hip_allreduce_extra.h; SURVEY.md §2
 * "Other Gloo collectives"), in libhydra_host_extra.so.  Same conventions as hydra_host.h.
 * Only the opt-in tests (pytest marker `extra`, HYDRA_EXTRA_TESTS=1) load it.
 */
#ifndef HYDRA_HOST_EXTRA_H_
#define HYDRA_HOST_EXTRA_H_

#include "hydra_host.h"

#ifdef __cplusplus
extern "C" {
#endif

/* hydra::HipAllreduceHalvingDoubling<T, W> (gloo::CudaAllreduceHalvingDoubling<T, W>,
 * cuda_allreduce_halving_doubling.cc), same arguments as hydra_host_hip_ring_threads. */
int hydra_host_hip_halving_doubling_threads(int P, int nptr, int dtype, size_t n,
                                            void** dev_bufs, int workspace, int user_streams,
                                            char* err, size_t errlen);

/* gloo::AllreduceHalvingDoubling<T>::run() (allreduce_halving_doubling.h:37-358), same
 * arguments as hydra_host_allreduce_ring_old_threads. */
int hydra_host_allreduce_halving_doubling_threads(int P, int nptr, int dtype, size_t n,
                                                  void** bufs, int reducer, hydra_inplace_fn fn,
                                                  char* err, size_t errlen);

/* Old-style gloo::AllreduceBcube<T>::run() (allreduce_bcube.h:255-691, base 2; P must be a
 * power of two), same arguments as hydra_host_allreduce_ring_old_threads. */
int hydra_host_allreduce_bcube_old_threads(int P, int nptr, int dtype, size_t n, void** bufs,
                                           int reducer, hydra_inplace_fn fn, char* err,
                                           size_t errlen);

/* gloo::AllreduceLocal<T>::run() (allreduce_local.cc:28-38): each rank's pointers only, same
 * arguments as hydra_host_allreduce_ring_old_threads. */
int hydra_host_allreduce_local_threads(int P, int nptr, int dtype, size_t n, void** bufs,
                                       int reducer, hydra_inplace_fn fn, char* err,
                                       size_t errlen);

/* hydra::HipAllreduceLocal<T> (gloo::CudaAllreduceLocal<T>, cuda_allreduce_local.cc), same
 * arguments as hydra_host_hip_ring_threads (workspace unused). */
int hydra_host_hip_local_threads(int P, int nptr, int dtype, size_t n, void** dev_bufs,
                                 int workspace, int user_streams, char* err, size_t errlen);

/* hydra::HipAllreduceBcube<T, W> (gloo::CudaAllreduceBcube<T, W>, cuda_allreduce_bcube.cc; P a
 * power of two), same arguments as hydra_host_hip_ring_threads. */
int hydra_host_hip_bcube_threads(int P, int nptr, int dtype, size_t n, void** dev_bufs,
                                 int workspace, int user_streams, char* err, size_t errlen);

#ifdef __cplusplus
}
#endif
#endif /* HYDRA_HOST_EXTRA_H_ */
