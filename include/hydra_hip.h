/*
 * hydra_hip.h -- C-ABI of the MI355X (gfx950) bucket-reduction hot path.
 *
 * libhydra_hip.so replaces the element-wise reduction that hydra/Gloo folds into every arriving
 * ring segment (new_allreduce_ring / bew_allreduce_a).  Plain C: pointers, sizes, ints; no HIP or
 * torch types in any signature (streams are opaque `hydra_stream_t` = hipStream_t).
 *
 * Every entry point returns 0 (HYDRA_OK) or a hydra_status_t; the message of the last failure on
 * the calling thread is hydra_last_error().  The C++ shim include/hydra/gloo_reduce.h turns
 * non-zero codes into exceptions, matching the reference's GLOO_ENFORCE -> gloo::EnforceNotMet
 * (gloo/gloo/common/logging.h:21,42) error model.
 *
 * Reference interfaces replaced (file:line under /root/reference):
 *   hydra_reduce / hydra_chunk_sum
 *       gloo::sum<T>(void* c, const void* a, const void* b, size_t n)  gloo/gloo/math.h:15-23
 *       gloo::product/max/min<T>                                        gloo/gloo/math.h:30-73
 *       the AllreduceOptions::Func plug-point it is bound to            gloo/gloo/allreduce.h:36,179-181
 *       (called at gloo/gloo/allreduce.cc:301-305 ring, :61-80 local reduce, :615-621 bcube)
 *       and cudaSum<T>(T* dst, const T* src, size_t n, stream)          gloo/gloo/cuda.cu:315-336
 *       as CudaReductionFunction<T>'s device function                    gloo/gloo/cuda.h:286-350
 *   hydra_reduce_host / hydra_chunk_sum_host
 *       the same gloo::sum<T> contract on HOST buffers (synchronous, like the reference), the form
 *       the ring actually hands over: c = out[0]+recvOffset, b = tmp scratch (allreduce.cc:301-305)
 *   hydra_acc_bf16_f32
 *       no reference counterpart: fp32 accumulate of a bf16 bucket (BASELINE config 5)
 *   hydra_ring_plan
 *       segment geometry of ring()                                      gloo/gloo/allreduce.cc:199-221
 */
#ifndef HYDRA_HIP_H_
#define HYDRA_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HYDRA_ABI_VERSION 2

typedef enum {
  HYDRA_INT8 = 0,
  HYDRA_UINT8 = 1,
  HYDRA_INT32 = 2,
  HYDRA_UINT32 = 3,
  HYDRA_INT64 = 4,
  HYDRA_UINT64 = 5,
  HYDRA_FLOAT32 = 6,
  HYDRA_FLOAT64 = 7,
  HYDRA_FLOAT16 = 8,  /* gloo::float16 semantics, incl. its store quirk */
  HYDRA_BFLOAT16 = 9  /* fp32 compute, RNE back to bf16 (no reference counterpart) */
} hydra_dtype_t;

typedef enum { HYDRA_SUM = 0, HYDRA_PRODUCT = 1, HYDRA_MAX = 2, HYDRA_MIN = 3 } hydra_op_t;

#define HYDRA_ACC_F32 1 /* flag: bf16 data, fp32 accumulation, one rounding */
/* flag (hydra_allreduce & co.): enqueue a multi-rank schedule even while the stream is being
 * captured into a hipGraph.  Without it such a call fails with HYDRA_ERR_UNSUPPORTED: on the
 * socket-linked ranks of the test box, ending the capture of RCCL's own ncclAllReduce segfaults
 * inside hipStreamEndCapture (profiles/r03g2_graph_ranks_rccl.log), so the library refuses
 * rather than let the caller's process die.  Set it on a node whose RCCL captures. */
#define HYDRA_ALLOW_CAPTURE 2

typedef enum {
  HYDRA_OK = 0,
  HYDRA_ERR_INVALID = 1,     /* bad argument (dtype, op, misaligned pointer, partial overlap) */
  HYDRA_ERR_HIP = 2,         /* HIP runtime error (message carries hipGetErrorString) */
  HYDRA_ERR_UNSUPPORTED = 3, /* op/dtype combination not provided */
  HYDRA_ERR_NO_DEVICE = 4,   /* no gfx950 device visible */
  HYDRA_ERR_TIMEOUT = 5      /* hydra_comm_wait: the enqueued work did not finish in time */
} hydra_status_t;

typedef void* hydra_stream_t; /* hipStream_t; NULL = the legacy default stream */
typedef struct hydra_ctx* hydra_ctx_t;

/* ---- library ---------------------------------------------------------------------------- */
int hydra_abi_version(void);
const char* hydra_last_error(void);      /* thread-local; "" when the last call succeeded */
int hydra_device_count(int* count);
int hydra_device_arch(int device, char* buf, size_t len); /* e.g. "gfx950:sramecc+:xnack-" */
/* Drain every stream of `device` and report a pending asynchronous error (a faulting kernel,
 * an illegal address).  Test attribution: the GPU suite calls it after every test. */
int hydra_device_check(int device);
/* Fault diagnostics.  After enable, a GPU memory fault prints to stderr its
 * virtual address and reason, the /proc/self/maps line holding it, and every range hydra knows
 * whose pages hold it (cache blocks, hydra_host_register ranges, per-call pins of pageable
 * operands; live or released, with times).  hydra_fault_last: the last fault seen (count 0 =
 * none).  hydra_fault_lookup: the same report for any address into buf (no fault needed).
 * The handler stays installed for the life of the process: do not unload the library after
 * enabling it. */
int hydra_fault_report_enable(void);
int hydra_fault_last(uint64_t* va, uint32_t* reason, uint64_t* count);
int hydra_fault_lookup(uint64_t va, char* buf, size_t len);

/* ---- device-resident reduction (the hot path) ---------------------------------------------
 * c[i] = op(a[i], b[i]) for i < n, enqueued on `stream` (asynchronous, graph-capturable: no
 * allocation, no synchronisation).  Pointers are device (or peer-accessible) addresses aligned
 * to the element size.  c may equal a or b exactly (the ring always calls c == a); partial
 * overlap is rejected.  n == 0 is a no-op.  Integer ops wrap modulo 2^bits; float ops round to
 * nearest even with subnormals kept, and NaNs propagate as on the reference's x86 build.      */
int hydra_reduce(int op, int dtype, void* c, const void* a, const void* b, size_t n,
                 hydra_stream_t stream);
int hydra_chunk_sum(int dtype, void* c, const void* a, const void* b, size_t n,
                    hydra_stream_t stream);
/* count independent segments c_k = op(a_k, b_k) in ONE launch (up to 32 segments per launch):
 * the same contract per segment as hydra_reduce.  Replaces `count` consecutive gloo::sum<T>
 * calls (allreduce.cc:301-305, one per arriving segment) for a caller that holds several
 * segments at once: below ~1 Mi elements a launch costs a dispatch plus one dependent HBM round
 * trip whatever its size, so K segments in one launch pay that once. */
typedef struct {
  void* c;
  const void* a;
  const void* b;
  size_t n; /* elements */
} hydra_segment_t;
int hydra_reduce_batch(int op, int dtype, const hydra_segment_t* segs, size_t count,
                       hydra_stream_t stream);

/* Mixed-precision bucket (BASELINE config 5): acc[i] = acc[i] + (float)b_bf16[i]. */
int hydra_acc_bf16_f32(float* acc, const void* b_bf16, size_t n, hydra_stream_t stream);
/* out_bf16[i] = bf16_rne(acc[i]) */
int hydra_f32_to_bf16(void* out_bf16, const float* acc, size_t n, hydra_stream_t stream);

/* P-way reduction in the reference ring's fold order (the owner step of the DIRECT/A2A
 * allreduce): dst[i] = srcs[0][i] op (srcs[1][i] op (... op srcs[nsrc-1][i])), where srcs[0]
 * is the owner's block x_q and srcs[j] rank q+j's contribution -- bit-identical to the
 * owner's P-1 in-place ring hops (allreduce.cc:301-305).  dst may equal srcs[0]; 1 <= nsrc <=
 * 16.  flags HYDRA_ACC_F32: bf16 data, fp32 accumulation, one rounding. */
int hydra_fold(int op, int dtype, int flags, void* dst, const void* const* srcs, int nsrc,
               size_t n, hydra_stream_t stream);

/* ---- library options -----------------------------------------------------------------------
 * The library reads no environment variable: every tunable is an option with the tuned default
 * (the reference's benchmark takes its settings as flags, benchmark/options.cc:144-172).
 * hydra_set_option sets the process-wide value, which applies to what starts afterwards (a
 * resident reducer instance, the staging copy pool, contexts created later); the keys marked
 * [ctx] are copied into each context at hydra_ctx_create and hydra_ctx_set_option overrides them
 * for that context alone.  Out-of-range values and unknown keys: HYDRA_ERR_INVALID.
 *   HYDRA_OPT_RESIDENT             [ctx] 1 (default): host calls are served by the device's
 *                                  resident reducer; 0: one batched launch per round
 *   HYDRA_OPT_STAGE_SPLIT          [ctx] rounds a staged call is cut into (4; 1..64)
 *   HYDRA_OPT_ROUND_MIN            [ctx] smallest staging round per operand, bytes (512 KiB;
 *                                  16 KiB..4 MiB)
 *   HYDRA_OPT_STAGE_RESULT_MAX     [ctx] results of calls of at most this many bytes per operand
 *                                  go through the pinned staging (0)
 *   HYDRA_OPT_STAGE_RESULT_REG_MAX [ctx] ... and results inside a hydra_host_register'ed range of
 *                                  at most this many bytes (8 MiB: such a bucket stays in the
 *                                  CPU's cache for the ring's next send)
 *   HYDRA_OPT_FORCE_STAGING        [ctx] 1: stage every operand, mapped or not (A/B; 0)
 *   HYDRA_OPT_COPY_THREADS         helper threads of the staging copies (4; 0..32: 0 = the
 *                                  calling thread alone); fixed once the first large copy ran
 *   HYDRA_OPT_RESIDENT_IDLE_US     a resident instance leaves after this long idle (2000)
 *   HYDRA_OPT_RESIDENT_GRACE_US    bound of every wait inside the resident grid (10 s)
 *   HYDRA_OPT_RESIDENT_QUEUE       0 (default): a greatest-priority queue of its own;
 *                                  1 a plain non-blocking stream; 2 a CU-masked stream (A/B)
 *   HYDRA_OPT_RESIDENT_BLOCKS, _BATCH, _SOLO, _TILES: the resident grid's shape (128, 4, 4, 4) */
typedef enum {
  HYDRA_OPT_RESIDENT = 1,
  HYDRA_OPT_STAGE_SPLIT = 2,
  HYDRA_OPT_ROUND_MIN = 3,
  HYDRA_OPT_STAGE_RESULT_MAX = 4,
  HYDRA_OPT_STAGE_RESULT_REG_MAX = 5,
  HYDRA_OPT_FORCE_STAGING = 6,
  HYDRA_OPT_COPY_THREADS = 7,
  HYDRA_OPT_RESIDENT_IDLE_US = 8,
  HYDRA_OPT_RESIDENT_GRACE_US = 9,
  HYDRA_OPT_RESIDENT_QUEUE = 10,
  HYDRA_OPT_RESIDENT_BLOCKS = 11,
  HYDRA_OPT_RESIDENT_BATCH = 12,
  HYDRA_OPT_RESIDENT_SOLO = 13,
  HYDRA_OPT_RESIDENT_TILES = 14
} hydra_opt_t;
int hydra_set_option(int key, long long value);
int hydra_get_option(int key, long long* value);

/* Test switches: process-wide values the library reads at the point they apply, so tests can
 * drive branches a one-GPU box never takes on its own.  Every switch is 0 in production (the
 * library never sets one itself).  hydra_test_set returns HYDRA_ERR_INVALID for an unknown or
 * read-only key; *prev (if given) receives the old value.
 *   HYDRA_TEST_LOCAL_STAGE         1: HipAllreduceRing's local steps are staged as if their two
 *                                  pointers were on devices without peer access (the
 *                                  cross-device staging branch on one GPU)
 *   HYDRA_TEST_RESIDENT_GEN_STRIDE >0: each resident-reducer launch advances the generation by
 *                                  this much instead of 1 (65536 wraps the job word's 16-bit
 *                                  generation tag on every launch)
 *   HYDRA_TEST_RESIDENT_REGRESSIONS  (read-only) completion words the resident reducer's waits
 *                                  saw move backwards, over every slot of every device */
typedef enum {
  HYDRA_TEST_LOCAL_STAGE = 1,
  HYDRA_TEST_RESIDENT_GEN_STRIDE = 2,
  HYDRA_TEST_RESIDENT_REGRESSIONS = 3
} hydra_test_key_t;
int hydra_test_set(int key, int64_t value, int64_t* prev);
int hydra_test_get(int key, int64_t* value);

/* ---- host-resident reduction --------------------------------------------------------------
 * Same contract on HOST buffers, synchronous like gloo::sum<T>: the kernel reads and writes the
 * mapped parts of a, b and c in place over PCIe (see below) and the rest through the context's
 * pinned staging, which the CPU fills and empties; one batched round per call (per 4 MiB of
 * staged bytes per operand, or per 16 intervals, beyond that: the CPU fills round r + 1 while
 * round r runs).  Device pointers are rejected (HYDRA_ERR_INVALID: use hydra_reduce).  One
 * context per calling thread (bew_allreduce_a runs two rails concurrently: one context each).
 * hydra_ctx_set_option: a [ctx] key of hydra_opt_t for this context alone (e.g.
 * HYDRA_OPT_FORCE_STAGING stages every operand for A/B measurements; HYDRA_OPT_RESIDENT 0
 * returns the context's resident slot). */
int hydra_ctx_create(int device, hydra_ctx_t* out);
int hydra_ctx_destroy(hydra_ctx_t ctx);
int hydra_ctx_set_option(hydra_ctx_t ctx, int key, long long value);
int hydra_reduce_host(hydra_ctx_t ctx, int op, int dtype, void* c, const void* a, const void* b,
                      size_t n);
int hydra_chunk_sum_host(hydra_ctx_t ctx, int dtype, void* c, const void* a, const void* b,
                         size_t n);
/* Low latency: the rounds are served by the device's RESIDENT reducer -- ONE launch of 128
 * workgroups per device per process, kept running while calls keep coming on a stream with a
 * hardware queue of its own (no other stream's work waits behind it), woken by a host-mapped
 * doorbell instead of a fresh dispatch.  Each context leases one of its 32 slots at
 * hydra_ctx_create (a context created when all are leased launches instead).  The instance
 * leaves after HYDRA_OPT_RESIDENT_IDLE_US (default 2000) without a call and at process exit.
 * HYDRA_OPT_RESIDENT 0 turns it off (every round is one launch on the context's stream).  Stats
 * (tests): rounds this context had served by it, and instances launched on its device. */
int hydra_ctx_stats(hydra_ctx_t ctx, uint64_t* resident_calls, uint64_t* resident_launches);
/* Per-call trace of hydra_reduce_host (measurement: where a call's time goes).  While enabled,
 * every call appends one record (at most 1 Mi records are kept): its size, how many intervals
 * and rounds it was cut into, the bytes of each operand the kernel touched in place (zero-copy)
 * and the bytes staged through the context's pinned buffers, whether the rounds went to the
 * resident reducer, and the call's wall time split into CPU copies in, waits for the GPU and
 * CPU copies out.  hydra_host_trace(1) clears and starts, (0) stops. */
typedef struct {
  uint64_t n, elem_bytes;
  uint32_t intervals, rounds, resident, reserved;
  uint64_t zero_copy_bytes[3]; /* c, a, b */
  uint64_t staged_bytes[3];    /* c, a, b (c: staged results copied back) */
  double total_us, copy_in_us, wait_us, copy_out_us;
} hydra_host_call_t;
int hydra_host_trace(int enable);
int hydra_host_trace_read(hydra_host_call_t* out, size_t cap, size_t* count);
/* Which host memory the kernel reads / writes in place (zero-copy over PCIe), per operand: a
 * range registered with hydra_host_register, a pinned block from hydra_malloc_host, or memory
 * the caller pinned / registered itself (hipHostMalloc, hipHostRegister, torch pinned tensors;
 * the caller keeps it so for the call, as for any copy from it).  Everything else -- pageable
 * memory, and the ragged first and last page of a registered range, which hold memory outside
 * it -- is read and written by the CPU only (memcpy through the context's pinned staging).
 * hydra never registers host memory on its own and never hands a caller's pageable range to a
 * HIP copy: on ROCm 7.2 host pages once registered and released, then reused and copied by the
 * runtime's page-locking pageable copy path, faulted the GPU.  Its
 * registrations never overlap one another and never cover a page holding memory outside the
 * range it was asked for. */
/* Page-lock caller memory for zero-copy use (optional): registers the whole pages inside
 * [ptr, ptr + bytes) (the ragged edges stay staged).  Reference-counted per start address: every
 * hydra_host_register needs one hydra_host_unregister, and a second register of the same address
 * may not cover more bytes.  Pages already mapped by their owner (hipHostRegister /
 * hipHostMalloc) are used as they are and never released here; pages another hydra registration
 * holds are shared with it; unregistering an address not registered here is a no-op.  The pages
 * stay registered until the last unregister AND the last in-flight call using them are done.
 * Register long-lived buffers only: do not free a registered range and hand its pages to
 * pageable HIP copies afterwards in the same process (the fault described above). */
int hydra_host_register(void* ptr, size_t bytes);
int hydra_host_unregister(void* ptr);
/* Inspection (tests): the whole pages inside [ptr, ptr + bytes), [*lo, *hi) (empty: equal). */
void hydra_page_interior(uint64_t ptr, size_t bytes, uint64_t* lo, uint64_t* hi);
/* Inspection (tests): hydra's live host mappings (registrations and pinned blocks),
 * how many hipHostRegister calls hydra has made, and how many of those covered a byte outside
 * the caller range they were made for (0 by construction). */
typedef struct {
  uint64_t lo, hi;  /* mapped host range */
  int32_t kind;     /* 1 hydra_host_register, 3 pinned block */
  int32_t owners;   /* hydra_host_register owners */
  int32_t users;    /* in-flight calls using it */
  uint64_t owner_lo, owner_hi; /* the caller range it was made for */
} hydra_host_mapping_t;
int hydra_host_mappings(hydra_host_mapping_t* out, size_t cap, size_t* count,
                        uint64_t* registrations, uint64_t* outside);

/* ---- streams / memory helpers for C callers (the Python layer uses torch instead) -------- */
/* Streams, events, device blocks and pinned blocks come from process-wide caches, like torch's
 * caching allocator: a destroy / free first waits for the work that may still use the object
 * (stream synchronise, event synchronise, device drain -- hipFree's own implicit
 * synchronisation), then keeps it for the next create / malloc of the same kind, size class
 * (64 KiB granules) and device.  At most 4 GiB of device blocks per device, 2 GiB of pinned
 * blocks and 64 streams / events per device are kept; the rest is really released.  Pointers
 * and handles the caches did not hand out are released directly.  hydra_cache_trim() really
 * releases everything kept (e.g. before handing the memory to another allocator). */
int hydra_cache_trim(void);
int hydra_stream_create(int device, hydra_stream_t* out);
int hydra_stream_destroy(hydra_stream_t s);
int hydra_stream_synchronize(hydra_stream_t s);
/* Events (hipEvent_t, timing disabled): completion markers an owner records on a caller's
 * stream, so it can later wait for ITS work without touching a stream it does not own. */
typedef void* hydra_event_t;
int hydra_event_create(hydra_event_t* out);                 /* on the caller's current device */
int hydra_event_create_on(int device, hydra_event_t* out);  /* on `device` (-1: current) */
int hydra_event_record(hydra_event_t e, hydra_stream_t s);
int hydra_event_synchronize(hydra_event_t e);
int hydra_event_destroy(hydra_event_t e);
/* Cross-stream ordering (cudaStreamWaitEvent, as CudaLocalNativeReduce orders its tree,
 * cuda_collectives_native.h:100-115): work enqueued on `s` after this call waits for `e`'s last
 * record.  The event and the stream may belong to different devices. */
int hydra_stream_wait_event(hydra_stream_t s, hydra_event_t e);
/* Peer access for the local reduce tree of several GPUs in one process
 * (cuda_collectives_native.h:63-84): *can = hipDeviceCanAccessPeer(device, peer); when it can,
 * `device`'s access to `peer`'s memory is enabled (idempotent; device == peer: *can = 1).  The
 * caller's current device is left as it was. */
int hydra_device_peer_access(int device, int peer, int* can);
/* Topology between two devices (inspection; the N>1 bench line records it, so a multi-GPU line
 * shows which fabric its links were): *link = hipExtGetLinkTypeAndHopCount's link type
 * (2 PCIe, 4 xGMI; hsa_amd_link_info_type_t), *hops its hop count, *can_peer =
 * hipDeviceCanAccessPeer.  Changes no device state (peer access is not enabled here). */
int hydra_device_link(int device, int peer, int* link, int* hops, int* can_peer);
int hydra_malloc(int device, size_t bytes, void** out);
int hydra_free(void* p);
int hydra_memcpy(void* dst, const void* src, size_t bytes); /* hipMemcpyDefault, synchronous */
int hydra_memcpy_async(void* dst, const void* src, size_t bytes, hydra_stream_t stream);
/* Pinned host memory (CudaHostPointer<T>::alloc, cuda.cu:231-240). */
int hydra_malloc_host(size_t bytes, void** out);
int hydra_free_host(void* p);
/* Device of a device allocation, -1 for host memory (CudaDevicePointer::create, cuda.cu:175-188). */
int hydra_pointer_device(const void* p, int* device);

/* ---- ring geometry (allreduce.cc:199-221), shared by the host ring and the xGMI ring ----- */
void hydra_ring_plan(int P, size_t n, size_t esize, size_t max_segment, size_t* num_segments,
                     size_t* segment_bytes, size_t* segments_per_rank);

/* ---- multi-GPU bucket allreduce over RCCL / xGMI ------------------------------------------
 * One process per GPU.  Replaces gloo::allreduce(opts) with RING (allreduce.cc:99-422) for
 * device-resident buckets: block ownership and per-element fold order are the reference's, so
 * results are bit-identical to the reference ring for every dtype/op.
 *   HYDRA_ALGO_RING    the reference schedule: P-1 reduce-scatter hops to rank-1 with the HIP
 *                      sum fused into each hop, then P-1 all-gather hops (one link per direction)
 *   HYDRA_ALGO_DIRECT  all-to-all reduce-scatter in one p2p group (all 7 xGMI links), then ONE
 *                      fold kernel per chunk in the reference order, then a direct all-gather
 *   HYDRA_ALGO_RCCL    ncclAllReduce (RCCL's own fold order: a tolerance, not bit-exact)
 *   HYDRA_ALGO_A2A     equal blocks only: ncclAllToAll of the blocks, ONE fold kernel in the
 *                      reference order, ncclAllGather in place (bit-exact, 3 launches)
 *   HYDRA_ALGO_RING_OLD  the old-style gloo::AllreduceRing<T> (allreduce_ring.h:20-125) on
 *                      device: P-1 whole-bucket rounds, each rank left-folds x_r op x_{r-1} op
 *                      ... (ranks differ, exactly as the reference; max_segment unused)
 *   HYDRA_ALGO_RING_CHUNKED  gloo::AllreduceRingChunked<T> (allreduce_ring_chunked.h:20-248):
 *                      2P chunks of max(256, ceil(n/2P)) elements, pipelined reduce pass +
 *                      broadcast pass; identical bits on every rank (max_segment, chunk_bytes
 *                      unused)
 *   HYDRA_ALGO_BCUBE   gloo::allreduce BCUBE (allreduce.cc:423-700): hypercube reduce-scatter
 *                      over the factors of P, then the reverse all-gather; the reference's
 *                      BCUBE bits (max_segment, chunk_bytes unused)
 *   HYDRA_ALGO_HALVING_DOUBLING  gloo::AllreduceHalvingDoubling<T>
 *                      (allreduce_halving_doubling.h:37-358): recursive halving / doubling in
 *                      binary blocks of P, bit-reversed exchange between blocks; identical
 *                      bits on every rank (max_segment, chunk_bytes unused)
 *   HYDRA_ALGO_RCCL_RS_AG  ncclReduceScatter in place + ncclAllGather in place: RCCL's own
 *                      ring reduce-scatter / all-gather (SURVEY 8(e)'s comparison point; RCCL's
 *                      order, a tolerance, not bit-exact; n a multiple of P)
 *   HYDRA_ALGO_AUTO    A2A when the reference blocks are equal (n*E a multiple of P*S*segmentBytes),
 *                      else DIRECT
 * max_segment: the reference's maxSegmentSize (0 = 1 MiB, allreduce.h:78) -- it fixes block
 * ownership; chunk_bytes: pipelining granularity (0 = 16 MiB), does not change results.
 * flags: HYDRA_ACC_F32 -- bf16 bucket, fp32 accumulation, one rounding (BASELINE config 5;
 * DIRECT/A2A/AUTO). */
#define HYDRA_UNIQUE_ID_BYTES 128
typedef enum {
  HYDRA_ALGO_AUTO = 0,
  HYDRA_ALGO_RING = 1,
  HYDRA_ALGO_DIRECT = 2,
  HYDRA_ALGO_RCCL = 3,
  HYDRA_ALGO_A2A = 4,
  HYDRA_ALGO_RING_OLD = 5,
  HYDRA_ALGO_RING_CHUNKED = 6,
  HYDRA_ALGO_BCUBE = 7,
  HYDRA_ALGO_HALVING_DOUBLING = 8,
  HYDRA_ALGO_RCCL_RS_AG = 9
} hydra_algo_t;
typedef struct hydra_comm* hydra_comm_t;

/* A plan op (one rank's schedule entry; see hydra_amd/csrc/xgmi_plan.h). */
typedef struct {
  int32_t kind; /* 1 SEND, 2 RECV, 3 GROUP end, 4 REDUCE (ring hop), 5 FOLD (owner),
                   6 ALLTOALL, 7 ALLGATHER (collectives over the whole bucket) */
  int32_t peer; /* FOLD: -1 contributor-ordered slots, >= 0 rank-ordered slots rotated by it */
  int32_t buf;  /* 0 user bucket, 1 scratch */
  int32_t nsrc;
  int64_t off, bytes, src_off, slot_stride;
  int32_t wait0, wait1;
} hydra_plan_op_t;

int hydra_comm_get_unique_id(void* id /* HYDRA_UNIQUE_ID_BYTES */);
int hydra_comm_init(hydra_comm_t* out, int nranks, int rank, const void* id, int device);
int hydra_comm_destroy(hydra_comm_t comm);
/* What RCCL itself reports for the communicator: ncclCommCount, ncclCommUserRank and
 * ncclCommCuDevice (the bench line records them, so a multi-GPU line shows RCCL saw N ranks). */
int hydra_comm_info(hydra_comm_t comm, int* nranks, int* rank, int* device);
int hydra_allreduce(hydra_comm_t comm, int algo, int op, int dtype, int flags, void* buf,
                    size_t n, size_t max_segment, size_t chunk_bytes, hydra_stream_t stream);

/* gloo::reduce (gloo/gloo/reduce.cc:21-262) of a device bucket to `root`, in place, on
 * `stream`: gloo::reduce's own block geometry (reduce.cc:87-135), a DIRECT-style reduce-scatter
 * whose owner folds are the reference's order, then every owner sends its block to the root.
 * Only the root's bucket is defined afterwards (as in the reference).  flags: HYDRA_ACC_F32
 * for bf16 buckets, as DIRECT. */
int hydra_reduce_root(hydra_comm_t comm, int root, int op, int dtype, int flags, void* buf,
                      size_t n, size_t max_segment, size_t chunk_bytes, hydra_stream_t stream);
/* The reference's per-op timeout (AllreduceOptions::setTimeout, allreduce.h:52; waitRecv /
 * waitSend(opts.timeout) -> IoException "Timed out waiting ...", tcp/unbound_buffer.cc:60-85)
 * for the asynchronous device path: wait until everything enqueued on `stream` so far is done.
 * Past `timeout_ms` the communicator is aborted (ncclCommAbort: no rank stays stuck in RCCL)
 * and HYDRA_ERR_TIMEOUT is returned with "Timed out waiting <ms>ms for ..."; the communicator
 * is then unusable (destroy it).  RCCL's asynchronous errors are reported the same way. */
int hydra_comm_wait(hydra_comm_t comm, hydra_stream_t stream, int64_t timeout_ms);

/* Per-phase timing of a communicator's allreduces (measurement, not for the timed region): while
 * profiling is on, every p2p group / collective on the comm stream and every fold kernel on the
 * compute stream is bracketed by timing events.  hydra_comm_phases waits for the profiled work
 * and returns the totals since profiling was switched on:
 *   link_ms   comm-stream busy time (sum over p2p groups and collectives)
 *   fold_ms   compute-stream busy time (sum over REDUCE / FOLD kernels)
 *   span_ms   sum over calls of first enqueue (the call's start on the caller's stream) to the
 *             last op's end; link_ms + fold_ms - span_ms > 0 is the overlap of the two streams
 *   sent_bytes / recv_bytes   this rank's link bytes (p2p sends / receives and the collectives'
 *             off-rank share), peers = distinct peers it sent to (links used per call)
 *   fold_hbm_bytes   the fold kernels' algorithmic HBM bytes ((nsrc + 1) x block bytes per FOLD,
 *             3 x segment bytes per REDUCE)
 * A communicator's own device is used whatever the caller's current device is. */
typedef struct {
  uint64_t calls, link_ops, fold_ops;
  double link_ms, fold_ms, span_ms;
  uint64_t sent_bytes, recv_bytes, fold_hbm_bytes;
  int32_t peers, reserved;
} hydra_comm_phases_t;
int hydra_comm_profile(hydra_comm_t comm, int enable); /* 1: on, totals reset; 0: off */
int hydra_comm_phases(hydra_comm_t comm, hydra_comm_phases_t* out);

/* ---- bew_allreduce_a on device: two rails (pipeallreduce-a.cc:27-61) ---------------------- */
#ifndef HYDRA_SPLIT_AA
#define HYDRA_SPLIT_AA 0 /* calculateElements_AA, pipeallreduce-a.h:296-376 (default) */
#define HYDRA_SPLIT_AG 1 /* calculateElements_AG, pipeallreduce-a.h:137-294 (ALLREDUCE_GLEX) */
#endif
/* e1 elements for rail 1 (opts3), e2 = n - e1 for rail 2 (opts2). */
void hydra_split_elements(int table, int P, size_t n, size_t* e1, size_t* e2);
/* [0, e1) allreduced on rail1 and [e1, n) on rail2, concurrently on the rails' own streams
 * forked from and joined back into `stream` (the reference spawns two threads per call).  Each
 * part equals gloo::allreduce RING on that slice with its own geometry (bit-exact for the
 * plan algorithms).  One part empty: one allreduce on the other rail, as the reference does.
 * The rails are two communicators over the same ranks (e.g. two hydra_comm_init calls). */
int hydra_apipe_allreduce(hydra_comm_t rail1, hydra_comm_t rail2, int table, int algo, int op,
                          int dtype, int flags, void* buf, size_t n, size_t max_segment,
                          size_t chunk_bytes, hydra_stream_t stream);
/* Executor test hook: run `ops` (e.g. a hydra_plan with peers remapped) through the RCCL
 * executor of `comm`.  Every op is validated against buf_bytes / scratch_bytes (collectives:
 * against the communicator size) first.  On a 1-rank communicator, RCCL's send/recv-to-self runs the real
 * executor (groups, both streams, event edges) on one GPU. */
int hydra_comm_run_plan(hydra_comm_t comm, const hydra_plan_op_t* ops, size_t nops, int op,
                        int dtype, int flags, void* buf, size_t buf_bytes, size_t scratch_bytes,
                        hydra_stream_t stream);
/* The same split on P simulated ranks of one GPU (see hydra_allreduce_simulate). */
int hydra_apipe_allreduce_simulate(int table, int algo, int op, int dtype, int flags, int P,
                                   void** bufs, size_t n, size_t max_segment, size_t chunk_bytes);

/* The schedule rank `rank` of P executes (for inspection / host-side tests). */
int hydra_plan(int algo, int P, int rank, size_t n, size_t esize, size_t max_segment,
               size_t chunk_bytes, hydra_plan_op_t* ops, size_t cap, size_t* count,
               size_t* scratch_bytes);

/* All P ranks' plans on ONE GPU (device copies stand in for xGMI, same kernels, same
 * cross-stream dependencies): bufs[r] is rank r's bucket.  Synchronous.  For testing the
 * multi-GPU path on a single-GPU machine. */
int hydra_allreduce_simulate(int algo, int op, int dtype, int flags, int P, void** bufs,
                             size_t n, size_t max_segment, size_t chunk_bytes);
/* hydra_reduce_root's schedule: the op list of `rank`, and all P ranks simulated on one GPU
 * (bufs: P device buckets, in place; bufs[root] ends with the reduction). */
int hydra_reduce_root_plan(int root, int P, int rank, size_t n, size_t esize, size_t max_segment,
                           size_t chunk_bytes, hydra_plan_op_t* ops, size_t cap, size_t* count,
                           size_t* scratch_bytes);
int hydra_reduce_root_simulate(int root, int op, int dtype, int flags, int P, void** bufs,
                               size_t n, size_t max_segment, size_t chunk_bytes);

/* ---- peer-access bucket allreduce over xGMI (no RCCL) --------------------------------------
 * The MI355X-first form of gloo::allreduce RING (allreduce.cc:147-422) for device-resident
 * buckets on one fully connected node: the peers' buckets are mapped into every rank by hipIpc
 * handles and ONE kernel per allreduce reads the other ranks' data over xGMI, folding it in the
 * reference's order (owner block q = x_q + (x_{q+1} + (... + x_{q-1})), blocks from
 * allreduce.cc:199-221) -- so results are bit-identical to RING/DIRECT and to the reference.
 *   HYDRA_PEER_TWO_SHOT  each rank folds its own block pulling from all P buckets (in place),
 *                        then pulls the other finished blocks (2(P-1)/P * n * E link bytes)
 *   HYDRA_PEER_ONE_SHOT  each rank folds the whole bucket into scratch, then copies it back
 *                        ((P-1) * n * E link bytes, 2 barriers)
 *   HYDRA_PEER_TWO_SHOT_PUSH  each rank folds its own block pulling from all P buckets and
 *                        stores the result into EVERY bucket (its own in place, the peers' over
 *                        xGMI): no second pull, 2 barriers, the same link bytes as TWO_SHOT and
 *                        n * E read + n * E written per rank.  Needs every rank's bucket at the
 *                        same address modulo 16 (else it runs as TWO_SHOT, on every rank alike)
 *   HYDRA_PEER_AUTO      ONE_SHOT up to HYDRA_PEER_OPT_ONE_SHOT_MAX bytes (default 0), else
 *                        TWO_SHOT_PUSH
 * Setup (every rank, same order; the byte blobs travel over any channel the caller has, e.g.
 * the rendezvous store): hydra_peer_create -> exchange sig handles -> hydra_peer_connect; for
 * each bucket: hydra_peer_register -> exchange -> hydra_peer_open.  Every rank must then issue
 * the same sequence of hydra_peer_allreduce calls (like any collective).  A call is one kernel
 * launch and is graph-capturable: barrier epochs live on the device, so replays need no new
 * arguments.  Eager calls on one group run one after another on the device even when issued on
 * different streams (each waits for the previous eager call's completion event).  A captured
 * call neither waits for nor records that event (a capture cannot wait on an outside event):
 * the caller orders a graph's replays against each other and against eager calls of the same
 * group on other streams (e.g. one stream for all of them).  A peer that never arrives ends
 * the kernel after the timeout (default 20 s) and leaves an error code readable with
 * hydra_peer_error; later calls on the group fail with HYDRA_ERR_HIP.  1 <= nranks <= 8.
 * Ranks of one group on the same GPU (each rank's GPU travels in its signal handle) must have
 * every rank's whole grid resident at once: an explicit HYDRA_PEER_OPT_BLOCKS beyond the GPU's
 * capacity / (the most ranks of the group on one GPU) is refused with HYDRA_ERR_INVALID, and the
 * derived grid shrinks to fit -- the same grid on every rank of the group. */
#define HYDRA_PEER_HANDLE_BYTES 128
typedef enum {
  HYDRA_PEER_AUTO = 0,
  HYDRA_PEER_TWO_SHOT = 1,
  HYDRA_PEER_ONE_SHOT = 2,
  HYDRA_PEER_TWO_SHOT_PUSH = 3
} hydra_peer_algo_t;
typedef enum {
  HYDRA_PEER_OPT_TIMEOUT_MS = 1,  /* barrier timeout (default 20000) */
  HYDRA_PEER_OPT_BLOCKS = 2,      /* workgroups per launch (0 = derived from the bucket, <= 1024) */
  HYDRA_PEER_OPT_ONE_SHOT_MAX = 3 /* AUTO threshold in bytes (default 0: always the push) */
} hydra_peer_opt_t;
typedef struct hydra_peer* hydra_peer_t;
/* sig_handle: HYDRA_PEER_HANDLE_BYTES out, to be gathered in rank order for hydra_peer_connect */
int hydra_peer_create(int nranks, int rank, int device, hydra_peer_t* out, void* sig_handle);
int hydra_peer_connect(hydra_peer_t peer, const void* sig_handles /* nranks * HANDLE_BYTES */);
/* buf: device memory (any sub-range of one allocation, e.g. a torch tensor) */
int hydra_peer_register(hydra_peer_t peer, void* buf, size_t bytes, void* handle);
int hydra_peer_open(hydra_peer_t peer, void* buf, size_t bytes, const void* handles);
int hydra_peer_close(hydra_peer_t peer, void* buf);
int hydra_peer_set_option(hydra_peer_t peer, int key, long long value);
int hydra_peer_error(hydra_peer_t peer, int* code); /* 0 = healthy */
/* buf must lie inside a buffer opened with hydra_peer_open, at the same offset on every rank */
int hydra_peer_allreduce(hydra_peer_t peer, int algo, int op, int dtype, int flags, void* buf,
                         size_t n, size_t max_segment, hydra_stream_t stream);
/* Teardown is collective, in this order on every rank:
 *   hydra_peer_detach  (closes every mapping this rank holds of the other ranks' memory)
 *   -> a barrier on the caller's channel
 *   -> hydra_peer_destroy (frees this rank's signal area), and only then free the buckets.
 * A rank never frees memory another rank still has mapped.  detach is local and idempotent;
 * allreduce calls fail once it ran.  hydra_peer_close(buf) has the same rule per buffer: close
 * on every rank, barrier, then free.  Register long-lived buckets: freeing a registered
 * allocation and registering a new one in the same process intermittently gave a peer a
 * mapping of the wrong memory on ROCm 7.2.  Enforced: every handle carries the
 * exporter's allocation id (HIP_POINTER_ATTRIBUTE_BUFFER_ID) and peers key their mappings by
 * it, and hydra_peer_register refuses (HYDRA_ERR_INVALID) an address whose allocation changed
 * since this group exported it, until hydra_peer_close released the old registration. */
int hydra_peer_detach(hydra_peer_t peer);
int hydra_peer_destroy(hydra_peer_t peer);

#ifdef __cplusplus
}
#endif
#endif /* HYDRA_HIP_H_ */
