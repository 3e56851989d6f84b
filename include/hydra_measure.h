/* hydra_measure.h -- measurement-only entry points of libhydra_measure.so.
 *
 * libhydra_measure.so is the product library (include/hydra_hip.h, every symbol) built again
 * with -DHYDRA_MEASURE: it adds the A/B kernel variants the tuning scripts compare against the
 * shipped defaults and the peer kernel's phase clocks.  Only scripts/ and the variant parity
 * tests load it; libhydra_hip.so exports none of these, and nothing in the product path
 * selects a variant. */
#ifndef HYDRA_MEASURE_H_
#define HYDRA_MEASURE_H_

#include "hydra_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Kernel variant selection (0 = the shipped default; process-wide; returns the previous value):
 *   1..52      hydra_reduce / hydra_chunk_sum (fp32 / int32 sum): unroll, cache policy, grid,
 *              LDS-DMA double buffering (13, 18), wave-shuffle tail (44), persistent (45-47)
 *   1..7       hydra_fold (the DIRECT / A2A owner fold): load policy, grid cap, XCD map
 *   2001..2007 hydra_peer_allreduce (fp32 sum): nontemporal loads / stores, deeper pipelining;
 *   2016       the same with the 1-3-source folds as deep as the others;
 *   2032       the push schedule's slabs handed out by a ticket counter (dynamic balance) */
int hydra_set_variant(int variant);

/* Phase clocks of the peer-access allreduce (fp32 sum only while set): every later
 * hydra_peer_allreduce on `peer` runs the shipped kernel (or variant 2032's) plus, per workgroup b, kPeerStamps = 6
 * s_memrealtime values (100 MHz) written to dev_buf[6 b + k]: kernel entry, after barrier 1,
 * end of the fold phase, after barrier 2, end of the copy phase, after barrier 3.  dev_buf
 * holds max_workgroups x 6 uint64 (device memory); a larger grid is refused.  NULL: off. */
int hydra_measure_peer_stamps(hydra_peer_t peer, void* dev_buf, size_t max_workgroups);

#ifdef __cplusplus
}
#endif

#endif /* HYDRA_MEASURE_H_ */
