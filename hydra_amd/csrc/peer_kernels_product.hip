// peer_kernels_product.hip -- the peer-access allreduce kernels of one reduction op (product), every
// dtype (peer_fold.h); launch_peer (peer_kernels.hip) dispatches here.
#include "peer_fold.h"

namespace hydra {

hipError_t launch_peer_product(int algo, int dtype, bool acc32, const PeerLaunch& A, unsigned grid,
                        hipStream_t s, int* occ) {
  return dispatch<kProduct>(algo, dtype, acc32, A, grid, s, occ);
}

}  // namespace hydra
