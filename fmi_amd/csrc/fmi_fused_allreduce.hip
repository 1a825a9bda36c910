// Fused single-pass kernels in the order of reference PeerToPeer::allreduce_no_order
// (src/comm/PeerToPeer.cpp:96-130), P = 2..16; 17..31 in fmi_fused_allreduce_wide.hip.
#include "fmi_fused_impl.h"

namespace fmi::dev {
int launch_fused_allreduce(int op, int dtype, int P, const PeerPtrs& ptrs, size_t n, int rank, hipStream_t s) {
    if (P > sched::kMaxFusedPeers) return launch_fused_allreduce_wide(op, dtype, P, ptrs, n, rank, s);
    return launch_fused<sched::kAllreduce, true>(op, dtype, P, ptrs, n, rank, s);
}
}  // namespace fmi::dev
