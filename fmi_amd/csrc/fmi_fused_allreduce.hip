// Fused single-pass kernels in the order of reference PeerToPeer::allreduce_no_order
// (src/comm/PeerToPeer.cpp:96-130).
#include "fmi_fused_impl.h"

namespace fmi::dev {
int launch_fused_allreduce(int op, int dtype, int P, const PeerPtrs& ptrs, size_t n, int rank, hipStream_t s) {
    return launch_fused<sched::kAllreduce, true>(op, dtype, P, ptrs, n, rank, s);
}
}  // namespace fmi::dev
