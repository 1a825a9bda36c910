// Fused single-pass kernels in the order of reference PeerToPeer::reduce_no_order
// (src/comm/PeerToPeer.cpp:59-84) and PeerToPeer::reduce_ltr (src/comm/PeerToPeer.cpp:44-57); the reduce with
// every peer's final sendbuf as an output (its partial, :72) for the reference-faithful sharded reduce.
#include "fmi_fused_impl.h"

namespace fmi::dev {
int launch_fused_reduce(int op, int dtype, int P, const PeerPtrs& ptrs, size_t n, hipStream_t s) {
    return launch_fused<sched::kReduce, false>(op, dtype, P, ptrs, n, 0, s);
}
int launch_fused_reduce_ltr(int op, int dtype, int P, const PeerPtrs& ptrs, size_t n, hipStream_t s) {
    return launch_fused<sched::kReduceLtr, false>(op, dtype, P, ptrs, n, 0, s);
}
int launch_fused_reduce_partials(int op, int dtype, int P, const PeerPtrs& ptrs, size_t n, hipStream_t s) {
    return launch_fused<sched::kReducePartials, false>(op, dtype, P, ptrs, n, 0, s);
}
}  // namespace fmi::dev
