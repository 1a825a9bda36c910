// Fused single-pass kernels in the order of reference PeerToPeer::allreduce_no_order
// (src/comm/PeerToPeer.cpp:96-130), P = 2..16; 17..31 in fmi_fused_allreduce_wide.hip.
#include "fmi_fused_impl.h"

namespace fmi::dev {
int launch_fused_allreduce(int op, int dtype, int P, const PeerPtrs& ptrs, size_t n, int rank, hipStream_t s) {
    if (P > sched::kMaxFusedPeers) return launch_fused_allreduce_wide(op, dtype, P, ptrs, n, rank, s);
    if ((P & (P - 1)) == 0 && rank > 0 && rank < P) {
        // For P = 2^k, recursive doubling is symmetric under relabelling peers p -> p ^ rank: the value
        // peer `rank` ends with is rank 0's expression over inputs x[p ^ rank] (every operand order
        // included; checked against the schedule in tests/test_abi.py). So the rank-0 kernel over
        // permuted pointers replaces the rank-selecting one, which has to evaluate every peer's value.
        PeerPtrs perm = ptrs;
        for (int p = 0; p < P; ++p) perm.in[p] = ptrs.in[p ^ rank];
        return launch_fused<sched::kAllreduce, false>(op, dtype, P, perm, n, 0, s);
    }
    return launch_fused<sched::kAllreduce, true>(op, dtype, P, ptrs, n, rank, s);
}
}  // namespace fmi::dev
