// Fused single-pass allreduce_no_order (reference src/comm/PeerToPeer.cpp:96-130) for P = 17..31: the
// pre-fold of peers 16.. into peers 0.. (:100-107) and the 16-peer recursive doubling (:108-121) in one pass
// over all P inputs. Its own translation unit: these programs are the largest and build in parallel with
// the rest.
#include "fmi_fused_impl.h"

namespace fmi::dev {
int launch_fused_allreduce_wide(int op, int dtype, int P, const PeerPtrs& ptrs, size_t n, int rank, hipStream_t s) {
    return launch_fused<sched::kAllreduce, true, sched::kMaxFusedPeers + 1, sched::kMaxFusedAllreducePeers>(
        op, dtype, P, ptrs, n, rank, s);
}

int launch_fused_allreduce_prefold16(int op, int dtype, const PeerPtrs& ptrs, size_t n, int rank, hipStream_t s) {
    // the 16-peer recursive doubling is symmetric under p -> p ^ rank (fmi_fused_allreduce.hip); each
    // peer's partner moves with it
    PeerPtrs perm = ptrs;
    for (int j = 0; j < 16; ++j) {
        perm.in[j] = ptrs.in[j ^ (rank & 15)];
        perm.in[16 + j] = ptrs.in[16 + (j ^ (rank & 15))];
    }
    return launch_fused<sched::kAllreducePrefold16, false, 32, 32>(op, dtype, 32, perm, n, 0, s);
}
}  // namespace fmi::dev
