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
}  // namespace fmi::dev
