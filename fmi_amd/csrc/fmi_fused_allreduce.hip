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

// Every peer's value of the same program at once (ptrs.out[r] = the value peer r holds), for the
// operand-order-sensitive ops only (float max / min): a sharded allreduce hands each rank the shard
// reductions in that rank's own order. One pass: P reads, P writes.
template <class Op, class T, int P>
void all_ranks_one(const PeerPtrs& ptrs, size_t n, int, hipStream_t s) {
    const size_t nvec = n / kVecLanes<T>;
    const unsigned grid = static_cast<unsigned>(std::min<size_t>(grid_for(nvec, kFusedBlock), kFusedGridCap));
    scan_kernel<Op, T, sched::kAllreduce, P><<<grid, kFusedBlock, fused_lds_bytes(P, kFusedBlock * 16), s>>>(ptrs, n, fused_policy(true, P));
}

template <class Op, class T, int... I>
constexpr std::array<FusedFn, sizeof...(I)> all_ranks_table(std::integer_sequence<int, I...>) {
    return {&all_ranks_one<Op, T, I + 2>...};
}

int launch_fused_allreduce_all_ranks(int op, int dtype, int P, const PeerPtrs& ptrs, size_t n, hipStream_t s) {
    if (P < 2 || P > sched::kMaxFusedPeers)
        return fail(FMI_ERR_INVALID, "all-ranks allreduce kernel needs 2 <= P <= 16, got " + std::to_string(P));
    return with_op_dtype<false>(op, dtype, [&]<class Op, class T>() -> int {
        if constexpr (std::is_floating_point_v<T> && (std::is_same_v<Op, OpMax> || std::is_same_v<Op, OpMin>)) {
            static constexpr auto table = all_ranks_table<Op, T>(std::make_integer_sequence<int, sched::kMaxFusedPeers - 1>{});
            table[P - 2](ptrs, n, 0, s);
            return check_launch("all-ranks allreduce kernel launch");
        } else {
            return fail(FMI_ERR_INVALID, "all-ranks allreduce kernel: only float max / min depend on the rank");
        }
    });
}
}  // namespace fmi::dev
