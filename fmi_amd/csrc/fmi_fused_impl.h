// fmi_fused_impl.h — launch tables for the fused P-way kernels (included by one TU per algorithm).
#pragma once

#include <algorithm>
#include <array>
#include <type_traits>

#include "fmi_internal.h"

namespace fmi::dev {

inline int check_launch(const char* what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(FMI_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
    return FMI_OK;
}

constexpr unsigned kFusedBlock = 256;

using FusedFn = void (*)(const PeerPtrs&, size_t, int, hipStream_t);

template <class Op, class T, int ALG, bool ALL_RANKS, int P>
void fused_one(const PeerPtrs& ptrs, size_t n, int rank, hipStream_t s) {
    const size_t nvec = n / kVecLanes<T>;
    const unsigned grid = static_cast<unsigned>(std::min<size_t>(grid_for(nvec, kFusedBlock), kFusedGridCap));
    const size_t lds = fused_lds_bytes(P, kFusedBlock * 16);
    if constexpr (sched::stores_all_outputs(ALG))
        scan_kernel<Op, T, ALG, P><<<grid, kFusedBlock, lds, s>>>(ptrs, n, fused_policy(true, P));
    else
        tree_kernel<Op, T, ALG, P, ALL_RANKS><<<grid, kFusedBlock, lds, s>>>(ptrs, n, rank, fused_policy(false, P));
}

template <class Op, class T, int ALG, bool ALL_RANKS, int LO, int... I>
constexpr std::array<FusedFn, sizeof...(I)> fused_table(std::integer_sequence<int, I...>) {
    return {&fused_one<Op, T, ALG, ALL_RANKS, I + LO>...};
}

// RANK_AWARE: the algorithm hands different operand orders to different peers (allreduce); the
// rank-selecting kernel is instantiated only where that can change bits (float max/min).
// [LO, HI]: the peer counts this translation unit instantiates.
template <int ALG, bool RANK_AWARE, int LO = 2, int HI = sched::kMaxFusedPeers>
int launch_fused(int op, int dtype, int P, const PeerPtrs& ptrs, size_t n, int rank, hipStream_t s) {
    static_assert(2 <= LO && LO <= HI && HI <= sched::max_fused_peers(ALG), "fused peer range");
    if (P < LO || P > HI)
        return fail(FMI_ERR_INVALID, "fused kernel needs " + std::to_string(LO) + " <= P <= " + std::to_string(HI) +
                                         ", got " + std::to_string(P));
    return with_op_dtype<false>(op, dtype, [&]<class Op, class T>() -> int {
        constexpr bool order_sensitive =
            RANK_AWARE && std::is_floating_point_v<T> && (std::is_same_v<Op, OpMax> || std::is_same_v<Op, OpMin>);
        static constexpr auto table =
            fused_table<Op, T, ALG, order_sensitive, LO>(std::make_integer_sequence<int, HI - LO + 1>{});
        table[P - LO](ptrs, n, order_sensitive ? rank : 0, s);
        return check_launch("fused P-way kernel launch");
    });
}

}  // namespace fmi::dev
