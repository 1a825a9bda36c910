// One-pass left-to-right chains beyond 31 peers (P <= 128 per launch; longer chains run as segments of 127
// peers continued from the previous segment's running value, fmi_dev.hip chain_superblocks): scan_ltr (reference PeerToPeer::scan_ltr,
// src/comm/PeerToPeer.cpp:141-152: peer k combines f(prefix of k-1, own)) and reduce_ltr (:44-57: the root
// folds the gathered buckets ((x0 + x1) + x2) + ..). The blocked launches (fmi_dev.hip) run 15 peers at a
// time from a carry bucket; here one thread carries the running value in registers through all P peers,
// 16 loads in flight per step of the runtime block loop. Same operand order, so the same bits; P (+P) bucket
// passes instead of P + 2 ceil((P - 16) / 15) (+P).
#include "fmi_fused_impl.h"

namespace fmi::dev {
namespace {

constexpr int BL = sched::kScanBlock;  // 16

// Peers [base, base + m) of the chain: all loads first, then the combines, then the stores (as the fused
// kernels; a first version that stored each prefix right after its combine ran scan_ltr P = 64 at 0.43 of
// peak, below the blocked launches).
template <class Op, class T, int W, bool SCAN, bool FULL>
__device__ __forceinline__ void chain_block(const BlockedScanPtrs& ptrs, int base, int m, size_t elem, Lanes<T, W>& acc) {
    using L = Lanes<T, W>;
    L x[BL];
#pragma unroll
    for (int q = 0; q < BL; ++q)
        if (FULL || q < m) x[q] = load_lanes<kFusedNT, T, W>(static_cast<const T*>(ptrs.in[base + q]) + elem);
#pragma unroll
    for (int q = 0; q < BL; ++q)
        if (FULL || q < m) x[q] = acc = combine<Op, T, W>(acc, x[q]);
    if constexpr (SCAN) {
#pragma unroll
        for (int q = 0; q < BL; ++q)
            if (FULL || q < m) store_lanes<kFusedNT, T, W>(static_cast<T*>(ptrs.out[base + q]) + elem, x[q]);
    }
}

// carry_in: ptrs.in[0] is the running value of an earlier segment (the previous peer's prefix), not a peer
// of this segment, so its output is not stored again.
template <class Op, class T, int W, bool SCAN>
__device__ __forceinline__ void chain_group(const BlockedScanPtrs& ptrs, int P, size_t elem, bool carry_in) {
    Lanes<T, W> acc = load_lanes<kFusedNT, T, W>(static_cast<const T*>(ptrs.in[0]) + elem);
    if constexpr (SCAN)
        if (!carry_in) store_lanes<kFusedNT, T, W>(static_cast<T*>(ptrs.out[0]) + elem, acc);
    int base = 1;
    for (; base + BL <= P; base += BL) chain_block<Op, T, W, SCAN, true>(ptrs, base, BL, elem, acc);  // uniform
    if (base < P) chain_block<Op, T, W, SCAN, false>(ptrs, base, P - base, elem, acc);
    if constexpr (!SCAN) store_lanes<kFusedNT, T, W>(static_cast<T*>(ptrs.out[0]) + elem, acc);
}

template <class Op, class T, bool SCAN>
__global__ void __launch_bounds__(256) chain_kernel(BlockedScanPtrs ptrs, int P, size_t n, int carry_in) {
    constexpr int W = kVecLanes<T>;
    const size_t nvec = n / W;
    const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
    for (size_t g = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; g < nvec; g += stride)
        chain_group<Op, T, W, SCAN>(ptrs, P, g * W, carry_in != 0);
    const size_t first = nvec * W;
    if (blockIdx.x == 0 && first + threadIdx.x < n) chain_group<Op, T, 1, SCAN>(ptrs, P, first + threadIdx.x, carry_in != 0);
}

}  // namespace

int launch_chain_one_pass(int op, int dtype, bool scan, int P, const BlockedScanPtrs& ptrs, size_t n, hipStream_t s,
                          bool carry_in) {
    if (P < 2 || P > kMaxOnePassScanBlocks * BL)
        return fail(FMI_ERR_INVALID, "one-pass chain needs 2 <= P <= " + std::to_string(kMaxOnePassScanBlocks * BL));
    return with_op_dtype<false>(op, dtype, [&]<class Op, class T>() -> int {
        const size_t nvec = n / kVecLanes<T>;
        const unsigned grid = static_cast<unsigned>(std::min<size_t>(grid_for(nvec, kFusedBlock), kFusedGridCap));
        const size_t lds = fused_lds_bytes(BL, kFusedBlock * 16);  // 16 streams in flight at a time
        if (scan)
            chain_kernel<Op, T, true><<<grid, kFusedBlock, lds, s>>>(ptrs, P, n, carry_in ? 1 : 0);
        else
            chain_kernel<Op, T, false><<<grid, kFusedBlock, lds, s>>>(ptrs, P, n, carry_in ? 1 : 0);
        return check_launch("one-pass chain launch");
    });
}

}  // namespace fmi::dev
