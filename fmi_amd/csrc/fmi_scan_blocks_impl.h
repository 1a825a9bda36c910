// fmi_scan_blocks_impl.h — the one-pass blocked scan kernel (see fmi_fused_scan_blocked.hip), included by
// the translation units that instantiate it for their range of block counts.
#pragma once

#include "fmi_fused_impl.h"

namespace fmi::dev::scan_blocks {

constexpr int BL = sched::kScanBlock;  // 16

template <int B>
struct LevelReady {
    static constexpr std::array<int, sched::kFusedInputCap + sched::kFusedStepCap> compute() {
        std::array<int, sched::kFusedInputCap + sched::kFusedStepCap> r{};
        const auto& prog = sched::Fused<sched::kScan, B>::prog;
        for (int v = 0; v < B; ++v) r[v] = v;
        for (int s = 0; s < prog.nsteps; ++s) r[B + s] = std::max(r[prog.step[s].a], r[prog.step[s].b]);
        return r;
    }
    static constexpr auto ready = compute();
    static constexpr bool outputs_causal() {
        for (int b = 0; b < B; ++b)
            if (ready[sched::Fused<sched::kScan, B>::prog.out[b]] != b) return false;
        return true;
    }
    static_assert(outputs_causal(), "scan output b must depend on blocks 0..b only");
};

template <int B, size_t S>
inline constexpr int kLevelReady = LevelReady<B>::ready[B + S];

// Block-level scan steps that become computable once T_b is known, in program order.
template <class Op, class T, int W, int B, int b, size_t... S>
__device__ __forceinline__ void level_steps(Lanes<T, W>* lv, std::index_sequence<S...>) {
    (
        [&] {
            if constexpr (kLevelReady<B, S> == b)
                lv[B + S] = combine<Op, T, W>(lv[kStepA<sched::kScan, B, S>], lv[kStepB<sched::kScan, B, S>]);
        }(),
        ...);
}

template <class T, int W, size_t... Q>
__device__ __forceinline__ void load_block(Lanes<T, W>* x, const BlockedScanPtrs& ptrs, int b, size_t elem,
                                           std::index_sequence<Q...>) {
    ((x[Q] = load_lanes<kFusedNT, T, W>(static_cast<const T*>(ptrs.in[b * BL + Q]) + elem)), ...);
}

template <class Op, class T, int W, int B, int b>
__device__ __forceinline__ void scan_block(const BlockedScanPtrs& ptrs, size_t elem, Lanes<T, W>* lv,
                                           Lanes<T, W>& carry) {
    using L = Lanes<T, W>;
    if constexpr (b == 0) {
        L v[BL + kNumSteps<sched::kScan, BL>];
        load_block<T, W>(v, ptrs, 0, elem, std::make_index_sequence<BL>{});
        run_steps<Op, T, W, sched::kScan, BL>(v, std::make_index_sequence<kNumSteps<sched::kScan, BL>>{});
        [&]<size_t... R>(std::index_sequence<R...>) {
            ((store_lanes<kFusedNT, T, W>(static_cast<T*>(ptrs.out[R]) + elem, v[kOut<sched::kScan, BL, R>])), ...);
        }(std::make_index_sequence<BL>{});
        lv[0] = v[kOut<sched::kScan, BL, BL - 1>];
        carry = lv[0];
    } else {
        L x[BL];
        load_block<T, W>(x, ptrs, b, elem, std::make_index_sequence<BL>{});
        // T_b: reduce program over the block in reverse order (value j = peer 16 b + 15 - j)
        L rv[BL + kNumSteps<sched::kReduce, BL>];
        [&]<size_t... J>(std::index_sequence<J...>) { ((rv[J] = x[BL - 1 - J]), ...); }(std::make_index_sequence<BL>{});
        run_steps<Op, T, W, sched::kReduce, BL>(rv, std::make_index_sequence<kNumSteps<sched::kReduce, BL>>{});
        lv[b] = rv[kOut<sched::kReduce, BL, 0>];
        level_steps<Op, T, W, B, b>(lv, std::make_index_sequence<kNumSteps<sched::kScan, B>>{});
        const L sb = lv[kOut<sched::kScan, B, b>];
        // the block's first 15 outputs: the carry program from S_{b-1} (value 0) over inputs q = 0..14
        L cv[BL + kNumSteps<sched::kScanCarry, BL>];
        cv[0] = carry;
        [&]<size_t... Q>(std::index_sequence<Q...>) { ((cv[1 + Q] = x[Q]), ...); }(std::make_index_sequence<BL - 1>{});
        run_steps<Op, T, W, sched::kScanCarry, BL>(cv, std::make_index_sequence<kNumSteps<sched::kScanCarry, BL>>{});
        [&]<size_t... Q>(std::index_sequence<Q...>) {
            ((store_lanes<kFusedNT, T, W>(static_cast<T*>(ptrs.out[b * BL + Q]) + elem, cv[kOut<sched::kScanCarry, BL, Q + 1>])),
             ...);
        }(std::make_index_sequence<BL - 1>{});
        store_lanes<kFusedNT, T, W>(static_cast<T*>(ptrs.out[b * BL + BL - 1]) + elem, sb);
        carry = sb;
    }
}

template <class Op, class T, int W, int B>
__device__ __forceinline__ void scan_blocks_group(const BlockedScanPtrs& ptrs, size_t elem) {
    Lanes<T, W> lv[B + kNumSteps<sched::kScan, B>];
    Lanes<T, W> carry;
    [&]<int... b>(std::integer_sequence<int, b...>) {
        (scan_block<Op, T, W, B, b>(ptrs, elem, lv, carry), ...);
    }(std::make_integer_sequence<int, B>{});
}

template <class Op, class T, int B>
__global__ void __launch_bounds__(256) scan_blocks_kernel(BlockedScanPtrs ptrs, size_t n) {
    constexpr int W = kVecLanes<T>;
    const size_t nvec = n / W;
    const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
    for (size_t g = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; g < nvec; g += stride)
        scan_blocks_group<Op, T, W, B>(ptrs, g * W);
    const size_t first = nvec * W;
    if (blockIdx.x == 0 && first + threadIdx.x < n) scan_blocks_group<Op, T, 1, B>(ptrs, first + threadIdx.x);
}

using BlocksFn = void (*)(const BlockedScanPtrs&, size_t, hipStream_t);

template <class Op, class T, int B>
void blocks_one(const BlockedScanPtrs& ptrs, size_t n, hipStream_t s) {
    const size_t nvec = n / kVecLanes<T>;
    const unsigned grid = static_cast<unsigned>(std::min<size_t>(grid_for(nvec, kFusedBlock), kFusedGridCap));
    // one block's 16 streams in flight per thread at a time: the residency of the 16-peer fused kernels
    const size_t lds = fused_lds_bytes(BL, kFusedBlock * 16);
    scan_blocks_kernel<Op, T, B><<<grid, kFusedBlock, lds, s>>>(ptrs, n);
}


// Launch table for B in [LO, HI] full blocks.
template <int LO, int HI>
int launch_range(int op, int dtype, int B, const BlockedScanPtrs& ptrs, size_t n, hipStream_t s) {
    if (B < LO || B > HI)
        return fail(FMI_ERR_INVALID, "one-pass blocked scan: B = " + std::to_string(B) + " outside [" +
                                         std::to_string(LO) + ", " + std::to_string(HI) + "]");
    return with_op_dtype<false>(op, dtype, [&]<class Op, class T>() -> int {
        static constexpr auto table = []<int... I>(std::integer_sequence<int, I...>) {
            return std::array<BlocksFn, sizeof...(I)>{&blocks_one<Op, T, I + LO>...};
        }(std::make_integer_sequence<int, HI - LO + 1>{});
        table[B - LO](ptrs, n, s);
        return check_launch("one-pass blocked scan launch");
    });
}

}  // namespace fmi::dev::scan_blocks
