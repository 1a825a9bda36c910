// One-pass tree reductions beyond the fused kernels, up to 128 peers (blocks of 16 peers):
// reduce_no_order (reference src/comm/PeerToPeer.cpp:59-84; any 17..128 peers, ragged last block included,
// reduce_any_kernel below), allreduce_no_order (:96-130) for
// P = 32, 64, 128 (no pre-fold) and, in prefold_blocks_kernel, P = 48, 80, 96, 112 (whole blocks pre-fold).
// tree_blocked (fmi_dev.hip) evaluates the same bracketing as a launch per block, each writing its block value
// to a temp, then a launch over the B temps: P + 2 B + 1 bucket passes. Here one thread computes its lane
// group's block values in registers and then the block-level program: P + 1 passes. Same programs, same
// operand order, so the same bits.
//   reduce:     binomial rounds 0..3 stay inside each block (the block's 16-peer reduce program); rounds 4..
//               combine the block values at spans 16, 32, ..: the reduce program over the B values.
//   allreduce:  recursive-doubling rounds 0..3 give position p the block's 16-peer allreduce for rank p % 16;
//               rounds 4.. pair positions with equal p % 16: the allreduce program over B values for rank
//               p / 16. Where the bits depend on the rank (float max / min on ±0 / NaN) each block keeps the
//               value of rank % 16 and the block level that of rank / 16 (pick_rank, as the fused kernels);
//               otherwise rank 0's expression is every rank's.
#include "fmi_fused_impl.h"

namespace fmi::dev {
namespace {

constexpr int BL = sched::kScanBlock;  // 16

// Block b's 16-peer program value (its inputs loaded once): the value of block rank `r`.
template <class Op, class T, int W, int ALG, bool ALL_RANKS, size_t... Q>
__device__ __forceinline__ Lanes<T, W> block_value(const BlockedScanPtrs& ptrs, int b, int r, size_t elem,
                                                   std::index_sequence<Q...>) {
    Lanes<T, W> v[BL + kNumSteps<ALG, BL>];
    ((v[Q] = load_lanes<kFusedNT, T, W>(static_cast<const T*>(ptrs.in[b * BL + Q]) + elem)), ...);
    run_steps<Op, T, W, ALG, BL>(v, std::make_index_sequence<kNumSteps<ALG, BL>>{});
    if constexpr (ALL_RANKS)
        return pick_rank<T, W, ALG, BL>(v, r, std::make_index_sequence<BL>{});
    else
        return v[kOut<ALG, BL, 0>];
}

template <class Op, class T, int W, int ALG, int B, bool ALL_RANKS, size_t... b>
__device__ __forceinline__ void tree_blocks_group(const BlockedScanPtrs& ptrs, int rank, size_t elem,
                                                  std::index_sequence<b...>) {
    using L = Lanes<T, W>;
    L bv[B + kNumSteps<ALG, B>];
    ((bv[b] = block_value<Op, T, W, ALG, ALL_RANKS>(ptrs, static_cast<int>(b), rank % BL, elem,
                                                     std::make_index_sequence<BL>{})),
     ...);
    run_steps<Op, T, W, ALG, B>(bv, std::make_index_sequence<kNumSteps<ALG, B>>{});
    L r;
    if constexpr (ALL_RANKS)
        r = pick_rank<T, W, ALG, B>(bv, rank / BL, std::make_index_sequence<B>{});
    else
        r = bv[kOut<ALG, B, 0>];
    store_lanes<kFusedNT, T, W>(static_cast<T*>(ptrs.out[0]) + elem, r);
}

template <class Op, class T, int ALG, int B, bool ALL_RANKS>
__global__ void __launch_bounds__(256) tree_blocks_kernel(BlockedScanPtrs ptrs, size_t n, int rank) {
    constexpr int W = kVecLanes<T>;
    const size_t nvec = n / W;
    const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
    for (size_t g = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; g < nvec; g += stride)
        tree_blocks_group<Op, T, W, ALG, B, ALL_RANKS>(ptrs, rank, g * W, std::make_index_sequence<B>{});
    const size_t first = nvec * W;
    if (blockIdx.x == 0 && first + threadIdx.x < n)
        tree_blocks_group<Op, T, 1, ALG, B, ALL_RANKS>(ptrs, rank, first + threadIdx.x, std::make_index_sequence<B>{});
}

template <class Op, class T, int ALG, int B, bool ALL_RANKS = false>
void tree_blocks_one(const BlockedScanPtrs& ptrs, size_t n, int rank, hipStream_t s) {
    const size_t nvec = n / kVecLanes<T>;
    const unsigned grid = static_cast<unsigned>(std::min<size_t>(grid_for(nvec, kFusedBlock), kFusedGridCap));
    const size_t lds = fused_lds_bytes(BL, kFusedBlock * 16);  // one block's 16 streams in flight at a time
    tree_blocks_kernel<Op, T, ALG, B, ALL_RANKS><<<grid, kFusedBlock, lds, s>>>(ptrs, n, rank);
}

// allreduce_no_order over P = 2^k + 16 F peers (F full blocks pre-fold a partner, :100-107): block b < F is the
// 32-input kAllreducePrefold16 program over its 16 peers and their partners 2^k + 16 b + q, the other blocks the
// 16-peer recursive doubling; then the doubling over the B = 2^k / 16 block values. The caller permutes each
// block's pointers by rank % 16 (the doubling is symmetric under p -> p ^ rank, partners move along), so every
// block value is rank 0's expression; the block level keeps rank / 16's value where the bits depend on it.
template <class Op, class T, int W, int B, bool PREFOLD>
__device__ __forceinline__ Lanes<T, W> prefold_block_value(const BlockedScanPtrs& ptrs, int b, size_t elem) {
    constexpr int ALG = PREFOLD ? sched::kAllreducePrefold16 : sched::kAllreduce;
    constexpr int NIN = PREFOLD ? 2 * BL : BL;
    Lanes<T, W> v[NIN + kNumSteps<ALG, NIN>];
    [&]<size_t... Q>(std::index_sequence<Q...>) {
        ((v[Q] = load_lanes<kFusedNT, T, W>(static_cast<const T*>(ptrs.in[b * BL + Q]) + elem)), ...);
        if constexpr (PREFOLD)
            ((v[BL + Q] = load_lanes<kFusedNT, T, W>(static_cast<const T*>(ptrs.in[B * BL + b * BL + Q]) + elem)), ...);
    }(std::make_index_sequence<BL>{});
    run_steps<Op, T, W, ALG, NIN>(v, std::make_index_sequence<kNumSteps<ALG, NIN>>{});
    return v[kOut<ALG, NIN, 0>];
}

template <class Op, class T, int W, int B, int F, bool RANKED, size_t... b>
__device__ __forceinline__ void prefold_blocks_group(const BlockedScanPtrs& ptrs, int rank_hi, size_t elem,
                                                     std::index_sequence<b...>) {
    using L = Lanes<T, W>;
    L bv[B + kNumSteps<sched::kAllreduce, B>];
    ((bv[b] = prefold_block_value<Op, T, W, B, (static_cast<int>(b) < F)>(ptrs, static_cast<int>(b), elem)), ...);
    run_steps<Op, T, W, sched::kAllreduce, B>(bv, std::make_index_sequence<kNumSteps<sched::kAllreduce, B>>{});
    L r;
    if constexpr (RANKED)
        r = pick_rank<T, W, sched::kAllreduce, B>(bv, rank_hi, std::make_index_sequence<B>{});
    else
        r = bv[kOut<sched::kAllreduce, B, 0>];
    store_lanes<kFusedNT, T, W>(static_cast<T*>(ptrs.out[0]) + elem, r);
}

template <class Op, class T, int B, int F, bool RANKED>
__global__ void __launch_bounds__(256) prefold_blocks_kernel(BlockedScanPtrs ptrs, size_t n, int rank_hi) {
    constexpr int W = kVecLanes<T>;
    const size_t nvec = n / W;
    const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
    for (size_t g = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; g < nvec; g += stride)
        prefold_blocks_group<Op, T, W, B, F, RANKED>(ptrs, rank_hi, g * W, std::make_index_sequence<B>{});
    const size_t first = nvec * W;
    if (blockIdx.x == 0 && first + threadIdx.x < n)
        prefold_blocks_group<Op, T, 1, B, F, RANKED>(ptrs, rank_hi, first + threadIdx.x, std::make_index_sequence<B>{});
}

template <class Op, class T, int B, int F, bool RANKED>
void prefold_blocks_one(const BlockedScanPtrs& ptrs, size_t n, int rank_hi, hipStream_t s) {
    const size_t nvec = n / kVecLanes<T>;
    const unsigned grid = static_cast<unsigned>(std::min<size_t>(grid_for(nvec, kFusedBlock), kFusedGridCap));
    const size_t lds = fused_lds_bytes(2 * BL, kFusedBlock * 16);  // a pre-fold block's 32 streams at a time
    prefold_blocks_kernel<Op, T, B, F, RANKED><<<grid, kFusedBlock, lds, s>>>(ptrs, n, rank_hi);
}

// reduce_no_order over any 17..128 peers in one kernel: the binomial rounds with compile-time operand indices
// and a uniform runtime guard `t + span < m`, which is exactly the m-peer program's step list (the fused
// kReduce program restricted to the steps whose right operand exists). Block b (m_b = min(16, P - 16 b)
// peers) is reduced that way, then the ceil(P / 16) block values likewise: tree_blocked's bracketing,
// ragged last block included.
template <class Op, class T, int W, int N>
__device__ __forceinline__ void binomial_reduce(Lanes<T, W>* v, int m) {
#pragma unroll
    for (int span = 1; span < N; span *= 2) {
#pragma unroll
        for (int t = 0; t + span < N; t += 2 * span)
            if (t + span < m) v[t] = combine<Op, T, W>(v[t], v[t + span]);
    }
}

template <class Op, class T, int W>
__device__ __forceinline__ void reduce_any_group(const BlockedScanPtrs& ptrs, int P, size_t elem) {
    using L = Lanes<T, W>;
    constexpr int NB = kMaxOnePassScanBlocks;
    const int nb = (P + BL - 1) / BL;
    L bv[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        if (b < nb) {
            const int m = P - b * BL < BL ? P - b * BL : BL;
            L v[BL];
#pragma unroll
            for (int q = 0; q < BL; ++q)
                if (q < m) v[q] = load_lanes<kFusedNT, T, W>(static_cast<const T*>(ptrs.in[b * BL + q]) + elem);
            binomial_reduce<Op, T, W, BL>(v, m);
            bv[b] = v[0];
        }
    }
    binomial_reduce<Op, T, W, NB>(bv, nb);
    store_lanes<kFusedNT, T, W>(static_cast<T*>(ptrs.out[0]) + elem, bv[0]);
}

template <class Op, class T>
__global__ void __launch_bounds__(256) reduce_any_kernel(BlockedScanPtrs ptrs, int P, size_t n) {
    constexpr int W = kVecLanes<T>;
    const size_t nvec = n / W;
    const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
    for (size_t g = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; g < nvec; g += stride)
        reduce_any_group<Op, T, W>(ptrs, P, g * W);
    const size_t first = nvec * W;
    if (blockIdx.x == 0 && first + threadIdx.x < n) reduce_any_group<Op, T, 1>(ptrs, P, first + threadIdx.x);
}

}  // namespace

bool tree_blocks_one_pass_covers(int op, int dtype, int alg, int P) {
    if (alg == FMI_ALG_REDUCE) return P > sched::kMaxFusedPeers && P <= kMaxOnePassScanBlocks * BL;
    if (alg != FMI_ALG_ALLREDUCE || P % BL != 0) return false;
    const int B = P / BL;
    return B >= 2 && B <= kMaxOnePassScanBlocks && (B & (B - 1)) == 0;
}

int launch_tree_blocks_one_pass(int op, int dtype, int alg, int P, const BlockedScanPtrs& ptrs, size_t n, int rank,
                                hipStream_t s) {
    if (!tree_blocks_one_pass_covers(op, dtype, alg, P))
        return fail(FMI_ERR_INVALID, "one-pass blocked tree: unsupported (alg, P, op, dtype)");
    const int B = P / BL;
    return with_op_dtype<false>(op, dtype, [&]<class Op, class T>() -> int {
        static_assert(kMaxOnePassScanBlocks == 8, "allreduce covers B = 2, 4, 8");
        constexpr bool ranked = std::is_floating_point_v<T> && (std::is_same_v<Op, OpMax> || std::is_same_v<Op, OpMin>);
        if (alg == FMI_ALG_REDUCE) {
            const size_t nvec = n / kVecLanes<T>;
            const unsigned grid = static_cast<unsigned>(std::min<size_t>(grid_for(nvec, kFusedBlock), kFusedGridCap));
            reduce_any_kernel<Op, T><<<grid, kFusedBlock, fused_lds_bytes(BL, kFusedBlock * 16), s>>>(ptrs, P, n);
        } else {
            switch (B) {
                case 2: tree_blocks_one<Op, T, sched::kAllreduce, 2, ranked>(ptrs, n, rank, s); break;
                case 4: tree_blocks_one<Op, T, sched::kAllreduce, 4, ranked>(ptrs, n, rank, s); break;
                default: tree_blocks_one<Op, T, sched::kAllreduce, 8, ranked>(ptrs, n, rank, s); break;
            }
        }
        return check_launch("one-pass blocked tree launch");
    });
}

bool prefold_blocks_one_pass_covers(int alg, int P) {
    if (alg != FMI_ALG_ALLREDUCE || P > kMaxOnePassScanBlocks * BL) return false;
    const int pow2 = 1 << sched::floor_log2(P);
    const int folded = P - pow2;
    return (pow2 == 32 || pow2 == 64) && folded > 0 && folded % BL == 0;
}

int launch_prefold_blocks_one_pass(int op, int dtype, int P, const BlockedScanPtrs& ptrs, size_t n, int rank_hi,
                                   hipStream_t s) {
    if (!prefold_blocks_one_pass_covers(FMI_ALG_ALLREDUCE, P))
        return fail(FMI_ERR_INVALID, "one-pass pre-fold allreduce: unsupported P = " + std::to_string(P));
    const int pow2 = 1 << sched::floor_log2(P);
    const int F = (P - pow2) / BL;
    return with_op_dtype<false>(op, dtype, [&]<class Op, class T>() -> int {
        constexpr bool ranked = std::is_floating_point_v<T> && (std::is_same_v<Op, OpMax> || std::is_same_v<Op, OpMin>);
        if (pow2 == 32) {
            prefold_blocks_one<Op, T, 2, 1, ranked>(ptrs, n, rank_hi, s);
        } else {
            switch (F) {
                case 1: prefold_blocks_one<Op, T, 4, 1, ranked>(ptrs, n, rank_hi, s); break;
                case 2: prefold_blocks_one<Op, T, 4, 2, ranked>(ptrs, n, rank_hi, s); break;
                default: prefold_blocks_one<Op, T, 4, 3, ranked>(ptrs, n, rank_hi, s); break;
            }
        }
        return check_launch("one-pass pre-fold allreduce launch");
    });
}

}  // namespace fmi::dev
