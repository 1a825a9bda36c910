// One-pass tree reductions over B full blocks of 16 peers (P = 16 B, 2 <= B <= kMaxOnePassScanBlocks):
// reduce_no_order (reference src/comm/PeerToPeer.cpp:59-84) for any such P, allreduce_no_order (:96-130) for
// P = 32, 64, 128 (no pre-fold). tree_blocked (fmi_dev.hip) evaluates the same bracketing as a launch per
// block, each writing its block value to a temp, then a launch over the B temps: P + 2 B + 1 bucket passes.
// Here one thread computes its lane group's B block values in registers and then the block-level program:
// P + 1 passes. Same programs, same operand order, so the same bits.
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

using TreeBlocksFn = void (*)(const BlockedScanPtrs&, size_t, int, hipStream_t);

template <class Op, class T, int ALG, int B, bool ALL_RANKS = false>
void tree_blocks_one(const BlockedScanPtrs& ptrs, size_t n, int rank, hipStream_t s) {
    const size_t nvec = n / kVecLanes<T>;
    const unsigned grid = static_cast<unsigned>(std::min<size_t>(grid_for(nvec, kFusedBlock), kFusedGridCap));
    const size_t lds = fused_lds_bytes(BL, kFusedBlock * 16);  // one block's 16 streams in flight at a time
    tree_blocks_kernel<Op, T, ALG, B, ALL_RANKS><<<grid, kFusedBlock, lds, s>>>(ptrs, n, rank);
}

}  // namespace

bool tree_blocks_one_pass_covers(int op, int dtype, int alg, int P) {
    if (P % BL != 0) return false;
    const int B = P / BL;
    if (B < 2 || B > kMaxOnePassScanBlocks) return false;
    if (alg == FMI_ALG_REDUCE) return true;
    return alg == FMI_ALG_ALLREDUCE && (B & (B - 1)) == 0;
}

int launch_tree_blocks_one_pass(int op, int dtype, int alg, int P, const BlockedScanPtrs& ptrs, size_t n, int rank,
                                hipStream_t s) {
    if (!tree_blocks_one_pass_covers(op, dtype, alg, P))
        return fail(FMI_ERR_INVALID, "one-pass blocked tree: unsupported (alg, P, op, dtype)");
    const int B = P / BL;
    return with_op_dtype<false>(op, dtype, [&]<class Op, class T>() -> int {
        static constexpr TreeBlocksFn reduce_table[] = {
            &tree_blocks_one<Op, T, sched::kReduce, 2>, &tree_blocks_one<Op, T, sched::kReduce, 3>,
            &tree_blocks_one<Op, T, sched::kReduce, 4>, &tree_blocks_one<Op, T, sched::kReduce, 5>,
            &tree_blocks_one<Op, T, sched::kReduce, 6>, &tree_blocks_one<Op, T, sched::kReduce, 7>,
            &tree_blocks_one<Op, T, sched::kReduce, 8>};
        static_assert(kMaxOnePassScanBlocks == 8, "tables cover B = 2..8");
        constexpr bool ranked = std::is_floating_point_v<T> && (std::is_same_v<Op, OpMax> || std::is_same_v<Op, OpMin>);
        if (alg == FMI_ALG_REDUCE) {
            reduce_table[B - 2](ptrs, n, 0, s);
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

}  // namespace fmi::dev
