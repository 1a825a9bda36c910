// fmi_internal.h — declarations shared by the translation units of libfmi_dev.so (not installed).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <exception>
#include <new>
#include <string>

#include "../../include/fmi_dev.h"
#include "fmi_kernels.h"

namespace fmi::dev {

// Records a failure message for fmi_last_error() and returns `code`.
int fail(int code, const std::string& msg);

// Runs a C-ABI entry point's body: no C++ exception may cross the extern "C" boundary (it would call
// std::terminate in the caller). std::bad_alloc (e.g. a host program or expression for millions of peers)
// becomes FMI_ERR_ALLOC, anything else FMI_ERR_INVALID, with the message for fmi_last_error().
template <class F>
int guarded(const char* what, F&& body) noexcept {
    try {
        return body();
    } catch (const std::bad_alloc&) {
        return fail(FMI_ERR_ALLOC, std::string(what) + ": out of host memory");
    } catch (const std::exception& e) {
        return fail(FMI_ERR_INVALID, std::string(what) + ": " + e.what());
    } catch (...) {
        return fail(FMI_ERR_INVALID, std::string(what) + ": unknown exception");
    }
}

// The library's default stream (what a NULL fmi_stream_t means); nullptr before fmi_dev_init.
hipStream_t library_stream();

// Dynamic LDS a fused P-way launch reserves (the kernels use none) so that the peer loads its resident
// workgroups keep in flight per CU stay within FMI_TUNE_FUSED_INFLIGHT_KIB: fewer concurrent HBM streams
// at large P, better DRAM row locality. `wg_load_bytes_per_peer` = bytes one workgroup loads per peer.
size_t fused_lds_bytes(int P, size_t wg_load_bytes_per_peer);
int fused_policy(bool scan, int P);  // FMI_TUNE_FUSED_POLICY: the fused kernels' `pol` argument

// The dtypes every kernel is instantiated for (the fused P-way kernels included).
inline bool is_core_dtype(int dtype) { return dtype >= FMI_F32 && dtype <= FMI_I64; }

// Invoke f.template operator()<T>() for a runtime dtype (ALL: every fmi_dtype_t; else the core four);
// returns FMI_ERR_INVALID if unknown.
template <bool ALL, class F>
int with_dtype(int dtype, F&& f) {
    switch (dtype) {
        case FMI_F32: return f.template operator()<float>();
        case FMI_F64: return f.template operator()<double>();
        case FMI_I32: return f.template operator()<int32_t>();
        case FMI_I64: return f.template operator()<int64_t>();
        default: break;
    }
    if constexpr (ALL) {
        switch (dtype) {
            case FMI_U32: return f.template operator()<uint32_t>();
            case FMI_U64: return f.template operator()<uint64_t>();
            case FMI_I8: return f.template operator()<int8_t>();
            case FMI_U8: return f.template operator()<uint8_t>();
            case FMI_I16: return f.template operator()<int16_t>();
            case FMI_U16: return f.template operator()<uint16_t>();
            default: break;
        }
    }
    return fail(FMI_ERR_INVALID, "unknown dtype " + std::to_string(dtype));
}

// Invoke f.template operator()<Op, T>() for a runtime (op, dtype); returns FMI_ERR_INVALID if unknown.
template <bool ALL = true, class F>
int with_op_dtype(int op, int dtype, F&& f) {
    auto by_dtype = [&]<class Op>() -> int {
        return with_dtype<ALL>(dtype, [&]<class T>() -> int { return f.template operator()<Op, T>(); });
    };
    switch (op) {
        case FMI_OP_SUM: return by_dtype.template operator()<OpSum>();
        case FMI_OP_PROD: return by_dtype.template operator()<OpProd>();
        case FMI_OP_MAX: return by_dtype.template operator()<OpMax>();
        case FMI_OP_MIN: return by_dtype.template operator()<OpMin>();
        default: return fail(FMI_ERR_INVALID, "unknown op " + std::to_string(op));
    }
}

inline size_t dtype_size(int dtype) {
    switch (dtype) {
        case FMI_F32: case FMI_I32: case FMI_U32: return 4;
        case FMI_F64: case FMI_I64: case FMI_U64: return 8;
        case FMI_I8: case FMI_U8: return 1;
        case FMI_I16: case FMI_U16: return 2;
        default: return 0;
    }
}

inline bool is_float(int dtype) { return dtype == FMI_F32 || dtype == FMI_F64; }

// Fused single-pass launches (P in [2, kMaxFusedPeers], all pointers 16-B aligned). One function per
// algorithm family, each defined in its own translation unit so the ~1.2k instantiations build in
// parallel. Return 0 or a negative fmi_status_t.
int launch_fused_allreduce(int op, int dtype, int P, const PeerPtrs& ptrs, size_t n, int rank, hipStream_t s);
// a 16-peer allreduce block whose peers all pre-fold a partner: ins[0..16) the block, ins[16..32) the
// partners; out[0] = the value of block peer `rank` (< 16)
int launch_fused_allreduce_prefold16(int op, int dtype, const PeerPtrs& ptrs, size_t n, int rank, hipStream_t s);
// allreduce_no_order's value for every peer at once (outs[r] for r < P), float max / min only
int launch_fused_allreduce_all_ranks(int op, int dtype, int P, const PeerPtrs& ptrs, size_t n, hipStream_t s);
// float max / min: which operand is kept on a tie (±0) or a NaN depends on the order, so every peer of an
// allreduce can end with different bits
inline bool order_sensitive(int op, int dtype) { return is_float(dtype) && (op == FMI_OP_MAX || op == FMI_OP_MIN); }
// allreduce for P = 17..31 (the pre-folded programs), reached through launch_fused_allreduce
int launch_fused_allreduce_wide(int op, int dtype, int P, const PeerPtrs& ptrs, size_t n, int rank, hipStream_t s);
int launch_fused_reduce(int op, int dtype, int P, const PeerPtrs& ptrs, size_t n, hipStream_t s);
int launch_fused_reduce_ltr(int op, int dtype, int P, const PeerPtrs& ptrs, size_t n, hipStream_t s);
// reduce_no_order with every (transformed) peer's final sendbuf stored: ptrs.out[t] for t < P
int launch_fused_reduce_partials(int op, int dtype, int P, const PeerPtrs& ptrs, size_t n, hipStream_t s);
// The same for any P and any alignment / dtype (fused kernel where it applies, pairwise passes otherwise):
// outs[t] = the value transformed peer t of reduce_no_order holds in its sendbuf at the end
// (src/comm/PeerToPeer.cpp:66-78); ins in transformed order. Defined in fmi_dev.hip.
int reduce_partials(int op, int dtype, void* const* outs, const void* const* ins, int P, size_t n, hipStream_t s);
int launch_fused_scan(int op, int dtype, int P, const PeerPtrs& ptrs, size_t n, hipStream_t s);
int launch_fused_scan_ltr(int op, int dtype, int P, const PeerPtrs& ptrs, size_t n, hipStream_t s);
// scans for P = 17..31 (alg = sched::kScan or kScanLtr), reached through the two launches above
int launch_fused_scan_wide(int op, int dtype, int alg, int P, const PeerPtrs& ptrs, size_t n, hipStream_t s);
// Blocks of a scan beyond 16 peers (sched::kScanCarry / kScanLtrCarry): ptrs.in[0] is the carry, out[0] unused.
int launch_fused_scan_carry(int op, int dtype, int P, const PeerPtrs& ptrs, size_t n, hipStream_t s);
int launch_fused_scan_ltr_carry(int op, int dtype, int P, const PeerPtrs& ptrs, size_t n, hipStream_t s);
// scan_no_order over B full blocks of 16 peers (2 <= B <= kMaxOnePassScanBlocks, P = 32..143) in one pass: every input read
// once, all 16 B outputs written (fmi_fused_scan_blocked.hip); a ragged last block is left to the caller.
inline constexpr int kMaxOnePassScanBlocks = 8;
inline constexpr int kOnePassScanBlocksNarrow = 4;  // B <= 4 in one translation unit, 5..8 in another
struct BlockedScanPtrs {
    const void* in[sched::kScanBlock * kMaxOnePassScanBlocks];
    void* out[sched::kScanBlock * kMaxOnePassScanBlocks];
};
int launch_scan_blocks_one_pass(int op, int dtype, int B, const BlockedScanPtrs& ptrs, size_t n, hipStream_t s);
int launch_scan_blocks_one_pass_wide(int op, int dtype, int B, const BlockedScanPtrs& ptrs, size_t n, hipStream_t s);
// reduce_no_order over any 17..128 peers (ragged last block included) and allreduce_no_order over P = 32, 64, 128
// in one pass: ptrs.in[0..P) the (transformed) inputs, ptrs.out[0] the result of peer `rank` (allreduce)
// (fmi_fused_tree_blocked.hip)
bool tree_blocks_one_pass_covers(int op, int dtype, int alg, int P);
// allreduce_no_order over P = 48, 80, 96, 112 (full blocks pre-fold) in one pass: ptrs.in[0..2^k) the doubling
// group and ptrs.in[2^k..P) the partners, each block permuted by rank % 16 by the caller; rank_hi = rank / 16
bool prefold_blocks_one_pass_covers(int alg, int P);
int launch_prefold_blocks_one_pass(int op, int dtype, int P, const BlockedScanPtrs& ptrs, size_t n, int rank_hi,
                                   hipStream_t s);
// scan_ltr (scan = true: ptrs.out[0..P)) and reduce_ltr (ptrs.out[0]) over 2..128 peers in one pass, the running
// value carried in registers (fmi_fused_chain.hip)
// carry_in: ptrs.in[0] is an earlier segment's running value (scan: ptrs.out[0] is not written).
int launch_chain_one_pass(int op, int dtype, bool scan, int P, const BlockedScanPtrs& ptrs, size_t n, hipStream_t s,
                          bool carry_in = false);
int launch_tree_blocks_one_pass(int op, int dtype, int alg, int P, const BlockedScanPtrs& ptrs, size_t n, int rank,
                                hipStream_t s);

// Many independent pairwise combines in one launch (fmi_dev_reduce_pair_batch, fmi_pair_batch.hip): up to
// kPairBatchMax descriptors, every pointer 16-B aligned; workgroup t works on tile t - first_tile[k] of the
// descriptor k with first_tile[k] <= t < first_tile[k + 1] (kPairBatchTile lane groups per tile).
inline constexpr int kPairBatchMax = 64;
inline constexpr unsigned kPairBatchBlock = 256;
inline constexpr int kPairBatchUnroll = 4;
inline constexpr size_t kPairBatchTile = size_t(kPairBatchBlock) * kPairBatchUnroll;
struct PairBatch {
    void* inout[kPairBatchMax];
    const void* in[kPairBatchMax];
    unsigned long long n[kPairBatchMax];         // elements
    unsigned first_tile[kPairBatchMax + 1];      // prefix sums of the descriptors' tile counts
    int count;
};
int launch_pair_batch(int op, int dtype, const PairBatch& pb, hipStream_t s);

// dst <- src (bytes) on stream s: the copy_tile kernel (nontemporal, ≈ the chip's copy rate) when both are
// 16-B aligned, non-overlapping device allocations of >= kDeviceCopyMin bytes; hipMemcpyAsync otherwise
// (host or unknown pointers, small or overlapping copies).
inline constexpr size_t kDeviceCopyMin = size_t(256) << 10;
int device_copy(void* dst, const void* src, size_t bytes, hipStream_t s);

// Workgroups to cover `items` with `block` threads each (at least 1). Callers cap it before narrowing.
inline size_t grid_for(size_t items, unsigned block) {
    const size_t g = (items + block - 1) / block;
    return g == 0 ? 1 : g;
}

}  // namespace fmi::dev
