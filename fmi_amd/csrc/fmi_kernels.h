// fmi_kernels.h — gfx950 (CDNA4) kernels for FMI's bucket reduction.
//
// All kernels here are HBM-streaming element-wise kernels (≈1/12 flop per byte for f32 add): there is
// no dense contraction, so no MFMA and no LDS staging — the work is to keep enough 16-byte
// loads in flight per CU that HBM3E, not latency, is the limit (MI355X_MICROARCH.md §HBM).
//
//   pair_tile / pair_stride   out[i] = op(a[i], b[i])          one pass: 2 reads + 1 write per element
//   tree_kernel               out    = program(x0..x{P-1})     one pass: P reads + 1 write
//   scan_kernel               outs[k]= program_k(x0..x{P-1})   one pass: P reads + P writes
//   synth_kernel              counter-based synthetic buckets (splitmix64), identical to the host
//
// Every access is a 16-B global_load_dwordx4 / global_store_dwordx4 (4 f32/i32 or 2 f64/i64 lanes);
// the < 16-B remainder of a bucket is handled by the first threads of block 0 with scalar accesses,
// so a launch never touches a byte outside [0, n).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <type_traits>
#include <utility>

#include "fmi_schedule.h"

namespace fmi::dev {

// ---------------------------------------------------------------------------------------------------
// Element ops. Semantics are the reference's built-ins (reference python/PythonCommunicator.h:131-149):
// std::plus, std::multiplies, std::max(a,b) = (a<b)?b:a, std::min(a,b) = (b<a)?b:a — NOT fmaxf/fminf,
// which differ on NaN and on signed zeros. Integer sum/prod wrap (computed in the unsigned type).
// ---------------------------------------------------------------------------------------------------
template <class T>
struct Wrap {
    using type = T;
};
template <>
struct Wrap<int32_t> {
    using type = uint32_t;
};
template <>
struct Wrap<int64_t> {
    using type = uint64_t;
};
// Sub-dword integers compute in 32 bits (no promotion to a signed int that could overflow) and keep the
// low bits on conversion back, as the reference's std::plus / std::multiplies on A do.
template <>
struct Wrap<int8_t> {
    using type = uint32_t;
};
template <>
struct Wrap<uint8_t> {
    using type = uint32_t;
};
template <>
struct Wrap<int16_t> {
    using type = uint32_t;
};
template <>
struct Wrap<uint16_t> {
    using type = uint32_t;
};

struct OpSum {
    template <class T>
    __device__ __forceinline__ static T apply(T a, T b) {
        using U = typename Wrap<T>::type;
        return static_cast<T>(static_cast<U>(a) + static_cast<U>(b));
    }
};
struct OpProd {
    template <class T>
    __device__ __forceinline__ static T apply(T a, T b) {
        using U = typename Wrap<T>::type;
        return static_cast<T>(static_cast<U>(a) * static_cast<U>(b));
    }
};
struct OpMax {
    template <class T>
    __device__ __forceinline__ static T apply(T a, T b) {
        return (a < b) ? b : a;
    }
};
struct OpMin {
    template <class T>
    __device__ __forceinline__ static T apply(T a, T b) {
        return (b < a) ? b : a;
    }
};

// ---------------------------------------------------------------------------------------------------
// 16-byte lane groups and their loads/stores.
// ---------------------------------------------------------------------------------------------------
// Sub-dword elements are held as a clang vector (<16 x i8>, <8 x i16>): reinterpreting one as 32-bit
// words is then free, where a plain array is split per element and reassembled (it turned the 16-B loads
// of the 8-bit kernels into 2-byte ones).
template <class T, int W, bool VEC = (sizeof(T) < 4 && W > 1)>
struct LaneStorage {
    T v[W];
};
template <class T, int W>
struct LaneStorage<T, W, true> {
    T __attribute__((ext_vector_type(W))) v;
};

template <class T, int W>
struct alignas(sizeof(T) * W) Lanes : LaneStorage<T, W> {};

template <class T>
inline constexpr int kVecLanes = 16 / static_cast<int>(sizeof(T));

using u32x4 = unsigned int __attribute__((ext_vector_type(4)));

template <bool NT, class T, int W>
__device__ __forceinline__ Lanes<T, W> load_lanes(const T* p) {
    if constexpr (NT && sizeof(T) * W == 16) {
        const u32x4 r = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
        return __builtin_bit_cast(Lanes<T, W>, r);
    } else {
        return *reinterpret_cast<const Lanes<T, W>*>(p);
    }
}

template <bool NT, class T, int W>
__device__ __forceinline__ void store_lanes(T* p, const Lanes<T, W>& x) {
    if constexpr (NT && sizeof(T) * W == 16) {
        __builtin_nontemporal_store(__builtin_bit_cast(u32x4, x), reinterpret_cast<u32x4*>(p));
    } else {
        *reinterpret_cast<Lanes<T, W>*>(p) = x;
    }
}

// 8-bit lanes, four bytes per 32-bit word: sum by SWAR (the carry out of each byte is dropped, exactly
// the wrap of the per-byte add), prod / max / min on packed 16-bit halves (even bytes and odd bytes; the
// low byte of a 16-bit product is the wrapped byte product, signed or not), one or two instructions per
// 2-4 bytes instead of several per byte.
using u16x2 = unsigned short __attribute__((ext_vector_type(2)));
using i16x2 = short __attribute__((ext_vector_type(2)));

template <class Op, class T>
__device__ __forceinline__ uint32_t combine_bytes(uint32_t a, uint32_t b) {
    if constexpr (std::is_same_v<Op, OpSum>) {
        return ((a & 0x7F7F7F7Fu) + (b & 0x7F7F7F7Fu)) ^ ((a ^ b) & 0x80808080u);
    } else if constexpr (std::is_same_v<Op, OpProd>) {
        const u16x2 ae = __builtin_bit_cast(u16x2, a & 0x00FF00FFu), be = __builtin_bit_cast(u16x2, b & 0x00FF00FFu);
        const u16x2 ao = __builtin_bit_cast(u16x2, (a >> 8) & 0x00FF00FFu), bo = __builtin_bit_cast(u16x2, (b >> 8) & 0x00FF00FFu);
        const uint32_t e = __builtin_bit_cast(uint32_t, static_cast<u16x2>(ae * be)) & 0x00FF00FFu;
        const uint32_t o = __builtin_bit_cast(uint32_t, static_cast<u16x2>(ao * bo)) & 0x00FF00FFu;
        return e | (o << 8);
    } else {
        using V = std::conditional_t<std::is_signed_v<T>, i16x2, u16x2>;
        const V a16 = __builtin_bit_cast(V, a), b16 = __builtin_bit_cast(V, b);
        const V ae = (a16 << 8) >> 8, be = (b16 << 8) >> 8;  // even bytes, widened
        const V ao = a16 >> 8, bo = b16 >> 8;                  // odd bytes, widened
        V e, o;
        if constexpr (std::is_same_v<Op, OpMax>) {
            e = __builtin_elementwise_max(ae, be);
            o = __builtin_elementwise_max(ao, bo);
        } else {
            e = __builtin_elementwise_min(ae, be);
            o = __builtin_elementwise_min(ao, bo);
        }
        return (__builtin_bit_cast(uint32_t, e) & 0x00FF00FFu) | ((__builtin_bit_cast(uint32_t, o) & 0x00FF00FFu) << 8);
    }
}

template <class Op, class T, int W>
__device__ __forceinline__ Lanes<T, W> combine(const Lanes<T, W>& a, const Lanes<T, W>& b) {
    if constexpr (sizeof(T) == 1 && W % 4 == 0) {
        struct Words {
            uint32_t w[W / 4];
        };
        const Words x = __builtin_bit_cast(Words, a), y = __builtin_bit_cast(Words, b);
        Words r;
#pragma unroll
        for (int k = 0; k < W / 4; ++k) r.w[k] = combine_bytes<Op, T>(x.w[k], y.w[k]);
        return __builtin_bit_cast(Lanes<T, W>, r);
    } else {
        Lanes<T, W> r;
#pragma unroll
        for (int k = 0; k < W; ++k) r.v[k] = Op::template apply<T>(a.v[k], b.v[k]);
        return r;
    }
}

// Buffer-op form of the fused kernels' 16-B accesses (pol = 1, FMI_TUNE_FUSED_POLICY): every access of a
// 256-thread tile goes through a descriptor based at the tile's first byte of that bucket (a uniform
// 64-bit address, so any bucket size) with the lane's 32-bit byte offset, and carries an explicit cache
// policy: loads nt; the tree's one output stream sc1 (written lines leave the XCD L2 at once), the scan's
// P output streams nt sc1. tools/microbench_cachepol.hip measured, on the same buffers, tree P = 8 3.3 %
// and scan P = 8 4.6 % faster than global_load / global_store nt (bit-identical results) with few rotating
// sets; with no set re-read from the MALL (tools/ab_fused_policy.py --footprint-gib 6) the scans keep ~2 %,
// trees of 4 peers 2.4 %, trees of 8 / 16 are within 1 % either way. The pairwise kernel keeps global nt
// accesses and stores some of its tiles with sc1 (pair_tile below).
inline constexpr int kAuxNT = 2, kAuxSC1 = 16;
inline constexpr int kTreeStoreAux = kAuxSC1, kScanStoreAux = kAuxNT | kAuxSC1, kFusedLoadAux = kAuxNT;
using b128 = unsigned int __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(const void* tile_base) {
    // raw (stride 0) descriptor, 32-bit data format; num_records covers any tile (<= 64 KiB past its base)
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(tile_base), 0, 1 << 30, 0x00020000);
}
template <int AUX, class T, int W>
__device__ __forceinline__ Lanes<T, W> load_tile(const void* bucket, size_t tile_byte, unsigned lane_byte) {
    static_assert(sizeof(T) * W == 16, "16-B lane groups");
    const b128 r = __builtin_amdgcn_raw_buffer_load_b128(tile_rsrc(static_cast<const char*>(bucket) + tile_byte), lane_byte, 0, AUX);
    return __builtin_bit_cast(Lanes<T, W>, r);
}
template <int AUX, class T, int W>
__device__ __forceinline__ void store_tile(void* bucket, size_t tile_byte, unsigned lane_byte, const Lanes<T, W>& x) {
    static_assert(sizeof(T) * W == 16, "16-B lane groups");
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(b128, x), tile_rsrc(static_cast<char*>(bucket) + tile_byte),
                                           lane_byte, 0, AUX);
}

// Device copy (device_copy in fmi_dev.hip: the reference's P = 1 allreduce and every staging copy of the
// communicator): the pair tile's shape with one stream in and one out — U 16-B vectors per thread (U = 1 in
// the library, profiles/r04_copy_unroll.jsonl), one tile per workgroup. Whole tiles load nontemporal and store with sc1 through a buffer descriptor (the tree kernel's
// policy, above): 4.6 % faster than global nontemporal stores at 256 MiB, 3 % at 64 MiB, with no set
// re-read from the MALL (profiles/archive/r03_copypol.jsonl). The partial last tile
// goes through bounds-checked global accesses; workgroup 0 copies the sub-16-B tail. Algorithmic HBM bytes:
// 2 x bytes. Both pointers 16-B aligned.
template <int U>
__global__ void __launch_bounds__(256) copy_tile(char* out, const char* in, size_t bytes) {
    const size_t nvec = bytes / 16;
    const size_t base = static_cast<size_t>(blockIdx.x) * U * 256 + threadIdx.x;
    if (static_cast<size_t>(blockIdx.x + 1) * U * 256 <= nvec) {
        const size_t tile_byte = static_cast<size_t>(blockIdx.x) * U * 256 * 16;
        Lanes<unsigned, 4> v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            v[u] = load_tile<kAuxNT, unsigned, 4>(in, tile_byte, static_cast<unsigned>((u * 256 + threadIdx.x) * 16));
#pragma unroll
        for (int u = 0; u < U; ++u)
            store_tile<kAuxSC1, unsigned, 4>(out, tile_byte, static_cast<unsigned>((u * 256 + threadIdx.x) * 16), v[u]);
    } else {
        const u32x4* src = reinterpret_cast<const u32x4*>(in);
        u32x4* dst = reinterpret_cast<u32x4*>(out);
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (base + u * 256 < nvec) v[u] = __builtin_nontemporal_load(src + base + u * 256);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (base + u * 256 < nvec) __builtin_nontemporal_store(v[u], dst + base + u * 256);
    }
    if (blockIdx.x == 0 && nvec * 16 + threadIdx.x < bytes) out[nvec * 16 + threadIdx.x] = in[nvec * 16 + threadIdx.x];
}

// ---------------------------------------------------------------------------------------------------
// Pairwise combine. A "tile" is U vectors per thread: thread t of block b owns vectors
// b*U*B + u*B + t (u < U), so each of the U wave-instructions is one contiguous 1-KiB access and each
// thread keeps 2U independent 16-B loads in flight before its first add.
// ---------------------------------------------------------------------------------------------------
// NT: cache policy bitmask — bit 0 nontemporal loads, bit 1 nontemporal stores. `sc1` (uniform per tile):
// store this tile with sc1 instead (pair_tile's sc1 tiles, FMI_TUNE_PAIR_SC1_OF_8).
template <class Op, class T, int U, int NT>
__device__ __forceinline__ void pair_tile_body(T* out, const T* a, const T* b, size_t nvec, size_t tile, bool sc1 = false) {
    constexpr int W = kVecLanes<T>;
    constexpr bool NTL = (NT & 1) != 0;
    constexpr bool NTS = (NT & 2) != 0;
    using L = Lanes<T, W>;
    const size_t B = blockDim.x;
    const size_t base = tile * U * B + threadIdx.x;
    L va[U], vb[U];
    if (tile * U * B + U * B <= nvec) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            va[u] = load_lanes<NTL, T, W>(a + (base + u * B) * W);
            vb[u] = load_lanes<NTL, T, W>(b + (base + u * B) * W);
        }
        // one descriptor at the tile's first output byte, lane offsets < U * B * 16 (U = 8: not taken; the
        // second store path spills the 8-bit max / min forms to scratch under the 1024-thread bound)
        if (U <= 4 && sc1) {
            const size_t tile_byte = tile * U * B * 16;
#pragma unroll
            for (int u = 0; u < U; ++u)
                store_tile<kAuxSC1, T, W>(out, tile_byte, static_cast<unsigned>((u * B + threadIdx.x) * 16),
                                          combine<Op, T, W>(va[u], vb[u]));
        } else {
#pragma unroll
            for (int u = 0; u < U; ++u) store_lanes<NTS, T, W>(out + (base + u * B) * W, combine<Op, T, W>(va[u], vb[u]));
        }
    } else {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + u * B;
            if (i < nvec) {
                va[u] = load_lanes<NTL, T, W>(a + i * W);
                vb[u] = load_lanes<NTL, T, W>(b + i * W);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = base + u * B;
            if (i < nvec) store_lanes<NTS, T, W>(out + i * W, combine<Op, T, W>(va[u], vb[u]));
        }
    }
}

template <class Op, class T>
__device__ __forceinline__ void pair_tail(T* out, const T* a, const T* b, size_t n) {
    constexpr int W = kVecLanes<T>;
    const size_t first = (n / W) * W;
    if (blockIdx.x == 0 && first + threadIdx.x < n) {
        const size_t i = first + threadIdx.x;
        out[i] = Op::template apply<T>(a[i], b[i]);
    }
}

// One-shot grid: one tile per workgroup. Pointers must be 16-B aligned. Whole tiles t with t % 8 < sc1_k
// store with sc1, the rest nontemporal (default 0: none, the round-1 kernel the exploration tools compare
// against). Consecutive workgroups are dispatched to different XCDs, so sc1_k of the 8 XCDs store sc1
// (FMI_TUNE_PAIR_SC1_OF_8; tools/ab_pair_sc1.py).
template <class Op, class T, int U, int NT>
__global__ void __launch_bounds__(1024) pair_tile(T* out, const T* a, const T* b, size_t n, unsigned sc1_k = 0) {
    const size_t nvec = n / kVecLanes<T>;
    pair_tile_body<Op, T, U, NT>(out, a, b, nvec, blockIdx.x, (blockIdx.x & 7u) < sc1_k);
    pair_tail<Op, T>(out, a, b, n);
}

// Grid-stride: a fixed grid (k workgroups per CU) walks the tiles. Pointers must be 16-B aligned. Every
// tile stores nontemporal (a second store path inside the loop spills the U = 8 forms to scratch).
template <class Op, class T, int U, int NT>
__global__ void __launch_bounds__(1024) pair_stride(T* out, const T* a, const T* b, size_t n) {
    const size_t nvec = n / kVecLanes<T>;
    const size_t ntiles = (nvec + static_cast<size_t>(U) * blockDim.x - 1) / (static_cast<size_t>(U) * blockDim.x);
    for (size_t t = blockIdx.x; t < ntiles; t += gridDim.x) pair_tile_body<Op, T, U, NT>(out, a, b, nvec, t);
    pair_tail<Op, T>(out, a, b, n);
}

// Any alignment: scalar grid-stride loop.
template <class Op, class T>
__global__ void __launch_bounds__(256) pair_scalar(T* out, const T* a, const T* b, size_t n) {
    for (size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
         i += static_cast<size_t>(gridDim.x) * blockDim.x)
        out[i] = Op::template apply<T>(a[i], b[i]);
}

// ---------------------------------------------------------------------------------------------------
// Fused P-way kernels: evaluate a sched::Fused<ALG,P> program per 16-B lane group, every value in
// registers. Indices into the value array are template constants (fold over index_sequence), so the
// array is promoted to VGPRs — no scratch.
// ---------------------------------------------------------------------------------------------------
// Peer buckets are streamed exactly once per launch: nontemporal loads/stores (global_* nt) keep them
// from displacing other data in L2/MALL, as for the pairwise kernel (tools/tune_pair.py: +13%).
inline constexpr bool kFusedNT = true;

struct PeerPtrs {
    const void* in[sched::kFusedInputCap];
    void* out[sched::kFusedInputCap];
};

// Program fields as integral constants: reading them through these variable templates guarantees the
// value-array indices are folded in the front end, so SROA keeps every value in VGPRs (no scratch).
template <int ALG, int P, size_t S>
inline constexpr int kStepA = sched::Fused<ALG, P>::prog.step[S].a;
template <int ALG, int P, size_t S>
inline constexpr int kStepB = sched::Fused<ALG, P>::prog.step[S].b;
template <int ALG, int P, size_t R>
inline constexpr int kOut = sched::Fused<ALG, P>::prog.out[R];
template <int ALG, int P>
inline constexpr int kNumSteps = sched::Fused<ALG, P>::prog.nsteps;

template <class Op, class T, int W, int ALG, int P, size_t... S>
__device__ __forceinline__ void run_steps(Lanes<T, W>* v, std::index_sequence<S...>) {
    ((v[P + S] = combine<Op, T, W>(v[kStepA<ALG, P, S>], v[kStepB<ALG, P, S>])), ...);
}

template <class T, int W, int P, size_t... I>
__device__ __forceinline__ void load_peers(Lanes<T, W>* v, const PeerPtrs& ptrs, size_t elem,
                                           std::index_sequence<I...>) {
    ((v[I] = load_lanes<kFusedNT, T, W>(static_cast<const T*>(ptrs.in[I]) + elem)), ...);
}

// The value as an opaque register operand. A select chain over loads from one array (pick_rank below) is
// otherwise folded by LLVM into a single load at a rank-dependent index, which pins the whole value array
// in scratch memory (it did, for every rank-aware instantiation, up to 1.3 KiB per thread at P = 16).
template <class T, int W>
__device__ __forceinline__ Lanes<T, W> opaque(Lanes<T, W> x) {
    if constexpr (sizeof(x) == 16) {
        u32x4 b = __builtin_bit_cast(u32x4, x);
        asm("" : "+v"(b));
        return __builtin_bit_cast(Lanes<T, W>, b);
    } else if constexpr (sizeof(x) == 8) {
        uint64_t b = __builtin_bit_cast(uint64_t, x);
        asm("" : "+v"(b));
        return __builtin_bit_cast(Lanes<T, W>, b);
    } else {
        static_assert(sizeof(x) == 4, "lane group of 4, 8 or 16 bytes");
        uint32_t b = __builtin_bit_cast(uint32_t, x);
        asm("" : "+v"(b));
        return __builtin_bit_cast(Lanes<T, W>, b);
    }
}

template <class T, int W, int ALG, int P, size_t... R>
__device__ __forceinline__ Lanes<T, W> pick_rank(const Lanes<T, W>* v, int rank, std::index_sequence<R...>) {
    Lanes<T, W> r = v[kOut<ALG, P, 0>];
    ((r = (rank == static_cast<int>(R)) ? opaque(v[kOut<ALG, P, R>]) : r), ...);
    return r;
}

template <class T, int W, int ALG, int P, size_t... R>
__device__ __forceinline__ void store_all(const Lanes<T, W>* v, const PeerPtrs& ptrs, size_t elem,
                                          std::index_sequence<R...>) {
    ((store_lanes<kFusedNT, T, W>(static_cast<T*>(ptrs.out[R]) + elem, v[kOut<ALG, P, R>])), ...);
}

template <class T, int W, int P, size_t... I>
__device__ __forceinline__ void load_peers_tile(Lanes<T, W>* v, const PeerPtrs& ptrs, size_t tile_byte, unsigned lane_byte,
                                                std::index_sequence<I...>) {
    ((v[I] = load_tile<kFusedLoadAux, T, W>(ptrs.in[I], tile_byte, lane_byte)), ...);
}

// ALL_RANKS: honour `rank` (output = the value peer `rank` holds). Needed only where operand order can
// change bits (float max/min on ±0); otherwise rank 0's expression is bit-identical for every peer.
template <class Op, class T, int ALG, int P, bool ALL_RANKS, int W>
__device__ __forceinline__ void tree_group(const PeerPtrs& ptrs, int rank, size_t elem) {
    Lanes<T, W> v[P + kNumSteps<ALG, P>];
    load_peers<T, W, P>(v, ptrs, elem, std::make_index_sequence<P>{});
    run_steps<Op, T, W, ALG, P>(v, std::make_index_sequence<kNumSteps<ALG, P>>{});
    Lanes<T, W> r;
    if constexpr (ALL_RANKS)
        r = pick_rank<T, W, ALG, P>(v, rank, std::make_index_sequence<P>{});
    else
        r = v[kOut<ALG, P, 0>];
    store_lanes<kFusedNT, T, W>(static_cast<T*>(ptrs.out[0]) + elem, r);
}

template <class Op, class T, int ALG, int P, bool ALL_RANKS, int W>
__device__ __forceinline__ void tree_group_tile(const PeerPtrs& ptrs, int rank, size_t tile_byte, unsigned lane_byte) {
    Lanes<T, W> v[P + kNumSteps<ALG, P>];
    load_peers_tile<T, W, P>(v, ptrs, tile_byte, lane_byte, std::make_index_sequence<P>{});
    run_steps<Op, T, W, ALG, P>(v, std::make_index_sequence<kNumSteps<ALG, P>>{});
    Lanes<T, W> r;
    if constexpr (ALL_RANKS)
        r = pick_rank<T, W, ALG, P>(v, rank, std::make_index_sequence<P>{});
    else
        r = v[kOut<ALG, P, 0>];
    store_tile<kTreeStoreAux, T, W>(ptrs.out[0], tile_byte, lane_byte, r);
}

// Launched with one thread per 16-B lane group up to kFusedGridCap workgroups; beyond that (buckets of
// > 2^30 lane groups) each thread strides over the rest, so the grid never exceeds HIP's 2^32-thread limit.
inline constexpr size_t kFusedGridCap = size_t(1) << 22;

// pol = 1: buffer accesses tile by tile (the tile index is uniform, so each tile's descriptors are scalar);
// pol = 0: global accesses.
template <class Op, class T, int ALG, int P, bool ALL_RANKS>
__global__ void __launch_bounds__(256) tree_kernel(PeerPtrs ptrs, size_t n, int rank, int pol) {
    constexpr int W = kVecLanes<T>;
    const size_t nvec = n / W;
    if (pol == 1) {
        const size_t B = blockDim.x;
        for (size_t tile = blockIdx.x; tile * B < nvec; tile += gridDim.x)
            if (tile * B + threadIdx.x < nvec)
                tree_group_tile<Op, T, ALG, P, ALL_RANKS, W>(ptrs, rank, tile * B * 16, threadIdx.x * 16u);
    } else {
        const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
        for (size_t g = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; g < nvec; g += stride)
            tree_group<Op, T, ALG, P, ALL_RANKS, W>(ptrs, rank, g * W);
    }
    const size_t first = nvec * W;
    if (blockIdx.x == 0 && first + threadIdx.x < n) tree_group<Op, T, ALG, P, ALL_RANKS, 1>(ptrs, rank, first + threadIdx.x);
}

// Carry programs (sched::is_carry_alg) leave output 0 alone: value 0 is the carry itself.
template <class T, int W, int ALG, int P, size_t... R>
__device__ __forceinline__ void store_after_carry(const Lanes<T, W>* v, const PeerPtrs& ptrs, size_t elem,
                                                  std::index_sequence<R...>) {
    ((store_lanes<kFusedNT, T, W>(static_cast<T*>(ptrs.out[R + 1]) + elem, v[kOut<ALG, P, R + 1>])), ...);
}

template <class Op, class T, int ALG, int P, int W>
__device__ __forceinline__ void scan_group(const PeerPtrs& ptrs, size_t elem) {
    Lanes<T, W> v[P + kNumSteps<ALG, P>];
    load_peers<T, W, P>(v, ptrs, elem, std::make_index_sequence<P>{});
    run_steps<Op, T, W, ALG, P>(v, std::make_index_sequence<kNumSteps<ALG, P>>{});
    if constexpr (sched::is_carry_alg(ALG))
        store_after_carry<T, W, ALG, P>(v, ptrs, elem, std::make_index_sequence<P - 1>{});
    else
        store_all<T, W, ALG, P>(v, ptrs, elem, std::make_index_sequence<P>{});
}

template <class Op, class T, int ALG, int P, int W>
__device__ __forceinline__ void scan_group_tile(const PeerPtrs& ptrs, size_t tile_byte, unsigned lane_byte) {
    Lanes<T, W> v[P + kNumSteps<ALG, P>];
    load_peers_tile<T, W, P>(v, ptrs, tile_byte, lane_byte, std::make_index_sequence<P>{});
    run_steps<Op, T, W, ALG, P>(v, std::make_index_sequence<kNumSteps<ALG, P>>{});
    constexpr int first_out = sched::is_carry_alg(ALG) ? 1 : 0;  // carry programs leave output 0 alone
    [&]<size_t... R>(std::index_sequence<R...>) {
        ((store_tile<kScanStoreAux, T, W>(ptrs.out[R + first_out], tile_byte, lane_byte, v[kOut<ALG, P, R + first_out>])), ...);
    }(std::make_index_sequence<P - first_out>{});
}

template <class Op, class T, int ALG, int P>
__global__ void __launch_bounds__(256) scan_kernel(PeerPtrs ptrs, size_t n, int pol) {
    constexpr int W = kVecLanes<T>;
    const size_t nvec = n / W;
    if (pol == 1) {
        const size_t B = blockDim.x;
        for (size_t tile = blockIdx.x; tile * B < nvec; tile += gridDim.x)
            if (tile * B + threadIdx.x < nvec) scan_group_tile<Op, T, ALG, P, W>(ptrs, tile * B * 16, threadIdx.x * 16u);
    } else {
        const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
        for (size_t g = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; g < nvec; g += stride)
            scan_group<Op, T, ALG, P, W>(ptrs, g * W);
    }
    const size_t first = nvec * W;
    if (blockIdx.x == 0 && first + threadIdx.x < n) scan_group<Op, T, ALG, P, 1>(ptrs, first + threadIdx.x);
}

// ---------------------------------------------------------------------------------------------------
// Synthetic buckets: h = splitmix64(seed ^ (peer << 40) ^ i).
// ---------------------------------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

template <class T>
__host__ __device__ __forceinline__ T synth_value(uint64_t h) {
    if constexpr (std::is_same_v<T, float>) {
        return static_cast<float>(h >> 40) * 0x1p-24f * 2.0f - 1.0f;
    } else if constexpr (std::is_same_v<T, double>) {
        return static_cast<double>(h >> 11) * 0x1p-53 * 2.0 - 1.0;
    } else {
        // integers: the top 8·sizeof(T) bits of h (i32 = h >> 32, i64 = h, as before)
        using U = std::make_unsigned_t<T>;
        return static_cast<T>(static_cast<U>(h >> (64 - 8 * sizeof(T))));
    }
}

template <class T>
__global__ void __launch_bounds__(256) synth_kernel(T* buf, size_t n, uint64_t seed, uint32_t peer, uint64_t first) {
    const uint64_t key = seed ^ (static_cast<uint64_t>(peer) << 40);
    for (size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
         i += static_cast<size_t>(gridDim.x) * blockDim.x)
        buf[i] = synth_value<T>(splitmix64(key ^ (first + i)));
}

}  // namespace fmi::dev
