// microbench_cachepol.hip — exploration harness (not part of the library): do gfx950's other vector
// cache policies beat the production nontemporal loads / stores on the streaming kernels?
//
// MI355X_MICROARCH.md: plain / sc0 / nt stores keep the written line in the XCD's L2, sc1 / sc0 sc1 drop it;
// sc1 / sc0 sc1 / nt loads bypass L1. The production kernels use __builtin_nontemporal_load / _store (nt
// both sides). Here the same tiles are issued as raw buffer loads / stores with an explicit aux policy
// (bit 0 sc0, bit 1 nt, bit 4 sc1) on the three production shapes:
//   pair   f32 sum, 256 MiB buckets (C2): 2 reads + 1 write, 256 threads, 4 lane groups per thread
//   scan8  f32 peer scan P = 8 x 64 MiB (C3): 8 reads + 8 writes, 256 threads, 2 workgroups per CU
//   tree8  f32 allreduce P = 8 x 64 MiB: 8 reads + 1 write, 256 threads, 2 workgroups per CU
// Every variant's output is compared with the production policy's (bit-exact, same arithmetic).
// Timing: K back-to-back launches over rotating buffer sets between two events, per variant, variants
// interleaved over R rounds; median over rounds.
//
// Build: hipcc -std=c++20 -O3 --offload-arch=gfx950 -ffp-contract=off tools/microbench_cachepol.hip -o build/mbc
// Run:   build/mbc [rounds, default 5] [name filter]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "../fmi_amd/csrc/fmi_internal.h"

using namespace fmi::dev;

#define CHECK(x)                                                                                   \
    do {                                                                                           \
        hipError_t e = (x);                                                                        \
        if (e != hipSuccess) {                                                                     \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            std::exit(1);                                                                          \
        }                                                                                          \
    } while (0)

using u32x4v = __attribute__((__vector_size__(4 * sizeof(unsigned)))) unsigned;
constexpr int kRsrcWord3 = 0x00020000;  // raw 32-bit buffer, gfx9 family
constexpr int PROD = -1;                // the production builtin (nontemporal)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, bytes, kRsrcWord3);
}

template <int LA>
__device__ __forceinline__ u32x4v ld(const void* base, __amdgpu_buffer_rsrc_t r, unsigned off) {
    if constexpr (LA == PROD)
        return __builtin_nontemporal_load(reinterpret_cast<const u32x4v*>(static_cast<const char*>(base) + off));
    else
        return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, LA);
}
template <int SA>
__device__ __forceinline__ void st(void* base, __amdgpu_buffer_rsrc_t r, unsigned off, u32x4v v) {
    if constexpr (SA == PROD)
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4v*>(static_cast<char*>(base) + off));
    else
        __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, SA);
}
__device__ __forceinline__ u32x4v addf(u32x4v a, u32x4v b) {
    u32x4v o;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = __float_as_uint(__uint_as_float(a[i]) + __uint_as_float(b[i]));
    return o;
}

// pair: out = a + b, U = 4 groups of 16 B per thread, stride 256 threads
template <int LA, int SA>
__global__ void __launch_bounds__(256) pair_k(float* out, const float* a, const float* b, unsigned bytes) {
    const auto ra = rsrc(a, bytes), rb = rsrc(b, bytes), ro = rsrc(out, bytes);
    const unsigned base = (blockIdx.x * 4u * 256u + threadIdx.x) * 16u;
    u32x4v x[4], y[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        x[u] = ld<LA>(a, ra, base + u * 4096u);
        y[u] = ld<LA>(b, rb, base + u * 4096u);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) st<SA>(out, ro, base + u * 4096u, addf(x[u], y[u]));
}

// Production candidate: the tile's base as a uniform (scalar) pointer, each lane a 32-bit byte offset from
// it (global_load saddr form: no per-lane 64-bit address arithmetic), compile-time block size, the same
// uniform full-tile / ragged-tile split and tail as pair_tile.
template <class Op, class T, int U, int B>
__global__ void __launch_bounds__(B) pair_saddr(T* out, const T* a, const T* b, size_t n) {
    constexpr int W = kVecLanes<T>;
    using L = Lanes<T, W>;
    const size_t nvec = n / W;
    const size_t tile0 = static_cast<size_t>(blockIdx.x) * U * B;  // first lane group of this tile
    const T* ta = a + tile0 * W;
    const T* tb = b + tile0 * W;
    T* to = out + tile0 * W;
    const unsigned t = threadIdx.x;
    L va[U], vb[U];
    if (tile0 + U * B <= nvec) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            va[u] = load_lanes<true, T, W>(ta + (u * B + t) * W);
            vb[u] = load_lanes<true, T, W>(tb + (u * B + t) * W);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) store_lanes<true, T, W>(to + (u * B + t) * W, combine<Op, T, W>(va[u], vb[u]));
    } else {
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (tile0 + u * B + t < nvec) {
                va[u] = load_lanes<true, T, W>(ta + (u * B + t) * W);
                vb[u] = load_lanes<true, T, W>(tb + (u * B + t) * W);
            }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (tile0 + u * B + t < nvec) store_lanes<true, T, W>(to + (u * B + t) * W, combine<Op, T, W>(va[u], vb[u]));
    }
    pair_tail<Op, T>(out, a, b, n);
}

// saddr form done right: uniform tile base pointers, each access a 32-bit unsigned byte offset from them
// (global_load v, v_off, s[base] — no per-lane 64-bit address arithmetic); same full / ragged split and tail.
template <class Op, class T, int U, unsigned B>
__global__ void __launch_bounds__(B) pair_saddr2(T* out, const T* a, const T* b, size_t n) {
    constexpr int W = kVecLanes<T>;
    using L = Lanes<T, W>;
    const size_t nvec = n / W;
    const size_t tile0 = static_cast<size_t>(blockIdx.x) * U * B;  // first lane group of the tile
    const char* ta = reinterpret_cast<const char*>(a + tile0 * W);
    const char* tb = reinterpret_cast<const char*>(b + tile0 * W);
    char* to = reinterpret_cast<char*>(out + tile0 * W);
    const unsigned lane = threadIdx.x * 16u;
    L va[U], vb[U];
    if (tile0 + U * B <= nvec) {
        // each group's 32-bit offset as an opaque register, so every access is (tile base SGPRs) + offset
        unsigned off[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            off[u] = lane + u * B * 16u;
            asm("" : "+v"(off[u]));
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            va[u] = load_lanes<true, T, W>(reinterpret_cast<const T*>(ta + off[u]));
            vb[u] = load_lanes<true, T, W>(reinterpret_cast<const T*>(tb + off[u]));
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            store_lanes<true, T, W>(reinterpret_cast<T*>(to + off[u]), combine<Op, T, W>(va[u], vb[u]));
    } else {
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (tile0 + u * B + threadIdx.x < nvec) {
                const unsigned off = lane + u * B * 16u;
                va[u] = load_lanes<true, T, W>(reinterpret_cast<const T*>(ta + off));
                vb[u] = load_lanes<true, T, W>(reinterpret_cast<const T*>(tb + off));
            }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (tile0 + u * B + threadIdx.x < nvec)
                store_lanes<true, T, W>(reinterpret_cast<T*>(to + lane + u * B * 16u), combine<Op, T, W>(va[u], vb[u]));
    }
    pair_tail<Op, T>(out, a, b, n);
}

// the production pair_tile with __launch_bounds__(256) instead of 1024 (same body and tail)
template <class Op, class T, int U, int NT>
__global__ void __launch_bounds__(256) pair_tile_lb256(T* out, const T* a, const T* b, size_t n) {
    const size_t nvec = n / kVecLanes<T>;
    pair_tile_body<Op, T, U, NT>(out, a, b, nvec, blockIdx.x);
    pair_tail<Op, T>(out, a, b, n);
}

// global nt loads, buffer store with policy SA through a per-tile descriptor
template <int SA>
__global__ void __launch_bounds__(256) pair_mix_k(float* out, const float* a, const float* b) {
    const size_t tile = static_cast<size_t>(blockIdx.x) * 4 * 256 * 16;  // bytes
    const unsigned lane = threadIdx.x * 16u;
    const char* ta = reinterpret_cast<const char*>(a) + tile;
    const char* tb = reinterpret_cast<const char*>(b) + tile;
    u32x4v x[4], y[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        x[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4v*>(ta + lane + u * 4096u));
        y[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4v*>(tb + lane + u * 4096u));
    }
    const auto ro = rsrc(reinterpret_cast<char*>(out) + tile, 1 << 30);
#pragma unroll
    for (int u = 0; u < 4; ++u) __builtin_amdgcn_raw_buffer_store_b128(addf(x[u], y[u]), ro, lane + u * 4096u, 0, SA);
}

struct P8 {
    const float* in[8];
    float* out[8];
};

// scan8: out[k] = in[0] + ... + in[k] (left fold; the arithmetic order is the same in every variant)
template <int LA, int SA, bool SCAN>
__global__ void __launch_bounds__(256) p8_k(P8 p, unsigned bytes) {
    extern __shared__ char lds_cap[];  // residency cap: the launch reserves LDS for 2 workgroups per CU
    if (bytes == 0) lds_cap[threadIdx.x] = 0;
    const unsigned off = (blockIdx.x * 256u + threadIdx.x) * 16u;
    u32x4v v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = ld<LA>(p.in[k], rsrc(p.in[k], bytes), off);
    u32x4v acc = v[0];
    if constexpr (SCAN) st<SA>(p.out[0], rsrc(p.out[0], bytes), off, acc);
#pragma unroll
    for (int k = 1; k < 8; ++k) {
        acc = addf(acc, v[k]);
        if constexpr (SCAN) st<SA>(p.out[k], rsrc(p.out[k], bytes), off, acc);
    }
    if constexpr (!SCAN) st<SA>(p.out[0], rsrc(p.out[0], bytes), off, acc);
}

// The production fused programs (reference bracketing, fmi_schedule.h) with buffer loads / stores: one
// descriptor per bucket (buckets < 4 GiB), 32-bit byte offsets, explicit aux policy.
template <int LA, int SA, class T, int W, int P, size_t... I>
__device__ __forceinline__ void load_peers_buf(Lanes<T, W>* v, const PeerPtrs& ptrs, unsigned off, unsigned bytes,
                                               std::index_sequence<I...>) {
    ((v[I] = __builtin_bit_cast(Lanes<T, W>, __builtin_amdgcn_raw_buffer_load_b128(rsrc(ptrs.in[I], bytes), off, 0, LA))), ...);
}
template <int SA, class T, int W, int ALG, int P, size_t... R>
__device__ __forceinline__ void store_all_buf(const Lanes<T, W>* v, const PeerPtrs& ptrs, unsigned off, unsigned bytes,
                                              std::index_sequence<R...>) {
    ((__builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, v[kOut<ALG, P, R>]), rsrc(ptrs.out[R], bytes), off, 0, SA)),
     ...);
}
template <class Op, class T, int ALG, int P, int LA, int SA, bool ALL_OUT>
__global__ void __launch_bounds__(256) fused_buf_kernel(PeerPtrs ptrs, size_t n) {
    constexpr int W = kVecLanes<T>;
    const size_t nvec = n / W;
    const unsigned bytes = static_cast<unsigned>(n * sizeof(T));
    const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
    for (size_t g = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; g < nvec; g += stride) {
        const unsigned off = static_cast<unsigned>(g * 16);
        Lanes<T, W> v[P + kNumSteps<ALG, P>];
        load_peers_buf<LA, SA, T, W, P>(v, ptrs, off, bytes, std::make_index_sequence<P>{});
        run_steps<Op, T, W, ALG, P>(v, std::make_index_sequence<kNumSteps<ALG, P>>{});
        if constexpr (ALL_OUT)
            store_all_buf<SA, T, W, ALG, P>(v, ptrs, off, bytes, std::make_index_sequence<P>{});
        else
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, v[kOut<ALG, P, 0>]), rsrc(ptrs.out[0], bytes), off, 0, SA);
    }
}

void* dalloc(size_t bytes) {
    void* p = nullptr;
    CHECK(hipMalloc(&p, bytes));
    CHECK(hipMemset(p, 0, bytes));
    return p;
}

__global__ void fill_k(float* p, size_t n, unsigned seed) {
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
        p[i] = float((i * 2654435761u + seed) % 1000003u) * 0.001f;
}

struct Variant {
    std::string name;
    std::function<void(int)> launch;
    double bytes;
    std::vector<double> us;
};

// the library's residency cap (fused_lds_bytes, 64 KiB budget of peer loads per CU, >= 2 workgroups)
size_t fused_lds(int P) {
    const size_t per_wg = size_t(P) * 4096, budget = 64 << 10;
    const size_t cap = std::max<size_t>(2, (budget + per_wg - 1) / per_wg);
    return cap >= 32 ? 0 : ((160 << 10) / cap) & ~size_t(255);
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 5;
    constexpr int K = 20;
    const size_t pair_bytes = size_t(256) << 20, p8_bytes = size_t(64) << 20;
    constexpr int PSETS = 2, SSETS = 2;
    float *pa[PSETS], *pb[PSETS], *po[PSETS];
    for (int s = 0; s < PSETS; ++s) {
        pa[s] = static_cast<float*>(dalloc(pair_bytes));
        pb[s] = static_cast<float*>(dalloc(pair_bytes));
        po[s] = static_cast<float*>(dalloc(pair_bytes));
        fill_k<<<4096, 256>>>(pa[s], pair_bytes / 4, 11 + s);
        fill_k<<<4096, 256>>>(pb[s], pair_bytes / 4, 17 + s);
    }
    P8 sp[SSETS], tp[SSETS];
    for (int s = 0; s < SSETS; ++s)
        for (int k = 0; k < 8; ++k) {
            float* in = static_cast<float*>(dalloc(p8_bytes));
            fill_k<<<4096, 256>>>(in, p8_bytes / 4, 100 * s + k);
            sp[s].in[k] = tp[s].in[k] = in;
            sp[s].out[k] = static_cast<float*>(dalloc(p8_bytes));
            tp[s].out[k] = k == 0 ? static_cast<float*>(dalloc(p8_bytes)) : nullptr;
        }
    CHECK(hipDeviceSynchronize());
    const unsigned pgrid = unsigned(pair_bytes / (16 * 4 * 256)), sgrid = unsigned(p8_bytes / (16 * 256));
    const size_t lds = 80 << 10;  // 160 KiB per CU / 2
    std::vector<Variant> vs;
#define PAIR(LA, SA)                                                                                         \
    vs.push_back({"pair ld" #LA " st" #SA, [&](int k) {                                                      \
                      pair_k<LA, SA><<<pgrid, 256>>>(po[k % PSETS], pa[k % PSETS], pb[k % PSETS], unsigned(pair_bytes)); \
                  }, 3.0 * pair_bytes, {}});
#define P8V(LA, SA, SCAN, NAME, BYTES)                                                                        \
    vs.push_back({std::string(NAME) + " ld" #LA " st" #SA, [&](int k) {                                      \
                      p8_k<LA, SA, SCAN><<<sgrid, 256, lds>>>((SCAN ? sp : tp)[k % SSETS], unsigned(p8_bytes)); \
                  }, BYTES, {}});
    const size_t pn = pair_bytes / 4;
    vs.push_back({"pair production pair_tile<OpSum,float,4,3>", [&](int k) {
                      pair_tile<OpSum, float, 4, 3><<<pgrid, 256>>>(po[k % PSETS], pa[k % PSETS], pb[k % PSETS], pn);
                  }, 3.0 * pair_bytes, {}});
    vs.push_back({"pair saddr candidate U4 B256", [&](int k) {
                      pair_saddr<OpSum, float, 4, 256><<<pgrid, 256>>>(po[k % PSETS], pa[k % PSETS], pb[k % PSETS], pn);
                  }, 3.0 * pair_bytes, {}});
    vs.push_back({"pair saddr candidate U2 B512", [&](int k) {
                      pair_saddr<OpSum, float, 2, 512><<<pgrid, 512>>>(po[k % PSETS], pa[k % PSETS], pb[k % PSETS], pn);
                  }, 3.0 * pair_bytes, {}});
    // the production P = 8 kernels against buffer-op versions of the same programs
    PeerPtrs psp[SSETS], ptp[SSETS];
    for (int s = 0; s < SSETS; ++s) {
        std::memset(&psp[s], 0, sizeof(PeerPtrs));
        std::memset(&ptp[s], 0, sizeof(PeerPtrs));
        for (int k = 0; k < 8; ++k) {
            psp[s].in[k] = ptp[s].in[k] = sp[s].in[k];
            psp[s].out[k] = sp[s].out[k];
        }
        ptp[s].out[0] = tp[s].out[0];
    }
    const size_t pn8 = p8_bytes / 4;
    constexpr int SC = fmi::sched::kScan, AR = fmi::sched::kAllreduce;
    vs.push_back({"pscan8 production scan_kernel", [&](int k) {
                      scan_kernel<OpSum, float, SC, 8><<<sgrid, 256, lds>>>(psp[k % SSETS], pn8, 0);
                  }, 16.0 * p8_bytes, {}});
#define PSCAN(LA, SA)                                                                                        \
    vs.push_back({"pscan8 buffer ld" #LA " st" #SA, [&](int k) {                                             \
                      fused_buf_kernel<OpSum, float, SC, 8, LA, SA, true><<<sgrid, 256, lds>>>(psp[k % SSETS], pn8); \
                  }, 16.0 * p8_bytes, {}});
    PSCAN(2, 2) PSCAN(2, 18) PSCAN(18, 18)
    vs.push_back({"pscan8 production scan_kernel pol1", [&](int k) {
                      scan_kernel<OpSum, float, SC, 8><<<sgrid, 256, lds>>>(psp[k % SSETS], pn8, 1);
                  }, 16.0 * p8_bytes, {}});
    vs.push_back({"ptree8 production tree_kernel", [&](int k) {
                      tree_kernel<OpSum, float, AR, 8, false><<<sgrid, 256, lds>>>(ptp[k % SSETS], pn8, 0, 0);
                  }, 9.0 * p8_bytes, {}});
#define PTREE(LA, SA)                                                                                        \
    vs.push_back({"ptree8 buffer ld" #LA " st" #SA, [&](int k) {                                             \
                      fused_buf_kernel<OpSum, float, AR, 8, LA, SA, false><<<sgrid, 256, lds>>>(ptp[k % SSETS], pn8); \
                  }, 9.0 * p8_bytes, {}});
    PTREE(2, 2) PTREE(2, 16)
    vs.push_back({"ptree8 production tree_kernel pol1", [&](int k) {
                      tree_kernel<OpSum, float, AR, 8, false><<<sgrid, 256, lds>>>(ptp[k % SSETS], pn8, 0, 1);
                  }, 9.0 * p8_bytes, {}});
    // store policies of the production programs at P = 2 and 4 (scan and tree)
#define PVAR(TAG, ALG, P_, ALLOUT, SA, BYTES)                                                                \
    vs.push_back({std::string(TAG) + " buffer ld2 st" #SA, [&](int k) {                                      \
                      fused_buf_kernel<OpSum, float, ALG, P_, 2, SA, ALLOUT><<<sgrid, 256, fused_lds(P_)>>>((ALLOUT ? psp : ptp)[k % SSETS], pn8); \
                  }, BYTES, {}});
#define PPROD(TAG, ALG, P_, ALLOUT, POL, BYTES)                                                              \
    vs.push_back({std::string(TAG) + " production pol" #POL, [&](int k) {                                    \
                      if constexpr (ALLOUT)                                                                  \
                          scan_kernel<OpSum, float, ALG, P_><<<sgrid, 256, fused_lds(P_)>>>(psp[k % SSETS], pn8, POL); \
                      else                                                                                   \
                          tree_kernel<OpSum, float, ALG, P_, false><<<sgrid, 256, fused_lds(P_)>>>(ptp[k % SSETS], pn8, 0, POL); \
                  }, BYTES, {}});
    PPROD("s2", SC, 2, true, 0, 4.0 * p8_bytes) PPROD("s2", SC, 2, true, 1, 4.0 * p8_bytes)
    PVAR("s2", SC, 2, true, 2, 4.0 * p8_bytes) PVAR("s2", SC, 2, true, 16, 4.0 * p8_bytes) PVAR("s2", SC, 2, true, 18, 4.0 * p8_bytes)
    PPROD("s4", SC, 4, true, 0, 8.0 * p8_bytes) PPROD("s4", SC, 4, true, 1, 8.0 * p8_bytes)
    PVAR("s4", SC, 4, true, 2, 8.0 * p8_bytes) PVAR("s4", SC, 4, true, 16, 8.0 * p8_bytes) PVAR("s4", SC, 4, true, 18, 8.0 * p8_bytes)
    PPROD("s8", SC, 8, true, 0, 16.0 * p8_bytes) PPROD("s8", SC, 8, true, 1, 16.0 * p8_bytes)
    PVAR("s8", SC, 8, true, 2, 16.0 * p8_bytes) PVAR("s8", SC, 8, true, 16, 16.0 * p8_bytes) PVAR("s8", SC, 8, true, 18, 16.0 * p8_bytes)
    PPROD("t2", AR, 2, false, 0, 3.0 * p8_bytes) PPROD("t2", AR, 2, false, 1, 3.0 * p8_bytes)
    PVAR("t2", AR, 2, false, 2, 3.0 * p8_bytes) PVAR("t2", AR, 2, false, 18, 3.0 * p8_bytes)
    PPROD("t4", AR, 4, false, 0, 5.0 * p8_bytes) PPROD("t4", AR, 4, false, 1, 5.0 * p8_bytes)
    PVAR("t4", AR, 4, false, 2, 5.0 * p8_bytes) PVAR("t4", AR, 4, false, 18, 5.0 * p8_bytes)
    PPROD("t8", AR, 8, false, 0, 9.0 * p8_bytes) PPROD("t8", AR, 8, false, 1, 9.0 * p8_bytes)
    PVAR("t8", AR, 8, false, 2, 9.0 * p8_bytes) PVAR("t8", AR, 8, false, 18, 9.0 * p8_bytes)
    vs.push_back({"pair saddr2 candidate U4 B256", [&](int k) {
                      pair_saddr2<OpSum, float, 4, 256><<<pgrid, 256>>>(po[k % PSETS], pa[k % PSETS], pb[k % PSETS], pn);
                  }, 3.0 * pair_bytes, {}});
    vs.push_back({"pair production body, launch_bounds 256", [&](int k) {
                      pair_tile_lb256<OpSum, float, 4, 3><<<pgrid, 256>>>(po[k % PSETS], pa[k % PSETS], pb[k % PSETS], pn);
                  }, 3.0 * pair_bytes, {}});
#define PMIX(SA)                                                                                              \
    vs.push_back({"pair mix global-nt loads, buffer st" #SA, [&](int k) {                                    \
                      pair_mix_k<SA><<<pgrid, 256>>>(po[k % PSETS], pa[k % PSETS], pb[k % PSETS]);           \
                  }, 3.0 * pair_bytes, {}});
    PMIX(2) PMIX(16) PMIX(18) PMIX(0)
    // aux bits: 1 sc0, 2 nt, 16 sc1
    PAIR(PROD, PROD) PAIR(2, 2) PAIR(2, 16) PAIR(2, 17) PAIR(2, 18) PAIR(2, 0) PAIR(16, 2) PAIR(18, 18) PAIR(0, 2)
    P8V(PROD, PROD, true, "scan8", 16.0 * p8_bytes) P8V(2, 2, true, "scan8", 16.0 * p8_bytes)
    P8V(2, 16, true, "scan8", 16.0 * p8_bytes) P8V(2, 17, true, "scan8", 16.0 * p8_bytes)
    P8V(2, 18, true, "scan8", 16.0 * p8_bytes) P8V(2, 0, true, "scan8", 16.0 * p8_bytes)
    P8V(16, 2, true, "scan8", 16.0 * p8_bytes) P8V(18, 18, true, "scan8", 16.0 * p8_bytes)
    P8V(PROD, PROD, false, "tree8", 9.0 * p8_bytes) P8V(2, 16, false, "tree8", 9.0 * p8_bytes)
    P8V(16, 2, false, "tree8", 9.0 * p8_bytes) P8V(18, 18, false, "tree8", 9.0 * p8_bytes)
    // bit-exactness of every variant against the production policy of its shape
    {
        std::vector<float> want, got;
        const std::string shapes[] = {"pair", "scan8", "tree8", "pscan8", "ptree8", "s2", "s4", "s8", "t2", "t4", "t8"};
        for (const auto& shape : shapes) {
            bool first = true;
            for (auto& v : vs) {
                if (v.name.rfind(shape + " ", 0) != 0) continue;
                v.launch(0);
                CHECK(hipDeviceSynchronize());
                const float* src = shape == "pair" ? po[0]
                                   : (shape == "scan8" || shape == "pscan8" || shape == "s8") ? sp[0].out[5]
                                   : (shape == "s2" || shape == "s4") ? sp[0].out[1] : tp[0].out[0];
                const size_t bytes = shape == "pair" ? pair_bytes : p8_bytes;
                (first ? want : got).resize(bytes / 4);
                CHECK(hipMemcpy((first ? want : got).data(), src, bytes, hipMemcpyDeviceToHost));
                if (!first && std::memcmp(want.data(), got.data(), bytes) != 0) {
                    std::printf("{\"variant\": \"%s\", \"error\": \"result differs from production policy\"}\n", v.name.c_str());
                    return 1;
                }
                first = false;
            }
        }
    }
    if (argc > 2) {  // keep only the variants whose name contains one of argv[2]'s '|'-separated parts
        std::vector<std::string> parts;
        for (std::string f = argv[2];;) {
            const size_t bar = f.find('|');
            parts.push_back(f.substr(0, bar));
            if (bar == std::string::npos) break;
            f = f.substr(bar + 1);
        }
        std::vector<Variant> keep;
        for (auto& v : vs)
            for (const auto& part : parts)
                if (v.name.find(part) != std::string::npos) {
                    keep.push_back(v);
                    break;
                }
        vs.swap(keep);
    }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int r = 0; r < rounds; ++r)
        for (auto& v : vs) {
            for (int k = 0; k < 2; ++k) v.launch(k);
            CHECK(hipEventRecord(e0));
            for (int k = 0; k < K; ++k) v.launch(k);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            v.us.push_back(ms * 1e3 / K);
        }
    for (auto& v : vs) {
        std::sort(v.us.begin(), v.us.end());
        const double us = v.us[v.us.size() / 2];
        std::printf("{\"variant\": \"%s\", \"median_us\": %.2f, \"min_us\": %.2f, \"frac\": %.4f, \"bit_exact\": true}\n",
                    v.name.c_str(), us, v.us.front(), v.bytes / (us * 1e-6) / 8e12);
    }
    return 0;
}
