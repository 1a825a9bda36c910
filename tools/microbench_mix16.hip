// microbench_mix16.hip — exploration harness (not part of the library): what does the chip stream for C3's
// peer-scan shape — 8 input buckets read and 8 output buckets written in one kernel, 64 MiB each, every
// bucket its own hipMalloc as the caller's buckets are — when the kernel does no arithmetic at all? That is
// the ceiling the scan kernel (scan_kernel<OpSum, float, ., 8>, P reads + P writes, 2·P·n·4 bytes) can be held
// against (VERDICT r02 "next" 7). Kernels, all with the production tile (256 threads, U = 4 lane groups of
// 16 B per thread per bucket, nontemporal loads and stores), on the same 16 buckets per draw:
//   copy8      out_p = in_p, p < 8                     8 read + 8 write streams (the scan's traffic)
//   read16     acc ^= in_p for 16 buckets, 1 store of the xor per workgroup-tile row (read-only bound)
//   write16    out_p = const for 16 buckets            (write-only bound)
//   copy8_2ph  copy8 storing outputs 0..3 of the tile first, then 4..7, the loads of 4..7 after the first
//              stores (4 + 4 write streams per phase)
//   scan8      the library's own peer scan (fmi_dev_scan_peers, scan_no_order, f32 sum) on the same buckets
//   copy8_xcd  copy8 with an XCD-contiguous tile order: workgroup b (dispatched to XCD b % 8) copies tile
//              (b % 8) * T/8 + b / 8, so each XCD streams its own eighth of every bucket instead of all XCDs
//              sharing one moving window (does DRAM locality improve on the slow placements?)
//   pair3 / pair3_xcd   C2's shape (2 reads + 1 write, f32 sum) on buckets 0..2 of the set, both tile orders
//   sum8       8 reads + 1 write, plain f32 sum in index order (no reference bracketing): the traffic of the
//              N = 8 shard kernel / C3's 8-peer tree
//   tree8      the library's fused 8-peer allreduce (fmi_dev_reduce_tree, allreduce_no_order order)
// Draws: each draw allocates a fresh set of 2 x 16 x 64 MiB buckets (two rotating sets, 2 GiB, beyond the
// 256 MB MALL), so placement varies draw to draw as it does between callers; per draw, the kernels run
// interleaved over R rounds of K back-to-back launches (events), median per kernel.
//
// Build: hipcc -std=c++20 -O3 --offload-arch=gfx950 -ffp-contract=off tools/microbench_mix16.hip
//          -Lfmi_amd/lib -lfmi_dev -Wl,-rpath,$PWD/fmi_amd/lib -o build/mbm16
// Run:   build/mbm16 [draws, default 6] [rounds, default 5]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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

constexpr int kP = 8;
constexpr int kU = 4;
using V = u32x4;

struct Ptrs16 {
    const V* in[16];
    V* out[16];
};

__device__ __forceinline__ V ld(const V* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void st(V* p, V v) { __builtin_nontemporal_store(v, p); }

__global__ void __launch_bounds__(256) copy8(Ptrs16 b) {
    const size_t base = static_cast<size_t>(blockIdx.x) * kU * 256 + threadIdx.x;
    V v[kP][kU];
#pragma unroll
    for (int p = 0; p < kP; ++p)
#pragma unroll
        for (int u = 0; u < kU; ++u) v[p][u] = ld(b.in[p] + base + u * 256);
#pragma unroll
    for (int p = 0; p < kP; ++p)
#pragma unroll
        for (int u = 0; u < kU; ++u) st(b.out[p] + base + u * 256, v[p][u]);
}

__device__ __forceinline__ size_t xcd_tile(unsigned b, unsigned tiles) {
    const unsigned per = tiles / 8;  // tiles % 8 == 0 (64 MiB buckets)
    return static_cast<size_t>(b % 8) * per + b / 8;
}

__global__ void __launch_bounds__(256) copy8_xcd(Ptrs16 b) {
    const size_t base = xcd_tile(blockIdx.x, gridDim.x) * kU * 256 + threadIdx.x;
    V v[kP][kU];
#pragma unroll
    for (int p = 0; p < kP; ++p)
#pragma unroll
        for (int u = 0; u < kU; ++u) v[p][u] = ld(b.in[p] + base + u * 256);
#pragma unroll
    for (int p = 0; p < kP; ++p)
#pragma unroll
        for (int u = 0; u < kU; ++u) st(b.out[p] + base + u * 256, v[p][u]);
}

template <bool XCD>
__global__ void __launch_bounds__(256) pair3(Ptrs16 b) {
    const size_t t = XCD ? xcd_tile(blockIdx.x, gridDim.x) : blockIdx.x;
    const size_t base = t * kU * 256 + threadIdx.x;
    using F4 = float __attribute__((ext_vector_type(4)));
    V x[kU], y[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        x[u] = ld(b.in[0] + base + u * 256);
        y[u] = ld(b.in[1] + base + u * 256);
    }
#pragma unroll
    for (int u = 0; u < kU; ++u)
        st(b.out[0] + base + u * 256, __builtin_bit_cast(V, __builtin_bit_cast(F4, x[u]) + __builtin_bit_cast(F4, y[u])));
}

__global__ void __launch_bounds__(256) sum8(Ptrs16 b) {
    const size_t base = static_cast<size_t>(blockIdx.x) * kU * 256 + threadIdx.x;
    using F4 = float __attribute__((ext_vector_type(4)));
    F4 acc[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) acc[u] = __builtin_bit_cast(F4, ld(b.in[0] + base + u * 256));
#pragma unroll
    for (int p = 1; p < kP; ++p)
#pragma unroll
        for (int u = 0; u < kU; ++u) acc[u] += __builtin_bit_cast(F4, ld(b.in[p] + base + u * 256));
#pragma unroll
    for (int u = 0; u < kU; ++u) st(b.out[0] + base + u * 256, __builtin_bit_cast(V, acc[u]));
}

__global__ void __launch_bounds__(256) copy8_2ph(Ptrs16 b) {
    const size_t base = static_cast<size_t>(blockIdx.x) * kU * 256 + threadIdx.x;
    V v[kP / 2][kU];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int p = 0; p < kP / 2; ++p)
#pragma unroll
            for (int u = 0; u < kU; ++u) v[p][u] = ld(b.in[h * 4 + p] + base + u * 256);
#pragma unroll
        for (int p = 0; p < kP / 2; ++p)
#pragma unroll
            for (int u = 0; u < kU; ++u) st(b.out[h * 4 + p] + base + u * 256, v[p][u]);
    }
}

__global__ void __launch_bounds__(256) read16(Ptrs16 b, V* sink) {
    const size_t base = static_cast<size_t>(blockIdx.x) * kU * 256 + threadIdx.x;
    V acc = {0, 0, 0, 0};
#pragma unroll
    for (int p = 0; p < 16; ++p) {
        const V* src = p < 8 ? b.in[p] : reinterpret_cast<const V*>(b.out[p - 8]);
#pragma unroll
        for (int u = 0; u < kU; ++u) acc ^= ld(src + base + u * 256);
    }
    if (acc[0] == 0x9E3779B9u && acc[1] == 0x7F4A7C15u) st(sink + threadIdx.x, acc);  // never true: keeps the loads
}

__global__ void __launch_bounds__(256) write16(Ptrs16 b) {
    const size_t base = static_cast<size_t>(blockIdx.x) * kU * 256 + threadIdx.x;
    const V c = {blockIdx.x, threadIdx.x, 7u, 9u};
#pragma unroll
    for (int p = 0; p < 16; ++p) {
        V* dst = p < 8 ? const_cast<V*>(b.in[p]) : b.out[p - 8];
#pragma unroll
        for (int u = 0; u < kU; ++u) st(dst + base + u * 256, c);
    }
}

struct Kernel {
    std::string name;
    double bytes;  // per launch
    std::function<void(int)> launch;
    std::vector<double> us;
};

int main(int argc, char** argv) {
    const int draws = argc > 1 ? std::atoi(argv[1]) : 6;
    const int rounds = argc > 2 ? std::atoi(argv[2]) : 5;
    constexpr int K = 12;
    constexpr size_t kBytes = size_t(64) << 20;
    const size_t nvec = kBytes / 16;
    const unsigned grid = static_cast<unsigned>(nvec / (kU * 256));
    CHECK(hipSetDevice(0));
    if (fmi_dev_init(0) != FMI_OK) {
        std::fprintf(stderr, "fmi_dev_init: %s\n", fmi_last_error());
        return 1;
    }
    V* sink = nullptr;
    CHECK(hipMalloc(&sink, 4096));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipStream_t s = nullptr;  // one explicit stream for every launch, the library's scan included
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    for (int d = 0; d < draws; ++d) {
        std::vector<void*> bufs;
        Ptrs16 sets[2];
        for (int k = 0; k < 2; ++k)
            for (int p = 0; p < kP; ++p) {
                void *i = nullptr, *o = nullptr;
                CHECK(hipMalloc(&i, kBytes));
                CHECK(hipMalloc(&o, kBytes));
                CHECK(hipMemset(i, 0x3c, kBytes));  // finite f32 values for the scan
                CHECK(hipMemset(o, 0, kBytes));
                sets[k].in[p] = static_cast<const V*>(i);
                sets[k].out[p] = static_cast<V*>(o);
                bufs.push_back(i);
                bufs.push_back(o);
            }
        CHECK(hipDeviceSynchronize());
        const double rw = 2.0 * kP * kBytes;
        std::vector<Kernel> ks = {
            {"copy8", rw, [&](int k) { copy8<<<grid, 256, 0, s>>>(sets[k & 1]); }, {}},
            {"copy8_2ph", rw, [&](int k) { copy8_2ph<<<grid, 256, 0, s>>>(sets[k & 1]); }, {}},
            {"copy8_xcd", rw, [&](int k) { copy8_xcd<<<grid, 256, 0, s>>>(sets[k & 1]); }, {}},
            {"pair3", 3.0 * kBytes, [&](int k) { pair3<false><<<grid, 256, 0, s>>>(sets[k & 1]); }, {}},
            {"pair3_xcd", 3.0 * kBytes, [&](int k) { pair3<true><<<grid, 256, 0, s>>>(sets[k & 1]); }, {}},
            {"sum8", 9.0 * kBytes, [&](int k) { sum8<<<grid, 256, 0, s>>>(sets[k & 1]); }, {}},
            {"tree8", 9.0 * kBytes, [&](int k) {
                 const Ptrs16& b = sets[k & 1];
                 const void* ins[kP];
                 for (int p = 0; p < kP; ++p) ins[p] = b.in[p];
                 if (fmi_dev_reduce_tree(FMI_OP_SUM, FMI_F32, FMI_ALG_ALLREDUCE, b.out[0], ins, kP, 0, kBytes / 4, s) != FMI_OK) {
                     std::fprintf(stderr, "tree: %s\n", fmi_last_error());
                     std::exit(1);
                 }
             }, {}},
            {"read16", rw, [&](int k) { read16<<<grid, 256, 0, s>>>(sets[k & 1], sink); }, {}},
            {"write16", rw, [&](int k) { write16<<<grid, 256, 0, s>>>(sets[k & 1]); }, {}},
            {"scan8", rw, [&](int k) {
                 const Ptrs16& b = sets[k & 1];
                 void* outs[kP];
                 const void* ins[kP];
                 for (int p = 0; p < kP; ++p) {
                     outs[p] = b.out[p];
                     ins[p] = b.in[p];
                 }
                 if (fmi_dev_scan_peers(FMI_OP_SUM, FMI_F32, FMI_ALG_SCAN, outs, ins, kP, kBytes / 4, s) != FMI_OK) {
                     std::fprintf(stderr, "scan: %s\n", fmi_last_error());
                     std::exit(1);
                 }
             }, {}},
        };
        for (int r = 0; r < rounds; ++r)
            for (auto& kn : ks) {
                for (int k = 0; k < 2; ++k) kn.launch(k);
                CHECK(hipEventRecord(e0, s));
                for (int k = 0; k < K; ++k) kn.launch(k);
                CHECK(hipEventRecord(e1, s));
                CHECK(hipEventSynchronize(e1));
                float ms = 0;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                kn.us.push_back(ms * 1e3 / K);
            }
        for (auto& kn : ks) {
            std::sort(kn.us.begin(), kn.us.end());
            const double us = kn.us[kn.us.size() / 2];
            std::printf("{\"draw\": %d, \"kernel\": \"%s\", \"median_us\": %.2f, \"min_us\": %.2f, \"frac\": %.4f}\n", d,
                        kn.name.c_str(), us, kn.us.front(), kn.bytes / (us * 1e-6) / 8e12);
        }
        std::fflush(stdout);
        for (void* p : bufs) CHECK(hipFree(p));
    }
    return 0;
}
