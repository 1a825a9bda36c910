// microbench_sc1tail.hip — exploration harness (not part of the library): with NO MALL re-use (enough
// rotating sets that no bucket comes back while the MALL can still hold its sc1 lines, and a rotation that
// runs on across warm-up and timed launches), does storing the LAST X MiB of a launch with sc1 shorten
// its drain, alone or on top of the library's one-XCD mix (tile t % 8 == 0 sc1)? In place, i64 max at
// 64 MiB (C3) and f32 sum at 256 MiB (C2).
//
// (microbench_sc1mix3.hip) third sweep. The library took
// sweep 2's rule (k of every 8 tiles sc1, ~128 MiB per launch) and C2 got SLOWER (122 -> 130 us) while C3
// got faster (31.9 -> 30.1 us): the sweeps wrote a third buffer, but FMI's combine is in place (a = a + b,
// reference include/Communicator.h:180-189). Here every pattern runs both in place (out = a) and out of
// place, with the tail patterns (the last X MiB of tiles sc1) beside the mixes.
//
// (sweep 2) second sweep of
// microbench_sc1mix.hip (profiles/r02_sc1mix_events.jsonl: interleaving sc1 and nt tiles, 1 of 2 up to
// 256 MiB and 1 of 4 at 512 MiB, beat every tail / head / pure form, C2 126.7 -> 111.1 us). Here: the
// sc1 fraction against the bucket size (32 MiB ... 1 GiB), and the mix inside a tile (store instruction u
// of every thread sc1 when u % m < k) against the mix across tiles. First sweep's notes:
//
// (microbench_sc1mix.hip) the follow-up of
// microbench_tailsweep.hip (profiles/r02_tailsweep_events.jsonl): storing the last HALF of a pairwise
// launch's output with sc1 beat both all-nt and all-sc1 at 64 and 256 MiB (C2 121.6 -> 115.5 us). Is it the
// position (the tail) or the mix of the two store kinds in flight? Which tiles store sc1:
//   tail f    tiles b >= grid (1 - f)
//   head f    tiles b <  grid f
//   mix k/m   tiles with b % m < k (interleaved over the whole launch)
// Kernel: the production tile (U = 4 lane groups per thread, 256 threads, nt loads), sc1 tiles through a
// per-tile buffer descriptor with aux 16, the others global nt stores.
// Sizes 16 … 512 MiB per bucket, f32 sum and i64 max, rotating sets so that >= 1.5 GiB is touched per lap.
// Timing: events around K back-to-back launches per variant, variants interleaved over R rounds, median.
// Every variant's output is compared with X = 0's (bit-exact).
//
// Build: hipcc -std=c++20 -O3 --offload-arch=gfx950 -ffp-contract=off tools/microbench_sc1tail.hip -o build/mbt4
// Run:   build/mbt4 [rounds, default 5]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
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

constexpr int kRsrcWord3 = 0x00020000;  // raw 32-bit buffer, gfx9 family
constexpr unsigned kTileBytes = 4 * 256 * 16;

__device__ __forceinline__ bool sc1_tile(unsigned b, int mode, unsigned p1, unsigned p2) {
    if (mode == 5) return (b % 8) == 0 || b >= p1;  // one-XCD mix plus a tail from tile p1
    if (mode == 0) return b >= p1;       // tail: from tile p1
    if (mode == 1) return b < p1;        // head: below tile p1
    if (mode == 2) return (b % p2) < p1; // mix: p1 of every p2 tiles
    return false;                        // mode 3: per store instruction (below)
}

template <class Op, class T>
__global__ void __launch_bounds__(256) pair_mixk(T* out, const T* a, const T* b, int mode, unsigned p1, unsigned p2) {
    constexpr int W = kVecLanes<T>;
    constexpr int U = 4;
    using L = Lanes<T, W>;
    const size_t base = static_cast<size_t>(blockIdx.x) * U * 256 + threadIdx.x;
    L va[U], vb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        va[u] = load_lanes<true, T, W>(a + (base + u * 256) * W);
        vb[u] = load_lanes<true, T, W>(b + (base + u * 256) * W);
    }
    if (mode == 3) {  // intra: store instruction u sc1 when u % p2 < p1, in every tile
        char* tile = reinterpret_cast<char*>(out + static_cast<size_t>(blockIdx.x) * U * 256 * W);
        const auto r = __builtin_amdgcn_make_buffer_rsrc(tile, 0, kTileBytes, kRsrcWord3);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const L x = combine<Op, T, W>(va[u], vb[u]);
            if ((u % p2) < p1)
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, x), r, (u * 256 + threadIdx.x) * 16u, 0, 16);
            else
                store_lanes<true, T, W>(out + (base + u * 256) * W, x);
        }
    } else if (sc1_tile(blockIdx.x, mode, p1, p2)) {
        char* tile = reinterpret_cast<char*>(out + static_cast<size_t>(blockIdx.x) * U * 256 * W);
        const auto r = __builtin_amdgcn_make_buffer_rsrc(tile, 0, kTileBytes, kRsrcWord3);
#pragma unroll
        for (int u = 0; u < U; ++u)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, combine<Op, T, W>(va[u], vb[u])), r,
                                                   (u * 256 + threadIdx.x) * 16u, 0, 16);
    } else {
#pragma unroll
        for (int u = 0; u < U; ++u)
            store_lanes<true, T, W>(out + (base + u * 256) * W, combine<Op, T, W>(va[u], vb[u]));
    }
}

__global__ void fill_k(unsigned* p, size_t n, unsigned seed) {
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
        p[i] = static_cast<unsigned>((i * 2654435761u) ^ (seed * 40503u + (i >> 7)));
}

struct Variant {
    std::string name;
    std::function<void(int)> launch;
    double bytes;
    std::vector<double> us;
    std::string shape;
    void* check_out;
    size_t check_bytes;
};

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 5;
    constexpr int K = 24;
    struct Pat {
        const char* name;
        int mode;
        int num, den;
    };
    // tails in MiB of output (mode 4 -> kernel mode 0; mode 6 -> kernel mode 5 with a tail)
    const Pat pats[] = {{"nt", 0, 0, 1},          {"mix 1/8", 2, 1, 8},          {"tail 4MiB", 4, 4, 0},
                        {"tail 8MiB", 4, 8, 0},   {"tail 16MiB", 4, 16, 0},      {"tail 32MiB", 4, 32, 0},
                        {"mix 1/8 + tail 4MiB", 6, 4, 0}, {"mix 1/8 + tail 8MiB", 6, 8, 0},
                        {"mix 1/8 + tail 16MiB", 6, 16, 0}};
    std::vector<Variant> vs;
    std::vector<void*> keep;
    for (int shape_id = 0; shape_id < 2; ++shape_id) {
        const bool i64 = shape_id == 0;
        const size_t mib = i64 ? 64 : 256;
        const size_t bytes = mib << 20;
        const int sets = static_cast<int>((size_t(6) << 30) / (2 * bytes));  // 6 GiB of buckets in place
        char *A = nullptr, *B = nullptr;
        CHECK(hipMalloc(&A, bytes * sets));
        CHECK(hipMalloc(&B, bytes * sets));
        fill_k<<<4096, 256>>>(reinterpret_cast<unsigned*>(A), bytes * sets / 4, 11 + mib);
        fill_k<<<4096, 256>>>(reinterpret_cast<unsigned*>(B), bytes * sets / 4, 97 + mib);
        keep.insert(keep.end(), {A, B});
        const unsigned grid = static_cast<unsigned>(bytes / kTileBytes);
        const std::string shape = std::string(i64 ? "i64max " : "f32sum ") + std::to_string(mib) + "MiB";
        auto pos = std::make_shared<size_t>(0);  // running set index, shared by the shape's variants
        for (const Pat& pt : pats) {
            int kmode = pt.mode;
            unsigned p1 = 0, p2 = 1;
            if (pt.mode == 4 || pt.mode == 6) {
                p1 = grid - static_cast<unsigned>(std::min<size_t>(grid, (size_t(pt.num) << 20) / kTileBytes));
                kmode = pt.mode == 4 ? 0 : 5;
            } else if (pt.mode == 2) {
                p1 = pt.num, p2 = pt.den;
            } else {
                p1 = grid;  // nt: tail from the end, i.e. none
            }
            auto launch = [=](int) {
                const size_t off = (*pos % sets) * bytes;
                ++*pos;
                if (i64)
                    pair_mixk<OpMax, long><<<grid, 256>>>(reinterpret_cast<long*>(A + off), reinterpret_cast<const long*>(A + off),
                                                          reinterpret_cast<const long*>(B + off), kmode, p1, p2);
                else
                    pair_mixk<OpSum, float><<<grid, 256>>>(reinterpret_cast<float*>(A + off), reinterpret_cast<const float*>(A + off),
                                                           reinterpret_cast<const float*>(B + off), kmode, p1, p2);
            };
            vs.push_back({shape + " " + pt.name, launch, 3.0 * bytes, {}, "inplace", A, bytes});
        }
    }
    CHECK(hipDeviceSynchronize());
    {  // bit-exactness: every variant of a shape against its all-nt form
        std::vector<unsigned char> want, got;
        std::string cur;
        for (auto& v : vs) {
            if (v.shape.rfind("inplace", 0) == 0) continue;  // in place rewrites its input: timing only
            CHECK(hipMemset(v.check_out, 0xA5, v.check_bytes));
            v.launch(0);
            CHECK(hipDeviceSynchronize());
            auto& dst = v.shape != cur ? want : got;
            dst.resize(v.check_bytes);
            CHECK(hipMemcpy(dst.data(), v.check_out, v.check_bytes, hipMemcpyDeviceToHost));
            if (v.shape == cur && std::memcmp(want.data(), got.data(), v.check_bytes) != 0) {
                std::printf("{\"variant\": \"%s\", \"error\": \"result differs from X = 0\"}\n", v.name.c_str());
                return 1;
            }
            cur = v.shape;
        }
    }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int r = 0; r < rounds; ++r)
        for (auto& v : vs) {
            for (int k = 0; k < 3; ++k) v.launch(k);
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
        std::printf("{\"variant\": \"%s\", \"median_us\": %.3f, \"min_us\": %.3f, \"frac\": %.4f, \"bit_exact\": true}\n",
                    v.name.c_str(), us, v.us.front(), v.bytes / (us * 1e-6) / 8e12);
    }
    for (void* p : keep) CHECK(hipFree(p));
    return 0;
}
