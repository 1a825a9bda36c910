// microbench_tailsweep.hip — exploration harness (not part of the library), the follow-up of
// microbench_tailpol.hip: that run (profiles/r02_tailpol_*) found the pairwise launch faster when only its
// last workgroups store with sc1 — at C3 (64 MiB i64) when the last 32 MiB of output did, at C2 (256 MiB f32)
// also when the last 32 MiB did. Is the right rule "the last X bytes of output", and which X, across sizes?
//
// Kernel: the production tile (U = 4 lane groups per thread, 256 threads, nt loads); workgroups
// b >= tail_from (a kernel argument, as the library would pass it) store with buffer aux 16 (sc1), the
// others with global nt stores. X = (grid - tail_from) tiles x 16 KiB of output.
// Sizes 1 … 512 MiB per bucket, f32 sum and i64 max, rotating sets so that >= 1.5 GiB is touched per lap.
// Timing: events around K back-to-back launches per variant, variants interleaved over R rounds, median.
// Every variant's output is compared with X = 0's (bit-exact).
//
// Build: hipcc -std=c++20 -O3 --offload-arch=gfx950 -ffp-contract=off tools/microbench_tailsweep.hip -o build/mbs
// Run:   build/mbs [rounds, default 5]
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

constexpr int kRsrcWord3 = 0x00020000;  // raw 32-bit buffer, gfx9 family
constexpr unsigned kTileBytes = 4 * 256 * 16;

template <class Op, class T>
__global__ void __launch_bounds__(256) pair_tailx(T* out, const T* a, const T* b, unsigned tail_from) {
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
    if (blockIdx.x >= tail_from) {
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
    const size_t mibs[] = {1, 4, 16, 64, 256, 512};
    const size_t xs_mib[] = {0, 4, 8, 16, 24, 32, 48, 64, 96, 128};
    std::vector<Variant> vs;
    std::vector<void*> keep;
    for (int dt = 0; dt < 2; ++dt)
        for (size_t mib : mibs) {
            const size_t bytes = mib << 20;
            const int sets = static_cast<int>(std::max<size_t>(2, (size_t(1536) << 20) / (3 * bytes)));
            // one allocation per role, carved into sets (the small sizes would otherwise need thousands)
            char *A = nullptr, *B = nullptr, *O = nullptr;
            CHECK(hipMalloc(&A, bytes * sets));
            CHECK(hipMalloc(&B, bytes * sets));
            CHECK(hipMalloc(&O, bytes * sets));
            fill_k<<<4096, 256>>>(reinterpret_cast<unsigned*>(A), bytes * sets / 4, 11 + mib);
            fill_k<<<4096, 256>>>(reinterpret_cast<unsigned*>(B), bytes * sets / 4, 97 + mib);
            keep.insert(keep.end(), {A, B, O});
            const unsigned grid = static_cast<unsigned>(bytes / kTileBytes);
            const std::string shape = std::string(dt ? "i64max " : "f32sum ") + std::to_string(mib) + "MiB";
            std::vector<size_t> xs;
            for (size_t x : xs_mib)
                if (x < mib) xs.push_back(x);
            xs.push_back(mib);  // every tile
            for (size_t x : xs) {
                const unsigned tail_tiles = static_cast<unsigned>(std::min<size_t>(grid, (x << 20) / kTileBytes));
                const unsigned tail_from = grid - tail_tiles;
                auto launch = [=](int k) {
                    const size_t off = static_cast<size_t>(k % sets) * bytes;
                    if (dt)
                        pair_tailx<OpMax, long><<<grid, 256>>>(reinterpret_cast<long*>(O + off), reinterpret_cast<const long*>(A + off),
                                                               reinterpret_cast<const long*>(B + off), tail_from);
                    else
                        pair_tailx<OpSum, float><<<grid, 256>>>(reinterpret_cast<float*>(O + off), reinterpret_cast<const float*>(A + off),
                                                                reinterpret_cast<const float*>(B + off), tail_from);
                };
                vs.push_back({shape + " tail " + std::to_string(x) + "MiB", launch, 3.0 * bytes, {}, shape, O, bytes});
            }
        }
    CHECK(hipDeviceSynchronize());
    {  // bit-exactness: every variant of a shape against its X = 0
        std::vector<unsigned char> want, got;
        std::string cur;
        for (auto& v : vs) {
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
