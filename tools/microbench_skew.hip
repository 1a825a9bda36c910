// microbench_skew.hip — exploration harness (not part of the library): the P = 8 peer scan's 16 buckets
// (8 inputs + 8 outputs, 64 MiB f32) carved out of ONE allocation at controlled offsets, to find a bucket
// placement rule that avoids the slow placements seen with tools/microbench_placement.hip (a 3 GiB arena
// with buckets at multiples of 64 MiB is consistently slow: 0.68–0.71 of peak vs 0.74–0.80 for separate
// allocations).
//
//   offset_k = k · (64 MiB + skew)                      ("stride" schemes)
//   offset_k = k · 64 MiB + ((k · m) mod c) · unit      ("color" schemes)
//
// Build: hipcc -std=c++20 -O3 --offload-arch=gfx950 -ffp-contract=off tools/microbench_skew.hip -o build/mbs
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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

constexpr int P = 8;

template <class F>
double median_us(F&& launch, int iters) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    launch();
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    std::vector<double> t;
    for (int r = 0; r < iters; ++r) {
        CHECK(hipEventRecord(e0));
        launch();
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        t.push_back(ms * 1e3);
    }
    CHECK(hipGetLastError());
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

struct Scheme {
    std::string name;
    std::vector<size_t> off;  // 16 byte offsets into the arena
};

int main() {
    const size_t n = (64u << 20) / 4, bytes = n * 4, nvec = n / 4;
    const size_t KiB = 1024, MiB = 1024 * 1024;
    std::vector<Scheme> schemes;
    auto stride = [&](const char* name, size_t skew) {
        Scheme s{name, {}};
        for (int k = 0; k < 16; ++k) s.off.push_back(k * (bytes + skew));
        schemes.push_back(s);
    };
    auto color = [&](const char* name, size_t mult, size_t colors, size_t unit) {
        Scheme s{name, {}};
        for (size_t k = 0; k < 16; ++k) s.off.push_back(k * (bytes + colors * unit) + ((k * mult) % colors) * unit);
        schemes.push_back(s);
    };
    stride("stride skew 0", 0);
    stride("stride skew 4 KiB", 4 * KiB);
    stride("stride skew 4352 B", 4352);
    stride("stride skew 64 KiB", 64 * KiB);
    stride("stride skew 68 KiB", 68 * KiB);
    stride("stride skew 256 KiB", 256 * KiB);
    stride("stride skew 1 MiB", MiB);
    stride("stride skew 2 MiB", 2 * MiB);
    stride("stride skew 2 MiB + 4352 B", 2 * MiB + 4352);
    stride("stride skew 3 MiB", 3 * MiB);
    stride("stride skew 6 MiB", 6 * MiB);
    stride("stride skew 10 MiB", 10 * MiB);
    color("color k*5 mod 16 x 4 KiB", 5, 16, 4 * KiB);
    color("color k*5 mod 16 x 64 KiB", 5, 16, 64 * KiB);
    color("color k*7 mod 16 x 256 KiB", 7, 16, 256 * KiB);
    color("color k*3 mod 16 x 1 MiB", 3, 16, MiB);
    color("color k*5 mod 8 x 2 MiB", 5, 8, 2 * MiB);
    size_t need = 0;
    for (auto& s : schemes) need = std::max(need, s.off.back() + bytes);
    char* arena;
    CHECK(hipMalloc(&arena, need));
    CHECK(hipMemset(arena, 0, need));
    std::printf("{\"arena_bytes\": %zu}\n", need);
    const unsigned grid = static_cast<unsigned>(nvec / 256);
    const double scan_bytes = 2.0 * P * bytes, tree_bytes = (P + 1.0) * bytes;
    for (int round = 0; round < 2; ++round)
        for (auto& s : schemes) {
            PeerPtrs p{};
            for (int j = 0; j < P; ++j) {
                p.in[j] = arena + s.off[j];
                p.out[j] = arena + s.off[8 + j];
            }
            const double us_scan = median_us([&] { scan_kernel<OpSum, float, fmi::sched::kScan, P><<<grid, 256>>>(p, n, 0); }, 9);
            const double us_tree =
                median_us([&] { tree_kernel<OpSum, float, fmi::sched::kAllreduce, P, false><<<grid, 256>>>(p, n, 0, 0); }, 9);
            std::printf("{\"round\": %d, \"scheme\": \"%s\", \"scan8_us\": %.2f, \"scan8_frac\": %.4f, \"tree8_us\": %.2f, "
                        "\"tree8_frac\": %.4f}\n",
                        round, s.name.c_str(), us_scan, scan_bytes / (us_scan * 1e-6) / 8e12, us_tree,
                        tree_bytes / (us_tree * 1e-6) / 8e12);
            std::fflush(stdout);
        }
    return 0;
}
