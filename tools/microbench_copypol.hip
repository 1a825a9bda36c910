// microbench_copypol.hip — exploration harness (not part of the library): access policy of the library's
// device copy (copy_tile, fmi_kernels.h: the one-rank allreduce and the communicator's staging copies). The
// fused scan's buffer stores with nt sc1 beat a plain nontemporal 8-in / 8-out copy of the same buckets by
// 3–10 % (profiles/r03_c3_scan_vs_16stream_ceiling.jsonl, r03_xcd_tile_order_rejected.jsonl): does a single
// copy stream gain the same way? Variants, all with the production tile (256 threads, U = 4 x 16 B per thread):
//   nt        global nontemporal loads and stores (the library's copy_tile)
//   buf_ntsc1 buffer loads nt, buffer stores nt sc1 (the scan's policy)
//   buf_sc1   buffer loads nt, buffer stores sc1 (the tree's policy)
//   xcd1_sc1  global nt, but tiles t % 8 == 0 (one XCD) store sc1 (the pair kernel's policy)
// Bucket: 256 MiB (and 64 MiB), separate hipMallocs, rotating sets covering >= 8 GiB so that no set is re-read
// from the 256 MB MALL; events around K back-to-back launches per variant, interleaved over R rounds, median;
// every variant's output compared with the source (bit-exact).
//
// Build: hipcc -std=c++20 -O3 --offload-arch=gfx950 -ffp-contract=off tools/microbench_copypol.hip -o build/mbcp
// Run:   build/mbcp [rounds, default 5]
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

constexpr int kU = 4;
using V = u32x4;

// MODE 0 nt, 1 buffer nt-load / nt-sc1-store, 2 buffer nt-load / sc1-store, 3 global nt with one XCD's tiles sc1
template <int MODE>
__global__ void __launch_bounds__(256) copy_pol(char* out, const char* in) {
    const size_t tile_byte = static_cast<size_t>(blockIdx.x) * kU * 256 * 16;
    const size_t base = static_cast<size_t>(blockIdx.x) * kU * 256 + threadIdx.x;
    V v[kU];
    if constexpr (MODE == 1 || MODE == 2) {
#pragma unroll
        for (int u = 0; u < kU; ++u)
            v[u] = __builtin_bit_cast(V, load_tile<kAuxNT, unsigned, 4>(in, tile_byte, (u * 256 + threadIdx.x) * 16u));
#pragma unroll
        for (int u = 0; u < kU; ++u)
            store_tile<MODE == 1 ? (kAuxNT | kAuxSC1) : kAuxSC1, unsigned, 4>(
                out, tile_byte, (u * 256 + threadIdx.x) * 16u, __builtin_bit_cast(Lanes<unsigned, 4>, v[u]));
    } else {
        const V* src = reinterpret_cast<const V*>(in);
#pragma unroll
        for (int u = 0; u < kU; ++u) v[u] = __builtin_nontemporal_load(src + base + u * 256);
        if (MODE == 3 && (blockIdx.x & 7u) == 0) {
#pragma unroll
            for (int u = 0; u < kU; ++u)
                store_tile<kAuxSC1, unsigned, 4>(out, tile_byte, (u * 256 + threadIdx.x) * 16u,
                                                 __builtin_bit_cast(Lanes<unsigned, 4>, v[u]));
        } else {
            V* dst = reinterpret_cast<V*>(out);
#pragma unroll
            for (int u = 0; u < kU; ++u) __builtin_nontemporal_store(v[u], dst + base + u * 256);
        }
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
};

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 5;
    constexpr int K = 20;
    std::vector<Variant> vs;
    std::vector<void*> keep;
    for (size_t mib : {size_t(256), size_t(64)}) {
        const size_t bytes = mib << 20;
        const int sets = static_cast<int>(std::max<size_t>(4, (size_t(8) << 30) / (2 * bytes)));
        std::vector<char*> a(sets), b(sets);
        for (int k = 0; k < sets; ++k) {
            CHECK(hipMalloc(&a[k], bytes));
            CHECK(hipMalloc(&b[k], bytes));
            fill_k<<<4096, 256>>>(reinterpret_cast<unsigned*>(a[k]), bytes / 4, 7 + k);
            keep.push_back(a[k]);
            keep.push_back(b[k]);
        }
        const unsigned grid = static_cast<unsigned>(bytes / (kU * 256 * 16));
        const std::string shape = std::to_string(mib) + "MiB sets=" + std::to_string(sets) + " ";
        auto add = [&](const char* name, void (*k)(char*, const char*)) {
            vs.push_back({shape + name, [=](int i) { k<<<grid, 256>>>(b[i % sets], a[i % sets]); }, 2.0 * bytes, {}});
        };
        add("nt", copy_pol<0>);
        add("buf_ntsc1", copy_pol<1>);
        add("buf_sc1", copy_pol<2>);
        add("xcd1_sc1", copy_pol<3>);
        CHECK(hipDeviceSynchronize());
        for (size_t v = vs.size() - 4; v < vs.size(); ++v) {  // bit-exactness of every variant
            CHECK(hipMemset(b[0], 0, bytes));
            vs[v].launch(0);
            CHECK(hipDeviceSynchronize());
            std::vector<unsigned char> x(bytes), y(bytes);
            CHECK(hipMemcpy(x.data(), a[0], bytes, hipMemcpyDeviceToHost));
            CHECK(hipMemcpy(y.data(), b[0], bytes, hipMemcpyDeviceToHost));
            if (std::memcmp(x.data(), y.data(), bytes) != 0) {
                std::printf("{\"variant\": \"%s\", \"error\": \"copy differs\"}\n", vs[v].name.c_str());
                return 1;
            }
        }
    }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::vector<int> next(vs.size(), 0);
    for (int r = 0; r < rounds; ++r)
        for (size_t v = 0; v < vs.size(); ++v) {
            for (int k = 0; k < 3; ++k) vs[v].launch(next[v]++);
            CHECK(hipEventRecord(e0));
            for (int k = 0; k < K; ++k) vs[v].launch(next[v]++);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            vs[v].us.push_back(ms * 1e3 / K);
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
