// microbench_tailpol.hip — exploration harness (not part of the library): does the end of a pairwise launch
// (the ≈ 1.7 µs per launch that does not scale with size, DESIGN.md §5 "Where C3's time goes") shrink when
// only the LAST workgroups store with sc1 (the written line leaves the XCD L2 at once, MI355X_MICROARCH.md),
// so the release at the end of the kernel has less dirty L2 data to write back, while the bulk of the
// launch keeps the production nontemporal stores (sc1 stores on every tile cost 1-2 % at C2)?
//
// Variants (i64 max 64 MiB = C3, 8 rotating sets; f32 sum 256 MiB = C2, 4 rotating sets):
//   production   pair_tile<Op,T,4,3>: global nt loads and stores
//   tail<A,F>    the same tiles; workgroups b >= grid - grid*F/16 store through a per-tile buffer descriptor
//                with aux A (16 = sc1, 18 = nt sc1, 17 = sc0 sc1), the rest with global nt stores
// Every variant's result is compared with the production kernel's (bit-exact). Timing: events around K
// back-to-back launches per variant, variants interleaved over R rounds (median over rounds); run it under
// `rocprofv3 --kernel-trace` for per-launch medians (each variant is its own template instantiation).
//
// Build: hipcc -std=c++20 -O3 --offload-arch=gfx950 -ffp-contract=off tools/microbench_tailpol.hip -o build/mbt
// Run:   build/mbt [rounds, default 7]
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

// pair tile of U = 4 lane groups per thread, 256 threads, whole tiles only (the buckets here are multiples
// of the tile); the last F/16 of the grid stores with buffer aux A.
template <class Op, class T, int A, int F>
__global__ void __launch_bounds__(256) pair_tailpol(T* out, const T* a, const T* b) {
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
    const unsigned tail_from = gridDim.x - (gridDim.x * F) / 16;
    if (blockIdx.x >= tail_from) {  // uniform per workgroup
        char* tile = reinterpret_cast<char*>(out + static_cast<size_t>(blockIdx.x) * U * 256 * W);
        const auto r = __builtin_amdgcn_make_buffer_rsrc(tile, 0, U * 256 * 16, kRsrcWord3);
#pragma unroll
        for (int u = 0; u < U; ++u)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, combine<Op, T, W>(va[u], vb[u])), r,
                                                   (u * 256 + threadIdx.x) * 16u, 0, A);
    } else {
#pragma unroll
        for (int u = 0; u < U; ++u)
            store_lanes<true, T, W>(out + (base + u * 256) * W, combine<Op, T, W>(va[u], vb[u]));
    }
}

void* dalloc(size_t bytes) {
    void* p = nullptr;
    CHECK(hipMalloc(&p, bytes));
    return p;
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

template <class T>
struct Sets {
    std::vector<T*> a, b, o;
    size_t n = 0;
    Sets(size_t bytes, int sets) : n(bytes / sizeof(T)) {
        for (int s = 0; s < sets; ++s) {
            a.push_back(static_cast<T*>(dalloc(bytes)));
            b.push_back(static_cast<T*>(dalloc(bytes)));
            o.push_back(static_cast<T*>(dalloc(bytes)));
            fill_k<<<4096, 256>>>(reinterpret_cast<unsigned*>(a.back()), bytes / 4, 11 + s);
            fill_k<<<4096, 256>>>(reinterpret_cast<unsigned*>(b.back()), bytes / 4, 97 + s);
        }
    }
};

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 7;
    constexpr int K = 24;
    Sets<long> c3(size_t(64) << 20, 8);
    Sets<float> c2(size_t(256) << 20, 4);
    CHECK(hipDeviceSynchronize());
    const unsigned g3 = unsigned(c3.n * sizeof(long) / (16 * 4 * 256)), g2 = unsigned(c2.n * 4 / (16 * 4 * 256));
    std::vector<Variant> vs;
    const double b3 = 3.0 * (64 << 20), b2 = 3.0 * (256 << 20);
    vs.push_back({"c3 production pair_tile<OpMax,long,4,3>", [&](int k) {
                      const int s = k % 8;
                      pair_tile<OpMax, long, 4, 3><<<g3, 256>>>(c3.o[s], c3.a[s], c3.b[s], c3.n);
                  }, b3, {}});
#define C3V(A, F)                                                                                        \
    vs.push_back({"c3 tail aux" #A " F" #F "/16", [&](int k) {                                           \
                      const int s = k % 8;                                                                \
                      pair_tailpol<OpMax, long, A, F><<<g3, 256>>>(c3.o[s], c3.a[s], c3.b[s]);            \
                  }, b3, {}});
    C3V(16, 0) C3V(16, 1) C3V(16, 2) C3V(16, 4) C3V(16, 8) C3V(16, 16)
    C3V(18, 1) C3V(18, 2) C3V(18, 4) C3V(18, 16) C3V(17, 2) C3V(17, 16)
    vs.push_back({"c2 production pair_tile<OpSum,float,4,3>", [&](int k) {
                      const int s = k % 4;
                      pair_tile<OpSum, float, 4, 3><<<g2, 256>>>(c2.o[s], c2.a[s], c2.b[s], c2.n);
                  }, b2, {}});
#define C2V(A, F)                                                                                        \
    vs.push_back({"c2 tail aux" #A " F" #F "/16", [&](int k) {                                           \
                      const int s = k % 4;                                                                \
                      pair_tailpol<OpSum, float, A, F><<<g2, 256>>>(c2.o[s], c2.a[s], c2.b[s]);           \
                  }, b2, {}});
    C2V(16, 0) C2V(16, 1) C2V(16, 2) C2V(18, 1) C2V(18, 2)
    // bit-exactness against the production kernel of the same shape (set 0)
    for (const char* shape : {"c3 ", "c2 "}) {
        const bool is3 = shape[1] == '3';
        const size_t bytes = is3 ? c3.n * 8 : c2.n * 4;
        std::vector<unsigned char> want(bytes), got(bytes);
        bool first = true;
        for (auto& v : vs) {
            if (v.name.rfind(shape, 0) != 0) continue;
            CHECK(hipMemset(is3 ? static_cast<void*>(c3.o[0]) : static_cast<void*>(c2.o[0]), 0xA5, bytes));
            v.launch(0);
            CHECK(hipDeviceSynchronize());
            CHECK(hipMemcpy((first ? want : got).data(), is3 ? static_cast<void*>(c3.o[0]) : static_cast<void*>(c2.o[0]),
                            bytes, hipMemcpyDeviceToHost));
            if (!first && std::memcmp(want.data(), got.data(), bytes) != 0) {
                std::printf("{\"variant\": \"%s\", \"error\": \"result differs from production\"}\n", v.name.c_str());
                return 1;
            }
            first = false;
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
        std::printf("{\"variant\": \"%s\", \"median_us\": %.2f, \"min_us\": %.2f, \"frac\": %.4f, \"bit_exact\": true}\n",
                    v.name.c_str(), us, v.us.front(), v.bytes / (us * 1e-6) / 8e12);
    }
    return 0;
}
