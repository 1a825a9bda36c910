// microbench_chainpol.hip — exploration harness (not part of the library): the many-peer scan_ltr regime
// (P = 256 peers x 4 MiB runs at 0.15 of peak, while reduce_ltr over the same inputs, one
// output, runs at 0.71). Is it the P output streams? The production chain step (16 loads, the running
// value, 16 stores) with the stores as global nt (production), global plain, buffer sc1, buffer nt sc1, and a
// variant that stores only every 16th output (the same loads and arithmetic, 1/16 of the write streams).
// One launch per variant covers all P peers (pointer tables in device memory); outputs rotate over sets.
//
// Build: hipcc -std=c++20 -O3 --offload-arch=gfx950 -ffp-contract=off tools/microbench_chainpol.hip -o build/mbch
// Run:   build/mbch [rounds, default 5]
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

constexpr int BL = 16;

// MODE: 0 global nt, 1 global plain, 2 buffer sc1, 3 buffer nt sc1, 4 global nt but only q == 15 stored
template <int MODE>
__device__ __forceinline__ void put(float* bucket, size_t tile_byte, unsigned lane_byte, const Lanes<float, 4>& v, int q) {
    if constexpr (MODE == 0) {
        store_lanes<true, float, 4>(reinterpret_cast<float*>(reinterpret_cast<char*>(bucket) + tile_byte + lane_byte), v);
    } else if constexpr (MODE == 1) {
        store_lanes<false, float, 4>(reinterpret_cast<float*>(reinterpret_cast<char*>(bucket) + tile_byte + lane_byte), v);
    } else if constexpr (MODE == 2) {
        store_tile<kAuxSC1, float, 4>(bucket, tile_byte, lane_byte, v);
    } else if constexpr (MODE == 3) {
        store_tile<kAuxNT | kAuxSC1, float, 4>(bucket, tile_byte, lane_byte, v);
    } else {
        if (q == BL - 1)
            store_lanes<true, float, 4>(reinterpret_cast<float*>(reinterpret_cast<char*>(bucket) + tile_byte + lane_byte), v);
    }
}

template <int MODE>
__global__ void __launch_bounds__(256) chain_scan(const float* const* __restrict__ ins, float* const* __restrict__ outs,
                                                  int P, size_t nvec) {
    extern __shared__ char lds_cap[];  // residency cap: the launch reserves LDS as the library's chain does
    if (nvec == 0) lds_cap[threadIdx.x] = 0;
    const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
    for (size_t g = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; g < nvec; g += stride) {
        const size_t tile_byte = (g - threadIdx.x) * 16;
        const unsigned lane_byte = threadIdx.x * 16u;
        Lanes<float, 4> acc = load_lanes<true, float, 4>(ins[0] + g * 4);
        put<MODE>(outs[0], tile_byte, lane_byte, acc, BL - 1);
        for (int base = 1; base < P; base += BL) {
            const int m = std::min(BL, P - base);
            Lanes<float, 4> x[BL];
#pragma unroll
            for (int q = 0; q < BL; ++q)
                if (q < m) x[q] = load_lanes<true, float, 4>(ins[base + q] + g * 4);
#pragma unroll
            for (int q = 0; q < BL; ++q)
                if (q < m) x[q] = acc = combine<OpSum, float, 4>(acc, x[q]);
#pragma unroll
            for (int q = 0; q < BL; ++q)
                if (q < m) put<MODE>(outs[base + q], tile_byte, lane_byte, x[q], q);
        }
    }
}

// The same chain with the pointer table passed by value in the kernel arguments (the library's
// BlockedScanPtrs, <= 128 peers), global nt stores.
__global__ void __launch_bounds__(256) chain_scan_kernarg(BlockedScanPtrs ptrs, int P, size_t nvec) {
    extern __shared__ char lds_cap[];
    if (nvec == 0) lds_cap[threadIdx.x] = 0;
    const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
    for (size_t g = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; g < nvec; g += stride) {
        const size_t tile_byte = (g - threadIdx.x) * 16;
        const unsigned lane_byte = threadIdx.x * 16u;
        Lanes<float, 4> acc = load_lanes<true, float, 4>(static_cast<const float*>(ptrs.in[0]) + g * 4);
        put<0>(static_cast<float*>(ptrs.out[0]), tile_byte, lane_byte, acc, BL - 1);
        for (int base = 1; base < P; base += BL) {
            const int m = std::min(BL, P - base);
            Lanes<float, 4> x[BL];
#pragma unroll
            for (int q = 0; q < BL; ++q)
                if (q < m) x[q] = load_lanes<true, float, 4>(static_cast<const float*>(ptrs.in[base + q]) + g * 4);
#pragma unroll
            for (int q = 0; q < BL; ++q)
                if (q < m) x[q] = acc = combine<OpSum, float, 4>(acc, x[q]);
#pragma unroll
            for (int q = 0; q < BL; ++q)
                if (q < m) put<0>(static_cast<float*>(ptrs.out[base + q]), tile_byte, lane_byte, x[q], q);
        }
    }
}

__global__ void fill_k(unsigned* p, size_t n, unsigned seed) {
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
        p[i] = 0x3f800000u | (static_cast<unsigned>((i * 2654435761u) ^ (seed * 40503u)) & 0x007fffffu);
}

struct Variant {
    std::string name;
    std::function<void(int)> launch;
    double bytes;
    std::vector<double> us;
};

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 5;
    constexpr int K = 4, SETS = 3;
    const size_t bytes = size_t(4) << 20, n = bytes / 4, nvec = n / 4;
    const size_t lds = 80 << 10;  // 2 workgroups per CU, as the library's 16-stream kernels
    std::vector<Variant> vs;
    for (int P : {64, 128, 256}) {
        std::vector<float*> hin(P);
        for (int p = 0; p < P; ++p) {
            CHECK(hipMalloc(&hin[p], bytes));
            fill_k<<<1024, 256>>>(reinterpret_cast<unsigned*>(hin[p]), n, 100 + p);
        }
        float** din = nullptr;
        CHECK(hipMalloc(&din, P * sizeof(float*)));
        CHECK(hipMemcpy(din, hin.data(), P * sizeof(float*), hipMemcpyHostToDevice));
        std::vector<float**> dout(SETS);
        std::vector<BlockedScanPtrs> kargs(SETS);
        for (int s = 0; s < SETS; ++s) {
            std::vector<float*> h(P);
            for (int p = 0; p < P; ++p) CHECK(hipMalloc(&h[p], bytes));
            CHECK(hipMalloc(&dout[s], P * sizeof(float*)));
            CHECK(hipMemcpy(dout[s], h.data(), P * sizeof(float*), hipMemcpyHostToDevice));
            std::memset(&kargs[s], 0, sizeof(BlockedScanPtrs));
            for (int p = 0; p < std::min(P, 128); ++p) {
                kargs[s].in[p] = hin[p];
                kargs[s].out[p] = h[p];
            }
        }
        const unsigned grid = static_cast<unsigned>(nvec / 256);
        const double algo = 2.0 * P * bytes;
        auto pos = std::make_shared<int>(0);
#define V(MODE, NAME)                                                                                            \
        vs.push_back({"P=" + std::to_string(P) + " " NAME, [=](int) {                                          \
                          chain_scan<MODE><<<grid, 256, lds>>>(din, dout[(*pos)++ % SETS], P, nvec);             \
                      }, algo, {}});
        V(0, "global nt, device table") V(1, "global plain") V(2, "buffer sc1") V(3, "buffer nt sc1")
        V(4, "global nt, only every 16th output stored")
#undef V
        if (P <= 128)
            vs.push_back({"P=" + std::to_string(P) + " global nt, kernarg table (library form)", [=](int) {
                              chain_scan_kernarg<<<grid, 256, lds>>>(kargs[(*pos)++ % SETS], P, nvec);
                          }, algo, {}});
    }
    CHECK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int r = 0; r < rounds; ++r)
        for (auto& v : vs) {
            v.launch(0);
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
        std::printf("{\"variant\": \"%s\", \"median_us\": %.1f, \"frac\": %.4f}\n", v.name.c_str(), us,
                    v.bytes / (us * 1e-6) / 8e12);
    }
    return 0;
}
