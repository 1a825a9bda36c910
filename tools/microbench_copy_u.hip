// microbench_copy_u.hip — exploration harness (not part of the library): does the device copy kernel
// (copy_tile<U>, fmi_kernels.h: the reference's P = 1 allreduce and every staging copy of the communicator) run
// faster with fewer 16-B vectors per thread? The round-1 calibration saw a plain copy reach 0.815 of peak at
// U = 1 against 0.77 at U = 4 (profiles/archive/r01_hbm_calibration.jsonl); the library ships U = 4. This runs
// the library's own kernel template at U = 1, 2, 4, 8 on the same buffers: 256 MiB (16 rotating src/dst pairs,
// 8 GiB) and 64 MiB (64 pairs), interleaved over R rounds of K back-to-back launches (events), median per
// variant; every variant's output compared in full with the source.
//
// Build: hipcc -std=c++20 -O3 --offload-arch=gfx950 -ffp-contract=off tools/microbench_copy_u.hip -o build/mbcu
// Run:   build/mbcu [rounds, default 5]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "../fmi_amd/csrc/fmi_kernels.h"

using namespace fmi::dev;

#define CHECK(x)                                                                                   \
    do {                                                                                           \
        hipError_t e = (x);                                                                        \
        if (e != hipSuccess) {                                                                     \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            std::exit(1);                                                                          \
        }                                                                                          \
    } while (0)

__global__ void fill(unsigned* p, size_t n, unsigned seed) {
    for (size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += static_cast<size_t>(gridDim.x) * blockDim.x)
        p[i] = static_cast<unsigned>(i * 2654435761u) ^ seed;
}

__global__ void count_mismatch(const unsigned* a, const unsigned* b, size_t n, unsigned long long* bad) {
    unsigned long long k = 0;
    for (size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += static_cast<size_t>(gridDim.x) * blockDim.x)
        k += a[i] != b[i];
    if (k) atomicAdd(bad, k);
}

template <int U>
void launch(char* dst, const char* src, size_t bytes, hipStream_t s) {
    const size_t tiles = (bytes / 16 + U * 256 - 1) / (U * 256);
    copy_tile<U><<<static_cast<unsigned>(tiles), 256, 0, s>>>(dst, src, bytes);
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 5;
    constexpr int K = 32;
    CHECK(hipSetDevice(0));
    hipStream_t s = nullptr;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    unsigned long long* bad = nullptr;
    CHECK(hipMalloc(&bad, sizeof(*bad)));
    for (const size_t mib : {size_t(256), size_t(64)}) {
        const size_t bytes = mib << 20;
        const int sets = static_cast<int>(4096 / mib);  // 4 GiB of sources + 4 GiB of destinations
        std::vector<char*> src(sets), dst(sets);
        for (int k = 0; k < sets; ++k) {
            CHECK(hipMalloc(&src[k], bytes));
            CHECK(hipMalloc(&dst[k], bytes));
            fill<<<4096, 256, 0, s>>>(reinterpret_cast<unsigned*>(src[k]), bytes / 4, k);
        }
        CHECK(hipStreamSynchronize(s));
        struct V {
            std::string name;
            std::function<void(char*, const char*)> f;
            std::vector<double> us;
        };
        std::vector<V> vs = {
            {"copy_tile<1>", [&](char* d, const char* c) { launch<1>(d, c, bytes, s); }, {}},
            {"copy_tile<2>", [&](char* d, const char* c) { launch<2>(d, c, bytes, s); }, {}},
            {"copy_tile<4> (library)", [&](char* d, const char* c) { launch<4>(d, c, bytes, s); }, {}},
            {"copy_tile<8>", [&](char* d, const char* c) { launch<8>(d, c, bytes, s); }, {}},
        };
        for (auto& v : vs) {  // bits: the whole copy of set 0 equals its source
            CHECK(hipMemsetAsync(dst[0], 0xff, bytes, s));
            v.f(dst[0], src[0]);
            CHECK(hipMemsetAsync(bad, 0, sizeof(*bad), s));
            count_mismatch<<<4096, 256, 0, s>>>(reinterpret_cast<const unsigned*>(src[0]), reinterpret_cast<const unsigned*>(dst[0]), bytes / 4, bad);
            unsigned long long h = 0;
            CHECK(hipMemcpyAsync(&h, bad, sizeof(h), hipMemcpyDeviceToHost, s));
            CHECK(hipStreamSynchronize(s));
            std::printf("{\"mib\": %zu, \"kernel\": \"%s\", \"mismatches\": %llu}\n", mib, v.name.c_str(), h);
        }
        int next = 0;
        for (int r = 0; r < rounds; ++r)
            for (auto& v : vs) {
                for (int k = 0; k < 2; ++k, ++next) v.f(dst[next % sets], src[next % sets]);
                CHECK(hipEventRecord(e0, s));
                for (int k = 0; k < K; ++k, ++next) v.f(dst[next % sets], src[next % sets]);
                CHECK(hipEventRecord(e1, s));
                CHECK(hipEventSynchronize(e1));
                float ms = 0;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                v.us.push_back(ms * 1e3 / K);
            }
        for (auto& v : vs) {
            std::sort(v.us.begin(), v.us.end());
            const double us = v.us[v.us.size() / 2];
            std::printf("{\"mib\": %zu, \"kernel\": \"%s\", \"median_us\": %.2f, \"min_us\": %.2f, \"frac\": %.4f, \"sets\": %d}\n",
                        mib, v.name.c_str(), us, v.us.front(), 2.0 * bytes / (us * 1e-6) / 8e12, sets);
        }
        std::fflush(stdout);
        for (int k = 0; k < sets; ++k) {
            CHECK(hipFree(src[k]));
            CHECK(hipFree(dst[k]));
        }
    }
    return 0;
}
