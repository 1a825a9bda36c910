// microbench_pipeline.hip — exploration harness (not part of the library): does a persistent, software-
// pipelined pairwise kernel (grid = resident capacity; each thread issues tile k+1's loads before tile k's
// stores) beat the production one-shot tiles (pair_tile: one tile per workgroup, all loads, then all
// stores) at config C3's size, where the one-shot kernel sits at 0.69-0.73 of peak and a MALL-resident
// run is no faster (VERDICT r01 "What's weak" 2)? Also at C2's size, so a win there is not a loss here.
//
// Every variant runs in one process, interleaved over rounds, on rotating buffer sets (C3: 8 x 192 MiB,
// C2: 4 x 768 MiB), timed by two HIP events around K back-to-back launches (as bench.py), and is checked
// bit for bit against the production kernel's output.
//
// Build: hipcc -std=c++20 -O3 --offload-arch=gfx950 -ffp-contract=off tools/microbench_pipeline.hip -o build/mbp
// Run:   build/mbp [rounds] [c3|c2]   (one JSON line per (config, variant, round))
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

// Persistent grid-stride over tiles of U lane groups per thread (the production tile shape), double-
// buffered in registers: tile t + grid's loads are in flight while tile t is combined and stored.
// nvec must be a multiple of U * blockDim.x (checked on the host).
template <class Op, class T, int U>
__device__ __forceinline__ void load_tile(Lanes<T, kVecLanes<T>>* va, Lanes<T, kVecLanes<T>>* vb, const T* a,
                                          const T* b, size_t tile) {
    constexpr int W = kVecLanes<T>;
    const size_t B = blockDim.x;
    const size_t base = tile * U * B + threadIdx.x;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        va[u] = load_lanes<true, T, W>(a + (base + u * B) * W);
        vb[u] = load_lanes<true, T, W>(b + (base + u * B) * W);
    }
}

template <class Op, class T, int U>
__device__ __forceinline__ void store_tile(T* out, const Lanes<T, kVecLanes<T>>* va, const Lanes<T, kVecLanes<T>>* vb,
                                           size_t tile) {
    constexpr int W = kVecLanes<T>;
    const size_t B = blockDim.x;
    const size_t base = tile * U * B + threadIdx.x;
#pragma unroll
    for (int u = 0; u < U; ++u) store_lanes<true, T, W>(out + (base + u * B) * W, combine<Op, T, W>(va[u], vb[u]));
}

template <class Op, class T, int U>
__global__ void __launch_bounds__(1024) pair_pipe(T* out, const T* a, const T* b, size_t ntiles) {
    using L = Lanes<T, kVecLanes<T>>;
    L a0[U], b0[U], a1[U], b1[U];
    size_t t = blockIdx.x;
    if (t >= ntiles) return;
    load_tile<Op, T, U>(a0, b0, a, b, t);
    for (;;) {
        const size_t t1 = t + gridDim.x;
        if (t1 < ntiles) load_tile<Op, T, U>(a1, b1, a, b, t1);
        store_tile<Op, T, U>(out, a0, b0, t);
        if (t1 >= ntiles) break;
        const size_t t2 = t1 + gridDim.x;
        if (t2 < ntiles) load_tile<Op, T, U>(a0, b0, a, b, t2);
        store_tile<Op, T, U>(out, a1, b1, t1);
        if (t2 >= ntiles) break;
        t = t2;
    }
}

// Each workgroup owns one contiguous run of tiles (blockIdx.x * per .. + per) and walks it pipelined.
template <class Op, class T, int U>
__global__ void __launch_bounds__(1024) pair_pipe_chunk(T* out, const T* a, const T* b, size_t ntiles) {
    using L = Lanes<T, kVecLanes<T>>;
    L a0[U], b0[U], a1[U], b1[U];
    const size_t per = (ntiles + gridDim.x - 1) / gridDim.x;
    size_t t = blockIdx.x * per;
    const size_t end = std::min(ntiles, t + per);
    if (t >= end) return;
    load_tile<Op, T, U>(a0, b0, a, b, t);
    for (;;) {
        const size_t t1 = t + 1;
        if (t1 < end) load_tile<Op, T, U>(a1, b1, a, b, t1);
        store_tile<Op, T, U>(out, a0, b0, t);
        if (t1 >= end) break;
        const size_t t2 = t1 + 1;
        if (t2 < end) load_tile<Op, T, U>(a0, b0, a, b, t2);
        store_tile<Op, T, U>(out, a1, b1, t1);
        if (t2 >= end) break;
        t = t2;
    }
}

struct Variant {
    std::string name;
    std::function<void(void*, const void*, const void*, size_t, hipStream_t)> launch;
};

template <class Op, class T>
std::vector<Variant> variants(int cus) {
    std::vector<Variant> v;
    auto tile = [&]<int U, int B>() {
        v.push_back({"tile U" + std::to_string(U) + " B" + std::to_string(B),
                     [](void* o, const void* a, const void* b, size_t n, hipStream_t s) {
                         const size_t nvec = n / kVecLanes<T>;
                         const unsigned grid = static_cast<unsigned>((nvec + U * B - 1) / (U * B));
                         pair_tile<Op, T, U, 3><<<grid, B, 0, s>>>(static_cast<T*>(o), static_cast<const T*>(a),
                                                                 static_cast<const T*>(b), n);
                     }});
    };
    tile.template operator()<4, 256>();  // production
    tile.template operator()<8, 256>();
    tile.template operator()<2, 256>();
    tile.template operator()<1, 256>();
    tile.template operator()<2, 512>();
    tile.template operator()<1, 1024>();
    auto pipe = [&]<int U, int B, bool CHUNK>(int per_cu) {
        v.push_back({std::string(CHUNK ? "pipe-chunk" : "pipe") + " U" + std::to_string(U) + " B" +
                         std::to_string(B) + " grid " + std::to_string(per_cu) + "/CU",
                     [per_cu, cus](void* o, const void* a, const void* b, size_t n, hipStream_t s) {
                         const size_t nvec = n / kVecLanes<T>;
                         const size_t ntiles = nvec / (U * B);
                         const unsigned grid = static_cast<unsigned>(std::min<size_t>(ntiles, size_t(per_cu) * cus));
                         if constexpr (CHUNK)
                             pair_pipe_chunk<Op, T, U><<<grid, B, 0, s>>>(static_cast<T*>(o), static_cast<const T*>(a),
                                                                          static_cast<const T*>(b), ntiles);
                         else
                             pair_pipe<Op, T, U><<<grid, B, 0, s>>>(static_cast<T*>(o), static_cast<const T*>(a),
                                                                    static_cast<const T*>(b), ntiles);
                     }});
    };
    for (int k : {2, 4, 8}) {
        pipe.template operator()<1, 256, false>(k);
        pipe.template operator()<2, 256, false>(k);
        pipe.template operator()<4, 256, false>(k);
    }
    for (int k : {4, 8}) pipe.template operator()<2, 256, true>(k);
    pipe.template operator()<1, 1024, false>(2);
    pipe.template operator()<2, 512, false>(4);
    return v;
}

template <class Op, class T>
void run_config(const char* cfg, size_t mib, int nsets, int K, int rounds, int cus) {
    const size_t n = mib * (size_t(1) << 20) / sizeof(T);
    const size_t bytes = n * sizeof(T);
    std::vector<T*> A(nsets), Bv(nsets);
    std::vector<T> host(n);
    for (int s = 0; s < nsets; ++s) {
        CHECK(hipMalloc(&A[s], bytes));
        CHECK(hipMalloc(&Bv[s], bytes));
        for (int side = 0; side < 2; ++side) {
            uint64_t key = 1234 + 2 * s + side;
            for (size_t i = 0; i < n; ++i) host[i] = synth_value<T>(splitmix64(key ^ i));
            CHECK(hipMemcpy(side ? Bv[s] : A[s], host.data(), bytes, hipMemcpyHostToDevice));
        }
    }
    T* ref = nullptr;
    T* got = nullptr;
    CHECK(hipMalloc(&ref, bytes));
    CHECK(hipMalloc(&got, bytes));
    auto vs = variants<Op, T>(cus);
    // correctness: out-of-place against the production kernel
    vs[0].launch(ref, A[0], Bv[0], n, nullptr);
    std::vector<T> h_ref(n), h_got(n);
    CHECK(hipMemcpy(h_ref.data(), ref, bytes, hipMemcpyDeviceToHost));
    std::vector<int> ok(vs.size());
    for (size_t k = 0; k < vs.size(); ++k) {
        CHECK(hipMemset(got, 0, bytes));
        vs[k].launch(got, A[0], Bv[0], n, nullptr);
        CHECK(hipGetLastError());
        CHECK(hipMemcpy(h_got.data(), got, bytes, hipMemcpyDeviceToHost));
        ok[k] = std::memcmp(h_ref.data(), h_got.data(), bytes) == 0;
    }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const double algo = 3.0 * bytes;
    for (int r = 0; r < rounds; ++r) {
        for (size_t k = 0; k < vs.size(); ++k) {
            for (int w = 0; w < 3; ++w) vs[k].launch(A[w % nsets], A[w % nsets], Bv[w % nsets], n, nullptr);
            CHECK(hipEventRecord(e0, nullptr));
            for (int i = 0; i < K; ++i) vs[k].launch(A[i % nsets], A[i % nsets], Bv[i % nsets], n, nullptr);
            CHECK(hipEventRecord(e1, nullptr));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            const double us = 1e3 * ms / K;
            std::printf("{\"config\": \"%s\", \"variant\": \"%s\", \"round\": %d, \"us\": %.2f, \"frac\": %.4f, "
                        "\"bit_exact\": %s}\n",
                        cfg, vs[k].name.c_str(), r, us, algo / (us * 1e-6) / 8e12, ok[k] ? "true" : "false");
            std::fflush(stdout);
        }
    }
    for (int s = 0; s < nsets; ++s) {
        CHECK(hipFree(A[s]));
        CHECK(hipFree(Bv[s]));
    }
    CHECK(hipFree(ref));
    CHECK(hipFree(got));
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 3;
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const std::string only = argc > 2 ? argv[2] : "";  // "c3" or "c2": one config (e.g. under rocprofv3)
    if (only != "c2") run_config<OpMax, int64_t>("C3 i64 max 64MiB", 64, 8, 60, rounds, cus);
    if (only != "c3") run_config<OpSum, float>("C2 f32 sum 256MiB", 256, 4, 30, rounds, cus);
    return 0;
}
