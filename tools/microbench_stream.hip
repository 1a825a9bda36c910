// microbench_stream.hip — exploration harness (not part of the library): HBM rate of the write-heavy
// shapes on gfx950 under different cache policies, tile sizes and block sizes, to choose the production
// variants of scan_kernel (P reads + P writes) and tree_kernel (P reads + 1 write).
//
//   copy      out = in                     1 read : 1 write (calibration, MI355X_MICROARCH.md: 6.29 TB/s)
//   scan8     8 outputs = peer-axis prefix of 8 inputs (allreduce_no_order-style scan program, f32 sum)
//   tree8     1 output  = fused allreduce of 8 inputs
//
// Build: hipcc -std=c++20 -O3 --offload-arch=gfx950 -ffp-contract=off tools/microbench_stream.hip -o build/mb
// Run:   build/mb [MiB per bucket, default 64] [skew bytes between consecutive buckets, default 0]
//        [quick: 1 = production variants only]
// All buckets are carved from one arena, bucket k at k * (size + skew): skew tests whether buckets whose
// base addresses are congruent modulo the HBM channel/bank interleave collide (partition camping).
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
using L = Lanes<float, 4>;

template <int NTL, int NTS, int U>
__global__ void __launch_bounds__(1024) copy_k(float* out, const float* in, size_t nvec) {
    const size_t B = blockDim.x;
    const size_t base = static_cast<size_t>(blockIdx.x) * U * B + threadIdx.x;
    L v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (base + u * B < nvec) v[u] = load_lanes<NTL != 0, float, 4>(in + (base + u * B) * 4);
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (base + u * B < nvec) store_lanes<NTS != 0, float, 4>(out + (base + u * B) * 4, v[u]);
}

template <int ALG, int NTL, size_t... I>
__device__ __forceinline__ void ld(L* v, const PeerPtrs& p, size_t e, std::index_sequence<I...>) {
    ((v[I] = load_lanes<NTL != 0, float, 4>(static_cast<const float*>(p.in[I]) + e)), ...);
}
template <int ALG, int NTS, size_t... R>
__device__ __forceinline__ void st(const L* v, const PeerPtrs& p, size_t e, std::index_sequence<R...>) {
    ((store_lanes<NTS != 0, float, 4>(static_cast<float*>(p.out[R]) + e, v[kOut<ALG, P, R>])), ...);
}

// U lane groups per thread, stride B (each wave-instruction stays one contiguous 1-KiB access).
template <int ALG, bool ALL_OUT, int NTL, int NTS, int U>
__global__ void __launch_bounds__(1024) fused_k(PeerPtrs ptrs, size_t nvec) {
    const size_t B = blockDim.x;
    const size_t base = static_cast<size_t>(blockIdx.x) * U * B + threadIdx.x;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t g = base + u * B;
        if (g >= nvec) break;
        L v[P + kNumSteps<ALG, P>];
        ld<ALG, NTL>(v, ptrs, g * 4, std::make_index_sequence<P>{});
        run_steps<OpSum, float, 4, ALG, P>(v, std::make_index_sequence<kNumSteps<ALG, P>>{});
        if constexpr (ALL_OUT)
            st<ALG, NTS>(v, ptrs, g * 4, std::make_index_sequence<P>{});
        else
            store_lanes<NTS != 0, float, 4>(static_cast<float*>(ptrs.out[0]) + g * 4, v[kOut<ALG, P, 0>]);
    }
}

// Same, but U groups loaded first for all peers, then computed and stored (more loads in flight).
template <int ALG, bool ALL_OUT, int NTL, int NTS>
__global__ void __launch_bounds__(1024) fused2_k(PeerPtrs ptrs, size_t nvec) {
    const size_t B = blockDim.x;
    const size_t base = static_cast<size_t>(blockIdx.x) * 2 * B + threadIdx.x;
    if (base + B >= nvec) return;  // exploration only: sizes are multiples of the tile
    L v0[P + kNumSteps<ALG, P>], v1[P + kNumSteps<ALG, P>];
    ld<ALG, NTL>(v0, ptrs, base * 4, std::make_index_sequence<P>{});
    ld<ALG, NTL>(v1, ptrs, (base + B) * 4, std::make_index_sequence<P>{});
    run_steps<OpSum, float, 4, ALG, P>(v0, std::make_index_sequence<kNumSteps<ALG, P>>{});
    run_steps<OpSum, float, 4, ALG, P>(v1, std::make_index_sequence<kNumSteps<ALG, P>>{});
    if constexpr (ALL_OUT) {
        st<ALG, NTS>(v0, ptrs, base * 4, std::make_index_sequence<P>{});
        st<ALG, NTS>(v1, ptrs, (base + B) * 4, std::make_index_sequence<P>{});
    } else {
        store_lanes<NTS != 0, float, 4>(static_cast<float*>(ptrs.out[0]) + base * 4, v0[kOut<ALG, P, 0>]);
        store_lanes<NTS != 0, float, 4>(static_cast<float*>(ptrs.out[0]) + (base + B) * 4, v1[kOut<ALG, P, 0>]);
    }
}

struct Timer {
    hipEvent_t a, b;
    Timer() {
        CHECK(hipEventCreate(&a));
        CHECK(hipEventCreate(&b));
    }
};

template <class F>
double median_us(F&& launch, int iters) {
    std::vector<double> t;
    Timer tm;
    for (int k = 0; k < 3; ++k) launch(k);
    CHECK(hipDeviceSynchronize());
    for (int k = 0; k < iters; ++k) {
        CHECK(hipEventRecord(tm.a));
        launch(k);
        CHECK(hipEventRecord(tm.b));
        CHECK(hipEventSynchronize(tm.b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, tm.a, tm.b));
        t.push_back(ms * 1e3);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

void report(const std::string& name, double bytes, double us) {
    const double gbs = bytes / (us * 1e-6) / 1e9;
    std::printf("{\"variant\": \"%s\", \"us\": %.2f, \"GB_s\": %.1f, \"frac\": %.4f}\n", name.c_str(), us, gbs,
                gbs / 8000.);
    std::fflush(stdout);
}

int main(int argc, char** argv) {
    const size_t mib = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 64;
    const size_t n = mib * (1 << 20) / 4;
    const size_t nvec = n / 4;
    const size_t skew = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 0;
    const bool quick = argc > 3 && argv[3][0] == '1';
    std::printf("{\"bucket_mib\": %zu, \"skew_bytes\": %zu}\n", mib, skew);
    const int iters = 20;
    constexpr int SETS = 2;
    const size_t stride = n * 4 + skew;
    char* arena;
    CHECK(hipMalloc(&arena, stride * (2 * P * SETS + 1)));
    CHECK(hipMemset(arena, 0, stride * (2 * P * SETS + 1)));
    PeerPtrs ptrs[SETS];
    size_t k = 0;
    for (int s = 0; s < SETS; ++s)
        for (int j = 0; j < P; ++j) {
            ptrs[s].in[j] = arena + stride * k++;
            ptrs[s].out[j] = arena + stride * k++;
        }
    // copy calibration: P*n floats in, P*n floats out (the scan's byte count), as 8 launches' worth in one
    float* cin = reinterpret_cast<float*>(arena);
    float* cout = reinterpret_cast<float*>(arena + ((P * n * 4 + skew + 4095) / 4096) * 4096 + skew);
    const double copy_bytes = 2.0 * P * n * 4;
#define COPY(NTL, NTS, U, B)                                                                              \
    report("copy ntl" #NTL " nts" #NTS " U" #U " B" #B, copy_bytes, median_us([&](int) {                 \
               copy_k<NTL, NTS, U><<<grid_for(P * nvec, U * B), B>>>(cout, cin, P * nvec);                \
           }, iters));
    COPY(1, 1, 1, 256)
    if (!quick) {
    COPY(0, 0, 1, 256)
    COPY(1, 0, 1, 256)
    COPY(0, 1, 1, 256)
    COPY(1, 1, 4, 256)
    COPY(0, 0, 4, 256)
    COPY(1, 1, 2, 512)
    CHECK(hipMemcpy(cout, cin, 16, hipMemcpyDeviceToDevice));
    report("hipMemcpyAsync d2d", copy_bytes, median_us([&](int) {
               CHECK(hipMemcpyAsync(cout, cin, P * n * 4, hipMemcpyDeviceToDevice, nullptr));
           }, iters));
    }

    constexpr int S = fmi::sched::kScan;
    constexpr int A = fmi::sched::kAllreduce;
    const double scan_bytes = 2.0 * P * n * 4;
    const double tree_bytes = (P + 1.0) * n * 4;
#define FUSED(ALG, ALL, NTL, NTS, U, B, NAME, BYTES)                                                      \
    report(std::string(NAME) + " ntl" #NTL " nts" #NTS " U" #U " B" #B, BYTES, median_us([&](int k) {    \
               fused_k<ALG, ALL, NTL, NTS, U><<<grid_for(nvec, U * B), B>>>(ptrs[k % SETS], nvec);       \
           }, iters));
#define FUSED2(ALG, ALL, NTL, NTS, B, NAME, BYTES)                                                        \
    report(std::string(NAME) + " 2-stage ntl" #NTL " nts" #NTS " B" #B, BYTES, median_us([&](int k) {    \
               fused2_k<ALG, ALL, NTL, NTS><<<grid_for(nvec, 2 * B), B>>>(ptrs[k % SETS], nvec);         \
           }, iters));
    FUSED(S, true, 1, 1, 1, 256, "scan8", scan_bytes)  // = production scan_kernel
    FUSED(A, false, 1, 1, 1, 256, "tree8", tree_bytes)  // = production tree_kernel
    if (quick) return 0;
    FUSED(S, true, 0, 0, 1, 256, "scan8", scan_bytes)
    FUSED(S, true, 1, 0, 1, 256, "scan8", scan_bytes)
    FUSED(S, true, 0, 1, 1, 256, "scan8", scan_bytes)
    FUSED(S, true, 1, 1, 2, 256, "scan8", scan_bytes)
    FUSED(S, true, 1, 1, 1, 512, "scan8", scan_bytes)
    FUSED(S, true, 1, 1, 1, 128, "scan8", scan_bytes)
    FUSED(S, true, 1, 1, 1, 64, "scan8", scan_bytes)
    FUSED2(S, true, 1, 1, 256, "scan8", scan_bytes)
    FUSED2(S, true, 1, 0, 256, "scan8", scan_bytes)
    FUSED(A, false, 0, 0, 1, 256, "tree8", tree_bytes)
    FUSED(A, false, 1, 0, 1, 256, "tree8", tree_bytes)
    FUSED(A, false, 1, 1, 2, 256, "tree8", tree_bytes)
    FUSED(A, false, 1, 1, 1, 512, "tree8", tree_bytes)
    FUSED(A, false, 1, 1, 1, 128, "tree8", tree_bytes)
    FUSED2(A, false, 1, 1, 256, "tree8", tree_bytes)
    return 0;
}
