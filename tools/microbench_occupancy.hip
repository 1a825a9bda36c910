// microbench_occupancy.hip — exploration harness (not part of the library): does capping the number of
// workgroups resident per CU (and so the number of HBM requests in flight chip-wide) change the rate of
// the production streaming kernels? The cap is set with dynamic LDS: 160 KiB of LDS per CU on gfx950, so
// a launch that asks for 160 KiB / k bytes fits at most k workgroups per CU. Also tried: an XCD-contiguous
// tile order for the pairwise kernel (blocks b and b+8 share an XCD, MI355X_MICROARCH.md §Workgroup
// dispatch), which gives each XCD one contiguous eighth of the bucket instead of every eighth tile.
//
//   pair   production pair_tile<sum, f32, U=4, nt/nt>, 256 threads, 256 MiB buckets (C2)
//   tree8  production tree_kernel, allreduce_no_order, P = 8 × 64 MiB (C3 shape)
//   scan8  production scan_kernel, scan_no_order,      P = 8 × 64 MiB (C3)
//
// Build: hipcc -std=c++20 -O3 --offload-arch=gfx950 -ffp-contract=off tools/microbench_occupancy.hip -o build/mbo
// Run:   build/mbo   (one JSON line per variant; two interleaved rounds)
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

// pair_tile with an XCD-contiguous tile order: the G tiles are dealt so that the blocks one XCD runs
// (b ≡ x mod 8) cover tiles [x·G/8, (x+1)·G/8) in order. Requires G % 8 == 0.
template <int U>
__global__ void __launch_bounds__(256) pair_xcd(float* out, const float* a, const float* b, size_t n) {
    const size_t nvec = n / 4;
    const size_t G = gridDim.x;
    const size_t tile = (blockIdx.x % 8) * (G / 8) + blockIdx.x / 8;
    pair_tile_body<OpSum, float, U, 3>(out, a, b, nvec, tile);
}

template <class F>
double median_us(F&& launch, int iters) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int k = 0; k < 3; ++k) launch(k);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    std::vector<double> t;
    for (int r = 0; r < iters; ++r) {
        CHECK(hipEventRecord(e0));
        for (int k = 0; k < 4; ++k) launch(k);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        t.push_back(ms * 1e3 / 4);
    }
    CHECK(hipGetLastError());
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

void report(const std::string& name, int cap, double bytes, double us) {
    const double gbs = bytes / (us * 1e-6) / 1e9;
    std::printf("{\"variant\": \"%s\", \"wg_per_cu_cap\": %d, \"us\": %.2f, \"GB_s\": %.1f, \"frac\": %.4f}\n",
                name.c_str(), cap, us, gbs, gbs / 8000.);
    std::fflush(stdout);
}

int main() {
    constexpr int SETS = 4;
    // C2: 256 MiB f32 pair
    const size_t n2 = (256u << 20) / 4;
    float* a[SETS];
    float* b[SETS];
    for (int s = 0; s < SETS; ++s) {
        CHECK(hipMalloc(&a[s], n2 * 4));
        CHECK(hipMalloc(&b[s], n2 * 4));
        CHECK(hipMemset(a[s], 0, n2 * 4));
        CHECK(hipMemset(b[s], 0, n2 * 4));
    }
    const unsigned grid2 = static_cast<unsigned>(n2 / 4 / (4 * 256));  // 16,384 tiles
    // C3: 8 × 64 MiB f32 inputs (+ 8 outputs for the scan); 2 sets of 16 buckets = 2 GiB
    const size_t n3 = (64u << 20) / 4;
    PeerPtrs ptrs[2];
    for (int s = 0; s < 2; ++s)
        for (int j = 0; j < P; ++j) {
            void* p;
            CHECK(hipMalloc(&p, n3 * 4));
            CHECK(hipMemset(p, 0, n3 * 4));
            ptrs[s].in[j] = p;
            CHECK(hipMalloc(&p, n3 * 4));
            CHECK(hipMemset(p, 0, n3 * 4));
            ptrs[s].out[j] = p;
        }
    const unsigned grid3 = static_cast<unsigned>(n3 / 4 / 256);
    constexpr int A = fmi::sched::kAllreduce;
    constexpr int S = fmi::sched::kScan;
    const double pair_bytes = 3.0 * n2 * 4, tree_bytes = (P + 1.0) * n3 * 4, scan_bytes = 2.0 * P * n3 * 4;

    // caps: 0 = no dynamic LDS (occupancy set by registers alone)
    const bool wide = std::getenv("MBO_WIDE") != nullptr;
    std::vector<int> caps = wide ? std::vector<int>{0, 16, 12, 8, 6, 4, 3, 2} : std::vector<int>{0, 3, 2, 1};
    auto lds_for = [](int cap) -> size_t { return cap ? (160u * 1024u / cap) & ~size_t(255) : 0; };
    int max_lds = 0;
    CHECK(hipDeviceGetAttribute(&max_lds, hipDeviceAttributeMaxSharedMemoryPerBlock, 0));
    std::printf("{\"max_lds_per_workgroup\": %d}\n", max_lds);
    caps.erase(std::remove_if(caps.begin(), caps.end(), [&](int c) { return lds_for(c) > size_t(max_lds); }),
               caps.end());
    // C3 i64 max pair: 64 MiB buckets, 8 rotating sets (1.5 GiB) as in tools/bench_configs.py
    const size_t n64 = (64u << 20) / 8;
    int64_t* qa[8];
    int64_t* qb[8];
    for (int s = 0; s < 8; ++s) {
        CHECK(hipMalloc(&qa[s], n64 * 8));
        CHECK(hipMalloc(&qb[s], n64 * 8));
        CHECK(hipMemset(qa[s], 0, n64 * 8));
        CHECK(hipMemset(qb[s], 0, n64 * 8));
    }
    const unsigned grid64 = static_cast<unsigned>(n64 / 2 / (4 * 256));
    const double q_bytes = 3.0 * n64 * 8;
    for (int round = 0; round < 2; ++round) {
        for (int cap : caps) {
            const size_t lds = lds_for(cap);
            report("pair U4 B256 nt", cap, pair_bytes, median_us([&](int k) {
                       pair_tile<OpSum, float, 4, 3><<<grid2, 256, lds>>>(a[k % SETS], a[k % SETS], b[k % SETS], n2);
                   }, 15));
            if (wide)
                report("pair xcd-contiguous U4 B256 nt", cap, pair_bytes, median_us([&](int k) {
                           pair_xcd<4><<<grid2, 256, lds>>>(a[k % SETS], a[k % SETS], b[k % SETS], n2);
                       }, 15));
            report("pair i64 max 64MiB U4 B256 nt", cap, q_bytes, median_us([&](int k) {
                       pair_tile<OpMax, int64_t, 4, 3><<<grid64, 256, lds>>>(qa[k % 8], qa[k % 8], qb[k % 8], n64);
                   }, 15));
            report("tree8 allreduce B256 nt", cap, tree_bytes, median_us([&](int k) {
                       tree_kernel<OpSum, float, A, P, false><<<grid3, 256, lds>>>(ptrs[k % 2], n3, 0, 0);
                   }, 15));
            report("scan8 B256 nt", cap, scan_bytes, median_us([&](int k) {
                       scan_kernel<OpSum, float, S, P><<<grid3, 256, lds>>>(ptrs[k % 2], n3, 0);
                   }, 15));
            // persistent grid-stride form: cap workgroups per CU × 256 CUs, each thread walks the bucket
            if (cap) {
                report("scan8 B256 nt grid-stride", cap, scan_bytes, median_us([&](int k) {
                           scan_kernel<OpSum, float, S, P><<<256 * cap, 256, lds>>>(ptrs[k % 2], n3, 0);
                       }, 15));
                report("tree8 B256 nt grid-stride", cap, tree_bytes, median_us([&](int k) {
                           tree_kernel<OpSum, float, A, P, false><<<256 * cap, 256, lds>>>(ptrs[k % 2], n3, 0, 0);
                       }, 15));
            }
        }
    }
    return 0;
}
