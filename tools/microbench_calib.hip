// microbench_calib.hip — exploration harness (not part of the library): what HBM rate does this chip
// reach for pure streaming reads, pure streaming writes, a 1:1 copy and the C2 pairwise combine (2 reads :
// 1 write, in place and out of place), all with the production access shape (16 B per lane, 4 lane groups
// per thread, 256-thread workgroups, nontemporal loads and stores) over buffers well beyond the 256 MiB
// Infinity Cache? It calibrates the "achievable" end of the C2 roofline.
//
// Build: hipcc -std=c++20 -O3 --offload-arch=gfx950 -ffp-contract=off tools/microbench_calib.hip -o build/mbc
// Run:   build/mbc   (one JSON line per variant; three interleaved rounds)
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

using L = Lanes<float, 4>;
constexpr int U = 4;
constexpr int B = 256;

// Pure read: every lane group is loaded once and folded into a register; one float per thread is written
// only if the fold hits an impossible value (keeps the loads live without adding write traffic).
__global__ void __launch_bounds__(B) read_only(const float* in, size_t nvec, float* sink) {
    const size_t base = static_cast<size_t>(blockIdx.x) * U * B + threadIdx.x;
    L v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = load_lanes<true, float, 4>(in + (base + u * B) * 4);
    float acc = 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u].v[0] + v[u].v[1] + v[u].v[2] + v[u].v[3];
    if (acc == 12345.678f) sink[threadIdx.x] = acc;
}

__global__ void __launch_bounds__(B) write_only(float* out, size_t nvec, float x) {
    const size_t base = static_cast<size_t>(blockIdx.x) * U * B + threadIdx.x;
    L v;
    v.v[0] = v.v[1] = v.v[2] = v.v[3] = x;
#pragma unroll
    for (int u = 0; u < U; ++u) store_lanes<true, float, 4>(out + (base + u * B) * 4, v);
}

__global__ void __launch_bounds__(B) copy_k(float* out, const float* in, size_t nvec) {
    const size_t base = static_cast<size_t>(blockIdx.x) * U * B + threadIdx.x;
    L v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = load_lanes<true, float, 4>(in + (base + u * B) * 4);
#pragma unroll
    for (int u = 0; u < U; ++u) store_lanes<true, float, 4>(out + (base + u * B) * 4, v[u]);
}

// Write-only variants: U stores per thread (stride B lane groups), cache policy through the buffer
// instruction's aux bits (gfx950: bit 0 sc0, bit 1 nt, bit 4 sc1).
template <int UW, int AUX>
__global__ void __launch_bounds__(1024) write_buf(float* out, unsigned nbytes, float x) {
    const auto r = __builtin_amdgcn_make_buffer_rsrc(out, 0, static_cast<int>(nbytes), 0x00020000);
    const unsigned base = (blockIdx.x * UW * blockDim.x + threadIdx.x) * 16u;
    u32x4 v = {__float_as_uint(x), __float_as_uint(x), __float_as_uint(x), __float_as_uint(x)};
#pragma unroll
    for (int u = 0; u < UW; ++u) __builtin_amdgcn_raw_buffer_store_b128(v, r, base + u * blockDim.x * 16u, 0, AUX);
}

// Wave-contiguous tiles: wave w of a workgroup owns U consecutive 1-KiB wave-rows (4·U KiB per operand in
// one run), instead of the production layout where the U rows of a wave are B/64 rows apart.
template <int UW, int MODE>  // MODE 0 = pair a=a+b, 1 = copy, 2 = write-only
__global__ void __launch_bounds__(256) wave_contig(float* out, const float* a, const float* b) {
    const size_t wave = threadIdx.x / 64, lane = threadIdx.x % 64;
    const size_t base = static_cast<size_t>(blockIdx.x) * UW * 256 + wave * UW * 64 + lane;
    L va[UW], vb[UW];
    if constexpr (MODE != 2) {
#pragma unroll
        for (int u = 0; u < UW; ++u) {
            va[u] = load_lanes<true, float, 4>(a + (base + u * 64) * 4);
            if constexpr (MODE == 0) vb[u] = load_lanes<true, float, 4>(b + (base + u * 64) * 4);
        }
    } else {
#pragma unroll
        for (int u = 0; u < UW; ++u) va[u].v[0] = va[u].v[1] = va[u].v[2] = va[u].v[3] = 1.f;
    }
#pragma unroll
    for (int u = 0; u < UW; ++u)
        store_lanes<true, float, 4>(out + (base + u * 64) * 4, MODE == 0 ? combine<OpSum, float, 4>(va[u], vb[u]) : va[u]);
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

void report(const std::string& name, double bytes, double us) {
    const double gbs = bytes / (us * 1e-6) / 1e9;
    std::printf("{\"variant\": \"%s\", \"bytes\": %.0f, \"us\": %.2f, \"GB_s\": %.1f, \"frac\": %.4f}\n", name.c_str(),
                bytes, us, gbs, gbs / 8000.);
    std::fflush(stdout);
}

int main() {
    constexpr int SETS = 4;
    const size_t n = (256u << 20) / 4;  // 256 MiB buckets (C2)
    const size_t nvec = n / 4;
    const unsigned grid = static_cast<unsigned>(nvec / (U * B));  // exact: 16,384 tiles
    float* a[SETS];
    float* b[SETS];
    float* c[SETS];
    for (int s = 0; s < SETS; ++s) {
        CHECK(hipMalloc(&a[s], n * 4));
        CHECK(hipMalloc(&b[s], n * 4));
        CHECK(hipMalloc(&c[s], n * 4));
        CHECK(hipMemset(a[s], 0, n * 4));
        CHECK(hipMemset(b[s], 0, n * 4));
        CHECK(hipMemset(c[s], 0, n * 4));
    }
    float* sink;
    CHECK(hipMalloc(&sink, B * sizeof(float)));
    const double S = n * 4.0;
    for (int round = 0; round < 3; ++round) {
        // 512 MiB per launch (two 256 MiB buckets back to back in one launch would need contiguity:
        // instead two launches' worth are timed as one 'pair' of launches below for read/write)
        report("read-only 256MiB", S, median_us([&](int k) { read_only<<<grid, B>>>(a[k % SETS], nvec, sink); }, 15));
        report("write-only 256MiB", S, median_us([&](int k) { write_only<<<grid, B>>>(c[k % SETS], nvec, 1.f); }, 15));
#define WB(UW, AUX, BLK)                                                                                  \
        report("write-only buffer U" #UW " aux" #AUX " B" #BLK, S, median_us([&](int k) {                      \
                   write_buf<UW, AUX><<<static_cast<unsigned>(nvec / (UW * BLK)), BLK>>>(c[k % SETS],        \
                                                                                        unsigned(S), 1.f); \
               }, 15));
        WB(4, 2, 256)
        WB(4, 0, 256)
        WB(4, 16, 256)
        WB(4, 18, 256)
        WB(1, 2, 256)
        WB(2, 2, 256)
        WB(8, 2, 256)
        WB(1, 2, 1024)
        WB(4, 2, 1024)
        WB(1, 0, 1024)
        report("copy 256MiB (1R:1W)", 2 * S,
               median_us([&](int k) { copy_k<<<grid, B>>>(c[k % SETS], a[k % SETS], nvec); }, 15));
        report("pair in place a=a+b (2R:1W, production C2)", 3 * S, median_us([&](int k) {
                   pair_tile<OpSum, float, 4, 3><<<grid, B>>>(a[k % SETS], a[k % SETS], b[k % SETS], n);
               }, 15));
        report("pair in place wave-contiguous U4", 3 * S, median_us([&](int k) {
                   wave_contig<4, 0><<<grid, B>>>(a[k % SETS], a[k % SETS], b[k % SETS]);
               }, 15));
        report("pair in place wave-contiguous U2", 3 * S, median_us([&](int k) {
                   wave_contig<2, 0><<<grid * 2, B>>>(a[k % SETS], a[k % SETS], b[k % SETS]);
               }, 15));
        report("pair in place production-layout U1", 3 * S, median_us([&](int k) {
                   pair_tile<OpSum, float, 1, 3><<<grid * 4, B>>>(a[k % SETS], a[k % SETS], b[k % SETS], n);
               }, 15));
        report("pair in place production-layout U2", 3 * S, median_us([&](int k) {
                   pair_tile<OpSum, float, 2, 3><<<grid * 2, B>>>(a[k % SETS], a[k % SETS], b[k % SETS], n);
               }, 15));
        report("copy wave-contiguous U4", 2 * S, median_us([&](int k) {
                   wave_contig<4, 1><<<grid, B>>>(c[k % SETS], a[k % SETS], nullptr);
               }, 15));
        report("copy U1", 2 * S, median_us([&](int k) {
                   wave_contig<1, 1><<<grid * 4, B>>>(c[k % SETS], a[k % SETS], nullptr);
               }, 15));
        report("write-only wave-contiguous U4", S, median_us([&](int k) {
                   wave_contig<4, 2><<<grid, B>>>(c[k % SETS], nullptr, nullptr);
               }, 15));
        report("pair out of place c=a+b (2R:1W)", 3 * S, median_us([&](int k) {
                   pair_tile<OpSum, float, 4, 3><<<grid, B>>>(c[k % SETS], a[k % SETS], b[k % SETS], n);
               }, 15));
    }
    return 0;
}
