// microbench_policy.hip — exploration harness (not part of the library): the C2 pairwise f32 sum
// (256 MiB buckets, U = 4 lane groups per thread, 256 threads) with every gfx950 cache-policy combination
// on its loads and stores, through raw buffer instructions whose aux operand carries the policy bits
// (gfx94x/gfx950: bit 0 = sc0, bit 1 = nt, bit 4 = sc1). The production kernel (global_load/store … nt)
// runs in the same process for reference.
//
// Build: hipcc -std=c++20 -O3 --offload-arch=gfx950 tools/microbench_policy.hip -o build/mbp
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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

using v4f = float __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, static_cast<int>(bytes), 0x00020000);
}

// One buffer covers the whole 256 MiB bucket (offsets < 2^31).
template <int LAUX, int SAUX>
__global__ void __launch_bounds__(256) pair_buf(float* out, const float* a, const float* b, unsigned nbytes) {
    constexpr int U = 4;
    const auto ra = rsrc(a, nbytes), rb = rsrc(b, nbytes), ro = rsrc(out, nbytes);
    const int base = (blockIdx.x * U * 256 + threadIdx.x) * 16;
    v4f x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        x[u] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(ra, base + u * 256 * 16, 0, LAUX));
        y[u] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(rb, base + u * 256 * 16, 0, LAUX));
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, x[u] + y[u]), ro, base + u * 256 * 16, 0, SAUX);
}

template <class F>
double median_us(F&& launch, int iters) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int k = 0; k < 3; ++k) launch(k);
    CHECK(hipDeviceSynchronize());
    std::vector<double> t;
    for (int r = 0; r < iters; ++r) {
        CHECK(hipEventRecord(e0));
        for (int k = 0; k < 8; ++k) launch(k);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        t.push_back(ms * 1e3 / 8);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main() {
    const size_t n = (256u << 20) / 4;
    const unsigned nbytes = static_cast<unsigned>(n * 4);
    constexpr int SETS = 4;
    float* a[SETS];
    float* b[SETS];
    for (int s = 0; s < SETS; ++s) {
        CHECK(hipMalloc(&a[s], n * 4));
        CHECK(hipMalloc(&b[s], n * 4));
        CHECK(hipMemset(a[s], 0, n * 4));
        CHECK(hipMemset(b[s], 0, n * 4));
    }
    const unsigned grid = static_cast<unsigned>(n / 4 / (4 * 256));
    const double bytes = 3.0 * n * 4;
    auto report = [&](const char* name, double us) {
        const double gbs = bytes / (us * 1e-6) / 1e9;
        std::printf("{\"variant\": \"%s\", \"us\": %.2f, \"GB_s\": %.1f, \"frac\": %.4f}\n", name, us, gbs, gbs / 8000.);
        std::fflush(stdout);
    };
    for (int round = 0; round < 2; ++round) {
        report("production pair_tile global nt/nt", median_us([&](int k) {
                   pair_tile<OpSum, float, 4, 3><<<grid, 256>>>(a[k % SETS], a[k % SETS], b[k % SETS], n);
               }, 15));
#define V(L, S)                                                                                  \
    report("buffer load aux " #L " store aux " #S, median_us([&](int k) {                        \
               pair_buf<L, S><<<grid, 256>>>(a[k % SETS], a[k % SETS], b[k % SETS], nbytes);     \
           }, 15));
        V(0, 0)
        V(2, 2)
        V(3, 2)
        V(16, 2)
        V(18, 2)
        V(19, 2)
        V(2, 0)
        V(2, 16)
        V(2, 18)
        V(2, 19)
        V(17, 17)
        V(8, 8)
        V(10, 10)
        V(11, 11)
    }
    return 0;
}
