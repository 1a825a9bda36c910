// microbench_tree_u.hip — exploration harness (not part of the library), round 5: with the buckets in distinct
// 4 KiB slots, does the fused 8-way tree gain from more 16-B lane groups per thread (U) or a different
// cap on workgroups per CU? The library's tree_kernel runs U = 1 (one lane group per thread per peer, 8 loads in
// flight) at 2 workgroups per CU (the LDS reservation of FMI_TUNE_FUSED_INFLIGHT_KIB = 64). Here an 8-in / 1-out
// f32 sum of the same access pattern (buffer loads nt, buffer stores sc1, 256-thread workgroups, one tile per
// workgroup) for U = 1, 2, 4 and caps of 2, 4 or 8 workgroups per CU (none = registers decide), interleaved in one
// process over rotating sets of slotted buckets. Wall time per launch from events around `launches` launches;
// every variant's output checked against a host sum on one window. Also U = 1 / 2 at 2 per CU with each XCD taking a
// contiguous eighth of the tiles instead of every eighth tile.
//
// Build: hipcc -std=c++20 -O3 --offload-arch=gfx950 tools/microbench_tree_u.hip -o build/mbtreeu
// Run:   build/mbtreeu [rounds, default 3]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CHECK(x)                                                                                   \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                          \
        }                                                                                          \
    } while (0)

using f32x4 = float __attribute__((ext_vector_type(4)));
using b128 = __attribute__((ext_vector_type(4))) unsigned int;
constexpr int P = 8;
constexpr int kAuxNT = 2, kAuxSC1 = 16;

struct Ptrs {
    const float* in[P];
    float* out;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 1 << 30, 0x00020000);
}

// XCD: 0 = tile = workgroup index (consecutive tiles on consecutive XCDs, the library's order); 1 = each XCD takes
// a contiguous eighth of the tiles (workgroup w runs on XCD w % 8)
template <int U, int XCD>
__global__ void __launch_bounds__(256) tree8(Ptrs p, size_t n16) {
    const size_t per_xcd = gridDim.x / 8;
    const size_t tile = XCD ? (blockIdx.x % 8) * per_xcd + blockIdx.x / 8 : blockIdx.x;
    const size_t first = tile * U * 256;
    if (first + U * 256 > n16) return;  // whole tiles only (sizes here are multiples)
    const size_t tile_byte = first * 16;
    f32x4 v[U][P];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
        for (int q = 0; q < P; ++q)
            v[u][q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                    rsrc(reinterpret_cast<const char*>(p.in[q]) + tile_byte),
                                                    (u * 256 + threadIdx.x) * 16, 0, kAuxNT));
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const f32x4 r = ((v[u][0] + v[u][4]) + (v[u][1] + v[u][5])) + ((v[u][2] + v[u][6]) + (v[u][3] + v[u][7]));
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(b128, r), rsrc(reinterpret_cast<char*>(p.out) + tile_byte),
                                               (u * 256 + threadIdx.x) * 16, 0, kAuxSC1);
    }
}

struct Set {
    std::vector<void*> base;
    Ptrs p;
};

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 3;
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const size_t lds_cu = prop.maxSharedMemoryPerMultiProcessor;
    struct Shape {
        size_t mib;
        int sets, launches;
    };
    const Shape shapes[] = {{1024, 2, 10}, {32, 8, 96}};
    unsigned slot = 0;
    for (const Shape& sh : shapes) {
        const size_t bytes = sh.mib << 20, n16 = bytes / 16;
        std::vector<Set> sets(sh.sets);
        for (int s = 0; s < sh.sets; ++s) {
            for (int q = 0; q <= P; ++q) {
                void* b = nullptr;
                CHECK(hipMalloc(&b, bytes + 65536));
                sets[s].base.push_back(b);
                char* at = static_cast<char*>(b) + (slot++ % 16) * 4096;  // fmi_dev_alloc's rotating slots
                if (q < P) {
                    sets[s].p.in[q] = reinterpret_cast<float*>(at);
                    std::vector<float> h(1 << 20);
                    for (size_t i = 0; i < h.size(); ++i) h[i] = float((i * 7 + q * 13 + s) % 1000) * 0.25f;
                    for (size_t o = 0; o < bytes; o += h.size() * 4)
                        CHECK(hipMemcpy(at + o, h.data(), std::min(bytes - o, h.size() * 4), hipMemcpyHostToDevice));
                } else {
                    sets[s].p.out = reinterpret_cast<float*>(at);
                }
            }
        }
        struct V {
            int u, cap, xcd;
            std::vector<double> us;
        };
        std::vector<V> vs;
        for (int u : {1, 2, 4})
            for (int cap : {2, 4, 8, 0}) vs.push_back({u, cap, 0, {}});
        for (int u : {1, 2}) vs.push_back({u, 2, 1, {}});
        hipEvent_t e0, e1;
        CHECK(hipEventCreate(&e0));
        CHECK(hipEventCreate(&e1));
        for (int r = 0; r < rounds; ++r)
            for (auto& v : vs) {
                const size_t lds = v.cap ? (lds_cu / v.cap) & ~size_t(255) : 0;
                const unsigned grid = static_cast<unsigned>(n16 / (v.u * 256));
                auto launch = [&](int s) {
                    if (v.xcd) {
                        if (v.u == 1) tree8<1, 1><<<grid, 256, lds>>>(sets[s].p, n16);
                        if (v.u == 2) tree8<2, 1><<<grid, 256, lds>>>(sets[s].p, n16);
                        return;
                    }
                    if (v.u == 1) tree8<1, 0><<<grid, 256, lds>>>(sets[s].p, n16);
                    if (v.u == 2) tree8<2, 0><<<grid, 256, lds>>>(sets[s].p, n16);
                    if (v.u == 4) tree8<4, 0><<<grid, 256, lds>>>(sets[s].p, n16);
                };
                for (int s = 0; s < sh.sets; ++s) launch(s);
                CHECK(hipEventRecord(e0));
                for (int k = 0; k < sh.launches; ++k) launch(k % sh.sets);
                CHECK(hipEventRecord(e1));
                CHECK(hipEventSynchronize(e1));
                float ms = 0;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                v.us.push_back(ms * 1e3 / sh.launches);
            }
        // check one window of every set once (the last variant's output)
        bool ok = true;
        for (int s = 0; s < sh.sets && ok; ++s) {
            std::vector<float> x[P], y(4096);
            for (int q = 0; q < P; ++q) {
                x[q].resize(4096);
                CHECK(hipMemcpy(x[q].data(), sets[s].p.in[q], 4096 * 4, hipMemcpyDeviceToHost));
            }
            CHECK(hipMemcpy(y.data(), sets[s].p.out, 4096 * 4, hipMemcpyDeviceToHost));
            for (int i = 0; i < 4096 && ok; ++i) {
                const float w = ((x[0][i] + x[4][i]) + (x[1][i] + x[5][i])) + ((x[2][i] + x[6][i]) + (x[3][i] + x[7][i]));
                ok = std::memcmp(&w, &y[i], 4) == 0;
            }
        }
        for (auto& v : vs) {
            std::sort(v.us.begin(), v.us.end());
            const double med = v.us[v.us.size() / 2];
            std::printf("{\"mib_per_peer\": %zu, \"U\": %d, \"wg_per_cu_cap\": %d, \"xcd_contiguous\": %d, \"median_us\": %.2f, "
                        "\"min_us\": %.2f, \"frac\": %.4f, \"bits_ok\": %s}\n",
                        sh.mib, v.u, v.cap, v.xcd, med, v.us.front(), 9.0 * bytes / (med * 1e-6) / 8e12, ok ? "true" : "false");
        }
        std::fflush(stdout);
        for (auto& s : sets)
            for (void* b : s.base) CHECK(hipFree(b));
    }
    return 0;
}
