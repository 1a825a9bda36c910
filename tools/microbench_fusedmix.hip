// microbench_fusedmix.hip — exploration harness (not part of the library): does the pairwise kernel's
// finding (microbench_sc1mix*.hip: splitting the store policy across XCDs, sc1 on k of every 8 consecutive
// tiles and nontemporal on the rest, streams faster than either policy alone) carry over to the fused P-way
// kernels? Production (FMI_TUNE_FUSED_POLICY = 1) stores trees of >= 4 peers with sc1 and scans of >= 8 with
// nt sc1 on every tile.
//
// Kernel: the production fused programs (reference bracketing, fmi_schedule.h) with buffer loads nt and
// buffer stores whose aux is SA on tiles t with t % m < k and SB on the others; the production launch shape
// (256 threads, one tile per workgroup, the residency cap of fused_lds_bytes). Shapes at 64 MiB per bucket
// (C3's scan P = 8; tree P = 8, the N = 8 shard kernel's program) and the N = 2 / 4 shard shapes (tree P = 2
// at 128 MiB, P = 4 at 64 MiB). Rotating sets >= 1.5 GiB. Every variant is compared with the production
// kernel's output (bit-exact). Timing: events around K back-to-back launches, variants interleaved over R
// rounds, median.
//
// Build: hipcc -std=c++20 -O3 --offload-arch=gfx950 -ffp-contract=off tools/microbench_fusedmix.hip -o build/mbf
// Run:   build/mbf [rounds, default 5]
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

template <int SA, class T, int W, int ALG, int P, bool ALL_OUT>
__device__ __forceinline__ void store_outs(const Lanes<T, W>* v, const PeerPtrs& ptrs, size_t tile_byte, unsigned lane_byte) {
    if constexpr (ALL_OUT) {
        [&]<size_t... R>(std::index_sequence<R...>) {
            ((store_tile<SA, T, W>(ptrs.out[R], tile_byte, lane_byte, v[kOut<ALG, P, R>])), ...);
        }(std::make_index_sequence<P>{});
    } else {
        store_tile<SA, T, W>(ptrs.out[0], tile_byte, lane_byte, v[kOut<ALG, P, 0>]);
    }
}

template <class Op, class T, int ALG, int P, bool ALL_OUT, int SA, int SB>
__global__ void __launch_bounds__(256) fused_mix(PeerPtrs ptrs, size_t n, unsigned k, unsigned m) {
    constexpr int W = kVecLanes<T>;
    const size_t nvec = n / W;
    const size_t B = blockDim.x;
    for (size_t tile = blockIdx.x; tile * B < nvec; tile += gridDim.x) {
        if (tile * B + threadIdx.x >= nvec) continue;
        const size_t tile_byte = tile * B * 16;
        const unsigned lane_byte = threadIdx.x * 16u;
        Lanes<T, W> v[P + kNumSteps<ALG, P>];
        load_peers_tile<T, W, P>(v, ptrs, tile_byte, lane_byte, std::make_index_sequence<P>{});
        run_steps<Op, T, W, ALG, P>(v, std::make_index_sequence<kNumSteps<ALG, P>>{});
        if ((tile % m) < k)
            store_outs<SA, T, W, ALG, P, ALL_OUT>(v, ptrs, tile_byte, lane_byte);
        else
            store_outs<SB, T, W, ALG, P, ALL_OUT>(v, ptrs, tile_byte, lane_byte);
    }
}

__global__ void fill_k(unsigned* p, size_t n, unsigned seed) {
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
        p[i] = 0x3f800000u | (static_cast<unsigned>((i * 2654435761u) ^ (seed * 40503u)) & 0x007fffffu);  // [1, 2)
}

size_t fused_lds(int P) {  // the library's residency cap (fused_lds_bytes, 64 KiB budget per CU)
    const size_t per_wg = size_t(P) * 4096, budget = 64 << 10;
    const size_t cap = std::max<size_t>(2, (budget + per_wg - 1) / per_wg);
    return cap >= 32 ? 0 : ((160 << 10) / cap) & ~size_t(255);
}

struct Variant {
    std::string name, shape;
    std::function<void(int)> launch;
    double bytes;
    std::vector<double> us;
    float* check;
    size_t check_bytes;
};

struct Shape {
    std::vector<PeerPtrs> sets;
    size_t n;
    int nsets;
};

Shape make_shape(int P, size_t bytes, bool all_out) {
    Shape sh;
    sh.n = bytes / 4;
    const size_t per_set = bytes * (P + (all_out ? P : 1));
    sh.nsets = static_cast<int>(std::max<size_t>(2, ((size_t(1536) << 20) + per_set - 1) / per_set));
    for (int s = 0; s < sh.nsets; ++s) {
        PeerPtrs p{};
        for (int j = 0; j < P; ++j) {
            void* in = nullptr;
            CHECK(hipMalloc(&in, bytes));
            fill_k<<<4096, 256>>>(static_cast<unsigned*>(in), bytes / 4, 100 * s + j);
            p.in[j] = in;
        }
        for (int j = 0; j < (all_out ? P : 1); ++j) CHECK(hipMalloc(&p.out[j], bytes));
        sh.sets.push_back(p);
    }
    return sh;
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 5;
    constexpr int K = 20;
    constexpr int SC = fmi::sched::kScan, AR = fmi::sched::kAllreduce;
    constexpr int NT = kAuxNT, S1 = kAuxSC1, NS = kAuxNT | kAuxSC1;
    std::vector<Variant> vs;
    std::vector<Shape> shapes;
    shapes.reserve(4);
    // (k, m) patterns: production = one policy everywhere (k = m)
    struct Pat {
        const char* name;
        unsigned k, m;
    };
    const Pat mixes[] = {{"4/8", 4, 8}, {"2/8", 2, 8}, {"6/8", 6, 8}};
#define ADD(TAG, SH, ALG, P_, ALLOUT, SA, SB, PNAME, K_, M_, BYTES)                                               \
    {                                                                                                              \
        Shape* sh = &(SH);                                                                                         \
        const unsigned grid = static_cast<unsigned>(sh->n / 4 / 256);                                              \
        const size_t lds = fused_lds(P_);                                                                          \
        const unsigned kk = K_, mm = M_;                                                                           \
        vs.push_back({std::string(TAG) + " " + PNAME, TAG, [=](int k) {                                            \
                          fused_mix<OpSum, float, ALG, P_, ALLOUT, SA, SB><<<grid, 256, lds>>>(sh->sets[k % sh->nsets], sh->n, kk, mm); \
                      }, BYTES, {}, static_cast<float*>(sh->sets[0].out[0]), sh->n * 4});                          \
    }
    const size_t MB64 = size_t(64) << 20, MB128 = size_t(128) << 20;
    shapes.push_back(make_shape(8, MB64, true));   // scan8
    shapes.push_back(make_shape(8, MB64, false));  // tree8
    shapes.push_back(make_shape(4, MB64, false));  // tree4
    shapes.push_back(make_shape(2, MB128, false)); // tree2
    CHECK(hipDeviceSynchronize());
    const double bs8 = 16.0 * MB64, bt8 = 9.0 * MB64, bt4 = 5.0 * MB64, bt2 = 3.0 * MB128;
    // scan8: production nt sc1 everywhere; alternatives
    ADD("scan8", shapes[0], SC, 8, true, NS, NS, "prod ntsc1", 1, 1, bs8)
    ADD("scan8", shapes[0], SC, 8, true, NT, NT, "nt", 1, 1, bs8)
    ADD("scan8", shapes[0], SC, 8, true, S1, S1, "sc1", 1, 1, bs8)
    for (const Pat& p : mixes) {
        ADD("scan8", shapes[0], SC, 8, true, S1, NT, std::string("sc1|nt ") + p.name, p.k, p.m, bs8)
        ADD("scan8", shapes[0], SC, 8, true, NS, NT, std::string("ntsc1|nt ") + p.name, p.k, p.m, bs8)
    }
    // trees: production sc1 everywhere (P >= 4), global nt for P = 2 (here: buffer nt)
    ADD("tree8", shapes[1], AR, 8, false, S1, S1, "prod sc1", 1, 1, bt8)
    ADD("tree8", shapes[1], AR, 8, false, NT, NT, "nt", 1, 1, bt8)
    ADD("tree4", shapes[2], AR, 4, false, S1, S1, "prod sc1", 1, 1, bt4)
    ADD("tree4", shapes[2], AR, 4, false, NT, NT, "nt", 1, 1, bt4)
    ADD("tree2", shapes[3], AR, 2, false, NT, NT, "prod nt", 1, 1, bt2)
    ADD("tree2", shapes[3], AR, 2, false, S1, S1, "sc1", 1, 1, bt2)
    for (const Pat& p : mixes) {
        ADD("tree8", shapes[1], AR, 8, false, S1, NT, std::string("sc1|nt ") + p.name, p.k, p.m, bt8)
        ADD("tree4", shapes[2], AR, 4, false, S1, NT, std::string("sc1|nt ") + p.name, p.k, p.m, bt4)
        ADD("tree2", shapes[3], AR, 2, false, S1, NT, std::string("sc1|nt ") + p.name, p.k, p.m, bt2)
    }
    {  // bit-exactness against the first (production) variant of each shape
        std::vector<unsigned char> want, got;
        std::string cur;
        for (auto& v : vs) {
            CHECK(hipMemset(v.check, 0xA5, v.check_bytes));
            v.launch(0);
            CHECK(hipDeviceSynchronize());
            auto& dst = v.shape != cur ? want : got;
            dst.resize(v.check_bytes);
            CHECK(hipMemcpy(dst.data(), v.check, v.check_bytes, hipMemcpyDeviceToHost));
            if (v.shape == cur && std::memcmp(want.data(), got.data(), v.check_bytes) != 0) {
                std::printf("{\"variant\": \"%s\", \"error\": \"result differs from production\"}\n", v.name.c_str());
                return 1;
            }
            cur = v.shape;
        }
    }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int r = 0; r < rounds; ++r)
        for (auto& v : vs) {
            for (int k = 0; k < 2; ++k) v.launch(k);
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
