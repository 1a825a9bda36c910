// microbench_storepol.hip — exploration harness (not part of the library): which workgroups of the pairwise
// kernel should store their output tile with a buffer store carrying cache-policy bits (sc1 / nt sc1 / sc0 sc1)
// instead of the global nontemporal store, and does that depend on the position in the launch (head, tail,
// the last X MiB), on an interleave (k of every m tiles — consecutive workgroups land on different XCDs, so
// k of 8 = k XCDs), on the individual store instruction, or on the bucket size and placement (in / out of
// place)? One parametrised harness; round 2 asked these questions with six forks of it (tailpol, tailsweep,
// sc1mix 1/2/3, sc1tail; git history at cabc6be), whose evidence stays in profiles/archive/r02_{tailpol,tailsweep,
// sc1mix*,sc1tail*}*.jsonl. The library's answer is FMI_TUNE_PAIR_SC1_OF_8 (k = 1: one XCD's tiles sc1,
// tools/ab_pair_sc1.py, measured with no MALL re-use).
//
// Kernel: the production tile (U = 4 lane groups per thread, 256 threads, nontemporal loads); policy tiles go
// through a per-tile buffer descriptor with store aux A, the others through global nt stores.
// Timing: events around K back-to-back launches per variant, variants interleaved over R rounds, median; the
// operand sets rotate so that >= --footprint-mib is touched per lap (MALL re-use inflates the sc1 forms when
// the footprint is small: use >= 8192 for no re-use at all). Every out-of-place variant's output is compared
// with the all-nt form's (bit-exact).
//
// Build: hipcc -std=c++20 -O3 --offload-arch=gfx950 -ffp-contract=off tools/microbench_storepol.hip -o build/mbsp
// Run:   build/mbsp [--dtype f32|i64] [--sizes 64,256] [--patterns nt,mix:1/8,tail:1/2,tailmib:32,head:1/4,
//                   intra:1/2,xcdtail:32] [--aux 16|17|18] [--inplace 0|1|2=both] [--footprint-mib 1536]
//                   [--rounds 5] [--k 24]
// Patterns (tile b of a grid of G 16-KiB output tiles):
//   nt           no policy tile (the reference form)
//   tail:n/d     b >= G (1 - n/d)          head:n/d    b < G n/d
//   tailmib:X    the last X MiB of output  mix:k/m     b % m < k
//   intra:k/m    in every tile, store instruction u with u % m < k
//   xcdtail:X    b % 8 == 0 (one XCD) plus the last X MiB
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <sstream>
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
constexpr int kU = 4;
constexpr unsigned kTileBytes = kU * 256 * 16;

enum Mode : int { kTail = 0, kHead = 1, kMix = 2, kIntra = 3, kXcdTail = 5 };

__device__ __forceinline__ bool policy_tile(unsigned b, int mode, unsigned p1, unsigned p2) {
    switch (mode) {
        case kTail: return b >= p1;
        case kHead: return b < p1;
        case kMix: return (b % p2) < p1;
        case kXcdTail: return (b % 8) == 0 || b >= p1;
        default: return false;
    }
}

template <class Op, class T, int AUX>
__global__ void __launch_bounds__(256) pair_storepol(T* out, const T* a, const T* b, int mode, unsigned p1, unsigned p2) {
    constexpr int W = kVecLanes<T>;
    using L = Lanes<T, W>;
    const size_t base = static_cast<size_t>(blockIdx.x) * kU * 256 + threadIdx.x;
    L va[kU], vb[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        va[u] = load_lanes<true, T, W>(a + (base + u * 256) * W);
        vb[u] = load_lanes<true, T, W>(b + (base + u * 256) * W);
    }
    char* tile = reinterpret_cast<char*>(out + static_cast<size_t>(blockIdx.x) * kU * 256 * W);
    const auto r = __builtin_amdgcn_make_buffer_rsrc(tile, 0, kTileBytes, kRsrcWord3);
    const bool whole = mode != kIntra && policy_tile(blockIdx.x, mode, p1, p2);
#pragma unroll
    for (int u = 0; u < kU; ++u) {
        const L x = combine<Op, T, W>(va[u], vb[u]);
        if (whole || (mode == kIntra && (u % p2) < p1))
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, x), r, (u * 256 + threadIdx.x) * 16u, 0, AUX);
        else
            store_lanes<true, T, W>(out + (base + u * 256) * W, x);
    }
}

__global__ void fill_k(unsigned* p, size_t n, unsigned seed) {
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
        p[i] = static_cast<unsigned>((i * 2654435761u) ^ (seed * 40503u + (i >> 7)));
}

template <class Op, class T>
void launch_aux(int aux, unsigned grid, T* o, const T* a, const T* b, int mode, unsigned p1, unsigned p2) {
    switch (aux) {
        case 17: pair_storepol<Op, T, 17><<<grid, 256>>>(o, a, b, mode, p1, p2); break;
        case 18: pair_storepol<Op, T, 18><<<grid, 256>>>(o, a, b, mode, p1, p2); break;
        default: pair_storepol<Op, T, 16><<<grid, 256>>>(o, a, b, mode, p1, p2); break;
    }
}

struct Pattern {
    std::string name;
    int mode;
    unsigned p1, p2;  // resolved per grid
};

// name -> (mode, p1, p2) for a grid of G tiles
bool resolve(const std::string& spec, unsigned G, Pattern* out) {
    const auto colon = spec.find(':');
    const std::string kind = spec.substr(0, colon);
    const std::string arg = colon == std::string::npos ? "" : spec.substr(colon + 1);
    unsigned n = 0, d = 1;
    if (arg.find('/') != std::string::npos) {
        n = static_cast<unsigned>(std::atoi(arg.substr(0, arg.find('/')).c_str()));
        d = static_cast<unsigned>(std::atoi(arg.substr(arg.find('/') + 1).c_str()));
    } else if (!arg.empty()) {
        n = static_cast<unsigned>(std::atoi(arg.c_str()));
    }
    const auto tail_tiles = [&](size_t mib) { return static_cast<unsigned>(std::min<size_t>(G, (mib << 20) / kTileBytes)); };
    out->name = spec;
    if (kind == "nt") *out = {spec, kTail, G, 1};
    else if (kind == "tail" && d) *out = {spec, kTail, G - static_cast<unsigned>(size_t(G) * n / d), 1};
    else if (kind == "head" && d) *out = {spec, kHead, static_cast<unsigned>(size_t(G) * n / d), 1};
    else if (kind == "tailmib") *out = {spec, kTail, G - tail_tiles(n), 1};
    else if (kind == "mix" && d) *out = {spec, kMix, n, d};
    else if (kind == "intra" && d) *out = {spec, kIntra, n, d};
    else if (kind == "xcdtail") *out = {spec, kXcdTail, G - tail_tiles(n), 1};
    else return false;
    return true;
}

std::vector<std::string> split(const std::string& s) {
    std::vector<std::string> v;
    std::stringstream ss(s);
    for (std::string x; std::getline(ss, x, ',');)
        if (!x.empty()) v.push_back(x);
    return v;
}

struct Variant {
    std::string name, shape;
    std::function<void(int)> launch;
    double bytes;
    std::vector<double> us;
    void* check_out;
    size_t check_bytes;
    bool checked;
};

int main(int argc, char** argv) {
    std::string dtype = "f32", sizes = "64,256", pats = "nt,mix:1/8,tail:1/2,tailmib:32,head:1/4,intra:1/2,xcdtail:32";
    int aux = 16, inplace = 2, rounds = 5, K = 24;
    size_t footprint_mib = 1536;
    for (int i = 1; i + 1 < argc; i += 2) {
        const std::string k = argv[i], v = argv[i + 1];
        if (k == "--dtype") dtype = v;
        else if (k == "--sizes") sizes = v;
        else if (k == "--patterns") pats = v;
        else if (k == "--aux") aux = std::atoi(v.c_str());
        else if (k == "--inplace") inplace = std::atoi(v.c_str());
        else if (k == "--footprint-mib") footprint_mib = std::strtoull(v.c_str(), nullptr, 10);
        else if (k == "--rounds") rounds = std::atoi(v.c_str());
        else if (k == "--k") K = std::atoi(v.c_str());
        else {
            std::fprintf(stderr, "unknown option %s\n", k.c_str());
            return 2;
        }
    }
    if (aux != 16 && aux != 17 && aux != 18) {
        std::fprintf(stderr, "--aux must be 16 (sc1), 17 (sc0 sc1) or 18 (nt sc1)\n");
        return 2;
    }
    const bool i64 = dtype == "i64";
    std::vector<Variant> vs;
    std::vector<void*> keep;
    for (int ip = 0; ip < 2; ++ip) {
        if (inplace != 2 && ip != inplace) continue;
        for (const std::string& mibs : split(sizes)) {
            const size_t mib = std::strtoull(mibs.c_str(), nullptr, 10);
            const size_t bytes = mib << 20;
            if (bytes == 0 || bytes % kTileBytes) {
                std::fprintf(stderr, "size %zu MiB is not a whole number of 16-KiB tiles\n", mib);
                return 2;
            }
            const int sets = static_cast<int>(std::max<size_t>(2, (footprint_mib << 20) / (3 * bytes)));
            char *A = nullptr, *B = nullptr, *O = nullptr;
            CHECK(hipMalloc(&A, bytes * sets));
            CHECK(hipMalloc(&B, bytes * sets));
            CHECK(hipMalloc(&O, bytes * sets));
            fill_k<<<4096, 256>>>(reinterpret_cast<unsigned*>(A), bytes * sets / 4, 11 + static_cast<unsigned>(mib));
            fill_k<<<4096, 256>>>(reinterpret_cast<unsigned*>(B), bytes * sets / 4, 97 + static_cast<unsigned>(mib));
            keep.insert(keep.end(), {A, B, O});
            const unsigned grid = static_cast<unsigned>(bytes / kTileBytes);
            const std::string shape = std::string(ip ? "inplace " : "outplace ") + dtype + " " + std::to_string(mib) +
                                      "MiB sets=" + std::to_string(sets);
            for (const std::string& spec : split(pats)) {
                Pattern pt;
                if (!resolve(spec, grid, &pt)) {
                    std::fprintf(stderr, "unknown pattern %s\n", spec.c_str());
                    return 2;
                }
                char* dst = ip ? A : O;
                auto launch = [=](int k) {
                    const size_t off = static_cast<size_t>(k % sets) * bytes;
                    if (i64)
                        launch_aux<OpMax, long>(aux, grid, reinterpret_cast<long*>(dst + off), reinterpret_cast<const long*>(A + off),
                                                reinterpret_cast<const long*>(B + off), pt.mode, pt.p1, pt.p2);
                    else
                        launch_aux<OpSum, float>(aux, grid, reinterpret_cast<float*>(dst + off), reinterpret_cast<const float*>(A + off),
                                                 reinterpret_cast<const float*>(B + off), pt.mode, pt.p1, pt.p2);
                };
                vs.push_back({shape + " " + spec + " aux" + std::to_string(aux), shape, launch, 3.0 * bytes, {}, dst, bytes, !ip});
            }
        }
    }
    CHECK(hipDeviceSynchronize());
    {  // bit-exactness: every out-of-place variant of a shape against the shape's first pattern
        std::vector<unsigned char> want, got;
        std::string cur;
        for (auto& v : vs) {
            if (!v.checked) continue;  // in place rewrites its input: timing only
            CHECK(hipMemset(v.check_out, 0xA5, v.check_bytes));
            v.launch(0);
            CHECK(hipDeviceSynchronize());
            auto& dst = v.shape != cur ? want : got;
            dst.resize(v.check_bytes);
            CHECK(hipMemcpy(dst.data(), v.check_out, v.check_bytes, hipMemcpyDeviceToHost));
            if (v.shape == cur && std::memcmp(want.data(), got.data(), v.check_bytes) != 0) {
                std::printf("{\"variant\": \"%s\", \"error\": \"result differs from the shape's first pattern\"}\n", v.name.c_str());
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
        std::printf("{\"variant\": \"%s\", \"median_us\": %.3f, \"min_us\": %.3f, \"frac\": %.4f, \"bit_exact\": %s}\n",
                    v.name.c_str(), us, v.us.front(), v.bytes / (us * 1e-6) / 8e12, v.checked ? "true" : "null");
    }
    for (void* p : keep) CHECK(hipFree(p));
    return 0;
}
