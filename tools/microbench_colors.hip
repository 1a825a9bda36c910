// microbench_colors.hip — exploration harness (not part of the library): does a per-bucket address skew
// ("colouring") remove the placement spread of the multi-stream kernels? C3's peer scan reads 8 and writes 8
// separately allocated 64 MiB buckets at the same element offset at the same time; its time varies 170-220 us
// with the allocation draw, the write side bimodal. Hypothesis: the DRAM channel / bank of an
// address is a function of its low bits XOR a function of the bucket's base, so buckets whose bases hash alike
// collide at every offset; skewing bucket k by k x `skew` bytes changes the low bits that meet at one offset.
// Per draw: 16 buckets of 64 MiB + 1 MiB slack, each its own hipMalloc (a random spacer allocation before each
// draw varies placement); the same physical buckets are then timed through every skew scheme (views base_k +
// (k * skew) mod 1 MiB), interleaved over R rounds of K back-to-back launches (events), median per scheme:
//   write8   out_k = const for the 8 output buckets           (the write side alone)
//   copy8    out_k = in_k                                      (the scan's traffic, no arithmetic)
//   scan8    the library's peer scan (fmi_dev_scan_peers, scan_no_order, f32 sum)
// Build: hipcc -std=c++20 -O3 --offload-arch=gfx950 -ffp-contract=off tools/microbench_colors.hip
//          -Lfmi_amd/lib -lfmi_dev -Wl,-rpath,$PWD/fmi_amd/lib -o build/mbcol
// Run:   build/mbcol [draws, default 6] [rounds, default 4]    |    build/mbcol rot|rotwarm|streams|contig|libcontig|vmm [draws] [rounds]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
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

constexpr int kP = 8;
constexpr int kU = 4;
using V = u32x4;

struct Ptrs {
    const V* in[kP];
    V* out[kP];
};

template <int N>
struct Ptrs16N {
    V* p[N];
};

__device__ __forceinline__ V ld(const V* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void st(V* p, V v) { __builtin_nontemporal_store(v, p); }

__global__ void __launch_bounds__(256) copy8(Ptrs b) {
    const size_t base = static_cast<size_t>(blockIdx.x) * kU * 256 + threadIdx.x;
    V v[kP][kU];
#pragma unroll
    for (int p = 0; p < kP; ++p)
#pragma unroll
        for (int u = 0; u < kU; ++u) v[p][u] = ld(b.in[p] + base + u * 256);
#pragma unroll
    for (int p = 0; p < kP; ++p)
#pragma unroll
        for (int u = 0; u < kU; ++u) st(b.out[p] + base + u * 256, v[p][u]);
}

__global__ void __launch_bounds__(256) write8(Ptrs b) {
    const size_t base = static_cast<size_t>(blockIdx.x) * kU * 256 + threadIdx.x;
    const V c = {blockIdx.x, threadIdx.x, 7u, 9u};
#pragma unroll
    for (int p = 0; p < kP; ++p)
#pragma unroll
        for (int u = 0; u < kU; ++u) st(b.out[p] + base + u * 256, c);
}

// Touches one 16-B word per 64 KiB of every bucket of a set (address translations only, a few us): run
// before a launch, outside its events, it tells translation misses apart from placement ("rotwarm").
__global__ void __launch_bounds__(256) touch16(Ptrs b, V* sink) {
    const size_t i = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x;  // page index within a bucket
    const int k = blockIdx.y;
    const V* base = k < kP ? b.in[k] : b.out[k - kP];
    const V v = __builtin_nontemporal_load(base + i * (65536 / 16));
    if (v[0] == 0x12345678u && v[1] == 0x9abcdef0u) sink[threadIdx.x] = v;  // never true: keeps the load
}

// Mode "rot": the bench's protocol — S sets of 16 buckets rotating (no set re-used within 3 GiB of traffic), an
// event pair around every launch, median per set; allocation size exactly 64 MiB ("exact") or 64 MiB + 16 MiB
// ("slack", the bucket at the allocation's base), or bucket k at (k x skew) mod 16 MiB into it ("skew*").
int rotating(int draws, int rounds, bool warm) {
    constexpr size_t kBytes = size_t(64) << 20;
    constexpr size_t kSlack = size_t(16) << 20;
    constexpr int S = 4;
    const size_t nvec = kBytes / 16;
    const unsigned grid = static_cast<unsigned>(nvec / (kU * 256));
    hipStream_t s = nullptr;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<hipEvent_t> ev(2 * S * rounds);
    V* sink = nullptr;
    CHECK(hipMalloc(&sink, 4096));
    for (auto& evt : ev) CHECK(hipEventCreate(&evt));
    struct Mode {
        const char* name;
        size_t alloc;
        size_t skew;
    };
    const Mode modes[] = {{"exact", kBytes, 0},           {"slack", kBytes + kSlack, 0},
                          {"skew4k", kBytes + kSlack, 4096}, {"skew64k", kBytes + kSlack, 65536},
                          {"skew256k", kBytes + kSlack, 262144}, {"skew1m", kBytes + kSlack, 1 << 20},
                          {"skew2m64k", kBytes + kSlack, (2 << 20) + 65536}};
    for (int d = 0; d < draws; ++d)
        for (const Mode& m : modes) {
            std::vector<char*> bufs;
            Ptrs sets[S];
            for (int j = 0; j < S; ++j)
                for (int k = 0; k < 2 * kP; ++k) {
                    char* b = nullptr;
                    CHECK(hipMalloc(reinterpret_cast<void**>(&b), m.alloc));
                    CHECK(hipMemset(b, 0x3c, m.alloc));
                    bufs.push_back(b);
                    char* v = b + (k * m.skew) % kSlack;
                    if (k < kP) sets[j].in[k] = reinterpret_cast<const V*>(v);
                    else sets[j].out[k - kP] = reinterpret_cast<V*>(v);
                }
            CHECK(hipDeviceSynchronize());
            for (const char* kern : {"write8", "scan8"}) {
                auto launch = [&](int j) {
                    const Ptrs& p = sets[j];
                    if (kern[0] == 'w') {
                        write8<<<grid, 256, 0, s>>>(p);
                        return;
                    }
                    void* outs[kP];
                    const void* ins[kP];
                    for (int k = 0; k < kP; ++k) {
                        outs[k] = p.out[k];
                        ins[k] = p.in[k];
                    }
                    if (fmi_dev_scan_peers(FMI_OP_SUM, FMI_F32, FMI_ALG_SCAN, outs, ins, kP, kBytes / 4, s) != FMI_OK) {
                        std::fprintf(stderr, "scan: %s\n", fmi_last_error());
                        std::exit(1);
                    }
                };
                for (int j = 0; j < S; ++j) launch(j);
                for (int r = 0; r < rounds; ++r)
                    for (int j = 0; j < S; ++j) {
                        if (warm) touch16<<<dim3(kBytes / 65536 / 256, 2 * kP), 256, 0, s>>>(sets[j], sink);
                        CHECK(hipEventRecord(ev[2 * (r * S + j)], s));
                        launch(j);
                        CHECK(hipEventRecord(ev[2 * (r * S + j) + 1], s));
                    }
                CHECK(hipStreamSynchronize(s));
                const double bytes = (kern[0] == 'w' ? 1.0 : 2.0) * kP * kBytes;
                for (int j = 0; j < S; ++j) {
                    std::vector<double> us;
                    for (int r = 0; r < rounds; ++r) {
                        float ms = 0;
                        CHECK(hipEventElapsedTime(&ms, ev[2 * (r * S + j)], ev[2 * (r * S + j) + 1]));
                        us.push_back(ms * 1e3);
                    }
                    std::sort(us.begin(), us.end());
                    const double u = us[us.size() / 2];
                    std::printf("{\"warm\": %d, \"mode\": \"%s\", \"draw\": %d, \"set\": %d, \"kernel\": \"%s\", \"median_us\": %.2f, "
                                "\"frac\": %.4f}\n", int(warm), m.name, d, j, kern, u, bytes / (u * 1e-6) / 8e12);
                }
            }
            std::fflush(stdout);
            for (char* b : bufs) CHECK(hipFree(b));
        }
    return 0;
}

// Mode "streams": the same 512 MiB written (or read) as N concurrent streams of 512/N MiB each (N = 1, 2, 4, 8,
// 16), S = 4 rotating sets of separate allocations, an event pair per launch, median per set: does the write
// rate depend on how many streams are open at once?
template <int N, bool WRITE>
__global__ void __launch_bounds__(256) streamsN(Ptrs16N<N> b, V* sink) {
    const size_t base = static_cast<size_t>(blockIdx.x) * kU * 256 + threadIdx.x;
    if constexpr (WRITE) {
        const V c = {blockIdx.x, threadIdx.x, 7u, 9u};
#pragma unroll
        for (int p = 0; p < N; ++p)
#pragma unroll
            for (int u = 0; u < kU; ++u) st(b.p[p] + base + u * 256, c);
    } else {
        V acc = {0, 0, 0, 0};
#pragma unroll
        for (int p = 0; p < N; ++p)
#pragma unroll
            for (int u = 0; u < kU; ++u) acc ^= ld(b.p[p] + base + u * 256);
        if (acc[0] == 0x12345678u && acc[1] == 0x9abcdef0u) sink[threadIdx.x] = acc;
    }
}

template <int N, bool WRITE>
void run_streams(int draws, int rounds, hipStream_t s, std::vector<hipEvent_t>& ev, V* sink, unsigned flags = 0) {
    constexpr size_t kTotal = size_t(512) << 20;
    constexpr size_t kEach = kTotal / N;
    constexpr int S = 4;
    const unsigned grid = static_cast<unsigned>(kEach / 16 / (kU * 256));
    for (int d = 0; d < draws; ++d) {
        std::vector<void*> bufs;
        Ptrs16N<N> sets[S];
        for (int j = 0; j < S; ++j)
            for (int k = 0; k < N; ++k) {
                void* b = nullptr;
                if (flags) CHECK(hipExtMallocWithFlags(&b, kEach, flags));
                else CHECK(hipMalloc(&b, kEach));
                CHECK(hipMemset(b, 0x3c, kEach));
                bufs.push_back(b);
                sets[j].p[k] = static_cast<V*>(b);
            }
        CHECK(hipDeviceSynchronize());
        for (int j = 0; j < S; ++j) streamsN<N, WRITE><<<grid, 256, 0, s>>>(sets[j], sink);
        for (int r = 0; r < rounds; ++r)
            for (int j = 0; j < S; ++j) {
                CHECK(hipEventRecord(ev[2 * (r * S + j)], s));
                streamsN<N, WRITE><<<grid, 256, 0, s>>>(sets[j], sink);
                CHECK(hipEventRecord(ev[2 * (r * S + j) + 1], s));
            }
        CHECK(hipStreamSynchronize(s));
        for (int j = 0; j < S; ++j) {
            std::vector<double> us;
            for (int r = 0; r < rounds; ++r) {
                float ms = 0;
                CHECK(hipEventElapsedTime(&ms, ev[2 * (r * S + j)], ev[2 * (r * S + j) + 1]));
                us.push_back(ms * 1e3);
            }
            std::sort(us.begin(), us.end());
            const double u = us[us.size() / 2];
            std::printf("{\"streams\": %d, \"op\": \"%s\", \"alloc_flags\": %u, \"draw\": %d, \"set\": %d, \"median_us\": %.2f, "
                        "\"frac\": %.4f}\n", N, WRITE ? "write" : "read", flags, d, j, u, kTotal / (u * 1e-6) / 8e12);
        }
        std::fflush(stdout);
        for (void* b : bufs) CHECK(hipFree(b));
    }
}

int streams(int draws, int rounds) {
    hipStream_t s = nullptr;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<hipEvent_t> ev(2 * 4 * rounds);
    for (auto& evt : ev) CHECK(hipEventCreate(&evt));
    V* sink = nullptr;
    CHECK(hipMalloc(&sink, 4096));
    run_streams<1, true>(draws, rounds, s, ev, sink);
    run_streams<2, true>(draws, rounds, s, ev, sink);
    run_streams<4, true>(draws, rounds, s, ev, sink);
    run_streams<8, true>(draws, rounds, s, ev, sink);
    run_streams<16, true>(draws, rounds, s, ev, sink);
    run_streams<1, false>(draws, rounds, s, ev, sink);
    run_streams<8, false>(draws, rounds, s, ev, sink);
    return 0;
}

// Mode "contig": 8 write streams from hipMalloc against hipExtMallocWithFlags(hipDeviceMallocContiguous)
// (physically contiguous buckets), interleaved draw by draw.
int contig(int draws, int rounds) {
    hipStream_t s = nullptr;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<hipEvent_t> ev(2 * 4 * rounds);
    for (auto& evt : ev) CHECK(hipEventCreate(&evt));
    V* sink = nullptr;
    CHECK(hipMalloc(&sink, 4096));
    for (int d = 0; d < draws; ++d) {
        run_streams<8, true>(1, rounds, s, ev, sink, 0);
        run_streams<8, true>(1, rounds, s, ev, sink, hipDeviceMallocContiguous);
        run_streams<1, true>(1, rounds, s, ev, sink, 0);
        run_streams<1, true>(1, rounds, s, ev, sink, hipDeviceMallocContiguous);
    }
    return 0;
}

// Mode "libcontig": the library's own C2 pair kernel (fmi_dev_reduce_pair, f32 sum, 256 MiB, 16 rotating pairs)
// and C3 scan (fmi_dev_scan_peers, 8 x 64 MiB, 4 rotating sets) on buckets from hipMalloc against
// hipExtMallocWithFlags(hipDeviceMallocContiguous); two HIP events around each pass of back-to-back launches.
double lib_pass(bool scan, unsigned flags, int passes, hipStream_t s) {
    const int S = scan ? 4 : 16;
    const size_t bytes = scan ? size_t(64) << 20 : size_t(256) << 20;
    const int per = scan ? 16 : 2;
    std::vector<void*> b(static_cast<size_t>(S) * per);
    for (auto& p : b) {
        if (flags) CHECK(hipExtMallocWithFlags(&p, bytes, flags));
        else CHECK(hipMalloc(&p, bytes));
        CHECK(hipMemset(p, 0x3c, bytes));
    }
    CHECK(hipDeviceSynchronize());
    auto launch = [&](int j) {
        void** q = &b[static_cast<size_t>(j) * per];
        int rc;
        if (scan) {
            const void* ins[kP];
            void* outs[kP];
            for (int k = 0; k < kP; ++k) {
                ins[k] = q[k];
                outs[k] = q[kP + k];
            }
            rc = fmi_dev_scan_peers(FMI_OP_SUM, FMI_F32, FMI_ALG_SCAN, outs, ins, kP, bytes / 4, s);
        } else {
            rc = fmi_dev_reduce_pair(FMI_OP_SUM, FMI_F32, q[0], q[1], bytes / 4, s);
        }
        if (rc != FMI_OK) {
            std::fprintf(stderr, "launch: %s\n", fmi_last_error());
            std::exit(1);
        }
    };
    for (int j = 0; j < S; ++j) launch(j);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipEventRecord(e0, s));
    for (int r = 0; r < passes; ++r)
        for (int j = 0; j < S; ++j) launch(j);
    CHECK(hipEventRecord(e1, s));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
    for (void* p : b) CHECK(hipFree(p));
    return ms * 1e3 / (passes * S);
}

int libcontig(int draws) {
    hipStream_t s = nullptr;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    for (int d = 0; d < draws; ++d)
        for (bool scan : {false, true})
            for (unsigned flags : {0u, unsigned(hipDeviceMallocContiguous)}) {
                const double us = lib_pass(scan, flags, scan ? 6 : 4, s);
                const double bytes = scan ? 2.0 * kP * (64 << 20) : 3.0 * (256 << 20);
                std::printf("{\"kernel\": \"%s\", \"alloc_flags\": %u, \"draw\": %d, \"mean_us\": %.2f, \"frac\": %.4f}\n",
                            scan ? "scan8" : "pair_c2", flags, d, us, bytes / (us * 1e-6) / 8e12);
                std::fflush(stdout);
            }
    return 0;
}

// Mode "vmm": 8 write streams into buckets placed with the HIP virtual-memory API — physical memory from
// hipMemCreate mapped at virtual addresses aligned to 1 GiB (one reservation per bucket), or all 8 buckets
// back to back in one 1 GiB-aligned reservation — against hipMalloc, rotating sets as in "streams". Does the
// virtual placement (translation fragments, alignment) decide the write rate?
struct VmmBuf {
    void* va = nullptr;
    size_t reserved = 0;
    hipMemGenericAllocationHandle_t h{};
};

void run_vmm_mode(int mode, int rounds, hipStream_t s, std::vector<hipEvent_t>& ev, V* sink, int d) {
    constexpr size_t kEach = size_t(64) << 20;
    constexpr int N = 8, S = 4;
    const unsigned grid = static_cast<unsigned>(kEach / 16 / (kU * 256));
    hipMemAllocationProp prop{};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    hipMemAccessDesc acc{};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    std::vector<void*> plain;
    std::vector<VmmBuf> vm;
    std::vector<void*> ranges;
    Ptrs16N<N> sets[S];
    for (int j = 0; j < S; ++j) {
        char* block = nullptr;
        if (mode == 2) {
            CHECK(hipMemAddressReserve(reinterpret_cast<void**>(&block), N * kEach, size_t(1) << 30, nullptr, 0));
            ranges.push_back(block);
        }
        for (int k = 0; k < N; ++k) {
            void* p = nullptr;
            if (mode == 0) {
                CHECK(hipMalloc(&p, kEach));
                plain.push_back(p);
            } else {
                VmmBuf b;
                if (mode == 1) {
                    CHECK(hipMemAddressReserve(&b.va, kEach, size_t(1) << 30, nullptr, 0));
                    b.reserved = kEach;
                } else {
                    b.va = block + k * kEach;
                }
                CHECK(hipMemCreate(&b.h, kEach, &prop, 0));
                CHECK(hipMemMap(b.va, kEach, 0, b.h, 0));
                CHECK(hipMemSetAccess(b.va, kEach, &acc, 1));
                p = b.va;
                vm.push_back(b);
            }
            CHECK(hipMemset(p, 0x3c, kEach));
            sets[j].p[k] = static_cast<V*>(p);
        }
    }
    CHECK(hipDeviceSynchronize());
    for (int j = 0; j < S; ++j) streamsN<N, true><<<grid, 256, 0, s>>>(sets[j], sink);
    for (int r = 0; r < rounds; ++r)
        for (int j = 0; j < S; ++j) {
            CHECK(hipEventRecord(ev[2 * (r * S + j)], s));
            streamsN<N, true><<<grid, 256, 0, s>>>(sets[j], sink);
            CHECK(hipEventRecord(ev[2 * (r * S + j) + 1], s));
        }
    CHECK(hipStreamSynchronize(s));
    for (int j = 0; j < S; ++j) {
        std::vector<double> us;
        for (int r = 0; r < rounds; ++r) {
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, ev[2 * (r * S + j)], ev[2 * (r * S + j) + 1]));
            us.push_back(ms * 1e3);
        }
        std::sort(us.begin(), us.end());
        const double u = us[us.size() / 2];
        std::printf("{\"vmm_mode\": %d, \"draw\": %d, \"set\": %d, \"median_us\": %.2f, \"frac\": %.4f}\n", mode, d, j, u,
                    N * kEach / (u * 1e-6) / 8e12);
    }
    std::fflush(stdout);
    for (void* p : plain) CHECK(hipFree(p));
    for (auto& b : vm) {
        CHECK(hipMemUnmap(b.va, kEach));
        CHECK(hipMemRelease(b.h));
        if (b.reserved) CHECK(hipMemAddressFree(b.va, b.reserved));
    }
    for (void* r : ranges) CHECK(hipMemAddressFree(r, N * kEach));
}

int vmm(int draws, int rounds) {
    hipStream_t s = nullptr;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<hipEvent_t> ev(2 * 4 * rounds);
    for (auto& evt : ev) CHECK(hipEventCreate(&evt));
    V* sink = nullptr;
    CHECK(hipMalloc(&sink, 4096));
    for (int d = 0; d < draws; ++d)
        for (int mode : {0, 1, 2}) run_vmm_mode(mode, rounds, s, ev, sink, d);
    return 0;
}

int main(int argc, char** argv) {
    if (argc > 1 && std::string(argv[1]) == "vmm") {
        CHECK(hipSetDevice(0));
        return vmm(argc > 2 ? std::atoi(argv[2]) : 3, argc > 3 ? std::atoi(argv[3]) : 6);
    }
    if (argc > 1 && std::string(argv[1]) == "libcontig") {
        CHECK(hipSetDevice(0));
        if (fmi_dev_init(0) != FMI_OK) return 1;
        return libcontig(argc > 2 ? std::atoi(argv[2]) : 4);
    }
    if (argc > 1 && std::string(argv[1]) == "contig") {
        CHECK(hipSetDevice(0));
        return contig(argc > 2 ? std::atoi(argv[2]) : 3, argc > 3 ? std::atoi(argv[3]) : 6);
    }
    if (argc > 1 && std::string(argv[1]) == "streams") {
        CHECK(hipSetDevice(0));
        return streams(argc > 2 ? std::atoi(argv[2]) : 2, argc > 3 ? std::atoi(argv[3]) : 6);
    }
    if (argc > 1 && (std::string(argv[1]) == "rot" || std::string(argv[1]) == "rotwarm")) {
        CHECK(hipSetDevice(0));
        if (fmi_dev_init(0) != FMI_OK) return 1;
        return rotating(argc > 2 ? std::atoi(argv[2]) : 3, argc > 3 ? std::atoi(argv[3]) : 5,
                        std::string(argv[1]) == "rotwarm");
    }
    const int draws = argc > 1 ? std::atoi(argv[1]) : 6;
    const int rounds = argc > 2 ? std::atoi(argv[2]) : 4;
    constexpr int K = 10;
    constexpr size_t kBytes = size_t(64) << 20;
    constexpr size_t kSlack = size_t(1) << 20;
    const size_t nvec = kBytes / 16;
    const unsigned grid = static_cast<unsigned>(nvec / (kU * 256));
    const size_t skews[] = {0, 4096, 8192, 65536, 4352, 256 * 1024 + 4096};
    CHECK(hipSetDevice(0));
    if (fmi_dev_init(0) != FMI_OK) {
        std::fprintf(stderr, "fmi_dev_init: %s\n", fmi_last_error());
        return 1;
    }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipStream_t s = nullptr;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::mt19937 rng(12345);
    std::vector<void*> spacers;
    for (int d = 0; d < draws; ++d) {
        void* sp = nullptr;
        CHECK(hipMalloc(&sp, (size_t(2) << 20) * (1 + rng() % 48)));  // kept: later draws land elsewhere
        spacers.push_back(sp);
        char* buf[2 * kP];
        for (auto& b : buf) {
            CHECK(hipMalloc(reinterpret_cast<void**>(&b), kBytes + kSlack));
            CHECK(hipMemset(b, 0x3c, kBytes + kSlack));  // finite f32 values for the scan
        }
        CHECK(hipDeviceSynchronize());
        struct Row {
            const char* kernel;
            size_t skew;
            double bytes;
            std::vector<double> us;
        };
        std::vector<Row> rows;
        for (size_t sk : skews)
            for (const char* k : {"write8", "copy8", "scan8"})
                rows.push_back({k, sk, (k[0] == 'w' ? 1.0 : 2.0) * kP * kBytes, {}});
        for (int r = 0; r < rounds; ++r)
            for (auto& row : rows) {
                Ptrs p{};
                for (int k = 0; k < kP; ++k) {
                    p.in[k] = reinterpret_cast<const V*>(buf[k] + (k * row.skew) % kSlack);
                    p.out[k] = reinterpret_cast<V*>(buf[kP + k] + ((kP + k) * row.skew) % kSlack);
                }
                auto launch = [&] {
                    if (row.kernel[0] == 'w') {
                        write8<<<grid, 256, 0, s>>>(p);
                    } else if (row.kernel[0] == 'c') {
                        copy8<<<grid, 256, 0, s>>>(p);
                    } else {
                        void* outs[kP];
                        const void* ins[kP];
                        for (int k = 0; k < kP; ++k) {
                            outs[k] = p.out[k];
                            ins[k] = p.in[k];
                        }
                        if (fmi_dev_scan_peers(FMI_OP_SUM, FMI_F32, FMI_ALG_SCAN, outs, ins, kP, kBytes / 4, s) != FMI_OK) {
                            std::fprintf(stderr, "scan: %s\n", fmi_last_error());
                            std::exit(1);
                        }
                    }
                };
                launch();
                CHECK(hipEventRecord(e0, s));
                for (int k = 0; k < K; ++k) launch();
                CHECK(hipEventRecord(e1, s));
                CHECK(hipEventSynchronize(e1));
                float ms = 0;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                row.us.push_back(ms * 1e3 / K);
            }
        for (auto& row : rows) {
            std::sort(row.us.begin(), row.us.end());
            const double us = row.us[row.us.size() / 2];
            std::printf("{\"draw\": %d, \"kernel\": \"%s\", \"skew\": %zu, \"median_us\": %.2f, \"frac\": %.4f}\n", d,
                        row.kernel, row.skew, us, row.bytes / (us * 1e-6) / 8e12);
        }
        std::fflush(stdout);
        for (char* b : buf) CHECK(hipFree(b));
    }
    for (void* sp : spacers) CHECK(hipFree(sp));
    return 0;
}
