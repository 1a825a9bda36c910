// microbench_scan_lds.hip — VERDICT r03 item 5: one bounded experiment on the write side of C3's peer scan
// (scan_no_order, f32 sum, P = 8 x 64 MiB), the BASELINE kernel furthest below its roofline. Exploration
// harness, not part of the library.
//
// Hypothesis: the scan's 8 output streams are written by every wave of every workgroup in 1 KiB pieces (each
// thread stores its 16 B of all 8 outputs); staging the workgroup's outputs in LDS and letting each wave write
// a longer contiguous run of ONE output bucket (fewer output streams open per CU at a time) could lift the
// write side, which DESIGN §5 locates as the loss. Variants scan8_lds<B, U>: B threads, U lane groups of
// 16 B per thread per peer, so a workgroup's tile is B·U·16 bytes of every bucket; the outputs of all U lane
// groups are evaluated with the library's own program (run_steps / kOut of fmi_kernels.h, the reference's
// scan_no_order bracketing) and written to LDS (8·B·U·16 bytes); after a barrier, wave w stores bucket
// (w·8/waves ...) as contiguous runs of B·U·16 / max(1, waves/8) bytes, with the library's store policy
// (buffer stores, nt sc1). Loads: the library's (buffer, nt).
//
// Protocol (the stop rule's): 8 sets of 16 freshly hipMalloc'd 64 MiB buckets (8 GiB, beyond the 256 MB MALL),
// synthetic f32 inputs; each kernel launched 2 x warm-up then 3 passes over the 8 sets (24 launches) back to
// back between two events; the library's scan (fmi_dev_scan_peers) in the same process, interleaved by
// round. Bits: every variant's 8 outputs of set 0 compared in full with the library's (a mismatch count kernel).
// Run under `rocprofv3 --kernel-trace --stats` for the trace averages the stop rule reads: a variant stays only
// if its trace average falls below 176 µs (>= 0.76 of 8 TB/s).
//
// Build: hipcc -std=c++20 -O3 --offload-arch=gfx950 -ffp-contract=off tools/microbench_scan_lds.hip
//          -Lfmi_amd/lib -lfmi_dev -Wl,-rpath,$PWD/fmi_amd/lib -o build/mbscanlds
// Run:   build/mbscanlds [rounds, default 3]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "../fmi_amd/csrc/fmi_internal.h"

using namespace fmi::dev;
namespace sched = fmi::sched;

#define CHECK(x)                                                                                   \
    do {                                                                                           \
        hipError_t e = (x);                                                                        \
        if (e != hipSuccess) {                                                                     \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            std::exit(1);                                                                          \
        }                                                                                          \
    } while (0)

constexpr int kP = 8;
constexpr int kAlg = sched::kScan;
using L = Lanes<float, 4>;

template <int B, int U>
__global__ void __launch_bounds__(B) scan8_lds(PeerPtrs ptrs) {
    __shared__ L stage[kP * B * U];  // stage[p * B * U + j]: bucket p, lane group j of this tile
    const size_t tile_byte = static_cast<size_t>(blockIdx.x) * B * U * 16;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const unsigned lane_byte = static_cast<unsigned>((u * B + threadIdx.x) * 16);
        L v[kP + kNumSteps<kAlg, kP>];
        load_peers_tile<float, 4, kP>(v, ptrs, tile_byte, lane_byte, std::make_index_sequence<kP>{});
        run_steps<OpSum, float, 4, kAlg, kP>(v, std::make_index_sequence<kNumSteps<kAlg, kP>>{});
        [&]<size_t... R>(std::index_sequence<R...>) {
            ((stage[R * B * U + u * B + threadIdx.x] = v[kOut<kAlg, kP, R>]), ...);
        }(std::make_index_sequence<kP>{});
    }
    __syncthreads();
    constexpr int kWaves = B / 64;
    const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
    if constexpr (kWaves <= kP) {
        // wave w writes buckets w, w + kWaves, ...: each a contiguous run of B·U·16 bytes
        for (int p = wave; p < kP; p += kWaves)
            for (int j = lane; j < B * U; j += 64)
                store_tile<kScanStoreAux, float, 4>(ptrs.out[p], tile_byte, static_cast<unsigned>(j * 16), stage[p * B * U + j]);
    } else {
        // kWaves / kP waves share a bucket, each a contiguous part of its run
        constexpr int per = kWaves / kP;
        const int p = wave / per, part = wave % per;
        constexpr int span = B * U / per;
        for (int j = part * span + lane; j < (part + 1) * span; j += 64)
            store_tile<kScanStoreAux, float, 4>(ptrs.out[p], tile_byte, static_cast<unsigned>(j * 16), stage[p * B * U + j]);
    }
}

__global__ void count_mismatch(const unsigned* a, const unsigned* b, size_t n, unsigned long long* bad) {
    unsigned long long k = 0;
    for (size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += static_cast<size_t>(gridDim.x) * blockDim.x)
        k += a[i] != b[i];
    if (k) atomicAdd(bad, k);
}

struct Kernel {
    std::string name;
    std::function<void(const PeerPtrs&)> launch;
    std::vector<double> us;
};

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 3;
    constexpr int kSets = 8, kPasses = 3;
    constexpr size_t kBytes = size_t(64) << 20, n = kBytes / 4;
    CHECK(hipSetDevice(0));
    if (fmi_dev_init(0) != FMI_OK) {
        std::fprintf(stderr, "fmi_dev_init: %s\n", fmi_last_error());
        return 1;
    }
    hipStream_t s = nullptr;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<void*> bufs;
    std::vector<PeerPtrs> sets(kSets);
    for (int k = 0; k < kSets; ++k)
        for (int p = 0; p < kP; ++p) {
            void *i = nullptr, *o = nullptr;
            CHECK(hipMalloc(&i, kBytes));
            CHECK(hipMalloc(&o, kBytes));
            if (fmi_dev_fill_synthetic(FMI_F32, i, n, 7 + k, p, s) != FMI_OK) return 1;
            sets[k].in[p] = i;
            sets[k].out[p] = o;
            bufs.push_back(i);
            bufs.push_back(o);
        }
    CHECK(hipStreamSynchronize(s));
    auto lib = [&](const PeerPtrs& b) {
        void* outs[kP];
        const void* ins[kP];
        for (int p = 0; p < kP; ++p) {
            outs[p] = b.out[p];
            ins[p] = b.in[p];
        }
        if (fmi_dev_scan_peers(FMI_OP_SUM, FMI_F32, FMI_ALG_SCAN, outs, ins, kP, n, s) != FMI_OK) {
            std::fprintf(stderr, "scan: %s\n", fmi_last_error());
            std::exit(1);
        }
    };
    const size_t nvec = n / 4;
    std::vector<Kernel> ks = {
        {"library_scan", lib, {}},
        {"lds_b256_u1", [&](const PeerPtrs& b) { scan8_lds<256, 1><<<nvec / 256, 256, 0, s>>>(b); }, {}},
        {"lds_b256_u2", [&](const PeerPtrs& b) { scan8_lds<256, 2><<<nvec / 512, 256, 0, s>>>(b); }, {}},
        {"lds_b512_u1", [&](const PeerPtrs& b) { scan8_lds<512, 1><<<nvec / 512, 512, 0, s>>>(b); }, {}},
        {"lds_b512_u2", [&](const PeerPtrs& b) { scan8_lds<512, 2><<<nvec / 1024, 512, 0, s>>>(b); }, {}},
        {"lds_b1024_u1", [&](const PeerPtrs& b) { scan8_lds<1024, 1><<<nvec / 1024, 1024, 0, s>>>(b); }, {}},
    };
    // bits: every variant's outputs of set 0 against the library's, in full
    std::vector<void*> ref(kP);
    for (int p = 0; p < kP; ++p) CHECK(hipMalloc(&ref[p], kBytes));
    unsigned long long* bad = nullptr;
    CHECK(hipMalloc(&bad, sizeof(*bad)));
    lib(sets[0]);
    for (int p = 0; p < kP; ++p) CHECK(hipMemcpyAsync(ref[p], sets[0].out[p], kBytes, hipMemcpyDeviceToDevice, s));
    for (size_t k = 1; k < ks.size(); ++k) {
        for (int p = 0; p < kP; ++p) CHECK(hipMemsetAsync(sets[0].out[p], 0xff, kBytes, s));
        ks[k].launch(sets[0]);
        CHECK(hipGetLastError());
        CHECK(hipMemsetAsync(bad, 0, sizeof(*bad), s));
        for (int p = 0; p < kP; ++p)
            count_mismatch<<<4096, 256, 0, s>>>(static_cast<const unsigned*>(ref[p]), static_cast<const unsigned*>(sets[0].out[p]), n, bad);
        unsigned long long h = 0;
        CHECK(hipMemcpyAsync(&h, bad, sizeof(h), hipMemcpyDeviceToHost, s));
        CHECK(hipStreamSynchronize(s));
        std::printf("{\"kernel\": \"%s\", \"bit_mismatches_vs_library\": %llu, \"elements_compared\": %zu}\n", ks[k].name.c_str(), h,
                    n * kP);
    }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int r = 0; r < rounds; ++r)
        for (auto& kn : ks) {
            kn.launch(sets[6]);
            kn.launch(sets[7]);
            CHECK(hipEventRecord(e0, s));
            for (int i = 0; i < kPasses * kSets; ++i) kn.launch(sets[i % kSets]);
            CHECK(hipEventRecord(e1, s));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            kn.us.push_back(ms * 1e3 / (kPasses * kSets));
        }
    const double bytes = 2.0 * kP * kBytes;
    for (auto& kn : ks) {
        std::sort(kn.us.begin(), kn.us.end());
        const double us = kn.us[kn.us.size() / 2];
        std::printf("{\"kernel\": \"%s\", \"median_of_rounds_us\": %.2f, \"min_us\": %.2f, \"frac\": %.4f, \"launches_per_round\": %d}\n",
                    kn.name.c_str(), us, kn.us.front(), bytes / (us * 1e-6) / 8e12, kPasses * kSets);
    }
    for (void* p : bufs) CHECK(hipFree(p));
    for (void* p : ref) CHECK(hipFree(p));
    CHECK(hipFree(bad));
    return 0;
}
