// microbench_pcie_peers.hip — exploration harness (not part of the library), VERDICT r04 item 1: what ceiling
// does C5's co-resident shape have on one GPU, and how must the copies be issued to reach it? P peers each
// stream a 1 GiB page-locked bucket host -> device and 1 GiB device -> host, in 64 MiB chunks, no compute:
//   own-sdma      every peer has its own H2D and D2H stream (hipMemcpyAsync), as LOCAL ranks' HostPipes do
//   own-sdma-def  the same with hipMemcpyDefault (the kind fmi_comm_allreduce_host passes)
//   shared-sdma   ONE H2D and ONE D2H stream for all peers, chunks in rank-major order
//   own-kernel    every peer copies with a kernel through the bucket's device mapping, on its own two streams
//   shared-kernel the kernel copies on one H2D and one D2H stream for all peers
// Each peer's chunks are issued by its own host thread (as the LOCAL ranks do), except the shared variants,
// which one thread feeds. Wall time from host clocks around issue .. last stream drained; 1 GiB = 2^30 B.
// "streams_before" opens that many idle streams first (where the runtime hands out its DMA engines by stream).
// "busy" (third argument 1): the shared-stream variants again while a third stream keeps HBM busy with device
// copies of 256 MiB (the co-resident ranks' exchange copies and kernels, as fmi_comm_allreduce_host runs them
// beside its DMA): does the link's duplex rate hold when the chip is also streaming HBM?
//
// Build: hipcc -std=c++20 -O3 --offload-arch=gfx950 tools/microbench_pcie_peers.hip -o build/mbpciepeers
// Run:   build/mbpciepeers [rounds, default 3] [streams_before, default 0] [busy, default 0]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <barrier>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#define CHECK(x)                                                                                   \
    do {                                                                                           \
        hipError_t e = (x);                                                                        \
        if (e != hipSuccess) {                                                                     \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            std::exit(1);                                                                          \
        }                                                                                          \
    } while (0)

using u32x4 = unsigned int __attribute__((ext_vector_type(4)));

// dst[i] = src[i] over n16 16-B groups, grid-stride; the HBM side is nontemporal
template <bool H2D>
__global__ void __launch_bounds__(256) copy_k(u32x4* __restrict__ dst, const u32x4* __restrict__ src, size_t n16) {
    for (size_t i = blockIdx.x * size_t(256) + threadIdx.x; i < n16; i += size_t(gridDim.x) * 256) {
        if constexpr (H2D) {
            const u32x4 v = src[i];
            __builtin_nontemporal_store(v, dst + i);
        } else {
            dst[i] = __builtin_nontemporal_load(src + i);
        }
    }
}

constexpr size_t kBytes = size_t(1) << 30;
constexpr size_t kChunk = size_t(64) << 20;

struct Peer {
    char *hsrc = nullptr, *hdst = nullptr;      // page-locked buckets
    char *hsrc_d = nullptr, *hdst_d = nullptr;  // their device mappings
    char *din = nullptr, *dout = nullptr;       // HBM
    hipStream_t h2d = nullptr, d2h = nullptr;
};

static void enqueue(Peer& p, size_t off, bool kernel, hipMemcpyKind hk, hipMemcpyKind dk, hipStream_t sh, hipStream_t sd,
                    int grid) {
    if (kernel) {
        copy_k<true><<<grid, 256, 0, sh>>>(reinterpret_cast<u32x4*>(p.din + off), reinterpret_cast<const u32x4*>(p.hsrc_d + off),
                                           kChunk / 16);
        copy_k<false><<<grid, 256, 0, sd>>>(reinterpret_cast<u32x4*>(p.hdst_d + off), reinterpret_cast<const u32x4*>(p.dout + off),
                                            kChunk / 16);
    } else {
        CHECK(hipMemcpyAsync(p.din + off, p.hsrc + off, kChunk, hk, sh));
        CHECK(hipMemcpyAsync(p.hdst + off, p.dout + off, kChunk, dk, sd));
    }
}

__global__ void __launch_bounds__(256) hbm_copy(u32x4* __restrict__ dst, const u32x4* __restrict__ src, size_t n16) {
    for (size_t i = blockIdx.x * size_t(256) + threadIdx.x; i < n16; i += size_t(gridDim.x) * 256)
        __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 3;
    const int streams_before = argc > 2 ? std::atoi(argv[2]) : 0;
    const bool busy = argc > 3 && std::atoi(argv[3]) != 0;
    std::vector<hipStream_t> idle(streams_before);
    for (auto& s : idle) CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    constexpr int kMaxPeers = 8;
    hipStream_t shared_h2d, shared_d2h;
    CHECK(hipStreamCreateWithFlags(&shared_h2d, hipStreamNonBlocking));
    CHECK(hipStreamCreateWithFlags(&shared_d2h, hipStreamNonBlocking));
    std::vector<Peer> peers(kMaxPeers);
    for (int r = 0; r < kMaxPeers; ++r) {
        Peer& p = peers[r];
        CHECK(hipHostMalloc(reinterpret_cast<void**>(&p.hsrc), kBytes, hipHostMallocDefault));
        CHECK(hipHostMalloc(reinterpret_cast<void**>(&p.hdst), kBytes, hipHostMallocDefault));
        CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&p.hsrc_d), p.hsrc, 0));
        CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&p.hdst_d), p.hdst, 0));
        CHECK(hipMalloc(&p.din, kBytes));
        CHECK(hipMalloc(&p.dout, kBytes));
        for (size_t i = 0; i < kBytes / 8; ++i) reinterpret_cast<uint64_t*>(p.hsrc)[i] = (i + r) * 0x9E3779B97F4A7C15ull;
        CHECK(hipMemcpy(p.dout, p.hsrc, kBytes, hipMemcpyHostToDevice));
        CHECK(hipStreamCreateWithFlags(&p.h2d, hipStreamNonBlocking));
        CHECK(hipStreamCreateWithFlags(&p.d2h, hipStreamNonBlocking));
    }
    CHECK(hipDeviceSynchronize());

    struct V {
        std::string name;
        int peers;
        bool shared, kernel, deflt;
        int grid;
    };
    std::vector<V> vs;
    if (busy) {
        vs.push_back({"shared-sdma+hbm-busy", 8, true, false, false, 0});
        vs.push_back({"shared-sdma", 8, true, false, false, 0});
        vs.push_back({"shared-sdma+hbm-busy", 8, true, false, false, 0});
        vs.push_back({"shared-sdma", 8, true, false, false, 0});
    }
    for (int P : {1, 2, 8}) {
        if (busy) break;
        vs.push_back({"own-sdma", P, false, false, false, 0});
        vs.push_back({"own-sdma-def", P, false, false, true, 0});
        vs.push_back({"shared-sdma", P, true, false, false, 0});
        vs.push_back({"shared-sdma-def", P, true, false, true, 0});
        for (int g : {64, 256}) {
            vs.push_back({"own-kernel", P, false, true, false, P == 1 ? g : std::max(8, g / P)});
            vs.push_back({"shared-kernel", P, true, true, false, g});
        }
    }
    // the busy stream's buffers: 2 x 256 MiB in HBM
    constexpr size_t kBusyBytes = size_t(256) << 20;
    u32x4 *busy_a = nullptr, *busy_b = nullptr;
    hipStream_t busy_s = nullptr;
    if (busy) {
        CHECK(hipMalloc(&busy_a, kBusyBytes));
        CHECK(hipMalloc(&busy_b, kBusyBytes));
        CHECK(hipMemset(busy_a, 1, kBusyBytes));
        CHECK(hipStreamCreateWithFlags(&busy_s, hipStreamNonBlocking));
    }
    for (auto& v : vs) {
        std::vector<double> ms;
        const bool keep_busy = v.name.find("hbm-busy") != std::string::npos;
        for (int rep = 0; rep < rounds + 1; ++rep) {
            CHECK(hipDeviceSynchronize());
            const hipMemcpyKind hk = v.deflt ? hipMemcpyDefault : hipMemcpyHostToDevice;
            const hipMemcpyKind dk = v.deflt ? hipMemcpyDefault : hipMemcpyDeviceToHost;
            std::atomic<bool> stop{false};
            std::thread feeder;
            if (keep_busy)  // keep 2 copies queued at a time until the DMA is done (~0.1 ms each)
                feeder = std::thread([&] {
                    hipEvent_t done[2];
                    for (auto& ev : done) CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
                    for (int k = 0; !stop.load(); ++k) {
                        if (k >= 2) CHECK(hipEventSynchronize(done[k & 1]));
                        hbm_copy<<<2048, 256, 0, busy_s>>>(busy_b, busy_a, kBusyBytes / 16);
                        CHECK(hipEventRecord(done[k & 1], busy_s));
                    }
                    CHECK(hipStreamSynchronize(busy_s));
                    for (auto& ev : done) CHECK(hipEventDestroy(ev));
                });
            const auto t0 = std::chrono::steady_clock::now();
            if (v.shared) {
                for (size_t off = 0; off < kBytes; off += kChunk)
                    for (int r = 0; r < v.peers; ++r) enqueue(peers[r], off, v.kernel, hk, dk, shared_h2d, shared_d2h, v.grid);
                CHECK(hipStreamSynchronize(shared_h2d));
                CHECK(hipStreamSynchronize(shared_d2h));
            } else {
                std::barrier go(v.peers);
                std::vector<std::thread> th;
                for (int r = 0; r < v.peers; ++r)
                    th.emplace_back([&, r] {
                        Peer& p = peers[r];
                        go.arrive_and_wait();
                        for (size_t off = 0; off < kBytes; off += kChunk) enqueue(p, off, v.kernel, hk, dk, p.h2d, p.d2h, v.grid);
                        CHECK(hipStreamSynchronize(p.h2d));
                        CHECK(hipStreamSynchronize(p.d2h));
                    });
                for (auto& t : th) t.join();
            }
            const double t = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            stop.store(true);
            if (feeder.joinable()) feeder.join();
            if (rep > 0) ms.push_back(t);  // the first is a warm-up
        }
        // byte-exact: every peer's device copy of its source, and its host copy of the device bucket
        bool ok = true;
        std::vector<char> back(kChunk);
        for (int r = 0; r < v.peers && ok; ++r) {
            CHECK(hipMemcpy(back.data(), peers[r].din + kBytes - kChunk, kChunk, hipMemcpyDeviceToHost));
            ok = std::memcmp(back.data(), peers[r].hsrc + kBytes - kChunk, kChunk) == 0 &&
                 std::memcmp(peers[r].hdst, peers[r].hsrc, kChunk) == 0;
        }
        std::sort(ms.begin(), ms.end());
        const double med = ms[ms.size() / 2];
        std::printf("{\"variant\": \"%s\", \"peers\": %d, \"grid\": %d, \"streams_before\": %d, \"median_ms\": %.2f, \"min_ms\": %.2f, "
                    "\"pcie_GB_s_both_directions\": %.1f, \"bytes_ok\": %s}\n",
                    v.name.c_str(), v.peers, v.grid, streams_before, med, ms.front(), 2.0 * v.peers * kBytes / (med * 1e-3) / 1e9,
                    ok ? "true" : "false");
        std::fflush(stdout);
        for (int r = 0; r < v.peers; ++r) std::memset(peers[r].hdst, 0, kChunk);
    }
    return 0;
}
