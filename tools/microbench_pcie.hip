// microbench_pcie.hip — exploration harness (not part of the library): can config C5's host path (a 1 GiB
// page-locked bucket in, the reduced bucket out) move more than the 91 GB/s both directions
// that fmi_comm_allreduce_host reaches with hipMemcpyAsync (SDMA) copies? Each direction alone runs at
// ~57 GB/s (1 GiB in 18.8 ms); together only ~46 GB/s each. Here, 1 GiB each way:
//   sdma      hipMemcpyAsync (the runtime's DMA engines), one stream per direction, or split in P streams
//   kernel    a copy kernel on G workgroups reading (H2D) or writing (D2H) the page-locked host bucket through
//             its device mapping, 16 B per lane, nontemporal on the device side
// alone and with the other direction concurrent, in every combination. Wall time per variant from events
// on a common start / end (max over the streams); the copies are checked byte-exact once.
//
// Build: hipcc -std=c++20 -O3 --offload-arch=gfx950 tools/microbench_pcie.hip -o build/mbpcie
// Run:   build/mbpcie [rounds, default 5]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
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

// dst[i] = src[i] over n16 16-B groups, grid-stride; DEV_DST: the device side is the destination (H2D)
template <bool H2D>
__global__ void __launch_bounds__(256) copy_k(u32x4* dst, const u32x4* src, size_t n16) {
    for (size_t i = blockIdx.x * size_t(256) + threadIdx.x; i < n16; i += size_t(gridDim.x) * 256) {
        if constexpr (H2D) {
            const u32x4 v = src[i];                   // host memory over PCIe
            __builtin_nontemporal_store(v, dst + i);  // HBM
        } else {
            const u32x4 v = __builtin_nontemporal_load(src + i);
            dst[i] = v;
        }
    }
}

struct Variant {
    std::string name;
    std::function<void()> run;  // enqueue on the streams (after the start event, before the end events)
    double bytes;               // PCIe bytes moved (both directions)
    std::vector<double> ms;
};

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 5;
    const size_t bytes = size_t(1) << 30, n16 = bytes / 16;
    void *hsrc = nullptr, *hdst = nullptr, *dA = nullptr, *dB = nullptr;
    CHECK(hipHostMalloc(&hsrc, bytes, hipHostMallocDefault));
    CHECK(hipHostMalloc(&hdst, bytes, hipHostMallocDefault));
    CHECK(hipMalloc(&dA, bytes));
    CHECK(hipMalloc(&dB, bytes));
    void *hsrc_d = nullptr, *hdst_d = nullptr;
    CHECK(hipHostGetDevicePointer(&hsrc_d, hsrc, 0));
    CHECK(hipHostGetDevicePointer(&hdst_d, hdst, 0));
    for (size_t i = 0; i < bytes / 8; ++i) static_cast<uint64_t*>(hsrc)[i] = i * 0x9E3779B97F4A7C15ull;
    CHECK(hipMemcpy(dB, hsrc, bytes, hipMemcpyHostToDevice));
    constexpr int S = 8;
    hipStream_t st[S];
    for (auto& s : st) CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t start, ends[S];
    CHECK(hipEventCreate(&start));
    for (auto& ev : ends) CHECK(hipEventCreate(&ev));

    auto sdma = [&](int first_stream, int parts, bool h2d) {
        const size_t part = bytes / parts;
        for (int p = 0; p < parts; ++p) {
            char* d = static_cast<char*>(h2d ? dA : hdst) + p * part;
            const char* s = static_cast<const char*>(h2d ? hsrc : dB) + p * part;
            CHECK(hipMemcpyAsync(d, s, part, h2d ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost, st[first_stream + p]));
        }
    };
    auto kern = [&](int stream, int grid, bool h2d) {
        if (h2d)
            copy_k<true><<<grid, 256, 0, st[stream]>>>(static_cast<u32x4*>(dA), static_cast<const u32x4*>(hsrc_d), n16);
        else
            copy_k<false><<<grid, 256, 0, st[stream]>>>(static_cast<u32x4*>(hdst_d), static_cast<const u32x4*>(dB), n16);
    };
    std::vector<Variant> vs;
    const double one = double(bytes), two = 2.0 * bytes;
    vs.push_back({"h2d sdma", [&] { sdma(0, 1, true); }, one, {}});
    vs.push_back({"d2h sdma", [&] { sdma(0, 1, false); }, one, {}});
    vs.push_back({"both sdma", [&] { sdma(0, 1, true); sdma(1, 1, false); }, two, {}});
    vs.push_back({"both sdma 2+2 streams", [&] { sdma(0, 2, true); sdma(2, 2, false); }, two, {}});
    vs.push_back({"both sdma 4+4 streams", [&] { sdma(0, 4, true); sdma(4, 4, false); }, two, {}});
    for (int g : {32, 64, 128, 256, 512}) {
        vs.push_back({"h2d kernel g" + std::to_string(g), [&, g] { kern(0, g, true); }, one, {}});
        vs.push_back({"d2h kernel g" + std::to_string(g), [&, g] { kern(0, g, false); }, one, {}});
        vs.push_back({"both kernel g" + std::to_string(g), [&, g] { kern(0, g, true); kern(1, g, false); }, two, {}});
        vs.push_back({"h2d kernel g" + std::to_string(g) + " + d2h sdma", [&, g] { kern(0, g, true); sdma(1, 1, false); }, two, {}});
        vs.push_back({"h2d sdma + d2h kernel g" + std::to_string(g), [&, g] { sdma(0, 1, true); kern(1, g, false); }, two, {}});
    }
    // byte-exact once: kernel H2D, kernel D2H
    kern(0, 256, true);
    CHECK(hipStreamSynchronize(st[0]));
    CHECK(hipMemcpy(hdst, dA, bytes, hipMemcpyDeviceToHost));
    if (std::memcmp(hdst, hsrc, bytes) != 0) {
        std::printf("{\"error\": \"kernel H2D copy differs\"}\n");
        return 1;
    }
    std::memset(hdst, 0, bytes);
    kern(0, 256, false);
    CHECK(hipStreamSynchronize(st[0]));
    if (std::memcmp(hdst, hsrc, bytes) != 0) {
        std::printf("{\"error\": \"kernel D2H copy differs\"}\n");
        return 1;
    }
    for (int r = 0; r < rounds; ++r)
        for (auto& v : vs) {
            CHECK(hipDeviceSynchronize());
            CHECK(hipEventRecord(start, st[0]));
            for (int s = 1; s < S; ++s) CHECK(hipStreamWaitEvent(st[s], start, 0));
            v.run();
            for (int s = 0; s < S; ++s) CHECK(hipEventRecord(ends[s], st[s]));
            CHECK(hipDeviceSynchronize());
            float worst = 0;
            for (int s = 0; s < S; ++s) {
                float ms = 0;
                CHECK(hipEventElapsedTime(&ms, start, ends[s]));
                worst = std::max(worst, ms);
            }
            v.ms.push_back(worst);
        }
    for (auto& v : vs) {
        std::sort(v.ms.begin(), v.ms.end());
        const double ms = v.ms[v.ms.size() / 2];
        std::printf("{\"variant\": \"%s\", \"median_ms\": %.3f, \"min_ms\": %.3f, \"pcie_GB_s\": %.1f}\n", v.name.c_str(),
                    ms, v.ms.front(), v.bytes / (ms * 1e-3) / 1e9);
    }
    return 0;
}
