// ipc_probe.hip — exploration harness (not part of the library): does cross-process HIP IPC work on this
// platform the way path DIRECT uses it? Two processes (forked before either touches HIP) on one GPU:
// the owner allocates a bucket, fills it, exports hipIpcGetMemHandle and passes the handle over a pipe;
// the peer opens it with hipIpcMemLazyEnablePeerAccess (the flag fmi_comm's map_window uses), reads it
// with a kernel into its own memory, and reports whether every element matched. The owner keeps the
// allocation alive until the peer has closed the mapping.
//
// Build: hipcc -std=c++20 -O3 --offload-arch=gfx950 tools/ipc_probe.hip -o build/ipc_probe
#include <hip/hip_runtime.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                                    \
    do {                                                                                            \
        hipError_t e = (x);                                                                         \
        if (e != hipSuccess) {                                                                      \
            std::fprintf(stderr, "[%d] %s:%d %s: %s\n", getpid(), __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            std::_Exit(1);                                                                          \
        }                                                                                           \
    } while (0)

__global__ void fill(unsigned* p, size_t n) {
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
        p[i] = static_cast<unsigned>(i * 2654435761u);
}

__global__ void copy(unsigned* dst, const unsigned* src, size_t n) {
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
        dst[i] = src[i];
}

int main() {
    const size_t n = (64u << 20) / 4;
    int to_peer[2], to_owner[2];
    if (pipe(to_peer) || pipe(to_owner)) return 1;
    const pid_t pid = fork();
    if (pid == 0) {  // peer
        hipIpcMemHandle_t h;
        if (read(to_peer[0], &h, sizeof(h)) != sizeof(h)) std::_Exit(1);
        CHECK(hipSetDevice(0));
        void* remote = nullptr;
        CHECK(hipIpcOpenMemHandle(&remote, h, hipIpcMemLazyEnablePeerAccess));
        unsigned* mine = nullptr;
        CHECK(hipMalloc(&mine, n * 4));
        copy<<<4096, 256>>>(mine, static_cast<const unsigned*>(remote), n);
        CHECK(hipDeviceSynchronize());
        std::vector<unsigned> host(n);
        CHECK(hipMemcpy(host.data(), mine, n * 4, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (size_t i = 0; i < n; ++i) bad += host[i] != static_cast<unsigned>(i * 2654435761u);
        CHECK(hipIpcCloseMemHandle(remote));
        CHECK(hipFree(mine));
        const int ok = bad == 0;
        if (write(to_owner[1], &ok, sizeof(ok)) != sizeof(ok)) std::_Exit(1);
        std::printf("{\"role\": \"peer\", \"opened\": true, \"mismatches\": %zu}\n", bad);
        std::fflush(stdout);
        std::_Exit(ok ? 0 : 2);
    }
    // owner
    CHECK(hipSetDevice(0));
    unsigned* buf = nullptr;
    CHECK(hipMalloc(&buf, n * 4));
    fill<<<4096, 256>>>(buf, n);
    CHECK(hipDeviceSynchronize());
    hipIpcMemHandle_t h;
    CHECK(hipIpcGetMemHandle(&h, buf));
    if (write(to_peer[1], &h, sizeof(h)) != sizeof(h)) return 1;
    int ok = 0;
    if (read(to_owner[0], &ok, sizeof(ok)) != sizeof(ok)) ok = 0;
    int status = 0;
    waitpid(pid, &status, 0);
    CHECK(hipFree(buf));
    std::printf("{\"role\": \"owner\", \"peer_ok\": %s, \"peer_exit\": %d}\n", ok ? "true" : "false",
                WIFEXITED(status) ? WEXITSTATUS(status) : -1);
    return ok ? 0 : 1;
}
