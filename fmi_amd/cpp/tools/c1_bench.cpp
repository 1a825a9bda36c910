// c1_bench.cpp — BASELINE.json config C1 on the host: a 2-peer float32 sum-allreduce of 1 MiB buckets
// through FMI::Communicator, the two peers as fork()ed processes over a socketpair channel (LocalSocket),
// the stand-in for the reference's TCPunch Direct channel (tests/communicator.cpp:145-192 with
// config/fmi_test.json; the rendezvous server it needs is not available).
//
// Two combine paths, same transport and algorithm (recursive doubling, reference
// src/comm/PeerToPeer.cpp:96-130):
//   lambda    an untagged Function<std::vector<float>> lambda: the reference adapter
//             (include/Communicator.h:180-189 — copies both buckets into vectors, calls by value, memcpy back)
//   builtin   Function<std::vector<float>>(Op::sum): the same combine in place, no copies, each transfer
//             then its combine
//   overlap   the built-in op with the transfer cut into --overlap-chunk pieces, piece k combined while
//             piece k+1 moves (PeerToPeer::set_overlap_chunk; identical bits)
//
//   c1_bench [--mib M] [--reps K] [--peers P] [--overlap-chunk BYTES] [--device D]
//            one JSON line (peer 0): median ms per allreduce and bucket GiB/s per path. --device D runs
//            the built-in combines of the host buckets on GPU D (Communicator::use_device: each combine,
//            or each piece of an overlapped one, is fmi_host_reduce_pair)
#include <sys/mman.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "fmi/fmi.h"

using FMI::Communicator;
using FMI::Comm::Data;
using FMI::Utils::Function;
using FMI::Utils::peer_num;

namespace {

double median(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

// One peer's run: K timed allreduces per path, each bracketed by barriers; returns median ms per path.
void run_peer(std::vector<int> fds, peer_num p, peer_num P, size_t n, int reps, size_t chunk, int device,
              double* out) {
    Communicator comm(p, P, "", "c1");
    if (device >= 0) comm.use_device(device, true);  // every combine on the GPU, whatever the crossover
    auto channel = std::make_shared<FMI::Comm::LocalSocket>(std::move(fds), 60000);
    comm.register_channel("Local", channel);
    std::vector<float> init(n);
    for (size_t i = 0; i < n; ++i) init[i] = static_cast<float>((i * 2654435761u + p) % 1000) * 0.001f;
    Function<std::vector<float>> lambda(
        [](std::vector<float> a, std::vector<float> b) {
            for (size_t i = 0; i < a.size(); ++i) a[i] += b[i];
            return a;
        },
        true, true);
    Function<std::vector<float>> builtin(FMI::Utils::Op::sum);
    std::vector<float> result[3];
    for (int path = 0; path < 3; ++path) {
        channel->set_overlap_chunk(path == 2 ? chunk : 0);
        std::vector<double> ms;
        for (int k = 0; k < reps + 1; ++k) {
            Data<std::vector<float>> send(init), recv{std::vector<float>(n)};
            comm.barrier();
            const auto t0 = std::chrono::steady_clock::now();
            comm.allreduce(send, recv, path == 0 ? lambda : builtin);
            comm.barrier();
            const auto t1 = std::chrono::steady_clock::now();
            if (k) ms.push_back(std::chrono::duration<double, std::milli>(t1 - t0).count());
            if (k == reps) result[path] = recv.get();
        }
        out[path] = median(ms);
    }
    // the three paths evaluate the same bracketing: identical bits
    out[3] = std::memcmp(result[1].data(), result[2].data(), n * sizeof(float)) == 0 &&
             std::memcmp(result[0].data(), result[1].data(), n * sizeof(float)) == 0;
}

}  // namespace

int main(int argc, char** argv) {
    size_t mib = 1;
    int reps = 21;
    peer_num P = 2;
    size_t chunk = 2u << 20;
    int device = -1;
    for (int i = 1; i + 1 < argc; i += 2) {
        const std::string k = argv[i];
        if (k == "--mib") mib = std::strtoull(argv[i + 1], nullptr, 10);
        else if (k == "--reps") reps = std::atoi(argv[i + 1]);
        else if (k == "--peers") P = static_cast<peer_num>(std::atoi(argv[i + 1]));
        else if (k == "--overlap-chunk") chunk = std::strtoull(argv[i + 1], nullptr, 10);
        else if (k == "--device") device = std::atoi(argv[i + 1]);
    }
    const size_t n = mib * (1u << 20) / sizeof(float);
    auto* res = static_cast<double*>(
        mmap(nullptr, 4 * P * sizeof(double), PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0));
    FMI::Comm::SocketMesh mesh(P);
    std::vector<pid_t> kids;
    for (peer_num p = 1; p < P; ++p) {
        const pid_t pid = fork();
        if (pid == 0) {
            try {
                run_peer(mesh.claim(p), p, P, n, reps, chunk, device, res + 4 * p);
            } catch (const std::exception& e) {
                std::fprintf(stderr, "peer %u: %s\n", p, e.what());
                _exit(1);
            }
            _exit(0);
        }
        kids.push_back(pid);
    }
    int rc = 0;
    try {
        run_peer(mesh.claim(0), 0, P, n, reps, chunk, device, res);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "peer 0: %s\n", e.what());
        rc = 1;
    }
    for (pid_t k : kids) {
        int status = 0;
        waitpid(k, &status, 0);
        if (!WIFEXITED(status) || WEXITSTATUS(status) != 0) rc = 1;
    }
    if (rc) return rc;
    double lam = 0, bi = 0, ov = 0;  // max over peers
    bool same = true;
    for (peer_num p = 0; p < P; ++p) {
        lam = std::max(lam, res[4 * p]);
        bi = std::max(bi, res[4 * p + 1]);
        ov = std::max(ov, res[4 * p + 2]);
        same = same && res[4 * p + 3] == 1.0;
    }
    const double gib = static_cast<double>(n * sizeof(float)) / (1u << 30);
    std::printf("{\"config\": \"C1\", \"peers\": %u, \"bucket_mib\": %zu, \"reps\": %d, \"combine_on\": \"%s\", \"transport\": "
                "\"fork + socketpair (LocalSocket)\", \"lambda_adapter_ms\": %.4f, \"builtin_inplace_ms\": %.4f, "
                "\"builtin_overlap_ms\": %.4f, \"overlap_chunk_bytes\": %zu, \"lambda_adapter_gib_s\": %.4f, "
                "\"builtin_inplace_gib_s\": %.4f, \"builtin_overlap_gib_s\": %.4f, \"paths_bit_identical\": %s}\n",
                P, mib, reps, device >= 0 ? "gpu (fmi_host_reduce_pair)" : "host", lam, bi, ov, chunk, gib / (lam * 1e-3), gib / (bi * 1e-3), gib / (ov * 1e-3),
                same ? "true" : "false");
    return 0;
}
