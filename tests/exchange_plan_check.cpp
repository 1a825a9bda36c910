// Host check of the communicator's exchange plans (fmi_amd/csrc/fmi_exchange_plan.h), built and run by
// tests/test_exchange_plan.py. For every plan, N ranks and a set of sizes, it simulates the exchange on
// tagged host buffers exactly as RCCL pairs a group's point-to-point calls (per ordered pair of ranks, the
// k-th send matches the k-th receive) and checks:
//   - pairing: per ordered pair, as many sends as receives, of equal lengths (else RCCL would hang);
//   - bounds: every transfer and the local copy stay inside the buffers the collective defines;
//   - no receive region is written twice;
//   - the result: every byte of every receive buffer holds what the exchange's definition says, and
//     bytes the exchange must not touch keep their sentinel.
// Prints one summary line and exits 0, or prints the first failure and exits 1.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "fmi_exchange_plan.h"

using fmi::plan::Plan;
using fmi::plan::span;
using fmi::plan::Xfer;

namespace {

constexpr uint64_t kSentinel = ~uint64_t(0);
uint64_t tag(int rank, size_t byte) { return (uint64_t(rank) << 40) | byte; }

struct Case {
    std::string name;
    int n;
    std::function<Plan(int)> plan;                 // plan of rank r
    std::function<size_t(int)> send_len, recv_len;  // buffer sizes of rank r (bytes)
    // expected source of recv byte b at rank r: {rank, byte} or {-1, 0} = untouched
    std::function<std::pair<int, size_t>(int, size_t)> expect;
};

long g_cases = 0, g_xfers = 0;

bool fail(const Case& c, const std::string& what) {
    std::printf("FAIL %s N=%d: %s\n", c.name.c_str(), c.n, what.c_str());
    return false;
}

bool run(const Case& c) {
    const int N = c.n;
    std::vector<Plan> plans(N);
    for (int r = 0; r < N; ++r) plans[r] = c.plan(r);
    std::vector<std::vector<uint64_t>> send(N), recv(N);
    for (int r = 0; r < N; ++r) {
        send[r].resize(c.send_len(r));
        for (size_t b = 0; b < send[r].size(); ++b) send[r][b] = tag(r, b);
        recv[r].assign(c.recv_len(r), kSentinel);
    }
    std::vector<std::vector<char>> written(N);
    for (int r = 0; r < N; ++r) written[r].assign(recv[r].size(), 0);
    auto write = [&](int r, size_t off, const uint64_t* src, size_t len) -> bool {
        if (off + len > recv[r].size()) return fail(c, "rank " + std::to_string(r) + " writes past its receive buffer");
        for (size_t t = 0; t < len; ++t) {
            if (written[r][off + t]) return fail(c, "rank " + std::to_string(r) + " receives byte " + std::to_string(off + t) + " twice");
            written[r][off + t] = 1;
            recv[r][off + t] = src[t];
        }
        return true;
    };
    for (int i = 0; i < N; ++i) {
        for (const Xfer& x : plans[i].sends)
            if (x.peer < 0 || x.peer >= N || x.len == 0 || x.off + x.len > send[i].size())
                return fail(c, "rank " + std::to_string(i) + " posts a send out of range");
        for (const Xfer& x : plans[i].recvs)
            if (x.peer < 0 || x.peer >= N || x.len == 0) return fail(c, "rank " + std::to_string(i) + " posts a bad receive");
    }
    // pair every ordered (i -> j): k-th send of i to j with k-th receive of j from i
    std::vector<std::vector<std::vector<Xfer>>> sends_to(N, std::vector<std::vector<Xfer>>(N)), recvs_from = sends_to;
    for (int i = 0; i < N; ++i) {
        for (const Xfer& x : plans[i].sends) sends_to[i][x.peer].push_back(x);
        for (const Xfer& x : plans[i].recvs) recvs_from[i][x.peer].push_back(x);
    }
    for (int i = 0; i < N; ++i) {
        for (int j = 0; j < N; ++j) {
            const std::vector<Xfer>& s = sends_to[i][j];
            const std::vector<Xfer>& r = recvs_from[j][i];
            if (s.size() != r.size())
                return fail(c, std::to_string(i) + " -> " + std::to_string(j) + ": " + std::to_string(s.size()) + " sends, " +
                                   std::to_string(r.size()) + " receives");
            for (size_t k = 0; k < s.size(); ++k) {
                if (s[k].len != r[k].len)
                    return fail(c, std::to_string(i) + " -> " + std::to_string(j) + ": send of " + std::to_string(s[k].len) +
                                       " B meets a receive of " + std::to_string(r[k].len) + " B");
                if (!write(j, r[k].off, send[i].data() + s[k].off, s[k].len)) return false;
                ++g_xfers;
            }
        }
    }
    for (int r = 0; r < N; ++r) {
        const Plan& p = plans[r];
        if (!p.copy_len) continue;
        if (p.copy_src + p.copy_len > send[r].size()) return fail(c, "local copy reads past the send buffer");
        if (!write(r, p.copy_dst, send[r].data() + p.copy_src, p.copy_len)) return false;
    }
    for (int r = 0; r < N; ++r) {
        for (size_t b = 0; b < recv[r].size(); ++b) {
            const auto [src, sb] = c.expect(r, b);
            const uint64_t want = src < 0 ? kSentinel : tag(src, sb);
            if (recv[r][b] != want)
                return fail(c, "rank " + std::to_string(r) + " byte " + std::to_string(b) + ": got rank " +
                                   std::to_string(recv[r][b] >> 40) + " byte " + std::to_string(recv[r][b] & ((uint64_t(1) << 40) - 1)) +
                                   (src < 0 ? ", want untouched" : ", want rank " + std::to_string(src) + " byte " + std::to_string(sb)));
        }
    }
    ++g_cases;
    return true;
}

bool check_all(int N, size_t unit) {
    using P = std::pair<int, size_t>;
    const P none{-1, 0};
    // fixed-size exchanges, `unit` bytes per block
    const size_t B = unit;
    if (!run({"all_to_all", N, [=](int r) { return fmi::plan::all_to_all(N, r, B); },
              [=](int) { return N * B; }, [=](int) { return N * B; },
              [=](int r, size_t b) { return P{int(b / B), r * B + b % B}; }}))
        return false;
    // the shard kernel's receive at a stride (each shard in its own 4 KiB slot): the gap bytes stay untouched
    for (size_t gap : {size_t(1), size_t(5)}) {
        const size_t S = B + gap;
        if (!run({"all_to_all stride +" + std::to_string(gap), N, [=](int r) { return fmi::plan::all_to_all(N, r, B, S); },
                  [=](int) { return N * B; }, [=](int) { return N * S; },
                  [=](int r, size_t b) { return b % S < B ? P{int(b / S), r * B + b % S} : none; }}))
            return false;
    }
    if (!run({"all_gather", N, [=](int r) { return fmi::plan::all_gather(N, r, B); }, [=](int) { return B; },
              [=](int) { return N * B; }, [=](int, size_t b) { return P{int(b / B), b % B}; }}))
        return false;
    for (int root : {0, N / 2, N - 1}) {
        if (!run({"gather root " + std::to_string(root), N, [=](int r) { return fmi::plan::gather(N, r, B, root); },
                  [=](int) { return B; }, [=](int r) { return r == root ? N * B : 0; },
                  [=](int, size_t b) { return P{int(b / B), b % B}; }}))
            return false;
        if (!run({"scatter root " + std::to_string(root), N, [=](int r) { return fmi::plan::scatter(N, r, B, root); },
                  [=](int r) { return r == root ? N * B : 0; }, [=](int) { return B; },
                  [=](int r, size_t b) { return P{root, r * B + b}; }}))
            return false;
    }
    // ragged exchanges: shard bytes and totals that leave the last shards short, empty, or exact
    const size_t shard = unit;
    std::vector<size_t> totals = {0, 1, shard - 1, shard, shard + 1, N * shard, N * shard - 1, (N - 1) * shard + 1,
                                  N * shard / 2 + 3};
    for (size_t total : totals) {
        if (total > N * shard) continue;
        const std::string t = " total " + std::to_string(total);
        if (!run({"all_to_all_ragged" + t, N, [=](int r) { return fmi::plan::all_to_all_ragged(N, r, shard, total); },
                  [=](int) { return total; }, [=](int) { return N * shard; },
                  [=](int r, size_t b) {
                      const int j = int(b / shard);
                      return b % shard < span(r, shard, total) ? P{j, r * shard + b % shard} : none;
                  }}))
            return false;
        if (!run({"all_gather_ragged" + t, N, [=](int r) { return fmi::plan::all_gather_ragged(N, r, shard, total); },
                  [=](int r) { return span(r, shard, total); }, [=](int) { return total; },
                  [=](int, size_t b) {
                      const int j = int(b / shard);
                      return b < total ? P{j, b % shard} : none;
                  }}))
            return false;
        for (int root : {0, N - 1}) {
            if (!run({"gather_ragged root " + std::to_string(root) + t, N,
                      [=](int r) { return fmi::plan::gather_ragged(N, r, shard, total, root); },
                      [=](int r) { return span(r, shard, total); }, [=](int r) { return r == root ? total : 0; },
                      [=](int, size_t b) { return b < total ? P{int(b / shard), b % shard} : none; }}))
                return false;
        }
        if (!run({"all_to_all_back_ragged" + t, N,
                  [=](int r) { return fmi::plan::all_to_all_back_ragged(N, r, shard, total); },
                  [=](int) { return N * shard; }, [=](int) { return total; },
                  [=](int r, size_t b) {
                      const int j = int(b / shard);
                      return b % shard < span(j, shard, total) ? P{j, r * shard + b % shard} : none;
                  }}))
            return false;
    }
    return true;
}

}  // namespace

int main(int argc, char** argv) {
    const int max_n = argc > 1 ? std::atoi(argv[1]) : 40;
    std::vector<int> ns;
    for (int n = 1; n <= max_n; ++n) ns.push_back(n);
    for (int n : {64, 100, 257})
        if (n > max_n) ns.push_back(n);
    for (int n : ns)
        for (size_t unit : {size_t(1), size_t(7), size_t(64)})
            if (!check_all(n, unit)) return 1;
    std::printf("ok: %ld exchanges, %ld matched transfers, N = 1..%d, 64, 100, 257\n", g_cases, g_xfers, max_n);
    return 0;
}
