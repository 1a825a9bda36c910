// Tests of the C++ FMI surface (fmi_amd/cpp/include/fmi), modelled on the reference's Boost suites
// tests/communicator.cpp and tests/channels.cpp: the same known answers, peers as threads over Loopback
// or as fork()ed processes over LocalSocket (results returned through MAP_SHARED memory, as the
// reference does), plus order, error and device tests. Run by tests/test_cpp_communicator.py.
//
//   test_communicator [--gpu] [name-filter]      run the suite (device tests only with --gpu)
//   test_communicator --proc-channel P           device collectives over the Rccl channel with the PROC
//        transport, P fork()ed peers on GPU 0, against the same collectives on host buckets
//   test_communicator --dump KIND P N OUT [--device|--offload]
//   test_communicator --dump-move bcast|gather|scatter P N ROOT OUT
//        run KIND (allreduce|reduce|scan|reduce_ltr|allreduce_ltr|scan_ltr) over P peers holding
//        synthetic f32 buckets of N elements (seed 42, peer p) and write every peer's recvbuf, then every
//        peer's sendbuf, as raw f32 to OUT — compared against the oracle by the Python wrapper.
#include <sys/mman.h>
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <functional>
#include <iostream>
#include <string>
#include <thread>
#include <vector>

#include "fmi/fmi.h"

using FMI::Communicator;
using FMI::Comm::Data;
using FMI::Utils::Function;
using FMI::Utils::Op;
using FMI::Utils::peer_num;
namespace Dev = FMI::Dev;

// ---- minimal harness ---------------------------------------------------------------------------------
struct TestCase {
    std::string name;
    bool gpu;
    std::function<void()> body;
};
static std::vector<TestCase>& registry() {
    static std::vector<TestCase> r;
    return r;
}
static std::atomic<int> g_failures{0};
struct Register {
    Register(const char* n, bool gpu, std::function<void()> f) { registry().push_back({n, gpu, std::move(f)}); }
};
#define TEST(name) \
    static void name(); \
    static Register reg_##name(#name, false, name); \
    static void name()
#define GPU_TEST(name) \
    static void name(); \
    static Register reg_##name(#name, true, name); \
    static void name()
#define CHECK(cond)                                                                                   \
    do {                                                                                              \
        if (!(cond)) {                                                                                \
            ++g_failures;                                                                             \
            std::fprintf(stderr, "  CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond);            \
        }                                                                                             \
    } while (0)
#define CHECK_THROWS(expr, Type)                     \
    do {                                             \
        bool thrown_ = false;                        \
        try {                                        \
            expr;                                    \
        } catch (const Type&) {                      \
            thrown_ = true;                          \
        }                                            \
        CHECK(thrown_ && "expected " #Type);         \
    } while (0)

// Run body(comm) for P peers as threads sharing one Loopback mailbox.
template <class Body>
static void with_peers(peer_num P, Body body, std::chrono::milliseconds timeout = std::chrono::seconds(60)) {
    auto mailbox = std::make_shared<FMI::Comm::Mailbox>();
    std::vector<std::thread> threads;
    std::vector<std::string> errors(P);
    for (peer_num p = 0; p < P; ++p)
        threads.emplace_back([&, p] {
            try {
                Communicator comm(p, P, "", "test");
                comm.register_channel("Loopback", std::make_shared<FMI::Comm::Loopback>(mailbox, timeout));
                body(comm, p);
            } catch (const std::exception& e) {
                errors[p] = e.what();
            }
        });
    for (auto& t : threads) t.join();
    for (peer_num p = 0; p < P; ++p)
        if (!errors[p].empty()) {
            ++g_failures;
            std::fprintf(stderr, "  peer %u threw: %s\n", p, errors[p].c_str());
        }
}

// Run body(channel, peer) in P fork()ed processes over LocalSocket; results go through `shared`.
template <class Body>
static void with_processes(peer_num P, Body body) {
    FMI::Comm::SocketMesh mesh(P);
    std::vector<pid_t> kids;
    for (peer_num p = 1; p < P; ++p) {
        pid_t pid = fork();
        if (pid == 0) {
            int rc = 0;
            try {
                auto ch = std::make_shared<FMI::Comm::LocalSocket>(mesh.claim(p), 30000);
                ch->set_peer_id(p);
                ch->set_num_peers(P);
                body(*ch, p);
                ch->finalize();
            } catch (const std::exception& e) {
                std::fprintf(stderr, "  child %u threw: %s\n", p, e.what());
                rc = 1;
            }
            _exit(rc);
        }
        kids.push_back(pid);
    }
    try {
        auto ch = std::make_shared<FMI::Comm::LocalSocket>(mesh.claim(0), 30000);
        ch->set_peer_id(0);
        ch->set_num_peers(P);
        body(*ch, 0);
        ch->finalize();
    } catch (const std::exception& e) {
        ++g_failures;
        std::fprintf(stderr, "  peer 0 threw: %s\n", e.what());
    }
    for (pid_t k : kids) {
        int status = 0;
        waitpid(k, &status, 0);
        if (!WIFEXITED(status) || WEXITSTATUS(status) != 0) ++g_failures;
    }
}

template <class T>
static T* shared_array(std::size_t n) {
    void* p = mmap(nullptr, n * sizeof(T), PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    return static_cast<T*>(p);
}

// ---- reference tests/communicator.cpp known answers (P = 4) ---------------------------------------------
TEST(sending_receiving) {  // tests/communicator.cpp:12-33
    with_peers(2, [](Communicator& c, peer_num p) {
        Data<int> single = 1, single_rcv;
        Data<std::vector<int>> mult = {{1, 2, 3}}, mult_rcv(3);
        if (p == 0) {
            c.send(single, 1);
            c.send(mult, 1);
        } else {
            c.recv(single_rcv, 0);
            c.recv(mult_rcv, 0);
            CHECK(single_rcv.get() == 1);
            CHECK((mult_rcv.get() == std::vector<int>{1, 2, 3}));
        }
    });
}

TEST(bcast) {  // tests/communicator.cpp:35-50
    for (peer_num root : {0u, 2u})
        with_peers(4, [root](Communicator& c, peer_num p) {
            Data<int> d = (p == root) ? 1 : 0;
            c.bcast(d, root);
            CHECK(d.get() == 1);
        });
}

TEST(scatter_gather) {  // tests/communicator.cpp:52-92
    for (peer_num root : {0u, 1u, 3u})
        with_peers(5, [root](Communicator& c, peer_num p) {
            Data<std::vector<int>> all(std::vector<int>{1, 2, 3, 4, 5});
            Data<std::vector<int>> mine(1);
            c.scatter(all, mine, root);
            CHECK(mine.get()[0] == static_cast<int>(p) + 1);
            Data<std::vector<int>> back(5);
            c.gather(mine, back, root);
            if (p == root) CHECK((back.get() == std::vector<int>{1, 2, 3, 4, 5}));
        });
}

TEST(reduce) {  // tests/communicator.cpp:94-116
    with_peers(4, [](Communicator& c, peer_num p) {
        Data<int> d = static_cast<int>(p) + 1, res;
        c.reduce(d, res, 0, Function<int>([](int a, int b) { return a + b; }, true, true));
        if (p == 0) CHECK(res.get() == 10);
    });
}

TEST(reduce_vector) {  // tests/communicator.cpp:118-143
    with_peers(4, [](Communicator& c, peer_num p) {
        const int r = static_cast<int>(p) + 1;
        Data<std::vector<int>> d(std::vector<int>{r, 2 * r}), res(2);
        Function<std::vector<int>> f([](auto a, auto b) { return std::vector<int>{a[0] + b[0], a[1] * b[1]}; }, true, true);
        c.reduce(d, res, 0, f);
        if (p == 0) CHECK((res.get() == std::vector<int>{10, 384}));
    });
}

TEST(allreduce) {  // tests/communicator.cpp:145-165
    with_peers(4, [](Communicator& c, peer_num p) {
        Data<int> d = static_cast<int>(p) + 1, res;
        c.allreduce(d, res, Function<int>([](int a, int b) { return a + b; }, true, true));
        CHECK(res.get() == 10);
    });
}

TEST(allreduce_vector) {  // tests/communicator.cpp:167-192
    with_peers(4, [](Communicator& c, peer_num p) {
        const int r = static_cast<int>(p) + 1;
        Data<std::vector<int>> d(std::vector<int>{r, 2 * r, r}), res(3);
        Function<std::vector<int>> f(
            [](auto a, auto b) { return std::vector<int>{a[0] + b[0], a[1] * b[1], std::max(a[2], b[2])}; }, true, true);
        c.allreduce(d, res, f);
        CHECK((res.get() == std::vector<int>{10, 384, 4}));
    });
}

TEST(scan) {  // tests/communicator.cpp:194-219
    with_peers(4, [](Communicator& c, peer_num p) {
        Data<int> d = static_cast<int>(p) + 1, res;
        c.scan(d, res, Function<int>([](int a, int b) { return a + b; }, true, true));
        int expect = 0;
        for (peer_num i = 0; i <= p; ++i) expect += static_cast<int>(i) + 1;
        CHECK(res.get() == expect);
    });
}

TEST(scan_vector) {  // tests/communicator.cpp:221-254
    with_peers(4, [](Communicator& c, peer_num p) {
        const int r = static_cast<int>(p) + 1;
        Data<std::vector<int>> d(std::vector<int>{r, 2 * r, r}), res(3);
        Function<std::vector<int>> f(
            [](auto a, auto b) { return std::vector<int>{a[0] + b[0], a[1] * b[1], std::max(a[2], b[2])}; }, true, true);
        c.scan(d, res, f);
        int sum = 0, prod = 1;
        for (peer_num i = 0; i <= p; ++i) {
            sum += static_cast<int>(i) + 1;
            prod *= 2 * (static_cast<int>(i) + 1);
        }
        CHECK(res.get()[0] == sum && res.get()[1] == prod && res.get()[2] == r);
    });
}

// ---- reference tests/channels.cpp known answers: fork()ed peers, raw functions ---------------------------
static raw_function int_op(char which, bool comm_assoc) {
    return raw_function{[which](char* a, char* b) {
                            int* x = reinterpret_cast<int*>(a);
                            const int y = *reinterpret_cast<int*>(b);
                            if (which == '*')
                                *x = static_cast<int>(static_cast<unsigned>(*x) * static_cast<unsigned>(y));
                            else if (which == '-')
                                *x = *x - y;
                            else
                                *x = *x + y;
                        },
                        comm_assoc, comm_assoc};
}

TEST(reduce_multiple) {  // tests/channels.cpp:419-465: 13 peers, root 5, product wraps in int32
    int* res = shared_array<int>(1);
    with_processes(13, [res](FMI::Comm::Channel& ch, peer_num p) {
        int val = static_cast<int>(p) + 1;
        if (p == 5)
            ch.reduce({reinterpret_cast<char*>(&val), sizeof(int)}, {reinterpret_cast<char*>(res), sizeof(int)}, 5, int_op('*', true));
        else
            ch.reduce({reinterpret_cast<char*>(&val), sizeof(int)}, {nullptr, 0}, 5, int_op('*', true));
    });
    CHECK(*res == 1932053504);
}

TEST(reduce_multiple_ltr) {  // tests/channels.cpp:467-513
    int* res = shared_array<int>(1);
    with_processes(8, [res](FMI::Comm::Channel& ch, peer_num p) {
        int val = static_cast<int>(p) + 1;
        ch.reduce({reinterpret_cast<char*>(&val), sizeof(int)}, {p == 0 ? reinterpret_cast<char*>(res) : nullptr, sizeof(int)},
                  0, int_op('-', false));
    });
    CHECK(*res == -34);
}

TEST(allreduce_multiple) {  // tests/channels.cpp:515-558
    int* res = shared_array<int>(8);
    with_processes(8, [res](FMI::Comm::Channel& ch, peer_num p) {
        int val = static_cast<int>(p) + 1;
        ch.allreduce({reinterpret_cast<char*>(&val), sizeof(int)}, {reinterpret_cast<char*>(res + p), sizeof(int)}, int_op('+', true));
    });
    for (int i = 0; i < 8; ++i) CHECK(res[i] == 36);
}

TEST(allreduce_multiple_ltr) {  // tests/channels.cpp:560-604
    int* res = shared_array<int>(8);
    with_processes(8, [res](FMI::Comm::Channel& ch, peer_num p) {
        int val = static_cast<int>(p) + 1;
        ch.allreduce({reinterpret_cast<char*>(&val), sizeof(int)}, {reinterpret_cast<char*>(res + p), sizeof(int)}, int_op('-', false));
    });
    for (int i = 0; i < 8; ++i) CHECK(res[i] == -34);
}

TEST(scan_multiple) {  // tests/channels.cpp:606-647: 32 peers
    int* res = shared_array<int>(32);
    with_processes(32, [res](FMI::Comm::Channel& ch, peer_num p) {
        int val = static_cast<int>(p) + 1;
        ch.scan({reinterpret_cast<char*>(&val), sizeof(int)}, {reinterpret_cast<char*>(res + p), sizeof(int)}, int_op('+', true));
    });
    int prefix = 0;
    for (int i = 0; i < 32; ++i) {
        prefix += i + 1;
        CHECK(res[i] == prefix);
    }
}

TEST(scan_ltr) {  // tests/channels.cpp:649-690
    int* res = shared_array<int>(8);
    with_processes(8, [res](FMI::Comm::Channel& ch, peer_num p) {
        int val = static_cast<int>(p);
        ch.scan({reinterpret_cast<char*>(&val), sizeof(int)}, {reinterpret_cast<char*>(res + p), sizeof(int)}, int_op('-', false));
    });
    int result = 0;
    for (int i = 0; i < 8; ++i) {
        result -= i;
        CHECK(res[i] == result);
    }
}

TEST(barrier_and_large_buckets_over_sockets) {  // 4 MiB messages exceed the socket buffers: no deadlock
    float* res = shared_array<float>(4);
    with_processes(4, [res](FMI::Comm::Channel& ch, peer_num p) {
        ch.barrier();
        std::vector<float> a(1 << 20, static_cast<float>(p + 1)), r(1 << 20);
        raw_function sum{[](char* x, char* y) {
                             float* fx = reinterpret_cast<float*>(x);
                             const float* fy = reinterpret_cast<const float*>(y);
                             for (int i = 0; i < (1 << 20); ++i) fx[i] += fy[i];
                         },
                         true, true};
        ch.allreduce({reinterpret_cast<char*>(a.data()), a.size() * 4}, {reinterpret_cast<char*>(r.data()), r.size() * 4}, sum);
        res[p] = r[12345];
        ch.barrier();
    });
    for (int i = 0; i < 4; ++i) CHECK(res[i] == 10.0f);
}

// ---- transfer overlapped with the combine (stream transports, ranged built-in combines) --------------
// Every peer runs each collective twice on the same inputs, chunked (1 MiB pieces, combine of piece k on
// the worker while piece k+1 moves) and serial (overlap chunk 0); the results must agree bit for bit. The
// buckets (3 MiB + 7 floats) give three full pieces and a ragged one; P covers the recursive-doubling fold.
static raw_function ranged_float_op(char kind, bool comm_assoc) {
    auto part = [kind](char* a, char* b, std::size_t off, std::size_t len) {
        float* x = reinterpret_cast<float*>(a + off);
        const float* y = reinterpret_cast<const float*>(b + off);
        for (std::size_t i = 0; i < len / sizeof(float); ++i) x[i] = kind == '+' ? x[i] + y[i] : x[i] - y[i];
    };
    raw_function f{nullptr, comm_assoc, comm_assoc};  // f.f is set per bucket size by the caller
    f.part = part;
    f.granule = sizeof(float);
    return f;
}

TEST(overlapped_transfer_combine_is_bit_identical) {
    constexpr std::size_t n = (3u << 20) / 4 + 7;
    for (peer_num P : {2u, 3u, 5u}) {
        // [run][kind][peer][n]: kind 0 allreduce, 1 reduce (root 1), 2 scan, 3 scan_ltr (a - b)
        float* res = shared_array<float>(2 * 4 * P * n);
        std::size_t* pieces = shared_array<std::size_t>(2 * P);
        with_processes(P, [res, pieces, P](FMI::Comm::Channel& ch, peer_num p) {
            auto& p2p = dynamic_cast<FMI::Comm::PeerToPeer&>(ch);
            for (int run = 0; run < 2; ++run) {
                const std::size_t before = p2p.overlapped_pieces();
                p2p.set_overlap_chunk(run == 0 ? (1u << 20) : 0);
                for (int kind = 0; kind < 4; ++kind) {
                    std::vector<float> send(n), recv(n, 0.f);
                    for (std::size_t i = 0; i < n; ++i) send[i] = std::sin(0.001f * static_cast<float>(i) + static_cast<float>(p));
                    raw_function f = ranged_float_op(kind == 3 ? '-' : '+', kind != 3);
                    const std::size_t bytes = n * sizeof(float);
                    f.f = [part = f.part, bytes](char* a, char* b) { part(a, b, 0, bytes); };
                    channel_data sd{reinterpret_cast<char*>(send.data()), bytes};
                    channel_data rd{reinterpret_cast<char*>(recv.data()), bytes};
                    if (kind == 0) ch.allreduce(sd, rd, f);
                    if (kind == 1) ch.reduce(sd, rd, 1 % P, f);
                    if (kind == 2 || kind == 3) ch.scan(sd, rd, f);
                    std::memcpy(res + ((run * 4 + kind) * P + p) * n, recv.data(), bytes);
                }
                pieces[run * P + p] = p2p.overlapped_pieces() - before;
            }
        });
        std::size_t chunked = 0;
        for (peer_num p = 0; p < P; ++p) {
            chunked += pieces[p];
            CHECK(pieces[P + p] == 0);  // overlap chunk 0: the serial path
        }
        CHECK(chunked > 0);  // the chunked run really overlapped
        for (int kind = 0; kind < 4; ++kind)
            for (peer_num p = 0; p < P; ++p) {
                if (kind == 1 && p != 1 % P) continue;  // reduce: only the root's recvbuf is defined
                const float* a = res + ((0 * 4 + kind) * P + p) * n;
                const float* b = res + ((1 * 4 + kind) * P + p) * n;
                CHECK(std::memcmp(a, b, n * sizeof(float)) == 0);
            }
        // and the chunked results are right: allreduce of sin(0.001 i + p) at a few indices, to 1e-5
        for (std::size_t i : {std::size_t(0), std::size_t(262147), n - 1}) {
            double want = 0;
            for (peer_num q = 0; q < P; ++q) want += std::sin(0.001f * static_cast<float>(i) + static_cast<float>(q));
            CHECK(std::fabs(res[(0 * 4 + 0) * P * n + i] - want) < 1e-4);
        }
        munmap(res, 2 * 4 * P * n * sizeof(float));
        munmap(pieces, 2 * P * sizeof(std::size_t));
    }
}

// ---- evaluation order: symbolic buffers through the channel algorithms ----------------------------------
constexpr std::size_t kSym = 8192;
static raw_function sym_combine(bool comm_assoc) {
    return raw_function{[](char* a, char* b) {
                            std::string r = std::string("(") + a + "+" + b + ")";
                            if (r.size() + 1 > kSym) throw std::runtime_error("expression too long");
                            std::memcpy(a, r.c_str(), r.size() + 1);
                        },
                        comm_assoc, comm_assoc};
}

static std::string schedule(int alg, int P, int rank) {
    std::vector<char> buf(1 << 16);
    Dev::check(fmi_schedule_expr(alg, P, rank, buf.data(), buf.size()), "fmi_schedule_expr");
    return buf.data();
}

TEST(order_matches_kernel_schedules) {
    // The C++ channel algorithms, the fused kernels' programs (fmi_schedule.h) and, through the Python
    // wrapper, the oracle must all agree on every peer's bracketing.
    for (peer_num P = 1; P <= 17; ++P) {
        std::vector<std::string> ar(P), ar_send(P), sc(P), scl(P), arl(P);
        std::vector<std::vector<std::string>> red(P, std::vector<std::string>(P));
        auto mailbox = std::make_shared<FMI::Comm::Mailbox>();
        auto run = [&](auto fn) {
            std::vector<std::thread> ts;
            for (peer_num p = 0; p < P; ++p)
                ts.emplace_back([&, p] {
                    FMI::Comm::Loopback ch(mailbox, std::chrono::seconds(10));
                    ch.set_peer_id(p);
                    ch.set_num_peers(P);
                    fn(ch, p);
                });
            for (auto& t : ts) t.join();
        };
        run([&](FMI::Comm::Loopback& ch, peer_num p) {
            std::vector<char> s(kSym), r(kSym);
            std::snprintf(s.data(), kSym, "x%u", p);
            ch.allreduce({s.data(), kSym}, {r.data(), kSym}, sym_combine(true));
            ar[p] = r.data();
            ar_send[p] = s.data();
        });
        run([&](FMI::Comm::Loopback& ch, peer_num p) {
            std::vector<char> s(kSym), r(kSym);
            std::snprintf(s.data(), kSym, "x%u", p);
            ch.scan({s.data(), kSym}, {r.data(), kSym}, sym_combine(true));
            sc[p] = r.data();
        });
        run([&](FMI::Comm::Loopback& ch, peer_num p) {
            std::vector<char> s(kSym), r(kSym);
            std::snprintf(s.data(), kSym, "x%u", p);
            ch.scan({s.data(), kSym}, {r.data(), kSym}, sym_combine(false));
            scl[p] = r.data();
        });
        run([&](FMI::Comm::Loopback& ch, peer_num p) {
            std::vector<char> s(kSym), r(kSym);
            std::snprintf(s.data(), kSym, "x%u", p);
            ch.allreduce({s.data(), kSym}, {r.data(), kSym}, sym_combine(false));
            arl[p] = r.data();
        });
        for (peer_num root = 0; root < P; ++root)
            run([&](FMI::Comm::Loopback& ch, peer_num p) {
                std::vector<char> s(kSym), r(kSym);
                std::snprintf(s.data(), kSym, "x%u", p);
                ch.reduce({s.data(), kSym}, {r.data(), kSym}, root, sym_combine(true));
                if (p == root) red[root][0] = r.data();
            });
        for (peer_num p = 0; p < P; ++p) {
            CHECK(ar[p] == schedule(FMI_ALG_ALLREDUCE, P, p));
            CHECK(ar_send[p] == ar[p]);  // sendbuf clobbered with the result (reference :129)
            CHECK(sc[p] == schedule(FMI_ALG_SCAN, P, p));
            CHECK(scl[p] == schedule(FMI_ALG_SCAN_LTR, P, p));
            CHECK(arl[p] == schedule(FMI_ALG_REDUCE_LTR, P, p));
        }
        for (peer_num root = 0; root < P; ++root) {
            // reduce programs are in transformed ids (root -> 0): map x<t> to x<(t + root) % P>
            std::string t = schedule(FMI_ALG_REDUCE, P, 0), real;
            for (std::size_t i = 0; i < t.size(); ++i) {
                if (t[i] == 'x') {
                    std::size_t j = i + 1;
                    unsigned v = 0;
                    while (j < t.size() && std::isdigit(static_cast<unsigned char>(t[j]))) v = v * 10 + (t[j++] - '0');
                    real += "x" + std::to_string((v + root) % P);
                    i = j - 1;
                } else {
                    real += t[i];
                }
            }
            CHECK(red[root][0] == real);
        }
    }
}

// ---- errors, policy, configuration ------------------------------------------------------------------------
TEST(dimension_mismatch_throws) {
    with_peers(1, [](Communicator& c, peer_num) {
        Data<std::vector<float>> a(4), b(5);
        CHECK_THROWS(c.allreduce(a, b, Function<std::vector<float>>(Op::sum)), std::runtime_error);
        CHECK_THROWS(c.scan(a, b, Function<std::vector<float>>(Op::sum)), std::runtime_error);
        CHECK_THROWS(c.reduce(a, b, 0, Function<std::vector<float>>(Op::sum)), std::runtime_error);
    });
}

TEST(receive_timeout_raises_timeout) {
    auto mailbox = std::make_shared<FMI::Comm::Mailbox>();
    FMI::Comm::Loopback ch(mailbox, std::chrono::milliseconds(50));
    ch.set_peer_id(0);
    ch.set_num_peers(2);
    int x = 0;
    CHECK_THROWS(ch.recv({reinterpret_cast<char*>(&x), sizeof(int)}, 1), FMI::Utils::Timeout);
}

TEST(policy_picks_by_hint) {
    auto mailbox = std::make_shared<FMI::Comm::Mailbox>();
    Communicator c(0, 1, "", "policy");
    // "Slow": cheap (price 0) but slow; "Fast": quick but priced per request
    struct Priced : FMI::Comm::Loopback {
        using Loopback::Loopback;
        double get_price(peer_num, peer_num, std::size_t) override { return 1.0; }
    };
    c.register_channel("Slow", std::make_shared<FMI::Comm::Loopback>(mailbox, std::chrono::seconds(1), 1.0, 50.0));
    c.register_channel("Fast", std::make_shared<Priced>(mailbox, std::chrono::seconds(1), 1e6, 0.001));
    FMI::Utils::ChannelPolicy policy = [&] {
        static std::map<std::string, std::shared_ptr<FMI::Comm::Channel>> chans;
        chans["Slow"] = std::make_shared<FMI::Comm::Loopback>(mailbox, std::chrono::seconds(1), 1.0, 50.0);
        chans["Fast"] = std::make_shared<Priced>(mailbox, std::chrono::seconds(1), 1e6, 0.001);
        for (auto& kv : chans) kv.second->set_num_peers(4);  // models scale with the peer count
        return FMI::Utils::ChannelPolicy(chans, 4, 0.0000166667 / 8, FMI::Utils::fast);
    }();
    CHECK(policy.get_channel({FMI::Utils::allreduce, 1 << 20}) == "Fast");
    policy.set_hint(FMI::Utils::cheap);
    CHECK(policy.get_channel({FMI::Utils::allreduce, 1 << 20}) == "Slow");
    // the communicator itself dispatches through its policy
    Data<std::vector<float>> a(std::vector<float>{1, 2}), b(2);
    c.hint(FMI::Utils::fast);
    c.allreduce(a, b, Function<std::vector<float>>(Op::sum));
    CHECK((b.get() == std::vector<float>{1, 2}));
}

TEST(configuration_reads_reference_schema) {
    const char* path = "/tmp/fmi_amd_test_config.json";
    {
        std::ofstream f(path);
        f << R"({"backends": {"S3": {"enabled": false, "bucket_name": "b", "timeout": 100},
                 "Direct": {"enabled": true, "host": "127.0.0.1", "port": 10000, "max_timeout": 1000}},
                "model": {"FaaS": {"gib_second_price": 0.0000166667},
                          "Direct": {"bandwidth": 400.0, "overhead": 0.34, "include_infrastructure_costs": true}}})";
    }
    FMI::Utils::Configuration cfg(path);
    auto b = cfg.get_active_channels();
    CHECK(b.size() == 1 && b.count("Direct") == 1);
    CHECK(b["Direct"].first["host"] == "127.0.0.1" && b["Direct"].first["port"] == "10000");
    CHECK(b["Direct"].second["bandwidth"] == "400.0" && b["Direct"].second["include_infrastructure_costs"] == "true");
    CHECK(std::fabs(cfg.get_faas_price() - 0.0000166667) < 1e-12);
    CHECK_THROWS(FMI::Utils::Configuration("/nonexistent/fmi.json"), std::runtime_error);
    std::remove(path);
}

TEST(builtin_host_functions_match_lambdas) {
    with_peers(5, [](Communicator& c, peer_num p) {
        std::vector<int64_t> v = {static_cast<int64_t>(p) - 2, INT64_MAX - static_cast<int64_t>(p), static_cast<int64_t>(p) * 7};
        Data<std::vector<int64_t>> a(v), r(3), a2(v), r2(3);
        c.allreduce(a, r, Function<std::vector<int64_t>>(Op::max));
        Function<std::vector<int64_t>> lam(
            [](auto x, auto y) {
                for (std::size_t i = 0; i < x.size(); ++i) x[i] = std::max(x[i], y[i]);
                return x;
            },
            true, true);
        c.allreduce(a2, r2, lam);
        CHECK(r.get() == r2.get());
        CHECK(r.get()[0] == 2 && r.get()[1] == INT64_MAX && r.get()[2] == 28);
    });
}

// ---- device buckets (MI355X) ----------------------------------------------------------------------------
static uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
static std::vector<float> synth_f32(std::size_t n, uint64_t seed, uint32_t peer) {
    std::vector<float> v(n);
    const uint64_t key = seed ^ (static_cast<uint64_t>(peer) << 40);
    for (std::size_t i = 0; i < n; ++i) v[i] = static_cast<float>(splitmix64(key ^ i) >> 40) * 0x1p-24f * 2.0f - 1.0f;
    return v;
}

GPU_TEST(device_buckets_match_host_path_bitwise) {
    Dev::init(0);
    const std::size_t n = 100003;
    for (peer_num P : {2u, 3u, 5u, 8u}) {
        std::vector<std::vector<float>> host_ar(P), dev_ar(P), host_sc(P), dev_sc(P), dev_send(P);
        std::vector<float> host_red, dev_red;
        with_peers(P, [&](Communicator& c, peer_num p) {
            Data<std::vector<float>> a(synth_f32(n, 42, p)), r(n);
            c.allreduce(a, r, Function<std::vector<float>>(Op::sum));
            host_ar[p] = r.get();
            Data<std::vector<float>> s(synth_f32(n, 42, p)), sr(n);
            c.scan(s, sr, Function<std::vector<float>>(Op::sum));
            host_sc[p] = sr.get();
            Data<std::vector<float>> d(synth_f32(n, 42, p)), dr(n);
            c.reduce(d, dr, P - 1, Function<std::vector<float>>(Op::sum));
            if (p == P - 1) host_red = dr.get();
        });
        with_peers(P, [&](Communicator& c, peer_num p) {
            Data<Dev::Bucket<float>> a(synth_f32(n, 42, p)), r(n);
            c.allreduce(a, r, Function<Dev::Bucket<float>>(Op::sum));
            dev_ar[p] = r.get();
            dev_send[p] = a.get();
            Data<Dev::Bucket<float>> s(synth_f32(n, 42, p)), sr(n);
            c.scan(s, sr, Function<Dev::Bucket<float>>(Op::sum));
            dev_sc[p] = sr.get();
            Data<Dev::Bucket<float>> d(synth_f32(n, 42, p)), dr(n);
            c.reduce(d, dr, P - 1, Function<Dev::Bucket<float>>(Op::sum));
            if (p == P - 1) dev_red = dr.get();
        });
        for (peer_num p = 0; p < P; ++p) {
            CHECK(std::memcmp(host_ar[p].data(), dev_ar[p].data(), n * 4) == 0);
            CHECK(std::memcmp(dev_send[p].data(), dev_ar[p].data(), n * 4) == 0);  // sendbuf side effect
            CHECK(std::memcmp(host_sc[p].data(), dev_sc[p].data(), n * 4) == 0);
        }
        CHECK(std::memcmp(host_red.data(), dev_red.data(), n * 4) == 0);
    }
}

// Any fundamental integer width is a device dtype (reference Data<std::vector<A>>, include/comm/Data.h:50-73):
// the reference's allreduce_vector known answers (tests/communicator.cpp:167-192, P = 4, peer p holds p + 1)
// for sum / prod / max on uint16 device buckets, and on int8 host buckets offloaded to the GPU.
GPU_TEST(small_integer_buckets_known_answers) {
    Dev::init(0);
    std::vector<uint16_t> dsum(4), dprod(4), dmax(4);
    std::vector<int8_t> hsum(4), hprod(4);
    with_peers(4, [&](Communicator& c, peer_num p) {
        const std::size_t n = 4099;
        auto run = [&](Op op) {
            Data<Dev::Bucket<uint16_t>> a(std::vector<uint16_t>(n, static_cast<uint16_t>(p + 1))), r(n);
            c.allreduce(a, r, Function<Dev::Bucket<uint16_t>>(op));
            return r.get()[n - 1];
        };
        dsum[p] = run(Op::sum);
        dprod[p] = run(Op::prod);
        dmax[p] = run(Op::max);
    });
    with_peers(4, [&](Communicator& c, peer_num p) {
        c.use_device(0, true);  // every combine on the GPU, whatever the crossover
        const std::size_t n = 70001;
        Data<std::vector<int8_t>> a(std::vector<int8_t>(n, static_cast<int8_t>(p + 1))), r(n);
        c.allreduce(a, r, Function<std::vector<int8_t>>(Op::sum));
        hsum[p] = r.get()[n / 2];
        Data<std::vector<int8_t>> b(std::vector<int8_t>(n, static_cast<int8_t>(100 + p))), rb(n);
        c.allreduce(b, rb, Function<std::vector<int8_t>>(Op::prod));  // 100·101·102·103 wraps in 8 bits
        hprod[p] = rb.get()[7];
    });
    const int8_t wrapped = static_cast<int8_t>(static_cast<uint8_t>(100u * 101u * 102u * 103u));
    for (int p = 0; p < 4; ++p) {
        CHECK(dsum[p] == 10);
        CHECK(dprod[p] == 24);
        CHECK(dmax[p] == 4);
        CHECK(hsum[p] == 10);
        CHECK(hprod[p] == wrapped);
    }
}

GPU_TEST(device_bcast_scatter_gather) {
    Dev::init(0);
    with_peers(5, [](Communicator& c, peer_num p) {
        std::vector<int64_t> all(5 * 3);
        for (std::size_t i = 0; i < all.size(); ++i) all[i] = static_cast<int64_t>(i) * 11;
        Data<Dev::Bucket<int64_t>> src(all), mine(3), back(15);
        c.scatter(src, mine, 2);
        auto m = mine.get();
        CHECK(m[0] == static_cast<int64_t>(3 * p) * 11 && m[2] == static_cast<int64_t>(3 * p + 2) * 11);
        c.gather(mine, back, 2);
        if (p == 2) CHECK(back.get() == all);
        Data<Dev::Bucket<int64_t>> b(std::vector<int64_t>{static_cast<int64_t>(p), 7});
        c.bcast(b, 4);
        CHECK((b.get() == std::vector<int64_t>{4, 7}));
    });
}

GPU_TEST(host_offload_matches_host_path) {
    const std::size_t n = (1 << 20) + 11;
    std::vector<std::vector<float>> off(4), host(4);
    with_peers(4, [&](Communicator& c, peer_num p) {
        Data<std::vector<float>> a(synth_f32(n, 7, p)), r(n);
        c.allreduce(a, r, Function<std::vector<float>>(Op::sum));
        host[p] = r.get();
    });
    with_peers(4, [&](Communicator& c, peer_num p) {
        c.use_device(0, true);  // every combine on the GPU, whatever the crossover
        Data<std::vector<float>> a(synth_f32(n, 7, p)), r(n);
        c.allreduce(a, r, Function<std::vector<float>>(Op::sum));
        off[p] = r.get();
    });
    for (int p = 0; p < 4; ++p) CHECK(std::memcmp(off[p].data(), host[p].data(), n * 4) == 0);
}

// The Rccl channel over the LOCAL transport (peers = threads sharing the GPU): bootstrapped through the
// Loopback host channel, selected by the policy for device buckets, results equal to the host path.
GPU_TEST(rccl_channel_collectives_local_transport) {
    Dev::init(0);
    for (peer_num P : {2u, 3u, 4u, 5u, 8u}) {
        const std::size_t n = 300007;
        std::vector<std::vector<float>> host_ar(P), dev_ar(P), dev_send(P), host_sc(P), dev_sc(P);
        std::vector<std::vector<float>> host_red_send(P), dev_red_send(P);  // reduce partials (PeerToPeer.cpp:72)
        std::vector<float> host_red, dev_red;
        std::vector<std::string> picked(P);
        with_peers(P, [&](Communicator& c, peer_num p) {
            Data<std::vector<float>> a(synth_f32(n, 5, p)), r(n);
            c.allreduce(a, r, Function<std::vector<float>>(Op::sum));
            host_ar[p] = r.get();
            Data<std::vector<float>> s(synth_f32(n, 5, p)), sr(n);
            c.scan(s, sr, Function<std::vector<float>>(Op::sum));
            host_sc[p] = sr.get();
            Data<std::vector<float>> d(synth_f32(n, 5, p)), dr(n);
            c.reduce(d, dr, 1 % P, Function<std::vector<float>>(Op::sum));
            if (p == 1 % P) host_red = dr.get();
            host_red_send[p] = d.get();
        });
        auto mailbox = std::make_shared<FMI::Comm::Mailbox>();
        std::vector<std::thread> ts;
        std::vector<std::string> errors(P);
        for (peer_num p = 0; p < P; ++p)
            ts.emplace_back([&, p] {
                try {
                    Communicator c(p, P, "", "rccl-test");
                    auto loop = std::make_shared<FMI::Comm::Loopback>(mailbox, std::chrono::seconds(60));
                    c.register_channel("Loopback", loop);
                    c.register_channel("Rccl", FMI::Comm::Rccl::connect(*loop, p, P, FMI_TRANSPORT_LOCAL));
                    Data<Dev::Bucket<float>> a(synth_f32(n, 5, p)), r(n);
                    c.allreduce(a, r, Function<Dev::Bucket<float>>(Op::sum));
                    dev_ar[p] = r.get();
                    dev_send[p] = a.get();
                    Data<Dev::Bucket<float>> s(synth_f32(n, 5, p)), sr(n);
                    c.scan(s, sr, Function<Dev::Bucket<float>>(Op::sum));
                    dev_sc[p] = sr.get();
                    Data<Dev::Bucket<float>> d(synth_f32(n, 5, p)), dr(n);
                    c.reduce(d, dr, 1 % P, Function<Dev::Bucket<float>>(Op::sum));
                    if (p == 1 % P) dev_red = dr.get();
                    dev_red_send[p] = d.get();
                    Data<Dev::Bucket<int64_t>> b(std::vector<int64_t>{static_cast<int64_t>(p), 9});
                    c.bcast(b, P - 1);
                    if (b.get()[0] != static_cast<int64_t>(P - 1)) throw std::runtime_error("bcast over Rccl");
                    c.barrier();
                } catch (const std::exception& e) {
                    errors[p] = e.what();
                }
            });
        for (auto& t : ts) t.join();
        for (peer_num p = 0; p < P; ++p) {
            if (!errors[p].empty()) {
                ++g_failures;
                std::fprintf(stderr, "  peer %u threw: %s\n", p, errors[p].c_str());
                continue;
            }
            CHECK(std::memcmp(host_ar[p].data(), dev_ar[p].data(), n * 4) == 0);
            CHECK(std::memcmp(dev_send[p].data(), dev_ar[p].data(), n * 4) == 0);  // sendbuf = result
            CHECK(std::memcmp(host_sc[p].data(), dev_sc[p].data(), n * 4) == 0);
            // every peer's sendbuf after reduce: the reference's partial (interior), own bucket (leaf), result (root)
            CHECK(std::memcmp(host_red_send[p].data(), dev_red_send[p].data(), n * 4) == 0);
        }
        CHECK(host_red.size() == n && dev_red.size() == n && std::memcmp(host_red.data(), dev_red.data(), n * 4) == 0);
    }
}

// A peer that never arrives: the Rccl channel's collective throws FMI::Utils::Timeout once its timeout
// passes, as the reference's channels do when a peer stays away (src/comm/Direct.cpp:28-30,40-42), and the
// channel is unusable (std::runtime_error) until destroyed. LOCAL transport (peers = threads on one GPU).
GPU_TEST(rccl_channel_absent_peer_raises_timeout) {
    Dev::init(0);
    auto mailbox = std::make_shared<FMI::Comm::Mailbox>();
    const std::size_t n = 4096;
    bool timed_out = false, unusable = false;
    double waited_s = 0;
    std::string error;
    auto member = [&](peer_num p, bool participate) {
        try {
            Communicator c(p, 2, "", "timeout-test");
            auto loop = std::make_shared<FMI::Comm::Loopback>(mailbox, std::chrono::seconds(60));
            c.register_channel("Loopback", loop);
            c.register_channel("Rccl", FMI::Comm::Rccl::connect(*loop, p, 2, FMI_TRANSPORT_LOCAL, 300., 1.0));
            if (!participate) return;  // joined the communicator, never calls the collective
            Data<Dev::Bucket<float>> a(synth_f32(n, 3, p)), r(n);
            const auto t0 = std::chrono::steady_clock::now();
            try {
                c.allreduce(a, r, Function<Dev::Bucket<float>>(Op::sum));
            } catch (const FMI::Utils::Timeout&) {
                timed_out = true;
            }
            waited_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            try {
                c.allreduce(a, r, Function<Dev::Bucket<float>>(Op::sum));
            } catch (const FMI::Utils::Timeout&) {
            } catch (const std::runtime_error&) {
                unusable = true;  // the aborted communicator refuses further work
            }
        } catch (const std::exception& e) {
            error = e.what();
        }
    };
    std::thread present(member, 0u, true), absent(member, 1u, false);
    present.join();
    absent.join();
    if (!error.empty()) std::fprintf(stderr, "  threw: %s\n", error.c_str());
    CHECK(error.empty());
    CHECK(timed_out);
    CHECK(waited_s >= 0.9 && waited_s < 30.0);
    CHECK(unusable);
}

GPU_TEST(policy_routes_device_buckets_to_rccl) {
    Dev::init(0);
    std::map<std::string, std::shared_ptr<FMI::Comm::Channel>> chans;
    auto mailbox = std::make_shared<FMI::Comm::Mailbox>();
    auto loop = std::make_shared<FMI::Comm::Loopback>(mailbox);
    loop->set_num_peers(1);
    chans["Loopback"] = loop;
    chans["Rccl"] = FMI::Comm::Rccl::connect(*loop, 0, 1, FMI_TRANSPORT_LOCAL);
    FMI::Utils::ChannelPolicy policy(chans, 1, 0.0000166667 / 8, FMI::Utils::cheap);
    for (std::size_t bytes : {std::size_t(1) << 10, std::size_t(1) << 20, std::size_t(256) << 20}) {
        CHECK(policy.get_device_channel({FMI::Utils::allreduce, bytes}) == "Rccl");
        CHECK(policy.get_channel({FMI::Utils::allreduce, bytes}) == "Loopback");  // host buffers never go to Rccl
    }
}

// Host buckets over the Rccl channel (host ingress, config C5 shape): with only Rccl registered, every
// collective of host vectors runs through the GPU (allreduce pipelined, the rest staged) and must equal
// the host-channel results bit for bit; sendbuf side effects as in the reference.
GPU_TEST(rccl_channel_host_ingress_local_transport) {
    Dev::init(0);
    for (peer_num P : {2u, 3u, 8u}) {
        const std::size_t n = 200003;
        std::vector<std::vector<float>> host_ar(P), host_sc(P), dev_ar(P), dev_send(P), dev_sc(P), host_ord(P),
            dev_ord(P);
        std::vector<float> host_red, dev_red;
        auto ordered_sum = [] {
            Function<std::vector<float>> f(Op::sum);
            f.commutative = false;
            f.associative = false;
            return f;
        };
        with_peers(P, [&](Communicator& c, peer_num p) {
            Data<std::vector<float>> a(synth_f32(n, 8, p)), r(n);
            c.allreduce(a, r, Function<std::vector<float>>(Op::sum));
            host_ar[p] = r.get();
            Data<std::vector<float>> s(synth_f32(n, 8, p)), sr(n);
            c.scan(s, sr, Function<std::vector<float>>(Op::sum));
            host_sc[p] = sr.get();
            Data<std::vector<float>> d(synth_f32(n, 8, p)), dr(n);
            c.reduce(d, dr, P - 1, Function<std::vector<float>>(Op::sum));
            if (p == P - 1) host_red = dr.get();
            Data<std::vector<float>> o(synth_f32(n, 8, p)), orr(n);
            c.allreduce(o, orr, ordered_sum());
            host_ord[p] = orr.get();
        });
        auto mailbox = std::make_shared<FMI::Comm::Mailbox>();
        std::vector<std::thread> ts;
        std::vector<std::string> errors(P);
        for (peer_num p = 0; p < P; ++p)
            ts.emplace_back([&, p] {
                try {
                    Communicator c(p, P, "", "rccl-host");
                    FMI::Comm::Loopback boot(mailbox, std::chrono::seconds(60));
                    boot.set_peer_id(p);
                    boot.set_num_peers(P);
                    auto rccl = FMI::Comm::Rccl::connect(boot, p, P, FMI_TRANSPORT_LOCAL);
                    rccl->set_host_ingress(true);
                    c.register_channel("Rccl", rccl);
                    Data<std::vector<float>> a(synth_f32(n, 8, p)), r(n);
                    c.allreduce(a, r, Function<std::vector<float>>(Op::sum));
                    dev_ar[p] = r.get();
                    dev_send[p] = a.get();
                    Data<std::vector<float>> s(synth_f32(n, 8, p)), sr(n);
                    c.scan(s, sr, Function<std::vector<float>>(Op::sum));
                    dev_sc[p] = sr.get();
                    Data<std::vector<float>> d(synth_f32(n, 8, p)), dr(n);
                    c.reduce(d, dr, P - 1, Function<std::vector<float>>(Op::sum));
                    if (p == P - 1) dev_red = dr.get();
                    Data<std::vector<float>> o(synth_f32(n, 8, p)), orr(n);
                    c.allreduce(o, orr, ordered_sum());  // reduce_ltr order through the host pipeline
                    dev_ord[p] = orr.get();
                    Data<std::vector<int64_t>> b(std::vector<int64_t>{static_cast<int64_t>(p), 9});
                    c.bcast(b, P - 1);
                    if (b.get()[0] != static_cast<int64_t>(P - 1)) throw std::runtime_error("host bcast over Rccl");
                    Data<std::vector<int32_t>> g(std::vector<int32_t>{static_cast<int32_t>(p)}), all(P);
                    c.gather(g, all, 0);
                    if (p == 0)
                        for (peer_num j = 0; j < P; ++j)
                            if (all.get()[j] != static_cast<int32_t>(j)) throw std::runtime_error("host gather over Rccl");
                    c.barrier();
                } catch (const std::exception& e) {
                    errors[p] = e.what();
                }
            });
        for (auto& t : ts) t.join();
        for (peer_num p = 0; p < P; ++p) {
            if (!errors[p].empty()) {
                ++g_failures;
                std::fprintf(stderr, "  peer %u threw: %s\n", p, errors[p].c_str());
                continue;
            }
            CHECK(std::memcmp(host_ar[p].data(), dev_ar[p].data(), n * 4) == 0);
            CHECK(std::memcmp(dev_send[p].data(), dev_ar[p].data(), n * 4) == 0);  // sendbuf = result
            CHECK(std::memcmp(host_sc[p].data(), dev_sc[p].data(), n * 4) == 0);
            CHECK(std::memcmp(host_ord[p].data(), dev_ord[p].data(), n * 4) == 0);
        }
        CHECK(host_red.size() == n && dev_red.size() == n && std::memcmp(host_red.data(), dev_red.data(), n * 4) == 0);
    }
}

// FMI_PATH_DIRECT through the C++ surface: window buckets from the channel, the fused kernel reading every
// peer's window in place; bit-identical to the host-channel allreduce, sendbuf = result as in the reference.
GPU_TEST(rccl_channel_direct_path_window_buckets) {
    Dev::init(0);
    for (peer_num P : {2u, 4u, 7u}) {
        const std::size_t n = 100003;
        std::vector<std::vector<float>> host(P), dev(P), sent(P);
        with_peers(P, [&](Communicator& c, peer_num p) {
            Data<std::vector<float>> a(synth_f32(n, 11, p)), r(n);
            c.allreduce(a, r, Function<std::vector<float>>(Op::sum));
            host[p] = r.get();
        });
        auto mailbox = std::make_shared<FMI::Comm::Mailbox>();
        std::vector<std::thread> ts;
        std::vector<std::string> errors(P);
        for (peer_num p = 0; p < P; ++p)
            ts.emplace_back([&, p] {
                try {
                    Communicator c(p, P, "", "rccl-direct");
                    FMI::Comm::Loopback boot(mailbox, std::chrono::seconds(60));
                    boot.set_peer_id(p);
                    boot.set_num_peers(P);
                    auto rccl = FMI::Comm::Rccl::connect(boot, p, P, FMI_TRANSPORT_LOCAL);
                    rccl->set_path(FMI_PATH_DIRECT);
                    c.register_channel("Rccl", rccl);
                    Data<Dev::Bucket<float>> a(rccl->window<float>(n)), r(n);
                    a.bucket().upload(synth_f32(n, 11, p));
                    c.allreduce(a, r, Function<Dev::Bucket<float>>(Op::sum));
                    dev[p] = r.get();
                    sent[p] = a.get();
                } catch (const std::exception& e) {
                    errors[p] = e.what();
                }
            });
        for (auto& t : ts) t.join();
        for (peer_num p = 0; p < P; ++p) {
            if (!errors[p].empty()) {
                ++g_failures;
                std::fprintf(stderr, "  peer %u threw: %s\n", p, errors[p].c_str());
                continue;
            }
            CHECK(std::memcmp(host[p].data(), dev[p].data(), n * 4) == 0);
            CHECK(std::memcmp(sent[p].data(), dev[p].data(), n * 4) == 0);
        }
    }
}

GPU_TEST(policy_host_ingress_keeps_user_functions_and_small_buckets_on_host) {
    Dev::init(0);
    std::map<std::string, std::shared_ptr<FMI::Comm::Channel>> chans;
    auto mailbox = std::make_shared<FMI::Comm::Mailbox>();
    auto loop = std::make_shared<FMI::Comm::Loopback>(mailbox);
    loop->set_num_peers(1);
    chans["Loopback"] = loop;
    auto rccl = FMI::Comm::Rccl::connect(*loop, 0, 1, FMI_TRANSPORT_LOCAL);
    rccl->set_host_ingress(true);
    chans["Rccl"] = rccl;
    FMI::Utils::ChannelPolicy policy(chans, 1, 0.0000166667 / 8, FMI::Utils::fast);
    for (std::size_t bytes : {std::size_t(1) << 10, std::size_t(256) << 20}) {
        FMI::Utils::OperationInfo user{FMI::Utils::allreduce, bytes, false, false, true};
        CHECK(policy.get_channel(user) == "Loopback");  // Rccl cannot run an opaque user function
    }
    CHECK(policy.get_channel({FMI::Utils::send, 64}) == "Loopback");  // PCIe crossing outweighs it
    CHECK(policy.get_device_channel({FMI::Utils::allreduce, std::size_t(1) << 20}) == "Rccl");
}

TEST(policy_host_combine_crossover) {
    // the built-in combine of two host buckets goes to the GPU only past the measured
    // crossover (profiles/r05_host_crossover.jsonl); both sides of it, pinned and pageable, and an override
    std::map<std::string, std::shared_ptr<FMI::Comm::Channel>> chans;
    FMI::Utils::ChannelPolicy policy(chans, 2, 0.0000166667 / 8, FMI::Utils::fast);
    using P = FMI::Utils::ChannelPolicy;
    const std::size_t cross = P::kHostCombinePinnedMinBytes;
    CHECK(!policy.host_combine_on_device(64 << 10, true));
    CHECK(!policy.host_combine_on_device(cross - 1, true));
    CHECK(policy.host_combine_on_device(cross, true));
    CHECK(policy.host_combine_on_device(std::size_t(1) << 30, true));
    CHECK(!policy.host_combine_on_device(64 << 10, false));
    CHECK(!policy.host_combine_on_device(cross, false));  // pageable buckets did not pay at any size measured
    CHECK(!policy.host_combine_on_device(std::size_t(1) << 30, false));
    policy.set_host_combine_min_bytes(std::size_t(1) << 20, 0);
    CHECK(!policy.host_combine_on_device((std::size_t(1) << 20) - 4, false));
    CHECK(policy.host_combine_on_device(std::size_t(1) << 20, false));
    CHECK(policy.host_combine_on_device(4, true));
}

GPU_TEST(host_combine_follows_the_policy_crossover) {
    // use_device(0): a 1 MiB pageable combine stays on the host (below the crossover); use_device(0, true) and a
    // policy whose crossover is 0 send it to the GPU; every result is the same, bit for bit
    const std::size_t n = (1 << 18) + 5;
    std::vector<float> got[3][2];
    bool on_device[3][2] = {};
    for (int mode = 0; mode < 3; ++mode)
        with_peers(2, [&](Communicator& c, peer_num p) {
            c.use_device(0, mode == 1);
            if (mode == 2) c.channel_policy()->set_host_combine_min_bytes(0, 0);
            Data<std::vector<float>> a(synth_f32(n, 5, p)), r(n);
            c.allreduce(a, r, Function<std::vector<float>>(Op::sum));
            got[mode][p] = r.get();
            on_device[mode][p] = c.last_host_combine_on_device();
        });
    for (int p = 0; p < 2; ++p) {
        CHECK(!on_device[0][p]);
        CHECK(on_device[1][p]);
        CHECK(on_device[2][p]);
        CHECK(std::memcmp(got[0][p].data(), got[1][p].data(), n * 4) == 0);
        CHECK(std::memcmp(got[0][p].data(), got[2][p].data(), n * 4) == 0);
    }
}

GPU_TEST(pageable_host_combine_sets_no_error_text) {
    // VERDICT r05 item 4 / ADVICE r05: a pageable bucket is the ordinary answer of the per-combine pinning probe,
    // not an error. Below the policy's smallest GPU size no probe runs; above it the probe is a query
    // (fmi_host_page_locked). Either way the peer thread's fmi_last_error() stays empty and the combine stays on
    // the host (Loopback runs each combine on the peer's own thread).
    for (std::size_t n : {std::size_t(1) << 18, (std::size_t(40) << 20) / 4 + 3}) {
        bool clean[2] = {}, on_device[2] = {true, true};
        with_peers(2, [&](Communicator& c, peer_num p) {
            c.use_device(0);
            Data<std::vector<float>> a(synth_f32(n, 9, p)), r(n);
            c.allreduce(a, r, Function<std::vector<float>>(Op::sum));
            clean[p] = std::string(fmi_last_error()).empty();
            on_device[p] = c.last_host_combine_on_device();
        });
        for (int p = 0; p < 2; ++p) {
            CHECK(clean[p]);
            CHECK(!on_device[p]);
        }
    }
}

GPU_TEST(bucket_group_places_each_bucket_by_index) {
    // Dev::Bucket<A>::group (fmi_dev_alloc_group): bucket j in 4 KiB slot j mod 16 modulo 64 KiB,
    // whatever was allocated before; each is a working bucket freed by its destructor
    Dev::init(0);
    const std::size_t n = (std::size_t(1) << 20) / 4 + 7;
    Dev::Bucket<float> before(n);
    auto g = Dev::Bucket<float>::group(18, n);
    CHECK(g.size() == 18);
    for (std::size_t j = 0; j < g.size(); ++j) {
        CHECK((reinterpret_cast<std::uintptr_t>(g[j].data()) % 65536) / 4096 == j % 16);
        CHECK(g[j].size() == n);
    }
    g[3].fill_synthetic(4, 1);
    const std::vector<float> x = g[3].download();
    g[17].upload(x);
    CHECK(std::memcmp(g[17].download().data(), x.data(), n * sizeof(float)) == 0);
}

GPU_TEST(device_buckets_need_builtin_op) {
    Dev::init(0);
    with_peers(1, [](Communicator& c, peer_num) {
        Data<Dev::Bucket<float>> a(4), r(4);
        Function<Dev::Bucket<float>> user([](Dev::Bucket<float> x, Dev::Bucket<float>) { return x; }, true, true);
        CHECK_THROWS(c.allreduce(a, r, user), std::runtime_error);
    });
}

// ---- dump mode -----------------------------------------------------------------------------------------
static int dump(const std::string& kind, peer_num P, std::size_t n, const std::string& out, const std::string& mode) {
    std::vector<std::vector<float>> recv(P), send(P);
    if (mode != "host") Dev::init(0);
    const bool ordered = kind.size() > 4 && kind.substr(kind.size() - 4) == "_ltr";
    const std::string base = ordered ? kind.substr(0, kind.size() - 4) : kind;
    auto run = [&](Communicator& c, peer_num p, auto& a, auto& r, auto f) {
        if (base == "allreduce") c.allreduce(a, r, f);
        else if (base == "reduce") c.reduce(a, r, 0, f);
        else if (base == "scan") c.scan(a, r, f);
        else throw std::runtime_error("unknown kind " + kind);
        recv[p] = r.get();
        send[p] = a.get();
    };
    with_peers(P, [&](Communicator& c, peer_num p) {
        if (mode == "device") {
            Data<Dev::Bucket<float>> a(synth_f32(n, 42, p)), r(n);
            Function<Dev::Bucket<float>> f(Op::sum);
            if (ordered) {
                f.commutative = false;
                f.associative = false;
            }
            run(c, p, a, r, f);
        } else {
            if (mode == "offload") c.use_device(0, true);  // every combine on the GPU
            Data<std::vector<float>> a(synth_f32(n, 42, p)), r(n);
            Function<std::vector<float>> f(Op::sum);
            if (ordered) {
                f.commutative = false;
                f.associative = false;
            }
            run(c, p, a, r, f);
        }
    });
    std::ofstream f(out, std::ios::binary);
    for (auto& v : recv) f.write(reinterpret_cast<const char*>(v.data()), static_cast<std::streamsize>(n * 4));
    for (auto& v : send) f.write(reinterpret_cast<const char*>(v.data()), static_cast<std::streamsize>(n * 4));
    return g_failures.load() ? 1 : 0;
}

// --dump-move KIND P N ROOT OUT (KIND = bcast | gather | scatter, host buckets over the Loopback channel): the
// data-movement collectives, for a check against the reference's own PeerToPeer (tests/test_cpp_communicator.py).
// Written per peer: bcast the peer's bucket after the call (n); gather the root's P x n receive buffer on the
// root, zeros elsewhere; scatter the peer's received n-element slice of the root's P x n bucket.
static int dump_move(const std::string& kind, peer_num P, std::size_t n, peer_num root, const std::string& out) {
    std::vector<std::vector<float>> got(P);
    with_peers(P, [&](Communicator& c, peer_num p) {
        if (kind == "bcast") {
            Data<std::vector<float>> b(synth_f32(n, 42, p));
            c.bcast(b, root);
            got[p] = b.get();
        } else if (kind == "gather") {
            Data<std::vector<float>> a(synth_f32(n, 42, p)), r(p == root ? P * n : n);
            c.gather(a, r, root);
            got[p] = p == root ? r.get() : std::vector<float>(P * n, 0.0f);
        } else if (kind == "scatter") {
            Data<std::vector<float>> a(synth_f32(P * n, 42, p)), r(n);
            c.scatter(a, r, root);
            got[p] = r.get();
        } else {
            throw std::runtime_error("unknown kind " + kind);
        }
    });
    std::ofstream f(out, std::ios::binary);
    for (auto& v : got) f.write(reinterpret_cast<const char*>(v.data()), static_cast<std::streamsize>(v.size() * 4));
    return g_failures.load() ? 1 : 0;
}

// --proc-channel P: P peers as fork()ed processes (forked before anything touches the GPU), each with a
// LocalSocket channel and an Rccl channel over the PROC transport (every process on GPU 0). Device-bucket
// allreduce / scan / reduce / bcast through the Rccl channel must equal, bit for bit, the same collectives
// on host buckets through the socket channel. Exit status 0 = every peer agreed.
static int proc_channel(peer_num P) {
    const std::size_t n = 300007;
    FMI::Comm::SocketMesh mesh(P);
    std::vector<pid_t> kids;
    for (peer_num p = 0; p < P; ++p) {
        const pid_t pid = fork();
        if (pid != 0) {
            kids.push_back(pid);
            continue;
        }
        int bad = 0;
        try {
            Communicator c(p, P, "", "proc-test");
            auto sock = std::make_shared<FMI::Comm::LocalSocket>(mesh.claim(p), 60000);
            c.register_channel("Local", sock);
            std::vector<float> host_ar, host_sc, host_red;
            {
                Data<std::vector<float>> a(synth_f32(n, 5, p)), r(n);
                c.allreduce(a, r, Function<std::vector<float>>(Op::sum));
                host_ar = r.get();
                Data<std::vector<float>> sc(synth_f32(n, 5, p)), sr(n);
                c.scan(sc, sr, Function<std::vector<float>>(Op::sum));
                host_sc = sr.get();
                Data<std::vector<float>> d(synth_f32(n, 5, p)), dr(n);
                c.reduce(d, dr, 1 % P, Function<std::vector<float>>(Op::sum));
                host_red = dr.get();
            }
            Dev::init(0);
            c.register_channel("Rccl", FMI::Comm::Rccl::connect(*sock, p, P, FMI_TRANSPORT_PROC));
            Data<Dev::Bucket<float>> a(synth_f32(n, 5, p)), r(n);
            c.allreduce(a, r, Function<Dev::Bucket<float>>(Op::sum));
            bad += std::memcmp(r.get().data(), host_ar.data(), n * 4) != 0;
            Data<Dev::Bucket<float>> sc(synth_f32(n, 5, p)), sr(n);
            c.scan(sc, sr, Function<Dev::Bucket<float>>(Op::sum));
            bad += std::memcmp(sr.get().data(), host_sc.data(), n * 4) != 0;
            Data<Dev::Bucket<float>> d(synth_f32(n, 5, p)), dr(n);
            c.reduce(d, dr, 1 % P, Function<Dev::Bucket<float>>(Op::sum));
            if (p == 1 % P) bad += std::memcmp(dr.get().data(), host_red.data(), n * 4) != 0;
            Data<Dev::Bucket<int64_t>> b(std::vector<int64_t>{static_cast<int64_t>(p), 9});
            c.bcast(b, P - 1);
            bad += b.get()[0] != static_cast<int64_t>(P - 1);
            c.barrier();
        } catch (const std::exception& e) {
            std::fprintf(stderr, "peer %u threw: %s\n", p, e.what());
            _exit(3);
        }
        if (bad) std::fprintf(stderr, "peer %u: %d mismatching results\n", p, bad);
        _exit(bad ? 1 : 0);
    }
    int rc = 0;
    for (pid_t k : kids) {
        int status = 0;
        waitpid(k, &status, 0);
        if (!WIFEXITED(status) || WEXITSTATUS(status) != 0) rc = 1;
    }
    std::fprintf(stderr, "proc_channel P=%u: %s\n", P, rc ? "FAIL" : "OK");
    return rc;
}

int main(int argc, char** argv) {
    std::vector<std::string> args(argv + 1, argv + argc);
    if (args.size() == 2 && args[0] == "--proc-channel") return proc_channel(static_cast<peer_num>(std::stoul(args[1])));
    if (args.size() == 6 && args[0] == "--dump-move")
        return dump_move(args[1], static_cast<peer_num>(std::stoul(args[2])), std::stoull(args[3]),
                         static_cast<peer_num>(std::stoul(args[4])), args[5]);
    if (!args.empty() && args[0] == "--dump") {
        if (args.size() < 5) return 2;
        const std::string mode = args.size() > 5 ? args[5].substr(2) : "host";
        return dump(args[1], static_cast<peer_num>(std::stoul(args[2])), std::stoull(args[3]), args[4], mode);
    }
    bool gpu = false;
    std::string filter;
    for (const auto& a : args) {
        if (a == "--gpu") gpu = true;
        else filter = a;
    }
    int ran = 0;
    for (const auto& t : registry()) {
        if (t.gpu != gpu) continue;  // --gpu runs the device tests, the default run the host tests
        if (!filter.empty() && t.name.find(filter) == std::string::npos) continue;
        const int before = g_failures.load();
        std::fprintf(stderr, "[ RUN  ] %s\n", t.name.c_str());
        try {
            t.body();
        } catch (const std::exception& e) {
            ++g_failures;
            std::fprintf(stderr, "  threw: %s\n", e.what());
        }
        std::fprintf(stderr, "[ %s ] %s\n", g_failures.load() == before ? " OK " : "FAIL", t.name.c_str());
        ++ran;
    }
    std::fprintf(stderr, "%d tests, %d failed checks\n", ran, g_failures.load());
    return g_failures.load() == 0 ? 0 : 1;
}
