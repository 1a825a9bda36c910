// ORACLE — TEST INFRASTRUCTURE ONLY (built into oracle/_ref/libfmi_ref.so by oracle/Makefile; loaded only by
// tests/, tests/golden/make_ref_vectors.py and bench.py's cpu_baseline leg — never by the product, smoke() or
// bench.py's timed regions).
//
// Runs the REFERENCE's own collective algorithms — /root/reference/src/comm/PeerToPeer.cpp, compiled unmodified
// from where it lies and linked beside this file — over an in-memory transport, so that the float evaluation
// order of FMI's reduce / allreduce / scan comes from the reference itself rather than from a restatement.
//
// What is the reference and what is this harness:
//   * reference (compiled from /root/reference, never copied): PeerToPeer::{reduce, reduce_ltr, reduce_no_order,
//     allreduce, allreduce_no_order, scan, scan_ltr, scan_no_order, bcast, gather, scatter, barrier}
//     (src/comm/PeerToPeer.cpp:6-293) and the headers it includes (include/comm/{PeerToPeer,Channel,Data}.h,
//     include/utils/{Function,Common}.h).
//   * this harness: `Loopback`, a PeerToPeer channel — the plug-in point the reference defines for transports
//     (include/comm/PeerToPeer.h:47-50, send_object / recv_object; the reference's own Direct channel fills it
//     with TCP sockets, src/comm/Direct.cpp:25-45) — whose per-peer-pair FIFO mailboxes live in memory; the
//     peers run as threads; and the element-wise combine f.f(a, b): a[i] = op(a[i], b[i]) with the reference's
//     built-in functors (std::plus / std::multiplies / std::max / std::min, python/PythonCommunicator.h:131-149),
//     i.e. what Communicator::convert_to_raw_function (include/Communicator.h:180-189) hands the channel. That
//     adapter itself is not compiled: include/Communicator.h needs include/utils/Configuration.h and so
//     boost::property_tree, which the image lacks. Its copies do not change any value.
//   * not built: src/comm/Channel.cpp (the S3 / Redis / Direct factory and Channel's default gather / scatter /
//     allreduce, all overridden by PeerToPeer; it needs aws-sdk-cpp, hiredis and TCPunch). Both files are built
//     with -fno-rtti because Channel's type_info would be emitted there (key function Channel::gather); no code
//     of Channel.cpp runs on any path used here. No stand-in for any missing header or library is written.
//
// C-ABI (oracle/fmi_ref.py wraps it with ctypes):
//   fmi_ref_run   numeric collective over P peers' buckets: every peer's recvbuf and sendbuf after the call.
//   fmi_ref_expr  symbolic run: each element is a handle to an expression; f.f(a, b) makes "(a+b)" (left operand
//                 = arg 0 of f.f), so the result is the exact bracketing the reference evaluates.
//   fmi_ref_time_allreduce  CPU time of the reference's allreduce (bench.py's C1 / C2 rows of the CPU baseline).
//   fmi_ref_time_scan       CPU time of the reference's scan (bench.py's C3 row of the CPU baseline).
//   fmi_ref_time_combine    CPU time of the combine alone, on 1 or several concurrent threads (C2 row).
//   fmi_ref_run_bound / fmi_ref_time_allreduce_bound  the same reference collectives with f.f bound to a
//                 bucket-reduction C-ABI whose entry points the caller passes by address (INTEGRATION.md §B.2;
//                 tests/test_gpu_ref_binding.py binds libfmi_dev.so). Nothing of that library is linked here.
#include "comm/PeerToPeer.h"

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <new>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#define FMI_REF_API extern "C" __attribute__((visibility("default")))

namespace {

using FMI::Utils::peer_num;

// Per-peer-pair FIFO mailboxes: send never blocks (the reference's Direct channel writes into a socket
// buffer), recv blocks until the message from that peer is there and must read exactly buf.len bytes.
struct Mailbox {
    explicit Mailbox(int p) : P(p), q(static_cast<size_t>(p) * p) {}
    int P;
    std::mutex mu;
    std::condition_variable cv;
    std::vector<std::deque<std::vector<char>>> q;  // q[src * P + dst]
    std::string error;                              // first failure; every waiting peer gives up on it
    size_t dropped = 0;                             // sends to a peer id >= P (reference scan_ltr at P = 1)
    std::vector<std::vector<char>> pool;            // consumed message buffers, reused (no mmap / munmap per message)
};

constexpr double kRecvTimeoutS = 60.0;

class Loopback final : public FMI::Comm::PeerToPeer {
public:
    Loopback(Mailbox* mb, peer_num id, peer_num P) : mb_(mb) {
        set_peer_id(id);
        set_num_peers(P);  // (comm_name stays empty: PeerToPeer never reads it)
    }
    void send_object(channel_data buf, peer_num dst) override {
        std::lock_guard<std::mutex> lk(mb_->mu);
        if (dst >= static_cast<peer_num>(mb_->P)) {  // no such peer: nothing would ever read it
            ++mb_->dropped;
            return;
        }
        std::vector<char> msg;
        if (!mb_->pool.empty()) {
            msg = std::move(mb_->pool.back());
            mb_->pool.pop_back();
        }
        msg.assign(buf.buf, buf.buf + buf.len);
        mb_->q[static_cast<size_t>(peer_id) * mb_->P + dst].push_back(std::move(msg));
        mb_->cv.notify_all();
    }
    void recv_object(channel_data buf, peer_num src) override {
        std::unique_lock<std::mutex> lk(mb_->mu);
        if (src >= static_cast<peer_num>(mb_->P)) throw std::runtime_error("recv from a peer id >= P");
        auto& box = mb_->q[static_cast<size_t>(src) * mb_->P + peer_id];
        const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(kRecvTimeoutS);
        while (box.empty() && mb_->error.empty()) {
            if (mb_->cv.wait_until(lk, deadline) == std::cv_status::timeout && box.empty())
                throw FMI::Utils::Timeout();
        }
        if (!mb_->error.empty()) throw std::runtime_error("another peer failed");
        std::vector<char> msg = std::move(box.front());
        box.pop_front();
        if (msg.size() != buf.len)
            throw std::runtime_error("message of " + std::to_string(msg.size()) + " B received into a " +
                                     std::to_string(buf.len) + " B buffer");
        std::memcpy(buf.buf, msg.data(), msg.size());
        mb_->pool.push_back(std::move(msg));
    }
    double get_latency(peer_num, peer_num, std::size_t) override { return 0.0; }
    double get_price(peer_num, peer_num, std::size_t) override { return 0.0; }

private:
    Mailbox* mb_;
};

enum Coll { kAllreduce = 0, kReduce = 1, kScan = 2, kBcast = 3, kGather = 4, kScatter = 5, kBarrier = 6 };
enum Op { kSum = 0, kProd = 1, kMax = 2, kMin = 3, kSub = 4 };
enum Dtype { kF32 = 0, kF64 = 1, kI32 = 2, kI64 = 3, kU32 = 4, kU64 = 5 };

size_t dtype_size(int d) {
    switch (d) {
        case kF32: case kI32: case kU32: return 4;
        case kF64: case kI64: case kU64: return 8;
        default: return 0;
    }
}

// a[i] = op(a[i], b[i]) for i < n — the channel-level combine f.f(a, b) (a overwritten, b read-only).
template <typename T>
raw_func elementwise(int op, size_t n) {
    std::function<T(T, T)> g;
    switch (op) {
        case kSum: g = std::plus<T>(); break;
        case kProd: g = std::multiplies<T>(); break;
        case kMax: g = [](T a, T b) { return std::max(a, b); }; break;
        case kMin: g = [](T a, T b) { return std::min(a, b); }; break;
        default: g = std::minus<T>(); break;  // the reference KATs' non-commutative op
    }
    return [g, n](char* a, char* b) {
        T* x = reinterpret_cast<T*>(a);
        const T* y = reinterpret_cast<const T*>(b);
        std::transform(x, x + n, y, x, g);
    };
}

raw_func make_combine(int op, int dtype, size_t n) {
    switch (dtype) {
        case kF32: return elementwise<float>(op, n);
        case kF64: return elementwise<double>(op, n);
        case kI32: return elementwise<int32_t>(op, n);
        case kI64: return elementwise<int64_t>(op, n);
        case kU32: return elementwise<uint32_t>(op, n);
        default: return elementwise<uint64_t>(op, n);
    }
}

void set_err(char* err, size_t len, const std::string& msg) {
    if (!err || !len) return;
    const size_t k = std::min(len - 1, msg.size());
    std::memcpy(err, msg.data(), k);
    err[k] = '\0';
}

// Runs `body(channel, peer)` on P threads, one Loopback per peer. Returns "" or the first failure.
std::string run_peers(int P, const std::function<void(Loopback&, int)>& body, size_t* dropped) {
    Mailbox mb(P);
    std::vector<std::thread> th;
    th.reserve(P);
    for (int p = 0; p < P; ++p) {
        th.emplace_back([&, p] {
            try {
                // Built in place and never destroyed: Channel has no virtual destructor and its implicit one
                // would name Channel's vtable, which only the unbuilt Channel.cpp emits. Nothing is leaked:
                // the object holds a non-owning mailbox pointer and an empty in-place string.
                alignas(Loopback) unsigned char storage[sizeof(Loopback)];
                Loopback& ch = *new (storage) Loopback(&mb, static_cast<peer_num>(p), static_cast<peer_num>(P));
                body(ch, p);
            } catch (const std::exception& e) {
                std::lock_guard<std::mutex> lk(mb.mu);
                if (mb.error.empty()) mb.error = "peer " + std::to_string(p) + ": " + e.what();
                mb.cv.notify_all();
            }
        });
    }
    for (auto& t : th) t.join();
    if (mb.error.empty()) {
        for (const auto& box : mb.q)
            if (!box.empty()) return "unconsumed messages after the collective";
    }
    if (dropped) *dropped = mb.dropped;
    return mb.error;
}

}  // namespace

// Numeric collective. ins: P buckets of n elements (peer-major). recv_out / send_out: P buckets each, the
// recvbuf (pre-filled from recv_init when not null, else zero) and the sendbuf of every peer after the call.
// ordered = 1: the raw_function is flagged non-commutative (the reference then takes its LTR algorithms).
// root: reduce / bcast / gather / scatter root. gather's recvbuf at the root is P buckets (recv_out holds
// P * P buckets for gather: peer p's slot is recv_out + p * P * n). Returns 0, or -1 with a message in err.
FMI_REF_API int fmi_ref_run(int coll, int op, int dtype, int ordered, int P, int root, size_t n, const void* ins,
                            const void* recv_init, void* recv_out, void* send_out, size_t* dropped, char* err,
                            size_t errlen) {
    const size_t es = dtype_size(dtype);
    if (P < 1 || es == 0 || root < 0 || root >= P || (!ins && coll != kBarrier)) {
        set_err(err, errlen, "invalid argument");
        return -1;
    }
    const size_t S = n * es;
    const size_t recv_buckets = coll == kGather ? static_cast<size_t>(P) : 1;
    const size_t send_buckets = coll == kScatter ? static_cast<size_t>(P) : 1;
    std::vector<std::vector<char>> send(P), recv(P);
    for (int p = 0; p < P; ++p) {
        if (ins)
            send[p].assign(static_cast<const char*>(ins) + p * send_buckets * S,
                           static_cast<const char*>(ins) + (p + 1) * send_buckets * S);
        else
            send[p].assign(send_buckets * S, 0);
        recv[p].assign(recv_buckets * S, 0);
        if (recv_init)
            std::memcpy(recv[p].data(), static_cast<const char*>(recv_init) + p * recv_buckets * S, recv_buckets * S);
    }
    const raw_function f{make_combine(op, dtype, n), /*associative=*/true, /*commutative=*/ordered == 0};
    const std::string e = run_peers(
        P,
        [&](Loopback& ch, int p) {
            channel_data sd{send[p].data(), send[p].size()};
            channel_data rd{recv[p].data(), recv[p].size()};
            switch (coll) {
                case kAllreduce: ch.allreduce(sd, rd, f); break;
                case kReduce: ch.reduce(sd, rd, static_cast<peer_num>(root), f); break;
                case kScan: ch.scan(sd, rd, f); break;
                case kBcast: ch.bcast(sd, static_cast<peer_num>(root)); break;
                case kGather: ch.gather(sd, rd, static_cast<peer_num>(root)); break;
                case kScatter: ch.scatter(sd, rd, static_cast<peer_num>(root)); break;
                default: ch.barrier(); break;
            }
        },
        dropped);
    if (!e.empty()) {
        set_err(err, errlen, e);
        return -1;
    }
    for (int p = 0; p < P; ++p) {
        if (recv_out) std::memcpy(static_cast<char*>(recv_out) + p * recv_buckets * S, recv[p].data(), recv[p].size());
        if (send_out) std::memcpy(static_cast<char*>(send_out) + p * send_buckets * S, send[p].data(), send[p].size());
    }
    return 0;
}

// Symbolic collective (one element per bucket): the expression peer `rank` ends with in its recvbuf (reduce:
// the root's), written to buf as "x0", "(x0+x1)", ... ; `which` = 1 returns the sendbuf after the call instead.
// Returns the expression length (buf may be too small: call again with a larger one), or -1 with err.
FMI_REF_API long fmi_ref_expr(int coll, int ordered, int P, int rank, int root, int which, char* buf, size_t len,
                              char* err, size_t errlen) {
    if (P < 1 || rank < 0 || rank >= P || root < 0 || root >= P || coll < kAllreduce || coll > kScan) {
        set_err(err, errlen, "invalid argument");
        return -1;
    }
    std::mutex mu;  // the expression table is shared by the peer threads
    std::vector<std::string> table;
    for (int p = 0; p < P; ++p) table.push_back("x" + std::to_string(p));
    auto combine = [&](char* a, char* b) {
        std::lock_guard<std::mutex> lk(mu);
        int32_t ia, ib;
        std::memcpy(&ia, a, 4);
        std::memcpy(&ib, b, 4);
        const std::string e = "(" + table.at(ia) + "+" + table.at(ib) + ")";
        table.push_back(e);
        const int32_t h = static_cast<int32_t>(table.size() - 1);
        std::memcpy(a, &h, 4);
    };
    const raw_function f{combine, true, ordered == 0};
    std::vector<int32_t> send(P), recv(P, -1);
    for (int p = 0; p < P; ++p) send[p] = p;
    const std::string e = run_peers(
        P,
        [&](Loopback& ch, int p) {
            channel_data sd{reinterpret_cast<char*>(&send[p]), 4};
            channel_data rd{reinterpret_cast<char*>(&recv[p]), 4};
            if (coll == kAllreduce) ch.allreduce(sd, rd, f);
            else if (coll == kReduce) ch.reduce(sd, rd, static_cast<peer_num>(root), f);
            else ch.scan(sd, rd, f);
        },
        nullptr);
    if (!e.empty()) {
        set_err(err, errlen, e);
        return -1;
    }
    const int who = coll == kReduce && which == 0 ? root : rank;
    const int32_t h = which ? send[who] : recv[who];
    if (h < 0 || h >= static_cast<int32_t>(table.size())) {
        set_err(err, errlen, "no value in that buffer");
        return -1;
    }
    const std::string& s = table[h];
    if (buf && len) {
        const size_t k = std::min(len - 1, s.size());
        std::memcpy(buf, s.data(), k);
        buf[k] = '\0';
    }
    return static_cast<long>(s.size());
}

// ---- The reference's combine site bound to a bucket-reduction C-ABI --------------------
// The entry points of such a library, passed in BY ADDRESS by the caller (tests/test_gpu_ref_binding.py takes
// them from libfmi_dev.so with ctypes): this file links nothing of the product and names none of its symbols.
// The signatures are those of include/fmi_dev.h; op ids (0 sum, 1 prod, 2 max, 3 min) and dtype ids (0 f32,
// 1 f64, 2 i32, 3 i64, 4 u32, 5 u64) coincide with this harness's own.
struct RefBinding {
    int (*host_pair)(int op, int dtype, void* inout, const void* in, size_t n);             // fmi_host_reduce_pair
    int (*dev_pair)(int op, int dtype, void* inout, const void* in, size_t n, void* stream); // fmi_dev_reduce_pair
    int (*stream_sync)(void* stream);                                                        // fmi_stream_sync
    const char* (*last_error)(void);                                                         // fmi_last_error
};

namespace {

// The raw_func §B.2 builds for a tagged Function: f.f(a, b) = "a = op(a, b)" through the library.
//   host entry point (dev_pair null): fmi_host_reduce_pair on whatever host memory the reference hands the
//     combine — the caller's buckets and the reference's own `new char[]` temporaries (PeerToPeer.cpp:47,63).
//   device entry point: fmi_dev_reduce_pair on the library stream + fmi_stream_sync, for buckets the GPU
//     addresses directly (page-locked, mapped). Operands outside [lo[k], lo[k] + len) of the `mapped` ranges
//     (the reference's pageable temporaries) are refused with an exception, never handed to a kernel.
raw_func bound_combine(const RefBinding& b, int op, int dtype, size_t n, std::vector<std::pair<const char*, size_t>> mapped) {
    const size_t bytes = n * dtype_size(dtype);
    return [b, op, dtype, n, bytes, mapped](char* x, char* y) {
        int rc;
        if (b.dev_pair) {
            for (const char* p : {static_cast<const char*>(x), static_cast<const char*>(y)}) {
                bool inside = false;
                for (const auto& r : mapped) inside = inside || (p >= r.first && p + bytes <= r.first + r.second);
                if (!inside) throw std::runtime_error("device binding: a combine operand is not a device-mapped bucket "
                                                      "(the reference's pageable temporary); use the host entry point");
            }
            rc = b.dev_pair(op, dtype, x, y, n, nullptr);
            if (rc == 0) rc = b.stream_sync(nullptr);
        } else {
            rc = b.host_pair(op, dtype, x, y, n);
        }
        if (rc != 0)
            throw std::runtime_error(std::string("bound combine failed (") + std::to_string(rc) + "): " +
                                     (b.last_error ? b.last_error() : ""));
    };
}

}  // namespace

// fmi_ref_run with the reference's combine bound to a C-ABI (struct RefBinding above) instead of the harness's
// std functors: the same PeerToPeer code, the same transport, only f.f differs. bufs: null (every peer's
// sendbuf / recvbuf are the harness's pageable vectors), or 2 * P caller-owned host-addressable buckets —
// bufs[p] = peer p's sendbuf, bufs[P + p] its recvbuf, each of n elements (page-locked and device-mapped for
// the device entry point, which requires them). ins / recv_init / recv_out / send_out as for fmi_ref_run
// (allreduce / reduce / scan only). Returns 0, or -1 with the first failure in err.
FMI_REF_API int fmi_ref_run_bound(int coll, int op, int dtype, int ordered, int P, int root, size_t n, const void* ins,
                                  const void* recv_init, void* recv_out, void* send_out, const RefBinding* binding,
                                  void* const* bufs, char* err, size_t errlen) {
    const size_t es = dtype_size(dtype);
    if (P < 1 || es == 0 || root < 0 || root >= P || !ins || !binding || coll < kAllreduce || coll > kScan ||
        op < kSum || op > kMin || (!binding->host_pair && !binding->dev_pair) ||
        (binding->dev_pair && (!binding->stream_sync || !bufs))) {
        set_err(err, errlen, "invalid argument");
        return -1;
    }
    const size_t S = n * es;
    std::vector<std::vector<char>> own(bufs ? 0 : 2 * static_cast<size_t>(P), std::vector<char>(S));
    std::vector<char*> send(P), recv(P);
    std::vector<std::pair<const char*, size_t>> mapped;
    for (int p = 0; p < P; ++p) {
        send[p] = bufs ? static_cast<char*>(bufs[p]) : own[p].data();
        recv[p] = bufs ? static_cast<char*>(bufs[P + p]) : own[P + p].data();
        if (S) {
            std::memcpy(send[p], static_cast<const char*>(ins) + p * S, S);
            if (recv_init) std::memcpy(recv[p], static_cast<const char*>(recv_init) + p * S, S);
            else std::memset(recv[p], 0, S);
        }
        mapped.emplace_back(send[p], S);
        mapped.emplace_back(recv[p], S);
    }
    const raw_function f{bound_combine(*binding, op, dtype, n, mapped), /*associative=*/true,
                         /*commutative=*/ordered == 0};
    const std::string e = run_peers(
        P,
        [&](Loopback& ch, int p) {
            channel_data sd{send[p], S};
            channel_data rd{recv[p], S};
            switch (coll) {
                case kAllreduce: ch.allreduce(sd, rd, f); break;
                case kReduce: ch.reduce(sd, rd, static_cast<peer_num>(root), f); break;
                default: ch.scan(sd, rd, f); break;
            }
        },
        nullptr);
    if (!e.empty()) {
        set_err(err, errlen, e);
        return -1;
    }
    for (int p = 0; p < P && S; ++p) {
        if (recv_out) std::memcpy(static_cast<char*>(recv_out) + p * S, recv[p], S);
        if (send_out) std::memcpy(static_cast<char*>(send_out) + p * S, send[p], S);
    }
    return 0;
}

namespace {

// Reusable barrier for the peer threads of fmi_ref_time.
class Barrier {
public:
    explicit Barrier(int n) : n_(n) {}
    void wait() {
        std::unique_lock<std::mutex> lk(mu_);
        const long gen = gen_;
        if (++count_ == n_) {
            count_ = 0;
            ++gen_;
            cv_.notify_all();
            return;
        }
        cv_.wait(lk, [&] { return gen_ != gen; });
    }

private:
    int n_;
    int count_ = 0;
    long gen_ = 0;
    std::mutex mu_;
    std::condition_variable cv_;
};

}  // namespace

namespace {

// P peer threads run the reference's allreduce (coll = kAllreduce) or scan (kScan) of n-element f32 buckets.
int time_collective(int coll, int P, size_t n, int reps, const raw_func& f, double* median_ms, char* err,
                    size_t errlen) {
    const size_t S = n * sizeof(float);
    std::vector<std::vector<float>> init(P, std::vector<float>(n)), send(P), recv(P, std::vector<float>(n));
    for (int p = 0; p < P; ++p)
        for (size_t i = 0; i < n; ++i) init[p][i] = static_cast<float>((i * 2654435761u + p * 40503u) % 2048) / 1024.0f - 1.0f;
    const raw_function rf{f, true, true};
    Barrier bar(P);
    std::vector<double> ms(reps);
    const std::string e = run_peers(
        P,
        [&](Loopback& ch, int p) {
            for (int r = 0; r < reps; ++r) {
                send[p] = init[p];
                bar.wait();
                const auto t0 = std::chrono::steady_clock::now();
                const channel_data sd{reinterpret_cast<char*>(send[p].data()), S};
                const channel_data rd{reinterpret_cast<char*>(recv[p].data()), S};
                if (coll == kScan)
                    ch.scan(sd, rd, rf);
                else
                    ch.allreduce(sd, rd, rf);
                bar.wait();
                if (p == 0) ms[r] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            }
        },
        nullptr);
    if (!e.empty()) {
        set_err(err, errlen, e);
        return -1;
    }
    std::sort(ms.begin(), ms.end());
    *median_ms = ms[ms.size() / 2];
    return 0;
}

}  // namespace

namespace {

// The raw_func Communicator::convert_to_raw_function builds for a Data<std::vector<float>> bucket
// (include/Communicator.h:180-189, restated: that header needs boost) around the reference's own
// FMI::Utils::Function (include/utils/Function.h, compiled here: its operator() takes both buckets by value and
// calls the std::function, which copies them again) holding the Python layer's built-in sum
// (python/PythonCommunicator.h:131-149: get_vec_function's SUM, std::transform with std::plus into its first
// by-value argument, which it returns).
raw_func reference_adapter(size_t n) {
    const size_t S = n * sizeof(float);
    const FMI::Utils::Function<std::vector<float>> user(  // get_vec_function's SUM, PythonCommunicator.h:135
        [](std::vector<float> a, std::vector<float> b) {
            std::transform(a.begin(), a.end(), b.begin(), a.begin(), std::plus<float>());
            return a;
        },
        true, true);
    return [user, S](char* a, char* b) {
        std::vector<float> va(reinterpret_cast<float*>(a), reinterpret_cast<float*>(a + S));
        std::vector<float> vb(reinterpret_cast<float*>(b), reinterpret_cast<float*>(b + S));
        std::vector<float> res = user(va, vb);
        std::memcpy(a, res.data(), S);
    };
}

}  // namespace

// The combine alone, outside any collective: `threads` threads each apply the f32 sum combine (adapter = 1: the
// reference's vector adapter; 0: std::transform in place) to their own pair of n-element buckets at the same
// time, released together by a barrier; the time of one repetition is the slowest thread's. With threads = 1 it
// is what oracle/cpu_baseline.cpp times; with threads = P it is the load the P peers of an allreduce put on the
// host at once (bench.py's cpu_baseline.c2_reference separates the two). Writes the median of `reps`, after one
// untimed warm-up.
FMI_REF_API int fmi_ref_time_combine(int threads, size_t n, int reps, int adapter, double* median_ms, char* err,
                                     size_t errlen) {
    if (threads < 1 || reps < 1 || !median_ms) {
        set_err(err, errlen, "invalid argument");
        return -1;
    }
    const raw_func f = adapter ? reference_adapter(n) : make_combine(kSum, kF32, n);
    std::vector<std::vector<float>> a(threads, std::vector<float>(n)), b(threads, std::vector<float>(n));
    for (int t = 0; t < threads; ++t)
        for (size_t i = 0; i < n; ++i) {
            a[t][i] = static_cast<float>((i * 2654435761u + t * 40503u) % 2048) / 1024.0f - 1.0f;
            b[t][i] = static_cast<float>((i * 40503u + t * 2654435761u) % 2048) / 1024.0f - 1.0f;
        }
    Barrier bar(threads);
    std::vector<std::vector<double>> ms(threads, std::vector<double>(reps));
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t)
        th.emplace_back([&, t] {
            for (int r = -1; r < reps; ++r) {  // r = -1: one untimed warm-up, as oracle/cpu_baseline.cpp does
                bar.wait();
                const auto t0 = std::chrono::steady_clock::now();
                f(reinterpret_cast<char*>(a[t].data()), reinterpret_cast<char*>(b[t].data()));
                if (r >= 0)
                    ms[t][r] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
                bar.wait();
            }
        });
    for (auto& x : th) x.join();
    std::vector<double> slowest(reps, 0.0);
    for (int r = 0; r < reps; ++r)
        for (int t = 0; t < threads; ++t) slowest[r] = std::max(slowest[r], ms[t][r]);
    std::sort(slowest.begin(), slowest.end());
    *median_ms = slowest[reps / 2];
    return 0;
}

// fmi_ref_time_allreduce with the combine bound to a C-ABI's host entry point (the
// reference's own allreduce, every f.f a fmi_host_reduce_pair on the harness's pageable buckets).
FMI_REF_API int fmi_ref_time_allreduce_bound(int P, size_t n, int reps, const RefBinding* binding, double* median_ms,
                                             char* err, size_t errlen) {
    if (P < 1 || reps < 1 || !median_ms || !binding || !binding->host_pair) {
        set_err(err, errlen, "invalid argument");
        return -1;
    }
    RefBinding host_only = *binding;
    host_only.dev_pair = nullptr;
    return time_collective(kAllreduce, P, n, reps, bound_combine(host_only, kSum, kF32, n, {}), median_ms, err, errlen);
}

// CPU timing of the reference's own allreduce (PeerToPeer::allreduce -> allreduce_no_order, f32 sum) over P
// peer threads and the in-memory transport: bench.py's cpu_baseline leg reports it for config C1 (2 peers,
// 1 MiB) beside the C++ port. adapter = 1: the combine is the reference's vector adapter as Communicator
// builds it for Data<std::vector<float>> (include/Communicator.h:180-189: both buckets copied into vectors,
// the reference's own FMI::Utils::Function called by value, the result memcpy'd back) around the Python layer's
// std::transform(std::plus) (python/PythonCommunicator.h:131-149) — the lambda restated (reference_adapter),
// since Communicator.h cannot be compiled (boost::property_tree); adapter = 0: std::transform in place; adapter = 2: a no-op
// combine, i.e. the collective's transport and copies alone (what separates the allreduce from its combine). Every repetition starts
// from the same buckets (restored outside the timed span); the time of one repetition is peer 0's, from a
// barrier that releases every peer to a barrier every peer reaches after its allreduce. Writes the median.
FMI_REF_API int fmi_ref_time_allreduce(int P, size_t n, int reps, int adapter, double* median_ms, char* err,
                                       size_t errlen) {
    if (P < 1 || reps < 1 || !median_ms) {
        set_err(err, errlen, "invalid argument");
        return -1;
    }
    raw_func f;
    if (adapter == 1) {
        f = reference_adapter(n);
    } else if (adapter == 2) {
        f = [](char*, char*) {};  // the reference's own no-op combine (its barrier, PeerToPeer.cpp:30)
    } else {
        f = make_combine(kSum, kF32, n);
    }
    return time_collective(kAllreduce, P, n, reps, f, median_ms, err, errlen);
}

// The same for the reference's scan (PeerToPeer::scan -> scan_no_order, f32 sum; PeerToPeer.cpp:132-184): bench.py's
// cpu_baseline reports it beside config C3's peer scan (8 peers x 64 MiB). adapter as for fmi_ref_time_allreduce.
FMI_REF_API int fmi_ref_time_scan(int P, size_t n, int reps, int adapter, double* median_ms, char* err,
                                  size_t errlen) {
    if (P < 1 || reps < 1 || !median_ms) {
        set_err(err, errlen, "invalid argument");
        return -1;
    }
    const raw_func f = adapter == 1 ? reference_adapter(n) : make_combine(kSum, kF32, n);
    return time_collective(kScan, P, n, reps, f, median_ms, err, errlen);
}
