// FMI::Comm::PeerToPeer — collectives for directly addressable peers (mirrors reference
// include/comm/PeerToPeer.h and src/comm/PeerToPeer.cpp). Transports implement send_object / recv_object;
// everything else — and in particular the combine ORDER of reduce / allreduce / scan — is fixed here and
// is identical to the reference's (verified against fmi_amd/csrc/fmi_schedule.h and the oracle by
// tests/test_cpp_communicator.py).
//
// Device-resident buckets (channel_data::on_device): transfers are staged through a page-locked host
// buffer owned by the channel, temporaries are allocated in HBM, and the combine `f.f` is the HIP kernel
// closure the Communicator built, so a PeerToPeer transport carries device buckets unchanged.
#ifndef FMI_AMD_COMM_PEERTOPEER_H
#define FMI_AMD_COMM_PEERTOPEER_H

#include <cmath>
#include <condition_variable>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <utility>
#include <vector>

#include "Channel.h"

namespace FMI::Comm {

//! One background thread that runs the chunk combines of an overlapped transfer, one job at a time (the
//! thread starts on first use, so channels that never overlap never create it).
class CombineWorker {
public:
    CombineWorker() = default;
    CombineWorker(const CombineWorker&) = delete;
    CombineWorker& operator=(const CombineWorker&) = delete;
    ~CombineWorker() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            quit_ = true;
        }
        cv_.notify_all();
        if (thread_.joinable()) thread_.join();
    }

    //! Queue `job` once the previous one has finished (rethrowing what that one threw).
    void submit(std::function<void()> job) {
        wait();
        std::lock_guard<std::mutex> lk(mu_);
        if (!thread_.joinable()) thread_ = std::thread([this] { loop(); });
        job_ = std::move(job);
        busy_ = true;
        cv_.notify_all();
    }

    //! Block until no job is running; rethrow the exception of the last one, if any.
    void wait() {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return !busy_; });
        if (error_) std::rethrow_exception(std::exchange(error_, nullptr));
    }

    //! wait() for use on an error path: never throws.
    void drain() noexcept {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return !busy_; });
        error_ = nullptr;
    }

private:
    void loop() {
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            cv_.wait(lk, [&] { return busy_ || quit_; });
            if (!busy_) return;  // quit with nothing pending
            std::function<void()> job = std::move(job_);
            lk.unlock();
            std::exception_ptr err;
            try {
                job();
            } catch (...) {
                err = std::current_exception();
            }
            lk.lock();
            error_ = err;
            busy_ = false;
            cv_.notify_all();
        }
    }

    std::mutex mu_;
    std::condition_variable cv_;
    std::thread thread_;
    std::function<void()> job_;
    std::exception_ptr error_;
    bool busy_ = false;
    bool quit_ = false;
};

class PeerToPeer : public Channel {
public:
    ~PeerToPeer() override { release_staging(); }

    //! Transport primitives the concrete channel provides (reference PeerToPeer.h:47-50).
    virtual void send_object(channel_data buf, Utils::peer_num peer) = 0;
    virtual void recv_object(channel_data buf, Utils::peer_num peer) = 0;

    //! A byte-stream transport (no message framing): one send_object may be received as several
    //! consecutive recv_objects and vice versa, which is what lets a combine overlap the transfer.
    virtual bool stream_transport() const { return false; }

    //! Chunk size of the overlapped transfer + combine on stream transports (0 = never overlap, the
    //! default: fmi_amd/cpp/tools/c1_bench.cpp measured it 5-20 % faster at 64 MiB but up to 2.4x slower
    //! at 16 and 256 MiB on the GPU box's 256-thread EPYC host, where the worker thread's combine reads
    //! pieces the receiving thread just wrote, often from another CCD).
    void set_overlap_chunk(std::size_t bytes) { overlap_chunk_ = bytes; }
    std::size_t overlap_chunk() const { return overlap_chunk_; }
    //! Pieces moved by overlapped transfers so far (introspection for tests and benchmarks).
    std::size_t overlapped_pieces() const { return overlapped_pieces_; }

    void send(channel_data buf, Utils::peer_num dest) override {
        if (!buf.on_device) return send_object(buf, dest);
        char* host = staging(buf.len);
        Dev::copy_bytes(host, false, buf.buf, true, buf.len);
        send_object({host, buf.len}, dest);
    }

    void recv(channel_data buf, Utils::peer_num src) override {
        if (!buf.on_device) return recv_object(buf, src);
        char* host = staging(buf.len);
        recv_object({host, buf.len}, src);
        Dev::copy_bytes(buf.buf, true, host, false, buf.len);
    }

    //! Binomial broadcast from `root` (reference PeerToPeer.cpp:14-27).
    void bcast(channel_data buf, Utils::peer_num root) override {
        const unsigned v = virt(peer_id, root);
        for (int i = ceil_log2(num_peers) - 1; i >= 0; --i) {
            const unsigned step = 1u << i;
            if (v % (2 * step) == 0 && v + step < num_peers)
                send(buf, real(v + step, root));
            else if (v % step == 0 && v % (2 * step) != 0)
                recv(buf, real(v - step, root));
        }
    }

    //! Allreduce of one byte with a no-op combine (reference PeerToPeer.cpp:29-33).
    void barrier() override {
        char token = 1;
        raw_function nop{[](char*, char*) {}, true, true};
        allreduce({&token, 1}, {&token, 1}, nop);
    }

    //! Binomial gather; the root's recvbuf receives the buckets in real peer order
    //! (reference PeerToPeer.cpp:186-239, wraparound for root != 0).
    void gather(channel_data sendbuf, channel_data recvbuf, Utils::peer_num root) override {
        const std::size_t S = sendbuf.len;
        const unsigned v = virt(peer_id, root);
        const bool dev = sendbuf.on_device;
        // Subtree buffer in virtual order: [v, v + held). The root of peer 0 gathers straight into recvbuf.
        Dev::Scratch own;
        char* mine;
        bool mine_dev;
        if (peer_id == root && root == 0) {
            mine = recvbuf.buf;
            mine_dev = recvbuf.on_device;
        } else {
            own = Dev::Scratch(S * subtree_size(v), dev);
            mine = own.get();
            mine_dev = dev;
        }
        Dev::copy_bytes(mine, mine_dev, sendbuf.buf, dev, S);
        for (int i = 0; i < ceil_log2(num_peers); ++i) {
            const unsigned step = 1u << i;
            if (v % (2 * step) == 0 && v + step < num_peers) {
                const unsigned count = std::min(step, num_peers - (v + step));
                recv({mine + step * S, count * S, mine_dev}, real(v + step, root));
            } else if (v % step == 0 && v % (2 * step) != 0) {
                const unsigned count = std::min(step, num_peers - v);
                send({mine, count * S, mine_dev}, real(v - step, root));
            }
        }
        if (peer_id == root && root != 0) {
            // virtual slot t holds real peer (t + root) % P: rotate into real order
            const std::size_t tail = (num_peers - root) * S;  // virtual [0, P-root) -> real [root, P)
            Dev::copy_bytes(recvbuf.buf + root * S, recvbuf.on_device, mine, mine_dev, tail);
            Dev::copy_bytes(recvbuf.buf, recvbuf.on_device, mine + tail, mine_dev, root * S);
        }
    }

    //! Binomial scatter of root's sendbuf (real peer order) (reference PeerToPeer.cpp:241-285).
    void scatter(channel_data sendbuf, channel_data recvbuf, Utils::peer_num root) override {
        const std::size_t S = recvbuf.len;
        const unsigned v = virt(peer_id, root);
        const bool dev = recvbuf.on_device;
        Dev::Scratch own;
        char* mine = nullptr;
        bool mine_dev = dev;
        if (peer_id == root) {
            mine_dev = sendbuf.on_device;
            if (root == 0) {
                mine = sendbuf.buf;
            } else {  // rotate into virtual order first
                own = Dev::Scratch(S * num_peers, mine_dev);
                mine = own.get();
                const std::size_t tail = (num_peers - root) * S;
                Dev::copy_bytes(mine, mine_dev, sendbuf.buf + root * S, sendbuf.on_device, tail);
                Dev::copy_bytes(mine + tail, mine_dev, sendbuf.buf, sendbuf.on_device, root * S);
            }
        } else {
            own = Dev::Scratch(S * subtree_size(v), dev);
            mine = own.get();
        }
        for (int i = ceil_log2(num_peers) - 1; i >= 0; --i) {
            const unsigned step = 1u << i;
            if (v % (2 * step) == 0 && v + step < num_peers) {
                const unsigned count = std::min(step, num_peers - (v + step));
                send({mine + step * S, count * S, mine_dev}, real(v + step, root));
            } else if (v % step == 0 && v % (2 * step) != 0) {
                const unsigned count = std::min(step, num_peers - v);
                recv({mine, count * S, mine_dev}, real(v - step, root));
            }
        }
        Dev::copy_bytes(recvbuf.buf, recvbuf.on_device, mine, mine_dev, S);
    }

    void reduce(channel_data sendbuf, channel_data recvbuf, Utils::peer_num root, raw_function f) override {
        if (ordered(f))
            reduce_ltr(sendbuf, recvbuf, root, f);
        else
            reduce_no_order(sendbuf, recvbuf, root, f);
    }

    void allreduce(channel_data sendbuf, channel_data recvbuf, raw_function f) override {
        if (ordered(f)) {  // reference PeerToPeer.cpp:88-90
            reduce(sendbuf, recvbuf, 0, f);
            bcast(recvbuf, 0);
        } else {
            allreduce_no_order(sendbuf, recvbuf, f);
        }
    }

    void scan(channel_data sendbuf, channel_data recvbuf, raw_function f) override {
        if (ordered(f))
            scan_ltr(sendbuf, recvbuf, f);
        else
            scan_no_order(sendbuf, recvbuf, f);
    }

    // ---- performance / cost model (reference PeerToPeer.cpp:295-406), in units of the channel's
    //      get_latency / get_price --------------------------------------------------------------------
    double get_operation_latency(Utils::OperationInfo info) override {
        const double P = num_peers;
        const double up = std::ceil(std::log2(P));
        const double down = std::floor(std::log2(P));
        // device buckets cross PCIe twice per message (D2H before the send, H2D after the receive)
        const double stage_ms = info.on_device ? 2 * 0.02 : 0.;
        const double stage_gb_s = 25.;
        auto hop = [&](std::size_t bytes) {
            double t = get_latency(1, 1, bytes);
            if (info.on_device) t += stage_ms + 2 * static_cast<double>(bytes) / 1e9 / stage_gb_s * 1e3;
            return t;
        };
        auto tree_growing = [&](std::size_t bytes) {  // gather/scatter: buffers grow per round
            double t = 0.;
            for (int i = 1; i <= static_cast<int>(down); ++i) t += hop(i * bytes);
            return t + hop(static_cast<std::size_t>(P - std::pow(2., down)) * bytes);
        };
        std::size_t bytes = info.data_size;
        switch (info.op) {
            case Utils::send: return hop(bytes);
            case Utils::bcast: return up * hop(bytes);
            case Utils::reduce:
                if (!info.left_to_right) return up * hop(bytes);
                return tree_growing(bytes);
            case Utils::gather:
            case Utils::scatter: return tree_growing(bytes);
            case Utils::barrier: bytes = 1; [[fallthrough]];
            case Utils::allreduce:
                if (info.left_to_right) return tree_growing(bytes) + up * hop(bytes);
                // the reference adds the two fold messages unconditionally (floor(log2 P) != P)
                return 2 * down * hop(bytes) + 2 * hop(bytes);
            case Utils::scan:
                return info.left_to_right ? (P - 1) * hop(bytes) : 2 * down * hop(bytes);
        }
        throw std::runtime_error("Operation not implemented");
    }

    double get_operation_price(Utils::OperationInfo info) override {
        const double P = num_peers;
        const double down = std::floor(std::log2(P));
        auto msg = [&](std::size_t bytes) { return get_price(1, 1, bytes); };
        auto tree_cost = [&](std::size_t bytes) {
            double c = 0.;
            for (int i = 1; i <= static_cast<int>(std::ceil(std::log2(P))); ++i) c += std::pow(2., down - i) * msg(i * bytes);
            return c;
        };
        std::size_t bytes = info.data_size;
        switch (info.op) {
            case Utils::send: return msg(bytes);
            case Utils::bcast: return (P - 1) * msg(bytes);
            case Utils::reduce:
                if (!info.left_to_right) return (P - 1) * msg(bytes);
                return tree_cost(bytes);
            case Utils::gather:
            case Utils::scatter: return tree_cost(bytes);
            case Utils::barrier: bytes = 1; [[fallthrough]];
            case Utils::allreduce:
                if (info.left_to_right) return tree_cost(bytes) + (P - 1) * msg(bytes);
                return 2 * (P - 1) * msg(bytes);
            case Utils::scan: return info.left_to_right ? (P - 1) * msg(bytes) : 2 * P * msg(bytes);
        }
        throw std::runtime_error("Operation not implemented");
    }

protected:
    //! LTR reduce: gather to root, then ((x0 f x1) f x2) ... (reference PeerToPeer.cpp:44-57).
    void reduce_ltr(channel_data sendbuf, channel_data recvbuf, Utils::peer_num root, const raw_function& f) {
        const std::size_t S = sendbuf.len;
        if (peer_id != root) {
            gather(sendbuf, {nullptr, 0, sendbuf.on_device}, root);
            return;
        }
        Dev::Scratch all(S * num_peers, sendbuf.on_device);
        gather(sendbuf, {all.get(), S * num_peers, sendbuf.on_device}, root);
        Dev::copy_bytes(recvbuf.buf, recvbuf.on_device, all.get(), sendbuf.on_device, S);
        for (unsigned p = 1; p < num_peers; ++p) f.f(recvbuf.buf, all.get() + p * S);
    }

    //! Binomial-tree reduce toward root on virtual ids, f(own, received) (reference PeerToPeer.cpp:59-84).
    void reduce_no_order(channel_data sendbuf, channel_data recvbuf, Utils::peer_num root, const raw_function& f) {
        const unsigned v = virt(peer_id, root);
        Dev::Scratch incoming(sendbuf.len, sendbuf.on_device);
        for (int i = 0; i < ceil_log2(num_peers); ++i) {
            const unsigned step = 1u << i;
            if (v % (2 * step) == 0 && v + step < num_peers) {
                const channel_data in{incoming.get(), sendbuf.len, sendbuf.on_device};
                recv_then_combine(in, real(v + step, root), sendbuf, in, f);
            } else if (v % step == 0 && v % (2 * step) != 0) {
                send(sendbuf, real(v - step, root));
            }
        }
        if (peer_id == root) Dev::copy_bytes(recvbuf.buf, recvbuf.on_device, sendbuf.buf, sendbuf.on_device, sendbuf.len);
    }

    //! Recursive doubling with a fold for the peers above the largest power of two
    //! (reference PeerToPeer.cpp:96-130). sendbuf ends holding the result (the reference's side effect).
    void allreduce_no_order(channel_data sendbuf, channel_data recvbuf, const raw_function& f) {
        const int rounds = floor_log2(num_peers);
        const unsigned pow2 = 1u << rounds;
        const bool folded_in = peer_id < pow2 && peer_id + pow2 < num_peers;  // receives a folded bucket
        const bool folded_out = peer_id >= pow2;                               // hands its bucket down
        channel_data tmp = recvbuf;  // the reference receives into recvbuf
        if (folded_in) {
            recv_then_combine(tmp, peer_id + pow2, sendbuf, tmp, f);
        } else if (folded_out) {
            send(sendbuf, peer_id - pow2);
        }
        if (peer_id < pow2) {
            for (int i = 0; i < rounds; ++i) {
                const unsigned partner = peer_id ^ (1u << i);
                if (partner < peer_id) {
                    send(sendbuf, partner);
                    recv_then_combine(tmp, partner, sendbuf, tmp, f);
                } else {
                    recv(tmp, partner);
                    send_then_combine(sendbuf, partner, sendbuf, tmp, f);
                }
            }
        }
        if (folded_in)
            send(sendbuf, peer_id + pow2);
        else if (folded_out)
            recv(sendbuf, peer_id - pow2);
        Dev::copy_bytes(recvbuf.buf, recvbuf.on_device, sendbuf.buf, sendbuf.on_device, sendbuf.len);
    }

    //! Linear chain scan, f(prefix, own) (reference PeerToPeer.cpp:141-152).
    void scan_ltr(channel_data sendbuf, channel_data recvbuf, const raw_function& f) {
        if (peer_id == 0) {
            if (num_peers > 1) send(sendbuf, 1);
            Dev::copy_bytes(recvbuf.buf, recvbuf.on_device, sendbuf.buf, sendbuf.on_device, sendbuf.len);
            return;
        }
        recv_then_combine(recvbuf, peer_id - 1, recvbuf, sendbuf, f);
        if (peer_id + 1 < num_peers) send(recvbuf, peer_id + 1);
    }

    //! Binomial up-sweep / down-sweep scan, f(own, received) (reference PeerToPeer.cpp:154-184).
    void scan_no_order(channel_data sendbuf, channel_data recvbuf, const raw_function& f) {
        const int rounds = floor_log2(num_peers);
        const unsigned id = peer_id;
        auto ones = [](int k) { return (1u << k) - 1u; };
        for (int i = 0; i < rounds; ++i) {
            if ((id & ones(i + 1)) == ones(i + 1)) {
                recv_then_combine(recvbuf, id - (1u << i), sendbuf, recvbuf, f);
            } else if ((id & ones(i)) == ones(i) && id + (1u << i) < num_peers) {
                send(sendbuf, id + (1u << i));
                break;
            }
        }
        for (int i = rounds; i > 0; --i) {
            const unsigned half = 1u << (i - 1);
            if ((id & ones(i)) == ones(i)) {
                if (id + half < num_peers) send(sendbuf, id + half);
            } else if ((id & ones(i - 1)) == ones(i - 1) && id > half) {
                recv_then_combine(recvbuf, id - half, sendbuf, recvbuf, f);
            }
        }
        Dev::copy_bytes(recvbuf.buf, recvbuf.on_device, sendbuf.buf, sendbuf.on_device, sendbuf.len);
    }

    static bool ordered(const raw_function& f) { return !(f.commutative && f.associative); }

    //! recv(`target`) from `src`, then left = f(left, right), where target is left or right. On a stream
    //! transport with a ranged combine and host buckets, the receive is cut into chunks and chunk k is
    //! combined on the worker thread while chunk k+1 arrives: the same element-wise combines on the same
    //! operands, so the same bits, in max(transfer, combine) instead of their sum.
    void recv_then_combine(channel_data target, Utils::peer_num src, channel_data left, channel_data right,
                           const raw_function& f) {
        const std::size_t chunk = overlap_chunk_for(f, left, right);
        if (!chunk) {
            recv(target, src);
            f.f(left.buf, right.buf);
            return;
        }
        overlapped(target, chunk, [&](channel_data piece) { recv_object(piece, src); }, left, right, f);
    }

    //! send(`source`) to `dst`, then left = f(left, right), where source is left: chunk k is combined as
    //! soon as it has been handed to the transport (it is not read again), while chunk k+1 is being sent.
    void send_then_combine(channel_data source, Utils::peer_num dst, channel_data left, channel_data right,
                           const raw_function& f) {
        const std::size_t chunk = overlap_chunk_for(f, left, right);
        if (!chunk) {
            send(source, dst);
            f.f(left.buf, right.buf);
            return;
        }
        overlapped(source, chunk, [&](channel_data piece) { send_object(piece, dst); }, left, right, f);
    }

    static int ceil_log2(unsigned v) {
        int r = 0;
        while ((1u << r) < v) ++r;
        return r;
    }
    static int floor_log2(unsigned v) {
        int r = 0;
        while ((2u << r) <= v) ++r;
        return r;
    }

private:
    // transform_peer_id (reference PeerToPeer.cpp:287-293): the root becomes virtual peer 0
    unsigned virt(unsigned id, unsigned root) const { return (id + num_peers - root) % num_peers; }
    unsigned real(unsigned v, unsigned root) const { return (v + root) % num_peers; }

    // buckets held by virtual peer v in a binomial gather: itself plus its children's subtrees
    unsigned subtree_size(unsigned v) const {
        unsigned count = 1;
        for (int i = 0; i < ceil_log2(num_peers); ++i) {
            const unsigned step = 1u << i;
            if (v % (2 * step) != 0) break;
            if (v + step < num_peers) count += std::min(step, num_peers - (v + step));
        }
        return count;
    }

    std::size_t overlap_chunk_for(const raw_function& f, const channel_data& left, const channel_data& right) const {
        if (!f.part || f.granule == 0 || overlap_chunk_ == 0 || !stream_transport()) return 0;
        if (left.on_device || right.on_device || left.len != right.len) return 0;
        const std::size_t chunk = std::max(f.granule, overlap_chunk_ / f.granule * f.granule);
        return left.len >= 2 * chunk ? chunk : 0;
    }

    // Move `buf` piece by piece with `io`; after piece k, its combine runs on the worker.
    template <class Io>
    void overlapped(channel_data buf, std::size_t chunk, Io&& io, channel_data left, channel_data right,
                    const raw_function& f) {
        try {
            for (std::size_t off = 0; off < buf.len; off += chunk) {
                const std::size_t len = std::min(chunk, buf.len - off);
                io(channel_data{buf.buf + off, len, false});
                ++overlapped_pieces_;
                worker_.submit([part = f.part, l = left.buf, r = right.buf, off, len] { part(l, r, off, len); });
            }
            worker_.wait();
        } catch (...) {
            worker_.drain();  // no combine may outlive the buffers it writes
            throw;
        }
    }

    char* staging(std::size_t len) {
        if (staging_bytes_ < len) {
            release_staging();
            void* p = nullptr;
            Dev::check(fmi_host_pin_alloc(&p, len), "fmi_host_pin_alloc (channel staging)");
            staging_ = static_cast<char*>(p);
            staging_bytes_ = len;
        }
        return staging_;
    }
    void release_staging() {
        if (staging_) (void)fmi_host_pin_free(staging_);
        staging_ = nullptr;
        staging_bytes_ = 0;
    }

    char* staging_ = nullptr;
    std::size_t staging_bytes_ = 0;
    std::size_t overlap_chunk_ = 0;  // opt-in: measured mixed on the GPU box's host
    std::size_t overlapped_pieces_ = 0;
    CombineWorker worker_;
};

}  // namespace FMI::Comm

#endif
