// FMI::Comm::Rccl — a Channel for buckets resident in MI355X HBM, one peer per GPU, over RCCL / xGMI
// (SURVEY.md §8f rank 2). It plugs in through the reference's own extension point,
// Communicator::register_channel (reference include/Communicator.h:153), and competes in ChannelPolicy
// (reference src/utils/ChannelPolicy.cpp:9-29) through its latency/price model; for device buckets it
// beats any host-staged channel, so the policy routes them here.
//
// The collectives are the C-ABI's sharded schedules (fmi_comm_*): all-to-all of shards, one pass of the
// fused kernel in the reference's order, all-gather / gather / all-to-all back — so every result has the
// reference's bracketing, each peer with its own operand order (float max/min ties and NaNs included).
// Side effects reproduced from the reference: commutative allreduce and scan leave sendbuf = result
// (reference src/comm/PeerToPeer.cpp:129,183); commutative reduce leaves every peer's sendbuf as the
// reference does (:72): the partial it forwarded up the binomial tree, the root's = the result
// (fmi_comm_reduce_sendbuf); the ordered (LTR) collectives leave it intact.
//
// Host ingress (config C5), opt-in with set_host_ingress(): the channel then also
// carries host buckets — the recv buffers FMI's transports fill (reference src/comm/Direct.cpp:36-45).
// allreduce streams them through the GPU with fmi_comm_allreduce_host (H2D, sharded allreduce and D2H of
// successive chunks overlapped); every other collective stages the host bucket through HBM. The model
// charges the PCIe crossing, so ChannelPolicy keeps small host operations on the host channels.
#ifndef FMI_AMD_COMM_RCCL_H
#define FMI_AMD_COMM_RCCL_H

#include <array>
#include <cmath>
#include <memory>
#include <stdexcept>
#include <string>

#include "Channel.h"

namespace FMI::Comm {

class Rccl : public Channel {
public:
    //! Join a communicator: peer 0 creates the id, `bootstrap` (any host channel of the same peers)
    //! broadcasts it, every peer initialises its rank. transport: FMI_TRANSPORT_RCCL (one process per GPU),
    //! FMI_TRANSPORT_PROC (peers are processes of one node, e.g. several sharing one GPU) or
    //! FMI_TRANSPORT_LOCAL (peers are threads of one process sharing one GPU).
    //! timeout_s bounds every wait for the peers (the init rendezvous, barriers, each collective's
    //! completion); on expiry the call throws Utils::Timeout, as the reference's channels do
    //! (src/comm/Direct.cpp:28-30), and the channel is unusable. <= 0: the library default
    //! (FMI_COMM_TIMEOUT_S, else 300 s).
    static std::shared_ptr<Rccl> connect(Channel& bootstrap, Utils::peer_num peer, Utils::peer_num num_peers,
                                         int transport = FMI_TRANSPORT_RCCL, double link_gb_s = 300.,
                                         double timeout_s = 0.) {
        std::array<char, FMI_COMM_ID_BYTES> id{};
        if (peer == 0) Dev::check(fmi_comm_unique_id(transport, id.data(), id.size()), "fmi_comm_unique_id");
        bootstrap.bcast({id.data(), id.size()}, 0);
        fmi_comm_t comm = nullptr;
        Dev::check(fmi_comm_init_timeout(&comm, id.data(), static_cast<int>(num_peers), static_cast<int>(peer), timeout_s),
                   "fmi_comm_init");
        auto ch = std::shared_ptr<Rccl>(new Rccl(comm, link_gb_s));
        ch->set_peer_id(peer);
        ch->set_num_peers(num_peers);
        return ch;
    }

    ~Rccl() override { finalize(); }

    bool supports_host_buffers() const override { return host_ingress_; }
    bool supports_user_functions() const override { return false; }

    //! Accept host buckets too (staged through HBM; allreduce pipelined). pcie_gb_s prices the crossing.
    void set_host_ingress(bool on, double pcie_gb_s = 50.) {
        host_ingress_ = on;
        pcie_gb_s_ = pcie_gb_s;
    }

    void send(channel_data buf, Utils::peer_num dest) override {
        Staged b(this, buf, true);
        run(fmi_comm_send(comm_, b.ptr(), buf.len, static_cast<int>(dest), nullptr), "fmi_comm_send");
    }
    void recv(channel_data buf, Utils::peer_num src) override {
        Staged b(this, buf, false);
        run(fmi_comm_recv(comm_, b.ptr(), buf.len, static_cast<int>(src), nullptr), "fmi_comm_recv");
        b.store();
    }
    void bcast(channel_data buf, Utils::peer_num root) override {
        Staged b(this, buf, peer_id == root);
        run(fmi_comm_bcast(comm_, b.ptr(), buf.len, static_cast<int>(root), nullptr), "fmi_comm_bcast");
        if (peer_id != root) b.store();
    }
    void barrier() override { run(fmi_comm_barrier(comm_, nullptr), "fmi_comm_barrier"); }

    void gather(channel_data sendbuf, channel_data recvbuf, Utils::peer_num root) override {
        const bool is_root = peer_id == root;
        Staged s(this, sendbuf, true);
        Staged r(this, is_root ? recvbuf : channel_data{nullptr, 0, true}, false);
        run(fmi_comm_gather(comm_, s.ptr(), is_root ? r.ptr() : nullptr, sendbuf.len, static_cast<int>(root), nullptr),
            "fmi_comm_gather");
        if (is_root) r.store();
    }
    void scatter(channel_data sendbuf, channel_data recvbuf, Utils::peer_num root) override {
        const bool is_root = peer_id == root;
        Staged s(this, is_root ? sendbuf : channel_data{nullptr, 0, true}, true);
        Staged r(this, recvbuf, false);
        run(fmi_comm_scatter(comm_, is_root ? s.ptr() : nullptr, r.ptr(), recvbuf.len, static_cast<int>(root), nullptr),
            "fmi_comm_scatter");
        r.store();
    }

    void reduce(channel_data sendbuf, channel_data recvbuf, Utils::peer_num root, raw_function f) override {
        const device_op& d = device_of(f, sendbuf);
        const int alg = ordered(f) ? FMI_ALG_REDUCE_LTR : FMI_ALG_REDUCE;
        const bool is_root = peer_id == root;
        Staged s(this, sendbuf, true);
        Staged r(this, is_root ? recvbuf : channel_data{nullptr, 0, true}, false);
        if (ordered(f)) {
            run(fmi_comm_reduce(comm_, d.op, d.dtype, alg, s.ptr(), is_root ? r.ptr() : nullptr, d.count,
                                static_cast<int>(root), nullptr),
                "fmi_comm_reduce");
        } else {  // every sendbuf ends as the reference leaves it
            run(fmi_comm_reduce_sendbuf(comm_, d.op, d.dtype, alg, s.ptr(), is_root ? r.ptr() : nullptr, d.count,
                                        static_cast<int>(root), nullptr),
                "fmi_comm_reduce_sendbuf");
            s.store();
        }
        if (is_root) r.store();
    }

    void allreduce(channel_data sendbuf, channel_data recvbuf, raw_function f) override {
        const device_op& d = device_of(f, sendbuf);
        carries(recvbuf);
        const int alg = ordered(f) ? FMI_ALG_REDUCE_LTR : FMI_ALG_ALLREDUCE;
        if (!sendbuf.on_device || !recvbuf.on_device) {  // host ingress: pipelined through the GPU
            Dev::check(fmi_comm_allreduce_host(comm_, d.op, d.dtype, alg, path_, sendbuf.buf, recvbuf.buf, d.count, 0),
                       "fmi_comm_allreduce_host");
        } else {
            run(fmi_comm_allreduce(comm_, d.op, d.dtype, alg, path_, sendbuf.buf, recvbuf.buf, d.count, nullptr),
                "fmi_comm_allreduce");
        }
        if (!ordered(f)) mirror(sendbuf, recvbuf);
    }

    void scan(channel_data sendbuf, channel_data recvbuf, raw_function f) override {
        const device_op& d = device_of(f, sendbuf);
        const int alg = ordered(f) ? FMI_ALG_SCAN_LTR : FMI_ALG_SCAN;
        Staged s(this, sendbuf, true);
        Staged r(this, recvbuf, false);
        run(fmi_comm_scan(comm_, d.op, d.dtype, alg, s.ptr(), r.ptr(), d.count, nullptr), "fmi_comm_scan");
        r.store();
        if (!ordered(f)) mirror(sendbuf, recvbuf);
    }

    //! FMI_PATH_TREE (default, reference order), FMI_PATH_RCCL (reduce-scatter, RCCL's order) or
    //! FMI_PATH_DIRECT (fused kernel over the peers' windows, reference order; buckets from window()).
    void set_path(int path) { path_ = path; }

    //! A device bucket in a symmetric window (collective: every peer, same n), readable by every peer
    //! over xGMI — the bucket kind FMI_PATH_DIRECT needs. It lives until the channel finalizes.
    template <class A>
    Dev::Bucket<A> window(std::size_t n) {
        void* p = nullptr;
        Dev::check(fmi_comm_window_alloc(comm_, n * sizeof(A), &p), "fmi_comm_window_alloc");
        return Dev::Bucket<A>::borrow(static_cast<A*>(p), n);
    }

    void finalize() override {
        if (comm_) (void)fmi_comm_destroy(comm_);
        comm_ = nullptr;
    }

    // xGMI model in ms: latency + bytes over the per-GPU link bandwidth; sharded collectives move
    // 2 (N-1)/N of the bucket per GPU (reduce-scatter + all-gather), point-to-point moves it once.
    double get_latency(Utils::peer_num producer, Utils::peer_num consumer, std::size_t size_in_bytes) override {
        return 0.01 + producer * consumer * (static_cast<double>(size_in_bytes) / 1e9) / link_gb_s_ * 1e3;
    }
    double get_price(Utils::peer_num, Utils::peer_num, std::size_t) override { return 0.; }
    double get_operation_latency(Utils::OperationInfo info) override {
        const double P = num_peers;
        const double frac = P > 1 ? (P - 1) / P : 0.;
        const std::size_t bytes = info.data_size;
        // host buckets cross PCIe once each way (overlapped with the exchange for allreduce)
        const double pcie = info.on_device || info.op == Utils::barrier
                                ? 0.
                                : (info.op == Utils::allreduce ? 1. : 2.) * static_cast<double>(bytes) / 1e9 /
                                      pcie_gb_s_ * 1e3;
        switch (info.op) {
            case Utils::send: return pcie + get_latency(1, 1, bytes);
            case Utils::barrier: return 0.02;
            case Utils::bcast:
            case Utils::gather:
            case Utils::scatter: return pcie + 0.01 + frac * get_latency(1, 1, bytes);
            case Utils::reduce:
            case Utils::allreduce:
            case Utils::scan: return pcie + 0.02 + 2 * frac * get_latency(1, 1, bytes);
        }
        throw std::runtime_error("Operation not implemented");
    }
    double get_operation_price(Utils::OperationInfo) override { return 0.; }

private:
    Rccl(fmi_comm_t comm, double link_gb_s) : comm_(comm), link_gb_s_(link_gb_s) {}

    static bool ordered(const raw_function& f) { return !(f.commutative && f.associative); }

    void carries(const channel_data& b) const {
        if (!b.on_device && b.len && !host_ingress_)
            throw std::runtime_error("Rccl channel carries device buckets only (see set_host_ingress)");
    }
    const device_op& device_of(const raw_function& f, const channel_data& b) const {
        carries(b);
        if (!f.device.valid())
            throw std::runtime_error("Rccl channel needs a built-in reduction op (Function<T>(Utils::Op::...))");
        return f.device;
    }
    // FMI collectives are blocking: wait for completion within the communicator's timeout
    // (FMI_ERR_TIMEOUT -> Utils::Timeout, Dev::check)
    void run(int status, const char* what) const {
        Dev::check(status, what);
        Dev::check(fmi_comm_sync(comm_, nullptr), "fmi_comm_sync");
    }
    static void mirror(const channel_data& sendbuf, const channel_data& recvbuf) {
        if (sendbuf.buf != recvbuf.buf)
            Dev::copy_bytes(sendbuf.buf, sendbuf.on_device, recvbuf.buf, recvbuf.on_device, sendbuf.len);
    }

    // A device view of a channel buffer: the buffer itself when it lives in HBM, else an HBM copy of the
    // host bucket (loaded on construction if `load`, written back by store()).
    class Staged {
    public:
        Staged(const Rccl* ch, const channel_data& b, bool load) : user_(b), host_(!b.on_device && b.buf) {
            ch->carries(b);
            if (!host_) return;
            scratch_ = Dev::Scratch(b.len, true);
            if (load) Dev::copy_bytes(scratch_.get(), true, b.buf, false, b.len);
        }
        char* ptr() const { return host_ ? scratch_.get() : user_.buf; }
        void store() const {
            if (host_) Dev::copy_bytes(user_.buf, false, scratch_.get(), true, user_.len);
        }

    private:
        channel_data user_;
        bool host_;
        Dev::Scratch scratch_;
    };

    fmi_comm_t comm_ = nullptr;
    double link_gb_s_;
    int path_ = FMI_PATH_TREE;
    bool host_ingress_ = false;
    double pcie_gb_s_ = 50.;
};

}  // namespace FMI::Comm

#endif
