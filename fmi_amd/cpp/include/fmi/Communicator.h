// FMI::Communicator — the user-facing SPMD communicator, source-compatible with the reference
// (include/Communicator.h:10-190, src/Communicator.cpp:5-44): same constructor, same templated
// send / recv / bcast / barrier / gather / scatter / reduce / allreduce / scan, same plugin points
// (register_channel, set_channel_policy, hint), same exceptions.
//
// What changes is the local bucket reduction, the hot path of reduce / allreduce / scan:
//   * Data<Dev::Bucket<A>> (bucket in MI355X HBM) + a built-in Function (Function<T>(Utils::Op::sum)):
//     every combine the channel algorithm performs is the gfx950 kernel fmi_dev_reduce_pair, on the
//     buffers where they live — no host round trip, no copies.
//   * Data<std::vector<A>> + a built-in Function, after use_device(d): each combine whose buckets are large
//     enough to pay (ChannelPolicy::host_combine_on_device, the measured crossover) streams the two host buckets
//     through the GPU (fmi_host_reduce_pair: zero-copy over PCIe if page-locked, else chunked H2D / kernel /
//     D2H); smaller ones run in place on the host. use_device(d, true) sends every combine to the GPU.
//   * Data<std::vector<A>> + a built-in Function without use_device: the combine runs in place on the
//     host buckets (no bucket copies).
//   * any user lambda: the reference's adapter, unchanged (include/Communicator.h:180-189 semantics).
// The evaluation order is the reference's in every case (it is fixed by the channel algorithm).
#ifndef FMI_AMD_COMMUNICATOR_H
#define FMI_AMD_COMMUNICATOR_H

#include <atomic>
#include <cstring>
#include <iostream>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "comm/Channel.h"
#include "dev/Device.h"
#include "utils/ChannelPolicy.h"
#include "utils/Configuration.h"

namespace FMI {

class Communicator {
public:
    /*!
     * @param peer_id ID of the peer in [0, num_peers)
     * @param num_peers number of peers in the communicator
     * @param config_path FMI JSON configuration (reference schema); "" = no configured backends, register
     *        channels with register_channel()
     * @param comm_name unique name of the communicator
     * @param faas_memory MiB of memory of the function, for the price model
     */
    Communicator(Utils::peer_num peer_id, Utils::peer_num num_peers, std::string config_path, std::string comm_name,
                 unsigned int faas_memory = 128)
        : peer_id(peer_id), num_peers(num_peers), comm_name(std::move(comm_name)) {
        double gib_second_price = 0.0000166667;  // reference config/fmi.json model.FaaS.gib_second_price
        if (!config_path.empty()) {
            Utils::Configuration config(config_path);
            for (const auto& [name, params] : config.get_active_channels()) {
                // The reference's bundled transports (Direct over TCPunch, Redis, S3) carry host bytes
                // between FaaS instances and are outside this engine; their role is taken by channels
                // registered through register_channel (LocalSocket, Loopback, Rccl).
                std::cerr << "fmi_amd: configured backend '" << name
                          << "' is not bundled; register a channel with register_channel()\n";
            }
            gib_second_price = config.get_faas_price();
        }
        const double faas_price = static_cast<double>(faas_memory) / 1024. * gib_second_price;
        set_channel_policy(std::make_shared<Utils::ChannelPolicy>(channels, num_peers, faas_price, channel_hint));
    }

    //! Finalizes all channels (reference src/Communicator.cpp:31-35).
    ~Communicator() {
        for (auto const& [name, channel] : channels) channel->finalize();
    }

    Communicator(const Communicator&) = delete;
    Communicator& operator=(const Communicator&) = delete;

    template <typename T>
    void send(Comm::Data<T>& buf, Utils::peer_num dest) {
        channel_for({Utils::send, buf.size_in_bytes()}, on_device(buf))->send(view(buf), dest);
    }

    template <typename T>
    void recv(Comm::Data<T>& buf, Utils::peer_num src) {
        channel_for({Utils::send, buf.size_in_bytes()}, on_device(buf))->recv(view(buf), src);
    }

    template <typename T>
    void bcast(Comm::Data<T>& buf, Utils::peer_num root) {
        channel_for({Utils::bcast, buf.size_in_bytes()}, on_device(buf))->bcast(view(buf), root);
    }

    void barrier() { channel_for({Utils::barrier, 0}, false)->barrier(); }

    template <typename T>
    void gather(Comm::Data<T>& sendbuf, Comm::Data<T>& recvbuf, Utils::peer_num root) {
        channel_for({Utils::gather, sendbuf.size_in_bytes()}, on_device(sendbuf))
            ->gather(view(sendbuf), view(recvbuf), root);
    }

    template <typename T>
    void scatter(Comm::Data<T>& sendbuf, Comm::Data<T>& recvbuf, Utils::peer_num root) {
        channel_for({Utils::scatter, recvbuf.size_in_bytes()}, on_device(recvbuf))
            ->scatter(view(sendbuf), view(recvbuf), root);
    }

    //! Reduction to `root`; for commutative + associative f the sendbuf is overwritten with partials,
    //! as in the reference (src/comm/PeerToPeer.cpp:72).
    template <typename T>
    void reduce(Comm::Data<T>& sendbuf, Comm::Data<T>& recvbuf, Utils::peer_num root, Utils::Function<T> f) {
        if (peer_id == root && sendbuf.size_in_bytes() != recvbuf.size_in_bytes())
            throw std::runtime_error("Dimensions of send and receive data must match");
        const bool ltr = !(f.commutative && f.associative);
        raw_function raw = convert_to_raw_function(f, sendbuf.size_in_bytes());
        auto ch = channel_for({Utils::reduce, sendbuf.size_in_bytes(), ltr, false, !raw.device.valid()}, on_device(sendbuf));
        ch->reduce(view(sendbuf), view(recvbuf), root, std::move(raw));
    }

    template <typename T>
    void allreduce(Comm::Data<T>& sendbuf, Comm::Data<T>& recvbuf, Utils::Function<T> f) {
        if (sendbuf.size_in_bytes() != recvbuf.size_in_bytes())
            throw std::runtime_error("Dimensions of send and receive data must match");
        const bool ltr = !(f.commutative && f.associative);
        raw_function raw = convert_to_raw_function(f, sendbuf.size_in_bytes());
        auto ch = channel_for({Utils::allreduce, sendbuf.size_in_bytes(), ltr, false, !raw.device.valid()},
                              on_device(sendbuf));
        ch->allreduce(view(sendbuf), view(recvbuf), std::move(raw));
    }

    //! Inclusive prefix across peers: peer k receives x0 f ... f xk.
    template <typename T>
    void scan(Comm::Data<T>& sendbuf, Comm::Data<T>& recvbuf, Utils::Function<T> f) {
        if (sendbuf.size_in_bytes() != recvbuf.size_in_bytes())
            throw std::runtime_error("Dimensions of send and receive data must match");
        // the reference does not pass left_to_right here (include/Communicator.h:140)
        raw_function raw = convert_to_raw_function(f, sendbuf.size_in_bytes());
        auto ch = channel_for({Utils::scan, sendbuf.size_in_bytes(), false, false, !raw.device.valid()}, on_device(sendbuf));
        ch->scan(view(sendbuf), view(recvbuf), std::move(raw));
    }

    //! Add a channel under `name` (reference src/Communicator.cpp:24-29).
    void register_channel(std::string name, std::shared_ptr<Comm::Channel> c) {
        c->set_peer_id(peer_id);
        c->set_num_peers(num_peers);
        c->set_comm_name(comm_name);
        channels[std::move(name)] = std::move(c);
    }

    void set_channel_policy(std::shared_ptr<Utils::ChannelPolicy> p) { policy = std::move(p); }
    //! The policy the communicator dispatches through (extension: e.g. to move the host-combine crossover).
    std::shared_ptr<Utils::ChannelPolicy> channel_policy() const { return policy; }

    void hint(Utils::Hint h) {
        channel_hint = h;
        policy->set_hint(h);
    }

    //! MI355X extension: run the combines of built-in Functions on host buckets on GPU `device` where the
    //! policy's crossover says the GPU pays (ChannelPolicy::host_combine_on_device); `always`: every one.
    void use_device(int device, bool always = false) {
        Dev::init(device);
        offload_host_ = true;
        offload_always_ = always;
    }

    //! Where the last built-in combine of host buckets ran (tests, diagnostics): true = the GPU.
    bool last_host_combine_on_device() const { return last_on_device_->load(); }

    Utils::peer_num get_peer_id() const { return peer_id; }
    Utils::peer_num get_num_peers() const { return num_peers; }

private:
    template <typename T>
    static bool on_device(Comm::Data<T>& d) {
        return d.on_device();
    }

    template <typename T>
    static channel_data view(Comm::Data<T>& d) {
        return channel_data{d.data(), d.size_in_bytes(), d.on_device()};
    }

    std::shared_ptr<Comm::Channel> channel_for(Utils::OperationInfo info, bool device) {
        const std::string name = device ? policy->get_device_channel(info) : policy->get_channel(info);
        auto it = channels.find(name);
        if (it == channels.end()) throw std::runtime_error("channel '" + name + "' is not registered");
        return it->second;
    }

    //! Scalars: *a = f(*a, *b) (reference include/Communicator.h:170-177).
    template <typename T>
    raw_function convert_to_raw_function(Utils::Function<T> f, std::size_t) {
        return raw_function{[f](char* a, char* b) {
                                T* dst = reinterpret_cast<T*>(a);
                                *dst = f(*reinterpret_cast<T*>(a), *reinterpret_cast<T*>(b));
                            },
                            f.associative, f.commutative};
    }

    //! Host buckets (include/Communicator.h:180-189).
    template <typename A>
    raw_function convert_to_raw_function(Utils::Function<std::vector<A>> f, std::size_t size_in_bytes) {
        const Utils::Op op = f.builtin();
        if constexpr (Dev::device_type<A>) {
            if (op != Utils::Op::none) {
                const std::size_t count = size_in_bytes / sizeof(A);
                const device_op dop{static_cast<int>(op), Dev::dtype_of<A>(), count};
                if (offload_host_) {
                    // per combine: the GPU where it pays, else the host loop (the same op, so the same bits)
                    auto part = [dop, op, policy = policy, always = offload_always_, last = last_on_device_](
                                    char* a, char* b, std::size_t off, std::size_t len) {
                        // below the policy's smallest GPU size the answer is the host whatever the pinning: no
                        // probe; above it a query that sets no error text (a pageable bucket is no error)
                        const bool device = always || (len >= policy->host_combine_min_bytes() &&
                                                       policy->host_combine_on_device(
                                                           len, fmi_host_page_locked(a + off, len) == 1 &&
                                                                    fmi_host_page_locked(b + off, len) == 1));
                        if (device) {
                            last->store(true);
                            Dev::check(fmi_host_reduce_pair(dop.op, dop.dtype, a + off, b + off, len / sizeof(A)),
                                       "fmi_host_reduce_pair");
                            return;
                        }
                        last->store(false);
                        A* x = reinterpret_cast<A*>(a + off);
                        const A* y = reinterpret_cast<const A*>(b + off);
                        for (std::size_t i = 0, m = len / sizeof(A); i < m; ++i)
                            x[i] = Utils::detail::apply_op<A>(op, x[i], y[i]);
                    };
                    return raw_function{[part, size_in_bytes](char* a, char* b) { part(a, b, 0, size_in_bytes); },
                                        f.associative, f.commutative, dop, part, sizeof(A)};
                }
                auto part = [op](char* a, char* b, std::size_t off, std::size_t len) {
                    A* x = reinterpret_cast<A*>(a + off);
                    const A* y = reinterpret_cast<const A*>(b + off);
                    for (std::size_t i = 0, m = len / sizeof(A); i < m; ++i) x[i] = Utils::detail::apply_op<A>(op, x[i], y[i]);
                };
                return raw_function{[part, size_in_bytes](char* a, char* b) { part(a, b, 0, size_in_bytes); },
                                    f.associative, f.commutative, dop, part, sizeof(A)};
            }
        }
        // The reference adapter: copy both buckets, call the user function by value, copy back.
        return raw_function{[f, size_in_bytes](char* a, char* b) {
                                std::vector<A> va(reinterpret_cast<A*>(a), reinterpret_cast<A*>(a + size_in_bytes));
                                std::vector<A> vb(reinterpret_cast<A*>(b), reinterpret_cast<A*>(b + size_in_bytes));
                                std::vector<A> res = f(va, vb);
                                if (res.size() * sizeof(A) != size_in_bytes)
                                    throw std::runtime_error("reduction function changed the bucket size");
                                std::memcpy(a, res.data(), size_in_bytes);
                            },
                            f.associative, f.commutative};
    }

    //! Device buckets: every combine is the gfx950 kernel on HBM-resident buffers.
    template <typename A>
    raw_function convert_to_raw_function(Utils::Function<Dev::Bucket<A>> f, std::size_t size_in_bytes) {
        if (f.builtin() == Utils::Op::none)
            throw std::runtime_error("device buckets need a built-in reduction op (Function<T>(Utils::Op::...))");
        const device_op dop{static_cast<int>(f.builtin()), Dev::dtype_of<A>(), size_in_bytes / sizeof(A)};
        return raw_function{[dop](char* a, char* b) {
                                Dev::check(fmi_dev_reduce_pair(dop.op, dop.dtype, a, b, dop.count, nullptr),
                                           "fmi_dev_reduce_pair");
                                Dev::check(fmi_stream_sync(nullptr), "fmi_stream_sync");
                            },
                            f.associative, f.commutative, dop};
    }

    std::shared_ptr<Utils::ChannelPolicy> policy;
    std::map<std::string, std::shared_ptr<Comm::Channel>> channels;
    Utils::peer_num peer_id;
    Utils::peer_num num_peers;
    std::string comm_name;
    Utils::Hint channel_hint = Utils::Hint::cheap;
    bool offload_host_ = false;
    bool offload_always_ = false;
    std::shared_ptr<std::atomic<bool>> last_on_device_ = std::make_shared<std::atomic<bool>>(false);
};

}  // namespace FMI

#endif
