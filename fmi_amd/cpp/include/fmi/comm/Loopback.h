// FMI::Comm::Loopback — in-process PeerToPeer transport: P peers (threads) share one Mailbox of
// per-(src, dst) FIFO queues. The reference has no such fake (its tests need a live TCPunch server,
// SURVEY.md §4); it stands in for the Direct channel's per-pair TCP streams (reference
// src/comm/Direct.cpp:25-45) with the same semantics: ordered, message-boundary-preserving, blocking
// receive with a timeout that raises Utils::Timeout.
#ifndef FMI_AMD_COMM_LOOPBACK_H
#define FMI_AMD_COMM_LOOPBACK_H

#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "PeerToPeer.h"

namespace FMI::Comm {

class Mailbox {
public:
    void put(Utils::peer_num src, Utils::peer_num dst, const char* data, std::size_t len) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            boxes_[{src, dst}].emplace_back(data, data + len);
        }
        cv_.notify_all();
    }

    void take(Utils::peer_num src, Utils::peer_num dst, char* data, std::size_t len, std::chrono::milliseconds timeout) {
        std::unique_lock<std::mutex> lk(mu_);
        auto& q = boxes_[{src, dst}];
        if (!cv_.wait_for(lk, timeout, [&] { return !q.empty(); })) throw Utils::Timeout();
        std::vector<char> msg = std::move(q.front());
        q.pop_front();
        if (msg.size() != len)
            throw std::runtime_error("Loopback: message of " + std::to_string(msg.size()) + " bytes, expected " +
                                     std::to_string(len));
        if (len) std::memcpy(data, msg.data(), len);
    }

private:
    std::mutex mu_;
    std::condition_variable cv_;
    std::map<std::pair<Utils::peer_num, Utils::peer_num>, std::deque<std::vector<char>>> boxes_;
};

class Loopback : public PeerToPeer {
public:
    explicit Loopback(std::shared_ptr<Mailbox> mailbox, std::chrono::milliseconds timeout = std::chrono::seconds(60),
                      double bandwidth_mb_s = 20000., double overhead_ms = 0.001)
        : mailbox_(std::move(mailbox)), timeout_(timeout), bandwidth_(bandwidth_mb_s), overhead_(overhead_ms) {}

    void send_object(channel_data buf, Utils::peer_num peer) override { mailbox_->put(peer_id, peer, buf.buf, buf.len); }
    void recv_object(channel_data buf, Utils::peer_num peer) override {
        mailbox_->take(peer, peer_id, buf.buf, buf.len, timeout_);
    }

    // memcpy-speed model in ms (same shape as Direct's: overhead + size / bandwidth); every bundled channel
    // models in ms so ChannelPolicy compares like with like
    double get_latency(Utils::peer_num producer, Utils::peer_num consumer, std::size_t size_in_bytes) override {
        return overhead_ + producer * consumer * (static_cast<double>(size_in_bytes) / 1e6) / bandwidth_ * 1e3;
    }
    double get_price(Utils::peer_num, Utils::peer_num, std::size_t) override { return 0.; }

private:
    std::shared_ptr<Mailbox> mailbox_;
    std::chrono::milliseconds timeout_;
    double bandwidth_;
    double overhead_;
};

}  // namespace FMI::Comm

#endif
