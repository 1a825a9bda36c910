// FMI::Comm::LocalSocket — PeerToPeer transport over AF_UNIX stream socketpairs for peers that are
// fork()ed processes on one host (the shape of the reference's own tests, tests/communicator.cpp:40-46,
// without the TCPunch rendezvous server they need). Same semantics as Direct (reference
// src/comm/Direct.cpp:25-71): blocking ordered byte streams per peer pair, send/receive timeouts raising
// Utils::Timeout — but partial sends are completed instead of dropped (reference quirk: Direct.cpp:27).
#ifndef FMI_AMD_COMM_LOCALSOCKET_H
#define FMI_AMD_COMM_LOCALSOCKET_H

#include <sys/socket.h>
#include <sys/time.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "PeerToPeer.h"

namespace FMI::Comm {

// All pairwise connections of P peers, created before the peers fork.
class SocketMesh {
public:
    explicit SocketMesh(Utils::peer_num P) : P_(P), fd_(static_cast<std::size_t>(P) * P, -1) {
        for (Utils::peer_num a = 0; a < P; ++a)
            for (Utils::peer_num b = a + 1; b < P; ++b) {
                int sv[2];
                if (socketpair(AF_UNIX, SOCK_STREAM, 0, sv) != 0)
                    throw std::runtime_error(std::string("socketpair: ") + std::strerror(errno));
                fd_[a * P + b] = sv[0];  // a's end towards b
                fd_[b * P + a] = sv[1];  // b's end towards a
            }
    }

    // The fds peer `me` uses (index = other peer, -1 for itself); closes every other end in this process.
    std::vector<int> claim(Utils::peer_num me) {
        std::vector<int> mine(P_, -1);
        for (Utils::peer_num a = 0; a < P_; ++a)
            for (Utils::peer_num b = 0; b < P_; ++b) {
                int& f = fd_[a * P_ + b];
                if (f < 0) continue;
                if (a == me)
                    mine[b] = f;
                else
                    ::close(f);
                f = -1;
            }
        return mine;
    }

private:
    Utils::peer_num P_;
    std::vector<int> fd_;
};

class LocalSocket : public PeerToPeer {
public:
    LocalSocket(std::vector<int> fds, int timeout_ms = 60000, double bandwidth_mb_s = 8000., double overhead_ms = 0.01)
        : fds_(std::move(fds)), bandwidth_(bandwidth_mb_s), overhead_(overhead_ms) {
        timeval tv{timeout_ms / 1000, (timeout_ms % 1000) * 1000};
        for (int f : fds_) {
            if (f < 0) continue;
            setsockopt(f, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
            setsockopt(f, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
        }
    }

    void send_object(channel_data buf, Utils::peer_num peer) override {
        const int f = fd(peer);
        std::size_t done = 0;
        while (done < buf.len) {
            const ssize_t k = ::send(f, buf.buf + done, buf.len - done, MSG_NOSIGNAL);
            if (k > 0) {
                done += static_cast<std::size_t>(k);
            } else if (k < 0 && errno == EINTR) {
                continue;
            } else if (k < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
                throw Utils::Timeout();
            } else {
                throw std::runtime_error(std::string("LocalSocket send: ") + std::strerror(errno));
            }
        }
    }

    void recv_object(channel_data buf, Utils::peer_num peer) override {
        const int f = fd(peer);
        std::size_t done = 0;
        while (done < buf.len) {
            const ssize_t k = ::recv(f, buf.buf + done, buf.len - done, MSG_WAITALL);
            if (k > 0) {
                done += static_cast<std::size_t>(k);
            } else if (k == 0) {
                throw std::runtime_error("LocalSocket recv: peer " + std::to_string(peer) + " closed the connection");
            } else if (errno == EINTR) {
                continue;
            } else if (errno == EAGAIN || errno == EWOULDBLOCK) {
                throw Utils::Timeout();
            } else {
                throw std::runtime_error(std::string("LocalSocket recv: ") + std::strerror(errno));
            }
        }
    }

    bool stream_transport() const override { return true; }

    void finalize() override {
        for (int& f : fds_)
            if (f >= 0) {
                ::close(f);
                f = -1;
            }
    }

    double get_latency(Utils::peer_num producer, Utils::peer_num consumer, std::size_t size_in_bytes) override {
        return overhead_ + producer * consumer * (static_cast<double>(size_in_bytes) / 1e6) / bandwidth_ * 1e3;  // ms
    }
    double get_price(Utils::peer_num, Utils::peer_num, std::size_t) override { return 0.; }

private:
    int fd(Utils::peer_num peer) const {
        if (peer >= fds_.size() || fds_[peer] < 0) throw std::runtime_error("LocalSocket: no connection to peer " + std::to_string(peer));
        return fds_[peer];
    }
    std::vector<int> fds_;
    double bandwidth_;
    double overhead_;
};

}  // namespace FMI::Comm

#endif
