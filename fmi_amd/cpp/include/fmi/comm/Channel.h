// FMI::Comm::Channel — the transport/collective plugin interface (mirrors reference
// include/comm/Channel.h:16-136 and src/comm/Channel.cpp:19-54).
//
// The type-erased op and buffer keep the reference's shape — raw_function{f, associative, commutative}
// and channel_data{buf, len}, so `{f, true, true}` and `{ptr, len}` still aggregate-initialise — with
// one defaulted field each:
//   raw_function::device   the built-in op as (op, dtype, count) when the Function carries one;
//   channel_data::on_device  buf points into HBM (channels stage transfers and run combines on the GPU).
#ifndef FMI_AMD_COMM_CHANNEL_H
#define FMI_AMD_COMM_CHANNEL_H

#include <cstddef>
#include <functional>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>

#include "../dev/Device.h"
#include "../utils/Common.h"
#include "../utils/Function.h"
#include "Data.h"

//! Type-erased combine: overwrites its first argument with f(first, second) (reference Channel.h:16).
using raw_func = std::function<void(char*, char*)>;

//! Built-in op of a raw_function, evaluable by the device kernels (C-ABI fmi_op_t / fmi_dtype_t).
struct device_op {
    int op = -1;
    int dtype = -1;
    std::size_t count = 0;
    bool valid() const { return op >= 0 && dtype >= 0; }
};

//! The same combine restricted to bytes [offset, offset + len) of both buckets; len and offset are whole
//! elements. Lets a stream transport combine chunk k while chunk k+1 is still in flight.
using raw_part_func = std::function<void(char*, char*, std::size_t offset, std::size_t len)>;

struct raw_function {
    raw_func f;  // overwrites the left argument
    bool associative;
    bool commutative;
    device_op device{};
    raw_part_func part{};     // optional (built-in ops on host buckets)
    std::size_t granule = 0;  // element size in bytes for `part`
};

struct channel_data {
    char* buf;
    std::size_t len;
    bool on_device = false;
};

namespace FMI::Comm {

class Channel {
public:
    virtual ~Channel() = default;

    virtual void send(channel_data buf, FMI::Utils::peer_num dest) = 0;
    virtual void recv(channel_data buf, FMI::Utils::peer_num src) = 0;
    virtual void bcast(channel_data buf, FMI::Utils::peer_num root) = 0;
    virtual void barrier() = 0;

    //! Default gather: every peer sends to root, root receives in peer order (reference Channel.cpp:19-32).
    virtual void gather(channel_data sendbuf, channel_data recvbuf, FMI::Utils::peer_num root) {
        if (peer_id != root) {
            send(sendbuf, root);
            return;
        }
        for (FMI::Utils::peer_num p = 0; p < num_peers; ++p) {
            channel_data slot{recvbuf.buf + p * sendbuf.len, sendbuf.len, recvbuf.on_device};
            if (p == root)
                Dev::copy_bytes(slot.buf, slot.on_device, sendbuf.buf, sendbuf.on_device, sendbuf.len);
            else
                recv(slot, p);
        }
    }

    //! Default scatter: root sends each peer its slice (reference Channel.cpp:34-49).
    virtual void scatter(channel_data sendbuf, channel_data recvbuf, FMI::Utils::peer_num root) {
        if (peer_id != root) {
            recv(recvbuf, root);
            return;
        }
        for (FMI::Utils::peer_num p = 0; p < num_peers; ++p) {
            channel_data slice{sendbuf.buf + p * recvbuf.len, recvbuf.len, sendbuf.on_device};
            if (p == root)
                Dev::copy_bytes(recvbuf.buf, recvbuf.on_device, slice.buf, slice.on_device, recvbuf.len);
            else
                send(slice, p);
        }
    }

    virtual void reduce(channel_data sendbuf, channel_data recvbuf, FMI::Utils::peer_num root, raw_function f) = 0;

    //! Default allreduce = reduce to peer 0 + bcast (reference Channel.cpp:51-54).
    virtual void allreduce(channel_data sendbuf, channel_data recvbuf, raw_function f) {
        reduce(sendbuf, recvbuf, 0, f);
        bcast(recvbuf, 0);
    }

    virtual void scan(channel_data sendbuf, channel_data recvbuf, raw_function f) = 0;

    void set_peer_id(FMI::Utils::peer_num num) { peer_id = num; }
    void set_num_peers(FMI::Utils::peer_num num) { num_peers = num; }
    void set_comm_name(std::string name) { comm_name = std::move(name); }

    //! Called by the Communicator's destructor before the channel is released.
    virtual void finalize() {}

    //! Whether the channel can move buffers that live in device memory (all channels here can; the
    //! policy uses it to keep device buckets off channels that cannot).
    virtual bool supports_device_buffers() const { return true; }
    virtual bool supports_host_buffers() const { return true; }
    //! Whether reductions may be opaque user functions (raw_function::f); device collectives need a
    //! built-in op (raw_function::device).
    virtual bool supports_user_functions() const { return true; }

    virtual double get_latency(Utils::peer_num producer, Utils::peer_num consumer, std::size_t size_in_bytes) = 0;
    virtual double get_price(Utils::peer_num producer, Utils::peer_num consumer, std::size_t size_in_bytes) = 0;
    virtual double get_operation_latency(Utils::OperationInfo op_info) = 0;
    virtual double get_operation_price(Utils::OperationInfo op_info) = 0;

protected:
    FMI::Utils::peer_num peer_id = 0;
    FMI::Utils::peer_num num_peers = 1;
    std::string comm_name;
};

}  // namespace FMI::Comm

#endif
