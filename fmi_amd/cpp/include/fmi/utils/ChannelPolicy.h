// FMI::Utils::ChannelPolicy — per-operation channel choice (mirrors reference include/utils/ChannelPolicy.h
// and src/utils/ChannelPolicy.cpp:9-29): argmin of the model latency for Hint::fast, argmin of channel
// price + FaaS runtime price for Hint::cheap. Channels are compared through their own
// get_operation_latency / get_operation_price, so an RCCL channel competes on the same terms.
// Added: channels that cannot carry the operation's buffers (host vs device), or cannot run an opaque user
// reduction function, are skipped; and the cost model of a built-in combine of two HOST buckets (after
// Communicator::use_device): the GPU (fmi_host_reduce_pair) against the host loop in place, by bucket size.
#ifndef FMI_AMD_UTILS_CHANNELPOLICY_H
#define FMI_AMD_UTILS_CHANNELPOLICY_H

#include <limits>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>

#include "../comm/Channel.h"
#include "Common.h"

namespace FMI::Utils {

class ChannelPolicy {
public:
    ChannelPolicy(std::map<std::string, std::shared_ptr<FMI::Comm::Channel>>& channels, peer_num num_peers,
                  double faas_price, Hint hint)
        : channels_(channels), num_peers_(num_peers), faas_price_(faas_price), hint_(hint) {}
    virtual ~ChannelPolicy() = default;

    virtual std::string get_channel(OperationInfo op_info) { return pick(op_info, false); }

    //! Same choice for an operation on device-resident buffers.
    virtual std::string get_device_channel(OperationInfo op_info) {
        op_info.on_device = true;
        return pick(op_info, true);
    }

    void set_hint(Hint hint) { hint_ = hint; }

    //! Host-combine crossover: smallest bucket, in bytes, whose built-in combine of two host
    //! buckets runs faster through the GPU (fmi_host_reduce_pair: the buckets cross PCIe, 2 in and 1 out) than as
    //! the host loop in place on the calling thread. Measured on MI355X by tools/host_crossover.py
    //! (profiles/r05_host_crossover_512.jsonl): page-locked buckets (the zero-copy kernel) pay from 32 MiB (GPU /
    //! host 0.98 at 32 MiB, 0.89 at 64 MiB, 0.77-0.81 from 128 MiB; 1.02 at 16 MiB); pageable buckets (staged H2D /
    //! kernel / D2H) at no size measured, up to 512 MiB (1.11-1.22); both lose by 15-40x at 64 KiB, where the call
    //! costs its launch and PCIe latency, not its bytes.
    static constexpr std::size_t kHostCombinePinnedMinBytes = std::size_t(32) << 20;
    static constexpr std::size_t kHostCombinePageableMinBytes = std::numeric_limits<std::size_t>::max();

    //! Does a built-in combine of two host buckets of `bucket_bytes` pay on the GPU? (Communicator::use_device
    //! asks this per combine; use_device(d, true) skips it.)
    virtual bool host_combine_on_device(std::size_t bucket_bytes, bool page_locked) const {
        return bucket_bytes >= (page_locked ? host_pinned_min_ : host_pageable_min_);
    }
    //! Below this no host combine goes to the GPU, page-locked or not: the Communicator asks nothing more then.
    virtual std::size_t host_combine_min_bytes() const { return std::min(host_pageable_min_, host_pinned_min_); }
    void set_host_combine_min_bytes(std::size_t pageable, std::size_t page_locked) {
        host_pageable_min_ = pageable;
        host_pinned_min_ = page_locked;
    }

protected:
    std::string pick(const OperationInfo& op_info, bool on_device) {
        std::string best;
        double best_score = std::numeric_limits<double>::infinity();
        for (const auto& [name, channel] : channels_) {
            if (on_device ? !channel->supports_device_buffers() : !channel->supports_host_buffers()) continue;
            if (op_info.user_function && !channel->supports_user_functions()) continue;
            const double latency = channel->get_operation_latency(op_info);
            const double score = hint_ == fast ? latency : channel->get_operation_price(op_info) + latency * faas_price_;
            if (best.empty() || score < best_score) {
                best = name;
                best_score = score;
            }
        }
        if (best.empty())
            throw std::runtime_error(std::string("no registered channel can carry ") + (on_device ? "device" : "host") +
                                     " buffers");
        return best;
    }

    std::map<std::string, std::shared_ptr<FMI::Comm::Channel>>& channels_;
    peer_num num_peers_;
    double faas_price_;
    Hint hint_;
    std::size_t host_pageable_min_ = kHostCombinePageableMinBytes;
    std::size_t host_pinned_min_ = kHostCombinePinnedMinBytes;
};

}  // namespace FMI::Utils

#endif
