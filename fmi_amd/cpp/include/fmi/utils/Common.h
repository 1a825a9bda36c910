// FMI::Utils — the vocabulary every other header uses. Names, enumerator order and the timeout message are
// those of reference include/utils/Common.h:8-32, so code written against the reference compiles and
// behaves unchanged; OperationInfo carries two extra, defaulted fields for the device-aware cost models.
#ifndef FMI_AMD_UTILS_COMMON_H
#define FMI_AMD_UTILS_COMMON_H

#include <cstddef>
#include <exception>

namespace FMI::Utils {

// Collectives, in the reference's enumerator order (ChannelPolicy and the cost models switch on them).
enum Operation { send, bcast, barrier, gather, scatter, reduce, allreduce, scan };

// What ChannelPolicy minimises: modelled latency (fast) or modelled price (cheap).
enum Hint { fast, cheap };

// A peer's rank in [0, num_peers).
using peer_num = unsigned int;

// Raised when a transport stops waiting for a peer: socket SO_RCVTIMEO / SO_SNDTIMEO expiry (LocalSocket,
// the reference's Direct), a Loopback wait, or a device/RCCL wait.
class Timeout : public std::exception {
public:
    const char* what() const noexcept override;
};
inline const char* Timeout::what() const noexcept { return "Timeout was reached"; }

// Per-call facts the policy and the channel cost models see.
struct OperationInfo {
    Operation op;
    std::size_t data_size;                // bytes per peer bucket
    bool left_to_right = false;           // the op is not both commutative and associative
    bool on_device = false;               // extension: buckets live in GPU memory
    bool user_function = false;           // extension: opaque user lambda (no built-in op id)
};

}  // namespace FMI::Utils

#endif
