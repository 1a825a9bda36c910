// FMI::Utils common vocabulary (mirrors reference include/utils/Common.h:8-32 — same names and meaning, so
// code written against the reference compiles unchanged).
#ifndef FMI_AMD_UTILS_COMMON_H
#define FMI_AMD_UTILS_COMMON_H

#include <cstddef>
#include <exception>

namespace FMI::Utils {

// Peer ids are 0 .. num_peers-1.
using peer_num = unsigned int;

// Thrown when a transport gives up waiting (reference: SO_RCVTIMEO expiry in Direct, poll expiry in
// ClientServer). Device/RCCL timeouts surface as the same type.
struct Timeout : public std::exception {
    const char* what() const noexcept override { return "Timeout was reached"; }
};

// Optimisation objective of the channel policy.
enum Hint { fast, cheap };

// Collectives a channel implements; the policy is consulted per operation.
enum Operation { send, bcast, barrier, gather, scatter, reduce, allreduce, scan };

struct OperationInfo {
    Operation op;
    std::size_t data_size;
    bool left_to_right = false;
    bool on_device = false;  // extension: the buffers live in GPU memory (channel models add staging)
    bool user_function = false;  // extension: the reduction is an opaque user function (no built-in op)
};

}  // namespace FMI::Utils

#endif
