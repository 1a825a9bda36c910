// FMI::Utils::Function — the reduction function object passed to reduce / allreduce / scan.
//
// Source-compatible with the reference (include/utils/Function.h:6-21): Function<T>(std::function<T(T,T)>,
// commutative, associative), call operator, public `commutative` / `associative` flags.
//
// MI355X extension: the reference's closure is opaque — no op id, no dtype — so a device
// cannot evaluate it. A Function built from a *built-in op* (Function<T>(Op::sum)) carries the op id the
// reference's Python layer already names (python/PythonCommunicator.h:13-15, 131-149) next to an
// equivalent host closure; channels then run the combine as a HIP kernel when the buckets are
// device-resident (or when host offload is enabled), and the host closure otherwise. User lambdas keep
// the reference's host-only behaviour.
#ifndef FMI_AMD_UTILS_FUNCTION_H
#define FMI_AMD_UTILS_FUNCTION_H

#include <algorithm>
#include <functional>
#include <stdexcept>
#include <type_traits>
#include <vector>

#include "fmi_dev.h"

namespace FMI::Dev {
template <class A>
class Bucket;
}

namespace FMI::Utils {

// Built-in reduction ops; numeric values are the C-ABI's fmi_op_t.
enum class Op : int { none = -1, sum = FMI_OP_SUM, prod = FMI_OP_PROD, max = FMI_OP_MAX, min = FMI_OP_MIN };

namespace detail {

// Integers wrap: computed in an unsigned type at least as wide as unsigned int (so sub-int types do not
// promote to a signed int that could overflow), then converted back to A, keeping the low bits.
template <class A>
using wrap_t = std::common_type_t<std::make_unsigned_t<A>, unsigned int>;

template <class A>
A apply_op(Op op, A a, A b) {
    switch (op) {
        case Op::sum:
            if constexpr (std::is_integral_v<A>)
                return static_cast<A>(static_cast<wrap_t<A>>(a) + static_cast<wrap_t<A>>(b));
            else
                return a + b;
        case Op::prod:
            if constexpr (std::is_integral_v<A>)
                return static_cast<A>(static_cast<wrap_t<A>>(a) * static_cast<wrap_t<A>>(b));
            else
                return a * b;
        case Op::max: return std::max(a, b);  // (a < b) ? b : a
        case Op::min: return std::min(a, b);  // (b < a) ? b : a
        default: throw std::runtime_error("Function: no built-in op");
    }
}

// The host closure equivalent to a built-in op, for each kind of T.
template <class T>
struct HostBuiltin {
    static std::function<T(T, T)> make(Op op) {
        return [op](T a, T b) { return apply_op<T>(op, a, b); };
    }
};

template <class A>
struct HostBuiltin<std::vector<A>> {
    static std::function<std::vector<A>(std::vector<A>, std::vector<A>)> make(Op op) {
        return [op](std::vector<A> a, std::vector<A> b) {
            std::transform(a.begin(), a.end(), b.begin(), a.begin(), [op](A x, A y) { return apply_op<A>(op, x, y); });
            return a;
        };
    }
};

// Device buckets have no host closure: their combine is always the kernel.
template <class A>
struct HostBuiltin<Dev::Bucket<A>> {
    static std::function<Dev::Bucket<A>(Dev::Bucket<A>, Dev::Bucket<A>)> make(Op) { return nullptr; }
};

}  // namespace detail

template <typename T>
class Function {
public:
    // Reference constructor: an arbitrary host function; host-only.
    Function(std::function<T(T, T)> f, bool commutative, bool associative)
        : commutative(commutative), associative(associative), f_(std::move(f)) {}

    // Built-in op: commutative and associative (the reference's built-ins are registered as such,
    // python/PythonCommunicator.h:133-149), evaluable on the device.
    explicit Function(Op op) : commutative(true), associative(true), f_(detail::HostBuiltin<T>::make(op)), op_(op) {
        if (op == Op::none) throw std::runtime_error("Function: Op::none is not a built-in op");
    }

    T operator()(T a, T b) const {
        if (!f_) throw std::runtime_error("Function: device-bucket functions have no host evaluation");
        return f_(std::move(a), std::move(b));
    }

    Op builtin() const { return op_; }

    //! User provided information about commutativity
    bool commutative;
    //! User provided information about associativity
    bool associative;

private:
    std::function<T(T, T)> f_;
    Op op_ = Op::none;
};

}  // namespace FMI::Utils

#endif
