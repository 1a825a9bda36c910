// FMI::Comm::Data — the buffer views the collectives move and combine.
//
// The public members are those of reference include/comm/Data.h:11-97 (size_in_bytes(), data(), get(),
// the same constructors and the same runtime error for a non-fundamental scalar), for four payloads:
//   Data<T>                 one scalar, held by value
//   Data<std::vector<A>>    an owned host bucket
//   Data<void*>             a caller-owned byte range (host, or device when flagged)
//   Data<Dev::Bucket<A>>    an owned bucket resident in MI355X HBM (extension)
// Every view also answers on_device(), which the channels use to route the combine to the HIP kernels and
// transfers through device-aware staging.
#ifndef FMI_AMD_COMM_DATA_H
#define FMI_AMD_COMM_DATA_H

#include <cstddef>
#include <ostream>
#include <stdexcept>
#include <type_traits>
#include <utility>
#include <vector>

#include "../dev/Device.h"

namespace FMI::Comm {

namespace detail {
// The (pointer, byte count) face every payload shows the channels; Derived supplies bytes() and base().
template <class Derived>
class ByteView {
public:
    std::size_t size_in_bytes() { return self().bytes(); }
    char* data() { return reinterpret_cast<char*>(self().base()); }

private:
    Derived& self() { return static_cast<Derived&>(*this); }
};
}  // namespace detail

template <typename T>
class Data : public detail::ByteView<Data<T>> {
public:
    Data() = default;
    Data(T value) : value_(value) {}

    T get() const { return value_; }
    static constexpr bool on_device() { return false; }

    friend std::ostream& operator<<(std::ostream& os, const Data& d) { return os << d.value_; }
    friend bool operator==(const Data& a, const Data& b) { return a.value_ == b.value_; }

private:
    friend class detail::ByteView<Data<T>>;
    std::size_t bytes() const {
        if constexpr (!std::is_fundamental_v<T>)
            throw std::runtime_error("Cannot get size in bytes of non-fundamental type");
        return sizeof(T);
    }
    void* base() { return &value_; }

    T value_{};
};

template <typename A>
class Data<std::vector<A>> : public detail::ByteView<Data<std::vector<A>>> {
public:
    Data() = default;
    Data(std::size_t n) : elems_(n) {}
    Data(std::vector<A> value) : elems_(std::move(value)) {}

    std::vector<A> get() const { return elems_; }
    static constexpr bool on_device() { return false; }

private:
    friend class detail::ByteView<Data<std::vector<A>>>;
    std::size_t bytes() const { return elems_.size() * sizeof(A); }
    void* base() { return elems_.data(); }

    std::vector<A> elems_;
};

template <>
class Data<void*> : public detail::ByteView<Data<void*>> {
public:
    Data() = default;
    // `device` marks a range in device memory (a raw HBM buffer the caller owns).
    Data(void* buf, std::size_t len, bool device = false) : ptr_(buf), len_(len), device_(device) {}

    void* get() { return ptr_; }
    bool on_device() const { return device_; }

private:
    friend class detail::ByteView<Data<void*>>;
    std::size_t bytes() const { return len_; }
    void* base() { return ptr_; }

    void* ptr_ = nullptr;
    std::size_t len_ = 0;
    bool device_ = false;
};

// A peer's bucket resident in HBM (move-only; get() downloads a host copy).
template <typename A>
class Data<Dev::Bucket<A>> : public detail::ByteView<Data<Dev::Bucket<A>>> {
public:
    Data() = default;
    explicit Data(std::size_t n) : bucket_(n) {}
    explicit Data(const std::vector<A>& host) : bucket_(host) {}
    Data(Dev::Bucket<A>&& bucket) : bucket_(std::move(bucket)) {}

    std::vector<A> get() const { return bucket_.download(); }
    Dev::Bucket<A>& bucket() { return bucket_; }
    static constexpr bool on_device() { return true; }

private:
    friend class detail::ByteView<Data<Dev::Bucket<A>>>;
    std::size_t bytes() const { return bucket_.size_in_bytes(); }
    void* base() { return bucket_.data(); }

    Dev::Bucket<A> bucket_;
};

}  // namespace FMI::Comm

#endif
