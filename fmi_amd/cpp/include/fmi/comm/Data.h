// FMI::Comm::Data — buffer views handed to the collectives.
//
// Same API as the reference (include/comm/Data.h:11-97): scalar Data<T>, owning Data<std::vector<A>>,
// non-owning Data<void*>, each with size_in_bytes() and data(). Added: Data<Dev::Bucket<A>>, a bucket
// resident in MI355X HBM — its data() is a device pointer and on_device() tells the channels so, which
// routes combines to the HIP kernels and transfers through device-aware staging.
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

template <typename T>
class Data {
public:
    Data() = default;
    Data(T value) : val(value) {}

    std::size_t size_in_bytes() {
        if constexpr (std::is_fundamental_v<T>) {
            return sizeof(T);
        } else {
            throw std::runtime_error("Cannot get size in bytes of non-fundamental type");
        }
    }
    char* data() { return reinterpret_cast<char*>(&val); }
    T get() const { return val; }
    static constexpr bool on_device() { return false; }

    friend std::ostream& operator<<(std::ostream& o, const Data& d) { return o << d.get(); }
    friend bool operator==(const Data& l, const Data& r) { return l.get() == r.get(); }

private:
    T val{};
};

template <typename A>
class Data<std::vector<A>> {
public:
    Data() = default;
    Data(std::size_t n) : val(n) {}
    Data(std::vector<A> value) : val(std::move(value)) {}

    std::size_t size_in_bytes() { return sizeof(A) * val.size(); }
    char* data() { return reinterpret_cast<char*>(val.data()); }
    std::vector<A> get() const { return val; }
    static constexpr bool on_device() { return false; }

private:
    std::vector<A> val;
};

template <>
class Data<void*> {
public:
    Data() = default;
    // `device` marks a pointer into device memory (a raw HBM buffer owned by the caller).
    Data(void* buf, std::size_t len, bool device = false) : buf(buf), len(len), device(device) {}

    std::size_t size_in_bytes() { return len; }
    char* data() { return reinterpret_cast<char*>(buf); }
    void* get() { return buf; }
    bool on_device() const { return device; }

private:
    void* buf = nullptr;
    std::size_t len = 0;
    bool device = false;
};

// A peer's bucket resident in HBM (move-only; get() copies it back to the host).
template <typename A>
class Data<Dev::Bucket<A>> {
public:
    Data() = default;
    explicit Data(std::size_t n) : val(n) {}
    explicit Data(const std::vector<A>& host) : val(host) {}
    Data(Dev::Bucket<A>&& bucket) : val(std::move(bucket)) {}

    std::size_t size_in_bytes() { return val.size_in_bytes(); }
    char* data() { return reinterpret_cast<char*>(val.data()); }
    std::vector<A> get() const { return val.download(); }
    Dev::Bucket<A>& bucket() { return val; }
    static constexpr bool on_device() { return true; }

private:
    Dev::Bucket<A> val;
};

}  // namespace FMI::Comm

#endif
