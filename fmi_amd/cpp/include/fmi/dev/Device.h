// FMI::Dev — C++ RAII layer over the C-ABI in include/fmi_dev.h (libfmi_dev.so, gfx950).
//
// Error convention: a C-ABI FMI_ERR_TIMEOUT becomes FMI::Utils::Timeout (reference
// include/utils/Common.h:11-15, what its channels throw when a peer stays away, src/comm/Direct.cpp:28-30);
// every other status != 0 a std::runtime_error carrying fmi_last_error(), the exception type the reference
// itself throws for usage errors (reference include/Communicator.h:90,114,138).
#ifndef FMI_AMD_DEV_DEVICE_H
#define FMI_AMD_DEV_DEVICE_H

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <limits>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "../utils/Common.h"
#include "fmi_dev.h"  // C-ABI: add -I<repo>/include

namespace FMI::Dev {

inline void check(int status, const char* what) {
    if (status == FMI_ERR_TIMEOUT) throw Utils::Timeout();
    if (status != FMI_OK) throw std::runtime_error(std::string(what) + ": " + fmi_last_error());
}

// The C-ABI element type of a fundamental A (any integer type by width and signedness, so long long and
// char map too), or -1: bool, long double and non-arithmetic types stay on the host.
template <class A>
constexpr int dtype_of() {
    if constexpr (std::is_same_v<A, float>) return FMI_F32;
    else if constexpr (std::is_same_v<A, double>) return FMI_F64;
    else if constexpr (std::is_integral_v<A> && !std::is_same_v<A, bool>) {
        constexpr bool s = std::is_signed_v<A>;
        switch (sizeof(A)) {
            case 1: return s ? FMI_I8 : FMI_U8;
            case 2: return s ? FMI_I16 : FMI_U16;
            case 4: return s ? FMI_I32 : FMI_U32;
            case 8: return s ? FMI_I64 : FMI_U64;
            default: return -1;
        }
    } else {
        return -1;
    }
}

template <class A>
constexpr bool device_type = dtype_of<A>() >= 0;

// Select the device for this process (one process per GPU, as FMI runs one peer per process).
inline void init(int device = 0) { check(fmi_dev_init(device), "fmi_dev_init"); }

inline bool available() {
    int n = 0;
    return fmi_dev_count(&n) == FMI_OK && n > 0;
}

inline void sync() { check(fmi_dev_sync(), "fmi_dev_sync"); }

// A device-resident bucket of n elements of A (owning, move-only).
template <class A>
class Bucket {
    static_assert(device_type<A>, "device buckets hold float, double or 8/16/32/64-bit integers");

public:
    using value_type = A;
    Bucket() = default;
    explicit Bucket(std::size_t n) : n_(n) {
        void* p = nullptr;
        check(fmi_dev_alloc(&p, n * sizeof(A)), "fmi_dev_alloc");
        ptr_ = static_cast<A*>(p);
    }
    explicit Bucket(const std::vector<A>& host) : Bucket(host.size()) { upload(host); }
    //! `count` buckets of n elements that one kernel streams together (a peer set's inputs and outputs): bucket j
    //! in 4 KiB slot j mod 16 whatever was allocated before (fmi_dev_alloc_group).
    static std::vector<Bucket> group(std::size_t count, std::size_t n) {
        if (count > static_cast<std::size_t>(std::numeric_limits<int>::max()))
            throw std::runtime_error("Bucket::group: too many buckets");
        std::vector<void*> ptrs(count);
        check(fmi_dev_alloc_group(ptrs.data(), static_cast<int>(count), n * sizeof(A)), "fmi_dev_alloc_group");
        std::vector<Bucket> out(count);
        for (std::size_t j = 0; j < count; ++j) {
            out[j].ptr_ = static_cast<A*>(ptrs[j]);
            out[j].n_ = n;
        }
        return out;
    }
    //! A bucket over memory owned elsewhere (e.g. a communicator window): never freed by the bucket.
    static Bucket borrow(A* ptr, std::size_t n) {
        Bucket b;
        b.ptr_ = ptr;
        b.n_ = n;
        b.owns_ = false;
        return b;
    }
    Bucket(const Bucket&) = delete;
    Bucket& operator=(const Bucket&) = delete;
    Bucket(Bucket&& o) noexcept
        : ptr_(std::exchange(o.ptr_, nullptr)), n_(std::exchange(o.n_, 0)), owns_(std::exchange(o.owns_, true)) {}
    Bucket& operator=(Bucket&& o) noexcept {
        if (this != &o) {
            release();
            ptr_ = std::exchange(o.ptr_, nullptr);
            n_ = std::exchange(o.n_, 0);
            owns_ = std::exchange(o.owns_, true);
        }
        return *this;
    }
    ~Bucket() { release(); }

    A* data() const { return ptr_; }
    std::size_t size() const { return n_; }
    std::size_t size_in_bytes() const { return n_ * sizeof(A); }

    void upload(const std::vector<A>& host) {
        if (host.size() != n_) throw std::runtime_error("Bucket::upload: size mismatch");
        check(fmi_dev_h2d_async(ptr_, host.data(), size_in_bytes(), nullptr), "fmi_dev_h2d_async");
        check(fmi_stream_sync(nullptr), "fmi_stream_sync");
    }
    std::vector<A> download() const {
        std::vector<A> host(n_);
        check(fmi_dev_d2h_async(host.data(), ptr_, size_in_bytes(), nullptr), "fmi_dev_d2h_async");
        check(fmi_stream_sync(nullptr), "fmi_stream_sync");
        return host;
    }
    void fill_synthetic(uint64_t seed, uint32_t peer) {
        check(fmi_dev_fill_synthetic(dtype_of<A>(), ptr_, n_, seed, peer, nullptr), "fmi_dev_fill_synthetic");
    }

private:
    void release() noexcept {
        if (ptr_ && owns_) (void)fmi_dev_free(ptr_);
        ptr_ = nullptr;
        n_ = 0;
        owns_ = true;
    }
    A* ptr_ = nullptr;
    std::size_t n_ = 0;
    bool owns_ = true;
};

// Untyped device scratch used by the channel algorithms for temporaries of device-resident buckets.
class Scratch {
public:
    Scratch() = default;
    Scratch(std::size_t bytes, bool on_device) : bytes_(bytes), device_(on_device) {
        if (device_) {
            void* p = nullptr;
            check(fmi_dev_alloc(&p, bytes ? bytes : 1), "fmi_dev_alloc (scratch)");
            ptr_ = static_cast<char*>(p);
        } else {
            ptr_ = new char[bytes ? bytes : 1];
        }
    }
    Scratch(const Scratch&) = delete;
    Scratch& operator=(const Scratch&) = delete;
    Scratch& operator=(Scratch&& o) noexcept {
        if (this != &o) {
            release();
            ptr_ = std::exchange(o.ptr_, nullptr);
            bytes_ = o.bytes_;
            device_ = o.device_;
        }
        return *this;
    }
    ~Scratch() { release(); }
    char* get() const { return ptr_; }

private:
    void release() noexcept {
        if (!ptr_) return;
        if (device_)
            (void)fmi_dev_free(ptr_);
        else
            delete[] ptr_;
        ptr_ = nullptr;
    }
    char* ptr_ = nullptr;
    std::size_t bytes_ = 0;
    bool device_ = false;
};

// Page-locks an existing host range for its lifetime (fmi_host_register), e.g. the storage of a
// Data<std::vector<A>> recv buffer reused across collectives, so host-bucket combines take the zero-copy
// path. The range must outlive the registration. Move-only.
class HostRegistration {
public:
    HostRegistration() = default;
    HostRegistration(void* ptr, std::size_t bytes) : ptr_(ptr) { check(fmi_host_register(ptr, bytes), "fmi_host_register"); }
    template <class A>
    explicit HostRegistration(std::vector<A>& v) : HostRegistration(v.data(), v.size() * sizeof(A)) {}
    HostRegistration(const HostRegistration&) = delete;
    HostRegistration& operator=(const HostRegistration&) = delete;
    HostRegistration(HostRegistration&& o) noexcept : ptr_(std::exchange(o.ptr_, nullptr)) {}
    HostRegistration& operator=(HostRegistration&& o) noexcept {
        if (this != &o) {
            release();
            ptr_ = std::exchange(o.ptr_, nullptr);
        }
        return *this;
    }
    ~HostRegistration() { release(); }

private:
    void release() noexcept {
        if (ptr_) (void)fmi_host_unregister(ptr_);
        ptr_ = nullptr;
    }
    void* ptr_ = nullptr;
};

// Byte copy that knows where both sides live (host-host memcpy, device-device D2D, staged otherwise).
inline void copy_bytes(char* dst, bool dst_dev, const char* src, bool src_dev, std::size_t len) {
    if (len == 0 || dst == src) return;
    if (!dst_dev && !src_dev) {
        std::copy(src, src + len, dst);
        return;
    }
    int rc;
    if (dst_dev && src_dev) rc = fmi_dev_d2d_async(dst, src, len, nullptr);
    else if (dst_dev) rc = fmi_dev_h2d_async(dst, src, len, nullptr);
    else rc = fmi_dev_d2h_async(dst, src, len, nullptr);
    check(rc, "device copy");
    check(fmi_stream_sync(nullptr), "fmi_stream_sync");
}

}  // namespace FMI::Dev

#endif
