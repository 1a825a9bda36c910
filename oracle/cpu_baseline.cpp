// ORACLE / CPU BASELINE — TEST INFRASTRUCTURE ONLY. Built by __graft_entry__.build() into
// oracle/build/cpu_baseline and run only by bench.py's cpu_baseline leg and tests/; never linked into
// the product.
//
// A C++ restatement ("port") of the reference's CPU bucket reduction as it actually executes, so the
// GPU numbers can be reported beside it on the same host:
//   adapter  — Communicator::convert_to_raw_function for vector buckets (reference
//              include/Communicator.h:180-189): copy both buckets into std::vectors, call the typed
//              Function by value (reference include/utils/Function.h:11-13 — another two copies through
//              std::function), memcpy the result back; the functor is the reference's built-in
//              std::transform loop (reference python/PythonCommunicator.h:131-149). Single thread, as FMI.
//   bare     — the std::transform loop alone, single thread.
//   omp      — the same loop over all host cores (a CPU roofline, not something FMI does).
// Inputs: the counter-based generator of SURVEY.md §8d (identical to fmi_dev_fill_synthetic).
// Output: one JSON object on stdout; with --dump PATH also the combined bucket as raw bytes (for
// tests/test_oracle.py, which checks the port's bits against the numpy oracle).
#include <omp.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

namespace {

uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

template <class T>
T synth(uint64_t h) {
    if constexpr (std::is_same_v<T, float>) return static_cast<float>(h >> 40) * 0x1p-24f * 2.0f - 1.0f;
    if constexpr (std::is_same_v<T, double>) return static_cast<double>(h >> 11) * 0x1p-53 * 2.0 - 1.0;
    if constexpr (std::is_same_v<T, int32_t>) return static_cast<int32_t>(static_cast<uint32_t>(h >> 32));
    if constexpr (std::is_same_v<T, int64_t>) return static_cast<int64_t>(h);
}

template <class T>
void fill(std::vector<T>& v, uint64_t seed, uint32_t peer) {
    const uint64_t key = seed ^ (static_cast<uint64_t>(peer) << 40);
#pragma omp parallel for schedule(static)
    for (size_t i = 0; i < v.size(); ++i) v[i] = synth<T>(splitmix64(key ^ i));
}

// The typed reduction function object: std::function + flags, called by value (the reference's
// Function<T>::operator()(T a, T b) const takes both buckets by value).
template <class T>
struct TypedFunction {
    std::function<T(T, T)> f;
    bool commutative;
    bool associative;
    T operator()(T a, T b) const { return f(a, b); }
};

template <class A, class Op>
std::function<void(char*, char*)> adapter(TypedFunction<std::vector<A>> fn, size_t bytes) {
    // restates include/Communicator.h:182-187: two vector copies in, by-value call, memcpy out
    return [fn, bytes](char* a, char* b) {
        std::vector<A> va(reinterpret_cast<A*>(a), reinterpret_cast<A*>(a + bytes));
        std::vector<A> vb(reinterpret_cast<A*>(b), reinterpret_cast<A*>(b + bytes));
        std::vector<A> r = fn(va, vb);
        std::memcpy(a, r.data(), bytes);
    };
}

// The reference's built-in element functors (python/PythonCommunicator.h:133-143): std::plus and a
// lambda around std::max; both inline into std::transform.
template <class A>
struct MaxOf {
    A operator()(A x, A y) const { return std::max(x, y); }
};

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <class A, class Elem>
int run(const std::string& mode, const std::string& op, size_t n, int reps, const std::string& dump) {
    std::vector<A> a(n), b(n), a0;
    fill(a, 42, 0);
    fill(b, 42, 1);
    a0 = a;
    const Elem elem{};
    TypedFunction<std::vector<A>> fn{[elem](std::vector<A> x, std::vector<A> y) {
                                         std::transform(x.begin(), x.end(), y.begin(), x.begin(), elem);
                                         return x;
                                     },
                                     true, true};
    const size_t bytes = n * sizeof(A);
    auto raw = adapter<A, void>(fn, bytes);
    std::vector<double> times;
    for (int r = 0; r <= reps; ++r) {  // first iteration is the warm-up
        std::memcpy(a.data(), a0.data(), bytes);
        const double t0 = now_ms();
        if (mode == "adapter") {
            raw(reinterpret_cast<char*>(a.data()), reinterpret_cast<char*>(b.data()));
        } else if (mode == "bare") {
            std::transform(a.begin(), a.end(), b.begin(), a.begin(), elem);
        } else {
#pragma omp parallel for schedule(static)
            for (size_t i = 0; i < n; ++i) a[i] = elem(a[i], b[i]);
        }
        const double t1 = now_ms();
        if (r > 0) times.push_back(t1 - t0);
    }
    // check the combine against a plain loop (all three modes compute the same bits)
    size_t bad = 0;
    for (size_t i = 0; i < n; ++i) {
        const A w = elem(a0[i], b[i]);
        bad += std::memcmp(&w, &a[i], sizeof(A)) != 0;
    }
    if (!dump.empty()) {
        FILE* f = std::fopen(dump.c_str(), "wb");
        if (!f || std::fwrite(a.data(), 1, bytes, f) != bytes) return 4;
        std::fclose(f);
    }
    std::sort(times.begin(), times.end());
    const double med = times[times.size() / 2];
    const int threads = mode == "omp" ? omp_get_max_threads() : 1;
    std::printf(
        "{\"mode\": \"%s\", \"op\": \"%s\", \"n\": %zu, \"bytes\": %zu, \"reps\": %d, \"threads\": %d, "
        "\"median_ms\": %.4f, \"min_ms\": %.4f, \"bucket_gib_s\": %.4f, \"traffic_gb_s\": %.4f, \"mismatches\": %zu}\n",
        mode.c_str(), op.c_str(), n, bytes, reps, threads, med, times.front(), bytes / (med * 1e-3) / (1u << 30),
        3.0 * bytes / (med * 1e-3) / 1e9, bad);
    return bad == 0 ? 0 : 3;
}

}  // namespace

int main(int argc, char** argv) {
    std::string mode = "adapter", dtype = "f32", op = "sum", dump;
    double mib = 256;
    int reps = 5;
    for (int i = 1; i + 1 < argc; i += 2) {
        const std::string k = argv[i], v = argv[i + 1];
        if (k == "--mode") mode = v;
        else if (k == "--dtype") dtype = v;
        else if (k == "--op") op = v;
        else if (k == "--mib") mib = std::atof(v.c_str());
        else if (k == "--reps") reps = std::atoi(v.c_str());
        else if (k == "--dump") dump = v;
        else {
            std::fprintf(stderr, "unknown option %s\n", k.c_str());
            return 2;
        }
    }
    if (mode != "adapter" && mode != "bare" && mode != "omp") return 2;
    const size_t bytes = static_cast<size_t>(mib * (1 << 20));
    const bool mx = op == "max";
    if (op != "sum" && op != "max") return 2;
    if (dtype == "f32") return mx ? run<float, MaxOf<float>>(mode, op, bytes / 4, reps, dump) : run<float, std::plus<float>>(mode, op, bytes / 4, reps, dump);
    if (dtype == "f64") return mx ? run<double, MaxOf<double>>(mode, op, bytes / 8, reps, dump) : run<double, std::plus<double>>(mode, op, bytes / 8, reps, dump);
    if (dtype == "i32") return mx ? run<int32_t, MaxOf<int32_t>>(mode, op, bytes / 4, reps, dump) : run<int32_t, std::plus<int32_t>>(mode, op, bytes / 4, reps, dump);
    if (dtype == "i64") return mx ? run<int64_t, MaxOf<int64_t>>(mode, op, bytes / 8, reps, dump) : run<int64_t, std::plus<int64_t>>(mode, op, bytes / 8, reps, dump);
    return 2;
}
