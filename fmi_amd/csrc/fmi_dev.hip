// fmi_dev.hip — C-ABI implementation (include/fmi_dev.h): device state, memory, streams, events, the
// pairwise hot kernel's launch policy, P-way dispatch, the host-ingress pipeline and synthetic buckets.
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <vector>

#include "fmi_internal.h"

namespace fmi::dev {

namespace {

thread_local std::string t_last_error;

struct DeviceState {
    int device = -1;
    int num_cus = 256;
    size_t lds_per_cu = 160 * 1024;  // gfx950
    size_t lds_per_wg = 160 * 1024;
    hipStream_t stream = nullptr;
    // scratch arena for the pairwise-pass execution of P-way programs; arena_free marks when the work
    // that last used it has drained (the next user's stream waits on it)
    void* arena = nullptr;
    size_t arena_bytes = 0;
    hipEvent_t arena_free = nullptr;
};

std::mutex g_mu;
DeviceState g_state;

// Bucket placement (fmi_dev_alloc / fmi_dev_alloc_group). A fused kernel reads its P buckets at the same
// offset at the same time. Separate hipMallocs of large buckets start on 2 MiB boundaries, so those P streams sit at
// the same offset modulo every HBM interleave period below 2 MiB, and they collide: the 8-way tree at 512 MiB per
// peer ran 0.71 of peak on separate allocations, 0.62 with the buckets packed back to back, and 0.83 with bucket j
// shifted by j x 4 KiB (profiles/r05_skew_sweep.jsonl, tools/skew_sweep.py). Shifts of 16, 32 or 64 KiB collide
// again: what counts is a distinct 4 KiB slot modulo 64 KiB for each stream. The pairwise kernel is the other way
// round: it runs fastest with both operands at their 2 MiB-aligned base, and 1.8-1.9 % slower when they sit in
// nonzero slots (profiles/r06a_placement_ab.jsonl, r06b_placement_ab.jsonl: two boxes, kernel traces). So a plain
// fmi_dev_alloc is a plain hipMalloc (FMI_TUNE_ALLOC_SLOTS = 0, the default since round 6), and the buckets one fused
// kernel streams together are allocated as one group (fmi_dev_alloc_group): carved from ONE allocation, bucket j in
// slot j mod 16, whatever was allocated before. One allocation matters as much as the slots: the 8-way tree over 1 GiB
// buckets reads 0.83 carved against 0.79-0.81 for the same slots in separate hipMallocs, whose rate also swings with
// where each allocation's memory comes from (profiles/r06f_placement_ab_trace.jsonl, r06b_placement_ab_trace.jsonl).
// FMI_TUNE_ALLOC_SLOTS = 1 restores round 5's rotation of every fmi_dev_alloc over the 16 slots.
constexpr size_t kSlotBytes = 4096, kSlots = 16, kSlotSpan = kSlotBytes * kSlots, kSlotMinBytes = size_t(1) << 20;
std::mutex g_slots_mu;
size_t g_next_slot = 0;
std::map<void*, void*> g_slotted;  // pointer handed out -> its hipMalloc base
struct Group {
    void* base;  // the group's one hipMalloc
    int live;    // its buckets not yet freed
};
std::map<void*, Group*> g_grouped;  // a group's bucket -> its group

// Host-ingress pipeline of fmi_host_reduce_pair: two slots of (a, b) device staging and two streams per SET. The
// reference's peers combine concurrently when they are threads of one process (its allreduce's peers each call
// f.f at once), and one shared set serialised them: 2 / 4 threads took exactly 2 / 4 x one combine
// (profiles/r04_host_pair_threads_shared.jsonl). So a call leases a set from a per-process pool for its own
// duration and hands it back when it returns (no per-thread state: the reference spawns threads per collective).
// Bounded: at most kMaxHostPipes sets per device exist; a caller past the cap waits until a set comes
// back (the PCIe link is saturated well before that many concurrent combines). A set's staging grows to the
// largest chunk it has served, rounded up to a power of two and capped at the host chunk (FMI_TUNE_HOST_CHUNK):
// small combines keep small staging. fmi_dev_finalize frees every set; it holds g_pipes_life exclusively, which
// every call holds shared for its whole duration, so no lease is outstanding then.
constexpr size_t kMaxHostPipes = 8;
struct HostPipe {
    int device = -1;
    void* stage[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};
    size_t stage_bytes = 0;
    hipStream_t pipe[2] = {nullptr, nullptr};
    void release() {
        for (int k = 0; k < 2; ++k) {
            if (pipe[k]) (void)hipStreamSynchronize(pipe[k]);
            for (int j = 0; j < 2; ++j)
                if (stage[k][j]) (void)hipFree(stage[k][j]);
            if (pipe[k]) (void)hipStreamDestroy(pipe[k]);
        }
        *this = HostPipe{};
    }
};
std::shared_mutex g_pipes_life;  // shared by every fmi_host_reduce_pair in flight, exclusive in init / finalize
struct PipeRegistry {
    std::mutex mu;
    std::condition_variable back;                // a set came back to the pool
    std::vector<std::unique_ptr<HostPipe>> all;  // every set (owning)
    std::vector<HostPipe*> idle;                 // sets no call holds; most recently returned last
};
// Never destroyed: a thread still running while the process exits may hand its set back after static
// destruction has begun.
PipeRegistry& pipes() {
    static PipeRegistry* r = new PipeRegistry;
    return *r;
}

// One call's set: leased on construction (waiting while the device's kMaxHostPipes sets are all in use), returned
// to the pool on destruction. No HIP call on return: the call synchronised the set's streams before returning.
struct PipeLease {
    HostPipe* p = nullptr;
    explicit PipeLease(int device) {
        PipeRegistry& reg = pipes();
        std::unique_lock<std::mutex> lk(reg.mu);
        for (;;) {
            for (size_t i = reg.idle.size(); i-- > 0;)
                if (reg.idle[i]->device == device) {
                    p = reg.idle[i];
                    reg.idle.erase(reg.idle.begin() + static_cast<std::ptrdiff_t>(i));
                    return;
                }
            size_t mine = 0;
            for (auto& q : reg.all) mine += q->device == device;
            if (mine < kMaxHostPipes) {
                reg.all.push_back(std::make_unique<HostPipe>());
                p = reg.all.back().get();
                p->device = device;
                return;
            }
            reg.back.wait(lk);
        }
    }
    ~PipeLease() {
        PipeRegistry& reg = pipes();
        {
            std::lock_guard<std::mutex> lk(reg.mu);
            reg.idle.push_back(p);
        }
        reg.back.notify_one();
    }
    PipeLease(const PipeLease&) = delete;
    PipeLease& operator=(const PipeLease&) = delete;
};

size_t host_pipe_count(size_t* idle, size_t* staging_bytes) {
    std::lock_guard<std::mutex> lk(pipes().mu);
    if (idle) *idle = pipes().idle.size();
    if (staging_bytes) {
        *staging_bytes = 0;
        for (auto& p : pipes().all) *staging_bytes += 4 * p->stage_bytes;
    }
    return pipes().all.size();
}

// Defaults from tools/tune_pair.py on MI355X (C2, 256 MiB f32): nontemporal one-shot tiles, 4 × 16 B per
// operand per thread, 256-thread workgroups — 125 µs = 6.4 TB/s vs 142 µs for plain loads/stores.
std::atomic<long long> g_tune[16] = {2 /*variant: nontemporal tiles*/, 4 /*unroll*/, 256 /*block*/,
                                     8 /*grid per CU*/, 64ll << 20 /*host chunk*/, 1 /*host zero-copy*/,
                                     64 /*fused in-flight KiB per CU (tools/ab_fused_cap.py)*/,
                                     1 /*one-pass blocked scan*/, 0 /*ncclAllToAll*/, 0 /*ncclAllGather*/,
                                     0 /*no allreduce pipelining*/, 1 /*fused kernels: buffer ops where measured faster*/,
                                     1 /*pairwise: tiles t % 8 < 1 (one XCD) store sc1 (tools/ab_pair_sc1.py)*/,
                                     0 /*one-rank communicators copy*/,
                                     0 /*plain allocations; groups take slots (profiles/r06a_placement_ab.jsonl)*/,
                                     1 /*shard kernel inputs in their own 4 KiB slots (profiles/r06a_shard_layout.jsonl)*/};

int hip_fail(const char* what, hipError_t e) {
    return fail(FMI_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define FMI_HIP_TRY(call)                                   \
    do {                                                    \
        const hipError_t fmi_e_ = (call);                   \
        if (fmi_e_ != hipSuccess) return hip_fail(#call, fmi_e_); \
    } while (0)

#define FMI_RC_TRY(call)                  \
    do {                                  \
        const int fmi_rc_ = (call);       \
        if (fmi_rc_ != FMI_OK) return fmi_rc_; \
    } while (0)

int require_device() {
    if (g_state.device < 0) return fail(FMI_ERR_NO_DEVICE, "fmi_dev_init has not been called");
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess || cur != g_state.device) FMI_HIP_TRY(hipSetDevice(g_state.device));
    return FMI_OK;
}

hipStream_t resolve(fmi_stream_t s) { return s ? static_cast<hipStream_t>(s) : g_state.stream; }

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// Is `p` page-locked host memory the device can address? Returns its device-side address.
bool host_mapped_at(void* p, void** dev) {
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable memory reports an error: clear it
        return false;
    }
    if (attr.type != hipMemoryTypeHost || attr.devicePointer == nullptr) return false;
    *dev = attr.devicePointer;
    return true;
}

// Is all of [p, p + bytes) page-locked and device-mapped as one contiguous range (first and last byte
// mapped, at device addresses bytes - 1 apart)? A bucket that only starts inside a pinned or registered
// range must not be read zero-copy past its end.
bool host_mapped(void* p, size_t bytes, void** dev) {
    void* first = nullptr;
    void* last = nullptr;
    if (!host_mapped_at(p, &first)) return false;
    if (!host_mapped_at(static_cast<char*>(p) + bytes - 1, &last)) return false;
    if (static_cast<char*>(last) - static_cast<char*>(first) != static_cast<std::ptrdiff_t>(bytes - 1)) return false;
    *dev = first;
    return true;
}

// ----------------------------------------------------------------------------------------------------
// Pairwise launch policy.
// ----------------------------------------------------------------------------------------------------
template <class Op, class T, int NT>
int launch_pair_vec(T* out, const T* a, const T* b, size_t n, hipStream_t s) {
    const long long variant = g_tune[FMI_TUNE_PAIR_VARIANT].load();
    const long long unroll = g_tune[FMI_TUNE_PAIR_UNROLL].load();
    const unsigned block = static_cast<unsigned>(g_tune[FMI_TUNE_BLOCK].load());
    const size_t nvec = n / kVecLanes<T>;
    const size_t per_block = static_cast<size_t>(block) * static_cast<size_t>(unroll);
    const size_t ntiles = std::max<size_t>(1, (nvec + per_block - 1) / per_block);
    const unsigned sc1_k = static_cast<unsigned>(g_tune[FMI_TUNE_PAIR_SC1_OF_8].load());  // one-shot tiles t % 8 < k: sc1
    // One-shot tiles unless the grid would pass HIP's 2^32-thread limit (buckets of > 2^31 tiles' worth):
    // then the grid-stride form walks the tiles.
    constexpr size_t kMaxGridThreads = size_t(1) << 31;
    if (variant == 1 || ntiles * block > kMaxGridThreads) {
        const size_t cap = static_cast<size_t>(g_state.num_cus) * static_cast<size_t>(g_tune[FMI_TUNE_GRID_PER_CU].load());
        const unsigned grid = static_cast<unsigned>(std::max<size_t>(1, std::min(ntiles, cap)));
        switch (unroll) {
            case 1: pair_stride<Op, T, 1, NT><<<grid, block, 0, s>>>(out, a, b, n); break;
            case 2: pair_stride<Op, T, 2, NT><<<grid, block, 0, s>>>(out, a, b, n); break;
            case 4: pair_stride<Op, T, 4, NT><<<grid, block, 0, s>>>(out, a, b, n); break;
            case 8: pair_stride<Op, T, 8, NT><<<grid, block, 0, s>>>(out, a, b, n); break;
            default: return fail(FMI_ERR_INVALID, "unroll must be 1, 2, 4 or 8");
        }
    } else {
        const unsigned grid = static_cast<unsigned>(ntiles);
        switch (unroll) {
            case 1: pair_tile<Op, T, 1, NT><<<grid, block, 0, s>>>(out, a, b, n, sc1_k); break;
            case 2: pair_tile<Op, T, 2, NT><<<grid, block, 0, s>>>(out, a, b, n, sc1_k); break;
            case 4: pair_tile<Op, T, 4, NT><<<grid, block, 0, s>>>(out, a, b, n, sc1_k); break;
            case 8: pair_tile<Op, T, 8, NT><<<grid, block, 0, s>>>(out, a, b, n, sc1_k); break;
            default: return fail(FMI_ERR_INVALID, "unroll must be 1, 2, 4 or 8");
        }
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail("pairwise kernel launch", e);
    return FMI_OK;
}

int launch_combine(int op, int dtype, void* out, const void* a, const void* b, size_t n, hipStream_t s) {
    if (n == 0) return FMI_OK;
    if (!out || !a || !b) return fail(FMI_ERR_INVALID, "null buffer");
    return with_op_dtype(op, dtype, [&]<class Op, class T>() -> int {
        T* o = static_cast<T*>(out);
        const T* x = static_cast<const T*>(a);
        const T* y = static_cast<const T*>(b);
        if (aligned16(o) && aligned16(x) && aligned16(y)) {
            // The cache-policy variants are instantiated for the core dtypes only (tools/tune_pair.py
            // sweeps them); the other integer widths always take the default policy.
            if constexpr (!(std::is_same_v<T, float> || std::is_same_v<T, double> || std::is_same_v<T, int32_t> ||
                            std::is_same_v<T, int64_t>)) {
                return launch_pair_vec<Op, T, 3>(o, x, y, n, s);
            } else {
                switch (g_tune[FMI_TUNE_PAIR_VARIANT].load()) {
                    case 2: return launch_pair_vec<Op, T, 3>(o, x, y, n, s);  // nt loads + nt stores
                    case 3: return launch_pair_vec<Op, T, 1>(o, x, y, n, s);  // nt loads only
                    case 4: return launch_pair_vec<Op, T, 2>(o, x, y, n, s);  // nt stores only
                    default: return launch_pair_vec<Op, T, 0>(o, x, y, n, s);
                }
            }
        }
        const unsigned grid = static_cast<unsigned>(std::min<size_t>(grid_for(n, 256), 65536));
        pair_scalar<Op, T><<<grid, 256, 0, s>>>(o, x, y, n);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return hip_fail("pairwise scalar kernel launch", e);
        return FMI_OK;
    });
}

// ----------------------------------------------------------------------------------------------------
// Scratch arena for P-way temporaries (caller holds g_mu). Stream s waits until the previous user's work
// has drained; the caller records g_state.arena_free on s after its last launch touching the arena.
// ----------------------------------------------------------------------------------------------------
int arena_acquire(size_t need, hipStream_t s) {
    // The arena is ordered by an event recorded outside any graph: a captured call would record arena_free
    // inside the graph, and its replays would write the arena unordered against later direct calls.
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    FMI_HIP_TRY(hipStreamIsCapturing(s, &cap));
    if (cap != hipStreamCaptureStatusNone)
        return fail(FMI_ERR_UNSUPPORTED, "this call needs the library's scratch arena (unaligned or 8/16-bit buckets, "
                                         "or a P-way program beyond the fused kernels) and cannot be captured in a graph");
    if (!g_state.arena_free) FMI_HIP_TRY(hipEventCreateWithFlags(&g_state.arena_free, hipEventDisableTiming));
    if (g_state.arena_bytes < need) {
        FMI_HIP_TRY(hipEventSynchronize(g_state.arena_free));  // previous users have drained
        if (g_state.arena) FMI_HIP_TRY(hipFree(g_state.arena));
        g_state.arena = nullptr;
        g_state.arena_bytes = 0;
        const hipError_t e = hipMalloc(&g_state.arena, need);
        if (e != hipSuccess) return fail(FMI_ERR_ALLOC, std::string("hipMalloc (P-way scratch): ") + hipGetErrorString(e));
        g_state.arena_bytes = need;
    }
    FMI_HIP_TRY(hipStreamWaitEvent(s, g_state.arena_free, 0));
    return FMI_OK;
}

size_t arena_stride(size_t n, size_t esz) { return (std::max<size_t>(n * esz, 16) + 255) / 256 * 256; }

// ----------------------------------------------------------------------------------------------------
// P-way programs for unaligned buckets, the byte/16-bit dtypes and the scans beyond 16 peers: the same
// schedule, one pairwise pass per step. Only the steps the requested outputs depend on run (an allreduce
// for one rank needs P - 1 of its P log P steps). Temp buckets live in the arena; slots are assigned on
// the host (a value's slot is recycled right after its last use) so the arena holds only the peak number
// of live temps.
// ----------------------------------------------------------------------------------------------------
int run_program_stepwise(int op, int dtype, const sched::HostProgram& prog, void* const* outs, int nouts,
                         const int* out_value, const void* const* ins, size_t n, hipStream_t s) {
    const size_t esz = dtype_size(dtype);
    const int P = prog.peers;
    const int nv = prog.nvalues();
    std::vector<char> live(nv, 0);
    for (int k = 0; k < nouts; ++k) live[out_value[k]] = 1;
    for (int st = prog.nsteps - 1; st >= 0; --st)
        if (live[P + st]) live[prog.step[st].a] = live[prog.step[st].b] = 1;
    std::vector<int> last_use(nv, -1);
    for (int st = 0; st < prog.nsteps; ++st) {
        if (!live[P + st]) continue;
        last_use[prog.step[st].a] = st;
        last_use[prog.step[st].b] = st;
    }
    for (int k = 0; k < nouts; ++k) last_use[out_value[k]] = prog.nsteps;  // outputs live to the end
    // host-side slot assignment
    std::vector<int> slot(nv, -1), free_slots;
    int nslots = 0;
    for (int st = 0; st < prog.nsteps; ++st) {
        if (!live[P + st]) continue;
        int d;
        if (!free_slots.empty()) {
            d = free_slots.back();
            free_slots.pop_back();
        } else {
            d = nslots++;
        }
        slot[P + st] = d;
        const int a = prog.step[st].a, b = prog.step[st].b;
        if (a >= P && last_use[a] == st) free_slots.push_back(slot[a]);
        if (b >= P && b != a && last_use[b] == st) free_slots.push_back(slot[b]);
    }
    const size_t stride = arena_stride(n, esz);
    std::lock_guard<std::mutex> lk(g_mu);
    FMI_RC_TRY(arena_acquire(stride * static_cast<size_t>(nslots), s));
    auto addr = [&](int v) -> const void* {
        return v < P ? ins[v] : static_cast<const char*>(g_state.arena) + stride * static_cast<size_t>(slot[v]);
    };
    int rc = FMI_OK;
    for (int st = 0; st < prog.nsteps && rc == FMI_OK; ++st)
        if (live[P + st])
            rc = launch_combine(op, dtype, const_cast<void*>(addr(P + st)), addr(prog.step[st].a), addr(prog.step[st].b), n, s);
    for (int k = 0; k < nouts && rc == FMI_OK; ++k) {
        const void* src = addr(out_value[k]);
        if (src != outs[k] && n > 0) {
            rc = device_copy(outs[k], src, n * esz, s);
        }
    }
    FMI_HIP_TRY(hipEventRecord(g_state.arena_free, s));
    return rc;
}

// ----------------------------------------------------------------------------------------------------
// Tree algorithms beyond the fused kernels as fused sub-programs. Each program splits along blocks of 16
// consecutive (transformed) peers, and every piece is exactly one of the fused kernels' own programs
// (fmi_schedule.h), so the bracketing is the reference's:
//   reduce_ltr  ((x0 + .. + x15) + x16 + .. + x30) + ..: a fused 16-peer fold, then fused folds of the
//               running value and the next 15 peers.
//   reduce      binomial rounds 0..3 stay inside blocks of 16 (the block's own reduce program); rounds 4..
//               combine the block values at spans 16, 32, .. = the reduce program over ceil(P/16) values.
//   allreduce   (P > 31; up to 31 it is one fused kernel) after the pre-fold of peers >= 2^k into
//               peer - 2^k, recursive-doubling rounds 0..3 stay inside blocks of 16 and leave position p
//               holding the block's 16-peer allreduce for rank p % 16; rounds 4.. pair positions with
//               equal p % 16 = the allreduce program over the 2^k / 16 block values, for rank p / 16. A
//               block pre-folds its partners inside its own kernel (16 + m inputs, or 32 for m = 16).
// Every input is read once; temps cost one write + one read per block value (P = 64: 73 bucket passes
// instead of 189 for pairwise steps). A dry run only counts the temps.
// ----------------------------------------------------------------------------------------------------
struct TreeTemps {
    bool dry = true;  // dry run: count the temps, launch nothing
    char* base = nullptr;
    size_t stride = 0;
    int used = 0;
    void* next() { return dry ? (++used, nullptr) : base + stride * static_cast<size_t>(used++); }
};

int tree_blocked(int op, int dtype, int alg, void* out, const void* const* ins, int P, int rank, size_t n,
                 hipStream_t s, TreeTemps& t) {
    const bool dry = t.dry;
    constexpr int B16 = sched::kMaxFusedPeers;
    if (P == 1) {
        if (!dry && out != ins[0]) FMI_RC_TRY(device_copy(out, ins[0], n * dtype_size(dtype), s));
        return FMI_OK;
    }
    if (P <= sched::max_fused_peers(alg)) {
        if (dry) return FMI_OK;
        PeerPtrs ptrs{};
        for (int p = 0; p < P; ++p) ptrs.in[p] = ins[p];
        ptrs.out[0] = out;
        switch (alg) {
            case FMI_ALG_ALLREDUCE: return launch_fused_allreduce(op, dtype, P, ptrs, n, rank, s);
            case FMI_ALG_REDUCE: return launch_fused_reduce(op, dtype, P, ptrs, n, s);
            default: return launch_fused_reduce_ltr(op, dtype, P, ptrs, n, s);
        }
    }
    switch (alg) {
        case FMI_ALG_REDUCE_LTR: {
            void* acc = t.next();
            FMI_RC_TRY(tree_blocked(op, dtype, alg, acc, ins, B16, 0, n, s, t));
            for (int p = B16; p < P; p += B16 - 1) {
                const int m = std::min(B16 - 1, P - p);
                if (dry) continue;
                PeerPtrs ptrs{};
                ptrs.in[0] = acc;
                for (int j = 0; j < m; ++j) ptrs.in[1 + j] = ins[p + j];
                ptrs.out[0] = p + m == P ? out : acc;  // elementwise: reading and writing acc in one pass is safe
                FMI_RC_TRY(launch_fused_reduce_ltr(op, dtype, 1 + m, ptrs, n, s));
            }
            return FMI_OK;
        }
        case FMI_ALG_REDUCE: {
            const int B = (P + B16 - 1) / B16;
            std::vector<const void*> vals(B);
            for (int b = 0; b < B; ++b) {
                const int m = std::min(B16, P - b * B16);
                if (m == 1) {
                    vals[b] = ins[b * B16];
                    continue;
                }
                void* v = t.next();
                FMI_RC_TRY(tree_blocked(op, dtype, alg, v, ins + b * B16, m, 0, n, s, t));
                vals[b] = v;
            }
            return tree_blocked(op, dtype, alg, out, vals.data(), B, 0, n, s, t);
        }
        default: {  // allreduce, P > 31
            const int pow2 = 1 << sched::floor_log2(P);
            const int folded = P - pow2;
            const int r = rank < pow2 ? rank : rank - pow2;  // folded peers get their partner's value back
            const int B = pow2 / B16;
            // A block of m < 16 pre-folded peers is the fused allreduce program of 16 + m peers (it pre-folds
            // them itself); a block whose 16 peers all take a pre-fold is the 32-input kAllreducePrefold16.
            std::vector<const void*> vals(B);
            for (int b = 0; b < B; ++b) {
                const int lo = b * B16;
                const int m = std::clamp(folded - lo, 0, B16);
                std::vector<const void*> y(ins + lo, ins + lo + B16);
                y.insert(y.end(), ins + pow2 + lo, ins + pow2 + lo + m);
                void* v = t.next();
                if (m == B16) {
                    if (!dry) {
                        PeerPtrs ptrs{};
                        for (int j = 0; j < 2 * B16; ++j) ptrs.in[j] = y[j];
                        ptrs.out[0] = v;
                        FMI_RC_TRY(launch_fused_allreduce_prefold16(op, dtype, ptrs, n, r % B16, s));
                    }
                } else {
                    FMI_RC_TRY(tree_blocked(op, dtype, alg, v, y.data(), static_cast<int>(y.size()), r % B16, n, s, t));
                }
                vals[b] = v;
            }
            return tree_blocked(op, dtype, alg, out, vals.data(), B, r / B16, n, s, t);
        }
    }
}

// ----------------------------------------------------------------------------------------------------
// Beyond one one-pass kernel (its pointer table holds 128 peers): superblocks of 128 peers. The programs
// split at 128 exactly as they split at 16 (tree_blocked above), one level up:
//   reduce_ltr / scan_ltr: segments of 127 peers continued from the previous segment's running value (the
//     chain kernel with a carry-in): P + ceil((P - 128) / 127) bucket reads, instead of the blocked
//     launches' P + 2 ceil((P - 16) / 15).
//   reduce_no_order: binomial rounds 0..6 stay inside each superblock (the one-pass reduce over its <= 128
//     peers), rounds 7+ are the reduce program over the ceil(P / 128) superblock values.
// Every input is read once; the superblock values cost 2 ceil(P / 128) bucket passes. Measured over 1 GiB
// of input (tools/ab_superblocks.py): reduce P = 256 / 300 13 / 9 % faster than the block launches,
// reduce_ltr P = 256 25 %, scan_ltr P = 256 14 %. allreduce_no_order, P = 2^k, would split the same way
// (rounds 0..6 inside superblocks, each the one-pass 128-peer allreduce for rank r % 128; rounds 7+ over
// the superblock values for rank r / 128) but was 16-25 % SLOWER than the 16-peer block launches at
// P = 256 / 512 (128 streams per one-pass kernel against 16 per launch); allreduce splits at 64 instead
// (allreduce_superblocks below).
// ----------------------------------------------------------------------------------------------------
constexpr int kSuperPeers = kMaxOnePassScanBlocks * sched::kScanBlock;  // 128

// scan (outs[0..P)) or reduce (out) left to right over P > 128 peers. For reduce, `out` carries the running
// value between segments, so it must not be one of the inputs a later segment reads (checked by the caller).
int chain_superblocks(int op, int dtype, bool scan, void* const* outs, void* out, const void* const* ins, int P,
                      size_t n, hipStream_t s) {
    for (int k = 0; k < P;) {
        BlockedScanPtrs ptrs{};
        const bool carry = k > 0;
        const int first = carry ? 1 : 0;
        const int m = std::min(kSuperPeers - first, P - k);
        if (carry) ptrs.in[0] = scan ? outs[k - 1] : out;
        for (int j = 0; j < m; ++j) {
            ptrs.in[first + j] = ins[k + j];
            if (scan) ptrs.out[first + j] = outs[k + j];
        }
        if (!scan) ptrs.out[0] = out;
        FMI_RC_TRY(launch_chain_one_pass(op, dtype, scan, m + first, ptrs, n, s, carry));
        k += m;
    }
    return FMI_OK;
}

// reduce_no_order over up to 128 values (transformed ids, root 0): fused up to 16 peers, one pass beyond.
int reduce_level(int op, int dtype, void* out, const void* const* vals, int P, size_t n, hipStream_t s) {
    if (P == 1) {
        if (out != vals[0]) FMI_RC_TRY(device_copy(out, vals[0], n * dtype_size(dtype), s));
        return FMI_OK;
    }
    if (P <= sched::kMaxFusedPeers) {
        PeerPtrs ptrs{};
        for (int p = 0; p < P; ++p) ptrs.in[p] = vals[p];
        ptrs.out[0] = out;
        return launch_fused_reduce(op, dtype, P, ptrs, n, s);
    }
    BlockedScanPtrs ptrs{};
    for (int p = 0; p < P; ++p) ptrs.in[p] = vals[p];
    ptrs.out[0] = out;
    return launch_tree_blocks_one_pass(op, dtype, FMI_ALG_REDUCE, P, ptrs, n, 0, s);
}

bool tree_superblocks_cover(int op, int dtype, int alg, int P) {
    if (alg != FMI_ALG_REDUCE || P <= kSuperPeers || P > kSuperPeers * kSuperPeers) return false;
    const int S = (P + kSuperPeers - 1) / kSuperPeers;
    const int last = P - (S - 1) * kSuperPeers;
    return tree_blocks_one_pass_covers(op, dtype, alg, kSuperPeers) &&
           (last <= sched::kMaxFusedPeers || tree_blocks_one_pass_covers(op, dtype, alg, last)) &&
           (S <= sched::kMaxFusedPeers || tree_blocks_one_pass_covers(op, dtype, alg, S));
}

// reduce_no_order over P > 128 peers (transformed ids, root 0) as superblocks of 128.
int reduce_superblocks(int op, int dtype, void* out, const void* const* ins, int P, size_t n, hipStream_t s) {
    const int S = (P + kSuperPeers - 1) / kSuperPeers;
    std::lock_guard<std::mutex> lk(g_mu);
    const size_t stride = arena_stride(n, dtype_size(dtype));
    FMI_RC_TRY(arena_acquire(stride * static_cast<size_t>(S), s));
    char* base = static_cast<char*>(g_state.arena);
    std::vector<const void*> vals(S);
    int rc = FMI_OK;
    for (int b = 0; b < S && rc == FMI_OK; ++b) {
        const int lo = b * kSuperPeers;
        const int m = std::min(kSuperPeers, P - lo);
        if (m == 1) {  // a lone last peer is its own superblock value
            vals[b] = ins[lo];
            continue;
        }
        void* v = base + stride * static_cast<size_t>(b);
        rc = reduce_level(op, dtype, v, ins + lo, m, n, s);
        vals[b] = v;
    }
    if (rc == FMI_OK) rc = reduce_level(op, dtype, out, vals.data(), S, n, s);
    FMI_HIP_TRY(hipEventRecord(g_state.arena_free, s));
    return rc;
}

// allreduce_no_order over P = 2^k >= 128 peers as superblocks of 64 peers (profiles/archive/r02_ab_allreduce_superblocks64.jsonl, 1 GiB of
// input: P = 256 / 512 / 1024 19 / 24 / 4 % faster than the 16-peer block launches; P = 128 28-31 % faster
// than its one-pass 128-peer kernel, profiles/archive/r02_ab_allreduce128.jsonl; superblocks of 128 were slower than the
// launches, above): recursive-doubling rounds 0..5 stay inside each superblock — its
// one-pass 64-peer allreduce for rank r % 64, the same for every superblock — and rounds 6+ are the
// allreduce over the P / 64 superblock values for rank r / 64 (fused up to 16 values, one pass beyond).
constexpr int kAllreduceSuper = 64;

bool allreduce_superblocks_cover(int op, int dtype, int P) {
    const int S = P / kAllreduceSuper;
    return P >= kSuperPeers && (P & (P - 1)) == 0 && S <= kSuperPeers &&
           tree_blocks_one_pass_covers(op, dtype, FMI_ALG_ALLREDUCE, kAllreduceSuper) &&
           (S <= sched::kMaxFusedPeers || tree_blocks_one_pass_covers(op, dtype, FMI_ALG_ALLREDUCE, S));
}

int allreduce_superblocks(int op, int dtype, void* out, const void* const* ins, int P, int rank, size_t n,
                          hipStream_t s) {
    const int S = P / kAllreduceSuper;
    std::lock_guard<std::mutex> lk(g_mu);
    const size_t stride = arena_stride(n, dtype_size(dtype));
    FMI_RC_TRY(arena_acquire(stride * static_cast<size_t>(S), s));
    char* base = static_cast<char*>(g_state.arena);
    std::vector<const void*> vals(S);
    int rc = FMI_OK;
    for (int b = 0; b < S && rc == FMI_OK; ++b) {
        BlockedScanPtrs ptrs{};
        for (int p = 0; p < kAllreduceSuper; ++p) ptrs.in[p] = ins[b * kAllreduceSuper + p];
        void* v = base + stride * static_cast<size_t>(b);
        ptrs.out[0] = v;
        rc = launch_tree_blocks_one_pass(op, dtype, FMI_ALG_ALLREDUCE, kAllreduceSuper, ptrs, n, rank % kAllreduceSuper, s);
        vals[b] = v;
    }
    if (rc == FMI_OK) {
        if (S <= sched::kMaxFusedPeers) {
            PeerPtrs ptrs{};
            for (int b = 0; b < S; ++b) ptrs.in[b] = vals[b];
            ptrs.out[0] = out;
            rc = launch_fused_allreduce(op, dtype, S, ptrs, n, rank / kAllreduceSuper, s);
        } else {
            BlockedScanPtrs ptrs{};
            for (int b = 0; b < S; ++b) ptrs.in[b] = vals[b];
            ptrs.out[0] = out;
            rc = launch_tree_blocks_one_pass(op, dtype, FMI_ALG_ALLREDUCE, S, ptrs, n, rank / kAllreduceSuper, s);
        }
    }
    FMI_HIP_TRY(hipEventRecord(g_state.arena_free, s));
    return rc;
}

int run_tree_blocked(int op, int dtype, int alg, void* out, const void* const* ins, int P, int rank, size_t n,
                     hipStream_t s) {
    if (g_tune[FMI_TUNE_BLOCKS_ONE_PASS].load() != 0 && P >= kSuperPeers) {
        if (alg == FMI_ALG_REDUCE_LTR && std::find(ins + kSuperPeers, ins + P, static_cast<const void*>(out)) == ins + P)
            return chain_superblocks(op, dtype, false, nullptr, out, ins, P, n, s);
        if (tree_superblocks_cover(op, dtype, alg, P)) return reduce_superblocks(op, dtype, out, ins, P, n, s);
        if (alg == FMI_ALG_ALLREDUCE && allreduce_superblocks_cover(op, dtype, P))
            return allreduce_superblocks(op, dtype, out, ins, P, rank, n, s);
    }
    if (g_tune[FMI_TUNE_BLOCKS_ONE_PASS].load() != 0 && alg == FMI_ALG_REDUCE_LTR && P <= kMaxOnePassScanBlocks * 16) {
        BlockedScanPtrs ptrs{};
        for (int p = 0; p < P; ++p) ptrs.in[p] = ins[p];
        ptrs.out[0] = out;
        return launch_chain_one_pass(op, dtype, false, P, ptrs, n, s);
    }
    if (g_tune[FMI_TUNE_BLOCKS_ONE_PASS].load() != 0 && prefold_blocks_one_pass_covers(alg, P)) {
        const int pow2 = 1 << sched::floor_log2(P);
        const int r = rank < pow2 ? rank : rank - pow2;  // folded peers get their partner's value back
        const int lo = r & 15;
        BlockedScanPtrs ptrs{};
        for (int p = 0; p < pow2; ++p) ptrs.in[p] = ins[(p & ~15) | ((p & 15) ^ lo)];
        for (int p = 0; p < P - pow2; ++p) ptrs.in[pow2 + p] = ins[pow2 + ((p & ~15) | ((p & 15) ^ lo))];
        ptrs.out[0] = out;
        return launch_prefold_blocks_one_pass(op, dtype, P, ptrs, n, r >> 4, s);
    }
    if (g_tune[FMI_TUNE_BLOCKS_ONE_PASS].load() != 0 && tree_blocks_one_pass_covers(op, dtype, alg, P)) {
        BlockedScanPtrs ptrs{};
        for (int p = 0; p < P; ++p) ptrs.in[p] = ins[p];
        ptrs.out[0] = out;
        return launch_tree_blocks_one_pass(op, dtype, alg, P, ptrs, n, alg == FMI_ALG_ALLREDUCE ? rank : 0, s);
    }
    TreeTemps count;
    FMI_RC_TRY(tree_blocked(op, dtype, alg, out, ins, P, rank, n, s, count));
    std::lock_guard<std::mutex> lk(g_mu);
    TreeTemps t;
    t.dry = false;
    t.stride = arena_stride(n, dtype_size(dtype));
    FMI_RC_TRY(arena_acquire(t.stride * static_cast<size_t>(count.used), s));
    t.base = static_cast<char*>(g_state.arena);
    const int rc = tree_blocked(op, dtype, alg, out, ins, P, rank, n, s, t);
    FMI_HIP_TRY(hipEventRecord(g_state.arena_free, s));
    return rc;
}

// ----------------------------------------------------------------------------------------------------
// Scans beyond 16 peers. scan_no_order splits along blocks of 16 (kScanCarry's derivation in
// fmi_schedule.h):
//   1. block 0 as the fused 16-peer scan (its last output is T_0), and every later full block's up-sweep
//      total T_b, which is the binomial reduce over the block in reverse order;
//   2. the block-level prefixes S_b = scan_no_order over the T_b, written straight into the output of
//      peer 16b + 15 (S_0 = T_0);
//   3. every later block as the carry program from S_{b-1}.
// scan_ltr: block 0 fused, then 15 peers at a time continued from the previous peer's prefix. No input is
// read more than twice (P = 64: 184 bucket passes, one pass would be 128, pairwise steps about 490).
// ----------------------------------------------------------------------------------------------------
int scan_blocked(int op, int dtype, int alg, void* const* outs, const void* const* ins, int P, size_t n,
                 hipStream_t s, TreeTemps& t) {
    constexpr int BL = sched::kScanBlock;
    const bool dry = t.dry;
    if (P == 1) {
        if (!dry && outs[0] != ins[0]) FMI_RC_TRY(device_copy(outs[0], ins[0], n * dtype_size(dtype), s));
        return FMI_OK;
    }
    if (P <= sched::max_fused_peers(alg)) {
        if (dry) return FMI_OK;
        PeerPtrs ptrs{};
        for (int p = 0; p < P; ++p) {
            ptrs.in[p] = ins[p];
            ptrs.out[p] = outs[p];
        }
        return alg == FMI_ALG_SCAN ? launch_fused_scan(op, dtype, P, ptrs, n, s) : launch_fused_scan_ltr(op, dtype, P, ptrs, n, s);
    }
    auto carry_block = [&](int lo, int m, const void* carry) -> int {
        if (dry) return FMI_OK;
        PeerPtrs ptrs{};
        ptrs.in[0] = carry;
        for (int j = 0; j < m; ++j) {
            ptrs.in[1 + j] = ins[lo + j];
            ptrs.out[1 + j] = outs[lo + j];
        }
        return alg == FMI_ALG_SCAN ? launch_fused_scan_carry(op, dtype, m + 1, ptrs, n, s)
                                   : launch_fused_scan_ltr_carry(op, dtype, m + 1, ptrs, n, s);
    };
    if (alg == FMI_ALG_SCAN_LTR) {
        FMI_RC_TRY(scan_blocked(op, dtype, alg, outs, ins, BL, n, s, t));
        for (int p = BL; p < P; p += BL - 1) FMI_RC_TRY(carry_block(p, std::min(BL - 1, P - p), outs[p - 1]));
        return FMI_OK;
    }
    // Block 0 first: the fused 16-peer scan, whose q = 15 output is T_0 = S_0. It reads its inputs before
    // the block-level scan writes any output (outs may alias ins).
    FMI_RC_TRY(scan_blocked(op, dtype, alg, outs, ins, BL, n, s, t));
    const int B = P / BL;  // full blocks; a partial last block takes no part in the block-level rounds
    if (B >= 2) {
        std::vector<const void*> totals(B);
        std::vector<void*> prefix(B);
        totals[0] = prefix[0] = outs[BL - 1];  // rewritten in place with the same bits
        for (int b = 1; b < B; ++b) {
            void* tb = t.next();
            totals[b] = tb;
            prefix[b] = outs[b * BL + BL - 1];
            if (dry) continue;
            PeerPtrs r{};
            for (int j = 0; j < BL; ++j) r.in[j] = ins[b * BL + BL - 1 - j];
            r.out[0] = tb;
            FMI_RC_TRY(launch_fused_reduce(op, dtype, BL, r, n, s));
        }
        FMI_RC_TRY(scan_blocked(op, dtype, FMI_ALG_SCAN, prefix.data(), totals.data(), B, n, s, t));
    }
    for (int b = 1; b * BL < P; ++b) FMI_RC_TRY(carry_block(b * BL, std::min(BL - 1, P - b * BL), outs[b * BL - 1]));
    return FMI_OK;
}

int run_scan_blocked(int op, int dtype, int alg, void* const* outs, const void* const* ins, int P, size_t n,
                     hipStream_t s) {
    constexpr int BL = sched::kScanBlock;
    const int B = P / BL, r = P % BL;
    if (alg == FMI_ALG_SCAN_LTR && P > kSuperPeers && g_tune[FMI_TUNE_BLOCKS_ONE_PASS].load() != 0)
        return chain_superblocks(op, dtype, true, outs, nullptr, ins, P, n, s);
    if (alg == FMI_ALG_SCAN_LTR && P <= kMaxOnePassScanBlocks * BL && g_tune[FMI_TUNE_BLOCKS_ONE_PASS].load() != 0) {
        BlockedScanPtrs ptrs{};
        for (int p = 0; p < P; ++p) {
            ptrs.in[p] = ins[p];
            ptrs.out[p] = outs[p];
        }
        return launch_chain_one_pass(op, dtype, true, P, ptrs, n, s);
    }
    if (alg == FMI_ALG_SCAN && B >= 2 && B <= kMaxOnePassScanBlocks && g_tune[FMI_TUNE_BLOCKS_ONE_PASS].load() != 0) {
        // every full block in one pass (fmi_fused_scan_blocked.hip), then a ragged block as scan_blocked's
        // carry program from S_{B-1} = outs[16 B - 1]
        BlockedScanPtrs ptrs{};
        for (int p = 0; p < B * BL; ++p) {
            ptrs.in[p] = ins[p];
            ptrs.out[p] = outs[p];
        }
        FMI_RC_TRY(launch_scan_blocks_one_pass(op, dtype, B, ptrs, n, s));
        if (r == 0) return FMI_OK;
        PeerPtrs c{};
        c.in[0] = outs[B * BL - 1];
        for (int j = 0; j < r; ++j) {
            c.in[1 + j] = ins[B * BL + j];
            c.out[1 + j] = outs[B * BL + j];
        }
        return launch_fused_scan_carry(op, dtype, r + 1, c, n, s);
    }
    TreeTemps count;
    FMI_RC_TRY(scan_blocked(op, dtype, alg, outs, ins, P, n, s, count));
    std::lock_guard<std::mutex> lk(g_mu);
    TreeTemps t;
    t.dry = false;
    t.stride = arena_stride(n, dtype_size(dtype));
    FMI_RC_TRY(arena_acquire(t.stride * static_cast<size_t>(count.used), s));
    t.base = static_cast<char*>(g_state.arena);
    const int rc = scan_blocked(op, dtype, alg, outs, ins, P, n, s, t);
    FMI_HIP_TRY(hipEventRecord(g_state.arena_free, s));
    return rc;
}

int check_peer_args(int op, int dtype, int P) {
    if (op < FMI_OP_SUM || op > FMI_OP_MIN) return fail(FMI_ERR_INVALID, "unknown op " + std::to_string(op));
    if (dtype_size(dtype) == 0) return fail(FMI_ERR_INVALID, "unknown dtype " + std::to_string(dtype));
    if (P < 1 || P > sched::kMaxPeers)
        return fail(FMI_ERR_INVALID, "P must be in [1, " + std::to_string(sched::kMaxPeers) + "], got " + std::to_string(P));
    return FMI_OK;
}

// Symbolic evaluation of a program, for fmi_schedule_expr.
// Iterative (an LTR chain over P peers nests P deep): a stack of pending tokens, written left to right.
std::string expr_of(const sched::HostProgram& prog, int v) {
    std::string e;
    std::vector<int> todo{v};  // >= 0: a value id to expand; -1: "+"; -2: ")"
    while (!todo.empty()) {
        const int t = todo.back();
        todo.pop_back();
        if (t == -1) {
            e += '+';
        } else if (t == -2) {
            e += ')';
        } else if (t < prog.peers) {
            e += 'x';
            e += std::to_string(t);
        } else {
            const auto& st = prog.step[t - prog.peers];
            e += '(';
            todo.insert(todo.end(), {-2, st.b, -1, st.a});
        }
    }
    return e;
}

}  // namespace

int reduce_partials(int op, int dtype, void* const* outs, const void* const* ins, int P, size_t n, hipStream_t s) {
    if (n == 0) return FMI_OK;
    bool aligned = true;
    for (int p = 0; p < P; ++p) aligned = aligned && aligned16(ins[p]) && aligned16(outs[p]);
    if (P >= 2 && P <= sched::kMaxFusedPeers && aligned && is_core_dtype(dtype)) {
        PeerPtrs ptrs{};
        for (int p = 0; p < P; ++p) {
            ptrs.in[p] = ins[p];
            ptrs.out[p] = outs[p];
        }
        return launch_fused_reduce_partials(op, dtype, P, ptrs, n, s);
    }
    const sched::HostProgram prog = sched::build_host(sched::kReducePartials, P);
    if (!prog.ok) return fail(FMI_ERR_INVALID, "schedule construction failed");
    std::vector<int> values(prog.out.begin(), prog.out.end());
    return run_program_stepwise(op, dtype, prog, outs, P, values.data(), ins, n, s);
}

int fail(int code, const std::string& msg) {
    t_last_error = msg;
    return code;
}

hipStream_t library_stream() { return g_state.stream; }

// A device allocation (this process's, or another's mapped over IPC): what copy_tile may touch. Host and
// unknown pointers answer false, and the failed query is cleared from the runtime's last-error slot (the
// launch checks below read it).
static bool device_memory(const void* p) {
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeDevice;
}

int device_copy(void* dst, const void* src, size_t bytes, hipStream_t s) {
    if (bytes == 0 || dst == src) return FMI_OK;
    const char* d = static_cast<const char*>(dst);
    const char* c = static_cast<const char*>(src);
    const bool disjoint = d + bytes <= c || c + bytes <= d;
    if (bytes >= kDeviceCopyMin && disjoint && aligned16(dst) && aligned16(src) && device_memory(dst) &&
        device_memory(src)) {
        // One 16-B vector per thread: 3.2 % faster than four at 256 MiB and 2 % at 64 MiB, interleaved on the same
        // buffers with no MALL re-use (profiles/r04_copy_unroll.jsonl); four per thread only where one would
        // pass HIP's 2^31-thread grid (copies beyond 32 GiB).
        const size_t nvec = bytes / 16;
        if (nvec <= (size_t(1) << 31)) {
            const size_t tiles = (nvec + 255) / 256;
            copy_tile<1><<<static_cast<unsigned>(std::max<size_t>(1, tiles)), 256, 0, s>>>(static_cast<char*>(dst), c, bytes);
        } else {
            const size_t tiles = (nvec + 4 * 256 - 1) / (4 * 256);
            copy_tile<4><<<static_cast<unsigned>(tiles), 256, 0, s>>>(static_cast<char*>(dst), c, bytes);
        }
        FMI_HIP_TRY(hipGetLastError());
        return FMI_OK;
    }
    FMI_HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s));
    return FMI_OK;
}

// The fused kernels' `pol` argument. Auto (1): buffer accesses where tools/ab_fused_policy.py measured them
// ahead with >= 1.5 GiB of rotating buckets (tree P >= 4: +1.6..3.2 %; scan P >= 8: +0.8..0.9 %), global
// accesses where they were not (tree P = 2: -0.7 %, scan P = 2 / 4: +0.3 / -2.4 %).
int fused_policy(bool scan, int P) {
    const long long v = g_tune[FMI_TUNE_FUSED_POLICY].load();
    if (v == 1) return (scan ? P >= 8 : P >= 4) ? 1 : 0;
    return v == 2 ? 1 : 0;
}

size_t fused_lds_bytes(int P, size_t wg_load_bytes_per_peer) {
    const long long budget = g_tune[FMI_TUNE_FUSED_INFLIGHT_KIB].load() << 10;
    if (budget <= 0 || P <= 0) return 0;
    const size_t per_wg = static_cast<size_t>(P) * wg_load_bytes_per_peer;
    // never below 2 workgroups per CU: one alone leaves too few loads in flight (P = 8: 12 % slower)
    const size_t cap = std::max<size_t>(2, (static_cast<size_t>(budget) + per_wg - 1) / per_wg);
    if (cap >= 32) return 0;  // beyond any register-limited occupancy: no reservation needed
    return std::min(g_state.lds_per_cu / cap, g_state.lds_per_wg) & ~size_t(255);
}

}  // namespace fmi::dev

using namespace fmi::dev;
namespace sched = fmi::sched;

extern "C" {

int fmi_abi_version(void) { return FMI_DEV_ABI_VERSION; }

const char* fmi_last_error(void) { return t_last_error.c_str(); }

int fmi_dev_count(int* count) {
    if (!count) return fail(FMI_ERR_INVALID, "count is null");
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *count = c;
    return FMI_OK;
}

int fmi_dev_init(int device) {
    std::lock_guard<std::mutex> lk(g_mu);
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0)
        return fail(FMI_ERR_NO_DEVICE, "no HIP device visible");
    if (device < 0 || device >= count)
        return fail(FMI_ERR_NO_DEVICE, "device " + std::to_string(device) + " out of range (" + std::to_string(count) + " visible)");
    hipDeviceProp_t prop;
    FMI_HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(FMI_ERR_NO_DEVICE, std::string("device arch ") + prop.gcnArchName + " is not gfx950 (MI355X)");
    if (g_state.device == device && g_state.stream) return FMI_OK;
    FMI_HIP_TRY(hipSetDevice(device));
    hipStream_t s = nullptr;
    FMI_HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::unique_lock<std::shared_mutex> life(g_pipes_life);  // fmi_host_reduce_pair reads g_state under it, shared
    g_state.device = device;
    g_state.num_cus = prop.multiProcessorCount;
    g_state.lds_per_cu = prop.maxSharedMemoryPerMultiProcessor;
    g_state.lds_per_wg = prop.sharedMemPerBlock;
    g_state.stream = s;
    return FMI_OK;
}

int fmi_dev_finalize(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_state.device < 0) return FMI_OK;
    (void)hipSetDevice(g_state.device);
    (void)hipDeviceSynchronize();
    // exclusive: no fmi_host_reduce_pair is in flight (each holds it shared throughout), and none starts until
    // g_state says there is no device
    std::unique_lock<std::shared_mutex> life(g_pipes_life);
    {
        std::lock_guard<std::mutex> lk(pipes().mu);
        for (auto& p : pipes().all) p->release();
        pipes().all.clear();
        pipes().idle.clear();
    }
    if (g_state.arena) (void)hipFree(g_state.arena);
    if (g_state.arena_free) (void)hipEventDestroy(g_state.arena_free);
    if (g_state.stream) (void)hipStreamDestroy(g_state.stream);
    g_state = DeviceState{};
    return FMI_OK;
}

int fmi_dev_sync(void) {
    if (int rc = require_device()) return rc;
    FMI_HIP_TRY(hipDeviceSynchronize());
    return FMI_OK;
}

int fmi_dev_describe(char* buf, size_t len) {
    if (!buf || len == 0) return fail(FMI_ERR_INVALID, "null buffer");
    if (int rc = require_device()) return rc;
    hipDeviceProp_t prop;
    FMI_HIP_TRY(hipGetDeviceProperties(&prop, g_state.device));
    std::string d = std::string(prop.name) + " " + prop.gcnArchName + " CUs=" + std::to_string(prop.multiProcessorCount) +
                    " HBM=" + std::to_string(prop.totalGlobalMem >> 20) + "MiB";
    size_t idle = 0, staging = 0;
    const size_t pipes = host_pipe_count(&idle, &staging);  // fmi_host_reduce_pair's pooled staging sets
    d += " host_pipelines=" + std::to_string(pipes) + " idle=" + std::to_string(idle) +
         " host_staging_bytes=" + std::to_string(staging) + " host_pipelines_max=" + std::to_string(kMaxHostPipes);
    std::snprintf(buf, len, "%s", d.c_str());
    return FMI_OK;
}

int fmi_dev_pci_bus_id(int device, char* buf, size_t len) {
    if (!buf || len == 0) return fail(FMI_ERR_INVALID, "null buffer");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count)
        return fail(FMI_ERR_NO_DEVICE, "no device " + std::to_string(device));
    char id[64] = {};
    FMI_HIP_TRY(hipDeviceGetPCIBusId(id, sizeof(id), device));
    std::snprintf(buf, len, "%s", id);
    return FMI_OK;
}

// ---- memory ----------------------------------------------------------------------------------------
int fmi_dev_alloc(void** ptr, size_t bytes) {
    if (!ptr) return fail(FMI_ERR_INVALID, "ptr is null");
    if (int rc = require_device()) return rc;
    const bool slotted = bytes >= kSlotMinBytes && bytes <= SIZE_MAX - kSlotSpan && g_tune[FMI_TUNE_ALLOC_SLOTS].load() != 0;
    void* base = nullptr;
    const hipError_t e = hipMalloc(&base, std::max<size_t>(bytes, 1) + (slotted ? kSlotSpan : 0));
    if (e != hipSuccess) {
        (void)hipGetLastError();  // not left for the next launch's error check to find
        return fail(FMI_ERR_ALLOC, "hipMalloc(" + std::to_string(bytes) + "): " + hipGetErrorString(e));
    }
    if (!slotted) {
        *ptr = base;
        return FMI_OK;
    }
    std::lock_guard<std::mutex> lk(g_slots_mu);
    char* p = static_cast<char*>(base) + (g_next_slot++ % kSlots) * kSlotBytes;
    g_slotted[p] = base;
    *ptr = p;
    return FMI_OK;
}

int fmi_dev_alloc_group(void** ptrs, int count, size_t bytes) {
    if (!ptrs || count < 0) return fail(FMI_ERR_INVALID, "bad group");
    for (int j = 0; j < count; ++j) ptrs[j] = nullptr;
    if (int rc = require_device()) return rc;
    if (count == 0) return FMI_OK;
    if (bytes < kSlotMinBytes) {  // small buckets: plain allocations, nothing to place
        for (int j = 0; j < count; ++j) {
            const hipError_t e = hipMalloc(&ptrs[j], std::max<size_t>(bytes, 1));
            if (e != hipSuccess) {
                (void)hipGetLastError();  // not left for the next launch's error check to find
                for (int i = 0; i < j; ++i) (void)hipFree(ptrs[i]);
                for (int i = 0; i < count; ++i) ptrs[i] = nullptr;
                return fail(FMI_ERR_ALLOC, "hipMalloc(" + std::to_string(bytes) + ") for group bucket " +
                                               std::to_string(j) + ": " + hipGetErrorString(e));
            }
        }
        return FMI_OK;
    }
    // One allocation for the whole group, bucket j at j x stride: each bucket in its own 4 KiB slot (stride = the
    // bucket rounded up to 64 KiB, plus 4 KiB), and the group's memory one range (see the placement note above).
    const size_t n = static_cast<size_t>(count);
    if (bytes > SIZE_MAX - 2 * kSlotSpan) return fail(FMI_ERR_INVALID, "group too large");
    const size_t stride = (bytes + kSlotSpan - 1) / kSlotSpan * kSlotSpan + kSlotBytes;
    size_t total = 0;  // the buckets, plus room to start the range on a 64 KiB boundary
    if (__builtin_mul_overflow(n - 1, stride, &total) || __builtin_add_overflow(total, bytes + kSlotSpan, &total))
        return fail(FMI_ERR_INVALID, "group too large");
    void* base = nullptr;
    const hipError_t e = hipMalloc(&base, total);
    if (e != hipSuccess) {
        (void)hipGetLastError();  // not left for the next launch's error check to find
        return fail(FMI_ERR_ALLOC, "hipMalloc(" + std::to_string(total) + ") for a group of " + std::to_string(count) +
                                       " buckets of " + std::to_string(bytes) + " B: " + hipGetErrorString(e));
    }
    char* first = static_cast<char*>(base) + (kSlotSpan - reinterpret_cast<uintptr_t>(base) % kSlotSpan) % kSlotSpan;
    std::lock_guard<std::mutex> lk(g_slots_mu);
    auto* g = new Group{base, count};
    for (size_t j = 0; j < n; ++j) {
        ptrs[j] = first + j * stride;
        g_grouped[ptrs[j]] = g;
    }
    return FMI_OK;
}

int fmi_dev_free(void* ptr) {
    if (!ptr) return FMI_OK;
    if (int rc = require_device()) return rc;
    void* base = ptr;
    {
        std::lock_guard<std::mutex> lk(g_slots_mu);
        auto it = g_slotted.find(ptr);
        if (it != g_slotted.end()) {
            base = it->second;
            g_slotted.erase(it);
        }
        auto gt = g_grouped.find(ptr);
        if (gt != g_grouped.end()) {  // a group's bucket: its range goes with the group's last bucket
            Group* g = gt->second;
            g_grouped.erase(gt);
            if (--g->live > 0) return FMI_OK;
            base = g->base;
            delete g;
        }
    }
    FMI_HIP_TRY(hipFree(base));
    return FMI_OK;
}

int fmi_host_pin_alloc(void** ptr, size_t bytes) {
    if (!ptr) return fail(FMI_ERR_INVALID, "ptr is null");
    if (int rc = require_device()) return rc;
    const hipError_t e = hipHostMalloc(ptr, std::max<size_t>(bytes, 1), hipHostMallocDefault);
    if (e != hipSuccess) return fail(FMI_ERR_ALLOC, "hipHostMalloc(" + std::to_string(bytes) + "): " + hipGetErrorString(e));
    return FMI_OK;
}

int fmi_host_pin_free(void* ptr) {
    if (!ptr) return FMI_OK;
    FMI_HIP_TRY(hipHostFree(ptr));
    return FMI_OK;
}

int fmi_host_register(void* ptr, size_t bytes) {
    if (!ptr || bytes == 0) return fail(FMI_ERR_INVALID, "fmi_host_register: null or empty range");
    if (int rc = require_device()) return rc;
    const hipError_t e = hipHostRegister(ptr, bytes, hipHostRegisterMapped);
    if (e != hipSuccess) return fail(FMI_ERR_ALLOC, "hipHostRegister(" + std::to_string(bytes) + "): " + hipGetErrorString(e));
    return FMI_OK;
}

int fmi_host_unregister(void* ptr) {
    if (!ptr) return fail(FMI_ERR_INVALID, "fmi_host_unregister: null pointer");
    if (int rc = require_device()) return rc;
    FMI_HIP_TRY(hipHostUnregister(ptr));
    return FMI_OK;
}

int fmi_host_device_ptr(const void* host, size_t bytes, void** dev) {
    if (!host || !dev || bytes == 0) return fail(FMI_ERR_INVALID, "fmi_host_device_ptr: null pointer or empty range");
    if (int rc = require_device()) return rc;
    if (!host_mapped(const_cast<void*>(host), bytes, dev))
        return fail(FMI_ERR_INVALID, "fmi_host_device_ptr: the range is not wholly inside one page-locked, device-mapped "
                                     "range (fmi_host_pin_alloc / fmi_host_register)");
    return FMI_OK;
}

int fmi_host_page_locked(const void* host, size_t bytes) {
    if (!host || bytes == 0 || g_state.device < 0) return 0;
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess || (cur != g_state.device && hipSetDevice(g_state.device) != hipSuccess)) {
        (void)hipGetLastError();
        return 0;
    }
    void* d = nullptr;
    return host_mapped(const_cast<void*>(host), bytes, &d) ? 1 : 0;
}

static int copy_async(void* dst, const void* src, size_t bytes, hipMemcpyKind kind, fmi_stream_t stream) {
    if (bytes == 0) return FMI_OK;
    if (!dst || !src) return fail(FMI_ERR_INVALID, "null buffer");
    if (int rc = require_device()) return rc;
    FMI_HIP_TRY(hipMemcpyAsync(dst, src, bytes, kind, resolve(stream)));
    return FMI_OK;
}

int fmi_dev_h2d_async(void* dst, const void* src, size_t bytes, fmi_stream_t stream) {
    return copy_async(dst, src, bytes, hipMemcpyHostToDevice, stream);
}
int fmi_dev_d2h_async(void* dst, const void* src, size_t bytes, fmi_stream_t stream) {
    return copy_async(dst, src, bytes, hipMemcpyDeviceToHost, stream);
}
int fmi_dev_d2d_async(void* dst, const void* src, size_t bytes, fmi_stream_t stream) {
    if (bytes == 0) return FMI_OK;
    if (!dst || !src) return fail(FMI_ERR_INVALID, "null buffer");
    if (int rc = require_device()) return rc;
    return device_copy(dst, src, bytes, resolve(stream));
}

int fmi_dev_memset_async(void* dst, int value, size_t bytes, fmi_stream_t stream) {
    if (bytes == 0) return FMI_OK;
    if (!dst) return fail(FMI_ERR_INVALID, "null buffer");
    if (int rc = require_device()) return rc;
    FMI_HIP_TRY(hipMemsetAsync(dst, value, bytes, resolve(stream)));
    return FMI_OK;
}

// ---- streams / events --------------------------------------------------------------------------------
int fmi_stream_create(fmi_stream_t* stream) {
    if (!stream) return fail(FMI_ERR_INVALID, "stream is null");
    if (int rc = require_device()) return rc;
    hipStream_t s = nullptr;
    FMI_HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    *stream = s;
    return FMI_OK;
}

int fmi_stream_destroy(fmi_stream_t stream) {
    if (!stream) return FMI_OK;
    FMI_HIP_TRY(hipStreamDestroy(static_cast<hipStream_t>(stream)));
    return FMI_OK;
}

int fmi_stream_sync(fmi_stream_t stream) {
    if (int rc = require_device()) return rc;
    FMI_HIP_TRY(hipStreamSynchronize(resolve(stream)));
    return FMI_OK;
}

int fmi_event_create(fmi_event_t* event) {
    if (!event) return fail(FMI_ERR_INVALID, "event is null");
    if (int rc = require_device()) return rc;
    hipEvent_t e = nullptr;
    FMI_HIP_TRY(hipEventCreate(&e));
    *event = e;
    return FMI_OK;
}

int fmi_event_destroy(fmi_event_t event) {
    if (!event) return FMI_OK;
    FMI_HIP_TRY(hipEventDestroy(static_cast<hipEvent_t>(event)));
    return FMI_OK;
}

int fmi_event_record(fmi_event_t event, fmi_stream_t stream) {
    if (!event) return fail(FMI_ERR_INVALID, "event is null");
    if (int rc = require_device()) return rc;
    FMI_HIP_TRY(hipEventRecord(static_cast<hipEvent_t>(event), resolve(stream)));
    return FMI_OK;
}

int fmi_stream_wait_event(fmi_stream_t stream, fmi_event_t event) {
    if (!event) return fail(FMI_ERR_INVALID, "event is null");
    if (int rc = require_device()) return rc;
    FMI_HIP_TRY(hipStreamWaitEvent(resolve(stream), static_cast<hipEvent_t>(event), 0));
    return FMI_OK;
}

int fmi_event_sync(fmi_event_t event) {
    if (!event) return fail(FMI_ERR_INVALID, "event is null");
    FMI_HIP_TRY(hipEventSynchronize(static_cast<hipEvent_t>(event)));
    return FMI_OK;
}

int fmi_event_elapsed_ms(float* ms, fmi_event_t start, fmi_event_t stop) {
    if (!ms || !start || !stop) return fail(FMI_ERR_INVALID, "null argument");
    FMI_HIP_TRY(hipEventElapsedTime(ms, static_cast<hipEvent_t>(start), static_cast<hipEvent_t>(stop)));
    return FMI_OK;
}

// ---- HIP graphs -----------------------------------------------------------------------------------------
int fmi_graph_capture_begin(fmi_stream_t stream) {
    if (int rc = require_device()) return rc;
    if (!stream) return fail(FMI_ERR_INVALID, "graph capture needs a stream from fmi_stream_create");
    FMI_HIP_TRY(hipStreamBeginCapture(static_cast<hipStream_t>(stream), hipStreamCaptureModeThreadLocal));
    return FMI_OK;
}

int fmi_graph_capture_end(fmi_stream_t stream, fmi_graph_t* graph) {
    if (!stream || !graph) return fail(FMI_ERR_INVALID, "null argument");
    *graph = nullptr;
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(static_cast<hipStream_t>(stream), &g);
    if (e != hipSuccess || !g) {
        if (g) (void)hipGraphDestroy(g);
        // the failed call inside the capture left HIP's sticky last error set: clear it, so the next launch
        // on this (now ordinary) stream does not report it as its own
        (void)hipGetLastError();
        return fail(FMI_ERR_HIP, std::string("graph capture failed (a call in the sequence is not capture-safe?): ") +
                                     hipGetErrorString(e));
    }
    hipGraphExec_t x = nullptr;
    const hipError_t ei = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (ei != hipSuccess) return fail(FMI_ERR_HIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(ei));
    *graph = x;
    return FMI_OK;
}

int fmi_graph_launch(fmi_graph_t graph, fmi_stream_t stream) {
    if (!graph) return fail(FMI_ERR_INVALID, "null graph");
    if (int rc = require_device()) return rc;
    FMI_HIP_TRY(hipGraphLaunch(static_cast<hipGraphExec_t>(graph), resolve(stream)));
    return FMI_OK;
}

int fmi_graph_destroy(fmi_graph_t graph) {
    if (graph) FMI_HIP_TRY(hipGraphExecDestroy(static_cast<hipGraphExec_t>(graph)));
    return FMI_OK;
}

// ---- hot path ----------------------------------------------------------------------------------------
int fmi_dev_reduce_pair(int op, int dtype, void* inout, const void* in, size_t n, fmi_stream_t stream) {
    if (int rc = require_device()) return rc;
    return launch_combine(op, dtype, inout, inout, in, n, resolve(stream));
}

int fmi_dev_reduce_pair_batch(int op, int dtype, const fmi_pair_desc_t* descs, int count, fmi_stream_t stream) {
    if (int rc = require_device()) return rc;
    if (op < FMI_OP_SUM || op > FMI_OP_MIN) return fail(FMI_ERR_INVALID, "unknown op " + std::to_string(op));
    const size_t esz = dtype_size(dtype);
    if (esz == 0) return fail(FMI_ERR_INVALID, "unknown dtype " + std::to_string(dtype));
    if (count < 0 || (count > 0 && !descs)) return fail(FMI_ERR_INVALID, "bad descriptor array");
    // no descriptor may write bytes another one reads or writes (one launch runs them concurrently)
    std::vector<std::pair<uintptr_t, uintptr_t>> writes;
    for (int k = 0; k < count; ++k) {
        if (descs[k].n == 0) continue;
        if (!descs[k].inout || !descs[k].in) return fail(FMI_ERR_INVALID, "null bucket in descriptor " + std::to_string(k));
        const uintptr_t w = reinterpret_cast<uintptr_t>(descs[k].inout);
        writes.emplace_back(w, w + descs[k].n * esz);
    }
    std::sort(writes.begin(), writes.end());
    for (size_t k = 1; k < writes.size(); ++k)
        if (writes[k].first < writes[k - 1].second) return fail(FMI_ERR_INVALID, "batch descriptors' inout buckets overlap");
    for (int k = 0; k < count; ++k) {
        if (descs[k].n == 0) continue;
        const uintptr_t r = reinterpret_cast<uintptr_t>(descs[k].in), re = r + descs[k].n * esz;
        const uintptr_t own = reinterpret_cast<uintptr_t>(descs[k].inout);
        auto it = std::upper_bound(writes.begin(), writes.end(), std::make_pair(re, uintptr_t(0)));
        while (it != writes.begin()) {  // write ranges starting before `re`, latest first
            --it;
            if (it->second <= r) break;  // sorted and disjoint: nothing earlier reaches r
            if (it->first != own) return fail(FMI_ERR_INVALID, "a batch descriptor reads another one's inout bucket");
        }
    }
    hipStream_t s = resolve(stream);
    const size_t W = 16 / esz;
    PairBatch pb{};
    int k = 0;
    unsigned tiles = 0;
    auto flush = [&]() -> int {
        if (k == 0) return FMI_OK;
        pb.count = k;
        pb.first_tile[k] = tiles;
        const int rc = launch_pair_batch(op, dtype, pb, s);
        pb = PairBatch{};
        k = 0;
        tiles = 0;
        return rc;
    };
    for (int d = 0; d < count; ++d) {
        const fmi_pair_desc_t& x = descs[d];
        if (x.n == 0) continue;
        const size_t t = std::max<size_t>(1, (x.n / W + kPairBatchTile - 1) / kPairBatchTile);
        if (!aligned16(x.inout) || !aligned16(x.in) || t > (size_t(1) << 20)) {  // unaligned, or large enough alone
            if (int rc = launch_combine(op, dtype, x.inout, x.inout, x.in, x.n, s)) return rc;
            continue;
        }
        if (k == kPairBatchMax || tiles + t > (size_t(1) << 22))
            if (int rc = flush()) return rc;
        pb.inout[k] = x.inout;
        pb.in[k] = x.in;
        pb.n[k] = x.n;
        pb.first_tile[k] = tiles;
        tiles += static_cast<unsigned>(t);
        ++k;
    }
    return flush();
}

int fmi_dev_combine(int op, int dtype, void* out, const void* a, const void* b, size_t n, fmi_stream_t stream) {
    if (int rc = require_device()) return rc;
    return launch_combine(op, dtype, out, a, b, n, resolve(stream));
}

static int reduce_tree_impl(int op, int dtype, int alg, void* out, const void* const* ins, int P, int rank, size_t n,
                            fmi_stream_t stream) {
    if (int rc = check_peer_args(op, dtype, P)) return rc;
    if (alg != FMI_ALG_ALLREDUCE && alg != FMI_ALG_REDUCE && alg != FMI_ALG_REDUCE_LTR)
        return fail(FMI_ERR_INVALID, "fmi_dev_reduce_tree: alg must be ALLREDUCE, REDUCE or REDUCE_LTR");
    if (rank < 0 || rank >= P) return fail(FMI_ERR_INVALID, "rank/root out of range");
    if (!out || !ins) return fail(FMI_ERR_INVALID, "null buffer");
    for (int p = 0; p < P; ++p)
        if (!ins[p]) return fail(FMI_ERR_INVALID, "null input bucket");
    if (int rc = require_device()) return rc;
    if (n == 0) return FMI_OK;
    hipStream_t s = resolve(stream);
    // reduce_no_order works on transformed ids t = (id - root) mod P (PeerToPeer.cpp:287-293):
    // input slot t takes real peer (t + root) % P.
    std::vector<const void*> order(P);
    for (int t = 0; t < P; ++t) order[t] = ins[alg == FMI_ALG_REDUCE ? (t + rank) % P : t];
    bool aligned = aligned16(out);
    for (int p = 0; p < P; ++p) aligned = aligned && aligned16(order[p]);
    if (P >= 2 && aligned && is_core_dtype(dtype)) {
        if (P > sched::max_fused_peers(alg)) return run_tree_blocked(op, dtype, alg, out, order.data(), P, rank, n, s);
        PeerPtrs ptrs{};
        for (int p = 0; p < P; ++p) ptrs.in[p] = order[p];
        ptrs.out[0] = out;
        switch (alg) {
            case FMI_ALG_ALLREDUCE: return launch_fused_allreduce(op, dtype, P, ptrs, n, rank, s);
            case FMI_ALG_REDUCE: return launch_fused_reduce(op, dtype, P, ptrs, n, s);
            default: return launch_fused_reduce_ltr(op, dtype, P, ptrs, n, s);
        }
    }
    const sched::HostProgram prog = sched::build_host(alg, P);
    if (!prog.ok) return fail(FMI_ERR_INVALID, "schedule construction failed");
    const int value = prog.out[alg == FMI_ALG_ALLREDUCE ? rank : 0];
    void* outs[1] = {out};
    return run_program_stepwise(op, dtype, prog, outs, 1, &value, order.data(), n, s);
}

static int scan_peers_impl(int op, int dtype, int alg, void* const* outs, const void* const* ins, int P, size_t n,
                           fmi_stream_t stream) {
    if (int rc = check_peer_args(op, dtype, P)) return rc;
    if (alg != FMI_ALG_SCAN && alg != FMI_ALG_SCAN_LTR)
        return fail(FMI_ERR_INVALID, "fmi_dev_scan_peers: alg must be SCAN or SCAN_LTR");
    if (!outs || !ins) return fail(FMI_ERR_INVALID, "null buffer");
    for (int p = 0; p < P; ++p)
        if (!ins[p] || !outs[p]) return fail(FMI_ERR_INVALID, "null bucket");
    if (int rc = require_device()) return rc;
    if (n == 0) return FMI_OK;
    hipStream_t s = resolve(stream);
    bool aligned = true;
    for (int p = 0; p < P; ++p) aligned = aligned && aligned16(ins[p]) && aligned16(outs[p]);
    if (P >= 2 && aligned && is_core_dtype(dtype)) {
        if (P > sched::max_fused_peers(alg)) return run_scan_blocked(op, dtype, alg, outs, ins, P, n, s);
        PeerPtrs ptrs{};
        for (int p = 0; p < P; ++p) {
            ptrs.in[p] = ins[p];
            ptrs.out[p] = outs[p];
        }
        return alg == FMI_ALG_SCAN ? launch_fused_scan(op, dtype, P, ptrs, n, s)
                                   : launch_fused_scan_ltr(op, dtype, P, ptrs, n, s);
    }
    const sched::HostProgram prog = sched::build_host(alg, P);
    if (!prog.ok) return fail(FMI_ERR_INVALID, "schedule construction failed");
    std::vector<int> values(P);
    for (int p = 0; p < P; ++p) values[p] = prog.out[p];
    return run_program_stepwise(op, dtype, prog, outs, P, values.data(), ins, n, s);
}

// Host-ingress pipeline: chunk c uses slot c % 2 (its own staging pair and its own stream). Stream order
// keeps a slot's staging from being overwritten before its previous D2H finished, while the other slot's
// H2D overlaps this slot's kernel + D2H.
int fmi_host_reduce_pair(int op, int dtype, void* inout, const void* in, size_t n) {
    if (op < FMI_OP_SUM || op > FMI_OP_MIN) return fail(FMI_ERR_INVALID, "unknown op " + std::to_string(op));
    const size_t esz = dtype_size(dtype);
    if (esz == 0) return fail(FMI_ERR_INVALID, "unknown dtype " + std::to_string(dtype));
    if (n == 0) return FMI_OK;
    if (!inout || !in) return fail(FMI_ERR_INVALID, "null buffer");
    if (int rc = require_device()) return rc;
    // A bucket partly inside a page-locked range: the zero-copy kernel must not read past that range, and
    // the runtime rejects copies that start or end inside one. Pin or register all of it, or none.
    for (const void* p : {static_cast<const void*>(inout), in}) {
        void* d = nullptr;
        char* c = static_cast<char*>(const_cast<void*>(p));
        const bool head = host_mapped_at(c, &d), tail = host_mapped_at(c + n * esz - 1, &d);
        if ((head || tail) && !host_mapped(c, n * esz, &d))
            return fail(FMI_ERR_INVALID, "fmi_host_reduce_pair: a bucket straddles the end of a page-locked range "
                                         "(pin or register the whole bucket, or none of it)");
    }
    std::shared_lock<std::shared_mutex> life(g_pipes_life);
    const int device = g_state.device;  // read under the lock: a finalize between require_device() and here
    if (device < 0) return fail(FMI_ERR_NO_DEVICE, "fmi_dev_finalize ran before this fmi_host_reduce_pair started");
    PipeLease lease(device);  // this call's streams and staging: concurrent callers do not serialise (up to the cap)
    HostPipe& hp = *lease.p;
    for (int k = 0; k < 2; ++k)
        if (!hp.pipe[k]) FMI_HIP_TRY(hipStreamCreateWithFlags(&hp.pipe[k], hipStreamNonBlocking));
    if (g_tune[FMI_TUNE_HOST_ZERO_COPY].load()) {
        // Page-locked buckets: the kernel streams them straight over PCIe (reads of both operands and the
        // write-back share the link concurrently, no staging copies, no DMA-engine serialisation).
        void* dx = nullptr;
        void* dy = nullptr;
        if (host_mapped(inout, n * esz, &dx) && host_mapped(const_cast<void*>(in), n * esz, &dy)) {
            hipStream_t s = hp.pipe[0];
            int rc = launch_combine(op, dtype, dx, dx, dy, n, s);
            if (rc != FMI_OK) return rc;
            FMI_HIP_TRY(hipStreamSynchronize(s));
            return FMI_OK;
        }
    }
    size_t chunk_elems = static_cast<size_t>(std::max<long long>(g_tune[FMI_TUNE_HOST_CHUNK].load(), 1 << 16)) / esz;
    chunk_elems = std::max<size_t>(16, chunk_elems / 16 * 16);
    const size_t chunk_bytes = chunk_elems * esz;
    // this call's largest chunk, rounded up to a power of two (>= 64 KiB), never above the tuned chunk
    size_t need = 64 << 10;
    while (need < std::min(chunk_bytes, n * esz)) need <<= 1;
    need = std::min(need, chunk_bytes);
    if (hp.stage_bytes < need) {
        for (int k = 0; k < 2; ++k) FMI_HIP_TRY(hipStreamSynchronize(hp.pipe[k]));
        for (int k = 0; k < 2; ++k)
            for (int j = 0; j < 2; ++j) {
                if (hp.stage[k][j]) FMI_HIP_TRY(hipFree(hp.stage[k][j]));
                hp.stage[k][j] = nullptr;
            }
        for (int k = 0; k < 2; ++k)
            for (int j = 0; j < 2; ++j) {
                const hipError_t e = hipMalloc(&hp.stage[k][j], need);
                if (e != hipSuccess) {
                    hp.stage_bytes = 0;
                    return fail(FMI_ERR_ALLOC, std::string("hipMalloc (host pipeline staging): ") + hipGetErrorString(e));
                }
            }
        hp.stage_bytes = need;
    }
    char* hx = static_cast<char*>(inout);
    const char* hy = static_cast<const char*>(in);
    int rc = FMI_OK;
    size_t chunk = 0;
    for (size_t off = 0; off < n && rc == FMI_OK; off += chunk_elems, ++chunk) {
        const int slot = static_cast<int>(chunk & 1);
        hipStream_t s = hp.pipe[slot];
        const size_t cnt = std::min(chunk_elems, n - off);
        const size_t bytes = cnt * esz;
        void* da = hp.stage[slot][0];
        void* db = hp.stage[slot][1];
        FMI_HIP_TRY(hipMemcpyAsync(da, hx + off * esz, bytes, hipMemcpyHostToDevice, s));
        FMI_HIP_TRY(hipMemcpyAsync(db, hy + off * esz, bytes, hipMemcpyHostToDevice, s));
        rc = launch_combine(op, dtype, da, da, db, cnt, s);
        if (rc != FMI_OK) break;
        FMI_HIP_TRY(hipMemcpyAsync(hx + off * esz, da, bytes, hipMemcpyDeviceToHost, s));
    }
    for (int k = 0; k < 2; ++k) FMI_HIP_TRY(hipStreamSynchronize(hp.pipe[k]));
    return rc;
}

int fmi_dev_fill_synthetic_at(int dtype, void* buf, size_t n, uint64_t seed, uint32_t peer, uint64_t first,
                              fmi_stream_t stream) {
    if (n == 0) return FMI_OK;
    if (!buf) return fail(FMI_ERR_INVALID, "null buffer");
    if (int rc = require_device()) return rc;
    hipStream_t s = resolve(stream);
    const unsigned grid = static_cast<unsigned>(std::min<size_t>(grid_for(n, 256), 16384));
    if (int rc = with_dtype<true>(dtype, [&]<class T>() -> int {
            synth_kernel<T><<<grid, 256, 0, s>>>(static_cast<T*>(buf), n, seed, peer, first);
            return FMI_OK;
        }))
        return rc;
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail("synthetic fill launch", e);
    return FMI_OK;
}

int fmi_dev_fill_synthetic(int dtype, void* buf, size_t n, uint64_t seed, uint32_t peer, fmi_stream_t stream) {
    return fmi_dev_fill_synthetic_at(dtype, buf, n, seed, peer, 0, stream);
}

static int schedule_expr_impl(int alg, int P, int rank, char* buf, size_t len) {
    if (!buf || len == 0) return fail(FMI_ERR_INVALID, "null buffer");
    if (P < 1 || P > sched::kMaxPeers) return fail(FMI_ERR_INVALID, "P out of range");
    if (rank < 0 || rank >= P) return fail(FMI_ERR_INVALID, "rank out of range");
    if (alg < FMI_ALG_ALLREDUCE || alg > FMI_ALG_SCAN_LTR) return fail(FMI_ERR_INVALID, "unknown algorithm " + std::to_string(alg));
    const sched::HostProgram prog = sched::build_host(alg, P);
    if (!prog.ok) return fail(FMI_ERR_INVALID, "unknown algorithm " + std::to_string(alg));
    const std::string e = expr_of(prog, prog.out[rank]);
    if (e.size() + 1 > len) return fail(FMI_ERR_INVALID, "buffer too small (" + std::to_string(e.size() + 1) + " needed)");
    std::memcpy(buf, e.c_str(), e.size() + 1);
    return FMI_OK;
}

int fmi_dev_reduce_tree(int op, int dtype, int alg, void* out, const void* const* ins, int P, int rank, size_t n,
                        fmi_stream_t stream) {
    return guarded("fmi_dev_reduce_tree", [&] { return reduce_tree_impl(op, dtype, alg, out, ins, P, rank, n, stream); });
}

int fmi_dev_scan_peers(int op, int dtype, int alg, void* const* outs, const void* const* ins, int P, size_t n,
                       fmi_stream_t stream) {
    return guarded("fmi_dev_scan_peers", [&] { return scan_peers_impl(op, dtype, alg, outs, ins, P, n, stream); });
}

int fmi_schedule_expr(int alg, int P, int rank, char* buf, size_t len) {
    return guarded("fmi_schedule_expr", [&] { return schedule_expr_impl(alg, P, rank, buf, len); });
}

int fmi_tune_set(int key, long long value) {
    switch (key) {
        case FMI_TUNE_PAIR_VARIANT:
            if (value < 0 || value > 4) return fail(FMI_ERR_INVALID, "variant must be in [0, 4]");
            break;
        case FMI_TUNE_PAIR_UNROLL:
            if (value != 1 && value != 2 && value != 4 && value != 8) return fail(FMI_ERR_INVALID, "unroll must be 1, 2, 4 or 8");
            break;
        case FMI_TUNE_BLOCK:
            if (value != 64 && value != 128 && value != 256 && value != 512 && value != 1024)
                return fail(FMI_ERR_INVALID, "block must be 64..1024 (power of two)");
            break;
        case FMI_TUNE_GRID_PER_CU:
            if (value < 1 || value > 64) return fail(FMI_ERR_INVALID, "grid per CU must be in [1, 64]");
            break;
        case FMI_TUNE_HOST_CHUNK:
            if (value < (1 << 16)) return fail(FMI_ERR_INVALID, "host chunk must be >= 64 KiB");
            break;
        case FMI_TUNE_HOST_ZERO_COPY:
            if (value != 0 && value != 1) return fail(FMI_ERR_INVALID, "host zero-copy must be 0 or 1");
            break;
        case FMI_TUNE_FUSED_INFLIGHT_KIB:
            if (value < 0 || value > 4096) return fail(FMI_ERR_INVALID, "fused in-flight budget must be in [0, 4096] KiB");
            break;
        case FMI_TUNE_BLOCKS_ONE_PASS:
            if (value != 0 && value != 1) return fail(FMI_ERR_INVALID, "one-pass blocked scan must be 0 or 1");
            break;
        case FMI_TUNE_COMM_A2A:
        case FMI_TUNE_COMM_GATHER:
            if (value != 0 && value != 1) return fail(FMI_ERR_INVALID, "exchange variant must be 0 or 1");
            break;
        case FMI_TUNE_COMM_PIPELINE:
            if (value < 0 || value > 64) return fail(FMI_ERR_INVALID, "pipeline chunks must be in [0, 64]");
            break;
        case FMI_TUNE_FUSED_POLICY:
            if (value < 0 || value > 2) return fail(FMI_ERR_INVALID, "fused access policy must be 0, 1 or 2");
            break;
        case FMI_TUNE_PAIR_SC1_OF_8:
            if (value < 0 || value > 8) return fail(FMI_ERR_INVALID, "pair sc1 tiles per 8 must be in [0, 8]");
            break;
        case FMI_TUNE_COMM_ONE_RANK_EXCHANGE:
            if (value != 0 && value != 1) return fail(FMI_ERR_INVALID, "one-rank exchange must be 0 or 1");
            break;
        case FMI_TUNE_ALLOC_SLOTS:
            if (value != 0 && value != 1) return fail(FMI_ERR_INVALID, "allocation slots must be 0 or 1");
            break;
        case FMI_TUNE_COMM_SHARD_SKEW:
            if (value != 0 && value != 1) return fail(FMI_ERR_INVALID, "shard skew must be 0 or 1");
            break;
        default: return fail(FMI_ERR_INVALID, "unknown tuning key");
    }
    g_tune[key].store(value);
    return FMI_OK;
}

int fmi_tune_get(int key, long long* value) {
    if (!value || key < 0 || key > FMI_TUNE_COMM_SHARD_SKEW) return fail(FMI_ERR_INVALID, "bad tuning query");
    *value = g_tune[key].load();
    return FMI_OK;
}

}  // extern "C"
