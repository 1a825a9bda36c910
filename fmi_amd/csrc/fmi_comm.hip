// fmi_comm.hip — sharded device collectives across GPUs (include/fmi_dev.h, "sharded device collectives").
//
// One rank = one FMI peer = one GPU. The reference's allreduce / reduce / scan (src/comm/PeerToPeer.cpp)
// exchange whole buckets peer to peer; here every bucket is cut into N shards so that all of a GPU's xGMI
// links carry traffic at once, and the combine of each shard is ONE pass of the fused P-way kernel in the
// reference's evaluation order (fmi_schedule.h):
//
//   allreduce  all-to-all(shards) -> fused tree over the N partials of my shard -> all-gather
//   reduce     all-to-all(shards) -> fused tree in reduce order for `root`       -> gather to root
//   scan       all-to-all(shards) -> fused peer-axis scan (N prefixes of my shard) -> all-to-all back
//
// Transports: RCCL (librccl resolved with dlopen on first use, so processes that never use it never load
// it) and LOCAL (ranks are threads of one process on one device; the exchanges are device-to-device
// copies) — the latter runs the exact same schedules, which is how the multi-rank logic is tested on a
// single MI355X.
#include <dlfcn.h>
#include <fcntl.h>
#include <rccl/rccl.h>

#include "fmi_exchange_plan.h"
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "fmi_internal.h"

namespace fmi::dev {
namespace {

constexpr size_t kShardAlign = 64;  // elements: shards stay 256-B aligned for the 16-B vector kernels

int hip_err(const char* what, hipError_t e) { return fail(FMI_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e)); }

long long tune(int key) {
    long long v = 0;
    (void)fmi_tune_get(key, &v);
    return v;
}

#define FMI_COMM_HIP(call)                                 \
    do {                                                   \
        const hipError_t e_ = (call);                      \
        if (e_ != hipSuccess) return hip_err(#call, e_);   \
    } while (0)
#define FMI_COMM_RC(call)              \
    do {                               \
        const int rc_ = (call);        \
        if (rc_ != FMI_OK) return rc_; \
    } while (0)

// ---------------------------------------------------------------------------------------------------
// RCCL entry points (dlopen'd once)
// ---------------------------------------------------------------------------------------------------
struct RcclApi {
    ncclResult_t (*GetUniqueId)(ncclUniqueId*);
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int);
    ncclResult_t (*CommDestroy)(ncclComm_t);
    const char* (*GetErrorString)(ncclResult_t);
    ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
    ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
    ncclResult_t (*GroupStart)();
    ncclResult_t (*GroupEnd)();
    ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t);
    ncclResult_t (*ReduceScatter)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t);
    ncclResult_t (*Broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
    ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t);
    // RCCL's native all-to-all (optional symbol; grouped send/recv otherwise)
    ncclResult_t (*AllToAll)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t);
    // optional: bounded waits (non-blocking init, asynchronous errors, abort on timeout) and introspection
    ncclResult_t (*CommInitRankConfig)(ncclComm_t*, int, ncclUniqueId, int, ncclConfig_t*);
    ncclResult_t (*CommGetAsyncError)(ncclComm_t, ncclResult_t*);
    ncclResult_t (*CommAbort)(ncclComm_t);
    ncclResult_t (*CommFinalize)(ncclComm_t);
    ncclResult_t (*CommCount)(const ncclComm_t, int*);
    ncclResult_t (*GetVersion)(int*);
    ncclResult_t (*CommUserRank)(const ncclComm_t, int*);
    ncclResult_t (*CommCuDevice)(const ncclComm_t, int*);
    bool bounded() const { return CommInitRankConfig && CommGetAsyncError && CommAbort; }
};

const RcclApi* rccl_api() {
    static std::once_flag once;
    static RcclApi api;
    static bool ok = false;
    static std::string err;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
        if (!h) {
            err = std::string("cannot load librccl: ") + dlerror();
            return;
        }
#define FMI_RCCL_SYM(name)                                                                  \
    api.name = reinterpret_cast<decltype(api.name)>(dlsym(h, "nccl" #name));                \
    if (!api.name) {                                                                        \
        err = "librccl lacks nccl" #name;                                                   \
        return;                                                                             \
    }
        FMI_RCCL_SYM(GetUniqueId)
        FMI_RCCL_SYM(CommInitRank)
        FMI_RCCL_SYM(CommDestroy)
        FMI_RCCL_SYM(GetErrorString)
        FMI_RCCL_SYM(Send)
        FMI_RCCL_SYM(Recv)
        FMI_RCCL_SYM(GroupStart)
        FMI_RCCL_SYM(GroupEnd)
        FMI_RCCL_SYM(AllGather)
        FMI_RCCL_SYM(ReduceScatter)
        FMI_RCCL_SYM(Broadcast)
        FMI_RCCL_SYM(AllReduce)
#undef FMI_RCCL_SYM
        api.AllToAll = reinterpret_cast<decltype(api.AllToAll)>(dlsym(h, "ncclAllToAll"));
#define FMI_RCCL_OPT(name) api.name = reinterpret_cast<decltype(api.name)>(dlsym(h, "nccl" #name));
        FMI_RCCL_OPT(CommInitRankConfig)
        FMI_RCCL_OPT(CommGetAsyncError)
        FMI_RCCL_OPT(CommAbort)
        FMI_RCCL_OPT(CommFinalize)
        FMI_RCCL_OPT(CommCount)
        FMI_RCCL_OPT(CommUserRank)
        FMI_RCCL_OPT(CommCuDevice)
        FMI_RCCL_OPT(GetVersion)
#undef FMI_RCCL_OPT
        ok = true;
    });
    if (!ok) {
        fail(FMI_ERR_COMM, err);
        return nullptr;
    }
    return &api;
}

int nccl_fail(const RcclApi* api, const char* what, ncclResult_t r) {
    return fail(FMI_ERR_COMM, std::string(what) + ": " + api->GetErrorString(r));
}

#define FMI_NCCL(api, call)                                        \
    do {                                                           \
        const ncclResult_t r_ = (api)->call;                       \
        if (r_ != ncclSuccess) return nccl_fail((api), #call, r_); \
    } while (0)

// ---------------------------------------------------------------------------------------------------
// transports
// ---------------------------------------------------------------------------------------------------
using Clock = std::chrono::steady_clock;

double env_seconds(const char* name, double fallback) {
    const char* e = std::getenv(name);
    if (!e || !*e) return fallback;
    const double v = std::atof(e);
    return v > 0 ? v : fallback;
}

// The default timeout of a communicator (fmi_comm_init): FMI_COMM_TIMEOUT_S, then (PROC) the older
// FMI_PROC_TIMEOUT_S, then 300 s.
double default_timeout_s(bool proc) {
    return env_seconds("FMI_COMM_TIMEOUT_S", proc ? env_seconds("FMI_PROC_TIMEOUT_S", 300.0) : 300.0);
}

// Poll with back-off: spin ~1k times, then sleep 5 us, then 200 us between checks.
void backoff(int k) {
    if (k < 1000) return;
    std::this_thread::sleep_for(std::chrono::microseconds(k < 10000 ? 5 : 200));
}

class Transport {
public:
    Transport(int n, int rank) : n_(n), rank_(rank) {}
    virtual ~Transport() = default;

    // ---- bounded waits (reference FMI::Utils::Timeout semantics) ----
    void set_timeout(double seconds) { timeout_s_ = seconds; }
    double timeout_s() const { return timeout_s_; }
    bool aborted() const { return aborted_; }
    // An asynchronous error of the transport (a peer's connection failed), FMI_OK if none.
    virtual int poll() { return FMI_OK; }
    // Give up on the peers: release what waits for them (RCCL: ncclCommAbort ends its kernels). Idempotent.
    virtual void abort() { aborted_ = true; }
    // Abort and report a timeout.
    int timed_out(const std::string& what) {
        abort();
        return fail(FMI_ERR_TIMEOUT, "Timeout was reached: " + what + " (not complete within " +
                                         std::to_string(timeout_s_) + " s; communicator aborted)");
    }
    // Wait for the work on s within the timeout, watching for transport errors. The limit covers everything
    // queued on s when the wait starts: callers that queue long pipelines wait per stage (wait_event), so the
    // limit bounds one stage's progress, not the whole call.
    int wait_stream(hipStream_t s, const char* what) {
        return wait_until_done([s] { return hipStreamQuery(s); }, s, what);
    }
    // Wait for `ev`'s last record within the timeout (a fresh deadline per call), watching for transport errors.
    int wait_event(hipEvent_t ev, hipStream_t s, const char* what) {
        return wait_until_done([ev] { return hipEventQuery(ev); }, s, what);
    }
    template <class Query>
    int wait_until_done(Query&& query, hipStream_t s, const char* what) {
        const auto t0 = Clock::now();
        for (int k = 0;; ++k) {
            const hipError_t e = query();
            if (e == hipSuccess) return FMI_OK;
            if (e != hipErrorNotReady) return fail(FMI_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
            if (int rc = poll()) {
                abort();
                return rc;
            }
            if (std::chrono::duration<double>(Clock::now() - t0).count() > timeout_s_) {
                const int rc = timed_out(what);
                drain(s, 10.0);  // the aborted transport's kernels end; do not leave them running
                return rc;
            }
            backoff(k);
        }
    }
    // Bounded wait for s (after an abort: never block forever). True if it drained.
    static bool drain(hipStream_t s, double seconds) {
        return drain_query([s] { return hipStreamQuery(s); }, seconds);
    }
    static bool drain_event(hipEvent_t ev, double seconds) {
        return drain_query([ev] { return hipEventQuery(ev); }, seconds);
    }
    template <class Query>
    static bool drain_query(Query&& query, double seconds) {
        const auto t0 = Clock::now();
        for (int k = 0;; ++k) {
            const hipError_t e = query();
            if (e != hipErrorNotReady) return e == hipSuccess;
            if (std::chrono::duration<double>(Clock::now() - t0).count() > seconds) return false;
            backoff(k);
        }
    }
    // What the transport reports about itself (fmi_comm_query).
    virtual int query(int* count, int* rank, int* device) {
        *count = n_;
        *rank = rank_;
        FMI_COMM_HIP(hipGetDevice(device));
        return FMI_OK;
    }
    // recv[j*bytes ...] = rank j's send[rank*bytes ...]
    virtual int all_to_all(const char* send, char* recv, size_t bytes, hipStream_t s) = 0;
    // all_to_all with rank j's block landing at recv + j * stride (stride >= bytes; the gaps untouched), for the
    // shard kernel's inputs (shard_stride). Only transports whose all-to-all posts one receive per peer anyway take a
    // stride other than bytes: for them the stride changes where the bytes land, never which operations run.
    virtual bool receives_per_peer() const { return false; }
    virtual int all_to_all_strided(const char* send, char* recv, size_t bytes, size_t stride, hipStream_t s) {
        if (stride == bytes) return all_to_all(send, recv, bytes, s);
        return fail(FMI_ERR_UNSUPPORTED, "transport has no strided all-to-all");
    }
    // recv[j*bytes ...] = rank j's send[0 .. bytes)
    virtual int all_gather(const char* send, char* recv, size_t bytes, hipStream_t s) = 0;
    virtual int gather(const char* send, char* recv, size_t bytes, int root, hipStream_t s) = 0;
    virtual int scatter(const char* send, char* recv, size_t bytes, int root, hipStream_t s) = 0;
    virtual int bcast(char* buf, size_t bytes, int root, hipStream_t s) = 0;
    virtual int send(const char* buf, size_t bytes, int peer, hipStream_t s) = 0;
    virtual int recv(char* buf, size_t bytes, int peer, hipStream_t s) = 0;
    virtual int barrier(hipStream_t s) = 0;
    // Stream-ordered barrier: work enqueued on s after it starts only once every rank has reached it.
    virtual int barrier_async(hipStream_t s) = 0;
    // Symmetric window: map every rank's `base` into this process (peers[j] = rank j's base, peers[rank] =
    // base). Collective, and all-or-nothing: `ok` is this rank's own readiness (its allocation succeeded);
    // every rank returns FMI_OK only if every rank could export and map, so no rank is left waiting.
    virtual int map_window(char* base, bool ok, std::vector<char*>& peers, hipStream_t s) = 0;
    virtual void unmap_window(const std::vector<char*>& peers) = 0;
    // Blocking element-wise max over ranks of k <= kAgreeMax host int64 values (in place): used to check
    // that every rank passed the same arguments (FMI_CHECK_DIRECT).
    static constexpr int kAgreeMax = 4;
    virtual int agree_max(int64_t* vals, int k, hipStream_t s) = 0;
    virtual int reduce_scatter(int, int, const void*, void*, size_t, hipStream_t) {
        return fail(FMI_ERR_UNSUPPORTED, "path RCCL needs the RCCL transport");
    }
    // Ragged exchanges: shard j covers bytes [j * shard, min(total, (j + 1) * shard)) of a bucket (the last
    // shards short or empty), so a bucket needs no zero padding. all_to_all_ragged: recv[j * shard ...] = rank
    // j's shard `rank` (span(rank) bytes); all_gather_ragged: recv[j * shard ...] = rank j's send (span(j)).
    virtual bool ragged() const { return false; }
    // Several ranks of this communicator drive the same device from this process: their host pipelines share one
    // H2D and one D2H stream (copy_streams). Every other rank owns its pair (HostPipe::init).
    virtual bool co_resident() const { return false; }
    virtual int copy_streams(hipStream_t*, hipStream_t*) {
        return fail(FMI_ERR_UNSUPPORTED, "copy streams are shared only among co-resident ranks");
    }
    virtual int all_to_all_ragged(const char*, char*, size_t, size_t, hipStream_t) {
        return fail(FMI_ERR_UNSUPPORTED, "transport has no ragged exchanges");
    }
    virtual int all_gather_ragged(const char*, char*, size_t, size_t, hipStream_t) {
        return fail(FMI_ERR_UNSUPPORTED, "transport has no ragged exchanges");
    }
    // gather_ragged: root's recv[j * shard ...] = rank j's send (span(j) bytes).
    virtual int gather_ragged(const char*, char*, size_t, size_t, int, hipStream_t) {
        return fail(FMI_ERR_UNSUPPORTED, "transport has no ragged exchanges");
    }
    // all_to_all_back_ragged: recv[j * shard ...] = rank j's send[rank * shard ...] (span(j) bytes): the
    // inverse of all_to_all_ragged, every owner handing each rank its version of the owner's shard.
    virtual int all_to_all_back_ragged(const char*, char*, size_t, size_t, hipStream_t) {
        return fail(FMI_ERR_UNSUPPORTED, "transport has no ragged exchanges");
    }
    static size_t span(int j, size_t shard, size_t total) { return plan::span(j, shard, total); }
    // A second communicator over the same ranks (collective), so two exchanges can be in flight at once on
    // two streams. nullptr: this transport's exchanges are host-synchronous, use it as is.
    virtual int split(std::unique_ptr<Transport>* out, hipStream_t) {
        out->reset();
        return FMI_OK;
    }
    int n() const { return n_; }
    int rank() const { return rank_; }

protected:
    int n_;
    int rank_;
    double timeout_s_ = 300.0;
    bool aborted_ = false;
};

// RCCL element type of a dtype; false for the 16-bit integers, which RCCL has no reduction type for.
bool nccl_type(int dtype, ncclDataType_t* t) {
    switch (dtype) {
        case FMI_F32: *t = ncclFloat32; return true;
        case FMI_F64: *t = ncclFloat64; return true;
        case FMI_I32: *t = ncclInt32; return true;
        case FMI_I64: *t = ncclInt64; return true;
        case FMI_U32: *t = ncclUint32; return true;
        case FMI_U64: *t = ncclUint64; return true;
        case FMI_I8: *t = ncclInt8; return true;
        case FMI_U8: *t = ncclUint8; return true;
        default: return false;
    }
}

ncclRedOp_t nccl_op(int op) {
    switch (op) {
        case FMI_OP_SUM: return ncclSum;
        case FMI_OP_PROD: return ncclProd;
        case FMI_OP_MAX: return ncclMax;
        default: return ncclMin;
    }
}

// An RCCL call of this transport: ncclInProgress (a non-blocking communicator still connecting or enqueuing)
// is waited out within the timeout, any other failure is returned.
#define FMI_RCCL(call)                                      \
    do {                                                    \
        const int rc_ = ck(api_->call, #call);              \
        if (rc_ != FMI_OK) return rc_;                      \
    } while (0)

class RcclTransport final : public Transport {
public:
    // nonblocking: the communicator was made with config.blocking = 0 (fmi_comm_init with a librccl that has
    // ncclCommInitRankConfig / ncclCommGetAsyncError / ncclCommAbort): every wait for the peers is bounded.
    RcclTransport(const RcclApi* api, ncclComm_t comm, int n, int rank, bool nonblocking)
        : Transport(n, rank), api_(api), comm_(comm), nonblocking_(nonblocking) {}
    ~RcclTransport() override {
        if (token_) (void)hipFree(token_);
        if (aborted_ || !comm_) return;  // ncclCommAbort released it
        if (nonblocking_ && api_->CommFinalize) {
            // flush, bounded: a peer that never arrives must not hang the destructor
            const ncclResult_t r = api_->CommFinalize(comm_);
            if ((r != ncclSuccess && r != ncclInProgress) || wait_ready("ncclCommFinalize") != FMI_OK) {
                abort();
                return;
            }
        }
        (void)api_->CommDestroy(comm_);
    }

    // Wait until the communicator has no operation in progress (non-blocking init / connect / enqueue).
    int wait_ready(const char* what) {
        if (!nonblocking_) return FMI_OK;
        const auto t0 = Clock::now();
        for (int k = 0;; ++k) {
            ncclResult_t st = ncclSuccess;
            const ncclResult_t r = api_->CommGetAsyncError(comm_, &st);
            if (r != ncclSuccess) return nccl_fail(api_, "ncclCommGetAsyncError", r);
            if (st == ncclSuccess) return FMI_OK;
            if (st != ncclInProgress) {
                abort();
                return fail(FMI_ERR_COMM, std::string(what) + ": " + api_->GetErrorString(st) + " (communicator aborted)");
            }
            if (std::chrono::duration<double>(Clock::now() - t0).count() > timeout_s_) return timed_out(what);
            backoff(k);
        }
    }
    int poll() override {
        if (!nonblocking_ || aborted_) return FMI_OK;
        ncclResult_t st = ncclSuccess;
        if (api_->CommGetAsyncError(comm_, &st) != ncclSuccess) return FMI_OK;
        if (st == ncclSuccess || st == ncclInProgress) return FMI_OK;
        return fail(FMI_ERR_COMM, std::string("RCCL asynchronous error: ") + api_->GetErrorString(st) +
                                      " (communicator aborted)");
    }
    void abort() override {
        if (!aborted_ && api_->CommAbort && comm_) (void)api_->CommAbort(comm_);
        aborted_ = true;
    }
    int query(int* count, int* rank, int* device) override {
        if (!api_->CommCount || !api_->CommUserRank) return Transport::query(count, rank, device);
        FMI_RCCL(CommCount(comm_, count));
        FMI_RCCL(CommUserRank(comm_, rank));
        if (api_->CommCuDevice) {
            FMI_RCCL(CommCuDevice(comm_, device));
        } else {
            FMI_COMM_HIP(hipGetDevice(device));
        }
        return FMI_OK;
    }

    int all_to_all(const char* send, char* recv, size_t bytes, hipStream_t s) override {
        if (api_->AllToAll && tune(FMI_TUNE_COMM_A2A) == 0) {
            FMI_RCCL(AllToAll(send, recv, bytes, ncclUint8, comm_, s));
            return FMI_OK;
        }
        return run_plan(plan::all_to_all(n_, rank_, bytes), send, recv, s);
    }
    // ncclAllToAll receives one contiguous buffer: only the grouped form (FMI_TUNE_COMM_A2A = 1, or a librccl
    // without ncclAllToAll) takes a stride, with the same sends and receives as without one
    bool receives_per_peer() const override { return !(api_->AllToAll && tune(FMI_TUNE_COMM_A2A) == 0); }
    int all_to_all_strided(const char* send, char* recv, size_t bytes, size_t stride, hipStream_t s) override {
        if (stride == bytes) return all_to_all(send, recv, bytes, s);
        if (!receives_per_peer()) return fail(FMI_ERR_UNSUPPORTED, "ncclAllToAll takes no receive stride");
        return run_plan(plan::all_to_all(n_, rank_, bytes, stride), send, recv, s);
    }
    int all_gather(const char* send, char* recv, size_t bytes, hipStream_t s) override {
        if (tune(FMI_TUNE_COMM_GATHER) == 0) {
            FMI_RCCL(AllGather(send, recv, bytes, ncclUint8, comm_, s));
            return FMI_OK;
        }
        return run_plan(plan::all_gather(n_, rank_, bytes), send, recv, s);  // one link per peer, no ring
    }
    bool ragged() const override { return true; }
    int all_to_all_ragged(const char* send, char* recv, size_t shard, size_t total, hipStream_t s) override {
        return run_plan(plan::all_to_all_ragged(n_, rank_, shard, total), send, recv, s);
    }
    int all_gather_ragged(const char* send, char* recv, size_t shard, size_t total, hipStream_t s) override {
        return run_plan(plan::all_gather_ragged(n_, rank_, shard, total), send, recv, s);
    }
    int gather_ragged(const char* send, char* recv, size_t shard, size_t total, int root, hipStream_t s) override {
        return run_plan(plan::gather_ragged(n_, rank_, shard, total, root), send, recv, s);
    }
    int all_to_all_back_ragged(const char* send, char* recv, size_t shard, size_t total, hipStream_t s) override {
        return run_plan(plan::all_to_all_back_ragged(n_, rank_, shard, total), send, recv, s);
    }
    int gather(const char* send, char* recv, size_t bytes, int root, hipStream_t s) override {
        return run_plan(plan::gather(n_, rank_, bytes, root), send, recv, s);
    }
    int scatter(const char* send, char* recv, size_t bytes, int root, hipStream_t s) override {
        return run_plan(plan::scatter(n_, rank_, bytes, root), send, recv, s);
    }
    int bcast(char* buf, size_t bytes, int root, hipStream_t s) override {
        FMI_RCCL(Broadcast(buf, buf, bytes, ncclUint8, root, comm_, s));
        return FMI_OK;
    }
    int send(const char* buf, size_t bytes, int peer, hipStream_t s) override {
        FMI_RCCL(Send(buf, bytes, ncclUint8, peer, comm_, s));
        return FMI_OK;
    }
    int recv(char* buf, size_t bytes, int peer, hipStream_t s) override {
        FMI_RCCL(Recv(buf, bytes, ncclUint8, peer, comm_, s));
        return FMI_OK;
    }
    int barrier(hipStream_t s) override {
        if (!token_) FMI_COMM_HIP(hipMalloc(&token_, sizeof(int)));
        FMI_RCCL(AllReduce(token_, token_, 1, ncclInt32, ncclSum, comm_, s));
        return wait_stream(s, "barrier");
    }
    int reduce_scatter(int op, int dtype, const void* send, void* recv, size_t count, hipStream_t s) override {
        ncclDataType_t t;
        if (!nccl_type(dtype, &t)) return fail(FMI_ERR_UNSUPPORTED, "path RCCL: RCCL has no 16-bit integer reductions");
        FMI_RCCL(ReduceScatter(send, recv, count, t, nccl_op(op), comm_, s));
        return FMI_OK;
    }
    int barrier_async(hipStream_t s) override {
        if (!token_) FMI_COMM_HIP(hipMalloc(&token_, sizeof(int)));
        FMI_RCCL(AllReduce(token_, token_, 1, ncclInt32, ncclSum, comm_, s));
        return FMI_OK;
    }
    // IPC handles travel by all-gather; the peer mappings are opened with lazy peer access (xGMI). A final
    // all-reduce(min) of every rank's success flag makes the outcome identical on all ranks.
    int map_window(char* base, bool ok, std::vector<char*>& peers, hipStream_t s) override {
        constexpr size_t H = sizeof(hipIpcMemHandle_t);
        hipIpcMemHandle_t mine{};
        if (ok) ok = hipIpcGetMemHandle(&mine, base) == hipSuccess;
        char* d = nullptr;
        FMI_COMM_HIP(hipMalloc(&d, (n_ + 1) * H + 2 * sizeof(int)));
        std::vector<hipIpcMemHandle_t> all(n_);
        int flag = 0;
        int rc = [&]() -> int {
            FMI_COMM_HIP(hipMemcpyAsync(d + n_ * H, &mine, H, hipMemcpyHostToDevice, s));
            FMI_RCCL(AllGather(d + n_ * H, d, H, ncclUint8, comm_, s));
            FMI_COMM_HIP(hipMemcpyAsync(all.data(), d, n_ * H, hipMemcpyDeviceToHost, s));
            FMI_COMM_RC(wait_stream(s, "window (handle exchange)"));
            peers.assign(n_, nullptr);
            peers[rank_] = base;
            for (int j = 0; j < n_ && ok; ++j) {
                if (j == rank_) continue;
                void* p = nullptr;
                if (hipIpcOpenMemHandle(&p, all[j], hipIpcMemLazyEnablePeerAccess) != hipSuccess) ok = false;
                peers[j] = static_cast<char*>(p);
            }
            int* f = reinterpret_cast<int*>(d + (n_ + 1) * H);
            const int mine_ok = ok ? 1 : 0;
            FMI_COMM_HIP(hipMemcpyAsync(f, &mine_ok, sizeof(int), hipMemcpyHostToDevice, s));
            FMI_RCCL(AllReduce(f, f + 1, 1, ncclInt32, ncclMin, comm_, s));
            FMI_COMM_HIP(hipMemcpyAsync(&flag, f + 1, sizeof(int), hipMemcpyDeviceToHost, s));
            FMI_COMM_RC(wait_stream(s, "window (map result)"));
            return FMI_OK;
        }();
        if (!aborted_) (void)hipFree(d);  // after an abort the stream may not have drained: leak, never free in use
        if (rc != FMI_OK || flag != 1) {
            unmap_window(peers);
            peers.clear();
            return rc != FMI_OK ? rc : fail(FMI_ERR_COMM, "window: a rank could not export or map its window (IPC)");
        }
        return FMI_OK;
    }
    void unmap_window(const std::vector<char*>& peers) override {
        for (int j = 0; j < static_cast<int>(peers.size()); ++j)
            if (j != rank_ && peers[j]) (void)hipIpcCloseMemHandle(peers[j]);
    }
    // The second communicator is made like the first: rank 0 draws a fresh id, this communicator broadcasts
    // it on s, every rank joins it (non-blocking init bounded by the timeout when this one is non-blocking).
    // Not ncclCommSplit: with a non-blocking parent the child's handle is published asynchronously, and the
    // librccl torch ships (2.26) handed back a handle that was not valid yet (ncclCommGetAsyncError: invalid
    // argument), with the library's pointer to it written later by RCCL's own thread.
    int split(std::unique_ptr<Transport>* out, hipStream_t s) override {
        ncclUniqueId id{};
        if (rank_ == 0) FMI_RCCL(GetUniqueId(&id));
        char* d = nullptr;
        FMI_COMM_HIP(hipMalloc(&d, sizeof(id)));
        const int rc = [&]() -> int {
            FMI_COMM_HIP(hipMemcpyAsync(d, &id, sizeof(id), hipMemcpyHostToDevice, s));
            FMI_RCCL(Broadcast(d, d, sizeof(id), ncclUint8, 0, comm_, s));
            FMI_COMM_HIP(hipMemcpyAsync(&id, d, sizeof(id), hipMemcpyDeviceToHost, s));
            return wait_stream(s, "second communicator (id broadcast)");
        }();
        if (!aborted_) (void)hipFree(d);
        FMI_COMM_RC(rc);
        ncclComm_t nc = nullptr;
        if (nonblocking_) {
            ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
            cfg.blocking = 0;
            const ncclResult_t r = api_->CommInitRankConfig(&nc, n_, id, rank_, &cfg);
            if (r != ncclSuccess && r != ncclInProgress) return nccl_fail(api_, "ncclCommInitRankConfig (second)", r);
        } else {
            FMI_NCCL(api_, CommInitRank(&nc, n_, id, rank_));
        }
        auto child = std::make_unique<RcclTransport>(api_, nc, n_, rank_, nonblocking_);
        child->set_timeout(timeout_s_);
        FMI_COMM_RC(child->wait_ready("ncclCommInitRankConfig (second communicator)"));
        *out = std::move(child);
        return FMI_OK;
    }
    int agree_max(int64_t* vals, int k, hipStream_t s) override {
        int64_t* d = nullptr;
        FMI_COMM_HIP(hipMalloc(&d, kAgreeMax * sizeof(int64_t)));
        const int rc = [&]() -> int {
            FMI_COMM_HIP(hipMemcpyAsync(d, vals, k * sizeof(int64_t), hipMemcpyHostToDevice, s));
            FMI_RCCL(AllReduce(d, d, k, ncclInt64, ncclMax, comm_, s));
            FMI_COMM_HIP(hipMemcpyAsync(vals, d, k * sizeof(int64_t), hipMemcpyDeviceToHost, s));
            return wait_stream(s, "agree");
        }();
        if (!aborted_) (void)hipFree(d);
        return rc;
    }

private:
    int ck(ncclResult_t r, const char* what) {
        if (r == ncclSuccess) return FMI_OK;
        if (r == ncclInProgress) return wait_ready(what);
        return nccl_fail(api_, what, r);
    }

    // One group of the plan's sends and receives (RCCL pairs them per peer in posting order), then the
    // local part on the stream.
    int run_plan(const plan::Plan& p, const char* send, char* recv, hipStream_t s) {
        if (!p.sends.empty() || !p.recvs.empty()) {
            FMI_RCCL(GroupStart());
            int rc = FMI_OK;
            for (size_t i = 0; i < p.sends.size() && rc == FMI_OK; ++i) {
                const plan::Xfer& x = p.sends[i];
                rc = ck(api_->Send(send + x.off, x.len, ncclUint8, x.peer, comm_, s), "Send");
            }
            for (size_t i = 0; i < p.recvs.size() && rc == FMI_OK; ++i) {
                const plan::Xfer& x = p.recvs[i];
                rc = ck(api_->Recv(recv + x.off, x.len, ncclUint8, x.peer, comm_, s), "Recv");
            }
            // the group is closed even after a failed post, so this thread's later RCCL calls are not grouped
            const int end = ck(api_->GroupEnd(), "GroupEnd");
            FMI_COMM_RC(rc);
            FMI_COMM_RC(end);
        }
        if (p.copy_len && recv + p.copy_dst != send + p.copy_src)
            FMI_COMM_RC(device_copy(recv + p.copy_dst, send + p.copy_src, p.copy_len, s));
        return FMI_OK;
    }
    const RcclApi* api_;
    ncclComm_t comm_;
    bool nonblocking_;
    void* token_ = nullptr;
};

// Ranks of one process on one device: a rendezvous hub per communicator id.
struct Hub {
    explicit Hub(int n) : n(n), ptrs(n, nullptr) {}
    ~Hub() {
        // A poisoned hub's ranks may have left copies queued that never drain: leak the streams then.
        if (!poisoned)
            for (hipStream_t st : {h2d, d2h})
                if (st) (void)hipStreamDestroy(st);
    }
    int n;
    // The host pipelines' copy streams, shared by this communicator's ranks only (LocalTransport::copy_streams).
    hipStream_t h2d = nullptr, d2h = nullptr;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t generation = 0;
    std::vector<const char*> ptrs;
    struct Msg {
        const char* buf;
        size_t bytes;
        bool done;
    };
    std::map<std::pair<int, int>, std::deque<Msg*>> box;
    // Set when any rank's wait on the hub times out. A timed-out rank has left its barrier (its arrival
    // withdrawn) and may free the buffer it published: no later barrier, exchange or mailbox wait of this hub
    // may complete and read it, so every one of them fails as a timeout instead (the communicator is aborted).
    bool poisoned = false;

    // false: not every rank arrived before the deadline, or the hub is poisoned
    bool barrier(Clock::time_point deadline) {
        std::unique_lock<std::mutex> lk(mu);
        if (poisoned) return false;
        const uint64_t g = generation;
        if (++arrived == n) {
            arrived = 0;
            ++generation;
            cv.notify_all();
            return true;
        }
        if (cv.wait_until(lk, deadline, [&] { return generation != g || poisoned; }) && generation != g) return true;
        if (generation == g) --arrived;  // withdraw: this rank no longer waits in this barrier
        poison_locked();
        return false;
    }
    void poison_locked() {
        poisoned = true;
        cv.notify_all();
    }
};

std::mutex g_hub_mu;
std::map<uint64_t, std::weak_ptr<Hub>> g_hubs;
std::atomic<uint64_t> g_hub_counter{1};
constexpr char kLocalMagic[8] = {'F', 'M', 'I', 'L', 'O', 'C', 'A', 'L'};

class LocalTransport final : public Transport {
public:
    LocalTransport(std::shared_ptr<Hub> hub, int n, int rank) : Transport(n, rank), hub_(std::move(hub)) {}

    bool co_resident() const override { return n_ > 1; }  // the ranks are threads sharing this device
    int copy_streams(hipStream_t* h2d, hipStream_t* d2h) override {
        std::lock_guard<std::mutex> lk(hub_->mu);
        for (hipStream_t* st : {&hub_->h2d, &hub_->d2h})
            if (!*st) FMI_COMM_HIP(hipStreamCreateWithFlags(st, hipStreamNonBlocking));
        *h2d = hub_->h2d;
        *d2h = hub_->d2h;
        return FMI_OK;
    }

    // Every exchange below runs the RCCL transport's own plan (fmi_exchange_plan.h): each receive copies
    // from the matching send of the peer's plan (same peer order, same length, or the call fails), so the
    // LOCAL ranks of the GPU tests exercise the pairings RCCL is given between GPUs.
    int all_to_all(const char* send, char* recv, size_t bytes, hipStream_t s) override {
        return run_plan([&](int r) { return plan::all_to_all(n_, r, bytes); }, send, recv, s);
    }
    bool receives_per_peer() const override { return true; }
    int all_to_all_strided(const char* send, char* recv, size_t bytes, size_t stride, hipStream_t s) override {
        return run_plan([&](int r) { return plan::all_to_all(n_, r, bytes, stride); }, send, recv, s);
    }
    int all_gather(const char* send, char* recv, size_t bytes, hipStream_t s) override {
        return run_plan([&](int r) { return plan::all_gather(n_, r, bytes); }, send, recv, s);
    }
    bool ragged() const override { return true; }
    int all_to_all_ragged(const char* send, char* recv, size_t shard, size_t total, hipStream_t s) override {
        return run_plan([&](int r) { return plan::all_to_all_ragged(n_, r, shard, total); }, send, recv, s);
    }
    int all_gather_ragged(const char* send, char* recv, size_t shard, size_t total, hipStream_t s) override {
        return run_plan([&](int r) { return plan::all_gather_ragged(n_, r, shard, total); }, send, recv, s);
    }
    int gather_ragged(const char* send, char* recv, size_t shard, size_t total, int root, hipStream_t s) override {
        return run_plan([&](int r) { return plan::gather_ragged(n_, r, shard, total, root); }, send, recv, s);
    }
    int all_to_all_back_ragged(const char* send, char* recv, size_t shard, size_t total, hipStream_t s) override {
        return run_plan([&](int r) { return plan::all_to_all_back_ragged(n_, r, shard, total); }, send, recv, s);
    }
    int gather(const char* send, char* recv, size_t bytes, int root, hipStream_t s) override {
        return run_plan([&](int r) { return plan::gather(n_, r, bytes, root); }, send, recv, s);
    }
    int scatter(const char* send, char* recv, size_t bytes, int root, hipStream_t s) override {
        return run_plan([&](int r) { return plan::scatter(n_, r, bytes, root); }, send, recv, s);
    }
    int bcast(char* buf, size_t bytes, int root, hipStream_t s) override {
        return exchange(buf, s, [&](const std::vector<const char*>& all) -> int {
            if (rank_ != root && bytes) FMI_COMM_RC(device_copy(buf, all[root], bytes, s));
            return FMI_OK;
        });
    }
    int send(const char* buf, size_t bytes, int peer, hipStream_t s) override {
        FMI_COMM_HIP(hipStreamSynchronize(s));
        Hub::Msg msg{buf, bytes, false};
        std::unique_lock<std::mutex> lk(hub_->mu);
        auto& q = hub_->box[{rank_, peer}];
        q.push_back(&msg);
        hub_->cv.notify_all();
        // rendezvous: the receiver has copied it
        if (!hub_->cv.wait_until(lk, deadline(), [&] { return msg.done || hub_->poisoned; }) || !msg.done) {
            const auto it = std::find(q.begin(), q.end(), &msg);
            if (it == q.end()) {  // the receiver took it and is copying: it is alive, let it finish
                hub_->cv.wait(lk, [&] { return msg.done; });
                return FMI_OK;
            }
            q.erase(it);  // never leave a pointer to this frame behind
            hub_->poison_locked();
            lk.unlock();
            return timed_out("local transport send to rank " + std::to_string(peer));
        }
        return FMI_OK;
    }
    int recv(char* buf, size_t bytes, int peer, hipStream_t s) override {
        Hub::Msg* msg = nullptr;
        {
            std::unique_lock<std::mutex> lk(hub_->mu);
            auto& q = hub_->box[{peer, rank_}];
            if (!hub_->cv.wait_until(lk, deadline(), [&] { return !q.empty() || hub_->poisoned; }) || q.empty()) {
                hub_->poison_locked();
                lk.unlock();
                return timed_out("local transport recv from rank " + std::to_string(peer));
            }
            msg = q.front();
            q.pop_front();
        }
        int rc = FMI_OK;
        if (msg->bytes != bytes) {
            rc = fail(FMI_ERR_COMM, "local transport: message of " + std::to_string(msg->bytes) + " bytes, expected " +
                                        std::to_string(bytes));
        } else if (bytes) {
            rc = device_copy(buf, msg->buf, bytes, s);
            if (rc == FMI_OK) {
                const hipError_t e = hipStreamSynchronize(s);
                if (e != hipSuccess) rc = hip_err("local transport recv", e);
            }
        }
        std::lock_guard<std::mutex> lk(hub_->mu);
        msg->done = true;
        hub_->cv.notify_all();
        return rc;
    }
    int barrier(hipStream_t s) override {
        FMI_COMM_HIP(hipStreamSynchronize(s));
        if (!hub_->barrier(deadline())) return timed_out("local transport barrier");
        return FMI_OK;
    }
    int barrier_async(hipStream_t s) override { return barrier(s); }
    // Ranks share the process and the device: the window pointers themselves are the mapping.
    int map_window(char* base, bool ok, std::vector<char*>& peers, hipStream_t s) override {
        bool all_ok = true;
        const int rc = exchange(ok ? base : nullptr, s, [&](const std::vector<const char*>& all) -> int {
            peers.assign(n_, nullptr);
            for (int j = 0; j < n_; ++j) {
                peers[j] = const_cast<char*>(all[j]);
                if (!all[j]) all_ok = false;
            }
            return FMI_OK;
        });
        if (rc != FMI_OK) return rc;
        if (!all_ok) {
            peers.clear();
            return fail(FMI_ERR_ALLOC, "window: a rank could not allocate its window");
        }
        return FMI_OK;
    }
    void unmap_window(const std::vector<char*>&) override {}
    int agree_max(int64_t* vals, int k, hipStream_t s) override {
        int64_t out[kAgreeMax];
        const int rc = exchange(reinterpret_cast<const char*>(vals), s, [&](const std::vector<const char*>& all) -> int {
            for (int i = 0; i < k; ++i) {
                out[i] = reinterpret_cast<const int64_t*>(all[0])[i];
                for (int j = 1; j < n_; ++j) out[i] = std::max(out[i], reinterpret_cast<const int64_t*>(all[j])[i]);
            }
            return FMI_OK;
        });
        if (rc == FMI_OK) std::copy(out, out + k, vals);  // after the closing barrier: every rank has read
        return rc;
    }

private:
    // Execute plan_of(rank_) against the published buffers: my k-th receive from peer j copies from the k-th
    // send to me in plan_of(j); a receive without a send of its length fails (RCCL would hang on it).
    template <class PlanOf>
    int run_plan(PlanOf&& plan_of, const char* send, char* recv, hipStream_t s) {
        const plan::Plan mine = plan_of(rank_);
        return exchange(send, s, [&](const std::vector<const char*>& all) -> int {
            std::vector<plan::Plan> peer(n_);
            std::vector<char> built(n_, 0);
            std::vector<size_t> next(n_, 0);  // per peer: where to look for its next send to me
            for (const plan::Xfer& r : mine.recvs) {
                const int j = r.peer;
                if (!built[j]) {
                    peer[j] = plan_of(j);
                    built[j] = 1;
                }
                const std::vector<plan::Xfer>& sends = peer[j].sends;
                size_t& k = next[j];
                while (k < sends.size() && sends[k].peer != rank_) ++k;
                if (k == sends.size() || sends[k].len != r.len)
                    return fail(FMI_ERR_COMM, "exchange plan: rank " + std::to_string(j) + " posts no send of " +
                                                  std::to_string(r.len) + " B to rank " + std::to_string(rank_));
                FMI_COMM_RC(device_copy(recv + r.off, all[j] + sends[k].off, r.len, s));
                ++k;
            }
            if (mine.copy_len && recv + mine.copy_dst != send + mine.copy_src)
                FMI_COMM_RC(device_copy(recv + mine.copy_dst, send + mine.copy_src, mine.copy_len, s));
            return FMI_OK;
        });
    }

    // Publish my buffer, wait for everyone, run `work` over all ranks' buffers, wait until everyone's
    // copies have completed (so no rank reuses a published buffer while another still reads it).
    int exchange(const char* mine, hipStream_t s, const std::function<int(const std::vector<const char*>&)>& work) {
        FMI_COMM_HIP(hipStreamSynchronize(s));
        {
            std::lock_guard<std::mutex> lk(hub_->mu);
            hub_->ptrs[rank_] = mine;
        }
        if (!hub_->barrier(deadline())) return timed_out("local transport exchange (published)");
        std::vector<const char*> all;
        {
            std::lock_guard<std::mutex> lk(hub_->mu);
            all = hub_->ptrs;
        }
        int rc = work(all);
        const hipError_t e = hipStreamSynchronize(s);
        if (!hub_->barrier(deadline())) return timed_out("local transport exchange (consumed)");
        if (rc == FMI_OK && e != hipSuccess) rc = hip_err("local transport exchange", e);
        return rc;
    }

    Clock::time_point deadline() const {
        return Clock::now() + std::chrono::duration_cast<Clock::duration>(std::chrono::duration<double>(timeout_s_));
    }

    std::shared_ptr<Hub> hub_;
};

// ---------------------------------------------------------------------------------------------------
// PROC: ranks are processes of one node. One POSIX shared-memory segment per communicator holds a control
// block (barrier, point-to-point mailboxes, window IPC handles) and one staging slot per rank, page-locked
// in every process so the slots move at DMA rate. Every exchange is: write my part into my slot, barrier,
// read the parts I need from the peers' slots, barrier — in pieces of the slot size.
// ---------------------------------------------------------------------------------------------------
constexpr char kProcMagic[8] = {'F', 'M', 'I', 'P', 'R', 'O', 'C', '\0'};
constexpr int kProcMaxRanks = 64;
constexpr size_t kProcSlot = size_t(32) << 20;
constexpr size_t kProcCtrlBytes = size_t(64) << 10;

struct ProcCtrl {  // lives in the shared segment; all-zero is the initial state
    std::atomic<uint64_t> arrived;
    std::atomic<uint64_t> generation;
    // set by a rank whose wait for the peers timed out: its arrival may still be counted and its slot may be
    // stale, so no later barrier or mailbox wait of any rank may complete on it (the LOCAL hub's rule)
    std::atomic<int> poisoned;
    struct Mail {  // what rank src's slot holds for point-to-point: a message for `dst` until ack == seq
        std::atomic<int> dst;
        std::atomic<uint64_t> bytes;
        std::atomic<uint64_t> seq;
        std::atomic<uint64_t> ack;
    } mail[kProcMaxRanks];
    hipIpcMemHandle_t handle[kProcMaxRanks];
    std::atomic<int> ok[kProcMaxRanks];
    int64_t agree[kProcMaxRanks][4];  // Transport::agree_max inputs, one row per rank
};
static_assert(sizeof(ProcCtrl) <= kProcCtrlBytes, "control block");

std::string proc_shm_name(const void* id) {
    uint64_t key;
    std::memcpy(&key, static_cast<const char*>(id) + 8, 8);
    char name[64];
    std::snprintf(name, sizeof(name), "/fmi_proc_%016llx", static_cast<unsigned long long>(key));
    return name;
}

class ProcTransport final : public Transport {
public:
    ProcTransport(int n, int rank) : Transport(n, rank) {}
    ~ProcTransport() override {
        if (registered_) (void)hipHostUnregister(base_);
        if (base_) munmap(base_, bytes_);
        if (fd_ >= 0) close(fd_);
        if (!unlinked_ && !name_.empty()) shm_unlink(name_.c_str());
    }

    // Collective: map the segment, then a barrier; rank 0 unlinks the name once everyone holds it.
    int join(const void* id) {
        if (n_ > kProcMaxRanks) return fail(FMI_ERR_INVALID, "PROC transport: at most 64 ranks");
        name_ = proc_shm_name(id);
        bytes_ = kProcCtrlBytes + static_cast<size_t>(n_) * kProcSlot;
        fd_ = shm_open(name_.c_str(), O_CREAT | O_RDWR, 0600);
        if (fd_ < 0) return fail(FMI_ERR_COMM, "shm_open(" + name_ + "): " + std::strerror(errno));
        struct stat st{};
        if (fstat(fd_, &st) != 0) return fail(FMI_ERR_COMM, std::string("fstat: ") + std::strerror(errno));
        if (st.st_size != 0 && static_cast<size_t>(st.st_size) != bytes_)
            return fail(FMI_ERR_INVALID, "PROC communicator joined with a different size");
        if (st.st_size == 0 && ftruncate(fd_, static_cast<off_t>(bytes_)) != 0)
            return fail(FMI_ERR_COMM, std::string("ftruncate: ") + std::strerror(errno));
        void* m = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd_, 0);
        if (m == MAP_FAILED) return fail(FMI_ERR_COMM, std::string("mmap: ") + std::strerror(errno));
        base_ = static_cast<char*>(m);
        ctrl_ = reinterpret_cast<ProcCtrl*>(base_);
        if (int rc = host_barrier("join")) return rc;
        if (rank_ == 0) shm_unlink(name_.c_str());
        unlinked_ = true;
        return FMI_OK;
    }

    int all_to_all(const char* send, char* recv, size_t bytes, hipStream_t s) override {
        return all_to_all_strided(send, recv, bytes, bytes, s);
    }
    bool receives_per_peer() const override { return true; }
    int all_to_all_strided(const char* send, char* recv, size_t bytes, size_t stride, hipStream_t s) override {
        const size_t c = std::max<size_t>(1, kProcSlot / static_cast<size_t>(n_));
        return pieces(bytes, c, s,
                      [&](size_t o, size_t len) -> int {
                          for (int d = 0; d < n_; ++d)
                              FMI_COMM_HIP(hipMemcpyAsync(slot(rank_) + d * c, send + d * bytes + o, len, hipMemcpyDeviceToHost, s));
                          return FMI_OK;
                      },
                      [&](size_t o, size_t len) -> int {
                          for (int j = 0; j < n_; ++j)
                              FMI_COMM_HIP(hipMemcpyAsync(recv + j * stride + o, slot(j) + rank_ * c, len, hipMemcpyHostToDevice, s));
                          return FMI_OK;
                      });
    }
    int all_gather(const char* send, char* recv, size_t bytes, hipStream_t s) override {
        return gather_to(send, recv, bytes, -1, s);
    }
    int gather(const char* send, char* recv, size_t bytes, int root, hipStream_t s) override {
        return gather_to(send, recv, bytes, root, s);
    }
    int scatter(const char* send, char* recv, size_t bytes, int root, hipStream_t s) override {
        const size_t c = std::max<size_t>(1, kProcSlot / static_cast<size_t>(n_));
        return pieces(bytes, c, s,
                      [&](size_t o, size_t len) -> int {
                          if (rank_ != root) return FMI_OK;
                          for (int d = 0; d < n_; ++d)
                              FMI_COMM_HIP(hipMemcpyAsync(slot(root) + d * c, send + d * bytes + o, len, hipMemcpyDeviceToHost, s));
                          return FMI_OK;
                      },
                      [&](size_t o, size_t len) -> int {
                          FMI_COMM_HIP(hipMemcpyAsync(recv + o, slot(root) + rank_ * c, len, hipMemcpyHostToDevice, s));
                          return FMI_OK;
                      });
    }
    int bcast(char* buf, size_t bytes, int root, hipStream_t s) override {
        return pieces(bytes, kProcSlot, s,
                      [&](size_t o, size_t len) -> int {
                          if (rank_ == root) FMI_COMM_HIP(hipMemcpyAsync(slot(root), buf + o, len, hipMemcpyDeviceToHost, s));
                          return FMI_OK;
                      },
                      [&](size_t o, size_t len) -> int {
                          if (rank_ != root) FMI_COMM_HIP(hipMemcpyAsync(buf + o, slot(root), len, hipMemcpyHostToDevice, s));
                          return FMI_OK;
                      });
    }
    // Rendezvous point-to-point through the sender's slot: one message in flight per sender, consumed
    // (ack == seq) before the next is written.
    int send(const char* buf, size_t bytes, int peer, hipStream_t s) override {
        FMI_COMM_RC(ensure_registered());
        auto& m = ctrl_->mail[rank_];
        size_t o = 0;
        do {
            const size_t len = std::min(kProcSlot, bytes - o);
            FMI_COMM_RC(wait_until([&] { return m.ack.load(std::memory_order_acquire) == m.seq.load(std::memory_order_acquire); }, "send"));
            if (len) {
                FMI_COMM_HIP(hipMemcpyAsync(slot(rank_), buf + o, len, hipMemcpyDeviceToHost, s));
                FMI_COMM_HIP(hipStreamSynchronize(s));
            }
            m.dst.store(peer, std::memory_order_relaxed);
            m.bytes.store(len, std::memory_order_relaxed);
            const uint64_t seq = m.seq.fetch_add(1, std::memory_order_acq_rel) + 1;
            FMI_COMM_RC(wait_until([&] { return m.ack.load(std::memory_order_acquire) == seq; }, "send (ack)"));
            o += len;
        } while (o < bytes);
        return FMI_OK;
    }
    int recv(char* buf, size_t bytes, int peer, hipStream_t s) override {
        FMI_COMM_RC(ensure_registered());
        auto& m = ctrl_->mail[peer];
        size_t o = 0;
        do {
            FMI_COMM_RC(wait_until([&] {
                return m.dst.load(std::memory_order_acquire) == rank_ &&
                       m.seq.load(std::memory_order_acquire) != m.ack.load(std::memory_order_acquire);
            }, "recv"));
            const size_t len = m.bytes.load(std::memory_order_relaxed);
            if (o + len > bytes) return fail(FMI_ERR_COMM, "PROC transport: message longer than the receive buffer");
            if (len) {
                FMI_COMM_HIP(hipMemcpyAsync(buf + o, slot(peer), len, hipMemcpyHostToDevice, s));
                FMI_COMM_HIP(hipStreamSynchronize(s));
            }
            m.ack.store(m.seq.load(std::memory_order_acquire), std::memory_order_release);
            o += len;
        } while (o < bytes);
        return FMI_OK;
    }
    int barrier(hipStream_t s) override {
        FMI_COMM_HIP(hipStreamSynchronize(s));
        return host_barrier("barrier");
    }
    int barrier_async(hipStream_t s) override { return barrier(s); }
    // HIP IPC handles through the control block; all-or-nothing like the RCCL transport's.
    int map_window(char* base, bool ok, std::vector<char*>& peers, hipStream_t s) override {
        FMI_COMM_HIP(hipStreamSynchronize(s));
        hipIpcMemHandle_t mine{};
        if (ok) ok = hipIpcGetMemHandle(&mine, base) == hipSuccess;
        ctrl_->handle[rank_] = mine;
        ctrl_->ok[rank_].store(ok ? 1 : 0, std::memory_order_release);
        FMI_COMM_RC(host_barrier("window (export)"));
        bool all = true;
        for (int j = 0; j < n_; ++j) all = all && ctrl_->ok[j].load(std::memory_order_acquire) == 1;
        peers.assign(n_, nullptr);
        peers[rank_] = base;
        bool opened = all;
        for (int j = 0; j < n_ && opened; ++j) {
            if (j == rank_) continue;
            void* p = nullptr;
            if (hipIpcOpenMemHandle(&p, ctrl_->handle[j], hipIpcMemLazyEnablePeerAccess) != hipSuccess) opened = false;
            peers[j] = static_cast<char*>(p);
        }
        FMI_COMM_RC(host_barrier("window (flags read)"));
        ctrl_->ok[rank_].store(opened ? 1 : 0, std::memory_order_release);
        FMI_COMM_RC(host_barrier("window (map)"));
        for (int j = 0; j < n_; ++j) opened = opened && ctrl_->ok[j].load(std::memory_order_acquire) == 1;
        FMI_COMM_RC(host_barrier("window (result read)"));
        if (!opened) {
            unmap_window(peers);
            peers.clear();
            return fail(FMI_ERR_COMM, "window: a rank could not export or map its window (IPC)");
        }
        return FMI_OK;
    }
    void unmap_window(const std::vector<char*>& peers) override {
        for (int j = 0; j < static_cast<int>(peers.size()); ++j)
            if (j != rank_ && peers[j]) (void)hipIpcCloseMemHandle(peers[j]);
    }
    int agree_max(int64_t* vals, int k, hipStream_t s) override {
        FMI_COMM_HIP(hipStreamSynchronize(s));
        std::copy(vals, vals + k, ctrl_->agree[rank_]);
        FMI_COMM_RC(host_barrier("agree (published)"));
        for (int i = 0; i < k; ++i)
            for (int j = 0; j < n_; ++j) vals[i] = std::max(vals[i], ctrl_->agree[j][i]);
        return host_barrier("agree (read)");
    }

private:
    char* slot(int r) const { return base_ + kProcCtrlBytes + static_cast<size_t>(r) * kProcSlot; }

    int ensure_registered() {
        if (registered_) return FMI_OK;
        FMI_COMM_HIP(hipHostRegister(base_ + kProcCtrlBytes, bytes_ - kProcCtrlBytes, hipHostRegisterDefault));
        registered_ = true;
        return FMI_OK;
    }

    // Split `bytes` per destination into pieces of `c`; each piece: write(o, len), sync, barrier,
    // read(o, len), sync, barrier (the second barrier frees the slots for the next piece).
    template <class W, class Rd>
    int pieces(size_t bytes, size_t c, hipStream_t s, W&& write, Rd&& read) {
        FMI_COMM_RC(ensure_registered());
        FMI_COMM_HIP(hipStreamSynchronize(s));
        for (size_t o = 0; o < bytes; o += c) {
            const size_t len = std::min(c, bytes - o);
            FMI_COMM_RC(write(o, len));
            FMI_COMM_HIP(hipStreamSynchronize(s));
            FMI_COMM_RC(host_barrier("exchange (published)"));
            FMI_COMM_RC(read(o, len));
            FMI_COMM_HIP(hipStreamSynchronize(s));
            FMI_COMM_RC(host_barrier("exchange (consumed)"));
        }
        return FMI_OK;
    }

    int gather_to(const char* send, char* recv, size_t bytes, int root, hipStream_t s) {
        return pieces(bytes, kProcSlot, s,
                      [&](size_t o, size_t len) -> int {
                          FMI_COMM_HIP(hipMemcpyAsync(slot(rank_), send + o, len, hipMemcpyDeviceToHost, s));
                          return FMI_OK;
                      },
                      [&](size_t o, size_t len) -> int {
                          if (root >= 0 && rank_ != root) return FMI_OK;
                          for (int j = 0; j < n_; ++j)
                              FMI_COMM_HIP(hipMemcpyAsync(recv + j * bytes + o, slot(j), len, hipMemcpyHostToDevice, s));
                          return FMI_OK;
                      });
    }

    int host_barrier(const char* what) {
        if (ctrl_->poisoned.load(std::memory_order_acquire))
            return timed_out(std::string("PROC transport: a peer timed out earlier (") + what + ")");
        const uint64_t g = ctrl_->generation.load(std::memory_order_acquire);
        if (ctrl_->arrived.fetch_add(1, std::memory_order_acq_rel) + 1 == static_cast<uint64_t>(n_)) {
            ctrl_->arrived.store(0, std::memory_order_relaxed);
            ctrl_->generation.fetch_add(1, std::memory_order_acq_rel);
            return FMI_OK;
        }
        return wait_until([&] { return ctrl_->generation.load(std::memory_order_acquire) != g; }, what);
    }

    // Spin, then back off to short sleeps; give up after the communicator's timeout (FMI_COMM_TIMEOUT_S /
    // FMI_PROC_TIMEOUT_S, default 300 s) so a dead peer surfaces as FMI_ERR_TIMEOUT instead of a hang.
    template <class Pred>
    int wait_until(Pred&& ready, const char* what) {
        const auto t0 = Clock::now();
        for (int k = 0; !ready(); ++k) {
            backoff(k);
            if (k >= 1000 && (k & 255) == 0) {
                if (ctrl_->poisoned.load(std::memory_order_acquire))
                    return timed_out(std::string("PROC transport: a peer timed out (") + what + ")");
                if (std::chrono::duration<double>(Clock::now() - t0).count() > timeout_s_) {
                    ctrl_->poisoned.store(1, std::memory_order_release);
                    return timed_out(std::string("PROC transport: waiting for peers (") + what + ")");
                }
            }
        }
        return FMI_OK;
    }

    std::string name_;
    int fd_ = -1;
    char* base_ = nullptr;
    size_t bytes_ = 0;
    ProcCtrl* ctrl_ = nullptr;
    bool registered_ = false;
    bool unlinked_ = false;
};

// ---------------------------------------------------------------------------------------------------
// communicator
// ---------------------------------------------------------------------------------------------------
// Streams and events of the host-ingress pipeline (fmi_comm_allreduce_host), created on first use: the chunk's
// sharded allreduce runs on the communicator's own stream, the copies on one H2D and one D2H stream.
//
// Whose copy streams. The runtime hands its DMA engines to streams: with one stream per direction the two
// directions run on separate engines at the link's duplex rate (1 GiB each way in 22.4 ms, 96 GB/s); with a pair per
// co-resident LOCAL rank (8 ranks, 16 copy streams) the directions land on shared engines and serialise, 178-241 ms
// for 8 GiB each way depending on the streams the runtime had handed out before, against 178.0 ms on one shared pair
// every time (profiles/r05_pcie_peers.jsonl, tools/microbench_pcie_peers.hip). So the co-resident ranks of ONE
// communicator share one pair (Transport::copy_streams, owned by their hub): each rank's order is kept by its own
// events, and their chunks interleave in the order their threads issue them, which the LOCAL rendezvous of every
// chunk keeps rank-major per chunk. Nothing wider shares a pair: two communicators whose loads waited
// on each other's device events in one shared stream could be queued X-then-Y in one process and Y-then-X in
// another and deadlock across processes, and an aborted communicator's undrained copies would block every later
// one. Every other communicator's pipeline (one rank per device: RCCL, PROC, one-rank LOCAL) owns its pair.
struct HostPipe {
    // Chunk slots in flight: the load of chunk k waits for the allreduce of chunk k - depth. One rank per device: 2 —
    // the wait paces the loads to the results draining, and the two directions stay overlapped (a 1 GiB one-rank
    // pipeline 23.2-24.3 ms at 2, 32.7-33.0 ms at 3). Co-resident ranks sharing their copy streams: 3 — one rank's
    // load waiting for its allreduce of chunk k - 2 would hold every other rank's loads behind it on the shared
    // stream, and at depth 3 that wait is long finished when the load is queued (8 ranks x 1 GiB: 203-204 ms at 3,
    // 217-240 ms at 2; profiles/r05_depth_ab.jsonl).
    static constexpr int kDepth = 3;  // slots allocated
    hipStream_t cs = nullptr;   // the chunk's sharded allreduce (this communicator's own)
    hipStream_t h2d = nullptr;  // host -> device loads
    hipStream_t d2h = nullptr;  // device -> host results
    bool owns_copy_streams = false;  // false: the co-resident ranks' pair (their hub owns it)
    hipEvent_t loaded[kDepth] = {}, reduced[kDepth] = {}, drained[kDepth] = {};
    bool ready = false;

    int depth() const { return owns_copy_streams ? 2 : kDepth; }

    int init(Transport& t) {
        if (ready) return FMI_OK;
        if (!h2d || !d2h) {  // (a failed creation is retried on the next call)
            if (t.co_resident()) {
                FMI_COMM_RC(t.copy_streams(&h2d, &d2h));
            } else {
                owns_copy_streams = true;
                for (hipStream_t* st : {&h2d, &d2h})
                    if (!*st) FMI_COMM_HIP(hipStreamCreateWithFlags(st, hipStreamNonBlocking));
            }
        }
        if (!cs) FMI_COMM_HIP(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
        for (int k = 0; k < kDepth; ++k)
            for (hipEvent_t* ev : {&loaded[k], &reduced[k], &drained[k]})
                if (!*ev) FMI_COMM_HIP(hipEventCreateWithFlags(ev, hipEventDisableTiming));
        ready = true;
        return FMI_OK;
    }
    ~HostPipe() {
        if (cs) (void)hipStreamDestroy(cs);
        if (owns_copy_streams)
            for (hipStream_t st : {h2d, d2h})
                if (st) (void)hipStreamDestroy(st);
        for (int k = 0; k < kDepth; ++k)
            for (hipEvent_t ev : {loaded[k], reduced[k], drained[k]})
                if (ev) (void)hipEventDestroy(ev);
    }
};

// A symmetric window (fmi_comm_window_alloc): 2 * bytes per rank — the caller's bucket area [0, bytes)
// and the reduced-shard area [bytes, 2 * bytes) — mapped into every rank's address space.
struct Window {
    size_t bytes = 0;
    std::vector<char*> peers;  // peers[j] = rank j's window base, as seen from this rank
    char** shards = nullptr;   // device table: peers[j] + bytes (rank j's reduced-shard area), any N
};

// Streams, events and the second transport of the pipelined allreduce (FMI_TUNE_COMM_PIPELINE).
struct ChunkPipe {
    std::unique_ptr<Transport> t2;  // nullptr with LOCAL / PROC: their exchanges are host-synchronous
    bool split_done = false;
    bool no_split = false;  // the transport could not make a second communicator: never pipeline
    hipStream_t gs = nullptr;  // all-gathers
    hipEvent_t reduced[2] = {}, gathered[2] = {}, start = nullptr;
    bool ready = false;

    int init(Transport* t, hipStream_t s) {
        if (!split_done) {
            const int rc = t->split(&t2, s);
            if (rc == FMI_ERR_UNSUPPORTED) no_split = true;  // every rank loads the same librccl: all fall back
            if (rc != FMI_OK) return rc;
            split_done = true;
        }
        if (ready) return FMI_OK;
        FMI_COMM_HIP(hipStreamCreateWithFlags(&gs, hipStreamNonBlocking));
        for (int k = 0; k < 2; ++k)
            for (hipEvent_t* ev : {&reduced[k], &gathered[k]}) FMI_COMM_HIP(hipEventCreateWithFlags(ev, hipEventDisableTiming));
        FMI_COMM_HIP(hipEventCreateWithFlags(&start, hipEventDisableTiming));
        ready = true;
        return FMI_OK;
    }
    ~ChunkPipe() {
        if (gs) {
            (void)hipStreamSynchronize(gs);
            (void)hipStreamDestroy(gs);
        }
        for (int k = 0; k < 2; ++k)
            for (hipEvent_t ev : {reduced[k], gathered[k]})
                if (ev) (void)hipEventDestroy(ev);
        if (start) (void)hipEventDestroy(start);
    }
};

// Live timing of the shard kernels (fmi_comm_timing): an event pair around every shard-kernel launch of the
// collectives, on the stream the kernel runs on, read back as a total by fmi_comm_timing_read.
struct KernelTiming {
    static constexpr size_t kMaxPairs = 8192;
    bool on = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pool;
    size_t used = 0;

    int begin(hipStream_t s) {
        if (!on || used >= kMaxPairs) return FMI_OK;
        if (used == pool.size()) {
            std::pair<hipEvent_t, hipEvent_t> e{};
            FMI_COMM_HIP(hipEventCreate(&e.first));
            FMI_COMM_HIP(hipEventCreate(&e.second));
            pool.push_back(e);
        }
        FMI_COMM_HIP(hipEventRecord(pool[used].first, s));
        return FMI_OK;
    }
    int end(hipStream_t s) {
        if (!on || used >= kMaxPairs) return FMI_OK;
        FMI_COMM_HIP(hipEventRecord(pool[used].second, s));
        ++used;
        return FMI_OK;
    }
    ~KernelTiming() {
        for (auto& [a, b] : pool) {
            (void)hipEventDestroy(a);
            (void)hipEventDestroy(b);
        }
    }
};

struct Comm {
    // 0-3: collective scratch; 4-7 and 16-17: host-pipeline chunk slots (in / out x HostPipe::kDepth);
    // 8-15: pipelined-allreduce slots (2 x 4)
    static constexpr int kSlots = 18;
    std::unique_ptr<Transport> t;
    std::mutex mu;
    KernelTiming timing;
    void* buf[kSlots] = {};
    size_t cap[kSlots] = {};
    HostPipe pipe;
    ChunkPipe chunks;
    std::map<char*, Window> windows;  // keyed by this rank's base
    // The end of the last collective queued on each caller stream (not the library's): an aborted communicator
    // must not free scratch that work on those streams may still read (events outlive the caller's streams).
    std::map<hipStream_t, hipEvent_t> user_tail;

    void note_user_stream(hipStream_t s) {
        if (!s || s == library_stream()) return;
        if (user_tail.size() >= 64 && !user_tail.count(s)) {  // many caller streams: forget the drained ones
            for (auto it = user_tail.begin(); it != user_tail.end();) {
                if (hipEventQuery(it->second) == hipSuccess) {
                    (void)hipEventDestroy(it->second);
                    it = user_tail.erase(it);
                } else {
                    ++it;
                }
            }
        }
        hipEvent_t& ev = user_tail[s];
        if (!ev && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
            user_tail.erase(s);
            return;
        }
        (void)hipEventRecord(ev, s);
    }

    ~Comm() {
        if (t && t->aborted()) {
            // A timed-out or failed communicator: no peer is waited for again. Its device memory may still
            // be referenced by work that never drained: free only if everything drained within a bound,
            // otherwise leak it (and the streams) rather than free memory a kernel may still touch.
            bool drained = Transport::drain(library_stream(), 10.0);
            for (hipStream_t st : {pipe.cs, chunks.gs})
                if (st) drained = Transport::drain(st, 10.0) && drained;
            // copy streams shared with the other co-resident ranks carry their chunks too: only this rank's copies
            // are waited for (its own pair is drained whole)
            if (pipe.owns_copy_streams)
                for (hipStream_t st : {pipe.h2d, pipe.d2h})
                    if (st) drained = Transport::drain(st, 10.0) && drained;
            for (int k = 0; k < HostPipe::kDepth; ++k)
                for (hipEvent_t ev : {pipe.loaded[k], pipe.drained[k]})
                    if (ev) drained = Transport::drain_event(ev, 10.0) && drained;
            for (auto& [st, ev] : user_tail) drained = Transport::drain_event(ev, 10.0) && drained;
            if (!drained) {
                pipe.cs = chunks.gs = nullptr;
                pipe.owns_copy_streams = false;  // leaked with the rest
                for (int k = 0; k < HostPipe::kDepth; ++k) pipe.loaded[k] = pipe.reduced[k] = pipe.drained[k] = nullptr;
                for (void*& b : buf) b = nullptr;
                windows.clear();
                return;
            }
            for (auto& [st, ev] : user_tail) (void)hipEventDestroy(ev);
            for (void* b : buf)
                if (b) (void)hipFree(b);
            for (auto& [base, w] : windows) {
                t->unmap_window(w.peers);
                if (w.shards) (void)hipFree(w.shards);
                (void)hipFree(base);
            }
            return;
        }
        if (pipe.cs) (void)hipStreamSynchronize(pipe.cs);
        for (int k = 0; k < HostPipe::kDepth; ++k)
            for (hipEvent_t ev : {pipe.loaded[k], pipe.drained[k]})
                if (ev) (void)hipEventSynchronize(ev);
        if (chunks.gs) (void)hipStreamSynchronize(chunks.gs);
        for (auto& [st, ev] : user_tail) {
            (void)hipEventSynchronize(ev);
            (void)hipEventDestroy(ev);
        }
        // Windows are read by the peers: wait until every rank is done with them (communicators are torn
        // down collectively, as the reference's Communicator destructor finalizes every channel). A path
        // DIRECT collective may have run on any stream of this process and still be reading a peer's window
        // through its mapping, so drain the whole device before the barrier releases the peers.
        if (!windows.empty()) {
            (void)hipDeviceSynchronize();
            (void)t->barrier(library_stream());
        }
        for (void* b : buf)
            if (b) (void)hipFree(b);
        for (auto& [base, w] : windows) {
            t->unmap_window(w.peers);
            if (w.shards) (void)hipFree(w.shards);
            (void)hipFree(base);
        }
    }

    // The window holding [p, p + len), or nullptr.
    const Window* window_of(const void* p, size_t len, size_t* offset) const {
        const char* c = static_cast<const char*>(p);
        auto it = windows.upper_bound(const_cast<char*>(c));
        if (it == windows.begin()) return nullptr;
        --it;
        if (c < it->first || c + len > it->first + it->second.bytes) return nullptr;
        *offset = static_cast<size_t>(c - it->first);
        return &it->second;
    }

    // scratch slot k of at least `bytes` (grown after draining the stream that used it)
    int scratch(int k, size_t bytes, hipStream_t s, char** out) {
        if (cap[k] < bytes) {
            FMI_COMM_HIP(hipStreamSynchronize(s));
            if (buf[k]) FMI_COMM_HIP(hipFree(buf[k]));
            buf[k] = nullptr;
            cap[k] = 0;
            const hipError_t e = hipMalloc(&buf[k], bytes);
            if (e != hipSuccess) return fail(FMI_ERR_ALLOC, std::string("hipMalloc (comm scratch): ") + hipGetErrorString(e));
            cap[k] = bytes;
        }
        *out = static_cast<char*>(buf[k]);
        return FMI_OK;
    }
};

size_t shard_elems(size_t n, int ranks) {
    const size_t per = (n + ranks - 1) / ranks;
    return (per + kShardAlign - 1) / kShardAlign * kShardAlign;
}

// Where the all-to-all lands the N shards the fused shard kernel then streams together. Back to
// back at `bytes` (a multiple of 64 KiB for the headline's buckets), all N streams sit at one offset modulo HBM's
// 64 KiB interleave and collide, as DESIGN §4 measured for buckets; at a stride of bytes rounded up to 64 KiB plus
// 4 KiB, shard j sits in 4 KiB slot j mod 16 and the reduced shard in slot N mod 16 of the same range. The fused 8-way kernel
// at the N = 8 shard shape (32 MiB): 0.738 packed, 0.790 skewed; N = 4: 0.741 / 0.764; N = 2: 0.784 / 0.806
// (profiles/r06a_shard_layout.jsonl, tools/shard_layout_ab.py). Taken where the transport posts a receive per peer
// anyway (receives_per_peer) and FMI_TUNE_COMM_SHARD_SKEW is on; shards under 1 MiB stay back to back.
constexpr size_t kShardSlot = 4096, kShardSpan = 16 * kShardSlot;
size_t shard_stride(const Transport& t, size_t bytes) {
    if (!tune(FMI_TUNE_COMM_SHARD_SKEW) || bytes < (size_t(1) << 20) || !t.receives_per_peer()) return bytes;
    return (bytes + kShardSpan - 1) / kShardSpan * kShardSpan + kShardSlot;
}

int aborted_error() {
    return fail(FMI_ERR_COMM, "communicator was aborted (a timeout or a transport error); destroy it");
}

int check_common(fmi_comm_t comm, int op, int dtype) {
    if (!comm) return fail(FMI_ERR_INVALID, "null communicator");
    if (op < FMI_OP_SUM || op > FMI_OP_MIN) return fail(FMI_ERR_INVALID, "unknown op " + std::to_string(op));
    if (dtype_size(dtype) == 0) return fail(FMI_ERR_INVALID, "unknown dtype " + std::to_string(dtype));
    if (!library_stream()) return fail(FMI_ERR_NO_DEVICE, "fmi_dev_init has not been called");
    if (static_cast<Comm*>(comm)->t->aborted()) return aborted_error();
    return FMI_OK;
}

// NULL stream = the library's stream (fmi_stream_sync(NULL) then waits for the collective).
hipStream_t resolve_stream(fmi_stream_t s) { return s ? static_cast<hipStream_t>(s) : library_stream(); }

// Copy `send` (n elements) into a zero-padded staging bucket when the shard grid needs padding.
int padded_source(Comm* c, size_t n, size_t padded, size_t esz, const void* send, hipStream_t s, const char** out) {
    if (padded == n) {
        *out = static_cast<const char*>(send);
        return FMI_OK;
    }
    char* pad = nullptr;
    FMI_COMM_RC(c->scratch(0, padded * esz, s, &pad));
    FMI_COMM_RC(device_copy(pad, send, n * esz, s));
    FMI_COMM_HIP(hipMemsetAsync(pad + n * esz, 0, (padded - n) * esz, s));
    *out = pad;
    return FMI_OK;
}

// recv[i] = (reduced-shard area of the rank owning element i)[i], for the byte range [0, nbytes). The owners'
// reduced-shard areas come from a device table (`shards`, one pointer per rank: no limit on the number of
// ranks); blockIdx.y strides over the owners, so each block copies from one owner through a uniform (scalar)
// pointer, and blockIdx.x over that owner's 16-B groups: nontemporal accesses over xGMI when every pointer is
// 16-B aligned, bytes otherwise. Shards are whole multiples of 256 B: only the last owner has a ragged tail.
template <bool VEC>
__global__ void __launch_bounds__(256) gather_shards(const char* const* shards, size_t off, char* dst, size_t nbytes,
                                                     size_t shard_bytes, int nranks) {
    const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
    const size_t first = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    for (int j = blockIdx.y; j < nranks; j += gridDim.y) {
        const size_t lo = static_cast<size_t>(j) * shard_bytes;
        if (lo >= nbytes) break;
        const size_t len = nbytes - lo < shard_bytes ? nbytes - lo : shard_bytes;
        const char* src = shards[j] + off + lo;
        char* out = dst + lo;
        if constexpr (VEC) {
            const size_t nvec = len / 16;
            for (size_t g = first; g < nvec; g += stride)
                __builtin_nontemporal_store(__builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src) + g),
                                            reinterpret_cast<u32x4*>(out) + g);
            if (blockIdx.x == 0 && nvec * 16 + threadIdx.x < len) out[nvec * 16 + threadIdx.x] = src[nvec * 16 + threadIdx.x];
        } else {
            for (size_t b = first; b < len; b += stride) out[b] = src[b];
        }
    }
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// Path DIRECT: no staging and no all-to-all. Rank k's fused kernel reads shard k of every rank's window
// over xGMI and reduces it in the reference's order into its reduced-shard area; every rank then gathers
// the N reduced shards straight from the peers' windows. Two stream-ordered barriers: before the reduce
// (every bucket written) and before the gather (every shard reduced). The next call's first barrier keeps
// a rank from overwriting its reduced shard while a peer still gathers it.
int allreduce_direct(Comm* c, const Window& w, size_t off, int op, int dtype, int alg, void* recv, size_t n,
                     hipStream_t s) {
    const int N = c->t->n();
    const int k = c->t->rank();
    const size_t esz = dtype_size(dtype);
    const size_t shard = shard_elems(n, N);
    static const bool check = [] {
        const char* e = std::getenv("FMI_CHECK_DIRECT");
        return e && e[0] == '1';
    }();
    if (check) {  // every rank must read the peers' windows at the offset and length it uses itself
        int64_t v[4] = {static_cast<int64_t>(off), -static_cast<int64_t>(off), static_cast<int64_t>(n),
                        -static_cast<int64_t>(n)};
        FMI_COMM_RC(c->t->agree_max(v, 4, s));
        if (v[0] != -v[1] || v[2] != -v[3])
            return fail(FMI_ERR_INVALID, "path DIRECT: ranks passed different window offsets or lengths (offset " +
                                             std::to_string(-v[1]) + ".." + std::to_string(v[0]) + ", n " +
                                             std::to_string(-v[3]) + ".." + std::to_string(v[2]) + ")");
    }
    FMI_COMM_RC(c->t->barrier_async(s));
    const size_t lo = std::min(n, static_cast<size_t>(k) * shard);
    const size_t len = std::min(shard, n - lo);
    if (len > 0) {
        std::vector<const void*> ins(N);
        for (int j = 0; j < N; ++j) ins[j] = w.peers[j] + off + lo * esz;
        char* out = w.peers[k] + w.bytes + off + lo * esz;
        FMI_COMM_RC(c->timing.begin(s));
        FMI_COMM_RC(fmi_dev_reduce_tree(op, dtype, alg, out, ins.data(), N, 0, len, s));
        FMI_COMM_RC(c->timing.end(s));
    }
    FMI_COMM_RC(c->t->barrier_async(s));
    // Window bases are allocation starts (256-B aligned) and w.bytes is a multiple of 256, so every owner's
    // source is 16-B aligned exactly when the common offset is.
    const bool vec = aligned16(recv) && off % 16 == 0;
    const size_t nbytes = n * esz;
    const size_t shard_bytes = shard * esz;
    const unsigned gy = static_cast<unsigned>(std::min(N, 65535));
    const size_t per_owner = std::max<size_t>(1, 16384 / gy);
    const unsigned gx = static_cast<unsigned>(std::min(grid_for(vec ? shard_bytes / 16 : shard_bytes, 256), per_owner));
    const dim3 grid(gx, gy);
    if (vec)
        gather_shards<true><<<grid, 256, 0, s>>>(w.shards, off, static_cast<char*>(recv), nbytes, shard_bytes, N);
    else
        gather_shards<false><<<grid, 256, 0, s>>>(w.shards, off, static_cast<char*>(recv), nbytes, shard_bytes, N);
    FMI_COMM_HIP(hipGetLastError());
    return FMI_OK;
}

// Path TREE pipelined over K chunks (FMI_TUNE_COMM_PIPELINE = K): every chunk is its own sharded allreduce
// of a sub-range (element-wise, so the bits are those of the whole-bucket call), with chunk c's all-gather
// on a second stream and communicator while chunk c + 1's all-to-all and kernel run on `s`. Two buffer slots;
// events order their reuse: the kernel of chunk c + 2 waits until chunk c's gather has read its shard.
int allreduce_tree_pipelined(Comm* c, int op, int dtype, int alg, const void* send, void* recv, size_t n,
                             hipStream_t s, size_t K) {
    const int N = c->t->n();
    const size_t esz = dtype_size(dtype);
    ChunkPipe& p = c->chunks;
    FMI_COMM_RC(p.init(c->t.get(), s));
    Transport* tg = p.t2 ? p.t2.get() : c->t.get();
    const size_t step = kShardAlign * static_cast<size_t>(N);
    const size_t ce = ((n + K - 1) / K + step - 1) / step * step;  // chunk elements, whole shards
    const size_t nchunks = (n + ce - 1) / ce;
    FMI_COMM_HIP(hipEventRecord(p.start, s));
    FMI_COMM_HIP(hipStreamWaitEvent(p.gs, p.start, 0));  // the gathers follow the caller's earlier work
    for (size_t k = 0; k < nchunks; ++k) {
        const int j = static_cast<int>(k & 1);
        const size_t lo = k * ce;
        const size_t cn = std::min(ce, n - lo);
        const size_t shard = shard_elems(cn, N);
        const size_t padded = shard * N;
        const char* src = static_cast<const char*>(send) + lo * esz;
        char* dst = static_cast<char*>(recv) + lo * esz;
        if (padded != cn) {  // only the last chunk can need padding
            char* pad = nullptr;
            FMI_COMM_RC(c->scratch(8 + 4 * j, padded * esz, s, &pad));
            FMI_COMM_RC(device_copy(pad, src, cn * esz, s));
            FMI_COMM_HIP(hipMemsetAsync(pad + cn * esz, 0, (padded - cn) * esz, s));
            src = pad;
        }
        char* staging = nullptr;
        char* red = nullptr;
        FMI_COMM_RC(c->scratch(9 + 4 * j, padded * esz, s, &staging));
        if (k >= 2) FMI_COMM_HIP(hipStreamWaitEvent(s, p.gathered[j], 0));  // chunk k - 2 has read red[j]
        FMI_COMM_RC(c->scratch(10 + 4 * j, shard * esz, s, &red));
        FMI_COMM_RC(c->t->all_to_all(src, staging, shard * esz, s));
        std::vector<const void*> parts(N);
        for (int r = 0; r < N; ++r) parts[r] = staging + r * shard * esz;
        FMI_COMM_RC(c->timing.begin(s));
        FMI_COMM_RC(fmi_dev_reduce_tree(op, dtype, alg, red, parts.data(), N, 0, shard, s));
        FMI_COMM_RC(c->timing.end(s));
        FMI_COMM_HIP(hipEventRecord(p.reduced[j], s));
        FMI_COMM_HIP(hipStreamWaitEvent(p.gs, p.reduced[j], 0));
        if (padded == cn) {
            FMI_COMM_RC(tg->all_gather(red, dst, shard * esz, p.gs));
        } else {
            char* out = nullptr;
            FMI_COMM_RC(c->scratch(11 + 4 * j, padded * esz, p.gs, &out));
            FMI_COMM_RC(tg->all_gather(red, out, shard * esz, p.gs));
            FMI_COMM_RC(device_copy(dst, out, cn * esz, p.gs));
        }
        FMI_COMM_HIP(hipEventRecord(p.gathered[j], p.gs));
    }
    // the caller's stream sees the whole result
    FMI_COMM_HIP(hipStreamWaitEvent(s, p.gathered[(nchunks - 1) & 1], 0));
    return FMI_OK;
}

// The sharded allreduce of one device bucket on stream s (caller holds c->mu; arguments validated).
int allreduce_device(Comm* c, int op, int dtype, int alg, int path, const void* send, void* recv, size_t n,
                     hipStream_t s) {
    const int N = c->t->n();
    const size_t esz = dtype_size(dtype);
    if (N == 1 && !tune(FMI_TUNE_COMM_ONE_RANK_EXCHANGE)) {  // reference P = 1: a copy
        if (send != recv) FMI_COMM_RC(device_copy(recv, send, n * esz, s));
        return FMI_OK;
    }
    // Float max / min: every peer of the reference allreduce keeps its own operand order, so on ±0 ties
    // and NaNs the peers' results differ. Each shard owner then computes the shard in every rank's order
    // and an all-to-all (instead of the all-gather) hands rank r the versions in its order. Same exchange
    // volume; the owner's kernel writes N versions of its shard. Path DIRECT takes this exchange too.
    const bool per_rank = path != FMI_PATH_RCCL && alg == FMI_ALG_ALLREDUCE && order_sensitive(op, dtype);
    if (path == FMI_PATH_DIRECT) {
        size_t off = 0;
        const Window* w = c->window_of(send, n * esz, &off);
        if (!w) return fail(FMI_ERR_INVALID, "path DIRECT: send must lie inside a window from fmi_comm_window_alloc");
        if (!per_rank) return allreduce_direct(c, *w, off, op, dtype, alg, recv, n, s);
    }
    if (path == FMI_PATH_TREE && !per_rank) {
        const long long K = tune(FMI_TUNE_COMM_PIPELINE);
        // worth it only for chunks of at least 1 MiB per rank; without a second communicator the unpipelined
        // path below runs (same bits)
        if (K >= 2 && n * esz / static_cast<size_t>(K) >= (size_t(1) << 20) * static_cast<size_t>(N) &&
            !c->chunks.no_split) {
            const int rc = c->chunks.init(c->t.get(), s);
            if (rc == FMI_OK) return allreduce_tree_pipelined(c, op, dtype, alg, send, recv, n, s, static_cast<size_t>(K));
            if (rc != FMI_ERR_UNSUPPORTED) return rc;
        }
    }
    const size_t shard = shard_elems(n, N);
    const size_t padded = shard * N;
    if (padded != n && path == FMI_PATH_TREE && !per_rank && c->t->ragged()) {
        // no zero-padded copies in or out: the last shards are short (or empty) and move at their length
        char* staging = nullptr;
        char* red = nullptr;
        FMI_COMM_RC(c->scratch(1, padded * esz, s, &staging));
        FMI_COMM_RC(c->scratch(2, shard * esz, s, &red));
        FMI_COMM_RC(c->t->all_to_all_ragged(static_cast<const char*>(send), staging, shard * esz, n * esz, s));
        const size_t len = Transport::span(c->t->rank(), shard, n);  // elements of my shard
        if (len) {
            std::vector<const void*> parts(N);
            for (int j = 0; j < N; ++j) parts[j] = staging + j * shard * esz;
            FMI_COMM_RC(c->timing.begin(s));
            FMI_COMM_RC(fmi_dev_reduce_tree(op, dtype, alg, red, parts.data(), N, 0, len, s));
            FMI_COMM_RC(c->timing.end(s));
        }
        return c->t->all_gather_ragged(red, static_cast<char*>(recv), shard * esz, n * esz, s);
    }
    const char* src = nullptr;
    FMI_COMM_RC(padded_source(c, n, padded, esz, send, s, &src));
    // skewed (shard_stride): the shard kernel's N inputs and its output carved from one scratch range, each in its
    // own 4 KiB slot (a carved group); otherwise the inputs back to back and the output apart
    const size_t stride = path != FMI_PATH_RCCL && !per_rank ? shard_stride(*c->t, shard * esz) : shard * esz;
    const bool skewed = stride != shard * esz;
    char* red = nullptr;
    char* staging = nullptr;
    if (skewed) {
        FMI_COMM_RC(c->scratch(1, (static_cast<size_t>(N) + 1) * stride, s, &staging));
        red = staging + static_cast<size_t>(N) * stride;
    } else {
        FMI_COMM_RC(c->scratch(2, (per_rank ? padded : shard) * esz, s, &red));
    }
    if (path != FMI_PATH_RCCL) {
        if (!skewed) FMI_COMM_RC(c->scratch(1, padded * esz, s, &staging));
        FMI_COMM_RC(c->t->all_to_all_strided(src, staging, shard * esz, stride, s));
        std::vector<const void*> parts(N);
        for (int j = 0; j < N; ++j) parts[j] = staging + j * stride;
        if (per_rank) {
            FMI_COMM_RC(c->timing.begin(s));
            if (N >= 2 && N <= sched::kMaxFusedPeers) {
                PeerPtrs ptrs{};
                for (int j = 0; j < N; ++j) {
                    ptrs.in[j] = parts[j];
                    ptrs.out[j] = red + j * shard * esz;
                }
                FMI_COMM_RC(launch_fused_allreduce_all_ranks(op, dtype, N, ptrs, shard, s));
            } else {
                for (int r = 0; r < N; ++r)
                    FMI_COMM_RC(fmi_dev_reduce_tree(op, dtype, alg, red + r * shard * esz, parts.data(), N, r, shard, s));
            }
            FMI_COMM_RC(c->timing.end(s));
            if (padded == n) return c->t->all_to_all(red, static_cast<char*>(recv), shard * esz, s);
            char* out = nullptr;
            FMI_COMM_RC(c->scratch(3, padded * esz, s, &out));
            FMI_COMM_RC(c->t->all_to_all(red, out, shard * esz, s));
            FMI_COMM_RC(device_copy(recv, out, n * esz, s));
            return FMI_OK;
        }
        FMI_COMM_RC(c->timing.begin(s));
        FMI_COMM_RC(fmi_dev_reduce_tree(op, dtype, alg, red, parts.data(), N, 0, shard, s));
        FMI_COMM_RC(c->timing.end(s));
    } else {
        FMI_COMM_RC(c->t->reduce_scatter(op, dtype, src, red, shard, s));
    }
    if (padded == n) return c->t->all_gather(red, static_cast<char*>(recv), shard * esz, s);
    char* out = nullptr;
    FMI_COMM_RC(c->scratch(3, padded * esz, s, &out));
    FMI_COMM_RC(c->t->all_gather(red, out, shard * esz, s));
    FMI_COMM_RC(device_copy(recv, out, n * esz, s));
    return FMI_OK;
}

int comm_init(fmi_comm_t* comm, const void* id, int nranks, int rank, double timeout_s);

int check_allreduce_args(int alg, int path) {
    if (alg != FMI_ALG_ALLREDUCE && alg != FMI_ALG_REDUCE_LTR)
        return fail(FMI_ERR_INVALID, "allreduce: alg must be ALLREDUCE or REDUCE_LTR");
    if (path != FMI_PATH_TREE && path != FMI_PATH_RCCL && path != FMI_PATH_DIRECT)
        return fail(FMI_ERR_INVALID, "unknown path");
    if (path == FMI_PATH_RCCL && alg != FMI_ALG_ALLREDUCE)
        return fail(FMI_ERR_INVALID, "ordered (LTR) allreduce needs the tree path");
    return FMI_OK;
}

}  // namespace
}  // namespace fmi::dev

using namespace fmi::dev;

extern "C" {

static int comm_unique_id_impl(int transport, void* id, size_t len) {
    if (!id || len < FMI_COMM_ID_BYTES) return fail(FMI_ERR_INVALID, "id buffer must hold FMI_COMM_ID_BYTES");
    std::memset(id, 0, FMI_COMM_ID_BYTES);
    if (transport == FMI_TRANSPORT_LOCAL) {
        const uint64_t key = (static_cast<uint64_t>(getpid()) << 32) ^ g_hub_counter.fetch_add(1);
        std::memcpy(id, kLocalMagic, 8);
        std::memcpy(static_cast<char*>(id) + 8, &key, 8);
        return FMI_OK;
    }
    if (transport == FMI_TRANSPORT_PROC) {
        const uint64_t t = static_cast<uint64_t>(std::chrono::steady_clock::now().time_since_epoch().count());
        const uint64_t key = (static_cast<uint64_t>(getpid()) << 40) ^ (g_hub_counter.fetch_add(1) << 24) ^ t;
        std::memcpy(id, kProcMagic, 8);
        std::memcpy(static_cast<char*>(id) + 8, &key, 8);
        return FMI_OK;
    }
    if (transport != FMI_TRANSPORT_RCCL) return fail(FMI_ERR_INVALID, "unknown transport");
    const RcclApi* api = rccl_api();
    if (!api) return FMI_ERR_COMM;
    ncclUniqueId uid;
    FMI_NCCL(api, GetUniqueId(&uid));
    static_assert(sizeof(ncclUniqueId) == FMI_COMM_ID_BYTES, "RCCL unique id size");
    std::memcpy(id, &uid, FMI_COMM_ID_BYTES);
    return FMI_OK;
}

int fmi_comm_init(fmi_comm_t* comm, const void* id, int nranks, int rank) {
    return fmi_comm_init_timeout(comm, id, nranks, rank, 0.0);
}

int fmi_comm_init_timeout(fmi_comm_t* comm, const void* id, int nranks, int rank, double timeout_s) {
    return guarded("fmi_comm_init", [&] { return comm_init(comm, id, nranks, rank, timeout_s); });
}

}  // extern "C"

namespace fmi::dev {
namespace {

int comm_init(fmi_comm_t* comm, const void* id, int nranks, int rank, double timeout_s) {
    if (!comm || !id) return fail(FMI_ERR_INVALID, "null argument");
    if (nranks < 1 || rank < 0 || rank >= nranks) return fail(FMI_ERR_INVALID, "rank out of range");
    if (nranks > fmi::sched::kMaxPeers)  // value ids of a P = nranks program must fit 31 bits
        return fail(FMI_ERR_INVALID, "at most " + std::to_string(fmi::sched::kMaxPeers) + " ranks per communicator");
    auto c = std::make_unique<Comm>();
    if (std::memcmp(id, kLocalMagic, 8) == 0) {
        uint64_t key;
        std::memcpy(&key, static_cast<const char*>(id) + 8, 8);
        std::shared_ptr<Hub> hub;
        {
            std::lock_guard<std::mutex> lk(g_hub_mu);
            hub = g_hubs[key].lock();
            if (!hub) {
                hub = std::make_shared<Hub>(nranks);
                g_hubs[key] = hub;
            }
        }
        if (hub->n != nranks) return fail(FMI_ERR_INVALID, "local communicator joined with a different size");
        c->t = std::make_unique<LocalTransport>(hub, nranks, rank);
        c->t->set_timeout(timeout_s > 0 ? timeout_s : default_timeout_s(false));
    } else if (std::memcmp(id, kProcMagic, 8) == 0) {
        auto t = std::make_unique<ProcTransport>(nranks, rank);
        t->set_timeout(timeout_s > 0 ? timeout_s : default_timeout_s(true));
        FMI_COMM_RC(t->join(id));
        c->t = std::move(t);
    } else {
        const RcclApi* api = rccl_api();
        if (!api) return FMI_ERR_COMM;
        ncclUniqueId uid;
        std::memcpy(&uid, id, FMI_COMM_ID_BYTES);
        ncclComm_t nc = nullptr;
        const double limit = timeout_s > 0 ? timeout_s : default_timeout_s(false);
        // Non-blocking init, polled against the timeout (a peer that never joins ends in FMI_ERR_TIMEOUT and
        // ncclCommAbort, not a hang). FMI_COMM_BLOCKING=1, or a librccl without the config / async-error /
        // abort entry points, takes the blocking ncclCommInitRank (unbounded).
        const char* blocking = std::getenv("FMI_COMM_BLOCKING");
        if (api->bounded() && !(blocking && blocking[0] == '1')) {
            ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
            cfg.blocking = 0;
            const ncclResult_t r = api->CommInitRankConfig(&nc, nranks, uid, rank, &cfg);
            if (r != ncclSuccess && r != ncclInProgress) {
                if (nc) (void)api->CommAbort(nc);
                return nccl_fail(api, "ncclCommInitRankConfig", r);
            }
            auto t = std::make_unique<RcclTransport>(api, nc, nranks, rank, true);
            t->set_timeout(limit);
            FMI_COMM_RC(t->wait_ready("ncclCommInitRankConfig (waiting for every rank to join)"));
            c->t = std::move(t);
        } else {
            FMI_NCCL(api, CommInitRank(&nc, nranks, uid, rank));
            c->t = std::make_unique<RcclTransport>(api, nc, nranks, rank, false);
            c->t->set_timeout(limit);
        }
    }
    *comm = c.release();
    return FMI_OK;
}

}  // namespace
}  // namespace fmi::dev

extern "C" {

int fmi_comm_destroy(fmi_comm_t comm) {
    delete static_cast<Comm*>(comm);
    return FMI_OK;
}

int fmi_comm_size(fmi_comm_t comm, int* nranks, int* rank) {
    if (!comm || !nranks || !rank) return fail(FMI_ERR_INVALID, "null argument");
    Comm* c = static_cast<Comm*>(comm);
    *nranks = c->t->n();
    *rank = c->t->rank();
    return FMI_OK;
}

static int comm_window_alloc_impl(fmi_comm_t comm, size_t bytes, void** ptr) {
    if (!comm || !ptr) return fail(FMI_ERR_INVALID, "null argument");
    if (!library_stream()) return fail(FMI_ERR_NO_DEVICE, "fmi_dev_init has not been called");
    Comm* c = static_cast<Comm*>(comm);
    std::lock_guard<std::mutex> lk(c->mu);
    if (c->t->aborted()) return aborted_error();
    bytes = std::max<size_t>(256, (bytes + 255) / 256 * 256);
    const int N = c->t->n();
    // Everything this rank needs is allocated BEFORE the collective mapping and its success goes into the
    // mapping's all-or-nothing flag; the table fill after it is agreed on by every rank too, so either every
    // rank holds the window or every rank has released it (no peer keeps a mapping of a freed base).
    char* base = nullptr;
    Window w;
    w.bytes = bytes;
    bool ok = hipMalloc(&base, 2 * bytes) == hipSuccess;
    ok = ok && hipMalloc(&w.shards, static_cast<size_t>(N) * sizeof(char*)) == hipSuccess;
    auto release = [&] {
        if (w.shards) (void)hipFree(w.shards);
        if (base) (void)hipFree(base);
    };
    int rc = c->t->map_window(ok ? base : nullptr, ok, w.peers, library_stream());
    if (rc != FMI_OK) {
        release();
        return rc;
    }
    std::vector<char*> table(w.peers.size());
    for (size_t j = 0; j < table.size(); ++j) table[j] = w.peers[j] + bytes;
    const hipError_t e = hipMemcpy(w.shards, table.data(), table.size() * sizeof(char*), hipMemcpyHostToDevice);
    int64_t failed[1] = {e == hipSuccess ? 0 : 1};
    rc = c->t->agree_max(failed, 1, library_stream());
    if (rc != FMI_OK || failed[0] != 0) {
        c->t->unmap_window(w.peers);
        release();
        if (rc != FMI_OK) return rc;
        return fail(FMI_ERR_ALLOC, e != hipSuccess ? std::string("window shard table: ") + hipGetErrorString(e)
                                                   : std::string("window shard table: failed on another rank"));
    }
    c->windows[base] = std::move(w);
    *ptr = base;
    return FMI_OK;
}

static int comm_window_free_impl(fmi_comm_t comm, void* ptr) {
    if (!comm || !ptr) return fail(FMI_ERR_INVALID, "null argument");
    Comm* c = static_cast<Comm*>(comm);
    std::lock_guard<std::mutex> lk(c->mu);
    if (c->t->aborted()) return aborted_error();  // the window goes with the communicator
    auto it = c->windows.find(static_cast<char*>(ptr));
    if (it == c->windows.end()) return fail(FMI_ERR_INVALID, "not a window of this communicator");
    // No peer may still be reading it, and this rank must be done reading the peers' windows: a path
    // DIRECT collective on any stream (not only the library's) reads them through the mappings that are
    // closed below, so the whole device drains before the barrier.
    FMI_COMM_HIP(hipDeviceSynchronize());
    FMI_COMM_RC(c->t->barrier(library_stream()));
    c->t->unmap_window(it->second.peers);
    if (it->second.shards) FMI_COMM_HIP(hipFree(it->second.shards));
    FMI_COMM_HIP(hipFree(it->first));
    c->windows.erase(it);
    return FMI_OK;
}

int fmi_comm_timing(fmi_comm_t comm, int enable) {
    if (!comm) return fail(FMI_ERR_INVALID, "null communicator");
    Comm* c = static_cast<Comm*>(comm);
    std::lock_guard<std::mutex> lk(c->mu);
    c->timing.on = enable != 0;
    c->timing.used = 0;
    return FMI_OK;
}

int fmi_comm_timing_read(fmi_comm_t comm, float* total_ms, int* launches) {
    if (!comm || !total_ms || !launches) return fail(FMI_ERR_INVALID, "null argument");
    Comm* c = static_cast<Comm*>(comm);
    std::lock_guard<std::mutex> lk(c->mu);
    float total = 0.f;
    for (size_t k = 0; k < c->timing.used; ++k) {
        auto& [a, b] = c->timing.pool[k];
        FMI_COMM_HIP(hipEventSynchronize(b));
        float ms = 0.f;
        FMI_COMM_HIP(hipEventElapsedTime(&ms, a, b));
        total += ms;
    }
    *total_ms = total;
    *launches = static_cast<int>(c->timing.used);
    c->timing.used = 0;
    return FMI_OK;
}

static int comm_allreduce_impl(fmi_comm_t comm, int op, int dtype, int alg, int path, const void* send, void* recv, size_t n,
                       fmi_stream_t stream) {
    FMI_COMM_RC(check_common(comm, op, dtype));
    FMI_COMM_RC(check_allreduce_args(alg, path));
    if (n == 0) return FMI_OK;
    if (!send || !recv) return fail(FMI_ERR_INVALID, "null bucket");
    Comm* c = static_cast<Comm*>(comm);
    std::lock_guard<std::mutex> lk(c->mu);
    return allreduce_device(c, op, dtype, alg, path, send, recv, n, resolve_stream(stream));
}

// Three-stage pipeline over HostPipe::depth() chunk slots: while chunk k is allreduced on pipe.cs, chunk k+1 loads on
// pipe.h2d and chunk k-1 drains on pipe.d2h (HostPipe: whose copy streams). Slot reuse is
// ordered by events: a load into slot j waits until the allreduce that read it (chunk k - kDepth) has finished
// (reduced), an allreduce into slot j waits until the previous result in it has drained to the host.
static int comm_allreduce_host_impl(fmi_comm_t comm, int op, int dtype, int alg, int path, const void* send, void* recv,
                            size_t n, size_t chunk) {
    FMI_COMM_RC(check_common(comm, op, dtype));
    FMI_COMM_RC(check_allreduce_args(alg, path));
    if (n == 0) return FMI_OK;
    if (!send || !recv) return fail(FMI_ERR_INVALID, "null bucket");
    Comm* c = static_cast<Comm*>(comm);
    std::lock_guard<std::mutex> lk(c->mu);
    HostPipe& p = c->pipe;
    FMI_COMM_RC(p.init(*c->t));
    const int D = p.depth();
    const size_t esz = dtype_size(dtype);
    if (chunk == 0) {
        long long bytes = 0;
        (void)fmi_tune_get(FMI_TUNE_HOST_CHUNK, &bytes);
        chunk = std::max<size_t>(static_cast<size_t>(bytes) / esz, kShardAlign);
    }
    chunk = std::min(chunk, n);
    const size_t nchunks = (n + chunk - 1) / chunk;
    static constexpr int kIn[HostPipe::kDepth] = {4, 5, 16}, kOut[HostPipe::kDepth] = {6, 7, 17};  // Comm scratch slots
    char* in[HostPipe::kDepth] = {};
    char* out[HostPipe::kDepth] = {};
    for (int j = 0; j < D && static_cast<size_t>(j) < nchunks; ++j) {
        FMI_COMM_RC(c->scratch(kIn[j], chunk * esz, p.cs, &in[j]));
        FMI_COMM_RC(c->scratch(kOut[j], chunk * esz, p.cs, &out[j]));
    }
    const char* src = static_cast<const char*>(send);
    char* dst = static_cast<char*>(recv);
    auto span = [&](size_t k) { return std::min(chunk, n - k * chunk); };
    auto load = [&](size_t k) -> int {
        const int j = static_cast<int>(k % D);
        if (k >= static_cast<size_t>(D)) FMI_COMM_HIP(hipStreamWaitEvent(p.h2d, p.reduced[j], 0));
        FMI_COMM_HIP(hipMemcpyAsync(in[j], src + k * chunk * esz, span(k) * esz, hipMemcpyDefault, p.h2d));
        FMI_COMM_HIP(hipEventRecord(p.loaded[j], p.h2d));
        return FMI_OK;
    };
    FMI_COMM_RC(load(0));
    for (size_t k = 0; k < nchunks; ++k) {
        if (k + 1 < nchunks) FMI_COMM_RC(load(k + 1));
        const int j = static_cast<int>(k % D);
        FMI_COMM_HIP(hipStreamWaitEvent(p.cs, p.loaded[j], 0));
        if (k >= static_cast<size_t>(D)) {
            // Host-side too: chunk k - D has drained before chunk k is queued. The device would wait for it anyway
            // (the stream wait above); waiting here as well gives the communicator's timeout a fresh deadline per
            // chunk, so it bounds the progress of one chunk, never the whole bucket's transfer time.
            FMI_COMM_HIP(hipStreamWaitEvent(p.cs, p.drained[j], 0));
            FMI_COMM_RC(c->t->wait_event(p.drained[j], p.d2h, "fmi_comm_allreduce_host (a chunk's exchange)"));
        }
        FMI_COMM_RC(allreduce_device(c, op, dtype, alg, path, in[j], out[j], span(k), p.cs));
        FMI_COMM_HIP(hipEventRecord(p.reduced[j], p.cs));
        FMI_COMM_HIP(hipStreamWaitEvent(p.d2h, p.reduced[j], 0));
        FMI_COMM_HIP(hipMemcpyAsync(dst + k * chunk * esz, out[j], span(k) * esz, hipMemcpyDefault, p.d2h));
        FMI_COMM_HIP(hipEventRecord(p.drained[j], p.d2h));
    }
    // this communicator's last result copy (the shared D2H stream may already carry other ranks' later chunks)
    FMI_COMM_RC(c->t->wait_event(p.drained[(nchunks - 1) % D], p.d2h, "fmi_comm_allreduce_host"));
    return c->t->wait_stream(p.cs, "fmi_comm_allreduce_host");
}

static int comm_reduce_impl(fmi_comm_t comm, int op, int dtype, int alg, const void* send, void* recv, size_t n, int root,
                    fmi_stream_t stream) {
    FMI_COMM_RC(check_common(comm, op, dtype));
    if (alg != FMI_ALG_REDUCE && alg != FMI_ALG_REDUCE_LTR)
        return fail(FMI_ERR_INVALID, "reduce: alg must be REDUCE or REDUCE_LTR");
    Comm* c = static_cast<Comm*>(comm);
    const int N = c->t->n();
    if (root < 0 || root >= N) return fail(FMI_ERR_INVALID, "root out of range");
    if (n == 0) return FMI_OK;
    if (!send || (c->t->rank() == root && !recv)) return fail(FMI_ERR_INVALID, "null bucket");
    std::lock_guard<std::mutex> lk(c->mu);
    hipStream_t s = resolve_stream(stream);
    const size_t esz = dtype_size(dtype);
    if (N == 1 && !tune(FMI_TUNE_COMM_ONE_RANK_EXCHANGE)) {
        if (send != recv) FMI_COMM_RC(device_copy(recv, send, n * esz, s));
        return FMI_OK;
    }
    const size_t shard = shard_elems(n, N);
    const size_t padded = shard * N;
    const bool is_root = c->t->rank() == root;
    char* staging = nullptr;
    char* red = nullptr;
    FMI_COMM_RC(c->scratch(1, padded * esz, s, &staging));
    FMI_COMM_RC(c->scratch(2, shard * esz, s, &red));
    std::vector<const void*> parts(N);
    for (int j = 0; j < N; ++j) parts[j] = staging + j * shard * esz;
    if (padded != n && c->t->ragged()) {  // short last shards at their own length: no padded copies
        FMI_COMM_RC(c->t->all_to_all_ragged(static_cast<const char*>(send), staging, shard * esz, n * esz, s));
        const size_t len = Transport::span(c->t->rank(), shard, n);
        FMI_COMM_RC(fmi_dev_reduce_tree(op, dtype, alg, red, parts.data(), N, root, len, s));
        return c->t->gather_ragged(red, is_root ? static_cast<char*>(recv) : nullptr, shard * esz, n * esz, root, s);
    }
    const char* src = nullptr;
    FMI_COMM_RC(padded_source(c, n, padded, esz, send, s, &src));
    FMI_COMM_RC(c->t->all_to_all(src, staging, shard * esz, s));
    FMI_COMM_RC(fmi_dev_reduce_tree(op, dtype, alg, red, parts.data(), N, root, shard, s));
    if (padded == n) return c->t->gather(red, is_root ? static_cast<char*>(recv) : nullptr, shard * esz, root, s);
    char* out = nullptr;
    FMI_COMM_RC(c->scratch(3, padded * esz, s, &out));
    FMI_COMM_RC(c->t->gather(red, out, shard * esz, root, s));
    if (is_root) FMI_COMM_RC(device_copy(recv, out, n * esz, s));
    return FMI_OK;
}

// The reference's reduce with its side effect on every sendbuf (PeerToPeer.cpp:59-84): all-to-all of shards
// -> on every shard owner, the reduce_no_order program with ALL N peers' final values as outputs (fused
// kReducePartials kernel: N reads, N writes) -> all-to-all back into each rank's `send`; the root then
// copies its value (the result) into recv. reduce_ltr leaves every sendbuf intact (:44-57), so it is the
// plain reduce.
static int comm_reduce_sendbuf_impl(fmi_comm_t comm, int op, int dtype, int alg, void* send, void* recv, size_t n, int root,
                            fmi_stream_t stream) {
    if (alg == FMI_ALG_REDUCE_LTR) return comm_reduce_impl(comm, op, dtype, alg, send, recv, n, root, stream);
    FMI_COMM_RC(check_common(comm, op, dtype));
    if (alg != FMI_ALG_REDUCE) return fail(FMI_ERR_INVALID, "reduce: alg must be REDUCE or REDUCE_LTR");
    Comm* c = static_cast<Comm*>(comm);
    const int N = c->t->n();
    if (root < 0 || root >= N) return fail(FMI_ERR_INVALID, "root out of range");
    if (n == 0) return FMI_OK;
    if (!send || (c->t->rank() == root && !recv)) return fail(FMI_ERR_INVALID, "null bucket");
    std::lock_guard<std::mutex> lk(c->mu);
    hipStream_t s = resolve_stream(stream);
    const size_t esz = dtype_size(dtype);
    const bool is_root = c->t->rank() == root;
    if (N > 1 || tune(FMI_TUNE_COMM_ONE_RANK_EXCHANGE)) {
        const size_t shard = shard_elems(n, N);
        const size_t padded = shard * N;
        const bool ragged = padded != n && c->t->ragged();  // short last shards at their own length
        char* staging = nullptr;
        char* partial = nullptr;
        FMI_COMM_RC(c->scratch(1, padded * esz, s, &staging));
        FMI_COMM_RC(c->scratch(2, padded * esz, s, &partial));
        if (ragged) {
            FMI_COMM_RC(c->t->all_to_all_ragged(static_cast<const char*>(send), staging, shard * esz, n * esz, s));
        } else {
            const char* src = nullptr;
            FMI_COMM_RC(padded_source(c, n, padded, esz, send, s, &src));
            FMI_COMM_RC(c->t->all_to_all(src, staging, shard * esz, s));
        }
        // transformed id t = (rank - root) mod N (PeerToPeer.cpp:287-293): input t is real rank (t + root) % N,
        // and output t goes to the block of that real rank (the all-to-all back delivers block j to rank j)
        std::vector<const void*> ins(N);
        std::vector<void*> outs(N);
        for (int t = 0; t < N; ++t) {
            const int real = (t + root) % N;
            ins[t] = staging + real * shard * esz;
            outs[t] = partial + real * shard * esz;
        }
        const size_t len = ragged ? Transport::span(c->t->rank(), shard, n) : shard;
        FMI_COMM_RC(reduce_partials(op, dtype, outs.data(), ins.data(), N, len, s));
        if (ragged) {
            FMI_COMM_RC(c->t->all_to_all_back_ragged(partial, static_cast<char*>(send), shard * esz, n * esz, s));
        } else if (padded == n) {
            FMI_COMM_RC(c->t->all_to_all(partial, static_cast<char*>(send), shard * esz, s));
        } else {
            char* out = nullptr;
            FMI_COMM_RC(c->scratch(3, padded * esz, s, &out));
            FMI_COMM_RC(c->t->all_to_all(partial, out, shard * esz, s));
            FMI_COMM_RC(device_copy(send, out, n * esz, s));
        }
    }
    if (is_root && recv != send) FMI_COMM_RC(device_copy(recv, send, n * esz, s));
    return FMI_OK;
}

static int comm_scan_impl(fmi_comm_t comm, int op, int dtype, int alg, const void* send, void* recv, size_t n,
                  fmi_stream_t stream) {
    FMI_COMM_RC(check_common(comm, op, dtype));
    if (alg != FMI_ALG_SCAN && alg != FMI_ALG_SCAN_LTR) return fail(FMI_ERR_INVALID, "scan: alg must be SCAN or SCAN_LTR");
    if (n == 0) return FMI_OK;
    if (!send || !recv) return fail(FMI_ERR_INVALID, "null bucket");
    Comm* c = static_cast<Comm*>(comm);
    std::lock_guard<std::mutex> lk(c->mu);
    hipStream_t s = resolve_stream(stream);
    const int N = c->t->n();
    const size_t esz = dtype_size(dtype);
    if (N == 1 && !tune(FMI_TUNE_COMM_ONE_RANK_EXCHANGE)) {
        if (send != recv) FMI_COMM_RC(device_copy(recv, send, n * esz, s));
        return FMI_OK;
    }
    const size_t shard = shard_elems(n, N);
    const size_t padded = shard * N;
    char* staging = nullptr;
    char* prefix = nullptr;
    FMI_COMM_RC(c->scratch(1, padded * esz, s, &staging));
    FMI_COMM_RC(c->scratch(2, padded * esz, s, &prefix));
    std::vector<const void*> ins(N);
    std::vector<void*> outs(N);
    for (int j = 0; j < N; ++j) {
        ins[j] = staging + j * shard * esz;
        outs[j] = prefix + j * shard * esz;  // prefix of rank j over my shard
    }
    if (padded != n && c->t->ragged()) {  // short last shards at their own length: no padded copies
        FMI_COMM_RC(c->t->all_to_all_ragged(static_cast<const char*>(send), staging, shard * esz, n * esz, s));
        const size_t len = Transport::span(c->t->rank(), shard, n);
        FMI_COMM_RC(fmi_dev_scan_peers(op, dtype, alg, outs.data(), ins.data(), N, len, s));
        return c->t->all_to_all_back_ragged(prefix, static_cast<char*>(recv), shard * esz, n * esz, s);
    }
    const char* src = nullptr;
    FMI_COMM_RC(padded_source(c, n, padded, esz, send, s, &src));
    FMI_COMM_RC(c->t->all_to_all(src, staging, shard * esz, s));
    FMI_COMM_RC(fmi_dev_scan_peers(op, dtype, alg, outs.data(), ins.data(), N, shard, s));
    // rank k gathers its prefix shard j from rank j: an all-to-all back
    if (padded == n) return c->t->all_to_all(prefix, static_cast<char*>(recv), shard * esz, s);
    char* out = nullptr;
    FMI_COMM_RC(c->scratch(3, padded * esz, s, &out));
    FMI_COMM_RC(c->t->all_to_all(prefix, out, shard * esz, s));
    FMI_COMM_RC(device_copy(recv, out, n * esz, s));
    return FMI_OK;
}

#define FMI_COMM_PRELUDE()                                                        \
    if (!comm) return fail(FMI_ERR_INVALID, "null communicator");                 \
    if (!library_stream()) return fail(FMI_ERR_NO_DEVICE, "fmi_dev_init has not been called"); \
    Comm* c = static_cast<Comm*>(comm);                                           \
    std::lock_guard<std::mutex> lk(c->mu);                                        \
    if (c->t->aborted()) return aborted_error();                                  \
    hipStream_t s = resolve_stream(stream);

static int comm_bcast_impl(fmi_comm_t comm, void* buf, size_t bytes, int root, fmi_stream_t stream) {
    FMI_COMM_PRELUDE();
    if (root < 0 || root >= c->t->n()) return fail(FMI_ERR_INVALID, "root out of range");
    return c->t->bcast(static_cast<char*>(buf), bytes, root, s);
}

static int comm_gather_impl(fmi_comm_t comm, const void* send, void* recv, size_t bytes, int root, fmi_stream_t stream) {
    FMI_COMM_PRELUDE();
    if (root < 0 || root >= c->t->n()) return fail(FMI_ERR_INVALID, "root out of range");
    return c->t->gather(static_cast<const char*>(send), static_cast<char*>(recv), bytes, root, s);
}

static int comm_scatter_impl(fmi_comm_t comm, const void* send, void* recv, size_t bytes, int root, fmi_stream_t stream) {
    FMI_COMM_PRELUDE();
    if (root < 0 || root >= c->t->n()) return fail(FMI_ERR_INVALID, "root out of range");
    return c->t->scatter(static_cast<const char*>(send), static_cast<char*>(recv), bytes, root, s);
}

static int comm_send_impl(fmi_comm_t comm, const void* buf, size_t bytes, int peer, fmi_stream_t stream) {
    FMI_COMM_PRELUDE();
    if (peer < 0 || peer >= c->t->n()) return fail(FMI_ERR_INVALID, "peer out of range");
    return c->t->send(static_cast<const char*>(buf), bytes, peer, s);
}

static int comm_recv_impl(fmi_comm_t comm, void* buf, size_t bytes, int peer, fmi_stream_t stream) {
    FMI_COMM_PRELUDE();
    if (peer < 0 || peer >= c->t->n()) return fail(FMI_ERR_INVALID, "peer out of range");
    return c->t->recv(static_cast<char*>(buf), bytes, peer, s);
}

static int comm_barrier_impl(fmi_comm_t comm, fmi_stream_t stream) {
    FMI_COMM_PRELUDE();
    return c->t->barrier(s);
}


}  // extern "C"

// ---- entry points: no C++ exception crosses the C-ABI (guarded) ----
// A collective on a caller stream: afterwards (whatever its status — a failure may follow enqueued work) the
// stream's tail is noted, so destroying an aborted communicator waits for it before freeing scratch.
template <class F>
int on_stream(const char* name, fmi_comm_t comm, fmi_stream_t stream, F&& f) {
    const int rc = guarded(name, f);
    if (comm && stream) {
        Comm* c = static_cast<Comm*>(comm);
        std::lock_guard<std::mutex> lk(c->mu);
        c->note_user_stream(static_cast<hipStream_t>(stream));
    }
    return rc;
}

extern "C" {
int fmi_comm_window_alloc(fmi_comm_t comm, size_t bytes, void** ptr) {
    return guarded("fmi_comm_window_alloc", [&] { return comm_window_alloc_impl(comm, bytes, ptr); });
}

int fmi_comm_window_free(fmi_comm_t comm, void* ptr) {
    return guarded("fmi_comm_window_free", [&] { return comm_window_free_impl(comm, ptr); });
}

int fmi_comm_allreduce(fmi_comm_t comm, int op, int dtype, int alg, int path, const void* send, void* recv, size_t n,
                       fmi_stream_t stream) {
    return on_stream("fmi_comm_allreduce", comm, stream, [&] { return comm_allreduce_impl(comm, op, dtype, alg, path, send, recv, n, stream); });
}

int fmi_comm_allreduce_host(fmi_comm_t comm, int op, int dtype, int alg, int path, const void* send, void* recv,
                            size_t n, size_t chunk) {
    return guarded("fmi_comm_allreduce_host", [&] { return comm_allreduce_host_impl(comm, op, dtype, alg, path, send, recv, n, chunk); });
}

int fmi_comm_reduce(fmi_comm_t comm, int op, int dtype, int alg, const void* send, void* recv, size_t n, int root,
                    fmi_stream_t stream) {
    return on_stream("fmi_comm_reduce", comm, stream, [&] { return comm_reduce_impl(comm, op, dtype, alg, send, recv, n, root, stream); });
}

int fmi_comm_reduce_sendbuf(fmi_comm_t comm, int op, int dtype, int alg, void* send, void* recv, size_t n, int root,
                            fmi_stream_t stream) {
    return on_stream("fmi_comm_reduce_sendbuf", comm, stream, [&] { return comm_reduce_sendbuf_impl(comm, op, dtype, alg, send, recv, n, root, stream); });
}

int fmi_comm_scan(fmi_comm_t comm, int op, int dtype, int alg, const void* send, void* recv, size_t n,
                  fmi_stream_t stream) {
    return on_stream("fmi_comm_scan", comm, stream, [&] { return comm_scan_impl(comm, op, dtype, alg, send, recv, n, stream); });
}

int fmi_comm_bcast(fmi_comm_t comm, void* buf, size_t bytes, int root, fmi_stream_t stream) {
    return on_stream("fmi_comm_bcast", comm, stream, [&] { return comm_bcast_impl(comm, buf, bytes, root, stream); });
}

int fmi_comm_gather(fmi_comm_t comm, const void* send, void* recv, size_t bytes, int root, fmi_stream_t stream) {
    return on_stream("fmi_comm_gather", comm, stream, [&] { return comm_gather_impl(comm, send, recv, bytes, root, stream); });
}

int fmi_comm_scatter(fmi_comm_t comm, const void* send, void* recv, size_t bytes, int root, fmi_stream_t stream) {
    return on_stream("fmi_comm_scatter", comm, stream, [&] { return comm_scatter_impl(comm, send, recv, bytes, root, stream); });
}

int fmi_comm_send(fmi_comm_t comm, const void* buf, size_t bytes, int peer, fmi_stream_t stream) {
    return on_stream("fmi_comm_send", comm, stream, [&] { return comm_send_impl(comm, buf, bytes, peer, stream); });
}

int fmi_comm_recv(fmi_comm_t comm, void* buf, size_t bytes, int peer, fmi_stream_t stream) {
    return on_stream("fmi_comm_recv", comm, stream, [&] { return comm_recv_impl(comm, buf, bytes, peer, stream); });
}

int fmi_comm_barrier(fmi_comm_t comm, fmi_stream_t stream) {
    return on_stream("fmi_comm_barrier", comm, stream, [&] { return comm_barrier_impl(comm, stream); });
}

int fmi_comm_unique_id(int transport, void* id, size_t len) {
    return guarded("fmi_comm_unique_id", [&] { return comm_unique_id_impl(transport, id, len); });
}

int fmi_comm_sync(fmi_comm_t comm, fmi_stream_t stream) {
    return guarded("fmi_comm_sync", [&]() -> int {
        if (!comm) return fail(FMI_ERR_INVALID, "null communicator");
        if (!library_stream()) return fail(FMI_ERR_NO_DEVICE, "fmi_dev_init has not been called");
        Comm* c = static_cast<Comm*>(comm);
        std::lock_guard<std::mutex> lk(c->mu);
        if (c->t->aborted()) return aborted_error();
        return c->t->wait_stream(resolve_stream(stream), "fmi_comm_sync");
    });
}

int fmi_comm_query(fmi_comm_t comm, int* count, int* rank, int* device) {
    return guarded("fmi_comm_query", [&]() -> int {
        if (!comm || !count || !rank || !device) return fail(FMI_ERR_INVALID, "null argument");
        Comm* c = static_cast<Comm*>(comm);
        std::lock_guard<std::mutex> lk(c->mu);
        if (c->t->aborted()) return aborted_error();
        return c->t->query(count, rank, device);
    });
}

int fmi_comm_rccl_info(int* version, char* path, size_t len) {
    return guarded("fmi_comm_rccl_info", [&]() -> int {
        const RcclApi* api = rccl_api();
        if (!api) return FMI_ERR_COMM;  // rccl_api() set the message (librccl missing or incomplete)
        int v = 0;
        if (api->GetVersion && api->GetVersion(&v) != ncclSuccess) v = 0;
        if (version) *version = v;
        if (path && len) {
            path[0] = '\0';
            Dl_info info{};
            if (dladdr(reinterpret_cast<void*>(api->GetUniqueId), &info) && info.dli_fname) {
                char real[4096];
                const char* name = realpath(info.dli_fname, real) ? real : info.dli_fname;
                std::snprintf(path, len, "%s", name);
            }
        }
        return FMI_OK;
    });
}

}  // extern "C"
