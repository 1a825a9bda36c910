/*
 * fmi_dev.h — C-ABI of the MI355X (gfx950) bucket-reduction engine behind FMI's collectives.
 *
 * This is the drop-in boundary for FMI's local element-wise bucket reduction. In the reference the
 * reduction is an opaque host closure, `raw_func = std::function<void(char*, char*)>`
 * (reference include/comm/Channel.h:16-23), built by Communicator::convert_to_raw_function
 * (reference include/Communicator.h:170-189) and applied by the PeerToPeer collectives as
 * `f.f(inout, in)` (reference src/comm/PeerToPeer.cpp:51,72,103,119,147,160,179).
 * Here the same combine is a HIP kernel launch on device-resident buckets, addressed by an explicit
 * op/dtype descriptor because the reference's closure carries neither.
 *
 * Conventions:
 *   - every entry point returns int: 0 = success, negative = fmi_status_t error; the message of the
 *     last failure on the calling thread is available from fmi_last_error(). No exception ever
 *     crosses this boundary; the C++ layer (fmi_amd/cpp/include/fmi/) rethrows std::runtime_error.
 *   - plain pointers and element counts only; no torch / HIP types in signatures. A stream is an
 *     opaque handle (hipStream_t underneath); NULL means the library's default stream of the device
 *     selected by fmi_dev_init.
 *   - the caller owns every buffer passed in; the library owns only its streams, events and scratch.
 *   - `inout`/`in` follow raw_func: argument 0 is overwritten, argument 1 is read-only, equal length.
 *   - all launches are asynchronous on the given stream; fmi_stream_sync / fmi_dev_sync wait.
 *
 * Element semantics match the reference's built-in ops (reference python/PythonCommunicator.h:116-149):
 *   SUM = a + b (std::plus), PROD = a * b (std::multiplies), MAX = std::max(a,b) = (a < b) ? b : a,
 *   MIN = std::min(a,b) = (b < a) ? b : a. Integer SUM/PROD wrap modulo 2^bits (two's complement), as
 *   the reference's int32 13! test relies on (reference tests/channels.cpp:419-465). Floats use IEEE
 *   round-to-nearest-even with denormals preserved and no contraction: a single device combine is
 *   bit-identical to the host one.
 */
#ifndef FMI_DEV_H
#define FMI_DEV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FMI_DEV_ABI_VERSION 1

/* ---- status ------------------------------------------------------------------------------------ */
typedef enum {
    FMI_OK = 0,
    FMI_ERR_INVALID = -1,     /* bad argument (null pointer, unknown op/dtype, P out of range ...) */
    FMI_ERR_HIP = -2,         /* a HIP runtime call failed; message names the call */
    FMI_ERR_NO_DEVICE = -3,   /* no gfx950 device visible / fmi_dev_init not called */
    FMI_ERR_UNSUPPORTED = -4, /* combination not implemented */
    FMI_ERR_ALLOC = -5,       /* device or pinned allocation failed */
    FMI_ERR_COMM = -6,        /* a communicator / transport (RCCL) call failed */
    FMI_ERR_TIMEOUT = -7      /* a peer did not arrive within the communicator's timeout (the reference's
                                 FMI::Utils::Timeout, include/utils/Common.h:11-15, raised by its channels
                                 when a peer stays away, src/comm/Direct.cpp:28-30,40-42). The communicator
                                 is aborted: later calls on it fail with FMI_ERR_COMM; destroy it. */
} fmi_status_t;

/* ---- op / dtype / algorithm descriptors -------------------------------------------------------- */
/* Op ids mirror the reference Python enum SUM/PROD/MAX/MIN (reference python/PythonCommunicator.h:13-15). */
typedef enum { FMI_OP_SUM = 0, FMI_OP_PROD = 1, FMI_OP_MAX = 2, FMI_OP_MIN = 3 } fmi_op_t;
/* Element types. The reference's buckets are Data<std::vector<A>> for any fundamental A
 * (include/comm/Data.h:50-73); f32 / f64 / i32 / i64 run every kernel, including the fused P-way ones.
 * The other integer widths run the pairwise kernel, and their P-way programs run as pairwise passes in
 * the same order (integer results do not depend on it). Integer sum / prod wrap, as the reference's
 * std::plus / std::multiplies do after conversion back to A. */
typedef enum {
    FMI_F32 = 0, FMI_F64 = 1, FMI_I32 = 2, FMI_I64 = 3,
    FMI_U32 = 4, FMI_U64 = 5, FMI_I8 = 6, FMI_U8 = 7, FMI_I16 = 8, FMI_U16 = 9
} fmi_dtype_t;

/* Evaluation orders reproduced by the P-way kernels; each is the combine order of one reference
 * collective, so a P-bucket reduction on one device is bit-identical to the distributed one. */
typedef enum {
    FMI_ALG_ALLREDUCE = 0,  /* recursive doubling + non-power-of-2 fold: PeerToPeer.cpp:96-130   */
    FMI_ALG_REDUCE = 1,     /* binomial tree toward root (transformed ids): PeerToPeer.cpp:59-84  */
    FMI_ALG_REDUCE_LTR = 2, /* gather + sequential left fold at root: PeerToPeer.cpp:44-57         */
    FMI_ALG_SCAN = 3,       /* binomial up/down sweep, own-op-received: PeerToPeer.cpp:154-184     */
    FMI_ALG_SCAN_LTR = 4    /* linear chain, prefix-op-own: PeerToPeer.cpp:141-152                 */
} fmi_alg_t;

typedef void* fmi_stream_t;
typedef void* fmi_event_t;

/* ---- library / device -------------------------------------------------------------------------- */
int fmi_abi_version(void);
/* Message of the last failed call on this thread ("" if none). Valid until the next failing call. */
const char* fmi_last_error(void);
/* Number of visible HIP devices (0 on a host without a GPU; never fails for lack of a device). */
int fmi_dev_count(int* count);
/* Select the device for this thread and create the library's default stream for it.
 * Fails with FMI_ERR_NO_DEVICE if the device is missing or is not gfx950. */
int fmi_dev_init(int device);
/* Release the library's streams and scratch (mirrors Channel::finalize, reference
 * include/comm/Channel.h:106). Buffers allocated by the caller are not touched. */
int fmi_dev_finalize(void);
/* Wait for all work on the selected device. */
int fmi_dev_sync(void);
/* Device name + arch string (e.g. "AMD Instinct MI355X gfx950"), CU count, HBM size, and the number of
 * fmi_host_reduce_pair staging sets ("host_pipelines=N idle=M": one per calling thread alive, idle ones are
 * those of exited threads, reused by the next new caller), NUL-terminated into buf. */
int fmi_dev_describe(char* buf, size_t len);
/* PCI bus id ("dddd:bb:dd.f") of a visible device, NUL-terminated into buf (hipDeviceGetPCIBusId): with
 * fmi_comm_query, lets the ranks of a communicator show they sit on distinct GPUs. */
int fmi_dev_pci_bus_id(int device, char* buf, size_t len);

/* ---- memory (replaces the reference's new[]/std::vector bucket storage, include/comm/Data.h:50-97)
 * fmi_dev_alloc: device memory, 4 KiB aligned: a plain hipMalloc (the pairwise kernel's best placement), or with
 * FMI_TUNE_ALLOC_SLOTS = 1 buckets of >= 1 MiB in rotating 4 KiB slots. Free with fmi_dev_free only (a slotted
 * pointer lies inside its hipMalloc, up to 60 KiB past its base, so it is not a hipIpcGetMemHandle base either:
 * memory shared across processes comes from fmi_comm_window_alloc). */
int fmi_dev_alloc(void** ptr, size_t bytes);
/* fmi_dev_alloc_group: `count` buckets of `bytes` each that one kernel streams together (a fused kernel's P
 * inputs and its outputs). Buckets of >= 1 MiB are carved from ONE allocation at a stride of `bytes` rounded up to
 * 64 KiB plus 4 KiB, so bucket j sits in 4 KiB slot j mod 16 (modulo 64 KiB) whatever was allocated before and
 * whatever FMI_TUNE_ALLOC_SLOTS says, and the group's streams never collide in HBM; smaller ones are
 * plain allocations. All or nothing: on failure every ptrs[j] is NULL. Free each with fmi_dev_free, in any order: a
 * carved group's memory is released with its last bucket. */
int fmi_dev_alloc_group(void** ptrs, int count, size_t bytes);
int fmi_dev_free(void* ptr);
int fmi_host_pin_alloc(void** ptr, size_t bytes);  /* page-locked host memory for recv buffers */
int fmi_host_pin_free(void* ptr);
/* Page-lock an existing host range in place (hipHostRegister, mapped), e.g. a channel recv buffer that is
 * reused across collectives (reference include/comm/Data.h:50-73 std::vector storage), so that
 * fmi_host_reduce_pair combines it zero-copy and the host pipelines move it at DMA rate. Registering
 * costs about as much as one copy of the range: worth it only for buffers used more than once. The range
 * must stay allocated until fmi_host_unregister(ptr) with the same ptr. A bucket handed to
 * fmi_host_reduce_pair must lie wholly inside one page-locked range or wholly outside any
 * (FMI_ERR_INVALID otherwise). */
int fmi_host_register(void* ptr, size_t bytes);
int fmi_host_unregister(void* ptr);
/* The device address of [host, host + bytes), a range wholly inside one page-locked, device-mapped range
 * (fmi_host_pin_alloc / fmi_host_register): what a caller hands to fmi_dev_reduce_pair to combine host recv
 * buffers in place over PCIe. FMI_ERR_INVALID for pageable or straddling ranges. */
int fmi_host_device_ptr(const void* host, size_t bytes, void** dev);
/* 1 if [host, host + bytes) lies wholly inside one page-locked, device-mapped range, else 0 (also before
 * fmi_dev_init). A query, not a request: it never sets fmi_last_error (the Communicator asks it per host combine,
 * where a pageable bucket is the ordinary answer, ChannelPolicy::host_combine_on_device). */
int fmi_host_page_locked(const void* host, size_t bytes);
int fmi_dev_h2d_async(void* dst, const void* src, size_t bytes, fmi_stream_t stream);
int fmi_dev_d2h_async(void* dst, const void* src, size_t bytes, fmi_stream_t stream);
int fmi_dev_d2d_async(void* dst, const void* src, size_t bytes, fmi_stream_t stream);
int fmi_dev_memset_async(void* dst, int value, size_t bytes, fmi_stream_t stream);

/* ---- streams / events (timing is taken on the stream the kernels run on) ----------------------- */
int fmi_stream_create(fmi_stream_t* stream);
int fmi_stream_destroy(fmi_stream_t stream);
int fmi_stream_sync(fmi_stream_t stream);
int fmi_event_create(fmi_event_t* event);
int fmi_event_destroy(fmi_event_t event);
int fmi_event_record(fmi_event_t event, fmi_stream_t stream);
int fmi_event_sync(fmi_event_t event);
/* Work enqueued on `stream` after this call waits for `event`'s last record (cross-stream ordering, e.g.
 * a combine on one stream feeding a collective on another). */
int fmi_stream_wait_event(fmi_stream_t stream, fmi_event_t event);
int fmi_event_elapsed_ms(float* ms, fmi_event_t start, fmi_event_t stop);

/* ---- HIP graphs: a launch-bound sequence (many small bucket combines, e.g. FMI's 1 MiB messages) is
 * recorded once and replayed as one submission. Between capture_begin and capture_end on a stream made by
 * fmi_stream_create, calls on that stream are recorded, not run. Capture-safe: fmi_dev_reduce_pair,
 * fmi_dev_combine, the d2d / memset copies, and fmi_dev_reduce_tree / fmi_dev_scan_peers up to 16 peers
 * (one fused kernel each). Everything else (host-ingress paths, communicators, P > 16 programs, which
 * may allocate or synchronise) is not: that call or capture_end fails, the graph is discarded, and the
 * stream must be destroyed and replaced (HIP leaves a stream whose capture was invalidated unusable).
 * Pointers and sizes are frozen in the graph; replays recompute the same buckets. */
typedef void* fmi_graph_t;
int fmi_graph_capture_begin(fmi_stream_t stream);
int fmi_graph_capture_end(fmi_stream_t stream, fmi_graph_t* graph);
int fmi_graph_launch(fmi_graph_t graph, fmi_stream_t stream);
int fmi_graph_destroy(fmi_graph_t graph);

/* ---- the hot path ------------------------------------------------------------------------------ */
/* Pairwise bucket combine: inout[i] = op(inout[i], in[i]) for i < n.
 * Replaces one application of the raw_func built by Communicator::convert_to_raw_function
 * (reference include/Communicator.h:180-189) at the PeerToPeer combine sites
 * (reference src/comm/PeerToPeer.cpp:51,72,103,119,147,160,179). inout == in is allowed. */
int fmi_dev_reduce_pair(int op, int dtype, void* inout, const void* in, size_t n, fmi_stream_t stream);

/* Batched pairwise combine: for every descriptor k, descs[k].inout[i] = op(inout[i], in[i]) for
 * i < descs[k].n, all of them in as few launches as possible (up to 64 descriptors per launch): the same
 * bits as `count` calls of fmi_dev_reduce_pair, without a launch and its ramp per bucket — for many small
 * buckets (FMI's 1 MiB messages). `descs` is host memory, read during the call. A descriptor's inout must
 * not overlap another descriptor's inout or in (FMI_ERR_INVALID); inout == in is allowed. n = 0 entries are
 * skipped; unaligned or very large buckets are combined by their own launch. Graph-capturable. */
typedef struct {
    void* inout;
    const void* in;
    size_t n;
} fmi_pair_desc_t;
int fmi_dev_reduce_pair_batch(int op, int dtype, const fmi_pair_desc_t* descs, int count, fmi_stream_t stream);

/* Out-of-place pairwise combine: out[i] = op(a[i], b[i]); out may alias a or b. */
int fmi_dev_combine(int op, int dtype, void* out, const void* a, const void* b, size_t n,
                    fmi_stream_t stream);

/* P-way reduction of P device buckets in one pass with the evaluation order of `alg`
 * (FMI_ALG_ALLREDUCE / FMI_ALG_REDUCE / FMI_ALG_REDUCE_LTR): out = the value peer `rank` holds at the
 * end of the reference collective (for FMI_ALG_REDUCE `rank` is the root; for ALLREDUCE it selects
 * whose operand order is reproduced, which differs only for float MAX/MIN on signed zeros).
 * Replaces the whole chain of f.f calls of reference PeerToPeer::allreduce_no_order / reduce_no_order /
 * reduce_ltr (src/comm/PeerToPeer.cpp:96-130, :59-84, :44-57) for buckets that sit on one device.
 * ins[p] = bucket of peer p (p < P); out may alias any ins[p]. Any P >= 1 (no peer cap, as in the
 * reference). One fused kernel (a single
 * pass over the P buckets) for P <= 16, and for ALLREDUCE up to 31; larger P as fused sub-programs of the
 * identical order over blocks of 16 peers (every input read once, plus one write and one read per block
 * value). Unaligned buckets and the 8/16-bit dtypes run the same order as pairwise passes. */
int fmi_dev_reduce_tree(int op, int dtype, int alg, void* out, const void* const* ins, int P, int rank,
                        size_t n, fmi_stream_t stream);

/* Peer-axis inclusive scan of P device buckets: outs[k] = x0 (+) ... (+) xk with the evaluation order
 * of `alg` (FMI_ALG_SCAN or FMI_ALG_SCAN_LTR). Replaces reference PeerToPeer::scan_no_order / scan_ltr
 * (src/comm/PeerToPeer.cpp:154-184, :141-152) and Communicator::scan (include/Communicator.h:135-150)
 * when the P buckets sit on one device. outs[k] may alias ins[k]. Any P >= 1: one fused pass up to 31
 * peers; beyond, every input is read at most twice (block totals, then the blocks continued from their
 * carry). */
int fmi_dev_scan_peers(int op, int dtype, int alg, void* const* outs, const void* const* ins, int P,
                       size_t n, fmi_stream_t stream);

/* Host-resident pairwise combine through the device: pinned (or pageable) host `inout`/`in` are
 * streamed through device staging in chunks (H2D, kernel, D2H overlapped on two streams).
 * This is the path a recv buffer arriving over a host channel takes (reference
 * src/comm/Direct.cpp:36-45 → PeerToPeer.cpp:119). Synchronous: returns when inout is updated. */
int fmi_host_reduce_pair(int op, int dtype, void* inout, const void* in, size_t n);

/* ---- sharded device collectives across GPUs (one process per GPU, RCCL over xGMI) ----------------
 * The reference's collectives exchange whole buckets peer to peer over host sockets
 * (src/comm/PeerToPeer.cpp). Between MI355X GPUs the same collectives run sharded, so every GPU's 7
 * xGMI links carry traffic at once, with the combine done by the fused kernels above in the reference's
 * order:
 *   allreduce (path TREE): all-to-all of N shards -> fused P-way kernel over the N partials of this
 *       GPU's shard (allreduce_no_order / reduce_ltr order) -> all-gather. Bit-identical to the
 *       reference's N-peer allreduce on every rank, each rank with its OWN operand order: for float
 *       max/min (whose ±0 ties and NaNs depend on it) the shard owner computes its shard in every rank's
 *       order and an all-to-all replaces the all-gather, so rank r receives what reference peer r holds.
 *   allreduce (path RCCL): RCCL reduce-scatter + all-gather (RCCL's order; within (N-1)*u*sum|x|).
 *   reduce: all-to-all -> fused kernel in reduce_no_order / reduce_ltr order for `root` -> gather.
 *   scan:   all-to-all -> fused peer-axis scan -> all-to-all back.
 * One rank = one peer = one GPU. Transports: FMI_TRANSPORT_RCCL (librccl, loaded on first use; with
 * torch imported first it is torch's copy), FMI_TRANSPORT_LOCAL (ranks are threads of ONE process
 * sharing one device: the same schedules over device-to-device copies — used to test the multi-rank
 * schedules on a single GPU and to serve several peers co-resident on one GPU) and FMI_TRANSPORT_PROC
 * (ranks are processes of one node, on the same or different GPUs: data staged through a page-locked
 * POSIX shared-memory segment, windows mapped with HIP IPC — the same schedules again, so multi-process
 * runs, FMI_PATH_DIRECT's cross-process mappings included, are testable on a single GPU).
 * All calls enqueue on `stream` (NULL = library stream); results are valid after fmi_stream_sync.
 * Buckets are device pointers; recv may alias send.
 * Side effect on `send` — a deliberate divergence from the reference: the reference's commutative
 * allreduce / scan leave the result in the caller's sendbuf and its reduce leaves partials in interior
 * peers' sendbufs (src/comm/PeerToPeer.cpp:72,103,119,160,179). Here `send` is never modified by
 * allreduce, reduce or scan, so a C-ABI caller that relied on the clobber passes recv == send (allreduce,
 * scan) to get it. The C++ channel FMI::Comm::Rccl (fmi_amd/cpp/include/fmi/comm/Rccl.h) restores the
 * reference's side effects itself, so Communicator callers see the reference behaviour. */
#define FMI_COMM_ID_BYTES 128
typedef void* fmi_comm_t;
typedef enum { FMI_TRANSPORT_RCCL = 0, FMI_TRANSPORT_LOCAL = 1, FMI_TRANSPORT_PROC = 2 } fmi_transport_t;
/* FMI_PATH_DIRECT: no RCCL data movement. `send` must lie in a window (fmi_comm_window_alloc) at the SAME
 * byte offset and with the same n on every rank: rank k reads every peer's window at its own offset (windows
 * are equal-sized, so a mismatch reads wrong data, never outside a window). With FMI_CHECK_DIRECT=1 in the
 * environment every call first compares the (offset, n) pairs across ranks (a blocking all-reduce) and a
 * mismatch fails the call on every rank with FMI_ERR_INVALID. Rank k's fused kernel reads shard k of every rank's window over xGMI (IPC-mapped peer
 * memory) and reduces it in the reference's order, then every rank reads the N reduced shards from the
 * peers' windows. Bit-identical to FMI_PATH_TREE. */
typedef enum { FMI_PATH_TREE = 0, FMI_PATH_RCCL = 1, FMI_PATH_DIRECT = 2 } fmi_path_t;

/* A fresh communicator id (FMI_COMM_ID_BYTES) made by one rank and handed to the others by any host
 * channel (FMI: Communicator::bcast over the host channel, reference include/Communicator.h:43-47). */
int fmi_comm_unique_id(int transport, void* id, size_t len);
/* Timeouts. Every wait of a communicator for its peers is bounded by its timeout: the rendezvous of
 * fmi_comm_init (RCCL: non-blocking ncclCommInitRankConfig, polled), the transport's own host-side waits
 * (PROC / LOCAL barriers and mailboxes, RCCL barriers and window setup) and fmi_comm_sync. On expiry the
 * call returns FMI_ERR_TIMEOUT and the communicator is aborted (RCCL: ncclCommAbort, which also ends its
 * kernels still waiting for the absent peer). fmi_comm_init uses FMI_COMM_TIMEOUT_S from the environment
 * (seconds; for PROC also FMI_PROC_TIMEOUT_S), default 300; fmi_comm_init_timeout takes it explicitly
 * (timeout_s <= 0: that default). An asynchronous transport error seen while waiting (RCCL
 * ncclCommGetAsyncError: a peer's connection failed) also aborts the communicator, with FMI_ERR_COMM. */
int fmi_comm_init(fmi_comm_t* comm, const void* id, int nranks, int rank);
int fmi_comm_init_timeout(fmi_comm_t* comm, const void* id, int nranks, int rank, double timeout_s);
int fmi_comm_destroy(fmi_comm_t comm);
int fmi_comm_size(fmi_comm_t comm, int* nranks, int* rank);
/* Wait until the work enqueued on `stream` (NULL = library stream) has completed — the blocking point of
 * the collectives, which enqueue asynchronously — within the communicator's timeout, polling the transport
 * for asynchronous errors (FMI_ERR_TIMEOUT / FMI_ERR_COMM as above). */
int fmi_comm_sync(fmi_comm_t comm, fmi_stream_t stream);
/* What the transport itself reports: RCCL ncclCommCount / ncclCommUserRank / ncclCommCuDevice (the device
 * RCCL bound this rank to); LOCAL / PROC the communicator's size, rank and the calling thread's device.
 * Lets a caller prove the topology it runs on (bench.py: RCCL saw N ranks on N distinct GPUs). */
int fmi_comm_query(fmi_comm_t comm, int* count, int* rank, int* device);
/* The librccl the RCCL transport uses (loaded on first use: with torch imported first, torch's copy): its
 * ncclGetVersion (0 if it lacks the symbol) and the real path of the mapped object, NUL-terminated into
 * path. FMI_ERR_COMM if librccl cannot be loaded. Lets a failed multi-GPU run name the RCCL it ran on. */
int fmi_comm_rccl_info(int* version, char* path, size_t len);
/* Symmetric window for FMI_PATH_DIRECT (collective: every rank calls it with the same `bytes`). Returns a
 * device bucket of `bytes` that every peer of the communicator can read directly (RCCL transport: HIP IPC
 * handles exchanged by all-gather, mapped with peer access over xGMI). All-or-nothing: if any rank cannot
 * allocate, export or map, every rank gets an error. Freed (collectively) by fmi_comm_window_free or with
 * the communicator: both first wait for all work on this rank's device (any stream may still be reading
 * a peer's window through its mapping), then barrier with the peers, then unmap and free. */
int fmi_comm_window_alloc(fmi_comm_t comm, size_t bytes, void** ptr);
int fmi_comm_window_free(fmi_comm_t comm, void* ptr);
/* Live timing of the collectives' shard kernels (the fused P-way kernel each rank runs on its shard, path
 * TREE / DIRECT allreduce): while enabled, an event pair is recorded around every such launch on the stream
 * it runs on (up to 8192 launches). fmi_comm_timing_read waits for them and returns the summed kernel time
 * and the launch count, then starts a new tally. Enabling also starts a new tally. */
int fmi_comm_timing(fmi_comm_t comm, int enable);
int fmi_comm_timing_read(fmi_comm_t comm, float* total_ms, int* launches);
/* alg: FMI_ALG_ALLREDUCE (commutative+associative) or FMI_ALG_REDUCE_LTR (ordered) */
int fmi_comm_allreduce(fmi_comm_t comm, int op, int dtype, int alg, int path, const void* send, void* recv, size_t n,
                       fmi_stream_t stream);
/* Host-ingress allreduce (BASELINE config C5): `send` / `recv` are HOST buckets, i.e. the channel recv
 * buffers FMI's transports deliver into (reference src/comm/Direct.cpp:36-45, PeerToPeer.cpp:110-129).
 * The bucket streams through the GPU in chunks of `chunk` elements (0 = FMI_TUNE_HOST_CHUNK bytes):
 * H2D of chunk k+1, the sharded allreduce of chunk k and D2H of chunk k-1 overlap on three streams.
 * Every rank must pass the same n and chunk. Page-locked buckets (fmi_host_pin_alloc) move at PCIe DMA
 * rate; pageable ones work but copy synchronously. Element-wise results are identical to
 * fmi_comm_allreduce over the whole bucket. Blocking: returns when `recv` holds the result. */
int fmi_comm_allreduce_host(fmi_comm_t comm, int op, int dtype, int alg, int path, const void* send, void* recv,
                            size_t n, size_t chunk);
/* alg: FMI_ALG_REDUCE or FMI_ALG_REDUCE_LTR; recv is used on root only (may be NULL elsewhere) */
int fmi_comm_reduce(fmi_comm_t comm, int op, int dtype, int alg, const void* send, void* recv, size_t n, int root,
                    fmi_stream_t stream);
/* fmi_comm_reduce with the reference's side effect on every rank's sendbuf (src/comm/PeerToPeer.cpp:59-84,
 * combine site :72): after the call rank r's `send` holds what reference peer r leaves in its sendbuf —
 * for FMI_ALG_REDUCE the partial it forwarded up the binomial tree (a leaf's own bucket, the root's
 * result), for FMI_ALG_REDUCE_LTR its own bucket unchanged (:44-57). recv (root only) gets the result, as
 * with fmi_comm_reduce. Costs N shard writes on each owner and an all-to-all back instead of a gather. */
int fmi_comm_reduce_sendbuf(fmi_comm_t comm, int op, int dtype, int alg, void* send, void* recv, size_t n, int root,
                            fmi_stream_t stream);
/* alg: FMI_ALG_SCAN or FMI_ALG_SCAN_LTR; rank k receives x0 (+) ... (+) xk */
int fmi_comm_scan(fmi_comm_t comm, int op, int dtype, int alg, const void* send, void* recv, size_t n,
                  fmi_stream_t stream);
int fmi_comm_bcast(fmi_comm_t comm, void* buf, size_t bytes, int root, fmi_stream_t stream);
/* recv holds nranks * bytes on root (rank order); scatter sends root's nranks * bytes */
int fmi_comm_gather(fmi_comm_t comm, const void* send, void* recv, size_t bytes, int root, fmi_stream_t stream);
int fmi_comm_scatter(fmi_comm_t comm, const void* send, void* recv, size_t bytes, int root, fmi_stream_t stream);
int fmi_comm_send(fmi_comm_t comm, const void* buf, size_t bytes, int peer, fmi_stream_t stream);
int fmi_comm_recv(fmi_comm_t comm, void* buf, size_t bytes, int peer, fmi_stream_t stream);
int fmi_comm_barrier(fmi_comm_t comm, fmi_stream_t stream);

/* ---- synthetic buckets (identical on host and device: SURVEY.md §8d generator) ------------------
 * h = splitmix64(seed ^ ((uint64)peer << 40) ^ i);  f32 = (float)((h >> 40) * 2^-24) * 2 - 1,
 * f64 = (double)((h >> 11) * 2^-53) * 2 - 1,  i32 = (int32)(h >> 32),  i64 = (int64)h. */
int fmi_dev_fill_synthetic(int dtype, void* buf, size_t n, uint64_t seed, uint32_t peer,
                           fmi_stream_t stream);
/* Elements [first, first + n) of the same synthetic bucket (i runs from `first`): lets a rank rebuild any
 * window of every peer's bucket locally, e.g. to check a sharded collective's result on sampled ranges. */
int fmi_dev_fill_synthetic_at(int dtype, void* buf, size_t n, uint64_t seed, uint32_t peer, uint64_t first,
                              fmi_stream_t stream);

/* ---- schedule introspection (host-only logic, no device needed) --------------------------------
 * Writes the symbolic combine expression peer `rank` ends with, e.g. "((x0+x1)+(x2+x3))", as the
 * fused kernels evaluate it. Used by the parity tests to pin the order against the reference's. */
int fmi_schedule_expr(int alg, int P, int rank, char* buf, size_t len);

/* ---- tuning knobs (performance only, never semantics) ------------------------------------------ */
typedef enum {
    FMI_TUNE_PAIR_VARIANT = 0, /* 0 = one-shot tiles, 1 = grid-stride, 2 = nontemporal tiles (default),
                                  3 = tiles with nontemporal loads only, 4 = nontemporal stores only */
    FMI_TUNE_PAIR_UNROLL = 1,  /* 16-B vectors per thread per operand: 1, 2, 4, 8 */
    FMI_TUNE_BLOCK = 2,        /* threads per workgroup: 256, 512, 1024 */
    FMI_TUNE_GRID_PER_CU = 3,  /* workgroups per CU for the grid-stride variant */
    FMI_TUNE_HOST_CHUNK = 4,   /* bytes per chunk of fmi_host_reduce_pair's staged pipeline */
    FMI_TUNE_HOST_ZERO_COPY = 5, /* 1: page-locked host buckets are combined in place over PCIe by the
                                   kernel (no staging); 0: always the staged H2D/kernel/D2H pipeline */
    FMI_TUNE_FUSED_INFLIGHT_KIB = 6, /* fused P-way kernels (tree, scan): budget of peer-load bytes in
                                       flight per CU, in KiB; a workgroup of the P-way kernel loads
                                       4 KiB x P, so at most max(2, ceil(budget / (4 P))) workgroups stay
                                       resident per CU (an LDS reservation enforces it); 0 = no cap. Default 64
                                       (fewer concurrent HBM streams at large P) */
    FMI_TUNE_BLOCKS_ONE_PASS = 7, /* P-way programs beyond 31 peers in one pass over every input (default 1):
                                    scan_no_order over 32..143 peers, reduce_no_order over 17..128 peers
                                    (beyond: superblocks of 128, one pass each, up to 16384 peers),
                                    allreduce_no_order over 32 / 48 / 64 / 80 / 96 / 112 / 128
                                    peers (2^k >= 128 peers: superblocks of 64), scan_ltr and
                                    reduce_ltr over 32..128 peers (beyond: segments of 127 continued
                                    from the running value, any P);
                                    0 = the blocked launches (block values through temps; the scan reads
                                    the inputs of blocks >= 1 twice). Same bits either way */
    FMI_TUNE_COMM_A2A = 8,        /* RCCL transport all-to-all: 0 = ncclAllToAll where librccl has it (default),
                                    1 = grouped ncclSend / ncclRecv to every peer. Same bytes either way.
                                    EVERY rank of a communicator must use the same value: the two forms post
                                    different RCCL operations, and ranks that disagree hang (until the
                                    communicator's timeout) */
    FMI_TUNE_COMM_GATHER = 9,     /* RCCL transport all-gather: 0 = ncclAllGather (default), 1 = grouped
                                    ncclSend / ncclRecv of this rank's shard to every peer (each peer link
                                    carries one shard, no ring). Same bytes either way. EVERY rank must use the
                                    same value (as FMI_TUNE_COMM_A2A) */
    FMI_TUNE_COMM_PIPELINE = 10,  /* EXPERIMENTAL (not yet run over RCCL with more than one rank). Path TREE
                                    allreduce in K chunks (0 or 1 = off, default; 2..64): chunk k's
                                    all-gather runs on a second stream and a second communicator (made
                                    once: a fresh id broadcast over the first, then a bounded init)
                                    while chunk k + 1's all-to-all and kernel run; chunks of >= 1 MiB per
                                    rank only. If the second communicator cannot be made, the unpipelined path runs.
                                    Same bits (element-wise); EVERY rank must set the same K */
    FMI_TUNE_FUSED_POLICY = 11,   /* fused P-way kernels (tree, scan; <= 16 peers), 16-B accesses: 2 = buffer
                                    loads nt with sc1 (tree) / nt sc1 (scan) stores; 0 = global_load /
                                    global_store nt; 1 = auto (default): 2 for trees of >= 4 and scans of
                                    >= 8 peers, 0 otherwise (tools/ab_fused_policy.py). Same bits always */
    FMI_TUNE_PAIR_SC1_OF_8 = 12,  /* pairwise kernel (16-B aligned buckets, one-shot tiles): tiles t with
                                    t % 8 < k store with sc1 instead of nontemporal (k = 0..8). Consecutive
                                    workgroups are dispatched to different XCDs, so k of the 8 XCDs store sc1.
                                    Default 1 (tools/ab_pair_sc1.py, measured with no MALL re-use). Same bits
                                    always */
    FMI_TUNE_COMM_ONE_RANK_EXCHANGE = 13, /* 1: a ONE-rank communicator runs the full sharded schedule —
                                    all-to-all, shard kernel, all-gather / gather / all-to-all back, RCCL
                                    reduce-scatter, window mapping, the pipelined split — exchanging with
                                    itself, instead of the reference's P = 1 copy. Same bits; exists so that
                                    a 1-GPU box runs the RCCL transport's real collectives (tests). Default 0 */
    FMI_TUNE_ALLOC_SLOTS = 14     /* fmi_dev_alloc of >= 1 MiB: 0 (default since round 6) = plain hipMalloc;
                                    1 = place successive buckets in successive of 16 4-KiB slots (modulo 64 KiB)
                                    of a hipMalloc 64 KiB larger (round 5). The buckets of one fused kernel belong
                                    in one fmi_dev_alloc_group, which places them whatever this says.
                                    fmi_dev_free takes either. Same bits */,
    FMI_TUNE_COMM_SHARD_SKEW = 15 /* sharded collectives (path TREE allreduce): 1 (default) = the all-to-all lands
                                    the N shards the fused shard kernel streams together in distinct 4 KiB slots
                                    (stride: the shard rounded up to 64 KiB plus 4 KiB), its output in the next one,
                                    where the transport posts a receive per peer anyway (LOCAL, PROC, RCCL's grouped
                                    form, FMI_TUNE_COMM_A2A set to 1; never ncclAllToAll); 0 = back to back. Shards under
                                    1 MiB stay back to back. Ranks may differ (only local placement changes). Same
                                    bits */
} fmi_tune_key_t;
int fmi_tune_set(int key, long long value);
int fmi_tune_get(int key, long long* value);

#ifdef __cplusplus
}
#endif

#endif /* FMI_DEV_H */
