// Batched pairwise combine: K independent bucket pairs (descriptors) in ONE launch, for buckets too small
// to amortise a launch and its ramp each (FMI's 1 MiB messages: one launch per combine costs ~4.8 µs for
// ~0.5 µs of HBM traffic). Every element is combined exactly as by fmi_dev_reduce_pair (same pair_tile
// body, same tail), so the bits are those of K separate calls (reference include/Communicator.h:180-189,
// one raw_function application per descriptor).
#include "fmi_internal.h"
#include "fmi_kernels.h"

namespace fmi::dev {
namespace {

template <class Op, class T>
__global__ void __launch_bounds__(kPairBatchBlock) pair_batch_kernel(PairBatch pb) {
    constexpr int W = kVecLanes<T>;
    const unsigned t = blockIdx.x;
    int lo = 0, hi = pb.count - 1;  // the descriptor whose tile range holds t (uniform: scalar search)
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (pb.first_tile[mid] <= t)
            lo = mid;
        else
            hi = mid - 1;
    }
    T* out = static_cast<T*>(pb.inout[lo]);
    const T* b = static_cast<const T*>(pb.in[lo]);
    const size_t n = pb.n[lo];
    const size_t nvec = n / W;
    const size_t tile = t - pb.first_tile[lo];
    pair_tile_body<Op, T, kPairBatchUnroll, 3>(out, out, b, nvec, tile);
    if (t + 1 == pb.first_tile[lo + 1] && nvec * W + threadIdx.x < n) {  // the last tile takes the < 16-B tail
        const size_t i = nvec * W + threadIdx.x;
        out[i] = Op::template apply<T>(out[i], b[i]);
    }
}

}  // namespace

int launch_pair_batch(int op, int dtype, const PairBatch& pb, hipStream_t s) {
    if (pb.count <= 0) return FMI_OK;
    return with_op_dtype(op, dtype, [&]<class Op, class T>() -> int {
        pair_batch_kernel<Op, T><<<pb.first_tile[pb.count], kPairBatchBlock, 0, s>>>(pb);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return fail(FMI_ERR_HIP, std::string("batched pairwise kernel launch: ") + hipGetErrorString(e));
        return FMI_OK;
    });
}

}  // namespace fmi::dev
