// Fused single-pass peer-axis scans in the order of reference PeerToPeer::scan_no_order
// (src/comm/PeerToPeer.cpp:154-184) and PeerToPeer::scan_ltr (src/comm/PeerToPeer.cpp:141-152), P = 2..16;
// 17..31 in fmi_fused_scan_wide.hip.
#include "fmi_fused_impl.h"

namespace fmi::dev {
int launch_fused_scan(int op, int dtype, int P, const PeerPtrs& ptrs, size_t n, hipStream_t s) {
    if (P > sched::kMaxFusedPeers) return launch_fused_scan_wide(op, dtype, sched::kScan, P, ptrs, n, s);
    return launch_fused<sched::kScan, false>(op, dtype, P, ptrs, n, 0, s);
}
int launch_fused_scan_ltr(int op, int dtype, int P, const PeerPtrs& ptrs, size_t n, hipStream_t s) {
    if (P > sched::kMaxFusedPeers) return launch_fused_scan_wide(op, dtype, sched::kScanLtr, P, ptrs, n, s);
    return launch_fused<sched::kScanLtr, false>(op, dtype, P, ptrs, n, 0, s);
}
int launch_fused_scan_carry(int op, int dtype, int P, const PeerPtrs& ptrs, size_t n, hipStream_t s) {
    return launch_fused<sched::kScanCarry, false>(op, dtype, P, ptrs, n, 0, s);
}
int launch_fused_scan_ltr_carry(int op, int dtype, int P, const PeerPtrs& ptrs, size_t n, hipStream_t s) {
    return launch_fused<sched::kScanLtrCarry, false>(op, dtype, P, ptrs, n, 0, s);
}
}  // namespace fmi::dev
