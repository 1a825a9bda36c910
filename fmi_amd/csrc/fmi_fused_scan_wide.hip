// Fused single-pass peer-axis scans for P = 17..31 (reference PeerToPeer::scan_no_order,
// src/comm/PeerToPeer.cpp:154-184, and scan_ltr, :141-152): all P inputs read and all P outputs written in
// one pass. Its own translation unit so these larger programs build in parallel with the rest.
#include "fmi_fused_impl.h"

namespace fmi::dev {
int launch_fused_scan_wide(int op, int dtype, int alg, int P, const PeerPtrs& ptrs, size_t n, hipStream_t s) {
    constexpr int LO = sched::kMaxFusedPeers + 1, HI = sched::kMaxFusedScanPeers;
    return alg == sched::kScan ? launch_fused<sched::kScan, false, LO, HI>(op, dtype, P, ptrs, n, 0, s)
                               : launch_fused<sched::kScanLtr, false, LO, HI>(op, dtype, P, ptrs, n, 0, s);
}
}  // namespace fmi::dev
