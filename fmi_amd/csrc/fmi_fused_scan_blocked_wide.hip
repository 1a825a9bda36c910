// The one-pass blocked scan (fmi_fused_scan_blocked.hip) for 5..8 full blocks of 16 peers (P = 80..143): its own
// translation unit so these larger programs build in parallel with the rest.
#include "fmi_fused_impl.h"
#include "fmi_scan_blocks_impl.h"

namespace fmi::dev {

int launch_scan_blocks_one_pass_wide(int op, int dtype, int B, const BlockedScanPtrs& ptrs, size_t n, hipStream_t s) {
    return scan_blocks::launch_range<kOnePassScanBlocksNarrow + 1, kMaxOnePassScanBlocks>(op, dtype, B, ptrs, n, s);
}

}  // namespace fmi::dev
