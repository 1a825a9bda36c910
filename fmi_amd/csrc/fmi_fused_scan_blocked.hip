// One-pass peer-axis scan_no_order beyond 31 peers (reference PeerToPeer::scan_no_order,
// src/comm/PeerToPeer.cpp:154-184): P = 16 B + r with 2 <= B <= kMaxOnePassScanBlocks full blocks of 16 peers.
//
// scan_blocked (fmi_dev.hip) evaluates the same bracketing as separate launches — block 0's scan, every
// later block's up-sweep total, the scan over the totals, then each block's carry program — which reads
// every input of blocks >= 1 twice. Here one thread walks the blocks of its lane group in peer order:
//   block 0:   the fused 16-peer scan; its last output is T_0 = S_0;
//   block b:   load the block's 16 inputs once; T_b = the block's up-sweep total (the binomial reduce over
//              the block in reverse order); the block-level scan's steps whose operands are all known by
//              now (the steps "ready at b": their leaves are T_0..T_b) give S_b; the kScanCarry program
//              from S_{b-1} gives the block's first 15 outputs, S_b its last.
// Output b of scan_no_order depends only on inputs 0..b (a down-sweep round never sends from a later peer),
// so S_b is ready at b — static_assert'ed in fmi_scan_blocks_impl.h. The bits are those of scan_blocked: same programs, same
// operand order. A ragged last block (r > 0) is the same carry launch scan_blocked uses, from S_{B-1}.
// Bucket passes: 2P, plus one carry read for a ragged block (P = 64: 128 instead of scan_blocked's 184).
#include "fmi_fused_impl.h"
#include "fmi_scan_blocks_impl.h"

namespace fmi::dev {

int launch_scan_blocks_one_pass(int op, int dtype, int B, const BlockedScanPtrs& ptrs, size_t n, hipStream_t s) {
    if (B > kOnePassScanBlocksNarrow) return launch_scan_blocks_one_pass_wide(op, dtype, B, ptrs, n, s);
    return scan_blocks::launch_range<2, kOnePassScanBlocksNarrow>(op, dtype, B, ptrs, n, s);
}

}  // namespace fmi::dev
