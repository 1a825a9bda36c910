// fmi_schedule.h — combine order of FMI's PeerToPeer collectives as a static single-assignment program.
//
// Each reference collective (reference src/comm/PeerToPeer.cpp) is a fixed pattern of sends, receives
// and local combines `f.f(mine, received)`. Because every peer's sequence depends only on (P, peer id),
// the whole collective collapses into a straight-line program over value ids:
//
//     values 0..P-1          = the peers' input buckets (x0 .. x{P-1})
//     value  P+s             = op(value[step[s].a], value[step[s].b])     (left operand = arg 0 of f.f)
//     out[r]                 = the value id peer r holds when the collective returns
//
// The fused HIP kernels (fmi_kernels.h) evaluate this program per element with every value in VGPRs,
// so P buckets resident on one device reduce in ONE pass over HBM with the reference's exact bracketing.
// Everything here is constexpr: the device instantiates programs at compile time (static register
// indices after unrolling), the host builds the same programs at run time for P > kMaxFusedPeers.
//
// Round-synchronous restatement: in every round of every algorithm below a peer either sends or
// receives+combines, never both, so a peer's outgoing value in round i is its value after round i-1.
// That is why a single pass over peers per round reproduces the message-passing order exactly.
#pragma once

#include <cstdint>
#include <type_traits>
#include <vector>

namespace fmi::sched {

enum Alg : int {
    kAllreduce = 0,  // reference PeerToPeer::allreduce_no_order  (src/comm/PeerToPeer.cpp:96-130)
    kReduce = 1,     // reference PeerToPeer::reduce_no_order     (src/comm/PeerToPeer.cpp:59-84)
    kReduceLtr = 2,  // reference PeerToPeer::reduce_ltr          (src/comm/PeerToPeer.cpp:44-57)
    kScan = 3,       // reference PeerToPeer::scan_no_order       (src/comm/PeerToPeer.cpp:154-184)
    kScanLtr = 4,    // reference PeerToPeer::scan_ltr            (src/comm/PeerToPeer.cpp:141-152)
    // Internal pieces of the scans beyond kMaxFusedPeers (not in the C-ABI): value 0 is a carry, the
    // prefix of every peer before this block; values 1..P-1 are the block's peers; out[0] is not stored.
    kScanCarry = 5,     // one block of 16 consecutive scan_no_order peers, b >= 1, after the block rounds
    kScanLtrCarry = 6,  // the scan_ltr chain continued from the carry
    // One 16-peer block of allreduce_no_order (P_all > 32) whose 16 peers all take a pre-fold: 32 inputs,
    // values 16 + j are the partners peer j folds in first; then the 16-peer recursive doubling.
    kAllreducePrefold16 = 7,
    // reduce_no_order's program with every peer's final value as an output: out[t] is the value transformed
    // peer t leaves in its sendbuf (the partial it forwarded; a leaf's own bucket; the root's result).
    kReducePartials = 8,
};

inline constexpr bool is_carry_alg(int alg) { return alg == kScanCarry || alg == kScanLtrCarry; }
// Programs whose kernels store every peer's output (not one peer's).
inline constexpr bool stores_all_outputs(int alg) {
    return alg == kScan || alg == kScanLtr || is_carry_alg(alg) || alg == kReducePartials;
}
inline constexpr int kScanBlock = 16;  // kScanCarry's block: P - 1 <= 15 of its 16 peers are inputs

inline constexpr int kMaxFusedPeers = 16;   // fused single-pass kernels are instantiated for P <= 16
// ... and allreduce_no_order up to 31: the pre-fold of peers 16.. into 0.. then the 16-peer recursive
// doubling, in one pass (also the block program of larger non-power-of-two P, fmi_dev.hip tree_blocked)
inline constexpr int kMaxFusedAllreducePeers = 31;
inline constexpr int kMaxFusedScanPeers = 31;  // the peer-axis scans likewise (P outputs, one pass)
inline constexpr int kFusedInputCap = 32;
inline constexpr int kFusedStepCap = 80;    // >= max steps of a fused program (allreduce P=31: 79)

constexpr int max_fused_peers(int alg) {
    return alg == 0 /*kAllreduce*/                    ? kMaxFusedAllreducePeers
           : alg == 3 || alg == 4 /*kScan, kScanLtr*/ ? kMaxFusedScanPeers
           : alg == 7 /*kAllreducePrefold16*/         ? 32
                                                      : kMaxFusedPeers;
}
// No cap on the number of peers, as in the reference (src/comm/PeerToPeer.cpp:59-184 take any num_peers):
// host programs (HostProgram below) are sized at run time; only the value ids must fit 31 bits.
inline constexpr int kMaxPeers = 1 << 24;

struct Step {
    uint16_t a;  // left operand (the buffer f.f overwrites)
    uint16_t b;  // right operand (the received buffer)
};

// Fixed-capacity program: the fused kernels' compile-time programs (value ids < 2^16).
template <int CapSteps, int CapPeers>
struct Program {
    using Id = uint16_t;
    using Ids = Id[CapPeers];
    int peers = 0;
    int nsteps = 0;
    bool ok = true;  // false if the capacity was exceeded or arguments were invalid
    Step step[CapSteps] = {};
    uint16_t out[CapPeers] = {};

    constexpr int nvalues() const { return peers + nsteps; }
    constexpr bool fits(int P) const { return P >= 1 && P <= CapPeers; }

    constexpr uint16_t emit(uint16_t a, uint16_t b) {
        if (nsteps >= CapSteps) {
            ok = false;
            return a;
        }
        step[nsteps] = Step{a, b};
        return static_cast<uint16_t>(peers + nsteps++);
    }
};

// Run-time program for any P (host side: fmi_schedule_expr, the pairwise-pass execution, the oracle
// checks). Same member names as Program, so host code indexes either alike.
struct HostStep {
    int32_t a;
    int32_t b;
};
struct HostProgram {
    using Id = int32_t;
    int peers = 0;
    int nsteps = 0;
    bool ok = true;
    std::vector<HostStep> step;
    std::vector<int32_t> out;

    int nvalues() const { return peers + nsteps; }
    bool fits(int P) const { return P >= 1 && P <= kMaxPeers; }
    int32_t emit(int32_t a, int32_t b) {
        step.push_back(HostStep{a, b});
        return peers + nsteps++;
    }
};

constexpr int floor_log2(int v) {
    int r = 0;
    while ((2 << r) <= v) ++r;
    return r;
}

constexpr int ceil_log2(int v) {
    int r = 0;
    while ((1 << r) < v) ++r;
    return r;
}

// The peers' current value ids: a fixed array for Program (constexpr), a vector for HostProgram.
template <class Prog>
struct IdVec {
    typename Prog::Ids v = {};
    constexpr explicit IdVec(int) {}
    constexpr auto& operator[](int i) { return v[i]; }
    constexpr const auto& operator[](int i) const { return v[i]; }
};
template <>
struct IdVec<HostProgram> {
    std::vector<int32_t> v;
    explicit IdVec(int P) : v(static_cast<size_t>(P)) {}
    int32_t& operator[](int i) { return v[static_cast<size_t>(i)]; }
    const int32_t& operator[](int i) const { return v[static_cast<size_t>(i)]; }
};

// Build the program of `alg` for P peers into `prog`. Ids are *transformed* ids for kReduce (root -> 0,
// reference PeerToPeer::transform_peer_id, src/comm/PeerToPeer.cpp:287-293): the caller rotates its inputs so
// that input t is real peer (t + root) % P; out[0] is then the root's result.
template <class Prog>
constexpr void build_into(Prog& prog, int alg, int P) {
    using Id = typename Prog::Id;
    if (!prog.fits(P)) {
        prog.ok = false;
        return;
    }
    prog.peers = P;
    IdVec<Prog> cur(P);
    for (int p = 0; p < P; ++p) cur[p] = static_cast<Id>(p);

    switch (alg) {
        case kAllreduce: {
            // Peers >= 2^floor(log2 P) first hand their bucket to peer - 2^k, which combines it as
            // f(own, received) (:100-107); recursive doubling over the power-of-two group, every pair
            // combining f(own, partner's value from the previous round) (:108-121); the folded peers
            // get the final value back (:122-128).
            const int rounds = floor_log2(P);
            const int pow2 = 1 << rounds;
            for (int p = pow2; p < P; ++p) cur[p - pow2] = prog.emit(cur[p - pow2], cur[p]);
            for (int i = 0; i < rounds; ++i) {
                IdVec<Prog> prev = cur;
                for (int p = 0; p < pow2; ++p) cur[p] = prog.emit(prev[p], prev[p ^ (1 << i)]);
            }
            for (int p = pow2; p < P; ++p) cur[p] = cur[p - pow2];
            break;
        }
        case kReduce:
        case kReducePartials: {
            // Binomial tree on transformed ids: in round i every t that is a multiple of 2^(i+1)
            // receives from t + 2^i (if it exists) and combines f(own, received) (:66-78).
            const int rounds = ceil_log2(P);
            for (int i = 0; i < rounds; ++i) {
                const int span = 1 << i;
                for (int t = 0; t + span < P; t += 2 * span) cur[t] = prog.emit(cur[t], cur[t + span]);
            }
            break;  // out[t != 0] is a non-root's partial (its sendbuf after the call, :72); out[0] the root's
        }
        case kReduceLtr: {
            // Root gathers all buckets by real id and folds left to right: ((x0 + x1) + x2) + ... (:49-52).
            // The allreduce variant broadcasts the root's result, so every peer ends with it.
            Id acc = 0;
            for (int p = 1; p < P; ++p) acc = prog.emit(acc, static_cast<Id>(p));
            for (int p = 0; p < P; ++p) cur[p] = acc;
            break;
        }
        case kScan: {
            // Up-sweep: in round i a peer whose low i+1 bits are all ones receives from peer - 2^i and
            // combines f(own, received); its partner (low i bits ones, bit i zero) sends (:156-168).
            // Down-sweep from round floor(log2 P) to 1: peers with low i bits all ones send to
            // peer + 2^(i-1); peers with only the low i-1 bits ones receive from peer - 2^(i-1) (if > 0)
            // and combine f(own, received) (:169-182).
            const int rounds = floor_log2(P);
            for (int i = 0; i < rounds; ++i) {
                const int full = (1 << (i + 1)) - 1;
                for (int p = 0; p < P; ++p)
                    if ((p & full) == full) cur[p] = prog.emit(cur[p], cur[p - (1 << i)]);
            }
            for (int i = rounds; i > 0; --i) {
                const int hi = (1 << i) - 1;
                const int lo = (1 << (i - 1)) - 1;
                for (int p = 0; p < P; ++p) {
                    if ((p & hi) == hi) continue;  // sender this round
                    const int src = p - (1 << (i - 1));
                    if ((p & lo) == lo && src > 0) cur[p] = prog.emit(cur[p], cur[src]);
                }
            }
            break;
        }
        case kScanLtr:
        case kScanLtrCarry: {
            // Linear chain: peer k receives the prefix of k-1 and combines f(prefix, own) (:146-147).
            for (int p = 1; p < P; ++p) cur[p] = prog.emit(cur[p - 1], static_cast<Id>(p));
            break;
        }
        case kAllreducePrefold16: {
            // allreduce_no_order's pre-fold (:100-107) for 16 peers at once, then its recursive doubling
            // (:108-121) over them: the program of a block whose peers all have a partner >= 2^k.
            if (P != 32) {
                prog.ok = false;
                return;
            }
            for (int j = 0; j < 16; ++j) cur[j] = prog.emit(cur[j], cur[16 + j]);
            for (int i = 0; i < 4; ++i) {
                IdVec<Prog> prev = cur;
                for (int p = 0; p < 16; ++p) cur[p] = prog.emit(prev[p], prev[p ^ (1 << i)]);
            }
            for (int p = 16; p < 32; ++p) cur[p] = cur[p - 16];
            break;
        }
        case kScanCarry: {
            // scan_no_order over P_all > 16 peers, restricted to block b >= 1 (peers 16b .. 16b+15, local
            // q = peer - 16b, value 1 + q). Up-sweep rounds 0..3 stay inside the block; rounds >= 4 and
            // down-sweep rounds >= 5 only touch q = 15 (the block totals), which leaves peer 16b - 1 holding
            // the prefix of blocks < b: the carry, value 0. Down-sweep rounds 4..1 then run inside the block,
            // except that a receiver whose source lies before the block (q - 2^(i-1) < 0) combines with the
            // carry (at full size that source is peer 16b - 1 > 0). The block's q = 15 input is never read:
            // its result is the block-level prefix, computed separately, so P - 1 <= 15 inputs.
            if (P - 1 > kScanBlock - 1) {
                prog.ok = false;
                return;
            }
            const int m = P - 1;
            for (int i = 0; i < 4; ++i) {
                const int full = (1 << (i + 1)) - 1;
                for (int q = 0; q < m; ++q)
                    if ((q & full) == full) cur[1 + q] = prog.emit(cur[1 + q], cur[1 + q - (1 << i)]);
            }
            for (int i = 4; i > 0; --i) {
                const int hi = (1 << i) - 1;
                const int lo = (1 << (i - 1)) - 1;
                for (int q = 0; q < m; ++q) {
                    if ((q & hi) == hi || (q & lo) != lo) continue;
                    const int src = q - (1 << (i - 1));
                    cur[1 + q] = prog.emit(cur[1 + q], src >= 0 ? cur[1 + src] : cur[0]);
                }
            }
            break;
        }
        default:
            prog.ok = false;
            return;
    }
    if constexpr (std::is_same_v<Prog, HostProgram>) prog.out.assign(static_cast<size_t>(P), 0);
    for (int p = 0; p < P; ++p) prog.out[p] = cur[p];
}

template <int CapSteps, int CapPeers>
constexpr Program<CapSteps, CapPeers> build(int alg, int P) {
    Program<CapSteps, CapPeers> prog{};
    build_into(prog, alg, P);
    return prog;
}

template <int Alg_, int P>
struct Fused {
    static constexpr Program<kFusedStepCap, kFusedInputCap> prog = build<kFusedStepCap, kFusedInputCap>(Alg_, P);
    static_assert(prog.ok, "fused schedule exceeds capacity");
};

inline HostProgram build_host(int alg, int P) {
    HostProgram prog;
    build_into(prog, alg, P);
    return prog;
}

}  // namespace fmi::sched
