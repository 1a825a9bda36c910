// fmi_exchange_plan.h — the point-to-point plans of the communicator's exchanges (host-only, no HIP).
//
// Every exchange the RCCL transport builds from grouped send / recv (all-to-all and all-gather in their
// grouped realisations, gather, scatter, and the four ragged exchanges whose last shards are short) is
// written here once, as a pure function of (ranks, rank, sizes): the list of sends and receives this rank
// posts plus one local copy. The RCCL transport issues a plan as one ncclGroupStart/End; the LOCAL
// transport executes the same plans by copying each receive from the matching send of the peer's plan,
// so the GPU tests over LOCAL ranks run the exact pairings the RCCL transport posts between GPUs; and
// tests/test_exchange_plan.py checks every plan for N = 1…257 ranks on the host: for each ordered pair the
// sends and the receives agree in count and length (a mismatch would hang RCCL), and the bytes land where
// the exchange's definition says.
#pragma once

#include <cstddef>
#include <vector>

namespace fmi::plan {

struct Xfer {
    int peer;
    size_t off;  // bytes into this rank's send (for a send) or recv (for a receive) buffer
    size_t len;  // bytes, never 0 (empty transfers are not posted, on either side alike)
};

struct Plan {
    std::vector<Xfer> sends;  // posted in this order; per peer, matched in order with the peer's receives
    std::vector<Xfer> recvs;
    size_t copy_src = 0;  // local part: recv[copy_dst ..] = send[copy_src ..], copy_len bytes (0: none)
    size_t copy_dst = 0;
    size_t copy_len = 0;
};

// Bytes of shard j when shards of `shard` bytes tile a `total`-byte bucket (the last ones short or empty).
inline size_t span(int j, size_t shard, size_t total) {
    const size_t lo = static_cast<size_t>(j) * shard;
    return lo >= total ? 0 : (total - lo < shard ? total - lo : shard);
}

namespace detail {
inline void add(std::vector<Xfer>& v, int peer, size_t off, size_t len) {
    if (len) v.push_back({peer, off, len});
}
}  // namespace detail

// recv[j * stride ...] = rank j's send[rank * bytes ...] (stride 0: bytes, the blocks back to back); the own part
// travels as a send / receive to self. The stride changes only where this rank's receives land, never the pairing.
inline Plan all_to_all(int n, int rank, size_t bytes, size_t recv_stride = 0) {
    (void)rank;
    const size_t stride = recv_stride ? recv_stride : bytes;
    Plan p;
    for (int j = 0; j < n; ++j) {
        detail::add(p.sends, j, j * bytes, bytes);
        detail::add(p.recvs, j, j * stride, bytes);
    }
    return p;
}

// recv[j * bytes ...] = rank j's send[0 .. bytes): this rank's block straight to every peer, no ring.
inline Plan all_gather(int n, int rank, size_t bytes) {
    Plan p;
    for (int j = 0; j < n; ++j) {
        if (j == rank) continue;
        detail::add(p.sends, j, 0, bytes);
        detail::add(p.recvs, j, j * bytes, bytes);
    }
    p.copy_dst = rank * bytes;
    p.copy_len = bytes;
    return p;
}

// root's recv[j * bytes ...] = rank j's send[0 .. bytes)
inline Plan gather(int n, int rank, size_t bytes, int root) {
    Plan p;
    if (rank == root) {
        for (int j = 0; j < n; ++j)
            if (j != root) detail::add(p.recvs, j, j * bytes, bytes);
        p.copy_dst = root * bytes;
        p.copy_len = bytes;
    } else {
        detail::add(p.sends, root, 0, bytes);
    }
    return p;
}

// recv[0 .. bytes) = root's send[rank * bytes ...]
inline Plan scatter(int n, int rank, size_t bytes, int root) {
    Plan p;
    if (rank == root) {
        for (int j = 0; j < n; ++j)
            if (j != root) detail::add(p.sends, j, j * bytes, bytes);
        p.copy_src = root * bytes;
        p.copy_len = bytes;
    } else {
        detail::add(p.recvs, root, 0, bytes);
    }
    return p;
}

// Ragged forms: shard j covers bytes [j * shard, j * shard + span(j)) of a `total`-byte bucket.

// recv[j * shard ...] = rank j's send[rank * shard ...], span(rank) bytes (every rank's copy of my shard).
inline Plan all_to_all_ragged(int n, int rank, size_t shard, size_t total) {
    Plan p;
    const size_t mine = span(rank, shard, total);
    for (int j = 0; j < n; ++j) {
        detail::add(p.sends, j, j * shard, span(j, shard, total));
        detail::add(p.recvs, j, j * shard, mine);
    }
    return p;
}

// recv[j * shard ...] = rank j's send[0 ..], span(j) bytes (every owner's reduced shard).
inline Plan all_gather_ragged(int n, int rank, size_t shard, size_t total) {
    Plan p;
    const size_t mine = span(rank, shard, total);
    for (int j = 0; j < n; ++j) {
        if (j == rank) continue;
        detail::add(p.sends, j, 0, mine);
        detail::add(p.recvs, j, j * shard, span(j, shard, total));
    }
    p.copy_dst = rank * shard;
    p.copy_len = mine;
    return p;
}

// root's recv[j * shard ...] = rank j's send[0 ..], span(j) bytes.
inline Plan gather_ragged(int n, int rank, size_t shard, size_t total, int root) {
    Plan p;
    const size_t mine = span(rank, shard, total);
    if (rank == root) {
        for (int j = 0; j < n; ++j)
            if (j != root) detail::add(p.recvs, j, j * shard, span(j, shard, total));
        p.copy_dst = root * shard;
        p.copy_len = mine;
    } else {
        detail::add(p.sends, root, 0, mine);
    }
    return p;
}

// recv[j * shard ...] = rank j's send[rank * shard ...], span(j) bytes: the inverse of all_to_all_ragged,
// every owner handing each rank that rank's version of the owner's shard.
inline Plan all_to_all_back_ragged(int n, int rank, size_t shard, size_t total) {
    Plan p;
    const size_t mine = span(rank, shard, total);
    for (int j = 0; j < n; ++j) {
        detail::add(p.sends, j, j * shard, mine);
        detail::add(p.recvs, j, j * shard, span(j, shard, total));
    }
    return p;
}

}  // namespace fmi::plan
