// The one-shot peer areas' layout, shared by the peer all-reduce kernel
// (collective.hip, PeerSum) and the in-kernel QN exchange across ranks
// (fb_kernels.hip, PeerX).  Every rank owns an area in uncached device
// memory, mapped into every member (IPC, or the pointer itself in one
// process): [2 parities][nranks][kPeerCap] double slots, then [2][nranks]
// [kPeerFlags] 64-bit flags, then the poison word (padded to 16 bytes).  A
// call with sequence number seq writes parity seq & 1: member r stores its
// values into slot [par][r] of every member's area, raises flag [par][r][f]
// there (system-scope release of seq) and reads the members' slots in its own
// area once every member's flag f has reached seq.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace wfsa {

constexpr size_t kPeerCap = size_t(1) << 16;      // doubles per rank slot (512 KiB)
constexpr int kPeerChunk = 1024;                  // doubles per block of the peer all-reduce
constexpr int kPeerMaxChunks = int(kPeerCap / kPeerChunk);   // its chunks: flags [0, 64)
constexpr int kPeerFlags = 4096;                  // flags per [parity][rank]
constexpr int kPeerQnFlag0 = kPeerMaxChunks;      // the in-kernel QN batches' flags: [64, 64 + batches)
constexpr int kPeerFinFlag = kPeerFlags - 2;      // the finishes' exchanges: flags 4094 (the finish
                                                  // wave) and 4095 (a launch finishing its own step)
constexpr size_t kPeerFinSlot = kPeerCap - 8;     // ... their data: 4 slots each
constexpr int kPeerMaxQnBatches = kPeerFinFlag - kPeerQnFlag0;
constexpr int kLocalMaxRanks = 16;

__host__ __device__ inline size_t peer_area_bytes(int nranks) {
    return 2 * size_t(nranks) * kPeerCap * sizeof(double) + 2 * size_t(nranks) * kPeerFlags * sizeof(uint64_t) + 16;
}
__host__ __device__ inline uint64_t* peer_flags(double* area, int nranks) {
    return reinterpret_cast<uint64_t*>(area + 2 * size_t(nranks) * kPeerCap);
}
__host__ __device__ inline uint64_t* peer_poison(double* area, int nranks) {
    return peer_flags(area, nranks) + 2 * size_t(nranks) * kPeerFlags;
}

// An in-kernel exchange's view of the areas (the QN waves' per-batch member
// partials, the finishes' log-likelihood and rmin), one sequence number per
// launch (Collective::peer_exchange)
struct PeerX {
    double* const* area;            // [nranks] rank r's area as mapped in this process (a device table:
                                    // indexed per lane, a kernel-argument array would go to scratch)
    int32_t on, nranks, me, pad;
    uint64_t seq;
    uint64_t timeout;               // s_memrealtime ticks (100 MHz)
    unsigned* status;               // host-mapped: set to 1 when an exchange failed (Collective::check)
};

}  // namespace wfsa
