// Rank-combination transports of the data-parallel path.
//
// Every place the context combines its shard's values with the other ranks'
// -- the constant trivial-word gradient once at preparation, [LL, grad] per
// evaluation, the used-parameter mask of the structural pass (max), the
// Learner's corpus statistics, the rmin column (min) and the H_f pattern
// values -- calls Collective::allreduce.  Two transports implement it:
//
//  * RCCL (the product across processes: one process per GPU, ring/tree
//    collectives over xGMI, stream-ordered);
//  * an in-process group: several contexts of ONE process (threads), each
//    with its own stream, on one device or on peer-enabled devices.  Every
//    member synchronises its stream, the members meet at a host barrier, each
//    sums the members' buffers in rank order into its own scratch, a second
//    barrier, then copies the sum back.  Deterministic (rank order), blocking.
//    This is what lets a single-GPU test run the product's multi-rank
//    branches -- sharding, the per-step all-reduce, the max-reduced masks --
//    end to end (tests/test_gpu_ranks.py).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>

namespace wfsa {

enum class RedOp { SumF64, MinF64, MaxU8 };

class PeerSum;

class Collective {
public:
    virtual ~Collective();
    int nranks() const { return n_; }
    int rank() const { return r_; }
    // in-place all-reduce of n elements of buf (device memory) on stream s;
    // 0 on success, else last_error() says why.  Sums of at most kPeerCap
    // doubles take the one-shot peer path when it is on (below).
    int allreduce(void* buf, size_t n, RedOp op, hipStream_t s);
    const char* last_error() const { return err_.c_str(); }
    virtual const char* kind() const = 0;
    // the one-shot peer all-reduce: "on", "off", "failed" (its set-up check
    // disagreed on some rank: the transport is used), "untried"
    const char* peer_state() const;

protected:
    // the transport's own all-reduce
    virtual int transport_allreduce(void* buf, size_t n, RedOp op, hipStream_t s) = 0;
    // the members share this process's address space (no IPC mapping)
    virtual bool same_process() const { return false; }
    // the peer path by default (WFSA_PEER=1 / 0 overrides)
    virtual bool peer_default() const { return false; }
    int n_ = 1, r_ = 0;
    std::string err_;

private:
    int try_peer(hipStream_t s);
    std::unique_ptr<PeerSum> peer_;
    int peer_st_ = 0;   // 0 untried, 1 on, -1 off, -2 failed
};

// One-shot peer all-reduce of doubles: every rank owns an area
// of [2 parities][nranks][kPeerCap] receive slots plus per-chunk flags in
// uncached device memory, mapped into every member (IPC, or the pointer
// itself in one process).  A call is one kernel: each block stores its chunk
// of the rank's vector into its slot in every member's area (remote stores
// over xGMI), raises its flag there (release, system scope), waits for the
// chunk's flags of all ranks in its own area and sums the slots in rank
// order -- deterministic, stream-ordered, no host step.  The parity (call
// sequence & 1) keeps a fast rank from overwriting slots a slow one still
// reads.  A wait gives up after WFSA_PEER_TIMEOUT_S (default 10 s): the
// result becomes NaN and the status word is set, never a hang.
constexpr size_t kPeerCap = size_t(1) << 16;      // doubles per rank slot (512 KiB)
constexpr int kPeerChunk = 1024;                  // doubles per block
constexpr int kPeerMaxChunks = int(kPeerCap / kPeerChunk);

constexpr int kCommIdBytes = 128;   // WFSA_COMM_ID_BYTES
constexpr int kLocalMaxRanks = 16;

// a fresh in-process group id (magic prefix, serial, size)
void local_group_id(int nranks, uint8_t id[kCommIdBytes]);
bool is_local_group_id(const uint8_t id[kCommIdBytes]);

// nullptr on failure (err says why)
std::unique_ptr<Collective> make_rccl_collective(int nranks, int rank, const uint8_t id[kCommIdBytes],
                                                 std::string& err);
std::unique_ptr<Collective> make_local_collective(int nranks, int rank, const uint8_t id[kCommIdBytes],
                                                  int device, std::string& err);
int rccl_unique_id(uint8_t id[kCommIdBytes], std::string& err);

// a transport over a host callback (e.g. torch.distributed over gloo, MPI):
// fn(user, host buffer, count, op) all-reduces in place, op 0 = sum of
// doubles, 1 = min of doubles, 2 = max of bytes; non-zero = failure.  One
// process per rank; several may share a GPU.
using HostAllreduceFn = int (*)(void* user, void* buf, int64_t count, int32_t op);
std::unique_ptr<Collective> make_host_collective(int nranks, int rank, HostAllreduceFn fn, void* user,
                                                 std::string& err);

}  // namespace wfsa
