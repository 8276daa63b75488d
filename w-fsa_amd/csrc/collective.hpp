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

#include "peer_layout.hpp"

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
    // why the peer path is off or failed ("" when on or untried)
    const char* peer_reason() const { return peer_why_.c_str(); }

    // 0 while the group is healthy; 1 (last_error() says why) once a peer
    // wait gave up, another member poisoned the group, or abort() ran.  Free
    // to call at any host sync point: the peer kernels report through
    // host-mapped memory.
    int check();
    // check() plus the transport's own liveness, for a host that has been
    // waiting `waited_s` seconds for device work that includes collectives:
    // an RCCL communicator with an asynchronous error, or a wait longer than
    // WFSA_COMM_TIMEOUT_S (default 300 s), is aborted here and reported (1)
    virtual int watchdog(double waited_s) { return check(); }
    // this member failed: every later call on this communicator fails, and
    // the members hear of it as follows (failure semantics):
    //  * in-process group: poisoned -- every member waiting in, or later
    //    entering, a collective fails at once;
    //  * peer all-reduce (the per-step [LL, grad] sums): every member's area
    //    gets its poison word -- their current or next peer call fails at once;
    //  * RCCL: the communicator is aborted (ncclCommAbort).  The other
    //    processes' pending RCCL calls are NOT woken by that: each rank's own
    //    watchdog ends them (its asynchronous error, or WFSA_COMM_TIMEOUT_S);
    //  * host callback (gloo, MPI): a poisoned header exchange (every call
    //    starts with one) -- every member waiting in, or later entering, a
    //    collective fails at once.  A member that dies without aborting
    //    leaves the others to the callback transport's own timeout.
    void abort(const char* why);
    bool aborted() const { return aborted_; }
    // the in-kernel exchange's view of the peer areas with the next sequence
    // number (one per launch that exchanges); false when the peer path is not
    // on (x.on = 0)
    bool peer_exchange(PeerX& x);

protected:
    // the transport's own all-reduce
    virtual int transport_allreduce(void* buf, size_t n, RedOp op, hipStream_t s) = 0;
    // the transport's part of abort()
    virtual void abort_transport(const std::string& why) {}
    // the members share this process's address space (no IPC mapping)
    virtual bool same_process() const { return false; }
    // the device ordinal this member's kernels run on
    virtual int device() const { return -1; }
    // the peer path by default (WFSA_PEER=1 / 0 overrides)
    virtual bool peer_default() const { return false; }
    int n_ = 1, r_ = 0;
    std::string err_;

    // device memory for the peer set-up's exchanges, reserved when the
    // communicator is made, so the set-up never lacks a buffer for its
    // agreement (every member then takes part in every exchange)
    void* agree_buf_ = nullptr;
public:
    // (the make_*_collective functions reserve it BEFORE joining the group or
    // creating the communicator -- a member that cannot reserve it then fails
    // alone, never leaving the others a member short -- and hand it over)
    static void* reserve_agreement(std::string& err);
    void adopt_agreement(void* buf) { agree_buf_ = buf; }
protected:

private:
    int try_peer(hipStream_t s);
    std::unique_ptr<PeerSum> peer_;
    int peer_st_ = 0;   // 0 untried, 1 on, -1 off, -2 failed
    std::string peer_why_;
    bool aborted_ = false;
    std::string abort_why_;
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
// reads.  A wait gives up after WFSA_PEER_TIMEOUT_S (default 120 s, the
// in-process group's barrier limit): the result becomes NaN, the rank's
// host-mapped status word is set and a poison word goes into EVERY member's
// area, so every member's next peer call fails at entry without waiting;
// Collective::check() turns the status into an error at the next host sync
// point -- an error on every rank, never a hang and never a silent NaN.
// The peer kernels of the members must run concurrently: members on distinct
// devices, or in distinct processes (distinct hardware queues).  Two contexts
// of one process on one device have no such guarantee -- HIP may put their
// streams on one hardware queue, where a spinning kernel holds back the
// other -- so an in-process group on one device keeps the transport.

constexpr int kCommIdBytes = 128;   // WFSA_COMM_ID_BYTES

// Checks the peer kernel on one device without a second process: the other
// members' areas are local and their contributions / flags are written
// beforehand (mode 0: all present, the sum must equal the rank-order sum;
// mode 1: member `nranks-1` never arrives, the call must give up after
// timeout_s with NaN, the status set and every area poisoned; mode 2: the
// own area poisoned before the call, which must fail at entry, well inside
// timeout_s).  out[0..3] = {max |error| (mode 0) or NaN count, status,
// poisoned areas, elapsed seconds}.  0 = ran (the caller judges out), else err.
int peer_selftest(int nranks, int64_t n, double timeout_s, int mode, double out[4], std::string& err);

// a fresh in-process group id (magic prefix, serial, size)
void local_group_id(int nranks, uint8_t id[kCommIdBytes]);
bool is_local_group_id(const uint8_t id[kCommIdBytes]);

// nullptr on failure (err says why)
std::unique_ptr<Collective> make_rccl_collective(int nranks, int rank, const uint8_t id[kCommIdBytes],
                                                 std::string& err);
std::unique_ptr<Collective> make_local_collective(int nranks, int rank, const uint8_t id[kCommIdBytes],
                                                  int device, std::string& err);
int rccl_unique_id(uint8_t id[kCommIdBytes], std::string& err);
// the host watchdog's limit (WFSA_COMM_TIMEOUT_S, default 300 s)
double comm_timeout_s();

// a transport over a host callback (e.g. torch.distributed over gloo, MPI):
// fn(user, host buffer, count, op) all-reduces in place, op 0 = sum of
// doubles, 1 = min of doubles, 2 = max of bytes; non-zero = failure.  One
// process per rank; several may share a GPU.
using HostAllreduceFn = int (*)(void* user, void* buf, int64_t count, int32_t op);
std::unique_ptr<Collective> make_host_collective(int nranks, int rank, HostAllreduceFn fn, void* user,
                                                 std::string& err);

}  // namespace wfsa
