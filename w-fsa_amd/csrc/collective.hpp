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

class Collective {
public:
    virtual ~Collective() = default;
    int nranks() const { return n_; }
    int rank() const { return r_; }
    // in-place all-reduce of n elements of buf (device memory) on stream s;
    // 0 on success, else last_error() says why
    virtual int allreduce(void* buf, size_t n, RedOp op, hipStream_t s) = 0;
    const char* last_error() const { return err_.c_str(); }
    virtual const char* kind() const = 0;

protected:
    int n_ = 1, r_ = 0;
    std::string err_;
};

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

}  // namespace wfsa
