// Learner: host-side mirror of the reference's Learner (inc/Learner.h:17-169)
// with the hot path moved behind the device boundary (include/wfsa_dev.h).
//
// What stays the same: the public methods, BuildConstraints, Trim,
// GetWeight, Renormalize, LambdaUpdate, Finalize's plogp, parameter
// numbering.  What changes: BuildPaths no longer enumerates paths and no
// P / M matrices exist -- the device's structural pass supplies the
// recognized strings, path counts and used parameters, and
// ComputeModeledProbs + ComputeObjective + the gradient come from one
// forward-backward launch per iteration.
//
// Data parallelism: with a communicator attached the corpus is split into
// contiguous shards (balanced on total length), each rank uploads only its
// shard, and the device sums [loglik, grad] over ranks with one RCCL
// all-reduce; host-side scalars (plogp, counts) are all-reduced once after
// BuildFrom.  Every rank then runs the identical O(n) optimizer update.
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "Corpus.hpp"
#include "Fsa.hpp"
#include "text.hpp"
#include "wfsa_dev.h"

namespace wfsa {

struct LearnerError : public MyError {
    using MyError::MyError;
};
// a call made out of order or with bad arguments, found before any rank
// collective: it fails this call only (the communicator is not aborted)
struct LearnerUsageError : public LearnerError {
    using LearnerError::LearnerError;
};

class Learner {
public:
    Learner();
    virtual ~Learner();
    Learner(const Learner&) = delete;
    Learner& operator=(const Learner&) = delete;

    // Device / sharding setup (new; call before BuildFrom).
    void SetDevice(int device);
    void SetCommunicator(int nranks, int rank, const uint8_t* unique_id);
    // the same over a host callback (wfsa_dev_comm_init_host)
    void SetHostCommunicator(int nranks, int rank, wfsa_host_allreduce_fn fn, void* user);
    // this rank failed: the other ranks' current or next collective fails at
    // once (wfsa_dev_comm_abort); a no-op before BuildFrom or on one rank
    void AbortCommunicator(const char* why);

    // `corpus` weights must already be normalized over the whole corpus
    // (main.cpp renormalizes before BuildFrom).  With a communicator, every
    // rank passes the full corpus and keeps its own shard.  `bfs` is
    // accepted for interface parity; the trellis has no BFS/DFS choice.
    void BuildFrom(const Fsa& fsa, const Corpus& corpus, bool bfs = true);
    // Same from packed strings (sym/off) and normalized weights.
    void BuildFromPacked(const Fsa& fsa, const uint8_t* sym, const int64_t* off, const double* weights,
                         int64_t n_strings);

    // Matrix-file mode (src/Learner.cpp:82-199): LoadMatrices reads
    // prefix.{C,M,P,prob,aux} in the reference's text CSR format
    // (ReadCsrMtx, src/Utils.cpp:184-202) and hands P/M/p to the device
    // (wfsa_dev_load_paths) instead of BuildFrom; throws LearnerError with the
    // reference's messages.  SaveMatrices writes the same files -- possible
    // only for matrices that were loaded: this build never enumerates paths.
    bool LoadMatrices(const std::string& prefix);
    bool SaveMatrices(const std::string& prefix) const;
    bool FromMatrices() const { return matrices != nullptr; }
    // The reference's P / M (paths x parameters counts, strings x paths) after
    // BuildFrom + Trim, enumerated on the host in the reference's path order
    // (Paths.hpp; src/Learner.cpp:276-348 and Trim's renumbering :397-419) --
    // for -p and -m >prefix only, one rank.  Then PrintC/M/P
    // (src/Learner.cpp:60-80) print them and SaveMatrices writes them.
    void EnumeratePaths(const Fsa& fsa, const Corpus& corpus, bool bfs = true);
    bool HasPathMatrices() const { return matrices != nullptr || enumerated != nullptr; }
    void PrintC(FILE* f) const;
    void PrintM(FILE* f) const;
    void PrintP(FILE* f) const;

    void Renormalize();
    void RewriteWeights(Fsa& fsa) const;
    const double* GetWeights() const { return _x.data(); }

    virtual std::vector<double> GetOptimizationInfo();
    virtual std::string GetOptimizationHeader() const;
    virtual std::vector<double> GetOptimizationResult(bool verbose = false);
    virtual bool HaltCondition(double tol);
    // the constraints' multipliers (the reference keeps them after x in _x)
    virtual std::vector<double> GetLagrangeMultipliers() const { return {}; }

    double GetCommonSupport() const { return common_support; }

    // log q for every (local) recognized string, then q (src/Learner.cpp:515-547)
    void ComputeModeledProbs();
    // kl = plogp - p.log q (src/Learner.cpp:549-553)
    void ComputeObjective();

    int32_t GetNumberOfStrings() const { return int32_t(n_strings_global); }
    int64_t GetNumberOfPaths() const { return n_paths_global; }
    int32_t GetNumberOfParameters() const { return int32_t(Ccol.size()); }
    int32_t GetNumberOfConstraints() const { return Ccol.empty() ? 0 : Ccol.back() + 1; }
    int32_t GetNumberOfLocalStrings() const { return int32_t(p.size()); }
    int32_t GetNumberOfFullParameters() const { return n_full; }

    bool HasUniquePaths() const { return unique_paths; }
    // the rmin info column (src/QuasiNewtonLearner.cpp:80-84): available with
    // ambiguous strings on one rank off the dense path; otherwise (0, 0) as
    // the reference reports for unique paths
    bool RminAvailable() const;
    // the rmin column is on by default (the reference prints it every epoch);
    // off, columns rmin / index read 0 and no (min, x) pass runs
    void SetInfoRmin(bool on) { info_rmin = on; }
    // out[0] = smallest relative path probability at the last evaluation,
    // out[1] = index of the string holding that path
    void ComputeRmin(double* out) const;
    double GetKLDistance() const { return kl; }
    double gKLDistance() const { return kl + mxlogx(common_support); }

    virtual void OptimizationStep(double eta = 1.0, bool verbose = false) = 0;
    virtual void Init(int flags, const double* initialx = nullptr);

    double LogModelVolume() const { return model_volume; }
    double LogAuxiliaryVolume() const { return log_simplex_volume(auxiliary_parameters); }
    double LogVolume() const { return LogModelVolume() + LogAuxiliaryVolume(); }
    double LogDetAuxiliaryHessian() const { return aux_hessian; }
    int32_t GetNumberOfAuxParameters() const { return int32_t(auxiliary_parameters); }

    void Finalize();

    // accessors used by the C-ABI / tests
    const std::vector<double>& GetP() const { return p; }
    const std::vector<double>& GetLastGradient() const { return grad_cache; }   // trimmed, last evaluation
    const std::vector<double>& GetLogQ();           // fetches log q from the device
    const std::vector<int32_t>& GetTrimmedIndex() const { return trimmed_weights; }
    const std::vector<double>& GetPathCounts() const { return path_count_local; }   // per local corpus string
    const std::vector<uint8_t>& GetRecognized() const { return recognized_local; }
    double GetWeight(int32_t i) const;
    void SetWeights(const double* x);
    double GetLogLikelihood() const { return loglik; }
    double GetPLogP() const { return plogp; }
    wfsa_dev* Device() const { return dev; }
    const FlatModel* Model() const { return flat.get(); }
    int64_t ShardBegin() const { return shard_begin; }
    int64_t ShardEnd() const { return shard_end; }

protected:
    virtual void FinalizeCallback();
    virtual void InitCallback(int flags);
    void LambdaUpdate(double* lstep, double* l, double eta = 1.0, bool exponential = false) const;

    // One device evaluation at the current _x: loglik, gradient (trimmed,
    // reference sign: -sum p E[count]) into `grad_out`.
    void EvaluateDevice(std::vector<double>& grad_out, bool want_logq);
    // The same, split: Begin enqueues the device work at the current _x and
    // returns, so the caller can do host work that does not need the
    // gradient; End waits and fills grad_out.  (ComputeModeledProbs ==
    // BeginModeledProbs + EndModeledProbs.)
    void BeginModeledProbs(bool want_logq = false);
    void EndModeledProbs(std::vector<double>& grad_out);
    // results of an evaluation that ran elsewhere (the device-resident QN run)
    void SetEvaluated(double loglik_value);
    double AllReduceSum(double v) const;

    std::vector<double> _x;
    std::vector<double> grad_cache;   // gradient of the last ComputeModeledProbs
    std::vector<double> p;
    std::vector<double> logq;
    std::vector<double> aux;
    std::vector<int32_t> Crow, Ccol;

private:
    void BuildConstraints(const Fsa& fsa);
    void BuildPaths(const Fsa& fsa, const uint8_t* sym, const int64_t* off, const double* weights, int64_t n);
    void Trim();
    void EnsureDevice();

    double common_support = 0, plogp = 0, kl = 0, aux_hessian = 0, model_volume = 0, loglik = 0;
    int64_t auxiliary_parameters = 0;
    int64_t n_strings_global = 0, n_paths_global = 0;
    bool unique_paths = true;
    bool info_rmin = true;
    int32_t n_full = 0;
    std::vector<int32_t> trimmed_weights;
    std::vector<double> w_full, grad_full;
    std::vector<double> path_count_local;
    std::vector<uint8_t> recognized_local;
    bool logq_valid = false;
    bool eval_in_flight = false, eval_logq = false;

    int device = 0;
    wfsa_dev* dev = nullptr;
    int nranks = 1, rank = 0;
    std::vector<uint8_t> comm_id;
    wfsa_host_allreduce_fn host_fn = nullptr;
    void* host_user = nullptr;
    std::unique_ptr<FlatModel> flat;
    int64_t shard_begin = 0, shard_end = 0;
    struct Matrices {   // the loaded path matrices (matrix-file mode)
        std::vector<double> cdata, mdata, pdata;
        std::vector<int32_t> crow, ccol, mrow, mcol, prow, pcol;
    };
    std::unique_ptr<Matrices> matrices;
    std::unique_ptr<Matrices> enumerated;   // EnumeratePaths (after BuildFrom)
    const Matrices* PathMatrices() const { return matrices ? matrices.get() : enumerated.get(); }
};

void ThrowOnDevError(int rc, const char* what);

// Contiguous shard of `rank` over strings with offsets off[0..n], balanced on
// total length: [begin, end).
struct ShardRange {
    int64_t begin, end;
};
ShardRange shard_range(const int64_t* off, int64_t n, int nranks, int rank);

}  // namespace wfsa
