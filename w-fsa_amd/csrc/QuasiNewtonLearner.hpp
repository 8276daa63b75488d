// QuasiNewtonLearner: mirror of the reference's optimizer
// (inc/QuasiNewtonLearner.h, src/QuasiNewtonLearner.cpp).  The KKT-diagonal
// update is O(n + k) host work; ComputeGrad is one device forward-backward.
#pragma once

#include "Learner.hpp"

namespace wfsa {

class QuasiNewtonLearner : public Learner {
public:
    QuasiNewtonLearner() {}
    void OptimizationStep(double eta = 1.0, bool verbose = false) override;
    std::vector<double> GetOptimizationInfo() override;
    std::string GetOptimizationHeader() const override;
    bool HaltCondition(double tol) override;

    const std::vector<double>& GetGradient() const { return grad; }
    const std::vector<double>& GetLambda() const { return lambda; }
    std::vector<double> GetLagrangeMultipliers() const override { return lambda; }

    void ComputeExpX();
    void ComputeG();
    void ComputeGrad();

    // The epoch loop of src/main.cpp:276-303 run device-resident
    // (wfsa_dev_qn_run): up to max_epochs OptimizationSteps, info_rows[7*e..]
    // (nullable) per epoch, stops after the epoch whose HaltCondition(tol)
    // holds; a non-finite info value throws LearnerError like the reference
    // after the row is recorded.  *epochs_done = the epochs run (set before
    // any throw).
    void RunDevice(double eta, double tol, int32_t max_epochs, double* info_rows, int32_t* epochs_done);

    // RunDevice leaves (x, lambda, grad) on the device: consecutive runs pass
    // them on without a host round trip.  Every other use of the learner
    // first pulls them back (PullDeviceState); one that may change x or
    // lambda on the host then marks the device copy out of date
    // (HostStateChanged), so the next run uploads it.  The C ABI
    // (host_api.cpp) does both at its entry points.
    void PullDeviceState();
    void HostStateChanged() { dev_state_valid = false; }

    struct Timing {
        int64_t steps = 0;
        double begin_ms = 0, overlap_ms = 0, wait_ms = 0, post_ms = 0;
    };
    const Timing& StepTiming() const { return timing; }

protected:
    void FinalizeCallback() override;
    void InitCallback(int flags) override;
    void ComputeLambdaNext(std::vector<double>& result);

private:
    std::vector<double> grad, expx, lambda, g, rhs;
    double grad_error = 0, lambda_min = 0, g_min = 0, g_max = 0;
    double rmin[2] = {0, 0};   // rmin column of the last step
    bool exponential_lambda = false;
    bool dev_qn_ready = false, dev_qn_exp = false;   // wfsa_dev_qn_setup done for this build
    int32_t dev_qn_rmin = -1;                        // ... with this info_rmin
    bool dev_state_valid = false;   // the device holds this learner's (x, lambda)
    bool host_state_stale = false;  // the device's (x, lambda, grad) are newer than the host's
    Timing timing;
    std::vector<double> rows_buf;   // RunDevice's info rows
    std::vector<double> laux_buf, lx_buf;   // OptimizationStep scratch (k, n)
    std::vector<int32_t> cptr_runs;         // constraint c's members: [cptr_runs[c], cptr_runs[c + 1])
    bool ccol_runs = false;                 // Ccol non-decreasing: cptr_runs is valid
};

}  // namespace wfsa
