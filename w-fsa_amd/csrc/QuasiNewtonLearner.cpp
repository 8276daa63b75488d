#include "QuasiNewtonLearner.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>

namespace wfsa {

void QuasiNewtonLearner::FinalizeCallback() {   // src/QuasiNewtonLearner.cpp:17-27
    const size_t n = size_t(GetNumberOfParameters()), k = size_t(GetNumberOfConstraints());
    grad.assign(n, 0.0);
    expx.assign(n, 0.0);
    rhs.assign(n, 0.0);
    lambda.assign(k, 1.0);
    g.assign(k, 0.0);
    // the constraints' member runs, when Ccol is non-decreasing (the host
    // update's fast form)
    ccol_runs = true;
    cptr_runs.assign(k + 1, 0);
    for (size_t i = 0; i < n; ++i) {
        if ((i > 0 && Ccol[i] < Ccol[i - 1]) || Ccol[i] < 0 || size_t(Ccol[i]) >= k) {
            ccol_runs = false;
            break;
        }
        cptr_runs[size_t(Ccol[i]) + 1]++;
    }
    for (size_t c = 0; c < k && ccol_runs; ++c) cptr_runs[c + 1] += cptr_runs[c];
    dev_qn_ready = false;
    dev_state_valid = host_state_stale = false;
}

void QuasiNewtonLearner::InitCallback(int flags) {   // :29-51
    if (flags & 1) std::fill(_x.begin(), _x.end(), 0.0);
    if (flags & 2) Renormalize();
    if (flags & 4) {
        ComputeExpX();
        ComputeGrad();
        std::fill(lambda.begin(), lambda.end(), 0.0);   // lambda <- -C^T grad
        for (size_t i = 0; i < grad.size(); ++i) lambda[size_t(Ccol[i])] -= grad[i];
    }
    exponential_lambda = (flags & 32) != 0;
}

void QuasiNewtonLearner::ComputeExpX() {
    for (size_t i = 0; i < _x.size(); ++i) expx[i] = std::exp(_x[i]);
}

std::string QuasiNewtonLearner::GetOptimizationHeader() const {
    return "       KL   graderr     g_min     g_max lambdamin      rmin";
}

// [KL, graderr, g_min, g_max, lambda_min, rmin, rmin index]: rmin is the
// smallest relative path probability (src/QuasiNewtonLearner.cpp:80-84) at
// the step's weights, from the device's (min, x) pass (wfsa_dev_rmin); its
// index is the string holding that path (the reference's BFS path index has
// no counterpart without enumerating paths).
std::vector<double> QuasiNewtonLearner::GetOptimizationInfo() {
    return {GetKLDistance(), grad_error, g_min, g_max, lambda_min, rmin[0], rmin[1]};
}

bool QuasiNewtonLearner::HaltCondition(double tol) {   // :88-91
    return grad_error <= tol && std::abs(g_min) <= tol && std::abs(g_max) <= tol;
}

// grad = -sum_s p_s E[count | s] straight from the device; the reference's
// grad_aux / relative_path_probs bookkeeping (:93-125) has no counterpart.
void QuasiNewtonLearner::ComputeGrad() {
    ComputeModeledProbs();
    grad = grad_cache;
}

void QuasiNewtonLearner::ComputeLambdaNext(std::vector<double>& result) {   // :127-146
    const size_t k = size_t(GetNumberOfConstraints());
    result.resize(k);
    for (size_t c = 0; c < k; ++c) result[c] = lambda[c] * g[c];
    for (size_t i = 0; i < grad.size(); ++i) result[size_t(Ccol[i])] -= grad[i];
    for (size_t c = 0; c < k; ++c) {
        g[c] += 1.0;
        result[c] /= g[c];
    }
}

void QuasiNewtonLearner::ComputeG() {   // :148-160: g = C^T exp(x) - 1
    std::fill(g.begin(), g.end(), -1.0);
    for (size_t i = 0; i < expx.size(); ++i) g[size_t(Ccol[i])] += expx[i];
    if (g.empty()) {
        g_min = g_max = 0.0;
        return;
    }
    g_min = *std::min_element(g.begin(), g.end());
    g_max = *std::max_element(g.begin(), g.end());
}

namespace {

// OptimizationStep's O(n + k) update after the gradient (:170-199): aux,
// rhs and graderr, the next lambda (ComputeLambdaNext), x and LambdaUpdate's
// argument.  Every value is formed by the same operations in the same order
// as the plain loops (Ccol is non-decreasing -- BuildConstraints numbers a
// group's members consecutively -- so a constraint's members are one run,
// subtracted in ascending order), so the results are the same bits; the max
// runs in four accumulators (NaN is never selected, as with std::max).
// Compiled twice, the AVX2 clone picked at load time (AVX2 alone has no FMA,
// so nothing is contracted).
struct QnHostUpdate {
    size_t n, k;
    const int32_t* ccol;
    const int32_t* cptr;
    const double* grad;
    const double* expx;
    const double* lambda;
    double* g;
    double* aux;
    double* rhs;
    double* x;
    double* laux;   // k: lambda - lambda_next on return
    double* lx;     // n: scratch
    double eta;
};

__attribute__((target_clones("avx2", "default"))) double qn_host_update(const QnHostUpdate& u) {
    const size_t n = u.n, k = u.k;
    const int32_t* __restrict ccol = u.ccol;
    const int32_t* __restrict cptr = u.cptr;
    const double* __restrict grad = u.grad;
    const double* __restrict expx = u.expx;
    const double* __restrict lambda = u.lambda;
    double* __restrict g = u.g;
    double* __restrict aux = u.aux;
    double* __restrict rhs = u.rhs;
    double* __restrict x = u.x;
    double* __restrict laux = u.laux;
    double* __restrict lx = u.lx;
    for (size_t i = 0; i < n; ++i) lx[i] = lambda[ccol[i]];
    double m[4] = {0.0, 0.0, 0.0, 0.0};
    size_t i = 0;
    for (; i + 4 <= n; i += 4)
        for (int q = 0; q < 4; ++q) {
            const double a = expx[i + q] * lx[i + q];   // J_g . lambda
            aux[i + q] = a;
            const double r = grad[i + q] + a;
            rhs[i + q] = r;
            const double ar = std::fabs(r);
            m[q] = m[q] < ar ? ar : m[q];
        }
    for (; i < n; ++i) {
        const double a = expx[i] * lx[i];
        aux[i] = a;
        const double r = grad[i] + a;
        rhs[i] = r;
        const double ar = std::fabs(r);
        m[0] = m[0] < ar ? ar : m[0];
    }
    m[0] = m[0] < m[1] ? m[1] : m[0];
    m[2] = m[2] < m[3] ? m[3] : m[2];
    const double graderr = m[0] < m[2] ? m[2] : m[0];
    for (size_t c = 0; c < k; ++c) {   // ComputeLambdaNext (:127-146)
        double v = lambda[c] * g[c];
        for (int32_t j = cptr[c]; j < cptr[c + 1]; ++j) v -= grad[j];
        const double gc = g[c] + 1.0;
        g[c] = gc;
        laux[c] = v / gc;
    }
    for (size_t j = 0; j < n; ++j) lx[j] = laux[ccol[j]];
    for (size_t j = 0; j < n; ++j) {
        const double r = (grad[j] + expx[j] * lx[j]) / aux[j];
        rhs[j] = r;
        x[j] -= u.eta * r;
    }
    for (size_t c = 0; c < k; ++c) laux[c] = lambda[c] - laux[c];
    return graderr;
}

}  // namespace

void QuasiNewtonLearner::OptimizationStep(double eta, bool) {   // :162-201
    // ComputeExpX and ComputeG do not depend on the gradient: run them on
    // the host while the device evaluates (same results as the reference's
    // ExpX, G, Grad order).
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    BeginModeledProbs();
    const auto t1 = clk::now();
    ComputeExpX();
    ComputeG();
    const auto t2 = clk::now();
    EndModeledProbs(grad_cache);
    ComputeRmin(rmin);
    const auto t3 = clk::now();
    grad = grad_cache;
    ComputeObjective();
    const size_t n = _x.size(), k = lambda.size();
    aux.resize(n);
    lambda_min = k ? *std::min_element(lambda.begin(), lambda.end()) : 0.0;
    if (ccol_runs) {
        laux_buf.resize(k);
        lx_buf.resize(n);
        const QnHostUpdate u{n, k, Ccol.data(), cptr_runs.data(), grad.data(), expx.data(), lambda.data(), g.data(),
                             aux.data(), rhs.data(), _x.data(), laux_buf.data(), lx_buf.data(), eta};
        grad_error = qn_host_update(u);
    } else {   // the plain loops (any constraint numbering)
        grad_error = 0.0;
        for (size_t i = 0; i < n; ++i) {
            aux[i] = expx[i] * lambda[size_t(Ccol[i])];   // J_g . lambda
            rhs[i] = grad[i] + aux[i];
            grad_error = std::max(grad_error, std::abs(rhs[i]));
        }
        ComputeLambdaNext(laux_buf);
        for (size_t i = 0; i < n; ++i) {
            rhs[i] = (grad[i] + expx[i] * laux_buf[size_t(Ccol[i])]) / aux[i];
            _x[i] -= eta * rhs[i];
        }
        for (size_t c = 0; c < k; ++c) laux_buf[c] = lambda[c] - laux_buf[c];
    }
    LambdaUpdate(laux_buf.data(), lambda.data(), eta, exponential_lambda);
    const auto t4 = clk::now();
    auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    timing.steps += 1;
    timing.begin_ms += ms(t0, t1);
    timing.overlap_ms += ms(t1, t2);
    timing.wait_ms += ms(t2, t3);
    timing.post_ms += ms(t3, t4);
}

void QuasiNewtonLearner::RunDevice(double eta, double tol, int32_t max_epochs, double* info_rows,
                                   int32_t* epochs_done) {
    using clk = std::chrono::steady_clock;
    const auto te = clk::now();
    if (epochs_done) *epochs_done = 0;
    wfsa_dev* d = Device();
    if (!d) throw LearnerUsageError("BuildFrom has not run");
    wfsa_qn_desc desc{};
    desc.n_params = GetNumberOfParameters();
    desc.n_constraints = GetNumberOfConstraints();
    desc.trim = GetTrimmedIndex().data();
    desc.ccol = Ccol.data();
    desc.plogp = GetPLogP();
    desc.exponential_lambda = exponential_lambda ? 1 : 0;
    desc.info_rmin = RminAvailable() ? 1 : 0;
    auto check = [](int rc, const char* what) {
        if (rc != WFSA_OK) throw LearnerError(what, ": ", wfsa_dev_last_error());
    };
    if (!dev_qn_ready || dev_qn_exp != exponential_lambda || dev_qn_rmin != desc.info_rmin) {   // once per Finalize (and mode)
        PullDeviceState();   // (the set-up may move the device buffers)
        check(wfsa_dev_qn_setup(d, &desc), "wfsa_dev_qn_setup");
        dev_qn_ready = true;
        dev_qn_exp = exponential_lambda;
        dev_qn_rmin = desc.info_rmin;
        dev_state_valid = false;
    }
    static const bool trace = std::getenv("WFSA_VERBOSE") != nullptr;
    const auto t0 = clk::now();
    if (!dev_state_valid) {
        check(wfsa_dev_qn_set_state(d, _x.data(), lambda.data()), "wfsa_dev_qn_set_state");
        dev_state_valid = true;
    }
    const auto t1 = clk::now();
    rows_buf.resize(size_t(std::max(max_epochs, 0)) * 7);
    std::vector<double>& rows = rows_buf;
    int32_t done = 0, status = 0;
    const int rc = wfsa_dev_qn_run(d, eta, tol, max_epochs, rows.data(), &done, &status);
    host_state_stale = true;   // even a failed run may have moved the device state
    check(rc, "wfsa_dev_qn_run");
    if (trace) {
        const auto t2 = clk::now();
        auto us = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
        std::fprintf(stderr, "[wfsa] RunDevice: entry at %lld ns, set-up %.1f us, set_state %.1f us, qn_run %.1f\n",
                     (long long)std::chrono::duration_cast<std::chrono::nanoseconds>(te.time_since_epoch()).count(),
                     us(te, t0), us(t0, t1), us(t1, t2));
    }
    if (info_rows) std::copy(rows.begin(), rows.begin() + std::ptrdiff_t(done) * 7, info_rows);
    if (epochs_done) *epochs_done = done;
    if (done > 0) {
        const double* r = rows.data() + size_t(done - 1) * 7;
        grad_error = r[1];
        g_min = r[2];
        g_max = r[3];
        lambda_min = r[4];
        rmin[0] = r[5];
        rmin[1] = r[6];
        SetEvaluated(GetPLogP() - r[0]);
        timing.steps += done;
        if (status == 2)
            for (int i = 0; i < 7; ++i)
                if (!std::isfinite(r[i])) throw LearnerError(r[i], " detected at epoch ", done);
    }
}

void QuasiNewtonLearner::PullDeviceState() {
    if (!host_state_stale) return;
    wfsa_dev* d = Device();
    if (!d) return;
    if (wfsa_dev_qn_get_state(d, _x.data(), lambda.data(), grad.data()) != WFSA_OK)
        throw LearnerError("wfsa_dev_qn_get_state: ", wfsa_dev_last_error());
    grad_cache = grad;
    host_state_stale = false;
}

}  // namespace wfsa
