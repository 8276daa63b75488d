#include "HessianLearner.hpp"

#include <unordered_map>

#include <string>

#include <cstdlib>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <limits>
#include <numeric>

namespace wfsa {

// ---------------------------------------------------------------- LDL^T ----

void DenseLdlt::Factor(std::vector<double>& A, int64_t n) {
    n_ = n;
    perm_.resize(size_t(n));
    std::iota(perm_.begin(), perm_.end(), int64_t(0));
    block_.assign(size_t(n), 1);
    positive = negative = zero = 0;
    log_abs_det = 0.0;
    det_sign = 1;
    const double alpha = (1.0 + std::sqrt(17.0)) / 8.0;   // Bunch-Kaufman
    auto at = [&](int64_t i, int64_t j) -> double& { return A[size_t(i * n + j)]; };
    auto swap_sym = [&](int64_t p, int64_t q) {   // rows and columns p <-> q, L columns included
        if (p == q) return;
        for (int64_t j = 0; j < n; ++j) std::swap(at(p, j), at(q, j));
        for (int64_t i = 0; i < n; ++i) std::swap(at(i, p), at(i, q));
        std::swap(perm_[size_t(p)], perm_[size_t(q)]);
    };
    std::vector<double> c1(static_cast<size_t>(n)), c2(static_cast<size_t>(n));
    auto account = [&](double d) {
        if (d > 0) ++positive;
        else if (d < 0) ++negative;
        else ++zero;
        if (d == 0) {
            log_abs_det = -std::numeric_limits<double>::infinity();
            det_sign = 0;
        } else {
            log_abs_det += std::log(std::abs(d));
            if (d < 0) det_sign = -det_sign;
        }
    };
    int64_t k = 0;
    while (k < n) {
        int64_t kstep = 1, kp = k;
        const double absakk = std::abs(at(k, k));
        int64_t imax = k;
        double colmax = 0.0;
        for (int64_t i = k + 1; i < n; ++i)
            if (std::abs(at(i, k)) > colmax) {
                colmax = std::abs(at(i, k));
                imax = i;
            }
        // (imax == k: no nonzero below the diagonal -- also a NaN column, where
        // a 2x2 pivot could reach past the last row)
        if (imax == k || std::max(absakk, colmax) == 0.0 || absakk >= alpha * colmax) {
            kp = k;
        } else {
            double rowmax = 0.0;
            for (int64_t j = k; j < n; ++j)
                if (j != imax) rowmax = std::max(rowmax, std::abs(at(imax, j)));
            if (absakk >= alpha * colmax * (colmax / rowmax)) {
                kp = k;
            } else if (std::abs(at(imax, imax)) >= alpha * rowmax) {
                kp = imax;
            } else {
                kp = imax;
                kstep = 2;
            }
        }
        const int64_t kk = k + kstep - 1;
        if (kp != kk) swap_sym(kk, kp);
        if (kstep == 1) {
            const double d = at(k, k);
            account(d);
            for (int64_t i = k + 1; i < n; ++i) c1[size_t(i)] = at(i, k);
            for (int64_t i = k + 1; i < n; ++i) {
                const double li = d != 0.0 ? c1[size_t(i)] / d : 0.0;
                if (li != 0.0)
                    for (int64_t j = k + 1; j < n; ++j) at(i, j) -= li * c1[size_t(j)];
                at(i, k) = li;
            }
        } else {
            block_[size_t(k)] = 2;
            block_[size_t(k) + 1] = 0;
            const double d11 = at(k, k), d21 = at(k + 1, k), d22 = at(k + 1, k + 1);
            const double det = d11 * d22 - d21 * d21;
            if (det < 0) {
                ++positive;
                ++negative;
            } else if (det > 0) {
                if (d11 + d22 > 0) positive += 2;
                else negative += 2;
            } else {
                ++zero;
                if (d11 + d22 > 0) ++positive;
                else if (d11 + d22 < 0) ++negative;
                else ++zero;
            }
            if (det == 0) {
                log_abs_det = -std::numeric_limits<double>::infinity();
                det_sign = 0;
            } else {
                log_abs_det += std::log(std::abs(det));
                if (det < 0) det_sign = -det_sign;
            }
            for (int64_t i = k + 2; i < n; ++i) {
                c1[size_t(i)] = at(i, k);
                c2[size_t(i)] = at(i, k + 1);
            }
            for (int64_t i = k + 2; i < n; ++i) {
                const double l1 = (c1[size_t(i)] * d22 - c2[size_t(i)] * d21) / det;
                const double l2 = (c2[size_t(i)] * d11 - c1[size_t(i)] * d21) / det;
                for (int64_t j = k + 2; j < n; ++j) at(i, j) -= l1 * c1[size_t(j)] + l2 * c2[size_t(j)];
                at(i, k) = l1;
                at(i, k + 1) = l2;
            }
        }
        k += kstep;
    }
    a_.swap(A);
}

void DenseLdlt::Solve(const double* b, double* x) const {
    const int64_t n = n_;
    auto L = [&](int64_t i, int64_t j) { return a_[size_t(i * n + j)]; };
    std::vector<double> y(static_cast<size_t>(n));
    for (int64_t i = 0; i < n; ++i) y[size_t(i)] = b[perm_[size_t(i)]];
    for (int64_t k = 0; k < n;) {   // L z = y
        if (block_[size_t(k)] == 1) {
            for (int64_t i = k + 1; i < n; ++i) y[size_t(i)] -= L(i, k) * y[size_t(k)];
            k += 1;
        } else {
            for (int64_t i = k + 2; i < n; ++i) y[size_t(i)] -= L(i, k) * y[size_t(k)] + L(i, k + 1) * y[size_t(k) + 1];
            k += 2;
        }
    }
    for (int64_t k = 0; k < n;) {   // D w = z
        if (block_[size_t(k)] == 1) {
            y[size_t(k)] /= L(k, k);
            k += 1;
        } else {
            const double d11 = L(k, k), d21 = L(k + 1, k), d22 = L(k + 1, k + 1);
            const double det = d11 * d22 - d21 * d21;
            const double r1 = y[size_t(k)], r2 = y[size_t(k) + 1];
            y[size_t(k)] = (d22 * r1 - d21 * r2) / det;
            y[size_t(k) + 1] = (d11 * r2 - d21 * r1) / det;
            k += 2;
        }
    }
    for (int64_t k = n - 1; k >= 0;) {   // L^T u = w
        if (block_[size_t(k)] == 0) {   // second of a 2x2: the pair is (k-1, k)
            const int64_t f = k - 1;
            for (int64_t i = k + 1; i < n; ++i) {
                y[size_t(f)] -= L(i, f) * y[size_t(i)];
                y[size_t(k)] -= L(i, k) * y[size_t(i)];
            }
            k -= 2;
        } else {
            for (int64_t i = k + 1; i < n; ++i) y[size_t(k)] -= L(i, k) * y[size_t(i)];
            k -= 1;
        }
    }
    for (int64_t i = 0; i < n; ++i) x[perm_[size_t(i)]] = y[size_t(i)];
}

// ------------------------------------------------------- HessianLearner ----

void HessianLearner::FinalizeCallback() {   // src/HessianLearner.cpp:19-26
    const size_t n = size_t(GetNumberOfParameters()), k = size_t(GetNumberOfConstraints());
    rhs.assign(n + k, 0.0);
    expx.assign(n, 0.0);
    grad.assign(n, 0.0);
    lambda.assign(k, 1.0);   // _x.resize(n + k, 1.0)
    hf_ready = false;
}

void HessianLearner::InitCallback(int flags) {   // :132-191
    exponential_lambda = (flags & 32) != 0;
    if (flags & 1) {
        std::fill(_x.begin(), _x.end(), 0.0);
        std::fill(lambda.begin(), lambda.end(), 1.0);
    }
    if (flags & 2) Renormalize();
    if (flags & 4) InitSlackVariables();
    include_Hf = (flags & 8) != 0;   // AssembleH(include_Hf)
    if (include_Hf && !HasUniquePaths()) SetupHf();
    reorder = (flags & 16) != 0;   // METIS in the reference: approximate minimum degree for the sparse LDL^T
    degenerate = false;
}

void HessianLearner::InitSlackVariables() {   // :554-563: lambda <- -C^T grad f
    ComputeExpX();
    ComputeGrad();
    std::fill(lambda.begin(), lambda.end(), 0.0);
    for (size_t i = 0; i < grad.size(); ++i) lambda[size_t(Ccol[i])] -= grad[i];
}

void HessianLearner::ComputeExpX() {
    for (size_t i = 0; i < _x.size(); ++i) expx[i] = std::exp(_x[i]);
}

void HessianLearner::ComputeGrad() {   // :565-597, from the device
    ComputeModeledProbs();
    grad = grad_cache;
}

void HessianLearner::ComputeRhs() {   // :610-620: rhs <- [grad f + J_g lambda, C^T exp(x) - 1]
    ComputeExpX();
    ComputeGrad();
    const size_t n = _x.size(), k = lambda.size();
    for (size_t c = 0; c < k; ++c) rhs[n + c] = -1.0;
    for (size_t i = 0; i < n; ++i) {
        rhs[n + size_t(Ccol[i])] += expx[i];
        rhs[i] = grad[i] + expx[i] * lambda[size_t(Ccol[i])];
    }
}

void HessianLearner::SetupHf() {
    if (hf_ready) return;
    wfsa_dev* d = Device();
    int64_t np = 0;
    ThrowOnDevError(wfsa_dev_hf_setup(d, &np), "wfsa_dev_hf_setup");
    std::vector<int32_t> pairs(size_t(2 * np));
    ThrowOnDevError(wfsa_dev_hf_pairs(d, pairs.data()), "wfsa_dev_hf_pairs");
    const auto& tw = GetTrimmedIndex();
    hf_j.resize(size_t(np));
    hf_k.resize(size_t(np));
    for (int64_t t = 0; t < np; ++t) {
        const int32_t a = tw[size_t(pairs[size_t(2 * t)])], b = tw[size_t(pairs[size_t(2 * t) + 1])];
        hf_j[size_t(t)] = a >= 0 ? a : -1;
        hf_k[size_t(t)] = b >= 0 ? b : -1;
    }
    hf_vals.resize(size_t(np));
    hf_ready = true;
}

bool HessianLearner::AddHf(SymEntries& A, bool per_weight) {   // ComputeHf, :498-547
    SetupHf();
    const int32_t nf = GetNumberOfFullParameters();
    w_hf.resize(size_t(nf));
    for (int32_t j = 0; j < nf; ++j) w_hf[size_t(j)] = GetWeight(j);
    ThrowOnDevError(wfsa_dev_hf_eval(Device(), w_hf.data(), hf_vals.data()), "wfsa_dev_hf_eval");
    bool offdiag = false;
    for (size_t t = 0; t < hf_vals.size(); ++t) {
        const int64_t a = hf_j[t], b = hf_k[t];
        if (a < 0 || b < 0) continue;
        const double v = per_weight ? hf_vals[t] / (expx[size_t(a)] * expx[size_t(b)]) : hf_vals[t];
        A.add(a, b, -v);
        offdiag |= a != b;
    }
    return offdiag;
}

namespace {

// WFSA_KKT=host / device / sparse forces one factorisation
std::string kkt_forced() {
    const char* e = std::getenv("WFSA_KKT");
    return e ? std::string(e) : std::string();
}

struct Factored {
    int64_t positive = 0, negative = 0;
    double log_abs_det = 0.0;
    int det_sign = 1;
    char kind = 'h';   // h: host dense, b: device blocked, d: device full Bunch-Kaufman, s: sparse
};

// the sparse LDL^T where it pays (above kHostDense unknowns and within
// kSparseFlops of work, or beyond the dense limit), else the dense
// Bunch-Kaufman factorisation on the host or in HBM; a sparse factorisation
// with a tiny pivot or a solve whose residual is off falls back to the dense
// one (when it fits)
Factored factor_and_solve(wfsa_dev* dev, const SymEntries& A, int order, const double* rhs, double* x) {
    Factored r;
    const int64_t N = A.n;
    const std::string forced = kkt_forced();
    const bool dense_fits = N <= HessianLearner::kMaxDense;
    if (forced == "sparse" || (forced.empty() && N > HessianLearner::kHostDense)) {
        // the requested ordering first; when its factorisation fails, the other
        // one before giving up (a different elimination order meets different
        // pivots and supernodes)
        for (int attempt = 0; attempt < 2; ++attempt) {
            const int other = order == SparseLdlt::kIdentity ? SparseLdlt::kApproxMinimumDegree : SparseLdlt::kIdentity;
            const int ord = attempt == 0 ? order : other;
            SparseLdlt s;
            const bool ordered = s.Analyze(A, ord);
            if (std::getenv("WFSA_VERBOSE"))
                std::fprintf(stderr, "[kkt] N %lld entries %zu order %d%s nnz(L) %lld flops %.3g supernodes %lld front %lld\n",
                             (long long)N, A.v.size(), ord, ordered ? "" : " (work bound: identity)", (long long)s.nnz_l,
                             s.flops, (long long)s.supernodes, (long long)s.max_front);
            if (!(forced == "sparse" || !dense_fits || s.flops <= HessianLearner::kSparseFlops)) break;
            bool ok = s.Factor(A) && (s.min_pivot_ratio > HessianLearner::kSparsePivotFloor || !dense_fits);
            if (ok && rhs) {   // normwise backward error per row: |Ax - b|_i <= tol (|A||x| + |b|)_i
                s.SolveRefined(A, rhs, x);
                std::vector<double> ax(static_cast<size_t>(N)), mag(static_cast<size_t>(N), 0.0);
                A.multiply(x, ax.data());
                for (size_t t = 0; t < A.v.size(); ++t) {
                    const double v = std::abs(A.v[t]);
                    mag[size_t(A.i[t])] += v * std::abs(x[A.j[t]]);
                    if (A.i[t] != A.j[t]) mag[size_t(A.j[t])] += v * std::abs(x[A.i[t]]);
                }
                for (int64_t i = 0; i < N && ok; ++i) {
                    const double res = std::abs(ax[size_t(i)] - rhs[i]);
                    ok = std::isfinite(res) && res <= 1e-9 * (mag[size_t(i)] + std::abs(rhs[i]));
                }
            }
            if (ok) {
                r.positive = s.positive;
                r.negative = s.negative;
                r.log_abs_det = s.log_abs_det;
                r.det_sign = s.det_sign;
                r.kind = 's';
                return r;
            }
        }
        if (!dense_fits) {   // degenerate: no inertia from a partial factorisation
            if (rhs) std::fill(x, x + N, std::numeric_limits<double>::quiet_NaN());
            r.positive = r.negative = 0;
            r.log_abs_det = -std::numeric_limits<double>::infinity();
            r.det_sign = 0;
            r.kind = 's';
            return r;
        }
    }
    if (!dense_fits)   // only a forced dense factorisation gets here
        throw LearnerError("KKT system of ", N, " unknowns: beyond the dense factorisation's ", HessianLearner::kMaxDense,
                           " (WFSA_KKT=", forced, ")");
    const bool device = forced == "device" || (forced != "host" && forced != "sparse" && N > HessianLearner::kHostDense);
    if (!device) {
        std::vector<double> H = A.dense();
        DenseLdlt f;
        f.Factor(H, N);
        r.positive = f.positive;
        r.negative = f.negative;
        r.log_abs_det = f.log_abs_det;
        r.det_sign = f.det_sign;
        if (rhs) f.Solve(rhs, x);
        return r;
    }
    if (!dev) throw LearnerError("no device for the KKT factorisation");
    // assembled in HBM from the entries (no dense host copy): the blocked
    // factorisation, or the full Bunch-Kaufman when it does not hold up
    int64_t inertia[3] = {0, 0, 0};
    int32_t sign = 1, method = 0;
    if (rhs) std::copy(rhs, rhs + N, x);
    ThrowOnDevError(wfsa_dev_sym_factor_coo(dev, N, int64_t(A.v.size()), A.i.data(), A.j.data(), A.v.data(),
                                            rhs ? x : nullptr, inertia, &r.log_abs_det, &sign, &method),
                    "wfsa_dev_sym_factor_coo");
    r.positive = inertia[0];
    r.negative = inertia[1];
    r.det_sign = sign;
    r.kind = method == 1 ? 'b' : 'd';
    if (std::getenv("WFSA_VERBOSE"))
        std::fprintf(stderr, "[kkt] N %lld device %s\n", (long long)N, method == 1 ? "blocked" : "full Bunch-Kaufman");
    return r;
}

}  // namespace

// The reference's sparse KKT layout (AssembleH, :381-467): row i < n holds
// its diagonal, the equivocal pattern's columns j > i (with H_f), then the
// constraint column n + C(i); rows n.. hold their (zero) diagonal.
// with_jg = false: the n x n Hessian of ComputeLogDetHessian (:219-260), the
// constraint column dropped.  Prints it as PrintCsrMtx does (PrintEq with rhs,
// PrintH without, :262-270).
void HessianLearner::PrintKkt(FILE* f, const SymEntries& A, bool with_hf, bool with_jg,
                              const std::vector<double>* rhs_print) {
    const int64_t n = int64_t(_x.size()), k = with_jg ? int64_t(lambda.size()) : 0;
    std::unordered_map<int64_t, double> H;   // (row, col) of the upper triangle -> value, duplicates summed
    H.reserve(A.v.size());
    for (size_t t = 0; t < A.v.size(); ++t) H[int64_t(A.i[t]) * A.n + A.j[t]] += A.v[t];
    auto at = [&](int64_t r, int64_t c) {
        const auto it = H.find(r * A.n + c);
        return it == H.end() ? 0.0 : it->second;
    };
    std::vector<std::vector<int32_t>> upper(static_cast<size_t>(n));
    if (with_hf && !HasUniquePaths()) {
        SetupHf();
        for (size_t t = 0; t < hf_j.size(); ++t)
            if (hf_j[t] >= 0 && hf_k[t] >= 0 && hf_j[t] != hf_k[t])
                upper[size_t(std::min(hf_j[t], hf_k[t]))].push_back(std::max(hf_j[t], hf_k[t]));
    }
    std::vector<int32_t> rows(1, 0), cols;
    std::vector<double> vals;
    for (int64_t i = 0; i < n; ++i) {
        auto& u = upper[size_t(i)];
        std::sort(u.begin(), u.end());
        u.erase(std::unique(u.begin(), u.end()), u.end());
        cols.push_back(int32_t(i));
        for (int32_t j : u) cols.push_back(j);
        if (with_jg) cols.push_back(int32_t(n + Ccol[size_t(i)]));
        rows.push_back(int32_t(cols.size()));
    }
    for (int64_t i = n; i < n + k; ++i) {
        cols.push_back(int32_t(i));
        rows.push_back(int32_t(cols.size()));
    }
    for (size_t r = 0; r + 1 < rows.size(); ++r)
        for (int32_t q = rows[r]; q < rows[r + 1]; ++q) vals.push_back(at(int64_t(r), cols[size_t(q)]));
    print_csr(f, vals.data(), rows, cols, rhs_print);
}

void HessianLearner::OptimizationStep(double eta, bool verbose) {   // :63-130
    ComputeRhs();
    ComputeObjective();
    ComputeRmin(rmin);
    const int64_t n = int64_t(_x.size()), k = int64_t(lambda.size()), N = n + k;
    SymEntries A(N);   // AssembleH's pattern (:381-467), upper triangle
    if (include_Hf && !HasUniquePaths()) AddHf(A, false);
    for (int64_t i = 0; i < n; ++i) {   // ComputeHg, :622-639
        A.add(i, i, expx[size_t(i)] * lambda[size_t(Ccol[size_t(i)])]);
        A.add(i, n + Ccol[size_t(i)], expx[size_t(i)]);
    }
    if (verbose) {   // (:76-80)
        std::fputs("H:\n", stderr);
        PrintKkt(stderr, A, include_Hf, true, &rhs);
    }
    lambda_min = k ? *std::min_element(lambda.begin(), lambda.end()) : 0.0;
    step.assign(size_t(N), 0.0);
    const Factored f = factor_and_solve(Device(), A, reorder ? SparseLdlt::kApproxMinimumDegree : SparseLdlt::kIdentity, rhs.data(), step.data());
    kkt_kind = f.kind;
    inertia_pos = f.positive;
    inertia_neg = f.negative;
    const auto bad = [](double v) { return !std::isfinite(v); };
    if (std::any_of(step.begin(), step.end(), bad)) {
        degenerate = true;
        std::fprintf(stderr,
                     "Solution of Newton step is degenerate at %f%% of the parameters and %f%% of the constraints!\n",
                     100.0 * double(std::count_if(step.begin(), step.begin() + n, bad)) / double(n),
                     100.0 * double(std::count_if(step.begin() + n, step.end(), bad)) / double(std::max<int64_t>(k, 1)));
    } else {
        for (int64_t i = 0; i < n; ++i) _x[size_t(i)] -= eta * step[size_t(i)];
        LambdaUpdate(step.data() + n, lambda.data(), eta, exponential_lambda);
    }
}

std::string HessianLearner::GetOptimizationHeader() const {   // :272-282
    return "       KL   graderr     g_min     g_max         +         - lambdamin      rmin";
}

// [KL, graderr, g_min, g_max, inertia +, inertia -, lambda_min, rmin, rmin
// index] (:284-347); rmin (smallest relative path probability) needs an
// explicit path list and is reported as 0
std::vector<double> HessianLearner::GetOptimizationInfo() {
    std::vector<double> r(9, 0.0);
    const size_t n = _x.size();
    r[0] = GetKLDistance();
    for (size_t i = 0; i < n; ++i) r[1] = std::max(r[1], std::abs(rhs[i]));
    if (rhs.size() > n) {
        r[2] = *std::min_element(rhs.begin() + std::ptrdiff_t(n), rhs.end());
        r[3] = *std::max_element(rhs.begin() + std::ptrdiff_t(n), rhs.end());
    }
    error = std::max(std::max(r[1], std::abs(r[2])), std::abs(r[3]));
    if (!degenerate) {
        r[4] = double(inertia_pos);
        r[5] = double(inertia_neg);
    }
    r[6] = lambda_min;
    r[7] = rmin[0];   // :313-317 (index: the string holding the path, see QuasiNewtonLearner)
    r[8] = rmin[1];
    return r;
}

bool HessianLearner::HaltCondition(double tol) {   // :374-379
    if (degenerate) throw LearnerError("Unable to continue!");
    return error <= tol;
}

// log det of the objective's Hessian in the weights w = exp(x):
// (H_f - diag(grad f)) / (exp(x_j) exp(x_k)) (:219-260)
double HessianLearner::ComputeLogDetHessian(bool verbose) {
    const int64_t n = int64_t(_x.size());
    SymEntries A(n);
    ComputeExpX();
    ComputeGrad();
    const bool offdiag = !HasUniquePaths() && AddHf(A, true);
    for (int64_t j = 0; j < n; ++j) A.add(j, j, -grad[size_t(j)] / (expx[size_t(j)] * expx[size_t(j)]));
    if (verbose) log_det_h = A;   // for PrintH after the Hessian line (:360)
    const double inf = std::numeric_limits<double>::infinity();
    if (!offdiag) {   // diagonal (src/Utils.cpp:300-311)
        std::vector<double> d(static_cast<size_t>(n), 0.0);
        for (size_t t = 0; t < A.v.size(); ++t)
            if (A.i[t] == A.j[t]) d[size_t(A.i[t])] += A.v[t];
        double r = 0.0;
        for (int64_t i = 0; i < n; ++i) {
            if (!(d[size_t(i)] > 0)) return inf;
            r += std::log(d[size_t(i)]);
        }
        return r;
    }
    const Factored f = factor_and_solve(Device(), A, reorder ? SparseLdlt::kApproxMinimumDegree : SparseLdlt::kIdentity, nullptr, nullptr);
    if (f.det_sign <= 0) return inf;   // (:351-352)
    return f.log_abs_det;
}

std::vector<double> HessianLearner::GetOptimizationResult(bool verbose) {   // :349-372
    ComputeModeledProbs();
    ComputeObjective();
    const double logdet = ComputeLogDetHessian(verbose);
    const int64_t n = int64_t(_x.size());
    int64_t nnz = n;
    if (hf_ready)
        for (size_t t = 0; t < hf_j.size(); ++t)
            if (hf_j[t] >= 0 && hf_k[t] >= 0 && hf_j[t] != hf_k[t]) ++nnz;
    std::fprintf(stderr, "Hessian:\n\trows: %lld\n\tnnz: %lld\n\tfill: %g\n", (long long)n, (long long)nnz,
                 n ? double(nnz) / double(n) : 0.0);
    if (verbose && log_det_h.n > 0) {
        PrintKkt(stderr, log_det_h, true, false, nullptr);
        log_det_h = SymEntries();
    }
    return {GetKLDistance(),
            mxlogx(GetCommonSupport()),
            LogModelVolume(),
            LogAuxiliaryVolume(),
            logdet,
            LogDetAuxiliaryHessian(),
            double(GetNumberOfParameters() - GetNumberOfConstraints()),
            double(std::max<int64_t>(0, GetNumberOfAuxParameters() - 1))};
}

}  // namespace wfsa
