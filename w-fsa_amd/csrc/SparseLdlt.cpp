#include "SparseLdlt.hpp"

#include <algorithm>
#include <cmath>
#include <limits>
#include <numeric>
#include <set>
#include <utility>

namespace wfsa {

std::vector<double> SymEntries::dense() const {
    std::vector<double> h(size_t(n * n), 0.0);
    for (size_t t = 0; t < v.size(); ++t) {
        h[size_t(int64_t(i[t]) * n + j[t])] += v[t];
        if (i[t] != j[t]) h[size_t(int64_t(j[t]) * n + i[t])] += v[t];
    }
    return h;
}

void SymEntries::multiply(const double* x, double* y) const {
    std::fill(y, y + n, 0.0);
    for (size_t t = 0; t < v.size(); ++t) {
        y[i[t]] += v[t] * x[j[t]];
        if (i[t] != j[t]) y[j[t]] += v[t] * x[i[t]];
    }
}

// Exact minimum degree on the elimination graph: eliminating v joins its
// neighbours into a clique.  Ties go to the lower index (deterministic).  A
// node with a zero diagonal (the KKT system's constraint rows) waits until a
// neighbour is eliminated -- its pivot is then a Schur complement, not 0 --
// since the static order has no 2x2 pivots.
bool minimum_degree_order(const SymEntries& a, std::vector<int32_t>& perm, double work_bound) {
    const int32_t n = int32_t(a.n);
    std::vector<std::vector<int32_t>> adj(static_cast<size_t>(n));
    std::vector<double> diag(static_cast<size_t>(n), 0.0);
    for (size_t t = 0; t < a.v.size(); ++t) {
        if (a.i[t] != a.j[t]) {
            adj[size_t(a.i[t])].push_back(a.j[t]);
            adj[size_t(a.j[t])].push_back(a.i[t]);
        } else {
            diag[size_t(a.i[t])] += a.v[t];
        }
    }
    std::set<std::pair<int32_t, int32_t>> queue;
    std::vector<char> waiting(static_cast<size_t>(n), 0), done(static_cast<size_t>(n), 0);
    for (int32_t u = 0; u < n; ++u) {
        auto& l = adj[size_t(u)];
        std::sort(l.begin(), l.end());
        l.erase(std::unique(l.begin(), l.end()), l.end());
        if (diag[size_t(u)] != 0.0 || l.empty()) queue.insert({int32_t(l.size()), u});
        else waiting[size_t(u)] = 1;
    }
    perm.clear();
    perm.reserve(size_t(n));
    double work = 0.0;
    std::vector<int32_t> merged;
    int32_t next_waiting = 0;
    while (int32_t(perm.size()) < n) {
        if (queue.empty()) {   // only waiting nodes remain: take them in index order
            while (!waiting[size_t(next_waiting)] || done[size_t(next_waiting)]) ++next_waiting;
            waiting[size_t(next_waiting)] = 0;
            queue.insert({int32_t(adj[size_t(next_waiting)].size()), next_waiting});
        }
        const int32_t v = queue.begin()->second;
        queue.erase(queue.begin());
        perm.push_back(v);
        done[size_t(v)] = 1;
        const std::vector<int32_t> nb = std::move(adj[size_t(v)]);
        adj[size_t(v)].clear();
        for (int32_t u : nb) {
            auto& l = adj[size_t(u)];
            if (!waiting[size_t(u)]) queue.erase({int32_t(l.size()), u});
            waiting[size_t(u)] = 0;
            merged.clear();
            std::set_union(l.begin(), l.end(), nb.begin(), nb.end(), std::back_inserter(merged));
            merged.erase(std::remove_if(merged.begin(), merged.end(), [&](int32_t w) { return w == u || w == v; }),
                         merged.end());
            l.swap(merged);
            queue.insert({int32_t(l.size()), u});
            work += double(l.size()) + double(nb.size());
        }
        if (work > work_bound) {
            perm.resize(size_t(n));
            std::iota(perm.begin(), perm.end(), 0);
            return false;
        }
    }
    return true;
}

bool SparseLdlt::Analyze(const SymEntries& a, int order) {
    const int32_t n = int32_t(a.n);
    n_ = n;
    bool ok = true;
    if (order == 1) {
        ok = minimum_degree_order(a, perm);
    } else {
        perm.resize(size_t(n));
        std::iota(perm.begin(), perm.end(), 0);
    }
    pinv_.assign(size_t(n), 0);
    for (int32_t k = 0; k < n; ++k) pinv_[size_t(perm[size_t(k)])] = k;
    // the permuted upper pattern by column (rows < k), and the diagonal's entries
    std::vector<int64_t> cnt(size_t(n) + 1, 0), dcnt(size_t(n) + 1, 0);
    for (size_t t = 0; t < a.v.size(); ++t) {
        const int32_t r = pinv_[size_t(a.i[t])], c = pinv_[size_t(a.j[t])];
        if (r == c) ++dcnt[size_t(r) + 1];
        else ++cnt[size_t(std::max(r, c)) + 1];
    }
    std::partial_sum(cnt.begin(), cnt.end(), cnt.begin());
    std::partial_sum(dcnt.begin(), dcnt.end(), dcnt.begin());
    ap_ = cnt;
    dp_ = dcnt;
    ai_.assign(size_t(ap_.back()), 0);
    src_.assign(size_t(ap_.back()), 0);
    dsrc_.assign(size_t(dp_.back()), 0);
    for (size_t t = 0; t < a.v.size(); ++t) {
        const int32_t r = pinv_[size_t(a.i[t])], c = pinv_[size_t(a.j[t])];
        if (r == c) {
            dsrc_[size_t(dcnt[size_t(r)]++)] = int64_t(t);
        } else {
            const int32_t col = std::max(r, c);
            const int64_t q = cnt[size_t(col)]++;
            ai_[size_t(q)] = std::min(r, c);
            src_[size_t(q)] = int64_t(t);
        }
    }
    // elimination tree and column counts of L (Liu; the LDL package's symbolic pass)
    parent_.assign(size_t(n), -1);
    lnz_.assign(size_t(n), 0);
    std::vector<int32_t> flag(size_t(n), -1);
    for (int32_t k = 0; k < n; ++k) {
        flag[size_t(k)] = k;
        for (int64_t p = ap_[size_t(k)]; p < ap_[size_t(k) + 1]; ++p)
            for (int32_t i = ai_[size_t(p)]; flag[size_t(i)] != k; i = parent_[size_t(i)]) {
                if (parent_[size_t(i)] == -1) parent_[size_t(i)] = k;
                ++lnz_[size_t(i)];
                flag[size_t(i)] = k;
            }
    }
    lp_.assign(size_t(n) + 1, 0);
    flops = 0.0;
    for (int32_t k = 0; k < n; ++k) {
        lp_[size_t(k) + 1] = lp_[size_t(k)] + lnz_[size_t(k)];
        flops += double(lnz_[size_t(k)]) * double(lnz_[size_t(k)]);
    }
    nnz_l = lp_[size_t(n)];
    li_.assign(size_t(nnz_l), 0);
    lx_.assign(size_t(nnz_l), 0.0);
    d_.assign(size_t(n), 0.0);
    return ok;
}

bool SparseLdlt::Factor(const SymEntries& a) {
    const int32_t n = int32_t(n_);
    positive = negative = zero = 0;
    log_abs_det = 0.0;
    det_sign = 1;
    min_pivot_ratio = 0.0;
    std::vector<double> y(size_t(n), 0.0), rowmax(size_t(n), 0.0);
    for (size_t t = 0; t < a.v.size(); ++t) {
        const double x = std::abs(a.v[t]);
        const int32_t r = pinv_[size_t(a.i[t])], c = pinv_[size_t(a.j[t])];
        rowmax[size_t(r)] = std::max(rowmax[size_t(r)], x);
        rowmax[size_t(c)] = std::max(rowmax[size_t(c)], x);
    }
    std::vector<int32_t> pattern(static_cast<size_t>(n)), flag(static_cast<size_t>(n), -1);
    double ratio = std::numeric_limits<double>::infinity();
    for (int32_t k = 0; k < n; ++k) {
        int32_t top = n;
        flag[size_t(k)] = k;
        lnz_[size_t(k)] = 0;
        double dk = 0.0;
        for (int64_t p = dp_[size_t(k)]; p < dp_[size_t(k) + 1]; ++p) dk += a.v[size_t(dsrc_[size_t(p)])];
        for (int64_t p = ap_[size_t(k)]; p < ap_[size_t(k) + 1]; ++p) {
            int32_t i = ai_[size_t(p)];
            y[size_t(i)] += a.v[size_t(src_[size_t(p)])];
            int32_t len = 0;
            for (; flag[size_t(i)] != k; i = parent_[size_t(i)]) {
                pattern[size_t(len++)] = i;
                flag[size_t(i)] = k;
            }
            while (len > 0) pattern[size_t(--top)] = pattern[size_t(--len)];
        }
        for (; top < n; ++top) {   // row k of L: the reach of column k in the etree, topological order
            const int32_t i = pattern[size_t(top)];
            const double yi = y[size_t(i)];
            y[size_t(i)] = 0.0;
            const int64_t p2 = lp_[size_t(i)] + lnz_[size_t(i)];
            for (int64_t p = lp_[size_t(i)]; p < p2; ++p) y[size_t(li_[size_t(p)])] -= lx_[size_t(p)] * yi;
            const double l = yi / d_[size_t(i)];
            dk -= l * yi;
            li_[size_t(p2)] = k;
            lx_[size_t(p2)] = l;
            ++lnz_[size_t(i)];
        }
        d_[size_t(k)] = dk;
        if (!(dk != 0.0) || !std::isfinite(dk)) return false;
        if (rowmax[size_t(k)] > 0) ratio = std::min(ratio, std::abs(dk) / rowmax[size_t(k)]);
        if (dk > 0) ++positive;
        else ++negative;
        log_abs_det += std::log(std::abs(dk));
        if (dk < 0) det_sign = -det_sign;
    }
    min_pivot_ratio = ratio;
    return true;
}

void SparseLdlt::Solve(const double* b, double* x) const {
    const int32_t n = int32_t(n_);
    std::vector<double> y(static_cast<size_t>(n));
    for (int32_t k = 0; k < n; ++k) y[size_t(k)] = b[perm[size_t(k)]];
    for (int32_t j = 0; j < n; ++j)   // L z = y (L by columns)
        for (int64_t p = lp_[size_t(j)]; p < lp_[size_t(j) + 1]; ++p) y[size_t(li_[size_t(p)])] -= lx_[size_t(p)] * y[size_t(j)];
    for (int32_t j = 0; j < n; ++j) y[size_t(j)] /= d_[size_t(j)];
    for (int32_t j = n - 1; j >= 0; --j)   // L^T
        for (int64_t p = lp_[size_t(j)]; p < lp_[size_t(j) + 1]; ++p) y[size_t(j)] -= lx_[size_t(p)] * y[size_t(li_[size_t(p)])];
    for (int32_t k = 0; k < n; ++k) x[perm[size_t(k)]] = y[size_t(k)];
}

}  // namespace wfsa
