#include "SparseLdlt.hpp"

#include <algorithm>
#include <cmath>
#include <limits>
#include <numeric>
#include <set>
#include <utility>
#include <vector>

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

// Approximate minimum degree on the quotient graph (Amestoy, Davis & Duff):
// an eliminated pivot becomes an element whose member list stands for the
// clique it would create; each remaining variable keeps its variable
// neighbours not yet covered by an element and its adjacent elements, and an
// approximate external degree |A_i| + |L_p \ i| + sum over its other
// elements e of |L_e \ L_p| (an upper bound of the true degree).  Elements
// adjacent to the pivot are absorbed into the new one, and so is any element
// whose members all lie in the new one.  A variable with a zero diagonal (a
// constraint row of the KKT system) becomes eligible once a neighbour is
// eliminated; ties go to the most recently updated variable of the lowest
// degree bucket (deterministic).
bool approximate_minimum_degree_order(const SymEntries& a, std::vector<int32_t>& perm) {
    const int32_t n = int32_t(a.n);
    std::vector<std::vector<int32_t>> av(static_cast<size_t>(n)), ev(static_cast<size_t>(n)), le(static_cast<size_t>(n));
    std::vector<double> diag(static_cast<size_t>(n), 0.0);
    for (size_t t = 0; t < a.v.size(); ++t) {
        if (a.i[t] != a.j[t]) {
            av[size_t(a.i[t])].push_back(a.j[t]);
            av[size_t(a.j[t])].push_back(a.i[t]);
        } else {
            diag[size_t(a.i[t])] += a.v[t];
        }
    }
    // 0 variable (in a degree bucket), 1 eliminated, 2 waiting (zero diagonal)
    std::vector<int8_t> state(static_cast<size_t>(n), 0);
    std::vector<char> alive(static_cast<size_t>(n), 0);   // element p not absorbed
    std::vector<int32_t> deg(static_cast<size_t>(n), 0), head(static_cast<size_t>(n) + 1, -1),
        nxt(static_cast<size_t>(n), -1), prv(static_cast<size_t>(n), -1);
    auto insert = [&](int32_t i) {
        const int32_t d = deg[size_t(i)];
        nxt[size_t(i)] = head[size_t(d)];
        prv[size_t(i)] = -1;
        if (head[size_t(d)] >= 0) prv[size_t(head[size_t(d)])] = i;
        head[size_t(d)] = i;
    };
    auto remove = [&](int32_t i) {
        if (prv[size_t(i)] >= 0) nxt[size_t(prv[size_t(i)])] = nxt[size_t(i)];
        else head[size_t(deg[size_t(i)])] = nxt[size_t(i)];
        if (nxt[size_t(i)] >= 0) prv[size_t(nxt[size_t(i)])] = prv[size_t(i)];
    };
    for (int32_t i = 0; i < n; ++i) {
        auto& l = av[size_t(i)];
        std::sort(l.begin(), l.end());
        l.erase(std::unique(l.begin(), l.end()), l.end());
        deg[size_t(i)] = int32_t(l.size());
        if (diag[size_t(i)] != 0.0 || l.empty()) insert(i);
        else state[size_t(i)] = 2;
    }
    std::vector<int32_t> mark(static_cast<size_t>(n), -1), wstamp(static_cast<size_t>(n), -1), wval(static_cast<size_t>(n), 0);
    std::vector<int32_t> lp;
    perm.clear();
    perm.reserve(size_t(n));
    int32_t mindeg = 0, next_waiting = 0;
    for (int32_t k = 0; k < n; ++k) {
        while (mindeg <= n && head[size_t(mindeg)] < 0) ++mindeg;
        int32_t p;
        if (mindeg > n) {   // only waiting variables remain: the lowest index
            while (state[size_t(next_waiting)] != 2) ++next_waiting;
            p = next_waiting;
        } else {
            p = head[size_t(mindeg)];
            remove(p);
        }
        state[size_t(p)] = 1;
        perm.push_back(p);
        // L_p: the pivot's variable neighbours and its elements' members
        lp.clear();
        mark[size_t(p)] = k;
        for (int32_t v : av[size_t(p)])
            if (state[size_t(v)] != 1 && mark[size_t(v)] != k) {
                mark[size_t(v)] = k;
                lp.push_back(v);
            }
        for (int32_t e : ev[size_t(p)]) {
            if (!alive[size_t(e)]) continue;
            for (int32_t v : le[size_t(e)])
                if (state[size_t(v)] != 1 && mark[size_t(v)] != k) {
                    mark[size_t(v)] = k;
                    lp.push_back(v);
                }
            alive[size_t(e)] = 0;   // absorbed into p
            std::vector<int32_t>().swap(le[size_t(e)]);
        }
        std::vector<int32_t>().swap(av[size_t(p)]);
        std::vector<int32_t>().swap(ev[size_t(p)]);
        le[size_t(p)] = lp;
        alive[size_t(p)] = 1;
        // prune the members' lists: elements absorbed -> p; variables now covered by p dropped
        for (int32_t i : lp) {
            if (state[size_t(i)] == 0) remove(i);
            else state[size_t(i)] = 0;   // (a waiting row: its neighbour p is eliminated now)
            auto& e = ev[size_t(i)];
            e.erase(std::remove_if(e.begin(), e.end(), [&](int32_t x) { return !alive[size_t(x)]; }), e.end());
            e.push_back(p);
            auto& v = av[size_t(i)];
            v.erase(std::remove_if(v.begin(), v.end(), [&](int32_t x) { return mark[size_t(x)] == k || state[size_t(x)] == 1; }),
                    v.end());
        }
        // |L_e \ L_p| for the other elements of the members
        for (int32_t i : lp)
            for (int32_t e : ev[size_t(i)]) {
                if (e == p) continue;
                if (wstamp[size_t(e)] != k) {
                    auto& m = le[size_t(e)];
                    m.erase(std::remove_if(m.begin(), m.end(), [&](int32_t x) { return state[size_t(x)] == 1; }), m.end());
                    wstamp[size_t(e)] = k;
                    wval[size_t(e)] = int32_t(m.size());
                }
                --wval[size_t(e)];
            }
        // approximate degrees; an element inside L_p is absorbed
        const int32_t np = int32_t(lp.size());
        for (int32_t i : lp) {
            int64_t d = int64_t(av[size_t(i)].size()) + (np - 1);
            auto& e = ev[size_t(i)];
            for (int32_t x : e) {
                if (x == p) continue;
                if (wval[size_t(x)] <= 0) {
                    alive[size_t(x)] = 0;
                    std::vector<int32_t>().swap(le[size_t(x)]);
                } else {
                    d += wval[size_t(x)];
                }
            }
            e.erase(std::remove_if(e.begin(), e.end(), [&](int32_t x) { return !alive[size_t(x)]; }), e.end());
            d = std::min<int64_t>(d, n - k - 1);
            deg[size_t(i)] = int32_t(d);
            insert(i);
            mindeg = std::min(mindeg, int32_t(d));
        }
    }
    return true;
}

namespace {

constexpr double kBkAlpha = 0.6403882032022076;   // (1 + sqrt(17)) / 8: Bunch-Kaufman's growth bound
constexpr double kPivotThreshold = 0.1;           // a pivot's multipliers at most 1 / u (MA57 allows 0.01 .. 0.1)

}  // namespace

bool SparseLdlt::Analyze(const SymEntries& a, int order) {
    const int32_t n = int32_t(a.n);
    n_ = n;
    bool ok = true;
    if (order == kMinimumDegree) {
        ok = minimum_degree_order(a, perm);
    } else if (order == kApproxMinimumDegree) {
        ok = approximate_minimum_degree_order(a, perm);
    } else {
        perm.resize(size_t(n));
        std::iota(perm.begin(), perm.end(), 0);
    }
    // the elimination tree and column counts (Liu) of the pattern under an
    // order; ap/ai: the permuted upper pattern by column (rows < k)
    std::vector<int32_t> pinv(static_cast<size_t>(n)), parent, lnz;
    std::vector<int64_t> ap;
    std::vector<int32_t> ai;
    auto symbolic = [&]() {
        for (int32_t k = 0; k < n; ++k) pinv[size_t(perm[size_t(k)])] = k;
        std::vector<int64_t> cnt(size_t(n) + 1, 0);
        for (size_t t = 0; t < a.v.size(); ++t) {
            const int32_t r = pinv[size_t(a.i[t])], c = pinv[size_t(a.j[t])];
            if (r != c) ++cnt[size_t(std::max(r, c)) + 1];
        }
        std::partial_sum(cnt.begin(), cnt.end(), cnt.begin());
        ap = cnt;
        ai.assign(size_t(ap.back()), 0);
        for (size_t t = 0; t < a.v.size(); ++t) {
            const int32_t r = pinv[size_t(a.i[t])], c = pinv[size_t(a.j[t])];
            if (r != c) ai[size_t(cnt[size_t(std::max(r, c))]++)] = std::min(r, c);
        }
        parent.assign(size_t(n), -1);
        lnz.assign(size_t(n), 0);
        std::vector<int32_t> flag(size_t(n), -1);
        for (int32_t k = 0; k < n; ++k) {
            flag[size_t(k)] = k;
            for (int64_t q = ap[size_t(k)]; q < ap[size_t(k) + 1]; ++q)
                for (int32_t i = ai[size_t(q)]; flag[size_t(i)] != k; i = parent[size_t(i)]) {
                    if (parent[size_t(i)] == -1) parent[size_t(i)] = k;
                    ++lnz[size_t(i)];
                    flag[size_t(i)] = k;
                }
        }
    };
    symbolic();
    // postorder the elimination tree (children in index order, iteratively)
    // and renumber, so that every subtree is a contiguous range
    {
        std::vector<int32_t> first_child(size_t(n), -1), sibling(size_t(n), -1), post;
        post.reserve(size_t(n));
        for (int32_t j = n - 1; j >= 0; --j)
            if (parent[size_t(j)] >= 0) {
                sibling[size_t(j)] = first_child[size_t(parent[size_t(j)])];
                first_child[size_t(parent[size_t(j)])] = j;
            }
        std::vector<int32_t> stack;
        for (int32_t r = 0; r < n; ++r) {
            if (parent[size_t(r)] != -1) continue;
            stack.push_back(r);
            while (!stack.empty()) {
                const int32_t v = stack.back();
                if (first_child[size_t(v)] >= 0) {   // descend into the next unvisited child
                    const int32_t c = first_child[size_t(v)];
                    first_child[size_t(v)] = sibling[size_t(c)];
                    stack.push_back(c);
                } else {
                    post.push_back(v);
                    stack.pop_back();
                }
            }
        }
        std::vector<int32_t> np(static_cast<size_t>(n));
        for (int32_t k = 0; k < n; ++k) np[size_t(k)] = perm[size_t(post[size_t(k)])];
        perm.swap(np);
        symbolic();
    }
    pinv_ = pinv;
    flops = 0.0;
    for (int32_t k = 0; k < n; ++k) flops += double(lnz[size_t(k)]) * double(lnz[size_t(k)]);
    // fundamental supernodes: j joins j - 1's when j is j - 1's parent, its
    // only child, and the structures nest (count(j - 1) = count(j) + 1)
    std::vector<int32_t> nchild(size_t(n), 0);
    for (int32_t j = 0; j < n; ++j)
        if (parent[size_t(j)] >= 0) ++nchild[size_t(parent[size_t(j)])];
    sn_.clear();
    std::vector<int32_t> sn_of(static_cast<size_t>(n), -1);
    for (int32_t j = 0; j < n; ++j) {
        const bool join = j > 0 && parent[size_t(j) - 1] == j && nchild[size_t(j)] == 1 &&
                          lnz[size_t(j) - 1] == lnz[size_t(j)] + 1;
        if (!join) {
            sn_.emplace_back();
            sn_.back().first = j;
        }
        sn_.back().ncol++;
        sn_of[size_t(j)] = int32_t(sn_.size()) - 1;
    }
    // each supernode's rows: its columns, then the structure below its last
    // column -- the entries below of its columns and its children's rows
    std::vector<int64_t> lo_ptr(size_t(n) + 1, 0);   // the permuted lower pattern by column (rows > k)
    for (size_t q = 0; q < ai.size(); ++q) ++lo_ptr[size_t(ai[q]) + 1];
    std::partial_sum(lo_ptr.begin(), lo_ptr.end(), lo_ptr.begin());
    std::vector<int32_t> lo_idx(ai.size());
    {
        std::vector<int64_t> fill(lo_ptr.begin(), lo_ptr.end() - 1);
        for (int32_t k = 0; k < n; ++k)
            for (int64_t q = ap[size_t(k)]; q < ap[size_t(k) + 1]; ++q) lo_idx[size_t(fill[size_t(ai[size_t(q)])]++)] = k;
    }
    std::vector<int32_t> mark(static_cast<size_t>(n), -1), below;
    nnz_l = 0;
    supernodes = int64_t(sn_.size());
    max_front = 0;
    for (size_t s = 0; s < sn_.size(); ++s) {
        Super& S = sn_[s];
        const int32_t last = S.first + S.ncol - 1;
        S.parent = parent[size_t(last)] >= 0 ? sn_of[size_t(parent[size_t(last)])] : -1;
        below.clear();
        for (int32_t j = S.first; j <= last; ++j)
            for (int64_t q = lo_ptr[size_t(j)]; q < lo_ptr[size_t(j) + 1]; ++q) {
                const int32_t r = lo_idx[size_t(q)];
                if (r > last && mark[size_t(r)] != int32_t(s)) {
                    mark[size_t(r)] = int32_t(s);
                    below.push_back(r);
                }
            }
        S.rows.clear();
        for (int32_t j = S.first; j <= last; ++j) S.rows.push_back(j);
        std::sort(below.begin(), below.end());
        S.rows.insert(S.rows.end(), below.begin(), below.end());   // (children merged below, in postorder)
    }
    // the children's rows (postorder: every child precedes its parent)
    for (size_t s = 0; s < sn_.size(); ++s) {
        const Super& S = sn_[s];
        if (S.parent < 0) continue;
        Super& P = sn_[size_t(S.parent)];
        const int32_t plast = P.first + P.ncol - 1;
        below.clear();
        for (size_t q = size_t(P.ncol); q < P.rows.size(); ++q) below.push_back(P.rows[q]);
        const size_t nb0 = below.size();
        for (size_t q = size_t(S.ncol); q < S.rows.size(); ++q)
            if (S.rows[q] > plast) below.push_back(S.rows[q]);
        if (below.size() > nb0) {
            std::sort(below.begin(), below.end());
            below.erase(std::unique(below.begin(), below.end()), below.end());
            P.rows.resize(size_t(P.ncol));
            P.rows.insert(P.rows.end(), below.begin(), below.end());
        }
    }
    for (const Super& S : sn_) {
        const int64_t m = int64_t(S.rows.size()), nf = S.ncol;
        nnz_l += nf * (nf - 1) / 2 + nf * (m - nf);
        max_front = std::max(max_front, m);
    }
    fr_.assign(sn_.size(), Front{});
    return ok;
}

bool SparseLdlt::Factor(const SymEntries& a) {
    const int32_t n = int32_t(n_);
    positive = negative = zero = two_by_two = delayed = 0;
    nnz_l = max_front = 0;
    log_abs_det = 0.0;
    det_sign = 1;
    min_pivot_ratio = 0.0;
    // the entries by supernode (of their lower column), and each row's largest |entry|
    std::vector<int32_t> sn_of(static_cast<size_t>(n), 0);
    for (size_t s = 0; s < sn_.size(); ++s)
        for (int32_t j = sn_[s].first; j < sn_[s].first + sn_[s].ncol; ++j) sn_of[size_t(j)] = int32_t(s);
    std::vector<int64_t> eptr(sn_.size() + 1, 0);
    std::vector<double> rowmax(static_cast<size_t>(n), 0.0);
    for (size_t t = 0; t < a.v.size(); ++t) {
        const int32_t r = pinv_[size_t(a.i[t])], c = pinv_[size_t(a.j[t])];
        ++eptr[size_t(sn_of[size_t(std::min(r, c))]) + 1];
        rowmax[size_t(r)] = std::max(rowmax[size_t(r)], std::abs(a.v[t]));
        rowmax[size_t(c)] = std::max(rowmax[size_t(c)], std::abs(a.v[t]));
    }
    std::partial_sum(eptr.begin(), eptr.end(), eptr.begin());
    std::vector<int64_t> ent(a.v.size());
    {
        std::vector<int64_t> fill(eptr.begin(), eptr.end() - 1);
        for (size_t t = 0; t < a.v.size(); ++t) {
            const int32_t r = pinv_[size_t(a.i[t])], c = pinv_[size_t(a.j[t])];
            ent[size_t(fill[size_t(sn_of[size_t(std::min(r, c))])]++)] = int64_t(t);
        }
    }
    struct Update {
        std::vector<int32_t> rows;   // the delayed columns first, then the structure
        int32_t ndelay = 0;
        std::vector<double> u;       // rows.size()^2, row-major, the lower triangle
    };
    std::vector<Update> stack;
    std::vector<int32_t> nkids(sn_.size(), 0);
    for (const Super& S : sn_)
        if (S.parent >= 0) ++nkids[size_t(S.parent)];
    std::vector<int32_t> rel(static_cast<size_t>(n), -1), rows, lperm;
    std::vector<double> F, l1, l2;
    double ratio = std::numeric_limits<double>::infinity();
    for (size_t s = 0; s < sn_.size(); ++s) {
        const Super& S = sn_[s];
        // the front: the children's delayed columns, the supernode's columns, the structure below
        rows.clear();
        const size_t nstack = stack.size(), kid0 = nstack - size_t(nkids[s]);
        for (size_t q = kid0; q < nstack; ++q)
            rows.insert(rows.end(), stack[q].rows.begin(), stack[q].rows.begin() + stack[q].ndelay);
        const int32_t ndel_in = int32_t(rows.size());
        rows.insert(rows.end(), S.rows.begin(), S.rows.end());
        const int32_t m = int32_t(rows.size()), nf = ndel_in + S.ncol;
        max_front = std::max<int64_t>(max_front, m);
        F.assign(size_t(m) * size_t(m), 0.0);   // row-major, the lower triangle held
        for (int32_t q = 0; q < m; ++q) rel[size_t(rows[size_t(q)])] = q;
        auto at = [&](int32_t i, int32_t j) -> double& { return F[size_t(i) * size_t(m) + size_t(j)]; };
        auto sym = [&](int32_t i, int32_t j) { return i >= j ? at(i, j) : at(j, i); };
        for (int64_t q = eptr[s]; q < eptr[s + 1]; ++q) {   // the entries
            const int64_t t = ent[size_t(q)];
            const int32_t r = rel[size_t(pinv_[size_t(a.i[size_t(t)])])], c = rel[size_t(pinv_[size_t(a.j[size_t(t)])])];
            at(std::max(r, c), std::min(r, c)) += a.v[size_t(t)];
        }
        for (size_t q = kid0; q < nstack; ++q) {   // extend-add of the children's updates (postorder: the stack's top)
            const Update& U = stack[q];
            const int32_t mu = int32_t(U.rows.size());
            std::vector<int32_t> map(static_cast<size_t>(mu));
            for (int32_t x = 0; x < mu; ++x) map[size_t(x)] = rel[size_t(U.rows[size_t(x)])];
            for (int32_t x = 0; x < mu; ++x)
                for (int32_t y = 0; y <= x; ++y) {
                    const int32_t r = map[size_t(x)], c = map[size_t(y)];
                    at(std::max(r, c), std::min(r, c)) += U.u[size_t(x) * size_t(mu) + size_t(y)];
                }
        }
        stack.resize(kid0);
        // partial Bunch-Kaufman over the fully summed columns [0, nf)
        lperm.resize(size_t(m));
        std::iota(lperm.begin(), lperm.end(), 0);
        Front& R = fr_[s];
        R.piv.assign(size_t(nf), 1);
        R.d.assign(size_t(nf) * 2, 0.0);
        auto swap_sym = [&](int32_t p, int32_t q) {   // rows and columns p, q of the lower triangle
            if (p == q) return;
            if (p > q) std::swap(p, q);
            for (int32_t j = 0; j < p; ++j) std::swap(at(p, j), at(q, j));
            for (int32_t j = p + 1; j < q; ++j) std::swap(at(j, p), at(q, j));
            for (int32_t i = q + 1; i < m; ++i) std::swap(at(i, p), at(i, q));
            std::swap(at(p, p), at(q, q));
            std::swap(lperm[size_t(p)], lperm[size_t(q)]);
        };
        auto global_rowmax = [&](int32_t t) { return rowmax[size_t(rows[size_t(lperm[size_t(t)])])]; };
        // the whole remaining column lies in the block at a root: plain
        // Bunch-Kaufman, any nonsingular pivot; elsewhere a pivot must also
        // pass the threshold test (|l| <= 1 / u), else its columns are delayed
        const bool whole = m == nf;
        int32_t k = 0;
        while (k < nf) {
            int32_t size = 0, p = -1, q = -1;
            for (int32_t c = k; c < nf && size == 0; ++c) {   // lead candidates, in order
                const double acc = std::abs(at(c, c));
                double colmax = 0.0, cmax = 0.0;
                int32_t r = -1;   // the largest candidate partner among the fully summed columns
                for (int32_t i = k; i < m; ++i) {
                    if (i == c) continue;
                    const double x = std::abs(sym(i, c));
                    colmax = std::max(colmax, x);
                    if (i < nf && x > cmax) {
                        cmax = x;
                        r = i;
                    }
                }
                if (acc == 0.0 && colmax == 0.0) return false;   // a zero column: singular
                int32_t sz = 1, pp = c;
                double rowmx = 0.0;
                if (acc < kBkAlpha * colmax && r >= 0) {
                    for (int32_t j = k; j < m; ++j)
                        if (j != r) rowmx = std::max(rowmx, std::abs(sym(r, j)));
                    if (acc * rowmx >= kBkAlpha * colmax * colmax) {
                        pp = c;
                    } else if (std::abs(at(r, r)) >= kBkAlpha * rowmx) {
                        pp = r;
                    } else {
                        sz = 2;
                    }
                }
                bool ok;
                if (sz == 1) {
                    const double d = at(pp, pp), cm = pp == c ? colmax : rowmx;
                    ok = d != 0.0 && std::isfinite(d) && (whole || std::abs(d) >= kPivotThreshold * cm);
                } else {
                    const double a11 = at(c, c), a21 = sym(r, c), a22 = at(r, r), det = a11 * a22 - a21 * a21;
                    ok = det != 0.0 && std::isfinite(det);
                    if (ok && !whole) {   // the multipliers of the rows below the block
                        double lmax = 0.0;
                        for (int32_t i = k; i < m; ++i) {
                            if (i == c || i == r) continue;
                            const double w1 = sym(i, c), w2 = sym(i, r);
                            lmax = std::max({lmax, std::abs((w1 * a22 - w2 * a21) / det), std::abs((w2 * a11 - w1 * a21) / det)});
                        }
                        ok = lmax <= 1.0 / kPivotThreshold;
                    }
                }
                if (ok) {
                    size = sz;
                    p = pp;
                    q = sz == 2 ? r : -1;
                }
            }
            if (size == 0) {
                if (whole) return false;   // (no pivot in the whole remaining matrix: singular)
                break;                     // the rest go to the parent's front
            }
            if (size == 1) {
                swap_sym(k, p);
                const double d = at(k, k);
                for (int32_t i = k + 1; i < m; ++i) {
                    const double w = at(i, k);
                    if (w == 0.0) continue;
                    const double l = w / d;
                    for (int32_t j = k + 1; j <= i; ++j) at(i, j) -= l * at(j, k);
                }
                for (int32_t i = k + 1; i < m; ++i) at(i, k) /= d;
                R.piv[size_t(k)] = 1;
                R.d[2 * size_t(k)] = d;
                if (d > 0) ++positive;
                else ++negative;
                log_abs_det += std::log(std::abs(d));
                if (d < 0) det_sign = -det_sign;
                if (global_rowmax(k) > 0) ratio = std::min(ratio, std::abs(d) / global_rowmax(k));
                k += 1;
            } else {
                if (q == k) q = p;   // (the lead's swap moves its partner)
                swap_sym(k, p);
                swap_sym(k + 1, q);
                const double a11 = at(k, k), a21 = at(k + 1, k), a22 = at(k + 1, k + 1);
                const double det = a11 * a22 - a21 * a21;
                // W D^-1 for the rows below, then the trailing update W D^-1 W^T
                l1.assign(size_t(m), 0.0);
                l2.assign(size_t(m), 0.0);
                for (int32_t i = k + 2; i < m; ++i) {
                    const double w1 = at(i, k), w2 = at(i, k + 1);
                    l1[size_t(i)] = (w1 * a22 - w2 * a21) / det;
                    l2[size_t(i)] = (w2 * a11 - w1 * a21) / det;
                }
                for (int32_t i = k + 2; i < m; ++i) {
                    if (l1[size_t(i)] == 0.0 && l2[size_t(i)] == 0.0) continue;
                    for (int32_t j = k + 2; j <= i; ++j) at(i, j) -= l1[size_t(i)] * at(j, k) + l2[size_t(i)] * at(j, k + 1);
                }
                for (int32_t i = k + 2; i < m; ++i) {
                    at(i, k) = l1[size_t(i)];
                    at(i, k + 1) = l2[size_t(i)];
                }
                at(k + 1, k) = 0.0;   // (the block lives in D)
                R.piv[size_t(k)] = 2;
                R.piv[size_t(k) + 1] = 0;
                R.d[2 * size_t(k)] = a11;
                R.d[2 * size_t(k) + 1] = a21;
                R.d[2 * size_t(k) + 2] = a22;
                ++two_by_two;
                if (det < 0) {
                    ++positive;
                    ++negative;
                    det_sign = -det_sign;
                } else if (a11 + a22 > 0) {
                    positive += 2;
                } else {
                    negative += 2;
                }
                log_abs_det += std::log(std::abs(det));
                const double big = std::max({std::abs(a11), std::abs(a21), std::abs(a22)}),
                             rm = std::max(global_rowmax(k), global_rowmax(k + 1));
                if (big > 0 && rm > 0) ratio = std::min(ratio, std::abs(det) / big / rm);
                k += 2;
            }
        }
        const int32_t ne = k;
        delayed += nf - ne;
        // keep the front's rows in pivot order and L (m x ne, column-major);
        // the delayed columns and the Schur complement go to the parent
        R.nelim = ne;
        R.rows.resize(size_t(m));
        for (int32_t t = 0; t < m; ++t) R.rows[size_t(t)] = rows[size_t(lperm[size_t(t)])];
        R.piv.resize(size_t(ne));
        R.d.resize(size_t(ne) * 2 + 1);
        R.l.assign(size_t(m) * size_t(ne), 0.0);
        for (int32_t t = 0; t < ne; ++t)
            for (int32_t i = t + 1; i < m; ++i) R.l[size_t(t) * size_t(m) + size_t(i)] = at(i, t);
        nnz_l += int64_t(ne) * (ne - 1) / 2 + int64_t(ne) * (m - ne);
        if (S.parent >= 0) {
            Update U;
            U.rows.assign(R.rows.begin() + ne, R.rows.end());
            U.ndelay = nf - ne;
            const int32_t mu = m - ne;
            U.u.resize(size_t(mu) * size_t(mu));
            for (int32_t x = 0; x < mu; ++x)
                for (int32_t y = 0; y <= x; ++y) U.u[size_t(x) * size_t(mu) + size_t(y)] = at(ne + x, ne + y);
            stack.push_back(std::move(U));
        } else if (ne < m) {
            return false;   // (a root with columns left: singular)
        }
        for (int32_t q = 0; q < m; ++q) rel[size_t(rows[size_t(q)])] = -1;
    }
    min_pivot_ratio = ratio;
    return true;
}

void SparseLdlt::Solve(const double* b, double* x) const {
    const int32_t n = int32_t(n_);
    std::vector<double> y(static_cast<size_t>(n)), z;
    for (int32_t k = 0; k < n; ++k) y[size_t(k)] = b[perm[size_t(k)]];
    for (size_t s = 0; s < fr_.size(); ++s) {   // L z = y, front by front
        const Front& R = fr_[s];
        const int32_t m = int32_t(R.rows.size()), ne = R.nelim;
        z.resize(size_t(ne));
        for (int32_t t = 0; t < ne; ++t) z[size_t(t)] = y[size_t(R.rows[size_t(t)])];
        for (int32_t t = 0; t < ne; ++t) {
            const double zt = z[size_t(t)];
            if (zt == 0.0) continue;
            const double* l = &R.l[size_t(t) * size_t(m)];
            for (int32_t i = t + 1; i < ne; ++i) z[size_t(i)] -= l[i] * zt;
            for (int32_t i = ne; i < m; ++i) y[size_t(R.rows[size_t(i)])] -= l[i] * zt;
        }
        for (int32_t t = 0; t < ne; ++t) y[size_t(R.rows[size_t(t)])] = z[size_t(t)];
    }
    for (const Front& R : fr_) {   // D
        for (int32_t t = 0; t < R.nelim; ++t) {
            double& y1 = y[size_t(R.rows[size_t(t)])];
            if (R.piv[size_t(t)] == 1) {
                y1 /= R.d[2 * size_t(t)];
            } else if (R.piv[size_t(t)] == 2) {
                double& y2 = y[size_t(R.rows[size_t(t) + 1])];
                const double a11 = R.d[2 * size_t(t)], a21 = R.d[2 * size_t(t) + 1], a22 = R.d[2 * size_t(t) + 2];
                const double det = a11 * a22 - a21 * a21;
                const double u = (a22 * y1 - a21 * y2) / det, v = (a11 * y2 - a21 * y1) / det;
                y1 = u;
                y2 = v;
            }
        }
    }
    for (size_t s = fr_.size(); s-- > 0;) {   // L^T
        const Front& R = fr_[s];
        const int32_t m = int32_t(R.rows.size()), ne = R.nelim;
        z.resize(size_t(ne));
        for (int32_t t = 0; t < ne; ++t) z[size_t(t)] = y[size_t(R.rows[size_t(t)])];
        for (int32_t t = ne - 1; t >= 0; --t) {
            const double* l = &R.l[size_t(t) * size_t(m)];
            double acc = z[size_t(t)];
            for (int32_t i = t + 1; i < ne; ++i) acc -= l[i] * z[size_t(i)];
            for (int32_t i = ne; i < m; ++i) acc -= l[i] * y[size_t(R.rows[size_t(i)])];
            z[size_t(t)] = acc;
        }
        for (int32_t t = 0; t < ne; ++t) y[size_t(R.rows[size_t(t)])] = z[size_t(t)];
    }
    for (int32_t k = 0; k < n; ++k) x[perm[size_t(k)]] = y[size_t(k)];
}

int SparseLdlt::SolveRefined(const SymEntries& a, const double* b, double* x, int max_steps) const {
    const size_t n = size_t(n_);
    Solve(b, x);
    std::vector<double> r(n), dx(n), xt(n), mag(n);
    auto backward_error = [&](const double* xv) {   // max_i |b - A x|_i / (|A||x| + |b|)_i, r = b - A x
        a.multiply(xv, r.data());
        std::fill(mag.begin(), mag.end(), 0.0);
        for (size_t t = 0; t < a.v.size(); ++t) {
            const double v = std::abs(a.v[t]);
            mag[size_t(a.i[t])] += v * std::abs(xv[a.j[t]]);
            if (a.i[t] != a.j[t]) mag[size_t(a.j[t])] += v * std::abs(xv[a.i[t]]);
        }
        double e = 0.0;
        for (size_t i = 0; i < n; ++i) {
            r[i] = b[i] - r[i];
            const double d = mag[i] + std::abs(b[i]);
            if (d > 0) e = std::max(e, std::abs(r[i]) / d);
        }
        return e;
    };
    double err = backward_error(x);
    int steps = 0;
    while (steps < max_steps && err > 4 * std::numeric_limits<double>::epsilon()) {
        Solve(r.data(), dx.data());
        for (size_t i = 0; i < n; ++i) xt[i] = x[i] + dx[i];
        const double e2 = backward_error(xt.data());
        if (!(e2 < err)) break;
        std::copy(xt.begin(), xt.end(), x);
        err = e2;
        ++steps;
    }
    return steps;
}

}  // namespace wfsa
