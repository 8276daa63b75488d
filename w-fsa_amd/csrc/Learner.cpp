#include "Learner.hpp"

#include "Paths.hpp"

#include <algorithm>
#include <cmath>
#include <limits>
#include <fstream>
#include <iomanip>
#include <numeric>
#include <sstream>
#include <cstring>

namespace wfsa {

void ThrowOnDevError(int rc, const char* what) {
    if (rc != WFSA_OK) throw LearnerError(what, " failed (", rc, "): ", wfsa_dev_last_error());
}

ShardRange shard_range(const int64_t* off, int64_t n, int nranks, int rank) {
    const int64_t total = off[n];
    auto bound = [&](int r) -> int64_t {
        if (r <= 0) return 0;
        if (r >= nranks) return n;
        const long double thr = (long double)total * r / nranks;
        return int64_t(std::lower_bound(off, off + n, int64_t(std::ceil(thr))) - off);
    };
    const int64_t b = bound(rank);
    return ShardRange{b, std::max(b, bound(rank + 1))};
}

Learner::Learner() {}

Learner::~Learner() {
    if (dev) wfsa_dev_destroy(dev);
}

void Learner::SetDevice(int d) {
    if (dev) throw LearnerUsageError("SetDevice must come before BuildFrom");
    device = d;
}

void Learner::SetCommunicator(int n, int r, const uint8_t* id) {
    if (dev) throw LearnerUsageError("SetCommunicator must come before BuildFrom");
    if (n < 1 || r < 0 || r >= n) throw LearnerUsageError("bad communicator: rank ", r, " of ", n);
    nranks = n;
    rank = r;
    if (n > 1) {
        if (!id) throw LearnerError("null communicator id");
        comm_id.assign(id, id + WFSA_COMM_ID_BYTES);
    }
    host_fn = nullptr;
}

void Learner::SetHostCommunicator(int n, int r, wfsa_host_allreduce_fn fn, void* user) {
    if (dev) throw LearnerUsageError("SetCommunicator must come before BuildFrom");
    if (n < 1 || r < 0 || r >= n || (n > 1 && !fn)) throw LearnerError("bad communicator: rank ", r, " of ", n);
    nranks = n;
    rank = r;
    host_fn = fn;
    host_user = user;
}

void Learner::AbortCommunicator(const char* why) {
    if (dev && nranks > 1) (void)wfsa_dev_comm_abort(dev, why);
}

void Learner::EnsureDevice() {
    if (dev) return;
    ThrowOnDevError(wfsa_dev_create(device, &dev), "wfsa_dev_create");
    if (nranks > 1) {
        if (host_fn) ThrowOnDevError(wfsa_dev_comm_init_host(dev, nranks, rank, host_fn, host_user), "wfsa_dev_comm_init_host");
        else ThrowOnDevError(wfsa_dev_comm_init(dev, nranks, rank, comm_id.data()), "wfsa_dev_comm_init");
    }
}

double Learner::AllReduceSum(double v) const {
    if (nranks > 1) ThrowOnDevError(wfsa_dev_allreduce(dev, &v, 1), "wfsa_dev_allreduce");
    return v;
}

// Constraint matrix C (n x k, one 1 per row) and x from the file weights, in
// map iteration order: equivocal emissions, then equivocal transitions, of
// every state (src/Learner.cpp:221-265).
void Learner::BuildConstraints(const Fsa& fsa) {
    model_volume = 0;
    Crow.clear();
    Ccol.clear();
    n_full = int32_t(fsa.GetNumberOfParameters());
    _x.assign(size_t(n_full), 0.0);
    int32_t k = 0;
    auto collect = [&](const auto& group) {
        if (group.size() <= 1) return;
        for (const auto& member : group) {
            if (member.index != int32_t(Ccol.size()))
                throw LearnerError("Indexing error: ", member.index, " != ", Ccol.size());
            Crow.push_back(int32_t(Ccol.size()));
            Ccol.push_back(k);
            _x[size_t(member.index)] = member.logprob;
        }
        ++k;
        model_volume += log_simplex_volume(group.size());
    };
    for (const auto& t : fsa.GetTransitionMtx()) {
        collect(t.second.emissions);
        collect(t.second.transitions);
    }
    Crow.push_back(int32_t(Ccol.size()));
}

void Learner::BuildFrom(const Fsa& fsa, const Corpus& corpus, bool) {
    PackedStrings ps;
    std::vector<double> w;
    w.reserve(corpus.size());
    for (const auto& e : corpus) {
        ps.add(e.first);
        w.push_back(e.second);
    }
    BuildFromPacked(fsa, ps.sym.data(), ps.off.data(), w.data(), ps.size());
}

void Learner::BuildFromPacked(const Fsa& fsa, const uint8_t* sym, const int64_t* off, const double* weights,
                              int64_t n_strings) {
    BuildConstraints(fsa);
    BuildPaths(fsa, sym, off, weights, n_strings);
    Trim();
}

// Replacement of Learner::BuildPaths (src/Learner.cpp:276-348): the device
// counting pass gives, per string, recognized / path count, and the used
// parameters (OR over ranks); p keeps the recognized strings' weights in
// corpus order.
void Learner::BuildPaths(const Fsa& fsa, const uint8_t* sym, const int64_t* off, const double* weights, int64_t n) {
    EnsureDevice();
    const ShardRange sr = shard_range(off, n, nranks, rank);
    shard_begin = sr.begin;
    shard_end = sr.end;
    const int64_t ln = shard_end - shard_begin;
    std::vector<int64_t> loff(size_t(ln) + 1);
    for (int64_t s = 0; s <= ln; ++s) loff[size_t(s)] = off[shard_begin + s] - off[shard_begin];
    const uint8_t* lsym = sym + off[shard_begin];
    const double* lw = weights + shard_begin;

    flat.reset(new FlatModel(fsa));
    const wfsa_model_desc desc = flat->desc();
    ThrowOnDevError(wfsa_dev_load_model(dev, &desc), "wfsa_dev_load_model");
    ThrowOnDevError(wfsa_dev_load_corpus(dev, lsym, loff.data(), lw, ln), "wfsa_dev_load_corpus");
    recognized_local.assign(size_t(ln), 0);
    path_count_local.assign(size_t(ln), 0.0);
    std::vector<uint8_t> used(size_t(std::max(n_full, 1)), 0);
    ThrowOnDevError(wfsa_dev_recognize(dev, recognized_local.data(), path_count_local.data(), used.data()),
                    "wfsa_dev_recognize");

    // p over recognized strings; the rest become auxiliary parameters
    p.clear();
    PackedStrings rec;
    double stats[5] = {0, 0, 0, 0, 0};   // support, #aux, aux_hessian, #strings, #paths
    double non_unique = 0;
    for (int64_t s = 0; s < ln; ++s) {
        if (recognized_local[size_t(s)]) {
            p.push_back(lw[s]);
            stats[0] += lw[s];
            stats[3] += 1;
            stats[4] += path_count_local[size_t(s)];
            if (path_count_local[size_t(s)] != 1.0) non_unique += 1;
            rec.sym.insert(rec.sym.end(), lsym + loff[size_t(s)], lsym + loff[size_t(s) + 1]);
            rec.off.push_back(int64_t(rec.sym.size()));
        } else {
            stats[1] += 1;
            stats[2] -= std::log(lw[s]);
        }
    }
    if (nranks > 1) {
        double buf[6] = {stats[0], stats[1], stats[2], stats[3], stats[4], non_unique};
        ThrowOnDevError(wfsa_dev_allreduce(dev, buf, 6), "wfsa_dev_allreduce");
        std::copy(buf, buf + 5, stats);
        non_unique = buf[5];
    }
    common_support = stats[0];
    auxiliary_parameters = int64_t(stats[1]);
    aux_hessian = stats[2];
    n_strings_global = int64_t(stats[3]);
    n_paths_global = int64_t(stats[4]);
    unique_paths = non_unique == 0;

    trimmed_weights.assign(size_t(n_full), -2);   // unused unless on an accepting path
    for (int32_t j = 0; j < n_full; ++j)
        if (used[size_t(j)]) trimmed_weights[size_t(j)] = 0;

    // the per-iteration launches see only the recognized strings
    ThrowOnDevError(wfsa_dev_load_corpus(dev, rec.sym.data(), rec.off.data(), p.data(), int64_t(p.size())),
                    "wfsa_dev_load_corpus");
    w_full.assign(size_t(n_full), 0.0);
    grad_full.assign(size_t(n_full), 0.0);
    logq_valid = false;
}

namespace {

// ReadCsrMtx (src/Utils.cpp:184-202): a row per line, "col value" pairs
// until the line stops parsing (a trailing half pair is dropped)
void read_csr(std::istream& is, std::vector<double>& data, std::vector<int32_t>& rows, std::vector<int32_t>& cols) {
    data.clear();
    rows.clear();
    cols.clear();
    std::string line;
    while (std::getline(is, line)) {
        rows.push_back(int32_t(cols.size()));
        std::istringstream iss(line);
        int32_t c;
        double d;
        while (iss >> c >> d) {
            cols.push_back(c);
            data.push_back(d);
        }
    }
    rows.push_back(int32_t(cols.size()));
}

// WriteCsrMtx (src/Utils.cpp:204-214)
void write_csr(std::ostream& os, const std::vector<double>* data, const std::vector<int32_t>& rows,
               const std::vector<int32_t>& cols) {
    for (size_t r = 0; r + 1 < rows.size(); ++r) {
        for (int32_t k = rows[r]; k < rows[r + 1]; ++k) os << cols[size_t(k)] << ' ' << (data ? (*data)[size_t(k)] : 1.0) << ' ';
        os << '\n';
    }
}

}  // namespace

bool Learner::LoadMatrices(const std::string& prefix) {   // src/Learner.cpp:125-199
    if (nranks > 1) throw LearnerError("matrix-file mode runs on one rank");
    auto m = std::make_unique<Matrices>();
    auto open = [&](const char* ext) {
        std::ifstream ifs(prefix + ext);
        if (!ifs) throw LearnerError("Unable to open \"", prefix + ext, "\"!");
        return ifs;
    };
    {
        auto ifs = open(".C");
        read_csr(ifs, m->cdata, m->crow, m->ccol);
    }
    {
        auto ifs = open(".M");
        read_csr(ifs, m->mdata, m->mrow, m->mcol);
    }
    {
        auto ifs = open(".P");
        read_csr(ifs, m->pdata, m->prow, m->pcol);
    }
    std::vector<double> prob;
    {
        std::ifstream ifs(prefix + ".prob");
        double v;
        while (ifs >> v) prob.push_back(v);
    }
    {
        auto ifs = open(".aux");
        double cs, pl, mv, ah;
        int64_t na;
        if (!(ifs >> cs >> pl >> mv >> ah >> na)) throw LearnerError("Invalid data in \"", prefix + ".aux", "\"!");
        common_support = cs;
        plogp = pl;
        model_volume = mv;
        aux_hessian = ah;
        auxiliary_parameters = na;
    }
    const int64_t n = int64_t(m->ccol.size());
    const int64_t n_paths = int64_t(m->prow.size()) - 1, S = int64_t(prob.size());
    if (S + 1 != int64_t(m->mrow.size())) throw LearnerError("Size mismatch: ", S + 1, " != ", m->mrow.size());
    if (!m->pcol.empty() && *std::max_element(m->pcol.begin(), m->pcol.end()) >= n)
        throw LearnerError("Size mismatch: more path indexes than parameters in the automaton!");
    if (m->mcol.empty() || m->mcol.back() + 1 != n_paths) throw LearnerError("M cols != P rows");
    for (size_t i = 1; i < m->ccol.size(); ++i)
        if (m->ccol[i] < m->ccol[i - 1]) throw LearnerError("constraint columns must be non-decreasing");

    Crow = m->crow;
    Ccol = m->ccol;
    p = prob;
    _x.assign(size_t(n), 0.0);
    n_full = int32_t(n);
    trimmed_weights.resize(size_t(n));
    std::iota(trimmed_weights.begin(), trimmed_weights.end(), 0);
    n_strings_global = S;
    n_paths_global = int64_t(m->mcol.size());
    unique_paths = m->mrow.size() == m->mcol.size() + 1;   // Learner::HasUniquePaths (:585-588)
    shard_begin = 0;
    shard_end = S;
    path_count_local.assign(size_t(S), 0.0);
    recognized_local.assign(size_t(S), 1);
    for (int64_t s = 0; s < S; ++s) path_count_local[size_t(s)] = double(m->mrow[size_t(s) + 1] - m->mrow[size_t(s)]);

    EnsureDevice();
    std::vector<int64_t> prow(m->prow.begin(), m->prow.end()), mrow(m->mrow.begin(), m->mrow.end()),
        mcol(m->mcol.begin(), m->mcol.end());
    ThrowOnDevError(wfsa_dev_load_paths(dev, int32_t(n), n_paths, prow.data(), m->pcol.data(), m->pdata.data(), S,
                                        mrow.data(), mcol.data(), p.data()),
                    "wfsa_dev_load_paths");
    flat.reset();
    w_full.assign(size_t(n), 0.0);
    grad_full.assign(size_t(n), 0.0);
    logq_valid = false;
    matrices = std::move(m);
    return true;
}

void Learner::EnumeratePaths(const Fsa& fsa, const Corpus& corpus, bool bfs) {
    if (nranks > 1) throw LearnerError("path enumeration runs on one rank");
    auto m = std::make_unique<Matrices>();
    typedef std::vector<std::pair<int32_t, double>> Path;   // (parameter, count), sorted
    auto add = [](Path& h, int32_t j) {   // SortedInsert(history, j) += 1
        auto it = std::lower_bound(h.begin(), h.end(), j, [](const auto& a, int32_t b) { return a.first < b; });
        if (it == h.end() || it->first != j) it = h.insert(it, {j, 0.0});
        it->second += 1.0;
    };
    const char* end_state = fsa.GetEndState();
    bool has_path = false;
    auto acc = [&](Path& h, const Fsa::NextState& t, const Fsa::NamedProb& e) {
        if (t.index >= 0) add(h, t.index);
        if (std::strcmp(t.next->first, end_state) != 0 && e.index >= 0) add(h, e.index);
    };
    auto done = [&](const Path& path) {
        if (!has_path) m->mrow.push_back(int32_t(m->mcol.size()));
        has_path = true;
        m->prow.push_back(int32_t(m->pcol.size()));
        for (const auto& v : path) {
            m->pdata.push_back(v.second);
            m->pcol.push_back(v.first);
        }
        m->mcol.push_back(int32_t(m->mcol.size()));
    };
    auto rec = make_recognizer<Path>(fsa, acc, done);
    for (const auto& word : corpus) {
        has_path = false;
        rec.Recognize(word.first.c_str(), Path(), bfs);
    }
    m->mrow.push_back(int32_t(m->mcol.size()));
    m->prow.push_back(int32_t(m->pcol.size()));
    // Trim's renumbering of P (src/Learner.cpp:397-419): unused and fixed
    // parameters drop out, the rest take their trimmed index
    std::vector<int32_t> pcol;
    std::vector<double> pdata;
    int32_t start = m->prow[0];
    for (size_t r = 0; r + 1 < m->prow.size(); ++r) {
        const int32_t stop = m->prow[r + 1];
        for (int32_t q = start; q < stop; ++q) {
            const int32_t t = trimmed_weights[size_t(m->pcol[size_t(q)])];
            if (t >= 0) {
                pcol.push_back(t);
                pdata.push_back(m->pdata[size_t(q)]);
            }
        }
        start = stop;
        m->prow[r + 1] = int32_t(pcol.size());
    }
    m->pcol.swap(pcol);
    m->pdata.swap(pdata);
    m->crow = Crow;
    m->ccol = Ccol;
    if (int64_t(m->mcol.size()) != n_paths_global || int64_t(m->mrow.size()) - 1 != n_strings_global)
        throw LearnerError("path enumeration found ", m->mrow.size() - 1, " strings and ", m->mcol.size(),
                           " paths; the device counted ", n_strings_global, " and ", n_paths_global);
    enumerated = std::move(m);
}

// PrintC / PrintM / PrintP (src/Learner.cpp:60-80)
void Learner::PrintC(FILE* f) const { print_csr(f, nullptr, Crow, Ccol); }

void Learner::PrintM(FILE* f) const {
    if (const Matrices* m = PathMatrices()) print_csr(f, nullptr, m->mrow, m->mcol);
}

void Learner::PrintP(FILE* f) const {
    if (const Matrices* m = PathMatrices()) print_csr(f, m->pdata.data(), m->prow, m->pcol);
}

bool Learner::SaveMatrices(const std::string& prefix) const {   // src/Learner.cpp:82-123
    if (!HasPathMatrices()) return false;   // after BuildFrom: EnumeratePaths first
    auto put = [&](const char* ext, auto&& body) {
        std::ofstream ofs(prefix + ext);
        if (!ofs) return false;
        ofs.precision(15);   // DBL_DIG
        body(ofs);
        return bool(ofs);
    };
    const Matrices& m = *PathMatrices();
    return put(".C", [&](std::ostream& o) { write_csr(o, nullptr, m.crow, m.ccol); }) &&
           put(".M", [&](std::ostream& o) { write_csr(o, nullptr, m.mrow, m.mcol); }) &&
           put(".P", [&](std::ostream& o) { write_csr(o, &m.pdata, m.prow, m.pcol); }) &&
           put(".prob", [&](std::ostream& o) { for (double v : p) o << v << '\n'; }) &&
           put(".aux", [&](std::ostream& o) {
               o << common_support << '\n' << plogp << '\n' << model_volume << '\n' << aux_hessian << '\n'
                 << auxiliary_parameters << '\n';
           });
}

bool Learner::RminAvailable() const {
    if (!info_rmin || unique_paths || !dev) return false;
    return true;   // every tier, the dense path included (its (min, +) trellis)
}

void Learner::ComputeRmin(double* out) const {
    out[0] = out[1] = 0.0;
    if (!RminAvailable()) return;
    double r = 0.0;
    int64_t s = -1;
    ThrowOnDevError(wfsa_dev_rmin(dev, &r, &s), "wfsa_dev_rmin");
    out[0] = r;
    out[1] = double(s);
}

// Learner::Trim (src/Learner.cpp:350-425) without the P matrix.  Ccol is
// sorted, so a constraint is a run of equal entries.  Entry states before:
// 0 used, -2 unused.  (1) a constraint whose used members number exactly one
// has that member fixed (-1: weight log 1); (2) the members still free get
// consecutive indices in their order, x is compacted the same way, and the
// constraints that keep a free member are renumbered consecutively.
void Learner::Trim() {
    const size_t n = Ccol.size();
    for (size_t run = 0; run < n;) {
        size_t end = run, n_used = 0, only = 0;
        for (; end < n && Ccol[end] == Ccol[run]; ++end)
            if (trimmed_weights[end] >= 0) {
                ++n_used;
                only = end;
            }
        if (n_used == 1) trimmed_weights[only] = -1;
        run = end;
    }
    std::vector<int32_t> con_of_free;   // the renumbered constraint of each free member
    con_of_free.reserve(n);
    int32_t n_free = 0, n_con = 0, cur_con = 0;
    for (size_t j = 0; j < n; ++j) {
        if (trimmed_weights[j] != 0) continue;
        if (n_free == 0 || Ccol[j] != cur_con) {   // the first free member of its constraint
            cur_con = Ccol[j];
            ++n_con;
        }
        _x[size_t(n_free)] = _x[j];   // (n_free <= j: compaction in place)
        trimmed_weights[j] = n_free++;
        con_of_free.push_back(n_con - 1);
    }
    Ccol = std::move(con_of_free);
    Crow.resize(size_t(n_free) + 1);
    _x.resize(size_t(n_free));
}

double Learner::GetWeight(int32_t i) const {   // src/Learner.cpp:427-436
    switch (trimmed_weights[size_t(i)]) {
        case -2: return -std::numeric_limits<double>::infinity();
        case -1: return 0.0;
        default: return _x[size_t(trimmed_weights[size_t(i)])];
    }
}

void Learner::SetWeights(const double* x) { std::copy(x, x + _x.size(), _x.begin()); }

void Learner::Renormalize() {   // src/Learner.cpp:23-43: x -= C log(C^T exp(x))
    const int32_t k = GetNumberOfConstraints();
    std::vector<double> g(size_t(k), 0.0);
    for (size_t i = 0; i < _x.size(); ++i) g[size_t(Ccol[i])] += std::exp(_x[i]);
    for (auto& v : g) v = std::log(v);
    for (size_t i = 0; i < _x.size(); ++i) _x[i] -= g[size_t(Ccol[i])];
}

void Learner::RewriteWeights(Fsa& fsa) const {   // src/Learner.cpp:45-58
    for (auto& t : fsa.GetTransitionMtx()) {
        for (auto& e : t.second.emissions) e.logprob = e.index >= 0 ? GetWeight(e.index) : 0.0;
        for (auto& e : t.second.transitions) e.logprob = e.index >= 0 ? GetWeight(e.index) : 0.0;
    }
}

std::vector<double> Learner::GetOptimizationInfo() { return {}; }
std::string Learner::GetOptimizationHeader() const { return std::string(); }
std::vector<double> Learner::GetOptimizationResult(bool) { return {}; }
bool Learner::HaltCondition(double) { return false; }

void Learner::LambdaUpdate(double* lstep, double* l, double eta, bool exponential) const {
    const int32_t k = GetNumberOfConstraints();
    if (!exponential) {
        for (int32_t c = 0; c < k; ++c) l[c] -= eta * lstep[c];
    } else {   // lambda *= exp(-eta * lstep / lambda)
        for (int32_t c = 0; c < k; ++c) l[c] *= std::exp(-eta * (lstep[c] / l[c]));
    }
}

void Learner::FinalizeCallback() {}
void Learner::InitCallback(int) {}

void Learner::Finalize() {   // src/Learner.cpp:466-488
    double local = 0;
    for (double v : p) local += v * std::log(v);
    plogp = AllReduceSum(local);
    logq.assign(p.size(), 0.0);
    grad_cache.assign(_x.size(), 0.0);
    FinalizeCallback();
}

void Learner::Init(int flags, const double* initialx) {
    if (initialx) std::copy(initialx, initialx + _x.size(), _x.begin());
    InitCallback(flags);
}

namespace {
// GetWeight(j) for every full parameter (src/Learner.cpp:427-436): x of its
// trimmed index, log 1 for a fixed singleton (-1), -inf for an unused one (-2)
__attribute__((target_clones("avx2", "default"))) void get_weights(int32_t n, const int32_t* __restrict tw,
                                                                   const double* __restrict x, double* __restrict w) {
    const double ninf = -std::numeric_limits<double>::infinity();
    for (int32_t j = 0; j < n; ++j) {
        const int32_t t = tw[j];
        const double xv = x[t >= 0 ? t : 0];
        w[j] = t >= 0 ? xv : (t == -1 ? 0.0 : ninf);
    }
}
}  // namespace

void Learner::BeginModeledProbs(bool want_logq) {
    if (!dev) throw LearnerUsageError("BuildFrom has not run");
    if (eval_in_flight) throw LearnerUsageError("an evaluation is already in flight");
    // straight into the device's host-mapped staging area (one copy fewer)
    double* staged = n_full > 0 ? wfsa_dev_weights_staging(dev) : nullptr;
    double* w = staged ? staged : w_full.data();
    const double none = 0.0;   // (no kept parameter: every index is negative, x is never read)
    get_weights(n_full, trimmed_weights.data(), _x.empty() ? &none : _x.data(), w);
    ThrowOnDevError(wfsa_dev_objective_grad_begin(dev, staged ? nullptr : w, want_logq ? 1 : 0),
                    "wfsa_dev_objective_grad_begin");
    eval_in_flight = true;
    eval_logq = want_logq;
}

void Learner::EndModeledProbs(std::vector<double>& grad_out) {
    if (!eval_in_flight) throw LearnerUsageError("no evaluation in flight");
    eval_in_flight = false;
    if (eval_logq) logq.resize(p.size());
    ThrowOnDevError(wfsa_dev_objective_grad_end(dev, &loglik, grad_full.data(),
                                                eval_logq ? logq.data() : nullptr),
                    "wfsa_dev_objective_grad_end");
    logq_valid = eval_logq;
    grad_out.resize(_x.size());
    const int32_t* tw = trimmed_weights.data();
    const double* gf = grad_full.data();
    double* go = grad_out.data();
    for (int32_t j = 0; j < n_full; ++j) {   // every kept parameter has exactly one full index
        const int32_t t = tw[j];
        if (t >= 0) go[t] = gf[j];
    }
}

void Learner::EvaluateDevice(std::vector<double>& grad_out, bool want_logq) {
    BeginModeledProbs(want_logq);
    EndModeledProbs(grad_out);
}

void Learner::ComputeModeledProbs() { EvaluateDevice(grad_cache, false); }

void Learner::SetEvaluated(double loglik_value) {
    loglik = loglik_value;
    kl = plogp - loglik;
    logq_valid = false;
}

void Learner::ComputeObjective() { kl = plogp - loglik; }

const std::vector<double>& Learner::GetLogQ() {
    if (!logq_valid) EvaluateDevice(grad_cache, true);
    return logq;
}

}  // namespace wfsa
