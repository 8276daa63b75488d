// C ABI over the host mirror (include/wfsa_host.h).  Exceptions stop here.
#include "wfsa_host.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <memory>
#include <new>
#include <string>
#include <vector>

#include "Corpus.hpp"
#include "Fsa.hpp"
#include "HessianLearner.hpp"
#include "Learner.hpp"
#include "QuasiNewtonLearner.hpp"
#include "SparseLdlt.hpp"
#include "synth.hpp"
#include "trellis_model.hpp"

using namespace wfsa;

struct wfsa_fsa {
    Fsa fsa;
    std::unique_ptr<FlatModel> flat;
};

struct wfsa_corpus {
    Corpus corpus;
    PackedStrings packed;
    std::vector<double> weights;
};

struct wfsa_learner {
    std::unique_ptr<Learner> base;
    QuasiNewtonLearner* qn = nullptr;   // exactly one of these is set
    HessianLearner* hs = nullptr;
    int width() const { return hs ? 9 : 7; }   // GetOptimizationInfo values
    // the learner for a host-side use: (x, lambda, grad) the device-resident
    // loop left on the device come back first; a use that may change x or
    // lambda (writes) makes the next wfsa_learner_run upload them again
    Learner& host(bool writes) {
        if (qn) {
            qn->PullDeviceState();
            if (writes) qn->HostStateChanged();
        }
        return *base;
    }
};

struct wfsa_synth {
    SynthOutput out;
};

namespace {

thread_local std::string g_host_error;

template <class F>
int guarded(F&& f) {
    try {
        f();
        return WFSA_OK;
    } catch (const std::bad_alloc&) {
        g_host_error = "out of memory";
    } catch (const std::exception& e) {
        g_host_error = e.what();
    }
    return WFSA_ERR_ARG;
}

// guarded() for a learner call that may sit between rank collectives: a
// failure on this rank aborts its communicator (wfsa_dev_comm_abort), so the
// other ranks fail at their current or next collective instead of waiting
// (a LearnerUsageError -- a call out of order or with bad arguments, found
// before any collective -- fails the call only, as wfsa_dev's rank guard
// exempts WFSA_ERR_ARG)
template <class F>
int rank_guarded(wfsa_learner* l, F&& f) {
    try {
        f();
        return WFSA_OK;
    } catch (const wfsa::LearnerUsageError& e) {
        g_host_error = e.what();
        return WFSA_ERR_ARG;
    } catch (const std::bad_alloc&) {
        g_host_error = "out of memory";
    } catch (const std::exception& e) {
        g_host_error = e.what();
    }
    l->base->AbortCommunicator(g_host_error.c_str());
    return WFSA_ERR_ARG;
}

int null_arg(const char* what) {
    g_host_error = std::string("null argument: ") + what;
    return WFSA_ERR_ARG;
}

}  // namespace

extern "C" {

const char* wfsa_host_last_error(void) { return g_host_error.c_str(); }

int wfsa_fsa_read_text(const char* text, wfsa_fsa** out) {
    if (!text || !out) return null_arg("text/out");
    *out = nullptr;
    return guarded([&] {
        std::unique_ptr<wfsa_fsa> f(new wfsa_fsa());
        f->fsa.ReadText(text);
        *out = f.release();
    });
}

int wfsa_fsa_read_file(const char* path, wfsa_fsa** out) {
    if (!path || !out) return null_arg("path/out");
    *out = nullptr;
    return guarded([&] {
        FILE* fp = std::fopen(path, "rb");
        if (!fp) throw FsaError("Unable to open \"", path, "\"!");
        std::unique_ptr<wfsa_fsa> f(new wfsa_fsa());
        try {
            f->fsa.Read(fp);
        } catch (...) {
            std::fclose(fp);
            throw;
        }
        std::fclose(fp);
        *out = f.release();
    });
}

void wfsa_fsa_free(wfsa_fsa* f) { delete f; }

int wfsa_fsa_desc(wfsa_fsa* f, wfsa_model_desc* out) {
    if (!f || !out) return null_arg("fsa/out");
    return guarded([&] {
        if (!f->flat) f->flat.reset(new FlatModel(f->fsa));
        *out = f->flat->desc();
    });
}

int wfsa_fsa_counts(wfsa_fsa* f, int64_t out[6]) {
    if (!f || !out) return null_arg("fsa/out");
    out[0] = int64_t(f->fsa.GetNumberOfStates());
    out[1] = int64_t(f->fsa.GetNumberOfTransitions());
    out[2] = int64_t(f->fsa.GetNumberOfEmissions());
    out[3] = int64_t(f->fsa.GetNumberOfParameters());
    out[4] = int64_t(f->fsa.GetNumberOfConstraints());
    out[5] = int64_t(f->fsa.GetNumberOfFreeParameters());
    return WFSA_OK;
}

int wfsa_fsa_param_name(wfsa_fsa* f, int32_t j, const char** state, int32_t* kind, const char** label) {
    if (!f || !state || !kind || !label) return null_arg("fsa/outputs");
    return guarded([&] {
        if (!f->flat) f->flat.reset(new FlatModel(f->fsa));
        if (j < 0 || j >= f->flat->n_params) throw FsaError("parameter index ", j, " out of range");
        *state = f->flat->state_names[size_t(f->flat->param_state[size_t(j)])];
        *kind = f->flat->param_kind[size_t(j)];
        *label = f->flat->param_label[size_t(j)];
    });
}

static void pack_corpus(wfsa_corpus* c) {
    c->packed = PackedStrings();
    c->weights.clear();
    for (const auto& e : c->corpus) {
        c->packed.add(e.first);
        c->weights.push_back(e.second);
    }
}

int wfsa_corpus_read_text(const char* text, wfsa_corpus** out) {
    if (!text || !out) return null_arg("text/out");
    *out = nullptr;
    return guarded([&] {
        std::unique_ptr<wfsa_corpus> c(new wfsa_corpus());
        c->corpus.ReadText(text);
        pack_corpus(c.get());
        *out = c.release();
    });
}

int wfsa_corpus_read_file(const char* path, wfsa_corpus** out) {
    if (!path || !out) return null_arg("path/out");
    *out = nullptr;
    return guarded([&] {
        FILE* fp = std::fopen(path, "rb");
        if (!fp) throw CorpusError("Unable to open \"", path, "\"!");
        std::unique_ptr<wfsa_corpus> c(new wfsa_corpus());
        try {
            c->corpus.Read(fp);
        } catch (...) {
            std::fclose(fp);
            throw;
        }
        std::fclose(fp);
        pack_corpus(c.get());
        *out = c.release();
    });
}

void wfsa_corpus_free(wfsa_corpus* c) { delete c; }

int wfsa_corpus_view(wfsa_corpus* c, const uint8_t** sym, const int64_t** off, const double** weights,
                     int64_t* n) {
    if (!c || !sym || !off || !weights || !n) return null_arg("corpus/outputs");
    *sym = c->packed.sym.data();
    *off = c->packed.off.data();
    *weights = c->weights.data();
    *n = c->packed.size();
    return WFSA_OK;
}

int wfsa_learner_create(const char* optimizer, int device, wfsa_learner** out) {
    if (!optimizer || !out) return null_arg("optimizer/out");
    *out = nullptr;
    return guarded([&] {
        std::unique_ptr<wfsa_learner> l(new wfsa_learner());
        if (std::strcmp(optimizer, "QuasiNewton") == 0) {
            l->qn = new QuasiNewtonLearner();
            l->base.reset(l->qn);
        } else if (std::strcmp(optimizer, "Hessian") == 0) {
            l->hs = new HessianLearner();
            l->base.reset(l->hs);
        } else {
            throw LearnerError("unknown optimizer \"", optimizer, "\" (Hessian or QuasiNewton)");
        }
        l->base->SetDevice(device);
        *out = l.release();
    });
}

void wfsa_learner_destroy(wfsa_learner* l) { delete l; }

int wfsa_learner_set_comm(wfsa_learner* l, int nranks, int rank, const uint8_t id[WFSA_COMM_ID_BYTES]) {
    if (!l) return null_arg("learner");
    return guarded([&] { l->host(true).SetCommunicator(nranks, rank, id); });
}

int wfsa_learner_comm_abort(wfsa_learner* l, const char* why) {
    if (!l) return null_arg("learner");
    l->base->AbortCommunicator(why ? why : "wfsa_learner_comm_abort");
    return WFSA_OK;
}

int wfsa_learner_set_comm_host(wfsa_learner* l, int nranks, int rank, wfsa_host_allreduce_fn fn, void* user) {
    if (!l) return null_arg("learner");
    return guarded([&] { l->host(true).SetHostCommunicator(nranks, rank, fn, user); });
}

int wfsa_learner_build_packed(wfsa_learner* l, wfsa_fsa* f, const uint8_t* sym, const int64_t* off,
                              const double* weights, int64_t n) {
    if (!l || !f || !off || (n > 0 && (!weights || !sym))) return null_arg("learner/fsa/corpus");
    return rank_guarded(l, [&] {
        double sum = 0.0;
        for (int64_t s = 0; s < n; ++s) sum += weights[s];
        std::vector<double> w(weights, weights + n);
        for (auto& v : w) v /= sum;   // Corpus::Renormalize (main.cpp:154)
        l->host(true).BuildFromPacked(f->fsa, sym, off, w.data(), n);
    });
}

int wfsa_learner_build(wfsa_learner* l, wfsa_fsa* f, wfsa_corpus* c) {
    if (!l || !f || !c) return null_arg("learner/fsa/corpus");
    return wfsa_learner_build_packed(l, f, c->packed.sym.data(), c->packed.off.data(), c->weights.data(),
                                     c->packed.size());
}

int wfsa_learner_set_info_rmin(wfsa_learner* l, int on) {
    if (!l) return null_arg("learner");
    return guarded([&] { l->base->SetInfoRmin(on != 0); });
}

int wfsa_learner_load_matrices(wfsa_learner* l, const char* prefix) {
    if (!l || !prefix) return null_arg("learner/prefix");
    return rank_guarded(l, [&] { l->host(true).LoadMatrices(prefix); });
}

int wfsa_learner_save_matrices(wfsa_learner* l, const char* prefix) {
    if (!l || !prefix) return null_arg("learner/prefix");
    return guarded([&] {
        if (!l->host(false).SaveMatrices(prefix))
            throw LearnerError("no path matrices to save: only matrices that were loaded exist on this build");
    });
}

int wfsa_learner_finalize(wfsa_learner* l) {
    if (!l) return null_arg("learner");
    return rank_guarded(l, [&] {
        l->host(true);
        if (l->base->GetNumberOfParameters() == 0) throw LearnerError("Empty automaton!");
        if (l->base->GetNumberOfStrings() == 0) throw LearnerError("Automaton cannot generate any of the strings!");
        l->base->Finalize();
    });
}

int wfsa_learner_info_get(wfsa_learner* l, wfsa_learner_info* o) {
    if (!l || !o) return null_arg("learner/out");
    Learner& q = *l->base;
    o->n_strings = q.GetNumberOfStrings();
    o->n_local_strings = q.GetNumberOfLocalStrings();
    o->n_paths = q.GetNumberOfPaths();
    o->n_full = q.GetNumberOfFullParameters();
    o->n_params = q.GetNumberOfParameters();
    o->n_constraints = q.GetNumberOfConstraints();
    o->unique_paths = q.HasUniquePaths() ? 1 : 0;
    o->aux_params = q.GetNumberOfAuxParameters();
    o->common_support = q.GetCommonSupport();
    o->plogp = q.GetPLogP();
    o->model_volume = q.LogModelVolume();
    o->aux_hessian = q.LogDetAuxiliaryHessian();
    o->kl = q.GetKLDistance();
    o->loglik = q.GetLogLikelihood();
    o->shard_begin = q.ShardBegin();
    o->shard_end = q.ShardEnd();
    return WFSA_OK;
}

int wfsa_learner_init(wfsa_learner* l, int flags, const double* x0) {
    if (!l) return null_arg("learner");
    return rank_guarded(l, [&] { l->host(true).Init(flags, x0); });
}

int wfsa_learner_info_width(wfsa_learner* l) { return l ? l->width() : 0; }

int wfsa_learner_step(wfsa_learner* l, double eta, double tol, double* info, int32_t* halt) {
    if (!l) return null_arg("learner");
    return rank_guarded(l, [&] {
        l->host(true).OptimizationStep(eta, false);
        const auto v = l->base->GetOptimizationInfo();
        if (info)
            for (size_t i = 0; i < size_t(l->width()); ++i) info[i] = i < v.size() ? v[i] : 0.0;
        if (halt) *halt = l->base->HaltCondition(tol) ? 1 : 0;
    });
}

int wfsa_learner_run(wfsa_learner* l, double eta, double tol, int32_t max_epochs, double* info_rows,
                     int32_t* epochs_done) {
    if (!l) return null_arg("learner");
    if (epochs_done) *epochs_done = 0;
    return rank_guarded(l, [&] {   // src/main.cpp:276-303
        if (l->qn) {   // device-resident
            l->qn->RunDevice(eta, tol, max_epochs, info_rows, epochs_done);
            return;
        }
        const int w = l->width();
        for (int32_t e = 1; e <= max_epochs; ++e) {
            l->base->OptimizationStep(eta, false);
            const auto v = l->base->GetOptimizationInfo();
            if (info_rows)
                for (int i = 0; i < w; ++i) info_rows[size_t(e - 1) * size_t(w) + size_t(i)] = v[size_t(i)];
            if (epochs_done) *epochs_done = e;
            for (double x : v)
                if (!std::isfinite(x)) throw LearnerError(x, " detected at epoch ", e);
            if (l->base->HaltCondition(tol)) break;
        }
    });
}

int wfsa_learner_objective_grad(wfsa_learner* l, double* kl, double* grad, double* logq) {
    if (!l) return null_arg("learner");
    return rank_guarded(l, [&] {
        const std::vector<double>* g;
        l->host(false);
        if (l->qn) {
            l->qn->ComputeExpX();
            l->qn->ComputeGrad();
            g = &l->qn->GetGradient();
        } else {
            l->hs->ComputeExpX();
            l->hs->ComputeGrad();
            g = &l->hs->GetGradient();
        }
        Learner& q = *l->base;
        q.ComputeObjective();
        if (kl) *kl = q.GetKLDistance();
        if (grad) std::memcpy(grad, g->data(), g->size() * sizeof(double));
        if (logq) {
            const auto& lq = q.GetLogQ();
            std::memcpy(logq, lq.data(), lq.size() * sizeof(double));
        }
    });
}

int wfsa_learner_get_x(wfsa_learner* l, double* x) {
    if (!l || !x) return null_arg("learner/x");
    return guarded([&] {
        std::memcpy(x, l->host(false).GetWeights(), size_t(l->base->GetNumberOfParameters()) * sizeof(double));
    });
}

int wfsa_learner_get_grad(wfsa_learner* l, double* grad) {
    if (!l || !grad) return null_arg("learner/grad");
    return guarded([&] {
        const auto& g = l->host(false).GetLastGradient();
        std::memcpy(grad, g.data(), g.size() * sizeof(double));
    });
}

int wfsa_learner_set_x(wfsa_learner* l, const double* x) {
    if (!l || !x) return null_arg("learner/x");
    return guarded([&] { l->host(true).SetWeights(x); });
}

int wfsa_learner_get_p(wfsa_learner* l, double* p) {
    if (!l || !p) return null_arg("learner/p");
    const auto& v = l->base->GetP();
    std::memcpy(p, v.data(), v.size() * sizeof(double));
    return WFSA_OK;
}

int wfsa_learner_trimmed_index(wfsa_learner* l, int32_t* out) {
    if (!l || !out) return null_arg("learner/out");
    const auto& v = l->base->GetTrimmedIndex();
    std::memcpy(out, v.data(), v.size() * sizeof(int32_t));
    return WFSA_OK;
}

int wfsa_learner_path_counts(wfsa_learner* l, double* out, uint8_t* recognized) {
    if (!l) return null_arg("learner");
    const auto& pc = l->base->GetPathCounts();
    const auto& rc = l->base->GetRecognized();
    if (out) std::memcpy(out, pc.data(), pc.size() * sizeof(double));
    if (recognized) std::memcpy(recognized, rc.data(), rc.size());
    return WFSA_OK;
}

int wfsa_learner_renormalize(wfsa_learner* l) {
    if (!l) return null_arg("learner");
    return guarded([&] { l->host(true).Renormalize(); });
}

int wfsa_learner_dump(wfsa_learner* l, wfsa_fsa* f, const char* path) {
    if (!l || !f || !path) return null_arg("learner/fsa/path");
    return guarded([&] {
        l->host(false).RewriteWeights(f->fsa);
        FILE* fp = std::fopen(path, "wb");
        if (!fp) throw LearnerError("Unable to open output file \"", path, "\" for writing!");
        f->fsa.Dump(fp);
        std::fclose(fp);
    });
}

int wfsa_learner_result(wfsa_learner* l, double out[8]) {
    if (!l || !out) return null_arg("learner/out");
    return guarded([&] {
        const auto v = l->host(true).GetOptimizationResult(false);
        for (size_t i = 0; i < 8; ++i) out[i] = i < v.size() ? v[i] : 0.0;
        if (v.empty()) throw LearnerError("this optimizer has no evaluation result");
    });
}

int wfsa_learner_stats(wfsa_learner* l, wfsa_dev_stats* out) {
    if (!l || !out) return null_arg("learner/out");
    if (!l->base->Device()) {
        g_host_error = "learner has no device context yet";
        return WFSA_ERR_ARG;
    }
    const int rc = wfsa_dev_get_stats(l->base->Device(), out);
    if (rc == WFSA_OK && l->qn) {
        const auto& t = l->qn->StepTiming();
        out->host_steps = t.steps;
        out->host_begin_ms = t.begin_ms;
        out->host_overlap_ms = t.overlap_ms;
        out->host_wait_ms = t.wait_ms;
        out->host_post_ms = t.post_ms;
    }
    return rc;
}

int wfsa_shard_range(const int64_t* off, int64_t n, int nranks, int rank, int64_t* begin, int64_t* end) {
    if (!off || !begin || !end || n < 0 || nranks < 1 || rank < 0 || rank >= nranks) return null_arg("shard arguments");
    const ShardRange r = shard_range(off, n, nranks, rank);
    *begin = r.begin;
    *end = r.end;
    return WFSA_OK;
}

int wfsa_sym_sparse_solve(int64_t n, int64_t nnz, const int32_t* i, const int32_t* j, const double* v, int order,
                          const double* b, double* x, int64_t out_i[8], double out_d[3]) {
    if (n < 0 || nnz < 0 || (nnz > 0 && (!i || !j || !v)) || (b && !x) || !out_i || !out_d) return null_arg("matrix");
    if (n > std::numeric_limits<int32_t>::max()) return null_arg("n");
    try {
        SymEntries a(n);
        for (int64_t t = 0; t < nnz; ++t) {
            if (i[t] < 0 || j[t] < 0 || i[t] >= n || j[t] >= n) return null_arg("entry index");
            a.add(i[t], j[t], v[t]);
        }
        SparseLdlt s;
        const bool ordered = s.Analyze(a, order);
        const bool ok = s.Factor(a);
        out_i[0] = s.positive;
        out_i[1] = s.negative;
        out_i[2] = s.nnz_l;
        out_i[3] = ordered ? 1 : 0;
        out_i[4] = s.supernodes;
        out_i[5] = s.two_by_two;
        out_i[6] = s.max_front;
        out_i[7] = s.delayed;
        out_d[0] = s.log_abs_det;
        out_d[1] = s.det_sign;
        out_d[2] = s.min_pivot_ratio;
        if (!ok) {
            g_host_error = "sparse LDL^T: singular (a zero column or a zero / non-finite pivot)";
            return WFSA_ERR_ARG;
        }
        if (b) s.SolveRefined(a, b, x);
        return WFSA_OK;
    } catch (const std::bad_alloc&) {
        g_host_error = "out of host memory";
        return WFSA_ERR_CAPACITY;
    }
}

int wfsa_trellis_compile_stats(const wfsa_model_desc* model, int64_t out[4]) {
    if (!model || !out) return null_arg("model/out");
    TrellisModel tm;
    const std::string err = compile_trellis_model(*model, tm);
    if (!err.empty()) {
        g_host_error = "automaton rejected: " + err;
        return WFSA_ERR_MODEL;
    }
    out[0] = tm.n_nodes;
    out[1] = int64_t(tm.o_byte.size());
    out[2] = int64_t(tm.x_pptr.size()) - 1;
    out[3] = int64_t(tm.o_pidx.size() + tm.x_pidx.size());
    return WFSA_OK;
}

int wfsa_synth_make(int32_t n_states, int32_t degree, int32_t vocab, int32_t emissions, int32_t dense,
                    int64_t n_strings, int32_t max_len, uint64_t seed, wfsa_synth** out) {
    if (!out) return null_arg("out");
    *out = nullptr;
    return guarded([&] {
        SynthSpec spec;
        spec.n_states = n_states;
        spec.degree = degree;
        spec.vocab = vocab;
        spec.emissions = emissions;
        spec.dense = dense;
        spec.n_strings = n_strings;
        spec.max_len = max_len;
        spec.seed = seed;
        std::unique_ptr<wfsa_synth> s(new wfsa_synth());
        const std::string err = make_synthetic(spec, s->out);
        if (!err.empty()) throw MyError(err);
        *out = s.release();
    });
}

void wfsa_synth_free(wfsa_synth* s) { delete s; }

const char* wfsa_synth_wfsa_text(wfsa_synth* s) { return s ? s->out.wfsa_text.c_str() : ""; }

int wfsa_synth_corpus(wfsa_synth* s, const uint8_t** sym, const int64_t** off, const double** weights,
                      int64_t* n) {
    if (!s || !sym || !off || !weights || !n) return null_arg("synth/outputs");
    *sym = s->out.sym.data();
    *off = s->out.off.data();
    *weights = s->out.weights.data();
    *n = int64_t(s->out.weights.size());
    return WFSA_OK;
}

}  // extern "C"
