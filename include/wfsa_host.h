/*
 * wfsa_host.h -- C ABI over the host-side mirror of the reference's Learner
 * stack (Fsa / Corpus / Learner / QuasiNewtonLearner), for FFI callers
 * (Python ctypes in this repo's tests and bench).  Each call maps to the
 * reference method named beside it; errors are returned as negative codes
 * with a thread-local message (the reference's MyError::what()).
 */
#ifndef WFSA_HOST_H
#define WFSA_HOST_H

#include <stdint.h>

#include "wfsa_dev.h"

#ifdef __cplusplus
extern "C" {
#endif

const char* wfsa_host_last_error(void);

/* ---- Fsa (inc/Fsa.h) ---------------------------------------------------- */
typedef struct wfsa_fsa wfsa_fsa;
int wfsa_fsa_read_text(const char* text, wfsa_fsa** out);     /* Fsa::Read */
int wfsa_fsa_read_file(const char* path, wfsa_fsa** out);
void wfsa_fsa_free(wfsa_fsa* fsa);
/* the flattened graph handed to wfsa_dev_load_model (valid while fsa lives) */
int wfsa_fsa_desc(wfsa_fsa* fsa, wfsa_model_desc* out);
/* counts: states, transitions, emissions, parameters, constraints, free params */
int wfsa_fsa_counts(wfsa_fsa* fsa, int64_t out[6]);
/* Fsa parameter j -> owning state name, kind (0 emission / 1 transition), label */
int wfsa_fsa_param_name(wfsa_fsa* fsa, int32_t j, const char** state, int32_t* kind, const char** label);

/* ---- Corpus (inc/Corpus.h) ---------------------------------------------- */
typedef struct wfsa_corpus wfsa_corpus;
int wfsa_corpus_read_text(const char* text, wfsa_corpus** out);   /* Corpus::Read */
int wfsa_corpus_read_file(const char* path, wfsa_corpus** out);
void wfsa_corpus_free(wfsa_corpus* c);
/* packed view: strings back to back, off[n+1]; weights as read (not normalized) */
int wfsa_corpus_view(wfsa_corpus* c, const uint8_t** sym, const int64_t** off, const double** weights,
                     int64_t* n_strings);

/* ---- Learner (inc/Learner.h, inc/QuasiNewtonLearner.h) ------------------ */
typedef struct wfsa_learner wfsa_learner;

typedef struct {
    int64_t n_strings;        /* recognized, all ranks (GetNumberOfStrings)   */
    int64_t n_local_strings;  /* recognized on this rank                      */
    int64_t n_paths;          /* sum of path counts (GetNumberOfPaths)        */
    int32_t n_full;           /* Fsa parameters                               */
    int32_t n_params;         /* after Trim (GetNumberOfParameters)           */
    int32_t n_constraints;
    int32_t unique_paths;
    int64_t aux_params;
    double common_support, plogp, model_volume, aux_hessian, kl, loglik;
    int64_t shard_begin, shard_end;
} wfsa_learner_info;

/* optimizer: "Hessian" (inc/HessianLearner.h, the reference's default) or
 * "QuasiNewton" (inc/QuasiNewtonLearner.h) */
int wfsa_learner_create(const char* optimizer, int device, wfsa_learner** out);
/* values per GetOptimizationInfo row: 9 (Hessian), 7 (QuasiNewton) */
int wfsa_learner_info_width(wfsa_learner* l);
void wfsa_learner_destroy(wfsa_learner* l);
int wfsa_learner_set_comm(wfsa_learner* l, int nranks, int rank, const uint8_t id[WFSA_COMM_ID_BYTES]);
/* this rank failed outside the library: every other rank's current or next
 * collective fails at once (wfsa_dev_comm_abort).  The learner calls that
 * sit between collectives (build, finalize, init, step, run, objective_grad,
 * load_matrices) do this themselves when they fail. */
int wfsa_learner_comm_abort(wfsa_learner* l, const char* why);
/* the same over a host all-reduce callback (wfsa_dev_comm_init_host) */
int wfsa_learner_set_comm_host(wfsa_learner* l, int nranks, int rank, wfsa_host_allreduce_fn fn, void* user);
/* Learner::BuildFrom on (Fsa, Corpus); the corpus is renormalized first as
 * main.cpp does.  With a communicator each rank keeps its shard. */
int wfsa_learner_build(wfsa_learner* l, wfsa_fsa* fsa, wfsa_corpus* corpus);
/* the same from packed strings + raw weights (renormalized here) */
int wfsa_learner_build_packed(wfsa_learner* l, wfsa_fsa* fsa, const uint8_t* sym, const int64_t* off,
                              const double* weights, int64_t n_strings);
/* The rmin info column (on by default, as the reference prints it every
 * epoch); off: its two columns read 0 and no (min, x) pass runs. */
int wfsa_learner_set_info_rmin(wfsa_learner* l, int on);
/* Matrix-file mode: Learner::LoadMatrices / SaveMatrices (src/Learner.cpp:82-199),
 * prefix.{C,M,P,prob,aux} in the reference's text CSR format; load replaces
 * BuildFrom (no automaton); save works only for loaded matrices. */
int wfsa_learner_load_matrices(wfsa_learner* l, const char* prefix);
int wfsa_learner_save_matrices(wfsa_learner* l, const char* prefix);
int wfsa_learner_finalize(wfsa_learner* l);                                 /* Learner::Finalize */
int wfsa_learner_info_get(wfsa_learner* l, wfsa_learner_info* out);
int wfsa_learner_init(wfsa_learner* l, int flags, const double* x0);       /* Learner::Init */
/* OptimizationStep + GetOptimizationInfo (info_width values) + HaltCondition(tol) */
int wfsa_learner_step(wfsa_learner* l, double eta, double tol, double* info, int32_t* halt);
/* main.cpp's epoch loop (src/main.cpp:276-303) without the per-epoch FFI
 * round trip (QuasiNewton: device-resident): up to max_epochs steps,
 * info_rows[info_width*e..] (nullable) gets each
 * epoch's info, stops after the epoch whose HaltCondition(tol) holds; a
 * non-finite info value fails with "<x> detected at epoch <e>" (the
 * reference's LearnerError) after recording that row. */
int wfsa_learner_run(wfsa_learner* l, double eta, double tol, int32_t max_epochs, double* info_rows,
                     int32_t* epochs_done);
/* ComputeExpX, ComputeGrad, ComputeObjective at the current x:
 * kl, grad[n_params] (trimmed order), logq[n_local_strings] (nullable) */
int wfsa_learner_objective_grad(wfsa_learner* l, double* kl, double* grad, double* logq);
int wfsa_learner_get_x(wfsa_learner* l, double* x);
/* the (trimmed) gradient of the last evaluation: after a device-resident
 * run, the gradient of its last step (at the weights that step started from) */
int wfsa_learner_get_grad(wfsa_learner* l, double* grad);
int wfsa_learner_set_x(wfsa_learner* l, const double* x);
int wfsa_learner_get_p(wfsa_learner* l, double* p);                 /* [n_local_strings] */
int wfsa_learner_trimmed_index(wfsa_learner* l, int32_t* out);      /* [n_full]          */
int wfsa_learner_path_counts(wfsa_learner* l, double* out, uint8_t* recognized); /* [shard size] */
int wfsa_learner_renormalize(wfsa_learner* l);                      /* Learner::Renormalize */
/* RewriteWeights into the fsa, then Fsa::Dump to path */
int wfsa_learner_dump(wfsa_learner* l, wfsa_fsa* fsa, const char* path);
int wfsa_learner_stats(wfsa_learner* l, wfsa_dev_stats* out);
/* GetOptimizationResult (src/HessianLearner.cpp:349-372; the -eval output):
 * KL, mxlogx(support), LogModelVolume, LogAuxVolume, logdetHessian,
 * LogDetAuxHessian, n - k, aux - 1 (Hessian only) */
int wfsa_learner_result(wfsa_learner* l, double out[8]);

/* ---- host-only helpers (no device needed) -------------------------------- */
/* Contiguous shard [begin, end) of rank `rank` out of `nranks` over strings
 * with offsets off[0..n], balanced on total length (what Learner::BuildFrom
 * keeps on each rank). */
int wfsa_shard_range(const int64_t* off, int64_t n, int nranks, int rank, int64_t* begin, int64_t* end);
/* Compile the automaton to the byte-step trellis the device walks, without a
 * device: out = {nodes, byte edges, end edges, parameter-list entries}.
 * Fails (WFSA_ERR_MODEL) e.g. on epsilon cycles. */
int wfsa_trellis_compile_stats(const wfsa_model_desc* model, int64_t out[4]);

/* The HessianLearner's sparse LDL^T (SparseLdlt.hpp; MKL DSS's role,
 * src/HessianLearner.cpp:28-57,100-113) on a symmetric matrix given as
 * upper-triangle coordinates (i[t] <= j[t], duplicates add): the order (0
 * identity -- MKL_DSS_MY_ORDER --, 1 exact minimum degree, 2 approximate
 * minimum degree -- init flag 16, the reference's METIS), the multifrontal
 * supernodal Bunch-Kaufman factorisation, and -- when b is given -- x = A^-1 b.
 * out_i = {positive pivots, negative pivots, nnz(L), ordering within its work
 * bound, supernodes, 2x2 pivots, largest front, delayed columns}; out_d = {log|det|, det sign,
 * min pivot ratio}.  Pivots pass a threshold test or their columns are
 * delayed to the parent front; the solve adds up to two steps of iterative
 * refinement.  WFSA_ERR_ARG when singular (a zero column, or no nonsingular
 * pivot left at a root). */
int wfsa_sym_sparse_solve(int64_t n, int64_t nnz, const int32_t* i, const int32_t* j, const double* v, int order,
                          const double* b, double* x, int64_t out_i[8], double out_d[3]);

/* ---- synthetic corpora (bench / tests) ---------------------------------- */
/* family: N states, out-degree D (+ end), E distinct symbols per state out of
 * V printable bytes, stop probability 1/32 per step, lengths capped at
 * max_len; n_strings distinct strings sampled from the automaton; integer
 * weights 1..10.  dense != 0: every state to every state (D ignored). */
typedef struct wfsa_synth wfsa_synth;
int wfsa_synth_make(int32_t n_states, int32_t degree, int32_t vocab, int32_t emissions, int32_t dense,
                    int64_t n_strings, int32_t max_len, uint64_t seed, wfsa_synth** out);
void wfsa_synth_free(wfsa_synth* s);
const char* wfsa_synth_wfsa_text(wfsa_synth* s);
int wfsa_synth_corpus(wfsa_synth* s, const uint8_t** sym, const int64_t** off, const double** weights,
                      int64_t* n_strings);

#ifdef __cplusplus
}
#endif

#endif /* WFSA_HOST_H */
