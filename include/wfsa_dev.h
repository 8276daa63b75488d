/*
 * wfsa_dev.h -- the drop-in device boundary of the MI355X w-fsa path.
 *
 * The reference (gaebor/w-fsa) has no FFI: its hot path is the body of the
 * Learner class hierarchy.  These C entry points replace, one for one, the
 * hot functions a host-side Learner calls:
 *
 *   wfsa_dev_load_model     <- the Fsa graph walked by Recognizer
 *                              (inc/Fsa.h:26-66, inc/Recognize.h:35-96)
 *   wfsa_dev_load_corpus    <- Corpus strings + p (inc/Corpus.h:16-26,
 *                              src/Learner.cpp:297-302)
 *   wfsa_dev_recognize      <- Learner::BuildPaths (src/Learner.cpp:276-348):
 *                              recognized flag, exact path count per string and
 *                              the "used parameter" marks Trim consumes
 *                              (src/Learner.cpp:310, :350-425)
 *   wfsa_dev_objective_grad <- Learner::ComputeModeledProbs + ComputeObjective
 *                              (src/Learner.cpp:515-553) and
 *                              QuasiNewtonLearner::ComputeGrad
 *                              (src/QuasiNewtonLearner.cpp:93-125) ==
 *                              HessianLearner::ComputeGrad
 *                              (src/HessianLearner.cpp:565-597)
 *   wfsa_dev_comm_*         <- (new) one all-reduce per iteration when the
 *                              corpus is sharded over GPUs (RCCL, or an
 *                              in-process group of contexts)
 *
 * Conventions: plain pointers and sizes, host buffers caller-owned and only
 * touched during the call; all device memory belongs to the context.  Every
 * entry point returns WFSA_OK (0) or a negative code and sets a thread-local
 * message readable with wfsa_dev_last_error() -- the reference throws MyError
 * subclasses with a message (inc/Utils.h:130-141); no exception crosses this
 * ABI.  A context is bound to one device and is not re-entrant.
 */
#ifndef WFSA_DEV_H
#define WFSA_DEV_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WFSA_OK 0
#define WFSA_ERR_ARG (-1)      /* invalid argument / call order            */
#define WFSA_ERR_HIP (-2)      /* HIP runtime failure                       */
#define WFSA_ERR_MODEL (-3)    /* automaton rejected (e.g. epsilon cycle)   */
#define WFSA_ERR_CAPACITY (-4) /* a string's trellis exceeds device limits  */
#define WFSA_ERR_RCCL (-5)     /* collective failure                        */
#define WFSA_ERR_NODEV (-6)    /* no usable gfx950 device / kernels missing */

typedef struct wfsa_dev wfsa_dev;

/* The automaton after Fsa::AssignIndices (src/Fsa.cpp:207-238), flattened.
 * States are 0..n_states-1; per state its emissions (byte strings, possibly
 * empty or multi-byte) and its transitions.  *_param is the Fsa parameter
 * index, or -1 for an unequivocal (single-member) group, whose weight is
 * log 1.  `end` is the end state's id or -1 when nothing transitions to it. */
typedef struct {
    int32_t n_states;
    int32_t start;
    int32_t end;
    int32_t n_params;          /* Fsa::GetNumberOfParameters() ("n_full")   */
    const int32_t* em_ptr;     /* [n_states+1]                              */
    const int64_t* em_off;     /* [n_em] offset of the emission in em_bytes */
    const int32_t* em_len;     /* [n_em]                                    */
    const int32_t* em_param;   /* [n_em]                                    */
    const uint8_t* em_bytes;
    const int32_t* tr_ptr;     /* [n_states+1]                              */
    const int32_t* tr_dst;     /* [n_tr]                                    */
    const int32_t* tr_param;   /* [n_tr]                                    */
} wfsa_model_desc;

typedef struct {
    int64_t n_strings;         /* strings resident on this device           */
    int64_t total_symbols;     /* sum of their lengths                      */
    int32_t max_len;
    int32_t n_nodes;           /* trellis nodes after epsilon removal       */
    int64_t n_edges;           /* byte-consuming composite edges            */
    int64_t n_end_edges;
    int64_t compiled_strings;  /* served by the compiled-stream kernel      */
    int64_t fallback_strings;  /* served by the traversal kernel            */
    int64_t stream_words;      /* compiled main-stream words                */
    int64_t stream_bytes;      /* main-stream bytes incl. chunk padding     */
    int64_t bubble_words;
    int64_t n_bubbles;         /* compiled bubbles (bubble kernel lanes)    */
    int64_t fb_launches;       /* objective_grad calls timed so far         */
    double fb_kernel_ms;       /* sum of their forward-backward kernel time */
    double last_fb_kernel_ms;  /* last call: compiled + traversal kernels   */
    double last_compiled_ms;   /* last call: compiled-stream kernel alone   */
    double last_call_ms;       /* last call, device side, end to end        */
    int64_t last_live_edges;   /* traversal-path trellis edges, last call   */
    int32_t tier1_strings;     /* strings needing the large-slab tier       */
    int32_t waves_per_block;
    double prepare_ms;         /* structural pass + stream compilation      */
    double compiled_kernel_ms; /* sum over calls of the compiled kernel     */
    int32_t graph;             /* last call replayed a captured hipGraph    */
    int32_t dense;             /* the dense fp64 MFMA path serves the model */
    /* filled by wfsa_learner_stats (zero from wfsa_dev_get_stats): host time
     * of the learner's optimization steps, summed over host_steps steps --
     * before the device call is enqueued, overlapped with it, waiting for
     * it, after it (gradient mapping + update) */
    int64_t host_steps;
    double host_begin_ms, host_overlap_ms, host_wait_ms, host_post_ms;
    /* dense path (dense == 1): row slots R and trellis steps T of the packed
     * corpus; each evaluation runs 3 GEMMs of 2 np^2 R flops per step */
    int32_t dense_rows, dense_steps, dense_np;
    int32_t tier2_strings;     /* strings on the global-scratch traversal tier */
    int32_t wave_strings;      /* traversal strings on the wave-per-string pair-table kernel */
    int64_t wave_row_entries;  /* per evaluation: alpha entries it writes (and reads back), sum |D| */
    int64_t wave_pair_edges;   /* per evaluation: pair-list edges one pass walks */
    int32_t comm_ranks;        /* communicator size (1: none) */
    int32_t comm_peer;         /* the one-shot peer all-reduce: 1 on, 0 off / untried, -1 its set-up check failed */
    int64_t slot_chunks;       /* bubble contribution slots, in 16-slot chunks (8 B a slot) */
    int32_t max_group_chunks;  /* chunks of the largest constraint's slot group (one QN block sums it) */
    int32_t wave_pull;         /* the wave kernel pulls (wave_pull_kernel): nodes per lane (4, 6, 8); 0: it pushes (wide2_kernel) */
    int32_t dense_blas;        /* dense path GEMM engine (WFSA_DENSE_ENGINE): 0 our fused MFMA kernels, 1 rocBLAS dgemm + our epilogues, 2 our split-K MFMA kernels + epilogues, 3 our LDS-DMA pipelined MFMA kernels + epilogues */
    int32_t qn_inkernel_waves; /* last device QN run: its update ran inside the stream kernel on this many waves (0: the separate QN step kernel) */
    int32_t qn_batches;        /* ... in this many batches of constraints (at most 64 members each) */
} wfsa_dev_stats;

/* context ---------------------------------------------------------------- */
int wfsa_dev_create(int device, wfsa_dev** out);
void wfsa_dev_destroy(wfsa_dev* ctx);
const char* wfsa_dev_last_error(void);

/* One-time uploads -------------------------------------------------------- */
int wfsa_dev_load_model(wfsa_dev* ctx, const wfsa_model_desc* model);
/* sym: packed bytes, off[n_strings+1] offsets into sym, p[n_strings] weights
 * (the reference's p: corpus weight / sum over ALL strings). */
int wfsa_dev_load_corpus(wfsa_dev* ctx, const uint8_t* sym, const int64_t* off,
                         const double* p, int64_t n_strings);

/* Structural pass (weights ignored) over the loaded strings.  Any output may
 * be NULL.  recognized[s] = 1 iff the string has an accepting path;
 * path_count[s] = number of accepting paths (exact below 2^53);
 * used_param[j] = 1 iff Fsa parameter j lies on an accepting path of some
 * string (OR over ranks when a communicator is attached). */
int wfsa_dev_recognize(wfsa_dev* ctx, uint8_t* recognized, double* path_count,
                       uint8_t* used_param);

/* Dense symmetric-indefinite factorisation in HBM for the HessianLearner's
 * KKT system (MKL DSS in the reference: dss_factor_real / dss_statistics
 * "Inertia", "Determinant" / dss_solve_real, src/HessianLearner.cpp:28-57,
 * 100-113; RealSymmetricLogDet src/Utils.cpp:296-350): Bunch-Kaufman LDL^T
 * (our own right-looking kernels, sym_solver.hip, with LAPACK dsytf2's pivot rule
 * and storage) of a[n*n] (symmetric, either layout); inertia =
 * {positive, negative, zero} pivots of D, log|det| and its sign.  sym_solve
 * overwrites b[n] with A^-1 b (one-workgroup dsytrs kernel). */
int wfsa_dev_sym_factor(wfsa_dev* ctx, int64_t n, const double* a, int64_t inertia[3], double* log_abs_det,
                        int32_t* det_sign);
int wfsa_dev_sym_solve(wfsa_dev* ctx, double* b);
/* The same from the matrix's entries -- upper-triangle coordinates
 * (i[t] <= j[t]; duplicates add), no dense host copy -- assembled in HBM and
 * factored blockwise: Bunch-Kaufman pivots within 128-column diagonal blocks
 * (MKL DSS's supernode-restricted pivoting), the trailing updates as fp64
 * library GEMMs (rocBLAS dsyrkx on MFMA); b (nullable) is solved in place and
 * refined against the entries.  When a block pivot falls under 1e-12 max|A|,
 * L grows past 1e8, or the refined solve misses a backward error of 1e-12,
 * the full Bunch-Kaufman factorisation above is used instead.  *method = 1
 * blocked, 2 full.  sym_solve works after either. */
int wfsa_dev_sym_factor_coo(wfsa_dev* ctx, int64_t n, int64_t nnz, const int32_t* i, const int32_t* j,
                            const double* v, double* b, int64_t inertia[3], double* log_abs_det, int32_t* det_sign,
                            int32_t* method);

/* Matrix-file mode (Learner::LoadMatrices, src/Learner.cpp:125-199; main.cpp
 * -m "<file"): instead of an automaton and strings, the path matrices the
 * reference's BuildPaths builds.  P: n_paths x n_params CSR (prow[n_paths+1],
 * pcol/pdata[prow[n_paths]], parameter counts); M: n_strings x n_paths CSR
 * of ones (mrow[n_strings+1], mcol = path indices); p[n_strings].  Replaces
 * any loaded model and corpus; objective_grad then takes w_full = x
 * (n_params values, no trimming) and computes the reference's SpMV chain
 * (logq = log M exp(P x), grad = -P^T (rpp (.) M^T p)); recognize reports
 * the path counts of M and the parameters P uses; rmin reports the
 * reference's path index.  Leave the mode with wfsa_dev_load_model. */
int wfsa_dev_load_paths(wfsa_dev* ctx, int32_t n_params, int64_t n_paths, const int64_t* prow, const int32_t* pcol,
                        const double* pdata, int64_t n_strings, const int64_t* mrow, const int64_t* mcol,
                        const double* p);

/* The rmin info column (QuasiNewtonLearner::GetOptimizationInfo,
 * src/QuasiNewtonLearner.cpp:80-84; HessianLearner :313-317) at the weights
 * of the last evaluation: *rmin = the smallest relative path probability
 * exp(P x)_path / q_s over all paths of ambiguous strings (path count > 1),
 * exact; *string_index = the loaded string holding that path (-1 when no
 * string is ambiguous).  The reference reports the path's index in its BFS
 * enumeration instead, which has no counterpart without enumerating paths
 * (in matrix-file mode, where paths are given, *string_index is that path
 * index).  On the dense path the candidates are every non-empty string
 * (a (min, +) trellis over its row slots; WFSA_ERR_ARG until an evaluation
 * at real weights has run). */
int wfsa_dev_rmin(wfsa_dev* ctx, double* rmin, int64_t* string_index);

/* Where each loaded string runs (after compilation): tier[s] = -1 compiled
 * stream (trivial words + bubbles), 0 / 1 LDS-slab traversal, 2 wide
 * traversal (global scratch), 3 dense MFMA path, 4 matrix-file mode. */
int wfsa_dev_string_tiers(wfsa_dev* ctx, int8_t* tier);

/* Per-iteration hot path.  w_full[n_params] = Learner::GetWeight(j)
 * (src/Learner.cpp:427-436): x[trim[j]], 0 or -inf.  Outputs:
 *   *loglik        = sum_s p_s log q_s
 *   grad_full[j]   = -sum_s p_s E_{path|s}[count_j]   (NULL allowed)
 *   logq[s]        = log q_s for the loaded strings     (NULL allowed)
 * With a communicator attached, loglik and grad_full are summed over ranks
 * (one RCCL all-reduce) and logq stays local. */
int wfsa_dev_objective_grad(wfsa_dev* ctx, const double* w_full, double* loglik,
                            double* grad_full, double* logq);
/* The same split in two so host work can overlap the device: _begin copies
 * w_full and enqueues the evaluation (plus the all-reduce) and returns;
 * _end waits and writes the outputs.  Exactly one _end per _begin. */
int wfsa_dev_objective_grad_begin(wfsa_dev* ctx, const double* w_full, int want_logq);
int wfsa_dev_objective_grad_end(wfsa_dev* ctx, double* loglik, double* grad_full, double* logq);
/* The host-mapped area _begin copies w_full into (n_params doubles; NULL
 * before a model is loaded; valid until the next load).  A caller may write
 * the weights there itself and pass w_full = NULL to _begin: one copy of
 * the weights fewer per evaluation (the host QN binding does).  Not while an
 * evaluation is in flight.  _begin accepts w_full = NULL only when this was
 * called since the previous _begin (else WFSA_ERR_ARG). */
double* wfsa_dev_weights_staging(wfsa_dev* ctx);

/* Device-resident QuasiNewton: QuasiNewtonLearner::OptimizationStep
 * (src/QuasiNewtonLearner.cpp:162-201) and the epoch loop (src/main.cpp:276-303)
 * with x, lambda and w_full kept in HBM -- one step = the objective/gradient
 * kernels at x, the (all-reduce), and a one-workgroup KKT-diagonal update that
 * writes the next step's weights; steps are enqueued ahead and the host only
 * reads each step's info row.
 *   qn_setup:     once after Trim: trim[n_full] = Learner::trimmed_weights,
 *                 ccol[n_params] = the constraint of each kept parameter (C),
 *                 plogp = sum p log p (over all ranks), InitCallback flag 32.
 *   qn_set_state: x[n_params], lambda[n_constraints] (after Init).
 *   qn_get_state: x, lambda and the last step's gradient (any may be NULL).
 *   qn_run:       up to max_steps steps; info_rows[7*s ..] gets step s's
 *                 GetOptimizationInfo row (KL, graderr, g_min, g_max, lambda_min,
 *                 rmin, rmin string -- both 0 unless info_rmin); stops after the step whose HaltCondition(tol) holds
 *                 (*status = 1) or whose info is not finite (*status = 2). */
typedef struct {
    int32_t n_params;
    int32_t n_constraints;
    const int32_t* trim;       /* [n_full]                                   */
    const int32_t* ccol;       /* [n_params]                                 */
    double plogp;
    int32_t exponential_lambda;
    int32_t info_rmin;         /* fill the rmin columns (wfsa_dev_rmin per step) */
} wfsa_qn_desc;
int wfsa_dev_qn_setup(wfsa_dev* ctx, const wfsa_qn_desc* desc);
int wfsa_dev_qn_set_state(wfsa_dev* ctx, const double* x, const double* lambda);
int wfsa_dev_qn_get_state(wfsa_dev* ctx, double* x, double* lambda, double* grad);
int wfsa_dev_qn_run(wfsa_dev* ctx, double eta, double tol, int32_t max_steps, double* info_rows,
                    int32_t* steps_done, int32_t* status);

/* Second-order term of the objective's Hessian for HessianLearner
 * (ComputeHf, src/HessianLearner.cpp:498-547; pattern as AssembleH :381-446):
 *   hf_setup: builds the pattern -- the pairs (j, k), j <= k, of Fsa
 *             parameters whose counts vary together on some string -- after the
 *             corpus is compiled (bubbles per bubble, traversal-tier strings
 *             per string over their equivocal parameters); fails
 *             (WFSA_ERR_CAPACITY) when a string has more than 512 equivocal
 *             parameters (on any rank), and on the dense path.  With a
 *             communicator the pattern is the union over the ranks and
 *             hf_eval's values are all-reduced.
 *   hf_pairs: the pattern, pairs[2 t], pairs[2 t + 1] (ascending).
 *   hf_eval:  values[t] = sum_s p_s Cov_s(count_j, count_k) at w_full
 *             (HessianLearner adds -values to H). */
int wfsa_dev_hf_setup(wfsa_dev* ctx, int64_t* n_pairs);
int wfsa_dev_hf_pairs(wfsa_dev* ctx, int32_t* pairs);
int wfsa_dev_hf_eval(wfsa_dev* ctx, const double* w_full, double* values);

/* Multi-GPU: one process per GPU.  Rank 0 creates the id, the launcher
 * broadcasts the 128 bytes, every rank attaches.  wfsa_dev_allreduce sums
 * `count` doubles of a host buffer in place over the ranks.
 * wfsa_dev_comm_local_id makes the id of an in-process group instead: up to
 * 16 contexts of ONE process, each driven by its own thread, on one device
 * or on peer-enabled devices; comm_init with that id attaches a member.  The
 * group combines the same values at the same points as RCCL (rank order,
 * blocking), so one GPU runs every multi-rank branch of the path. */
#define WFSA_COMM_ID_BYTES 128
int wfsa_dev_comm_unique_id(uint8_t id[WFSA_COMM_ID_BYTES]);
int wfsa_dev_comm_local_id(int nranks, uint8_t id[WFSA_COMM_ID_BYTES]);
int wfsa_dev_comm_init(wfsa_dev* ctx, int nranks, int rank, const uint8_t id[WFSA_COMM_ID_BYTES]);
int wfsa_dev_allreduce(wfsa_dev* ctx, double* host_buf, int64_t count);

/* Failure semantics across ranks.  A call that takes part in
 * collectives (recognize, objective_grad_begin/_end, qn_setup, qn_run,
 * hf_setup, hf_eval, rmin, allreduce) and fails on one rank for any reason
 * but a bad argument aborts that rank's communicator.  How the others hear
 * of it depends on the transport:
 *   - in-process group: poisoned -- every waiting member wakes with
 *     WFSA_ERR_RCCL now, a later one fails at entry;
 *   - peer sums (the per-step [LL, grad]): every member's peer area gets its
 *     poison word -- their next peer sum fails at entry;
 *   - host callback (gloo, MPI): a poisoned header exchange -- every member
 *     waiting in, or later entering, any collective fails at once;
 *   - RCCL: the communicator is aborted (ncclCommAbort), which does NOT wake
 *     the other processes' pending RCCL calls: each rank's host watchdog
 *     ends them (an asynchronous error, or no progress within
 *     WFSA_COMM_TIMEOUT_S, default 300 s), unless the peer path carried the
 *     call.
 * A peer sum whose wait gives up (WFSA_PEER_TIMEOUT_S, default 120 s)
 * poisons every area too and is reported as WFSA_ERR_RCCL at the next host
 * sync point, never as a NaN result.  wfsa_dev_comm_abort does the same for
 * a failure outside the library (the caller's own work between
 * collectives). */
int wfsa_dev_comm_abort(wfsa_dev* ctx, const char* why);

/* Test entry: the peer all-reduce kernel on one device, the other members'
 * areas local and written beforehand (no second process, no concurrency
 * needed).  mode 0: every member present, out[0] = max |sum - rank-order
 * sum|; 1: the last member never arrives, out[0] = NaN results (the call
 * must give up after timeout_s); 2: the area poisoned before the call, which
 * must fail at entry.  out[1] = status word, out[2] = poisoned areas,
 * out[3] = seconds the call took. */
int wfsa_dev_peer_selftest(int device, int nranks, int64_t n, double timeout_s, int mode, double out[4]);

/* A communicator over a host callback instead of RCCL (one process per rank,
 * several may share a GPU; e.g. torch.distributed over gloo, or MPI):
 * fn(user, buf, count, op) all-reduces a HOST buffer in place -- op 0: sum
 * of doubles, 1: min of doubles, 2: max of bytes -- and returns 0 on
 * success.  Called from the thread that drives ctx.  (New; the reference
 * has no multi-process path.)
 *
 * Sums of up to 65536 doubles (the per-iteration [LL, grad] and the other
 * small vectors) take the one-shot peer all-reduce when it is on: one
 * kernel stores the rank's vector into every member's receive slot over
 * xGMI (IPC-mapped device memory; the pointer itself in an in-process
 * group), raises a flag per chunk and sums the members' slots in rank
 * order -- stream-ordered, no host step.  On by default over RCCL, off
 * otherwise; WFSA_PEER=1 / 0 overrides.  The first such sum checks the
 * path on every rank and all ranks fall back to the transport when any
 * check fails (stats.comm_peer = -1).  Refused (stats.comm_peer = 0) for an
 * in-process group whose members share a device: nothing guarantees their
 * spinning kernels run concurrently there. */
typedef int (*wfsa_host_allreduce_fn)(void* user, void* buf, int64_t count, int32_t op);
int wfsa_dev_comm_init_host(wfsa_dev* ctx, int nranks, int rank, wfsa_host_allreduce_fn fn, void* user);

int wfsa_dev_get_stats(wfsa_dev* ctx, wfsa_dev_stats* out);

#ifdef __cplusplus
}
#endif

#endif /* WFSA_DEV_H */
