/*
 * wfsa_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C99) of gaebor/w-fsa's objective/gradient path, used
 * as the parity checker for the MI355X product.  Nothing in the product links
 * or calls this file; only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg load it (through oracle/oracle.py).
 *
 * Two independent engines:
 *   ENUM    -- the reference algorithm: enumerate every accepting path of every
 *              string (BFS, inc/Recognize.h:62-96 without the 1 s clock cap),
 *              build P (paths x params) and M (strings x paths) exactly as
 *              Learner::BuildPaths (src/Learner.cpp:276-348), Trim
 *              (src/Learner.cpp:350-425), then every iteration the SpMV chain
 *              of ComputeModeledProbs / ComputeObjective / ComputeGrad
 *              (src/Learner.cpp:515-553, src/QuasiNewtonLearner.cpp:93-125).
 *   TRELLIS -- a dense float64 forward-backward over (position, state) with
 *              epsilon emissions in topological order.  Used where ENUM cannot
 *              finish (ambiguous automata); must agree with ENUM elsewhere.
 *
 * Parameter numbering is the oracle's own (states in creation order); results
 * are compared with the product by (state, kind, label) names.
 *
 * PARITY UNPINNED.  The reference cannot be built here (its sources include
 * Intel MKL headers the image lacks), and the only outputs it holds are its
 * CTest exit codes (CMakeLists.txt:34-57), which tests/test_oracle.py
 * reproduces.  The oracle is also checked against SURVEY.md Appendix A
 * (tests/golden/appendix_a.json), but those values came from a build of the
 * reference sources against stand-in MKL headers, so
 * they are a consistency check, not a pin to a reference run.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define OR_OK 0
#define OR_ERR -1

/* ------------------------------------------------------------------------ */
/* small helpers                                                              */
/* ------------------------------------------------------------------------ */

static void* xrealloc(void* p, size_t n) {
    void* q = realloc(p, n ? n : 1);
    if (!q) { fprintf(stderr, "oracle: out of memory\n"); abort(); }
    return q;
}

#define VEC(T) struct { T* a; int64_t n, cap; }
#define VPUSH(v, x) do { if ((v).n == (v).cap) { (v).cap = (v).cap ? 2 * (v).cap : 16; \
    (v).a = xrealloc((v).a, sizeof(*(v).a) * (size_t)(v).cap); } (v).a[(v).n++] = (x); } while (0)
#define VFREE(v) do { free((v).a); (v).a = NULL; (v).n = (v).cap = 0; } while (0)

/* GetWord: restatement of src/Utils.cpp:20-80, including its quirks (a
 * trailing separator before '\n' leaves the cursor on the '\n'; a failed
 * partial separator match does not re-examine the current byte; a separator
 * matched right before end-of-buffer is not cut). */
typedef struct { char* word; char term; } word_t;

static word_t get_word(char** input, const char* separator) {
    char* in = *input;
    char* result = in;
    const char* sep = separator;
    int in_sep = 0;
    while (*in) {
        if (!in_sep) {
            if (*in == *sep) { in_sep = 1; ++sep; }
            else if (*in == '\n') { *(in++) = '\0'; *input = in; return (word_t){result, '\n'}; }
        } else {
            if (*in == *sep) { ++sep; }
            else if (*in == '\n' && *sep == '\0') {
                for (char* w = in - (sep - separator); w < in; ++w) *w = '\0';
                *input = in; return (word_t){result, '\n'};
            } else if (*in == '\n') { *(in++) = '\0'; *input = in; return (word_t){result, '\n'}; }
            else if (*sep == '\0') {
                for (char* w = in - (sep - separator); w < in; ++w) *w = '\0';
                *input = in; return (word_t){result, *(sep - 1)};
            } else { sep = separator; in_sep = 0; }
        }
        ++in;
    }
    *input = in;
    return (word_t){result, '\0'};
}

static int starts_with(const char* word, const char* prefix) {   /* src/Utils.cpp:216-219 */
    return strncmp(word, prefix, strlen(prefix)) == 0;
}

static double log_factorial(size_t d) {
    double r = 0; for (size_t i = 2; i <= d; ++i) r += log((double)i); return r;
}
static double log_simplex_volume(size_t d) {                       /* src/Utils.cpp:221-227 */
    return d > 0 ? 0.5 * log((double)d) - log_factorial(d - 1) : 0.0;
}

/* ------------------------------------------------------------------------ */
/* automaton (src/Fsa.cpp restated)                                           */
/* ------------------------------------------------------------------------ */

typedef struct { char* str; int len; double logprob; int index; } emis_t;
typedef struct { int dst; double logprob; int index; } trans_t;
typedef struct {
    char* name;
    VEC(emis_t) em;
    VEC(trans_t) tr;
    int defined;
} state_t;

typedef struct {
    char* content;         /* owned, mutated by get_word */
    char *sep, *start_name, *end_name;
    VEC(state_t) st;
    int* htab; int64_t hcap;
    int start, end;
    int n_params;
    /* per parameter: owner state, kind (0 emission, 1 transition), label */
    int *p_state, *p_kind; const char** p_label;
} fsa_t;

static uint64_t fnv(const char* s) {
    uint64_t h = 14695981039346656037ULL;
    for (; *s; ++s) { h ^= (uint64_t)(unsigned char)*s; h *= 1099511628211ULL; }
    return h;
}

static int fsa_find(const fsa_t* f, const char* name) {
    if (!f->hcap) return -1;
    uint64_t m = (uint64_t)f->hcap - 1, h = fnv(name) & m;
    while (f->htab[h] >= 0) {
        if (strcmp(f->st.a[f->htab[h]].name, name) == 0) return f->htab[h];
        h = (h + 1) & m;
    }
    return -1;
}

static int fsa_get(fsa_t* f, const char* name) {
    int id = fsa_find(f, name);
    if (id >= 0) return id;
    if ((f->st.n + 1) * 2 > f->hcap) {
        int64_t nc = f->hcap ? f->hcap * 2 : 64;
        while ((f->st.n + 1) * 2 > nc) nc *= 2;
        free(f->htab);
        f->htab = xrealloc(NULL, sizeof(int) * (size_t)nc);
        for (int64_t i = 0; i < nc; ++i) f->htab[i] = -1;
        f->hcap = nc;
        for (int64_t i = 0; i < f->st.n; ++i) {
            uint64_t h = fnv(f->st.a[i].name) & (uint64_t)(nc - 1);
            while (f->htab[h] >= 0) h = (h + 1) & (uint64_t)(nc - 1);
            f->htab[h] = (int)i;
        }
    }
    state_t s; memset(&s, 0, sizeof s); s.name = (char*)name;
    VPUSH(f->st, s);
    id = (int)f->st.n - 1;
    uint64_t h = fnv(name) & (uint64_t)(f->hcap - 1);
    while (f->htab[h] >= 0) h = (h + 1) & (uint64_t)(f->hcap - 1);
    f->htab[h] = id;
    return id;
}

static void fsa_free(fsa_t* f) {
    for (int64_t i = 0; i < f->st.n; ++i) { VFREE(f->st.a[i].em); VFREE(f->st.a[i].tr); }
    VFREE(f->st); free(f->htab); free(f->content);
    free(f->p_state); free(f->p_kind); free(f->p_label);
    memset(f, 0, sizeof *f);
}

/* Fsa::Read + ReadOneState + AssignIndices (src/Fsa.cpp:73-238). */
static int fsa_parse(fsa_t* f, const char* text, char* err, int errlen) {
    memset(f, 0, sizeof *f);
    size_t len = strlen(text);
    f->content = xrealloc(NULL, len + 1);
    memcpy(f->content, text, len + 1);
    size_t lines = 0; for (size_t i = 0; i < len; ++i) lines += text[i] == '\n';
    size_t expected = ((lines > 3 ? lines : 3) - 3) / 2 + 1;      /* Fsa::AllocateStates */
    char* c = f->content;
    f->sep = get_word(&c, "\n").word;
    f->start_name = get_word(&c, "\n").word;
    f->end_name = get_word(&c, "\n").word;
    if (!*f->sep) f->sep = " ";
    if (starts_with(f->start_name, f->sep) || starts_with(f->end_name, f->sep)) {
        snprintf(err, errlen, "Invalid FSA format! Start or end state contains the separator!"); return OR_ERR;
    }
    if (strcmp(f->start_name, f->end_name) == 0) {
        snprintf(err, errlen, "Invalid FSA format! Start and end states should be different!"); return OR_ERR;
    }
    while (*c) {
        word_t r = get_word(&c, f->sep);
        char* this_state = r.word;
        if (!*this_state || starts_with(this_state, f->end_name)) { get_word(&c, "\n"); continue; }
        VEC(emis_t) em = {0}; VEC(trans_t) tr = {0};
        int is_start = strcmp(this_state, f->start_name) == 0;
        do {
            r = get_word(&c, f->sep);
            char* w = r.word;
            if (is_start && *w) { snprintf(err, errlen, "Invalid FSA format! Start state should emit empty string instead of \"%s\"!", w); VFREE(em); VFREE(tr); return OR_ERR; }
            for (int64_t k = 0; k < em.n; ++k) if (strcmp(em.a[k].str, w) == 0) {
                snprintf(err, errlen, "Invalid FSA format! Emission \"%s\" of state \"%s\" appears more than once!", w, this_state); VFREE(em); VFREE(tr); return OR_ERR; }
            r = get_word(&c, f->sep);
            emis_t e = { w, (int)strlen(w), atof(r.word), -1 };
            VPUSH(em, e);
        } while (r.term != '\n' && r.term != '\0');
        if (strcmp(this_state, get_word(&c, f->sep).word) != 0) {
            snprintf(err, errlen, "Invalid FSA format! You should enlist transitions of \"%s\" after emissions of the same state!", this_state); VFREE(em); VFREE(tr); return OR_ERR;
        }
        VEC(char*) tnames = {0}; VEC(double) tw = {0};
        do {
            r = get_word(&c, f->sep);
            char* w = r.word;
            for (int64_t k = 0; k < tnames.n; ++k) if (strcmp(tnames.a[k], w) == 0) {
                snprintf(err, errlen, "Invalid FSA format! Transition \"%s\" -> \"%s\" appears more than once!", this_state, w); VFREE(em); VFREE(tnames); VFREE(tw); return OR_ERR; }
            if (strcmp(w, f->start_name) == 0) {
                snprintf(err, errlen, "Invalid FSA format! \"%s\" connects to start state \"%s\"!", this_state, f->start_name); VFREE(em); VFREE(tnames); VFREE(tw); return OR_ERR; }
            VPUSH(tnames, w);
            r = get_word(&c, f->sep);
            VPUSH(tw, atof(r.word));
        } while (r.term != '\n' && r.term != '\0');
        for (int64_t k = 0; k < tnames.n; ++k) {
            trans_t t = { fsa_get(f, tnames.a[k]), tw.a[k], -1 };
            VPUSH(tr, t);
        }
        VFREE(tnames); VFREE(tw);
        int id = fsa_get(f, this_state);
        state_t* s = &f->st.a[id];
        VFREE(s->em); VFREE(s->tr);                      /* a re-definition replaces */
        s->em.a = em.a; s->em.n = em.n; s->em.cap = em.cap;
        s->tr.a = tr.a; s->tr.n = tr.n; s->tr.cap = tr.cap;
        s->defined = 1;
    }
    if ((size_t)f->st.n > expected) {
        snprintf(err, errlen, "Invalid FSA format! There are more states than rows in the automaton file! %lld > %zu", (long long)f->st.n, expected); return OR_ERR;
    }
    /* AssignIndices: a group with one member is unequivocal (-1) */
    int n = 0;
    for (int64_t i = 0; i < f->st.n; ++i) {
        state_t* s = &f->st.a[i];
        if (s->em.n > 1) for (int64_t k = 0; k < s->em.n; ++k) s->em.a[k].index = n++;
        if (s->tr.n > 1) for (int64_t k = 0; k < s->tr.n; ++k) s->tr.a[k].index = n++;
    }
    f->n_params = n;
    f->p_state = xrealloc(NULL, sizeof(int) * (size_t)(n + 1));
    f->p_kind = xrealloc(NULL, sizeof(int) * (size_t)(n + 1));
    f->p_label = xrealloc(NULL, sizeof(char*) * (size_t)(n + 1));
    for (int64_t i = 0; i < f->st.n; ++i) {
        state_t* s = &f->st.a[i];
        for (int64_t k = 0; k < s->em.n; ++k) if (s->em.a[k].index >= 0) {
            int j = s->em.a[k].index; f->p_state[j] = (int)i; f->p_kind[j] = 0; f->p_label[j] = s->em.a[k].str; }
        for (int64_t k = 0; k < s->tr.n; ++k) if (s->tr.a[k].index >= 0) {
            int j = s->tr.a[k].index; f->p_state[j] = (int)i; f->p_kind[j] = 1; f->p_label[j] = f->st.a[s->tr.a[k].dst].name; }
    }
    f->start = fsa_find(f, f->start_name);
    f->end = fsa_find(f, f->end_name);
    if (f->start < 0) { snprintf(err, errlen, "start state \"%s\" is not defined", f->start_name); return OR_ERR; }
    return OR_OK;
}

/* ------------------------------------------------------------------------ */
/* corpus (src/Corpus.cpp:9-61 restated)                                      */
/* ------------------------------------------------------------------------ */

typedef struct {
    char* content;
    VEC(char*) words;   /* owned copies */
    VEC(int) lens;
    VEC(double) w;
} corpus_t;

static void corpus_free(corpus_t* c) {
    for (int64_t i = 0; i < c->words.n; ++i) free(c->words.a[i]);
    VFREE(c->words); VFREE(c->lens); VFREE(c->w); free(c->content);
    memset(c, 0, sizeof *c);
}

/* duplicate detection: open addressing over word strings */
typedef struct { int64_t* t; int64_t cap; } wset_t;
static int wset_insert(wset_t* s, char** words, int64_t id) {
    if (!s->cap) return 1;
    uint64_t m = (uint64_t)s->cap - 1, h = fnv(words[id]) & m;
    while (s->t[h] >= 0) { if (strcmp(words[s->t[h]], words[id]) == 0) return 0; h = (h + 1) & m; }
    s->t[h] = id; return 1;
}

static int corpus_finish(corpus_t* cp, char* err, int errlen) {
    for (int64_t i = 0; i < cp->w.n; ++i) {
        double v = cp->w.a[i];
        if (!(isnormal(v)) || v < 0) { snprintf(err, errlen, "\"%s\" has probability %g!", cp->words.a[i], v); return OR_ERR; }
    }
    return OR_OK;
}

static int corpus_parse(corpus_t* cp, const char* text, char* err, int errlen) {
    memset(cp, 0, sizeof *cp);
    size_t len = strlen(text);
    cp->content = xrealloc(NULL, len + 1);
    memcpy(cp->content, text, len + 1);
    char* c = cp->content;
    word_t r = get_word(&c, "\n");
    const char* sep = *r.word ? r.word : " ";
    VEC(char) word = {0};
    wset_t set = {0};
    size_t lines = 1; for (size_t i = 0; i < len; ++i) lines += text[i] == '\n';
    set.cap = 64; while ((size_t)set.cap < 2 * lines) set.cap *= 2;
    set.t = xrealloc(NULL, sizeof(int64_t) * (size_t)set.cap);
    for (int64_t i = 0; i < set.cap; ++i) set.t[i] = -1;
    while (r.term != '\0') {
        word.n = 0;
        int empty = 1;
        do {
            r = get_word(&c, sep);
            if (r.term == '\n' || r.term == '\0') {
                if (!empty) {
                    VPUSH(word, '\0');
                    char* copy = xrealloc(NULL, (size_t)word.n);
                    memcpy(copy, word.a, (size_t)word.n);
                    VPUSH(cp->words, copy);
                    if (!wset_insert(&set, cp->words.a, cp->words.n - 1)) {
                        snprintf(err, errlen, "\"%s\" is duplicate!", copy); VFREE(word); free(set.t); return OR_ERR;
                    }
                    VPUSH(cp->lens, (int)(word.n - 1));
                    VPUSH(cp->w, atof(r.word));
                }
                break;
            }
            empty = 0;
            for (const char* p = r.word; *p; ++p) VPUSH(word, *p);
        } while (r.term);
    }
    VFREE(word); free(set.t);
    return corpus_finish(cp, err, errlen);
}

/* ------------------------------------------------------------------------ */
/* learner state                                                              */
/* ------------------------------------------------------------------------ */

typedef struct { int idx; double cnt; } pc_t;

typedef struct {
    fsa_t fsa;
    corpus_t corpus;
    int mode;                 /* 0 ENUM, 1 TRELLIS */
    int n_full;               /* Fsa params */
    int n, k;                 /* trimmed params, constraints */
    int* trimmed;             /* [n_full]: >=0 trimmed index, -1 fixed 0, -2 unused */
    int* Ccol;                /* [n] constraint of trimmed param */
    double* x;                /* [n] */
    double model_volume, common_support, plogp, aux_hessian, kl;
    int64_t aux_params;
    /* recognized strings */
    int64_t S;
    int64_t* str_of;          /* [S] corpus index */
    double* p;                /* [S] */
    double* logq;             /* [S] */
    int64_t* path_count;      /* [corpus size] (ENUM: exact, TRELLIS: count semiring) */
    /* ENUM matrices */
    int64_t n_paths;
    int64_t *Prow, *Mrow;     /* Prow [n_paths+1]; Mrow [S+1] */
    int* Pcol; double* Pdata;
    double* rpp;              /* [n_paths] */
    double* grad_aux;
    int grad_aux_init;
    int unique;
    /* QN state */
    double *grad, *expx, *lambda, *g, *rhs, *aux;
    double grad_error, lambda_min, g_min, g_max;
    int exp_lambda;
    int64_t max_paths;
    int threads;              /* OpenMP threads of the per-iteration passes (cpu_baseline); 1 = serial */
} learner_t;

static double get_weight(const learner_t* L, int j) {             /* src/Learner.cpp:427-436 */
    int t = L->trimmed[j];
    if (t == -2) return -INFINITY;
    if (t == -1) return 0.0;
    return L->x[t];
}

/* ---- BuildConstraints (src/Learner.cpp:221-265) ---- */

static void build_constraints(learner_t* L, double* x_full, int* Ccol_full) {
    int k = 0, pos = 0;
    L->model_volume = 0;
    for (int64_t i = 0; i < L->fsa.st.n; ++i) {
        state_t* s = &L->fsa.st.a[i];
        if (s->em.n > 1) {
            for (int64_t e = 0; e < s->em.n; ++e) { x_full[s->em.a[e].index] = s->em.a[e].logprob; Ccol_full[pos++] = k; }
            ++k; L->model_volume += log_simplex_volume((size_t)s->em.n);
        }
        if (s->tr.n > 1) {
            for (int64_t t = 0; t < s->tr.n; ++t) { x_full[s->tr.a[t].index] = s->tr.a[t].logprob; Ccol_full[pos++] = k; }
            ++k; L->model_volume += log_simplex_volume((size_t)s->tr.n);
        }
    }
}

/* ---- Trim (src/Learner.cpp:350-425) ---- */
static void trim(learner_t* L, const double* x_full, const int* Ccol_full) {
    int n = L->n_full, c = -1, nnz_in_c = -1;
    int* tw = L->trimmed;
    for (int i = 0; i < n; ++i) {
        int this_c = Ccol_full[i];
        if (this_c != c) { c = this_c; if (nnz_in_c >= 0) tw[nnz_in_c] = -1; nnz_in_c = -1; }
        if (tw[i] >= 0) nnz_in_c = (nnz_in_c == -1) ? i : -2;
    }
    if (nnz_in_c >= 0) tw[nnz_in_c] = -1;
    int good = 0, good_c = -1; c = -1;
    L->x = xrealloc(NULL, sizeof(double) * (size_t)(n + 1));
    L->Ccol = xrealloc(NULL, sizeof(int) * (size_t)(n + 1));
    for (int i = 0; i < n; ++i) {
        if (tw[i] == 0) {
            tw[i] = good++;
            L->x[tw[i]] = x_full[i];
            if (c < Ccol_full[i]) { ++good_c; c = Ccol_full[i]; }
            L->Ccol[tw[i]] = good_c;
        }
    }
    L->n = good;
    L->k = good ? L->Ccol[good - 1] + 1 : 0;
}

/* ---- BFS path enumeration (inc/Recognize.h:62-96, no clock cap) ---- */
typedef struct { int word_off; int state; int64_t hist_off; int hist_len; } qitem_t;

typedef struct {
    VEC(qitem_t) q;
    VEC(pc_t) hist;        /* arena of histories */
} bfs_ws_t;

static int64_t sorted_insert(pc_t* h, int len, int idx) {   /* returns new len; h has room for len+1 */
    int lo = 0, hi = len;
    while (lo < hi) { int mid = (lo + hi) / 2; if (h[mid].idx < idx) lo = mid + 1; else hi = mid; }
    if (lo < len && h[lo].idx == idx) { h[lo].cnt += 1; return len; }
    memmove(h + lo + 1, h + lo, sizeof(pc_t) * (size_t)(len - lo));
    h[lo].idx = idx; h[lo].cnt = 1;
    return len + 1;
}

/* Appends every accepting path's (param,count) list via the callback arrays.
 * Returns number of paths, or -1 if more than max_paths. */
typedef struct { VEC(int64_t) prow; VEC(int) pcol; VEC(double) pdata; } paths_out_t;

static int64_t bfs_paths(const fsa_t* f, const char* word, bfs_ws_t* ws, paths_out_t* out, int64_t max_paths) {
    ws->q.n = 0; ws->hist.n = 0;
    qitem_t q0 = { 0, f->start, 0, 0 };
    VPUSH(ws->q, q0);
    int64_t head = 0, npaths = 0;
    while (head < ws->q.n) {
        qitem_t w = ws->q.a[head++];
        const char* cur = word + w.word_off;
        const state_t* s = &f->st.a[w.state];
        for (int64_t t = 0; t < s->tr.n; ++t) {
            const trans_t* tr = &s->tr.a[t];
            if (tr->dst == f->end) {
                if (cur[0] == '\0') {
                    /* accepting path: history + transition param */
                    int64_t base = ws->hist.n;
                    for (int i = 0; i < w.hist_len + 1; ++i) { pc_t z = {0, 0}; VPUSH(ws->hist, z); }
                    pc_t* h = ws->hist.a + base;
                    memcpy(h, ws->hist.a + w.hist_off, sizeof(pc_t) * (size_t)w.hist_len);
                    int len = w.hist_len;
                    if (tr->index >= 0) len = (int)sorted_insert(h, len, tr->index);
                    VPUSH(out->prow, out->pcol.n);
                    for (int i = 0; i < len; ++i) { VPUSH(out->pcol, h[i].idx); VPUSH(out->pdata, h[i].cnt); }
                    ws->hist.n = base;
                    if (++npaths > max_paths) return -1;
                }
                continue;
            }
            const state_t* ns = &f->st.a[tr->dst];
            for (int64_t e = 0; e < ns->em.n; ++e) {
                const emis_t* em = &ns->em.a[e];
                if (strncmp(cur, em->str, (size_t)em->len) == 0) {
                    int64_t base = ws->hist.n;
                    for (int i = 0; i < w.hist_len + 2; ++i) { pc_t z = {0, 0}; VPUSH(ws->hist, z); }
                    pc_t* h = ws->hist.a + base;
                    memcpy(h, ws->hist.a + w.hist_off, sizeof(pc_t) * (size_t)w.hist_len);
                    int len = w.hist_len;
                    if (tr->index >= 0) len = (int)sorted_insert(h, len, tr->index);
                    if (em->index >= 0) len = (int)sorted_insert(h, len, em->index);
                    qitem_t nq = { w.word_off + em->len, tr->dst, base, len };
                    VPUSH(ws->q, nq);
                    if (ws->q.n > 64 * max_paths + 1000000) return -1;  /* epsilon blow-up guard */
                }
            }
        }
    }
    return npaths;
}

/* ---- trellis forward/backward (dense, float64) ---- */
typedef struct {
    int N;
    int* topo;          /* states in topological order of epsilon edges */
    double* alpha;      /* [(L+1) * N] */
    double* beta;
    int cap_L;
    int* eb;            /* [N * 256] single-byte emission of state s with byte b, or -1 */
    int* oth_ptr;       /* [N + 1] the other (epsilon / multi-byte) emissions of s ... */
    int* oth;           /* ... as indices into s's emission list */
} trellis_ws_t;

static int eps_topo(const fsa_t* f, int* order, char* err, int errlen) {
    int N = (int)f->st.n;
    int* indeg = calloc((size_t)N, sizeof(int));
    for (int s = 0; s < N; ++s) {
        const state_t* st = &f->st.a[s];
        for (int64_t t = 0; t < st->tr.n; ++t) {
            int d = st->tr.a[t].dst; if (d == f->end) continue;
            const state_t* ds = &f->st.a[d];
            for (int64_t e = 0; e < ds->em.n; ++e) if (ds->em.a[e].len == 0) { indeg[d]++; break; }
        }
    }
    int head = 0, tail = 0;
    for (int s = 0; s < N; ++s) if (!indeg[s]) order[tail++] = s;
    while (head < tail) {
        int s = order[head++];
        const state_t* st = &f->st.a[s];
        for (int64_t t = 0; t < st->tr.n; ++t) {
            int d = st->tr.a[t].dst; if (d == f->end) continue;
            const state_t* ds = &f->st.a[d];
            int has_eps = 0;
            for (int64_t e = 0; e < ds->em.n; ++e) if (ds->em.a[e].len == 0) has_eps = 1;
            if (has_eps && --indeg[d] == 0) order[tail++] = d;
        }
    }
    free(indeg);
    if (tail != N) { snprintf(err, errlen, "epsilon cycle in automaton"); return OR_ERR; }
    return OR_OK;
}

/* emission lookup: every emission of state s is either the single byte b
 * (eb[s*256+b]) or in s's "other" list; the matching rule is unchanged
 * (inc/Recognize.h:52: the emission must be a prefix of the rest of the word) */
static void trellis_tables(const fsa_t* f, trellis_ws_t* ws) {
    if (ws->eb) return;
    int N = ws->N;
    ws->eb = xrealloc(NULL, sizeof(int) * (size_t)N * 256);
    ws->oth_ptr = xrealloc(NULL, sizeof(int) * (size_t)(N + 1));
    for (size_t k = 0; k < (size_t)N * 256; ++k) ws->eb[k] = -1;
    int n_oth = 0;
    for (int s = 0; s < N; ++s)
        for (int64_t e = 0; e < f->st.a[s].em.n; ++e) if (f->st.a[s].em.a[e].len != 1) ++n_oth;
    ws->oth = xrealloc(NULL, sizeof(int) * (size_t)(n_oth + 1));
    n_oth = 0;
    for (int s = 0; s < N; ++s) {
        ws->oth_ptr[s] = n_oth;
        const state_t* st = &f->st.a[s];
        for (int64_t e = 0; e < st->em.n; ++e) {
            const emis_t* em = &st->em.a[e];
            if (em->len == 1) ws->eb[(size_t)s * 256 + (unsigned char)em->str[0]] = (int)e;
            else ws->oth[n_oth++] = (int)e;
        }
    }
    ws->oth_ptr[N] = n_oth;
}

static void trellis_free(trellis_ws_t* ws) {
    free(ws->topo); free(ws->alpha); free(ws->beta); free(ws->eb); free(ws->oth_ptr); free(ws->oth);
}

static void trellis_alloc(trellis_ws_t* ws, int L) {
    if (L + 1 > ws->cap_L) {
        ws->cap_L = L + 1;
        free(ws->alpha); free(ws->beta);
        ws->alpha = xrealloc(NULL, sizeof(double) * (size_t)ws->cap_L * (size_t)ws->N);
        ws->beta = xrealloc(NULL, sizeof(double) * (size_t)ws->cap_L * (size_t)ws->N);
    }
}

/* Calls BODY for every emission em (index EI in state D's list) of state D
 * that matches the word at position i. */
#define FOR_MATCHING_EMISSIONS(D, EI, BODY)                                          \
    do {                                                                             \
        const state_t* ds_ = &f->st.a[(D)];                                          \
        if (i < L) {                                                                 \
            int EI = ws->eb[(size_t)(D) * 256 + (unsigned char)word[i]];              \
            if (EI >= 0) { BODY }                                                    \
        }                                                                            \
        for (int k_ = ws->oth_ptr[(D)]; k_ < ws->oth_ptr[(D) + 1]; ++k_) {           \
            int EI = ws->oth[k_];                                                    \
            const emis_t* e_ = &ds_->em.a[EI];                                       \
            if (i + e_->len > L) continue;                                           \
            if (memcmp(word + i, e_->str, (size_t)e_->len) != 0) continue;           \
            { BODY }                                                                 \
        }                                                                            \
    } while (0)

/* Forward-backward on one string.  Returns q (not log).  ew[j] = exp(w_j)
 * for Fsa parameter j; NULL = all weights 1 (counting semiring: q = path
 * count).  If counts != NULL, adds scale * E[count_j] into counts[j]. */
static double trellis_string(const fsa_t* f, trellis_ws_t* ws, const char* word, int L,
                             const double* ew, double* counts, double scale,
                             unsigned char* used) {
    int N = ws->N;
    trellis_tables(f, ws);
    trellis_alloc(ws, L);
    double* A = ws->alpha; double* B = ws->beta;
    memset(A, 0, sizeof(double) * (size_t)(L + 1) * (size_t)N);
    memset(B, 0, sizeof(double) * (size_t)(L + 1) * (size_t)N);
#define EW(j) ((j) < 0 || !ew ? 1.0 : ew[(j)])
    A[f->start] = 1.0;
    for (int i = 0; i <= L; ++i) {
        double* Ai = A + (size_t)i * N;
        for (int oi = 0; oi < N; ++oi) {
            int s = ws->topo[oi];
            double a = Ai[s];
            if (a == 0.0) continue;
            const state_t* st = &f->st.a[s];
            for (int64_t t = 0; t < st->tr.n; ++t) {
                const trans_t* tr = &st->tr.a[t];
                if (tr->dst == f->end) continue;
                const double wt = EW(tr->index);
                FOR_MATCHING_EMISSIONS(tr->dst, ei, {
                    const emis_t* em = &ds_->em.a[ei];
                    A[(size_t)(i + em->len) * N + tr->dst] += a * (wt * EW(em->index));
                });
            }
        }
    }
    double q = 0;
    double* AL = A + (size_t)L * N;
    double* BL = B + (size_t)L * N;
    for (int s = 0; s < N; ++s) {
        const state_t* st = &f->st.a[s];
        for (int64_t t = 0; t < st->tr.n; ++t) if (st->tr.a[t].dst == f->end) {
            double we = EW(st->tr.a[t].index);
            BL[s] += we;
            q += AL[s] * we;
        }
    }
    for (int i = L; i >= 0; --i) {
        double* Bi = B + (size_t)i * N;
        for (int oi = N - 1; oi >= 0; --oi) {
            int s = ws->topo[oi];
            const state_t* st = &f->st.a[s];
            double acc = 0;
            for (int64_t t = 0; t < st->tr.n; ++t) {
                const trans_t* tr = &st->tr.a[t];
                if (tr->dst == f->end) continue;
                const double wt = EW(tr->index);
                FOR_MATCHING_EMISSIONS(tr->dst, ei, {
                    const emis_t* em = &ds_->em.a[ei];
                    acc += (wt * EW(em->index)) * B[(size_t)(i + em->len) * N + tr->dst];
                });
            }
            Bi[s] += acc;
        }
    }
    if (q > 0 && (counts || used)) {
        for (int i = 0; i <= L; ++i) {
            double* Ai = A + (size_t)i * N;
            for (int s = 0; s < N; ++s) {
                double a = Ai[s];
                if (a == 0.0) continue;
                const state_t* st = &f->st.a[s];
                for (int64_t t = 0; t < st->tr.n; ++t) {
                    const trans_t* tr = &st->tr.a[t];
                    if (tr->dst == f->end) {
                        if (i != L) continue;
                        double xi = a * EW(tr->index) / q;
                        if (xi > 0 && tr->index >= 0) {
                            if (counts) counts[tr->index] += scale * xi;
                            if (used) used[tr->index] = 1;
                        }
                        continue;
                    }
                    const double wt = EW(tr->index);
                    FOR_MATCHING_EMISSIONS(tr->dst, ei, {
                        const emis_t* em = &ds_->em.a[ei];
                        double b = B[(size_t)(i + em->len) * N + tr->dst];
                        double xi = a * (wt * EW(em->index)) * b / q;
                        if (xi > 0) {
                            if (tr->index >= 0) { if (counts) counts[tr->index] += scale * xi; if (used) used[tr->index] = 1; }
                            if (em->index >= 0) { if (counts) counts[em->index] += scale * xi; if (used) used[em->index] = 1; }
                        }
                    });
                }
            }
        }
    }
#undef EW
    return q;
}

/* exp of the weights in GetWeight form, by Fsa parameter */
static double* exp_weights(const learner_t* L, const double* w_full) {
    double* ew = xrealloc(NULL, sizeof(double) * (size_t)(L->n_full + 1));
    for (int j = 0; j < L->n_full; ++j) ew[j] = exp(w_full ? w_full[j] : get_weight(L, j));
    return ew;
}


/* ------------------------------------------------------------------------ */
/* public API                                                                 */
/* ------------------------------------------------------------------------ */

typedef struct {
    int64_t n_corpus, n_strings, n_paths;
    int n_full, n_params, n_constraints, unique;
    int64_t aux_params;
    double plogp, common_support, model_volume, aux_hessian;
    int n_states;
} oracle_info_t;

void oracle_free(learner_t* L) {
    if (!L) return;
    fsa_free(&L->fsa); corpus_free(&L->corpus);
    free(L->trimmed); free(L->Ccol); free(L->x); free(L->str_of); free(L->p); free(L->logq);
    free(L->path_count); free(L->Prow); free(L->Mrow); free(L->Pcol); free(L->Pdata); free(L->rpp);
    free(L->grad_aux); free(L->grad); free(L->expx); free(L->lambda); free(L->g); free(L->rhs); free(L->aux);
    free(L);
}

static learner_t* build_common(learner_t* L, int mode, int64_t max_paths, char* err, int errlen) {
    L->mode = mode;
    L->max_paths = max_paths > 0 ? max_paths : 1000000;
    fsa_t* f = &L->fsa;
    corpus_t* cp = &L->corpus;
    /* Corpus::Renormalize (src/Corpus.cpp:67-72), done by main before BuildFrom */
    double sum = 0; for (int64_t i = 0; i < cp->w.n; ++i) sum += cp->w.a[i];
    for (int64_t i = 0; i < cp->w.n; ++i) cp->w.a[i] /= sum;

    int nf = f->n_params;
    L->n_full = nf;
    double* x_full = xrealloc(NULL, sizeof(double) * (size_t)(nf + 1));
    int* Ccol_full = xrealloc(NULL, sizeof(int) * (size_t)(nf + 1));
    build_constraints(L, x_full, Ccol_full);
    L->trimmed = xrealloc(NULL, sizeof(int) * (size_t)(nf + 1));
    for (int j = 0; j < nf; ++j) L->trimmed[j] = -2;

    int64_t NC = cp->words.n;
    L->path_count = calloc((size_t)(NC + 1), sizeof(int64_t));
    L->str_of = xrealloc(NULL, sizeof(int64_t) * (size_t)(NC + 1));
    L->p = xrealloc(NULL, sizeof(double) * (size_t)(NC + 1));
    L->common_support = 0; L->aux_params = 0; L->aux_hessian = 0;
    int64_t S = 0;
    if (f->end < 0) {
        /* no transition reaches the end state: nothing is recognized */
        for (int64_t i = 0; i < NC; ++i) { L->aux_params++; L->aux_hessian -= log(cp->w.a[i]); }
    } else if (mode == 0) {
        /* BuildPaths (src/Learner.cpp:276-348): strings enumerated in chunks
         * on OpenMP threads, each into its own arrays, then concatenated in
         * string order -- the same P, M and numbering as one thread */
        int nt = omp_get_max_threads();
        const char* bt = getenv("ORACLE_BUILD_THREADS");   /* (tests: force a split) */
        if (bt && atoi(bt) > 0) nt = atoi(bt);
        else if (NC < 4096) nt = 1;
        if (nt < 1) nt = 1;
        paths_out_t* po_t = calloc((size_t)nt, sizeof(paths_out_t));
        int64_t* np_of = calloc((size_t)(NC + 1), sizeof(int64_t));
        int failed = 0;
        int64_t fail_at = -1;
#pragma omp parallel num_threads(nt) if (nt > 1)
        {
            const int t = omp_get_thread_num();
            const int64_t b = NC * t / nt, e = NC * (t + 1) / nt;
            bfs_ws_t ws = {0};
            for (int64_t i = b; i < e && !failed; ++i) {
                int64_t np = bfs_paths(f, cp->words.a[i], &ws, &po_t[t], L->max_paths);
                np_of[i] = np;
                if (np < 0) {
#pragma omp critical
                    { if (!failed || i < fail_at) fail_at = i; failed = 1; }
                }
            }
            VFREE(ws.q); VFREE(ws.hist);
        }
        if (failed) {
            snprintf(err, errlen, "string %lld exceeds max_paths", (long long)fail_at);
            for (int t = 0; t < nt; ++t) { VFREE(po_t[t].prow); VFREE(po_t[t].pcol); VFREE(po_t[t].pdata); }
            free(po_t); free(np_of); free(x_full); free(Ccol_full); return NULL;
        }
        paths_out_t po = {0};
        VEC(int64_t) mrow = {0};
        int64_t tot_rows = 0, tot_nz = 0;
        for (int t = 0; t < nt; ++t) { tot_rows += po_t[t].prow.n; tot_nz += po_t[t].pcol.n; }
        po.prow.a = xrealloc(NULL, sizeof(int64_t) * (size_t)(tot_rows + 1)); po.prow.cap = tot_rows + 1;
        po.pcol.a = xrealloc(NULL, sizeof(int) * (size_t)(tot_nz + 1)); po.pcol.cap = tot_nz + 1;
        po.pdata.a = xrealloc(NULL, sizeof(double) * (size_t)(tot_nz + 1)); po.pdata.cap = tot_nz + 1;
        for (int t = 0; t < nt; ++t) {
            const int64_t row0 = po.prow.n, nz0 = po.pcol.n;
            for (int64_t r = 0; r < po_t[t].prow.n; ++r) po.prow.a[row0 + r] = po_t[t].prow.a[r] + nz0;
            po.prow.n += po_t[t].prow.n;
            memcpy(po.pcol.a + nz0, po_t[t].pcol.a, sizeof(int) * (size_t)po_t[t].pcol.n);
            memcpy(po.pdata.a + nz0, po_t[t].pdata.a, sizeof(double) * (size_t)po_t[t].pdata.n);
            po.pcol.n += po_t[t].pcol.n;
            po.pdata.n += po_t[t].pdata.n;
            VFREE(po_t[t].prow); VFREE(po_t[t].pcol); VFREE(po_t[t].pdata);
        }
        free(po_t);
        int64_t row = 0;
        for (int64_t i = 0; i < NC; ++i) {
            const int64_t np = np_of[i];
            L->path_count[i] = np;
            if (np > 0) {
                VPUSH(mrow, row);
                L->common_support += cp->w.a[i];
                L->str_of[S] = i; L->p[S] = cp->w.a[i]; ++S;
                const int64_t k_end = row + np < po.prow.n ? po.prow.a[row + np] : po.pcol.n;
                for (int64_t k = po.prow.a[row]; k < k_end; ++k) L->trimmed[po.pcol.a[k]] = 0;
                row += np;
            } else {
                L->aux_params++; L->aux_hessian -= log(cp->w.a[i]);
            }
        }
        free(np_of);
        VPUSH(mrow, po.prow.n);
        VPUSH(po.prow, po.pcol.n);
        L->n_paths = po.prow.n - 1;
        L->Prow = po.prow.a; L->Pcol = po.pcol.a; L->Pdata = po.pdata.a;
        L->Mrow = mrow.a;
    } else {
        trellis_ws_t ws = {0};
        ws.N = (int)f->st.n;
        ws.topo = xrealloc(NULL, sizeof(int) * (size_t)(ws.N + 1));
        if (eps_topo(f, ws.topo, err, errlen) != OR_OK) { free(ws.topo); free(x_full); free(Ccol_full); return NULL; }
        unsigned char* used = calloc((size_t)(nf + 1), 1);
        L->n_paths = 0;
        for (int64_t i = 0; i < NC; ++i) {
            double q = trellis_string(f, &ws, cp->words.a[i], cp->lens.a[i], NULL, NULL, 0, used);
            L->path_count[i] = (int64_t)q;
            if (q > 0) {
                L->common_support += cp->w.a[i];
                L->str_of[S] = i; L->p[S] = cp->w.a[i]; ++S;
                L->n_paths += (int64_t)q;
            } else { L->aux_params++; L->aux_hessian -= log(cp->w.a[i]); }
        }
        for (int j = 0; j < nf; ++j) if (used[j]) L->trimmed[j] = 0;
        free(used); trellis_free(&ws);
    }
    L->S = S;
    trim(L, x_full, Ccol_full);
    if (mode == 0) {
        /* Trim also renumbers P columns and drops trimmed entries */
        int64_t w = 0, start = L->Prow[0];
        for (int64_t r = 0; r < L->n_paths; ++r) {
            int64_t end = L->Prow[r + 1];
            for (int64_t k = start; k < end; ++k) {
                int t = L->trimmed[L->Pcol[k]];
                if (t >= 0) { L->Pcol[w] = t; L->Pdata[w] = L->Pdata[k]; ++w; }
            }
            start = end; L->Prow[r + 1] = w;
        }
        L->unique = (L->n_paths == S);
    } else {
        L->unique = (L->n_paths == S);
    }
    free(x_full); free(Ccol_full);
    /* Finalize (src/Learner.cpp:466-488) */
    L->plogp = 0;
    for (int64_t s = 0; s < S; ++s) L->plogp += L->p[s] * log(L->p[s]);
    L->logq = xrealloc(NULL, sizeof(double) * (size_t)(S + 1));
    if (mode == 0) L->rpp = xrealloc(NULL, sizeof(double) * (size_t)(L->n_paths + 1));
    int n = L->n, k = L->k;
    L->grad = calloc((size_t)n + 1, sizeof(double));
    L->expx = calloc((size_t)n + 1, sizeof(double));
    L->rhs = calloc((size_t)n + 1, sizeof(double));
    L->aux = calloc((size_t)n + 1, sizeof(double));
    L->lambda = xrealloc(NULL, sizeof(double) * (size_t)(k + 1));
    for (int c = 0; c < k; ++c) L->lambda[c] = 1.0;
    L->g = calloc((size_t)k + 1, sizeof(double));
    return L;
}

learner_t* oracle_build_text(const char* wfsa_text, const char* corpus_text, int mode,
                             int64_t max_paths, char* err, int errlen) {
    learner_t* L = calloc(1, sizeof(learner_t));
    if (fsa_parse(&L->fsa, wfsa_text, err, errlen) != OR_OK) { oracle_free(L); return NULL; }
    if (corpus_parse(&L->corpus, corpus_text, err, errlen) != OR_OK) { oracle_free(L); return NULL; }
    if (!build_common(L, mode, max_paths, err, errlen)) { oracle_free(L); return NULL; }
    return L;
}

/* corpus given as packed bytes + offsets + raw weights (renormalized here) */
learner_t* oracle_build_arrays(const char* wfsa_text, const unsigned char* sym, const int64_t* off,
                               const double* weights, int64_t n_strings, int mode, int64_t max_paths,
                               char* err, int errlen) {
    learner_t* L = calloc(1, sizeof(learner_t));
    if (fsa_parse(&L->fsa, wfsa_text, err, errlen) != OR_OK) { oracle_free(L); return NULL; }
    corpus_t* cp = &L->corpus;
    for (int64_t i = 0; i < n_strings; ++i) {
        int64_t len = off[i + 1] - off[i];
        char* w = xrealloc(NULL, (size_t)len + 1);
        memcpy(w, sym + off[i], (size_t)len); w[len] = '\0';
        VPUSH(cp->words, w); VPUSH(cp->lens, (int)len); VPUSH(cp->w, weights[i]);
    }
    if (corpus_finish(cp, err, errlen) != OR_OK) { oracle_free(L); return NULL; }
    if (!build_common(L, mode, max_paths, err, errlen)) { oracle_free(L); return NULL; }
    return L;
}

void oracle_get_info(const learner_t* L, oracle_info_t* o) {
    o->n_corpus = L->corpus.words.n; o->n_strings = L->S; o->n_paths = L->n_paths;
    o->n_full = L->n_full; o->n_params = L->n; o->n_constraints = L->k; o->unique = L->unique;
    o->aux_params = L->aux_params; o->plogp = L->plogp; o->common_support = L->common_support;
    o->model_volume = L->model_volume; o->aux_hessian = L->aux_hessian;
    o->n_states = (int)L->fsa.st.n;
}

/* name of trimmed parameter t: state, kind (0 emission / 1 transition), label */
int oracle_param_name(const learner_t* L, int t, const char** state, int* kind, const char** label) {
    for (int j = 0; j < L->n_full; ++j) if (L->trimmed[j] == t) {
        *state = L->fsa.st.a[L->fsa.p_state[j]].name; *kind = L->fsa.p_kind[j]; *label = L->fsa.p_label[j];
        return OR_OK;
    }
    return OR_ERR;
}

void oracle_path_counts(const learner_t* L, int64_t* out) {
    memcpy(out, L->path_count, sizeof(int64_t) * (size_t)L->corpus.words.n);
}

void oracle_get_x(const learner_t* L, double* x) { memcpy(x, L->x, sizeof(double) * (size_t)L->n); }
void oracle_set_x(learner_t* L, const double* x) { memcpy(L->x, x, sizeof(double) * (size_t)L->n); }
void oracle_get_logq(const learner_t* L, double* out) { memcpy(out, L->logq, sizeof(double) * (size_t)L->S); }
void oracle_get_p(const learner_t* L, double* out) { memcpy(out, L->p, sizeof(double) * (size_t)L->S); }
void oracle_get_grad(const learner_t* L, double* out) { memcpy(out, L->grad, sizeof(double) * (size_t)L->n); }
double oracle_kl(const learner_t* L) { return L->kl; }

/* ComputeModeledProbs (src/Learner.cpp:515-547) */
static void modeled_probs(learner_t* L) {
    int64_t S = L->S;
    if (L->mode == 0) {
        const int nt = L->threads > 1 ? L->threads : 1;
        (void)nt;
        if (L->unique) {
#pragma omp parallel for num_threads(nt) if (nt > 1) schedule(static)
            for (int64_t s = 0; s < S; ++s) {          /* logq = P.x (row s = path s) */
                double a = 0;
                for (int64_t k = L->Prow[s]; k < L->Prow[s + 1]; ++k) a += L->Pdata[k] * L->x[L->Pcol[k]];
                L->logq[s] = a;
            }
        } else {
#pragma omp parallel for num_threads(nt) if (nt > 1) schedule(static)
            for (int64_t r = 0; r < L->n_paths; ++r) {
                double a = 0;
                for (int64_t k = L->Prow[r]; k < L->Prow[r + 1]; ++k) a += L->Pdata[k] * L->x[L->Pcol[k]];
                L->rpp[r] = exp(a);
            }
#pragma omp parallel for num_threads(nt) if (nt > 1) schedule(static)
            for (int64_t s = 0; s < S; ++s) {
                double q = 0;
                for (int64_t r = L->Mrow[s]; r < L->Mrow[s + 1]; ++r) q += L->rpp[r];
                L->logq[s] = log(q);
                for (int64_t r = L->Mrow[s]; r < L->Mrow[s + 1]; ++r) L->rpp[r] /= q;
            }
        }
    } else {
        trellis_ws_t ws = {0};
        ws.N = (int)L->fsa.st.n;
        ws.topo = xrealloc(NULL, sizeof(int) * (size_t)(ws.N + 1));
        char err[64];
        eps_topo(&L->fsa, ws.topo, err, 64);
        double* counts = calloc((size_t)L->n_full + 1, sizeof(double));
        double* ew = exp_weights(L, NULL);
        for (int64_t s = 0; s < S; ++s) {
            int64_t i = L->str_of[s];
            double q = trellis_string(&L->fsa, &ws, L->corpus.words.a[i], L->corpus.lens.a[i],
                                      ew, counts, -L->p[s], NULL);
            L->logq[s] = log(q);
        }
        for (int j = 0; j < L->n_full; ++j) if (L->trimmed[j] >= 0) L->grad[L->trimmed[j]] = counts[j];
        free(ew); free(counts); trellis_free(&ws);
    }
}

/* ComputeObjective (src/Learner.cpp:549-553) */
static void objective(learner_t* L) {
    double d = 0; for (int64_t s = 0; s < L->S; ++s) d += L->p[s] * L->logq[s];
    L->kl = L->plogp - d;
}

/* QuasiNewtonLearner::ComputeGrad (src/QuasiNewtonLearner.cpp:93-125) */
static void compute_grad(learner_t* L) {
    int n = L->n;
    if (L->mode == 1) { modeled_probs(L); return; }
    if (!L->grad_aux_init) {
        L->grad_aux_init = 1;
        if (L->unique) {
            L->grad_aux = calloc((size_t)n + 1, sizeof(double));
            for (int64_t s = 0; s < L->S; ++s)
                for (int64_t k = L->Prow[s]; k < L->Prow[s + 1]; ++k) L->grad_aux[L->Pcol[k]] -= L->Pdata[k] * L->p[s];
        } else {
            L->grad_aux = calloc((size_t)L->n_paths + 1, sizeof(double));
            for (int64_t s = 0; s < L->S; ++s)
                for (int64_t r = L->Mrow[s]; r < L->Mrow[s + 1]; ++r) L->grad_aux[r] = -L->p[s];
        }
    }
    modeled_probs(L);
    if (L->unique) {
        memcpy(L->grad, L->grad_aux, sizeof(double) * (size_t)n);
    } else if (L->threads <= 1) {
        for (int j = 0; j < n; ++j) L->grad[j] = 0;
        for (int64_t r = 0; r < L->n_paths; ++r) {
            double a = L->rpp[r] * L->grad_aux[r];
            for (int64_t k = L->Prow[r]; k < L->Prow[r + 1]; ++k) L->grad[L->Pcol[k]] += L->Pdata[k] * a;
        }
    } else {   /* P^T. with per-thread partial vectors, summed in thread order */
        const int nt = L->threads;
        double* part = calloc((size_t)nt * (size_t)(n + 1), sizeof(double));
#pragma omp parallel num_threads(nt)
        {
#ifdef _OPENMP
            const int t = omp_get_thread_num();
#else
            const int t = 0;
#endif
            double* g = part + (size_t)t * (size_t)(n + 1);
#pragma omp for schedule(static)
            for (int64_t r = 0; r < L->n_paths; ++r) {
                double a = L->rpp[r] * L->grad_aux[r];
                for (int64_t k = L->Prow[r]; k < L->Prow[r + 1]; ++k) g[L->Pcol[k]] += L->Pdata[k] * a;
            }
        }
        for (int j = 0; j < n; ++j) {
            double a = 0;
            for (int t = 0; t < nt; ++t) a += part[(size_t)t * (size_t)(n + 1) + (size_t)j];
            L->grad[j] = a;
        }
        free(part);
    }
}

/* objective + gradient at the current x: the per-iteration hot path */
void oracle_objective_grad(learner_t* L, double* kl, double* loglik) {
    compute_grad(L);
    objective(L);
    if (kl) *kl = L->kl;
    if (loglik) *loglik = L->plogp - L->kl;
}

/* Learner::Renormalize (src/Learner.cpp:23-43) */
void oracle_renormalize(learner_t* L) {
    int n = L->n, k = L->k;
    double* g = calloc((size_t)k + 1, sizeof(double));
    for (int i = 0; i < n; ++i) g[L->Ccol[i]] += exp(L->x[i]);
    for (int c = 0; c < k; ++c) g[c] = log(g[c]);
    for (int i = 0; i < n; ++i) L->x[i] -= g[L->Ccol[i]];
    free(g);
}

static void compute_expx(learner_t* L) { for (int i = 0; i < L->n; ++i) L->expx[i] = exp(L->x[i]); }

/* QuasiNewtonLearner::InitCallback (src/QuasiNewtonLearner.cpp:29-51) */
void oracle_qn_init(learner_t* L, int flags) {
    if (flags & 1) for (int i = 0; i < L->n; ++i) L->x[i] = 0.0;
    if (flags & 2) oracle_renormalize(L);
    if (flags & 4) {
        compute_expx(L);
        compute_grad(L);
        for (int c = 0; c < L->k; ++c) L->lambda[c] = 0.0;
        for (int i = 0; i < L->n; ++i) L->lambda[L->Ccol[i]] -= L->grad[i];
    }
    L->exp_lambda = (flags & 32) != 0;
}

/* QuasiNewtonLearner::OptimizationStep (src/QuasiNewtonLearner.cpp:162-201)
 * info7: KL, graderr, g_min, g_max, lambda_min, rmin, rmin index */
int oracle_qn_step(learner_t* L, double eta, double* info7) {
    int n = L->n, k = L->k;
    compute_expx(L);
    /* ComputeG (:148-160) */
    for (int c = 0; c < k; ++c) L->g[c] = -1.0;
    for (int i = 0; i < n; ++i) L->g[L->Ccol[i]] += L->expx[i];
    L->g_min = INFINITY; L->g_max = -INFINITY;
    for (int c = 0; c < k; ++c) { if (L->g[c] < L->g_min) L->g_min = L->g[c]; if (L->g[c] > L->g_max) L->g_max = L->g[c]; }
    compute_grad(L);
    objective(L);
    for (int i = 0; i < n; ++i) L->aux[i] = L->expx[i] * L->lambda[L->Ccol[i]];   /* Jg.lambda */
    double ge = 0;
    for (int i = 0; i < n; ++i) { L->rhs[i] = L->grad[i] + L->aux[i]; if (fabs(L->rhs[i]) > ge) ge = fabs(L->rhs[i]); }
    L->grad_error = ge;
    L->lambda_min = INFINITY;
    for (int c = 0; c < k; ++c) if (L->lambda[c] < L->lambda_min) L->lambda_min = L->lambda[c];
    /* ComputeLambdaNext (:127-146) */
    double* laux = calloc((size_t)k + 1, sizeof(double));
    for (int c = 0; c < k; ++c) laux[c] = L->lambda[c] * L->g[c];
    for (int i = 0; i < n; ++i) laux[L->Ccol[i]] -= L->grad[i];
    for (int c = 0; c < k; ++c) { L->g[c] += 1.0; laux[c] /= L->g[c]; }
    for (int i = 0; i < n; ++i) {
        double r = L->grad[i] + L->expx[i] * laux[L->Ccol[i]];
        r /= L->aux[i];
        L->x[i] -= eta * r;
    }
    for (int c = 0; c < k; ++c) laux[c] = L->lambda[c] - laux[c];
    /* LambdaUpdate (src/Learner.cpp:438-462) */
    if (!L->exp_lambda) {
        for (int c = 0; c < k; ++c) L->lambda[c] -= eta * laux[c];
    } else {
        for (int c = 0; c < k; ++c) L->lambda[c] *= exp(-eta * laux[c] / L->lambda[c]);
    }
    free(laux);
    if (info7) {
        info7[0] = L->kl; info7[1] = L->grad_error; info7[2] = L->g_min; info7[3] = L->g_max;
        info7[4] = L->lambda_min; info7[5] = 0; info7[6] = 0;
        if (!L->unique && L->mode == 0) {
            int64_t best = 0;
            for (int64_t r = 1; r < L->n_paths; ++r) if (fabs(L->rpp[r]) < fabs(L->rpp[best])) best = r;
            info7[5] = L->rpp[best]; info7[6] = (double)best;
        }
    }
    return OR_OK;
}

int oracle_qn_halt(const learner_t* L, double tol) {            /* :88-91 */
    return L->grad_error <= tol && fabs(L->g_min) <= tol && fabs(L->g_max) <= tol;
}

/* per-string trellis evaluation at Fsa-indexed log-weights w_full (index -1
 * -> 0): writes logq per corpus string and grad_full[j] = -sum p E[count_j]
 * over strings with q > 0 using the renormalized corpus weights.  Used to
 * check the device path directly at arbitrary weights. */
int oracle_trellis_eval(learner_t* L, const double* w_full, double* logq_corpus, double* grad_full,
                        double* loglik, char* err, int errlen) {
    int* topo = xrealloc(NULL, sizeof(int) * (size_t)(L->fsa.st.n + 1));
    if (eps_topo(&L->fsa, topo, err, errlen) != OR_OK) { free(topo); return OR_ERR; }
    double* ew = exp_weights(L, w_full);
    const int nt = L->threads > 1 ? L->threads : 1;
    const int64_t NC = L->corpus.words.n;
    const size_t nf = (size_t)L->n_full + 1;
    /* per-thread workspaces and gradient partials, summed in thread order
     * (one thread: the serial sum) */
    double* part = calloc((size_t)nt * nf, sizeof(double));
#pragma omp parallel num_threads(nt) if (nt > 1)
    {
#ifdef _OPENMP
        const int t = omp_get_thread_num();
#else
        const int t = 0;
#endif
        trellis_ws_t ws = {0};
        ws.N = (int)L->fsa.st.n;
        ws.topo = xrealloc(NULL, sizeof(int) * (size_t)(ws.N + 1));
        memcpy(ws.topo, topo, sizeof(int) * (size_t)ws.N);
        double* g = part + (size_t)t * nf;
#pragma omp for schedule(dynamic, 64)
        for (int64_t i = 0; i < NC; ++i) {
            double q = trellis_string(&L->fsa, &ws, L->corpus.words.a[i], L->corpus.lens.a[i],
                                      ew, g, -L->corpus.w.a[i], NULL);
            logq_corpus[i] = q > 0 ? log(q) : -INFINITY;
        }
        trellis_free(&ws);
    }
    for (int j = 0; j < L->n_full; ++j) {
        double a = 0;
        for (int t = 0; t < nt; ++t) a += part[(size_t)t * nf + (size_t)j];
        grad_full[j] = a;
    }
    double ll = 0;
    for (int64_t i = 0; i < NC; ++i)
        if (logq_corpus[i] > -INFINITY) ll += L->corpus.w.a[i] * logq_corpus[i];
    *loglik = ll;
    free(part); free(ew); free(topo);
    return OR_OK;
}

/* full-parameter weight vector in GetWeight form (for feeding the device) */
void oracle_get_w_full(const learner_t* L, double* w_full) {
    for (int j = 0; j < L->n_full; ++j) w_full[j] = get_weight(L, j);
}

/* Fsa-index name of parameter j */
int oracle_full_param_name(const learner_t* L, int j, const char** state, int* kind, const char** label) {
    if (j < 0 || j >= L->n_full) return OR_ERR;
    *state = L->fsa.st.a[L->fsa.p_state[j]].name; *kind = L->fsa.p_kind[j]; *label = L->fsa.p_label[j];
    return OR_OK;
}
int oracle_trimmed_index(const learner_t* L, int j) { return L->trimmed[j]; }

/* OpenMP threads of the per-iteration passes (ENUM SpMV chain, trellis
 * evaluation); 1 (the default) = serial, like the reference (mkl_sequential) */
void oracle_set_threads(learner_t* L, int threads) { L->threads = threads > 1 ? threads : 1; }

/* ENUM path matrices (src/Learner.cpp BuildFrom: P rows = paths, M rows =
 * strings) and the trimmed constraint of each parameter (Ccol), for the
 * second-order restatement in oracle/hessian.py.  nnz = Prow[n_paths]. */
int64_t oracle_path_nnz(const learner_t* L) { return L->mode == 0 && L->Prow ? L->Prow[L->n_paths] : -1; }
int oracle_get_paths(const learner_t* L, int64_t* prow, int* pcol, double* pdata, int64_t* mrow) {
    if (L->mode != 0 || !L->Prow) return OR_ERR;
    int64_t nnz = L->Prow[L->n_paths];
    memcpy(prow, L->Prow, sizeof(int64_t) * (size_t)(L->n_paths + 1));
    memcpy(pcol, L->Pcol, sizeof(int) * (size_t)nnz);
    memcpy(pdata, L->Pdata, sizeof(double) * (size_t)nnz);
    memcpy(mrow, L->Mrow, sizeof(int64_t) * (size_t)(L->S + 1));
    return OR_OK;
}
void oracle_get_ccol(const learner_t* L, int* out) { memcpy(out, L->Ccol, sizeof(int) * (size_t)L->n); }
