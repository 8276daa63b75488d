// Device-side views and launchers of the trellis kernels.
//
// Two kernels carry the hot path:
//   * trav_kernel<MODE> -- one wavefront per string, re-derives the string's
//     trellis from the automaton (LDS slab).  MODE_COUNT is the one-time
//     structural pass (recognition, path counts, used parameters, compiled
//     stream sizes), MODE_EMIT writes the compiled streams, MODE_WEIGHTED is
//     the per-iteration fallback for strings whose trellis does not compile.
//   * fbc_kernel -- the per-iteration forward-backward over compiled
//     streams, one lane per string, 64 strings of similar stream length per
//     wavefront, stream words interleaved so every load is coalesced, and the
//     gradient accumulated in LDS.
#pragma once

#include <hip/hip_runtime.h>

#include "peer_layout.hpp"

#include <cstddef>
#include <cstdint>
#include <cstdlib>

// Timing experiments that skip work on purpose (WFSA_FBS_DBG, WFSA_BUB_DBG,
// WFSA_QN_DBG, WFSA_W2_DBG) exist only in a build made with
// `make EXPERIMENTS=1`; the release library ignores those variables and its
// kernels carry no such branch.
#ifdef WFSA_EXPERIMENTS
#define WFSA_KDBG(x) (x)
inline int experiment_knob(const char* name) {
    const char* e = std::getenv(name);
    return e ? std::atoi(e) : 0;
}
#else
#define WFSA_KDBG(x) 0
inline int experiment_knob(const char*) { return 0; }
#endif

namespace wfsa {

constexpr int kMaxBubbleNodes = 32;    // nodes of one compiled bubble
constexpr int kMaxBubbleEdges = 255;   // edges of one compiled bubble
constexpr int kBubbleRegEdges = 8;     // bubbles up to this many edges run from registers
constexpr int kBubbleRegNodes = 8;     // (and so at most this many nodes)
// bubble record: 4 header words + 2 per edge, rounded up to 16 bytes
__host__ __device__ inline int bubble_record_words(int edges) { return (4 + 2 * edges + 3) & ~3; }
constexpr int kBubbleSlackWords = 4 * (1 + kBubbleRegEdges / 2);   // over-read of the last record
constexpr int kStreamPrefetch = 4;     // 16-byte chunks in flight per lane (per register set)
// slack after the last group's chunks (the prepare-time pass over-reads)
constexpr int kStreamTailChunks = 64 * 8;
// Each lane's first chunk of a group starts with a header: p of the lane's
// string (64 bits) and the group's chunk rows (low 16 bits of the next word),
// so the per-iteration kernel streams a wave's groups as one run.  Narrow
// (16-bit) words: the header takes words 0..4, wide (32-bit): words 0..2;
// the string's words follow.
__host__ __device__ inline int stream_hdr_words(int wide) { return wide ? 3 : 5; }

// Delta stream (the per-iteration stream kernel's format when the weights
// are staged in LDS and no word is a multi-parameter composite): a string's
// trivial words as a multiset -- their sum does not depend on the order --
// sorted, each a 10-bit step forward from the previous index.  The staged
// table is remapped with a zero-weight slot every kDeltaPeriod entries
// (slot 0 included): a gap longer than a step is bridged by steps onto zero
// slots, the lane starts each string on slot 0 and ends it on a zero slot,
// so padding fields (0) add nothing.  Row layout (16 bytes per lane): three
// 10-bit fields per dword (field i in dword i / 3 at bit 10 (i % 3); no
// field straddles a dword), 12 fields; the lane's first row of a group
// carries p (dwords 0-1) and the group's row count (bits 0-15 of dword 2) in
// place of fields 0-7.  c3: 10.5 bits per word against 16 (profiles/r04/
// stream_format_micro_v4b.txt).
constexpr int kDeltaBits = 10;
constexpr uint32_t kDeltaMax = (1u << kDeltaBits) - 1u;
// zero slots at the multiples of kDeltaPeriod (<= kDeltaMax: a zero slot is
// always within one step); odd, so the zero slots fall on different LDS
// banks -- the lanes whose strings have ended sit on them, as do the steps
// bridging long gaps (at 512 every zero slot was on bank 0: N-way conflicts)
constexpr int kDeltaPeriod = 511;
constexpr int kDeltaFields = 12, kDeltaHdrFields = 4;
// rows per register set of the delta pass (two sets in flight): 12 gathers
// per row, so fewer rows than the 16-bit pass's kStreamPrefetch (the stream
// micro: D = 2 17.9 us, D = 3 19.0 us)
#ifndef WFSA_DELTA_D
#define WFSA_DELTA_D 2
#endif
constexpr int kDeltaPrefetch = WFSA_DELTA_D;
__host__ __device__ inline int32_t delta_slot(int32_t j) { return j + 1 + j / (kDeltaPeriod - 1); }
// the zero slot after the last weight's: a string whose words end in the
// last period steps onto it (not onto the next multiple of kDeltaPeriod)
__host__ __device__ inline int32_t delta_end_slot(int32_t n_params) {
    return n_params > 0 ? delta_slot(n_params - 1) + 1 : 0;
}
// table entries (even: the kernel stages 16-byte pieces)
__host__ __device__ inline int32_t delta_table(int32_t n_params) { return (delta_end_slot(n_params) + 2) & ~1; }

// Per-iteration record of a combined edge, one 16-byte gather in the
// compiled kernel: its log-weight and its parameter list (p0 when np == 1).
struct alignas(16) EdgeRec {
    double lw;
    int32_t p0;   // first parameter (np >= 1)
    int32_t np;   // number of parameters
};

// Compiled trellis automaton resident in HBM (see trellis_model.hpp).
// Edge ids: [0, E) byte-consuming edges, [E, E+X) end edges ("combined").
struct ModelView {
    const int32_t* o_ptr;    // [n_nodes+1] out-edges by source node, sorted by byte
    const uint8_t* o_byte;
    const int32_t* o_dst;
    const int32_t* x_ptr;    // [n_nodes+1] end edges by source node (ids relative to E)
    const int32_t* pptr;     // [E+X+1] parameter list of each combined edge
    const int32_t* pidx;
    const double* ew;        // [E+X] exp(log-weight), per iteration
    const double* lw;        // [E+X] log-weight, per iteration
    const EdgeRec* erec;     // [E+X] log-weight + parameters, per iteration
    const double* node_end;  // [n_nodes] sum of the node's end-edge weights
    const double* node_end_count;  // [n_nodes] number of end edges (counting mode)
    const int32_t* multi_of;       // [E+X] index among multi-parameter edges, or -1
    const int32_t* multi_edge;     // [n_multi] combined edge of each multi-parameter edge
    int32_t n_nodes;
    int32_t start;
    int32_t n_edges;         // E
    int32_t n_params;        // Fsa parameters (w has a zero slot at n_params)
};

// Parameter code of combined edge g in a bubble record: its parameter when
// it has exactly one, n_params (the zero slot: weight log 1) when it has
// none, -(g + 2) when it has several.  The edge weight is then exp(w[code])
// straight from the weight table in the common case.
__host__ __device__ inline int32_t edge_code(const int32_t* pptr, const int32_t* pidx, int32_t g, int32_t n_params) {
    const int32_t np = pptr[g + 1] - pptr[g];
    return np == 1 ? pidx[pptr[g]] : (np == 0 ? n_params : -(g + 2));
}

// Per-wave LDS slab holding one string's trellis: frontier nodes (alpha,
// beta, node id) for every position, the live edges between consecutive
// positions, per-position offsets/scale exponents and the node->slot map.
struct SlabConfig {
    int32_t cap_f;           // frontier entries over all positions
    int32_t cap_e;           // live edges over all positions
    int32_t max_len;         // longest string
    int32_t n_nodes;
    int32_t bytes;           // bytes per wave
    int32_t waves_per_block;
};

struct SlabLayout {
    int32_t alpha, beta, state, eg, esrc, edst, fpos, epos, dsc, slot, total;
};

inline SlabLayout slab_layout(int32_t cap_f, int32_t cap_e, int32_t max_len, int32_t n_nodes) {
    SlabLayout l;
    const int32_t np = max_len + 2;
    l.alpha = 0;
    l.beta = l.alpha + 8 * cap_f;
    l.state = l.beta + 8 * cap_f;
    l.eg = l.state + 4 * cap_f;
    l.esrc = l.eg + 4 * cap_e;
    l.edst = l.esrc + 4 * cap_e;
    l.fpos = l.edst + 4 * cap_e;
    l.epos = l.fpos + 4 * np;
    l.dsc = l.epos + 4 * np;
    l.slot = l.dsc + 4 * np;
    l.total = (l.slot + 4 * n_nodes + 15) & ~15;
    return l;
}

// MODE_MIN: the weighted forward plus the (min, x) forward of the rmin info
// column -- log(min path weight / q) per string into rmin_log, no backward.
enum TravMode { MODE_WEIGHTED = 0, MODE_COUNT = 1, MODE_EMIT = 2, MODE_MIN = 3 };

struct TravArgs {
    ModelView m;
    const uint8_t* sym;      // packed corpus bytes
    const int64_t* off;      // [S+1]
    const double* p;         // [S]
    const int32_t* list;     // strings this launch serves
    int32_t n_list;
    SlabConfig slab;
    SlabLayout lay;
    // weighted mode
    double* grad;            // [n_params]  accumulates -p_s * E[count]
    double* ll_part;         // [waves in grid]
    double* logq;            // [S] or null
    // counting mode
    double* path_count;      // [S] or null
    uint8_t* recognized;     // [S] or null
    uint8_t* used;           // [n_params] or null
    int32_t* c_main;         // [S] compiled main-stream words, or null
    int32_t* c_bub;          // [S] compiled bubble words (-1: does not compile)
    int32_t* c_nbub;         // [S] number of bubbles
    // emit mode
    void* stream;            // interleaved main streams (see CompiledArgs)
    int32_t wide;            // 32-bit words (else 16-bit)
    const int64_t* s_base;   // [S] element index of the string's first main word
    int32_t* bub;            // bubble buffer
    const int64_t* b_base;   // [S] word index of the string's first bubble word
    const int32_t* b_first;  // [S] ordinal of the string's first bubble
    int32_t* bub_off;        // [n_bubbles] word offset of each bubble
    uint8_t* overflow;       // [S] string did not fit the slab
    unsigned long long* live_edges;
    const unsigned* halted;  // device-resident QN run: nonzero = skip (or null)
    double* rmin_log;        // min mode: [S] log of the string's smallest relative path probability
};

// Tier 2 of the traversal: strings whose trellis overflows every LDS slab
// (ambiguous automata: hundreds of live nodes per position).  One block per
// string; alpha of every position is a dense vector over the trellis nodes in
// global scratch, built by gathering through the byte-indexed in-edge lists
// (each destination node summed by one thread: no atomics); beta rolls over
// two vectors, gathered through the out-edges; the gradient accumulates in
// LDS when n_params fits (else global atomics).
// Byte-pair tables of the tier-2 wave kernel.  The nodes live at position i
// are D(c_{i-1}) (the nodes a byte-c_{i-1} edge enters; at 0 the start node,
// pseudo-byte K), so a trellis step (a = c_{i-1}, b = c_i) only ever joins
// D(a) to D(b).  Rows are indexed by position in D (compact), and every pair
// (a, b), a in [0, K], b in [0, K), owns the list of its edges -- the edges
// consuming b whose source is in D(a) -- as
//   ent = (src index | dst index << 16, edge id, param0, param1)
// (param -1: none; param0 = -2: more than two, read pptr/pidx) and, rewritten
// each evaluation, its ew and lw.  A wave walks a pair's list with one edge
// per lane (contiguous loads, no padding) and sums into its LDS rows.
struct PairTables {
    int32_t K;               // compact alphabet (bytes some edge consumes)
    const int32_t* bidx;     // [256] byte -> compact index, -1
    const int32_t* n;        // [K + 1] |D(b)| (< 65536); n[K] = 1 (start)
    const int32_t* dl_ptr;   // [K + 2] D(b) node list offsets into dl_node
    const int32_t* dl_node;  // node ids
    const int32_t* e_ptr;    // [(K + 1) K + 1] edge range of pair a K + b
    const int32_t* sd;       // [entries] the ent .x alone (the forward's contiguous loads)
    const int4* ent;
    const double* w;         // this evaluation's ew per entry
    const double* lw;        // and lw
    int32_t max_n;
};

// The same steps laid out for pulling (wave_pull_kernel): the forward sums
// each destination of D(b) over its in-edges, the backward each source of
// D(a) over its out-edges, one lane per node -- no LDS atomics, each node's
// sum in a fixed order, one LDS row per wave (a lane holds its nodes' sums in
// registers until every lane has read the row, then overwrites it).  Per
// pair the nodes are dealt to the 64 lanes (largest first, to the least
// loaded lane, at most `items` per lane) and each lane's entries are its
// nodes' edge lists back to back, lane-strided: entry t of lane l at
// base + 64 t + l, T entries per lane (the most loaded lane; the rest padded).
// A node's last entry carries the flag bit and the node; a node without edges
// gets one empty flagged entry (its sum is 0).  The backward's entries start
// with one more row: per lane its sources in item order, 16 bits each
// (0xffff: none), so a lane loads their alpha at the step's start; the
// forward's destinations are listed the same way in fhdr (per pair, per lane).
//   forward code:  src index | dst index << 16 | last << 31
//   backward code: dst index | src index << 16 | last << 31
// (src in D(a), dst in D(b), both < 2^15).
constexpr int kPullItemsMax = 8;
struct PullTables {
    int32_t items;           // nodes per lane at most: 4, 6 or 8 (the kernel's register queues)
    const int4* info;        // [(K + 1) K] per pair: forward base, forward T, backward base, backward T
    const int4* fhdr;        // [(K + 1) K][64] each lane's destinations, 16 bits each (0xffff: none)
    const int32_t* fcode;    // forward entries
    const double* fw;        // their ew this evaluation (0: padding / empty node)
    const double* flw;       // their lw (rmin column; -inf: padding)
    const int4* bent;        // backward entries: code, edge id, param0, param1 (as PairTables::ent)
    const double* bw;        // their ew this evaluation
};

struct WideModel {
    const int32_t* c_ptr;    // [257] destination entries of byte c: [c_ptr[c], c_ptr[c+1])
    const int32_t* dst;      // [n_dst] the node (every destination of a byte-c edge, once)
    const int32_t* e_ptr;    // [n_dst + 1] its in-edges with that byte
    const int32_t* e_src;    // [E] source node
    const int32_t* e_g;      // [E] edge id (ModelView numbering)
};
constexpr int kWideBlock = 256;
struct WideArgs {
    ModelView m;
    WideModel w;
    const uint8_t* sym;
    const int64_t* off;
    const double* p;
    const int32_t* list;
    int32_t n_list;
    int32_t max_len;
    double* scratch;         // per block: alpha [(max_len+1) n_nodes], beta [2 n_nodes], exponents
    int64_t scratch_stride;  // doubles per block
    int32_t grad_lds;        // weighted: the gradient accumulates in LDS (n_params doubles)
    int32_t dbg;             // wide2 timing experiments (WFSA_W2_DBG): 1 no backward, 2 no edge loops, 3 both
    double* grad;            // [n_params]  -p_s E[count]
    double* ll_part;         // [grid]
    double* logq;            // [S] or null
    double* path_count;      // counting: [S] or null
    uint8_t* recognized;
    uint8_t* used;
    const unsigned* halted;
    unsigned long long* live_edges;   // counting: += the edges the forward gathers over (or null)
    double* rmin_log;        // min mode: [S] log(min path weight / q)
    // weighted mode, wave per string (wide2_kernel over the byte-pair tables)
    PairTables pt;
    PullTables pl;           // wave_pull_kernel (info null: not built)
    double* scratch2;       // per wave: alpha rows (compact, 1 + max_len * max_n), min-forward rows
                             // [2 max_n], exponents [max_len + 2]
    int64_t stride2;         // doubles per wave
    int64_t hrows2;          // wave_pull_kernel: doubles of a wave's alpha rows (the min-forward rows follow)
    unsigned* ctr;           // [2] work and block-exit counters (zero between launches)
    // wide2_kernel's order-independent sums (fixed point, fix128_* in
    // fb_kernels.hip): [2 n_params] gradient accumulators (lo, hi words, fix_frac
    // fraction bits), [2] the log-likelihood's (64 fraction bits), [1] flags
    // (kFix*); zero between launches
    unsigned long long* fix;
    int32_t fix_frac;
};
// doubles of scratch per block
inline int64_t wide_scratch_stride(int32_t max_len, int32_t n_nodes) {
    return (int64_t(max_len) + 3) * int64_t(n_nodes) + (int64_t(max_len) + 3) / 2 + 2;
}
hipError_t launch_wide(bool counting, const WideArgs& a, int grid, hipStream_t stream, bool min_mode = false);
// Tier 2 weighted pass, one wavefront per string (kWide2Block threads per
// block, the blocks' waves take strings from a work counter): alpha rows in
// HBM (zeroed behind the backward), gradient in one LDS table per block
// when n_params fits.  grid: blocks.
constexpr int kWide2Block = 1024;
// wave_pull_kernel's largest block: its launch bound sets the register budget
// (1024 threads: 4 waves per SIMD, 128 VGPRs)
#ifndef WFSA_PULL_BLOCK
#define WFSA_PULL_BLOCK 1024
#endif
constexpr int kPullBlock = WFSA_PULL_BLOCK;
// alpha rows of a wave: compact (wide2_kernel, 1 + max_len * max_n), or in
// wave_pull_kernel's slot layout (a row per step of items * 64 slots, slot
// k * 64 + lane the lane's k-th backward source); the larger of the two
inline int64_t wide2_rows(int32_t max_len, int32_t max_n, int32_t items) {
    const int64_t compact = 1 + int64_t(max_len) * max_n, slots = int64_t(max_len) * items * 64;
    return compact > slots ? compact : slots;
}
inline int64_t wide2_stride(int32_t max_len, int32_t max_n, int32_t items = 0) {
    return wide2_rows(max_len, max_n, items) + 2 * int64_t(max_n) + (int64_t(max_len) + 3) / 2 + 2;
}
// LDS of a block: the gradient table (grad_lds, + 64 spare slots) + per wave 2 rows of max_n doubles
inline size_t wide2_lds(int32_t n_params, bool grad_lds, int waves, int32_t max_n) {
    return (grad_lds ? size_t((n_params + 64 + 1) & ~1) * 8 : 0) + size_t(waves) * 2 * size_t(max_n) * 8;
}
// waves: per block (blockDim = 64 waves); lds from wide2_lds
hipError_t launch_wide2(const WideArgs& a, int grid, int waves, size_t lds, hipStream_t stream);
// LDS of a wave_pull_kernel block: the gradient table + one row per wave
inline size_t pull_lds(int32_t n_params, bool grad_lds, int waves, int32_t max_n) {
    return (grad_lds ? size_t((n_params + 64 + 1) & ~1) * 8 : 0) + size_t(waves) * size_t(max_n) * 8;
}
hipError_t launch_wave_pull(const WideArgs& a, int grid, int waves, size_t lds, hipStream_t stream);
// the pull tables' per-evaluation weights: w[i] = ew[g[i]] (0 where g < 0),
// and for i < n_lw, lw_out[i] = lw[g[i]] (-inf where g < 0)
hipError_t launch_pull_weights(const int32_t* g, int64_t n, int64_t n_lw, const double* ew, const double* lw,
                               double* w, double* lw_out, hipStream_t stream);
// the pair tables' per-evaluation weights pw[0, n) = ew, pw[n, 2n) = lw
hipError_t launch_pair_weights(const int4* ent, int64_t n, const double* ew, const double* lw, double* pw,
                               hipStream_t stream);

// The rmin info column (QuasiNewtonLearner::GetOptimizationInfo,
// src/QuasiNewtonLearner.cpp:80-84; HessianLearner :313-317): the smallest
// relative path probability min_paths exp(P x)_path / q_s over every string.
// A compiled string's path posterior factors over its bubbles, so its
// smallest one is the product of each bubble's smallest (min, x) path over
// the bubble's sum (rmin_bubble_kernel, lane per bubble); traversal strings
// get log(min path / q) from trav_kernel<MODE_MIN> / wide_kernel min mode;
// rmin_strings_kernel (lane per ambiguous string) sums each string's run and
// takes the minimum, ties to the lower index; rmin_final_kernel merges the
// block minima.
struct RminArgs {
    ModelView m;
    const int32_t* bub;
    const int32_t* bub_off;  // [n_bub]
    int32_t n_bub;
    int32_t max_nodes;       // largest bubble: sizes the kernel's LDS node vectors
    double* vb;              // [n_bub] log(min path / Z) per bubble; null: the evaluation's bubble
                             // passes accumulated them per string into rmin_log (read and re-zeroed)
    const double* w;         // [n_params + 1] weights (multi-parameter edges)
    const double* ewp;       // [n_params + 1] exp(w)
    double* rmin_log;        // [S] traversal strings' values
    const double* sv;        // [n_bub] or null: per-bubble values at list positions (BubbleArgs::rmin_sv)
    const int32_t* bpos;     // [n_bub] list position of bubble b
    const int4* amb;         // [n_amb] (string, first bubble, bubble count | -1 traversal, 0), ascending
    int64_t n_amb;
    double* part;            // [blocks][2]
    double* res;             // [2]: rmin, string index (-1: no ambiguous string)
    const unsigned* halted;
};
constexpr int kRminBlock = 256;
// final = false: leave the block minima in part[] (log values, string index)
// for the QN finish to reduce (QnArgs::rmin_part)
hipError_t launch_rmin(const RminArgs& a, hipStream_t stream, bool final = true);
// rmin across ranks: the phases around the two Min all-reduces (fb_kernels.hip)
hipError_t launch_rmin_rank(double* res, double* key, double base, int phase, hipStream_t stream);
inline int rmin_blocks(int64_t n_amb) { return int(n_amb > 0 ? (n_amb + kRminBlock - 1) / kRminBlock : 1); }

// Second-order term of the Hessian (HessianLearner::ComputeHf,
// src/HessianLearner.cpp:498-547): sum_s p_s Cov_s(count_j, count_k).  The
// segments of a compiled string are independent, so a string's covariance is
// the sum of its bubbles' (trivial words have constant counts).  One
// wavefront per bubble: alpha, beta, the node-to-node path sums R (<= 16 x 16)
// and, for every ordered pair of its edges (e, f),
//   v(e, f) = P(e and f on the path) - P(e) P(f),
//   P(e and f) = alpha(src e) w_e R(dst e, src f) w_f beta(dst f) / Z (e before f),
// written p-scaled into the bubble's slots: one slot per (e, f, j in e, k in
// f, j <= k), in that nesting order (hf_slots counts them the same way).
struct HfArgs {
    ModelView m;
    const int32_t* bub;        // bubble records (BubbleArgs)
    const int32_t* bub_off;    // [n_bubbles]
    const int64_t* slot_base;  // [n_bubbles + 1]
    int32_t n_bubbles;
    const double* w;           // [n_params + 1] weights (GetWeight form)
    const double* ewp;         // [n_params + 1] exp(w)
    double* slot_val;          // [slots]
    // the pattern sums: entry t = sum of slot_val[t_slot[t_ptr[t] .. t_ptr[t+1])]
    const int64_t* t_ptr;
    const int64_t* t_slot;
    int64_t n_pattern;
    double* out;               // [n_pattern]
};
constexpr int kHfBlock = 256;   // four bubbles per block

// H_f of the strings the traversal kernels carry (no bubble decomposition):
// per string s, over its equivocal parameters V_s (the parameters whose count
// differs between its paths, at most kHfTravMaxV; the host finds them at set-up
// from exact min / max counts), the count covariance from one backward and one
// forward pass: with G_i(u)[j] the path-weighted count of parameter j over the
// paths into node u at position i (G rolls forward with alpha),
//   E[c c^T] = D + A + A^T,  D = sum_e P(e) c(e) c(e)^T,
//   A[j][k] = sum_e (w_e beta(dst) / Z) G(src)[j] c_k(e)   (pairs strictly before e),
//   E[c] = sum_e P(e) c(e);   slot (a <= b) = p_s Cov(a, b).
// One wavefront per string: lanes over nodes for the alpha / beta rows, lanes
// over j for G and A; every sum in a fixed order (deterministic).
constexpr int kHfTravMaxV = 512;   // (8 columns per lane)
struct HfTravArgs {
    ModelView m;
    WideModel w;             // in-edges by byte
    const uint8_t* sym;
    const int64_t* off;
    const double* p;
    const int4* list;        // (string, offset of V_s, |V_s|, 0)
    const int32_t* vlist;    // V_s, ascending Fsa parameter ids
    const int64_t* slot_base;   // [n_list] first slot of the string
    int32_t n_list;
    int32_t max_len;
    const double* wt;        // [n_params + 1] weights (GetWeight form)
    double* scratch;         // per wave: hf_trav_stride doubles
    int64_t stride;
    int32_t vm;              // columns of G / A / D: max |V_s| rounded up to 64, <= kHfTravMaxV
    double* slot_val;
};
inline int64_t hf_trav_stride(int32_t max_len, int32_t n_nodes, int32_t vm) {
    return (int64_t(max_len) + 1) * (n_nodes + 1) + 4 * int64_t(n_nodes) + 2 * int64_t(n_nodes) * vm +
           2 * int64_t(vm) * vm + vm + 16;
}
hipError_t launch_hf(const HfArgs& a, hipStream_t stream, const HfTravArgs* trav = nullptr, int trav_grid = 0);

// Device-resident QuasiNewton step (qn_kernel.hip): qn_step_kernel, one
// block per constraint, completes the gradient of the constraint's members
// (the traversal tiers' part in out, the constant trivial-word part, and --
// fused -- the sums of their bubble contribution slots in a fixed order),
// updates x and lambda, writes the next w_full, and leaves its block partial
// (g, g, lambda, graderr).  The step's FINISH -- the info row [KL, graderr,
// g_min, g_max, lambda_min, rmin, rmin string, status] from those partials
// and the log-likelihood partials, into a host-mapped ring slot, then the
// flag -- runs in the first block of the NEXT step's stream kernel (which
// does not depend on it; no arrival ticket: 1024 same-address atomics cost
// ~8 ns each, serialised), or as its own one-block launch after the last
// step of a run / when the next step has no stream kernel.
//
// Halting: the finish of step e sets halt_pending; the QN kernel of step
// e + 1 (a later launch) sees it, publishes its row as skipped and sets
// halted, which every evaluation kernel of the later steps checks at entry.
// A launch never reads a flag that the same launch writes.
constexpr int kQnRow = 8;
// kQnTimedOut: an in-kernel QN wave's arrival wait gave up (its constraints
// were not updated; the finish reports it and the host fails the run)
constexpr unsigned kQnRan = 0, kQnHalted = 1, kQnNonFinite = 2, kQnSkipped = 3, kQnTimedOut = 4;
constexpr int kQnBlock = 256;
constexpr int kQnMaxSeg = 1024;   // members of a constraint the fused kernel keeps in LDS
struct QnFinish {
    int32_t active;              // (stream kernel: its block 0 finishes the previous step)
    const double* partial;       // [n_blocks][4] the QN kernel's block partials
    int32_t n_blocks;
    const double* ll_part;       // log-likelihood partials (fixed-order sum), or null: out0
    int32_t n_ll;
    const double* out0;
    const double* rmin;          // [2] the step's rmin column (rmin, string index), or null (0, 0)
    const double* rmin_part;     // or: [n][2] block minima (log rmin, string index)
    int32_t rmin_n_part;
    int32_t k;
    double plogp, tol;
    int32_t ring_slot;           // ring slot of the step
    // across ranks (px.on): the step's log-likelihood sum and rmin minimum
    // exchanged through the peer areas (PeerX) in flag / slot px_slot of the
    // finish's exchanges; rm_base: this rank's first global string
    PeerX px;
    int32_t px_slot;
    double rm_base;
    uint32_t tag;                // the row's sequence number as the host expects it: written into the row
                                 // with the status (row[7] = status + 16 tag), so a reader that sees the
                                 // flag before the row's data waits for the row itself
    const unsigned* halted;      // [0] halted, [1] halt_pending (the finish writes [1]),
                                 // [2] an in-kernel QN wave's wait timed out (sc1)
    unsigned* halt_pending;
    unsigned* seq;               // device sequence counter
    unsigned* host_flag;         // host-mapped completion flag
    double* host_ring;           // host-mapped [slots][kQnRow]
};
struct QnArgs {
    const double* out;           // [1 + n_full]: gradient parts accumulated so far
    double* ll_stash;            // non-null (across ranks): out[0], the step's all-reduced log-likelihood,
                                 // copied here for the step's finish (which rides in the next stream kernel,
                                 // which zeroes out)
    int32_t use_out;             // (fused: 0 when no traversal string adds to out)
    const double* fixed;         // [n_full] constant trivial-word gradient to add, or null
    const double* fixed_t;       // fused: the same in trimmed order ([n]), or null (then fixed[full_of])
    const double* contrib;       // fused: bubble contribution slots, or null
    const int64_t* grp_base;     // fused: physical slot base of constraint c's group
    const int32_t* grp_nch;      // fused: its chunk count
    const int32_t* seg_ptr;      // fused: [n + 1] logical slot run of kept parameter i (trimmed order)
    const int32_t* chunk_ptr;    // fused: [n + 1] its chunks (cumulative)
    int32_t n_full, n, k;
    const int32_t* full_of;      // [n] full index of each kept parameter
    const int32_t* trim;         // [n_full] trimmed index / -1 / -2
    const int32_t* cptr;         // [k+1] constraint c owns parameters [cptr[c], cptr[c+1])
    double* x;
    double* lambda;
    double* expx;
    double* grad;
    double* w_full;              // [n_full + 1] (zero slot)
    double* ewp;                 // [n_full + 1] exp(w_full), for the bubble kernel
    double* partial;             // [max(k, 1)][4] block partials (the finish reads them)
    double eta;
    int32_t exp_lambda;
    unsigned* halted;            // [0] halted, [1] halt_pending
    QnFinish fin;                // this step's finish (publication of skipped rows)
    int32_t dbg;                 // timing experiments only (WFSA_QN_DBG)
    int32_t seg_cap;             // LDS capacity: members of the largest constraint (<= kQnMaxSeg; 0: that)
    int32_t chunk_cap;           // ... and its slot chunks (<= kMaxChunks; 0: that)
    RminArgs rm;                 // rm_on: the rmin strings pass folded into this launch (its block c runs
    int32_t rm_on, rm_blocks;    // the pass's block c, c < rm_blocks; the grid covers both)
};

// Bubble evaluation.  Contributions (-p_s x edge posterior) go straight to
// their slots in `contrib`, which is parameter-major: parameter j owns the
// contiguous range [slot_ptr[j], slot_ptr[j+1]) -- the tail kernel then sums
// contiguous runs, no gather.
//   small bubbles (every edge with at most one parameter) in two classes,
//     A: <= 4 nodes and edges, B: <= kBubbleRegNodes nodes, <= kBubbleRegEdges
//     edges; each a structure-of-arrays table of 16-byte quads -- quad k of
//     bubble b at tbl[k * n + b]: [header: nodes | edges << 16, string, p (2
//     words)], RE/2 x [(code, src | dst << 16) x 2], RE/4 x [slot x 4] (-1:
//     the edge has no parameter) -- one lane per bubble, coalesced loads.
//   big bubbles (the rest, rare): variable records in `bub` at big_off[i]
//     (bubble record layout above), one wavefront per bubble; the slots of
//     edge e of big bubble i are big_eslot[big_eslot_ptr[big_edge_base[i] + e] ..].
constexpr int kSmallBubbleQuads = 7;
constexpr int kBigEdgeLds = 256;   // > kMaxBubbleEdges: per-wave staging of a big bubble
// per-wave LDS staging of a big bubble of at most E edges in the stream
// kernel (E even): weights / contributions and alpha, beta (doubles), then
// the edges' nodes (ints); 16-byte multiple
__host__ __device__ inline int big_stage_bytes(int E) { return ((E + 2 * kMaxBubbleNodes) * 8 + E * 4 + 15) & ~15; }
// The big bubbles' wave order in the stream kernel: wave rank r takes big
// bubbles r, r + (waves - 1), ...  Ranks run from the blocks' last waves
// backwards (those waves take no small bubbles); block 0's last wave, the QN
// finish's, takes none; the QN waves (wave wpb - 2 of blocks [0, qw_waves))
// come last, so they take one only when every other wave has: a QN wave with
// a big bubble started its update late (with the rmin column its deferred
// (min, x) pass came first too)
__host__ __device__ inline int big_rank(int bid, int wib, int nblk, int wpb, int qw_waves) {
    int r = (nblk - 1 - bid) + nblk * (wpb - 1 - wib);
    r -= r > nblk - 1 ? 1 : 0;
    if (qw_waves <= 0) return r;
    if (wib == wpb - 2 && bid < qw_waves) return nblk * wpb - 1 - qw_waves + bid;
    return r >= 2 * nblk - 1 - qw_waves ? r - qw_waves : r;
}
constexpr int kSmallBubbleQuads4 = 4;   // class A: <= 4 nodes, <= 4 edges (1 + 2 + 1 quads)
struct BubbleArgs {
    ModelView m;
    const int4* sm4_tbl;     // class A table (most bubbles: diamonds)
    int32_t n_small4;
    const int4* sm_tbl;      // class B table (<= 8 nodes, <= 8 edges)
    int32_t n_small;
    const int32_t* bub;
    const int32_t* big_off;
    int32_t n_big;
    int32_t small_wpb;       // fused: waves [0, small_wpb) of every block take 64 small bubbles each
    int32_t qw_waves;        // fused: the layout's QN waves (big_rank; whether or not this launch runs them)
    int32_t big_lds_edges;   // fused: max edges of a big bubble (even) ...
    int32_t big_lds_off;     // ... and the byte offset of the waves' staging in the stream kernel's LDS
    const int32_t* big_edge_base;
    const int32_t* big_eslot_ptr;
    const int32_t* big_eslot;
    double* contrib;
    double* ll_part;         // [waves in grid]
    double* logq;            // [S] or null: log Z added to the string's entry
    double* rmin_acc;        // [S] or null: log(min path / Z) added to the string's entry (rmin column;
                             // small bubbles only in the RMIN kernel variants)
    double* rmin_sv;         // [n_bubbles] or null: the same value stored per bubble at its list position
                             // (small4, small, big) instead of added -- coalesced, summed per string in
                             // bubble order by rmin_strings_kernel (deterministic)
    const double* w;         // [n_params + 1] weights (GetWeight form) with the zero slot
    const double* ewp;       // [n_params + 1] exp(w), ewp[n_params] = 1 (per iteration)
    const unsigned* halted;
    int32_t dbg;             // timing experiments only (WFSA_BUB_DBG): 1 no slot stores, 2 no weight gathers
    int32_t wt;              // contribution slots stored write-through (sc1): read in the same launch (QnWave)
};

// Compiled streams of the per-iteration kernels.
//   main stream: only "trivial" words (edges whose posterior is 1).  Narrow
//     (16-bit) words: j < 0x8000 a single-parameter edge with parameter j,
//     0x8000 + m the m-th multi-parameter edge, 0xFFFF padding.  Wide (32-bit)
//     words: j >= 0 a parameter, -(g+2) multi-parameter combined edge g, -1
//     padding.  Each lane's words are cut into 16-byte chunks (8 narrow / 4
//     wide words); chunk c of lane l of group g sits at chunk index
//     g_base[g] + 64 c + l, so one wavefront reads 1 KiB per load.
//   bubble buffer: per bubble [nodes | edges << 16, string, p (2 words),
//     (edge code, src | dst << 16) x edges] (edge_code above), 16-byte aligned
//     (padded), so edge e of the bubble at word offset o owns contribution
//     slot o / 2 + 2 + e.
// The QN update inside the stream kernel (one rank, every string compiled,
// delta stream, no rmin column): the bubble waves store their contribution
// slots write-through (sc1), and each block, once all its waves' stores have
// retired (the last wave of the block by an LDS counter), adds one arrival to
// a per-launch counter (agent-scope atomic).  The QN waves -- wave wpb - 2 of
// blocks [0, n_waves), charged by the dealer -- stream their (shorter) share
// of rows, then poll the counter (sc1 loads) until every block has arrived,
// read the slots with sc1 loads and run the QuasiNewton update of their
// batches of constraints: a batch is a run of consecutive constraints with at
// most 64 members, a lane per member, the per-constraint sums in member order
// by lane shuffles (the host's order: bitwise the same update as
// qn_step_kernel).  The finish wave of the same launch (the previous step's
// info row and halt decision) arrives like the bubble waves, so the QN waves
// read its halt_pending (stored sc1) after the same poll.  The updated weights
// go to the other parity's buffers (w_next, ewp_next): the blocks of this
// launch still read the current ones.  Launch e uses arrive[e & 1] and zeroes
// arrive[(e + 1) & 1] for the next launch.  A poll that outlasts its limit
// writes NaN partials (the step's row then reports non-finite) instead of
// hanging.
constexpr int kQnWaveMembers = 64;
constexpr int kQnWaveChunkRounds = 4;   // a batch's slot chunks, one per lane per round: at most 256
struct QnWave {
    int32_t on;
    int32_t n_batches;
    int32_t n_waves;             // QN waves: wave wpb - 2 of blocks [0, n_waves)
    int32_t parity;
    int32_t n_arrive;            // arrivals to wait for (the grid's blocks)
    const int4* batch;           // [n_batches][2] (first constraint, end constraint, first member, end member),
                                 // (slot chunks, their first slot: low, high word, 0)
    const int32_t* con_of;       // [n] constraint of each member (trimmed order)
    const int32_t* mfirst;       // [n] the member's first chunk within its batch
    const int32_t* mnch;         // [n] its chunk count
    const int32_t* cptr;         // [k + 1]
    const int32_t* full_of;      // [n]
    const double* fixed_t;       // [n] constant trivial-word gradient, trimmed order
    const double* out;           // [1 + n_full] the traversal strings' gradient (kernels before this launch), or null
    const double* contrib;
    double* x;
    double* lambda;
    double* grad;
    double* w_next;              // [n_full + 1] the next step's weights (the other parity)
    double* ewp_next;
    double* partial;             // [k][4] (g, g, lambda, graderr), read by the next finish
    double eta;
    int32_t exp_lambda;
    unsigned* arrive;            // [2] per-parity arrival counters
    unsigned* halted;            // [0] halted (earlier launches), [1] halt_pending (this launch's finish, sc1),
                                 // [2] set by a QN wave whose arrival wait timed out
    QnFinish fin;                // this step's publication (a skipped row after a halt; with self_finish, its row)
    int32_t self_finish;         // the launch's last finisher (after every block's log-likelihood partial and
                                 // every QN wave's partials, write-through) runs this step's finish itself
    unsigned* done;              // [2] per-parity counters of those arrivals (each launch zeroes the other's)
    PeerX px;                    // px.on: across ranks -- each batch's member partials (the slot sums and
                                 // the traversal part) summed over the ranks through the peer areas
    uint32_t poll_limit;         // polls before a QN wave gives up (0: kQnPollLimit)
    int32_t poll_fault;          // fault injection (tests): QN wave 0 waits for one arrival too many
    unsigned* go;                // [n_waves][kQnGoStride]: wave r's go line (r > 0), set to fin.tag by wave 0
};

// QN waves' go lines: 256 bytes apart (their polls spread over the memory
// channels), at most kQnMaxWaves of them
constexpr int kQnGoStride = 64;
constexpr int kQnMaxWaves = 1024;

// The rmin column inside the in-kernel QN step (fbs_kernel<..., RMIN, DELTA,
// QN>; GetOptimizationInfo's smallest relative path probability,
// src/QuasiNewtonLearner.cpp:80-84): no strings pass of its own.  A bubble
// whose string has one bubble is that string's candidate at once (its lane's
// log(min path / Z)); a string of k > 1 bubbles stores each bubble's value
// write-through, and after the wave's arrival (its stores retired) adds one
// to the string's counter -- the k-th adder sums the k values in bubble order
// (the strings pass's order: the same bits) and holds the candidate.
// Ambiguous traversal strings' values (rmin_log, written by the traversal
// kernels before this launch) are read at the block's end.  Each block's
// (min, string) pair -- ties to the lower string, an order-free minimum --
// goes to part[block] beside its log-likelihood partial; the step's finish
// reduces them.
struct RminFold {
    const int2* bk;          // [bubble positions] (k, run): k = bubbles of the bubble's string if it is
                             // ambiguous, else 0; run = the string's first entry in mpos (k > 1)
    const int32_t* mpos;     // the bubble positions of each multi-bubble string, in bubble order
    unsigned* cnt;           // [mpos entries] the arrivals per multi-bubble string (at its run's first
                             // entry; the k-th arrival re-zeroes it for the next launch)
    const int32_t* trav;     // [n_trav] ambiguous traversal strings
    int32_t n_trav;
    const double* rmin_log;  // [S] their values
    double* part;            // [blocks][2] this launch's block minima (log rmin, string index)
};

// a lane's small bubble in the folded column: its value and string, and its
// string's bubble count and run (RminFold::bk) for the wave's end
struct RminLane {
    double rv;
    int32_t str, k, run;
    int32_t big;             // a big bubble's index whose (min, x) pass is still due (rv: its Z), or -1
};

struct CompiledArgs {
    ModelView m;
    const double* p;         // [S]
    const uint4* stream;     // 16-byte chunks
    const int64_t* g_base;   // [G] first chunk of the group
    const int32_t* g_len;    // [G] chunk rows of the group (its longest lane, header included)
    const int32_t* l_str;    // [64 G] string of each lane, -1 = padding
    const int32_t* l_len;    // [64 G] words of each lane (header excluded)
    const int32_t* wave_first;   // [stream waves + 1] the per-iteration kernel's groups of
                                 // wave w: [wave_first[w], wave_first[w + 1]), contiguous
    int32_t n_groups;
    int32_t n_params;
    int32_t d_tab;           // > 0: the stream is in the delta format, its LDS table has d_tab entries
    int32_t tables;          // with_grad: 2 w and grad staged in LDS, 1 grad in LDS, 0 global;
                             // else: >= 1 w staged in LDS, 0 global
    int32_t wide;
    int32_t with_grad;       // accumulate the (weight-independent) trivial-word gradient
    int32_t no_slice;        // skip edge_weight_slice (nothing after this launch reads it)
    int32_t no_streams;      // bubbles only (the pipelined QN loop's update chain): no table
                             // staging, no stream pass, no per-edge weight slice
    // bub_on: the stream waves also evaluate the bubbles before their
    // streams (no separate bubble kernel) -- the small ones one per lane from
    // the first waves, the big ones one per wavefront from the last
    BubbleArgs bub;
    int32_t bub_on;
    int32_t multi;           // the automaton has multi-parameter (epsilon-composite) edges
    const double* w;         // [n_params] w_full (GetWeight form)
    double* grad;            // [n_params] (TABLES == 0: atomics straight into it)
    double* gpart;           // [grid][n_params] per-block partial gradients (TABLES >= 1)
    // prologue work folded into this launch when TABLES >= 1 (no other kernel
    // then runs before it): per-edge weights of all combined edges and the
    // zeroing of the result vector
    int64_t n_comb;          // E + X
    double* lw_out;
    double* ew_out;
    EdgeRec* erec_out;
    double* out;             // [1 + n_params], zeroed by block 0
    double* ll_part;         // [waves in grid] (per-iteration stream kernel: [blocks])
    double* logq;            // [S] or null
    const unsigned* halted;  // device-resident QN run: nonzero = skip (or null)
    QnFinish fin;            // fin.active: block 0 finishes the previous QN step first
    QnWave qw;               // qw.on: this step's QN update runs in this launch
    RminFold rf;             // rf.part: the rmin column folded into this launch (with qw.on)
    unsigned long long* trace;   // timing experiments only (WFSA_FBS_TRACE): [waves][8] s_memrealtime stamps
};


// The per-iteration reduction, one launch, deterministic: parameters in
// slot order are cut into tiles (consecutive positions, bounded slots); a
// block per tile adds to out[1 + j] the constant trivial-word gradient (when
// `fixed` is given) and the fixed-order sum of j's bubble contribution slots
// (seg_sums, qn_device.hpp); one more block writes out[0] = the sum of the
// log-likelihood partials in a fixed order.  No atomics: the same inputs give
// the same bits on every launch.

constexpr int kReduceBlock = 256;
constexpr int kReduceTileParams = 1024;
// The bubble contribution slots of a parameter are summed in chunks of
// kSlotChunk (seg_sums, qn_device.hpp); a reduction group's chunk sums fit in
// LDS up to kMaxChunks (a run-of-positions group is cut to fit).
constexpr int kSlotChunk = 16;
constexpr int kMaxChunks = 1024;
struct ReduceArgs {
    const double* contrib;       // bubble contribution slots, or null
    const int64_t* grp_base;     // [n_tiles + 1] physical slot base of each group (chunk-transposed)
    const int32_t* seg_ptr;      // [n_pos + 1] logical slot run of the parameter at each position
    const int32_t* chunk_ptr;    // [n_pos + 1] its chunks (cumulative)
    const int32_t* param_at;     // [n_pos] full parameter index at each position
    const int32_t* tile_ptr;     // [n_tiles + 1] position range of each reduction group
    int32_t n_tiles;
    const double* fixed;         // [n_params] added when non-null
    const double* ll_part;
    int32_t n_ll;
    double* out;                 // [1 + n_params]
    const unsigned* halted;
};
// Completion without a DMA copy or a stream synchronisation: a one-block
// kernel copies out[0, n) into host-mapped memory (adding `add` to out[1..]
// when given), fences at system scope and then stores the next sequence
// number into a host-mapped flag the host polls.
struct Publish {
    double* host_out;            // host-mapped [n rounded up to even]
    int32_t n;
    const double* add;           // [n - 1] added to out[1 ..] (the all-reduced constant gradient), or null
    unsigned* seq;               // device sequence counter
    unsigned* host_flag;         // host-mapped: last published sequence number
};

// sum of p[t], p[t + nt], p[t + 2 nt], ... below n, in that order, with the
// loads issued eight at a time (a plain strided loop waits on every load)
__device__ __forceinline__ double strided_sum(const double* __restrict__ p, int n, int t, int nt) {
    double s = 0.0;
    for (int i0 = t; i0 < n; i0 += 8 * nt) {
        double v[8];
#pragma unroll
        for (int b = 0; b < 8; ++b) v[b] = p[min(i0 + b * nt, n - 1)];
#pragma unroll
        for (int b = 0; b < 8; ++b)
            if (i0 + b * nt < n) s += v[b];
    }
    return s;
}

hipError_t configure_kernels(int max_dynamic_lds);
hipError_t launch_trav(TravMode mode, const TravArgs& a, int grid, hipStream_t stream);
hipError_t launch_stream_headers(uint4* stream, const int64_t* g_base, const int32_t* g_len, const double* p_lane,
                                int32_t n_groups, int32_t wide, hipStream_t s);
// ev0 / ev1 (optional, timing events): the stream kernel's dispatch start and
// end (hipExtLaunchKernel's profiling timestamps, the launch gap excluded)
hipError_t launch_compiled(const CompiledArgs& a, int grid, int block, size_t lds, hipStream_t stream,
                           hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr);
constexpr int kBubbleBlock = 128;
// waves: n_big (one per big bubble) + ceil(n_small / 64)
// Small bubbles run 64 to a wavefront: the class-A chunks first (the last
// one partial), then the class-B chunks from list entry n4 on -- so no
// wavefront holds both classes (a mixed one ran both code paths, twice a
// wave's time, and was the launch's last bubble arrival, profiles/r05).
// Chunk c, lane l -> small-list entry b (class A: b < n4, class B: b >= n4),
// or -1 for an idle lane; b is also the bubble's position (rmin, the slot
// layout's lane groups, which are aligned within each class's chunks)
__host__ __device__ inline int64_t small_chunks(int64_t n4, int64_t ns) { return (n4 + 63) / 64 + (ns + 63) / 64; }
__host__ __device__ inline int64_t small_entry(int64_t c, int l, int64_t n4, int64_t ns) {
    const int64_t na = (n4 + 63) / 64;
    if (c < na) {
        const int64_t b = c * 64 + l;
        return b < n4 ? b : -1;
    }
    const int64_t b = n4 + (c - na) * 64 + l;
    return b < n4 + ns ? b : -1;
}
int bubble_waves(int32_t n_small4, int32_t n_small, int32_t n_big);
// blocks of the stream kernel with the in-kernel QN update that one CU holds
// at once (block threads, dynamic LDS bytes); 0 on error
int fbs_qn_blocks_per_cu(int block, size_t lds);
hipError_t launch_bubbles(const BubbleArgs& a, hipStream_t stream);
hipError_t launch_reduce(const ReduceArgs& a, hipStream_t stream);
// out[1 + j] = sum over k of gpart[k][j] in k order (the preparation-time gradient slabs)
hipError_t launch_slab_sum(const double* gpart, int32_t n_slabs, int32_t n_params, double* out, hipStream_t stream);
// out[0, n) -> host-mapped memory, then the flag (one block)
hipError_t launch_publish(const double* out, const Publish& pub, hipStream_t stream);
// host-mapped weights w[0, n) and the zero slot w[n] -> device, with
// ewp = exp(w) (all buffers padded to an even count)
hipError_t launch_stage(const double* host_w, double* w, double* ewp, int32_t n, hipStream_t stream);
// fused: the member gradients include the bubble slot sums (every constraint
// has at most kQnMaxSeg members); grid max(k, 1)
hipError_t launch_qn_step(const QnArgs& a, bool fused, hipStream_t stream);
// dst[i] = src[idx[i]], i < n
hipError_t launch_gather(const double* src, const int32_t* idx, int32_t n, double* dst, hipStream_t stream);
// a step's finish as its own one-block launch
hipError_t launch_qn_finish(const QnFinish& f, hipStream_t stream);
hipError_t launch_qn_weights(const double* x, const int32_t* trim, int32_t n_full, double* w_full, double* ewp,
                             hipStream_t stream);
// n doubles src -> dst by a kernel (host-mapped memory on either side: no
// staging copy of pageable memory)
hipError_t launch_copy(const double* src, double* dst, int64_t n, hipStream_t stream);
hipError_t launch_edge_weights(const double* w_full, const int32_t* pptr, const int32_t* pidx, double* lw,
                               double* ew, EdgeRec* erec, int64_t n_edges, double* out, int64_t n_out,
                               hipStream_t stream);
hipError_t launch_node_end(const int32_t* x_ptr, const double* x_w, double* node_end, int32_t n_nodes,
                           hipStream_t stream);

}  // namespace wfsa
