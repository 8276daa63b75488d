// Dense-automaton forward-backward on fp64 MFMA (see dense_path.hpp).
//
// Per evaluation, on one stream:
//   dense_weights   exp(w) tables: A (np x np), E^T ((V+1) x np), start and
//                   end vectors; zeroes the result vector
//   gemm<FWD>  x T  alpha[t+1] = (alpha[t] / rowsum) A (.) E[sym]  (row slots
//                   that start a string take a (.) E[sym] instead)
//   dense_final     log q per string, p . log q partials
//   gemm<BWD>  x T  beta[t] = (Y[t+1] / rowsum) A^T, or e where a string ends;
//                   writes Y[t] = E[sym] (.) beta[t], z[t] (Y scaled for the
//                   gradient GEMM) and gamma[t] = alpha beta / q (scaled)
//   gemm<GRAD>      G = alpha[0..T-2]^T z[1..T-1]; grad(S->T) = -A (.) G
//   dense_reduce    gamma summed per (emitted symbol, state), per start and
//                   end state, in fixed row chunks
//   dense_scatter   chunk sums -> the emission / start / end gradients, LL
// Every sum runs in a fixed order: results are deterministic.
//
// GEMM: 256 threads, 128 x 128 block tile, 64 x 64 per wavefront (4 x 4
// tiles of v_mfma_f64_16x16x4f64), K staged through LDS in slices of 16,
// double-buffered; operands are stored in LDS as [row][k] with a 2-double pad
// (a fragment read of 64 lanes is bank-conflict free).  Blocks are dealt so
// that each XCD owns a contiguous range of tiles (column panels shared in its
// L2).
#include "dense_path.hpp"

#include <rocblas/rocblas.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <numeric>
#include <queue>
#include <string>

namespace wfsa {

namespace {

typedef double d4 __attribute__((ext_vector_type(4)));
// staging registers of the operand slices: a native vector, not HIP's double2
// class (whose assignment is a struct memcpy that SROA leaves in scratch: the
// prefetch then went through scratch stores waited for right after issue)
typedef double d2 __attribute__((ext_vector_type(2)));

constexpr int kT = kDenseTile;        // 128
// K slice per LDS stage: 32 for the per-step GEMMs (one block per CU, the
// longer slice hides the slice-boundary barrier), 16 for the gradient GEMM
// (two blocks per CU)
constexpr int kBkStep = 32, kBkGrad = 16;
// waves per block: 8 for the per-step GEMMs (one block per CU: two waves per
// SIMD hide each other's LDS and barrier time), 4 for the gradient GEMM (two
// blocks per CU do that)
constexpr int kNwStep = 8, kNwGrad = 4;
// engine 2's step GEMMs: K in two halves, 4-wave blocks, slices of 16 --
// twice the blocks of a step's tile grid, two per CU (the gradient GEMM's shape)
constexpr int kSplitK = 2;
// LDS images of an operand slice (128 rows r x BK k), never transposed on
// the way in, so every store is a plain conflict-free 16-byte write:
//  * KC (the operand's rows contiguous along k in memory): [r][k], padded
//    row of BK + 1 doubles: the compiler pairs a fragment's reads for kk and
//    kk + 1 into ds_read2_b64, banked per 16 lanes mod 32 dwords, where an
//    odd pitch puts the 16 rows on distinct bank pairs (round 3's BK + 2,
//    conflict-free for single ds_read_b64, left a third of the A reads'
//    LDS cycles in conflicts: SQ_LDS_BANK_CONFLICT, profiles/r04/
//    gemm_pmc.txt); the pitch is odd, so its stores are 8 bytes wide;
//  * RC (memory rows run along r): [k][r], padded row of kLdn = 144
//    doubles (2 kLdn == 32 mod 64: the fragment read's two k rows of a
//    32-lane group fall on the two bank halves).
// (Round 2's kernels stored RC slices transposed into [r][k]: 8-byte
// stores four-way conflicted, a burst at every slice end while the MFMA
// pipe idled -- 0.67 of the fp64 peak.)
#ifdef WFSA_GEMM_LDK_EVEN   // (layout-variant builds: round 3's padding)
template <int BK> constexpr int ldk() { return BK + 2; }
#else
template <int BK> constexpr int ldk() { return BK + 1; }
#endif
constexpr int kLdn = kDenseTile + 16;
template <bool KC, int BK> constexpr int op_size() { return KC ? kT * ldk<BK>() : BK * kLdn; }
template <int MODE, int BK> constexpr int stage();   // doubles per stage (A and B), below
constexpr int kRedThreads = 128;      // dense_reduce: one column per thread
// row pitch of the row-slot buffers = np + 16 doubles: a 128-row tile read
// along k then spreads over memory channels and L2 sets (a power-of-two pitch
// puts every row of the tile on the same ones)
constexpr int kRowPad = 16;
constexpr int kRedWindow = 64;        // symbols per LDS pass of dense_reduce
#ifndef WFSA_RED_BATCH   // (variant builds: batch sizes)
#define WFSA_RED_BATCH 32
#endif
#ifndef WFSA_EPI_BATCH
#define WFSA_EPI_BATCH 4
#endif
constexpr int kRedBatch = WFSA_RED_BATCH;   // dense_reduce: rows whose loads are in flight together (batch 8 / 16 / 32: 4.35 -> 1.68 / 1.27 / 1.12 ms per c5 evaluation)
constexpr int kEpiBatch = WFSA_EPI_BATCH;   // epilogues: columns per thread loaded before the stores (29.1 / 47.7 -> 24.7 / 45.5 us)

// RAW: a plain product (the forward's or the backward's operand layouts)
// into out (K split s: into out2 for s = 1), the epilogue left to the
// epilogue kernels -- split-K gives the 256-tile step GEMMs two blocks per CU
enum GemmMode { FWD = 0, BWD = 1, GRAD = 2, RAW = 3 };

struct GemmArgs {
    int32_t R, np, nct;
    int32_t ldx;               // row pitch of the row-slot buffers (alpha, Y, z, gamma)
    int64_t kg;                // GRAD: K = (T - 1) R
    const double* x;           // FWD alpha[t] / BWD Y[t+1] / GRAD alpha (steps 0..T-2)
    const double* bm;          // FWD, BWD: A / GRAD: z from step 1
    int32_t no_mma;            // every row of the step starts (FWD) / ends (BWD) a string
    const int32_t* meta;       // [R] meta of the output step
    const int32_t* sid;        // [R] (BWD)
    const double* part_in;     // [nct][R] row-sum partials of the input rows
    double* part_out;          // [nct][R] of the output rows
    const double* et;          // [(V+1)][np]
    const double* a0;
    const double* aend;
    double* out;               // FWD alpha[t+1] / BWD Y[t]
    const double* la_in;       // FWD la[t]
    double* la_out;            // FWD la[t+1]
    const double* lb_in;       // BWD lb[t+1]
    double* lb_out;            // BWD lb[t]
    const double* la_t;        // BWD la[t]
    const double* la_prev;     // BWD la[t-1] or null
    const double* alpha_t;     // BWD alpha[t]
    double* gam;               // BWD gamma[t]
    double* z;                 // BWD z[t]
    const double* p;
    const double* logq;
    const int32_t* code_a;     // GRAD
    const double* amat;
    double* grad;              // GRAD: out + 1
    int32_t n_params;
    const unsigned* halted;
    double* out2;              // RAW: the second K half's product
    int32_t splits;            // RAW: K halves (1 or 2); else 1
};

// Global -> registers -> LDS staging of one 128 x 16 operand slice.  KC: the
// operand's row r is contiguous along k (element (r, k) at base[r ld + k]);
// RC: rows of memory run along the operand's rows (element (r, k) at
// base[k ld + r]).  LDS holds KC slices as [r][k], RC slices as [k][r].
// chunks of 16 bytes per thread for one 128 x BK slice
template <int BK, int NT> constexpr int slice_chunks() { return kT * BK / 2 / NT; }

template <bool KC, int BK, int NT>
__device__ __forceinline__ void load_slice(const double* __restrict__ base, int64_t ld, int r0, int64_t k0, int tid,
                                           d2 (&v)[slice_chunks<BK, NT>()]) {
    constexpr int kPairs = BK / 2;   // 16-byte chunks per row of the slice
#pragma unroll
    for (int c = 0; c < slice_chunks<BK, NT>(); ++c) {
        const int idx = c * NT + tid;
        if (KC) {
            const int row = idx / kPairs, kp = idx % kPairs;
            v[c] = *reinterpret_cast<const d2*>(base + int64_t(r0 + row) * ld + k0 + 2 * kp);
        } else {
            const int kk = idx >> 6, rp = idx & 63;
            v[c] = *reinterpret_cast<const d2*>(base + (k0 + kk) * ld + r0 + 2 * rp);
        }
    }
}

template <bool KC, int BK, int NT>
__device__ __forceinline__ void store_slice(double* __restrict__ s, int tid, const d2 (&v)[slice_chunks<BK, NT>()]) {
    constexpr int kPairs = BK / 2, L = ldk<BK>();
#pragma unroll
    for (int c = 0; c < slice_chunks<BK, NT>(); ++c) {
        const int idx = c * NT + tid;
        if (KC) {   // (an odd row pitch: 8-byte stores)
            const int row = idx / kPairs, kp = idx % kPairs;
            s[row * L + 2 * kp] = v[c].x;
            s[row * L + 2 * kp + 1] = v[c].y;
        } else {
            const int kk = idx >> 6, rp = idx & 63;
            *reinterpret_cast<d2*>(s + kk * kLdn + 2 * rp) = v[c];
        }
    }
}

template <int MODE, int BK> constexpr int stage() { return op_size<MODE != 2, BK>() + op_size<false, BK>(); }

// NW waves per 128 x 128 block: 2 x (NW / 2), each a 64 x (256 / NW) tile
// of 16 x 16 MFMA tiles (NJ of them per row of tiles)
template <int MODE, int BK, int NW>
__global__ __launch_bounds__(NW * 64, ((MODE == GRAD || MODE == RAW) && (NW == 4 || NW == 8) && BK == 16 ? 2 : 1)) void dense_gemm_kernel(GemmArgs a) {
    if (a.halted && *a.halted) return;
    constexpr int NT = NW * 64, NWN = NW / 2, NJ = 16 / NW, WCOLS = 16 * NJ;
    constexpr int kLdk = ldk<BK>(), kStage = stage<MODE, BK>();
    constexpr int CH = slice_chunks<BK, NT>();
    __shared__ __attribute__((aligned(16))) double lds[2 * kStage];
    __shared__ double red[NWN][kT];
    __shared__ double rs0[kT], rs1[kT], rs2[kT];
    __shared__ int32_t rmeta[kT];

    constexpr bool A_KC = MODE != GRAD;   // FWD / BWD: x rows are contiguous along k
    constexpr bool B_KC = false;          // FWD: A, BWD: A^T (stored), GRAD: z -- all along memory rows
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / NWN, wn = wave % NWN;
    const int np = a.np, ldx = a.ldx;
    const int mtiles = (MODE == GRAD ? np : a.R) / kT, ntiles = np / kT;
    const int nb = mtiles * ntiles, splits = MODE == RAW ? a.splits : 1, total = nb * splits;
    int bid = int(blockIdx.x);
    if ((total & 7) == 0) bid = (bid & 7) * (total >> 3) + (bid >> 3);   // XCD x: tiles [x total/8, (x+1) total/8)
    const int sidx = bid / nb, tile = bid % nb;   // (RAW: K half sidx)
    const int mt_ = tile % mtiles, nt_ = tile / mtiles;
    const int r0 = mt_ * kT, c0 = nt_ * kT;

    // per-row scalars of the block's output rows (read by the epilogue)
    auto row_scalars = [&]() {
    if ((MODE == FWD || MODE == BWD) && tid < kT) {
        const int r = r0 + tid;
        const int m = a.meta[r];
        const bool start = (m >> 9) & 1, end = (m >> 10) & 1;
        if (MODE == FWD) {
            double inv = 0.0, la = 0.0;
            if (!a.no_mma) {
                double s = 0.0;
                for (int ct = 0; ct < a.nct; ++ct) s += a.part_in[int64_t(ct) * a.R + r];
                inv = s > 0.0 ? 1.0 / s : 0.0;
                la = start ? 0.0 : a.la_in[r] + log(s);
            }
            rs0[tid] = inv;
            if (nt_ == 0) a.la_out[r] = la;
        } else {
            double inv = 0.0, lb = 0.0;
            if (!end && !a.no_mma) {
                double u = 0.0;
                for (int ct = 0; ct < a.nct; ++ct) u += a.part_in[int64_t(ct) * a.R + r];
                inv = u > 0.0 ? 1.0 / u : 0.0;
                lb = a.lb_in[r] + log(u);
            }
            if (nt_ == 0) a.lb_out[r] = lb;
            double f1 = 0.0, f2 = 0.0;
            const int s = a.sid[r];
            if (s >= 0) {
                const double lq = a.logq[s];
                if (lq > -INFINITY) {
                    f1 = a.p[s] * exp(a.la_t[r] + lb - lq);
                    if (!start && a.la_prev) f2 = a.p[s] * exp(a.la_prev[r] + lb - lq);
                }
            }
            rs0[tid] = inv;
            rs1[tid] = f1;
            rs2[tid] = f2;
        }
        rmeta[tid] = m;
    }
    };

    d4 acc[4][NJ];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = d4{0.0, 0.0, 0.0, 0.0};

    if (!a.no_mma) {
        const int64_t klen = (MODE == GRAD ? a.kg : int64_t(np)) / splits, kofs = int64_t(sidx) * klen;
        const int64_t nk = klen / BK;
        const double* xa = a.x;
        const double* xb = a.bm;
        d2 va[CH], vb[CH];
        const int ldb = MODE == GRAD ? ldx : np;   // z / A, A^T
        load_slice<A_KC, BK, NT>(xa, ldx, r0, kofs, tid, va);
        load_slice<B_KC, BK, NT>(xb, ldb, c0, kofs, tid, vb);
        row_scalars();   // its loads overlap the first slice's
        store_slice<A_KC, BK, NT>(lds, tid, va);
        store_slice<B_KC, BK, NT>(lds + op_size<A_KC, BK>(), tid, vb);
        __syncthreads();
        for (int64_t kt = 0; kt < nk; ++kt) {
            const bool more = kt + 1 < nk;
            if (more) {
                load_slice<A_KC, BK, NT>(xa, ldx, r0, kofs + (kt + 1) * BK, tid, va);
                load_slice<B_KC, BK, NT>(xb, ldb, c0, kofs + (kt + 1) * BK, tid, vb);
            }
            const double* As = lds + (kt & 1) * kStage;
            const double* Bs = As + op_size<A_KC, BK>();
            // a wave's fragments of k-step kk: 4 A values (its 64 rows) and NJ B values
            auto frag = [&](int kk, double (&av)[4], double (&bv)[NJ]) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    av[i] = A_KC ? As[(wm * 64 + i * 16 + (lane & 15)) * kLdk + kk * 4 + (lane >> 4)]
                                 : As[(kk * 4 + (lane >> 4)) * kLdn + wm * 64 + i * 16 + (lane & 15)];
#pragma unroll
                for (int j = 0; j < NJ; ++j) bv[j] = Bs[(kk * 4 + (lane >> 4)) * kLdn + wn * WCOLS + j * 16 + (lane & 15)];
            };
#ifdef WFSA_GEMM_FRAG_PF
            double fa[2][4], fb[2][NJ];
#endif
#pragma unroll
            for (int kk = 0; kk < BK / 4; ++kk) {
                // the next slice into the other stage half-way through this
                // one (its loads have landed by then; every wave finished
                // reading that stage before the last barrier): the stores
                // then overlap this wave's MFMAs instead of idling the matrix
                // pipe before the barrier
#ifdef WFSA_GEMM_STORE_END   // (layout-variant builds: the stores after the slice's MFMAs)
                if (kk == BK / 4 - 1 && more) {
#else
                if (kk == BK / 8 && more) {
#endif
                    double* s = lds + ((kt + 1) & 1) * kStage;
                    store_slice<A_KC, BK, NT>(s, tid, va);
                    store_slice<B_KC, BK, NT>(s + op_size<A_KC, BK>(), tid, vb);
                }
#ifdef WFSA_GEMM_FRAG_PF   // (variant builds: fragments of k-step kk + 1 read before kk's MFMAs)
                if (kk == 0) frag(0, fa[0], fb[0]);
                if (kk + 1 < BK / 4) frag(kk + 1, fa[(kk + 1) & 1], fb[(kk + 1) & 1]);
                double (&av)[4] = fa[kk & 1];
                double (&bv)[NJ] = fb[kk & 1];
#else
                double av[4], bv[NJ];
                frag(kk, av, bv);
#endif
#ifndef WFSA_GEMM_NOPRIO   // (MFMA clusters at raised priority: 537 -> 528 us per step GEMM, profiles/r04/gemm_variants.txt)
                __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < NJ; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[i], bv[j], acc[i][j], 0, 0, 0);
#ifndef WFSA_GEMM_NOPRIO
                __builtin_amdgcn_s_setprio(0);
#endif
            }
            __syncthreads();
        }
    } else {
        row_scalars();
        __syncthreads();
    }

    // epilogue: element (i, j, e) of this lane is row wm*64 + 16 i + (lane>>4)
    // + 4 e, column wn*WCOLS + 16 j + (lane & 15) of the block tile
    if (MODE == RAW) {   // the raw product (4 rows x 16 columns = 128-byte runs per store)
        double* o = sidx ? a.out2 : a.out;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int row = r0 + wm * 64 + 16 * i + (lane >> 4) + 4 * e;
                    const int col = c0 + wn * WCOLS + 16 * j + (lane & 15);
                    o[int64_t(row) * ldx + col] = acc[i][j][e];
                }
        return;
    }
    if (MODE == GRAD) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int row = r0 + wm * 64 + 16 * i + (lane >> 4) + 4 * e;
                    const int col = c0 + wn * WCOLS + 16 * j + (lane & 15);
                    const int64_t o = int64_t(row) * np + col;
                    const int32_t code = a.code_a[o];
                    if (code >= 0 && code < a.n_params) a.grad[code] = -a.amat[o] * acc[i][j][e];
                }
        return;
    }
    double rsum[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) rsum[i][e] = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int rl = wm * 64 + 16 * i + (lane >> 4) + 4 * e;
            const int row = r0 + rl;
            const int m = rmeta[rl];
            const int sym = m & 511;
            const double* erow = a.et + int64_t(sym) * np;
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int col = c0 + wn * WCOLS + 16 * j + (lane & 15);
                const int64_t o = int64_t(row) * ldx + col;
                double v;
                if (MODE == FWD) {
                    v = ((m >> 9) & 1) ? a.a0[col] : acc[i][j][e] * rs0[rl];
                    v *= erow[col];
                    a.out[o] = v;
                } else {
                    const double beta = ((m >> 10) & 1) ? a.aend[col] : acc[i][j][e] * rs0[rl];
                    a.gam[o] = a.alpha_t[o] * beta * rs1[rl];
                    v = erow[col] * beta;
                    a.out[o] = v;
                    a.z[o] = v * rs2[rl];
                }
                rsum[i][e] += v;
            }
        }
    // row sums over the tile's 128 columns: 16 lanes per row, then the
    // NWN column groups (wn) through LDS
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            double v = rsum[i][e];
            v += __shfl_xor(v, 1);
            v += __shfl_xor(v, 2);
            v += __shfl_xor(v, 4);
            v += __shfl_xor(v, 8);
            if ((lane & 15) == 0) red[wn][wm * 64 + 16 * i + (lane >> 4) + 4 * e] = v;
        }
    __syncthreads();
    if (tid < kT) {
        double v = red[0][tid];
#pragma unroll
        for (int g = 1; g < NWN; ++g) v += red[g][tid];
        a.part_out[int64_t(nt_) * a.R + r0 + tid] = v;
    }
}

struct WeightsArgs {
    const double* ewp;          // exp(w_full) (or all ones)
    const int32_t* code_a;
    const int32_t* code_em;
    const int32_t* code_s;
    const int32_t* code_e;
    double* amat;
    double* et;
    double* a0;
    double* aend;
    int64_t n_a, n_em;
    int32_t np;
    double* out;                // [1 + n_params] zeroed
    int32_t n_out;
    const unsigned* halted;
};

__device__ __forceinline__ double code_weight(const double* ewp, int32_t c) {
    return c >= 0 ? ewp[c] : (c == kCodeOne ? 1.0 : 0.0);
}

__global__ __launch_bounds__(256) void dense_weights_kernel(WeightsArgs a) {
    if (a.halted && *a.halted) return;
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    const int64_t t0 = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    for (int64_t i = t0; i < a.n_a; i += stride) a.amat[i] = code_weight(a.ewp, a.code_a[i]);
    for (int64_t i = t0; i < a.n_em; i += stride) a.et[i] = code_weight(a.ewp, a.code_em[i]);
    for (int64_t i = t0; i < a.np; i += stride) {
        a.a0[i] = code_weight(a.ewp, a.code_s[i]);
        a.aend[i] = code_weight(a.ewp, a.code_e[i]);
    }
    for (int64_t i = t0; i < a.n_out; i += stride) a.out[i] = 0.0;
}

// A^T for the backward GEMM (its B operand then streams along rows of
// memory like the forward GEMM's): 32 x 32 tiles through LDS
__global__ __launch_bounds__(256) void dense_transpose_kernel(const double* __restrict__ a, double* __restrict__ at,
                                                              int32_t np, const unsigned* halted) {
    if (halted && *halted) return;
    __shared__ double tile[32][33];
    const int bx = blockIdx.x * 32, by = blockIdx.y * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
#pragma unroll
    for (int k = 0; k < 32; k += 8) tile[ty + k][tx] = a[int64_t(by + ty + k) * np + bx + tx];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 32; k += 8) at[int64_t(bx + ty + k) * np + by + tx] = tile[tx][ty + k];
}

struct FinalArgs {
    const double* alpha;        // [T][R][np]
    const double* la;           // [T][R]
    const double* aend;
    const int32_t* end_at;      // [S]
    const double* p;
    const double* ewp;
    int32_t code_se;
    int64_t n_strings;
    int32_t np, ldx;
    double* logq;               // [S]
    double* logq_user;          // [S] or null
    double* ll_part;            // [blocks]
    const unsigned* halted;
};

// one wavefront per string: log q = la + log(alpha_L . e)
__global__ __launch_bounds__(256) void dense_final_kernel(FinalArgs a) {
    if (a.halted && *a.halted) return;
    __shared__ double wsum[4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t s = int64_t(blockIdx.x) * 4 + w;
    double contrib = 0.0;
    if (s < a.n_strings) {
        const int32_t at = a.end_at[s];
        double lq;
        if (at >= 0) {
            const double* row = a.alpha + int64_t(at) * a.ldx;
            double d = 0.0;
            for (int c = lane; c < a.np; c += 64) d += row[c] * a.aend[c];
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) d += __shfl_xor(d, o);
            lq = a.la[at] + log(d);
        } else {
            lq = log(code_weight(a.ewp, a.code_se));
        }
        if (lane == 0) {
            a.logq[s] = lq;
            if (a.logq_user) a.logq_user[s] = lq;
        }
        contrib = a.p[s] > 0.0 ? a.p[s] * lq : 0.0;
    }
    if (lane == 0) wsum[w] = contrib;
    __syncthreads();
    if (threadIdx.x == 0) a.ll_part[blockIdx.x] = ((wsum[0] + wsum[1]) + wsum[2]) + wsum[3];
}

struct ReduceArgs {
    const double* gam;          // [T R][np]
    const int32_t* meta;        // [T R]
    int64_t rows;               // T R
    int64_t rows_per_chunk;
    int32_t np, vocab, ldx;
    double* red;                // [chunks][vocab + 2][np]
    const unsigned* halted;
};

// gamma rows of chunk blockIdx.y, columns [128 blockIdx.x, +128): sums per
// emitted symbol, per start row (-> ^->T) and per end row (-> S->$)
__global__ __launch_bounds__(kRedThreads) void dense_reduce_kernel(ReduceArgs a) {
    if (a.halted && *a.halted) return;
    __shared__ double acc[(kRedWindow + 2) * kRedThreads];
    const int t = threadIdx.x;
    const int col = int(blockIdx.x) * kRedThreads + t;
    const int64_t rbeg = int64_t(blockIdx.y) * a.rows_per_chunk;
    const int64_t rend = min(a.rows, rbeg + a.rows_per_chunk);
    const int V = a.vocab;
    double* outp = a.red + int64_t(blockIdx.y) * (V + 2) * a.np;
    for (int vb = 0; vb < V || vb == 0; vb += kRedWindow) {
        const int wv = min(kRedWindow, V - vb);
        for (int k = 0; k < kRedWindow + 2; ++k) acc[k * kRedThreads + t] = 0.0;
        double st = 0.0, en = 0.0;
        auto add = [&](int m, double g) {
            const int sym = m & 511;
            if (sym >= V) return;   // idle slot
            const int k = sym - vb;
            if (k >= 0 && k < wv) acc[k * kRedThreads + t] += g;
            if (vb == 0) {
                if ((m >> 9) & 1) st += g;
                if ((m >> 10) & 1) en += g;
            }
        };
        int64_t r = rbeg;
        for (; r + kRedBatch <= rend; r += kRedBatch) {   // a batch of rows' loads in flight, then the adds in row order
            int mb[kRedBatch];
            double gb[kRedBatch];
#pragma unroll
            for (int u = 0; u < kRedBatch; ++u) {
                mb[u] = a.meta[r + u];
                gb[u] = a.gam[(r + u) * a.ldx + col];   // (an idle slot's row is read and skipped)
            }
#pragma unroll
            for (int u = 0; u < kRedBatch; ++u) add(mb[u], gb[u]);
        }
        for (; r < rend; ++r) add(a.meta[r], a.gam[r * a.ldx + col]);
        for (int k = 0; k < wv; ++k) outp[int64_t(vb + k) * a.np + col] = acc[k * kRedThreads + t];
        if (vb == 0) {
            outp[int64_t(V) * a.np + col] = st;
            outp[int64_t(V + 1) * a.np + col] = en;
        }
        if (V == 0) break;
    }
}

struct ScatterArgs {
    const double* red;          // [chunks][vocab + 2][np]
    int32_t chunks;
    int32_t np, vocab;
    const int32_t* code_em;     // [vocab + 1][np]
    const int32_t* code_s;
    const int32_t* code_e;
    int32_t code_se;
    int32_t n_params;
    double empty_p;             // sum of p over empty strings (posterior 1 on ^->$)
    const double* ll_part;
    int32_t n_ll;
    double* out;                // [1 + n_params]
    const unsigned* halted;
};

__global__ __launch_bounds__(256) void dense_scatter_kernel(ScatterArgs a) {
    if (a.halted && *a.halted) return;
    const int64_t n = int64_t(a.vocab + 2) * a.np;
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n) {
        const int slot = int(i / a.np), col = int(i % a.np);
        double s = 0.0;
        for (int c = 0; c < a.chunks; ++c) s += a.red[(int64_t(c) * (a.vocab + 2) + slot) * a.np + col];
        const int32_t code =
            slot < a.vocab ? a.code_em[int64_t(slot) * a.np + col] : (slot == a.vocab ? a.code_s[col] : a.code_e[col]);
        if (code >= 0 && code < a.n_params) a.out[1 + code] = -s;
    }
    if (i == 0) {
        double ll = 0.0;
        for (int b = 0; b < a.n_ll; ++b) ll += a.ll_part[b];
        a.out[0] = ll;
        if (a.code_se >= 0 && a.code_se < a.n_params) a.out[1 + a.code_se] = -a.empty_p;
    }
}

// ---- the staged-pipeline GEMM (engine 3) -----------------------------------
// One 4-wave block per 128 x 128 tile (64 x 64 per wave), K in slices of 16
// moved global -> LDS by global_load_lds_dwordx4 (LDS-DMA: no staging
// registers, no LDS store instructions) into four LDS stages, three slices
// ahead.  Each wave waits (counted vmcnt, never 0 in the loop) for its own
// pieces of the next slice half-way through the current one, then a raw
// s_barrier -- past it every wave's pieces of that slice are in LDS and every
// wave has finished the slice before, whose stage the next issue refills.
// The LDS images are lane-linear per 1 KiB DMA piece:
//  * [k][r] rows of 144 doubles for an operand whose memory rows run along r
//    (B always; A in the gradient GEMM) -- one piece per k row;
//  * [r][k] rows of 16 doubles for the step GEMMs' A (alpha / Y rows run
//    along k): 16-byte chunk c of row r stored at chunk c ^ ((r >> 1) & 7) --
//    the permutation applied to the pieces' global source addresses and
//    undone by the fragment reads, so a fragment read (16 rows x 2 k per
//    32 lanes) touches 64 distinct banks.
// Epilogue: RAW the plain product into out; GRADEPI the gradient's scatter
// -A (.) G by parameter code (as dense_gemm_kernel<GRAD>).
constexpr int kMmBK = 16, kMmStages = 4;
constexpr int kMmKc = kT * kMmBK;     // doubles of a swizzled [r][k] image
constexpr int kMmRc = kMmBK * kLdn;   // doubles of a padded [k][r] image
template <bool AKC> constexpr int mm_stage() { return (AKC ? kMmKc : kMmRc) + kMmRc; }
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

template <bool AKC, bool GRADEPI>
__global__ __launch_bounds__(256, 1) void dense_mm_kernel(GemmArgs a) {
    if (a.halted && *a.halted) return;
    constexpr int kStage = mm_stage<AKC>(), kBOff = AKC ? kMmKc : kMmRc;
    __shared__ __attribute__((aligned(16))) double lds[kMmStages * kStage];
    const int tid = int(threadIdx.x), lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int np = a.np, ldx = a.ldx;
    const int mtiles = (GRADEPI ? np : a.R) / kT, ntiles = np / kT, nb = mtiles * ntiles;
    int bid = int(blockIdx.x);
    if ((nb & 7) == 0) bid = (bid & 7) * (nb >> 3) + (bid >> 3);   // XCD x: tiles [x nb/8, (x+1) nb/8)
    const int mt_ = bid % mtiles, nt_ = bid / mtiles;
    const int r0 = mt_ * kT, c0 = nt_ * kT;
    const int nk = int((GRADEPI ? a.kg : int64_t(np)) / kMmBK);
    const int ldb = GRADEPI ? ldx : np;   // z / A, A^T
    const double* xa = a.x;
    const double* xb = a.bm;
    // slice s into stage s % 4: 4 A pieces and 4 B pieces of 1 KiB per wave
    auto issue = [&](int s) {
        double* st = lds + (s % kMmStages) * kStage;
        const int64_t k0 = int64_t(s) * kMmBK;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int q = wave * 4 + i;
            const double* ga;
            double* la;
            if (AKC) {   // rows 8q .. 8q + 7; lane l fills chunk l % 8 of row 8q + l / 8
                const int row = 8 * q + (lane >> 3);
                const int c = (lane & 7) ^ ((row >> 1) & 7);
                ga = xa + int64_t(r0 + row) * ldx + k0 + 2 * c;
                la = st + q * 128;
            } else {     // k row q
                ga = xa + (k0 + q) * ldx + r0 + 2 * lane;
                la = st + q * kLdn;
            }
            __builtin_amdgcn_global_load_lds((glb_void*)ga, (lds_void*)la, 16, 0, 0);
            const double* gb = xb + (k0 + q) * ldb + c0 + 2 * lane;
            __builtin_amdgcn_global_load_lds((glb_void*)gb, (lds_void*)(st + kBOff + q * kLdn), 16, 0, 0);
        }
    };
    d4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = d4{0.0, 0.0, 0.0, 0.0};
    // a wave's fragments of k-step kk of slice s (4 A, 4 B values), and the
    // k-step's 16 MFMAs: the fragments of the next k-step are read before
    // this one's MFMAs are issued (one wave per SIMD: nothing else hides the
    // LDS latency), across the mid-slice barrier too
    auto frag = [&](int s, int kk, double (&av)[4], double (&bv)[4]) {
        const double* As = lds + (s % kMmStages) * kStage;
        const double* Bs = As + kBOff;
        const int kr = kk * 4 + (lane >> 4);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = wm * 64 + i * 16 + (lane & 15);
            av[i] = AKC ? As[row * kMmBK + ((((kr >> 1) ^ ((row >> 1) & 7))) << 1) + (kr & 1)]
                        : As[kr * kLdn + row];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) bv[j] = Bs[kr * kLdn + wn * 64 + j * 16 + (lane & 15)];
    };
    auto mma = [&](const double (&av)[4], const double (&bv)[4], int i0 = 0, int i1 = 4) {   // A rows i0 .. i1 - 1
#ifdef WFSA_MM_PRIO
        __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
        for (int i = i0; i < i1; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[i], bv[j], acc[i][j], 0, 0, 0);
#ifdef WFSA_MM_PRIO
        __builtin_amdgcn_s_setprio(0);
#endif
    };
    // (every wave issues 8 DMA pieces per slice: "slice t landed" = at most
    // 8 x (slices issued after t) still outstanding)
    auto barrier = [] {
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
    };
    issue(0);
    if (nk > 1) issue(1);
    if (nk > 2) issue(2);
    if (nk > 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (nk > 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier();
    double a0[4], b0[4], a1[4], b1[4];
    frag(0, 0, a0, b0);
    for (int t = 0; t < nk; ++t) {
        frag(t, 1, a1, b1);
        mma(a0, b0);
        frag(t, 2, a0, b0);
        mma(a1, b1);
        // slice t + 1 in LDS (past the last slice: every DMA done); stage
        // (t + 3) % 4 = (t - 1) % 4 free.  (Unconditional barrier and reads:
        // one LDS-counter state on every path, so the compiler's waits for
        // the fragments stay counted, not drained.)
        if (t + 2 < nk) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        barrier();
        if (t + 3 < nk) issue(t + 3);
        frag(t, 3, a1, b1);
        mma(a0, b0);
        // the next slice's first fragments read half-way through the last
        // k-step (pinned there: hoisted above it, the wait for k-step 3's
        // fragments drained them too, with no MFMA in between)
        mma(a1, b1, 0, 2);
        __builtin_amdgcn_sched_barrier(0);
        frag(t + 1, 0, a0, b0);   // (past the last slice: a stale stage, unused)
        __builtin_amdgcn_sched_barrier(0);
        mma(a1, b1, 2, 4);
    }
    // epilogue: element (i, j, e) of this lane is row wm*64 + 16 i + (lane>>4)
    // + 4 e, column wn*64 + 16 j + (lane & 15) of the block tile
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int row = r0 + wm * 64 + 16 * i + (lane >> 4) + 4 * e;
                const int col = c0 + wn * 64 + 16 * j + (lane & 15);
                if (GRADEPI) {
                    const int64_t o = int64_t(row) * np + col;
                    const int32_t code = a.code_a[o];
                    if (code >= 0 && code < a.n_params) a.grad[code] = -a.amat[o] * acc[i][j][e];
                } else {
                    a.out[int64_t(row) * ldx + col] = acc[i][j][e];
                }
            }
}

// ---- epilogues of the library GEMMs (enqueue_blas) ------------------------
// One block per row slot r of the step; the row's new values and their sum
// (a fixed-order block reduction: deterministic) for the next step's scale.

constexpr int kEpiThreads = 256;

__device__ __forceinline__ double epi_block_sum(double v, double* red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    const int w = int(threadIdx.x) >> 6;
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    double t = 0.0;
    for (int i = 0; i < kEpiThreads / 64; ++i) t += red[i];
    return t;
}

struct EpiArgs {
    int32_t np, ldx;
    int32_t first;             // FWD: step 0 (every row starts) / BWD: step T-1 (every row ends)
    const int32_t* meta;       // [R] of the output step
    const int32_t* sid;        // [R] (BWD)
    const double* sum_in;      // [R] row sums of the input step
    double* sum_out;           // [R] of the output step
    const double* et;
    const double* a0;
    const double* aend;
    double* io;                // FWD: alpha[t+1] (the GEMM's alpha[t] A in, the values out); BWD: Y[t] likewise
    const double* io2;         // a split-K GEMM's second product (added to io's), or null
    const double* la_in;       // FWD
    double* la_out;
    const double* lb_in;       // BWD
    double* lb_out;
    const double* la_t;
    const double* la_prev;
    const double* alpha_t;
    double* gam;
    double* z;
    const double* p;
    const double* logq;
    const unsigned* halted;
};

// alpha[t+1] = (alpha[t] A / rowsum(alpha[t])) (.) E[sym], a0 (.) E[sym] where a string starts
__global__ __launch_bounds__(kEpiThreads) void dense_fwd_epi_kernel(EpiArgs a) {
    if (a.halted && *a.halted) return;
    __shared__ double red[kEpiThreads / 64];
    const int r = int(blockIdx.x);
    const int m = a.meta[r];
    const bool start = (m >> 9) & 1;
    double inv = 0.0, la = 0.0;
    if (!a.first) {
        const double s = a.sum_in[r];
        inv = s > 0.0 ? 1.0 / s : 0.0;
        la = start ? 0.0 : a.la_in[r] + log(s);
    }
    if (threadIdx.x == 0) a.la_out[r] = la;
    const double* erow = a.et + int64_t(m & 511) * a.np;
    double* row = a.io + int64_t(r) * a.ldx;
    const double* row2 = a.io2 ? a.io2 + int64_t(r) * a.ldx : nullptr;
    double acc = 0.0;
    // kEpiBatch columns per thread loaded before any is stored (the stores
    // into the row would otherwise order every later load behind them);
    // the sum runs over the thread's columns in the same ascending order
    for (int c0 = int(threadIdx.x); c0 < a.np; c0 += kEpiBatch * kEpiThreads) {
        double raw[kEpiBatch], e[kEpiBatch], s0[kEpiBatch];
#pragma unroll
        for (int u = 0; u < kEpiBatch; ++u) {
            const int c = c0 + u * kEpiThreads;
            const bool in = c < a.np;
            raw[u] = in && !a.first ? (row2 ? row[c] + row2[c] : row[c]) : 0.0;
            e[u] = in ? erow[c] : 0.0;
            s0[u] = in && start ? a.a0[c] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < kEpiBatch; ++u) {
            const int c = c0 + u * kEpiThreads;
            if (c >= a.np) break;
            const double v = (start ? s0[u] : raw[u] * inv) * e[u];
            row[c] = v;
            acc += v;
        }
    }
    acc = epi_block_sum(acc, red);
    if (threadIdx.x == 0) a.sum_out[r] = acc;
}

// beta[t] = Y[t+1] A^T / rowsum(Y[t+1]) (e where a string ends); Y[t] = E (.)
// beta, z[t] = Y[t] f2, gamma[t] = alpha[t] beta f1 (the fused kernel's epilogue)
__global__ __launch_bounds__(kEpiThreads) void dense_bwd_epi_kernel(EpiArgs a) {
    if (a.halted && *a.halted) return;
    __shared__ double red[kEpiThreads / 64];
    const int r = int(blockIdx.x);
    const int m = a.meta[r];
    const bool start = (m >> 9) & 1, end = (m >> 10) & 1;
    double inv = 0.0, lb = 0.0;
    if (!end && !a.first) {
        const double u = a.sum_in[r];
        inv = u > 0.0 ? 1.0 / u : 0.0;
        lb = a.lb_in[r] + log(u);
    }
    if (threadIdx.x == 0) a.lb_out[r] = lb;
    double f1 = 0.0, f2 = 0.0;
    const int s = a.sid[r];
    if (s >= 0) {
        const double lq = a.logq[s];
        if (lq > -INFINITY) {
            f1 = a.p[s] * exp(a.la_t[r] + lb - lq);
            if (!start && a.la_prev) f2 = a.p[s] * exp(a.la_prev[r] + lb - lq);
        }
    }
    const double* erow = a.et + int64_t(m & 511) * a.np;
    const int64_t o0 = int64_t(r) * a.ldx;
    double* row = a.io + o0;
    const double* row2 = a.io2 ? a.io2 + o0 : nullptr;
    double acc = 0.0;
    for (int c0 = int(threadIdx.x); c0 < a.np; c0 += kEpiBatch * kEpiThreads) {   // (batched as the forward's)
        double raw[kEpiBatch], e[kEpiBatch], al[kEpiBatch], ae[kEpiBatch];
#pragma unroll
        for (int u = 0; u < kEpiBatch; ++u) {
            const int c = c0 + u * kEpiThreads;
            const bool in = c < a.np;
            raw[u] = in && !a.first ? (row2 ? row[c] + row2[c] : row[c]) : 0.0;
            e[u] = in ? erow[c] : 0.0;
            al[u] = in ? a.alpha_t[o0 + c] : 0.0;
            ae[u] = in && end ? a.aend[c] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < kEpiBatch; ++u) {
            const int c = c0 + u * kEpiThreads;
            if (c >= a.np) break;
            const double beta = end ? ae[u] : raw[u] * inv;
            a.gam[o0 + c] = al[u] * beta * f1;
            const double v = e[u] * beta;
            row[c] = v;
            a.z[o0 + c] = v * f2;
            acc += v;
        }
    }
    acc = epi_block_sum(acc, red);
    if (threadIdx.x == 0) a.sum_out[r] = acc;
}

// grad(S -> T) = -A(S, T) G(S, T) for the transition parameters
__global__ __launch_bounds__(256) void dense_grad_scatter_kernel(const double* __restrict__ g, const double* __restrict__ amat,
                                                                 const int32_t* __restrict__ code_a, int64_t n,
                                                                 int32_t n_params, double* grad, const unsigned* halted) {
    if (halted && *halted) return;
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t o = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; o < n; o += stride) {
        const int32_t code = code_a[o];
        if (code >= 0 && code < n_params) grad[code] = -amat[o] * g[o];
    }
}

// ---- the rmin info column: a (min, +) trellis in the log domain ----------
//
// m_1[T] = log a[T] + log E[T][c_0],  m_{j+1}[T] = min_S (m_j[S] + log A[S][T])
// + log E[T][c_j], and the string's smallest path weight is min_T (m_L[T] +
// log e[T]); its relative probability divides by q (log q from the
// evaluation).  Missing edges are +inf, so they never win a minimum.

// log tables of the evaluation's exp-weight tables (+inf where the weight is 0)
__global__ __launch_bounds__(256) void dense_log_kernel(const double* __restrict__ amat, const double* __restrict__ et,
                                                        const double* __restrict__ a0, const double* __restrict__ aend,
                                                        double* lmat, double* let, double* l0, double* lend,
                                                        int64_t n_a, int64_t n_e, int32_t np, const unsigned* halted) {
    if (halted && *halted) return;
    const int64_t n = n_a + n_e + 2 * int64_t(np);
    for (int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) {
        const double* src;
        double* dst;
        int64_t j = i;
        if (j < n_a) { src = amat; dst = lmat; }
        else if ((j -= n_a) < n_e) { src = et; dst = let; }
        else if ((j -= n_e) < np) { src = a0; dst = l0; }
        else { j -= np; src = aend; dst = lend; }
        const double v = src[j];
        dst[j] = v > 0.0 ? log(v) : INFINITY;
    }
}

struct MinPlusArgs {
    const double* x;        // [R][np] the previous step's log minima (unused at step 0)
    const double* lmat;     // [np][np]
    const double* let;      // [vocab+1][np]
    const double* l0;       // [np]
    const double* lend;     // [np]
    const int32_t* meta;    // [R] this step
    const int32_t* sid;     // [R] this step
    double* y;              // [R][np] this step's log minima
    double* spart;          // [nct][S] per column tile: a string's end minimum
    int64_t n_strings;
    int32_t np, vocab;
    const unsigned* halted;
};

constexpr int kMpK = 16;   // K slice of the min-plus tile

// One step of the (min, +) trellis for all R row slots: y = (x (min,+) lA)
// + lE[sym] on a 128 x 128 tile per block (256 threads, 8 x 8 per thread at
// stride 16: the LDS reads of a slice broadcast within each 16-lane row
// group), K staged through LDS in slices of 16 with the next slice's global
// loads in registers during the current one's arithmetic.  Rows that start a
// string take log a + lE instead; rows that end one reduce min_T (y + log e)
// over the tile's columns into spart.
template <bool FIRST>
__global__ __launch_bounds__(256) void dense_minplus_kernel(MinPlusArgs a) {
    if (a.halted && *a.halted) return;
    __shared__ double xs[kMpK][kT + 1];   // [k][row]
    __shared__ double ls[kMpK][kT];       // [k][column]
    const int tid = int(threadIdx.x), tx = tid & 15, ty = tid >> 4;
    const int c0 = int(blockIdx.x) * kT, r0 = int(blockIdx.y) * kT;
    const size_t np = size_t(a.np);
    double acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = INFINITY;
    if (!FIRST) {
        // loaders: x row tid/2, k half (tid&1)*8; lA k row tid/16, columns (tid&15)*8
        const int xr = tid >> 1, xk = (tid & 1) * 8, lk = tid >> 4, lc = (tid & 15) * 8;
        const double2* xp = reinterpret_cast<const double2*>(a.x + size_t(r0 + xr) * np + size_t(xk));
        const double2* lp = reinterpret_cast<const double2*>(a.lmat + size_t(lk) * np + size_t(c0 + lc));
        const size_t lstep = kMpK * np / 2;   // double2 per K slice of lA
        double2 xv[4], lv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            xv[q] = xp[q];
            lv[q] = lp[q];
        }
        for (int k0 = 0; k0 < a.np; k0 += kMpK) {
            __syncthreads();   // the previous slice's reads are done
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                xs[xk + 2 * q][xr] = xv[q].x;
                xs[xk + 2 * q + 1][xr] = xv[q].y;
                ls[lk][lc + 2 * q] = lv[q].x;
                ls[lk][lc + 2 * q + 1] = lv[q].y;
            }
            __syncthreads();
            if (k0 + kMpK < a.np) {
                xp += kMpK / 2;
                lp += lstep;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    xv[q] = xp[q];
                    lv[q] = lp[q];
                }
            }
#pragma unroll 4
            for (int kk = 0; kk < kMpK; ++kk) {
                double xa[8], lb[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) xa[i] = xs[kk][ty + 16 * i];
#pragma unroll
                for (int j = 0; j < 8; ++j) lb[j] = ls[kk][tx + 16 * j];
#pragma unroll
                for (int i = 0; i < 8; ++i)
#pragma unroll
                    for (int j = 0; j < 8; ++j) acc[i][j] = fmin(acc[i][j], xa[i] + lb[j]);
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int r = r0 + ty + 16 * i;
        const int32_t m = a.meta[r];
        const int sym = m & 0x1ff;
        const bool idle = sym >= a.vocab, start = (m >> 9) & 1, end = (m >> 10) & 1;
        double endmin = INFINITY;
        double* yr = a.y + size_t(r) * np;
        const double* le = a.let + size_t(idle ? a.vocab : sym) * np;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int T = c0 + tx + 16 * j;
            const double v = idle ? INFINITY : ((start || FIRST) ? a.l0[T] : acc[i][j]) + le[T];
            yr[T] = v;
            endmin = fmin(endmin, v + a.lend[T]);
        }
        // the 16 lanes of this row (one row group of the wavefront)
#pragma unroll
        for (int o = 8; o >= 1; o >>= 1) endmin = fmin(endmin, __shfl_xor(endmin, o, 64));
        if (end && !idle && tx == 0) a.spart[size_t(blockIdx.x) * size_t(a.n_strings) + size_t(a.sid[r])] = endmin;
    }
}

__device__ __forceinline__ void dense_min_pair(double& v, double& i, double v2, double i2) {
    if (v2 < v || (v2 == v && i2 < i)) {
        v = v2;
        i = i2;
    }
}

// per string: log(min path / q) = min over column tiles - log q; block minima
// (value, string), ties to the lower string
__global__ __launch_bounds__(256) void dense_rmin_strings_kernel(const double* __restrict__ spart, int32_t nct,
                                                                 const int32_t* __restrict__ end_at,
                                                                 const double* __restrict__ logq, int64_t n_strings,
                                                                 double* rpart, const unsigned* halted) {
    if (halted && *halted) return;
    __shared__ double wv[4], wi[4];
    const int64_t s = int64_t(blockIdx.x) * 256 + threadIdx.x;
    double v = INFINITY, idx = -1.0;
    if (s < n_strings && end_at[s] >= 0) {
        double m = INFINITY;
        for (int c = 0; c < nct; ++c) m = fmin(m, spart[size_t(c) * size_t(n_strings) + size_t(s)]);
        v = m - logq[s];
        idx = double(s);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) dense_min_pair(v, idx, __shfl_xor(v, o, 64), __shfl_xor(idx, o, 64));
    if ((threadIdx.x & 63) == 0) {
        wv[threadIdx.x >> 6] = v;
        wi[threadIdx.x >> 6] = idx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < 4; ++k) dense_min_pair(v, idx, wv[k], wi[k]);
        rpart[2 * blockIdx.x] = v;
        rpart[2 * blockIdx.x + 1] = idx;
    }
}

// the block minima -> res = (exp(value), string), (0, -1) without a string
__global__ __launch_bounds__(256) void dense_rmin_final_kernel(const double* __restrict__ rpart, int n_part, double* res,
                                                               const unsigned* halted) {
    if (halted && *halted) return;
    __shared__ double wv[4], wi[4];
    double v = INFINITY, idx = -1.0;
    for (int k = int(threadIdx.x); k < n_part; k += 256) dense_min_pair(v, idx, rpart[2 * k], rpart[2 * k + 1]);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) dense_min_pair(v, idx, __shfl_xor(v, o, 64), __shfl_xor(idx, o, 64));
    if ((threadIdx.x & 63) == 0) {
        wv[threadIdx.x >> 6] = v;
        wi[threadIdx.x >> 6] = idx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < 4; ++k) dense_min_pair(v, idx, wv[k], wi[k]);
        res[0] = idx >= 0.0 ? exp(v) : 0.0;
        res[1] = idx;
    }
}

template <typename T>
hipError_t dalloc(T*& p, size_t n) {
    if (p) (void)hipFree(p);
    p = nullptr;
    return hipMalloc(reinterpret_cast<void**>(&p), std::max<size_t>(n, 1) * sizeof(T));
}

template <typename T>
void dfree(T*& p) {
    if (p) (void)hipFree(p);
    p = nullptr;
}

#define DTRY(x)                                     \
    do {                                            \
        const hipError_t e_ = (x);                  \
        if (e_ != hipSuccess) return e_;            \
    } while (0)

}  // namespace

std::string dense_model_build(const wfsa_model_desc& d, bool force, DenseModel& out) {
    const int32_t N = d.n_states;
    if (N <= 0 || d.start < 0 || d.start >= N) return "no start state";
    std::vector<int32_t> idx(size_t(N), -1);
    int32_t n_int = 0;
    for (int32_t s = 0; s < N; ++s)
        if (s != d.start && s != d.end) idx[size_t(s)] = n_int++;
    if (n_int == 0) return "no interior states";
    // single-byte emissions only
    bool used[256] = {};
    for (int32_t s = 0; s < N; ++s) {
        if (idx[size_t(s)] < 0) continue;
        for (int32_t e = d.em_ptr[s]; e < d.em_ptr[s + 1]; ++e) {
            if (d.em_len[e] != 1) return "an emission is not a single byte";
            used[d.em_bytes[d.em_off[e]]] = true;
        }
    }
    int64_t n_tr = 0;
    for (int32_t s = 0; s < N; ++s)
        if (idx[size_t(s)] >= 0)
            for (int32_t t = d.tr_ptr[s]; t < d.tr_ptr[s + 1]; ++t)
                if (d.tr_dst[t] != d.end && d.tr_dst[t] != d.start) ++n_tr;
    if (!force) {
        if (n_int < 64) return "fewer than 64 interior states";
        if (double(n_tr) * 4.0 < double(n_int) * double(n_int)) return "transition matrix sparser than 1/4";
    }
    DenseModel m;
    m.n_states = n_int;
    m.np = (n_int + kDenseTile - 1) / kDenseTile * kDenseTile;
    m.n_params = d.n_params;
    m.n_transitions = n_tr;
    int32_t V = 0;
    for (int b = 0; b < 256; ++b) m.sym_of_byte[b] = -1;
    for (int b = 0; b < 256; ++b)
        if (used[b]) m.sym_of_byte[b] = int16_t(V++);
    for (int b = 0; b < 256; ++b)
        if (m.sym_of_byte[b] < 0) m.sym_of_byte[b] = int16_t(V);
    m.vocab = V;
    const size_t np = size_t(m.np);
    auto code_of = [](int32_t param) { return param >= 0 ? param : kCodeOne; };
    m.code_a.assign(np * np, kCodeNone);
    m.code_s.assign(np, kCodeNone);
    m.code_e.assign(np, kCodeNone);
    m.code_em.assign(size_t(V + 1) * np, kCodeNone);
    for (int32_t s = 0; s < N; ++s) {
        const int32_t is = idx[size_t(s)];
        if (s == d.end) continue;   // $ has no way out on an accepting path
        for (int32_t t = d.tr_ptr[s]; t < d.tr_ptr[s + 1]; ++t) {
            const int32_t dst = d.tr_dst[t];
            if (dst == d.start) return "a transition into the start state";
            int32_t* slot;
            if (s == d.start) {
                slot = dst == d.end ? &m.code_se : &m.code_s[size_t(idx[size_t(dst)])];
            } else {
                slot = dst == d.end ? &m.code_e[size_t(is)] : &m.code_a[size_t(is) * np + size_t(idx[size_t(dst)])];
            }
            if (*slot != kCodeNone) return "duplicate transition";
            *slot = code_of(d.tr_param[t]);
        }
        if (is < 0) continue;
        for (int32_t e = d.em_ptr[s]; e < d.em_ptr[s + 1]; ++e) {
            const int32_t v = m.sym_of_byte[d.em_bytes[d.em_off[e]]];
            int32_t& slot = m.code_em[size_t(v) * np + size_t(is)];
            if (slot != kCodeNone) return "duplicate emission";
            slot = code_of(d.em_param[e]);
        }
    }
    out = std::move(m);
    return std::string();
}

DensePath::~DensePath() {
    free_corpus();
    free_model();
}

void DensePath::free_model() {
    dfree(code_a_); dfree(code_s_); dfree(code_e_); dfree(code_em_);
    dfree(amat_); dfree(amat_t_); dfree(et_); dfree(a0_); dfree(aend_); dfree(ones_); dfree(gbuf_);
    if (blas_) (void)rocblas_destroy_handle(static_cast<rocblas_handle>(blas_));
    blas_ = nullptr;
}

void DensePath::free_corpus() {
    dfree(meta_); dfree(sid_); dfree(end_at_); dfree(p_); dfree(pones_); dfree(logq_);
    dfree(la_); dfree(lb_); dfree(alpha_); dfree(gam_); dfree(z_); dfree(y_); dfree(ysplit_); dfree(part_);
    dfree(ll_part_); dfree(red_);
    dfree(lmat_); dfree(let_); dfree(l0_); dfree(lend_); dfree(mrow_); dfree(spart_); dfree(rpart_);
    n_strings_ = 0;
    R_ = T_ = 0;
    weighted_ = false;
}

hipError_t DensePath::load_model(const DenseModel& m, hipStream_t s) {
#ifdef WFSA_EXPERIMENTS   // GEMM block configurations for timing experiments (experiments build only)
    if (const char* e = std::getenv("WFSA_DENSE_GRAD_CFG")) grad_cfg_ = std::atoi(e);
    if (const char* e = std::getenv("WFSA_DENSE_STEP_CFG")) step_cfg_ = std::atoi(e);
#endif
    free_corpus();
    free_model();
    n_params_ = m.n_params;
    np_ = m.np;
    vocab_ = m.vocab;
    nct_ = m.np / kT;
    code_se_ = m.code_se;
    std::memcpy(sym_of_byte_, m.sym_of_byte, sizeof sym_of_byte_);
    const size_t np = size_t(np_);
    DTRY(dalloc(code_a_, np * np));
    DTRY(dalloc(code_s_, np));
    DTRY(dalloc(code_e_, np));
    DTRY(dalloc(code_em_, size_t(vocab_ + 1) * np));
    DTRY(hipMemcpyAsync(code_a_, m.code_a.data(), np * np * 4, hipMemcpyHostToDevice, s));
    DTRY(hipMemcpyAsync(code_s_, m.code_s.data(), np * 4, hipMemcpyHostToDevice, s));
    DTRY(hipMemcpyAsync(code_e_, m.code_e.data(), np * 4, hipMemcpyHostToDevice, s));
    DTRY(hipMemcpyAsync(code_em_, m.code_em.data(), size_t(vocab_ + 1) * np * 4, hipMemcpyHostToDevice, s));
    DTRY(dalloc(amat_, np * np));
    DTRY(dalloc(amat_t_, np * np));
    DTRY(dalloc(et_, size_t(vocab_ + 1) * np));
    DTRY(dalloc(a0_, np));
    DTRY(dalloc(aend_, np));
    std::vector<double> ones(size_t(n_params_) + 2, 1.0);
    DTRY(dalloc(ones_, ones.size()));
    DTRY(hipMemcpyAsync(ones_, ones.data(), ones.size() * 8, hipMemcpyHostToDevice, s));
    if (const char* e = std::getenv("WFSA_DENSE_ENGINE")) {
        const std::string v(e);
        if (v == "fused") engine_ = 0;
        else if (v == "blas") engine_ = 1;
        else if (v == "split") engine_ = 2;
        else if (v == "dma") engine_ = 3;
        else return hipErrorInvalidValue;
    }
    if (engine_ == 1) {
        rocblas_handle h = nullptr;
        if (rocblas_create_handle(&h) != rocblas_status_success) return hipErrorNotInitialized;
        blas_ = h;
        // no atomics: every GEMM's sums in a fixed order (deterministic results)
        if (rocblas_set_atomics_mode(h, rocblas_atomics_not_allowed) != rocblas_status_success)
            return hipErrorNotInitialized;
        DTRY(dalloc(gbuf_, np * np));
    }
    return hipStreamSynchronize(s);
}

hipError_t DensePath::load_corpus(const uint8_t* sym, const int64_t* off, const double* p, int64_t n_strings,
                                  hipStream_t s) {
    free_corpus();
    n_strings_ = n_strings;
    const size_t S = size_t(n_strings);
    int64_t total = 0, lmax = 0;
    p0_sum_ = 0.0;
    n0_ = 0.0;
    std::vector<int32_t> order;
    order.reserve(S);
    for (size_t i = 0; i < S; ++i) {
        const int64_t L = off[i + 1] - off[i];
        total += L;
        lmax = std::max(lmax, L);
        if (L > 0) order.push_back(int32_t(i));
        else { p0_sum_ += p[i]; n0_ += 1.0; }
    }
    total_sym_ = total;
    // slots: R rows (a multiple of the tile) and T >= max(lmax, total / R)
    // steps; a step's GEMM is (R / 128) x (np / 128) blocks, which run in
    // ceil(blocks / CUs) rounds -- pick the R with the fewest step-rounds
    int64_t R = kT;
    {
        const int64_t cap = std::max<int64_t>(1, (int64_t(order.size()) + kT - 1) / kT);
        double best = -1.0;
        for (int64_t k = 1; k <= cap; ++k) {
            const int64_t r = k * kT;
            const int64_t t = std::max<int64_t>(lmax, (total + r - 1) / r);
            const int64_t blocks = k * int64_t(nct_);
            const double cost = double(std::max<int64_t>(t - 1, 1)) * double((blocks + n_cu_ - 1) / n_cu_);
            if (best < 0.0 || cost < best - 1e-9) {
                best = cost;
                R = r;
            }
        }
    }
    std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) {
        return off[a + 1] - off[a] > off[b + 1] - off[b];
    });
    // longest first, each to the least loaded slot
    std::vector<std::vector<int32_t>> slot(static_cast<size_t>(R));
    std::vector<int64_t> load(static_cast<size_t>(R), 0);
    {
        using E = std::pair<int64_t, int32_t>;
        std::priority_queue<E, std::vector<E>, std::greater<E>> pq;
        for (int32_t r = 0; r < int32_t(R); ++r) pq.push({0, r});
        for (int32_t str : order) {
            E e = pq.top();
            pq.pop();
            slot[size_t(e.second)].push_back(str);
            e.first += off[str + 1] - off[str];
            load[size_t(e.second)] = e.first;
            pq.push(e);
        }
    }
    int64_t T = 0;
    for (int64_t l : load) T = std::max(T, l);
    T = std::max<int64_t>(T, 1);
    if (T * R >= (int64_t(1) << 31)) return hipErrorInvalidValue;
    R_ = int32_t(R);
    T_ = int32_t(T);
    const size_t TR = size_t(T) * size_t(R);
    std::vector<int32_t> meta(TR, vocab_), sid(TR, -1), end_at(S, -1);
    for (int32_t r = 0; r < int32_t(R); ++r) {
        int64_t t = 0;
        for (int32_t str : slot[size_t(r)]) {
            const int64_t L = off[str + 1] - off[str];
            for (int64_t j = 0; j < L; ++j, ++t) {
                const size_t o = size_t(t) * size_t(R) + size_t(r);
                meta[o] = int32_t(sym_of_byte_[sym[off[str] + j]]) | (j == 0 ? 1 << 9 : 0) | (j == L - 1 ? 1 << 10 : 0);
                sid[o] = str;
                if (j == L - 1) end_at[size_t(str)] = int32_t(o);
            }
        }
    }
    const size_t np = size_t(np_);
    DTRY(dalloc(meta_, TR));
    DTRY(dalloc(sid_, TR));
    DTRY(dalloc(end_at_, S));
    DTRY(dalloc(p_, S));
    DTRY(dalloc(pones_, S));
    DTRY(dalloc(logq_, S));
    DTRY(hipMemcpyAsync(meta_, meta.data(), TR * 4, hipMemcpyHostToDevice, s));
    DTRY(hipMemcpyAsync(sid_, sid.data(), TR * 4, hipMemcpyHostToDevice, s));
    DTRY(hipMemcpyAsync(end_at_, end_at.data(), S * 4, hipMemcpyHostToDevice, s));
    if (S) DTRY(hipMemcpyAsync(p_, p, S * 8, hipMemcpyHostToDevice, s));
    std::vector<double> ones(std::max<size_t>(S, 1), 1.0);
    DTRY(hipMemcpyAsync(pones_, ones.data(), S * 8, hipMemcpyHostToDevice, s));
    DTRY(dalloc(la_, TR));
    DTRY(dalloc(lb_, TR));
    ldx_ = np_ + kRowPad;
    const size_t ld = size_t(ldx_);
    DTRY(dalloc(alpha_, TR * ld));
    DTRY(dalloc(gam_, TR * ld));
    DTRY(dalloc(z_, TR * ld));
    DTRY(dalloc(y_, 2 * size_t(R) * ld));
    if (engine_ == 2) DTRY(dalloc(ysplit_, size_t(R) * ld));   // (engine 3: no split)
    DTRY(dalloc(part_, 2 * size_t(nct_) * size_t(R)));
    n_ll_ = int32_t((S + 3) / 4);
    DTRY(dalloc(ll_part_, size_t(std::max(n_ll_, 1))));
    // gamma reduction: enough row chunks to fill the chip with column blocks
    const int64_t cols = np / kRedThreads;
    int64_t chunks = std::max<int64_t>(1, (1024 + cols - 1) / cols);
    chunks = std::min<int64_t>(chunks, int64_t(TR));
    reduce_chunks_ = int32_t(chunks);
    DTRY(dalloc(red_, size_t(chunks) * size_t(vocab_ + 2) * np));
    return hipStreamSynchronize(s);
}

double DensePath::issued_flops() const {
    const double np = double(np_), R = double(R_), T = double(T_);
    return 2.0 * np * np * R * (T - 1) * 3.0;
}

hipError_t DensePath::enqueue(const double* ewp, bool structural, double* out, double* logq, const unsigned* halted,
                              hipStream_t s) {
    const size_t np = size_t(np_), R = size_t(R_);
    const double* w = structural ? ones_ : ewp;
    const double* p = structural ? pones_ : p_;
    weighted_ = !structural;
    if (engine() != 0 && n_strings_ > 0 && total_sym_ > 0) return enqueue_lib(w, p, structural, out, logq, halted, s);
    {
        WeightsArgs a{};
        a.ewp = w;
        a.code_a = code_a_; a.code_em = code_em_; a.code_s = code_s_; a.code_e = code_e_;
        a.amat = amat_; a.et = et_; a.a0 = a0_; a.aend = aend_;
        a.n_a = int64_t(np * np);
        a.n_em = int64_t(size_t(vocab_ + 1) * np);
        a.np = np_;
        a.out = out;
        a.n_out = n_params_ + 1;
        a.halted = halted;
        dense_weights_kernel<<<1024, 256, 0, s>>>(a);
        DTRY(hipGetLastError());
        dense_transpose_kernel<<<dim3(unsigned(np / 32), unsigned(np / 32)), 256, 0, s>>>(amat_, amat_t_, np_, halted);
        DTRY(hipGetLastError());
    }
    if (n_strings_ == 0 || total_sym_ == 0) {
        FinalArgs f{};
        if (n_strings_ > 0) {
            f.alpha = alpha_; f.la = la_; f.aend = aend_; f.end_at = end_at_; f.p = p; f.ewp = w;
            f.code_se = code_se_; f.n_strings = n_strings_; f.np = np_; f.ldx = ldx_; f.logq = logq_; f.logq_user = logq;
            f.ll_part = ll_part_; f.halted = halted;
            dense_final_kernel<<<n_ll_, 256, 0, s>>>(f);
            DTRY(hipGetLastError());
        }
        ScatterArgs c{};
        c.red = red_; c.chunks = 0; c.np = np_; c.vocab = vocab_;
        c.code_em = code_em_; c.code_s = code_s_; c.code_e = code_e_; c.code_se = code_se_;
        c.n_params = n_params_; c.empty_p = structural ? n0_ : p0_sum_;
        c.ll_part = ll_part_; c.n_ll = n_strings_ > 0 ? n_ll_ : 0; c.out = out; c.halted = halted;
        dense_scatter_kernel<<<1, 256, 0, s>>>(c);
        return hipGetLastError();
    }
    const size_t step = R * size_t(ldx_);
    GemmArgs g{};
    g.R = R_; g.np = np_; g.nct = nct_; g.ldx = ldx_;
    g.et = et_; g.a0 = a0_; g.aend = aend_;
    g.p = p; g.logq = logq_;
    g.n_params = n_params_;
    g.halted = halted;
    const int fb_blocks = int((R / kT) * (np / kT));
    // forward: step 0 (every row starts a string), then t -> t+1
    for (int64_t t = -1; t + 1 < T_; ++t) {
        GemmArgs f = g;
        f.no_mma = t < 0;
        f.x = t < 0 ? alpha_ : alpha_ + size_t(t) * step;
        f.bm = amat_;
        f.meta = meta_ + size_t(t + 1) * R;
        f.part_in = part_ + size_t(t & 1) * nct_ * R;
        f.part_out = part_ + size_t((t + 1) & 1) * nct_ * R;
        f.out = alpha_ + size_t(t + 1) * step;
        f.la_in = t < 0 ? la_ : la_ + size_t(t) * R;
        f.la_out = la_ + size_t(t + 1) * R;
        if (step_cfg_ == 1) dense_gemm_kernel<FWD, kBkStep, 4><<<fb_blocks, 4 * 64, 0, s>>>(f);
        else if (step_cfg_ == 2) dense_gemm_kernel<FWD, kBkGrad, kNwStep><<<fb_blocks, kNwStep * 64, 0, s>>>(f);
        else dense_gemm_kernel<FWD, kBkStep, kNwStep><<<fb_blocks, kNwStep * 64, 0, s>>>(f);
        DTRY(hipGetLastError());
    }
    {
        FinalArgs f{};
        f.alpha = alpha_; f.la = la_; f.aend = aend_; f.end_at = end_at_; f.p = p; f.ewp = w;
        f.code_se = code_se_; f.n_strings = n_strings_; f.np = np_; f.ldx = ldx_; f.logq = logq_; f.logq_user = logq;
        f.ll_part = ll_part_; f.halted = halted;
        dense_final_kernel<<<n_ll_, 256, 0, s>>>(f);
        DTRY(hipGetLastError());
    }
    // backward: step T-1 (every row ends), then t+1 -> t
    for (int64_t t = T_ - 1; t >= 0; --t) {
        GemmArgs b = g;
        b.no_mma = t == T_ - 1;
        b.x = y_ + size_t((t + 1) & 1) * step;
        b.bm = amat_t_;
        b.meta = meta_ + size_t(t) * R;
        b.sid = sid_ + size_t(t) * R;
        b.part_in = part_ + size_t((t + 1) & 1) * nct_ * R;
        b.part_out = part_ + size_t(t & 1) * nct_ * R;
        b.out = y_ + size_t(t & 1) * step;
        b.lb_in = lb_ + size_t(std::min<int64_t>(t + 1, T_ - 1)) * R;
        b.lb_out = lb_ + size_t(t) * R;
        b.la_t = la_ + size_t(t) * R;
        b.la_prev = t > 0 ? la_ + size_t(t - 1) * R : nullptr;
        b.alpha_t = alpha_ + size_t(t) * step;
        b.gam = gam_ + size_t(t) * step;
        b.z = z_ + size_t(t) * step;
        if (step_cfg_ == 1) dense_gemm_kernel<BWD, kBkStep, 4><<<fb_blocks, 4 * 64, 0, s>>>(b);
        else if (step_cfg_ == 2) dense_gemm_kernel<BWD, kBkGrad, kNwStep><<<fb_blocks, kNwStep * 64, 0, s>>>(b);
        else dense_gemm_kernel<BWD, kBkStep, kNwStep><<<fb_blocks, kNwStep * 64, 0, s>>>(b);
        DTRY(hipGetLastError());
    }
    if (T_ >= 2) {
        GemmArgs q = g;
        q.no_mma = 0;
        q.kg = int64_t(T_ - 1) * int64_t(R);
        q.x = alpha_;
        q.bm = z_ + step;
        q.code_a = code_a_;
        q.amat = amat_;
        q.grad = out + 1;
        if (grad_cfg_ == 1)
            dense_gemm_kernel<GRAD, kBkStep, kNwStep><<<int((np / kT) * (np / kT)), kNwStep * 64, 0, s>>>(q);
        else
            dense_gemm_kernel<GRAD, kBkGrad, kNwGrad><<<int((np / kT) * (np / kT)), kNwGrad * 64, 0, s>>>(q);
        DTRY(hipGetLastError());
    }
    {
        ReduceArgs r{};
        r.gam = gam_; r.meta = meta_;
        r.rows = int64_t(T_) * int64_t(R);
        r.rows_per_chunk = (r.rows + reduce_chunks_ - 1) / reduce_chunks_;
        r.np = np_; r.vocab = vocab_; r.ldx = ldx_; r.red = red_; r.halted = halted;
        dim3 grid(unsigned(np / kRedThreads), unsigned(reduce_chunks_));
        dense_reduce_kernel<<<grid, kRedThreads, 0, s>>>(r);
        DTRY(hipGetLastError());
    }
    {
        ScatterArgs c{};
        c.red = red_; c.chunks = reduce_chunks_; c.np = np_; c.vocab = vocab_;
        c.code_em = code_em_; c.code_s = code_s_; c.code_e = code_e_; c.code_se = code_se_;
        c.n_params = n_params_; c.empty_p = structural ? n0_ : p0_sum_;
        c.ll_part = ll_part_; c.n_ll = n_ll_; c.out = out; c.halted = halted;
        const int64_t n = int64_t(vocab_ + 2) * int64_t(np);
        dense_scatter_kernel<<<unsigned((n + 255) / 256), 256, 0, s>>>(c);
        DTRY(hipGetLastError());
    }
    return hipSuccess;
}

// The same evaluation with the GEMMs as plain products and the fused
// kernels' epilogues as their own per-row kernels.  Engine 1: rocBLAS dgemm
// calls (fp64 MFMA): the row slot buffers are row-major [R][ldx]; seen
// column-major they are np x R (ld = ldx), so alpha[t+1]^T = A^T alpha[t]^T
// is dgemm(N, N) with the row-major A as its column-major transpose, Y[t+1]
// A^T likewise with op T, and G = alpha[0..T-2]^T z[1..T-1] as (G^T)^T =
// dgemm(N, T) over K = (T-1) R rows.  Engine 2: dense_gemm_kernel<RAW> with
// K in two halves (the second into ysplit_, summed by the epilogue) and the
// fused gradient kernel.  Row sums: one full sum per row ([R], nct = 1).
hipError_t DensePath::enqueue_lib(const double* w, const double* p, bool structural, double* out, double* logq,
                                  const unsigned* halted, hipStream_t s) {
    const size_t np = size_t(np_), R = size_t(R_);
    const bool ours = engine() >= 2, dma = engine() == 3;
    rocblas_handle h = static_cast<rocblas_handle>(blas_);
    if (!ours && rocblas_set_stream(h, s) != rocblas_status_success) return hipErrorInvalidHandle;
    auto rb = [](rocblas_status st) { return st == rocblas_status_success ? hipSuccess : hipErrorLaunchFailure; };
    GemmArgs raw{};
    raw.R = R_; raw.np = np_; raw.nct = nct_; raw.ldx = ldx_; raw.halted = halted;
    raw.out2 = ysplit_; raw.splits = kSplitK;
    const int raw_blocks = int((R / kT) * (np / kT)) * kSplitK, mm_blocks = int((R / kT) * (np / kT));
    {
        WeightsArgs a{};
        a.ewp = w;
        a.code_a = code_a_; a.code_em = code_em_; a.code_s = code_s_; a.code_e = code_e_;
        a.amat = amat_; a.et = et_; a.a0 = a0_; a.aend = aend_;
        a.n_a = int64_t(np * np);
        a.n_em = int64_t(size_t(vocab_ + 1) * np);
        a.np = np_;
        a.out = out;
        a.n_out = n_params_ + 1;
        a.halted = halted;
        dense_weights_kernel<<<1024, 256, 0, s>>>(a);
        DTRY(hipGetLastError());
        if (ours) {
            dense_transpose_kernel<<<dim3(unsigned(np / 32), unsigned(np / 32)), 256, 0, s>>>(amat_, amat_t_, np_, halted);
            DTRY(hipGetLastError());
        }
    }
    const size_t step = R * size_t(ldx_);
    const double one = 1.0, zero = 0.0;
    const rocblas_int inp = rocblas_int(np_), iR = rocblas_int(R_), ild = rocblas_int(ldx_);
    EpiArgs g{};
    g.np = np_; g.ldx = ldx_; g.et = et_; g.a0 = a0_; g.aend = aend_; g.p = p; g.logq = logq_; g.halted = halted;
    // forward
    for (int64_t t = -1; t + 1 < T_; ++t) {
        double* nxt = alpha_ + size_t(t + 1) * step;
        if (t >= 0 && ours) {   // alpha[t+1] = alpha[t] A (raw products; the epilogue scales)
            GemmArgs m = raw;
            m.x = alpha_ + size_t(t) * step;
            m.bm = amat_;
            m.out = nxt;
            if (dma) dense_mm_kernel<true, false><<<mm_blocks, 256, 0, s>>>(m);
            else if (step_cfg_ == 3) dense_gemm_kernel<RAW, kBkStep, 4><<<raw_blocks, 4 * 64, 0, s>>>(m);
            else if (step_cfg_ >= 5) dense_gemm_kernel<RAW, kBkGrad, 8><<<raw_blocks, 8 * 64, 0, s>>>(m);   // (8 waves, 64 x 32 each)
            else dense_gemm_kernel<RAW, kBkGrad, kNwGrad><<<raw_blocks, kNwGrad * 64, 0, s>>>(m);
            DTRY(hipGetLastError());
        } else if (t >= 0) {   // alpha[t+1]^T = A^T alpha[t]^T
            DTRY(rb(rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_none, inp, iR, inp, &one, amat_, inp,
                                  alpha_ + size_t(t) * step, ild, &zero, nxt, ild)));
        }
        EpiArgs f = g;
        f.io2 = ours && !dma && t >= 0 ? ysplit_ : nullptr;
        f.first = t < 0;
        f.meta = meta_ + size_t(t + 1) * R;
        f.sum_in = part_ + size_t(t & 1) * R;
        f.sum_out = part_ + size_t((t + 1) & 1) * R;
        f.io = nxt;
        f.la_in = t < 0 ? la_ : la_ + size_t(t) * R;
        f.la_out = la_ + size_t(t + 1) * R;
        dense_fwd_epi_kernel<<<unsigned(R), kEpiThreads, 0, s>>>(f);
        DTRY(hipGetLastError());
    }
    {
        FinalArgs f{};
        f.alpha = alpha_; f.la = la_; f.aend = aend_; f.end_at = end_at_; f.p = p; f.ewp = w;
        f.code_se = code_se_; f.n_strings = n_strings_; f.np = np_; f.ldx = ldx_; f.logq = logq_; f.logq_user = logq;
        f.ll_part = ll_part_; f.halted = halted;
        dense_final_kernel<<<n_ll_, 256, 0, s>>>(f);
        DTRY(hipGetLastError());
    }
    // backward
    for (int64_t t = T_ - 1; t >= 0; --t) {
        double* cur = y_ + size_t(t & 1) * step;
        if (t < T_ - 1 && ours) {   // beta[t] = Y[t+1] A^T (raw)
            GemmArgs m = raw;
            m.x = y_ + size_t((t + 1) & 1) * step;
            m.bm = amat_t_;
            m.out = cur;
            if (dma) dense_mm_kernel<true, false><<<mm_blocks, 256, 0, s>>>(m);
            else if (step_cfg_ == 3) dense_gemm_kernel<RAW, kBkStep, 4><<<raw_blocks, 4 * 64, 0, s>>>(m);
            else if (step_cfg_ >= 5) dense_gemm_kernel<RAW, kBkGrad, 8><<<raw_blocks, 8 * 64, 0, s>>>(m);   // (8 waves, 64 x 32 each)
            else dense_gemm_kernel<RAW, kBkGrad, kNwGrad><<<raw_blocks, kNwGrad * 64, 0, s>>>(m);
            DTRY(hipGetLastError());
        } else if (t < T_ - 1) {   // beta[t]^T = A Y[t+1]^T
            DTRY(rb(rocblas_dgemm(h, rocblas_operation_transpose, rocblas_operation_none, inp, iR, inp, &one, amat_, inp,
                                  y_ + size_t((t + 1) & 1) * step, ild, &zero, cur, ild)));
        }
        EpiArgs b = g;
        b.io2 = ours && !dma && t < T_ - 1 ? ysplit_ : nullptr;
        b.first = t == T_ - 1;
        b.meta = meta_ + size_t(t) * R;
        b.sid = sid_ + size_t(t) * R;
        b.sum_in = part_ + size_t((t + 1) & 1) * R;
        b.sum_out = part_ + size_t(t & 1) * R;
        b.io = cur;
        b.lb_in = lb_ + size_t(std::min<int64_t>(t + 1, T_ - 1)) * R;
        b.lb_out = lb_ + size_t(t) * R;
        b.la_t = la_ + size_t(t) * R;
        b.la_prev = t > 0 ? la_ + size_t(t - 1) * R : nullptr;
        b.alpha_t = alpha_ + size_t(t) * step;
        b.gam = gam_ + size_t(t) * step;
        b.z = z_ + size_t(t) * step;
        dense_bwd_epi_kernel<<<unsigned(R), kEpiThreads, 0, s>>>(b);
        DTRY(hipGetLastError());
    }
    if (T_ >= 2 && ours) {   // G = alpha[0..T-2]^T z[1..T-1], scattered into the gradient by the kernel
        GemmArgs q{};
        q.R = R_; q.np = np_; q.nct = nct_; q.ldx = ldx_; q.halted = halted; q.n_params = n_params_; q.splits = 1;
        q.kg = int64_t(T_ - 1) * int64_t(R);
        q.x = alpha_;
        q.bm = z_ + step;
        q.code_a = code_a_;
        q.amat = amat_;
        q.grad = out + 1;
        if (dma && step_cfg_ == 4) dense_mm_kernel<false, true><<<int((np / kT) * (np / kT)), 256, 0, s>>>(q);
        else if (step_cfg_ == 6) dense_gemm_kernel<GRAD, kBkGrad, 8><<<int((np / kT) * (np / kT)), 8 * 64, 0, s>>>(q);
        else dense_gemm_kernel<GRAD, kBkGrad, kNwGrad><<<int((np / kT) * (np / kT)), kNwGrad * 64, 0, s>>>(q);
        DTRY(hipGetLastError());
    } else if (T_ >= 2) {   // G^T = z[1..]^T alpha[0..] over K = (T-1) R rows: g[S np + T] = G(S, T)
        const int64_t K = int64_t(T_ - 1) * int64_t(R);
        if (K >= (int64_t(1) << 31)) return hipErrorInvalidValue;
        DTRY(rb(rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_transpose, inp, inp, rocblas_int(K), &one,
                              z_ + step, ild, alpha_, ild, &zero, gbuf_, inp)));
        dense_grad_scatter_kernel<<<1024, 256, 0, s>>>(gbuf_, amat_, code_a_, int64_t(np * np), n_params_, out + 1,
                                                        halted);
        DTRY(hipGetLastError());
    }
    {
        ReduceArgs r{};
        r.gam = gam_; r.meta = meta_;
        r.rows = int64_t(T_) * int64_t(R);
        r.rows_per_chunk = (r.rows + reduce_chunks_ - 1) / reduce_chunks_;
        r.np = np_; r.vocab = vocab_; r.ldx = ldx_; r.red = red_; r.halted = halted;
        dim3 grid(unsigned(np / kRedThreads), unsigned(reduce_chunks_));
        dense_reduce_kernel<<<grid, kRedThreads, 0, s>>>(r);
        DTRY(hipGetLastError());
    }
    {
        ScatterArgs c{};
        c.red = red_; c.chunks = reduce_chunks_; c.np = np_; c.vocab = vocab_;
        c.code_em = code_em_; c.code_s = code_s_; c.code_e = code_e_; c.code_se = code_se_;
        c.n_params = n_params_; c.empty_p = structural ? n0_ : p0_sum_;
        c.ll_part = ll_part_; c.n_ll = n_ll_; c.out = out; c.halted = halted;
        const int64_t n = int64_t(vocab_ + 2) * int64_t(np);
        dense_scatter_kernel<<<unsigned((n + 255) / 256), 256, 0, s>>>(c);
        DTRY(hipGetLastError());
    }
    return hipSuccess;
}

hipError_t DensePath::enqueue_rmin(double* res, const unsigned* halted, hipStream_t s) {
    const size_t np = size_t(np_), R = size_t(R_), S = size_t(std::max<int64_t>(n_strings_, 1));
    const int nb = int((S + 255) / 256);
    if (!lmat_) {   // first call: the pass's buffers
        DTRY(dalloc(lmat_, np * np));
        DTRY(dalloc(let_, size_t(vocab_ + 1) * np));
        DTRY(dalloc(l0_, np));
        DTRY(dalloc(lend_, np));
    }
    if (!mrow_ && R > 0) {
        DTRY(dalloc(mrow_, 2 * R * np));
        DTRY(dalloc(spart_, size_t(nct_) * S));
        DTRY(dalloc(rpart_, 2 * size_t(nb)));
    }
    if (n_strings_ == 0 || total_sym_ == 0 || R == 0) {   // no string with a path of positive length
        static const double none[2] = {0.0, -1.0};
        return hipMemcpyAsync(res, none, sizeof none, hipMemcpyHostToDevice, s);
    }
    dense_log_kernel<<<1024, 256, 0, s>>>(amat_, et_, a0_, aend_, lmat_, let_, l0_, lend_, int64_t(np * np),
                                          int64_t(size_t(vocab_ + 1) * np), np_, halted);
    DTRY(hipGetLastError());
    MinPlusArgs g{};
    g.lmat = lmat_; g.let = let_; g.l0 = l0_; g.lend = lend_;
    g.spart = spart_;
    g.n_strings = n_strings_;
    g.np = np_;
    g.vocab = vocab_;
    g.halted = halted;
    const dim3 grid(unsigned(np / kT), unsigned(R / kT));
    for (int64_t t = 0; t < T_; ++t) {
        MinPlusArgs f = g;
        f.x = mrow_ + size_t((t + 1) & 1) * R * np;
        f.y = mrow_ + size_t(t & 1) * R * np;
        f.meta = meta_ + size_t(t) * R;
        f.sid = sid_ + size_t(t) * R;
        if (t == 0) dense_minplus_kernel<true><<<grid, 256, 0, s>>>(f);
        else dense_minplus_kernel<false><<<grid, 256, 0, s>>>(f);
        DTRY(hipGetLastError());
    }
    dense_rmin_strings_kernel<<<unsigned(nb), 256, 0, s>>>(spart_, nct_, end_at_, logq_, n_strings_, rpart_, halted);
    DTRY(hipGetLastError());
    dense_rmin_final_kernel<<<1, 256, 0, s>>>(rpart_, nb, res, halted);
    return hipGetLastError();
}

}  // namespace wfsa
