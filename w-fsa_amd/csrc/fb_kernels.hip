// Forward-backward over the (position, node) trellis of each corpus string.
//
// Replaces, per iteration, the reference's SpMV chain over the path matrices
// (Learner::ComputeModeledProbs / ComputeObjective, src/Learner.cpp:515-553;
// QuasiNewtonLearner::ComputeGrad, src/QuasiNewtonLearner.cpp:93-125) and,
// once, its path enumeration (Learner::BuildPaths, src/Learner.cpp:276-348,
// with Recognizer::RecognizeBFS, inc/Recognize.h:62-96).
//
// Per string s of length L (bytes c_0..c_{L-1}):
//   forward   alpha_0 = {start: 1};  alpha_{i+1}(T) = sum over edges S->T with
//             byte c_i of alpha_i(S) * w_edge;
//   end       q = sum_S alpha_L(S) * w_end(S)
//   backward  beta_L(S) = w_end(S);  beta_i(S) = sum_edges w * beta_{i+1}(T);
//             an edge's posterior alpha_i(S) w beta_{i+1}(T) / q is added
//             (times -p_s) to every parameter of the edge.
//
// trav_kernel (one wavefront per string) walks the automaton: frontier nodes
// are created on first touch through a node->slot map in LDS (CAS claim,
// ballot compaction), summed with LDS fp64 atomics, every position rescaled
// by an exact power of two.  Its counting mode (all weights 1) gives the path
// count, the used parameters and the compiled stream of the string:
//
// Compiled stream.  A position with exactly one live node (one on an
// accepting path) is a cut: every path passes through it.  Between two
// consecutive cuts the trellis is either ONE edge (a "trivial" word: the edge
// id; its posterior is exactly 1) or a "bubble" (a small DAG stored once in a
// bubble buffer).  With the posterior of a bubble edge taken relative to the
// bubble's own start and end, alpha_seg(src) w beta_seg(dst) / Z_seg, the
// whole string decomposes into independent segments, and
//   log q = sum_trivial lw_e + sum_bubbles log Z_seg.
// fbc_kernel evaluates these streams every iteration, one lane per string.
#include "fb_kernels.hpp"
#include "qn_device.hpp"

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>


namespace wfsa {

namespace {

constexpr int kWave = 64;
constexpr double kLn2 = 0.69314718055994530942;

__device__ __forceinline__ int lane_id() { return int(threadIdx.x) & (kWave - 1); }

// number of set bits of m below this lane
__device__ __forceinline__ int rank_below(unsigned long long m) {
    return int(__builtin_amdgcn_mbcnt_hi(unsigned(m >> 32), __builtin_amdgcn_mbcnt_lo(unsigned(m), 0u)));
}

// LDS is processed in issue order for one wavefront; the fence only stops
// the compiler from moving LDS accesses across the phase boundary.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

__device__ __forceinline__ int ld_rlx(const int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}
__device__ __forceinline__ void st_rlx(int* p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}
__device__ __forceinline__ void lds_add(double* p, double v) {
    __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}
__device__ __forceinline__ void block_add(double* p, double v) {
    __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void global_add(double* p, double v) {
    __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Fixed-point sums whose bits do not depend on the order of the adds (integer
// addition is associative): the wave kernel's gradient and log-likelihood,
// whose strings go to waves through a work counter.  A value is rounded once
// to a multiple of 2^-frac; a 128-bit accumulator {lo, hi} in global memory
// takes a signed 64-bit (or a 128-bit) addend with an atomic add on the low
// word whose returned old value gives the carry into the high word.
constexpr unsigned long long kFixLlNegInf = 1, kFixLlPosInf = 2, kFixLlNan = 4, kFixGradBad = 8;
__device__ __forceinline__ long long fix_of(double v, int frac) { return (long long)rint(ldexp(v, frac)); }
__device__ __forceinline__ void fix128_add(unsigned long long* acc, unsigned long long lo, long long hi) {
    const unsigned long long old = __hip_atomic_fetch_add(acc, lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    hi += (old + lo < old) ? 1 : 0;   // carry out of the low word
    if (hi) __hip_atomic_fetch_add(acc + 1, (unsigned long long)hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void fix128_add(unsigned long long* acc, long long v) {
    fix128_add(acc, (unsigned long long)v, v < 0 ? -1ll : 0ll);
}
// v * 2^64 rounded to an integer, as {lo, hi} (|v| < 2^63)
__device__ __forceinline__ void fix128_of(double v, unsigned long long& lo, long long& hi) {
    const double r = rint(ldexp(v, 64));
    if (fabs(r) < 0x1p63) {
        const long long i = (long long)r;
        lo = (unsigned long long)i;
        hi = i < 0 ? -1 : 0;
    } else {   // r is a multiple of 2^11: r - h 2^64 is exact
        const double h = floor(ldexp(r, -64));
        hi = (long long)h;
        lo = (unsigned long long)(r - ldexp(h, 64));
    }
}
__device__ __forceinline__ double fix128_value(unsigned long long lo, long long hi, int frac) {
    const long long s = (long long)lo;
    if (hi == (s < 0 ? -1 : 0)) return ldexp(double(s), -frac);   // fits 64 bits: one rounding
    return ldexp(double(hi), 64 - frac) + ldexp(double(lo), -frac);
}
__device__ __forceinline__ void block_add_fix(long long* p, long long v) {
    __hip_atomic_fetch_add(reinterpret_cast<unsigned long long*>(p), (unsigned long long)v, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ unsigned long long ld_agent(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void flag_agent(unsigned long long* p, unsigned long long bits) {
    __hip_atomic_fetch_or(p, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Doubles as order-preserving 64-bit keys (an LDS atomicMin on the key is a
// min on the value): sign bit set -> all bits flipped, else the sign bit set.
__device__ __forceinline__ unsigned long long okey(double d) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(d);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double odec(unsigned long long k) {
    return __longlong_as_double((long long)((k >> 63) ? (k & 0x7fffffffffffffffull) : ~k));
}

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, kWave));
    return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, kWave));
    return v;
}
__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}

// [lo, lo+cnt): out-edges of node S that consume byte c (edges sorted by byte)
__device__ __forceinline__ void edge_range(const ModelView& m, int S, int c, int& lo, int& cnt) {
    const int b = m.o_ptr[S], e = m.o_ptr[S + 1];
    int l = b, h = e;
    while (l < h) {
        const int mid = (l + h) >> 1;
        if (int(m.o_byte[mid]) < c) l = mid + 1; else h = mid;
    }
    int l2 = l, h2 = e;
    while (l2 < h2) {
        const int mid = (l2 + h2) >> 1;
        if (int(m.o_byte[mid]) <= c) l2 = mid + 1; else h2 = mid;
    }
    lo = l;
    cnt = l2 - l;
}

// sum of the weights of node S's end edges (this iteration)
__device__ __forceinline__ double end_weight(const ModelView& m, int S) {
    double s = 0.0;
    for (int x = m.x_ptr[S]; x < m.x_ptr[S + 1]; ++x) s += m.ew[m.n_edges + x];
    return s;
}

struct Slab {
    double* alpha;
    double* beta;
    int* state;
    int* e_g;
    int* e_src;
    int* e_dst;
    int* fpos;
    int* epos;
    int* dsc;
    int* slot;
};

// Main-stream word of a trivial edge g (posterior 1): an edge with one
// parameter is stored as that parameter's index (log-weight w[j], gradient
// slot j); an edge without parameters (weight log 1) is not stored; an edge
// with several parameters (epsilon composites) by its multi-edge index.
__device__ __forceinline__ bool put_trivial(const ModelView& m, int g, bool write, void* stream, int wide,
                                            int64_t s_base, int& n_main) {
    const int np = m.pptr[g + 1] - m.pptr[g];
    if (np == 0) return false;
    if (write) {
        const int k = n_main + stream_hdr_words(wide);   // after the lane's group header
        if (wide) {
            const int v = np == 1 ? m.pidx[m.pptr[g]] : -(g + 2);
            static_cast<int32_t*>(stream)[s_base + int64_t(k >> 2) * 256 + (k & 3)] = v;
        } else {
            const int v = np == 1 ? m.pidx[m.pptr[g]] : 0x8000 + m.multi_of[g];
            static_cast<uint16_t*>(stream)[s_base + int64_t(k >> 3) * 512 + (k & 7)] = uint16_t(v);
        }
    }
    ++n_main;
    return true;
}

// Compiled stream of one string from its counted trellis (lane 0 only;
// beta > 0 marks live entries).  Trivial segments go to the main stream,
// bubbles to the bubble buffer.  Returns false when a bubble exceeds the
// kernel limits; the string then stays on the traversal path.
template <bool WRITE>
__device__ bool compile_walk(const Slab& sl, const ModelView& m, int L, int sidx, double p, int& n_main,
                             int& n_bub, int& n_nb, void* stream, int wide, int64_t s_base, int32_t* bub,
                             int64_t b_base, int32_t* bub_off, int32_t b_first) {
    long long* lid = reinterpret_cast<long long*>(sl.alpha);   // alpha is dead in counting mode
    n_main = 0;
    n_bub = 0;
    n_nb = 0;
    int a = 0, fa = 0;
    while (a <= L) {
        int b = a + 1, fbn = -1;
        for (; b <= L; ++b) {
            int cnt = 0, last = -1;
            for (int f = sl.fpos[b]; f < sl.fpos[b + 1]; ++f)
                if (sl.beta[f] > 0.0) { ++cnt; last = f; }
            if (cnt == 1) { fbn = last; break; }
        }
        const bool to_end = b > L;
        // trivial segments
        if (!to_end && b == a + 1) {
            int cnt = 0, ge = -1;
            for (int e = sl.epos[a]; e < sl.epos[a + 1]; ++e)
                if (sl.beta[sl.e_dst[e]] > 0.0) { ++cnt; ge = e; }
            if (cnt == 1) {
                put_trivial(m, sl.e_g[ge], WRITE, stream, wide, s_base, n_main);
                a = b;
                fa = fbn;
                continue;
            }
        }
        if (to_end && a == L) {
            const int S = sl.state[fa];
            if (m.x_ptr[S + 1] - m.x_ptr[S] == 1) {
                put_trivial(m, m.n_edges + m.x_ptr[S], WRITE, stream, wide, s_base, n_main);
                break;
            }
        }
        // bubble: local ids in position order
        int nodes = 0;
        lid[fa] = nodes++;
        const int last_pos = to_end ? L : b - 1;
        for (int pos = a + 1; pos <= last_pos; ++pos)
            for (int f = sl.fpos[pos]; f < sl.fpos[pos + 1]; ++f)
                if (sl.beta[f] > 0.0) lid[f] = nodes++;
        const int end_id = nodes++;   // the cut node b, or the virtual end node
        if (!to_end) lid[fbn] = end_id;
        const int e_hi = sl.epos[to_end ? L : b];
        int edges = 0;
        for (int e = sl.epos[a]; e < e_hi; ++e)
            if (sl.beta[sl.e_dst[e]] > 0.0) ++edges;
        if (to_end)
            for (int f = sl.fpos[L]; f < sl.fpos[L + 1]; ++f)
                if (sl.beta[f] > 0.0) edges += m.x_ptr[sl.state[f] + 1] - m.x_ptr[sl.state[f]];
        if (nodes > kMaxBubbleNodes || edges > kMaxBubbleEdges) return false;
        if (WRITE) {
            int64_t w = b_base + n_bub;
            bub_off[b_first + n_nb] = int32_t(w);
            bub[w++] = nodes | (edges << 16);
            bub[w++] = sidx;
            const unsigned long long pb = __double_as_longlong(p);
            bub[w++] = int32_t(uint32_t(pb));
            bub[w++] = int32_t(uint32_t(pb >> 32));
            for (int e = sl.epos[a]; e < e_hi; ++e) {
                const int h = sl.e_dst[e];
                if (!(sl.beta[h] > 0.0)) continue;
                bub[w++] = edge_code(m.pptr, m.pidx, sl.e_g[e], m.n_params);
                bub[w++] = int(lid[sl.e_src[e]]) | (int(lid[h]) << 16);
            }
            if (to_end) {
                for (int f = sl.fpos[L]; f < sl.fpos[L + 1]; ++f) {
                    if (!(sl.beta[f] > 0.0)) continue;
                    const int S = sl.state[f];
                    for (int x = m.x_ptr[S]; x < m.x_ptr[S + 1]; ++x) {
                        bub[w++] = edge_code(m.pptr, m.pidx, m.n_edges + x, m.n_params);
                        bub[w++] = int(lid[f]) | (end_id << 16);
                    }
                }
            }
        }
        n_bub += bubble_record_words(edges);
        ++n_nb;
        if (to_end) break;
        a = b;
        fa = fbn;
    }
    return true;
}

template <int MODE>
__global__ __launch_bounds__(256) void trav_kernel(TravArgs a) {
    constexpr bool COUNTING = MODE == MODE_COUNT || MODE == MODE_EMIT;
    constexpr bool MINM = MODE == MODE_MIN;   // beta holds the (min, x) forward as okey(log)
    if (a.halted && *a.halted) return;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = lane_id();
    const int wib = int(threadIdx.x) / kWave;
    const int wpb = int(blockDim.x) / kWave;
    const int gw = int(blockIdx.x) * wpb + wib;
    const int nw = int(gridDim.x) * wpb;

    unsigned char* base = smem + size_t(wib) * size_t(a.slab.bytes);
    Slab sl;
    sl.alpha = reinterpret_cast<double*>(base + a.lay.alpha);
    sl.beta = reinterpret_cast<double*>(base + a.lay.beta);
    sl.state = reinterpret_cast<int*>(base + a.lay.state);
    sl.e_g = reinterpret_cast<int*>(base + a.lay.eg);
    sl.e_src = reinterpret_cast<int*>(base + a.lay.esrc);
    sl.e_dst = reinterpret_cast<int*>(base + a.lay.edst);
    sl.fpos = reinterpret_cast<int*>(base + a.lay.fpos);
    sl.epos = reinterpret_cast<int*>(base + a.lay.epos);
    sl.dsc = reinterpret_cast<int*>(base + a.lay.dsc);
    sl.slot = reinterpret_cast<int*>(base + a.lay.slot);
    double* falpha = sl.alpha;
    double* fbeta = sl.beta;
    int* fstate = sl.state;
    int* slot = sl.slot;

    const ModelView& m = a.m;
    const int cap_f = a.slab.cap_f, cap_e = a.slab.cap_e;
    const bool want_back = !MINM && (!COUNTING || a.used || a.c_main || MODE == MODE_EMIT);
    // the (min, x) forward: min mode, or a weighted pass asked for the rmin
    // column too (beta holds the keys until the backward re-zeroes it)
    const bool track = MINM || (MODE == MODE_WEIGHTED && a.rmin_log != nullptr);
    unsigned long long* fkey = reinterpret_cast<unsigned long long*>(fbeta);

    for (int j = lane; j < m.n_nodes; j += kWave) st_rlx(&slot[j], -1);
    wave_sync();

    double ll_acc = 0.0;
    unsigned long long edges_acc = 0;

    for (int li = gw; li < a.n_list; li += nw) {
        const int sidx = a.list[li];
        const int64_t o0 = a.off[sidx];
        const int L = int(a.off[sidx + 1] - o0);
        const uint8_t* str = a.sym + o0;

        if (lane == 0) {
            fstate[0] = m.start;
            falpha[0] = 1.0;
            if (track) fkey[0] = okey(0.0);
            else fbeta[0] = 0.0;
            sl.fpos[0] = 0;
            sl.fpos[1] = 1;
            sl.epos[0] = 0;
            sl.dsc[0] = 0;
        }
        int nF = 1, nE = 0;
        bool ovf = false;
        bool alive = true;
        wave_sync();

        // ---------------- forward ----------------
        uint32_t chunk = 0;
        for (int i = 0; i < L; ++i) {
            if ((i & (kWave - 1)) == 0) {
                const int k = i + lane;
                chunk = k < L ? uint32_t(str[k]) : 0u;
            }
            const int c = __builtin_amdgcn_readlane(int(chunk), i & (kWave - 1));
            const int fb = sl.fpos[i];
            const int fe = nF;
            for (int fbase = fb; fbase < fe && !ovf; fbase += kWave) {
                const int f = fbase + lane;
                const bool act = f < fe;
                int lo = 0, cnt = 0;
                double af = 0.0, mf = 0.0;
                if (act) {
                    af = falpha[f];
                    if (track) mf = odec(fkey[f]);
                    edge_range(m, fstate[f], c, lo, cnt);
                }
                const int maxc = wave_max_i(cnt);
                for (int t = 0; t < maxc; ++t) {
                    const bool has = t < cnt;
                    const int g = lo + t;
                    int d = 0;
                    double v = 0.0;
                    if (has) {
                        d = m.o_dst[g];
                        v = COUNTING ? af : af * m.ew[g];
                    }
                    int slv = has ? ld_rlx(&slot[d]) : 0;
                    const bool need = has && slv < 0;
                    bool won = false;
                    if (need) won = atomicCAS(&slot[d], -1, -2) == -1;
                    const unsigned long long wm = __ballot(won);
                    const unsigned long long hm = __ballot(has);
                    const int nwon = __popcll(wm);
                    const int nhas = __popcll(hm);
                    if (nF + nwon > cap_f || nE + nhas > cap_e) {
                        ovf = true;
                        break;
                    }
                    if (won) {
                        const int idx = nF + rank_below(wm);
                        st_rlx(&slot[d], idx);
                        fstate[idx] = d;
                        falpha[idx] = 0.0;
                        if (track) fkey[idx] = okey(INFINITY);
                        else fbeta[idx] = 0.0;
                    }
                    nF += nwon;
                    wave_sync();
                    if (need) slv = ld_rlx(&slot[d]);
                    if (has) {
                        lds_add(&falpha[slv], v);
                        if (track && m.lw[g] > -INFINITY) atomicMin(&fkey[slv], okey(mf + m.lw[g]));
                        const int k = nE + rank_below(hm);
                        sl.e_g[k] = g;
                        sl.e_src[k] = f;
                        sl.e_dst[k] = slv;
                    }
                    nE += nhas;
                    wave_sync();
                }
            }
            wave_sync();
            if (ovf) break;
            // release the slot map entries of the new frontier, rescale it
            double mx = 0.0;
            for (int j = fe + lane; j < nF; j += kWave) {
                st_rlx(&slot[fstate[j]], -1);
                mx = fmax(mx, falpha[j]);
            }
            mx = wave_max(mx);
            int ex = 0;
            if (mx > 0.0) ex = __builtin_amdgcn_frexp_exp(mx);
            if (ex != 0)
                for (int j = fe + lane; j < nF; j += kWave) falpha[j] = ldexp(falpha[j], -ex);
            if (lane == 0) {
                sl.fpos[i + 2] = nF;
                sl.epos[i + 1] = nE;
                sl.dsc[i + 1] = ex;
            }
            wave_sync();
            if (nF == fe) {   // empty frontier: no accepting path
                alive = false;
                break;
            }
        }

        if (ovf) {
            // slot entries of the unfinished position may still be claimed
            for (int j = lane; j < m.n_nodes; j += kWave) st_rlx(&slot[j], -1);
            wave_sync();
            if (lane == 0) a.overflow[sidx] = 1;
            continue;
        }

        // ---------------- end + log q ----------------
        double qh = 0.0;
        int esum = 0;
        const int fl0 = alive ? sl.fpos[L] : 0;
        const int fl1 = alive ? nF : 0;
        for (int j = fl0 + lane; j < fl1; j += kWave) {
            const int S = fstate[j];
            qh += falpha[j] * (COUNTING ? m.node_end_count[S] : end_weight(m, S));
        }
        qh = wave_sum(qh);
        if (alive) {
            int es = 0;
            for (int j = 1 + lane; j <= L; j += kWave) es += sl.dsc[j];
            esum = wave_sum_i(es);
        }
        const double lq = qh > 0.0 ? log(qh) + kLn2 * double(esum) : -INFINITY;
        const double ps = COUNTING ? 0.0 : a.p[sidx];
        if (track) {
            double mn = INFINITY;
            for (int j = fl0 + lane; j < fl1; j += kWave) {
                const double we = end_weight(m, fstate[j]);
                if (we > 0.0) mn = fmin(mn, odec(fkey[j]) + log(we));
            }
            mn = -wave_max(-mn);
            if (lane == 0) a.rmin_log[sidx] = qh > 0.0 ? mn - lq : INFINITY;
            if (!MINM) {   // the backward accumulates into beta from zero
                for (int j = lane; j < nF; j += kWave) fbeta[j] = 0.0;
                wave_sync();
            }
        }
        if (lane == 0) {
            if (MODE == MODE_COUNT) {
                if (a.path_count) a.path_count[sidx] = qh > 0.0 ? ldexp(qh, esum) : 0.0;
                if (a.recognized) a.recognized[sidx] = qh > 0.0 ? 1 : 0;
                if (a.c_bub && !(qh > 0.0)) a.c_bub[sidx] = -1;
            } else if (MODE == MODE_WEIGHTED && a.logq) {
                a.logq[sidx] = lq;
            }
        }
        if (!COUNTING && !MINM) ll_acc += ps * lq;
        edges_acc += (unsigned long long)nE;
        if (!(qh > 0.0) || !want_back) continue;

        // ---------------- backward ----------------
        const double inv_q = 1.0 / qh;
        for (int j = fl0 + lane; j < fl1; j += kWave) {
            const int S = fstate[j];
            const double af = falpha[j];
            fbeta[j] = (COUNTING ? m.node_end_count[S] : end_weight(m, S)) * inv_q;
            for (int x = m.x_ptr[S]; x < m.x_ptr[S + 1]; ++x) {
                const int gx = m.n_edges + x;
                const double xi = af * (COUNTING ? 1.0 : m.ew[gx]) * inv_q;
                if (!(xi > 0.0)) continue;
                for (int k = m.pptr[gx]; k < m.pptr[gx + 1]; ++k) {
                    if (COUNTING) { if (a.used) a.used[m.pidx[k]] = 1; }
                    else global_add(&a.grad[m.pidx[k]], -ps * xi);
                }
            }
        }
        wave_sync();
        for (int i = L - 1; i >= 0; --i) {
            const double sc = ldexp(1.0, -sl.dsc[i + 1]);
            const int eb = sl.epos[i], ee = sl.epos[i + 1];
            for (int k = eb + lane; k < ee; k += kWave) {
                const int g = sl.e_g[k];
                const int f = sl.e_src[k];
                const int h = sl.e_dst[k];
                const double b = (COUNTING ? 1.0 : m.ew[g]) * fbeta[h] * sc;
                if (b != 0.0) lds_add(&fbeta[f], b);
                const double xi = falpha[f] * b;
                if (xi > 0.0) {
                    for (int q = m.pptr[g]; q < m.pptr[g + 1]; ++q) {
                        if (COUNTING) { if (a.used) a.used[m.pidx[q]] = 1; }
                        else global_add(&a.grad[m.pidx[q]], -ps * xi);
                    }
                }
            }
            wave_sync();
        }

        // ---------------- compiled stream ----------------
        if (COUNTING && (a.c_main || MODE == MODE_EMIT)) {
            if (lane == 0) {
                int n_main = 0, n_bub = 0, n_nb = 0;
                bool ok;
                if (MODE == MODE_EMIT)
                    ok = compile_walk<true>(sl, m, L, sidx, a.p[sidx], n_main, n_bub, n_nb, a.stream, a.wide,
                                            a.s_base[sidx], a.bub, a.b_base[sidx], a.bub_off, a.b_first[sidx]);
                else
                    ok = compile_walk<false>(sl, m, L, sidx, 0.0, n_main, n_bub, n_nb, nullptr, 0, 0, nullptr, 0,
                                             nullptr, 0);
                if (MODE == MODE_COUNT) {
                    a.c_main[sidx] = ok ? n_main : 0;
                    a.c_bub[sidx] = ok ? n_bub : -1;
                    a.c_nbub[sidx] = ok ? n_nb : 0;
                }
            }
            wave_sync();
        }
    }

    if (lane == 0) {
        if (!COUNTING && !MINM) a.ll_part[gw] = ll_acc;
        if (a.live_edges && edges_acc) atomicAdd(a.live_edges, edges_acc);
    }
}

// block-wide reductions (every thread gets the result)
__device__ __forceinline__ double block_sum(double v, double* red) {
    v = wave_sum(v);
    const int w = int(threadIdx.x) >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    double s = 0.0;
    for (int i = 0; i < int(blockDim.x) / kWave; ++i) s += red[i];
    return s;
}
__device__ __forceinline__ double block_max(double v, double* red) {
    v = wave_max(v);
    const int w = int(threadIdx.x) >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    double s = red[0];
    for (int i = 1; i < int(blockDim.x) / kWave; ++i) s = fmax(s, red[i]);
    return s;
}

// Tier 2 (fb_kernels.hpp WideArgs): one block per string, alpha per position
// as a dense node vector in global scratch.  Position i+1 is nonzero only on
// the destinations of byte c_i (the list D_c), so the forward writes exactly
// D_c and the backward visits exactly those nodes; the rows are zeroed per
// string because an in-edge gather reads arbitrary sources.
template <bool COUNTING, bool MINM = false>
__global__ __launch_bounds__(kWideBlock) void wide_kernel(WideArgs a) {
    if (a.halted && *a.halted) return;
    extern __shared__ __attribute__((aligned(16))) double gl[];   // [n_params] (weighted, grad_lds)
    __shared__ double red[kWideBlock / kWave];
    const int tid = int(threadIdx.x);
    const ModelView& m = a.m;
    const WideModel& W = a.w;
    const int N = m.n_nodes;
    double* A = a.scratch + int64_t(blockIdx.x) * a.scratch_stride;
    double* B = A + (int64_t(a.max_len) + 1) * N;             // [2][N]
    int* dsc = reinterpret_cast<int*>(B + 2 * int64_t(N));    // [max_len + 2]
    const bool lgrad = !COUNTING && !MINM && a.grad_lds;
    const bool track = MINM || (!COUNTING && a.rmin_log != nullptr);   // (min, x) forward in B's rows
    if (lgrad)
        for (int j = tid; j < m.n_params; j += kWideBlock) gl[j] = 0.0;
    double ll = 0.0;
    // parameters of edge g get -p xi (weighted) / are marked used (counting)
    auto credit = [&](int g, double xi, double ps) {
        for (int q = m.pptr[g]; q < m.pptr[g + 1]; ++q) {
            if (COUNTING) { if (a.used) a.used[m.pidx[q]] = 1; }
            else if (lgrad) block_add(&gl[m.pidx[q]], -ps * xi);
            else global_add(&a.grad[m.pidx[q]], -ps * xi);
        }
    };
    __syncthreads();
    for (int li = int(blockIdx.x); li < a.n_list; li += int(gridDim.x)) {
        const int sidx = a.list[li];
        const int64_t o0 = a.off[sidx];
        const int L = int(a.off[sidx + 1] - o0);
        const uint8_t* str = a.sym + o0;
        for (int64_t k = tid; k < (int64_t(L) + 1) * N; k += kWideBlock) A[k] = 0.0;
        __syncthreads();
        if (tid == 0) {
            A[m.start] = 1.0;
            dsc[0] = 0;
            if (track) B[m.start] = 0.0;   // (min, x) forward in log form, rolling over B's two rows
        }
        __syncthreads();
        bool alive = true;
        if (COUNTING && a.live_edges && tid == 0) {   // the edges the forward gathers over, per position
            unsigned long long ne = 0;
            for (int i = 0; i < L; ++i) ne += (unsigned long long)(W.e_ptr[W.c_ptr[str[i] + 1]] - W.e_ptr[W.c_ptr[str[i]]]);
            atomicAdd(a.live_edges, ne);
        }
        for (int i = 0; i < L; ++i) {
            const int c = str[i];
            const double* Ai = A + int64_t(i) * N;
            double* An = A + int64_t(i + 1) * N;
            const int cb = W.c_ptr[c], ce = W.c_ptr[c + 1];
            double mx = 0.0;
            for (int k = cb + tid; k < ce; k += kWideBlock) {
                double v = 0.0;
                for (int e = W.e_ptr[k]; e < W.e_ptr[k + 1]; ++e)
                    v += COUNTING ? Ai[W.e_src[e]] : Ai[W.e_src[e]] * m.ew[W.e_g[e]];
                An[W.dst[k]] = v;
                mx = fmax(mx, v);
                if (track) {
                    const double* Mi = B + int64_t(i & 1) * N;
                    double mn = INFINITY;
                    for (int e = W.e_ptr[k]; e < W.e_ptr[k + 1]; ++e) {
                        const double lwe = m.lw[W.e_g[e]];
                        if (Ai[W.e_src[e]] > 0.0 && lwe > -INFINITY) mn = fmin(mn, Mi[W.e_src[e]] + lwe);
                    }
                    B[int64_t((i + 1) & 1) * N + W.dst[k]] = mn;
                }
            }
            mx = block_max(mx, red);
            if (!(mx > 0.0)) {
                alive = false;
                break;
            }
            const int ex = __builtin_amdgcn_frexp_exp(mx);
            if (ex != 0)
                for (int k = cb + tid; k < ce; k += kWideBlock) An[W.dst[k]] = ldexp(An[W.dst[k]], -ex);
            if (tid == 0) dsc[i + 1] = ex;
            __syncthreads();
        }
        // nodes live at position j: the destinations of byte c_{j-1}; at 0 the start
        auto fr_begin = [&](int j) { return j == 0 ? 0 : W.c_ptr[str[j - 1]]; };
        auto fr_end = [&](int j) { return j == 0 ? 1 : W.c_ptr[str[j - 1] + 1]; };
        auto fr_node = [&](int j, int k) { return j == 0 ? m.start : W.dst[k]; };
        double qh = 0.0;
        int esum = 0;
        if (alive) {
            for (int k = fr_begin(L) + tid; k < fr_end(L); k += kWideBlock) {
                const int S = fr_node(L, k);
                qh += A[int64_t(L) * N + S] * (COUNTING ? m.node_end_count[S] : end_weight(m, S));
            }
            qh = block_sum(qh, red);
            double es = 0.0;
            for (int j = 1 + tid; j <= L; j += kWideBlock) es += double(dsc[j]);
            esum = int(block_sum(es, red));
        }
        const double lq = qh > 0.0 ? log(qh) + kLn2 * double(esum) : -INFINITY;
        const double ps = COUNTING ? 1.0 : a.p[sidx];
        if (track) {
            double mn = INFINITY;
            if (alive)
                for (int k = fr_begin(L) + tid; k < fr_end(L); k += kWideBlock) {
                    const int S = fr_node(L, k);
                    const double we = end_weight(m, S);
                    if (A[int64_t(L) * N + S] > 0.0 && we > 0.0) mn = fmin(mn, B[int64_t(L & 1) * N + S] + log(we));
                }
            mn = -block_max(-mn, red);
            if (tid == 0) a.rmin_log[sidx] = qh > 0.0 ? mn - lq : INFINITY;
            __syncthreads();
            if (MINM) continue;
        }
        if (tid == 0) {
            if (COUNTING) {
                if (a.path_count) a.path_count[sidx] = qh > 0.0 ? ldexp(qh, esum) : 0.0;
                if (a.recognized) a.recognized[sidx] = qh > 0.0 ? 1 : 0;
            } else {
                if (a.logq) a.logq[sidx] = lq;
                ll += ps * lq;
            }
        }
        if (!(qh > 0.0) || (COUNTING && !a.used)) {
            __syncthreads();
            continue;
        }
        // backward, scaled so that alpha_i beta_i is the posterior of the node
        const double inv_q = 1.0 / qh;
        {
            double* BL = B + int64_t(L & 1) * N;
            for (int k = fr_begin(L) + tid; k < fr_end(L); k += kWideBlock) {
                const int S = fr_node(L, k);
                const double af = A[int64_t(L) * N + S];
                BL[S] = (COUNTING ? m.node_end_count[S] : end_weight(m, S)) * inv_q;
                if (!(af > 0.0)) continue;
                for (int x = m.x_ptr[S]; x < m.x_ptr[S + 1]; ++x) {
                    const int gx = m.n_edges + x;
                    const double xi = af * (COUNTING ? 1.0 : m.ew[gx]) * inv_q;
                    if (xi > 0.0) credit(gx, xi, ps);
                }
            }
        }
        __syncthreads();
        for (int i = L - 1; i >= 0; --i) {
            const int c = str[i];
            const double sc = ldexp(1.0, -dsc[i + 1]);
            const double* Bn = B + int64_t((i + 1) & 1) * N;
            double* Bi = B + int64_t(i & 1) * N;
            for (int k = fr_begin(i) + tid; k < fr_end(i); k += kWideBlock) {
                const int S = fr_node(i, k);
                const double af = A[int64_t(i) * N + S];
                double bs = 0.0;
                if (af > 0.0) {
                    int lo, cnt;
                    edge_range(m, S, c, lo, cnt);
                    for (int g = lo; g < lo + cnt; ++g) {
                        const double b = (COUNTING ? 1.0 : m.ew[g]) * Bn[m.o_dst[g]] * sc;
                        bs += b;
                        const double xi = af * b;
                        if (xi > 0.0) credit(g, xi, ps);
                    }
                }
                Bi[S] = bs;
            }
            __syncthreads();
        }
    }
    if (!COUNTING && !MINM && tid == 0) a.ll_part[blockIdx.x] = ll;
    if (lgrad) {
        __syncthreads();
        for (int j = tid; j < m.n_params; j += kWideBlock)
            if (gl[j] != 0.0) global_add(&a.grad[j], gl[j]);
    }
}

// Tier 2, weighted, one wavefront per string, over the byte-pair tables
// (fb_kernels.hpp PairTables).  The trellis sums of wide_kernel<false>, laid
// out for the gather rate that bounds this pass: a block's waves each take a
// string from a work counter (16 strings per CU at once instead of one per
// 256-thread block); a step (a, b) walks the pair's edge list one edge per
// lane -- contiguous loads, no per-destination padding, only the edges whose
// source is live -- and sums into the wave's LDS rows (LDS atomics, issued in
// lane order within the wave: run-to-run stable); the forward keeps the
// current row in LDS and writes each row once to HBM (compact, coalesced) for
// the backward, which gathers alpha from that row and sums beta in LDS; no
// block barriers; the gradient in one LDS table per block when it fits,
// flushed once per launch.  The gradient and the log-likelihood are summed in
// fixed point (fix128_*): which wave drew which string changes the order of
// the adds, not their result, so an evaluation gives the same bits every run;
// the last block out turns the accumulators into doubles.
__device__ __forceinline__ void wave_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }
constexpr int kU = 4;   // wide2: edges per lane in flight
constexpr int kExpNone = -4096;   // below every frexp exponent of a double
// wave max of frexp exponents (kExpNone where a lane has none) by 13 ballots
// over the offset value's bits -- VALU compares, no LDS round trips
__device__ __forceinline__ int wave_max_exp(int e) {
    const unsigned u = unsigned(e - kExpNone);   // 0 .. 5120
    unsigned r = 0;
#pragma unroll
    for (int bit = 12; bit >= 0; --bit) {
        const unsigned c = r | (1u << bit);
        if (__ballot(u >= c)) r = c;
    }
    return int(r) + kExpNone;
}

template <bool TRACK>
__global__ __launch_bounds__(kWide2Block) void wide2_kernel(WideArgs a) {
    if (a.halted && *a.halted) return;
    extern __shared__ __attribute__((aligned(16))) double lds2[];
    __shared__ int last_block;
    const int lane = lane_id(), wv = int(threadIdx.x) >> 6, nwv = int(blockDim.x) >> 6;
    const ModelView& m = a.m;
    const PairTables& P = a.pt;
    const int K = P.K, MN = P.max_n;
    const bool lgrad = a.grad_lds != 0;
    long long* gl = reinterpret_cast<long long*>(lds2);   // fixed point, a.fix_frac fraction bits
    const int F = a.fix_frac;
    unsigned long long* gfix = a.fix;                       // [2 n_params]
    unsigned long long* llfix = a.fix + 2 * int64_t(m.n_params);
    double* rows = lds2 + (lgrad ? ((m.n_params + kWave + 1) & ~1) : 0) + int64_t(wv) * 2 * MN;
    double* R0 = rows;              // the two rows (alternating)
    double* R1 = rows + MN;
    if (lgrad)
        for (int j = int(threadIdx.x); j < m.n_params + kWave; j += int(blockDim.x)) gl[j] = 0;   // + spare slots
    __syncthreads();
    double* H = a.scratch2 + (int64_t(blockIdx.x) * nwv + wv) * a.stride2;
    double* Mg = H + 1 + int64_t(a.max_len) * MN;   // [2][max_n] min-forward rows (rmin column)
    int* ex = reinterpret_cast<int*>(Mg + 2 * int64_t(MN));   // [max_len + 2]
    auto add_fix = [&](int j, long long iv) {
        if (lgrad) block_add_fix(&gl[j], iv); else fix128_add(gfix + 2 * int64_t(j), iv);
    };
    auto credit = [&](int p0, int p1, int g, double v) {
        if (!(fabs(v) < INFINITY)) flag_agent(llfix + 2, kFixGradBad);
        const long long iv = fix_of(v, F);
        if (p0 >= 0) {
            add_fix(p0, iv);
            if (p1 >= 0) add_fix(p1, iv);
        } else if (p0 == -2) {
            for (int q = m.pptr[g]; q < m.pptr[g + 1]; ++q) add_fix(m.pidx[q], iv);
        }
    };
    for (;;) {
        int li = 0;
        if (lane == 0) li = int(__hip_atomic_fetch_add(a.ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        li = __builtin_amdgcn_readfirstlane(__shfl(li, 0, kWave));
        if (li >= a.n_list) break;
        const int sidx = a.list[li];
        const int64_t o0 = a.off[sidx];
        const int L = int(a.off[sidx + 1] - o0);
        const uint8_t* str = a.sym + o0;
        // step info, 64 steps at a time in lane registers (lane j: step c*64+j):
        // the pair (D of position p, byte p) range, |D(byte p)| (-1: no edge
        // consumes the byte), |D of position p|; read per step with readlane
        int veb = 0, vee = 0, vnb = 0, vna = 0;
        auto load_chunk = [&](int c) {
            const int p = c * kWave + lane;
            veb = vee = vnb = vna = 0;
            if (p < L) {
                const int bp = P.bidx[str[p]];
                const int apv = p == 0 ? K : P.bidx[str[p - 1]];
                if (bp < 0 || apv < 0) {
                    vnb = -1;
                } else {
                    veb = P.e_ptr[apv * K + bp];
                    vee = P.e_ptr[apv * K + bp + 1];
                    vnb = P.n[bp];
                    vna = P.n[apv];
                }
            }
        };
        // forward: the current row in A (LDS), every row also to H + roff (HBM)
        double* A = R0;
        double* Nx = R1;
        if (lane == 0) {
            A[0] = 1.0;
            H[0] = 1.0;
            ex[0] = 0;
            if (TRACK) Mg[0] = 0.0;
        }
        wave_sync();
        int exi = 0, esum = 0, last_n = 1;   // last_n: size of the current row
        int64_t roff = 0;
        bool alive = true;
        for (int i = 0; i < L; ++i) {
            if ((i & (kWave - 1)) == 0) load_chunk(i / kWave);
            const int nb = __builtin_amdgcn_readlane(vnb, i & (kWave - 1));
            if (nb < 0) {   // no edge consumes the byte
                alive = false;
                break;
            }
            const int eb = __builtin_amdgcn_readlane(veb, i & (kWave - 1));
            const int ee = __builtin_amdgcn_readlane(vee, i & (kWave - 1));
            const double sc = ldexp(1.0, -exi);
            const int64_t rn = roff + last_n;
            for (int d = lane; d < nb; d += kWave) Nx[d] = 0.0;
            wave_sync();
            for (int e0 = eb + lane; e0 < ((WFSA_KDBG(a.dbg) & 2) ? eb : ee); e0 += kU * kWave) {   // kU edges per lane in flight
                int sd[kU];
                double w[kU], r[kU];
#pragma unroll
                for (int u = 0; u < kU; ++u) {
                    const int e = e0 + u * kWave;
                    sd[u] = e < ee ? P.sd[e] : -1;
                    w[u] = e < ee ? P.w[e] : 0.0;
                }
                // branch-free: a padding lane adds 0 to its own entry (distinct banks)
                const int own = lane < nb ? lane : 0;
#pragma unroll
                for (int u = 0; u < kU; ++u) r[u] = A[sd[u] >= 0 ? (sd[u] & 0xffff) : 0];
#pragma unroll
                for (int u = 0; u < kU; ++u)
                    lds_add(&Nx[sd[u] >= 0 ? int(unsigned(sd[u]) >> 16) : own], sd[u] >= 0 ? r[u] * w[u] : 0.0);
            }
            wave_sync();
            int emx = kExpNone;   // the row's largest exponent (ballots, no LDS)
            for (int d = lane; d < nb; d += kWave) {
                const double v = Nx[d] * sc;
                Nx[d] = v;
                H[rn + d] = v;
                if (v > 0.0) emx = max(emx, __builtin_amdgcn_frexp_exp(v));
            }
            emx = wave_max_exp(emx);
            wave_sync();
            double* t = A; A = Nx; Nx = t;
            if (TRACK) {   // (min, x) forward: keys summed in the free row, sources' liveness from H
                unsigned long long* KN = reinterpret_cast<unsigned long long*>(Nx);
                const double* Mi = Mg + int64_t(i & 1) * MN;
                double* Mn = Mg + int64_t((i + 1) & 1) * MN;
                for (int d = lane; d < nb; d += kWave) KN[d] = ~0ull;
                wave_sync();
                for (int e = eb + lane; e < ee; e += kWave) {
                    const int4 en = P.ent[e];
                    const int src = en.x & 0xffff, dst = int(unsigned(en.x) >> 16);
                    const double lwe = P.lw[e];
                    if (H[roff + src] > 0.0 && lwe > -INFINITY) atomicMin(&KN[dst], okey(Mi[src] + lwe));
                }
                wave_sync();
                for (int d = lane; d < nb; d += kWave) Mn[d] = odec(KN[d]);
                wave_fence();   // the next min pass reads this row from H
            }
            roff = rn;
            last_n = nb;
            if (emx == kExpNone) {   // every node of the row is zero
                alive = false;
                break;
            }
            exi = emx;
            esum += exi;
            if (lane == 0) ex[i + 1] = exi;
        }
        double qh = 0.0;
        const double scL = ldexp(1.0, -exi);
        const int aL = L > 0 ? P.bidx[str[L - 1]] : K;
        const int nL = alive ? last_n : 0;
        const int32_t* dL = P.dl_node + P.dl_ptr[alive ? aL : K];
        for (int d = lane; d < nL; d += kWave) qh += A[d] * scL * end_weight(m, dL[d]);
        qh = wave_sum(qh);
        const double lq = qh > 0.0 ? log(qh) + kLn2 * double(esum) : -INFINITY;
        const double ps = a.p[sidx];
        if (TRACK) {
            double mn = INFINITY;
            for (int d = lane; d < nL; d += kWave) {
                const double we = end_weight(m, dL[d]);
                if (A[d] > 0.0 && we > 0.0) mn = fmin(mn, Mg[int64_t(L & 1) * MN + d] + log(we));
            }
            mn = -wave_max(-mn);
            if (lane == 0) a.rmin_log[sidx] = qh > 0.0 ? mn - lq : INFINITY;
        }
        if (lane == 0) {
            if (a.logq) a.logq[sidx] = lq;
            const double c = ps * lq;
            if (fabs(c) < 0x1p62) {
                unsigned long long lo;
                long long hi;
                fix128_of(c, lo, hi);
                fix128_add(llfix, lo, hi);
            } else {
                flag_agent(llfix + 2, c != c ? kFixLlNan : (c < 0.0 ? kFixLlNegInf : kFixLlPosInf));
            }
        }
        if (!(qh > 0.0) || (WFSA_KDBG(a.dbg) & 1)) continue;
        wave_fence();   // the rows in H (and ex) are visible to every lane
        // backward (beta scaled so that alpha_i beta_i is the node posterior):
        // beta_{i+1} in Bn (LDS), beta_i summed into Bi (LDS)
        const double inv_q = 1.0 / qh;
        double* Bn = R1;
        double* Bi = R0;
        for (int d = lane; d < nL; d += kWave) {
            const int S = dL[d];
            const double af = A[d] * scL;
            Bn[d] = end_weight(m, S) * inv_q;
            if (!(af > 0.0)) continue;
            for (int x = m.x_ptr[S]; x < m.x_ptr[S + 1]; ++x) {
                const int gx = m.n_edges + x;
                const double xi = af * m.ew[gx] * inv_q;
                if (xi > 0.0) credit(-2, -1, gx, -ps * xi);
            }
        }
        wave_sync();
        int ex_next = exi, vex = 0;
        for (int i = L - 1; i >= 0; --i) {
            if (i == L - 1 || (i & (kWave - 1)) == kWave - 1) {   // this step's chunk (steps and row exponents)
                load_chunk(i / kWave);
                const int p = (i / kWave) * kWave + lane;
                vex = p <= L ? ex[p] : 0;
            }
            const int eb = __builtin_amdgcn_readlane(veb, i & (kWave - 1));
            const int ee = __builtin_amdgcn_readlane(vee, i & (kWave - 1));
            const int na = __builtin_amdgcn_readlane(vna, i & (kWave - 1));
            const int ex_i = __builtin_amdgcn_readlane(vex, i & (kWave - 1));
            roff -= na;
            const double sc = ldexp(1.0, -ex_next), sci = ldexp(1.0, -ex_i);
            for (int d = lane; d < na; d += kWave) Bi[d] = 0.0;
            wave_sync();
            for (int e0 = eb + lane; e0 < ((WFSA_KDBG(a.dbg) & 2) ? eb : ee); e0 += kU * kWave) {
                int4 en[kU];
                double w[kU], af[kU], bn[kU];
#pragma unroll
                for (int u = 0; u < kU; ++u) {
                    const int e = e0 + u * kWave;
                    en[u] = e < ee ? P.ent[e] : make_int4(-1, 0, -1, -1);
                    w[u] = e < ee ? P.w[e] : 0.0;
                }
                // branch-free: a padding / dead lane adds 0 to its own entries
                const int own = lane < na ? lane : 0;
#pragma unroll
                for (int u = 0; u < kU; ++u) af[u] = en[u].x >= 0 ? H[roff + (en[u].x & 0xffff)] * sci : 0.0;
#pragma unroll
                for (int u = 0; u < kU; ++u) bn[u] = Bn[en[u].x >= 0 ? int(unsigned(en[u].x) >> 16) : 0];
#pragma unroll
                for (int u = 0; u < kU; ++u) {
                    const bool on = af[u] > 0.0;
                    const double bv = on ? w[u] * bn[u] * sc : 0.0;
                    lds_add(&Bi[on ? (en[u].x & 0xffff) : own], bv);
                    const double v = -ps * (af[u] * bv);
                    if (lgrad) {   // two parameters per edge in one table; the rest to this lane's spare slot
                        const int spare = m.n_params + lane;
                        if (on && !(fabs(v) < INFINITY)) flag_agent(llfix + 2, kFixGradBad);
                        const long long iv = on ? fix_of(v, F) : 0;
                        block_add_fix(&gl[on && en[u].z >= 0 ? en[u].z : spare], iv);
                        block_add_fix(&gl[on && en[u].w >= 0 ? en[u].w : spare], iv);
                        if (on && en[u].z == -2) credit(-2, -1, en[u].y, v);
                    } else if (on && af[u] * bv > 0.0) {
                        credit(en[u].z, en[u].w, en[u].y, v);
                    }
                }
            }
            wave_sync();
            double* t = Bn; Bn = Bi; Bi = t;
            ex_next = ex_i;
        }
        wave_sync();
    }
    __syncthreads();   // every wave of the block is past its last string
    if (lgrad)
        for (int j = int(threadIdx.x); j < m.n_params; j += int(blockDim.x))
            if (gl[j] != 0) fix128_add(gfix + 2 * int64_t(j), gl[j]);
    __threadfence();   // this thread's accumulator adds before the block's arrival
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned d = __hip_atomic_fetch_add(a.ctr + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        last_block = d + 1 == gridDim.x;
    }
    __syncthreads();
    if (!last_block) return;
    // the last block out: the sums into doubles, the accumulators and
    // counters zeroed for the next launch
    __threadfence();
    const unsigned long long flags = ld_agent(llfix + 2);
    for (int j = int(threadIdx.x); j < m.n_params; j += int(blockDim.x)) {
        unsigned long long* q = gfix + 2 * int64_t(j);
        const unsigned long long lo = ld_agent(q), hi = ld_agent(q + 1);
        if (flags & kFixGradBad) a.grad[j] = __builtin_nan("");
        else if (lo | hi) a.grad[j] += fix128_value(lo, (long long)hi, F);
        if (lo | hi) {
            st_agent(q, 0);
            st_agent(q + 1, 0);
        }
    }
    for (int b = int(threadIdx.x); b < int(gridDim.x); b += int(blockDim.x)) {
        double v = 0.0;
        if (b == 0) {
            const bool ninf = flags & kFixLlNegInf, pinf = flags & kFixLlPosInf;
            v = (flags & kFixLlNan) || (ninf && pinf) ? __builtin_nan("")
                : ninf ? -INFINITY : pinf ? INFINITY : fix128_value(ld_agent(llfix), (long long)ld_agent(llfix + 1), 64);
            st_agent(llfix, 0);
            st_agent(llfix + 1, 0);
            st_agent(llfix + 2, 0);
            __hip_atomic_store(a.ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a.ctr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        a.ll_part[b] = v;   // the log-likelihood in the first slot
    }
}

// Tier 2, weighted, one wavefront per string, pulling (fb_kernels.hpp
// PullTables): the forward sums each destination of D(b) over its in-edges
// and the backward each source of D(a) over its out-edges, a lane per node
// -- no LDS atomics on the rows, each node's sum in one fixed order -- and a
// wave needs one LDS row, not two: a lane keeps its finished node sums in a
// shift register (the newest in acc[0]) until the whole wave has read the
// row, then writes them over it.  With the gradient table that fits 16 waves
// per block where wide2_kernel fits 12.  The backward reads alpha of an
// edge's source from the row the forward wrote to HBM (the lane's consecutive
// entries share a source: one row read per source: the pair's first entry row
// lists each lane's sources).  Scaling, alpha history, fixed-point
// gradient / log-likelihood and the last block's conversion as wide2_kernel.
#ifndef WFSA_PULL_UF
#define WFSA_PULL_UF 8   // forward entries per lane in flight
#endif
#ifndef WFSA_PULL_UB
#define WFSA_PULL_UB 2   // backward entries per lane in flight
#endif
// timing variants only (make var, never the release build): 1 no alpha
// gather in the backward, 2 no gradient credits, 3 no alpha history at all
// (neither the forward's row stores nor the backward's gather)
#ifndef WFSA_PULL_EXP
#define WFSA_PULL_EXP 0
#endif
// 1: the alpha history in slot layout (fb_kernels.hpp wide2_rows): the forward
// copies each finished row from LDS into the slots the backward's lanes read,
// 64-lane coalesced both ways, and the backward needs no source lists.  As
// fast as the compact rows, bitwise equal (profiles/r05/famb/alpha_history.txt)
#ifndef WFSA_PULL_SLOT
#define WFSA_PULL_SLOT 0
#endif
template <int NI, bool TRACK>
__global__ __launch_bounds__(kPullBlock) void wave_pull_kernel(WideArgs a) {
    constexpr int kUF = TRACK && WFSA_PULL_UF > 4 ? 4 : WFSA_PULL_UF, kUB = WFSA_PULL_UB;   // (the min forward's registers)
    if (a.halted && *a.halted) return;
    extern __shared__ __attribute__((aligned(16))) double lds2[];
    __shared__ int last_block;
    const int lane = lane_id(), wv = int(threadIdx.x) >> 6, nwv = int(blockDim.x) >> 6;
    const ModelView& m = a.m;
    const PairTables& P = a.pt;
    const PullTables& Q = a.pl;
    const int K = P.K, MN = P.max_n;
    const bool lgrad = a.grad_lds != 0;
    long long* gl = reinterpret_cast<long long*>(lds2);   // fixed point, a.fix_frac fraction bits
    const int F = a.fix_frac;
    unsigned long long* gfix = a.fix;                       // [2 n_params]
    unsigned long long* llfix = a.fix + 2 * int64_t(m.n_params);
    double* R = lds2 + (lgrad ? ((m.n_params + kWave + 1) & ~1) : 0) + int64_t(wv) * MN;   // the wave's row
    if (lgrad)
        for (int j = int(threadIdx.x); j < m.n_params + kWave; j += int(blockDim.x)) gl[j] = 0;   // + spare slots
    __syncthreads();
    double* H = a.scratch2 + (int64_t(blockIdx.x) * nwv + wv) * a.stride2;
    double* Mg = H + a.hrows2;   // [2][max_n] min-forward rows (rmin column)
    int* ex = reinterpret_cast<int*>(Mg + 2 * int64_t(MN));   // [max_len + 2]
    constexpr int kS = NI * kWave;   // a row of the slot layout
    auto add_fix = [&](int j, long long iv) {
        if (lgrad) block_add_fix(&gl[j], iv); else fix128_add(gfix + 2 * int64_t(j), iv);
    };
    auto credit = [&](int p0, int p1, int g, double v) {
        if (!(fabs(v) < INFINITY)) flag_agent(llfix + 2, kFixGradBad);
        const long long iv = fix_of(v, F);
        if (p0 >= 0) {
            add_fix(p0, iv);
            if (p1 >= 0) add_fix(p1, iv);
        } else if (p0 == -2) {
            for (int q = m.pptr[g]; q < m.pptr[g + 1]; ++q) add_fix(m.pidx[q], iv);
        }
    };
    // slot layout: the lane's backward sources (16-bit row indices, 0xffff
    // none) of row 0 of a pair's backward entries, copied from the LDS row
    auto put_slots = [&](int64_t row, int4 sl) {
        const unsigned sw[4] = {unsigned(sl.x), unsigned(sl.y), unsigned(sl.z), unsigned(sl.w)};
#pragma unroll
        for (int k = 0; k < NI; ++k) {
            const unsigned u = (sw[k >> 1] >> (16 * (k & 1))) & 0xffffu;
            H[row * kS + k * kWave + lane] = u != 0xffffu ? R[u] : 0.0;
        }
    };
    for (;;) {
        int li = 0;
        if (lane == 0) li = int(__hip_atomic_fetch_add(a.ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        li = __builtin_amdgcn_readfirstlane(__shfl(li, 0, kWave));
        if (li >= a.n_list) break;
        const int sidx = a.list[li];
        const int64_t o0 = a.off[sidx];
        const int L = int(a.off[sidx + 1] - o0);
        const uint8_t* str = a.sym + o0;
        // step info, 64 steps at a time in lane registers (lane j: step c*64+j):
        // the pair's forward base / T and backward base / T, |D(byte p)| (-1:
        // no edge consumes the byte), |D of position p|; read with readlane
        // (slot layout: vbn, the backward base of step p + 1)
        int vfb = 0, vft = 0, vbb = 0, vbt = 0, vnb = 0, vna = 0, vq = 0, vbn = 0;
        auto load_chunk = [&](int c) {
            const int p = c * kWave + lane;
            vfb = vft = vbb = vbt = vnb = vna = vq = vbn = 0;
            if (WFSA_PULL_SLOT && p + 1 < L) {
                const int b1 = P.bidx[str[p + 1]], a1 = P.bidx[str[p]];
                if (b1 >= 0 && a1 >= 0) vbn = Q.info[a1 * K + b1].z;
            }
            if (p < L) {
                const int bp = P.bidx[str[p]];
                const int apv = p == 0 ? K : P.bidx[str[p - 1]];
                if (bp < 0 || apv < 0) {
                    vnb = -1;
                } else {
                    vq = apv * K + bp;
                    const int4 inf = Q.info[vq];
                    vfb = inf.x;
                    vft = inf.y;
                    vbb = inf.z;
                    vbt = inf.w;
                    vnb = P.n[bp];
                    vna = P.n[apv];
                }
            }
        };
        if (lane == 0) {
            R[0] = 1.0;
            H[0] = 1.0;
            ex[0] = 0;
            if (TRACK) Mg[0] = 0.0;
        }
        wave_sync();
        int exi = 0, esum = 0, last_n = 1;   // last_n: size of the current row
        int64_t roff = 0;
        bool alive = true;
        // a step's header and first kUF entries per lane are loaded during the
        // step before (they depend only on the string's bytes), so the step's
        // chain starts at its LDS gathers, not at a global load
        int pcd[kUF];
        double pw[kUF], plw[kUF];
        int4 pdh = make_int4(-1, -1, -1, -1);
        auto load_entries = [&](int fb, int T, int t0, int* cd, double* w, double* lwv) {
#pragma unroll
            for (int u = 0; u < kUF; ++u) {
                const int t = t0 + u;
                const int64_t e = int64_t(fb) + int64_t(t) * kWave + lane;
                cd[u] = t < T ? Q.fcode[e] : 0;
                w[u] = t < T ? Q.fw[e] : 0.0;
                if (TRACK) lwv[u] = t < T ? Q.flw[e] : -INFINITY;
            }
        };
        auto prefetch = [&](int i) {   // step i's info is in the chunk registers
            const int ii = i & (kWave - 1);
            if (__builtin_amdgcn_readlane(vnb, ii) < 0) return;
            pdh = Q.fhdr[int64_t(__builtin_amdgcn_readlane(vq, ii)) * kWave + lane];
            load_entries(__builtin_amdgcn_readlane(vfb, ii), __builtin_amdgcn_readlane(vft, ii), 0, pcd, pw, plw);
        };
#ifndef WFSA_PULL_NOSTEPPF
        if (L > 0) {
            load_chunk(0);
            prefetch(0);
        }
#elif WFSA_PULL_SLOT
#error "the slot layout loads the first chunk before the forward"
#endif
        if (WFSA_PULL_SLOT && L > 0 && __builtin_amdgcn_readlane(vnb, 0) >= 0)   // the start row's slots
            put_slots(0, Q.bent[int64_t(__builtin_amdgcn_readlane(vbb, 0)) + lane]);
        for (int i = 0; i < L; ++i) {
#ifdef WFSA_PULL_NOSTEPPF
            if ((i & (kWave - 1)) == 0) load_chunk(i / kWave);
            prefetch(i);
#endif
            const int ii = i & (kWave - 1);
            const int nb = __builtin_amdgcn_readlane(vnb, ii);
            if (nb < 0) {   // no edge consumes the byte
                alive = false;
                break;
            }
            const int fb = __builtin_amdgcn_readlane(vfb, ii);
            const int T = __builtin_amdgcn_readlane(vft, ii);
            const int4 dh = pdh;   // the lane's destinations
            // slot layout: the sources of step i + 1's backward, in flight over this step
            const int4 slf = WFSA_PULL_SLOT && i + 1 < L
                ? Q.bent[int64_t(__builtin_amdgcn_readlane(vbn, ii)) + lane] : make_int4(-1, -1, -1, -1);
            const double sc = ldexp(1.0, -exi);
            const int64_t rn = roff + last_n;
            const double* Mi = Mg + int64_t(i & 1) * MN;
            double* Mn = Mg + int64_t((i + 1) & 1) * MN;
            double acc[NI], amin[NI];
#pragma unroll
            for (int k = 0; k < NI; ++k) {
                acc[k] = 0.0;
                amin[k] = INFINITY;
            }
            double s = 0.0, smin = INFINITY;
            for (int t0 = 0; t0 < T; t0 += kUF) {
                int cd[kUF];
                double w[kUF], r[kUF], lwv[kUF], mv[kUF];
                if (t0 == 0) {
#pragma unroll
                    for (int u = 0; u < kUF; ++u) {
                        cd[u] = pcd[u];
                        w[u] = pw[u];
                        lwv[u] = plw[u];
                    }
                } else {
                    load_entries(fb, T, t0, cd, w, lwv);
                }
#pragma unroll
                for (int u = 0; u < kUF; ++u) r[u] = R[cd[u] & 0xffff];
                if (TRACK) {
#pragma unroll
                    for (int u = 0; u < kUF; ++u) mv[u] = Mi[cd[u] & 0xffff];
                }
#pragma unroll
                for (int u = 0; u < kUF; ++u) {
                    if (t0 + u >= T) break;   // uniform
                    s += r[u] * w[u];
                    if (TRACK && r[u] > 0.0 && lwv[u] > -INFINITY) smin = fmin(smin, mv[u] + lwv[u]);
                    const bool f = cd[u] < 0;   // the node's last entry
#pragma unroll
                    for (int k = 0; k + 1 < NI; ++k) {   // (a queue: the lane's first node ends up in acc[0])
                        acc[k] = f ? acc[k + 1] : acc[k];
                        if (TRACK) amin[k] = f ? amin[k + 1] : amin[k];
                    }
                    acc[NI - 1] = f ? s : acc[NI - 1];
                    s = f ? 0.0 : s;
                    if (TRACK) {
                        amin[NI - 1] = f ? smin : amin[NI - 1];
                        smin = f ? INFINITY : smin;
                    }
                }
            }
#ifndef WFSA_PULL_NOSTEPPF
            if (i + 1 < L) {   // the next step's header and entries, in flight over this step's row write
                if (((i + 1) & (kWave - 1)) == 0) load_chunk((i + 1) / kWave);
                prefetch(i + 1);
            }
#endif
            wave_sync();   // every lane has read the row
            int emx = kExpNone;   // the row's largest exponent (ballots, no LDS)
            {
                // the lane's n nodes sit in acc[NI - n .. NI) in its item order: node k
                // (header slot k) in acc[NI - n + k]; shift them down to acc[k]
                const unsigned hw[4] = {unsigned(dh.x), unsigned(dh.y), unsigned(dh.z), unsigned(dh.w)};
                int n = 0;
#pragma unroll
                for (int k = 0; k < NI; ++k) n += ((hw[k >> 1] >> (16 * (k & 1))) & 0xffffu) != 0xffffu ? 1 : 0;
#pragma unroll
                for (int r = 0; r < NI; ++r) {   // NI - n rounds of a one-place shift
                    const bool sh = r < NI - n;
#pragma unroll
                    for (int k = 0; k + 1 < NI; ++k) {
                        acc[k] = sh ? acc[k + 1] : acc[k];
                        if (TRACK) amin[k] = sh ? amin[k + 1] : amin[k];
                    }
                }
#pragma unroll
                for (int k = 0; k < NI; ++k) {
                    const unsigned d = (hw[k >> 1] >> (16 * (k & 1))) & 0xffffu;
                    if (d == 0xffffu) continue;
                    const double v = acc[k] * sc;
                    R[d] = v;
                    if (WFSA_PULL_EXP != 3 && !WFSA_PULL_SLOT) H[rn + d] = v;
                    if (v > 0.0) emx = max(emx, __builtin_amdgcn_frexp_exp(v));
                    if (TRACK) Mn[d] = amin[k];
                }
            }
            emx = wave_max_exp(emx);
            wave_sync();
            if (WFSA_PULL_SLOT && WFSA_PULL_EXP != 3 && i + 1 < L) put_slots(i + 1, slf);
            if (TRACK) wave_fence();   // the next step reads the min row from HBM
            roff = rn;
            last_n = nb;
            if (emx == kExpNone) {   // every node of the row is zero
                alive = false;
                break;
            }
            exi = emx;
            esum += exi;
            if (lane == 0) ex[i + 1] = exi;
        }
        double qh = 0.0;
        const double scL = ldexp(1.0, -exi);
        const int aL = L > 0 ? P.bidx[str[L - 1]] : K;
        const int nL = alive ? last_n : 0;
        const int32_t* dL = P.dl_node + P.dl_ptr[alive ? aL : K];
        for (int d = lane; d < nL; d += kWave) qh += R[d] * scL * end_weight(m, dL[d]);
        qh = wave_sum(qh);
        const double lq = qh > 0.0 ? log(qh) + kLn2 * double(esum) : -INFINITY;
        const double ps = a.p[sidx];
        if (TRACK) {
            double mn = INFINITY;
            for (int d = lane; d < nL; d += kWave) {
                const double we = end_weight(m, dL[d]);
                if (R[d] > 0.0 && we > 0.0) mn = fmin(mn, Mg[int64_t(L & 1) * MN + d] + log(we));
            }
            mn = -wave_max(-mn);
            if (lane == 0) a.rmin_log[sidx] = qh > 0.0 ? mn - lq : INFINITY;
        }
        if (lane == 0) {
            if (a.logq) a.logq[sidx] = lq;
            const double c = ps * lq;
            if (fabs(c) < 0x1p62) {
                unsigned long long lo;
                long long hi;
                fix128_of(c, lo, hi);
                fix128_add(llfix, lo, hi);
            } else {
                flag_agent(llfix + 2, c != c ? kFixLlNan : (c < 0.0 ? kFixLlNegInf : kFixLlPosInf));
            }
        }
        if (!(qh > 0.0)) continue;
        wave_fence();   // the rows in H (and ex) are visible to every lane
        // backward (beta scaled so that alpha_i beta_i is the node posterior):
        // beta_L from the end weights, over the last alpha row (each lane
        // reads, then overwrites, its own entries)
        const double inv_q = 1.0 / qh;
        for (int d = lane; d < nL; d += kWave) {
            const int S = dL[d];
            const double af = R[d] * scL;
            R[d] = end_weight(m, S) * inv_q;
            if (!(af > 0.0)) continue;
            for (int x = m.x_ptr[S]; x < m.x_ptr[S + 1]; ++x) {
                const int gx = m.n_edges + x;
                const double xi = af * m.ew[gx] * inv_q;
                if (xi > 0.0) credit(-2, -1, gx, -ps * xi);
            }
        }
        wave_sync();
        int ex_next = exi, vex = 0;
        int4 sl_next = make_int4(-1, -1, -1, -1);   // the next (lower) step's source list, loaded a step early
        bool have_next = false;
        // entries: each round's loads issued before the round before it is
        // summed, the next step's first round during this step's row write
        // (within a chunk of step registers)
        int4 ben[kUB];
        double bwn[kUB];
        bool have_ent = false;
        auto load_b = [&](int bb, int T, int t0, int4* en, double* w) {
#pragma unroll
            for (int u = 0; u < kUB; ++u) {
                const int t = t0 + u;
                const int64_t e = int64_t(bb) + int64_t(t + 1) * kWave + lane;   // (row 0: the lane's sources)
                en[u] = t < T ? Q.bent[e] : make_int4(0, -1, -1, -1);
                w[u] = t < T ? Q.bw[e] : 0.0;
            }
        };
        for (int i = L - 1; i >= 0; --i) {
            if (i == L - 1 || (i & (kWave - 1)) == kWave - 1) {   // this step's chunk (steps and row exponents)
                load_chunk(i / kWave);
                const int p = (i / kWave) * kWave + lane;
                vex = p <= L ? ex[p] : 0;
            }
            const int ii = i & (kWave - 1);
            const int bb = __builtin_amdgcn_readlane(vbb, ii);
            const int T = __builtin_amdgcn_readlane(vbt, ii);
            const int na = __builtin_amdgcn_readlane(vna, ii);
            const int ex_i = __builtin_amdgcn_readlane(vex, ii);
            roff -= na;
            const double sc = ldexp(1.0, -ex_next), sci = ldexp(1.0, -ex_i);
            double acc[NI], av[NI];
            int dd[NI];
            if (WFSA_PULL_SLOT && WFSA_PULL_EXP != 1 && WFSA_PULL_EXP != 3) {   // the row's slots, coalesced
#pragma unroll
                for (int k = 0; k < NI; ++k) av[k] = H[int64_t(i) * kS + k * kWave + lane] * sci;
            } else {   // alpha of the lane's sources, in its item order (row 0 of the pair's entries)
                const int4 sl = have_next ? sl_next : Q.bent[int64_t(bb) + lane];
#ifdef WFSA_PULL_NOPF   // (layout-variant builds: no prefetch)
                have_next = false;
#else
                have_next = (ii & (kWave - 1)) != 0;   // step i - 1 in this chunk of step registers
#endif
                if (have_next) sl_next = Q.bent[int64_t(__builtin_amdgcn_readlane(vbb, ii - 1)) + lane];
                const unsigned sw[4] = {unsigned(sl.x), unsigned(sl.y), unsigned(sl.z), unsigned(sl.w)};
#pragma unroll
                for (int k = 0; k < NI; ++k) {
                    const unsigned u = (sw[k >> 1] >> (16 * (k & 1))) & 0xffffu;
                    av[k] = WFSA_PULL_EXP == 1 || WFSA_PULL_EXP == 3 ? (u != 0xffffu ? 1e-3 * sci : 0.0)
                                               : (u != 0xffffu ? H[roff + int(u)] * sci : 0.0);
                }
            }
#pragma unroll
            for (int k = 0; k < NI; ++k) {
                acc[k] = 0.0;
                dd[k] = -1;
            }
            double s = 0.0;
#ifdef WFSA_PULL_NOSTEPPF
            have_ent = false;
#endif
            if (!have_ent) load_b(bb, T, 0, ben, bwn);
            for (int t0 = 0; t0 < T; t0 += kUB) {
                int4 en[kUB];
                double w[kUB], bn[kUB];
#ifdef WFSA_PULL_NOSTEPPF   // (A/B variant: round 3's load, gather, sum)
                if (t0 > 0) load_b(bb, T, t0, ben, bwn);
#endif
#pragma unroll
                for (int u = 0; u < kUB; ++u) {
                    en[u] = ben[u];
                    w[u] = bwn[u];
                }
#ifndef WFSA_PULL_NOSTEPPF
                if (t0 + kUB < T) load_b(bb, T, t0 + kUB, ben, bwn);
#endif
#pragma unroll
                for (int u = 0; u < kUB; ++u) bn[u] = R[en[u].x & 0xffff];
#pragma unroll
                for (int u = 0; u < kUB; ++u) {
                    if (t0 + u >= T) break;   // uniform
                    const double afu = av[0];   // alpha of the lane's current source
                    const bool on = afu > 0.0;
                    const double bv = on ? w[u] * bn[u] * sc : 0.0;
                    s += bv;
                    const double v = -ps * (afu * bv);
                    if (WFSA_PULL_EXP == 2) {
                    } else if (lgrad) {   // two parameters per edge in one table; the rest to this lane's spare slot
                        const int spare = m.n_params + lane;
                        if (on && !(fabs(v) < INFINITY)) flag_agent(llfix + 2, kFixGradBad);
                        const long long iv = on ? fix_of(v, F) : 0;
                        block_add_fix(&gl[on && en[u].z >= 0 ? en[u].z : spare], iv);
                        block_add_fix(&gl[on && en[u].w >= 0 ? en[u].w : spare], iv);
                        if (on && en[u].z == -2) credit(-2, -1, en[u].y, v);
                    } else if (on && afu * bv > 0.0) {
                        credit(en[u].z, en[u].w, en[u].y, v);
                    }
                    const bool f = en[u].x < 0;   // the source's last entry
#pragma unroll
                    for (int k = NI - 1; k > 0; --k) {
                        acc[k] = f ? acc[k - 1] : acc[k];
                        dd[k] = f ? dd[k - 1] : dd[k];
                    }
#pragma unroll
                    for (int k = 0; k + 1 < NI; ++k) av[k] = f ? av[k + 1] : av[k];
                    av[NI - 1] = f ? 0.0 : av[NI - 1];
                    acc[0] = f ? s : acc[0];
                    dd[0] = f ? ((en[u].x >> 16) & 0x7fff) : dd[0];
                    s = f ? 0.0 : s;
                }
            }
#ifndef WFSA_PULL_NOSTEPPF
            have_ent = ii != 0;   // step i - 1 in this chunk of step registers
#endif
            if (have_ent)
                load_b(__builtin_amdgcn_readlane(vbb, ii - 1), __builtin_amdgcn_readlane(vbt, ii - 1), 0, ben, bwn);
            wave_sync();   // every lane has read the row
#pragma unroll
            for (int k = 0; k < NI; ++k)
                if (dd[k] >= 0) R[dd[k]] = acc[k];
            wave_sync();
            ex_next = ex_i;
        }
        wave_sync();
    }
    __syncthreads();   // every wave of the block is past its last string
    if (lgrad)
        for (int j = int(threadIdx.x); j < m.n_params; j += int(blockDim.x))
            if (gl[j] != 0) fix128_add(gfix + 2 * int64_t(j), gl[j]);
    __threadfence();   // this thread's accumulator adds before the block's arrival
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned d = __hip_atomic_fetch_add(a.ctr + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        last_block = d + 1 == gridDim.x;
    }
    __syncthreads();
    if (!last_block) return;
    __threadfence();
    const unsigned long long flags = ld_agent(llfix + 2);
    for (int j = int(threadIdx.x); j < m.n_params; j += int(blockDim.x)) {
        unsigned long long* q = gfix + 2 * int64_t(j);
        const unsigned long long lo = ld_agent(q), hi = ld_agent(q + 1);
        if (flags & kFixGradBad) a.grad[j] = __builtin_nan("");
        else if (lo | hi) a.grad[j] += fix128_value(lo, (long long)hi, F);
        if (lo | hi) {
            st_agent(q, 0);
            st_agent(q + 1, 0);
        }
    }
    for (int b = int(threadIdx.x); b < int(gridDim.x); b += int(blockDim.x)) {
        double v = 0.0;
        if (b == 0) {
            const bool ninf = flags & kFixLlNegInf, pinf = flags & kFixLlPosInf;
            v = (flags & kFixLlNan) || (ninf && pinf) ? __builtin_nan("")
                : ninf ? -INFINITY : pinf ? INFINITY : fix128_value(ld_agent(llfix), (long long)ld_agent(llfix + 1), 64);
            st_agent(llfix, 0);
            st_agent(llfix + 1, 0);
            st_agent(llfix + 2, 0);
            __hip_atomic_store(a.ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a.ctr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        a.ll_part[b] = v;   // the log-likelihood in the first slot
    }
}

__global__ __launch_bounds__(256) void pull_weights_kernel(const int32_t* __restrict__ g, int64_t n, int64_t n_lw,
                                                           const double* __restrict__ ew,
                                                           const double* __restrict__ lw, double* __restrict__ w,
                                                           double* __restrict__ lw_out) {
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        const int32_t k = g[i];
        w[i] = k >= 0 ? ew[k] : 0.0;
        if (i < n_lw) lw_out[i] = k >= 0 ? lw[k] : -INFINITY;
    }
}

__global__ __launch_bounds__(256) void pair_weights_kernel(const int4* ent, int64_t n, const double* ew,
                                                           const double* lw, double* pw) {
    const int64_t stride = int64_t(gridDim.x) * blockDim.x;
    for (int64_t e = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; e < n; e += stride) {
        const int g = ent[e].y;
        pw[e] = ew[g];
        pw[n + e] = lw[g];
    }
}

__device__ __forceinline__ void wave_fence_hf() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }

// Hessian second-order term per bubble (fb_kernels.hpp HfArgs).  The
// bubble's local node ids are in position order, so its edges (listed by
// source position) are already topologically sorted.
__global__ __launch_bounds__(kHfBlock) void hf_kernel(HfArgs a) {
    constexpr int NW = kHfBlock / kWave;
    constexpr int NN = kMaxBubbleNodes;
    __shared__ double s_w[NW][kMaxBubbleEdges + 1];
    __shared__ int s_sd[NW][kMaxBubbleEdges + 1];
    __shared__ int s_code[NW][kMaxBubbleEdges + 1];
    __shared__ double s_R[NW][NN * NN];
    __shared__ double s_ab[NW][2 * NN];
    const int lane = lane_id(), w = int(threadIdx.x) / kWave;
    const int b = int(blockIdx.x) * NW + w;
    if (b >= a.n_bubbles) return;
    const int32_t* rec = a.bub + a.bub_off[b];
    const int nodes = rec[0] & 0xffff, edges = rec[0] >> 16;
    const double p = __longlong_as_double((long long)(uint32_t(rec[2])) | ((long long)(uint32_t(rec[3])) << 32));
    double* lw = s_w[w];
    int* sd = s_sd[w];
    int* code = s_code[w];
    double* R = s_R[w];
    double* A = s_ab[w];
    double* B = s_ab[w] + NN;
    for (int e = lane; e < edges; e += kWave) {
        const int c = rec[4 + 2 * e];
        sd[e] = rec[5 + 2 * e];
        code[e] = c;
        double wgt;
        if (c >= 0) {
            wgt = a.ewp[c];
        } else {
            const int g = -c - 2;
            double t = 0.0;
            for (int q = a.m.pptr[g]; q < a.m.pptr[g + 1]; ++q) t += a.w[a.m.pidx[q]];
            wgt = exp(t);
        }
        lw[e] = wgt;
    }
    // R(u, v) = sum of the path weights from u to v: lane v owns column v
    for (int u = 0; u < nodes; ++u)
        if (lane < nodes) R[u * NN + lane] = u == lane ? 1.0 : 0.0;
    wave_sync();
    if (lane < nodes) {
        for (int e = edges - 1; e >= 0; --e) {
            const int src = sd[e] & 0xffff, dst = sd[e] >> 16;
            R[src * NN + lane] += lw[e] * R[dst * NN + lane];
        }
    }
    wave_sync();
    if (lane < nodes) {   // alpha = R(0, .) (paths from the entry), beta = R(., end)
        A[lane] = R[lane];
        B[lane] = R[lane * NN + nodes - 1];
    }
    wave_sync();
    const double Z = B[0];
    const double inv_z = 1.0 / Z;
    // slots: every ordered edge pair (e, f), every parameter pair (j in e,
    // k in f) with j <= k, in nesting order; lanes take the (e, f) pairs
    auto params = [&](int c, int* out) {   // the edge's parameters (in list order)
        if (c >= 0) {
            if (c < a.m.n_params) { out[0] = c; return 1; }
            return 0;
        }
        const int g = -c - 2;
        int n = 0;
        for (int q = a.m.pptr[g]; q < a.m.pptr[g + 1] && n < 8; ++q) out[n++] = a.m.pidx[q];
        return n;
    };
    // slot offsets of the ordered pairs are prefix sums over (e, f); lane 0
    // walks them in order and the lanes fill pair by pair
    int64_t slot = a.slot_base[b];
    for (int ef0 = 0; ef0 < edges * edges; ef0 += kWave) {
        const int ef = ef0 + lane;
        int pe[8], pf[8], ne = 0, nf = 0, cnt = 0;
        double v = 0.0;
        if (ef < edges * edges) {
            const int e = ef / edges, f = ef % edges;
            ne = params(code[e], pe);
            nf = params(code[f], pf);
            for (int x = 0; x < ne; ++x)
                for (int y = 0; y < nf; ++y) cnt += pe[x] <= pf[y];
            const int se = sd[e] & 0xffff, de = sd[e] >> 16, sf = sd[f] & 0xffff, df = sd[f] >> 16;
            const double Pe = A[se] * lw[e] * B[de] * inv_z;
            const double Pf = A[sf] * lw[f] * B[df] * inv_z;
            double both;
            if (e == f) both = Pe;
            else if (R[de * NN + sf] > 0.0) both = A[se] * lw[e] * R[de * NN + sf] * lw[f] * B[df] * inv_z;
            else if (R[df * NN + se] > 0.0) both = A[sf] * lw[f] * R[df * NN + se] * lw[e] * B[de] * inv_z;
            else both = 0.0;
            v = p * (both - Pe * Pf);
        }
        // exclusive prefix of cnt over the lanes (pair order = lane order)
        int incl = cnt;
#pragma unroll
        for (int o = 1; o < kWave; o <<= 1) {
            const int t = __shfl_up(incl, o, kWave);
            if (lane >= o) incl += t;
        }
        int64_t my = slot + (incl - cnt);
        for (int x = 0; x < ne; ++x)
            for (int y = 0; y < nf; ++y)
                if (pe[x] <= pf[y]) a.slot_val[my++] = v;
        slot += __shfl(incl, kWave - 1, kWave);
    }
}

// pattern entry t = its slots' sum, in slot order (deterministic)
// weight of combined edge g (exp of its parameters' sum)
__device__ __forceinline__ double hf_edge_weight(const ModelView& m, const double* wt, int g) {
    double t = 0.0;
    for (int q = m.pptr[g]; q < m.pptr[g + 1]; ++q) t += wt[m.pidx[q]];
    return exp(t);
}

// (local index, count) of edge g's parameters in V (ascending), at most 8
__device__ __forceinline__ int hf_local(const ModelView& m, const int32_t* V, int nV, int g, int* kk, double* cc) {
    int n = 0;
    for (int q = m.pptr[g]; q < m.pptr[g + 1] && n < 8; ++q) {
        const int j = m.pidx[q];
        int lo = 0, hi = nV;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (V[mid] < j) lo = mid + 1; else hi = mid;
        }
        if (lo < nV && V[lo] == j) {
            int t = 0;
            while (t < n && kk[t] != lo) ++t;
            if (t == n) {
                kk[n] = lo;
                cc[n] = 0.0;
                ++n;
            }
            cc[t] += 1.0;
        }
    }
    return n;
}

// hf_trav_kernel (fb_kernels.hpp HfTravArgs): one wavefront per string;
// lane l owns the V columns l, l + 64, ... (R of them) of G and the rows of A.
template <int R>
__device__ void hf_trav_string(const HfTravArgs& a, int li, int lane, double* Bt) {
    const ModelView& m = a.m;
    const WideModel& W = a.w;
    const int N = m.n_nodes;
    const int VM = a.vm;
    double* Be = Bt + (int64_t(a.max_len) + 1) * N;                // [max_len + 1] their exponents
    double* Ar = Be + (a.max_len + 1);                             // [2][N] scaled alpha rows
    double* Gr = Ar + 2 * int64_t(N);                              // [2][N][VM] scaled G rows
    double* Am = Gr + 2 * int64_t(N) * VM;                         // [VM][VM]
    double* Dm = Am + int64_t(VM) * VM;                            // [VM][VM]
    double* Mv = Dm + int64_t(VM) * VM;                            // [VM]
    const int4 it = a.list[li];
    const int sidx = it.x, nV = it.z;
    const int32_t* V = a.vlist + it.y;
    const int64_t o0 = a.off[sidx];
    const int L = int(a.off[sidx + 1] - o0);
    const uint8_t* str = a.sym + o0;
    // backward: beta rows, each scaled to a power of two (exponent kept)
    for (int S = lane; S < N; S += kWave) {
        double b = 0.0;
        for (int x = m.x_ptr[S]; x < m.x_ptr[S + 1]; ++x) b += hf_edge_weight(m, a.wt, m.n_edges + x);
        Bt[int64_t(L) * N + S] = b;
    }
    wave_fence_hf();
    auto rescale = [&](double* row, int n) -> int {
        double mx = 0.0;
        for (int S = lane; S < n; S += kWave) mx = fmax(mx, row[S]);
        mx = wave_max(mx);
        const int e = mx > 0.0 ? __builtin_amdgcn_frexp_exp(mx) : 0;
        if (e != 0)
            for (int S = lane; S < n; S += kWave) row[S] = ldexp(row[S], -e);
        wave_fence_hf();
        return e;
    };
    int eb = rescale(Bt + int64_t(L) * N, N);
    if (lane == 0) Be[L] = double(eb);
    for (int i = L - 1; i >= 0; --i) {
        const int c = str[i];
        const double* Bn = Bt + int64_t(i + 1) * N;
        for (int S = lane; S < N; S += kWave) {
            int lo, cnt;
            edge_range(m, S, c, lo, cnt);
            double b = 0.0;
            for (int g = lo; g < lo + cnt; ++g) b += hf_edge_weight(m, a.wt, g) * Bn[m.o_dst[g]];
            Bt[int64_t(i) * N + S] = b;
        }
        wave_fence_hf();
        eb += rescale(Bt + int64_t(i) * N, N);
        if (lane == 0) Be[i] = double(eb);
    }
    wave_fence_hf();
    // Z = beta_0(start); true beta_i = Bt_i 2^Be[i]
    const double zt = Bt[m.start];
    const int ez = int(Be[0]);
    if (!(zt > 0.0)) return;   // not recognized (the host lists recognized strings only)
    // forward: alpha and G rows (both scaled by 2^-ea), A, D, m
    for (int64_t j = lane; j < int64_t(VM) * VM; j += kWave) {
        Am[j] = 0.0;
        Dm[j] = 0.0;
    }
    for (int j = lane; j < VM; j += kWave) Mv[j] = 0.0;
    for (int S = lane; S < N; S += kWave) Ar[S] = S == m.start ? 1.0 : 0.0;
    for (int64_t q = lane; q < int64_t(N) * VM; q += kWave) Gr[q] = 0.0;
    wave_fence_hf();
    int ea = 0;
    int kk[8];
    double cc[8];
    // one edge: alpha / G into its destination (an, gn), A rows and D, m
    auto edge = [&](const double* Gi, int S, double as, int g, double coef, double* gn) {
        const int n = hf_local(m, V, nV, g, kk, cc);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int j = lane + r * kWave;
            const double gs = Gi[int64_t(S) * VM + j];
            double cl = 0.0;
            for (int t = 0; t < n; ++t) {
                cl += kk[t] == j ? cc[t] : 0.0;
                if (j < nV) Am[int64_t(j) * VM + kk[t]] += coef * gs * cc[t];
            }
            if (gn) gn[r] += gs + as * cl;   // (times the edge weight by the caller)
        }
        if (lane == 0) {
            const double pe = coef * as;
            for (int t = 0; t < n; ++t) {
                Mv[kk[t]] += pe * cc[t];
                for (int u = 0; u < n; ++u) Dm[int64_t(kk[t]) * VM + kk[u]] += pe * cc[t] * cc[u];
            }
        }
    };
    for (int i = 0; i < L; ++i) {
        const int c = str[i];
        const double* Ai = Ar + int64_t(i & 1) * N;
        double* An = Ar + int64_t((i + 1) & 1) * N;
        const double* Gi = Gr + int64_t(i & 1) * N * VM;
        double* Gn = Gr + int64_t((i + 1) & 1) * N * VM;
        const double* Bn = Bt + int64_t(i + 1) * N;
        // P(e) = a~ w b~ 2^(ea + Be[i+1] - ez) / z~
        const double f = ldexp(1.0, ea + int(Be[i + 1]) - ez) / zt;
        for (int S = lane; S < N; S += kWave) An[S] = 0.0;
        for (int64_t q = lane; q < int64_t(N) * VM; q += kWave) Gn[q] = 0.0;
        wave_fence_hf();
        for (int k = W.c_ptr[c]; k < W.c_ptr[c + 1]; ++k) {   // destinations of byte c, in order
            const int T = W.dst[k];
            double an = 0.0, gn[R];
#pragma unroll
            for (int r = 0; r < R; ++r) gn[r] = 0.0;
            const double bT = Bn[T];
            for (int e = W.e_ptr[k]; e < W.e_ptr[k + 1]; ++e) {
                const int S = W.e_src[e], g = W.e_g[e];
                const double as = Ai[S];
                if (!(as > 0.0)) continue;
                const double we = hf_edge_weight(m, a.wt, g);
                double ge[R];
#pragma unroll
                for (int r = 0; r < R; ++r) ge[r] = 0.0;
                edge(Gi, S, as, g, we * bT * f, ge);
                an += we * as;
#pragma unroll
                for (int r = 0; r < R; ++r) gn[r] += we * ge[r];
            }
            if (lane == 0) An[T] = an;
#pragma unroll
            for (int r = 0; r < R; ++r) Gn[int64_t(T) * VM + lane + r * kWave] = gn[r];
        }
        wave_fence_hf();
        // rescale alpha and G together
        double mx = 0.0;
        for (int S = lane; S < N; S += kWave) mx = fmax(mx, An[S]);
        mx = wave_max(mx);
        const int e = mx > 0.0 ? __builtin_amdgcn_frexp_exp(mx) : 0;
        if (e != 0) {
            for (int S = lane; S < N; S += kWave) An[S] = ldexp(An[S], -e);
            for (int64_t q = lane; q < int64_t(N) * VM; q += kWave) Gn[q] = ldexp(Gn[q], -e);
        }
        ea += e;
        wave_fence_hf();
    }
    {   // end edges (beta = 1 past them)
        const double* Ai = Ar + int64_t(L & 1) * N;
        const double* Gi = Gr + int64_t(L & 1) * N * VM;
        const double f = ldexp(1.0, ea - ez) / zt;
        for (int S = 0; S < N; ++S) {
            const double as = Ai[S];
            if (!(as > 0.0)) continue;
            for (int x = m.x_ptr[S]; x < m.x_ptr[S + 1]; ++x) {
                const int g = m.n_edges + x;
                edge(Gi, S, as, g, hf_edge_weight(m, a.wt, g) * f, nullptr);
            }
        }
    }
    wave_fence_hf();
    // slots (a <= b, row-major): p_s Cov(a, b)
    const double ps = a.p[sidx];
    const int64_t base = a.slot_base[li];
    for (int ra = lane; ra < nV; ra += kWave) {
        int64_t q = base + int64_t(ra) * nV - int64_t(ra) * (ra - 1) / 2;   // sum_{r < ra} (nV - r)
        for (int rb = ra; rb < nV; ++rb, ++q) {
            const double e2 = Dm[int64_t(ra) * VM + rb] + Am[int64_t(ra) * VM + rb] + Am[int64_t(rb) * VM + ra];
            a.slot_val[q] = ps * (e2 - Mv[ra] * Mv[rb]);
        }
    }
    wave_fence_hf();
}

template <int R>
__global__ __launch_bounds__(kHfBlock) void hf_trav_kernel(HfTravArgs a) {
    const int lane = lane_id();
    const int gw = int(blockIdx.x) * (kHfBlock / kWave) + int(threadIdx.x) / kWave;
    const int nwv = int(gridDim.x) * (kHfBlock / kWave);
    double* Bt = a.scratch + int64_t(gw) * a.stride;               // [(max_len + 1)][N] scaled beta rows
    for (int li = gw; li < a.n_list; li += nwv) hf_trav_string<R>(a, li, lane, Bt);
}

__global__ __launch_bounds__(256) void hf_sum_kernel(HfArgs a) {
    const int64_t t = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (t >= a.n_pattern) return;
    double s = 0.0;
    for (int64_t q = a.t_ptr[t]; q < a.t_ptr[t + 1]; ++q) s += a.slot_val[a.t_slot[q]];
    a.out[t] = s;
}

// Main streams: one lane per string, 64 strings of similar stream length per
// wavefront.  Every word is an edge on all of the string's paths (posterior
// 1): log q accumulates its log-weight and its parameters get -p_s.  A
// single-parameter word j reads w[j] and adds to gradient slot j; with
// TABLES == 2 both live in LDS (w staged per block), so the only global
// traffic is the stream itself, one 16-byte chunk per lane per load (the next
// chunk in flight while the current one is applied).  Multi-parameter words
// (rare) read the edge's log-weight and parameter list from global memory.
// Groups are dealt to waves in snake order (longest first) to balance them.
//
// GRAD == false is the per-iteration form: a trivial word's posterior is 1
// whatever the weights, so its gradient contribution -p_s is a constant of
// the corpus (the reference keeps the same constant for unique-path corpora,
// grad_aux = -P^T p, src/QuasiNewtonLearner.cpp:95-101).  It is accumulated
// once (GRAD == true, at preparation) and added by the tail kernel; every
// iteration then only sums the words' log-weights per string (log q) -- no
// atomics.  TABLES then means: 2 or 1 = w staged in LDS, 0 = w from global.
template <int TABLES, bool WIDE, bool GRAD>   // GRAD: TABLES 2 w + grad in LDS, 1 grad in LDS, 0 none
__global__ __launch_bounds__(1024) void fbc_kernel(CompiledArgs a) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* gacc = lds;                              // [n_params] when GRAD && TABLES >= 1
    double* wl = GRAD ? lds + a.n_params : lds;      // [n_params] when w is staged
    constexpr bool W_LDS = GRAD ? TABLES == 2 : TABLES >= 1;
    constexpr bool G_LDS = GRAD && TABLES >= 1;
    const int lane = lane_id();
    const int wpb = int(blockDim.x) / kWave;
    const int gw = int(blockIdx.x) * wpb + int(threadIdx.x) / kWave;
    const int nw = int(gridDim.x) * wpb;
    if (TABLES >= 1) {
        for (int j = int(threadIdx.x); j < a.n_params; j += int(blockDim.x)) {
            if (G_LDS) gacc[j] = 0.0;
            if (W_LDS) wl[j] = a.w[j];
        }
        // this block's slice of the per-edge weights (bubbles and the
        // traversal fallback read them after this launch), and the zeroed
        // result vector
        const int64_t per = (a.n_comb + gridDim.x - 1) / gridDim.x;
        const int64_t e_end = min(a.n_comb, per * int64_t(blockIdx.x + 1));
        for (int64_t g = per * int64_t(blockIdx.x) + threadIdx.x; g < e_end; g += blockDim.x) {
            const int32_t b = a.m.pptr[g], e = a.m.pptr[g + 1];
            double sum = 0.0;
            for (int32_t k = b; k < e; ++k) sum += a.w[a.m.pidx[k]];
            a.lw_out[g] = sum;
            a.ew_out[g] = exp(sum);
            a.erec_out[g] = EdgeRec{sum, e > b ? a.m.pidx[b] : 0, e - b};
        }
        if (blockIdx.x == 0)
            for (int j = int(threadIdx.x); j <= a.n_params; j += int(blockDim.x)) a.out[j] = 0.0;
        __syncthreads();
    }
    const double* wsrc = W_LDS ? wl : a.w;
    constexpr int PER = WIDE ? 4 : 8;   // words per 16-byte chunk
    const uint4 pad = make_uint4(0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu);
    double ll_acc = 0.0;

    // the gradient pass runs one wavefront per block: its accumulation (LDS,
    // or the block's own slab in HBM) sees one instruction stream, so the
    // slabs -- summed in slab order afterwards -- are the same bits every time
    double* gslab = a.gpart + size_t(blockIdx.x) * size_t(a.n_params);
    auto apply = [&](int j_single, int g_multi, double p, double& acc) {
        if (j_single >= 0) {
            acc += wsrc[j_single];
            if (G_LDS) block_add(&gacc[j_single], -p);
            else if (GRAD) global_add(&gslab[j_single], -p);
        } else if (g_multi >= 0) {
            for (int q = a.m.pptr[g_multi]; q < a.m.pptr[g_multi + 1]; ++q) {
                const int j = a.m.pidx[q];
                acc += wsrc[j];
                if (G_LDS) block_add(&gacc[j], -p);
                else if (GRAD) global_add(&gslab[j], -p);
            }
        }
    };

    for (int round = 0;; ++round) {
        const int grp = round * nw + ((round & 1) ? (nw - 1 - gw) : gw);
        if (grp >= a.n_groups) break;
        const int s = a.l_str[grp * kWave + lane];
        const int nch = (a.l_len[grp * kWave + lane] + stream_hdr_words(WIDE) + PER - 1) / PER;
        const int gch = a.g_len[grp];
        const uint4* st = a.stream + a.g_base[grp] + lane;
        const double p = s >= 0 ? a.p[s] : 0.0;
        double acc = 0.0;
        // ring of D chunks in flight per lane (~64 KB per CU with 16 waves)
        constexpr int D = 4;
        uint4 buf[D];
#pragma unroll
        for (int d = 0; d < D; ++d) buf[d] = d < nch ? st[int64_t(kWave) * d] : pad;
        for (int c0 = 0; c0 < gch; c0 += D) {
#pragma unroll
            for (int d = 0; d < D; ++d) {
                const int c = c0 + d;
                if (c >= gch) break;
                uint4 cur = buf[d];
                buf[d] = (c + D < nch) ? st[int64_t(kWave) * (c + D)] : pad;
                if (c == 0) {   // the group header reads as padding
                    cur.x = 0xffffffffu;
                    cur.y = 0xffffffffu;
                    cur.z = WIDE ? 0xffffffffu : (cur.z | 0xffffu);
                }
                const uint32_t v[4] = {cur.x, cur.y, cur.z, cur.w};
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    if (WIDE) {
                        const int x = int(v[i]);
                        apply(x, x < -1 ? -(x + 2) : -1, p, acc);
                    } else {
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            const int x = int((v[i] >> (16 * h)) & 0xffffu);
                            if (x < 0x8000) apply(x, -1, p, acc);
                            else if (x != 0xffff) apply(-1, a.m.multi_edge[x - 0x8000], p, acc);
                        }
                    }
                }
            }
        }
        if (s >= 0) {
            ll_acc += p * acc;
            if (a.logq) a.logq[s] = acc;
        }
    }
    ll_acc = wave_sum(ll_acc);
    if (lane == 0) a.ll_part[gw] = ll_acc;
    if (G_LDS) {   // this block's partial gradient, summed by slab_sum_kernel
        __syncthreads();
        for (int j = int(threadIdx.x); j < a.n_params; j += int(blockDim.x)) gslab[j] = gacc[j];
    }
}

// Prologue of the per-iteration stream kernel (no other kernel runs before
// it): this block's slice of the per-edge weights (bubbles and the traversal
// fallback read them after this launch) and, by block 0, the zeroed result.
__device__ __forceinline__ void edge_weight_slice(const CompiledArgs& a, int bid, int nblk) {
    const int64_t per = (a.n_comb + nblk - 1) / nblk;
    const int64_t e_end = min(a.n_comb, per * int64_t(bid + 1));
    for (int64_t g = per * int64_t(bid) + threadIdx.x; g < e_end; g += blockDim.x) {
        const int32_t b = a.m.pptr[g], e = a.m.pptr[g + 1];
        double sum = 0.0;
        for (int32_t k = b; k < e; ++k) sum += a.w[a.m.pidx[k]];
        a.lw_out[g] = sum;
        a.ew_out[g] = exp(sum);
        a.erec_out[g] = EdgeRec{sum, e > b ? a.m.pidx[b] : 0, e - b};
    }
    if (bid == 0)
        for (int j = int(threadIdx.x); j <= a.n_params; j += int(blockDim.x)) a.out[j] = 0.0;
}


// Bubbles.  Local forward from the bubble's first cut, local backward from
// its last cut; an edge's posterior is alpha(src) w beta(dst) / Z, -p_s times
// it goes to the edge's slot(s) in the parameter-major contribution array;
// log Z joins the string's log q.  The weight of an edge is exp(w[code]) from
// the per-iteration table ewp (edge_code).
//
// Small bubbles, one lane each: the bubble's quads are loaded in one round
// (structure-of-arrays, coalesced), the weights gathered in a second, and
// alpha/beta of its at most 8 nodes live in registers, addressed through a
// tree of selects on the node id.
// r[i] for i < 8 as a tree of selects on the bits of i (a compare chain is
// re-formed into an indexed scratch load by the compiler)
template <int N>
__device__ __forceinline__ double reg_get(const double (&r)[N], int i) {
    static_assert(N == 4 || N == 8, "register bubbles have 4 or 8 nodes");
    const bool b0 = i & 1, b1 = i & 2;
    const double s0 = b0 ? r[1] : r[0], s1 = b0 ? r[3] : r[2];
    const double t0 = b1 ? s1 : s0;
    if constexpr (N == 4) {
        return t0;
    } else {
        const double s2 = b0 ? r[5] : r[4], s3 = b0 ? r[7] : r[6];
        const double t1 = b1 ? s3 : s2;
        return (i & 4) ? t1 : t0;
    }
}
template <int N>
__device__ __forceinline__ void reg_add(double (&r)[N], int i, double v) {
#pragma unroll
    for (int k = 0; k < N; ++k) r[k] = i == k ? r[k] + v : r[k];
}

// A small bubble of class (N nodes, RE edges): quads of bubble b at
// tbl[k * n + b] -- [header], RE/2 x [(code, sd) x 2], RE/4 x [slot x 4].
// The partner's value at butterfly level d (1, 2, ..., 32) of an aligned
// group sum, without the LDS crossbar (ds_bpermute): DPP within a 16-lane
// row, the gfx950 permlane swaps across rows.  At level d every aligned
// d-lane group already holds one value, so the half-row / row mirrors pair
// the same groups as xor 4 / xor 8 (tools/micro/permlane_probe.hip: the swaps'
// lane mapping).
template <int D>
__device__ __forceinline__ double bfly_partner(double v) {
    const int lo = __double2loint(v), hi = __double2hiint(v);
    if constexpr (D == 16 || D == 32) {
        const auto l = D == 16 ? __builtin_amdgcn_permlane16_swap(lo, lo, false, false)
                               : __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
        const auto h = D == 16 ? __builtin_amdgcn_permlane16_swap(hi, hi, false, false)
                               : __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
        const bool up = (lane_id() & D) != 0;   // (out[0]: the lower row's lanes, out[1]: the upper row's)
        return __hiloint2double(up ? h[0] : h[1], up ? l[0] : l[1]);
    } else {
        constexpr int ctrl = D == 1 ? 0xB1 : D == 2 ? 0x4E : D == 4 ? 0x141 : 0x140;   // quad_perm / half mirror / mirror
        return __hiloint2double(__builtin_amdgcn_mov_dpp(hi, ctrl, 0xF, 0xF, false),
                                __builtin_amdgcn_mov_dpp(lo, ctrl, 0xF, 0xF, false));
    }
}
// v summed over the lane's aligned group of 2^k lanes, levels below kmax
// (wave-uniform) exchanged: every lane of the group ends with the same bits
__device__ __forceinline__ double group_sum(double v, int k, int kmax) {
    if (kmax >= 1) { const double t = bfly_partner<1>(v); if (k >= 1) v += t; }
    if (kmax >= 2) { const double t = bfly_partner<2>(v); if (k >= 2) v += t; }
    if (kmax >= 3) { const double t = bfly_partner<4>(v); if (k >= 3) v += t; }
    if (kmax >= 4) { const double t = bfly_partner<8>(v); if (k >= 4) v += t; }
    if (kmax >= 5) { const double t = bfly_partner<16>(v); if (k >= 5) v += t; }
    if (kmax >= 6) { const double t = bfly_partner<32>(v); if (k >= 6) v += t; }
    return v;
}

// The big bubbles' wave priority: above the small-bubble waves' 2 -- a big
// bubble is one wave's serial sweep, and the small-bubble waves on its SIMD
// otherwise issue first (c3 26.6 vs 26.9 us per step, with the rmin column
// 29.6 vs 31.5; priority 2: no gain; profiles/r06/big_prio_ab.txt)
#ifndef WFSA_BIG_PRIO
#define WFSA_BIG_PRIO 3
#endif
#ifndef WFSA_UNI_BUBBLES   // (variant builds: the uniform-structure path of small bubbles)
#define WFSA_UNI_BUBBLES 0
#endif
// (tr: timing experiments only, stamps 8..11 of the wave's trace row)
#define WFSA_BSTAMP(k)                                                   \
    if (tr) {                                                            \
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");     \
        if (lane_id() == 0) tr[k] = __builtin_amdgcn_s_memrealtime();    \
    }
// The rmin column's (min, x) forward over a small bubble's edges (weights
// ew, nodes sd, header h), log(min path / Z).  The node vector is indexed
// register-direct: by the wave's shared structure (uni), else by a
// waterfall over the wave's bubble shapes (sorted by shape: few) -- the
// first pending lane's structure, read into scalars, runs for every lane and
// the lanes of that shape keep the result (per-lane node indices put the
// vector in scratch memory).  min(a, b) x w = min(a x w, b x w) exactly, so
// any topological order gives the same bits.
template <int N, int RE>
__device__ __forceinline__ double min_path_log(const double (&ew)[RE], const int (&sd)[RE], int h, bool uni, double Z) {
    double rv = 0.0;
    bool pending = true;
    while (true) {
        const unsigned long long m = __ballot(pending);
        if (m == 0ull) break;
        const int lead = uni ? 0 : __ffsll(m) - 1;
        const int hu = __builtin_amdgcn_readlane(h, lead);
        bool mine = pending && (uni || h == hu);
        int su[RE];
#pragma unroll
        for (int e = 0; e < RE; ++e) {
            su[e] = __builtin_amdgcn_readlane(sd[e], lead);
            mine = mine && (uni || sd[e] == su[e]);
        }
        const int eu = hu >> 16, nu = hu & 0xffff;
        double B[N];
#pragma unroll
        for (int k = 0; k < N; ++k) B[k] = k == 0 ? 1.0 : INFINITY;
#pragma unroll
        for (int e = 0; e < RE; ++e)
            if (e < eu) {
                const double v = B[su[e] & 0xffff] * ew[e];
                B[su[e] >> 16] = ew[e] > 0.0 ? fmin(B[su[e] >> 16], v) : B[su[e] >> 16];
            }
        if (mine) {
            rv = log(B[nu - 1] / Z);
            pending = false;
        }
    }
    return rv;
}

// rl (RMIN, optional): the folded rmin column's record of the bubble
// (RminLane: the bubble's value, its string and the string's bubble count
// and run; FOLD: the (min, x) pass after the backward -- VALU work beside the
// slot stores' latency -- and a multi-bubble string's value stored for its
// last arrival, settled at the wave's end)
template <int N, int RE, bool RMIN = false, bool FOLD = false>
__device__ __forceinline__ double small_bubble(const BubbleArgs& a, const int4* __restrict__ tbl, int n, int b,
                                               int pos, unsigned long long* tr = nullptr, const RminFold* rf = nullptr,
                                               RminLane* rl = nullptr) {
#pragma clang fp contract(off)   // (both forms below: the same bits)
    constexpr int NQ = 1 + RE / 2 + RE / 4;
    int4 q[NQ];
#pragma unroll
    for (int k = 0; k < NQ; ++k) q[k] = tbl[size_t(k) * size_t(n) + size_t(b)];
    const int2 bk = rf ? rf->bk[pos] : make_int2(0, 0);   // (in flight with the quads)
    WFSA_BSTAMP(8)
    const int nodes = q[0].x & 0xffff, edges = q[0].x >> 16;
    const double p = __longlong_as_double((long long)(uint32_t(q[0].z)) | ((long long)(uint32_t(q[0].w)) << 32));
    int code[RE], sd[RE], slot[RE];
#pragma unroll
    for (int k = 0; k < RE / 2; ++k) {
        code[2 * k] = q[1 + k].x;
        sd[2 * k] = q[1 + k].y;
        code[2 * k + 1] = q[1 + k].z;
        sd[2 * k + 1] = q[1 + k].w;
    }
#pragma unroll
    for (int k = 0; k < RE / 4; ++k) {
        slot[4 * k] = q[1 + RE / 2 + k].x;
        slot[4 * k + 1] = q[1 + RE / 2 + k].y;
        slot[4 * k + 2] = q[1 + RE / 2 + k].z;
        slot[4 * k + 3] = q[1 + RE / 2 + k].w;
    }
    double ew[RE];
#pragma unroll
    for (int e = 0; e < RE; ++e) ew[e] = (WFSA_KDBG(a.dbg) & 2) ? 1.0 + 1e-3 * code[e] : a.ewp[code[e]];   // padding edges carry the zero-slot code
    WFSA_BSTAMP(9)
    double A[N], B[N];
#pragma unroll
    for (int k = 0; k < N; ++k) {
        A[k] = k == 0 ? 1.0 : 0.0;
        B[k] = 0.0;
    }
    // Bubbles are sorted by shape, so the lanes of a wave mostly share one
    // structure (header and every edge's nodes): then the node indices are
    // wave-uniform and address the registers directly (s_set_gpr_idx), else
    // every access is a tree of selects (reg_get / reg_add)
    bool same = q[0].x == __builtin_amdgcn_readfirstlane(q[0].x);
#pragma unroll
    for (int e = 0; e < RE; ++e) same = same && sd[e] == __builtin_amdgcn_readfirstlane(sd[e]);
    const bool uni = WFSA_UNI_BUBBLES && __all(same);
    if (uni) {
        const int eu = __builtin_amdgcn_readfirstlane(edges);
#pragma unroll
        for (int e = 0; e < RE; ++e)
            if (e < eu) {
                const int s = __builtin_amdgcn_readfirstlane(sd[e]);
                const double v = A[s & 0xffff] * ew[e];
                A[s >> 16] = A[s >> 16] + v;
            }
    } else {
#pragma unroll
        for (int e = 0; e < RE; ++e)
            if (e < edges) reg_add(A, sd[e] >> 16, reg_get(A, sd[e] & 0xffff) * ew[e]);
    }
    const double Z = uni ? A[__builtin_amdgcn_readfirstlane(nodes) - 1] : reg_get(A, nodes - 1);
    const double scale = -p / Z;

    WFSA_BSTAMP(10)
    auto rmin_pass = [&]() {   // (the min path never exceeds Z)
        const double rv = min_path_log<N, RE>(ew, sd, q[0].x, uni, Z);
        if (a.rmin_sv) {
            if (a.wt) store_wt(&a.rmin_sv[pos], rv);
            else a.rmin_sv[pos] = rv;
        } else {
            global_add(&a.rmin_acc[q[0].y], rv);
        }
    };
    if (RMIN && !FOLD && a.rmin_acc) rmin_pass();
    if (uni) B[__builtin_amdgcn_readfirstlane(nodes) - 1] = 0.0 + 1.0;
    else reg_add(B, nodes - 1, 1.0);
    // lanes of an aligned 2^k group sharing edge e's parameter (slot field
    // level k, layout_slots) sum their contributions by a butterfly -- every
    // lane of the group gets the same bits, in a fixed order -- and the
    // group's first lane stores the one slot; the partners of a grouped lane
    // are active (their edge e exists), the rest ignore what they read
    int kl = 0, kmax = 0;   // (ballots: over the active lanes only -- this runs inside the class branch)
#pragma unroll
    for (int e = 0; e < RE; ++e) kl = max(kl, slot[e] >= 0 ? (slot[e] >> 28) : 0);
#pragma unroll
    for (int t = 1; t <= 6; ++t) kmax = __ballot(kl >= t) ? t : kmax;
    const int lane = lane_id();
    auto contribute = [&](int e, double v) {   // edge e's slot (its group's sum, by the group's first lane)
        const int k = slot[e] >= 0 ? (slot[e] >> 28) : 0;
        v = group_sum(v, k, kmax);
        if (slot[e] >= 0 && (lane & ((1 << k) - 1)) == 0 && !(WFSA_KDBG(a.dbg) & 1)) {
            if (a.wt) store_wt(&a.contrib[slot[e] & 0x0fffffff], v);
            else a.contrib[slot[e] & 0x0fffffff] = v;
        }
    };
    if (uni) {
        const int eu = __builtin_amdgcn_readfirstlane(edges);
#pragma unroll
        for (int e = RE - 1; e >= 0; --e)
            if (e < eu) {
                const int s = __builtin_amdgcn_readfirstlane(sd[e]);
                const double bb = ew[e] * B[s >> 16];
                B[s & 0xffff] = B[s & 0xffff] + bb;
                contribute(e, A[s & 0xffff] * bb * scale);
            }
    } else {
#pragma unroll
        for (int e = RE - 1; e >= 0; --e)
            if (e < edges) {
                const int src = sd[e] & 0xffff;
                const double bb = ew[e] * reg_get(B, sd[e] >> 16);
                reg_add(B, src, bb);
                contribute(e, reg_get(A, src) * bb * scale);
            }
    }
    WFSA_BSTAMP(11)
    const double lz = log(Z);
    if (a.logq) global_add(&a.logq[q[0].y], lz);
    if (FOLD) {
        const double rv = min_path_log<N, RE>(ew, sd, q[0].x, uni, Z);
        rl->rv = rv;
        rl->str = q[0].y;
        rl->k = bk.x;
        rl->run = bk.y;
        if (bk.x > 1) store_wt(&a.rmin_sv[pos], rv);   // (retired by the wave's arrival)
    }
    return p * lz;
}
#undef WFSA_BSTAMP

// Big bubbles, one wavefront each: the lanes stage the edges (code, nodes,
// weight) in LDS in parallel, lane 0 runs the two sweeps over the staged
// edges, and the lanes write the contributions (an edge may have several
// parameters, hence several slots).
// The folded rmin column (RminFold): the candidate of the bubble at position
// pos (value rv, string str) -- a one-bubble string's at once; a k-bubble
// string's value stored write-through, then (the store retired) the
// string's arrival: the k-th sums the k stored values in bubble order.
__device__ __forceinline__ void rmin_settle(const RminFold& rf, double* sv, int pos, double rv, int str,
                                            double& cv, double& ci) {
    const int2 bk = rf.bk[pos];
    double v = INFINITY, idx = -1.0;
    if (bk.x == 1) {
        v = rv;
        idx = double(str);
    } else if (bk.x > 1) {
        store_wt(sv + pos, rv);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned old = __hip_atomic_fetch_add(rf.cnt + bk.y, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == unsigned(bk.x - 1)) {   // the last of the string's bubbles: every value is stored
            rf.cnt[bk.y] = 0u;             // (for the next launch)
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");   // (a compiler barrier)
            double r = 0.0;
            for (int j = 0; j < bk.x; ++j) r += load_wt(sv + rf.mpos[bk.y + j]);
            v = r;
            idx = double(str);
        }
    }
    if (v < cv || (v == cv && idx < ci)) {
        cv = v;
        ci = idx;
    }
}

// The folded column's (min, x) pass over big bubble i at the wave's end (a
// wave-wide call; Z from the sum forward): the edges staged again -- the
// backward overwrote the weights with contributions -- and lane 0's serial
// sweep, as big_bubble's (the same bits); lane 0 settles the candidate
__device__ __forceinline__ void big_bubble_min(const BubbleArgs& a, const RminFold& rf, int i, double Z, int* lsd,
                                               double* lw, double* AB, double& cv, double& ci) {
    const int lane = lane_id();
    const int32_t* rec = a.bub + a.big_off[i];
    const int hdr = rec[0];
    const int nodes = hdr & 0xffff, edges = hdr >> 16;
    for (int e = lane; e < edges; e += kWave) {
        const int code = rec[4 + 2 * e];
        lsd[e] = rec[5 + 2 * e];
        double wgt;
        if (code >= 0) {
            wgt = a.ewp[code];
        } else {
            const int g = -code - 2;
            double s = 0.0;
            for (int q = a.m.pptr[g]; q < a.m.pptr[g + 1]; ++q) s += a.w[a.m.pidx[q]];
            wgt = exp(s);
        }
        lw[e] = wgt;
    }
    wave_sync();
    if (lane == 0) {
        double* B = AB + kMaxBubbleNodes;
        for (int v = 0; v < nodes; ++v) B[v] = v == 0 ? 1.0 : INFINITY;
        for (int e = 0; e < edges; ++e)
            if (lw[e] > 0.0) B[lsd[e] >> 16] = fmin(B[lsd[e] >> 16], B[lsd[e] & 0xffff] * lw[e]);
        const double rv = log(B[nodes - 1] / Z);
        rmin_settle(rf, a.rmin_sv, a.n_small4 + a.n_small + i, rv, rec[1], cv, ci);
    }
    wave_sync();
}

// A multi-bubble string's arrival (its value stored write-through and
// retired): the k-th arrival sums the k values in bubble order
__device__ __forceinline__ void rmin_arrive(const RminFold& rf, const double* sv, const RminLane& l, double& cv,
                                            double& ci) {
    const unsigned old = __hip_atomic_fetch_add(rf.cnt + l.run, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == unsigned(l.k - 1)) {   // the string's last bubble: every value is stored
        rf.cnt[l.run] = 0u;            // (for the next launch)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");   // (a compiler barrier)
        double r = 0.0;
        for (int j = 0; j < l.k; ++j) r += load_wt(sv + rf.mpos[l.run + j]);
        if (r < cv || (r == cv && double(l.str) < ci)) {
            cv = r;
            ci = double(l.str);
        }
    }
}

// rf (the folded rmin column, or null): lane 0 settles the bubble's string
// at once -- rare bubbles: its store retired, its string's arrival, the sum
// by the k-th arrival -- and min-folds the candidate into (cv, ci)
__device__ __forceinline__ double big_bubble(const BubbleArgs& a, int i, int* lsd, double* lw, double* lv, double* AB,
                             const RminFold* rf = nullptr, double* cv = nullptr, double* ci = nullptr,
                             RminLane* pend = nullptr) {
    const int lane = lane_id();
    const int off = a.big_off[i];
    const int32_t* rec = a.bub + off;
    const int hdr = rec[0];
    const int nodes = hdr & 0xffff, edges = hdr >> 16;
    const double p = __longlong_as_double((long long)(uint32_t(rec[2])) | ((long long)(uint32_t(rec[3])) << 32));
    for (int e = lane; e < edges; e += kWave) {
        const int code = rec[4 + 2 * e];
        lsd[e] = rec[5 + 2 * e];
        double wgt;
        if (code >= 0) {
            wgt = a.ewp[code];
        } else {
            const int g = -code - 2;
            double s = 0.0;
            for (int q = a.m.pptr[g]; q < a.m.pptr[g + 1]; ++q) s += a.w[a.m.pidx[q]];
            wgt = exp(s);
        }
        lw[e] = wgt;
    }
    wave_sync();
    double res = 0.0;
    if (lane == 0) {
        double* A = AB;
        double* B = AB + kMaxBubbleNodes;
        for (int v = 0; v < nodes; ++v) {
            A[v] = v == 0 ? 1.0 : 0.0;
            B[v] = 0.0;
        }
        for (int e = 0; e < edges; ++e) A[lsd[e] >> 16] += A[lsd[e] & 0xffff] * lw[e];
        const double Z = A[nodes - 1];
        const double scale = -p / Z;
        // the folded column: this bubble's (min, x) pass at the wave's end,
        // off the path to the QN update (big_bubble_min) -- unless the wave
        // holds another already (a second big bubble: here, as before)
        const bool defer = rf && pend->big < 0;
        if (defer) *pend = RminLane{Z, rec[1], 0, 0, i};
        if (a.rmin_acc && !defer) {   // (min, x) forward in B's storage, then B is re-zeroed
            for (int v = 0; v < nodes; ++v) B[v] = v == 0 ? 1.0 : INFINITY;
            for (int e = 0; e < edges; ++e)
                if (lw[e] > 0.0) B[lsd[e] >> 16] = fmin(B[lsd[e] >> 16], B[lsd[e] & 0xffff] * lw[e]);
            const double rv = log(B[nodes - 1] / Z);
            const int pos = a.n_small4 + a.n_small + i;
            if (a.rmin_sv) {
                if (a.wt) store_wt(&a.rmin_sv[pos], rv);
                else a.rmin_sv[pos] = rv;
            } else {
                global_add(&a.rmin_acc[rec[1]], rv);
            }
            if (rf) rmin_settle(*rf, a.rmin_sv, pos, rv, rec[1], *cv, *ci);
            for (int v = 0; v < nodes; ++v) B[v] = 0.0;
        }
        B[nodes - 1] = 1.0;
        for (int e = edges - 1; e >= 0; --e) {
            const int src = lsd[e] & 0xffff;
            const double bb = lw[e] * B[lsd[e] >> 16];
            B[src] += bb;
            lv[e] = A[src] * bb * scale;
        }
        const double lz = log(Z);
        if (a.logq) global_add(&a.logq[rec[1]], lz);
        res = p * lz;
    }
    wave_sync();
    const int base = a.big_edge_base[i];
    for (int e = lane; e < edges; e += kWave)
        for (int q = a.big_eslot_ptr[base + e]; q < a.big_eslot_ptr[base + e + 1]; ++q) {
            if (a.wt) store_wt(&a.contrib[a.big_eslot[q]], lv[e]);
            else a.contrib[a.big_eslot[q]] = lv[e];
        }
    return res;
}

template <bool RMIN>
__global__ __launch_bounds__(kBubbleBlock) void bubble_kernel(BubbleArgs a) {
    if (a.halted && *a.halted) return;
    constexpr int WPB = kBubbleBlock / kWave;
    __shared__ int lsd[WPB][kBigEdgeLds];
    __shared__ double lw[WPB][kBigEdgeLds], lv[WPB][kBigEdgeLds], lab[WPB][2 * kMaxBubbleNodes];
    const int lane = lane_id();
    const int wib = int(threadIdx.x) / kWave;
    const int gw = int(blockIdx.x) * WPB + wib;
    double ll_acc = 0.0;
    if (gw < a.n_big) {
        ll_acc = big_bubble(a, gw, lsd[wib], lw[wib], lv[wib], lab[wib]);
    } else {
        // class A (4 nodes / 4 edges: most bubbles) first, then class B
        const int b = int(small_entry(gw - a.n_big, lane, a.n_small4, a.n_small));
        if (b >= 0 && b < a.n_small4) ll_acc = small_bubble<4, 4, RMIN>(a, a.sm4_tbl, a.n_small4, b, b);
        else if (b >= a.n_small4)
            ll_acc = small_bubble<8, 8, RMIN>(a, a.sm_tbl, a.n_small, b - a.n_small4, b);
    }
    ll_acc = wave_sum(ll_acc);
    if (lane == 0) a.ll_part[gw] = ll_acc;
}

// Per-iteration stream kernel: log q of every compiled string's trivial
// words, sum_words w[j], one lane per string, no atomics (their gradient is
// the constant added by the tail kernel).  w[n_params] is a zero slot, so a
// padding word (0xFFFF / -1), a header word and -- in the fast path -- a
// multi-parameter word read 0.0 without a branch: index = min(word,
// n_params).  Chunks that hold multi-parameter words (MULTI, automata with
// epsilon composites) take a second, per-word pass.
//
// Each wave owns a contiguous run of groups (wave_first, balanced at
// preparation on chunk rows and bubble work) and streams it as one run of
// 1 KiB rows: two register sets of D rows, one applied while the other's
// loads are in flight, across group boundaries (a group starts with its
// header row: p of each lane's string and the group's row count), so the
// prefetch never drains between strings.  Load rows are clamped to the run
// (a clamped load re-reads the last row from cache, no over-read of HBM).
// The first set is issued before the weights are staged and the bubbles
// evaluated, so its latency hides behind that work (both sets would spill).
// DBG (timing experiments only, WFSA_FBS_DBG): 1 no table gathers, 3 no
// stream pass at all, 4 neither stream pass nor table staging, 5 the QN finish only, 6 / 7
// prefetch sets of 2 / 6 rows, 8 no bubble code, 9 stream loads only; the
// delta kernel also: 11 no table staging, 12 no QN finish, 13 neither bubbles
// nor finish (the stream pass and the staging alone)
// One delta-format row (fb_kernels.hpp) of a lane: three 10-bit fields per
// dword; each steps the lane's LDS address in the staged table forward and
// gathers that entry -- three VALU per field (extract, shift-add, f64 add).
// HDR: the group's first row, whose fields 0-7 hold p and the row count.  A
// valid stream never leaves the table (its last step lands on the final zero
// slot); a corrupt one reads zeros past the allocation, never faults.
typedef __attribute__((address_space(3))) const double lds_double;
// the LDS address of the staged table (32-bit; the lane's cursor is kept as
// one, so a gather needs no base add)
__device__ __forceinline__ uint32_t lds_addr(const double* p) {
    return uint32_t(reinterpret_cast<uintptr_t>((lds_double*)p));   // (an address-space cast)
}
// field k (0..2) of a dword: one v_bfe_u32 (written out: the compiler turns
// a bfe followed by the << 3 into a shift and a mask, an instruction more)
__device__ __forceinline__ uint32_t delta_field(uint32_t d, int k) {   // (k a constant after unrolling)
    uint32_t f;
    if (k == 0) asm("v_bfe_u32 %0, %1, 0, 10" : "=v"(f) : "v"(d));
    else if (k == 1) asm("v_bfe_u32 %0, %1, 10, 10" : "=v"(f) : "v"(d));
    else asm("v_bfe_u32 %0, %1, 20, 10" : "=v"(f) : "v"(d));
    return f;
}
template <bool HDR>
__device__ __forceinline__ void delta_row(const uint4 v, uint32_t& cur, double& a0, double& a1) {
    const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = HDR ? kDeltaFields - kDeltaHdrFields : 0; i < kDeltaFields; ++i) {
        const uint32_t f = delta_field(d[i / 3], i % 3);
        // (written out too: the compiler reassociates cur + (f << 3) into
        // prefix sums of the fields plus a shift-add each, a third VALU)
        asm("v_lshl_add_u32 %0, %1, 3, %2" : "=v"(cur) : "v"(f), "v"(cur));
        const double t = *(lds_double*)uintptr_t(cur);
        if (i & 1) a1 += t;
        else a0 += t;
    }
}

// The QuasiNewton update of one batch of constraints (QnWave) by one
// wavefront, a lane per member: the arithmetic and the summation orders of
// qn_step_kernel<true> (qn_kernel.hip: ComputeExpX, ComputeG,
// ComputeLambdaNext, the x update, LambdaUpdate -- src/QuasiNewtonLearner.cpp:
// 53-56,127-201, src/Learner.cpp:438-462), so the trajectory is the same bit
// for bit.  The per-constraint sums run in member order on the constraint's
// first lane, which reads its members' values by shuffles.  ok == false (the
// arrival poll gave up): NaN partials, no update.
// a batch's member data: loaded before the QN wave's poll (none of it is
// written in this launch)
struct QnBatchIn {
    int c0, nc, m0, m1, nchunk;
    int64_t cbase;
    int con, fo, nch, fc, cpl;
    double x, ft, laml, gout;
};
__device__ __forceinline__ QnBatchIn qn_wave_load(const QnWave& q, int b) {
    const int lane = lane_id();
    const int4 bd = q.batch[2 * b], bc = q.batch[2 * b + 1];
    QnBatchIn in;
    in.c0 = bd.x;
    in.nc = bd.y - bd.x;
    in.m0 = bd.z;
    in.m1 = bd.w;
    in.nchunk = bc.x;
    in.cbase = int64_t(uint32_t(bc.y)) | (int64_t(bc.z) << 32);
    const int m = in.m0 + lane;
    in.con = in.c0;
    in.fo = in.nch = in.fc = in.cpl = 0;
    in.x = in.ft = in.laml = in.gout = 0.0;
    if (m < in.m1) {
        in.con = q.con_of[m];
        in.fo = q.full_of[m];
        if (q.out) in.gout = q.out[1 + in.fo];   // (the traversal strings' part)
        in.x = q.x[m];
        in.ft = q.fixed_t[m];
        in.fc = q.mfirst[m];
        in.nch = q.mnch[m];
    }
    if (lane < in.nc) {
        in.cpl = q.cptr[in.c0 + lane];
        in.laml = q.lambda[in.c0 + lane];
    }
    return in;
}

typedef __attribute__((address_space(3))) void lds_void;   // (LDS-DMA operands)
typedef __attribute__((address_space(1))) void glb_void;
template <bool PX>
__device__ __forceinline__ void qn_wave_batch(const QnWave& q, const QnBatchIn& in, bool ok_in, const unsigned& halt,
                                              int bi, unsigned long long* tr = nullptr) {   // (tr: timing experiments, stamps 8-11)
#pragma clang fp contract(off)
    const int lane = lane_id();
    const int c0 = in.c0, nc = in.nc, m0 = in.m0, m1 = in.m1, nchunk = in.nchunk;
    const int64_t cbase = in.cbase;
    const int m = m0 + lane;
    const bool valid = m < m1;
    const int con = in.con, fo = in.fo, nch = in.nch, fc = in.fc, cpl = in.cpl;
    const double x = in.x, ft = in.ft, laml = in.laml;
    const int j = con - c0;                        // the member's constraint within the batch
    const int first = __shfl(cpl, j, kWave);       // its first member
    const int nxt = __shfl(cpl, min(j + 1, kWave - 1), kWave);
    const int end = j + 1 < nc ? nxt : m1;
    const double lam = __shfl(laml, j, kWave);
    const int nm = end - first, ld = first - m0;   // members, and the first member's lane
    const bool leader = valid && m == first;
    int maxnm = valid ? nm : 0, maxnch = valid ? nch : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        maxnm = max(maxnm, __shfl_xor(maxnm, o, kWave));
        maxnch = max(maxnch, __shfl_xor(maxnch, o, kWave));
    }
    // the batch's bubble contribution chunks (stored write-through by this
    // launch's bubble waves: sc1 loads), one per lane per round, each summed
    // by chunk_tree; then every member adds its chunks' sums in chunk order
    // Eight lanes read a chunk (lane piece = two consecutive slots, so a load
    // instruction covers eight whole chunks, 1 KiB, instead of 64 lanes each
    // on its own chunk's line) and reduce it by xor shuffles in chunk_tree's
    // order; chunk 64 r + l's sum then moves to lane l of round r
    double cs[kQnWaveChunkRounds];
#pragma unroll
    for (int r = 0; r < kQnWaveChunkRounds; ++r) cs[r] = 0.0;
    const int sub = lane & 7;
#pragma nounroll
    for (int r = 0; r < kQnWaveChunkRounds; ++r) {   // (a round at a time: 16 loads in flight, no spills)
        if (r * kWave >= nchunk) break;   // (uniform)
        double s8[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int c = r * kWave + 8 * k + (lane >> 3);
            const double* p = q.contrib + cbase + int64_t(kSlotChunk) * c + 2 * sub;
            s8[k] = c < nchunk ? load_wt(p) : 0.0;
            const double hi = c < nchunk ? load_wt(p + 1) : 0.0;
            s8[k] += hi;   // p_sub = x[2 sub] + x[2 sub + 1]
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
#pragma unroll
            for (int o = 1; o < 8; o <<= 1) s8[k] += __shfl_xor(s8[k], o, kWave);
        }
        double v = 0.0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const double t = __shfl(s8[k], sub * 8, kWave);
            if (k == (lane >> 3)) v = t;
        }
#pragma unroll
        for (int i = 0; i < kQnWaveChunkRounds; ++i)   // (static indices: the array stays in registers)
            if (i == r) cs[i] = v;
    }
    if (tr && lane_id() == 0) tr[8] = __builtin_amdgcn_s_memrealtime();
    double sm = 0.0;   // the member's chunk sums in chunk order, four chunks' shuffles per round
    for (int t0 = 0; t0 < maxnch; t0 += 4) {
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int qc = fc + t0 + u, src = qc & (kWave - 1), rr = qc >> 6;
            v[u] = 0.0;
#pragma unroll
            for (int r = 0; r < kQnWaveChunkRounds; ++r) {
                if (r * kWave >= nchunk) break;   // (uniform)
                const double s = __shfl(cs[r], src, kWave);
                if (rr == r) v[u] = s;
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (t0 + u < nch) sm += v[u];
    }
    bool ok = ok_in;
    double sg;
    if (PX && q.px.on) {
        // across ranks: the members' partials (their traversal part and slot
        // sums) summed over the ranks through the peer areas, in rank order,
        // then the trivial words' constant (all-reduced at preparation); a
        // halted step skips the exchange on every rank alike
        double g = 0.0;
        if (ok && halt == 0u) {
            ok = peer_post_wait(q.px, size_t(m0), m1 - m0, valid ? in.gout + sm : 0.0, kPeerQnFlag0 + bi);
            if (ok && valid)
                for (int r = 0; r < q.px.nranks; ++r) g += peer_slot(q.px, r, size_t(m));
            if (!ok && lane == 0) store_wt(q.halted + 2, 1u);   // (the finish reports it; the host the member's failure)
        }
        sg = g + ft;
    } else {
        double gi = in.gout;   // qn_step_kernel's order: the traversal part, + the trivial words', + the slots'
        gi += ft;
        sg = gi + sm;
    }
    const double e = exp(x);
    // the per-constraint sums, in member order on the leader lane: eight
    // members' values fetched per round (the shuffles independent, in flight
    // together), then added in order -- the same sums, without a shuffle's
    // latency per member
    double gg = -1.0;   // ComputeG: -1 + sum exp(x) in member order
    for (int t0 = 0; t0 < maxnm; t0 += 8) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = __shfl(e, min(lane + t0 + u, kWave - 1), kWave);
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (leader && t0 + u < nm) gg += v[u];
    }
    double r = lam * gg;   // ComputeLambdaNext
    for (int t0 = 0; t0 < maxnm; t0 += 8) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = __shfl(sg, min(lane + t0 + u, kWave - 1), kWave);
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (leader && t0 + u < nm) r -= v[u];
    }
    const double laux_l = r / (gg + 1.0);
    const double g = __shfl(gg, ld, kWave), laux = __shfl(laux_l, ld, kWave);
    if (tr && lane == 0) tr[9] = __builtin_amdgcn_s_memrealtime();
    // the previous step's halt decision (loaded beside the chunks): a halted
    // run skips this step -- no update at all (qn_wave_run publishes it)
    if (halt != 0u) return;
    double gerr = 0.0;
    if (valid && ok) {
        const double aux = e * lam;
        gerr = fabs(sg + aux);
        const double xn = x - q.eta * ((sg + e * laux) / aux);
        q.x[m] = xn;
        q.grad[m] = sg;
        q.w_next[fo] = xn;   // GetWeight for the next step
        q.ewp_next[fo] = exp(xn);
    }
    if (tr && lane == 0) tr[10] = __builtin_amdgcn_s_memrealtime();
    double ge = 0.0;
    for (int t0 = 0; t0 < maxnm; t0 += 8) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = __shfl(gerr, min(lane + t0 + u, kWave - 1), kWave);
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (leader && t0 + u < nm) ge = fmax(ge, v[u]);
    }
    if (leader) {
        double4 pv;
        if (ok) {
            const double d = lam - laux_l;   // LambdaUpdate (src/Learner.cpp:438-462)
            q.lambda[con] = q.exp_lambda ? lam * exp(-q.eta * (d / lam)) : lam - q.eta * d;
            pv.x = g;
            pv.y = g;
            pv.z = lam;
            pv.w = ge;
        } else {
            pv.x = pv.y = pv.z = pv.w = NAN;
        }
        if (q.self_finish) {   // read by this launch's finisher
            double* pp = q.partial + 4 * size_t(con);
            store_wt(pp, pv.x);
            store_wt(pp + 1, pv.y);
            store_wt(pp + 2, pv.z);
            store_wt(pp + 3, pv.w);
        } else {
            reinterpret_cast<double4*>(q.partial)[con] = pv;
        }
    }
}

// QN wave r of the launch: wait for every block's arrival (its bubble slots
// and the finish wave's halt decision), then its batches r, r + n_waves, ...
constexpr unsigned kQnPollLimit = 1u << 22;   // polls of ~0.5 us under load (s_sleep 1 + an sc1 load): ~1 s, then give up
template <bool PX>
__device__ __forceinline__ void qn_wave_run(const QnWave& q, int r, unsigned long long* tr) {
    const int lane = lane_id();
    QnBatchIn first{};
    if (r < q.n_batches) first = qn_wave_load(q, r);   // (in flight during the poll)
    int ok = 1;
    if (lane == 0) {
        unsigned it = 0;
        const unsigned limit = q.poll_limit ? q.poll_limit : kQnPollLimit;
#ifdef WFSA_EXPERIMENTS
        if (tr) tr[11] = __builtin_amdgcn_s_memrealtime();
#endif
        // Wave 0 alone polls the arrival counter and then releases the other
        // waves' go lines (this launch's tag; no reset needed).  Every QN
        // wave polling the counter's line -- which the blocks' atomics
        // update -- slowed the whole launch once the waves polled from their
        // stream's end (c3 46 vs 27.5 us, 500k strings 37 vs 23.7;
        // profiles/r06/poll_modes.txt)
        const bool lead = r == 0;
        const unsigned* line = lead ? q.arrive + q.parity : q.go + size_t(r) * kQnGoStride;
        const unsigned want = lead ? unsigned(q.n_arrive) + (q.poll_fault ? 1u : 0u) : q.fin.tag;   // (fault injection)
        while (lead ? load_wt(line) < want : load_wt(line) != want) {
#ifdef WFSA_EXPERIMENTS
            if (tr && it == 0) tr[13] = __builtin_amdgcn_s_memrealtime();
#endif
            __builtin_amdgcn_s_sleep(1);
            if (++it > limit) {
                ok = 0;
                break;
            }
        }
#ifdef WFSA_EXPERIMENTS
        if (tr) tr[12] = it;
#endif
        // a wave that gave up leaves its constraints un-updated: the timeout
        // word makes this step's finish report kQnTimedOut (its NaN partials
        // alone would be dropped by the finish's fmin / fmax), and the host
        // then fails the run instead of stepping on inconsistent weights
        if (!ok) store_wt(q.halted + 2, 1u);
    }
    if (r == 0)   // (after a timeout too: the step then fails by the timeout word, not by every wave's wait)
        for (int v = 1 + lane; v < q.n_waves; v += kWave) store_wt(q.go + size_t(v) * kQnGoStride, q.fin.tag);
    // (a compiler barrier: no load below moves above the poll; on the
    // hardware a workgroup-scope acquire is only a vmcnt wait -- see the
    // ordering note at the arrival in fbs_kernel)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    ok = __shfl(ok, 0, kWave);
    if (tr && lane == 0) tr[5] = __builtin_amdgcn_s_memrealtime();   // (timing experiments)
    // the halt decision of this launch's finish wave: issued now, waited for
    // only before the first store (beside the batch's chunk loads)
    const unsigned halt = ok ? load_wt(q.halted + 1) : 0u;
    if (r < q.n_batches) qn_wave_batch<PX>(q, first, ok != 0, halt, r, tr);
    for (int b = r + q.n_waves; b < q.n_batches && halt == 0u; b += q.n_waves)
        qn_wave_batch<PX>(q, qn_wave_load(q, b), ok != 0, halt, b);
    if (halt != 0u && r == 0 && lane == 0) {   // the previous step halted: this one is skipped
        q.halted[0] = 1u;   // for the later launches
        qn_publish_row(q.fin, nullptr, kQnSkipped);
    }
    if (tr && lane == 0) tr[6] = __builtin_amdgcn_s_memrealtime();
}

// A field of the stream kernel's argument block read where it is used,
// through a pointer into the kernel-argument segment the compiler cannot see
// through: kernel arguments are otherwise loaded at the entry and kept in
// scalar registers to the end, and the QN waves' and the finishes' ~60
// dwords of them spilled the kernel's scalar registers into vector lanes
// (616 lane reads in the in-kernel QN variant; 131 with these three late)
template <typename T>
__device__ __forceinline__ T late_arg(size_t off) {
    static_assert(sizeof(T) % 4 == 0, "argument blocks are dword multiples");
    typedef __attribute__((address_space(4))) const char kchar;
    typedef __attribute__((address_space(4))) const uint32_t kword;
    kchar* kp = (kchar*)(__builtin_amdgcn_kernarg_segment_ptr());
    asm volatile("" : "+s"(kp));
    kword* src = reinterpret_cast<kword*>(kp + off);
    T v;
    uint32_t* dst = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
    for (size_t i = 0; i < sizeof(T) / 4; ++i) dst[i] = src[i];
    return v;
}
#define WFSA_LATE_ARG(field) late_arg<decltype(CompiledArgs::field)>(offsetof(CompiledArgs, field))

// PX: the QN update across ranks (QnWave::px, the finishes' exchanges): its own variants
template <bool WIDE, bool W_LDS, bool MULTI, int DBG = 0, bool RMIN = false, bool DELTA = false, bool QN = false,
          bool PX = false>
#ifdef WFSA_FBS_VGPR64   // (variant builds: a 64-VGPR budget, two 1024-thread blocks per CU)
#define WFSA_FBS_ATTR __attribute__((amdgpu_num_vgpr(64)))
#else
#define WFSA_FBS_ATTR
#endif
__global__ __launch_bounds__(1024, (DBG == 10 ? 8 : 1)) WFSA_FBS_ATTR void fbs_kernel(CompiledArgs a) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int lane = lane_id();
    const int wpb = int(blockDim.x) / kWave;
    const int nblk = int(gridDim.x);
    const int nw = nblk * wpb;
    const int bid = int(blockIdx.x);
    const int w = int(threadIdx.x) / kWave;
    const int gw = __builtin_amdgcn_readfirstlane(bid * wpb + w);
#ifdef WFSA_EXPERIMENTS
    unsigned long long* tr = a.trace ? a.trace + size_t(gw) * 16 : nullptr;   // (timing experiments)
#define WFSA_STAMP(k) \
    if (tr && lane == 0) tr[k] = __builtin_amdgcn_s_memrealtime();
#else
#define WFSA_STAMP(k)
#endif
    WFSA_STAMP(0)
    // The delta table's first round of loads before anything else is waited
    // for (the halted flag, the wave's stream setup, the first row set): at
    // entry these scalar load chains took ~2 us ahead of the table's loads
    constexpr int kTB = 12;   // 16-byte pieces per thread and round (one round for 12k-entry tables at 512 threads)
    const bool pre = DELTA && !a.no_streams && DBG != 4 && DBG != 11;
    const int tlast = a.n_params - 1;
    // A piece is slots (s2, s2 + 1): weights j0 = s2 - 1 - s2 / kDeltaPeriod
    // and j0 + 1 whenever neither slot is a zero slot, and on a period
    // boundary one of the two is zero and the other is still w[j0] or
    // w[j0 + 1] -- so one 16-byte load of (w[j0], w[j0 + 1]) serves every
    // piece (8-byte aligned; w holds n_params + 2 doubles, so j0 + 1 <=
    // tlast + 1 stays inside), the zeros by selects: half the load
    // instructions of two 8-byte gathers (the staging 5.4 -> ~3.4 us in
    // tools/micro/stage_table.hip, profiles/r05)
    auto table_round = [&](int q0, int nthr, double2 (&t)[kTB]) {
#pragma unroll
        for (int b = 0; b < kTB; ++b) {
            const int s2 = 2 * (q0 + b * nthr);
            const int j0 = s2 - 1 - s2 / kDeltaPeriod;
            const int jc = min(max(j0, 0), tlast);
            const double2 v = *reinterpret_cast<const double2*>(a.w + jc);
            const bool z0 = (s2 % kDeltaPeriod) == 0 || j0 > tlast;
            const bool z1 = ((s2 + 1) % kDeltaPeriod) == 0 || j0 + 1 > tlast;
            t[b].x = z0 ? 0.0 : v.x;
            t[b].y = z1 ? 0.0 : (j0 < 0 ? v.x : v.y);
        }
    };
    double2 t0[kTB];
    if (pre) table_round(int(threadIdx.x), int(blockDim.x), t0);
    if (QN && bid == 0 && threadIdx.x == 0) {   // for the next launch
        a.qw.arrive[a.qw.parity ^ 1] = 0u;
        if (a.qw.done) a.qw.done[a.qw.parity ^ 1] = 0u;   // (also when only a Run's last launch finishes itself)
    }
    // halted is written only by an earlier launch (the QN step's finish)
    if (a.halted && *a.halted) {
        if (QN && bid == 0 && threadIdx.x == 0) qn_publish_row(a.qw.fin, nullptr, kQnSkipped);   // (no QN kernel)
        return;
    }
    __shared__ unsigned q_arrived;   // QN: this block's waves whose bubble slots have retired
    __shared__ unsigned blk_in;      // this block's waves whose partials are in LDS (wsum, wrv, wri)
    if (threadIdx.x == 0) {   // (ordered by the staging barrier)
        blk_in = 0u;
        if (QN) q_arrived = 0u;
    }
    const uint32_t zslot = uint32_t(a.n_params);
    // this wave's run of chunk rows
    const int g0 = a.wave_first[gw], g1 = a.wave_first[gw + 1];
    const int64_t cb = a.g_base[g0];
    const int rows = int((a.g_base[g1] - cb) / kWave);
    const int last = max(rows - 1, 0);   // no groups: row 0 of the slack after the last group
    const uint4* st = a.stream + cb + lane;
    constexpr int D = DELTA ? kDeltaPrefetch : (DBG == 6 ? 2 : (DBG == 7 ? 6 : kStreamPrefetch));
    uint4 A[D], B[D];
    auto load = [&](uint4 (&r)[D], int c0) {
#pragma unroll
        for (int d = 0; d < D; ++d) r[d] = st[int64_t(kWave) * min(c0 + d, last)];
    };
    const bool kStreams = DBG != 3 && DBG != 4 && !a.no_streams;   // (timing experiments; bubbles-only launches)
    // the first row set in flight from the start (its latency hides behind
    // the staging and the bubbles)
    if (kStreams) load(A, 0);
    if (pre) {   // the table: the first round's pieces (loaded at entry), then any further rounds
        const int T2 = (a.d_tab + 1) / 2, nthr = int(blockDim.x);
        double2* dst = reinterpret_cast<double2*>(lds);
#pragma unroll
        for (int b = 0; b < kTB; ++b) {
            const int q = int(threadIdx.x) + b * nthr;
            if (q < T2) dst[q] = t0[b];
        }
        for (int q0 = int(threadIdx.x) + kTB * nthr; q0 < T2; q0 += kTB * nthr) {
            double2 t[kTB];
            table_round(q0, nthr, t);
#pragma unroll
            for (int b = 0; b < kTB; ++b) {
                const int q = q0 + b * nthr;
                if (q < T2) dst[q] = t[b];
            }
        }
        __syncthreads();
    }
    // the previous QN step's finish runs in a wave of its own -- the last
    // wave of block 0, which the host gives no groups and no bubbles -- after
    // the staging barrier, beside the other waves' work
    const bool fin_wave = bid == 0 && w == wpb - 1;
    auto finish = [&]() {
        if (fin_wave && a.fin.active && DBG != 12 && DBG != 13) {
            double finfo[7];
            unsigned fstat = kQnRan;
            const QnFinish fin = WFSA_LATE_ARG(fin);
            qn_finish_compute<true, false, PX>(fin, nullptr, finfo, fstat);
            if (lane == 0) qn_finish_publish(fin, finfo, fstat);
        }
    };
    if (DBG == 5) {   // the launch and the finish only
        finish();
        return;
    }
    double ll_acc = 0.0;
    bool stored = fin_wave;   // (QN: this wave's stores must retire before it arrives)
    // the folded rmin column (RMIN && QN, RminFold): the lane's small bubble
    // (position, value, string) until its wave arrived, and the lane's candidate
    constexpr bool RF = RMIN && QN;
    RminLane rm_lane{0.0, -1, 0, 0, -1};   // the lane's small bubble
    RminLane rm_big{0.0, -1, 0, 0, -1};    // lane 0: a big bubble whose (min, x) pass is due at the wave's end
    int rm_pos = -1;
    double rm_cv = INFINITY, rm_ci = -1.0;
    const bool small_wave = a.bub_on && DBG != 8 && DBG != 10 && DBG != 13 && !fin_wave && w < a.bub.small_wpb;
    auto small_bubbles = [&]() {   // one per lane, from the first small_wpb waves of every block (spread over all CUs)
        stored = true;
        // chunk w * nblk + bid: consecutive chunks (one class, one cost) on
        // different blocks, so the costly class-B chunks spread over the CUs
        const int b = int(small_entry(int64_t(w) * nblk + bid, lane, a.bub.n_small4, a.bub.n_small));
#ifdef WFSA_EXPERIMENTS
        unsigned long long* btr = tr;
#else
        unsigned long long* btr = nullptr;
#endif
        // (the bubbles are on the QN update's critical path; the stream waves
        // beside them mostly wait for memory: the bubble waves issue first)
        __builtin_amdgcn_s_setprio(2);
        const BubbleArgs bub = WFSA_LATE_ARG(bub);
        const RminFold rf = WFSA_LATE_ARG(rf);
        const RminFold* rfp = RF ? &rf : nullptr;
        RminLane* rlp = RF ? &rm_lane : nullptr;
        if (b >= 0 && b < bub.n_small4)
            ll_acc += small_bubble<4, 4, RMIN, RF>(bub, bub.sm4_tbl, bub.n_small4, b, b, btr, rfp, rlp);
        else if (b >= bub.n_small4)
            ll_acc += small_bubble<8, 8, RMIN, RF>(bub, bub.sm_tbl, bub.n_small, b - bub.n_small4, b, btr, rfp, rlp);
        if (RF && b >= 0) {
            rm_pos = int(b);
            if (rm_lane.k == 1) min_pair(rm_cv, rm_ci, rm_lane.rv, double(rm_lane.str));
        }
        __builtin_amdgcn_s_setprio(0);
    };
    // big bubbles, one wavefront each, from the last blocks' last waves down
    // (the finish wave's rank, nblk - 1, skipped), staged in LDS after the table
    auto big_bubbles = [&]() {
        const int r = big_rank(bid, w, nblk, wpb, a.bub.qw_waves);
        if (r < a.bub.n_big) {
            stored = true;
            const int E = a.bub.big_lds_edges;
            char* stg = reinterpret_cast<char*>(lds) + a.bub.big_lds_off + w * big_stage_bytes(E);
            double* lw = reinterpret_cast<double*>(stg);
            int* lsd = reinterpret_cast<int*>(lw + E + 2 * kMaxBubbleNodes);
            const BubbleArgs bub = WFSA_LATE_ARG(bub);
            const RminFold rf = WFSA_LATE_ARG(rf);
            if (WFSA_BIG_PRIO) __builtin_amdgcn_s_setprio(WFSA_BIG_PRIO);
            for (int i = r; i < bub.n_big; i += nw - 1)
                ll_acc += big_bubble(bub, i, lsd, lw, lw, lw + E, RF ? &rf : nullptr, &rm_cv, &rm_ci, &rm_big);
            if (WFSA_BIG_PRIO) __builtin_amdgcn_s_setprio(0);
        }
    };
    if (!DELTA && W_LDS && DBG != 4 && !a.no_streams) {
        // stage w[0, n_params] in 16-byte pieces, all of a thread's loads
        // issued before its first store (loads and stores unconditional --
        // an index past the end is clamped to the last piece, which is then
        // written twice with the same value -- so nothing is branched around)
        const int n2 = (a.n_params + 2) / 2;
        const double2* src = reinterpret_cast<const double2*>(a.w);
        double2* dst = reinterpret_cast<double2*>(lds);
        constexpr int kB = 12;   // one round for tables up to 12k params at 512 threads
        for (int j0 = int(threadIdx.x); j0 < n2; j0 += kB * int(blockDim.x)) {
            double2 t[kB];
#pragma unroll
            for (int b = 0; b < kB; ++b) t[b] = src[min(j0 + b * int(blockDim.x), n2 - 1)];
#pragma unroll
            for (int b = 0; b < kB; ++b) dst[min(j0 + b * int(blockDim.x), n2 - 1)] = t[b];
        }
        __syncthreads();
    }
    WFSA_STAMP(1)
    finish();
    const double* wsrc = W_LDS ? lds : a.w;
    if (a.bub_on && DBG != 8 && DBG != 10 && DBG != 13 && !fin_wave) {   // this wave's bubbles, before its streams
        if (small_wave) small_bubbles();   // (small_wpb <= waves per block: bubbles_fused)
        big_bubbles();
    }
    WFSA_STAMP(2)
    // Ordering of the in-launch hand-off (slot stores -> arrival -> the QN
    // waves' reads).  The arrival is a RELAXED agent-scope atomic and the
    // poll a relaxed sc1 load, so the HIP memory model alone gives no
    // happens-before; an agent-scope release / acquire would, but on gfx950
    // it is an L2 write-back / invalidate per wave (round 2's grid barrier:
    // 38 -> 88 us).  The hardware argument instead: (1) every slot store is
    // write-through (store_wt: sc1, to memory past the XCD's L2); (2) the
    // storing wave waits vmcnt(0) -- its stores acknowledged by memory --
    // before its LDS arrival, and the block's last wave adds to the global
    // counter only after every wave of the block arrived (LDS atomics order
    // within the block); (3) the consumer's loads are sc1 (they bypass the
    // stale L2) and are issued after its poll matched (a compiler barrier
    // there; vector loads are not speculated).  So a consumer that saw the
    // count reads the stored values.  The same argument covers the done
    // counter and the self-finish's partials.
    if (QN) {   // this wave's slot stores (and the finish wave's halt decision) retired: arrive
        if (stored) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        unsigned prev = 0u;
        if (lane == 0) prev = atomicAdd(&q_arrived, 1u);
        prev = __shfl(prev, 0, kWave);
        if (lane == 0 && prev == unsigned(wpb - 1)) {   // the block's last wave: one arrival for all its stores
            const unsigned o =
                __hip_atomic_fetch_add(a.qw.arrive + a.qw.parity, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#ifdef WFSA_EXPERIMENTS
            if (a.trace) {   // (the atomic's return: when it landed, in which order)
                a.trace[size_t(blockIdx.x) * wpb * 16 + 14] = __builtin_amdgcn_s_memrealtime();
                a.trace[size_t(blockIdx.x) * wpb * 16 + 15] = o;
            }
#else
            (void)o;
#endif
        }
        WFSA_STAMP(3)
    }
    if (kStreams) load(B, D);
    double p = 0.0, acc0 = 0.0, acc1 = 0.0;
    int hdr = 0, grp = g0 - 1;   // the next header row, the current group
    auto flush = [&]() {   // the lane's string of the current group is complete
        const double acc = acc0 + acc1;
        ll_acc += p * acc;
        if (a.logq && grp >= g0) {
            const int s = a.l_str[grp * kWave + lane];
            if (s >= 0) a.logq[s] = acc;
        }
    };
    // DELTA: the lane's LDS address in the remapped table (its slot 0 at a group start)
    const uint32_t tab0 = lds_addr(lds);
    uint32_t cur = tab0;
    auto apply = [&](const uint4 (&r)[D], int c0) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int c = c0 + d;
            if (c >= rows) break;
            uint4 v = r[d];
            if constexpr (DELTA) {
                if (DBG == 9 || DBG == 1) {   // (timing variants: loads only / no table gathers)
                    if (c == hdr) {
                        flush();
                        acc0 = 0.0;
                        acc1 = 0.0;
                        hdr += __builtin_amdgcn_readfirstlane(int(v.z & 0xffffu));
                        ++grp;
                    }
                    if (DBG == 9) {
                        acc0 += double(v.x ^ v.y ^ v.z ^ v.w);
                    } else {
                        const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                        for (int i = 0; i < kDeltaFields; ++i) {
                            const uint32_t f = delta_field(d[i / 3], i % 3);
                            asm("v_lshl_add_u32 %0, %1, 3, %2" : "=v"(cur) : "v"(f), "v"(cur));
                            if (i & 1) acc1 += double(cur);
                            else acc0 += double(cur);
                        }
                    }
                    continue;
                }
                if (c == hdr) {   // uniform: the first row of the next group
                    flush();
                    acc0 = 0.0;
                    acc1 = 0.0;
                    p = __longlong_as_double((long long)(v.x) | ((long long)(v.y) << 32));
                    hdr += __builtin_amdgcn_readfirstlane(int(v.z & 0xffffu));
                    ++grp;
                    cur = tab0;
                    delta_row<true>(v, cur, acc0, acc1);
                } else {
                    delta_row<false>(v, cur, acc0, acc1);
                }
                continue;
            }
            if (c == hdr) {   // uniform: the first row of the next group
                flush();
                acc0 = 0.0;
                acc1 = 0.0;
                p = __longlong_as_double((long long)(v.x) | ((long long)(v.y) << 32));
                hdr += __builtin_amdgcn_readfirstlane(int(WIDE ? v.z : (v.z & 0xffffu)));
                ++grp;
                v.x = 0xffffffffu;
                v.y = 0xffffffffu;
                v.z = WIDE ? 0xffffffffu : (v.z | 0xffffu);
            }
            const uint32_t vw[4] = {v.x, v.y, v.z, v.w};
            if (DBG == 9) {   // loads only
                acc0 += double(vw[0] ^ vw[1] ^ vw[2] ^ vw[3]);
                continue;
            }
            bool multi = false;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (WIDE) {
                    const uint32_t x = vw[i];
                    const double t = wsrc[min(x, zslot)];
                    if (i & 1) acc1 += t; else acc0 += t;
                    if (MULTI) multi |= int(x) < -1;
                } else {
                    const uint32_t lo = vw[i] & 0xffffu, hi = vw[i] >> 16;
                    if (DBG == 1) {
                        acc0 += double(lo);
                        acc1 += double(hi);
                    } else {
                        acc0 += wsrc[min(lo, zslot)];
                        acc1 += wsrc[min(hi, zslot)];
                    }
                    if (MULTI) multi |= (lo >= 0x8000u && lo != 0xffffu) || (hi >= 0x8000u && hi != 0xffffu);
                }
            }
            if (MULTI && multi) {   // rare: epsilon-composite edges
                for (int i = 0; i < 4; ++i) {
                    for (int h = 0; h < (WIDE ? 1 : 2); ++h) {
                        int g = -1;
                        if (WIDE) {
                            if (int(vw[i]) < -1) g = -(int(vw[i]) + 2);
                        } else {
                            const uint32_t x = (vw[i] >> (16 * h)) & 0xffffu;
                            if (x >= 0x8000u && x != 0xffffu) g = a.m.multi_edge[x - 0x8000u];
                        }
                        if (g >= 0)
                            for (int q = a.m.pptr[g]; q < a.m.pptr[g + 1]; ++q) acc0 += wsrc[a.m.pidx[q]];
                    }
                }
            }
        }
    };
    if (kStreams && rows > 0) {
        for (int c0 = 0;;) {   // A holds rows [c0, c0 + D), B [c0 + D, c0 + 2D)
            apply(A, c0);
            if (c0 + D >= rows) break;
            load(A, c0 + 2 * D);
            apply(B, c0 + D);
            c0 += 2 * D;
            if (c0 >= rows) break;
            load(B, c0 + D);
        }
    }
    flush();
    WFSA_STAMP(4)
    // the folded rmin column: a multi-bubble string's arrival, the k-th one
    // summing the string's stored values (retired at this wave's arrival) --
    // at the wave's end, off the stream pass and the QN update
    if (RF && rm_pos >= 0 && rm_lane.k > 1) {   // (its value stored: retired by now)
        const RminFold rf = WFSA_LATE_ARG(rf);
        rmin_arrive(rf, WFSA_LATE_ARG(bub.rmin_sv), rm_lane, rm_cv, rm_ci);
    }
    if (RF) {   // a big bubble's (min, x) pass (lane 0 held its index and Z; the staging is this wave's)
        const int big = __builtin_amdgcn_readfirstlane(rm_big.big);
        if (big >= 0) {
            const BubbleArgs bub = WFSA_LATE_ARG(bub);
            const RminFold rf = WFSA_LATE_ARG(rf);
            const double z = __shfl(rm_big.rv, 0, kWave);
            const int E = bub.big_lds_edges;
            char* stg = reinterpret_cast<char*>(lds) + bub.big_lds_off + w * big_stage_bytes(E);
            double* lw = reinterpret_cast<double*>(stg);
            int* lsd = reinterpret_cast<int*>(lw + E + 2 * kMaxBubbleNodes);
            big_bubble_min(bub, rf, big, z, lsd, lw, lw + E, rm_cv, rm_ci);
        }
    }
    // one log-likelihood partial per block (the QN finish sums them)
    __shared__ double wsum[1024 / kWave];
    __shared__ double wrv[1024 / kWave], wri[1024 / kWave];   // (RF: the waves' rmin candidates)
    ll_acc = wave_sum(ll_acc);
    if (lane == 0) wsum[w] = ll_acc;
    if (RF) {
        // the ambiguous traversal strings (values from the kernels before this launch), strided over the grid
        for (int i = bid * int(blockDim.x) + int(threadIdx.x); i < a.rf.n_trav; i += nblk * int(blockDim.x)) {
            const int st = a.rf.trav[i];
            min_pair(rm_cv, rm_ci, a.rf.rmin_log[st], double(st));
        }
        for (int o = 32; o > 0; o >>= 1) min_pair(rm_cv, rm_ci, __shfl_xor(rm_cv, o, kWave), __shfl_xor(rm_ci, o, kWave));
        if (lane == 0) {
            wrv[w] = rm_cv;
            wri[w] = rm_ci;
        }
    }
    // The block's partials: the last of its waves to get here sums them (an
    // LDS counter, no block barrier), so a QN wave goes on to its update as
    // soon as its own stream share is done -- behind a block barrier it
    // started only once the slowest stream wave of its block was done (c3:
    // polls matched at 20-24 us for arrivals landed by 20,
    // profiles/r06/fbs_trace_polls.log).  (The workgroup-scope release /
    // acquire orders each wave's LDS partials before its count.)
    unsigned prev_in = 0u;
    if (lane == 0) prev_in = __hip_atomic_fetch_add(&blk_in, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
    prev_in = __builtin_amdgcn_readfirstlane(prev_in);   // (every lane active: lane 0's)
    const bool writer = prev_in == unsigned(wpb - 1);
    const bool self_fin = QN && a.qw.self_finish;
    if (writer && lane == 0) {
        double t = 0.0;
        for (int i = 0; i < wpb; ++i) t += wsum[i];
        if (self_fin) store_wt(a.ll_part + bid, t);   // (read by this launch's finisher)
        else a.ll_part[bid] = t;
        if (RF) {
            double v = wrv[0], idx = wri[0];
            for (int i = 1; i < wpb; ++i) min_pair(v, idx, wrv[i], wri[i]);
            if (self_fin) {
                store_wt(a.rf.part + 2 * bid, v);
                store_wt(a.rf.part + 2 * bid + 1, idx);
            } else {
                a.rf.part[2 * bid] = v;
                a.rf.part[2 * bid + 1] = idx;
            }
        }
    }
    // this block's slice of the per-edge weights and the zeroed result, for
    // the kernels after this one (nothing in this launch reads them; skipped
    // when the QN update rides in the launch)
    if (W_LDS && !a.no_streams && !a.no_slice) edge_weight_slice(a, bid, nblk);
    const bool qn_wave = QN && w == wpb - 2 && bid < a.qw.n_waves;
    if (qn_wave) {   // this step's QN update
        const QnWave qw = WFSA_LATE_ARG(qw);
#ifdef WFSA_EXPERIMENTS
        qn_wave_run<PX>(qw, bid, tr);
#else
        qn_wave_run<PX>(qw, bid, nullptr);
#endif
    }
    // Self-finish: every block's partials writer (its log-likelihood
    // partial) and every QN wave (its constraints' partials) arrive once
    // their stores retired -- a wave in both roles counts twice; the last
    // arrival runs this step's finish (the wave form, write-through loads,
    // the same sums as the next launch's finish wave) and publishes the row
    // -- no finish left for the next launch, and the Run's last row needs no
    // finish kernel of its own.  A step the previous finish halted publishes
    // its skipped row from its QN waves instead.
    if (self_fin && (writer || qn_wave)) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned add = unsigned(writer) + unsigned(qn_wave);
        unsigned before = 0u;
        if (lane == 0) before = __hip_atomic_fetch_add(a.qw.done + a.qw.parity, add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        before = __shfl(before, 0, kWave);
        if (before + add == unsigned(nblk + a.qw.n_waves) && load_wt(a.qw.halted + 1) == 0u) {
            double info[7];
            unsigned st = kQnRan;
            const QnFinish fin = WFSA_LATE_ARG(qw.fin);
            qn_finish_compute<true, true, PX>(fin, nullptr, info, st);
            if (lane == 0) qn_finish_publish(fin, info, st);
        }
    }
    WFSA_STAMP(7)
#undef WFSA_STAMP
}

// Group headers (stream_hdr_words), written after the streams are emitted:
// lane l's first chunk of group g gets p of its string and the group's row
// count; the string's words follow in the same chunk.
__global__ void stream_headers_kernel(uint4* stream, const int64_t* g_base, const int32_t* g_len,
                                      const double* p_lane, int32_t n_groups, int32_t wide) {
    const int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (k >= int64_t(n_groups) * kWave) return;
    const int g = int(k / kWave), l = int(k % kWave);
    uint4 v = stream[g_base[g] + l];
    const unsigned long long pb = (unsigned long long)(__double_as_longlong(p_lane[k]));
    v.x = uint32_t(pb);
    v.y = uint32_t(pb >> 32);
    v.z = wide ? uint32_t(g_len[g]) : ((v.z & 0xffff0000u) | uint32_t(g_len[g]));
    stream[g_base[g] + l] = v;
}

// One block copies out[0, n) to host-mapped memory in 16-byte stores (n
// rounded up to even; both buffers are padded), fences at system scope and
// stores the next sequence number into the host-mapped flag.  A separate
// launch after the reductions: the kernel boundary makes their results
// visible, where a last-block ticket would need an L2 write-back per block.
__global__ __launch_bounds__(256) void publish_kernel(const double* out, Publish pub) {
    const int n2 = (pub.n + 1) / 2;
    const double2* src = reinterpret_cast<const double2*>(out);
    double2* dst = reinterpret_cast<double2*>(pub.host_out);
    for (int i = int(threadIdx.x); i < n2; i += int(blockDim.x)) {
        double2 v = src[i];
        if (pub.add) {   // out[1 + j] += add[j]: add[2i - 1], add[2i]
            if (2 * i >= 1 && 2 * i - 1 < pub.n - 1) v.x += pub.add[2 * i - 1];
            if (2 * i < pub.n - 1) v.y += pub.add[2 * i];
        }
        dst[i] = v;
    }
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) {   // (the sequence counter is an agent-scope atomic everywhere: qn_publish_row)
        const unsigned v = __hip_atomic_fetch_add(pub.seq, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
        __hip_atomic_store(pub.host_flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Per-iteration reduction (ReduceArgs): a block per tile of consecutive
// parameters in slot order, one more for the log-likelihood.  No atomics.
__global__ __launch_bounds__(kReduceBlock) void reduce_kernel(ReduceArgs a) {
    if (a.halted && *a.halted) return;
    const int t = int(threadIdx.x);
    const int tb = int(blockIdx.x);
    if (tb == a.n_tiles) {   // log-likelihood, fixed order
        __shared__ double red[kReduceBlock];
        red[t] = strided_sum(a.ll_part, a.n_ll, t, kReduceBlock);
        __syncthreads();
        for (int w = kReduceBlock / 2; w > 0; w >>= 1) {
            if (t < w) red[t] += red[t + w];
            __syncthreads();
        }
        if (t == 0) a.out[0] = red[0];
        return;
    }
    __shared__ int sp[kReduceTileParams + 1], cb[kReduceTileParams + 1];
    __shared__ double res[kReduceTileParams], cp[kMaxChunks];
    const int p0 = a.tile_ptr[tb], ns = a.tile_ptr[tb + 1] - p0;
    if (a.contrib) {
        const int s0 = a.seg_ptr[p0], c0 = a.chunk_ptr[p0];
        for (int i = t; i <= ns; i += kReduceBlock) {
            sp[i] = a.seg_ptr[p0 + i] - s0;
            cb[i] = a.chunk_ptr[p0 + i] - c0;
        }
        __syncthreads();
        seg_sums<kReduceBlock>(a.contrib + a.grp_base[tb], sp, cb, ns, res, cp);
    }
    for (int i = t; i < ns; i += kReduceBlock) {
        const int j = a.param_at[p0 + i];
        double v = a.out[1 + j];
        if (a.fixed) v += a.fixed[j];
        if (a.contrib) v += res[i];
        a.out[1 + j] = v;
    }
}

// out[1 + j] = sum of the preparation-time gradient slabs, in slab order
__global__ __launch_bounds__(256) void slab_sum_kernel(const double* __restrict__ gpart, int32_t n_slabs,
                                                      int32_t n_params, double* __restrict__ out) {
    const int j = int(blockIdx.x) * 256 + int(threadIdx.x);
    if (j >= n_params) return;
    double s = 0.0;
    for (int k0 = 0; k0 < n_slabs; k0 += 8) {
        double v[8];
#pragma unroll
        for (int b = 0; b < 8; ++b) v[b] = gpart[size_t(min(k0 + b, n_slabs - 1)) * size_t(n_params) + size_t(j)];
#pragma unroll
        for (int b = 0; b < 8; ++b)
            if (k0 + b < n_slabs) s += v[b];
    }
    out[1 + j] = s;
}

// host-mapped weights -> device, 16-byte loads (both buffers padded to even)
__global__ __launch_bounds__(256) void stage_kernel(const double2* __restrict__ host_w, double2* __restrict__ w,
                                                    double2* __restrict__ ewp, int32_t n2) {
    for (int32_t i = int32_t(blockIdx.x * blockDim.x + threadIdx.x); i < n2; i += int32_t(gridDim.x * blockDim.x)) {
        const double2 v = host_w[i];
        w[i] = v;
        ewp[i] = make_double2(exp(v.x), exp(v.y));
    }
}

// Per iteration: log-weight, weight and parameter record of every combined
// edge from the GetWeight-expanded parameter vector.
__global__ void edge_weights_kernel(const double* __restrict__ w_full, const int32_t* __restrict__ pptr,
                                    const int32_t* __restrict__ pidx, double* __restrict__ lw,
                                    double* __restrict__ ew, EdgeRec* __restrict__ erec, int64_t n,
                                    double* __restrict__ out, int64_t n_out) {
    const int64_t g = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (g < n_out) out[g] = 0.0;
    if (g >= n) return;
    const int32_t b = pptr[g], e = pptr[g + 1];
    double s = 0.0;
    for (int32_t k = b; k < e; ++k) s += w_full[pidx[k]];
    lw[g] = s;
    ew[g] = exp(s);
    erec[g] = EdgeRec{s, e > b ? pidx[b] : 0, e - b};
}

__global__ void node_end_kernel(const int32_t* __restrict__ x_ptr, const double* __restrict__ x_w,
                                double* __restrict__ node_end, int32_t n_nodes) {
    const int32_t u = int32_t(blockIdx.x * blockDim.x + threadIdx.x);
    if (u >= n_nodes) return;
    double s = 0.0;
    for (int32_t x = x_ptr[u]; x < x_ptr[u + 1]; ++x) s += x_w[x];
    node_end[u] = s;
}

}  // namespace

hipError_t configure_kernels(int max_dynamic_lds) {
    const void* fns[] = {reinterpret_cast<const void*>(&trav_kernel<MODE_WEIGHTED>),
                         reinterpret_cast<const void*>(&trav_kernel<MODE_MIN>),
                         reinterpret_cast<const void*>(&trav_kernel<MODE_COUNT>),
                         reinterpret_cast<const void*>(&trav_kernel<MODE_EMIT>),
                         reinterpret_cast<const void*>(&fbc_kernel<0, false, true>),
                         reinterpret_cast<const void*>(&fbc_kernel<1, false, true>),
                         reinterpret_cast<const void*>(&fbc_kernel<2, false, true>),
                         reinterpret_cast<const void*>(&fbc_kernel<0, true, true>),
                         reinterpret_cast<const void*>(&fbc_kernel<1, true, true>),
                         reinterpret_cast<const void*>(&fbc_kernel<2, true, true>),
                         reinterpret_cast<const void*>(&fbs_kernel<false, true, false>),
                         reinterpret_cast<const void*>(&fbs_kernel<false, true, true>),
                         reinterpret_cast<const void*>(&fbs_kernel<true, true, false>),
                         reinterpret_cast<const void*>(&fbs_kernel<true, true, true>),
                         reinterpret_cast<const void*>(&fbs_kernel<false, true, false, 0, true>),
                         reinterpret_cast<const void*>(&fbs_kernel<false, true, true, 0, true>),
                         reinterpret_cast<const void*>(&fbs_kernel<true, true, false, 0, true>),
                         reinterpret_cast<const void*>(&fbs_kernel<true, true, true, 0, true>),
                         reinterpret_cast<const void*>(&fbs_kernel<false, true, false, 0, false, true>),
                         reinterpret_cast<const void*>(&fbs_kernel<false, true, false, 0, true, true>),
                         reinterpret_cast<const void*>(&fbs_kernel<false, true, false, 0, false, true, true>),
#ifdef WFSA_EXPERIMENTS
                         reinterpret_cast<const void*>(&fbs_kernel<false, true, false, 1>),
                         reinterpret_cast<const void*>(&fbs_kernel<false, true, false, 3>),
                         reinterpret_cast<const void*>(&fbs_kernel<false, true, false, 4>),
                         reinterpret_cast<const void*>(&fbs_kernel<false, true, false, 5>),
                         reinterpret_cast<const void*>(&fbs_kernel<false, true, false, 6>),
                         reinterpret_cast<const void*>(&fbs_kernel<false, true, false, 7>),
                         reinterpret_cast<const void*>(&fbs_kernel<false, true, false, 8>),
                         reinterpret_cast<const void*>(&fbs_kernel<false, true, false, 9>),
                         reinterpret_cast<const void*>(&fbs_kernel<false, true, false, 10>),
                         reinterpret_cast<const void*>(&fbs_kernel<false, true, false, 1, false, true>),
                         reinterpret_cast<const void*>(&fbs_kernel<false, true, false, 3, false, true>),
                         reinterpret_cast<const void*>(&fbs_kernel<false, true, false, 4, false, true>),
                         reinterpret_cast<const void*>(&fbs_kernel<false, true, false, 5, false, true>),
                         reinterpret_cast<const void*>(&fbs_kernel<false, true, false, 8, false, true>),
                         reinterpret_cast<const void*>(&fbs_kernel<false, true, false, 9, false, true>),
                         reinterpret_cast<const void*>(&fbs_kernel<false, true, false, 11, false, true>),
                         reinterpret_cast<const void*>(&fbs_kernel<false, true, false, 12, false, true>),
                         reinterpret_cast<const void*>(&fbs_kernel<false, true, false, 13, false, true>),
#endif
                         reinterpret_cast<const void*>(&wide_kernel<false>)};
    for (const void* f : fns) {   // (static LDS counts against the same 160 KiB)
        hipFuncAttributes attr{};
        hipError_t e = hipFuncGetAttributes(&attr, f);
        if (e != hipSuccess) return e;
        e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                max_dynamic_lds - int(attr.sharedSizeBytes));
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_trav(TravMode mode, const TravArgs& a, int grid, hipStream_t stream) {
    const dim3 block(unsigned(a.slab.waves_per_block * kWave));
    const size_t lds = size_t(a.slab.bytes) * size_t(a.slab.waves_per_block);
    switch (mode) {
        case MODE_WEIGHTED:
            hipLaunchKernelGGL(trav_kernel<MODE_WEIGHTED>, dim3(unsigned(grid)), block, lds, stream, a);
            break;
        case MODE_COUNT:
            hipLaunchKernelGGL(trav_kernel<MODE_COUNT>, dim3(unsigned(grid)), block, lds, stream, a);
            break;
        case MODE_EMIT:
            hipLaunchKernelGGL(trav_kernel<MODE_EMIT>, dim3(unsigned(grid)), block, lds, stream, a);
            break;
        case MODE_MIN:
            hipLaunchKernelGGL(trav_kernel<MODE_MIN>, dim3(unsigned(grid)), block, lds, stream, a);
            break;
    }
    return hipGetLastError();
}

// Lane per bubble, 64-lane blocks: sum forward and (min, x) forward over the
// bubble's topologically listed edges with the node vectors in LDS
// ([node][lane], conflict-free); the min path never exceeds the sum, so both
// stay linear and one log per bubble gives vb = log(min path / Z).
__global__ __launch_bounds__(64) void rmin_bubble_kernel(RminArgs a) {
    if (a.halted && *a.halted) return;
    extern __shared__ double rmin_lds[];   // [max_nodes][64] sum, then [max_nodes][64] min
    double (*sA)[64] = reinterpret_cast<double (*)[64]>(rmin_lds);
    double (*sM)[64] = reinterpret_cast<double (*)[64]>(rmin_lds + size_t(a.max_nodes) * 64);
    const int lane = int(threadIdx.x);
    const int b = int(blockIdx.x) * 64 + lane;
    if (b >= a.n_bub) return;
    const int32_t* rec = a.bub + a.bub_off[b];
    const int nodes = rec[0] & 0xffff, edges = rec[0] >> 16;
    for (int u = 0; u < nodes; ++u) {
        sA[u][lane] = u == 0 ? 1.0 : 0.0;
        sM[u][lane] = u == 0 ? 1.0 : INFINITY;
    }
    const int2* ed = reinterpret_cast<const int2*>(rec + 4);   // (code, src | dst << 16), 8-byte aligned
    for (int e = 0; e < edges; ++e) {
        const int2 cs = ed[e];
        double wgt;
        if (cs.x >= 0) {
            wgt = a.ewp[cs.x];
        } else {
            const int g = -cs.x - 2;
            double t = 0.0;
            for (int q = a.m.pptr[g]; q < a.m.pptr[g + 1]; ++q) t += a.w[a.m.pidx[q]];
            wgt = exp(t);
        }
        const int src = cs.y & 0xffff, dst = cs.y >> 16;
        sA[dst][lane] += sA[src][lane] * wgt;
        if (wgt > 0.0) sM[dst][lane] = fmin(sM[dst][lane], sM[src][lane] * wgt);
    }
    a.vb[b] = log(sM[nodes - 1][lane] / sA[nodes - 1][lane]);
}

// Lane per ambiguous string (rmin_strings_block, qn_device.hpp): block minima to part[].
__global__ __launch_bounds__(kRminBlock) void rmin_strings_kernel(RminArgs a) {
    if (a.halted && *a.halted) return;
    __shared__ double wv[kRminBlock / kWave], wi[kRminBlock / kWave];
    rmin_strings_block(a, int(blockIdx.x), wv, wi);
}

// the block minima -> res (a second launch: the kernel boundary orders the
// partials; a device-scope fence per block costs an L2 write-back on gfx950)
__global__ __launch_bounds__(256) void rmin_final_kernel(RminArgs a, int n_part) {
    if (a.halted && *a.halted) return;
    __shared__ double wv[4], wi[4];
    const int lane = int(threadIdx.x);
    double v = INFINITY, idx = -1.0;
    for (int k = lane; k < n_part; k += 256) min_pair(v, idx, a.part[2 * k], a.part[2 * k + 1]);
    for (int o = 32; o > 0; o >>= 1) min_pair(v, idx, __shfl_xor(v, o, 64), __shfl_xor(idx, o, 64));
    if ((lane & 63) == 0) {
        wv[lane >> 6] = v;
        wi[lane >> 6] = idx;
    }
    __syncthreads();
    if (lane == 0) {
        for (int k = 1; k < 4; ++k) min_pair(v, idx, wv[k], wi[k]);
        a.res[0] = idx >= 0.0 ? exp(v) : 0.0;
        a.res[1] = idx;
    }
}

// The rmin column across ranks, between two Min all-reduces of key
// (phase 0: key[0] = this rank's value, +inf without an ambiguous string;
// 1: key[1] = its global string index if it holds the global minimum, else
// +inf -- ties to the lower string, as within a rank; 2: res = the result,
// (0, -1) when no rank has an ambiguous string).
__global__ void rmin_rank_kernel(double* res, double* key, double base, int phase) {
    if (threadIdx.x != 0) return;
    if (phase == 0) key[0] = res[1] >= 0.0 ? res[0] : INFINITY;
    else if (phase == 1) key[1] = (res[1] >= 0.0 && res[0] == key[0]) ? res[1] + base : INFINITY;
    else {
        const bool any = key[1] < INFINITY;
        res[0] = any ? key[0] : 0.0;
        res[1] = any ? key[1] : -1.0;
    }
}

hipError_t launch_rmin_rank(double* res, double* key, double base, int phase, hipStream_t stream) {
    hipLaunchKernelGGL(rmin_rank_kernel, dim3(1), dim3(64), 0, stream, res, key, base, phase);
    return hipGetLastError();
}

hipError_t launch_rmin(const RminArgs& a, hipStream_t stream, bool final) {
    if (a.n_bub > 0 && a.vb)
        hipLaunchKernelGGL(rmin_bubble_kernel, dim3(unsigned((a.n_bub + 63) / 64)), dim3(64),
                           2 * size_t(a.max_nodes) * 64 * sizeof(double), stream, a);
    const unsigned g = unsigned(std::max<int64_t>(1, (a.n_amb + kRminBlock - 1) / kRminBlock));
    hipLaunchKernelGGL(rmin_strings_kernel, dim3(g), dim3(kRminBlock), 0, stream, a);
    if (final) hipLaunchKernelGGL(rmin_final_kernel, dim3(1), dim3(256), 0, stream, a, int(g));
    return hipGetLastError();
}

hipError_t launch_hf(const HfArgs& a, hipStream_t stream, const HfTravArgs* trav, int trav_grid) {
    constexpr int NW = kHfBlock / kWave;
    if (a.n_bubbles > 0)
        hipLaunchKernelGGL(hf_kernel, dim3(unsigned((a.n_bubbles + NW - 1) / NW)), dim3(kHfBlock), 0, stream, a);
    if (trav && trav->n_list > 0)
    {
        const dim3 g(static_cast<unsigned>(trav_grid)), b(kHfBlock);
        switch (trav->vm / kWave) {
        case 1: hipLaunchKernelGGL(hf_trav_kernel<1>, g, b, 0, stream, *trav); break;
        case 2: hipLaunchKernelGGL(hf_trav_kernel<2>, g, b, 0, stream, *trav); break;
        case 4: hipLaunchKernelGGL(hf_trav_kernel<4>, g, b, 0, stream, *trav); break;
        default: hipLaunchKernelGGL(hf_trav_kernel<8>, g, b, 0, stream, *trav); break;
        }
    }
    if (a.n_pattern > 0)
        hipLaunchKernelGGL(hf_sum_kernel, dim3(unsigned((a.n_pattern + 255) / 256)), dim3(256), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_wide(bool counting, const WideArgs& a, int grid, hipStream_t stream, bool min_mode) {
    const size_t lds = (!counting && !min_mode && a.grad_lds) ? size_t(a.m.n_params) * sizeof(double) : 0;
    if (min_mode)
        hipLaunchKernelGGL((wide_kernel<false, true>), dim3(unsigned(grid)), dim3(kWideBlock), 0, stream, a);
    else if (counting)
        hipLaunchKernelGGL(wide_kernel<true>, dim3(unsigned(grid)), dim3(kWideBlock), 0, stream, a);
    else
        hipLaunchKernelGGL(wide_kernel<false>, dim3(unsigned(grid)), dim3(kWideBlock), lds, stream, a);
    return hipGetLastError();
}

hipError_t launch_wide2(const WideArgs& a, int grid, int waves, size_t lds, hipStream_t stream) {
    if (a.rmin_log)
        hipLaunchKernelGGL(wide2_kernel<true>, dim3(unsigned(grid)), dim3(unsigned(waves * kWave)), lds, stream, a);
    else
        hipLaunchKernelGGL(wide2_kernel<false>, dim3(unsigned(grid)), dim3(unsigned(waves * kWave)), lds, stream, a);
    return hipGetLastError();
}

template <int NI>
void launch_wave_pull_ni(const WideArgs& a, int grid, int waves, size_t lds, hipStream_t stream) {
    if (a.rmin_log)
        hipLaunchKernelGGL((wave_pull_kernel<NI, true>), dim3(unsigned(grid)), dim3(unsigned(waves * kWave)), lds, stream, a);
    else
        hipLaunchKernelGGL((wave_pull_kernel<NI, false>), dim3(unsigned(grid)), dim3(unsigned(waves * kWave)), lds, stream, a);
}

hipError_t launch_wave_pull(const WideArgs& a, int grid, int waves, size_t lds, hipStream_t stream) {
    switch (a.pl.items) {
    case 4: launch_wave_pull_ni<4>(a, grid, waves, lds, stream); break;
    case 6: launch_wave_pull_ni<6>(a, grid, waves, lds, stream); break;
    case 8: launch_wave_pull_ni<8>(a, grid, waves, lds, stream); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_pull_weights(const int32_t* g, int64_t n, int64_t n_lw, const double* ew, const double* lw,
                               double* w, double* lw_out, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const unsigned nb = unsigned(std::min<int64_t>((n + 255) / 256, 4096));
    hipLaunchKernelGGL(pull_weights_kernel, dim3(nb), dim3(256), 0, stream, g, n, n_lw, ew, lw, w, lw_out);
    return hipGetLastError();
}

hipError_t launch_pair_weights(const int4* ent, int64_t n, const double* ew, const double* lw, double* pw,
                               hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const unsigned g = unsigned(std::min<int64_t>((n + 255) / 256, 4096));
    hipLaunchKernelGGL(pair_weights_kernel, dim3(g), dim3(256), 0, stream, ent, n, ew, lw, pw);
    return hipGetLastError();
}

hipError_t launch_stream_headers(uint4* stream, const int64_t* g_base, const int32_t* g_len, const double* p_lane,
                                int32_t n_groups, int32_t wide, hipStream_t s) {
    const int64_t n = int64_t(n_groups) * kWave;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(stream_headers_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, s, stream, g_base, g_len,
                       p_lane, n_groups, wide);
    return hipGetLastError();
}

static hipError_t launch_compiled_impl(const CompiledArgs& a, int grid, int block, size_t lds, hipStream_t stream);

// one launch of a stream-kernel instance, with dispatch timestamps when
// events are given (hipExtLaunchKernelGGL: the kernel itself, as rocprof
// measures it)
template <typename K>
static hipError_t go(K k, int grid, int block, size_t lds, hipStream_t stream, hipEvent_t ev0, hipEvent_t ev1,
                     const CompiledArgs& a) {
    const dim3 g{unsigned(grid), 1, 1}, b{unsigned(block), 1, 1};
    if (ev0 || ev1) hipExtLaunchKernelGGL(k, g, b, uint32_t(lds), stream, ev0, ev1, 0u, a);
    else hipLaunchKernelGGL(k, g, b, lds, stream, a);
    return hipGetLastError();
}

hipError_t launch_compiled(const CompiledArgs& a, int grid, int block, size_t lds, hipStream_t stream, hipEvent_t ev0,
                           hipEvent_t ev1) {
    if (ev0 || ev1) {   // no dispatch events inside a stream capture (the graph path records none)
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(stream, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) ev0 = ev1 = nullptr;
    }
    if (!a.with_grad && a.d_tab > 0) {   // the delta stream kernel: narrow words, no composites, w staged (the host checks)
#ifdef WFSA_EXPERIMENTS
        static const int dbg = experiment_knob("WFSA_FBS_DBG");
        switch (dbg) {   // timing variants of the delta kernel (results wrong by design)
        case 1: return go(fbs_kernel<false, true, false, 1, false, true>, grid, block, lds, stream, ev0, ev1, a);
        case 3: return go(fbs_kernel<false, true, false, 3, false, true>, grid, block, lds, stream, ev0, ev1, a);
        case 4: return go(fbs_kernel<false, true, false, 4, false, true>, grid, block, lds, stream, ev0, ev1, a);
        case 5: return go(fbs_kernel<false, true, false, 5, false, true>, grid, block, lds, stream, ev0, ev1, a);
        case 8: return go(fbs_kernel<false, true, false, 8, false, true>, grid, block, lds, stream, ev0, ev1, a);
        case 9: return go(fbs_kernel<false, true, false, 9, false, true>, grid, block, lds, stream, ev0, ev1, a);
        case 11: return go(fbs_kernel<false, true, false, 11, false, true>, grid, block, lds, stream, ev0, ev1, a);
        case 12: return go(fbs_kernel<false, true, false, 12, false, true>, grid, block, lds, stream, ev0, ev1, a);
        case 13: return go(fbs_kernel<false, true, false, 13, false, true>, grid, block, lds, stream, ev0, ev1, a);
        default: break;
        }
#endif
        if (a.qw.on && a.qw.px.on && a.rf.part)   // ... across ranks (the peer exchange)
            return go(fbs_kernel<false, true, false, 0, true, true, true, true>, grid, block, lds, stream, ev0, ev1, a);
        if (a.qw.on && a.qw.px.on)
            return go(fbs_kernel<false, true, false, 0, false, true, true, true>, grid, block, lds, stream, ev0, ev1, a);
        if (a.qw.on && a.rf.part)   // with this step's QN update and the rmin column folded in
            return go(fbs_kernel<false, true, false, 0, true, true, true>, grid, block, lds, stream, ev0, ev1, a);
        if (a.qw.on)   // with this step's QN update (the host checks: bubbles fused or none)
            return go(fbs_kernel<false, true, false, 0, false, true, true>, grid, block, lds, stream, ev0, ev1, a);
        if (a.bub_on && a.bub.rmin_acc)
            return go(fbs_kernel<false, true, false, 0, true, true>, grid, block, lds, stream, ev0, ev1, a);
        return go(fbs_kernel<false, true, false, 0, false, true>, grid, block, lds, stream, ev0, ev1, a);
    }
    if (ev0) {
        const hipError_t e = hipEventRecord(ev0, stream);
        if (e != hipSuccess) return e;
    }
    const hipError_t e = launch_compiled_impl(a, grid, block, lds, stream);
    if (e != hipSuccess || !ev1) return e;
    return hipEventRecord(ev1, stream);
}

static hipError_t launch_compiled_impl(const CompiledArgs& a, int grid, int block, size_t lds, hipStream_t stream) {
    const dim3 g{unsigned(grid), 1, 1}, b{unsigned(block), 1, 1};
    if (!a.with_grad) {   // per-iteration form: w staged in LDS or read from global
#ifdef WFSA_EXPERIMENTS
        static const int dbg = experiment_knob("WFSA_FBS_DBG");
        if (dbg == 1) {
            hipLaunchKernelGGL((fbs_kernel<false, true, false, 1>), g, b, lds, stream, a);
            return hipGetLastError();
        }
        if (dbg == 2) {
            hipLaunchKernelGGL((fbs_kernel<false, false, false, 0>), g, b, 0, stream, a);
            return hipGetLastError();
        }
        if (dbg == 3) {
            hipLaunchKernelGGL((fbs_kernel<false, true, false, 3>), g, b, lds, stream, a);
            return hipGetLastError();
        }
        if (dbg == 4) {
            hipLaunchKernelGGL((fbs_kernel<false, true, false, 4>), g, b, lds, stream, a);
            return hipGetLastError();
        }
        if (dbg == 5) {
            hipLaunchKernelGGL((fbs_kernel<false, true, false, 5>), g, b, lds, stream, a);
            return hipGetLastError();
        }
        if (dbg == 6) {
            hipLaunchKernelGGL((fbs_kernel<false, true, false, 6>), g, b, lds, stream, a);
            return hipGetLastError();
        }
        if (dbg == 7) {
            hipLaunchKernelGGL((fbs_kernel<false, true, false, 7>), g, b, lds, stream, a);
            return hipGetLastError();
        }
        if (dbg == 10) {   // no bubble code, two blocks per CU (<= 64 VGPRs): needs WFSA_FUSE_BUBBLES=0
            hipLaunchKernelGGL((fbs_kernel<false, true, false, 10>), g, b, lds, stream, a);
            return hipGetLastError();
        }
        if (dbg == 8) {
            hipLaunchKernelGGL((fbs_kernel<false, true, false, 8>), g, b, lds, stream, a);
            return hipGetLastError();
        }
        if (dbg == 9) {
            hipLaunchKernelGGL((fbs_kernel<false, true, false, 9>), g, b, lds, stream, a);
            return hipGetLastError();
        }
#endif
        const int key = (a.tables >= 1 ? 4 : 0) + (a.wide ? 2 : 0) + (a.multi ? 1 : 0);
        if (a.bub_on && a.bub.rmin_acc) {   // the bubbles also feed the rmin column
            switch (key) {
                case 0: hipLaunchKernelGGL((fbs_kernel<false, false, false, 0, true>), g, b, 0, stream, a); break;
                case 1: hipLaunchKernelGGL((fbs_kernel<false, false, true, 0, true>), g, b, 0, stream, a); break;
                case 2: hipLaunchKernelGGL((fbs_kernel<true, false, false, 0, true>), g, b, 0, stream, a); break;
                case 3: hipLaunchKernelGGL((fbs_kernel<true, false, true, 0, true>), g, b, 0, stream, a); break;
                case 4: hipLaunchKernelGGL((fbs_kernel<false, true, false, 0, true>), g, b, lds, stream, a); break;
                case 5: hipLaunchKernelGGL((fbs_kernel<false, true, true, 0, true>), g, b, lds, stream, a); break;
                case 6: hipLaunchKernelGGL((fbs_kernel<true, true, false, 0, true>), g, b, lds, stream, a); break;
                default: hipLaunchKernelGGL((fbs_kernel<true, true, true, 0, true>), g, b, lds, stream, a); break;
            }
            return hipGetLastError();
        }
        switch (key) {
            case 0: hipLaunchKernelGGL((fbs_kernel<false, false, false>), g, b, 0, stream, a); break;
            case 1: hipLaunchKernelGGL((fbs_kernel<false, false, true>), g, b, 0, stream, a); break;
            case 2: hipLaunchKernelGGL((fbs_kernel<true, false, false>), g, b, 0, stream, a); break;
            case 3: hipLaunchKernelGGL((fbs_kernel<true, false, true>), g, b, 0, stream, a); break;
            case 4: hipLaunchKernelGGL((fbs_kernel<false, true, false>), g, b, lds, stream, a); break;
            case 5: hipLaunchKernelGGL((fbs_kernel<false, true, true>), g, b, lds, stream, a); break;
            case 6: hipLaunchKernelGGL((fbs_kernel<true, true, false>), g, b, lds, stream, a); break;
            default: hipLaunchKernelGGL((fbs_kernel<true, true, true>), g, b, lds, stream, a); break;
        }
        return hipGetLastError();
    }
    const int key = a.tables * 2 + (a.wide ? 1 : 0);
    switch (key) {
        case 4: hipLaunchKernelGGL((fbc_kernel<2, false, true>), g, b, lds, stream, a); break;
        case 5: hipLaunchKernelGGL((fbc_kernel<2, true, true>), g, b, lds, stream, a); break;
        case 2: hipLaunchKernelGGL((fbc_kernel<1, false, true>), g, b, lds, stream, a); break;
        case 3: hipLaunchKernelGGL((fbc_kernel<1, true, true>), g, b, lds, stream, a); break;
        case 1: hipLaunchKernelGGL((fbc_kernel<0, true, true>), g, b, 0, stream, a); break;
        default: hipLaunchKernelGGL((fbc_kernel<0, false, true>), g, b, 0, stream, a); break;
    }
    return hipGetLastError();
}

int fbs_qn_blocks_per_cu(int block, size_t lds) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fbs_kernel<false, true, false, 0, false, true, true>, block,
                                                     lds) != hipSuccess)
        return 0;
    return nb;
}

int bubble_waves(int32_t n_small4, int32_t n_small, int32_t n_big) { return n_big + int(small_chunks(n_small4, n_small)); }

hipError_t launch_bubbles(const BubbleArgs& a, hipStream_t stream) {
    const int waves = bubble_waves(a.n_small4, a.n_small, a.n_big);
    if (waves <= 0) return hipSuccess;
    constexpr int WPB = kBubbleBlock / kWave;
    if (a.rmin_acc)
        hipLaunchKernelGGL(bubble_kernel<true>, dim3(unsigned((waves + WPB - 1) / WPB)), dim3(kBubbleBlock), 0, stream, a);
    else
        hipLaunchKernelGGL(bubble_kernel<false>, dim3(unsigned((waves + WPB - 1) / WPB)), dim3(kBubbleBlock), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_reduce(const ReduceArgs& a, hipStream_t stream) {
    hipLaunchKernelGGL(reduce_kernel, dim3(unsigned(a.n_tiles + 1)), dim3(kReduceBlock), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_slab_sum(const double* gpart, int32_t n_slabs, int32_t n_params, double* out, hipStream_t stream) {
    if (n_params <= 0 || n_slabs <= 0) return hipSuccess;
    hipLaunchKernelGGL(slab_sum_kernel, dim3(unsigned((n_params + 255) / 256)), dim3(256), 0, stream, gpart, n_slabs,
                       n_params, out);
    return hipGetLastError();
}

hipError_t launch_publish(const double* out, const Publish& pub, hipStream_t stream) {
    hipLaunchKernelGGL(publish_kernel, dim3(1), dim3(256), 0, stream, out, pub);
    return hipGetLastError();
}

hipError_t launch_stage(const double* host_w, double* w, double* ewp, int32_t n, hipStream_t stream) {
    const int32_t n2 = (n + 2) / 2;   // n weights and the zero slot w[n]
    const unsigned blocks = unsigned(std::min<int32_t>(8, (n2 + 255) / 256));
    hipLaunchKernelGGL(stage_kernel, dim3(blocks), dim3(256), 0, stream, reinterpret_cast<const double2*>(host_w),
                       reinterpret_cast<double2*>(w), reinterpret_cast<double2*>(ewp), n2);
    return hipGetLastError();
}

hipError_t launch_edge_weights(const double* w_full, const int32_t* pptr, const int32_t* pidx, double* lw,
                               double* ew, EdgeRec* erec, int64_t n_edges, double* out, int64_t n_out,
                               hipStream_t stream) {
    const int64_t n = std::max(n_edges, n_out);
    if (n <= 0) return hipSuccess;
    const unsigned blocks = unsigned((n + 255) / 256);
    hipLaunchKernelGGL(edge_weights_kernel, dim3(blocks), dim3(256), 0, stream, w_full, pptr, pidx, lw, ew, erec,
                       n_edges, out, n_out);
    return hipGetLastError();
}

hipError_t launch_node_end(const int32_t* x_ptr, const double* x_w, double* node_end, int32_t n_nodes,
                           hipStream_t stream) {
    if (n_nodes <= 0) return hipSuccess;
    const unsigned blocks = unsigned((n_nodes + 255) / 256);
    hipLaunchKernelGGL(node_end_kernel, dim3(blocks), dim3(256), 0, stream, x_ptr, x_w, node_end, n_nodes);
    return hipGetLastError();
}

}  // namespace wfsa
