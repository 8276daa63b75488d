// Device helpers shared by the QN step kernel and the reduction kernel: wave
// reductions and the deterministic segmented sum of bubble contribution slots.
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>

#include "fb_kernels.hpp"

namespace wfsa {

__device__ inline double wave_reduce(double v, int op) {   // op 0 min, 1 max, 2 sum (fixed order)
    for (int o = 32; o > 0; o >>= 1) {
        const double t = __shfl_xor(v, o, 64);
        v = op == 0 ? fmin(v, t) : (op == 1 ? fmax(v, t) : v + t);
    }
    return v;
}

// Per-parameter sums of the bubble contribution slots, in an order that
// depends on the parameter's own slots only (not on the slot layout, the
// reduction groups or the block size), so the same contributions give the
// same bits under every layout: parameter q's slots are cut into chunks of
// kSlotChunk (16) from its first slot, each chunk summed by a fixed tree
// (chunk_tree: pairs, then pairs of pairs), then the chunk sums added in
// chunk order.
//
// One reduction group (a QN constraint, or a run of positions) holds nseg
// parameters: q owns logical slots [sp[q], sp[q+1]) and chunks [cb[q],
// cb[q+1]) (both relative to the group, in LDS).  Chunk c of the group is
// stored contiguously at v[16 c, 16 c + 16) (a chunk's tail is zero padding),
// so the bubble kernels' stores -- lanes holding same-shaped bubbles write a
// parameter's consecutive slots -- coalesce, and so do these loads: eight
// lanes read a chunk as eight 16-byte pieces and reduce it by shuffles in the
// tree's order.  The chunk sums go to LDS (cp, kMaxChunks, fb_kernels.hpp)
// and a thread per parameter adds them; a group with more chunks sums each
// parameter's chunks in one thread straight from memory (same tree).
static_assert(kSlotChunk == 16, "chunk_tree and the 8-lane chunk loads assume 16-slot chunks");
__device__ inline double chunk_tree(const double* x) {   // ((p0+p1)+(p2+p3)) + ((p4+p5)+(p6+p7)), pk = x2k + x2k+1
    double p[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) p[k] = x[2 * k] + x[2 * k + 1];
    return ((p[0] + p[1]) + (p[2] + p[3])) + ((p[4] + p[5]) + (p[6] + p[7]));
}
// the chunk sums of a group (nch <= kMaxChunks) into cp; no barrier
template <int NT>
__device__ inline void chunk_sums(const double* __restrict__ v, int nch, double* cp) {
    const int t = int(threadIdx.x);
    {
        // a wave reads 8 chunks per round (lane: chunk lane / 8, piece lane % 8),
        // kR rounds in flight; the shuffles follow chunk_tree's order
        constexpr int kR = NT >= 512 ? 2 : (NT >= 256 ? 4 : 8);
        const int lane = t & 63, wv = t >> 6, sub = lane & 7;
        constexpr int NW = NT / 64;
        const double2* v2 = reinterpret_cast<const double2*>(v);
        for (int c0 = wv * 8 * kR; c0 < nch; c0 += NW * 8 * kR) {
            double2 x[kR];
#pragma unroll
            for (int r = 0; r < kR; ++r) {
                const int c = c0 + 8 * r + (lane >> 3);
                x[r] = c < nch ? v2[size_t(c) * 8 + sub] : make_double2(0.0, 0.0);
            }
#pragma unroll
            for (int r = 0; r < kR; ++r) {
                double sr = x[r].x + x[r].y;
#pragma unroll
                for (int o = 1; o < 8; o <<= 1) sr += __shfl_xor(sr, o, 64);
                const int c = c0 + 8 * r + (lane >> 3);
                if (sub == 0 && c < nch) cp[c] = sr;
            }
        }
    }
}
// parameter q's sum from the chunk sums in cp (after a barrier); no barrier
template <int NT>
__device__ inline void member_sums(const int* cb, int nseg, const double* cp, double* res) {
    const int t = int(threadIdx.x);
    {
        for (int q = t; q < nseg; q += NT) {
            const int c0 = cb[q], c1 = cb[q + 1];
            double s = 0.0;
            int c = c0;
            for (; c + 8 <= c1; c += 8) {   // eight LDS loads in flight, added in order
                double y[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) y[i] = cp[c + i];
#pragma unroll
                for (int i = 0; i < 8; ++i) s += y[i];
            }
            for (; c < c1; ++c) s += cp[c];
            res[q] = s;
        }
    }
}
// cp holds cap chunk sums (kMaxChunks unless the caller sized it smaller)
template <int NT>
__device__ void seg_sums(const double* __restrict__ v, const int* sp, const int* cb, int nseg, double* res,
                         double* cp, int cap = kMaxChunks) {
    const int t = int(threadIdx.x);
    const int nch = cb[nseg];
    if (nch <= cap) {
        chunk_sums<NT>(v, nch, cp);
        __syncthreads();
        member_sums<NT>(cb, nseg, cp, res);
    } else {
        for (int q = t; q < nseg; q += NT) {
            double s = 0.0;
            for (int c = cb[q]; c < cb[q + 1]; ++c) {
                double x[kSlotChunk];
#pragma unroll
                for (int b = 0; b < kSlotChunk; ++b) x[b] = v[size_t(c) * kSlotChunk + size_t(b)];
                s += chunk_tree(x);
            }
            res[q] = s;
        }
    }
    __syncthreads();
}

// Write-through (sc1) 8-byte stores and sc1 loads: the hand-off inside one
// launch across CUs and XCDs (MI355X_MICROARCH.md, inter-workgroup
// visibility: sc1 stores, every storing wave's vmcnt(0) before its arrival,
// sc1 loads by the consumer after its poll has matched)
__device__ __forceinline__ void store_wt(double* p, double v) {
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)(__double_as_longlong(v)),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double load_wt(const double* p) {
    return __longlong_as_double((long long)(__hip_atomic_load(reinterpret_cast<unsigned long long*>(const_cast<double*>(p)),
                                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
}
__device__ __forceinline__ unsigned load_wt(const unsigned* p) {
    return __hip_atomic_load(const_cast<unsigned*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void store_wt(unsigned* p, unsigned v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the info row of a step into its host ring slot, then the flag; the
// system-scope release orders the row before the flag.  The sequence counter
// is an agent-scope atomic: two rows of one launch (a finish and a skipped
// step) may be published from different CUs.
__device__ inline void qn_publish_row(const QnFinish& f, const double* info, unsigned status) {
    double* row = f.host_ring + size_t(f.ring_slot) * kQnRow;
    for (int i = 0; i < 7; ++i) row[i] = info ? info[i] : 0.0;
    // the status and tag word last, released after the data: a reader that
    // sees the tag sees the row
    const double tw = double(status) + 16.0 * double(f.tag);
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(row + 7), (unsigned long long)(__double_as_longlong(tw)),
                       __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned v = __hip_atomic_fetch_add(f.seq, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    __hip_atomic_store(f.host_flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

constexpr int kMaxBlockWaves = 16;

// The in-kernel exchange across ranks (PeerX, peer_layout.hpp), by one
// wavefront: lane l's value v (l < nv) into slot [par][me][base + l] of every
// member's area, then flag fl there; then every member's flag fl awaited in
// this rank's area.  false: a member is late past the timeout or an area was
// poisoned -- then every area is poisoned and the status word set, so every
// member fails (Collective::check) instead of waiting.
__device__ inline bool peer_post_wait(const PeerX& x, size_t base, int nv, double v, int fl) {
    const int lane = int(threadIdx.x) & 63;
    const int n = x.nranks, par = int(x.seq & 1);
    const size_t mine = (size_t(par) * n + x.me) * kPeerCap + base;
    if (lane < nv)
        for (int r = 0; r < n; ++r) x.area[r][mine + lane] = v;   // (uncached: the stores reach the member)
    __threadfence_system();   // the slots before the flags, on every member
    bool ok = true;
    if (lane < n) {
        __hip_atomic_store(peer_flags(x.area[lane], n) + (size_t(par) * n + x.me) * kPeerFlags + fl, x.seq,
                           __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        const uint64_t* f = peer_flags(x.area[x.me], n) + (size_t(par) * n + lane) * kPeerFlags + fl;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < x.seq) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > x.timeout ||
                __hip_atomic_load(peer_poison(x.area[x.me], n), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) {
                ok = false;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
    ok = !__any(!ok);
    __threadfence_system();
    if (!ok) {
        if (lane < n)
            __hip_atomic_store(peer_poison(x.area[lane], n), uint64_t(1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (lane == 0) __hip_atomic_store(x.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    return ok;
}
// member r's value at slot base + l of this rank's area (after peer_post_wait)
__device__ inline double peer_slot(const PeerX& x, int r, size_t idx) {
    const int par = int(x.seq & 1);
    return __hip_atomic_load(x.area[x.me] + (size_t(par) * x.nranks + r) * kPeerCap + idx, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
}

// rmin column (fb_kernels.hpp RminArgs).  (value, index) minimum, ties to
// the lower index.
__device__ __forceinline__ void min_pair(double& v, double& i, double v2, double i2) {
    if (v2 < v || (v2 == v && i2 < i)) {
        v = v2;
        i = i2;
    }
}

// Block bid of the rmin strings pass (kRminBlock threads): lane per ambiguous
// string -- a compiled string sums its run of bubbles in order
// (deterministic), a traversal string's value is already in rmin_log -- and
// the block minimum to part[2 bid].  Run by rmin_strings_kernel, or folded
// into the QN step kernel's blocks (QnArgs::rm_on).  wv, wi: LDS, one per wave.
__device__ inline void rmin_strings_block(const RminArgs& a, int bid, double* wv, double* wi) {
    const int lane = int(threadIdx.x);
    const int64_t i = int64_t(bid) * kRminBlock + lane;
    double v = INFINITY, idx = -1.0;
    if (i < a.n_amb) {
        const int4 ent = a.amb[i];   // (string, first bubble, bubble count or -1, 0)
        double r = 0.0;
        if (ent.z < 0) {
            r = a.rmin_log[ent.x];
        } else if (a.sv) {   // stored per bubble by the evaluation: summed in bubble order
            for (int b = ent.y; b < ent.y + ent.z; ++b) r += a.sv[a.bpos[b]];
        } else if (!a.vb) {   // accumulated by the evaluation's bubble passes: read, re-arm
            r = a.rmin_log[ent.x];
            a.rmin_log[ent.x] = 0.0;
        } else {
            for (int b = ent.y; b < ent.y + ent.z; ++b) r += a.vb[b];
        }
        v = r;
        idx = double(ent.x);
    }
    for (int o = 32; o > 0; o >>= 1) min_pair(v, idx, __shfl_xor(v, o, 64), __shfl_xor(idx, o, 64));
    if ((lane & 63) == 0) {
        wv[lane >> 6] = v;
        wi[lane >> 6] = idx;
    }
    __syncthreads();
    if (lane == 0) {
        for (int k = 1; k < kRminBlock / 64; ++k) min_pair(v, idx, wv[k], wi[k]);
        a.part[2 * bid] = v;
        a.part[2 * bid + 1] = idx;
    }
    __syncthreads();   // (wv, wi reused by the caller)
}

// block-wide reduction by a fixed tree (every thread gets the result);
// red: kMaxBlockWaves doubles of LDS
__device__ inline double block_reduce(double v, int op, double* red) {
    const int t = int(threadIdx.x), nw = int(blockDim.x) / 64;
    v = wave_reduce(v, op);
    __syncthreads();
    if ((t & 63) == 0) red[t >> 6] = v;
    __syncthreads();
    double r = red[0];
    for (int i = 1; i < nw; ++i) r = op == 0 ? fmin(r, red[i]) : (op == 1 ? fmax(r, red[i]) : r + red[i]);
    __syncthreads();   // red is reused
    return r;
}

// A QN step's finish (QnFinish, fb_kernels.hpp), by every thread of one
// block: the info row from the QN block partials and the log-likelihood
// partials (fixed order) into thread 0's info[7] and status; then
// qn_finish_publish (thread 0): the halt decision (halt_pending, read by the
// next QN launch) and the publication.  red: kMaxBlockWaves doubles of LDS.
// WAVE: one wavefront computes it alone (the stream kernel's reserved finish
// wave; no block barriers), red unused
// PX: across ranks through the peer areas (f.px; its own kernel variants:
// the exchange's registers stay out of the one-rank kernels)
template <bool WAVE = false, bool WT = false, bool PX = false>   // WT: the partials read write-through (sc1): inside the launch that wrote them
__device__ inline void qn_finish_compute(const QnFinish& f, double* red, double* info, unsigned& status) {
    const int t = WAVE ? int(threadIdx.x) % 64 : int(threadIdx.x), nt = WAVE ? 64 : int(blockDim.x), nw = nt / 64;
    double gmin = INFINITY, gmax = -INFINITY, lmin = INFINITY, ge = 0.0;
    // a NaN partial (fmin / fmax would drop it) makes the row non-finite:
    // counted beside the minima
    double nanp = 0.0;
    for (int j0 = t; j0 < f.n_blocks; j0 += 4 * nt) {   // four blocks' partials in flight per thread
        double4 v[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            if constexpr (WT) {
                const double* p = f.partial + 4 * size_t(min(j0 + b * nt, f.n_blocks - 1));
                v[b] = make_double4(load_wt(p), load_wt(p + 1), load_wt(p + 2), load_wt(p + 3));
            } else {
                v[b] = reinterpret_cast<const double4*>(f.partial)[min(j0 + b * nt, f.n_blocks - 1)];
            }
        }
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            gmin = fmin(gmin, v[b].x);
            gmax = fmax(gmax, v[b].y);
            lmin = fmin(lmin, v[b].z);
            ge = fmax(ge, v[b].w);
            if (isnan(v[b].x) || isnan(v[b].y) || isnan(v[b].z) || isnan(v[b].w)) nanp = 1.0;
        }
    }
    // the log-likelihood partials in one order whichever form runs (the
    // first wavefront's strided sums, then its shuffle tree): a run's last
    // row (the one-block finish) and the others (the stream kernel's finish
    // wave) sum the same way
    double ll = 0.0;
    if constexpr (WT) {   // strided_sum's order, write-through loads
        if (f.ll_part && t < 64)
            for (int i0 = t; i0 < f.n_ll; i0 += 8 * 64) {
                double v[8];
#pragma unroll
                for (int b = 0; b < 8; ++b) v[b] = load_wt(f.ll_part + min(i0 + b * 64, f.n_ll - 1));
#pragma unroll
                for (int b = 0; b < 8; ++b)
                    if (i0 + b * 64 < f.n_ll) ll += v[b];
            }
    } else {
        ll = (f.ll_part && t < 64) ? strided_sum(f.ll_part, f.n_ll, t, 64) : 0.0;
    }
    ll = wave_reduce(ll, 2);
    double rv = INFINITY, ri = -1.0;   // rmin column from block minima, ties to the lower string
    if (f.rmin_part)   // (eight pairs' loads in flight per thread: the folded column has a pair per block)
        for (int j0 = t; j0 < f.rmin_n_part; j0 += 8 * nt) {
            double v[8], i[8];
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                const int j = min(j0 + b * nt, f.rmin_n_part - 1);
                v[b] = WT ? load_wt(f.rmin_part + 2 * j) : f.rmin_part[2 * j];
                i[b] = WT ? load_wt(f.rmin_part + 2 * j + 1) : f.rmin_part[2 * j + 1];
            }
#pragma unroll
            for (int b = 0; b < 8; ++b)
                if (v[b] < rv || (v[b] == rv && i[b] < ri)) {
                    rv = v[b];
                    ri = i[b];
                }
        }
    if (WAVE) {
        gmin = wave_reduce(gmin, 0);
        gmax = wave_reduce(gmax, 1);
        lmin = wave_reduce(lmin, 0);
        ge = wave_reduce(ge, 1);
        nanp = wave_reduce(nanp, 1);
    } else {
        gmin = block_reduce(gmin, 0, red);
        gmax = block_reduce(gmax, 1, red);
        lmin = block_reduce(lmin, 0, red);
        ge = block_reduce(ge, 1, red);
        nanp = block_reduce(nanp, 1, red);
    }
    for (int o = 32; o > 0; o >>= 1) {
        const double v = __shfl_xor(rv, o, 64), i = __shfl_xor(ri, o, 64);
        if (v < rv || (v == rv && i < ri)) {
            rv = v;
            ri = i;
        }
    }
    __shared__ double rr[kMaxBlockWaves][2];
    if (!WAVE) {
        if ((t & 63) == 0) {
            rr[t >> 6][0] = rv;
            rr[t >> 6][1] = ri;
        }
        __syncthreads();
        if (t < 64)   // (every lane of wave 0: the block's minimum)
            for (int w = 1; w < nw; ++w)
                if (rr[w][0] < rv || (rr[w][0] == rv && rr[w][1] < ri)) {
                    rv = rr[w][0];
                    ri = rr[w][1];
                }
    }
    if (PX && f.px.on && t < 64) {
        // across ranks: this rank's log-likelihood and rmin pair through the
        // peer areas; the sum in rank order, the minimum ties to the lower
        // (global) string
        const double rg = ri >= 0.0 ? ri + f.rm_base : -1.0;
        const size_t base = kPeerFinSlot + 4 * size_t(f.px_slot);
        const double v = t == 0 ? ll : (t == 1 ? rv : rg);
        if (peer_post_wait(f.px, base, 3, v, kPeerFinFlag + f.px_slot)) {
            double lls = 0.0, mv = INFINITY, mi = -1.0;
            for (int r = 0; r < f.px.nranks; ++r) {
                lls += peer_slot(f.px, r, base);
                min_pair(mv, mi, peer_slot(f.px, r, base + 1), peer_slot(f.px, r, base + 2));
            }
            ll = lls;
            rv = mv;
            ri = mi;
        } else {
            ll = NAN;   // (the host reports the member's failure: Collective::check)
        }
    }
    if (t == 0) {
        if (f.k == 0) gmin = gmax = lmin = 0.0;
        info[0] = f.plogp - (f.ll_part ? ll : *f.out0);
        info[1] = ge;
        info[2] = gmin;
        info[3] = gmax;
        info[4] = lmin;
        info[5] = 0.0;
        info[6] = 0.0;
        if (f.rmin_part) {
            info[5] = ri >= 0.0 ? exp(rv) : 0.0;
            info[6] = ri;
        } else if (f.rmin) {
            info[5] = f.rmin[0];
            info[6] = f.rmin[1];
        }
        bool finite = nanp == 0.0;
        for (int i = 0; i < 7; ++i) finite = finite && isfinite(info[i]);
        const bool halt = ge <= f.tol && fabs(gmin) <= f.tol && fabs(gmax) <= f.tol;
        status = !finite ? kQnNonFinite : (halt ? kQnHalted : kQnRan);
        if (f.halted && load_wt(f.halted + 2) != 0u) status = kQnTimedOut;   // (a QN wave's wait gave up)
    }
}

__device__ inline void qn_finish_publish(const QnFinish& f, const double* info, unsigned status) {
    // read by the next QN launch, or (write-through) by the QN waves of the
    // stream kernel this finish runs in
    if (status != kQnRan) __hip_atomic_store(f.halt_pending, status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    qn_publish_row(f, info, status);
}

template <bool PX = false>
__device__ inline void qn_finish(const QnFinish& f, double* red) {
    double info[7];
    unsigned status = kQnRan;
    qn_finish_compute<false, false, PX>(f, red, info, status);
    if (threadIdx.x == 0) qn_finish_publish(f, info, status);
}

}  // namespace wfsa
