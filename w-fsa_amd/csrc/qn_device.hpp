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

// Deterministic per-segment sums over one contiguous run of bubble
// contribution slots (the runs of consecutive parameters in slot order).
// Segment q of nseg owns v[sp[q], sp[q+1]) (sp relative, sp[0] = 0, in LDS).
// The block's NT threads cut the run into pieces of C consecutive slots,
// thread t the t-th; a thread sums its piece segment by segment in slot
// order (a segment wholly inside the piece is written at once), and a
// segment that crosses pieces is completed by adding its piece partials in
// thread order.  The order of every addition depends only on the segment
// lengths and C, never on timing: the same inputs give the same bits.
template <int NT>
struct SegScratch {
    double pf[NT], pl[NT];   // partial of the piece's first / last segment
    int fs[NT], ls[NT];      // the piece's first / last segment (-1: empty piece)
};

// C: slots per piece, at least ceil(sp[nseg] / NT)
__device__ inline int seg_piece(int total, int nt) { return max((total + nt - 1) / nt, 16); }

template <int NT>
__device__ void seg_sums(const double* __restrict__ v, const int* sp, int nseg, int C, double* res,
                         SegScratch<NT>& sc) {
    const int t = int(threadIdx.x);
    const int total = sp[nseg];
    for (int q = t; q < nseg; q += NT) res[q] = 0.0;
    __syncthreads();
    const int a0 = t * C, a1 = min(a0 + C, total);
    int f = -1, q = -1;
    double p0 = 0.0, acc = 0.0;
    if (a0 < a1) {
        int lo = 0, hi = nseg;   // the segment holding slot a0: last q with sp[q] <= a0
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (sp[mid] <= a0) lo = mid; else hi = mid;
        }
        q = f = lo;
        int nxt = sp[q + 1];
        for (int s0 = a0; s0 < a1; s0 += 8) {
            double x[8];
#pragma unroll
            for (int b = 0; b < 8; ++b) x[b] = v[min(s0 + b, a1 - 1)];
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                const int s = s0 + b;
                if (s >= a1) break;
                while (s >= nxt) {   // segment q ends inside this piece
                    if (q == f) p0 = acc; else res[q] = acc;
                    acc = 0.0;
                    ++q;
                    nxt = sp[q + 1];
                }
                acc += x[b];
            }
        }
        if (q == f) p0 = acc;
    }
    sc.pf[t] = p0;
    sc.pl[t] = acc;
    sc.fs[t] = f;
    sc.ls[t] = q;
    __syncthreads();
    for (int k = t; k < nseg; k += NT) {
        const int b0 = sp[k], b1 = sp[k + 1];
        if (b0 == b1) continue;
        const int ta = b0 / C, tb = (b1 - 1) / C;
        if (ta == tb) {
            if (k == sc.fs[ta]) res[k] = sc.pf[ta];
            else if (k == sc.ls[ta]) res[k] = sc.pl[ta];   // (else written by the piece itself)
        } else {   // k is the last segment of piece ta and the first of tb
            double s = sc.pl[ta];
            for (int u = ta + 1; u < tb; ++u) s += sc.pf[u];
            res[k] = s + sc.pf[tb];
        }
    }
    __syncthreads();
}

}  // namespace wfsa
