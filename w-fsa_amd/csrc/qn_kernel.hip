// Device-resident QuasiNewton step: the KKT-diagonal update of
// QuasiNewtonLearner::OptimizationStep (src/QuasiNewtonLearner.cpp:162-201,
// with ComputeExpX :53-56, ComputeG :148-160, ComputeLambdaNext :127-146,
// Learner::LambdaUpdate src/Learner.cpp:438-462, HaltCondition :88-91 and
// GetOptimizationInfo :68-86) after the objective/gradient kernels of the
// same step, in ONE launch: qn_step_kernel, one block per constraint; the
// step's finish (qn_finish, qn_device.hpp: the info row, the halt decision)
// runs in the first block of the next step's stream kernel, or as a
// one-block launch (fb_kernels.hpp, QnFinish).  It keeps x, lambda and the
// next step's w_full in HBM, so consecutive steps need nothing from the host;
// each step publishes its info row to host-mapped memory and bumps the flag.
//
// Fused form: the members' gradients are completed here from the bubble
// contribution slots (the slots are laid out in trimmed-parameter order, so a
// constraint's members own one contiguous run, summed by seg_sums in a fixed
// order) -- no separate reduction launch.
//
// The arithmetic follows the host code operation for operation (the same
// summation orders, no FMA contraction) so the device and host trajectories
// agree to the last bits up to exp()'s rounding and the gradient's summation.
#include "fb_kernels.hpp"
#include "qn_device.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>

#pragma clang fp contract(off)

namespace wfsa {

namespace {

template <bool FUSED, int NT = kQnBlock>
__global__ __launch_bounds__(NT) void qn_step_kernel(QnArgs a) {
    const int t = int(threadIdx.x);
    const int c = int(blockIdx.x);
    // LDS sized by the host to the largest constraint (a.seg_cap members,
    // a.chunk_cap slot chunks), so every block of the grid is resident at once
    extern __shared__ __attribute__((aligned(16))) double qlds[];
    double* sg = qlds;
    double* se = sg + a.seg_cap;
    double* cp = se + a.seg_cap;
    int* sp = reinterpret_cast<int*>(cp + a.chunk_cap);
    int* cb = sp + a.seg_cap + 1;
    int* sfo = cb + a.seg_cap + 1;
    __shared__ double bc[2], red[kMaxBlockWaves];
    // The loads are issued in dependent rounds (the kernel is a chain of
    // global-memory latencies): the flags with the constraint's extent and its
    // slot group; its members' slot runs, full indices and x together with the
    // group's slot chunks; the members' constant gradient parts.
    if (WFSA_KDBG(a.dbg) == 3) return;   // (timing experiments: the launch alone)
    const bool have = c < a.k;
    const bool slots = FUSED && a.contrib && WFSA_KDBG(a.dbg) != 5;   // (5: timing experiments, no slot sums)
    int b = 0, e = 0, gnch = 0;
    int64_t gb = 0;
    double lam = 0.0;
    if (have) {
        b = a.cptr[c];
        e = a.cptr[c + 1];
        lam = a.lambda[c];
        if (slots) {
            gb = a.grp_base[c];
            gnch = a.grp_nch[c];
        }
    }
    // halted and halt_pending are written only by earlier launches: every
    // block of this one sees the same values
    if (a.halted[0] || a.halted[1]) {   // a step enqueued after the halt: published as skipped
        if (c == 0 && t == 0) {
            a.halted[0] = 1u;   // for the evaluation kernels of the later steps
            qn_publish_row(a.fin, nullptr, kQnSkipped);
        }
        return;
    }
    if (a.ll_stash && c == 0 && t == 0) *a.ll_stash = a.out[0];
    if (a.rm_on && c < a.rm_blocks) {   // the rmin strings pass's block c (one launch fewer per step)
        static_assert(kRminBlock == kQnBlock, "the folded rmin pass runs in the QN step's blocks");
        rmin_strings_block(a.rm, c, red, red + kMaxBlockWaves / 2);
    }
    if (c >= max(a.k, 1)) return;   // (blocks beyond the constraints: the rmin pass only)
    if (WFSA_KDBG(a.dbg) == 1) return;   // (timing experiments, WFSA_QN_DBG: the launch and first round only)
    double gerr = 0.0, g = 0.0;
    if (have) {
        const int nm = e - b;
        double laux;
        if (nm <= a.seg_cap) {
            constexpr int PT = kQnMaxSeg / NT;   // members per thread (at most)
            double xr[PT], ft[PT];
#pragma unroll
            for (int i = 0; i < PT; ++i) {
                const int m = t + i * NT;
                xr[i] = 0.0;
                ft[i] = 0.0;
                if (m < nm) {
                    sfo[m] = a.full_of[b + m];
                    xr[i] = a.x[b + m];
                    if (a.fixed_t) ft[i] = a.fixed_t[b + m];
                }
            }
            if (slots)   // the members' bubble slot runs and chunks (the host guarantees nm <= kQnMaxSeg)
                for (int i = t; i <= nm; i += NT) {
                    sp[i] = a.seg_ptr[b + i];
                    cb[i] = a.chunk_ptr[b + i];
                }
            const bool in_lds = slots && gnch <= a.chunk_cap;   // (else more than kMaxChunks: seg_sums from memory)
            if (in_lds && WFSA_KDBG(a.dbg) != 7) chunk_sums<NT>(a.contrib + gb, gnch, cp);   // the group's chunks, this round (7: timing, skipped)
            __syncthreads();
            const int s0 = slots ? sp[0] : 0, c0 = slots ? cb[0] : 0;
            double gp[PT];   // this thread's members: trivial-word + traversal parts
#pragma unroll
            for (int i = 0; i < PT; ++i) {
                const int m = t + i * NT;
                double gi = 0.0;
                if (m < nm) {
                    const int fo = sfo[m];
                    if (a.use_out) gi = a.out[1 + fo];
                    if (a.fixed_t) gi += ft[i];
                    else if (a.fixed) gi += a.fixed[fo];
                }
                gp[i] = gi;
            }
            if (in_lds) {   // each thread its members' chunk sums, in chunk order (member_sums' order)
#pragma unroll
                for (int i = 0; i < PT; ++i) {
                    const int m = t + i * NT;
                    if (m < nm) {
                        const int q0 = cb[m] - c0, q1 = WFSA_KDBG(a.dbg) == 6 ? q0 : cb[m + 1] - c0;   // (6: timing, no sums)
                        double sm = 0.0;
                        int q = q0;
                        for (; q + 8 <= q1; q += 8) {
                            double y[8];
#pragma unroll
                            for (int k = 0; k < 8; ++k) y[k] = cp[q + k];
#pragma unroll
                            for (int k = 0; k < 8; ++k) sm += y[k];
                        }
                        for (; q < q1; ++q) sm += cp[q];
                        sg[m] = gp[i] + sm;
                        se[m] = exp(xr[i]);
                    }
                }
            } else {
                if (slots) {
                    __syncthreads();   // every sp read as absolute above
                    for (int i = t; i <= nm; i += NT) {
                        sp[i] -= s0;
                        cb[i] -= c0;
                    }
                    __syncthreads();
                    seg_sums<NT>(a.contrib + gb, sp, cb, nm, sg, cp, a.chunk_cap);
                }
#pragma unroll
                for (int i = 0; i < PT; ++i) {
                    const int m = t + i * NT;
                    if (m < nm) {
                        sg[m] = slots ? gp[i] + sg[m] : gp[i];
                        se[m] = exp(xr[i]);
                    }
                }
            }
            __syncthreads();
            if (t == 0) {   // ComputeG, ComputeLambdaNext in member order
                double gg = -1.0;
                for (int m = 0; m < nm; ++m) gg += se[m];
                double r = lam * gg;
                for (int m = 0; m < nm; ++m) r -= sg[m];
                bc[0] = gg;
                bc[1] = r / (gg + 1.0);
            }
            __syncthreads();
            g = bc[0];
            laux = bc[1];
#pragma unroll
            for (int i = 0; i < PT; ++i) {   // graderr (old lambda), x update (lambda_next)
                const int m = t + i * NT;
                if (m >= nm) break;
                const double gi = sg[m], ei = se[m];
                const double aux = ei * lam;
                gerr = fmax(gerr, fabs(gi + aux));
                const double xn = xr[i] - a.eta * ((gi + ei * laux) / aux);
                const int fo = sfo[m];
                a.x[b + m] = xn;
                a.grad[b + m] = gi;
                a.w_full[fo] = xn;   // GetWeight for the next step
                a.ewp[fo] = exp(xn);
            }
        } else {   // large groups (dense automata; never fused): members strided
                   // over the threads, sums by a fixed tree (deterministic; the
                   // host's member-order sums differ from it by rounding only)
            double gs = 0.0, gv = 0.0;
            for (int i = b + t; i < e; i += NT) {
                const double ex = exp(a.x[i]);
                const int fo = a.full_of[i];
                double gi = a.out[1 + fo];
                if (a.fixed) gi += a.fixed[fo];
                a.expx[i] = ex;
                a.grad[i] = gi;
                gs += ex;
                gv += gi;
            }
            gs = block_reduce(gs, 2, red);
            gv = block_reduce(gv, 2, red);
            g = -1.0 + gs;
            laux = (lam * g - gv) / (g + 1.0);
            for (int i = b + t; i < e; i += NT) {
                const double ex = a.expx[i], gi = a.grad[i];
                const double aux = ex * lam;
                gerr = fmax(gerr, fabs(gi + aux));
                const double xn = a.x[i] - a.eta * ((gi + ex * laux) / aux);
                a.x[i] = xn;
                a.w_full[a.full_of[i]] = xn;
                a.ewp[a.full_of[i]] = exp(xn);
            }
        }
        if (t == 0) {   // LambdaUpdate (src/Learner.cpp:438-462)
            const double d = lam - laux;
            a.lambda[c] = a.exp_lambda ? lam * exp(-a.eta * (d / lam)) : lam - a.eta * d;
        }
    }
    // (max is exact in any order: members in wave 0 alone need no block barrier)
    gerr = (e - b <= 64) ? wave_reduce(gerr, 1) : block_reduce(gerr, 1, red);
    if (t == 0) {   // the block's partial for the step's finish (a later launch)
        double4 pv;
        pv.x = have ? g : INFINITY;
        pv.y = have ? g : -INFINITY;
        pv.z = have ? lam : INFINITY;
        pv.w = gerr;
        reinterpret_cast<double4*>(a.partial)[c] = pv;
    }
}

template <bool PX>
__global__ __launch_bounds__(kQnBlock) void qn_finish_kernel(QnFinish f) {
    if (f.halted[0] || f.halted[1]) return;   // the step was skipped (and published so)
    __shared__ double red[kMaxBlockWaves];
    qn_finish<PX>(f, red);
}

// initial w_full from x (qn_set_state)
__global__ void qn_weights_kernel(const double* x, const int32_t* trim, int32_t n_full, double* w_full, double* ewp) {
    const int j = int(blockIdx.x * blockDim.x + threadIdx.x);
    if (j < n_full) {
        const int tj = trim[j];
        w_full[j] = tj >= 0 ? x[tj] : (tj == -1 ? 0.0 : -INFINITY);
        ewp[j] = exp(w_full[j]);
    }
    if (j == n_full) {   // the zero slot of the stream kernel
        w_full[j] = 0.0;
        ewp[j] = 1.0;
    }
}

}  // namespace

hipError_t launch_qn_step(const QnArgs& a_in, bool fused, hipStream_t stream) {
    static const int dbg = experiment_knob("WFSA_QN_DBG");
    QnArgs a = a_in;
    a.dbg = dbg;
    if (a.seg_cap <= 0 || a.seg_cap > kQnMaxSeg) a.seg_cap = kQnMaxSeg;
    if (a.chunk_cap <= 0 || a.chunk_cap > kMaxChunks) a.chunk_cap = kMaxChunks;
    const size_t lds = (2 * size_t(a.seg_cap) + size_t(a.chunk_cap)) * sizeof(double) +
                       (3 * size_t(a.seg_cap) + 2) * sizeof(int);
    dim3 grid(unsigned(std::max({a.k, 1, a.rm_on ? a.rm_blocks : 0})));
    if (dbg == 4) {   // (timing experiments: an empty launch of a quarter of the blocks)
        grid = dim3(unsigned(std::max((a.k + 3) / 4, 1)));
        a.dbg = 3;
    }
    if (fused) hipLaunchKernelGGL((qn_step_kernel<true>), grid, dim3(kQnBlock), lds, stream, a);
    else hipLaunchKernelGGL((qn_step_kernel<false>), grid, dim3(kQnBlock), lds, stream, a);
    return hipGetLastError();
}

__global__ void copy_kernel(const double* __restrict__ src, double* __restrict__ dst, int64_t n) {
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[i];
}

__global__ void gather_kernel(const double* src, const int32_t* idx, int32_t n, double* dst) {
    const int i = int(blockIdx.x * blockDim.x + threadIdx.x);
    if (i < n) dst[i] = src[idx[i]];
}

hipError_t launch_gather(const double* src, const int32_t* idx, int32_t n, double* dst, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(gather_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, stream, src, idx, n, dst);
    return hipGetLastError();
}

hipError_t launch_qn_finish(const QnFinish& f, hipStream_t stream) {
    if (f.px.on) hipLaunchKernelGGL(qn_finish_kernel<true>, dim3(1), dim3(kQnBlock), 0, stream, f);
    else hipLaunchKernelGGL(qn_finish_kernel<false>, dim3(1), dim3(kQnBlock), 0, stream, f);
    return hipGetLastError();
}

hipError_t launch_copy(const double* src, double* dst, int64_t n, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(copy_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, stream, src, dst, n);
    return hipGetLastError();
}

hipError_t launch_qn_weights(const double* x, const int32_t* trim, int32_t n_full, double* w_full, double* ewp,
                             hipStream_t stream) {
    const unsigned blocks = unsigned((n_full + 1 + 255) / 256);
    hipLaunchKernelGGL(qn_weights_kernel, dim3(blocks), dim3(256), 0, stream, x, trim, n_full, w_full, ewp);
    return hipGetLastError();
}

}  // namespace wfsa
