// Device-resident QuasiNewton step: the KKT-diagonal update of
// QuasiNewtonLearner::OptimizationStep (src/QuasiNewtonLearner.cpp:162-201,
// with ComputeExpX :53-56, ComputeG :148-160, ComputeLambdaNext :127-146,
// Learner::LambdaUpdate src/Learner.cpp:438-462, HaltCondition :88-91 and
// GetOptimizationInfo :68-86) after the objective/gradient kernels of the
// same step: qn_update (wave per constraint) + qn_finish (one wave).  It keeps x, lambda and the next step's w_full in
// HBM, so consecutive steps need nothing from the host; each step publishes
// its info row to host-mapped memory and bumps the completion flag.
//
// The arithmetic follows the host code operation for operation (the same
// summation orders, no FMA contraction) so the device and host trajectories
// agree to the last bits up to exp()'s rounding.
#include "fb_kernels.hpp"
#include "qn_device.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>

#pragma clang fp contract(off)

namespace wfsa {

namespace {

constexpr int kQnUpdateBlock = 256;   // four constraints (one wavefront each) per block

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

// qn_update: one wavefront per constraint.  Every quantity of the update is
// local to a constraint (its members are a contiguous, ascending range of
// parameters), so waves are independent; each block writes its partial
// (g_min, g_max, lambda_min, graderr) and qn_finish reduces them.  Up to 64
// members: lane m owns member m (exp and the x update); g and the
// lambda_next numerator are summed by lane 0 in member order, as the host
// does.  Larger groups stride their members over the lanes.
__global__ __launch_bounds__(kQnUpdateBlock) void qn_update_kernel(QnArgs a) {
    if (*a.halted) return;
    constexpr int W = kQnUpdateBlock / 64;
    __shared__ double sh_ev[W][64], sh_gv[W][64];
    __shared__ double sh_bc[W][2];
    __shared__ double red[W][4];
    const int lane = int(threadIdx.x) & 63, w = int(threadIdx.x) >> 6;
    const int c = int(blockIdx.x) * W + w;
    double gmin = INFINITY, gmax = -INFINITY, lmin = INFINITY, gerr = 0.0;
    if (c < a.k) {
        const int b = a.cptr[c], e = a.cptr[c + 1], nm = e - b;
        const double lam = a.lambda[c];
        double g, laux;
        if (nm <= 64) {
            double xi = 0.0, gi = 0.0;
            int fo = 0;
            if (lane < nm) {
                xi = a.x[b + lane];
                fo = a.full_of[b + lane];
                gi = a.out[1 + fo] + (a.fixed ? a.fixed[fo] : 0.0);
            }
            const double ei = lane < nm ? exp(xi) : 0.0;
            sh_ev[w][lane] = ei;
            sh_gv[w][lane] = gi;
            wave_sync();
            if (lane == 0) {   // ComputeG, ComputeLambdaNext in member order
                double gg = -1.0;
                for (int m = 0; m < nm; ++m) gg += sh_ev[w][m];
                double r = lam * gg;
                for (int m = 0; m < nm; ++m) r -= sh_gv[w][m];
                sh_bc[w][0] = gg;
                sh_bc[w][1] = r / (gg + 1.0);
            }
            wave_sync();
            g = sh_bc[w][0];
            laux = sh_bc[w][1];
            if (lane < nm) {   // graderr (old lambda), x update (lambda_next), next weights
                const double aux = ei * lam;
                gerr = fabs(gi + aux);
                const double xn = xi - a.eta * ((gi + ei * laux) / aux);
                a.x[b + lane] = xn;
                a.grad[b + lane] = gi;
                a.w_full[fo] = xn;   // GetWeight for the next step
                a.ewp[fo] = exp(xn);
            }
        } else {   // large groups (dense automata): members strided over the lanes,
                   // lane sums combined by a fixed xor tree (deterministic; the
                   // host's member-order sums differ from it by rounding only)
            double gs = 0.0, gv = 0.0;
            for (int i = b + lane; i < e; i += 64) {
                const double ex = exp(a.x[i]);
                const int fo = a.full_of[i];
                const double gi = a.out[1 + fo] + (a.fixed ? a.fixed[fo] : 0.0);
                a.expx[i] = ex;
                a.grad[i] = gi;
                gs += ex;
                gv += gi;
            }
            for (int o = 32; o > 0; o >>= 1) {
                gs += __shfl_xor(gs, o, 64);
                gv += __shfl_xor(gv, o, 64);
            }
            g = -1.0 + gs;
            laux = (lam * g - gv) / (g + 1.0);
            for (int i = b + lane; i < e; i += 64) {
                const double ex = a.expx[i], gi = a.grad[i];
                const double aux = ex * lam;
                gerr = fmax(gerr, fabs(gi + aux));
                const double xn = a.x[i] - a.eta * ((gi + ex * laux) / aux);
                a.x[i] = xn;
                a.w_full[a.full_of[i]] = xn;
                a.ewp[a.full_of[i]] = exp(xn);
            }
        }
        if (lane == 0) {   // LambdaUpdate (src/Learner.cpp:438-462)
            const double d = lam - laux;
            a.lambda[c] = a.exp_lambda ? lam * exp(-a.eta * (d / lam)) : lam - a.eta * d;
        }
        gmin = g;
        gmax = g;
        lmin = lam;
    }
    for (int o = 32; o > 0; o >>= 1) gerr = fmax(gerr, __shfl_xor(gerr, o, 64));
    if (lane == 0) {
        red[w][0] = gmin;
        red[w][1] = gmax;
        red[w][2] = lmin;
        red[w][3] = gerr;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        if (blockIdx.x == 0 && !a.ll_part) *a.ll_val = a.out[0];   // the finish may run after out is reused
        double r0 = red[0][0], r1 = red[0][1], r2 = red[0][2], r3 = red[0][3];
        for (int v = 1; v < W; ++v) {
            r0 = fmin(r0, red[v][0]);
            r1 = fmax(r1, red[v][1]);
            r2 = fmin(r2, red[v][2]);
            r3 = fmax(r3, red[v][3]);
        }
        double* p = a.partial + size_t(blockIdx.x) * 4;
        p[0] = r0;
        p[1] = r1;
        p[2] = r2;
        p[3] = r3;
    }
}

// qn_finish: the info row of the step (the reductions of qn_update's
// partials and, without the tail kernel, of the per-wave log-likelihood
// partials in a fixed order), the halt decision, then the publication.
__global__ __launch_bounds__(64) void qn_finish_kernel(QnArgs a) { qn_finish_wave(a); }

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

int qn_update_blocks(int32_t k) {
    constexpr int W = kQnUpdateBlock / 64;
    return std::max(1, (k + W - 1) / W);
}

hipError_t launch_qn_update(const QnArgs& a, hipStream_t stream) {
    hipLaunchKernelGGL(qn_update_kernel, dim3(unsigned(qn_update_blocks(a.k))), dim3(kQnUpdateBlock), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_qn_finish(const QnArgs& a, hipStream_t stream) {
    hipLaunchKernelGGL(qn_finish_kernel, dim3(1), dim3(64), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_qn_weights(const double* x, const int32_t* trim, int32_t n_full, double* w_full, double* ewp,
                             hipStream_t stream) {
    const unsigned blocks = unsigned((n_full + 1 + 255) / 256);
    hipLaunchKernelGGL(qn_weights_kernel, dim3(blocks), dim3(256), 0, stream, x, trim, n_full, w_full, ewp);
    return hipGetLastError();
}

}  // namespace wfsa
