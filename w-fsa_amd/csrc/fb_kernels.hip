// Forward-backward over the (position, node) trellis of each corpus string,
// one wavefront per string, the whole trellis of the string kept in a
// per-wave LDS slab.
//
// Replaces, per iteration, the reference's SpMV chain over the path matrices
// (Learner::ComputeModeledProbs / ComputeObjective, src/Learner.cpp:515-553;
// QuasiNewtonLearner::ComputeGrad, src/QuasiNewtonLearner.cpp:93-125) and,
// once, its path enumeration (Learner::BuildPaths, src/Learner.cpp:276-348,
// with Recognizer::RecognizeBFS, inc/Recognize.h:62-96).
//
// Per string s of length L (bytes c_0..c_{L-1}):
//   forward   alpha_0 = {start: 1};  alpha_{i+1}(T) = sum over edges S->T with
//             byte c_i of alpha_i(S) * w_edge;  every position is rescaled by
//             an exact power of two (its max -> [0.5, 1)), so no underflow and
//             no rounding is added by the scaling;
//   end       q_hat = sum_S alpha_L(S) * w_end(S);  log q = log q_hat + ln2 * E
//   backward  beta_L(S) = w_end(S) / q_hat;  beta_i(S) = sum_edges w * beta_{i+1}(T)
//             * 2^-d_{i+1};  an edge's posterior is alpha_i(S) * w * beta_{i+1}(T)
//             * 2^-d_{i+1}, added (times -p_s) to every parameter of the edge.
// Counting mode runs the same passes with every weight 1: q is the number of
// accepting paths, and an edge is "used" when its posterior is positive.
//
// Frontier nodes of a position are created on first touch through a node ->
// slot map in LDS (CAS claim, ballot compaction) and summed with LDS fp64
// atomics; live edges are logged for the backward pass, so the backward pass
// never searches the automaton again.
#include "fb_kernels.hpp"

#include <hip/hip_runtime.h>

#include <cmath>

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
__device__ __forceinline__ void global_add(double* p, double v) {
    __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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

template <bool COUNTING>
__global__ __launch_bounds__(256) void fb_kernel(FBArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = lane_id();
    const int wib = int(threadIdx.x) / kWave;
    const int wpb = int(blockDim.x) / kWave;
    const int gw = int(blockIdx.x) * wpb + wib;
    const int nw = int(gridDim.x) * wpb;

    unsigned char* base = smem + size_t(wib) * size_t(a.slab.bytes);
    double* falpha = reinterpret_cast<double*>(base + a.lay.alpha);
    double* fbeta = reinterpret_cast<double*>(base + a.lay.beta);
    int* fstate = reinterpret_cast<int*>(base + a.lay.state);
    int* e_g = reinterpret_cast<int*>(base + a.lay.eg);
    int* e_src = reinterpret_cast<int*>(base + a.lay.esrc);
    int* e_dst = reinterpret_cast<int*>(base + a.lay.edst);
    int* fpos = reinterpret_cast<int*>(base + a.lay.fpos);
    int* epos = reinterpret_cast<int*>(base + a.lay.epos);
    int* dsc = reinterpret_cast<int*>(base + a.lay.dsc);
    int* slot = reinterpret_cast<int*>(base + a.lay.slot);

    const ModelView& m = a.m;
    const int cap_f = a.slab.cap_f, cap_e = a.slab.cap_e;

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
            fbeta[0] = 0.0;
            fpos[0] = 0;
            fpos[1] = 1;
            epos[0] = 0;
            dsc[0] = 0;
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
            const int fb = fpos[i];
            const int fe = nF;
            for (int fbase = fb; fbase < fe && !ovf; fbase += kWave) {
                const int f = fbase + lane;
                const bool act = f < fe;
                int lo = 0, cnt = 0;
                double af = 0.0;
                if (act) {
                    af = falpha[f];
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
                        v = COUNTING ? af : af * m.o_w[g];
                    }
                    int sl = has ? ld_rlx(&slot[d]) : 0;
                    const bool need = has && sl < 0;
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
                        fbeta[idx] = 0.0;
                    }
                    nF += nwon;
                    wave_sync();
                    if (need) sl = ld_rlx(&slot[d]);
                    if (has) {
                        lds_add(&falpha[sl], v);
                        const int k = nE + rank_below(hm);
                        e_g[k] = g;
                        e_src[k] = f;
                        e_dst[k] = sl;
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
                fpos[i + 2] = nF;
                epos[i + 1] = nE;
                dsc[i + 1] = ex;
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
        const int fl0 = alive ? fpos[L] : 0;
        const int fl1 = alive ? nF : 0;
        for (int j = fl0 + lane; j < fl1; j += kWave) {
            const int S = fstate[j];
            qh += falpha[j] * (COUNTING ? m.node_end_count[S] : m.node_end[S]);
        }
        qh = wave_sum(qh);
        if (alive) {
            int es = 0;
            for (int j = 1 + lane; j <= L; j += kWave) es += dsc[j];
            esum = wave_sum_i(es);
        }
        const double lq = qh > 0.0 ? log(qh) + kLn2 * double(esum) : -INFINITY;
        const double ps = COUNTING ? 0.0 : a.p[sidx];
        if (lane == 0) {
            if (COUNTING) {
                if (a.path_count) a.path_count[sidx] = qh > 0.0 ? ldexp(qh, esum) : 0.0;
                if (a.recognized) a.recognized[sidx] = qh > 0.0 ? 1 : 0;
            } else if (a.logq) {
                a.logq[sidx] = lq;
            }
        }
        if (!COUNTING) ll_acc += ps * lq;
        edges_acc += (unsigned long long)nE;
        if (!(qh > 0.0)) continue;
        if (COUNTING && !a.used) continue;

        // ---------------- backward ----------------
        const double inv_q = 1.0 / qh;
        for (int j = fl0 + lane; j < fl1; j += kWave) {
            const int S = fstate[j];
            const double af = falpha[j];
            fbeta[j] = (COUNTING ? m.node_end_count[S] : m.node_end[S]) * inv_q;
            for (int x = m.x_ptr[S]; x < m.x_ptr[S + 1]; ++x) {
                const double xi = af * (COUNTING ? 1.0 : m.x_w[x]) * inv_q;
                if (!(xi > 0.0)) continue;
                for (int k = m.x_pptr[x]; k < m.x_pptr[x + 1]; ++k) {
                    if (COUNTING) a.used[m.x_pidx[k]] = 1;
                    else global_add(&a.grad[m.x_pidx[k]], -ps * xi);
                }
            }
        }
        wave_sync();
        for (int i = L - 1; i >= 0; --i) {
            const double sc = ldexp(1.0, -dsc[i + 1]);
            const int eb = epos[i], ee = epos[i + 1];
            for (int k = eb + lane; k < ee; k += kWave) {
                const int g = e_g[k];
                const int f = e_src[k];
                const int h = e_dst[k];
                const double b = (COUNTING ? 1.0 : m.o_w[g]) * fbeta[h] * sc;
                if (b != 0.0) lds_add(&fbeta[f], b);
                const double xi = falpha[f] * b;
                if (xi > 0.0) {
                    for (int q = m.o_pptr[g]; q < m.o_pptr[g + 1]; ++q) {
                        if (COUNTING) a.used[m.o_pidx[q]] = 1;
                        else global_add(&a.grad[m.o_pidx[q]], -ps * xi);
                    }
                }
            }
            wave_sync();
        }
    }

    if (lane == 0) {
        if (!COUNTING) a.ll_part[gw] = ll_acc;
        if (a.live_edges && edges_acc) atomicAdd(a.live_edges, edges_acc);
    }
}

__global__ void edge_weights_kernel(const double* __restrict__ w_full, const int32_t* __restrict__ pptr,
                                    const int32_t* __restrict__ pidx, double* __restrict__ out, int64_t n) {
    const int64_t g = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (g >= n) return;
    double s = 0.0;
    for (int32_t k = pptr[g]; k < pptr[g + 1]; ++k) s += w_full[pidx[k]];
    out[g] = exp(s);
}

__global__ void node_end_kernel(const int32_t* __restrict__ x_ptr, const double* __restrict__ x_w,
                                double* __restrict__ node_end, int32_t n_nodes) {
    const int32_t u = int32_t(blockIdx.x * blockDim.x + threadIdx.x);
    if (u >= n_nodes) return;
    double s = 0.0;
    for (int32_t x = x_ptr[u]; x < x_ptr[u + 1]; ++x) s += x_w[x];
    node_end[u] = s;
}

// out[0] = sum of the per-wave log-likelihood partials, in a fixed order
__global__ __launch_bounds__(256) void finalize_kernel(const double* __restrict__ part, int32_t n,
                                                       double* __restrict__ out) {
    __shared__ double red[256];
    double s = 0.0;
    for (int32_t i = int32_t(threadIdx.x); i < n; i += 256) s += part[i];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (int(threadIdx.x) < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[0] = red[0];
}

}  // namespace

hipError_t configure_fb_kernels(int max_dynamic_lds) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&fb_kernel<true>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, max_dynamic_lds);
    if (e != hipSuccess) return e;
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&fb_kernel<false>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, max_dynamic_lds);
}

hipError_t launch_fb(bool counting, const FBArgs& a, int grid, hipStream_t stream) {
    const dim3 block(unsigned(a.slab.waves_per_block * kWave));
    const size_t lds = size_t(a.slab.bytes) * size_t(a.slab.waves_per_block);
    if (counting)
        hipLaunchKernelGGL(fb_kernel<true>, dim3(unsigned(grid)), block, lds, stream, a);
    else
        hipLaunchKernelGGL(fb_kernel<false>, dim3(unsigned(grid)), block, lds, stream, a);
    return hipGetLastError();
}

hipError_t launch_edge_weights(const double* w_full, const int32_t* pptr, const int32_t* pidx, double* out,
                               int64_t n_edges, hipStream_t stream) {
    if (n_edges <= 0) return hipSuccess;
    const unsigned blocks = unsigned((n_edges + 255) / 256);
    hipLaunchKernelGGL(edge_weights_kernel, dim3(blocks), dim3(256), 0, stream, w_full, pptr, pidx, out, n_edges);
    return hipGetLastError();
}

hipError_t launch_node_end(const int32_t* x_ptr, const double* x_w, double* node_end, int32_t n_nodes,
                           hipStream_t stream) {
    if (n_nodes <= 0) return hipSuccess;
    const unsigned blocks = unsigned((n_nodes + 255) / 256);
    hipLaunchKernelGGL(node_end_kernel, dim3(blocks), dim3(256), 0, stream, x_ptr, x_w, node_end, n_nodes);
    return hipGetLastError();
}

hipError_t launch_finalize(const double* ll_part, int32_t n_part, double* out, hipStream_t stream) {
    hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(256), 0, stream, ll_part, n_part, out);
    return hipGetLastError();
}

}  // namespace wfsa
