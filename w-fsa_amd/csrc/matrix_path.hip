// Matrix-file mode: the reference's SpMV chain over explicit path matrices
// (matrix_path.hpp).
#include "matrix_path.hpp"

#include <algorithm>
#include <cmath>
#include <map>

namespace wfsa {
namespace {

constexpr int kBlock = 256;

// lw[l] = sum_k pdata[k] x[pcol[k]] over path l's row
__global__ __launch_bounds__(kBlock) void mp_logw_kernel(const int64_t* __restrict__ prow, const int32_t* __restrict__ pcol,
                                                         const double* __restrict__ pdata, const double* __restrict__ x,
                                                         int64_t n_paths, double* __restrict__ lw, const unsigned* halted) {
    if (halted && *halted) return;
    const int64_t l = int64_t(blockIdx.x) * kBlock + threadIdx.x;
    if (l >= n_paths) return;
    double a = 0.0;
    for (int64_t k = prow[l]; k < prow[l + 1]; ++k) a += pdata[k] * x[pcol[k]];
    lw[l] = a;
}

__device__ __forceinline__ void min_pair(double& v, double& i, double v2, double i2) {
    if (v2 < v || (v2 == v && i2 < i)) {
        v = v2;
        i = i2;
    }
}

// string per lane: log q_s, then lw[l] <- -p_s rpp_l; block partials of
// sum p log q (fixed order) and of the smallest rpp of ambiguous strings
__global__ __launch_bounds__(kBlock) void mp_string_kernel(const int64_t* __restrict__ mrow, const int64_t* __restrict__ mcol,
                                                           const double* __restrict__ p, int64_t n_strings,
                                                           double* __restrict__ lw, double* __restrict__ logq,
                                                           double* __restrict__ rpp, double* __restrict__ part,
                                                           const unsigned* halted) {
    if (halted && *halted) return;
    __shared__ double sll[kBlock / 64], sv[kBlock / 64], si[kBlock / 64];
    const int t = int(threadIdx.x);
    const int64_t s = int64_t(blockIdx.x) * kBlock + t;
    double ll = 0.0, rv = INFINITY, ri = -1.0;
    if (s < n_strings) {
        const int64_t a = mrow[s], b = mrow[s + 1];
        double mx = -INFINITY;
        for (int64_t k = a; k < b; ++k) mx = fmax(mx, lw[mcol[k]]);
        double sum = 0.0;
        for (int64_t k = a; k < b; ++k) sum += exp(lw[mcol[k]] - mx);
        const double lq = mx + log(sum);
        const double ps = p[s];
        for (int64_t k = a; k < b; ++k) {
            const int64_t l = mcol[k];
            const double r = exp(lw[l] - lq);
            if (b - a > 1) min_pair(rv, ri, r, double(l));
            lw[l] = -ps * r;
            rpp[l] = r;
        }
        if (logq) logq[s] = lq;
        ll = ps * lq;
    }
    for (int o = 32; o > 0; o >>= 1) {
        ll += __shfl_xor(ll, o, 64);
        min_pair(rv, ri, __shfl_xor(rv, o, 64), __shfl_xor(ri, o, 64));
    }
    if ((t & 63) == 0) {
        sll[t >> 6] = ll;
        sv[t >> 6] = rv;
        si[t >> 6] = ri;
    }
    __syncthreads();
    if (t == 0) {
        for (int k = 1; k < kBlock / 64; ++k) {
            ll += sll[k];
            min_pair(rv, ri, sv[k], si[k]);
        }
        part[3 * blockIdx.x] = ll;
        part[3 * blockIdx.x + 1] = rv;
        part[3 * blockIdx.x + 2] = ri;
    }
}

// parameter per lane over P^T: grad_j = sum_l P_lj (-p_s rpp_l); block 0
// also sums the log-likelihood partials in block order
__global__ __launch_bounds__(kBlock) void mp_grad_kernel(const int64_t* __restrict__ trow, const int64_t* __restrict__ tcol,
                                                         const double* __restrict__ tdata, const double* __restrict__ coef,
                                                         int32_t n_params, const double* __restrict__ part, int n_part,
                                                         double* __restrict__ out, const unsigned* halted) {
    if (halted && *halted) return;
    const int64_t j = int64_t(blockIdx.x) * kBlock + threadIdx.x;
    if (j < n_params) {
        double g = 0.0;
        for (int64_t k = trow[j]; k < trow[j + 1]; ++k) g += tdata[k] * coef[tcol[k]];
        out[1 + j] = g;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        double ll = 0.0;
        for (int k = 0; k < n_part; ++k) ll += part[3 * k];
        out[0] = ll;
    }
}

__global__ __launch_bounds__(64) void mp_rmin_kernel(const double* __restrict__ part, int n_part, double* res,
                                                     const unsigned* halted) {
    if (halted && *halted) return;
    double v = INFINITY, i = -1.0;
    for (int k = int(threadIdx.x); k < n_part; k += 64) min_pair(v, i, part[3 * k + 1], part[3 * k + 2]);
    for (int o = 32; o > 0; o >>= 1) min_pair(v, i, __shfl_xor(v, o, 64), __shfl_xor(i, o, 64));
    if (threadIdx.x == 0) {
        res[0] = i >= 0.0 ? v : 0.0;
        res[1] = i;
    }
}

// H_f slot (string t, equivocal columns a <= b) -> p_s (E[c_a c_b] - E[c_a] E[c_b])
__global__ __launch_bounds__(kBlock) void mp_hf_slot_kernel(const int4* __restrict__ str, const double* __restrict__ tab,
                                                            const int4* __restrict__ slot, int64_t n_slots,
                                                            const int64_t* __restrict__ mcol, const double* __restrict__ rpp,
                                                            const double* __restrict__ p, double* __restrict__ val) {
    const int64_t i = int64_t(blockIdx.x) * kBlock + threadIdx.x;
    if (i >= n_slots) return;
    const int4 sl = slot[i];               // (equivocal string, a, b, string)
    const int4 st = str[sl.x];             // (table offset, paths, equivocal params, first M entry)
    const double* T = tab + st.x;
    double ea = 0.0, eb = 0.0, eab = 0.0;
    for (int l = 0; l < st.y; ++l) {
        const double r = rpp[mcol[st.w + l]];
        const double ca = T[l * st.z + sl.y], cb = T[l * st.z + sl.z];
        ea += ca * r;
        eb += cb * r;
        eab += ca * cb * r;
    }
    val[i] = p[sl.w] * (eab - ea * eb);
}

__global__ __launch_bounds__(kBlock) void mp_hf_sum_kernel(const int64_t* __restrict__ tptr, const int64_t* __restrict__ tslot,
                                                           const double* __restrict__ val, int64_t n_pairs,
                                                           double* __restrict__ out) {
    const int64_t t = int64_t(blockIdx.x) * kBlock + threadIdx.x;
    if (t >= n_pairs) return;
    double v = 0.0;
    for (int64_t k = tptr[t]; k < tptr[t + 1]; ++k) v += val[tslot[k]];
    out[t] = v;
}

template <typename T>
hipError_t upload(T*& dst, const T* src, size_t n, hipStream_t s) {
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&dst), std::max<size_t>(n, 1) * sizeof(T));
    if (e != hipSuccess || n == 0) return e;
    return hipMemcpyAsync(dst, src, n * sizeof(T), hipMemcpyHostToDevice, s);
}

}  // namespace

void MatrixPath::release() {
    for (void* ptr : {static_cast<void*>(prow_), static_cast<void*>(pcol_), static_cast<void*>(pdata_),
                      static_cast<void*>(mrow_), static_cast<void*>(mcol_), static_cast<void*>(p_),
                      static_cast<void*>(trow_), static_cast<void*>(tcol_), static_cast<void*>(tdata_),
                      static_cast<void*>(lw_), static_cast<void*>(part_), static_cast<void*>(rpp_),
                      static_cast<void*>(hf_str_), static_cast<void*>(hf_tab_), static_cast<void*>(hf_slot_),
                      static_cast<void*>(hf_tptr_), static_cast<void*>(hf_tslot_), static_cast<void*>(hf_val_)})
        if (ptr) (void)hipFree(ptr);
    rpp_ = nullptr;
    hf_str_ = nullptr;
    hf_tab_ = nullptr;
    hf_slot_ = nullptr;
    hf_tptr_ = nullptr;
    hf_tslot_ = nullptr;
    hf_val_ = nullptr;
    hf_n_slots_ = hf_n_pairs_ = 0;
    prow_ = nullptr;
    pcol_ = nullptr;
    pdata_ = nullptr;
    mrow_ = nullptr;
    mcol_ = nullptr;
    p_ = nullptr;
    trow_ = nullptr;
    tcol_ = nullptr;
    tdata_ = nullptr;
    lw_ = nullptr;
    part_ = nullptr;
}

MatrixPath::~MatrixPath() { release(); }

hipError_t MatrixPath::load(int32_t n_params, int64_t n_paths, const int64_t* prow, const int32_t* pcol,
                            const double* pdata, int64_t n_strings, const int64_t* mrow, const int64_t* mcol,
                            const double* p, hipStream_t s) {
    release();
    n_params_ = n_params;
    n_paths_ = n_paths;
    n_strings_ = n_strings;
    const int64_t nnz = prow[n_paths];
    // P^T by counting sort on the column (paths ascending within a column)
    std::vector<int64_t> trow(static_cast<size_t>(n_params) + 1, 0), tcol(static_cast<size_t>(nnz));
    std::vector<double> tdata(static_cast<size_t>(nnz));
    for (int64_t k = 0; k < nnz; ++k) trow[size_t(pcol[k]) + 1]++;
    for (int32_t j = 0; j < n_params; ++j) trow[size_t(j) + 1] += trow[size_t(j)];
    std::vector<int64_t> fill(trow.begin(), trow.end() - 1);
    for (int64_t l = 0; l < n_paths; ++l)
        for (int64_t k = prow[l]; k < prow[l + 1]; ++k) {
            const int64_t q = fill[size_t(pcol[k])]++;
            tcol[size_t(q)] = l;
            tdata[size_t(q)] = pdata[k];
        }
    h_counts_.assign(size_t(n_strings), 0.0);
    for (int64_t i = 0; i < n_strings; ++i) h_counts_[size_t(i)] = double(mrow[i + 1] - mrow[i]);
    h_used_.assign(size_t(std::max(n_params, 1)), 0);
    for (int32_t j = 0; j < n_params; ++j) h_used_[size_t(j)] = trow[size_t(j) + 1] > trow[size_t(j)] ? 1 : 0;
    blocks_s_ = int(std::max<int64_t>(1, (n_strings + kBlock - 1) / kBlock));
    hipError_t e;
    if ((e = upload(prow_, prow, size_t(n_paths) + 1, s)) != hipSuccess) return e;
    if ((e = upload(pcol_, pcol, size_t(nnz), s)) != hipSuccess) return e;
    if ((e = upload(pdata_, pdata, size_t(nnz), s)) != hipSuccess) return e;
    if ((e = upload(mrow_, mrow, size_t(n_strings) + 1, s)) != hipSuccess) return e;
    if ((e = upload(mcol_, mcol, size_t(mrow[n_strings]), s)) != hipSuccess) return e;
    if ((e = upload(p_, p, size_t(n_strings), s)) != hipSuccess) return e;
    if ((e = upload(trow_, trow.data(), trow.size(), s)) != hipSuccess) return e;
    if ((e = upload(tcol_, tcol.data(), tcol.size(), s)) != hipSuccess) return e;
    if ((e = upload(tdata_, tdata.data(), tdata.size(), s)) != hipSuccess) return e;
    if ((e = hipMalloc(reinterpret_cast<void**>(&lw_), std::max<size_t>(size_t(n_paths), 1) * sizeof(double))) != hipSuccess)
        return e;
    if ((e = hipMalloc(reinterpret_cast<void**>(&part_), size_t(blocks_s_) * 3 * sizeof(double))) != hipSuccess)
        return e;
    if ((e = hipMalloc(reinterpret_cast<void**>(&rpp_), std::max<size_t>(size_t(n_paths), 1) * sizeof(double))) != hipSuccess)
        return e;
    h_prow_.assign(prow, prow + n_paths + 1);
    h_pcol_.assign(pcol, pcol + nnz);
    h_pdata_.assign(pdata, pdata + nnz);
    h_mrow_.assign(mrow, mrow + n_strings + 1);
    h_mcol_.assign(mcol, mcol + mrow[n_strings]);
    return hipStreamSynchronize(s);   // the host vectors above are freed on return
}

hipError_t MatrixPath::enqueue(const double* w, double* out, double* logq, const unsigned* halted, hipStream_t s) {
    const unsigned gp = unsigned(std::max<int64_t>(1, (n_paths_ + kBlock - 1) / kBlock));
    hipLaunchKernelGGL(mp_logw_kernel, dim3(gp), dim3(kBlock), 0, s, prow_, pcol_, pdata_, w, n_paths_, lw_, halted);
    hipLaunchKernelGGL(mp_string_kernel, dim3(unsigned(blocks_s_)), dim3(kBlock), 0, s, mrow_, mcol_, p_, n_strings_,
                       lw_, logq, rpp_, part_, halted);
    const unsigned gj = unsigned(std::max<int64_t>(1, (int64_t(n_params_) + kBlock - 1) / kBlock));
    hipLaunchKernelGGL(mp_grad_kernel, dim3(gj), dim3(kBlock), 0, s, trow_, tcol_, tdata_, lw_, n_params_, part_,
                       blocks_s_, out, halted);
    return hipGetLastError();
}

hipError_t MatrixPath::hf_setup(std::vector<int32_t>& pairs, hipStream_t s) {
    std::vector<int4> strs, slots;
    std::vector<double> tab;
    std::vector<int64_t> keys;
    const int64_t np = std::max<int64_t>(n_params_, 1);
    for (int64_t i = 0; i < n_strings_; ++i) {
        const int64_t a = h_mrow_[size_t(i)], b = h_mrow_[size_t(i) + 1];
        if (b - a < 2) continue;
        // parameters whose count is not the same on every path (AssembleH's
        // union minus the intersection of (column, count))
        std::map<int32_t, std::vector<double>> cnt;
        for (int64_t k = a; k < b; ++k) {
            const int64_t l = h_mcol_[size_t(k)];
            for (int64_t q = h_prow_[size_t(l)]; q < h_prow_[size_t(l) + 1]; ++q) {
                auto& v = cnt[h_pcol_[size_t(q)]];
                v.resize(size_t(b - a), 0.0);
                v[size_t(k - a)] += h_pdata_[size_t(q)];
            }
        }
        std::vector<int32_t> eq;
        for (auto& kv : cnt)
            if (std::any_of(kv.second.begin(), kv.second.end(), [&](double c) { return c != kv.second[0]; }))
                eq.push_back(kv.first);
        if (eq.empty()) continue;
        const int32_t ne = int32_t(eq.size()), sid = int32_t(strs.size());
        strs.push_back(make_int4(int32_t(tab.size()), int32_t(b - a), ne, int32_t(a)));
        for (int64_t l = 0; l < b - a; ++l)
            for (int32_t e = 0; e < ne; ++e) tab.push_back(cnt[eq[size_t(e)]][size_t(l)]);
        for (int32_t x = 0; x < ne; ++x)
            for (int32_t y = x; y < ne; ++y) {
                slots.push_back(make_int4(sid, x, y, int32_t(i)));
                keys.push_back(int64_t(eq[size_t(x)]) * np + eq[size_t(y)]);
            }
    }
    if (tab.size() >= (size_t(1) << 31)) return hipErrorOutOfMemory;
    const int64_t ns = int64_t(slots.size());
    std::vector<int64_t> order(static_cast<size_t>(ns));
    for (int64_t i = 0; i < ns; ++i) order[size_t(i)] = i;
    std::stable_sort(order.begin(), order.end(), [&](int64_t x, int64_t y) { return keys[size_t(x)] < keys[size_t(y)]; });
    std::vector<int64_t> tptr(1, 0);
    pairs.clear();
    for (int64_t i = 0; i < ns; ++i) {
        const int64_t key = keys[size_t(order[size_t(i)])];
        if (i == 0 || key != keys[size_t(order[size_t(i) - 1])]) {
            if (i > 0) tptr.push_back(i);
            pairs.push_back(int32_t(key / np));
            pairs.push_back(int32_t(key % np));
        }
    }
    if (ns > 0) tptr.push_back(ns);
    for (void* ptr : {static_cast<void*>(hf_str_), static_cast<void*>(hf_tab_), static_cast<void*>(hf_slot_),
                      static_cast<void*>(hf_tptr_), static_cast<void*>(hf_tslot_), static_cast<void*>(hf_val_)})
        if (ptr) (void)hipFree(ptr);
    hipError_t e;
    if ((e = upload(hf_str_, strs.data(), strs.size(), s)) != hipSuccess) return e;
    if ((e = upload(hf_tab_, tab.data(), tab.size(), s)) != hipSuccess) return e;
    if ((e = upload(hf_slot_, slots.data(), slots.size(), s)) != hipSuccess) return e;
    if ((e = upload(hf_tptr_, tptr.data(), tptr.size(), s)) != hipSuccess) return e;
    if ((e = upload(hf_tslot_, order.data(), order.size(), s)) != hipSuccess) return e;
    if ((e = hipMalloc(reinterpret_cast<void**>(&hf_val_), std::max<size_t>(size_t(ns), 1) * sizeof(double))) != hipSuccess)
        return e;
    hf_n_slots_ = ns;
    hf_n_pairs_ = int64_t(pairs.size() / 2);
    return hipStreamSynchronize(s);
}

hipError_t MatrixPath::hf_eval(const double* w, double* out, hipStream_t s) {
    // the evaluation leaves the relative path probabilities in rpp_ (and
    // overwrites nothing the caller reads: out is the context's H_f buffer)
    const unsigned gp = unsigned(std::max<int64_t>(1, (n_paths_ + kBlock - 1) / kBlock));
    hipLaunchKernelGGL(mp_logw_kernel, dim3(gp), dim3(kBlock), 0, s, prow_, pcol_, pdata_, w, n_paths_, lw_, nullptr);
    hipLaunchKernelGGL(mp_string_kernel, dim3(unsigned(blocks_s_)), dim3(kBlock), 0, s, mrow_, mcol_, p_, n_strings_,
                       lw_, nullptr, rpp_, part_, nullptr);
    if (hf_n_slots_ > 0) {
        hipLaunchKernelGGL(mp_hf_slot_kernel, dim3(unsigned((hf_n_slots_ + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                           hf_str_, hf_tab_, hf_slot_, hf_n_slots_, mcol_, rpp_, p_, hf_val_);
        hipLaunchKernelGGL(mp_hf_sum_kernel, dim3(unsigned((hf_n_pairs_ + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                           hf_tptr_, hf_tslot_, hf_val_, hf_n_pairs_, out);
    }
    return hipGetLastError();
}

hipError_t MatrixPath::enqueue_rmin(double* res, const unsigned* halted, hipStream_t s) {
    hipLaunchKernelGGL(mp_rmin_kernel, dim3(1), dim3(64), 0, s, part_, blocks_s_, res, halted);
    return hipGetLastError();
}

}  // namespace wfsa
