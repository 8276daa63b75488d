// Stream-format micro v4: the trivial-word pass of fbs_kernel in isolation
// (c3-like: 1M strings of 30-42 edges on 1024 nodes x 9 out-slots, 9,216
// weights staged in LDS), one wave per run of 64-string groups, 16-byte rows
// of every lane contiguous per wave instruction, two register sets of D rows.
// What it separates:
//   * the LDS gathers' bank conflicts: words of every string in stream order
//     ("rand") against the same words reordered at compile time so that at
//     each row position the 32 lanes of a half-wave read distinct banks
//     ("sched": a bipartite matching of lanes to the 32 bank classes of
//     j mod 32 -- a string's sum does not depend on its word order);
//   * the stream's bytes: 16-bit words (8 per row) against 14-bit words
//     (9 per row);
//   * the stream loads alone ("loads") at D = 4 and 8 rows per set.
// Rows carry words only; p and the group row counts are separate arrays.
// Prints the event-timed kernel time per launch and the log-likelihood
// against the host's.  Run under rocprofv3 --pmc for the LDS counters.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <functional>
#include <numeric>
#include <random>
#include <thread>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int kWave = 64;
constexpr int kNodes = 1024, kDeg = 9, kSlots = kNodes * kDeg;   // zero weight at kSlots
constexpr int kMinLen = 30, kMaxLen = 42;

__device__ inline double wave_sum(double v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// FMT 16: words at bits 16i (i < 8); FMT 14: at bits 14i (i < 9)
template <int FMT>
__device__ __forceinline__ void words(const uint4 v, uint32_t (&o)[FMT == 16 ? 8 : 9]) {
    if constexpr (FMT == 16) {
        const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            o[2 * i] = d[i] & 0xffffu;
            o[2 * i + 1] = d[i] >> 16;
        }
    } else {
        constexpr uint32_t M = 0x3fffu;
        o[0] = v.x & M;
        o[1] = (v.x >> 14) & M;
        o[2] = __builtin_amdgcn_alignbit(v.y, v.x, 28) & M;
        o[3] = (v.y >> 10) & M;
        o[4] = __builtin_amdgcn_alignbit(v.z, v.y, 24) & M;
        o[5] = (v.z >> 6) & M;
        o[6] = __builtin_amdgcn_alignbit(v.w, v.z, 20) & M;
        o[7] = (v.w >> 2) & M;
        o[8] = (v.w >> 16) & M;
    }
}

// delta formats (FMT = 100 + b): 128 / b fields of b bits per row, each a
// step forward from the lane's previous index (the string's words sorted,
// remapped to leave a zero slot every 2^(b-1) entries, long gaps bridged by
// steps to zero slots); every field gathers the weight at its index
template <int B>
__device__ __forceinline__ void fields(const uint4 v, uint32_t (&o)[128 / B]) {
    const uint32_t d[4] = {v.x, v.y, v.z, v.w};
    constexpr uint32_t M = (1u << B) - 1u;
#pragma unroll
    for (int i = 0; i < 128 / B; ++i) {
        const int b0 = i * B, w0 = b0 / 32, sh = b0 % 32;
        if (sh + B <= 32) o[i] = (d[w0] >> sh) & M;
        else o[i] = __builtin_amdgcn_alignbit(d[w0 + 1], d[w0], sh) & M;
    }
}

// MODE 0: gathers; 1: stream loads only
template <int FMT, int D, int MODE, int OCC>
__global__ __launch_bounds__(1024, OCC) void pass(const uint4* __restrict__ st, const int* __restrict__ wave_row0,
                                                   const int* __restrict__ wave_g0, const int* __restrict__ grp_rows,
                                                   const double* __restrict__ w, const double* __restrict__ p,
                                                   double* ll_part) {
    constexpr bool DEL = FMT > 100;
    constexpr int DB = DEL ? FMT - 100 : 16;
    constexpr int PER = DEL ? (1 << (DB - 1)) : 1 << 30;   // zero-slot period
    constexpr int TSZ = DEL ? kSlots + kSlots / (PER - 1) + PER : kSlots + 2;
    __shared__ double lw[TSZ];
    if (DEL) {
        for (int j = threadIdx.x; j < TSZ; j += blockDim.x) {
            const int src = j - j / PER;   // remapped slot j holds weight src unless a zero slot
            lw[j] = ((j % PER) == PER - 1 || src >= kSlots) ? 0.0 : w[src];
        }
    } else {
        for (int j = threadIdx.x; j < kSlots + 1; j += blockDim.x) lw[j] = w[j];
    }
    __syncthreads();
    constexpr int NW = DEL ? 128 / DB : (FMT == 16 ? 8 : 9);
    const int lane = threadIdx.x % kWave;
    const int gw = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave);
    const int r0 = wave_row0[gw], rows = wave_row0[gw + 1] - r0;
    int g = wave_g0[gw];
    int bound = rows > 0 ? grp_rows[g] : 1 << 30;
    const uint4* s = st + int64_t(r0) * kWave + lane;
    const int last = max(rows - 1, 0);
    uint4 A[D], B[D];
    auto load = [&](uint4 (&r)[D], int c0) {
#pragma unroll
        for (int d = 0; d < D; ++d) r[d] = s[int64_t(kWave) * min(c0 + d, last)];
    };
    double ll = 0.0, acc0 = 0.0, acc1 = 0.0;
    uint32_t cur = 0;
    auto apply = [&](const uint4 (&r)[D], int c0) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int c = c0 + d;
            if (c >= rows) break;
            if (c == bound) {
                ll += p[int64_t(g) * kWave + lane] * (acc0 + acc1);
                acc0 = acc1 = 0.0;
                cur = 0;
                ++g;
                bound += grp_rows[g];
            }
            if (MODE == 1) {
                acc0 += double(r[d].x ^ r[d].y ^ r[d].z ^ r[d].w);
                continue;
            }
            uint32_t o[NW];
            if constexpr (DEL) {
                fields<DB>(r[d], o);
#pragma unroll
                for (int i = 0; i < NW; ++i) {
                    cur += o[i];
                    const double t = lw[min(cur, uint32_t(TSZ - 1))];
                    if (i & 1) acc1 += t; else acc0 += t;
                }
            } else {
                words<FMT>(r[d], o);
#pragma unroll
                for (int i = 0; i < NW; ++i) {
                    const double t = lw[min(o[i], uint32_t(kSlots))];
                    if (i & 1) acc1 += t; else acc0 += t;
                }
            }
        }
    };
    if (rows > 0) {
        load(A, 0);
        load(B, D);
        for (int c0 = 0;;) {
            apply(A, c0);
            if (c0 + D >= rows) break;
            load(A, c0 + 2 * D);
            apply(B, c0 + D);
            c0 += 2 * D;
            if (c0 >= rows) break;
            load(B, c0 + D);
        }
        ll += p[int64_t(g) * kWave + lane] * (acc0 + acc1);
    }
    ll = wave_sum(ll);
    if (lane == 0) ll_part[gw] = ll;
}

// ---------------------------------------------------------------- host side
struct Layout {
    std::vector<uint32_t> rows;   // uint4 rows as 4 x u32
    std::vector<int> wave_row0, wave_g0, grp_rows;
    double bytes = 0;
};

// order[g][lane] = the lane's words in stream order
static Layout build(const std::vector<std::vector<std::vector<uint16_t>>>& order, const std::vector<int>& wave_groups_ptr,
                    int fmt) {
    const int per_row = fmt > 100 ? 128 / (fmt - 100) : fmt == 16 ? 8 : 9;
    const int pad = fmt > 100 ? 0 : fmt == 16 ? 0xffff : 0x3fff;
    const int fb = fmt > 100 ? fmt - 100 : fmt;
    Layout L;
    const int G = int(order.size());
    const int nwaves = int(wave_groups_ptr.size()) - 1;
    L.grp_rows.resize(size_t(G) + 1, 0);
    L.wave_row0.resize(size_t(nwaves) + 1);
    L.wave_g0.resize(size_t(nwaves) + 1);
    int64_t total_rows = 0;
    for (int g = 0; g < G; ++g) {
        size_t mx = 0;
        for (const auto& v : order[g]) mx = std::max(mx, v.size());
        L.grp_rows[g] = int((mx + per_row - 1) / per_row);
        total_rows += L.grp_rows[g];
    }
    L.rows.assign(size_t(total_rows) * kWave * 4, 0);
    int64_t r = 0;
    for (int wv = 0; wv < nwaves; ++wv) {
        L.wave_row0[wv] = int(r);
        L.wave_g0[wv] = wave_groups_ptr[wv];
        for (int g = wave_groups_ptr[wv]; g < wave_groups_ptr[wv + 1]; ++g) {
            for (int l = 0; l < kWave; ++l) {
                const auto& v = order[g][l];
                for (int c = 0; c < L.grp_rows[g]; ++c) {
                    uint32_t* d = &L.rows[((size_t(r + c)) * kWave + l) * 4];
                    for (int i = 0; i < per_row; ++i) {
                        const size_t k = size_t(c) * per_row + i;
                        const uint32_t x = k < v.size() ? v[k] : uint32_t(pad);
                        if (fmt == 16) {
                            d[i / 2] |= x << (16 * (i % 2));
                        } else {
                            const int b = fb * i, wd = b / 32, sh = b % 32;
                            d[wd] |= x << sh;
                            if (sh + fb > 32) d[wd + 1] |= x >> (32 - sh);
                        }
                    }
                }
            }
            r += L.grp_rows[g];
        }
    }
    L.wave_row0[nwaves] = int(r);
    L.wave_g0[nwaves] = G;
    L.bytes = double(L.rows.size()) * 4;
    return L;
}

// the delta encoding of one string's words as b-bit fields (see fields<>)
static std::vector<uint16_t> delta_fields(std::vector<uint16_t> w, int b) {
    const uint32_t M = (1u << b) - 1u, P = 1u << (b - 1);
    std::vector<uint32_t> r;
    for (uint16_t j : w) r.push_back(uint32_t(j) + uint32_t(j) / (P - 1));
    std::sort(r.begin(), r.end());
    std::vector<uint16_t> f;
    uint32_t cur = 0;
    for (uint32_t t : r) {
        while (t - cur > M) {   // to the farthest zero slot within reach
            const uint32_t z = ((cur + M + 1) / P) * P - 1;
            f.push_back(uint16_t(z - cur));
            cur = z;
        }
        f.push_back(uint16_t(t - cur));
        cur = t;
    }
    const uint32_t z = (cur / P) * P + P - 1;   // the end: onto a zero slot (the pads then add 0)
    if (z != cur) f.push_back(uint16_t(z - cur));
    return f;
}

// reorder every string of a group so that at each position the lanes of a
// half-wave read distinct classes j mod 32 where a matching allows
static void schedule_group(std::vector<std::vector<uint16_t>>& lanes, int64_t& conflicts_before, int64_t& conflicts_after) {
    auto count_conf = [&](const std::vector<std::vector<uint16_t>>& L) {
        int64_t c = 0;
        size_t mx = 0;
        for (const auto& v : L) mx = std::max(mx, v.size());
        for (int h = 0; h < 2; ++h)
            for (size_t t = 0; t < mx; ++t) {
                int cnt[32] = {0};
                bool padseen = false;
                for (int l = 32 * h; l < 32 * h + 32; ++l) {
                    if (t < L[l].size()) ++cnt[L[l][t] % 32];
                    else padseen = true;
                }
                if (padseen) ++cnt[kSlots % 32];
                int m = 0;
                for (int k = 0; k < 32; ++k) m = std::max(m, cnt[k]);
                c += m - 1;   // extra cycles of this half's gather
            }
        return c;
    };
    conflicts_before += count_conf(lanes);
    for (int h = 0; h < 2; ++h) {
        std::vector<std::vector<uint16_t>> rem(32);
        size_t mx = 0;
        for (int l = 0; l < 32; ++l) {
            rem[l] = lanes[32 * h + l];
            mx = std::max(mx, rem[l].size());
        }
        std::vector<std::vector<uint16_t>> out(32);
        for (size_t t = 0; t < mx; ++t) {
            uint32_t mask[32];
            for (int l = 0; l < 32; ++l) {
                mask[l] = 0;
                for (uint16_t j : rem[l]) mask[l] |= 1u << (j % 32);
            }
            int owner[32];   // class -> lane
            std::fill(owner, owner + 32, -1);
            bool padseen = false;
            for (int l = 0; l < 32; ++l) padseen |= rem[l].empty();
            if (padseen) owner[kSlots % 32] = 99;   // the pad's bank is taken
            int match[32];
            std::fill(match, match + 32, -1);
            // lanes with the most words left first (they must not fall behind)
            int ord[32];
            std::iota(ord, ord + 32, 0);
            std::sort(ord, ord + 32, [&](int a, int b) { return rem[a].size() > rem[b].size(); });
            std::function<bool(int, uint32_t&)> aug = [&](int l, uint32_t& seen) -> bool {
                uint32_t m = mask[l] & ~seen;
                while (m) {
                    const int c = __builtin_ctz(m);
                    m &= m - 1;
                    seen |= 1u << c;
                    if (owner[c] == -1 || (owner[c] != 99 && aug(owner[c], seen))) {
                        owner[c] = l;
                        match[l] = c;
                        return true;
                    }
                }
                return false;
            };
            for (int oi = 0; oi < 32; ++oi) {
                const int l = ord[oi];
                if (rem[l].empty()) continue;
                uint32_t seen = 0;
                aug(l, seen);
            }
            int load[32] = {0};
            for (int c = 0; c < 32; ++c) load[c] = owner[c] >= 0 ? 1 : 0;
            for (int l = 0; l < 32; ++l) {
                if (rem[l].empty()) continue;
                int pick = -1;
                if (match[l] >= 0) {
                    for (size_t i = 0; i < rem[l].size(); ++i)
                        if (int(rem[l][i] % 32) == match[l]) { pick = int(i); break; }
                } else {   // the least loaded class it has
                    int best = 1 << 30;
                    for (size_t i = 0; i < rem[l].size(); ++i)
                        if (load[rem[l][i] % 32] < best) { best = load[rem[l][i] % 32]; pick = int(i); }
                    ++load[rem[l][size_t(pick)] % 32];
                }
                out[l].push_back(rem[l][size_t(pick)]);
                rem[l].erase(rem[l].begin() + pick);
            }
        }
        for (int l = 0; l < 32; ++l) lanes[32 * h + l] = out[l];
    }
    conflicts_after += count_conf(lanes);
}

int main() {
    const int S = 1 << 20, G = S / kWave;
    std::mt19937_64 rng(11);
    std::vector<double> sw(kSlots + 1);
    std::vector<int> succ(kSlots);
    for (int j = 0; j < kSlots; ++j) {
        succ[j] = int(rng() % kNodes);
        sw[j] = -1.0 - double(rng() % 1000) * 1e-3;
    }
    sw[kSlots] = 0.0;
    // strings: a walk from node 0, lengths 30..42; sorted longest first into groups
    std::vector<std::vector<uint16_t>> str(S);
    std::vector<double> p(S);
    for (int s = 0; s < S; ++s) {
        const int L = kMinLen + int(rng() % (kMaxLen - kMinLen + 1));
        int u = 0;
        for (int e = 0; e < L; ++e) {
            const int j = u * kDeg + int(rng() % kDeg);
            str[s].push_back(uint16_t(j));
            u = succ[j];
        }
        p[s] = (1.0 + double(rng() % 100)) / (50.5 * S);
    }
    std::vector<int> ordr(S);
    std::iota(ordr.begin(), ordr.end(), 0);
    std::stable_sort(ordr.begin(), ordr.end(), [&](int a, int b) { return str[a].size() > str[b].size(); });
    // groups dealt to waves in snake order, then laid out wave-contiguous
    // STREAM_WAVES=8192: the layout for two 1024-thread blocks per CU (32 waves)
    const int nwaves = std::getenv("STREAM_WAVES") ? std::atoi(std::getenv("STREAM_WAVES")) : 256 * 16;
    std::vector<std::vector<int>> wg(nwaves);
    for (int g = 0; g < G; ++g) {
        const int round = g / nwaves, k = g % nwaves;
        wg[(round % 2) ? nwaves - 1 - k : k].push_back(g);
    }
    std::vector<int> gperm, wptr(1, 0);
    for (int wv = 0; wv < nwaves; ++wv) {
        for (int g : wg[wv]) gperm.push_back(g);
        wptr.push_back(int(gperm.size()));
    }
    std::vector<std::vector<std::vector<uint16_t>>> order(G, std::vector<std::vector<uint16_t>>(kWave));
    std::vector<double> pg(size_t(G) * kWave);
    double ref = 0.0;
    for (int gi = 0; gi < G; ++gi) {
        const int g = gperm[gi];
        for (int l = 0; l < kWave; ++l) {
            const int s = ordr[size_t(g) * kWave + l];
            order[gi][l] = str[s];
            pg[size_t(gi) * kWave + l] = p[s];
            double a = 0.0;
            for (uint16_t j : str[s]) a += sw[j];
            ref += p[s] * a;
        }
    }
    auto sched = order;
    {
        const int nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        std::vector<int64_t> cb(nt, 0), ca(nt, 0);
        std::vector<std::thread> th;
        for (int t = 0; t < nt; ++t)
            th.emplace_back([&, t] {
                for (int g = t; g < G; g += nt) schedule_group(sched[g], cb[t], ca[t]);
            });
        for (auto& x : th) x.join();
        const int64_t b = std::accumulate(cb.begin(), cb.end(), int64_t(0)), a = std::accumulate(ca.begin(), ca.end(), int64_t(0));
        int64_t gathers = 0;
        for (int g = 0; g < G; ++g) {
            size_t mx = 0;
            for (const auto& v : order[g]) mx = std::max(mx, v.size());
            gathers += int64_t(mx) * 2;
        }
        printf("half-wave gathers %lld: extra conflict cycles in stream order %lld (%.2f per gather), scheduled %lld (%.3f)\n",
               (long long)gathers, (long long)b, double(b) / gathers, (long long)a, double(a) / gathers);
    }
    Layout l16r = build(order, wptr, 16), l16s = build(sched, wptr, 16);
    Layout l14r = build(order, wptr, 14), l14s = build(sched, wptr, 14);
    Layout ld[3];
    const int dbits[3] = {8, 9, 10};
    for (int q = 0; q < 3; ++q) {
        auto enc = order;
        int64_t nf = 0;
        for (auto& grp : enc)
            for (auto& v : grp) {
                v = delta_fields(v, dbits[q]);
                nf += int64_t(v.size());
            }
        ld[q] = build(enc, wptr, 100 + dbits[q]);
        printf("delta %d-bit: %.3f fields per word, stream %.1f MB\n", dbits[q], double(nf) / 37748736.0 * 1.0, ld[q].bytes / 1e6);
    }
    double *dw, *dp, *dll;
    CK(hipMalloc(&dw, (kSlots + 2) * 8));
    CK(hipMalloc(&dp, pg.size() * 8));
    CK(hipMalloc(&dll, size_t(nwaves) * 8 * 4));
    CK(hipMemcpy(dw, sw.data(), (kSlots + 1) * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dp, pg.data(), pg.size() * 8, hipMemcpyHostToDevice));
    struct Dev { uint4* st; int *wr, *wg, *gr; double bytes; };
    auto up = [&](const Layout& L, Dev& d) -> int {
        CK(hipMalloc(&d.st, L.rows.size() * 4));
        CK(hipMalloc(&d.wr, L.wave_row0.size() * 4));
        CK(hipMalloc(&d.wg, L.wave_g0.size() * 4));
        CK(hipMalloc(&d.gr, L.grp_rows.size() * 4));
        CK(hipMemcpy(d.st, L.rows.data(), L.rows.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(d.wr, L.wave_row0.data(), L.wave_row0.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(d.wg, L.wave_g0.data(), L.wave_g0.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(d.gr, L.grp_rows.data(), L.grp_rows.size() * 4, hipMemcpyHostToDevice));
        d.bytes = L.bytes;
        return 0;
    };
    Dev d16r, d16s, d14r, d14s, dd[3];
    if (up(l16r, d16r) || up(l16s, d16s) || up(l14r, d14r) || up(l14s, d14s)) return 1;
    for (int q = 0; q < 3; ++q)
        if (up(ld[q], dd[q])) return 1;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto kern, const Dev& d, int blocks, bool check) -> int {
        auto launch = [&] { hipLaunchKernelGGL(kern, dim3(blocks), dim3(1024), 0, 0, d.st, d.wr, d.wg, d.gr, dw, dp, dll); };
        for (int r = 0; r < 3; ++r) launch();
        CK(hipDeviceSynchronize());
        const int reps = 50;
        CK(hipEventRecord(e0, 0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::vector<double> part(nwaves);
        CK(hipMemcpy(part.data(), dll, size_t(nwaves) * 8, hipMemcpyDeviceToHost));
        double ll = 0.0;
        for (double v : part) ll += v;
        const double us = ms * 1e3 / reps, bytes = d.bytes + double(S) * 8;
        printf("%-30s %8.2f us  stream+p %6.1f MB  %7.1f GB/s", name, us, bytes / 1e6, bytes / us / 1e3);
        if (check) printf("  ll %.15g (ref %.15g, rel %.1e)", ll, ref, std::abs(ll - ref) / std::abs(ref));
        printf("\n");
        return 0;
    };
    const int b1 = nwaves / 16;   // 1024-thread blocks: 256 (one per CU, 16 waves) or 512 (two per CU)
    if (nwaves == 8192) {   // the 32-waves-per-CU form of the delta pass (64 VGPRs)
        if (run("delta 10-bit D2 gather occ2", pass<110, 2, 0, 2>, dd[2], b1, true)) return 1;
        if (run("delta 10-bit D3 gather occ2", pass<110, 3, 0, 2>, dd[2], b1, true)) return 1;
        if (run("delta 10-bit D2 loads occ2", pass<110, 2, 1, 2>, dd[2], b1, false)) return 1;
        return 0;
    }
    if (run("16-bit rand  D4 gather", pass<16, 4, 0, 1>, d16r, b1, true)) return 1;
    if (run("16-bit sched D4 gather", pass<16, 4, 0, 1>, d16s, b1, true)) return 1;
    if (run("14-bit rand  D4 gather", pass<14, 4, 0, 1>, d14r, b1, true)) return 1;
    if (run("14-bit sched D4 gather", pass<14, 4, 0, 1>, d14s, b1, true)) return 1;
    if (run("16-bit sched D2 gather", pass<16, 2, 0, 1>, d16s, b1, true)) return 1;
    if (run("14-bit sched D2 gather", pass<14, 2, 0, 1>, d14s, b1, true)) return 1;
    if (run("14-bit sched D3 gather", pass<14, 3, 0, 1>, d14s, b1, true)) return 1;
    if (run("delta 8-bit D2 gather", pass<108, 2, 0, 1>, dd[0], b1, true)) return 1;
    if (run("delta 9-bit D2 gather", pass<109, 2, 0, 1>, dd[1], b1, true)) return 1;
    if (run("delta 10-bit D2 gather", pass<110, 2, 0, 1>, dd[2], b1, true)) return 1;
    if (run("delta 10-bit D3 gather", pass<110, 3, 0, 1>, dd[2], b1, true)) return 1;
    if (run("delta 9-bit D3 gather", pass<109, 3, 0, 1>, dd[1], b1, true)) return 1;
    if (run("delta 10-bit D2 loads", pass<110, 2, 1, 1>, dd[2], b1, false)) return 1;
    if (run("16-bit loads D4", pass<16, 4, 1, 1>, d16r, b1, false)) return 1;
    if (run("16-bit loads D2", pass<16, 2, 1, 1>, d16r, b1, false)) return 1;
    if (run("16-bit loads D8", pass<16, 8, 1, 1>, d16r, b1, false)) return 1;
    if (run("14-bit loads D4", pass<14, 4, 1, 1>, d14r, b1, false)) return 1;
    if (run("14-bit loads D2", pass<14, 2, 1, 1>, d14r, b1, false)) return 1;
    return 0;
}
