#include "trellis_model.hpp"

#include <algorithm>
#include <numeric>
#include <string>

namespace wfsa {

namespace {

constexpr int64_t kMaxCompositeEdges = int64_t(1) << 28;
constexpr int kMaxEpsilonDepth = 100000;

struct RawEdge {
    uint8_t byte;
    int32_t dst;
    int32_t pbeg, pend;  // into scratch param pool
};

}  // namespace

std::string compile_trellis_model(const wfsa_model_desc& d, TrellisModel& out) {
    const int32_t N = d.n_states;
    if (N <= 0 || !d.em_ptr || !d.tr_ptr) return "empty automaton description";
    if (d.start < 0 || d.start >= N) return "start state out of range";
    if (d.end >= N) return "end state out of range";
    const int32_t n_em = d.em_ptr[N], n_tr = d.tr_ptr[N];
    for (int32_t s = 0; s < N; ++s) {
        if (d.em_ptr[s] > d.em_ptr[s + 1] || d.tr_ptr[s] > d.tr_ptr[s + 1]) return "non-monotone CSR pointers";
    }
    for (int32_t e = 0; e < n_em; ++e) {
        if (d.em_len[e] < 0) return "negative emission length";
        if (d.em_param[e] < -1 || d.em_param[e] >= d.n_params) return "emission parameter out of range";
    }
    for (int32_t t = 0; t < n_tr; ++t) {
        if (d.tr_dst[t] < 0 || d.tr_dst[t] >= N) return "transition target out of range";
        if (d.tr_param[t] < -1 || d.tr_param[t] >= d.n_params) return "transition parameter out of range";
    }

    // chain nodes for multi-byte emissions: emission e of state U with |e|=m
    // gets nodes chain_base[e] .. chain_base[e]+m-2
    std::vector<int32_t> chain_base(size_t(n_em), -1);
    int64_t n_nodes = N;
    for (int32_t e = 0; e < n_em; ++e) {
        if (d.em_len[e] >= 2) {
            chain_base[e] = int32_t(n_nodes);
            n_nodes += d.em_len[e] - 1;
        }
    }
    if (n_nodes >= (int64_t(1) << 31) - 1) return "too many trellis nodes";
    std::vector<int32_t> em_owner(static_cast<size_t>(n_em));
    for (int32_t s = 0; s < N; ++s)
        for (int32_t e = d.em_ptr[s]; e < d.em_ptr[s + 1]; ++e) em_owner[e] = s;

    std::vector<std::vector<RawEdge>> edges(static_cast<size_t>(n_nodes));
    std::vector<std::vector<std::pair<int32_t, int32_t>>> ends(static_cast<size_t>(n_nodes));
    std::vector<int32_t> pool;      // parameter lists
    int64_t n_composite = 0;

    // epsilon-removal DFS from every state S
    std::vector<char> on_path(size_t(N), 0);
    std::vector<int32_t> cur;   // parameter list along the current epsilon path
    std::string err;

    auto push_list = [&](int32_t extra1, int32_t extra2, int32_t& b, int32_t& e) {
        b = int32_t(pool.size());
        pool.insert(pool.end(), cur.begin(), cur.end());
        if (extra1 >= 0) pool.push_back(extra1);
        if (extra2 >= 0) pool.push_back(extra2);
        e = int32_t(pool.size());
    };

    // explicit-stack DFS to survive long epsilon chains
    struct Frame { int32_t state; int32_t t; int32_t e; size_t cur_len; };
    for (int32_t S = 0; S < N && err.empty(); ++S) {
        std::vector<Frame> stack;
        stack.push_back({S, d.tr_ptr[S], -1, 0});
        on_path[S] = 1;
        while (!stack.empty() && err.empty()) {
            Frame& fr = stack.back();
            const int32_t X = fr.state;
            if (fr.t >= d.tr_ptr[X + 1]) {
                on_path[X] = 0;
                cur.resize(fr.cur_len);
                stack.pop_back();
                continue;
            }
            const int32_t T = d.tr_dst[fr.t];
            const int32_t tp = d.tr_param[fr.t];
            if (T == d.end) {
                int32_t b, e;
                push_list(tp, -1, b, e);
                ends[S].push_back({b, e});
                if (++n_composite > kMaxCompositeEdges) err = "too many composite edges";
                ++fr.t;
                continue;
            }
            // iterate emissions of T
            if (fr.e < 0) fr.e = d.em_ptr[T];
            if (fr.e >= d.em_ptr[T + 1]) { fr.e = -1; ++fr.t; continue; }
            const int32_t e = fr.e++;
            const int32_t ep = d.em_param[e];
            const int32_t len = d.em_len[e];
            if (len == 0) {
                if (on_path[T]) { err = "epsilon cycle through state " + std::to_string(T); break; }
                if (int(stack.size()) >= kMaxEpsilonDepth) { err = "epsilon chain too deep"; break; }
                const size_t saved = cur.size();
                if (tp >= 0) cur.push_back(tp);
                if (ep >= 0) cur.push_back(ep);
                on_path[T] = 1;
                stack.push_back({T, d.tr_ptr[T], -1, saved});
                continue;
            }
            int32_t b, en;
            push_list(tp, ep, b, en);
            const uint8_t first = d.em_bytes[d.em_off[e]];
            const int32_t dst = (len == 1) ? T : chain_base[e];
            edges[S].push_back({first, dst, b, en});
            if (++n_composite > kMaxCompositeEdges) err = "too many composite edges";
        }
        if (!err.empty()) break;
    }
    if (!err.empty()) return err;

    // chain edges
    for (int32_t e = 0; e < n_em; ++e) {
        if (chain_base[e] < 0) continue;
        const int32_t len = d.em_len[e];
        const uint8_t* bytes = d.em_bytes + d.em_off[e];
        for (int32_t k = 1; k < len; ++k) {
            const int32_t node = chain_base[e] + k - 1;
            const int32_t dst = (k + 1 < len) ? node + 1 : em_owner[e];
            const int32_t b = int32_t(pool.size());
            edges[node].push_back({bytes[k], dst, b, b});
        }
    }

    out = TrellisModel();
    out.n_params = d.n_params;
    out.n_nodes = int32_t(n_nodes);
    out.start = d.start;
    out.o_ptr.assign(size_t(n_nodes) + 1, 0);
    out.x_ptr.assign(size_t(n_nodes) + 1, 0);
    out.node_end_count.assign(size_t(n_nodes), 0.0);
    out.o_pptr.push_back(0);
    out.x_pptr.push_back(0);
    for (int64_t u = 0; u < n_nodes; ++u) {
        auto& ev = edges[size_t(u)];
        std::stable_sort(ev.begin(), ev.end(), [](const RawEdge& a, const RawEdge& b) { return a.byte < b.byte; });
        for (const auto& re : ev) {
            out.o_byte.push_back(re.byte);
            out.o_dst.push_back(re.dst);
            out.o_pidx.insert(out.o_pidx.end(), pool.begin() + re.pbeg, pool.begin() + re.pend);
            out.o_pptr.push_back(int32_t(out.o_pidx.size()));
        }
        out.o_ptr[size_t(u) + 1] = int32_t(out.o_byte.size());
        for (const auto& xe : ends[size_t(u)]) {
            out.x_pidx.insert(out.x_pidx.end(), pool.begin() + xe.first, pool.begin() + xe.second);
            out.x_pptr.push_back(int32_t(out.x_pidx.size()));
        }
        out.x_ptr[size_t(u) + 1] = int32_t(out.x_pptr.size() - 1);
        out.node_end_count[size_t(u)] = double(ends[size_t(u)].size());
        ev.clear(); ev.shrink_to_fit();
    }
    if (out.o_pidx.size() >= size_t(1) << 31) return "parameter lists too large";
    return std::string();
}

}  // namespace wfsa
