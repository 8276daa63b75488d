// Synthetic automata + corpora for the benchmark configurations
// ("family A" / "family B"): N states with D random successors
// plus the end state, E emitted symbols per state out of V printable bytes,
// strings sampled by walking the automaton (stop probability 1/32 per step,
// capped length), all distinct, integer weights 1..10.
#include "synth.hpp"

#include <cmath>
#include <cstdio>
#include <string>
#include <unordered_set>
#include <vector>

namespace wfsa {

namespace {

struct Rng {   // xoshiro256**
    uint64_t s[4];
    explicit Rng(uint64_t seed) {
        uint64_t z = seed;
        for (auto& v : s) {   // splitmix64
            z += 0x9e3779b97f4a7c15ULL;
            uint64_t x = z;
            x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
            x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
            v = x ^ (x >> 31);
        }
    }
    static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
    uint64_t next() {
        const uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
        s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl(s[3], 45);
        return r;
    }
    uint32_t below(uint32_t n) { return uint32_t((next() >> 32) * uint64_t(n) >> 32); }
    double unit() { return double(next() >> 11) * (1.0 / 9007199254740992.0); }
};

const char kAlphabet[] =
    "0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz+-*/=<>?!#%&()[]{}:;,.@_~|^";

// k distinct values from [0, n)
std::vector<int32_t> sample(Rng& rng, int32_t n, int32_t k) {
    std::vector<int32_t> out;
    if (k >= n) {
        for (int32_t i = 0; i < n; ++i) out.push_back(i);
        return out;
    }
    std::unordered_set<int32_t> seen;
    while (int32_t(out.size()) < k) {
        const int32_t v = int32_t(rng.below(uint32_t(n)));
        if (seen.insert(v).second) out.push_back(v);
    }
    return out;
}

}  // namespace

std::string make_synthetic(const SynthSpec& spec, SynthOutput& out) {
    const int32_t N = spec.n_states, V = spec.vocab, E = spec.emissions;
    const int32_t D = spec.dense ? N : spec.degree;
    if (N < 1 || V < 1 || V > int32_t(sizeof(kAlphabet) - 1) || E < 1 || E > V || D < 1 || D > N)
        return "bad synthetic specification";
    if (spec.max_len < 1) return "max_len must be positive";
    Rng rng(spec.seed);
    std::vector<std::vector<int32_t>> succ(static_cast<size_t>(N) + 1);   // index N = start state
    std::vector<std::vector<int32_t>> emit(static_cast<size_t>(N));
    for (int32_t s = 0; s < N; ++s) {
        emit[size_t(s)] = sample(rng, V, E);
        succ[size_t(s)] = sample(rng, N, D);
    }
    succ[size_t(N)] = sample(rng, N, D);

    // automaton text: empty separator line -> " "
    std::string& t = out.wfsa_text;
    t.clear();
    t += "\n^\n$\n^  0\n^";
    char buf[64];
    const double w_start = std::log(1.0 / D);
    for (int32_t d : succ[size_t(N)]) {
        std::snprintf(buf, sizeof buf, " q%d %.17g", d, w_start);
        t += buf;
    }
    t += "\n";
    const double w_step = std::log((1.0 - 1.0 / 32.0) / D), w_end = std::log(1.0 / 32.0);
    const double w_emit = std::log(1.0 / E);
    for (int32_t s = 0; s < N; ++s) {
        std::snprintf(buf, sizeof buf, "q%d", s);
        t += buf;
        for (int32_t e : emit[size_t(s)]) {
            std::snprintf(buf, sizeof buf, " %c %.17g", kAlphabet[e], w_emit);
            t += buf;
        }
        std::snprintf(buf, sizeof buf, "\nq%d", s);
        t += buf;
        for (int32_t d : succ[size_t(s)]) {
            std::snprintf(buf, sizeof buf, " q%d %.17g", d, w_step);
            t += buf;
        }
        std::snprintf(buf, sizeof buf, " $ %.17g\n", w_end);
        t += buf;
    }

    // distinct strings by walking the automaton
    out.sym.clear();
    out.off.assign(1, 0);
    out.weights.clear();
    std::unordered_set<std::string> seen;
    seen.reserve(size_t(spec.n_strings) * 2);
    std::string w;
    int64_t attempts = 0;
    const int64_t max_attempts = 64 * spec.n_strings + 1000;
    while (int64_t(out.weights.size()) < spec.n_strings) {
        if (++attempts > max_attempts) return "could not sample enough distinct strings";
        w.clear();
        int32_t s = succ[size_t(N)][rng.below(uint32_t(D))];
        w += kAlphabet[emit[size_t(s)][rng.below(uint32_t(E))]];
        while (int32_t(w.size()) < spec.max_len && rng.unit() >= 1.0 / 32.0) {
            s = succ[size_t(s)][rng.below(uint32_t(D))];
            w += kAlphabet[emit[size_t(s)][rng.below(uint32_t(E))]];
        }
        if (!seen.insert(w).second) continue;
        out.sym.insert(out.sym.end(), w.begin(), w.end());
        out.off.push_back(int64_t(out.sym.size()));
        out.weights.push_back(double(1 + rng.below(10)));
    }
    return std::string();
}

}  // namespace wfsa
