#include "Fsa.hpp"

#include <algorithm>
#include <cstdlib>
#include <numeric>
#include <unordered_map>

namespace wfsa {

Fsa::Fsa() {}

Fsa::Fsa(const Fsa& other) { *this = other; }

Fsa& Fsa::operator=(const Fsa& other) {
    // Names and NextPtr targets point into `content` and into the map, so a
    // copy re-parses the source text instead of rebasing pointers.
    if (this == &other) return *this;
    Clear();
    source = other.source;
    if (!source.empty()) Parse();
    return *this;
}

void Fsa::Clear() {
    m1 = m2 = n = 0;
    separator = start_state = end_state = "";
    transition_probs.clear();
}

size_t Fsa::AllocateStates() {
    // rows: 3 header lines + 2 per state (src/Fsa.cpp:112-120 semantics)
    const size_t lines = size_t(std::count(content.begin(), content.end(), '\n'));
    const size_t expected = (std::max<size_t>(lines, 3) - 3) / 2 + 1;
    transition_probs.reserve(expected);
    transition_probs.max_load_factor(0.8f);
    return expected;
}

void Fsa::Read(FILE* input) {
    Clear();
    source.clear();
    if (!read_content(input, source)) throw FsaError("Unable to read file!");
    Parse();
}

void Fsa::ReadText(const char* text) {
    Clear();
    source.assign(text, text + std::strlen(text));
    source.push_back('\0');
    Parse();
}

void Fsa::Parse() {
    // the tokenizer writes NULs: parse a private copy (names point into it)
    // and keep `source` intact so copies can re-parse
    content = source;
    const size_t expected = AllocateStates();
    char* c = content.data();
    separator = get_word(c, "\n").first;
    start_state = get_word(c, "\n").first;
    end_state = get_word(c, "\n").first;
    if (is_empty(separator)) separator = " ";
    for (CStr x : {start_state, end_state}) {
        if (contains_prefix(x, separator))
            throw FsaError("Invalid FSA format! Start or end state contains the separator! \"", separator,
                           "\" is in \"", x, "\"");
    }
    if (StrEq()(start_state, end_state))
        throw FsaError("Invalid FSA format! Start and end states should be different! \"", start_state, "\"==\"",
                       end_state, "\"");
    while (*c) ReadOneState(c);
    if (transition_probs.size() > expected)
        throw FsaError("Invalid FSA format! There are more states than rows in the automaton file! ",
                       transition_probs.size(), " > ", expected);
    AssignIndices();
}

namespace {

// The (key, value) tokens after a row's head, up to the line end: a state's
// emission row "name e1 w1 e2 w2 ..." or its transition row "name t1 w1 ...".
using Pairs = std::vector<std::pair<CStr, CStr>>;
void read_pairs(char*& c, CStr sep, Pairs& out) {
    out.clear();
    std::pair<CStr, char> value;
    do {
        const CStr key = get_word(c, sep).first;
        value = get_word(c, sep);
        out.emplace_back(key, value.first);
    } while (value.second != '\n' && value.second != '\0');
}

}  // namespace

// One state: its emission row, then its transition row, which must name the
// same state (src/Fsa.cpp:122-205).  A row starting blank or with the end
// state's name is skipped.  The emissions / transitions are collected in
// Keyed maps and copied out in their iteration order, and every successor is
// entered into transition_probs before the state itself: both orders decide
// the parameter numbering (AssignIndices), so they follow the reference's.
void Fsa::ReadOneState(char*& c) {
    const CStr name = get_word(c, separator).first;
    if (is_empty(name) || contains_prefix(name, end_state)) {
        get_word(c, "\n");
        return;
    }
    const bool is_start = StrEq()(name, start_state);
    Pairs row;
    read_pairs(c, separator, row);
    Keyed<double> emissions;
    for (const auto& kv : row) {
        if (is_start && !is_empty(kv.first))
            throw FsaError("Invalid FSA format! Start state should emit empty string instead of \"", kv.first, "\"!");
        if (!emissions.emplace(kv.first, std::atof(kv.second)).second)
            throw FsaError("Invalid FSA format! Emission \"", kv.first, "\" of state \"", name,
                           "\" appears more than once!");
    }
    if (emissions.empty())
        throw FsaError("Invalid FSA format! State \"", name,
                       "\" should have positive number of emissions, even if empty emission!");
    if (!StrEq()(name, get_word(c, separator).first))
        throw FsaError("Invalid FSA format! You should enlist transitions of \"", name,
                       "\" after emissions of the same state!");
    read_pairs(c, separator, row);
    Keyed<double> transitions;
    for (const auto& kv : row) {
        if (!transitions.emplace(kv.first, std::atof(kv.second)).second)
            throw FsaError("Invalid FSA format! Transition \"", name, "\" -> \"", kv.first,
                           "\" appears more than once!");
        if (StrEq()(kv.first, start_state))
            throw FsaError("Invalid FSA format! \"", name, "\" connects to start state \"", start_state, "\"!");
    }
    if (transitions.empty())
        throw FsaError("Invalid FSA format! State \"", name, "\" should have positive number of transitions!");

    State st;
    for (const auto& e : emissions) st.emissions.emplace_back(e.first, e.second);
    for (const auto& t : transitions)
        st.transitions.emplace_back(&(*transition_probs.emplace(t.first, State()).first), t.second);
    transition_probs[name] = st;
}

void Fsa::AssignIndices() {
    m1 = m2 = n = 0;
    for (auto& s : transition_probs) {
        auto& em = s.second.emissions;
        auto& tr = s.second.transitions;
        if (em.size() == 1) em.front().index = -1;   // unequivocal
        else for (auto& e : em) e.index = int32_t(n++);
        if (tr.size() == 1) tr.front().index = -1;
        else for (auto& t : tr) t.index = int32_t(n++);
        m1 += tr.size();
        m2 += em.size();
    }
}

size_t Fsa::GetNumberOfFreeParameters() const {
    return m1 + m2 - 2 * (transition_probs.size() - 1);
}

void Fsa::Dump(FILE* out) const {
    std::fprintf(out, "%s\n%s\n%s\n", separator, start_state, end_state);
    for (const auto& s : transition_probs) {
        if (StrEq()(s.first, end_state)) continue;
        std::fprintf(out, "%s", s.first);
        for (const auto& e : s.second.emissions)
            std::fprintf(out, "%s%s%s%g", separator, e.str, separator, e.logprob);
        std::fprintf(out, "\n%s", s.first);
        for (const auto& t : s.second.transitions)
            std::fprintf(out, "%s%s%s%g", separator, t.next->first, separator, t.logprob);
        std::fprintf(out, "\n");
    }
}

FlatModel::FlatModel(const Fsa& fsa) {
    const auto& mtx = fsa.GetTransitionMtx();
    std::unordered_map<const void*, int32_t> id;
    id.reserve(mtx.size());
    for (const auto& s : mtx) {
        id.emplace(&s, int32_t(state_names.size()));
        state_names.push_back(s.first);
    }
    auto find = [&](const char* name) -> int32_t {
        auto it = mtx.find(name);
        return it == mtx.end() ? -1 : id.at(&(*it));
    };
    start = find(fsa.GetStartState());
    end = find(fsa.GetEndState());
    n_params = int32_t(fsa.GetNumberOfParameters());
    param_state.assign(size_t(n_params), -1);
    param_kind.assign(size_t(n_params), -1);
    param_label.assign(size_t(n_params), "");
    em_ptr.push_back(0);
    tr_ptr.push_back(0);
    for (const auto& s : mtx) {
        const int32_t sid = id.at(&s);
        for (const auto& e : s.second.emissions) {
            const size_t len = std::strlen(e.str);
            em_off.push_back(int64_t(em_bytes.size()));
            em_len.push_back(int32_t(len));
            em_param.push_back(e.index);
            em_bytes.insert(em_bytes.end(), e.str, e.str + len);
            if (e.index >= 0) { param_state[e.index] = sid; param_kind[e.index] = 0; param_label[e.index] = e.str; }
        }
        em_ptr.push_back(int32_t(em_len.size()));
        for (const auto& t : s.second.transitions) {
            tr_dst.push_back(id.at(t.next));
            tr_param.push_back(t.index);
            if (t.index >= 0) { param_state[t.index] = sid; param_kind[t.index] = 1; param_label[t.index] = t.next->first; }
        }
        tr_ptr.push_back(int32_t(tr_dst.size()));
    }
    if (em_bytes.empty()) em_bytes.push_back(0);
}

wfsa_model_desc FlatModel::desc() const {
    wfsa_model_desc d;
    d.n_states = int32_t(state_names.size());
    d.start = start;
    d.end = end;
    d.n_params = n_params;
    d.em_ptr = em_ptr.data();
    d.em_off = em_off.data();
    d.em_len = em_len.data();
    d.em_param = em_param.data();
    d.em_bytes = em_bytes.data();
    d.tr_ptr = tr_ptr.data();
    d.tr_dst = tr_dst.data();
    d.tr_param = tr_param.data();
    return d;
}

}  // namespace wfsa
