// Weighted automaton: the .wfsa reader/writer and parameter numbering.
// Public interface mirrors the reference's Fsa (inc/Fsa.h:24-106) so a
// Learner written against it drops in; FlatModel is the new part: the graph
// flattened into the wfsa_model_desc the device boundary takes.
#pragma once

#include <cstdint>
#include <cstdio>
#include <vector>

#include "text.hpp"
#include "wfsa_dev.h"

namespace wfsa {

struct FsaError : public MyError {
    using MyError::MyError;
};

class Fsa {
public:
    struct NamedProb {          // an emission (inc/Fsa.h:26-34)
        const char* str;
        double logprob;
        int32_t index;
        NamedProb(const char* s = "", double l = 0.0, int32_t i = -1) : str(s), logprob(l), index(i) {}
    };
    struct State;
    typedef Keyed<State> TransitionMtx;
    typedef const std::pair<const CStr, State>* NextPtr;
    struct NextState {          // a transition (inc/Fsa.h:51-59)
        NextPtr next;
        double logprob;
        int32_t index;
        NextState(NextPtr n, double l = 0.0, int32_t i = -1) : next(n), logprob(l), index(i) {}
    };
    typedef std::vector<NamedProb> Emissions;
    typedef std::vector<NextState> Transitions;
    struct State {
        Emissions emissions;
        Transitions transitions;
    };

    Fsa();
    Fsa(const Fsa& other);
    Fsa& operator=(const Fsa& other);

    void Read(FILE* input);
    void ReadText(const char* text);   // same parser over an in-memory buffer
    void Dump(FILE* out) const;

    size_t GetNumberOfStates() const { return transition_probs.size(); }
    size_t GetNumberOfTransitions() const { return m1; }
    size_t GetNumberOfEmissions() const { return m2; }
    size_t GetNumberOfFreeParameters() const;
    size_t GetNumberOfParameters() const { return n; }
    size_t GetNumberOfConstraints() const { return n - GetNumberOfFreeParameters(); }

    const char* GetStartState() const { return start_state; }
    const char* GetEndState() const { return end_state; }
    const TransitionMtx& GetTransitionMtx() const { return transition_probs; }
    TransitionMtx& GetTransitionMtx() { return transition_probs; }

private:
    void Parse();
    void AssignIndices();
    size_t AllocateStates();
    void Clear();
    void ReadOneState(char*& c);

    TransitionMtx transition_probs;
    size_t m1 = 0, m2 = 0, n = 0;
    CStr separator = "", start_state = "", end_state = "";
    std::vector<char> source;    // file text as read
    std::vector<char> content;   // tokenized copy; state/emission names live here
};

// The automaton flattened for wfsa_dev_load_model.  State ids follow the
// Fsa's map iteration order; names are kept for reporting.
struct FlatModel {
    std::vector<const char*> state_names;
    int32_t start = -1, end = -1, n_params = 0;
    std::vector<int32_t> em_ptr, em_len, em_param, tr_ptr, tr_dst, tr_param;
    std::vector<int64_t> em_off;
    std::vector<uint8_t> em_bytes;
    // per Fsa parameter: owning state, kind (0 emission, 1 transition), label
    std::vector<int32_t> param_state, param_kind;
    std::vector<const char*> param_label;

    explicit FlatModel(const Fsa& fsa);
    wfsa_model_desc desc() const;
};

}  // namespace wfsa
