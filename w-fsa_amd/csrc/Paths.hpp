// Host path enumeration over the parsed automaton: the reference's
// Recognizer (inc/Recognize.h:34-96), for the features that print or save
// explicit paths -- the -p / -pr listing (src/main.cpp:178-203), the P / M
// matrices of -p and of -m >prefix (Learner::BuildPaths, src/Learner.cpp:
// 276-348).  The objective and gradient never use it: they run on the device
// trellis.  Same visiting order as the reference (its containers' iteration
// order, BFS queue or DFS recursion), so paths come out in the same order;
// the reference's one-second BFS clock is replaced by a cap on the states
// visited per word (an error, not a silent truncation).
#pragma once

#include <cstring>
#include <deque>
#include <string>

#include "Fsa.hpp"

namespace wfsa {

struct PathError : public MyError {
    using MyError::MyError;
};

// acc(Path& history, const Fsa::NextState& transition, const Fsa::NamedProb& emission):
// extends the history by one transition and the emission of its target (a
// default emission for the end transition); done(const Path&): one accepting path.
template <class Path, class Acc, class Done>
class HostRecognizer {
public:
    HostRecognizer(const Fsa& fsa, Acc acc, Done done, int64_t cap = int64_t(1) << 24)
        : fsa_(fsa), acc_(acc), done_(done), cap_(cap) {}

    void Recognize(const char* word, const Path& start, bool bfs) {
        const Fsa::State& s0 = fsa_.GetTransitionMtx().at(fsa_.GetStartState());
        visited_ = 0;
        if (bfs) Bfs(word, s0, start);
        else Dfs(word, s0, start);
    }

private:
    bool is_end(const Fsa::NextState& t) const { return std::strcmp(t.next->first, fsa_.GetEndState()) == 0; }
    void count() {
        if (++visited_ > cap_) throw PathError("Path enumeration: more than ", cap_, " partial paths for one string");
    }

    void Dfs(const char* word, const Fsa::State& state, const Path& history) {   // inc/Recognize.h:34-60
        count();
        for (const auto& t : state.transitions) {
            if (is_end(t)) {
                if (word[0] == '\0') {
                    Path path(history);
                    acc_(path, t, Fsa::NamedProb());
                    done_(path);
                }
                continue;
            }
            const Fsa::State& next = t.next->second;
            for (const auto& e : next.emissions) {
                if (!contains_prefix(word, e.str)) continue;
                Path path(history);
                acc_(path, t, e);
                Dfs(word + std::strlen(e.str), next, path);
            }
        }
    }

    void Bfs(const char* word, const Fsa::State& state, const Path& history) {   // inc/Recognize.h:62-96
        struct Item {
            const char* word;
            const Fsa::State* state;
            Path history;
        };
        std::deque<Item> queue;   // push_back keeps references to the front valid
        queue.push_back(Item{word, &state, history});
        while (!queue.empty()) {
            count();
            const Item& w = queue.front();
            for (const auto& t : w.state->transitions) {
                if (is_end(t)) {
                    if (w.word[0] == '\0') {
                        Path path(w.history);
                        acc_(path, t, Fsa::NamedProb());
                        done_(path);
                    }
                    continue;
                }
                const Fsa::State& next = t.next->second;
                for (const auto& e : next.emissions) {
                    if (!contains_prefix(w.word, e.str)) continue;
                    queue.push_back(Item{w.word + std::strlen(e.str), &next, w.history});
                    acc_(queue.back().history, t, e);
                }
            }
            queue.pop_front();
        }
    }

    const Fsa& fsa_;
    Acc acc_;
    Done done_;
    int64_t cap_, visited_ = 0;
};

template <class Path, class Acc, class Done>
HostRecognizer<Path, Acc, Done> make_recognizer(const Fsa& fsa, Acc acc, Done done) {
    return HostRecognizer<Path, Acc, Done>(fsa, acc, done);
}

}  // namespace wfsa
