// The string store: the .corpus reader and the packed layout that goes to
// HBM.  Interface mirrors the reference's Corpus (inc/Corpus.h:16-26).
#pragma once

#include <cstdint>
#include <cstdio>
#include <string>
#include <utility>
#include <vector>

#include "text.hpp"

namespace wfsa {

struct CorpusError : public MyError {
    using MyError::MyError;
};

class Corpus : public std::vector<std::pair<std::string, double>> {
public:
    void Read(FILE* input);
    void ReadText(const char* text);
    void Renormalize();
    double Sum() const;

private:
    void Parse(std::vector<char>& content);
    std::string separator;
};

// Strings packed for the device: sym = all bytes back to back,
// off[s]..off[s+1] the bytes of string s.
struct PackedStrings {
    std::vector<uint8_t> sym;
    std::vector<int64_t> off{0};
    void add(const std::string& s) {
        sym.insert(sym.end(), s.begin(), s.end());
        off.push_back(int64_t(sym.size()));
    }
    int64_t size() const { return int64_t(off.size()) - 1; }
};

}  // namespace wfsa
