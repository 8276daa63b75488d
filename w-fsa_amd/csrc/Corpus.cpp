#include "Corpus.hpp"

#include <cmath>
#include <cstdlib>
#include <unordered_set>

namespace wfsa {

void Corpus::Read(FILE* input) {
    std::vector<char> content;
    if (!read_content(input, content)) throw CorpusError("Cannot read file!");
    Parse(content);
}

void Corpus::ReadText(const char* text) {
    std::vector<char> content(text, text + std::strlen(text));
    content.push_back('\0');
    Parse(content);
}

// Line 1 is the separator (" " when empty).  Every later line is a string:
// its tokens are concatenated and the last token is the weight
// (src/Corpus.cpp:9-61); duplicates and weights that are not positive normal
// numbers are errors.
void Corpus::Parse(std::vector<char>& content) {
    clear();
    char* c = content.data();
    auto result = get_word(c, "\n");
    separator = result.first;
    if (separator.empty()) separator = " ";
    std::unordered_set<std::string> seen;
    std::string word;
    while (result.second != '\0') {
        word.clear();
        bool empty = true;
        do {
            result = get_word(c, separator.c_str());
            if (result.second == '\n' || result.second == '\0') {
                if (!empty) {
                    if (!seen.insert(word).second) throw CorpusError("\"", word, "\" is duplicate!");
                    emplace_back(word, std::atof(result.first));
                }
                break;
            }
            empty = false;
            word += result.first;
        } while (result.second);
    }
    for (const auto& w : *this) {
        if (!std::isnormal(w.second) || w.second < 0)
            throw CorpusError("\"", w.first, "\" has probability ", w.second, "!");
    }
}

void Corpus::Renormalize() {
    const double s = Sum();
    for (auto& w : *this) w.second /= s;
}

double Corpus::Sum() const {
    double s = 0.0;
    for (const auto& w : *this) s += w.second;
    return s;
}

}  // namespace wfsa
