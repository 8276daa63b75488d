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

// Line 1 is the separator (" " when empty).  Every later line is a list of
// tokens: all but the last, concatenated, form the string and the last is its
// weight; a line of one token holds no string (src/Corpus.cpp:9-61).
// Duplicates and weights that are not positive normal numbers are errors.
void Corpus::Parse(std::vector<char>& content) {
    clear();
    char* cursor = content.data();
    const auto head = get_word(cursor, "\n");
    separator = *head.first ? head.first : " ";
    std::unordered_set<std::string> seen;
    std::vector<CStr> tokens;   // the current line's tokens (pointers into content)
    for (char end = head.second; end != '\0';) {
        tokens.clear();
        do {
            const auto tok = get_word(cursor, separator.c_str());
            tokens.push_back(tok.first);
            end = tok.second;
        } while (end != '\n' && end != '\0');
        if (tokens.size() < 2) continue;
        std::string str;
        for (size_t i = 0; i + 1 < tokens.size(); ++i) str += tokens[i];
        if (!seen.insert(str).second) throw CorpusError("\"", str, "\" is duplicate!");
        const double weight = std::atof(tokens.back());
        emplace_back(std::move(str), weight);
    }
    for (const auto& entry : *this)
        if (!std::isnormal(entry.second) || entry.second < 0)
            throw CorpusError("\"", entry.first, "\" has probability ", entry.second, "!");
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
