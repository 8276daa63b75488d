// Text and container helpers shared by the .wfsa / .corpus readers.
//
// Behaviour follows the reference's tokenizer and containers so that files
// parse identically and parameters get the same numbering:
//   * get_word  <- GetWord (src/Utils.cpp:20-80), quirks included
//   * StrHash   <- FNV-1a over signed chars (src/Utils.cpp:276-294)
//   * Keyed<T>  <- std::unordered_map<const char*, T, StrHash, StrEq>
//                  (inc/Utils.h:104-108): iteration order of this container
//                  decides parameter numbering in Fsa::AssignIndices.
#pragma once

#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <exception>
#include <sstream>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace wfsa {

typedef const char* CStr;

struct StrEq {
    bool operator()(const CStr& a, const CStr& b) const { return std::strcmp(a, b) == 0; }
};

struct StrHash {
    size_t operator()(const CStr& s) const {
        size_t h = sizeof(size_t) == 8 ? size_t(14695981039346656037ULL) : size_t(2166136261U);
        const size_t prime = sizeof(size_t) == 8 ? size_t(1099511628211ULL) : size_t(16777619U);
        for (const char* p = s; *p; ++p) {
            h ^= size_t(*p);  // sign-extends bytes >= 0x80, as the reference does
            h *= prime;
        }
        return h;
    }
};

template <class T>
struct Keyed : std::unordered_map<CStr, T, StrHash, StrEq> {};

// The reference's error hierarchy (inc/Utils.h:130-141): a message built
// from any streamable arguments.
class MyError : public std::exception {
public:
    template <typename... Args>
    explicit MyError(const Args&... args) {
        std::ostringstream oss;
        (void)std::initializer_list<int>{(oss << args, 0)...};
        msg_ = oss.str();
    }
    const char* what() const noexcept override { return msg_.c_str(); }

private:
    std::string msg_;
};

// (word, terminator): terminator is the last separator byte, '\n' or '\0'.
std::pair<const char*, char> get_word(char*& input, const char* separator = " ");

bool is_empty(const char* s);
bool contains_prefix(const char* word, const char* prefix);
bool read_content(FILE* input, std::vector<char>& content);
double log_simplex_volume(size_t d);
double mxlogx(double x);

// PrintFixedWidth (src/Utils.cpp:82-97): the epoch table's and the matrix
// printer's number format
void print_fixed_width(FILE* out, double x, int width = 7);
// PrintCsrMtx (src/Utils.cpp:157-182): one text row per matrix row, every
// stored entry in its column (8 characters per column, blanks for the gaps),
// optionally "|" and the row's right-hand side.  data == nullptr: all ones.
void print_csr(FILE* out, const double* data, const std::vector<int32_t>& rows, const std::vector<int32_t>& cols,
               const std::vector<double>* rhs = nullptr);

}  // namespace wfsa
