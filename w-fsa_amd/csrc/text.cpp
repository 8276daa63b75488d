#include "text.hpp"

#include <limits>

namespace wfsa {

std::pair<const char*, char> get_word(char*& input, const char* separator) {
    const char* word = input;
    const char* sep = separator;
    bool matching = false;  // inside a (possibly partial) separator match
    for (; *input; ++input) {
        if (!matching) {
            if (*input == *sep) {
                matching = true;
                ++sep;
            } else if (*input == '\n') {
                *input++ = '\0';
                return {word, '\n'};
            }
            continue;
        }
        if (*input == *sep) {
            ++sep;
        } else if (*input == '\n') {
            if (*sep == '\0') {
                // separator complete right before the line end: cut it, stay on '\n'
                std::memset(input - (sep - separator), 0, size_t(sep - separator));
                return {word, '\n'};
            }
            *input++ = '\0';
            return {word, '\n'};
        } else if (*sep == '\0') {
            std::memset(input - (sep - separator), 0, size_t(sep - separator));
            return {word, *(sep - 1)};
        } else {
            sep = separator;  // not a separator after all; this byte is not re-examined
            matching = false;
        }
    }
    return {word, '\0'};
}

bool is_empty(const char* s) { return s[0] == '\0'; }

bool contains_prefix(const char* word, const char* prefix) {
    return std::strncmp(word, prefix, std::strlen(prefix)) == 0;
}

bool read_content(FILE* input, std::vector<char>& content) {
    if (!input) return false;
    const long begin = std::ftell(input);
    if (std::fseek(input, 0, SEEK_END) != 0) return false;
    long length = std::ftell(input);
    if (length == -1L) return false;
    length -= begin;
    if (std::fseek(input, begin, SEEK_SET) != 0) return false;
    content.resize(size_t(length));
    content.resize(std::fread(content.data(), 1, size_t(length), input));
    content.push_back('\0');
    return true;
}

double log_simplex_volume(size_t d) {
    if (d == 0) return 0.0;
    double log_fact = 0.0;  // log((d-1)!)
    for (size_t i = 2; i < d; ++i) log_fact += std::log(double(i));
    return 0.5 * std::log(double(d)) - log_fact;
}

double mxlogx(double x) {
    if (x > 0) return -x * std::log(x);
    if (x == 0) return 0.0;
    return std::numeric_limits<double>::infinity();
}

}  // namespace wfsa
