#include "text.hpp"

#include <algorithm>
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

void print_fixed_width(FILE* out, double x, int width) {
    const int mag = (x == 0) ? 0 : int(std::floor(std::log10(std::abs(x))));
    if (mag <= width - 2 && mag >= 0) {
        if (std::floor(x) == x) std::fprintf(out, "%*.0f", width, x);
        else std::fprintf(out, "%*.*f", width, std::max(0, width - 3 - mag), x);
    } else if (-4 < mag && mag < 0) {
        std::fprintf(out, "%*.*f", width, width - 3, x);
    } else {
        std::fprintf(out, "%*.*e", width, width - 7, x);
    }
}

void print_csr(FILE* out, const double* data, const std::vector<int32_t>& rows, const std::vector<int32_t>& cols,
               const std::vector<double>* rhs) {
    if (rows.empty()) return;
    const int64_t width = int64_t(rows.size()) - 1;
    for (size_t r = 0; r + 1 < rows.size(); ++r) {
        int64_t col = -1;   // the last column printed
        for (int32_t q = rows[r]; q < rows[r + 1]; ++q) {
            for (; col < int64_t(cols[size_t(q)]) - 1; ++col) std::fputs("        ", out);
            col = cols[size_t(q)];
            print_fixed_width(out, data ? data[q] : 1.0, 7);
            std::fputs(" ", out);
        }
        if (rhs && rhs->size() > r) {
            for (; col < width - 1; ++col) std::fputs("        ", out);
            std::fputs("|", out);
            print_fixed_width(out, (*rhs)[r], 7);
        }
        std::fputs("\n", out);
    }
}

}  // namespace wfsa
