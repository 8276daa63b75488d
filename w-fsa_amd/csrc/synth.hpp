// Synthetic benchmark inputs (see synth.cpp).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace wfsa {

struct SynthSpec {
    int32_t n_states = 1024, degree = 8, vocab = 64, emissions = 1, dense = 0;
    int64_t n_strings = 1000;
    int32_t max_len = 128;
    uint64_t seed = 1;
};

struct SynthOutput {
    std::string wfsa_text;
    std::vector<uint8_t> sym;
    std::vector<int64_t> off;
    std::vector<double> weights;
};

// Returns an empty string on success, else the reason.
std::string make_synthetic(const SynthSpec& spec, SynthOutput& out);

}  // namespace wfsa
