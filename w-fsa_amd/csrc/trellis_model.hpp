// Compiles an Fsa (flat wfsa_model_desc) into the byte-step trellis automaton
// the device kernels walk.
//
// The reference enumerates paths by following a transition S->T and then an
// emission e of T that is a prefix of the remaining word (inc/Recognize.h:
// 49-57); the end transition is taken only when the word is consumed
// (:39-47).  Here every such hyper-edge (S->T, e) becomes a "composite edge"
// that consumes exactly ONE byte, so the trellis advances one position per
// byte:
//   * epsilon emissions are removed: a path S->T1(eps)->...->Tk->U(e) becomes
//     one composite edge whose parameter list is the multiset of all the
//     transition/emission parameters on the way (the epsilon sub-graph must be
//     acyclic -- the reference would never terminate on a cycle);
//   * a multi-byte emission e of U gets |e|-1 private chain nodes, so the edge
//     lands on the first chain node and the chain spells the rest of e with
//     weight 1; the parameters sit on the first edge;
//   * end transitions (reached directly or through epsilon states) become end
//     edges with their own parameter lists.
// Paths of the original automaton and paths of the compiled trellis are in
// bijection, so path sums, path counts and expected counts are unchanged.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "wfsa_dev.h"

namespace wfsa {

struct TrellisModel {
    int32_t n_params = 0;   // Fsa parameters (n_full)
    int32_t n_nodes = 0;    // Fsa states + chain nodes
    int32_t start = 0;
    // byte-consuming composite edges, CSR by source node, sorted by byte
    std::vector<int32_t> o_ptr;    // [n_nodes+1]
    std::vector<uint8_t> o_byte;   // [E]
    std::vector<int32_t> o_dst;    // [E]
    std::vector<int32_t> o_pptr;   // [E+1] parameter list CSR
    std::vector<int32_t> o_pidx;
    // end edges, CSR by source node
    std::vector<int32_t> x_ptr;    // [n_nodes+1]
    std::vector<int32_t> x_pptr;   // [X+1]
    std::vector<int32_t> x_pidx;
    std::vector<double> node_end_count;  // [n_nodes] number of end edges
};

// Returns an empty string on success, otherwise the reason the model was
// rejected.
std::string compile_trellis_model(const wfsa_model_desc& d, TrellisModel& out);

}  // namespace wfsa
