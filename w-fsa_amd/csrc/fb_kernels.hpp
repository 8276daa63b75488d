// Device-side views and launchers of the forward-backward kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace wfsa {

// Compiled trellis automaton resident in HBM (see trellis_model.hpp).
struct ModelView {
    const int32_t* o_ptr;    // [n_nodes+1] out-edges by source node, sorted by byte
    const uint8_t* o_byte;
    const int32_t* o_dst;
    const int32_t* o_pptr;   // [E+1] parameter list of each edge
    const int32_t* o_pidx;
    const double* o_w;       // [E] exp(sum of the edge's log-weights), per iteration
    const int32_t* x_ptr;    // [n_nodes+1] end edges by source node
    const int32_t* x_pptr;
    const int32_t* x_pidx;
    const double* x_w;       // [X] per iteration
    const double* node_end;  // [n_nodes] sum of the node's end-edge weights
    const double* node_end_count;  // [n_nodes] number of end edges (counting mode)
    int32_t n_nodes;
    int32_t start;
};

// Per-wave LDS slab holding one string's trellis: frontier nodes (alpha,
// beta, node id) for every position, the live edges between consecutive
// positions, per-position offsets/scale exponents and the node->slot map.
struct SlabConfig {
    int32_t cap_f;           // frontier entries over all positions
    int32_t cap_e;           // live edges over all positions
    int32_t max_len;         // longest string
    int32_t n_nodes;
    int32_t bytes;           // bytes per wave
    int32_t waves_per_block;
};

struct SlabLayout {
    int32_t alpha, beta, state, eg, esrc, edst, fpos, epos, dsc, slot, total;
};

inline SlabLayout slab_layout(int32_t cap_f, int32_t cap_e, int32_t max_len, int32_t n_nodes) {
    SlabLayout l;
    const int32_t np = max_len + 2;
    l.alpha = 0;
    l.beta = l.alpha + 8 * cap_f;
    l.state = l.beta + 8 * cap_f;
    l.eg = l.state + 4 * cap_f;
    l.esrc = l.eg + 4 * cap_e;
    l.edst = l.esrc + 4 * cap_e;
    l.fpos = l.edst + 4 * cap_e;
    l.epos = l.fpos + 4 * np;
    l.dsc = l.epos + 4 * np;
    l.slot = l.dsc + 4 * np;
    l.total = (l.slot + 4 * n_nodes + 15) & ~15;
    return l;
}

struct FBArgs {
    ModelView m;
    const uint8_t* sym;      // packed corpus bytes
    const int64_t* off;      // [S+1]
    const double* p;         // [S]
    const int32_t* list;     // strings this launch serves
    int32_t n_list;
    SlabConfig slab;
    SlabLayout lay;
    // weighted mode outputs
    double* grad;            // [n_params]  accumulates -p_s * E[count]
    double* ll_part;         // [waves in grid]  sum of p_s log q_s per wave
    double* logq;            // [S] or null
    // counting mode outputs
    double* path_count;      // [S] or null
    uint8_t* recognized;     // [S] or null
    uint8_t* used;           // [n_params] or null
    uint8_t* overflow;       // [S] string did not fit the slab
    unsigned long long* live_edges;  // total live edges touched
};

hipError_t configure_fb_kernels(int max_dynamic_lds);
hipError_t launch_fb(bool counting, const FBArgs& a, int grid, hipStream_t stream);
hipError_t launch_edge_weights(const double* w_full, const int32_t* pptr, const int32_t* pidx, double* out,
                               int64_t n_edges, hipStream_t stream);
hipError_t launch_node_end(const int32_t* x_ptr, const double* x_w, double* node_end, int32_t n_nodes,
                           hipStream_t stream);
hipError_t launch_finalize(const double* ll_part, int32_t n_part, double* out, hipStream_t stream);

}  // namespace wfsa
