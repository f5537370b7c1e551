// Machine description (host) and its flattened device form.
// Blob format: include/zkm_hip.h.  Semantics: crates/stark/src/chip.rs:19-175,
// crates/stark/src/permutation.rs:16-23 (width), :355-388 (constraint count).
#pragma once
#include <string>
#include <vector>

#include "internal.hpp"

namespace zkm {

enum Op : uint32_t {
    OP_END = 0, OP_MAIN_L, OP_MAIN_N, OP_PREP_L, OP_PREP_N, OP_CONST, OP_PV,
    OP_IS_FIRST, OP_IS_LAST, OP_IS_TRANS, OP_ADD, OP_SUB, OP_MUL, OP_NEG, OP_EMIT,
    OP_LET, OP_GET  // shared subexpressions: LET s pops the top into value slot s, GET s pushes it
};

struct VPC {
    std::vector<uint32_t> cols;     // bit31 = main
    std::vector<uint32_t> weights;  // canonical
    uint32_t constant = 0;          // canonical
};
struct LookupDesc {
    uint32_t kind = 0, scope = 0;
    bool is_send = true;
    std::vector<VPC> values;
    VPC mult;
};
struct ChipDesc {
    std::string name;
    int prep_w = 0, main_w = 0, scope = 0, local_only = 0, log_qd = 0, n_main = 0;
    std::vector<uint32_t> code;        // canonical constants
    std::vector<LookupDesc> local;     // local-scope lookups, sends then receives
    int perm_w = 0;                    // EF columns
    int n_constraints = 0;
    int max_stack = 0;
    int n_slots = 0;                   // value slots of shared subexpressions (1 + largest LET slot)
};
struct Machine {
    int num_pv = 0;
    std::vector<ChipDesc> chips;
    int index_of(const std::string &n) const {
        for (size_t i = 0; i < chips.size(); i++)
            if (chips[i].name == n) return (int)i;
        return -1;
    }
};

Machine parse_machine(const uint32_t *w, size_t n);

// Device program of one chip (u32 words, constants in Montgomery form):
//   [0] code_len, [1] code offset, [2] n_local, [3] lookup table offset
//   code: ops with Montgomery constants
//   lookup i (at lookup table offset + 4*i): kind_mont, is_send, nvalues, vpc offset of values
//   vpc: nterms, (col, weight_mont) * nterms, const_mont ; values' vpcs back to back, then mult
std::vector<uint32_t> flatten_chip(const ChipDesc &c);

}  // namespace zkm
