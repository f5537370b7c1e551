// ORACLE — TEST INFRASTRUCTURE ONLY.  A C-ABI wrapper around the reference's own host field type,
// kb31_t (crates/core/machine/include/kb31_t.hpp, host branch :451-625: Montgomery form with
// R = 2^32, the in-memory form of KoalaBear in the reference's Rust and C++ alike).  The header is
// compiled from where it lies under /root/reference (never copied; oracle/Makefile target `ref`)
// into oracle/_ref/libkb31_ref.so.  Tests use it to pin the field arithmetic and the Montgomery
// encoding that the C ABI's ZKM_REPR_MONTGOMERY inputs are in.  Not part of the product.
#include <cstddef>
#include <cstdint>
#include "kb31_t.hpp"

extern "C" {
// canonical -> the reference's in-memory (Montgomery) word, and back
void ref_kb31_to_monty(const uint32_t *x, uint32_t *out, uint64_t n) {
    for (uint64_t i = 0; i < n; i++) out[i] = kb31_t::from_canonical_u32(x[i]).val;
}
void ref_kb31_from_monty(const uint32_t *x, uint32_t *out, uint64_t n) {
    for (uint64_t i = 0; i < n; i++) out[i] = kb31_t(x[i]).as_canonical_u32();
}
// op on canonical inputs, canonical outputs: 0 add, 1 sub, 2 mul, 3 reciprocal(a), 4 a^(2^b)
void ref_kb31_binop(int op, const uint32_t *a, const uint32_t *b, uint32_t *out, uint64_t n) {
    for (uint64_t i = 0; i < n; i++) {
        kb31_t x = kb31_t::from_canonical_u32(a[i]), y = kb31_t::from_canonical_u32(b[i]);
        switch (op) {
            case 0: x += y; break;
            case 1: x -= y; break;
            case 2: x *= y; break;
            case 3: x = x.reciprocal(); break;
            default: x = x.exp_power_of_2(b[i]); break;
        }
        out[i] = x.as_canonical_u32();
    }
}
}
