// Argument block of JIT-compiled quotient kernels (shared verbatim by host code and the
// generated source, so the layout matches by construction).  Plain C, no HIP dependencies.
#ifndef ZKM_JIT_ABI_H
#define ZKM_JIT_ABI_H
struct ZkmQuotJitArgs {
    const unsigned *main, *prep, *perm;  // LDEs, column stride ld, bit-reversed rows
    const unsigned *pv;                  // public values (Montgomery)
    const unsigned *pows;                // alpha^(nc-1-k), EF (4 words each)
    const unsigned *beta_pows;           // beta^(j+1), EF
    const unsigned *tw;                  // forward twiddles
    unsigned *chunks;                    // 2^lqd chunks x 4 columns x n rows (bit-reversed rows)
    unsigned long long ld, n, q;
    unsigned long long cstride;          // words between chunk j and chunk j+1 (column stride is n)
    int log_n, log_q, step, pad0;
    unsigned gen, gen_pow_n, wn_inv, pad1;
    unsigned alpha_p[4], lcs[4];
    unsigned gcs[14];
    const unsigned *prog;                // flattened chip program (lookup table: chips with many lookups)
};
struct ZkmPermJitArgs {
    const unsigned *main, *prep;  // traces, column-major natural, column stride ld
    const unsigned *beta_pows;    // beta^(j+1), EF
    unsigned *out;                // perm trace batch columns (4 per batch), column stride ld
    unsigned *rowsum;             // per-row EF total (scan input)
    unsigned long long ld;        // rows
    unsigned alpha[4];
    const unsigned *prog;         // flattened chip program (lookup table: chips with many lookups)
};
#endif
