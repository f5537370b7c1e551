/*
 * zkm_hip.h — C ABI of the MI355X-native shard prover (libzkm_hip.so).
 *
 * Drop-in for the reference's per-shard prover surface, the Rust trait
 * `MachineProver<SC, A>` implemented by `CpuProver` (crates/stark/src/prover.rs:30-184, :210-694),
 * selected through `ZKMProverComponents::CoreProver` (crates/prover/src/components.rs:6-35).
 * The reference's own FFI precedent is `extern "C-unwind"` into a native library with
 * Montgomery-form KoalaBear values (crates/core/machine/src/sys.rs:14-42,
 * crates/core/machine/cpp/extern.cpp:6-37); this ABI follows it: plain pointers and sizes, no
 * language runtime types, status codes instead of panics.  INTEGRATION.md shows the Rust binding.
 *
 * Field elements: KoalaBear p = 2^31 - 2^24 + 1, one u32 each.  Inputs say whether they are
 * canonical residues or Montgomery form (R = 2^32, the in-memory form of p3 MontyField31);
 * challenger state and digests crossing this ABI are canonical.
 *
 * Thread safety: every entry point may be called concurrently from several host threads (the
 * reference calls commit/open from rayon workers for all shards of a batch,
 * crates/core/machine/src/utils/prove.rs:487-521); each call runs on its own HIP stream.
 */
#ifndef ZKM_HIP_H
#define ZKM_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---- */
#define ZKM_OK 0
#define ZKM_ERR_ARG (-1)          /* malformed argument / machine blob */
#define ZKM_ERR_HIP (-2)          /* HIP runtime error (message via zkm_last_error) */
#define ZKM_ERR_UNSATISFIED (-3)  /* constraints not satisfied: FRI final polynomial not constant */
#define ZKM_ERR_UNSUPPORTED (-4)  /* e.g. log_quotient_degree > log_blowup */
#define ZKM_ERR_NO_DEVICE (-5)    /* no usable gfx950 device */

#define ZKM_REPR_CANONICAL 0u
#define ZKM_REPR_MONTGOMERY 1u
#define ZKM_MEM_DEVICE 0x100u  /* OR into zkm_matrix_t.repr: `data` is a row-major buffer already
                                  resident in the context GPU's memory (e.g. a torch tensor) */

typedef struct zkm_ctx zkm_ctx;   /* one per GPU: device, stream pool, twiddle tables */
typedef struct zkm_pk zkm_pk;     /* DeviceProvingKey   (prover.rs:40, machine.rs:55-75)   */
typedef struct zkm_main zkm_main; /* ShardMainData<SC, DeviceMatrix, DeviceProverData> (types.rs:16-22) */
typedef struct zkm_machine zkm_machine; /* a machine layout (StarkMachine chips), no preprocessed data */

/* PCS / FRI configuration (crates/stark/src/kb31_poseidon2.rs:203-213). */
typedef struct {
    uint32_t num_queries;      /* FRI_QUERIES, default 84 */
    uint32_t pow_bits;         /* proof_of_work_bits, 16 */
    uint32_t log_blowup;       /* 1 (core config) or 2 (compressed_fri_config, kb31_poseidon2.rs:217-227) */
    uint32_t proof_montgomery; /* 0: field elements in proof bytes are canonical; 1: Montgomery */
} zkm_config_t;

/* DuplexChallenger<KoalaBear, Poseidon2KoalaBear<16>, 16, 8> state, canonical values
 * (semantics: crates/recursion/circuit/src/challenger.rs:60-233). */
typedef struct {
    uint32_t sponge_state[16];
    uint32_t num_inputs;
    uint32_t input_buffer[8];
    uint32_t num_outputs;
    uint32_t output_buffer[8];
} zkm_challenger_t;

/* A host row-major matrix, the layout of p3 RowMajorMatrix<KoalaBear>. */
typedef struct {
    const char *name;       /* chip name (MachineAir::name) */
    const uint32_t *data;   /* height * width values, row-major */
    uint64_t height;        /* power of two, >= 16 for traces */
    uint64_t width;
    uint32_t repr;          /* ZKM_REPR_CANONICAL or ZKM_REPR_MONTGOMERY, | ZKM_MEM_DEVICE */
} zkm_matrix_t;

/* ---- context ---- */
int zkm_init(int device, zkm_ctx **out);
void zkm_destroy(zkm_ctx *ctx);
const char *zkm_last_error(void);  /* thread-local message of the last failing call */
int zkm_device_count(void);

/* ---- page-locked host memory for traces ----
 * A trace generator that writes its RowMajorMatrix storage here hands the prover host buffers
 * the DMA engines read directly: the H2D copy runs asynchronously, overlapped with this and other
 * shards' kernels, at the PCIe rate.  Any other host pointer is also accepted (the runtime stages
 * it, and the call waits for the copy).  Backs the Rust shim's trace allocator. */
int zkm_host_alloc(size_t bytes, void **out);
void zkm_host_free(void *p);

/* ---- MachineProver::setup (prover.rs:52 -> machine.rs:332-439) ----
 * machine_blob: machine description (format below); prep[i] is the preprocessed trace of
 * machine chip i (data == NULL / width 0 for chips without one).  Writes the preprocessed
 * commitment (vk.commit) to commit_out[8] (canonical). */
int zkm_setup(zkm_ctx *ctx, const uint32_t *machine_blob, size_t nwords, const zkm_config_t *cfg,
              const zkm_matrix_t *prep, uint32_t nprep, uint32_t pc_start,
              const uint32_t initial_global_cumulative_sum[14], zkm_pk **pk_out, uint32_t commit_out[8]);
void zkm_pk_free(zkm_pk *pk);
/* StarkProvingKey::observe_into (machine.rs:77-85): commit, pc_start, gcs x/y, 0 */
int zkm_pk_observe(const zkm_pk *pk, zkm_challenger_t *ch);

/* ---- MachineProver::commit (prover.rs:111-115, :258-292) ----
 * traces: the shard's named main traces (any order; sorted here by (height desc, name)).
 * public_values: record.public_values() (the first num_pv_elts are observed by open).
 * On success *main_out owns the device LDEs + Merkle tree; main_commit_out[8] = root. */
int zkm_commit(zkm_ctx *ctx, const zkm_pk *pk, const zkm_matrix_t *traces, uint32_t ntraces,
               const uint32_t *public_values, uint32_t npv, zkm_main **main_out, uint32_t main_commit_out[8]);
/* The same commit against a key-free machine handle: the trait's commit receives no proving key
 * (prover.rs:111-115, called concurrently with other programs' setups by the compress workers,
 * prover/src/lib.rs:794-824), and commit reads only the machine layout (chip names, main widths,
 * blowup).  zkm_open rejects (ZKM_ERR_ARG) a shard committed under a different machine than its key. */
int zkm_machine_new(const uint32_t *machine_blob, size_t nwords, const zkm_config_t *cfg, zkm_machine **out);
void zkm_machine_free(zkm_machine *m);
int zkm_commit_machine(zkm_ctx *ctx, const zkm_machine *m, const zkm_matrix_t *traces, uint32_t ntraces,
                       const uint32_t *public_values, uint32_t npv, zkm_main **main_out,
                       uint32_t main_commit_out[8]);
void zkm_main_free(zkm_main *main);

/* ---- MachineProver::open (prover.rs:132-137, :298-653) ----
 * Consumes `main` (freed on return, success or not).  The challenger is advanced exactly as the
 * reference's is.  *proof_out receives the serialized ShardProof (bincode-1 layout, see
 * DESIGN.md "Proof bytes"); release it with zkm_free_bytes. */
int zkm_open(zkm_ctx *ctx, const zkm_pk *pk, zkm_main *main, zkm_challenger_t *ch,
             uint8_t **proof_out, uint64_t *proof_len);
void zkm_free_bytes(uint8_t *p);

/* ---- convenience: commit + open for one shard, challenger cloned from `base` ----
 * (the body of the reference's per-shard closure, prove.rs:492-497 / prover.rs:686-687) */
int zkm_prove_shard(zkm_ctx *ctx, const zkm_pk *pk, const zkm_matrix_t *traces, uint32_t ntraces,
                    const uint32_t *public_values, uint32_t npv, const zkm_challenger_t *base,
                    uint8_t **proof_out, uint64_t *proof_len);

/* ---- PCS commit only (TwoAdicFriPcs::commit for trace domains: LDE x2 on coset 3*H, bit-reversed
 * rows, MerkleTreeMmcs root).  Used for configuration 2 (S-COMMIT). */
int zkm_pcs_commit_root(zkm_ctx *ctx, const zkm_matrix_t *mats, uint32_t n, uint32_t root_out[8]);

/* ---- kernel-level entry points (parity tests, microbenchmarks) ---- */
/* out (host, row-major (h << 1) x w, canonical): bit-reversed coset LDE with the given shift */
int zkm_coset_lde(zkm_ctx *ctx, const zkm_matrix_t *m, uint32_t shift_canonical, uint32_t *out);
/* same; bitrev_in != 0: the input rows are the evaluations in bit-reversed order (quotient chunks) */
int zkm_coset_lde_ex(zkm_ctx *ctx, const zkm_matrix_t *m, uint32_t shift_canonical, int bitrev_in, uint32_t *out);
/* n independent Poseidon2-16 permutations of canonical states (in place, host memory) */
int zkm_poseidon2_permute(zkm_ctx *ctx, uint32_t *states, uint64_t n);
/* Timing helper: runs `iters` LDEs of a resident random h x w matrix, returns average ms of the
 * whole LDE and of each kernel stage via HIP events (see bench.py). */
int zkm_bench_lde(zkm_ctx *ctx, uint64_t h, uint64_t w, int iters, double *ms_out);
/* Generates and compiles (hiprtc, gfx950, no device needed) the per-chip specialised quotient
 * kernels zkm_setup builds for this machine blob; returns the total code-object size.  Build /
 * codegen check only.  zkm_setup compiles the same kernels (set ZKM_NO_JIT=1 to use the generic
 * interpreter kernel instead; ZKM_JIT_DUMP=<dir> writes the generated sources). */
int zkm_quotient_jit_compile(const uint32_t *blob, size_t nwords, uint64_t *code_bytes);

/* ---- stage profiling (HIP events on the launching stream; see bench.py) ----
 * zkm_profile_dump writes lines "stage count total_ms units" and returns the bytes needed. */
void zkm_profile_enable(int on);
void zkm_profile_reset(void);
size_t zkm_profile_dump(char *buf, size_t len);

/*
 * Machine blob (u32 words), produced by zkmips_amd/machine.py:
 *   'ZKMM' (0x4D4D4B5A), version 1, num_pv_elts, num_chips, then per chip:
 *     name_len, ceil(name_len/4) words of UTF-8 bytes (little-endian packing),
 *     prep_width, main_width, commit_scope (0 Local, 1 Global), local_only, log_quotient_degree,
 *     num_main_constraints, code_len, code[code_len]   (postfix AIR program, opcodes below),
 *     num_sends, num_receives, lookups (sends then receives):
 *       kind (LookupKind), scope (0 Local, 1 Global), num_values, VPC x num_values, VPC multiplicity
 *       VPC = num_terms, (col, weight) x num_terms, constant;  col bit31 = main, else preprocessed.
 *   Opcodes: 0 END, 1 MAIN_L c, 2 MAIN_N c, 3 PREP_L c, 4 PREP_N c, 5 CONST v, 6 PV i, 7 IS_FIRST,
 *            8 IS_LAST, 9 IS_TRANSITION, 10 ADD, 11 SUB, 12 MUL, 13 NEG, 14 EMIT (assert_zero),
 *            15 LET s (pop the top into value slot s), 16 GET s (push slot s).
 *   Shared subexpressions (the Rc-shared nodes of Plonky3's SymbolicExpression DAG, which
 *   get_symbolic_constraints returns) are defined once with LET, slots numbered 0, 1, 2, ... in
 *   order of definition, and read with GET after their definition; this keeps a chip's program
 *   linear in the size of its DAG (chained Poseidon2 layers, septic-extension products).  The JIT
 *   keeps slots in registers; the ZKM_NO_JIT interpreter in global scratch.
 */

#ifdef __cplusplus
}
#endif
#endif /* ZKM_HIP_H */
