/*
 * zkm_tracegen.h — device trace generation (libzkm_hip.so), SURVEY.md §8f row 2.
 *
 * Drop-in for the reference's native trace-row ABI, crates/core/machine/src/sys.rs:14-42 →
 * crates/core/machine/cpp/extern.cpp:6-37, which fills ONE row per call on the host:
 *
 *   cpu_event_to_row_koalabear(CpuEventFfi, shard, InstructionFfi, CpuCols*)      (include/cpu.hpp:37-108)
 *   add_sub_event_to_row_koalabear(const AluEvent*, AddSubCols*)                   (include/add_sub.hpp:26-39)
 *   memory_local_event_to_row_koalabear(const MemoryLocalEvent*, SingleMemoryLocal*) (include/memory_local.hpp:8-20)
 *   memory_global_event_to_row_koalabear(const MemoryInitializeFinalizeEvent*, bool, MemoryInitCols*)
 *                                                                                  (include/memory_global.hpp:9-43)
 *   syscall_event_to_row_koalabear(const SyscallEvent*, bool, SyscallCols*)        (include/syscall.hpp:8-16)
 *
 * and, beyond that ABI, the Global chip (the reference's Rust generate_trace, global/mod.rs:77-196), and
 * from the recursion machine's row ABI (crates/recursion/core/src/sys.rs:22-110) the Poseidon2WideDeg3
 *   poseidon2_wide_event_to_row_koalabear(const KoalaBear *input, KoalaBear *row, bool sbox_state)
 *   exp_reverse_bits_event_to_row_koalabear(const ExpReverseBitsEventFFI *, size_t i, ExpReverseBitsLenCols *)
 *
 * Here each entry point fills a WHOLE padded trace in GPU memory from an event array in GPU memory:
 * one thread per row, rows staged through LDS so the row-major trace is written in full cache
 * lines; padding rows get the chip's padding values, so the buffer needs no clearing.  The parts
 * the reference's Rust callers add around the row ABI are done on the device too: the Byte chip's
 * lookup multiplicities (`byte_mult`, the Byte chip's 65536 x 10 row-major main trace, added to with
 * atomics), the Program chip's multiplicities, and the cross-row columns of MemoryGlobalInit/Finalize
 * (`memory/global.rs:111-186`).  Output is canonical KoalaBear (the prover's ZKM_REPR_CANONICAL),
 * ready for zkm_prove_shard with ZKM_MEM_DEVICE.
 *
 * The event structs are the reference's #[repr(C)] layouts (cbindgen), so a Rust caller passes its
 * event vectors (after `.into()` for CpuEventFfi) byte for byte.  All pointers are device pointers;
 * `stream` is a hipStream_t (NULL = the null stream).  Calls are asynchronous on `stream` and return
 * ZKM_ERR_ARG for inconsistent sizes.
 */
#ifndef ZKM_TRACEGEN_H
#define ZKM_TRACEGEN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* MemoryReadRecord / MemoryWriteRecord / MemoryRecord (core/executor/src/events/memory.rs:12-19, :49-83) */
typedef struct { uint32_t value, shard, timestamp, prev_shard, prev_timestamp; } zkm_memory_read_record;
typedef struct { uint32_t value, shard, timestamp, prev_value, prev_shard, prev_timestamp; } zkm_memory_write_record;
typedef struct { uint32_t shard, timestamp, value; } zkm_memory_record;

/* OptionMemoryRecordEnum (events/cpu.rs:100-139): tag 0 Read, 1 Write, 2 None */
#define ZKM_RECORD_READ 0
#define ZKM_RECORD_WRITE 1
#define ZKM_RECORD_NONE 2
typedef struct {
    uint8_t tag;
    zkm_memory_read_record read;
    zkm_memory_write_record write;
} zkm_option_memory_record;  /* 48 bytes */

/* OptionU32 (core/executor/src/lib.rs:40-60): tag 0 Some, 1 None */
typedef struct { uint8_t tag; uint32_t value; } zkm_option_u32;

/* CpuEventFfi (events/cpu.rs:46-75), 280 bytes */
typedef struct {
    uint32_t clk, pc, next_pc, next_next_pc;
    uint32_t a;
    zkm_option_memory_record a_record;
    uint32_t b;
    zkm_option_memory_record b_record;
    uint32_t c;
    zkm_option_memory_record c_record;
    zkm_option_u32 hi;
    zkm_option_memory_record hi_record;
    zkm_option_memory_record memory_record;
    uint32_t exit_code;
} zkm_cpu_event_ffi;

/* InstructionFfi (core/executor/src/instruction.rs:29-45), 24 bytes; opcode = Opcode as u8 */
typedef struct {
    uint8_t opcode, op_a;
    uint32_t op_b, op_c;
    uint8_t imm_b, imm_c;
    zkm_option_u32 raw;
} zkm_instruction_ffi;

/* AluEvent (events/instr.rs:10-27), 28 bytes */
typedef struct { uint32_t pc, next_pc; uint8_t opcode; uint32_t hi, a, b, c; } zkm_alu_event;

/* MemoryLocalEvent (events/memory.rs:225-236), 28 bytes */
typedef struct { uint32_t addr; zkm_memory_record initial_mem_access, final_mem_access; } zkm_memory_local_event;

/* MemoryInitializeFinalizeEvent (events/memory.rs:135-148), 16 bytes */
typedef struct { uint32_t addr, value, shard, timestamp; } zkm_memory_init_final_event;

/* SyscallEvent (events/syscall.rs:8-29), 56 bytes */
typedef struct {
    uint32_t pc, next_pc, shard, clk;
    zkm_memory_write_record a_record;
    uint8_t a_record_is_real;
    uint32_t syscall_id, arg1, arg2;
} zkm_syscall_event;

/* GlobalLookupEvent (core/executor/src/events/global.rs:6-15), 32 bytes */
typedef struct { uint32_t message[7]; uint8_t is_receive; uint8_t kind; } zkm_global_lookup_event;

/* Trace widths (columns) of the chips filled here. */
#define ZKM_CPU_WIDTH 67
#define ZKM_ADD_SUB_WIDTH 19
#define ZKM_MEMORY_LOCAL_WIDTH 56      /* 4 SingleMemoryLocal of 14 per row (memory/local.rs:26) */
#define ZKM_MEMORY_GLOBAL_WIDTH 111
#define ZKM_SYSCALL_WIDTH 6
#define ZKM_GLOBAL_WIDTH 99
#define ZKM_BYTE_MULT_WIDTH 10         /* Byte chip main trace: 65536 rows x 10 (bytes/columns.rs) */

/* Cpu: rows [0, n) from events[i] with instruction program[(pc - pc_base) / 4] (Program::fetch),
 * rows [n, height) padding (imm_b = imm_c = is_rw_a = 1, cpu/trace.rs).  byte_mult (nullable): the
 * row's Byte lookups (shard/clk range checks, the register-access timestamp checks and op_a value
 * bytes, cpu/trace.rs:118-250).  program_mult (nullable, program_len x 1): +1 per executed
 * instruction (the Program chip's multiplicities, program/mod.rs:102-140). */
int zkm_cpu_events_to_trace(const zkm_cpu_event_ffi *events, uint64_t n, uint32_t shard,
                            const zkm_instruction_ffi *program, uint64_t program_len, uint32_t pc_base,
                            uint32_t *trace, uint64_t height, uint32_t *byte_mult, uint32_t *program_mult,
                            void *stream);

/* AddSub (alu/add_sub/mod.rs:82-163): AddOperation carries + the U8Range checks of both operands
 * and the sum into byte_mult (nullable). */
int zkm_add_sub_events_to_trace(const zkm_alu_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                                uint32_t *byte_mult, void *stream);

/* The other AluEvent chips, whose rows the reference fills in Rust (no C++ row ABI): Bitwise
 * (alu/bitwise/mod.rs:140-171, the byte op of every limb), Lt (alu/lt/mod.rs:179-263: the AND 0x7F
 * masks of both top bytes and the LTU comparison of the most significant differing byte), ShiftLeft
 * (alu/sll/mod.rs:200-260: U8Range of the result and carries; padding rows with shift_by_n_bits[0] =
 * shift_by_n_bytes[0] = bit_shift_multiplier = 1), ShiftRight (alu/sr/mod.rs:220-325: MSB of the operand,
 * ShrCarry of every byte, U8Range of the byte / bit results, carries and shifted bytes; padding rows with
 * shift_by_n_bits[0] = shift_by_n_bytes[0] = 1).  byte_mult (nullable) as above. */
#define ZKM_BITWISE_WIDTH 18
#define ZKM_LT_WIDTH 36
#define ZKM_SHIFT_LEFT_WIDTH 44
#define ZKM_SHIFT_RIGHT_WIDTH 71
int zkm_bitwise_events_to_trace(const zkm_alu_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                                uint32_t *byte_mult, void *stream);
int zkm_lt_events_to_trace(const zkm_alu_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                           uint32_t *byte_mult, void *stream);
int zkm_shift_left_events_to_trace(const zkm_alu_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                                   uint32_t *byte_mult, void *stream);
int zkm_shift_right_events_to_trace(const zkm_alu_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                                    uint32_t *byte_mult, void *stream);

/* BranchEvent (events/instr.rs:159-177, #[repr(C)]), 28 bytes */
typedef struct { uint32_t pc, next_pc, next_next_pc; uint8_t opcode; uint32_t a, b, c; } zkm_branch_event;
/* MemInstrEvent (events/instr.rs:112-135); its mem_access (a Rust enum MemoryRecordEnum, no fixed layout)
 * travels as an OptionMemoryRecordEnum with tag Read (loads) or Write (stores), as in CpuEventFfi; 84 bytes */
typedef struct {
    uint32_t shard, clk, pc, next_pc;
    uint8_t opcode;
    uint32_t a, b, c;
    zkm_option_memory_record mem_access;
    uint32_t prev_a_val;
} zkm_mem_instr_event;
#define ZKM_BRANCH_WIDTH 62
#define ZKM_MEMORY_INSTRS_WIDTH 79
/* Branch (control_flow/branch/trace.rs:85-130): the branch decision recomputed from opcode, a, b
 * (Executor::execute_branch), the word range checks of next_pc / next_next_pc, U8Range of both on the
 * rows not taken.  MemoryInstrs (memory/instructions/trace.rs:88-251): address b + c, its alignment and
 * range-check columns, the memory access (value, previous value, timestamp checks), the unsigned loaded
 * value and sign columns of LB / LH, the is-register-address test (LTU against 35 when the top three
 * address bytes are zero).  byte_mult (nullable) as above. */
int zkm_branch_events_to_trace(const zkm_branch_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                               uint32_t *byte_mult, void *stream);
int zkm_memory_instrs_events_to_trace(const zkm_mem_instr_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                                      uint32_t *byte_mult, void *stream);

/* JumpEvent (events/instr.rs:198-216, #[repr(C)]) and MovCondEvent (:283-301, #[repr(C)]), 28 bytes each */
typedef struct { uint32_t pc, next_pc, next_next_pc; uint8_t opcode; uint32_t a, b, c; } zkm_jump_event;
typedef struct { uint32_t pc, next_pc; uint8_t opcode; uint32_t a, b, c, prev_a; } zkm_movcond_event;
/* CompAluEvent (events/instr.rs:44-72; not #[repr(C)] there, so this is its field order with C layout):
 * the HI register write of MULT / MULTU (hi_record_is_real = 0 for MUL), 64 bytes */
typedef struct {
    uint32_t shard, clk, pc, next_pc;
    uint8_t opcode;
    uint32_t hi, a, b, c;
    zkm_memory_write_record hi_record;
    uint8_t hi_record_is_real;
} zkm_comp_alu_event;
#define ZKM_JUMP_WIDTH 66
#define ZKM_MOVCOND_WIDTH 32
#define ZKM_MUL_WIDTH 58
/* Jump (control_flow/jump/trace.rs:83-102) and MovCond (misc/mov_cond/mod.rs: IsZeroWordOperation of c)
 * record no Byte lookups.  Mul (alu/mul/mod.rs:218-318): the 64-bit product of the (sign-extended for
 * MULT) operands by byte limbs with carries, MSB of both top bytes, U16Range of the carries, U8Range of the
 * product bytes, and the HI write's access columns and timestamp checks. */
int zkm_jump_events_to_trace(const zkm_jump_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                             void *stream);
int zkm_movcond_events_to_trace(const zkm_movcond_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                                void *stream);
int zkm_mul_events_to_trace(const zkm_comp_alu_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                            uint32_t *byte_mult, void *stream);

#define ZKM_DIVREM_WIDTH 106
#define ZKM_CLO_CLZ_WIDTH 22
/* DivRem (alu/divrem/mod.rs:240-390) from CompAluEvents: quotient and remainder recomputed from b, c
 * (get_quotient_and_remainder, executor/src/utils.rs:33-43: c = 0 gives q = 0xFFFFFFFF, r = b; INT_MIN / -1
 * wraps), the is-zero / overflow word tests, |c|, |r|, max(1, |c|), c q + r by bytes with carries, the HI
 * write of DIV / DIVU; MSB of b, c, r, U8Range of q, r and the product bytes.  CloClz (alu/clo_clz/mod.rs:
 * 85-160) from AluEvents (a = the count): b or ~b, its shift by 31 - a, U8Range of it and LTU(a, 33); padding
 * rows clz(0) = 32.  Its SRL dependencies are ShiftRight events (zkm_shift_right_events_to_trace). */
int zkm_divrem_events_to_trace(const zkm_comp_alu_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                               uint32_t *byte_mult, void *stream);
int zkm_clo_clz_events_to_trace(const zkm_alu_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                                uint32_t *byte_mult, void *stream);

#define ZKM_SYSCALL_INSTRS_WIDTH 64
/* SyscallInstrs (syscall/instructions/trace.rs:82-162) from the shard's SyscallEvents (every syscall the
 * CPU executed): the syscall-id tests (IsZero against ENTER_UNCONSTRAINED, HINT_LEN, HALT, SYS_EXT_GROUP,
 * COMMIT, COMMIT_DEFERRED_PROOFS), the COMMIT word bitmap, the HALT / COMMIT_DEFERRED_PROOFS operand's
 * word range check; no Byte lookups. */
int zkm_syscall_instrs_events_to_trace(const zkm_syscall_event *events, uint64_t n, uint32_t *trace,
                                       uint64_t height, void *stream);

/* MiscEvent (events/instr.rs:236-260, #[repr(C)]), 60 bytes */
typedef struct {
    uint32_t shard, clk, pc, next_pc;
    uint8_t opcode;
    uint32_t a, b, c, prev_a;
    zkm_memory_write_record hi_record;
} zkm_misc_event;
#define ZKM_MISC_INSTRS_WIDTH 72
/* MiscInstrs (misc/others/trace.rs:81-262): SEXT / TEQ (sign bit and byte, a == b), EXT (lsb, msbd, the
 * shifted operand), INS (lsb, msb, the rotate / shift / sum chain), MADDU / MSUBU / MADD / MSUB (the product,
 * the (HI, LO) addend, the 64-bit AddDouble with its carries, the HI write), their Byte lookups. */
int zkm_misc_instrs_events_to_trace(const zkm_misc_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                                    uint32_t *byte_mult, void *stream);

/* ShaExtend (syscall/precompiles/sha256/extend/trace.rs:29-150): ShaExtendEvent holds Vecs (one read of
 * w[i-15], w[i-2], w[i-16], w[i-7] and one write of w[i] per step i = 16..63), so its rows travel flattened,
 * one record per step in call order (48 per call): the call's shard, clk and w_ptr, the four reads, the write.
 * Every row gets the 16/48-cycle flags (flags.rs:13-34), real rows the access columns, the rotate / shift
 * carries (ShrCarry lookups), the XORs and the Add4 of w[i-16] + s0 + w[i-7] + s1 (U8 range checks). */
typedef struct {
    uint32_t shard, clk, w_ptr;
    zkm_memory_read_record w_i_minus_15, w_i_minus_2, w_i_minus_16, w_i_minus_7;
    zkm_memory_write_record w_i;
} zkm_sha_extend_row;  /* 116 bytes */
#define ZKM_SHA_EXTEND_WIDTH 176
int zkm_sha_extend_events_to_trace(const zkm_sha_extend_row *rows, uint64_t n, uint32_t *trace, uint64_t height,
                                   uint32_t *byte_mult, void *stream);

/* Uint256MulMod (syscall/precompiles/uint256/air.rs:103-186): Uint256MulEvent as one fixed record: shard, clk,
 * x_ptr, y_ptr, the 8 reads of y and the 8 reads of the modulus (at clk), the 8 writes of x (at clk + 1; each
 * prev_value a word of x).  Each row: the accesses, IsZeroOperation of the modulus's byte sum, FieldOpCols of
 * x y mod m (2^256 when m = 0: result, carry, the vanishing polynomial's witness limbs), FieldLtCols
 * result < m when m != 0; padding rows multiply zeros modulo 2^256.  byte_mult (nullable): the U8 range
 * checks of the FieldOpCols limbs, the LTU comparison and the accesses' range checks.  480 columns. */
typedef struct {
    uint32_t shard, clk, x_ptr, y_ptr;
    zkm_memory_read_record y[8], modulus[8];
    zkm_memory_write_record x[8];
} zkm_uint256_mul_event;  /* 528 bytes */
#define ZKM_UINT256_MUL_WIDTH 480
int zkm_uint256_mul_events_to_trace(const zkm_uint256_mul_event *events, uint64_t n, uint32_t *trace,
                                    uint64_t height, uint32_t *byte_mult, void *stream);

/* U256XU2048Mul (syscall/precompiles/u256x2048_mul/air.rs:109-213): U256xU2048MulEvent as one fixed record:
 * shard, clk, a_ptr, b_ptr, lo_ptr, hi_ptr, the A2 / A3 register reads, the 8 reads of a and 64 of b (at
 * clk), the 64 writes of lo and 8 of hi (at clk + 1).  Each row: the accesses and the eight FieldOpCols
 * mul-and-carry operations a b_k + carry = lo_k + carry' 2^256 (field_op.rs populate_mul_and_carry); padding
 * rows hold them for zeros.  byte_mult (nullable): the limbs' U8 and the accesses' range checks.  3129
 * columns. */
typedef struct {
    uint32_t shard, clk, a_ptr, b_ptr, lo_ptr, hi_ptr;
    zkm_memory_read_record lo_ptr_reg, hi_ptr_reg, a[8], b[64];
    zkm_memory_write_record lo[64], hi[8];
} zkm_u256x2048_mul_event;  /* 3232 bytes */
#define ZKM_U256XU2048_MUL_WIDTH 3129
int zkm_u256x2048_mul_events_to_trace(const zkm_u256x2048_mul_event *events, uint64_t n, uint32_t *trace,
                                      uint64_t height, uint32_t *byte_mult, void *stream);

/* FpOpAssign of the bn254 / bls12-381 base fields (syscall/precompiles/fptower/fp.rs:90-160): FpOpEvent as
 * one fixed record: shard, clk, x_ptr, y_ptr, op (0 add, 1 sub, 2 mul), the reads of y (at clk) and the
 * writes of x (at clk + 1) -- 8 words each for bn254, 12 for bls12-381, in slots of 12.  Each row: op flags,
 * the accesses, FieldOpCols of x op y mod p (sub populated as r + y, field_op.rs populate_with_modulus);
 * padding rows are 0 + 0.  byte_mult (nullable): the limbs' U8 and the accesses' range checks.  372 (bn254)
 * or 556 (bls12-381) columns. */
#define ZKM_FIELD_BN254 0
#define ZKM_FIELD_BLS12381 1
typedef struct {
    uint32_t shard, clk, x_ptr, y_ptr, op;
    zkm_memory_read_record y[12];
    zkm_memory_write_record x[12];
} zkm_fp_op_event;  /* 548 bytes */
#define ZKM_FP_OP_WIDTH_BN254 372
#define ZKM_FP_OP_WIDTH_BLS12381 556
int zkm_fp_op_events_to_trace(int field, const zkm_fp_op_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                              uint32_t *byte_mult, void *stream);

/* Fp2AddSubAssign / Fp2MulAssign of the bn254 / bls12-381 quadratic extensions (fptower/fp2_addsub.rs:93-183,
 * fp2_mul.rs:122-210): one fixed record per call: shard, clk, x_ptr, y_ptr, op (0 add, 1 sub; unused for mul),
 * the reads of y = (y0, y1) at clk and the writes of x = (x0, x1) at clk + 1 (16 words for bn254, 24 for
 * bls12-381, in slots of 24).  Rows: AddSub c0 = x0 +- y0, c1 = x1 +- y1 (two FieldOpCols), Mul a0 b0, a1 b1,
 * a0 b1, a1 b0 and c0 = a0 b0 - a1 b1, c1 = a0 b1 + a1 b0 (six); padding rows the operations on zeros.
 * byte_mult (nullable): the limbs' U8 and the accesses' range checks.  mul: 0 AddSub, 1 Mul. */
typedef struct {
    uint32_t shard, clk, x_ptr, y_ptr, op;
    zkm_memory_read_record y[24];
    zkm_memory_write_record x[24];
} zkm_fp2_event;  /* 1076 bytes */
int zkm_fp2_events_to_trace(int field, int mul, const zkm_fp2_event *events, uint64_t n, uint32_t *trace,
                            uint64_t height, uint32_t *byte_mult, void *stream);

/* WeierstrassAddAssign on secp256k1 / secp256r1 / bn254 / bls12-381 (weierstrass/weierstrass_add.rs:192-252,
 * :384-420): EllipticCurveAddEvent as one fixed record: shard, clk, p_ptr, q_ptr, the reads of q at clk and
 * the writes of p at clk + 1 (16 words for the 256-bit curves, 24 for bls12-381, in slots of 24).  Each row:
 * the accesses and the nine FieldOpCols of the affine addition (the slope by a modular inverse on the
 * device); padding rows the operations on zero inputs.  byte_mult (nullable) as above. */
#define ZKM_CURVE_SECP256K1 0
#define ZKM_CURVE_SECP256R1 1
#define ZKM_CURVE_BN254 2
#define ZKM_CURVE_BLS12381 3
typedef struct {
    uint32_t shard, clk, p_ptr, q_ptr;
    zkm_memory_read_record q[24];
    zkm_memory_write_record p[24];
} zkm_ec_add_event;  /* 1072 bytes */
int zkm_ec_add_events_to_trace(int curve, const zkm_ec_add_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                               uint32_t *byte_mult, void *stream);

/* WeierstrassDoubleAssign on the same curves (weierstrass/weierstrass_double.rs:201-270, :411-440):
 * EllipticCurveDoubleEvent as one fixed record: shard, clk, p_ptr, the writes of p at clk (16 or 24 words, in
 * slots of 24).  Each row: the accesses and the eleven FieldOpCols of the affine doubling; padding rows: the
 * operations of p = (0, 1) and the dummy write record of y's first word.  byte_mult (nullable) as above. */
typedef struct {
    uint32_t shard, clk, p_ptr;
    zkm_memory_write_record p[24];
} zkm_ec_double_event;  /* 588 bytes */
int zkm_ec_double_events_to_trace(int curve, const zkm_ec_double_event *events, uint64_t n, uint32_t *trace,
                                  uint64_t height, uint32_t *byte_mult, void *stream);

/* WeierstrassDecompress on secp256k1 / secp256r1 / bls12-381 (weierstrass/weierstrass_decompress.rs:161-303):
 * EllipticCurveDecompressEvent as one fixed record: shard, clk, ptr, sign, the reads of x (at ptr + nl) and
 * the writes of y (at ptr), both at clk (8 or 12 words, in slots of 12).  Each row: the accesses, x < p,
 * x^2, x^3, a x + b, the square root of x^3 + a x + b (a^((p+1)/4) on the device), its range and lsb, -y,
 * and for bls12-381 the lexicographic choice columns; padding rows decompress the generator's x.  byte_mult
 * (nullable) as above. */
typedef struct {
    uint32_t shard, clk, ptr, sign;
    zkm_memory_read_record x[12];
    zkm_memory_write_record y[12];
} zkm_ec_decompress_event;  /* 544 bytes */
int zkm_ec_decompress_events_to_trace(int curve, const zkm_ec_decompress_event *events, uint64_t n, uint32_t *trace,
                                      uint64_t height, uint32_t *byte_mult, void *stream);

/* EdAddAssign (syscall/precompiles/edwards/ed_add.rs:111-238): the Ed25519 EllipticCurveAddEvent as one fixed
 * record: shard, clk, p_ptr, q_ptr, the 16 reads of q at clk, the 16 writes of p at clk + 1.  Each row: the
 * accesses, the two FieldInnerProductCols of the numerators, four FieldOpCols (x1 y1, x2 y2, f, d f) and the
 * two FieldDenCols of x3 and y3 (inverses on the device); padding rows the operations on zero inputs.
 * byte_mult (nullable) as above.  1861 columns. */
typedef struct {
    uint32_t shard, clk, p_ptr, q_ptr;
    zkm_memory_read_record q[16];
    zkm_memory_write_record p[16];
} zkm_ed_add_event;  /* 720 bytes */
#define ZKM_ED_ADD_WIDTH 1861
int zkm_ed_add_events_to_trace(const zkm_ed_add_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                               uint32_t *byte_mult, void *stream);

/* EdDecompress (syscall/precompiles/edwards/ed_decompress.rs:64-101, :214-247): EdDecompressEvent as one fixed
 * record: shard, clk, ptr, sign, the 8 reads of y (at ptr + 32) and the 8 writes of x (at ptr), both at clk.
 * Each row: the accesses, y < p, y^2, u, d y^2, v, u / v, its square root (lsb 0, ed25519.rs:75-113) as
 * FieldSqrtCols with range and lsb, -x; padding rows the operations of y = 0.  byte_mult (nullable) as
 * above.  1566 columns. */
typedef struct {
    uint32_t shard, clk, ptr, sign;
    zkm_memory_read_record y[8];
    zkm_memory_write_record x[8];
} zkm_ed_decompress_event;  /* 368 bytes */
#define ZKM_ED_DECOMPRESS_WIDTH 1566
int zkm_ed_decompress_events_to_trace(const zkm_ed_decompress_event *events, uint64_t n, uint32_t *trace,
                                      uint64_t height, uint32_t *byte_mult, void *stream);

/* KeccakSponge (syscall/precompiles/keccak_sponge/trace.rs:62-196): KeccakSpongeEvent holds Vecs, so it travels
 * as one record per absorbed block: the call's shard, clk, this block's input address, the output address,
 * the input length (words), the block's index and the call's block count, the xored state after absorbing
 * this block and the previous block's (zero for the first; the original state is its Keccak-f, computed on
 * the device), the block's 36 input reads, the length read, the 16 output writes (at clk + 1).  24 rows per
 * block (the p3-keccak-air round columns and the sponge columns); padding rows the zero input's rounds.
 * byte_mult (nullable): the XORs of the rate and the accesses' range checks.  3531 columns. */
typedef struct {
    uint32_t shard, clk, in_ptr, out_ptr, in_len, block, nblocks;
    uint32_t xored[50], prev_xored[50];
    zkm_memory_read_record in[36], len;
    zkm_memory_write_record out[16];
} zkm_keccak_block;  /* 1552 bytes */
#define ZKM_KECCAK_SPONGE_WIDTH 3531
int zkm_keccak_sponge_events_to_trace(const zkm_keccak_block *blocks, uint64_t n, uint32_t *trace, uint64_t height,
                                      uint32_t *byte_mult, void *stream);

/* SysLinux (syscall/precompiles/sys_linux/trace.rs:106-167): LinuxEvent as one fixed record: the call's
 * shard, clk, syscall code, a0, a1, the value returned in V0; the A3 (error) write; `io`: the brk register
 * read (BRK), the A2 read (WRITE; a read as a write record with prev_value = value), the heap write (MMAP /
 * MMAP2 with a0 = 0), unused otherwise.  One row per call (flags per syscall kind, GtColsBytes of BRK);
 * rows [n, height) zero.  byte_mult (nullable): the accesses' timestamp range checks and BRK's LTU / U8
 * lookups.  69 columns. */
typedef struct {
    uint32_t shard, clk, code, a0, a1, result;
    zkm_memory_write_record a3, io;
} zkm_sys_linux_event;  /* 72 bytes */
#define ZKM_SYS_LINUX_WIDTH 69
int zkm_sys_linux_events_to_trace(const zkm_sys_linux_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                                  uint32_t *byte_mult, void *stream);

/* Poseidon2Permute (syscall/precompiles/poseidon2/trace.rs event_to_row, columns.rs Poseidon2MemCols):
 * Poseidon2PermuteEvent as one fixed record: the call's shard, clk and state pointer, the 16 state words'
 * MemoryWriteRecords (prev_value = the word permuted, value = the permutation's output word).  Each row:
 * Poseidon2Degree3Cols of the permutation (the PermutationSBox layout of Poseidon2WideDeg3 above), shard,
 * clk, ptr, 16 MemoryWriteCols, the KoalaBearWordRangeChecker of every pre- and post-state word, is_real;
 * rows [n, height) the permutation of zero and zero elsewhere.  byte_mult (nullable): the accesses'
 * timestamp range checks (U16Range, U8Range).  973 columns. */
typedef struct {
    uint32_t shard, clk, ptr;
    zkm_memory_write_record state[16];
} zkm_poseidon2_permute_event;  /* 396 bytes */
#define ZKM_POSEIDON2_PERMUTE_WIDTH 973
int zkm_poseidon2_permute_events_to_trace(const zkm_poseidon2_permute_event *events, uint64_t n, uint32_t *trace,
                                          uint64_t height, uint32_t *byte_mult, void *stream);

/* ShaCompress (syscall/precompiles/sha256/compress/trace.rs:32-305): ShaCompressEvent's records (its w is a
 * Vec) as one fixed record per call: shard, clk, w_ptr, h_ptr, the 8 reads of h, the 64 reads of w, the 8
 * writes of h.  80 rows per call (init, 64 rounds, finalize): the round state is expanded on the device, then
 * every row gets its octet flags, access, state words, the Sigma rotations (ShrCarry), the ch / maj
 * AND / XOR bytes, the Add5 of temp1, the adds of temp2, d + temp1, temp1 + temp2 and the finalize add. */
typedef struct {
    uint32_t shard, clk, w_ptr, h_ptr;
    zkm_memory_read_record h_read_records[8];
    zkm_memory_read_record w_i_read_records[64];
    zkm_memory_write_record h_write_records[8];
} zkm_sha_compress_event;  /* 1648 bytes */
#define ZKM_SHA_COMPRESS_WIDTH 262
int zkm_sha_compress_events_to_trace(const zkm_sha_compress_event *events, uint64_t n, uint32_t *trace,
                                     uint64_t height, uint32_t *byte_mult, void *stream);

/* MemoryLocal (memory/local.rs:144-185): event i fills entry i % 4 of row i / 4; height rows. */
int zkm_memory_local_events_to_trace(const zkm_memory_local_event *events, uint64_t n, uint32_t *trace,
                                     uint64_t height, void *stream);

/* MemoryGlobalInit (is_receive = 0) / MemoryGlobalFinalize (1) (memory/global.rs:111-186): events
 * sorted by strictly increasing addr, all above prev_addr (the shard's previous_*_addr public value,
 * 0 for none) — the precondition the reference establishes with sort_by_key. */
int zkm_memory_global_events_to_trace(const zkm_memory_init_final_event *events, uint64_t n, int is_receive,
                                      uint32_t prev_addr, uint32_t *trace, uint64_t height, void *stream);

/* SyscallCore / SyscallPrecompile (syscall/chip.rs:138-183). */
int zkm_syscall_events_to_trace(const zkm_syscall_event *events, uint64_t n, int is_receive, uint32_t *trace,
                                uint64_t height, void *stream);

/* Global (global/mod.rs:77-196): each message lifted onto the septic curve y^2 = x^3 + 3z x - 3 over
 * F_p[z]/(z^7 + 2z - 8) with the smallest offset (GlobalLookupOperation::populate), the running sum
 * of the points from the zero digest as a parallel scan (the reference's par_iter().scan), padding
 * rows with the dummy point, U16Range(message[0]) into byte_mult (nullable).  final_digest (device,
 * nullable): the shard's global cumulative sum, 14 canonical words (x then y).  Synchronises `stream`
 * before returning; ZKM_ERR_UNSATISFIED if a message has no lift, the running sum reaches infinity
 * or message[0] is not 16-bit. */
int zkm_global_events_to_trace(const zkm_global_lookup_event *events, uint64_t n, uint32_t *trace,
                               uint64_t height, uint32_t *byte_mult, uint32_t *final_digest, void *stream);

/* ---- recursion machine (crates/recursion/core/src/sys.rs:22-110, include/poseidon2_wide.hpp) ---- */
#define ZKM_POSEIDON2_WIDE_DEG3_WIDTH 313  /* PermutationSBox (poseidon2_wide/columns/permutation.rs:20-72) */

/* Poseidon2Io<KoalaBear> = Poseidon2Event (recursion/core/src/lib.rs): input[16] then output[16] */
typedef struct {
    uint32_t input[16];
    uint32_t output[16];
} zkm_poseidon2_event;

/* Poseidon2WideDeg3 main trace: poseidon2_wide_event_to_row_koalabear(input, row, sbox_state = true)
 * (sys.rs:102-106, include/poseidon2_wide.hpp) for every event, rows [n, height) the permutation of
 * zero (poseidon2_wide/trace.rs dummy row).  repr: ZKM_REPR_MONTGOMERY for a Rust
 * Vec<Poseidon2Event<KoalaBear>> as it lies in memory, or ZKM_REPR_CANONICAL.  The output words are
 * not read (the permutation is recomputed). */
int zkm_poseidon2_wide_events_to_trace(const zkm_poseidon2_event *events, uint64_t n, uint32_t repr,
                                       uint32_t *trace, uint64_t height, void *stream);

#define ZKM_EXP_REVERSE_BITS_LEN_WIDTH 7  /* ExpReverseBitsLenCols (exp_reverse_bits.rs:44-53) */

/* ExpReverseBitsLen main trace: exp_reverse_bits_event_to_row_koalabear (sys.rs:50-54,
 * include/exp_reverse_bits.hpp) plus the accumulator columns the Rust caller fills around it
 * (exp_reverse_bits.rs:216-270): event e = (base[e], the bits at bits[offsets[e] .. offsets[e + 1]])
 * fills rows offsets[e] .. offsets[e + 1] - 1 (x, current_bit, prev_accum_squared,
 * prev_accum_squared_times_multiplier, accum, accum_squared, multiplier); rows from offsets[n] on are
 * zero.  offsets has n + 1 entries, offsets[0] = 0, offsets[n] <= height.  repr as above. */
int zkm_exp_reverse_bits_events_to_trace(const uint32_t *base, const uint32_t *bits, const uint64_t *offsets,
                                         uint64_t n, uint32_t repr, uint32_t *trace, uint64_t height, void *stream);

/* Recursion chips whose main rows are their events (cols.vals = event), several events per row for the
 * memory and ALU chips:
 *   BaseAlu      alu_base_event_to_row_koalabear   (sys.rs:22-25, include/alu_base.hpp)   3 words x 4 per row
 *   ExtAlu       alu_ext_event_to_row_koalabear    (sys.rs:31-34, include/alu_ext.hpp)   12 words x 4 per row
 *   BatchFRI     batch_fri_event_to_row_koalabear  (sys.rs:40-43, include/batch_fri.hpp) 13 words (acc[4],
 *                alpha_pow[4], p_at_z[4], p_at_x) x 1
 *   Select       select_event_to_row_koalabear     (sys.rs:83-86, include/select.hpp)     5 words x 1
 *   FriFold      fri_fold_event_to_row_koalabear   (sys.rs:62-65, include/fri_fold.hpp)  33 words x 1
 *   PublicValues public_values_event_to_row_koalabear (sys.rs:72-76, include/public_values.hpp): the
 *                digest's 8 elements, 1 word x 1
 *   MemoryVar    mem/variable.rs generate_trace: a hinted block, 4 words x 2 per row
 *   MemoryConst  mem/constant.rs generate_trace: main width 1, all zero (n = 0)
 * `events` holds n events of the chip's width back to back; row r gets events r*k .. r*k + k - 1 side by side;
 * rows past the events are zero (the chips' padding rows).  repr as above (the words are converted to
 * canonical on the way).  ZKM_ERR_ARG for an unknown chip, n events not fitting height rows, or a
 * height that is not a power of two >= 16. */
#define ZKM_REC_CHIP_BASE_ALU 0
#define ZKM_REC_CHIP_EXT_ALU 1
#define ZKM_REC_CHIP_BATCH_FRI 2
#define ZKM_REC_CHIP_SELECT 3
#define ZKM_REC_CHIP_FRI_FOLD 4
#define ZKM_REC_CHIP_PUBLIC_VALUES 5
#define ZKM_REC_CHIP_MEMORY_VAR 6
#define ZKM_REC_CHIP_MEMORY_CONST 7
int zkm_recursion_events_to_trace(uint32_t chip, const uint32_t *events, uint64_t n, uint32_t repr, uint32_t *trace,
                                  uint64_t height, void *stream);

/* Preprocessed traces of the recursion chips: the *_instr_to_row_koalabear functions of sys.rs:22-110
 * (include/alu_base.hpp, alu_ext.hpp, batch_fri.hpp, select.hpp, fri_fold.hpp, public_values.hpp,
 * exp_reverse_bits.hpp, poseidon2_wide.hpp; mem/{constant,variable}.rs) from n instruction records of
 * u32 words, field words in `repr`, integer words (opcodes, flags, indices) plain:
 *   BaseAlu / ExtAlu   5: addr out, in1, in2, opcode (0 add, 1 sub, 2 mul, 3 div), mult  -> 4 per row, 32 cols
 *   BatchFRI           5 per row: acc, alpha_pow, p_at_z, p_at_x addrs, is_end           -> 6 cols
 *   Select             7: bit, out1, out2, in1, in2 addrs, mult1, mult2                   -> 8 cols
 *   FriFold           12 per row: z, alpha, x, alpha_pow_in, ro_in, p_at_x, p_at_z, ro_out addrs, ro mult,
 *                      alpha_pow_out addr, alpha_pow mult, is_first                       -> 20 cols
 *   PublicValues       1: the digest element's address (n <= 8)                           -> 10 cols
 *   MemoryVar          2: addr, mult                                                      -> 2 per row, 4 cols
 *   MemoryConst        6: value[4], addr, mult (negative for a read)                      -> 2 per row, 12 cols
 *   ExpReverseBitsLen  6 per row: base addr, exponent-bit addr, result addr, mult, row index i, length L
 *                                                                                          -> 10 cols
 *   Poseidon2WideDeg3 48: input addrs[16], output addrs[16], output mults[16]             -> 49 cols
 * Rows past the records are zero. */
#define ZKM_REC_CHIP_EXP_REVERSE_BITS 8
#define ZKM_REC_CHIP_POSEIDON2_WIDE 9
int zkm_recursion_instrs_to_trace(uint32_t chip, const uint32_t *instrs, uint64_t n, uint32_t repr, uint32_t *trace,
                                  uint64_t height, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* ZKM_TRACEGEN_H */
