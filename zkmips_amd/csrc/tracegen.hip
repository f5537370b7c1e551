// Device trace generation: the reference's per-row trace ABI (crates/core/machine/src/sys.rs:14-42,
// cpp/extern.cpp:6-37, include/*.hpp) as whole-trace HIP kernels.  See include/zkm_tracegen.h.
//
// Every kernel is the same streaming shape, HBM-bound (no arithmetic worth the name): a workgroup
// of 128 threads owns 128 consecutive trace rows.  (1) The block's events are copied into LDS with
// coalesced dword loads (events are 16-280 byte structs; one thread per event would make every load
// instruction touch 64 cache lines).  (2) Each thread builds its row in registers from its event —
// the reference's event_to_row — and adds its Byte-chip lookups (wave-aggregated atomics: most
// lookups of a wave hit the same entry, e.g. the shard's U16 range check).  (3) The rows go back
// through LDS (odd pitch: conflict-free) and leave as full-line 16-byte stores of the block's
// contiguous row-major span.  Padding rows are written too, so the output needs no clearing.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "../../include/zkm_hip.h"
#include "../../include/zkm_tracegen.h"
#include "kb31.cuh"
#include "p2_rows.cuh"

namespace zkm {
extern thread_local std::string g_last_error;
}
using zkm::g_last_error;

static_assert(sizeof(zkm_option_memory_record) == 48, "OptionMemoryRecordEnum layout");
static_assert(sizeof(zkm_cpu_event_ffi) == 280, "CpuEventFfi layout");
static_assert(sizeof(zkm_instruction_ffi) == 24, "InstructionFfi layout");
static_assert(sizeof(zkm_alu_event) == 28, "AluEvent layout");
static_assert(sizeof(zkm_memory_local_event) == 28, "MemoryLocalEvent layout");
static_assert(sizeof(zkm_memory_init_final_event) == 16, "MemoryInitializeFinalizeEvent layout");
static_assert(sizeof(zkm_syscall_event) == 56, "SyscallEvent layout");
static_assert(sizeof(zkm_branch_event) == 28, "BranchEvent layout");
static_assert(sizeof(zkm_mem_instr_event) == 84, "MemInstrEvent layout");
static_assert(sizeof(zkm_jump_event) == 28, "JumpEvent layout");
static_assert(sizeof(zkm_movcond_event) == 28, "MovCondEvent layout");
static_assert(sizeof(zkm_comp_alu_event) == 64, "CompAluEvent layout");
static_assert(sizeof(zkm_misc_event) == 60, "MiscEvent layout");
static_assert(sizeof(zkm_sha_extend_row) == 116, "ShaExtend row record layout");
static_assert(sizeof(zkm_sha_compress_event) == 1648, "ShaCompress call record layout");

namespace zkm::tg {

constexpr uint32_t P = 0x7f000001u;
constexpr int NTH = 128;  // rows per workgroup

// Opcode (core/executor/src/opcode.rs:15-75)
enum Op : uint32_t {
    ADD = 0, SUB = 1, MULT = 3, MULTU = 4, DIV = 5, DIVU = 6,
    BEQ = 21, BGEZ = 22, BGTZ = 23, BLEZ = 24, BLTZ = 25, BNE = 26, JUMP = 27, JUMPI = 28, JUMPDIRECT = 29,
    SYSCALL = 30, LB = 31, LBU = 32, LH = 33, LHU = 34, LW = 35, LWL = 36, LWR = 37, LL = 38,
    SB = 39, SH = 40, SW = 41, SWL = 42, SWR = 43, SC = 44, INS = 45, MADDU = 46, MSUBU = 47, MADD = 48,
    MSUB = 49, MEQ = 50, MNE = 51,
};
// ByteOpcode (core/executor/src/events/byte.rs) and the Byte chip's multiplicity columns
constexpr uint32_t B_U8RANGE = 4, B_U16RANGE = 8, BYTE_COLS = ZKM_BYTE_MULT_WIDTH;
constexpr uint32_t SYS_EXT_GROUP = 4246;  // SyscallCode::SYS_EXT_GROUP (syscalls/code.rs:154)

// instruction predicates (include/instruction.hpp)
__device__ __forceinline__ bool is_branch(uint32_t op) { return op >= BEQ && op <= BNE; }
__device__ __forceinline__ bool is_jump(uint32_t op) { return op >= JUMP && op <= JUMPDIRECT; }
__device__ __forceinline__ bool is_mem(uint32_t op) { return op >= LB && op <= SC; }
__device__ __forceinline__ bool is_store_except_sc(uint32_t op) { return op >= SB && op <= SWR; }
__device__ __forceinline__ bool is_maddsub(uint32_t op) { return op >= MADDU && op <= MSUB; }
__device__ __forceinline__ bool is_mult_div(uint32_t op) { return op == MULT || op == MULTU || op == DIV || op == DIVU; }
__device__ __forceinline__ bool is_check_memory(uint32_t op) { return op == SYSCALL || is_maddsub(op) || is_mem(op); }
__device__ __forceinline__ bool is_rw_a(uint32_t op) {
    return op == SYSCALL || op == INS || is_maddsub(op) || op == MEQ || op == MNE || is_mem(op);
}

__device__ __forceinline__ uint32_t byte_of(uint32_t x, int i) { return (x >> (8 * i)) & 0xFF; }
__device__ __forceinline__ void put_word(uint32_t *v, uint32_t x) {  // write_word_from_u32_v2
#pragma unroll
    for (int i = 0; i < 4; i++) v[i] = byte_of(x, i);
}

// Lookup multiplicities (the Byte chip's 65536 x 10 counts, the Program chip's per-instruction
// counts).  Real traces are skewed — a shard's lookups hit few distinct entries (zero bytes, small
// timestamp gaps, the shard number) — so global atomics straight from every lane serialise on those
// entries.  Instead each workgroup (persistent, looping over row tiles) accumulates into an LDS hash
// table, after merging the lanes of a wave that agree with the first active lane; the table is
// flushed once per workgroup with one global atomic per distinct key.  Keys that find no slot within
// a few probes, and lookups known to be spread out (the 16-bit clk limb), go to global memory directly.
constexpr uint32_t LOG_HS = 11, HS = 1u << LOG_HS, EMPTY = 0xFFFFFFFFu, PROG_KEY = 0x80000000u;

struct Hist {
    uint32_t *keys, *vals;             // LDS, HS each (null when the chip records no lookups)
    uint32_t *byte_mult, *program_mult;  // global, nullable

    __device__ __forceinline__ void global_add(uint32_t key, uint32_t cnt) const {
        if (key & PROG_KEY) {
            if (program_mult) atomicAdd(program_mult + (key & ~PROG_KEY), cnt);
        } else if (byte_mult) {
            atomicAdd(byte_mult + key, cnt);
        }
    }
    __device__ __forceinline__ void insert(uint32_t key, uint32_t cnt) const {
        uint32_t h = (key * 2654435761u) >> (32 - LOG_HS);
#pragma unroll 1
        for (int p = 0; p < 8; p++) {
            const uint32_t k = atomicCAS(keys + h, EMPTY, key);
            if (k == EMPTY || k == key) {
                atomicAdd(vals + h, cnt);
                return;
            }
            h = (h + 1) & (HS - 1);
        }
        global_add(key, cnt);
    }
    // +1 at `key` for every lane with `on`; called by every lane of the wave (ballots)
    __device__ __forceinline__ void add(uint32_t key, bool on) const {
        const uint64_t act = __ballot(on);
        if (act == 0) return;
        const int leader = __ffsll((unsigned long long)act) - 1;
        const uint32_t lead = __shfl(key, leader);
        const uint64_t same = __ballot(on && key == lead);
        if ((int)(threadIdx.x & 63) == leader) insert(lead, (uint32_t)__popcll(same));
        if (on && key != lead) insert(key, 1u);
    }
    __device__ __forceinline__ void direct(uint32_t key, bool on) const {
        if (on) global_add(key, 1u);
    }
    __device__ __forceinline__ void byte(uint32_t op, uint32_t b, uint32_t c, bool on) const {
        if (byte_mult) add(((b << 8) | c) * BYTE_COLS + op, on);
    }
};

// Persistent workgroups over tiles of NTH rows: (1) the tile's events -> LDS (pitch EP dwords),
// (2) chip.row(v, event or nullptr, row, hist) per thread, (3) rows -> LDS (pitch W|1) -> 16-byte
// coalesced stores.  EVS: event stride in dwords, EVW: the leading dwords the row needs.
template <int EVS, int EVW, int W>
struct Tile {
    static constexpr int EP = EVW | 1, RP = W | 1;
    static constexpr int WORDS = NTH * (EP > RP ? EP : RP);
};

constexpr int WIDE_ROW = 128;  // rows wider than this are built in LDS, not registers

template <int EVS, int EVW, int W, bool HIST, class Chip>
__global__ __launch_bounds__(NTH) void k_events_to_rows(const uint32_t *__restrict__ ev, uint64_t n,
                                                        uint32_t *__restrict__ out, uint64_t nrows, Chip chip,
                                                        uint32_t *byte_mult, uint32_t *program_mult) {
    using T = Tile<EVS, EVW, W>;
    __shared__ uint32_t buf[T::WORDS];
    __shared__ uint32_t hkeys[HIST ? HS : 1], hvals[HIST ? HS : 1];
    const uint32_t t = threadIdx.x;
    Hist hist{hkeys, hvals, byte_mult, program_mult};
    if constexpr (HIST) {
        for (uint32_t i = t; i < HS; i += NTH) {
            hkeys[i] = EMPTY;
            hvals[i] = 0;
        }
    }
    const uint64_t ntiles = (nrows + NTH - 1) / NTH;
    for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const uint64_t row0 = tile * NTH;
        const uint32_t rows = (uint32_t)min<uint64_t>(NTH, nrows - row0);
        const uint32_t nev = n > row0 ? (uint32_t)min<uint64_t>(rows, n - row0) : 0u;
        const uint32_t *src = ev + row0 * EVS;
        __syncthreads();  // the previous tile's stores have read buf; the table is initialised
        if constexpr (EVS == EVW) {
            for (uint32_t i = t; i < nev * EVW; i += NTH) {
                const uint32_t r = i / EVW;
                buf[r * T::EP + (i - r * EVW)] = src[i];
            }
        } else {
            for (uint32_t i = t; i < nev * EVW; i += NTH) {
                const uint32_t r = i / EVW, k = i - r * EVW;
                buf[r * T::EP + k] = src[(uint64_t)r * EVS + k];
            }
        }
        __syncthreads();
        if constexpr (W > WIDE_ROW) {
            // wide rows (ShaExtend 176, ShaCompress 262 columns) would not fit in registers: the thread takes
            // its event into registers, then the chip writes the row straight into the LDS tile
            uint32_t ev[EVW];
            if (t < nev) {
#pragma unroll
                for (int k = 0; k < EVW; k++) ev[k] = buf[t * T::EP + k];
            }
            __syncthreads();
            chip.row(buf + t * T::RP, t < nev ? ev : nullptr, row0 + t, hist);
        } else {
            uint32_t v[W];
            chip.row(v, t < nev ? buf + t * T::EP : nullptr, row0 + t, hist);
            __syncthreads();
            if (t < rows) {
#pragma unroll
                for (int c = 0; c < W; c++) buf[t * T::RP + c] = v[c];
            }
        }
        __syncthreads();
        uint32_t *dst = out + row0 * W;
        const uint32_t total = rows * W;  // rows is a multiple of 16 (heights are powers of two >= 16)
        for (uint32_t q = t; q < total / 4; q += NTH) {
            uint32_t w4[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const uint32_t i = 4 * q + j, r = i / W;
                w4[j] = buf[r * T::RP + (i - r * W)];
            }
            reinterpret_cast<uint4 *>(dst)[q] = make_uint4(w4[0], w4[1], w4[2], w4[3]);
        }
    }
    if constexpr (HIST) {
        __syncthreads();
        for (uint32_t i = t; i < HS; i += NTH)
            if (hkeys[i] != EMPTY && hvals[i]) hist.global_add(hkeys[i], hvals[i]);
    }
}

// ------------------------------------------------------------------ Cpu (include/cpu.hpp:37-108)
// CpuCols (cpu/columns/mod.rs), canonical u32 per column
enum {
    C_SHARD = 0, C_CLK16 = 1, C_CLK8 = 2, C_SHARD_SEND = 3, C_CLK_SEND = 4, C_PC = 5, C_NPC = 6, C_NNPC = 7,
    C_OPCODE = 8, C_OPA = 9, C_OPB = 10, C_OPC = 14, C_OPA0 = 18, C_IMMB = 19, C_IMMC = 20,
    C_EXTRA = 21, C_RW_A = 22, C_CHECK_MEM = 23, C_HALT = 24, C_SEQ = 25, C_A_VAL = 26, C_HI_PREV_A = 30,
    C_A_ACC = 34, C_B_ACC = 47, C_C_ACC = 56, C_REAL = 65, C_A_IMM = 66,
};
enum { ACC_VALUE = 0, ACC_PREV_SHARD = 4, ACC_PREV_CLK = 5, ACC_COMPARE = 6, ACC_D16 = 7, ACC_D8 = 8 };
// CpuEventFfi dword offsets (zkm_tracegen.h): the three operand records, then hi
enum { E_CLK = 0, E_PC = 1, E_NPC = 2, E_NNPC = 3, E_A = 4, E_AREC = 5, E_B = 17, E_BREC = 18, E_C = 30,
       E_CREC = 31, E_HI_TAG = 43, E_HI = 44, E_WORDS = 45 };
// OptionMemoryRecordEnum: tag, read {value, shard, ts, prev_shard, prev_ts}, write {value, shard, ts,
// prev_value, prev_shard, prev_ts}
enum { R_TAG = 0, R_READ = 1, R_WRITE = 6 };

struct Access {  // one populated MemoryAccessCols (include/memory.hpp:10-32)
    bool on;
    uint32_t value, prev_value, prev_shard, prev_clk, compare, d16, d8;
};

// populate_read / populate_read_write (include/memory.hpp:34-93) of an OptionMemoryRecordEnum
__device__ __forceinline__ Access access_of(const uint32_t *rec) {
    Access a{};
    const uint32_t tag = rec[R_TAG] & 0xFF;
    if (tag != ZKM_RECORD_READ && tag != ZKM_RECORD_WRITE) return a;
    const uint32_t *r = rec + (tag == ZKM_RECORD_READ ? R_READ : R_WRITE);
    const uint32_t value = r[0], shard = r[1], ts = r[2];
    const uint32_t prev_value = tag == ZKM_RECORD_READ ? value : r[3];
    const uint32_t prev_shard = r[tag == ZKM_RECORD_READ ? 3 : 4], prev_ts = r[tag == ZKM_RECORD_READ ? 4 : 5];
    a.on = true;
    a.value = value;
    a.prev_value = prev_value;
    a.prev_shard = prev_shard;
    a.prev_clk = prev_ts;
    const bool cmp = prev_shard == shard;
    a.compare = cmp;
    const uint32_t diff_minus_one = (cmp ? ts : shard) - (cmp ? prev_ts : prev_shard) - 1u;
    a.d16 = diff_minus_one & 0xFFFF;
    a.d8 = (diff_minus_one >> 16) & 0xFF;
    return a;
}

__device__ __forceinline__ void put_access(uint32_t *v, int base, const Access &a) {
    put_word(v + base + ACC_VALUE, a.value);
    v[base + ACC_PREV_SHARD] = a.prev_shard;
    v[base + ACC_PREV_CLK] = a.prev_clk;
    v[base + ACC_COMPARE] = a.compare;
    v[base + ACC_D16] = a.d16;
    v[base + ACC_D8] = a.d8;
}

struct CpuChip {
    const uint32_t *program;  // InstructionFfi as 6 dwords each
    uint64_t program_len;
    uint32_t pc_base, shard;

    __device__ __forceinline__ void row(uint32_t *v, const uint32_t *e, uint64_t, const Hist &h) const {
#pragma unroll
        for (int c = 0; c < ZKM_CPU_WIDTH; c++) v[c] = 0;
        const bool real = e != nullptr;
        Access acc[3] = {};  // a, b, c
        uint32_t clk = 0, written = 0, idx = 0;
        if (real) {
            clk = e[E_CLK];
            const uint32_t pc = e[E_PC];
            idx = (pc - pc_base) >> 2;
            if (idx >= program_len) idx = (uint32_t)program_len - 1;  // Program::fetch precondition
            const uint32_t *ins = program + 6 * (uint64_t)idx;
            const uint32_t opcode = ins[0] & 0xFF, op_a = (ins[0] >> 8) & 0xFF;
            const uint32_t imm_b = ins[3] & 0xFF, imm_c = (ins[3] >> 8) & 0xFF;
            // populate_shard_clk
            v[C_SHARD] = shard;
            v[C_CLK16] = clk & 0xFFFF;
            v[C_CLK8] = (clk >> 16) & 0xFF;
            v[C_PC] = pc;
            v[C_NPC] = e[E_NPC];
            v[C_NNPC] = e[E_NNPC];
            // populate_instruction
            v[C_OPCODE] = opcode;
            v[C_OPA] = op_a;
            put_word(v + C_OPB, ins[1]);
            put_word(v + C_OPC, ins[2]);
            v[C_OPA0] = op_a == 0;
            v[C_IMMB] = imm_b != 0;
            v[C_IMMC] = imm_c != 0;
            v[C_A_IMM] = is_store_except_sc(opcode) || is_branch(opcode);
            v[C_RW_A] = is_rw_a(opcode);
            const bool check = is_mult_div(opcode) || is_check_memory(opcode);
            v[C_CHECK_MEM] = check;
            put_word(v + C_A_VAL, e[E_A]);
            if ((e[E_HI_TAG] & 0xFF) == 0) put_word(v + C_HI_PREV_A, e[E_HI]);
            if (check) {
                v[C_SHARD_SEND] = shard;
                v[C_CLK_SEND] = clk;
            }
            // operand values (cpu.hpp:70-72), then the access records overwrite where present
            put_word(v + C_A_ACC + 4 + ACC_VALUE, e[E_A]);
            put_word(v + C_B_ACC + ACC_VALUE, e[E_B]);
            put_word(v + C_C_ACC + ACC_VALUE, e[E_C]);
            acc[0] = access_of(e + E_AREC);
            if ((e[E_BREC] & 0xFF) == ZKM_RECORD_READ) acc[1] = access_of(e + E_BREC);
            if ((e[E_CREC] & 0xFF) == ZKM_RECORD_READ) acc[2] = access_of(e + E_CREC);
            if (acc[0].on) {
                put_word(v + C_A_ACC, acc[0].prev_value);
                put_access(v, C_A_ACC + 4, acc[0]);
            }
            if (acc[1].on) put_access(v, C_B_ACC, acc[1]);
            if (acc[2].on) put_access(v, C_C_ACC, acc[2]);
            written = acc[0].on ? acc[0].value : e[E_A];
            bool halt = false;
            if (opcode == SYSCALL) {
                const uint32_t id0 = v[C_A_ACC + 0], id1 = v[C_A_ACC + 1];
                halt = (id0 == 0 && id1 == 0) || (id0 == (SYS_EXT_GROUP & 0xFF) && id1 == ((SYS_EXT_GROUP >> 8) & 0xFF));
                v[C_HALT] = halt;
                v[C_EXTRA] = v[C_A_ACC + 3];
            }
            v[C_SEQ] = !halt && !is_branch(opcode) && !is_jump(opcode);
            v[C_REAL] = 1;
        } else {  // padding row (cpu/trace.rs:60-66)
            v[C_IMMB] = 1;
            v[C_IMMC] = 1;
            v[C_RW_A] = 1;
        }
        // Byte lookups (cpu/trace.rs:206-247, MemoryAccessCols::populate): every lane takes part
        h.byte(B_U16RANGE, shard >> 8, shard & 0xFF, real);
        if (h.byte_mult) h.direct(((clk & 0xFFFF) * BYTE_COLS) + B_U16RANGE, real);  // distinct per row
        h.byte(B_U8RANGE, 0, (clk >> 16) & 0xFF, real);
#pragma unroll
        for (int k = 2; k >= 0; k--) {  // c, b, a: the order the executor reads them
            h.byte(B_U16RANGE, acc[k].d16 >> 8, acc[k].d16 & 0xFF, real && acc[k].on);
            h.byte(B_U8RANGE, 0, acc[k].d8, real && acc[k].on);
        }
        h.byte(B_U8RANGE, byte_of(written, 0), byte_of(written, 1), real);
        h.byte(B_U8RANGE, byte_of(written, 2), byte_of(written, 3), real);
        if (h.program_mult) h.add(PROG_KEY | idx, real);
    }
};

// ------------------------------------------------------------------ AddSub (include/add_sub.hpp:9-39)
enum { AS_PC = 0, AS_NPC = 1, AS_VAL = 2, AS_CARRY = 6, AS_OP1 = 9, AS_OP2 = 13, AS_ADD = 17, AS_SUB = 18 };

struct AddSubChip {
    __device__ __forceinline__ void row(uint32_t *v, const uint32_t *e, uint64_t, const Hist &h) const {
#pragma unroll
        for (int c = 0; c < ZKM_ADD_SUB_WIDTH; c++) v[c] = 0;
        const bool real = e != nullptr;
        uint32_t x = 0, y = 0, sum = 0;
        if (real) {  // AluEvent: pc, next_pc, opcode, hi, a, b, c
            const bool is_add = (e[2] & 0xFF) == ADD;
            x = is_add ? e[5] : e[4];
            y = e[6];
            sum = x + y;
            v[AS_PC] = e[0];
            v[AS_NPC] = e[1];
            v[AS_ADD] = is_add;
            v[AS_SUB] = !is_add;
            uint32_t carry = 0;
#pragma unroll
            for (int k = 0; k < 3; k++) {  // AddOperation::populate
                carry = (byte_of(x, k) + byte_of(y, k) + carry) > 0xFF;
                v[AS_CARRY + k] = carry;
            }
            put_word(v + AS_VAL, sum);
            put_word(v + AS_OP1, x);
            put_word(v + AS_OP2, y);
        }
        const uint32_t words[3] = {x, y, sum};
#pragma unroll
        for (int w = 0; w < 3; w++) {
            h.byte(B_U8RANGE, byte_of(words[w], 0), byte_of(words[w], 1), real);
            h.byte(B_U8RANGE, byte_of(words[w], 2), byte_of(words[w], 3), real);
        }
    }
};

// ------------------------------------------------------------------ the other AluEvent chips
// The reference fills these rows in Rust (no C++ row ABI): Bitwise (alu/bitwise/mod.rs:140-171), Lt
// (alu/lt/mod.rs:179-263), ShiftLeft (alu/sll/mod.rs:200-260), ShiftRight (alu/sr/mod.rs:220-325), each
// with its Byte lookups.  AluEvent dwords: pc, next_pc, opcode, hi, a, b, c.
constexpr uint32_t B_AND = 0, B_OR = 1, B_XOR = 2, B_SHRCARRY = 5, B_LTU = 6, B_MSB = 7, B_NOR = 9;
enum : uint32_t { OP_SRL = 10, OP_SRA = 11, OP_ROR = 12, OP_SLT = 13, OP_AND = 15, OP_OR = 16, OP_XOR = 17 };

enum { BW_PC = 0, BW_NPC = 1, BW_A = 2, BW_B = 6, BW_C = 10, BW_NOR = 14, BW_XOR = 15, BW_OR = 16, BW_AND = 17 };
struct BitwiseChip {
    __device__ __forceinline__ void row(uint32_t *v, const uint32_t *e, uint64_t, const Hist &h) const {
#pragma unroll
        for (int c = 0; c < ZKM_BITWISE_WIDTH; c++) v[c] = 0;
        const bool real = e != nullptr;
        const uint32_t op = real ? e[2] & 0xFF : 0u, b = real ? e[5] : 0u, c = real ? e[6] : 0u;
        if (real) {
            v[BW_PC] = e[0];
            v[BW_NPC] = e[1];
            put_word(v + BW_A, e[4]);
            put_word(v + BW_B, b);
            put_word(v + BW_C, c);
            v[BW_AND] = op == OP_AND;
            v[BW_OR] = op == OP_OR;
            v[BW_XOR] = op == OP_XOR;
            v[BW_NOR] = op != OP_AND && op != OP_OR && op != OP_XOR;
        }
        const uint32_t bop = op == OP_AND ? B_AND : op == OP_OR ? B_OR : op == OP_XOR ? B_XOR : B_NOR;
#pragma unroll
        for (int k = 0; k < 4; k++) h.byte(bop, byte_of(b, k), byte_of(c, k), real);
    }
};

// (x mod p)^-1 of a canonical x (0 -> 0), by Fermat in Montgomery form (32-bit products, no 64-bit
// modulo)
__device__ __forceinline__ uint32_t inv_canonical(uint32_t x) {
    return x ? kb::from_mont(kb::inv(kb::to_mont(x))) : 0u;
}

enum { LT_PC = 0, LT_NPC = 1, LT_SLT = 2, LT_SLTU = 3, LT_A = 4, LT_B = 8, LT_C = 12, LT_FLAGS = 16, LT_BM = 20,
       LT_CM = 21, LT_INV = 22, LT_MSB_B = 23, LT_MSB_C = 24, LT_BIT_B = 25, LT_BIT_C = 26, LT_SLTU_R = 27,
       LT_COMP_EQ = 28, LT_SIGN_EQ = 29, LT_CMP = 30 };
struct LtChip {
    __device__ __forceinline__ void row(uint32_t *v, const uint32_t *e, uint64_t, const Hist &h) const {
#pragma unroll
        for (int c = 0; c < ZKM_LT_WIDTH; c++) v[c] = 0;
        const bool real = e != nullptr;
        const uint32_t b = real ? e[5] : 0u, c = real ? e[6] : 0u;
        const bool slt = real && (e[2] & 0xFF) == OP_SLT;
        const uint32_t b3 = byte_of(b, 3), c3 = byte_of(c, 3), bm = b3 & 0x7F, cm = c3 & 0x7F;
        h.byte(B_AND, b3, 0x7F, real);
        h.byte(B_AND, c3, 0x7F, real);
        uint32_t bc[4], cc[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            bc[i] = byte_of(b, i);
            cc[i] = byte_of(c, i);
        }
        if (slt) {
            bc[3] = bm;
            cc[3] = cm;
        }
        int first = -1;  // the most significant differing byte
#pragma unroll
        for (int i = 0; i < 4; i++)
            if (bc[i] != cc[i]) first = i;
        uint32_t bcb = 0, ccb = 0;
#pragma unroll
        for (int i = 0; i < 4; i++)
            if (i == first) {
                bcb = bc[i];
                ccb = cc[i];
            }
        h.byte(B_LTU, bcb, ccb, real);
        if (!real) return;
        const uint32_t msb_b = b3 >> 7, msb_c = c3 >> 7, sltu = bcb < ccb;
        v[LT_PC] = e[0];
        v[LT_NPC] = e[1];
        put_word(v + LT_A, e[4]);
        put_word(v + LT_B, b);
        put_word(v + LT_C, c);
        v[LT_BM] = bm;
        v[LT_CM] = cm;
#pragma unroll
        for (int i = 0; i < 4; i++) v[LT_FLAGS + i] = i == first;
        v[LT_INV] = inv_canonical(bcb >= ccb ? bcb - ccb : P - (ccb - bcb));
        v[LT_CMP] = bcb;
        v[LT_CMP + 1] = ccb;
        v[LT_SLTU_R] = sltu;
        v[LT_COMP_EQ] = first < 0;
        v[LT_MSB_B] = msb_b;
        v[LT_MSB_C] = msb_c;
        v[LT_SIGN_EQ] = slt ? msb_b == msb_c : 1u;
        v[LT_SLT] = slt;
        v[LT_SLTU] = !slt;
        v[LT_BIT_B] = slt ? msb_b : 0u;
        v[LT_BIT_C] = slt ? msb_c : 0u;
    }
};

enum { SL_PC = 0, SL_NPC = 1, SL_A = 2, SL_B = 6, SL_C = 10, SL_CBITS = 14, SL_NBITS = 22, SL_MULT = 30, SL_RES = 31,
       SL_CARRY = 35, SL_NBYTES = 39, SL_REAL = 43 };
struct ShiftLeftChip {
    __device__ __forceinline__ void row(uint32_t *v, const uint32_t *e, uint64_t, const Hist &h) const {
#pragma unroll
        for (int c = 0; c < ZKM_SHIFT_LEFT_WIDTH; c++) v[c] = 0;
        const bool real = e != nullptr;
        if (!real) {  // padding: shift_by_n_bits[0] = shift_by_n_bytes[0] = bit_shift_multiplier = 1 (:142-155)
            v[SL_NBITS] = v[SL_NBYTES] = v[SL_MULT] = 1;
        }
        const uint32_t b = real ? e[5] : 0u, c = real ? e[6] : 0u;
        const uint32_t nb = c & 7, mul = 1u << nb;
        uint32_t res = 0, cry = 0, carry = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t x = byte_of(b, i) * mul + carry;
            carry = x >> 8;
            res |= (x & 0xFF) << (8 * i);
            cry |= carry << (8 * i);
        }
        h.byte(B_U8RANGE, byte_of(res, 0), byte_of(res, 1), real);
        h.byte(B_U8RANGE, byte_of(res, 2), byte_of(res, 3), real);
        h.byte(B_U8RANGE, byte_of(cry, 0), byte_of(cry, 1), real);
        h.byte(B_U8RANGE, byte_of(cry, 2), byte_of(cry, 3), real);
        if (!real) return;
        v[SL_PC] = e[0];
        v[SL_NPC] = e[1];
        put_word(v + SL_A, e[4]);
        put_word(v + SL_B, b);
        put_word(v + SL_C, c);
#pragma unroll
        for (int i = 0; i < 8; i++) {
            v[SL_CBITS + i] = (c >> i) & 1;
            v[SL_NBITS + i] = (uint32_t)i == nb;
        }
        v[SL_MULT] = mul;
        put_word(v + SL_RES, res);
        put_word(v + SL_CARRY, cry);
        const uint32_t nbyte = (c & 31) >> 3;
#pragma unroll
        for (int i = 0; i < 4; i++) v[SL_NBYTES + i] = (uint32_t)i == nbyte;
        v[SL_REAL] = 1;
    }
};

enum { SR_PC = 0, SR_NPC = 1, SR_A = 2, SR_B = 6, SR_C = 10, SR_NBITS = 14, SR_NBYTES = 22, SR_BYTE_RES = 26,
       SR_BIT_RES = 34, SR_CARRY = 42, SR_SHIFTED = 50, SR_MSB = 58, SR_CBITS = 59, SR_SRL = 67, SR_ROR = 68,
       SR_SRA = 69, SR_REAL = 70 };
struct ShiftRightChip {
    __device__ __forceinline__ void row(uint32_t *v, const uint32_t *e, uint64_t, const Hist &h) const {
#pragma unroll
        for (int c = 0; c < ZKM_SHIFT_RIGHT_WIDTH; c++) v[c] = 0;
        const bool real = e != nullptr;
        if (!real) {  // padding: shift_by_n_bits[0] = shift_by_n_bytes[0] = 1
            v[SR_NBITS] = v[SR_NBYTES] = 1;
        }
        const uint32_t op = real ? e[2] & 0xFF : OP_SRL, b = real ? e[5] : 0u, c = real ? e[6] : 0u;
        const uint32_t nbyte = (c & 31) >> 3, nbit = c & 7;
        // the operand extended to 64 bits (sign for SRA, a second copy for ROR), shifted by whole bytes
        const uint64_t ext = op == OP_SRA ? (uint64_t)(int64_t)(int32_t)b
                             : op == OP_ROR ? ((uint64_t)b | ((uint64_t)b << 32)) : (uint64_t)b;
        const uint64_t bsr = ext >> (8 * nbyte);
        uint32_t byte_res[8], shifted[8], carry[8], bit_res[8];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            byte_res[i] = (uint32_t)(bsr >> (8 * i)) & 0xFF;
            shifted[i] = byte_res[i] >> nbit;
            carry[i] = byte_res[i] & ((1u << nbit) - 1);
        }
#pragma unroll
        for (int i = 0; i < 8; i++) bit_res[i] = i < 7 ? (shifted[i] + (carry[i + 1] << (8 - nbit))) & 0xFF : shifted[i];
        h.byte(B_MSB, byte_of(b, 3), 0, real);
#pragma unroll
        for (int i = 0; i < 8; i++) h.byte(B_SHRCARRY, byte_res[i], nbit, real);
        const uint32_t *words[4] = {byte_res, bit_res, carry, shifted};
#pragma unroll
        for (int w = 0; w < 4; w++)
#pragma unroll
            for (int k = 0; k < 8; k += 2) h.byte(B_U8RANGE, words[w][k], words[w][k + 1], real);
        if (!real) return;
        v[SR_PC] = e[0];
        v[SR_NPC] = e[1];
        put_word(v + SR_A, e[4]);
        put_word(v + SR_B, b);
        put_word(v + SR_C, c);
        v[SR_MSB] = b >> 31;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            v[SR_CBITS + i] = (c >> i) & 1;
            v[SR_NBITS + i] = (uint32_t)i == nbit;
            v[SR_BYTE_RES + i] = byte_res[i];
            v[SR_BIT_RES + i] = bit_res[i];
            v[SR_CARRY + i] = carry[i];
            v[SR_SHIFTED + i] = shifted[i];
        }
#pragma unroll
        for (int i = 0; i < 4; i++) v[SR_NBYTES + i] = (uint32_t)i == nbyte;
        v[SR_SRL] = op == OP_SRL;
        v[SR_SRA] = op == OP_SRA;
        v[SR_ROR] = op == OP_ROR;
        v[SR_REAL] = 1;
    }
};

// ------------------------------------------------------------------ Branch (control_flow/branch/trace.rs:85-130)
// BranchEvent dwords: pc, next_pc, next_next_pc, opcode, a, b, c.  KoalaBearWordRangeChecker of a word
// (operations/koala_bear_word.rs:34-52): the 8 bits of its top byte and their running products.
__device__ __forceinline__ void put_range_check(uint32_t *v, uint32_t x) {
    uint32_t acc = 1;
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = (x >> (24 + i)) & 1;
#pragma unroll
    for (int k = 0; k < 6; k++) {
        acc = k == 0 ? v[0] * v[1] : acc * v[k + 1];
        v[8 + k] = acc;
    }
}

enum { BR_PC = 0, BR_NPC = 1, BR_NPC_RC = 5, BR_TGT = 19, BR_NNPC = 23, BR_NNPC_RC = 27, BR_A = 41, BR_B = 45,
       BR_C = 49, BR_BEQ = 53, BR_BNE = 54, BR_BLTZ = 55, BR_BLEZ = 56, BR_BGTZ = 57, BR_BGEZ = 58, BR_BRANCHING = 59,
       BR_GT = 60, BR_LT = 61 };
struct BranchChip {
    __device__ __forceinline__ void row(uint32_t *v, const uint32_t *e, uint64_t, const Hist &h) const {
#pragma unroll
        for (int c = 0; c < ZKM_BRANCH_WIDTH; c++) v[c] = 0;
        const bool real = e != nullptr;
        uint32_t npc = 0, nnpc = 0;
        bool taken = false;
        if (real) {
            const uint32_t op = e[3] & 0xFF, a = e[4], b = e[5], c = e[6];
            npc = e[1];
            nnpc = e[2];
            const int32_t sa = (int32_t)a, sb = (int32_t)b;
            // Executor::execute_branch (executor.rs:2098-2120)
            taken = op == BEQ ? a == b : op == BNE ? a != b : op == BGEZ ? sa >= 0 : op == BLEZ ? sa <= 0
                  : op == BGTZ ? sa > 0 : sa < 0;
            v[BR_PC] = e[0];
            v[BR_BEQ] = op == BEQ;
            v[BR_BNE] = op == BNE;
            v[BR_BLTZ] = op == BLTZ;
            v[BR_BGTZ] = op == BGTZ;
            v[BR_BLEZ] = op == BLEZ;
            v[BR_BGEZ] = op == BGEZ;
            put_word(v + BR_A, a);
            put_word(v + BR_B, b);
            put_word(v + BR_C, c);
            v[BR_LT] = sa < sb;
            v[BR_GT] = sa > sb;
            put_word(v + BR_NPC, npc);
            put_word(v + BR_TGT, npc + c);
            put_word(v + BR_NNPC, nnpc);
            put_range_check(v + BR_NPC_RC, npc);
            put_range_check(v + BR_NNPC_RC, nnpc);
            v[BR_BRANCHING] = taken;
        }
        const bool nt = real && !taken;  // the not-taken rows range-check next_pc and next_next_pc
        h.byte(B_U8RANGE, byte_of(npc, 0), byte_of(npc, 1), nt);
        h.byte(B_U8RANGE, byte_of(npc, 2), byte_of(npc, 3), nt);
        h.byte(B_U8RANGE, byte_of(nnpc, 0), byte_of(nnpc, 1), nt);
        h.byte(B_U8RANGE, byte_of(nnpc, 2), byte_of(nnpc, 3), nt);
    }
};

// ------------------------------------------------------------------ MemoryInstrs (memory/instructions/trace.rs:88-251)
// zkm_mem_instr_event dwords: shard, clk, pc, next_pc, opcode, a, b, c, mem_access (OptionMemoryRecordEnum,
// 12 dwords), prev_a_val
enum { MI_PC = 0, MI_NPC = 1, MI_SHARD = 2, MI_CLK = 3, MI_A = 4, MI_B = 8, MI_C = 12, MI_SEL = 16, MI_ADDR = 30,
       MI_ALIGNED = 34, MI_LS2 = 35, MI_L1 = 36, MI_L2 = 37, MI_L3 = 38, MI_ADDR_RC = 39, MI_ACC = 53, MI_PREV_A = 66,
       MI_UMV = 70, MI_MSBIT = 74, MI_MSBYTE = 75, MI_NEG = 76, MI_MSBZ = 77 };
constexpr uint32_t B_LTU_NUM_REGISTERS_M1 = 35;  // REF_NUM_REGISTERS - 1 (executor/src/register.rs)

struct MemoryInstrsChip {
    __device__ __forceinline__ void row(uint32_t *v, const uint32_t *e, uint64_t, const Hist &h) const {
#pragma unroll
        for (int c = 0; c < ZKM_MEMORY_INSTRS_WIDTH; c++) v[c] = 0;
        const bool real = e != nullptr;
        Access acc{};
        uint32_t addr = 0, op = 0, umv = 0;
        if (real) {
            op = e[4] & 0xFF;
            const uint32_t a = e[5], b = e[6], c = e[7];
            addr = b + c;
            v[MI_PC] = e[2];
            v[MI_NPC] = e[3];
            v[MI_SHARD] = e[0];
            v[MI_CLK] = e[1];
            put_word(v + MI_A, a);
            put_word(v + MI_B, b);
            put_word(v + MI_C, c);
            put_word(v + MI_PREV_A, e[20]);
            put_word(v + MI_ADDR, addr);
#pragma unroll
            for (int k = 0; k < 14; k++) v[MI_SEL + k] = op == LB + (uint32_t)k;
            const uint32_t two = addr & 3;
            v[MI_ALIGNED] = addr - two;
            v[MI_LS2] = two;
            v[MI_L1] = two == 1;
            v[MI_L2] = two == 2;
            v[MI_L3] = two == 3;
            put_range_check(v + MI_ADDR_RC, addr);
            acc = access_of(e + 8);
            put_word(v + MI_ACC, acc.prev_value);
            put_access(v, MI_ACC + 4, acc);
            const uint32_t pmem = acc.prev_value;
            if (op >= LB && op <= LL) {  // the loaded value before sign extension
                umv = (op == LB || op == LBU) ? byte_of(pmem, (int)two)
                    : (op == LH || op == LHU) ? ((two >> 1) ? pmem >> 16 : pmem & 0xFFFF)
                    : (op == LWL || op == LWR) ? a : pmem;
            }
            put_word(v + MI_UMV, umv);
        }
        const bool sgn = real && (op == LB || op == LH);
        const uint32_t msbyte = op == LB ? umv & 0xFF : (umv >> 8) & 0xFF, msbit = msbyte >> 7;
        const uint32_t s = byte_of(addr, 1) + byte_of(addr, 2) + byte_of(addr, 3);
        if (real) {
            v[MI_MSBYTE] = sgn ? msbyte : 0u;
            v[MI_MSBIT] = sgn ? msbit : 0u;
            v[MI_NEG] = sgn && msbit == 1;
            v[MI_MSBZ] = inv_canonical(s);
            v[MI_MSBZ + 1] = s == 0;
        }
        h.byte(B_U16RANGE, acc.d16 >> 8, acc.d16 & 0xFF, real);
        h.byte(B_U8RANGE, 0, acc.d8, real);
        h.byte(B_AND, byte_of(addr, 0), 3, real);
        h.byte(B_MSB, msbyte, 0, sgn);
        h.byte(B_U8RANGE, byte_of(addr, 1), byte_of(addr, 2), real);
        h.byte(B_LTU, B_LTU_NUM_REGISTERS_M1, byte_of(addr, 0), real && s == 0);
    }
};

// ------------------------------------------------------------------ Jump (control_flow/jump/trace.rs:83-102)
// JumpEvent dwords: pc, next_pc, next_next_pc, opcode, a, b, c; no Byte lookups
enum { J_PC = 0, J_NPC = 1, J_NPC_RC = 5, J_NNPC = 19, J_NNPC_RC = 23, J_A = 37, J_B = 41, J_C = 45, J_JUMP = 49,
       J_JUMPI = 50, J_JDIRECT = 51, J_A_RC = 52 };
struct JumpChip {
    __device__ __forceinline__ void row(uint32_t *v, const uint32_t *e, uint64_t, const Hist &) const {
#pragma unroll
        for (int c = 0; c < ZKM_JUMP_WIDTH; c++) v[c] = 0;
        if (!e) return;
        const uint32_t op = e[3] & 0xFF;
        v[J_PC] = e[0];
        v[J_JUMP] = op == JUMP;
        v[J_JUMPI] = op == JUMPI;
        v[J_JDIRECT] = op == JUMPDIRECT;
        put_word(v + J_A, e[4]);
        put_word(v + J_B, e[5]);
        put_word(v + J_C, e[6]);
        put_word(v + J_NPC, e[1]);
        put_word(v + J_NNPC, e[2]);
        put_range_check(v + J_A_RC, e[4]);
        put_range_check(v + J_NPC_RC, e[1]);
        put_range_check(v + J_NNPC_RC, e[2]);
    }
};

// ------------------------------------------------------------------ MovCond (misc/mov_cond/mod.rs)
// MovCondEvent dwords: pc, next_pc, opcode, a, b, c, prev_a; IsZeroWordOperation of c's bytes
enum { MC_PC = 0, MC_NPC = 1, MC_A = 2, MC_PREV_A = 6, MC_B = 10, MC_C = 14, MC_C0 = 18, MC_MNE = 29, MC_MEQ = 30,
       MC_WSBH = 31 };
constexpr uint32_t OP_MEQ = 50, OP_MNE = 51, OP_WSBH = 52;
struct MovCondChip {
    __device__ __forceinline__ void row(uint32_t *v, const uint32_t *e, uint64_t, const Hist &) const {
#pragma unroll
        for (int c = 0; c < ZKM_MOVCOND_WIDTH; c++) v[c] = 0;
        if (!e) return;
        const uint32_t op = e[2] & 0xFF, c = e[5];
        v[MC_PC] = e[0];
        v[MC_NPC] = e[1];
        put_word(v + MC_A, e[3]);
        put_word(v + MC_B, e[4]);
        put_word(v + MC_C, c);
        put_word(v + MC_PREV_A, e[6]);
        uint32_t z[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {  // IsZeroWordOperation::populate_from_field_element
            const uint32_t x = byte_of(c, i);
            z[i] = x == 0;
            v[MC_C0 + 2 * i] = inv_canonical(x);
            v[MC_C0 + 2 * i + 1] = z[i];
        }
        v[MC_C0 + 8] = z[0] * z[1];
        v[MC_C0 + 9] = z[2] * z[3];
        v[MC_C0 + 10] = z[0] * z[1] * z[2] * z[3];
        v[MC_MEQ] = op == OP_MEQ;
        v[MC_MNE] = op == OP_MNE;
        v[MC_WSBH] = op == OP_WSBH;
    }
};

// ------------------------------------------------------------------ Mul (alu/mul/mod.rs:218-318)
// zkm_comp_alu_event dwords: shard, clk, pc, next_pc, opcode, hi, a, b, c, hi_record (6), hi_record_is_real
enum { MU_PC = 0, MU_NPC = 1, MU_HI = 2, MU_A = 6, MU_B = 10, MU_C = 14, MU_CARRY = 18, MU_PROD = 26, MU_BMSB = 34,
       MU_CMSB = 35, MU_BSE = 36, MU_CSE = 37, MU_MUL = 38, MU_MULT = 39, MU_MULTU = 40, MU_REAL = 41,
       MU_HI_ACC = 42, MU_HRR = 55, MU_SHARD = 56, MU_CLK = 57 };
constexpr uint32_t OP_MUL = 2;
struct MulChip {
    __device__ __forceinline__ void row(uint32_t *v, const uint32_t *e, uint64_t, const Hist &h) const {
#pragma unroll
        for (int c = 0; c < ZKM_MUL_WIDTH; c++) v[c] = 0;
        const bool real = e != nullptr;
        const uint32_t op = real ? e[4] & 0xFF : 0u, b = real ? e[7] : 0u, c = real ? e[8] : 0u;
        const uint32_t bmsb = byte_of(b, 3) >> 7, cmsb = byte_of(c, 3) >> 7;
        const bool bse = op == MULT && bmsb, cse = op == MULT && cmsb;
        uint32_t b8[8], c8[8], prod[8], carry[8];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            b8[i] = byte_of(b, i);
            c8[i] = byte_of(c, i);
            b8[4 + i] = bse ? 255u : 0u;
            c8[4 + i] = cse ? 255u : 0u;
        }
#pragma unroll
        for (int i = 0; i < 8; i++) prod[i] = 0;
#pragma unroll
        for (int i = 0; i < 8; i++)
#pragma unroll
            for (int j = 0; j < 8 - i; j++) prod[i + j] += b8[i] * c8[j];
#pragma unroll
        for (int i = 0; i < 8; i++) {
            carry[i] = prod[i] >> 8;
            prod[i] &= 0xFF;
            if (i + 1 < 8) prod[i + 1] += carry[i];
        }
        Access acc{};
        const bool hrr = real && (e[15] & 0xFF);
        if (hrr) {  // the HI register write (MemoryWriteRecord: value, shard, timestamp, prev_value, prev_shard, prev_ts)
            const uint32_t *r = e + 9;
            acc.on = true;
            acc.value = r[0];
            acc.prev_value = r[3];
            acc.prev_shard = r[4];
            acc.prev_clk = r[5];
            const bool cmp = r[4] == r[1];
            acc.compare = cmp;
            const uint32_t d = (cmp ? r[2] : r[1]) - (cmp ? r[5] : r[4]) - 1u;
            acc.d16 = d & 0xFFFF;
            acc.d8 = (d >> 16) & 0xFF;
        }
        h.byte(B_MSB, byte_of(b, 3), 0, real);
        h.byte(B_MSB, byte_of(c, 3), 0, real);
#pragma unroll
        for (int i = 0; i < 8; i++) h.byte(B_U16RANGE, carry[i] >> 8, carry[i] & 0xFF, real);
#pragma unroll
        for (int k = 0; k < 8; k += 2) h.byte(B_U8RANGE, prod[k], prod[k + 1], real);
        h.byte(B_U16RANGE, acc.d16 >> 8, acc.d16 & 0xFF, hrr);
        h.byte(B_U8RANGE, 0, acc.d8, hrr);
        if (!real) return;
        v[MU_PC] = e[2];
        v[MU_NPC] = e[3];
        put_word(v + MU_HI, e[5]);
        put_word(v + MU_A, e[6]);
        put_word(v + MU_B, b);
        put_word(v + MU_C, c);
#pragma unroll
        for (int i = 0; i < 8; i++) {
            v[MU_CARRY + i] = carry[i];
            v[MU_PROD + i] = prod[i];
        }
        v[MU_BMSB] = bmsb;
        v[MU_CMSB] = cmsb;
        v[MU_BSE] = bse;
        v[MU_CSE] = cse;
        v[MU_MUL] = op == OP_MUL;
        v[MU_MULT] = op == MULT;
        v[MU_MULTU] = op == MULTU;
        v[MU_REAL] = 1;
        v[MU_HRR] = hrr;
        if (hrr) {
            v[MU_SHARD] = e[0];
            v[MU_CLK] = e[1];
            put_word(v + MU_HI_ACC, acc.prev_value);
            put_access(v, MU_HI_ACC + 4, acc);
        }
    }
};

// ------------------------------------------------------------------ DivRem (alu/divrem/mod.rs:240-390)
// zkm_comp_alu_event as for Mul; quotient and remainder recomputed (get_quotient_and_remainder,
// executor/src/utils.rs:33-43), the HI write (DIV / DIVU) carries the remainder
enum { DV_PC = 0, DV_NPC = 1, DV_B = 2, DV_C = 6, DV_Q = 10, DV_R = 14, DV_ABS_R = 18, DV_ABS_C = 22, DV_MAXC = 26,
       DV_CTQ = 30, DV_CARRY = 38, DV_IS_C0 = 46, DV_DIV = 57, DV_DIVU = 58, DV_MOD = 59, DV_MODU = 60, DV_OVF = 61,
       DV_OVF_B = 62, DV_OVF_C = 73, DV_BMSB = 84, DV_RMSB = 85, DV_CMSB = 86, DV_BNEG = 87, DV_RNEG = 88,
       DV_CNEG = 89, DV_RCM = 90, DV_HI_ACC = 91, DV_SHARD = 104, DV_CLK = 105 };
constexpr uint32_t OP_MOD = 7, OP_MODU = 8;

// IsZeroWordOperation::populate_from_field_element of four field elements (11 columns)
__device__ __forceinline__ void put_is_zero_word(uint32_t *v, const uint32_t x[4]) {
    uint32_t z[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        z[i] = x[i] == 0;
        v[2 * i] = inv_canonical(x[i]);
        v[2 * i + 1] = z[i];
    }
    v[8] = z[0] * z[1];
    v[9] = z[2] * z[3];
    v[10] = z[0] * z[1] * z[2] * z[3];
}

struct DivRemChip {
    __device__ __forceinline__ void row(uint32_t *v, const uint32_t *e, uint64_t, const Hist &h) const {
#pragma unroll
        for (int c = 0; c < ZKM_DIVREM_WIDTH; c++) v[c] = 0;
        const bool real = e != nullptr;
        const uint32_t op = real ? e[4] & 0xFF : 0u, b = real ? e[7] : 0u, c = real ? e[8] : 0u;
        const bool sgn = op == DIV || op == OP_MOD;
        uint32_t q, r;
        if (c == 0) {
            q = 0xFFFFFFFFu;
            r = b;
        } else if (sgn) {
            if (b == 0x80000000u && c == 0xFFFFFFFFu) {  // wrapping_div / wrapping_rem
                q = b;
                r = 0;
            } else {
                q = (uint32_t)((int32_t)b / (int32_t)c);
                r = (uint32_t)((int32_t)b % (int32_t)c);
            }
        } else {
            q = b / c;
            r = b % c;
        }
        const uint32_t bmsb = b >> 31, cmsb = c >> 31, rmsb = r >> 31;
        const uint32_t abs_r = sgn && rmsb ? 0u - r : r, abs_c = sgn && cmsb ? 0u - c : c;
        // c * q + r in 64 bits, as bytes (signed operands sign-extended)
        const uint64_t ctq = sgn ? (uint64_t)((int64_t)(int32_t)q * (int64_t)(int32_t)c) : (uint64_t)q * (uint64_t)c;
        const uint64_t r64 = sgn ? (uint64_t)(int64_t)(int32_t)r : (uint64_t)r;
        uint32_t ctq_b[8], carry[8];
        uint32_t cy = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            ctq_b[i] = (uint32_t)(ctq >> (8 * i)) & 0xFF;
            cy = (ctq_b[i] + ((uint32_t)(r64 >> (8 * i)) & 0xFF) + cy) >> 8;
            carry[i] = cy;
        }
        Access acc{};
        const bool hrr = real && (e[15] & 0xFF);
        if (hrr) {
            const uint32_t *rr = e + 9;
            acc.on = true;
            acc.value = rr[0];
            acc.prev_value = rr[3];
            acc.prev_shard = rr[4];
            acc.prev_clk = rr[5];
            const bool cmp = rr[4] == rr[1];
            acc.compare = cmp;
            const uint32_t d = (cmp ? rr[2] : rr[1]) - (cmp ? rr[5] : rr[4]) - 1u;
            acc.d16 = d & 0xFFFF;
            acc.d8 = (d >> 16) & 0xFF;
        }
        h.byte(B_U16RANGE, acc.d16 >> 8, acc.d16 & 0xFF, hrr);
        h.byte(B_U8RANGE, 0, acc.d8, hrr);
        h.byte(B_MSB, byte_of(b, 3), 0, real);
        h.byte(B_MSB, byte_of(c, 3), 0, real);
        h.byte(B_MSB, byte_of(r, 3), 0, real);
        h.byte(B_U8RANGE, byte_of(q, 0), byte_of(q, 1), real);
        h.byte(B_U8RANGE, byte_of(q, 2), byte_of(q, 3), real);
        h.byte(B_U8RANGE, byte_of(r, 0), byte_of(r, 1), real);
        h.byte(B_U8RANGE, byte_of(r, 2), byte_of(r, 3), real);
#pragma unroll
        for (int k = 0; k < 8; k += 2) h.byte(B_U8RANGE, ctq_b[k], ctq_b[k + 1], real);
        if (!real) return;
        v[DV_PC] = e[2];
        v[DV_NPC] = e[3];
        put_word(v + DV_B, b);
        put_word(v + DV_C, c);
        put_word(v + DV_Q, q);
        put_word(v + DV_R, r);
        v[DV_DIV] = op == DIV;
        v[DV_DIVU] = op == DIVU;
        v[DV_MOD] = op == OP_MOD;
        v[DV_MODU] = op == OP_MODU;
        uint32_t x[4];
#pragma unroll
        for (int i = 0; i < 4; i++) x[i] = byte_of(c, i);
        put_is_zero_word(v + DV_IS_C0, x);
#pragma unroll
        for (int i = 0; i < 4; i++) {  // bytes of b minus (0, 0, 0, 0x80), as field elements
            const uint32_t bi = byte_of(b, i), k = i == 3 ? 0x80u : 0u;
            x[i] = bi >= k ? bi - k : P - (k - bi);
        }
        put_is_zero_word(v + DV_OVF_B, x);
#pragma unroll
        for (int i = 0; i < 4; i++) {  // bytes of c minus 255
            const uint32_t ci = byte_of(c, i);
            x[i] = ci == 255 ? 0u : P - (255 - ci);
        }
        put_is_zero_word(v + DV_OVF_C, x);
        v[DV_BMSB] = bmsb;
        v[DV_CMSB] = cmsb;
        v[DV_RMSB] = rmsb;
        v[DV_BNEG] = sgn ? bmsb : 0u;
        v[DV_CNEG] = sgn ? cmsb : 0u;
        v[DV_RNEG] = sgn ? rmsb : 0u;
        v[DV_OVF] = sgn && b == 0x80000000u && c == 0xFFFFFFFFu;
        put_word(v + DV_ABS_R, abs_r);
        put_word(v + DV_ABS_C, abs_c);
        put_word(v + DV_MAXC, abs_c > 1u ? abs_c : 1u);
        v[DV_RCM] = c != 0;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            v[DV_CTQ + i] = ctq_b[i];
            v[DV_CARRY + i] = carry[i];
        }
        if (hrr) {
            v[DV_SHARD] = e[0];
            v[DV_CLK] = e[1];
            put_word(v + DV_HI_ACC, acc.prev_value);
            put_access(v, DV_HI_ACC + 4, acc);
        }
    }
};

// ------------------------------------------------------------------ CloClz (alu/clo_clz/mod.rs:85-160)
enum { CZ_PC = 0, CZ_NPC = 1, CZ_A = 2, CZ_B = 6, CZ_BB = 10, CZ_BB_ZERO = 14, CZ_SR1 = 15, CZ_CLZ = 19, CZ_CLO = 20,
       CZ_REAL = 21 };
constexpr uint32_t OP_CLO = 20;
struct CloClzChip {
    __device__ __forceinline__ void row(uint32_t *v, const uint32_t *e, uint64_t, const Hist &h) const {
#pragma unroll
        for (int c = 0; c < ZKM_CLO_CLZ_WIDTH; c++) v[c] = 0;
        const bool real = e != nullptr;
        const uint32_t a = real ? e[4] : 32u, b = real ? e[5] : 0u;
        const bool clo = real && (e[2] & 0xFF) == OP_CLO;
        const uint32_t bb = clo ? ~b : b;
        h.byte(B_U8RANGE, byte_of(bb, 0), byte_of(bb, 1), real);
        h.byte(B_U8RANGE, byte_of(bb, 2), byte_of(bb, 3), real);
        h.byte(B_LTU, a & 0xFF, 33, real);
        if (!real) {  // padding: clz(0) = 32
            v[CZ_A] = 32;
            v[CZ_CLZ] = 1;
            v[CZ_BB_ZERO] = 1;
            return;
        }
        v[CZ_PC] = e[0];
        v[CZ_NPC] = e[1];
        put_word(v + CZ_A, a);
        put_word(v + CZ_B, b);
        put_word(v + CZ_BB, bb);
        v[CZ_BB_ZERO] = bb == 0;
        put_word(v + CZ_SR1, bb ? bb >> (31 - a) : 0u);
        v[CZ_CLZ] = !clo;
        v[CZ_CLO] = clo;
        v[CZ_REAL] = 1;
    }
};

// ------------------------------------------------------------------ SyscallInstrs (syscall/instructions/trace.rs:82-162)
// from SyscallEvents (a = a_record.value, prev_a = a_record.prev_value, b = arg1, c = arg2); no Byte lookups
enum { SI_PC = 0, SI_NPC = 1, SI_SHARD = 2, SI_CLK = 3, SI_EXTRA = 4, SI_HALT = 5, SI_LINUX = 6, SI_ID = 7, SI_A = 8,
       SI_B = 12, SI_C = 16, SI_PREV_A = 20, SI_IZ = 24, SI_BITMAP = 36, SI_RC_BITS = 44, SI_RC_AND = 52,
       SI_OPERAND = 58, SI_RCOP = 62, SI_REAL = 63 };
// syscall ids of the IsZero columns in order: ENTER_UNCONSTRAINED, HINT_LEN, HALT, SYS_EXT_GROUP, COMMIT,
// COMMIT_DEFERRED_PROOFS (syscalls/code.rs)
__constant__ uint32_t kSiCodes[6] = {0x03, 0xF0, 0x00, SYS_EXT_GROUP, 0x10, 0x1A};
struct SyscallInstrsChip {
    __device__ __forceinline__ void row(uint32_t *v, const uint32_t *e, uint64_t, const Hist &) const {
#pragma unroll
        for (int c = 0; c < ZKM_SYSCALL_INSTRS_WIDTH; c++) v[c] = 0;
        if (!e) return;
        const uint32_t a = e[4], prev = e[7], b = e[12], c = e[13], sid = prev & 0xFFFF;
        v[SI_PC] = e[0];
        v[SI_NPC] = e[1];
        v[SI_SHARD] = e[2];
        v[SI_CLK] = e[3];
        put_word(v + SI_A, a);
        put_word(v + SI_B, b);
        put_word(v + SI_C, c);
        put_word(v + SI_PREV_A, prev);
        v[SI_ID] = e[11];
        v[SI_EXTRA] = prev >> 24;
        const bool halt = sid == 0 || sid == SYS_EXT_GROUP;
        v[SI_HALT] = halt;
        v[SI_LINUX] = (prev & 0xFF00) != 0;
#pragma unroll
        for (int k = 0; k < 6; k++) {  // IsZeroOperation of sid - code (as a field element)
            const uint32_t code = kSiCodes[k], x = sid >= code ? sid - code : P - (code - sid);
            v[SI_IZ + 2 * k] = inv_canonical(x);
            v[SI_IZ + 2 * k + 1] = x == 0;
        }
        const bool cdp = sid == 0x1A;
        if ((sid == 0x10 || cdp) && b < 8) v[SI_BITMAP + b] = 1;
        const bool chk = halt || cdp;
        if (chk) {
            const uint32_t operand = halt ? b : c, msb = byte_of(operand, 3);
            put_word(v + SI_OPERAND, operand);
            uint32_t acc = 1;
#pragma unroll
            for (int i = 0; i < 8; i++) v[SI_RC_BITS + i] = (msb >> i) & 1;
#pragma unroll
            for (int k = 0; k < 6; k++) {
                acc = k == 0 ? v[SI_RC_BITS] * v[SI_RC_BITS + 1] : acc * v[SI_RC_BITS + k + 1];
                v[SI_RC_AND + k] = acc;
            }
        }
        v[SI_RCOP] = chk;
        v[SI_REAL] = 1;
    }
};

// ------------------------------------------------------------------ MiscInstrs (misc/others/trace.rs:81-262)
// MiscEvent dwords: shard, clk, pc, next_pc, opcode, a, b, c, prev_a, hi_record (6: value, shard, timestamp,
// prev_value, prev_shard, prev_timestamp); the opcode-specific columns share one union (MS_SPEC)
enum { MS_SHARD = 0, MS_CLK = 1, MS_PC = 2, MS_NPC = 3, MS_A = 4, MS_PREV_A = 8, MS_B = 12, MS_C = 16, MS_SPEC = 20,
       MS_SEL = 64 };
enum { MD_LO = 0, MD_HI = 4, MD_VAL = 8, MD_VALHI = 12, MD_CARRY = 16, MD_S2HI = 23, MD_S2LO = 27, MD_HIACC = 31 };
constexpr uint32_t OP_INS = 45, OP_MADDU = 46, OP_MSUBU = 47, OP_MADD = 48, OP_MSUB = 49, OP_EXT = 53, OP_TEQ = 54,
                   OP_SEXT = 55;
struct MiscInstrsChip {
    __device__ __forceinline__ void row(uint32_t *v, const uint32_t *e, uint64_t, const Hist &h) const {
#pragma unroll
        for (int c = 0; c < ZKM_MISC_INSTRS_WIDTH; c++) v[c] = 0;
        const bool real = e != nullptr;
        const uint32_t op = real ? e[4] & 0xFF : 0u, a = real ? e[5] : 0u, b = real ? e[6] : 0u;
        const uint32_t c = real ? e[7] : 0u, pa = real ? e[8] : 0u;
        uint32_t *S = v + MS_SPEC;
        // SEXT / TEQ (sext view: most_sig_bit, sig_byte, a_eq_b, is_seb, is_seh)
        const bool half = c > 0;
        const uint32_t sbyte = half ? (b >> 8) & 0xFF : b & 0xFF;
        h.byte(B_MSB, sbyte, 0, real && op == OP_SEXT);
        // EXT (lsb, msbd, sll_val) and INS (lsb, msb, ror_val, srl_val, sll_val, add_val)
        const uint32_t lsb = c & 31, hi5 = c >> 5;
        const bool ext = real && op == OP_EXT, ins = real && op == OP_INS;
        h.byte(B_U8RANGE, lsb, hi5, ext || ins);
        h.byte(B_LTU, lsb + hi5, 32, ext);
        h.byte(B_LTU, lsb, hi5 + 1, ins);
        h.byte(B_LTU, hi5, 32, ins);
        // MADDU / MSUBU / MADD / MSUB: the product plus the (HI, LO) addend as a 64-bit AddDouble
        const bool md = real && op >= OP_MADDU && op <= OP_MSUB;
        const bool sgn = op == OP_MADD || op == OP_MSUB, is_add = op == OP_MADDU || op == OP_MADD;
        const uint64_t prod = sgn ? (uint64_t)((int64_t)(int32_t)b * (int64_t)(int32_t)c) : (uint64_t)b * (uint64_t)c;
        const uint32_t hi_prev = real ? e[12] : 0u, hi_new = real ? e[9] : 0u;
        const uint32_t s2lo = is_add ? pa : a, s2hi = is_add ? hi_prev : hi_new;
        const uint64_t addend = ((uint64_t)s2hi << 32) | s2lo, tot = prod + addend;
        const uint32_t words[6] = {(uint32_t)prod, (uint32_t)(prod >> 32), s2lo, s2hi, (uint32_t)tot,
                                   (uint32_t)(tot >> 32)};
#pragma unroll
        for (int w = 0; w < 6; w++) {
            h.byte(B_U8RANGE, byte_of(words[w], 0), byte_of(words[w], 1), md);
            h.byte(B_U8RANGE, byte_of(words[w], 2), byte_of(words[w], 3), md);
        }
        Access acc{};
        if (md) {  // the HI write at clk + POS_HI
            const uint32_t *r = e + 9;
            acc.on = true;
            acc.value = r[0];
            acc.prev_value = r[3];
            acc.prev_shard = r[4];
            acc.prev_clk = r[5];
            const bool cmp = r[4] == r[1];
            acc.compare = cmp;
            const uint32_t d = (cmp ? r[2] : r[1]) - (cmp ? r[5] : r[4]) - 1u;
            acc.d16 = d & 0xFFFF;
            acc.d8 = (d >> 16) & 0xFF;
        }
        h.byte(B_U16RANGE, acc.d16 >> 8, acc.d16 & 0xFF, md);
        h.byte(B_U8RANGE, 0, acc.d8, md);
        if (!real) return;
        v[MS_PC] = e[2];
        v[MS_NPC] = e[3];
        put_word(v + MS_A, a);
        put_word(v + MS_B, b);
        put_word(v + MS_C, c);
        put_word(v + MS_PREV_A, pa);
        // selectors in MISC_OPS order: SEXT, INS, EXT, MADDU, MSUBU, MADD, MSUB, TEQ
        v[MS_SEL + 0] = op == OP_SEXT;
        v[MS_SEL + 1] = op == OP_INS;
        v[MS_SEL + 2] = op == OP_EXT;
        v[MS_SEL + 3] = op == OP_MADDU;
        v[MS_SEL + 4] = op == OP_MSUBU;
        v[MS_SEL + 5] = op == OP_MADD;
        v[MS_SEL + 6] = op == OP_MSUB;
        v[MS_SEL + 7] = op == OP_TEQ;
        if (op == OP_SEXT || op == OP_TEQ) {
            S[0] = half ? (b & 0xFFFF) >> 15 : (b & 0xFF) >> 7;
            S[1] = sbyte;
            S[2] = a == b;
            S[3] = !half;
            S[4] = half;
        } else if (ext) {
            S[0] = lsb;
            S[1] = hi5;
            const int sh = 31 - (int)lsb - (int)hi5;
            put_word(S + 2, sh >= 0 ? b << sh : 0u);
        } else if (ins) {
            S[0] = lsb;
            S[1] = hi5;
            const uint64_t p = pa;
            const uint32_t ror = (uint32_t)(((p >> lsb) | (p << (32 - lsb))) & 0xFFFFFFFFull);
            const uint32_t srl = (uint32_t)((uint64_t)ror >> (hi5 - lsb + 1));
            const uint32_t sll = (uint32_t)(((uint64_t)b << (31 - hi5 + lsb)) & 0xFFFFFFFFull);
            put_word(S + 2, ror);
            put_word(S + 6, srl);
            put_word(S + 10, sll);
            put_word(S + 14, srl + sll);
        } else if (md) {
            v[MS_SHARD] = e[0];
            v[MS_CLK] = e[1];
            uint32_t cy = 0;
#pragma unroll
            for (int j = 0; j < 7; j++) {
                cy = ((uint32_t)(prod >> (8 * j)) & 0xFF) + ((uint32_t)(addend >> (8 * j)) & 0xFF) + cy > 255;
                S[MD_CARRY + j] = cy;
            }
            put_word(S + MD_LO, words[0]);
            put_word(S + MD_HI, words[1]);
            put_word(S + MD_VAL, words[4]);
            put_word(S + MD_VALHI, words[5]);
            put_word(S + MD_S2HI, s2hi);
            put_word(S + MD_S2LO, s2lo);
            put_word(S + MD_HIACC, acc.prev_value);
            put_access(S, MD_HIACC + 4, acc);
        }
    }
};

// ------------------------------------------------------------------ ShaExtend (sha256/extend/trace.rs:29-150)
// One row per extension step: zkm_sha_extend_row dwords: shard, clk (the call's), w_ptr, then the reads of
// w[i-15], w[i-2], w[i-16], w[i-7] (MemoryReadRecord: value, shard, timestamp, prev_shard, prev_timestamp)
// and the write of w[i] (MemoryWriteRecord: value, shard, timestamp, prev_value, prev_shard, prev_timestamp)
enum { SE_SHARD = 0, SE_CLK = 1, SE_WPTR = 2, SE_I = 3, SE_C16 = 4, SE_C16S = 5, SE_C16E = 7, SE_C48 = 9, SE_C48S = 12,
       SE_C48E = 13, SE_W15 = 14, SE_RR7 = 23, SE_RR18 = 35, SE_RS3 = 47, SE_S0I = 59, SE_S0 = 63, SE_W2 = 67,
       SE_RR17 = 76, SE_RR19 = 88, SE_RS10 = 100, SE_S1I = 112, SE_S1 = 116, SE_W16 = 120, SE_W7 = 129, SE_S2 = 138,
       SE_WI = 162, SE_REAL = 175 };
constexpr uint32_t G16 = 148625052u;  // KoalaBear::two_adic_generator(4), order 16

// MemoryAccessCols of a read record (value, shard, timestamp, prev_shard, prev_timestamp) at its timestamp
__device__ __forceinline__ Access access_read(const uint32_t *r) {
    Access a{};
    a.on = true;
    a.value = a.prev_value = r[0];
    a.prev_shard = r[3];
    a.prev_clk = r[4];
    const bool cmp = r[3] == r[1];
    a.compare = cmp;
    const uint32_t d = (cmp ? r[2] : r[1]) - (cmp ? r[4] : r[3]) - 1u;
    a.d16 = d & 0xFFFF;
    a.d8 = (d >> 16) & 0xFF;
    return a;
}
__device__ __forceinline__ Access access_write(const uint32_t *r) {  // MemoryWriteRecord
    Access a{};
    a.on = true;
    a.value = r[0];
    a.prev_value = r[3];
    a.prev_shard = r[4];
    a.prev_clk = r[5];
    const bool cmp = r[4] == r[1];
    a.compare = cmp;
    const uint32_t d = (cmp ? r[2] : r[1]) - (cmp ? r[5] : r[4]) - 1u;
    a.d16 = d & 0xFFFF;
    a.d8 = (d >> 16) & 0xFF;
    return a;
}

// FixedRotateRightOperation / FixedShiftRightOperation::populate: value, shift, carry (4 bytes each) at v,
// ShrCarry lookups; returns the result word
template <int ROT, bool ROTATE>
__device__ __forceinline__ uint32_t shr_carry(uint32_t *v, uint32_t x, const Hist &h, bool on) {
    constexpr int NB = ROT / 8, NBITS = ROT % 8;
    constexpr uint32_t MULT = 1u << (8 - NBITS);
    uint32_t rb[4], sh[4], ca[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        rb[i] = ROTATE ? byte_of(x, (i + NB) % 4) : (i + NB < 4 ? byte_of(x, i + NB) : 0u);
        sh[i] = rb[i] >> NBITS;
        ca[i] = rb[i] & ((1u << NBITS) - 1);
        h.byte(B_SHRCARRY, rb[i], NBITS, on);
    }
    uint32_t w = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t val = i < 3 ? sh[i] + ca[i + 1] * MULT : sh[3] + (ROTATE ? ca[0] * MULT : 0u);
        v[i] = val;
        v[4 + i] = sh[i];
        v[8 + i] = ca[i];
        w |= (val & 0xFF) << (8 * i);
    }
    return w;
}
__device__ __forceinline__ uint32_t xor_word(uint32_t *v, uint32_t a, uint32_t b, const Hist &h, bool on) {
#pragma unroll
    for (int i = 0; i < 4; i++) {
        v[i] = byte_of(a, i) ^ byte_of(b, i);
        h.byte(B_XOR, byte_of(a, i), byte_of(b, i), on);
    }
    return a ^ b;
}

struct ShaExtendChip {
    // the 16-cycle flag values by (row + 1) mod 16: g^k and the inverses of g^k - g and g^k - 1 (0 for 0),
    // computed once on the host (16 distinct values: no per-row field inversion)
    uint32_t c16[16], inv_s[16], inv_e[16];
    __device__ __forceinline__ void row(uint32_t *v, const uint32_t *e, uint64_t r, const Hist &h) const {
#pragma unroll
        for (int c = 0; c < ZKM_SHA_EXTEND_WIDTH; c++) v[c] = 0;
        const bool real = e != nullptr;
        // populate_flags(i) (flags.rs:13-34), for every row
        const uint32_t k16 = (uint32_t)((r + 1) % 16);
        const uint32_t c16v = c16[k16];
        const uint32_t j = 16 + (uint32_t)(r % 48);
        const bool xs0 = k16 == 1, xe0 = k16 == 0;  // g^k = g, g^k = 1
        v[SE_I] = j;
        v[SE_C16] = c16v;
        v[SE_C16S] = inv_s[k16];
        v[SE_C16S + 1] = xs0;
        v[SE_C16E] = inv_e[k16];
        v[SE_C16E + 1] = xe0;
        const uint32_t third = (j - 16) / 16;
        v[SE_C48 + third] = 1;
        v[SE_C48S] = (third == 0 && xs0 && real);
        v[SE_C48E] = (third == 2 && xe0 && real);
        Access acc[5] = {};
        if (real) {
            v[SE_SHARD] = e[0];
            v[SE_CLK] = e[1];
            v[SE_WPTR] = e[2];
            const int bases[4] = {SE_W15, SE_W2, SE_W16, SE_W7};
#pragma unroll
            for (int k = 0; k < 4; k++) {
                acc[k] = access_read(e + 3 + 5 * k);
                put_access(v, bases[k], acc[k]);
            }
            acc[4] = access_write(e + 23);
            put_word(v + SE_WI, acc[4].prev_value);
            put_access(v, SE_WI + 4, acc[4]);
        }
        const uint32_t w15 = acc[0].value, w2 = acc[1].value, w16 = acc[2].value, w7 = acc[3].value;
        const uint32_t rr7 = shr_carry<7, true>(v + SE_RR7, w15, h, real);
        const uint32_t rr18 = shr_carry<18, true>(v + SE_RR18, w15, h, real);
        const uint32_t rs3 = shr_carry<3, false>(v + SE_RS3, w15, h, real);
        const uint32_t s0 = xor_word(v + SE_S0, xor_word(v + SE_S0I, rr7, rr18, h, real), rs3, h, real);
        const uint32_t rr17 = shr_carry<17, true>(v + SE_RR17, w2, h, real);
        const uint32_t rr19 = shr_carry<19, true>(v + SE_RR19, w2, h, real);
        const uint32_t rs10 = shr_carry<10, false>(v + SE_RS10, w2, h, real);
        const uint32_t s1 = xor_word(v + SE_S1, xor_word(v + SE_S1I, rr17, rr19, h, real), rs10, h, real);
        // Add4Operation::populate(w[i-16], s0, w[i-7], s1): bytes, carries, one-hot carries, U8 range checks
        const uint32_t ins[4] = {w16, s0, w7, s1};
        uint32_t carry = 0, sum = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            uint32_t t = carry;
#pragma unroll
            for (int k = 0; k < 4; k++) t += byte_of(ins[k], i);
            carry = t >> 8;
            sum |= (t & 0xFF) << (8 * i);
            if (real) {
                v[SE_S2 + i] = t & 0xFF;
#pragma unroll
                for (int k = 0; k < 4; k++) v[SE_S2 + 4 + 4 * k + i] = carry == (uint32_t)k;
                v[SE_S2 + 20 + i] = carry;
            }
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            h.byte(B_U8RANGE, byte_of(ins[k], 0), byte_of(ins[k], 1), real);
            h.byte(B_U8RANGE, byte_of(ins[k], 2), byte_of(ins[k], 3), real);
        }
        h.byte(B_U8RANGE, byte_of(sum, 0), byte_of(sum, 1), real);
        h.byte(B_U8RANGE, byte_of(sum, 2), byte_of(sum, 3), real);
#pragma unroll
        for (int k = 0; k < 5; k++) {
            h.byte(B_U16RANGE, acc[k].d16 >> 8, acc[k].d16 & 0xFF, real);
            h.byte(B_U8RANGE, 0, acc[k].d8, real);
        }
        if (real) v[SE_REAL] = 1;
        else {  // padding rows keep only the flags
#pragma unroll
            for (int c = SE_W15; c < ZKM_SHA_EXTEND_WIDTH; c++) v[c] = 0;
        }
    }
};

// ------------------------------------------------------------------ Uint256MulMod (uint256/air.rs:103-186)
// Uint256MulCols: shard, clk, x_ptr, y_ptr, x (8 MemoryWriteCols), y and modulus (8 MemoryReadCols each),
// IsZeroOperation (inverse, result), modulus_is_not_zero, FieldOpCols<U256Field> (result 32, carry 32,
// witness low 63, witness high 63), FieldLtCols (byte flags 32, the compared bytes), is_real.  One thread
// per row (the big-integer work is sequential): x y as 16 32-bit limbs, divided by the modulus (Knuth's
// algorithm D), the vanishing polynomial x(X) y(X) - r(X) - c(X) m(X) over byte limbs divided by X - 256
// (field_op.rs populate_with_modulus, util.rs compute_root_quotient_and_shift).
enum { U2_SHARD = 0, U2_CLK = 1, U2_XPTR = 2, U2_YPTR = 3, U2_X = 4, U2_Y = U2_X + 8 * 13, U2_M = U2_Y + 8 * 9,
       U2_IZINV = U2_M + 8 * 9, U2_IZRES = U2_IZINV + 1, U2_NZ = U2_IZRES + 1, U2_OUT = U2_NZ + 1, U2_LT = U2_OUT + 190,
       U2_REAL = U2_LT + 34, U2_EV = 4 + 40 + 40 + 48, U2_NW = 63, U2_OFFSET = 1 << 14 };
static_assert(U2_REAL + 1 == ZKM_UINT256_MUL_WIDTH, "Uint256MulCols layout");

// u (m limbs) = q v + r, v (n limbs, v[n-1] != 0); q gets m - n + 1 limbs, r n limbs (Knuth D, base 2^32)
__device__ inline void divmod_limbs(const uint32_t *u, int m, const uint32_t *v, int n, uint32_t *q, uint32_t *r) {
    if (n == 1) {
        uint64_t k = 0;
        for (int j = m - 1; j >= 0; j--) {
            const uint64_t t = (k << 32) | u[j];
            q[j] = (uint32_t)(t / v[0]);
            k = t - (uint64_t)q[j] * v[0];
        }
        r[0] = (uint32_t)k;
        return;
    }
    uint32_t un[17], vn[8];
    const int s = __clz(v[n - 1]);
    for (int i = n - 1; i > 0; i--) vn[i] = (uint32_t)(((uint64_t)v[i] << s) | ((uint64_t)v[i - 1] >> (32 - s)));
    vn[0] = v[0] << s;
    un[m] = (uint32_t)((uint64_t)u[m - 1] >> (32 - s));
    for (int i = m - 1; i > 0; i--) un[i] = (uint32_t)(((uint64_t)u[i] << s) | ((uint64_t)u[i - 1] >> (32 - s)));
    un[0] = u[0] << s;
    for (int j = m - n; j >= 0; j--) {
        const uint64_t num = ((uint64_t)un[j + n] << 32) | un[j + n - 1];
        uint64_t qhat = num / vn[n - 1], rhat = num - qhat * vn[n - 1];
        while (qhat >> 32 || qhat * vn[n - 2] > ((rhat << 32) | un[j + n - 2])) {
            qhat--;
            rhat += vn[n - 1];
            if (rhat >> 32) break;
        }
        int64_t t;
        uint64_t k = 0;
        for (int i = 0; i < n; i++) {  // un[j..j+n] -= qhat vn
            const uint64_t p = qhat * vn[i];
            t = (int64_t)un[i + j] - (int64_t)k - (int64_t)(p & 0xFFFFFFFFu);
            un[i + j] = (uint32_t)t;
            k = (p >> 32) - (uint64_t)(t >> 32);
        }
        t = (int64_t)un[j + n] - (int64_t)k;
        un[j + n] = (uint32_t)t;
        q[j] = (uint32_t)qhat;
        if (t < 0) {  // qhat was one too large: add vn back
            q[j]--;
            uint64_t c = 0;
            for (int i = 0; i < n; i++) {
                const uint64_t w = (uint64_t)un[i + j] + vn[i] + c;
                un[i + j] = (uint32_t)w;
                c = w >> 32;
            }
            un[j + n] += (uint32_t)c;
        }
    }
    for (int i = 0; i < n - 1; i++) r[i] = (uint32_t)(((uint64_t)un[i] >> s) | ((uint64_t)un[i + 1] << (32 - s)));
    r[n - 1] = un[n - 1] >> s;
}

__device__ __forceinline__ void byte_add(uint32_t *bm, uint32_t op, uint32_t b, uint32_t c) {
    if (bm) atomicAdd(bm + (((b << 8) | c) * BYTE_COLS + op), 1u);
}

// FieldOpCols<U256Field> at o for a b + c = res + car M (c nullable; M = the byte limbs of m, or X^32 for
// 2^256 when m is null): result and carry bytes, the witness limbs of the vanishing polynomial
// a(X) b(X) + c(X) - res(X) - car(X) M(X) divided by X - 256 and shifted by the offset (field_op.rs
// populate_with_modulus / populate_mul_and_carry, util.rs compute_root_quotient_and_shift), and the U8
// range checks of the four limb groups (pairs, a trailing single with 0) into bm (nullable)
__device__ inline void u256_field_op(uint32_t *o, const uint32_t a[8], const uint32_t b[8], const uint32_t *c,
                                     const uint32_t res[8], const uint32_t car[8], const uint32_t *m, uint32_t *bm) {
    int64_t van[U2_NW + 1];
    for (int k = 0; k <= U2_NW; k++) van[k] = 0;
    for (int i = 0; i < 32; i++) {
        const int64_t ai = byte_of(a[i >> 2], i & 3), ci = byte_of(car[i >> 2], i & 3);
        for (int j = 0; j < 32; j++) {
            van[i + j] += ai * (int64_t)byte_of(b[j >> 2], j & 3);
            if (m) van[i + j] -= ci * (int64_t)byte_of(m[j >> 2], j & 3);
        }
        van[i] -= byte_of(res[i >> 2], i & 3);
        if (c) van[i] += byte_of(c[i >> 2], i & 3);
        if (!m) van[i + 32] -= ci;  // M(X) = X^32
    }
    int64_t qw = van[U2_NW];
    uint32_t *W = o + 64;
    for (int k = U2_NW - 1; k >= 0; k--) {  // q_k = van_{k+1} + 256 q_{k+1}; column k = q_k + offset
        const uint32_t w = (uint32_t)(qw + U2_OFFSET);
        W[k] = w & 0xFF;
        W[U2_NW + k] = w >> 8;
        if (k) qw = van[k] + 256 * qw;
    }
    for (int i = 0; i < 32; i++) {
        o[i] = byte_of(res[i >> 2], i & 3);
        o[32 + i] = byte_of(car[i >> 2], i & 3);
    }
    for (int blk = 0; blk < 4; blk++) {
        const uint32_t *g = o + (blk < 2 ? 32 * blk : 64 + U2_NW * (blk - 2));
        const int len = blk < 2 ? 32 : U2_NW;
        for (int j = 0; j + 1 < len; j += 2) byte_add(bm, B_U8RANGE, g[j], g[j + 1]);
        if (len & 1) byte_add(bm, B_U8RANGE, g[len - 1], 0);
    }
}

__global__ __launch_bounds__(128) void k_uint256_rows(const uint32_t *__restrict__ ev, uint64_t n,
                                                      uint32_t *__restrict__ out, uint64_t height, uint32_t *bm) {
    const uint64_t row = (uint64_t)blockIdx.x * 128 + threadIdx.x;
    if (row >= height) return;
    uint32_t *v = out + row * ZKM_UINT256_MUL_WIDTH;
    for (int c = 0; c < ZKM_UINT256_MUL_WIDTH; c++) v[c] = 0;
    if (row >= n) {  // x = y = 0 mod 2^256: result, carry, vanishing 0; witness limbs = the offset
        for (int k = 0; k < U2_NW; k++) v[U2_OUT + 64 + U2_NW + k] = U2_OFFSET >> 8;
        return;
    }
    const uint32_t *e = ev + row * U2_EV;
    const uint32_t shard = e[0], clk = e[1];
    v[U2_SHARD] = shard;
    v[U2_CLK] = clk;
    v[U2_XPTR] = e[2];
    v[U2_YPTR] = e[3];
    v[U2_REAL] = 1;
    uint32_t x[8], y[8], m[8];
    for (int i = 0; i < 8; i++) {
        const Access ya = access_read(e + 4 + 5 * i), ma = access_read(e + 44 + 5 * i), xa = access_write(e + 84 + 6 * i);
        y[i] = ya.value;
        m[i] = ma.value;
        x[i] = xa.prev_value;
        put_access(v, U2_Y + 9 * i, ya);
        put_access(v, U2_M + 9 * i, ma);
        put_word(v + U2_X + 13 * i, xa.prev_value);
        put_access(v, U2_X + 13 * i + 4, xa);
        const Access as[3] = {ya, ma, xa};
        for (int k = 0; k < 3; k++) {
            byte_add(bm, B_U16RANGE, as[k].d16 >> 8, as[k].d16 & 0xFF);
            byte_add(bm, B_U8RANGE, 0, as[k].d8);
        }
    }
    // IsZeroOperation on the modulus's byte sum
    uint32_t bsum = 0;
    for (int i = 0; i < 32; i++) bsum += byte_of(m[i >> 2], i & 3);
    const bool mz = bsum == 0;
    v[U2_IZRES] = mz;
    v[U2_NZ] = !mz;
    v[U2_IZINV] = mz ? 0u : kb::from_mont(kb::inv(kb::to_mont(bsum)));
    // x y = carry m + result (m = 2^256 when zero)
    uint32_t prod[16];
    for (int i = 0; i < 16; i++) prod[i] = 0;
    for (int i = 0; i < 8; i++) {
        uint64_t c = 0;
        for (int j = 0; j < 8; j++) {
            const uint64_t t = (uint64_t)x[i] * y[j] + prod[i + j] + c;
            prod[i + j] = (uint32_t)t;
            c = t >> 32;
        }
        prod[i + 8] = (uint32_t)c;
    }
    uint32_t res[8] = {0, 0, 0, 0, 0, 0, 0, 0}, car[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (mz) {
        for (int i = 0; i < 8; i++) {
            res[i] = prod[i];
            car[i] = prod[8 + i];
        }
    } else {
        int nm = 8;
        while (m[nm - 1] == 0) nm--;
        uint32_t q[16], r[8];
        divmod_limbs(prod, 16, m, nm, q, r);
        for (int i = 0; i < nm; i++) res[i] = r[i];
        for (int i = 0; i < 8; i++) car[i] = q[i];  // below 2^256 for operands below the modulus
    }
    u256_field_op(v + U2_OUT, x, y, nullptr, res, car, mz ? nullptr : m, bm);
    // FieldLtCols: result < m at its most significant differing byte (only when m != 0)
    if (!mz) {
        for (int k = 31; k >= 0; k--) {
            const uint32_t a = byte_of(res[k >> 2], k & 3), b = byte_of(m[k >> 2], k & 3);
            if (a < b) {
                v[U2_LT + k] = 1;
                v[U2_LT + 32] = a;
                v[U2_LT + 33] = b;
                break;
            }
        }
        byte_add(bm, B_LTU, v[U2_LT + 32], v[U2_LT + 33]);
    }
}

// ------------------------------------------------------------------ U256XU2048Mul (u256x2048_mul/air.rs:109-213)
// U256x2048MulCols: shard, clk, a_ptr, b_ptr, lo_ptr, hi_ptr, the A2 / A3 register reads, a (8 reads), b (64
// reads), lo (64 writes), hi (8 writes), eight FieldOpCols (a b_k + carry_{k-1} = lo_k + carry_k 2^256), is_real.
enum { UX_APTR = 2, UX_BPTR = 3, UX_LOPTR = 4, UX_HIPTR = 5, UX_LOREG = 6, UX_HIREG = 15, UX_A = 24, UX_B = UX_A + 8 * 9,
       UX_LO = UX_B + 64 * 9, UX_HI = UX_LO + 64 * 13, UX_OUT = UX_HI + 8 * 13, UX_REAL = UX_OUT + 8 * 190,
       UX_EV = 6 + 10 + 40 + 320 + 384 + 48 };
static_assert(UX_REAL + 1 == ZKM_U256XU2048_MUL_WIDTH, "U256x2048MulCols layout");

__global__ __launch_bounds__(128) void k_u256x2048_rows(const uint32_t *__restrict__ ev, uint64_t n,
                                                        uint32_t *__restrict__ out, uint64_t height, uint32_t *bm) {
    const uint64_t row = (uint64_t)blockIdx.x * 128 + threadIdx.x;
    if (row >= height) return;
    uint32_t *v = out + row * ZKM_U256XU2048_MUL_WIDTH;
    for (int c = 0; c < ZKM_U256XU2048_MUL_WIDTH; c++) v[c] = 0;
    if (row >= n) {  // eight mul-and-carry operations of zeros: witness limbs = the offset
        for (int k = 0; k < 8; k++)
            for (int j = 0; j < U2_NW; j++) v[UX_OUT + 190 * k + 64 + U2_NW + j] = U2_OFFSET >> 8;
        return;
    }
    const uint32_t *e = ev + row * UX_EV;
    for (int i = 0; i < 6; i++) v[i] = e[i];
    v[UX_REAL] = 1;
    auto acc = [&](int col, const Access &a) {
        put_access(v, col, a);
        byte_add(bm, B_U16RANGE, a.d16 >> 8, a.d16 & 0xFF);
        byte_add(bm, B_U8RANGE, 0, a.d8);
    };
    acc(UX_LOREG, access_read(e + 6));
    acc(UX_HIREG, access_read(e + 11));
    uint32_t a[8];
    for (int i = 0; i < 8; i++) {
        const Access r = access_read(e + 16 + 5 * i);
        a[i] = r.value;
        acc(UX_A + 9 * i, r);
    }
    for (int i = 0; i < 64; i++) acc(UX_B + 9 * i, access_read(e + 56 + 5 * i));
    for (int i = 0; i < 72; i++) {
        const Access w = access_write(e + 376 + 6 * i);
        const int col = i < 64 ? UX_LO + 13 * i : UX_HI + 13 * (i - 64);
        put_word(v + col, w.prev_value);
        acc(col + 4, w);
    }
    uint32_t carry[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int k = 0; k < 8; k++) {
        uint32_t b[8], p[16];
        for (int i = 0; i < 8; i++) b[i] = e[56 + 5 * (8 * k + i)];
        for (int i = 0; i < 16; i++) p[i] = i < 8 ? carry[i] : 0u;  // a b_k + carry
        for (int i = 0; i < 8; i++) {
            uint64_t c = 0;
            for (int j = 0; j < 8; j++) {
                const uint64_t t = (uint64_t)a[i] * b[j] + p[i + j] + c;
                p[i + j] = (uint32_t)t;
                c = t >> 32;
            }
            for (int j = i + 8; c && j < 16; j++) {
                const uint64_t t = (uint64_t)p[j] + c;
                p[j] = (uint32_t)t;
                c = t >> 32;
            }
        }
        uint32_t prev[8];
        for (int i = 0; i < 8; i++) prev[i] = carry[i];
        u256_field_op(v + UX_OUT + 190 * k, a, b, prev, p, p + 8, nullptr, bm);
        for (int i = 0; i < 8; i++) carry[i] = p[8 + i];
    }
}

// ------------------------------------------------------------------ FpOpAssign (fptower/fp.rs:90-160)
// Generic emulated-field pieces over NL-byte limbs (bn254: 32, bls12-381: 48): big integers as 32-bit words.
// u (MU words) = q v + r with v of NV words, the top one nonzero (Knuth D; q MU - NV + 1 words, r NV words)
template <int MU, int NVMAX>
__device__ inline void divmod_words(const uint32_t *u, const uint32_t *v, int nv, uint32_t *q, uint32_t *r) {
    if (nv == 1) {
        uint64_t k = 0;
        for (int j = MU - 1; j >= 0; j--) {
            const uint64_t t = (k << 32) | u[j];
            q[j] = (uint32_t)(t / v[0]);
            k = t - (uint64_t)q[j] * v[0];
        }
        r[0] = (uint32_t)k;
        return;
    }
    uint32_t un[MU + 1], vn[NVMAX];
    const int s = __clz(v[nv - 1]);
    for (int i = nv - 1; i > 0; i--) vn[i] = (uint32_t)(((uint64_t)v[i] << s) | ((uint64_t)v[i - 1] >> (32 - s)));
    vn[0] = v[0] << s;
    un[MU] = (uint32_t)((uint64_t)u[MU - 1] >> (32 - s));
    for (int i = MU - 1; i > 0; i--) un[i] = (uint32_t)(((uint64_t)u[i] << s) | ((uint64_t)u[i - 1] >> (32 - s)));
    un[0] = u[0] << s;
    for (int j = MU - nv; j >= 0; j--) {
        const uint64_t num = ((uint64_t)un[j + nv] << 32) | un[j + nv - 1];
        uint64_t qhat = num / vn[nv - 1], rhat = num - qhat * vn[nv - 1];
        while (qhat >> 32 || qhat * vn[nv - 2] > ((rhat << 32) | un[j + nv - 2])) {
            qhat--;
            rhat += vn[nv - 1];
            if (rhat >> 32) break;
        }
        int64_t t;
        uint64_t k = 0;
        for (int i = 0; i < nv; i++) {
            const uint64_t p = qhat * vn[i];
            t = (int64_t)un[i + j] - (int64_t)k - (int64_t)(p & 0xFFFFFFFFu);
            un[i + j] = (uint32_t)t;
            k = (p >> 32) - (uint64_t)(t >> 32);
        }
        t = (int64_t)un[j + nv] - (int64_t)k;
        un[j + nv] = (uint32_t)t;
        q[j] = (uint32_t)qhat;
        if (t < 0) {
            q[j]--;
            uint64_t c = 0;
            for (int i = 0; i < nv; i++) {
                const uint64_t w = (uint64_t)un[i + j] + vn[i] + c;
                un[i + j] = (uint32_t)w;
                c = w >> 32;
            }
            un[j + nv] += (uint32_t)c;
        }
    }
    for (int i = 0; i < nv - 1; i++) r[i] = (uint32_t)(((uint64_t)un[i] >> s) | ((uint64_t)un[i + 1] << (32 - s)));
    r[nv - 1] = un[nv - 1] >> s;
}

// x (NX words) mod m (W words, canonical modulus): r (W words), q (NX - nv + 1 words, may be null)
template <int NX, int W>
__device__ inline void mod_words(const uint32_t *x, const uint32_t *m, uint32_t *r, uint32_t *qout) {
    int nv = W;
    while (m[nv - 1] == 0) nv--;
    uint32_t q[NX], rr[W];
    for (int i = 0; i < W; i++) rr[i] = 0;
    divmod_words<NX, W>(x, m, nv, q, rr);
    for (int i = 0; i < W; i++) r[i] = rr[i];
    if (qout)
        for (int i = 0; i < NX - nv + 1 && i < W; i++) qout[i] = q[i];
}

// FieldOpCols<NL bytes, NW witness limbs> at o: result `res_col`, carry, and the witness of the vanishing
// polynomial of a (op) b + c - mres - carry m, op = mul or add (field_op.rs populate_with_modulus: sub and div
// are populated as additions / products of the result); U8 range checks into bm
// FieldOpCols-shaped columns at o from a vanishing polynomial van (NW + 1 coefficients): result `res_col`,
// carry, the witness limbs of van / (X - 256) shifted by the offset, and the U8 range checks of the four limb
// groups (pairs, a trailing single with 0) into bm; `u8res` (nullable) replaces the result limbs in the range
// check (FieldSqrtCols checks its multiplication's result)
template <int NL, int NW, int OFF>
__device__ inline void field_cols(uint32_t *o, const int64_t *van, const uint32_t *res_col, const uint32_t *car,
                                  uint32_t *bm, const uint32_t *u8res = nullptr) {
    int64_t qw = van[NW];
    uint32_t *Wc = o + 2 * NL;
    for (int k = NW - 1; k >= 0; k--) {
        const uint32_t w = (uint32_t)(qw + OFF);
        Wc[k] = w & 0xFF;
        Wc[NW + k] = w >> 8;
        if (k) qw = van[k] + 256 * qw;
    }
    for (int i = 0; i < NL; i++) {
        o[i] = byte_of(res_col[i >> 2], i & 3);
        o[NL + i] = byte_of(car[i >> 2], i & 3);
    }
    for (int blk = 0; blk < 4; blk++) {
        const uint32_t *g = o + (blk < 2 ? NL * blk : 2 * NL + NW * (blk - 2));
        const int len = blk < 2 ? NL : NW;
        for (int j = 0; j + 1 < len; j += 2) {
            if (blk == 0 && u8res) byte_add(bm, B_U8RANGE, byte_of(u8res[j >> 2], j & 3), byte_of(u8res[(j + 1) >> 2], (j + 1) & 3));
            else byte_add(bm, B_U8RANGE, g[j], g[j + 1]);
        }
        if (len & 1) byte_add(bm, B_U8RANGE, g[len - 1], 0);
    }
}

// van += sign a(X) b(X) over byte limbs
template <int NL, int NW>
__device__ inline void van_mul(int64_t *van, const uint32_t *a, const uint32_t *b, int sign) {
    for (int i = 0; i < NL; i++) {
        const int64_t ai = sign * (int64_t)byte_of(a[i >> 2], i & 3);
        for (int j = 0; j < NL; j++) van[i + j] += ai * (int64_t)byte_of(b[j >> 2], j & 3);
    }
}

// FieldOpCols<NL bytes, NW witness limbs> at o: result `res_col`, carry, and the witness of the vanishing
// polynomial of a (op) b - mres - carry m, op = mul or add (field_op.rs populate_with_modulus: sub and div
// are populated as additions / products of the result); U8 range checks into bm
template <int NL, int NW, int OFF>
__device__ inline void field_op_cols(uint32_t *o, const uint32_t *a, const uint32_t *b, bool mul, const uint32_t *res_col,
                                     const uint32_t *mres, const uint32_t *car, const uint32_t *m, uint32_t *bm,
                                     const uint32_t *u8res = nullptr) {
    int64_t van[NW + 1];
    for (int k = 0; k <= NW; k++) van[k] = 0;
    if (mul) {
        van_mul<NL, NW>(van, a, b, 1);
    } else {
        for (int i = 0; i < NL; i++) van[i] += (int64_t)byte_of(a[i >> 2], i & 3) + byte_of(b[i >> 2], i & 3);
    }
    van_mul<NL, NW>(van, car, m, -1);
    for (int i = 0; i < NL; i++) van[i] -= byte_of(mres[i >> 2], i & 3);
    field_cols<NL, NW, OFF>(o, van, res_col, car, bm, u8res);
}

// FpOpCols: is_real, shard, clk, is_add, is_sub, is_mul, x_ptr, y_ptr, x (W MemoryWriteCols), y (W
// MemoryReadCols), FieldOpCols.  zkm_fp_op_event dwords: shard, clk, x_ptr, y_ptr, op, y reads (12 x 5), x
// writes (12 x 6) -- the first W of each used
enum { FO_REAL = 0, FO_SHARD = 1, FO_CLK = 2, FO_ADD = 3, FO_SUB = 4, FO_MUL = 5, FO_XPTR = 6, FO_YPTR = 7, FO_X = 8,
       FO_EV = 5 + 60 + 72 };
struct FpMod {
    uint32_t w[12];
};
// the base field moduli (crates/curves/src/weierstrass/{bn254,bls12_381}.rs FieldParameters), 32-bit words
constexpr FpMod kBn254{{0xd87cfd47u, 0x3c208c16u, 0x6871ca8du, 0x97816a91u, 0x8181585du, 0xb85045b6u, 0xe131a029u,
                        0x30644e72u, 0, 0, 0, 0}};
constexpr FpMod kSecp256k1{{0xfffffc2fu, 0xfffffffeu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu,
                            0xffffffffu, 0, 0, 0, 0}};
constexpr FpMod kSecp256r1{{0xffffffffu, 0xffffffffu, 0xffffffffu, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000001u,
                            0xffffffffu, 0, 0, 0, 0}};
constexpr FpMod kSqrtExpK1{{0xbfffff0cu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x3fffffffu, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u}};
constexpr FpMod kGenXK1{{0x16f81798u, 0x59f2815bu, 0x2dce28d9u, 0x029bfcdbu, 0xce870b07u, 0x55a06295u, 0xf9dcbbacu, 0x79be667eu, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u}};
constexpr FpMod kCurveAK1{{0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u}};
constexpr FpMod kCurveBK1{{0x00000007u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u}};
constexpr FpMod kSqrtExpR1{{0x00000000u, 0x00000000u, 0x40000000u, 0x00000000u, 0x00000000u, 0x40000000u, 0xc0000000u, 0x3fffffffu, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u}};
constexpr FpMod kGenXR1{{0xd898c296u, 0xf4a13945u, 0x2deb33a0u, 0x77037d81u, 0x63a440f2u, 0xf8bce6e5u, 0xe12c4247u, 0x6b17d1f2u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u}};
constexpr FpMod kCurveAR1{{0xfffffffcu, 0xffffffffu, 0xffffffffu, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000001u, 0xffffffffu, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u}};
constexpr FpMod kCurveBR1{{0x27d2604bu, 0x3bce3c3eu, 0xcc53b0f6u, 0x651d06b0u, 0x769886bcu, 0xb3ebbd55u, 0xaa3a93e7u, 0x5ac635d8u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u}};
constexpr FpMod kSqrtExpBLS{{0xffffeaabu, 0xee7fbfffu, 0xac54ffffu, 0x07aaffffu, 0x3dac3d89u, 0xd9cc34a8u, 0x3ce144afu, 0xd91dd2e1u, 0x90d2eb35u, 0x92c6e9edu, 0x8e5ff9a6u, 0x0680447au}};
constexpr FpMod kGenXBLS{{0xdb22c6bbu, 0xfb3af00au, 0xf97a1aefu, 0x6c55e83fu, 0x171bac58u, 0xa14e3a3fu, 0x9774b905u, 0xc3688c4fu, 0x4fa9ac0fu, 0x2695638cu, 0x3197d794u, 0x17f1d3a7u}};
constexpr FpMod kCurveABLS{{0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u}};
constexpr FpMod kCurveBBLS{{0x00000004u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u}};
constexpr FpMod kEd25519{{0xffffffedu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x7fffffffu, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u}};
constexpr FpMod kEdD{{0x135978a3u, 0x75eb4dcau, 0x4141d8abu, 0x00700a4du, 0x7779e898u, 0x8cc74079u, 0x2b6ffe73u, 0x52036ceeu, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u}};
constexpr FpMod kEdSqrtExp{{0xfffffffeu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x0fffffffu, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u}};
constexpr FpMod kEdSqrtM1{{0x4a0ea0b0u, 0xc4ee1b27u, 0xad2fe478u, 0x2f431806u, 0x3dfbd7a7u, 0x2b4d0099u, 0x4fc1df0bu, 0x2b832480u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u}};
constexpr FpMod kBls{{0xffffaaabu, 0xb9feffffu, 0xb153ffffu, 0x1eabfffeu, 0xf6b0f624u, 0x6730d2a0u, 0xf38512bfu,
                      0x64774b84u, 0x434bacd7u, 0x4b1ba7b6u, 0x397fe69au, 0x1a0111eau}};
// W-word helpers for the modular inverse (binary extended Euclid; p odd)
template <int W>
__device__ inline bool w_is(const uint32_t *u, uint32_t x) {
    bool r = u[0] == x;
    for (int i = 1; i < W; i++) r = r && u[i] == 0;
    return r;
}
template <int W>
__device__ inline void w_shr1(uint32_t *u, uint32_t top) {
    for (int i = 0; i < W - 1; i++) u[i] = (u[i] >> 1) | (u[i + 1] << 31);
    u[W - 1] = (u[W - 1] >> 1) | (top << 31);
}
template <int W>
__device__ inline bool w_ge(const uint32_t *a, const uint32_t *b) {
    for (int i = W - 1; i >= 0; i--)
        if (a[i] != b[i]) return a[i] > b[i];
    return true;
}
template <int W>
__device__ inline uint32_t w_sub(uint32_t *a, const uint32_t *b) {  // a -= b, returns the borrow
    int64_t bw = 0;
    for (int i = 0; i < W; i++) {
        const int64_t d = (int64_t)a[i] - b[i] - bw;
        a[i] = (uint32_t)d;
        bw = d < 0;
    }
    return (uint32_t)bw;
}
template <int W>
__device__ inline uint32_t w_add(uint32_t *a, const uint32_t *b) {  // a += b, returns the carry
    uint64_t c = 0;
    for (int i = 0; i < W; i++) {
        const uint64_t t = (uint64_t)a[i] + b[i] + c;
        a[i] = (uint32_t)t;
        c = t >> 32;
    }
    return (uint32_t)c;
}
// a^-1 mod p for 0 < a < p
template <int W>
__device__ inline void modinv(const uint32_t *a, const uint32_t *p, uint32_t *out) {
    uint32_t u[W], v[W], x1[W], x2[W];
    for (int i = 0; i < W; i++) {
        u[i] = a[i];
        v[i] = p[i];
        x1[i] = i == 0;
        x2[i] = 0;
    }
    while (!w_is<W>(u, 1) && !w_is<W>(v, 1)) {
        while (!(u[0] & 1)) {
            w_shr1<W>(u, 0);
            w_shr1<W>(x1, (x1[0] & 1) ? w_add<W>(x1, p) : 0u);  // x1 / 2 mod p
        }
        while (!(v[0] & 1)) {
            w_shr1<W>(v, 0);
            w_shr1<W>(x2, (x2[0] & 1) ? w_add<W>(x2, p) : 0u);
        }
        if (w_ge<W>(u, v)) {
            w_sub<W>(u, v);
            if (w_sub<W>(x1, x2)) w_add<W>(x1, p);
        } else {
            w_sub<W>(v, u);
            if (w_sub<W>(x2, x1)) w_add<W>(x2, p);
        }
    }
    const uint32_t *r = w_is<W>(u, 1) ? x1 : x2;
    for (int i = 0; i < W; i++) out[i] = r[i];
}

// One FieldOpCols of x op y in the base field (x, y: W words, reduced here; op 0 add, 1 sub, 2 mul, 3 div),
// its result r (mod p) into res (nullable) -- FieldOpCols::populate_with_modulus as pop_field_op: sub is
// populated as r + y = x + carry p, div as r y = x + carry p (r = 0 for 0 / 0)
template <int W, int NW, int OFF>
__device__ inline void fp_op(uint32_t *o, const uint32_t *x, const uint32_t *y, uint32_t op, const FpMod &mod,
                             uint32_t *bm, uint32_t *res) {
    constexpr int NL = 4 * W;
    uint32_t a[W], b[W], lhs[W], full[2 * W], mres[W], car[W];
    mod_words<W, W>(x, mod.w, a, nullptr);
    mod_words<W, W>(y, mod.w, b, nullptr);
    const bool mul = op >= 2;
    if (op == 1) {  // r = a + p - b mod p (a + p - b < 2p: one conditional subtraction)
        for (int i = 0; i < W; i++) lhs[i] = a[i];
        const uint32_t c = w_add<W>(lhs, mod.w);
        const uint32_t bw = w_sub<W>(lhs, b);
        uint32_t t[W];
        for (int i = 0; i < W; i++) t[i] = lhs[i];
        if ((c != bw) || w_ge<W>(t, mod.w)) w_sub<W>(lhs, mod.w);  // value >= p
    } else if (op == 3) {  // r = a / b
        for (int i = 0; i < W; i++) lhs[i] = 0;
        if (!w_is<W>(b, 0)) {
            uint32_t ib[W], pr[2 * W];
            modinv<W>(b, mod.w, ib);
            for (int i = 0; i < 2 * W; i++) pr[i] = 0;
            for (int i = 0; i < W; i++) {
                uint64_t c = 0;
                for (int j = 0; j < W; j++) {
                    const uint64_t t = (uint64_t)a[i] * ib[j] + pr[i + j] + c;
                    pr[i + j] = (uint32_t)t;
                    c = t >> 32;
                }
                pr[i + W] = (uint32_t)c;
            }
            mod_words<2 * W, W>(pr, mod.w, lhs, nullptr);
        }
    } else {
        for (int i = 0; i < W; i++) lhs[i] = a[i];
    }
    for (int i = 0; i < 2 * W; i++) full[i] = 0;
    for (int i = 0; i < W; i++) car[i] = 0;
    if (mul) {  // lhs b = carry p + mres
        for (int i = 0; i < W; i++) {
            uint64_t c = 0;
            for (int j = 0; j < W; j++) {
                const uint64_t t = (uint64_t)lhs[i] * b[j] + full[i + j] + c;
                full[i + j] = (uint32_t)t;
                c = t >> 32;
            }
            full[i + W] = (uint32_t)c;
        }
        mod_words<2 * W, W>(full, mod.w, mres, car);
    } else {  // lhs + b
        for (int i = 0; i < W; i++) full[i] = lhs[i];
        full[W] = w_add<W>(full, b);
        mod_words<W + 1, W>(full, mod.w, mres, car);
    }
    // the result column: add / mul the reduced value, sub / div the populated left-hand side
    const uint32_t *r = (op == 1 || op == 3) ? lhs : mres;
    field_op_cols<NL, NW, OFF>(o, lhs, b, mul, r, mres, car, mod.w, bm);
    if (res)
        for (int i = 0; i < W; i++) res[i] = r[i];
}

template <int W, int NW, int OFF>
__global__ __launch_bounds__(128) void k_fp_op_rows(const uint32_t *__restrict__ ev, uint64_t n, uint32_t *__restrict__ out,
                                                    uint64_t height, FpMod mod, uint32_t *bm) {
    constexpr int NL = 4 * W, Y = FO_X + 13 * W, OUT = Y + 9 * W, WIDTH = OUT + 2 * NL + 2 * NW;
    const uint64_t row = (uint64_t)blockIdx.x * 128 + threadIdx.x;
    if (row >= height) return;
    uint32_t *v = out + row * WIDTH;
    for (int c = 0; c < WIDTH; c++) v[c] = 0;
    v[FO_ADD] = 1;
    if (row >= n) {  // 0 + 0: witness limbs = the offset
        for (int k = 0; k < NW; k++) {
            v[OUT + 2 * NL + k] = OFF & 0xFF;
            v[OUT + 2 * NL + NW + k] = OFF >> 8;
        }
        return;
    }
    const uint32_t *e = ev + row * FO_EV;
    const uint32_t op = e[4];
    v[FO_REAL] = 1;
    v[FO_SHARD] = e[0];
    v[FO_CLK] = e[1];
    v[FO_XPTR] = e[2];
    v[FO_YPTR] = e[3];
    v[FO_ADD] = op == 0;
    v[FO_SUB] = op == 1;
    v[FO_MUL] = op == 2;
    uint32_t x[W], y[W];
    for (int i = 0; i < W; i++) {
        const Access ya = access_read(e + 5 + 5 * i), xa = access_write(e + 65 + 6 * i);
        y[i] = ya.value;
        x[i] = xa.prev_value;
        put_access(v, Y + 9 * i, ya);
        put_word(v + FO_X + 13 * i, xa.prev_value);
        put_access(v, FO_X + 13 * i + 4, xa);
        const Access as[2] = {ya, xa};
        for (int k = 0; k < 2; k++) {
            byte_add(bm, B_U16RANGE, as[k].d16 >> 8, as[k].d16 & 0xFF);
            byte_add(bm, B_U8RANGE, 0, as[k].d8);
        }
    }
    fp_op<W, NW, OFF>(v + OUT, x, y, op, mod, bm, nullptr);
}

// Fp2AddSubAssign / Fp2MulAssign (fptower/fp2_addsub.rs:93-183, fp2_mul.rs:122-210): x = (x0, x1), y = (y0, y1)
// of 2W words.  AddSub: is_real, shard, clk, is_add, x_ptr, y_ptr, x (2W writes), y (2W reads), c0, c1.  Mul:
// is_real, shard, clk, x_ptr, y_ptr, x, y, a0 b0, a1 b1, a0 b1, a1 b0, c0 = a0 b0 - a1 b1, c1 = a0 b1 + a1 b0.
// zkm_fp2_event dwords: shard, clk, x_ptr, y_ptr, op (0 add, 1 sub; mul: unused), y reads (24 x 5), x writes
// (24 x 6), the first 2W of each used
enum { F2_EV = 5 + 120 + 144 };
template <int W, int NW, int OFF, bool MUL>
__global__ __launch_bounds__(128) void k_fp2_rows(const uint32_t *__restrict__ ev, uint64_t n, uint32_t *__restrict__ out,
                                                  uint64_t height, FpMod mod, uint32_t *bm) {
    constexpr int NL = 4 * W, FW = 2 * NL + 2 * NW, H = MUL ? 5 : 6, X = H, Y = X + 2 * W * 13, OUT = Y + 2 * W * 9,
                  NOPS = MUL ? 6 : 2, WIDTH = OUT + NOPS * FW;
    const uint64_t row = (uint64_t)blockIdx.x * 128 + threadIdx.x;
    if (row >= height) return;
    uint32_t *v = out + row * WIDTH;
    for (int c = 0; c < WIDTH; c++) v[c] = 0;
    if (!MUL) v[3] = 1;  // is_add (padding rows add zeros)
    if (row >= n) {      // the operations on zeros: witness limbs = the offset
        for (int k = 0; k < NOPS; k++)
            for (int j = 0; j < NW; j++) {
                v[OUT + k * FW + 2 * NL + j] = OFF & 0xFF;
                v[OUT + k * FW + 2 * NL + NW + j] = OFF >> 8;
            }
        return;
    }
    const uint32_t *e = ev + row * F2_EV;
    v[0] = 1;
    v[1] = e[0];
    v[2] = e[1];
    v[H - 2] = e[2];
    v[H - 1] = e[3];
    const uint32_t op = e[4];
    if (!MUL) v[3] = op == 0;
    uint32_t x[2 * W], y[2 * W];
    for (int i = 0; i < 2 * W; i++) {
        const Access ya = access_read(e + 5 + 5 * i), xa = access_write(e + 125 + 6 * i);
        y[i] = ya.value;
        x[i] = xa.prev_value;
        put_access(v, Y + 9 * i, ya);
        put_word(v + X + 13 * i, xa.prev_value);
        put_access(v, X + 13 * i + 4, xa);
        const Access as[2] = {ya, xa};
        for (int k = 0; k < 2; k++) {
            byte_add(bm, B_U16RANGE, as[k].d16 >> 8, as[k].d16 & 0xFF);
            byte_add(bm, B_U8RANGE, 0, as[k].d8);
        }
    }
    if (!MUL) {
        fp_op<W, NW, OFF>(v + OUT, x, y, op, mod, bm, nullptr);
        fp_op<W, NW, OFF>(v + OUT + FW, x + W, y + W, op, mod, bm, nullptr);
    } else {
        uint32_t r00[W], r11[W], r01[W], r10[W];
        fp_op<W, NW, OFF>(v + OUT, x, y, 2, mod, bm, r00);
        fp_op<W, NW, OFF>(v + OUT + FW, x + W, y + W, 2, mod, bm, r11);
        fp_op<W, NW, OFF>(v + OUT + 2 * FW, x, y + W, 2, mod, bm, r01);
        fp_op<W, NW, OFF>(v + OUT + 3 * FW, x + W, y, 2, mod, bm, r10);
        fp_op<W, NW, OFF>(v + OUT + 4 * FW, r00, r11, 1, mod, bm, nullptr);
        fp_op<W, NW, OFF>(v + OUT + 5 * FW, r01, r10, 0, mod, bm, nullptr);
    }
}

// WeierstrassAddAssign (weierstrass_add.rs:192-252, :384-420): is_real, shard, clk, p_ptr, q_ptr, p (2W writes),
// q (2W reads), nine FieldOpCols in column order slope_denominator = qx - px, slope_numerator = qy - py,
// slope = num / den, slope_squared, p_x_plus_q_x, x3_ins = s^2 - (px + qx), p_x_minus_x = px - x3,
// y3_ins = s (px - x3) - py, slope_times_p_x_minus_x; padding rows: the operations on zero inputs.
// zkm_ec_add_event dwords: shard, clk, p_ptr, q_ptr, q reads (24 x 5), p writes (24 x 6)
enum { EA_EV = 4 + 120 + 144 };
template <int W, int NW, int OFF>
__global__ __launch_bounds__(128) void k_ec_add_rows(const uint32_t *__restrict__ ev, uint64_t n, uint32_t *__restrict__ out,
                                                     uint64_t height, FpMod mod, uint32_t *bm) {
    constexpr int NL = 4 * W, FW = 2 * NL + 2 * NW, PC = 5, QC = PC + 2 * W * 13, OUT = QC + 2 * W * 9, WIDTH = OUT + 9 * FW;
    enum { DEN = 0, NUM, SLOPE, S2, PXQX, X3, PMX, Y3, STP };
    const uint64_t row = (uint64_t)blockIdx.x * 128 + threadIdx.x;
    if (row >= height) return;
    uint32_t *v = out + row * WIDTH;
    for (int c = 0; c < WIDTH; c++) v[c] = 0;
    if (row >= n) {
        for (int k = 0; k < 9; k++)
            for (int j = 0; j < NW; j++) {
                v[OUT + k * FW + 2 * NL + j] = OFF & 0xFF;
                v[OUT + k * FW + 2 * NL + NW + j] = OFF >> 8;
            }
        return;
    }
    const uint32_t *e = ev + row * EA_EV;
    v[0] = 1;
    v[1] = e[0];
    v[2] = e[1];
    v[3] = e[2];
    v[4] = e[3];
    uint32_t pw[2 * W], qw[2 * W];
    for (int i = 0; i < 2 * W; i++) {
        const Access qa = access_read(e + 4 + 5 * i), pa = access_write(e + 124 + 6 * i);
        qw[i] = qa.value;
        pw[i] = pa.prev_value;
        put_access(v, QC + 9 * i, qa);
        put_word(v + PC + 13 * i, pa.prev_value);
        put_access(v, PC + 13 * i + 4, pa);
        const Access as[2] = {qa, pa};
        for (int k = 0; k < 2; k++) {
            byte_add(bm, B_U16RANGE, as[k].d16 >> 8, as[k].d16 & 0xFF);
            byte_add(bm, B_U8RANGE, 0, as[k].d8);
        }
    }
    const uint32_t *px = pw, *py = pw + W, *qx = qw, *qy = qw + W;
    uint32_t num[W], den[W], slope[W], s2[W], pq[W], x3[W], pmx[W], stp[W];
    fp_op<W, NW, OFF>(v + OUT + NUM * FW, qy, py, 1, mod, bm, num);
    fp_op<W, NW, OFF>(v + OUT + DEN * FW, qx, px, 1, mod, bm, den);
    fp_op<W, NW, OFF>(v + OUT + SLOPE * FW, num, den, 3, mod, bm, slope);
    fp_op<W, NW, OFF>(v + OUT + S2 * FW, slope, slope, 2, mod, bm, s2);
    fp_op<W, NW, OFF>(v + OUT + PXQX * FW, px, qx, 0, mod, bm, pq);
    fp_op<W, NW, OFF>(v + OUT + X3 * FW, s2, pq, 1, mod, bm, x3);
    fp_op<W, NW, OFF>(v + OUT + PMX * FW, px, x3, 1, mod, bm, pmx);
    fp_op<W, NW, OFF>(v + OUT + STP * FW, slope, pmx, 2, mod, bm, stp);
    fp_op<W, NW, OFF>(v + OUT + Y3 * FW, stp, py, 1, mod, bm, nullptr);
}

// WeierstrassDoubleAssign (weierstrass_double.rs:201-270, :411-440): is_real, shard, clk, p_ptr, p (2W writes
// at clk), eleven FieldOpCols in column order slope_denominator = 2 py, slope_numerator = a + 3 px^2, slope,
// p_x_squared, p_x_squared_times_3, slope_squared, p_x_plus_p_x, x3_ins, p_x_minus_x, y3_ins,
// slope_times_p_x_minus_x.  Padding rows: the operations of p = (0, 1) (no lookups) and the dummy write
// record of the first y word (prev_value 1, value 1, compare 1).  zkm_ec_double_event dwords: shard, clk,
// p_ptr, p writes (24 x 6)
enum { ED2_EV = 3 + 144 };
template <int W, int NW, int OFF>
__global__ __launch_bounds__(128) void k_ec_double_rows(const uint32_t *__restrict__ ev, uint64_t n,
                                                        uint32_t *__restrict__ out, uint64_t height, FpMod mod,
                                                        FpMod curve_a, uint32_t *bm) {
    constexpr int NL = 4 * W, FW = 2 * NL + 2 * NW, PC = 4, OUT = PC + 2 * W * 13, WIDTH = OUT + 11 * FW;
    enum { DEN = 0, NUM, SLOPE, X2, X23, S2, PP, X3, PMX, Y3, STP };
    const uint64_t row = (uint64_t)blockIdx.x * 128 + threadIdx.x;
    if (row >= height) return;
    uint32_t *v = out + row * WIDTH;
    for (int c = 0; c < WIDTH; c++) v[c] = 0;
    const bool real = row < n;
    uint32_t *b = real ? bm : nullptr;  // padding rows record no lookups
    uint32_t pw[2 * W];
    for (int i = 0; i < 2 * W; i++) pw[i] = 0;
    if (real) {
        const uint32_t *e = ev + row * ED2_EV;
        v[0] = 1;
        v[1] = e[0];
        v[2] = e[1];
        v[3] = e[2];
        for (int i = 0; i < 2 * W; i++) {
            const Access pa = access_write(e + 3 + 6 * i);
            pw[i] = pa.prev_value;
            put_word(v + PC + 13 * i, pa.prev_value);
            put_access(v, PC + 13 * i + 4, pa);
            byte_add(bm, B_U16RANGE, pa.d16 >> 8, pa.d16 & 0xFF);
            byte_add(bm, B_U8RANGE, 0, pa.d8);
        }
    } else {  // p = (0, 1) and the dummy record of y's first word
        pw[W] = 1;
        v[PC + 13 * W] = 1;
        v[PC + 13 * W + 4 + ACC_VALUE] = 1;
        v[PC + 13 * W + 4 + ACC_COMPARE] = 1;
    }
    const uint32_t *px = pw, *py = pw + W;
    uint32_t k2[W], k3[W];
    for (int i = 0; i < W; i++) k2[i] = k3[i] = 0;
    k2[0] = 2;
    k3[0] = 3;
    uint32_t x2[W], x23[W], num[W], den[W], slope[W], s2[W], pp[W], x3[W], pmx[W], stp[W];
    fp_op<W, NW, OFF>(v + OUT + X2 * FW, px, px, 2, mod, b, x2);
    fp_op<W, NW, OFF>(v + OUT + X23 * FW, x2, k3, 2, mod, b, x23);
    fp_op<W, NW, OFF>(v + OUT + NUM * FW, curve_a.w, x23, 0, mod, b, num);
    fp_op<W, NW, OFF>(v + OUT + DEN * FW, k2, py, 2, mod, b, den);
    fp_op<W, NW, OFF>(v + OUT + SLOPE * FW, num, den, 3, mod, b, slope);
    fp_op<W, NW, OFF>(v + OUT + S2 * FW, slope, slope, 2, mod, b, s2);
    fp_op<W, NW, OFF>(v + OUT + PP * FW, px, px, 0, mod, b, pp);
    fp_op<W, NW, OFF>(v + OUT + X3 * FW, s2, pp, 1, mod, b, x3);
    fp_op<W, NW, OFF>(v + OUT + PMX * FW, px, x3, 1, mod, b, pmx);
    fp_op<W, NW, OFF>(v + OUT + STP * FW, slope, pmx, 2, mod, b, stp);
    fp_op<W, NW, OFF>(v + OUT + Y3 * FW, stp, py, 1, mod, b, nullptr);
}

// W-word modular multiplication and exponentiation (square and multiply over the exponent's bits)
template <int W>
__device__ inline void mulmod(const uint32_t *a, const uint32_t *b, const uint32_t *m, uint32_t *r) {
    uint32_t pr[2 * W];
    for (int i = 0; i < 2 * W; i++) pr[i] = 0;
    for (int i = 0; i < W; i++) {
        uint64_t c = 0;
        for (int j = 0; j < W; j++) {
            const uint64_t t = (uint64_t)a[i] * b[j] + pr[i + j] + c;
            pr[i + j] = (uint32_t)t;
            c = t >> 32;
        }
        pr[i + W] = (uint32_t)c;
    }
    mod_words<2 * W, W>(pr, m, r, nullptr);
}
template <int W>
__device__ inline void powmod(const uint32_t *a, const uint32_t *e, const uint32_t *m, uint32_t *r) {
    uint32_t acc[W];
    for (int i = 0; i < W; i++) acc[i] = i == 0;
    for (int bit = 32 * W - 1; bit >= 0; bit--) {
        mulmod<W>(acc, acc, m, acc);
        if ((e[bit >> 5] >> (bit & 31)) & 1) mulmod<W>(acc, a, m, acc);
    }
    for (int i = 0; i < W; i++) r[i] = acc[i];
}

// FieldLtCols at o for lhs < rhs (the most significant differing byte), its LTU lookup into bm
template <int NL>
__device__ inline void field_lt(uint32_t *o, const uint32_t *lhs, const uint32_t *rhs, uint32_t *bm) {
    for (int k = NL - 1; k >= 0; k--) {
        const uint32_t a = byte_of(lhs[k >> 2], k & 3), b = byte_of(rhs[k >> 2], k & 3);
        if (a != b) {
            if (a < b) {
                o[k] = 1;
                o[NL] = a;
                o[NL + 1] = b;
            }
            break;
        }
    }
    byte_add(bm, B_LTU, o[NL], o[NL + 1]);
}

// WeierstrassDecompress (weierstrass_decompress.rs:161-303): is_real, shard, clk, ptr, sign, x (W reads), y (W
// writes at clk), range_x (x < p), x^2, x^3, a x + b (FieldInnerProductCols), x^3 + a x + b, FieldSqrtCols
// (the root times itself, the root in its result; range; lsb), -y; bls12-381 adds LexicographicChoiceCols.
// Padding rows decompress the generator's x (its words as the x reads' values) without lookups.
// zkm_ec_decompress_event dwords: shard, clk, ptr, sign, x reads (12 x 5), y writes (12 x 6)
enum { EDC_EV = 4 + 60 + 72 };
struct CurveConsts {
    FpMod p, sqrt_exp, gen_x, a, b;
};
template <int W, int NW, int OFF, bool LEX>
__global__ __launch_bounds__(128) void k_ec_decompress_rows(const uint32_t *__restrict__ ev, uint64_t n,
                                                            uint32_t *__restrict__ out, uint64_t height, CurveConsts cc,
                                                            uint32_t *bm) {
    constexpr int NL = 4 * W, FW = 2 * NL + 2 * NW, LW = NL + 2, XC = 5, YC = XC + 9 * W, RX = YC + 13 * W, X2 = RX + LW,
                  X3 = X2 + FW, AXB = X3 + FW, X3AXB = AXB + FW, SQ = X3AXB + FW, SQR = SQ + FW, LSB = SQR + LW,
                  NEGY = LSB + 1, CMP = NEGY + FW, NEGR = CMP + LW, ISEQ = NEGR + LW, WSQ = ISEQ + 1, WNEG = WSQ + 1,
                  WIDTH = LEX ? WNEG + 1 : NEGY + FW;
    const uint64_t row = (uint64_t)blockIdx.x * 128 + threadIdx.x;
    if (row >= height) return;
    uint32_t *v = out + row * WIDTH;
    for (int c = 0; c < WIDTH; c++) v[c] = 0;
    const bool real = row < n;
    uint32_t *b = real ? bm : nullptr;
    const uint32_t *m = cc.p.w;
    const uint32_t *e = ev + row * EDC_EV;
    uint32_t x[W], y[W];
    for (int i = 0; i < W; i++) y[i] = 0;
    if (real) {
        v[0] = 1;
        v[1] = e[0];
        v[2] = e[1];
        v[3] = e[2];
        v[4] = e[3];
        for (int i = 0; i < W; i++) {
            const Access xa = access_read(e + 4 + 5 * i), ya = access_write(e + 64 + 6 * i);
            x[i] = xa.value;
            y[i] = ya.value;
            put_access(v, XC + 9 * i, xa);
            put_word(v + YC + 13 * i, ya.prev_value);
            put_access(v, YC + 13 * i + 4, ya);
            const Access as[2] = {xa, ya};
            for (int k = 0; k < 2; k++) {
                byte_add(bm, B_U16RANGE, as[k].d16 >> 8, as[k].d16 & 0xFF);
                byte_add(bm, B_U8RANGE, 0, as[k].d8);
            }
        }
    } else {
        for (int i = 0; i < W; i++) {
            x[i] = cc.gen_x.w[i];
            put_word(v + XC + 9 * i + ACC_VALUE, x[i]);
        }
    }
    field_lt<NL>(v + RX, x, m, b);
    uint32_t x2[W], x3[W], axb[W], rhs[W], sq[W], zero[W], one[W];
    for (int i = 0; i < W; i++) zero[i] = one[i] = 0;
    one[0] = 1;
    fp_op<W, NW, OFF>(v + X2, x, x, 2, cc.p, b, x2);
    fp_op<W, NW, OFF>(v + X3, x2, x, 2, cc.p, b, x3);
    {  // a x + b 1 (field_inner_product.rs populate)
        uint32_t ip[2 * W + 1], car[W], t[2 * W];
        for (int i = 0; i < 2 * W + 1; i++) ip[i] = 0;
        for (int i = 0; i < W; i++) {
            uint64_t c = 0;
            for (int j = 0; j < W; j++) {
                const uint64_t u = (uint64_t)cc.a.w[i] * x[j] + ip[i + j] + c;
                ip[i + j] = (uint32_t)u;
                c = u >> 32;
            }
            ip[i + W] = (uint32_t)c;
        }
        for (int i = 0; i < 2 * W; i++) t[i] = ip[i];
        const uint32_t cb = w_add<W>(t, cc.b.w);
        uint64_t c = cb;
        for (int i = W; i < 2 * W; i++) {
            const uint64_t u = (uint64_t)t[i] + c;
            t[i] = (uint32_t)u;
            c = u >> 32;
        }
        for (int i = 0; i < W; i++) car[i] = 0;
        uint32_t qd[2 * W];
        {
            int nv = W;
            while (m[nv - 1] == 0) nv--;
            uint32_t rr[W];
            for (int i = 0; i < W; i++) rr[i] = 0;
            divmod_words<2 * W, W>(t, m, nv, qd, rr);
            for (int i = 0; i < W; i++) {
                axb[i] = rr[i];
                car[i] = qd[i];
            }
        }
        int64_t van[NW + 1];
        for (int k = 0; k <= NW; k++) van[k] = 0;
        van_mul<NL, NW>(van, cc.a.w, x, 1);
        van_mul<NL, NW>(van, cc.b.w, one, 1);
        van_mul<NL, NW>(van, car, m, -1);
        for (int i = 0; i < NL; i++) van[i] -= byte_of(axb[i >> 2], i & 3);
        field_cols<NL, NW, OFF>(v + AXB, van, axb, car, b);
    }
    fp_op<W, NW, OFF>(v + X3AXB, x3, axb, 0, cc.p, b, rhs);
    powmod<W>(rhs, cc.sqrt_exp.w, m, sq);
    {  // FieldSqrtCols: sq sq = rhs + carry p, the root in the result columns, the U8 check over rhs's limbs
        uint32_t pr[2 * W], mres[W], car[W];
        for (int i = 0; i < 2 * W; i++) pr[i] = 0;
        for (int i = 0; i < W; i++) {
            uint64_t c = 0;
            for (int j = 0; j < W; j++) {
                const uint64_t u = (uint64_t)sq[i] * sq[j] + pr[i + j] + c;
                pr[i + j] = (uint32_t)u;
                c = u >> 32;
            }
            pr[i + W] = (uint32_t)c;
        }
        for (int i = 0; i < W; i++) car[i] = 0;
        mod_words<2 * W, W>(pr, m, mres, car);
        field_op_cols<NL, NW, OFF>(v + SQ, sq, sq, true, sq, mres, car, m, b, rhs);
    }
    field_lt<NL>(v + SQR, sq, m, b);
    v[LSB] = sq[0] & 1;
    byte_add(b, B_AND, sq[0] & 0xFF, 1);
    for (int j = 0; j < NL; j += 2) byte_add(b, B_U8RANGE, byte_of(sq[j >> 2], j & 3), byte_of(sq[(j + 1) >> 2], (j + 1) & 3));
    uint32_t negy[W];
    fp_op<W, NW, OFF>(v + NEGY, zero, sq, 1, cc.p, b, negy);
    if (LEX && real) {
        const bool eq = (y[0] & 1) == (sq[0] & 1), sg = e[3] != 0;
        v[ISEQ] = eq;
        v[WSQ] = sg ? !eq : eq;
        v[WNEG] = sg ? eq : !eq;
        field_lt<NL>(v + NEGR, negy, m, bm);
        uint32_t neg[W];  // (p - y) mod p
        for (int i = 0; i < W; i++) neg[i] = m[i];
        w_sub<W>(neg, y);
        if (w_ge<W>(neg, m)) w_sub<W>(neg, m);
        field_lt<NL>(v + CMP, sg ? neg : y, sg ? y : neg, bm);
    }
}

// FieldInnerProductCols (field_inner_product.rs:33-94) of a0 b0 + a1 b1 and FieldDenCols (field_den.rs:33-94)
// of a / (1 +- b) (sign: 1 + b, else 1 - b) at o, their results into res; W-word operands below p
template <int W, int NW, int OFF>
__device__ inline void fp_ip2(uint32_t *o, const uint32_t *a0, const uint32_t *b0, const uint32_t *a1, const uint32_t *b1,
                              const uint32_t *m, uint32_t *bm, uint32_t *res) {
    constexpr int NL = 4 * W;
    uint32_t t0[2 * W], t1[2 * W + 1], car[W], r[W];
    for (int i = 0; i < 2 * W; i++) t0[i] = t1[i] = 0;
    t1[2 * W] = 0;
    for (int i = 0; i < W; i++) {
        uint64_t c = 0, d = 0;
        for (int j = 0; j < W; j++) {
            const uint64_t u = (uint64_t)a0[i] * b0[j] + t0[i + j] + c;
            t0[i + j] = (uint32_t)u;
            c = u >> 32;
            const uint64_t v = (uint64_t)a1[i] * b1[j] + t1[i + j] + d;
            t1[i + j] = (uint32_t)v;
            d = v >> 32;
        }
        t0[i + W] = (uint32_t)c;
        t1[i + W] = (uint32_t)d;
    }
    t1[2 * W] = w_add<2 * W>(t1, t0);
    for (int i = 0; i < W; i++) car[i] = 0;
    mod_words<2 * W + 1, W>(t1, m, r, car);
    int64_t van[NW + 1];
    for (int k = 0; k <= NW; k++) van[k] = 0;
    van_mul<NL, NW>(van, a0, b0, 1);
    van_mul<NL, NW>(van, a1, b1, 1);
    van_mul<NL, NW>(van, car, m, -1);
    for (int i = 0; i < NL; i++) van[i] -= byte_of(r[i >> 2], i & 3);
    field_cols<NL, NW, OFF>(o, van, r, car, bm);
    for (int i = 0; i < W; i++) res[i] = r[i];
}
template <int W, int NW, int OFF>
__device__ inline void fp_den(uint32_t *o, const uint32_t *a, const uint32_t *b, bool sign, const FpMod &mod,
                              uint32_t *bm, uint32_t *res) {
    constexpr int NL = 4 * W;
    const uint32_t *m = mod.w;
    uint32_t den[W], one[W], r[W];
    for (int i = 0; i < W; i++) one[i] = i == 0;
    if (sign) {  // b + 1 mod p
        for (int i = 0; i < W; i++) den[i] = b[i];
    } else {     // p - b + 1 mod p
        for (int i = 0; i < W; i++) den[i] = m[i];
        w_sub<W>(den, b);
    }
    const uint32_t c = w_add<W>(den, one);
    if (c || w_ge<W>(den, m)) w_sub<W>(den, m);
    for (int i = 0; i < W; i++) r[i] = 0;
    if (!w_is<W>(den, 0)) {
        uint32_t inv[W];
        modinv<W>(den, m, inv);
        mulmod<W>(a, inv, m, r);
    }
    // lhs = b r + (sign ? r : a), rhs = sign ? a : r; carry = (lhs - rhs) / p
    uint32_t l[2 * W + 1], q[2 * W + 1], rr[W], car[W];
    for (int i = 0; i < 2 * W + 1; i++) l[i] = 0;
    for (int i = 0; i < W; i++) {
        uint64_t cc = 0;
        for (int j = 0; j < W; j++) {
            const uint64_t u = (uint64_t)b[i] * r[j] + l[i + j] + cc;
            l[i + j] = (uint32_t)u;
            cc = u >> 32;
        }
        l[i + W] = (uint32_t)cc;
    }
    uint32_t add_t[2 * W];
    for (int i = 0; i < 2 * W; i++) add_t[i] = i < W ? (sign ? r[i] : a[i]) : 0u;
    l[2 * W] = w_add<2 * W>(l, add_t);
    uint32_t sub_t[2 * W + 1];
    for (int i = 0; i < 2 * W + 1; i++) sub_t[i] = i < W ? (sign ? a[i] : r[i]) : 0u;
    w_sub<2 * W + 1>(l, sub_t);  // lhs - rhs, a multiple of p
    int nv = W;
    while (m[nv - 1] == 0) nv--;
    for (int i = 0; i < W; i++) rr[i] = 0;
    divmod_words<2 * W + 1, W>(l, m, nv, q, rr);
    for (int i = 0; i < W; i++) car[i] = q[i];
    int64_t van[NW + 1];
    for (int k = 0; k <= NW; k++) van[k] = 0;
    van_mul<NL, NW>(van, b, r, 1);
    for (int i = 0; i < NL; i++) {
        const int64_t ri = byte_of(r[i >> 2], i & 3), ai = byte_of(a[i >> 2], i & 3);
        van[i] += sign ? ri - ai : ai - ri;
    }
    van_mul<NL, NW>(van, car, m, -1);
    field_cols<NL, NW, OFF>(o, van, r, car, bm);
    for (int i = 0; i < W; i++) res[i] = r[i];
}

// EdAddAssign (edwards/ed_add.rs:111-238): is_real, shard, clk, p_ptr, q_ptr, p (16 writes at clk + 1), q (16
// reads at clk), x3_numerator = x1 y2 + x2 y1, y3_numerator = y1 y2 + x1 x2, x1 y1, x2 y2, f = x1 y1 x2 y2,
// d f, x3 = x3n / (1 + d f), y3 = y3n / (1 - d f); padding rows: the operations on zero inputs.
// zkm_ed_add_event dwords: shard, clk, p_ptr, q_ptr, q reads (16 x 5), p writes (16 x 6)
enum { EDA_EV = 4 + 80 + 96 };
__global__ __launch_bounds__(128) void k_ed_add_rows(const uint32_t *__restrict__ ev, uint64_t n, uint32_t *__restrict__ out,
                                                     uint64_t height, uint32_t *bm) {
    constexpr int W = 8, NW = 62, OFF = 1 << 14, NL = 32, FW = 2 * NL + 2 * NW, PC = 5, QC = PC + 16 * 13,
                  OUT = QC + 16 * 9, WIDTH = OUT + 8 * FW;
    static_assert(WIDTH == ZKM_ED_ADD_WIDTH, "EdAddAssignCols layout");
    const uint64_t row = (uint64_t)blockIdx.x * 128 + threadIdx.x;
    if (row >= height) return;
    uint32_t *v = out + row * WIDTH;
    for (int c = 0; c < WIDTH; c++) v[c] = 0;
    const bool real = row < n;
    uint32_t *b = real ? bm : nullptr;
    uint32_t pw[16], qw[16];
    for (int i = 0; i < 16; i++) pw[i] = qw[i] = 0;
    if (real) {
        const uint32_t *e = ev + row * EDA_EV;
        v[0] = 1;
        v[1] = e[0];
        v[2] = e[1];
        v[3] = e[2];
        v[4] = e[3];
        for (int i = 0; i < 16; i++) {
            const Access qa = access_read(e + 4 + 5 * i), pa = access_write(e + 84 + 6 * i);
            qw[i] = qa.value;
            pw[i] = pa.prev_value;
            put_access(v, QC + 9 * i, qa);
            put_word(v + PC + 13 * i, pa.prev_value);
            put_access(v, PC + 13 * i + 4, pa);
            const Access as[2] = {qa, pa};
            for (int k = 0; k < 2; k++) {
                byte_add(bm, B_U16RANGE, as[k].d16 >> 8, as[k].d16 & 0xFF);
                byte_add(bm, B_U8RANGE, 0, as[k].d8);
            }
        }
    }
    const uint32_t *x1 = pw, *y1 = pw + 8, *x2 = qw, *y2 = qw + 8, *m = kEd25519.w;
    uint32_t x3n[W], y3n[W], x1y1[W], x2y2[W], f[W], df[W], t[W];
    fp_ip2<W, NW, OFF>(v + OUT, x1, y2, x2, y1, m, b, x3n);
    fp_ip2<W, NW, OFF>(v + OUT + FW, y1, y2, x1, x2, m, b, y3n);
    fp_op<W, NW, OFF>(v + OUT + 2 * FW, x1, y1, 2, kEd25519, b, x1y1);
    fp_op<W, NW, OFF>(v + OUT + 3 * FW, x2, y2, 2, kEd25519, b, x2y2);
    fp_op<W, NW, OFF>(v + OUT + 4 * FW, x1y1, x2y2, 2, kEd25519, b, f);
    fp_op<W, NW, OFF>(v + OUT + 5 * FW, f, kEdD.w, 2, kEd25519, b, df);
    fp_den<W, NW, OFF>(v + OUT + 6 * FW, x3n, df, true, kEd25519, b, t);
    fp_den<W, NW, OFF>(v + OUT + 7 * FW, y3n, df, false, kEd25519, b, t);
}

// EdDecompress (edwards/ed_decompress.rs:64-101, :214-247): is_real, shard, clk, ptr, sign, x (8 writes at clk),
// y (8 reads at clk), y < p, y^2, u = y^2 - 1, d y^2, v = 1 + d y^2, u / v, FieldSqrtCols of u / v (the root
// with lsb 0: ed25519.rs:75-113), its range and lsb, -x; padding rows: the operations of y = 0, no lookups.
// zkm_ed_decompress_event dwords: shard, clk, ptr, sign, y reads (8 x 5), x writes (8 x 6)
enum { EDD_EV = 4 + 40 + 48 };
__global__ __launch_bounds__(128) void k_ed_decompress_rows(const uint32_t *__restrict__ ev, uint64_t n,
                                                            uint32_t *__restrict__ out, uint64_t height, uint32_t *bm) {
    constexpr int W = 8, NW = 62, OFF = 1 << 14, NL = 32, FW = 2 * NL + 2 * NW, LW = NL + 2, XC = 5, YC = XC + 8 * 13,
                  YR = YC + 8 * 9, YY = YR + LW, U = YY + FW, DYY = U + FW, V = DYY + FW, UDV = V + FW, SQ = UDV + FW,
                  SQR = SQ + FW, LSB = SQR + LW, NEGX = LSB + 1, WIDTH = NEGX + FW;
    static_assert(WIDTH == ZKM_ED_DECOMPRESS_WIDTH, "EdDecompressCols layout");
    const uint64_t row = (uint64_t)blockIdx.x * 128 + threadIdx.x;
    if (row >= height) return;
    uint32_t *v = out + row * WIDTH;
    for (int c = 0; c < WIDTH; c++) v[c] = 0;
    const bool real = row < n;
    uint32_t *b = real ? bm : nullptr;
    const uint32_t *m = kEd25519.w;
    uint32_t y[W];
    for (int i = 0; i < W; i++) y[i] = 0;
    if (real) {
        const uint32_t *e = ev + row * EDD_EV;
        v[0] = 1;
        v[1] = e[0];
        v[2] = e[1];
        v[3] = e[2];
        v[4] = e[3];
        for (int i = 0; i < W; i++) {
            const Access ya = access_read(e + 4 + 5 * i), xa = access_write(e + 44 + 6 * i);
            y[i] = ya.value;
            put_access(v, YC + 9 * i, ya);
            put_word(v + XC + 13 * i, xa.prev_value);
            put_access(v, XC + 13 * i + 4, xa);
            const Access as[2] = {ya, xa};
            for (int k = 0; k < 2; k++) {
                byte_add(bm, B_U16RANGE, as[k].d16 >> 8, as[k].d16 & 0xFF);
                byte_add(bm, B_U8RANGE, 0, as[k].d8);
            }
        }
    }
    field_lt<NL>(v + YR, y, m, b);
    uint32_t one[W], zero[W], yy[W], u[W], dyy[W], vv[W], udv[W], sq[W], t[W];
    for (int i = 0; i < W; i++) one[i] = zero[i] = 0;
    one[0] = 1;
    fp_op<W, NW, OFF>(v + YY, y, y, 2, kEd25519, b, yy);
    fp_op<W, NW, OFF>(v + U, yy, one, 1, kEd25519, b, u);
    fp_op<W, NW, OFF>(v + DYY, kEdD.w, yy, 2, kEd25519, b, dyy);
    fp_op<W, NW, OFF>(v + V, one, dyy, 0, kEd25519, b, vv);
    fp_op<W, NW, OFF>(v + UDV, u, vv, 3, kEd25519, b, udv);
    {  // ed25519_sqrt: beta = a^((p+3)/8), times sqrt(-1) when beta^2 = -a, negated when odd
        powmod<W>(udv, kEdSqrtExp.w, m, sq);
        mulmod<W>(sq, sq, m, t);
        uint32_t na[W];
        for (int i = 0; i < W; i++) na[i] = m[i];
        w_sub<W>(na, udv);
        if (w_ge<W>(na, m)) w_sub<W>(na, m);
        bool eq = true;
        for (int i = 0; i < W; i++) eq = eq && t[i] == na[i];
        if (eq) mulmod<W>(sq, kEdSqrtM1.w, m, sq);
        if (sq[0] & 1) {
            uint32_t r[W];
            for (int i = 0; i < W; i++) r[i] = m[i];
            w_sub<W>(r, sq);
            if (w_ge<W>(r, m)) w_sub<W>(r, m);
            for (int i = 0; i < W; i++) sq[i] = r[i];
        }
    }
    {  // FieldSqrtCols: sq sq = u / v + carry p, the root in the result columns, the U8 check over u / v's limbs
        uint32_t pr[2 * W], mres[W], car[W];
        for (int i = 0; i < 2 * W; i++) pr[i] = 0;
        for (int i = 0; i < W; i++) {
            uint64_t c = 0;
            for (int j = 0; j < W; j++) {
                const uint64_t q = (uint64_t)sq[i] * sq[j] + pr[i + j] + c;
                pr[i + j] = (uint32_t)q;
                c = q >> 32;
            }
            pr[i + W] = (uint32_t)c;
        }
        for (int i = 0; i < W; i++) car[i] = 0;
        mod_words<2 * W, W>(pr, m, mres, car);
        field_op_cols<NL, NW, OFF>(v + SQ, sq, sq, true, sq, mres, car, m, b, udv);
    }
    field_lt<NL>(v + SQR, sq, m, b);
    v[LSB] = sq[0] & 1;
    byte_add(b, B_AND, sq[0] & 0xFF, 1);
    for (int j = 0; j < NL; j += 2) byte_add(b, B_U8RANGE, byte_of(sq[j >> 2], j & 3), byte_of(sq[(j + 1) >> 2], (j + 1) & 3));
    fp_op<W, NW, OFF>(v + NEGX, zero, sq, 1, kEd25519, b, t);
}

// ------------------------------------------------------------------ KeccakSponge (keccak_sponge/trace.rs:62-196)
// 24 rows per absorbed block.  Each row is built by its own thread: the block's xored state run through the
// rounds before it (Keccak-f[1600], lane index 5y + x), then the p3-keccak-air columns of that round (step
// flags, preimage, A limbs, C / C-prime / A-prime bits, A2 limbs, the bits of A2[0][0], the limbs of
// A3[0][0] = A2[0][0] ^ RC) and the sponge columns (flags, addresses, original state, on the block's first
// row the block reads and the xored rate, on the call's first row the length read, on its last row the
// output writes).  Padding rows: the zero input's rows, round = row mod 24.  zkm_keccak_block dwords: shard,
// clk, in_ptr (of this block), out_ptr, in_len (words), block index, blocks in the call, the xored state
// (50), the previous block's xored state (50; zero for the first), the block's 36 reads (5 each), the length
// read (5), the 16 output writes (6 each)
enum { KS_EV = 7 + 50 + 50 + 180 + 5 + 96, KK_STEP = 0, KK_PRE = 25, KK_A = 125, KK_C = 225, KK_CP = 545, KK_AP = 865,
       KK_APP = 2465, KK_APP00 = 2565, KK_APPP00 = 2629, KS_BLOCK_MEM = 2633, KS_SHARD = 2957, KS_CLK = 2958,
       KS_REAL = 2959, KS_READ_BLOCK = 2960, KS_IN_ADDR = 2961, KS_OUT_ADDR = 2962, KS_IN_LEN = 2963,
       KS_ABSORBED = 2964, KS_IS_ABSORBED = 2965, KS_RECV = 2966, KS_WRITE_OUT = 2967, KS_FIRST = 2968,
       KS_FINAL = 2969, KS_ORIG = 2970, KS_XORED = 3170, KS_LEN_MEM = 3314, KS_OUT_MEM = 3323 };
static_assert(KS_OUT_MEM + 16 * 13 == ZKM_KECCAK_SPONGE_WIDTH, "KeccakSpongeCols layout");
__constant__ uint64_t kKeccakRC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808aull, 0x8000000080008000ull, 0x000000000000808bull,
    0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull, 0x000000000000008aull, 0x0000000000000088ull,
    0x0000000080008009ull, 0x000000008000000aull, 0x000000008000808bull, 0x800000000000008bull, 0x8000000000008089ull,
    0x8000000000008003ull, 0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800aull, 0x800000008000000aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};
__constant__ uint8_t kKeccakR[5][5] = {{0, 36, 3, 41, 18}, {1, 44, 10, 45, 2}, {62, 6, 43, 15, 61}, {28, 55, 25, 21, 56},
                                       {27, 20, 39, 8, 14}};
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int s) { return s ? (x << s) | (x >> (64 - s)) : x; }

// one round on a (in place); c, cp, ap, app filled when c is non-null
__device__ inline void keccak_round(uint64_t a[25], int r, uint64_t *c, uint64_t *cp, uint64_t *ap, uint64_t *app) {
    uint64_t C[5], D[5], A1[25], B[25];
    for (int x = 0; x < 5; x++) C[x] = a[x] ^ a[5 + x] ^ a[10 + x] ^ a[15 + x] ^ a[20 + x];
    for (int x = 0; x < 5; x++) D[x] = C[x] ^ C[(x + 4) % 5] ^ rotl64(C[(x + 1) % 5], 1);
    for (int y = 0; y < 5; y++)
        for (int x = 0; x < 5; x++) A1[5 * y + x] = a[5 * y + x] ^ C[x] ^ D[x];
    for (int y = 0; y < 5; y++)
        for (int x = 0; x < 5; x++) {
            const int sx = (x + 3 * y) % 5;
            B[5 * y + x] = rotl64(A1[5 * x + sx], kKeccakR[sx][x]);
        }
    for (int y = 0; y < 5; y++)
        for (int x = 0; x < 5; x++) a[5 * y + x] = B[5 * y + x] ^ (~B[5 * y + (x + 1) % 5] & B[5 * y + (x + 2) % 5]);
    if (c) {
        for (int x = 0; x < 5; x++) {
            c[x] = C[x];
            cp[x] = D[x];
        }
        for (int i = 0; i < 25; i++) {
            ap[i] = A1[i];
            app[i] = a[i];
        }
    }
    a[0] ^= kKeccakRC[r];
}

__global__ __launch_bounds__(64) void k_keccak_sponge_rows(const uint32_t *__restrict__ ev, uint64_t nblocks,
                                                           uint32_t *__restrict__ out, uint64_t height, uint32_t *bm) {
    constexpr int WD = ZKM_KECCAK_SPONGE_WIDTH;
    const uint64_t row = (uint64_t)blockIdx.x * 64 + threadIdx.x;
    if (row >= height) return;
    uint32_t *v = out + row * WD;
    for (int c = 0; c < WD; c++) v[c] = 0;
    const uint64_t blk = row / 24;
    const int r = (int)(row % 24);
    const bool real = blk < nblocks;
    const uint32_t *e = ev + blk * KS_EV;  // dereferenced for real rows only
    uint64_t a[25];
    for (int i = 0; i < 25; i++) a[i] = real ? ((uint64_t)e[7 + 2 * i] | ((uint64_t)e[8 + 2 * i] << 32)) : 0ull;
    v[KK_STEP + r] = 1;
    for (int i = 0; i < 25; i++)
        for (int l = 0; l < 4; l++) v[KK_PRE + 4 * i + l] = (uint32_t)((a[i] >> (16 * l)) & 0xFFFF);
    for (int k = 0; k < r; k++) keccak_round(a, k, nullptr, nullptr, nullptr, nullptr);
    for (int i = 0; i < 25; i++)
        for (int l = 0; l < 4; l++) v[KK_A + 4 * i + l] = (uint32_t)((a[i] >> (16 * l)) & 0xFFFF);
    uint64_t c[5], cp[5], ap[25], app[25];
    keccak_round(a, r, c, cp, ap, app);
    for (int x = 0; x < 5; x++)
        for (int b = 0; b < 64; b++) {
            v[KK_C + 64 * x + b] = (uint32_t)((c[x] >> b) & 1);
            v[KK_CP + 64 * x + b] = (uint32_t)((cp[x] >> b) & 1);
        }
    for (int i = 0; i < 25; i++) {
        for (int b = 0; b < 64; b++) v[KK_AP + 64 * i + b] = (uint32_t)((ap[i] >> b) & 1);
        for (int l = 0; l < 4; l++) v[KK_APP + 4 * i + l] = (uint32_t)((app[i] >> (16 * l)) & 0xFFFF);
    }
    for (int b = 0; b < 64; b++) v[KK_APP00 + b] = (uint32_t)((app[0] >> b) & 1);
    for (int l = 0; l < 4; l++) v[KK_APPP00 + l] = (uint32_t)((a[0] >> (16 * l)) & 0xFFFF);
    if (!real) return;
    const uint32_t shard = e[0], clk = e[1], k = e[5], nblk = e[6];
    const bool first = k == 0, final = k + 1 == nblk;
    v[KS_SHARD] = shard;
    v[KS_CLK] = clk;
    v[KS_REAL] = 1;
    v[KS_IN_LEN] = e[4];
    v[KS_ABSORBED] = k * 36;
    v[KS_IS_ABSORBED] = r == 23 && !final;
    v[KS_FIRST] = first;
    v[KS_FINAL] = final;
    v[KS_READ_BLOCK] = r == 0;
    v[KS_RECV] = r == 0 && first;
    v[KS_WRITE_OUT] = r == 23 && final;
    v[KS_OUT_ADDR] = e[3];
    v[KS_IN_ADDR] = e[2];
    // the state before this block's absorption: Keccak-f of the previous block's xored state
    uint64_t o[25];
    for (int i = 0; i < 25; i++) o[i] = (uint64_t)e[57 + 2 * i] | ((uint64_t)e[58 + 2 * i] << 32);
    if (!first)
        for (int k2 = 0; k2 < 24; k2++) keccak_round(o, k2, nullptr, nullptr, nullptr, nullptr);
    uint32_t ow[50];
    for (int i = 0; i < 25; i++) {
        ow[2 * i] = (uint32_t)o[i];
        ow[2 * i + 1] = (uint32_t)(o[i] >> 32);
    }
    for (int i = 0; i < 50; i++) put_word(v + KS_ORIG + 4 * i, ow[i]);
    auto acc = [&](int col, const Access &x) {
        put_access(v, col, x);
        byte_add(bm, B_U16RANGE, x.d16 >> 8, x.d16 & 0xFF);
        byte_add(bm, B_U8RANGE, 0, x.d8);
    };
    if (r == 0) {
        for (int i = 0; i < 36; i++) {
            const Access x = access_read(e + 107 + 5 * i);
            acc(KS_BLOCK_MEM + 9 * i, x);
            for (int b = 0; b < 4; b++) {  // XorOperation of the original word and the input word
                const uint32_t ob = byte_of(ow[i], b), ib = byte_of(x.value, b);
                v[KS_XORED + 4 * i + b] = ob ^ ib;
                byte_add(bm, B_XOR, ob, ib);
            }
        }
        if (first) acc(KS_LEN_MEM, access_read(e + 287));
    }
    if (r == 23 && final) {
        for (int i = 0; i < 16; i++) {
            const Access w = access_write(e + 292 + 6 * i);
            put_word(v + KS_OUT_MEM + 13 * i, w.prev_value);
            acc(KS_OUT_MEM + 13 * i + 4, w);
        }
    }
}

// ------------------------------------------------------------------ SysLinux (sys_linux/trace.rs:106-167)
// SysLinuxCols (sys_linux/columns.rs); zkm_sys_linux_event dwords: shard, clk, code, a0, a1, result, the A3
// write, the io record
enum { LX_SHARD = 0, LX_CLK = 1, LX_ID = 2, LX_A0 = 3, LX_A1 = 7, LX_RES = 11, LX_IO = 15, LX_OUT = 28, LX_A0_0 = 41,
       LX_A0_1 = 42, LX_A0_2 = 43, LX_MMAP = 44, LX_MMAP2 = 45, LX_MMAP_A0_0 = 46, LX_PAGE_OFF = 47, LX_OFF_0 = 48,
       LX_UPPER = 49, LX_CLONE = 50, LX_EXIT = 51, LX_BRK = 52, LX_GT = 53, LX_FCNTL = 60, LX_A1_1 = 61, LX_A1_3 = 62,
       LX_F_A1_1 = 63, LX_F_A1_3 = 64, LX_READ = 65, LX_WRITE = 66, LX_NOP = 67, LX_REAL = 68, LX_EV = 18 };
static_assert(LX_REAL + 1 == ZKM_SYS_LINUX_WIDTH, "SysLinuxCols layout");
constexpr uint32_t SYS_READ_ = 4003, SYS_WRITE_ = 4004, SYS_BRK_ = 4045, SYS_FCNTL_ = 4055, SYS_MMAP2_ = 4090,
                   SYS_CLONE_ = 4120, SYS_MMAP_ = 4210, SYS_EXT_GROUP_ = 4246;  // executor/src/syscalls/code.rs

struct SysLinuxChip {
    // MemoryWriteCols at `base` (prev_value word, then MemoryAccessCols) with its range-check lookups
    __device__ __forceinline__ static void write(uint32_t *v, int base, const uint32_t *rec, const Hist &h) {
        const Access a = access_write(rec);
        put_word(v + base, a.prev_value);
        put_access(v, base + 4, a);
        h.byte(B_U16RANGE, a.d16 >> 8, a.d16 & 0xFF, true);
        h.byte(B_U8RANGE, 0, a.d8, true);
    }
    __device__ __forceinline__ void row(uint32_t *v, const uint32_t *e, uint64_t, const Hist &h) const {
#pragma unroll
        for (int c = 0; c < ZKM_SYS_LINUX_WIDTH; c++) v[c] = 0;
        // every lane takes part in the ballots of Hist::byte, with `on` false for the padding rows
        const bool real = e != nullptr;
        const uint32_t code = real ? e[2] : 0u, a0 = real ? e[3] : 0u, a1 = real ? e[4] : 0u;
        if (real) {
            v[LX_SHARD] = e[0];
            v[LX_CLK] = e[1];
            v[LX_ID] = code;
            v[LX_REAL] = 1;
            put_word(v + LX_A0, a0);
            put_word(v + LX_A1, a1);
            put_word(v + LX_RES, e[5]);
            v[LX_A0_0] = a0 == 0;
            v[LX_A0_1] = a0 == 1;
            v[LX_A0_2] = a0 == 2;
        }
        const Access out = real ? access_write(e + 6) : Access{};
        if (real) {
            put_word(v + LX_OUT, out.prev_value);
            put_access(v, LX_OUT + 4, out);
        }
        h.byte(B_U16RANGE, out.d16 >> 8, out.d16 & 0xFF, real);
        h.byte(B_U8RANGE, 0, out.d8, real);
        const bool brk = real && code == SYS_BRK_, wr = real && code == SYS_WRITE_;
        const bool mmap = real && (code == SYS_MMAP_ || code == SYS_MMAP2_);
        const bool io = brk || wr || (mmap && a0 == 0);
        const Access ia = io ? access_write(e + 12) : Access{};
        if (io) {
            put_word(v + LX_IO, ia.prev_value);
            put_access(v, LX_IO + 4, ia);
        }
        h.byte(B_U16RANGE, ia.d16 >> 8, ia.d16 & 0xFF, io);
        h.byte(B_U8RANGE, 0, ia.d8, io);
        // BRK: GtColsBytes::populate(a0, brk): the most significant differing byte, its values and a0 > brk
        uint32_t ac = 0, bc = 0;
        if (brk) {
            v[LX_BRK] = 1;
            const uint32_t b = ia.value;
            for (int j = 3; j >= 0; j--) {
                if (byte_of(a0, j) != byte_of(b, j)) {
                    v[LX_GT + j] = 1;
                    ac = byte_of(a0, j);
                    bc = byte_of(b, j);
                    v[LX_GT + 6] = ac > bc;
                    break;
                }
            }
            v[LX_GT + 4] = ac;
            v[LX_GT + 5] = bc;
        }
        h.byte(B_LTU, bc, ac, brk);
        h.byte(B_U8RANGE, byte_of(a0, 0), byte_of(a0, 1), brk);
        h.byte(B_U8RANGE, byte_of(a0, 2), byte_of(a0, 3), brk);
        h.byte(B_U8RANGE, byte_of(ia.value, 0), byte_of(ia.value, 1), brk);
        h.byte(B_U8RANGE, byte_of(ia.value, 2), byte_of(ia.value, 3), brk);
        if (!real || brk) return;
        if (code == SYS_CLONE_) {
            v[LX_CLONE] = 1;
        } else if (code == SYS_EXT_GROUP_) {
            v[LX_EXIT] = 1;
        } else if (code == SYS_FCNTL_) {
            v[LX_FCNTL] = 1;
            v[LX_A1_1] = v[LX_F_A1_1] = a1 == 1;
            v[LX_A1_3] = v[LX_F_A1_3] = a1 == 3;
        } else if (mmap) {
            v[LX_MMAP] = 1;
            v[LX_MMAP2] = code == SYS_MMAP2_;
            v[LX_MMAP_A0_0] = a0 == 0;
            v[LX_PAGE_OFF] = a1 & 0xFFF;
            v[LX_OFF_0] = (a1 & 0xFFF) == 0;
            v[LX_UPPER] = (a1 >> 12) << 12;
        } else if (code == SYS_READ_) {
            v[LX_READ] = 1;
        } else if (code == SYS_WRITE_) {
            v[LX_WRITE] = 1;
        } else {
            v[LX_NOP] = 1;
        }
    }
};

// ------------------------------------------------------------------ Poseidon2Permute (poseidon2/trace.rs)
// Poseidon2MemCols (poseidon2/columns.rs:9-20): Poseidon2Degree3Cols (the 313 PermutationSBox columns),
// shard, clk, ptr, 16 MemoryWriteCols (prev_value word + MemoryAccessCols), the range checkers of the
// pre- and post-state words, is_real.  Each 16-lane DPP row of a wavefront builds one trace row (lane l:
// state word l, as in the recursion chip's kernel); 16 rows per workgroup in a 62 KB LDS tile that leaves
// as one contiguous span of 16-byte stores.
enum { PM_SHARD = 313, PM_CLK = 314, PM_ADDR = 315, PM_MEM = 316, PM_PRE = PM_MEM + 16 * 13, PM_POST = PM_PRE + 16 * 14,
       PM_REAL = PM_POST + 16 * 14, PM_EV = 3 + 16 * 6, PM_ROWS = 16 };
static_assert(p2rows::COLS == PM_SHARD && PM_REAL + 1 == ZKM_POSEIDON2_PERMUTE_WIDTH, "Poseidon2MemCols layout");
static_assert(PM_ROWS * ZKM_POSEIDON2_PERMUTE_WIDTH % 4 == 0, "tile of whole 16-byte stores");

__global__ __launch_bounds__(16 * PM_ROWS) void k_p2permute_rows(const uint32_t *__restrict__ ev, uint64_t n,
                                                                 uint32_t *__restrict__ out, uint32_t *byte_mult) {
    constexpr int WD = ZKM_POSEIDON2_PERMUTE_WIDTH;
    __shared__ uint32_t tile[PM_ROWS * WD];
    const uint32_t t = threadIdx.x, rl = t >> 4, l = t & 15;
    const uint64_t row0 = (uint64_t)blockIdx.x * PM_ROWS, row = row0 + rl;
    uint32_t *my = tile + rl * WD;
    const bool real = row < n;
    const uint32_t *e = ev + row * PM_EV, *w = e + 3 + 6 * l;  // dereferenced for real rows only
    p2rows::fill(kb::to_mont(real ? w[3] : 0u), l, my);       // the state word: its write's previous value
    for (int c = p2rows::COLS + (int)l; c < WD; c += 16) my[c] = 0;
    __syncthreads();
    if (real) {
        if (l == 0) {
            my[PM_SHARD] = e[0];
            my[PM_CLK] = e[1];
            my[PM_ADDR] = e[2];
            my[PM_REAL] = 1;
        }
        const Access a = access_write(w);
        put_word(my + PM_MEM + 13 * l, a.prev_value);
        put_access(my, PM_MEM + 13 * l + 4, a);
        put_range_check(my + PM_PRE + 14 * l, a.prev_value);
        put_range_check(my + PM_POST + 14 * l, a.value);
        if (byte_mult) {  // the access's timestamp-difference range checks (memory/consistency/trace.rs)
            atomicAdd(byte_mult + (a.d16 * BYTE_COLS + B_U16RANGE), 1u);
            atomicAdd(byte_mult + (a.d8 * BYTE_COLS + B_U8RANGE), 1u);
        }
    }
    __syncthreads();
    uint4 *dst = reinterpret_cast<uint4 *>(out + row0 * WD);
    for (uint32_t q = t; q < PM_ROWS * WD / 4; q += 16 * PM_ROWS) {
        const uint32_t *src = tile + 4 * q;
        dst[q] = make_uint4(src[0], src[1], src[2], src[3]);
    }
}

// ------------------------------------------------------------------ ShaCompress (sha256/compress/trace.rs:32-305)
// 80 rows per call (8 reads of h, 64 rounds, 8 writes of h + the state).  The round state is sequential
// within a call, so a first kernel (one thread per call) expands each call into 80 row records: shard,
// clk, w_ptr, h_ptr, the row's memory access as a MemoryWriteRecord (reads: prev_value = value), the state
// a..h the row shows, w[j] and h[j]; the row kernel then fills every column from its record.
enum { SC2_SHARD = 0, SC2_CLK = 1, SC2_WPTR = 2, SC2_HPTR = 3, SC2_START = 4, SC2_OCTET = 5, SC2_OCTNUM = 13,
       SC2_MEM = 23, SC2_ADDR = 36, SC2_A = 37, SC2_K = 69, SC2_ERR6 = 73, SC2_ERR11 = 85, SC2_ERR25 = 97,
       SC2_S1I = 109, SC2_S1 = 113, SC2_EANDF = 117, SC2_ENOT = 121, SC2_ENOTG = 125, SC2_CH = 129, SC2_TEMP1 = 133,
       SC2_ARR2 = 161, SC2_ARR13 = 173, SC2_ARR22 = 185, SC2_S0I = 197, SC2_S0 = 201, SC2_AANDB = 205,
       SC2_AANDC = 209, SC2_BANDC = 213, SC2_MAJI = 217, SC2_MAJ = 221, SC2_TEMP2 = 225, SC2_DT1 = 232,
       SC2_T1T2 = 239, SC2_FOP = 246, SC2_FADD = 250, SC2_INIT = 257, SC2_COMP = 258, SC2_FIN = 259, SC2_LAST = 260,
       SC2_REAL = 261 };
__constant__ uint32_t kShaK[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5, 0xd807aa98,
    0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786,
    0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8,
    0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13,
    0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819,
    0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a,
    0x5b9cca4f, 0x682e6ff3, 0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
    0xc67178f2};
constexpr int SCR = 20;  // dwords of an expanded row record
__device__ __forceinline__ uint32_t rotr32(uint32_t x, int s) { return (x >> s) | (x << (32 - s)); }

// zkm_sha_compress_event dwords: shard, clk, w_ptr, h_ptr, h reads (8 x 5), w reads (64 x 5), h writes (8 x 6)
__global__ __launch_bounds__(64) void k_sha_compress_expand(const uint32_t *__restrict__ ev, uint64_t ncalls,
                                                            uint32_t *__restrict__ rows) {
    const uint64_t k = (uint64_t)blockIdx.x * 64 + threadIdx.x;
    if (k >= ncalls) return;
    const uint32_t *e = ev + k * 412;
    const uint32_t *hr = e + 4, *wr = e + 44, *hw = e + 364;
    uint32_t st[8], h0[8];
#pragma unroll
    for (int i = 0; i < 8; i++) st[i] = h0[i] = hr[5 * i];
    for (int p = 0; p < 80; p++) {
        uint32_t *o = rows + (k * 80 + (uint64_t)p) * SCR;
        o[0] = e[0];
        o[1] = e[1];
        o[2] = e[2];
        o[3] = e[3];
        uint32_t wj = 0, hj = 0;
        if (p < 8) {  // init: read h[p] (prev_value = value)
            const uint32_t *r = hr + 5 * p;
            o[4] = r[0]; o[5] = r[1]; o[6] = r[2]; o[7] = r[0]; o[8] = r[3]; o[9] = r[4];
        } else if (p < 72) {  // compression: read w[p - 8]
            const uint32_t *r = wr + 5 * (p - 8);
            o[4] = r[0]; o[5] = r[1]; o[6] = r[2]; o[7] = r[0]; o[8] = r[3]; o[9] = r[4];
            wj = r[0];
        } else {  // finalize: write h[p - 72]
            const uint32_t *r = hw + 6 * (p - 72);
#pragma unroll
            for (int q = 0; q < 6; q++) o[4 + q] = r[q];
            hj = h0[p - 72];
        }
#pragma unroll
        for (int i = 0; i < 8; i++) o[10 + i] = st[i];
        o[18] = wj;
        o[19] = hj;
        if (p >= 8 && p < 72) {  // the round (the row shows the state before it)
            const uint32_t a = st[0], b = st[1], c = st[2], d = st[3], ee = st[4], f = st[5], g = st[6], hh = st[7];
            const uint32_t s1 = rotr32(ee, 6) ^ rotr32(ee, 11) ^ rotr32(ee, 25), ch = (ee & f) ^ (~ee & g);
            const uint32_t t1 = hh + s1 + ch + kShaK[p - 8] + wj;
            const uint32_t s0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22), maj = (a & b) ^ (a & c) ^ (b & c);
            const uint32_t t2 = s0 + maj;
            st[7] = g; st[6] = f; st[5] = ee; st[4] = d + t1; st[3] = c; st[2] = b; st[1] = a; st[0] = t1 + t2;
        }
    }
}

__device__ __forceinline__ uint32_t and_word(uint32_t *v, uint32_t a, uint32_t b, const Hist &h, bool on) {
#pragma unroll
    for (int i = 0; i < 4; i++) {
        v[i] = byte_of(a, i) & byte_of(b, i);
        h.byte(B_AND, byte_of(a, i), byte_of(b, i), on);
    }
    return a & b;
}
// AddOperation::populate: value bytes, 3 carries, U8 range checks of a, b and the sum
__device__ __forceinline__ uint32_t add_word(uint32_t *v, uint32_t a, uint32_t b, const Hist &h, bool on) {
    const uint32_t sum = a + b;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        v[i] = byte_of(sum, i);
        if (i < 3) {
            c = (byte_of(a, i) + byte_of(b, i) + c) >> 8;
            v[4 + i] = c;
        }
    }
    const uint32_t w3[3] = {a, b, sum};
#pragma unroll
    for (int k = 0; k < 3; k++) {
        h.byte(B_U8RANGE, byte_of(w3[k], 0), byte_of(w3[k], 1), on);
        h.byte(B_U8RANGE, byte_of(w3[k], 2), byte_of(w3[k], 3), on);
    }
    return sum;
}

struct ShaCompressChip {
    uint64_t n;  // real rows (80 per call)
    __device__ __forceinline__ void row(uint32_t *v, const uint32_t *e, uint64_t r, const Hist &h) const {
#pragma unroll
        for (int c = 0; c < ZKM_SHA_COMPRESS_WIDTH; c++) v[c] = 0;
        const bool real = e != nullptr;
        const uint32_t pos = (uint32_t)(r < n ? r % 80 : (r - n) % 80), oc = pos % 8, on = pos / 8;
        v[SC2_OCTET + oc] = 1;
        v[SC2_OCTNUM + on] = 1;
        const bool compr = on >= 1 && on <= 8;
        if (compr) put_word(v + SC2_K, kShaK[(on - 1) * 8 + oc]);
        v[SC2_LAST] = oc == 7 && on == 9;
        Access acc{};
        if (real) {
            v[SC2_REAL] = 1;
            v[SC2_INIT] = on == 0;
            v[SC2_COMP] = compr;
            v[SC2_FIN] = on == 9;
            v[SC2_START] = on == 0 && oc == 0;
            v[SC2_SHARD] = e[0];
            v[SC2_CLK] = e[1];
            v[SC2_WPTR] = e[2];
            v[SC2_HPTR] = e[3];
            acc = access_write(e + 4);
            put_word(v + SC2_MEM, acc.prev_value);
            put_access(v, SC2_MEM + 4, acc);
            v[SC2_ADDR] = pos < 8 ? e[3] + 4 * pos : pos < 72 ? e[2] + 4 * (pos - 8) : e[3] + 4 * (pos - 72);
#pragma unroll
            for (int i = 0; i < 8; i++) put_word(v + SC2_A + 4 * i, e[10 + i]);
        }
        h.byte(B_U16RANGE, acc.d16 >> 8, acc.d16 & 0xFF, real);
        h.byte(B_U8RANGE, 0, acc.d8, real);
        const bool cr = real && compr;
        uint32_t st[8];
#pragma unroll
        for (int i = 0; i < 8; i++) st[i] = real ? e[10 + i] : 0u;
        const uint32_t a = st[0], b = st[1], c = st[2], d = st[3], ee = st[4], f = st[5], g = st[6], hh = st[7];
        uint32_t tmp[12];
        const uint32_t e6 = shr_carry<6, true>(cr ? v + SC2_ERR6 : tmp, ee, h, cr);
        const uint32_t e11 = shr_carry<11, true>(cr ? v + SC2_ERR11 : tmp, ee, h, cr);
        const uint32_t e25 = shr_carry<25, true>(cr ? v + SC2_ERR25 : tmp, ee, h, cr);
        const uint32_t s1i = xor_word(cr ? v + SC2_S1I : tmp, e6, e11, h, cr);
        const uint32_t s1 = xor_word(cr ? v + SC2_S1 : tmp, s1i, e25, h, cr);
        const uint32_t eandf = and_word(cr ? v + SC2_EANDF : tmp, ee, f, h, cr);
        const uint32_t enot = ~ee;
        if (cr) put_word(v + SC2_ENOT, enot);
        h.byte(B_U8RANGE, byte_of(ee, 0), byte_of(ee, 1), cr);
        h.byte(B_U8RANGE, byte_of(ee, 2), byte_of(ee, 3), cr);
        const uint32_t enotg = and_word(cr ? v + SC2_ENOTG : tmp, enot, g, h, cr);
        const uint32_t ch = xor_word(cr ? v + SC2_CH : tmp, eandf, enotg, h, cr);
        // Add5Operation (h, s1, ch, k, w): bytes, one-hot carries (5 x 4), carries, U8 range checks
        const uint32_t kj = compr ? kShaK[(on - 1) * 8 + oc] : 0u, wj = real ? e[18] : 0u;
        const uint32_t ins[5] = {hh, s1, ch, kj, wj};
        uint32_t carry = 0, t1 = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            uint32_t t = carry;
#pragma unroll
            for (int k = 0; k < 5; k++) t += byte_of(ins[k], i);
            carry = t >> 8;
            t1 |= (t & 0xFF) << (8 * i);
            if (cr) {
                v[SC2_TEMP1 + i] = t & 0xFF;
#pragma unroll
                for (int k = 0; k < 5; k++) v[SC2_TEMP1 + 4 + 4 * k + i] = carry == (uint32_t)k;
                v[SC2_TEMP1 + 24 + i] = carry;
            }
        }
#pragma unroll
        for (int k = 0; k < 5; k++) {
            h.byte(B_U8RANGE, byte_of(ins[k], 0), byte_of(ins[k], 1), cr);
            h.byte(B_U8RANGE, byte_of(ins[k], 2), byte_of(ins[k], 3), cr);
        }
        h.byte(B_U8RANGE, byte_of(t1, 0), byte_of(t1, 1), cr);
        h.byte(B_U8RANGE, byte_of(t1, 2), byte_of(t1, 3), cr);
        const uint32_t a2 = shr_carry<2, true>(cr ? v + SC2_ARR2 : tmp, a, h, cr);
        const uint32_t a13 = shr_carry<13, true>(cr ? v + SC2_ARR13 : tmp, a, h, cr);
        const uint32_t a22 = shr_carry<22, true>(cr ? v + SC2_ARR22 : tmp, a, h, cr);
        const uint32_t s0i = xor_word(cr ? v + SC2_S0I : tmp, a2, a13, h, cr);
        const uint32_t s0 = xor_word(cr ? v + SC2_S0 : tmp, s0i, a22, h, cr);
        const uint32_t ab = and_word(cr ? v + SC2_AANDB : tmp, a, b, h, cr);
        const uint32_t ac = and_word(cr ? v + SC2_AANDC : tmp, a, c, h, cr);
        const uint32_t bc = and_word(cr ? v + SC2_BANDC : tmp, b, c, h, cr);
        const uint32_t maji = xor_word(cr ? v + SC2_MAJI : tmp, ab, ac, h, cr);
        const uint32_t maj = xor_word(cr ? v + SC2_MAJ : tmp, maji, bc, h, cr);
        const uint32_t t2 = add_word(cr ? v + SC2_TEMP2 : tmp, s0, maj, h, cr);
        add_word(cr ? v + SC2_DT1 : tmp, d, t1, h, cr);
        add_word(cr ? v + SC2_T1T2 : tmp, t1, t2, h, cr);
        // finalize rows: the final state word j and h[j] + it
        const bool fr = real && on == 9;
        const uint32_t opnd = st[oc];
        if (fr) put_word(v + SC2_FOP, opnd);
        add_word(fr ? v + SC2_FADD : tmp, real ? e[19] : 0u, opnd, h, fr);
    }
};

// ------------------------------------------------------------------ MemoryLocal (include/memory_local.hpp:8-20)
// one SingleMemoryLocal (14 columns) per event; a trace row holds four
struct MemoryLocalChip {
    __device__ __forceinline__ void row(uint32_t *v, const uint32_t *e, uint64_t, const Hist &h) const {
#pragma unroll
        for (int c = 0; c < 14; c++) v[c] = 0;
        if (!e) return;
        v[0] = e[0];            // addr
        v[1] = e[1];            // initial_shard
        v[2] = e[4];            // final_shard
        v[3] = e[2];            // initial_clk
        v[4] = e[5];            // final_clk
        put_word(v + 5, e[3]);  // initial_value
        put_word(v + 9, e[6]);  // final_value
        v[13] = 1;              // is_real
    }
};

// ------------------------------------------------------------------ MemoryGlobalInit/Finalize
// (include/memory_global.hpp:9-43 per row; memory/global.rs:133-181 across rows)
enum { MG_SHARD = 0, MG_TS = 1, MG_ADDR = 2, MG_LT = 3, MG_BITS = 35, MG_AND = 67, MG_VALUE = 73, MG_REAL = 105,
       MG_NEXT_COMP = 106, MG_IZ_INV = 107, MG_IZ_RES = 108, MG_FIRST_COMP = 109, MG_LAST_ADDR = 110 };

struct MemoryGlobalChip {
    const uint32_t *events;  // 4 dwords each: addr, value, shard, timestamp
    uint64_t n;
    uint32_t prev_addr, prev_addr_inv;

    __device__ __forceinline__ static void lt_flags(uint32_t *v, uint32_t a, uint32_t b) {
        const uint32_t x = a ^ b;  // AssertLtColsBits: the most significant differing bit
        const int top = x ? 31 - __builtin_clz(x) : -1;
#pragma unroll
        for (int i = 0; i < 32; i++) v[MG_LT + i] = i == top;
    }

    __device__ __forceinline__ void row(uint32_t *v, const uint32_t *e, uint64_t r, const Hist &) const {
#pragma unroll
        for (int c = 0; c < ZKM_MEMORY_GLOBAL_WIDTH; c++) v[c] = 0;
        if (r == 0) {  // IsZeroOperation(prev_addr) on the first row, also with no events
            v[MG_IZ_INV] = prev_addr_inv;
            v[MG_IZ_RES] = prev_addr == 0;
        }
        if (!e) return;
        const uint32_t addr = e[0], value = e[1];
        v[MG_SHARD] = e[2];
        v[MG_TS] = e[3];
        v[MG_ADDR] = addr;
#pragma unroll
        for (int i = 0; i < 32; i++) v[MG_BITS + i] = (addr >> i) & 1;
        uint32_t acc = ((addr >> 24) & 1) * ((addr >> 25) & 1);
        v[MG_AND] = acc;
#pragma unroll
        for (int k = 1; k < 6; k++) {
            acc *= (addr >> (25 + k)) & 1;
            v[MG_AND + k] = acc;
        }
#pragma unroll
        for (int i = 0; i < 32; i++) v[MG_VALUE + i] = (value >> i) & 1;
        v[MG_REAL] = 1;
        if (r == 0) {
            v[MG_FIRST_COMP] = prev_addr != 0;
            if (prev_addr != 0) lt_flags(v, prev_addr, addr);
        } else {
            v[MG_NEXT_COMP] = 1;
            lt_flags(v, events[4 * (r - 1)], addr);
        }
        if (r == n - 1) v[MG_LAST_ADDR] = 1;
    }
};

// ------------------------------------------------------------------ Syscall (include/syscall.hpp:8-16)
struct SyscallChip {
    __device__ __forceinline__ void row(uint32_t *v, const uint32_t *e, uint64_t, const Hist &h) const {
#pragma unroll
        for (int c = 0; c < ZKM_SYSCALL_WIDTH; c++) v[c] = 0;
        if (!e) return;
        v[0] = e[2];   // shard
        v[1] = e[3];   // clk
        v[2] = e[11];  // syscall_id
        v[3] = e[12];  // arg1
        v[4] = e[13];  // arg2
        v[5] = 1;      // is_real
    }
};

template <int EVS, int EVW, int W, bool HIST, class Chip>
int launch(const void *events, uint64_t n, uint32_t *trace, uint64_t nrows, const Chip &chip, void *stream,
           const char *what, uint32_t *byte_mult = nullptr, uint32_t *program_mult = nullptr) {
    if (!trace || (n && !events) || n > nrows || nrows < 16 || (nrows & (nrows - 1))) {
        g_last_error = std::string(what) + ": bad arguments (need n <= height, height a power of two >= 16)";
        return ZKM_ERR_ARG;
    }
    auto kern = k_events_to_rows<EVS, EVW, W, HIST, Chip>;
    // persistent grid: as many workgroups as fit on the device at once (each loops over tiles, so the
    // LDS tables are flushed once per resident workgroup)
    static const uint64_t resident = [&] {
        int dev = 0, cus = 256, per_cu = 1;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            cus = 256;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, NTH, 0) != hipSuccess || per_cu < 1)
            per_cu = 1;
        return (uint64_t)cus * (uint64_t)per_cu;
    }();
    const uint64_t tiles = (nrows + NTH - 1) / NTH;
    const uint64_t blocks = tiles < resident ? tiles : resident;
    hipLaunchKernelGGL(kern, dim3((uint32_t)blocks), dim3(NTH), 0, (hipStream_t)stream, (const uint32_t *)events, n,
                       trace, nrows, chip, byte_mult, program_mult);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        g_last_error = std::string(what) + ": " + hipGetErrorString(err);
        return ZKM_ERR_HIP;
    }
    return ZKM_OK;
}

uint32_t inv_mod_p(uint32_t x) {
    uint64_t r = 1, b = x % P, e = P - 2;
    while (e) {
        if (e & 1) r = r * b % P;
        b = b * b % P;
        e >>= 1;
    }
    return (uint32_t)r;
}

uint32_t inv_or_zero(uint32_t x) { return x ? inv_mod_p(x) : 0u; }

}  // namespace zkm::tg

using namespace zkm::tg;

extern "C" {

int zkm_cpu_events_to_trace(const zkm_cpu_event_ffi *events, uint64_t n, uint32_t shard,
                            const zkm_instruction_ffi *program, uint64_t program_len, uint32_t pc_base,
                            uint32_t *trace, uint64_t height, uint32_t *byte_mult, uint32_t *program_mult,
                            void *stream) {
    if (n && (!program || program_len == 0)) {
        g_last_error = "zkm_cpu_events_to_trace: empty program";
        return ZKM_ERR_ARG;
    }
    CpuChip chip{(const uint32_t *)program, program_len, pc_base, shard};
    return launch<70, E_WORDS, ZKM_CPU_WIDTH, true>(events, n, trace, height, chip, stream, "zkm_cpu_events_to_trace",
                                                    byte_mult, program_mult);
}

int zkm_add_sub_events_to_trace(const zkm_alu_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                                uint32_t *byte_mult, void *stream) {
    AddSubChip chip{};
    return launch<7, 7, ZKM_ADD_SUB_WIDTH, true>(events, n, trace, height, chip, stream, "zkm_add_sub_events_to_trace",
                                                 byte_mult);
}

int zkm_bitwise_events_to_trace(const zkm_alu_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                                uint32_t *byte_mult, void *stream) {
    return launch<7, 7, ZKM_BITWISE_WIDTH, true>(events, n, trace, height, BitwiseChip{}, stream,
                                                 "zkm_bitwise_events_to_trace", byte_mult);
}

int zkm_lt_events_to_trace(const zkm_alu_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                           uint32_t *byte_mult, void *stream) {
    return launch<7, 7, ZKM_LT_WIDTH, true>(events, n, trace, height, LtChip{}, stream, "zkm_lt_events_to_trace",
                                            byte_mult);
}

int zkm_shift_left_events_to_trace(const zkm_alu_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                                   uint32_t *byte_mult, void *stream) {
    return launch<7, 7, ZKM_SHIFT_LEFT_WIDTH, true>(events, n, trace, height, ShiftLeftChip{}, stream,
                                                    "zkm_shift_left_events_to_trace", byte_mult);
}

int zkm_shift_right_events_to_trace(const zkm_alu_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                                    uint32_t *byte_mult, void *stream) {
    return launch<7, 7, ZKM_SHIFT_RIGHT_WIDTH, true>(events, n, trace, height, ShiftRightChip{}, stream,
                                                     "zkm_shift_right_events_to_trace", byte_mult);
}

int zkm_branch_events_to_trace(const zkm_branch_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                               uint32_t *byte_mult, void *stream) {
    return launch<7, 7, ZKM_BRANCH_WIDTH, true>(events, n, trace, height, BranchChip{}, stream,
                                                "zkm_branch_events_to_trace", byte_mult);
}

int zkm_memory_instrs_events_to_trace(const zkm_mem_instr_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                                      uint32_t *byte_mult, void *stream) {
    return launch<21, 21, ZKM_MEMORY_INSTRS_WIDTH, true>(events, n, trace, height, MemoryInstrsChip{}, stream,
                                                         "zkm_memory_instrs_events_to_trace", byte_mult);
}

int zkm_jump_events_to_trace(const zkm_jump_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                             void *stream) {
    return launch<7, 7, ZKM_JUMP_WIDTH, false>(events, n, trace, height, JumpChip{}, stream, "zkm_jump_events_to_trace");
}

int zkm_movcond_events_to_trace(const zkm_movcond_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                                void *stream) {
    return launch<7, 7, ZKM_MOVCOND_WIDTH, false>(events, n, trace, height, MovCondChip{}, stream,
                                                  "zkm_movcond_events_to_trace");
}

int zkm_mul_events_to_trace(const zkm_comp_alu_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                            uint32_t *byte_mult, void *stream) {
    return launch<16, 16, ZKM_MUL_WIDTH, true>(events, n, trace, height, MulChip{}, stream, "zkm_mul_events_to_trace",
                                               byte_mult);
}

int zkm_divrem_events_to_trace(const zkm_comp_alu_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                               uint32_t *byte_mult, void *stream) {
    return launch<16, 16, ZKM_DIVREM_WIDTH, true>(events, n, trace, height, DivRemChip{}, stream,
                                                  "zkm_divrem_events_to_trace", byte_mult);
}

int zkm_clo_clz_events_to_trace(const zkm_alu_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                                uint32_t *byte_mult, void *stream) {
    return launch<7, 7, ZKM_CLO_CLZ_WIDTH, true>(events, n, trace, height, CloClzChip{}, stream,
                                                 "zkm_clo_clz_events_to_trace", byte_mult);
}

int zkm_syscall_instrs_events_to_trace(const zkm_syscall_event *events, uint64_t n, uint32_t *trace,
                                       uint64_t height, void *stream) {
    return launch<14, 14, ZKM_SYSCALL_INSTRS_WIDTH, false>(events, n, trace, height, SyscallInstrsChip{}, stream,
                                                          "zkm_syscall_instrs_events_to_trace");
}

int zkm_misc_instrs_events_to_trace(const zkm_misc_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                                    uint32_t *byte_mult, void *stream) {
    return launch<15, 15, ZKM_MISC_INSTRS_WIDTH, true>(events, n, trace, height, MiscInstrsChip{}, stream,
                                                       "zkm_misc_instrs_events_to_trace", byte_mult);
}

int zkm_sha_extend_events_to_trace(const zkm_sha_extend_row *rows, uint64_t n, uint32_t *trace, uint64_t height,
                                   uint32_t *byte_mult, void *stream) {
    if (n % 48) {
        g_last_error = "zkm_sha_extend_events_to_trace: the rows of whole calls (a multiple of 48) are needed";
        return ZKM_ERR_ARG;
    }
    ShaExtendChip chip{};
    uint64_t gk = 1;
    for (int k = 0; k < 16; k++, gk = gk * G16 % P) {
        chip.c16[k] = (uint32_t)gk;
        chip.inv_s[k] = inv_or_zero((uint32_t)((gk + P - G16) % P));
        chip.inv_e[k] = inv_or_zero((uint32_t)((gk + P - 1) % P));
    }
    return launch<29, 29, ZKM_SHA_EXTEND_WIDTH, true>(rows, n, trace, height, chip, stream,
                                                      "zkm_sha_extend_events_to_trace", byte_mult);
}

int zkm_uint256_mul_events_to_trace(const zkm_uint256_mul_event *events, uint64_t n, uint32_t *trace,
                                    uint64_t height, uint32_t *byte_mult, void *stream) {
    static_assert(sizeof(zkm_uint256_mul_event) == 4 * U2_EV, "Uint256MulEvent record");
    if (!trace || (n && !events) || n > height || height < 16 || (height & (height - 1))) {
        g_last_error = "zkm_uint256_mul_events_to_trace: bad arguments (need n <= height, a power of two >= 16)";
        return ZKM_ERR_ARG;
    }
    hipLaunchKernelGGL(k_uint256_rows, dim3((unsigned)((height + 127) / 128)), dim3(128), 0, (hipStream_t)stream,
                       (const uint32_t *)events, n, trace, height, byte_mult);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        g_last_error = std::string("zkm_uint256_mul_events_to_trace: ") + hipGetErrorString(err);
        return ZKM_ERR_HIP;
    }
    return ZKM_OK;
}

int zkm_u256x2048_mul_events_to_trace(const zkm_u256x2048_mul_event *events, uint64_t n, uint32_t *trace,
                                      uint64_t height, uint32_t *byte_mult, void *stream) {
    static_assert(sizeof(zkm_u256x2048_mul_event) == 4 * UX_EV, "U256xU2048MulEvent record");
    if (!trace || (n && !events) || n > height || height < 16 || (height & (height - 1))) {
        g_last_error = "zkm_u256x2048_mul_events_to_trace: bad arguments (need n <= height, a power of two >= 16)";
        return ZKM_ERR_ARG;
    }
    hipLaunchKernelGGL(k_u256x2048_rows, dim3((unsigned)((height + 127) / 128)), dim3(128), 0, (hipStream_t)stream,
                       (const uint32_t *)events, n, trace, height, byte_mult);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        g_last_error = std::string("zkm_u256x2048_mul_events_to_trace: ") + hipGetErrorString(err);
        return ZKM_ERR_HIP;
    }
    return ZKM_OK;
}

int zkm_fp_op_events_to_trace(int field, const zkm_fp_op_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                              uint32_t *byte_mult, void *stream) {
    static_assert(sizeof(zkm_fp_op_event) == 4 * FO_EV, "FpOpEvent record");
    if (!trace || (n && !events) || n > height || height < 16 || (height & (height - 1)) ||
        (field != ZKM_FIELD_BN254 && field != ZKM_FIELD_BLS12381)) {
        g_last_error = "zkm_fp_op_events_to_trace: bad arguments (need n <= height, a power of two >= 16, a known field)";
        return ZKM_ERR_ARG;
    }
    const dim3 grid((unsigned)((height + 127) / 128)), block(128);
    if (field == ZKM_FIELD_BN254)
        hipLaunchKernelGGL((k_fp_op_rows<8, 62, 1 << 14>), grid, block, 0, (hipStream_t)stream, (const uint32_t *)events, n,
                           trace, height, kBn254, byte_mult);
    else
        hipLaunchKernelGGL((k_fp_op_rows<12, 94, 1 << 15>), grid, block, 0, (hipStream_t)stream, (const uint32_t *)events,
                           n, trace, height, kBls, byte_mult);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        g_last_error = std::string("zkm_fp_op_events_to_trace: ") + hipGetErrorString(err);
        return ZKM_ERR_HIP;
    }
    return ZKM_OK;
}

int zkm_fp2_events_to_trace(int field, int mul, const zkm_fp2_event *events, uint64_t n, uint32_t *trace,
                            uint64_t height, uint32_t *byte_mult, void *stream) {
    static_assert(sizeof(zkm_fp2_event) == 4 * F2_EV, "Fp2 event record");
    if (!trace || (n && !events) || n > height || height < 16 || (height & (height - 1)) ||
        (field != ZKM_FIELD_BN254 && field != ZKM_FIELD_BLS12381)) {
        g_last_error = "zkm_fp2_events_to_trace: bad arguments (need n <= height, a power of two >= 16, a known field)";
        return ZKM_ERR_ARG;
    }
    const dim3 grid((unsigned)((height + 127) / 128)), block(128);
    hipStream_t s = (hipStream_t)stream;
    const uint32_t *ev = (const uint32_t *)events;
    if (field == ZKM_FIELD_BN254) {
        if (mul) hipLaunchKernelGGL((k_fp2_rows<8, 62, 1 << 14, true>), grid, block, 0, s, ev, n, trace, height, kBn254, byte_mult);
        else hipLaunchKernelGGL((k_fp2_rows<8, 62, 1 << 14, false>), grid, block, 0, s, ev, n, trace, height, kBn254, byte_mult);
    } else {
        if (mul) hipLaunchKernelGGL((k_fp2_rows<12, 94, 1 << 15, true>), grid, block, 0, s, ev, n, trace, height, kBls, byte_mult);
        else hipLaunchKernelGGL((k_fp2_rows<12, 94, 1 << 15, false>), grid, block, 0, s, ev, n, trace, height, kBls, byte_mult);
    }
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        g_last_error = std::string("zkm_fp2_events_to_trace: ") + hipGetErrorString(err);
        return ZKM_ERR_HIP;
    }
    return ZKM_OK;
}

int zkm_ec_add_events_to_trace(int curve, const zkm_ec_add_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                               uint32_t *byte_mult, void *stream) {
    static_assert(sizeof(zkm_ec_add_event) == 4 * EA_EV, "EllipticCurveAddEvent record");
    if (!trace || (n && !events) || n > height || height < 16 || (height & (height - 1)) || curve < 0 || curve > 3) {
        g_last_error = "zkm_ec_add_events_to_trace: bad arguments (need n <= height, a power of two >= 16, a known curve)";
        return ZKM_ERR_ARG;
    }
    const dim3 grid((unsigned)((height + 127) / 128)), block(128);
    hipStream_t s = (hipStream_t)stream;
    const uint32_t *ev = (const uint32_t *)events;
    if (curve == ZKM_CURVE_BLS12381)
        hipLaunchKernelGGL((k_ec_add_rows<12, 94, 1 << 15>), grid, block, 0, s, ev, n, trace, height, kBls, byte_mult);
    else
        hipLaunchKernelGGL((k_ec_add_rows<8, 62, 1 << 14>), grid, block, 0, s, ev, n, trace, height,
                           curve == ZKM_CURVE_SECP256K1 ? kSecp256k1 : curve == ZKM_CURVE_SECP256R1 ? kSecp256r1 : kBn254,
                           byte_mult);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        g_last_error = std::string("zkm_ec_add_events_to_trace: ") + hipGetErrorString(err);
        return ZKM_ERR_HIP;
    }
    return ZKM_OK;
}

int zkm_ec_double_events_to_trace(int curve, const zkm_ec_double_event *events, uint64_t n, uint32_t *trace,
                                  uint64_t height, uint32_t *byte_mult, void *stream) {
    static_assert(sizeof(zkm_ec_double_event) == 4 * ED2_EV, "EllipticCurveDoubleEvent record");
    if (!trace || (n && !events) || n > height || height < 16 || (height & (height - 1)) || curve < 0 || curve > 3) {
        g_last_error = "zkm_ec_double_events_to_trace: bad arguments (need n <= height, a power of two >= 16, a known curve)";
        return ZKM_ERR_ARG;
    }
    // the curves' a: 0 except secp256r1 (p - 3)
    constexpr FpMod a0{{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}};
    constexpr FpMod a_r1{{0xfffffffcu, 0xffffffffu, 0xffffffffu, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000001u,
                          0xffffffffu, 0, 0, 0, 0}};
    const dim3 grid((unsigned)((height + 127) / 128)), block(128);
    hipStream_t s = (hipStream_t)stream;
    const uint32_t *ev = (const uint32_t *)events;
    if (curve == ZKM_CURVE_BLS12381)
        hipLaunchKernelGGL((k_ec_double_rows<12, 94, 1 << 15>), grid, block, 0, s, ev, n, trace, height, kBls, a0, byte_mult);
    else
        hipLaunchKernelGGL((k_ec_double_rows<8, 62, 1 << 14>), grid, block, 0, s, ev, n, trace, height,
                           curve == ZKM_CURVE_SECP256K1 ? kSecp256k1 : curve == ZKM_CURVE_SECP256R1 ? kSecp256r1 : kBn254,
                           curve == ZKM_CURVE_SECP256R1 ? a_r1 : a0, byte_mult);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        g_last_error = std::string("zkm_ec_double_events_to_trace: ") + hipGetErrorString(err);
        return ZKM_ERR_HIP;
    }
    return ZKM_OK;
}

int zkm_ec_decompress_events_to_trace(int curve, const zkm_ec_decompress_event *events, uint64_t n, uint32_t *trace,
                                      uint64_t height, uint32_t *byte_mult, void *stream) {
    static_assert(sizeof(zkm_ec_decompress_event) == 4 * EDC_EV, "EllipticCurveDecompressEvent record");
    if (!trace || (n && !events) || n > height || height < 16 || (height & (height - 1)) ||
        (curve != ZKM_CURVE_SECP256K1 && curve != ZKM_CURVE_SECP256R1 && curve != ZKM_CURVE_BLS12381)) {
        g_last_error = "zkm_ec_decompress_events_to_trace: bad arguments (need n <= height, a power of two >= 16, "
                       "secp256k1, secp256r1 or bls12-381)";
        return ZKM_ERR_ARG;
    }
    const dim3 grid((unsigned)((height + 127) / 128)), block(128);
    hipStream_t s = (hipStream_t)stream;
    const uint32_t *ev = (const uint32_t *)events;
    if (curve == ZKM_CURVE_BLS12381) {
        const CurveConsts cc{kBls, kSqrtExpBLS, kGenXBLS, kCurveABLS, kCurveBBLS};
        hipLaunchKernelGGL((k_ec_decompress_rows<12, 94, 1 << 15, true>), grid, block, 0, s, ev, n, trace, height, cc,
                           byte_mult);
    } else {
        const CurveConsts cc = curve == ZKM_CURVE_SECP256K1
                                   ? CurveConsts{kSecp256k1, kSqrtExpK1, kGenXK1, kCurveAK1, kCurveBK1}
                                   : CurveConsts{kSecp256r1, kSqrtExpR1, kGenXR1, kCurveAR1, kCurveBR1};
        hipLaunchKernelGGL((k_ec_decompress_rows<8, 62, 1 << 14, false>), grid, block, 0, s, ev, n, trace, height, cc,
                           byte_mult);
    }
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        g_last_error = std::string("zkm_ec_decompress_events_to_trace: ") + hipGetErrorString(err);
        return ZKM_ERR_HIP;
    }
    return ZKM_OK;
}

int zkm_ed_add_events_to_trace(const zkm_ed_add_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                               uint32_t *byte_mult, void *stream) {
    static_assert(sizeof(zkm_ed_add_event) == 4 * EDA_EV, "EllipticCurveAddEvent (Ed25519) record");
    if (!trace || (n && !events) || n > height || height < 16 || (height & (height - 1))) {
        g_last_error = "zkm_ed_add_events_to_trace: bad arguments (need n <= height, a power of two >= 16)";
        return ZKM_ERR_ARG;
    }
    hipLaunchKernelGGL(k_ed_add_rows, dim3((unsigned)((height + 127) / 128)), dim3(128), 0, (hipStream_t)stream,
                       (const uint32_t *)events, n, trace, height, byte_mult);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        g_last_error = std::string("zkm_ed_add_events_to_trace: ") + hipGetErrorString(err);
        return ZKM_ERR_HIP;
    }
    return ZKM_OK;
}

int zkm_ed_decompress_events_to_trace(const zkm_ed_decompress_event *events, uint64_t n, uint32_t *trace,
                                      uint64_t height, uint32_t *byte_mult, void *stream) {
    static_assert(sizeof(zkm_ed_decompress_event) == 4 * EDD_EV, "EdDecompressEvent record");
    if (!trace || (n && !events) || n > height || height < 16 || (height & (height - 1))) {
        g_last_error = "zkm_ed_decompress_events_to_trace: bad arguments (need n <= height, a power of two >= 16)";
        return ZKM_ERR_ARG;
    }
    hipLaunchKernelGGL(k_ed_decompress_rows, dim3((unsigned)((height + 127) / 128)), dim3(128), 0, (hipStream_t)stream,
                       (const uint32_t *)events, n, trace, height, byte_mult);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        g_last_error = std::string("zkm_ed_decompress_events_to_trace: ") + hipGetErrorString(err);
        return ZKM_ERR_HIP;
    }
    return ZKM_OK;
}

int zkm_keccak_sponge_events_to_trace(const zkm_keccak_block *blocks, uint64_t n, uint32_t *trace, uint64_t height,
                                      uint32_t *byte_mult, void *stream) {
    static_assert(sizeof(zkm_keccak_block) == 4 * KS_EV, "KeccakSponge block record");
    if (!trace || (n && !blocks) || 24 * n > height || height < 16 || (height & (height - 1))) {
        g_last_error = "zkm_keccak_sponge_events_to_trace: bad arguments (need 24 n <= height, a power of two >= 16)";
        return ZKM_ERR_ARG;
    }
    hipLaunchKernelGGL(k_keccak_sponge_rows, dim3((unsigned)((height + 63) / 64)), dim3(64), 0, (hipStream_t)stream,
                       (const uint32_t *)blocks, n, trace, height, byte_mult);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        g_last_error = std::string("zkm_keccak_sponge_events_to_trace: ") + hipGetErrorString(err);
        return ZKM_ERR_HIP;
    }
    return ZKM_OK;
}

int zkm_sys_linux_events_to_trace(const zkm_sys_linux_event *events, uint64_t n, uint32_t *trace, uint64_t height,
                                  uint32_t *byte_mult, void *stream) {
    static_assert(sizeof(zkm_sys_linux_event) == 4 * LX_EV, "LinuxEvent record");
    return launch<LX_EV, LX_EV, ZKM_SYS_LINUX_WIDTH, true>(events, n, trace, height, SysLinuxChip{}, stream,
                                                          "zkm_sys_linux_events_to_trace", byte_mult);
}

int zkm_poseidon2_permute_events_to_trace(const zkm_poseidon2_permute_event *events, uint64_t n, uint32_t *trace,
                                          uint64_t height, uint32_t *byte_mult, void *stream) {
    static_assert(sizeof(zkm_poseidon2_permute_event) == 4 * PM_EV, "Poseidon2PermuteEvent record");
    if (!trace || (n && !events) || n > height || height < 16 || (height & (height - 1))) {
        g_last_error = "zkm_poseidon2_permute_events_to_trace: bad arguments (need n <= height, a power of two >= 16)";
        return ZKM_ERR_ARG;
    }
    hipLaunchKernelGGL(k_p2permute_rows, dim3((unsigned)(height / PM_ROWS)), dim3(16 * PM_ROWS), 0, (hipStream_t)stream,
                       (const uint32_t *)events, n, trace, byte_mult);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        g_last_error = std::string("zkm_poseidon2_permute_events_to_trace: ") + hipGetErrorString(err);
        return ZKM_ERR_HIP;
    }
    return ZKM_OK;
}

int zkm_sha_compress_events_to_trace(const zkm_sha_compress_event *events, uint64_t n, uint32_t *trace,
                                     uint64_t height, uint32_t *byte_mult, void *stream) {
    const uint64_t nrows = 80 * n;
    if (!trace || (n && !events) || nrows > height || height < 16 || (height & (height - 1))) {
        g_last_error = "zkm_sha_compress_events_to_trace: bad arguments (need 80 n <= height, a power of two >= 16)";
        return ZKM_ERR_ARG;
    }
    hipStream_t s = (hipStream_t)stream;
    uint32_t *rows = nullptr;
    if (n) {
        if (hipMallocAsync((void **)&rows, nrows * SCR * 4, s) != hipSuccess) {
            g_last_error = "zkm_sha_compress_events_to_trace: out of device memory";
            return ZKM_ERR_HIP;
        }
        hipLaunchKernelGGL(k_sha_compress_expand, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, s,
                           (const uint32_t *)events, n, rows);
    }
    const int rc = launch<SCR, SCR, ZKM_SHA_COMPRESS_WIDTH, true>(rows, nrows, trace, height, ShaCompressChip{nrows},
                                                                  stream, "zkm_sha_compress_events_to_trace", byte_mult);
    if (rows) (void)hipFreeAsync(rows, s);  // stream-ordered: after the row kernel
    return rc;
}

int zkm_memory_local_events_to_trace(const zkm_memory_local_event *events, uint64_t n, uint32_t *trace,
                                     uint64_t height, void *stream) {
    if (height < 16 || (height & (height - 1)) || n > 4 * height) {
        g_last_error = "zkm_memory_local_events_to_trace: bad arguments";
        return ZKM_ERR_ARG;
    }
    MemoryLocalChip chip{};
    return launch<7, 7, 14, false>(events, n, trace, 4 * height, chip, stream, "zkm_memory_local_events_to_trace");
}

int zkm_memory_global_events_to_trace(const zkm_memory_init_final_event *events, uint64_t n, int is_receive,
                                      uint32_t prev_addr, uint32_t *trace, uint64_t height, void *stream) {
    (void)is_receive;  // the columns are the same for both chips (memory_global.hpp:11-20 builds an unused record)
    MemoryGlobalChip chip{(const uint32_t *)events, n, prev_addr, prev_addr ? inv_mod_p(prev_addr) : 0u};
    return launch<4, 4, ZKM_MEMORY_GLOBAL_WIDTH, false>(events, n, trace, height, chip, stream,
                                                 "zkm_memory_global_events_to_trace");
}

int zkm_syscall_events_to_trace(const zkm_syscall_event *events, uint64_t n, int is_receive, uint32_t *trace,
                                uint64_t height, void *stream) {
    (void)is_receive;  // syscall.hpp:8-16: the same row for SyscallCore and SyscallPrecompile
    SyscallChip chip{};
    return launch<14, 14, ZKM_SYSCALL_WIDTH, false>(events, n, trace, height, chip, stream, "zkm_syscall_events_to_trace");
}

}  // extern "C"
