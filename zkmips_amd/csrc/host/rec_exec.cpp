// The recursion runtime (recursion/core/src/runtime/mod.rs:336-625) as native host code, for the compress
// nodes' witness generation: the program arrives flattened by instruction kind (zkmips_amd/recursion.py
// FlatProgram: every kind's operand arrays concatenated in program order, a block table giving each run
// of same-kind instructions its kind, first entry, length, row length and first flat row) and executes
// block by block with the semantics of recursion.execute_numpy:
//   * memory is write-once: every read must hit an address an earlier block wrote, every write a fresh one;
//   * a block's reads are checked before any of its writes (instructions of one block are independent);
//   * constant-memory reads must equal the stated value.
// The events come back as the chips' main-trace rows (alu_base.hpp / alu_ext.hpp / select.hpp /
// batch_fri.hpp / fri_fold.hpp / exp_reverse_bits.hpp event_to_row; Poseidon2 as (input, output) pairs),
// canonical words, concatenated per kind in program order.  Single-threaded: the callers are
// witness-generation worker processes, one per core.
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <memory>
#include <vector>

#include "../p2.cuh"

namespace zkm_host {
uint64_t p2_simd_permute(const uint32_t *in, size_t in_stride, uint32_t *out, size_t out_stride, uint64_t n);
}

namespace {
constexpr uint64_t P = 0x7f000001u;

enum Kind { K_MEM, K_HINT, K_BASE, K_EXT, K_P2, K_SELECT, K_EXPREV, K_BATCHFRI, K_FRIFOLD, K_COMMIT };
// pointer slots (recursion.py _RX_SLOTS has the same order)
enum Slot {
    MEM_ADDR, MEM_VALS, MEM_WRITE, HINT_ADDR, HINT_VALS,
    BASE_OP, BASE_OUT, BASE_IN1, BASE_IN2, BASE_EV,
    EXT_OP, EXT_OUT, EXT_IN1, EXT_IN2, EXT_EV,
    P2_OUT, P2_INP, P2_EV,
    SEL_BIT, SEL_OUT1, SEL_OUT2, SEL_IN1, SEL_IN2, SEL_EV,
    ER_BASE, ER_RESULT, ER_EXPS, ER_ROWS,
    BF_ACC, BF_AP, BF_PZ, BF_PX, BF_ROWS,
    FF_X, FF_Z, FF_ALPHA, FF_PX, FF_PZ, FF_API, FF_ROI, FF_APO, FF_ROO, FF_ROWS,
    PV_ADDRS, PV_EV, MEM_IMAGE, NUM_SLOTS
};
constexpr int NUM_PVS = 231;
constexpr uint64_t OP_ADD = 0, OP_SUB = 1, OP_MUL = 2, OP_DIV = 3;

inline uint64_t fadd(uint64_t a, uint64_t b) {  // a, b < P
    const uint64_t s = a + b;
    return s >= P ? s - P : s;
}
inline uint64_t fsub(uint64_t a, uint64_t b) { return a >= b ? a - b : a + P - b; }  // a, b < P
inline uint64_t fmul(uint64_t a, uint64_t b) { return a * b % P; }
inline uint64_t fpow(uint64_t a, uint64_t e) {
    uint64_t r = 1;
    for (a %= P; e; e >>= 1, a = a * a % P)
        if (e & 1) r = r * a % P;
    return r;
}
inline uint64_t finv(uint64_t a) { return fpow(a, P - 2); }  // 0 -> 0, as the numpy runtime

struct Ef {
    uint64_t c[4];
};
inline Ef ef_mul(const Ef &a, const Ef &b) {  // X^4 = 3; coefficients < P: four products < 4 P^2 < 2^64
    uint64_t t[7] = {0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) t[i + j] += a.c[i] * b.c[j];
    Ef r;
    for (int k = 0; k < 4; k++) r.c[k] = (t[k] % P + (k < 3 ? 3 * (t[k + 4] % P) : 0)) % P;
    return r;
}
inline Ef ef_add(const Ef &a, const Ef &b) {
    Ef r;
    for (int k = 0; k < 4; k++) r.c[k] = fadd(a.c[k], b.c[k]);
    return r;
}
inline Ef ef_sub(const Ef &a, const Ef &b) {
    Ef r;
    for (int k = 0; k < 4; k++) r.c[k] = fsub(a.c[k], b.c[k]);
    return r;
}
// a^-1 by a(x) a(-x) = b0 + b2 x^2 and (b0 + b2 y)(b0 - b2 y) = b0^2 - 3 b2^2 (recursion.ext_inv); 0 -> 0
inline Ef ef_inv(const Ef &a) {
    const Ef conj{{a.c[0], (P - a.c[1]) % P, a.c[2], (P - a.c[3]) % P}};
    const Ef b = ef_mul(a, conj);
    const uint64_t n = fsub(fmul(b.c[0], b.c[0]), fmul(3, fmul(b.c[2], b.c[2])));
    const uint64_t ni = finv(n);
    const Ef c{{b.c[0], 0, (P - b.c[2]) % P, 0}};
    Ef r = ef_mul(conj, c);
    for (int k = 0; k < 4; k++) r.c[k] = fmul(r.c[k], ni);
    return r;
}

struct Vm {
    uint64_t n_addrs;
    std::unique_ptr<uint32_t[]> mem;  // not zeroed: a word is read only after its address was written
    std::vector<uint8_t> written;
    char *err;
    uint64_t err_len;
    int64_t block = 0;

    int fail(const char *what) {
        if (err && err_len) snprintf(err, err_len, "%s (block %lld)", what, (long long)block);
        return 1;
    }
    bool readable(int64_t a) const { return a >= 0 && (uint64_t)a < n_addrs && written[a]; }
    int check_reads(const int64_t *addrs, uint64_t n) {
        for (uint64_t i = 0; i < n; i++)
            if (!readable(addrs[i])) return fail("read of an unassigned address");
        return 0;
    }
    uint64_t rd(int64_t a) const { return mem[4 * a]; }
    Ef rd_ef(int64_t a) const { return Ef{{mem[4 * a], mem[4 * a + 1], mem[4 * a + 2], mem[4 * a + 3]}}; }
    int wr(int64_t a, const uint64_t v[4]) {
        if (a < 0 || (uint64_t)a >= n_addrs || written[a]) return fail("write to an assigned address");
        for (int k = 0; k < 4; k++) mem[4 * a + k] = (uint32_t)(v[k] % P);
        written[a] = 1;
        return 0;
    }
    int wr1(int64_t a, uint64_t v) {
        const uint64_t b[4] = {v, 0, 0, 0};
        return wr(a, b);
    }
    int wr_ef(int64_t a, const Ef &e) { return wr(a, e.c); }
};

template <class T>
inline const T *cp(const void *const *s, int i) { return static_cast<const T *>(s[i]); }
template <class T>
inline T *mp(void *const *s, int i) { return static_cast<T *>(s[i]); }
}  // namespace

// table: nblocks x 5 int64 (kind, entry start, count, row length L, flat start); slots: NUM_SLOTS pointers
// (inputs const, outputs written; unused kinds may be null).  Returns 0, or 1 with a message in err.
extern "C" int zkm_host_recursion_execute(uint64_t num_addrs, uint64_t nblocks, const int64_t *table,
                                          void *const *slots, char *err, uint64_t err_len) {
    Vm vm{num_addrs, std::unique_ptr<uint32_t[]>(new uint32_t[4 * num_addrs]), std::vector<uint8_t>(num_addrs, 0), err,
          err_len};
    const void *const *in = const_cast<const void *const *>(slots);
    uint64_t n_commit = 0;
    for (uint64_t bi = 0; bi < nblocks; bi++) {
        vm.block = (int64_t)bi;
        const int64_t *t = table + 5 * bi;
        const int kind = (int)t[0];
        const uint64_t s = (uint64_t)t[1], n = (uint64_t)t[2], L = (uint64_t)t[3], fs = (uint64_t)t[4];
        switch (kind) {
            case K_MEM: {
                const int64_t *addr = cp<int64_t>(in, MEM_ADDR) + s;
                const uint32_t *vals = cp<uint32_t>(in, MEM_VALS) + 4 * s;
                const uint8_t *w = cp<uint8_t>(in, MEM_WRITE) + s;
                for (uint64_t i = 0; i < n; i++)
                    if (!w[i] && !vm.readable(addr[i])) return vm.fail("read of an unassigned address");
                for (uint64_t i = 0; i < n; i++)
                    if (!w[i])
                        for (int k = 0; k < 4; k++)
                            if (vm.mem[4 * addr[i] + k] != vals[4 * i + k] % P)
                                return vm.fail("stored memory value should be the specified value");
                for (uint64_t i = 0; i < n; i++)
                    if (w[i]) {
                        const uint64_t v[4] = {vals[4 * i], vals[4 * i + 1], vals[4 * i + 2], vals[4 * i + 3]};
                        if (vm.wr(addr[i], v)) return 1;
                    }
                break;
            }
            case K_HINT: {
                const int64_t *addr = cp<int64_t>(in, HINT_ADDR) + s;
                const uint32_t *vals = cp<uint32_t>(in, HINT_VALS) + 4 * s;
                for (uint64_t i = 0; i < n; i++) {
                    const uint64_t v[4] = {vals[4 * i], vals[4 * i + 1], vals[4 * i + 2], vals[4 * i + 3]};
                    if (vm.wr(addr[i], v)) return 1;
                }
                break;
            }
            case K_BASE:
            case K_EXT: {
                const bool ext = kind == K_EXT;
                const int64_t *op = cp<int64_t>(in, ext ? EXT_OP : BASE_OP) + s;
                const int64_t *out = cp<int64_t>(in, ext ? EXT_OUT : BASE_OUT) + s;
                const int64_t *i1 = cp<int64_t>(in, ext ? EXT_IN1 : BASE_IN1) + s;
                const int64_t *i2 = cp<int64_t>(in, ext ? EXT_IN2 : BASE_IN2) + s;
                if (vm.check_reads(i1, n) || vm.check_reads(i2, n)) return 1;
                uint32_t *ev = mp<uint32_t>(slots, ext ? EXT_EV : BASE_EV) + (ext ? 12 : 3) * s;
                for (uint64_t i = 0; i < n; i++) {
                    if (ext) {
                        const Ef x = vm.rd_ef(i1[i]), y = vm.rd_ef(i2[i]);
                        Ef o;
                        switch (op[i]) {
                            case OP_ADD: o = ef_add(x, y); break;
                            case OP_SUB: o = ef_sub(x, y); break;
                            case OP_MUL: o = ef_mul(x, y); break;
                            case OP_DIV:
                            default: o = ef_mul(x, ef_inv(y)); break;
                        }
                        for (int k = 0; k < 4; k++) {
                            ev[12 * i + k] = (uint32_t)o.c[k];
                            ev[12 * i + 4 + k] = (uint32_t)x.c[k];
                            ev[12 * i + 8 + k] = (uint32_t)y.c[k];
                        }
                    } else {
                        const uint64_t x = vm.rd(i1[i]), y = vm.rd(i2[i]);
                        const uint64_t o = op[i] == (int64_t)OP_ADD   ? fadd(x, y)
                                           : op[i] == (int64_t)OP_SUB ? fsub(x, y)
                                           : op[i] == (int64_t)OP_MUL ? fmul(x, y)
                                                                      : fmul(x, finv(y));
                        ev[3 * i] = (uint32_t)o;
                        ev[3 * i + 1] = (uint32_t)x;
                        ev[3 * i + 2] = (uint32_t)y;
                    }
                }
                for (uint64_t i = 0; i < n; i++) {
                    if (ext) {
                        const Ef o{{ev[12 * i], ev[12 * i + 1], ev[12 * i + 2], ev[12 * i + 3]}};
                        if (vm.wr_ef(out[i], o)) return 1;
                    } else if (vm.wr1(out[i], ev[3 * i])) {
                        return 1;
                    }
                }
                break;
            }
            case K_P2: {
                const int64_t *inp = cp<int64_t>(in, P2_INP) + 16 * s;
                const int64_t *out = cp<int64_t>(in, P2_OUT) + 16 * s;
                if (vm.check_reads(inp, 16 * n)) return 1;
                uint32_t *ev = mp<uint32_t>(slots, P2_EV) + 32 * s;
                for (uint64_t i = 0; i < 16 * n; i++) ev[32 * (i / 16) + i % 16] = (uint32_t)vm.rd(inp[i]);
                // sixteen permutations at a time where the CPU has AVX-512 (p2_simd.cpp), else one by one
                for (uint64_t i = zkm_host::p2_simd_permute(ev, 32, ev + 16, 32, n); i < n; i++) {
                    uint32_t st[16];
                    for (int j = 0; j < 16; j++) st[j] = kb::to_mont(ev[32 * i + j]);
                    p2::permute(st);
                    for (int j = 0; j < 16; j++) ev[32 * i + 16 + j] = kb::from_mont(st[j]);
                }
                for (uint64_t i = 0; i < 16 * n; i++)
                    if (vm.wr1(out[i], ev[32 * (i / 16) + 16 + i % 16])) return 1;
                break;
            }
            case K_SELECT: {
                const int64_t *bit = cp<int64_t>(in, SEL_BIT) + s, *o1 = cp<int64_t>(in, SEL_OUT1) + s,
                              *o2 = cp<int64_t>(in, SEL_OUT2) + s, *i1 = cp<int64_t>(in, SEL_IN1) + s,
                              *i2 = cp<int64_t>(in, SEL_IN2) + s;
                if (vm.check_reads(bit, n) || vm.check_reads(i1, n) || vm.check_reads(i2, n)) return 1;
                uint32_t *ev = mp<uint32_t>(slots, SEL_EV) + 5 * s;
                for (uint64_t i = 0; i < n; i++) {
                    const uint64_t b = vm.rd(bit[i]), x = vm.rd(i1[i]), y = vm.rd(i2[i]);
                    ev[5 * i] = (uint32_t)b;
                    if (b <= 1) {  // a bit: the products pick
                        ev[5 * i + 1] = (uint32_t)(b ? y : x);
                        ev[5 * i + 2] = (uint32_t)(b ? x : y);
                    } else {
                        const uint64_t nb = (P + 1 - b) % P;
                        ev[5 * i + 1] = (uint32_t)fadd(fmul(b, y), fmul(nb, x));
                        ev[5 * i + 2] = (uint32_t)fadd(fmul(b, x), fmul(nb, y));
                    }
                    ev[5 * i + 3] = (uint32_t)x;
                    ev[5 * i + 4] = (uint32_t)y;
                }
                for (uint64_t i = 0; i < n; i++)
                    if (vm.wr1(o1[i], ev[5 * i + 1])) return 1;
                for (uint64_t i = 0; i < n; i++)
                    if (vm.wr1(o2[i], ev[5 * i + 2])) return 1;
                break;
            }
            case K_EXPREV: {
                const int64_t *base = cp<int64_t>(in, ER_BASE) + s, *res = cp<int64_t>(in, ER_RESULT) + s;
                const int64_t *exps = cp<int64_t>(in, ER_EXPS) + fs;
                if (vm.check_reads(base, n) || vm.check_reads(exps, n * L)) return 1;
                uint32_t *rows = mp<uint32_t>(slots, ER_ROWS) + 7 * fs;
                std::vector<uint64_t> acc(n, 1);
                for (uint64_t q = 0; q < n; q++) {
                    const uint64_t x = vm.rd(base[q]);
                    uint64_t a = 1;
                    for (uint64_t i = 0; i < L; i++) {
                        const uint64_t bit = vm.rd(exps[q * L + i]);
                        const uint64_t mult = bit == 1 ? x : 1;
                        const uint64_t psq = fmul(a, a);
                        a = fmul(psq, mult);
                        uint32_t *r = rows + 7 * (q * L + i);
                        r[0] = (uint32_t)x;
                        r[1] = (uint32_t)bit;
                        r[2] = (uint32_t)psq;
                        r[3] = (uint32_t)a;
                        r[4] = (uint32_t)a;
                        r[5] = (uint32_t)fmul(a, a);
                        r[6] = (uint32_t)mult;
                    }
                    acc[q] = a;
                }
                for (uint64_t q = 0; q < n; q++)
                    if (vm.wr1(res[q], acc[q])) return 1;
                break;
            }
            case K_BATCHFRI: {
                const int64_t *acc = cp<int64_t>(in, BF_ACC) + s;
                const int64_t *ap = cp<int64_t>(in, BF_AP) + fs, *pz = cp<int64_t>(in, BF_PZ) + fs,
                              *px = cp<int64_t>(in, BF_PX) + fs;
                if (vm.check_reads(px, n * L) || vm.check_reads(pz, n * L) || vm.check_reads(ap, n * L)) return 1;
                uint32_t *rows = mp<uint32_t>(slots, BF_ROWS) + 13 * fs;
                std::vector<Ef> res(n, Ef{{0, 0, 0, 0}});
                for (uint64_t q = 0; q < n; q++) {
                    Ef run{{0, 0, 0, 0}};
                    for (uint64_t i = 0; i < L; i++) {
                        const uint64_t e = q * L + i;
                        const Ef al = vm.rd_ef(ap[e]), z = vm.rd_ef(pz[e]);
                        const uint64_t x = vm.rd(px[e]);
                        Ef d = z;
                        d.c[0] = fsub(d.c[0], x);
                        run = ef_add(run, ef_mul(al, d));
                        uint32_t *r = rows + 13 * e;
                        for (int k = 0; k < 4; k++) {
                            r[k] = (uint32_t)run.c[k];
                            r[4 + k] = (uint32_t)al.c[k];
                            r[8 + k] = (uint32_t)z.c[k];
                        }
                        r[12] = (uint32_t)x;
                    }
                    res[q] = run;
                }
                for (uint64_t q = 0; q < n; q++)
                    if (vm.wr_ef(acc[q], res[q])) return 1;
                break;
            }
            case K_FRIFOLD: {
                const int64_t xa = cp<int64_t>(in, FF_X)[s], za = cp<int64_t>(in, FF_Z)[s],
                              aa = cp<int64_t>(in, FF_ALPHA)[s];
                const int64_t *pxa = cp<int64_t>(in, FF_PX) + fs, *pza = cp<int64_t>(in, FF_PZ) + fs,
                              *apa = cp<int64_t>(in, FF_API) + fs, *roa = cp<int64_t>(in, FF_ROI) + fs,
                              *apo = cp<int64_t>(in, FF_APO) + fs, *roo = cp<int64_t>(in, FF_ROO) + fs;
                if (vm.check_reads(&xa, 1) || vm.check_reads(&za, 1) || vm.check_reads(&aa, 1) ||
                    vm.check_reads(pxa, L) || vm.check_reads(pza, L) || vm.check_reads(apa, L) ||
                    vm.check_reads(roa, L))
                    return 1;
                const uint64_t x = vm.rd(xa);
                const Ef z = vm.rd_ef(za), alpha = vm.rd_ef(aa);
                Ef xz{{(P - z.c[0]) % P, (P - z.c[1]) % P, (P - z.c[2]) % P, (P - z.c[3]) % P}};
                xz.c[0] = fadd(xz.c[0], x);
                const Ef xzi = ef_inv(xz);
                uint32_t *rows = mp<uint32_t>(slots, FF_ROWS) + 33 * fs;
                std::vector<Ef> nro(L), nap(L);
                for (uint64_t i = 0; i < L; i++) {
                    const Ef px = vm.rd_ef(pxa[i]), pz = vm.rd_ef(pza[i]), ap = vm.rd_ef(apa[i]), ro = vm.rd_ef(roa[i]);
                    const Ef q = ef_mul(ef_sub(px, pz), xzi);
                    nro[i] = ef_add(ro, ef_mul(ap, q));
                    nap[i] = ef_mul(ap, alpha);
                    uint32_t *r = rows + 33 * i;
                    for (int k = 0; k < 4; k++) {
                        r[k] = (uint32_t)z.c[k];
                        r[4 + k] = (uint32_t)alpha.c[k];
                        r[9 + k] = (uint32_t)px.c[k];
                        r[13 + k] = (uint32_t)pz.c[k];
                        r[17 + k] = (uint32_t)ap.c[k];
                        r[21 + k] = (uint32_t)ro.c[k];
                        r[25 + k] = (uint32_t)nap[i].c[k];
                        r[29 + k] = (uint32_t)nro[i].c[k];
                    }
                    r[8] = (uint32_t)x;
                }
                for (uint64_t i = 0; i < L; i++)
                    if (vm.wr_ef(roo[i], nro[i])) return 1;
                for (uint64_t i = 0; i < L; i++)
                    if (vm.wr_ef(apo[i], nap[i])) return 1;
                break;
            }
            case K_COMMIT: {
                const int64_t *pv = cp<int64_t>(in, PV_ADDRS) + NUM_PVS * s;
                if (vm.check_reads(pv, NUM_PVS)) return 1;
                uint32_t *ev = mp<uint32_t>(slots, PV_EV) + NUM_PVS * s;
                for (int i = 0; i < NUM_PVS; i++) ev[i] = (uint32_t)vm.rd(pv[i]);
                n_commit++;
                break;
            }
            default:
                return vm.fail("unknown instruction kind");
        }
    }
    if (slots[MEM_IMAGE]) {  // (the image has zeros at unwritten addresses)
        uint32_t *img = static_cast<uint32_t *>(slots[MEM_IMAGE]);
        for (uint64_t a = 0; a < num_addrs; a++)
            for (int k = 0; k < 4; k++) img[4 * a + k] = vm.written[a] ? vm.mem[4 * a + k] : 0u;
    }
    (void)n_commit;
    return 0;
}
