// Host trace generation for the Global chip: the septic extension F_{p^7} = F_p[z]/(z^7 + 2z - 8),
// the curve y^2 = x^3 + 3z x - 3 over it, lift_x, and the cumulative sum of lookup digests.
//
// Reference (restated, canonical u32 residues):
//   crates/stark/src/septic_extension.rs   mul :300-316, frobenius :575-598, inverse :601-613,
//                                          sqrt :615-674, is_send/is_receive/is_exception :677-693
//   crates/stark/src/septic_curve.rs       curve_formula :101-122, add_incomplete :53-58,
//                                          double :69-84, lift_x :130-154, complete add :198-217
//   crates/stark/src/septic_digest.rs      zero / starting digests :8-50, Sum :57-73
//   crates/core/machine/src/operations/global_lookup.rs   get_digest :26-38 (x = message + kind << 16)
//   crates/core/machine/src/global/mod.rs  generate_trace :110-196 (scan from the zero digest)
// sqrt may return either root; lift_x normalises the sign (y_6 in [1, (p-1)/2]), so the result is the
// reference's whatever square-root algorithm computes it.
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

constexpr uint32_t P = 0x7f000001u;

inline uint32_t add(uint32_t a, uint32_t b) { uint32_t s = a + b; return s >= P ? s - P : s; }
inline uint32_t sub(uint32_t a, uint32_t b) { return a >= b ? a - b : a + P - b; }
inline uint32_t mul(uint32_t a, uint32_t b) { return (uint32_t)((uint64_t)a * b % P); }
inline uint32_t pw(uint32_t a, uint64_t e) {
    uint32_t r = 1;
    while (e) { if (e & 1) r = mul(r, a); a = mul(a, a); e >>= 1; }
    return r;
}
inline uint32_t inv(uint32_t a) { return pw(a, P - 2); }

struct S7 { uint32_t c[7]; };
S7 s_zero() { S7 r; memset(r.c, 0, sizeof r.c); return r; }
S7 s_base(uint32_t a) { S7 r = s_zero(); r.c[0] = a; return r; }
bool s_eq(const S7 &a, const S7 &b) { return !memcmp(a.c, b.c, sizeof a.c); }
S7 s_add(S7 a, const S7 &b) { for (int i = 0; i < 7; i++) a.c[i] = add(a.c[i], b.c[i]); return a; }
S7 s_sub(S7 a, const S7 &b) { for (int i = 0; i < 7; i++) a.c[i] = sub(a.c[i], b.c[i]); return a; }
S7 s_neg(S7 a) { for (int i = 0; i < 7; i++) a.c[i] = sub(0, a.c[i]); return a; }
S7 s_scale(S7 a, uint32_t k) { for (int i = 0; i < 7; i++) a.c[i] = mul(a.c[i], k); return a; }
S7 s_mul(const S7 &a, const S7 &b) {
    uint64_t t[13] = {0};
    for (int i = 0; i < 7; i++)
        for (int j = 0; j < 7; j++) t[i + j] = (t[i + j] + (uint64_t)a.c[i] * b.c[j]) % P;
    // z^7 = 8 - 2z
    for (int i = 12; i >= 7; i--) {
        t[i - 7] = (t[i - 7] + 8 * t[i]) % P;
        t[i - 6] = (t[i - 6] + (uint64_t)(P - 2) * t[i]) % P;
    }
    S7 r;
    for (int i = 0; i < 7; i++) r.c[i] = (uint32_t)t[i];
    return r;
}
S7 s_sq(const S7 &a) { return s_mul(a, a); }

// Frobenius x -> x^p is F_p-linear: column i of FROB is z^{i p}.  FROB2 is its square.
struct Frob {
    S7 col[7];
    S7 apply(const S7 &a) const {
        S7 r = s_zero();
        for (int i = 0; i < 7; i++) r = s_add(r, s_scale(col[i], a.c[i]));
        return r;
    }
};
S7 s_pow_big(S7 a, uint64_t e) {  // a^e for e < 2^64
    S7 r = s_base(1);
    while (e) { if (e & 1) r = s_mul(r, a); a = s_sq(a); e >>= 1; }
    return r;
}
struct Tables {
    Frob f1, f2, f3, f5;  // x^p, x^{p^2}, x^{p^3}, x^{p^5}
    Tables() {
        S7 z = s_zero();
        z.c[1] = 1;
        S7 zp = s_pow_big(z, P);  // z^p
        S7 acc = s_base(1);
        for (int i = 0; i < 7; i++) { f1.col[i] = acc; acc = s_mul(acc, zp); }
        for (int i = 0; i < 7; i++) f2.col[i] = f1.apply(f1.col[i]);
        for (int i = 0; i < 7; i++) f3.col[i] = f1.apply(f2.col[i]);
        for (int i = 0; i < 7; i++) f5.col[i] = f2.apply(f3.col[i]);
    }
};
const Tables &T() { static Tables t; return t; }

// x^{p + p^2 + ... + p^6} (so that x * it = N(x) in F_p)
S7 s_pow_r_1(const S7 &a) {
    const Tables &t = T();
    S7 b = s_mul(t.f1.apply(a), t.f2.apply(a));  // a^{p + p^2}
    S7 b2 = t.f2.apply(b), b4 = t.f2.apply(b2);  // a^{p^3 + p^4}, a^{p^5 + p^6}
    return s_mul(s_mul(b, b2), b4);
}
uint32_t s_norm(const S7 &a) { return s_mul(s_pow_r_1(a), a).c[0]; }
S7 s_inv(const S7 &a) { S7 r1 = s_pow_r_1(a); return s_scale(r1, inv(s_mul(r1, a).c[0])); }

// Tonelli-Shanks in F_p: p - 1 = 127 * 2^24, 3 generates F_p^* (a non-residue)
bool sqrt_p(uint32_t n, uint32_t &out) {
    if (n == 0) { out = 0; return true; }
    if (pw(n, (P - 1) / 2) != 1) return false;
    uint32_t M = 24, c = pw(3, 127), t = pw(n, 127), R = pw(n, 64);
    while (t != 1) {
        uint32_t i = 0, tt = t;
        while (tt != 1) { tt = mul(tt, tt); i++; }
        uint32_t b = c;
        for (uint32_t k = 0; k + i + 1 < M; k++) b = mul(b, b);
        M = i; c = mul(b, b); t = mul(t, c); R = mul(R, b);
    }
    out = R;
    return true;
}

// sqrt(a) = a * (a^{(p+1)/2})^{p + p^3 + p^5} * sqrt(N(a))^-1   (septic_extension.rs:626-674)
bool s_sqrt(const S7 &a, S7 &out) {
    S7 one = s_base(1);
    if (s_eq(a, s_zero()) || s_eq(a, one)) { out = a; return true; }
    uint32_t nrm = s_norm(a), r;
    if (!sqrt_p(inv(nrm), r)) return false;
    const Tables &t = T();
    S7 h = s_pow_big(a, ((uint64_t)P + 1) / 2);
    S7 d = s_mul(s_mul(t.f1.apply(h), t.f3.apply(h)), t.f5.apply(h));
    out = s_scale(s_mul(d, a), r);
    return true;
}

S7 curve_formula(const S7 &x) {  // x^3 + 3z x - 3
    S7 z3 = s_zero();
    z3.c[1] = 3;
    return s_sub(s_add(s_mul(s_sq(x), x), s_mul(x, z3)), s_base(3));
}

struct Pt { S7 x, y; bool inf; };
Pt add_incomplete(const Pt &a, const Pt &b) {
    S7 slope = s_mul(s_sub(b.y, a.y), s_inv(s_sub(b.x, a.x)));
    Pt r;
    r.x = s_sub(s_sub(s_sq(slope), a.x), b.x);
    r.y = s_sub(s_mul(slope, s_sub(a.x, r.x)), a.y);
    r.inf = false;
    return r;
}
Pt dbl(const Pt &a) {
    S7 z3 = s_zero();
    z3.c[1] = 3;
    S7 num = s_add(s_scale(s_sq(a.x), 3), z3);
    S7 slope = s_mul(num, s_inv(s_scale(a.y, 2)));
    Pt r;
    r.x = s_sub(s_sq(slope), s_scale(a.x, 2));
    r.y = s_sub(s_mul(slope, s_sub(a.x, r.x)), a.y);
    r.inf = false;
    return r;
}
Pt add_complete(const Pt &a, const Pt &b) {
    if (a.inf) return b;
    if (b.inf) return a;
    if (!s_eq(a.x, b.x)) return add_incomplete(a, b);
    if (s_eq(a.y, b.y)) return dbl(a);
    Pt r;
    r.x = s_zero(); r.y = s_zero(); r.inf = true;
    return r;
}

const uint32_t HALF = (P - 1) / 2;
bool is_send(const S7 &y) { return y.c[6] > HALF; }            // (p+1)/2 <= y6 <= p-1
bool is_exception(const S7 &y) { return y.c[6] == 0; }

}  // namespace

extern "C" {

// GlobalLookupOperation::get_digest for n messages (7 canonical words each): x = message with
// kind << 16 added to coefficient 0, lifted with the smallest offset; sends are negated.
// out_xy: n x 14 (x then y); out_offset: n.  Returns 0, or -1 if some x has no lift.
int zkm_septic_lift(const uint32_t *msg, const uint32_t *kind, const uint8_t *is_receive, uint64_t n,
                    uint32_t *out_xy, uint32_t *out_offset) {
    int bad = 0;
#pragma omp parallel for schedule(dynamic, 256) reduction(| : bad)
    for (uint64_t e = 0; e < n; e++) {
        S7 m;
        for (int i = 0; i < 7; i++) m.c[i] = msg[7 * e + i] % P;
        m.c[0] = add(m.c[0], (kind[e] << 16) % P);
        bool ok = false;
        for (uint32_t off = 0; off < 256 && !ok; off++) {
            S7 x = m;
            x.c[6] = add(mul(m.c[6], 256), off);
            S7 y;
            if (!s_sqrt(curve_formula(x), y) || is_exception(y)) continue;
            if (is_send(y)) y = s_neg(y);
            if (!is_receive[e]) y = s_neg(y);
            memcpy(out_xy + 14 * e, x.c, 28);
            memcpy(out_xy + 14 * e + 7, y.c, 28);
            out_offset[e] = off;
            ok = true;
        }
        if (!ok) bad = 1;
    }
    return bad ? -1 : 0;
}

// Inclusive running sums start + P_0 + ... + P_i with complete addition (global/mod.rs:126-166):
// out: (n + 1) x 15 = (x[7], y[7], is_infinity) with out[0] = start.
void zkm_septic_cumsum(const uint32_t *start14, const uint32_t *pts, uint64_t n, uint32_t *out) {
    Pt acc;
    memcpy(acc.x.c, start14, 28);
    memcpy(acc.y.c, start14 + 7, 28);
    acc.inf = false;
    auto put = [&](uint64_t i, const Pt &p) {
        memcpy(out + 15 * i, p.x.c, 28);
        memcpy(out + 15 * i + 7, p.y.c, 28);
        out[15 * i + 14] = p.inf ? 1u : 0u;
    };
    put(0, acc);
    for (uint64_t i = 0; i < n; i++) {
        Pt q;
        memcpy(q.x.c, pts + 14 * i, 28);
        memcpy(q.y.c, pts + 14 * i + 7, 28);
        q.inf = false;
        acc = add_complete(acc, q);
        put(i + 1, acc);
    }
}

// Septic helpers for tests and trace columns.
void zkm_septic_mul(const uint32_t *a, const uint32_t *b, uint32_t *out) {
    S7 x, y;
    memcpy(x.c, a, 28); memcpy(y.c, b, 28);
    S7 r = s_mul(x, y);
    memcpy(out, r.c, 28);
}
void zkm_septic_frobenius_col(int i, uint32_t *out) { memcpy(out, T().f1.col[i].c, 28); }
int zkm_septic_on_curve(const uint32_t *xy) {
    S7 x, y;
    memcpy(x.c, xy, 28); memcpy(y.c, xy + 7, 28);
    return s_eq(s_sq(y), curve_formula(x));
}
// SepticCurve::sum_checker_x(p1, p2, p3) = (x1 + x2 + x3)(x2 - x1)^2 - (y2 - y1)^2
void zkm_septic_sum_checker_x(const uint32_t *p1, const uint32_t *p2, const uint32_t *p3, uint32_t *out) {
    S7 x1, y1, x2, y2, x3;
    memcpy(x1.c, p1, 28); memcpy(y1.c, p1 + 7, 28); memcpy(x2.c, p2, 28); memcpy(y2.c, p2 + 7, 28);
    memcpy(x3.c, p3, 28);
    S7 r = s_sub(s_mul(s_add(s_add(x1, x2), x3), s_sq(s_sub(x2, x1))), s_sq(s_sub(y2, y1)));
    memcpy(out, r.c, 28);
}
// SepticDigest sum (septic_digest.rs:57-73): start + sum_i (d_i - zero) + zero - start
void zkm_septic_digest_sum(const uint32_t *digests, uint64_t n, const uint32_t *zero14, const uint32_t *start14,
                           uint32_t *out14) {
    Pt zero, start, acc;
    memcpy(zero.x.c, zero14, 28); memcpy(zero.y.c, zero14 + 7, 28); zero.inf = false;
    memcpy(start.x.c, start14, 28); memcpy(start.y.c, start14 + 7, 28); start.inf = false;
    Pt nzero = zero; nzero.y = s_neg(zero.y);
    Pt nstart = start; nstart.y = s_neg(start.y);
    acc = start;
    for (uint64_t i = 0; i < n; i++) {
        Pt d;
        memcpy(d.x.c, digests + 14 * i, 28); memcpy(d.y.c, digests + 14 * i + 7, 28); d.inf = false;
        acc = add_incomplete(add_incomplete(acc, d), nzero);
    }
    acc = add_incomplete(add_incomplete(acc, zero), nstart);
    memcpy(out14, acc.x.c, 28);
    memcpy(out14 + 7, acc.y.c, 28);
}

}  // extern "C"
