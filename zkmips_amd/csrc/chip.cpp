// Machine blob parser and device flattening (format: include/zkm_hip.h).
#include "chip.hpp"

#include <algorithm>

namespace zkm {

namespace {
struct Rd {
    const uint32_t *w;
    size_t n, p = 0;
    uint32_t get() {
        ARG_CHECK(p < n, "machine blob truncated");
        return w[p++];
    }
};
VPC read_vpc(Rd &r) {
    VPC v;
    uint32_t nt = r.get();
    ARG_CHECK(nt < 4096, "VPC too long");
    for (uint32_t i = 0; i < nt; i++) {
        v.cols.push_back(r.get());
        v.weights.push_back(r.get() % kb::P);
    }
    v.constant = r.get() % kb::P;
    return v;
}
}  // namespace

Machine parse_machine(const uint32_t *w, size_t n) {
    Rd r{w, n};
    ARG_CHECK(r.get() == 0x4D4D4B5Au, "bad machine magic");
    ARG_CHECK(r.get() == 1u, "unsupported machine blob version");
    Machine m;
    m.num_pv = (int)r.get();
    uint32_t nchips = r.get();
    ARG_CHECK(nchips < 1024, "too many chips");
    for (uint32_t ci = 0; ci < nchips; ci++) {
        ChipDesc c;
        uint32_t nl = r.get();
        ARG_CHECK(nl < 256, "chip name too long");
        std::string name;
        for (uint32_t i = 0; i < (nl + 3) / 4; i++) {
            uint32_t x = r.get();
            for (int b = 0; b < 4 && 4 * i + b < nl; b++) name.push_back((char)((x >> (8 * b)) & 0xff));
        }
        c.name = name;
        c.prep_w = (int)r.get();
        c.main_w = (int)r.get();
        c.scope = (int)r.get();
        c.local_only = (int)r.get();
        c.log_qd = (int)r.get();
        c.n_main = (int)r.get();
        uint32_t cl = r.get();
        for (uint32_t i = 0; i < cl; i++) c.code.push_back(r.get());
        // validate program and its stack depth
        int sp = 0, emits = 0;
        for (size_t pc = 0; pc < c.code.size();) {
            uint32_t op = c.code[pc++];
            switch (op) {
            case OP_MAIN_L: case OP_MAIN_N:
                ARG_CHECK(pc < c.code.size() && (int)c.code[pc] < c.main_w, "MAIN column out of range");
                pc++; sp++; break;
            case OP_PREP_L: case OP_PREP_N:
                ARG_CHECK(pc < c.code.size() && (int)c.code[pc] < c.prep_w, "PREP column out of range");
                pc++; sp++; break;
            case OP_CONST: ARG_CHECK(pc < c.code.size(), "CONST operand"); c.code[pc] %= kb::P; pc++; sp++; break;
            case OP_PV: ARG_CHECK(pc < c.code.size(), "PV operand"); pc++; sp++; break;
            case OP_IS_FIRST: case OP_IS_LAST: case OP_IS_TRANS: sp++; break;
            case OP_ADD: case OP_SUB: case OP_MUL: ARG_CHECK(sp >= 2, "stack underflow"); sp--; break;
            case OP_NEG: ARG_CHECK(sp >= 1, "stack underflow"); break;
            case OP_EMIT: ARG_CHECK(sp >= 1, "stack underflow"); sp--; emits++; break;
            case OP_LET:
                ARG_CHECK(pc < c.code.size() && sp >= 1, "LET operand / stack underflow");
                ARG_CHECK(c.code[pc] == (uint32_t)c.n_slots, "LET slots must be defined in order 0, 1, 2, ...");
                c.n_slots++; pc++; sp--; break;
            case OP_GET:
                ARG_CHECK(pc < c.code.size() && (int)c.code[pc] < c.n_slots, "GET of an undefined slot");
                pc++; sp++; break;
            default: ARG_CHECK(false, "bad opcode");
            }
            c.max_stack = std::max(c.max_stack, sp);
        }
        ARG_CHECK(emits == c.n_main, "EMIT count != num_main_constraints");
        ARG_CHECK(c.max_stack <= 24, "constraint program stack deeper than 24");
        uint32_t ns = r.get(), nr = r.get();
        for (uint32_t i = 0; i < ns + nr; i++) {
            LookupDesc l;
            l.kind = r.get();
            l.scope = r.get();
            uint32_t nv = r.get();
            ARG_CHECK(nv < 256, "lookup arity");
            for (uint32_t v = 0; v < nv; v++) l.values.push_back(read_vpc(r));
            l.mult = read_vpc(r);
            l.is_send = i < ns;
            for (auto *vp : {&l.mult}) for (uint32_t col : vp->cols) (void)col;
            // scoped_lookups (permutation.rs:73-98): keep Local, stable order
            if (l.scope == 0) c.local.push_back(std::move(l));
        }
        for (auto &l : c.local)
            for (const VPC *v : [&] { std::vector<const VPC *> a; for (auto &x : l.values) a.push_back(&x); a.push_back(&l.mult); return a; }())
                for (uint32_t col : v->cols) {
                    if (col & 0x80000000u) ARG_CHECK((int)(col & 0x7fffffffu) < c.main_w, "lookup main column");
                    else ARG_CHECK((int)col < c.prep_w, "lookup prep column");
                }
        const int batch = 1 << c.log_qd;
        const int nloc = (int)c.local.size();
        c.perm_w = nloc ? (nloc + batch - 1) / batch + 1 : 0;
        int pc_ = 0;
        if (nloc) pc_ += c.perm_w - 1 + 3;
        if (c.scope == 1) pc_ += 14;
        c.n_constraints = c.n_main + pc_;
        ARG_CHECK(c.scope != 1 || c.main_w >= 14, "global chip needs 14 digest columns");
        m.chips.push_back(std::move(c));
    }
    return m;
}

std::vector<uint32_t> flatten_chip(const ChipDesc &c) {
    std::vector<uint32_t> out(4, 0);
    out[0] = (uint32_t)c.code.size();
    out[1] = 4;
    for (size_t pc = 0; pc < c.code.size();) {
        uint32_t op = c.code[pc++];
        out.push_back(op);
        if (op == OP_CONST) out.push_back(kb::to_mont(c.code[pc++]));
        else if (op == OP_MAIN_L || op == OP_MAIN_N || op == OP_PREP_L || op == OP_PREP_N || op == OP_PV ||
                 op == OP_LET || op == OP_GET)
            out.push_back(c.code[pc++]);
    }
    out[0] = (uint32_t)(out.size() - 4);
    out[2] = (uint32_t)c.local.size();
    out[3] = (uint32_t)out.size();
    size_t table = out.size();
    out.resize(table + 4 * c.local.size());
    auto push_vpc = [&](const VPC &v) {
        out.push_back((uint32_t)v.cols.size());
        for (size_t i = 0; i < v.cols.size(); i++) {
            out.push_back(v.cols[i]);
            out.push_back(kb::to_mont(v.weights[i]));
        }
        out.push_back(kb::to_mont(v.constant));
    };
    for (size_t i = 0; i < c.local.size(); i++) {
        const LookupDesc &l = c.local[i];
        out[table + 4 * i + 0] = kb::to_mont(l.kind);
        out[table + 4 * i + 1] = l.is_send ? 1u : 0u;
        out[table + 4 * i + 2] = (uint32_t)l.values.size();
        out[table + 4 * i + 3] = (uint32_t)out.size();
        for (auto &v : l.values) push_vpc(v);
        push_vpc(l.mult);
    }
    return out;
}

}  // namespace zkm
