"""Machine description ("machine blob") for the MI355X shard prover.

The reference describes each chip by Rust code: `MachineAir::eval` for its own constraints and
`Chip::sends/receives` for its lookups (crates/stark/src/chip.rs:19-28, :65-90).  Across the
C ABI (include/zkm_hip.h) we describe the same information as plain data:

* AIR constraints as a postfix program (one EMIT per `assert_zero`), evaluated by the quotient
  kernel in the order the reference's `ProverConstraintFolder` would see them
  (crates/stark/src/folder.rs:79-102);
* lookups as `VirtualPairCol` linear combinations (crates/stark/src/lookup/lookup.rs:8-77),
  fingerprinted exactly as `populate_local_permutation_row` does (permutation.rs:29-69).

`log_quotient_degree` follows chip.rs:81-87: max constraint degree (selectors count 1), raised
to 3 when the chip has lookups, then log2_ceil(deg - 1).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

P = 0x7F000001
MAGIC = 0x4D4D4B5A
VERSION = 1

OP_END, OP_MAIN_L, OP_MAIN_N, OP_PREP_L, OP_PREP_N, OP_CONST, OP_PV = 0, 1, 2, 3, 4, 5, 6
OP_IS_FIRST, OP_IS_LAST, OP_IS_TRANS, OP_ADD, OP_SUB, OP_MUL, OP_NEG, OP_EMIT = 7, 8, 9, 10, 11, 12, 13, 14
# shared subexpressions (the Rc-shared nodes of Plonky3's SymbolicExpression DAG): LET s pops the top
# into value slot s, GET s pushes it.  A chip's program starts with its shared definitions (each
# evaluated once per row, in creation order, which is a topological order), then its constraints.
OP_LET, OP_GET = 15, 16
# builder-only opcode (never in a blob): a reference to shared definition `gid` of _SHARED
OP_REF = 0x10000
_OPERAND_OPS = frozenset((OP_MAIN_L, OP_MAIN_N, OP_PREP_L, OP_PREP_N, OP_CONST, OP_PV, OP_LET, OP_GET, OP_REF))
_SHARED: List[List[int]] = []  # gid -> code of the shared definition (builder registry)


def _refs(code: List[int]):
    """gids of the shared definitions `code` references directly."""
    i, n = 0, len(code)
    while i < n:
        op = code[i]
        if op == OP_REF:
            yield code[i + 1]
        i += 2 if op in _OPERAND_OPS else 1

SCOPE_GLOBAL_ENUM = 1  # commit_scope encoding in the blob: 0 = Local, 1 = Global
LOOKUP_LOCAL, LOOKUP_GLOBAL = 0, 1

# LookupKind discriminants, crates/stark/src/lookup/lookup.rs:23-44
KIND_MEMORY, KIND_PROGRAM, KIND_INSTRUCTION, KIND_BYTE, KIND_RANGE, KIND_SYSCALL, KIND_GLOBAL = range(1, 8)


class Expr:
    """Postfix expression over one row pair of a chip (base field)."""

    __slots__ = ("code", "deg")

    def __init__(self, code: List[int], deg: int):
        self.code = code
        self.deg = deg

    @staticmethod
    def lift(x) -> "Expr":
        if isinstance(x, Expr):
            return x
        return Expr([OP_CONST, int(x) % P], 0)

    def __add__(self, o):
        o = Expr.lift(o)
        return Expr(self.code + o.code + [OP_ADD], max(self.deg, o.deg))

    __radd__ = lambda self, o: Expr.lift(o) + self

    def __sub__(self, o):
        o = Expr.lift(o)
        return Expr(self.code + o.code + [OP_SUB], max(self.deg, o.deg))

    def __rsub__(self, o):
        return Expr.lift(o) - self

    def __mul__(self, o):
        o = Expr.lift(o)
        return Expr(self.code + o.code + [OP_MUL], self.deg + o.deg)

    __rmul__ = lambda self, o: Expr.lift(o) * self

    def __neg__(self):
        return Expr(self.code + [OP_NEG], self.deg)

    def share(self) -> "Expr":
        """This expression as a shared node: every use reads one value per row (OP_GET) instead of
        repeating its code, as Plonky3 shares Rc'd SymbolicExpression nodes.  Columns and constants are
        returned as they are (re-reading them is as cheap as a slot)."""
        if len(self.code) <= 2:
            return self
        _SHARED.append(self.code)
        return Expr([OP_REF, len(_SHARED) - 1], self.deg)


def main(c: int) -> Expr:
    return Expr([OP_MAIN_L, c], 1)


def main_next(c: int) -> Expr:
    return Expr([OP_MAIN_N, c], 1)


def prep(c: int) -> Expr:
    return Expr([OP_PREP_L, c], 1)


def prep_next(c: int) -> Expr:
    return Expr([OP_PREP_N, c], 1)


def pv(i: int) -> Expr:
    return Expr([OP_PV, i], 0)


IS_FIRST = Expr([OP_IS_FIRST], 1)
IS_LAST = Expr([OP_IS_LAST], 1)
# Plonky3 SymbolicExpression::degree_multiple: IsFirstRow / IsLastRow count 1, IsTransition 0 (the
# reference's CpuChip has when_transition().when(next).when_not(next) constraints of degree 3 under
# its blowup-2 config, which only holds with a degree-0 transition selector)
IS_TRANSITION = Expr([OP_IS_TRANS], 0)


@dataclass
class VirtualPairCol:
    """constant + sum(weight * column); column = ("main"|"prep", index)."""

    terms: List[Tuple[str, int, int]] = field(default_factory=list)
    constant: int = 0

    @staticmethod
    def single_main(c: int) -> "VirtualPairCol":
        return VirtualPairCol([("main", c, 1)], 0)

    @staticmethod
    def single_prep(c: int) -> "VirtualPairCol":
        return VirtualPairCol([("prep", c, 1)], 0)

    @staticmethod
    def const(v: int) -> "VirtualPairCol":
        return VirtualPairCol([], v % P)

    def words(self) -> List[int]:
        w = [len(self.terms)]
        for kind, idx, weight in self.terms:
            w += [(0x80000000 | idx) if kind == "main" else idx, weight % P]
        return w + [self.constant % P]


@dataclass
class Lookup:
    values: List[VirtualPairCol]
    multiplicity: VirtualPairCol
    kind: int
    scope: int = LOOKUP_LOCAL

    def words(self) -> List[int]:
        w = [self.kind, self.scope, len(self.values)]
        for v in self.values:
            w += v.words()
        return w + self.multiplicity.words()


@dataclass
class ChipDesc:
    name: str
    prep_width: int
    main_width: int
    commit_scope: int = 0
    local_only: bool = False
    constraints: List[Expr] = field(default_factory=list)
    sends: List[Lookup] = field(default_factory=list)
    receives: List[Lookup] = field(default_factory=list)

    def assert_zero(self, e: Expr):
        self.constraints.append(Expr.lift(e))

    @property
    def max_constraint_degree(self) -> int:
        d = max([c.deg for c in self.constraints], default=0)
        if self.sends or self.receives:
            d = max(d, 3)
        return d

    @property
    def log_quotient_degree(self) -> int:
        d = self.max_constraint_degree - 1
        return 0 if d <= 1 else math.ceil(math.log2(d))

    @property
    def num_local_lookups(self) -> int:
        return sum(1 for l in self.sends + self.receives if l.scope == LOOKUP_LOCAL)

    @property
    def perm_width_ef(self) -> int:
        n = self.num_local_lookups
        b = 1 << self.log_quotient_degree
        return 0 if n == 0 else (n + b - 1) // b + 1

    @property
    def num_constraints(self) -> int:
        c = len(self.constraints)
        if self.num_local_lookups:
            c += self.perm_width_ef - 1 + 3
        if self.commit_scope == 1:
            c += 14
        return c

    def program(self) -> List[int]:
        """The chip's postfix program: its shared definitions (LET), then one EMIT per constraint."""
        need, stack = set(), []
        for c in self.constraints:
            stack.extend(_refs(c.code))
        while stack:
            g = stack.pop()
            if g not in need:
                need.add(g)
                stack.extend(_refs(_SHARED[g]))
        slot = {g: k for k, g in enumerate(sorted(need))}

        def lower(code):
            out, i, n = [], 0, len(code)
            while i < n:
                op = code[i]
                if op == OP_REF:
                    out += [OP_GET, slot[code[i + 1]]]
                    i += 2
                elif op in _OPERAND_OPS:
                    out += code[i:i + 2]
                    i += 2
                else:
                    out.append(op)
                    i += 1
            return out
        prog: List[int] = []
        for g in sorted(need):
            prog += lower(_SHARED[g]) + [OP_LET, slot[g]]
        for c in self.constraints:
            prog += lower(c.code) + [OP_EMIT]
        return prog

    def words(self) -> List[int]:
        nb = self.name.encode()
        w = [len(nb)]
        padded = nb + b"\0" * (-len(nb) % 4)
        w += [int.from_bytes(padded[i:i + 4], "little") for i in range(0, len(padded), 4)]
        code = self.program()
        w += [self.prep_width, self.main_width, self.commit_scope, int(self.local_only),
              self.log_quotient_degree, len(self.constraints), len(code)] + code
        w += [len(self.sends), len(self.receives)]
        for l in self.sends + self.receives:
            w += l.words()
        return w


@dataclass
class MachineDesc:
    chips: List[ChipDesc]
    num_pv: int
    # MachineProgram::pc_start of the programs it proves, observed by every shard's transcript and hashed into the
    # vk: the MIPS program's entry (crates/core/executor/src/program.rs:329), 0 for recursion programs
    # (crates/recursion/core/src/runtime/program.rs:20-22)
    pc_start: int = 0x00400000

    def blob(self):
        import numpy as np
        w = [MAGIC, VERSION, self.num_pv, len(self.chips)]
        for c in self.chips:
            w += c.words()
        return np.asarray(w, dtype=np.uint32)

    def chip_index(self, name: str) -> int:
        for i, c in enumerate(self.chips):
            if c.name == name:
                return i
        raise KeyError(name)
