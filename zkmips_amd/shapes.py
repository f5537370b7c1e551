"""MIPS core shards padded to a reference shard shape (crates/core/machine/src/shape/maximal_shapes.json).

With shapes enabled the reference pads every chip of a shard to the log height its shape fixes
(`fixed_log2_rows` -> `next_power_of_two(n, Some(log))`, crates/core/machine/src/utils/mod.rs:87-110), so
a shard's proving cost is set by the shape, not by how full the chips are.  `shape_program` generates a
counted loop whose instruction mix stays inside a given shape; `shape_shard` runs it and pads each chip's
trace to the shape with the chip's own padding row (absent chips of the shape as all-padding traces).
Heights below 16 rows are raised to 16, this framework's minimum trace height.
"""
from __future__ import annotations

import numpy as np

from . import mips_alu as A
from . import mips_core as C
from . import mips_syscall as SY
from .workloads import splitmix64

MIN_LOG = 4
# instruction kinds and the chips their events land in (with the executor's dependency events)
_KINDS = ("add", "bit", "lt", "sll", "sr", "mem", "branch", "movcond")


def _fractions(shape: dict) -> dict:
    """Per-instruction-kind share of the loop body that keeps every chip below its shape height with the
    CPU running ~80% of 2^Cpu rows (the 24-bit clk bound: at most 2^24 / 5 instructions per shard)."""
    cpu = shape["Cpu"]
    cap = lambda chip: 2.0 ** (shape.get(chip, 0) - cpu) if chip in shape else 0.0
    f = {"mem": 0.7 * cap("MemoryInstrs"), "bit": 0.8 * cap("Bitwise"), "sll": 0.8 * cap("ShiftLeft"),
         "sr": 0.8 * cap("ShiftRight"), "movcond": 0.7 * cap("MovCond")}
    # each branch sends two Lt events (and an AddSub when taken); memory ops send an AddSub each
    f["branch"] = min(0.6 * cap("Branch"), 0.3 * cap("Lt"))
    f["lt"] = max(0.0, 0.8 * cap("Lt") - 2 * f["branch"])
    used = sum(f.values())
    f["add"] = max(0.0, min(0.8 * cap("AddSub") - f["mem"] - f["branch"], 1.0 - used))
    tot = sum(f.values())
    return {k: v / tot for k, v in f.items()} if tot > 1 else f


_OPS = {"add": [(A.OP_ADD, 0), (A.OP_ADD, 1), (A.OP_SUB, 0)],
        "bit": [(A.OP_AND, 0), (A.OP_OR, 1), (A.OP_XOR, 0), (A.OP_NOR, 0), (A.OP_AND, 1)],
        "lt": [(A.OP_SLT, 0), (A.OP_SLTU, 0), (A.OP_SLT, 1)],
        "sll": [(A.OP_SLL, 1), (A.OP_SLL, 0)],
        "sr": [(A.OP_SRL, 1), (A.OP_SRA, 1), (A.OP_SRL, 0)],
        "movcond": [(C.OP_MEQ, 0), (C.OP_MNE, 0)]}
_AVOID = (C.COUNTER,)


def shape_program(shape: dict, seed: int = 1, body: int = 512, fill: float = 0.8, rows: int = None):
    """A counted loop (`r3` counts down) whose body mixes ALU, memory, forward-branch and conditional-move
    instructions in the proportions `_fractions(shape)`; iterations sized to `fill` of the shape's Cpu
    rows (capped by the 24-bit clk), or to `rows` instructions in all (an execution of several shards)."""
    frac = _fractions(shape)
    kinds = list(frac)
    p = np.asarray([frac[k] for k in kinds])
    r = splitmix64(0x5AA9E00 + seed, 8 * body + 64)
    pick = (r[:body] % np.uint64(1 << 30)).astype(np.float64) / (1 << 30)
    cum = np.cumsum(p / p.sum())
    regs = [x for x in range(1, 32) if x not in _AVOID]
    prog = [(A.OP_ADD, C.COUNTER, 0, 0, 0, 1)]  # iterations patched below
    k = 0
    while k < body:
        kind = kinds[min(int(np.searchsorted(cum, pick[k])), len(kinds) - 1)]
        w = r[8 * k + 64:8 * k + 72]
        ra = regs[int(w[1] % len(regs))]
        rb, rc = int(w[2] % 32), int(w[3] % 32)
        if kind == "branch" and k + 2 < body:  # forward over its delay slot and 0..1 instructions
            op = C.BRANCH_OPS[int(w[0] % 6)]
            skip = int(w[4] % 2)
            if op in (C.OP_BEQ, C.OP_BNE):
                prog.append((op, rb, rc, 4 * (skip + 1), 0, 1))
            else:
                prog.append((op, rb, 0, 4 * (skip + 1), 1, 1))
            prog.append((A.OP_ADD, ra, rb, int(w[5] & np.uint64(0xFFFF)), 0, 1))  # delay slot
            k += 2
            continue
        if kind == "mem":
            op = (C.OP_LW, C.OP_SW, C.OP_LBU, C.OP_SB, C.OP_LH, C.OP_SH)[int(w[0] % 6)]
            off = 4 * int(w[4] % 4096) + (0 if op in (C.OP_LW, C.OP_SW) else int(w[5] % 2) * 2)
            prog.append((op, ra if op not in C.STORE_OPS else rb, 0, C.DATA_BASE + off, 0, 1))
        elif kind in ("branch", "add"):
            op, imm = _OPS["add"][int(w[0] % 3)]
            prog.append((op, ra, rb, int(w[4] & np.uint64(0xFFFFFFFF)) if imm else rc, 0, imm))
        else:
            op, imm = _OPS[kind][int(w[0] % len(_OPS[kind]))]
            c = int(w[4] % 32) if imm and kind in ("sll", "sr") else (int(w[4] & np.uint64(0xFFFFFFFF)) if imm else rc)
            prog.append((op, ra, rb, c, 0, imm))
        k += 1
    prog.append((A.OP_ADD, C.COUNTER, C.COUNTER, C.M32, 0, 1))
    back = (1 - (len(prog) + 1)) * 4
    prog.append((C.OP_BNE, C.COUNTER, 0, back & C.M32, 0, 1))
    prog.append((A.OP_ADD, 0, 0, 0, 0, 1))  # delay slot
    prog += [(A.OP_ADD, SY.REG_V0, 0, SY.HALT, 0, 1), (A.OP_ADD, SY.REG_A0, 0, 0, 0, 1),
             (SY.OP_SYSCALL, SY.REG_V0, SY.REG_A0, SY.REG_A1, 0, 0)]
    if rows is None:
        rows = min(int(fill * (1 << shape["Cpu"])), (1 << 24) // 5 - 64)
    per_iter = len(prog) - 4  # the body's untaken-branch path, roughly
    iters = max(1, rows // per_iter - 1)
    prog[0] = (A.OP_ADD, C.COUNTER, 0, iters, 0, 1)
    return prog


def scaled(shape: dict, down: int) -> dict:
    """The shape with every log height lowered by `down` (not below MIN_LOG)."""
    return {k: max(MIN_LOG, v - down) for k, v in shape.items()}


def pad_to_shape(machine, traces: dict, shape: dict) -> dict:
    """Each chip of `shape` padded to 2^max(log, MIN_LOG) rows with its padding row (its trace's last row,
    which every builder leaves as padding); chips of the shape with no events get an all-padding trace."""
    out = dict(traces)
    widths = {c.name: c.main_width for c in machine.chips}
    for name, log in shape.items():
        h = 1 << max(MIN_LOG, log)
        t = out.get(name)
        if t is None:
            out[name] = np.zeros((h, widths[name]), np.uint32)
            continue
        if len(t) > h:
            raise ValueError(f"{name}: {len(t)} rows do not fit the shape's 2^{log}")
        if len(t) < h:
            out[name] = np.concatenate([t, np.repeat(t[-1:], h - len(t), axis=0)])
    return out


def shape_shard(shape: dict, seed: int = 1, down: int = 0, fill: float = 0.8, capture: dict = None):
    """(machine, prep_traces, traces, public_values) of one CPU shard padded to `shape` scaled down by
    2^down.  The execution halts in the shard (HALT), so its MemoryLocal/Global close the shard's
    accesses like any continuation shard.  `capture` receives the executor's records (program_shard)."""
    sh = scaled(shape, down)
    prog = shape_program(sh, seed, fill=fill)
    m, prep, traces, pvs = C.program_shard(prog, seed, 1, (1 << 24) // 5 - 1, capture=capture)
    for name, t in traces.items():
        if name not in sh and name not in ("Program", "Byte"):
            raise ValueError(f"{name} ({len(t)} rows) is not in the shape")
    return m, prep, pad_to_shape(m, traces, sh), pvs


def shape_execution(shape: dict, cpu_shards: int, down: int = 0, seed: int = 1, fill: float = 0.8):
    """One execution of a shape_program loop cut into `cpu_shards` consecutive CPU shards (continuations,
    mips_core.program_shards: registers, memory and access records carry over; each shard about `fill` of
    the scaled shape's Cpu rows) each padded to the scaled `shape`, then the memory shard that closes the
    execution -- the leaves the reference's recursion chains (consecutive shard numbers and pcs, one proving
    key, global sums adding to zero).  Returns the list of (machine, prep_traces, traces, public_values)."""
    sh = scaled(shape, down)
    per = min(int(fill * (1 << sh["Cpu"])), (1 << 24) // 5 - 64)
    prog = shape_program(sh, seed, fill=fill, rows=per)
    # the loop's executed instructions per iteration (branches skip part of the body), measured on two short
    # runs, set the iteration count: the last CPU shard about half full
    def steps(iters):
        q = list(prog)
        q[0] = (A.OP_ADD, C.COUNTER, 0, iters, 0, 1)
        return len(C._execute(q, C.initial_registers(seed), 1, 1 << 30)[0])
    s2, s3 = steps(2), steps(3)
    per_iter, fixed = s3 - s2, s2 - 2 * (s3 - s2)
    iters = max(1, (per * cpu_shards - per // 2 - fixed) // per_iter)
    prog[0] = (A.OP_ADD, C.COUNTER, 0, iters, 0, 1)
    out = C.program_shards(prog, seed, shard_size=per)
    if sum("Cpu" in t for _, _, t, _ in out) != cpu_shards:
        raise AssertionError("shape_execution: CPU shard count")
    # one shape for every CPU shard (one recursion program structure): the scaled shape, raised where a small
    # scale's fixed per-shard records (the register entries of MemoryLocal, ...) need more rows
    common = dict(sh)
    for m, prep, traces, pvs in out:
        if "Cpu" in traces:
            for name, t in traces.items():
                if name not in sh and name not in ("Program", "Byte"):
                    raise ValueError(f"{name} ({len(t)} rows) is not in the shape")
                if name in common:
                    common[name] = max(common[name], (len(t) - 1).bit_length())
    res = []
    for m, prep, traces, pvs in out:
        if "Cpu" in traces:
            traces = pad_to_shape(m, traces, common)
        res.append((m, prep, traces, pvs))
    return res


def shape_shards(shape: dict, seeds, down: int = 0, fill: float = 0.8):
    """Several CPU shards of ONE program (one proving key, as the shards of one ELF's executions share it)
    padded to `shape`: the program of shape_shard(seeds[0]) run from the initial registers of each seed, so
    the traces differ while the preprocessed Program table is the same."""
    sh = scaled(shape, down)
    prog = shape_program(sh, seeds[0], fill=fill)
    out = []
    for s in seeds:
        m, prep, traces, pvs = C.program_shard(prog, s, 1, (1 << 24) // 5 - 1)
        out.append((m, prep, pad_to_shape(m, traces, sh), pvs))
    return out


# maximal_shapes.json["22"][2] (crates/core/machine/src/shape/maximal_shapes.json; tests/golden pins it):
# Cpu 22 / AddSub 21 / Lt, MemoryInstrs, Bitwise 20 / Branch, ShiftRight 19 / ShiftLeft 18 / Global 17 /
# MemoryLocal, MovCond 14 / Jump 6 / Mul, SyscallInstrs, SyscallCore 1
MAXIMAL_22 = {"Cpu": 22, "MemoryLocal": 14, "MovCond": 14, "Lt": 20, "MemoryInstrs": 20, "SyscallInstrs": 1,
              "ShiftLeft": 18, "Bitwise": 20, "ShiftRight": 19, "Mul": 1, "Global": 17, "Branch": 19, "Jump": 6,
              "AddSub": 21, "SyscallCore": 1}
