"""MIPS core shard: the reference's Cpu, Program, Branch, Jump, Mul, DivRem, MovCond, MemoryInstrs and
MiscInstrs chips (zkmips_amd/mips_core.py) on top of the ALU slice, with the memory argument closed by the
MemoryLocal and Global chips (zkmips_amd/mips_memory.py).  The reference's own instruction-test programs are fixtures.

CPU part: the trace satisfies every constraint and every lookup balances (direct evaluation,
tests/_air_check.py); the oracle proves it and its verifier accepts; forged ALU results, register
values, timestamps, pcs, program rows and branch decisions are rejected.  Programs are straight-line
code and counted loops with forward branches of all six kinds (delay slots as the executor runs them).
GPU part: the HIP prover's proofs are byte-identical to the oracle's, and shards whose Cpu chip has
2^22 rows (the §8 "Cpu-shaped chip" at the bench height) verify."""
import numpy as np
import pytest

from tests import _air_check
from tests import _oracle as O
from zkmips_amd import mips_alu as A
from zkmips_amd import mips_core as C
from zkmips_amd import mips_memory as MM


@pytest.fixture(scope="module")
def shard():
    return C.core_shard(700, seed=4)


@pytest.fixture(scope="module")
def oracle(shard):
    m, prep, _, _ = shard
    return O.OracleProver(m, prep, num_queries=16)


def test_core_chip_shapes(shard):
    m, prep, tr, pv = shard
    cpu = m.chips[m.chip_index("Cpu")]
    # cpu/columns/mod.rs: 67 main columns; 21 local lookups -> 11 EF permutation columns (§8 "Cpu-shaped")
    assert cpu.main_width == 67 and cpu.perm_width_ef == 11 and cpu.log_quotient_degree == 1
    assert tr["Cpu"].shape == (1024, 67) and prep["Program"].shape == (1024, 14)
    assert tr["Program"][:700].all() and not tr["Program"][700:].any()
    assert tr["Cpu"][699, C.C_REAL] == 1 and tr["Cpu"][700, C.C_REAL] == 0


@pytest.mark.parametrize("n,seed", [(1, 2), (17, 3), (700, 4), (5000, 5)])
def test_core_trace_satisfies_air(n, seed):
    bad, unbalanced = _air_check.check(*C.core_shard(n, seed=seed))
    assert bad == [] and unbalanced == []


def test_core_shard_proves_and_verifies(shard, oracle):
    _, _, tr, pv = shard
    rc, proof = oracle.prove(tr, pv)
    assert rc == 0 and oracle.verify(proof) == 0


def _tamper(tr, what):
    bad = {k: v.copy() for k, v in tr.items()}
    t = bad["Cpu"]
    if what == "alu_result":  # the CPU claims a result the ALU chips never produced
        t[10, C.C_A_VAL] = (int(t[10, C.C_A_VAL]) + 1) % 256
    elif what == "register_read":  # a forged register value read by op_b
        t[20, C.C_B_ACC + C.ACC_VALUE] ^= 1
    elif what == "timestamp":  # an access whose previous timestamp is after the current one
        t[30, C.C_B_ACC + C.ACC_PREV_CLK] += 7
    elif what == "pc":
        t[40, C.C_NPC] += 4
    elif what == "program":  # the executed instruction is not the committed program's
        t[50, C.C_OPC] = (int(t[50, C.C_OPC]) + 1) % 256
    elif what == "register_final":  # the value MemoryLocal says a register holds at the shard's end
        bad["MemoryLocal"][0, MM.ML_ENTRY_WIDTH + MM.ML_FVAL] ^= 1
    elif what == "clk":
        t[60, C.C_CLK16] += 1
    return bad


@pytest.mark.parametrize("what", ["alu_result", "register_read", "timestamp", "pc", "program", "register_final",
                                  "clk"])
def test_core_tamper_rejected(shard, oracle, what):
    m, prep, tr, pv = shard
    bad = _tamper(tr, what)
    assert _air_check.check(m, prep, bad, pv) != ([], [])
    rc, proof = oracle.prove(bad, pv)
    assert rc == 0
    assert oracle.verify(proof) != 0


def _branch_kinds_program():
    """Every branch kind on a positive, a negative and a zero operand (BEQ/BNE on equal and unequal
    registers), each followed by its delay slot and one instruction it skips when taken."""
    prog = [(A.OP_ADD, 1, 0, 5, 0, 1), (A.OP_ADD, 2, 0, C.M32 - 4, 0, 1), (A.OP_ADD, 6, 0, 5, 0, 1)]
    for op in C.BRANCH_OPS:
        for rs, rt in ((1, 6), (2, 1), (0, 0)):
            if op in (C.OP_BEQ, C.OP_BNE):
                prog.append((op, rs, rt, 8, 0, 1))  # target = next_pc + 8
            else:
                prog.append((op, rs, 0, 8, 1, 1))
            prog.append((A.OP_ADD, 4, 4, 1, 0, 1))  # delay slot: always runs
            prog.append((A.OP_ADD, 5, 5, 1, 0, 1))  # skipped when taken
    # offset 0 targets the delay slot itself: it runs twice, the first time with next_pc == pc
    prog += [(C.OP_BEQ, 0, 0, 0, 0, 1), (A.OP_ADD, 7, 7, 3, 0, 1)]
    return prog


def test_branch_kinds():
    prog = _branch_kinds_program()
    m, prep, tr, pv = C.program_shard(prog, seed=2)
    br = tr["Branch"]
    assert br.shape == (32, C.BR_WIDTH)
    taken = list(br[:18, C.BR_BRANCHING])
    # (5, 5), (-5, 5), (0, 0) per kind in BRANCH_OPS order: BEQ, BGEZ, BGTZ, BLEZ, BLTZ, BNE
    assert taken == [1, 0, 1,  1, 0, 1,  1, 0, 0,  0, 1, 1,  0, 1, 0,  0, 1, 0]
    assert list(br[:18, C.BR_LT]) == [0, 1, 0] * 6 and list(br[:18, C.BR_GT]) == [0, 0, 0] + [1, 0, 0] * 4 + [0, 0, 0]
    cpu = tr["Cpu"]
    n = int(cpu[:, C.C_REAL].sum())
    assert n == 3 + 18 * 3 - sum(taken) + 3
    assert br[18, C.BR_BRANCHING] == 1 and list(cpu[n - 2:n, C.C_PC]) == [cpu[n - 3, C.C_PC] + 4] * 2
    assert _air_check.check(m, prep, tr, pv) == ([], [])
    o = O.OracleProver(m, prep, num_queries=8)
    rc, proof = o.prove(tr, pv)
    assert rc == 0 and o.verify(proof) == 0


def test_jump_kinds():
    """j, jal, jr, jalr and bal (the executor's Jumpi / Jump / JumpDirect), each with its delay slot."""
    S = C.PC_BASE + 4 * 12
    prog = [(A.OP_ADD, 30, 0, S, 0, 1),                    # 0: r30 = S
            (C.OP_JUMPI, 31, S, 0, 1, 1),                  # 1: jal S
            (A.OP_ADD, 4, 4, 1, 0, 1),                     # 2: delay slot
            (C.OP_JUMP, 31, 30, 0, 0, 1),                  # 3: jalr r31, r30
            (A.OP_ADD, 4, 4, 1, 0, 1),                     # 4: delay slot
            (C.OP_JUMPDIRECT, 31, 8, 0, 1, 1),             # 5: bal +8 (skips 7)
            (A.OP_ADD, 4, 4, 1, 0, 1),                     # 6: delay slot
            (A.OP_ADD, 5, 5, 1, 0, 1),                     # 7: skipped
            (C.OP_JUMPI, 0, C.PC_BASE + 4 * 16, 0, 1, 1),  # 8: j END
            (A.OP_ADD, 4, 4, 1, 0, 1),                     # 9: delay slot
            (A.OP_ADD, 5, 5, 1, 0, 1),                     # 10: skipped
            (A.OP_ADD, 5, 5, 1, 0, 1),                     # 11: skipped
            (A.OP_ADD, 6, 6, 7, 0, 1),                     # 12: S
            (C.OP_JUMP, 0, 31, 0, 0, 1),                   # 13: jr r31
            (A.OP_ADD, 6, 6, 1, 0, 1),                     # 14: delay slot
            (A.OP_ADD, 5, 5, 1, 0, 1)]                     # 15: skipped
    m, prep, tr, pv = C.program_shard(prog, seed=2)
    j = tr["Jump"]
    pcs = [int(x) for x in tr["Cpu"][tr["Cpu"][:, C.C_REAL] == 1, C.C_PC]]
    assert [(p - C.PC_BASE) // 4 for p in pcs] == [0, 1, 2, 12, 13, 14, 3, 4, 12, 13, 14, 5, 6, 8, 9]
    assert int(j[:, C.J_JUMP].sum()) == 3 and int(j[:, C.J_JUMPI].sum()) == 2 and int(j[:, C.J_JDIRECT].sum()) == 1
    assert _air_check.check(m, prep, tr, pv) == ([], [])
    o = O.OracleProver(m, prep, num_queries=8)
    rc, proof = o.prove(tr, pv)
    assert rc == 0 and o.verify(proof) == 0


@pytest.mark.parametrize("body,iters,seed", [(4, 3, 1), (12, 7, 1), (40, 25, 2), (60, 40, 3)])
def test_loop_trace_satisfies_air(body, iters, seed):
    m, prep, tr, pv = C.loop_shard(body, iters, seed)
    assert int(tr["Program"][body + 3, 0]) == iters  # the loop-closing bne ran iters times
    assert _air_check.check(m, prep, tr, pv) == ([], [])


@pytest.fixture(scope="module")
def loop():
    return C.loop_shard(40, 25, seed=2)


def test_loop_shard_proves_and_verifies(loop):
    m, prep, tr, pv = loop
    o = O.OracleProver(m, prep, num_queries=16)
    rc, proof = o.prove(tr, pv)
    assert rc == 0 and o.verify(proof) == 0


@pytest.mark.parametrize("what", ["flip_taken", "target", "lt_flag", "delay_slot_npc", "link", "jump_target"])
def test_branch_tamper_rejected(loop, what):
    m, prep, tr, pv = loop
    bad = {k: v.copy() for k, v in tr.items()}
    br = bad["Branch"]
    if what == "flip_taken":  # claims the branch was not taken (next_next_pc unchanged)
        i = int(np.nonzero(br[:, C.BR_BRANCHING])[0][0])
        br[i, C.BR_BRANCHING] = 0
    elif what == "target":  # only constrained when the branch is taken (the ADD lookup's multiplicity)
        i = int(np.nonzero(br[:, C.BR_BRANCHING])[0][1])
        br[i, C.BR_TGT] ^= 4
    elif what == "lt_flag":
        br[5, C.BR_LT] ^= 1
    elif what == "link":  # a jump-and-link that stores a wrong return address
        bad["Jump"][2, C.J_A] += 4
    elif what == "jump_target":  # j / jal / jr whose next_next_pc is not its target
        j = bad["Jump"]
        i = int(np.nonzero(j[:, C.J_JUMPI] + j[:, C.J_JUMP])[0][0])
        j[i, C.J_NNPC] += 4
    else:  # the CPU continues somewhere else after a taken branch's delay slot
        cpu = bad["Cpu"]
        i = int(np.nonzero(cpu[:, C.C_SEQ] == 0)[0][0]) + 1
        cpu[i, C.C_NPC] += 4
    assert _air_check.check(m, prep, bad, pv) != ([], [])
    o = O.OracleProver(m, prep, num_queries=16)
    rc, proof = o.prove(bad, pv)
    assert rc == 0 and o.verify(proof) != 0


def test_core_register_chain(shard):
    """MemoryLocal holds every register the shard accessed, then every data word it touched, each once
    with its value at the shard's start and end; the Global chip receives two messages per entry."""
    _, _, tr, _ = shard
    e = MM.local_entries(tr["MemoryLocal"])
    regs = e[e[:, 0] < C.NUM_REGS, 0]
    words = e[e[:, 0] >= C.NUM_REGS, 0]
    assert len(regs) and (np.diff(regs) > 0).all() and len(words) and (words >= C.DATA_BASE).all()
    assert (np.diff(words) > 0).all() and len(regs) + len(words) == len(e)
    assert (e[:, 5] <= 5 * 699 + C.POS_HI).all() and (e[:, 4] == 1).all() and (e[:, 1:3] == 0).all()
    assert int(tr["Global"][:, MM.G_REAL].sum()) == 2 * len(e)
    if 0 in regs:
        assert e[e[:, 0] == 0, 3][0] == 0 and e[e[:, 0] == 0, 6][0] == 0  # r0 stays 0


def _word(row, base):
    return int(sum(int(row[base + i]) << (8 * i) for i in range(4)))


def test_mul_kinds():
    """MUL / MULT / MULTU on sign and carry edge cases; LO and HI end up in registers 32 and 33."""
    vals = [(7, 6), (C.M32, C.M32), (C.M32 - 2, 5), (0x80000000, 0x80000000), (0x12345678, 0x9ABCDEF0), (0, C.M32)]
    prog = []
    for b, c in vals:
        prog += [(A.OP_ADD, 1, 0, b, 0, 1), (A.OP_ADD, 2, 0, c, 0, 1)]
        prog += [(C.OP_MUL, 3, 1, 2, 0, 0), (C.OP_MULT, C.REG_LO, 1, 2, 0, 0), (C.OP_MULTU, C.REG_LO, 1, 2, 0, 0)]
    m, prep, tr, pv = C.program_shard(prog, seed=3)
    mu = tr["Mul"]
    assert mu.shape == (32, C.MU_WIDTH)
    for k, (b, c) in enumerate(vals):
        sb = b - (1 << 32) if b >> 31 else b
        sc = c - (1 << 32) if c >> 31 else c
        r_mul, r_mult, r_multu = mu[3 * k], mu[3 * k + 1], mu[3 * k + 2]
        assert _word(r_mul, C.MU_A) == (b * c) & C.M32 and r_mul[C.MU_HRR] == 0
        p = (sb * sc) & ((1 << 64) - 1)
        assert (_word(r_mult, C.MU_A), _word(r_mult, C.MU_HI)) == (p & C.M32, p >> 32) and r_mult[C.MU_HRR] == 1
        assert (_word(r_multu, C.MU_A), _word(r_multu, C.MU_HI)) == ((b * c) & C.M32, (b * c) >> 32)
    b, c = vals[-1]
    assert _final(tr, C.REG_LO) == (b * c) & C.M32 and _final(tr, C.REG_HI) == (b * c) >> 32
    assert _air_check.check(m, prep, tr, pv) == ([], [])
    o = O.OracleProver(m, prep, num_queries=8)
    rc, proof = o.prove(tr, pv)
    assert rc == 0 and o.verify(proof) == 0


_DIV_VALUES = [(7, 2), (C.M32 - 6, 2), (7, C.M32 - 1), (C.M32 - 6, C.M32 - 1), (0x80000000, C.M32), (5, 0), (0, 5),
               (C.M32, C.M32), (0x80000000, 1), (123456789, 1000)]


def test_divrem_kinds():
    """DIV / DIVU / MOD / MODU on signs, i32::MIN / -1 overflow and division by zero (the AIR's c = 0
    branch: quotient 2^32 - 1, remainder b); DIV/DIVU leave (quotient, remainder) in (LO, HI)."""
    prog = []
    for b, c in _DIV_VALUES:
        prog += [(A.OP_ADD, 1, 0, b, 0, 1), (A.OP_ADD, 2, 0, c, 0, 1)]
        prog += [(C.OP_DIV, C.REG_LO, 1, 2, 0, 0), (C.OP_DIVU, C.REG_LO, 1, 2, 0, 0), (C.OP_MOD, 3, 1, 2, 0, 0),
                 (C.OP_MODU, 4, 1, 2, 0, 0)]
    m, prep, tr, pv = C.program_shard(prog, seed=3)
    d = tr["DivRem"]
    s32 = lambda x: x - (1 << 32) if x >> 31 else x
    for k, (b, c) in enumerate(_DIV_VALUES):
        rows = d[4 * k:4 * k + 4]
        if c == 0:
            want_s = want_u = (C.M32, b)
        elif s32(b) == -(1 << 31) and s32(c) == -1:
            want_s, want_u = (b, 0), (b // c, b % c)
        else:
            q = int(abs(s32(b)) // abs(s32(c))) * (1 if (s32(b) < 0) == (s32(c) < 0) else -1)
            want_s, want_u = (q & C.M32, (s32(b) - q * s32(c)) & C.M32), (b // c, b % c)
        assert (_word(rows[0], C.DV_Q), _word(rows[0], C.DV_R)) == want_s
        assert (_word(rows[1], C.DV_Q), _word(rows[1], C.DV_R)) == want_u
        assert _word(rows[2], C.DV_R) == want_s[1] and _word(rows[3], C.DV_R) == want_u[1]
        assert rows[0, C.DV_OVF] == (b == 0x80000000 and c == C.M32) and rows[0, C.DV_IS_C0 + 10] == (c == 0)
    assert _air_check.check(m, prep, tr, pv) == ([], [])
    o = O.OracleProver(m, prep, num_queries=8)
    rc, proof = o.prove(tr, pv)
    assert rc == 0 and o.verify(proof) == 0


def test_movcond_reference_fixture():
    """The program of the reference's test_mov_cond_prove (misc/mov_cond/mod.rs tests): MOVZ/MOVN (MEQ/MNE)
    with zero and nonzero conditions, to r0 and r30, and WSBH into LO and r0."""
    prog = [(A.OP_ADD, 29, 0, 0xF, 0, 1), (A.OP_ADD, 28, 0, 0x8F8F, 0, 1),
            (C.OP_MEQ, 30, 29, 0, 0, 0), (C.OP_MEQ, 30, 29, 28, 0, 0), (C.OP_MEQ, 0, 29, 0, 0, 0),
            (C.OP_MEQ, 0, 29, 29, 0, 0), (C.OP_MNE, 30, 29, 28, 0, 0), (C.OP_MNE, 0, 29, 0, 0, 0),
            (C.OP_WSBH, 32, 29, 0, 0, 1), (C.OP_WSBH, 32, 31, 0, 0, 1), (C.OP_WSBH, 0, 29, 0, 0, 1)]
    m, prep, tr, pv = C.program_shard(prog, seed=4)
    mc = tr["MovCond"]
    assert int(mc[:, C.MC_MEQ].sum()) == 4 and int(mc[:, C.MC_MNE].sum()) == 2 and int(mc[:, C.MC_WSBH].sum()) == 3
    assert _word(mc[0], C.MC_A) == 0xF and _word(mc[4], C.MC_A) == 0xF  # MOVZ with rt = r0, MOVN with rt = r28
    assert _word(mc[6], C.MC_A) == 0x0F00  # WSBH swaps the bytes of each halfword
    r31 = _initial(tr, 31)
    want = ((r31 >> 16 & 0xFF) << 24) | ((r31 >> 24 & 0xFF) << 16) | ((r31 & 0xFF) << 8) | (r31 >> 8 & 0xFF)
    assert _final(tr, C.REG_LO) == want
    assert _air_check.check(m, prep, tr, pv) == ([], [])
    o = O.OracleProver(m, prep, num_queries=8)
    rc, proof = o.prove(tr, pv)
    assert rc == 0 and o.verify(proof) == 0


_ADD = A.OP_ADD
# crates/core/machine/src/programs.rs:126-196 and mips/mod.rs:1042-1054 (Instruction::new(op, a, b, c, imm_b, imm_c))
SIMPLE_MEMORY_PROGRAM = [
    (_ADD, 29, 0, 0x12348765, 0, 1), (C.OP_SW, 29, 0, 0x27654320, 0, 1), (C.OP_LW, 28, 0, 0x27654320, 0, 1),
    (C.OP_LBU, 27, 0, 0x27654320, 0, 1), (C.OP_LBU, 26, 0, 0x27654321, 0, 1), (C.OP_LBU, 25, 0, 0x27654322, 0, 1),
    (C.OP_LBU, 24, 0, 0x27654323, 0, 1), (C.OP_LB, 23, 0, 0x27654320, 0, 1), (C.OP_LB, 22, 0, 0x27654321, 0, 1),
    (C.OP_LHU, 21, 0, 0x27654320, 0, 1), (C.OP_LHU, 20, 0, 0x27654322, 0, 1), (C.OP_LH, 19, 0, 0x27654320, 0, 1),
    (C.OP_LH, 18, 0, 0x27654322, 0, 1), (_ADD, 17, 0, 0x38276525, 0, 1), (C.OP_SW, 29, 0, 0x43627530, 0, 1),
    (C.OP_SB, 17, 0, 0x43627530, 0, 1), (C.OP_LW, 16, 0, 0x43627530, 0, 1), (C.OP_SB, 17, 0, 0x43627531, 0, 1),
    (C.OP_LW, 15, 0, 0x43627530, 0, 1), (C.OP_SB, 17, 0, 0x43627532, 0, 1), (C.OP_LW, 14, 0, 0x43627530, 0, 1),
    (C.OP_SB, 17, 0, 0x43627533, 0, 1), (C.OP_LW, 13, 0, 0x43627530, 0, 1), (C.OP_SW, 29, 0, 0x43627530, 0, 1),
    (C.OP_SH, 17, 0, 0x43627530, 0, 1), (C.OP_LW, 12, 0, 0x43627530, 0, 1), (C.OP_SH, 17, 0, 0x43627532, 0, 1),
    (C.OP_LW, 11, 0, 0x43627530, 0, 1)]
OTHER_MEMORY_PROGRAM = [
    (_ADD, 29, 0, (1 << 20) + (1 << 15) + (1 << 6) - 1, 0, 1), (_ADD, 27, 0, 3325, 0, 1),
    (_ADD, 25, 0, (1 << 28) + (1 << 12) + (1 << 18) - 1, 0, 1), (_ADD, 17, 0, 0x43627530, 0, 1),
    (_ADD, 22, 0, 80, 0, 1), (_ADD, 10, 0, 100, 0, 1), (C.OP_LWR, 29, 27, 1, 0, 1), (C.OP_LWL, 29, 27, 1, 0, 1),
    (C.OP_LL, 29, 27, 3, 0, 1), (_ADD, 15, 0, (1 << 20) + (1 << 15) + (1 << 6) - 1, 0, 1),
    (C.OP_SWL, 15, 22, 2, 0, 1), (C.OP_SWR, 15, 22, 2, 0, 1), (C.OP_SWL, 26, 10, 2, 0, 1),
    (C.OP_SWR, 26, 10, 2, 0, 1), (C.OP_LWR, 29, 27, 0, 0, 1), (C.OP_LWL, 29, 27, 0, 0, 1)]
SC_PROGRAM = [(_ADD, 29, 0, 0x12348765, 0, 1), (C.OP_SW, 29, 0, 0x27654320, 0, 1), (C.OP_LL, 28, 0, 0x27654320, 0, 1),
              (_ADD, 28, 28, 1, 0, 1), (C.OP_SC, 28, 0, 0x27654320, 0, 1), (C.OP_LW, 29, 0, 0x27654320, 0, 1)]


def _reference_alu_fixtures():
    """The straight-line programs of the reference's per-instruction tests (core/machine/src/mips/mod.rs:
    test_simple_prove, test_shift_prove, test_sub/add/add_overflow_prove, test_mul_mod_prove,
    test_mult_div_prove, test_lt_prove, test_bitwise_prove, test_divrem_prove, test_cloclz_prove)."""
    M32 = C.M32
    progs = [[(_ADD, 29, 0, 5, 0, 1), (_ADD, 30, 0, 37, 0, 1), (_ADD, 31, 30, 29, 0, 0)]]
    pairs = [(1, 1), (1234, 5678), (0xFFFF, 0xFFFF - 1), (M32 - 1, M32), (M32, 0)]
    for op in (A.OP_SRL, A.OP_ROR, A.OP_SRA, A.OP_SLL):
        progs += [[(_ADD, 29, 0, b, 0, 1), (_ADD, 30, 0, c, 0, 1), (op, 31, 29, 3, 0, 0)] for b, c in pairs]
    for op, b in ((A.OP_SUB, 5), (_ADD, 5), (_ADD, 0xEFFFFFFF)):
        progs.append([(_ADD, 29, 0, b, 0, 1), (_ADD, 30, 0, 8 if b == 5 else 2, 0, 1), (op, 31, 30, 29, 0, 0)])
    pairs = [(1, 1), (1234, 5678), (8765, 4321), (0xFFFF, 0xFFFF - 1), (M32 - 1, M32)]
    for op in (C.OP_MUL, C.OP_MOD, C.OP_MODU):
        progs += [[(_ADD, 29, 0, b, 0, 1), (_ADD, 30, 0, c, 0, 1), (op, 31, 30, 29, 0, 0)] for b, c in pairs]
    for op in (C.OP_MULT, C.OP_MULTU, C.OP_DIV, C.OP_DIVU):
        progs += [[(_ADD, 29, 0, b, 0, 1), (_ADD, 30, 0, c, 0, 1), (op, 32, 30, 29, 0, 0)] for b, c in pairs]
    for op in (A.OP_SLT, A.OP_SLTU, A.OP_XOR, A.OP_OR, A.OP_AND):
        progs.append([(_ADD, 29, 0, 5, 0, 1), (_ADD, 30, 0, 8, 0, 1), (op, 31, 30, 29, 0, 0)])
    pairs = [(1, 1), (123, 456 * 789), (123 * 456, 789), (0xFFFF * (0xFFFF - 1), 0xFFFF), (M32 - 5, M32 - 7)]
    for op in (C.OP_DIV, C.OP_DIVU):
        progs += [[(_ADD, 29, 0, b, 0, 1), (_ADD, 30, 0, c, 0, 1), (op, 32, 29, 30, 0, 0)] for b, c in pairs]
    for op in (A.OP_CLZ, A.OP_CLO):
        progs += [[(_ADD, 29, 0, v, 0, 1), (op, 30, 29, 0, 0, 1)]
                  for v in (0, 0x0A0B0C0D, 0x1000, 0xFF7FFFFF, 0x7FFFFFFF, 0x80000000, 0xFFFFFFFF)]
    return progs


def _reference_control_fixtures():
    """test_beq/bne_(not_)branching_prove, test_rest_branch_prove, test_j/jr/jal/jalr_prove
    (core/machine/src/mips/mod.rs:751-1039): each leaves the program through its branch or jump."""
    progs = [[(_ADD, 29, 0, x, 0, 1), (_ADD, 30, 0, y, 0, 1), (op, 29, 30, 100, 0, 1)]
             for op, x, y in ((C.OP_BEQ, 1, 1), (C.OP_BEQ, 1, 2), (C.OP_BNE, 1, 2), (C.OP_BNE, 0, 0))]
    for op in (C.OP_BLTZ, C.OP_BGEZ, C.OP_BLEZ, C.OP_BGTZ):
        progs += [[(_ADD, 29, 0, v, 0, 1), (op, 29, 0, 100, 1, 1)] for v in (0, 1, C.M32)]
    progs += [[(_ADD, 11, 0, 100, 0, 1), (C.OP_JUMPI, 0, 100, 0, 1, 1)],
              [(_ADD, 11, 0, 100, 0, 1), (C.OP_JUMP, 0, 11, 0, 0, 1)],
              [(_ADD, 31, 0, 0, 0, 1), (C.OP_JUMPI, 31, 100, 0, 1, 1)],
              [(_ADD, 5, 0, 0, 0, 1), (_ADD, 11, 11, 100, 0, 1), (C.OP_JUMP, 5, 11, 0, 0, 1)]]
    return progs


def test_reference_instruction_programs():
    """All straight-line programs of the reference's per-instruction tests, run back to back in one shard."""
    prog = [ins for p in _reference_alu_fixtures() for ins in p]
    m, prep, tr, pv = C.program_shard(prog, seed=6)
    assert int(tr["Cpu"][:, C.C_REAL].sum()) == len(prog)
    assert _air_check.check(m, prep, tr, pv) == ([], [])
    o = O.OracleProver(m, prep, num_queries=8)
    rc, proof = o.prove(tr, pv)
    assert rc == 0 and o.verify(proof) == 0


@pytest.mark.parametrize("k", range(20))
def test_reference_control_programs(k):
    prog = _reference_control_fixtures()[k]
    m, prep, tr, pv = C.program_shard(prog, seed=k)
    assert _air_check.check(m, prep, tr, pv) == ([], [])
    o = O.OracleProver(m, prep, num_queries=8)
    rc, proof = o.prove(tr, pv)
    assert rc == 0 and o.verify(proof) == 0


# misc/others/mod.rs test_misc_prove
MISC_PROGRAM = [
    (_ADD, 29, 0, 0xF, 0, 1), (_ADD, 28, 0, 0x8F8F, 0, 1),
    (C.OP_SEXT, 30, 29, 0, 0, 1), (C.OP_SEXT, 31, 28, 0, 0, 1), (C.OP_SEXT, 0, 28, 0, 0, 1),
    (C.OP_SEXT, 30, 29, 1, 0, 1), (C.OP_SEXT, 31, 28, 1, 0, 1), (C.OP_SEXT, 0, 28, 1, 0, 1),
    (C.OP_EXT, 30, 28, 0x21, 0, 1), (C.OP_EXT, 30, 31, 0x1EF, 0, 1), (C.OP_EXT, 0, 28, 0x21, 0, 1),
    (C.OP_INS, 30, 29, 0x21, 0, 1), (C.OP_INS, 30, 31, 0x3EF, 0, 1), (C.OP_INS, 0, 29, 0x21, 0, 1),
    (C.OP_MADDU, 32, 31, 31, 0, 0), (C.OP_MADDU, 32, 29, 31, 0, 0), (C.OP_MADDU, 32, 29, 0, 0, 0),
    (C.OP_MSUBU, 32, 31, 31, 0, 0), (C.OP_MSUBU, 32, 29, 31, 0, 0), (C.OP_MSUBU, 32, 29, 0, 0, 0),
    (C.OP_MADD, 32, 31, 31, 0, 0), (C.OP_MADD, 32, 29, 31, 0, 0), (C.OP_MADD, 32, 29, 0, 0, 0),
    (C.OP_MSUB, 32, 31, 31, 0, 0), (C.OP_MSUB, 32, 29, 31, 0, 0), (C.OP_MSUB, 32, 29, 0, 0, 0),
    (C.OP_TEQ, 28, 29, 0, 0, 1), (C.OP_TEQ, 28, 0, 0, 0, 1), (C.OP_TEQ, 0, 28, 0, 0, 1)]


def test_misc_reference_fixture():
    """The reference's test_misc_prove program: SEB/SEH, EXT, INS, MADDU/MSUBU/MADD/MSUB (HI:LO
    accumulate and its 64-bit AddDouble), TEQ (non-trapping)."""
    m, prep, tr, pv = C.program_shard(MISC_PROGRAM, seed=1)
    ms = tr["MiscInstrs"]
    assert [int(ms[:, C.MS_SEL + k].sum()) for k in range(8)] == [6, 3, 3, 3, 3, 3, 3, 3]
    assert _final(tr, 31) == 0xFFFF8F8F  # SEH of 0x8F8F
    # MADDU, MSUBU, MADD and MSUB of the same operands cancel pairwise: HI:LO returns to its start
    assert _final(tr, C.REG_LO) == _initial(tr, C.REG_LO)
    assert _final(tr, C.REG_HI) == _initial(tr, C.REG_HI)
    assert _air_check.check(m, prep, tr, pv) == ([], [])
    o = O.OracleProver(m, prep, num_queries=8)
    rc, proof = o.prove(tr, pv)
    assert rc == 0 and o.verify(proof) == 0


@pytest.mark.parametrize("what", ["ins_result", "maddsub_carry", "sext_sign", "teq_equal"])
def test_misc_tamper_rejected(what):
    m, prep, tr, pv = C.program_shard(MISC_PROGRAM, seed=1)
    bad = {k: v.copy() for k, v in tr.items()}
    ms = bad["MiscInstrs"]
    if what == "ins_result":
        i = int(np.nonzero(ms[:, C.MS_SEL + 1])[0][0])
        ms[i, C.MS_A] ^= 4
    elif what == "maddsub_carry":
        i = int(np.nonzero(ms[:, C.MS_SEL + 3])[0][0])
        ms[i, C.MS_SPEC + 16] ^= 1
    elif what == "sext_sign":
        i = int(np.nonzero(ms[:, C.MS_SEL])[0][1])
        ms[i, C.MS_SPEC] ^= 1
    else:  # a TEQ that claims its operands are equal (it would have trapped)
        i = int(np.nonzero(ms[:, C.MS_SEL + 7])[0][0])
        ms[i, C.MS_SPEC + 2] = 1
    assert _air_check.check(m, prep, bad, pv) != ([], [])
    o = O.OracleProver(m, prep, num_queries=8)
    rc, proof = o.prove(bad, pv)
    assert rc == 0 and o.verify(proof) != 0


def _final(tr, addr):
    e = MM.local_entries(tr["MemoryLocal"])
    return int(e[e[:, 0] == addr, 6][0])


def _initial(tr, addr):
    e = MM.local_entries(tr["MemoryLocal"])
    return int(e[e[:, 0] == addr, 3][0])


@pytest.mark.parametrize("name", ["simple_memory", "other_memory", "sc"])
def test_memory_reference_programs(name):
    """The reference's own memory-instruction programs (programs.rs simple_memory_program /
    other_memory_program, mips/mod.rs test_sc_prove) prove and verify through the MemoryInstrs chip."""
    prog = {"simple_memory": SIMPLE_MEMORY_PROGRAM, "other_memory": OTHER_MEMORY_PROGRAM, "sc": SC_PROGRAM}[name]
    m, prep, tr, pv = C.program_shard(prog, seed=1)
    if name == "simple_memory":
        assert [_final(tr, r) for r in (28, 27, 26, 25, 24)] == [0x12348765, 0x65, 0x87, 0x34, 0x12]
        assert [_final(tr, r) for r in (23, 22, 21, 20, 19, 18)] == [0x65, 0xFFFFFF87, 0x8765, 0x1234, 0xFFFF8765,
                                                                      0x1234]
        assert [_final(tr, r) for r in (16, 15, 14, 13)] == [0x12348725, 0x12342525, 0x12252525, 0x25252525]
        assert [_final(tr, r) for r in (12, 11)] == [0x12346525, 0x65256525]
    elif name == "sc":
        assert _final(tr, 28) == 1 and _final(tr, 29) == 0x12348766 and _final(tr, 0x27654320) == 0x12348766
    assert _air_check.check(m, prep, tr, pv) == ([], [])
    o = O.OracleProver(m, prep, num_queries=8)
    rc, proof = o.prove(tr, pv)
    assert rc == 0 and o.verify(proof) == 0


@pytest.mark.parametrize("what", ["load_value", "store_merge", "memory_final", "address"])
def test_memory_tamper_rejected(shard, oracle, what):
    m, prep, tr, pv = shard
    bad = {k: v.copy() for k, v in tr.items()}
    mi = bad["MemoryInstrs"]
    if what == "load_value":  # an LW that returns something else than the word in memory
        i = int(np.nonzero(mi[:, C.MI_SEL + 4])[0][0])
        mi[i, C.MI_UMV] = (int(mi[i, C.MI_UMV]) + 1) % 256
        mi[i, C.MI_A] = mi[i, C.MI_UMV]
    elif what == "store_merge":  # an SB that also changes a neighbouring byte
        i = int(np.nonzero(mi[:, C.MI_SEL + 8])[0][0])
        j = (int(mi[i, C.MI_LS2]) + 1) % 4
        mi[i, C.MI_ACC + 4 + j] = (int(mi[i, C.MI_ACC + 4 + j]) + 1) % 256
    elif what == "memory_final":  # the memory argument's closing value of a data word
        ml = bad["MemoryLocal"].reshape(-1, MM.ML_ENTRY_WIDTH)
        k = int(np.nonzero(ml[:, MM.ML_ADDR] >= C.DATA_BASE)[0][0])
        ml[k, MM.ML_FVAL] ^= 1
    else:  # the access goes to another word than b + c
        mi[3, C.MI_ALIGNED] += 4
    assert _air_check.check(m, prep, bad, pv) != ([], [])
    rc, proof = oracle.prove(bad, pv)
    assert rc == 0 and oracle.verify(proof) != 0


@pytest.mark.parametrize("what", ["moved", "kept", "wsbh"])
def test_movcond_tamper_rejected(shard, oracle, what):
    m, prep, tr, pv = shard
    bad = {k: v.copy() for k, v in tr.items()}
    mc = bad["MovCond"]
    if what == "moved":  # a MOVZ/MOVN that moved, with a different value in both the chip and the CPU
        i = int(np.nonzero((mc[:, C.MC_MEQ] == 1) & (mc[:, C.MC_C0 + 10] == 1))[0][0])
    elif what == "kept":
        i = int(np.nonzero((mc[:, C.MC_MEQ] == 1) & (mc[:, C.MC_C0 + 10] == 0))[0][0])
    else:
        i = int(np.nonzero(mc[:, C.MC_WSBH])[0][0])
    mc[i, C.MC_A] = (int(mc[i, C.MC_A]) + 1) % 256
    assert _air_check.check(m, prep, bad, pv) != ([], [])
    rc, proof = oracle.prove(bad, pv)
    assert rc == 0 and oracle.verify(proof) != 0


@pytest.mark.parametrize("what", ["quotient", "remainder_sign", "div_carry", "c_is_zero"])
def test_divrem_tamper_rejected(shard, oracle, what):
    m, prep, tr, pv = shard
    bad = {k: v.copy() for k, v in tr.items()}
    d = bad["DivRem"]
    nz = np.nonzero(d[:, C.DV_IS_C0 + 10] == 0)[0]
    i = int(nz[0])
    if what == "quotient":  # q + 1 with the remainder unchanged
        d[i, C.DV_Q] = (int(d[i, C.DV_Q]) + 1) % 256
    elif what == "remainder_sign":
        j = int(np.nonzero(d[:, C.DV_DIV] + d[:, C.DV_MOD])[0][0])
        d[j, C.DV_RNEG] ^= 1
    elif what == "div_carry":
        d[i, C.DV_CARRY] ^= 1
    else:  # claims division by zero for a nonzero divisor
        d[i, C.DV_IS_C0 + 10] = 1
    assert _air_check.check(m, prep, bad, pv) != ([], [])
    rc, proof = oracle.prove(bad, pv)
    assert rc == 0 and oracle.verify(proof) != 0


@pytest.mark.parametrize("what", ["carry", "hi", "sign_extend", "hi_register"])
def test_mul_tamper_rejected(shard, oracle, what):
    m, prep, tr, pv = shard
    bad = {k: v.copy() for k, v in tr.items()}
    mu = bad["Mul"]
    i = int(np.nonzero(mu[:, C.MU_MULT] * mu[:, C.MU_HRR])[0][0])  # a CPU MULT (DivRem's have no HI record)
    if what == "carry":
        mu[i, C.MU_CARRY + 2] += 1
    elif what == "hi":  # a forged HI in both the chip and its register write
        mu[i, C.MU_HI] ^= 1
        mu[i, C.MU_HI_ACC + 4] ^= 1
    elif what == "sign_extend":  # MULT treated as unsigned
        j = int(np.nonzero(mu[:, C.MU_BSE])[0][0])
        mu[j, C.MU_BSE] = 0
    else:  # the HI write is dropped from the memory argument
        mu[i, C.MU_HRR] = 0
    assert _air_check.check(m, prep, bad, pv) != ([], [])
    rc, proof = oracle.prove(bad, pv)
    assert rc == 0 and oracle.verify(proof) != 0


def _with_global_chip(shard, seed=9):
    """The core shard plus a Global-scope chip (commit_scope Global, crates/core/machine/src/global/mod.rs:202):
    its last row's last 14 main columns are the shard's septic global cumulative sum, which the prover
    captures (prover.rs:352-361), observes, and the quotient ties to the trace with 14 last-row
    constraints (permutation.rs:331-343).  The septic-curve accumulation itself is not restated; the
    digest here is 14 synthetic field elements."""
    from zkmips_amd.machine import ChipDesc, MachineDesc, main
    from zkmips_amd.workloads import splitmix64
    m, prep, tr, pv = shard
    ch = ChipDesc("GlobalStandIn", prep_width=0, main_width=15, commit_scope=1)
    ch.assert_zero(main(0) * (main(0) - 1))
    mg = MachineDesc(m.chips + [ch], m.num_pv)
    g = np.zeros((64, 15), np.uint32)
    g[:40, 0] = 1
    g[:, 1:] = (splitmix64(0x61B0000 + seed, 64 * 14) % np.uint64(A.P)).astype(np.uint32).reshape(64, 14)
    return mg, prep, {**tr, "GlobalStandIn": g}, pv


def test_global_scope_chip(shard):
    mg, prep, tr, pv = _with_global_chip(shard)
    assert mg.chips[-1].num_constraints == 1 + 14
    o = O.OracleProver(mg, prep, num_queries=8)
    rc, proof = o.prove(tr, pv)
    assert rc == 0 and o.verify(proof) == 0
    assert tr["GlobalStandIn"][-1, 1:].astype("<u4").tobytes() in proof  # the captured digest


# ---------------------------------------------------------------- GPU parity
@pytest.fixture(scope="module")
def dev():
    from zkmips_amd._lib import Device
    d = Device(0)
    yield d
    d.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n,seed", [(17, 3), (700, 4), (20000, 6), (1 << 17, 7)])
def test_core_gpu_proof_bytes_identical(dev, n, seed):
    from zkmips_amd.prover import HipProver
    m, prep, tr, pv = C.core_shard(n, seed=seed)
    gpu = HipProver(dev, m, prep, num_queries=16)
    cpu = O.OracleProver(m, prep, num_queries=16)
    assert np.array_equal(gpu.vk_commit, cpu.commit)
    proof = gpu.prove_shard(tr, pv)
    rc, ref = cpu.prove(tr, pv)
    assert rc == 0 and proof == ref
    assert cpu.verify(proof) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["alu_fixtures", "simple_memory", "other_memory", "sc", "jalr", "misc"])
def test_reference_programs_gpu_proof_bytes_identical(dev, name):
    """The reference's own instruction-test programs: GPU proof bytes == oracle proof bytes."""
    from zkmips_amd.prover import HipProver
    prog = {"alu_fixtures": [ins for p in _reference_alu_fixtures() for ins in p],
            "simple_memory": SIMPLE_MEMORY_PROGRAM, "other_memory": OTHER_MEMORY_PROGRAM, "sc": SC_PROGRAM,
            "jalr": _reference_control_fixtures()[-1], "misc": MISC_PROGRAM}[name]
    m, prep, tr, pv = C.program_shard(prog, seed=6)
    gpu = HipProver(dev, m, prep, num_queries=16)
    cpu = O.OracleProver(m, prep, num_queries=16)
    proof = gpu.prove_shard(tr, pv)
    rc, ref = cpu.prove(tr, pv)
    assert rc == 0 and proof == ref and cpu.verify(proof) == 0


@pytest.mark.gpu
def test_global_scope_gpu_proof_bytes_identical(dev, shard):
    from zkmips_amd.prover import HipProver
    mg, prep, tr, pv = _with_global_chip(shard)
    gpu = HipProver(dev, mg, prep, num_queries=16)
    cpu = O.OracleProver(mg, prep, num_queries=16)
    proof = gpu.prove_shard(tr, pv)
    rc, ref = cpu.prove(tr, pv)
    assert rc == 0 and proof == ref and cpu.verify(proof) == 0
    assert tr["GlobalStandIn"][-1, 1:].astype("<u4").tobytes() in proof


@pytest.mark.gpu
@pytest.mark.parametrize("body,iters,seed", [(12, 7, 1), (40, 300, 2), (60, 4000, 3)])
def test_loop_gpu_proof_bytes_identical(dev, body, iters, seed):
    from zkmips_amd.prover import HipProver
    m, prep, tr, pv = C.loop_shard(body, iters, seed)
    gpu = HipProver(dev, m, prep, num_queries=16)
    cpu = O.OracleProver(m, prep, num_queries=16)
    assert np.array_equal(gpu.vk_commit, cpu.commit)
    proof = gpu.prove_shard(tr, pv)
    rc, ref = cpu.prove(tr, pv)
    assert rc == 0 and proof == ref
    assert cpu.verify(proof) == 0


@pytest.mark.gpu
def test_loop_gpu_full_size_verifies(dev):
    from zkmips_amd.prover import HipProver
    m, prep, tr, pv = C.loop_shard(60, 30000, seed=5)
    assert tr["Cpu"].shape == (1 << 22, 67)
    gpu = HipProver(dev, m, prep, num_queries=84)
    cpu = O.OracleProver(m, prep, num_queries=84)
    assert cpu.verify(gpu.prove_shard(tr, pv)) == 0
    bad = {k: v.copy() for k, v in tr.items()}
    bad["Branch"][777, C.BR_LT] ^= 1
    assert cpu.verify(gpu.prove_shard(bad, pv)) != 0


@pytest.mark.gpu
def test_core_gpu_full_size_verifies(dev):
    from zkmips_amd.prover import HipProver
    # random-instruction shard at the headline height: Cpu 2^22 rows (2.1M instructions, every
    # restated chip incl. MiscInstrs, MemoryLocal and Global; ~30 s of trace generation)
    n = (1 << 21) + 12345
    m, prep, tr, pv = C.core_shard(n, seed=11)
    assert tr["Cpu"].shape == (1 << 22, 67)
    gpu = HipProver(dev, m, prep, num_queries=84)
    cpu = O.OracleProver(m, prep, num_queries=84)
    proof = gpu.prove_shard(tr, pv)
    assert cpu.verify(proof) == 0
    rc, ref = cpu.prove(tr, pv)  # every restated chip at the headline height, byte for byte
    assert rc == 0 and proof == ref
    assert cpu.verify(gpu.prove_shard(_tamper(tr, "register_read"), pv)) != 0
