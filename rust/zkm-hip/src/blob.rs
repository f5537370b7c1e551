//! Machine blob (format: include/zkm_hip.h, end of file) from a `StarkMachine`: every chip's AIR as
//! the postfix program of its symbolic constraints (the same `get_symbolic_constraints` the reference
//! counts them with, crates/stark/src/machine.rs:357-362) and its sends / receives
//! (crates/stark/src/chip.rs:19-40) as VirtualPairCol descriptors.  This is how the real MIPS chips
//! reach the GPU without a hand restatement: the blob is derived from the Rust AIRs themselves.
use std::collections::HashMap;
use std::rc::Rc;

use p3_air::VirtualPairCol;
use p3_field::{AbstractField, PrimeField32};
use p3_uni_stark::{get_symbolic_constraints, Entry, SymbolicExpression};
use zkm_stark::air::{LookupScope, MachineAir, PROOF_MAX_NUM_PVS};
use zkm_stark::{Chip, Lookup, StarkGenericConfig, StarkMachine, Val};

const MAGIC: u32 = 0x4D4D_4B5A;
const VERSION: u32 = 1;

// postfix opcodes (zkm_hip.h)
const OP_MAIN_L: u32 = 1;
const OP_MAIN_N: u32 = 2;
const OP_PREP_L: u32 = 3;
const OP_PREP_N: u32 = 4;
const OP_CONST: u32 = 5;
const OP_PV: u32 = 6;
const OP_IS_FIRST: u32 = 7;
const OP_IS_LAST: u32 = 8;
const OP_IS_TRANS: u32 = 9;
const OP_ADD: u32 = 10;
const OP_SUB: u32 = 11;
const OP_MUL: u32 = 12;
const OP_NEG: u32 = 13;
const OP_EMIT: u32 = 14;

const OP_LET: u32 = 15;
const OP_GET: u32 = 16;

type Node<F> = SymbolicExpression<F>;

fn key<F>(e: &Node<F>) -> usize {
    e as *const _ as usize
}

fn children<F>(e: &Node<F>) -> Vec<&Node<F>> {
    match e {
        SymbolicExpression::Add { x, y, .. } | SymbolicExpression::Sub { x, y, .. } | SymbolicExpression::Mul { x, y, .. } => {
            vec![x.as_ref(), y.as_ref()]
        }
        SymbolicExpression::Neg { x, .. } => vec![x.as_ref()],
        _ => vec![],
    }
}

/// Parent references of every node of the constraints' DAG (an Rc'd node cloned into several parents
/// is one node with several references).
fn count_refs<F>(e: &Node<F>, refs: &mut HashMap<usize, u32>) {
    let n = refs.entry(key(e)).or_insert(0);
    *n += 1;
    if *n == 1 {
        for c in children(e) {
            count_refs(c, refs);
        }
    }
}

/// The chip program: every interior node referenced more than once becomes a shared subexpression,
/// defined once (its code, then LET slot) in post-order -- slots 0, 1, 2, ... before their first
/// use -- and read with GET wherever it is used; then one EMIT per constraint.  Linear in the size
/// of the DAG, where re-emitting shared nodes per use is exponential in the depth of chained layers
/// (e.g. Poseidon2's 13 internal rounds).
struct Lowering {
    refs: HashMap<usize, u32>,
    slot: HashMap<usize, u32>,
    defs: Vec<u32>,
}

impl Lowering {
    fn shared<F>(&self, e: &Node<F>) -> bool {
        !children(e).is_empty() && self.refs.get(&key(e)).copied().unwrap_or(0) > 1
    }

    /// Defines the shared nodes below (and including) `e`, children first.
    fn define<F: PrimeField32>(&mut self, e: &Node<F>) {
        if self.slot.contains_key(&key(e)) {
            return;
        }
        for c in children(e) {
            self.define(c);
        }
        if self.shared(e) {
            let mut code = Vec::new();
            self.emit(e, &mut code, true);
            let s = self.slot.len() as u32;
            code.extend([OP_LET, s]);
            self.defs.extend(code);
            self.slot.insert(key(e), s);
        }
    }

    /// Postfix code of `e`, shared nodes as GET (except `e` itself when it is being defined).
    fn emit<F: PrimeField32>(&self, e: &Node<F>, out: &mut Vec<u32>, top: bool) {
        if !top {
            if let Some(&s) = self.slot.get(&key(e)) {
                out.extend([OP_GET, s]);
                return;
            }
        }
        match e {
            SymbolicExpression::Variable(v) => match v.entry {
                Entry::Main { offset } => out.extend([if offset == 0 { OP_MAIN_L } else { OP_MAIN_N }, v.index as u32]),
                Entry::Preprocessed { offset } => {
                    out.extend([if offset == 0 { OP_PREP_L } else { OP_PREP_N }, v.index as u32])
                }
                Entry::Public => out.extend([OP_PV, v.index as u32]),
                Entry::Permutation { .. } | Entry::Challenge => {
                    panic!("main-trace constraints reference no permutation columns or challenges")
                }
            },
            SymbolicExpression::IsFirstRow => out.push(OP_IS_FIRST),
            SymbolicExpression::IsLastRow => out.push(OP_IS_LAST),
            SymbolicExpression::IsTransition => out.push(OP_IS_TRANS),
            SymbolicExpression::Constant(c) => out.extend([OP_CONST, c.as_canonical_u32()]),
            SymbolicExpression::Add { x, y, .. } => self.bin(x, y, OP_ADD, out),
            SymbolicExpression::Sub { x, y, .. } => self.bin(x, y, OP_SUB, out),
            SymbolicExpression::Mul { x, y, .. } => self.bin(x, y, OP_MUL, out),
            SymbolicExpression::Neg { x, .. } => {
                self.emit(x, out, false);
                out.push(OP_NEG);
            }
        }
    }

    fn bin<F: PrimeField32>(&self, x: &Rc<Node<F>>, y: &Rc<Node<F>>, op: u32, out: &mut Vec<u32>) {
        self.emit(x, out, false);
        self.emit(y, out, false);
        out.push(op);
    }
}

fn chip_program<F: PrimeField32>(constraints: &[Node<F>]) -> Vec<u32> {
    let mut l = Lowering { refs: HashMap::new(), slot: HashMap::new(), defs: Vec::new() };
    for c in constraints {
        count_refs(c, &mut l.refs);
    }
    for c in constraints {
        for ch in children(c) {
            l.define(ch);
        }
    }
    let mut code = std::mem::take(&mut l.defs);
    for c in constraints {
        l.emit(c, &mut code, true);
        code.push(OP_EMIT);
    }
    code
}

/// VirtualPairCol -> [num_terms, (col | main bit31, weight)..., constant], recovered through the
/// public `apply` (the column is an affine function of the row): constant = f(0), weight_j = f(e_j) - f(0).
fn vpc_words<F: PrimeField32>(v: &VirtualPairCol<F>, prep_w: usize, main_w: usize, out: &mut Vec<u32>) {
    let zp = vec![F::zero(); prep_w];
    let zm = vec![F::zero(); main_w];
    let c0: F = v.apply::<F, F>(&zp, &zm);
    let mut terms = Vec::new();
    for j in 0..prep_w {
        let mut p = zp.clone();
        p[j] = F::one();
        let w = v.apply::<F, F>(&p, &zm) - c0;
        if !w.is_zero() {
            terms.push((j as u32, w.as_canonical_u32()));
        }
    }
    for j in 0..main_w {
        let mut m = zm.clone();
        m[j] = F::one();
        let w = v.apply::<F, F>(&zp, &m) - c0;
        if !w.is_zero() {
            terms.push((0x8000_0000 | j as u32, w.as_canonical_u32()));
        }
    }
    out.push(terms.len() as u32);
    for (c, w) in terms {
        out.extend([c, w]);
    }
    out.push(c0.as_canonical_u32());
}

fn lookup_words<F: PrimeField32>(l: &Lookup<F>, prep_w: usize, main_w: usize, out: &mut Vec<u32>) {
    out.push(l.kind as u32);
    out.push(match l.scope {
        LookupScope::Local => 0,
        LookupScope::Global => 1,
    });
    out.push(l.values.len() as u32);
    for v in &l.values {
        vpc_words(v, prep_w, main_w, out);
    }
    vpc_words(&l.multiplicity, prep_w, main_w, out);
}

fn chip_words<SC, A>(chip: &Chip<Val<SC>, A>, out: &mut Vec<u32>)
where
    SC: StarkGenericConfig,
    Val<SC>: PrimeField32,
    A: MachineAir<Val<SC>> + for<'a> p3_air::Air<p3_uni_stark::SymbolicAirBuilder<Val<SC>>>,
{
    let name = chip.name();
    let bytes = name.as_bytes();
    out.push(bytes.len() as u32);
    for c in bytes.chunks(4) {
        let mut w = [0u8; 4];
        w[..c.len()].copy_from_slice(c);
        out.push(u32::from_le_bytes(w));
    }
    let prep_w = chip.preprocessed_width();
    let main_w = chip.width();
    let constraints = get_symbolic_constraints(&chip.air, prep_w, PROOF_MAX_NUM_PVS);
    let code = chip_program(&constraints);
    out.extend([
        prep_w as u32,
        main_w as u32,
        match chip.commit_scope() {
            LookupScope::Local => 0,
            LookupScope::Global => 1,
        },
        chip.local_only() as u32,
        chip.log_quotient_degree() as u32,
        constraints.len() as u32,
        code.len() as u32,
    ]);
    out.extend(code);
    out.push(chip.sends().len() as u32);
    out.push(chip.receives().len() as u32);
    for l in chip.sends().iter().chain(chip.receives()) {
        lookup_words(l, prep_w, main_w, out);
    }
}

/// The whole machine's blob, chips in machine order (the order zkm_setup's `prep` array follows).
pub fn machine_blob<SC, A>(machine: &StarkMachine<SC, A>) -> Vec<u32>
where
    SC: StarkGenericConfig,
    Val<SC>: PrimeField32,
    A: MachineAir<Val<SC>> + for<'a> p3_air::Air<p3_uni_stark::SymbolicAirBuilder<Val<SC>>>,
{
    let chips = machine.chips();
    let mut w = vec![MAGIC, VERSION, machine.num_pv_elts() as u32, chips.len() as u32];
    for chip in chips.iter() {
        chip_words::<SC, A>(chip, &mut w);
    }
    w
}
