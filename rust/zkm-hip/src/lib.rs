//! MI355X shard prover for Ziren behind the reference's `MachineProver` trait
//! (crates/stark/src/prover.rs:30-184), plus device trace generation for the chips the reference
//! exposes a native row ABI for (crates/core/machine/src/sys.rs:14-42).
//!
//! `ZKMProverComponents::CoreProver = HipProver<MipsAir<KoalaBear>>` (crates/prover/src/components.rs)
//! is the whole integration: `prove_with_context` keeps calling `commit` / `open` from its workers.
pub mod blob;
pub mod prover;
pub mod sys;
pub mod tracegen;

pub use prover::{HipProver, HipProverError};
