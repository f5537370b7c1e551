//! `HipProver`: the reference's `MachineProver` (crates/stark/src/prover.rs:30-184) over the C ABI of
//! libzkm_hip.so.  The shape follows `CpuProver` (prover.rs:201-694): `setup` builds the proving key,
//! `commit` hands the shard's traces to the GPU (sorted there by (height desc, name), as prover.rs
//! sorts them), `open` runs the rest of the shard proof on the GPU and returns the `ShardProof`,
//! which the ABI serialises in the bincode-1 layout of the reference's serde derive.
use std::collections::HashMap;
use std::ffi::CString;
use std::ptr;

use p3_field::{AbstractField, PrimeField32};
use p3_koala_bear::KoalaBear;
use p3_matrix::{dense::RowMajorMatrix, Matrix};
use zkm_stark::air::MachineAir;
use zkm_stark::septic_digest::SepticDigest;
use zkm_stark::{
    Com, KoalaBearPoseidon2, MachineProof, MachineProver, MachineProvingKey, MachineRecord, ShardMainData,
    ShardProof, StarkGenericConfig, StarkMachine, StarkProvingKey, StarkVerifyingKey, Val,
};

use crate::blob::machine_blob;
use crate::sys::*;

type SC = KoalaBearPoseidon2;
type Challenger = <SC as StarkGenericConfig>::Challenger;

#[derive(Debug, thiserror::Error)]
#[error("libzkm_hip: {0}")]
pub struct HipProverError(pub String);

fn check(rc: i32, what: &str) -> Result<(), HipProverError> {
    if rc == ZKM_OK {
        Ok(())
    } else {
        Err(HipProverError(format!("{what} failed ({rc}): {}", last_error())))
    }
}

/// One GPU context; the ABI is thread-safe (one HIP stream per call), so the handle is shared by the
/// `prove_with_context` workers.
struct Ctx(*mut zkm_ctx);
unsafe impl Send for Ctx {}
unsafe impl Sync for Ctx {}
impl Drop for Ctx {
    fn drop(&mut self) {
        unsafe { zkm_destroy(self.0) }
    }
}

/// The device proving key plus the host key the trait's accessors read.  Shared (`Arc`) across the
/// `prove_with_context` workers.
pub struct PkInner {
    pk: *mut zkm_pk,
    host: StarkProvingKey<SC>,
}
unsafe impl Send for PkInner {}
unsafe impl Sync for PkInner {}
impl Drop for PkInner {
    fn drop(&mut self) {
        unsafe { zkm_pk_free(self.pk) }
    }
}
#[derive(Clone)]
pub struct HipProvingKey(std::sync::Arc<PkInner>);

impl MachineProvingKey<SC> for HipProvingKey {
    fn preprocessed_commit(&self) -> Com<SC> {
        self.0.host.commit
    }
    fn pc_start(&self) -> Val<SC> {
        self.0.host.pc_start
    }
    fn initial_global_cumulative_sum(&self) -> SepticDigest<Val<SC>> {
        self.0.host.initial_global_cumulative_sum
    }
    fn observe_into(&self, challenger: &mut Challenger) {
        self.0.host.observe_into(challenger)
    }
}

/// The committed shard on the device (LDEs + Merkle tree), released by `open` or on drop.
pub struct HipMainData(*mut zkm_main);
unsafe impl Send for HipMainData {}
unsafe impl Sync for HipMainData {}
impl Drop for HipMainData {
    fn drop(&mut self) {
        if !self.0.is_null() {
            unsafe { zkm_main_free(self.0) }
        }
    }
}

/// The machine layout for `commit` (zkm_machine_new): the trait's `commit` receives no proving key,
/// and the compress workers call `setup(program)` and `commit` concurrently for different programs
/// (prover/src/lib.rs:794-824), so commit must not depend on whichever key was set up last.
struct MachineHandle(*mut zkm_machine);
unsafe impl Send for MachineHandle {}
unsafe impl Sync for MachineHandle {}
impl Drop for MachineHandle {
    fn drop(&mut self) {
        unsafe { zkm_machine_free(self.0) }
    }
}

pub struct HipProver<A> {
    machine: StarkMachine<SC, A>,
    ctx: Ctx,
    blob: Vec<u32>,
    cfg: zkm_config_t,
    layout: MachineHandle,
}

fn canonical(v: &[KoalaBear]) -> Vec<u32> {
    v.iter().map(|x| x.as_canonical_u32()).collect()
}

fn digest_words(d: &SepticDigest<KoalaBear>) -> [u32; 14] {
    let mut w = [0u32; 14];
    for i in 0..7 {
        w[i] = d.0.x.0[i].as_canonical_u32();
        w[7 + i] = d.0.y.0[i].as_canonical_u32();
    }
    w
}

/// A RowMajorMatrix<KoalaBear> as an ABI matrix: its storage is Montgomery u32 (MontyField31), so it
/// crosses without conversion (ZKM_REPR_MONTGOMERY), as the reference's own row ABI passes it
/// (crates/core/machine/src/sys.rs).
fn matrix(name: &CString, m: &RowMajorMatrix<KoalaBear>) -> zkm_matrix_t {
    zkm_matrix_t {
        name: name.as_ptr(),
        data: m.values.as_ptr() as *const u32,
        height: m.height() as u64,
        width: m.width() as u64,
        repr: ZKM_REPR_MONTGOMERY,
    }
}

fn to_abi(ch: &Challenger) -> zkm_challenger_t {
    let mut c = zkm_challenger_t::default();
    for (i, x) in ch.sponge_state.iter().enumerate() {
        c.sponge_state[i] = x.as_canonical_u32();
    }
    c.num_inputs = ch.input_buffer.len() as u32;
    for (i, x) in ch.input_buffer.iter().enumerate() {
        c.input_buffer[i] = x.as_canonical_u32();
    }
    c.num_outputs = ch.output_buffer.len() as u32;
    for (i, x) in ch.output_buffer.iter().enumerate() {
        c.output_buffer[i] = x.as_canonical_u32();
    }
    c
}

fn from_abi(c: &zkm_challenger_t, ch: &mut Challenger) {
    for i in 0..16 {
        ch.sponge_state[i] = KoalaBear::from_canonical_u32(c.sponge_state[i]);
    }
    ch.input_buffer = c.input_buffer[..c.num_inputs as usize].iter().map(|&x| KoalaBear::from_canonical_u32(x)).collect();
    ch.output_buffer =
        c.output_buffer[..c.num_outputs as usize].iter().map(|&x| KoalaBear::from_canonical_u32(x)).collect();
}

impl<A> HipProver<A>
where
    A: MachineAir<KoalaBear> + for<'a> p3_air::Air<p3_uni_stark::SymbolicAirBuilder<KoalaBear>>,
{
    /// Device `device` (one prover per GPU; deal shards round-robin for several).
    pub fn on_device(machine: StarkMachine<SC, A>, device: i32) -> Result<Self, HipProverError> {
        let mut ctx = ptr::null_mut();
        check(unsafe { zkm_init(device, &mut ctx) }, "zkm_init")?;
        let blob = machine_blob(&machine);
        // FRI parameters of the machine's config (kb31_poseidon2.rs:203-227): 84 queries, 16 PoW bits,
        // log_blowup 1 for the core, 2 for compressed_fri_config.
        let fri = machine.config().fri_config();
        let cfg = zkm_config_t {
            num_queries: fri.num_queries as u32,
            pow_bits: fri.proof_of_work_bits as u32,
            log_blowup: fri.log_blowup as u32,
            proof_montgomery: 0,
        };
        let mut layout = ptr::null_mut();
        check(unsafe { zkm_machine_new(blob.as_ptr(), blob.len(), &cfg, &mut layout) }, "zkm_machine_new")?;
        Ok(Self { machine, ctx: Ctx(ctx), blob, cfg, layout: MachineHandle(layout) })
    }

    fn device_pk(&self, program: &A::Program, host: StarkProvingKey<SC>) -> HipProvingKey {
        let prep: Vec<Option<RowMajorMatrix<KoalaBear>>> =
            self.machine.chips().iter().map(|c| c.generate_preprocessed_trace(program)).collect();
        self.upload_pk(prep, host)
    }

    /// The device key from the preprocessed traces in machine-chip order (None for chips without one).
    fn upload_pk(&self, prep: Vec<Option<RowMajorMatrix<KoalaBear>>>, host: StarkProvingKey<SC>) -> HipProvingKey {
        let chips = self.machine.chips();
        let names: Vec<CString> = chips.iter().map(|c| CString::new(c.name()).unwrap()).collect();
        let mats: Vec<zkm_matrix_t> = prep
            .iter()
            .zip(&names)
            .map(|(p, n)| match p {
                Some(m) => matrix(n, m),
                None => zkm_matrix_t { name: n.as_ptr(), data: ptr::null(), height: 0, width: 0, repr: 0 },
            })
            .collect();
        let gcs = digest_words(&host.initial_global_cumulative_sum);
        let mut pk = ptr::null_mut();
        let mut commit = [0u32; 8];
        let rc = unsafe {
            zkm_setup(
                self.ctx.0,
                self.blob.as_ptr(),
                self.blob.len(),
                &self.cfg,
                mats.as_ptr(),
                mats.len() as u32,
                host.pc_start.as_canonical_u32(),
                gcs.as_ptr(),
                &mut pk,
                commit.as_mut_ptr(),
            )
        };
        check(rc, "zkm_setup").expect("device setup");
        // the GPU's preprocessed commitment is the reference's (tests/test_gpu_prover.py pins it)
        let host_commit: [KoalaBear; 8] = host.commit.into();
        debug_assert_eq!(canonical(&host_commit), commit.to_vec());
        HipProvingKey(std::sync::Arc::new(PkInner { pk, host }))
    }
}

impl<A> MachineProver<SC, A> for HipProver<A>
where
    A: MachineAir<KoalaBear>
        + for<'a> p3_air::Air<p3_uni_stark::SymbolicAirBuilder<KoalaBear>>
        + for<'a> p3_air::Air<zkm_stark::ProverConstraintFolder<'a, SC>>
        + p3_air::Air<zkm_stark::lookup::LookupBuilder<KoalaBear>>
        + for<'a> p3_air::Air<zkm_stark::VerifierConstraintFolder<'a, SC>>,
    A::Record: MachineRecord,
{
    type DeviceMatrix = RowMajorMatrix<KoalaBear>;
    type DeviceProverData = HipMainData;
    type DeviceProvingKey = HipProvingKey;
    type Error = HipProverError;

    fn new(machine: StarkMachine<SC, A>) -> Self {
        Self::on_device(machine, 0).expect("no usable MI355X (gfx950) device")
    }

    fn machine(&self) -> &StarkMachine<SC, A> {
        &self.machine
    }

    fn setup(&self, program: &A::Program) -> (Self::DeviceProvingKey, StarkVerifyingKey<SC>) {
        let (pk, vk) = self.machine.setup(program);
        (self.device_pk(program, pk), vk)
    }

    fn pk_from_vk(&self, program: &A::Program, vk: &StarkVerifyingKey<SC>) -> Self::DeviceProvingKey {
        let (pk, _) = self.machine.setup_core(program, vk.initial_global_cumulative_sum);
        self.device_pk(program, pk)
    }

    fn pk_to_device(&self, pk: &StarkProvingKey<SC>) -> Self::DeviceProvingKey {
        // the host key's preprocessed traces are indexed by chip_ordering (machine.rs:383-403: sorted by
        // (height desc, name)); the ABI wants one slot per machine chip, in machine order
        let prep: Vec<Option<RowMajorMatrix<KoalaBear>>> = self
            .machine
            .chips()
            .iter()
            .map(|c| pk.chip_ordering.get(&c.name()).map(|&i| pk.traces[i].clone()))
            .collect();
        self.upload_pk(prep, pk.clone())
    }

    fn pk_to_host(&self, pk: &Self::DeviceProvingKey) -> StarkProvingKey<SC> {
        pk.0.host.clone()
    }

    fn commit(
        &self,
        record: &A::Record,
        traces: Vec<(String, RowMajorMatrix<KoalaBear>)>,
    ) -> ShardMainData<SC, Self::DeviceMatrix, Self::DeviceProverData> {
        // key-free: the machine layout is all commit reads; open checks it against the key's machine
        self.commit_layout(record, traces).expect("zkm_commit_machine")
    }

    fn open(
        &self,
        pk: &Self::DeviceProvingKey,
        mut data: ShardMainData<SC, Self::DeviceMatrix, Self::DeviceProverData>,
        challenger: &mut Challenger,
    ) -> Result<ShardProof<SC>, Self::Error> {
        let mut ch = to_abi(challenger);
        let mut out: *mut u8 = ptr::null_mut();
        let mut len = 0u64;
        let main = std::mem::replace(&mut data.main_data.0, ptr::null_mut());  // consumed by zkm_open
        check(unsafe { zkm_open(self.ctx.0, pk.0.pk, main, &mut ch, &mut out, &mut len) }, "zkm_open")?;
        let bytes = unsafe { std::slice::from_raw_parts(out, len as usize) }.to_vec();
        unsafe { zkm_free_bytes(out) };
        from_abi(&ch, challenger);
        bincode::deserialize(&bytes).map_err(|e| HipProverError(format!("proof bytes: {e}")))
    }

    fn prove(
        &self,
        pk: &Self::DeviceProvingKey,
        mut records: Vec<A::Record>,
        challenger: &mut Challenger,
        opts: <A::Record as MachineRecord>::Config,
    ) -> Result<MachineProof<SC>, Self::Error>
    where
        A: for<'a> p3_air::Air<zkm_stark::DebugConstraintBuilder<'a, KoalaBear, <SC as StarkGenericConfig>::Challenge>>,
    {
        self.machine
            .generate_dependencies(&mut records, &opts, None)
            .map_err(|_| HipProverError("generate_dependencies".into()))?;
        pk.observe_into(challenger);
        let mut shard_proofs = Vec::with_capacity(records.len());
        for record in records {
            let traces = self.generate_traces(&record).map_err(|_| HipProverError("generate_traces".into()))?;
            let data = self.commit_layout(&record, traces)?;
            shard_proofs.push(self.open(pk, data, &mut challenger.clone())?);
        }
        Ok(MachineProof { shard_proofs })
    }
}

impl<A> HipProver<A>
where
    A: MachineAir<KoalaBear>,
    A::Record: MachineRecord,
{
    /// MachineProver::commit with the device key (zkm_commit needs the machine layout it holds).
    pub fn commit_layout(
        &self,
        record: &A::Record,
        traces: Vec<(String, RowMajorMatrix<KoalaBear>)>,
    ) -> Result<ShardMainData<SC, RowMajorMatrix<KoalaBear>, HipMainData>, HipProverError> {
        let names: Vec<CString> = traces.iter().map(|(n, _)| CString::new(n.as_str()).unwrap()).collect();
        let mats: Vec<zkm_matrix_t> = traces.iter().zip(&names).map(|((_, m), n)| matrix(n, m)).collect();
        let pv = canonical(&record.public_values::<KoalaBear>());
        let mut main = ptr::null_mut();
        let mut root = [0u32; 8];
        check(
            unsafe {
                zkm_commit_machine(self.ctx.0, self.layout.0, mats.as_ptr(), mats.len() as u32, pv.as_ptr(),
                                   pv.len() as u32, &mut main, root.as_mut_ptr())
            },
            "zkm_commit_machine",
        )?;
        // chip ordering as prover.rs:262-285 builds it: (height desc, name)
        let mut order: Vec<(usize, &String)> = traces.iter().map(|(n, m)| (m.height(), n)).collect();
        order.sort_by(|a, b| b.0.cmp(&a.0).then(a.1.cmp(b.1)));
        let chip_ordering: HashMap<String, usize> =
            order.iter().enumerate().map(|(i, (_, n))| ((*n).clone(), i)).collect();
        let words: [KoalaBear; 8] = root.map(KoalaBear::from_canonical_u32);
        Ok(ShardMainData {
            traces: traces.into_iter().map(|(_, m)| m).collect(),
            main_commit: words.into(),
            main_data: HipMainData(main),
            chip_ordering,
            public_values: record.public_values::<KoalaBear>(),
        })
    }
}
