//! Raw bindings of include/zkm_hip.h and include/zkm_tracegen.h.  Every struct is `#[repr(C)]` with
//! the header's field order; the trace-generation records are the executor's own `#[repr(C)]` event
//! types, so they are passed straight through (see `tracegen.rs`).
#![allow(non_camel_case_types)]
use std::os::raw::{c_char, c_int, c_void};

use zkm_core_executor::events::{
    AluEvent, CpuEventFfi, GlobalLookupEvent, MemoryInitializeFinalizeEvent, MemoryLocalEvent, SyscallEvent,
};
use zkm_core_executor::InstructionFfi;

pub const ZKM_OK: c_int = 0;
pub const ZKM_ERR_ARG: c_int = -1;
pub const ZKM_ERR_HIP: c_int = -2;
pub const ZKM_ERR_UNSATISFIED: c_int = -3;
pub const ZKM_ERR_UNSUPPORTED: c_int = -4;
pub const ZKM_ERR_NO_DEVICE: c_int = -5;

pub const ZKM_REPR_CANONICAL: u32 = 0;
pub const ZKM_REPR_MONTGOMERY: u32 = 1;
pub const ZKM_MEM_DEVICE: u32 = 0x100;

#[repr(C)]
pub struct zkm_ctx {
    _p: [u8; 0],
}
#[repr(C)]
pub struct zkm_pk {
    _p: [u8; 0],
}
#[repr(C)]
pub struct zkm_main {
    _p: [u8; 0],
}
#[repr(C)]
pub struct zkm_machine {
    _p: [u8; 0],
}

#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct zkm_config_t {
    pub num_queries: u32,
    pub pow_bits: u32,
    pub log_blowup: u32,
    pub proof_montgomery: u32,
}

#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct zkm_challenger_t {
    pub sponge_state: [u32; 16],
    pub num_inputs: u32,
    pub input_buffer: [u32; 8],
    pub num_outputs: u32,
    pub output_buffer: [u32; 8],
}

#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct zkm_matrix_t {
    pub name: *const c_char,
    pub data: *const u32,
    pub height: u64,
    pub width: u64,
    pub repr: u32,
}

#[link(name = "zkm_hip")]
extern "C" {
    // ---- zkm_hip.h ----
    pub fn zkm_init(device: c_int, out: *mut *mut zkm_ctx) -> c_int;
    pub fn zkm_destroy(ctx: *mut zkm_ctx);
    pub fn zkm_last_error() -> *const c_char;
    pub fn zkm_device_count() -> c_int;
    pub fn zkm_host_alloc(bytes: usize, out: *mut *mut c_void) -> c_int;
    pub fn zkm_host_free(p: *mut c_void);
    pub fn zkm_setup(
        ctx: *mut zkm_ctx,
        machine_blob: *const u32,
        nwords: usize,
        cfg: *const zkm_config_t,
        prep: *const zkm_matrix_t,
        nprep: u32,
        pc_start: u32,
        initial_global_cumulative_sum: *const u32,
        pk_out: *mut *mut zkm_pk,
        commit_out: *mut u32,
    ) -> c_int;
    pub fn zkm_pk_free(pk: *mut zkm_pk);
    pub fn zkm_pk_observe(pk: *const zkm_pk, ch: *mut zkm_challenger_t) -> c_int;
    pub fn zkm_commit(
        ctx: *mut zkm_ctx,
        pk: *const zkm_pk,
        traces: *const zkm_matrix_t,
        ntraces: u32,
        public_values: *const u32,
        npv: u32,
        main_out: *mut *mut zkm_main,
        main_commit_out: *mut u32,
    ) -> c_int;
    pub fn zkm_main_free(main: *mut zkm_main);
    pub fn zkm_machine_new(blob: *const u32, nwords: usize, cfg: *const zkm_config_t, out: *mut *mut zkm_machine)
        -> c_int;
    pub fn zkm_machine_free(m: *mut zkm_machine);
    pub fn zkm_commit_machine(
        ctx: *mut zkm_ctx,
        m: *const zkm_machine,
        traces: *const zkm_matrix_t,
        ntraces: u32,
        public_values: *const u32,
        npv: u32,
        main_out: *mut *mut zkm_main,
        main_commit_out: *mut u32,
    ) -> c_int;
    pub fn zkm_open(
        ctx: *mut zkm_ctx,
        pk: *const zkm_pk,
        main: *mut zkm_main,
        ch: *mut zkm_challenger_t,
        proof_out: *mut *mut u8,
        proof_len: *mut u64,
    ) -> c_int;
    pub fn zkm_free_bytes(p: *mut u8);
    pub fn zkm_quotient_jit_compile(blob: *const u32, nwords: usize, code_bytes: *mut u64) -> c_int;

    // ---- zkm_tracegen.h (device pointers; `stream` is a hipStream_t, null = the null stream) ----
    /// Poseidon2WideDeg3 main trace (recursion/core/src/sys.rs:102-106); `repr` 1 = Montgomery records.
    pub fn zkm_poseidon2_wide_events_to_trace(
        events: *const u32,
        n: u64,
        repr: u32,
        trace: *mut u32,
        height: u64,
        stream: *mut c_void,
    ) -> c_int;
    /// ExpReverseBitsLen main trace (recursion/core/src/sys.rs:50-54 plus the accumulator columns).
    pub fn zkm_exp_reverse_bits_events_to_trace(
        base: *const u32,
        bits: *const u32,
        offsets: *const u64,
        n: u64,
        repr: u32,
        trace: *mut u32,
        height: u64,
        stream: *mut c_void,
    ) -> c_int;
    pub fn zkm_cpu_events_to_trace(
        events: *const CpuEventFfi,
        n: u64,
        shard: u32,
        program: *const InstructionFfi,
        program_len: u64,
        pc_base: u32,
        trace: *mut u32,
        height: u64,
        byte_mult: *mut u32,
        program_mult: *mut u32,
        stream: *mut c_void,
    ) -> c_int;
    pub fn zkm_add_sub_events_to_trace(
        events: *const AluEvent,
        n: u64,
        trace: *mut u32,
        height: u64,
        byte_mult: *mut u32,
        stream: *mut c_void,
    ) -> c_int;
    pub fn zkm_memory_local_events_to_trace(
        events: *const MemoryLocalEvent,
        n: u64,
        trace: *mut u32,
        height: u64,
        stream: *mut c_void,
    ) -> c_int;
    pub fn zkm_memory_global_events_to_trace(
        events: *const MemoryInitializeFinalizeEvent,
        n: u64,
        is_receive: c_int,
        prev_addr: u32,
        trace: *mut u32,
        height: u64,
        stream: *mut c_void,
    ) -> c_int;
    pub fn zkm_syscall_events_to_trace(
        events: *const SyscallEvent,
        n: u64,
        is_receive: c_int,
        trace: *mut u32,
        height: u64,
        stream: *mut c_void,
    ) -> c_int;
    pub fn zkm_global_events_to_trace(
        events: *const GlobalLookupEvent,
        n: u64,
        trace: *mut u32,
        height: u64,
        byte_mult: *mut u32,
        final_digest: *mut u32,
        stream: *mut c_void,
    ) -> c_int;
}

/// The thread-local message of the last failing call.
pub fn last_error() -> String {
    unsafe {
        let p = zkm_last_error();
        if p.is_null() {
            String::new()
        } else {
            std::ffi::CStr::from_ptr(p).to_string_lossy().into_owned()
        }
    }
}
