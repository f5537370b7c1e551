//! Device trace generation for the chips the reference exposes a native row ABI for
//! (crates/core/machine/src/sys.rs:14-42) plus the Global chip: the shard's event vectors are copied
//! to the GPU once and each chip's whole padded trace is filled there (include/zkm_tracegen.h),
//! then handed to `zkm_commit` as a ZKM_MEM_DEVICE matrix without coming back to the host.
//!
//! Replaces, per chip, the body of `generate_trace` (cpu/trace.rs:43-76, alu/add_sub/mod.rs:82-110,
//! memory/local.rs:144-185, syscall/chip.rs:138-183, global/mod.rs:110-196); the Byte chip's
//! multiplicities those chips add in `generate_dependencies` are accumulated on the device into the
//! Byte trace, so the host's Byte trace must leave these chips' lookups out.
use std::os::raw::{c_int, c_void};
use std::ptr;

use zkm_core_executor::events::{AluEvent, CpuEvent, CpuEventFfi, GlobalLookupEvent, MemoryLocalEvent};
use zkm_core_executor::{InstructionFfi, Program};

use crate::prover::HipProverError;
use crate::sys::*;

#[link(name = "amdhip64")]
extern "C" {
    fn hipMalloc(p: *mut *mut c_void, bytes: usize) -> c_int;
    fn hipFree(p: *mut c_void) -> c_int;
    fn hipMemcpy(dst: *mut c_void, src: *const c_void, bytes: usize, kind: c_int) -> c_int;
    fn hipMemset(p: *mut c_void, v: c_int, bytes: usize) -> c_int;
}
const H2D: c_int = 1;

/// A GPU buffer (freed on drop).
pub struct DeviceBuf {
    pub ptr: *mut c_void,
    pub bytes: usize,
}
unsafe impl Send for DeviceBuf {}
impl Drop for DeviceBuf {
    fn drop(&mut self) {
        unsafe { hipFree(self.ptr) };
    }
}

fn alloc(bytes: usize) -> Result<DeviceBuf, HipProverError> {
    let mut p = ptr::null_mut();
    if unsafe { hipMalloc(&mut p, bytes.max(4)) } != 0 {
        return Err(HipProverError(format!("hipMalloc({bytes})")));
    }
    Ok(DeviceBuf { ptr: p, bytes })
}

fn upload<T: Copy>(v: &[T]) -> Result<DeviceBuf, HipProverError> {
    let bytes = std::mem::size_of_val(v);
    let b = alloc(bytes)?;
    if bytes > 0 && unsafe { hipMemcpy(b.ptr, v.as_ptr() as *const c_void, bytes, H2D) } != 0 {
        return Err(HipProverError("hipMemcpy".into()));
    }
    Ok(b)
}

/// A chip's trace resident in HBM (canonical row-major u32), ready for commit as ZKM_MEM_DEVICE.
pub struct DeviceTrace {
    pub name: String,
    pub buf: DeviceBuf,
    pub height: usize,
    pub width: usize,
}

impl DeviceTrace {
    pub fn matrix(&self, name: &std::ffi::CString) -> zkm_matrix_t {
        zkm_matrix_t {
            name: name.as_ptr(),
            data: self.buf.ptr as *const u32,
            height: self.height as u64,
            width: self.width as u64,
            repr: ZKM_REPR_CANONICAL | ZKM_MEM_DEVICE,
        }
    }
}

fn height_for(n: usize) -> usize {
    n.next_power_of_two().max(16)
}

fn rc(r: c_int, what: &str) -> Result<(), HipProverError> {
    if r == ZKM_OK {
        Ok(())
    } else {
        Err(HipProverError(format!("{what} failed ({r}): {}", last_error())))
    }
}

/// The Byte chip's multiplicity trace (65536 x 10), zeroed, for the chips below to add into.
pub fn byte_multiplicities() -> Result<DeviceTrace, HipProverError> {
    let bytes = 65536 * 10 * 4;
    let buf = alloc(bytes)?;
    unsafe { hipMemset(buf.ptr, 0, bytes) };
    Ok(DeviceTrace { name: "Byte".into(), buf, height: 65536, width: 10 })
}

/// CpuChip::generate_trace on the GPU, the Program chip's multiplicities alongside.
pub fn cpu_trace(
    events: &[CpuEvent],
    program: &Program,
    shard: u32,
    byte_mult: &DeviceTrace,
) -> Result<(DeviceTrace, DeviceBuf), HipProverError> {
    let ffi: Vec<CpuEventFfi> = events.iter().map(CpuEventFfi::from).collect();
    let ins: Vec<InstructionFfi> = program.instructions.iter().map(|i| InstructionFfi::from(*i)).collect();
    let (d_ev, d_prog) = (upload(&ffi)?, upload(&ins)?);
    let height = height_for(events.len());
    let out = alloc(height * 67 * 4)?;
    let prog_mult = alloc(ins.len() * 4)?;
    unsafe { hipMemset(prog_mult.ptr, 0, ins.len() * 4) };
    rc(
        unsafe {
            zkm_cpu_events_to_trace(d_ev.ptr as _, ffi.len() as u64, shard, d_prog.ptr as _, ins.len() as u64,
                                    program.pc_base, out.ptr as _, height as u64, byte_mult.buf.ptr as _,
                                    prog_mult.ptr as _, ptr::null_mut())
        },
        "zkm_cpu_events_to_trace",
    )?;
    Ok((DeviceTrace { name: "Cpu".into(), buf: out, height, width: 67 }, prog_mult))
}

/// AddSubChip::generate_trace on the GPU.
pub fn add_sub_trace(events: &[AluEvent], byte_mult: &DeviceTrace) -> Result<DeviceTrace, HipProverError> {
    let d_ev = upload(events)?;
    let height = height_for(events.len());
    let out = alloc(height * 19 * 4)?;
    rc(
        unsafe {
            zkm_add_sub_events_to_trace(d_ev.ptr as _, events.len() as u64, out.ptr as _, height as u64,
                                        byte_mult.buf.ptr as _, ptr::null_mut())
        },
        "zkm_add_sub_events_to_trace",
    )?;
    Ok(DeviceTrace { name: "AddSub".into(), buf: out, height, width: 19 })
}

/// MemoryLocalChip::generate_trace on the GPU (four entries per row).
pub fn memory_local_trace(events: &[MemoryLocalEvent]) -> Result<DeviceTrace, HipProverError> {
    let d_ev = upload(events)?;
    let height = height_for(events.len().div_ceil(4));
    let out = alloc(height * 56 * 4)?;
    rc(
        unsafe {
            zkm_memory_local_events_to_trace(d_ev.ptr as _, events.len() as u64, out.ptr as _, height as u64,
                                             ptr::null_mut())
        },
        "zkm_memory_local_events_to_trace",
    )?;
    Ok(DeviceTrace { name: "MemoryLocal".into(), buf: out, height, width: 56 })
}

/// GlobalChip::generate_trace on the GPU; returns the trace and the shard's global cumulative sum.
pub fn global_trace(
    events: &[GlobalLookupEvent],
    byte_mult: &DeviceTrace,
) -> Result<(DeviceTrace, [u32; 14]), HipProverError> {
    let d_ev = upload(events)?;
    let height = height_for(events.len());
    let out = alloc(height * 99 * 4)?;
    let fin = alloc(14 * 4)?;
    rc(
        unsafe {
            zkm_global_events_to_trace(d_ev.ptr as _, events.len() as u64, out.ptr as _, height as u64,
                                       byte_mult.buf.ptr as _, fin.ptr as _, ptr::null_mut())
        },
        "zkm_global_events_to_trace",
    )?;
    let mut digest = [0u32; 14];
    unsafe { hipMemcpy(digest.as_mut_ptr() as _, fin.ptr, 56, 2) };
    Ok((DeviceTrace { name: "Global".into(), buf: out, height, width: 99 }, digest))
}
