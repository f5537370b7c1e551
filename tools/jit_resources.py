"""Resource usage of a JIT kernel source (ZKM_JIT_DUMP output) compiled with hiprtc as the library does:
VGPRs, spills and scratch per kernel, from the code object's AMDHSA metadata (no GPU needed).
python tools/jit_resources.py <chip>.hip [extra hiprtc options]"""
import ctypes
import re
import subprocess
import sys
import tempfile


def compile_co(src: bytes, opts):
    lib = ctypes.CDLL("/opt/rocm/lib/libhiprtc.so")
    prog = ctypes.c_void_p()
    assert lib.hiprtcCreateProgram(ctypes.byref(prog), src, b"quotient_jit.hip", 0, None, None) == 0
    o = [b"--offload-arch=gfx950", b"-O3", b"-std=c++17"] + [x.encode() for x in opts]
    arr = (ctypes.c_char_p * len(o))(*o)
    rc = lib.hiprtcCompileProgram(prog, len(o), arr)
    if rc:
        n = ctypes.c_size_t()
        lib.hiprtcGetProgramLogSize(prog, ctypes.byref(n))
        log = ctypes.create_string_buffer(n.value + 1)
        lib.hiprtcGetProgramLog(prog, log)
        raise SystemExit(log.value.decode()[:3000])
    n = ctypes.c_size_t()
    lib.hiprtcGetCodeSize(prog, ctypes.byref(n))
    buf = ctypes.create_string_buffer(n.value)
    lib.hiprtcGetCode(prog, buf)
    return buf.raw


def main():
    co = compile_co(open(sys.argv[1], "rb").read(), sys.argv[2:])
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(co)
        f.flush()
        notes = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", f.name], capture_output=True,
                               text=True).stdout
    for blk in notes.split("- .agpr_count")[1:]:
        name = re.search(r"\.name:\s+(\S+)", blk).group(1)
        get = lambda k: (re.search(rf"\.{k}:\s+(\S+)", blk) or [None, "?"])[1]
        print(f"{name:24s} vgpr {get('vgpr_count'):>4s} agpr {get('agpr_count') if 'agpr' in blk else '-':>3s} "
              f"vgpr_spill {get('vgpr_spill_count'):>4s} sgpr_spill {get('sgpr_spill_count'):>4s} "
              f"scratch {get('private_segment_fixed_size'):>6s} B")


if __name__ == "__main__":
    main()
