"""LDE microbench A/B of two library builds (ZKM_LIB=zkmips_amd/libzkm_hip_a.so is A, the in-tree build B),
alternated in fresh processes: ms per LDE of 2^L x W (zkm_bench_lde) for the heights given.
python tools/gpu/r06_lde_ab.py [rounds]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CHILD = ("import sys; sys.path.insert(0, %r); from zkmips_amd._lib import Device; d = Device(0); "
         "print(' '.join('%%.4f' %% d.bench_lde(1 << L, W, 20) for L, W in [(22, 67), (22, 44), (23, 64), (21, 67), (20, 67)]))"
         % ROOT)
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
print("cols: 2^22x67 2^22x44 2^23x64 2^21x67 2^20x67 (ms)")
for r in range(rounds):
    for v in ("A", "B"):
        env = dict(os.environ)
        if v == "A":
            env["ZKM_LIB"] = os.path.join(ROOT, "zkmips_amd", "libzkm_hip_a.so")
        else:
            env.pop("ZKM_LIB", None)
        out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        if out.returncode:
            print(v, "failed", out.stderr[-2000:])
            sys.exit(1)
        print(v, r, out.stdout.strip(), flush=True)
