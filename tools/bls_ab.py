"""A/B of BLS wave-program variants on the GPU box: tools/bls_probe.py (wave form, with the
kernel's shader-clock breakdown) once per library.  usage: python tools/bls_ab.py LIB [LIB ...]
(LIB: a path such as varlib/lib_t6.so, or 'main' for the in-tree library)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for lib in sys.argv[1:]:
    env = dict(os.environ, EDV_BLS_WAVE_CLOCKS="1")
    if lib != "main":
        env["PLENUM_EDVERIFY_LIB"] = os.path.join(ROOT, lib)
    print("==", lib, flush=True)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "bls_probe.py"), "wave", "1", "25", "25", "1024"],
                       env=env, timeout=300)
    if r.returncode:
        sys.exit(r.returncode)
