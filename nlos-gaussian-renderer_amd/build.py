"""Build the C-ABI HIP library in-tree: nlosgr/libnlosgr.so (gfx950 only).

    python nlos-gaussian-renderer_amd/build.py [--force] [--save-temps]

The library links only the HIP runtime (no torch).  At run time Python loads it with ctypes
after torch, so it binds to the libamdhip64.so.7 torch already loaded.
"""
import argparse
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "nlosgr", "libnlosgr.so")
ARCH = "gfx950"


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def deps():
    return sources() + sorted(glob.glob(os.path.join(CSRC, "*.hpp"))) + [os.path.join(ROOT, "include", "nlosgr.h")]


def needs_build():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(d) > t for d in deps())


def build(force=False, save_temps=False, verbose=True, out=None, defines=()):
    """out/defines: alternative in-tree builds for A/B timing (NLOSGR_LIB selects one at run time)."""
    out = out or OUT
    if out == OUT and not defines and not force and not needs_build():
        return OUT
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    # no SLP / loop vectorisation: packed-f32 VALU needs aligned register pairs, which raised the
    # backward kernel's VGPR count past the 3-waves/SIMD limit (measured: bwd 736 -> 701 ms at C3)
    cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-munsafe-fp-atomics", "-fno-slp-vectorize", "-fno-vectorize", "-fvisibility=hidden",
           "-I", os.path.join(ROOT, "include"), "-o", out + ".tmp"] + [f"-D{d}" for d in defines]
    if save_temps:
        cmd += ["-save-temps"]
    cmd += sources()
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True, cwd=os.path.join(HERE, "csrc") if save_temps else None)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--save-temps", action="store_true")
    ap.add_argument("--out", default=None, help="alternative output path (A/B builds)")
    ap.add_argument("-D", dest="defines", action="append", default=[], help="preprocessor define")
    a = ap.parse_args()
    print(build(force=a.force, save_temps=a.save_temps, out=a.out, defines=a.defines))
