"""Builds libpdp_hip.so in-tree for gfx950 (``python -m pipelinedp_amd.build``).

``--debug-build`` builds variants/libpdp_hip_debug.so with -DPDP_DEBUG_BUILD
instead: the experiment library that honours the PDP_* environment knobs and
the timing-ablation debug flags (load it with PDP_HIP_LIB=...).  The shipped
library reads no environment.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "pdp_kernels.hip")
OUT = os.path.join(HERE, "libpdp_hip.so")
DEBUG_OUT = os.path.join(ROOT, "variants", "libpdp_hip_debug.so")
CSRC = os.path.join(HERE, "csrc")
DEPS = [os.path.join(CSRC, f) for f in sorted(os.listdir(CSRC))] + [os.path.join(ROOT, "include", "pdp_hip.h")]


def build(force: bool = False, verbose: bool = True, debug: bool = False) -> str:
    out = DEBUG_OUT if debug else OUT
    if not force and os.path.exists(out) and all(os.path.getmtime(out) >= os.path.getmtime(d) for d in DEPS):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    cmd = [hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-I" + os.path.join(ROOT, "include"), "-o", out + ".tmp", SRC]
    if debug:
        cmd.insert(1, "-DPDP_DEBUG_BUILD")
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv, debug="--debug-build" in sys.argv)
