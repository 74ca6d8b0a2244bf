"""Build libldpc5g.so (gfx950) in-tree with hipcc.

    python -m python_5gtoolbox_amd.build [--force]

The shared library lands next to this file so it travels with the repo snapshot to the GPU box.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(ROOT, "include")
LIB = os.path.join(HERE, "libldpc5g.so")
SOURCES = [os.path.join(CSRC, "ldpc5g.hip")]
DEPS = SOURCES + [os.path.join(CSRC, "ldpc5g_tables.h"), os.path.join(INCLUDE, "ldpc5g.h")]
ARCH = os.environ.get("LDPC5G_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def cmd(out=LIB):
    return [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC",
            "-shared", "-Wno-unused-result", f"-I{INCLUDE}", f"-I{CSRC}", *SOURCES, "-o", out]


def up_to_date():
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(d) <= t for d in DEPS)


def build(force=False, verbose=True):
    if not force and up_to_date():
        if verbose:
            print("libldpc5g.so up to date")
        return LIB
    c = cmd(LIB + ".tmp")
    if verbose:
        print(" ".join(c), flush=True)
    subprocess.run(c, check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
