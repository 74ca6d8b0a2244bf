"""Build libldpc5g.so (gfx950) in-tree with hipcc.

    python -m python_5gtoolbox_amd.build [--force]

Each csrc/*.hip translation unit is compiled to an object in parallel, then linked into
python_5gtoolbox_amd/libldpc5g.so, which travels with the repo snapshot to the GPU box.
"""
import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(ROOT, "include")
OBJ = os.path.join(ROOT, "build", "obj")
LIB = os.path.join(HERE, "libldpc5g.so")
ARCH = os.environ.get("LDPC5G_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC",
         "-Wno-unused-result", f"-I{INCLUDE}", f"-I{CSRC}"]


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def deps():
    return sources() + glob.glob(os.path.join(CSRC, "*.h")) + [os.path.join(INCLUDE, "ldpc5g.h")]


def up_to_date():
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(d) <= t for d in deps())


def _compile(src, verbose):
    obj = os.path.join(OBJ, os.path.basename(src) + ".o")
    cmd = [HIPCC, *FLAGS, "-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return obj


def build(force=False, verbose=True):
    if not force and up_to_date():
        if verbose:
            print("libldpc5g.so up to date")
        return LIB
    os.makedirs(OBJ, exist_ok=True)
    srcs = sources()
    with ThreadPoolExecutor(max_workers=min(len(srcs), 8)) as ex:
        objs = list(ex.map(lambda s: _compile(s, verbose), srcs))
    link = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", LIB + ".tmp"]
    if verbose:
        print(" ".join(link), flush=True)
    subprocess.run(link, check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
