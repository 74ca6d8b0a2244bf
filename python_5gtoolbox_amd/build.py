"""Build libldpc5g.so (gfx950) in-tree with hipcc.

    python -m python_5gtoolbox_amd.build [--force] [--csrc DIR --out LIB]

(--csrc/--out build an alternative source tree into another library, for A/B timing on one GPU
box via LDPC5G_LIB=...; the default build is the in-tree one.)

Each csrc/*.hip translation unit is compiled to an object in parallel, then linked into
python_5gtoolbox_amd/libldpc5g.so, which travels with the repo snapshot to the GPU box.
"""
import glob
import hashlib
import json
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

# v_pk_add_f32 issues at ~1/3 the rate of two scalar v_add_f32 on gfx950 (tools/microbench/valu_rates.hip),
# so the layered decoder TU is built without the SLP vectorizer that forms it (the flooding TU keeps
# it: there the packed adds measure faster).
NO_SLP = {"ldpc5g_dec_l.hip", "ldpc5g_dec_l_dead.hip"}


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def deps():
    return sources() + glob.glob(os.path.join(CSRC, "*.h")) + [os.path.join(INCLUDE, "ldpc5g.h")]


def _digest(paths):
    """{path: sha1 of its contents} (missing files map to None)."""
    out = {}
    for p in paths:
        try:
            with open(p, "rb") as f:
                out[os.path.abspath(p)] = hashlib.sha1(f.read()).hexdigest()
        except OSError:
            out[os.path.abspath(p)] = None
    return out


def _stamp(dig=None):
    """Everything that decides the library's code: flags and arch (a library built with other
    flags or for another arch — an A/B build into the default path — is never reused as the
    product) and the contents of every source, as they were when the build STARTED (a source
    edited while the build ran leaves the library stale, not falsely up to date)."""
    dig = dig if dig is not None else _digest(deps())
    return " ".join([HIPCC, ARCH, *FLAGS, os.environ.get("LDPC5G_EXTRA_FLAGS", ""),
                     os.environ.get("LDPC5G_SLP", ""), *sorted(NO_SLP)]) + "\n" + \
        json.dumps(sorted((os.path.relpath(k, ROOT), v) for k, v in dig.items()))


def up_to_date():
    if not os.path.exists(LIB):
        return False
    try:
        with open(LIB + ".stamp") as f:
            return f.read() == _stamp()
    except OSError:
        return False


def _obj_fresh(obj, cmd):
    """The object exists, was built by exactly `cmd`, and every file its dependency list (hipcc
    -MMD) names still has the contents it had when that compile started (.dig)."""
    try:
        with open(obj + ".cmd") as f:
            if f.read() != " ".join(cmd):
                return False
        with open(obj + ".dig") as f:
            rec = json.load(f)
    except (OSError, ValueError):
        return False
    return bool(rec) and _digest(rec) == rec


def _compile(src, verbose, obj_dir=None, csrc=CSRC):
    obj = os.path.join(obj_dir or OBJ, os.path.basename(src) + ".o")
    flags = [f for f in FLAGS if f != f"-I{CSRC}"] + [f"-I{csrc}"]
    flags += os.environ.get("LDPC5G_EXTRA_FLAGS", "").split()   # A/B builds (-D...)
    if os.path.basename(src) in NO_SLP and not os.environ.get("LDPC5G_SLP"):
        flags.append("-fno-slp-vectorize")
    cmd = [HIPCC, *flags, "-c", src, "-o", obj]
    if _obj_fresh(obj, cmd):   # incremental: only translation units whose inputs changed
        return obj
    if verbose:
        print(" ".join(cmd), flush=True)
    _compile_recorded(cmd, obj)
    return obj


def _compile_recorded(cmd, obj):
    """Run one compile and record its command and the contents of its dependencies as they
    were when it started (every candidate file is hashed first; the -MMD list picks them)."""
    before = _digest(deps())
    subprocess.run(cmd + ["-MMD", "-MF", obj + ".d"], check=True)
    with open(obj + ".d") as f:
        text = f.read().replace("\\\n", " ")
    dl = text.split(":", 1)[1].split() if ":" in text else []
    rec = {}
    for d in dl:
        a = os.path.abspath(d)
        rec[a] = before[a] if a in before else _digest([a])[a]
    with open(obj + ".dig", "w") as f:
        json.dump(rec, f)
    with open(obj + ".cmd", "w") as f:
        f.write(" ".join(cmd))


def build(force=False, verbose=True, csrc=None, out=None):
    alt = csrc is not None or out is not None
    lib_path = out or LIB
    if not alt and not force and up_to_date():
        if verbose:
            print("libldpc5g.so up to date")
        return LIB
    stamp = _stamp()   # the sources as they are now: an edit during the build is not covered
    csrc = csrc or CSRC
    obj_dir = os.path.join(ROOT, "build", ("obj_alt_" + os.path.basename(lib_path)) if alt else "obj")
    os.makedirs(obj_dir, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(csrc, "*.hip")))
    with ThreadPoolExecutor(max_workers=min(len(srcs), 8)) as ex:
        objs = list(ex.map(lambda s: _compile(s, verbose, obj_dir, csrc), srcs))
    link = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", lib_path + ".tmp"]
    if verbose:
        print(" ".join(link), flush=True)
    subprocess.run(link, check=True)
    os.replace(lib_path + ".tmp", lib_path)
    if not alt:
        with open(LIB + ".stamp", "w") as f:
            f.write(stamp)
    return lib_path


ASAN_LIB = os.path.join(ROOT, "build", "asan", "libldpc5g.so")


def asan_runtime():
    """The clang ASan runtime a non-instrumented interpreter must preload to load ASAN_LIB."""
    res = subprocess.run([HIPCC, "--print-file-name=libclang_rt.asan-x86_64.so"], capture_output=True,
                         text=True)
    p = res.stdout.strip()
    if not os.path.isabs(p):   # older drivers: search the resource directory
        rd = subprocess.run([HIPCC, "-print-resource-dir"], capture_output=True, text=True).stdout.strip()
        p = os.path.join(rd, "lib", "linux", "libclang_rt.asan-x86_64.so")
    return p


ASAN_SAN = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
            "-Xarch_host", "-fno-sanitize-recover=undefined", "-Xarch_host", "-fno-omit-frame-pointer"]


def _asan_stamp():
    return " ".join([HIPCC, ARCH, *FLAGS, *ASAN_SAN, *sorted(NO_SLP)]) + "\n" + \
        json.dumps(sorted((os.path.relpath(k, ROOT), v) for k, v in _digest(deps()).items()))


def build_asan(force=False, verbose=False):
    """Host-code sanitizer build: every TU's HOST code compiled with
    AddressSanitizer + UndefinedBehaviorSanitizer (-Xarch_host: the device code is the normal
    gfx950 build, which the host registration code needs), into build/asan/libldpc5g.so, per
    translation unit incrementally like build().  It backs the CPU suite's validation /
    plan-building / configuration tests (tests/test_asan_host.py), which exercise exactly the
    C-ABI host code: argument checks, ldpc5g_sch_config, the mixed-Zc and per-TB plans.  Built
    lazily by that test, not by the product build()."""
    out_dir = os.path.dirname(ASAN_LIB)
    stamp = ASAN_LIB + ".stamp"
    want = _asan_stamp()   # the sources as they are when the build starts
    try:
        with open(stamp) as f:
            same = f.read() == want
    except OSError:
        same = False
    if not force and same and os.path.exists(ASAN_LIB):
        return ASAN_LIB
    os.makedirs(out_dir, exist_ok=True)
    san = list(ASAN_SAN)
    base = list(FLAGS)

    def one(src):
        obj = os.path.join(out_dir, os.path.basename(src) + ".o")
        cmd = [HIPCC, *base, *san, "-c", src, "-o", obj]
        if os.path.basename(src) in NO_SLP:
            cmd.insert(1, "-fno-slp-vectorize")
        if not force and _obj_fresh(obj, cmd):
            return obj
        if verbose:
            print(" ".join(cmd), flush=True)
        _compile_recorded(cmd, obj)
        return obj
    srcs = sources()
    with ThreadPoolExecutor(max_workers=min(len(srcs), 8)) as ex:
        objs = list(ex.map(one, srcs))
    link = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-Xarch_host", "-fsanitize=address", "-Xarch_host",
            "-fsanitize=undefined", "-shared-libasan", *objs, "-o", ASAN_LIB + ".tmp"]
    if verbose:
        print(" ".join(link), flush=True)
    subprocess.run(link, check=True)
    os.replace(ASAN_LIB + ".tmp", ASAN_LIB)
    with open(stamp, "w") as f:
        f.write(want)
    return ASAN_LIB


def _arg(name):
    return sys.argv[sys.argv.index(name) + 1] if name in sys.argv else None


if __name__ == "__main__":
    if "--asan" in sys.argv:
        print(build_asan(force="--force" in sys.argv, verbose=True))
    else:
        build(force="--force" in sys.argv, csrc=_arg("--csrc"), out=_arg("--out"))
