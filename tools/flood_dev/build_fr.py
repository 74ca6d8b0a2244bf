"""Build variants of the float64 frame kernel (ldpc5g_dec_frame.h) for side-by-side timing with
tools/flood_dev/run_dev.py (development tool, not product).

    python tools/flood_dev/build_fr.py NAME[:FLAG,FLAG...] ...

NAME is a key of PATCHES (string patches applied to a copy of csrc/) or any other name (no patch);
the optional FLAGs are -D definitions (e.g. v:LDPC5G_FR_PIPE=1).  Output: build/frdev/NAME.so.
"""
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "python_5gtoolbox_amd", "csrc")
HERE = os.path.dirname(os.path.abspath(__file__))
FR = "ldpc5g_dec_frame.h"

PATCHES = {
    # timing splits (wrong results)
    "noB": [("        if constexpr (LDPC5G_FR_PIPE) {", "        if constexpr (false) {"),
            ("                per_half([&](auto hc) {\n                    constexpr int H = decltype(hc)::value;\n"
             "                    sfor<kFrPlan<BG>.gstart[g], kFrPlan<BG>.gstart[g + 1]>([&](auto ic) {\n"
             "                        constexpr int i = decltype(ic)::value, e0 = P::RS[i], d = kFrPlan<BG>.deg(i);\n"
             "                        if constexpr (kFrPlan<BG>.lds[i]) {",
             "                per_half([&](auto hc) {\n                    constexpr int H = decltype(hc)::value;\n"
             "                    sfor<kFrPlan<BG>.gstart[g], kFrPlan<BG>.gstart[g + 1]>([&](auto ic) {\n"
             "                        constexpr int i = decltype(ic)::value, e0 = P::RS[i], d = kFrPlan<BG>.deg(i);\n"
             "                        if constexpr (false) {"),
            ("                        } else if constexpr (kFrPlan<BG>.owner[i] == H) {\n                            T a, b;",
             "                        } else if constexpr (false) {\n                            T a, b;")],
    "nobar": [("            lds_barrier();\n        });\n        }\n", "        });\n        }\n")],
    "plain": [("            else __hip_atomic_fetch_add(&acc, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);",
               "            else acc = r;")],
    # DEAD kernel probe: the prologue's liveness loads kept, the plain iterations always
    "onlyplain": [("        if (live_x != all) {", "        if (live_x == 12345) {")],
}


def make(spec):
    name, _, flags = spec.partition(":")
    d = os.path.join(ROOT, "build", "frv", name)
    shutil.rmtree(d, ignore_errors=True)
    shutil.copytree(CSRC, d)
    p = os.path.join(d, FR)
    s = open(p).read()
    for old, new in PATCHES.get(name.split("+")[0], []):
        assert old in s, (name, old[:80])
        s = s.replace(old, new)
    open(p, "w").write(s)
    out = os.path.join(ROOT, "build", "frdev", name + ".so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC",
           "-shared", f"-I{ROOT}/include", f"-I{d}", *[f"-D{f}" for f in flags.split(",") if f],
           "-Rpass-analysis=kernel-resource-usage", os.path.join(HERE, "frdev.hip"), "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True)
    res = [ln.split("remark:")[-1].strip() for ln in r.stderr.splitlines()
           if "VGPRs:" in ln or "ScratchSize" in ln]
    return name, r.returncode, (r.stderr[-3000:] if r.returncode else " ".join(x.replace(" [-Rpass-analysis=kernel-resource-usage]", "") for x in res))


if __name__ == "__main__":
    specs = sys.argv[1:]
    with ThreadPoolExecutor(min(6, len(specs))) as ex:
        for name, rc, msg in ex.map(make, specs):
            print(name, "rc", rc, msg)
