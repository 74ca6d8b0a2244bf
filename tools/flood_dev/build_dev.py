"""Build float64 flooding-kernel variants for side-by-side timing (development tool, not product).

    python tools/flood_dev/build_dev.py base noB nobar plain

Each variant: csrc/ copied to build/fdev/<name>/, string patches from VARIANTS applied to the
flooding header, tools/flood_dev/fdev.hip compiled against it into build/fdev/<name>.so.  A variant
named after a file tools/flood_dev/<name>.h uses that file as ldpc5g_dec_flood.h instead.
"""
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "python_5gtoolbox_amd", "csrc")
HERE = os.path.dirname(os.path.abspath(__file__))
FLOOD = "ldpc5g_dec_flood.h"

VARIANTS = {
    "base": [],
    # timing splits (wrong results)
    "noB": [("                        if constexpr (i < NLS) {   // LDS state: both halves, alternate edges",
             "                        if constexpr (i < 0) {"),
            ("                        } else if constexpr (kFloodPlan<BG, T, NP, CS>.owner[i] == decltype(hc)::value) {",
             "                        } else if constexpr (i < 0) {")],
    "nobar": [("            if (!gd) lds_barrier();\n        });", "        });")],
    "noX": [("                xr[p % XP] = llrx(kFloodPlan<BG, T, NP, CS>.xlist[hh][p]);",
             "                xr[p % XP] = T(1.5 + p);")],
    "plain": [("                        __hip_atomic_fetch_add(&acc, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);",
               "                        acc = r;")],
    # register-pressure probes of the gather phase B (compile only)
    "e_nolf": [("                        const T v = lf[x] + acc[x];", "                        const T v = acc[x];"),
               ("                                lf[x] = llr_core(j);", "")],
    "e_noadd": [("                                    acc[FP.cpos[j]] = acc[FP.cpos[j]] + r;",
                 "                                    asm volatile(\"\" :: \"v\"(r));")],
    "e_nowrite": [("                                    *(lds_V2*)(uintptr_t)(uint32_t)(so_b + so * 2 * TS) = v;", ""),
                  ("                                    *(lds_u32*)(uintptr_t)(uint32_t)(so_b + CS * 2 * TS + so * 4) = (u & 0xffffff00u) | x;", "")],
    "e_nogather": [("                                if constexpr (j < KC && FP.cown[j] == hh) {",
                    "                                if constexpr (j < 0) {")],
}


# compile-time flags per variant (the product header's LDPC5G_FLOOD_* knobs)
FLAGS = {
    "pre1": ["-DLDPC5G_FLOOD_APRE=1", "-DLDPC5G_FLOOD_ASB=0"],
    "pre2": ["-DLDPC5G_FLOOD_APRE=2", "-DLDPC5G_FLOOD_ASB=0"],
    "pre3": ["-DLDPC5G_FLOOD_APRE=3", "-DLDPC5G_FLOOD_ASB=0"],
    "pre1sb": ["-DLDPC5G_FLOOD_APRE=1", "-DLDPC5G_FLOOD_ASB=1"],
    "pre2sb": ["-DLDPC5G_FLOOD_APRE=2", "-DLDPC5G_FLOOD_ASB=1"],
    "pre3sb": ["-DLDPC5G_FLOOD_APRE=3", "-DLDPC5G_FLOOD_ASB=1"],
    "nosxpop": ["-DLDPC5G_FLOOD_SXPOP=0"],
    "x2": ["-DLDPC5G_FLOOD_XPRE=2"],
    "x6": ["-DLDPC5G_FLOOD_XPRE=6"],
    "x8": ["-DLDPC5G_FLOOD_XPRE=8"],
}
for _n in FLAGS:
    VARIANTS.setdefault(_n, [])


def make(name):
    d = os.path.join(ROOT, "build", "fdev", name)
    shutil.rmtree(d, ignore_errors=True)
    shutil.copytree(CSRC, d)
    alt = os.path.join(HERE, name + ".h")
    p = os.path.join(d, FLOOD)
    if os.path.exists(alt):
        shutil.copy(alt, p)
    else:
        s = open(p).read()
        for old, new in VARIANTS[name]:
            assert old in s, (name, old[:70])
            s = s.replace(old, new)
        open(p, "w").write(s)
    out = os.path.join(ROOT, "build", "fdev", name + ".so")
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC",
           "-shared", f"-I{ROOT}/include", f"-I{d}", "-DLDPC5G_FLOOD_FRAME=0", *os.environ.get("FDEV_FLAGS", "").split(), *FLAGS.get(name, []),
           os.path.join(HERE, "fdev.hip"), "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True)
    return name, r.returncode, r.stderr[-3000:]


if __name__ == "__main__":
    names = sys.argv[1:] or list(VARIANTS)
    with ThreadPoolExecutor(min(8, len(names))) as ex:
        for name, rc, err in ex.map(make, names):
            print(name, "rc", rc, err if rc else "")
