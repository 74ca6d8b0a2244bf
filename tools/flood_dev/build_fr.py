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
FRS = ("ldpc5g_dec_frame.h", "ldpc5g_dec_frame_iter.h")   # patched: the first file holding the text

PATCHES = {
    # timing splits (wrong results)
    "noB": [("            if (active && !gdead) {", "            if (false) {")],
    "nobar": [("            lds_barrier();\n        });\n        }\n", "        });\n        }\n")],
    "plain": [("            else __hip_atomic_fetch_add(&acc, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);",
               "            else acc = r;")],
    # phase A: the core edges' (LQ < 0) parity from f64 compares instead of the sign-word XOR
    "noa": [("                    r.px ^= FT<T>::sbits(a);   // a core LQ is never -0.0 (frame_body's load)",
             "                    r.par ^= a < T(0);")],
    # phase A: rotated LQ offsets by VALU (rot: two adds + a min) instead of the wrap table
    "A_rot": [("                tbs[p % kFrDT] = *(lds_u32*)(uintptr_t)(tz + (uint32_t)fr_cof<BG>(i, k) * 4u);",
               "                tbs[p % kFrDT] = rot(fr_cof<BG>(i, k));")],
    # phase A without the per-edge scheduling barrier
    "nosb": [("                    a = snext(ic, kc);\n                    __builtin_amdgcn_sched_barrier(0);",
              "                    a = snext(ic, kc);")],
    # phase-A latency splits (wrong results): no LDS reads of the core LQ / no ext LLR loads
    "A_nolds": [("                if constexpr (P::COL[e0 + k2] < KC) r.ab = at((uint32_t)(P::COL[e0 + k2] * kFrColB) + r.tb[k2 % 2]);",
                 "                if constexpr (P::COL[e0 + k2] < KC) r.ab = __builtin_bit_cast(T, ((uint64_t)r.tb[k2 % 2] << 32) | 0x3ff00000u);"),
                ("                if constexpr (P::COL[e0 + k3] < KC) r.tb[k3 % 2] = *(lds_u32*)(uintptr_t)(tz + (uint32_t)fr_cof<BG>(i, k3) * 4u);",
                 "                if constexpr (P::COL[e0 + k3] < KC) r.tb[k3 % 2] = tz + (uint32_t)fr_cof<BG>(i, k3) * 4u;")],
    "A_noxl": [("            if constexpr (p < kFrPlan<BG>.nx[hh]) xr[p % XP] = llrx(kFrPlan<BG>.xlist[hh][p]);",
                "            if constexpr (p < kFrPlan<BG>.nx[hh]) xr[p % XP] = T(1.5 + p) + T(sv);")],
    # DEAD kernel probe: the prologue's liveness loads kept, the plain iterations always
    "onlyplain": [("        if (live_x != all) {", "        if (live_x == 12345) {")],
}


def make(spec):
    name, _, flags = spec.partition(":")
    d = os.path.join(ROOT, "build", "frv", name)
    shutil.rmtree(d, ignore_errors=True)
    shutil.copytree(CSRC, d)
    texts = {f: open(os.path.join(d, f)).read() for f in FRS}
    for old, new in PATCHES.get(name.split("+")[0], []):
        hit = [f for f in FRS if old in texts[f]]
        assert hit, (name, old[:80])
        texts[hit[0]] = texts[hit[0]].replace(old, new)
    for f in FRS:
        open(os.path.join(d, f), "w").write(texts[f])
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
