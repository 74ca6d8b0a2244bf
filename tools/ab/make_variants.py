"""Decoder A/B variants (dev tool): copy python_5gtoolbox_amd/csrc into build/alt_src/<name>/,
apply string patches to one header, and build each into build/alt/<name>.so for one GPU call to
time them side by side (tools/gpu_round.sh ab; LDPC5G_LIB selects the library).  Variants that win
move into the product sources; the measured results of the rest are in DESIGN.md §4.2 / §4.2b,
not switches in csrc/.  Patches are written against the current sources, so a variant whose text
no longer matches fails loudly (assert) instead of building the unpatched library.

    python tools/ab/make_variants.py flood_noB lay_idx_inplace
"""
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "python_5gtoolbox_amd", "csrc")
LAYERED = "ldpc5g_dec_body.h"
FLOOD = "ldpc5g_dec_flood.h"

VARIANTS = {
    # timing split (wrong results): the flooding kernel without phase B's row-ordered sums
    "flood_noB": (FLOOD, [
        ("                        if constexpr (i < NLS) {   // LDS state: both halves, alternate edges",
         "                        if constexpr (i < 0) {"),
        ("                        } else if constexpr (kFloodPlan<BG, T, NP, CS>.owner[i] == decltype(hc)::value) {",
         "                        } else if constexpr (i < 0) {"),
    ]),
    # flooding phase A: rows of degree >= 12 as two independent two-min chains (even / odd edges)
    # merged at the row end, halving the dependent f64 min/max chain
    "flood_split2": (FLOOD, [
        ("""            T min1 = FT<T>::inf(), min2 = FT<T>::inf();
            uint32_t sx = 0, idx = 0, negs = 0;
            bool par = false;
            sfor<0, d>([&](auto kc) {""",
         """            T min1 = FT<T>::inf(), min2 = FT<T>::inf();
            T m1b = FT<T>::inf(), m2b = FT<T>::inf();
            uint32_t sx = 0, idx = 0, negs = 0, idxb = 0;
            constexpr bool SPL = d >= 12;
            bool par = false;
            sfor<0, d>([&](auto kc) {"""),
        ("""                idx = aq < min1 ? (uint32_t)k : idx;
                asm volatile("" : "+v"(idx));   // update in place: a sunk select chain keeps all
                                                // the compare masks live (scratch spills)
                negs = __builtin_amdgcn_alignbit(negs, FT<T>::sbits(q), 31);
                two_min(min1, min2, aq);
                sx ^= FT<T>::sbits(q);
            });""",
         """                if constexpr (SPL && (k & 1)) {
                    idxb = aq < m1b ? (uint32_t)k : idxb;
                    asm volatile("" : "+v"(idxb));
                    two_min(m1b, m2b, aq);
                } else {
                    idx = aq < min1 ? (uint32_t)k : idx;
                    asm volatile("" : "+v"(idx));
                    two_min(min1, min2, aq);
                }
                negs = __builtin_amdgcn_alignbit(negs, FT<T>::sbits(q), 31);
                sx ^= FT<T>::sbits(q);
            });
            if constexpr (SPL) {
                const bool c = m1b < min1;
                min2 = c ? fmin(min1, m2b) : fmin(min2, m1b);
                min1 = c ? m1b : min1;
                idx = c ? idxb : idx;
            }"""),
    ]),
    # flooding phase B in float32 with LDS atomic adds too (ds_add_f32): measured 4x slower
    "flood_atomic_f32": (FLOOD, [
        ("                    } else if constexpr (sizeof(T) == 8) {",
         "                    } else if constexpr (sizeof(T) >= 4) {"),
    ]),
    # layered pass 2: the argmin updated in place (the flooding kernel's fix for a sunk select
    # chain); here it moved 36 -> 60 B/lane of scratch and did not cut the SGPR spills
    "lay_idx_inplace": (LAYERED, [
        ("                idxn = isMin ? (uint32_t)k : idxn;\n",
         "                idxn = isMin ? (uint32_t)k : idxn;\n                asm volatile(\"\" : \"+v\"(idxn));\n"),
    ]),
}


def make(name):
    target, patches = VARIANTS[name]
    d = os.path.join(ROOT, "build", "alt_src", name)
    shutil.rmtree(d, ignore_errors=True)
    shutil.copytree(CSRC, d)
    p = os.path.join(d, target)
    s = open(p).read()
    for old, new in patches:
        assert old in s, (name, old[:60])
        s = s.replace(old, new)
    open(p, "w").write(s)
    out = os.path.join(ROOT, "build", "alt", name + ".so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    r = subprocess.run([sys.executable, "-m", "python_5gtoolbox_amd.build", "--csrc", d, "--out", out],
                       cwd=ROOT, capture_output=True, text=True)
    return name, r.returncode, r.stderr[-2000:]


if __name__ == "__main__":
    names = sys.argv[1:] or list(VARIANTS)
    with ThreadPoolExecutor(2) as ex:
        for name, rc, err in ex.map(make, names):
            print(name, "rc", rc, err if rc else "")
