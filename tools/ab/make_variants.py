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
sys.path.insert(0, ROOT)
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
# layered per-row overheads (ISA count per iteration, r02s: 5583 VALU, 316 edges)
_NOINIT = ("        T xlb[2][NXR] = {};", "        T xlb[2][NXR];")
_IDXOP = ("            const uint32_t idxo = pk >> 24;\n",
          "            uint32_t idxo = pk >> 24;\n            asm volatile(\"\" : \"+v\"(idxo));\n")
_NOPF = [("""            uint32_t csw[NPW];
#pragma unroll
            for (int x = 0; x < NPW; ++x) csw[x] = nsw[x];""",
          """            prefetch(gc);
            uint32_t csw[NPW];
#pragma unroll
            for (int x = 0; x < NPW; ++x) csw[x] = nsw[x];"""),
         ("            if constexpr (g + 1 < kGroups<BG>.n) prefetch(std::integral_constant<int, g + 1>{});\n"
          "            lds_barrier();", "            lds_barrier();")]
VARIANTS.update({
    # xlb zero-initialised every iteration (~90 v_mov)
    "lay_noinit": (LAYERED, [_NOINIT]),
    # rows 0-3: the argmin compare folded into v_cmp_eq_u32_sdwa BYTE_3 + a v_mov of k per edge
    "lay_idxop": (LAYERED, [_IDXOP]),
    # shift words loaded after the barrier (no double buffer: fewer SGPRs, no writelane spills)
    "lay_nopf": (LAYERED, _NOPF),
    "lay_combo": (LAYERED, [_NOINIT, _IDXOP] + _NOPF),
})

# r04, the Zc = 384 layered kernel (table reads with immediate offsets): how many rows keep their
# rotated offsets live from pass 1 to pass 2, and how many rows keep their state in LDS
VARIANTS.update({
    "lay_recomp8": (LAYERED, [("constexpr int kRecompDeg = 12;", "constexpr int kRecompDeg = 8;")]),
    "lay_recomp5": (LAYERED, [("constexpr int kRecompDeg = 12;", "constexpr int kRecompDeg = 5;")]),
    "lay_nlr12": (LAYERED, [("constexpr int lds_rows() { return BG == 1 ? 11 : 18; }",
                             "constexpr int lds_rows() { return BG == 1 ? 12 : 18; }")]),
    "lay_nlr10": (LAYERED, [("constexpr int lds_rows() { return BG == 1 ? 11 : 18; }",
                             "constexpr int lds_rows() { return BG == 1 ? 10 : 18; }")]),
})


def _pre(n):
    """Rotated-address table lookups of the next row group's first row (its first n core edges)
    issued BEFORE the row-group barrier: after the barrier the first data reads go out at once
    instead of waiting for a table round trip while all three waves of the SIMD sit idle."""
    return [
        ("    uint32_t mv = 0x80000000u;   // sign mask kept in a VGPR (all-VGPR bitop3 is full rate)\n",
         f"    constexpr int kNPre = {n};\n    uint32_t pre[kNPre];\n"
         "    uint32_t mv = 0x80000000u;   // sign mask kept in a VGPR (all-VGPR bitop3 is full rate)\n"),
        ("        auto layered_row = [&](auto ic, auto& gshift, T xl) {",
         "        auto layered_row = [&](auto ic, auto& gshift, T xl, auto npre) {"),
        ("                    rb[k] = (int)*(lds_u32*)(uintptr_t)(tzbT + (uint32_t)gshift(e0 + k) * GT);\n",
         "                    if constexpr (k < decltype(npre)::value) rb[k] = (int)pre[k];\n"
         "                    else rb[k] = (int)*(lds_u32*)(uintptr_t)(tzbT + (uint32_t)gshift(e0 + k) * GT);\n"),
        ("                    layered_row(ic, gshift, i >= 4 ? xlb[g & 1][i >= 4 ? i - r0 : 0] : T(0));\n",
         "                    layered_row(ic, gshift, i >= 4 ? xlb[g & 1][i >= 4 ? i - r0 : 0] : T(0),\n"
         "                                std::integral_constant<int, (g > 0 && i == kGroups<BG>.start[g]) ? kNPre : 0>{});\n"),
        ("            if constexpr (g + 1 < kGroups<BG>.n) prefetch(std::integral_constant<int, g + 1>{});\n"
         "            lds_barrier();",
         """            if constexpr (g + 1 < kGroups<BG>.n) {
                prefetch(std::integral_constant<int, g + 1>{});
                constexpr int i1 = kGroups<BG>.start[g + 1];
                constexpr int e1 = P::RS[i1], d1 = P::RS[i1 + 1] - P::RS[i1];
                sfor<0, kNPre>([&](auto kc) {
                    constexpr int k = decltype(kc)::value;
                    if constexpr (k < d1 && P::COL[e1 + k] < KC) {
                        const uint32_t w = nsw[((e1 + k) >> 1) - group_w0<BG>(g + 1)];
                        const uint32_t s = ((e1 + k) & 1) ? (w >> 16) : (w & 0xffffu);
                        pre[k] = *(lds_u32*)(uintptr_t)(tzbT + s * GT);
                    }
                });
            }
            lds_barrier();"""),
    ]


VARIANTS.update({
    # one codeblock per 384-thread layered workgroup (78 KB LDS), two workgroups per CU: the row-group
    # barriers of one workgroup overlap the other's work (full build: the mixed plan's G changes)
    "t384": ("ldpc5g_common.h", [("constexpr int kDecThreadsL = 768;", "constexpr int kDecThreadsL = 384;")]),
})
VARIANTS.update({
    # timing split (wrong results): the layered row loop without its row-group barriers — the
    # barrier-exposed share of the launch
    "lay_nobar": (LAYERED, [("            if constexpr (g + 1 < kGroups<BG>.n) prefetch(std::integral_constant<int, g + 1>{});\n"
                             "            lds_barrier();",
                             "            if constexpr (g + 1 < kGroups<BG>.n) prefetch(std::integral_constant<int, g + 1>{});\n")]),
})
# pass-1 two-min two edges at a time: min1' = min3(min1, x, y), min2' = min(min2, med3(min1, x, y))
# (the second smallest of {min1 <= min2, x, y}): 3 ops per 2 edges instead of 4, same selections
_MIN3 = [("""                asm("v_add_u32 %0, %1, %1" : "=v"(u) : "v"(u));   // u <<= 1, all-VGPR form
                const T aq = fabs(q[k]);
                min2 = FT<T>::med3(min1, min2, aq);
                min1 = fmin(min1, aq);
""", """                asm("v_add_u32 %0, %1, %1" : "=v"(u) : "v"(u));   // u <<= 1, all-VGPR form
                if constexpr (k % 2 == 1) {
                    const T x = fabs(q[k - 1]), y = fabs(q[k]);
                    min2 = fmin(min2, FT<T>::med3(min1, x, y));
                    min1 = fmin(fmin(min1, x), y);
                } else if constexpr (k == d - 1) {
                    const T aq = fabs(q[k]);
                    min2 = FT<T>::med3(min1, min2, aq);
                    min1 = fmin(min1, aq);
                }
""")]
VARIANTS.update({"lay_min3": (LAYERED, _MIN3)})
def _xl_ahead(n):
    """ext-column LLRs of row group g loaded n groups ahead (n + 1 buffers) instead of one: a row
    group lasts ~1.1 us, about one L2-miss round trip under load."""
    return [("        T xlb[2][NXR] = {};", f"        T xlb[{n + 1}][NXR] = {{}};"),
            ("                xlb[g & 1][i - r0] = lrow[(KB + i - pc) * Zc + zv];",
             f"                xlb[g % {n + 1}][i - r0] = lrow[(KB + i - pc) * Zc + zv];"),
            ("        prefetch_xl(std::integral_constant<int, 0>{});   // row 0 has no ext column: no load\n",
             "".join(f"        prefetch_xl(std::integral_constant<int, {j}>{{}});\n" for j in range(n))),
            ("            if constexpr (g + 1 < kGroups<BG>.n) prefetch_xl(std::integral_constant<int, g + 1>{});",
             f"            if constexpr (g + {n} < kGroups<BG>.n) prefetch_xl(std::integral_constant<int, g + {n}>{{}});"),
            ("layered_row(ic, gshift, i >= 4 ? xlb[g & 1][i >= 4 ? i - r0 : 0] : T(0));",
             f"layered_row(ic, gshift, i >= 4 ? xlb[g % {n + 1}][i >= 4 ? i - r0 : 0] : T(0));")]


VARIANTS.update({
    "lay_xl2": (LAYERED, _xl_ahead(2)), "lay_xl3": (LAYERED, _xl_ahead(3)),
    # timing split (wrong results): no ext-column LLR loads in the row loop
    "lay_noxl": (LAYERED, [("                xlb[g & 1][i - r0] = lrow[(KB + i - pc) * Zc + zv];",
                            "                xlb[g & 1][i - r0] = T(0.5f);")]),
})
# (IEEE mode off for the layered TU — -mno-amdgpu-ieee -fno-honor-nans, to drop the ~88
# canonicalising v_max_f32 per iteration — crashes this compiler: "illegal VGPR to SGPR copy".)
# stop-rule syndrome pass and final pass: rotated addresses from the wrap table (1 VALU + 1 LDS
# read per edge) instead of rot()'s two SGPR-operand adds and a min
VARIANTS.update({"lay_syntbl": (LAYERED, [
    ("par ^= at(j * CS * TS + rot(shift_of<BG>(ziv, e0 + k))) < T(0);",
     "par ^= at(j * CS * TS + (int)*(lds_u32*)(uintptr_t)(tzbT + (uint32_t)shift_of<BG>(ziv, e0 + k) * GT)) < T(0);"),
    ("if constexpr (j < KC) a = at(j * CS * TS + rot(shift_of<BG>(zi, e0 + k)));",
     "if constexpr (j < KC) a = at(j * CS * TS + (int)*(lds_u32*)(uintptr_t)(tzbT + (uint32_t)shift_of<BG>(zi, e0 + k) * GT));"),
])})
VARIANTS.update({"lay_pre4": (LAYERED, _pre(4)), "lay_pre8": (LAYERED, _pre(8)),
                 "lay_pre12": (LAYERED, _pre(12))})


# instrumentation (wrong ck rows): thread 0 of every workgroup records the real-time clock (100 MHz)
# at 7 points — start, after the prologue, after iteration 1, loop exit, after the final syndrome
# pass, after the ck store, and (slot 6) after the prologue's LLR loads were consumed — into the
# first 56 bytes of its first codeblock's ck row (tools/ts_probe.py reads them)
def _ts(flood):
    rt = "__builtin_amdgcn_s_memrealtime()"
    final = ("    lds_barrier();   // every LQ / state read is done: LDS below FLAG_B is free from here\n" if flood else
             "    lds_barrier();   // every APP / state read is done: LDS below FLAG_B is free from here\n")
    loads = ("        if constexpr (DEAD)\n            per_half_init(" if flood else
             "    for (int w = 0; w < 2 * NLR; ++w) at(ST_B + w * CS * TS + tzb) = T(0);\n")
    p = [
        ("    const int t = threadIdx.x;\n", f"    const int t = threadIdx.x;\n    uint64_t ts[7] = {{}};\n    ts[0] = {rt};\n"),
        ("    bool active = valid;\n    lds_barrier();\n", f"    bool active = valid;\n    lds_barrier();\n    ts[1] = {rt};\n"),
        ("        if (!block_any(active)) break;\n    }\n",
         f"        if (it == 0) ts[2] = {rt};\n        if (!block_any(active)) break;\n    }}\n    ts[3] = {rt};\n"),
        (final, final + f"    ts[4] = {rt};\n"),
        (loads, f"    ts[6] = {rt};\n" + loads),
        ("        }, slow, t, (int)blockDim.x);\n    }\n}\n",
         f"        }}, slow, t, (int)blockDim.x);\n    }}\n    __syncthreads();\n    ts[5] = {rt};\n"
         "    if (t == 0 && !work) {\n        uint64_t* o = (uint64_t*)(ck + (int64_t)((int)blockIdx.x * G) * ldc);\n"
         "        for (int k = 0; k < 7; ++k) o[k] = ts[k];\n    }\n}\n"),
    ]
    return p


VARIANTS.update({"lay_ts": (LAYERED, _ts(False)), "flood_ts": (FLOOD, _ts(True))})
# the per-thread output / LLR row of the layered kernel re-derived after the iteration loop from an
# opaque thread id, instead of keeping crow / out / lrow copies live across the loop (they were
# the kernel's only scratch spills: 40 B/lane, 63 MB of WRITE per 4096-codeblock launch)
_REDERIVE = [
    ("""                if (cand && flagB[cl] == 0) {
                    if (z == 0) status[out] = 1, iters[out] = it + 1;""",
     """                if (cand && flagB[cl] == 0) {
                    if (z == 0) {
                        int tq = t;
                        asm volatile("" : "+v"(tq));
                        const int cq = tq - zv * G;
                        const int oq = work ? cbs[work[blockIdx.x].first + cq].out : (int)blockIdx.x * G + cq;
                        status[oq] = 1, iters[oq] = it + 1;
                    }"""),
    ("""    zv = z;
    asm volatile("" : "+v"(zv));   // keep the output addresses out of the loop (no hoist/spill)
    if (active) {""",
     """    zv = z;
    asm volatile("" : "+v"(zv));   // keep the output addresses out of the loop (no hoist/spill)
    int t2 = t;
    asm volatile("" : "+v"(t2));
    const int cl2 = t2 - zv * G;   // zv = z here (no division)
    int out2 = 0;
    const T* lrow2 = llr;
    if (valid) {
        if (work) {
            const CbRef r2 = cbs[work[blockIdx.x].first + cl2];
            out2 = r2.out, lrow2 = llr + r2.llr_off;
        } else {
            out2 = (int)blockIdx.x * G + cl2, lrow2 = llr + (int64_t)out2 * ldl;
        }
    }
    auto llrx2 = [&](int i4) -> T { return lrow2[(KB + 4 + i4 - pc) * Zc + zv]; };
    if (active) {"""),
    ("""            sfor<x0, x1>([&](auto xc) { vx[decltype(xc)::value - x0] = llrx(decltype(xc)::value); });""",
     """            sfor<x0, x1>([&](auto xc) { vx[decltype(xc)::value - x0] = llrx2(decltype(xc)::value); });"""),
    ("""        if (fail) flagA[cl] = 1;
        uint32_t oc = 0;""", """        if (fail) flagA[cl2] = 1;
        uint32_t oc = 0;"""),
    ("""    if (active && z == 0) {
        status[out] = flagA[cl] == 0;
        iters[out] = L;
    }""", """    if (active && z == 0) {
        status[out2] = flagA[cl2] == 0;
        iters[out2] = L;
    }"""),
    ("""            const uint32_t sb = (uint32_t)(cl * ck_stage_stride(NFZ) + zv);""",
     """            const uint32_t sb = (uint32_t)(cl2 * ck_stage_stride(NFZ) + zv);"""),
    ("""        const bool slow = block_any(valid && !ck_row_aligned(NFZ, crow));   // orders the staging too""",
     """        int8_t* crow2 = ck;
        if (valid) crow2 = work ? ck + cbs[work[blockIdx.x].first + cl2].ck_off : ck + (int64_t)out2 * ldc;
        const bool slow = block_any(valid && !ck_row_aligned(NFZ, crow2));   // orders the staging too"""),
]
# ... and the stop rule's flag slot from the per-iteration opaque zv (its address was hoisted out of
# the loop and spilled)
_REDERIVE_FLAGS = [
    ("""        {
            // ---- layered stopping rule: no hard decision changed over the iteration, then an
            //      exact syndrome check of those decisions (oracle.decode_layered)
            uint32_t hdc = 0;""", """        const int clq = valid ? t - zv * G : 0;
        {
            // ---- layered stopping rule: no hard decision changed over the iteration, then an
            //      exact syndrome check of those decisions (oracle.decode_layered)
            uint32_t hdc = 0;"""),
    ("""            if (active && (hdc != hdc_prev || hdx != hdx_prev)) flagA[cl] = 1;""",
     """            if (active && (hdc != hdc_prev || hdx != hdx_prev)) flagA[clq] = 1;"""),
    ("""            const bool cand = active && flagA[cl] == 0;""", """            const bool cand = active && flagA[clq] == 0;"""),
    ("""                    if (sf) flagB[cl] = 1;""", """                    if (sf) flagB[clq] = 1;"""),
    ("""                if (cand && flagB[cl] == 0) {""", """                if (cand && flagB[clq] == 0) {"""),
    ("""        lds_barrier();
        if (z == 0 && valid) flagA[cl] = 0, flagB[cl] = 0;
        if (!block_any(active)) break;""", """        lds_barrier();
        if (z == 0 && valid) flagA[clq] = 0, flagB[clq] = 0;
        if (!block_any(active)) break;"""),
]
# (r04: lay_rederive2 = _REDERIVE + _REDERIVE_FLAGS measured 2.348 vs 2.371 ms / 8.843 vs 9.055 ms at
#  4096 / 16384 codeblocks, 0 B/lane scratch; adopted into ldpc5g_dec_body.h, so these patches no
#  longer apply and are kept as the record of the change)
# (a variant may also name a unified diff against python_5gtoolbox_amd/csrc, applied with patch -p3
#  in the copy; r04's lay_bitsyn diff was measured, rejected and deleted in r05: DESIGN.md §7)


def make(name):
    target, patches = VARIANTS[name]
    d = os.path.join(ROOT, "build", "alt_src", name)
    shutil.rmtree(d, ignore_errors=True)
    shutil.copytree(CSRC, d)
    p = os.path.join(d, target)
    if isinstance(patches, str):
        with open(os.path.join(ROOT, patches)) as f:
            r = subprocess.run(["patch", "-p3", "-d", d], stdin=f, capture_output=True, text=True)
        assert r.returncode == 0, (name, r.stdout, r.stderr)
    else:
        s = open(p).read()
        for old, new in patches:
            assert old in s, (name, old[:60])
            s = s.replace(old, new)
        open(p, "w").write(s)
    out = os.path.join(ROOT, "build", "alt", name + ".so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    if target == LAYERED and name.startswith("lay"):
        # only the layered TU instantiates the patched kernel: recompile it and link it with the
        # product objects of every other TU (build/obj, from the current product build)
        from python_5gtoolbox_amd import build as b
        assert not os.environ.get("LDPC5G_EXTRA_FLAGS"), "the product objects must be built without A/B flags"
        b.build(verbose=False)
        od = os.path.join(ROOT, "build", "obj_alt_" + name)
        os.makedirs(od, exist_ok=True)
        try:
            lay = b._compile(os.path.join(d, "ldpc5g_dec_l.hip"), False, od, d)
        except subprocess.CalledProcessError as e:
            return name, 1, str(e)
        objs = [lay] + [os.path.join(b.OBJ, os.path.basename(x) + ".o") for x in b.sources()
                        if os.path.basename(x) != "ldpc5g_dec_l.hip"]
        r = subprocess.run([b.HIPCC, f"--offload-arch={b.ARCH}", "-shared", "-fPIC", *objs, "-o", out],
                           capture_output=True, text=True)
        return name, r.returncode, r.stderr[-2000:]
    r = subprocess.run([sys.executable, "-m", "python_5gtoolbox_amd.build", "--csrc", d, "--out", out],
                       cwd=ROOT, capture_output=True, text=True)
    return name, r.returncode, r.stderr[-2000:]


if __name__ == "__main__":
    names = sys.argv[1:] or list(VARIANTS)
    with ThreadPoolExecutor(4) as ex:
        for name, rc, err in ex.map(make, names):
            print(name, "rc", rc, err if rc else "")
