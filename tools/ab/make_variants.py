"""Decoder A/B variants (dev tool): copy python_5gtoolbox_amd/csrc into build/alt_src/<name>/,
apply string patches, and build each into build/alt/<name>.so for one GPU call to time them side
by side (tools/gpu_round.sh ab).  Variants that win move into the product sources; the rest stay
recorded here and in DESIGN.md, not as switches in csrc/."""
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "python_5gtoolbox_amd", "csrc")
BODY = "ldpc5g_dec_body.h"

# pass 2: |q_k| == min1 via a full-rate sub (abs modifier) + arithmetic shift, selects as bitop3
NOTMIN_OLD = """                const bool isMin = fabs(q[k]) == min1;   // ties: nB == nA, either is right
                idxn = isMin ? (uint32_t)k : idxn;
                const T sel = isMin ? nBs : nAs;
                const T r = __uint_as_float(__builtin_amdgcn_bitop3_b32(qb, __float_as_uint(sel), mv, 0x6c));"""
NOTMIN_NEW = """                const uint32_t notMin = (uint32_t)((int32_t)__float_as_uint(min1 - fabsf(q[k])) >> 31);
                idxn = __builtin_amdgcn_bitop3_b32(notMin, idxn, (uint32_t)k, 0xca);
                const uint32_t sel = __builtin_amdgcn_bitop3_b32(notMin, __float_as_uint(nAs), __float_as_uint(nBs), 0xca);
                const T r = __uint_as_float(__builtin_amdgcn_bitop3_b32(qb, sel, mv, 0x6c));"""
# rotated address: second candidate by an all-VGPR subtract of Zc*G*4
ADDR_OLD = """    auto rot = [&](int s) -> int {
        const uint32_t S = (uint32_t)s * GT;
        return (int)min((uint32_t)tzb + S, tzbw + S);
    };"""
ADDR_NEW = """    uint32_t zgt_v = ZGT;
    asm volatile("" : "+v"(zgt_v));
    auto rot = [&](int s) -> int {
        const uint32_t a = (uint32_t)tzb + (uint32_t)s * GT;
        uint32_t b;
        asm("v_sub_u32 %0, %1, %2" : "=v"(b) : "v"(a), "v"(zgt_v));
        return (int)min(a, b);
    };"""

# static priority for the second half of the workgroup's waves (MI355X_MICROARCH.md, two waves per
# SIMD item 4)
PRIO_OLD = """    uint32_t mv = 0x80000000u;   // sign mask kept in a VGPR (all-VGPR bitop3 is full rate)"""
PRIO_NEW = """    if constexpr (LAYERED) {
        if ((t >> 6) >= (CS >> 7)) __builtin_amdgcn_s_setprio(1);
    }
    uint32_t mv = 0x80000000u;   // sign mask kept in a VGPR (all-VGPR bitop3 is full rate)"""
# stagger: in row groups of >= 2 rows the second half of the waves runs the rows in reverse order
STAG_OLD = """            if (active) {
                sfor<kGroups<BG>.start[g], kGroups<BG>.start[g + 1]>([&](auto ic) {
                    constexpr int i = decltype(ic)::value;
                    constexpr int r0 = kGroups<BG>.start[g] > 4 ? kGroups<BG>.start[g] : 4;
                    if constexpr (LAYERED) layered_row(ic, gshift, i >= 4 ? xlb[g & 1][i >= 4 ? i - r0 : 0] : T(0));
                    else flooding_row(ic, gshift);
                });
            }"""
STAG_NEW = """            constexpr int gs = kGroups<BG>.start[g], ge = kGroups<BG>.start[g + 1];
            if (active) {
                if (LAYERED && ge - gs >= 2 && (t >> 6) >= (CS >> 7)) {
                    sfor<gs, ge>([&](auto jc) {
                        constexpr int i = gs + ge - 1 - decltype(jc)::value;
                        constexpr int r0 = gs > 4 ? gs : 4;
                        if constexpr (LAYERED) layered_row(std::integral_constant<int, i>{}, gshift, i >= 4 ? xlb[g & 1][i >= 4 ? i - r0 : 0] : T(0));
                    });
                } else {
                    sfor<gs, ge>([&](auto ic) {
                        constexpr int i = decltype(ic)::value;
                        constexpr int r0 = gs > 4 ? gs : 4;
                        if constexpr (LAYERED) layered_row(ic, gshift, i >= 4 ? xlb[g & 1][i >= 4 ? i - r0 : 0] : T(0));
                        else flooding_row(ic, gshift);
                    });
                }
            }"""

# layered: rotated addresses from an LDS table indexed by the unwrapped offset (1 VALU + 1 LDS read
# per edge instead of 2 adds + a min)
TBL = [
    ("""           (LAYERED ? (size_t)2 * lds_rows<BG>() * CS * sizeof(T) : 0) + (2 * kMaxG + 4) * sizeof(int);""",
     """           (LAYERED ? (size_t)2 * lds_rows<BG>() * CS * sizeof(T) : 0) + (2 * kMaxG + 4) * sizeof(int) +
           (LAYERED ? (size_t)2 * CS * sizeof(uint32_t) : 0);"""),
    ("""    constexpr int FLAG_B = ST_B + 2 * NLR * CS * TS;""",
     """    constexpr int FLAG_B = ST_B + 2 * NLR * CS * TS;
    constexpr int TBL_B = FLAG_B + (2 * kMaxG + 4) * 4;   // layered: wrap table, 2*CS entries"""),
    ("""    if (z == 0 && valid) flagA[cl] = 0, flagB[cl] = 0;
    if (t == 0) *anyf = 0;
    bool active = valid;
    lds_barrier();""",
     """    if (z == 0 && valid) flagA[cl] = 0, flagB[cl] = 0;
    if (t == 0) *anyf = 0;
    using lds_u32 = __attribute__((address_space(3))) uint32_t;
    if constexpr (LAYERED) {   // T[e] = byte offset of entry e mod (Zc*G), e in [0, 2*Zc*G)
        const int ZG = Zc * G;
        if (t < ZG) {
            *(lds_u32*)(uintptr_t)(uint32_t)(TBL_B + t * 4) = (uint32_t)(t * 4);
            *(lds_u32*)(uintptr_t)(uint32_t)(TBL_B + (t + ZG) * 4) = (uint32_t)(t * 4);
        }
    }
    const uint32_t tzbT = (uint32_t)(TBL_B + (valid ? t : 0) * 4);
    bool active = valid;
    lds_barrier();"""),
    ("""                } else {
                    q[k] = xl;   // degree-1 column: q is the channel LLR itself
                }
                asm("v_add_u32 %0, %1, %1" : "=v"(u) : "v"(u));""",
     """                } else {
                    q[k] = xl;   // degree-1 column: q is the channel LLR itself
                }
                asm("v_add_u32 %0, %1, %1" : "=v"(u) : "v"(u));   // (tbl)"""),
    ("""#else
                    rb[k] = rot(gshift(e0 + k));
                    q[k] = at(j * CS * TS + rb[k]) - rold;
#endif""",
     """#else
                    rb[k] = (int)*(lds_u32*)(uintptr_t)(tzbT + (uint32_t)gshift(e0 + k) * GT);
                    q[k] = at(j * CS * TS + rb[k]) - rold;
#endif"""),
    ("""            constexpr bool RECOMP = d > kRecompDeg;
            uint32_t tzb2 = (uint32_t)tzb, tzbw2 = tzbw;
            if constexpr (RECOMP) {
                asm volatile("" : "+v"(tzb2));
                asm volatile("" : "+v"(tzbw2));
            }
            sfor<0, d>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                constexpr int j = P::COL[e0 + k];
                const uint32_t qb = FT<T>::sbits(q[k]);""",
     """            constexpr bool RECOMP = d > kRecompDeg;
            uint32_t tzbT2 = tzbT;
            if constexpr (RECOMP) asm volatile("" : "+v"(tzbT2));
            sfor<0, d>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                constexpr int j = P::COL[e0 + k];
                const uint32_t qb = FT<T>::sbits(q[k]);"""),
    ("""                        const uint32_t S = (uint32_t)gshift(e0 + k) * GT;
                        at(j * CS * TS + (int)min(tzb2 + S, tzbw2 + S)) = app;""",
     """                        const uint32_t S = (uint32_t)gshift(e0 + k) * GT;
                        at(j * CS * TS + (int)*(lds_u32*)(uintptr_t)(tzbT2 + S)) = app;"""),
]

VARIANTS = {
    "base": [],
    "notmin": [(NOTMIN_OLD, NOTMIN_NEW)],
    "addr": [(ADDR_OLD, ADDR_NEW)],
    "both": [(NOTMIN_OLD, NOTMIN_NEW), (ADDR_OLD, ADDR_NEW)],
    "prio": [(PRIO_OLD, PRIO_NEW)],
    "stagger": [(STAG_OLD, STAG_NEW)],
    "prio_stagger": [(PRIO_OLD, PRIO_NEW), (STAG_OLD, STAG_NEW)],
    "tbl": TBL,
    "tbl_notmin": TBL + [(NOTMIN_OLD, NOTMIN_NEW)],
}


def make(name, patches):
    d = os.path.join(ROOT, "build", "alt_src", name)
    shutil.rmtree(d, ignore_errors=True)
    shutil.copytree(CSRC, d)
    p = os.path.join(d, BODY)
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
        for name, rc, err in ex.map(lambda n: make(n, VARIANTS[n]), names):
            print(name, "rc", rc, err if rc else "")
