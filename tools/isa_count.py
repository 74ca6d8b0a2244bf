"""Static ISA counts of the layered decoder's headline kernel (dev tool): extracts the gfx950 code
object from a built library, disassembles ldpc_dec_kernel_l<1,float,true,false> and counts the
instructions of the row-group region of the iteration loop (first to last row-group barrier), by
opcode.  Used to compare A/B variants before spending GPU time on them.

    python tools/isa_count.py python_5gtoolbox_amd/libldpc5g.so build/alt/*.so
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
KERNEL = "_ZN11ldpc5g_impl12_GLOBAL__N_117ldpc_dec_kernel_lILi1EfLb1ELb0ELb0ELi384EEEvPKT0_PaPhPiiiiilliS2_S2_iPKNS_7DecWorkEPKNS_5CbRefE"


def disasm(lib):
    """All gfx950 code objects of a library (the linked .hip_fatbin holds one bundle per TU)."""
    out = []
    with tempfile.TemporaryDirectory() as d:
        fb = os.path.join(d, "fb")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", lib, os.path.join(d, "x")],
                       check=True)
        data = open(fb, "rb").read()
        magic = b"__CLANG_OFFLOAD_BUNDLE__"
        starts = [m.start() for m in re.finditer(re.escape(magic), data)]
        for i, s0 in enumerate(starts):
            part = os.path.join(d, f"b{i}")
            with open(part, "wb") as f:
                f.write(data[s0:starts[i + 1] if i + 1 < len(starts) else len(data)])
            co = os.path.join(d, f"co{i}")
            r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"],
                               capture_output=True)
            if r.returncode == 0 and os.path.getsize(co):
                out.append(subprocess.run([f"{LLVM}/llvm-objdump", "-d", co], capture_output=True,
                                          text=True).stdout)
    return "\n".join(out)


def kernel_lines(text, name=KERNEL):
    out, on = [], False
    for ln in text.splitlines():
        if ln.endswith(">:"):
            on = f"<{name}>:" in ln
            continue
        if on and ln.strip():
            out.append(ln.split("//")[0].strip())
    return out


def region(lines):
    bars = [i for i, ln in enumerate(lines) if ln.startswith("s_barrier")]
    # row-group barriers are the long run of barriers; the loop region spans the first 33 after
    # the setup barrier (32 row groups in BG1)
    return lines[bars[0]:bars[min(len(bars) - 1, 33)]]


def summary(lib):
    lines = kernel_lines(disasm(lib))
    reg = region(lines)
    ops = collections.Counter(ln.split()[0] for ln in reg if ln)
    valu = sum(v for k, v in ops.items() if k.startswith("v_"))
    scratch = sum(v for k, v in collections.Counter(ln.split()[0] for ln in lines).items() if "scratch" in k)
    keys = ["v_writelane_b32", "v_readlane_b32", "v_mov_b32_e32", "v_cmp_eq_u32_sdwa", "ds_read_b32",
            "global_load_dword", "s_waitcnt"]
    return valu, scratch, {k: ops.get(k, 0) for k in keys}


if __name__ == "__main__":
    for lib in sys.argv[1:]:
        valu, scratch, ks = summary(lib)
        print(f"{os.path.basename(lib):28s} VALU {valu:5d}  scratch instrs (whole kernel) {scratch:3d}  " +
              " ".join(f"{k.replace('_b32', '').replace('_e32', '')}={v}" for k, v in ks.items()))
