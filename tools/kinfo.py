"""Register / spill summary of the gfx950 kernels in built libraries (dev tool).

    python tools/kinfo.py PATTERN lib.so [lib2.so ...]

Prints, for every kernel whose mangled name contains PATTERN: vgpr count, vgpr / sgpr spills,
scratch bytes (from the code object's metadata notes).
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def notes(lib):
    with tempfile.TemporaryDirectory() as d:
        fb = os.path.join(d, "fb")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", lib, os.path.join(d, "x")],
                       check=True)
        data = open(fb, "rb").read()
        magic = b"__CLANG_OFFLOAD_BUNDLE__"
        starts = [m.start() for m in re.finditer(re.escape(magic), data)]
        out = []
        for i, s0 in enumerate(starts):
            part = os.path.join(d, f"b{i}")
            with open(part, "wb") as f:
                f.write(data[s0:starts[i + 1] if i + 1 < len(starts) else len(data)])
            co = os.path.join(d, f"co{i}")
            r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], capture_output=True)
            if r.returncode == 0 and os.path.getsize(co):
                out.append(subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True,
                                          text=True).stdout)
        return "\n".join(out)


def main():
    pat = sys.argv[1]
    for lib in sys.argv[2:]:
        cur = {}
        rows = []
        for ln in notes(lib).splitlines():
            ln = ln.strip()
            m = re.match(r"- \.args:|\.(name|vgpr_count|vgpr_spill_count|sgpr_spill_count|private_segment_fixed_size):\s+(\S+)", ln)
            if not m:
                continue
            if m.group(1) is None:
                continue
            cur[m.group(1)] = m.group(2)
            if m.group(1) == "name" or len(cur) == 5:
                pass
            if all(k in cur for k in ("name", "vgpr_count", "vgpr_spill_count", "sgpr_spill_count",
                                      "private_segment_fixed_size")):
                if pat in cur["name"]:
                    rows.append(cur)
                cur = {}
        for r in rows:
            print(f"{os.path.basename(lib)}: vgpr {r['vgpr_count']} vspill {r['vgpr_spill_count']} "
                  f"sspill {r['sgpr_spill_count']} scratch {r['private_segment_fixed_size']}  {r['name'][:110]}")


if __name__ == "__main__":
    main()
