"""Register / scratch / LDS use of every kernel in a built engine library
(the code-object notes of its gfx950 offload bundle).

    python tools/kernel_resources.py [logparser_amd/_lib/liblogparser_amd.so] [name-filter]
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def kernels(lib):
    """the gfx950 code objects of every offload bundle in the library's .hip_fatbin"""
    with tempfile.TemporaryDirectory() as d:
        fb = os.path.join(d, "fatbin")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "-O", "binary", "--only-section=.hip_fatbin", lib, fb],
                       check=True)
        data = open(fb, "rb").read()
        magic = b"__CLANG_OFFLOAD_BUNDLE__"
        starts = [m.start() for m in re.finditer(re.escape(magic), data)]
        res = []
        for i, s in enumerate(starts):
            e = starts[i + 1] if i + 1 < len(starts) else len(data)
            b = os.path.join(d, "b%d" % i)
            open(b, "wb").write(data[s:e])
            tl = subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--list", "--type=o", "--input=" + b],
                                capture_output=True, text=True).stdout.split()
            for j, t in enumerate(x for x in tl if "gfx950" in x):
                co = os.path.join(d, "k%d_%d.co" % (i, j))
                subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", "--input=" + b,
                                "--targets=" + t, "--output=" + co], check=True)
                res.append(subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True,
                                          capture_output=True, text=True).stdout)
        return "\n".join(res)


def parse(notes):
    out = []
    for blk in re.split(r"\n\s*- \.agpr_count", notes)[1:]:
        def g(k):
            m = re.search(r"\.%s:\s+(\S+)" % re.escape(k), blk)
            return m.group(1) if m else "?"
        out.append((g("name"), g("vgpr_count"), g("sgpr_count"), g("vgpr_spill_count"), g("sgpr_spill_count"),
                    g("private_segment_fixed_size"), g("group_segment_fixed_size")))
    return out


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 else "logparser_amd/_lib/liblogparser_amd.so"
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    rows = parse(kernels(lib))
    print("%-70s %5s %5s %6s %6s %7s" % ("kernel", "vgpr", "sgpr", "vspill", "sspill", "scratch"))
    for n, v, s, vs, ss, pr, gs in sorted(rows):
        if flt in n:
            print("%-70s %5s %5s %6s %6s %7s" % (n[:70], v, s, vs, ss, pr))
