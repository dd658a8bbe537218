#!/usr/bin/env python3
"""Per-kernel register / spill / LDS / occupancy table of one HIP source, from the compiler's
kernel-resource-usage remarks (gfx950, the library's own flags).

    python tools/kernel_resources.py [nr_trace.hip] [-DKNOB=..] [--filter k_trace]
"""
import os
import re
import subprocess
import sys

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cudaneuralrender_amd", "csrc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-Xclang",
         "-target-feature", "-Xclang", "-packed-fp32-ops", "-Wno-unused-function"]
KEYS = ("VGPRs", "AGPRs", "SGPRs Spill", "VGPRs Spill", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]",
        "LDS Size [bytes/block]")


def demangle(names):
    try:
        out = subprocess.run(["/opt/rocm/llvm/bin/llvm-cxxfilt"], input="\n".join(names), capture_output=True,
                             text=True).stdout.split("\n")
        return [o if o else n for o, n in zip(out, names)]
    except OSError:
        return names


def main():
    args = sys.argv[1:]
    flt = None
    if "--filter" in args:
        i = args.index("--filter")
        flt = args[i + 1]
        del args[i:i + 2]
    src = next((a for a in args if not a.startswith("-")), "nr_trace.hip")
    defs = [a for a in args if a.startswith("-D")]
    r = subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *defs, "-c", os.path.join(CSRC, src), "-o", "/dev/null",
                        "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True, cwd=CSRC)
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        for k in KEYS:
            m = re.search(r"remark:\s+" + re.escape(k) + r": (\d+)", line)
            if m and cur is not None:
                cur[k] = int(m.group(1))
    names = demangle([x["name"] for x in rows])
    print("%-70s %5s %5s %6s %6s %7s %4s %6s" % ("kernel", "VGPR", "AGPR", "SGsp", "VGsp", "scratch", "occ", "LDS"))
    for x, n in zip(rows, names):
        n = re.sub(r"\(nr::RenderArgs.*|\(nr::MlpArgs.*", "", n)
        if flt and flt not in n:
            continue
        print("%-70s %5s %5s %6s %6s %7s %4s %6s" % (n[:70], *(x.get(k, "-") for k in KEYS)))
    if r.returncode:
        print(r.stderr[-3000:])
        sys.exit(r.returncode)


if __name__ == "__main__":
    main()
