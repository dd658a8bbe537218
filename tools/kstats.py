"""Per-kernel register / scratch / instruction summary of a libnr source, from hipcc's gfx950
assembly (the Makefile's flags):

    python tools/kstats.py nr_trace.hip [NAME_SUBSTRING ...]

Prints, per kernel whose mangled name contains every substring: VGPRs, AGPRs, SGPRs, scratch
bytes per lane (spills), LDS, and the count of MFMA / VALU / SALU / LDS / global instructions
in its body -- the numbers an A/B of a code-shape change looks at first.
"""
import os
import re
import subprocess
import sys

CSRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "cudaneuralrender_amd", "csrc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
         "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops", "--cuda-device-only", "-S"]


def assemble(src, extra=()):
    out = "/tmp/kstats_" + os.path.basename(src) + ".s"
    subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *extra, os.path.join(CSRC, src), "-o", out], check=True)
    return open(out).read()


def kernels(asm):
    """{name: (body lines, metadata dict)}"""
    res = {}
    for m in re.finditer(r"^(\S+):\s*; @\S+\n(.*?)^\s*s_endpgm", asm, re.S | re.M):
        res[m.group(1)] = m.group(2).splitlines()
    meta = {}
    for m in re.finditer(r"\.amdhsa_kernel (\S+)\n(.*?)\.end_amdhsa_kernel", asm, re.S):
        d = dict(re.findall(r"\.amdhsa_(\w+) (\S+)", m.group(2)))
        meta[m.group(1)] = d
    for m in re.finditer(r"; (\S+)\n(?:.*\n)*?\s*; NumVgprs: (\d+)\n\s*; NumAgprs: (\d+)", asm):
        pass
    return res, meta


def classify(lines):
    c = {"mfma": 0, "valu": 0, "salu": 0, "lds": 0, "vmem": 0, "scratch": 0}
    for ln in lines:
        t = ln.strip().split()
        if not t or t[0].startswith(("; ", ".", ";")) or t[0].endswith(":"):
            continue
        op = t[0]
        if op.startswith("v_mfma"):
            c["mfma"] += 1
        elif op.startswith("scratch_") or (op.startswith("buffer_") and "off" in ln and "s[0:3]" in ln):
            c["scratch"] += 1
        elif op.startswith("v_"):
            c["valu"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
        elif op.startswith(("global_", "buffer_", "flat_")):
            c["vmem"] += 1
    return c


def main():
    src = sys.argv[1]
    subs = sys.argv[2:]
    asm = assemble(src)
    bodies, meta = kernels(asm)
    for name, body in bodies.items():
        if not all(s in name for s in subs) or name not in meta:
            continue
        d = meta[name]
        c = classify(body)
        print(f"{name}\n  vgpr {d.get('next_free_vgpr')} agpr_off {d.get('accum_offset')} sgpr {d.get('next_free_sgpr')} "
              f"scratch {d.get('private_segment_fixed_size')} lds {d.get('group_segment_fixed_size')} | "
              + " ".join(f"{k} {v}" for k, v in c.items()))


if __name__ == "__main__":
    main()
