"""Per-phase instruction counts of a k_trace instance from its assembly: build
nr_trace.hip with -DNR_PHASE_MARKS=1 (an assembler comment at each phase boundary of the loop,
csrc/nr_trace.hip NR_PHASE), cut the instance's listing at the markers and count the instructions
of each phase by class: VALU (v_*, MFMAs apart), MFMA, SALU (s_* but branches / waitcnt / nop),
LDS (ds_*), VMEM (global_ / buffer_ / flat_), branches, waitcnt, nop.  Static counts: a phase's
instructions once, whatever its trip count (the MLP, scene and step run every wave iteration; the
refill when >= 8 ray slots are free; the shading once per 16 converged rays).
usage: python tools/phase_isa.py [kernel-substring ...]  (default: the batched bf16 tracer with
fp32x3 normals, without and with the endgame)"""
import collections
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "cudaneuralrender_amd", "csrc", "nr_trace.hip")
OUT = "/tmp/nr_trace_phases.s"


def build():
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
           "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops", "--cuda-device-only", "-S",
           "-DNR_PHASE_MARKS=1", "-I", os.path.join(REPO, "include"), SRC, "-o", OUT]
    subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)


def klass(op):
    if op.startswith("v_mfma"):
        return "MFMA"
    if op.startswith("v_"):
        return "VALU"
    if op.startswith("ds_"):
        return "LDS"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "VMEM"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_swappc")):
        return "branch"
    if op.startswith("s_"):
        return "SALU"
    return None


def phases(listing, kernel):
    lines = listing.splitlines()
    start = next(i for i, ln in enumerate(lines) if ln.startswith(kernel) and ln.rstrip().endswith(":") or
                 (ln.startswith(kernel) and ":" in ln and not ln.startswith("\t")))
    counts = collections.OrderedDict()
    cur = "prologue"
    for ln in lines[start + 1:]:
        if ln.startswith("\t.section") or re.match(r"^\s*s_endpgm", ln):
            break
        m = re.search(r"NRPHASE (\w+)", ln)
        if m:
            cur = m.group(1)
            continue
        t = ln.strip()
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        k = klass(t.split()[0])
        if k:
            counts.setdefault(cur, collections.Counter())[k] += 1
    return counts


def main():
    build()
    listing = open(OUT).read()
    pats = sys.argv[1:] or ["_ZN2nr7k_traceILi1ELb0ELb0ELb1ELb1ELb0E", "_ZN2nr7k_traceILi1ELb0ELb0ELb1ELb1ELb1E"]
    cols = ["VALU", "MFMA", "SALU", "LDS", "VMEM", "branch", "waitcnt", "nop"]
    for pat in pats:
        name = next(ln.split(":")[0] for ln in listing.splitlines() if ln.startswith(pat))
        c = phases(listing, name)
        print(f"# {name}")
        print(f"{'phase':<12}" + "".join(f"{k:>8}" for k in cols))
        tot = collections.Counter()
        for ph, cnt in c.items():
            tot.update(cnt)
            print(f"{ph:<12}" + "".join(f"{cnt.get(k, 0):>8}" for k in cols))
        print(f"{'total':<12}" + "".join(f"{tot.get(k, 0):>8}" for k in cols))


if __name__ == "__main__":
    main()
