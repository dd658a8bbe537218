"""Generates tools/mlp_shape_asm.h: the bf16 MLP's 7 hidden layers on 128 points per wave as two
software-pipelined streams that differ only in the MFMA shape -- the A/B of VERDICT r4 item 1
("A/B k_mlp16 with a 16x16x32 generated stream"), timed by tools/mlp_shape_ab.hip.

  S32 (the product's shape, k_mlp16 / nr_mlp16_asm.h without its input layer): four 32-point tiles,
      per tile and layer two v_mfma_f32_32x32x16_bf16 (K = 16 each, bias as the first's
      accumulator init) and 8 v_cvt_pk_bf16_f32 ... clamp (ReLU) -> the next layer's B operand.
  S16: eight 16-point tiles, per tile and layer two v_mfma_f32_16x16x32_bf16 (output rows 0-15
      and 16-31, K = 32 each, bias as the accumulator init) and 4 v_cvt_pk_bf16_f32 ... clamp.
      Lane l of tile t holds rows 4(l >> 4) + i of each half = the k-slots 8(l >> 4) .. + 7 of the
      next layer's B operand under a fixed permutation of the hidden units (which a pack would
      fold into the weights), so no lane moves either.
Both: the conversions of tile t + 1 (S32) or t + 2 (S16) run beside tile t's MFMAs, the next layer's operands (A and bias
from LDS, ds_read_b128) load into the idle one of two register buffers a layer ahead, and every
hazard is checked (gen_mlp_asm.check).  Same FLOPs (7 x 128 x 2 x 32 x 32 per chunk), same LDS
bytes per layer for A (2 KB), the bias 1 KB (S32: 16 floats per lane) or 512 B (S16: 8).

The S16 summation (one K = 32 MFMA per output half) is not the product's (two K = 16 steps), so
an S16 product path would need its own oracle model; this is the timing A/B only.
Run:  python tools/gen_mlp_shape_asm.py        (writes tools/mlp_shape_asm.h)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_mlp_asm import NH, Stream, check, emit, rng  # noqa: E402


def build32(nt=4):
    """S32, hidden layers only: in = the accumulators v[0 : 16 nt) (the previous layer's f32 outputs)."""
    st = Stream(nt)
    ACC = lambda t: 16 * t
    KOP = lambda t, s: 16 * nt + 8 * t + 4 * s
    AOP = lambda b, s: 24 * nt + 8 * b + 4 * s
    BIAS = lambda b: 24 * nt + 16 + 16 * b

    def mfma(buf, t, s):
        d, a, b = ACC(t), AOP(buf, s), KOP(t, s)
        c = BIAS(buf) if s == 0 else ACC(t)
        reads = [("A", r) for r in rng(a, 4)] + [("B", r) for r in rng(b, 4)] + [("C", r) for r in rng(c, 16)]
        st.pad("mfma", reads, list(rng(d, 16)))
        st.add(f"v_mfma_f32_32x32x16_bf16 v[{d}:{d + 15}], v[{a}:{a + 3}], v[{b}:{b + 3}], v[{c}:{c + 15}]", "mfma",
               reads=reads, writes=list(rng(d, 16)))

    def conv(t, s):
        for q in range(4):
            src, dst = ACC(t) + 8 * s + 2 * q, KOP(t, s) + q
            st.pad("valu", [src, src + 1], [dst])
            st.add(f"v_cvt_pk_bf16_f32 v{dst}, v{src}, v{src + 1} clamp", "valu", reads=[src, src + 1], writes=[dst])

    def load(dst, addr, off):
        st.pad("lds", (), list(rng(dst, 4)))
        st.add(f"ds_read_b128 v[{dst}:{dst + 3}], %[{addr}]" + (f" offset:{off}" if off else ""), "lds",
               writes=list(rng(dst, 4)))

    def a_loads(buf, j):
        load(AOP(buf, 0), "va", 2048 * j)
        load(AOP(buf, 1), "va", 2048 * j + 1024)

    def b_load(buf, j, i):
        load(BIAS(buf) + 4 * i, "vb", 128 * j + 16 * i)

    wait = lambda: st.add("s_waitcnt lgkmcnt(0)", "wait")
    a_loads(1, 0)
    for i in range(4):
        b_load(1, 0, i)
    conv(0, 0)
    conv(0, 1)
    for l in range(1, NH + 1):
        buf, j, nxt = l % 2, l - 1, l < NH
        wait()
        for t in range(nt):
            for s in range(2):
                mfma(buf, t, s)
                conv(t + 1 if t < nt - 1 else 0, s)
                if nxt:
                    if (t, s) == (1, 0):
                        a_loads(1 - buf, j + 1)
                    elif (t, s) == (1, 1):
                        b_load(1 - buf, j + 1, 0)
                    elif (t, s) == (2, 0):
                        b_load(1 - buf, j + 1, 1)
                    elif (t, s) == (2, 1):
                        b_load(1 - buf, j + 1, 2)
                        b_load(1 - buf, j + 1, 3)
    for t in range(1, nt):
        conv(t, 0)
        conv(t, 1)
    _drain(st)
    check(st, inputs=list(rng(0, 16 * nt)))
    return st


def build16(nt=8):
    """S16, hidden layers only: in = the accumulators v[0 : 8 nt); tile t: v[8t : 8t+3] rows 0-15,
    v[8t+4 : 8t+7] rows 16-31; B operand of tile t v[8nt + 4t : +3]; A operands (halves 0, 1) and
    biases (8 registers) in two buffers each."""
    st = Stream(nt)
    ACC = lambda t, h: 8 * t + 4 * h
    KOP = lambda t: 8 * nt + 4 * t
    AOP = lambda b, h: 12 * nt + 8 * b + 4 * h
    BIAS = lambda b, h: 12 * nt + 16 + 8 * b + 4 * h

    def mfma(buf, t, h):
        d, a, b, c = ACC(t, h), AOP(buf, h), KOP(t), BIAS(buf, h)
        reads = [("A", r) for r in rng(a, 4)] + [("B", r) for r in rng(b, 4)] + [("C", r) for r in rng(c, 4)]
        st.pad("mfma", reads, list(rng(d, 4)))
        st.add(f"v_mfma_f32_16x16x32_bf16 v[{d}:{d + 3}], v[{a}:{a + 3}], v[{b}:{b + 3}], v[{c}:{c + 3}]", "mfma",
               reads=reads, writes=list(rng(d, 4)))

    def conv(t, h):  # half h of tile t's accumulators -> B-operand words 2h, 2h + 1
        for q in range(2):
            src, dst = ACC(t, h) + 2 * q, KOP(t) + 2 * h + q
            st.pad("valu", [src, src + 1], [dst])
            st.add(f"v_cvt_pk_bf16_f32 v{dst}, v{src}, v{src + 1} clamp", "valu", reads=[src, src + 1], writes=[dst])

    def load(dst, addr, off):
        st.pad("lds", (), list(rng(dst, 4)))
        st.add(f"ds_read_b128 v[{dst}:{dst + 3}], %[{addr}]" + (f" offset:{off}" if off else ""), "lds",
               writes=list(rng(dst, 4)))

    def loads(buf, j, part):
        if part == 0:
            load(AOP(buf, 0), "va", 2048 * j)
            load(AOP(buf, 1), "va", 2048 * j + 1024)
        else:
            load(BIAS(buf, 0), "vb", 128 * j)
            load(BIAS(buf, 1), "vb", 128 * j + 64)

    wait = lambda: st.add("s_waitcnt lgkmcnt(0)", "wait")
    loads(1, 0, 0)
    loads(1, 0, 1)
    for t in range(2):
        conv(t, 0)
        conv(t, 1)
    for l in range(1, NH + 1):
        buf, j, nxt = l % 2, l - 1, l < NH
        wait()
        for t in range(nt):
            for h in range(2):
                mfma(buf, t, h)
                # tile t + 2's conversions (two tiles ahead: a tile's one B operand takes both
                # halves' words, so one tile ahead left its last words just before its first MFMA)
                conv((t + 2) % nt, h)
                if nxt and (t, h) == (2, 0):
                    loads(1 - buf, j + 1, 0)
                elif nxt and (t, h) == (3, 0):
                    loads(1 - buf, j + 1, 1)
    for t in range(2, nt):
        conv(t, 0)
        conv(t, 1)
    _drain(st)
    check(st, inputs=list(rng(0, 8 * nt)))
    return st


def _drain(st):
    from gen_mlp_asm import MFMA_VALU_RAW, SRCAB_WAR, SRCC_WAR
    dist, need = 0, 0
    for text, k, rd, wr, states in reversed(st.ins):
        if k == "mfma":
            need = max(need, MFMA_VALU_RAW - dist, max(SRCC_WAR if role == "C" else SRCAB_WAR for role, _ in rd) - dist)
        dist += states
    st.nop(need)


def main():
    here = os.path.dirname(os.path.abspath(__file__))
    path = os.path.join(here, "mlp_shape_asm.h")
    parts = ["// mlp_shape_asm.h -- GENERATED by tools/gen_mlp_shape_asm.py (the MFMA-shape A/B streams; see there).",
             "#pragma once", ""]
    for name, st in (("NR_SHAPE_S32", build32()), ("NR_SHAPE_S16", build16())):
        nm = sum(1 for x in st.ins if x[1] == "mfma")
        nv = sum(1 for x in st.ins if x[1] == "valu")
        nl = sum(1 for x in st.ins if x[1] == "lds")
        nn = sum(x[4] for x in st.ins if x[1] == "nop")
        parts.append(f"// {len(st.ins)} instructions: {nm} MFMA, {nv} VALU, {nl} ds_read_b128, {nn} s_nop states")
        parts.append(f"#define {name} \\")
        parts.append(emit(st).replace("\n", " \\\n"))
        parts.append("")
    with open(path, "w") as f:
        f.write("\n".join(parts) + "\n")
    print(f"wrote {os.path.normpath(path)}")


if __name__ == "__main__":
    main()
