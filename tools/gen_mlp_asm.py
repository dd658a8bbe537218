"""Generates cudaneuralrender_amd/csrc/nr_mlp16_asm.h: the 16-bit MLP's hidden layers for four
32-point tiles (128 points per wave, k_mlp16) and for two (64 points, the tracer's march MLP:
k_trace) as software-pipelined instruction streams.

Why: compiled from builtins, every hidden layer issued its 8 MFMAs back to
back and then converted all four tiles' accumulators (32 v_cvt_pk) with no MFMA in flight, so a
wave alone kept the matrix pipe ~55 % busy and the waves of a SIMD, sharing the pipe, fell into
step.  Here the conversion of tile t + 1 runs in the shadow of tile t's two MFMAs, and the next
layer's tile 0 in the shadow of tile 3's, so one wave alone keeps the pipe nearly full:

    layer l:  M(l,0,0) C(l,1)s0  M(l,0,1) C(l,1)s1  M(l,1,0) C(l,2)s0 ...  M(l,3,0) C(l+1,0)s0  M(l,3,1) C(l+1,0)s1

M(l,t,s) = v_mfma_f32_32x32x16_{bf16,f16} of layer l, tile t, k-step s (s = 0 takes the bias as
its accumulator init, s = 1 the s = 0 result); C(l,t)s = the 4 v_cvt_pk (bf16: with the clamp bit
that is the ReLU on the clamped pack; otherwise + v_pk_max_i16) that turn registers 8s..8s+7 of
tile t's accumulator into the B operand of k-step s.  Every instruction and operand is the one the
builtin form issues, so the outputs are bit-identical; only the order changes.  With two tiles
the same pattern puts the next layer's tile-0 conversions right behind tile 0's own MFMAs, so
s_nop padding (inserted here wherever a distance falls short, then checked) covers the MFMA ->
VALU distance the other two tiles' MFMAs covered.

The stream runs inside one inline-asm statement, so the compiler neither pads its hazards nor
counts its LDS reads: this script places the operand reads (ds_read_b128 of the next layer's A
operands and biases into the idle one of two register buffers, one layer ahead) and CHECKS every
hazard of the stream before it writes the header (check()).  The registers are pinned
("{v[a:b]}" constraints), for NT tiles: accumulators v[0 : 16NT), B operands v[16NT : 24NT), A
operands 16 from v[24NT], biases 32 from v[24NT + 16] (four tiles: v0-v63, v64-v95, v96-v111,
v112-v143; two: v0-v31, v32-v47, v48-v63, v64-v95).

Run:  python tools/gen_mlp_asm.py   (writes the header; the CPU test suite checks it is current)
"""
import os
import sys

NH = 7                       # hidden layers of the bundled networks (others take the builtin form)


class Layout:
    """Pinned registers of an NT-tile stream."""
    def __init__(self, nt):
        self.nt = nt

    def ACC(self, t):            # accumulator of tile t: v[16t : 16t+15]
        return 16 * t

    def KOP(self, t, s):         # B operand of tile t, k-step s: 4 registers
        return 16 * self.nt + 8 * t + 4 * s

    def AOP(self, b, s):         # A operand of buffer b, k-step s: 4 registers
        return 24 * self.nt + 8 * b + 4 * s

    def BIAS(self, b):           # bias (accumulator init) of buffer b: 16 registers
        return 24 * self.nt + 16 + 16 * b

# hazard distances (wait states = instructions issued between producer and consumer; s_nop N
# counts N + 1).  MFMA_VALU_RAW: hipcc's own gfx950 padding of v_mfma_f32_32x32x16 -> VALU read
# is 12 (nr_trace.hip disassembly: MFMA, s_nop 10, read); one more here as margin.  The WAR rows
# are conservative (the ISA's 8-pass SrcC value is smaller).
MFMA_VALU_RAW = 13
VALU_MFMA_RAW = 3
SRCC_WAR = 16
SRCAB_WAR = 8
# v_permlane16/32_swap reading a register a VALU instruction wrote (LLVM's gfx950 hazard rule
# "VALU write vdst -> v_permlane read", cdna_hip_programming.md T21): 2 wait states.  Otherwise a
# swap is a VALU instruction that reads and writes both of its registers.
PERM_RAW = 2


class Stream:
    def __init__(self, nt=4, raw=None):
        self.ins = []   # (text, kind, reads, writes, states)
        self.nt = nt
        self.raw = MFMA_VALU_RAW if raw is None else raw   # MFMA -> VALU read distance of its MFMAs

    def add(self, text, kind, reads=(), writes=(), states=1):
        self.ins.append((text, kind, tuple(reads), tuple(writes), states))

    def nop(self, need):
        while need > 0:
            n = min(need, 16)
            self.add(f"s_nop {n - 1}", "nop", states=n)
            need -= n

    def pad(self, kind, reads=(), writes=()):
        """Appends the s_nop an instruction of `kind` reading / writing these registers needs after
        the stream so far (the distances check() enforces)."""
        regs = [r if isinstance(r, int) else r[1] for r in reads]
        need, dist = 0, 0
        for text, k, rd, wr, states in reversed(self.ins):
            if dist >= SRCC_WAR:
                break
            if k == "mfma" and kind != "mfma":
                if any(r in wr for r in regs) or any(r in wr for r in writes):
                    need = max(need, self.raw - dist)
                for role, r in rd:
                    if r in writes:
                        need = max(need, (SRCC_WAR if role == "C" else SRCAB_WAR) - dist)
            elif k in ("valu", "perm") and kind == "mfma" and any(r in wr for r in regs):
                need = max(need, VALU_MFMA_RAW - dist)
            elif k in ("valu", "perm") and kind == "perm" and any(r in wr for r in regs):
                need = max(need, PERM_RAW - dist)
            dist += states
        self.nop(need)


def rng(a, n):
    return range(a, a + n)


def build(prec, clamp, nt=4):
    dt = "bf16" if prec == "bf16" else "f16"
    st = Stream(nt)
    L = Layout(nt)
    ACC, KOP, AOP, BIAS = L.ACC, L.KOP, L.AOP, L.BIAS

    def mfma(buf, t, s, layer0=False):
        d = ACC(t)
        a = AOP(buf, 0) if layer0 else AOP(buf, s)
        b = KOP(t, s)
        c = BIAS(buf) if (layer0 or s == 0) else ACC(t)
        reads = [("A", r) for r in rng(a, 4)] + [("B", r) for r in rng(b, 4)] + [("C", r) for r in rng(c, 16)]
        st.pad("mfma", reads, list(rng(d, 16)))
        st.add(f"v_mfma_f32_32x32x16_{dt} v[{d}:{d + 15}], v[{a}:{a + 3}], v[{b}:{b + 3}], v[{c}:{c + 15}]", "mfma",
               reads=reads, writes=list(rng(d, 16)))

    def conv(t, s):
        for q in range(4):
            src = ACC(t) + 8 * s + 2 * q
            dst = KOP(t, s) + q
            st.pad("valu", [src, src + 1], [dst])
            if prec == "bf16" and clamp:
                st.add(f"v_cvt_pk_bf16_f32 v{dst}, v{src}, v{src + 1} clamp", "valu", reads=[src, src + 1], writes=[dst])
            else:
                cvt = "v_cvt_pk_bf16_f32" if prec == "bf16" else "v_cvt_pk_f16_f32"
                st.add(f"{cvt} v{dst}, v{src}, v{src + 1}", "valu", reads=[src, src + 1], writes=[dst])
                st.add(f"v_pk_max_i16 v{dst}, v{dst}, 0", "valu", reads=[dst], writes=[dst])

    def load(dst, addr, off):
        o = f" offset:{off}" if off else ""
        st.pad("lds", (), list(rng(dst, 4)))
        st.add(f"ds_read_b128 v[{dst}:{dst + 3}], %[{addr}]{o}", "lds", writes=list(rng(dst, 4)))

    def a_loads(buf, j):       # hidden layer j's A operands (both k-steps) into buffer buf
        load(AOP(buf, 0), "va", 1024 + 2048 * j)
        load(AOP(buf, 1), "va", 2048 + 2048 * j)

    def b_load(buf, j, i):     # quarter i of hidden layer j's bias into buffer buf
        load(BIAS(buf) + 4 * i, "vb", 128 + 128 * j + 16 * i)

    wait = lambda: st.add("s_waitcnt lgkmcnt(0)", "wait")
    # ---- layer 0 (buffer 0): its A operand (k-step-0 slot) and bias; the B operands are inputs
    load(AOP(0, 0), "va", 0)
    for i in range(4):
        load(BIAS(0) + 4 * i, "vb", 16 * i)
    wait()
    mfma(0, 0, 0, layer0=True)
    a_loads(1, 0)
    mfma(0, 1, 0, layer0=True)
    for i in range(4):
        b_load(1, 0, i)
    for t in range(2, nt):
        mfma(0, t, 0, layer0=True)
    conv(0, 0)
    conv(0, 1)
    # ---- hidden layers l = 1..NH (hidden layer j = l - 1, buffer l % 2); the next layer's
    # operands go to the other buffer once this layer's MFMAs no longer read the old ones there
    for l in range(1, NH + 1):
        buf, j, nxt = l % 2, l - 1, l < NH
        wait()
        for t in range(nt):
            for s in range(2):
                mfma(buf, t, s)
                conv(t + 1 if t < nt - 1 else 0, s)   # tile t + 1 of this layer, or tile 0 of the next
                if nxt and nt == 2 and (t, s) == (0, 0):
                    # two tiles: all of the next layer's operands right after this layer's first
                    # MFMA -- a whole layer (4 MFMAs) ahead of their use; the other buffer's last
                    # readers, the previous layer's tile-1 MFMAs, are just far enough back
                    a_loads(1 - buf, j + 1)
                    for i in range(4):
                        b_load(1 - buf, j + 1, i)
                elif nxt and nt == 4:
                    if (t, s) == (1, 0):
                        a_loads(1 - buf, j + 1)
                    elif (t, s) == (1, 1):
                        b_load(1 - buf, j + 1, 0)
                    elif (t, s) == (2, 0):
                        b_load(1 - buf, j + 1, 1)
                    elif (t, s) == (2, 1):
                        b_load(1 - buf, j + 1, 2)
                        b_load(1 - buf, j + 1, 3)
    # ---- tail: the final layer's B operands of tiles 1.. (tile 0's ran beside M(NH, nt - 1, *)),
    # then whatever padding the exit needs: no MFMA of the stream in flight when it ends
    for t in range(1, nt):
        conv(t, 0)
        conv(t, 1)
    dist, need = 0, 0
    for text, k, rd, wr, states in reversed(st.ins):
        if k == "mfma":
            need = max(need, MFMA_VALU_RAW - dist, max(SRCC_WAR if role == "C" else SRCAB_WAR for role, _ in rd) - dist)
        dist += states
    st.nop(need)
    check(st)
    return st


def build_s16(prec, clamp):
    """k_mlp16's 128-point MLP with the hidden layers on v_mfma_f32_16x16x32 (round 6, VERDICT r5
    item 1): the input layer as in build() (four 32-point tiles, v_mfma_f32_32x32x16), its outputs
    re-dealt to eight 16-point tiles by one v_permlane16_swap per word pair, the 7 hidden layers as
    two 16x16x32 MFMAs (output rows 0-15 and 16-31) per 16-point tile, and the last hidden layer's
    outputs re-dealt to the 32-point tiles' B operands by the same swaps, where the final layer (the
    caller's v_dot2c chains) reads them as it reads build()'s.

    Same values as build(), bit for bit: a 16x16x32 MFMA sums its K = 32 as two chained K = 16
    steps of the matrix core's 8-product blocks (profiles/r5_mfma_peak_random.txt (4)), and the
    pack (nr_pack.cpp pack_lowp_s16) orders the hidden units so that lane group g of a B operand
    holds the block the 32x32x16 form sums g-th; the input layer's rows are permuted so that the
    swap lands each block in its group, the last hidden layer's so that the swap back gives the
    32x32x16 form's final-layer operands.  Lane (j, g) of 16-point tile t: point 16t + j, block g.

    Registers: accumulators v0-v63 (16-point tile t: v[8t:8t+3] rows 0-15, v[8t+4:8t+7] rows
    16-31; 32-point tile T: v[16T:16T+15]), B operands v64-v95 (16-point tile t: v[64+4t:+3]; in:
    the input layer's B operand of 32-point tile T at v[64+8T:+3]; out: 32-point tile T's final
    operands, k-step s at v[64+8T+4s:+3] -- build()'s interface), A operands v96-v111 and biases
    v112-v127 (two buffers each); the input layer's bias is read into v48-v63, the accumulator of
    32-point tile 3, whose MFMA then accumulates in place.  %[va] = LDS byte address of the A
    operands + 16 lane, %[vb0] = of the biases + 64 (lane >> 5) (the input layer's 32-point
    layout), %[vb] = + 32 (lane >> 4) (the hidden layers': [group 4][half 2][4] per layer)."""
    dt = "bf16" if prec == "bf16" else "f16"
    st = Stream(8)
    ACC = lambda t, h: 8 * t + 4 * h
    ACC32 = lambda T: 16 * T
    KOP = lambda t: 64 + 4 * t
    AOP = lambda b, h: 96 + 8 * b + 4 * h
    BIAS = lambda b, h: 112 + 8 * b + 4 * h
    L0B = 48

    def cvt(dst, src):
        st.pad("valu", [src, src + 1], [dst])
        if prec == "bf16" and clamp:
            st.add(f"v_cvt_pk_bf16_f32 v{dst}, v{src}, v{src + 1} clamp", "valu", reads=[src, src + 1], writes=[dst])
        else:
            c = "v_cvt_pk_bf16_f32" if prec == "bf16" else "v_cvt_pk_f16_f32"
            st.add(f"{c} v{dst}, v{src}, v{src + 1}", "valu", reads=[src, src + 1], writes=[dst])
            st.add(f"v_pk_max_i16 v{dst}, v{dst}, 0", "valu", reads=[dst], writes=[dst])

    def mfma32(T):
        d, a, b, c = ACC32(T), AOP(0, 0), KOP(2 * T), L0B
        reads = [("A", r) for r in rng(a, 4)] + [("B", r) for r in rng(b, 4)] + [("C", r) for r in rng(c, 16)]
        st.pad("mfma", reads, list(rng(d, 16)))
        st.add(f"v_mfma_f32_32x32x16_{dt} v[{d}:{d + 15}], v[{a}:{a + 3}], v[{b}:{b + 3}], v[{c}:{c + 15}]", "mfma",
               reads=reads, writes=list(rng(d, 16)))

    def mfma16(buf, t, h):
        d, a, b, c = ACC(t, h), AOP(buf, h), KOP(t), BIAS(buf, h)
        reads = [("A", r) for r in rng(a, 4)] + [("B", r) for r in rng(b, 4)] + [("C", r) for r in rng(c, 4)]
        st.pad("mfma", reads, list(rng(d, 4)))
        st.add(f"v_mfma_f32_16x16x32_{dt} v[{d}:{d + 3}], v[{a}:{a + 3}], v[{b}:{b + 3}], v[{c}:{c + 3}]", "mfma",
               reads=reads, writes=list(rng(d, 4)))

    def conv32(T, s):   # input layer, 32-point tile T, registers 8s..8s+7 -> 16-point tile 2T + s's slots
        for q in range(4):
            cvt(KOP(2 * T + s) + q, ACC32(T) + 8 * s + 2 * q)

    def conv16(t, h):   # half h of 16-point tile t's accumulators -> B-operand words 2h, 2h + 1
        for q in range(2):
            cvt(KOP(t) + 2 * h + q, ACC(t, h) + 2 * q)

    def swap(T, q):     # word q of 16-point tiles 2T, 2T + 1 <-> 32-point tile T's k-steps 0, 1
        a, b = KOP(2 * T) + q, KOP(2 * T + 1) + q
        st.pad("perm", [a, b], [a, b])
        st.add(f"v_permlane16_swap_b32 v{a}, v{b}", "perm", reads=[a, b], writes=[a, b])

    def load(dst, addr, off):
        st.pad("lds", (), list(rng(dst, 4)))
        st.add(f"ds_read_b128 v[{dst}:{dst + 3}], %[{addr}]" + (f" offset:{off}" if off else ""), "lds",
               writes=list(rng(dst, 4)))

    def a_loads(buf, j):
        load(AOP(buf, 0), "va", 1024 + 2048 * j)
        load(AOP(buf, 1), "va", 2048 + 2048 * j)

    def b_loads(buf, j):
        load(BIAS(buf, 0), "vb", 128 + 128 * j)
        load(BIAS(buf, 1), "vb", 128 + 128 * j + 16)

    wait = lambda: st.add("s_waitcnt lgkmcnt(0)", "wait")
    # ---- input layer (32-point tiles); hidden layer 0's operands (buffer 1) load beside it
    load(AOP(0, 0), "va", 0)
    for i in range(4):
        load(L0B + 4 * i, "vb0", 16 * i)
    wait()
    mfma32(0)
    a_loads(1, 0)
    mfma32(1)
    b_loads(1, 0)
    mfma32(2)
    mfma32(3)
    conv32(0, 0)
    conv32(0, 1)
    for q in range(4):
        swap(0, q)
    # ---- hidden layers l = 1..NH (j = l - 1, buffer l % 2), the conversions two 16-point tiles
    # ahead; in layer 1 the input layer's 32-point tiles 1-3 are converted and swapped instead
    for l in range(1, NH + 1):
        buf, j, nxt = l % 2, l - 1, l < NH
        wait()
        for t in range(8):
            for h in range(2):
                mfma16(buf, t, h)
                if l == 1 and t < 6:
                    T = t // 2 + 1
                    if t % 2 == 0:
                        conv32(T, h)
                    else:
                        swap(T, 2 * h)
                        swap(T, 2 * h + 1)
                else:
                    conv16((t + 2) % 8, h)
                if nxt and (t, h) == (2, 0):
                    a_loads(1 - buf, j + 1)
                elif nxt and (t, h) == (3, 0):
                    b_loads(1 - buf, j + 1)
    # ---- the last hidden layer's outputs: tiles 2-7 converted, every pair swapped back
    for q in range(4):
        swap(0, q)
    for T in range(1, 4):
        for s in range(2):
            conv16(2 * T + s, 0)
            conv16(2 * T + s, 1)
        for q in range(4):
            swap(T, q)
    dist, need = 0, 0
    for text, k, rd, wr, states in reversed(st.ins):
        if k == "mfma":
            need = max(need, MFMA_VALU_RAW - dist, max(SRCC_WAR if role == "C" else SRCAB_WAR for role, _ in rd) - dist)
        dist += states
    st.nop(need)
    check(st, inputs=[r for T in range(4) for r in rng(KOP(2 * T), 4)])
    return st


# v_mfma_f32_16x16x4_f32 -> VALU read: hipcc pads 10 wait states on gfx950 (its minimum over the
# fp32 tracer's listing); two more here as margin
F32_MFMA_VALU_RAW = 12


def build_f32(nt):
    """The fp32 MLP's 7 hidden layers (clamped ReLU, the scaled pack: nr_mlp16.h mlp16_fp32_nt<NT, 0,
    true>) for NT <= 2 16-point tiles as one stream (round 6, VERDICT r5 item 4: the latency of a
    wave with few rays, the single frame's tail).  The compiled form issues a layer's 16 NT MFMAs,
    then waits for the last, then converts all 8 NT accumulators and only then requests the next
    layer's weights, so every layer boundary costs an MFMA drain, the ReLUs and an LDS round trip
    with the matrix pipe idle.  Here (the same instructions and operands, so the same values):
      * the next layer's weights and bias are read into the other of two register buffers during
        this layer (its first MFMAs / after its deferred ReLUs);
      * the accumulators alternate between two buffers by layer, so that the ReLU of row tile 1
        (units 16-31 = k-steps 4-7 of the next layer) is deferred until the next layer's k-steps
        0-3 have issued: at a boundary only row tile 0's four ReLUs stand between the last MFMA
        and the next one.
    MFMA(l, st, mt, t): acc(l % 2, t, mt) (+)= W[2 st + mt] x act(t, st), k-step st = 0 from 0 --
    the k-ascending fmaf chain of every output, as the compiled form.  Registers: accumulators
    v[0 : 16 NT) (buffer b, tile t, row tile mt at 8 NT b + 8 t + 4 mt), activations v[16 NT : 24 NT)
    (tile t, k-step st at 16 NT + 8 t + st: in = layer 0's ReLU'd outputs, out = the last hidden
    layer's), weights 2 x 16 from v[24 NT], biases 2 x 8 after them.  %[va] = LDS byte address of
    the pack's hidden layers + 16 lane, %[vb] = of their biases + 32 (lane >> 4)."""
    st = Stream(nt, raw=F32_MFMA_VALU_RAW)
    ACC = lambda b, t, mt: 8 * nt * b + 8 * t + 4 * mt
    ACT = lambda t, s: 16 * nt + 8 * t + s
    W = lambda b: 24 * nt + 16 * b
    BIAS = lambda b: 24 * nt + 32 + 8 * b
    STRIDE = 4 * (1024 + 32)   # bytes per hidden layer in the pack (nr_internal.h PK_HID_STRIDE)

    def load(dst, addr, off):
        o = f" offset:{off}" if off else ""
        st.pad("lds", (), list(rng(dst, 4)))
        st.add(f"ds_read_b128 v[{dst}:{dst + 3}], %[{addr}]{o}", "lds", writes=list(rng(dst, 4)))

    def w_loads(b, j):
        for q in range(4):
            load(W(b) + 4 * q, "va", j * STRIDE + 1024 * q)

    def b_loads(b, j):
        load(BIAS(b), "vb", j * STRIDE)
        load(BIAS(b) + 4, "vb", j * STRIDE + 16)

    def mfma(l, s, mt, t):
        b = l % 2
        d, a, bb = ACC(b, t, mt), W(b) + 2 * s + mt, ACT(t, s)
        reads = [("A", a), ("B", bb)] + ([("C", r) for r in rng(d, 4)] if s else [])
        st.pad("mfma", reads, list(rng(d, 4)))
        c = f"v[{d}:{d + 3}]" if s else "0"
        st.add(f"v_mfma_f32_16x16x4_f32 v[{d}:{d + 3}], v{a}, v{bb}, {c}", "mfma", reads=reads, writes=list(rng(d, 4)))

    def relu(l, mt):
        b = l % 2
        for t in range(nt):
            for r in range(4):
                src, bias, dst = ACC(b, t, mt) + r, BIAS(b) + 4 * mt + r, ACT(t, 4 * mt + r)
                st.pad("valu", [src, bias], [dst])
                st.add(f"v_add_f32_e64 v{dst}, v{src}, v{bias} clamp", "valu", reads=[src, bias], writes=[dst])

    wait = lambda: st.add("s_waitcnt lgkmcnt(0)", "wait")
    w_loads(0, 0)
    b_loads(0, 0)
    for l in range(NH):
        wait()
        nxt = l < NH - 1
        for s in range(8):
            if s == 4:
                if l > 0:
                    relu(l - 1, 1)              # the previous layer's row tile 1 -> k-steps 4-7
                if nxt:
                    b_loads((l + 1) % 2, l + 1)  # (its bias buffer's last reader was that ReLU)
            for mt in range(2):
                for t in range(nt):
                    mfma(l, s, mt, t)
            if s == 0 and nxt:
                w_loads((l + 1) % 2, l + 1)      # (the other buffer's readers: layer l - 1's MFMAs)
        relu(l, 0)                              # row tile 0 -> the next layer's k-steps 0-3
    relu(NH - 1, 1)
    dist, need = 0, 0
    for text, k, rd, wr, states in reversed(st.ins):
        if k == "mfma":
            need = max(need, max(SRCC_WAR if role == "C" else SRCAB_WAR for role, _ in rd) - dist)
        dist += states
    st.nop(need)
    check(st, inputs=[ACT(t, s) for t in range(nt) for s in range(8)])
    return st


def check(st, inputs=None):
    """Verifies every hazard of the stream (raises on the first violation).  inputs: the registers
    the compiler's VALU wrote just before the stream (default: the k-step-0 B operands)."""
    L = Layout(getattr(st, "nt", 4))
    pos = []   # wait-state position of each instruction
    p = 0
    for ins in st.ins:
        pos.append(p)
        p += ins[4]
    # the input B operands (k-step 0 slots) were written by the compiler's VALU just before the stream
    if inputs is None:
        inputs = [r for t in range(L.nt) for r in rng(L.KOP(t, 0), 4)]
    last_w = {r: (-1, "valu") for r in inputs}
    last_r = {}      # reg -> list of (index, operand role) of MFMA reads since the last write
    pending = set()  # regs with an LDS load not yet waited for
    for i, (text, kind, reads, writes, _) in enumerate(st.ins):
        if kind == "wait":
            pending.clear()
            continue
        regs_read = [r if isinstance(r, int) else r[1] for r in reads]
        for r in regs_read:
            if r in pending:
                raise AssertionError(f"{i}: {text}: reads v{r} before its LDS load is waited for")
            if r in last_w:
                wi, wk = last_w[r]
                dist = pos[i] - (pos[wi] + st.ins[wi][4]) if wi >= 0 else pos[i]   # states in between
                if wk == "mfma" and kind != "mfma" and dist < st.raw:
                    raise AssertionError(f"{i}: {text}: reads v{r} {dist} states after MFMA {wi}")
                if wk in ("valu", "perm") and kind == "mfma" and dist < VALU_MFMA_RAW:
                    raise AssertionError(f"{i}: {text}: reads v{r} {dist} states after VALU {wi}")
                if wk in ("valu", "perm") and kind == "perm" and dist < PERM_RAW:
                    raise AssertionError(f"{i}: {text}: swaps v{r} {dist} states after VALU {wi}")
                if wk == "mfma" and kind == "mfma":
                    # only an exact accumulate chain (same registers as C) may follow an MFMA
                    role = [x[0] for x in reads if x[1] == r][0]
                    if role != "C":
                        raise AssertionError(f"{i}: {text}: MFMA operand {role} v{r} written by MFMA {wi}")
        for r in writes:
            for (ri, role) in last_r.get(r, []):
                dist = pos[i] - (pos[ri] + st.ins[ri][4])
                need = SRCC_WAR if role == "C" else SRCAB_WAR
                if kind != "mfma" and dist < need:
                    raise AssertionError(f"{i}: {text}: writes v{r} {dist} states after MFMA {ri} read it as {role}")
            if r in last_w and last_w[r][1] == "mfma" and kind != "mfma":
                wi = last_w[r][0]
                if pos[i] - (pos[wi] + st.ins[wi][4]) < st.raw:
                    raise AssertionError(f"{i}: {text}: overwrites v{r} too soon after MFMA {wi}")
        for r in writes:
            last_w[r] = (i, kind)
            last_r[r] = []
            if kind == "lds":
                pending.add(r)
        if kind == "mfma":
            for role, r in reads:
                last_r.setdefault(r, []).append((i, role))
    if pending:
        raise AssertionError("LDS loads left outstanding at the end of the stream")
    # nothing in flight at the exit: the compiler may read or overwrite any register right after
    for r, (wi, wk) in last_w.items():
        if wk == "mfma" and p - (pos[wi] + st.ins[wi][4]) < st.raw:
            raise AssertionError(f"v{r}: MFMA {wi} may still be writing it when the stream ends")
    for r, lst in last_r.items():
        for (ri, role) in lst:
            if p - (pos[ri] + st.ins[ri][4]) < (SRCC_WAR if role == "C" else SRCAB_WAR):
                raise AssertionError(f"v{r}: MFMA {ri} may still be reading it when the stream ends")


def emit(st):
    out = []
    for text, kind, *_ in st.ins:
        out.append(f'    "{text}\\n"')
    return "\n".join(out)


def main():
    here = os.path.dirname(os.path.abspath(__file__))
    path = os.path.join(here, "..", "cudaneuralrender_amd", "csrc", "nr_mlp16_asm.h")
    parts = [
        "// nr_mlp16_asm.h -- GENERATED by tools/gen_mlp_asm.py (do not edit; rerun the script).",
        "// The 16-bit MLP's input layer + 7 hidden layers + the final layer's operand conversion for",
        "// four 32-point tiles as one software-pipelined stream (see the script's docstring).",
        "// Registers: accumulators v0-v63 (tile t: v[16t:16t+15]), B operands v64-v95 (tile t, k-step s:",
        "// v[64+8t+4s:+3]; in: the input layer's B operands in k-step 0's slot; out: the ReLU'd final",
        "// operands), A operands v96-v111 and biases v112-v143 (two buffers each); %[va] = LDS byte",
        "// address of the A operands + 16 lane, %[vb] = of the biases + 64 (lane >> 5).",
        "#pragma once",
        "",
    ]
    for name, prec, clamp, nt in (("NR_HID7_BF16_CLAMP", "bf16", True, 4), ("NR_HID7_BF16_MAX", "bf16", False, 4),
                                  ("NR_HID7_F16_MAX", "fp16", False, 4)):
        st = build(prec, clamp, nt)
        nm = sum(1 for x in st.ins if x[1] == "mfma")
        nv = sum(1 for x in st.ins if x[1] == "valu")
        nn = sum(x[4] for x in st.ins if x[1] == "nop")
        parts.append(f"// {prec}, {nt} tiles, {'clamped' if clamp else 'max'} ReLU: {len(st.ins)} instructions, {nm} MFMA, "
                     f"{nv} VALU, {nn} s_nop states")
        parts.append(f"#define {name} \\")
        parts.append(emit(st).replace("\n", " \\\n") + "")
        parts.append("")
    parts += [
        "// 16x16x32 hidden layers for k_mlp16 (build_s16): the same interface and values; registers",
        "// v0-v127 (accumulators v0-v63, B operands v64-v95, A operands v96-v111, biases v112-v127);",
        "// %[vb0] = LDS byte address of the biases + 64 (lane >> 5), %[vb] = + 32 (lane >> 4).",
        "",
    ]
    for name, prec, clamp in (("NR_S16_BF16_CLAMP", "bf16", True), ("NR_S16_BF16_MAX", "bf16", False),
                              ("NR_S16_F16_MAX", "fp16", False)):
        st = build_s16(prec, clamp)
        nm = sum(1 for x in st.ins if x[1] == "mfma")
        nv = sum(1 for x in st.ins if x[1] in ("valu", "perm"))
        nn = sum(x[4] for x in st.ins if x[1] == "nop")
        parts.append(f"// {prec}, 8 x 16-point tiles, {'clamped' if clamp else 'max'} ReLU: {len(st.ins)} instructions, "
                     f"{nm} MFMA, {nv} VALU, {nn} s_nop states")
        parts.append(f"#define {name} \\")
        parts.append(emit(st).replace("\n", " \\\n") + "")
        parts.append("")
    parts += [
        "// The fp32 MLP's 7 hidden layers, clamped ReLU, for NT = 1, 2 16-point tiles (build_f32): the",
        "// compiled form's instructions and operands, software-pipelined; registers v[0 : 24 NT + 48)",
        "// (accumulators v[0 : 16 NT), activations v[16 NT : 24 NT) in and out, weights and biases after);",
        "// %[va] = LDS byte address of the pack's hidden layers + 16 lane, %[vb] = of their biases + 32 (lane >> 4).",
        "",
    ]
    for nt in (1, 2):
        st = build_f32(nt)
        nm = sum(1 for x in st.ins if x[1] == "mfma")
        nv = sum(1 for x in st.ins if x[1] == "valu")
        nn = sum(x[4] for x in st.ins if x[1] == "nop")
        parts.append(f"// fp32, {nt} tile(s): {len(st.ins)} instructions, {nm} MFMA, {nv} VALU, {nn} s_nop states")
        parts.append(f"#define NR_F32_HID7_NT{nt} \\")
        parts.append(emit(st).replace("\n", " \\\n") + "")
        parts.append("")
    text = "\n".join(parts) + "\n"
    if len(sys.argv) > 1 and sys.argv[1] == "--check":
        with open(path) as f:
            if f.read() != text:
                sys.exit("nr_mlp16_asm.h is stale: rerun tools/gen_mlp_asm.py")
        return
    with open(path, "w") as f:
        f.write(text)
    print(f"wrote {os.path.normpath(path)}")


if __name__ == "__main__":
    main()
