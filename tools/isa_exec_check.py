"""ISA audit: cross-lane consumers whose operands were written under a partial EXEC.

    python tools/isa_exec_check.py KERNEL.s SYMBOL_SUBSTRING

MFMA, v_permlane*_swap, ds_bpermute/ds_permute and v_readlane read lanes other than the
writer's own, so a source VGPR whose reaching definitions were all executed with some
lanes disabled hands those lanes' stale contents to the consumer.  This reconstructs the
CFG of one function in a gfx950 assembly listing (hipcc --cuda-device-only -S), tracks
whether EXEC is the whole wave or a subset at each instruction (structurised if / else /
loop idioms: s_and_saveexec, s_xor exec, s_or exec, s_andn2 exec + execnz back edges,
s_mov exec), runs reaching definitions per VGPR in which a partial-EXEC write adds a
definition without killing the earlier ones, and reports every cross-lane source whose
reaching definitions include a partial write.  A report is a lead, not a verdict: the
stale lanes may be don't-care columns.
"""
import re
import sys
from collections import defaultdict

CROSS = re.compile(r"^(v_mfma|v_smfmac|v_permlane|ds_bpermute|ds_permute|v_readlane|v_readfirstlane|v_mov_b32_dpp|.*_dpp)")
NODEST = re.compile(r"^(ds_write|ds_store|global_store|flat_store|buffer_store|scratch_store|s_|v_cmp_|v_cmpx_|exp|v_readlane|v_readfirstlane)")


def regs(tok):
    tok = tok.strip()
    m = re.fullmatch(r"v(\d+)", tok)
    if m:
        return [int(m.group(1))]
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return list(range(int(m.group(1)), int(m.group(2)) + 1))
    return []


def parse(lines, sym):
    start = None
    for i, l in enumerate(lines):
        if l.startswith(sym) and l.rstrip().endswith(sym + ":") or (l.split(":")[0] == sym):
            start = i
            break
    if start is None:
        cands = [i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and sym in l]
        start = cands[0]
    end = next(i for i in range(start + 1, len(lines)) if lines[i].strip().startswith("s_endpgm"))
    body = []
    for i in range(start + 1, end + 1):
        s = lines[i].split(";")[0].rstrip()
        if not s.strip():
            continue
        if re.match(r"^\.LBB\S*:", s.strip()) or re.match(r"^\.LBB\S*:", s):
            body.append((i + 1, "label", s.strip()[:-1], []))
            continue
        if s.startswith("\t") or s.startswith(" "):
            parts = s.strip().split(None, 1)
            op = parts[0]
            args = [a.strip() for a in re.split(r",(?![^\[]*\])", parts[1])] if len(parts) > 1 else []
            body.append((i + 1, "ins", op, args))
    return body


def build_blocks(body):
    blocks, cur, labels = [], [], {}
    for it in body:
        if it[1] == "label":
            if cur:
                blocks.append(cur)
            cur = []
            labels[it[2]] = len(blocks)
            cur.append(it)
            continue
        cur.append(it)
        if it[2].startswith("s_cbranch") or it[2] in ("s_branch", "s_endpgm"):
            blocks.append(cur)
            cur = []
    if cur:
        blocks.append(cur)
    # re-map labels to block indices
    labels = {}
    for bi, b in enumerate(blocks):
        for it in b:
            if it[1] == "label":
                labels[it[2]] = bi
    succ = defaultdict(list)
    for bi, b in enumerate(blocks):
        last = [x for x in b if x[1] == "ins"]
        last = last[-1] if last else None
        if last and last[2] == "s_branch":
            succ[bi].append(labels[last[3][0]])
        elif last and last[2].startswith("s_cbranch"):
            succ[bi].append(labels[last[3][0]])
            if bi + 1 < len(blocks):
                succ[bi].append(bi + 1)
        elif last and last[2] == "s_endpgm":
            pass
        elif bi + 1 < len(blocks):
            succ[bi].append(bi + 1)
    return blocks, succ


def exec_states(blocks, succ):
    """Forward dataflow over (exec_full, origin): origin maps an SGPR pair that a region
    opened with (saveexec destination, loop break mask, a copy of exec) to whether EXEC was
    the whole wave when that region began; closing the region (s_or_b64 exec, exec, X)
    restores that state.  Joins: partial wins; origins kept only where both sides agree."""
    def tr(state, op, args):
        full, origin = state
        origin = dict(origin)
        a0 = args[0] if args else ""
        if op in ("s_and_saveexec_b64", "s_andn2_saveexec_b64"):
            origin[a0] = full
            return False, tuple(sorted(origin.items()))
        if op == "s_or_saveexec_b64":  # else-start: exec |= src (the region's lanes come back)
            f = origin.get(args[1], False)
            origin[a0] = f
            return f, tuple(sorted(origin.items()))
        if op == "s_mov_b64" and a0 == "exec":
            return bool(origin.get(args[1], False)) and False, tuple(sorted(origin.items()))
        if op == "s_mov_b64" and len(args) > 1 and args[1] == "exec":
            origin[a0] = full
            return full, tuple(sorted(origin.items()))
        if op == "s_or_b64" and a0 == "exec":
            other = args[2] if args[1] == "exec" else args[1]
            return (full or bool(origin.get(other, False))), tuple(sorted(origin.items()))
        if op == "s_andn2_b64" and a0 == "exec" and args[1] == "exec":
            origin.setdefault(args[2], full)
            return False, tuple(sorted(origin.items()))
        if op in ("s_and_b64", "s_xor_b64", "s_or_b64", "s_andn2_b64", "s_mov_b64") and a0 == "exec":
            return False, tuple(sorted(origin.items()))
        if op.startswith("v_cmpx"):
            return False, tuple(sorted(origin.items()))
        return full, tuple(sorted(origin.items()))

    def join(a, b):
        da, db = dict(a[1]), dict(b[1])
        o = {k: da[k] and db[k] for k in da if k in db}
        return (a[0] and b[0], tuple(sorted(o.items())))

    IN = {0: (True, ())}
    work = [0]
    per_ins = {}
    while work:
        bi = work.pop()
        st = IN[bi]
        for it in blocks[bi]:
            if it[1] != "ins":
                continue
            per_ins[it[0]] = st[0] if it[0] not in per_ins else (per_ins[it[0]] and st[0])
            st = tr(st, it[2], it[3])
        ins = [x for x in blocks[bi] if x[1] == "ins"]
        last = ins[-1] if ins else None
        for s in succ[bi]:
            ns = st
            if last and last[2] == "s_cbranch_execnz":
                ns = (False, st[1])
            old = IN.get(s)
            if old is None:
                IN[s] = ns
                work.append(s)
            else:
                j = join(old, ns)
                if j != old:
                    IN[s] = j
                    work.append(s)
    return per_ins


def dests_srcs(op, args):
    if op.startswith("v_permlane16_swap") or op.startswith("v_permlane32_swap"):
        r = regs(args[0]) + regs(args[1])
        return r, r
    if NODEST.match(op):
        srcs = [x for a in args for x in regs(a)]
        if op.startswith("v_readlane") or op.startswith("v_readfirstlane"):
            srcs = [x for a in args[1:] for x in regs(a)]
        return [], srcs
    if op.startswith("global_atomic") or op.startswith("flat_atomic") or op.startswith("buffer_atomic"):
        if "sc0" in args[-1] or "glc" in " ".join(args):
            return regs(args[0]), [x for a in args[1:] for x in regs(a)]
        return [], [x for a in args for x in regs(a)]
    if op.startswith("v_writelane"):
        return regs(args[0]), [x for a in args[1:] for x in regs(a)]
    if op.startswith("v_") or op.startswith("ds_") or op.startswith("global_load") or op.startswith("flat_load") \
            or op.startswith("buffer_load") or op.startswith("scratch_load"):
        d = regs(args[0]) if args else []
        return d, [x for a in args[1:] for x in regs(a)]
    return [], []


def main():
    path, sym = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    body = parse(lines, sym)
    blocks, succ = build_blocks(body)
    full_at = exec_states(blocks, succ)
    # reaching definitions: per block, gen/kill with partial writes non-killing
    defs_of = {}
    for b in blocks:
        for it in b:
            if it[1] == "ins":
                d, _ = dests_srcs(it[2], it[3])
                partial = (not full_at.get(it[0], True)) or it[2].startswith("v_writelane")
                defs_of[it[0]] = (d, partial)
    pred = defaultdict(list)
    for b, ss in succ.items():
        for s in ss:
            pred[s].append(b)
    IN = [dict() for _ in blocks]
    OUT = [dict() for _ in blocks]

    def transfer(bi, inmap):
        m = {k: set(v) for k, v in inmap.items()}
        for it in blocks[bi]:
            if it[1] != "ins":
                continue
            d, partial = defs_of[it[0]]
            for r in d:
                if partial:
                    m.setdefault(r, set()).add(it[0])
                else:
                    m[r] = {it[0]}
        return m

    changed = True
    while changed:
        changed = False
        for bi in range(len(blocks)):
            inm = {}
            for p in pred[bi]:
                for r, s in OUT[p].items():
                    inm.setdefault(r, set()).update(s)
            out = transfer(bi, inm)
            if out != OUT[bi]:
                OUT[bi] = out
                changed = True
            IN[bi] = inm
    nrep = 0
    for bi, b in enumerate(blocks):
        m = {k: set(v) for k, v in IN[bi].items()}
        for it in b:
            if it[1] != "ins":
                continue
            op, args = it[2], it[3]
            d, srcs = dests_srcs(op, args)
            if CROSS.match(op) and full_at.get(it[0], True):
                cs = srcs
                if op.startswith("v_mfma") or op.startswith("v_smfmac"):
                    cs = [x for a in args[1:3] for x in regs(a)]  # A and B read every lane
                bad = []
                for r in cs:
                    rd = m.get(r, set())
                    pd = [x for x in rd if defs_of[x][1]]
                    if pd:
                        fulls = [x for x in rd if not defs_of[x][1]]
                        bad.append((r, sorted(pd), sorted(fulls)))
                if bad:
                    nrep += 1
                    print(f"line {it[0]}: {op} {', '.join(args)}")
                    for r, pd, fu in bad:
                        print(f"    v{r}: partial defs at {pd[:6]}{'...' if len(pd) > 6 else ''}; full defs {fu[:6]}")
            partial = defs_of[it[0]][1]
            for r in d:
                if partial:
                    m.setdefault(r, set()).add(it[0])
                else:
                    m[r] = {it[0]}
    print(f"{nrep} cross-lane instructions with partial-EXEC reaching definitions "
          f"({sum(1 for v in full_at.values() if not v)} of {len(full_at)} instructions under partial EXEC)")


if __name__ == "__main__":
    main()
