"""Wait-state lint for the hand-written inline asm of the inflate kernel (gfx950).

LLVM's hazard recognizer pads the code it generates, but not for an inline-asm consumer of a
register the compiler wrote just before it (e.g. an SGPR restored from a spill by v_readlane).
This scans the compiler's assembly (hipcc --cuda-device-only -S) and, for every instruction
between ;;#ASMSTART and ;;#ASMEND, checks the instructions before it:

  * a VMEM instruction reading an SGPR base (saddr) needs 5 wait states after a VALU write of it;
  * global_load_lds_* reads M0: 1 wait state after a SALU write, 5 after a VALU write;
  * v_readlane / v_writelane with an SGPR or M0 lane select: 4 wait states after a VALU write.

A plain instruction counts one wait state, s_nop N counts N + 1.  The scan runs backwards over
every predecessor path: at a label it follows both the fall-through predecessor (unless that is an
unconditional s_branch) and every branch that jumps to the label (s_branch / s_cbranch_*, named
.LBB labels and the asm's numeric local labels "1b"/"1f"), and takes the fewest wait states over
all paths.  Exit status 1 lists the violations.
(Found with amdgpu_num_sgpr(64): a spilled far-load base restored right before the load faulted.)

  python tools/hazard_lint.py file.s [kernel-name-substring]
"""
import re
import sys

SREG = re.compile(r"\bs\[(\d+):(\d+)\]|\bs(\d+)\b|\b(m0)\b|\b(vcc)\b")


def sregs(tok):
    out = set()
    for m in SREG.finditer(tok):
        if m.group(1):
            out |= {f"s{i}" for i in range(int(m.group(1)), int(m.group(2)) + 1)}
        elif m.group(3):
            out.add(f"s{m.group(3)}")
        elif m.group(4):
            out.add("m0")
    return out


def parse(line):
    s = line.split(";")[0].strip()
    if not s or s.startswith("."):
        if s.startswith(".L") and s.endswith(":"):
            return ("label", s[:-1])
        return None
    if s.endswith(":"):
        return ("label", s[:-1])
    parts = s.split(None, 1)
    ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
    return parts[0], ops


BRANCH = re.compile(r"s_(branch|cbranch_\w+)$")


def writes(mn, ops):
    """(kind, registers written) for VALU / SALU instructions."""
    if not ops:
        return None, set()
    if mn.startswith("v_"):
        dst = sregs(ops[0])
        if re.match(r"v_(add|sub|subrev)_co|v_(addc|subb|subbrev)_co|v_mad_(u|i)64|v_div_scale", mn) and len(ops) > 1:
            dst |= sregs(ops[1])
        return "valu", dst
    if mn.startswith("s_") and not re.match(r"s_(nop|waitcnt|cbranch|branch|barrier|setprio|sleep|endpgm|dcache|icache)", mn):
        return "salu", sregs(ops[0])
    return None, set()


def needs(mn, ops):
    """[(registers, wait states after VALU write, after SALU write)] this asm instruction reads."""
    out = []
    if mn.startswith("global_") or mn.startswith("buffer_") or mn.startswith("scratch_"):
        for o in ops[1:]:
            r = sregs(o)
            if r:
                out.append((r, 5, 0))
        if "_lds_" in mn:
            out.append(({"m0"}, 5, 1))
    if mn in ("v_readlane_b32", "v_writelane_b32") and len(ops) >= 3:
        r = sregs(ops[2])
        if r:
            out.append((r, 4, 0))
    return out


def lint(lines, kernel=None):
    in_kernel = kernel is None
    insts = []          # (index in file, mnemonic or "label", ops or label name, in_asm)
    in_asm = False
    for i, line in enumerate(lines):
        if kernel is not None and re.match(r"^[_A-Za-z0-9.$]+:", line):
            name = line.split(":")[0]
            if not name.startswith(".L"):
                in_kernel = kernel in name
        if not in_kernel:
            continue
        if "ASMSTART" in line:
            in_asm = True
            continue
        if "ASMEND" in line:
            in_asm = False
            continue
        p = parse(line)
        if p:
            insts.append((i, p[0], p[1], in_asm))
    # branch sources of every label position: named labels anywhere, numeric local labels
    # ("1:" referenced as "1b" / "1f") resolved to the nearest one before / after the branch
    labels = {}
    numeric = {}
    for k, (_, mn, op, _) in enumerate(insts):
        if mn == "label":
            labels.setdefault(op, k)
            if op.isdigit():
                numeric.setdefault(op, []).append(k)
    preds = {}
    for k, (_, mn, ops, _) in enumerate(insts):
        if mn == "label" or not BRANCH.match(mn) or not ops:
            continue
        tgt = ops[-1]
        m = re.fullmatch(r"(\d+)([bf])", tgt)
        if m:
            cands = numeric.get(m.group(1), [])
            before = [c for c in cands if c < k]
            after = [c for c in cands if c > k]
            t = (before[-1] if before else None) if m.group(2) == "b" else (after[0] if after else None)
        else:
            t = labels.get(tgt)
        if t is not None:
            preds.setdefault(t, []).append(k)

    def fewest(k, regs, need_v, need_s, ws, seen):
        """(wait states, writer index) on the worst path back from instruction k, or None."""
        worst = None
        j = k - 1
        while j >= 0:
            _, mj, oj, _ = insts[j]
            if mj == "label":
                for src in preds.get(j, []):
                    if (src, ws) in seen:
                        continue
                    seen.add((src, ws))
                    r = fewest(src + 1, regs, need_v, need_s, ws, seen)   # the branch itself is the predecessor
                    if r and (worst is None or r[0] < worst[0]):
                        worst = r
                prev = insts[j - 1][1] if j > 0 else None
                if prev == "s_branch":
                    return worst
                j -= 1
                continue
            kind, w = writes(mj, oj)
            if w & regs:
                need = need_v if kind == "valu" else need_s
                if ws < need and (worst is None or ws < worst[0]):
                    worst = (ws, j, need)
                return worst
            ws += (int(oj[0], 0) + 1 if oj else 1) if mj == "s_nop" else 1
            if ws >= 5:
                return worst
            j -= 1
        return worst

    bad = []
    for k, (i, mn, ops, asm) in enumerate(insts):
        if not asm or mn == "label":
            continue
        for regs, need_v, need_s in needs(mn, ops):
            r = fewest(k, regs, need_v, need_s, 0, set())
            if r:
                ws, j, need = r
                bad.append((i + 1, mn, " ".join(ops), insts[j][0] + 1, insts[j][1], ws, need))
    return bad


if __name__ == "__main__":
    lines = open(sys.argv[1]).read().splitlines()
    bad = lint(lines, sys.argv[2] if len(sys.argv) > 2 else None)
    for line, mn, ops, wl, wm, ws, need in bad:
        print(f"line {line}: {mn} {ops}: written by {wm} at line {wl}, {ws} wait states < {need}")
    print(f"hazard_lint: {len(bad)} violation(s)")
    sys.exit(1 if bad else 0)
