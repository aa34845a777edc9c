"""Scan a gfx950 assembly file (hipcc -S) for packed-fp32 VALU reads of a VGPR that a VALU
instruction wrote a few instructions earlier (round 6).

For every v_pk_{fma,mul,add}_f32 it finds, per source operand, the nearest earlier writer of each
of its two registers inside the same straight-line block, the writer's kind (VALU / packed VALU /
LDS / VMEM / MFMA / SALU-move) and the distance in instructions, and which half (op_sel /
op_sel_hi) each lane reads.  Reported: the reads whose writer is a non-packed VALU at distance
<= --window (default 2), the pattern of the round-4 two-process mismatch.

    python tools/pkhaz/pk_hazard_scan.py file.s <kernel substring | ALL> [--window 2] [--brief]
"""
import argparse
import collections
import re

PK = re.compile(r"^\s*(v_pk_(?:fma|mul|add)_f32)\s+(v\[\d+:\d+\]),\s*(.+)$")
REG = re.compile(r"v\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(tok):
    out = []
    for m in REG.finditer(tok):
        if m.group(1):
            out += list(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.append(int(m.group(3)))
    return out


def kind(op):
    if "mfma" in op:
        return "mfma"
    if op.startswith("v_pk_"):
        return "pkvalu"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def kernel_lines(path, name):
    s = open(path).read().split("\n")
    start = next(i for i, l in enumerate(s) if re.match(r"^\S+:", l) and name in l and not l.startswith("."))
    end = next(i for i in range(start + 1, len(s)) if s[i].startswith(".Lfunc_end"))
    return s[start + 1:end]


def scan(lines, window):
    hist = []  # (op, dst regs) since the last label / branch
    hits, counts = [], collections.Counter()
    for ln in lines:
        t = ln.split(";")[0].strip()
        if not t:
            continue
        if t.endswith(":") or t.startswith(("s_branch", "s_cbranch", "s_setpc", "s_swappc")):
            hist = []  # block boundary: start over (conservative: no cross-block writer)
            continue
        op = t.split()[0]
        if op.startswith("."):
            continue
        args = t[len(op):].strip()
        m = PK.match(t)
        if m:
            counts[op] += 1
            counts["pk_total"] += 1
            dst, rest = m.group(2), m.group(3)
            parts = [p.strip() for p in rest.split(",")]
            srcs = [p for p in parts if p.startswith("v[") or re.match(r"^v\d+$", p)][:3]
            sel = re.search(r"op_sel:\[([01,]+)\]", t)
            selhi = re.search(r"op_sel_hi:\[([01,]+)\]", t)
            sel = [int(x) for x in sel.group(1).split(",")] if sel else [0, 0, 0]
            selhi = [int(x) for x in selhi.group(1).split(",")] if selhi else [1, 1, 1]
            for si, src in enumerate(srcs):
                r = regs(src)
                lo_reads = r[sel[si]] if len(r) > 1 else r[0]
                hi_reads = r[selhi[si]] if len(r) > 1 else r[0]
                bcast = len(r) > 1 and lo_reads == hi_reads  # one register of the pair read by both lanes
                for lane, reg in (("lo", lo_reads), ("hi", hi_reads)):
                    for d, (wop, wregs) in enumerate(reversed(hist)):
                        if reg in wregs:
                            if kind(wop) == "valu" and d < window:
                                hits.append((t, si, lane, reg, wop, d))
                                if bcast and lane == "lo":
                                    counts["bcast_of_fresh_valu"] += 1
                                    if wop.startswith("v_mov_b32"):
                                        counts["bcast_of_fresh_v_mov (the r4 sa_pre_kernel sequence)"] += 1
                            break
        dregs = regs(args.split(",")[0]) if args and (op.startswith("v_") or op.startswith(("ds_read", "global_load", "buffer_load", "flat_load", "scratch_load"))) else []
        hist.append((op, set(dregs)))
    return hits, counts


def kernels(path):
    return [m.group(1) for m in re.finditer(r"^(_Z\S+):", open(path).read(), re.M)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel")
    ap.add_argument("--window", type=int, default=2)
    ap.add_argument("--brief", action="store_true", help="one line per kernel")
    a = ap.parse_args()
    names = kernels(a.asm) if a.kernel == "ALL" else [a.kernel]
    for name in names:
        hits, counts = scan(kernel_lines(a.asm, name), a.window)
        if not counts["pk_total"]:
            continue
        print(f"{name[:90]}: packed fp32 ops {dict(counts)}; reads of a VALU result within {a.window} "
              f"instructions: {len(hits)}")
        if not a.brief:
            for t, si, lane, reg, wop, d in hits:
                print(f"  src{si} {lane}-lane v{reg} <- {wop} at distance {d}: {t}")


if __name__ == "__main__":
    main()
