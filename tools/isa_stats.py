#!/usr/bin/env python3
"""Static instruction counts of the gfx950 kernels in one HIP source, by class (MFMA, VALU, LDS,
global memory, scalar, s_nop), plus VGPR / spill figures from the assembler metadata. For before /
after comparisons of kernel changes (counts are static: a loop body counts once).
usage: isa_stats.py FILE.hip [KERNEL_SUBSTRING ...] [-D...]"""
import os
import re
import subprocess
import sys
import tempfile
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as g  # noqa: E402


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("v_permlane", "v_readlane", "v_writelane", "v_readfirstlane")):
        return "xlane"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op == "s_nop":
        return "s_nop"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    src = sys.argv[1]
    rest = sys.argv[2:]
    defs = [a for a in rest if a.startswith("-D")]
    keys = [a for a in rest if not a.startswith("-D")]
    with tempfile.TemporaryDirectory() as tmp:
        out = os.path.join(tmp, "k.s")
        cmd = [g.HIPCC] + g.HIP_FLAGS + g.EXTRA_FLAGS.get(os.path.basename(src), []) + defs + [
            "--cuda-device-only", "-S", src, "-o", out]
        g._run(cmd)
        text = open(out).read()
    # split into functions: "name:" label lines that start a .type'd function
    funcs = re.split(r"\n(?=[A-Za-z_][\w.$]*:\s*(?:;.*)?\n)", text)
    meta = {}
    for m in re.finditer(r"\.name:\s+(\S+)\n(?:.*\n)*?\s+\.sgpr_count:\s+(\d+)(?:.*\n)*?\s+\.vgpr_count:\s+(\d+)", text):
        meta[m.group(1)] = (int(m.group(2)), int(m.group(3)))
    for m in re.finditer(r"\.name:\s+(\S+)\n(?:.*\n)*?\s+\.private_segment_fixed_size:\s+(\d+)", text):
        pass
    rows = []
    for f in funcs:
        head = f.split("\n", 1)[0]
        name = head.split(":")[0].strip()
        if not name or name.startswith(".") or "kernel" not in name.lower() and "Kernel" not in name:
            continue
        if keys and not any(k in name for k in keys):
            continue
        c = Counter()
        lines = [ln.strip() for ln in f.split("\n")[1:]]
        for s in lines:
            if not s or s.startswith((";", ".", "//")) or s.endswith(":"):
                continue
            op = s.split()[0]
            c[classify(op)] += 1
        # the loop (label .. backward branch to it) holding the most MFMAs: the tile loop
        labels = {s.split(":")[0]: n for n, s in enumerate(lines) if s.startswith(".LBB") and ":" in s}
        best = None
        for n, s in enumerate(lines):
            if s.startswith("s_cbranch") or s.startswith("s_branch"):
                tgt = s.split()[-1]
                if tgt in labels and labels[tgt] < n:
                    body = lines[labels[tgt]:n + 1]
                    lc = Counter(classify(b.split()[0]) for b in body
                                 if b and not b.startswith((";", ".", "//")))
                    if best is None or lc["mfma"] > best["mfma"] or (lc["mfma"] == best["mfma"] and lc["valu"] > best["valu"]):
                        best = lc
        c["loop"] = best
        if c["mfma"] + c["valu"] == 0 and not keys:
            continue
        spill = re.search(r"; ScratchSize: (\d+)", f)
        vg = re.search(r"; NumVgprs: (\d+)", f)
        ag = re.search(r"; NumAgprs: (\d+)", f)
        rows.append((name, c, spill.group(1) if spill else "?", vg.group(1) if vg else "?", ag.group(1) if ag else "?"))
    for name, c, spill, vg, ag in rows:
        short = re.sub(r"^_ZN4nerf", "", name)[:70]
        ratio = c["valu"] / c["mfma"] if c["mfma"] else float("nan")
        print(f"{short:70s} mfma {c['mfma']:5d} valu {c['valu']:6d} ({ratio:5.2f}:1) lds {c['lds']:5d} vmem {c['vmem']:4d} "
              f"xlane {c['xlane']:3d} salu {c['salu']:5d} nop {c['s_nop']:4d} wait {c['waitcnt']:4d} vgpr {vg} agpr {ag} scratch {spill}")
        lc = c["loop"]
        if lc:
            print(f"{'  largest loop':70s} mfma {lc['mfma']:5d} valu {lc['valu']:6d} lds {lc['lds']:5d} vmem {lc['vmem']:4d} "
                  f"xlane {lc['xlane']:3d} salu {lc['salu']:5d} nop {lc['s_nop']:4d} wait {lc['waitcnt']:4d}")


if __name__ == "__main__":
    main()
