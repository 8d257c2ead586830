#!/usr/bin/env python3
"""Attribute a kernel's register spills to the kernel's phases.

Input: the device assembly of one kernel configuration built with
-gline-tables-only (tools/spill_attr.sh), whose .loc comments carry the
whole inlined-at chain.  For each kernel function in the file it prints

  * the resource notes (VGPRs, SGPRs, scratch, spills) from the .s metadata;
  * per phase (the outermost kernel function of the chain that names a phase:
    dp_solo, traceback, merge, ...): instructions, VGPR scratch spill stores /
    reloads, SGPR spill writelanes / readlanes (lanes of the compiler's spill
    VGPRs, which take immediate lane numbers), and the innermost source lines
    with the most spill traffic.

Static counts: a spill in a loop body counts once here; DESIGN.md pairs them
with the PMC per-row counts.

    python tools/spill_attr.py solo_g.s ccsx_amd/csrc/ccsx_kernel.hip [--json out.json]
"""
from __future__ import annotations

import argparse
import collections
import json
import re

PHASES = ["dp_solo", "dp_two_wave", "dp_wave_b", "dp_helper", "traceback", "merge", "columns_count", "call_columns",
          "find_breakpoint", "emit", "write_msa", "load_read", "stage_read", "win_load"]

FUNC_RE = re.compile(r"^(?:template\s*<[^>]*>\s*)?(?:__device__|__global__)[^(;]*?\b(\w+)\s*\(")


def source_functions(path: str):
    """[(first line, name)] of the kernel source's device functions."""
    out = []
    with open(path) as f:
        lines = f.readlines()
    for i, ln in enumerate(lines, 1):
        m = FUNC_RE.match(ln)
        if m and "{" in "".join(lines[i - 1:i + 8]):
            out.append((i, m.group(1)))
    return out


def func_of(funcs, line: int) -> str:
    name = "?"
    for start, n in funcs:
        if start > line:
            break
        name = n
    return name


LOC_CHAIN = re.compile(r"ccsx_kernel\.hip:(\d+):\d+")


def analyse(asm: str, src: str):
    funcs = source_functions(src)
    kernels = {}
    cur = None
    chain = []
    spill_vgprs = set()
    with open(asm) as f:
        lines = f.readlines()
    # spill VGPRs: written by v_writelane with an immediate lane
    for ln in lines:
        m = re.match(r"\s*v_writelane_b32 (v\d+), s\d+, (\d+)\s*$", ln.split(";")[0])
        if m:
            spill_vgprs.add(m.group(1))
    meta = {}
    for ln in lines:
        s = ln.strip()
        m = re.match(r"^(_Z\w+):", ln)
        if m and "ccsx_zmw_kernel" in m.group(1):
            cur = m.group(1)
            kernels[cur] = collections.defaultdict(lambda: collections.Counter())
            chain = []
            continue
        if s.startswith(".Lfunc_end"):
            cur = None
            continue
        if cur is None:
            for key in ("vgpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count", "private_segment_fixed_size",
                        ".name"):
                mm = re.match(r"^\s*\.?%s:\s+(\S+)" % re.escape(key.lstrip(".")), ln)
                if mm and ln.strip().startswith("." + key.lstrip(".")):
                    meta.setdefault("_pending", {})[key.lstrip(".")] = mm.group(1)
                    if key == ".name" and "ccsx_zmw_kernel" in mm.group(1) and not mm.group(1).endswith(".kd"):
                        meta[mm.group(1)] = meta.pop("_pending")
            continue
        if s.startswith(".loc"):
            if ";" in s:
                chain = [int(x) for x in LOC_CHAIN.findall(s.split(";", 1)[1])]
            continue
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        ins = s.split(";")[0].strip()
        op = ins.split()[0]
        names = [func_of(funcs, x) for x in reversed(chain)]  # outermost first
        phase = next((n for n in names if n in PHASES), "other")
        inner = f"{names[-1]}:{chain[0]}" if chain else "?"
        k = kernels[cur]
        k[phase]["insts"] += 1
        if op.startswith("scratch_store"):
            k[phase]["vgpr_spill_store"] += 1
            k[("line", phase)][inner] += 1
        elif op.startswith("scratch_load"):
            k[phase]["vgpr_spill_load"] += 1
            k[("line", phase)][inner] += 1
        elif op == "v_writelane_b32" and re.search(r"v_writelane_b32 (v\d+), s\d+, \d+$", ins) and \
                ins.split()[1].rstrip(",") in spill_vgprs:
            k[phase]["sgpr_spill_write"] += 1
            k[("sline", phase)][inner] += 1
        elif op == "v_readlane_b32" and re.search(r", (v\d+), \d+$", ins) and \
                re.search(r", (v\d+), \d+$", ins).group(1) in spill_vgprs:
            k[phase]["sgpr_spill_read"] += 1
            k[("sline", phase)][inner] += 1
    return kernels, meta, sorted(spill_vgprs, key=lambda v: int(v[1:]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("src")
    ap.add_argument("--json")
    ap.add_argument("--top", type=int, default=6)
    a = ap.parse_args()
    kernels, meta, spill_vgprs = analyse(a.asm, a.src)
    out = {"spill_vgprs": spill_vgprs, "kernels": {}}
    for kname, k in kernels.items():
        print(f"== {kname}  {meta.get(kname, {})}")
        print(f"   spill VGPRs (SGPR spill lanes): {len(spill_vgprs)}")
        rows = {}
        for ph in sorted((p for p in k if isinstance(p, str)), key=lambda p: -k[p]["insts"]):
            c = k[ph]
            rows[ph] = dict(c)
            print(f"   {ph:16s} insts {c['insts']:7d}  vgpr spill st/ld {c['vgpr_spill_store']:3d}/{c['vgpr_spill_load']:3d}"
                  f"  sgpr spill w/r {c['sgpr_spill_write']:4d}/{c['sgpr_spill_read']:4d}")
            for tag, title in (("line", "vgpr"), ("sline", "sgpr")):
                top = k[(tag, ph)].most_common(a.top)
                if top:
                    print(f"      {title} spills at: " + ", ".join(f"{l} x{n}" for l, n in top))
                    rows[ph][f"{title}_spill_lines"] = top
        out["kernels"][kname] = {"meta": meta.get(kname, {}), "phases": rows}
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
