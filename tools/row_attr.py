#!/usr/bin/env python3
"""Per-DP-row instruction attribution of the one-wave DP (dpS_row) from the
device assembly: static instruction counts of one FULL row (m >= W) of each
row class, by instruction type and by purpose, taken from the eight unrolled
rows of dpS_block (their inlined-at chains run through the unrolled call).

Input: the .s of one kernel configuration built with -gline-tables-only
(tools/row_attr.sh builds it).  Classes follow dpS_row / dpA_cold:

  fast0 / fast1   plain chain rows, band moved by 0 / 1 (predecessor cells by DPP)
  cold_*          dpA_cold's branches: far, chain (moved by 2 or spill-flagged),
                  np1, np2, gen (3-4 predecessors); each also runs the cold
                  instance of the row tail (cold_tail)
  row             the per-row bookkeeping both share: row info, band
                  placement's scalar chain, the fast / cold test, the
                  offset / key writelanes after the join

Static counts (a branchy path counts every alternative): pair them with
tools/row_kinds.py's class frequencies for a per-average-row estimate.

    python tools/row_attr.py solo16_g.s ccsx_amd/csrc/ccsx_kernel.hip [--json out.json]
"""
from __future__ import annotations

import argparse
import collections
import json
import re
import sys

LOC = re.compile(r"ccsx_kernel\.hip:(\d+):\d+")


def find_lines(src_path: str):
    """Source line numbers of the markers this attribution keys on."""
    src = open(src_path).read().split("\n")

    def line_of(pat, start=0, func=None):
        for i in range(start, len(src)):
            if re.search(pat, src[i]):
                return i + 1
        raise SystemExit(f"marker {pat!r} not found in {src_path}")
    m = {}
    m["dpS_row"] = line_of(r"__device__ __forceinline__ void dpS_row\(")
    m["dpS_block"] = line_of(r"__device__ __forceinline__ void dpS_block\(")
    m["dp_solo"] = line_of(r"__device__ __forceinline__ void dp_solo\(")
    m["dp_align"] = line_of(r"__device__ __forceinline__ void dp_align\(")
    m["dpA_cold"] = line_of(r"__device__ __forceinline__ void dpA_cold\(")
    m["row_record"] = line_of(r"__device__ __forceinline__ void row_record\(")
    # call sites
    m["full_call"] = line_of(r"dp_solo<true>\(", m["dp_align"])
    b = m["dpS_block"]
    m["unrolled_call"] = line_of(r"dpS_row<FULL>\(", b)
    r = m["dpS_row"]
    m["tail_sh0"] = line_of(r"tail\(coff, win_codes\(S\.qn, S\.pOff, 0\)", r)
    m["tail_sh1"] = line_of(r"tail\(coff, win_codes\(S\.qn, S\.pOff, 1\)", r)
    m["cold_call"] = line_of(r"dpA_cold<true>\(", r)
    m["tail_cold"] = line_of(r"tail\(off, qp, A, true\)", r)
    m["fast_if"] = line_of(r"if \(__builtin_expect\(fast, 1\)\)", r)
    m["row_end"] = line_of(r"^}", m["tail_cold"])
    c = m["dpA_cold"]
    m["c_far"] = line_of(r"far_terms<SLOTS>\(", c)
    m["c_chain"] = line_of(r"kind = 1;", c)
    m["c_np1"] = line_of(r"kind = 2;", c)
    m["c_np2"] = line_of(r"kind = 3;", c)
    m["c_gen"] = line_of(r"pred_terms<SLOTS>\(ring", c)
    m["c_end"] = line_of(r"off_o = off;", c)
    m["tail_begin"] = line_of(r"auto tail = \[&\]", r)
    return m, src


def itype(ins: str) -> str:
    op = ins.split()[0]
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith("s_cbranch") or op.startswith("s_branch") or op.startswith("s_setpc"):
        return "branch"
    if op.startswith("s_setprio") or op.startswith("s_barrier"):
        return "other"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_load") or op.startswith("s_buffer"):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu"
    return "other"


# purpose of an instruction by the source statement it comes from: the first
# line of its inlined-at chain inside the DP's own functions (the helpers --
# dpp, readlane, ring_val -- are attributed to their caller's statement)
RULES = [
    (r"S\.qn = rd_win16|rd_win16\(|win_codes\(", "read window"),
    (r"const int32_t j0 =|const int32_t srcu =|const int32_t src0 =", "source term"),
    (r"const bool mp0|const bool d0 = Dv0|const bool i0 =|const uint32_t hc0|const uint32_t hc1", "decision: code"),
    (r"const int32_t X1L|iext0 = |const int32_t ex1 = max\(Pex, X0\);$", "decision: iext"),
    (r"const int32_t M0 =|const int32_t M1 =|int32_t Dv0 = A|const int32_t hp0 =", "cells: M, D, H'"),
    (r"const int32_t X0 =|int32_t incl =|int32_t rk0 =|int32_t rk = max", "X, row key"),
    (r"wave_incl_max2|const int32_t Pex =", "scans (DPP)"),
    (r"int32_t nH0 =|ex1 \+ c\.cI1", "insertion, H"),
    (r"readlane\(rk, 63\)", "row key readlane"),
    (r"ring_store2|RingT \*row =", "ring store"),
    (r"nspill|sl < z\.d\.scap|rec\[256\]|int32_t \*rec =|reinterpret_cast<int2 \*>\(rec|kErrSpill|info & kInfoSpill", "spill record"),
    (r"S\.H0 = nH0|S\.pOff = off|S\.pArg =|row_key = key", "state, band chain"),
    (r"uint32_t w0 =|uint32_t w1 =", "record build"),
    (r"np > 63u|kExtWtag", "wide record"),
    (r"raw_buffer_store_b32\(w0", "record store"),
    (r"eb =|e0 = X0|e1 = X1|e01|bE|bKey|off == lim|c\.L2 == m - 1|readlane\(e1", "free-end"),
    (r"A\.Mh0 = |A\.Mh1 = |a0 = S\.|a1 = |A\.Dv0 = max|A\.ms0 = ", "pred terms (DPP)"),
    (r"A\.dx0 = ", "decision: D-ext"),
    (r"const uint32_t info =|const uint32_t base =|const uint32_t np =|const int32_t coff|const int32_t sh =|const uint32_t fast =|__builtin_expect\(fast", "row: info, band, fast test"),
    (r"S\.vOff = writelane|S\.vKey = writelane", "row: offset / key writelanes"),
]


def purpose(inner: int, m: dict, src: list) -> str:
    text = src[inner - 1].strip() if 0 < inner <= len(src) else ""
    for pat, name in RULES:
        if re.search(pat, text):
            return name
    if m["dpA_cold"] <= inner <= m["c_end"] + 2:
        return "cold: dispatch, placement"
    if 520 <= inner < m["dpA_cold"]:
        return "cold: pred reads / folds"
    return "other (" + text[:40] + ")"


def analyse(asm_path: str, src_path: str):
    m, src = find_lines(src_path)
    full = f"ccsx_kernel.hip:{m['full_call']}:"
    unr = f"ccsx_kernel.hip:{m['unrolled_call']}:"
    cls_site = {
        "fast0": m["tail_sh0"], "fast1": m["tail_sh1"],
    }
    cold_sites = {"cold_far": m["c_far"], "cold_chain": m["c_chain"], "cold_np1": m["c_np1"],
                  "cold_np2": m["c_np2"], "cold_gen": m["c_gen"]}
    counts = collections.defaultdict(lambda: collections.Counter())
    copies = set()  # inlined copies of the unrolled block (run_poa is inlined per mode)
    purposes = collections.defaultdict(lambda: collections.Counter())
    chain = ""
    inker = False
    for ln in open(asm_path):
        if re.match(r"^_Z\w*ccsx_zmw_kernel\w*:", ln):
            inker = True
            continue
        if not inker:
            continue
        if ln.startswith(".Lfunc_end"):
            break
        s = ln.strip()
        if s.startswith(".loc"):
            mm = re.search(r";\s*(.*)$", ln)
            chain = mm.group(1) if mm else ""
            continue
        if not s or s.startswith((".", ";")) or s.endswith(":"):
            continue
        if full not in chain or unr not in chain:
            continue
        lines = [int(x) for x in LOC.findall(chain)]
        inner = lines[0] if lines else 0
        for x in lines:  # the first frame inside the DP's own code
            if m["dpA_cold"] - 260 <= x <= m["row_end"] and not (60 <= x <= 160) and not (360 <= x <= 420):
                inner = x
                break
        copies.add(tuple(lines[lines.index(m["unrolled_call"]):]))
        # the dpS_row-level frame: the first chain entry inside dpS_row's body
        in_row = [x for x in lines if m["dpS_row"] <= x <= m["row_end"]]
        top = in_row[-1] if in_row else None  # outermost line within dpS_row
        cls = "row"
        if top is not None:
            if m["tail_begin"] <= top <= m["tail_cold"] - 30 and len(in_row) >= 2:
                # inside the tail lambda: which instance (the call site is the outermost)
                site = in_row[-1]
                cls = "row"
            if m["tail_sh0"] in lines:
                cls = "fast0"
            elif m["tail_sh1"] in lines:
                cls = "fast1"
            elif m["tail_cold"] in lines:
                cls = "cold_tail"
            elif m["cold_call"] in lines:
                cls = "cold_dispatch"
                dl = [x for x in lines if m["dpA_cold"] <= x <= m["c_end"]]
                if dl:
                    x = dl[-1]  # the dpA_cold statement this comes from
                    bounds = [("cold_far", m["c_far"] - 2, m["c_chain"] - 1), ("cold_chain", m["c_chain"] - 1, m["c_np1"] - 1),
                              ("cold_np1", m["c_np1"] - 1, m["c_np2"] - 1), ("cold_np2", m["c_np2"] - 1, m["c_np2"] + 13),
                              ("cold_gen", m["c_np2"] + 13, m["c_end"])]
                    for k, lo, hi in bounds:
                        if lo <= x < hi:
                            cls = k
            elif m["fast_if"] <= top < m["cold_call"]:
                # the fast rows' predecessor terms: which band move
                cls = "fast0" if top <= (m["fast_if"] + m["tail_sh1"]) // 2 else "fast1"
        t = itype(s)
        counts[cls][t] += 1
        if t in ("valu", "salu", "lds", "vmem"):
            purposes[cls][purpose(inner, m, src)] += 1
    return m, counts, purposes, len(copies)


def parse_blocks(asm_path: str):
    """The kernel's instructions in layout order as (label or None, text,
    chain) and a label -> index map."""
    ins, labels = [], {}
    chain, inker = "", False
    for ln in open(asm_path):
        if re.match(r"^_Z\w*ccsx_zmw_kernel\w*:", ln):
            inker = True
            continue
        if not inker:
            continue
        if ln.startswith(".Lfunc_end"):
            break
        s = ln.strip()
        if s.startswith(".loc"):
            mm = re.search(r";\s*(.*)$", ln)
            chain = mm.group(1) if mm else ""
            continue
        mlab = re.match(r"^(\.LBB\w+):", s)
        if mlab:
            labels[mlab.group(1)] = len(ins)
            continue
        if not s or s.startswith((".", ";")) or s.endswith(":"):
            continue
        ins.append((s.split(";")[0].strip(), chain))
    return ins, labels


def walk_fast(asm_path: str, m: dict, src: list):
    """Dynamic instruction path of one fast row of each band move (1 and 0)
    and of the per-row bookkeeping, on the FULL unrolled block's second row:
    from the row's join (the offset / key writelanes of the previous row)
    through the fast test, the fast row's straight line (conditional branches
    not taken: the rare paths -- off == lim, spill -- are laid out aside) to
    the next row's join."""
    ins, labels = parse_blocks(asm_path)
    full = f"ccsx_kernel.hip:{m['full_call']}:"
    unr = f"ccsx_kernel.hip:{m['unrolled_call']}:"
    wl = [i for i, (t, ch) in enumerate(ins) if full in ch and unr in ch and t.startswith("v_writelane")
          and re.search(r"ccsx_kernel\.hip:(\d+)", ch) and any(
              src[int(x) - 1].strip().startswith("S.vOff = writelane") for x in LOC.findall(ch))]
    if not wl:
        return None
    starts = sorted(labels.values())

    def block_start(i):
        b = 0
        for st in starts:
            if st > i:
                break
            b = st
        return b
    join_starts = {block_start(w) for w in wl}
    # the third join of the first copy: rows 2 -> 3 of the unrolled block
    j = block_start(wl[2] if len(wl) > 2 else wl[0])
    # back to the start of that join block's bookkeeping: after the previous s_branch / fast-row end
    out = {}

    def run(i, take_sh0):
        seq = []
        while i < len(ins) and len(seq) < 600:
            if seq and i in join_starts:
                break
            t, ch = ins[i]
            lines = [int(x) for x in LOC.findall(ch)]
            seq.append((t, ch))
            op = t.split()[0]
            if op == "s_branch":
                i = labels[t.split()[1]]
                continue
            if op.startswith("s_cbranch"):
                tgt = t.split()[1]
                # the sh == 0 test (dpS_row's `if (sh == 0)`) is the one branch taken for fast0
                is_sh = any(src[x - 1].strip().startswith("if (sh == 0)") for x in lines)
                is_fast = any("__builtin_expect(fast" in src[x - 1] for x in lines)
                if is_fast and op in ("s_cbranch_vccz", "s_cbranch_scc1", "s_cbranch_scc0"):
                    # the fast test: stay on the fast path (fall through when the branch leaves it)
                    pass
                if is_sh and take_sh0:
                    i = labels[tgt]
                    continue
                if op == "s_cbranch_execnz":  # the structurizer's joins: exec is never empty here
                    i = labels[tgt]
                    continue
            i += 1
        return seq

    for name, sh0 in (("fast1", False), ("fast0", True)):
        seq = run(j, sh0)
        c = collections.Counter(itype(t) for t, _ in seq)
        pc = collections.Counter()
        for t, ch in seq:
            if itype(t) in ("valu", "salu", "lds", "vmem"):
                lines = [int(x) for x in LOC.findall(ch)]
                inner = lines[0] if lines else 0
                for x in lines:
                    if m["dpA_cold"] - 260 <= x <= m["row_end"] and not (60 <= x <= 160) and not (360 <= x <= 420):
                        inner = x
                        break
                pc[purpose(inner, m, src)] += 1
        out[name] = {"types": dict(c), "purposes": dict(pc.most_common()), "listing": [t for t, _ in seq]}
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("src")
    ap.add_argument("--json")
    ap.add_argument("--unroll", type=int, default=8, help="rows per unrolled block (kBlkAB)")
    a = ap.parse_args()
    m, counts, purposes, ncopies = analyse(a.asm, a.src)
    U = a.unroll * ncopies
    print(f"{ncopies} inlined copies of the unrolled {a.unroll}-row block: counts / {U}")
    out = {"per_row_static": {}, "purposes": {}}
    order = ["row", "fast0", "fast1", "cold_dispatch", "cold_far", "cold_chain", "cold_np1", "cold_np2", "cold_gen",
             "cold_tail"]
    types = ["valu", "salu", "lds", "vmem", "branch", "waitcnt", "nop", "smem", "other"]
    print(f"{'class':14s} " + " ".join(f"{t:>7s}" for t in types))
    for k in order:
        if k not in counts:
            continue
        row = {t: round(counts[k][t] / U, 2) for t in types}
        out["per_row_static"][k] = row
        out["purposes"][k] = {p: round(v / U, 2) for p, v in purposes[k].most_common()}
        print(f"{k:14s} " + " ".join(f"{row[t]:7.2f}" for t in types))
    for k in order:
        if k in out["purposes"]:
            print(f"\n{k}: " + ", ".join(f"{p} {v}" for p, v in out["purposes"][k].items()))
    dyn = walk_fast(a.asm, m, open(a.src).read().split("\n"))
    if dyn:
        out["fast_row_path"] = dyn
        for k, v in dyn.items():
            t = v["types"]
            print(f"\n{k} row, dynamic path from the previous row's join (bookkeeping included): "
                  f"VALU {t.get('valu', 0)}, SALU {t.get('salu', 0)}, LDS {t.get('lds', 0)}, VMEM {t.get('vmem', 0)}, "
                  f"branch {t.get('branch', 0)}, waitcnt {t.get('waitcnt', 0)}, nop {t.get('nop', 0)}")
            print("   " + ", ".join(f"{p} {n}" for p, n in v["purposes"].items()))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
