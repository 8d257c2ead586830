#!/usr/bin/env python3
"""Resource notes of every kernel code object in a library (VGPRs, SGPRs,
spills, scratch, LDS), read from the AMDGPU metadata notes of the gfx950
code objects bundled in its .hip_fatbin section (llvm-objcopy + the clang
offload-bundle header + llvm-readelf --notes); no GPU needed.

    python tools/kernel_notes.py ccsx_amd/libccsx_amd.so [--json out.json] [--md out.md]
"""
from __future__ import annotations

import argparse
import json
import os
import re
import struct
import subprocess
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
KEYS = ("vgpr_count", "agpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
        "private_segment_fixed_size", "group_segment_fixed_size")


def code_objects(lib: str):
    """The amdgcn code objects (bytes) of every offload bundle in the library."""
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", f".hip_fatbin={fat}", lib, os.devnull],
                       check=True)
        data = open(fat, "rb").read()
    out = []
    for m in re.finditer(re.escape(MAGIC), data):
        b = m.start()
        n = struct.unpack_from("<Q", data, b + 24)[0]
        p = b + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tl].decode()
            p += 24 + tl
            if "amdgcn" in triple and size:
                out.append(data[b + off:b + off + size])
    return out


def notes(obj: bytes):
    """{kernel name: {key: value}} from one code object's metadata note."""
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(obj)
        f.flush()
        txt = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", f.name], capture_output=True,
                             text=True).stdout
    res, cur = {}, {}
    for line in txt.splitlines():
        s = line.strip().lstrip("- ").strip()
        m = re.match(r"\.(\w+):\s+(.*)$", s)
        if not m:
            continue
        k, v = m.group(1), m.group(2).strip()
        if k == "name" and not v.endswith(".kd"):
            cur = {}
            res[v] = cur
        elif k in KEYS and cur is not None:
            cur[k] = int(v)
    # the note lists each kernel's keys before its .name in some versions:
    # keep only complete entries
    return {k: v for k, v in res.items() if v}


def demangle(k: str) -> str:
    """_ZN4ccsx<n><ns><n><name>E... -> ns::name"""
    m = re.match(r"_ZN4ccsx(\d+)", k)
    if not m:
        return k
    p = m.end()
    n = int(m.group(1))
    ns = k[p:p + n]
    m2 = re.match(r"(\d+)", k[p + n:])
    if not m2:
        return k
    q = p + n + len(m2.group(1))
    return f"{ns}::{k[q:q + int(m2.group(1))]}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--json")
    ap.add_argument("--md")
    a = ap.parse_args()
    allk = {}
    for co in code_objects(a.lib):
        allk.update(notes(co))
    rows = sorted((k, v) for k, v in allk.items() if "ccsx_zmw_kernel" in k)
    lines = ["| kernel | VGPRs | SGPRs | VGPR spills | SGPR spills | scratch B/lane | static LDS |", "|---|---|---|---|---|---|---|"]
    for k, v in rows:
        lines.append(f"| {demangle(k)} | {v.get('vgpr_count')} | {v.get('sgpr_count')} | {v.get('vgpr_spill_count')} | "
                     f"{v.get('sgpr_spill_count')} | {v.get('private_segment_fixed_size')} | "
                     f"{v.get('group_segment_fixed_size')} |")
    print("\n".join(lines))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(dict(rows), f, indent=1)
    if a.md:
        with open(a.md, "w") as f:
            f.write(f"# Kernel resource notes: {os.path.basename(a.lib)}\n\n"
                    "From the gfx950 code objects' AMDGPU metadata (tools/kernel_notes.py).\n\n" + "\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
