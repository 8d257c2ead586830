"""Build oracle/_ref/ -- TEST INFRASTRUCTURE ONLY.

Compiles the reference's own subread-ingest sources (seqio.h, kseq.h,
kstring.c, bamlite.c under /root/reference, unmodified, compiled where they
lie) with this project's driver oracle/ref_seqio_driver.c into
oracle/_ref/ref_seqio.  Nothing else of the reference builds here: main.c
needs bsalign's dna.h / bsalign.h / bspoa.h, which are not vendored
(DESIGN.md §1), so it is treated as unbuildable.

Only tests/ and tools/make_host_golden.py run the result.
"""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("CCSX_REFERENCE", "/root/reference")
OUT = os.path.join(HERE, "_ref", "ref_seqio")


def build_ref(force: bool = False) -> str | None:
    srcs = [os.path.join(REF, f) for f in ("kstring.c", "bamlite.c")]
    if not all(os.path.exists(s) for s in srcs + [os.path.join(REF, "seqio.h")]):
        return None  # e.g. on the GPU box: the reference does not travel
    drv = os.path.join(HERE, "ref_seqio_driver.c")
    if not force and os.path.exists(OUT) and os.path.getmtime(OUT) >= os.path.getmtime(drv):
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    cmd = ["gcc", "-O2", "-w", "-D_FILE_OFFSET_BITS=64", "-D_GNU_SOURCE", "-I", REF, drv, *srcs, "-o", OUT, "-lz"]
    subprocess.run(cmd, check=True)
    return OUT


if __name__ == "__main__":
    print(build_ref(force=True))
