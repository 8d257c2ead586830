"""Build the in-tree native libraries.

* ``ccsx_amd/libccsx_amd.so`` -- the product: the gfx950 HIP kernel, its
  batched C-ABI (include/ccsx_gpu.h), the bspoa-compatible API
  (include/ccsx_bspoa.h) and the host preparation code (include/ccsx_host.h).
  Compiled with ``hipcc --offload-arch=gfx950``; works without a GPU present.
* ``ccsx_amd/bin/ccsx`` -- the C host program (ccsx's CLI, main.c:723-870).
* ``oracle/liboracle.so`` -- the CPU restatement used as the checker by the
  tests and bench.py's cpu_baseline leg (test infrastructure, not shipped).

Incremental: a target is rebuilt only when one of its sources is newer.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
INC = os.path.join(ROOT, "include")
OBJ = os.path.join(ROOT, "build", "obj")
LIB = os.path.join(HERE, "libccsx_amd.so")
BIN = os.path.join(HERE, "bin", "ccsx")
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "liboracle.so")

ARCH = os.environ.get("CCSX_OFFLOAD_ARCH", "gfx950")
# the kernel configurations (ccsx_layout.h KernelCfg): latency (8-row DP
# blocks, 32-row ring), occupancy (4-row blocks, 24-row ring), throughput
# (two-wave workgroups) and solo (one-wave workgroups)
KCFGS = [(n, [f"-DCCSX_KCFG={n}", f"-DCCSX_LAUNCH=ccsx_launch_zmw_{n}", f"-DCCSX_INFO=ccsx_kcfg_info_{n}"] + d)
         for n, d in [("lat", ["-DCCSX_RINGA=32", "-DCCSX_BLK=8"]),
                      ("occ", ["-DCCSX_RINGA=24", "-DCCSX_BLK=4"]),
                      # two-wave workgroups, a 16-row ring read back 8 rows
                      # no issue priorities: two wave 0s share each SIMD (A/B r03g: D 567 -> 550 ms)
                      ("tput", ["-DCCSX_RINGA=16", "-DCCSX_BLK=4", "-DCCSX_RING=8", "-DCCSX_HELPERS=1",
                                "-DCCSX_PRIO_WAVE0=0", "-DCCSX_PRIO_MERGE=0"]),
                      # one-wave workgroups (dp_solo), an 8-row ring, one traceback buffer;
                      # 8-row blocks (no barriers: only the unrolling; A/B r03u: D 363.6 -> 356.8 ms)
                      ("solo", ["-DCCSX_RINGA=8", "-DCCSX_BLK=8", "-DCCSX_RING=8", "-DCCSX_HELPERS=0",
                                "-DCCSX_PRIO_WAVE0=0", "-DCCSX_PRIO_MERGE=0", "-DCCSX_PRIO_TB=1", "-DCCSX_PRIO_MG=1"]),
                      # the solo object with an int16 ring (exact for reads <= 16,256 bases), one 16-row
                      # traceback block and 96 VGPRs: ~5.5 KB of LDS, 20 workgroups per CU
                      ("solo16", ["-DCCSX_RINGA=8", "-DCCSX_BLK=8", "-DCCSX_RING=8", "-DCCSX_HELPERS=0",
                                  "-DCCSX_PRIO_WAVE0=0", "-DCCSX_PRIO_MERGE=0", "-DCCSX_PRIO_TB=1", "-DCCSX_PRIO_MG=1",
                                  "-DCCSX_RING16", "-DCCSX_TB_ROWS=32",
                                  "-DCCSX_WAVES_PER_EU=5"]),
                      # solo16 at 80 VGPRs: 24 workgroups per CU, for slices of few-segment ZMWs
                      # (config E: 16,384 ZMWs per launch 582 -> 569 ms; config D's 30 passes keep
                      # solo16: 314 vs 319 ms, r06c)
                      ("solo16w", ["-DCCSX_RINGA=8", "-DCCSX_BLK=8", "-DCCSX_RING=8", "-DCCSX_HELPERS=0",
                                   "-DCCSX_PRIO_WAVE0=0", "-DCCSX_PRIO_MERGE=0", "-DCCSX_PRIO_TB=1", "-DCCSX_PRIO_MG=1",
                                   "-DCCSX_RING16", "-DCCSX_TB_ROWS=32",
                                   "-DCCSX_WAVES_PER_EU=6"])]]
# machine-scheduler strategy per kernel configuration (the others: max-ilp).
# The one-wave objects under LLVM's iterative ILP scheduler, interleaved A/B
# r08ad: E16k 541.2 -> 536.3 ms, config D 305.1 -> 302.2 ms; the latency
# object (config B) measured +1.7 % with it and keeps max-ilp
KSCHED: dict[str, str] = {n: "iterative-ilp" for n in ("solo", "solo16", "solo16w")}


def _hipcc() -> str:
    for c in (os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc"), shutil.which("hipcc") or ""):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm required to build ccsx_amd)")


def _rocm_inc() -> str:
    return os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "include")


def _stale(target: str, sources: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def _headers() -> list[str]:
    hs = []
    for d in (INC, CSRC, os.path.join(CSRC, "host")):
        for f in os.listdir(d):
            if f.endswith(".h"):
                hs.append(os.path.join(d, f))
    return hs


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout)
        raise RuntimeError("build failed: " + " ".join(cmd))


def _run_all(cmds: list[list[str]], verbose: bool = False) -> None:
    if verbose:
        for c in cmds:
            print(" ".join(c))
    jobs = int(os.environ.get("CCSX_BUILD_JOBS", "6"))
    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for f in [ex.submit(_run, c) for c in cmds]:
            f.result()


def build_product(verbose: bool = False) -> str:
    hipcc = _hipcc()
    os.makedirs(OBJ, exist_ok=True)
    hdrs = _headers()
    khdrs = [os.path.join(CSRC, "ccsx_layout.h")]  # all the kernel includes
    srcs = [
        os.path.join(CSRC, "ccsx_kernel.hip"),  # compiled once per kernel configuration (KCFGS)
        os.path.join(CSRC, "ccsx_gpu.cpp"),
        os.path.join(CSRC, "bspoa_gpu.cpp"),
        os.path.join(CSRC, "host", "prepare.cpp"),
        os.path.join(CSRC, "host", "pairwise.cpp"),
        os.path.join(CSRC, "host", "seqio.cpp"),
        os.path.join(CSRC, "host", "dispatch.cpp"),
        os.path.join(CSRC, "host", "ingest.cpp"),
    ]
    common = ["-O3", "-std=c++17", "-fPIC", "-I" + INC, "-I" + CSRC, "-I" + os.path.join(CSRC, "host")]
    # the kernel's per-ZMW chains are latency-bound: the ILP-maximising machine
    # scheduler measured -0.8 % per launch on config B (tools/abn.sh); per
    # configuration, KSCHED's strategy instead (A/B in DESIGN §9)
    def kflags_of(name: str) -> list[str]:
        return ["-mllvm", "-amdgpu-sched-strategy=" + KSCHED.get(name, "max-ilp")]
    # a flag change here must rebuild the kernel objects
    khdrs = khdrs + [os.path.abspath(__file__)]
    # every object is independent: compile them concurrently (the kernel
    # objects take minutes each; host objects seconds)
    objs, jobs = [], []
    for s in srcs:
        if s.endswith(".hip"):
            for name, defs in KCFGS:
                o = os.path.join(OBJ, f"ccsx_kernel_{name}.hip.o")
                objs.append(o)
                if _stale(o, [s] + khdrs):
                    jobs.append([hipcc, "-x", "hip", "--offload-arch=" + ARCH] + common + kflags_of(name) + defs + ["-c", s, "-o", o])
            continue
        o = os.path.join(OBJ, os.path.basename(s) + ".o")
        objs.append(o)
        if _stale(o, [s] + hdrs):
            jobs.append([hipcc, "-x", "c++"] + common + ["-D__HIP_PLATFORM_AMD__", "-I" + _rocm_inc(), "-c", s, "-o", o])
    # diagnostic variant with per-phase DP stamps (tools/phase_prof.py --diag)
    dobjs = []
    for name, defs in KCFGS:
        dobj = os.path.join(OBJ, f"ccsx_kernel_{name}_diag.hip.o")
        dobjs.append(dobj)
        if _stale(dobj, [srcs[0]] + khdrs):
            # the stamps' counters need registers: 2 waves per SIMD (occupancy
            # is not what this build measures; per-ZMW cycle counts are).  The
            # diagnostic flags come after the configuration's defines, so its
            # waves-per-EU wins over solo16's 5
            jobs.append([hipcc, "-x", "hip", "--offload-arch=" + ARCH] + common + kflags_of(name) + defs
                        + ["-Wno-macro-redefined", "-DCCSX_DP_STAMPS", "-DCCSX_WAVES_PER_EU=2", "-c", srcs[0], "-o", dobj])
    _run_all(jobs, verbose)
    if _stale(LIB, objs):
        cmd = [hipcc, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", LIB] + objs + ["-lz", "-lpthread"]
        if verbose:
            print(" ".join(cmd))
        _run(cmd)
    diag = os.path.join(HERE, "libccsx_amd_diag.so")
    host_objs = objs[len(KCFGS):]
    if _stale(diag, host_objs + dobjs):
        _run([hipcc, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", diag] + dobjs + host_objs + ["-lz", "-lpthread"])
    # the C host program
    main_src = os.path.join(CSRC, "host", "main.cpp")
    if os.path.exists(main_src) and _stale(BIN, [main_src, LIB] + hdrs):
        os.makedirs(os.path.dirname(BIN), exist_ok=True)
        cmd = [hipcc, "-x", "c++"] + common + ["-D__HIP_PLATFORM_AMD__", "-I" + _rocm_inc(), main_src, "-o", BIN,
                                               "-L" + HERE, "-lccsx_amd", "-Wl,-rpath,$ORIGIN/..", "-lz", "-lpthread"]
        if verbose:
            print(" ".join(cmd))
        _run(cmd)
    # tools/synth_fa: the synthetic subread FASTA streamer (CLI runs at config-E scale)
    gsrc = os.path.join(ROOT, "tools", "synth_fa.c")
    gexe = os.path.join(ROOT, "tools", "synth_fa")
    if os.path.exists(gsrc) and _stale(gexe, [gsrc, LIB]):
        _run(["gcc", "-O2", "-std=gnu11", "-I" + INC, "-o", gexe, gsrc, "-L" + HERE, "-lccsx_amd",
              "-Wl,-rpath,$ORIGIN/../ccsx_amd", "-lpthread"])
    return LIB


def build_oracle(verbose: bool = False) -> str:
    # the POA restatement (poa_*.c) and the ccs_prepare one (prep_oracle.c)
    srcs = [os.path.join(ORACLE_DIR, f) for f in sorted(os.listdir(ORACLE_DIR))
            if f.endswith(".c") and (f.startswith("poa_") or f.startswith("prep_"))]
    hdrs = [os.path.join(ORACLE_DIR, f) for f in os.listdir(ORACLE_DIR) if f.endswith(".h")]
    if _stale(ORACLE_LIB, srcs + hdrs):
        cmd = ["gcc", "-O2", "-std=gnu11", "-fPIC", "-shared", "-o", ORACLE_LIB] + srcs + ["-lpthread", "-lz"]
        if verbose:
            print(" ".join(cmd))
        _run(cmd)
    # the CPU-only ccsx of bench.py's cpu_baseline leg: the product's ingest
    # (pinned by the reference's seqio.h fixtures) around the oracle's own
    # ccs_prepare (prep_oracle.c) and POA
    cpu = os.path.join(ORACLE_DIR, "ccsx_cpu")
    csrc = os.path.join(ORACLE_DIR, "ccsx_cpu.c")
    if os.path.exists(LIB) and _stale(cpu, [csrc, LIB] + srcs + hdrs):
        cmd = ["gcc", "-O2", "-std=gnu11", "-o", cpu, csrc] + srcs + ["-L" + HERE, "-lccsx_amd",
                                                                       "-Wl,-rpath,$ORIGIN/../ccsx_amd", "-lpthread", "-lz"]
        if verbose:
            print(" ".join(cmd))
        _run(cmd)
    return ORACLE_LIB


def build_all(verbose: bool = False) -> None:
    build_product(verbose)
    build_oracle(verbose)


if __name__ == "__main__":
    build_all(verbose=True)
