#!/usr/bin/env python3
"""Wait until the given HIP devices have at least FRAC of their memory free
(the driver clears what a process that just exited held: a process that
follows one that used ~250 GB waits seconds in its first large allocation,
DESIGN.md §7).  Run as a short-lived child process by bench.py before its
one-process line, so that line times the product, not the release.

    python tools/mem_wait.py --devices 0,1 --frac 0.95 --timeout 120

Prints one JSON line: {"waited_s": s, "free_frac": {dev: frac}, "ok": bool}.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import time


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--devices", default="0")
    ap.add_argument("--frac", type=float, default=0.95)
    ap.add_argument("--timeout", type=float, default=120.0)
    a = ap.parse_args()
    devs = [int(x) for x in a.devices.split(",") if x != ""]
    try:
        hip = C.CDLL("libamdhip64.so")
    except OSError:
        hip = C.CDLL("/opt/rocm/lib/libamdhip64.so")
    hip.hipSetDevice.argtypes = [C.c_int]
    hip.hipMemGetInfo.argtypes = [C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]

    def fracs():
        out = {}
        for d in devs:
            f, t = C.c_size_t(0), C.c_size_t(0)
            if hip.hipSetDevice(d) != 0 or hip.hipMemGetInfo(C.byref(f), C.byref(t)) != 0 or not t.value:
                out[d] = None
            else:
                out[d] = f.value / t.value
        return out

    t0 = time.perf_counter()
    fr = fracs()
    while any(v is not None and v < a.frac for v in fr.values()) and time.perf_counter() - t0 < a.timeout:
        time.sleep(0.1)
        fr = fracs()
    ok = all(v is not None and v >= a.frac for v in fr.values())
    print(json.dumps({"waited_s": round(time.perf_counter() - t0, 3),
                      "free_frac": {str(k): (round(v, 4) if v is not None else None) for k, v in fr.items()},
                      "ok": ok}), flush=True)


if __name__ == "__main__":
    main()
