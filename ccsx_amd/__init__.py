"""ccsx_amd -- MI355X-native engine for ccsx's per-ZMW circular-consensus hot path.

See DESIGN.md.  The product is the in-tree ``libccsx_amd.so`` (HIP kernels for
gfx950 + C-ABI, include/*.h); this package holds its build script and ctypes
bindings.
"""
from .native import (MODE_PRIMITIVE, MODE_SHRED, Engine, GpuError, Prepared, lib, pairwise, partition,  # noqa: F401
                     prepare, prepare_segments, read_calls, read_zmws, revcomp, synth_zmw, zmw_cost)

__version__ = "0.1.0"
