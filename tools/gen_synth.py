"""Write a synthetic subread FASTA: `synth/<hole>/<qs>_<qe>` names,
single-line uppercase records.  Usage: gen_synth.py OUT.fa NZMW L PASSES [HOLE0]
(L = 0: per-hole insert length and passes of bench.py's config E)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ccsx_amd as cx  # noqa: E402


def write(path, nzmw, L, passes, hole0=0, seed=20201104, movie="synth"):
    with open(path, "wb") as f:
        for h in range(hole0, hole0 + nzmw):
            if L:
                subs, _ = cx.synth_zmw(seed, h, L, passes)
            else:
                from bench import CONFIGS, zmw_shape
                subs, _ = cx.synth_zmw(seed, h, *zmw_shape(CONFIGS["E"], h))
            qs = 0
            for s in subs:
                f.write(b">%s/%d/%d_%d\n%s\n" % (movie.encode(), h, qs, qs + len(s), s))
                qs += len(s)


if __name__ == "__main__":
    a = sys.argv
    write(a[1], int(a[2]), int(a[3]), int(a[4]), int(a[5]) if len(a) > 5 else 0)
