"""Development analysis (CPU): structure of the per-chroma mask profiles under a
range set, and how much of a uniform-byte batch each descriptor scheme sends
to the exact path.  Uses the oracle's exact masks of all 2^24 (Y,U,V) and the
numpy model of the chroma-run builder in tests/test_chroma_model.py.

usage: python scripts/chroma_profile_stats.py [n_ranges]
"""
import collections
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import oracle  # noqa: E402
import test_chroma_model as tcm  # noqa: E402


def runs_of(row):
    """[(value, start, end_exclusive)] of a 256-entry profile."""
    out, s = [], 0
    for y in range(1, 257):
        if y == 256 or row[y] != row[s]:
            out.append((int(row[s]), s, y))
            s = y
    return out


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    oracle.build()
    P = tcm.profiles(oracle, tcm.BENCH[:n])
    runs, blocks, _cut = tcm.build(P)
    Y = np.arange(256)[None, :]
    b1, b2 = (runs & 255)[:, None], (runs >> 8)[:, None]
    x = (runs == tcm.KEXC)
    flagged = x[:, None] | ((Y < b1) & (Y > b2))
    pf = flagged.mean(1)
    words = 1 - (1 - pf) ** 2
    kind = np.where(x, "exc", np.where((runs & 255) > (runs >> 8) + 1, "window", "runs"))
    print(f"ranges={n} flagged pixels {flagged.mean():.4f} words {words.mean():.4f}")
    for k in ("runs", "window", "exc"):
        sel = kind == k
        print(f"  {k:7s} chromas {sel.mean():.4f}  word share {words[sel].sum() / 65536:.4f}")
    # run-structure histogram (leading value zero?, number of runs incl. the trailing zero)
    shapes = collections.Counter()
    wshapes = collections.Counter()
    for c in range(65536):
        r = runs_of(P[c])
        sig = tuple(v for v, _, _ in r)
        shapes[len(r)] += 1
        if kind[c] != "runs":
            wshapes[sig] += words[c]
    print("runs per profile:", sorted(shapes.items()))
    print("top flagged-word profiles (value sequence: word share):")
    for sig, wsh in sorted(wshapes.items(), key=lambda t: -t[1])[:25]:
        print(f"   {sig}: {wsh / 65536:.5f}")


if __name__ == "__main__":
    main()
