"""CPU model (development only): how many of the chroma kernel's flagged words a
third block mask would remove.  A block of 16 chromas whose every profile
(the oracle's mask over Y) is M1* M2* M3* -- three runs in this order, any of
them empty -- for one (M1, M2, M3) would need no exact path at all.
Builds the bench ranges' tables with tests/test_chroma_model.py (the numpy
restatement of the device builder) and prints the flagged-word share before
and after.  usage: python scripts/chroma_m3_model.py   (~1 min, CPU)
"""
import itertools
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import oracle as om  # noqa: E402
import test_chroma_model as tm  # noqa: E402


def compress(p):
    out = [int(p[0])]
    for v in p[1:]:
        if v != out[-1]:
            out.append(int(v))
    return tuple(out)


def fits(seq, tri):
    j = 0
    for v in seq:
        while j < 3 and tri[j] != v:
            j += 1
        if j == 3:
            return False
        j += 1
    return True


def main():
    P = tm.profiles(om, tm.BENCH)
    runs, _, _ = tm.build(P)
    Y = np.arange(256)[None, :]
    b1, b2 = (runs & 255)[:, None], (runs >> 8)[:, None]
    flag = (runs == tm.KEXC)[:, None] | ((Y < b1) & (Y > b2))
    words = 1 - (1 - flag.mean(1)) ** 2  # per chroma: share of its words flagged
    seqs = [compress(P[c]) for c in range(65536)]
    saved, fixed, costly = 0.0, 0, 0
    for b in range(4096):
        cs = [((b >> 4) << 8) | ((b & 15) << 4) | i for i in range(16)]
        cost = sum(words[c] for c in cs)
        if cost == 0:
            continue
        costly += 1
        bs = set(seqs[c] for c in cs)
        if any(len(s) > 3 for s in bs):
            continue
        vals = sorted(set(v for s in bs for v in s))
        if any(all(fits(s, tri) for s in bs) for tri in itertools.product(vals, repeat=3)):
            fixed += 1
            saved += cost
    print(f"flagged words {words.mean():.4f}; blocks with flagged words {costly}; "
          f"exact with a third mask {fixed}; flagged words after {words.mean() - saved / 65536:.4f}")


if __name__ == "__main__":
    main()
