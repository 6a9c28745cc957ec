"""CPU model of the chroma-run hot kernel's tables (trik_hsv_chroma.hip:
chroma_summary_kernel, chroma_desc, chroma_block_kernel, chroma_palette_kernel,
select2), restated in numpy and checked against the oracle's exact mask of
every (Y, U, V).

It pins the descriptor semantics independently of the device: for every
chroma the fast path's select `le ? (lt ? M1 : M2) : 0` (lt = Y < b1,
le = Y <= b2, le cleared for the exception code) must equal the oracle's mask
at every Y that is not flagged for the exact path, and must give 0 at the
flagged ones (the exact path adds their masks).  The GPU tests
(tests/test_gpu_chroma.py) hold the device builder and kernel to the oracle on
the same 2^24 triples; this test documents why the construction is exact and
how much reaches the exact path.
"""
import numpy as np
import pytest

KEXC = 0x00FF
BENCH = [(0, 30, 50, 100, 30, 100), (90, 150, 40, 100, 20, 100),
         (200, 260, 40, 100, 20, 100), (330, 20, 30, 100, 30, 100)]


def profiles(oracle_mod, ranges):
    """[65536, 256] uint8: the oracle's mask of (Y, c), c = U | V << 8."""
    c = np.arange(65536, dtype=np.uint32)
    j = np.arange(128, dtype=np.uint32)
    w = (2 * j)[None, :] | ((c & 255) << 8)[:, None] | ((2 * j + 1) << 16)[None, :] | ((c >> 8) << 24)[:, None]
    fr = w.astype("<u4").view(np.uint8).reshape(4096, 8192)
    _, m = oracle_mod.frame(fr, 4096, 4096, 8192, oracle_mod.LAYOUT_YUYV, ranges, want_mask=True)
    return m.reshape(65536, 256).astype(np.int64)


def summaries(P):
    """chroma_summary_kernel: (n, v1, v2, a, ab) per chroma."""
    change = np.ones((P.shape[0], 256), bool)
    change[:, 1:] = P[:, 1:] != P[:, :-1]
    run_id = np.cumsum(change, axis=1) - 1                      # run index of each Y
    nz = P != 0
    any_nz = nz.any(1)
    last_nz_y = 255 - np.argmax(nz[:, ::-1], axis=1)            # valid where any_nz
    last_nz_run = np.where(any_nz, run_id[np.arange(P.shape[0]), last_nz_y], -1)
    n = last_nz_run + 1
    v1 = P[:, 0]
    a = np.argmax(run_id >= 1, axis=1)                          # end of run 1 (0 if a single run)
    a = np.where(run_id[:, -1] == 0, 256, a)
    second = np.where(run_id[:, -1] >= 1, P[np.arange(P.shape[0]), np.minimum(a, 255)], 0)
    v2 = np.where(n == 2, second, 0)
    last_nz_end = np.where(any_nz, last_nz_y + 1, 0)
    ab = np.where(n == 1, a, last_nz_end)
    return np.minimum(n, 3), v1, v2, a, ab


def desc(S, M1, M2):
    """chroma_desc for every chroma under block masks M1, M2 (arrays)."""
    n, v1, v2, a, ab = S
    out = np.full(n.shape, -1, np.int64)
    def put(cond, val):
        sel = (out < 0) & cond
        out[sel] = np.broadcast_to(val, out.shape)[sel]
    put((n == 0) & (M1 == 0), 255 | 254 << 8)
    put((n == 0) & (M2 == 0), 0 | 255 << 8)
    put(n == 0, KEXC)
    put((n == 1) & (v1 == M2), 0 | (a - 1) << 8)
    put((n == 1) & (v1 == M1) & (a <= 255), a | (a - 1) << 8)
    put((n == 2) & (v1 == M1) & (v2 == M2), a | (ab - 1) << 8)
    put((v1 != M1) | (ab > 255), KEXC)
    b2, b1 = a - 1, ab
    put((b2 == 0) & (b1 == 255), KEXC)
    put(np.ones_like(out, bool), b1 | b2 << 8)
    return out


def cost(d):
    b1, b2 = d & 255, d >> 8
    L = b1 - b2 - 1
    return np.where(d == KEXC, 65536, np.where(b1 <= b2 + 1, 0, L * (512 - L)))


def build(P):
    """chroma_block_kernel: per 16-chroma block the cheapest (M1, M2)."""
    S = summaries(P)
    n, v1, v2 = S[0], S[1], S[2]
    present = np.ones(65536, np.int64)
    present |= np.where(n > 0, 1 << v1, 0)
    present |= np.where(n == 2, 1 << v2, 0)
    present = np.bitwise_or.reduce(present.reshape(4096, 16), axis=1)
    best = np.full(4096, np.iinfo(np.int64).max)
    best_k = np.zeros(4096, np.int64)
    for k in range(256):
        M1, M2 = k & 15, k >> 4
        ok = ((present >> M1) & 1).astype(bool) & ((present >> M2) & 1).astype(bool)
        c = cost(desc(S, np.full(65536, M1), np.full(65536, M2))).reshape(4096, 16).sum(1)
        better = ok & (c < best)
        best[better] = c[better]
        best_k[better] = k
    # chroma_palette_kernel: the 32 most used pairs (ties: smaller k); a block
    # whose pair missed the palette takes the cheapest palette pair
    hist = np.bincount(best_k, minlength=256)
    order = sorted(range(256), key=lambda k: (-hist[k], k))
    palette = [k for k in order[:32] if hist[k] > 0]
    miss = ~np.isin(best_k, palette)
    if miss.any():
        costs = np.stack([cost(desc(S, np.full(65536, k & 15), np.full(65536, k >> 4))).reshape(4096, 16).sum(1)
                          for k in palette], axis=1)
        best_k = np.where(miss, np.asarray(palette)[np.argmin(costs, axis=1)], best_k)
    kk = np.repeat(best_k, 16)
    return desc(S, kk & 15, kk >> 4), best_k


@pytest.mark.parametrize("n_ranges,max_words", [(4, 0.065), (1, 0.005)])
def test_descriptors_exact_on_all_triples(oracle_mod, n_ranges, max_words):
    P = profiles(oracle_mod, BENCH[:n_ranges])
    runs, blocks = build(P)
    Y = np.arange(256)[None, :]
    b1, b2 = (runs & 255)[:, None], (runs >> 8)[:, None]
    kk = np.repeat(blocks, 16)
    M1, M2 = (kk & 15)[:, None], (kk >> 4)[:, None]
    x = (runs == KEXC)[:, None]
    lt, le = Y < b1, (Y <= b2) & ~x
    fast = np.where(le, np.where(lt, M1, M2), 0)
    flagged = x | (lt & (Y > b2))
    assert (fast[flagged] == 0).all()                     # the exact path adds these
    assert np.array_equal(np.where(flagged, P, fast), P)  # everything else is exact
    words = (1 - (1 - flagged.mean(1)) ** 2).mean()       # a word: two uniform Y of one chroma
    assert words < max_words
