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


def first_nonzero(P):
    """first_nz: the first Y with a nonzero mask (256: all zero)."""
    nz = P != 0
    return np.where(nz.any(1), np.argmax(nz, axis=1), 256)


def build(P):
    """chroma_summary_kernel + chroma_block_kernel + chroma_palette_kernel:
    per 16-chroma block the cheapest (cost, M1 | M2 << 4, cut A), ties by the
    smaller pair, then the smaller cut; A is 0 or the first nonzero Y of one of
    the block's chromas.  A chroma whose profile starts at A is described from
    A on (its leading zero run dropped), one that starts above A as before, one
    that starts below A is an exception."""
    N = P.shape[0]
    f = first_nonzero(P)
    Y = np.arange(256)[None, :]
    Pd = np.where(Y < f[:, None], P[np.arange(N), np.minimum(f, 255)][:, None], P)
    Sf, Sd = summaries(P), summaries(Pd)
    fb = f.reshape(4096, 16)

    def descs(k, A):  # A: per-chroma cut
        df = desc(Sf, np.full(N, k & 15), np.full(N, k >> 4))
        dd = desc(Sd, np.full(N, k & 15), np.full(N, k >> 4))
        return np.where(f > A, df, np.where(f == A, dd, KEXC))

    def choose(pairs, block_ok):
        best = np.full(4096, np.iinfo(np.int64).max)
        for k in pairs:
            ok = block_ok(k)
            if not ok.any():
                continue
            for j in range(-1, 16):
                A = np.zeros(4096, np.int64) if j < 0 else fb[:, j]
                if j >= 0:
                    valid = (A > 0) & (A < 256)
                c = cost(descs(k, np.repeat(A, 16))).reshape(4096, 16).sum(1)
                key = (c << 17) | (k << 9) | A
                take = ok & (key < best) if j < 0 else ok & valid & (key < best)
                best[take] = key[take]
        return best

    present = np.ones(N, np.int64)
    for S in (Sf, Sd):
        present |= np.where(S[0] > 0, 1 << S[1], 0)
        present |= np.where(S[0] == 2, 1 << S[2], 0)
    present = np.bitwise_or.reduce(present.reshape(4096, 16), axis=1)
    best = choose(range(256), lambda k: ((present >> (k & 15)) & (present >> (k >> 4)) & 1).astype(bool))
    best_k = (best >> 9) & 255
    # chroma_palette_kernel: the 32 most used pairs (ties: smaller k); then the
    # choice among the palette's pairs (the same where the pair made it)
    hist = np.bincount(best_k, minlength=256)
    order = sorted(range(256), key=lambda k: (-hist[k], k))
    palette = [k for k in order[:32] if hist[k] > 0]
    best = choose(palette, lambda k: np.ones(4096, bool))
    best_k, best_A = (best >> 9) & 255, best & 511
    return descs_for(best_k, best_A, descs), best_k, best_A


def descs_for(best_k, best_A, descs):
    runs = np.zeros(65536, np.int64)
    kk, AA = np.repeat(best_k, 16), np.repeat(best_A, 16)
    for k in np.unique(best_k):
        sel = kk == k
        runs[sel] = descs(k, AA)[sel]
    return runs


@pytest.mark.parametrize("n_ranges,max_words", [(4, 0.03), (1, 0.005)])
def test_descriptors_exact_on_all_triples(oracle_mod, n_ranges, max_words):
    P = profiles(oracle_mod, BENCH[:n_ranges])
    runs, blocks, cut = build(P)
    Y = np.arange(256)[None, :]
    b1, b2 = (runs & 255)[:, None], (runs >> 8)[:, None]
    kk, AA = np.repeat(blocks, 16), np.repeat(cut, 16)
    M1, M2, A = (kk & 15)[:, None], (kk >> 4)[:, None], AA[:, None]
    x = (runs == KEXC)[:, None]
    lt, le, ge = Y < b1, (Y <= b2) & ~x, Y >= A
    fast = np.where(le & ge, np.where(lt, M1, M2), 0)
    flagged = x | (lt & (Y > b2))
    assert not (flagged & ~ge & ~x).any()                 # windows lie above the cut
    assert (fast[flagged] == 0).all()                     # the exact path adds these
    assert np.array_equal(np.where(flagged, P, fast), P)  # everything else is exact
    words = (1 - (1 - flagged.mean(1)) ** 2).mean()       # a word: two uniform Y of one chroma
    assert words < max_words
