// Offline model of the chroma-run tables (development analysis, CPU only):
// the builder's per-chroma run summaries, per-block (mask pair, cut) choice
// and palette (trik_hsv_chroma.hip: chroma_summary_kernel, chroma_desc,
// chroma_cost, chroma_block_kernel) restated over the exhaustive mask table
// of scripts/chroma_masks.py, to see where the exact-path share comes from
// and what other encodings would give -- without a GPU.
//
// build: gcc -O2 -o /tmp/chroma_model scripts/chroma_model.c
// usage: /tmp/chroma_model MASKS.bin
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define NC 65536
static uint8_t* M;  // [NC][256]

typedef struct {
  int n;        // runs up to the last nonzero one (0: all zero)
  int v[4];     // first run values (v[0] = mask at Y = 0)
  int e[4];     // their exclusive ends
  int last_end; // end of the last nonzero run
} Runs;
static Runs R[NC];

static void runs_of(int c, Runs* r) {
  const uint8_t* p = M + (size_t)c * 256;
  int vals[256], ends[256], k = 0;
  int cur = p[0];
  for (int y = 1; y <= 256; ++y) {
    if (y == 256 || p[y] != cur) {
      vals[k] = cur;
      ends[k] = y;
      ++k;
      if (y < 256) cur = p[y];
    }
  }
  int last = -1;
  for (int i = 0; i < k; ++i)
    if (vals[i]) last = i;
  memset(r, 0, sizeof *r);
  r->n = last + 1;
  for (int i = 0; i < 4 && i < k; ++i) {
    r->v[i] = vals[i];
    r->e[i] = ends[i];
  }
  r->last_end = last >= 0 ? ends[last] : 0;
}

// the summary word (pack in chroma_summary_kernel)
static uint32_t pack(int nn, int v1, int v2, int a, int last_end) {
  if (nn == 0) return 0u;
  const int ab = nn == 1 ? a : last_end;
  return (uint32_t)(nn > 2 ? 3 : nn) | ((uint32_t)v1 << 4) | ((uint32_t)(nn == 2 ? v2 : 0) << 8) | ((uint32_t)a << 12) |
         ((uint32_t)ab << 21);
}
static uint32_t SF[NC], SD[NC];
static int FZ[NC];

#define EXC 0x00FFu
static uint32_t desc(uint32_t s, uint32_t M1, uint32_t M2) {
  const uint32_t n = s & 3u;
  if (n == 0) {
    if (M1 == 0) return 255u | (254u << 8);
    if (M2 == 0) return 0u | (255u << 8);
    return EXC;
  }
  const uint32_t v1 = (s >> 4) & 15u, v2 = (s >> 8) & 15u;
  const uint32_t a = (s >> 12) & 511u, ab = (s >> 21) & 511u;
  if (n == 1) {
    if (v1 == M2) return 0u | ((a - 1u) << 8);
    if (v1 == M1 && a <= 255u) return a | ((a - 1u) << 8);
  }
  if (n == 2 && v1 == M1 && v2 == M2) return a | ((ab - 1u) << 8);
  if (v1 != M1 || ab > 255u) return EXC;
  const uint32_t b2 = a - 1u, b1 = ab;
  if (b2 == 0u && b1 == 255u) return EXC;
  return b1 | (b2 << 8);
}
static uint32_t cost_words(uint32_t d) {  // per 65536 words
  if (d == EXC) return 65536u;
  const uint32_t b1 = d & 255u, b2 = d >> 8;
  if (b1 <= b2 + 1u) return 0u;
  const uint32_t L = b1 - b2 - 1u;
  return L * (512u - L);
}
static uint32_t desc_cut(int c, uint32_t k, uint32_t A) {
  if ((uint32_t)FZ[c] < A) return EXC;
  return desc((uint32_t)FZ[c] == A ? SD[c] : SF[c], k & 15u, k >> 4);
}

// block b's 16 chromas under a block layout
static int LAYOUT = 0;
static int BS = 16;  // chromas per block (16: the kernel's; 8: a finer variant)
static FILE* dump = NULL;  // 0: 16 along U (the kernel's), 1: 16 along V, 2: 4 x 4
static int chroma_in_block(int b, int i) {
  if (BS == 8) return ((b >> 5) << 8) | ((b & 31) << 3) | i;     // V = b >> 5, U = 8 (b & 31) + i
  if (LAYOUT == 0) return ((b >> 4) << 8) | ((b & 15) << 4) | i;  // V = b >> 4, U = 16 (b & 15) + i
  if (LAYOUT == 1) return (((b & 15) * 16 + i) << 8) | (b >> 4);  // U = b >> 4, V = 16 (b & 15) + i
  // 4 x 4: b = (V >> 2) << 6 | (U >> 2)
  const int U = ((b & 63) << 2) | (i & 3), V = ((b >> 6) << 2) | (i >> 2);
  return U | (V << 8);
}

typedef struct {
  uint64_t key;  // cost << 17 | k << 9 | A
} Best;

static uint64_t block_best(int b, const int* allowed /* [256] or NULL */) {
  int cs[16];
  for (int i = 0; i < BS; ++i) cs[i] = chroma_in_block(b, i);
  uint32_t cuts[17];
  int nc = 0;
  cuts[nc++] = 0;
  for (int i = 0; i < BS; ++i)
    if (FZ[cs[i]] != 0 && FZ[cs[i]] <= 255) cuts[nc++] = (uint32_t)FZ[cs[i]];
  uint32_t present = 1;
  if (!allowed)
    for (int i = 0; i < BS; ++i) {
      const uint32_t a = SF[cs[i]], d = SD[cs[i]];
      if (a & 3u) present |= 1u << ((a >> 4) & 15u);
      if ((a & 3u) == 2u) present |= 1u << ((a >> 8) & 15u);
      if (d & 3u) present |= 1u << ((d >> 4) & 15u);
      if ((d & 3u) == 2u) present |= 1u << ((d >> 8) & 15u);
    }
  uint64_t best = ~0ull;
  for (uint32_t k = 0; k < 256; ++k) {
    const int take = allowed ? allowed[k] : (((present >> (k & 15u)) & 1u) && ((present >> (k >> 4)) & 1u));
    if (!take) continue;
    for (int j = 0; j < nc; ++j) {
      uint64_t cost = 0;
      for (int i = 0; i < BS; ++i) cost += cost_words(desc_cut(cs[i], k, cuts[j]));
      const uint64_t key = (cost << 17) | ((uint64_t)k << 9) | cuts[j];
      if (key < best) best = key;
    }
  }
  return best;
}

static double model(int layout, int palette, const char* label, int verbose) {
  LAYOUT = layout;
  static uint64_t best[8192];
  static int hist[256];
  const int nb = NC / BS;
  memset(hist, 0, sizeof hist);
  for (int b = 0; b < nb; ++b) {
    best[b] = block_best(b, NULL);
    hist[(best[b] >> 9) & 255]++;
  }
  int allowed[256];
  for (int k = 0; k < 256; ++k) {
    int rank = 0;
    for (int j = 0; j < 256; ++j) rank += (hist[j] > hist[k]) || (hist[j] == hist[k] && j < k);
    allowed[k] = hist[k] > 0 && rank < palette;
  }
  uint64_t total = 0, exc_c = 0, win_c = 0, exc_cost = 0, win_cost = 0, pix = 0;
  uint64_t hL[257] = {0};
  for (int b = 0; b < nb; ++b) {
    uint64_t key = best[b];
    if (!allowed[(key >> 9) & 255]) key = block_best(b, allowed);
    const uint32_t k = (uint32_t)(key >> 9) & 255u, A = (uint32_t)key & 511u;
    for (int i = 0; i < BS; ++i) {
      const int c = chroma_in_block(b, i);
      const uint32_t d = desc_cut(c, k, A);
      const uint32_t cw = cost_words(d);
      total += cw;
      if (dump && (d == EXC || cw)) {
        fprintf(dump, "%s %d %u %u %u %u", d == EXC ? "EXC" : "WIN", c, k & 15u, k >> 4, A, cw);
        const uint8_t* p = M + (size_t)c * 256;
        fprintf(dump, " |");
        for (int y = 0; y < 256; ++y)
          if (y == 0 || p[y] != p[y - 1]) fprintf(dump, " %d@%d", p[y], y);
        fprintf(dump, "\n");
      }
      if (d == EXC) {
        exc_c++;
        exc_cost += cw;
        pix += 256;
      } else if (cw) {
        win_c++;
        win_cost += cw;
        const uint32_t L = (d & 255u) - (d >> 8) - 1u;
        pix += L;
        hL[L]++;
      }
    }
  }
  const double share = (double)total / 65536.0 / 65536.0;
  printf("%-28s word share %.4f  pixel share %.4f | exceptions %6llu chromas (%.4f) windows %6llu chromas (%.4f)\n",
         label, share, (double)pix / 65536.0 / 256.0, (unsigned long long)exc_c, (double)exc_cost / 4294967296.0,
         (unsigned long long)win_c, (double)win_cost / 4294967296.0);
  if (verbose) {
    printf("  window lengths (L: chromas):");
    int shown = 0;
    for (int L = 1; L < 257 && shown < 40; ++L)
      if (hL[L]) {
        printf(" %d:%llu", L, (unsigned long long)hL[L]);
        ++shown;
      }
    printf("\n");
  }
  return share;
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  M = malloc((size_t)NC * 256);
  FILE* f = fopen(argv[1], "rb");
  if (!f || fread(M, 1, (size_t)NC * 256, f) != (size_t)NC * 256) return 2;
  fclose(f);
  for (int c = 0; c < NC; ++c) {
    Runs* r = &R[c];
    runs_of(c, r);
    const int n = r->n;
    SF[c] = pack(n, r->v[0], r->v[1], r->e[0], r->last_end);
    const int lead0 = r->v[0] == 0 && n > 0;
    SD[c] = lead0 ? pack(n - 1, r->v[1], r->v[2], r->e[1], r->last_end) : SF[c];
    FZ[c] = n == 0 ? 256 : (lead0 ? r->e[0] : 0);
  }
  // profile shapes: runs up to the last nonzero one
  int hn[8] = {0};
  for (int c = 0; c < NC; ++c) hn[R[c].n < 7 ? R[c].n : 7]++;
  printf("chromas by runs (up to the last nonzero): 0:%d 1:%d 2:%d 3:%d 4:%d 5:%d 6:%d 7+:%d\n", hn[0], hn[1], hn[2],
         hn[3], hn[4], hn[5], hn[6], hn[7]);
  if (argc > 2) dump = fopen(argv[2], "w");
  model(0, 32, "kernel (16 along U, pal 32)", 1);
  if (dump) fclose(dump);
  dump = NULL;
  model(0, 256, "16 along U, pal 256", 0);
  model(1, 32, "16 along V, pal 32", 0);
  model(2, 32, "4 x 4, pal 32", 0);
  BS = 8;
  model(0, 32, "8 along U, pal 32", 0);
  model(0, 64, "8 along U, pal 64", 0);
  BS = 16;
  return 0;
}
