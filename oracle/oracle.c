/*
 * oracle.c -- CPU restatement (test infrastructure ONLY) of the reference's
 * two native helpers on the hot path.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this library, and only as the
 * checker / CPU baseline; the product path never links it.
 *
 *  oracle_medfilt   <- comancpipeline/Tools/median_filter/medianFilter.cpp:4-30
 *                      (+ Mediator.h:91-99 getMedian, medfilt.pyx:26-33)
 *     Semantics restated (not the two-heap data structure): in place,
 *       out[i] = median( x'[i-h], ..., x'[i-h+w-1] ),  h = w/2,
 *       x'[j] = x[0]   for j < h   (the w/2 head inserts of x[0] and the
 *                                  head outputs written over x[0..h) before
 *                                  they are read back),
 *       x'[j] = x[j]   for h <= j < n,
 *       x'[j] = x[n-1] for j >= n  (tail inserts of x[n-1]).
 *     Even w: (s[w/2-1] + s[w/2]) / 2 in double, the order Mediator uses.
 *     Implemented with a sorted window and binary-search insert/delete:
 *     O(n w) moves, exact.
 *
 *  oracle_medfilt_twoheap <- the same filter() driver (medianFilter.cpp:4-30) over
 *     the two-heap running median of Mediator.h:9-197, restated: a window ring
 *     of values, a max-heap (positions -1, -2, ...) below a median slot (0) above
 *     a min-heap (1, 2, ...), every comparison a plain '<' / '>' on doubles.
 *     Equal to oracle_medfilt on NaN-free input; with NaN every comparison with it
 *     is false, so the result follows the heap's insertion history -- this is the
 *     reference's NaN semantics, pinned against oracle/_ref (the reference's own
 *     medianFilter.cpp) in tests/test_oracle_golden.py.  Requires n >= ceil(w/2)
 *     (below that the reference reads and writes outside the array).
 *
 *  oracle_bin_values <- comancpipeline/Tools/binFuncs.pyx:7-32 (binValues):
 *     image[p] += w[i] (or += 1 when w == NULL) for 0 <= p < npix and
 *     mask[i] != 0 (mask == NULL: all).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static int64_t lower_bound_d(const double *s, int64_t n, double v)
{
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if (s[mid] < v) lo = mid + 1; else hi = mid;
    }
    return lo;
}

static double xprime(const double *x, int64_t n, int64_t h, int64_t j)
{
    if (j < h) return x[0];
    if (j >= n) return x[n - 1];
    return x[j];
}

int oracle_medfilt(double *x, int64_t n, int32_t w)
{
    if (w < 1 || n < 1 || n < w) return -1;
    /* the sorted window needs a total order: NaN is outside this restatement (the
       reference's two-heap result for it depends on its history) -- refuse it */
    for (int64_t i = 0; i < n; ++i)
        if (x[i] != x[i]) return -3;
    const int64_t h = w / 2;
    double *orig = (double *)malloc(sizeof(double) * (size_t)n);
    double *s = (double *)malloc(sizeof(double) * (size_t)w);
    if (!orig || !s) { free(orig); free(s); return -2; }
    memcpy(orig, x, sizeof(double) * (size_t)n);
    /* window for i = 0: x'[-h .. -h+w-1] */
    for (int64_t k = 0; k < w; ++k) s[k] = xprime(orig, n, h, k - h);
    /* insertion sort is fine for the first window */
    for (int64_t a = 1; a < w; ++a) {
        double v = s[a]; int64_t b = a - 1;
        while (b >= 0 && s[b] > v) { s[b + 1] = s[b]; --b; }
        s[b + 1] = v;
    }
    for (int64_t i = 0; i < n; ++i) {
        double med = (w % 2 == 0) ? (s[w / 2] + s[w / 2 - 1]) / 2.0 : s[w / 2];
        x[i] = med;
        if (i + 1 == n) break;
        double vout = xprime(orig, n, h, i - h);
        double vin = xprime(orig, n, h, i - h + w);
        int64_t po = lower_bound_d(s, w, vout);      /* s[po] == vout */
        memmove(s + po, s + po + 1, sizeof(double) * (size_t)(w - 1 - po));
        int64_t pi = lower_bound_d(s, w - 1, vin);
        memmove(s + pi + 1, s + pi, sizeof(double) * (size_t)(w - 1 - pi));
        s[pi] = vin;
    }
    free(orig); free(s);
    return 0;
}

/* ---- two-heap running median (Mediator.h restated) */
typedef struct {
    int32_t N;        /* window */
    double *val;      /* val[slot]: value held by ring slot                */
    int32_t *at;      /* at[slot]: heap position of the slot               */
    int32_t *hp;      /* hp[pos + N/2]: slot at heap position pos          */
    int32_t nlo, nhi; /* filled positions below (max-heap) / above (min-heap) */
    int32_t cur;      /* next ring slot to overwrite                       */
} twoheap;

#define HP(m, i) ((m)->hp[(i) + (m)->N / 2])

static int th_less(const twoheap *m, int32_t i, int32_t j) { return m->val[HP(m, i)] < m->val[HP(m, j)]; }

static void th_swap(twoheap *m, int32_t i, int32_t j)
{
    const int32_t a = HP(m, i), b = HP(m, j);
    HP(m, i) = b; HP(m, j) = a;
    m->at[b] = i; m->at[a] = j;
}

/* swaps positions i and j when the value at i is below the one at j */
static int th_order(twoheap *m, int32_t i, int32_t j)
{
    if (!th_less(m, i, j)) return 0;
    th_swap(m, i, j);
    return 1;
}

static int th_hi_up(twoheap *m, int32_t i)        /* min-heap side, towards the median */
{
    while (i > 0 && th_order(m, i, i / 2)) i /= 2;
    return i == 0;
}

static int th_lo_up(twoheap *m, int32_t i)        /* max-heap side, towards the median */
{
    while (i < 0 && th_order(m, i / 2, i)) i /= 2;
    return i == 0;
}

static void th_hi_down(twoheap *m, int32_t i)
{
    for (i *= 2; i <= m->nhi; i *= 2) {
        if (i < m->nhi && th_less(m, i + 1, i)) ++i;
        if (!th_order(m, i, i / 2)) break;
    }
}

static void th_lo_down(twoheap *m, int32_t i)
{
    for (i *= 2; i >= -m->nlo; i *= 2) {
        if (i > -m->nlo && th_less(m, i, i - 1)) --i;
        if (!th_order(m, i / 2, i)) break;
    }
}

static void th_push(twoheap *m, double v)
{
    const int32_t p = m->at[m->cur];
    const double old = m->val[m->cur];
    m->val[m->cur] = v;
    m->cur = (m->cur + 1) % m->N;
    if (p > 0) {
        if (m->nhi < (m->N - 1) / 2) m->nhi++;
        else if (v > old) { th_hi_down(m, p); return; }
        if (th_hi_up(m, p) && th_order(m, 0, -1)) th_lo_down(m, -1);
    } else if (p < 0) {
        if (m->nlo < m->N / 2) m->nlo++;
        else if (v < old) { th_lo_down(m, p); return; }
        if (th_lo_up(m, p) && m->nhi && th_order(m, 1, 0)) th_hi_down(m, 1);
    } else {
        if (m->nlo && th_lo_up(m, -1)) th_lo_down(m, -1);
        if (m->nhi && th_hi_up(m, 1)) th_hi_down(m, 1);
    }
}

static double th_median(const twoheap *m)
{
    double v = m->val[HP(m, 0)];
    if (m->nhi < m->nlo) v = (v + m->val[HP(m, -1)]) / 2;
    return v;
}

int oracle_medfilt_twoheap(double *x, int64_t n, int32_t w)
{
    if (w < 1 || n < (int64_t)(w / 2 + w % 2) || n < 1) return -1;
    twoheap m;
    m.N = w;
    m.val = (double *)calloc((size_t)w, sizeof(double));
    m.at = (int32_t *)malloc(sizeof(int32_t) * (size_t)w);
    m.hp = (int32_t *)malloc(sizeof(int32_t) * (size_t)w);
    if (!m.val || !m.at || !m.hp) { free(m.val); free(m.at); free(m.hp); return -2; }
    m.nlo = m.nhi = m.cur = 0;
    /* slot s starts at position 0, -1, +1, -2, +2, ... */
    for (int32_t s = w - 1; s >= 0; --s) {
        const int32_t pos = ((s + 1) / 2) * ((s & 1) ? -1 : 1);
        m.at[s] = pos;
        HP(&m, pos) = s;
    }
    /* filter()'s four phases, in place exactly as medianFilter.cpp runs them */
    const int64_t h = w / 2, off = w / 2 + w % 2;
    for (int64_t i = 0; i < h; ++i) { th_push(&m, x[0]); x[i] = th_median(&m); }
    for (int64_t i = 0; i < off; ++i) th_push(&m, x[i]);
    for (int64_t i = 0; i < n - off; ++i) { x[i] = th_median(&m); th_push(&m, x[i + off]); }
    for (int64_t i = n - off; i < n; ++i) { x[i] = th_median(&m); th_push(&m, x[n - 1]); }
    free(m.val); free(m.at); free(m.hp);
    return 0;
}

int oracle_bin_values(double *image, int64_t npix, const int64_t *pixels,
                      const double *weights, const int64_t *mask, int64_t n)
{
    for (int64_t i = 0; i < n; ++i) {
        if (mask && mask[i] == 0) continue;
        int64_t p = pixels[i];
        if (p >= 0 && p < npix) image[p] += weights ? weights[i] : 1.0;
    }
    return 0;
}
