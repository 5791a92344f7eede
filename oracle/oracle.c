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
