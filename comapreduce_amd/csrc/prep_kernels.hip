// prep_kernels.hip -- the destriper's data prep on the device
// (reference comancpipeline/MapMaking/COMAPData.py:72-117, 205-236, 247-427, 471-577).
//
// read_comap_data turns Level-2 files into flat (tod, weights, pointing, ...)
// vectors.  The reference does it per file and per feed in NumPy; here every
// O(samples) step runs on the device, per file for all its feeds and bands:
//
//   comap_prep_auto_rms     weights = 1/auto_rms(tod)^2 per (feed, band): NumPy's
//                           nanstd reproduced bit for bit (its pairwise summation tree)
//   comap_prep_percentiles  the az / el 10th and 90th percentiles per feed: exact
//                           order statistics (radix select) + NumPy's linear rule
//   comap_prep_gather       per output sample: the file row's tod / cal, the weight
//                           cuts (spikes, Sun < 10 deg, az / el percentile band, 10%
//                           scan edges), az / el, the Sun-centric distance and
//                           colatitude, feed id, obsid, and the pixel id (CAR / SIN /
//                           TAN world -> pixel, floor(p + 0.5), off-map -> -1)
//   comap_prep_highpass     tod -= the reflect-padded 400-sample running median of
//                           each (feed, scan, band)'s non-zero samples (median_kernels.hip)
//   comap_prep_cut          NaN -> 0, the offsets with all-zero weights dropped per
//                           band (keep mask), the union of kept offsets compacted
//
// The trigonometric leaves (Sun rotation, WCS) use the device's f64 libm, within
// an ulp or two of NumPy's; every other output is the reference's arithmetic in
// the reference's order (contraction off).
#include "comap_internal.h"

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

namespace {

constexpr double kD2R = M_PI / 180.0;   // np.pi / 180.0
constexpr double kR2D = 180.0 / M_PI;

inline unsigned grid_for(int64_t n, int64_t cap = 4096)
{
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, cap));
}

// ---------------------------------------------------------------- NumPy's pairwise sum
// np.sum of a contiguous f64 array = 0 + pw(b0) + pw(b1) + ... over the reduction
// buffer's 8192-element blocks b_k, where pw (pairwise_sum, loops_utils.h) sums
// n < 8 values one after the other from 0, n <= 128 values with 8 strided
// accumulators combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) plus the tail, and
// larger n as pw(first n2) + pw(rest) with n2 = n/2 rounded down to a multiple of 8.
// (Checked against numpy 2.2 np.sum / np.nanstd for lengths 1 .. 360k, NaNs included.)
constexpr int kPwBlock = 8192;
constexpr int kPwLeaf = 128;

// NumPy's pairwise sum (pw) of n <= 8192 values as a static plan, built on the host once
// per call (every series' last, partial buffer block has the same length): its leaves
// (<= 128 values, left to right) and its internal nodes in post-order, node = left +
// right.  Nodes 0 .. nleaf-1 are the leaves, nleaf + t the t-th internal node; the root
// is the last node.  (A device-side walk of the recursion on one thread kept its stack
// in scratch memory: ~0.19 ms per rms pass, all of it in the 76 partial blocks, r03s9.)
constexpr int kPwMaxLeaves = 80;   // pw splits at multiples of 8: <= 65 leaves below 8192
struct PwPlan {
    int16_t nleaf, ntri;
    int16_t loff[kPwMaxLeaves], llen[kPwMaxLeaves];
    uint8_t tri[3 * kPwMaxLeaves];   // (dst, left, right) node ids
};

static int pw_plan_rec(PwPlan &p, std::vector<int> &kids, int off, int n)
{
    if (n <= kPwLeaf) {
        const int id = p.nleaf++;
        p.loff[id] = (int16_t)off;
        p.llen[id] = (int16_t)n;
        return -1 - id;                        // leaf id, encoded negative until renumbering
    }
    int n2 = n / 2;
    n2 -= n2 % 8;
    const int a = pw_plan_rec(p, kids, off, n2);
    const int b = pw_plan_rec(p, kids, off + n2, n - n2);
    kids.push_back(a);
    kids.push_back(b);
    return (int)kids.size() / 2 - 1;           // internal node index (post-order)
}

static PwPlan pw_plan(int n)
{
    PwPlan p{};
    std::vector<int> kids;
    pw_plan_rec(p, kids, 0, n);
    p.ntri = (int16_t)(kids.size() / 2);
    auto id = [&](int v) { return v < 0 ? -1 - v : p.nleaf + v; };
    for (int t = 0; t < p.ntri; ++t) {
        p.tri[3 * t] = (uint8_t)(p.nleaf + t);
        p.tri[3 * t + 1] = (uint8_t)id(kids[2 * t]);
        p.tri[3 * t + 2] = (uint8_t)id(kids[2 * t + 1]);
    }
    return p;
}

// rms[r] = nanstd(d) / sqrt(2), d_i = x[1 + i] / s - x[0] / s, i < m = N - 1, N = n // 2 * 2
// (COMAPData.auto_rms with its tod[:-1:N] slice: COMAPData.py:205-208).  np.nanstd:
// NaN -> 0, avg = sum / count, (d - avg)^2 with NaN -> 0, var = sum / count; both sums
// are NumPy's pairwise sums: 0 + pw(b_0) + pw(b_1) + ... over 8192-value buffer blocks.
// Spread over the chip: one wave per (series, buffer block) computes pw(b_k) -- a full
// block is a balanced tree of 64 leaves of 128 values (lane l: leaf l, then a butterfly
// in the tree's pairing); the last, partial block walks pw's recursion -- and a final
// per-series step adds the block values in order.  PHASE 0 sums d (and counts the
// non-NaN d); PHASE 1 re-derives avg from the phase-0 block values and sums (d - avg)^2.
constexpr int kRmsWG = 512;   // one workgroup per (series, buffer block): 64 groups of 8 lanes

// One pw leaf of n values at lo by the 8 lanes of a group (j = lane % 8): lane j sums the
// values lo + j, lo + j + 8, ... below n - n % 8 (NumPy's accumulator r[j]), the group
// combines ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)), then the n % 8 tail is added
// in order; n < 8: a plain sequential sum.  The group's lane 0 holds the result.
template <typename Val>
__device__ __forceinline__ double pw_leaf8(Val v, int64_t lo, int n, int j)
{
#pragma clang fp contract(off)
    if (n < 8) {
        double r = 0.0;
        if (j == 0)
            for (int i = 0; i < n; ++i) r += v(lo + i);
        return r;
    }
    const int n8 = n - n % 8;
    double r = v(lo + j);
    for (int i = 8; i < n8; i += 8) r += v(lo + i + j);
    r = r + __shfl_xor(r, 1, 64);
    r = r + __shfl_xor(r, 2, 64);
    r = r + __shfl_xor(r, 4, 64);
    if (j == 0)
        for (int i = n8; i < n; ++i) r += v(lo + i);
    return r;
}

template <int PHASE>
__global__ void __launch_bounds__(kRmsWG) k_rms_blocks(const double *__restrict__ x, int64_t stride,
                                                       const int32_t *__restrict__ rows,
                                                       const double *__restrict__ scale, int64_t n, int32_t nrows,
                                                       int32_t nblk, const double *__restrict__ part0,
                                                       const int64_t *__restrict__ cnt0, double *__restrict__ part,
                                                       int64_t *__restrict__ cnt, const PwPlan plan)
{
#pragma clang fp contract(off)
    // leaf sums, then (partial block) the plan's internal nodes
    __shared__ double lsum[2 * kPwMaxLeaves];
    __shared__ unsigned long long cnt_s;
    const int64_t job = blockIdx.x;
    const int r = (int)(job / nblk), k = (int)(job % nblk);
    const int64_t m = n / 2 * 2 - 1;
    const double *xr = x + (int64_t)rows[r] * stride;
    const double s = scale[r];
    const double x0 = xr[0] / s;
    double avg = 0.0;
    if constexpr (PHASE == 1) {
        // numpy's sum over its 8192-element buffer blocks: 0 + b_0 + b_1 + ..., in order;
        // the block values are loaded 8 at a time before their adds (no load per add)
        double sum = 0.0;
        int64_t c = 0;
        const double *pp = part0 + (int64_t)r * nblk;
        const int64_t *cp = cnt0 + (int64_t)r * nblk;
        for (int q0 = 0; q0 < nblk; q0 += 8) {
            double pv[8];
            int64_t cv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                pv[u] = q0 + u < nblk ? pp[q0 + u] : 0.0;
                cv[u] = q0 + u < nblk ? cp[q0 + u] : 0;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (q0 + u < nblk) { sum += pv[u]; c += cv[u]; }
        }
        avg = sum / (double)c;
    }
    auto v = [&](int64_t i) {
        const double d = xr[1 + i] / s - x0;
        if (isnan(d)) return 0.0;
        if constexpr (PHASE == 0) {
            return d;
        } else {
            const double e = d - avg;
            return e * e;
        }
    };
    const int64_t b0 = (int64_t)k * kPwBlock;
    const int bn = (int)std::min<int64_t>(kPwBlock, m - b0);
    const bool full = bn == kPwBlock;
    if (threadIdx.x == 0) cnt_s = 0;
    __syncthreads();
    const int g = threadIdx.x >> 3, j = threadIdx.x & 7;
    unsigned long long c = 0;         // phase 0: non-NaN d (exact)
    if (full) {
        // one leaf per 8-lane group: lane j's 16 values (r[j]'s chain) loaded before any add
        const int64_t lo = b0 + (int64_t)kPwLeaf * g;
        double t[kPwLeaf / 8];
#pragma unroll
        for (int i = 0; i < kPwLeaf / 8; ++i) {
            const double d = xr[1 + lo + 8 * i + j] / s - x0;
            c += !isnan(d);
            if (isnan(d)) {
                t[i] = 0.0;
            } else if constexpr (PHASE == 0) {
                t[i] = d;
            } else {
                const double e = d - avg;
                t[i] = e * e;
            }
        }
        double r = t[0];
#pragma unroll
        for (int i = 1; i < kPwLeaf / 8; ++i) r += t[i];
        r = r + __shfl_xor(r, 1, 64);
        r = r + __shfl_xor(r, 2, 64);
        r = r + __shfl_xor(r, 4, 64);
        if (j == 0) lsum[g] = r;
    } else {
        if constexpr (PHASE == 0)
            for (int i = threadIdx.x; i < bn; i += kRmsWG) c += !isnan(xr[1 + b0 + i] / s - x0);
        for (int l = g; l < plan.nleaf; l += kRmsWG / 8) {
            const double t = pw_leaf8(v, b0 + plan.loff[l], plan.llen[l], j);
            if (j == 0) lsum[l] = t;
        }
    }
    if constexpr (PHASE == 0) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
        if ((threadIdx.x & 63) == 0) atomicAdd(&cnt_s, c);
    }
    __syncthreads();
    if (full) {
        // pw's balanced tree over the 64 leaves, level by level, left + right: lane i of
        // wave 0 holds leaf i, and at level o lane i (i % 2o == 0) adds lane i + o's
        // value -- the serial loop's additions in the same pairs, as 6 shuffles instead
        // of 63 dependent LDS read-modify-writes on one thread
        if (threadIdx.x < 64) {
            double v = lsum[threadIdx.x];
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const double w = __shfl_down(v, o, 64);
                if ((threadIdx.x & (2 * o - 1)) == 0) v = v + w;
            }
            if (threadIdx.x == 0) {
                part[job] = v;
                if constexpr (PHASE == 0) cnt[job] = (int64_t)cnt_s;
            }
        }
    } else if (threadIdx.x == 0) {
        for (int t = 0; t < plan.ntri; ++t)
            lsum[plan.tri[3 * t]] = lsum[plan.tri[3 * t + 1]] + lsum[plan.tri[3 * t + 2]];
        part[job] = lsum[plan.nleaf + plan.ntri - 1];
        if constexpr (PHASE == 0) cnt[job] = (int64_t)cnt_s;
    }
}

// rms[r] from the phase-1 block values: var = (0 + q_0 + q_1 + ...) / count
__global__ void k_rms_final(int32_t nrows, int32_t nblk, int64_t n, const double *__restrict__ part1,
                            const int64_t *__restrict__ cnt0, double *__restrict__ rms)
{
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nrows) return;
    if (n / 2 * 2 - 1 <= 0) { rms[r] = NAN; return; }
    double sq = 0.0;
    int64_t c = 0;
    for (int j = 0; j < nblk; ++j) { sq += part1[(int64_t)r * nblk + j]; c += cnt0[(int64_t)r * nblk + j]; }
    rms[r] = sqrt(sq / (double)c) / 1.4142135623730951;   // np.sqrt(2)
}

// ---------------------------------------------------------------- percentiles
__device__ __forceinline__ unsigned long long ord_key(double v)
{
    const unsigned long long u = __double_as_longlong(v);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}

__device__ __forceinline__ double from_key(unsigned long long k)
{
    const unsigned long long u = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
    return __longlong_as_double((long long)u);
}

// pct[r][2 which + {0, 1}] = np.percentile(v[good], {10, 90}), good = isfinite(az),
// v = az (which 0) or el (which 1) of row rows[r] (COMAPData.py:338-346).  NumPy's
// 'linear' rule: virtual index (n - 1) q, gamma its fraction, lerp between the order
// statistics at floor and floor + 1 (a + (b - a) g, or b - (b - a)(1 - g) for g >= 0.5);
// a NaN among the values makes the result NaN.  The order statistics come from one
// device-wide sort of every (row, which) series at once: orderable u64 keys (excluded
// samples last) sorted with their series id, then a stable sort by series id.
// (A per-series radix select in one workgroup took 1.6-2.2 ms per file: 38 workgroups
// and LDS-atomic histograms on nearly constant leading digits.)
__global__ void k_pct_keys(const double *__restrict__ az, const double *__restrict__ el, int64_t stride,
                           const int32_t *__restrict__ rows, int32_t nrows, int64_t n,
                           unsigned long long *__restrict__ key, uint16_t *__restrict__ sid,
                           unsigned long long *__restrict__ cnt)
{
    const int sg = blockIdx.y;                       // series = 2 r + which
    const int r = sg >> 1, which = sg & 1;
    const double *a = az + (int64_t)rows[r] * stride;
    const double *v = (which ? el : az) + (int64_t)rows[r] * stride;
    unsigned long long ng = 0, nn = 0;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
        const bool good = isfinite(a[t]);
        const double x = v[t];
        ng += good;
        nn += good && isnan(x);
        key[(int64_t)sg * n + t] = good ? ord_key(x) : ~0ull;
        if (sid) sid[(int64_t)sg * n + t] = (uint16_t)sg;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        ng += __shfl_xor(ng, o, 64);
        nn += __shfl_xor(nn, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&cnt[2 * sg], ng);
        atomicAdd(&cnt[2 * sg + 1], nn);
    }
}

// NumPy's linear-rule order statistics of a series with c good samples: ranks lo / hi of
// the 10th (k = 0) and 90th (k = 1) percentiles and the interpolation weight
__device__ __forceinline__ void pct_ranks(int64_t c, int k, int64_t &lo, int64_t &hi, double &g)
{
#pragma clang fp contract(off)
    const double q = k ? 0.9 : 0.1;   // np.true_divide(10, 100), (90, 100)
    const double virt = (double)(c - 1) * q;
    double prev = floor(virt);
    if (virt >= (double)(c - 1)) prev = -1.0;   // _get_indexes: above the last index -> the last value
    if (virt < 0) prev = 0.0;
    lo = prev < 0 ? c - 1 : (int64_t)prev;
    hi = prev < 0 ? c - 1 : std::min<int64_t>(lo + 1, c - 1);
    g = virt - prev;                            // gamma = virtual - previous index
}

// ---- exact order statistics by radix select (4 per series: the two percentiles' lo / hi
// ranks).  Six passes over the series' order-preserving keys, 11 bits at a time from the
// top (the last one 9): per pass a histogram of the next digit over the keys that match the target's
// prefix so far, then the digit whose cumulative count passes the remaining rank.  The
// selected key is the rank's value exactly (what a full sort would put there); 2 x 64-bit
// + 16-bit radix sorts of every series took 0.85 ms of the chain's 3.4 ms prep (r04zj).
constexpr int kSelBits = 11, kSelBins = 1 << kSelBits;
struct SelState {
    unsigned long long prefix;
    long long rank;
};

__global__ void k_sel_init(const unsigned long long *__restrict__ cnt, int32_t nseries, SelState *__restrict__ st)
{
    const int sg = blockIdx.x * blockDim.x + threadIdx.x;
    if (sg >= nseries) return;
    const int64_t c = (int64_t)cnt[2 * sg];
    for (int k = 0; k < 2; ++k) {
        int64_t lo = 0, hi = 0;
        double g;
        if (c > 0) pct_ranks(c, k, lo, hi, g);
        st[4 * sg + 2 * k] = {0ull, (long long)lo};
        st[4 * sg + 2 * k + 1] = {0ull, (long long)hi};
    }
}

// grid (chunks, series): the 4 targets' digit histograms of this chunk in LDS (a wave whose
// matching lanes share one digit adds once), merged into hist [series][4][kSelBins]
__global__ void __launch_bounds__(256) k_sel_hist(const unsigned long long *__restrict__ key, int64_t n, int shift,
                                                  int bits, const SelState *__restrict__ st,
                                                  uint32_t *__restrict__ hist)
{
    __shared__ uint32_t h[4][kSelBins];
    const int sg = blockIdx.y, lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 4 * kSelBins; i += blockDim.x) (&h[0][0])[i] = 0;
    __syncthreads();
    const int top = shift + bits;
    const unsigned long long hmask = top >= 64 ? 0ull : (~0ull << top);
    unsigned long long pre[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) pre[q] = st[4 * sg + q].prefix;
    const unsigned long long *k = key + (int64_t)sg * n;
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    for (int64_t t0 = (int64_t)blockIdx.x * blockDim.x; t0 < n; t0 += step) {   // wave-uniform trip count
        const int64_t t = t0 + threadIdx.x;
        const unsigned long long v = t < n ? k[t] : 0ull;
        const int d = (int)((v >> shift) & ((1u << bits) - 1u));
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const bool m = t < n && (v & hmask) == pre[q];
            const unsigned long long mb = __ballot(m);
            if (!mb) continue;
            const int l0 = __ffsll((long long)mb) - 1;
            const int d0 = __shfl(d, l0, 64);
            if (__ballot(m && d == d0) == mb) {
                if (lane == l0) atomicAdd(&h[q][d0], (uint32_t)__popcll(mb));
            } else if (m) {
                atomicAdd(&h[q][d], 1u);
            }
        }
    }
    __syncthreads();
    uint32_t *g = hist + (int64_t)sg * 4 * kSelBins;
    for (int i = threadIdx.x; i < 4 * kSelBins; i += blockDim.x) {
        const uint32_t c = (&h[0][0])[i];
        if (c) atomicAdd(g + i, c);
    }
}

// one wave per (series, target): the digit holding the remaining rank; zeroes the
// histogram for the next pass
__global__ void k_sel_pick(uint32_t *__restrict__ hist, int nt, int shift, SelState *__restrict__ st)
{
    const int lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    if (w >= nt) return;
    uint32_t *hb = hist + w * kSelBins;
    constexpr int per = kSelBins / 64;
    uint32_t c[per];
    long long tot = 0;
#pragma unroll
    for (int i = 0; i < per; ++i) {
        c[i] = hb[lane * per + i];
        tot += c[i];
    }
    long long inc = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const long long y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
    }
    const long long r = st[w].rank;
    const bool here = inc > r && inc - tot <= r;      // this lane's bins hold rank r
    const unsigned long long hb_ = __ballot(here);
    if (hb_) {
        const int ln = __ffsll((long long)hb_) - 1;
        if (lane == ln) {
            long long cum = inc - tot;
            int dsel = lane * per + per - 1;
            for (int i = 0; i < per; ++i) {
                if (cum + (long long)c[i] > r) { dsel = lane * per + i; break; }
                cum += c[i];
            }
            st[w].prefix |= (unsigned long long)dsel << shift;
            st[w].rank = r - cum;
        }
    }
#pragma unroll
    for (int i = 0; i < per; ++i) hb[lane * per + i] = 0u;
}

// the percentiles from the selected keys (sel: SelState [series][4])
__global__ void k_pct_pick_sel(const SelState *__restrict__ sel, const unsigned long long *__restrict__ cnt,
                               int32_t nseries, double *__restrict__ pct)
{
#pragma clang fp contract(off)
    const int sg = blockIdx.x * blockDim.x + threadIdx.x;
    if (sg >= nseries) return;
    const int r = sg >> 1, which = sg & 1;
    double *out = pct + 4 * (int64_t)r + 2 * which;
    const int64_t c = (int64_t)cnt[2 * sg];
    if (c == 0 || cnt[2 * sg + 1] > 0) { out[0] = NAN; out[1] = NAN; return; }
    for (int k = 0; k < 2; ++k) {
        int64_t lo, hi;
        double g;
        pct_ranks(c, k, lo, hi, g);
        const double av = from_key(sel[4 * sg + 2 * k].prefix), bv = from_key(sel[4 * sg + 2 * k + 1].prefix);
        const double diff = bv - av;
        double res = av + diff * g;
        if (g >= 0.5) res = bv - diff * (1.0 - g);
        out[k] = res;
    }
}

// sorted: series sg occupies [sg n, (sg + 1) n), its good samples first, ascending
__global__ void k_pct_pick(const unsigned long long *__restrict__ sorted, const unsigned long long *__restrict__ cnt,
                           int32_t nseries, int64_t n, double *__restrict__ pct)
{
#pragma clang fp contract(off)
    const int sg = blockIdx.x * blockDim.x + threadIdx.x;
    if (sg >= nseries) return;
    const int r = sg >> 1, which = sg & 1;
    double *out = pct + 4 * (int64_t)r + 2 * which;
    const int64_t c = cnt ? (int64_t)cnt[2 * sg] : 0;
    if (c == 0 || cnt[2 * sg + 1] > 0) { out[0] = NAN; out[1] = NAN; return; }
    const double q[2] = {0.1, 0.9};   // np.true_divide(10, 100), (90, 100)
    for (int k = 0; k < 2; ++k) {
        const double virt = (double)(c - 1) * q[k];
        double prev = floor(virt);
        if (virt >= (double)(c - 1)) prev = -1.0;   // _get_indexes: above the last index -> the last value
        if (virt < 0) prev = 0.0;
        const int64_t lo = prev < 0 ? c - 1 : (int64_t)prev;
        const int64_t hi = prev < 0 ? c - 1 : std::min<int64_t>(lo + 1, c - 1);
        const double g = virt - prev;                // gamma = virtual - previous index
        const double av = from_key(sorted[(int64_t)sg * n + lo]), bv = from_key(sorted[(int64_t)sg * n + hi]);
        const double diff = bv - av;
        double res = av + diff * g;
        if (g >= 0.5) res = bv - diff * (1.0 - g);
        out[k] = res;
    }
}

// ---------------------------------------------------------------- per-sample gather
// healpy Rotator.__call__ (astro.Rotator): (theta, phi) -> rotated (theta', phi').
__device__ __forceinline__ void rotate(const double *m, double theta, double phi, double &to, double &po)
{
#pragma clang fp contract(off)
    const double st = sin(theta);
    const double v0 = st * cos(phi), v1 = st * sin(phi), v2 = cos(theta);
    const double x = (m[0] * v0 + m[1] * v1) + m[2] * v2;
    const double y = (m[3] * v0 + m[4] * v1) + m[5] * v2;
    const double z = (m[6] * v0 + m[7] * v1) + m[8] * v2;
    const double rr = sqrt((x * x + y * y) + z * z);
    to = acos(z / rr);
    po = atan2(y, x);
}

// CelestialWCS world -> pixel + transform_to_1d (mapmaking/wcs.py; COMAPData.py:83-117)
__device__ __forceinline__ int32_t wcs_pixel(const comap_prep_wcs &w, double lng, double lat)
{
#pragma clang fp contract(off)
    if (w.galactic) {   // Rotator(coord=['C','G']) on ((90 - y) pi/180, x pi/180) (COMAPData.py:411-415)
        double gb, gl;
        rotate(w.gal_rot, (90.0 - lat) * M_PI / 180.0, lng * M_PI / 180.0, gb, gl);
        lng = gl * 180.0 / M_PI;
        lat = (M_PI / 2 - gb) * 180.0 / M_PI;
    }
    const double e0 = w.eul[0], e1 = w.eul[1], e2 = w.eul[2], ce1 = w.eul[3], se1 = w.eul[4];
    const double dl = (lng - e0) * kD2R;
    const double cl = cos(lat * kD2R), sl = sin(lat * kD2R);
    const double cdl = cos(dl);
    double x = sl * se1 - cl * ce1 * cdl;
    if (fabs(x) < 1e-5) x = -cos(lat * kD2R + e1 * kD2R) + cl * ce1 * (1 - cdl);
    const double y = -cl * sin(dl);
    double phi = e2 + atan2(y, x) * kR2D;
    phi = phi > 180 ? phi - 360 : (phi < -180 ? phi + 360 : phi);
    const double z = sl * ce1 + cl * se1 * cdl;
    const double theta = asin(fmin(fmax(z, -1.0), 1.0)) * kR2D;
    double ix, iy;
    if (w.proj == 0) {
        ix = phi;
        iy = theta;
    } else {
        const double r = w.proj == 1 ? kR2D * cos(theta * kD2R) : kR2D / tan(theta * kD2R);
        ix = r * sin(phi * kD2R);
        iy = -r * cos(phi * kD2R);
    }
    const double px = floor(((w.crpix[0] + ix / w.cdelt[0]) - 1) + 0.5);
    const double py = floor(((w.crpix[1] + iy / w.cdelt[1]) - 1) + 0.5);
    if (!(px >= 0 && px <= (double)(w.nx - 1)) || !(py >= 0 && py <= (double)(w.ny - 1))) return -1;
    return (int32_t)(py * (double)w.nx + px);
}

constexpr int kScanLds = 128;

// One thread per output sample (row, column) of one file (get_tod COMAPData.py:306-376,
// read_pixels :404-425): column -> (scan, sample) through the scan table.
__global__ void __launch_bounds__(256) k_prep_gather(comap_prep_file f, comap_prep_wcs wc, comap_prep_out o)
{
#pragma clang fp contract(off)
    // the scan of a column = the last scan whose first column is <= it (zero-length scans
    // share the next scan's first column and are skipped); a file of up to kScanLds scans
    // keeps its table in LDS, a longer one is binary-searched in global memory
    __shared__ int64_t sc[3 * kScanLds];
    const bool lds = f.n_scans <= kScanLds;
    if (lds) {
        for (int i = threadIdx.x; i < 3 * f.n_scans; i += blockDim.x) sc[i] = f.scans[i];
        __syncthreads();
    }
    const int64_t col = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int row = blockIdx.y;
    if (col >= f.datasize) return;
    const int64_t *tab = lds ? sc : f.scans;
    int lo = 0, hi = f.n_scans - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (tab[3 * mid + 2] <= col) lo = mid;
        else hi = mid - 1;
    }
    const int s = lo;
    const int64_t N = tab[3 * s + 1], j = col - tab[3 * s + 2], t = tab[3 * s] + j;
    const int64_t oi = o.offset + (int64_t)row * f.datasize + col;
    // pointing (read_pixels fills row i from the file row of output_feed_index[i])
    const int ps = f.pix_src[row];
    int32_t pix = 0;
    if (f.pixels) pix = (int32_t)f.pixels[(int64_t)row * f.datasize + col];
    else if (ps >= 0) pix = wcs_pixel(wc, f.ra[ps * f.point_stride + t], f.dec[ps * f.point_stride + t]);
    o.pix[oi] = pix;
    o.obsid[oi] = f.obsid;
    const int rs = f.row_src[row];
    if (rs < 0) {   // bad feed: the row stays zero (COMAPData.py:314-315)
        o.az[oi] = o.el[oi] = o.ra[oi] = o.dec[oi] = 0.0;
        o.feedid[oi] = 0;
        for (int b = 0; b < f.n_bands; ++b) o.tod[b * o.band_stride + oi] = o.w[b * o.band_stride + oi] = 0.0;
        return;
    }
    const int64_t pt = rs * f.point_stride + t;
    const double azv = f.az[pt], elv = f.el[pt], rav = f.ra[pt], decv = f.dec[pt];
    // get_sun_centric_coords + haversine (COMAPData.py:213-236, 326-327)
    double theta = M_PI / 2. - decv * M_PI / 180.;
    double phi = rav * M_PI / 180.;
    if (isfinite(rav) && isfinite(decv)) rotate(f.sun_rot, theta, phi, theta, phi);
    const double sp2 = sin(phi / 2), st2 = sin(theta / 2);
    const double dist = 2 * asin(sqrt(sp2 * sp2 + cos(0.0) * cos(phi) * (st2 * st2))) * 180.0 / M_PI;
    o.az[oi] = azv;
    o.el[oi] = elv;
    o.ra[oi] = dist;
    o.dec[oi] = theta;
    o.feedid[oi] = f.row_feed[row];
    const double *pc = f.row_pct + 4 * (int64_t)row;
    const int64_t nten = (int64_t)((double)N * 0.1);
    const bool cut = dist < 10 || azv < pc[0] || azv > pc[1] || elv < pc[2] || elv > pc[3] || j < nten ||
                     j >= N - nten;
    for (int b = 0; b < f.n_bands; ++b) {
        const int band = f.bands[b];
        const double tv = f.tod[rs * f.tod_feed_stride + band * f.tod_band_stride + t] / f.row_cal[row * 4 + b];
        double wv = f.row_w[row * 4 + b];
        if (cut || (f.spike && f.spike[rs * f.spike_feed_stride + band * f.spike_band_stride + t])) wv = 0.0;
        o.tod[b * o.band_stride + oi] = tv;
        o.w[b * o.band_stride + oi] = wv;
    }
}

// ---------------------------------------------------------------- running-median high-pass
// segment k = x[seg[2k] .. seg[2k] + seg[2k+1]); its median input = the non-zero samples
// (bad = tod == 0, COMAPData.py:357-360), NaN and +-inf included as in the reference.  A
// segment of <= 2w values takes np.nanmedian (:79, NaN ignored); a longer one the running
// median, where the order-statistics plan serves NaN-free segments and a segment holding
// NaN is replayed through the reference's two-heap (comap_median_replay), whose result for
// NaN follows its insertion history.
__device__ __forceinline__ bool hp_keep(double v) { return v != 0.0; }

// One 1024-thread workgroup per segment (a chain segment holds ~8 k samples: 16 waves
// keep enough loads in flight; 256 threads left the pass latency-bound at ~1.2 TB/s).
constexpr int kSegThreads = 1024;
constexpr int kSegItems = 4;     // consecutive samples per thread per compaction round

__global__ void __launch_bounds__(kSegThreads) k_seg_count(const double *__restrict__ x,
                                                           const int64_t *__restrict__ seg,
                                                           int64_t *__restrict__ cnt)
{
    // cnt[k] = median-input values of segment k, cnt[nseg + k] = NaN among them
    __shared__ unsigned c_s[kSegThreads / 64], q_s[kSegThreads / 64];
    const double *p = x + seg[2 * blockIdx.x];
    const int64_t n = seg[2 * blockIdx.x + 1];
    unsigned c = 0, q = 0;
    int64_t i = threadIdx.x;
    for (; i + kSegThreads < n; i += 2 * kSegThreads) {     // two independent loads per trip
        const double a = p[i], b = p[i + kSegThreads];
        c += hp_keep(a) + hp_keep(b);
        q += isnan(a) + isnan(b);
    }
    if (i < n) {
        c += hp_keep(p[i]);
        q += isnan(p[i]);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        c += __shfl_xor(c, o, 64);
        q += __shfl_xor(q, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        c_s[threadIdx.x >> 6] = c;
        q_s[threadIdx.x >> 6] = q;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0, u = 0;
        for (int v = 0; v < kSegThreads / 64; ++v) {
            t += c_s[v];
            u += q_s[v];
        }
        cnt[blockIdx.x] = (int64_t)t;
        cnt[gridDim.x + blockIdx.x] = (int64_t)u;
    }
}

// compacted values (in order) and their positions, one workgroup per segment: each round
// takes kSegThreads x kSegItems consecutive samples (kSegItems per thread), one block scan
__global__ void __launch_bounds__(kSegThreads) k_seg_compact(const double *__restrict__ x,
                                                             const int64_t *__restrict__ seg,
                                                             const int64_t *__restrict__ off,
                                                             double *__restrict__ vals, int32_t *__restrict__ pos)
{
    typedef hipcub::BlockScan<int, kSegThreads> Scan;
    __shared__ typename Scan::TempStorage ts;
    const double *p = x + seg[2 * blockIdx.x];
    const int64_t n = seg[2 * blockIdx.x + 1];
    double *vo = vals + off[blockIdx.x];
    int32_t *po = pos + off[blockIdx.x];
    int64_t run = 0;
    for (int64_t b = 0; b < n; b += (int64_t)kSegThreads * kSegItems) {
        const int64_t i0 = b + (int64_t)threadIdx.x * kSegItems;
        double v[kSegItems];
        int k[kSegItems], ex[kSegItems];
#pragma unroll
        for (int j = 0; j < kSegItems; ++j) {
            v[j] = i0 + j < n ? p[i0 + j] : 0.0;
            k[j] = i0 + j < n && hp_keep(v[j]);
        }
        int tot = 0;
        Scan(ts).ExclusiveSum(k, ex, tot);
#pragma unroll
        for (int j = 0; j < kSegItems; ++j)
            if (k[j]) {
                vo[run + ex[j]] = v[j];
                po[run + ex[j]] = (int32_t)(i0 + j);
            }
        run += tot;
        __syncthreads();     // the scan's temporary storage is reused next round
    }
}

// Segments with 1 .. 2w median-input values: np.nanmedian of the values (COMAPData.py:79),
// broadcast.  One workgroup per segment (the others exit at once): every non-NaN value's
// rank = the non-NaN values below it plus the equal ones before it (+-inf compare like any
// value), so the sorted order needs no sort; NaN is ignored (all NaN: the median is NaN);
// even counts average the two middle values as np.median does ((a + b) / 2).
constexpr int kSmallSeg = 2048;
__global__ void __launch_bounds__(256) k_seg_small_median(const double *__restrict__ vals,
                                                          const int64_t *__restrict__ off,
                                                          const int64_t *__restrict__ cnt, int64_t nmax,
                                                          double *__restrict__ filt)
{
    const int64_t n = cnt[blockIdx.x];
    if (n == 0 || n > nmax) return;
    __shared__ double v[kSmallSeg], srt[kSmallSeg];
    __shared__ int nn_s;
    const int64_t o0 = off[blockIdx.x];
    if (threadIdx.x == 0) nn_s = 0;
    __syncthreads();
    int nn = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        v[i] = vals[o0 + i];
        nn += !isnan(v[i]);
    }
    atomicAdd(&nn_s, nn);
    __syncthreads();
    const int m = nn_s;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const double x = v[i];
        if (isnan(x)) continue;
        int r = 0;
        for (int j = 0; j < n; ++j) r += (v[j] < x) || (v[j] == x && j < i);
        srt[r] = x;
    }
    __syncthreads();
    const double med = m == 0 ? (double)NAN : (m & 1) ? srt[m / 2] : (srt[m / 2 - 1] + srt[m / 2]) / 2.0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) filt[o0 + i] = med;
}

// grid (segment, 256-value chunk): every compacted value back to its sample
__global__ void __launch_bounds__(256) k_seg_subtract(double *__restrict__ x, const int64_t *__restrict__ seg,
                                                      const int64_t *__restrict__ off,
                                                      const int64_t *__restrict__ cnt,
                                                      const double *__restrict__ filt,
                                                      const int32_t *__restrict__ pos)
{
    const int64_t n = cnt[blockIdx.x];
    double *p = x + seg[2 * blockIdx.x];
    const int64_t o0 = off[blockIdx.x];
    for (int64_t i = (int64_t)blockIdx.y * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.y * 256)
        p[pos[o0 + i]] -= filt[o0 + i];
}

// ---------------------------------------------------------------- NaN and empty-offset cuts
// per band: tod NaN / inf -> tod = w = 0 (COMAPData.py:550-552); keep[b][o] = any w != 0
// over the offset (:554-557); kept[o] = any band keeps o
// One wave per offset (lanes over its samples, coalesced): NaN tod -> tod = w = 0, then
// keep[b][o] = any w != 0 in band b, kept[o] = any band keeps it.
__global__ void __launch_bounds__(256) k_cut_flags(double *__restrict__ tod, double *__restrict__ w,
                                                   int64_t band_stride, int nb, int64_t NO, int L,
                                                   uint8_t *__restrict__ keep, int32_t *__restrict__ kept)
{
    const int lane = threadIdx.x & 63;
    const int64_t o = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (o >= NO) return;
    int any_band = 0;
    for (int b = 0; b < nb; ++b) {
        double *tp = tod + b * band_stride + o * L, *wp = w + b * band_stride + o * L;
        bool any = false;
        for (int j = lane; j < L; j += 64) {
            if (!isfinite(tp[j])) { tp[j] = 0.0; wp[j] = 0.0; }
            any |= wp[j] != 0.0;
        }
        any = __ballot(any) != 0ull;
        if (lane == 0) keep[b * NO + o] = (uint8_t)any;
        any_band |= any;
    }
    if (lane == 0) kept[o] = any_band;
}
__global__ void k_cut_copy(const comap_prep_out in, comap_prep_out out, int nb, int64_t NO, int L,
                           const int32_t *__restrict__ kept, const int32_t *__restrict__ newo,
                           const uint8_t *__restrict__ keep, uint8_t *__restrict__ keep_out, int64_t NO_out)
{
    const int64_t total = NO * L;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t o = i / L;
        if (!kept[o]) continue;
        const int64_t k = (int64_t)newo[o] * L + i % L;
        for (int b = 0; b < nb; ++b) {
            out.tod[b * out.band_stride + k] = in.tod[b * in.band_stride + i];
            const double wv = in.w[b * in.band_stride + i];
            out.w[b * out.band_stride + k] = isfinite(wv) ? wv : 0.0;
            if (i % L == 0) keep_out[b * NO_out + newo[o]] = keep[b * NO + o];
        }
        out.az[k] = in.az[i];
        out.el[k] = in.el[i];
        out.ra[k] = in.ra[i];
        out.dec[k] = in.dec[i];
        out.feedid[k] = in.feedid[i];
        out.obsid[k] = in.obsid[i];
        out.pix[k] = in.pix[i];
    }
}

}  // namespace

extern "C" int comap_prep_auto_rms(comap_ctx *ctx, const double *x, int64_t row_stride, const int32_t *rows,
                                   const double *scale, int32_t nrows, int64_t n, double *rms)
{
    if (!ctx || !x || !rows || !scale || !rms || nrows < 0 || n < 0) return -1;
    COMAP_DEVICE_GUARD(ctx);
    if (nrows == 0) return 0;
    const int64_t m = n / 2 * 2 - 1;
    const int32_t nblk = (int32_t)std::max<int64_t>(1, (m + kPwBlock - 1) / kPwBlock);
    const size_t nj = (size_t)nrows * nblk;
    // block values in the context scratch (stream-ordered: no allocation or sync per call)
    void *sc = nullptr;
    if (int rc = comap_scratch(ctx, 24 * nj, &sc)) return rc;
    double *p0 = (double *)sc, *p1 = p0 + nj;
    int64_t *c0 = (int64_t *)(p1 + nj);
    if (m > 0) {
        const unsigned g = (unsigned)nj;
        const PwPlan plan = pw_plan((int)(m - (int64_t)(nblk - 1) * kPwBlock));   // the last block's tree
        k_rms_blocks<0><<<g, kRmsWG, 0, ctx->stream>>>(x, row_stride, rows, scale, n, nrows, nblk, nullptr, nullptr, p0,
                                                      c0, plan);
        k_rms_blocks<1><<<g, kRmsWG, 0, ctx->stream>>>(x, row_stride, rows, scale, n, nrows, nblk, p0, c0, p1, nullptr,
                                                      plan);
    }
    k_rms_final<<<(nrows + 255) / 256, 256, 0, ctx->stream>>>(nrows, nblk, n, p1, c0, rms);
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}

extern "C" int comap_prep_percentiles(comap_ctx *ctx, const double *az, const double *el, int64_t row_stride,
                                      const int32_t *rows, int32_t nrows, int64_t n, double *pct)
{
    if (!ctx || !az || !el || !rows || !pct || nrows < 0 || n < 0) return -1;
    COMAP_DEVICE_GUARD(ctx);
    if (nrows == 0) return 0;
    if (2 * (int64_t)nrows > 65535) return comap_fail(ctx, -1, "comap_prep_percentiles: too many rows");
    hipStream_t st = ctx->stream;
    const int ns = 2 * nrows;
    const int64_t tot = (int64_t)ns * n;
    if (tot >= (1ll << 31)) return comap_fail(ctx, -1, "comap_prep_percentiles: too many samples");
    if (n == 0) {
        k_pct_pick<<<(ns + 255) / 256, 256, 0, st>>>(nullptr, nullptr, ns, 0, pct);   // NaN: no good sample
        COMAP_LAUNCH_CHECK(ctx);
        return 0;
    }
    DevTemps tmp(st, false);   // freed behind the queued work (stream-safe cache): no host wait
    unsigned long long *k0 = nullptr, *cnt = nullptr;
    SelState *sel = nullptr;
    uint32_t *hist = nullptr;
    const int nt = 4 * ns;
    COMAP_CHECK(ctx, tmp.alloc(&k0, (size_t)tot));
    COMAP_CHECK(ctx, tmp.alloc(&cnt, 2 * (size_t)ns));
    COMAP_CHECK(ctx, tmp.alloc(&sel, (size_t)nt));
    COMAP_CHECK(ctx, tmp.alloc(&hist, (size_t)nt * kSelBins));
    COMAP_CHECK(ctx, hipMemsetAsync(cnt, 0, 16 * (size_t)ns, st));
    COMAP_CHECK(ctx, hipMemsetAsync(hist, 0, 4 * (size_t)nt * kSelBins, st));
    const dim3 g((unsigned)std::min<int64_t>(64, (n + 255) / 256), (unsigned)ns);
    k_pct_keys<<<g, 256, 0, st>>>(az, el, row_stride, rows, nrows, n, k0, nullptr, cnt);
    COMAP_LAUNCH_CHECK(ctx);
    k_sel_init<<<(ns + 255) / 256, 256, 0, st>>>(cnt, ns, sel);
    COMAP_LAUNCH_CHECK(ctx);
    const dim3 gh((unsigned)std::min<int64_t>(32, (n + 255) / 256), (unsigned)ns);
    for (int top = 64; top > 0; top -= kSelBits) {          // digits 53-63, 42-52, ..., 9-19, 0-8
        const int sh = std::max(top - kSelBits, 0), bits = top - sh;
        k_sel_hist<<<gh, 256, 0, st>>>(k0, n, sh, bits, sel, hist);
        COMAP_LAUNCH_CHECK(ctx);
        k_sel_pick<<<(nt + 3) / 4, 256, 0, st>>>(hist, nt, sh, sel);
        COMAP_LAUNCH_CHECK(ctx);
    }
    k_pct_pick_sel<<<(ns + 255) / 256, 256, 0, st>>>(sel, cnt, ns, pct);
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}

extern "C" int comap_prep_gather(comap_ctx *ctx, const comap_prep_file *f, const comap_prep_wcs *wcs,
                                 const comap_prep_out *out)
{
    if (!ctx || !f || !out || (!wcs && !f->pixels)) return -1;
    COMAP_DEVICE_GUARD(ctx);
    if (f->n_scans < 1) return comap_fail(ctx, -1, "comap_prep_gather: no scan in the file");
    if (f->n_bands < 1 || f->n_bands > 4) return comap_fail(ctx, -1, "comap_prep_gather: 1 to 4 bands");
    if (f->n_rows < 1 || f->datasize < 1) return 0;
    if (f->n_rows > 65535) return comap_fail(ctx, -1, "comap_prep_gather: too many rows");
    comap_prep_wcs w{};
    if (wcs) w = *wcs;
    const dim3 grid((unsigned)((f->datasize + 255) / 256), (unsigned)f->n_rows);
    k_prep_gather<<<grid, 256, 0, ctx->stream>>>(*f, w, *out);
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}

// Segments' median inputs -> medfilt (reflect-3 middle third, median_kernels.hip) for
// the segments with more than 2 w values, np.nanmedian of the values for the others
// (COMAPData.py:72-81) -> subtracted in place.  Synchronises the host once (the
// segment lengths size the median plan).
extern "C" int comap_prep_highpass(comap_ctx *ctx, double *x, const int64_t *seg_dev, int32_t nseg, int32_t w)
{
    if (!ctx || !x || (!seg_dev && nseg > 0) || w < 1) return -1;
    COMAP_DEVICE_GUARD(ctx);
    if (nseg == 0) return 0;
    hipStream_t st = ctx->stream;
    DevTemps tmp(st, false);   // freed behind the queued work (stream-safe cache): no host wait
    int64_t *cnt = nullptr, *off = nullptr;
    COMAP_CHECK(ctx, tmp.alloc(&cnt, 2 * (size_t)nseg));
    COMAP_CHECK(ctx, tmp.alloc(&off, (size_t)nseg));
    k_seg_count<<<nseg, kSegThreads, 0, st>>>(x, seg_dev, cnt);
    COMAP_LAUNCH_CHECK(ctx);
    std::vector<int64_t> c(2 * (size_t)nseg), o(nseg);     // counts, then NaN counts
    COMAP_CHECK(ctx, hipMemcpyAsync(c.data(), cnt, 16 * (size_t)nseg, hipMemcpyDeviceToHost, st));
    COMAP_CHECK(ctx, hipStreamSynchronize(st));
    int64_t total = 0, cmax = 0;
    for (int k = 0; k < nseg; ++k) {
        o[k] = total;
        total += c[k];
        cmax = std::max(cmax, c[k]);
    }
    if (total == 0) return 0;
    double *vals = nullptr, *filt = nullptr;
    int32_t *pos = nullptr;
    COMAP_CHECK(ctx, tmp.alloc(&vals, (size_t)total));
    COMAP_CHECK(ctx, tmp.alloc(&filt, (size_t)total));
    COMAP_CHECK(ctx, tmp.alloc(&pos, (size_t)total));
    COMAP_CHECK(ctx, comap_upload(off, o.data(), 8 * (size_t)nseg, st));
    k_seg_compact<<<nseg, kSegThreads, 0, st>>>(x, seg_dev, off, vals, pos);
    COMAP_LAUNCH_CHECK(ctx);
    std::vector<MedJob> jobs, replay;
    std::vector<int> small;      // short segments the device kernel cannot hold (2w > kSmallSeg)
    const int64_t nsmall_dev = 2 * (int64_t)w <= kSmallSeg ? 2 * (int64_t)w : 0;
    bool any_small_dev = false;
    for (int k = 0; k < nseg; ++k) {
        if (c[k] == 0) continue;
        if (c[k] <= nsmall_dev) {
            any_small_dev = true;
            continue;
        }
        if (c[k] > 2 * (int64_t)w) {
            MedJob j;
            j.src = vals + o[k];
            j.dst = filt + o[k];
            j.n = c[k];
            j.out_lo = c[k];
            j.out_hi = 2 * c[k];
            j.mode = 1;
            j.pad_ = 0;
            j.gate = nullptr;
            (c[nseg + k] > 0 ? replay : jobs).push_back(j);     // NaN: the two-heap's own order
        } else {
            small.push_back(k);
        }
    }
    int rc = comap_median_replay(ctx, replay, w, st);
    if (rc) return rc;
    // (a chunked small-window median -- one workgroup per 256 outputs bitonic-sorting its
    // union window in registers / LDS -- matched this bit for bit but ran 1.9 ms against
    // the plan's ~0.9 ms at the chain's 912 segments, r03t7: removed)
    if (!jobs.empty()) {
        MedPlan mp;
        const bool prof = getenv("COMAP_PREP_PROFILE") && getenv("COMAP_PREP_PROFILE")[0] == '1';
        auto now = [] { return std::chrono::steady_clock::now(); };
        const auto t0 = now();
        rc = comap_median_plan(ctx, &mp, jobs, w);
        const auto t1 = now();
        if (!rc) rc = comap_median_run(ctx, &mp);
        const auto t2 = now();
        // the plan's buffers go back to the temporaries cache behind an event after the walk
        // (reuse on another stream waits for it): no host wait
        comap_median_plan_free(&mp);
        const auto t3 = now();
        if (prof) {
            auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
            fprintf(stderr, "[comap_prep_highpass] plan %.0f us, run enqueue %.0f us, free %.0f us (%zu jobs)\n",
                    us(t0, t1), us(t1, t2), us(t2, t3), jobs.size());
        }
        if (rc) return rc;
    }
    // short segments: np.nanmedian of their (non-NaN) values -- a mean of the two middle
    // values for an even count -- broadcast (np.ones(n) * m)
    if (any_small_dev) {
        k_seg_small_median<<<nseg, 256, 0, st>>>(vals, off, cnt, nsmall_dev, filt);
        COMAP_LAUNCH_CHECK(ctx);
    }
    for (int k : small) {
        std::vector<double> v(c[k]);
        COMAP_CHECK(ctx, hipMemcpyAsync(v.data(), vals + o[k], 8 * v.size(), hipMemcpyDeviceToHost, st));
        COMAP_CHECK(ctx, hipStreamSynchronize(st));
        const size_t n = v.size();
        v.erase(std::remove_if(v.begin(), v.end(), [](double a) { return std::isnan(a); }), v.end());
        std::sort(v.begin(), v.end());
        const size_t m = v.size();     // np.nanmedian: NaN ignored, all NaN -> NaN
        const double med = m == 0 ? NAN : m % 2 ? v[m / 2] : (v[m / 2 - 1] + v[m / 2]) / 2.0;
        std::vector<double> f(n, med);
        COMAP_CHECK(ctx, comap_upload(filt + o[k], f.data(), 8 * n, st));
    }
    const unsigned chunks = (unsigned)std::min<int64_t>((cmax + 255) / 256, 4096);
    k_seg_subtract<<<dim3((unsigned)nseg, chunks), 256, 0, st>>>(x, seg_dev, off, cnt, filt, pos);
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}

// NaN cut, per-band keep mask, compaction of the union of kept offsets.  n_kept_out: the
// number of kept offsets (host; synchronises).  out arrays hold >= n_kept * L samples
// (out.band_stride >= that); keep_out [nb][n_kept] (row stride n_kept_cap).
extern "C" int comap_prep_cut(comap_ctx *ctx, const comap_prep_out *in, int32_t nb, int64_t n_samples,
                              int32_t offset_length, const comap_prep_out *out, uint8_t *keep_out,
                              int64_t n_kept_cap, int64_t *n_kept_out)
{
    if (!ctx || !in || !out || !keep_out || !n_kept_out || nb < 1 || nb > 4 || offset_length < 1) return -1;
    COMAP_DEVICE_GUARD(ctx);
    const int L = offset_length;
    if (n_samples % L) return comap_fail(ctx, -1, "comap_prep_cut: n_samples must be a multiple of offset_length");
    const int64_t NO = n_samples / L;
    *n_kept_out = 0;
    if (NO == 0) return 0;
    hipStream_t st = ctx->stream;
    DevTemps tmp(st, false);   // freed behind the queued work (stream-safe cache): no host wait
    uint8_t *keep = nullptr;
    int32_t *kept = nullptr, *newo = nullptr;
    COMAP_CHECK(ctx, tmp.alloc(&keep, (size_t)nb * NO));
    COMAP_CHECK(ctx, tmp.alloc(&kept, (size_t)NO + 1));
    COMAP_CHECK(ctx, tmp.alloc(&newo, (size_t)NO + 1));
    k_cut_flags<<<(unsigned)((NO + 3) / 4), 256, 0, st>>>(in->tod, in->w, in->band_stride, nb, NO, L, keep, kept);
    COMAP_LAUNCH_CHECK(ctx);
    size_t tb = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tb, kept, newo, (int)(NO + 1), st);
    char *ct = nullptr;
    COMAP_CHECK(ctx, tmp.alloc(&ct, tb));
    COMAP_CHECK(ctx, hipMemsetAsync(kept + NO, 0, 4, st));
    COMAP_CHECK(ctx, hipcub::DeviceScan::ExclusiveSum(ct, tb, kept, newo, (int)(NO + 1), st));
    int32_t nk = 0;
    COMAP_CHECK(ctx, hipMemcpyAsync(&nk, newo + NO, 4, hipMemcpyDeviceToHost, st));
    COMAP_CHECK(ctx, hipStreamSynchronize(st));
    if (nk > n_kept_cap) return comap_fail(ctx, -1, "comap_prep_cut: output capacity too small");
    k_cut_copy<<<grid_for(NO * L, 8192), 256, 0, st>>>(*in, *out, nb, NO, L, kept, newo, keep, keep_out, n_kept_cap);
    COMAP_LAUNCH_CHECK(ctx);
    *n_kept_out = nk;
    return 0;
}
