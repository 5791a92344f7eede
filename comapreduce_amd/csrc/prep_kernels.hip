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
#include <cmath>
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

// Post-order walk of pw's recursion over [0, n): leaf(off, len) is called for the
// leaves left to right and returns the leaf's value; returns left + right at every
// internal node.  Explicit stack (depth <= 8 for n <= 8192).
template <typename Leaf>
__device__ double pairwise_tree(int n, Leaf leaf)
{
    int so[24], sn[24], sst[24];
    double sv[24];
    int sp = 0;
    so[0] = 0; sn[0] = n; sst[0] = 0;
    double v = 0.0;
    bool have = false;   // v holds the value of the node just finished
    while (true) {
        if (!have) {
            if (sn[sp] <= kPwLeaf) {
                v = leaf(so[sp], sn[sp]);
                have = true;
                if (sp == 0) return v;
                --sp;
                continue;
            }
            int n2 = sn[sp] / 2;
            n2 -= n2 % 8;
            so[sp + 1] = so[sp]; sn[sp + 1] = n2; sst[sp + 1] = 0;
            sst[sp] = 0;
            ++sp;
        } else {
            int n2 = sn[sp] / 2;
            n2 -= n2 % 8;
            if (sst[sp] == 0) {   // left child done: keep it, walk the right child
                sv[sp] = v;
                sst[sp] = 1;
                have = false;
                so[sp + 1] = so[sp] + n2; sn[sp + 1] = sn[sp] - n2; sst[sp + 1] = 0;
                ++sp;
            } else {              // right child done
                v = sv[sp] + v;
                if (sp == 0) return v;
                --sp;
            }
        }
    }
}

// One leaf of pw: values v(lo .. lo + n - 1), n <= 128.
template <typename Val>
__device__ __forceinline__ double pw_leaf(Val v, int64_t lo, int n)
{
#pragma clang fp contract(off)
    if (n < 8) {
        double r = 0.0;
        for (int i = 0; i < n; ++i) r += v(lo + i);
        return r;
    }
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = v(lo + j);
    int i = 8;
    const int n8 = n - n % 8;
    for (; i < n8; i += 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] += v(lo + i + j);
    }
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += v(lo + i);
    return res;
}

constexpr int kRmsThreads = 256;
constexpr int kRmsGroup = 16;                                  // buffer blocks per LDS round
constexpr int kRmsLeafCap = kRmsGroup * (kPwBlock / 64) + 256;   // >= leaves of 16 blocks

// np.sum over m values v(0 .. m-1) with NumPy's tree, by one 256-thread block: leaves
// listed by thread 0, summed by all threads, folded by thread 0 in the tree's order.
template <typename Val>
__device__ double numpy_sum(Val v, int64_t m, int32_t *loff, int32_t *llen, double *lsum, int32_t *bleaf,
                            double *bcast)
{
    double total = 0.0;   // thread 0's running value
    const int64_t nblk = (m + kPwBlock - 1) / kPwBlock;
    for (int64_t g0 = 0; g0 < nblk; g0 += kRmsGroup) {
        const int gn = (int)std::min<int64_t>(kRmsGroup, nblk - g0);
        if (threadIdx.x == 0) {
            int nl = 0;
            for (int g = 0; g < gn; ++g) {
                const int64_t b0 = (g0 + g) * kPwBlock;
                const int bn = (int)std::min<int64_t>(kPwBlock, m - b0);
                bleaf[g] = nl;
                pairwise_tree(bn, [&](int off, int len) {
                    loff[nl] = (int32_t)(b0 - g0 * kPwBlock) + off;
                    llen[nl] = len;
                    ++nl;
                    return 0.0;
                });
            }
            bleaf[gn] = nl;
        }
        __syncthreads();
        const int64_t base = g0 * kPwBlock;
        for (int l = threadIdx.x; l < bleaf[gn]; l += blockDim.x) lsum[l] = pw_leaf(v, base + loff[l], llen[l]);
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int g = 0; g < gn; ++g) {
                const int bn = (int)std::min<int64_t>(kPwBlock, m - (g0 + g) * kPwBlock);
                int li = bleaf[g];
                total += pairwise_tree(bn, [&](int, int) { return lsum[li++]; });
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) *bcast = total;
    __syncthreads();
    const double t = *bcast;
    __syncthreads();
    return t;
}

// rms[r] = nanstd(d) / sqrt(2), d_i = x[1 + i] / s - x[0] / s, i < N - 1, N = n // 2 * 2
// (COMAPData.auto_rms with its tod[:-1:N] slice: COMAPData.py:205-208).  np.nanstd:
// NaN -> 0, avg = sum / count, (d - avg)^2 with NaN -> 0, var = sum / count.
__global__ void __launch_bounds__(kRmsThreads) k_prep_rms(const double *__restrict__ x, int64_t stride,
                                                          const int32_t *__restrict__ rows,
                                                          const double *__restrict__ scale, int64_t n,
                                                          double *__restrict__ rms)
{
#pragma clang fp contract(off)
    __shared__ int32_t loff[kRmsLeafCap], llen[kRmsLeafCap];
    __shared__ double lsum[kRmsLeafCap];
    __shared__ int32_t bleaf[kRmsGroup + 1];
    __shared__ double bc;
    __shared__ unsigned long long cnt_s;
    const int r = blockIdx.x;
    const double *xr = x + (int64_t)rows[r] * stride;
    const double s = scale[r];
    const int64_t m = n / 2 * 2 - 1;
    if (m <= 0) {
        if (threadIdx.x == 0) rms[r] = NAN;
        return;
    }
    const double x0 = xr[0] / s;
    auto d_at = [&](int64_t i) { return xr[1 + i] / s - x0; };
    // count of non-NaN differences (exact integer sum)
    if (threadIdx.x == 0) cnt_s = 0;
    __syncthreads();
    unsigned long long c = 0;
    for (int64_t i = threadIdx.x; i < m; i += blockDim.x) c += !isnan(d_at(i));
    atomicAdd(&cnt_s, c);
    __syncthreads();
    const double cnt = (double)cnt_s;
    const double sum = numpy_sum([&](int64_t i) { const double d = d_at(i); return isnan(d) ? 0.0 : d; }, m, loff,
                                 llen, lsum, bleaf, &bc);
    const double avg = sum / cnt;
    const double sq = numpy_sum([&](int64_t i) {
        const double d = d_at(i);
        if (isnan(d)) return 0.0;
        const double e = d - avg;
        return e * e;
    }, m, loff, llen, lsum, bleaf, &bc);
    if (threadIdx.x == 0) rms[r] = sqrt(sq / cnt) / 1.4142135623730951;   // np.sqrt(2)
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
// a NaN among the values makes the result NaN.  The four order statistics come from
// one block's radix select (8 passes of 8 bits over orderable u64 keys).
constexpr int kPctThreads = 1024;
__global__ void __launch_bounds__(kPctThreads) k_prep_pct(const double *__restrict__ az, const double *__restrict__ el,
                                                          int64_t stride, const int32_t *__restrict__ rows, int64_t n,
                                                          double *__restrict__ pct)
{
#pragma clang fp contract(off)
    __shared__ unsigned int hist[4][256];
    __shared__ unsigned long long pre[4];
    __shared__ long long rk[4];
    __shared__ unsigned long long ngood_s, nnan_s;
    const int r = blockIdx.x >> 1, which = blockIdx.x & 1;
    const double *a = az + (int64_t)rows[r] * stride;
    const double *v = (which ? el : az) + (int64_t)rows[r] * stride;
    if (threadIdx.x == 0) { ngood_s = 0; nnan_s = 0; }
    __syncthreads();
    unsigned long long ng = 0, nn = 0;
    for (int64_t t = threadIdx.x; t < n; t += blockDim.x) {
        if (isfinite(a[t])) { ++ng; nn += isnan(v[t]); }
    }
    atomicAdd(&ngood_s, ng);
    atomicAdd(&nnan_s, nn);
    __syncthreads();
    const int64_t cnt = (int64_t)ngood_s;
    double *out = pct + 4 * (int64_t)r + 2 * which;
    if (cnt == 0 || nnan_s > 0) {
        if (threadIdx.x < 2) out[threadIdx.x] = NAN;
        return;
    }
    const double q[2] = {0.1, 0.9};   // np.true_divide(10, 100), (90, 100)
    double virt[2];
    int64_t lo[2], hi[2];
    for (int k = 0; k < 2; ++k) {
        virt[k] = (double)(cnt - 1) * q[k];
        double prev = floor(virt[k]);
        if (virt[k] >= (double)(cnt - 1)) prev = -1.0;   // _get_indexes: above the last index -> the last value
        if (virt[k] < 0) prev = 0.0;
        lo[k] = prev < 0 ? cnt - 1 : (int64_t)prev;
        hi[k] = prev < 0 ? cnt - 1 : std::min<int64_t>(lo[k] + 1, cnt - 1);
        virt[k] = virt[k] - prev;                        // gamma = virtual - previous index
    }
    if (threadIdx.x < 4) {
        pre[threadIdx.x] = 0;
        rk[threadIdx.x] = threadIdx.x == 0 ? lo[0] : threadIdx.x == 1 ? hi[0] : threadIdx.x == 2 ? lo[1] : hi[1];
    }
    unsigned long long mask = 0;
    for (int pass = 7; pass >= 0; --pass) {
        const int sh = 8 * pass;
        for (int i = threadIdx.x; i < 4 * 256; i += blockDim.x) (&hist[0][0])[i] = 0;
        __syncthreads();
        unsigned long long p4[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) p4[s] = pre[s];
        for (int64_t t = threadIdx.x; t < n; t += blockDim.x) {
            if (!isfinite(a[t])) continue;
            const unsigned long long key = ord_key(v[t]);
            const unsigned dg = (unsigned)(key >> sh) & 255u;
#pragma unroll
            for (int s = 0; s < 4; ++s)
                if ((key & mask) == p4[s]) atomicAdd(&hist[s][dg], 1u);
        }
        __syncthreads();
        if (threadIdx.x < 4) {
            const int s = threadIdx.x;
            long long before = 0;
            int d = 0;
            for (; d < 255; ++d) {
                if (before + hist[s][d] > rk[s]) break;
                before += hist[s][d];
            }
            rk[s] -= before;
            pre[s] |= (unsigned long long)d << sh;
        }
        mask |= 255ull << sh;
        __syncthreads();
    }
    if (threadIdx.x < 2) {
        const int k = threadIdx.x;
        const double av = from_key(pre[2 * k]), bv = from_key(pre[2 * k + 1]), g = virt[k];
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

// One thread per output sample (row, column) of one file (get_tod COMAPData.py:306-376,
// read_pixels :404-425): column -> (scan, sample) through the scan table.
__global__ void __launch_bounds__(256) k_prep_gather(comap_prep_file f, comap_prep_wcs wc, comap_prep_out o)
{
#pragma clang fp contract(off)
    __shared__ int64_t sc[3 * 64];
    for (int i = threadIdx.x; i < 3 * f.n_scans; i += blockDim.x) sc[i] = f.scans[i];
    __syncthreads();
    const int64_t col = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int row = blockIdx.y;
    if (col >= f.datasize) return;
    int s = 0;
    while (s + 1 < f.n_scans && sc[3 * (s + 1) + 2] <= col) ++s;
    const int64_t N = sc[3 * s + 1], j = col - sc[3 * s + 2], t = sc[3 * s] + j;
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
// segment k = x[seg[2k] .. seg[2k] + seg[2k+1]); its median input = the non-zero finite samples
__device__ __forceinline__ bool hp_keep(double v) { return v != 0.0 && isfinite(v); }

__global__ void __launch_bounds__(256) k_seg_count(const double *__restrict__ x, const int64_t *__restrict__ seg,
                                                   int64_t *__restrict__ cnt)
{
    __shared__ unsigned long long c_s;
    const double *p = x + seg[2 * blockIdx.x];
    const int64_t n = seg[2 * blockIdx.x + 1];
    if (threadIdx.x == 0) c_s = 0;
    __syncthreads();
    unsigned long long c = 0;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) c += hp_keep(p[i]);
    atomicAdd(&c_s, c);
    __syncthreads();
    if (threadIdx.x == 0) cnt[blockIdx.x] = (int64_t)c_s;
}

// compacted values (in order) and their positions, one block per segment
__global__ void __launch_bounds__(256) k_seg_compact(const double *__restrict__ x, const int64_t *__restrict__ seg,
                                                     const int64_t *__restrict__ off, double *__restrict__ vals,
                                                     int32_t *__restrict__ pos)
{
    typedef hipcub::BlockScan<int, 256> Scan;
    __shared__ typename Scan::TempStorage ts;
    __shared__ int64_t run;
    const double *p = x + seg[2 * blockIdx.x];
    const int64_t n = seg[2 * blockIdx.x + 1];
    const int64_t o0 = off[blockIdx.x];
    if (threadIdx.x == 0) run = 0;
    __syncthreads();
    for (int64_t b = 0; b < n; b += 256) {
        const int64_t i = b + threadIdx.x;
        const double v = i < n ? p[i] : 0.0;
        const int k = i < n && hp_keep(v);
        int ex = 0, tot = 0;
        Scan(ts).ExclusiveSum(k, ex, tot);
        if (k) {
            vals[o0 + run + ex] = v;
            pos[o0 + run + ex] = (int32_t)i;
        }
        __syncthreads();
        if (threadIdx.x == 0) run += tot;
        __syncthreads();
    }
}

__global__ void k_seg_subtract(double *__restrict__ x, const int64_t *__restrict__ seg, const int64_t *__restrict__ off,
                               const int64_t *__restrict__ cnt, const double *__restrict__ filt,
                               const int32_t *__restrict__ pos)
{
    double *p = x + seg[2 * blockIdx.x];
    const int64_t o0 = off[blockIdx.x], n = cnt[blockIdx.x];
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) p[pos[o0 + i]] -= filt[o0 + i];
}

// ---------------------------------------------------------------- NaN and empty-offset cuts
// per band: tod NaN / inf -> tod = w = 0 (COMAPData.py:550-552); keep[b][o] = any w != 0
// over the offset (:554-557); kept[o] = any band keeps o
__global__ void k_cut_flags(double *__restrict__ tod, double *__restrict__ w, int64_t band_stride, int nb, int64_t NO,
                            int L, uint8_t *__restrict__ keep, int32_t *__restrict__ kept)
{
    for (int64_t o = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; o < NO; o += (int64_t)gridDim.x * blockDim.x) {
        int any_band = 0;
        for (int b = 0; b < nb; ++b) {
            double *tp = tod + b * band_stride + o * L, *wp = w + b * band_stride + o * L;
            int any = 0;
            for (int j = 0; j < L; ++j) {
                if (!isfinite(tp[j])) { tp[j] = 0.0; wp[j] = 0.0; }
                any |= wp[j] != 0.0;
            }
            keep[b * NO + o] = (uint8_t)any;
            any_band |= any;
        }
        kept[o] = any_band;
    }
}

// compaction of the kept offsets (L samples each) of every output array; non-finite
// weights -> 0 after the cut (COMAPData.py:568)
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
    k_prep_rms<<<nrows, kRmsThreads, 0, ctx->stream>>>(x, row_stride, rows, scale, n, rms);
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}

extern "C" int comap_prep_percentiles(comap_ctx *ctx, const double *az, const double *el, int64_t row_stride,
                                      const int32_t *rows, int32_t nrows, int64_t n, double *pct)
{
    if (!ctx || !az || !el || !rows || !pct || nrows < 0 || n < 0) return -1;
    COMAP_DEVICE_GUARD(ctx);
    if (nrows == 0) return 0;
    k_prep_pct<<<2 * nrows, kPctThreads, 0, ctx->stream>>>(az, el, row_stride, rows, n, pct);
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}

extern "C" int comap_prep_gather(comap_ctx *ctx, const comap_prep_file *f, const comap_prep_wcs *wcs,
                                 const comap_prep_out *out)
{
    if (!ctx || !f || !out || (!wcs && !f->pixels)) return -1;
    COMAP_DEVICE_GUARD(ctx);
    if (f->n_scans < 1 || f->n_scans > 64) return comap_fail(ctx, -1, "comap_prep_gather: 1 to 64 scans per file");
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
    DevTemps tmp(st);
    int64_t *cnt = nullptr, *off = nullptr;
    COMAP_CHECK(ctx, tmp.alloc(&cnt, (size_t)nseg));
    COMAP_CHECK(ctx, tmp.alloc(&off, (size_t)nseg));
    k_seg_count<<<nseg, 256, 0, st>>>(x, seg_dev, cnt);
    COMAP_LAUNCH_CHECK(ctx);
    std::vector<int64_t> c(nseg), o(nseg);
    COMAP_CHECK(ctx, hipMemcpyAsync(c.data(), cnt, 8 * (size_t)nseg, hipMemcpyDeviceToHost, st));
    COMAP_CHECK(ctx, hipStreamSynchronize(st));
    int64_t total = 0;
    for (int k = 0; k < nseg; ++k) { o[k] = total; total += c[k]; }
    if (total == 0) return 0;
    double *vals = nullptr, *filt = nullptr;
    int32_t *pos = nullptr;
    COMAP_CHECK(ctx, tmp.alloc(&vals, (size_t)total));
    COMAP_CHECK(ctx, tmp.alloc(&filt, (size_t)total));
    COMAP_CHECK(ctx, tmp.alloc(&pos, (size_t)total));
    COMAP_CHECK(ctx, hipMemcpyAsync(off, o.data(), 8 * (size_t)nseg, hipMemcpyHostToDevice, st));
    k_seg_compact<<<nseg, 256, 0, st>>>(x, seg_dev, off, vals, pos);
    COMAP_LAUNCH_CHECK(ctx);
    std::vector<MedJob> jobs;
    std::vector<int> small;
    for (int k = 0; k < nseg; ++k) {
        if (c[k] == 0) continue;
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
            jobs.push_back(j);
        } else {
            small.push_back(k);
        }
    }
    int rc = 0;
    if (!jobs.empty()) {
        MedPlan mp;
        rc = comap_median_plan(ctx, &mp, jobs, w);
        if (!rc) rc = comap_median_run(ctx, &mp);
        if (!rc) {
            // the plan's buffers are freed below: wait for the walk
            const hipError_t e = hipStreamSynchronize(st);
            if (e != hipSuccess) rc = comap_fail(ctx, -2, hipGetErrorString(e));
        }
        comap_median_plan_free(&mp);
        if (rc) return rc;
    }
    // short segments: np.nanmedian of their (finite) values -- a mean of the two middle
    // values for an even count -- broadcast (np.ones(n) * m)
    for (int k : small) {
        std::vector<double> v(c[k]);
        COMAP_CHECK(ctx, hipMemcpyAsync(v.data(), vals + o[k], 8 * v.size(), hipMemcpyDeviceToHost, st));
        COMAP_CHECK(ctx, hipStreamSynchronize(st));
        std::sort(v.begin(), v.end());
        const size_t n = v.size();
        const double med = n % 2 ? v[n / 2] : (v[n / 2 - 1] + v[n / 2]) / 2.0;
        std::vector<double> f(n, med);
        COMAP_CHECK(ctx, hipMemcpyAsync(filt + o[k], f.data(), 8 * n, hipMemcpyHostToDevice, st));
        COMAP_CHECK(ctx, hipStreamSynchronize(st));
    }
    k_seg_subtract<<<nseg, 256, 0, st>>>(x, seg_dev, off, cnt, filt, pos);
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
    DevTemps tmp(st);
    uint8_t *keep = nullptr;
    int32_t *kept = nullptr, *newo = nullptr;
    COMAP_CHECK(ctx, tmp.alloc(&keep, (size_t)nb * NO));
    COMAP_CHECK(ctx, tmp.alloc(&kept, (size_t)NO + 1));
    COMAP_CHECK(ctx, tmp.alloc(&newo, (size_t)NO + 1));
    k_cut_flags<<<grid_for(NO), 256, 0, st>>>(in->tod, in->w, in->band_stride, nb, NO, L, keep, kept);
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
