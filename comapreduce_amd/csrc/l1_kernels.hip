// l1_kernels.hip -- Level-1 -> Level-2 reduction on MI355X (gfx950).
//
// The reference reduces each (feed, scan) with NumPy/SciPy
// (comancpipeline/Analysis/Level1Averaging.py:792-872).  Here every step is a
// weighted sum of the raw f32 cube d[f][b][c][t] with per-channel f64
// coefficients, so the whole observation is three streaming passes over HBM:
//
//   pass A  k_moments      per channel, over t: sum d, sum A d, and the
//                          stride-4 difference moments (atmosphere fit +
//                          normalise_data rms)                  -> 4 B/samp·ch
//   pass B  k_band_sums    per t, over the listed median channels: the band
//                          mean of y = (d - o - a A)/rms (median input) AND
//                          every per-sample output sum (gain template, residual
//                          and original band sums)              -> 4 B/samp·ch
//           median_kernels.hip: the w = 6000 running median of the band means
//   pass C  k_regress      per channel, over t: sum d mf        -> 4 B/samp·ch
//
// The regression enters the outputs only through per-band constants (k_finish);
// k_gain_avg (the former pass D) runs only when a NaN regression coefficient
// changes a channel weight (k_coef_d phase 1 flags it).
//
// Layout: time is contiguous (the reference's [F][B][C][T]); a wave reads
// 64 lanes x 16 B of one channel row per instruction (coalesced).  Pass A/C
// waves own 4 / 8 channel rows and share the airmass / median loads; pass B
// workgroups own a sub-tile of a 1024-sample tile with one wave per band.  All
// arithmetic is f64 (the reference upcasts to f64 at subtract_fitted_atmosphere).
// Variants measured slower are listed in DESIGN.md §3 (code in git history).
#include "comap_internal.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <utility>

using namespace comap;

#ifndef COMAP_GROUPS
#define COMAP_GROUPS 1      // unit groups of the pass B / median / pass C pipeline (2 measured no faster with the sort-path median)
#endif

typedef float f32x4u __attribute__((ext_vector_type(4), aligned(4)));
// Streaming load of 4 cube samples, non-temporal: data read once never allocates in
// L2, which keeps the airmass / median-filter rows every wave shares resident
// (measured at C2: pass A 9.19 -> 8.82 ms, B 9.55 -> 8.75, C 8.86 -> 7.89).
__device__ __forceinline__ f32x4u ld4(const float *p)
{
    return __builtin_nontemporal_load(reinterpret_cast<const f32x4u *>(p));
}

__device__ __forceinline__ double wave_sum(double v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Block-wide sum for 256-thread blocks (4 waves); every thread gets the total.
__device__ __forceinline__ double block_sum256(double v, double *lds4)
{
    v = wave_sum(v);
    const int wid = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) lds4[wid] = v;
    __syncthreads();
    double t = lds4[0] + lds4[1] + lds4[2] + lds4[3];
    return t;
}

__device__ __forceinline__ bool atmos_channel(int c)
{   // fit_atmosphere channel set: arange(10,1014) minus 510..514 (Level1Averaging.py:201-202)
    return c >= 10 && c < 1014 && !(c >= 510 && c < 515);
}

__device__ __forceinline__ bool median_channel(int c)
{   // median_filter index: 10..1013 minus 507..517 (Level1Averaging.py:688-690)
    return c >= 10 && c < 1014 && !(c >= 507 && c <= 517);
}

__device__ __forceinline__ bool gain_masked(int c)
{   // gain_subtraction_fit: [:20], [-20:], 512-5:512+5 (GainSubtraction.py:190-196)
    return c < 20 || c >= 1004 || (c >= 507 && c < 517);
}

// ------------------------------------------------------------------ channel-list compaction
// Wave 0 of a block writes, in ascending order, the channels c with live(c)
// into list[0..cnt) and emit(j, c) for each, then pads list to a multiple of 8
// with channel 0 / pad(j) (weight-0 entries the streaming passes never let
// contribute).  Lane l scans channels 16l..16l+15.  Returns cnt on every lane.
template <typename Live, typename Emit, typename Pad>
__device__ __forceinline__ int wave_compact_channels(int lane, Live live, Emit emit, Pad pad, int32_t *list)
{
    const int c0 = lane * 16;
    uint32_t bits = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) bits |= (live(c0 + i) ? 1u : 0u) << i;
    const int m = __popc(bits);
    int incl = m;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    int pos = incl - m;
    for (int i = 0; i < 16; ++i)
        if ((bits >> i) & 1u) { list[pos] = c0 + i; emit(pos, c0 + i); ++pos; }
    const int cnt = __shfl(incl, 63, 64);
    const int j = cnt + lane;
    if (lane < 8 && j < ((cnt + 7) & ~7)) { list[j] = 0; pad(j); }
    return cnt;
}

// ------------------------------------------------------------------ airmass
// COMAPLevel1.airmass: 1/sin(el*pi/180) (DataHandling.py:398-401)
__global__ void k_airmass(const double *__restrict__ el, double *__restrict__ A, int64_t n)
{
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        A[i] = 1.0 / sin(el[i] * M_PI / 180.0);
}

// ------------------------------------------------------------------ per-unit airmass sums
// us[u] = {n, sum A, sum A^2, sum v, sum v^2, N4}, v_k = A[4k] - A[4k+2]
__global__ void __launch_bounds__(256) k_unit_sums(const int32_t *__restrict__ units,
                                                   const double *__restrict__ A, int64_t T,
                                                   double *__restrict__ us)
{
    __shared__ double red[4];
    const int u = blockIdx.x;
    const int f = units[4 * u], t0 = units[4 * u + 2], n = units[4 * u + 3];
    const double *a = A + (int64_t)f * T + t0;
    double sa = 0, saa = 0, sv = 0, svv = 0;
    for (int t = threadIdx.x; t < n; t += blockDim.x) {
        double x = a[t];
        sa += x;
        saa += x * x;
    }
    const int n4 = n / 4;
    for (int k = threadIdx.x; k < n4; k += blockDim.x) {
        double v = a[4 * k] - a[4 * k + 2];
        sv += v;
        svv += v * v;
    }
    sa = block_sum256(sa, red);
    saa = block_sum256(saa, red);
    sv = block_sum256(sv, red);
    svv = block_sum256(svv, red);
    if (threadIdx.x == 0) {
        double *o = us + 8 * (int64_t)u;
        o[0] = n; o[1] = sa; o[2] = saa; o[3] = sv; o[4] = svv; o[5] = n4;
    }
}

// ------------------------------------------------------------------ pass A
// Per (unit, band, channel): Sd = sum d, SAd = sum A d over the scan, and over
// the stride-4 pairs u_k = d[4k]-d[4k+2]: Su, Suu, Suv (v_k = A[4k]-A[4k+2]).
// normalise_data's rms for ANY atmosphere slope a follows in closed form:
//   diff_k = u_k - a v_k  (the offset cancels).
// Wave shape and load depth by measurement at C2 (where the rejected
// variants -- aligned loads with lane shifts, other wave shapes, forced occupancy --
// are listed): 4 channel rows per wave (8: 9.28 -> 10.13 ms), 4 sample groups per
// lane per trip with every row load issued before any is accumulated (1: 9.39 ms,
// 2: 9.15, 4: 8.82, 8: 9.08), the trip's airmass staged once per block in LDS
// (8.86 -> 8.65 ms).
constexpr int kCPW = 4;    // channel rows per wave
constexpr int kAUnr = 4;   // sample groups per lane per trip (loads in flight = kAUnr x kCPW)
__global__ void __launch_bounds__(256) k_moments(const float *__restrict__ tod, const double *__restrict__ A,
                                                 const int32_t *__restrict__ units, int64_t T,
                                                 double *__restrict__ mom, int64_t UC, int32_t *nan_count,
                                                 int32_t *__restrict__ rowbad)
{
    const int wid = uniform(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int groups_per_band = kChannels / (4 * kCPW);
    int bid = blockIdx.x;
    const int g = bid % groups_per_band; bid /= groups_per_band;
    const int b = bid % kBands;
    const int u = bid / kBands;
    const int f = units[4 * u], t0 = units[4 * u + 2], n = units[4 * u + 3];
    const int c0 = g * 4 * kCPW + wid * kCPW;
    const float *row0 = tod + ((int64_t)(f * kBands + b) * kChannels + c0) * T + t0;
    const double *a = A + (int64_t)f * T + t0;

    double sd[kCPW], sad[kCPW], su[kCPW], suu[kCPW], suv[kCPW];
    int bad[kCPW];
#pragma unroll
    for (int r = 0; r < kCPW; ++r) { sd[r] = sad[r] = su[r] = suu[r] = suv[r] = 0.0; bad[r] = 0; }
    const int n4 = n >> 2;
    auto group = [&](int k) {
        const double a0 = a[4 * k], a1 = a[4 * k + 1], a2 = a[4 * k + 2], a3 = a[4 * k + 3];
        const double v = a0 - a2;
#pragma unroll
        for (int r = 0; r < kCPW; ++r) {
            const f32x4u x = ld4(row0 + (int64_t)r * T + 4 * k);
            const double x0 = x.x, x1 = x.y, x2 = x.z, x3 = x.w;
            bad[r] += !isfinite(x.x) + !isfinite(x.y) + !isfinite(x.z) + !isfinite(x.w);
            sd[r] += (x0 + x1) + (x2 + x3);
            sad[r] = fma(a0, x0, sad[r]);
            sad[r] = fma(a1, x1, sad[r]);
            sad[r] = fma(a2, x2, sad[r]);
            sad[r] = fma(a3, x3, sad[r]);
            const double uu = x0 - x2;
            su[r] += uu;
            suu[r] = fma(uu, uu, suu[r]);
            suv[r] = fma(uu, v, suv[r]);
        }
    };
    // groups of 4 stay on the scan's stride-4 pairs (normalise_data); the scans' rows
    // start anywhere in a 16-B chunk, so the loads are unaligned
    int k = lane;
    // the block's 4 waves walk the same samples of 16 rows: each trip's airmass groups are
    // read from L2 once per block into LDS (double-buffered, one barrier per trip) instead
    // of once per wave.  Trips are block-uniform (whole trips only; the rest below).
    static_assert(kAUnr * 64 == 256, "one airmass group of 4 samples per thread");
    __shared__ double4 air[2][kAUnr * 64];
    {
        int par = 0;
        for (int kb = 0; kb + 64 * kAUnr <= n4; kb += 64 * kAUnr, par ^= 1) {
            f32x4u xs[kAUnr][kCPW];
#pragma unroll
            for (int j = 0; j < kAUnr; ++j)
#pragma unroll
                for (int r = 0; r < kCPW; ++r) xs[j][r] = ld4(row0 + (int64_t)r * T + 4 * (kb + 64 * j + lane));
            {
                const double *q = a + 4 * (kb + (int)threadIdx.x);
                air[par][threadIdx.x] = make_double4(q[0], q[1], q[2], q[3]);
            }
            __syncthreads();
#pragma unroll
            for (int j = 0; j < kAUnr; ++j) {
                const double4 av = air[par][64 * j + lane];
                const double a0 = av.x, a1 = av.y, a2 = av.z, a3 = av.w;
                const double v = a0 - a2;
#pragma unroll
                for (int r = 0; r < kCPW; ++r) {
                    const f32x4u x = xs[j][r];
                    const double x0 = x.x, x1 = x.y, x2 = x.z, x3 = x.w;
                    bad[r] += !isfinite(x.x) + !isfinite(x.y) + !isfinite(x.z) + !isfinite(x.w);
                    sd[r] += (x0 + x1) + (x2 + x3);
                    sad[r] = fma(a0, x0, sad[r]);
                    sad[r] = fma(a1, x1, sad[r]);
                    sad[r] = fma(a2, x2, sad[r]);
                    sad[r] = fma(a3, x3, sad[r]);
                    const double uu = x0 - x2;
                    su[r] += uu;
                    suu[r] = fma(uu, uu, suu[r]);
                    suv[r] = fma(uu, v, suv[r]);
                }
            }
            k = kb + 64 * kAUnr + lane;
        }
    }
    for (; k < n4; k += 64) group(k);
    // tail samples n4*4 .. n-1 (at most 3)
    const int tt = 4 * n4 + lane;
    if (lane < 4 && tt < n) {
        const double at = a[tt];
#pragma unroll
        for (int r = 0; r < kCPW; ++r) {
            const float xf = row0[(int64_t)r * T + tt];
            bad[r] += !isfinite(xf);
            sd[r] += (double)xf;
            sad[r] = fma(at, (double)xf, sad[r]);
        }
    }
    int tot = 0;
#pragma unroll
    for (int r = 0; r < kCPW; ++r) {
        const double s0 = wave_sum(sd[r]), s1 = wave_sum(sad[r]), s2 = wave_sum(su[r]);
        const double s3 = wave_sum(suu[r]), s4 = wave_sum(suv[r]);
        const int nb = (int)wave_sum((double)bad[r]);
        tot += nb;
        if (lane == 0) {
            const int64_t idx = (int64_t)u * kBC + b * kChannels + c0 + r;
            mom[idx] = s0;
            mom[UC + idx] = s1;
            mom[2 * UC + idx] = s2;
            mom[3 * UC + idx] = s3;
            mom[4 * UC + idx] = s4;
            rowbad[idx] = nb;
        }
    }
    if (lane == 0 && tot) atomicAdd(nan_count, tot);
}

// ------------------------------------------------------------------ NaN path: select_time + masked fit sums
// fit_atmosphere (Level1Averaging.py:204-213) fits only the samples where all
// 994 fitted channels of the band are finite.  One workgroup per
// (unit, band, 1024-sample tile) marks valid[t]; a second kernel recomputes
// the fit sums of that (unit, band) over the valid samples.
// The pairs: list[0 .. *count) of pair ids (grid-strided over blockIdx.y).
__global__ void __launch_bounds__(256) k_select_time(const float *__restrict__ tod, const int32_t *__restrict__ units,
                                                     const int32_t *__restrict__ pairs, int64_t T,
                                                     const int64_t *__restrict__ voff, uint8_t *__restrict__ valid,
                                                     const int32_t *__restrict__ list,
                                                     const int32_t *__restrict__ count)
{
    const int np = *count;
    for (int li = blockIdx.y; li < np; li += gridDim.y) {
        const int pr = list[li];
        const int u = pairs[2 * pr], b = pairs[2 * pr + 1];
        const int f = units[4 * u], t0 = units[4 * u + 2], n = units[4 * u + 3];
        const int t = blockIdx.x * blockDim.x + threadIdx.x;
        if (t >= n) continue;
        const float *p = tod + (int64_t)(f * kBands + b) * kChannels * T + t0 + t;
        bool ok = true;
        for (int c = 10; c < 1014; ++c)
            if (atmos_channel(c) && !isfinite(p[(int64_t)c * T])) ok = false;
        valid[voff[pr] + t] = ok;
    }
}

// per (pair, channel): Sd, SAd over valid t -> fs[0/1][u*4096+b*1024+c];
// per pair: n, SA, SAA -> ub[(u*4+b)*4 + {0,1,2}]
__global__ void __launch_bounds__(256) k_masked_fit_sums(const float *__restrict__ tod, const double *__restrict__ A,
                                                         const int32_t *__restrict__ units,
                                                         const int32_t *__restrict__ pairs, int64_t T,
                                                         const int64_t *__restrict__ voff,
                                                         const uint8_t *__restrict__ valid, int64_t UC,
                                                         double *__restrict__ fs, double *__restrict__ ub,
                                                         const int32_t *__restrict__ list,
                                                         const int32_t *__restrict__ count)
{
    const int np = *count;
    for (int li = blockIdx.y; li < np; li += gridDim.y) {
    const int pr = list[li];
    const int u = pairs[2 * pr], b = pairs[2 * pr + 1];
    const int f = units[4 * u], t0 = units[4 * u + 2], n = units[4 * u + 3];
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int c = blockIdx.x * 4 + wid;            // one wave per channel
    const float *p = tod + ((int64_t)(f * kBands + b) * kChannels + c) * T + t0;
    const double *a = A + (int64_t)f * T + t0;
    const uint8_t *v = valid + voff[pr];
    double s0 = 0, s1 = 0, cn = 0, sa = 0, saa = 0;
    for (int t = lane; t < n; t += 64) {
        if (!v[t]) continue;
        const double x = p[t], at = a[t];
        s0 += x;
        s1 = fma(at, x, s1);
        cn += 1.0;
        sa += at;
        saa = fma(at, at, saa);
    }
    s0 = wave_sum(s0); s1 = wave_sum(s1);
    cn = wave_sum(cn); sa = wave_sum(sa); saa = wave_sum(saa);
    if (lane == 0) {
        const int64_t i = (int64_t)u * kBC + b * kChannels + c;
        fs[i] = s0;
        fs[UC + i] = s1;
        if (c == 0) {
            double *o = ub + 4 * ((int64_t)u * kBands + b);
            o[0] = cn; o[1] = sa; o[2] = saa;
        }
    }
    }   // listed pairs
}

// flag[u*4+b]: pass A found a non-finite sample in one of the band's fitted channels (the
// (unit, band) pairs whose fit select_time restricts); one wave per pair
__global__ void __launch_bounds__(256) k_pair_flags(const int32_t *__restrict__ rowbad, int npairs,
                                                    int32_t *__restrict__ flag)
{
    const int lane = threadIdx.x & 63;
    const int pr = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (pr >= npairs) return;
    const int u = pr / kBands, b = pr % kBands;
    const int32_t *rb = rowbad + (int64_t)u * kBC + b * kChannels;
    bool any = false;
    for (int c = lane; c < kChannels; c += 64) any |= atmos_channel(c) && rb[c] > 0;
    any = __ballot(any) != 0ull;
    if (lane == 0) flag[pr] = any ? 1 : 0;
}

// the flagged pairs in order (one wave): list[0 .. count)
__global__ void k_pair_list(const int32_t *__restrict__ flag, int npairs, int32_t *__restrict__ list,
                            int32_t *__restrict__ count)
{
    const int lane = threadIdx.x & 63;
    int base = 0;
    for (int i0 = 0; i0 < npairs; i0 += 64) {
        const int i = i0 + lane;
        const bool f = i < npairs && flag[i];
        const unsigned long long m = __ballot(f);
        if (f) list[base + __popcll(m & ((1ull << lane) - 1ull))] = i;
        base += __popcll(m);
    }
    if (lane == 0) *count = base;
}

// ub[(u*4+b)] = unit airmass sums (NaN-free case: every sample is fitted)
__global__ void k_ub_from_units(const double *__restrict__ us, int U, double *__restrict__ ub)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= U * kBands) return;
    const double *q = us + 8 * (int64_t)(i / kBands);
    ub[4 * (int64_t)i] = q[0];
    ub[4 * (int64_t)i + 1] = q[1];
    ub[4 * (int64_t)i + 2] = q[2];
}

// fill_bad_data (Level1Averaging.py:658-665): NaN -> the row's nanmedian (f32).  The
// reference fills its per-feed copy (DataHandling.py:176-177 hands every stage a fresh
// h5py read); here the resident cube is filled for the duration of comap_l1_average
// and every overwritten position is recorded, so k_restore_nan puts the NaNs back.
__global__ void __launch_bounds__(256) k_fill_rows(float *__restrict__ tod, const int64_t *__restrict__ rows,
                                                   const float *__restrict__ med, int nrows, int64_t *__restrict__ pos,
                                                   int64_t cap, int64_t *__restrict__ npos)
{
    const int r = blockIdx.y;
    if (r >= nrows) return;
    const int64_t off = rows[2 * r];
    float *p = tod + off;
    const int64_t n = rows[2 * r + 1];
    const float m = med[r];
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        if (isnan(p[i])) {
            const unsigned long long k = atomicAdd(reinterpret_cast<unsigned long long *>(npos), 1ull);
            if ((int64_t)k < cap) {   // cap = the non-finite count of pass A >= NaN count
                pos[k] = off + i;
                p[i] = m;
            }
        }
}

__global__ void k_restore_nan(float *__restrict__ tod, const int64_t *__restrict__ pos, const int64_t *__restrict__ npos,
                              int64_t cap)
{
    const int64_t n = min(*npos, cap);
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        tod[pos[i]] = __int_as_float(0x7fc00000);
}

// constant-elevation scans (Level1Averaging.py:242-244): fit = (nanmedian, 0) for every channel
__global__ void k_fit_from_median(const int32_t *__restrict__ units, const int32_t *__restrict__ ulist, int nu,
                                  const float *__restrict__ med, int F, double *__restrict__ fit)
{
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= (int64_t)nu * kBC) return;
    const int k = (int)(i / kBC), bc = (int)(i % kBC);
    const int u = ulist[k];
    const int f = units[4 * u], s = units[4 * u + 1];
    const int b = bc / kChannels, c = bc % kChannels;
    double *o = fit + (((int64_t)s * F + f) * kBands + b) * 2 * kChannels;
    o[c] = (double)med[i];
    o[kChannels + c] = 0.0;
}

// ------------------------------------------------------------------ atmosphere fit
// AtmosphereRemoval.fit_atmosphere (Level1Averaging.py:197-227): the
// block-diagonal spsolve is an independent 2x2 normal-equation solve per
// channel: [[n, SA],[SA, SAA]] [o, a]^T = [Sd, SAd]^T.
// fs_sel / sel (select_time): the (unit, band) pairs flagged in sel read their sums from fs_sel
__global__ void k_atmos_fit(const int32_t *__restrict__ units, const double *__restrict__ ubs,
                            const double *__restrict__ fs, int64_t UC, int F, int U,
                            double *__restrict__ fit, const double *__restrict__ fs_sel = nullptr,
                            const int32_t *__restrict__ sel = nullptr)
{
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= (int64_t)U * kBC) return;
    const int u = (int)(i / kBC);
    const int bc = (int)(i % kBC);
    const int b = bc / kChannels, c = bc % kChannels;
    const int f = units[4 * u], s = units[4 * u + 1];
    const double *q = ubs + 4 * ((int64_t)u * kBands + b);
    const double n = q[0], sa = q[1], saa = q[2];
    double o = NAN, a = NAN;
    if (atmos_channel(c) && n >= 100.0) {    // MINIMUM_CHUNK_SIZE (Level1Averaging.py:207-208)
        const double *src = (sel && sel[(int64_t)u * kBands + b]) ? fs_sel : fs;
        const double sd = src[i], sad = src[UC + i];
        const double det = n * saa - sa * sa;
        o = (saa * sd - sa * sad) / det;
        a = (n * sad - sa * sd) / det;
    }
    double *out = fit + (((int64_t)s * F + f) * kBands + b) * 2 * kChannels;
    out[c] = o;
    out[kChannels + c] = a;
}

// ------------------------------------------------------------------ L1AGC coefficients I
// normalise_data (Level1Averaging.py:667-679): rms from the pass-A moments for
// the fit slope a; pass-B coefficients alpha_c = 1/rms on the median
// channels; per (unit, band): beta = sum alpha o, gamma = sum alpha a, N.
// Also gathers the (unit, channel) offsets / slopes L1AGC subtracts (k_gather_oa's job:
// the unit's scan fit, or (nanmedian, 0) for calibrators) into oa for k_coef_d, and
// block 0 clears the pass-D mismatch flag -- two launches fewer per step.
__global__ void __launch_bounds__(256) k_coef_b(const int32_t *__restrict__ units, const double *__restrict__ us,
                                                const double *__restrict__ mom, int64_t UC,
                                                const double *__restrict__ fit, int F, const float *__restrict__ med,
                                                double *__restrict__ oa,
                                                double *__restrict__ alpha, double *__restrict__ nf,
                                                double *__restrict__ bsum, int32_t *__restrict__ flag)
{
    __shared__ double red[4];
    const int ub = blockIdx.x;
    const int u = ub / kBands, b = ub % kBands;
    const int n = units[4 * u + 3];
    if (ub == 0 && threadIdx.x == 0) *flag = 0;
    const int fu = units[4 * u], su = units[4 * u + 1];
    const double *fo = fit + (((int64_t)su * F + fu) * kBands + b) * 2 * kChannels;
    const double *q = us + 8 * (int64_t)u;
    const double sv = q[3], svv = q[4], n4 = q[5];
    double beta = 0, gamma = 0, cnt = 0;
    for (int c = threadIdx.x; c < kChannels; c += blockDim.x) {
        const int64_t i = (int64_t)u * kBC + b * kChannels + c;
        const double o = med ? (double)med[i] : fo[c], a = med ? 0.0 : fo[kChannels + c];
        oa[2 * i] = o;
        oa[2 * i + 1] = a;
        double rms = NAN;
        if (n4 > 0 && isfinite(o) && isfinite(a)) {
            const double su = mom[2 * UC + i], suu = mom[3 * UC + i], suv = mom[4 * UC + i];
            const double mean = (su - a * sv) / n4;
            double var = (suu - 2.0 * a * suv + a * a * svv) / n4 - mean * mean;
            var = var < 0.0 ? 0.0 : var;
            rms = sqrt(var) / sqrt(2.0) * sqrt(kDnuTau);
        }
        nf[i] = rms;
        double al = 0.0;
        if (median_channel(c)) {
            al = 1.0 / rms;
            if (isfinite(al) && isfinite(o) && isfinite(a)) {
                beta += al * o;
                gamma += al * a;
                cnt += 1.0;
            } else {
                al = 0.0;
            }
        }
        alpha[i] = al;
    }
    beta = block_sum256(beta, red);
    gamma = block_sum256(gamma, red);
    cnt = block_sum256(cnt, red);
    if (threadIdx.x == 0) {
        double *o = bsum + 4 * (int64_t)ub;
        o[0] = beta; o[1] = gamma; o[2] = cnt;
        // median_filter skips the band when fewer than 2w finite band-mean samples
        o[3] = (cnt > 0 && n >= 2 * kMedfiltWindow) ? 1.0 : 0.0;
    }
}

// ------------------------------------------------------------------ pass B
// One read of the cube BEFORE the median serves every per-sample channel sum
// of the reduction (Level1Averaging.py:691-692, 841-867; GainSubtraction.py:201):
//   m_t   = (sum_c alpha_c d_ct - beta - gamma A_t) / N      band mean -> median
//   Sg_t  = sum_b sum_c kg_c d_ct                             gain template (dG)
//   Sr_bt = sum_c kr_c d_ct,  So_bt = sum_c ko_c d_ct         residual / original band sums
// The kappa weights (k_coef_d phase 0) depend on the regression only through
// a NaN coefficient, which phase 1 detects (then the legacy pass D runs), so
// they are known here; the regression enters later only through per-band
// constants (k_finish).  The wave walks its (unit, band)'s channel list
// (k_coef_d phase 0: the median channels with alpha != 0, a superset of the
// kappa channels) four entries at a time, 4 x kJB 16-B loads in flight.

// x[4g+e] = d[r0 + 256 g + e] (0 beyond the scan end, nv0 = n - r0)
constexpr int kJ = kTile / 256;
template <int J = kJ>
__device__ __forceinline__ void load_groups(const float *__restrict__ p, int nv0, double (&x)[4 * J])
{
#pragma unroll
    for (int g = 0; g < J; ++g) {
        const int nv = nv0 - 256 * g;
        if (nv >= 4) {
            const f32x4u v = *reinterpret_cast<const f32x4u *>(p + 256 * g);
            x[4 * g] = v.x; x[4 * g + 1] = v.y; x[4 * g + 2] = v.z; x[4 * g + 3] = v.w;
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) x[4 * g + e] = (e < nv) ? (double)p[256 * g + e] : 0.0;
        }
    }
}

// Raw f32 groups of one channel row: r[g] = d[r0 + 256 g .. +3] (zeros beyond
// the scan end; FULL = the whole sub-tile lies inside the scan, no checks).
template <int J, bool FULL>
__device__ __forceinline__ void load_raw(const float *__restrict__ p, int nv0, f32x4u (&r)[J])
{
#pragma unroll
    for (int g = 0; g < J; ++g) {
        const int nv = nv0 - 256 * g;
        if (FULL || nv >= 4) {
            r[g] = ld4(p + 256 * g);
        } else {
            f32x4u v = {0.f, 0.f, 0.f, 0.f};
            if (nv > 0) v.x = p[256 * g];
            if (nv > 1) v.y = p[256 * g + 1];
            if (nv > 2) v.z = p[256 * g + 2];
            r[g] = v;
        }
    }
}

// 4 groups x 4 samples per lane: a wave reads 4 KB of a channel row per load
// pair (measured: 1 KB 10.6 ms, 2 KB 9.9 ms, 4 KB 9.45 ms at C2)
constexpr int kJB = 4;                     // groups of 4 samples per lane
constexpr int kBB = 2;                     // channel-list entries per load batch (4: 8.76 -> 8.98 ms at C2)
constexpr int kSubB = kTile / (256 * kJB); // pass-B blocks per 1024-sample tile

struct BandAcc {
    double m[4 * kJB], g[4 * kJB], r[4 * kJB], o[4 * kJB];
};

__device__ __forceinline__ void band_fma(BandAcc &a, const double *__restrict__ w, const f32x4u (&r)[kJB])
{
    const double wa = w[0], wg = w[1], wr = w[2], wo = w[3];
#pragma unroll
    for (int g = 0; g < kJB; ++g)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int i = 4 * g + e;
            const double x = (double)r[g][e];
            a.m[i] = fma(wa, x, a.m[i]);
            a.g[i] = fma(wg, x, a.g[i]);
            a.r[i] = fma(wr, x, a.r[i]);
            a.o[i] = fma(wo, x, a.o[i]);
        }
}

template <bool FULL>
__device__ __forceinline__ void band_sums(const float *__restrict__ base, int64_t T, int nv0,
                                          const int32_t *__restrict__ lst, const double *__restrict__ wl, int cnt,
                                          BandAcc &a)
{
    int j = 0;
    for (; j + kBB <= cnt; j += kBB) {
        f32x4u r[kBB][kJB];
#pragma unroll
        for (int q = 0; q < kBB; ++q) load_raw<kJB, FULL>(base + (int64_t)lst[j + q] * T, nv0, r[q]);
#pragma unroll
        for (int q = 0; q < kBB; ++q) band_fma(a, wl + 4 * (j + q), r[q]);
    }
    for (; j < cnt; ++j) {
        f32x4u r[kJB];
        load_raw<kJB, FULL>(base + (int64_t)lst[j] * T, nv0, r);
        band_fma(a, wl + 4 * j, r);
    }
}

// Block = 4 waves (wave b = band b) on a 256 kJB-sample sub-tile of a 1024-sample tile.
__global__ void __launch_bounds__(256) k_band_sums(const float *__restrict__ tod, const double *__restrict__ A,
                                                   const int32_t *__restrict__ units, const int32_t *__restrict__ tiles,
                                                   int64_t tile0, int64_t T, const int32_t *__restrict__ dlist,
                                                   const int32_t *__restrict__ dcnt, const double *__restrict__ dw,
                                                   const double *__restrict__ bsum, double *__restrict__ mb,
                                                   double *__restrict__ sr_out, double *__restrict__ so_out,
                                                   double *__restrict__ sg_out)
{
    __shared__ double sg[kBands][256 * kJB];
    const int b = uniform(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int tile = (int)(tile0 + blockIdx.x / kSubB), sub = blockIdx.x % kSubB;
    const int u = tiles[2 * tile], toff = tiles[2 * tile + 1] + 256 * kJB * sub;
    const int f = units[4 * u], t0 = units[4 * u + 2], n = units[4 * u + 3];
    if (toff >= n) return;                          // whole block: past the scan end
    const int r0 = toff + 4 * lane;                 // first sample (relative) of this lane
    const int nv0 = n - r0;
    const float *base = tod + (int64_t)(f * kBands + b) * kChannels * T + t0 + r0;
    const int ub = u * kBands + b;
    BandAcc acc;
#pragma unroll
    for (int i = 0; i < 4 * kJB; ++i) acc.m[i] = acc.g[i] = acc.r[i] = acc.o[i] = 0.0;
    const int32_t *lst = dlist + (int64_t)ub * kChannels;
    const double *wl = dw + 4 * (int64_t)ub * kChannels;
    if (n - toff >= 256 * kJB) band_sums<true>(base, T, nv0, lst, wl, dcnt[ub], acc);
    else band_sums<false>(base, T, nv0, lst, wl, dcnt[ub], acc);
#pragma unroll
    for (int g = 0; g < kJB; ++g)
#pragma unroll
        for (int e = 0; e < 4; ++e) sg[b][256 * g + 4 * lane + e] = acc.g[4 * g + e];
    __syncthreads();
    const double *bs = bsum + 4 * (int64_t)ub;
    const double beta = bs[0], gamma = bs[1], cn = bs[2];
    const int64_t rowo = (int64_t)(f * kBands + b) * T + t0 + r0;
    const double *a = A + (int64_t)f * T + t0 + r0;
#pragma unroll
    for (int g = 0; g < kJB; ++g)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int i = 4 * g + e, o = 256 * g + e;
            if (o >= nv0 || r0 + o < 0) continue;   // before the scan: aligned-tile lead-in
            mb[rowo + o] = cn > 0 ? (acc.m[i] - beta - gamma * a[o]) / cn : NAN;
            sr_out[rowo + o] = acc.r[i];
            so_out[rowo + o] = acc.o[i];
            if (b == 0) {
                const int tl = 256 * g + 4 * lane + e;
                sg_out[(int64_t)f * T + t0 + r0 + o] = (sg[0][tl] + sg[1][tl]) + (sg[2][tl] + sg[3][tl]);
            }
        }
}

// ------------------------------------------------------------------ series sums for pass C
// ss[ub] = {sum mf, sum mf^2, sum A mf}; zeroes mf of skipped bands.
__global__ void __launch_bounds__(256) k_series_sums(int ub0, const int32_t *__restrict__ units, const double *__restrict__ A,
                                                     int64_t T, const double *__restrict__ bsum,
                                                     double *__restrict__ mf, double *__restrict__ ss)
{
    __shared__ double red[4];
    const int ub = ub0 + blockIdx.x;
    const int u = ub / kBands, b = ub % kBands;
    const int f = units[4 * u], t0 = units[4 * u + 2], n = units[4 * u + 3];
    const bool run = bsum[4 * (int64_t)ub + 3] > 0;
    double *m = mf + (int64_t)(f * kBands + b) * T + t0;
    const double *a = A + (int64_t)f * T + t0;
    double s0 = 0, s1 = 0, s2 = 0;
    for (int t = threadIdx.x; t < n; t += blockDim.x) {
        if (!run) { m[t] = 0.0; continue; }
        const double x = m[t];
        s0 += x;
        s1 = fma(x, x, s1);
        s2 = fma(a[t], x, s2);
    }
    s0 = block_sum256(s0, red);
    s1 = block_sum256(s1, red);
    s2 = block_sum256(s2, red);
    if (threadIdx.x == 0) {
        double *o = ss + 4 * (int64_t)ub;
        o[0] = s0; o[1] = s1; o[2] = s2;
    }
}

// ------------------------------------------------------------------ pass C
// Regression of each median channel on [1, mf] (Level1Averaging.py:701-705):
// only sum_t d mf is new (sum d came from pass A).  Row streaming like pass
// A: a wave owns kRPW entries of the (unit, band)'s channel list and walks
// the scan 4 samples per lane, sharing the mf loads between its rows.  Bands
// the median filter skipped need no regression and are not read.
// (measured at C2 and rejected: 4 or 16 rows per wave, 2-4 sample groups per trip,
// the median-filter groups staged through LDS -- DESIGN §3)
constexpr int kRPW = 8;
constexpr int kRegBlocks = kChannels / (4 * kRPW);   // blocks per (unit, band)
__global__ void __launch_bounds__(256) k_regress(int ub0, const float *__restrict__ tod, const double *__restrict__ mf,
                                                 const int32_t *__restrict__ units, int64_t T,
                                                 const double *__restrict__ bsum, const int32_t *__restrict__ dlist,
                                                 const int32_t *__restrict__ dcnt, double *__restrict__ sdm)
{
    const int wid = uniform(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int ub = ub0 + blockIdx.x / kRegBlocks, g = blockIdx.x % kRegBlocks;
    const int u = ub / kBands, b = ub % kBands;
    const int cnt = dcnt[ub];
    const int j0 = g * 4 * kRPW + wid * kRPW;
    if (bsum[4 * (int64_t)ub + 3] <= 0) return;      // band skipped by median_filter (block-uniform)
    if (j0 >= cnt) return;
    const int f = units[4 * u], t0 = units[4 * u + 2], n = units[4 * u + 3];
    const int32_t *lst = dlist + (int64_t)ub * kChannels;
    const float *band = tod + (int64_t)(f * kBands + b) * kChannels * T + t0;
    const float *row[kRPW];
#pragma unroll
    for (int r = 0; r < kRPW; ++r) row[r] = band + (int64_t)lst[j0 + r < cnt ? j0 + r : j0] * T;   // pad: re-read
    const double *m = mf + (int64_t)(f * kBands + b) * T + t0;
    double acc[kRPW];
#pragma unroll
    for (int r = 0; r < kRPW; ++r) acc[r] = 0.0;
    // peel the samples before the first 128-B boundary of the list's first row (every row
    // of the band shares it when T is a multiple of 32), so each wave load covers 8 whole
    // lines; block-uniform in any case
    const int head = (int)min((int64_t)n, (-(int64_t)(band + (int64_t)lst[0] * T - tod)) & 31);
    if (lane < head) {
#pragma unroll
        for (int r = 0; r < kRPW; ++r) acc[r] = fma(m[lane], (double)row[r][lane], acc[r]);
    }
#pragma unroll
    for (int r = 0; r < kRPW; ++r) row[r] += head;
    m += head;
    const int nb = n - head;
    const int n4 = nb >> 2;
    int k = lane;
    for (; k < n4; k += 64) {
        const double m0 = m[4 * k], m1 = m[4 * k + 1], m2 = m[4 * k + 2], m3 = m[4 * k + 3];
#pragma unroll
        for (int r = 0; r < kRPW; ++r) {
            const f32x4u x = ld4(row[r] + 4 * k);
            double s = acc[r];
            s = fma(m0, (double)x.x, s);
            s = fma(m1, (double)x.y, s);
            s = fma(m2, (double)x.z, s);
            s = fma(m3, (double)x.w, s);
            acc[r] = s;
        }
    }
    const int tt = 4 * n4 + lane;
    if (lane < 4 && tt < nb) {
#pragma unroll
        for (int r = 0; r < kRPW; ++r) acc[r] = fma(m[tt], (double)row[r][tt], acc[r]);
    }
    double *out = sdm + (int64_t)u * kBC + b * kChannels;
#pragma unroll
    for (int r = 0; r < kRPW; ++r) {
        const double s = wave_sum(acc[r]);
        if (lane == 0 && j0 + r < cnt) out[lst[j0 + r]] = s;
    }
}

// ------------------------------------------------------------------ gain template weights
// gain_subtraction_fit + AMatrix + cg (GainSubtraction.py:17-209) in closed
// form: A = P^T Z P = c I, so dG_t = sum_nu w_nu y_nu,t with w = ZP / c.
// mode: 0 solve, 1 all Tsys NaN (dG = 0), 2 C not finite (ValueError -> dG None).
__global__ void __launch_bounds__(1024) k_gain_weights(const double *__restrict__ tsys0,
                                                       double *__restrict__ gw, int32_t *__restrict__ gmode)
{
    __shared__ double red[16][7];
    const int f = blockIdx.x;
    const double *ts = tsys0 + (int64_t)f * kBC;
    double c00 = 0, c01 = 0, c11 = 0, b0 = 0, b1 = 0, nbad = 0, pp = 0;
    double t0v[4], t1v[4], pv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = threadIdx.x + r * 1024;
        const int c = i % kChannels;
        const double tsv = ts[i];
        const double v = -1.0 + 2.0 * (double)i / (double)(kBC - 1);   // linspace(-1,1,4096)
        double T0 = 1.0 / tsv, T1 = v / tsv, P = 1.0;
        const bool bad = isnan(tsv);
        if (bad) nbad += 1.0;
        if (gain_masked(c) || bad) { T0 = 0.0; T1 = 0.0; P = 0.0; }
        t0v[r] = T0; t1v[r] = T1; pv[r] = P;
        c00 += T0 * T0; c01 += T0 * T1; c11 += T1 * T1;
        b0 += T0 * P; b1 += T1 * P; pp += P;
    }
    double vals[7] = {c00, c01, c11, b0, b1, nbad, pp};
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        double s = wave_sum(vals[k]);
        if (lane == 0) red[wid][k] = s;
    }
    __syncthreads();
    double tot[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        double s = 0;
        for (int w = 0; w < 16; ++w) s += red[w][k];
        tot[k] = s;
    }
    c00 = tot[0]; c01 = tot[1]; c11 = tot[2]; b0 = tot[3]; b1 = tot[4]; nbad = tot[5];
    int mode = 0;
    if (nbad == (double)kBC) mode = 1;
    else if (!isfinite(c00 + c01 + c01 + c11)) mode = 2;
    // inv(C) applied to T01^T P
    const double det = c00 * c11 - c01 * c01;
    const double g0 = (c11 * b0 - c01 * b1) / det;
    const double g1 = (-c01 * b0 + c00 * b1) / det;
    // c = P^T Z P = sum P (P - T0 g0 - T1 g1)
    double cz = 0;
    double zp[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        zp[r] = pv[r] - (t0v[r] * g0 + t1v[r] * g1);
        cz += pv[r] * zp[r];
    }
    __syncthreads();
    double s = wave_sum(cz);
    if (lane == 0) red[wid][0] = s;
    __syncthreads();
    double ctot = 0;
    for (int w = 0; w < 16; ++w) ctot += red[w][0];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int i = threadIdx.x + r * 1024;
        gw[(int64_t)f * kBC + i] = (mode == 0) ? zp[r] / ctot : 0.0;
    }
    if (threadIdx.x == 0) gmode[f] = mode;
}

// ------------------------------------------------------------------ non-finite filtered rows
// After fill_bad_data only +-inf samples and rows whose normalisation failed (alpha = 0:
// rms NaN / 0, or a NaN atmosphere fit) make the filtered TOD y non-finite.  The reference
// then behaves as follows (Level1Averaging.py:681-708, 552-589, 834-867;
// GainSubtraction.py:127-128, 154-158):
//  * alpha = 0: the row is NaN throughout;
//  * a row with +-inf samples and a finite rms ("special"): A^T y of the median-filter
//    regression is non-finite, np.linalg.solve (LU with partial pivoting) returns non-finite
//    x, and y_t = m_t - (x0 + mf_t x1) is +-inf or NaN at EVERY sample;
//  * any non-finite y on the gain fit's channels makes b = P^T Z d non-finite: cg's first
//    matvec raises and solve_gain_solution returns dG = 0;
//  * +-inf anywhere in a band-0 row (the channel nanmean of fit_power_spectrum holds it)
//    makes the PSD bins NaN: IndexError, dG = None and the gain function's in-place
//    zeroing of y never happens;
//  * weighted_average_over_band zeroes a channel's weight when its residual at the scan's
//    first sample is NaN and turns NaN entries into 0 -- +-inf entries stay (and 0 * inf is
//    NaN for a zero weight).
// Special rows are therefore excluded from the fused channel sums and added per sample by
// k_special_rows, which evaluates them exactly as the reference does.

// ynf[u]: a gain-fit input row (band the median filter ran on, median channel, not zeroed
// by gain_subtraction_fit's mask or a NaN Tsys) is non-finite.  One block per unit.
__global__ void __launch_bounds__(256) k_unit_flags(const int32_t *__restrict__ units,
                                                    const double *__restrict__ alpha,
                                                    const int32_t *__restrict__ rowbad,
                                                    const double *__restrict__ bsum,
                                                    const double *__restrict__ tsys0, int32_t *__restrict__ ynf)
{
    __shared__ double red[4];
    const int u = blockIdx.x;
    const int f = units[4 * u];
    double any = 0.0;
    for (int k = threadIdx.x; k < kBC; k += blockDim.x) {
        const int b = k / kChannels, c = k % kChannels;
        if (bsum[4 * ((int64_t)u * kBands + b) + 3] <= 0 || !median_channel(c) || gain_masked(c)) continue;
        if (isnan(tsys0[(int64_t)f * kBC + k])) continue;
        const int64_t i = (int64_t)u * kBC + k;
        if (alpha[i] == 0.0 || rowbad[i] > 0) any = 1.0;
    }
    any = block_sum256(any, red);
    if (threadIdx.x == 0) ynf[u] = any > 0.0;
}

// The regression solve of Level1Averaging.py:704 for a non-finite right-hand side
// (sy = sum y, sym = sum mf y): np.linalg.solve's LU with partial pivoting on
// [[n, Smf], [Smf, Smm]], whose +-inf / NaN outcome differs from Cramer's rule when the
// pivot row swaps (|Smf| > n).
__device__ __forceinline__ void solve2_lu(double n, double Smf, double Smm, double sy, double sym, double &x0,
                                          double &x1)
{
    if (fabs(Smf) > fabs(n)) {            // idamax picks row 1
        const double l = n / Smf, u11 = Smf - l * Smm;
        const double y1 = sy - l * sym;
        x1 = y1 / u11;
        x0 = (sym - Smm * x1) / Smf;
    } else {
        const double l = Smf / n, u11 = Smm - l * Smf;
        const double y1 = sym - l * sy;
        x1 = y1 / u11;
        x0 = (sy - Smf * x1) / n;
    }
}

// A special row: band the median ran on, median channel, finite alpha, +-inf samples
__device__ __forceinline__ bool special_row(bool band_on, int c, double al, int32_t rb)
{
    return band_on && median_channel(c) && al != 0.0 && rb > 0;
}

// y_t of a special row (the reference's order: m_t - (x0 + mf_t x1))
__device__ __forceinline__ double special_y(double al, double o, double a, double x0, double x1, float d, double At,
                                            double mft)
{
    const double m = ((double)d - (o + a * At)) * al;
    return m - (x0 + mft * x1);
}

// weighted_average_over_band's weights for a special row: W (residual; zero when the
// residual at the scan's first sample is NaN) and Wo (tod_original; also zero when
// (y * Tsys) there is NaN)
__device__ __forceinline__ void special_weights(int c, double tsv, double nf, double g, double y0, double &W,
                                                double &Wo)
{
    W = 1.0 / (tsv * tsv);
    if (tsv == 0.0) W = 0.0;
    if (c < 50 || c >= 974 || c == 512 || (c >= 510 && c < 515)) W = 0.0;
    if (isnan(y0 * nf / g)) W = 0.0;
    Wo = W;
    if (isnan(tsv) || isnan(y0 * tsv)) Wo = 0.0;
}

// ------------------------------------------------------------------ L1AGC coefficients II
// Regression solve + the filtered-TOD coefficients f_ct = fa d + fb + fg A_t + fd mf_t
// and the three channel weightings pass D sums:
//   Kg   gain template weights (dG), zero unless the gain fit ran
//   Kres weighted_average_over_band weights * nf / g      (residual)
//   Korig the same weights * Tsys                          (tod_original)
// Level1Averaging.py:701-705, 710-725, 841-867; GainSubtraction.py:190-201.
// dsum[ub][..] = {Sg_b, Gg_b, Dg_b, Sr_b, Gr_b, Dr_b, So_b, Go_b, Do_b, SKr, SW, SWo}
__global__ void __launch_bounds__(256) k_coef_d(const int32_t *__restrict__ units, const double *__restrict__ us,
                                                const double *__restrict__ mom, int64_t UC,
                                                const double *__restrict__ oa,
                                                const double *__restrict__ alpha, const double *__restrict__ nf,
                                                const double *__restrict__ bsum, const double *__restrict__ ss,
                                                double *__restrict__ sdm, const double *__restrict__ tsys0,
                                                const double *__restrict__ gain0, const double *__restrict__ gw,
                                                const int32_t *__restrict__ gmode, int calibrator,
                                                double *__restrict__ kap, double *__restrict__ dsum,
                                                double *__restrict__ xreg, int phase,
                                                int32_t *__restrict__ flag, int32_t *__restrict__ dlist,
                                                int32_t *__restrict__ dcnt, double *__restrict__ dw,
                                                const int32_t *__restrict__ rowbad, const float *__restrict__ tod,
                                                int64_t T, const double *__restrict__ A,
                                                const double *__restrict__ mf, const int32_t *__restrict__ ynf,
                                                const int32_t *__restrict__ ugate)
{
    __shared__ double red[4];
    __shared__ double s_kap[4][kChannels];     // alpha, kg, kr, ko (phase 0 channel list)
    const int ub = blockIdx.x;
    const int u = ub / kBands, b = ub % kBands;
    const int f = units[4 * u];
    const double *q = us + 8 * (int64_t)u;
    const double n = q[0], SA = q[1];
    const double *bs = bsum + 4 * (int64_t)ub;
    const bool band_on = bs[3] > 0;
    const double *sq = ss + 4 * (int64_t)ub;
    const double Smf = sq[0], Smm = sq[1], SAm = sq[2];
    const int gm = gmode[f];
    // gain path (Level1Averaging.py:710-725, 834-838):
    //   zero: y zeroed on the gain mask (gain function was called)
    //   use_dg: dG enters the residual
    // gain_subtraction first runs fit_power_spectrum's gate (:552-589) on the band-0
    // channel mean: np.fft of n <= 4 samples leaves no finite PSD bin (ValueError /
    // IndexError), so dG = None and the gain function (and its in-place zeroing) never
    // runs.  For n >= 5 and finite samples the gate passes (every band-0 channel outside
    // the median set is 0, so the channel nanmean is finite).  A band-0 row holding +-inf
    // after the filter fails the gate too (ugate, k_special_rows); a non-finite gain-fit
    // input leaves dG = 0 (ynf, k_unit_flags) -- see "non-finite filtered rows" above.
    const bool gate = n >= 5.0 && !(ugate && ugate[u]);
    const bool gain_called = !calibrator && gate;
    const bool zero = gain_called;
    const bool use_dg = gain_called && gm == 0 && !ynf[u];
    const double det = n * Smm - Smf * Smf;
    double acc[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) acc[k] = 0.0;
    for (int c = threadIdx.x; c < kChannels; c += blockDim.x) {
        const int64_t i = (int64_t)u * kBC + b * kChannels + c;
        const double o = oa[2 * i], a = oa[2 * i + 1];
        const double al = alpha[i];
        const double tsv = tsys0[(int64_t)f * kBC + b * kChannels + c];
        const bool zeroed = zero && (gain_masked(c) || isnan(tsv));     // y row set to 0 in place
        // a special row (+-inf samples, finite rms) not zeroed: k_special_rows adds it
        const bool special = special_row(band_on, c, al, rowbad[i]) && !zeroed;
        // ---- filtered TOD coefficients
        double fa = 0, fb = 0, fg = 0, fd = 0, x0 = 0, x1 = 0;
        if (band_on && median_channel(c)) {
            if (al != 0.0) {
                const double sdmi = (phase != 0) ? sdm[i] : 0.0;   // pass C (every listed channel)
                const double sy = al * (mom[i] - n * o - a * SA);
                const double sym = al * (sdmi - o * Smf - a * SAm);
                if (phase != 0) {    // phase 0: x unknown yet; kappa never depends on x unless x is NaN
                    if (isfinite(sy) && isfinite(sym)) {
                        x0 = (Smm * sy - Smf * sym) / det;
                        x1 = (n * sym - Smf * sy) / det;
                    } else {
                        solve2_lu(n, Smf, Smm, sy, sym, x0, x1);
                    }
                }
                fa = al; fb = -(al * o + x0); fg = -al * a; fd = -x1;
            } else {                      // NaN channel inside the regression set
                fa = NAN; fb = NAN; fg = NAN; fd = NAN; x0 = NAN; x1 = NAN;
            }
        }
        xreg[2 * i] = x0;
        xreg[2 * i + 1] = x1;
        if (zeroed) { fa = fb = fg = fd = 0.0; }
        const bool fnan = isnan(fa) || isnan(fb) || isnan(fg) || isnan(fd);
        // ---- gain template weight
        const double kg = (use_dg && !special) ? gw[(int64_t)f * kBC + b * kChannels + c] : 0.0;
        // ---- band-average weights (Level1Averaging.py:841-845, 593-596)
        double W = 1.0 / (tsv * tsv);
        if (tsv == 0.0) W = 0.0;
        if (c < 50 || c >= 974 || c == 512 || (c >= 510 && c < 515)) W = 0.0;
        const double nfg = nf[i] / gain0[(int64_t)f * kBC + b * kChannels + c];
        if (isnan(nfg) || fnan) W = 0.0;                       // residual[...,0] NaN
        double kr = (W == 0.0) ? 0.0 : W * nfg;                // never 0 * NaN
        double Wo = W;
        if (isnan(tsv) || fnan) Wo = 0.0;                      // (clean*Tsys)[...,0] NaN
        double ko = (Wo == 0.0) ? 0.0 : Wo * tsv;
        if (special) {          // out of the fused sums; its weights from y at the scan's first sample
            kr = ko = 0.0;
            W = Wo = 0.0;
            if (phase != 0) {
                const int t0 = units[4 * u + 2];
                const float d0 = tod[((int64_t)f * kBC + b * kChannels + c) * T + t0];
                const double y0 = special_y(al, o, a, x0, x1, d0, A[(int64_t)f * T + t0],
                                            mf[((int64_t)f * kBands + b) * T + t0]);
                special_weights(c, tsv, nf[i], gain0[(int64_t)f * kBC + b * kChannels + c], y0, W, Wo);
            }
        }
        // ---- kappa (zero weights contribute exactly nothing, as NaN->0 does)
        const double kgfa = (kg == 0.0) ? 0.0 : kg * fa;
        const double krfa = (kr == 0.0) ? 0.0 : kr * fa;
        const double kofa = (ko == 0.0) ? 0.0 : ko * fa;
        if (phase >= 1) {        // kappa with the regression (and the gate) known must equal the earlier kappa
            if (__double_as_longlong(kap[i]) != __double_as_longlong(kgfa) ||
                __double_as_longlong(kap[UC + i]) != __double_as_longlong(krfa) ||
                __double_as_longlong(kap[2 * UC + i]) != __double_as_longlong(kofa))
                atomicOr(flag, 1);
        }
        kap[i] = kgfa;
        kap[UC + i] = krfa;
        kap[2 * UC + i] = kofa;
        s_kap[0][c] = al;
        s_kap[1][c] = kgfa;
        s_kap[2][c] = krfa;
        s_kap[3][c] = kofa;
        if (kg != 0.0) { acc[0] += kg * fb; acc[1] += kg * fg; acc[2] += kg * fd; }
        if (kr != 0.0) { acc[3] += kr * fb; acc[4] += kr * fg; acc[5] += kr * fd; acc[9] += kr; }
        if (ko != 0.0) { acc[6] += ko * fb; acc[7] += ko * fg; acc[8] += ko * fd; }
        acc[10] += W;
        acc[11] += Wo;
    }
#pragma unroll
    for (int k = 0; k < 12; ++k) acc[k] = block_sum256(acc[k], red);
    if (threadIdx.x == 0 && phase != 0) {
        double *o = dsum + 16 * (int64_t)ub;
#pragma unroll
        for (int k = 0; k < 12; ++k) o[k] = acc[k];
    }
    __syncthreads();
    if (phase == 0 && threadIdx.x < 64) {
        // channel list of passes B and C: the median channels with alpha != 0 (every kappa
        // channel is one of them: fa = alpha), with their (alpha, kg, kr, ko) weights
        double *w = dw + 4 * (int64_t)ub * kChannels;
        const int nc = wave_compact_channels(
            threadIdx.x, [&](int c) { return s_kap[0][c] != 0.0; },
            [&](int j, int c) {
#pragma unroll
                for (int k = 0; k < 4; ++k) w[4 * j + k] = s_kap[k][c];
            },
            [&](int j) {
#pragma unroll
                for (int k = 0; k < 4; ++k) w[4 * j + k] = 0.0;
            },
            dlist + (int64_t)ub * kChannels);
        if (threadIdx.x == 0) dcnt[ub] = nc;
    }
}

// ------------------------------------------------------------------ special rows
// One block per (unit, band).  mode 0 (after k_coef_d phase 1, before phase 2): ugate[u] =
// a band-0 special row's y holds +-inf somewhere (fit_power_spectrum's channel nanmean is
// then non-finite; evaluated before the gain function's zeroing).  mode 1 (after the
// outputs are formed): every special row that was not zeroed adds its residual and
// tod_original terms per sample exactly as weighted_average_over_band forms them
// (Level1Averaging.py:592-599): NaN entries -> 0, +-inf entries kept, times the row's
// weight (0 * inf = NaN), divided by the band's weight sum.  Launched only when pass A
// found non-finite samples after the NaN fill.
__global__ void __launch_bounds__(256) k_special_rows(int mode, const int32_t *__restrict__ units,
                                                      const float *__restrict__ tod, int64_t T,
                                                      const double *__restrict__ A, const double *__restrict__ mf,
                                                      const double *__restrict__ oa, const double *__restrict__ alpha,
                                                      const double *__restrict__ nf, const int32_t *__restrict__ rowbad,
                                                      const double *__restrict__ bsum, const double *__restrict__ xreg,
                                                      const double *__restrict__ tsys0, const double *__restrict__ gain0,
                                                      const double *__restrict__ dsum, int calibrator,
                                                      int32_t *__restrict__ ugate, double *__restrict__ tod_out,
                                                      double *__restrict__ orig_out)
{
    __shared__ int nrow;
    __shared__ int16_t rows[kChannels];
    __shared__ double rw[kChannels], rwo[kChannels];
    const int ub = blockIdx.x;
    const int u = ub / kBands, b = ub % kBands;
    if (mode == 0 && b != 0) return;
    const int f = units[4 * u], t0 = units[4 * u + 2], n = units[4 * u + 3];
    const bool band_on = bsum[4 * (int64_t)ub + 3] > 0;
    if (!band_on) return;
    const bool zero = mode == 1 && !calibrator && n >= 5 && !ugate[u];
    if (threadIdx.x == 0) nrow = 0;
    __syncthreads();
    const int64_t kb = (int64_t)u * kBC + b * kChannels, fb = (int64_t)f * kBC + b * kChannels;
    for (int c = threadIdx.x; c < kChannels; c += blockDim.x) {
        const int64_t i = kb + c;
        if (!special_row(band_on, c, alpha[i], rowbad[i])) continue;
        const double tsv = tsys0[fb + c];
        if (zero && (gain_masked(c) || isnan(tsv))) continue;       // y zeroed in place
        const float d0 = tod[(fb + c) * T + t0];
        const double y0 = special_y(alpha[i], oa[2 * i], oa[2 * i + 1], xreg[2 * i], xreg[2 * i + 1], d0,
                                    A[(int64_t)f * T + t0], mf[((int64_t)f * kBands + b) * T + t0]);
        double W, Wo;
        special_weights(c, tsv, nf[i], gain0[fb + c], y0, W, Wo);
        const int k = atomicAdd(&nrow, 1);
        rows[k] = (int16_t)c;
        rw[k] = W;
        rwo[k] = Wo;
    }
    __syncthreads();
    const int nr = nrow;
    if (nr == 0) return;
    const double *a = A + (int64_t)f * T + t0;
    const double *m = mf + ((int64_t)f * kBands + b) * T + t0;
    if (mode == 0) {
        bool inf = false;
        for (int t = threadIdx.x; t < n; t += blockDim.x)
            for (int k = 0; k < nr; ++k) {
                const int64_t i = kb + rows[k];
                const double y = special_y(alpha[i], oa[2 * i], oa[2 * i + 1], xreg[2 * i], xreg[2 * i + 1],
                                           tod[(fb + rows[k]) * T + t0 + t], a[t], m[t]);
                inf |= isinf(y);
            }
        if (inf) ugate[u] = 1;
        return;
    }
    const double *ds = dsum + 16 * (int64_t)ub;
    const double SW = ds[10], SWo = ds[11];
    double *to = tod_out + ((int64_t)f * kBands + b) * T + t0;
    double *oo = orig_out + ((int64_t)f * kBands + b) * T + t0;
    for (int t = threadIdx.x; t < n; t += blockDim.x) {
        double sr = 0.0, so = 0.0;
        for (int k = 0; k < nr; ++k) {
            const int c = rows[k];
            const int64_t i = kb + c;
            const double y = special_y(alpha[i], oa[2 * i], oa[2 * i + 1], xreg[2 * i], xreg[2 * i + 1],
                                       tod[(fb + c) * T + t0 + t], a[t], m[t]);
            double r = y * nf[i] / gain0[fb + c];
            if (isnan(r)) r = 0.0;
            sr += rw[k] * r;
            double q = y * tsys0[fb + c];
            if (isnan(q)) q = 0.0;
            so += rwo[k] * q;
        }
        to[t] += sr / SW;
        oo[t] += so / SWo;
    }
}

// ------------------------------------------------------------------ pass D
// Per 256-sample tile: wave b sums its band's 1024 channels with kappa_g,
// kappa_r, kappa_o; dG_t = sum over the 4 bands; then
//   tod_b  = (Sr_b - dG SKr_b) / SW_b           (residual band average)
//   orig_b = So_b / SWo_b                        (tod_original)
__global__ void __launch_bounds__(256) k_gain_avg(const float *__restrict__ tod, const double *__restrict__ A,
                                                  const int32_t *__restrict__ units, const int32_t *__restrict__ tiles,
                                                  int64_t T, int64_t UC, const double *__restrict__ kap,
                                                  const double *__restrict__ dsum, const double *__restrict__ mf,
                                                  double *__restrict__ tod_out, double *__restrict__ orig_out,
                                                  double *__restrict__ dG_out, const int32_t *__restrict__ flag)
{
    __shared__ double sg[kBands][kTile];
    if (*flag == 0) return;                         // legacy pass D: only after a fused-path mismatch
    const int b = uniform(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int u = tiles[2 * blockIdx.x], toff = tiles[2 * blockIdx.x + 1];
    const int f = units[4 * u], t0 = units[4 * u + 2], n = units[4 * u + 3];
    const int r0 = toff + 4 * lane;
    const float *base = tod + (int64_t)(f * kBands + b) * kChannels * T + t0 + r0;
    const int64_t kb = (int64_t)u * kBC + b * kChannels;
    const double *kg = kap + kb, *kr = kap + UC + kb, *ko = kap + 2 * UC + kb;
    double ag[4 * kJ], ar[4 * kJ], ao[4 * kJ];
#pragma unroll
    for (int i = 0; i < 4 * kJ; ++i) ag[i] = ar[i] = ao[i] = 0.0;
    const int nv0 = n - r0;
#pragma unroll 2
    for (int c = 0; c < kChannels; ++c) {
        const double wg = kg[c], wr = kr[c], wo = ko[c];
        // channels excluded from all three averages are not read at all: the
        // reference zeroes their weights (and NaN data must not leak as 0 * NaN)
        if (wg == 0.0 && wr == 0.0 && wo == 0.0) continue;
        double x[4 * kJ];
        load_groups(base + (int64_t)c * T, nv0, x);
#pragma unroll
        for (int i = 0; i < 4 * kJ; ++i) {
            ag[i] = fma(wg, x[i], ag[i]);
            ar[i] = fma(wr, x[i], ar[i]);
            ao[i] = fma(wo, x[i], ao[i]);
        }
    }
    const double *ds = dsum + 16 * ((int64_t)u * kBands + b);
    const double *a = A + (int64_t)f * T + t0 + r0;
    const double *m = mf + (int64_t)(f * kBands + b) * T + t0 + r0;
    double at[4 * kJ], mt[4 * kJ];
#pragma unroll
    for (int g = 0; g < kJ; ++g)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int i = 4 * g + e, o = 256 * g + e;
            const bool ok = o < nv0;
            at[i] = ok ? a[o] : 0.0;
            mt[i] = ok ? m[o] : 0.0;
            sg[b][256 * g + 4 * lane + e] = ag[i] + ds[0] + at[i] * ds[1] + mt[i] * ds[2];
        }
    __syncthreads();
    double *to = tod_out + (int64_t)(f * kBands + b) * T + t0 + r0;
    double *oo = orig_out + (int64_t)(f * kBands + b) * T + t0 + r0;
#pragma unroll
    for (int g = 0; g < kJ; ++g)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int i = 4 * g + e, o = 256 * g + e;
            if (o >= nv0) continue;
            const int tl = 256 * g + 4 * lane + e;
            const double dG = sg[0][tl] + sg[1][tl] + sg[2][tl] + sg[3][tl];
            const double sr = ar[i] + ds[3] + at[i] * ds[4] + mt[i] * ds[5];
            const double so = ao[i] + ds[6] + at[i] * ds[7] + mt[i] * ds[8];
            to[o] = (sr - dG * ds[9]) / ds[10];
            oo[o] = so / ds[11];
            if (b == 0) dG_out[(int64_t)f * T + t0 + r0 + o] = dG;
        }
}

// averaged_tod/weights = 1/auto_rms(residual)^2 per (band, scan)
// (Level1Averaging.py:512-518, 867): nanstd of odd-even differences, ddof 0, over the
// unit's n samples of one band, by one 256-thread block.
__device__ __forceinline__ void scan_weight_band(const double *__restrict__ r, int n, double *__restrict__ wo,
                                                 double *red)
{
    const int np = n / 2;
    double s = 0, cnt = 0;
    for (int k = threadIdx.x; k < np; k += blockDim.x) {
        const double d = r[2 * k + 1] - r[2 * k];
        if (!isnan(d)) { s += d; cnt += 1.0; }
    }
    s = block_sum256(s, red);
    cnt = block_sum256(cnt, red);
    const double mean = s / cnt;
    double v = 0;
    for (int k = threadIdx.x; k < np; k += blockDim.x) {
        const double d = r[2 * k + 1] - r[2 * k];
        if (!isnan(d)) v += (d - mean) * (d - mean);
    }
    v = block_sum256(v, red);
    const double rms = sqrt(v / cnt) / sqrt(2.0);
    const double wt = 1.0 / (rms * rms);
    for (int t = threadIdx.x; t < n; t += blockDim.x) wo[t] = wt;
}

__global__ void __launch_bounds__(256) k_scan_weights(const int32_t *__restrict__ units, int64_t T,
                                                      const double *__restrict__ tod_out, double *__restrict__ w_out)
{
    __shared__ double red[4];
    const int ub = blockIdx.x;
    const int u = ub / kBands, b = ub % kBands;
    const int f = units[4 * u], t0 = units[4 * u + 2], n = units[4 * u + 3];
    const int64_t o = (int64_t)(f * kBands + b) * T + t0;
    scan_weight_band(tod_out + o, n, w_out + o, red);
}

// Applies the per-band constants of k_coef_d phase 1 to the fused sums:
//   dG    = Sg + sum_b (Dg0_b + A Dg1_b + mf_b Dg2_b)
//   tod_b = (Sr_b + Dr0 + A Dr1 + mf Dr2 - dG SKr) / SW
//   orig_b = (So_b + Do0 + A Do1 + mf Do2) / SWo
// (Merging k_gain_avg into this kernel behind the flag branch -- one launch fewer --
// cost far more than the launch: the pass-D body's registers and 32 KB of LDS ride on
// every finish block, 103 -> 1448 us at C2, r03s2; reverted.)
__global__ void __launch_bounds__(256) k_finish(const int32_t *__restrict__ units, const int32_t *__restrict__ tiles,
                                                int64_t T, const double *__restrict__ A,
                                                const double *__restrict__ mf, const double *__restrict__ dsum,
                                                double *__restrict__ tod_out, double *__restrict__ orig_out,
                                                double *__restrict__ dG, const int32_t *__restrict__ flag)
{
    if (*flag != 0) return;                          // mismatch: the legacy passes produce the outputs
    const int u = tiles[2 * blockIdx.x];
    const int f = units[4 * u], t0 = units[4 * u + 2], n = units[4 * u + 3];
    const double *ds = dsum + 16 * (int64_t)u * kBands;
    for (int k = threadIdx.x; k < kTile; k += 256) {
        const int r = tiles[2 * blockIdx.x + 1] + k;
        if (r >= n) break;
        const int64_t t = t0 + r;
        const double a = A[(int64_t)f * T + t];
        double m[kBands], g = dG[(int64_t)f * T + t];
#pragma unroll
        for (int b = 0; b < kBands; ++b) {
            m[b] = mf[(int64_t)(f * kBands + b) * T + t];
            const double *d = ds + 16 * b;
            g += d[0] + a * d[1] + m[b] * d[2];
        }
        dG[(int64_t)f * T + t] = g;
#pragma unroll
        for (int b = 0; b < kBands; ++b) {
            const double *d = ds + 16 * b;
            const int64_t o = (int64_t)(f * kBands + b) * T + t;
            tod_out[o] = (tod_out[o] + d[3] + a * d[4] + m[b] * d[5] - g * d[9]) / d[10];
            orig_out[o] = (orig_out[o] + d[6] + a * d[7] + m[b] * d[8]) / d[11];
        }
    }
}

// ------------------------------------------------------------------ output gaps
// The Level-2 outputs are 0 wherever no unit of the plan writes (between scans, and a
// C3 shard's foreign units): zero exactly those samples of every (output, band) instead
// of clearing the whole [3][F][4][T] buffer first.  gap g = (feed, t0, n); grid.y = gap.
__global__ void __launch_bounds__(256) k_zero_gaps(const int64_t *__restrict__ gaps, int64_t T, int F,
                                                   double *__restrict__ tod_out, double *__restrict__ orig_out,
                                                   double *__restrict__ w_out)
{
    const int64_t *g = gaps + 3 * (int64_t)blockIdx.y;
    const int64_t f = g[0], t0 = g[1], n = g[2];
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
#pragma unroll
        for (int b = 0; b < kBands; ++b) {
            const int64_t o = (f * kBands + b) * T + t0 + k;
            tod_out[o] = 0.0;
            orig_out[o] = 0.0;
            w_out[o] = 0.0;
        }
    }
}

// ------------------------------------------------------------------ vane
// system_temperature_from_tod (VaneCalibration.py:67-82): per channel nanmean
// over the hot and cold samples of the vane event; one wave per channel row.
// system_temperature_from_tod (VaneCalibration.py:67-82) with the reference's
// numerics.  tod[..., hot] is a fancy-index gather, which numpy lays out
// F-ordered (strides (4, 4 n)), so its float32 nanmean reduces each channel
// SEQUENTIALLY: s = ((0 + x0) + x1) + ... in float32 with NaN -> 0, then
// float32(double(s) / count).  gain = double(float32(th - tc)) / (t_hot - 2.73)
// and tsys = tc / gain in float64 (t_hot is an np.float64).  Two threads per
// channel row -- the hot and the cold mean are independent sequential sums -- so a
// block is 128 rows x 2 sides; its rows read the same columns, so each cache line
// is fetched once and re-used from L1 for the next 15 columns.
__global__ void __launch_bounds__(256) k_vane(const float *__restrict__ tod, int64_t T, int F,
                                              int64_t vstart, const int32_t *__restrict__ hot,
                                              const int64_t *__restrict__ hoff, const int32_t *__restrict__ cold,
                                              const int64_t *__restrict__ coff, double t_hot,
                                              double *__restrict__ tsys, double *__restrict__ gain)
{
    __shared__ float s_cold[128];
    const int side = threadIdx.x >> 7;                               // wave-uniform: 0 hot, 1 cold
    const int64_t row = (int64_t)blockIdx.x * 128 + (threadIdx.x & 127);   // (f*4+b)*1024 + c
    const bool live = row < (int64_t)F * kBC;
    const int fb = live ? (int)(row / kChannels) : 0;               // uniform: 1024 % 128 == 0
    const float *p = tod + row * T + vstart;
    const int64_t h0 = hoff[fb], h1 = hoff[fb + 1], k0 = coff[fb], k1 = coff[fb + 1];
    float mean = 0.f;
    if (live && h1 != h0) {
        const int32_t *idx = side == 0 ? hot : cold;
        const int64_t j0 = side == 0 ? h0 : k0, j1 = side == 0 ? h1 : k1;
        float s = 0.f;
        int64_t cnt = 0;
        // the adds stay sequential (numpy's order); the loads are issued kV at a time
        // (one at a time the row's ~900 gathers made this a latency chain)
        constexpr int kV = 16;
        int64_t j = j0;
        for (; j + kV <= j1; j += kV) {
            float x[kV];
#pragma unroll
            for (int k = 0; k < kV; ++k) x[k] = p[idx[j + k]];
#pragma unroll
            for (int k = 0; k < kV; ++k) {
                const bool ok = !isnan(x[k]);
                s += ok ? x[k] : 0.f;
                cnt += ok;
            }
        }
        for (; j < j1; ++j) {
            const float x = p[idx[j]];
            const bool ok = !isnan(x);
            s += ok ? x : 0.f;
            cnt += ok;
        }
        mean = (float)((double)s / (double)cnt);   // empty list: nanmean([]) -> NaN
    }
    if (side == 1) s_cold[threadIdx.x & 127] = mean;
    __syncthreads();
    if (side == 1 || !live) return;
    if (h1 == h0) {                                // no hot/cold found (RuntimeError path): zeros
        gain[row] = 0.0;
        tsys[row] = 0.0;
        return;
    }
    const float mc = s_cold[threadIdx.x];
    const float d = mean - mc;
    const double g = (double)d / (t_hot - 2.73);
    gain[row] = g;
    tsys[row] = (double)mc / g;
}

// ------------------------------------------------------------------ generic channel binning
// Level1Averaging.average_tod (Level1Averaging.py:292-321): per (feed, band) and
// bin k of bw channels,
//   x_ct  = f32(d_ct / g_c)                   (tod /= system_gain, in place on the f32 copy)
//   avg_k = sum_c x w_c / W_k,   sq_k = sum_c f32(x x) w_c / W_k,   std = sqrt(sq - avg^2)
// with w = 1/Tsys^2 (edge channels zeroed by the caller) and W_k its per-bin sum.
// numpy reduces the middle (channel) axis sequentially: same order here, each
// product rounded before the add.  Block = 4 waves (wave = band) on a
// 1024-sample tile; every channel is read (masked ones too: NaN * 0 stays NaN).
__global__ void __launch_bounds__(256) k_channel_bin(const float *__restrict__ tod, int64_t T, int32_t bw,
                                                     int32_t nbin, const double *__restrict__ w,
                                                     const double *__restrict__ g, const double *__restrict__ wsum,
                                                     double *__restrict__ avg, double *__restrict__ sd)
{
#pragma clang fp contract(off)
    const int b = uniform(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int64_t ntile = (T + kTile - 1) / kTile;
    const int f = (int)(blockIdx.x / ntile);
    const int64_t t0 = (int64_t)(blockIdx.x % ntile) * kTile;
    const int64_t r0 = t0 + 4 * lane;
    const int nv0 = (int)std::max<int64_t>(-1, std::min<int64_t>(T - r0, 1 << 20));
    const int64_t fb = (int64_t)f * kBands + b;
    const float *base = tod + fb * kChannels * T + r0;
    const double *wc = w + fb * kChannels, *gc = g + fb * kChannels;
    const bool full = t0 + kTile <= T;
    for (int k = 0; k < nbin; ++k) {
        double s1[4 * kJ], s2[4 * kJ];
#pragma unroll
        for (int i = 0; i < 4 * kJ; ++i) s1[i] = s2[i] = 0.0;
        for (int c = k * bw; c < (k + 1) * bw; ++c) {
            const double wv = wc[c], gv = gc[c];
            f32x4u r[kJ];
            if (full) load_raw<kJ, true>(base + (int64_t)c * T, nv0, r);
            else load_raw<kJ, false>(base + (int64_t)c * T, nv0, r);
#pragma unroll
            for (int q = 0; q < kJ; ++q)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float x = (float)((double)r[q][e] / gv);
                    s1[4 * q + e] += (double)x * wv;
                    s2[4 * q + e] += (double)(x * x) * wv;
                }
        }
        const double W = wsum[fb * nbin + k];
        double *ao = avg + (fb * nbin + k) * T + r0, *so = sd + (fb * nbin + k) * T + r0;
#pragma unroll
        for (int q = 0; q < kJ; ++q)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int o = 256 * q + e;
                if (o >= nv0) continue;
                const double a = s1[4 * q + e] / W, sq = s2[4 * q + e] / W;
                ao[o] = a;
                so[o] = sqrt(sq - a * a);
            }
    }
}

// ================================================================== host side
// HIP events around each launch on the plan's stream (comap_l1_profile)
static int prof_begin(comap_l1_plan *p, int id, hipStream_t st)
{
    if (!p->prof_on) return -1;
    // level 1: the three streaming passes only (a bench's timed region: an event pair
    // costs a few us of gap, too much around every small kernel)
    if (p->prof_level == 1 && id != KV_MOMENTS && id != KV_BAND_SUMS && id != KV_REGRESS) return -1;
    const int idx = (int)p->prof_rec.size() * 2;
    while ((int)p->prof_pool.size() < idx + 2) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return -1;
        p->prof_pool.push_back(e);
    }
    (void)hipEventRecord(p->prof_pool[idx], st);
    return idx;
}

static void prof_end(comap_l1_plan *p, int id, int idx, hipStream_t st)
{
    if (idx < 0) return;
    (void)hipEventRecord(p->prof_pool[idx + 1], st);
    p->prof_rec.push_back({id, idx});
}

#define PROF_ON(p, id, st, ...)              \
    do {                                     \
        const int _pi = prof_begin(p, id, st); \
        __VA_ARGS__;                         \
        prof_end(p, id, _pi, st);            \
    } while (0)
#define PROF(p, id, ...) PROF_ON(p, id, (p)->ctx->stream, __VA_ARGS__)

extern "C" int comap_l1_profile(comap_l1_plan *p, int32_t enable)
{
    if (!p) return -1;
    p->prof_on = enable != 0;
    p->prof_level = enable >= 2 ? 2 : 1;
    return 0;
}

extern "C" int comap_l1_profile_collect(comap_l1_plan *p, double *ms, int64_t *counts, int32_t n)
{
    if (!p || !ms || !counts) return -1;
    COMAP_DEVICE_GUARD(p->ctx);
    comap_ctx *ctx = p->ctx;
    COMAP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
    for (auto &r : p->prof_rec) {
        float t = 0.f;
        COMAP_CHECK(ctx, hipEventElapsedTime(&t, p->prof_pool[r.second], p->prof_pool[r.second + 1]));
        p->prof_ms[r.first] += t;
        p->prof_n[r.first] += 1;
    }
    p->prof_rec.clear();
    for (int i = 0; i < n && i < 32; ++i) {
        ms[i] = p->prof_ms[i];
        counts[i] = p->prof_n[i];
        p->prof_ms[i] = 0;
        p->prof_n[i] = 0;
    }
    return 0;
}

static int upload(comap_ctx *ctx, void **dst, const void *src, size_t bytes)
{
    COMAP_CHECK(ctx, hipMalloc(dst, bytes ? bytes : 8));
    if (bytes) COMAP_CHECK(ctx, hipMemcpyAsync(*dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
    return 0;
}

template <typename T>
static int dalloc(comap_ctx *ctx, T **p, size_t count)
{
    COMAP_CHECK(ctx, hipMalloc((void **)p, sizeof(T) * (count ? count : 1)));
    return 0;
}

extern "C" int comap_l1_plan_create(comap_ctx *ctx, const comap_obs_desc *d, comap_l1_plan **out)
{
    if (!ctx || !d || !out) return -1;
    COMAP_DEVICE_GUARD(ctx);
    if (d->n_bands != kBands || d->n_channels != kChannels)
        return comap_fail(ctx, -1, "only 4 bands x 1024 channels are supported");
    if (d->n_units <= 0 || d->n_samples <= 0 || d->n_feeds <= 0)
        return comap_fail(ctx, -1, "empty observation");
    COMAP_CHECK(ctx, hipSetDevice(ctx->device));
    auto *p = new comap_l1_plan();
    p->ctx = ctx;
    p->F = d->n_feeds; p->S = d->n_scans; p->U = d->n_units; p->T = d->n_samples;
    p->tod = d->tod; p->el = d->el;
    p->units_h.assign(d->units_host, d->units_host + 4 * (size_t)d->n_units);
    for (int u = 0; u < p->U; ++u) {
        const int32_t *q = &p->units_h[4 * u];
        if (q[0] < 0 || q[0] >= p->F || q[1] < 0 || q[1] >= p->S || q[2] < 0 || q[3] < 1 ||
            (int64_t)q[2] + q[3] > p->T) {
            delete p;
            return comap_fail(ctx, -1, "unit out of range");
        }
    }
    std::vector<int32_t> tiles;
    for (int u = 0; u < p->U; ++u)
        for (int t = 0; t < p->units_h[4 * u + 3]; t += kTile) { tiles.push_back(u); tiles.push_back(t); }
    p->n_tiles = (int64_t)tiles.size() / 2;
    std::vector<int32_t> tiles_b;
    std::vector<int64_t> tub(p->U + 1, 0);
    for (int u = 0; u < p->U; ++u) {
        // pass B tiles start on 128-B boundaries (up to 31 samples before the scan, read from
        // the same row and never written): PMC bytes 56.9 -> 55.3 GB, time -2.5% at C2
        const int shift = (p->T % 32 == 0) ? (p->units_h[4 * u + 2] & 31) : 0;
        for (int t = -shift; t < p->units_h[4 * u + 3]; t += kTile) { tiles_b.push_back(u); tiles_b.push_back(t); }
        tub[u + 1] = (int64_t)tiles_b.size() / 2;
    }
    // uncovered samples per feed (the complement of the plan's units)
    std::vector<int64_t> gaps;
    {
        std::vector<std::vector<std::pair<int64_t, int64_t>>> cov(p->F);
        for (int u = 0; u < p->U; ++u)
            cov[p->units_h[4 * u]].push_back({p->units_h[4 * u + 2], p->units_h[4 * u + 2] + p->units_h[4 * u + 3]});
        for (int f = 0; f < p->F; ++f) {
            std::sort(cov[f].begin(), cov[f].end());
            int64_t t = 0;
            for (auto &c : cov[f]) {
                if (c.first > t) { gaps.push_back(f); gaps.push_back(t); gaps.push_back(c.first - t); }
                t = std::max(t, c.second);
            }
            if (t < p->T) { gaps.push_back(f); gaps.push_back(t); gaps.push_back(p->T - t); }
        }
        p->n_gaps = (int64_t)gaps.size() / 3;
        for (int64_t g = 0; g < p->n_gaps; ++g) p->max_gap = std::max(p->max_gap, gaps[3 * g + 2]);
    }
    const int64_t UC = (int64_t)p->U * kBC;
    int rc = 0;
    if (p->n_gaps) rc |= upload(ctx, (void **)&p->gaps, gaps.data(), gaps.size() * 8);
    rc |= dalloc(ctx, &p->flag, 1);
    rc |= dalloc(ctx, &p->dlist, (size_t)p->U * kBC);
    rc |= dalloc(ctx, &p->dcnt, (size_t)p->U * kBands);
    rc |= dalloc(ctx, &p->dw, 4 * (size_t)p->U * kBC);
    if (hipHostMalloc((void **)&p->nan_host, 4, hipHostMallocDefault) != hipSuccess) rc |= 1;
    if (hipEventCreateWithFlags(&p->mom_event, hipEventDisableTiming) != hipSuccess) rc |= 1;
    rc |= upload(ctx, (void **)&p->units, p->units_h.data(), p->units_h.size() * 4);
    rc |= upload(ctx, (void **)&p->tiles, tiles.data(), tiles.size() * 4);
    rc |= upload(ctx, (void **)&p->tiles_b, tiles_b.data(), tiles_b.size() * 4);
    rc |= dalloc(ctx, &p->airmass, (size_t)p->F * p->T);
    rc |= dalloc(ctx, &p->unit_sums, 8 * (size_t)p->U);
    rc |= dalloc(ctx, &p->mom, 5 * (size_t)UC);
    rc |= dalloc(ctx, &p->nan_count, 1);
    rc |= dalloc(ctx, &p->alpha, UC);
    rc |= dalloc(ctx, &p->nf, UC);
    rc |= dalloc(ctx, &p->bsum, 4 * (size_t)p->U * kBands);
    rc |= dalloc(ctx, &p->mb, (size_t)p->F * kBands * p->T);
    rc |= dalloc(ctx, &p->mf, (size_t)p->F * kBands * p->T);
    rc |= dalloc(ctx, &p->ssum, 4 * (size_t)p->U * kBands);
    rc |= dalloc(ctx, &p->sdm, UC);
    rc |= dalloc(ctx, &p->gw, (size_t)p->F * kBC);
    rc |= dalloc(ctx, &p->gmode, p->F);
    rc |= dalloc(ctx, &p->kap, 3 * (size_t)UC);
    rc |= dalloc(ctx, &p->dsum, 16 * (size_t)p->U * kBands);
    rc |= dalloc(ctx, &p->xreg, 2 * (size_t)UC);
    rc |= dalloc(ctx, &p->dG, (size_t)p->F * p->T);
    rc |= dalloc(ctx, &p->rowbad, UC);
    rc |= dalloc(ctx, &p->ubs, 4 * (size_t)p->U * kBands);
    rc |= dalloc(ctx, &p->fitsum, 2 * (size_t)UC);
    rc |= dalloc(ctx, &p->oa, 2 * (size_t)UC);
    rc |= dalloc(ctx, &p->ynf, (size_t)p->U);
    rc |= dalloc(ctx, &p->ugate, (size_t)p->U);
    if (rc) { delete p; return -2; }
    // pass B / median / pass C pipeline groups (comap_l1_average): contiguous unit ranges
    // COMAP_GROUPS (env) overrides the compiled default -- measurement knob
    int groups = COMAP_GROUPS;
    if (const char *g = getenv("COMAP_GROUPS")) groups = atoi(g);
    p->ngroups = std::max(1, std::min(std::min(groups, comap_l1_plan::kMaxGroups), (int)p->U));
    {
        std::vector<int64_t> tu(p->U + 1, 0);
        for (int u = 0; u < p->U; ++u) tu[u + 1] = tu[u] + (p->units_h[4 * u + 3] + kTile - 1) / kTile;
        for (int g = 0; g <= p->ngroups; ++g) {
            p->grp_u0[g] = (int32_t)((int64_t)p->U * g / p->ngroups);
            p->grp_tile0[g] = tu[p->grp_u0[g]];
            p->grpb_tile0[g] = tub[p->grp_u0[g]];
        }
    }
    // the median side stream may run at a higher priority than the streaming passes
    // (COMAP_SIDE_PRIO=1): its latency-bound kernels then take CU slots first while
    // the next group's bandwidth-bound pass B runs on the rest
    int prio = 0;
    if (const char *sp = getenv("COMAP_SIDE_PRIO"); sp && sp[0] == '1') {
        int lo = 0, hi = 0;
        if (hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess) prio = hi;
    }
    bool ok = hipStreamCreateWithPriority(&p->side, hipStreamNonBlocking, prio) == hipSuccess;
    for (int g = 0; g < p->ngroups && ok; ++g)
        ok = hipEventCreateWithFlags(&p->ev_b[g], hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&p->ev_m[g], hipEventDisableTiming) == hipSuccess;
    if (!ok) { comap_l1_plan_destroy(p); return comap_fail(ctx, -2, "side stream / events"); }
    // median jobs per group: (unit, band) series, reflect-3 padded [rev, x, rev], outputs [n, 2n)
    // (bands of scans shorter than 2w are skipped by median_filter: no outputs)
    for (int g = 0; g < p->ngroups; ++g) {
        std::vector<MedJob> jobs;
        for (int u = p->grp_u0[g]; u < p->grp_u0[g + 1]; ++u) {
            const int32_t f = p->units_h[4 * u], t0 = p->units_h[4 * u + 2], n = p->units_h[4 * u + 3];
            for (int b = 0; b < kBands; ++b) {
                MedJob j;
                const int64_t off = (int64_t)(f * kBands + b) * p->T + t0;
                j.src = p->mb + off;
                j.dst = p->mf + off;
                j.n = n;
                j.out_lo = n;
                j.out_hi = (n >= 2 * kMedfiltWindow) ? 2 * (int64_t)n : (int64_t)n;
                j.mode = 1;
                j.pad_ = 0;
                j.gate = p->bsum + 4 * ((int64_t)u * kBands + b) + 3;
                jobs.push_back(j);
            }
        }
        rc = comap_median_plan(ctx, &p->medg[g], jobs, kMedfiltWindow);
        if (rc) { comap_l1_plan_destroy(p); return rc; }
    }
    // airmass and per-unit airmass sums depend only on the pointing
    k_airmass<<<2048, 256, 0, ctx->stream>>>(p->el, p->airmass, (int64_t)p->F * p->T);
    COMAP_LAUNCH_CHECK(ctx);
    k_unit_sums<<<p->U, 256, 0, ctx->stream>>>(p->units, p->airmass, p->T, p->unit_sums);
    COMAP_LAUNCH_CHECK(ctx);
    *out = p;
    return 0;
}

extern "C" int comap_l1_plan_destroy(comap_l1_plan *p)
{
    if (!p) return 0;
    COMAP_DEVICE_GUARD(p->ctx);
    if (p->side) (void)hipStreamSynchronize(p->side);
    void *bufs[] = {p->units, p->tiles, p->tiles_b, p->gaps, p->airmass, p->unit_sums, p->mom,
                    p->nan_count, p->alpha, p->nf, p->bsum, p->mb, p->mf, p->ssum, p->sdm, p->gw,
                    p->gmode, p->kap, p->dsum, p->xreg, p->dG, p->rowbad, p->ubs, p->fitsum, p->oa,
                    p->flag, p->dlist, p->dcnt, p->dw, p->nanpos, p->nanpos_n, p->vane_dev,
                    p->sel_pairs, p->sel_voff, p->sel_flag, p->sel_valid, p->ynf, p->ugate};
    for (void *b : bufs)
        if (b) (void)hipFree(b);
    for (int g = 0; g < comap_l1_plan::kMaxGroups; ++g) {
        comap_median_plan_free(&p->medg[g]);
        if (p->ev_b[g]) (void)hipEventDestroy(p->ev_b[g]);
        if (p->ev_m[g]) (void)hipEventDestroy(p->ev_m[g]);
    }
    if (p->side) (void)hipStreamDestroy(p->side);
    if (p->nan_host) (void)hipHostFree(p->nan_host);
    if (p->mom_event) (void)hipEventDestroy(p->mom_event);
    if (p->vane_ev) (void)hipEventDestroy(p->vane_ev);
    if (p->pre_a_ev) (void)hipEventDestroy(p->pre_a_ev);
    if (p->vane_done) (void)hipEventDestroy(p->vane_done);
    if (p->vane_pinned) (void)hipHostFree(p->vane_pinned);
    for (hipEvent_t e : p->prof_pool) (void)hipEventDestroy(e);
    delete p;
    return 0;
}

// Pass A is enqueued without waiting: the 4-byte NaN count comes back through
// pinned memory behind an event, so host work (the vane sample search) can
// overlap the 56 GB read.  wait_moments() makes nan_total valid.
static int launch_moments(comap_l1_plan *p)
{
    comap_ctx *ctx = p->ctx;
    const int64_t UC = (int64_t)p->U * kBC;
    if (!p->pre_a_ev) COMAP_CHECK(ctx, hipEventCreateWithFlags(&p->pre_a_ev, hipEventDisableTiming));
    COMAP_CHECK(ctx, hipEventRecord(p->pre_a_ev, ctx->stream));
    p->pre_a_valid = true;
    COMAP_CHECK(ctx, hipMemsetAsync(p->nan_count, 0, 4, ctx->stream));
    const int64_t grid = (int64_t)p->U * kBands * (kChannels / (4 * kCPW));
    PROF(p, KV_MOMENTS, k_moments<<<grid, 256, 0, ctx->stream>>>(p->tod, p->airmass, p->units, p->T, p->mom, UC,
                                                                     p->nan_count, p->rowbad));
    COMAP_LAUNCH_CHECK(ctx);
    COMAP_CHECK(ctx, hipMemcpyAsync(p->nan_host, p->nan_count, 4, hipMemcpyDeviceToHost, ctx->stream));
    COMAP_CHECK(ctx, hipEventRecord(p->mom_event, ctx->stream));
    p->moments_pending = true;
    p->moments_valid = true;
    return 0;
}

static int wait_moments(comap_l1_plan *p)
{
    if (!p->moments_pending) return 0;
    COMAP_CHECK(p->ctx, hipEventSynchronize(p->mom_event));
    p->nan_total = *p->nan_host;
    p->moments_pending = false;
    return 0;
}

static int run_moments(comap_l1_plan *p)
{
    int rc = launch_moments(p);
    return rc ? rc : wait_moments(p);
}

extern "C" int comap_l1_prefetch(comap_l1_plan *p)
{
    if (!p) return -1;
    COMAP_DEVICE_GUARD(p->ctx);
    int rc = launch_moments(p);
    if (!rc) p->prefetched = true;
    return rc;
}

static int fetch_rowbad(comap_l1_plan *p, std::vector<int32_t> &rb)
{
    comap_ctx *ctx = p->ctx;
    rb.resize((size_t)p->U * kBC);
    COMAP_CHECK(ctx, hipMemcpyAsync(rb.data(), p->rowbad, 4 * rb.size(), hipMemcpyDeviceToHost, ctx->stream));
    COMAP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
    return 0;
}

// nanmedian (f32) of the given (unit, band*1024+channel) rows over their scans
static int unit_row_medians(comap_l1_plan *p, const std::vector<int64_t> &rowids, float *med_dev)
{
    std::vector<int64_t> rows(2 * rowids.size());
    for (size_t k = 0; k < rowids.size(); ++k) {
        const int64_t i = rowids[k];
        const int u = (int)(i / kBC), bc = (int)(i % kBC);
        const int32_t *q = &p->units_h[4 * u];
        rows[2 * k] = ((int64_t)q[0] * kBC + bc) * p->T + q[2];
        rows[2 * k + 1] = q[3];
    }
    return comap_row_nanmedian(p->ctx, p->tod, rows.data(), (int32_t)rowids.size(), med_dev);
}

extern "C" int comap_l1_atmosphere(comap_l1_plan *p, const int32_t *const_el_units, int32_t n_const_el,
                                   double *fit)
{
    if (!p || !fit) return -1;
    COMAP_DEVICE_GUARD(p->ctx);
    p->pre_a_valid = false;            // a later vane call orders itself after this stage
    comap_ctx *ctx = p->ctx;
    hipStream_t st = ctx->stream;
    // pass A, unless comap_l1_prefetch queued it; its NaN count is not waited for here: the
    // NaN path below is gated on the device by pass A's row flags, so this stage queues
    // behind pass A with no host round trip (comap_l1_average reads the count)
    int rc = p->prefetched ? 0 : launch_moments(p);
    p->prefetched = false;
    if (rc) return rc;
    const int64_t UC = (int64_t)p->U * kBC;
    const int UB = p->U * kBands;
    k_ub_from_units<<<(UB + 255) / 256, 256, 0, st>>>(p->unit_sums, p->U, p->ubs);
    COMAP_LAUNCH_CHECK(ctx);
    // select_time: the (unit, band) pairs with a non-finite sample in a fitted channel get
    // their fit sums over the samples where every fitted channel is finite (into fitsum);
    // every other pair keeps pass A's sums
    if (!p->sel_pairs) {
        std::vector<int32_t> pairs(2 * (size_t)UB);
        std::vector<int64_t> voff(UB + 1, 0);
        int maxn = 0;
        for (int u = 0; u < p->U; ++u)
            for (int b = 0; b < kBands; ++b) {
                const int pr = u * kBands + b;
                pairs[2 * pr] = u;
                pairs[2 * pr + 1] = b;
                voff[pr + 1] = voff[pr] + p->units_h[4 * u + 3];
                maxn = std::max(maxn, p->units_h[4 * u + 3]);
            }
        COMAP_CHECK(ctx, hipMalloc((void **)&p->sel_pairs, 4 * pairs.size()));
        COMAP_CHECK(ctx, hipMalloc((void **)&p->sel_voff, 8 * voff.size()));
        COMAP_CHECK(ctx, hipMalloc((void **)&p->sel_flag, 4 * (2 * (size_t)UB + 1)));   // flags, list, count
        COMAP_CHECK(ctx, hipMalloc((void **)&p->sel_valid, (size_t)voff.back() + 1));
        COMAP_CHECK(ctx, comap_upload(p->sel_pairs, pairs.data(), 4 * pairs.size(), st));
        COMAP_CHECK(ctx, comap_upload(p->sel_voff, voff.data(), 8 * voff.size(), st));
        p->sel_maxn = maxn;
    }
    int32_t *plist = p->sel_flag + UB, *pcount = p->sel_flag + 2 * UB;
    k_pair_flags<<<(UB + 3) / 4, 256, 0, st>>>(p->rowbad, UB, p->sel_flag);
    COMAP_LAUNCH_CHECK(ctx);
    k_pair_list<<<1, 64, 0, st>>>(p->sel_flag, UB, plist, pcount);
    COMAP_LAUNCH_CHECK(ctx);
    if (p->sel_maxn > 0) {
        // (a NaN-free cube lists no pair: both kernels return at once)
        const unsigned gy = (unsigned)std::min(UB, 16);    // a few blocks: the listed pairs are strided
        k_select_time<<<dim3((p->sel_maxn + 255) / 256, gy), 256, 0, st>>>(p->tod, p->units, p->sel_pairs, p->T,
                                                                           p->sel_voff, p->sel_valid, plist, pcount);
        COMAP_LAUNCH_CHECK(ctx);
        k_masked_fit_sums<<<dim3(kChannels / 4, gy), 256, 0, st>>>(p->tod, p->airmass, p->units, p->sel_pairs, p->T,
                                                                   p->sel_voff, p->sel_valid, UC, p->fitsum, p->ubs,
                                                                   plist, pcount);
        COMAP_LAUNCH_CHECK(ctx);
    }
    const double *fs = p->mom;
    PROF(p, KV_ATMOS_FIT, k_atmos_fit<<<(UC + 255) / 256, 256, 0, st>>>(p->units, p->ubs, fs, UC, p->F, p->U, fit,
                                                                        p->fitsum, p->sel_flag));
    COMAP_LAUNCH_CHECK(ctx);
    if (n_const_el > 0) {
        // constant-elevation scans: (nanmedian over the scan, 0) for every channel
        std::vector<int64_t> ids;
        for (int k = 0; k < n_const_el; ++k) {
            const int u = const_el_units[k];
            if (u < 0 || u >= p->U) return comap_fail(ctx, -1, "constant-elevation unit out of range");
            for (int bc = 0; bc < kBC; ++bc) ids.push_back((int64_t)u * kBC + bc);
        }
        float *med = nullptr;
        int32_t *dl = nullptr;
        DevTemps tmp(st);
        COMAP_CHECK(ctx, tmp.alloc(&med, ids.size()));
        COMAP_CHECK(ctx, tmp.alloc(&dl, (size_t)n_const_el));
        COMAP_CHECK(ctx, hipMemcpyAsync(dl, const_el_units, 4 * (size_t)n_const_el, hipMemcpyHostToDevice, st));
        if ((rc = unit_row_medians(p, ids, med))) return rc;
        const int64_t nt = (int64_t)n_const_el * kBC;
        k_fit_from_median<<<(nt + 255) / 256, 256, 0, st>>>(p->units, dl, n_const_el, med, p->F, fit);
        COMAP_LAUNCH_CHECK(ctx);
    }
    return 0;
}

// fill_bad_data for every row holding a NaN, then pass A again on the filled cube
static int fill_nan_rows(comap_l1_plan *p)
{
    comap_ctx *ctx = p->ctx;
    hipStream_t st = ctx->stream;
    std::vector<int32_t> rb;
    int rc = fetch_rowbad(p, rb);
    if (rc) return rc;
    std::vector<int64_t> ids;
    for (size_t i = 0; i < rb.size(); ++i)
        if (rb[i] > 0) ids.push_back((int64_t)i);
    if (ids.empty()) return 0;
    float *med = nullptr;
    int64_t *drows = nullptr;
    std::vector<int64_t> rows(2 * ids.size());
    for (size_t k = 0; k < ids.size(); ++k) {
        const int u = (int)(ids[k] / kBC), bc = (int)(ids[k] % kBC);
        const int32_t *q = &p->units_h[4 * u];
        rows[2 * k] = ((int64_t)q[0] * kBC + bc) * p->T + q[2];
        rows[2 * k + 1] = q[3];
    }
    DevTemps tmp(st);
    COMAP_CHECK(ctx, tmp.alloc(&med, ids.size()));
    COMAP_CHECK(ctx, tmp.alloc(&drows, rows.size()));
    // positions the fill overwrites (restored by restore_nan): at most pass A's non-finite count
    const int64_t cap = std::max<int64_t>(p->nan_total, 1);
    if (cap > p->nanpos_cap) {
        if (p->nanpos) (void)hipFree(p->nanpos);
        p->nanpos = nullptr;
        p->nanpos_cap = 0;
        COMAP_CHECK(ctx, hipMalloc((void **)&p->nanpos, 8 * (size_t)cap));
        p->nanpos_cap = cap;
    }
    if (!p->nanpos_n) COMAP_CHECK(ctx, hipMalloc((void **)&p->nanpos_n, 8));
    COMAP_CHECK(ctx, hipMemsetAsync(p->nanpos_n, 0, 8, st));
    COMAP_CHECK(ctx, hipMemcpyAsync(drows, rows.data(), 8 * rows.size(), hipMemcpyHostToDevice, st));
    if ((rc = comap_row_nanmedian(ctx, p->tod, rows.data(), (int32_t)ids.size(), med))) return rc;
    p->filled = true;   // from here on the cube must be restored (restore_nan), even after an error
    for (size_t r0 = 0; r0 < ids.size(); r0 += 65535) {
        const int nr = (int)std::min<size_t>(65535, ids.size() - r0);
        k_fill_rows<<<dim3(16, nr), 256, 0, st>>>(const_cast<float *>(p->tod), drows + 2 * r0, med + r0, nr,
                                                  p->nanpos, p->nanpos_cap, p->nanpos_n);
        COMAP_LAUNCH_CHECK(ctx);
    }
    return run_moments(p);
}

// Puts back the NaNs fill_nan_rows overwrote (stream-ordered after the reduction), so
// every later stage sees the raw cube again; the next pass A re-reads it.
static int restore_nan(comap_l1_plan *p)
{
    if (!p->filled) return 0;
    comap_ctx *ctx = p->ctx;
    k_restore_nan<<<256, 256, 0, ctx->stream>>>(const_cast<float *>(p->tod), p->nanpos, p->nanpos_n, p->nanpos_cap);
    p->filled = false;
    p->moments_valid = false;
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}

extern "C" int comap_l1_average(comap_l1_plan *p, const double *fit, const double *tsys0, const double *gain0,
                                int32_t calibrator, double *tod_out, double *orig_out, double *w_out)
{
    if (!p || !fit || !tsys0 || !gain0 || !tod_out || !orig_out || !w_out) return -1;
    COMAP_DEVICE_GUARD(p->ctx);
    p->pre_a_valid = false;            // the NaN fill below writes the cube
    comap_ctx *ctx = p->ctx;
    int rc = 0;
    if (!p->moments_valid && (rc = run_moments(p))) return rc;
    if ((rc = wait_moments(p))) return rc;
    // the NaN fill is undone (restore_nan) on every return from here on
    struct Restore {
        comap_l1_plan *p;
        ~Restore() { (void)restore_nan(p); }
    } restore{p};
    if (p->nan_total > 0 && !p->filled && (rc = fill_nan_rows(p))) return rc;
    const int64_t UC = (int64_t)p->U * kBC;
    const int UB = p->U * kBands;
    hipStream_t st = ctx->stream;
    DevTemps tmp(st);
    // offsets/slopes to subtract: the scan fits, or per-channel nanmedians for calibrators
    float *cmed = nullptr;
    if (calibrator) {
        std::vector<int64_t> ids(UC);
        for (int64_t i = 0; i < UC; ++i) ids[i] = i;
        COMAP_CHECK(ctx, tmp.alloc(&cmed, (size_t)UC));
        if ((rc = unit_row_medians(p, ids, cmed))) return rc;
    }
    if (p->n_gaps) {
        const unsigned gx = (unsigned)std::min<int64_t>(64, (p->max_gap + 255) / 256);
        k_zero_gaps<<<dim3(gx, (unsigned)p->n_gaps), 256, 0, st>>>(p->gaps, p->T, p->F, tod_out, orig_out, w_out);
        COMAP_LAUNCH_CHECK(ctx);
    }
    PROF(p, KV_COEF_B, k_coef_b<<<UB, 256, 0, st>>>(p->units, p->unit_sums, p->mom, UC, fit, p->F, cmed, p->oa,
                                                    p->alpha, p->nf, p->bsum, p->flag));
    COMAP_LAUNCH_CHECK(ctx);
    PROF(p, KV_GAIN_WEIGHTS, k_gain_weights<<<p->F, 1024, 0, st>>>(tsys0, p->gw, p->gmode));
    COMAP_LAUNCH_CHECK(ctx);
    k_unit_flags<<<p->U, 256, 0, st>>>(p->units, p->alpha, p->rowbad, p->bsum, tsys0, p->ynf);
    COMAP_LAUNCH_CHECK(ctx);
    // +-inf samples left after the NaN fill (pass A counted them): special rows (k_special_rows)
    const bool special = p->nan_total > 0;
    auto coef_d = [&](int phase, const int32_t *ugate) {
        k_coef_d<<<UB, 256, 0, st>>>(p->units, p->unit_sums, p->mom, UC, p->oa, p->alpha, p->nf, p->bsum, p->ssum,
                                     p->sdm, tsys0, gain0, p->gw, p->gmode, calibrator, p->kap, p->dsum, p->xreg,
                                     phase, p->flag, p->dlist, p->dcnt, p->dw, p->rowbad, p->tod, p->T, p->airmass,
                                     p->mf, p->ynf, ugate);
    };
    auto special_rows = [&](int mode) {
        k_special_rows<<<UB, 256, 0, st>>>(mode, p->units, p->tod, p->T, p->airmass, p->mf, p->oa, p->alpha, p->nf,
                                           p->rowbad, p->bsum, p->xreg, tsys0, gain0, p->dsum, calibrator, p->ugate,
                                           tod_out, orig_out);
    };
    // phase 0: the kappa weights and the channel list (no regression needed)
    PROF(p, KV_COEF_D, coef_d(0, nullptr));
    COMAP_LAUNCH_CHECK(ctx);
    // Pass B (band means + every per-sample output sum), the sliding median and pass C
    // (regression sums) are software-pipelined over the unit groups on two streams:
    //   main: B0 B1 .. | wait M0: C0 | wait M1: C1 ..     side: wait B0: M0 | wait B1: M1 ..
    // so each group's median (latency-bound) runs under the next group's streaming pass.
    // one group: the median stays on the main stream -- the two cross-stream event hops
    // cost ~20 us each at the C3 shard (r03s2 trace) and there is nothing to overlap
    hipStream_t side = p->ngroups > 1 ? p->side : st;
    for (int g = 0; g < p->ngroups; ++g) {
        const int64_t t0 = p->grpb_tile0[g], nt = p->grpb_tile0[g + 1] - t0;
        const int ub0 = p->grp_u0[g] * kBands, nub = (p->grp_u0[g + 1] - p->grp_u0[g]) * kBands;
            PROF(p, KV_BAND_SUMS, k_band_sums<<<kSubB * nt, 256, 0, st>>>(p->tod, p->airmass, p->units, p->tiles_b, t0,
                                                                        p->T, p->dlist, p->dcnt, p->dw, p->bsum,
                                                                        p->mb, tod_out, orig_out, p->dG));
        COMAP_LAUNCH_CHECK(ctx);
        if (side != st) {
            COMAP_CHECK(ctx, hipEventRecord(p->ev_b[g], st));
            COMAP_CHECK(ctx, hipStreamWaitEvent(side, p->ev_b[g], 0));
        }
        PROF_ON(p, KV_MEDIAN, side, rc = comap_median_run(ctx, &p->medg[g], side));
        if (rc) return rc;
        PROF_ON(p, KV_SERIES_SUMS, side, k_series_sums<<<nub, 256, 0, side>>>(ub0, p->units, p->airmass, p->T,
                                                                             p->bsum, p->mf, p->ssum));
        COMAP_LAUNCH_CHECK(ctx);
        if (side != st) COMAP_CHECK(ctx, hipEventRecord(p->ev_m[g], side));
    }
    for (int g = 0; g < p->ngroups; ++g) {
        const int ub0 = p->grp_u0[g] * kBands, nub = (p->grp_u0[g + 1] - p->grp_u0[g]) * kBands;
        if (side != st) COMAP_CHECK(ctx, hipStreamWaitEvent(st, p->ev_m[g], 0));
        PROF(p, KV_REGRESS, k_regress<<<nub * kRegBlocks, 256, 0, st>>>(ub0, p->tod, p->mf, p->units, p->T, p->bsum,
                                                                       p->dlist, p->dcnt, p->sdm));
        COMAP_LAUNCH_CHECK(ctx);
    }
    // phase 1: regression solve, per-band constants, kappa re-check
    PROF(p, KV_COEF_D, coef_d(1, nullptr));
    COMAP_LAUNCH_CHECK(ctx);
    if (special) {
        // the fit_power_spectrum gate of units whose band-0 special rows hold +-inf, then the
        // coefficients again with it (a kappa that changes sets the flag: legacy pass D)
        COMAP_CHECK(ctx, hipMemsetAsync(p->ugate, 0, 4 * (size_t)p->U, st));
        special_rows(0);
        COMAP_LAUNCH_CHECK(ctx);
        coef_d(2, p->ugate);
        COMAP_LAUNCH_CHECK(ctx);
        // pass B's fused sums took kappa 0 * inf = NaN at a special row's +-inf samples; the
        // legacy pass D re-forms every output and skips kappa-0 channels
        COMAP_CHECK(ctx, hipMemsetAsync(p->flag, 0xff, 4, st));
    }
    // legacy pass D: exits at once unless phase 1 found a kappa that depends on the
    // regression (a NaN regression coefficient), in which case it recomputes the outputs
    // exactly from phase 1's constants (a former separate phase-2 k_coef_d launch
    // recomputed what phase 1 had already written: dropped)
    PROF(p, KV_GAIN_AVG, k_gain_avg<<<p->n_tiles, 256, 0, st>>>(p->tod, p->airmass, p->units, p->tiles, p->T, UC,
                                                                p->kap, p->dsum, p->mf, tod_out, orig_out, p->dG,
                                                                p->flag));
    COMAP_LAUNCH_CHECK(ctx);
    PROF(p, KV_FINISH, k_finish<<<p->n_tiles, 256, 0, st>>>(p->units, p->tiles, p->T, p->airmass, p->mf, p->dsum,
                                                            tod_out, orig_out, p->dG, p->flag));
    COMAP_LAUNCH_CHECK(ctx);
    if (special) {
        special_rows(1);
        COMAP_LAUNCH_CHECK(ctx);
    }
    PROF(p, KV_SCAN_WEIGHTS, k_scan_weights<<<UB, 256, 0, st>>>(p->units, p->T, tod_out, w_out));
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}


extern "C" int comap_l1_vane(comap_l1_plan *p, int64_t vstart, int64_t vlen, const int32_t *hot_h,
                             const int64_t *hoff_h, const int32_t *cold_h, const int64_t *coff_h,
                             double t_hot, double *tsys, double *gain)
{
    if (!p || !hoff_h || !coff_h || !tsys || !gain) return -1;
    COMAP_DEVICE_GUARD(p->ctx);
    comap_ctx *ctx = p->ctx;
    const int FB = p->F * kBands;
    if (vstart < 0 || vstart + vlen > p->T) return comap_fail(ctx, -1, "vane event out of range");
    const int64_t nh = hoff_h[FB], nc = coff_h[FB];
    for (int64_t i = 0; i < nh; ++i)
        if (hot_h[i] < 0 || hot_h[i] >= vlen) return comap_fail(ctx, -1, "hot index out of range");
    for (int64_t i = 0; i < nc; ++i)
        if (cold_h[i] < 0 || cold_h[i] >= vlen) return comap_fail(ctx, -1, "cold index out of range");
    // index lists -> plan-owned pinned staging (the caller may free its arrays on return)
    // -> plan-owned device buffer, asynchronously: the host does not wait for the kernel
    const size_t off_c = (size_t)nh * 4, off_ho = (off_c + (size_t)nc * 4 + 15) & ~(size_t)15;
    const size_t off_co = off_ho + (size_t)(FB + 1) * 8, bytes = off_co + (size_t)(FB + 1) * 8;
    hipStream_t st = ctx->stream;
    // COMAP_VANE_SIDE=1: k_vane (it reads ~1% of the cube) on the side stream beside pass A
    // (queued by comap_l1_prefetch before the host search) instead of behind it.  Measured
    // at C2: 27.16 vs 27.09 ms per step -- its scattered row reads slow pass A by as much
    // as they hide (the kernel itself 0.23 -> 0.59 ms) -- so it stays on the main stream.
    static const bool use_side = getenv("COMAP_VANE_SIDE") && getenv("COMAP_VANE_SIDE")[0] == '1';
    hipStream_t vs = (use_side && p->side) ? p->side : st;
    if (vs != st) {
        if (!p->pre_a_ev) COMAP_CHECK(ctx, hipEventCreateWithFlags(&p->pre_a_ev, hipEventDisableTiming));
        if (!p->vane_done) COMAP_CHECK(ctx, hipEventCreateWithFlags(&p->vane_done, hipEventDisableTiming));
        if (!p->pre_a_valid) COMAP_CHECK(ctx, hipEventRecord(p->pre_a_ev, st));   // no prefetch: the stream's tail
        COMAP_CHECK(ctx, hipStreamWaitEvent(vs, p->pre_a_ev, 0));
    }
    if (!p->vane_ev) COMAP_CHECK(ctx, hipEventCreateWithFlags(&p->vane_ev, hipEventDisableTiming));
    else COMAP_CHECK(ctx, hipEventSynchronize(p->vane_ev));   // the previous call's upload has run
    if (bytes > p->vane_cap) {
        if (p->vane_pinned) (void)hipHostFree(p->vane_pinned);
        if (p->vane_dev) (void)hipFree(p->vane_dev);
        p->vane_pinned = p->vane_dev = nullptr;
        p->vane_cap = 0;
        COMAP_CHECK(ctx, hipHostMalloc((void **)&p->vane_pinned, bytes, hipHostMallocDefault));
        COMAP_CHECK(ctx, hipMalloc((void **)&p->vane_dev, bytes));
        p->vane_cap = bytes;
    }
    std::memcpy(p->vane_pinned, hot_h, (size_t)nh * 4);
    std::memcpy(p->vane_pinned + off_c, cold_h, (size_t)nc * 4);
    std::memcpy(p->vane_pinned + off_ho, hoff_h, (size_t)(FB + 1) * 8);
    std::memcpy(p->vane_pinned + off_co, coff_h, (size_t)(FB + 1) * 8);
    COMAP_CHECK(ctx, hipMemcpyAsync(p->vane_dev, p->vane_pinned, bytes, hipMemcpyHostToDevice, vs));
    COMAP_CHECK(ctx, hipEventRecord(p->vane_ev, vs));
    const int32_t *dh = (const int32_t *)p->vane_dev;
    const int32_t *dc = (const int32_t *)(p->vane_dev + off_c);
    const int64_t *dho = (const int64_t *)(p->vane_dev + off_ho);
    const int64_t *dco = (const int64_t *)(p->vane_dev + off_co);
    const int64_t rows = (int64_t)FB * kChannels;
    PROF_ON(p, KV_VANE, vs, k_vane<<<(rows + 127) / 128, 256, 0, vs>>>(p->tod, p->T, p->F, vstart, dh, dho, dc, dco,
                                                                      t_hot, tsys, gain));
    COMAP_LAUNCH_CHECK(ctx);
    if (vs != st) {
        COMAP_CHECK(ctx, hipEventRecord(p->vane_done, vs));
        COMAP_CHECK(ctx, hipStreamWaitEvent(st, p->vane_done, 0));
    }
    return 0;
}

extern "C" int comap_l1_debug_fetch(comap_l1_plan *p, int32_t what, double *out, int64_t n)
{
    if (!p || !out) return -1;
    COMAP_DEVICE_GUARD(p->ctx);
    comap_ctx *ctx = p->ctx;
    const int64_t UC = (int64_t)p->U * kBC;
    const double *src = nullptr;
    int64_t cnt = 0;
    switch (what) {
    case 0: src = p->nf; cnt = UC; break;
    case 1: src = p->mf; cnt = (int64_t)p->F * kBands * p->T; break;
    case 2: src = p->dG; cnt = (int64_t)p->F * p->T; break;
    case 3: src = p->xreg; cnt = 2 * UC; break;
    case 4: src = p->mb; cnt = (int64_t)p->F * kBands * p->T; break;
    case 5: src = p->kap; cnt = 3 * UC; break;
    case 6: src = p->dsum; cnt = (int64_t)p->U * kBands * 16; break;
    case 7: src = p->alpha; cnt = UC; break;
    case 8: src = p->oa; cnt = 2 * UC; break;
    case 9: {   // per (unit, band): channel-list length, median band on
        const int UB = p->U * kBands;
        if (n < 2 * (int64_t)UB) return comap_fail(ctx, -1, "debug buffer too small");
        std::vector<int32_t> c(UB);
        std::vector<double> bs(4 * (size_t)UB);
        COMAP_CHECK(ctx, hipMemcpyAsync(c.data(), p->dcnt, 4 * (size_t)UB, hipMemcpyDeviceToHost, ctx->stream));
        COMAP_CHECK(ctx, hipMemcpyAsync(bs.data(), p->bsum, 32 * (size_t)UB, hipMemcpyDeviceToHost, ctx->stream));
        COMAP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
        for (int i = 0; i < UB; ++i) { out[2 * i] = c[i]; out[2 * i + 1] = bs[4 * (size_t)i + 3] > 0 ? 1.0 : 0.0; }
        return 0;
    }
    default: return comap_fail(ctx, -1, "unknown debug array");
    }
    if (n < cnt) return comap_fail(ctx, -1, "debug buffer too small");
    COMAP_CHECK(ctx, hipMemcpyAsync(out, src, cnt * 8, hipMemcpyDeviceToHost, ctx->stream));
    COMAP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
    return 0;
}

extern "C" int comap_l1_channel_bin(comap_l1_plan *p, int32_t bin_size, const double *weights, const double *gain,
                                    const double *wsum, double *avg, double *stddev)
{
    if (!p || !weights || !gain || !wsum || !avg || !stddev) return -1;
    COMAP_DEVICE_GUARD(p->ctx);
    p->pre_a_valid = false;
    comap_ctx *ctx = p->ctx;
    if (bin_size < 1 || kChannels % bin_size) return comap_fail(ctx, -1, "bin_size must divide 1024");
    const int64_t ntile = (p->T + kTile - 1) / kTile;
    k_channel_bin<<<(unsigned)(p->F * ntile), 256, 0, ctx->stream>>>(p->tod, p->T, bin_size, kChannels / bin_size,
                                                                     weights, gain, wsum, avg, stddev);
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}
