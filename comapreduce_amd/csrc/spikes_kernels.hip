// spikes_kernels.hip -- Level-2 spike mask (reference Analysis/Statistics.py:31-105, Spikes).
//
// Per (feed, band):  rms = tod_auto_rms (DataHandling.py:591-597: non-zero
// samples of the whole band row, pairs (2k, 2k+1) of the compacted series,
// nanstd / sqrt 2).  Per (feed, band, scan):
//   mf   = medfilt(tod, MEDIAN_FILTER_STEP) (head/tail semantics of
//          medianFilter.cpp; zeros if the scan holds a non-finite sample;
//          nanmedian if shorter than the window)           (:63-73)
//   raw  = |tod - mf| > SPIKE_THRESHOLD * rms               (:78)
//   mask = raw dilated: fit_spikes marks [start - step, end + step) for each
//          run, with start = index BEFORE the run and end = its last index
//          (:79-93), i.e. mask[t] = any(raw[t - step + 1 .. t + step + 1]).
#include "comap_internal.h"

#include <cmath>

namespace {

__device__ __forceinline__ double wave_sum(double v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ double block_sum1024(double v, double *red)
{
    v = wave_sum(v);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    double s = 0;
    for (int i = 0; i < 16; ++i) s += red[i];
    return s;
}

// compaction of the non-zero samples of one (feed, band) row, in order
__global__ void __launch_bounds__(1024) k_compact_nonzero(const double *__restrict__ tod, int64_t T,
                                                          double *__restrict__ comp, int64_t *__restrict__ cnt)
{
    __shared__ int wsum[16];
    __shared__ int64_t base;
    const int64_t row = blockIdx.x;
    const double *r = tod + row * T;
    double *c = comp + row * T;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (threadIdx.x == 0) base = 0;
    __syncthreads();
    for (int64_t t0 = 0; t0 < T; t0 += 1024) {
        const int64_t t = t0 + threadIdx.x;
        const double v = t < T ? r[t] : 0.0;
        const bool nz = t < T && v != 0.0;           // NaN != 0 is true, as in tod[tod != 0]
        const unsigned long long m = __ballot(nz);
        const int before = __popcll(m & ((1ull << lane) - 1ull));
        if (lane == 0) wsum[w] = __popcll(m);
        __syncthreads();
        int off = 0, tot = 0;
        for (int i = 0; i < 16; ++i) { off += (i < w) ? wsum[i] : 0; tot += wsum[i]; }
        if (nz) c[base + off + before] = v;
        __syncthreads();
        if (threadIdx.x == 0) base += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) cnt[row] = base;
}

// rms = nanstd(c[0:N:2] - c[1:N:2]) / sqrt 2, N = cnt//2*2 (two-pass, ddof 0)
__global__ void __launch_bounds__(1024) k_pair_rms(const double *__restrict__ comp, const int64_t *__restrict__ cnt,
                                                   int64_t T, double *__restrict__ rms)
{
    __shared__ double red[16];
    const int64_t row = blockIdx.x;
    const double *c = comp + row * T;
    const int64_t np = cnt[row] / 2;
    double s = 0, n = 0;
    for (int64_t k = threadIdx.x; k < np; k += blockDim.x) {
        const double d = c[2 * k] - c[2 * k + 1];
        if (!isnan(d)) { s += d; n += 1.0; }
    }
    s = block_sum1024(s, red);
    n = block_sum1024(n, red);
    const double mean = s / n;
    double v = 0;
    for (int64_t k = threadIdx.x; k < np; k += blockDim.x) {
        const double d = c[2 * k] - c[2 * k + 1];
        if (!isnan(d)) v += (d - mean) * (d - mean);
    }
    v = block_sum1024(v, red);
    if (threadIdx.x == 0) rms[row] = sqrt(v / n) / sqrt(2.0);
}

// per job: gate[j] = 1 when the scan is all-finite and long enough for medfilt
// (else 0); short finite scans get their nanmedian (<= w-1 values, LDS sort)
__global__ void __launch_bounds__(256) k_spike_prep(const double *__restrict__ tod, int64_t T,
                                                    const int64_t *__restrict__ jobs, int w,
                                                    double *__restrict__ gate, double *__restrict__ mf)
{
    __shared__ double red[4];
    __shared__ double vals[1024];
    __shared__ int bad_s;
    const int j = blockIdx.x;
    const int64_t row = jobs[3 * j], s = jobs[3 * j + 1], n = jobs[3 * j + 2];
    const double *r = tod + row * T + s;
    if (threadIdx.x == 0) bad_s = 0;
    __syncthreads();
    int bad = 0;
    for (int64_t t = threadIdx.x; t < n; t += blockDim.x) bad |= !isfinite(r[t]);
    if (bad) atomicOr(&bad_s, 1);
    __syncthreads();
    const bool finite = bad_s == 0;
    if (finite && n >= w) {
        if (threadIdx.x == 0) gate[j] = 1.0;
        return;
    }
    if (threadIdx.x == 0) gate[j] = 0.0;
    double *m = mf + row * T + s;
    if (!finite) {                                  // median_filter returns zeros
        for (int64_t t = threadIdx.x; t < n; t += blockDim.x) m[t] = 0.0;
        return;
    }
    // finite and n < w (<= 1023 here): np.nanmedian via an LDS sort
    const int P = 1024;
    for (int i = threadIdx.x; i < P; i += blockDim.x) vals[i] = (i < n) ? r[i] : INFINITY;
    __syncthreads();
    for (int k = 2; k <= P; k <<= 1)
        for (int jj = k >> 1; jj > 0; jj >>= 1) {
            for (int i = threadIdx.x; i < P; i += blockDim.x) {
                const int l = i ^ jj;
                if (l > i) {
                    const bool up = (i & k) == 0;
                    const double a = vals[i], b = vals[l];
                    if ((a > b) == up) { vals[i] = b; vals[l] = a; }
                }
            }
            __syncthreads();
        }
    const double med = (n & 1) ? vals[n / 2] : (vals[n / 2 - 1] + vals[n / 2]) / 2.0;
    (void)red;
    for (int64_t t = threadIdx.x; t < n; t += blockDim.x) m[t] = med;
}

// raw flags -> dilated mask, one workgroup per (job, 1024-sample tile)
__global__ void __launch_bounds__(1024) k_spike_mask(const double *__restrict__ tod, const double *__restrict__ mf,
                                                     const double *__restrict__ rms, int64_t T,
                                                     const int64_t *__restrict__ jobs, double thr, int step,
                                                     uint8_t *__restrict__ mask)
{
    extern __shared__ int pre[];
    const int j = blockIdx.y;
    const int64_t row = jobs[3 * j], s = jobs[3 * j + 1], n = jobs[3 * j + 2];
    const int64_t t0 = (int64_t)blockIdx.x * 1024;
    if (t0 >= n) return;
    const double lim = thr * rms[row];
    const double *r = tod + row * T + s, *m = mf + row * T + s;
    // window of raw flags [t0 - (step-1), t0 + 1024 + step + 1)
    const int64_t lo = t0 - (step - 1);
    const int W = 1024 + 2 * step + 1;
    for (int i = threadIdx.x; i < W; i += blockDim.x) {
        const int64_t t = lo + i;
        int f = 0;
        if (t >= 0 && t < n) f = fabs(r[t] - m[t]) > lim;
        pre[i + 1] = f;
    }
    if (threadIdx.x == 0) pre[0] = 0;
    __syncthreads();
    // inclusive prefix over W entries (simple serial-per-chunk scan)
    if (threadIdx.x == 0)
        for (int i = 1; i <= W; ++i) pre[i] += pre[i - 1];
    __syncthreads();
    const int64_t t = t0 + threadIdx.x;
    if (t < n) {
        const int a = (int)(t - (step - 1) - lo);          // window start index in [0, W)
        const int b = (int)(t + step + 1 - lo);            // inclusive end
        mask[row * T + s + t] = (pre[b + 1] - pre[a]) > 0;
    }
}

}  // namespace

extern "C" int comap_spikes(comap_ctx *ctx, const double *tod, int32_t n_rows, int64_t T, const int64_t *edges,
                            int32_t n_scans, int32_t medfilt_window, int32_t step, double threshold, uint8_t *mask)
{
    if (!ctx || !tod || !mask || n_rows <= 0 || T <= 0) return -1;
    COMAP_DEVICE_GUARD(ctx);
    if (medfilt_window < 1 || medfilt_window > 1023 || step < 1) return comap_fail(ctx, -1, "unsupported spike window");
    hipStream_t st = ctx->stream;
    double *comp = nullptr, *rms = nullptr, *mf = nullptr, *gate = nullptr;
    int64_t *cnt = nullptr, *djobs = nullptr;
    std::vector<int64_t> jobs;
    for (int r = 0; r < n_rows; ++r)
        for (int k = 0; k < n_scans; ++k) {
            const int64_t s = edges[2 * k], e = edges[2 * k + 1];
            if (s < 0 || e > T || e < s) return comap_fail(ctx, -1, "scan edge out of range");
            if (e > s) { jobs.push_back(r); jobs.push_back(s); jobs.push_back(e - s); }
        }
    const int nj = (int)jobs.size() / 3;
    DevTemps tmps(st);   // freed on every return path, after the queued work
    COMAP_CHECK(ctx, tmps.alloc(&comp, (size_t)n_rows * T));
    COMAP_CHECK(ctx, tmps.alloc(&mf, (size_t)n_rows * T));
    COMAP_CHECK(ctx, tmps.alloc(&rms, (size_t)n_rows));
    COMAP_CHECK(ctx, tmps.alloc(&cnt, (size_t)n_rows));
    COMAP_CHECK(ctx, tmps.alloc(&gate, (size_t)nj + 1));
    COMAP_CHECK(ctx, tmps.alloc(&djobs, jobs.size() + 1));
    COMAP_CHECK(ctx, hipMemsetAsync(mask, 0, (size_t)n_rows * T, st));
    if (nj) COMAP_CHECK(ctx, hipMemcpyAsync(djobs, jobs.data(), 8 * jobs.size(), hipMemcpyHostToDevice, st));
    k_compact_nonzero<<<n_rows, 1024, 0, st>>>(tod, T, comp, cnt);
    COMAP_LAUNCH_CHECK(ctx);
    k_pair_rms<<<n_rows, 1024, 0, st>>>(comp, cnt, T, rms);
    COMAP_LAUNCH_CHECK(ctx);
    int rc = 0;
    if (nj) {
        k_spike_prep<<<nj, 256, 0, st>>>(tod, T, djobs, medfilt_window, gate, mf);
        COMAP_LAUNCH_CHECK(ctx);
        std::vector<MedJob> mj(nj);
        int64_t maxn = 0;
        for (int j = 0; j < nj; ++j) {
            MedJob &q = mj[j];
            const int64_t r = jobs[3 * j], s = jobs[3 * j + 1], n = jobs[3 * j + 2];
            q.src = tod + r * T + s;
            q.dst = mf + r * T + s;
            q.n = n;
            q.out_lo = 0;
            q.out_hi = n >= medfilt_window ? n : 0;
            q.mode = 0;
            q.pad_ = 0;
            q.gate = gate + j;
            maxn = std::max(maxn, n);
        }
        MedPlan mp;
        rc = comap_median_plan(ctx, &mp, mj, medfilt_window);
        if (!rc) rc = comap_median_run(ctx, &mp);
        if (!rc) {
            const size_t sm = 4 * (size_t)(1024 + 2 * step + 2);
            k_spike_mask<<<dim3((unsigned)((maxn + 1023) / 1024), nj), 1024, sm, st>>>(tod, mf, rms, T, djobs,
                                                                                        threshold, step, mask);
            hipError_t e = hipGetLastError();
            if (e != hipSuccess) rc = comap_fail(ctx, -2, hipGetErrorString(e));
        }
        hipError_t e = hipStreamSynchronize(st);
        if (!rc && e != hipSuccess) rc = comap_fail(ctx, -2, hipGetErrorString(e));
        comap_median_plan_free(&mp);
    }
    return rc;
}
