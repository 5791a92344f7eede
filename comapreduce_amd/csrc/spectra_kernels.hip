// Batched power spectra of Level-2 TOD scans for the FFT noise QA stages:
//   Level2FitPowerSpectrum.run     (Analysis/Level2Data.py:275-282)
//     power_spectrum = |fft(tod)|**2 / tod.size, freqs > 0
//   NoiseStatistics.power_spectrum (Analysis/Statistics.py:152-156), after the
//     spike interpolation of run_fit_noise (Statistics.py:216-221)
//     ps = |fft(tod)**2|
//
// Per scan (all rows share the scan edges, so one length per scan):
//   k_scan_gather  copies row r's scan slice into a dense [rows][n] f64 batch,
//                  replacing spike-masked samples by np.interp over the unmasked
//                  ones (previous / next good index by block max / min scans);
//   hipFFT D2Z     one batched real FFT per scan length (library FFT: the plain
//                  transform; everything around it is ours);
//   k_power        out[r][k-1] = |X_k|^2 (scaled) for k = 1 .. (n-1)/2, the
//                  bins np.fft.fftfreq marks > 0.
// Bandwidth: a few reads of the Level-2 TOD (F*4*T f64, ~110 MB at C2), far
// below the L1 cube; the host-side fits dominate these stages.
#include <hipcub/hipcub.hpp>
#include <hipfft/hipfft.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "comap_internal.h"

namespace {

constexpr int kGatherThreads = 256;

struct ScanJob {
    int64_t src;    // element offset of the scan start in tod (row r * T + s)
    int64_t dst;    // element offset in the dense batch
    int32_t n;
    int32_t pad_;
};

// np.interp(bad, good, x[good]) at position i with bracketing good indices j < i < k
// (numpy/_core/src/multiarray/compiled_base.c, arr_interp): slope*(x - xp[j]) + fp[j],
// then the other side if NaN; left/right clamps outside the good range.
__device__ __forceinline__ double interp_at(const double *x, int i, int j, int k, int n)
{
#pragma clang fp contract(off)
    if (j < 0 && k >= n) return __builtin_nan("");   // no good sample (the reference raises)
    if (j < 0) return x[k];
    if (k >= n) return x[j];
    const double yj = x[j], yk = x[k];
    const double slope = (yk - yj) / ((double)k - (double)j);
    double r = slope * ((double)i - (double)j) + yj;
    if (isnan(r)) {
        r = slope * ((double)i - (double)k) + yk;
        if (isnan(r) && yj == yk) r = yj;
    }
    return r;
}

// One block per (row, scan): dense copy, masked samples interpolated.
__global__ void __launch_bounds__(kGatherThreads) k_scan_gather(const double *__restrict__ tod,
                                                                const uint8_t *__restrict__ mask,
                                                                const ScanJob *__restrict__ jobs,
                                                                int32_t *__restrict__ prev_scratch,
                                                                double *__restrict__ out)
{
    using Scan = hipcub::BlockScan<int, kGatherThreads>;
    __shared__ typename Scan::TempStorage tmp;
    __shared__ int carry;
    const ScanJob jb = jobs[blockIdx.x];
    const double *x = tod + jb.src;
    double *y = out + jb.dst;
    const int n = jb.n;
    if (!mask) {
        for (int i = threadIdx.x; i < n; i += kGatherThreads) y[i] = x[i];
        return;
    }
    const uint8_t *m = mask + jb.src;
    int32_t *prev = prev_scratch + jb.dst;
    // forward: previous good index (inclusive max-scan of good positions)
    if (threadIdx.x == 0) carry = -1;
    __syncthreads();
    for (int base = 0; base < n; base += kGatherThreads) {
        const int i = base + threadIdx.x;
        const int v = (i < n && !m[i]) ? i : -1;
        int incl;
        Scan(tmp).InclusiveScan(v, incl, hipcub::Max());
        const int c = carry;
        incl = max(incl, c);
        if (i < n) prev[i] = incl;
        __syncthreads();
        if (threadIdx.x == kGatherThreads - 1) carry = incl;
        __syncthreads();
    }
    // backward: next good index (min-scan over reversed positions), then interpolate
    if (threadIdx.x == 0) carry = n;
    __syncthreads();
    for (int top = n - 1; top >= 0; top -= kGatherThreads) {
        const int i = top - (int)threadIdx.x;
        const int v = (i >= 0 && !m[i]) ? i : n;
        int incl;
        Scan(tmp).InclusiveScan(v, incl, hipcub::Min());
        const int c = carry;
        incl = min(incl, c);
        if (i >= 0) y[i] = m[i] ? interp_at(x, i, prev[i], incl, n) : x[i];
        __syncthreads();
        if (threadIdx.x == kGatherThreads - 1) carry = incl;
        __syncthreads();
    }
}

// out[r][k-1] for k = 1 .. nk from the D2Z half spectrum X[r][0 .. n/2].
// mode 0: |X|**2 / n   (np.abs(fft)**2 / size)    mode 1: |X**2|   (np.abs(fft**2))
__global__ void k_power(const hipfftDoubleComplex *__restrict__ X, int64_t rows, int32_t nh, int32_t nk, int32_t n,
                        int32_t mode, double *__restrict__ out)
{
#pragma clang fp contract(off)
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= rows * nk) return;
    const int64_t r = idx / nk;
    const int k = (int)(idx - r * nk) + 1;
    const hipfftDoubleComplex z = X[r * nh + k];
    double p;
    if (mode == 0) {
        const double a = hypot(z.x, z.y);
        p = a * a / (double)n;
    } else {
        p = hypot(z.x * z.x - z.y * z.y, z.x * z.y + z.y * z.x);
    }
    out[idx] = p;
}

const char *fft_err(hipfftResult r)
{
    switch (r) {
    case HIPFFT_SUCCESS: return "success";
    case HIPFFT_INVALID_PLAN: return "invalid plan";
    case HIPFFT_ALLOC_FAILED: return "alloc failed";
    case HIPFFT_INVALID_VALUE: return "invalid value";
    case HIPFFT_EXEC_FAILED: return "exec failed";
    case HIPFFT_SETUP_FAILED: return "setup failed";
    case HIPFFT_INVALID_SIZE: return "invalid size";
    default: return "hipfft error";
    }
}

}  // namespace

extern "C" int comap_power_spectra(comap_ctx *ctx, const double *tod, int32_t n_rows, int64_t T,
                                   const int64_t *edges, int32_t n_scans, const uint8_t *mask, int32_t mode,
                                   const int64_t *out_offsets, double *out)
{
    if (!ctx || !tod || !out || !edges || !out_offsets || n_rows <= 0 || T <= 0 || n_scans < 0)
        return comap_fail(ctx, -1, "comap_power_spectra: bad arguments");
    COMAP_DEVICE_GUARD(ctx);
    if (mode != 0 && mode != 1) return comap_fail(ctx, -1, "comap_power_spectra: mode must be 0 or 1");
    hipStream_t st = ctx->stream;
    int64_t nmax = 0;
    for (int k = 0; k < n_scans; ++k) {
        const int64_t s = edges[2 * k], e = edges[2 * k + 1];
        if (s < 0 || e > T || e < s) return comap_fail(ctx, -1, "scan edge out of range");
        if (e - s > (int64_t)INT32_MAX) return comap_fail(ctx, -1, "scan too long");
        nmax = std::max(nmax, e - s);
    }
    if (nmax < 2) return 0;
    const size_t in_bytes = 8 * (size_t)n_rows * nmax;
    const size_t cx_bytes = 16 * (size_t)n_rows * (nmax / 2 + 1);
    double *buf = nullptr;
    hipfftDoubleComplex *X = nullptr;
    int32_t *prev = nullptr;
    ScanJob *djobs = nullptr;
    int rc = 0;
    std::vector<ScanJob> jobs(n_rows);
    DevTemps tmps(st);   // freed on every return path, after the queued work
    COMAP_CHECK(ctx, tmps.alloc(&buf, in_bytes / 8));
    COMAP_CHECK(ctx, tmps.alloc(&X, cx_bytes / 16));
    COMAP_CHECK(ctx, tmps.alloc(&djobs, (size_t)n_rows * n_scans));
    if (mask) COMAP_CHECK(ctx, tmps.alloc(&prev, (size_t)n_rows * nmax));
    for (int k = 0; k < n_scans && rc == 0; ++k) {
        const int64_t s = edges[2 * k];
        const int n = (int)(edges[2 * k + 1] - s);
        const int nk = (n - 1) / 2;   // fftfreq(n) > 0
        if (nk <= 0) continue;
        for (int r = 0; r < n_rows; ++r) jobs[r] = ScanJob{(int64_t)r * T + s, (int64_t)r * n, n, 0};
        ScanJob *dj = djobs + (size_t)k * n_rows;
        if (hipMemcpyAsync(dj, jobs.data(), sizeof(ScanJob) * n_rows, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess) {   // jobs is reused by the next scan
            rc = comap_fail(ctx, -2, "comap_power_spectra: job upload failed");
            break;
        }
        k_scan_gather<<<n_rows, kGatherThreads, 0, st>>>(tod, mask, dj, prev, buf);
        if (hipGetLastError() != hipSuccess) { rc = comap_fail(ctx, -2, "k_scan_gather launch failed"); break; }
        hipfftHandle plan;
        int len = n, nh = n / 2 + 1;
        hipfftResult fr = hipfftPlanMany(&plan, 1, &len, &len, 1, n, &nh, 1, nh, HIPFFT_D2Z, n_rows);
        if (fr != HIPFFT_SUCCESS) { rc = comap_fail(ctx, -3, std::string("hipfftPlanMany: ") + fft_err(fr)); break; }
        fr = hipfftSetStream(plan, st);
        if (fr == HIPFFT_SUCCESS) fr = hipfftExecD2Z(plan, buf, X);
        if (fr != HIPFFT_SUCCESS) {
            hipfftDestroy(plan);
            rc = comap_fail(ctx, -3, std::string("hipfftExecD2Z: ") + fft_err(fr));
            break;
        }
        const int64_t total = (int64_t)n_rows * nk;
        k_power<<<(unsigned)((total + 255) / 256), 256, 0, st>>>(X, n_rows, nh, nk, n, mode, out + out_offsets[k]);
        if (hipGetLastError() != hipSuccess) rc = comap_fail(ctx, -2, "k_power launch failed");
        // the plan's work area must outlive the queued transform
        if (hipStreamSynchronize(st) != hipSuccess && rc == 0) rc = comap_fail(ctx, -2, "power spectra failed");
        hipfftDestroy(plan);
    }
    return rc;
}
