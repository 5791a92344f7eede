// rowmedian_kernels.hip -- np.nanmedian of float32 rows on the device.
//
// Used by the rare paths of the L1 reduction that take a per-channel median
// over a scan of the f32 cube:
//   fill_bad_data        NaN -> nanmedian over the scan   (Level1Averaging.py:658-665)
//   filter_atmosphere    constant-elevation scans          (Level1Averaging.py:242-244)
//   remove_atmosphere    calibrator sources                (Level1Averaging.py:647-648)
// NumPy semantics for float32: NaNs ignored; odd count -> middle value; even
// count -> (a + b) / 2 evaluated in float32 (np.mean of the two middle
// float32 values); no finite value -> NaN.
// Rows are sorted with hipcub's segmented radix sort on order-preserving u32
// keys (NaN keys sort last and are not counted).
#include "comap_internal.h"

#include <hipcub/hipcub.hpp>

namespace {

__device__ __forceinline__ uint32_t fkey(float v)
{
    if (isnan(v)) return 0xffffffffu;
    const uint32_t b = __float_as_uint(v);
    return (b >> 31) ? ~b : (b | 0x80000000u);
}

__device__ __forceinline__ float fval(uint32_t k)
{
    const uint32_t b = (k >> 31) ? (k & 0x7fffffffu) : ~k;
    return __uint_as_float(b);
}

// rows: (pointer offset into tod, length); seg = running offsets
__global__ void __launch_bounds__(256) k_row_keys(const float *__restrict__ tod, const int64_t *__restrict__ rows,
                                                  const int32_t *__restrict__ seg, int nrows, uint32_t *__restrict__ keys)
{
    const int r = blockIdx.y;
    if (r >= nrows) return;
    const float *p = tod + rows[2 * r];
    const int s0 = seg[r], n = seg[r + 1] - s0;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) keys[s0 + i] = fkey(p[i]);
}

__global__ void __launch_bounds__(256) k_row_median(const uint32_t *__restrict__ skeys, const int32_t *__restrict__ seg,
                                                    int nrows, float *__restrict__ med)
{
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nrows) return;
    const int s0 = seg[r], n = seg[r + 1] - s0;
    // number of finite entries = index of the first NaN key (binary search)
    int lo = 0, hi = n;
    while (lo < hi) {
        const int m = (lo + hi) >> 1;
        if (skeys[s0 + m] != 0xffffffffu) lo = m + 1; else hi = m;
    }
    const int nf = lo;
    float out;
    if (nf == 0) out = NAN;
    else if (nf & 1) out = fval(skeys[s0 + nf / 2]);
    else {
        const float a = fval(skeys[s0 + nf / 2 - 1]), b = fval(skeys[s0 + nf / 2]);
        out = (a + b) / 2.0f;
    }
    med[r] = out;
}

}  // namespace

// med_dev[r] = nanmedian(tod[rows[2r] : rows[2r] + rows[2r+1]]) (float32 semantics)
int comap_row_nanmedian(comap_ctx *ctx, const float *tod, const int64_t *rows_host, int32_t nrows, float *med_dev)
{
    if (nrows <= 0) return 0;
    hipStream_t st = ctx->stream;
    std::vector<int32_t> seg(nrows + 1, 0);
    for (int r = 0; r < nrows; ++r) {
        if ((int64_t)seg[r] + rows_host[2 * r + 1] >= (1ll << 31)) return comap_fail(ctx, -1, "row median too large");
        seg[r + 1] = seg[r] + (int32_t)rows_host[2 * r + 1];
    }
    const int64_t items = seg.back();
    size_t tb = 0;
    (void)hipcub::DeviceSegmentedRadixSort::SortKeys(nullptr, tb, (uint32_t *)nullptr, (uint32_t *)nullptr, (int)items,
                                                     nrows, (int32_t *)nullptr, (int32_t *)nullptr, 0, 32, st);
    int64_t *drows = nullptr;
    int32_t *dseg = nullptr;
    uint32_t *k0 = nullptr, *k1 = nullptr;
    char *tmp = nullptr;
    DevTemps tmps(st);   // freed on every return path, after the queued work
    COMAP_CHECK(ctx, tmps.alloc(&drows, 2 * (size_t)nrows));
    COMAP_CHECK(ctx, tmps.alloc(&dseg, (size_t)nrows + 1));
    COMAP_CHECK(ctx, tmps.alloc(&k0, (size_t)items));
    COMAP_CHECK(ctx, tmps.alloc(&k1, (size_t)items));
    COMAP_CHECK(ctx, tmps.alloc(&tmp, tb ? tb : 8));
    COMAP_CHECK(ctx, hipMemcpyAsync(drows, rows_host, 16 * (size_t)nrows, hipMemcpyHostToDevice, st));
    COMAP_CHECK(ctx, hipMemcpyAsync(dseg, seg.data(), 4 * (size_t)(nrows + 1), hipMemcpyHostToDevice, st));
    for (int r0 = 0; r0 < nrows; r0 += 65535) {
        const int nr = nrows - r0 < 65535 ? nrows - r0 : 65535;
        k_row_keys<<<dim3(16, nr), 256, 0, st>>>(tod, drows + 2 * r0, dseg + r0, nr, k0);
        COMAP_LAUNCH_CHECK(ctx);
    }
    COMAP_CHECK(ctx, hipcub::DeviceSegmentedRadixSort::SortKeys(tmp, tb, k0, k1, (int)items, nrows, dseg, dseg + 1,
                                                                0, 32, st));
    k_row_median<<<(nrows + 255) / 256, 256, 0, st>>>(k1, dseg, nrows, med_dev);
    COMAP_LAUNCH_CHECK(ctx);
    COMAP_CHECK(ctx, hipStreamSynchronize(st));
    return 0;
}
