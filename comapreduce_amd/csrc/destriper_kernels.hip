// destriper_kernels.hip -- destriping map-maker (reference MapMaking/Destriper.py:85-263, 402-503).
//
// The reference's matvec A x = F^T W Z F x (op_Ax) bins every sample twice
// per call (binFuncs.binValues, 97% of its time) and its BiCG calls it three
// times per iteration with bit-identical arguments (p == pb, r == rb).
//
// Pointing and weights are constant during CG, so the operator is rebuilt
// here once as a sparse offset<->pixel structure:
//   entry (o, p, s) with s = sum of w_i over the samples i of offset o that
//   fall in pixel p.  Then, with ws_o = sum_{i in o} w_i and h = weight map,
//     num = W x               num_p = sum_{e in pixel row p} s_e x_{o(e)}
//     m   = num / h           (m_p = num_p where h_p == 0, as share_map)
//     y_o = ws_o x_o - sum_{e in offset row o} s_e m_{p(e)}      (op_Z + F^T W)
// Off-map samples (pixel -1) are never binned but gather m[npix-1], the
// reference's m[-1] wrap (Destriper.py:211).  One CG iteration streams
// 2 nnz entries instead of 6 N samples; all reductions are fixed-order
// (deterministic).  The sample-level maps (weight map h, hits, naive
// numerator sum w tod) are summed per pixel in sample order after a stable
// radix sort, i.e. in exactly binValues' order (bit-exact on one rank).
#include "comap_internal.h"

#include <hipcub/hipcub.hpp>

#include <cmath>

struct comap_destriper {
    comap_ctx *ctx = nullptr;
    int64_t N = 0, NO = 0, npix = 0;
    int32_t L = 0;
    int64_t nnz = 0;       // offset-major entries (incl. off-map gathers)
    int64_t nnzp = 0;      // pixel-major entries (binned only)
    // offset-major
    int64_t *orow = nullptr;   // [NO+1]
    int32_t *opix = nullptr;   // [nnz]  pixel (-1 = off-map)
    double *ow = nullptr;      // [nnz]
    double *ws = nullptr;      // [NO] sum w
    double *tw = nullptr;      // [NO] sum w tod
    // pixel-major
    int64_t *prow = nullptr;   // [npix+1]
    int32_t *poff = nullptr;   // [nnzp]
    double *pw = nullptr;      // [nnzp]
    // sample-level maps (local)
    double *h = nullptr, *hits = nullptr, *nnum = nullptr;   // [npix]
    // reduction scratch
    double *part = nullptr;    // [2 kPartMax] block partials
    double *scal = nullptr;    // [16] device scalars: rr0, rr, pq, rr_new, threshold
    // device-resident CG of comap_destripe_solve (fixed pointers: graph-replayable)
    double *cg = nullptr;          // [4 NO + npix]: x, r, p, q | num
    int32_t *flags = nullptr;      // [2]: stop, iterations
    int32_t *hrow = nullptr;       // [nh] pixel rows with entries (the CG bin skips empty rows)
    int64_t nh = 0;
    int32_t *flags_host = nullptr; // pinned [2]
    double *thr_host = nullptr;    // pinned [1]
    hipStream_t cs = nullptr;      // CG stream (graph capture needs a non-default stream)
    hipEvent_t ev = nullptr;
    hipGraphExec_t batch = nullptr;   // kCgBatch iterations
};

namespace {

constexpr int kRedBlocks = 256;
constexpr int kPartMax = 8192;     // >= every reduction grid below
constexpr int kBinU = 4;           // entry loads in flight per lane (k_ds_bin)
constexpr int kProjU = 4;          // entry loads in flight per lane (k_ds_project)
constexpr int kCgBatch = 16;       // CG iterations per replayed graph (one host check per batch)

// Device-side CG stop flag (comap_destripe_solve): once set, every kernel of the
// remaining enqueued iterations returns at once, so iterations run as replayed
// hipGraph batches with one host round trip per batch.
__device__ __forceinline__ bool cg_done(const int32_t *done) { return done && *done; }

__device__ __forceinline__ double wave_sum(double v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Fixed-order sum of n block partials by one 256-thread block (k_dot_final's order).
__device__ __forceinline__ double block_final_sum(const double *__restrict__ part, int n, double *red)
{
    double acc = 0.0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) acc += part[i];
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    return (red[0] + red[1]) + (red[2] + red[3]);
}

// One wave per offset: lane l owns samples l, l + 64, ... (K per lane, L <= 64 K).
// Unique pixels in first-occurrence order, weights summed in sample order.
// pass 0 counts (and sums ws = sum w, tw = sum w tod), pass 1 fills.
template <int K>
__global__ void __launch_bounds__(256) k_ds_entries(const int32_t *__restrict__ pix, const double *__restrict__ w,
                                                    const double *__restrict__ tod, int64_t NO, int L, int pass,
                                                    int64_t *__restrict__ cnt, const int64_t *__restrict__ orow,
                                                    int32_t *__restrict__ opix, double *__restrict__ ow,
                                                    double *__restrict__ ws, double *__restrict__ tw)
{
    const int lane = threadIdx.x & 63;
    const int64_t o = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (o >= NO) return;
    int32_t p[K];
    double wi[K], gsum[K];
    bool first[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int sidx = lane + 64 * k;
        const bool in = sidx < L;
        p[k] = in ? pix[o * L + sidx] : -2;
        wi[k] = in ? w[o * L + sidx] : 0.0;
        first[k] = in;
        gsum[k] = 0.0;
    }
    // every sample in order (chunk kk, lane j): first occurrence and the in-order group sum
#pragma unroll
    for (int kk = 0; kk < K; ++kk)
        for (int j = 0; j < 64; ++j) {
            const int32_t pj = __shfl(p[kk], j, 64);
            const double wj = __shfl(wi[kk], j, 64);
#pragma unroll
            for (int k = 0; k < K; ++k)
                if (pj == p[k]) {
                    if (j + 64 * kk < lane + 64 * k) first[k] = false;
                    gsum[k] += wj;
                }
        }
    unsigned long long m[K];
#pragma unroll
    for (int k = 0; k < K; ++k) m[k] = __ballot(first[k] && gsum[k] != 0.0);
    if (pass == 0) {
        int64_t c = 0;
        double sw = 0.0, st = 0.0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            c += __popcll(m[k]);
            sw += wi[k];
            if (lane + 64 * k < L) st += wi[k] * tod[o * L + lane + 64 * k];
        }
        sw = wave_sum(sw);
        st = wave_sum(st);
        if (lane == 0) { cnt[o] = c; ws[o] = sw; tw[o] = st; }
        return;
    }
    int base = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        if ((m[k] >> lane) & 1ull) {
            const int64_t e = orow[o] + base + __popcll(m[k] & ((1ull << lane) - 1ull));
            opix[e] = p[k];
            ow[e] = gsum[k];
        }
        base += __popcll(m[k]);
    }
}

static void launch_entries(int L, unsigned blocks, hipStream_t st, const int32_t *pix, const double *w,
                           const double *tod, int64_t NO, int pass, int64_t *cnt, const int64_t *orow,
                           int32_t *opix, double *ow, double *ws, double *tw)
{
    if (L <= 64)
        k_ds_entries<1><<<blocks, 256, 0, st>>>(pix, w, tod, NO, L, pass, cnt, orow, opix, ow, ws, tw);
    else if (L <= 128)
        k_ds_entries<2><<<blocks, 256, 0, st>>>(pix, w, tod, NO, L, pass, cnt, orow, opix, ow, ws, tw);
    else
        k_ds_entries<4><<<blocks, 256, 0, st>>>(pix, w, tod, NO, L, pass, cnt, orow, opix, ow, ws, tw);
}

// keys for the pixel-major transpose: pixel of each offset-major entry (npix for off-map)
__global__ void k_entry_keys(const int64_t *__restrict__ orow, int64_t NO, const int32_t *__restrict__ opix,
                             int64_t npix, int32_t *__restrict__ key, int32_t *__restrict__ val,
                             int32_t *__restrict__ eoff)
{
    for (int64_t o = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; o < NO; o += (int64_t)gridDim.x * blockDim.x) {
        for (int64_t e = orow[o]; e < orow[o + 1]; ++e) {
            const int32_t p = opix[e];
            key[e] = (p >= 0 && p < npix) ? p : (int32_t)npix;
            val[e] = (int32_t)e;
            eoff[e] = (int32_t)o;
        }
    }
}

__device__ __forceinline__ int64_t lb32(const int32_t *a, int64_t n, int64_t v)
{
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t m = (lo + hi) >> 1;
        if (a[m] < v) lo = m + 1; else hi = m;
    }
    return lo;
}

__global__ void k_rowptr(const int32_t *__restrict__ skey, int64_t n, int64_t npix, int64_t *__restrict__ row)
{
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p <= npix; p += (int64_t)gridDim.x * blockDim.x)
        row[p] = lb32(skey, n, p);
}

__global__ void k_pixel_entries(const int32_t *__restrict__ sval, int64_t nnzp, const int32_t *__restrict__ eoff,
                                const double *__restrict__ ow, int32_t *__restrict__ poff, double *__restrict__ pw)
{
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < nnzp; k += (int64_t)gridDim.x * blockDim.x) {
        const int32_t e = sval[k];
        poff[k] = eoff[e];
        pw[k] = ow[e];
    }
}

// sample-level maps in binValues order (stable pixel sort keeps sample order)
__global__ void k_sample_keys(const int32_t *__restrict__ pix, int64_t N, int64_t npix, int32_t *__restrict__ key,
                              int32_t *__restrict__ val)
{
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < N; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t p = pix[i];
        key[i] = (p >= 0 && p < npix) ? p : (int32_t)npix;
        val[i] = (int32_t)i;
    }
}

__global__ void k_sample_maps(const int32_t *__restrict__ skey, const int32_t *__restrict__ sval, int64_t N,
                              int64_t npix, const double *__restrict__ w, const double *__restrict__ tod,
                              double *__restrict__ h, double *__restrict__ hits, double *__restrict__ nnum)
{
#pragma clang fp contract(off)   // binValues(weights=z*w): the product is rounded before the add
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < npix; p += (int64_t)gridDim.x * blockDim.x) {
        const int64_t lo = lb32(skey, N, p), hi = lb32(skey, N, p + 1);
        double sh = 0.0, sc = 0.0, sn = 0.0;
        for (int64_t k = lo; k < hi; ++k) {
            const int32_t i = sval[k];
            const double wi = w[i];
            sh += wi;
            sn += tod[i] * wi;
            sc += 1.0;
        }
        h[p] = sh;
        hits[p] = sc;
        nnum[p] = sn;
    }
}

__device__ __forceinline__ double map_value(const double *num, const double *h, int64_t q)
{
    const double hv = h[q];
    return hv != 0.0 ? num[q] / hv : num[q];
}

// num_p = sum_e s_e x_o(e); base != NULL: num = base - W x (final destriped numerator);
// hdiv != NULL: num = m = (W x) / h, the map itself (single rank: k_ds_project then gathers
// one array).  kBinLanes lanes per pixel row (rows hold 0 .. thousands of entries),
// lane-strided; each lane issues kBinU entry loads, then kBinU gathers, before its fmas
// (in entry order, so the sum is the plain lane-strided one), then a kBinLanes-lane reduction.
template <int kBinLanes>
__global__ void __launch_bounds__(256) k_ds_bin(const int64_t *__restrict__ prow, const int32_t *__restrict__ poff,
                                                const double *__restrict__ pw, const double *__restrict__ x,
                                                int64_t npix, const double *__restrict__ base,
                                                const double *__restrict__ hdiv, double *__restrict__ num,
                                                const int32_t *__restrict__ done, const int32_t *__restrict__ rows = nullptr)
{
    if (cg_done(done)) return;
    const int sub = threadIdx.x & (kBinLanes - 1);
    const int64_t step = (int64_t)gridDim.x * blockDim.x / kBinLanes;
    // rows != NULL: only the listed (non-empty) rows, npix = their count
    for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kBinLanes; i < npix; i += step) {
        const int64_t p = rows ? (int64_t)rows[i] : i;
        double s = 0.0;
        const int64_t e1 = prow[p + 1];
        for (int64_t k = prow[p] + sub; k < e1; k += kBinLanes * kBinU) {
            int32_t o[kBinU];
            double a[kBinU], xv[kBinU];
#pragma unroll
            for (int u = 0; u < kBinU; ++u) {
                const bool in = k + u * kBinLanes < e1;
                o[u] = in ? poff[k + u * kBinLanes] : 0;
                a[u] = in ? pw[k + u * kBinLanes] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < kBinU; ++u) xv[u] = x[o[u]];
#pragma unroll
            for (int u = 0; u < kBinU; ++u)
                if (k + u * kBinLanes < e1) s = fma(a[u], xv[u], s);
        }
#pragma unroll
        for (int o = kBinLanes / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, kBinLanes);
        if (sub == 0) {
            if (base) s = base[p] - s;
            else if (hdiv) { const double hv = hdiv[p]; s = hv != 0.0 ? s / hv : s; }
            num[p] = s;
        }
    }
}

// y_o = ws_o x_o - sum_e s_e m_p(e)  (x == NULL: y_o = tw_o - ..., the b vector).
// G lanes per offset (G = 16 for L <= 64: 256/G offsets per block sweep); each lane issues
// kProjU entry loads then kProjU map gathers before its fmas; m = num / h, or num itself
// when h == NULL (k_ds_bin already divided).  Block partials of y.x (dot_part != NULL).
template <int G>
__global__ void __launch_bounds__(256) k_ds_project(const int64_t *__restrict__ orow, const int32_t *__restrict__ opix,
                                                    const double *__restrict__ ow, const double *__restrict__ ws,
                                                    const double *__restrict__ tw, const double *__restrict__ x,
                                                    const double *__restrict__ num, const double *__restrict__ h,
                                                    int64_t NO, int64_t npix, double *__restrict__ y,
                                                    double *__restrict__ dot_part, const int32_t *__restrict__ done)
{
    __shared__ double red[4];
    if (cg_done(done)) return;
    constexpr int kPer = 256 / G;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, sub = threadIdx.x & (G - 1);
    double acc = 0.0;
    for (int64_t o0 = (int64_t)blockIdx.x * kPer; o0 < NO; o0 += (int64_t)gridDim.x * kPer) {
        const int64_t o = o0 + threadIdx.x / G;
        const bool valid = o < NO;
        const int64_t e1 = valid ? orow[o + 1] : 0;
        double g = 0.0;
        for (int64_t e = (valid ? orow[o] : 0) + sub; e < e1; e += G * kProjU) {
            int32_t q[kProjU];
            double a[kProjU], mv[kProjU];
#pragma unroll
            for (int u = 0; u < kProjU; ++u) {
                const bool in = e + u * G < e1;
                const int32_t pp = in ? opix[e + u * G] : 0;
                q[u] = pp >= 0 ? pp : (int32_t)(npix - 1);   // m[-1] for off-map samples
                a[u] = in ? ow[e + u * G] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < kProjU; ++u) mv[u] = h ? map_value(num, h, q[u]) : num[q[u]];
#pragma unroll
            for (int u = 0; u < kProjU; ++u)
                if (e + u * G < e1) g = fma(a[u], mv[u], g);
        }
#pragma unroll
        for (int s = G / 2; s > 0; s >>= 1) g += __shfl_xor(g, s, G);
        if (valid && sub == 0) {
            const double v = (x ? ws[o] * x[o] : tw[o]) - g;
            y[o] = v;
            if (dot_part) acc = fma(v, x[o], acc);
        }
    }
    if (dot_part) {
        acc = wave_sum(acc);
        if (lane == 0) red[wid] = acc;
        __syncthreads();
        if (threadIdx.x == 0) dot_part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
    }
}

__global__ void __launch_bounds__(256) k_dot_part(const double *__restrict__ a, const double *__restrict__ b, int64_t n,
                                                  double *__restrict__ part)
{
    __shared__ double red[4];
    double acc = 0.0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        acc = fma(a[i], b[i], acc);
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ void __launch_bounds__(256) k_dot_final(const double *__restrict__ part, int n, double *__restrict__ out,
                                                   const int32_t *__restrict__ done)
{
    __shared__ double red[4];
    if (cg_done(done)) return;
    const double sum = block_final_sum(part, n, red);
    if (threadIdx.x == 0) out[0] = sum;
}

// x += a p ; r -= a q ; a = rr / pq ; partials of r.r
__global__ void __launch_bounds__(256) k_cg_update(const double *__restrict__ rr, const double *__restrict__ pq,
                                                   double *__restrict__ x, double *__restrict__ r,
                                                   const double *__restrict__ p, const double *__restrict__ q,
                                                   int64_t n, double *__restrict__ part, const int32_t *__restrict__ done)
{
    __shared__ double red[4];
    if (cg_done(done)) return;
    const double a = rr[0] / pq[0];
    double acc = 0.0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        x[i] += a * p[i];
        const double ri = r[i] - a * q[i];
        r[i] = ri;
        acc = fma(ri, ri, acc);
    }
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// Fused single-rank CG tail (comap_destripe_solve): no separate final-sum or check
// launches.  Every block re-derives the global sums from the previous kernel's block
// partials in k_dot_final's order, so all blocks hold identical values and no block
// waits on another.  scal: [0] rr0, [1] rr of this iteration (for beta), [3] current rr.
//   k_cg_update_fused: pq = sum(pq partials); a = scal[3] / pq; x += a p; r -= a q;
//                      r.r partials into part_rr; block 0 saves scal[1] = scal[3]
//   k_cg_direction_fused: rr_new = sum(part_rr); p = r + (rr_new / scal[1]) p;
//                      block 0: scal[3] = rr_new, count, stop test (k_cg_check)
__global__ void __launch_bounds__(256) k_cg_update_fused(double *__restrict__ scal, const double *__restrict__ part_pq,
                                                         int npq, double *__restrict__ x, double *__restrict__ r,
                                                         const double *__restrict__ p, const double *__restrict__ q,
                                                         int64_t n, double *__restrict__ part_rr,
                                                         const int32_t *__restrict__ done)
{
    __shared__ double red[4];
    if (cg_done(done)) return;
    const double pq = block_final_sum(part_pq, npq, red);
    const double rr = scal[3];
    const double a = rr / pq;
    __syncthreads();
    double acc = 0.0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        x[i] += a * p[i];
        const double ri = r[i] - a * q[i];
        r[i] = ri;
        acc = fma(ri, ri, acc);
    }
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        part_rr[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
        if (blockIdx.x == 0) { scal[1] = rr; scal[2] = pq; }
    }
}

__global__ void __launch_bounds__(256) k_cg_direction_fused(double *__restrict__ scal, const double *__restrict__ part_rr,
                                                            int nrr, double *__restrict__ p, const double *__restrict__ r,
                                                            int64_t n, int32_t *flags)
{
    __shared__ double red[4];
    if (flags[0]) return;
    const double rrn = block_final_sum(part_rr, nrr, red);
    const double beta = rrn / scal[1];
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = r[i] + beta * p[i];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        scal[3] = rrn;
        flags[1] += 1;
        const double delta = rrn / scal[0];
        if (isnan(delta) || delta < scal[4]) flags[0] = 1;
    }
}

__global__ void k_cg_direction(const double *__restrict__ rr_new, const double *__restrict__ rr, double *__restrict__ p,
                               const double *__restrict__ r, int64_t n, const int32_t *__restrict__ done)
{
    if (cg_done(done)) return;
    const double beta = rr_new[0] / rr[0];
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = r[i] + beta * p[i];
}

// End of one CG iteration (Destriper.py:136-152): rr = rr_new, count it, stop when
// delta = rr_new / rr0 is NaN or below the threshold (scal[4]).
__global__ void k_cg_check(double *__restrict__ scal, int32_t *__restrict__ flags)
{
    if (threadIdx.x != 0 || flags[0]) return;
    const double rrn = scal[3];
    scal[1] = rrn;
    flags[1] += 1;
    const double delta = rrn / scal[0];
    if (isnan(delta) || delta < scal[4]) flags[0] = 1;
}

__global__ void k_div_map(const double *__restrict__ num, const double *__restrict__ h, int64_t npix,
                          double *__restrict__ out)
{
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < npix; p += (int64_t)gridDim.x * blockDim.x)
        out[p] = map_value(num, h, p);
}

inline unsigned grid_for(int64_t n, int64_t cap = 4096) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, cap)); }
// k_ds_bin with kBinLanes sized to the mean pixel-row length (sparse C4-like maps
// hold ~5 entries per pixel: 16 lanes per row would leave most lanes idle and
// need several latency-bound grid sweeps); one sweep over all rows.
// hit_rows: only the non-empty rows (d->hrow; the caller's num must hold 0 on the
// empty rows, as the CG's own map buffer does).
void launch_bin(const comap_destriper *d, hipStream_t st, const double *x, const double *base, const double *hdiv,
                double *num, const int32_t *done, bool hit_rows = false)
{
    const int64_t np = hit_rows ? d->nh : d->npix;
    const int32_t *rows = hit_rows ? d->hrow : nullptr;
    const int64_t mean = np ? d->nnzp / np : 0;
    const int lanes = mean >= 24 ? 16 : (mean >= 10 ? 8 : 4);
    const unsigned g = grid_for(np * lanes, 65536);
    if (lanes == 16)
        k_ds_bin<16><<<g, 256, 0, st>>>(d->prow, d->poff, d->pw, x, np, base, hdiv, num, done, rows);
    else if (lanes == 8)
        k_ds_bin<8><<<g, 256, 0, st>>>(d->prow, d->poff, d->pw, x, np, base, hdiv, num, done, rows);
    else
        k_ds_bin<4><<<g, 256, 0, st>>>(d->prow, d->poff, d->pw, x, np, base, hdiv, num, done, rows);
}

inline int project_lanes(int L) { return L <= 64 ? 16 : (L <= 128 ? 32 : 64); }
inline unsigned project_grid(int64_t NO, int L)
{
    const int64_t per = 256 / project_lanes(L);
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>((NO + per - 1) / per, kPartMax));
}

// k_ds_project with the lane group sized to the offset length; returns its grid (= partials).
unsigned launch_project(const comap_destriper *d, hipStream_t st, const double *x, const double *num,
                        const double *h, double *y, double *part, const int32_t *done)
{
    const unsigned pg = project_grid(d->NO, d->L);
    switch (project_lanes(d->L)) {
    case 16:
        k_ds_project<16><<<pg, 256, 0, st>>>(d->orow, d->opix, d->ow, d->ws, d->tw, x, num, h, d->NO, d->npix, y, part, done);
        break;
    case 32:
        k_ds_project<32><<<pg, 256, 0, st>>>(d->orow, d->opix, d->ow, d->ws, d->tw, x, num, h, d->NO, d->npix, y, part, done);
        break;
    default:
        k_ds_project<64><<<pg, 256, 0, st>>>(d->orow, d->opix, d->ow, d->ws, d->tw, x, num, h, d->NO, d->npix, y, part, done);
    }
    return pg;
}

template <typename T>
int dalloc(comap_ctx *ctx, T **p, size_t n)
{
    COMAP_CHECK(ctx, hipMalloc((void **)p, sizeof(T) * (n ? n : 1)));
    return 0;
}

int dot(comap_destriper *d, const double *a, const double *b, double *out)
{
    comap_ctx *ctx = d->ctx;
    k_dot_part<<<kRedBlocks, 256, 0, ctx->stream>>>(a, b, d->NO, d->part);
    COMAP_LAUNCH_CHECK(ctx);
    k_dot_final<<<1, 256, 0, ctx->stream>>>(d->part, kRedBlocks, out, nullptr);
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}

}  // namespace

extern "C" int comap_destripe_create(comap_ctx *ctx, const int32_t *pix, const double *tod, const double *w,
                                     int64_t N, int32_t L, int64_t npix, comap_destriper **out)
{
    if (!ctx || !pix || !tod || !w || !out) return -1;
    COMAP_DEVICE_GUARD(ctx);
    if (L < 1 || L > 256) return comap_fail(ctx, -1, "offset_length must be in [1, 256]");
    if (N <= 0 || N % L) return comap_fail(ctx, -1, "n_samples must be a positive multiple of offset_length");
    if (npix <= 0 || npix >= (1ll << 31) - 1 || N >= (1ll << 31)) return comap_fail(ctx, -1, "size limits exceeded");
    hipStream_t st = ctx->stream;
    auto *d = new comap_destriper();
    d->ctx = ctx; d->N = N; d->L = L; d->NO = N / L; d->npix = npix;
    int rc = 0;
    rc |= dalloc(ctx, &d->orow, d->NO + 1);
    rc |= dalloc(ctx, &d->ws, d->NO);
    rc |= dalloc(ctx, &d->tw, d->NO);
    rc |= dalloc(ctx, &d->prow, npix + 1);
    rc |= dalloc(ctx, &d->h, npix);
    rc |= dalloc(ctx, &d->hits, npix);
    rc |= dalloc(ctx, &d->nnum, npix);
    rc |= dalloc(ctx, &d->part, 2 * (size_t)kPartMax);   // [0, kPartMax): p.q / dots, then r.r of the fused CG
    rc |= dalloc(ctx, &d->scal, 16);
    if (rc) { comap_destripe_destroy(d); return -2; }
    // ---- offset-major entries
    int64_t *cnt = nullptr;
    if (dalloc(ctx, &cnt, d->NO + 1)) { comap_destripe_destroy(d); return -2; }
    const unsigned gblocks = (unsigned)((d->NO + 3) / 4);
    launch_entries(L, gblocks, st, pix, w, tod, d->NO, 0, cnt, nullptr, nullptr, nullptr, d->ws, d->tw);
    COMAP_LAUNCH_CHECK(ctx);
    size_t tb = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cnt, d->orow, (int)(d->NO + 1), st);
    void *tmp = nullptr;
    COMAP_CHECK(ctx, hipMalloc(&tmp, tb));
    COMAP_CHECK(ctx, hipMemsetAsync(cnt + d->NO, 0, 8, st));
    COMAP_CHECK(ctx, hipcub::DeviceScan::ExclusiveSum(tmp, tb, cnt, d->orow, (int)(d->NO + 1), st));
    COMAP_CHECK(ctx, hipMemcpyAsync(&d->nnz, d->orow + d->NO, 8, hipMemcpyDeviceToHost, st));
    COMAP_CHECK(ctx, hipStreamSynchronize(st));
    (void)hipFree(tmp);
    (void)hipFree(cnt);
    rc |= dalloc(ctx, &d->opix, d->nnz);
    rc |= dalloc(ctx, &d->ow, d->nnz);
    if (rc) { comap_destripe_destroy(d); return -2; }
    launch_entries(L, gblocks, st, pix, w, tod, d->NO, 1, nullptr, d->orow, d->opix, d->ow, nullptr, nullptr);
    COMAP_LAUNCH_CHECK(ctx);
    // ---- pixel-major transpose (stable radix sort keeps offset order within a pixel)
    const int64_t sortn = std::max<int64_t>(d->nnz, N);
    int32_t *k0 = nullptr, *k1 = nullptr, *v0 = nullptr, *v1 = nullptr, *eoff = nullptr;
    rc |= dalloc(ctx, &k0, sortn); rc |= dalloc(ctx, &k1, sortn);
    rc |= dalloc(ctx, &v0, sortn); rc |= dalloc(ctx, &v1, sortn);
    rc |= dalloc(ctx, &eoff, d->nnz);
    if (rc) { comap_destripe_destroy(d); return -2; }
    int end_bit = 1;
    while ((1ll << end_bit) <= npix) ++end_bit;
    k_entry_keys<<<grid_for(d->NO), 256, 0, st>>>(d->orow, d->NO, d->opix, npix, k0, v0, eoff);
    COMAP_LAUNCH_CHECK(ctx);
    tb = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tb, k0, k1, v0, v1, (int)sortn, 0, end_bit, st);
    COMAP_CHECK(ctx, hipMalloc(&tmp, tb));
    COMAP_CHECK(ctx, hipcub::DeviceRadixSort::SortPairs(tmp, tb, k0, k1, v0, v1, (int)d->nnz, 0, end_bit, st));
    k_rowptr<<<grid_for(npix + 1), 256, 0, st>>>(k1, d->nnz, npix, d->prow);
    COMAP_LAUNCH_CHECK(ctx);
    COMAP_CHECK(ctx, hipMemcpyAsync(&d->nnzp, d->prow + npix, 8, hipMemcpyDeviceToHost, st));
    {
        std::vector<int64_t> ph(npix + 1);
        COMAP_CHECK(ctx, hipMemcpyAsync(ph.data(), d->prow, 8 * (size_t)(npix + 1), hipMemcpyDeviceToHost, st));
        COMAP_CHECK(ctx, hipStreamSynchronize(st));
        std::vector<int32_t> hr;
        for (int64_t q = 0; q < npix; ++q)
            if (ph[q + 1] > ph[q]) hr.push_back((int32_t)q);
        d->nh = (int64_t)hr.size();
        rc |= dalloc(ctx, &d->hrow, hr.size());
        if (!rc && !hr.empty())
            COMAP_CHECK(ctx, hipMemcpyAsync(d->hrow, hr.data(), 4 * hr.size(), hipMemcpyHostToDevice, st));
        COMAP_CHECK(ctx, hipStreamSynchronize(st));
    }
    rc |= dalloc(ctx, &d->poff, d->nnzp);
    rc |= dalloc(ctx, &d->pw, d->nnzp);
    if (rc) { comap_destripe_destroy(d); return -2; }
    k_pixel_entries<<<grid_for(d->nnzp), 256, 0, st>>>(v1, d->nnzp, eoff, d->ow, d->poff, d->pw);
    COMAP_LAUNCH_CHECK(ctx);
    // ---- sample-level maps (binValues order)
    k_sample_keys<<<grid_for(N), 256, 0, st>>>(pix, N, npix, k0, v0);
    COMAP_LAUNCH_CHECK(ctx);
    COMAP_CHECK(ctx, hipcub::DeviceRadixSort::SortPairs(tmp, tb, k0, k1, v0, v1, (int)N, 0, end_bit, st));
    k_sample_maps<<<grid_for(npix), 256, 0, st>>>(k1, v1, N, npix, w, tod, d->h, d->hits, d->nnum);
    COMAP_LAUNCH_CHECK(ctx);
    COMAP_CHECK(ctx, hipStreamSynchronize(st));
    (void)hipFree(tmp); (void)hipFree(k0); (void)hipFree(k1); (void)hipFree(v0); (void)hipFree(v1); (void)hipFree(eoff);
    *out = d;
    return 0;
}

extern "C" int comap_destripe_destroy(comap_destriper *d)
{
    if (!d) return 0;
    COMAP_DEVICE_GUARD(d->ctx);
    if (d->cs) (void)hipStreamSynchronize(d->cs);
    void *b[] = {d->orow, d->opix, d->ow, d->ws, d->tw, d->prow, d->poff, d->pw, d->h, d->hits, d->nnum, d->part, d->scal,
                 d->cg, d->flags, d->hrow};
    for (void *p : b)
        if (p) (void)hipFree(p);
    if (d->flags_host) (void)hipHostFree(d->flags_host);
    if (d->thr_host) (void)hipHostFree(d->thr_host);
    if (d->batch) (void)hipGraphExecDestroy(d->batch);
    if (d->ev) (void)hipEventDestroy(d->ev);
    if (d->cs) (void)hipStreamDestroy(d->cs);
    delete d;
    return 0;
}

extern "C" int64_t comap_destripe_n_offsets(const comap_destriper *d) { return d ? d->NO : -1; }

extern "C" int comap_destripe_nnz(const comap_destriper *d, int64_t *nnz_offset_major, int64_t *nnz_pixel_major)
{
    if (!d) return -1;
    if (nnz_offset_major) *nnz_offset_major = d->nnz;
    if (nnz_pixel_major) *nnz_pixel_major = d->nnzp;
    return 0;
}

extern "C" int comap_destripe_local_maps(comap_destriper *d, double *h, double *hits, double *naive_num)
{
    if (!d) return -1;
    COMAP_DEVICE_GUARD(d->ctx);
    comap_ctx *ctx = d->ctx;
    const size_t b = 8 * (size_t)d->npix;
    if (h) COMAP_CHECK(ctx, hipMemcpyAsync(h, d->h, b, hipMemcpyDeviceToDevice, ctx->stream));
    if (hits) COMAP_CHECK(ctx, hipMemcpyAsync(hits, d->hits, b, hipMemcpyDeviceToDevice, ctx->stream));
    if (naive_num) COMAP_CHECK(ctx, hipMemcpyAsync(naive_num, d->nnum, b, hipMemcpyDeviceToDevice, ctx->stream));
    return 0;
}

extern "C" int comap_destripe_bin(comap_destriper *d, const double *x, int32_t mode, double *num)
{
    if (!d || !x || !num) return -1;
    COMAP_DEVICE_GUARD(d->ctx);
    comap_ctx *ctx = d->ctx;
    launch_bin(d, ctx->stream, x, mode == 1 ? d->nnum : nullptr, nullptr, num, nullptr);
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}

extern "C" int comap_destripe_project(comap_destriper *d, const double *x, const double *num, const double *h,
                                      double *y, double *dot_out)
{
    if (!d || !num || !y) return -1;
    COMAP_DEVICE_GUARD(d->ctx);
    comap_ctx *ctx = d->ctx;
    const double *hh = h ? h : d->h;
    const bool want = dot_out && x;
    const unsigned pg = launch_project(d, ctx->stream, x, num, hh, y, want ? d->part : nullptr, nullptr);
    COMAP_LAUNCH_CHECK(ctx);
    if (want) {
        k_dot_final<<<1, 256, 0, ctx->stream>>>(d->part, (int)pg, dot_out, nullptr);
        COMAP_LAUNCH_CHECK(ctx);
    }
    return 0;
}

extern "C" int comap_destripe_dot(comap_destriper *d, const double *a, const double *b, double *out)
{
    if (!d || !a || !b || !out) return -1;
    COMAP_DEVICE_GUARD(d->ctx);
    return dot(d, a, b, out);
}

extern "C" int comap_destripe_cg_update(comap_destriper *d, const double *rr, const double *pq, double *x, double *r,
                                        const double *p, const double *q, double *rr_new)
{
    if (!d) return -1;
    COMAP_DEVICE_GUARD(d->ctx);
    comap_ctx *ctx = d->ctx;
    k_cg_update<<<kRedBlocks, 256, 0, ctx->stream>>>(rr, pq, x, r, p, q, d->NO, d->part, nullptr);
    COMAP_LAUNCH_CHECK(ctx);
    k_dot_final<<<1, 256, 0, ctx->stream>>>(d->part, kRedBlocks, rr_new, nullptr);
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}

extern "C" int comap_destripe_cg_direction(comap_destriper *d, const double *rr_new, const double *rr, double *p,
                                           const double *r)
{
    if (!d) return -1;
    COMAP_DEVICE_GUARD(d->ctx);
    comap_ctx *ctx = d->ctx;
    k_cg_direction<<<grid_for(d->NO), 256, 0, ctx->stream>>>(rr_new, rr, p, r, d->NO, nullptr);
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}

extern "C" int comap_destripe_div_map(comap_destriper *d, const double *num, const double *h, double *out)
{
    if (!d || !num || !out) return -1;
    COMAP_DEVICE_GUARD(d->ctx);
    comap_ctx *ctx = d->ctx;
    k_div_map<<<grid_for(d->npix), 256, 0, ctx->stream>>>(num, h ? h : d->h, d->npix, out);
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}

// ---------------------------------------------------------------- multi-rank CG pieces
// One CG iteration split at its three all-reduce points (map numerator, p.q,
// r.r), every kernel gated by the device stop flag so the host can queue a
// batch of iterations (with the collectives between the pieces) and check the
// flag once per batch.  scal: [0] rr0, [1] rr, [2] pq, [3] rr_new, [4] threshold.
extern "C" int comap_destripe_dist_bin(comap_destriper *d, const double *p, double *num, const int32_t *flags)
{
    if (!d || !p || !num || !flags) return -1;
    COMAP_DEVICE_GUARD(d->ctx);
    comap_ctx *ctx = d->ctx;
    launch_bin(d, ctx->stream, p, nullptr, nullptr, num, flags);
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}

extern "C" int comap_destripe_dist_project(comap_destriper *d, const double *p, const double *num, const double *h,
                                           double *q, double *scal, const int32_t *flags)
{
    if (!d || !p || !num || !h || !q || !scal || !flags) return -1;
    COMAP_DEVICE_GUARD(d->ctx);
    comap_ctx *ctx = d->ctx;
    const unsigned pg = launch_project(d, ctx->stream, p, num, h, q, d->part, flags);
    k_dot_final<<<1, 256, 0, ctx->stream>>>(d->part, (int)pg, scal + 2, flags);
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}

extern "C" int comap_destripe_dist_update(comap_destriper *d, double *scal, double *x, double *r, const double *p,
                                          const double *q, const int32_t *flags)
{
    if (!d || !scal || !x || !r || !p || !q || !flags) return -1;
    COMAP_DEVICE_GUARD(d->ctx);
    comap_ctx *ctx = d->ctx;
    k_cg_update<<<kRedBlocks, 256, 0, ctx->stream>>>(scal + 1, scal + 2, x, r, p, q, d->NO, d->part, flags);
    k_dot_final<<<1, 256, 0, ctx->stream>>>(d->part, kRedBlocks, scal + 3, flags);
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}

extern "C" int comap_destripe_dist_direction(comap_destriper *d, double *scal, double *p, const double *r,
                                             int32_t *flags)
{
    if (!d || !scal || !p || !r || !flags) return -1;
    COMAP_DEVICE_GUARD(d->ctx);
    comap_ctx *ctx = d->ctx;
    k_cg_direction<<<grid_for(d->NO), 256, 0, ctx->stream>>>(scal + 3, scal + 1, p, r, d->NO, flags);
    k_cg_check<<<1, 64, 0, ctx->stream>>>(scal, flags);
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}

// ---------------------------------------------------------------- device-resident CG
// One CG iteration (Destriper.py:85-152 with p == pb, r == rb) on the problem's own
// vectors; every kernel returns at once after the stop flag is set.
static void enqueue_iteration(comap_destriper *d, hipStream_t st)
{
    const int64_t NO = d->NO;
    double *x = d->cg, *r = x + NO, *p = r + NO, *q = p + NO, *num = q + NO;
    const int32_t *done = d->flags;
    // the bin writes the map m = (W p) / h itself, so the projection gathers one array
    launch_bin(d, st, p, nullptr, d->h, num, done, true);   // empty rows of num stay 0
    // 4 launches per iteration: the p.q / r.r finals and the stop test are folded into
    // the update and direction kernels (same arithmetic and order as k_dot_final + k_cg_check)
    const unsigned pg = launch_project(d, st, p, num, nullptr, q, d->part, done);
    k_cg_update_fused<<<kRedBlocks, 256, 0, st>>>(d->scal, d->part, (int)pg, x, r, p, q, NO, d->part + kPartMax,
                                                  done);
    k_cg_direction_fused<<<grid_for(NO), 256, 0, st>>>(d->scal, d->part + kPartMax, kRedBlocks, p, r, NO,
                                                       d->flags);
}

// CG state, stream and the kCgBatch-iteration graph, created on first use.
static int cg_setup(comap_destriper *d)
{
    if (d->batch) return 0;
    comap_ctx *ctx = d->ctx;
    if (!d->cg && (dalloc(ctx, &d->cg, 4 * (size_t)d->NO + (size_t)d->npix) || dalloc(ctx, &d->flags, 2))) return -2;
    if (!d->flags_host) COMAP_CHECK(ctx, hipHostMalloc((void **)&d->flags_host, 8, hipHostMallocDefault));
    if (!d->thr_host) COMAP_CHECK(ctx, hipHostMalloc((void **)&d->thr_host, 8, hipHostMallocDefault));
    if (!d->cs) COMAP_CHECK(ctx, hipStreamCreateWithFlags(&d->cs, hipStreamNonBlocking));
    if (!d->ev) COMAP_CHECK(ctx, hipEventCreateWithFlags(&d->ev, hipEventDisableTiming));
    hipGraph_t g = nullptr;
    COMAP_CHECK(ctx, hipStreamBeginCapture(d->cs, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < kCgBatch; ++i) enqueue_iteration(d, d->cs);
    COMAP_CHECK(ctx, hipStreamEndCapture(d->cs, &g));
    const hipError_t e = hipGraphInstantiate(&d->batch, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    COMAP_CHECK(ctx, e);
    return 0;
}

// Single-rank destriper_iteration: CG (one matvec per iteration) to threshold /
// niter, then the final maps (:419-451).  Iterations are queued kCgBatch at a
// time as one graph launch; a device-side stop flag makes the iterations after
// convergence no-ops, so the iterates and the count equal a per-iteration loop's.
extern "C" int comap_destripe_solve(comap_destriper *d, double threshold, int32_t niter, double *x, double *map,
                                    double *naive, double *weight, double *hits, int32_t *iters_out)
{
    if (!d || !x || niter < 0) return -1;
    COMAP_DEVICE_GUARD(d->ctx);
    comap_ctx *ctx = d->ctx;
    int rc = cg_setup(d);
    if (rc) return rc;
    hipStream_t st = d->cs;
    const int64_t NO = d->NO, np = d->npix;
    double *cx = d->cg, *r = cx + NO, *p = r + NO, *num = p + 2 * NO;
    // inputs were produced on the caller's stream
    COMAP_CHECK(ctx, hipEventRecord(d->ev, ctx->stream));
    COMAP_CHECK(ctx, hipStreamWaitEvent(st, d->ev, 0));
    d->thr_host[0] = threshold;
    COMAP_CHECK(ctx, hipMemcpyAsync(d->scal + 4, d->thr_host, 8, hipMemcpyHostToDevice, st));
    COMAP_CHECK(ctx, hipMemsetAsync(cx, 0, 8 * NO, st));
    COMAP_CHECK(ctx, hipMemsetAsync(num, 0, 8 * np, st));   // the CG bin writes only the non-empty rows
    COMAP_CHECK(ctx, hipMemsetAsync(d->flags, 0, 8, st));
    // b = op_Ax(tod, extend=False); r = p = b (x0 = 0); rr = rr0 = b.b
    launch_project(d, st, nullptr, d->nnum, d->h, r, nullptr, nullptr);
    COMAP_LAUNCH_CHECK(ctx);
    COMAP_CHECK(ctx, hipMemcpyAsync(p, r, 8 * NO, hipMemcpyDeviceToDevice, st));
    k_dot_part<<<kRedBlocks, 256, 0, st>>>(r, r, NO, d->part);
    k_dot_final<<<1, 256, 0, st>>>(d->part, kRedBlocks, d->scal, nullptr);
    COMAP_LAUNCH_CHECK(ctx);
    COMAP_CHECK(ctx, hipMemcpyAsync(d->scal + 1, d->scal, 8, hipMemcpyDeviceToDevice, st));
    COMAP_CHECK(ctx, hipMemcpyAsync(d->scal + 3, d->scal, 8, hipMemcpyDeviceToDevice, st));   // current rr (fused CG)
    d->flags_host[0] = d->flags_host[1] = 0;
    for (int enq = 0; enq < niter;) {
        const int k = std::min(kCgBatch, niter - enq);
        if (k == kCgBatch) {
            COMAP_CHECK(ctx, hipGraphLaunch(d->batch, st));
        } else {
            for (int i = 0; i < k; ++i) enqueue_iteration(d, st);
            COMAP_LAUNCH_CHECK(ctx);
        }
        enq += k;
        COMAP_CHECK(ctx, hipMemcpyAsync(d->flags_host, d->flags, 8, hipMemcpyDeviceToHost, st));
        COMAP_CHECK(ctx, hipStreamSynchronize(st));
        if (d->flags_host[0]) break;
    }
    if (iters_out) *iters_out = d->flags_host[1];
    COMAP_CHECK(ctx, hipMemcpyAsync(x, cx, 8 * NO, hipMemcpyDeviceToDevice, st));
    // final maps: map = (sum w tod - W x) / h ; naive = sum w tod / h
    if (map) {
        launch_bin(d, st, cx, d->nnum, nullptr, num, nullptr);
        k_div_map<<<grid_for(np), 256, 0, st>>>(num, d->h, np, map);
    }
    if (naive) k_div_map<<<grid_for(np), 256, 0, st>>>(d->nnum, d->h, np, naive);
    COMAP_LAUNCH_CHECK(ctx);
    if (weight) COMAP_CHECK(ctx, hipMemcpyAsync(weight, d->h, 8 * np, hipMemcpyDeviceToDevice, st));
    if (hits) COMAP_CHECK(ctx, hipMemcpyAsync(hits, d->hits, 8 * np, hipMemcpyDeviceToDevice, st));
    COMAP_CHECK(ctx, hipStreamSynchronize(st));
    return 0;
}
