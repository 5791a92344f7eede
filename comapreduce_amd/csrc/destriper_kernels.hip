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
// Off-map samples (negative pixel ids p >= -npix) are never binned but gather m[npix + p],
// numpy's index wrap in the reference's m[pointing] (Destriper.py:211; -1 reads the last
// pixel); ids < -npix are rejected as numpy raises there.  One CG iteration streams
// 2 nnz entries instead of 6 N samples; all reductions are fixed-order
// (deterministic).  The sample-level maps (weight map h, hits, naive
// numerator sum w tod) are summed per pixel in sample order after a stable
// radix sort, i.e. in exactly binValues' order (bit-exact on one rank).
//
// Bands.  run_destriper.py:146-189 solves the 4 sidebands one after the other
// on the SAME pointing (only tod and weights differ per band).  A problem here
// holds NB in {1, 2, 4} bands as one batched system: the index structure
// (offset rows, pixel ids, pixel-major transpose) is shared and every per-band
// quantity is interleaved band-fastest -- entry weights [nnz][NB], CG vectors
// [N/L][NB], maps [npix][NB] -- so one entry-index load and one 8 NB-byte
// gather serve all bands, and one launch sequence advances every band's CG.
// Each band keeps its own scalars and stop flag (its iterates and iteration
// count are those of a separate solve).  An offset that a band's data prep
// drops (all weights zero, COMAPData.py:550-568) is marked in the per-band
// keep mask: its weights are zero, so it adds exactly nothing to that band's
// operator, and its samples are left out of that band's hit map.
//
// Layout of the device scalars (k-major, so one collective sums NB values):
//   scal[0:NB] rr0, [NB:2NB] rr, [2NB:3NB] p.q, [3NB:4NB] rr_new, [4NB] threshold
//   flags[0] all bands stopped, [1] iterations while any band ran,
//   [2+b] band b stopped, [2+NB+b] band b's iterations
// (NB = 1 is the single-band layout rr0, rr, pq, rr_new, threshold / stop, iterations.)
#include "comap_internal.h"

#include <hipcub/hipcub.hpp>
#include <rocprim/device/device_radix_sort.hpp>

#include <cmath>
#include <type_traits>
#include <cstdlib>
#include <cstring>

struct comap_destriper {
    comap_ctx *ctx = nullptr;
    int64_t N = 0, NO = 0, npix = 0;
    int32_t L = 0;
    int32_t nb = 1;        // bands solved together (interleaved, band fastest)
    int64_t nnz = 0;       // offset-major entries (incl. off-map gathers)
    int64_t nnzp = 0;      // pixel-major entries (binned only)
    // offset-major
    int64_t *orow = nullptr;   // [NO+1]
    int32_t *opix = nullptr;   // [nnz]  pixel (-1 = off-map)
    double *ow = nullptr;      // [nnz][nb]
    double *ws = nullptr;      // [NO][nb] sum w
    double *tw = nullptr;      // [NO][nb] sum w tod
    // pixel-major
    int64_t *prow = nullptr;   // [npix+1]
    int32_t *poff = nullptr;   // [nnzp]
    double *pw = nullptr;      // [nnzp][nb]
    // count form (cf): every offset's non-zero sample weights in band b equal one value
    // wbar[o][b] (COMAP's weights are per (feed, band, file), cuts set 0), so an entry
    // stores the number of non-zero-weight samples per band (uint8) instead of the f64
    // sums: s_e = wbar_o c_e.  opix / poff + ocnt / pcnt replace ow / pw (4 + NB bytes per
    // entry instead of 4 + 8 NB); the bin gathers pt = wbar o x (written by the direction
    // kernel, or by k_scale), the projection multiplies its row sum by wbar_o.
    bool cf = false;
    // launch shapes (defaults: the measured best; COMAP_DS_BL / BU / PG / PU / PB override)
    int bin_lanes = 0;         // lanes per pixel row (0: by the mean row length)
    int bin_u = 4;             // entry loads in flight per bin lane
    int proj_lanes = 0;        // lanes per offset row (0: by L)
    int proj_u = 4;            // entry loads in flight per projection lane
    int64_t proj_blocks = 1024;   // projection grid cap (its p.q partials are re-summed by every update block)
    // comap_destripe_solve replays a captured graph of kCgBatch iterations only for small
    // problems, whose 4 kernels per iteration run shorter than their host enqueue; larger
    // ones enqueue eagerly (no capture: 0.4 ms at C4 that no replay won back)
    int cg_graph = -1;          // -1: by size (COMAP_DS_CGGRAPH=0 / 1 overrides)
    // sliced-ELLPACK copy of the offset-major rows for the projection (COMAP_DS_SELL): chunk c
    // = 64 consecutive offsets (one wave, lane = offset), padded to its longest row and stored
    // column-major -- entry j of lane l at sbase[c] + 64 j + l -- so a lane streams its row
    // with coalesced loads, no row-pointer load and no cross-lane reduction
    bool sell = false;
    bool walk = false;         // sample-level maps by the member-mask walk (set-up)
    int64_t nsell = 0;         // padded entries
    int64_t *sbase = nullptr;  // [NC + 1]
    int32_t *spix = nullptr;   // [nsell] pixel, -1 off-map, kSellPad padding
    void *sco = nullptr;       // [nsell][nb] counts (uint8) or weights (f64)
    uint8_t *ocnt = nullptr;   // [nnz][nb]
    uint8_t *pcnt = nullptr;   // [nnzp][nb]
    double *wbar = nullptr;    // [NO][nb]
    double *pt = nullptr;      // [NO][nb] scaled bin input (CG direction / scratch)
    // sample-level maps (local), [npix][nb]
    double *h = nullptr, *hits = nullptr, *nnum = nullptr;
    // reduction scratch
    double *part = nullptr;    // [2 nb kPartMax] block partials (band b at b kPartMax)
    double *scal = nullptr;    // [4 nb + 1] device scalars (layout above)
    // device-resident CG of comap_destripe_solve (fixed pointers: graph-replayable)
    double *cg = nullptr;          // [(4 NO + npix) nb]: x, r, p, q | num
    int32_t *flags = nullptr;      // [2 + 2 nb]
    int32_t *hrow = nullptr;       // [nh] pixel rows with entries (the CG bin skips empty rows)
    int64_t *hprow = nullptr;      // [nh + 1] their entry ranges: hprow[i] = prow[hrow[i]] (no empty row between)
    int64_t nh = 0;
    int32_t *perm = nullptr;       // [NO] internal offset position -> caller's offset (NULL: identity)
    int32_t *flags_host = nullptr; // pinned [2 + 2 nb]
    double *thr_host = nullptr;    // pinned [1 + 4 nb]: threshold, then a copy of scal's rr0 .. rr_new
    hipStream_t cs = nullptr;      // CG stream (graph capture needs a non-default stream)
    hipEvent_t ev = nullptr;
    hipGraphExec_t batch = nullptr;   // kCgBatch iterations
};

namespace {

constexpr int kRedBlocks = 256;   // dot-product grids (k_dot_part)
constexpr int kUpdBlocks = 1024;  // CG update grid cap: its r.r partials are re-summed by every direction block
constexpr int kProjBlocks = 1024; // k_ds_project grid cap: its p.q partials are re-summed by every update block
constexpr int kDirBlocks = 1024;  // CG direction grid cap
constexpr int kPartMax = 8192;     // >= every reduction grid below
constexpr int kCgBatch = 16;       // CG iterations per replayed graph (one host check per batch)
constexpr int64_t kSellMinOffsets = 131072;   // sliced-ELLPACK projection by default from this many offsets

typedef double d2v __attribute__((ext_vector_type(2)));

// Device-side CG stop flags: flags[0] (every band stopped) makes every kernel of the
// remaining enqueued iterations return at once, so iterations run as replayed
// hipGraph batches with one host round trip per batch; flags[2+b] freezes band b.
__device__ __forceinline__ bool cg_done(const int32_t *flags) { return flags && flags[0]; }
__device__ __forceinline__ bool band_stopped(const int32_t *flags, int b) { return flags && flags[2 + b]; }

// v[0..NB) = p[0..NB) (16-B loads when NB is even; p is 8 NB-byte aligned)
template <int NB>
__device__ __forceinline__ void ldb(const double *__restrict__ p, double (&v)[NB])
{
    if constexpr (NB % 2 == 0) {
#pragma unroll
        for (int b = 0; b < NB; b += 2) {
            const d2v t = *reinterpret_cast<const d2v *>(p + b);
            v[b] = t.x;
            v[b + 1] = t.y;
        }
    } else {
#pragma unroll
        for (int b = 0; b < NB; ++b) v[b] = p[b];
    }
}

template <int NB>
__device__ __forceinline__ void stb(double *__restrict__ p, const double (&v)[NB])
{
    if constexpr (NB % 2 == 0) {
#pragma unroll
        for (int b = 0; b < NB; b += 2) {
            d2v t;
            t.x = v[b];
            t.y = v[b + 1];
            *reinterpret_cast<d2v *>(p + b) = t;
        }
    } else {
#pragma unroll
        for (int b = 0; b < NB; ++b) p[b] = v[b];
    }
}

// Entry coefficients of NB bands: the f64 weight sums (full form) or the uint8
// non-zero-sample counts (count form, CF), as doubles.
template <int NB, bool CF>
__device__ __forceinline__ void ld_coef(const void *__restrict__ base, int64_t k, double (&a)[NB])
{
    if constexpr (CF) {
        const uint8_t *c = reinterpret_cast<const uint8_t *>(base) + k * NB;
        if constexpr (NB == 4) {
            const uint32_t v = *reinterpret_cast<const uint32_t *>(c);
#pragma unroll
            for (int b = 0; b < 4; ++b) a[b] = (double)((v >> (8 * b)) & 0xffu);
        } else if constexpr (NB == 2) {
            const uint32_t v = *reinterpret_cast<const uint16_t *>(c);
            a[0] = (double)(v & 0xffu);
            a[1] = (double)(v >> 8);
        } else {
            a[0] = (double)c[0];
        }
    } else {
        ldb<NB>(reinterpret_cast<const double *>(base) + k * NB, a);
    }
}

// One entry's coefficients held in registers between its load and its use (the bin's
// software pipeline): the count form keeps the packed uint8 counts (one dword for up to
// 4 bands), the full form the NB doubles.
template <int NB, bool CF>
struct Coef;
template <int NB>
struct Coef<NB, true> {
    uint32_t v = 0;
    __device__ __forceinline__ void load(const void *__restrict__ base, int64_t k)
    {
        const uint8_t *c = reinterpret_cast<const uint8_t *>(base) + k * NB;
        if constexpr (NB == 4) v = *reinterpret_cast<const uint32_t *>(c);
        else if constexpr (NB == 2) v = *reinterpret_cast<const uint16_t *>(c);
        else v = *c;
    }
    __device__ __forceinline__ double get(int b) const { return (double)((v >> (8 * b)) & 0xffu); }
};
template <int NB>
struct Coef<NB, false> {
    double v[NB] = {};
    __device__ __forceinline__ void load(const void *__restrict__ base, int64_t k)
    {
        ldb<NB>(reinterpret_cast<const double *>(base) + k * NB, v);
    }
    __device__ __forceinline__ double get(int b) const { return v[b]; }
};

// Inclusive prefix sum over the 64 lanes by DPP: row_shr 1 / 2 / 4 / 8 inside each 16-lane
// row (zeros shifted in), then row_bcast 15 / 31 carry the row totals into the later rows.
// Every lane must be active.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v)
{
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);   // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);   // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);   // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);   // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);   // row_bcast:15 -> rows 1, 3
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);   // row_bcast:31 -> rows 2, 3
    return v;
}

__device__ __forceinline__ double wave_sum(double v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Wave sums of V values per lane (V a power of two <= 64) by a reduce-scatter butterfly:
// the first log2 V steps exchange half of the remaining values (each lane keeps the half
// its lane bit selects), the rest reduce the single value left, so V sums cost V - 1 + 6 -
// log2 V exchanges instead of 6 V.  Afterwards x[0] holds value lane / (64 / V)'s total (a
// fixed order; a + b == b + a, so both lanes of a pair hold the same bits).
template <int V>
__device__ __forceinline__ void wave_sum_scatter(double (&x)[V], int lane)
{
    // (values held in named registers and selected as values: a select between two array
    // elements was turned into a lane-dependent index, i.e. v_cndmask chains over all V)
    static_assert(V == 2 || V == 4 || V == 8, "V");
    double y[V];
#pragma unroll
    for (int j = 0; j < V; ++j) y[j] = x[j];
    int h = V / 2, sft = 32;
    if constexpr (V >= 8) {
        const bool up = (lane & sft) != 0;
        const double s0 = up ? y[0] : y[4], s1 = up ? y[1] : y[5], s2 = up ? y[2] : y[6], s3 = up ? y[3] : y[7];
        const double k0 = up ? y[4] : y[0], k1 = up ? y[5] : y[1], k2 = up ? y[6] : y[2], k3 = up ? y[7] : y[3];
        y[0] = k0 + __shfl_xor(s0, sft, 64);
        y[1] = k1 + __shfl_xor(s1, sft, 64);
        y[2] = k2 + __shfl_xor(s2, sft, 64);
        y[3] = k3 + __shfl_xor(s3, sft, 64);
        h >>= 1;
        sft >>= 1;
    }
    if constexpr (V >= 4) {
        const bool up = (lane & sft) != 0;
        const double s0 = up ? y[0] : y[2], s1 = up ? y[1] : y[3];
        const double k0 = up ? y[2] : y[0], k1 = up ? y[3] : y[1];
        y[0] = k0 + __shfl_xor(s0, sft, 64);
        y[1] = k1 + __shfl_xor(s1, sft, 64);
        h >>= 1;
        sft >>= 1;
    }
    {
        const bool up = (lane & sft) != 0;
        const double s0 = up ? y[0] : y[1], k0 = up ? y[1] : y[0];
        y[0] = k0 + __shfl_xor(s0, sft, 64);
        sft >>= 1;
    }
    (void)h;
#pragma unroll
    for (int o = 32 / V; o > 0; o >>= 1) y[0] += __shfl_xor(y[0], o, 64);
    x[0] = y[0];
}

// v of lane `src` (wave-uniform) by two v_readlane
__device__ __forceinline__ double read_lane(double v, int src)
{
    const uint64_t u = __double_as_longlong(v);
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)u, src), hi = __builtin_amdgcn_readlane((uint32_t)(u >> 32), src);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// Fixed-order sum of n block partials by one 256-thread block (k_dot_final's order).
// Each thread adds part[tid], part[tid + 256], ... in that order; the loads are issued
// 8 at a time before the adds (a serial load -> add chain costs one L2 round trip per
// partial: ~40 us for 4 bands x 2k partials at C4, most of the CG update kernel).
__device__ __forceinline__ double block_final_sum(const double *__restrict__ part, int n, double *red)
{
    double acc = 0.0;
    constexpr int kB = 8;
    int i = threadIdx.x;
    for (; i + (kB - 1) * 256 < n; i += kB * 256) {
        double v[kB];
#pragma unroll
        for (int k = 0; k < kB; ++k) v[k] = part[i + k * 256];
#pragma unroll
        for (int k = 0; k < kB; ++k) acc += v[k];
    }
    for (; i < n; i += 256) acc += part[i];
    acc = wave_sum(acc);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    return (red[0] + red[1]) + (red[2] + red[3]);
}

// block_final_sum for NB bands at once (band b's partials at part + b kPartMax): the
// same per-band order and result, with every band's loads in flight together.
// red: 4 NB doubles.
template <int NB>
__device__ __forceinline__ void block_final_sums(const double *__restrict__ part, int n, double *red, double (&out)[NB],
                                                 int64_t stride = kPartMax)
{
    double acc[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[b] = 0.0;
    constexpr int kB = 4;
    int i = threadIdx.x;
    for (; i + (kB - 1) * 256 < n; i += kB * 256) {
        double v[NB][kB];
#pragma unroll
        for (int b = 0; b < NB; ++b)
#pragma unroll
            for (int k = 0; k < kB; ++k) v[b][k] = part[(int64_t)b * stride + i + k * 256];
#pragma unroll
        for (int b = 0; b < NB; ++b)
#pragma unroll
            for (int k = 0; k < kB; ++k) acc[b] += v[b][k];
    }
    for (; i < n; i += 256) {
#pragma unroll
        for (int b = 0; b < NB; ++b) acc[b] += part[(int64_t)b * stride + i];
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[b] = wave_sum(acc[b]);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int b = 0; b < NB; ++b) red[4 * b + (threadIdx.x >> 6)] = acc[b];
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < NB; ++b) out[b] = (red[4 * b] + red[4 * b + 1]) + (red[4 * b + 2] + red[4 * b + 3]);
}

// Partial slots [used, stride) of every band set to 0 (by one block).  The multi-rank
// partial buffers (stride kDistParts) are all-reduced in place, so a rank whose grid
// is smaller than another's must clear the slots it does not write each time.
template <int NB>
__device__ __forceinline__ void zero_tail(double *__restrict__ part, int64_t stride, int64_t used)
{
    for (int64_t t = used + threadIdx.x; t < stride; t += blockDim.x)
#pragma unroll
        for (int b = 0; b < NB; ++b) part[(int64_t)b * stride + t] = 0.0;
}

// block_partial of NB accumulators with one pair of barriers; band b's partial goes to
// part[b kPartMax] (same value as block_partial per band).  red: 4 NB doubles.
template <int NB>
__device__ __forceinline__ void block_partials(double (&acc)[NB], double *red, double *part, int64_t stride = kPartMax)
{
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[b] = wave_sum(acc[b]);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int b = 0; b < NB; ++b) red[4 * b + (threadIdx.x >> 6)] = acc[b];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int b = 0; b < NB; ++b)
            part[(int64_t)b * stride] = (red[4 * b] + red[4 * b + 1]) + (red[4 * b + 2] + red[4 * b + 3]);
    }
}

// ---------------------------------------------------------------- set-up (comap_destripe_create_bands)
// Processing order of the offsets.  In time order the offsets in flight at once
// cover the whole scan pattern, so the projection's map gathers (npix x 8 NB bytes,
// 7.4 MB for 4 bands at 480^2) miss the 4 MB XCD L2s.  Sorting offsets by the pixel
// of their first on-map sample makes concurrently processed offsets look at one band
// of map rows, and puts offsets that cross the same pixels next to each other in the
// CG vectors (the bin's x gathers).  Key: that pixel (npix when the offset is all
// off-map); a stable sort keeps time order among equal keys.
// (one wave per offset: its pixels by coalesced loads, the first on-map one by a ballot;
// a thread per offset walked an off-map offset's L pixels one dependent load at a time)
__global__ void __launch_bounds__(256) k_offset_keys(const int32_t *__restrict__ pix, int64_t NO, int L, int64_t npix,
                                                     int32_t *__restrict__ key, int32_t *__restrict__ val)
{
    const int lane = threadIdx.x & 63;
    for (int64_t o = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); o < NO; o += (int64_t)gridDim.x * 4) {
        int32_t k = (int32_t)npix;
        if (!pix) {                 // keys given by the caller: the sort's values only
            if (lane == 0) val[o] = (int32_t)o;
            continue;
        }
        for (int j0 = 0; j0 < L; j0 += 64) {
            const int j = j0 + lane;
            const int32_t p = j < L ? pix[o * L + j] : -1;
            const unsigned long long v = __ballot(p >= 0);
            if (v) {
                k = __shfl(p, __ffsll((long long)v) - 1, 64);
                break;
            }
        }
        if (lane == 0) {
            key[o] = k;
            val[o] = (int32_t)o;
        }
    }
}

__global__ void k_iota32(int32_t *__restrict__ v, int64_t n)
{
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        v[i] = (int32_t)i;
}

// Member-mask walk: a kept entry's slot record, written by the count pass at slot
// k L + r (offset k's r-th entry) -- pixel, packed per-band non-zero counts, member mask
// (sample j of the offset = bit j) -- one 16-B-aligned gather for the sample walk
template <int K>
struct alignas(16) SlotRec {
    int32_t pix;
    uint32_t cnt;
    uint64_t mask[K];
};
static_assert(sizeof(SlotRec<1>) == 16 && sizeof(SlotRec<2>) == 32 && sizeof(SlotRec<4>) == 48, "SlotRec");

// Orders a wave's LDS writes before its later LDS reads by other lanes (and reads before
// later overwrites) where each wave owns its LDS region: one wave's LDS operations execute
// in issue order, so only the compiler must keep them in place.  A workgroup-scope fence
// would also wait for every global load and store the wave has in flight (s_waitcnt
// vmcnt(0)): the next chunk's prefetched loads and the previous chunk's stores.
__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Offset rows of the sparse operator, one wave per row k (offset o = perm[k]): lane l
// holds samples l, l + 64, ... (K per lane, L <= 64 K).  The distinct pixels of the
// offset are found in first-occurrence order by a leader loop (the first pending
// sample leads, one ballot per chunk collects every sample with its pixel), so the
// work is one short scalar loop per distinct pixel instead of an L x L compare.  The
// group's head lane then sums its samples' weights per band in sample order (the
// reference's binValues order within the offset; the offset's rows are L1-resident
// after the coalesced loads).  An entry is kept when any band's sum is non-zero.
//   FILL = false: cnt[k] (kept entries), ws / tw (sum w, sum w tod per band: lane
//                 order, then a fixed butterfly), and per sample the sort key of the
//                 sample-level maps (pixel, npix when not binned), its index, and the
//                 packed payload {w_b, tod_b w_b} [N][2 NB] (the product rounded, as
//                 binValues(weights = tod * w) rounds it).  The row's kept entries
//                 also go to slots [k L, k L + cnt[k]) of eval (pixel) / eoff (packed
//                 uint8 counts), in entry order: the count form's fill is then a
//                 compaction (k_ds_compact_cf) instead of a second leader loop.
//   FILL = true:  the row's entries at orow[k]: pixel (-1 = off-map), weights, and the
//                 pixel-major transpose's key / entry id / row.
// w, tod: band-major [NB][N].
template <int K, int NB, bool FILL, bool CF>
__global__ void __launch_bounds__(256) k_ds_rows(const int32_t *__restrict__ pix, const double *__restrict__ w,
                                                 const double *__restrict__ tod, int64_t N, int64_t NO, int L,
                                                 int64_t npix, const int32_t *__restrict__ perm,
                                                 int64_t *__restrict__ cnt, double *__restrict__ ws,
                                                 double *__restrict__ tw, double *__restrict__ payload,
                                                 int32_t *__restrict__ skey, int32_t *__restrict__ sval,
                                                 double *__restrict__ wbar, int32_t *__restrict__ nonuni,
                                                 const int64_t *__restrict__ orow, int32_t *__restrict__ opix,
                                                 double *__restrict__ ow, uint8_t *__restrict__ ocnt,
                                                 int32_t *__restrict__ ekey, int32_t *__restrict__ eval,
                                                 int32_t *__restrict__ eoff, uint64_t *__restrict__ epay,
                                                 SlotRec<K> *__restrict__ srec, uint32_t *__restrict__ hextra,
                                                 const uint8_t *__restrict__ keep, int32_t *__restrict__ nonfin)
{
#pragma clang fp contract(off)
    const int lane = threadIdx.x & 63;
    constexpr int32_t kNone = INT32_MIN;    // lanes past the offset's end (real pixels are >= -1)
    // the offset's weights, staged in LDS: the group sums below read their members from
    // here instead of one dependent global load per member (the count pass took 3.2 ms at
    // C5 with 4 bands, 80 % of its wave cycles waiting)
    __shared__ double wsh[4][K * 64 * NB];
    double *wl = wsh[threadIdx.x >> 6];
    // waves walk offsets k, k + nw, ... (grid-stride; the launch covers every offset
    // once by default -- a persistent grid that loaded the next offset during the current
    // one's leader loop took 100+ VGPRs, half the occupancy, and was no faster, r04z)
    const int64_t nw = (int64_t)gridDim.x * 4;
    int64_t k = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    int32_t qn[K];
    double wn[K][NB], tn[K][NB];
    auto fetch = [&](int64_t kk) {
        const int64_t bs = (perm ? (int64_t)perm[kk] : kk) * L;
#pragma unroll
        for (int m = 0; m < K; ++m) {
            const int j = lane + 64 * m;
            qn[m] = j < L ? pix[bs + j] : kNone;
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                wn[m][b] = j < L ? w[(int64_t)b * N + bs + j] : 0.0;
                if constexpr (!FILL) tn[m][b] = j < L ? tod[(int64_t)b * N + bs + j] : 0.0;
            }
        }
    };
    for (; k < NO; k += nw) {
    fetch(k);
    const int64_t o = perm ? (int64_t)perm[k] : k;
    const int64_t base = o * L;
    int32_t q[K];
    unsigned long long rem[K];
    double ti[K][NB];
#pragma unroll
    for (int m = 0; m < K; ++m) {
        q[m] = qn[m];
        rem[m] = __ballot(lane + 64 * m < L);
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            if constexpr (FILL) wl[(64 * m + lane) * NB + b] = wn[m][b];
            else ti[m][b] = tn[m][b];
        }
    }
    // (the fill pass reads group members' weights from LDS; the count pass stages them only
    // for an offset whose weights fail the count-form test, below)
    if constexpr (FILL) wave_lds_sync();
    // leader loop: head lanes and their members (per chunk of the leader)
    bool head[K];
    unsigned long long mem[K][K];
#pragma unroll
    for (int m = 0; m < K; ++m) {
        head[m] = false;
#pragma unroll
        for (int c = 0; c < K; ++c) mem[m][c] = 0ull;
    }
    if constexpr (K == 1) {
        // one sample per lane: the groups by an LDS hash table instead of the leader loop's
        // ~30 dependent readlane / ballot rounds per offset -- every lane inserts its pixel
        // (linear probing, compare-and-swap), the slot keeps the smallest lane (the first
        // occurrence: the group's head, as the leader loop picks it) and the OR of the
        // members' lane bits.  Same heads, same masks.
        constexpr int kSlots = 128;
        constexpr int32_t kEmpty = INT32_MIN + 1;
        __shared__ int32_t hkey[4][kSlots], hmin[4][kSlots];
        __shared__ unsigned long long hmsk[4][kSlots];
        int32_t *hk = hkey[threadIdx.x >> 6], *hm = hmin[threadIdx.x >> 6];
        unsigned long long *hb = hmsk[threadIdx.x >> 6];
#pragma unroll
        for (int z = lane; z < kSlots; z += 64) {
            hk[z] = kEmpty;
            hm[z] = 64;
            hb[z] = 0ull;
        }
        wave_lds_sync();
        const bool valid = lane < L;
        int slot = (int)(((uint32_t)q[0] * 2654435761u) >> 25);
        if (valid) {
            for (;;) {
                const int32_t old = atomicCAS(&hk[slot], kEmpty, q[0]);
                if (old == kEmpty || old == q[0]) break;
                slot = (slot + 1) & (kSlots - 1);
            }
            atomicMin(&hm[slot], lane);
            atomicOr(&hb[slot], 1ull << lane);
        }
        wave_lds_sync();
        head[0] = valid && hm[slot] == lane;
        mem[0][0] = head[0] ? hb[slot] : 0ull;
    } else {
#pragma unroll
    for (int m = 0; m < K; ++m) {
        while (rem[m]) {
            // the leader's pixel by v_readlane (rem is wave-uniform): no LDS round trip
            // (ds_bpermute) on this loop's dependent chain
            const int ld = __builtin_amdgcn_readfirstlane(__ffsll((long long)rem[m]) - 1);
            const int32_t pl = __builtin_amdgcn_readlane(q[m], ld);
            unsigned long long mm[K];
#pragma unroll
            for (int c = 0; c < K; ++c) {
                mm[c] = c < m ? 0ull : __ballot(q[c] == pl);
                rem[c] &= ~mm[c];
            }
            if (lane == ld) {
                head[m] = true;
#pragma unroll
                for (int c = 0; c < K; ++c) mem[m][c] = mm[c];
            }
        }
    }
    }   // K > 1: the leader loop
    // count pass: the count-form test first -- per band, every non-zero weight finite and
    // equal to the first one (ballot + readlane) -- with the non-zero masks
    double wi[K][NB], refb[NB];
    unsigned long long nzm[NB][K];
    bool uni = true;
    if constexpr (!FILL) {
#pragma unroll
        for (int m = 0; m < K; ++m)
#pragma unroll
            for (int b = 0; b < NB; ++b) wi[m][b] = wn[m][b];
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            double ref = 0.0;
            bool found = false, bad = false;
#pragma unroll
            for (int m = 0; m < K; ++m) {
                nzm[b][m] = __ballot(wi[m][b] != 0.0);
                if (!found && nzm[b][m]) {
                    found = true;
                    ref = read_lane(wi[m][b], __ffsll((long long)nzm[b][m]) - 1);
                }
            }
#pragma unroll
            for (int m = 0; m < K; ++m) {
                const double v = wi[m][b];
                bad |= v != 0.0 && (!isfinite(v) || v != ref);
            }
            refb[b] = ref;
            uni &= __ballot(bad) == 0ull;
        }
        if (!uni) {      // wave-uniform: the group sums below read members' weights
#pragma unroll
            for (int m = 0; m < K; ++m)
#pragma unroll
                for (int b = 0; b < NB; ++b) wl[(64 * m + lane) * NB + b] = wi[m][b];
            wave_lds_sync();
        }
    }
    // per head: the group's in-order weight sums per band (and, for the count form, its
    // number of non-zero-weight samples).  A uniform offset in the count pass needs only
    // the counts (its group sums are count x weight: non-zero iff the count is), which are
    // popcounts of member mask & non-zero mask -- no per-member loop
    double gs[K][NB];
    int gc[K][NB];
    bool keepe[K];
#pragma unroll
    for (int m = 0; m < K; ++m) {
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            gs[m][b] = 0.0;
            gc[m][b] = 0;
        }
        if (!FILL && uni) {
            bool any = false;
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                int n = 0;
#pragma unroll
                for (int c = 0; c < K; ++c) n += __popcll(mem[m][c] & nzm[b][c]);
                gc[m][b] = n;
                any |= n != 0;
            }
            keepe[m] = head[m] && any;
            continue;
        }
        if (head[m]) {
            // members in sample order, all bands per member (one NB-wide LDS read each);
            // every band's sum keeps the member order
#pragma unroll
            for (int c = 0; c < K; ++c)
                for (unsigned long long bits = mem[m][c]; bits; bits &= bits - 1) {
                    const double *src = wl + (64 * c + (__ffsll((long long)bits) - 1)) * NB;
                    double v[NB];
#pragma unroll
                    for (int b = 0; b < NB; ++b) v[b] = src[b];
#pragma unroll
                    for (int b = 0; b < NB; ++b) {
                        gs[m][b] += v[b];
                        gc[m][b] += v[b] != 0.0;
                    }
                }
        }
        bool any = false;
#pragma unroll
        for (int b = 0; b < NB; ++b) any |= gs[m][b] != 0.0;
        keepe[m] = head[m] && any;
    }
    if constexpr (!FILL) {
        int64_t c0 = 0;
#pragma unroll
        for (int m = 0; m < K; ++m) c0 += __popcll(__ballot(keepe[m]));
        bool nf = false;
#pragma unroll
        for (int m = 0; m < K; ++m) {
            const int j = lane + 64 * m;
            if (j < L) {
                const int64_t i = base + j;
                if (payload && srec) {
                    // member-mask walk: (tod w) per band, sample-major (NB doubles a sample)
                    // in the internal offset order (slot k L + j), so the walk needs no perm
                    double pt[NB];
#pragma unroll
                    for (int b = 0; b < NB; ++b) pt[b] = ti[m][b] * wi[m][b];
                    stb<NB>(payload + (k * L + j) * NB, pt);
                } else if (payload) {
                    double pl[2 * NB];
#pragma unroll
                    for (int b = 0; b < NB; ++b) { pl[b] = wi[m][b]; pl[NB + b] = ti[m][b] * wi[m][b]; }
                    stb<2 * NB>(payload + i * 2 * NB, pl);
                    skey[i] = (q[m] >= 0 && q[m] < npix) ? q[m] : (int32_t)npix;
                    sval[i] = (int32_t)i;
                }
#pragma unroll
                for (int b = 0; b < NB; ++b) nf |= !isfinite(ti[m][b]);
            }
        }
        // flags[1]: a pixel index >= npix or < -npix (the caller's error: numpy's m[pointing]
        // raises IndexError there; a negative id marks an unbinned sample that reads m[npix + p])
        if (nonfin) {
            bool ob = false;
#pragma unroll
            for (int m = 0; m < K; ++m) ob |= q[m] != kNone && (q[m] >= npix || q[m] < -npix);
            if (__ballot(ob) && lane == 0) nonfin[1] = 1;
        }
        // member-mask walk (no payload): hits of the groups that hold no entry (every weight
        // zero) by integer adds -- order-free, exact -- and a flag for non-finite tod, which
        // such groups would carry into the naive numerator (the set-up then takes the
        // payload walk, which reproduces that)
        if (srec) {
            if (nonfin && __ballot(nf) && lane == 0) nonfin[0] = 1;
#pragma unroll
            for (int m = 0; m < K; ++m)
                if (head[m] && !keepe[m] && q[m] >= 0 && q[m] < npix) {
                    uint32_t cnt_m = 0;
#pragma unroll
                    for (int c = 0; c < K; ++c) cnt_m += (uint32_t)__popcll(mem[m][c]);
#pragma unroll
                    for (int b = 0; b < NB; ++b)
                        if (!keep || keep[(int64_t)b * NO + o]) atomicAdd(hextra + (int64_t)q[m] * NB + b, cnt_m);
                }
        }
        // per band: the offset's sums (lane order, then wave_sum_scatter's fixed butterfly) and
        // the count-form test's result (ballot + readlane above instead of two more 6-step
        // reductions per band: most of the count pass's LDS-pipe time was 4 x 4 bpermute
        // butterflies, r04w)
        if (!uni && lane == 0) nonuni[0] = 1;
        double red[2 * NB];
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            double sw = 0.0, st = 0.0;
#pragma unroll
            for (int m = 0; m < K; ++m) {
                sw += wi[m][b];
                if (lane + 64 * m < L) st = fma(wi[m][b], ti[m][b], st);   // fused, as before the rewrite
            }
            red[2 * b] = sw;
            red[2 * b + 1] = st;
            if (lane == 0) wbar[k * NB + b] = refb[b];
        }
        wave_sum_scatter<2 * NB>(red, lane);
        if ((lane & (64 / (2 * NB) - 1)) == 0) {
            const int idx = lane / (64 / (2 * NB));           // value held: band idx / 2, sum idx % 2
            (idx & 1 ? tw : ws)[k * NB + (idx >> 1)] = red[0];
        }
        if (lane == 0) cnt[k] = c0;
        if (eval || srec) {
            int64_t r0 = k * L;
#pragma unroll
            for (int m = 0; m < K; ++m) {
                const unsigned long long bm = __ballot(keepe[m]);
                if (keepe[m]) {
                    const int64_t si = r0 + __popcll(bm & ((1ull << lane) - 1ull));
                    uint32_t pk = 0;
#pragma unroll
                    for (int b = 0; b < NB; ++b) pk |= (uint32_t)(gc[m][b] & 255) << (8 * b);
                    if (srec) {
                        SlotRec<K> rc;
                        rc.pix = q[m];
                        rc.cnt = pk;
#pragma unroll
                        for (int c = 0; c < K; ++c) rc.mask[c] = mem[m][c];
                        srec[si] = rc;
                    } else {
                        eval[si] = q[m];
                        eoff[si] = (int32_t)pk;
                    }
                }
                r0 += __popcll(bm);
            }
        }
    } else {
        int64_t e = orow[k];
#pragma unroll
        for (int m = 0; m < K; ++m) {
            const unsigned long long bm = __ballot(keepe[m]);
            if (keepe[m]) {
                const int64_t ei = e + __popcll(bm & ((1ull << lane) - 1ull));
                opix[ei] = q[m];
                // (the count form's fill is k_ds_compact_cf over the count pass's slots)
#pragma unroll
                for (int b = 0; b < NB; ++b) ow[ei * NB + b] = gs[m][b];
                ekey[ei] = (q[m] >= 0 && q[m] < npix) ? q[m] : (int32_t)npix;
                eval[ei] = (int32_t)ei;
                eoff[ei] = (int32_t)k;
            }
            e += __popcll(bm);
        }
    }
    }   // offsets of this wave
}

// Count-form fill: row k's kept entries, left by the count pass in slots
// [k L, k L + cnt_k) (pixel, packed uint8 counts per band), copied to the CSR rows at
// orow[k] with the transpose's sort pairs (pixel key, offset << 32 | counts) -- the
// same entries, in the same order, as the leader-loop fill pass wrote (1.2 ms of the
// C5 4-band set-up, r03l).  One wave per row.
template <int NB>
__global__ void __launch_bounds__(256) k_ds_compact_cf(const int64_t *__restrict__ orow, int64_t NO, int L,
                                                       int64_t npix, const int32_t *__restrict__ spx,
                                                       const int32_t *__restrict__ spk, int32_t *__restrict__ opix,
                                                       uint8_t *__restrict__ ocnt, int32_t *__restrict__ ekey,
                                                       uint64_t *__restrict__ epay)
{
    const int lane = threadIdx.x & 63;
    const int64_t k = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (k >= NO) return;
    const int64_t e0 = orow[k], c = orow[k + 1] - e0;
    for (int64_t r = lane; r < c; r += 64) {
        const int32_t q = spx[k * L + r];
        const uint32_t pk = (uint32_t)spk[k * L + r];
        const int64_t ei = e0 + r;
        opix[ei] = q;
        if constexpr (NB == 4) {
            *reinterpret_cast<uint32_t *>(ocnt + ei * 4) = pk;
        } else if constexpr (NB == 2) {
            *reinterpret_cast<uint16_t *>(ocnt + ei * 2) = (uint16_t)pk;
        } else {
            ocnt[ei] = (uint8_t)pk;
        }
        epay[ei] = ((uint64_t)(uint32_t)k << 32) | pk;
        ekey[ei] = (q >= 0 && q < npix) ? q : (int32_t)npix;
    }
}

template <int NB, bool FILL, bool CF>
void launch_rows(int L, hipStream_t st, const int32_t *pix, const double *w, const double *tod, int64_t N,
                 int64_t NO, int64_t npix, const int32_t *perm, int64_t *cnt, double *ws, double *tw, double *payload,
                 int32_t *skey, int32_t *sval, double *wbar, int32_t *nonuni, const int64_t *orow, int32_t *opix,
                 double *ow, uint8_t *ocnt, int32_t *ekey, int32_t *eval, int32_t *eoff, uint64_t *epay = nullptr,
                 void *srec = nullptr, uint32_t *hextra = nullptr, const uint8_t *keep = nullptr,
                 int32_t *nonfin = nullptr)
{
    // k_ds_rows' grid: COMAP_DS_RB blocks at most (default: one offset per wave)
    static const int64_t cap = [] {
        const char *v = getenv("COMAP_DS_RB");
        const int64_t x = v ? atoll(v) : 0;
        return x >= 256 && x <= (1 << 20) ? x : (int64_t)(1 << 20);
    }();
    const unsigned blocks = (unsigned)std::min<int64_t>((NO + 3) / 4, cap);
#define COMAP_ROWS(K) k_ds_rows<K, NB, FILL, CF><<<blocks, 256, 0, st>>>(pix, w, tod, N, NO, L, npix, perm, cnt, ws, \
                                                                          tw, payload, skey, sval, wbar, nonuni, orow, \
                                                                          opix, ow, ocnt, ekey, eval, eoff, epay, \
                                                                          (SlotRec<K> *)srec, hextra, keep, nonfin)
    if (L <= 64) COMAP_ROWS(1);
    else if (L <= 128) COMAP_ROWS(2);
    else COMAP_ROWS(4);
#undef COMAP_ROWS
}

// x_out[perm[k]] = x[k] per band (internal offset order -> the caller's)
template <int NB>
__global__ void k_unpermute(const double *__restrict__ x, const int32_t *__restrict__ perm, int64_t NO,
                            double *__restrict__ out)
{
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < NO; k += (int64_t)gridDim.x * blockDim.x) {
        double v[NB];
        ldb<NB>(x + k * NB, v);
        stb<NB>(out + (int64_t)perm[k] * NB, v);
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

// Stable sort of int32 (key, value) pairs on key bits [0, end_bit): nine = rocprim's onesweep
// with 9-bit digits (match-based ranking: 512 buckets do not fit the basic rank's LDS) and
// no merge-sort path -- for the spatial offset sort, 18-bit pixel keys of 547 k offsets in
// 2 passes (63 us) instead of hipcub's ~20 block-merge kernels (131 us) at C5.  The
// transpose (15.4 M pairs) stays on hipcub's 8-bit onesweep: 410 us in 3 passes against
// 537 us in 2 with the match ranking (r04zr).  Keys are non-negative.
using Sort9Config = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<256, 12>, rocprim::kernel_config<256, 12>, 9,
                                        rocprim::block_radix_rank_algorithm::match>,
    0>;

// (rocprim onesweep with 8-bit digits at 256 x 16 / 256 x 8 / 256 x 20 threads x items ran
// the transpose in 1.52 / 2.92 / 1.29 ms against hipcub's 0.43, r04ts: removed)
hipError_t sort_pairs_i32(bool nine, void *tmp, size_t &bytes, const int32_t *kin, int32_t *kout,
                          const int32_t *vin, int32_t *vout, int64_t n, int end_bit, hipStream_t st)
{
    if (nine)
        return rocprim::radix_sort_pairs<Sort9Config>(tmp, bytes, kin, kout, vin, vout, (unsigned)n, 0u,
                                                      (unsigned)end_bit, st);
    return hipcub::DeviceRadixSort::SortPairs(tmp, bytes, kin, kout, vin, vout, (int)n, 0, end_bit, st);
}

// row[p] = first sorted position with key >= p, p in [0, npix]
__global__ void k_rowptr(const int32_t *__restrict__ skey, int64_t n, int64_t npix, int64_t *__restrict__ row)
{
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p <= npix; p += (int64_t)gridDim.x * blockDim.x)
        row[p] = lb32(skey, n, p);
}

// The set-up's first host read-back in one piece: nnz, the SELL slot count, the count-form
// and tod / pixel-range flags (four pageable copies cost ~20 us of idle GPU each)
__global__ void k_setup_sizes(const int64_t *__restrict__ orow, int64_t NO, const int64_t *__restrict__ sbase,
                              int64_t NCs, const int32_t *__restrict__ nonuni, const int32_t *__restrict__ flags,
                              int64_t *__restrict__ out)
{
    if (threadIdx.x == 0) {
        out[0] = orow[NO];
        out[1] = sbase ? sbase[NCs] : 0;
        out[2] = nonuni[0];
        out[3] = flags[0];
        out[4] = flags[1];
    }
}

// nat0[k] = orow_nat[perm[k]]: each internal row's first slot in the caller's-order entry
// array, gathered once so the compaction's rows need no dependent perm -> orow_nat load
__global__ void k_nat_base(const int64_t *__restrict__ orow_nat, const int32_t *__restrict__ perm, int64_t NO,
                           int64_t *__restrict__ nat0)
{
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < NO; k += (int64_t)gridDim.x * blockDim.x)
        nat0[k] = orow_nat[perm ? (int64_t)perm[k] : k];
}

// cnt_nat[perm[k]] = cnt[k]: the offsets' kept-entry counts in the caller's offset order
__global__ void k_cnt_natural(const int64_t *__restrict__ cnt, const int32_t *__restrict__ perm, int64_t NO,
                              int64_t *__restrict__ cnt_nat)
{
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k <= NO; k += (int64_t)gridDim.x * blockDim.x)
        cnt_nat[k < NO ? (perm ? (int64_t)perm[k] : k) : NO] = k < NO ? cnt[k] : 0;
}

// kint[k] = bit b set when band b keeps offset perm[k] (keep [nb][NO] in the caller's
// offset order): the sample walk reads one byte per entry by its internal offset k
__global__ void k_keep_bits(const uint8_t *__restrict__ keep, const int32_t *__restrict__ perm, int64_t NO, int nb,
                            uint8_t *__restrict__ kint)
{
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < NO; k += (int64_t)gridDim.x * blockDim.x) {
        const int64_t o = perm ? (int64_t)perm[k] : k;
        uint32_t m = 0;
        for (int b = 0; b < nb; ++b) m |= (uint32_t)(keep[(int64_t)b * NO + o] != 0) << b;
        kint[k] = (uint8_t)m;
    }
}

// Count-form fill for the member-mask walk: row k's kept entries from the count pass's slots
// into the CSR rows (pixel, packed counts), and the transpose's sort pairs (pixel key, slot
// k L + r: the entry's walk record) in the caller's offset order (row k's first slot there:
// orow_nat[perm[k]], or orow_nat[k] when perm is NULL -- the set-up passes k_nat_base's
// gathered bases), so the stable
// sort by pixel leaves each pixel's entries in sample order -- the order binValues adds
// them in.  16 lanes per row (rows hold ~30 entries; a wave per row waited on its loads:
// 0.6 ms at C5).
template <int NB, int K>
__global__ void __launch_bounds__(256) k_ds_compact_walk(const int64_t *__restrict__ orow,
                                                         const int64_t *__restrict__ orow_nat,
                                                         const int32_t *__restrict__ perm, int64_t NO, int L,
                                                         int64_t npix, const SlotRec<K> *__restrict__ srec,
                                                         int32_t *__restrict__ opix, uint8_t *__restrict__ ocnt,
                                                         int32_t *__restrict__ ekey, int32_t *__restrict__ eval)
{
    const int sub = threadIdx.x & 15;
    const int64_t k = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
    if (k >= NO) return;
    const int64_t o = perm ? (int64_t)perm[k] : k;
    const int64_t e0 = orow[k], c = orow[k + 1] - e0, n0 = orow_nat[o];
    for (int64_t r = sub; r < c; r += 16) {
        const int32_t q = srec[k * L + r].pix;
        const uint32_t pk = srec[k * L + r].cnt;
        const int64_t ei = e0 + r;
        opix[ei] = q;
        if constexpr (NB == 4) {
            *reinterpret_cast<uint32_t *>(ocnt + ei * 4) = pk;
        } else if constexpr (NB == 2) {
            *reinterpret_cast<uint16_t *>(ocnt + ei * 2) = (uint16_t)pk;
        } else {
            ocnt[ei] = (uint8_t)pk;
        }
        ekey[n0 + r] = (q >= 0 && q < npix) ? q : (int32_t)npix;
        eval[n0 + r] = (int32_t)(k * L + r);
    }
}

// pixel-major entries: sorted position k < nnzp (= prow[npix], read on the device) takes
// offset-major entry sval[k] (entries of one pixel come from spatially adjacent rows)
template <int NB>
__global__ void k_pixel_entries(const int32_t *__restrict__ sval, const int64_t *__restrict__ nnzp_dev,
                                const int32_t *__restrict__ eoff, const double *__restrict__ ow,
                                const uint8_t *__restrict__ ocnt, int32_t *__restrict__ poff, double *__restrict__ pw,
                                uint8_t *__restrict__ pcnt)
{
    const int64_t nnzp = *nnzp_dev;
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < nnzp; k += (int64_t)gridDim.x * blockDim.x) {
        const int32_t e = sval[k];
        poff[k] = eoff[e];
        if (ocnt) {
#pragma unroll
            for (int b = 0; b < NB; ++b) pcnt[k * NB + b] = ocnt[(int64_t)e * NB + b];
        } else {
            double v[NB];
            ldb<NB>(ow + (int64_t)e * NB, v);
            stb<NB>(pw + k * NB, v);
        }
    }
}

// count form: pixel-major entries straight from the sorted (offset << 32 | counts) values
template <int NB>
__global__ void k_pixel_entries_cf(const uint64_t *__restrict__ pay, const int64_t *__restrict__ nnzp_dev,
                                   int32_t *__restrict__ poff, uint8_t *__restrict__ pcnt)
{
    const int64_t nnzp = *nnzp_dev;
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < nnzp; k += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t v = pay[k];
        poff[k] = (int32_t)(v >> 32);
        const uint32_t c = (uint32_t)v;
        if constexpr (NB == 4) *reinterpret_cast<uint32_t *>(pcnt + k * 4) = c;
        else if constexpr (NB == 2) *reinterpret_cast<uint16_t *>(pcnt + k * 2) = (uint16_t)c;
        else pcnt[k] = (uint8_t)c;
    }
}

// xs = wbar o x per band (the count form's bin input); gated by the CG stop flags
template <int NB>
__global__ void k_scale(const double *__restrict__ wbar, const double *__restrict__ x, int64_t NO,
                        double *__restrict__ xs, const int32_t *__restrict__ flags)
{
    if (cg_done(flags)) return;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < NO; i += (int64_t)gridDim.x * blockDim.x) {
        double a[NB], v[NB];
        ldb<NB>(wbar + i * NB, a);
        ldb<NB>(x + i * NB, v);
#pragma unroll
        for (int b = 0; b < NB; ++b) v[b] *= a[b];
        stb<NB>(xs + i * NB, v);
    }
}

// Non-empty pixel rows for the CG bin: flag, exclusive scan, then the compact list with
// each row's entry range (hprow[i] = prow[hrow[i]], hprow[nh] = nnzp) and nh itself.
// h != NULL (member-mask walk, which visits the non-empty rows only): an empty row's
// sample-level maps here -- h = naive numerator = 0, hits = its zero-weight samples' count
__global__ void k_hit_flags(const int64_t *__restrict__ prow, int64_t npix, int32_t *__restrict__ flag, int nb,
                            const uint32_t *__restrict__ hextra, double *__restrict__ h, double *__restrict__ hits,
                            double *__restrict__ nnum, int64_t *__restrict__ counts)
{
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < npix; p += (int64_t)gridDim.x * blockDim.x) {
        const bool hit = prow[p + 1] > prow[p];
        flag[p] = hit ? 1 : 0;
        if (p == 0) counts[2] = 0;     // k_hit_rows' heavy-row count
        if (h && !hit)
            for (int b = 0; b < nb; ++b) {
                h[p * nb + b] = 0.0;
                nnum[p * nb + b] = 0.0;
                hits[p * nb + b] = (double)hextra[p * nb + b];
            }
    }
}

// heavy != NULL: also the list of the rows with more than heavy_min entries (any order,
// count in counts[2], which k_hit_flags zeroed) -- the sample walk starts them first
__global__ void k_hit_rows(const int64_t *__restrict__ prow, const int32_t *__restrict__ flag,
                           const int32_t *__restrict__ pos, int64_t npix, int32_t *__restrict__ hrow,
                           int64_t *__restrict__ hprow, int64_t *__restrict__ counts, int64_t heavy_min,
                           int32_t *__restrict__ heavy)
{
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < npix; p += (int64_t)gridDim.x * blockDim.x) {
        if (flag[p]) {
            hrow[pos[p]] = (int32_t)p;
            hprow[pos[p]] = prow[p];
            if (heavy && prow[p + 1] - prow[p] > heavy_min)
                heavy[atomicAdd(reinterpret_cast<unsigned long long *>(counts + 2), 1ull)] = pos[p];
        }
        if (p == npix - 1) {
            const int64_t nh = (int64_t)pos[p] + flag[p];
            hprow[nh] = prow[npix];
            counts[0] = prow[npix];   // nnzp
            counts[1] = nh;
        }
    }
}

// Sample-level maps in binValues order: h = sum w, hits = sum 1, nnum = sum tod w per
// pixel and band, over the samples of the offsets the band keeps (keep [NB][NO], NULL =
// all), each pixel's samples added one after the other in sample order (the stable
// pixel sort keeps it) -- the reference's sequential loop, bit for bit.
// One wave per pixel: per chunk of 64 of its samples every lane gathers one sample's
// packed payload (64 B for 4 bands) and keep mask into LDS, then lanes 0 .. 3 NB - 1
// each run one of the 3 NB ordered sums (h, nnum, hits per band) over the chunk.  The
// thread-per-pixel walk this replaces kept 8 gathers in flight per pixel, so the most
// hit pixel (thousands of samples) set the kernel time: 545 us on the chain's 3.4 M
// samples, 690 us at C5 (r03s2, r03l).
template <int NB>
__global__ void __launch_bounds__(256) k_sample_walk(const int64_t *__restrict__ srow, const int32_t *__restrict__ sval,
                                                     const double *__restrict__ payload, int64_t npix, int L, int64_t NO,
                                                     const uint8_t *__restrict__ keep, double *__restrict__ h,
                                                     double *__restrict__ hits, double *__restrict__ nnum)
{
    __shared__ double spl[4][64 * 2 * NB];
    __shared__ uint32_t smk[4][64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    double *pl = spl[wv];
    uint32_t *mk = smk[wv];
    const int kind = lane / NB, b = lane % NB;     // this lane's ordered sum (lanes < 3 NB)
    const int col = kind == 2 ? 0 : kind * NB + b;
    for (int64_t p = (int64_t)blockIdx.x * 4 + wv; p < npix; p += (int64_t)gridDim.x * 4) {
        const int64_t lo = srow[p], hi = srow[p + 1];
        double acc = 0.0;
        for (int64_t c = lo; c < hi; c += 64) {
            const int n = (int)((hi - c) < 64 ? (hi - c) : 64);
            if (lane < n) {
                const int32_t i = sval[c + lane];
                double v[2 * NB];
                ldb<2 * NB>(payload + (int64_t)i * 2 * NB, v);
#pragma unroll
                for (int q = 0; q < 2 * NB; ++q) pl[lane * 2 * NB + q] = v[q];
                const int64_t o = i / L;
                uint32_t m = 0;
#pragma unroll
                for (int bb = 0; bb < NB; ++bb) m |= (uint32_t)(!keep || keep[(int64_t)bb * NO + o]) << bb;
                mk[lane] = m;
            }
            wave_lds_sync();   // the chunk, before other lanes read it
            if (lane < 3 * NB) {
                if (kind == 2) {
                    for (int t = 0; t < n; ++t) acc = ((mk[t] >> b) & 1u) ? acc + 1.0 : acc;
                } else {
#pragma unroll 8
                    for (int t = 0; t < n; ++t) {
                        const double v = pl[t * 2 * NB + col];
                        acc = ((mk[t] >> b) & 1u) ? acc + v : acc;
                    }
                }
            }
            wave_lds_sync();   // read before the next chunk overwrites
        }
        if (lane < 3 * NB) (kind == 0 ? h : kind == 1 ? nnum : hits)[p * NB + b] = acc;
    }
}

// every band's non-zero-weight count of a group is 0 or all n of its members (packed
// 8-bit counts): the group's weights are the offset's wb or zero
template <int NB>
__device__ __forceinline__ bool uniform_counts(uint32_t gc, uint32_t n)
{
    bool u = true;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const uint32_t c = (gc >> (8 * b)) & 255u;
        u = u && (c == 0u || c == n);
    }
    return u;
}

// position of the r-th (0-based) set bit of x (r < popcount(x)): six halving steps
__device__ __forceinline__ int select_bit(uint64_t x, int r)
{
    int pos = 0;
#pragma unroll
    for (int sh = 32; sh > 0; sh >>= 1) {
        const int c = __popcll(x & ((1ull << sh) - 1ull));
        if (r >= c) { r -= c; x >>= sh; pos += sh; }
    }
    return pos;
}

// Sample-level maps from the pixel-major entries (member-mask walk): one wave per pixel.
// Per chunk the wave takes the row's next entries (caller's offset order) whose members
// fit 64 M slots, one entry per lane (one packed-record gather each, which also writes the
// entry's pixel-major offset / counts for the CG bin); then every lane fills member slots
// t = lane + 64 u: the owning entry from the chunk's start-position mask, the member's
// sample from the entry's mask (sample order: an entry's members ascending, entries by
// offset), and its (w, tod w) per band into LDS.  tod w comes from the count pass's
// sample-major copy (ptw, one 8 NB-byte read); w is the offset's weight wb when all the
// group's members have a non-zero weight in the band (count form: they all equal wb), 0
// when none has, and only a mixed group reads w itself.  Then 2 NB lanes run the ordered
// sums of h and the naive numerator exactly as k_sample_walk does over the sorted samples.  Samples of groups without
// an entry carry zero weights (they add nothing to h or to the naive numerator); their
// hits come from the count pass's integer adds.
//
// The hits per band are integer counts (each kept member adds 1): they are summed as
// integers per entry instead of a third LDS column -- the same bits (exact below 2^53), a
// third less LDS per slot and 2 NB serial chains instead of 3 NB.
// entries above which a row is walked first (COMAP_DS_HEAVY, 0 = row order only).  Field walk
// (ms, r06w / r06x): 256: 9.00, 512: 8.20, 1024: 7.19, 1536: 6.89, 2048: 6.77-6.89, 3072: 7.00,
// 4096: 8.85 (15 rows), none: 9.45; C5 (max row 1047 entries) unaffected
int64_t heavy_env()
{
    const char *e = getenv("COMAP_DS_HEAVY");
    return e ? (int64_t)atoll(e) : (int64_t)2048;
}

// the walk's rows dealt to the XCDs in contiguous ranges (COMAP_DS_WXCD=1; default 0:
// field set-up walk 8.23 vs 7.86 ms, r06l)
int walk_xcd_env()
{
    const char *e = getenv("COMAP_DS_WXCD");
    return e ? atoi(e) : 0;
}

// the walk's record prefetch one chunk ahead (COMAP_DS_WPF, default 1; field walk 7.23 vs
// 7.83 ms, C5 1.17 vs 1.20 ms, r06m.  Its 73 VGPRs give 6 waves per SIMD; capped for 7:
// 7.28 ms, for 8: 9.05 ms with spills, r06n)
int walk_pf_env()
{
    const char *e = getenv("COMAP_DS_WPF");
    return e ? atoi(e) : 1;
}

template <int NB, int K, int M, bool PF>
__global__ void __launch_bounds__(256) k_sample_walk2(const int32_t *__restrict__ hrow,
                                                      const int64_t *__restrict__ hprow,
                                                      const int64_t *__restrict__ counts,
                                                      const int32_t *__restrict__ sval,
                                                      const SlotRec<K> *__restrict__ srec,
                                                      const int32_t *__restrict__ perm,
                                                      const double *__restrict__ wbar,
                                                      const double *__restrict__ w, const double *__restrict__ ptw,
                                                      int64_t N, int64_t npix, int L, int64_t NO,
                                                      const uint8_t *__restrict__ kint,
                                                      const uint32_t *__restrict__ hextra, double *__restrict__ h,
                                                      double *__restrict__ hits, double *__restrict__ nnum,
                                                      int32_t *__restrict__ poff, uint8_t *__restrict__ pcnt,
                                                      const int32_t *__restrict__ heavy, int64_t heavy_min, int xcd)
{
#pragma clang fp contract(off)
    constexpr int CAP = 64 * M;
    // per member slot, 2 NB doubles: w and tod w per band, each 0 where the band does not
    // keep the member's offset -- adding +0 leaves a sum that never holds -0 unchanged, so
    // lane l < 2 NB runs its ordered sum as one unconditional chain over column l.  Slots are
    // SW doubles apart, SW odd: the 16 lanes of a ds_write_b64 group then hit distinct bank
    // pairs (an even stride would share bank pairs between lanes: multi-way conflicts)
    constexpr int SW = (2 * NB) | 1;
    __shared__ double spl[4][CAP * SW];
    __shared__ uint8_t sfl[4][CAP];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    double *pl = spl[wv];
    uint8_t *fl = sfl[wv];
    const int kind = lane / NB, b = lane % NB;     // this lane's ordered sum (lanes < 2 NB)
    // the non-empty rows only (k_hit_flags wrote the empty ones): row i of nh = counts[1]
    // Each wave walks its heavy rows first (the long walks start at once, dealt round-robin
    // over the XCDs), then its rows of the row list.  xcd: the row list in 8 contiguous
    // ranges, one per XCD (block b runs on XCD b % 8), so an XCD's concurrent waves walk
    // neighbouring pixels, whose entries share offsets -- their sample lines -- in its L2.
    const int64_t nh = counts[1], nhv = heavy ? counts[2] : 0;
    const int64_t W = (int64_t)gridDim.x * 4, w0 = (int64_t)blockIdx.x * 4 + wv;
    int64_t p0 = w0;
    if (xcd) {
        const int64_t x = blockIdx.x & 7, q = gridDim.x >> 3, r = gridDim.x & 7;
        p0 = (x * q + (x < r ? x : r) + (blockIdx.x >> 3)) * 4 + wv;
    }
    // virtual rows: heavy v < nhv (this wave's w0, w0 + W, ...), then row v - nhv (p0, p0 + W, ...)
    auto next = [&](int64_t v) {
        if (v >= nhv) return v + W;
        v += W;
        return v < nhv ? v : nhv + p0;
    };
    for (int64_t ii = w0 < nhv ? w0 : nhv + p0; ii < nh + nhv; ii = next(ii)) {
        const int64_t i = ii < nhv ? (int64_t)heavy[ii] : ii - nhv;
        const int64_t lo = hprow[i], hi = hprow[i + 1];
        if (ii >= nhv && heavy && hi - lo > heavy_min) continue;     // walked from the heavy list
        const int64_t p = hrow[i];
        double acc = 0.0;
        uint32_t hc[NB];               // this lane's entries' kept members per band (hits)
#pragma unroll
        for (int q = 0; q < NB; ++q) hc[q] = 0;
        // slot ids of a chunk's entries: each chunk loads the next chunk's as soon as its own
        // extent is known (lanes past the row's end re-read its last entry: an unconditional
        // load, no select waiting on it).  PF: the next chunk's records (member masks, counts,
        // keep bits) are gathered too, once those ids are in, while this chunk's member
        // gathers are in flight -- one dependent memory round trip per chunk instead of two
        // (every gather below is unconditional -- lanes past the chunk re-read valid entries --
        // so the compiler's wait for one load never has to drain the later ones: a load under
        // a branch makes it wait for all of them at the join)
        constexpr uint32_t kAll = (1u << NB) - 1u;
        const uint8_t *kip = kint ? kint : reinterpret_cast<const uint8_t *>(sval);
        int64_t si_c = sval[lo + lane < hi ? lo + lane : hi - 1];
        // the prefetched record as raw 16-B words (decoded at use: a SlotRec copy made the
        // compiler move the loaded registers at once, waiting for the load right there)
        constexpr int NQ = (int)(sizeof(SlotRec<K>) / 16);
        uint4 rq_n[NQ];
        uint32_t kb_n = kAll;
        if constexpr (PF) {
#pragma unroll
            for (int q = 0; q < NQ; ++q) rq_n[q] = reinterpret_cast<const uint4 *>(srec + si_c)[q];
            kb_n = kip[si_c / L];
        }
        for (int64_t c = lo; c < hi;) {
            const int64_t e = c + lane;
            const bool live = e < hi;
            // the entry's slot si = k L + r: its record from the count pass, the offset's
            // weights and keep bits from k
            const int64_t si = si_c;
            const int64_t kk = si / L;
            SlotRec<K> rc;
            double wb[NB];
            uint32_t kb = kAll;
            if constexpr (PF) {
                const uint32_t *wd = reinterpret_cast<const uint32_t *>(rq_n);
                rc.pix = (int32_t)wd[0];
                rc.cnt = wd[1];
#pragma unroll
                for (int q = 0; q < K; ++q) rc.mask[q] = (uint64_t)wd[2 + 2 * q] | ((uint64_t)wd[3 + 2 * q] << 32);
                kb = kint ? kb_n : kAll;
            } else if (live) {
                rc = srec[si];
                if (kint) kb = kint[kk];
            }
            ldb<NB>(wbar + kk * NB, wb);          // used after the member gathers are issued
            if (!live) {
                rc.pix = 0;
                rc.cnt = 0;
#pragma unroll
                for (int q = 0; q < K; ++q) rc.mask[q] = 0ull;
#pragma unroll
                for (int q = 0; q < NB; ++q) wb[q] = 0.0;
            }
            uint32_t cnt = 0;
#pragma unroll
            for (int q = 0; q < K; ++q) cnt += (uint32_t)__popcll(rc.mask[q]);
            // inclusive prefix of the member counts over the wave (DPP, no LDS permutes)
            const uint32_t inc = wave_incl_scan(cnt);
            const bool take = live && inc <= (uint32_t)CAP;
            const int ntake = __popcll(__ballot(take));     // >= 1: one entry holds <= L <= CAP members
            const int total = (int)__shfl(inc, ntake - 1, 64);
            const uint32_t excl = inc - cnt;
            if (take) {
#pragma unroll
                for (int q = 0; q < NB; ++q) hc[q] += ((kb >> q) & 1u) ? cnt : 0u;
                // the taken entries' pixel-major offset / counts for the CG bin
                poff[e] = (int32_t)kk;
                if constexpr (NB == 4) *reinterpret_cast<uint32_t *>(pcnt + e * 4) = rc.cnt;
                else if constexpr (NB == 2) *reinterpret_cast<uint16_t *>(pcnt + e * 2) = (uint16_t)rc.cnt;
                else pcnt[e] = (uint8_t)rc.cnt;
            }
            {
                const int64_t en = c + ntake + lane;
                si_c = sval[en < hi ? en : hi - 1];            // the next chunk's slot ids
            }
            // the chunk's entry start positions (taken entries hold >= 1 member each): each
            // taken entry flags its first slot in LDS, a ballot per 64 slots reads them back
            uint64_t sm[M];
#pragma unroll
            for (int u = 0; u < M; ++u) fl[lane + 64 * u] = 0;
            wave_lds_sync();
            if (take) fl[excl] = 1;
            wave_lds_sync();
#pragma unroll
            for (int u = 0; u < M; ++u) sm[u] = __ballot(fl[lane + 64 * u] != 0);
            // member slots t = lane + 64 u, first the owning entries and the member gathers ...
            int before = 0;                 // start positions in the slot words below u
            const uint64_t upto_lane = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
            int ju[M], bit[M];
            uint32_t nmu[M], ku[M], kbu[M], gcu[M];
            double pv[M][NB];
#pragma unroll
            for (int u = 0; u < M; ++u) {
                const int t = lane + 64 * u;
                // owning entry: start positions at or before t, minus one
                int j = before + __popcll(sm[u] & upto_lane);
                before += __popcll(sm[u]);
                j = t < total ? j - 1 : 0;
                ju[u] = j;
                const uint32_t exj = (uint32_t)__shfl((int)excl, j, 64);
                nmu[u] = (uint32_t)__shfl((int)cnt, j, 64);
                ku[u] = (uint32_t)__shfl((int)kk, j, 64);
                kbu[u] = (uint32_t)__shfl((int)kb, j, 64);
                gcu[u] = (uint32_t)__shfl((int)rc.cnt, j, 64);
                uint64_t mj[K];
#pragma unroll
                for (int q = 0; q < K; ++q) mj[q] = (uint64_t)__shfl((long long)rc.mask[q], j, 64);
                int r = t - (int)exj, bitpos = 0;
#pragma unroll
                for (int q = 0; q < K; ++q) {
                    const int cq = __popcll(mj[q]);
                    if (r >= 0 && r < cq) bitpos = 64 * q + select_bit(mj[q], r);
                    r -= cq;
                }
                bit[u] = bitpos;
                // (slots past the chunk: entry 0's first member, a valid address)
                ldb<NB>(ptw + ((int64_t)ku[u] * L + bitpos) * NB, pv[u]);
            }
            // a mixed group (some members zero-weight in a band): the sample's own weights
            double wmix[M][NB];
#pragma unroll
            for (int u = 0; u < M; ++u) {
                const int t = lane + 64 * u;
                if (t < total && !uniform_counts<NB>(gcu[u], nmu[u])) {
                    const int64_t on = perm ? (int64_t)perm[ku[u]] : (int64_t)ku[u];
#pragma unroll
                    for (int bb = 0; bb < NB; ++bb) {
                        const uint32_t gc = (gcu[u] >> (8 * bb)) & 255u;
                        wmix[u][bb] = gc != 0 && gc != nmu[u] ? w[(int64_t)bb * N + on * L + bit[u]] : 0.0;
                    }
                }
            }
            if constexpr (PF) {
                // ... then the next chunk's records (waits for its slot ids only) ...
#pragma unroll
                for (int q = 0; q < NQ; ++q) rq_n[q] = reinterpret_cast<const uint4 *>(srec + si_c)[q];
                kb_n = kip[si_c / L];
            }
            // ... then the slots' (w, tod w) per band into LDS
#pragma unroll
            for (int u = 0; u < M; ++u) {
                const int t = lane + 64 * u;
                double wbj[NB];
#pragma unroll
                for (int q = 0; q < NB; ++q) wbj[q] = __shfl(wb[q], ju[u], 64);
                if (t < total) {
                    const uint32_t gcj = gcu[u], nmj = nmu[u];
                    double wvs[NB];
#pragma unroll
                    for (int bb = 0; bb < NB; ++bb) {
                        const uint32_t gc = (gcj >> (8 * bb)) & 255u;
                        wvs[bb] = gc == nmj ? wbj[bb] : 0.0;
                    }
                    if (!uniform_counts<NB>(gcj, nmj)) {
#pragma unroll
                        for (int bb = 0; bb < NB; ++bb) {
                            const uint32_t gc = (gcj >> (8 * bb)) & 255u;
                            if (gc != 0 && gc != nmj) wvs[bb] = wmix[u][bb];
                        }
                    }
#pragma unroll
                    for (int bb = 0; bb < NB; ++bb) {
                        const bool kept = (kbu[u] >> bb) & 1u;
                        pl[t * SW + bb] = kept ? wvs[bb] : 0.0;
                        pl[t * SW + NB + bb] = kept ? pv[u][bb] : 0.0;
                    }
                }
            }
            wave_lds_sync();   // the chunk, before other lanes read it
            if (lane < 2 * NB) {
#pragma unroll 8
                for (int t = 0; t < total; ++t) acc += pl[t * SW + lane];
            }
            wave_lds_sync();   // read before the next chunk overwrites
            c += ntake;
        }
        uint32_t hv = 0;               // lane q < NB: band q's hits over the row
#pragma unroll
        for (int q = 0; q < NB; ++q) {
            const uint32_t tq = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(hc[q]), 63);
            hv = lane == q ? tq : hv;
        }
        if (lane < 2 * NB) (kind == 0 ? h : nnum)[p * NB + b] = acc;
        if (lane < NB) hits[p * NB + lane] = (double)(hv + hextra[p * NB + lane]);
    }
}

// The map pixel a projection entry gathers: op_Z reads m[pointing] (Destriper.py:206-213),
// so an unbinned sample's negative id p in [-npix, -1] reads m[npix + p] -- numpy's index
// wrap (-1: the last pixel).  The set-up rejects p < -npix (numpy's IndexError).
__device__ __forceinline__ int64_t wrap_pixel(int32_t p, int64_t npix) { return p >= 0 ? (int64_t)p : npix + p; }

__device__ __forceinline__ double map_value(const double *num, const double *h, int64_t q)
{
    const double hv = h[q];
    return hv != 0.0 ? num[q] / hv : num[q];
}

// num_p = sum_e s_e x_o(e) per band; base != NULL: num = base - W x (final destriped
// numerator); hdiv != NULL: num = m = (W x) / h, the map itself (single rank: k_ds_project
// then gathers one array).  kBinLanes lanes per pixel row (rows hold 0 .. thousands of
// entries), lane-strided; each lane issues kBinU entry loads, then kBinU gathers of the
// NB-band x vectors, before its fmas (in entry order, so the sum is the plain
// lane-strided one), then a kBinLanes-lane reduction.
template <int kBinLanes, int NB, bool CF, int kBinU>
__global__ void __launch_bounds__(256) k_ds_bin(const int64_t *__restrict__ prow, const int32_t *__restrict__ poff,
                                                const void *__restrict__ pw, const double *__restrict__ x,
                                                int64_t npix, const double *__restrict__ base,
                                                const double *__restrict__ hdiv, double *__restrict__ num,
                                                const int32_t *__restrict__ flags, const int32_t *__restrict__ rows)
{
    if (cg_done(flags)) return;
    const int sub = threadIdx.x & (kBinLanes - 1);
    const int64_t step = (int64_t)gridDim.x * blockDim.x / kBinLanes;
    // rows != NULL: only the listed (non-empty) rows, npix = their count, and prow holds
    // their entry ranges (hprow: row i spans [prow[i], prow[i + 1]), no dependent row load)
    for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kBinLanes; i < npix; i += step) {
        const int64_t p = rows ? (int64_t)rows[i] : i;
        double s[NB];
#pragma unroll
        for (int b = 0; b < NB; ++b) s[b] = 0.0;
        // the row's base / h values, loaded by the lead lane up front (their latency
        // overlaps the row's gathers instead of following its reduction)
        double tail[NB];
#pragma unroll
        for (int b = 0; b < NB; ++b) tail[b] = 0.0;
        if (sub == 0 && (base || hdiv)) ldb<NB>((base ? base : hdiv) + p * NB, tail);
        const int64_t e1 = prow[i + 1];
        // software pipeline: the next group's entry loads are issued before this group's
        // x gathers are consumed, so a lane has one dependent latency per group, not two
        int64_t k = prow[i] + sub;
        int32_t o[kBinU];
        Coef<NB, CF> a[kBinU];
#pragma unroll
        for (int u = 0; u < kBinU; ++u) {
            const bool in = k + u * kBinLanes < e1;
            o[u] = in ? poff[k + u * kBinLanes] : 0;
            if (in) a[u].load(pw, k + u * kBinLanes);
        }
        while (k < e1) {
            double xv[kBinU][NB];
#pragma unroll
            for (int u = 0; u < kBinU; ++u) ldb<NB>(x + (int64_t)o[u] * NB, xv[u]);
            const int64_t kn = k + kBinLanes * kBinU;
            int32_t on[kBinU];
            Coef<NB, CF> an[kBinU];
#pragma unroll
            for (int u = 0; u < kBinU; ++u) {
                const bool in = kn + u * kBinLanes < e1;
                on[u] = in ? poff[kn + u * kBinLanes] : 0;
                if (in) an[u].load(pw, kn + u * kBinLanes);
            }
#pragma unroll
            for (int u = 0; u < kBinU; ++u)
                if (k + u * kBinLanes < e1) {
#pragma unroll
                    for (int b = 0; b < NB; ++b) s[b] = fma(a[u].get(b), xv[u][b], s[b]);
                }
#pragma unroll
            for (int u = 0; u < kBinU; ++u) { o[u] = on[u]; a[u] = an[u]; }
            k = kn;
        }
#pragma unroll
        for (int b = 0; b < NB; ++b) {
#pragma unroll
            for (int o = kBinLanes / 2; o > 0; o >>= 1) s[b] += __shfl_xor(s[b], o, kBinLanes);
        }
        if (sub == 0) {
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                if (base) s[b] = tail[b] - s[b];
                else if (hdiv) { const double hv = tail[b]; s[b] = hv != 0.0 ? s[b] / hv : s[b]; }
            }
            stb<NB>(num + p * NB, s);
        }
    }
}

// y_o = ws_o x_o - sum_e s_e m_p(e) per band  (x == NULL: y_o = tw_o - ..., the b vector).
// G lanes per offset (G = 16 for L <= 64: 256/G offsets per block sweep); each lane issues
// kProjU entry loads then kProjU map gathers before its fmas; m = num / h, or num itself
// when h == NULL (k_ds_bin already divided).  Block partials of y.x per band
// (dot_part + b kPartMax, when dot_part != NULL).
template <int G, int NB, bool CF, int kProjU>
__global__ void __launch_bounds__(256) k_ds_project(const int64_t *__restrict__ orow, const int32_t *__restrict__ opix,
                                                    const void *__restrict__ ow, const double *__restrict__ wbar,
                                                    const double *__restrict__ ws,
                                                    const double *__restrict__ tw, const double *__restrict__ x,
                                                    const double *__restrict__ num, const double *__restrict__ h,
                                                    int64_t NO, int64_t npix, double *__restrict__ y,
                                                    double *__restrict__ dot_part, const int32_t *__restrict__ flags,
                                                    int64_t pstride = kPartMax)
{
    __shared__ double red[4 * NB];
    if (cg_done(flags)) return;
    constexpr int kPer = 256 / G;
    const int sub = threadIdx.x & (G - 1);
    double acc[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[b] = 0.0;
    // Software pipeline over the block's sweeps (kPer offsets each): while this sweep's
    // map gathers are in flight, the next sweep's first pass of entries (and the row
    // bounds of the one after) are already being loaded -- a lane waits on one dependent
    // latency per sweep instead of three.  Rows longer than one pass (G kProjU entries)
    // finish with plain passes.
    const int64_t stride = (int64_t)gridDim.x * kPer;
    int64_t o = (int64_t)blockIdx.x * kPer + threadIdx.x / G;
    int64_t b0 = 0, b1 = 0, nb0 = 0, nb1 = 0;
    if (o < NO) { b0 = orow[o]; b1 = orow[o + 1]; }
    if (o + stride < NO) { nb0 = orow[o + stride]; nb1 = orow[o + stride + 1]; }
    int32_t cq[kProjU];
    Coef<NB, CF> ca[kProjU];
    auto load_pass = [&](int64_t e, int64_t e1, int32_t (&q)[kProjU], Coef<NB, CF> (&a)[kProjU]) {
#pragma unroll
        for (int u = 0; u < kProjU; ++u) {
            const bool in = e + u * G < e1;
            q[u] = in ? (int32_t)wrap_pixel(opix[e + u * G], npix) : 0;   // numpy's m[p] wrap for p < 0
            if (in) a[u].load(ow, e + u * G);
            else a[u] = Coef<NB, CF>();
        }
    };
    auto gather = [&](const int32_t (&q)[kProjU], double (&mv)[kProjU][NB]) {
#pragma unroll
        for (int u = 0; u < kProjU; ++u) {
            if (h) {
#pragma unroll
                for (int b = 0; b < NB; ++b) mv[u][b] = map_value(num, h, (int64_t)q[u] * NB + b);
            } else {
                ldb<NB>(num + (int64_t)q[u] * NB, mv[u]);
            }
        }
    };
    load_pass(b0 + sub, b1, cq, ca);
    for (; o - threadIdx.x / G < NO; o += stride) {
        const bool valid = o < NO;
        const int64_t e0 = b0, e1 = b1;
        double g[NB];
#pragma unroll
        for (int b = 0; b < NB; ++b) g[b] = 0.0;
        double mv[kProjU][NB];
        gather(cq, mv);
        // next sweep: its first pass of entries, and the row bounds of the sweep after it
        int32_t nq[kProjU];
        Coef<NB, CF> na[kProjU];
        load_pass(nb0 + sub, nb1, nq, na);
        b0 = nb0; b1 = nb1;
        nb0 = nb1 = 0;
        if (o + 2 * stride < NO) { nb0 = orow[o + 2 * stride]; nb1 = orow[o + 2 * stride + 1]; }
#pragma unroll
        for (int u = 0; u < kProjU; ++u)
            if (e0 + sub + u * G < e1) {
#pragma unroll
                for (int b = 0; b < NB; ++b) g[b] = fma(ca[u].get(b), mv[u][b], g[b]);
            }
        for (int64_t e = e0 + sub + G * kProjU; e < e1; e += G * kProjU) {   // long rows
            int32_t q[kProjU];
            Coef<NB, CF> a[kProjU];
            load_pass(e, e1, q, a);
            double mw[kProjU][NB];
            gather(q, mw);
#pragma unroll
            for (int u = 0; u < kProjU; ++u)
                if (e + u * G < e1) {
#pragma unroll
                    for (int b = 0; b < NB; ++b) g[b] = fma(a[u].get(b), mw[u][b], g[b]);
                }
        }
#pragma unroll
        for (int u = 0; u < kProjU; ++u) { cq[u] = nq[u]; ca[u] = na[u]; }
#pragma unroll
        for (int b = 0; b < NB; ++b) {
#pragma unroll
            for (int s = G / 2; s > 0; s >>= 1) g[b] += __shfl_xor(g[b], s, G);
        }
        if (valid && sub == 0) {
            // (loading x / wbar / ws at the top of the sweep, beside the gathers, measured
            // slower: 124.6 -> 136.4 us at C5 4 bands, r03t4)
            double xo[NB], v[NB];
            if (x) {
                ldb<NB>(x + o * NB, xo);
            } else {
#pragma unroll
                for (int b = 0; b < NB; ++b) xo[b] = 0.0;
            }
            if constexpr (CF) {   // the row's sum of counts x m, times the offset's weight
                double wb[NB];
                ldb<NB>(wbar + o * NB, wb);
#pragma unroll
                for (int b = 0; b < NB; ++b) g[b] *= wb[b];
            }
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                v[b] = (x ? ws[o * NB + b] * xo[b] : tw[o * NB + b]) - g[b];
                if (dot_part) acc[b] = fma(v[b], xo[b], acc[b]);
            }
            stb<NB>(y + o * NB, v);
        }
    }
    if (dot_part) {
        block_partials<NB>(acc, red, dot_part + blockIdx.x, pstride);
        if (pstride < kPartMax && blockIdx.x == 0) zero_tail<NB>(dot_part, pstride, gridDim.x);
    }
}

// ---------------------------------------------------------------- sliced-ELLPACK projection
constexpr int32_t kSellPad = (int32_t)0x80808080;   // memset pattern 0x80: a padding slot

// chunk widths: sw[c] = 64 x the longest row of offsets [64 c, 64 c + 64); sw[NC] = 0.
__global__ void k_sell_width(const int64_t *__restrict__ orow, int64_t NO, int64_t NC, int64_t *__restrict__ sw)
{
    const int64_t c = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (c > NC) return;
    const int64_t o = c * 64 + (threadIdx.x & 63);
    int64_t len = (c < NC && o < NO) ? orow[o + 1] - orow[o] : 0;
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) len = max(len, (int64_t)__shfl_xor(len, s, 64));
    if ((threadIdx.x & 63) == 0) sw[c] = 64 * len;
}

// The sliced-ELLPACK fill, one workgroup per chunk: the chunk's CSR range (contiguous: its offsets are
// consecutive rows) is staged in LDS with coalesced loads, then the padded column-major
// slots are written in order (coalesced, padding included: no memset).  Chunks holding more
// than kSellStage entries read their rows straight from global memory.
constexpr int kSellStage = 4096;
template <int NB, bool CF>
__global__ void __launch_bounds__(256) k_sell_fill_lds(const int64_t *__restrict__ orow,
                                                       const int32_t *__restrict__ opix,
                                                       const void *__restrict__ oco,
                                                       const int64_t *__restrict__ sbase, int64_t NO,
                                                       int32_t *__restrict__ spix, void *__restrict__ sco)
{
    // count form: an entry's NB uint8 counts moved as one NB-byte word (4 byte loads and
    // stores per entry were most of this kernel's instructions)
    using PackT = typename std::conditional<NB == 4, uint32_t, typename std::conditional<NB == 2, uint16_t, uint8_t>::type>::type;
    __shared__ int32_t lp[kSellStage];
    __shared__ PackT lc[CF ? kSellStage : 1];
    __shared__ int32_t rs[64], rn[64];
    constexpr int cw = 64;
    const int64_t c = blockIdx.x;
    const int64_t o0 = c * cw;
    const int nrow = (int)std::min<int64_t>(cw, NO - o0);
    const int64_t e0 = orow[o0];
    const int64_t ne = orow[o0 + nrow] - e0;
    if (threadIdx.x < cw) {
        const int r = threadIdx.x;
        rs[r] = r < nrow ? (int)(orow[o0 + r] - e0) : 0;
        rn[r] = r < nrow ? (int)(orow[o0 + r + 1] - orow[o0 + r]) : 0;
    }
    const bool staged = ne <= kSellStage && CF;
    if (staged) {
        for (int64_t i = threadIdx.x; i < ne; i += blockDim.x) {
            lp[i] = opix[e0 + i];
            lc[i] = reinterpret_cast<const PackT *>(oco)[e0 + i];
        }
    }
    __syncthreads();
    const int64_t b0 = sbase[c], nslot = sbase[c + 1] - b0;
    for (int64_t sl = threadIdx.x; sl < nslot; sl += blockDim.x) {
        const int r = (int)(sl % cw);
        const int64_t j = sl / cw;
        const bool in = j < rn[r];
        const int64_t ei = (int64_t)rs[r] + j;
        int32_t q = kSellPad;
        if constexpr (CF) {
            PackT a = 0;
            if (in) {
                q = staged ? lp[ei] : opix[e0 + ei];
                a = staged ? lc[ei] : reinterpret_cast<const PackT *>(oco)[e0 + ei];
            }
            spix[b0 + sl] = q;
            reinterpret_cast<PackT *>(sco)[b0 + sl] = a;
        } else {
            double a[NB];
#pragma unroll
            for (int k = 0; k < NB; ++k) a[k] = 0;
            if (in) {
                q = opix[e0 + ei];
#pragma unroll
                for (int k = 0; k < NB; ++k) a[k] = reinterpret_cast<const double *>(oco)[(e0 + ei) * NB + k];
            }
            spix[b0 + sl] = q;
#pragma unroll
            for (int k = 0; k < NB; ++k) reinterpret_cast<double *>(sco)[(b0 + sl) * NB + k] = a[k];
        }
    }
}

// k_ds_project on the sliced-ELLPACK rows: one wave per chunk of 64 offsets (chunks dealt
// to the grid's waves round-robin), lane = offset.  Each lane walks its row in groups of U
// entries: the group's pixel ids and coefficients are coalesced loads issued one group
// ahead of its map gathers, and the row sum is a plain in-order fma chain per lane (no
// shuffles).  Same outputs as k_ds_project (y, block partials of y.x per band).
template <int NB, bool CF, int U>
__global__ void __launch_bounds__(256) k_ds_project_sell(const int64_t *__restrict__ sbase,
                                                         const int32_t *__restrict__ spix, const void *__restrict__ sco,
                                                         const double *__restrict__ wbar, const double *__restrict__ ws,
                                                         const double *__restrict__ tw, const double *__restrict__ x,
                                                         const double *__restrict__ num, const double *__restrict__ h,
                                                         int64_t NO, int64_t npix, double *__restrict__ y,
                                                         double *__restrict__ dot_part, const int32_t *__restrict__ flags,
                                                         int64_t pstride)
{
    __shared__ double red[4 * NB];
    if (cg_done(flags)) return;
    const int lane = threadIdx.x & 63;
    const int64_t NC = (NO + 63) >> 6;
    const int64_t nw = (int64_t)gridDim.x * 4;
    double acc[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[b] = 0.0;
    for (int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); c < NC; c += nw) {
        const int64_t b0 = sbase[c], W = (sbase[c + 1] - b0) >> 6;
        const int64_t o = c * 64 + lane;
        const int32_t *pp = spix + b0 + lane;
        double g[NB];
#pragma unroll
        for (int b = 0; b < NB; ++b) g[b] = 0.0;
        int32_t q[U];
        Coef<NB, CF> a[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool in = u < W;
            q[u] = in ? pp[64 * u] : kSellPad;
            if (in) a[u].load(sco, b0 + 64 * u + lane);
        }
        for (int64_t j = 0; j < W; j += U) {
            double mv[U][NB];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (q[u] != kSellPad) {
                    const int64_t qq = wrap_pixel(q[u], npix);     // m[p] with numpy's wrap for p < 0
                    if (h) {
#pragma unroll
                        for (int b = 0; b < NB; ++b) mv[u][b] = map_value(num, h, qq * NB + b);
                    } else {
                        ldb<NB>(num + qq * NB, mv[u]);
                    }
                }
            }
            const int64_t jn = j + U;
            int32_t qn[U];
            Coef<NB, CF> an[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const bool in = jn + u < W;
                qn[u] = in ? pp[64 * (jn + u)] : kSellPad;
                if (in) an[u].load(sco, b0 + 64 * (jn + u) + lane);
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (q[u] != kSellPad) {
#pragma unroll
                    for (int b = 0; b < NB; ++b) g[b] = fma(a[u].get(b), mv[u][b], g[b]);
                }
#pragma unroll
            for (int u = 0; u < U; ++u) { q[u] = qn[u]; a[u] = an[u]; }
        }
        if (o < NO) {
            double v[NB], xo[NB], wb[NB], wsv[NB];
            if (x) ldb<NB>(x + o * NB, xo);
            if constexpr (CF) ldb<NB>(wbar + o * NB, wb);
            ldb<NB>((x ? ws : tw) + o * NB, wsv);
            if (!x) {
#pragma unroll
                for (int b = 0; b < NB; ++b) xo[b] = 0.0;
            }
            if constexpr (CF) {
#pragma unroll
                for (int b = 0; b < NB; ++b) g[b] *= wb[b];
            }
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                v[b] = (x ? wsv[b] * xo[b] : wsv[b]) - g[b];
                if (dot_part) acc[b] = fma(v[b], xo[b], acc[b]);
            }
            stb<NB>(y + o * NB, v);
        }
    }
    if (dot_part) {
        block_partials<NB>(acc, red, dot_part + blockIdx.x, pstride);
        if (pstride < kPartMax && blockIdx.x == 0) zero_tail<NB>(dot_part, pstride, gridDim.x);
    }
}

// per-band block partials of sum_o a[o][b] c[o][b]
template <int NB>
__global__ void __launch_bounds__(256) k_dot_part(const double *__restrict__ a, const double *__restrict__ c, int64_t n,
                                                  double *__restrict__ part)
{
    __shared__ double red[4 * NB];
    double acc[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[b] = 0.0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        double av[NB], cv[NB];
        ldb<NB>(a + i * NB, av);
        ldb<NB>(c + i * NB, cv);
#pragma unroll
        for (int b = 0; b < NB; ++b) acc[b] = fma(av[b], cv[b], acc[b]);
    }
    block_partials<NB>(acc, red, part + blockIdx.x);
}

// out[b] = fixed-order sum of band b's n partials
template <int NB>
__global__ void __launch_bounds__(256) k_dot_final(const double *__restrict__ part, int n, double *__restrict__ out,
                                                   const int32_t *__restrict__ flags)
{
    __shared__ double red[4];
    if (cg_done(flags)) return;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const double sum = block_final_sum(part + (int64_t)b * kPartMax, n, red);
        if (threadIdx.x == 0) out[b] = sum;
    }
}

// one offset's x += a p ; r -= a q for the live bands, accumulating r.r (16-B vector access)
template <int NB>
__device__ __forceinline__ void update_row(double *__restrict__ x, double *__restrict__ r, const double *__restrict__ p,
                                           const double *__restrict__ q, const double (&a)[NB], const bool (&live)[NB],
                                           double (&acc)[NB])
{
    double xv[NB], rv[NB], pv[NB], qv[NB];
    ldb<NB>(r, rv);
    ldb<NB>(p, pv);
    ldb<NB>(q, qv);
    ldb<NB>(x, xv);
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        if (live[b]) {
            xv[b] += a[b] * pv[b];
            rv[b] = rv[b] - a[b] * qv[b];
        }
        acc[b] = fma(rv[b], rv[b], acc[b]);
    }
    stb<NB>(x, xv);
    stb<NB>(r, rv);
}

// p = r + beta p for the live bands of one offset; wbar != NULL (count form): also
// pt = wbar o p, the next bin's input
template <int NB>
__device__ __forceinline__ void direction_row(double *__restrict__ p, const double *__restrict__ r,
                                              const double (&beta)[NB], const bool (&live)[NB],
                                              const double *__restrict__ wbar = nullptr, double *__restrict__ pt = nullptr)
{
    double pv[NB], rv[NB];
    ldb<NB>(p, pv);
    ldb<NB>(r, rv);
#pragma unroll
    for (int b = 0; b < NB; ++b)
        if (live[b]) pv[b] = rv[b] + beta[b] * pv[b];
    stb<NB>(p, pv);
    if (wbar) {
        double a[NB];
        ldb<NB>(wbar, a);
#pragma unroll
        for (int b = 0; b < NB; ++b) pv[b] *= a[b];
        stb<NB>(pt, pv);
    }
}

// x += a p ; r -= a q ; a = rr / pq per band (bands already stopped are left alone);
// per-band partials of r.r
template <int NB>
__global__ void __launch_bounds__(256) k_cg_update(const double *__restrict__ rr, const double *__restrict__ pq,
                                                   double *__restrict__ x, double *__restrict__ r,
                                                   const double *__restrict__ p, const double *__restrict__ q,
                                                   int64_t n, double *__restrict__ part, const int32_t *__restrict__ flags)
{
    __shared__ double red[4 * NB];
    if (cg_done(flags)) return;
    double a[NB], acc[NB];
    bool live[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) { a[b] = rr[b] / pq[b]; live[b] = !band_stopped(flags, b); acc[b] = 0.0; }
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        update_row<NB>(x + i * NB, r + i * NB, p + i * NB, q + i * NB, a, live, acc);
    block_partials<NB>(acc, red, part + blockIdx.x);
}

// End-of-iteration bookkeeping (Destriper.py:136-152) by one thread, per band still
// running: rr = rr_new, count it, stop when delta = rr_new / rr0 is NaN or below the
// threshold; flags[1] counts iterations any band ran, flags[0] = every band stopped.
template <int NB, bool kSetRr = true>
__device__ __forceinline__ void cg_check(double *__restrict__ scal, int32_t *__restrict__ flags, const double *rrn)
{
    bool any = false, all = true;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        if (!flags[2 + b]) {
            any = true;
            if (kSetRr) scal[NB + b] = rrn[b];   // the per-piece update reads rr there
            scal[3 * NB + b] = rrn[b];
            flags[2 + NB + b] += 1;
            const double delta = rrn[b] / scal[b];
            if (isnan(delta) || delta < scal[4 * NB]) flags[2 + b] = 1;
        }
        all = all && flags[2 + b];
    }
    if (any) flags[1] += 1;
    if (all) flags[0] = 1;
}

// Fused single-rank CG tail (comap_destripe_solve): no separate final-sum or check
// launches.  Every block re-derives the global sums from the previous kernel's block
// partials in k_dot_final's order, so all blocks hold identical values and no block
// waits on another.  Per band: scal[b] rr0, scal[NB+b] rr of this iteration (for beta),
// scal[3NB+b] current rr.
//   k_cg_update_fused: pq = sum(pq partials); a = rr / pq; x += a p; r -= a q;
//                      r.r partials into part_rr; block 0 saves rr and pq
//   k_cg_direction_fused: rr_new = sum(part_rr); p = r + (rr_new / rr) p;
//                      block 0: rr = rr_new, count, stop test (cg_check)
template <int NB>
__global__ void __launch_bounds__(256) k_cg_update_fused(double *__restrict__ scal, const double *__restrict__ part_pq,
                                                         int npq, double *__restrict__ x, double *__restrict__ r,
                                                         const double *__restrict__ p, const double *__restrict__ q,
                                                         int64_t n, double *__restrict__ part_rr,
                                                         const int32_t *__restrict__ flags, int64_t pstride = kPartMax)
{
    __shared__ double red[4 * NB];
    if (cg_done(flags)) return;
    double pq[NB], rr[NB], a[NB], acc[NB];
    bool live[NB];
    block_final_sums<NB>(part_pq, npq, red, pq, pstride);
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        rr[b] = scal[3 * NB + b];
        a[b] = rr[b] / pq[b];
        live[b] = !band_stopped(flags, b);
        acc[b] = 0.0;
    }
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        update_row<NB>(x + i * NB, r + i * NB, p + i * NB, q + i * NB, a, live, acc);
    block_partials<NB>(acc, red, part_rr + blockIdx.x, pstride);
    if (pstride < kPartMax && blockIdx.x == 0) zero_tail<NB>(part_rr, pstride, gridDim.x);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
#pragma unroll
        for (int b = 0; b < NB; ++b)
            if (live[b]) { scal[NB + b] = rr[b]; scal[2 * NB + b] = pq[b]; }
    }
}

template <int NB>
__global__ void __launch_bounds__(256) k_cg_direction_fused(double *__restrict__ scal, const double *__restrict__ part_rr,
                                                            int nrr, double *__restrict__ p, const double *__restrict__ r,
                                                            int64_t n, int32_t *flags, int64_t pstride = kPartMax,
                                                            const double *__restrict__ wbar = nullptr,
                                                            double *__restrict__ pt = nullptr)
{
    __shared__ double red[4 * NB];
    if (flags[0]) return;
    double rrn[NB], beta[NB];
    bool live[NB];
    block_final_sums<NB>(part_rr, nrr, red, rrn, pstride);
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        beta[b] = rrn[b] / scal[NB + b];
        live[b] = !flags[2 + b];
    }
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        direction_row<NB>(p + i * NB, r + i * NB, beta, live, wbar ? wbar + i * NB : nullptr,
                          wbar ? pt + i * NB : nullptr);
    // block 0 only, after its own sweep: a band that stops here never reads p again.
    // scal[NB+b] is left alone -- other blocks may still be reading it for beta; the
    // fused update takes rr from scal[3NB+b] and rewrites scal[NB+b] itself.
    if (blockIdx.x == 0 && threadIdx.x == 0) cg_check<NB, false>(scal, flags, rrn);
}

// p = r + (rr_new / rr) p per band still running
template <int NB>
__global__ void k_cg_direction(const double *__restrict__ rr_new, const double *__restrict__ rr, double *__restrict__ p,
                               const double *__restrict__ r, int64_t n, const int32_t *__restrict__ flags)
{
    if (cg_done(flags)) return;
    double beta[NB];
    bool live[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) { beta[b] = rr_new[b] / rr[b]; live[b] = !band_stopped(flags, b); }
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        direction_row<NB>(p + i * NB, r + i * NB, beta, live);
}

template <int NB>
__global__ void k_cg_check(double *__restrict__ scal, int32_t *__restrict__ flags)
{
    if (threadIdx.x != 0 || flags[0]) return;
    double rrn[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) rrn[b] = scal[3 * NB + b];
    cg_check<NB>(scal, flags, rrn);
}

__global__ void k_div_map(const double *__restrict__ num, const double *__restrict__ h, int64_t n,
                          double *__restrict__ out)
{
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x)
        out[p] = map_value(num, h, p);
}

inline unsigned grid_for(int64_t n, int64_t cap = 4096) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, cap)); }
// CG update grid: one offset row per thread up to kUpdBlocks blocks (the fused and the
// per-piece paths use the same grid, hence the same r.r partials)
inline unsigned upd_grid(int64_t NO) { return grid_for(NO, kUpdBlocks); }

// every templated launch dispatches on the problem's band count (1, 2 or 4)
#define COMAP_NB_SWITCH(nb, ...)                                 \
    switch (nb) {                                                \
    case 1: { constexpr int NB = 1; __VA_ARGS__; } break;       \
    case 2: { constexpr int NB = 2; __VA_ARGS__; } break;       \
    default: { constexpr int NB = 4; __VA_ARGS__; } break;      \
    }

// k_ds_bin with kBinLanes sized to the mean pixel-row length (sparse C4-like maps
// hold ~5 entries per pixel: 16 lanes per row would leave most lanes idle and
// need several latency-bound grid sweeps); one sweep over all rows.
// hit_rows: only the non-empty rows (d->hrow; the caller's num must hold 0 on the
// empty rows, as the CG's own map buffer does).  Count form: x must already be
// scaled (wbar o x, x_scaled) or is scaled into d->pt first.
template <int NB, bool CF, int U>
void launch_bin_u(const comap_destriper *d, hipStream_t st, const double *x, const double *base, const double *hdiv,
                  double *num, const int32_t *flags, bool hit_rows)
{
    const int64_t np = hit_rows ? d->nh : d->npix;
    const int32_t *rows = hit_rows ? d->hrow : nullptr;
    const int64_t *rp = hit_rows ? d->hprow : d->prow;
    const int64_t mean = np ? d->nnzp / np : 0;
    const void *co = CF ? (const void *)d->pcnt : (const void *)d->pw;
    // (rows of >= 256 entries -- the field's 415 -- with 8 loads per lane: 32 lanes, field 4 bands
    // 1.354 -> 1.336 ms, 1 band 0.655 -> 0.623 ms per iteration, profiles/r06/r06cg)
    const int lanes = d->bin_lanes ? d->bin_lanes
                                   : (mean >= 256 && U == 8 ? 32 : (mean >= 24 ? 16 : (mean >= 10 ? 8 : 4)));
    const unsigned g = grid_for(np * lanes, 65536);
#define COMAP_BIN(LN) k_ds_bin<LN, NB, CF, U><<<g, 256, 0, st>>>(rp, d->poff, co, x, np, base, hdiv, num, flags, rows)
    switch (lanes) {
    case 64: COMAP_BIN(64); break;
    case 32: COMAP_BIN(32); break;
    case 16: COMAP_BIN(16); break;
    case 8: COMAP_BIN(8); break;
    default: COMAP_BIN(4);
    }
#undef COMAP_BIN
}

template <int NB, bool CF>
void launch_bin_cf(const comap_destriper *d, hipStream_t st, const double *x, const double *base, const double *hdiv,
                   double *num, const int32_t *flags, bool hit_rows)
{
    if (d->bin_u == 8) launch_bin_u<NB, CF, 8>(d, st, x, base, hdiv, num, flags, hit_rows);
    else launch_bin_u<NB, CF, 4>(d, st, x, base, hdiv, num, flags, hit_rows);
}

void launch_bin(const comap_destriper *d, hipStream_t st, const double *x, const double *base, const double *hdiv,
                double *num, const int32_t *flags, bool hit_rows = false, bool x_scaled = false)
{
    if (d->cf && !x_scaled) {
        COMAP_NB_SWITCH(d->nb, k_scale<NB><<<grid_for(d->NO), 256, 0, st>>>(d->wbar, x, d->NO, d->pt, flags));
        x = d->pt;
    }
    if (d->cf) {
        COMAP_NB_SWITCH(d->nb, (launch_bin_cf<NB, true>(d, st, x, base, hdiv, num, flags, hit_rows)));
    } else {
        COMAP_NB_SWITCH(d->nb, (launch_bin_cf<NB, false>(d, st, x, base, hdiv, num, flags, hit_rows)));
    }
}

// lanes per offset row: the fewest whose one pass of kProjU loads covers the mean row
// (C5: 28 entries per offset -> 8 lanes, 32 offsets per block sweep; C4: 14 -> 4).
// Measured at C5 (r03e, ms per CG iteration, 1 / 4 bands): 16 lanes 0.152 / 0.347,
// 8 lanes 0.132 / 0.307; 8 loads per lane or a 2048-block grid: within noise or slower.
inline int project_lanes(const comap_destriper *d)
{
    if (d->proj_lanes) return d->proj_lanes;
    const int64_t mean = d->NO ? (d->nnz + d->NO - 1) / d->NO : 0;
    int g = 4;
    while (g < 64 && g * d->proj_u < mean) g *= 2;
    return g;
}
inline unsigned project_grid(const comap_destriper *d, int64_t cap)
{
    const int64_t per = d->sell ? 256 : 256 / project_lanes(d);   // offsets per block sweep
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>((d->NO + per - 1) / per, std::min<int64_t>(cap, d->proj_blocks)));
}

// k_ds_project with the lane group sized to the offset length; returns its grid (= partials).
template <int NB, bool CF, int U>
unsigned launch_project_u(const comap_destriper *d, hipStream_t st, const double *x, const double *num,
                          const double *h, double *y, double *part, const int32_t *flags, int64_t pstride)
{
    const unsigned pg = project_grid(d, pstride);
    if (d->sell) {
        k_ds_project_sell<NB, CF, 8><<<pg, 256, 0, st>>>(d->sbase, d->spix, d->sco, d->wbar, d->ws, d->tw, x, num, h,
                                                        d->NO, d->npix, y, part, flags, pstride);
        return pg;
    }
    const void *co = CF ? (const void *)d->ocnt : (const void *)d->ow;
#define COMAP_PROJ(G) k_ds_project<G, NB, CF, U><<<pg, 256, 0, st>>>(d->orow, d->opix, co, d->wbar, d->ws, d->tw, x, \
                                                                     num, h, d->NO, d->npix, y, part, flags, pstride)
    switch (project_lanes(d)) {
    case 4: COMAP_PROJ(4); break;
    case 8: COMAP_PROJ(8); break;
    case 16: COMAP_PROJ(16); break;
    case 32: COMAP_PROJ(32); break;
    default: COMAP_PROJ(64);
    }
#undef COMAP_PROJ
    return pg;
}

template <int NB, bool CF>
unsigned launch_project_cf(const comap_destriper *d, hipStream_t st, const double *x, const double *num,
                           const double *h, double *y, double *part, const int32_t *flags, int64_t pstride)
{
    return d->proj_u == 8 ? launch_project_u<NB, CF, 8>(d, st, x, num, h, y, part, flags, pstride)
                          : launch_project_u<NB, CF, 4>(d, st, x, num, h, y, part, flags, pstride);
}

unsigned launch_project(const comap_destriper *d, hipStream_t st, const double *x, const double *num,
                        const double *h, double *y, double *part, const int32_t *flags, int64_t pstride = kPartMax)
{
    unsigned pg = 0;
    if (d->cf) {
        COMAP_NB_SWITCH(d->nb, (pg = launch_project_cf<NB, true>(d, st, x, num, h, y, part, flags, pstride)));
    } else {
        COMAP_NB_SWITCH(d->nb, (pg = launch_project_cf<NB, false>(d, st, x, num, h, y, part, flags, pstride)));
    }
    return pg;
}

// a problem's persistent buffers come from the cached device pool (comap_tmp_alloc) in
// the context stream's order; comap_destripe_destroy returns them after a device sync
template <typename T>
int dalloc(comap_ctx *ctx, T **p, size_t n)
{
    void *q = nullptr;
    COMAP_CHECK(ctx, comap_tmp_alloc(&q, sizeof(T) * (n ? n : 1), ctx->stream));
    *p = (T *)q;
    return 0;
}

int dot(comap_destriper *d, hipStream_t st, const double *a, const double *b, double *out, const int32_t *flags)
{
    comap_ctx *ctx = d->ctx;
    COMAP_NB_SWITCH(d->nb, k_dot_part<NB><<<kRedBlocks, 256, 0, st>>>(a, b, d->NO, d->part);
                    k_dot_final<NB><<<1, 256, 0, st>>>(d->part, kRedBlocks, out, flags));
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}

// destroys a partly built problem on every early return of comap_destripe_create_bands
struct ProblemOwner {
    comap_destriper *d;
    ~ProblemOwner()
    {
        if (d) comap_destripe_destroy(d);
    }
};

// One device allocation carved into the set-up's scratch arrays (256-B aligned), so the
// set-up makes one hipMalloc / hipFree pair for its temporaries instead of one per array.
struct Arena {
    char *base = nullptr;
    size_t used = 0, cap = 0;
    template <typename T>
    T *take(size_t n)
    {
        const size_t b = (sizeof(T) * (n ? n : 1) + 255) & ~(size_t)255;
        T *p = reinterpret_cast<T *>(base + used);
        used += b;
        return p;
    }
    template <typename T>
    static size_t bytes(size_t n) { return (sizeof(T) * (n ? n : 1) + 255) & ~(size_t)255; }
};

}  // namespace

// Set-up of the constant operator (pointing and weights do not change during CG):
//   1. spatial offset order: first on-map pixel per offset, stable radix sort -> perm
//   2. k_ds_rows count pass: kept entries per row, ws / tw, the sample sort keys and
//      the packed sample payload; scan -> orow; nnz back to the host (sync 1)
//   3. k_ds_rows fill pass: the offset-major entries + the transpose's keys
//   4. pixel-major transpose: stable radix sort of the entries by pixel, row pointers,
//      gathered entry weights, the non-empty row list
//   5. sample-level maps: stable radix sort of the samples by pixel, ordered walk
//   nnzp and the non-empty row count back to the host (sync 2).
extern "C" int comap_destripe_create_bands(comap_ctx *ctx, const int32_t *pix, const double *tod, const double *w,
                                           const uint8_t *keep, int64_t N, int32_t L, int64_t npix, int32_t nb,
                                           comap_destriper **out)
{
    return comap_destripe_create_keyed(ctx, pix, tod, w, keep, nullptr, 0, N, L, npix, nb, out);
}

extern "C" int comap_destripe_create_keyed(comap_ctx *ctx, const int32_t *pix, const double *tod, const double *w,
                                           const uint8_t *keep, const int32_t *okey, int64_t okey_max, int64_t N,
                                           int32_t L, int64_t npix, int32_t nb, comap_destriper **out)
{
    if (!ctx || !pix || !tod || !w || !out) return -1;
    COMAP_DEVICE_GUARD(ctx);
    *out = nullptr;
    if (nb != 1 && nb != 2 && nb != 4) return comap_fail(ctx, -1, "bands per problem must be 1, 2 or 4");
    if (L < 1 || L > 256) return comap_fail(ctx, -1, "offset_length must be in [1, 256]");
    if (N <= 0 || N % L) return comap_fail(ctx, -1, "n_samples must be a positive multiple of offset_length");
    // (npix below the SELL padding id's magnitude, so no pixel id in [-npix, npix) is the pad)
    if (npix <= 0 || npix >= 0x7f7f7f7fll || N >= (1ll << 31)) return comap_fail(ctx, -1, "size limits exceeded");
    hipStream_t st = ctx->stream;
    auto *d = new comap_destriper();
    d->ctx = ctx; d->N = N; d->L = L; d->NO = N / L; d->npix = npix; d->nb = nb;
    const int64_t NO = d->NO;
    const size_t NB = (size_t)nb;
    ProblemOwner own{d};   // frees d on every early return; released at the end
    int rc = 0;
    rc |= dalloc(ctx, &d->orow, NO + 1);
    rc |= dalloc(ctx, &d->ws, NO * NB);
    rc |= dalloc(ctx, &d->tw, NO * NB);
    rc |= dalloc(ctx, &d->wbar, NO * NB);
    rc |= dalloc(ctx, &d->pt, NO * NB);
    rc |= dalloc(ctx, &d->prow, npix + 1);
    rc |= dalloc(ctx, &d->h, npix * NB);
    rc |= dalloc(ctx, &d->hits, npix * NB);
    rc |= dalloc(ctx, &d->nnum, npix * NB);
    rc |= dalloc(ctx, &d->part, 2 * NB * (size_t)kPartMax);   // [0, NB kPartMax): p.q / dots, then r.r of the fused CG
    rc |= dalloc(ctx, &d->scal, 4 * NB + 4);
    rc |= dalloc(ctx, &d->hrow, npix);
    rc |= dalloc(ctx, &d->hprow, npix + 1);
    const char *ord = getenv("COMAP_DS_ORDER");          // 0: keep the offsets in time order
    const bool spatial = !(ord && ord[0] == '0');
    if (spatial) rc |= dalloc(ctx, &d->perm, NO);
    if (rc) return -2;
    int end_bit = 1;
    while ((1ll << end_bit) <= npix) ++end_bit;
    if (okey && (okey_max < 1 || okey_max >= (1ll << 31))) return comap_fail(ctx, -1, "okey_max must be in [1, 2^31)");
    int key_bit = 1;          // radix bits of the offset order keys (the caller's bound, or npix)
    while ((1ll << key_bit) <= (okey ? okey_max - 1 : npix)) ++key_bit;
    // ---- scratch: sizes first (hipcub temp storage for the largest sort / scan), one allocation
    size_t sort_tb = 0, scan_tb = 0, scan32_tb = 0;
    (void)sort_pairs_i32(false, nullptr, sort_tb, nullptr, nullptr, nullptr, nullptr, N, end_bit, st);
    {
        size_t tb9 = 0;       // the spatial offset sort (NO pairs)
        (void)sort_pairs_i32(true, nullptr, tb9, nullptr, nullptr, nullptr, nullptr, NO, key_bit, st);
        sort_tb = std::max(sort_tb, tb9);
    }
    size_t sort64_tb = 0;   // the count form's transpose: (pixel, u64 offset|counts) pairs
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, sort64_tb, (int32_t *)nullptr, (int32_t *)nullptr,
                                             (uint64_t *)nullptr, (uint64_t *)nullptr, (int)N, 0, end_bit, st);
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, scan_tb, (int64_t *)nullptr, (int64_t *)nullptr, (int)(NO + 1), st);
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, scan32_tb, (int32_t *)nullptr, (int32_t *)nullptr, (int)npix, st);
    const size_t cub_tb = std::max({sort_tb, sort64_tb, scan_tb, scan32_tb});
    const int KW = L <= 64 ? 1 : (L <= 128 ? 2 : 4);     // member-mask words per entry (k_ds_rows' K)
    const int64_t rec_words = KW == 1 ? 2 : (KW == 2 ? 4 : 6);   // sizeof(SlotRec<KW>) / 8
    Arena ar;
    ar.cap = Arena::bytes<char>(cub_tb) + Arena::bytes<int64_t>(NO + 1) + 8 * Arena::bytes<int32_t>(N) +
             Arena::bytes<double>((size_t)N * 2 * NB) + Arena::bytes<int64_t>(npix + 1) +
             3 * Arena::bytes<int32_t>(npix) + Arena::bytes<int64_t>(8) + Arena::bytes<int32_t>(N) +
             Arena::bytes<int32_t>(1) + 2 * Arena::bytes<uint64_t>(N) + Arena::bytes<int64_t>(NO / 32 + 2) +
             Arena::bytes<uint64_t>((size_t)N * rec_words) +
             Arena::bytes<uint32_t>((size_t)npix * NB) +
             2 * Arena::bytes<int64_t>(NO + 1) + Arena::bytes<int32_t>(2) + Arena::bytes<uint8_t>(NO);
    COMAP_CHECK(ctx, comap_tmp_alloc((void **)&ar.base, ar.cap, st));
    struct ArenaFree {
        Arena *a;
        hipStream_t s;
        ~ArenaFree()
        {
            (void)hipStreamSynchronize(s);
            comap_tmp_free_on((void *const *)&a->base, 1, s, true);
        }
    } arena_free{&ar, st};
    char *cub_tmp = ar.take<char>(cub_tb);
    int64_t *cnt = ar.take<int64_t>(NO + 1);
    int32_t *skey = ar.take<int32_t>(N), *sval = ar.take<int32_t>(N);      // samples by pixel (sort in)
    int32_t *skey2 = ar.take<int32_t>(N), *sval2 = ar.take<int32_t>(N);    // (sort out)
    int32_t *ekey = ar.take<int32_t>(N), *eval = ar.take<int32_t>(N);      // entries by pixel (nnz <= N)
    int32_t *ekey2 = ar.take<int32_t>(N), *eval2 = ar.take<int32_t>(N);
    int32_t *eoff = ar.take<int32_t>(N);
    double *payload = ar.take<double>((size_t)N * 2 * NB);
    int64_t *srow = ar.take<int64_t>(npix + 1);
    int32_t *hflag = ar.take<int32_t>(npix), *hpos = ar.take<int32_t>(npix);
    int32_t *hheavy = ar.take<int32_t>(npix);   // the walk's heavy rows (indices into hrow)
    int64_t *counts = ar.take<int64_t>(8);      // [nnzp, nh] (k_hit_rows); first the set-up sizes (k_setup_sizes)
    int32_t *nonuni = ar.take<int32_t>(1);
    uint64_t *epay = ar.take<uint64_t>(N), *epay2 = ar.take<uint64_t>(N);   // count form: offset << 32 | counts
    const int64_t NC = (NO + 31) / 32;                      // sliced-ELLPACK chunks (at most, CW >= 32)
    int64_t *swid = ar.take<int64_t>(NC + 1);
    // member-mask walk (count form): slot / entry member masks, integer hits of the groups
    // without an entry, the transpose's rows in the caller's offset order
    void *srec = ar.take<uint64_t>((size_t)N * rec_words);       // SlotRec<KW> per slot
    uint32_t *hextra = ar.take<uint32_t>((size_t)npix * NB);
    int64_t *cnt_nat = ar.take<int64_t>(NO + 1), *orow_nat = ar.take<int64_t>(NO + 1);
    int32_t *nonfin = ar.take<int32_t>(2);       // [non-finite tod, pixel index >= npix]
    uint8_t *kint = keep ? ar.take<uint8_t>(NO) : nullptr;   // keep bits by internal offset (sample walk)
    bool walk = true;
    {
        const char *we = getenv("COMAP_DS_WALK");        // 0: the sorted-sample payload walk
        walk = !(we && we[0] == '0');
    }
    // ---- 1. spatial processing order of the offsets
    if (spatial) {
        // the caller's keys (comap_offset_centroid_keys: the centroid's internal pixel), or
        // the first on-map pixel of each offset
        if (okey)     // the sort's values only: a thread per offset
            k_iota32<<<grid_for(NO, 8192), 256, 0, st>>>(eval, NO);
        else
            k_offset_keys<<<(unsigned)std::min<int64_t>((NO + 3) / 4, 65536), 256, 0, st>>>(pix, NO, L, npix, ekey,
                                                                                             eval);
        COMAP_LAUNCH_CHECK(ctx);
        size_t tb = cub_tb;
        // (the caller's keys may exceed npix -- a compacted problem keeps its tiled-layout
        // keys -- so they sort on the bits of the caller's bound)
        COMAP_CHECK(ctx, sort_pairs_i32(true, cub_tmp, tb, okey ? okey : ekey, ekey2, eval, d->perm, NO, key_bit, st));
    }
    // ---- 2. count pass (+ the count-form test: non-zero weights uniform per offset and band)
    COMAP_CHECK(ctx, hipMemsetAsync(nonuni, 0, 4, st));
    // (eval / eoff: the count-form fill's entry slots, unused by the f64 path until its
    // own fill pass overwrites them).  Member-mask walk: no per-sample payload or sample
    // sort keys, but the slots' member masks, the empty groups' hits and the tod check
    auto count_pass = [&](bool with_payload) {
        COMAP_NB_SWITCH(nb, (launch_rows<NB, false, false>(
                                L, st, pix, w, tod, N, NO, npix, d->perm, cnt, d->ws, d->tw,
                                payload, skey, sval, d->wbar, nonuni, nullptr, nullptr,
                                nullptr, nullptr, nullptr, eval, eoff, nullptr, with_payload ? nullptr : srec,
                                with_payload ? nullptr : hextra, keep, nonfin)));
    };
    COMAP_CHECK(ctx, hipMemsetAsync(nonfin, 0, 8, st));
    if (walk) {
        COMAP_CHECK(ctx, hipMemsetAsync(hextra, 0, 4 * (size_t)npix * NB, st));
    }
    count_pass(!walk);
    COMAP_LAUNCH_CHECK(ctx);
    COMAP_CHECK(ctx, hipMemsetAsync(cnt + NO, 0, 8, st));
    COMAP_CHECK(ctx, hipcub::DeviceScan::ExclusiveSum(cub_tmp, scan_tb, cnt, d->orow, (int)(NO + 1), st));
    if (walk) {
        k_cnt_natural<<<grid_for(NO + 1, 8192), 256, 0, st>>>(cnt, d->perm, NO, cnt_nat);
        COMAP_LAUNCH_CHECK(ctx);
        COMAP_CHECK(ctx, hipcub::DeviceScan::ExclusiveSum(cub_tmp, scan_tb, cnt_nat, orow_nat, (int)(NO + 1), st));
        k_nat_base<<<grid_for(NO, 8192), 256, 0, st>>>(orow_nat, d->perm, NO, cnt_nat);   // (cnt_nat is free)
        COMAP_LAUNCH_CHECK(ctx);
    }
    {
        // sliced-ELLPACK projection: default for large problems (C5, 547k offsets: 1 band
        // 0.112 -> 0.098 ms per CG iteration, 4 bands 0.261 -> 0.236, r04j); a C4-size problem
        // (35k offsets) gains nothing its extra set-up pass would not cost.  COMAP_DS_SELL=0/1
        const char *se = getenv("COMAP_DS_SELL");
        d->sell = se ? se[0] == '1' : NO >= kSellMinOffsets;
    }
    int64_t NCs = NC;
    if (d->sell) {
        NCs = (NO + 63) / 64;
        if (dalloc(ctx, &d->sbase, NCs + 1)) return -2;
        const unsigned wg = (unsigned)(((NCs + 1) * 64 + 255) / 256);
        k_sell_width<<<wg, 256, 0, st>>>(d->orow, NO, NCs, swid);
        COMAP_LAUNCH_CHECK(ctx);
        COMAP_CHECK(ctx, hipcub::DeviceScan::ExclusiveSum(cub_tmp, scan_tb, swid, d->sbase, (int)(NCs + 1), st));
    }
    // one read-back into a page-locked block (sizes + flags), one sync
    struct PinnedWords {
        int64_t *p = nullptr;
        ~PinnedWords() { if (p) comap_pinned_free(p); }
    } hw;
    COMAP_CHECK(ctx, comap_pinned_alloc((void **)&hw.p, 8 * 8));
    k_setup_sizes<<<1, 64, 0, st>>>(d->orow, NO, d->sell ? d->sbase : nullptr, NCs, nonuni, nonfin, counts);
    COMAP_LAUNCH_CHECK(ctx);
    COMAP_CHECK(ctx, hipMemcpyAsync(hw.p, counts, 5 * 8, hipMemcpyDeviceToHost, st));
    COMAP_CHECK(ctx, hipStreamSynchronize(st));
    d->nnz = hw.p[0];
    if (d->sell) d->nsell = hw.p[1];
    const int32_t nonuni_h = (int32_t)hw.p[2], nonfin_h = (int32_t)hw.p[3];
    if (hw.p[4]) return comap_fail(ctx, -3, "pixel index out of range for the map (>= npix or < -npix)");
    {
        const char *cfe = getenv("COMAP_DS_CF");             // 0: always the f64 entry weights
        d->cf = !nonuni_h && L <= 255 && !(cfe && cfe[0] == '0');
        // launch-shape overrides (measurement knobs; invalid values keep the defaults)
        auto env_int = [](const char *k, int dflt, std::initializer_list<int> ok) {
            const char *v = getenv(k);
            if (!v) return dflt;
            const int x = atoi(v);
            for (int o : ok)
                if (x == o) return x;
            return dflt;
        };
        d->bin_lanes = env_int("COMAP_DS_BL", 0, {4, 8, 16, 32, 64});
        // long pixel rows (the field: 376 entries per pixel) keep 8 entry loads in flight per
        // bin lane, and a problem of millions of offsets runs its SELL projection at 8192
        // blocks (field 4 bands: 1.446 -> 1.380 ms per iteration; C5 1 / 4 bands unchanged,
        // profiles/r06/r06cg).  Neither changes a result: a bin lane adds its entries in the
        // same order, and single-rank p.q partials are re-summed in one fixed order.
        const bool long_rows = d->nnz >= 256 * npix;
        d->bin_u = env_int("COMAP_DS_BU", long_rows ? 8 : 4, {4, 8});
        d->proj_lanes = env_int("COMAP_DS_PG", 0, {4, 8, 16, 32, 64});
        d->proj_u = env_int("COMAP_DS_PU", 4, {4, 8});
        // the SELL projection runs one chunk per wave at 2048 blocks (1024: 0.254 vs 0.244 ms per
        // 4-band C5 iteration, r04h); its p.q partials fit kPartMax and the dist slots below
        d->proj_blocks = env_int("COMAP_DS_PB", d->sell ? (NO >= (2 << 20) ? 8192 : 2 * kProjBlocks) : kProjBlocks,
                                 {256, 512, 1024, 2048, 4096, 8192});
        d->cg_graph = env_int("COMAP_DS_CGGRAPH", -1, {0, 1});
    }
    // the member-mask walk needs the count form and finite tod everywhere; otherwise the
    // count pass runs again with the per-sample payload for the sorted-sample walk
    if (walk && (!d->cf || nonfin_h)) {
        walk = false;
        count_pass(true);
        COMAP_LAUNCH_CHECK(ctx);
    }
    rc |= dalloc(ctx, &d->opix, d->nnz);
    rc |= dalloc(ctx, &d->poff, d->nnz);          // nnzp <= nnz (off-map entries are not binned)
    if (d->cf) {
        rc |= dalloc(ctx, &d->ocnt, d->nnz * NB);
        rc |= dalloc(ctx, &d->pcnt, d->nnz * NB);
    } else {
        rc |= dalloc(ctx, &d->ow, d->nnz * NB);
        rc |= dalloc(ctx, &d->pw, d->nnz * NB);
    }
    if (rc) return -2;
    // ---- 3. fill pass
    int32_t *evn = skey2, *evn2 = sval2;   // walk: the sample-sort arrays are free
    if (walk) {
#define COMAP_CW(KK) k_ds_compact_walk<NB, KK><<<(unsigned)((NO + 15) / 16), 256, 0, st>>>(                     \
        d->orow, cnt_nat, nullptr, NO, L, npix, (const SlotRec<KK> *)srec, d->opix, d->ocnt, ekey, evn)
        if (KW == 1) { COMAP_NB_SWITCH(nb, COMAP_CW(1)); }
        else if (KW == 2) { COMAP_NB_SWITCH(nb, COMAP_CW(2)); }
        else { COMAP_NB_SWITCH(nb, COMAP_CW(4)); }
#undef COMAP_CW
    } else if (d->cf) {
        COMAP_NB_SWITCH(nb, (k_ds_compact_cf<NB><<<(unsigned)((NO + 3) / 4), 256, 0, st>>>(
                                d->orow, NO, L, npix, eval, eoff, d->opix, d->ocnt, ekey, epay)));
    } else {
        COMAP_NB_SWITCH(nb, (launch_rows<NB, true, false>(L, st, pix, w, tod, N, NO, npix, d->perm, nullptr, nullptr,
                                                          nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, d->orow,
                                                          d->opix, d->ow, nullptr, ekey, eval, eoff)));
    }
    COMAP_LAUNCH_CHECK(ctx);
    if (d->sell) {
        if (dalloc(ctx, &d->spix, d->nsell)) return -2;
        if (d->cf ? dalloc(ctx, (uint8_t **)&d->sco, d->nsell * NB) : dalloc(ctx, (double **)&d->sco, d->nsell * NB))
            return -2;
        const unsigned nch = (unsigned)((NO + 63) / 64);
        if (d->cf) {
            COMAP_NB_SWITCH(nb, (k_sell_fill_lds<NB, true><<<nch, 256, 0, st>>>(
                                    d->orow, d->opix, d->ocnt, d->sbase, NO, d->spix, d->sco)));
        } else {
            COMAP_NB_SWITCH(nb, (k_sell_fill_lds<NB, false><<<nch, 256, 0, st>>>(
                                    d->orow, d->opix, d->ow, d->sbase, NO, d->spix, d->sco)));
        }
        COMAP_LAUNCH_CHECK(ctx);
    }
    // ---- 4. pixel-major transpose (stable: offset order within a pixel)
    if (walk) {
        size_t tb = cub_tb;
        COMAP_CHECK(ctx, sort_pairs_i32(false, cub_tmp, tb, ekey, ekey2, evn, evn2, d->nnz, end_bit, st));
    } else if (d->cf) {
        COMAP_CHECK(ctx, hipcub::DeviceRadixSort::SortPairs(cub_tmp, sort64_tb, ekey, ekey2, epay, epay2, (int)d->nnz,
                                                            0, end_bit, st));
    } else {
        COMAP_CHECK(ctx, hipcub::DeviceRadixSort::SortPairs(cub_tmp, sort_tb, ekey, ekey2, eval, eval2, (int)d->nnz, 0,
                                                            end_bit, st));
    }
    k_rowptr<<<grid_for(npix + 1), 256, 0, st>>>(ekey2, d->nnz, npix, d->prow);
    COMAP_LAUNCH_CHECK(ctx);
    if (walk) {
        // (the sample walk below writes the pixel-major offsets / counts)
    } else if (d->cf) {
        COMAP_NB_SWITCH(nb, k_pixel_entries_cf<NB><<<grid_for(d->nnz, 8192), 256, 0, st>>>(epay2, d->prow + npix,
                                                                                            d->poff, d->pcnt));
    } else {
        COMAP_NB_SWITCH(nb, k_pixel_entries<NB><<<grid_for(d->nnz, 8192), 256, 0, st>>>(eval2, d->prow + npix, eoff,
                                                                                         d->ow, d->ocnt, d->poff, d->pw,
                                                                                         d->pcnt));
    }
    COMAP_LAUNCH_CHECK(ctx);
    k_hit_flags<<<grid_for(npix), 256, 0, st>>>(d->prow, npix, hflag, nb, hextra, walk ? d->h : nullptr, d->hits,
                                                d->nnum, counts);
    COMAP_LAUNCH_CHECK(ctx);
    COMAP_CHECK(ctx, hipcub::DeviceScan::ExclusiveSum(cub_tmp, scan32_tb, hflag, hpos, (int)npix, st));
    // the walk's heavy rows: more entries than kHeavyRow (the Lissajous turn-round pixels hold
    // up to ~100x the mean; walked last they set the kernel's tail)
    k_hit_rows<<<grid_for(npix), 256, 0, st>>>(d->prow, hflag, hpos, npix, d->hrow, d->hprow, counts,
                                               heavy_env(), walk && heavy_env() > 0 ? hheavy : nullptr);
    COMAP_LAUNCH_CHECK(ctx);
    // ---- 5. sample-level maps (binValues order)
    const unsigned wgrid = (unsigned)std::min<int64_t>((npix + 3) / 4, 65536);
    if (walk) {
        if (kint) {
            k_keep_bits<<<grid_for(NO, 8192), 256, 0, st>>>(keep, d->perm, NO, nb, kint);
            COMAP_LAUNCH_CHECK(ctx);
        }
        // member slots per lane and chunk: 64 KW (one entry's members fit a chunk); one wave per
        // row (a fixed 2048-block grid: C5 0.80 -> 1.04 ms)
#define COMAP_W2(KK, MM) (walk_pf_env() ? k_sample_walk2<NB, KK, MM, true> \
                                         : k_sample_walk2<NB, KK, MM, false>)<<<wgrid, 256, 0, st>>>(                                   \
        d->hrow, d->hprow, counts, evn2, (const SlotRec<KK> *)srec, d->perm, d->wbar, w, payload, N, npix, L, NO, kint, \
        hextra, d->h, d->hits, d->nnum, d->poff, d->pcnt, heavy_env() > 0 ? hheavy : nullptr, heavy_env(), \
        walk_xcd_env())
        if (KW == 1) { COMAP_NB_SWITCH(nb, COMAP_W2(1, 1)); }
        else if (KW == 2) { COMAP_NB_SWITCH(nb, COMAP_W2(2, 2)); }
        else { COMAP_NB_SWITCH(nb, COMAP_W2(4, 4)); }
#undef COMAP_W2
    } else {
        COMAP_CHECK(ctx, hipcub::DeviceRadixSort::SortPairs(cub_tmp, sort_tb, skey, skey2, sval, sval2, (int)N, 0,
                                                            end_bit, st));
        k_rowptr<<<grid_for(npix + 1), 256, 0, st>>>(skey2, N, npix, srow);
        COMAP_LAUNCH_CHECK(ctx);
        COMAP_NB_SWITCH(nb, k_sample_walk<NB><<<wgrid, 256, 0, st>>>(srow, sval2, payload, npix, L, NO, keep, d->h,
                                                                     d->hits, d->nnum));
    }
    COMAP_LAUNCH_CHECK(ctx);
    d->walk = walk;
    COMAP_CHECK(ctx, hipMemcpyAsync(hw.p, counts, 16, hipMemcpyDeviceToHost, st));
    COMAP_CHECK(ctx, hipStreamSynchronize(st));
    d->nnzp = hw.p[0];
    d->nh = hw.p[1];
    own.d = nullptr;
    *out = d;
    return 0;
}

namespace {
__device__ __forceinline__ int32_t relabel_one(int32_t p32, const int32_t *__restrict__ lut, int64_t npix, int64_t nt)
{
    const int64_t p = p32;
    if (p >= npix || p < -npix) return (int32_t)nt;
    return p >= 0 ? lut[p] : (int32_t)((int64_t)lut[npix + p] - nt);
}

// The tiled layout's id of row-major pixel p (destriper.tiled_layout): T x T tiles in
// row-major tile order (ntx tiles a row), Morton order inside (bits of x at even, of y at
// odd positions) -- computed, not looked up: the table gathers ran at 1.9 TB/s on the field.
__device__ __forceinline__ int32_t tiled_id(int32_t p, int32_t nx, int32_t ntx, int tb, double inv)
{
    int32_t y = (int32_t)((double)p * inv);
    int32_t x = p - y * nx;
    if (x < 0) { --y; x += nx; }
    else if (x >= nx) { ++y; x -= nx; }
    const int32_t T = 1 << tb;
    const uint32_t ix = (uint32_t)(x & (T - 1)), iy = (uint32_t)(y & (T - 1));
    uint32_t z = 0;
    for (int b = 0; b < tb; ++b) z |= (((ix >> b) & 1u) << (2 * b)) | (((iy >> b) & 1u) << (2 * b + 1));
    return (((y >> tb) * ntx + (x >> tb)) << (2 * tb)) + (int32_t)z;
}

__device__ __forceinline__ int32_t relabel_tiled_one(int32_t p, int32_t npix, int32_t nx, int32_t ntx, int tb,
                                                     double inv, int32_t nt)
{
    if (p >= npix || p < -npix) return nt;
    return p >= 0 ? tiled_id(p, nx, ntx, tb, inv) : tiled_id(npix + p, nx, ntx, tb, inv) - nt;
}

__global__ void k_relabel_tiled(const int32_t *__restrict__ pix, int64_t n, int32_t npix, int32_t nx, int32_t ntx,
                                int tb, int32_t nt, int32_t *__restrict__ out)
{
    const double inv = 1.0 / (double)nx;
    const int64_t n4 = ((uintptr_t)pix % 16 == 0 && (uintptr_t)out % 16 == 0) ? n / 4 : 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t t0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    for (int64_t i = t0; i < n4; i += stride) {
        const int4 v = reinterpret_cast<const int4 *>(pix)[i];
        int4 r;
        r.x = relabel_tiled_one(v.x, npix, nx, ntx, tb, inv, nt);
        r.y = relabel_tiled_one(v.y, npix, nx, ntx, tb, inv, nt);
        r.z = relabel_tiled_one(v.z, npix, nx, ntx, tb, inv, nt);
        r.w = relabel_tiled_one(v.w, npix, nx, ntx, tb, inv, nt);
        reinterpret_cast<int4 *>(out)[i] = r;
    }
    for (int64_t i = 4 * n4 + t0; i < n; i += stride) out[i] = relabel_tiled_one(pix[i], npix, nx, ntx, tb, inv, nt);
}

// four ids per thread (16-B loads and stores; torch's blocks are 256-B aligned), the tail
// one by one
__global__ void k_relabel_pixels(const int32_t *__restrict__ pix, int64_t n, const int32_t *__restrict__ lut,
                                 int64_t npix, int64_t nt, int32_t *__restrict__ out)
{
    const int64_t n4 = ((uintptr_t)pix % 16 == 0 && (uintptr_t)out % 16 == 0) ? n / 4 : 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t t0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    for (int64_t i = t0; i < n4; i += stride) {
        const int4 v = reinterpret_cast<const int4 *>(pix)[i];
        int4 r;
        r.x = relabel_one(v.x, lut, npix, nt);
        r.y = relabel_one(v.y, lut, npix, nt);
        r.z = relabel_one(v.z, lut, npix, nt);
        r.w = relabel_one(v.w, lut, npix, nt);
        reinterpret_cast<int4 *>(out)[i] = r;
    }
    for (int64_t i = 4 * n4 + t0; i < n; i += stride) out[i] = relabel_one(pix[i], lut, npix, nt);
}
}  // namespace

// key[o] = lut[round(mean y) nx + round(mean x)] over offset o's on-map samples
// (0 <= p < nx ny, row-major ids), n_internal when it has none.  One wave per offset, a lane
// per sample (coalesced), 32-bit sums reduced across the wave; p = y nx + x by a double
// reciprocal and one integer fix-up (exact for p < 2^31).  (64-bit divisions and sums took
// 1.7 ms on the field's 4.38 M offsets, a thread per offset with strided loads as long,
// profiles/r06/r06c-d.)
__global__ void __launch_bounds__(256) k_offset_centroid_keys(const int32_t *__restrict__ pix, int64_t NO, int L,
                                                              int32_t nx, int32_t ny, const int32_t *__restrict__ lut,
                                                              int32_t n_internal, int32_t *__restrict__ key)
{
    const int lane = threadIdx.x & 63;
    const double inv = 1.0 / (double)nx;
    const int32_t npix = nx * ny;
    // L <= 64 (one sample per lane) and per-offset coordinate sums below 2^16
    const bool packed = L <= 64 && (int64_t)L * (nx - 1) < 65536 && (int64_t)L * (ny - 1) < 65536;
    for (int64_t o = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); o < NO; o += (int64_t)gridDim.x * 4) {
        int32_t sy = 0, sx = 0, c = 0;
        for (int j = lane; j < L; j += 64) {
            const int32_t p = pix[o * L + j];
            if (p >= 0 && p < npix) {
                int32_t y = (int32_t)((double)p * inv);
                int32_t x = p - y * nx;
                if (x < 0) { --y; x += nx; }
                else if (x >= nx) { ++y; x -= nx; }
                sy += y;
                sx += x;
                c += 1;
            }
        }
        if (packed) {
            // y in the low, x in the high 16 bits (their offset sums fit): one DPP scan, the
            // count by a ballot -- no LDS permutes
            const uint32_t t = wave_incl_scan((uint32_t)sy | ((uint32_t)sx << 16));
            const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)t, 63);
            sy = (int32_t)(tot & 0xffffu);
            sx = (int32_t)(tot >> 16);
            c = __popcll(__ballot(c != 0));
        } else {
#pragma unroll
            for (int sh = 32; sh > 0; sh >>= 1) {
                sy += __shfl_xor(sy, sh, 64);
                sx += __shfl_xor(sx, sh, 64);
                c += __shfl_xor(c, sh, 64);
            }
        }
        if (lane == 0) {
            int32_t k = n_internal;
            if (c > 0) {
                const int32_t yi = (2 * sy + c) / (2 * c), xi = (2 * sx + c) / (2 * c);   // round half up
                k = lut[yi * nx + xi];
            }
            key[o] = k;
        }
    }
}

// The same keys for L <= 64, a block per 128 offsets: the block's 128 L pixel ids are one
// contiguous run, staged in LDS by coalesced loads (every load of the block in flight at
// once), then a thread per offset sums its samples from LDS -- one memory round trip per
// 128 offsets instead of one per offset (the wave-per-offset kernel above: 765 us on the
// field's 4.38 M offsets, latency-bound at 1.1 TB/s).
constexpr int kCkOffsets = 128;
__global__ void __launch_bounds__(256) k_offset_centroid_keys_lds(const int32_t *__restrict__ pix, int64_t NO, int L,
                                                                  int32_t nx, int32_t ny,
                                                                  const int32_t *__restrict__ lut, int32_t n_internal,
                                                                  int32_t *__restrict__ key)
{
    __shared__ int32_t sp[kCkOffsets * 64];
    const int64_t o0 = (int64_t)blockIdx.x * kCkOffsets;
    const int no = (int)min<int64_t>(kCkOffsets, NO - o0);
    const int cnt = no * L;
    const int32_t *src = pix + o0 * L;
    for (int i = threadIdx.x; i < cnt; i += 256) sp[i] = src[i];
    __syncthreads();
    const int t = threadIdx.x;
    if (t >= no) return;
    const double inv = 1.0 / (double)nx;
    const int32_t npix = nx * ny;
    int32_t sy = 0, sx = 0, c = 0;
    for (int j = 0; j < L; ++j) {
        const int32_t p = sp[t * L + j];
        if (p >= 0 && p < npix) {
            int32_t y = (int32_t)((double)p * inv);
            int32_t x = p - y * nx;
            if (x < 0) { --y; x += nx; }
            else if (x >= nx) { ++y; x -= nx; }
            sy += y;
            sx += x;
            c += 1;
        }
    }
    int32_t k = n_internal;
    if (c > 0) {
        const int32_t yi = (2 * sy + c) / (2 * c), xi = (2 * sx + c) / (2 * c);   // round half up
        k = lut[yi * nx + xi];
    }
    key[o0 + t] = k;
}

extern "C" int comap_offset_centroid_keys(comap_ctx *ctx, const int32_t *pix, int64_t n, int32_t L, int64_t nx,
                                          int64_t ny, const int32_t *lut, int64_t n_internal, int32_t *key)
{
    if (!ctx || L < 1 || n < 0 || n % L || nx < 1 || ny < 1 || n_internal < nx * ny || n_internal >= (1ll << 31) ||
        (n > 0 && (!pix || !lut || !key)))
        return -1;
    COMAP_DEVICE_GUARD(ctx);
    const int64_t NO = n / L;
    if (NO == 0) return 0;
    if ((int64_t)L * (nx - 1 + ny - 1) >= (1ll << 30) / 2)     // the per-offset int32 sums
        return comap_fail(ctx, -1, "comap_offset_centroid_keys: map too large for the offset length");
    if (L <= 64 && (NO + kCkOffsets - 1) / kCkOffsets < (1ll << 31))
        k_offset_centroid_keys_lds<<<(unsigned)((NO + kCkOffsets - 1) / kCkOffsets), 256, 0, ctx->stream>>>(
            pix, NO, L, (int32_t)nx, (int32_t)ny, lut, (int32_t)n_internal, key);
    else
        k_offset_centroid_keys<<<(unsigned)std::min<int64_t>((NO + 3) / 4, 65536), 256, 0, ctx->stream>>>(
            pix, NO, L, (int32_t)nx, (int32_t)ny, lut, (int32_t)n_internal, key);
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}

extern "C" int comap_relabel_pixels(comap_ctx *ctx, const int32_t *pix, int64_t n, const int32_t *lut, int64_t npix,
                                    int64_t n_internal, int32_t *out)
{
    if (!ctx || (n > 0 && (!pix || !lut || !out)) || n < 0 || npix <= 0 || n_internal < npix ||
        n_internal >= (1ll << 31))
        return -1;
    COMAP_DEVICE_GUARD(ctx);
    if (n == 0) return 0;
    k_relabel_pixels<<<grid_for((n + 3) / 4, 16384), 256, 0, ctx->stream>>>(pix, n, lut, npix, n_internal, out);
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}

extern "C" int comap_relabel_pixels_tiled(comap_ctx *ctx, const int32_t *pix, int64_t n, int64_t nx, int64_t ny,
                                          int32_t T, int32_t *out)
{
    if (!ctx || (n > 0 && (!pix || !out)) || n < 0 || nx < 1 || ny < 1 || T < 1 || (T & (T - 1)))
        return -1;
    int tb = 0;
    while ((1 << tb) < T) ++tb;
    const int64_t ntx = (nx + T - 1) / T, nty = (ny + T - 1) / T, nt = ntx * nty * T * T;
    if (nt >= (1ll << 31)) return -1;
    COMAP_DEVICE_GUARD(ctx);
    if (n == 0) return 0;
    k_relabel_tiled<<<grid_for((n + 3) / 4, 16384), 256, 0, ctx->stream>>>(pix, n, (int32_t)(nx * ny), (int32_t)nx,
                                                                           (int32_t)ntx, tb, (int32_t)nt, out);
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}

extern "C" int comap_destripe_create(comap_ctx *ctx, const int32_t *pix, const double *tod, const double *w,
                                     int64_t N, int32_t L, int64_t npix, comap_destriper **out)
{
    return comap_destripe_create_bands(ctx, pix, tod, w, nullptr, N, L, npix, 1, out);
}

extern "C" int comap_destripe_destroy(comap_destriper *d)
{
    if (!d) return 0;
    COMAP_DEVICE_GUARD(d->ctx);
    // every stream that may still read the buffers (the CG stream, the caller's) is idle
    // after a device sync; the blocks then go back to the caches
    (void)hipDeviceSynchronize();
    void *b[] = {d->orow, d->opix, d->ow, d->ws, d->tw, d->prow, d->poff, d->pw, d->h, d->hits, d->nnum, d->part, d->scal,
                 d->cg, d->flags, d->hrow, d->hprow, d->perm, d->ocnt, d->pcnt, d->wbar, d->pt, d->sbase, d->spix,
                 d->sco};
    comap_tmp_free_on(b, (int)(sizeof(b) / sizeof(b[0])), nullptr, true);
    comap_pinned_free(d->flags_host);
    comap_pinned_free(d->thr_host);
    if (d->batch) (void)hipGraphExecDestroy(d->batch);
    if (d->ev) (void)hipEventDestroy(d->ev);
    comap_stream_release(d->cs);
    delete d;
    return 0;
}

extern "C" int64_t comap_destripe_n_offsets(const comap_destriper *d) { return d ? d->NO : -1; }
extern "C" int32_t comap_destripe_n_bands(const comap_destriper *d) { return d ? d->nb : -1; }

extern "C" int64_t comap_destripe_sell_entries(const comap_destriper *d) { return d && d->sell ? d->nsell : -1; }

extern "C" int32_t comap_destripe_entry_bytes(const comap_destriper *d)
{
    return d ? (d->cf ? 4 + d->nb : 4 + 8 * d->nb) : -1;
}

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
    const size_t b = 8 * (size_t)d->npix * d->nb;
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
        COMAP_NB_SWITCH(d->nb, k_dot_final<NB><<<1, 256, 0, ctx->stream>>>(d->part, (int)pg, dot_out, nullptr));
        COMAP_LAUNCH_CHECK(ctx);
    }
    return 0;
}

extern "C" int comap_destripe_dot(comap_destriper *d, const double *a, const double *b, double *out)
{
    if (!d || !a || !b || !out) return -1;
    COMAP_DEVICE_GUARD(d->ctx);
    return dot(d, d->ctx->stream, a, b, out, nullptr);
}

extern "C" int comap_destripe_cg_update(comap_destriper *d, const double *rr, const double *pq, double *x, double *r,
                                        const double *p, const double *q, double *rr_new)
{
    if (!d) return -1;
    COMAP_DEVICE_GUARD(d->ctx);
    comap_ctx *ctx = d->ctx;
    COMAP_NB_SWITCH(d->nb, k_cg_update<NB><<<upd_grid(d->NO), 256, 0, ctx->stream>>>(rr, pq, x, r, p, q, d->NO, d->part,
                                                                                 nullptr);
                    k_dot_final<NB><<<1, 256, 0, ctx->stream>>>(d->part, (int)upd_grid(d->NO), rr_new, nullptr));
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}

extern "C" int comap_destripe_cg_direction(comap_destriper *d, const double *rr_new, const double *rr, double *p,
                                           const double *r)
{
    if (!d) return -1;
    COMAP_DEVICE_GUARD(d->ctx);
    comap_ctx *ctx = d->ctx;
    COMAP_NB_SWITCH(d->nb, k_cg_direction<NB><<<grid_for(d->NO), 256, 0, ctx->stream>>>(rr_new, rr, p, r, d->NO,
                                                                                         nullptr));
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}

extern "C" int comap_destripe_offsets_natural(comap_destriper *d, const double *x_internal, double *x_out)
{
    if (!d || !x_internal || !x_out || x_internal == x_out) return -1;
    COMAP_DEVICE_GUARD(d->ctx);
    comap_ctx *ctx = d->ctx;
    if (d->perm) {
        COMAP_NB_SWITCH(d->nb, k_unpermute<NB><<<grid_for(d->NO), 256, 0, ctx->stream>>>(x_internal, d->perm, d->NO,
                                                                                         x_out));
    } else {
        COMAP_CHECK(ctx, hipMemcpyAsync(x_out, x_internal, 8 * (size_t)d->NO * d->nb, hipMemcpyDeviceToDevice,
                                        ctx->stream));
    }
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}

extern "C" int comap_destripe_div_map(comap_destriper *d, const double *num, const double *h, double *out)
{
    if (!d || !num || !out) return -1;
    COMAP_DEVICE_GUARD(d->ctx);
    comap_ctx *ctx = d->ctx;
    const int64_t n = d->npix * d->nb;
    k_div_map<<<grid_for(n), 256, 0, ctx->stream>>>(num, h ? h : d->h, n, out);
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}

// ---------------------------------------------------------------- multi-rank CG pieces
// One CG iteration split at its three all-reduce points (map numerator, p.q,
// r.r), every kernel gated by the device stop flags so the host can queue a
// batch of iterations (with the collectives between the pieces) and check the
// flags once per batch.  Scalar / flag layout: see the top of this file.
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
    const int nb = d->nb;
    const unsigned pg = launch_project(d, ctx->stream, p, num, h, q, d->part, flags);
    COMAP_NB_SWITCH(nb, k_dot_final<NB><<<1, 256, 0, ctx->stream>>>(d->part, (int)pg, scal + 2 * nb, flags));
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}

extern "C" int comap_destripe_dist_update(comap_destriper *d, double *scal, double *x, double *r, const double *p,
                                          const double *q, const int32_t *flags)
{
    if (!d || !scal || !x || !r || !p || !q || !flags) return -1;
    COMAP_DEVICE_GUARD(d->ctx);
    comap_ctx *ctx = d->ctx;
    const int nb = d->nb;
    COMAP_NB_SWITCH(nb, k_cg_update<NB><<<upd_grid(d->NO), 256, 0, ctx->stream>>>(scal + nb, scal + 2 * nb, x, r, p, q,
                                                                              d->NO, d->part, flags);
                    k_dot_final<NB><<<1, 256, 0, ctx->stream>>>(d->part, (int)upd_grid(d->NO), scal + 3 * nb, flags));
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}

extern "C" int comap_destripe_dist_direction(comap_destriper *d, double *scal, double *p, const double *r,
                                             int32_t *flags)
{
    if (!d || !scal || !p || !r || !flags) return -1;
    COMAP_DEVICE_GUARD(d->ctx);
    comap_ctx *ctx = d->ctx;
    const int nb = d->nb;
    COMAP_NB_SWITCH(nb, k_cg_direction<NB><<<grid_for(d->NO), 256, 0, ctx->stream>>>(scal + 3 * nb, scal + nb, p, r,
                                                                                      d->NO, flags);
                    k_cg_check<NB><<<1, 64, 0, ctx->stream>>>(scal, flags));
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}

// Partial-sum variant of the multi-rank pieces: the native solve's kernels, with the p.q
// and r.r block partials (one slot per block, kDistParts per band, zero beyond the grid)
// all-reduced between them instead of final sums.  Adding the zero slots changes no bit,
// so on one rank the iterates equal comap_destripe_solve's.
constexpr int kDistParts = 1024;   // >= kProjBlocks, kUpdBlocks
static_assert(kDistParts >= kProjBlocks && kDistParts >= kUpdBlocks, "partial slots");

extern "C" int32_t comap_destripe_dist_parts(void) { return kDistParts; }

extern "C" int comap_destripe_dist_project_parts(comap_destriper *d, const double *p, const double *num,
                                                 const double *h, double *q, double *pq_part, const int32_t *flags)
{
    if (!d || !p || !num || !h || !q || !pq_part || !flags) return -1;
    COMAP_DEVICE_GUARD(d->ctx);
    comap_ctx *ctx = d->ctx;
    launch_project(d, ctx->stream, p, num, h, q, pq_part, flags, kDistParts);
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}

extern "C" int comap_destripe_dist_update_fused(comap_destriper *d, double *scal, const double *pq_part, double *x,
                                                double *r, const double *p, const double *q, double *rr_part,
                                                const int32_t *flags)
{
    if (!d || !scal || !pq_part || !x || !r || !p || !q || !rr_part || !flags) return -1;
    COMAP_DEVICE_GUARD(d->ctx);
    comap_ctx *ctx = d->ctx;
    COMAP_NB_SWITCH(d->nb, k_cg_update_fused<NB><<<upd_grid(d->NO), 256, 0, ctx->stream>>>(
                               scal, pq_part, kDistParts, x, r, p, q, d->NO, rr_part, flags, kDistParts));
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}

extern "C" int comap_destripe_dist_direction_fused(comap_destriper *d, double *scal, const double *rr_part, double *p,
                                                   const double *r, int32_t *flags)
{
    if (!d || !scal || !rr_part || !p || !r || !flags) return -1;
    COMAP_DEVICE_GUARD(d->ctx);
    comap_ctx *ctx = d->ctx;
    COMAP_NB_SWITCH(d->nb, k_cg_direction_fused<NB><<<grid_for(d->NO, kDirBlocks), 256, 0, ctx->stream>>>(
                               scal, rr_part, kDistParts, p, r, d->NO, flags, kDistParts));
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}

// ---------------------------------------------------------------- device-resident CG
// One CG iteration (Destriper.py:85-152 with p == pb, r == rb) on the problem's own
// vectors for every band; every kernel returns at once after all bands stopped.
static void enqueue_iteration(comap_destriper *d, hipStream_t st)
{
    const int64_t n = d->NO * d->nb;
    double *x = d->cg, *r = x + n, *p = r + n, *q = p + n, *num = q + n;
    const int32_t *flags = d->flags;
    // the bin writes the map m = (W p) / h itself, so the projection gathers one array
    // (count form: it bins pt = wbar o p, which the previous direction kernel wrote)
    launch_bin(d, st, d->cf ? d->pt : p, nullptr, d->h, num, flags, true, d->cf);   // empty rows of num stay 0
    // 4 launches per iteration: the p.q / r.r finals and the stop test are folded into
    // the update and direction kernels (same arithmetic and order as k_dot_final + k_cg_check)
    const unsigned pg = launch_project(d, st, p, num, nullptr, q, d->part, flags);
    double *part_rr = d->part + (size_t)d->nb * kPartMax;
    COMAP_NB_SWITCH(d->nb,
                    k_cg_update_fused<NB><<<upd_grid(d->NO), 256, 0, st>>>(d->scal, d->part, (int)pg, x, r, p, q,
                                                                           d->NO, part_rr, flags);
                    k_cg_direction_fused<NB><<<grid_for(d->NO, kDirBlocks), 256, 0, st>>>(
                        d->scal, part_rr, (int)upd_grid(d->NO), p, r, d->NO, d->flags, kPartMax,
                        d->cf ? d->wbar : nullptr, d->cf ? d->pt : nullptr));
}

// graph replay pays when an iteration's kernels are shorter than enqueueing them
// (~20 us of host time for 4 launches): below ~300k entries (C4's 4-band iteration of
// 0.5 M entries already runs 34 us)
static bool cg_use_graph(const comap_destriper *d)
{
    if (d->cg_graph >= 0) return d->cg_graph == 1;
    return d->nnz + d->nnzp < 300000;
}

// CG state, stream and (small problems) the kCgBatch-iteration graph, created on first use.
static int cg_setup(comap_destriper *d)
{
    if (d->batch || (d->cs && !cg_use_graph(d))) return 0;
    comap_ctx *ctx = d->ctx;
    const size_t nb = (size_t)d->nb;
    if (!d->cg && (dalloc(ctx, &d->cg, (4 * (size_t)d->NO + (size_t)d->npix) * nb) ||
                   dalloc(ctx, &d->flags, 2 + 2 * nb)))
        return -2;
    if (!d->flags_host) COMAP_CHECK(ctx, comap_pinned_alloc((void **)&d->flags_host, 4 * (2 + 2 * nb)));
    if (!d->thr_host) COMAP_CHECK(ctx, comap_pinned_alloc((void **)&d->thr_host, 8 * (1 + 4 * nb)));
    if (!d->cs) COMAP_CHECK(ctx, comap_stream_acquire(&d->cs));
    if (!d->ev) COMAP_CHECK(ctx, hipEventCreateWithFlags(&d->ev, hipEventDisableTiming));
    if (!cg_use_graph(d)) return 0;
    hipGraph_t g = nullptr;
    COMAP_CHECK(ctx, hipStreamBeginCapture(d->cs, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < kCgBatch; ++i) enqueue_iteration(d, d->cs);
    COMAP_CHECK(ctx, hipStreamEndCapture(d->cs, &g));
    const hipError_t e = hipGraphInstantiate(&d->batch, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    COMAP_CHECK(ctx, e);
    return 0;
}

// Single-rank destriper_iteration for every band: CG (one matvec per iteration) to
// threshold / niter, then the final maps (:419-451).  Iterations are queued kCgBatch
// at a time as one graph launch; the device-side stop flags make a band's iterations
// after its convergence no-ops, so its iterates and count equal a per-iteration loop's.
extern "C" int comap_destripe_solve(comap_destriper *d, double threshold, int32_t niter, double *x, double *map,
                                    double *naive, double *weight, double *hits, int32_t *iters_out)
{
    if (!d || !x || niter < 0) return -1;
    COMAP_DEVICE_GUARD(d->ctx);
    comap_ctx *ctx = d->ctx;
    int rc = cg_setup(d);
    if (rc) return rc;
    hipStream_t st = d->cs;
    const int nb = d->nb;
    const int64_t n = d->NO * nb, np = d->npix * nb;
    double *cx = d->cg, *r = cx + n, *p = r + n, *num = p + 2 * n;
    // inputs were produced on the caller's stream
    COMAP_CHECK(ctx, hipEventRecord(d->ev, ctx->stream));
    COMAP_CHECK(ctx, hipStreamWaitEvent(st, d->ev, 0));
    d->thr_host[0] = threshold;
    COMAP_CHECK(ctx, hipMemcpyAsync(d->scal + 4 * nb, d->thr_host, 8, hipMemcpyHostToDevice, st));
    COMAP_CHECK(ctx, hipMemsetAsync(cx, 0, 8 * n, st));
    COMAP_CHECK(ctx, hipMemsetAsync(num, 0, 8 * np, st));   // the CG bin writes only the non-empty rows
    COMAP_CHECK(ctx, hipMemsetAsync(d->flags, 0, 4 * (2 + 2 * nb), st));
    // b = op_Ax(tod, extend=False); r = p = b (x0 = 0); rr = rr0 = b.b
    launch_project(d, st, nullptr, d->nnum, d->h, r, nullptr, nullptr);
    COMAP_LAUNCH_CHECK(ctx);
    COMAP_CHECK(ctx, hipMemcpyAsync(p, r, 8 * n, hipMemcpyDeviceToDevice, st));
    if (d->cf) {   // the first bin's input pt = wbar o p (later ones come from the direction kernel)
        COMAP_NB_SWITCH(nb, k_scale<NB><<<grid_for(d->NO), 256, 0, st>>>(d->wbar, p, d->NO, d->pt, nullptr));
        COMAP_LAUNCH_CHECK(ctx);
    }
    if ((rc = dot(d, st, r, r, d->scal, nullptr))) return rc;
    COMAP_CHECK(ctx, hipMemcpyAsync(d->scal + nb, d->scal, 8 * nb, hipMemcpyDeviceToDevice, st));
    COMAP_CHECK(ctx, hipMemcpyAsync(d->scal + 3 * nb, d->scal, 8 * nb, hipMemcpyDeviceToDevice, st));   // current rr
    for (int i = 0; i < 2 + 2 * nb; ++i) d->flags_host[i] = 0;
    // Batches of kCgBatch iterations between host checks; after the first, the next batch
    // is sized from each running band's convergence rate over the last batch (delta =
    // rr / rr0 falls geometrically), so a solve that needs 2 more iterations does not
    // enqueue 14 no-op ones (4 launches each).  The iterates are unchanged: every
    // kernel still stops on the device flags.
    double *hs = d->thr_host + 1;                       // rr0 [nb] | rr [nb] | pq [nb] | rr_new [nb]
    std::vector<double> prev_delta(nb, -1.0);
    int next = kCgBatch;
    for (int enq = 0; enq < niter;) {
        const int k = std::min(next, niter - enq);
        if (k == kCgBatch && d->batch) {
            COMAP_CHECK(ctx, hipGraphLaunch(d->batch, st));
        } else {
            for (int i = 0; i < k; ++i) enqueue_iteration(d, st);
            COMAP_LAUNCH_CHECK(ctx);
        }
        enq += k;
        COMAP_CHECK(ctx, hipMemcpyAsync(d->flags_host, d->flags, 4 * (2 + 2 * nb), hipMemcpyDeviceToHost, st));
        COMAP_CHECK(ctx, hipMemcpyAsync(hs, d->scal, 8 * 4 * (size_t)nb, hipMemcpyDeviceToHost, st));
        COMAP_CHECK(ctx, hipStreamSynchronize(st));
        if (d->flags_host[0]) break;
        next = kCgBatch;
        if (threshold > 0) {
            int est = 0;
            for (int b = 0; b < nb; ++b) {
                if (d->flags_host[2 + b]) continue;
                const double delta = hs[3 * nb + b] / hs[b];
                const double pd = prev_delta[b] > 0 ? prev_delta[b] : 1.0;
                prev_delta[b] = delta;
                if (!(delta > 0) || !(delta < pd)) { est = kCgBatch; break; }
                const double need = std::log(threshold / delta) / (std::log(delta / pd) / k);
                est = std::max(est, (int)std::ceil(std::max(need, 0.0)) + 1);
            }
            next = std::max(1, std::min(kCgBatch, est));
        }
    }
    if (iters_out)
        for (int b = 0; b < nb; ++b) iters_out[b] = d->flags_host[2 + nb + b];
    if (d->perm) {
        COMAP_NB_SWITCH(nb, k_unpermute<NB><<<grid_for(d->NO), 256, 0, st>>>(cx, d->perm, d->NO, x));
        COMAP_LAUNCH_CHECK(ctx);
    } else {
        COMAP_CHECK(ctx, hipMemcpyAsync(x, cx, 8 * n, hipMemcpyDeviceToDevice, st));
    }
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
