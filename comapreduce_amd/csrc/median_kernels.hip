// median_kernels.hip -- exact sliding median (window w) on gfx950.
//
// Replaces the reference's serial two-heap filter (Tools/median_filter/
// Mediator.h:9-197, medianFilter.cpp:4-30) with an order-statistics
// formulation that is bit-exact for NaN-free input: the median of a window is
// a pure function of its multiset; even w averages s[w/2-1] and s[w/2] as
// (hi + lo) / 2 in f64, the order Mediator::getMedian uses (Mediator.h:91-99).
//
// 1. k_med_range + k_med_keys: every series (job) contributes the Ns = n_out + w - 1
//    values its windows touch, as 32-bit order-preserving proxies -- the value's u64
//    key relative to the series' smallest, scaled so the series' key range spans 32
//    bits (a monotone map, so the f64 order only differs inside runs of equal
//    proxies, which need keys within range / 2^32 of each other) + positions.
// 2. rocprim segmented radix sort (4 digit passes instead of 8); k_med_fix then
//    re-sorts every run of equal proxies by the exact u64 key of the f64 value
//    (runs are a few elements on real data).  A segment with a run longer than
//    kFixRun is flagged and re-sorted whole on 64-bit keys (a second segmented
//    sort over the flagged segments only -- the others are passed as empty).
//    k_med_rank inverts the permutation (rank of every position).
// 3. k_med_walk, one workgroup per segment of up to 4 chunks of L = 128 consecutive
//    outputs, chunk by chunk:
//    a. the chunk's union window U = positions [c, c+w+L-1) is marked in an
//       LDS bitmap indexed by rank (built once per segment from coalesced reads
//       of rank[], then slid: L positions leave and L enter per chunk), together
//       with its "zone" Z (offsets < L-1 or >= w: excluded by some output's window);
//       word popcount prefixes turn a rank into its index within U;
//    b. the zone entries, in rank order, form the list E = (U index, offset);
//    c. lane k walks E (4 entries per wave-uniform LDS read): from q = r, every
//       excluded zone entry with U index <= q pushes q up by one -> q = index in
//       U of the r-th smallest element of k's window; a binary search over the
//       word prefixes maps q back to a rank, hence to the value.
// Series longer than kMaxOut outputs are split into independent sub-jobs so
// the per-chunk bitmaps stay within LDS.
#include "comap_internal.h"

#include <hipcub/hipcub.hpp>
#include <rocprim/block/block_radix_sort.hpp>
#include <rocprim/device/device_segmented_radix_sort.hpp>

#include <algorithm>
#include <cstdlib>
#include <cstring>

namespace {

__device__ __forceinline__ uint64_t key_of(double v)
{
    const uint64_t b = __double_as_longlong(v);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

// index into j.src of the virtual series' element at pos (see xprime)
__device__ __forceinline__ int64_t src_index(const MedJob &j, int64_t pos, int h)
{
    const int64_t n = j.n;
    if (j.mode == 0) return pos < h ? 0 : (pos >= n ? n - 1 : pos);
    if (pos < 0) pos = 0;
    if (pos < n) return n - 1 - pos;
    if (pos < 2 * n) return pos - n;
    const int64_t q = 3 * n - 1 - pos;
    return q < 0 ? 0 : q;
}

// virtual series x'(pos), pos relative to the start of the (virtual) series
__device__ __forceinline__ double xprime(const MedJob &j, int64_t pos, int h)
{
    const int64_t n = j.n;
    if (j.mode == 0) {   // medfilt: x'[j<h] = x[0] (head inserts + overwritten head), x'[j>=n] = x[n-1]
        if (pos < h) return j.src[0];
        if (pos >= n) return j.src[n - 1];
        return j.src[pos];
    }
    // reflect-3: [x[::-1], x, x[::-1]] of length 3n
    if (pos < 0) pos = 0;
    if (pos < n) return j.src[n - 1 - pos];
    if (pos < 2 * n) return j.src[pos - n];
    int64_t q = 3 * n - 1 - pos;
    return j.src[q < 0 ? 0 : q];
}

// Source-index interval [lo, hi) that virtual positions [p0, p1) of a job read (src_index
// is monotone on each piece and the pieces meet, so the set is one interval: its ends
// are at the range ends or at the piece boundaries)
__host__ __device__ inline void src_interval(const MedJob &j, int64_t p0, int64_t p1, int h, int64_t &lo, int64_t &hi)
{
    const int64_t n = j.n;
    auto src = [&](int64_t pos) -> int64_t {
        if (j.mode == 0) return pos < h ? 0 : (pos >= n ? n - 1 : pos);
        if (pos < 0) pos = 0;
        if (pos < n) return n - 1 - pos;
        if (pos < 2 * n) return pos - n;
        const int64_t q = 3 * n - 1 - pos;
        return q < 0 ? 0 : q;
    };
    int64_t a = src(p0), b = a;
    const int64_t pts[6] = {p1 - 1, (int64_t)h - 1, n - 1, n, 2 * n - 1, 2 * n};
    for (int t = 0; t < 6; ++t)
        if (pts[t] >= p0 && pts[t] < p1) {
            const int64_t v = src(pts[t]);
            a = v < a ? v : a;
            b = v > b ? v : b;
        }
    lo = a;
    hi = b + 1;
}

// Element i of job jb's sort segment: with per-job source offsets (slo, the distinct-
// source layout of the wavelet-matrix walk) source slo[jb] + i, else virtual position
// base + i.
__device__ __forceinline__ double seg_elem(const MedJob &job, const int32_t *__restrict__ slo, int jb, int64_t base,
                                           int h, int64_t i)
{
    return slo ? job.src[slo[jb] + i] : xprime(job, base + i, h);
}

// Per-series range of the u64 keys (kr[2j] = min, kr[2j+1] = max), one 1024-thread
// workgroup per series (a C3 shard has ~110 series: 16 waves each keep 4x the loads
// in flight of the former 256-thread block).
// (also clears the job's re-sort flag for k_med_fix: no separate memset launch)
constexpr int kRangeThreads = 1024;
__global__ void __launch_bounds__(kRangeThreads) k_med_range(const MedJob *__restrict__ jobs,
                                                             const int32_t *__restrict__ seg, int32_t njobs, int32_t w,
                                                             unsigned long long *__restrict__ kr,
                                                             const int32_t *__restrict__ slo,
                                                             int32_t *__restrict__ flag = nullptr)
{
    __shared__ unsigned long long s_lo[kRangeThreads / 64], s_hi[kRangeThreads / 64];
    const int jb = blockIdx.x;
    if (jb >= njobs) return;
    const MedJob job = jobs[jb];
    const int32_t s0 = seg[jb], ns = seg[jb + 1] - s0;
    const int h = w / 2;
    const int64_t base = job.out_lo - h;
    unsigned long long lo = ~0ull, hi = 0ull;
    for (int i = threadIdx.x; i < ns; i += blockDim.x) {
        const unsigned long long k = key_of(seg_elem(job, slo, jb, base, h, i));
        lo = k < lo ? k : lo;
        hi = k > hi ? k : hi;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long a = __shfl_xor(lo, o, 64), b = __shfl_xor(hi, o, 64);
        lo = a < lo ? a : lo;
        hi = b > hi ? b : hi;
    }
    if ((threadIdx.x & 63) == 0) { s_lo[threadIdx.x >> 6] = lo; s_hi[threadIdx.x >> 6] = hi; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int v = 1; v < kRangeThreads / 64; ++v) {
            lo = s_lo[v] < lo ? s_lo[v] : lo;
            hi = s_hi[v] > hi ? s_hi[v] : hi;
        }
        kr[2 * jb] = lo;
        kr[2 * jb + 1] = hi;
        if (flag) flag[jb] = 0;
    }
}

// Order-preserving 32-bit proxy of a u64 key: its offset from the series' smallest key,
// scaled so the series' key range spans 32 bits (monotone non-decreasing in the key;
// two values share a proxy only when their keys are within range / 2^32).
__device__ __forceinline__ uint32_t key32_of(uint64_t k, uint64_t kmin, int shift)
{
    return (uint32_t)((k - kmin) >> shift);
}

template <typename K>
__global__ void __launch_bounds__(256) k_med_keys(const MedJob *__restrict__ jobs, const int32_t *__restrict__ seg,
                                                  int32_t njobs, int32_t w, K *__restrict__ keys,
                                                  int32_t *__restrict__ vals, const unsigned long long *__restrict__ kr,
                                                  const int32_t *__restrict__ slo, int pbits = 32)
{
    const int jb = blockIdx.y;
    if (jb >= njobs) return;
    const MedJob job = jobs[jb];
    const int32_t s0 = seg[jb], ns = seg[jb + 1] - s0;
    const int h = w / 2;
    const int64_t base = job.out_lo - h;
    uint64_t kmin = 0;
    int shift = 0;
    if constexpr (sizeof(K) == 4) {
        kmin = kr[2 * jb];
        const uint64_t range = kr[2 * jb + 1] - kmin;
        const int bits = range ? 64 - __clzll((long long)range) : 0;
        shift = bits > pbits ? bits - pbits : 0;
    }
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < ns; i += gridDim.x * blockDim.x) {
        const uint64_t k = key_of(seg_elem(job, slo, jb, base, h, i));
        if constexpr (sizeof(K) == 4) keys[s0 + i] = key32_of(k, kmin, shift);
        else keys[s0 + i] = k;
        vals[s0 + i] = i;
    }
}

constexpr int kFixRun = 32;   // longest run of equal proxies k_med_fix re-sorts in place

// Exact order inside runs of equal proxy keys: the thread at a run's first element
// insertion-sorts the run's positions by (u64 key of the f64 value, position) --
// the order the 64-bit sort gives.  Longer runs flag the segment for the full re-sort.
__global__ void __launch_bounds__(256) k_med_fix(const MedJob *__restrict__ jobs, const int32_t *__restrict__ seg,
                                                 int32_t njobs, int32_t w, const uint32_t *__restrict__ skeys,
                                                 int32_t *__restrict__ svals, int32_t *__restrict__ redo,
                                                 const int32_t *__restrict__ slo)
{
    const int jb = blockIdx.y;
    if (jb >= njobs) return;
    const int32_t s0 = seg[jb], ns = seg[jb + 1] - s0;
    const int h = w / 2;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < ns; i += gridDim.x * blockDim.x) {
        const uint32_t k = skeys[s0 + i];
        if (i + 1 >= ns || skeys[s0 + i + 1] != k) continue;     // not part of a run, or not its start
        if (i > 0 && skeys[s0 + i - 1] == k) continue;
        int e = i + 2;
        while (e < ns && e - i <= kFixRun && skeys[s0 + e] == k) ++e;
        if (e - i > kFixRun) { redo[jb] = 1; continue; }
        const MedJob job = jobs[jb];
        const int64_t base = job.out_lo - h;
        const int n = e - i;
        // the common run: equal values (one source element seen at several positions --
        // reflection padding, medfilt edges -- or equal samples): their relative order
        // cannot change any order statistic's value
        {
            const uint64_t k0 = key_of(seg_elem(job, slo, jb, base, h, svals[s0 + i]));
            bool same = true;
            for (int t = 1; t < n && same; ++t) same = key_of(seg_elem(job, slo, jb, base, h, svals[s0 + i + t])) == k0;
            if (same) continue;
        }
        auto before = [](uint64_t ka, int32_t pa, uint64_t kb, int32_t pb) { return ka < kb || (ka == kb && pa < pb); };
        if (n <= 8) {
            // the common case: a register-resident odd-even transposition sort (padded to 8)
            uint64_t kk[8];
            int32_t pp[8];
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                if (t < n) {
                    pp[t] = svals[s0 + i + t];
                    kk[t] = key_of(seg_elem(job, slo, jb, base, h, pp[t]));
                } else {
                    kk[t] = ~0ull;
                    pp[t] = 0x7fffffff;
                }
            }
#pragma unroll
            for (int rnd = 0; rnd < 8; ++rnd) {
#pragma unroll
                for (int t = rnd & 1; t + 1 < 8; t += 2) {
                    if (before(kk[t + 1], pp[t + 1], kk[t], pp[t])) {
                        const uint64_t tk = kk[t]; kk[t] = kk[t + 1]; kk[t + 1] = tk;
                        const int32_t tp = pp[t]; pp[t] = pp[t + 1]; pp[t + 1] = tp;
                    }
                }
            }
#pragma unroll
            for (int t = 0; t < 8; ++t)
                if (t < n) svals[s0 + i + t] = pp[t];
            continue;
        }
        uint64_t rk[kFixRun];
        int32_t rp[kFixRun];
        for (int t = 0; t < n; ++t) {
            const int32_t p = svals[s0 + i + t];
            const uint64_t kk = key_of(seg_elem(job, slo, jb, base, h, p));
            int u = t;
            while (u > 0 && (rk[u - 1] > kk || (rk[u - 1] == kk && rp[u - 1] > p))) {
                rk[u] = rk[u - 1];
                rp[u] = rp[u - 1];
                --u;
            }
            rk[u] = kk;
            rp[u] = p;
        }
        for (int t = 0; t < n; ++t) svals[s0 + i + t] = rp[t];
    }
}

// Segments flagged by k_med_fix: full 64-bit keys and the [begin, end) of the
// second sort (empty for the others).
__global__ void __launch_bounds__(256) k_med_redo(const MedJob *__restrict__ jobs, const int32_t *__restrict__ seg,
                                                  int32_t njobs, int32_t w, const int32_t *__restrict__ redo,
                                                  uint64_t *__restrict__ keys, int32_t *__restrict__ vals,
                                                  int32_t *__restrict__ beg, int32_t *__restrict__ end,
                                                  const int32_t *__restrict__ slo)
{
    const int jb = blockIdx.y;
    if (jb >= njobs) return;
    const int32_t s0 = seg[jb], ns = seg[jb + 1] - s0;
    const bool on = redo[jb] != 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        beg[jb] = s0;
        end[jb] = on ? s0 + ns : s0;
    }
    if (!on) return;
    const MedJob job = jobs[jb];
    const int h = w / 2;
    const int64_t base = job.out_lo - h;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < ns; i += gridDim.x * blockDim.x) {
        keys[s0 + i] = key_of(seg_elem(job, slo, jb, base, h, i));
        vals[s0 + i] = i;
    }
}

// rank[position] = sorted index, and sval[sorted index] = the value (so the walk's
// final lookup is one load)
__global__ void __launch_bounds__(256) k_med_rank(const MedJob *__restrict__ jobs, const int32_t *__restrict__ seg,
                                                  int32_t njobs, int32_t w, const int32_t *__restrict__ svals,
                                                  int32_t *__restrict__ rank, double *__restrict__ sval)
{
    const int jb = blockIdx.y;
    if (jb >= njobs) return;
    const MedJob job = jobs[jb];
    const int32_t s0 = seg[jb], ns = seg[jb + 1] - s0;
    const int h = w / 2;
    const int64_t base = job.out_lo - h;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < ns; i += gridDim.x * blockDim.x) {
        const int32_t p = svals[s0 + i];
        rank[s0 + p] = i;
        sval[s0 + i] = xprime(job, base + p, h);
    }
}

// One workgroup per walk segment: S consecutive chunks of LT outputs of one job.  The
// union-window bitmap U is built once for the segment's first chunk and then slid:
// moving to the next chunk clears the LT positions that leave and sets the LT that
// enter (3 LT rank reads per chunk instead of w + LT - 1).
template <int LT>   // threads = outputs per chunk
__global__ void __launch_bounds__(LT) k_med_walk(const MedJob *__restrict__ jobs, const SlideSeg *__restrict__ wsegs,
                                                 const int32_t *__restrict__ seg, const double *__restrict__ sval,
                                                 const int32_t *__restrict__ rank, int32_t w, int32_t nwmax)
{
    // LDS: E (16-B aligned for 4-entry reads) | U bitmap | Z bitmap | U, Z word prefixes | scans
    extern __shared__ __align__(16) unsigned char smem[];
    uint32_t *E = reinterpret_cast<uint32_t *>(smem);
    uint32_t *Ub = E + (2 * LT + 16);
    uint32_t *Zb = Ub + nwmax;
    int32_t *Up = reinterpret_cast<int32_t *>(Zb + nwmax);
    int32_t *Zp = Up + nwmax;
    int *scanU = Zp + nwmax;
    int *scanZ = scanU + LT;

    const int tid = threadIdx.x;
    const int lane = tid & 63, wv = tid >> 6;
    const SlideSeg sg = wsegs[blockIdx.x];
    const int jb = sg.job;
    const MedJob job = jobs[jb];
    if (job.gate && *job.gate <= 0.0) return;
    const int32_t s0 = seg[jb], ns = seg[jb + 1] - s0;
    const int nw = (ns + 31) >> 5;
    const int32_t *rk = rank + s0;                 // rank of series position p
    const double *sv = sval + s0;                  // value of rank r
    const int r_lo = (w % 2 == 0) ? (w / 2 - 1) : (w / 2);
    const int wpt = (nw + LT - 1) / LT;            // per-thread contiguous word ranges
    const int wb = min(nw, tid * wpt), we = min(nw, wb + wpt);

    int64_t i0 = sg.o0;
    int L = (int)min((int64_t)LT, sg.o1 - i0);
    int c0 = (int)(i0 - job.out_lo);               // chunk offset inside the series' position space
    // ---- a0. U of the first chunk: positions [c0, c0 + w + L - 1)
    for (int i = tid; i < nw; i += LT) Ub[i] = 0u;
    __syncthreads();
    for (int i = tid; i < w + L - 1; i += LT) {
        const int r = rk[c0 + i];
        atomicOr(&Ub[r >> 5], 1u << (r & 31));
    }
    for (;;) {
        const int M = w + L - 1;
        // ---- a. zone Z: offsets < L-1 or >= w (excluded by some output's window)
        for (int i = tid; i < nw; i += LT) Zb[i] = 0u;
        __syncthreads();
        int zr0 = -1, zr1 = -1;                   // this thread's zone entries: offsets tid and w + tid
        if (tid < L - 1) {
            zr0 = rk[c0 + tid];
            atomicOr(&Zb[zr0 >> 5], 1u << (zr0 & 31));
            zr1 = rk[c0 + w + tid];
            atomicOr(&Zb[zr1 >> 5], 1u << (zr1 & 31));
        }
        __syncthreads();
        int cu = 0, cz = 0;
        for (int k = wb; k < we; ++k) { cu += __popc(Ub[k]); cz += __popc(Zb[k]); }
        // inclusive scans of (cu, cz): within each wave by shuffles, then across waves
        int iu = cu, iz = cz;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int yu = __shfl_up(iu, off, 64), yz = __shfl_up(iz, off, 64);
            if (lane >= off) { iu += yu; iz += yz; }
        }
        if (lane == 63) { scanU[wv] = iu; scanZ[wv] = iz; }
        __syncthreads();
        int bu = 0, bz = 0, tz = 0;
        for (int v = 0; v < LT / 64; ++v) {
            if (v < wv) { bu += scanU[v]; bz += scanZ[v]; }
            tz += scanZ[v];
        }
        // ---- b. word prefixes; each zone entry's place in rank order (its Z prefix) and
        //         its union index (its U prefix) -> the zone list E, sorted by rank
        int u = bu + iu - cu, z = bz + iz - cz;
        for (int k = wb; k < we; ++k) {
            Up[k] = u;
            Zp[k] = z;
            u += __popc(Ub[k]);
            z += __popc(Zb[k]);
        }
        __syncthreads();
        if (tid < L - 1) {
            const int rr[2] = {zr0, zr1};
            const int pp[2] = {tid, w + tid};
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const int r = rr[t], k = r >> 5;
                const uint32_t below = (1u << (r & 31)) - 1u;
                const int ui = Up[k] + __popc(Ub[k] & below);
                const int zi = Zp[k] + __popc(Zb[k] & below);
                E[zi] = ((uint32_t)ui << 16) | (uint32_t)pp[t];
            }
        }
        if (tid < 16) E[tz + tid] = 0xffffffffu;   // sentinels: index 0xffff > any q
        __syncthreads();

        // ---- c. walk
        if (tid < L) {
            const int k = tid;
            int q = r_lo;
            int j = 0;
            int jstop = 0;
            for (;;) {
                const uint4 v = *reinterpret_cast<const uint4 *>(E + j);
                const uint32_t es[4] = {v.x, v.y, v.z, v.w};
                bool stop = false;
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    if (!stop) {
                        const uint32_t e = es[t];
                        if ((int)(e >> 16) > q) {
                            stop = true;
                            jstop = j + t;
                        } else {
                            const int pp = (int)(e & 0xffff);
                            q += (pp < k) | (pp >= k + w);
                        }
                    }
                }
                if (stop) break;
                j += 4;
            }
            // U index -> rank: the last word whose prefix is <= q holds it
            auto select = [&](int qi) -> int {
                int lo = 0, hi = nw - 1;
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (Up[mid] <= qi) lo = mid; else hi = mid - 1;
                }
                uint32_t bits = Ub[lo];
                for (int t = qi - Up[lo]; t > 0; --t) bits &= bits - 1u;
                return 32 * lo + __builtin_ctz(bits);
            };
            auto value = [&](int qi) -> double { return sv[select(qi)]; };
            const int q1 = q;
            const double v1 = value(q1);
            double out;
            if (w % 2 == 0) {
                q = q1 + 1;
                for (j = jstop;; ++j) {
                    const uint32_t e = E[j];
                    if ((int)(e >> 16) > q) break;
                    const int pp = (int)(e & 0xffff);
                    q += (pp < k) | (pp >= k + w);
                }
                out = (value(q) + v1) / 2.0;
            } else {
                out = v1;
            }
            job.dst[i0 + k - job.out_lo] = out;
        }
        // ---- next chunk: positions [c0, c0 + L) leave, [c0 + M, c0 + L + w + L1 - 1) enter
        const int64_t i1 = i0 + L;
        if (i1 >= sg.o1) break;
        const int L1 = (int)min((int64_t)LT, sg.o1 - i1);
        __syncthreads();          // the walk's reads of Ub / Up / E are done
        if (tid < L) {
            const int r = rk[c0 + tid];
            atomicAnd(&Ub[r >> 5], ~(1u << (r & 31)));
        }
        if (tid < L1) {
            const int r = rk[c0 + M + tid];
            atomicOr(&Ub[r >> 5], 1u << (r & 31));
        }
        i0 = i1;
        c0 += L;
        L = L1;
    }
}

// ------------------------------------------------------------------ wavelet-matrix walk
// k_med_wm: one workgroup per segment of consecutive outputs [o0, o1) of one job.  The
// ranks of the segment's positions P = [c0, c0 + ns), ns = (o1 - o0) + w - 1, are a
// sequence of L-bit integers; output k needs the r_lo-th (and for even w the next)
// smallest rank among positions [k, k + w) of it -- a range order statistic.  The
// workgroup builds the sequence's wavelet matrix in LDS (Claude & Navarro): level l
// (from the top bit down) holds bit l of every element of the current sequence, packed
// 32 to a word with the count of zeros before the word, and the next level's sequence
// is the stable partition of this one by that bit (zeros first).  A query then walks
// the L levels, each narrowing the range with two rank0 lookups (one LDS read each);
// the two middle order statistics share their path until the level where they part.
// Same ranks as the bitmap walk, so the same (bit-exact) values.
constexpr int kWmThreads = 1024;
#ifndef COMAP_WM_Q
#define COMAP_WM_Q 2
#endif
constexpr int kWmQ = COMAP_WM_Q;   // outputs per thread walking the levels together

__device__ __forceinline__ int wm_rank0(const uint64_t *__restrict__ lv, int i)
{
    const uint64_t e = lv[i >> 5];
    return (int)(e >> 32) + __popc(~(uint32_t)e & ((1u << (i & 31)) - 1u));
}

__global__ void __launch_bounds__(kWmThreads) k_med_wm(const MedJob *__restrict__ jobs,
                                                       const SlideSeg *__restrict__ wsegs,
                                                       const int32_t *__restrict__ seg,
                                                       const int32_t *__restrict__ sidx,
                                                       const int32_t *__restrict__ slo, int32_t w, int32_t L)
{
    extern __shared__ __align__(16) unsigned char smem[];
    __shared__ int wtot[kWmThreads / 64];
    __shared__ int zt[32];
    const SlideSeg sg = wsegs[blockIdx.x];
    const MedJob job = jobs[sg.job];
    if (job.gate && *job.gate <= 0.0) return;
    // the job's sort segment: its distinct sources [sl, sl + nu) in sorted order (sidx holds
    // source - sl); u(s) = sorted index of source s, so u order refines value order
    const int32_t s0 = seg[sg.job], nu = seg[sg.job + 1] - s0, sl = slo[sg.job];
    const int c0 = (int)(sg.o0 - job.out_lo);
    const int nout = (int)(sg.o1 - sg.o0);
    const int ns = nout + w - 1;
    const int nw = (ns + 31) >> 5;                 // <= kWmThreads (plan)
    const int ld = nw + 1;                         // words per level (+ the total-zeros entry)
    const int h = w / 2;
    const int64_t base = job.out_lo - h;           // virtual position of sort element 0
    uint64_t *lev = reinterpret_cast<uint64_t *>(smem);                 // [L][ld]
    const size_t lbytes = max((size_t)L * ld * 8, (size_t)nw * 64 + 16);
    uint16_t *S = reinterpret_cast<uint16_t *>(smem + lbytes);          // [nw * 32]
    uint16_t *uinv = reinterpret_cast<uint16_t *>(smem);                // [b - a], before the levels
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint16_t pad = (uint16_t)((1u << L) - 1u);   // padding sorts last at every level
    // sequence: u of the source every segment position reads
    int64_t a, b;
    src_interval(job, base + c0, base + c0 + ns, h, a, b);
    for (int i = tid; i < nu; i += kWmThreads) {
        const int64_t sidx_i = sl + sidx[s0 + i];
        if (sidx_i >= a && sidx_i < b) uinv[sidx_i - a] = (uint16_t)i;
    }
    __syncthreads();
    for (int i = tid; i < nw * 32; i += kWmThreads)
        S[i] = i < ns ? uinv[src_index(job, base + c0 + i, h) - a] : pad;
    __syncthreads();
    const bool own = tid < nw;
    for (int l = L - 1; l >= 0; --l) {
        uint16_t v[32];
        uint32_t bits = 0;
        if (own) {
            const uint4 *p = reinterpret_cast<const uint4 *>(S + 32 * tid);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint4 x = p[q];
                const uint32_t xw[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    v[8 * q + 2 * t] = (uint16_t)(xw[t] & 0xffffu);
                    v[8 * q + 2 * t + 1] = (uint16_t)(xw[t] >> 16);
                }
            }
#pragma unroll
            for (int j = 0; j < 32; ++j) bits |= (uint32_t)((v[j] >> l) & 1u) << j;
        }
        const int z = own ? 32 - __popc(bits) : 0;
        int incl = z;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        if (lane == 63) wtot[wv] = incl;
        __syncthreads();
        int before = 0, Z = 0;
#pragma unroll
        for (int u = 0; u < kWmThreads / 64; ++u) {
            const int t = wtot[u];
            before += u < wv ? t : 0;
            Z += t;
        }
        const int zpre = before + incl - z;
        uint64_t *lv = lev + (size_t)l * ld;
        if (own) lv[tid] = ((uint64_t)(uint32_t)zpre << 32) | bits;
        if (tid == 0) { lv[nw] = (uint64_t)(uint32_t)Z << 32; zt[l] = Z; }
        __syncthreads();                           // every read of S (and wtot) is done
        if (own && l > 0) {
            const int opre = 32 * tid - zpre;      // ones before this word
#pragma unroll
            for (int j = 0; j < 32; ++j) {
                const uint32_t below = (1u << j) - 1u;
                const int dst = ((bits >> j) & 1u) ? Z + opre + __popc(bits & below) : zpre + __popc(~bits & below);
                S[dst] = v[j];
            }
        }
        __syncthreads();
    }
    const bool two = (w % 2) == 0;
    const int r_lo = two ? (w / 2 - 1) : (w / 2);
    const int32_t *sp = sidx + s0;
    auto value = [&](uint32_t u) { return job.src[sl + sp[u]]; };   // value of sorted index u
    // kWmQ outputs per thread walk the levels together: their rank lookups are
    // independent, so each level's LDS reads of all of them are in flight at once
    // (one output's walk is a chain of dependent LDS round trips)
    struct Walk {
        int a, b, r, a2, b2, r2;
        uint32_t v1, v2;
        bool split;
    };
    for (int k0 = tid; k0 < nout; k0 += kWmThreads * kWmQ) {
        Walk q[kWmQ];
#pragma unroll
        for (int i = 0; i < kWmQ; ++i) {
            const int k = k0 + i * kWmThreads;
            const int ka = k < nout ? k : 0;           // idle slots walk output 0 (valid ranges)
            q[i] = Walk{ka, ka + w, r_lo, 0, 0, 0, 0u, 0u, false};
        }
        for (int l = L - 1; l >= 0; --l) {
            const uint64_t *lv = lev + (size_t)l * ld;
            const int Z = zt[l];
#pragma unroll
            for (int i = 0; i < kWmQ; ++i) {
                Walk &t = q[i];
                if (t.split) {                     // the upper statistic on its own path
                    const int za = wm_rank0(lv, t.a2), zb = wm_rank0(lv, t.b2), nz = zb - za;
                    if (t.r2 < nz) { t.a2 = za; t.b2 = zb; }
                    else { t.r2 -= nz; t.a2 = Z + t.a2 - za; t.b2 = Z + t.b2 - zb; t.v2 |= 1u << l; }
                }
                const int za = wm_rank0(lv, t.a), zb = wm_rank0(lv, t.b), nz = zb - za;
                if (two && !t.split && t.r < nz && t.r + 1 >= nz) {   // the two part here: upper = first one
                    t.split = true;
                    t.a2 = Z + t.a - za; t.b2 = Z + t.b - zb; t.r2 = 0; t.v2 = t.v1 | (1u << l);
                    t.a = za; t.b = zb;
                } else if (t.r < nz) {
                    t.a = za; t.b = zb;
                } else {
                    t.r -= nz; t.a = Z + t.a - za; t.b = Z + t.b - zb; t.v1 |= 1u << l;
                }
            }
        }
#pragma unroll
        for (int i = 0; i < kWmQ; ++i) {
            const int k = k0 + i * kWmThreads;
            if (k >= nout) continue;
            const double lo = value(q[i].v1);
            double out = lo;
            if (two) out = (value(q[i].split ? q[i].v2 : q[i].v1) + lo) / 2.0;
            job.dst[sg.o0 + k - job.out_lo] = out;
        }
    }
}

// LDS of a wavelet-matrix segment: the level words (whose space first holds the 16-bit
// source -> sorted-index table, at most one entry per position) + the 16-bit sequence;
// L levels of 8-B words
size_t wm_smem(int L, int nw)
{
    const size_t lv = (size_t)L * (nw + 1) * 8;
    return std::max<size_t>(lv, (size_t)nw * 64 + 16) + (size_t)nw * 64;
}

// Segmented radix sort of the series keys (u64 keys, i32 positions).
#ifndef COMAP_SORT_RB
#define COMAP_SORT_RB 8
#endif
#ifndef COMAP_SORT_IPT
#define COMAP_SORT_IPT 8
#endif
using SegSortConfig = rocprim::segmented_radix_sort_config<COMAP_SORT_RB, rocprim::kernel_config<256, COMAP_SORT_IPT>,
                                                           rocprim::DisabledWarpSortConfig, false>;
// the sort runs one workgroup per segment: wider workgroups finish each segment in
// fewer tiles per digit pass, which matters most with few segments (a C3 shard:
// ~100 series for 256 CUs)
using SegSortConfigWide = rocprim::segmented_radix_sort_config<8, rocprim::kernel_config<1024, 8>,
                                                               rocprim::DisabledWarpSortConfig, false>;
template <typename K>
hipError_t seg_sort(void *tmp, size_t &tb, const K *k0, K *k1, const int32_t *v0, int32_t *v1, int n, int nseg,
                    const int32_t *beg, const int32_t *end, hipStream_t st, bool wide = false,
                    unsigned end_bit = 8u * (unsigned)sizeof(K))
{
    if (wide)
        return rocprim::segmented_radix_sort_pairs<SegSortConfigWide>(tmp, tb, k0, k1, v0, v1, (unsigned)n,
                                                                      (unsigned)nseg, beg, end, 0u, end_bit, st);
    return rocprim::segmented_radix_sort_pairs<SegSortConfig>(tmp, tb, k0, k1, v0, v1, (unsigned)n, (unsigned)nseg,
                                                              beg, end, 0u, end_bit, st);
}

// Segments of up to kBlockSortMax elements are sorted whole in LDS by one 1024-thread
// workgroup: proxies computed from the values (k_med_keys' map), a block radix sort of
// (proxy, position) pairs on the pbits significant bits (rocprim block_radix_sort, 8-bit
// match ranking: pbits / 8 passes through LDS instead of through HBM), written as the
// sorted keys / positions the fix-up reads.  Stable (blocked input = position order), so
// the result equals the segmented device sort's.  Longer segments get their keys written
// and a [begin, end) range for that sort (empty ranges for the others).
constexpr int kBsThreads = 1024, kBsItems = 16;
constexpr int64_t kBlockSortMax = (int64_t)kBsThreads * kBsItems;
__global__ void __launch_bounds__(kBsThreads) k_med_blocksort(const MedJob *__restrict__ jobs,
                                                              const int32_t *__restrict__ seg, int32_t njobs, int32_t w,
                                                              const unsigned long long *__restrict__ kr,
                                                              const int32_t *__restrict__ slo, int pbits,
                                                              uint32_t *__restrict__ k0, int32_t *__restrict__ v0,
                                                              uint32_t *__restrict__ k1, int32_t *__restrict__ v1,
                                                              int32_t *__restrict__ beg, int32_t *__restrict__ end)
{
    using BS = rocprim::block_radix_sort<uint32_t, kBsThreads, kBsItems, int32_t>;
    __shared__ typename BS::storage_type bst;
    const int jb = blockIdx.x;
    if (jb >= njobs) return;
    const MedJob job = jobs[jb];
    const int32_t s0 = seg[jb], ns = seg[jb + 1] - s0;
    const int h = w / 2;
    const int64_t base = job.out_lo - h;
    const uint64_t kmin = kr[2 * jb];
    const uint64_t range = kr[2 * jb + 1] - kmin;
    const int bits = range ? 64 - __clzll((long long)range) : 0;
    const int shift = bits > pbits ? bits - pbits : 0;
    const bool large = ns > kBlockSortMax;
    if (threadIdx.x == 0) {
        beg[jb] = s0;
        end[jb] = large ? s0 + ns : s0;
    }
    if (large) {        // the segmented device sort's input
        for (int i = threadIdx.x; i < ns; i += kBsThreads) {
            k0[s0 + i] = key32_of(key_of(seg_elem(job, slo, jb, base, h, i)), kmin, shift);
            v0[s0 + i] = i;
        }
        return;
    }
    if (ns == 0) return;
    uint32_t k[kBsItems];
    int32_t v[kBsItems];
#pragma unroll
    for (int u = 0; u < kBsItems; ++u) {
        const int i = threadIdx.x * kBsItems + u;         // blocked: position order = input order
        v[u] = i;
        // padding sorts last: all-ones in the sorted bits, after every real key (stable)
        k[u] = i < ns ? key32_of(key_of(seg_elem(job, slo, jb, base, h, i)), kmin, shift) : 0xffffffffu;
    }
    BS().sort_to_striped(k, v, bst, 0, (unsigned)pbits);
#pragma unroll
    for (int u = 0; u < kBsItems; ++u) {
        const int i = threadIdx.x + kBsThreads * u;       // striped: coalesced stores
        if (i < ns) {
            k1[s0 + i] = k[u];
            v1[s0 + i] = v[u];
        }
    }
}

size_t walk_smem(int nwmax, int lt) { return 4 * (2 * (size_t)lt + 16) + 16 * (size_t)nwmax + 8 * (size_t)lt + 64; }

}  // namespace

// ------------------------------------------------------------------ plan
// Jobs with more than kMaxOut outputs are split into sub-jobs (each its own
// sorted segment), so a segment never exceeds kMaxOut + w - 1 values.
constexpr int64_t kMaxOut = 65536;
constexpr int32_t kMaxWindow = 32768;   // keeps U indices and offsets within 16 bits

int comap_median_plan(comap_ctx *ctx, MedPlan *mp, const std::vector<MedJob> &jobs_in, int32_t w)
{
    mp->w = w;
    // outputs per walk chunk (64 / 128 / 256 / 512): per output, the chunk's bitmap
    // setup costs ~(w + L) / L and the walk ~L zone entries; 128 measured fastest at w = 6000
    const char *lenv = getenv("COMAP_MEDIAN_L");
    mp->lc = lenv ? atoi(lenv) : 128;
    if (mp->lc != 64 && mp->lc != 256 && mp->lc != 512) mp->lc = 128;
    const char *k32 = getenv("COMAP_MEDIAN_KEY32");           // 0: sort the full u64 keys directly
    mp->key32 = !(k32 && !strcmp(k32, "0"));
    // proxy bits: the series' key range is scaled onto 32 bits, 4 radix digit passes
    // (24 bits: one pass less but more proxy collisions for k_med_fix, measured slower:
    // C2 median 1.18 vs 1.00 ms with the device sort, 1.06 vs 0.88 with the block sort)
    mp->pbits = 32;
    if (w < 1 || w > kMaxWindow) return comap_fail(ctx, -1, "median window must be 1 <= w <= 32768");
    // Sub-job length: at most kMaxOut outputs (LDS bitmaps).  (Splitting series further to
    // put more sort segments on the chip at C3 shard size measured slower: each extra
    // segment re-sorts w - 1 values.)
    int64_t total_out = 0;
    for (const MedJob &j : jobs_in) total_out += std::max<int64_t>(0, j.out_hi - j.out_lo);
    // the walk: wavelet matrix (default) or the bitmap walk (COMAP_MEDIAN_WALK=bitmap);
    // the wavelet matrix keeps ranks in 16 bits, so sub-jobs stay within 65536 positions
    const char *walk_env = getenv("COMAP_MEDIAN_WALK");
    mp->wm = !(walk_env && !strcmp(walk_env, "bitmap")) && w <= 16384;
    const int64_t max_out = mp->wm ? std::min<int64_t>(kMaxOut, 65536 - (int64_t)w + 1) : kMaxOut;
    std::vector<MedJob> jobs;
    for (const MedJob &j : jobs_in) {
        if (j.out_hi - j.out_lo <= max_out) { jobs.push_back(j); continue; }
        const int64_t nsub = (j.out_hi - j.out_lo + max_out - 1) / max_out;
        const int64_t len = ((j.out_hi - j.out_lo + nsub - 1) / nsub + mp->lc - 1) / mp->lc * mp->lc;
        for (int64_t lo = j.out_lo; lo < j.out_hi; lo += len) {
            MedJob sj = j;
            sj.out_lo = lo;
            sj.out_hi = std::min(j.out_hi, lo + len);
            sj.dst = j.dst + (lo - j.out_lo);      // dst is indexed from out_lo
            jobs.push_back(sj);
        }
    }
    // sort segments: the Ns = n_out + w - 1 virtual positions of each job (bitmap walk), or
    // for the wavelet-matrix walk the distinct source elements those positions read
    // (reflection padding and medfilt's edge repeats read some sources several times;
    // equal values need no order between them, so each source is sorted once)
    std::vector<int32_t> seg(jobs.size() + 1, 0), slo(jobs.size(), 0);
    int64_t nsmax = 0, numax = 0, nchunks = 0;
    for (size_t j = 0; j < jobs.size(); ++j) {
        const int64_t nout = jobs[j].out_hi - jobs[j].out_lo;
        const int64_t ns = nout > 0 ? nout + w - 1 : 0;
        int64_t ne = ns;
        if (mp->wm && ns > 0) {
            int64_t a = 0, b = 0;
            src_interval(jobs[j], jobs[j].out_lo - w / 2, jobs[j].out_lo - w / 2 + ns, w / 2, a, b);
            slo[j] = (int32_t)a;
            ne = b - a;
        }
        if ((int64_t)seg[j] + ne >= (1ll << 31)) return comap_fail(ctx, -1, "median plan too large");
        seg[j + 1] = seg[j] + (int32_t)ne;
        nsmax = std::max(nsmax, ns);
        numax = std::max(numax, ne);
        if (nout > 0) nchunks += (nout + mp->lc - 1) / mp->lc;
    }
    // walk segments of up to S chunks per workgroup (the bitmaps slide from chunk to
    // chunk); measured at w = 6000: C2 (107k chunks) S = 4 best, a C3 shard (13k) S = 1-2
    const char *senv = getenv("COMAP_MEDIAN_S");
    int64_t S = senv ? atoll(senv) : std::min<int64_t>(4, std::max<int64_t>(1, nchunks / 16384));
    S = std::max<int64_t>(1, S);
    std::vector<SlideSeg> wsegs;
    for (size_t j = 0; j < jobs.size(); ++j) {
        const int64_t span = S * mp->lc;
        for (int64_t o = jobs[j].out_lo; o < jobs[j].out_hi; o += span) {
            SlideSeg sg;
            sg.job = (int32_t)j; sg.pad_ = 0; sg.o0 = o; sg.o1 = std::min(jobs[j].out_hi, o + span);
            wsegs.push_back(sg);
        }
    }
    if (mp->wm) {
        // wavelet-matrix segments: short enough that L levels of (nw + 1) words plus the
        // 16-bit sequence fit the LDS budget, and enough of them to fill the chip
        int L = 1;
        while ((int64_t)1 << L < numax) ++L;
        const int64_t budget = 150 * 1024;
        const int64_t nwcap = std::min<int64_t>(kWmThreads, (budget - 8 * L) / (std::max(8 * L, 64) + 64));
        const int64_t seg_cap = nwcap * 32 - (w - 1);
        const char *te = getenv("COMAP_MEDIAN_WMSEGS");
        // measured at the C3 shard (r02sw2): 1 / 64 -> 0.255 ms, 128 / 192 -> 0.218, 256 -> 0.265, 512 -> 0.28;
        // C2 is cap-driven (>= 600 segments) and unchanged
        const int64_t target = te ? std::max(1, atoi(te)) : 128;
        if (L > 16 || seg_cap < 1) {
            return comap_fail(ctx, -1, "median plan: wavelet-matrix walk does not fit (use COMAP_MEDIAN_WALK=bitmap)");
        } else {
            wsegs.clear();
            size_t smax = 0;
            for (size_t j = 0; j < jobs.size(); ++j) {
                const int64_t nout = jobs[j].out_hi - jobs[j].out_lo;
                if (nout <= 0) continue;
                const int64_t want = total_out > 0 ? (nout * target + total_out - 1) / total_out : 1;
                const int64_t nseg = std::max<int64_t>((nout + seg_cap - 1) / seg_cap, std::max<int64_t>(1, want));
                const int64_t len = (nout + nseg - 1) / nseg;
                for (int64_t o = jobs[j].out_lo; o < jobs[j].out_hi; o += len) {
                    SlideSeg sg;
                    sg.job = (int32_t)j; sg.pad_ = 0; sg.o0 = o; sg.o1 = std::min(jobs[j].out_hi, o + len);
                    wsegs.push_back(sg);
                    smax = std::max(smax, wm_smem(L, (int)((sg.o1 - sg.o0 + w - 1 + 31) / 32)));
                }
            }
            mp->wmL = L;
            mp->wm_smem = smax;
        }
    }
    mp->nwmax = (int32_t)((nsmax + 31) / 32);
    mp->numax = numax;
    {
        const char *be = getenv("COMAP_MEDIAN_BLOCKSORT");     // 0: every segment on the device-wide sort
        mp->blocksort = !(be && be[0] == '0');
    }
    mp->njobs = (int32_t)jobs.size();
    mp->nitems = seg.back();
    mp->nchunks = nchunks;
    mp->nsegs = (int32_t)wsegs.size();
    hipStream_t st = ctx->stream;
    mp->alloc_stream = st;
    auto alloc = [&](void **p, size_t b) { return comap_tmp_alloc(p, b ? b : 8, st); };
    COMAP_CHECK(ctx, alloc((void **)&mp->jobs, sizeof(MedJob) * jobs.size()));
    COMAP_CHECK(ctx, alloc((void **)&mp->seg, 4 * seg.size()));
    COMAP_CHECK(ctx, alloc((void **)&mp->segs, sizeof(SlideSeg) * wsegs.size()));
    COMAP_CHECK(ctx, alloc((void **)&mp->k0, 8 * (size_t)mp->nitems));
    COMAP_CHECK(ctx, alloc((void **)&mp->k1, 8 * (size_t)mp->nitems));
    COMAP_CHECK(ctx, alloc((void **)&mp->v0, 4 * (size_t)mp->nitems));
    COMAP_CHECK(ctx, alloc((void **)&mp->v1, 4 * (size_t)mp->nitems));
    COMAP_CHECK(ctx, alloc((void **)&mp->rank, 4 * (size_t)mp->nitems));
    COMAP_CHECK(ctx, alloc((void **)&mp->redo, 4 * 3 * jobs.size()));   // flags | begin | end
    if (mp->wm) {
        COMAP_CHECK(ctx, alloc((void **)&mp->slo, 4 * jobs.size()));
        COMAP_CHECK(ctx, comap_upload(mp->slo, slo.data(), 4 * slo.size(), st));
    }
    COMAP_CHECK(ctx, alloc((void **)&mp->krange, 16 * jobs.size()));    // per-series key min, max
    COMAP_CHECK(ctx, comap_upload(mp->jobs, jobs.data(), sizeof(MedJob) * jobs.size(), st));
    COMAP_CHECK(ctx, comap_upload(mp->seg, seg.data(), 4 * seg.size(), st));
    if (!wsegs.empty()) COMAP_CHECK(ctx, comap_upload(mp->segs, wsegs.data(), sizeof(SlideSeg) * wsegs.size(), st));
    {
        // measured: C3 shard (106 series) 0.49 -> 0.40 ms of median, C2 (836) 2.06 -> 2.03
        const char *wenv = getenv("COMAP_SORT_WIDE");
        mp->wide = wenv ? atoi(wenv) != 0 : true;
    }
    size_t tb = 0, tb32 = 0;
    COMAP_CHECK(ctx, seg_sort(nullptr, tb, mp->k0, mp->k1, mp->v0, mp->v1, (int)mp->nitems, mp->njobs, mp->seg,
                              mp->seg + 1, st, mp->wide));
    COMAP_CHECK(ctx, seg_sort(nullptr, tb32, (const uint32_t *)mp->k0, (uint32_t *)mp->k1, mp->v0, mp->v1,
                              (int)mp->nitems, mp->njobs, mp->seg, mp->seg + 1, st, mp->wide));
    tb = std::max(tb, tb32);
    mp->temp_bytes = tb;
    COMAP_CHECK(ctx, alloc(&mp->temp, tb));
    // the plan's uploads are ordered on alloc_stream only: a run on another stream waits
    // for this event first (comap_median_run)
    COMAP_CHECK(ctx, hipEventCreateWithFlags(&mp->plan_ev, hipEventDisableTiming));
    COMAP_CHECK(ctx, hipEventRecord(mp->plan_ev, st));
    if (mp->wm) {
        COMAP_CHECK(ctx, hipFuncSetAttribute((const void *)k_med_wm,
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)std::max<size_t>(mp->wm_smem, 16)));
        return 0;   // (the uploads went through staging: no host wait for the host vectors)
    }
    const size_t sm = walk_smem(mp->nwmax, mp->lc);
    if (sm > 160 * 1024) return comap_fail(ctx, -1, "median plan: LDS budget exceeded");
    const void *wk = mp->lc == 64 ? (const void *)k_med_walk<64> : mp->lc == 128 ? (const void *)k_med_walk<128>
                   : mp->lc == 512 ? (const void *)k_med_walk<512> : (const void *)k_med_walk<256>;
    COMAP_CHECK(ctx, hipFuncSetAttribute(wk, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sm));
    return 0;
}

void comap_median_plan_free(MedPlan *mp)
{
    void *b[] = {mp->jobs, mp->seg, mp->k0, mp->k1, mp->v0, mp->v1, mp->rank, mp->temp, mp->segs, mp->redo, mp->krange,
                 mp->slo};
    // the last use is the last walk (whose stream waited for the plan's uploads on the
    // allocation stream): one event there guards every buffer's reuse
    comap_tmp_free_on(b, (int)(sizeof(b) / sizeof(b[0])), mp->run_stream ? mp->run_stream : mp->alloc_stream, false);
    if (mp->plan_ev) (void)hipEventDestroy(mp->plan_ev);
    *mp = MedPlan();
}

int comap_median_run(comap_ctx *ctx, MedPlan *mp, hipStream_t st)
{
    mp->run_stream = st;
    if (mp->nchunks == 0) return 0;
    if (mp->plan_ev && st != mp->alloc_stream) COMAP_CHECK(ctx, hipStreamWaitEvent(st, mp->plan_ev, 0));
    dim3 g1(64, (unsigned)mp->njobs);
    size_t tb = mp->temp_bytes;
    if (mp->key32) {
        uint32_t *k0 = (uint32_t *)mp->k0, *k1 = (uint32_t *)mp->k1;
        int32_t *flag = mp->redo, *beg = mp->redo + mp->njobs, *end = beg + mp->njobs;
        unsigned long long *kr = (unsigned long long *)mp->krange;
        k_med_range<<<mp->njobs, kRangeThreads, 0, st>>>(mp->jobs, mp->seg, mp->njobs, mp->w, kr, mp->slo, flag);
        COMAP_LAUNCH_CHECK(ctx);
        if (mp->blocksort) {
            // segments <= kBlockSortMax sorted in LDS; the longer ones (if any) by the device sort
            k_med_blocksort<<<mp->njobs, kBsThreads, 0, st>>>(mp->jobs, mp->seg, mp->njobs, mp->w, kr, mp->slo,
                                                             mp->pbits, k0, mp->v0, k1, mp->v1, beg, end);
            COMAP_LAUNCH_CHECK(ctx);
            if (mp->numax > kBlockSortMax)
                COMAP_CHECK(ctx, seg_sort(mp->temp, tb, (const uint32_t *)k0, k1, mp->v0, mp->v1, (int)mp->nitems,
                                          mp->njobs, beg, end, st, mp->wide, (unsigned)mp->pbits));
        } else {
            k_med_keys<uint32_t><<<g1, 256, 0, st>>>(mp->jobs, mp->seg, mp->njobs, mp->w, k0, mp->v0, kr, mp->slo,
                                                     mp->pbits);
            COMAP_LAUNCH_CHECK(ctx);
            COMAP_CHECK(ctx, seg_sort(mp->temp, tb, (const uint32_t *)k0, k1, mp->v0, mp->v1, (int)mp->nitems,
                                      mp->njobs, mp->seg, mp->seg + 1, st, mp->wide, (unsigned)mp->pbits));
        }
        k_med_fix<<<g1, 256, 0, st>>>(mp->jobs, mp->seg, mp->njobs, mp->w, k1, mp->v1, flag, mp->slo);
        COMAP_LAUNCH_CHECK(ctx);
        // the flagged segments (if any) again on exact 64-bit keys; the rest are empty ranges
        k_med_redo<<<g1, 256, 0, st>>>(mp->jobs, mp->seg, mp->njobs, mp->w, flag, mp->k0, mp->v0, beg, end, mp->slo);
        COMAP_LAUNCH_CHECK(ctx);
        tb = mp->temp_bytes;
        COMAP_CHECK(ctx, seg_sort(mp->temp, tb, (const uint64_t *)mp->k0, mp->k1, mp->v0, mp->v1, (int)mp->nitems,
                                  mp->njobs, beg, end, st, mp->wide));
    } else {
        k_med_keys<uint64_t><<<g1, 256, 0, st>>>(mp->jobs, mp->seg, mp->njobs, mp->w, mp->k0, mp->v0, nullptr,
                                                 mp->slo);
        COMAP_LAUNCH_CHECK(ctx);
        COMAP_CHECK(ctx, seg_sort(mp->temp, tb, (const uint64_t *)mp->k0, mp->k1, mp->v0, mp->v1, (int)mp->nitems,
                                  mp->njobs, mp->seg, mp->seg + 1, st, mp->wide));
    }
    if (mp->wm) {   // the wavelet-matrix walk reads the sorted positions directly
        if (mp->nsegs > 0)
            k_med_wm<<<mp->nsegs, kWmThreads, mp->wm_smem, st>>>(mp->jobs, mp->segs, mp->seg, mp->v1, mp->slo, mp->w,
                                                                 mp->wmL);
        COMAP_LAUNCH_CHECK(ctx);
        return 0;
    }
    // k0 (sort keys) is free now: it holds the values in sorted order for the walk
    double *sval = (double *)mp->k0;
    k_med_rank<<<g1, 256, 0, st>>>(mp->jobs, mp->seg, mp->njobs, mp->w, mp->v1, mp->rank, sval);
    COMAP_LAUNCH_CHECK(ctx);
    const size_t sm = walk_smem(mp->nwmax, mp->lc);
#define COMAP_WALK(LT) k_med_walk<LT><<<mp->nsegs, LT, sm, st>>>(mp->jobs, mp->segs, mp->seg, sval, mp->rank, mp->w, \
                                                                 mp->nwmax)
    switch (mp->lc) {
    case 64: COMAP_WALK(64); break;
    case 128: COMAP_WALK(128); break;
    case 512: COMAP_WALK(512); break;
    default: COMAP_WALK(256); break;
    }
#undef COMAP_WALK
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}

// ------------------------------------------------------------------ two-heap replay
// The order statistics above are the reference's result only when every comparison is a
// total order.  For a series holding NaN, Mediator's comparisons with NaN are all false,
// so which value sits at the median slot follows the heap's whole insertion history
// (Mediator.h:36-99); the drop-in (medfilt.pyx:26-33) and the data prep's running median
// (COMAPData.py:72-81, 357-360) feed such series to it.  They are replayed here exactly:
// one workgroup per series, the series materialised in a work array, one lane running
// medianFilter.cpp:4-30's four phases on it in place over a two-heap kept in LDS (or in a
// global scratch block for windows above kReplayLdsWindow), then the requested outputs
// copied out.  The series are rare (NaN-bearing) and independent, so a serial lane per
// series is the exact and sufficient shape.
namespace {

constexpr int kReplayThreads = 256;
constexpr int kReplayLdsWindow = 10240;          // 16 B per window slot: <= 160 KiB of LDS

struct ReplayHeap {
    int n;              // window
    double *val;        // ring slot -> value
    int *at;            // ring slot -> heap position
    int *hp;            // heap position + n/2 -> ring slot
    int nlo, nhi, cur;

    __device__ int &slot(int pos) { return hp[pos + n / 2]; }
    __device__ bool below(int i, int j) { return val[slot(i)] < val[slot(j)]; }
    __device__ bool order(int i, int j)      // swap positions i, j when value(i) < value(j)
    {
        const int a = slot(i), b = slot(j);
        if (!(val[a] < val[b])) return false;
        slot(i) = b; slot(j) = a;
        at[b] = i; at[a] = j;
        return true;
    }
    __device__ bool hi_up(int i) { while (i > 0 && order(i, i / 2)) i /= 2; return i == 0; }
    __device__ bool lo_up(int i) { while (i < 0 && order(i / 2, i)) i /= 2; return i == 0; }
    __device__ void hi_down(int i)
    {
        for (i *= 2; i <= nhi; i *= 2) {
            if (i < nhi && below(i + 1, i)) ++i;
            if (!order(i, i / 2)) break;
        }
    }
    __device__ void lo_down(int i)
    {
        for (i *= 2; i >= -nlo; i *= 2) {
            if (i > -nlo && below(i, i - 1)) --i;
            if (!order(i / 2, i)) break;
        }
    }
    __device__ void init()
    {
        nlo = nhi = cur = 0;
        for (int s = n - 1; s >= 0; --s) {      // slot s starts at 0, -1, +1, -2, +2, ...
            const int pos = ((s + 1) / 2) * ((s & 1) ? -1 : 1);
            at[s] = pos;
            slot(pos) = s;
            val[s] = 0.0;
        }
    }
    __device__ void push(double v)
    {
        const int p = at[cur];
        const double old = val[cur];
        val[cur] = v;
        cur = cur + 1 == n ? 0 : cur + 1;
        if (p > 0) {
            if (nhi < (n - 1) / 2) ++nhi;
            else if (v > old) { hi_down(p); return; }
            if (hi_up(p) && order(0, -1)) lo_down(-1);
        } else if (p < 0) {
            if (nlo < n / 2) ++nlo;
            else if (v < old) { lo_down(p); return; }
            if (lo_up(p) && nhi && order(1, 0)) hi_down(1);
        } else {
            if (nlo && lo_up(-1)) lo_down(-1);
            if (nhi && hi_up(1)) hi_down(1);
        }
    }
    __device__ double median()
    {
        double v = val[slot(0)];
        if (nhi < nlo) v = (v + val[slot(-1)]) / 2;
        return v;
    }
};

// job j: work[woff[j] .. + m) = the (virtual) series, m = n (mode 0) or 3n (mode 1); the
// filter runs on it in place; outputs [out_lo, out_hi) -> dst.  heap_g (global heap
// arrays, 16 w bytes per job) is used when w > kReplayLdsWindow.
__global__ void __launch_bounds__(kReplayThreads) k_med_replay(const MedJob *__restrict__ jobs,
                                                               const int64_t *__restrict__ woff,
                                                               double *__restrict__ work, int w,
                                                               char *__restrict__ heap_g)
{
    extern __shared__ double replay_lds[];
    const MedJob j = jobs[blockIdx.x];
    const int64_t n = j.n, m = j.mode == 0 ? n : 3 * n;
    double *z = work + woff[blockIdx.x];
    for (int64_t i = threadIdx.x; i < m; i += kReplayThreads) {
        int64_t s = i;
        if (j.mode != 0) s = i < n ? n - 1 - i : (i < 2 * n ? i - n : 3 * n - 1 - i);
        z[i] = j.src[s];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        ReplayHeap h;
        h.n = w;
        char *base = w <= kReplayLdsWindow ? (char *)replay_lds : heap_g + 16 * (int64_t)w * blockIdx.x;
        h.val = (double *)base;
        h.at = (int *)(base + 8 * (int64_t)w);
        h.hp = h.at + w;
        h.init();
        const int64_t hw = w / 2, off = w / 2 + w % 2;
        for (int64_t i = 0; i < hw; ++i) { h.push(z[0]); z[i] = h.median(); }
        for (int64_t i = 0; i < off; ++i) h.push(z[i]);
        for (int64_t i = 0; i < m - off; ++i) { z[i] = h.median(); h.push(z[i + off]); }
        for (int64_t i = m - off; i < m; ++i) { z[i] = h.median(); h.push(z[m - 1]); }
    }
    __syncthreads();
    for (int64_t i = j.out_lo + threadIdx.x; i < j.out_hi; i += kReplayThreads) j.dst[i - j.out_lo] = z[i];
}

}  // namespace

int comap_median_replay(comap_ctx *ctx, const std::vector<MedJob> &jobs, int32_t w, hipStream_t st)
{
    if (jobs.empty()) return 0;
    if (w < 1) return comap_fail(ctx, -1, "median window must be >= 1");
    std::vector<int64_t> woff(jobs.size() + 1, 0);
    for (size_t k = 0; k < jobs.size(); ++k) {
        const MedJob &j = jobs[k];
        const int64_t m = j.mode == 0 ? j.n : 3 * j.n;
        // medianFilter.cpp reads and writes outside the array below ceil(w/2) values
        if (m < (int64_t)(w / 2 + w % 2) || j.n < 1)
            return comap_fail(ctx, -1, "median replay: series shorter than ceil(w/2)");
        if (j.out_lo < 0 || j.out_hi > m || j.out_lo > j.out_hi) return comap_fail(ctx, -1, "median replay: bad range");
        woff[k + 1] = woff[k] + m;
    }
    const int nj = (int)jobs.size();
    DevTemps tmp(st, false);     // freed behind the queued work
    MedJob *djobs = nullptr;
    int64_t *dwoff = nullptr;
    double *work = nullptr;
    char *heap_g = nullptr;
    COMAP_CHECK(ctx, tmp.alloc(&djobs, jobs.size()));
    COMAP_CHECK(ctx, tmp.alloc(&dwoff, woff.size()));
    COMAP_CHECK(ctx, tmp.alloc(&work, (size_t)woff.back()));
    const bool lds = w <= kReplayLdsWindow;
    if (!lds) COMAP_CHECK(ctx, tmp.alloc(&heap_g, 16 * (size_t)w * jobs.size()));
    COMAP_CHECK(ctx, comap_upload(djobs, jobs.data(), sizeof(MedJob) * jobs.size(), st));
    COMAP_CHECK(ctx, comap_upload(dwoff, woff.data(), 8 * woff.size(), st));
    const size_t sm = lds ? 16 * (size_t)w : 0;
    COMAP_CHECK(ctx, hipFuncSetAttribute((const void *)k_med_replay, hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)std::max<size_t>(sm, 16)));
    k_med_replay<<<nj, kReplayThreads, sm, st>>>(djobs, dwoff, work, w, heap_g);
    COMAP_LAUNCH_CHECK(ctx);
    return 0;
}
