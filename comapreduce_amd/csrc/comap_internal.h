// Internal declarations shared by the HIP translation units of libcomap_hip.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/comap_hip.h"

struct comap_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    // scratch reused by the host-array drop-ins
    void *scratch = nullptr;
    size_t scratch_bytes = 0;
};

#define COMAP_CHECK(ctx, expr)                                                         \
    do {                                                                               \
        hipError_t _e = (expr);                                                        \
        if (_e != hipSuccess) {                                                        \
            (ctx)->err = std::string(#expr) + ": " + hipGetErrorString(_e);            \
            return -2;                                                                 \
        }                                                                              \
    } while (0)

#define COMAP_LAUNCH_CHECK(ctx) COMAP_CHECK(ctx, hipGetLastError())

// Every entry point that allocates or launches makes its context's device current
// for the call and restores the caller's device on return: the process shares one
// HIP runtime with torch, whose current device must not move under it.
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        else if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard()
    {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard &) = delete;
    DeviceGuard &operator=(const DeviceGuard &) = delete;
};
#define COMAP_DEVICE_GUARD(ctx) DeviceGuard _comap_dg((ctx)->device)

// Device buffers owned by one call: freed on every return path (error returns
// included).  With a stream, the destructor first waits for the work queued on
// it (kernels may still read the buffers).
// Process-wide stream-ordered pool for the current device's temporaries (created on
// first use, release threshold unbounded): hipMallocFromPoolAsync / hipFreeAsync then
// reuse cached memory instead of mapping and unmapping hundreds of MB per call
// (the prep high-pass lost 1.8 ms per call to that, r03h).
hipMemPool_t comap_tmp_pool();
// Temporaries through a host-side cache of freed blocks (8 size classes per octave, per
// device) in front of that pool: a free is a list push, an allocation of a cached class a
// list pop -- no allocation call.  hipFreeAsync of a median plan's 12 buffers cost
// 0.75-0.8 ms of host time per prep call (r03j).  Reuse is stream-safe: a free records
// one event after the blocks' last use (on `st`, default the stream each block was
// allocated on; none when `idle`, i.e. the caller synchronised), and a block handed out
// on another stream makes that stream wait for the event first (same stream: stream
// order suffices).  Cached bytes are capped (COMAP_TMP_CACHE_MB); comap_tmp_trim releases
// every cached block (comap_cache_trim in the C ABI; also tried once on out-of-memory).
hipError_t comap_tmp_alloc(void **p, size_t bytes, hipStream_t st);
void comap_tmp_free(void *p);
void comap_tmp_free_on(void *const *ps, int n, hipStream_t st, bool idle);
void comap_tmp_trim();
// Small pinned host blocks (CG flag / scalar read-back, result blocks) through the same
// kind of cache (capped by COMAP_PINNED_CACHE_MB): hipHostMalloc costs 0.1-0.3 ms a
// call, once per destriper problem before this (r03l).  A block is freed by its owner
// once no copy into or out of it is pending.
hipError_t comap_pinned_alloc(void **p, size_t bytes);
void comap_pinned_free(void *p);
void comap_pinned_trim();
// Non-blocking streams for the current device, reused across objects (a problem's CG
// stream): hipStreamCreate / hipStreamDestroy per destriper problem cost ~0.1 ms and a
// device sync.  Released streams must be idle (the caller synchronised them).
hipError_t comap_stream_acquire(hipStream_t *s);
void comap_stream_release(hipStream_t s);

// Host -> device copy through a page-locked staging block: the host array may be reused
// or freed as soon as this returns (the staging block is handed out again only once the
// copy has run), so no stream synchronisation is needed for the host buffer's lifetime.
hipError_t comap_upload(void *dst_dev, const void *src_host, size_t bytes, hipStream_t st);

struct DevTemps {
    std::vector<void *> p;
    hipStream_t st = nullptr;
    bool sync = true;     // false: no host wait on exit, the blocks are freed behind the stream's work
    explicit DevTemps(hipStream_t s = nullptr, bool sync_on_exit = true) : st(s), sync(sync_on_exit) {}
    DevTemps(const DevTemps &) = delete;
    DevTemps &operator=(const DevTemps &) = delete;
    // stream-ordered pool allocations (the context keeps the device pool's memory cached,
    // comap_ctx_create): no page mapping per call; freed after the stream sync
    template <typename T>
    hipError_t alloc(T **out, size_t n)
    {
        void *q = nullptr;
        const hipError_t e = comap_tmp_alloc(&q, sizeof(T) * (n ? n : 1), st);
        if (e == hipSuccess) p.push_back(q);
        *out = (T *)q;
        return e;
    }
    ~DevTemps()
    {
        if (p.empty()) return;
        if (sync) (void)hipStreamSynchronize(st);
        comap_tmp_free_on(p.data(), (int)p.size(), st, sync);
    }
};

int comap_fail(comap_ctx *ctx, int code, const std::string &msg);
int comap_scratch(comap_ctx *ctx, size_t bytes, void **out);
// med_dev[r] = np.nanmedian(float32 row r), rows_host[2r] = element offset in tod, [2r+1] = length
int comap_row_nanmedian(comap_ctx *ctx, const float *tod, const int64_t *rows_host, int32_t nrows, float *med_dev);

inline bool atmos_channel_host(int c) { return c >= 10 && c < 1014 && !(c >= 510 && c < 515); }

// ------------------------------------------------------------------ constants
namespace comap {
constexpr int kBands = 4;
constexpr int kChannels = 1024;
constexpr int kBC = kBands * kChannels;
constexpr int kMedfiltWindow = 6000;           // int(50*120), Level1Averaging.py:833
constexpr int kTile = 1024;                    // samples per pass-B/D workgroup (multiple of 256)
constexpr double kDnuTau = (2e9 / 1024.0) * (1.0 / 50.0);   // Level1Averaging.py:671-672
}  // namespace comap

// ------------------------------------------------------------------ sliding median
// One job = one series with a virtual accessor; outputs [out_lo, out_hi) of the
// (virtual) series are written to dst[i - out_lo].
struct MedJob {
    const double *src;
    double *dst;
    int64_t n;          // source length
    int64_t out_lo;
    int64_t out_hi;
    int32_t mode;       // 0: medfilt head/tail semantics on src; 1: reflect3 [rev, x, rev]
    int32_t pad_;
    const double *gate; // optional: skip the job when *gate <= 0 (band count N_b)
};

// A walk work item (k_med_wm / k_med_walk segment): outputs [o0, o1) of one job.
struct SlideSeg {
    int32_t job, pad_;
    int64_t o0, o1;
};

// Sliding-median plan: jobs, per-job sorted-key segments, walk segments in `segs`,
// buffers.
struct MedPlan {
    SlideSeg *segs = nullptr;    // dev [nsegs] k_med_wm or k_med_walk segments
    int32_t nsegs = 0;
    int32_t w = 0, lc = 0, nwmax = 0, njobs = 0;
    int32_t nitems = 0;
    int64_t nchunks = 0;
    MedJob *jobs = nullptr;      // dev [njobs]
    int32_t *seg = nullptr;      // dev [njobs+1] segment offsets
    uint64_t *k0 = nullptr, *k1 = nullptr;
    int32_t *v0 = nullptr, *v1 = nullptr;
    int32_t *rank = nullptr;     // dev [nitems] position -> sorted index
    bool key32 = true;           // sort 32-bit proxies + exact run fix-up (else u64 keys)
    int32_t pbits = 32;          // significant proxy bits (radix-sort digit passes = pbits / 8)
    bool wide = false;           // segmented sort with 1024-thread workgroups (few series)
    bool wm = false;             // walk = wavelet-matrix range order statistics (k_med_wm)
    int32_t wmL = 0;             // wavelet-matrix levels (bits of the largest rank)
    size_t wm_smem = 0;          // its dynamic LDS bytes
    int32_t *slo = nullptr;      // dev [njobs] first source index of each job (wavelet-matrix walk: the
                                 // sort segments hold the distinct sources a job reads, not positions)
    int32_t *redo = nullptr;     // dev [3][njobs]: segment re-sort flags, begin, end
    void *krange = nullptr;      // dev [njobs][2] u64: per-series key min, max (proxy scaling)
    void *temp = nullptr;
    size_t temp_bytes = 0;
    int64_t numax = 0;           // longest sort segment (the block sort takes those <= kBlockSortMax)
    bool blocksort = true;       // segments sorted whole in LDS by one workgroup (k_med_blocksort)
    hipEvent_t plan_ev = nullptr;         // recorded on alloc_stream after the plan's uploads
    hipStream_t alloc_stream = nullptr;   // its buffers come from the device pool on this stream
    hipStream_t run_stream = nullptr;     // the stream of its last comap_median_run (their last use)
};

int comap_median_plan(comap_ctx *ctx, MedPlan *mp, const std::vector<MedJob> &jobs, int32_t w);
void comap_median_plan_free(MedPlan *mp);
int comap_median_run(comap_ctx *ctx, MedPlan *mp, hipStream_t stream);
inline int comap_median_run(comap_ctx *ctx, MedPlan *mp) { return comap_median_run(ctx, mp, ctx->stream); }
// Exact replay of the reference's two-heap filter (Mediator.h / medianFilter.cpp) for the
// series the order-statistics plan does not serve: NaN-bearing series (the two-heap's NaN
// result follows its insertion history) and ceil(w/2) <= length < w.  One workgroup per
// job; job.mode 0 = medfilt on src[0..n), 1 = medfilt on [src[::-1], src, src[::-1]]
// (3n values); outputs [out_lo, out_hi) of the filtered array go to dst.  Enqueued on st.
int comap_median_replay(comap_ctx *ctx, const std::vector<MedJob> &jobs, int32_t w, hipStream_t st);

// ------------------------------------------------------------------ L1 plan
struct comap_l1_plan {
    comap_ctx *ctx = nullptr;
    int32_t F = 0, S = 0, U = 0;
    int64_t T = 0;
    const float *tod = nullptr;
    const double *el = nullptr;
    std::vector<int32_t> units_h;      // [U][4]
    int32_t *units = nullptr;          // dev [U][4]
    int32_t *tiles = nullptr;          // dev [NT][2] (unit, t_off)
    int64_t n_tiles = 0;
    // pass-B tiles: per unit from t_off = -(t0 mod 32) when T is a multiple of 32, so the
    // 4 KB row runs start on 128-B boundaries (the few samples before the scan are read
    // from the same row and never written out)
    int32_t *tiles_b = nullptr;        // dev [NTB][2] (unit, t_off)
    // samples of each feed that no unit of this plan covers (scan gaps, and in a C3 shard
    // the other ranks' units): (feed, t0, n); comap_l1_average zeroes the outputs there
    int64_t *gaps = nullptr;           // dev [NG][3]
    int64_t n_gaps = 0, max_gap = 0;
    // pass B -> median -> pass C software pipeline over unit groups (comap_l1_average):
    // group g = units [grp_u0[g], grp_u0[g+1]) = tiles [grp_tile0[g], grp_tile0[g+1]);
    // its sliding medians (one job per (unit, band)) run on the side stream
    static constexpr int kMaxGroups = 4;
    int32_t ngroups = 0;
    int32_t grp_u0[kMaxGroups + 1] = {0};
    int64_t grp_tile0[kMaxGroups + 1] = {0};
    int64_t grpb_tile0[kMaxGroups + 1] = {0};
    MedPlan medg[kMaxGroups];
    hipStream_t side = nullptr;
    hipEvent_t ev_b[kMaxGroups] = {}, ev_m[kMaxGroups] = {};
    // device workspaces
    double *airmass = nullptr;         // [F][T]
    double *unit_sums = nullptr;       // [U][8]: n, SA, SAA, Sv, Svv, N4
    double *mom = nullptr;             // [5][U*4096]: Sd, SAd, Su, Suu, Suv
    int32_t *nan_count = nullptr;      // [1]
    bool moments_valid = false;
    bool moments_pending = false;      // pass A enqueued, NaN count not read back yet
    bool prefetched = false;           // comap_l1_prefetch launched pass A for the next atmosphere call
    int32_t *nan_host = nullptr;       // pinned [1]
    hipEvent_t mom_event = nullptr;
    double *alpha = nullptr;           // [U*4096] 1/rms on median channels (0 off-set, NaN bad)
    double *nf = nullptr;              // [U*4096] rms (normalisation factor)
    double *bsum = nullptr;            // [U*4][4]: beta, gamma, N, skip
    double *mb = nullptr;              // [F][4][T] band mean
    double *mf = nullptr;              // [F][4][T] median-filtered band mean
    double *ssum = nullptr;            // [U*4][4]: Smf, Smm, SAm
    double *sdm = nullptr;             // [U*4096] sum_t d mf
    double *gw = nullptr;              // [F][4096] gain weights w
    int32_t *gmode = nullptr;          // [F]
    double *kap = nullptr;             // [3][U*4096] kappa_g, kappa_r, kappa_o
    double *dsum = nullptr;            // [U*4][16] per-band constants for pass D
    double *xreg = nullptr;            // [U*4096][2] regression x0,x1 (debug)
    double *dG = nullptr;              // [F][T]
    // NaN / calibrator paths
    int32_t *rowbad = nullptr;         // [U*4096] non-finite samples per row (pass A)
    int32_t nan_total = 0;             // total from the last pass A
    bool filled = false;               // fill_bad_data applied to the device cube (until restore_nan)
    int64_t *nanpos = nullptr;         // [nanpos_cap] cube element offsets the fill overwrote
    int64_t nanpos_cap = 0;
    int64_t *nanpos_n = nullptr;       // [1] entries used
    // select_time over every (unit, band) pair, gated on the device by pass A's row flags
    // (comap_l1_atmosphere enqueues it without waiting for pass A's NaN count)
    int32_t *sel_pairs = nullptr;      // [U*4][2] (unit, band)
    int64_t *sel_voff = nullptr;       // [U*4 + 1] offsets of each pair's valid mask
    int32_t *sel_flag = nullptr;       // [U*4] pair has a non-finite sample in a fitted channel
    uint8_t *sel_valid = nullptr;      // [sel_voff[U*4] + 1]
    int sel_maxn = 0;
    // comap_l1_vane's hot/cold index lists: host arrays are copied into pinned staging
    // and uploaded asynchronously (no host wait); the event guards the staging reuse
    char *vane_pinned = nullptr, *vane_dev = nullptr;
    size_t vane_cap = 0;
    hipEvent_t vane_ev = nullptr;
    // the vane kernel runs on the side stream beside pass A: it waits only for the main
    // stream's work up to pass A's launch (pre_a_ev), and the main stream waits for it
    // (vane_done) before anything queued after the vane call
    hipEvent_t pre_a_ev = nullptr, vane_done = nullptr;
    bool pre_a_valid = false;          // pre_a_ev marks the cube as final (no fill/restore since)
    double *ubs = nullptr;             // [U*4][4] fit normal-equation sums n, SA, SAA per (unit, band)
    double *fitsum = nullptr;          // [2][U*4096] masked Sd, SAd (select_time path)
    double *oa = nullptr;              // [U*4096][2] offset/slope L1AGC subtracts
    int32_t *flag = nullptr;           // [1] phase-1 kappa mismatch -> legacy passes C, D run
    // non-finite filtered rows (k_unit_flags, k_special_rows): ynf[u] = the gain fit's input
    // holds a non-finite value (dG = 0); ugate[u] = a band-0 row's filtered values hold
    // +-inf (fit_power_spectrum raises: dG None, no in-place zeroing)
    int32_t *ynf = nullptr;            // [U]
    int32_t *ugate = nullptr;          // [U]
    // channel list per (unit, band) for passes B and C: the median channels with alpha != 0,
    // ascending (k_coef_d phase 0)
    int32_t *dlist = nullptr;          // [U*4][1024]
    int32_t *dcnt = nullptr;           // [U*4]
    double *dw = nullptr;              // [U*4][1024][4] (alpha, kg, kr, ko) of each listed channel
    // per-kernel HIP-event timing (comap_l1_profile)
    bool prof_on = false;
    int prof_level = 2;                // 1: streaming passes only, 2: every kernel
    std::vector<hipEvent_t> prof_pool;
    std::vector<std::pair<int, int>> prof_rec;   // (kernel id, index of start event)
    double prof_ms[32] = {0};
    int64_t prof_n[32] = {0};
};

// kernel ids for comap_l1_profile_collect
enum L1Kernel {
    KV_VANE = 0, KV_MOMENTS, KV_ATMOS_FIT, KV_COEF_B, KV_BAND_SUMS, KV_MEDIAN, KV_SERIES_SUMS,
    KV_REGRESS, KV_GAIN_WEIGHTS, KV_COEF_D, KV_GAIN_AVG, KV_SCAN_WEIGHTS, KV_REGRESS_AVG, KV_FINISH, KV_COUNT
};
