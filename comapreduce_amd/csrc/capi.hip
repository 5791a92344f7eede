// capi.hip -- context management and the host-array drop-ins of the C ABI.
//
//   comap_medfilt_f64     replaces medfilt.medfilt   (Tools/median_filter/medfilt.pyx:26-33)
//   comap_bin_values_f64  replaces binFuncs.binValues (Tools/binFuncs.pyx:7-32)
//
// binValues is reproduced bit-exactly: samples are stably radix-sorted by
// pixel (hipcub, keeps sample order inside a pixel) and each pixel's weights
// are then added to image[p] in sample order, exactly the sequence of the
// reference's serial loop.
#include "comap_internal.h"

#include <map>
#include <memory>
#include <mutex>
#include <tuple>
#include <utility>
#include <vector>

#include <hipcub/hipcub.hpp>

#include <cmath>
#include <cstring>

int comap_fail(comap_ctx *ctx, int code, const std::string &msg)
{
    if (ctx) ctx->err = msg;
    return code;
}

namespace {
// Cached bytes above which a freed block goes back to the pool instead of the cache
// (COMAP_TMP_CACHE_MB, default 16 GiB of device temporaries per device; the pool itself
// keeps at most the same amount mapped between synchronisations).
uint64_t tmp_cache_cap()
{
    static uint64_t cap = [] {
        const char *e = getenv("COMAP_TMP_CACHE_MB");
        return (uint64_t)(e ? atoll(e) : 16384) << 20;
    }();
    return cap;
}
uint64_t pinned_cache_cap()
{
    static uint64_t cap = [] {
        const char *e = getenv("COMAP_PINNED_CACHE_MB");
        return (uint64_t)(e ? atoll(e) : 2048) << 20;
    }();
    return cap;
}
}  // namespace

hipMemPool_t comap_tmp_pool()
{
    static std::mutex mu;
    static std::map<int, hipMemPool_t> pools;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lock(mu);
    auto it = pools.find(dev);
    if (it != pools.end()) return it->second;
    hipMemPoolProps props{};
    props.allocType = hipMemAllocationTypePinned;
    props.handleTypes = hipMemHandleTypeNone;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = dev;
    hipMemPool_t pool = nullptr;
    if (hipMemPoolCreate(&pool, &props) != hipSuccess || !pool) {
        (void)hipGetLastError();
        (void)hipDeviceGetDefaultMemPool(&pool, dev);
    }
    if (pool) {
        uint64_t keep = tmp_cache_cap();
        (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
    }
    pools[dev] = pool;
    return pool;
}

namespace {
// A freed block's last use: the stream it ran on and, unless the block was already idle,
// an event recorded there after that use.  One event serves every block of one free call.
struct LastUse {
    hipStream_t st = nullptr;
    std::shared_ptr<hipEvent_t> ev;      // null: idle (the caller synchronised)
};
struct TmpBlock {
    void *p = nullptr;
    LastUse use;
};
struct TmpCache {
    std::mutex mu;
    std::map<std::pair<int, size_t>, std::vector<TmpBlock>> free;   // (device, class bytes) -> blocks
    std::map<void *, std::tuple<int, size_t, hipStream_t>> live;     // block -> (device, class, alloc stream)
    std::map<int, uint64_t> cached;                                  // device -> bytes on the free lists
};
TmpCache &tmp_cache()
{
    static TmpCache *c = new TmpCache();   // never destroyed: frees may run during exit
    return *c;
}
// 8 size classes per octave above 4 KiB: a request wastes at most 1/8 of its block
size_t tmp_class(size_t b)
{
    if (b <= 4096) return 4096;
    size_t top = 4096;
    while ((top << 1) <= b) top <<= 1;
    const size_t step = top / 8;
    return (b + step - 1) / step * step;
}
bool capturing(hipStream_t st)
{
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    return st && hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}
std::shared_ptr<hipEvent_t> record_use(hipStream_t st)
{
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
    if (hipEventRecord(e, st) != hipSuccess) {
        (void)hipEventDestroy(e);
        return nullptr;
    }
    return std::shared_ptr<hipEvent_t>(new hipEvent_t(e), [](hipEvent_t *q) {
        (void)hipEventDestroy(*q);
        delete q;
    });
}
// the block's last use has completed, or is ordered before work that st enqueues next
bool make_safe(const LastUse &u, hipStream_t st)
{
    if (!u.ev || u.st == st) return true;            // idle, or same stream: stream order
    if (!*u.ev) return false;                        // freed under capture: its own stream only
    // no cross-stream edge into a graph: under capture only completed blocks are reused
    const hipError_t e = capturing(st) ? hipEventQuery(*u.ev) : hipStreamWaitEvent(st, *u.ev, 0);
    if (e == hipSuccess) return true;
    (void)hipGetLastError();      // NotReady / a failed wait must not surface in a later launch check
    return false;
}
// COMAP_POISON=1 (debug): every temporary block handed out is filled with 0xff bytes (NaN
// for f64 / f32, -1 for integers), so a kernel that reads what no kernel wrote shows it
bool poison_on()
{
    static const bool on = [] {
        const char *e = getenv("COMAP_POISON");
        return e && e[0] == '1';
    }();
    return on;
}
}  // namespace

hipError_t comap_tmp_alloc(void **p, size_t bytes, hipStream_t st)
{
    int dev = 0;
    (void)hipGetDevice(&dev);
    const size_t cls = tmp_class(bytes ? bytes : 1);
    TmpCache &c = tmp_cache();
    {
        std::lock_guard<std::mutex> lock(c.mu);
        auto it = c.free.find({dev, cls});
        if (it != c.free.end()) {
            auto &v = it->second;
            for (size_t i = v.size(); i-- > 0;) {
                if (!make_safe(v[i].use, st)) continue;
                *p = v[i].p;
                v.erase(v.begin() + (std::ptrdiff_t)i);
                c.cached[dev] -= cls;
                c.live[*p] = {dev, cls, st};
                return poison_on() ? hipMemsetAsync(*p, 0xff, cls, st) : hipSuccess;
            }
        }
    }
    hipError_t e = hipMallocFromPoolAsync(p, cls, comap_tmp_pool(), st);
    if (e == hipErrorOutOfMemory) {       // cached blocks of other sizes hold the memory
        (void)hipGetLastError();
        comap_tmp_trim();
        e = hipMallocFromPoolAsync(p, cls, comap_tmp_pool(), st);
    }
    if (e == hipSuccess) {
        std::lock_guard<std::mutex> lock(c.mu);
        c.live[*p] = {dev, cls, st};
    }
    if (e == hipSuccess && poison_on()) e = hipMemsetAsync(*p, 0xff, cls, st);
    return e;
}

void comap_tmp_free_on(void *const *ps, int n, hipStream_t st, bool idle)
{
    TmpCache &c = tmp_cache();
    std::shared_ptr<hipEvent_t> ev;
    bool recorded = false;
    for (int i = 0; i < n; ++i) {
        void *p = ps[i];
        if (!p) continue;
        std::unique_lock<std::mutex> lock(c.mu);
        auto it = c.live.find(p);
        if (it == c.live.end()) continue;
        const int dev = std::get<0>(it->second);
        const size_t cls = std::get<1>(it->second);
        const hipStream_t use_st = st ? st : std::get<2>(it->second);
        c.live.erase(it);
        if (c.cached[dev] + cls > tmp_cache_cap()) {
            lock.unlock();
            DeviceGuard g(dev);
            (void)hipFreeAsync(p, use_st);            // stream-ordered release to the pool
            continue;
        }
        LastUse u;
        u.st = use_st;
        if (!idle) {
            if (capturing(use_st)) {
                // no event can be recorded into a capture: reuse stays on this stream only
                u.ev = std::shared_ptr<hipEvent_t>(new hipEvent_t(nullptr), [](hipEvent_t *q) { delete q; });
            } else {
                if (!recorded) {
                    lock.unlock();
                    ev = record_use(use_st);
                    recorded = true;
                    lock.lock();
                }
                if (!ev) {                              // could not record: wait here instead
                    lock.unlock();
                    (void)hipStreamSynchronize(use_st);
                    lock.lock();
                }
                u.ev = ev;
            }
        }
        c.free[{dev, cls}].push_back({p, u});
        c.cached[dev] += cls;
    }
}

void comap_tmp_free(void *p) { comap_tmp_free_on(&p, 1, nullptr, false); }

void comap_tmp_trim()
{
    TmpCache &c = tmp_cache();
    std::map<std::pair<int, size_t>, std::vector<TmpBlock>> fl;
    {
        std::lock_guard<std::mutex> lock(c.mu);
        fl.swap(c.free);
        c.cached.clear();
    }
    std::map<int, bool> devs;
    for (auto &kv : fl) {
        DeviceGuard g(kv.first.first);
        for (TmpBlock &b : kv.second) {
            if (b.use.ev && *b.use.ev) (void)hipEventSynchronize(*b.use.ev);
            else if (b.use.ev) (void)hipStreamSynchronize(b.use.st);
            (void)hipFree(b.p);
        }
        devs[kv.first.first] = true;
    }
    for (auto &d : devs) {
        DeviceGuard g(d.first);
        (void)hipMemPoolTrimTo(comap_tmp_pool(), 0);
    }
}

namespace {
struct PinnedCache {
    std::mutex mu;
    std::map<size_t, std::vector<void *>> free;
    std::map<void *, size_t> live;
    uint64_t cached = 0;
};
PinnedCache &pinned_cache()
{
    static PinnedCache *c = new PinnedCache();
    return *c;
}
struct StreamPool {
    std::mutex mu;
    std::map<int, std::vector<hipStream_t>> idle;
    std::map<hipStream_t, int> dev_of;
};
StreamPool &stream_pool()
{
    static StreamPool *s = new StreamPool();
    return *s;
}
}  // namespace

hipError_t comap_pinned_alloc(void **p, size_t bytes)
{
    const size_t cls = tmp_class(bytes ? bytes : 1);
    PinnedCache &c = pinned_cache();
    {
        std::lock_guard<std::mutex> lock(c.mu);
        auto it = c.free.find(cls);
        if (it != c.free.end() && !it->second.empty()) {
            *p = it->second.back();
            it->second.pop_back();
            c.cached -= cls;
            c.live[*p] = cls;
            return hipSuccess;
        }
    }
    const hipError_t e = hipHostMalloc(p, cls, hipHostMallocDefault);
    if (e == hipSuccess) {
        std::lock_guard<std::mutex> lock(c.mu);
        c.live[*p] = cls;
    }
    return e;
}

// Host blocks are returned by their owner once no copy into or out of them is pending
// (the Python side frees a result block when its last NumPy view is gone).
void comap_pinned_free(void *p)
{
    if (!p) return;
    PinnedCache &c = pinned_cache();
    std::unique_lock<std::mutex> lock(c.mu);
    auto it = c.live.find(p);
    if (it == c.live.end()) return;
    const size_t cls = it->second;
    c.live.erase(it);
    if (c.cached + cls > pinned_cache_cap()) {
        lock.unlock();
        (void)hipHostFree(p);
        return;
    }
    c.free[cls].push_back(p);
    c.cached += cls;
}

void comap_pinned_trim()
{
    PinnedCache &c = pinned_cache();
    std::map<size_t, std::vector<void *>> fl;
    {
        std::lock_guard<std::mutex> lock(c.mu);
        fl.swap(c.free);
        c.cached = 0;
    }
    for (auto &kv : fl)
        for (void *p : kv.second) (void)hipHostFree(p);
}

namespace {
struct StageBlock {
    void *p = nullptr;
    size_t bytes = 0;
    hipEvent_t ev = nullptr;    // recorded after the block's last copy
};
struct StagePool {
    std::mutex mu;
    std::vector<StageBlock> idle;
};
StagePool &stage_pool()
{
    static StagePool *s = new StagePool();
    return *s;
}
}  // namespace

hipError_t comap_upload(void *dst_dev, const void *src_host, size_t bytes, hipStream_t st)
{
    if (!bytes) return hipSuccess;
    StagePool &sp = stage_pool();
    StageBlock b;
    {
        std::lock_guard<std::mutex> lock(sp.mu);
        for (size_t i = 0; i < sp.idle.size(); ++i) {
            StageBlock &c = sp.idle[i];
            if (c.bytes < bytes) continue;
            if (c.ev && hipEventQuery(c.ev) != hipSuccess) {
                (void)hipGetLastError();          // NotReady is not an error of the next launch
                continue;
            }
            b = c;
            sp.idle.erase(sp.idle.begin() + (std::ptrdiff_t)i);
            break;
        }
    }
    if (!b.p) {
        b.bytes = tmp_class(std::max<size_t>(bytes, 65536));
        hipError_t e = hipHostMalloc(&b.p, b.bytes, hipHostMallocDefault);
        if (e != hipSuccess) return e;
        e = hipEventCreateWithFlags(&b.ev, hipEventDisableTiming);
        if (e != hipSuccess) {
            (void)hipHostFree(b.p);
            return e;
        }
    }
    std::memcpy(b.p, src_host, bytes);
    hipError_t e = hipMemcpyAsync(dst_dev, b.p, bytes, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipEventRecord(b.ev, st);
    if (e != hipSuccess) (void)hipStreamSynchronize(st);    // the block is idle again either way
    std::lock_guard<std::mutex> lock(sp.mu);
    sp.idle.push_back(b);
    return e;
}

static void stage_trim()
{
    StagePool &sp = stage_pool();
    std::vector<StageBlock> v;
    {
        std::lock_guard<std::mutex> lock(sp.mu);
        v.swap(sp.idle);
    }
    for (StageBlock &b : v) {
        if (b.ev) {
            (void)hipEventSynchronize(b.ev);
            (void)hipEventDestroy(b.ev);
        }
        (void)hipHostFree(b.p);
    }
}

extern "C" int comap_cache_trim(void)
{
    comap_tmp_trim();
    comap_pinned_trim();
    stage_trim();
    return 0;
}

extern "C" int comap_cache_bytes(int64_t *device_cached, int64_t *device_live, int64_t *host_cached)
{
    TmpCache &c = tmp_cache();
    int dev = 0;
    (void)hipGetDevice(&dev);
    {
        std::lock_guard<std::mutex> lock(c.mu);
        if (device_cached) *device_cached = (int64_t)c.cached[dev];
        if (device_live) {
            int64_t s = 0;
            for (auto &kv : c.live)
                if (std::get<0>(kv.second) == dev) s += (int64_t)std::get<1>(kv.second);
            *device_live = s;
        }
    }
    if (host_cached) {
        PinnedCache &pc = pinned_cache();
        std::lock_guard<std::mutex> lock(pc.mu);
        *host_cached = (int64_t)pc.cached;
    }
    return 0;
}

hipError_t comap_stream_acquire(hipStream_t *s)
{
    int dev = 0;
    (void)hipGetDevice(&dev);
    StreamPool &sp = stream_pool();
    {
        std::lock_guard<std::mutex> lock(sp.mu);
        auto &v = sp.idle[dev];
        if (!v.empty()) {
            *s = v.back();
            v.pop_back();
            return hipSuccess;
        }
    }
    const hipError_t e = hipStreamCreateWithFlags(s, hipStreamNonBlocking);
    if (e == hipSuccess) {
        std::lock_guard<std::mutex> lock(sp.mu);
        sp.dev_of[*s] = dev;
    }
    return e;
}

void comap_stream_release(hipStream_t s)
{
    if (!s) return;
    StreamPool &sp = stream_pool();
    std::lock_guard<std::mutex> lock(sp.mu);
    auto it = sp.dev_of.find(s);
    if (it != sp.dev_of.end()) sp.idle[it->second].push_back(s);
}

int comap_scratch(comap_ctx *ctx, size_t bytes, void **out)
{
    if (bytes > ctx->scratch_bytes) {
        if (ctx->scratch) {
            COMAP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
            COMAP_CHECK(ctx, hipFree(ctx->scratch));
            ctx->scratch = nullptr;
            ctx->scratch_bytes = 0;
        }
        size_t nb = bytes + bytes / 4 + 4096;
        COMAP_CHECK(ctx, hipMalloc(&ctx->scratch, nb));
        ctx->scratch_bytes = nb;
    }
    *out = ctx->scratch;
    return 0;
}

extern "C" const char *comap_version(void) { return "comap_hip gfx950 " __DATE__; }

extern "C" int comap_host_alloc(size_t bytes, void **out)
{
    if (!out) return -1;
    *out = nullptr;
    return comap_pinned_alloc(out, bytes) == hipSuccess ? 0 : -2;
}

extern "C" void comap_host_free(void *p) { comap_pinned_free(p); }

extern "C" int comap_ctx_create(int device, comap_ctx **out)
{
    if (!out) return -1;
    *out = nullptr;
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev <= device || device < 0) return -6;
    // the caller's current device is left as it was (DeviceGuard restores it)
    DeviceGuard g(device);
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess || cur != device) return -6;
    (void)comap_tmp_pool();
    auto *c = new comap_ctx();
    c->device = device;
    *out = c;
    return 0;
}

extern "C" int comap_ctx_destroy(comap_ctx *ctx)
{
    if (!ctx) return 0;
    COMAP_DEVICE_GUARD(ctx);
    if (ctx->scratch) {
        (void)hipStreamSynchronize(ctx->stream);
        (void)hipFree(ctx->scratch);
    }
    delete ctx;
    return 0;
}

extern "C" const char *comap_last_error(const comap_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

extern "C" int comap_set_stream(comap_ctx *ctx, void *stream)
{
    if (!ctx) return -1;
    ctx->stream = (hipStream_t)stream;
    return 0;
}

extern "C" int comap_synchronize(comap_ctx *ctx)
{
    if (!ctx) return -1;
    COMAP_DEVICE_GUARD(ctx);
    COMAP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
    return 0;
}

// ------------------------------------------------------------------ medfilt drop-in
extern "C" int comap_medfilt_f64(comap_ctx *ctx, double *x, int64_t n, int32_t w)
{
    if (!ctx || !x) return -1;
    COMAP_DEVICE_GUARD(ctx);
    // medianFilter.cpp:4-30 stays inside the array for n >= ceil(w/2)
    if (w < 1 || n < (int64_t)(w / 2 + w % 2)) return comap_fail(ctx, -1, "medfilt requires 1 <= w and ceil(w/2) <= n");
    if (n + w >= (1ll << 31)) return comap_fail(ctx, -1, "medfilt series too long");
    bool nan = false;
    for (int64_t i = 0; i < n && !nan; ++i) nan = std::isnan(x[i]);
    char *s = nullptr;
    int rc = comap_scratch(ctx, 16 * (size_t)n + 64, (void **)&s);
    if (rc) return rc;
    double *dsrc = (double *)s;
    double *ddst = dsrc + n;
    MedJob job;
    job.src = dsrc; job.dst = ddst; job.n = n; job.out_lo = 0; job.out_hi = n; job.mode = 0; job.pad_ = 0;
    job.gate = nullptr;
    hipStream_t st = ctx->stream;
    COMAP_CHECK(ctx, hipMemcpyAsync(dsrc, x, 8 * n, hipMemcpyHostToDevice, st));
    MedPlan mp;
    // NaN (history-dependent two-heap order) or a series shorter than the window: the exact
    // two-heap replay; otherwise the order-statistics plan
    const bool replay = nan || n < w || w > 32768;
    if (replay) rc = comap_median_replay(ctx, std::vector<MedJob>{job}, w, st);
    else {
        rc = comap_median_plan(ctx, &mp, std::vector<MedJob>{job}, w);
        if (!rc) rc = comap_median_run(ctx, &mp);
    }
    if (!rc) {
        hipError_t e = hipMemcpyAsync(x, ddst, 8 * n, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) rc = comap_fail(ctx, -2, hipGetErrorString(e));
    }
    comap_median_plan_free(&mp);
    return rc;
}

// ------------------------------------------------------------------ batched median
// Series s = x[offsets[s] .. offsets[s+1]).  mode 0: medfilt semantics, all
// outputs; mode 1: the middle third of medfilt on [x[::-1], x, x[::-1]]
// (Level1Averaging.py:696-700, COMAPData.py:72-81), computed without the pad.  Series
// holding NaN, or shorter than the window, take the exact two-heap replay.
extern "C" int comap_medfilt_batch_f64(comap_ctx *ctx, const double *x, const int64_t *offsets, int32_t nseries,
                                       int32_t w, int32_t mode, double *out)
{
    if (!ctx || !x || !offsets || !out || nseries < 0 || (mode != 0 && mode != 1)) return -1;
    COMAP_DEVICE_GUARD(ctx);
    if (nseries == 0) return 0;
    if (w < 1) return comap_fail(ctx, -1, "medfilt requires w >= 1");
    const int64_t total = offsets[nseries];
    const int64_t need = w / 2 + w % 2;     // medianFilter.cpp stays inside the array from ceil(w/2) values
    for (int s = 0; s < nseries; ++s) {
        const int64_t n = offsets[s + 1] - offsets[s];
        if (n < 0) return comap_fail(ctx, -1, "offsets must be non-decreasing");
        if (n > 0 && (mode == 0 ? n : 3 * n) < need) return comap_fail(ctx, -1, "series shorter than ceil(w/2)");
    }
    char *s = nullptr;
    int rc = comap_scratch(ctx, 16 * (size_t)total + 64, (void **)&s);
    if (rc) return rc;
    double *dsrc = (double *)s;
    double *ddst = dsrc + total;
    std::vector<MedJob> jobs, replay;
    for (int k = 0; k < nseries; ++k) {
        const int64_t n = offsets[k + 1] - offsets[k];
        if (n == 0) continue;
        MedJob j;
        j.src = dsrc + offsets[k];
        j.dst = ddst + offsets[k];
        j.n = n;
        j.mode = mode;
        j.pad_ = 0;
        j.gate = nullptr;
        j.out_lo = mode == 0 ? 0 : n;
        j.out_hi = mode == 0 ? n : 2 * n;
        bool nan = false;
        for (int64_t i = offsets[k]; i < offsets[k + 1] && !nan; ++i) nan = std::isnan(x[i]);
        // mode 1 equals medfilt on the padded array on the order-statistics path only when
        // no output window reaches the pad's head / tail replacement: n >= w
        (nan || n < w || w > 32768 ? replay : jobs).push_back(j);
    }
    hipStream_t st = ctx->stream;
    COMAP_CHECK(ctx, hipMemcpyAsync(dsrc, x, 8 * total, hipMemcpyHostToDevice, st));
    MedPlan mp;
    if (!jobs.empty()) {
        rc = comap_median_plan(ctx, &mp, jobs, w);
        if (!rc) rc = comap_median_run(ctx, &mp);
    }
    if (!rc) rc = comap_median_replay(ctx, replay, w, st);
    if (!rc) {
        hipError_t e = hipMemcpyAsync(out, ddst, 8 * total, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) rc = comap_fail(ctx, -2, hipGetErrorString(e));
    }
    comap_median_plan_free(&mp);
    return rc;
}

// ------------------------------------------------------------------ binValues drop-in
__global__ void k_bin_keys(const int64_t *__restrict__ pix, const int64_t *__restrict__ mask, int64_t n,
                           int64_t npix, int32_t *__restrict__ keys, int32_t *__restrict__ vals)
{
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t p = pix[i];
        const bool ok = (p >= 0) && (p < npix) && (!mask || mask[i] != 0);
        keys[i] = ok ? (int32_t)p : (int32_t)npix;
        vals[i] = (int32_t)i;
    }
}

__device__ __forceinline__ int64_t lb32(const int32_t *a, int64_t n, int32_t v)
{
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t m = (lo + hi) >> 1;
        if (a[m] < v) lo = m + 1; else hi = m;
    }
    return lo;
}

// image[p] += w[i] in sample order (the reference's serial sequence).
__global__ void k_bin_ordered(const int32_t *__restrict__ keys, const int32_t *__restrict__ vals, int64_t n,
                              const double *__restrict__ w, int64_t npix, double *__restrict__ image)
{
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < npix; p += (int64_t)gridDim.x * blockDim.x) {
        const int64_t lo = lb32(keys, n, (int32_t)p), hi = lb32(keys, n, (int32_t)(p + 1));
        if (lo == hi) continue;
        double acc = image[p];
        if (w) for (int64_t j = lo; j < hi; ++j) acc += w[vals[j]];
        else for (int64_t j = lo; j < hi; ++j) acc += 1.0;
        image[p] = acc;
    }
}

extern "C" int comap_bin_values_f64(comap_ctx *ctx, double *image, int64_t npix, const int64_t *pixels,
                                    const double *weights, const int64_t *mask, int64_t n)
{
    if (!ctx || !image || (!pixels && n > 0)) return -1;
    COMAP_DEVICE_GUARD(ctx);
    if (npix <= 0 || n <= 0) return 0;
    if (npix >= (1ll << 31) - 1 || n >= (1ll << 31)) return comap_fail(ctx, -1, "binValues size limit exceeded");
    int end_bit = 1;
    while ((1ll << end_bit) <= npix) ++end_bit;
    size_t tmp_bytes = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, (int32_t *)nullptr, (int32_t *)nullptr,
                                       (int32_t *)nullptr, (int32_t *)nullptr, (int)n, 0, end_bit, ctx->stream);
    const size_t bytes = 8 * (size_t)n * 3 + 8 * (size_t)npix + 16 * (size_t)n + tmp_bytes + 4096;
    char *s = nullptr;
    int rc = comap_scratch(ctx, bytes, (void **)&s);
    if (rc) return rc;
    auto align = [](char *p) { return (char *)(((uintptr_t)p + 255) & ~(uintptr_t)255); };
    int64_t *dpix = (int64_t *)align(s);
    double *dw = (double *)align((char *)(dpix + n));
    int64_t *dmask = (int64_t *)align((char *)(dw + n));
    double *dimg = (double *)align((char *)(dmask + n));
    int32_t *k0 = (int32_t *)align((char *)(dimg + npix));
    int32_t *k1 = (int32_t *)align((char *)(k0 + n));
    int32_t *v0 = (int32_t *)align((char *)(k1 + n));
    int32_t *v1 = (int32_t *)align((char *)(v0 + n));
    void *tmp = (void *)align((char *)(v1 + n));
    hipStream_t st = ctx->stream;
    COMAP_CHECK(ctx, hipMemcpyAsync(dpix, pixels, 8 * n, hipMemcpyHostToDevice, st));
    if (weights) COMAP_CHECK(ctx, hipMemcpyAsync(dw, weights, 8 * n, hipMemcpyHostToDevice, st));
    if (mask) COMAP_CHECK(ctx, hipMemcpyAsync(dmask, mask, 8 * n, hipMemcpyHostToDevice, st));
    COMAP_CHECK(ctx, hipMemcpyAsync(dimg, image, 8 * npix, hipMemcpyHostToDevice, st));
    k_bin_keys<<<1024, 256, 0, st>>>(dpix, mask ? dmask : nullptr, n, npix, k0, v0);
    COMAP_LAUNCH_CHECK(ctx);
    COMAP_CHECK(ctx, hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, k0, k1, v0, v1, (int)n, 0, end_bit, st));
    k_bin_ordered<<<1024, 256, 0, st>>>(k1, v1, n, weights ? dw : nullptr, npix, dimg);
    COMAP_LAUNCH_CHECK(ctx);
    COMAP_CHECK(ctx, hipMemcpyAsync(image, dimg, 8 * npix, hipMemcpyDeviceToHost, st));
    COMAP_CHECK(ctx, hipStreamSynchronize(st));
    return 0;
}
