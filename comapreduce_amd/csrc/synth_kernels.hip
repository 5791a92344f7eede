// synth_kernels.hip -- device-side synthetic Level-1 cube for the benchmark.
//
// The C2 configuration (19 feeds x 4 x 1024 x 180,000 f32 = 56 GB) is too big
// to build with NumPy and push over PCIe, so bench.py generates it in HBM:
//   tod[f,b,c,t] = G_fbc * ((Tsys_fbc + level_ft + hot_ft) * mult_ft) * (1 + s n_fbct)
// with Tsys ~ U(35,45) K, G ~ 1e6 U(0.9,1.1), n ~ N(0,1) (counter-based hash +
// Box-Muller, fully deterministic in (seed, f, b, c, t) with f the feed's index in
// the whole observation, so a feed shard generates the same samples), s = 1/sqrt(dnu tau).
// level/mult/hot (atmosphere, 1/f gain drift, vane load) come from the host
// generator (comapreduce_amd/synthetic.py), so the statistics match
// SURVEY.md §8(d).  band_average = channel mean (what the spectrometer stores).
#include "comap_internal.h"

namespace {

__device__ __forceinline__ uint64_t mix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ double u01(uint64_t h) { return ((h >> 11) + 0.5) * (1.0 / 9007199254740992.0); }

__global__ void __launch_bounds__(256) k_synth(int F, int64_t T, uint64_t seed, const double *__restrict__ level,
                                               const double *__restrict__ mult, const double *__restrict__ hot,
                                               float *__restrict__ tod, int64_t row0, int64_t grow0)
{
    const int64_t row = row0 + blockIdx.y;                // (f*4+b)*1024 + c in this call's cube
    const int f = (int)(row / comap::kBC);
    const uint64_t grow = (uint64_t)(grow0 + row);        // the same row in the whole observation
    const uint64_t rs = mix64(seed ^ (0x1234567ull + grow * 0x9E3779B97F4A7C15ull));
    const double tsys = 35.0 + 10.0 * u01(mix64(rs ^ 0x51ull));
    const double g = 1e6 * (0.9 + 0.2 * u01(mix64(rs ^ 0xa3ull)));
    const float sig = (float)(1.0 / sqrt(comap::kDnuTau));
    float *out = tod + row * T;
    const double *lv = level + (int64_t)f * T, *mu = mult + (int64_t)f * T, *ho = hot + (int64_t)f * T;
    for (int64_t t = 2 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x); t < T;
         t += 2 * (int64_t)gridDim.x * blockDim.x) {
        const uint64_t h = mix64(rs + (uint64_t)t);
        const float u1 = ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);
        const float u2 = (float)((h >> 8) & 0xffffff) * (1.0f / 16777216.0f);
        const float r = sqrtf(-2.0f * __logf(u1));
        float s, c;
        __sincosf(6.28318530718f * u2, &s, &c);
        const float n0 = r * c, n1 = r * s;
        out[t] = (float)(g * ((tsys + lv[t] + ho[t]) * mu[t]) * (1.0 + (double)(sig * n0)));
        if (t + 1 < T) out[t + 1] = (float)(g * ((tsys + lv[t + 1] + ho[t + 1]) * mu[t + 1]) * (1.0 + (double)(sig * n1)));
    }
}

__global__ void __launch_bounds__(256) k_band_average(int F, int64_t T, const float *__restrict__ tod,
                                                      float *__restrict__ ba)
{
    const int fb = blockIdx.y;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < T; t += (int64_t)gridDim.x * blockDim.x) {
        const float *p = tod + (int64_t)fb * comap::kChannels * T + t;
        double s = 0;
        for (int c = 0; c < comap::kChannels; ++c) s += p[(int64_t)c * T];
        ba[(int64_t)fb * T + t] = (float)(s / comap::kChannels);
    }
}

}  // namespace

extern "C" int comap_synth_tod(comap_ctx *ctx, int32_t F, int32_t feed0, int64_t T, uint64_t seed,
                               const double *level, const double *mult, const double *hot, float *tod, float *ba)
{
    if (!ctx || !level || !mult || !hot || !tod || F <= 0 || T <= 0 || feed0 < 0) return -1;
    COMAP_DEVICE_GUARD(ctx);
    hipStream_t st = ctx->stream;
    const int64_t rows = (int64_t)F * comap::kBC;
    for (int64_t r0 = 0; r0 < rows; r0 += 65535) {
        const int64_t nr = rows - r0 < 65535 ? rows - r0 : 65535;
        dim3 grid((unsigned)((T / 2 + 255) / 256 < 64 ? (T / 2 + 255) / 256 : 64), (unsigned)nr);
        k_synth<<<grid, 256, 0, st>>>(F, T, seed, level, mult, hot, tod, r0, (int64_t)feed0 * comap::kBC);
        COMAP_LAUNCH_CHECK(ctx);
    }
    if (ba) {
        dim3 grid((unsigned)((T + 255) / 256 < 1024 ? (T + 255) / 256 : 1024), (unsigned)(F * comap::kBands));
        k_band_average<<<grid, 256, 0, st>>>(F, T, tod, ba);
        COMAP_LAUNCH_CHECK(ctx);
    }
    return 0;
}
