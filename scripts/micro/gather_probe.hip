// Microbenchmark (round 5): what bounds the destriper CG pair's scattered map gathers?
// A [NPIX][4] f64 map (7.4 MB, the C5 480 x 480 map with 4 bands interleaved) is gathered
// at E entry indices laid out like the sliced-ELLPACK projection (column-major chunks of
// 64 lanes: entry j of lane l at 64 j + l), each lane walking its own column with 8 loads
// in flight, in several lane <-> (entry, band) shapes:
//   A  lane = entry, 2 x 16-B loads (bands 0-1, 2-3): the production kernel's shape
//   B  4 lanes per entry, lane = band, one 8-B load each (a quad reads 32 contiguous B)
//   C  lane = entry, one 8-B load (band 0 only: the 1-band problem's shape)
//   D  lane = entry, 4 x 8-B loads
// over index patterns: uniform random pixels; Lissajous-like tracks (each lane a random
// walk of unit pixel steps from a start pixel, starts sorted across lanes as the spatial
// offset order sorts them); and every lane of a column on the same pixel (broadcast).
// Prints us per pass and ns per entry.  Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

typedef double d2v __attribute__((ext_vector_type(2)));
constexpr int U = 8;

__global__ void __launch_bounds__(256) kA(const int *__restrict__ idx, int W, int nchunk, const double *__restrict__ m,
                                          double *__restrict__ out)
{
    const int lane = threadIdx.x & 63;
    for (int c = blockIdx.x * 4 + (threadIdx.x >> 6); c < nchunk; c += gridDim.x * 4) {
        const int *p = idx + (size_t)c * W * 64 + lane;
        double s0 = 0, s1 = 0, s2 = 0, s3 = 0;
        for (int j = 0; j < W; j += U) {
            int q[U];
#pragma unroll
            for (int u = 0; u < U; ++u) q[u] = p[64 * (j + u)];
            d2v a[U], b[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                a[u] = *reinterpret_cast<const d2v *>(m + 4 * (size_t)q[u]);
                b[u] = *reinterpret_cast<const d2v *>(m + 4 * (size_t)q[u] + 2);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) { s0 += a[u].x; s1 += a[u].y; s2 += b[u].x; s3 += b[u].y; }
        }
        out[(size_t)c * 64 + lane] = s0 + s1 + s2 + s3;
    }
}

__global__ void __launch_bounds__(256) kB(const int *__restrict__ idx, int W, int nchunk, const double *__restrict__ m,
                                          double *__restrict__ out)
{
    const int lane = threadIdx.x & 63, band = lane & 3, sub = lane >> 2;   // 16 entries-lanes x 4 bands
    // a wave covers 16 of the chunk's 64 columns: 4 waves per chunk
    for (int cw = blockIdx.x * 4 + (threadIdx.x >> 6); cw < nchunk * 4; cw += gridDim.x * 4) {
        const int c = cw >> 2, col = (cw & 3) * 16 + sub;
        const int *p = idx + (size_t)c * W * 64 + col;
        double s = 0;
        for (int j = 0; j < W; j += U) {
            int q[U];
#pragma unroll
            for (int u = 0; u < U; ++u) q[u] = p[64 * (j + u)];
            double a[U];
#pragma unroll
            for (int u = 0; u < U; ++u) a[u] = m[4 * (size_t)q[u] + band];
#pragma unroll
            for (int u = 0; u < U; ++u) s += a[u];
        }
        out[(size_t)c * 256 + (cw & 3) * 64 + lane] = s;
    }
}

__global__ void __launch_bounds__(256) kC(const int *__restrict__ idx, int W, int nchunk, const double *__restrict__ m1,
                                          double *__restrict__ out)
{
    const int lane = threadIdx.x & 63;
    for (int c = blockIdx.x * 4 + (threadIdx.x >> 6); c < nchunk; c += gridDim.x * 4) {
        const int *p = idx + (size_t)c * W * 64 + lane;
        double s = 0;
        for (int j = 0; j < W; j += U) {
            int q[U];
#pragma unroll
            for (int u = 0; u < U; ++u) q[u] = p[64 * (j + u)];
            double a[U];
#pragma unroll
            for (int u = 0; u < U; ++u) a[u] = m1[q[u]];
#pragma unroll
            for (int u = 0; u < U; ++u) s += a[u];
        }
        out[(size_t)c * 64 + lane] = s;
    }
}

__global__ void __launch_bounds__(256) kD(const int *__restrict__ idx, int W, int nchunk, const double *__restrict__ m,
                                          double *__restrict__ out)
{
    const int lane = threadIdx.x & 63;
    for (int c = blockIdx.x * 4 + (threadIdx.x >> 6); c < nchunk; c += gridDim.x * 4) {
        const int *p = idx + (size_t)c * W * 64 + lane;
        double s = 0;
        for (int j = 0; j < W; j += U) {
            int q[U];
#pragma unroll
            for (int u = 0; u < U; ++u) q[u] = p[64 * (j + u)];
            double a[U][4];
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int b = 0; b < 4; ++b) a[u][b] = m[4 * (size_t)q[u] + b];
#pragma unroll
            for (int u = 0; u < U; ++u) s += (a[u][0] + a[u][1]) + (a[u][2] + a[u][3]);
        }
        out[(size_t)c * 64 + lane] = s;
    }
}

int main(int argc, char **argv)
{
    const int NX = 480, NPIX = NX * NX, W = 40;          // 40 entries per lane (C5: ~37 per offset)
    const int nchunk = argc > 1 ? atoi(argv[1]) : 8192;  // 8192 chunks x 64 lanes x 40 = 21 M entries
    const size_t E = (size_t)nchunk * 64 * W;
    double *m, *out;
    int *idx;
    hipMalloc(&m, 8 * 4 * (size_t)NPIX);
    hipMalloc(&out, 8 * (size_t)nchunk * 256);
    hipMalloc(&idx, 4 * E);
    std::vector<double> hm(4 * (size_t)NPIX);
    for (size_t i = 0; i < hm.size(); ++i) hm[i] = 1e-3 * (double)(i % 977);
    hipMemcpy(m, hm.data(), 8 * hm.size(), hipMemcpyHostToDevice);
    std::mt19937_64 rng(7);
    std::vector<int> hi(E);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const char *pats[] = {"uniform", "tracks", "broadcast"};
    for (int pat = 0; pat < 3; ++pat) {
        if (pat == 0) {
            for (auto &v : hi) v = (int)(rng() % NPIX);
        } else if (pat == 1) {
            // per chunk: 64 sorted start pixels in a band of rows, each lane a unit-step walk
            for (int c = 0; c < nchunk; ++c) {
                std::vector<int> st(64);
                const int row0 = (int)(((size_t)c * NX) / nchunk);
                for (auto &s : st) s = row0 * NX + (int)(rng() % (3 * NX));
                std::sort(st.begin(), st.end());
                for (int l = 0; l < 64; ++l) {
                    int x = st[l] % NX, y = std::min(st[l] / NX, NX - 1);
                    const int dx = (int)(rng() % 3) - 1, dy = (int)(rng() % 3) - 1;
                    for (int j = 0; j < W; ++j) {
                        hi[(size_t)c * W * 64 + 64 * (size_t)j + l] = y * NX + x;
                        if (rng() % 2) x = std::min(std::max(x + (dx ? dx : 1), 0), NX - 1);
                        else y = std::min(std::max(y + (dy ? dy : 1), 0), NX - 1);
                    }
                }
            }
        } else {
            for (size_t i = 0; i < E; ++i) hi[i] = (int)((i / 64) % NPIX);
        }
        hipMemcpy(idx, hi.data(), 4 * E, hipMemcpyHostToDevice);
        for (int k = 0; k < 4; ++k) {
            auto run = [&]() {
                if (k == 0) kA<<<2048, 256>>>(idx, W, nchunk, m, out);
                if (k == 1) kB<<<2048, 256>>>(idx, W, nchunk, m, out);
                if (k == 2) kC<<<2048, 256>>>(idx, W, nchunk, m, out);
                if (k == 3) kD<<<2048, 256>>>(idx, W, nchunk, m, out);
            };
            for (int w = 0; w < 3; ++w) run();
            const int R = 20;
            hipEventRecord(a);
            for (int r = 0; r < R; ++r) run();
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            const double us = ms * 1e3 / R;
            printf("%-9s kernel %c  %8.1f us  %.3f ns/entry\n", pats[pat], "ABCD"[k], us, us * 1e3 / (double)E);
        }
    }
    return 0;
}
