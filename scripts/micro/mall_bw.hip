// Microbenchmark: streaming-read bandwidth vs working-set size (HBM vs Infinity Cache).
// Reads a buffer of S bytes R times (sum of floats, one f32x4 per lane per step).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void __launch_bounds__(256) k_read(const float4 *__restrict__ p, size_t n4, float *out)
{
    float s = 0.f;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll 8
    for (; i < n4; i += stride) {
        float4 v = p[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 12345.f) out[0] = s;
}

int main()
{
    const size_t maxb = (size_t)8 << 30;
    float *buf, *out;
    hipMalloc(&buf, maxb);
    hipMalloc(&out, 64);
    hipMemset(buf, 0, maxb);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    size_t sizes[] = {16ull << 20, 32ull << 20, 64ull << 20, 96ull << 20, 128ull << 20, 160ull << 20,
                      192ull << 20, 224ull << 20, 256ull << 20, 384ull << 20, 1ull << 30, 8ull << 30};
    for (size_t S : sizes) {
        for (int grid : {2048, 8192}) {
            const size_t n4 = S / 16;
            for (int w = 0; w < 3; ++w) k_read<<<grid, 256>>>((const float4 *)buf, n4, out);
            const int R = S >= (1ull << 30) ? 5 : 50;
            hipEventRecord(a);
            for (int r = 0; r < R; ++r) k_read<<<grid, 256>>>((const float4 *)buf, n4, out);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            printf("S=%8.1f MB grid=%5d  %.3f us/read  %.2f TB/s\n", S / 1048576.0, grid, ms * 1e3 / R,
                   (double)S * R / (ms * 1e-3) / 1e12);
        }
    }
    return 0;
}
