// STREAM copy probe: which float4 copy form reaches the highest HBM rate on this box.
// usage: ./stream_probe   (prints GB/s per variant; 2 GiB read + 2 GiB written per copy)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

typedef float v4f __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_k(const v4f* __restrict__ s, v4f* __restrict__ d, long n) {
    const long stride = (long)gridDim.x * 256 * U;
    for (long i = (long)blockIdx.x * 256 * U + threadIdx.x; i < n; i += stride) {
        v4f v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long k = i + 256 * u;
            if (k < n) v[u] = NT ? __builtin_nontemporal_load(s + k) : s[k];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long k = i + 256 * u;
            if (k < n) { if (NT) __builtin_nontemporal_store(v[u], d + k); else d[k] = v[u]; }
        }
    }
}

template <int U, bool NT>
static void run(const char* name, const v4f* s, v4f* d, long n, int grid) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    std::vector<float> t;
    for (int it = 0; it < 8; ++it) {
        hipEventRecord(a);
        hipLaunchKernelGGL((copy_k<U, NT>), dim3(grid), dim3(256), 0, 0, s, d, n);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        if (it) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    const double ms = t[t.size() / 2];
    printf("%-28s grid %6d  %.3f ms  %.0f GB/s\n", name, grid, ms, 2.0 * n * 16 / (ms * 1e-3) / 1e9);
}

int main() {
    const long bytes = 1L << 31, n = bytes / 16;
    v4f *s, *d;
    hipMalloc(&s, bytes); hipMalloc(&d, bytes);
    hipMemset(s, 1, bytes); hipMemset(d, 0, bytes);
    for (int grid : {4096, 8192, 16384, 32768}) {
        run<4, false>("U4 plain", s, d, n, grid);
        run<4, true>("U4 nontemporal", s, d, n, grid);
        run<8, false>("U8 plain", s, d, n, grid);
        run<8, true>("U8 nontemporal", s, d, n, grid);
        run<2, false>("U2 plain", s, d, n, grid);
        run<1, false>("U1 plain", s, d, n, grid);
    }
    return 0;
}
