// Probe: latency of a hand-off between TWO workgroups of one launch (a pair per example, as a
// two-workgroup split of the C3 forward would need): workgroup A stores NV floats and a flag,
// B polls the flag and reads the floats, then answers the same way -- R round trips.  Stores and
// loads of the handed-off words are relaxed agent-scope atomics (global_store / load ... sc1: the
// MI355X guide's hand-off row without an acquire); pairs on one XCD (blocks b, b + 8) and on two.
//   build: hipcc -O3 --offload-arch=gfx950 pair_probe.hip -o pair_probe
//   run:   ./pair_probe     (us per one-way hand-off, p50 over pairs, both placements)
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int NPAIR = 100, BT = 512, NV = 128, R = 50;
constexpr int SPIN_MAX = 1 << 20;               // bounded polls: every wave exits

__device__ __forceinline__ void st(float* p, float v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld(const float* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// same_xcd: pair p = blocks (A, A + 8) with A = 16 (p / 8) + p % 8; else (2p, 2p + 1)
__global__ __launch_bounds__(BT) void k_pair(float* buf, int* flags, unsigned long long* t,
                                             int* err, int same_xcd) {
    extern __shared__ float sm[];
    const int b = blockIdx.x;
    int p, side;
    if (same_xcd) { p = (b / 16) * 8 + (b % 8); side = (b % 16) >= 8; }
    else { p = b / 2; side = b & 1; }
    if (p >= NPAIR) return;
    float* mine = buf + (size_t)(2 * p + side) * NV;
    const float* theirs = buf + (size_t)(2 * p + 1 - side) * NV;
    int* myflag = flags + (2 * p + side) * 32;
    const int* theirflag = flags + (2 * p + 1 - side) * 32;
    sm[threadIdx.x] = 0.f;
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    float acc = 0.f;
    for (int r = 1; r <= R; ++r) {
        const bool send_first = side == 0;
        for (int ph = 0; ph < 2; ++ph) {
            const bool sending = (ph == 0) == send_first;
            if (sending) {
                if (threadIdx.x < NV) st(mine + threadIdx.x, (float)(r * 1000 + p) + acc * 0.f);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                if (threadIdx.x == 0)
                    __hip_atomic_store(myflag, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                if (threadIdx.x == 0) {
                    int n = 0;
                    while (__hip_atomic_load(theirflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < r &&
                           ++n < SPIN_MAX) {}
                    if (n >= SPIN_MAX) atomicAdd(err, 1);
                }
                __syncthreads();
                if (threadIdx.x < NV) {
                    const float v = ld(theirs + threadIdx.x);
                    if (v != (float)(r * 1000 + p)) atomicAdd(err + 1, 1);
                    acc += v;
                }
            }
        }
    }
    if (threadIdx.x == 0 && side == 0) t[p] = __builtin_amdgcn_s_memrealtime() - t0;
    sm[threadIdx.x] += acc;
}

int main() {
    float* buf; int* flags; unsigned long long* t; int* err;
    CHK(hipMalloc(&buf, sizeof(float) * 2 * NPAIR * NV));
    CHK(hipMalloc(&flags, sizeof(int) * 2 * NPAIR * 32));
    CHK(hipMalloc(&t, sizeof(unsigned long long) * NPAIR));
    CHK(hipMalloc(&err, sizeof(int) * 2));
    const size_t lds = 100 * 1024;                 // one workgroup per CU, as the forward
    CHK(hipFuncSetAttribute((const void*)k_pair, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    for (int same = 1; same >= 0; --same) {
        std::vector<double> med;
        for (int rep = 0; rep < 5; ++rep) {
            CHK(hipMemset(flags, 0, sizeof(int) * 2 * NPAIR * 32));
            CHK(hipMemset(err, 0, sizeof(int) * 2));
            const int grid = same ? 16 * ((NPAIR + 7) / 8) : 2 * NPAIR;
            hipLaunchKernelGGL(k_pair, dim3(grid), dim3(BT), lds, 0, buf, flags, t, err, same);
            CHK(hipDeviceSynchronize());
            std::vector<unsigned long long> h(NPAIR);
            int he[2];
            CHK(hipMemcpy(h.data(), t, sizeof(unsigned long long) * NPAIR, hipMemcpyDeviceToHost));
            CHK(hipMemcpy(he, err, sizeof(he), hipMemcpyDeviceToHost));
            std::sort(h.begin(), h.end());
            const double us = h[NPAIR / 2] / 100.0 / (2.0 * R);   // s_memrealtime: 100 MHz
            med.push_back(us);
            printf("%s rep %d: one-way hand-off p50 %.3f us (max pair %.3f us), timeouts %d, stale %d\n",
                   same ? "same XCD" : "two XCDs", rep, us, h[NPAIR - 1] / 100.0 / (2.0 * R), he[0], he[1]);
        }
    }
    return 0;
}
