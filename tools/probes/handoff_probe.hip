// Probe: producer -> consumer hand-off inside ONE launch (agent-scope release / acquire and an
// arrival counter) against the same work as two launches, on MI355X.  Shapes mirror the C5
// forward's k_bil_enc -> k_bil_mt pass: 100 producer workgroups (a dependent-load chain, then a
// 1288-float record each) and 325 consumer workgroups (stage 51 KB of a 16 MB tensor into LDS,
// then read the first 100 floats of every record).  Consumers check every value they read
// against this iteration's (stale-data detector) and count mismatches.
//   build: hipcc -O3 --offload-arch=gfx950 handoff_probe.hip -o handoff_probe
//   run:   ./handoff_probe            (prints us per iteration of each form, and errors)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
    printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int NP = 100, NC = 325, BT = 512, REC = 1288, NREAD = 100;
constexpr int CHAIN = 6;                      // dependent loads per producer (~encoder latency)
constexpr long RSZ = 16L << 20;               // bytes of the staged tensor
constexpr int STAGE = 8 * 16 * 100;           // floats staged per consumer (51 KB)
constexpr long CHN = 16L << 20;               // ints in the chase buffer (64 MB)
constexpr int SPIN_MAX = 1 << 22;             // bounded wait: every wave exits

struct Args {
    const int* chase; float* rec; const float* R; float* out; int* cnt; int* err; int iter;
};

template <int F>
__device__ void produce(const Args& a, int b, float* sm) {
    if (threadIdx.x == 0) {
        int x = (b * 7919) & (CHN - 1);
        for (int k = 0; k < CHAIN; ++k) x = a.chase[x];
        sm[0] = (float)(x & 1);
    }
    __syncthreads();
    const float v = (float)(a.iter * 1000 + b) + 0.f * sm[0];
    for (int t = threadIdx.x; t < REC; t += BT) {
        if (F == 2) __hip_atomic_store(a.rec + (long)b * REC + t, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else a.rec[(long)b * REC + t] = v;
    }
}

__device__ void consume(const Args& a, int c, float* sm) {
    const float4* R4 = reinterpret_cast<const float4*>(a.R);
    const long base = ((long)c * STAGE / 4) % (RSZ / 16 - STAGE / 4);
    for (int e = threadIdx.x; e < STAGE / 4; e += BT) reinterpret_cast<float4*>(sm)[e] = R4[base + e];
    __syncthreads();
}

template <int F>
__device__ void consume_tail(const Args& a, int c, float* sm) {
    float s = sm[threadIdx.x % STAGE];
    int bad = 0;
    for (int e = threadIdx.x; e < NP * NREAD; e += BT) {
        const int b = e / NREAD, k = e - b * NREAD;
        const float v = (F >= 2) ? __hip_atomic_load(a.rec + (long)b * REC + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                 : a.rec[(long)b * REC + k];
        bad += v != (float)(a.iter * 1000 + b);
        s += v;
    }
    if (bad) atomicAdd(a.err, bad);
    a.out[(long)c * BT + threadIdx.x] = s;
}

__global__ __launch_bounds__(BT) void k_prod(Args a) {
    __shared__ float sm[16];
    produce<0>(a, blockIdx.x, sm);
}
__global__ __launch_bounds__(BT) void k_cons(Args a) {
    extern __shared__ float sm[];
    consume(a, blockIdx.x, sm);
    consume_tail<0>(a, blockIdx.x, sm);
}
// one launch: workgroups [0, NP) produce, [NP, NP + NC) consume after all producers arrived
template <int F>
__global__ __launch_bounds__(BT) void k_fused(Args a) {
    extern __shared__ float sm[];
    __shared__ int ok;
    if (blockIdx.x < NP) {
        produce<F>(a, blockIdx.x, sm);
        if (F == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            if (F != 2) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            __hip_atomic_fetch_add(a.cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
    const int c = blockIdx.x - NP;
    consume(a, c, sm);
    if (threadIdx.x == 0) {
        int it = 0;
        while (__hip_atomic_load(a.cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < NP && ++it < SPIN_MAX)
            __builtin_amdgcn_s_sleep(1);
        if (it >= SPIN_MAX) atomicAdd(a.err, 1 << 20);
        if (F == 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        ok = 1;
    }
    __syncthreads();
    consume_tail<F>(a, c, sm);
    __syncthreads();
    if (threadIdx.x == 0) {          // the last consumer resets the counters for the next launch
        const int d = __hip_atomic_fetch_add(a.cnt + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (d == NC - 1) {
            __hip_atomic_store(a.cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a.cnt + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

int main() {
    int *chase, *cnt, *err;
    float *rec, *R, *out;
    CHK(hipMalloc(&chase, CHN * 4));
    CHK(hipMalloc(&rec, (long)NP * REC * 4));
    CHK(hipMalloc(&R, RSZ));
    CHK(hipMalloc(&out, (long)NC * BT * 4));
    CHK(hipMalloc(&cnt, 8));
    CHK(hipMalloc(&err, 4));
    std::vector<int> h(CHN);
    unsigned s = 12345;
    for (long i = 0; i < CHN; ++i) { s = s * 1103515245u + 12345u; h[i] = (int)((s >> 4) & (CHN - 1)); }
    CHK(hipMemcpy(chase, h.data(), CHN * 4, hipMemcpyHostToDevice));
    CHK(hipMemset(R, 0, RSZ));
    CHK(hipMemset(cnt, 0, 8));
    CHK(hipMemset(err, 0, 4));
    const size_t lds = STAGE * 4;
    CHK(hipFuncSetAttribute((const void*)k_cons, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    CHK(hipFuncSetAttribute((const void*)k_fused<1>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    CHK(hipFuncSetAttribute((const void*)k_fused<2>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    CHK(hipFuncSetAttribute((const void*)k_fused<3>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    hipStream_t st;
    CHK(hipStreamCreate(&st));
    const int NIT = 64;
    const char* names[4] = {"two launches", "one launch, release/acquire fences",
                            "one launch, coherent (sc1) stores + loads, no fences",
                            "one launch, release fence + coherent loads"};
    for (int form = 0; form < 4; ++form) {
        for (int rep = 0; rep < 3; ++rep) {
            hipGraph_t g;
            hipGraphExec_t ge;
            CHK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
            for (int i = 0; i < NIT; ++i) {
                Args a{chase, rec, R, out, cnt, err, rep * NIT + i + 1};
                if (form == 0) {
                    hipLaunchKernelGGL(k_prod, dim3(NP), dim3(BT), 0, st, a);
                    hipLaunchKernelGGL(k_cons, dim3(NC), dim3(BT), lds, st, a);
                } else if (form == 1) {
                    hipLaunchKernelGGL(k_fused<1>, dim3(NP + NC), dim3(BT), lds, st, a);
                } else if (form == 2) {
                    hipLaunchKernelGGL(k_fused<2>, dim3(NP + NC), dim3(BT), lds, st, a);
                } else {
                    hipLaunchKernelGGL(k_fused<3>, dim3(NP + NC), dim3(BT), lds, st, a);
                }
            }
            CHK(hipStreamEndCapture(st, &g));
            CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            CHK(hipGraphUpload(ge, st));
            CHK(hipStreamSynchronize(st));
            hipEvent_t e0, e1;
            CHK(hipEventCreate(&e0));
            CHK(hipEventCreate(&e1));
            CHK(hipEventRecord(e0, st));
            CHK(hipGraphLaunch(ge, st));
            CHK(hipEventRecord(e1, st));
            CHK(hipStreamSynchronize(st));
            float ms = 0;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            int herr = 0;
            CHK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
            printf("%s rep %d: %.2f us per iteration, errors %d (spin timeouts %d)\n",
                   names[form], rep, ms * 1e3 / NIT,
                   herr & ((1 << 20) - 1), herr >> 20);
            CHK(hipMemset(err, 0, 4));
            CHK(hipGraphExecDestroy(ge));
            CHK(hipGraphDestroy(g));
        }
    }
    return 0;
}
