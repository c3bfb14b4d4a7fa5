// Probe (tools only): cost of a cross-workgroup barrier on MI355X -- a cluster of P workgroups
// meets at a device-scope counter S times (release fence + atomic add, polling loads with a bounded
// spin, acquire fence), optionally exchanging a 77 KB image through L2 between meetings.
//   hipcc -O3 --offload-arch=gfx950 -o gridsync gridsync.hip && ./gridsync
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__device__ __forceinline__ bool cluster_barrier(unsigned *ctr, unsigned target) {
    bool ok = true;
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        atomicAdd(ctr, 1u);
        int it = 0;
        while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            if (++it > (1 << 22)) { ok = false; break; }  // never hang: give up and report
            __builtin_amdgcn_s_sleep(1);
        }
        __threadfence();
    }
    __syncthreads();
    return ok;
}

// cluster c = blockIdx % nclusters (spread) or blockIdx / P (packed); every block writes its strip of
// a [P][strip] image and, after the barrier, reads the whole image
__global__ void probe(unsigned *ctrs, int P, int S, int nclusters, int packed, float *img, int strip, int *fail) {
    const int c = packed ? blockIdx.x / P : blockIdx.x % nclusters;
    const int i = packed ? blockIdx.x % P : blockIdx.x / nclusters;
    float *base = img + (size_t)c * P * strip;
    float acc = 0.0f;
    for (int s = 0; s < S; s++) {
        for (int e = threadIdx.x; e < strip; e += blockDim.x) base[(size_t)i * strip + e] = acc + e + s;
        if (!cluster_barrier(ctrs + c, (unsigned)(P * (s + 1)))) { if (threadIdx.x == 0) atomicAdd(fail, 1); return; }
        for (int e = threadIdx.x; e < P * strip; e += blockDim.x * 8) acc += base[e];
    }
    if (acc == 12345.0f) img[0] = acc;
}

int main() {
    unsigned *ctrs;
    float *img;
    int *fail;
    CHECK(hipMalloc(&ctrs, 64 * sizeof(unsigned)));
    CHECK(hipMalloc(&img, 64 << 20));
    CHECK(hipMalloc(&fail, sizeof(int)));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int S = 15;
    for (int packed = 0; packed < 2; packed++)
        for (int P : {4, 8, 13, 16})
            for (int strip : {0, 196 * 196 / 13}) {
                const int nc = 2;
                float best = 1e9f;
                for (int rep = 0; rep < 5; rep++) {
                    CHECK(hipMemset(ctrs, 0, 64 * sizeof(unsigned)));
                    CHECK(hipMemset(fail, 0, sizeof(int)));
                    CHECK(hipEventRecord(e0));
                    hipLaunchKernelGGL(probe, dim3(P * nc), dim3(256), 0, 0, ctrs, P, S, nc, packed, img, strip, fail);
                    CHECK(hipEventRecord(e1));
                    CHECK(hipEventSynchronize(e1));
                    float ms;
                    CHECK(hipEventElapsedTime(&ms, e0, e1));
                    best = ms < best ? ms : best;
                }
                int f;
                CHECK(hipMemcpy(&f, fail, sizeof(int), hipMemcpyDeviceToHost));
                printf("packed=%d P=%2d strip=%5d floats: %d barriers %7.2f us total, %.2f us each, fail=%d\n", packed,
                       P, strip, S, best * 1e3f, best * 1e3f / S, f);
            }
    return 0;
}
