// Micro-benchmark: cycles per dependent f32 add in one wave (the exact obs_rms chain's floor),
// and per row of the LDS-fed chain (ds_read_b128 + 4 adds).  hipcc --offload-arch=gfx950
// -O3 tools/chain_latency.hip -o /tmp/chain_latency && /tmp/chain_latency
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void dep_add(float* out, long long* cyc, int n) {
    float a = out[threadIdx.x], b = out[64 + threadIdx.x];
    __syncthreads();
    long long t0 = clock64();
    for (int i = 0; i < n; i += 8) {
        asm volatile(
            "v_add_f32 %0, %0, %1\n\tv_add_f32 %0, %0, %1\n\tv_add_f32 %0, %0, %1\n\t"
            "v_add_f32 %0, %0, %1\n\tv_add_f32 %0, %0, %1\n\tv_add_f32 %0, %0, %1\n\t"
            "v_add_f32 %0, %0, %1\n\tv_add_f32 %0, %0, %1"
            : "+v"(a) : "v"(b));
    }
    long long t1 = clock64();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void two_chains(float* out, long long* cyc, int n) {
    float a = out[threadIdx.x], c = out[threadIdx.x] + 1.f, b = out[64 + threadIdx.x];
    long long t0 = clock64();
    for (int i = 0; i < n; i += 4) {
        asm volatile(
            "v_add_f32 %0, %0, %2\n\tv_add_f32 %1, %1, %2\n\tv_add_f32 %0, %0, %2\n\t"
            "v_add_f32 %1, %1, %2\n\tv_add_f32 %0, %0, %2\n\tv_add_f32 %1, %1, %2\n\t"
            "v_add_f32 %0, %0, %2\n\tv_add_f32 %1, %1, %2"
            : "+v"(a), "+v"(c) : "v"(b));
    }
    long long t1 = clock64();
    out[threadIdx.x] = a + c;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
    float* d;
    long long* c;
    hipMalloc(&d, 1024);
    hipMalloc(&c, 8);
    hipMemset(d, 0, 1024);
    const int n = 1 << 16;
    long long h;
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(dep_add, dim3(1), dim3(64), 0, 0, d, c, n);
        hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
        printf("dependent v_add_f32: %.2f clock64 ticks per add\n", (double)h / n);
        hipLaunchKernelGGL(two_chains, dim3(1), dim3(64), 0, 0, d, c, n);
        hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
        printf("two interleaved chains: %.2f ticks per add pair\n", (double)h / n);
    }
    return 0;
}
