// ds_add_f32 throughput by address pattern (the texel scatter's LDS adds).
// Each wave issues `iters` no-return LDS float adds; reports LDS cycles per
// wave-instruction per CU.  build: hipcc -O3 --offload-arch=gfx950 tools/exp_ldsatomic.hip -o tools/exp_ldsatomic
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef __attribute__((address_space(3))) float LdsF;

__device__ __forceinline__ uint32_t hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

template <int Pat>
__global__ void __launch_bounds__(512) k(float *out, uint32_t iters, uint32_t n_floats) {
    extern __shared__ float lds[];
    LdsF *acc = (LdsF *)lds;
    for (uint32_t i = threadIdx.x; i < n_floats; i += blockDim.x) acc[i] = 0.f;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t s = hash(threadIdx.x * 7919u + blockIdx.x * 104729u);
    for (uint32_t it = 0; it < iters; ++it) {
        uint32_t a;
        if (Pat == 0) a = lane;                              // distinct, conflict-free
        else if (Pat == 1) a = lane * 3u + (it & 31u) * 192u;  // stride 3 (texel * 3 + c)
        else if (Pat == 2) { s = hash(s + it); a = s & 8191u; }  // random over 8192
        else if (Pat == 3) a = 17u;                          // one address
        else if (Pat == 4) a = (lane >> 3) * 3u;             // 8 addresses, 8 lanes each
        else a = (lane >> 1) * 3u;                           // 32 addresses, 2 lanes each
        if (Pat == 6) { s = hash(s + it); a = s & 8191u; acc[a] = acc[a] + 1.f; }  // random RMW, not atomic
        else if (Pat >= 7) {  // other atomic types, random addresses
            s = hash(s + it); a = s & 4095u;
            if (Pat == 7) __hip_atomic_fetch_add((__attribute__((address_space(3))) uint32_t *)acc + a, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            else if (Pat == 8) __hip_atomic_fetch_add((__attribute__((address_space(3))) unsigned long long *)acc + a, (unsigned long long)s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            else if (Pat == 9) __hip_atomic_fetch_add((__attribute__((address_space(3))) double *)acc + a, (double)lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            else if (Pat == 10) out[blockIdx.x] += __hip_atomic_fetch_add(acc + a, (float)lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            else __hip_atomic_fetch_max((__attribute__((address_space(3))) uint32_t *)acc + a, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        else __hip_atomic_fetch_add(acc + a, (float)lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = acc[17];
}

template <int Pat>
void run(const char *name, int cus, float *out, hipEvent_t e0, hipEvent_t e1) {
    const uint32_t iters = 4096, n_floats = 12288, threads = 512, per_cu = 3;
    const uint32_t blocks = cus * per_cu;
    hipLaunchKernelGGL(k<Pat>, dim3(blocks), dim3(threads), n_floats * 4, 0, out, iters, n_floats);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<Pat>, dim3(blocks), dim3(threads), n_floats * 4, 0, out, iters, n_floats);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    const double inst_per_cu = (double)per_cu * (threads / 64) * iters;
    printf("%-34s %8.3f ms  %6.2f cycles per wave-instruction per CU (2.4 GHz)\n", name, ms,
           ms * 1e-3 * 2.4e9 / inst_per_cu);
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float *out;
    hipMalloc(&out, 4096 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    run<0>("ds_add lane (distinct banks)", cus, out, e0, e1);
    run<1>("ds_add 3*lane (texel*3+c)", cus, out, e0, e1);
    run<2>("ds_add random over 12288", cus, out, e0, e1);
    run<3>("ds_add one address", cus, out, e0, e1);
    run<4>("ds_add 8 addresses x 8 lanes", cus, out, e0, e1);
    run<5>("ds_add 32 addresses x 2 lanes", cus, out, e0, e1);
    run<6>("read+add+write random (not atomic)", cus, out, e0, e1);
    run<7>("ds_add_u32 random", cus, out, e0, e1);
    run<8>("ds_add_u64 random", cus, out, e0, e1);
    run<9>("ds_add_f64 random", cus, out, e0, e1);
    run<10>("ds_add_rtn_f32 random (value used)", cus, out, e0, e1);
    run<11>("ds_max_u32 random", cus, out, e0, e1);
    return 0;
}
