// Exhaustive / sampled check of short reciprocal and division sequences
// against the correctly rounded 1/x and a/b (-fhip-fp32-correctly-rounded-divide-sqrt).
// build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt tools/exp_rcp.hip -o /tmp/exp_rcp
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>

__device__ __forceinline__ float rcp_nr(float b) {
    const float y = __builtin_amdgcn_rcpf(b);
    const float e = __builtin_fmaf(-b, y, 1.f);
    return __builtin_fmaf(e, y, y);
}
__device__ __forceinline__ float rcp_nr_fix(float b) { return __builtin_amdgcn_div_fixupf(rcp_nr(b), b, 1.f); }
// a/b from y = RN(1/b): q0 = a*y, two residual corrections
__device__ __forceinline__ float div_nr1(float a, float b, float y) {
    const float q = a * y;
    const float r = __builtin_fmaf(-b, q, a);
    return __builtin_fmaf(r, y, q);
}
__device__ __forceinline__ float div_nr2(float a, float b, float y) {
    const float q1 = div_nr1(a, b, y);
    const float r = __builtin_fmaf(-b, q1, a);
    return __builtin_fmaf(r, y, q1);
}

__device__ __forceinline__ bool same(float x, float y) {
    return __float_as_uint(x) == __float_as_uint(y) || (x != x && y != y);
}
// bucket by the biased exponent of the input: 0 = zero/denormal, 1 = [2^-126, 2^-64), 2 = [2^-64, 2^64), 3 = [2^64, 2^126), 4 = >= 2^126 finite, 5 = inf/nan
__device__ __forceinline__ int bucket(float x) {
    const uint32_t e = (__float_as_uint(x) >> 23) & 0xffu;
    if (e == 0) return 0;
    if (e == 255) return 5;
    if (e < 127 - 64) return 1;
    if (e < 127 + 64) return 2;
    if (e < 127 + 126) return 3;
    return 4;
}

__global__ void k_rcp(unsigned long long *cnt) {
    const uint64_t total = 1ull << 32;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
        const float b = __uint_as_float((uint32_t)i);
        const float ref = 1.0f / b;
        const int k = bucket(b);
        if (!same(rcp_nr(b), ref)) atomicAdd(&cnt[k], 1ull);
        if (!same(rcp_nr_fix(b), ref)) atomicAdd(&cnt[8 + k], 1ull);
    }
}

__device__ __forceinline__ uint32_t hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

// random (a, b) with exponents in [-40, 40] plus structured mantissas; bucket 0: nr1 mismatch, 1: nr2 mismatch
__global__ void k_div(unsigned long long *cnt, uint32_t salt) {
    const uint64_t total = 1ull << 32;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t h1 = hash((uint32_t)i ^ salt), h2 = hash((uint32_t)(i >> 32) ^ h1 ^ 0x9e3779b9u);
        uint32_t ma = h1 & 0x7fffffu, mb = h2 & 0x7fffffu;
        if ((h1 >> 28) == 0) ma = 0x7fffffu;       // all-ones mantissas
        if ((h2 >> 28) == 0) mb = 0x7fffffu;
        if ((h1 >> 28) == 1) mb = 0;
        const uint32_t ea = 127 - 40 + ((h1 >> 23) % 81u), eb = 127 - 40 + ((h2 >> 23) % 81u);
        const float a = __uint_as_float((h2 & 0x80000000u) | (ea << 23) | ma);
        const float b = __uint_as_float((h1 & 0x80000000u) | (eb << 23) | mb);
        const float ref = a / b;
        const float y = 1.0f / b;
        if (!same(div_nr1(a, b, y), ref)) atomicAdd(&cnt[0], 1ull);
        if (!same(div_nr2(a, b, y), ref)) atomicAdd(&cnt[1], 1ull);
        if (!same(div_nr1(a, b, rcp_nr_fix(b)), ref)) atomicAdd(&cnt[2], 1ull);
    }
}

int main_rcp() {
    unsigned long long *d, h[16];
    hipMalloc(&d, sizeof(h));
    hipMemset(d, 0, sizeof(h));
    hipLaunchKernelGGL(k_rcp, dim3(8192), dim3(256), 0, 0, d);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    const char *nm[6] = {"zero/denorm", "[2^-126,2^-64)", "[2^-64,2^64)", "[2^64,2^126)", ">=2^126", "inf/nan"};
    printf("reciprocal, all 2^32 inputs: mismatches vs 1.0f/b\n");
    for (int k = 0; k < 6; ++k) printf("  %-16s rcp+nr %12llu   rcp+nr+fixup %12llu\n", nm[k], h[k], h[8 + k]);
    hipMemset(d, 0, sizeof(h));
    hipLaunchKernelGGL(k_div, dim3(8192), dim3(256), 0, 0, d, 12345u);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("division, 2^32 random pairs (exponents +-40): nr1 %llu  nr2 %llu  nr1(fast rcp) %llu\n", h[0], h[1], h[2]);
    return hipDeviceSynchronize() != hipSuccess;
}

// ---- square root: raw v_sqrt_f32 and v_sqrt_f32 + a Tuckerman rounding step (no range scaling)
__device__ __forceinline__ float sqrt_tuck(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sdn = __uint_as_float(__float_as_uint(s) - 1u), sup = __uint_as_float(__float_as_uint(s) + 1u);
    const float rdn = __builtin_fmaf(-sdn, s, x), rup = __builtin_fmaf(-sup, s, x);
    float r = rdn <= 0.f ? sdn : s;
    return rup > 0.f ? sup : r;
}
__global__ void k_sqrt(unsigned long long *cnt) {
    const uint64_t total = 1ull << 31;  // non-negative inputs
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
        const float x = __uint_as_float((uint32_t)i);
        const float ref = __builtin_sqrtf(x);
        const int k = bucket(x);
        if (!same(__builtin_amdgcn_sqrtf(x), ref)) atomicAdd(&cnt[k], 1ull);
        if (!same(sqrt_tuck(x), ref)) atomicAdd(&cnt[8 + k], 1ull);
    }
}
int main_sqrt() {
    unsigned long long *d, h[16];
    hipMalloc(&d, sizeof(h));
    hipMemset(d, 0, sizeof(h));
    hipLaunchKernelGGL(k_sqrt, dim3(8192), dim3(256), 0, 0, d);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    const char *nm[6] = {"zero/denorm", "[2^-126,2^-64)", "[2^-64,2^64)", "[2^64,2^126)", ">=2^126", "inf/nan"};
    printf("sqrt, all 2^31 non-negative inputs: mismatches vs sqrtf\n");
    for (int k = 0; k < 6; ++k) printf("  %-16s v_sqrt %12llu   v_sqrt+tuckerman %12llu\n", nm[k], h[k], h[8 + k]);
    return hipDeviceSynchronize() != hipSuccess;
}
int main() { return main_rcp() | main_sqrt(); }
