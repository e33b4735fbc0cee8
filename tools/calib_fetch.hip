// calib_fetch.hip — known-byte kernels that calibrate rocprofv3's FETCH_SIZE /
// WRITE_SIZE on gfx950 for the access patterns of the bounce kernels
// (MI355X_MICROARCH.md: FETCH_SIZE reads 1/2 of a 16-B/lane streaming read;
// other widths are uncalibrated).
//
//   k_read4    P planes of 4 B per lane   (WfState / WfPrb: k_wf_bounce_prb)
//   k_read16   P planes of 16 B per lane  (WfPacked: k_wf_bounce)
//   k_write4 / k_write16                  the matching stores
// Each kernel touches n lanes x P planes once; the planes (P x n x width) far
// exceed the 256 MiB Infinity Cache, so every byte comes from / goes to HBM.
// The sink store of the read kernels is predicated on an impossible value.
//
// usage (on the GPU box): calib_fetch        prints the known bytes per kernel
//   rocprofv3 --kernel-trace --pmc FETCH_SIZE -- tools/calib_fetch
//   rocprofv3 --kernel-trace --pmc WRITE_SIZE -- tools/calib_fetch
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr int P = 20;  // planes, as the bounce kernels' state

__global__ void k_read4(const float *__restrict__ base, size_t stride, size_t n, float *sink) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float s = 0.f;
#pragma unroll
    for (int p = 0; p < P; ++p) s += base[p * stride + i];
    if (s == -12345.f) sink[i] = s;
}

__global__ void k_read16(const float4 *__restrict__ base, size_t stride, size_t n, float *sink) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float s = 0.f;
#pragma unroll
    for (int p = 0; p < P / 4; ++p) {
        const float4 v = base[p * stride + i];
        s += (v.x + v.y) + (v.z + v.w);
    }
    if (s == -12345.f) sink[i] = s;
}

__global__ void k_write4(float *__restrict__ base, size_t stride, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
#pragma unroll
    for (int p = 0; p < P; ++p) base[p * stride + i] = (float)(p + i);
}

__global__ void k_write16(float4 *__restrict__ base, size_t stride, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
#pragma unroll
    for (int p = 0; p < P / 4; ++p) base[p * stride + i] = make_float4(p, i, 0.f, 1.f);
}

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
            return 1;                                                            \
        }                                                                        \
    } while (0)

int main() {
    const size_t n = 1u << 24;  // lanes (one 2^24-path wavefront chunk)
    const size_t bytes = (size_t)P * n * 4;
    float *buf = nullptr, *sink = nullptr;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&sink, n * 4));
    CK(hipMemset(buf, 0, bytes));
    const dim3 g((unsigned)(n / 256)), b(256);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_write4, g, b, 0, 0, buf, n, n);
        hipLaunchKernelGGL(k_read4, g, b, 0, 0, buf, n, n, sink);
        hipLaunchKernelGGL(k_write16, g, b, 0, 0, reinterpret_cast<float4 *>(buf), n, n);
        hipLaunchKernelGGL(k_read16, g, b, 0, 0, reinterpret_cast<const float4 *>(buf), n, n, sink);
    }
    CK(hipDeviceSynchronize());
    printf("{\"bytes_per_launch\": %zu, \"lanes\": %zu, \"planes\": %d}\n", bytes, n, P);
    CK(hipFree(buf));
    CK(hipFree(sink));
    return 0;
}
