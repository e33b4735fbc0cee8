// Grid-gradient scatter experiment (prbvolpath sigma_t_backward): the 8
// trilinear taps of a lookup as
//   mode 0: 8 float atomics per lane into the linear (z, y, x) gradient
//           (every wave-instruction: up to 64 lanes in 64 different rows),
//   mode 1: the lanes' (cell, 8 weights) staged in wave LDS and re-issued
//           transposed into a per-cell corner buffer (8 contiguous floats per
//           cell), so one wave-instruction covers the corners of ~8 cells,
//   mode 2: per-cell corner buffer, each lane its own 8 atomics (no transpose),
// with a fraction of lanes active (divergent call sites), then the corner
// buffer gathered into the linear gradient (k_gather) and checked against mode 0.
// build: hipcc -O3 --offload-arch=gfx950 tools/exp_cellgrad.hip -o tools/exp_cellgrad
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cmath>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__device__ __forceinline__ uint32_t hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

template <int MODE>
__global__ __launch_bounds__(256) void k_scatter(float *lin, float *cell, int R, uint32_t iters, uint32_t act, uint32_t salt) {
    __shared__ float st[4][64 * 9];
    float *sc = st[threadIdx.x >> 6];
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t R1 = (uint32_t)R + 1;
    for (uint32_t it = 0; it < iters; ++it) {
        const uint32_t h = hash(tid * iters + it + salt);
        if ((h & 0xffffu) >= act) continue;
        const uint32_t h1 = hash(h ^ 0x1234567u), h2 = hash(h1), h3 = hash(h2);
        const float px = (h1 >> 8) * (1.f / 16777216.f) * R - 0.5f, py = (h2 >> 8) * (1.f / 16777216.f) * R - 0.5f,
                    pz = (h3 >> 8) * (1.f / 16777216.f) * R - 0.5f;
        const int ix = (int)floorf(px), iy = (int)floorf(py), iz = (int)floorf(pz);
        const float w1x = px - ix, w1y = py - iy, w1z = pz - iz;
        const float as = (float)(h >> 16) * 1e-6f;
        float v[8];
#pragma unroll
        for (int c = 0; c < 8; ++c)
            v[c] = as * (((c >> 2) ? w1z : 1.f - w1z) * (((c >> 1) & 1) ? w1y : 1.f - w1y)) * ((c & 1) ? w1x : 1.f - w1x);
        if (MODE == 0) {
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const int x = min(max(ix + (c & 1), 0), R - 1), y = min(max(iy + ((c >> 1) & 1), 0), R - 1),
                          z = min(max(iz + (c >> 2), 0), R - 1);
                unsafeAtomicAdd(lin + ((size_t)z * R + y) * R + x, v[c]);
            }
        } else {
            const uint32_t ci = ((uint32_t)(iz + 1) * R1 + (uint32_t)(iy + 1)) * R1 + (uint32_t)(ix + 1);
            if (MODE == 2) {
#pragma unroll
                for (int c = 0; c < 8; ++c) unsafeAtomicAdd(cell + (size_t)ci * 8 + c, v[c]);
            } else {
                const uint64_t m = __ballot(1);
                const uint32_t n = (uint32_t)__popcll(m);
                const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                sc[r * 9] = __uint_as_float(ci);
#pragma unroll
                for (int c = 0; c < 8; ++c) sc[r * 9 + 1 + c] = v[c];
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
                for (uint32_t j = 0; j < 8; ++j) {
                    const uint32_t t = j * n + r, src = t >> 3, c = t & 7u;
                    const uint32_t cc = __float_as_uint(sc[src * 9]);
                    unsafeAtomicAdd(cell + (size_t)cc * 8 + c, sc[src * 9 + 1 + c]);
                }
                __builtin_amdgcn_wave_barrier();
            }
        }
    }
}

// linear gradient += the corners of every cell that has the texel as a tap:
// per axis, the cell index i (offset by one: i = ix + 1 in [0, R]) with
// clamp(ix + b) == x, i.e. ix = x - b, plus ix = -1 (b = 0, x = 0) and
// ix = R - 1 (b = 1, x = R - 1)
__global__ void k_gather(const float *cell, float *lin, int R) {
    const size_t n = (size_t)R * R * R;
    const uint32_t R1 = (uint32_t)R + 1;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const int x = (int)(i % R), y = (int)((i / R) % R), z = (int)(i / ((size_t)R * R));
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const int bx = c & 1, by = (c >> 1) & 1, bz = c >> 2;
            int cx[2], cy[2], cz[2], nx = 1, ny = 1, nz = 1;
            cx[0] = x - bx + 1; cy[0] = y - by + 1; cz[0] = z - bz + 1;
            if (bx == 0 && x == 0) cx[nx++] = 0; else if (bx == 1 && x == R - 1) cx[nx++] = R;
            if (by == 0 && y == 0) cy[ny++] = 0; else if (by == 1 && y == R - 1) cy[ny++] = R;
            if (bz == 0 && z == 0) cz[nz++] = 0; else if (bz == 1 && z == R - 1) cz[nz++] = R;
            for (int a = 0; a < nz; ++a)
                for (int b = 0; b < ny; ++b)
                    for (int d = 0; d < nx; ++d) s += cell[(((size_t)cz[a] * R1 + cy[b]) * R1 + cx[d]) * 8 + c];
        }
        lin[i] += s;
    }
}

int main(int argc, char **argv) {
    const int R = argc > 1 ? atoi(argv[1]) : 256;
    const uint32_t threads = 1u << 24, iters = 16;
    const size_t n = (size_t)R * R * R, ncell = (size_t)(R + 1) * (R + 1) * (R + 1);
    float *lin, *lin2, *cell;
    CK(hipMalloc(&lin, n * 4)); CK(hipMalloc(&lin2, n * 4)); CK(hipMalloc(&cell, ncell * 32));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const uint32_t acts[3] = {65536, 32768, 16384};
    for (int ai = 0; ai < 3; ++ai) {
        const uint32_t act = acts[ai];
        float ms[4] = {0, 0, 0, 0};
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipMemset(lin, 0, n * 4)); CK(hipMemset(lin2, 0, n * 4)); CK(hipMemset(cell, 0, ncell * 32));
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0)); k_scatter<0><<<threads / 256, 256>>>(lin, cell, R, iters, act, 7); CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms[0], e0, e1));
            CK(hipEventRecord(e0)); k_scatter<1><<<threads / 256, 256>>>(lin, cell, R, iters, act, 7); CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms[1], e0, e1));
            CK(hipEventRecord(e0)); k_gather<<<4096, 256>>>(cell, lin2, R); CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms[3], e0, e1));
        }
        // check the transposed scatter + gather against the direct one
        std::vector<float> a(n), b(n);
        CK(hipMemcpy(a.data(), lin, n * 4, hipMemcpyDeviceToHost)); CK(hipMemcpy(b.data(), lin2, n * 4, hipMemcpyDeviceToHost));
        double worst = 0, sa = 0, sb = 0;
        for (size_t i = 0; i < n; ++i) {
            worst = fmax(worst, fabs((double)a[i] - b[i]) / fmax(1e-3, fabs((double)a[i])));
            sa += a[i]; sb += b[i];
        }
        CK(hipMemset(cell, 0, ncell * 32)); CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0)); k_scatter<2><<<threads / 256, 256>>>(lin, cell, R, iters, act, 7); CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms[2], e0, e1));
        const double lookups = (double)threads * iters * act / 65536.0;
        printf("R=%d active=%.2f lookups=%.0fM  direct %.2f ms  corner-transposed %.2f ms  corner-own %.2f ms  gather %.3f ms  "
               "(atomics/s direct %.2fG transposed %.2fG)  check: max rel %.2e sums %.6e %.6e\n",
               R, act / 65536.0, lookups / 1e6, ms[0], ms[1], ms[2], ms[3], 8 * lookups / ms[0] / 1e6, 8 * lookups / ms[1] / 1e6,
               worst, sa, sb);
    }
    return 0;
}
