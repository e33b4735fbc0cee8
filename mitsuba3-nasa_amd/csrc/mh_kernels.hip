// mh_kernels.hip — gfx950 kernels for the `path` / `prb` integrator loop.
//
// Kernels:
//   k_trace<Shadow>     SoA rays -> SoA hits / occlusion (the OptiX slot,
//                       scene_optix.inl:592-721): BVH2 nodes + prim records
//                       staged into LDS, per-lane traversal stack in LDS.
//   k_path              per-lane PathIntegrator::sample (path.cpp:95-287)
//                       incl. camera ray-gen (integrator.cpp:1139-1240);
//                       writes L and sample_pos SoA.
//   k_prb_primal        per-lane PRB primal (prb.py:59-257) for mi.render(prb).
//   k_splat_px          ImageBlock::put, coalesced Gaussian (imageblock.cpp:418-531):
//                       16 lanes per pixel, 5x5x4 partial sums in VGPRs summed
//                       across the DPP row, one global atomic per footprint
//                       texel per pixel.
//   k_splat_generic     ImageBlock::put for every other filter/spp case.
//   k_develop           HDRFilm::develop (hdrfilm.cpp:349-405).
//   k_prb_weights       W image of render_backward (common.py:936-947).
//   k_prb_backward      per-lane dL gather + PRB primal + adjoint replay with
//                       wave/block-reduced gradient atomics (common.py:828-983).
#include <algorithm>

#include "mh_shading.hpp"

namespace mh {
// ===========================================================================
// Kernels
// ===========================================================================
// this wave's contiguous share of n items (the stream engine refills lanes
// from it); wave-uniform
MH_DEV void stream_wave_range(uint64_t n, uint32_t &r0, uint32_t &r1) {
    const uint32_t waves = gridDim.x * (blockDim.x / 64u), w = blockIdx.x * (blockDim.x / 64u) + threadIdx.x / 64u;
    const uint64_t per = (n + waves - 1) / waves;
    r0 = (uint32_t)std::min<uint64_t>(n, (uint64_t)w * per);
    r1 = (uint32_t)std::min<uint64_t>(n, (uint64_t)r0 + per);
}

template <bool InLds>
__global__ void __launch_bounds__(256)
k_trace_closest(DScene S, uint64_t n, const float *__restrict__ rays, float *__restrict__ t_out,
                float *__restrict__ u_out, float *__restrict__ v_out, uint32_t *__restrict__ prim_out,
                uint32_t *__restrict__ shape_out, uint32_t *__restrict__ inst_out) {
    extern __shared__ uint4 lds[];
    LdsBvh B = stage_bvh<InLds>(S, lds);
    // the OptiX payload (scene_optix.inl:602-657, optix/common.h:43-58):
    // prim_index 0 for rectangles (rectangle.cuh:42) and for misses (the
    // payload's initial value; the miss program sets only t and shape),
    // prim_uv (0, 0) on a miss; no instancing: instance = null
    auto load = [&](uint64_t i) {
        RayT r;
        r.o = v3(rays[i], rays[n + i], rays[2 * n + i]);
        r.d = v3(rays[3 * n + i], rays[4 * n + i], rays[5 * n + i]);
        r.maxt = fminf(rays[6 * n + i], kFloatMax);
        return r;
    };
    auto store = [&](uint64_t i, const Hit &h, bool) {
        const bool hit = h.shape != MH_INVALID;
        t_out[i] = h.t;
        u_out[i] = hit ? h.u : 0.f;
        v_out[i] = hit ? h.v : 0.f;
        prim_out[i] = hit && h.prim != MH_INVALID ? h.prim : 0u;
        shape_out[i] = h.shape;
        if (inst_out) inst_out[i] = MH_INVALID;
    };
    if (!InLds && (B.qnodes || B.nodes4)) {
        // a BVH in global memory: the wavefront's per-lane stream engine (the
        // launcher keeps n < 2^32), items in contiguous per-wave ranges
        uint32_t r0, r1;
        stream_wave_range(n, r0, r1);
        trace_stream_any<false>(B, r0, r1, load, store);
        return;
    }
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        Hit h;
        traverse<false>(B.nodes, B.prims, B.stack, B.stride, load(i), h);
        store(i, h, true);
    }
}

template <bool InLds>
__global__ void __launch_bounds__(256)
k_trace_shadow(DScene S, uint64_t n, const float *__restrict__ rays, uint32_t *__restrict__ occ) {
    extern __shared__ uint4 lds[];
    LdsBvh B = stage_bvh<InLds>(S, lds);
    auto load = [&](uint64_t i) {
        RayT r;
        r.o = v3(rays[i], rays[n + i], rays[2 * n + i]);
        r.d = v3(rays[3 * n + i], rays[4 * n + i], rays[5 * n + i]);
        r.maxt = fminf(rays[6 * n + i], kFloatMax);
        return r;
    };
    if (!InLds && (B.qnodes || B.nodes4)) {
        uint32_t r0, r1;
        stream_wave_range(n, r0, r1);
        trace_stream_any<true>(B, r0, r1, load, [&](uint64_t i, const Hit &, bool f) { occ[i] = f ? 1u : 0u; });
        return;
    }
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        Hit h;
        occ[i] = traverse<true>(B.nodes, B.prims, B.stack, B.stride, load(i), h) ? 1u : 0u;
    }
}

// Forward render of one chunk: lane k in [0, n) -> samples of every pass.
// out planes (each `plane` floats apart): Lr, Lg, Lb, posx, posy; sample
// (k, pass) stored at pass * n + k.
// Kind: MH_INTEGRATOR_PATH / MH_INTEGRATOR_PRB (primal) / MH_INTEGRATOR_VOLPATH /
// MH_INTEGRATOR_PRBVOLPATH (primal)
#ifndef MH_VOL_WAVES
#define MH_VOL_WAVES 4  // volpath: 128 VGPRs (+ some scratch) measured +10 % over 2 waves (tools/exp_volwaves.sh)
#endif
template <int Kind, bool InLds>
__global__ void __launch_bounds__(256, (Kind == MH_INTEGRATOR_VOLPATH || Kind == MH_INTEGRATOR_PRBVOLPATH) ? MH_VOL_WAVES : 1)
k_render(DScene S, IntegratorParams in, LaneMap lm, uint32_t seed_value, uint32_t n_passes,
         uint64_t n, uint64_t plane, float *__restrict__ out, unsigned long long *__restrict__ counters,
         int alpha) {
    extern __shared__ uint4 lds[];
    LdsBvh B = stage_bvh<InLds>(S, lds);
    uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t n_closest = 0, n_shadow = 0;
    if (k < n) {
        uint32_t lane, px, py;
        lane_of(lm, k, lane, px, py);
        Pcg rng;
        rng.seed(seed_value, lane);
        const float sw = S.inv_width, sh = S.inv_height;
        for (uint32_t pass = 0; pass < n_passes; ++pass) {
            float jx = rng.next_float(), jy = rng.next_float();
            float sx = (float)px + jx, sy = (float)py + jy;
            RayT r = camera_ray(S, __builtin_fmaf(sx, sw, -0.f), __builtin_fmaf(sy, sh, -0.f));
            V3 L;
            bool valid = false;
            if (Kind == MH_INTEGRATOR_PRB)
                L = prb_sample<false>(S, B, in, rng, r, v3(0, 0, 0), v3(0, 0, 0), nullptr, n_closest, n_shadow,
                                      &valid);
            else if (Kind == MH_INTEGRATOR_VOLPATH)
                L = volpath_sample(S, B, in, rng, r, n_closest, n_shadow, &valid);
            else if (Kind == MH_INTEGRATOR_PRBVOLPATH)
                L = prbvol_sample<0>(S, B, in, rng, r, v3(0, 0, 0), v3(0, 0, 0), nullptr, n_closest, n_shadow,
                                         &valid);
            else
                L = path_sample(S, B, in, rng, r, n_closest, n_shadow, &valid);
            uint64_t o = (uint64_t)pass * n + k;
            out[o] = L.x;
            out[plane + o] = L.y;
            out[2 * plane + o] = L.z;
            out[3 * plane + o] = sx;
            out[4 * plane + o] = sy;
            if (alpha) out[5 * plane + o] = valid ? 1.f : 0.f;  // aovs[3] (integrator.cpp:1229-1231)
        }
    }
    if (counters) {
        wave_count(&counters[0], n_closest);
        wave_count(&counters[1], n_shadow);
    }
}

// ---------------------------------------------------------------------------
// Splat: one lane per pixel, coalesced Gaussian footprint (count = 5)
// ---------------------------------------------------------------------------
MH_DEV void splat_one_atomic(const DScene &S, float *film, float px, float py, const float *vals,
                             int nch, int ch0) {
    const uint32_t W = S.width, H = S.height;
    int32_t pix = (int32_t)floorf(px) - 2, piy = (int32_t)floorf(py) - 2;
    uint32_t x = (uint32_t)pix, y = (uint32_t)piy;
    float relx = ((float)pix + 0.5f) - px, rely = ((float)piy + 0.5f) - py;
    for (int ys = 0; ys < 5; ++ys) {
        float wy = gaussian_eval(S.filter_coeff, rely + (float)ys);
        for (int xs = 0; xs < 5; ++xs) {
            float wx = gaussian_eval(S.filter_coeff, relx + (float)xs);
            float w = wx * wy;
            if ((y + ys) < H && (x + xs) < W) {
                float *p = film + ((uint64_t)(y + ys) * W + (x + xs)) * 4;
                for (int c = 0; c < nch; ++c) atomicAdd(p + ch0 + c, vals[c] * w);
            }
        }
    }
}

// Mode 0: RGBW film from stored (L, pos); mode 1: W-only image from the RNG
// jitter (PRB weights; film has 1 channel); mode 2: the alpha channel of an
// rgba / ya / xyza film from the stored (alpha, pos) (1 channel).
//
// kSplatLanes (16) lanes share a pixel: lane g of the group takes samples
// g, g + 16, ... (16 consecutive floats per plane read: one 64-B segment),
// and the 16 partial footprints are summed across the DPP row before one
// lane issues the footprint's atomics.  (A lane per pixel left a chunk of
// 32k pixels at 512 waves for 1024 SIMDs, each walking 256 samples alone.)
constexpr uint32_t kSplatLanes = 16;

// sum over the 16 lanes of a DPP row; every lane of the row gets the total
MH_DEV float row16_sum(float x) {
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x141, 0xF, 0xF, false));  // row_half_mirror
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x140, 0xF, 0xF, false));  // row_mirror
    return x;
}

// ImageBlock::put's sample check (imageblock.cpp:180-204: warn_negative
// `v >= -1e-5`, warn_invalid `isfinite(v)`), counted instead of logged
MH_DEV bool sample_invalid(const float *v) {
    bool bad = false;
#pragma unroll
    for (int c = 0; c < 3; ++c) bad = bad || !(v[c] >= -1e-5f) || !isfinite(v[c]);
    return bad;
}

template <int Mode>
__global__ void __launch_bounds__(128)
k_splat_px(DScene S, uint32_t pixel_begin, uint32_t n_pix, uint32_t Sn, uint32_t n_passes,
           uint64_t n, uint64_t plane, const float *__restrict__ in, float *__restrict__ film,
           uint32_t seed_value, uint32_t spp_pp, uint32_t s_begin, unsigned long long *__restrict__ invalid,
           uint64_t in_lim, unsigned long long *__restrict__ viol) {
    uint32_t n_bad = 0;
    const uint32_t gl = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t pl = gl / kSplatLanes, g = gl % kSplatLanes;
    if (pl >= n_pix) return;  // whole DPP rows leave together (n_pix granularity = 16 lanes)
    // bounds guard (the host checks the same contract per launch): the last
    // float this pixel's row reads must lie inside the in planes; a row that
    // would read past them counts a violation and leaves whole
    if (Mode != 1) {
        const uint64_t last = (uint64_t)(n_passes - 1) * n + (uint64_t)(pl + 1) * Sn - 1 + (Mode == 2 ? 5 : 4) * plane;
        if (last >= in_lim) {
            if (g == 0) atomicAdd(viol, 1ull);
            return;
        }
    }
    const uint32_t W = S.width, H = S.height;
    const uint32_t pixel = pixel_begin + pl;
    const uint32_t py = pixel / W, px = pixel - py * W;
    float acc[5][5][4];
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
        for (int j = 0; j < 5; ++j)
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[i][j][c] = 0.f;
    for (uint32_t pass = 0; pass < n_passes; ++pass) {
        // Mode 0: the next sample's five floats are in flight while this one
        // is weighted (one wave has the SIMD to itself at this VGPR count)
        const float *src = in + (uint64_t)pass * n + (uint64_t)pl * Sn;
        float nv[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
        if (Mode == 0 && g < Sn) {
#pragma unroll
            for (int c = 0; c < 5; ++c) nv[c] = src[c * plane + g];
        }
        if (Mode == 2 && g < Sn) {
            nv[0] = src[5 * plane + g];
            nv[3] = src[3 * plane + g];
            nv[4] = src[4 * plane + g];
        }
        for (uint32_t j = g; j < Sn; j += kSplatLanes) {
            float sx, sy, vals[4];
            if (Mode == 0) {
                vals[0] = nv[0];
                vals[1] = nv[1];
                vals[2] = nv[2];
                vals[3] = 1.f;
                sx = nv[3];
                sy = nv[4];
                n_bad += sample_invalid(vals) ? 1u : 0u;
                const uint32_t jn = j + kSplatLanes;
                if (jn < Sn) {
#pragma unroll
                    for (int c = 0; c < 5; ++c) nv[c] = src[c * plane + jn];
                }
            } else if (Mode == 2) {
                vals[0] = vals[1] = vals[2] = 0.f;
                vals[3] = nv[0];
                sx = nv[3];
                sy = nv[4];
                const uint32_t jn = j + kSplatLanes;
                if (jn < Sn) {
                    nv[0] = src[5 * plane + jn];
                    nv[3] = src[3 * plane + jn];
                    nv[4] = src[4 * plane + jn];
                }
            } else {
                Pcg rng;
                rng.seed(seed_value, pixel * spp_pp + s_begin + j);
                sx = (float)px + rng.next_float();
                sy = (float)py + rng.next_float();
                vals[0] = vals[1] = vals[2] = 0.f;
                vals[3] = 1.f;
            }
            int32_t fx = (int32_t)floorf(sx), fy = (int32_t)floorf(sy);
            if (fx != (int32_t)px || fy != (int32_t)py) {  // jitter rounded onto the next pixel
                if (Mode == 0) splat_one_atomic(S, film, sx, sy, vals, 4, 0);
                else {
                    const float one = vals[3];  // 1 (W image) or the sample's alpha
                    // 1-channel film (W image / alpha): the footprint of one sample
                    const uint32_t Wd = S.width, Hd = S.height;
                    int32_t pix = fx - 2, piy = fy - 2;
                    float relx = ((float)pix + 0.5f) - sx, rely = ((float)piy + 0.5f) - sy;
                    for (int ys = 0; ys < 5; ++ys) {
                        float wy = gaussian_eval(S.filter_coeff, rely + (float)ys);
                        for (int xs = 0; xs < 5; ++xs) {
                            float wx = gaussian_eval(S.filter_coeff, relx + (float)xs);
                            uint32_t xx = (uint32_t)(pix + xs), yy = (uint32_t)(piy + ys);
                            if (xx < Wd && yy < Hd) atomicAdd(film + (uint64_t)yy * Wd + xx, one * (wx * wy));
                        }
                    }
                }
                continue;
            }
            float relx = ((float)(fx - 2) + 0.5f) - sx, rely = ((float)(fy - 2) + 0.5f) - sy;
            float wx[5], wy[5];
#pragma unroll
            for (int i = 0; i < 5; ++i) {
                wx[i] = gaussian_eval(S.filter_coeff, relx + (float)i);
                wy[i] = gaussian_eval(S.filter_coeff, rely + (float)i);
            }
#pragma unroll
            for (int ys = 0; ys < 5; ++ys)
#pragma unroll
                for (int xs = 0; xs < 5; ++xs) {
                    float w = wx[xs] * wy[ys];
                    if (Mode == 0) {
#pragma unroll
                        for (int c = 0; c < 4; ++c) acc[ys][xs][c] += vals[c] * w;
                    } else {
                        acc[ys][xs][3] += vals[3] * w;
                    }
                }
        }
    }
    if (Mode == 0 && invalid && n_bad) atomicAdd(invalid, (unsigned long long)n_bad);  // rare: no reduction
#pragma unroll
    for (int ys = 0; ys < 5; ++ys)
#pragma unroll
        for (int xs = 0; xs < 5; ++xs)
#pragma unroll
            for (int c = (Mode == 0 ? 0 : 3); c < 4; ++c) acc[ys][xs][c] = row16_sum(acc[ys][xs][c]);
    if (g != 0) return;
#pragma unroll
    for (int ys = 0; ys < 5; ++ys) {
        uint32_t yy = py - 2 + ys;
        if (yy >= H) continue;
#pragma unroll
        for (int xs = 0; xs < 5; ++xs) {
            uint32_t xx = px - 2 + xs;
            if (xx >= W) continue;
            if (Mode == 0) {
                float *p = film + ((uint64_t)yy * W + xx) * 4;
#pragma unroll
                for (int c = 0; c < 4; ++c) atomicAdd(p + c, acc[ys][xs][c]);
            } else {
                atomicAdd(film + (uint64_t)yy * W + xx, acc[ys][xs][3]);
            }
        }
    }
}

// The film splat (mode 0) on 4 x 4 tiles of source pixels: a 256-thread
// workgroup is 16 pixel rows of kSplatLanes lanes, as in k_splat_px, but the
// rows' footprint sums go to the tile's 8 x 8 film block in LDS (ds_add_f64)
// and the block is added to the film once, coalesced: 256 lanes, one float
// each, film rows of 8 pixels x 4 channels contiguous.  k_splat_px issues
// 100 memory-side atomics per source pixel from 4 lanes of a wave; this
// issues 16 (the film's halo pixels still receive up to four tiles' adds).
// Same values and filter as k_splat_px; only the float summation order
// differs (as between any two atomic runs).
#ifndef MH_SPLAT_TILE
#define MH_SPLAT_TILE 1
#endif
constexpr uint32_t kSplatTile = 4;                    // source pixels per tile side
constexpr uint32_t kSplatTileFilm = kSplatTile + 4;   // film pixels per tile side (the 5 x 5 footprint)
// Mode 0: the RGBW film from the stored (L, pos); Mode 1: the W image of the
// PRB weights, its jitter regenerated from the RNG as k_splat_px<1> does
// (1 channel; round 5: 25 memory-side atomics per source pixel from 4 lanes
// of a wave were 0.44 ms of the bench step)
template <int Mode>
__global__ void __launch_bounds__(256)
k_splat_tile(DScene S, uint32_t pixel_begin, uint32_t n_pix, uint32_t row_first, uint32_t tiles_x, uint32_t Sn,
             uint32_t n_passes, uint64_t n, uint64_t plane, const float *__restrict__ in, float *__restrict__ film,
             unsigned long long *__restrict__ invalid, uint64_t in_lim, unsigned long long *__restrict__ viol,
             uint32_t seed_value, uint32_t spp_pp, uint32_t s_begin) {
    constexpr uint32_t NC = Mode == 0 ? 4u : 1u, kTileN = kSplatTileFilm * kSplatTileFilm * NC;
    // double: ds_add_f64 runs ~7x the rate of ds_add_f32 on gfx950 (LdsDouble)
    __shared__ double tile[kTileN];
    const uint32_t W = S.width, H = S.height;
    const uint32_t tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x;
    const uint32_t grp = threadIdx.x / kSplatLanes, g = threadIdx.x % kSplatLanes;
    const uint32_t ti = grp % kSplatTile, tj = grp / kSplatTile;
    const uint32_t px = tx * kSplatTile + ti, py = row_first + ty * kSplatTile + tj;
    for (uint32_t e = threadIdx.x; e < kTileN; e += 256) tile[e] = 0.0;
    const uint32_t pixel = py * W + px;
    bool live = px < W && py < H && pixel >= pixel_begin && pixel - pixel_begin < n_pix;
    const uint32_t pl = pixel - pixel_begin;
    if (Mode == 0 && live) {  // the bounds guard of k_splat_px: a row that would read past the planes leaves whole
        const uint64_t last = (uint64_t)(n_passes - 1) * n + (uint64_t)(pl + 1) * Sn - 1 + 4 * plane;
        if (last >= in_lim) {
            if (g == 0) atomicAdd(viol, 1ull);
            live = false;
        }
    }
    __syncthreads();
    uint32_t n_bad = 0;
    float acc[5][5][NC];
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
        for (int j = 0; j < 5; ++j)
#pragma unroll
            for (uint32_t c = 0; c < NC; ++c) acc[i][j][c] = 0.f;
    if (live) {
        for (uint32_t pass = 0; pass < n_passes; ++pass) {
            const float *src = in + (uint64_t)pass * n + (uint64_t)pl * Sn;
            float nv[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
            if (Mode == 0 && g < Sn) {
#pragma unroll
                for (int c = 0; c < 5; ++c) nv[c] = src[c * plane + g];
            }
            for (uint32_t j = g; j < Sn; j += kSplatLanes) {
                float vals[4] = {nv[0], nv[1], nv[2], 1.f};
                float sx = nv[3], sy = nv[4];
                if (Mode == 0) {
                    n_bad += sample_invalid(vals) ? 1u : 0u;
                    const uint32_t jn = j + kSplatLanes;
                    if (jn < Sn) {
#pragma unroll
                        for (int c = 0; c < 5; ++c) nv[c] = src[c * plane + jn];
                    }
                } else {
                    Pcg rng;
                    rng.seed(seed_value, pixel * spp_pp + s_begin + j);
                    sx = (float)px + rng.next_float();
                    sy = (float)py + rng.next_float();
                }
                const int32_t fx = (int32_t)floorf(sx), fy = (int32_t)floorf(sy);
                if (fx != (int32_t)px || fy != (int32_t)py) {  // jitter rounded onto the next pixel
                    if (Mode == 0) {
                        splat_one_atomic(S, film, sx, sy, vals, 4, 0);
                    } else {
                        const int32_t pix = fx - 2, piy = fy - 2;
                        const float relx = ((float)pix + 0.5f) - sx, rely = ((float)piy + 0.5f) - sy;
                        for (int ys = 0; ys < 5; ++ys) {
                            const float wy = gaussian_eval(S.filter_coeff, rely + (float)ys);
                            for (int xs = 0; xs < 5; ++xs) {
                                const float wx = gaussian_eval(S.filter_coeff, relx + (float)xs);
                                const uint32_t xx = (uint32_t)(pix + xs), yy = (uint32_t)(piy + ys);
                                if (xx < W && yy < H) atomicAdd(film + (uint64_t)yy * W + xx, 1.f * (wx * wy));
                            }
                        }
                    }
                    continue;
                }
                const float relx = ((float)(fx - 2) + 0.5f) - sx, rely = ((float)(fy - 2) + 0.5f) - sy;
                // the 10 filter weights on packed f32 pairs (gaussian_eval2:
                // bit-identical to gaussian_eval, half the instructions)
                const F2 wa = gaussian_eval2(S.filter_coeff, pair(relx + 0.f, relx + 1.f)),
                         wb = gaussian_eval2(S.filter_coeff, pair(relx + 2.f, relx + 3.f)),
                         wc = gaussian_eval2(S.filter_coeff, pair(relx + 4.f, rely + 0.f)),
                         wd = gaussian_eval2(S.filter_coeff, pair(rely + 1.f, rely + 2.f)),
                         we = gaussian_eval2(S.filter_coeff, pair(rely + 3.f, rely + 4.f));
                const float wx[5] = {wa.x, wa.y, wb.x, wb.y, wc.x}, wy[5] = {wc.y, wd.x, wd.y, we.x, we.y};
#pragma unroll
                for (int ys = 0; ys < 5; ++ys)
#pragma unroll
                    for (int xs = 0; xs < 5; ++xs) {
                        const float w = wx[xs] * wy[ys];
                        if (Mode == 0) {
#pragma unroll
                            for (int c = 0; c < 4; ++c) acc[ys][xs][c] += vals[c] * w;
                        } else {
                            acc[ys][xs][0] += 1.f * w;
                        }
                    }
            }
        }
    }
    if (Mode == 0 && invalid && n_bad) atomicAdd(invalid, (unsigned long long)n_bad);  // rare: no reduction
#pragma unroll
    for (int ys = 0; ys < 5; ++ys)
#pragma unroll
        for (int xs = 0; xs < 5; ++xs)
#pragma unroll
            for (uint32_t c = 0; c < NC; ++c) acc[ys][xs][c] = row16_sum(acc[ys][xs][c]);
    if (live && g == 0) {
#pragma unroll
        for (int ys = 0; ys < 5; ++ys)
#pragma unroll
            for (int xs = 0; xs < 5; ++xs)
#pragma unroll
                for (uint32_t c = 0; c < NC; ++c)
                    __hip_atomic_fetch_add((LdsDouble *)&tile[((tj + ys) * kSplatTileFilm + (ti + xs)) * NC + c],
                                           (double)acc[ys][xs][c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __syncthreads();
    // the film block: element e = (row, column, channel) of the tile's 8 x 8 x NC
    const int32_t ox = (int32_t)(tx * kSplatTile) - 2, oy = (int32_t)(row_first + ty * kSplatTile) - 2;
    for (uint32_t e = threadIdx.x; e < kTileN; e += 256) {
        const float v = (float)tile[e];
        const int32_t x = ox + (int32_t)((e / NC) % kSplatTileFilm), y = oy + (int32_t)((e / NC) / kSplatTileFilm);
        if (v != 0.f && x >= 0 && y >= 0 && (uint32_t)x < W && (uint32_t)y < H)
            atomicAdd(film + ((uint64_t)y * W + (uint32_t)x) * NC + (e % NC), v);
    }
}

// sample check of a chunk's (L, pos) planes for the deterministic splat
__global__ void k_count_invalid(uint64_t total, uint64_t n, uint64_t plane, const float *__restrict__ in,
                                unsigned long long *__restrict__ invalid) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const float v[3] = {in[i], in[plane + i], in[2 * plane + i]};  // sample (k, pass) at pass * n + k
    if (sample_invalid(v)) atomicAdd(invalid, 1ull);
}

// Deterministic splat (MH_FLAG_DETERMINISTIC / MH_DETERMINISTIC=1; the
// ordered-reduction build of SURVEY.md §5): every film pixel of the rows a
// chunk can reach gathers, in a fixed order (source row, source column,
// pass, sample), the weighted values of the chunk's samples whose coalesced
// footprint covers it, and adds the sum once.  A sample's footprint starts at
// floor(pos) - 2 and floor(pos) is its pixel or, when the jitter rounds up,
// the next one, so the sources of pixel o are the pixels o - 3 .. o + 2.
// Each contribution is the scatter's own `value * (wx * wy)`; only the
// summation order differs from k_splat_px, and it no longer depends on
// scheduling, so the film is bit-reproducible from run to run.
template <int Mode>
__global__ void __launch_bounds__(256)
k_splat_gather(DScene S, uint32_t pixel_begin, uint32_t n_pix, uint32_t row0, uint32_t n_rows, uint32_t Sn,
               uint32_t n_passes, uint64_t n, uint64_t plane, const float *__restrict__ in,
               float *__restrict__ film, uint32_t seed_value, uint32_t spp_pp, uint32_t s_begin) {
    const uint32_t W = S.width, H = S.height;
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint64_t)n_rows * W) return;
    const int32_t oy = (int32_t)(row0 + t / W), ox = (int32_t)(t % W);
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int32_t qy = oy - 3; qy <= oy + 2; ++qy) {
        if (qy < 0 || qy >= (int32_t)H) continue;
        for (int32_t qx = ox - 3; qx <= ox + 2; ++qx) {
            if (qx < 0 || qx >= (int32_t)W) continue;
            const uint32_t q = (uint32_t)qy * W + (uint32_t)qx;
            if (q < pixel_begin || q - pixel_begin >= n_pix) continue;
            const uint32_t pl = q - pixel_begin;
            for (uint32_t pass = 0; pass < n_passes; ++pass) {
                const float *src = in + (uint64_t)pass * n + (uint64_t)pl * Sn;
                for (uint32_t j = 0; j < Sn; ++j) {
                    float sx, sy, vals[4];
                    if (Mode == 1) {
                        Pcg rng;
                        rng.seed(seed_value, q * spp_pp + s_begin + j);
                        sx = (float)qx + rng.next_float();
                        sy = (float)qy + rng.next_float();
                        vals[0] = vals[1] = vals[2] = 0.f;
                        vals[3] = 1.f;
                    } else {
                        sx = src[3 * plane + j];
                        sy = src[4 * plane + j];
                        if (Mode == 0) {
                            vals[0] = src[j]; vals[1] = src[plane + j]; vals[2] = src[2 * plane + j]; vals[3] = 1.f;
                        } else {
                            vals[0] = vals[1] = vals[2] = 0.f;
                            vals[3] = src[5 * plane + j];
                        }
                    }
                    const int32_t p0x = (int32_t)floorf(sx) - 2, p0y = (int32_t)floorf(sy) - 2;
                    const int32_t dx = ox - p0x, dy = oy - p0y;
                    if (dx < 0 || dx > 4 || dy < 0 || dy > 4) continue;
                    const float relx = ((float)p0x + 0.5f) - sx, rely = ((float)p0y + 0.5f) - sy;
                    const float w = gaussian_eval(S.filter_coeff, relx + (float)dx) *
                                    gaussian_eval(S.filter_coeff, rely + (float)dy);
                    if (Mode == 0) {
#pragma unroll
                        for (int c = 0; c < 4; ++c) acc[c] += vals[c] * w;
                    } else {
                        acc[3] += vals[3] * w;
                    }
                }
            }
        }
    }
    const uint64_t o = (uint64_t)oy * W + (uint32_t)ox;
    if (Mode == 0) {
        float4 *f = reinterpret_cast<float4 *>(film) + o;
        float4 v = *f;
        v.x += acc[0]; v.y += acc[1]; v.z += acc[2]; v.w += acc[3];
        *f = v;
    } else {
        film[o] += acc[3];
    }
}

// Generic per-sample splat (box filter / non-coalesced spp < 4 / other radii)
// — ImageBlock::put (imageblock.cpp:210-233, 264-409, 418-531)
template <int Mode>
__global__ void __launch_bounds__(256)
k_splat_generic(DScene S, LaneMap lm, uint32_t n_passes, uint64_t n, uint64_t plane,
                const float *__restrict__ in, float *__restrict__ film, uint32_t seed_value,
                int coalesce, unsigned long long *__restrict__ invalid) {
    uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint32_t W = S.width, H = S.height;
    const int nch = Mode == 0 ? 4 : 1;
    uint32_t lane, pxi, pyi;
    lane_of(lm, k, lane, pxi, pyi);
    Pcg rng;
    if (Mode == 1) rng.seed(seed_value, lane);
    for (uint32_t pass = 0; pass < n_passes; ++pass) {
        float vals[4], px, py;
        if (Mode == 0) {
            uint64_t o = (uint64_t)pass * n + k;
            vals[0] = in[o]; vals[1] = in[plane + o]; vals[2] = in[2 * plane + o]; vals[3] = 1.f;
            px = in[3 * plane + o]; py = in[4 * plane + o];
            if (invalid && sample_invalid(vals)) atomicAdd(invalid, 1ull);
        } else if (Mode == 2) {
            uint64_t o = (uint64_t)pass * n + k;
            vals[0] = in[5 * plane + o];
            px = in[3 * plane + o]; py = in[4 * plane + o];
        } else {
            px = (float)pxi + rng.next_float();
            py = (float)pyi + rng.next_float();
            vals[0] = 1.f;
        }
        auto add = [&](uint32_t xx, uint32_t yy, float w) {
            if (Mode == 0) {
                float *p = film + ((uint64_t)yy * W + xx) * 4;
                for (int c = 0; c < 4; ++c) atomicAdd(p + c, vals[c] * w);
            } else {
                atomicAdd(film + (uint64_t)yy * W + xx, vals[0] * w);
            }
        };
        if (S.rfilter == MH_RFILTER_BOX) {
            uint32_t ux = (uint32_t)(int32_t)floorf(px), uy = (uint32_t)(int32_t)floorf(py);
            if (ux < W && uy < H) add(ux, uy, 1.f);
            continue;
        }
        const float radius = S.rfilter_radius;
        if (coalesce) {
            int32_t nn = (int32_t)ceilf(radius - 0.5f), count = 2 * nn + 1;
            int32_t pix = (int32_t)floorf(px) - nn, piy = (int32_t)floorf(py) - nn;
            float relx = ((float)pix + 0.5f) - px, rely = ((float)piy + 0.5f) - py;
            for (int32_t ys = 0; ys < count; ++ys) {
                float wy = gaussian_eval(S.filter_coeff, rely + (float)ys);
                for (int32_t xs = 0; xs < count; ++xs) {
                    float wx = gaussian_eval(S.filter_coeff, relx + (float)xs);
                    uint32_t xx = (uint32_t)(pix + xs), yy = (uint32_t)(piy + ys);
                    if (xx < W && yy < H) add(xx, yy, wx * wy);
                }
            }
        } else {
            float pfx = px - 0.5f, pfy = py - 0.5f;
            int32_t a0x = max((int32_t)ceilf(pfx - radius), 0), a0y = max((int32_t)ceilf(pfy - radius), 0);
            int32_t a1x = min((int32_t)floorf(pfx + radius), (int32_t)W - 1);
            int32_t a1y = min((int32_t)floorf(pfy + radius), (int32_t)H - 1);
            if (!(a0x <= a1x && a0y <= a1y)) continue;
            uint32_t count = (uint32_t)ceilf(2.f * radius);
            float relx = (float)a0x - pfx, rely = (float)a0y - pfy;
            for (uint32_t ys = 0; ys < count; ++ys) {
                float wy = gaussian_eval(S.filter_coeff, rely + (float)ys);
                for (uint32_t xs = 0; xs < count; ++xs) {
                    float wx = gaussian_eval(S.filter_coeff, relx + (float)xs);
                    if ((int32_t)(a0x + xs) <= a1x && (int32_t)(a0y + ys) <= a1y)
                        add((uint32_t)a0x + xs, (uint32_t)a0y + ys, wx * wy);
                }
            }
        }
    }
    (void)nch;
}

// adjoint of develop: grad_in / (W == 0 ? 1 : W), once per pixel (the
// division Dr.Jit's AD of `rgb / W` performs); gathered per sample by gather_dL
__global__ void k_grad_over_w(uint64_t n_px, const float *__restrict__ grad_in, const float *__restrict__ w,
                              float *__restrict__ out) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_px) return;
    const float Wp = w[i] == 0.f ? 1.f : w[i];
    // float4 per pixel: gather_dL reads a footprint texel with one load
    reinterpret_cast<float4 *>(out)[i] =
        make_float4(grad_in[3 * i] / Wp, grad_in[3 * i + 1] / Wp, grad_in[3 * i + 2] / Wp, 0.f);
}

// HDRFilm::develop (films/hdrfilm.cpp:349-405): rgb / w, or luminance(rgb) / w
// (spectrum.h:431-434), or srgb_to_xyz(rgb) / w (spectrum.h:396-402, matrix
// product as column fmadds); with alpha (rgba / ya / xyza) the film holds
// R G B A W and the image gets the alpha channel after the colour channels
template <int Fmt, bool Alpha>
__global__ void k_develop(uint64_t n_px, const float *__restrict__ film, float *__restrict__ out) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_px) return;
    float4 v;
    float al = 0.f;
    if (Alpha) {
        const float *f = film + 5 * i;
        v = make_float4(f[0], f[1], f[2], f[4]);
        al = f[3];
    } else {
        v = reinterpret_cast<const float4 *>(film)[i];
    }
    float d = v.w == 0.f ? 1.f : v.w;
    if (Fmt == MH_PIXEL_Y) {
        out[(Alpha ? 2 : 1) * i] = ((v.x * 0.212671f + v.y * 0.715160f) + v.z * 0.072169f) / d;
        if (Alpha) out[2 * i + 1] = al / d;
        return;
    }
    float a = v.x, b = v.y, c = v.z;
    if (Fmt == MH_PIXEL_XYZ) {
        a = __builtin_fmaf(0.180423f, v.z, __builtin_fmaf(0.357580f, v.y, 0.412453f * v.x));
        b = __builtin_fmaf(0.072169f, v.z, __builtin_fmaf(0.715160f, v.y, 0.212671f * v.x));
        c = __builtin_fmaf(0.950227f, v.z, __builtin_fmaf(0.119193f, v.y, 0.019334f * v.x));
    }
    const uint32_t ch = Alpha ? 4 : 3;
    out[ch * i] = a / d;
    out[ch * i + 1] = b / d;
    out[ch * i + 2] = c / d;
    if (Alpha) out[4 * i + 3] = al / d;
}

// ---------------------------------------------------------------------------
// render_forward (common.py:696-826): per sample the tangent radiance dL,
// written to the (L, pos, alpha) planes of k_render for the film splat.
// prb: prb_forward, one traversal.  prbvolpath: the reference's primal +
// forward-mode replay, the replay run once per colour channel c with dL = e_c
// through the adjoint sinks in forward mode (GradCtx::fwd), whose
// <adj, tangent> sum is then dL_c (the medium's sigma_t adjoint mixes the
// channels, so one replay cannot give all three)
// ---------------------------------------------------------------------------
template <bool Vol, bool InLds>
__global__ void __launch_bounds__(256, Vol ? MH_VOL_WAVES : 1)
k_render_forward(DScene S, IntegratorParams in, LaneMap lm, uint32_t seed_value, uint64_t n, uint64_t plane,
                 float *__restrict__ out, GradArgs ga, unsigned long long *__restrict__ counters, int alpha) {
    extern __shared__ uint4 lds[];
    LdsBvh B = stage_bvh<InLds>(S, lds);
    GradCtx g = make_grad_ctx(ga);
    g.fwd = true;
    uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t n_closest = 0, n_shadow = 0;
    if (k < n) {
        uint32_t lane, px, py;
        lane_of(lm, k, lane, px, py);
        Pcg rng;
        rng.seed(seed_value, lane);
        const float sx = (float)px + rng.next_float(), sy = (float)py + rng.next_float();
        RayT r = camera_ray(S, __builtin_fmaf(sx, S.inv_width, -0.f),
                            __builtin_fmaf(sy, S.inv_height, -0.f));
        V3 dL;
        bool valid = false;
        if (Vol) {
            Pcg rng_primal = rng;  // sampler.clone()
            const V3 Lp = prbvol_sample<0>(S, B, in, rng_primal, r, v3(0, 0, 0), v3(0, 0, 0), nullptr, n_closest,
                                           n_shadow, &valid);
            float d[3];
#pragma unroll 1
            for (int c = 0; c < 3; ++c) {
                Pcg rc = rng;
                g.fsum = 0.f;
                prbvol_sample<1>(S, B, in, rc, r, v3(c == 0 ? 1.f : 0.f, c == 1 ? 1.f : 0.f, c == 2 ? 1.f : 0.f), Lp,
                                 &g, n_closest, n_shadow);
                d[c] = g.fsum;
            }
            dL = v3(d[0], d[1], d[2]);
        } else {
            dL = prb_forward(S, B, in, rng, r, g, n_closest, n_shadow, &valid);
        }
        out[k] = dL.x;
        out[plane + k] = dL.y;
        out[2 * plane + k] = dL.z;
        out[3 * plane + k] = sx;
        out[4 * plane + k] = sy;
        if (alpha) out[5 * plane + k] = valid ? 1.f : 0.f;  // common.py:803-804
    }
    if (counters) {
        wave_count(&counters[0], n_closest);
        wave_count(&counters[1], n_shadow);
    }
}

// ---------------------------------------------------------------------------
// PRB backward: dL gather + primal + adjoint per lane (common.py:900-983)
// ---------------------------------------------------------------------------
#ifndef MH_PRB_WAVES
#define MH_PRB_WAVES 4  // replay backward: 128 VGPRs (4 waves/SIMD, ~28 spilled) measured faster than 3 waves
#endif
template <bool InLds, bool Fused>
__global__ void __launch_bounds__(256, Fused ? 1 : MH_PRB_WAVES)
k_prb_backward(DScene S, IntegratorParams in, LaneMap lm, uint32_t seed_value, uint64_t n,
               int coalesce, const float *__restrict__ grad_in, const float *__restrict__ weights,
               GradArgs ga, unsigned long long *__restrict__ counters) {
    extern __shared__ uint4 lds[];
    LdsBvh B = stage_bvh<InLds>(S, lds);
    GradCtx g = make_grad_ctx(ga);
    // one bitmap parameter small enough for LDS: texel gradients accumulate per
    // workgroup (after the BVH staging region) and are flushed once at the end;
    // the grid is then persistent (grid-stride over the samples)
    float *tex_acc = nullptr;
    if (!Fused && ga.lds_slot >= 0) {
        tex_acc = reinterpret_cast<float *>(reinterpret_cast<uint8_t *>(lds) + ga.lds_offset);
        for (uint32_t i = threadIdx.x; i < ga.lds_floats; i += blockDim.x) tex_acc[i] = 0.f;
        __syncthreads();
        g.lds_slot = ga.lds_slot;
        g.lds_acc = tex_acc;
        g.lds_floats = ga.lds_floats;
    }
    uint32_t n_closest = 0, n_shadow = 0;
    const uint64_t stride = tex_acc ? (uint64_t)gridDim.x * blockDim.x : n;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += stride) {
        uint32_t lane, px, py;
        lane_of(lm, k, lane, px, py);
        Pcg rng;
        rng.seed(seed_value, lane);
        float sx = (float)px + rng.next_float(), sy = (float)py + rng.next_float();
        RayT r = camera_ray(S, __builtin_fmaf(sx, S.inv_width, -0.f),
                            __builtin_fmaf(sy, S.inv_height, -0.f));
        V3 dL = gather_dL_wave(S, coalesce, grad_in, sx, sy);  // grad_in: pre-divided by W (k_grad_over_w)
        if (Fused) {
            prb_fused(S, B, in, rng, r, dL, ga.n_rgb, g, n_closest, n_shadow);
        } else {
            Pcg rng_primal = rng;  // sampler.clone()
            V3 Lp = prb_sample<false>(S, B, in, rng_primal, r, v3(0, 0, 0), v3(0, 0, 0), nullptr,
                                      n_closest, n_shadow);
            prb_sample<true>(S, B, in, rng, r, dL, Lp, &g, n_closest, n_shadow);
        }
    }
    if (tex_acc) {
        __syncthreads();
        float *dst = ga.bufs[ga.lds_slot];
        for (uint32_t i = threadIdx.x; i < ga.lds_floats; i += blockDim.x)
            if (tex_acc[i] != 0.f) gatomic_add(dst + i, tex_acc[i]);
    }
    flush_small_slots(g, ga);
    if (counters) {
        wave_count(&counters[0], n_closest);
        wave_count(&counters[1], n_shadow);
    }
}

// prbvolpath backward: dL gather + primal + adjoint replay per lane
// (RBIntegrator.render_backward, common.py:900-983, with prbvolpath.sample)
// PvpWork: a persistent grid (one NEE log region per thread) pulling
// 64-sample batches per wave from an atomic head; log == nullptr: one thread
// per sample, adjoint NEE walks replayed
struct PvpWork {
    float4 *log;                  // [cap][threads] NeeLog entries
    uint32_t cap;
    unsigned long long *head;     // work counter (zeroed by the launcher)
    float4 *main;                 // [4 main_cap][threads] MainLog entries (nullptr: primal + adjoint replay)
    uint32_t main_cap;
};

template <bool InLds>
__global__ void __launch_bounds__(256, MH_VOL_WAVES)
k_prbvol_backward(DScene S, IntegratorParams in, LaneMap lm, uint32_t seed_value, uint64_t n, int coalesce,
                  const float *__restrict__ grad_in, GradArgs ga, unsigned long long *__restrict__ counters,
                  PvpWork wk) {
    extern __shared__ uint4 lds[];
    LdsBvh B = stage_bvh<InLds>(S, lds);
    GradCtx g = make_grad_ctx(ga);
    uint32_t n_closest = 0, n_shadow = 0;
    NeeLog nl;
    nl.buf = wk.log;
    nl.stride = gridDim.x * blockDim.x;
    nl.cap = wk.cap;
    nl.t = blockIdx.x * blockDim.x + threadIdx.x;
    nl.n = 0;
    nl.med = 0;
    nl.overflow = false;
    uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (;;) {
        if (wk.log) {  // next batch of 64 samples for this wave
            unsigned long long b = 0;
            if ((threadIdx.x & 63u) == 0) b = atomicAdd(wk.head, 64ull);
            b = __builtin_amdgcn_readfirstlane((uint32_t)b) | ((unsigned long long)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32);
            if (b >= n) break;
            k = b + (threadIdx.x & 63u);
        }
        if (k < n) {
            uint32_t lane, px, py;
            lane_of(lm, k, lane, px, py);
            Pcg rng;
            rng.seed(seed_value, lane);
            float sx = (float)px + rng.next_float(), sy = (float)py + rng.next_float();
            RayT r = camera_ray(S, __builtin_fmaf(sx, S.inv_width, -0.f),
                                __builtin_fmaf(sy, S.inv_height, -0.f));
            V3 dL = gather_dL_wave(S, coalesce, grad_in, sx, sy);  // grad_in: pre-divided by W (k_grad_over_w)
            Pcg rng_primal = rng;  // sampler.clone()
            if (wk.main) {  // single pass: primal + logged adjoint terms, replay only on overflow
                MainLog ml{wk.main, nl.stride, wk.main_cap, nl.t, 0u, false};
                const V3 Lp = prbvol_sample<2>(S, B, in, rng_primal, r, dL, v3(0, 0, 0), &g, n_closest, n_shadow,
                                               nullptr, &nl, &ml);
                if (!ml.overflow) pvp_log_apply(S, ml, Lp, g);
                else prbvol_sample<3>(S, B, in, rng, r, dL, Lp, &g, n_closest, n_shadow);
            } else {
                V3 Lp = prbvol_sample<0>(S, B, in, rng_primal, r, v3(0, 0, 0), v3(0, 0, 0), nullptr, n_closest,
                                         n_shadow);
                prbvol_sample<1>(S, B, in, rng, r, dL, Lp, &g, n_closest, n_shadow, nullptr, wk.log ? &nl : nullptr);
            }
        }
        if (!wk.log) break;
    }
    flush_small_slots(g, ga);
    if (counters) {
        wave_count(&counters[0], n_closest);
        wave_count(&counters[1], n_shadow);
    }
}

// ===========================================================================
// Host-side launchers (declared in mh_internal.hpp)
// ===========================================================================
static inline uint32_t blocks_for(uint64_t n, uint32_t bs) { return (uint32_t)((n + bs - 1) / bs); }

#ifdef MH_DEBUG
// this unit's device guard counters (mh_device.hpp MH_GUARD), read and reset
hipError_t guard_read_k(unsigned long long *out) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mh_guard), sizeof(g_mh_guard));
    const unsigned long long z[kGuardCount] = {};
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_mh_guard), z, sizeof(z));
    return e;
}
#endif

size_t lds_bytes(const DScene &S, uint32_t block) {
    return (size_t)S.lds_bytes_bvh + (size_t)S.stack_size * block * sizeof(uint32_t);
}

hipError_t launch_trace(const DScene &S, bool shadow, uint64_t n, const float *rays, float *t,
                        float *u, float *v, uint32_t *prim, uint32_t *shape, uint32_t *inst, uint32_t *occ,
                        uint32_t grid, hipStream_t st) {
    const uint32_t bs = 256;
    uint32_t g = grid ? grid : blocks_for(n, bs);
    if (g == 0) return hipSuccess;
    const bool lds = S.lds_bytes_bvh != 0, stream = !lds && (S.qnodes || S.nodes4);
    if (stream && n >= (1ull << 32)) return hipErrorInvalidValue;  // 32-bit stream items
    // the stream engine: its LDS stack, and at most one overflow column per thread
    if (stream && S.stack_ovf) g = std::min<uint32_t>(g, S.ovf_threads / bs);
    const size_t sh = stream ? stream_lds_bytes(S, bs) : lds_bytes(S, bs);
    if (shadow) {
        if (lds) hipLaunchKernelGGL(k_trace_shadow<true>, dim3(g), dim3(bs), sh, st, S, n, rays, occ);
        else hipLaunchKernelGGL(k_trace_shadow<false>, dim3(g), dim3(bs), sh, st, S, n, rays, occ);
    } else {
        if (lds) hipLaunchKernelGGL(k_trace_closest<true>, dim3(g), dim3(bs), sh, st, S, n, rays, t, u, v, prim, shape, inst);
        else hipLaunchKernelGGL(k_trace_closest<false>, dim3(g), dim3(bs), sh, st, S, n, rays, t, u, v, prim, shape, inst);
    }
    return hipGetLastError();
}

hipError_t launch_render(const DScene &S, const IntegratorParams &in, const LaneMap &lm,
                         uint32_t seed_value, uint32_t n_passes, uint64_t n, uint64_t plane,
                         float *out, unsigned long long *counters, hipStream_t st, int alpha) {
    const uint32_t bs = 256;
    size_t sh = lds_bytes(S, bs);
    if (n == 0) return hipSuccess;
    const bool lds = S.lds_bytes_bvh != 0;
    const dim3 g(blocks_for(n, bs)), b(bs);
#define MH_LAUNCH_RENDER(K)                                                                                   \
    do {                                                                                                      \
        if (lds) hipLaunchKernelGGL((k_render<K, true>), g, b, sh, st, S, in, lm, seed_value, n_passes, n, plane, out, counters, alpha); \
        else hipLaunchKernelGGL((k_render<K, false>), g, b, sh, st, S, in, lm, seed_value, n_passes, n, plane, out, counters, alpha);    \
    } while (0)
    if (in.type == MH_INTEGRATOR_PRB) MH_LAUNCH_RENDER(MH_INTEGRATOR_PRB);
    else if (in.type == MH_INTEGRATOR_VOLPATH) MH_LAUNCH_RENDER(MH_INTEGRATOR_VOLPATH);
    else if (in.type == MH_INTEGRATOR_PRBVOLPATH) MH_LAUNCH_RENDER(MH_INTEGRATOR_PRBVOLPATH);
    else MH_LAUNCH_RENDER(MH_INTEGRATOR_PATH);
#undef MH_LAUNCH_RENDER
    return hipGetLastError();
}

hipError_t launch_render_forward(const DScene &S, const IntegratorParams &in, const LaneMap &lm,
                                 uint32_t seed_value, uint64_t n, uint64_t plane, float *out, const GradArgs &ga,
                                 unsigned long long *counters, hipStream_t st, int alpha) {
    const uint32_t bs = 256;
    if (n == 0) return hipSuccess;
    const size_t sh = lds_bytes(S, bs);
    const bool lds = S.lds_bytes_bvh != 0, vol = in.type == MH_INTEGRATOR_PRBVOLPATH;
    const dim3 g(blocks_for(n, bs)), b(bs);
    if (vol && lds) hipLaunchKernelGGL((k_render_forward<true, true>), g, b, sh, st, S, in, lm, seed_value, n, plane, out, ga, counters, alpha);
    else if (vol) hipLaunchKernelGGL((k_render_forward<true, false>), g, b, sh, st, S, in, lm, seed_value, n, plane, out, ga, counters, alpha);
    else if (lds) hipLaunchKernelGGL((k_render_forward<false, true>), g, b, sh, st, S, in, lm, seed_value, n, plane, out, ga, counters, alpha);
    else hipLaunchKernelGGL((k_render_forward<false, false>), g, b, sh, st, S, in, lm, seed_value, n, plane, out, ga, counters, alpha);
    return hipGetLastError();
}

hipError_t launch_splat(const DScene &S, const LaneMap &lm, int mode, bool fast,
                        uint32_t n_pix, uint32_t n_passes, uint64_t n, uint64_t plane,
                        const float *in, float *film, uint32_t seed_value, int coalesce,
                        hipStream_t st, unsigned long long *invalid, bool deterministic, uint64_t in_floats,
                        uint64_t film_floats, unsigned long long *viol) {
    if (n == 0) return hipSuccess;
    // the splat's bounds contract, checked before every launch: sample (k, pass)
    // of pixel pl sits at pass * n + pl * S + k of each plane (k < S), the
    // planes are `plane` floats apart (5 in planes, 6 with alpha), and the
    // film holds W * H pixels of 4 (mode 0) or 1 (W image / alpha) floats
    const uint64_t film_need = (uint64_t)S.width * S.height * (mode == kSplatFilm ? 4 : 1);
    if (film_floats < film_need || (uint64_t)n_pix * lm.S > n || (uint64_t)lm.pixel_begin + n_pix > (uint64_t)S.width * S.height)
        return hipErrorInvalidValue;
    if (mode != kSplatWeights &&
        (plane < (uint64_t)n_passes * n || in_floats < (uint64_t)(mode == kSplatAlpha ? 6 : 5) * plane || !in))
        return hipErrorInvalidValue;
#define MH_SPLAT_PX(M)                                                                                          \
    hipLaunchKernelGGL(k_splat_px<M>, dim3(blocks_for(lanes, bs)), dim3(bs), 0, st, S, lm.pixel_begin, n_pix, \
                       lm.S, n_passes, n, plane, in, film, seed_value, lm.spp_pp, lm.s_begin, invalid, in_floats, viol)
#define MH_SPLAT_GEN(M)                                                                                         \
    hipLaunchKernelGGL(k_splat_generic<M>, dim3(blocks_for(n, bs)), dim3(bs), 0, st, S, lm, n_passes, n, plane, \
                       in, film, seed_value, coalesce, invalid)
#define MH_SPLAT_GATHER(M)                                                                                      \
    hipLaunchKernelGGL(k_splat_gather<M>, dim3(blocks_for((uint64_t)n_rows * S.width, 256)), dim3(256), 0, st, S, \
                       lm.pixel_begin, n_pix, row0, n_rows, lm.S, n_passes, n, plane, in, film, seed_value,      \
                       lm.spp_pp, lm.s_begin)
    if (fast && deterministic) {
        // film rows the chunk's footprints reach: its first row - 2 .. its last row + 3
        const uint32_t r_first = lm.pixel_begin / S.width, r_last = (lm.pixel_begin + n_pix - 1) / S.width;
        const uint32_t row0 = r_first >= 2 ? r_first - 2 : 0, row1 = std::min<uint32_t>(S.height - 1, r_last + 3);
        const uint32_t n_rows = row1 - row0 + 1;
        if (mode == kSplatWeights) MH_SPLAT_GATHER(1);
        else if (mode == kSplatAlpha) MH_SPLAT_GATHER(2);
        else MH_SPLAT_GATHER(0);
        if (mode == kSplatFilm && invalid)  // the sample check of the atomic path, counted by the generic kernel's rule
            hipLaunchKernelGGL(k_count_invalid, dim3(blocks_for(n * n_passes, 256)), dim3(256), 0, st, n * n_passes,
                               n, plane, in, invalid);
    } else if (fast && (mode == kSplatFilm || mode == kSplatWeights) && MH_SPLAT_TILE) {
        const uint32_t r_first = lm.pixel_begin / S.width, r_last = (lm.pixel_begin + n_pix - 1) / S.width;
        const uint32_t tiles_x = (S.width + kSplatTile - 1) / kSplatTile;
        const uint32_t tiles_y = (r_last - r_first + 1 + kSplatTile - 1) / kSplatTile;
        if (mode == kSplatFilm)
            hipLaunchKernelGGL(k_splat_tile<0>, dim3(tiles_x * tiles_y), dim3(256), 0, st, S, lm.pixel_begin, n_pix,
                               r_first, tiles_x, lm.S, n_passes, n, plane, in, film, invalid, in_floats, viol,
                               seed_value, lm.spp_pp, lm.s_begin);
        else
            hipLaunchKernelGGL(k_splat_tile<1>, dim3(tiles_x * tiles_y), dim3(256), 0, st, S, lm.pixel_begin, n_pix,
                               r_first, tiles_x, lm.S, n_passes, n, plane, in, film, invalid, in_floats, viol,
                               seed_value, lm.spp_pp, lm.s_begin);
    } else if (fast) {
        const uint32_t bs = 128;
        const uint64_t lanes = (uint64_t)n_pix * kSplatLanes;
        if (mode == kSplatWeights) MH_SPLAT_PX(1);
        else if (mode == kSplatAlpha) MH_SPLAT_PX(2);
        else MH_SPLAT_PX(0);
    } else {
        const uint32_t bs = 256;
        if (mode == kSplatWeights) MH_SPLAT_GEN(1);
        else if (mode == kSplatAlpha) MH_SPLAT_GEN(2);
        else MH_SPLAT_GEN(0);
    }
#undef MH_SPLAT_PX
#undef MH_SPLAT_GEN
#undef MH_SPLAT_GATHER
    return hipGetLastError();
}

// an alpha film's storage (hdrfilm.cpp:304-327: base_ch = 5, R G B A W) from
// the RGBW film and the alpha plane the splat kernels accumulate
__global__ void k_film_rgbaw(uint64_t n_px, const float *__restrict__ rgbw, const float *__restrict__ a,
                             float *__restrict__ out) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_px) return;
    const float4 v = reinterpret_cast<const float4 *>(rgbw)[i];
    float *o = out + 5 * i;
    o[0] += v.x;
    o[1] += v.y;
    o[2] += v.z;
    o[3] += a[i];
    o[4] += v.w;
}

hipError_t launch_film_rgbaw(uint64_t n_px, const float *rgbw, const float *a, float *out, hipStream_t st) {
    if (n_px == 0) return hipSuccess;
    hipLaunchKernelGGL(k_film_rgbaw, dim3(blocks_for(n_px, 256)), dim3(256), 0, st, n_px, rgbw, a, out);
    return hipGetLastError();
}

hipError_t launch_grad_over_w(uint64_t n_px, const float *grad_in, const float *w, float *out, hipStream_t st) {
    if (n_px == 0) return hipSuccess;
    hipLaunchKernelGGL(k_grad_over_w, dim3(blocks_for(n_px, 256)), dim3(256), 0, st, n_px, grad_in, w, out);
    return hipGetLastError();
}

// order-preserving float -> uint key (negative floats reversed)
__global__ void k_grid_max(const float *__restrict__ data, uint64_t n, uint32_t *__restrict__ key) {
    uint32_t best = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t u = __float_as_uint(data[i]);
        const uint32_t k = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
        best = max(best, k);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) best = max(best, (uint32_t)__shfl_xor((int)best, off));
    if ((threadIdx.x & 63) == 0) atomicMax(key, best);
}

hipError_t launch_grid_max(const float *data, uint64_t n, uint32_t *key, hipStream_t st) {
    hipError_t e = hipMemsetAsync(key, 0, 4, st);
    if (e != hipSuccess || n == 0) return e;
    const uint32_t g = (uint32_t)std::min<uint64_t>(blocks_for(n, 256), 2048);
    hipLaunchKernelGGL(k_grid_max, dim3(g), dim3(256), 0, st, data, n, key);
    return hipGetLastError();
}

__global__ void k_accumulate(float *__restrict__ dst, const float *__restrict__ src, uint64_t n) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] += src[i];
}

// the device layout of a density grid (mh_shading.hpp grid_setup: 4^3
// bricks), in floats
uint64_t grid_bricked_size(const uint32_t res[3]) {
    return (uint64_t)((res[0] + 3) / 4) * ((res[1] + 3) / 4) * ((res[2] + 3) / 4) * 64u;
}

void grid_to_bricks(const float *src, const uint32_t res[3], float *dst) {
    const int32_t rx = (int32_t)res[0], ry = (int32_t)res[1], rz = (int32_t)res[2];
    std::fill(dst, dst + grid_bricked_size(res), 0.f);
    for (int32_t z = 0; z < rz; ++z)
        for (int32_t y = 0; y < ry; ++y)
            for (int32_t x = 0; x < rx; ++x)
                dst[grid_index(x, y, z, rx, ry)] = src[((uint64_t)z * ry + y) * rx + x];
}

__global__ void k_grid_to_bricks(const float *__restrict__ src, int32_t rx, int32_t ry, int32_t rz,
                                 float *__restrict__ dst) {
    const uint64_t n = (uint64_t)rx * ry * rz;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const int32_t x = (int32_t)(i % rx), y = (int32_t)((i / rx) % ry), z = (int32_t)(i / ((uint64_t)rx * ry));
        dst[grid_index(x, y, z, rx, ry)] = src[i];
    }
}

hipError_t launch_grid_to_bricks(const float *src, const uint32_t res[3], float *dst, hipStream_t st) {
    const uint64_t n = std::max<uint64_t>((uint64_t)res[0] * res[1] * res[2], grid_bricked_size(res));
    if ((uint64_t)res[0] * res[1] * res[2] == 0) return hipSuccess;
    const uint32_t g = (uint32_t)std::min<uint64_t>(blocks_for(n, 256), 4096);
    hipLaunchKernelGGL(k_grid_to_bricks, dim3(g), dim3(256), 0, st, src, (int32_t)res[0], (int32_t)res[1],
                       (int32_t)res[2], dst);
    return hipGetLastError();
}

// grad (z, y, x) += the corner block of sigma_t_backward's corner_scatter:
// texel x receives tap b of every cell ix with clamp(ix + b) == x, per axis
// ix = x - b, plus ix = -1 for (b = 0, x = 0) and ix = r - 1 for (b = 1, x = r - 1)
// (cell index ix + 1 in [0, r])
__global__ void k_corner_gather(const float *__restrict__ cb, float *__restrict__ grad, int32_t rx, int32_t ry,
                                int32_t rz) {
    const uint64_t n = (uint64_t)rx * ry * rz;
    const uint64_t sy = (uint64_t)rx + 1, sz = sy * (uint64_t)(ry + 1);
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const int32_t x = (int32_t)(i % rx), y = (int32_t)((i / rx) % ry), z = (int32_t)(i / ((uint64_t)rx * ry));
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const int32_t b[3] = {c & 1, (c >> 1) & 1, c >> 2}, v[3] = {x, y, z}, r[3] = {rx, ry, rz};
            int32_t cell[3][2], cnt[3];
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                cell[a][0] = v[a] - b[a] + 1;
                cnt[a] = 1;
                if (b[a] == 0 && v[a] == 0) cell[a][cnt[a]++] = 0;
                else if (b[a] == 1 && v[a] == r[a] - 1) cell[a][cnt[a]++] = r[a];
            }
            for (int kz = 0; kz < cnt[2]; ++kz)
                for (int ky = 0; ky < cnt[1]; ++ky)
                    for (int kx = 0; kx < cnt[0]; ++kx)
                        s += cb[((uint64_t)cell[2][kz] * sz + (uint64_t)cell[1][ky] * sy + (uint64_t)cell[0][kx]) * 8 + c];
        }
        grad[i] += s;
    }
}

// the fixed-point form: exact int64 sums, one conversion per texel
__global__ void k_corner_gather_fx(const long long *__restrict__ cb, float *__restrict__ grad, int32_t rx, int32_t ry,
                                   int32_t rz, double inv_scale) {
    const uint64_t n = (uint64_t)rx * ry * rz;
    const uint64_t sy = (uint64_t)rx + 1, sz = sy * (uint64_t)(ry + 1);
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const int32_t x = (int32_t)(i % rx), y = (int32_t)((i / rx) % ry), z = (int32_t)(i / ((uint64_t)rx * ry));
        long long s = 0;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const int32_t b[3] = {c & 1, (c >> 1) & 1, c >> 2}, v[3] = {x, y, z}, r[3] = {rx, ry, rz};
            int32_t cell[3][2], cnt[3];
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                cell[a][0] = v[a] - b[a] + 1;
                cnt[a] = 1;
                if (b[a] == 0 && v[a] == 0) cell[a][cnt[a]++] = 0;
                else if (b[a] == 1 && v[a] == r[a] - 1) cell[a][cnt[a]++] = r[a];
            }
            for (int kz = 0; kz < cnt[2]; ++kz)
                for (int ky = 0; ky < cnt[1]; ++ky)
                    for (int kx = 0; kx < cnt[0]; ++kx)
                        s += cb[((uint64_t)cell[2][kz] * sz + (uint64_t)cell[1][ky] * sy + (uint64_t)cell[0][kx]) * 8 + c];
        }
        grad[i] += (float)((double)s * inv_scale);
    }
}

hipError_t launch_corner_gather_fx(const long long *corner, float *grad, const uint32_t res[3], double inv_scale,
                                   hipStream_t st) {
    const uint64_t n = (uint64_t)res[0] * res[1] * res[2];
    if (n == 0) return hipSuccess;
    const uint32_t g = (uint32_t)std::min<uint64_t>(blocks_for(n, 256), 8192);
    hipLaunchKernelGGL(k_corner_gather_fx, dim3(g), dim3(256), 0, st, corner, grad, (int32_t)res[0], (int32_t)res[1],
                       (int32_t)res[2], inv_scale);
    return hipGetLastError();
}

// deterministic bitmap texels (replay kernel): grad[i] += (float)(fx[i] / scale)
__global__ void k_fx_to_float(const long long *__restrict__ fx, float *__restrict__ grad, uint64_t n, double inv_scale) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        if (const long long q = fx[i]) grad[i] += (float)((double)q * inv_scale);
}

hipError_t launch_fx_to_float(const long long *fx, float *grad, uint64_t n, double inv_scale, hipStream_t st) {
    if (n == 0) return hipSuccess;
    const uint32_t g = (uint32_t)std::min<uint64_t>(blocks_for(n, 256), 8192);
    hipLaunchKernelGGL(k_fx_to_float, dim3(g), dim3(256), 0, st, fx, grad, n, inv_scale);
    return hipGetLastError();
}

uint64_t corner_floats(const uint32_t res[3]) {
    return (uint64_t)(res[0] + 1) * (res[1] + 1) * (res[2] + 1) * 8u;
}

hipError_t launch_corner_gather(const float *corner, float *grad, const uint32_t res[3], hipStream_t st) {
    const uint64_t n = (uint64_t)res[0] * res[1] * res[2];
    if (n == 0) return hipSuccess;
    const uint32_t g = (uint32_t)std::min<uint64_t>(blocks_for(n, 256), 8192);
    hipLaunchKernelGGL(k_corner_gather, dim3(g), dim3(256), 0, st, corner, grad, (int32_t)res[0], (int32_t)res[1],
                       (int32_t)res[2]);
    return hipGetLastError();
}

hipError_t launch_accumulate(float *dst, const float *src, uint64_t n, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_accumulate, dim3(blocks_for(n, 256)), dim3(256), 0, st, dst, src, n);
    return hipGetLastError();
}

hipError_t launch_develop(uint64_t n_px, const float *film, float *rgb, uint32_t fmt, hipStream_t st) {
    if (n_px == 0) return hipSuccess;
    const dim3 g(blocks_for(n_px, 256)), b(256);
    switch (fmt) {
    case MH_PIXEL_Y: hipLaunchKernelGGL((k_develop<MH_PIXEL_Y, false>), g, b, 0, st, n_px, film, rgb); break;
    case MH_PIXEL_XYZ: hipLaunchKernelGGL((k_develop<MH_PIXEL_XYZ, false>), g, b, 0, st, n_px, film, rgb); break;
    case MH_PIXEL_RGBA: hipLaunchKernelGGL((k_develop<MH_PIXEL_RGB, true>), g, b, 0, st, n_px, film, rgb); break;
    case MH_PIXEL_YA: hipLaunchKernelGGL((k_develop<MH_PIXEL_Y, true>), g, b, 0, st, n_px, film, rgb); break;
    case MH_PIXEL_XYZA: hipLaunchKernelGGL((k_develop<MH_PIXEL_XYZ, true>), g, b, 0, st, n_px, film, rgb); break;
    default: hipLaunchKernelGGL((k_develop<MH_PIXEL_RGB, false>), g, b, 0, st, n_px, film, rgb);
    }
    return hipGetLastError();
}

hipError_t launch_prb_backward(const DScene &S, const IntegratorParams &in, const LaneMap &lm,
                               uint32_t seed_value, uint64_t n, int coalesce,
                               const float *grad_in, const float *weights, const GradArgs &ga_in,
                               bool fused, unsigned long long *counters, hipStream_t st,
                               float4 *nee_log, uint32_t nee_cap, uint32_t nee_blocks,
                               unsigned long long *head, float4 *main_log, uint32_t main_cap) {
    const uint32_t bs = 256;
    if (n == 0) return hipSuccess;
    size_t sh = lds_bytes(S, bs);
    dim3 g(blocks_for(n, bs)), b(bs);
    GradArgs ga = ga_in;
    if (in.type != MH_INTEGRATOR_PRBVOLPATH && !fused && ga.lds_slot >= 0) {
        // persistent grid: as many workgroups as fit beside the texel accumulator
        // the accumulator must fit the device's per-workgroup LDS beside the
        // BVH / stack staging; otherwise the texels take the global-atomic path
        int dev = 0, cus = 256, max_wg = 64 << 10, per_cu_lds = 160 << 10;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipDeviceGetAttribute(&max_wg, hipDeviceAttributeMaxSharedMemoryPerBlock, dev);
        (void)hipDeviceGetAttribute(&per_cu_lds, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev);
        // the kernel's static LDS (GradCtx's per-wave fixed-point sums,
        // g_fx_wave) comes on top of the dynamic bytes
        hipFuncAttributes fa{};
        const void *fn = S.lds_bytes_bvh ? (fused ? (const void *)k_prb_backward<true, true> : (const void *)k_prb_backward<true, false>)
                                         : (fused ? (const void *)k_prb_backward<false, true> : (const void *)k_prb_backward<false, false>);
        const size_t st_lds = hipFuncGetAttributes(&fa, fn) == hipSuccess ? fa.sharedSizeBytes : (size_t)kFxStaticLdsBytes;
        const uint32_t off = (uint32_t)((sh + 15) / 16 * 16);
        const size_t total = off + (size_t)ga.lds_floats * 4;
        if (total + st_lds <= (size_t)max_wg) {
            ga.lds_offset = off;
            sh = total;
            const size_t lds_cu = per_cu_lds > 0 ? (size_t)per_cu_lds : (size_t)max_wg;
            const uint32_t per_cu = (uint32_t)std::max<size_t>(1, std::min<size_t>(4, lds_cu / (sh + st_lds)));
            g = dim3(std::min<uint32_t>(blocks_for(n, bs), (uint32_t)cus * per_cu));
        } else {
            ga.lds_slot = -1;
        }
    } else {
        ga.lds_slot = -1;
    }
    if (in.type == MH_INTEGRATOR_PRBVOLPATH) {
        PvpWork wk{nullptr, 0, nullptr, nullptr, 0};
        if (nee_log && head && nee_cap && nee_blocks) {
            wk = PvpWork{nee_log, nee_cap, head, main_cap ? main_log : nullptr, main_cap};
            g = dim3(nee_blocks);
            hipError_t e = hipMemsetAsync(head, 0, sizeof(unsigned long long), st);
            if (e != hipSuccess) return e;
        }
        if (S.lds_bytes_bvh)
            hipLaunchKernelGGL((k_prbvol_backward<true>), g, b, sh, st, S, in, lm, seed_value, n, coalesce, grad_in, ga, counters, wk);
        else
            hipLaunchKernelGGL((k_prbvol_backward<false>), g, b, sh, st, S, in, lm, seed_value, n, coalesce, grad_in, ga, counters, wk);
    } else if (S.lds_bytes_bvh && fused)
        hipLaunchKernelGGL((k_prb_backward<true, true>), g, b, sh, st, S, in, lm, seed_value, n, coalesce, grad_in, weights, ga, counters);
    else if (S.lds_bytes_bvh)
        hipLaunchKernelGGL((k_prb_backward<true, false>), g, b, sh, st, S, in, lm, seed_value, n, coalesce, grad_in, weights, ga, counters);
    else if (fused)
        hipLaunchKernelGGL((k_prb_backward<false, true>), g, b, sh, st, S, in, lm, seed_value, n, coalesce, grad_in, weights, ga, counters);
    else
        hipLaunchKernelGGL((k_prb_backward<false, false>), g, b, sh, st, S, in, lm, seed_value, n, coalesce, grad_in, weights, ga, counters);
    return hipGetLastError();
}

}  // namespace mh
