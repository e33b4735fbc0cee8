// mh_device.hpp — gfx950 device-side data layout and per-lane math for the
// `path` / `prb` / `volpath` hot path.  Compiled only by hipcc for gfx950.
//
// Numerics contract: built with -ffp-contract=off and
// -fhip-fp32-correctly-rounded-divide-sqrt; an fma appears exactly where the
// reference (or Dr.Jit 0.4.4's LLVM backend) emits dr::fmadd, rcp(x) = 1/x,
// rsqrt(x) = sqrt(1/x), sincos = Cephes polynomial.  This makes every lane
// bit-comparable with the CPU oracle (oracle/mh_oracle.c).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mitsuba_hip.h"

namespace mh {

#define MH_DEV __device__ __forceinline__

// Debug build (tools/build_variant.sh <name> -DMH_DEBUG): device bounds
// guards.  A failed check counts into this translation unit's g_mh_guard[k];
// the entry points read every unit's counters after the call (guard_read_*)
// and fail it when one is nonzero.  Release builds compile them away.
enum {
    kGuardQueueSlot = 0,   // a queue item beyond its segment's capacity
    kGuardPathId = 1,      // a path id beyond the chunk's paths
    kGuardAppendSlot = 2,  // a compacted (appended) slot beyond the segment's capacity
    kGuardPlane = 3,       // a sample-plane index beyond the plane
    kGuardPixel = 4,       // a generated sample's pixel outside the film
    kGuardLds = 5,         // an LDS texel accumulator index beyond the accumulator
    kGuardCount = 8
};
#ifdef MH_DEBUG
static __device__ unsigned long long g_mh_guard[kGuardCount];
#define MH_GUARD(cond, k)                                           \
    do {                                                            \
        if (!(cond)) atomicAdd(&g_mh_guard[(k)], 1ull);             \
    } while (0)
#else
#define MH_GUARD(cond, k) \
    do {                  \
    } while (0)
#endif

// Atomic adds to device (global) memory through a generic pointer, emitted as
// global_atomic_*.  For a pointer it cannot prove global (loaded from a
// struct or a pointer table) the compiler emits flat_atomic_*, and a flat
// operation counts in lgkmcnt as well as vmcnt: every later LDS wait of the
// wave then waits for the atomic's round trip to memory (round 6: the
// prbvolpath backward's corner scatters, the bitmap / film scatters).
typedef __attribute__((address_space(1))) float g_float;
typedef __attribute__((address_space(1))) unsigned long long g_u64;
MH_DEV void gatomic_add(float *p, float v) {
    __hip_atomic_fetch_add((g_float *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
MH_DEV void gatomic_add(unsigned long long *p, unsigned long long v) {
    __hip_atomic_fetch_add((g_u64 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr float kPi = 3.14159265358979323846f;
constexpr float kInvPi = 0.31830988618379067154f;
constexpr float kRayEps = 1500.0f * 5.9604644775390625e-08f;  // core/math.h:18-23
constexpr float kShadowEps = kRayEps * 10.0f;
constexpr float kFloatMax = 3.40282346638528859812e+38f;      // dr::Largest<float>

// ---------------------------------------------------------------------------
// Device scene layout (HBM; the BVH + primitive records are staged into LDS)
// ---------------------------------------------------------------------------
struct alignas(16) Node {       // 64 B: two child boxes (Aila-Laine BVH2 layout)
    float4 lo0, hi0, lo1, hi1;  // .w of lo = child index / first prim, .w of hi = leaf word (0 = inner)
};
// leaf word: primitive count in the low 16 bits, number of rectangles (the
// leaf's primitives are ordered rectangles first) from bit 16
constexpr uint32_t kLeafCountMask = 0xffffu, kLeafRectShift = 16;

// 128 B: four child boxes in SoA (one float4 per plane), the per-lane stream
// engine's wide node for large scenes (collapsed from the BVH2, mh_bvh.cpp).
// ref: inner Node4 index, or kLeafBit | first << 5 | count, or kEmptyRef.
struct alignas(16) Node4 {
    float4 lox, loy, loz, hix, hiy, hiz;
    uint4 ref;
    uint4 pad;
};

struct alignas(16) Prim {       // 64 B primitive record
    float4 a, b, c;             // triangle: v0, e1 = v1 - v0, e2 = v2 - v0; rectangle: to_object rows
    uint4 info;                 // x: shape, y: prim index (face; ~0 for rectangles), z: type, w: scene-order key
};

// 64 B: the quantised wide node of the stream engine (round 4; mh_bvh.cpp
// build_qbvh4).  Child c's box on axis a is [o_a + qlo_a[c] * s_a, o_a +
// qhi_a[c] * s_a] with s_a = 2^(ebits byte a - 127), decoded by one fma per
// bound (exact product, one rounding); the host picks each byte so that the
// decoded float box contains the padded float box of the BVH2, so the slab
// test stays conservative and hits stay bit-identical.  Byte c of qlo[a] /
// qhi[a] is child c.  ref: as Node4.  A node's inner children are contiguous
// (children-contiguous depth-first order).
struct alignas(16) QNode4 {
    float ox, oy, oz;
    uint32_t ebits;
    uint32_t qlo[3], qhi_x;
    uint32_t qhi_y, qhi_z, pad0, pad1;
    uint32_t ref[4];
};

// 48 B: the compact primitive record of the stream engine, in the leaf order
// of Prim (same index): v0, e1, e2 of a triangle, the scene-order key, the
// face index and the shape (kPrimCRect set for a rectangle, whose test reads
// the full Prim of the same index).
struct alignas(16) PrimC {
    float v0x, v0y, v0z, e1x, e1y, e1z, e2x, e2y, e2z;
    uint32_t key, prim, shape;
};
constexpr uint32_t kPrimCRect = 0x80000000u;

struct DShape {                 // shading-time shape record
    uint32_t type, bsdf, emitter, face_offset;
    uint32_t vertex_offset, has_normals, has_texcoords, pad;
    float to_world[12];
    float frame_s[4], frame_t[4], frame_n[4];
    float inv_area;
    uint32_t interior, exterior, pad3;  // media (MH_INVALID = none)
};

struct DTexture {
    uint32_t type, width, height, channels;
    uint64_t data_offset;
    uint32_t filter, wrap;
    float value[4];
    float to_uv[8];
};

struct DEmitter {
    uint32_t type, shape, pad0, pad1;
    float radiance[4];
    float direction[4];
    float center[3], radius;   // constant / directional: scene bounding sphere
};

struct DMedium {
    uint32_t type, phase, flags, pad0;
    float g, scale, maj, sigma_t_const;   // maj = scale * max(grid) (heterogeneous.cpp:163)
    float albedo[4];
    uint32_t res[4];
    uint64_t grid_offset, pad1;   // grid_offset: first float of the medium's bricked grid (grid_index)
    float to_local[12];
    float bbox_min[4], bbox_max[4];
};

// PRBVolpathIntegrator.prepare_scene (prbvolpath.py:76-89), from the media of the shapes
constexpr uint32_t kVolHandleNull = 1u;       // some medium is heterogeneous
constexpr uint32_t kVolNeeHomogeneous = 2u;   // some medium is homogeneous

struct DScene {                 // kernel argument (by value)
    const Node *nodes;
    const Prim *prims;
    const DShape *shapes;
    const uint32_t *bsdf_type;     // per bsdf
    const uint32_t *bsdf_tex;      // per bsdf reflectance texture
    const DTexture *textures;
    const DEmitter *emitters;
    const float *positions;        // float3 (packed)
    const float *normals;
    const float *texcoords;
    const uint32_t *faces;
    const float *texels;
    const DMedium *media;
    const float *grid;             // volume grid data
    const Node4 *nodes4;           // wide BVH of the stream engine (nullptr: BVH2 only)
    const uint2 *key_sp;           // scene-order key -> (shape, prim) (packet engine)
    const Prim *prim_pairs;        // interleaved pair records of the packet engine (mh_shading.hpp pp())
    uint32_t n_nodes, n_prims, n_emitters, environment;
    uint32_t n_media, camera_medium;
    uint32_t vol_flags;            // prbvolpath prepare_scene flags (kVol*)
    // small shading tables (shapes .. faces) staged into LDS by the shade
    // kernels when tab_bytes != 0 (mh_shading.hpp stage_tables)
    uint32_t n_shapes, n_bsdfs, n_textures, n_vertices, n_faces, tab_bytes;
    uint32_t stack_size;           // BVH traversal stack entries per lane
    uint32_t lds_bytes_bvh;        // bytes of nodes + prims staged into LDS
    // sensor
    float cam_to_world[16];
    float sample_to_camera[16];
    float near_clip, far_clip;
    uint32_t width, height;
    uint32_t rfilter;
    float rfilter_radius;
    float filter_coeff[10];
    uint32_t sampler_seed;
    // (last: the fused bounce kernels never read them, and fields ahead of
    // the ones they do read shift the kernel-argument layout they are tuned on)
    const QNode4 *qnodes;          // quantised wide BVH of the stream engine (nullptr: Node4 / BVH2)
    const PrimC *primsc;           // its compact primitive records (with qnodes)
    // the per-lane stream engine's stack: stream_stack entries per lane in
    // LDS (<= stack_size), the deeper ones in stack_ovf (entry k of global
    // thread g at (k - stream_stack) * ovf_threads + g; nullptr: none needed)
    uint32_t *stack_ovf;
    uint32_t stream_stack, ovf_threads;
    // 1 / (float)width, 1 / (float)height, 1 / (float)n_emitters: divided on the host (correctly rounded,
    // as the device's division), so the bounce kernels hold no per-lane loop-invariant quotients
    float inv_width, inv_height, inv_n_emitters;
    float n_emitters_f, env_pdf;  // (float)n_emitters; kInv4Pi * inv_n_emitters (a constant emitter's pdf)
};

// lane -> (pixel, sample) map of one render call (sample-slab aware)
struct LaneMap {
    uint32_t W, spp_pp, log_spp;  // log_spp == 32 -> integer division
    uint32_t pixel_begin, S, s_begin, log_S;
};

// ---------------------------------------------------------------------------
// fp32 vector helpers (Dr.Jit semantics)
// ---------------------------------------------------------------------------
struct V3 { float x, y, z; };

MH_DEV V3 v3(float x, float y, float z) { return V3{x, y, z}; }
MH_DEV V3 operator+(V3 a, V3 b) { return V3{a.x + b.x, a.y + b.y, a.z + b.z}; }
MH_DEV V3 operator-(V3 a, V3 b) { return V3{a.x - b.x, a.y - b.y, a.z - b.z}; }
MH_DEV V3 operator*(V3 a, V3 b) { return V3{a.x * b.x, a.y * b.y, a.z * b.z}; }
MH_DEV V3 operator*(V3 a, float s) { return V3{a.x * s, a.y * s, a.z * s}; }
MH_DEV V3 operator-(V3 a) { return V3{-a.x, -a.y, -a.z}; }
MH_DEV V3 vdiv(V3 a, float s) { return V3{a.x / s, a.y / s, a.z / s}; }
// dr::fmadd(vector, scalar, vector)
MH_DEV V3 fma3s(V3 a, float b, V3 c) {
    return V3{__builtin_fmaf(a.x, b, c.x), __builtin_fmaf(a.y, b, c.y), __builtin_fmaf(a.z, b, c.z)};
}
MH_DEV V3 fma3(V3 a, V3 b, V3 c) {
    return V3{__builtin_fmaf(a.x, b.x, c.x), __builtin_fmaf(a.y, b.y, c.y), __builtin_fmaf(a.z, b.z, c.z)};
}
// dr::dot: a.x*b.x then an fmadd chain
MH_DEV float dot(V3 a, V3 b) {
    return __builtin_fmaf(a.z, b.z, __builtin_fmaf(a.y, b.y, a.x * b.x));
}
// dr::cross: fmsub(a.y, b.z, a.z*b.y), ...
MH_DEV V3 cross(V3 a, V3 b) {
    return V3{__builtin_fmaf(a.y, b.z, -(a.z * b.y)), __builtin_fmaf(a.z, b.x, -(a.x * b.z)),
              __builtin_fmaf(a.x, b.y, -(a.y * b.x))};
}
// rcp(x) == 1.0f / x correctly rounded (the numerics contract),
// in 3 VALU on the common path: v_rcp_f32 (<= 1 ulp) and one Newton step on
// fma give RN(1/x) for every 2^-126 <= |x| < 2^126 -- checked bit for bit
// against the IEEE division for all 2^32 inputs on gfx950
// (tools/exp_rcp.hip).  Lanes outside that range (zero, denormals,
// |x| >= 2^126, inf, NaN) take the full division behind a wave vote.
MH_DEV bool rcp_fast_ok(float x) { return (__builtin_fabsf(x) >= 0x1p-126f) & (__builtin_fabsf(x) < 0x1p126f); }
// some active lane is outside the fast range (two ballots straight off the
// compares, so no lane mask is materialised in a VGPR)
MH_DEV bool rcp_fast_any_bad(float x) {
    const float a = __builtin_fabsf(x);
    return (__builtin_amdgcn_ballot_w64(!(a >= 0x1p-126f)) | __builtin_amdgcn_ballot_w64(!(a < 0x1p126f))) != 0;
}
// the full division, kept behind its branch (a volatile asm cannot be
// speculated, so the compiler does not if-convert it into every lane's path)
MH_DEV float rcp_slow(float x) {
    asm volatile("" : "+v"(x));
    return 1.0f / x;
}
MH_DEV float rcp_core(float x) {
    const float y = __builtin_amdgcn_rcpf(x);
    return __builtin_fmaf(__builtin_fmaf(-x, y, 1.f), y, y);
}
MH_DEV float rcp(float x) {
    float y = rcp_core(x);
    if (rcp_fast_any_bad(x)) {
        if (!rcp_fast_ok(x)) y = rcp_slow(x);
    }
    return y;
}
MH_DEV float rsqrt_(float x) { return __builtin_sqrtf(rcp(x)); }
MH_DEV V3 normalize(V3 v) { return v * rsqrt_(dot(v, v)); }
MH_DEV float norm(V3 v) { return __builtin_sqrtf(dot(v, v)); }
MH_DEV float hmax(V3 v) { return fmaxf(fmaxf(v.x, v.y), v.z); }
MH_DEV V3 ld3(const float *p) { return V3{p[0], p[1], p[2]}; }
MH_DEV float mulsign(float a, float b) { return b >= 0.f ? a : -a; }
MH_DEV float mulsign_neg(float a, float b) { return b >= 0.f ? -a : a; }
MH_DEV bool isfinite_(float x) { return __builtin_fabsf(x) < __builtin_huge_valf(); }
MH_DEV bool nonzero(V3 v) { return v.x != 0.f || v.y != 0.f || v.z != 0.f; }

// Transform4f point / vector products (core/transform.h:104-141); 3x4 row-major
MH_DEV V3 xf_point(const float *m, V3 p) {
    return V3{__builtin_fmaf(m[2], p.z, __builtin_fmaf(m[1], p.y, __builtin_fmaf(m[0], p.x, m[3]))),
              __builtin_fmaf(m[6], p.z, __builtin_fmaf(m[5], p.y, __builtin_fmaf(m[4], p.x, m[7]))),
              __builtin_fmaf(m[10], p.z, __builtin_fmaf(m[9], p.y, __builtin_fmaf(m[8], p.x, m[11])))};
}
MH_DEV V3 xf_vector(const float *m, V3 v) {
    return V3{__builtin_fmaf(m[2], v.z, __builtin_fmaf(m[1], v.y, m[0] * v.x)),
              __builtin_fmaf(m[6], v.z, __builtin_fmaf(m[5], v.y, m[4] * v.x)),
              __builtin_fmaf(m[10], v.z, __builtin_fmaf(m[9], v.y, m[8] * v.x))};
}

// ---------------------------------------------------------------------------
// Cephes sincos (Dr.Jit 0.4.4 math.h sincos for JIT-LLVM float arrays)
// ---------------------------------------------------------------------------
MH_DEV float poly2(float x, float c0, float c1, float c2) {
    float x2 = x * x;
    return __builtin_fmaf(x2, c2, __builtin_fmaf(x, c1, c0));
}
MH_DEV void sincos_cephes(float x, float &s_out, float &c_out) {
    float xa = __builtin_fabsf(x);
    int32_t j = (int32_t)(xa * 1.2732395447351626862f);
    j = (j + 1) & ~1;
    float y = (float)j;
    uint32_t sign_sin = ((uint32_t)j << 29) ^ __float_as_uint(x);
    uint32_t sign_cos = (~(uint32_t)(j - 2)) << 29;
    y = xa - y * 0.78515625f - y * 2.4187564849853515625e-4f - y * 3.77489497744594108e-8f;
    float z = y * y;
    if (xa == __builtin_huge_valf()) z = __uint_as_float(0xffffffffu);
    float s = poly2(z, -1.6666654611e-1f, 8.3321608736e-3f, -1.9515295891e-4f) * z;
    float c = poly2(z, 4.166664568298827e-2f, -1.388731625493765e-3f, 2.443315711809948e-5f) * z;
    s = __builtin_fmaf(s, y, y);
    c = __builtin_fmaf(c, z, __builtin_fmaf(z, -0.5f, 1.0f));
    bool polymask = (j & 2) == 0;
    float rs = polymask ? s : c, rc = polymask ? c : s;
    s_out = __uint_as_float(__float_as_uint(rs) ^ (sign_sin & 0x80000000u));
    c_out = __uint_as_float(__float_as_uint(rc) ^ (sign_cos & 0x80000000u));
}

// ---------------------------------------------------------------------------
// TEA + PCG32 (core/random.h:77-90, render/sampler.cpp:115-134, [drjit] PCG32)
// ---------------------------------------------------------------------------
MH_DEV void tea4(uint32_t v0, uint32_t v1, uint32_t &o0, uint32_t &o1) {
    uint32_t sum = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        sum += 0x9e3779b9u;
        v0 += ((v1 << 4) + 0xa341316cu) ^ (v1 + sum) ^ ((v1 >> 5) + 0xc8013ea4u);
        v1 += ((v0 << 4) + 0xad90777du) ^ (v0 + sum) ^ ((v0 >> 5) + 0x7e95761eu);
    }
    o0 = v0;
    o1 = v1;
}

struct Pcg {
    uint64_t state, inc;
    MH_DEV uint32_t next() {
        uint64_t old = state;
        state = old * 0x5851f42d4c957f2dull + inc;
        uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
        uint32_t rot = (uint32_t)(old >> 59u);
        return (xs >> rot) | (xs << ((0u - rot) & 31u));
    }
    MH_DEV float next_float() { return __uint_as_float((next() >> 9) | 0x3f800000u) - 1.0f; }
    MH_DEV void seed(uint32_t seed_value, uint32_t lane) {
        uint32_t v0, v1;
        tea4(seed_value, lane, v0, v1);
        state = 0;
        inc = ((uint64_t)v1 << 1) | 1u;
        next();
        state += (uint64_t)v0;
        next();
    }
};

// ---------------------------------------------------------------------------
// Gaussian reconstruction filter (rfilters/gaussian.cpp:94-97, [drjit] Estrin)
// ---------------------------------------------------------------------------
MH_DEV float estrin10(float x, const float *k) {
    float c0 = __builtin_fmaf(x, k[1], k[0]), c1 = __builtin_fmaf(x, k[3], k[2]),
          c2 = __builtin_fmaf(x, k[5], k[4]), c3 = __builtin_fmaf(x, k[7], k[6]),
          c4 = __builtin_fmaf(x, k[9], k[8]);
    float x2 = x * x;
    float d0 = __builtin_fmaf(x2, c1, c0), d1 = __builtin_fmaf(x2, c3, c2);
    float x4 = x2 * x2;
    float e0 = __builtin_fmaf(x4, d1, d0);
    float x8 = x4 * x4;
    return __builtin_fmaf(x8, c4, e0);
}
MH_DEV float estrin6(float x, float c0, float c1, float c2, float c3, float c4, float c5) {
    float a0 = __builtin_fmaf(x, c1, c0), a1 = __builtin_fmaf(x, c3, c2), a2 = __builtin_fmaf(x, c5, c4);
    float x2 = x * x;
    float b0 = __builtin_fmaf(x2, a1, a0);
    float x4 = x2 * x2;
    return __builtin_fmaf(x4, a2, b0);
}

// Dr.Jit 0.4.4 math.h `exp`, single precision, non-CUDA branch (Cephes range
// reduction + Estrin polynomial + ldexp by exponent construction)
MH_DEV float exp_dr(float x) {
    const bool overflow = x > 88.3762626647949f, underflow = x < -88.3762626647949f;
    float n = floorf(__builtin_fmaf(1.44269504088896340736f, x, 0.5f));
    x = __builtin_fmaf(-n, 0.693359375f, x);
    x = __builtin_fmaf(-n, -2.12194440e-4f, x);
    float z = estrin6(x, 5.0000001201e-1f, 1.6666665459e-1f, 4.1665795894e-2f, 8.3334519073e-3f,
                      1.3981999507e-3f, 1.9875691500e-4f);
    z = __builtin_fmaf(z, x * x, x + 1.0f);
    z = z * __uint_as_float((uint32_t)((int32_t)n + 127) << 23);
    if (overflow) z = __builtin_huge_valf();
    if (underflow) z = 0.f;
    return z;
}

// Dr.Jit 0.4.4 math.h `log` (Cephes logf: frexp + polynomial)
MH_DEV float log_dr(float x) {
    if (!(x > 0.f)) return x == 0.f ? -__builtin_huge_valf() : __uint_as_float(0xffffffffu);
    if (x == __builtin_huge_valf()) return x;
    uint32_t bits = __float_as_uint(x);
    int e;
    float xm;
    if ((bits & 0x7f800000u) == 0) {
        xm = frexpf(x, &e);
    } else {
        e = (int)((bits >> 23) & 0xff) - 126;
        xm = __uint_as_float((bits & 0x807fffffu) | 0x3f000000u);
    }
    if (xm < 0.70710678118654752440f) {
        e -= 1;
        xm = xm + xm - 1.0f;
    } else {
        xm = xm - 1.0f;
    }
    float z = xm * xm;
    float y = 7.0376836292e-2f;
    y = __builtin_fmaf(y, xm, -1.1514610310e-1f);
    y = __builtin_fmaf(y, xm, 1.1676998740e-1f);
    y = __builtin_fmaf(y, xm, -1.2420140846e-1f);
    y = __builtin_fmaf(y, xm, 1.4249322787e-1f);
    y = __builtin_fmaf(y, xm, -1.6668057665e-1f);
    y = __builtin_fmaf(y, xm, 2.0000714765e-1f);
    y = __builtin_fmaf(y, xm, -2.4999993993e-1f);
    y = __builtin_fmaf(y, xm, 3.3333331174e-1f);
    y = y * xm * z;
    float fe = (float)e;
    y = __builtin_fmaf(fe, -2.12194440e-4f, y);
    y = __builtin_fmaf(z, -0.5f, y);
    float r = xm + y;
    return __builtin_fmaf(fe, 0.693359375f, r);
}

MH_DEV float gaussian_eval(const float *coeff, float x) {
    return fmaxf(estrin10(x * x, coeff), 0.f);
}

}  // namespace mh
