// mh_wavefront.hip — wavefront (stream) execution of the `path` integrator:
// PathIntegrator::sample (integrators/path.cpp:95-287) split at its two ray
// queries into separate persistent kernels over structure-of-arrays state.
//
//   k_wf_raygen   render_sample prologue (integrator.cpp:1139-1176): TEA/PCG32
//                 seeding, pixel jitter, perspective camera ray -> ray SoA
//   k_wf_trace    Scene::ray_intersect (scene.cpp:181-190): SoA ray in, SoA
//                 hit record out (t, u, v, prim, shape) — the OptiX slot
//   k_wf_shade    one loop iteration of path.cpp:142-281 up to the NEE
//                 visibility test: emission + MIS, light sample, BSDF sample,
//                 spawn, Russian roulette; survivors are compacted into the
//                 next queue, NEE candidates into the shadow queue (wave
//                 ballot + one atomic per wave)
//   k_wf_shadow   Scene::ray_test (scene.cpp:201-210) + the deferred
//                 `result = fma(throughput, bsdf_val*em_weight*mis, result)`
//
// Every per-lane operation is the one the megakernel executes (same device
// functions, same order), so results are bit-identical to k_render and the
// CPU oracle.  Work is pulled by waves from an atomic head (no host sync
// between bounces: queue counts stay on the device).
#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <cstring>

#include "mh_shading.hpp"

namespace mh {

// Path state is stored per queue SLOT, not per path id, in two ping-pong
// buffers: the shade kernel reads slot i of the current queue and writes the
// survivor's state to its compacted slot of the next queue, so every state
// access is a coalesced SoA stream.  The path id (for the output sample
// planes and the PCG32 stream) travels in the low 24 bits of `pd`, the depth
// in the high 8.
struct WfState {
    uint32_t *pd[2];
    float *ox[2], *oy[2], *oz[2], *dx[2], *dy[2], *dz[2], *mt[2];
    float *bx[2], *by[2], *bz[2], *ppx[2], *ppy[2], *ppz[2], *ppdf[2];
    uint64_t *rng[2];
    float *lx[2], *ly[2], *lz[2];                              // radiance so far (fused bounce kernel)
    float *ht, *hu, *hv;                                       // hit record of the current bounce
    uint32_t *hp, *hs;
    uint32_t *sid;                                             // shadow records
    float *sox, *soy, *soz, *sdx, *sdy, *sdz, *smt, *sax, *say, *saz, *sbx, *sby, *sbz;
};

// Queues are split into kSeg statically partitioned segments (paths never
// change segment).  Workgroup b serves one segment (seg_iter), so a segment's state
// stays on one XCD's L2 (blocks b, b+8, ... share an XCD) and every segment
// has its own counters on a private 128-B line: no single-word atomic hot
// spot (MI355X_MICROARCH.md "dequeue": one word saturates at ~88 ops/us).
// Per bounce: kSeg x 32 uint32: [s*32 + 0] queue length, [s*32 + 1] shadow length.
constexpr uint32_t kSeg = 64;
#ifndef MH_SEG_XCD
#define MH_SEG_XCD 0  // 1 measured slower: bench 1,859 -> 1,806, 1M-triangle mesh 558 -> 500 Msamples/s (round 4)
#endif
static_assert(kSeg == 64, "seg_iter's XCD-contiguous map assumes 64 segments over 8 XCDs");
#ifndef MH_BOUNCE_WAVES
#define MH_BOUNCE_WAVES 5  // fused bounce kernels: waves per SIMD the register budget targets
#endif
#ifndef MH_BOUNCE_PRB_WAVES
#define MH_BOUNCE_PRB_WAVES MH_BOUNCE_WAVES  // the fused PRB bounce kernel's
#endif
constexpr uint32_t kCtrStride = kSeg * 32;
// path id and depth share a word: 2^MH_PID_BITS paths per chunk, depth
// < 2^(32 - MH_PID_BITS) (the wavefront runs max_depth <= 64: 7 bits)
#ifndef MH_PID_BITS
#define MH_PID_BITS 25
#endif
constexpr uint32_t kPidBits = MH_PID_BITS, kPidMask = (1u << kPidBits) - 1u;
constexpr uint32_t kMaxWfBounces = (1u << (32 - kPidBits)) - 1u;

// Traversal engine of the stream kernels: wave-coherent packets for small
// BVHs (every wave visits about the whole tree anyway; no divergence, no
// per-lane stack, broadcast node reads), per-lane while-while otherwise.
// MH_TRAVERSAL=packet|lane overrides (tests cover both).
constexpr uint32_t kPacketMaxPrims = 64;
// MH_PACKET_MAX_PRIMS: experiments with larger packet scenes (read once)
uint32_t wf_packet_max_prims() {
    static const uint32_t v = [] {
        const char *e = getenv("MH_PACKET_MAX_PRIMS");
        return e ? (uint32_t)std::max(1, atoi(e)) : kPacketMaxPrims;
    }();
    return v;
}
static bool use_packet(const DScene &S) {
    const char *e = getenv("MH_TRAVERSAL");
    if (S.n_prims > wf_packet_max_prims()) return false;  // no pair records beyond (mh_api.hip)
    if (e && !strcmp(e, "packet")) return true;
    if (e && !strcmp(e, "lane")) return false;
    return true;
}
// MH_WF_FUSED=0 keeps the three-kernel pipeline (trace / shade / shadow)
static bool wf_unfused() {
    const char *e = getenv("MH_WF_FUSED");
    return e && !strcmp(e, "0");
}
// the stream kernels are instantiated per node format (Eng), so each one's
// register allocation is that of its own traversal engine
#define MH_WF_DISPATCH(K, ...)                                                                        \
    do {                                                                                              \
        const dim3 g_(grid), b_(256);                                                                 \
        if (lds && packet) hipLaunchKernelGGL((K<true, true, kEngBvh2>), g_, b_, sh, st, __VA_ARGS__);         \
        else if (lds) hipLaunchKernelGGL((K<true, false, kEngBvh2>), g_, b_, sh, st, __VA_ARGS__);           \
        else if (packet) hipLaunchKernelGGL((K<false, true, kEngBvh2>), g_, b_, sh, st, __VA_ARGS__);        \
        else switch (stream_engine(S)) {                                                              \
            case kEngQuant: hipLaunchKernelGGL((K<false, false, kEngQuant>), g_, b_, sh, st, __VA_ARGS__); break; \
            case kEngWideC: hipLaunchKernelGGL((K<false, false, kEngWideC>), g_, b_, sh, st, __VA_ARGS__); break; \
            case kEngWide: hipLaunchKernelGGL((K<false, false, kEngWide>), g_, b_, sh, st, __VA_ARGS__); break;   \
            default: hipLaunchKernelGGL((K<false, false, kEngBvh2>), g_, b_, sh, st, __VA_ARGS__); break;        \
        }                                                                                             \
    } while (0)
#define MH_WF_DISPATCH_NR(K, NR, ...)                                                                 \
    do {                                                                                              \
        const dim3 g_(grid), b_(256);                                                                 \
        if (lds && packet) hipLaunchKernelGGL((K<true, true, NR, kEngBvh2>), g_, b_, sh, st, __VA_ARGS__);     \
        else if (lds) hipLaunchKernelGGL((K<true, false, NR, kEngBvh2>), g_, b_, sh, st, __VA_ARGS__);       \
        else if (packet) hipLaunchKernelGGL((K<false, true, NR, kEngBvh2>), g_, b_, sh, st, __VA_ARGS__);    \
        else switch (stream_engine(S)) {                                                              \
            case kEngQuant: hipLaunchKernelGGL((K<false, false, NR, kEngQuant>), g_, b_, sh, st, __VA_ARGS__); break; \
            case kEngWideC: hipLaunchKernelGGL((K<false, false, NR, kEngWideC>), g_, b_, sh, st, __VA_ARGS__); break; \
            case kEngWide: hipLaunchKernelGGL((K<false, false, NR, kEngWide>), g_, b_, sh, st, __VA_ARGS__); break;   \
            default: hipLaunchKernelGGL((K<false, false, NR, kEngBvh2>), g_, b_, sh, st, __VA_ARGS__); break;        \
        }                                                                                             \
    } while (0)

static inline size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

uint32_t wf_counter_words(uint32_t n_bounces) { return kCtrStride * (n_bounces + 1); }

#ifdef MH_DEBUG
// this unit's device guard counters (mh_device.hpp MH_GUARD), read and reset
hipError_t guard_read_wf(unsigned long long *out) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mh_guard), sizeof(g_mh_guard));
    const unsigned long long z[kGuardCount] = {};
    if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_mh_guard), z, sizeof(z));
    return e;
}
#endif
uint64_t wf_max_chunk() { return 1ull << kPidBits; }

size_t wf_workspace_bytes(uint64_t cap) {
    // 55 4-byte planes + 2 8-byte planes, each 256-B aligned; capacity padded
    // to a whole number of segments
    cap = (cap + kSeg - 1) / kSeg * kSeg;
    return 55 * align_up(cap * 4) + 2 * align_up(cap * 8);
}

static WfState carve(void *ws, uint64_t cap) {
    cap = (cap + kSeg - 1) / kSeg * kSeg;
    uint8_t *p = reinterpret_cast<uint8_t *>(ws);
    auto f = [&]() { float *r = reinterpret_cast<float *>(p); p += align_up(cap * 4); return r; };
    auto u = [&]() { uint32_t *r = reinterpret_cast<uint32_t *>(p); p += align_up(cap * 4); return r; };
    WfState w;
    for (int k = 0; k < 2; ++k) {
        w.pd[k] = u();
        w.ox[k] = f(); w.oy[k] = f(); w.oz[k] = f(); w.dx[k] = f(); w.dy[k] = f(); w.dz[k] = f(); w.mt[k] = f();
        w.bx[k] = f(); w.by[k] = f(); w.bz[k] = f(); w.ppx[k] = f(); w.ppy[k] = f(); w.ppz[k] = f(); w.ppdf[k] = f();
        w.lx[k] = f(); w.ly[k] = f(); w.lz[k] = f();
    }
    w.ht = f(); w.hu = f(); w.hv = f(); w.hp = u(); w.hs = u();
    w.sid = u();
    w.sox = f(); w.soy = f(); w.soz = f(); w.sdx = f(); w.sdy = f(); w.sdz = f(); w.smt = f();
    w.sax = f(); w.say = f(); w.saz = f(); w.sbx = f(); w.sby = f(); w.sbz = f();
    for (int k = 0; k < 2; ++k) {
        w.rng[k] = reinterpret_cast<uint64_t *>(p);
        p += align_up(cap * 8);
    }
    return w;
}

// Path state of the fused bounce kernels: 16-B records, one plane per record
// field group (SoA of float4), ping-pong buffers b = 0, 1 -- five 16-B loads
// and stores per path-bounce instead of twenty 4-B ones, and two base
// addresses instead of a pointer per plane (kernel-argument SGPRs):
//   plane 0: o.x o.y o.z maxt        plane 3: prev_p.x .y .z rng.lo
//   plane 1: d.x d.y d.z pd          plane 4: L.x L.y L.z rng.hi    (PRB: dL.x .y .z rng.hi)
//   plane 2: tp.x tp.y tp.z prev_pdf
// (The PRB bounce kernel keeps the 4-B planes of WfState / WfPrb: packed, its
// extra registers cost more than the fewer memory instructions saved, measured
// bwd 20.0 -> 20.7 ms per bench step.)
constexpr uint32_t kPkPlanes = 5, kPkExt = 3;
struct WfPacked {
    float4 *base, *ext;
    uint64_t stride;  // float4 per plane
    uint32_t *tea_base;  // ping-pong: the TEA word of the path's PCG32 increment (WfPrb::tea)
    uint64_t tstride;    // uint32 per tea plane
    MH_DEV float4 *pl(int b, uint32_t k) const { return base + (uint64_t)(b * (int)kPkPlanes + (int)k) * stride; }
    MH_DEV float4 *ex(int b, uint32_t k) const { return ext + (uint64_t)(b * (int)kPkExt + (int)k) * stride; }
    MH_DEV uint32_t *tea(int b) const { return tea_base + (uint64_t)b * tstride; }
};
static WfPacked carve_packed(void *ws, void *ws_ext, uint64_t cap) {
    cap = (cap + kSeg - 1) / kSeg * kSeg;
    WfPacked p;
    p.stride = align_up(cap * 16) / 16;
    p.base = reinterpret_cast<float4 *>(ws);
    p.ext = reinterpret_cast<float4 *>(ws_ext);
    // two 4-B planes after the 2 x kPkPlanes records (inside wf_workspace_bytes)
    p.tea_base = reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(ws) + 2 * kPkPlanes * align_up(cap * 16));
    p.tstride = align_up(cap * 4) / 4;
    return p;
}

MH_DEV uint32_t lane_id() { return threadIdx.x & 63u; }

// Diagnostic build (-DMH_EXP_BPHASE): s_memtime cycles of the fused bounce
// kernels' phases, summed per wave and added once per wave into g_bph[group]
// (group: 0 / 1 k_wf_bounce generating / not, 2 / 3 k_wf_bounce_prb
// generating / not; phases: 0 state load or ray generation, 1 closest-hit
// packet trace, 2 shade, 3 compaction + state store, 4 shadow packet trace,
// 5 tail (NEE charge, radiance out), 6 iterations, 7 block prologue; 8-11
// spare).  A phase is charged with the waits that fall in it (a load issued
// earlier is paid where its value is first used: the state loads issued
// after the closest trace are paid in shade).  Read by mh_exp_bphase.
#ifdef MH_EXP_BPHASE
__device__ unsigned long long g_bph[4][12];
#define MH_BPH_DECL uint64_t bph_t = __builtin_amdgcn_s_memtime(); uint64_t bph[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#define MH_BPH(k) do { const uint64_t _t = __builtin_amdgcn_s_memtime(); bph[k] += _t - bph_t; bph_t = _t; } while (0)
#define MH_BPH_ITER() (bph[6] += 1)
#define MH_BPH_FLUSH(grp)                                                                 \
    do {                                                                                  \
        if (lane_id() == 0)                                                               \
            for (int _k = 0; _k < 12; ++_k) atomicAdd(&g_bph[grp][_k], (unsigned long long)bph[_k]); \
    } while (0)
#else
#define MH_BPH_DECL
#define MH_BPH(k) do {} while (0)
#define MH_BPH_ITER() do {} while (0)
#define MH_BPH_FLUSH(grp) do {} while (0)
#endif

// segment geometry of a launch: segment of this block, this wave's rank
// among the segment's waves and the number of waves serving the segment
struct SegIter {
    uint32_t seg, wave, nwaves;
};
MH_DEV SegIter seg_iter() {
    SegIter it;
    // Blocks are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md:
    // b and b + 8 share one).  Default: segment b % 64 (XCD x serves segments
    // x, x + 8, ...: pixel bands spread over the image, so every XCD gets a
    // share of every region's work).  MH_SEG_XCD = 1: XCD x serves segments
    // 8x .. 8x + 7, one contiguous eighth of the pixels, for L2 locality --
    // measured slower on the bench and the large meshes (the per-XCD loads
    // become uneven).  Either map gives a segment the blocks b = s' + 64 k.
#if MH_SEG_XCD
    it.seg = (blockIdx.x & 7u) * 8u + ((blockIdx.x >> 3) & 7u);
#else
    it.seg = blockIdx.x % kSeg;
#endif
    const uint32_t wpb = blockDim.x / 64u;
    it.wave = (blockIdx.x / kSeg) * wpb + threadIdx.x / 64u;
    it.nwaves = (gridDim.x / kSeg) * wpb;
    return it;
}
__host__ __device__ inline uint32_t seg_len(uint64_t n) { return (uint32_t)((n + kSeg - 1) / kSeg); }

// ballot-compacted append; must be reached by the whole wave
MH_DEV uint32_t wave_append(uint32_t *count, bool pred) {
    const unsigned long long m = __ballot(pred);
    const uint32_t tot = (uint32_t)__popcll(m);
    uint32_t base = 0;
    if (lane_id() == 0 && tot) base = atomicAdd(count, tot);
    base = __builtin_amdgcn_readfirstlane(base);
    // the lanes below this one (v_mbcnt: no 64-bit lane mask kept live across
    // the kernel's loop, which the PRB bounce spilled to scratch)
    const uint32_t off = lane_rank(m);
    return base + off;
}

// inc of the lane's PCG32 stream (sampler.cpp:115-134), recomputed from TEA
MH_DEV uint64_t pcg_inc(uint32_t seed_value, uint32_t lane) {
    uint32_t v0, v1;
    tea4(seed_value, lane, v0, v1);
    return ((uint64_t)v1 << 1) | 1u;
}

// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
k_wf_raygen(DScene S, LaneMap lm, uint32_t seed_value, uint64_t n, uint64_t plane, float *out,
            WfState w, uint32_t *ctr) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < kSeg) {
        const uint64_t L = seg_len(n), b = k * L;
        ctr[k * 32] = b >= n ? 0u : (uint32_t)std::min<uint64_t>(L, n - b);
    }
    if (k >= n) return;
    uint32_t lane, px, py;
    lane_of(lm, k, lane, px, py);
    Pcg rng;
    rng.seed(seed_value, lane);
    float sx = (float)px + rng.next_float(), sy = (float)py + rng.next_float();
    RayT r = camera_ray(S, __builtin_fmaf(sx, S.inv_width, -0.f),
                        __builtin_fmaf(sy, S.inv_height, -0.f));
    // slot k of buffer 0 == path k (segment s holds ids [s*L, (s+1)*L))
    w.pd[0][k] = (uint32_t)k;  // depth 0: prev_bsdf_delta = true on the first bounce
    w.ox[0][k] = r.o.x; w.oy[0][k] = r.o.y; w.oz[0][k] = r.o.z;
    w.dx[0][k] = r.d.x; w.dy[0][k] = r.d.y; w.dz[0][k] = r.d.z; w.mt[0][k] = r.maxt;
    w.bx[0][k] = 1.f; w.by[0][k] = 1.f; w.bz[0][k] = 1.f;
    w.ppx[0][k] = 0.f; w.ppy[0][k] = 0.f; w.ppz[0][k] = 0.f; w.ppdf[0][k] = 1.f;
    w.rng[0][k] = rng.state;
    w.lx[0][k] = 0.f; w.ly[0][k] = 0.f; w.lz[0][k] = 0.f;
    out[k] = 0.f; out[plane + k] = 0.f; out[2 * plane + k] = 0.f;
    out[3 * plane + k] = sx; out[4 * plane + k] = sy;
}

// does any wave of this workgroup get items of its segment?  (uniform per
// block: lets empty workgroups of short late-bounce queues exit before
// staging anything into LDS)
MH_DEV bool block_has_stride_work(const SegIter &it, uint32_t n) {
    const uint32_t first_wave = (blockIdx.x / kSeg) * (blockDim.x / 64u);
    return first_wave * 64u < n;
}
MH_DEV bool block_has_range_work(const SegIter &it, uint32_t n) {
    const uint32_t first_wave = (blockIdx.x / kSeg) * (blockDim.x / 64u);
    const uint32_t per = (n + it.nwaves - 1) / it.nwaves;
    return first_wave * per < n;
}

// contiguous share of a segment for this wave (refill traversal)
MH_DEV void wave_range(const SegIter &it, uint32_t n, uint32_t &r0, uint32_t &r1) {
    const uint32_t per = (n + it.nwaves - 1) / it.nwaves;
    r0 = min(n, it.wave * per);
    r1 = min(n, r0 + per);
}

// occupancy target of the unfused trace kernels (experiments: -DMH_STREAM_WAVES=n).
// With the LDS stack capped (DScene::stream_stack) registers set it: 6 waves
// per SIMD (80 VGPRs, 2 spilled) measured +3-4 % over 5 on 1M / 4M-triangle
// meshes (522 -> 536 / 434 -> 450 Msamples/s), 8 waves (64 VGPRs) -10 %.
#ifndef MH_STREAM_WAVES
#define MH_STREAM_WAVES 6
#endif
#define MH_STREAM_LB __launch_bounds__(256, MH_STREAM_WAVES)

// Packet: wave-coherent engine (small BVHs) instead of the per-lane stream engine
template <bool InLds, bool Packet, int Eng>
__global__ void MH_STREAM_LB
k_wf_trace(DScene S, WfState w, int cur, uint32_t seg_cap, uint32_t *ctr) {
    extern __shared__ uint4 lds[];
    const SegIter it = seg_iter();
    const uint32_t n = __hip_atomic_load(ctr + it.seg * 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!block_has_range_work(it, n)) return;
    LdsBvh B = stage_bvh<InLds && !Packet>(S, lds);  // the packet engine reads the BVH via s_load
    const uint32_t base = it.seg * seg_cap;
    const float *ox = w.ox[cur], *oy = w.oy[cur], *oz = w.oz[cur], *dx = w.dx[cur], *dy = w.dy[cur],
                *dz = w.dz[cur], *mt = w.mt[cur];
    uint32_t r0, r1;
    wave_range(it, n, r0, r1);
    auto load = [&](uint32_t i) {
        const uint32_t j = base + i;
        return RayT{v3(ox[j], oy[j], oz[j]), v3(dx[j], dy[j], dz[j]), mt[j]};
    };
    auto store = [&](uint32_t i, const Hit &h, bool) {
        const uint32_t j = base + i;
        w.ht[j] = h.t; w.hu[j] = h.u; w.hv[j] = h.v; w.hp[j] = h.prim; w.hs[j] = h.shape;
    };
    if (Packet) trace_packet<false>(S.nodes, S.prims, S.prim_pairs, S.key_sp, B, r0, r1, load, store);
    else trace_stream<false, Eng>(B, r0, r1, load, store);
}

// one iteration of PathIntegrator::sample for every queued path
// Staged: shading tables in LDS (stage_tables)
template <bool Staged>
__global__ void __launch_bounds__(256, 5)
k_wf_shade(DScene S0, IntegratorParams in, LaneMap lm, uint32_t seed_value, uint64_t plane,
           float *out, WfState w, int cur, uint32_t seg_cap, uint32_t *ctr, uint32_t *ctr_next, int alpha) {
    extern __shared__ uint4 lds[];
    const SegIter it = seg_iter();
    const uint32_t n = __hip_atomic_load(ctr + it.seg * 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!block_has_stride_work(it, n)) return;
    const DScene S = Staged ? stage_tables(S0, lds) : S0;
    const uint32_t sbase = it.seg * seg_cap;  // slots (state, hits, shadow records) of this segment
    const int nxt = cur ^ 1;
    for (uint32_t base = it.wave * 64u; base < n; base += it.nwaves * 64u) {
        const uint32_t i = base + lane_id();
        bool alive = false, shadow = false;
        uint32_t pid = 0;
        RayT ray, sray;
        V3 tp, a_nee, b_nee, prev_p;
        float eta = 1.f, prev_pdf = 1.f;
        uint32_t depth = 0;
        Pcg rng;
        if (i < n) {
            const uint32_t j = sbase + i;
            const uint32_t pd = w.pd[cur][j];
            pid = pd & kPidMask;
            depth = pd >> kPidBits;
            ray.o = v3(w.ox[cur][j], w.oy[cur][j], w.oz[cur][j]);
            ray.d = v3(w.dx[cur][j], w.dy[cur][j], w.dz[cur][j]);
            ray.maxt = w.mt[cur][j];
            Hit h;
            h.t = w.ht[j]; h.u = w.hu[j]; h.v = w.hv[j]; h.prim = w.hp[j]; h.shape = w.hs[j];
            tp = v3(w.bx[cur][j], w.by[cur][j], w.bz[cur][j]);
            // diffuse / null BSDFs only: eta stays 1 and only the camera vertex
            // (depth 0) has a delta "previous bsdf"
            eta = 1.f;
            const bool prev_delta = depth == 0;
            prev_p = v3(w.ppx[cur][j], w.ppy[cur][j], w.ppz[cur][j]);
            prev_pdf = w.ppdf[cur][j];
            uint32_t lane, px, py;
            lane_of(lm, pid, lane, px, py);
            rng.state = w.rng[cur][j];
            rng.inc = pcg_inc(seed_value, lane);
            SI si;
            compute_si(S, ray, h, si);

            // ---- direct emission (path.cpp:158-174); a camera ray that escapes
            // with the environment hidden returns 0 (valid_ray, path.cpp:115, 256, 284)
            const uint32_t em = si.valid ? S.shapes[si.shape].emitter : S.environment;
            const bool hidden = depth == 0 && !si.valid && in.hide_emitters;
            if (em != MH_INVALID && !hidden) {
                float em_pdf = prev_delta ? 0.f : emitter_pdf_direction(S, em, si, prev_p);
                float mis_bsdf = mis_weight(prev_pdf, em_pdf);
                V3 le = v3(0, 0, 0);
                if (prev_pdf > 0.f)
                    le = emitter_eval(S, em, si);
                V3 L = v3(out[pid], out[plane + pid], out[2 * plane + pid]);
                L = fma3(tp, le * mis_bsdf, L);
                out[pid] = L.x; out[plane + pid] = L.y; out[2 * plane + pid] = L.z;
            }
            // alpha: valid_ray (path.cpp:115, 256); a path ends at its first miss,
            // so the camera vertex decides it
            if (alpha && depth == 0)
                out[5 * plane + pid] = (si.valid || (!in.hide_emitters && S.environment != MH_INVALID)) ? 1.f : 0.f;
            const bool active_next = (depth + 1 < in.max_depth) && si.valid;
            const uint32_t b = si.valid ? S.shapes[si.shape].bsdf : MH_INVALID;
            const bool smooth = b != MH_INVALID && S.bsdf_type[b] == MH_BSDF_DIFFUSE;
            const bool active_em = active_next && smooth;

            // ---- emitter sampling (path.cpp:187-208); visibility is deferred
            float e0 = rng.next_float(), e1 = rng.next_float();
            DirS ds;
            ds.pdf = 0.f;
            ds.d = v3(0, 0, 0);
            ds.delta = false;
            V3 em_weight = v3(0, 0, 0), wo = v3(0, 0, 0);
            if (active_em) {
                em_weight = scene_sample_emitter_direction(S, si.p, e0, e1, ds);
                if (ds.pdf != 0.f && nonzero(em_weight)) {
                    shadow = true;
                    sray = spawn_ray_to(si.p, si.n, ds.p);
                }
                wo = to_local(si, ds.d);
            }

            // ---- BSDF eval + sample (path.cpp:212-216)
            (void)rng.next_float();
            float s2x = rng.next_float(), s2y = rng.next_float();
            V3 bsdf_val = v3(0, 0, 0), bsdf_weight = v3(0, 0, 0), bs_wo = v3(0, 0, 0);
            float bsdf_pdf = 0.f, bs_pdf = 0.f, bs_eta = 0.f;
            if (smooth) {
                V3 rho = tex_eval(S, S.bsdf_tex[b], si.uvx, si.uvy);
                diffuse_eval_pdf(rho, si.wi, wo, true, bsdf_val, bsdf_pdf);
                bs_wo = square_to_cosine_hemisphere(s2x, s2y);
                bs_pdf = kInvPi * bs_wo.z;
                bs_eta = 1.f;
                bsdf_weight = (si.wi.z > 0.f && bs_pdf > 0.f) ? rho : v3(0, 0, 0);
            }
            if (shadow) {  // (path.cpp:220-230), applied by k_wf_shadow if unoccluded
                a_nee = tp;
                b_nee = (bsdf_val * em_weight) * (ds.delta ? 1.f : mis_weight(ds.pdf, bsdf_pdf));
            }

            // ---- BSDF sampling, state update, Russian roulette (path.cpp:234-280)
            ray = spawn_ray(si.p, si.n, to_world(si, bs_wo));
            tp = tp * bsdf_weight;
            eta *= bs_eta;
            prev_p = si.p;
            prev_pdf = bs_pdf;
            if (si.valid) depth += 1;
            float tmax = hmax(tp);
            float rr_prob = fminf(tmax * (eta * eta), 0.95f);
            bool rr_active = depth >= in.rr_depth;
            bool rr_continue = rng.next_float() < rr_prob;
            if (rr_active) tp = tp * rcp(rr_prob);
            alive = active_next && (!rr_active || rr_continue) && tmax != 0.f;
        }
        // compaction: survivors -> next queue, NEE candidates -> shadow queue
        const uint32_t slot = sbase + wave_append(ctr_next + it.seg * 32, alive);
        const uint32_t sslot = sbase + wave_append(ctr + it.seg * 32 + 1, shadow);
        if (alive) {
            w.pd[nxt][slot] = pid | (depth << kPidBits);
            w.ox[nxt][slot] = ray.o.x; w.oy[nxt][slot] = ray.o.y; w.oz[nxt][slot] = ray.o.z;
            w.dx[nxt][slot] = ray.d.x; w.dy[nxt][slot] = ray.d.y; w.dz[nxt][slot] = ray.d.z;
            w.mt[nxt][slot] = ray.maxt;
            w.bx[nxt][slot] = tp.x; w.by[nxt][slot] = tp.y; w.bz[nxt][slot] = tp.z;
            w.ppx[nxt][slot] = prev_p.x; w.ppy[nxt][slot] = prev_p.y; w.ppz[nxt][slot] = prev_p.z;
            w.ppdf[nxt][slot] = prev_pdf;
            w.rng[nxt][slot] = rng.state;
        }
        if (shadow) {
            w.sid[sslot] = pid;
            w.sox[sslot] = sray.o.x; w.soy[sslot] = sray.o.y; w.soz[sslot] = sray.o.z;
            w.sdx[sslot] = sray.d.x; w.sdy[sslot] = sray.d.y; w.sdz[sslot] = sray.d.z; w.smt[sslot] = sray.maxt;
            w.sax[sslot] = a_nee.x; w.say[sslot] = a_nee.y; w.saz[sslot] = a_nee.z;
            w.sbx[sslot] = b_nee.x; w.sby[sslot] = b_nee.y; w.sbz[sslot] = b_nee.z;
        }
    }
}

// ---------------------------------------------------------------------------
// Fused bounce kernel (small scenes: packet engine + LDS-staged tables).  For
// every queued path of the bounce: the closest-hit packet trace, one
// iteration of PathIntegrator::sample (path.cpp:142-281), the NEE shadow
// packet trace and the deferred `result = fma(throughput, bsdf_val *
// em_weight * mis, result)`, with L carried in the path state and written to
// the sample planes once, when the path ends.  Same per-lane operations in
// the same order as k_wf_trace -> k_wf_shade -> k_wf_shadow (bit-identical),
// without the hit and shadow records in HBM, and with the traversal VALU of
// one wave overlapping the state streams of the others.
// LDS: shading tables (tab_bytes) + one traversal stack per wave.
// ---------------------------------------------------------------------------
// Gen: the first bounce generates its paths (k_wf_raygen's camera ray, PCG32
// state and film position) in registers instead of reading them from the
// queue -- the 80-B path state of every camera ray never goes to HBM.  Slot j
// of bounce 0 is path j; n_total: paths of the chunk.
template <bool Gen>
__global__ void __launch_bounds__(256, MH_BOUNCE_WAVES)
k_wf_bounce(DScene S0, IntegratorParams in, LaneMap lm, uint32_t seed_value, uint64_t plane, float *out,
            WfPacked w, int cur, uint32_t seg_cap, uint32_t *ctr, uint32_t *ctr_next, uint64_t n_total,
            uint64_t *carry, uint32_t pass, int alpha) {
    extern __shared__ uint4 lds[];
    const SegIter it = seg_iter();
    auto seg_count = [&](uint32_t sg) -> uint32_t {
        if (Gen) {
            const uint64_t b0 = (uint64_t)sg * seg_cap;
            return b0 >= n_total ? 0u : (uint32_t)std::min<uint64_t>(seg_cap, n_total - b0);
        }
        return __hip_atomic_load(ctr + sg * 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    const uint32_t n = seg_count(it.seg);
    if (Gen && blockIdx.x < kSeg && threadIdx.x == 0) ctr[it.seg * 32] = n;  // queue statistics
    if (!block_has_stride_work(it, n)) return;
    MH_BPH_DECL
    float *recs = reinterpret_cast<float *>(reinterpret_cast<uint8_t *>(lds) + fused_pairs_offset(S0));
    stage_pair_records(S0, recs);  // made visible by stage_tables' barrier
    const DScene S = stage_tables(S0, lds);
    uint32_t *ws = reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(lds) + S0.tab_bytes) +
                   (threadIdx.x >> 6) * S0.stack_size;
    uint8_t *dscr = reinterpret_cast<uint8_t *>(lds) + fused_scratch_offset(S0) + (threadIdx.x >> 6) * kDeferScratch;
    const int nxt = cur ^ 1;
    uint32_t n_shadow = 0;
    MH_BPH(7);
    const uint32_t seg = it.seg;
    for (uint32_t base = it.wave * 64u; base < n; base += it.nwaves * 64u) {
        const uint32_t sbase = seg * seg_cap;
        MH_BPH_ITER();
        const uint32_t i = base + lane_id();
        const bool has = i < n;
        const uint32_t j = sbase + i;
        MH_GUARD(!has || i < seg_cap, kGuardQueueSlot);
        bool alive = false, shadow = false;
        uint32_t pid = 0, depth = 0;
        RayT ray{v3(0, 0, 0), v3(0, 0, 1), -1.f}, sray{v3(0, 0, 0), v3(0, 0, 1), -1.f};
        V3 tp, a_nee, b_nee, prev_p, L;
        float eta = 1.f, prev_pdf = 1.f;
        Pcg rng;
        uint64_t gen_state = 0, gen_inc = 0;
        if (has) {
            if (Gen) {  // k_wf_raygen (integrator.cpp:1139-1176, perspective.cpp:240-281)
                pid = j;
                uint32_t lane, px, py;
                lane_of(lm, pid, lane, px, py);
                MH_GUARD(px < S0.width && py < S0.height, kGuardPixel);
                Pcg g;
                if (pass == 0) {
                    g.seed(seed_value, lane);
                } else {  // later pass: the lane's stream continues (integrator.cpp:353-357)
                    g.state = carry[pid];
                    g.inc = pcg_inc(seed_value, lane);
                }
                const float sx = (float)px + g.next_float(), sy = (float)py + g.next_float();
                ray = camera_ray(S0, __builtin_fmaf(sx, S0.inv_width, -0.f),
                                 __builtin_fmaf(sy, S0.inv_height, -0.f));
                gen_state = g.state;
                gen_inc = g.inc;  // the TEA of this lane, reused below
                out[3 * plane + pid] = sx;
                out[4 * plane + pid] = sy;
            } else {
                const float4 q0 = w.pl(cur, 0)[j], q1 = w.pl(cur, 1)[j];
                const uint32_t pd = __float_as_uint(q1.w);
                pid = pd & kPidMask;
                depth = pd >> kPidBits;
                ray.o = v3(q0.x, q0.y, q0.z);
                ray.d = v3(q1.x, q1.y, q1.z);
                ray.maxt = q0.w;
            }
            MH_GUARD(pid < n_total, kGuardPathId);
            MH_GUARD(pid < plane, kGuardPlane);
        }
        MH_BPH(0);
        const Hit h = packet_batch<false, true>(S0.nodes, S0.prims, S0.prim_pairs, S0.key_sp, ws, 1u, ray, has, recs, dscr);
        MH_BPH(1);
        if (has) {
            if (Gen) {
                tp = v3(1.f, 1.f, 1.f);
                L = v3(0.f, 0.f, 0.f);
                prev_p = v3(0.f, 0.f, 0.f);
                prev_pdf = 1.f;
                rng.state = gen_state;
            } else {
                const uint32_t jl = j;
                const float4 q2 = w.pl(cur, 2)[jl], q3 = w.pl(cur, 3)[jl], q4 = w.pl(cur, 4)[jl];
                tp = v3(q2.x, q2.y, q2.z);
                prev_pdf = q2.w;
                prev_p = v3(q3.x, q3.y, q3.z);
                L = v3(q4.x, q4.y, q4.z);
                rng.state = (uint64_t)__float_as_uint(q3.w) | ((uint64_t)__float_as_uint(q4.w) << 32);
            }
            eta = 1.f;  // diffuse / null BSDFs: eta stays 1, only the camera vertex is delta
            const bool prev_delta = depth == 0;
            rng.inc = Gen ? gen_inc : (((uint64_t)w.tea(cur)[j] << 1) | 1u);
            SI si;
            compute_si(S, ray, h, si);

            // ---- direct emission (path.cpp:158-174); a camera ray that escapes
            // with the environment hidden returns 0 (valid_ray, path.cpp:115, 256, 284)
            const uint32_t em = si.valid ? S.shapes[si.shape].emitter : S.environment;
            const bool hidden = depth == 0 && !si.valid && in.hide_emitters;
            if (em != MH_INVALID && !hidden) {
                float em_pdf = prev_delta ? 0.f : emitter_pdf_direction(S, em, si, prev_p);
                float mis_bsdf = mis_weight(prev_pdf, em_pdf);
                V3 le = v3(0, 0, 0);
                if (prev_pdf > 0.f) le = emitter_eval(S, em, si);
                L = fma3(tp, le * mis_bsdf, L);
            }
            if (Gen && alpha)  // valid_ray (path.cpp:115, 256): decided at the camera vertex
                out[5 * plane + pid] = (si.valid || (!in.hide_emitters && S.environment != MH_INVALID)) ? 1.f : 0.f;
            const bool active_next = (depth + 1 < in.max_depth) && si.valid;
            const uint32_t b = si.valid ? S.shapes[si.shape].bsdf : MH_INVALID;
            const bool smooth = b != MH_INVALID && S.bsdf_type[b] == MH_BSDF_DIFFUSE;
            const bool active_em = active_next && smooth;

            // ---- emitter sampling (path.cpp:187-208); visibility below
            float e0 = rng.next_float(), e1 = rng.next_float();
            DirS ds;
            ds.pdf = 0.f;
            ds.d = v3(0, 0, 0);
            ds.delta = false;
            V3 em_weight = v3(0, 0, 0), wo = v3(0, 0, 0);
            if (active_em) {
                em_weight = scene_sample_emitter_direction(S, si.p, e0, e1, ds);
                if (ds.pdf != 0.f && nonzero(em_weight)) {
                    shadow = true;
                    sray = spawn_ray_to(si.p, si.n, ds.p);
                }
                wo = to_local(si, ds.d);
            }

            // ---- BSDF eval + sample (path.cpp:212-216)
            (void)rng.next_float();
            float s2x = rng.next_float(), s2y = rng.next_float();
            V3 bsdf_val = v3(0, 0, 0), bsdf_weight = v3(0, 0, 0), bs_wo = v3(0, 0, 0);
            float bsdf_pdf = 0.f, bs_pdf = 0.f, bs_eta = 0.f;
            if (smooth) {
                V3 rho = tex_eval(S, S.bsdf_tex[b], si.uvx, si.uvy);
                diffuse_eval_pdf(rho, si.wi, wo, true, bsdf_val, bsdf_pdf);
                bs_wo = square_to_cosine_hemisphere(s2x, s2y);
                bs_pdf = kInvPi * bs_wo.z;
                bs_eta = 1.f;
                bsdf_weight = (si.wi.z > 0.f && bs_pdf > 0.f) ? rho : v3(0, 0, 0);
            }
            if (shadow) {  // (path.cpp:220-230), applied below if unoccluded
                a_nee = tp;
                b_nee = (bsdf_val * em_weight) * (ds.delta ? 1.f : mis_weight(ds.pdf, bsdf_pdf));
            }

            // ---- BSDF sampling, state update, Russian roulette (path.cpp:234-280)
            ray = spawn_ray(si.p, si.n, to_world(si, bs_wo));
            tp = tp * bsdf_weight;
            eta *= bs_eta;
            prev_p = si.p;
            prev_pdf = bs_pdf;
            if (si.valid) depth += 1;
            float tmax = hmax(tp);
            float rr_prob = fminf(tmax * (eta * eta), 0.95f);
            bool rr_active = depth >= in.rr_depth;
            bool rr_continue = rng.next_float() < rr_prob;
            if (rr_active) tp = tp * rcp(rr_prob);
            alive = active_next && (!rr_active || rr_continue) && tmax != 0.f;
        }
        MH_BPH(2);
        // ---- compaction: the survivor's next-bounce state leaves registers
        // before the shadow trace (only L and the NEE product stay live across it)
        const uint32_t slot = sbase + wave_append(ctr_next + seg * 32, alive);
        MH_GUARD(!alive || slot - sbase < seg_cap, kGuardAppendSlot);
        const float rng_hi = __uint_as_float((uint32_t)(rng.state >> 32));
        if (alive) {
            w.pl(nxt, 0)[slot] = make_float4(ray.o.x, ray.o.y, ray.o.z, ray.maxt);
            w.pl(nxt, 1)[slot] = make_float4(ray.d.x, ray.d.y, ray.d.z, __uint_as_float(pid | (depth << kPidBits)));
            w.pl(nxt, 2)[slot] = make_float4(tp.x, tp.y, tp.z, prev_pdf);
            w.pl(nxt, 3)[slot] = make_float4(prev_p.x, prev_p.y, prev_p.z, __uint_as_float((uint32_t)rng.state));
            w.tea(nxt)[slot] = (uint32_t)(rng.inc >> 1);
        } else if (has && carry) {
            carry[pid] = rng.state;  // multi-pass: the next pass continues the stream
        }
        MH_BPH(3);
        // ---- visibility of the NEE sample (scene.cpp:201-210)
        const Hit sh = packet_batch<true, true>(S0.nodes, S0.prims, S0.prim_pairs, S0.key_sp, ws, 1u, sray, shadow, recs, dscr);
        MH_BPH(4);
        if (shadow && sh.shape == MH_INVALID) L = fma3(a_nee, b_nee, L);
        n_shadow += (uint32_t)__popcll(__ballot(shadow));
        // ---- radiance: survivors carry it on, finished paths -> sample planes
        if (alive) {
            w.pl(nxt, 4)[slot] = make_float4(L.x, L.y, L.z, rng_hi);
        } else if (has) {
            out[pid] = L.x; out[plane + pid] = L.y; out[2 * plane + pid] = L.z;
        }
        MH_BPH(5);
    }
    if (lane_id() == 0 && n_shadow) atomicAdd(ctr + it.seg * 32 + 1, n_shadow);  // statistics only
    MH_BPH_FLUSH(Gen ? 0 : 1);
}

template <bool InLds, bool Packet, int Eng>
__global__ void MH_STREAM_LB
k_wf_shadow(DScene S, WfState w, uint64_t plane, float *out, uint32_t seg_cap, uint32_t *ctr) {
    extern __shared__ uint4 lds[];
    const SegIter it = seg_iter();
    const uint32_t n = __hip_atomic_load(ctr + it.seg * 32 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!block_has_range_work(it, n)) return;
    LdsBvh B = stage_bvh<InLds && !Packet>(S, lds);
    const uint32_t base = it.seg * seg_cap;
    uint32_t r0, r1;
    wave_range(it, n, r0, r1);
    auto load = [&](uint32_t i) {
        const uint32_t j = base + i;
        return RayT{v3(w.sox[j], w.soy[j], w.soz[j]), v3(w.sdx[j], w.sdy[j], w.sdz[j]), w.smt[j]};
    };
    auto store = [&](uint32_t i, const Hit &, bool occluded) {
        if (occluded) return;
        const uint32_t j = base + i, pid = w.sid[j];
        V3 L = v3(out[pid], out[plane + pid], out[2 * plane + pid]);
        L = fma3(v3(w.sax[j], w.say[j], w.saz[j]), v3(w.sbx[j], w.sby[j], w.sbz[j]), L);
        out[pid] = L.x; out[plane + pid] = L.y; out[2 * plane + pid] = L.z;
    };
    if (Packet) trace_packet<true>(S.nodes, S.prims, S.prim_pairs, S.key_sp, B, r0, r1, load, store);
    else trace_stream<true, Eng>(B, r0, r1, load, store);
}

// ---------------------------------------------------------------------------
// Host driver: one chunk of n <= capacity paths, all bounces queued on `st`
// without host synchronisation.  trace_ev: optional event pairs bracketing
// every k_wf_trace launch (roofline timing of the dominant kernel).
// ---------------------------------------------------------------------------
static hipError_t launch_wavefront_pass(const DScene &S, const IntegratorParams &in, const LaneMap &lm,
                                        uint32_t seed_value, uint64_t n, uint64_t plane, float *out, void *ws,
                                        uint64_t cap, uint32_t *ctr, uint32_t n_bounces, uint32_t grid,
                                        hipEvent_t *trace_ev, hipStream_t st, uint64_t *carry, uint32_t pass,
                                        int alpha);

hipError_t launch_wavefront(const DScene &S, const IntegratorParams &in, const LaneMap &lm,
                            uint32_t seed_value, uint64_t n, uint64_t plane, float *out, void *ws,
                            uint64_t cap, uint32_t *ctr, uint32_t n_bounces, uint32_t grid,
                            hipEvent_t *trace_ev, hipStream_t st, uint32_t n_passes, uint64_t *carry,
                            int alpha) {
    if (n == 0) return hipSuccess;
    if (n > (1ull << kPidBits) || n_bounces > kMaxWfBounces || n_passes == 0) return hipErrorInvalidValue;
    if (n_passes == 1)
        return launch_wavefront_pass(S, in, lm, seed_value, n, plane, out, ws, cap, ctr, n_bounces, grid, trace_ev,
                                     st, nullptr, 0, alpha);
    if (!wf_fused(S) || !carry) return hipErrorInvalidValue;
    // passes of one chunk run back to back (integrator.cpp:350-360): pass p
    // writes its samples at p * n of every plane and hands each lane's PCG32
    // state to pass p + 1 through `carry`; counters per pass; the bounce
    // launches of all passes are timed as one span
    if (trace_ev) (void)hipEventRecord(trace_ev[0], st);
    for (uint32_t p = 0; p < n_passes; ++p) {
        hipError_t e = launch_wavefront_pass(S, in, lm, seed_value, n, plane, out + (uint64_t)p * n, ws, cap,
                                             ctr + (size_t)p * wf_counter_words(n_bounces), n_bounces, grid,
                                             nullptr, st, carry, p, alpha);
        if (e != hipSuccess) return e;
    }
    if (trace_ev) (void)hipEventRecord(trace_ev[1], st);  // one span (wf_trace_pairs)
    return hipSuccess;
}

static hipError_t launch_wavefront_pass(const DScene &S, const IntegratorParams &in, const LaneMap &lm,
                                        uint32_t seed_value, uint64_t n, uint64_t plane, float *out, void *ws,
                                        uint64_t cap, uint32_t *ctr, uint32_t n_bounces, uint32_t grid,
                                        hipEvent_t *trace_ev, hipStream_t st, uint64_t *carry, uint32_t pass,
                                        int alpha) {
    const bool fused = wf_fused(S);
    WfState w = carve(ws, cap);
    const WfPacked pk = carve_packed(ws, nullptr, cap);
    hipError_t e = hipMemsetAsync(ctr, 0, sizeof(uint32_t) * kCtrStride * (n_bounces + 1), st);
    if (e != hipSuccess) return e;
    const bool lds = S.lds_bytes_bvh != 0, packet = use_packet(S);
    const size_t sh = packet ? lds_bytes(S, 256) : stream_lds_bytes(S, 256);
    const uint32_t seg_cap = seg_len(n);
    grid = std::max<uint32_t>(kSeg, grid / kSeg * kSeg);  // whole number of blocks per segment
    if (S.stack_ovf && (uint64_t)grid * 256 > S.ovf_threads) return hipErrorInvalidValue;  // overflow columns
    if (!fused)  // the fused first bounce generates its camera rays itself
        hipLaunchKernelGGL(k_wf_raygen, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, S, lm,
                           seed_value, n, plane, out, w, ctr);
    for (uint32_t b = 0; b < n_bounces; ++b) {
        uint32_t *c = ctr + kCtrStride * b, *cn = ctr + kCtrStride * (b + 1);
        const int cur = (int)(b & 1);
        if (fused) {
            // timed as one span: an event between two launches costs a ~5-10 us
            // gap (measured), so bounce 0 opens the span and the last bounce
            // closes it (wf_trace_pairs: the host reads that one pair; the
            // round-3 build recorded the other 2 n_bounces - 2 events empty
            // after it, ~75 us of idle GPU per chunk)
            if (trace_ev && b == 0) (void)hipEventRecord(trace_ev[0], st);
            const uint32_t gd = grid;
            if (b == 0)
                hipLaunchKernelGGL(k_wf_bounce<true>, dim3(gd), dim3(256), fused_lds_bytes(S), st, S,
                                   in, lm, seed_value, plane, out, pk, cur, seg_cap, c, cn, n, carry, pass, alpha);
            else
                hipLaunchKernelGGL(k_wf_bounce<false>, dim3(gd), dim3(256), fused_lds_bytes(S), st,
                                   S, in, lm, seed_value, plane, out, pk, cur, seg_cap, c, cn, n, carry, pass, alpha);
            if (trace_ev && b + 1 == n_bounces) (void)hipEventRecord(trace_ev[1], st);
            continue;
        }
        if (trace_ev) (void)hipEventRecord(trace_ev[2 * b], st);
        MH_WF_DISPATCH(k_wf_trace, S, w, cur, seg_cap, c);
        if (trace_ev) (void)hipEventRecord(trace_ev[2 * b + 1], st);
        if (S.tab_bytes)
            hipLaunchKernelGGL(k_wf_shade<true>, dim3(grid), dim3(256), S.tab_bytes, st, S, in, lm, seed_value,
                               plane, out, w, cur, seg_cap, c, cn, alpha);
        else
            hipLaunchKernelGGL(k_wf_shade<false>, dim3(grid), dim3(256), 0, st, S, in, lm, seed_value, plane, out,
                               w, cur, seg_cap, c, cn, alpha);
        MH_WF_DISPATCH(k_wf_shadow, S, w, plane, out, seg_cap, c);
    }
    return hipGetLastError();
}

// ===========================================================================
// Wavefront PRB gradient (rgb parameters): RBIntegrator.render_backward
// (common.py:828-983) in the single-traversal form of prb_fused
// (mh_shading.hpp).  Extra per-path state: dL (gathered at raygen) and the
// running adjoint factors A_s; a shadow record carries the gradient it
// contributes if unoccluded (dL e_j A_s / pi plus the direct-term adjoint of
// its own slot).  Gradients accumulate in per-thread registers across a
// kernel's items and are folded once per kernel into a per-block partial
// (plain read-modify-write: one block per index per launch, launches are
// stream-ordered), so no same-address atomics; k_wf_grad_reduce sums the
// partials in a fixed order (deterministic).
// ===========================================================================
constexpr int kG = kMaxRgbParams * 3;

// planes addressed arithmetically (base + plane * stride): a runtime-indexed
// pointer table in the kernel arguments would be copied to scratch
struct WfPrb {
    float *base;
    uint64_t stride;  // floats between planes
    float *partial;   // [grid][kG]
    const int32_t *slot_of_tex;
    uint32_t n_rgb;
    // ping-pong k: planes [k * (3 + kG), (k + 1) * (3 + kG)): dL xyz, then A
    MH_DEV float *dl(int k, int c) const { return base + (uint64_t)(k * (3 + kG) + c) * stride; }
    MH_DEV float *A(int k, int c) const { return base + (uint64_t)(k * (3 + kG) + 3 + c) * stride; }
    MH_DEV float *G(int c) const { return base + (uint64_t)(2 * (3 + kG) + c) * stride; }
    // ping-pong k: the TEA word behind the path's PCG32 increment
    // (inc = (v1 << 1) | 1, sampler.cpp:128-132): one 4-B load instead of
    // re-running TEA (64 integer ops) and the lane map every bounce
    MH_DEV uint32_t *tea(int k) const {
        return reinterpret_cast<uint32_t *>(base + (uint64_t)(2 * (3 + kG) + kG + k) * stride);
    }
};

size_t wf_prb_workspace_bytes(uint64_t cap) {
    cap = (cap + kSeg - 1) / kSeg * kSeg;
    return (size_t)(6 + 2 * kG + kG + 2) * align_up(cap * 4);
}

static WfPrb carve_prb(void *ws, uint64_t cap, float *partial, const int32_t *slot_of_tex, uint32_t n_rgb) {
    cap = (cap + kSeg - 1) / kSeg * kSeg;
    WfPrb q;
    q.base = reinterpret_cast<float *>(ws);
    q.stride = align_up(cap * 4) / 4;
    q.partial = partial;
    q.slot_of_tex = slot_of_tex;
    q.n_rgb = n_rgb;
    return q;
}

// MH_FLAG_DETERMINISTIC (the ordered-reduction build of SURVEY.md §5) for
// the rgb gradient slots: a thread's register accumulator sums whichever
// paths the queue compaction handed it, so its float sum depends on the
// wave-ballot order of the appends.  Instead each path carries its own sum
// (P, ping-pong planes by slot), writes it under its path id when it ends
// (fin), and k_wf_det_sum adds the fin planes in a fixed order: the gradient
// is then bit-reproducible from run to run.  Cost: 12 B per rgb slot more
// path state per bounce, and the fin planes.
struct WfDet {
    float *base = nullptr;
    uint64_t stride = 0;  // floats between planes
    MH_DEV float *P(int k, int c) const { return base + (uint64_t)(k * kG + c) * stride; }
    MH_DEV float *fin(int c) const { return base + (uint64_t)(2 * kG + c) * stride; }
    float *fin_host(int c) const { return base + (uint64_t)(2 * kG + c) * stride; }
    __host__ __device__ float *blocks() const { return base + (uint64_t)(3 * kG) * stride; }  // [kDetBlocks][kG]
};
constexpr uint32_t kDetBlocks = 1024;

size_t wf_det_workspace_bytes(uint64_t cap) {
    cap = (cap + kSeg - 1) / kSeg * kSeg;
    return (size_t)3 * kG * align_up(cap * 4) + (size_t)kDetBlocks * kG * 4;
}

static WfDet carve_det(void *ws, uint64_t cap) {
    cap = (cap + kSeg - 1) / kSeg * kSeg;
    WfDet d;
    d.base = reinterpret_cast<float *>(ws);
    d.stride = align_up(cap * 4) / 4;
    return d;
}

// block b sums the path ids [b * per, (b + 1) * per) of every fin plane: its
// threads in a fixed strided order, then a fixed tree
__global__ void __launch_bounds__(256) k_wf_det_sum(WfDet d, uint32_t m, uint32_t n_c) {
    __shared__ float red[256];
    const uint32_t per = (m + kDetBlocks - 1) / kDetBlocks;
    const uint32_t b0 = blockIdx.x * per, b1 = std::min<uint32_t>(m, b0 + per);
    for (uint32_t c = 0; c < n_c; ++c) {
        float s = 0.f;
        for (uint32_t i = b0 + threadIdx.x; i < b1; i += 256u) s += d.fin(c)[i];
        red[threadIdx.x] = s;
        __syncthreads();
        for (uint32_t o = 128; o > 0; o >>= 1) {
            if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
            __syncthreads();
        }
        if (threadIdx.x == 0) d.blocks()[(size_t)blockIdx.x * kG + c] = red[0];
        __syncthreads();
    }
}

// the block sums in block order, added into the first block partial (which
// k_wf_grad_reduce sums in a fixed order with the others)
__global__ void k_wf_det_fold(WfDet d, uint32_t n_c, float *partial) {
    const uint32_t c = threadIdx.x;
    if (c >= n_c) return;
    float s = 0.f;
    for (uint32_t b = 0; b < kDetBlocks; ++b) s += d.blocks()[(size_t)b * kG + c];
    partial[c] += s;
}

// block-reduce the per-thread accumulators into partial[blockIdx]
template <int NR>
MH_DEV void flush_partial(float (&acc)[NR][3], const WfPrb &q) {
    __shared__ float red[4][kG];
    const uint32_t wave = threadIdx.x >> 6;
#pragma unroll
    for (int kk = 0; kk < NR; ++kk) {
        if ((uint32_t)kk >= q.n_rgb) break;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            float v = acc[kk][c];
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
            if (lane_id() == 0) red[wave][kk * 3 + c] = v;
        }
    }
    __syncthreads();
    const uint32_t t = threadIdx.x;
    if (t < q.n_rgb * 3) {
        float s = 0.f;
        for (uint32_t w = 0; w < blockDim.x / 64u; ++w) s += red[w][t];
        q.partial[(size_t)blockIdx.x * kG + t] += s;
    }
}

__global__ void __launch_bounds__(256)
k_wf_raygen_prb(DScene S, LaneMap lm, uint32_t seed_value, uint64_t n, int coalesce,
                const float *__restrict__ grad_in, const float *__restrict__ weights, WfState w,
                WfPrb q, uint32_t *ctr) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < kSeg) {
        const uint64_t L = seg_len(n), b = k * L;
        ctr[k * 32] = b >= n ? 0u : (uint32_t)std::min<uint64_t>(L, n - b);
    }
    if (k >= n) return;
    uint32_t lane, px, py;
    lane_of(lm, k, lane, px, py);
    Pcg rng;
    rng.seed(seed_value, lane);
    float sx = (float)px + rng.next_float(), sy = (float)py + rng.next_float();
    RayT r = camera_ray(S, __builtin_fmaf(sx, S.inv_width, -0.f),
                        __builtin_fmaf(sy, S.inv_height, -0.f));
    V3 dL = gather_dL(S, coalesce, grad_in, sx, sy);  // grad_in: pre-divided by W
    w.pd[0][k] = (uint32_t)k;
    w.ox[0][k] = r.o.x; w.oy[0][k] = r.o.y; w.oz[0][k] = r.o.z;
    w.dx[0][k] = r.d.x; w.dy[0][k] = r.d.y; w.dz[0][k] = r.d.z; w.mt[0][k] = r.maxt;
    w.bx[0][k] = 1.f; w.by[0][k] = 1.f; w.bz[0][k] = 1.f;
    w.ppx[0][k] = 0.f; w.ppy[0][k] = 0.f; w.ppz[0][k] = 0.f; w.ppdf[0][k] = 1.f;
    w.rng[0][k] = rng.state;
    q.dl(0, 0)[k] = dL.x; q.dl(0, 1)[k] = dL.y; q.dl(0, 2)[k] = dL.z;
#pragma unroll
    for (int c = 0; c < kG; ++c)
        if ((uint32_t)c < q.n_rgb * 3) q.A(0, c)[k] = 0.f;
}

// one iteration of the prb_fused loop (prb.py:114-278) for every queued path
// NR: rgb slot arrays (1 when a single rgb parameter is differentiated)
template <bool Staged, int NR>
__global__ void __launch_bounds__(256, 5)
k_wf_shade_prb(DScene S0, IntegratorParams in, LaneMap lm, uint32_t seed_value, WfState w, WfPrb q,
               int cur, uint32_t seg_cap, uint32_t *ctr, uint32_t *ctr_next) {
    extern __shared__ uint4 lds[];
    const SegIter it = seg_iter();
    const uint32_t n = __hip_atomic_load(ctr + it.seg * 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!block_has_stride_work(it, n)) return;
    const DScene S = Staged ? stage_tables(S0, lds) : S0;
    const uint32_t sbase = it.seg * seg_cap;
    const int nxt = cur ^ 1;
    const uint32_t n_rgb = q.n_rgb;
    float acc[NR][3];
#pragma unroll
    for (int kk = 0; kk < NR; ++kk) acc[kk][0] = acc[kk][1] = acc[kk][2] = 0.f;
    const uint32_t n_iter = (n + it.nwaves * 64u - 1) / (it.nwaves * 64u);  // wave-uniform
    for (uint32_t itr = 0; itr < n_iter; ++itr) {
        const uint32_t i = (itr * it.nwaves + it.wave) * 64u + lane_id();
        bool alive = false, shadow = false;
        uint32_t pid = 0, depth = 0;
        RayT ray, sray;
        V3 beta, prev_p, dL;
        float prev_pdf = 1.f;
        float A[NR][3], G[NR][3];
        Pcg rng;
        if (i < n) {
            const uint32_t j = sbase + i;
            const uint32_t pd = w.pd[cur][j];
            pid = pd & kPidMask;
            depth = pd >> kPidBits;
            ray.o = v3(w.ox[cur][j], w.oy[cur][j], w.oz[cur][j]);
            ray.d = v3(w.dx[cur][j], w.dy[cur][j], w.dz[cur][j]);
            ray.maxt = w.mt[cur][j];
            Hit h;
            h.t = w.ht[j]; h.u = w.hu[j]; h.v = w.hv[j]; h.prim = w.hp[j]; h.shape = w.hs[j];
            beta = v3(w.bx[cur][j], w.by[cur][j], w.bz[cur][j]);
            prev_p = v3(w.ppx[cur][j], w.ppy[cur][j], w.ppz[cur][j]);
            prev_pdf = w.ppdf[cur][j];
            dL = v3(q.dl(cur, 0)[j], q.dl(cur, 1)[j], q.dl(cur, 2)[j]);
#pragma unroll
            for (int kk = 0; kk < NR; ++kk)
#pragma unroll
                for (int c = 0; c < 3; ++c) A[kk][c] = (uint32_t)kk < n_rgb ? q.A(cur, kk * 3 + c)[j] : 0.f;
            const bool prev_delta = depth == 0;  // diffuse / null BSDFs: only the camera vertex is delta
            const float eta = 1.f;
            uint32_t lane, px, py;
            lane_of(lm, pid, lane, px, py);
            rng.state = w.rng[cur][j];
            rng.inc = pcg_inc(seed_value, lane);
            SI si;
            compute_si(S, ray, h, si);
            const uint32_t b = si.valid ? S.shapes[si.shape].bsdf : MH_INVALID;
            const bool smooth = b != MH_INVALID && S.bsdf_type[b] == MH_BSDF_DIFFUSE;
            bool active_next = !(in.hide_emitters && depth == 0 && !si.valid);

            // ---- emission (prb.py:143-152): charged to the earlier vertices
            const uint32_t em = si.valid ? S.shapes[si.shape].emitter : S.environment;
            if (em != MH_INVALID) {
                float em_pdf = prev_delta ? 0.f : emitter_pdf_direction(S, em, si, prev_p);
                float mis = mis_weight(prev_pdf, em_pdf);
                V3 le = v3(0, 0, 0);
                if (active_next)
                    le = emitter_eval(S, em, si);
                charge(acc, A, n_rgb, dL * ((beta * mis) * le));
            }
            active_next = active_next && (depth + 1 < in.max_depth) && si.valid;
            const bool active_em0 = active_next && smooth;

            // ---- emitter sampling (prb.py:157-176); visibility deferred
            float e0 = rng.next_float(), e1 = rng.next_float();
            DirS ds;
            ds.pdf = 0.f;
            ds.d = v3(0, 0, 0);
            ds.delta = false;
            V3 em_weight = v3(0, 0, 0);
            if (active_em0) {
                em_weight = scene_sample_emitter_direction(S, si.p, e0, e1, ds);
                if (ds.pdf != 0.f && nonzero(em_weight)) {
                    shadow = true;
                    sray = spawn_ray_to(si.p, si.n, ds.p);
                }
            }
            V3 rho = v3(0, 0, 0);
            if (smooth) rho = tex_eval(S, S.bsdf_tex[b], si.uvx, si.uvy);
            const int32_t slot = smooth ? q.slot_of_tex[S.bsdf_tex[b]] : -1;
            if (shadow) {  // as if unoccluded; applied by k_wf_shadow_prb
                V3 wo_em = to_local(si, ds.d);
                V3 bsdf_value_em;
                float bsdf_pdf_em;
                diffuse_eval_pdf(rho, si.wi, wo_em, true, bsdf_value_em, bsdf_pdf_em);
                float mis_em = ds.delta ? 1.f : mis_weight(ds.pdf, bsdf_pdf_em);
                V3 beta_mis_em = beta * mis_em;
                V3 dLe = dL * ((beta_mis_em * bsdf_value_em) * em_weight);
#pragma unroll
                for (int kk = 0; kk < NR; ++kk) {
                    G[kk][0] = (dLe.x * (A[kk][0] * kInvPi));
                    G[kk][1] = (dLe.y * (A[kk][1] * kInvPi));
                    G[kk][2] = (dLe.z * (A[kk][2] * kInvPi));
                }
                if (slot >= 0 && si.wi.z > 0.f && wo_em.z > 0.f)
                    add_slot(G, slot, (((dL * em_weight) * beta_mis_em) * wo_em.z) * kInvPi);
            }

            // ---- BSDF sampling, RR (prb.py:181-278)
            (void)rng.next_float();
            float s2x = rng.next_float(), s2y = rng.next_float();
            V3 bs_wo = v3(0, 0, 0), bsdf_weight = v3(0, 0, 0);
            float bs_pdf = 0.f;
            if (smooth && active_next) {
                bs_wo = square_to_cosine_hemisphere(s2x, s2y);
                bs_pdf = kInvPi * bs_wo.z;
                bsdf_weight = (si.wi.z > 0.f && bs_pdf > 0.f) ? rho : v3(0, 0, 0);
            }
            ray = spawn_ray(si.p, si.n, to_world(si, bs_wo));
            beta = beta * bsdf_weight;
            prev_p = si.p;
            prev_pdf = bs_pdf;
            float beta_max = hmax(beta);
            active_next = active_next && beta_max != 0.f;
            float rr_prob = fminf(beta_max * (eta * eta), 0.95f);
            bool rr_active = depth >= in.rr_depth;
            if (rr_active) beta = beta * rcp(rr_prob);
            bool rr_continue = rng.next_float() < rr_prob;
            active_next = active_next && (!rr_active || rr_continue);
            if (slot >= 0)
                add_slot(A, slot, prb_indirect_factor(active_next, si, to_local(si, ray.d), bsdf_weight, bs_pdf));
            if (si.valid) depth += 1;
            alive = active_next;
        }
        const uint32_t slot_n = sbase + wave_append(ctr_next + it.seg * 32, alive);
        const uint32_t sslot = sbase + wave_append(ctr + it.seg * 32 + 1, shadow);
        if (alive) {
            w.pd[nxt][slot_n] = pid | (depth << kPidBits);
            w.ox[nxt][slot_n] = ray.o.x; w.oy[nxt][slot_n] = ray.o.y; w.oz[nxt][slot_n] = ray.o.z;
            w.dx[nxt][slot_n] = ray.d.x; w.dy[nxt][slot_n] = ray.d.y; w.dz[nxt][slot_n] = ray.d.z;
            w.mt[nxt][slot_n] = ray.maxt;
            w.bx[nxt][slot_n] = beta.x; w.by[nxt][slot_n] = beta.y; w.bz[nxt][slot_n] = beta.z;
            w.ppx[nxt][slot_n] = prev_p.x; w.ppy[nxt][slot_n] = prev_p.y; w.ppz[nxt][slot_n] = prev_p.z;
            w.ppdf[nxt][slot_n] = prev_pdf;
            w.rng[nxt][slot_n] = rng.state;
            q.dl(nxt, 0)[slot_n] = dL.x; q.dl(nxt, 1)[slot_n] = dL.y; q.dl(nxt, 2)[slot_n] = dL.z;
#pragma unroll
            for (int kk = 0; kk < NR; ++kk)
                if ((uint32_t)kk < n_rgb) {
                    q.A(nxt, kk * 3 + 0)[slot_n] = A[kk][0];
                    q.A(nxt, kk * 3 + 1)[slot_n] = A[kk][1];
                    q.A(nxt, kk * 3 + 2)[slot_n] = A[kk][2];
                }
        }
        if (shadow) {
            w.sox[sslot] = sray.o.x; w.soy[sslot] = sray.o.y; w.soz[sslot] = sray.o.z;
            w.sdx[sslot] = sray.d.x; w.sdy[sslot] = sray.d.y; w.sdz[sslot] = sray.d.z; w.smt[sslot] = sray.maxt;
#pragma unroll
            for (int kk = 0; kk < NR; ++kk)
                if ((uint32_t)kk < n_rgb) {
                    q.G(kk * 3 + 0)[sslot] = G[kk][0];
                    q.G(kk * 3 + 1)[sslot] = G[kk][1];
                    q.G(kk * 3 + 2)[sslot] = G[kk][2];
                }
        }
    }
    flush_partial(acc, q);
}

// Fused PRB bounce kernel (small scenes): closest-hit packet trace + one
// iteration of the prb_fused loop + the NEE packet visibility test, whose
// gradient record is charged at once (same operations and order as
// k_wf_trace -> k_wf_shade_prb -> k_wf_shadow_prb; only the order in which
// the per-thread gradient registers accumulate differs).
// First-bounce generation for the fused PRB bounce (k_wf_raygen_prb in
// registers): camera ray, PCG32 state and the dL gather of the sample.
struct PrbGen {
    uint64_t n_total;          // paths of the chunk (0: not the first bounce)
    const float *grad_in;      // grad_in / W (common.py:936-965)
    int coalesce;
};

// ---------------------------------------------------------------------------
// A bitmap parameter on the fused wavefront (Bm).  Its texels differ from
// vertex to vertex, so the A_s regrouping of the rgb slots does not apply;
// the replay's adjoint at a bitmap vertex k (prb.py:203-248),
//     adj_k = D_k + dL (L_total - P_k) q_k / pi,
// D_k = the NEE term (dL em_weight beta mis cos / pi, zero when occluded),
// q_k = cos / (rho pdf) of the sampled direction, P_k = the primal radiance
// through vertex k (Le and Lr_dir included, as prb.py's `L - Le - Lr_dir`),
// needs L_total, known only when the path ends.  The bounce kernel carries the
// running radiance L, logs (P_k, uv) (q_k) (D_k) per bitmap vertex under the
// path id, and writes (L_total, depth mask) (dL) when the path ends; after the
// chunk's last bounce k_wf_bitmap_scatter turns the records into texel
// gradients (bilinear taps of bitmap.cpp, per-workgroup LDS accumulator).
// ---------------------------------------------------------------------------
struct WfBmp {
    float4 *fin;         // [2][stride]: (L_total, mask as bits), (dL, 0) per path id
    float4 *rec;         // [n_depth][3][stride]: (P, uvx), (q, uvy), (D, 0) per path id
    uint32_t *mask[2];   // per queue slot, ping-pong: depths holding a record
    uint64_t stride;     // float4 per plane
    uint32_t n_depth;
    int32_t slot;        // gradient slot of the bitmap (-1: no bitmap on this launch)
    MH_DEV float4 *r(uint32_t d, uint32_t k) const { return rec + (uint64_t)(d * 3u + k) * stride; }
};

size_t wf_bmp_workspace_bytes(uint64_t cap, uint32_t n_depth) {
    cap = (cap + kSeg - 1) / kSeg * kSeg;
    return (size_t)(2 + 3 * n_depth) * align_up(cap * 16) + 2 * align_up(cap * 4);
}

static WfBmp carve_bmp(void *ws, uint64_t cap, uint32_t n_depth, int32_t slot) {
    cap = (cap + kSeg - 1) / kSeg * kSeg;
    WfBmp b;
    b.stride = align_up(cap * 16) / 16;
    b.fin = reinterpret_cast<float4 *>(ws);
    b.rec = b.fin + 2 * b.stride;
    uint8_t *m = reinterpret_cast<uint8_t *>(b.rec + (uint64_t)3 * n_depth * b.stride);
    b.mask[0] = reinterpret_cast<uint32_t *>(m);
    b.mask[1] = reinterpret_cast<uint32_t *>(m + align_up(cap * 4));
    b.n_depth = n_depth;
    b.slot = slot;
    return b;
}

#ifndef MH_BOUNCE_BMP_WAVES
#define MH_BOUNCE_BMP_WAVES 4  // the Bm instance carries ~20 more live values across the shadow trace
#endif
template <int NR, bool Gen, bool Bm, bool Det>
__global__ void __launch_bounds__(256, Bm ? MH_BOUNCE_BMP_WAVES : MH_BOUNCE_PRB_WAVES)
k_wf_bounce_prb(DScene S0, IntegratorParams in, LaneMap lm, uint32_t seed_value, WfState w, WfPrb q,
                int cur, uint32_t seg_cap, uint32_t *ctr, uint32_t *ctr_next, PrbGen gen, WfBmp bm, WfDet det) {
    extern __shared__ uint4 lds[];
    const SegIter it = seg_iter();
    auto seg_count = [&](uint32_t sg) -> uint32_t {
        if (Gen) {
            const uint64_t b0 = (uint64_t)sg * seg_cap;
            return b0 >= gen.n_total ? 0u : (uint32_t)std::min<uint64_t>(seg_cap, gen.n_total - b0);
        }
        return __hip_atomic_load(ctr + sg * 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    const uint32_t n = seg_count(it.seg);
    if (Gen && blockIdx.x < kSeg && threadIdx.x == 0) ctr[it.seg * 32] = n;  // queue statistics
    if (!block_has_stride_work(it, n)) return;
    MH_BPH_DECL
    float *recs = reinterpret_cast<float *>(reinterpret_cast<uint8_t *>(lds) + fused_pairs_offset(S0));
    stage_pair_records(S0, recs);  // made visible by stage_tables' barrier
    const DScene S = stage_tables(S0, lds);
    uint32_t *ws = reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(lds) + S0.tab_bytes) +
                   (threadIdx.x >> 6) * S0.stack_size;
    uint8_t *dscr = reinterpret_cast<uint8_t *>(lds) + fused_scratch_offset(S0) + (threadIdx.x >> 6) * kDeferScratch;
    uint32_t n_shadow = 0;
    const int nxt = cur ^ 1;
    const uint32_t n_rgb = q.n_rgb;
    float acc[NR][3];
#pragma unroll
    for (int kk = 0; kk < NR; ++kk) acc[kk][0] = acc[kk][1] = acc[kk][2] = 0.f;
    MH_BPH(7);
    const uint32_t seg = it.seg;
    const uint32_t n_iter = (n + it.nwaves * 64u - 1) / (it.nwaves * 64u);  // wave-uniform
    for (uint32_t itr = 0; itr < n_iter; ++itr) {
        const uint32_t i = (itr * it.nwaves + it.wave) * 64u + lane_id();
        const uint32_t sbase = seg * seg_cap;
        MH_BPH_ITER();
        bool alive = false, shadow = false;
        uint32_t pid = 0, depth = 0;
        RayT ray{v3(0, 0, 0), v3(0, 0, 1), -1.f}, sray{v3(0, 0, 0), v3(0, 0, 1), -1.f};
        V3 beta, prev_p, dL;
        float prev_pdf = 1.f;
        float A[NR][3], G[NR][3];
        float Pp[NR][3];  // Det: this path's own gradient sum
#pragma unroll
        for (int kk = 0; kk < NR; ++kk) Pp[kk][0] = Pp[kk][1] = Pp[kk][2] = 0.f;
        Pcg rng;
        const uint32_t j = sbase + i;
        MH_GUARD(i >= n || i < seg_cap, kGuardQueueSlot);
        uint64_t gen_state = 0, gen_inc = 0;
        // Bm: running radiance, this vertex's Le / potential Lr_dir / record
        V3 Lrun = v3(0, 0, 0), Le_b = v3(0, 0, 0), Lr_pot = v3(0, 0, 0), D_pot = v3(0, 0, 0), q_ind = v3(0, 0, 0);
        float b_uvx = 0.f, b_uvy = 0.f;
        uint32_t vmask = 0, depth_v = 0;
        bool bvtx = false;
        if (i < n) {
            if (Gen) {  // k_wf_raygen_prb (integrator.cpp:1139-1176, common.py:936-965)
                pid = j;
                uint32_t lane, px, py;
                lane_of(lm, pid, lane, px, py);
                MH_GUARD(px < S0.width && py < S0.height, kGuardPixel);
                Pcg g;
                g.seed(seed_value, lane);
                const float sx = (float)px + g.next_float(), sy = (float)py + g.next_float();
                ray = camera_ray(S0, __builtin_fmaf(sx, S0.inv_width, -0.f),
                                 __builtin_fmaf(sy, S0.inv_height, -0.f));
                gen_state = g.state;
                gen_inc = g.inc;  // the TEA of this lane, reused below
                dL = gather_dL_wave_lds(S0, gen.coalesce, gen.grad_in, sx, sy, dscr);
            } else {
                const uint32_t pd = w.pd[cur][j];
                pid = pd & kPidMask;
                depth = pd >> kPidBits;
                ray.o = v3(w.ox[cur][j], w.oy[cur][j], w.oz[cur][j]);
                ray.d = v3(w.dx[cur][j], w.dy[cur][j], w.dz[cur][j]);
                ray.maxt = w.mt[cur][j];
            }
            MH_GUARD(pid < gen.n_total, kGuardPathId);
        }
        MH_BPH(0);
        const Hit h = packet_batch<false, true>(S0.nodes, S0.prims, S0.prim_pairs, S0.key_sp, ws, 1u, ray, i < n, recs, dscr);
        MH_BPH(1);
        if (i < n) {
            if (Gen) {
                beta = v3(1.f, 1.f, 1.f);
                prev_p = v3(0.f, 0.f, 0.f);
                prev_pdf = 1.f;
#pragma unroll
                for (int kk = 0; kk < NR; ++kk) A[kk][0] = A[kk][1] = A[kk][2] = 0.f;
                rng.state = gen_state;
            } else {
                const uint32_t jl = j;
                beta = v3(w.bx[cur][jl], w.by[cur][jl], w.bz[cur][jl]);
                prev_p = v3(w.ppx[cur][jl], w.ppy[cur][jl], w.ppz[cur][jl]);
                prev_pdf = w.ppdf[cur][jl];
                dL = v3(q.dl(cur, 0)[jl], q.dl(cur, 1)[jl], q.dl(cur, 2)[jl]);
#pragma unroll
                for (int kk = 0; kk < NR; ++kk)
#pragma unroll
                    for (int c = 0; c < 3; ++c) A[kk][c] = (uint32_t)kk < n_rgb ? q.A(cur, kk * 3 + c)[jl] : 0.f;
                rng.state = w.rng[cur][jl];
                if (Det) {
#pragma unroll
                    for (int kk = 0; kk < NR; ++kk)
#pragma unroll
                        for (int c = 0; c < 3; ++c) Pp[kk][c] = (uint32_t)kk < n_rgb ? det.P(cur, kk * 3 + c)[j] : 0.f;
                }
                if (Bm) {
                    Lrun = v3(w.lx[cur][j], w.ly[cur][j], w.lz[cur][j]);
                    vmask = bm.mask[cur][j];
                }
            }
            const bool prev_delta = depth == 0;  // diffuse / null BSDFs: only the camera vertex is delta
            const float eta = 1.f;
            rng.inc = Gen ? gen_inc : (((uint64_t)q.tea(cur)[j] << 1) | 1u);
            SI si;
            compute_si(S, ray, h, si);
            const uint32_t b = si.valid ? S.shapes[si.shape].bsdf : MH_INVALID;
            const bool smooth = b != MH_INVALID && S.bsdf_type[b] == MH_BSDF_DIFFUSE;
            bool active_next = !(in.hide_emitters && depth == 0 && !si.valid);

            // ---- emission (prb.py:143-152): charged to the earlier vertices
            const uint32_t em = si.valid ? S.shapes[si.shape].emitter : S.environment;
            if (em != MH_INVALID) {
                float em_pdf = prev_delta ? 0.f : emitter_pdf_direction(S, em, si, prev_p);
                float mis = mis_weight(prev_pdf, em_pdf);
                V3 le = v3(0, 0, 0);
                if (active_next)
                    le = emitter_eval(S, em, si);
                const V3 Le = (beta * mis) * le;
                if (Det) charge(Pp, A, n_rgb, dL * Le);
                else charge(acc, A, n_rgb, dL * Le);
                if (Bm) Le_b = Le;
            }
            active_next = active_next && (depth + 1 < in.max_depth) && si.valid;
            const bool active_em0 = active_next && smooth;

            // ---- emitter sampling (prb.py:157-176); visibility deferred
            float e0 = rng.next_float(), e1 = rng.next_float();
            DirS ds;
            ds.pdf = 0.f;
            ds.d = v3(0, 0, 0);
            ds.delta = false;
            V3 em_weight = v3(0, 0, 0);
            if (active_em0) {
                em_weight = scene_sample_emitter_direction(S, si.p, e0, e1, ds);
                if (ds.pdf != 0.f && nonzero(em_weight)) {
                    shadow = true;
                    sray = spawn_ray_to(si.p, si.n, ds.p);
                }
            }
            V3 rho = v3(0, 0, 0);
            if (smooth) rho = tex_eval(S, S.bsdf_tex[b], si.uvx, si.uvy);
            const int32_t slot = smooth ? q.slot_of_tex[S.bsdf_tex[b]] : -1;
            if (Bm) {
                // every bitmap slot (kMaxRgbParams + b) records; b rides in depth_v's bits 8+
                bvtx = slot >= (int32_t)kMaxRgbParams && depth < bm.n_depth;
                depth_v = depth | (bvtx ? (uint32_t)(slot - (int32_t)kMaxRgbParams) << 8 : 0u);
                b_uvx = si.uvx;
                b_uvy = si.uvy;
            }
            if (shadow) {  // as if unoccluded; applied after the visibility test
                V3 wo_em = to_local(si, ds.d);
                V3 bsdf_value_em;
                float bsdf_pdf_em;
                diffuse_eval_pdf(rho, si.wi, wo_em, true, bsdf_value_em, bsdf_pdf_em);
                float mis_em = ds.delta ? 1.f : mis_weight(ds.pdf, bsdf_pdf_em);
                V3 beta_mis_em = beta * mis_em;
                const V3 Lr = (beta_mis_em * bsdf_value_em) * em_weight;
                V3 dLe = dL * Lr;
#pragma unroll
                for (int kk = 0; kk < NR; ++kk) {
                    G[kk][0] = (dLe.x * (A[kk][0] * kInvPi));
                    G[kk][1] = (dLe.y * (A[kk][1] * kInvPi));
                    G[kk][2] = (dLe.z * (A[kk][2] * kInvPi));
                }
                if (slot >= 0 && si.wi.z > 0.f && wo_em.z > 0.f)
                    add_slot(G, slot, (((dL * em_weight) * beta_mis_em) * wo_em.z) * kInvPi);
                if (Bm) {
                    Lr_pot = Lr;
                    if (bvtx && si.wi.z > 0.f && wo_em.z > 0.f)
                        D_pot = (((dL * em_weight) * beta_mis_em) * wo_em.z) * kInvPi;
                }
            }

            // ---- BSDF sampling, RR (prb.py:181-278)
            (void)rng.next_float();
            float s2x = rng.next_float(), s2y = rng.next_float();
            V3 bs_wo = v3(0, 0, 0), bsdf_weight = v3(0, 0, 0);
            float bs_pdf = 0.f;
            if (smooth && active_next) {
                bs_wo = square_to_cosine_hemisphere(s2x, s2y);
                bs_pdf = kInvPi * bs_wo.z;
                bsdf_weight = (si.wi.z > 0.f && bs_pdf > 0.f) ? rho : v3(0, 0, 0);
            }
            ray = spawn_ray(si.p, si.n, to_world(si, bs_wo));
            beta = beta * bsdf_weight;
            prev_p = si.p;
            prev_pdf = bs_pdf;
            float beta_max = hmax(beta);
            active_next = active_next && beta_max != 0.f;
            float rr_prob = fminf(beta_max * (eta * eta), 0.95f);
            bool rr_active = depth >= in.rr_depth;
            if (rr_active) beta = beta * rcp(rr_prob);
            bool rr_continue = rng.next_float() < rr_prob;
            active_next = active_next && (!rr_active || rr_continue);
            if (slot >= 0) {
                const V3 c = prb_indirect_factor(active_next, si, to_local(si, ray.d), bsdf_weight, bs_pdf);
                add_slot(A, slot, c);
                if (Bm && bvtx) q_ind = c;
            }
            if (si.valid) depth += 1;
            alive = active_next;
        }
        MH_BPH(2);
        const uint32_t slot_n = sbase + wave_append(ctr_next + seg * 32, alive);
        MH_GUARD(!alive || slot_n - sbase < seg_cap, kGuardAppendSlot);
        if (alive) {
            w.pd[nxt][slot_n] = pid | (depth << kPidBits);
            w.ox[nxt][slot_n] = ray.o.x; w.oy[nxt][slot_n] = ray.o.y; w.oz[nxt][slot_n] = ray.o.z;
            w.dx[nxt][slot_n] = ray.d.x; w.dy[nxt][slot_n] = ray.d.y; w.dz[nxt][slot_n] = ray.d.z;
            w.mt[nxt][slot_n] = ray.maxt;
            w.bx[nxt][slot_n] = beta.x; w.by[nxt][slot_n] = beta.y; w.bz[nxt][slot_n] = beta.z;
            w.ppx[nxt][slot_n] = prev_p.x; w.ppy[nxt][slot_n] = prev_p.y; w.ppz[nxt][slot_n] = prev_p.z;
            w.ppdf[nxt][slot_n] = prev_pdf;
            w.rng[nxt][slot_n] = rng.state;
            q.tea(nxt)[slot_n] = (uint32_t)(rng.inc >> 1);
            q.dl(nxt, 0)[slot_n] = dL.x; q.dl(nxt, 1)[slot_n] = dL.y; q.dl(nxt, 2)[slot_n] = dL.z;
#pragma unroll
            for (int kk = 0; kk < NR; ++kk)
                if ((uint32_t)kk < n_rgb) {
                    q.A(nxt, kk * 3 + 0)[slot_n] = A[kk][0];
                    q.A(nxt, kk * 3 + 1)[slot_n] = A[kk][1];
                    q.A(nxt, kk * 3 + 2)[slot_n] = A[kk][2];
                }
        }
        // ---- visibility of the NEE sample; the record is charged if unoccluded
        MH_BPH(3);
        const Hit sh = packet_batch<true, true, Gen>(S0.nodes, S0.prims, S0.prim_pairs, S0.key_sp, ws, 1u, sray, shadow, recs, dscr);
        MH_BPH(4);
        const bool unocc = shadow && sh.shape == MH_INVALID;
        if (unocc) {
            float (&ga)[NR][3] = Det ? Pp : acc;
#pragma unroll
            for (int kk = 0; kk < NR; ++kk)
                if ((uint32_t)kk < n_rgb) {
                    ga[kk][0] += G[kk][0];
                    ga[kk][1] += G[kk][1];
                    ga[kk][2] += G[kk][2];
                }
        }
        if (Det && i < n) {  // the path's sum travels with it, or lands under its id when it ends
#pragma unroll
            for (int kk = 0; kk < NR; ++kk)
                if ((uint32_t)kk < n_rgb)
#pragma unroll
                    for (int c = 0; c < 3; ++c) {
                        if (alive) det.P(nxt, kk * 3 + c)[slot_n] = Pp[kk][c];
                        else det.fin(kk * 3 + c)[pid] = Pp[kk][c];
                    }
        }
        if (Bm && i < n) {
            // primal state update L = (L + Le) + Lr_dir (prb.py:174-199), then the vertex record
            Lrun = (Lrun + Le_b) + (unocc ? Lr_pot : v3(0, 0, 0));
            const V3 D = unocc ? D_pot : v3(0, 0, 0);
            if (bvtx && (nonzero(q_ind) || nonzero(D))) {
                const uint32_t dv = depth_v & 0xffu;
                bm.r(dv, 0)[pid] = make_float4(Lrun.x, Lrun.y, Lrun.z, b_uvx);
                bm.r(dv, 1)[pid] = make_float4(q_ind.x, q_ind.y, q_ind.z, b_uvy);
                bm.r(dv, 2)[pid] = make_float4(D.x, D.y, D.z, __uint_as_float(depth_v >> 8));
                vmask |= 1u << dv;
            }
            if (alive) {
                w.lx[nxt][slot_n] = Lrun.x; w.ly[nxt][slot_n] = Lrun.y; w.lz[nxt][slot_n] = Lrun.z;
                bm.mask[nxt][slot_n] = vmask;
            } else {  // the path ends: L_total and the record mask under its id
                bm.fin[pid] = make_float4(Lrun.x, Lrun.y, Lrun.z, __uint_as_float(vmask));
                if (vmask) bm.fin[bm.stride + pid] = make_float4(dL.x, dL.y, dL.z, 0.f);
            }
        }
        n_shadow += (uint32_t)__popcll(__ballot(shadow));
        MH_BPH(5);
    }
    if (lane_id() == 0 && n_shadow) atomicAdd(ctr + it.seg * 32 + 1, n_shadow);  // statistics only
    flush_partial(acc, q);
    if (!Bm && !Det) MH_BPH_FLUSH(Gen ? 2 : 3);
}

// ---------------------------------------------------------------------------
// Forward-mode PRB on the fused wavefront (render_forward, common.py:696-826):
// prb_forward (mh_shading.hpp) as bounce kernels.  Per path the dL planes of
// WfPrb carry the tangent radiance and the first three A planes the tangent
// sum T = sum c_k t_k; a contribution e_j adds e_j T / pi, an unoccluded NEE
// sample also its direct term (em_weight beta mis cos / pi) t_k, and a path
// that ends writes dL to the sample planes of the film splat (L, pos, alpha:
// the layout of k_wf_bounce), which the generating bounce fills with pos.
// Tangents: the slot table and tangent arrays of a GradArgs (GradCtx::fwd).
// ---------------------------------------------------------------------------
struct WfFwdOut {
    float *out;          // sample planes: L.r L.g L.b pos.x pos.y [alpha]
    uint64_t plane;      // floats between planes
    int alpha;
    const int32_t *slot_of_tex;
    float *const *tan;   // per slot: tangent values (rgb: 3, bitmap: the texels)
    const uint32_t *is_rgb;
};

template <bool Gen>
__global__ void __launch_bounds__(256, MH_BOUNCE_PRB_WAVES)
k_wf_bounce_fwd(DScene S0, IntegratorParams in, LaneMap lm, uint32_t seed_value, WfState w, WfPrb q, int cur,
                uint32_t seg_cap, uint32_t *ctr, uint32_t *ctr_next, uint64_t n_total, WfFwdOut fo) {
    extern __shared__ uint4 lds[];
    const SegIter it = seg_iter();
    uint32_t n;
    if (Gen) {
        const uint64_t b0 = (uint64_t)it.seg * seg_cap;
        n = b0 >= n_total ? 0u : (uint32_t)std::min<uint64_t>(seg_cap, n_total - b0);
        if (blockIdx.x < kSeg && threadIdx.x == 0) ctr[it.seg * 32] = n;  // queue statistics
    } else {
        n = __hip_atomic_load(ctr + it.seg * 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (!block_has_stride_work(it, n)) return;
    float *recs = reinterpret_cast<float *>(reinterpret_cast<uint8_t *>(lds) + fused_pairs_offset(S0));
    stage_pair_records(S0, recs);  // made visible by stage_tables' barrier
    const DScene S = stage_tables(S0, lds);
    uint32_t *ws = reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(lds) + S0.tab_bytes) +
                   (threadIdx.x >> 6) * S0.stack_size;
    uint8_t *dscr = reinterpret_cast<uint8_t *>(lds) + fused_scratch_offset(S0) + (threadIdx.x >> 6) * kDeferScratch;
    GradCtx tg;  // tangent lookups only (tex_tangent)
    tg.slot_of_tex = fo.slot_of_tex;
    tg.bufs = fo.tan;
    tg.is_rgb = fo.is_rgb;
    uint32_t n_shadow = 0;
    const uint32_t sbase = it.seg * seg_cap;
    const int nxt = cur ^ 1;
    const uint32_t n_iter = (n + it.nwaves * 64u - 1) / (it.nwaves * 64u);  // wave-uniform
    for (uint32_t itr = 0; itr < n_iter; ++itr) {
        const uint32_t i = (itr * it.nwaves + it.wave) * 64u + lane_id();
        bool alive = false, shadow = false;
        uint32_t pid = 0, depth = 0;
        RayT ray{v3(0, 0, 0), v3(0, 0, 1), -1.f}, sray{v3(0, 0, 0), v3(0, 0, 1), -1.f};
        V3 beta, prev_p, dL = v3(0, 0, 0), T = v3(0, 0, 0), G = v3(0, 0, 0);
        float prev_pdf = 1.f;
        Pcg rng;
        const uint32_t j = sbase + i;
        uint64_t gen_state = 0, gen_inc = 0;
        if (i < n) {
            if (Gen) {  // camera ray and PCG32 state (integrator.cpp:1139-1176)
                pid = j;
                uint32_t lane, px, py;
                lane_of(lm, pid, lane, px, py);
                Pcg g;
                g.seed(seed_value, lane);
                const float sx = (float)px + g.next_float(), sy = (float)py + g.next_float();
                ray = camera_ray(S0, __builtin_fmaf(sx, S0.inv_width, -0.f),
                                 __builtin_fmaf(sy, S0.inv_height, -0.f));
                gen_state = g.state;
                gen_inc = g.inc;
                fo.out[3 * fo.plane + pid] = sx;
                fo.out[4 * fo.plane + pid] = sy;
            } else {
                const uint32_t pd = w.pd[cur][j];
                pid = pd & kPidMask;
                depth = pd >> kPidBits;
                ray.o = v3(w.ox[cur][j], w.oy[cur][j], w.oz[cur][j]);
                ray.d = v3(w.dx[cur][j], w.dy[cur][j], w.dz[cur][j]);
                ray.maxt = w.mt[cur][j];
            }
        }
        const Hit h = packet_batch<false, true>(S0.nodes, S0.prims, S0.prim_pairs, S0.key_sp, ws, 1u, ray, i < n, recs, dscr);
        if (i < n) {
            if (Gen) {
                beta = v3(1.f, 1.f, 1.f);
                prev_p = v3(0.f, 0.f, 0.f);
                prev_pdf = 1.f;
                rng.state = gen_state;
            } else {
                beta = v3(w.bx[cur][j], w.by[cur][j], w.bz[cur][j]);
                prev_p = v3(w.ppx[cur][j], w.ppy[cur][j], w.ppz[cur][j]);
                prev_pdf = w.ppdf[cur][j];
                dL = v3(q.dl(cur, 0)[j], q.dl(cur, 1)[j], q.dl(cur, 2)[j]);
                T = v3(q.A(cur, 0)[j], q.A(cur, 1)[j], q.A(cur, 2)[j]);
                rng.state = w.rng[cur][j];
            }
            const bool prev_delta = depth == 0;
            const float eta = 1.f;
            rng.inc = Gen ? gen_inc : (((uint64_t)q.tea(cur)[j] << 1) | 1u);
            SI si;
            compute_si(S, ray, h, si);
            const uint32_t b = si.valid ? S.shapes[si.shape].bsdf : MH_INVALID;
            const bool smooth = b != MH_INVALID && S.bsdf_type[b] == MH_BSDF_DIFFUSE;
            bool active_next = !(in.hide_emitters && depth == 0 && !si.valid);
            const uint32_t em = si.valid ? S.shapes[si.shape].emitter : S.environment;
            if (em != MH_INVALID) {
                float em_pdf = prev_delta ? 0.f : emitter_pdf_direction(S, em, si, prev_p);
                float mis = mis_weight(prev_pdf, em_pdf);
                V3 le = v3(0, 0, 0);
                if (active_next)
                    le = emitter_eval(S, em, si);
                dL = dL + ((beta * mis) * le) * (T * kInvPi);
            }
            active_next = active_next && (depth + 1 < in.max_depth) && si.valid;
            const bool active_em0 = active_next && smooth;
            float e0 = rng.next_float(), e1 = rng.next_float();
            DirS ds;
            ds.pdf = 0.f;
            ds.d = v3(0, 0, 0);
            ds.delta = false;
            V3 em_weight = v3(0, 0, 0);
            if (active_em0) {
                em_weight = scene_sample_emitter_direction(S, si.p, e0, e1, ds);
                if (ds.pdf != 0.f && nonzero(em_weight)) {
                    shadow = true;
                    sray = spawn_ray_to(si.p, si.n, ds.p);
                }
            }
            V3 rho = v3(0, 0, 0);
            if (smooth) rho = tex_eval(S, S.bsdf_tex[b], si.uvx, si.uvy);
            const bool tvtx = smooth && tg.slot_of_tex[S.bsdf_tex[b]] >= 0;
            const V3 t = tvtx ? tex_tangent(S, S.bsdf_tex[b], si.uvx, si.uvy, tg) : v3(0, 0, 0);
            if (shadow) {  // as if unoccluded; applied after the visibility test
                V3 wo_em = to_local(si, ds.d);
                V3 bsdf_value_em;
                float bsdf_pdf_em;
                diffuse_eval_pdf(rho, si.wi, wo_em, true, bsdf_value_em, bsdf_pdf_em);
                float mis_em = ds.delta ? 1.f : mis_weight(ds.pdf, bsdf_pdf_em);
                V3 beta_mis_em = beta * mis_em;
                G = ((beta_mis_em * bsdf_value_em) * em_weight) * (T * kInvPi);
                if (tvtx && si.wi.z > 0.f && wo_em.z > 0.f)
                    G = G + (((em_weight * beta_mis_em) * wo_em.z) * kInvPi) * t;
            }
            (void)rng.next_float();
            float s2x = rng.next_float(), s2y = rng.next_float();
            V3 bs_wo = v3(0, 0, 0), bsdf_weight = v3(0, 0, 0);
            float bs_pdf = 0.f;
            if (smooth && active_next) {
                bs_wo = square_to_cosine_hemisphere(s2x, s2y);
                bs_pdf = kInvPi * bs_wo.z;
                bsdf_weight = (si.wi.z > 0.f && bs_pdf > 0.f) ? rho : v3(0, 0, 0);
            }
            ray = spawn_ray(si.p, si.n, to_world(si, bs_wo));
            beta = beta * bsdf_weight;
            prev_p = si.p;
            prev_pdf = bs_pdf;
            float beta_max = hmax(beta);
            active_next = active_next && beta_max != 0.f;
            float rr_prob = fminf(beta_max * (eta * eta), 0.95f);
            bool rr_active = depth >= in.rr_depth;
            if (rr_active) beta = beta * rcp(rr_prob);
            bool rr_continue = rng.next_float() < rr_prob;
            active_next = active_next && (!rr_active || rr_continue);
            if (tvtx) T = T + prb_indirect_factor(active_next, si, to_local(si, ray.d), bsdf_weight, bs_pdf) * t;
            if (si.valid) depth += 1;
            alive = active_next;
        }
        const uint32_t slot_n = sbase + wave_append(ctr_next + it.seg * 32, alive);
        if (alive) {
            w.pd[nxt][slot_n] = pid | (depth << kPidBits);
            w.ox[nxt][slot_n] = ray.o.x; w.oy[nxt][slot_n] = ray.o.y; w.oz[nxt][slot_n] = ray.o.z;
            w.dx[nxt][slot_n] = ray.d.x; w.dy[nxt][slot_n] = ray.d.y; w.dz[nxt][slot_n] = ray.d.z;
            w.mt[nxt][slot_n] = ray.maxt;
            w.bx[nxt][slot_n] = beta.x; w.by[nxt][slot_n] = beta.y; w.bz[nxt][slot_n] = beta.z;
            w.ppx[nxt][slot_n] = prev_p.x; w.ppy[nxt][slot_n] = prev_p.y; w.ppz[nxt][slot_n] = prev_p.z;
            w.ppdf[nxt][slot_n] = prev_pdf;
            w.rng[nxt][slot_n] = rng.state;
            q.tea(nxt)[slot_n] = (uint32_t)(rng.inc >> 1);
            q.A(nxt, 0)[slot_n] = T.x; q.A(nxt, 1)[slot_n] = T.y; q.A(nxt, 2)[slot_n] = T.z;
        }
        // ---- visibility of the NEE sample; its tangent is charged if unoccluded
        const Hit sh = packet_batch<true, true>(S0.nodes, S0.prims, S0.prim_pairs, S0.key_sp, ws, 1u, sray, shadow, recs, dscr);
        if (shadow && sh.shape == MH_INVALID) dL = dL + G;
        if (alive) {
            q.dl(nxt, 0)[slot_n] = dL.x; q.dl(nxt, 1)[slot_n] = dL.y; q.dl(nxt, 2)[slot_n] = dL.z;
        } else if (i < n) {  // the path ends: its tangent radiance and validity (prb.py:253-257)
            fo.out[pid] = dL.x;
            fo.out[fo.plane + pid] = dL.y;
            fo.out[2 * fo.plane + pid] = dL.z;
            if (fo.alpha) fo.out[5 * fo.plane + pid] = depth != 0 ? 1.f : 0.f;
        }
        n_shadow += (uint32_t)__popcll(__ballot(shadow));
    }
    if (lane_id() == 0 && n_shadow) atomicAdd(ctr + it.seg * 32 + 1, n_shadow);  // statistics only
}

hipError_t launch_wavefront_fwd(const DScene &S, const IntegratorParams &in, const LaneMap &lm, uint32_t seed_value,
                                uint64_t n, const int32_t *slot_of_tex, float *const *tangents,
                                const uint32_t *is_rgb, float *out, uint64_t plane, int alpha, void *ws,
                                void *ws_prb, uint64_t cap, uint32_t *ctr, uint32_t n_bounces, uint32_t grid,
                                hipStream_t st) {
    if (n == 0) return hipSuccess;
    if (n > (1ull << kPidBits) || n_bounces > kMaxWfBounces || !wf_fused(S)) return hipErrorInvalidValue;
    WfState w = carve(ws, cap);
    WfPrb q = carve_prb(ws_prb, cap, nullptr, slot_of_tex, 1);
    hipError_t e = hipMemsetAsync(ctr, 0, sizeof(uint32_t) * kCtrStride * (n_bounces + 1), st);
    if (e != hipSuccess) return e;
    const uint32_t seg_cap = seg_len(n);
    const size_t sh_fused = fused_lds_bytes(S);
    const WfFwdOut fo{out, plane, alpha, slot_of_tex, tangents, is_rgb};
    for (uint32_t b = 0; b < n_bounces; ++b) {
        uint32_t *c = ctr + kCtrStride * b, *cn = ctr + kCtrStride * (b + 1);
        const int cur = (int)(b & 1);
        if (b == 0)
            hipLaunchKernelGGL(k_wf_bounce_fwd<true>, dim3(grid), dim3(256), sh_fused, st, S, in, lm, seed_value, w, q,
                               cur, seg_cap, c, cn, n, fo);
        else
            hipLaunchKernelGGL(k_wf_bounce_fwd<false>, dim3(grid), dim3(256), sh_fused, st, S, in, lm, seed_value, w,
                               q, cur, seg_cap, c, cn, n, fo);
    }
    return hipGetLastError();
}

// Texel gradients of the logged bitmap vertices of one chunk (see WfBmp):
// adj_k = D_k + dL (L_total - P_k) q_k / pi per record, spread over the
// bilinear taps (tex_backward's weights).  InLds: a persistent grid of
// kScatThreads-wide workgroups accumulating into a per-workgroup LDS copy of
// the texture, flushed once with one global atomic per non-zero texel; lane l
// of a wave takes path 64 c + l of a 4096-path tile (column c): coalesced
// loads, and one pixel's samples, whose camera vertices share texels, fold in
// lds_add_grouped (round 5, config 3(b): 3.27 -> 1.37 ms per scatter with the
// double accumulator below; the lanes 64 paths apart of
// round 4 re-read each 128-B line 8 times through a thrashed L2: 2.26 ms of
// the 3.27 were the loads).  Otherwise lane l takes
// path 64 l + c, 64 different pixels at 64 spp, and adds by global atomics,
// issued transposed: the wave's records
// stage (4 tap bases, 12 values) in LDS and the wave adds items (record,
// tap, channel) 64 at a time, so an instruction carries the two 24-B runs
// of ~5 records instead of 64 lanes in 64 rows (the float-atomic shape
// rule of corner_scatter; 1024^2 x 3 bitmap: 21.7 ms per scatter before).
MH_DEV float *bmp_stage() {
    __shared__ float st[4 * 64 * 16];
    return st + (threadIdx.x >> 6) * (64 * 16);
}
// the bitmap parameters of a scatter: record b (its r2.w) is texture tex[b],
// whose texels sit at float offset off[b] of the slot block grad (the
// bitmap slots' part of s->tmp_c, n_floats long with its padding)
// Fx (MH_FLAG_DETERMINISTIC; the global path only): 1 = the largest |value|
// into fx_max, nothing added; 2 = round(value * scale) as int64 into acc64
// (exact sums, folded into grad by k_fx_fold)
struct WfBmpTex {
    uint32_t tex[kMaxBitmapParams], off[kMaxBitmapParams];
    unsigned long long *acc64;
    uint32_t *fx_max;
    double scale;
    unsigned long long *n_rec;  // += records read (nullptr: not counted)
};
// the InLds accumulator: double (ds_add_f64 runs ~7x the rate of ds_add_f32
// on gfx950, mh_shading.hpp), or float with MH_SCAT_F64=0
#ifndef MH_SCAT_F64
#define MH_SCAT_F64 1
#endif
#if MH_SCAT_F64
using ScatT = double;
using ScatAcc = LdsDouble;
#else
using ScatT = float;
using ScatAcc = LdsFloat;
#endif
constexpr uint32_t kScatAccBytes = sizeof(ScatT);
#ifndef MH_SCAT_THREADS  // InLds: waves sharing one LDS copy of the texture
#define MH_SCAT_THREADS (MH_SCAT_F64 ? 1024 : 512)
#endif
constexpr uint32_t kScatThreads = MH_SCAT_THREADS;
template <bool InLds, int Fx = 0>
__global__ void __launch_bounds__(InLds ? kScatThreads : 256u)
k_wf_bitmap_scatter(DScene S, WfBmpTex bt, WfBmp bm, uint32_t n, float *__restrict__ grad, uint32_t n_floats) {
    static_assert(!(InLds && Fx), "the fixed-point passes use the global path");
    float fx_mx = 0.f;
    extern __shared__ uint4 lds[];
    ScatAcc *acc = (ScatAcc *)reinterpret_cast<ScatT *>(lds);
    if (InLds) {
        for (uint32_t i = threadIdx.x; i < n_floats; i += blockDim.x) acc[i] = (ScatT)0;
        __syncthreads();
    }
    // the global path: a workgroup owns whole 4096-path tiles (its waves take
    // the tile's 64 columns in turn), so the 64 lines a wave's transposed load
    // touches are re-read by the same CU's next columns from its L1 / L2
    const uint32_t n_tiles = (n + 4095u) / 4096u, waves = blockDim.x >> 6, wave = threadIdx.x >> 6,
                   lane = threadIdx.x & 63u;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    const DTexture tx0 = S.textures[bt.tex[0]];
    uint32_t n_recs = 0;  // this lane's records (mh_stats.aux_items)
#ifndef MH_SCAT_BAL  // float accumulators, 3 workgroups per CU: 2.44 vs 2.23 ms without; double, 1 per CU: 1.36 vs 1.39
#define MH_SCAT_BAL MH_SCAT_F64
#endif
    // InLds: the waves of the grid take 64-path columns in turn, so every
    // wave gets the same number of columns (+-1) instead of whole tiles
    const bool bal = InLds && MH_SCAT_BAL;
    const uint32_t n_outer = bal ? 1u : n_tiles, outer0 = bal ? 0u : blockIdx.x, outer_step = bal ? 1u : gridDim.x;
    const uint32_t col0 = bal ? blockIdx.x * waves + wave : wave, col_step = bal ? gridDim.x * waves : waves,
                   n_cols = bal ? (n + 63u) / 64u : 64u;
    for (uint32_t tile = outer0; tile < n_outer; tile += outer_step) {
      for (uint32_t col = col0; col < n_cols; col += col_step) {
        // InLds: lane l takes path 64 c + l (one pixel's samples: the camera
        // vertices share texels and lds_add_grouped folds them; coalesced
        // loads); the global path keeps the transposed lanes described above
        const uint32_t pid = InLds ? tile * 4096u + col * 64u + lane : tile * 4096u + lane * 64u + col;
        uint32_t mask = 0;
        float4 f0 = z4, f1 = z4;
        if (pid < n) {
            f0 = bm.fin[pid];
            mask = __float_as_uint(f0.w);
            if (mask) f1 = bm.fin[bm.stride + pid];
        }
        n_recs += (uint32_t)__popc(mask);
        const V3 Ltot = v3(f0.x, f0.y, f0.z), dL = v3(f1.x, f1.y, f1.z);
        // the next record's loads are issued before this record's adds
        bool on = mask != 0;
        float4 r0 = z4, r1 = z4, r2 = z4;
        if (on) {
            const uint32_t d = (uint32_t)__ffs(mask) - 1u;
            r0 = bm.r(d, 0)[pid]; r1 = bm.r(d, 1)[pid]; r2 = bm.r(d, 2)[pid];
        }
        while (__ballot(on)) {
            mask &= mask - 1u;
            const bool on_next = mask != 0;
            float4 q0 = z4, q1 = z4, q2 = z4;
            if (on_next) {
                const uint32_t d = (uint32_t)__ffs(mask) - 1u;
                q0 = bm.r(d, 0)[pid]; q1 = bm.r(d, 1)[pid]; q2 = bm.r(d, 2)[pid];
            }
            V3 adj = v3(0, 0, 0);
            float uvx = 0.f, uvy = 0.f;
            uint32_t bi = 0;
            if (on) {
                const V3 Lsuf = Ltot - v3(r0.x, r0.y, r0.z);  // prb.py: L - Le - Lr_dir
                adj = v3(r2.x, r2.y, r2.z) + ((dL * Lsuf) * v3(r1.x, r1.y, r1.z)) * kInvPi;
                uvx = r0.w;
                uvy = r1.w;
                bi = min(__float_as_uint(r2.w), (uint32_t)kMaxBitmapParams - 1u);
            }
            // a wave whose records all belong to the first bitmap (the common
            // case) takes its texture from the hoisted scalar copy instead of
            // five dependent loads per record
            DTexture tx = tx0;
            uint32_t goff = bt.off[0];
            if (__ballot(bi != 0)) {
                tx = S.textures[bt.tex[bi]];
                goff = bt.off[bi];
            }
            Taps tp;
            bitmap_taps(tx, uvx, uvy, tp);
            float w4[4] = {1.f, 0.f, 0.f, 0.f};
            if (tp.n != 1) {
                w4[0] = tp.w0y * tp.w0x; w4[1] = tp.w0y * tp.w1x; w4[2] = tp.w1y * tp.w0x; w4[3] = tp.w1y * tp.w1x;
            }
            if constexpr (!InLds) {
                const uint64_t onm = __ballot(on);
                const uint32_t n_on = (uint32_t)__popcll(onm);
                const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(onm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)onm, 0u));
                const uint32_t nc = tx.channels == 3 ? 3u : 1u, per = 4u * nc;  // every bitmap of a call has the same channel count
                float *st = bmp_stage();
                if (on) {
#pragma unroll
                    for (uint32_t k = 0; k < 4; ++k)
                        st[r * 16 + k] = __uint_as_float(k < tp.n ? goff + (uint32_t)(tp.idx[k] - tx.data_offset) : 0xffffffffu);
#pragma unroll
                    for (uint32_t k = 0; k < 4; ++k) {
                        if (nc == 3) {
                            st[r * 16 + 4 + k * 3 + 0] = adj.x * w4[k];
                            st[r * 16 + 4 + k * 3 + 1] = adj.y * w4[k];
                            st[r * 16 + 4 + k * 3 + 2] = adj.z * w4[k];
                        } else {
                            st[r * 16 + 4 + k * 3] = (adj.x + adj.y + adj.z) * w4[k];
                        }
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                const uint32_t total = n_on * per;
                for (uint32_t t = lane; t < total; t += 64u) {
                    const uint32_t src = t / per, rem = t - src * per, k = rem / nc, c = rem - k * nc;
                    const uint32_t base = __float_as_uint(st[src * 16 + k]);
                    if (base == 0xffffffffu) continue;
                    const float val = st[src * 16 + 4 + k * 3 + c];
                    if constexpr (Fx == 1) fx_mx = fmaxf(fx_mx, fabsf(val));
                    else if constexpr (Fx == 2)
                        gatomic_add(bt.acc64 + base + c, (unsigned long long)__double2ll_rn((double)val * bt.scale));
                    else gatomic_add(grad + base + c, val);
                }
                __builtin_amdgcn_wave_barrier();
            } else {
#pragma unroll
                for (uint32_t k = 0; k < 4; ++k) {
                    const bool tap = on && k < tp.n;
                    const uint32_t base = goff + (uint32_t)(tp.idx[k] - tx.data_offset);
                    if (tx.channels == 3) {
                        const float v[3] = {adj.x * w4[k], adj.y * w4[k], adj.z * w4[k]};
                        lds_add_grouped<3>(acc, base, tap, v);
                    } else {
                        const float v[1] = {(adj.x + adj.y + adj.z) * w4[k]};
                        lds_add_grouped<1>(acc, base, tap, v);
                    }
                }
            }
            on = on_next;
            r0 = q0; r1 = q1; r2 = q2;
        }
      }
    }
    if (bt.n_rec && Fx != 1) wave_count(bt.n_rec, n_recs);
    if (InLds) {
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < n_floats; i += blockDim.x)
            if (acc[i] != (ScatT)0) gatomic_add(grad + i, (float)acc[i]);
    }
    if constexpr (Fx == 1) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) fx_mx = fmaxf(fx_mx, __shfl_xor(fx_mx, off));
        if ((threadIdx.x & 63u) == 0 && fx_mx > 0.f) atomicMax(bt.fx_max, __float_as_uint(fx_mx));
    }
}

// grad += the exact int64 sums of the fixed-point scatter, once per texel float
__global__ void k_fx_fold(const long long *__restrict__ acc, float *__restrict__ grad, uint32_t n, double inv) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        grad[i] += (float)((double)acc[i] * inv);
}

template <bool InLds, bool Packet, int NR, int Eng>
__global__ void MH_STREAM_LB
k_wf_shadow_prb(DScene S, WfState w, WfPrb q, uint32_t seg_cap, uint32_t *ctr) {
    extern __shared__ uint4 lds[];
    const SegIter it = seg_iter();
    const uint32_t n = __hip_atomic_load(ctr + it.seg * 32 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!block_has_range_work(it, n)) return;
    LdsBvh B = stage_bvh<InLds && !Packet>(S, lds);
    const uint32_t base = it.seg * seg_cap;
    const uint32_t n_rgb = q.n_rgb;
    float acc[NR][3];
#pragma unroll
    for (int kk = 0; kk < NR; ++kk) acc[kk][0] = acc[kk][1] = acc[kk][2] = 0.f;
    uint32_t r0, r1;
    wave_range(it, n, r0, r1);
    auto load = [&](uint32_t i) {
        const uint32_t j = base + i;
        return RayT{v3(w.sox[j], w.soy[j], w.soz[j]), v3(w.sdx[j], w.sdy[j], w.sdz[j]), w.smt[j]};
    };
    auto store = [&](uint32_t i, const Hit &, bool occluded) {
        if (occluded) return;
        const uint32_t j = base + i;
#pragma unroll
        for (int kk = 0; kk < NR; ++kk)
            if ((uint32_t)kk < n_rgb) {
                acc[kk][0] += q.G(kk * 3 + 0)[j];
                acc[kk][1] += q.G(kk * 3 + 1)[j];
                acc[kk][2] += q.G(kk * 3 + 2)[j];
            }
    };
    if (Packet) trace_packet<true>(S.nodes, S.prims, S.prim_pairs, S.key_sp, B, r0, r1, load, store);
    else trace_stream<true, Eng>(B, r0, r1, load, store);
    flush_partial(acc, q);
}

// partials -> gradient buffers; block t sums entry t over all blocks
__global__ void __launch_bounds__(256)
k_wf_grad_reduce(const float *__restrict__ partial, uint32_t grid, float *const *bufs) {
    __shared__ float red[4];
    const uint32_t t = blockIdx.x;
    float s = 0.f;
    for (uint32_t b = threadIdx.x; b < grid; b += blockDim.x) s += partial[(size_t)b * kG + t];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    if (lane_id() == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) bufs[t / 3][t % 3] += (red[0] + red[1]) + (red[2] + red[3]);
}

hipError_t launch_wavefront_prb(const DScene &S, const IntegratorParams &in, const LaneMap &lm,
                                uint32_t seed_value, uint64_t n, int coalesce, const float *grad_in,
                                const float *weights, const int32_t *slot_of_tex, uint32_t n_rgb,
                                void *ws, void *ws_prb, uint64_t cap, uint32_t *ctr, uint32_t n_bounces,
                                uint32_t grid, float *partial, hipStream_t st, hipEvent_t *span,
                                const WfBitmapArgs *bmp, void *ws_det) {
    if (n == 0) return hipSuccess;
    if (n > (1ull << kPidBits) || n_bounces > kMaxWfBounces || n_rgb > (uint32_t)kMaxRgbParams) return hipErrorInvalidValue;
    WfState w = carve(ws, cap);
    WfPrb q = carve_prb(ws_prb, cap, partial, slot_of_tex, n_rgb);
    hipError_t e = hipMemsetAsync(ctr, 0, sizeof(uint32_t) * kCtrStride * (n_bounces + 1), st);
    if (e != hipSuccess) return e;
    const bool lds = S.lds_bytes_bvh != 0, packet = use_packet(S);
    const size_t sh = packet ? lds_bytes(S, 256) : stream_lds_bytes(S, 256);
    const uint32_t seg_cap = seg_len(n);
    const bool fused = packet && S.tab_bytes != 0 && !wf_unfused();
    const size_t sh_fused = fused_lds_bytes(S);
    if (S.stack_ovf && (uint64_t)grid * 256 > S.ovf_threads) return hipErrorInvalidValue;  // overflow columns
    const bool with_bmp = bmp != nullptr;
    if (with_bmp && (!fused || bmp->n_depth > 31 || bmp->n_depth + 1 < n_bounces || !bmp->ws)) return hipErrorInvalidValue;
    const WfBmp bm = with_bmp ? carve_bmp(bmp->ws, cap, bmp->n_depth, bmp->slot) : WfBmp{};
    const bool det_on = ws_det != nullptr;
    if (det_on && !fused) return hipErrorInvalidValue;
    const WfDet det = det_on ? carve_det(ws_det, cap) : WfDet{};
    if (det_on) {  // paths whose id is never written (segment gaps) add zeros
        e = hipMemsetAsync(det.fin_host(0), 0, (size_t)n_rgb * 3 * det.stride * 4, st);
        if (e != hipSuccess) return e;
    }
    if (!fused)  // the fused first bounce generates its camera rays itself
        hipLaunchKernelGGL(k_wf_raygen_prb, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, S, lm,
                           seed_value, n, coalesce, grad_in, weights, w, q, ctr);
    const PrbGen gen{n, grad_in, coalesce};
    if (span) (void)hipEventRecord(span[0], st);
#define MH_BOUNCE_PRB(NR, GEN, BM, DET)                                                                        \
    hipLaunchKernelGGL((k_wf_bounce_prb<NR, GEN, BM, DET>),                                                    \
                       dim3(grid), dim3(256),      \
                       sh_fused, st, S, in, lm, seed_value, w, q, cur, seg_cap, c, cn, gen, bm, det)
#define MH_BOUNCE_PRB_NR(GEN, BM, DET)                                                                         \
    do {                                                                                                       \
        if (n_rgb <= 1) MH_BOUNCE_PRB(1, GEN, BM, DET);                                                        \
        else MH_BOUNCE_PRB(kMaxRgbParams, GEN, BM, DET);                                                       \
    } while (0)
    for (uint32_t b = 0; b < n_bounces; ++b) {
        uint32_t *c = ctr + kCtrStride * b, *cn = ctr + kCtrStride * (b + 1);
        const int cur = (int)(b & 1);
        if (fused) {
            if (with_bmp && det_on) {
                if (b == 0) MH_BOUNCE_PRB_NR(true, true, true);
                else MH_BOUNCE_PRB_NR(false, true, true);
            } else if (with_bmp) {
                if (b == 0) MH_BOUNCE_PRB_NR(true, true, false);
                else MH_BOUNCE_PRB_NR(false, true, false);
            } else if (det_on) {
                if (b == 0) MH_BOUNCE_PRB_NR(true, false, true);
                else MH_BOUNCE_PRB_NR(false, false, true);
            } else {
                if (b == 0) MH_BOUNCE_PRB_NR(true, false, false);
                else MH_BOUNCE_PRB_NR(false, false, false);
            }
            continue;
        }
        MH_WF_DISPATCH(k_wf_trace, S, w, cur, seg_cap, c);
        if (n_rgb == 1) {
            if (S.tab_bytes)
                hipLaunchKernelGGL((k_wf_shade_prb<true, 1>), dim3(grid), dim3(256), S.tab_bytes, st, S, in, lm,
                                   seed_value, w, q, cur, seg_cap, c, cn);
            else
                hipLaunchKernelGGL((k_wf_shade_prb<false, 1>), dim3(grid), dim3(256), 0, st, S, in, lm, seed_value,
                                   w, q, cur, seg_cap, c, cn);
        } else {
            if (S.tab_bytes)
                hipLaunchKernelGGL((k_wf_shade_prb<true, kMaxRgbParams>), dim3(grid), dim3(256), S.tab_bytes, st, S,
                                   in, lm, seed_value, w, q, cur, seg_cap, c, cn);
            else
                hipLaunchKernelGGL((k_wf_shade_prb<false, kMaxRgbParams>), dim3(grid), dim3(256), 0, st, S, in, lm,
                                   seed_value, w, q, cur, seg_cap, c, cn);
        }
        if (n_rgb == 1) MH_WF_DISPATCH_NR(k_wf_shadow_prb, 1, S, w, q, seg_cap, c);
        else MH_WF_DISPATCH_NR(k_wf_shadow_prb, kMaxRgbParams, S, w, q, seg_cap, c);
    }
#undef MH_BOUNCE_PRB_NR
#undef MH_BOUNCE_PRB
    if (span) (void)hipEventRecord(span[1], st);  // the bounce span; span[1] -> span[2]: the scatter
    if (with_bmp) {
        const size_t acc_bytes = std::max<size_t>((size_t)bmp->n_floats * kScatAccBytes, 1);
        const bool in_lds = (size_t)bmp->n_floats * 4 <= bmp->lds_max && acc_bytes <= bmp->wg_lds;
        // accumulators per CU: as many as its LDS holds, at most the workgroups
        // of kScatThreads that are resident at once (more would only zero and
        // flush extra LDS copies)
        // (a thread-safe one-time query: calls on distinct scenes may run concurrently)
        static const int resident = [] {
            int r = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&r, k_wf_bitmap_scatter<true>, kScatThreads, 0) !=
                hipSuccess) {
                (void)hipGetLastError();
                r = 0;
            }
            return r;
        }();
        const uint32_t per_cu = (uint32_t)std::max<size_t>(
            1, std::min<size_t>(resident > 0 ? (size_t)resident : 8u, std::min<size_t>(8, bmp->cu_lds / acc_bytes)));
        const uint32_t blocks = std::max<uint32_t>(1, std::min<uint32_t>(bmp->cus * per_cu, (uint32_t)((n + 4095) / 4096)));
        WfBmpTex bt;
        for (int b = 0; b < kMaxBitmapParams; ++b) { bt.tex[b] = bmp->tex[b]; bt.off[b] = bmp->off[b]; }
        bt.acc64 = bmp->fx_acc;
        bt.fx_max = bmp->fx_word;
        bt.scale = 0.0;
        bt.n_rec = bmp->n_rec;
        const dim3 g_all((uint32_t)((n + 4095) / 4096));
        if (bmp->fx_acc) {  // deterministic: max pass, then int64 pass, then fold (this chunk's own scale)
            e = hipMemsetAsync(bmp->fx_word, 0, 4, st);
            if (e != hipSuccess) return e;
            hipLaunchKernelGGL((k_wf_bitmap_scatter<false, 1>), g_all, dim3(256), 0, st, S, bt, bm, (uint32_t)n,
                               bmp->grad, bmp->n_floats);
            uint32_t mb = 0;
            e = hipMemcpyAsync(&mb, bmp->fx_word, 4, hipMemcpyDeviceToHost, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
            if (e != hipSuccess) return e;
            float mx;
            memcpy(&mx, &mb, 4);
            int ex = 0;
            if (mx > 0.f && std::isfinite(mx)) (void)std::frexp(mx, &ex);
            bt.scale = std::ldexp(1.0, 31 - ex);
            e = hipMemsetAsync(bmp->fx_acc, 0, (size_t)bmp->n_floats * 8, st);
            if (e != hipSuccess) return e;
            hipLaunchKernelGGL((k_wf_bitmap_scatter<false, 2>), g_all, dim3(256), 0, st, S, bt, bm, (uint32_t)n,
                               bmp->grad, bmp->n_floats);
            hipLaunchKernelGGL(k_fx_fold, dim3(std::max<uint32_t>(1, std::min<uint32_t>(4096, (bmp->n_floats + 255) / 256))),
                               dim3(256), 0, st, reinterpret_cast<const long long *>(bmp->fx_acc), bmp->grad,
                               bmp->n_floats, std::ldexp(1.0, ex - 31));
        } else if (in_lds)
            hipLaunchKernelGGL(k_wf_bitmap_scatter<true>, dim3(blocks), dim3(kScatThreads), (size_t)bmp->n_floats * kScatAccBytes, st, S,
                               bt, bm, (uint32_t)n, bmp->grad, bmp->n_floats);
        else
            hipLaunchKernelGGL(k_wf_bitmap_scatter<false>, dim3((uint32_t)((n + 4095) / 4096)), dim3(256), 0, st, S,
                               bt, bm, (uint32_t)n, bmp->grad, bmp->n_floats);
    }
    if (span) (void)hipEventRecord(span[2], st);
    if (det_on) {
        hipLaunchKernelGGL(k_wf_det_sum, dim3(kDetBlocks), dim3(256), 0, st, det, (uint32_t)(seg_cap * kSeg), n_rgb * 3);
        hipLaunchKernelGGL(k_wf_det_fold, dim3(1), dim3(64), 0, st, det, n_rgb * 3, partial);
    }
    return hipGetLastError();
}

bool wf_fused(const DScene &S) { return use_packet(S) && S.tab_bytes != 0 && !wf_unfused(); }

uint32_t wf_grid(uint32_t grid) { return std::max<uint32_t>(kSeg, grid / kSeg * kSeg); }
// Workgroups of the wavefront kernels.  A wave's share of a queue is fixed
// (stride loop), and a CU holds 5 bounce workgroups at a time, so a grid of a
// few resident rounds leaves CUs idle in its last round; many small rounds
// even the tail out (MH_WF_BPC overrides for experiments: tools/exp_bpc.sh).
// shared: another call runs on the device at the same time
// (MH_FLAG_SHARED_DEVICE): each launch then takes a smaller share of the CUs' slots, so
// the two calls' launches interleave instead of queueing behind each other --
// the overlapped bench step (forward || gradient pass), 3 runs per point:
// 30 -> 2,074-2,094, 20 -> 2,098-2,106, 12 -> 2,105-2,129, 8 -> 2,105-2,117,
// 6 -> 2,070-2,082 Msamples/s (alone, 12 would cost 6 %: 1,824 vs 1,946)
uint32_t wf_blocks(int cus, bool shared) {
    uint32_t bpc = shared ? 12 : 30;  // measured alone: 8 -> 54.6, 20 -> 51.4, 30 -> 51.2, 60 -> 52.3 ms per bench step
    if (const char *e = getenv("MH_WF_BPC")) bpc = std::max(1, atoi(e));
    return (uint32_t)cus * bpc;
}

hipError_t launch_wf_grad_reduce(const float *partial, uint32_t grid, uint32_t n_rgb, float *const *bufs,
                                 hipStream_t st) {
    if (n_rgb == 0) return hipSuccess;
    hipLaunchKernelGGL(k_wf_grad_reduce, dim3(n_rgb * 3), dim3(256), 0, st, partial, grid, bufs);
    return hipGetLastError();
}

#ifdef MH_EXP_BPHASE
extern "C" int mh_exp_bphase(unsigned long long *out, int reset) {
    hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bph), sizeof(g_bph));
    if (reset) {
        unsigned long long z[48] = {0};
        hipMemcpyToSymbol(HIP_SYMBOL(g_bph), z, sizeof(z));
    }
    return 0;
}
#endif
#ifdef MH_EXP_COUNT
extern "C" int mh_exp_counters(unsigned long long *out, int reset) {
    hipMemcpyFromSymbol(out, HIP_SYMBOL(g_exp_cnt), sizeof(g_exp_cnt));
    if (reset) {
        unsigned long long z[32] = {0};
        hipMemcpyToSymbol(HIP_SYMBOL(g_exp_cnt), z, sizeof(z));
    }
    return 0;
}
#endif
}  // namespace mh
