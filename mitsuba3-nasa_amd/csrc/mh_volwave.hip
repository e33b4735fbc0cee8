// mh_volwave.hip — wavefront execution of the `volpath` integrator
// (integrators/volpath.cpp:95-450) for configuration 4.
//
// The per-lane megakernel (k_render<VOLPATH>) runs at 10-12 % lane
// utilisation: a lane's loop trips are mostly null collisions
// (volpath.cpp:161-205; ~17.5 trips per sample on config 4) and its emitter
// samples walk ratio-tracked shadow rays of very different lengths
// (volpath.cpp:361-448; ~25 steps per sample), so the 64 lanes of a wave sit
// in different loops most of the time.  Here the loop is cut at its one
// long inner loop, the NEE transmittance walk, into two persistent kernels
// that alternate in rounds:
//
//   k_vw_main  runs a path's loop trips (volpath_post of the previous trip,
//              then volpath_pre) until the path either ends -- it writes its
//              sample -- or starts a shadow walk: then it appends its state
//              to the next round's queue and the walk to the walk queue;
//   k_vw_walk  runs every queued walk to its end (nee_step until the
//              transmittance loop exits) and hands the transmittance x
//              emitter value and the lane's advanced PCG32 state back.
//
// Both kernels keep every lane busy with per-lane refill: a lane whose path
// suspends or ends (or whose walk ends) takes the wave's next item at once
// (the while-while scheme of trace_stream), so a wave no longer waits for
// its longest lane.  A path walks at most once per real scatter and depth <
// max_depth bounds those, so at most max_depth + 1 main rounds exist.
//
// Every per-lane operation and random draw is the megakernel's (the same
// volpath_pre / volpath_post / nee_step device functions in the same
// order, with the state a walk needs carried through HBM bit for bit), so
// samples are bit-identical to k_render<VOLPATH> and to the CPU oracle.
//
// HBM layout: 15 planes of 16-B records per path slot and side (ping-pong),
// slot-indexed by queue position; queues are split into kVwSeg static
// segments (a path never changes segment, each segment's counter has its
// own 128-B line; workgroup b serves segment b % kVwSeg).
//   path record    C0 d.xyz last_pdf      C1 throughput.xyz pid
//                  C2 result.xyz bits     C3 last_p.xyz pend_w
//                  C4 pend.xyz pcg_v1     C5 mei.p.xyz depth
//   surface NEE    X0 si.p.xyz wi.z       X1 si.n.xyz shape
//                  X2 si.s.xyz rho.x      X3 si.t.xyz rho.y    X4 si.sn.xyz rho.z
//   walk item      W0 o.xyz max_dist      W1 d.xyz medium
//                  W2 emitter_val.xyz ds.dist  (walk result: nee.xyz)
//                  W3 pcg.state lo hi, pcg_v1
#include <algorithm>
#include <cstring>
#include <type_traits>

#include "mh_internal.hpp"
#include "mh_shading.hpp"

namespace mh {
namespace {

constexpr uint32_t kVwSeg = 64;
constexpr uint32_t kVwCtr = kVwSeg * 32;  // counter words per round
constexpr uint32_t kVwPlanes = 15;        // per side
constexpr uint32_t kVwWaveRounds = 6;     // main / walk rounds before the finish launch (MH_VW_ROUNDS)
enum : uint32_t { kC0 = 0, kC1, kC2, kC3, kC4, kC5, kX0, kX1, kX2, kX3, kX4, kW0, kW1, kW2, kW3 };

// bits of C2.w
enum : uint32_t {
    kBitActScatter = 1u << 10, kBitActSurface = 1u << 11, kBitActMedium = 1u << 12, kBitActive = 1u << 13,
    kBitSpecChain = 1u << 14, kBitValid = 1u << 15
};

struct VwPlanes {
    float4 *p;     // side base: plane k at p + k * cap
    uint64_t cap;
    MH_DEV float4 &at(uint32_t k, uint64_t i) const { return p[k * cap + i]; }
};

MH_DEV uint32_t vw_lane() { return threadIdx.x & 63u; }

struct VwSeg {
    uint32_t seg, wave, nwaves;
};
MH_DEV VwSeg vw_seg() {
    VwSeg it;
    it.seg = blockIdx.x % kVwSeg;
    const uint32_t wpb = blockDim.x / 64u;
    it.wave = (blockIdx.x / kVwSeg) * wpb + threadIdx.x / 64u;
    it.nwaves = (gridDim.x / kVwSeg) * wpb;
    return it;
}

// ballot-compacted append to a segment counter; reached by the whole wave
MH_DEV uint32_t vw_append(uint32_t *count, bool pred) {
    const unsigned long long m = __ballot(pred);
    const uint32_t tot = (uint32_t)__popcll(m);
    uint32_t base = 0;
    if (vw_lane() == 0 && tot) base = atomicAdd(count, tot);
    base = __builtin_amdgcn_readfirstlane(base);
    return base + (uint32_t)__popcll(m & ((1ull << vw_lane()) - 1ull));
}

MH_DEV float4 f4(V3 a, float w) { return make_float4(a.x, a.y, a.z, w); }
MH_DEV float4 f4u(V3 a, uint32_t w) { return make_float4(a.x, a.y, a.z, __uint_as_float(w)); }
MH_DEV V3 xyz(const float4 &a) { return v3(a.x, a.y, a.z); }

// ---- the state a suspended path carries through HBM ------------------------
MH_DEV void vw_store_path(const VwPlanes &P, uint64_t i, const VolState &v, uint32_t pid, uint32_t v1) {
    const uint32_t med = v.medium == MH_INVALID ? 0xffu : v.medium;
    const uint32_t bits = med | (v.nee_kind << 8) | (v.act_scatter ? kBitActScatter : 0u) |
                          (v.active_surface ? kBitActSurface : 0u) | (v.active_medium ? kBitActMedium : 0u) |
                          (v.active ? kBitActive : 0u) | (v.specular_chain ? kBitSpecChain : 0u) |
                          (v.valid ? kBitValid : 0u);
    P.at(kC0, i) = f4(v.ray.d, v.last_pdf);
    P.at(kC1, i) = f4u(v.throughput, pid);
    P.at(kC2, i) = f4u(v.result, bits);
    P.at(kC3, i) = f4(v.last_p, v.pend_w);
    P.at(kC4, i) = f4u(v.pend, v1);
    P.at(kC5, i) = f4u(v.mei.p, v.depth);
    if (v.active_surface) {
        // a surface walk only starts from a non-null BSDF, whose sampling in
        // volpath_post reads wi.z alone (the null branch's -wi never runs)
        P.at(kX0, i) = f4(v.si.p, v.si.wi.z);
        P.at(kX1, i) = f4u(v.si.n, v.si.shape);
        P.at(kX2, i) = f4(v.si.s, v.rho.x);
        P.at(kX3, i) = f4(v.si.t_, v.rho.y);
        P.at(kX4, i) = f4(v.si.sn, v.rho.z);
    }
}

MH_DEV void vw_store_walk(const VwPlanes &P, uint64_t i, const VolState &v, const Pcg &rng, uint32_t v1) {
    const NeeState &ns = v.ns;
    P.at(kW0, i) = f4(ns.ray.o, ns.max_dist);
    P.at(kW1, i) = f4u(ns.ray.d, ns.medium);
    P.at(kW2, i) = f4(ns.emitter_val, v.ds.dist);
    P.at(kW3, i) = make_float4(__uint_as_float((uint32_t)rng.state), __uint_as_float((uint32_t)(rng.state >> 32)),
                               __uint_as_float(v1), 0.f);
}

// resume a suspended path in kVolPost mode with its walk's result
MH_DEV void vw_load_path(const DScene &S, const VwPlanes &P, uint64_t i, VolState &v, Pcg &rng, uint32_t &pid,
                         uint32_t &v1) {
    const float4 c0 = P.at(kC0, i), c1 = P.at(kC1, i), c2 = P.at(kC2, i), c3 = P.at(kC3, i), c4 = P.at(kC4, i),
                 c5 = P.at(kC5, i), w2 = P.at(kW2, i), w3 = P.at(kW3, i);
    const uint32_t bits = __float_as_uint(c2.w);
    v.ray.d = xyz(c0);
    v.last_pdf = c0.w;
    v.throughput = xyz(c1);
    pid = __float_as_uint(c1.w);
    v.result = xyz(c2);
    v.last_p = xyz(c3);
    v.pend_w = c3.w;
    v.pend = xyz(c4);
    v1 = __float_as_uint(c4.w);
    v.mei.p = xyz(c5);
    v.depth = __float_as_uint(c5.w);
    const uint32_t med = bits & 0xffu;
    v.medium = med == 0xffu ? MH_INVALID : med;
    v.nee_kind = (bits >> 8) & 3u;
    v.act_scatter = bits & kBitActScatter;
    v.active_surface = bits & kBitActSurface;
    v.active_medium = bits & kBitActMedium;
    v.active = bits & kBitActive;
    v.specular_chain = bits & kBitSpecChain;
    v.valid = bits & kBitValid;
    v.eta = 1.f;
    // the medium interaction's frame: Frame3f(ray.d) of sample_interaction
    v.mei.fn = v.ray.d;
    coordinate_system(v.ray.d, v.mei.fs, v.mei.ft);
    // the walk's transmittance x emitter value (x 1 keeps it exact)
    v.ns.transmittance = xyz(w2);
    v.ns.emitter_val = v3(1.f, 1.f, 1.f);
    rng.state = (uint64_t)__float_as_uint(w3.x) | ((uint64_t)__float_as_uint(w3.y) << 32);
    rng.inc = ((uint64_t)v1 << 1) | 1u;
    if (v.active_surface) {
        const float4 x0 = P.at(kX0, i), x1 = P.at(kX1, i), x2 = P.at(kX2, i), x3 = P.at(kX3, i), x4 = P.at(kX4, i);
        v.si.valid = true;
        v.si.p = xyz(x0);
        v.si.wi = v3(0.f, 0.f, x0.w);
        v.si.n = xyz(x1);
        v.si.shape = __float_as_uint(x1.w);
        v.si.s = xyz(x2);
        v.si.t_ = xyz(x3);
        v.si.sn = xyz(x4);
        v.rho = v3(x2.w, x3.w, x4.w);
    }
    v.mode = kVolPost;
}

MH_DEV void vw_write_sample(float *out, uint64_t plane, uint32_t pid, const VolState &v, int alpha) {
    out[pid] = v.result.x;
    out[plane + pid] = v.result.y;
    out[2 * plane + pid] = v.result.z;
    if (alpha) out[5 * plane + pid] = v.valid ? 1.f : 0.f;  // aovs[3] (integrator.cpp:1229-1231)
}

MH_DEV void vw_range(const VwSeg &it, uint32_t n, uint32_t &r0, uint32_t &r1) {
    const uint32_t per = (n + it.nwaves - 1) / it.nwaves;
    r0 = min(n, it.wave * per);
    r1 = min(n, r0 + per);
}

}  // namespace

// ---------------------------------------------------------------------------
// k_vw_main: the loop trips of every queued path up to its next shadow walk.
// Fresh (round 0): item j of segment s is path s * seg_cap + j, generated
// here exactly as k_render does (TEA/PCG32 seed, jitter, camera ray,
// volpath_init); film positions go to the sample planes.
// ---------------------------------------------------------------------------
#ifndef MH_VW_MAIN_WAVES
#define MH_VW_MAIN_WAVES 2
#endif
template <bool Fresh, bool InLds, bool Pk>
__global__ void __launch_bounds__(256, MH_VW_MAIN_WAVES)
k_vw_main(DScene S, IntegratorParams in, LaneMap lm, uint32_t seed_value, uint64_t n, uint64_t plane,
          float *__restrict__ out, VwPlanes cur, VwPlanes nxt, uint32_t seg_cap, const uint32_t *__restrict__ ctr_in,
          uint32_t *__restrict__ ctr_out, unsigned long long *__restrict__ counters, int alpha) {
    const VwSeg it = vw_seg();
    uint32_t count;
    if (Fresh) {
        const uint64_t b = (uint64_t)it.seg * seg_cap;
        count = b >= n ? 0u : (uint32_t)std::min<uint64_t>(seg_cap, n - b);
    } else {
        count = ctr_in[it.seg * 32];
    }
    {   // workgroups without items leave before staging anything
        const uint32_t first_wave = (blockIdx.x / kVwSeg) * (blockDim.x / 64u);
        const uint32_t per = (count + it.nwaves - 1) / it.nwaves;
        if (first_wave * per >= count) return;
    }
    extern __shared__ uint4 lds[];
    LdsBvh B = stage_bvh<InLds>(S, lds);
    uint32_t r0, r1;
    vw_range(it, count, r0, r1);
    const uint64_t base = (uint64_t)it.seg * seg_cap;
    uint32_t *ctr_next = ctr_out + it.seg * 32;
    const float sw = S.inv_width, sh = S.inv_height;
    uint32_t n_closest = 0;
#ifdef MH_EXP_VWCNT  // diagnostic build: loop trips / walk steps / wave iterations per round
    uint32_t n_trips = 0, n_iter = 0;
#endif

    VolState v;
    Pcg rng;
    uint32_t pid = 0, v1 = 0;
    auto load = [&](uint32_t item) {
        if (Fresh) {
            pid = (uint32_t)(base + item);
            uint32_t lane, px, py;
            lane_of(lm, pid, lane, px, py);
            rng.seed(seed_value, lane);
            v1 = (uint32_t)(rng.inc >> 1);
            const float sx = (float)px + rng.next_float(), sy = (float)py + rng.next_float();
            const RayT r = camera_ray(S, __builtin_fmaf(sx, sw, -0.f), __builtin_fmaf(sy, sh, -0.f));
            out[3 * plane + pid] = sx;
            out[4 * plane + pid] = sy;
            volpath_init(S, in, rng, r, v);
        } else {
            vw_load_path(S, cur, base + item, v, rng, pid, v1);
        }
    };
    uint32_t fetched = r0 + 64u;  // wave-uniform
    bool has = r0 + vw_lane() < r1;
    if (has) load(r0 + vw_lane());
    while (__builtin_amdgcn_ballot_w64(has) != 0) {
        bool ended = false, susp = false;
#ifdef MH_EXP_VWCNT
        ++n_iter;
#endif
        if (has) {
            bool alive = true;
#ifdef MH_EXP_VWCNT
            ++n_trips;
#endif
            if (v.mode == kVolPost) alive = volpath_post(S, in, rng, v);
            if (alive) alive = volpath_pre<Pk>(S, B, in, rng, v, n_closest);
            if (!alive) ended = true;
            else susp = v.mode == kVolNee;
        }
        const uint32_t pos = vw_append(ctr_next, susp);
        if (susp) {
            vw_store_path(nxt, base + pos, v, pid, v1);
            vw_store_walk(nxt, base + pos, v, rng, v1);
        }
        if (ended) vw_write_sample(out, plane, pid, v, alpha);
        const bool need = !has || ended || susp;
        const unsigned long long m = __ballot(need);
        if (need) {
            const uint32_t cand = fetched + (uint32_t)__popcll(m & ((1ull << vw_lane()) - 1ull));
            has = cand < r1;
            if (has) load(cand);
        }
        fetched += (uint32_t)__popcll(m);
    }
    if (counters) wave_count(&counters[0], n_closest);
#ifdef MH_EXP_VWCNT
    wave_count(reinterpret_cast<unsigned long long *>(ctr_out + it.seg * 32 + 2), n_trips);
    if (vw_lane() == 0) atomicAdd(ctr_out + it.seg * 32 + 6, n_iter);
#endif
}

// ---------------------------------------------------------------------------
// k_vw_finish: the tail.  After the first rounds few paths remain, and a
// round costs its longest walk or trip chain however few items it holds, so
// the remaining paths run to their end in one launch: each lane resumes a
// suspended path and advances it through its remaining trips and walks
// (volpath_advance, the megakernel's state machine), refilled per lane.
// ---------------------------------------------------------------------------
template <bool InLds, bool Pk>
__global__ void __launch_bounds__(256, MH_VW_MAIN_WAVES)
k_vw_finish(DScene S, IntegratorParams in, uint64_t plane, float *__restrict__ out, VwPlanes cur, uint32_t seg_cap,
            const uint32_t *__restrict__ ctr_in, unsigned long long *__restrict__ counters, int alpha) {
    const VwSeg it = vw_seg();
    const uint32_t count = ctr_in[it.seg * 32];
    {
        const uint32_t first_wave = (blockIdx.x / kVwSeg) * (blockDim.x / 64u);
        const uint32_t per = (count + it.nwaves - 1) / it.nwaves;
        if (first_wave * per >= count) return;
    }
    extern __shared__ uint4 lds[];
    LdsBvh B = stage_bvh<InLds>(S, lds);
    uint32_t r0, r1;
    vw_range(it, count, r0, r1);
    const uint64_t base = (uint64_t)it.seg * seg_cap;
    uint32_t n_closest = 0, n_shadow = 0;
    VolState v;
    Pcg rng;
    uint32_t pid = 0, v1 = 0;
    uint32_t fetched = r0 + 64u;
    bool has = r0 + vw_lane() < r1;
    if (has) vw_load_path(S, cur, base + r0 + vw_lane(), v, rng, pid, v1);
    while (__builtin_amdgcn_ballot_w64(has) != 0) {
        bool ended = false;
        if (has && !volpath_advance<Pk>(S, B, in, rng, v, n_closest, n_shadow)) {
            ended = true;
            vw_write_sample(out, plane, pid, v, alpha);
        }
        const bool need = !has || ended;
        const unsigned long long m = __ballot(need);
        if (need) {
            const uint32_t cand = fetched + (uint32_t)__popcll(m & ((1ull << vw_lane()) - 1ull));
            has = cand < r1;
            if (has) vw_load_path(S, cur, base + cand, v, rng, pid, v1);
        }
        fetched += (uint32_t)__popcll(m);
    }
    if (counters) {
        wave_count(&counters[0], n_closest);
        wave_count(&counters[1], n_shadow);
    }
}

// ---------------------------------------------------------------------------
// k_vw_walk: every queued shadow walk to its end (volpath.cpp:361-448,
// nee_step), starting from nee_begin's state; writes transmittance x
// emitter value and the lane's PCG32 state back into the walk record.
// ---------------------------------------------------------------------------
#ifndef MH_VW_WALK_WAVES
#define MH_VW_WALK_WAVES 4
#endif
template <bool InLds, bool Pk>
__global__ void __launch_bounds__(256, MH_VW_WALK_WAVES)
k_vw_walk(DScene S, VwPlanes P, uint32_t seg_cap, const uint32_t *__restrict__ ctr,
          unsigned long long *__restrict__ counters) {
    const VwSeg it = vw_seg();
    const uint32_t count = ctr[it.seg * 32];
    {
        const uint32_t first_wave = (blockIdx.x / kVwSeg) * (blockDim.x / 64u);
        const uint32_t per = (count + it.nwaves - 1) / it.nwaves;
        if (first_wave * per >= count) return;
    }
    extern __shared__ uint4 lds[];
    LdsBvh B = stage_bvh<InLds>(S, lds);
    uint32_t r0, r1;
    vw_range(it, count, r0, r1);
    const uint64_t base = (uint64_t)it.seg * seg_cap;
    uint32_t n_shadow = 0;
#ifdef MH_EXP_VWCNT
    uint32_t n_steps = 0, n_iter = 0;
#endif
    NeeState ns;
    DirS ds;
    Pcg rng;
    uint64_t slot = 0;
    auto load = [&](uint32_t item) {
        slot = base + item;
        const float4 w0 = P.at(kW0, slot), w1 = P.at(kW1, slot), w2 = P.at(kW2, slot), w3 = P.at(kW3, slot);
        // nee_begin's state after the emitter sample (mh_shading.hpp)
        ns.ray = RayT{xyz(w0), xyz(w1), w0.w};
        ns.max_dist = w0.w;
        ns.medium = __float_as_uint(w1.w);
        ns.emitter_val = xyz(w2);
        ds.dist = w2.w;
        ns.transmittance = v3(1.f, 1.f, 1.f);
        ns.total_dist = 0.f;
        ns.si.valid = false;
        ns.si_t = 0.f;
        ns.needs_intersection = true;
        rng.state = (uint64_t)__float_as_uint(w3.x) | ((uint64_t)__float_as_uint(w3.y) << 32);
        rng.inc = ((uint64_t)__float_as_uint(w3.z) << 1) | 1u;
    };
    uint32_t fetched = r0 + 64u;
    bool has = r0 + vw_lane() < r1;
    if (has) load(r0 + vw_lane());
    while (__builtin_amdgcn_ballot_w64(has) != 0) {
        bool fin = false;
#ifdef MH_EXP_VWCNT
        n_steps += has;
        ++n_iter;
#endif
        if (has && !nee_step<Pk>(S, B, rng, ds, ns, n_shadow)) {
            fin = true;
            const V3 r = nee_result(ns);
            P.at(kW2, slot) = f4(r, 0.f);
            P.at(kW3, slot) = make_float4(__uint_as_float((uint32_t)rng.state),
                                          __uint_as_float((uint32_t)(rng.state >> 32)), 0.f, 0.f);
        }
        const bool need = !has || fin;
        const unsigned long long m = __ballot(need);
        if (need) {
            const uint32_t cand = fetched + (uint32_t)__popcll(m & ((1ull << vw_lane()) - 1ull));
            has = cand < r1;
            if (has) load(cand);
        }
        fetched += (uint32_t)__popcll(m);
    }
    if (counters) wave_count(&counters[1], n_shadow);
#ifdef MH_EXP_VWCNT
    wave_count(reinterpret_cast<unsigned long long *>(const_cast<uint32_t *>(ctr) + it.seg * 32 + 4), n_steps);
    if (vw_lane() == 0) atomicAdd(const_cast<uint32_t *>(ctr) + it.seg * 32 + 7, n_iter);
#endif
}

// ===========================================================================
// Phase-scheduled volpath (k_vol_sched): one persistent launch, no rounds.
//
// The loop of volpath.cpp:139-330 and its NEE walk (:361-448) are cut into
// phases at every point where the work changes kind:
//   HEAD     loop head: Russian roulette, free-flight sampling in the medium
//            (sample_interaction), the null / real decision of a null
//            collision -- the light, frequent trip;
//   TRACE    a closest-hit query (medium segment, surface, or walk segment);
//   SCATTER  a real medium scatter: albedo weight, emitter sample, phase eval;
//   SURF     a surface interaction: emission + MIS, BSDF NEE setup;
//   WALK     one step of the ratio-tracked transmittance walk;
//   POST     after a walk: the sample's contribution, phase / BSDF sampling;
//   FREE     a lane without a path takes the wave's next sample (camera ray).
// Each trip of the wave runs ONE phase -- the one whose pending lanes times
// its weight is largest (a ballot per phase) -- for exactly the lanes pending
// in it; lanes of other phases wait.  Heavy, rare work (scatter, surface,
// traces) therefore runs for many lanes at once instead of costing the whole
// wave at a few active lanes per instruction, the light phases run nearly
// full, and a finished lane is refilled at once (no wave waits for its
// longest path, no barrier between rounds, no path state through HBM).
// Per lane, the operations and random draws are those of volpath_pre /
// volpath_post / nee_step in their order (bit-identical samples).
// ===========================================================================
enum : uint32_t {
    kPhFree = 0, kPhHead, kPhTraceM, kPhTraceS, kPhTraceWM, kPhTraceWS, kPhScatter, kPhSurf, kPhWalk, kPhPost, kPhEnd
};
// kGEnd: a finished path's own end-of-path work (machines with kDeferEnd:
// the backward's log application), scheduled like the other heavy phases
enum : uint32_t { kGFree = 0, kGHead, kGTrace, kGScatter, kGSurf, kGWalk, kGPost, kGEnd, kNGroups };
MH_DEV uint32_t ph_group(uint32_t ph) {
    return ph == kPhFree ? kGFree : ph == kPhHead ? kGHead : ph <= kPhTraceWS ? kGTrace : ph == kPhScatter ? kGScatter
         : ph == kPhSurf ? kGSurf : ph == kPhWalk ? kGWalk : ph == kPhPost ? kGPost : kGEnd;
}

// the walk's own medium interaction across its trace (nee_step's local mei)
struct WMei {
    float t, mint, maj, sigma_n;
    V3 p;
    bool valid;
};

// end of a trip that needs no walk (volpath_pre's tail + volpath_post)
MH_DEV uint32_t vs_no_walk(const DScene &S, const IntegratorParams &in, Pcg &rng, VolState &v) {
    if (v.nee_kind != kNeeNone) {  // ds.pdf == 0: emitted = 0
        v.ns.transmittance = v3(0, 0, 0);
        v.ns.emitter_val = v3(0, 0, 0);
    }
    return volpath_post(S, in, rng, v) ? kPhHead : kPhFree;
}

// the medium block of volpath_pre after its (optional) intersection, up to
// the scatter / surface split (volpath.cpp:166-223)
MH_DEV uint32_t vs_med_rest(const DScene &S, const IntegratorParams &in, Pcg &rng, VolState &v) {
    MEI &mei = v.mei;
    v.needs_intersection = v.needs_intersection && !v.si.valid;
    if (v.si_t < mei.t) { mei.t = __builtin_huge_valf(); mei.valid = false; }
    const DMedium &m = S.media[v.medium];
    const bool spectral = !(m.flags & MH_MEDIUM_NO_SPECTRAL_EXTINCTION);
    if (spectral) {
        const float t = fminf(mei.t, v.si_t) - mei.mint;
        const float tr = exp_dr((-t) * mei.maj);
        const float pdf = v.si_t < mei.t ? tr : tr * mei.maj;
        v.throughput = v.throughput * (pdf > 0.f ? tr / pdf : 0.f);
    }
    const bool escaped = !mei.valid;
    v.active_medium = mei.valid;
    bool null_scatter = false;
    if (v.active_medium) null_scatter = rng.next_float() >= mei.sigma_t / mei.maj;
    const bool act_null = null_scatter && v.active_medium;
    bool act_scatter = !act_null && v.active_medium;
    if (spectral && act_null) v.throughput = v.throughput * ((mei.sigma_n * mei.maj) / mei.sigma_n);
    if (act_scatter) { v.depth += 1; v.last_p = mei.p; }
    v.active = v.active && v.depth < in.max_depth;
    act_scatter = act_scatter && v.active;
    if (act_null) { v.ray.o = mei.p; v.si_t = v.si_t - mei.t; }
    v.nee_kind = kNeeNone;
    v.act_scatter = act_scatter;
    if (act_scatter) return kPhScatter;
    v.active_surface = v.active_surface || escaped;
    if (v.active_surface) return v.needs_intersection ? kPhTraceS : kPhSurf;
    // a null collision (or a scatter cut by max_depth): volpath_post's test
    v.active_surface = false;
    v.rho = v3(0, 0, 0);
    return (v.active && v.active_medium) ? kPhHead : kPhFree;
}

// HEAD: Russian roulette and free-flight sampling (volpath.cpp:143-165), cut
// at its medium sample: true with the sample's draw u when one is pending
// (v.medium, v.ray), else the next phase in nph
MH_DEV bool vs_head_pre(const DScene &S, const IntegratorParams &in, Pcg &rng, VolState &v, uint32_t &nph, float &u) {
    bool active = nonzero(v.throughput);
    const float q = fminf(hmax(v.throughput) * (v.eta * v.eta), 0.95f);
    const bool perform_rr = v.depth > in.rr_depth;
    if (active) active = rng.next_float() < q || !perform_rr;
    if (perform_rr) v.throughput = v.throughput * rcp(q);
    active = active && v.depth < in.max_depth;
    if (!active) { nph = kPhFree; return false; }
    v.active = true;
    v.active_medium = v.medium != MH_INVALID;
    v.active_surface = !v.active_medium;
    v.act_scatter = false;
    v.nee_kind = kNeeNone;
    v.mei.valid = false;
    v.mei.t = __builtin_huge_valf();
    if (v.active_medium) { u = rng.next_float(); return true; }
    nph = v.needs_intersection ? kPhTraceS : kPhSurf;
    return false;
}
// the rest of HEAD once v.mei holds the medium sample
MH_DEV uint32_t vs_head_post(const DScene &S, const IntegratorParams &in, Pcg &rng, VolState &v) {
    const DMedium &m = S.media[v.medium];
    if (m.type == MH_MEDIUM_HOMOGENEOUS && v.mei.valid) v.ray.maxt = v.mei.t;
    if (v.needs_intersection) return kPhTraceM;
    return vs_med_rest(S, in, rng, v);
}
MH_DEV uint32_t vs_head(const DScene &S, const IntegratorParams &in, Pcg &rng, VolState &v) {
    uint32_t nph = kPhFree;
    float u = 0.f;
    if (!vs_head_pre(S, in, rng, v, nph, u)) return nph;
    sample_interaction(S, v.medium, v.ray, u, v.mei);
    return vs_head_post(S, in, rng, v);
}

// SCATTER: a real medium interaction (volpath.cpp:224-252)
MH_DEV uint32_t vs_scatter(const DScene &S, const IntegratorParams &in, Pcg &rng, VolState &v) {
    mei_frame(v.mei);  // the merged medium step samples without it (identical values)
    const DMedium &m = S.media[v.medium];
    const MEI &mei = v.mei;
    const bool spectral = !(m.flags & MH_MEDIUM_NO_SPECTRAL_EXTINCTION);
    if (spectral) v.throughput = v.throughput * vdiv(mei.sigma_s * mei.maj, mei.sigma_t);
    else v.throughput = v.throughput * vdiv(mei.sigma_s, mei.sigma_t);
    const bool sample_emitters = !(m.flags & MH_MEDIUM_NO_EMITTER_SAMPLING);
    v.specular_chain = !sample_emitters;
    v.valid = true;  // valid_ray |= act_medium_scatter (volpath.cpp:223)
    bool walk = false;
    if (sample_emitters) {
        walk = nee_begin(S, mei.p, v3(0, 0, 0), nullptr, rng, v.medium, v.ds, v.ns);
        const float ph = phase_eval(m, mei_to_local(mei, v.ds.d));
        v.pend = v.throughput * ph;
        v.pend_w = mis_weight(v.ds.pdf, v.ds.delta ? 0.f : ph);
        v.nee_kind = kNeeMedium;
    }
    v.active_surface = false;
    v.rho = v3(0, 0, 0);
    return walk ? kPhWalk : vs_no_walk(S, in, rng, v);
}

// SURF: a surface interaction after its intersection (volpath.cpp:254-300)
MH_DEV uint32_t vs_surf(const DScene &S, const IntegratorParams &in, Pcg &rng, VolState &v) {
    const SI &si = v.si;
    const bool count_direct = v.depth == 0 || v.specular_chain;
    const uint32_t em = si.valid ? S.shapes[si.shape].emitter : S.environment;
    if (em != MH_INVALID && !(v.depth == 0 && in.hide_emitters)) {
        float emitter_pdf = 1.f;
        if (!count_direct) emitter_pdf = emitter_pdf_direction(S, em, si, v.last_p);
        const V3 emitted = emitter_eval(S, em, si);
        v.result = v.result + (count_direct ? v.throughput * emitted
                                            : (v.throughput * mis_weight(v.last_pdf, emitter_pdf)) * emitted);
    }
    v.active_surface = v.active_surface && si.valid;
    v.rho = v3(0, 0, 0);
    bool walk = false;
    if (v.active_surface) {
        const uint32_t b = S.shapes[si.shape].bsdf;
        const bool is_null = b == MH_INVALID || S.bsdf_type[b] == MH_BSDF_NULL;
        if (!is_null) v.rho = tex_eval(S, S.bsdf_tex[b], si.uvx, si.uvy);
        if (!is_null && v.depth + 1 < in.max_depth) {
            walk = nee_begin(S, si.p, si.n, &si, rng, v.medium, v.ds, v.ns);
            V3 bv;
            float bp;
            diffuse_eval_pdf(v.rho, si.wi, to_local(si, v.ds.d), true, bv, bp);
            const float w = mis_weight(v.ds.pdf, v.ds.delta ? 0.f : bp);
            v.pend = (v.throughput * bv) * w;
            v.nee_kind = kNeeSurface;
        }
    }
    return walk ? kPhWalk : vs_no_walk(S, in, rng, v);
}

// ---- the walk (nee_step, volpath.cpp:361-448) cut at its intersection ------
// common tail of a walk step; false when the walk has ended
MH_DEV bool walk_tail(const DScene &S, NeeState &ns, bool active_medium, bool escaped, bool active_surface0,
                      bool intersect, float remaining) {
    ns.needs_intersection = ns.needs_intersection && !intersect;
    bool active_surface = active_surface0 || escaped;
    if (active_surface) ns.total_dist += ns.si_t;
    active_surface = active_surface && ns.si.valid && !active_medium;
    if (active_surface) {
        const uint32_t b = S.shapes[ns.si.shape].bsdf;
        const float tn = (b != MH_INVALID && S.bsdf_type[b] == MH_BSDF_NULL) ? 1.f : 0.f;
        ns.transmittance = ns.transmittance * tn;
        ns.ray = spawn_ray(ns.si.p, ns.si.n, ns.ray.d);
    }
    ns.ray.maxt = remaining;
    ns.needs_intersection = ns.needs_intersection || active_surface;
    const bool active = (active_medium || active_surface) && nonzero(ns.transmittance);
    if (active_surface && is_medium_transition(S, ns.si)) ns.medium = target_medium(S, ns.si, ns.ray.d);
    return active;
}

// the medium part of a walk step after its (optional) intersection
MH_DEV bool walk_med_rest(const DScene &S, const DirS &ds, NeeState &ns, WMei &wm) {
    const float remaining = ns.max_dist - ns.total_dist;
    const DMedium &m = S.media[ns.medium];
    if (ns.si_t < wm.t) { wm.t = __builtin_huge_valf(); wm.valid = false; }
    ns.needs_intersection = ns.needs_intersection && !ns.si.valid;
    const bool spectral = !(m.flags & MH_MEDIUM_NO_SPECTRAL_EXTINCTION);
    if (spectral) {
        const float t = fminf(remaining, fminf(wm.t, ns.si_t)) - wm.mint;
        const float tr = exp_dr((-t) * wm.maj);
        const float pdf = (ns.si_t < wm.t || wm.t > remaining) ? tr : tr * wm.maj;
        ns.transmittance = ns.transmittance * (pdf > 0.f ? tr / pdf : 0.f);
    }
    if (wm.t > remaining && wm.valid) ns.total_dist = ds.dist;
    if (wm.t > remaining) { wm.t = __builtin_huge_valf(); wm.valid = false; }
    const bool escaped = !wm.valid, active_medium = wm.valid;
    if (active_medium) {
        ns.total_dist += wm.t;
        ns.ray.o = wm.p;
        ns.si_t = ns.si_t - wm.t;
        ns.transmittance = ns.transmittance * (spectral ? wm.sigma_n : wm.sigma_n / wm.maj);
    }
    return walk_tail(S, ns, active_medium, escaped, false, false, remaining);
}

// WALK: the start of a walk step, up to its intersection; cut at its medium
// sample like HEAD (pending: ns.medium, ns.ray and the draw u)
MH_DEV bool vs_walk_pre(const DScene &S, Pcg &rng, NeeState &ns, uint32_t &nph, float &u) {
    const float remaining = ns.max_dist - ns.total_dist;
    ns.ray.maxt = remaining;
    if (!(remaining > 0.f)) { nph = kPhPost; return false; }
    if (ns.medium != MH_INVALID) { u = rng.next_float(); return true; }
    if (ns.needs_intersection) { nph = kPhTraceWS; return false; }
    nph = walk_tail(S, ns, false, false, true, false, remaining) ? kPhWalk : kPhPost;
    return false;
}
MH_DEV uint32_t vs_walk_post(const DScene &S, const DirS &ds, NeeState &ns, WMei &wm, const MEI &mei) {
    const float remaining = ns.max_dist - ns.total_dist;
    const DMedium &m = S.media[ns.medium];
    if (m.type == MH_MEDIUM_HOMOGENEOUS && mei.valid) ns.ray.maxt = fminf(mei.t, remaining);
    wm.t = mei.t; wm.mint = mei.mint; wm.maj = mei.maj; wm.sigma_n = mei.sigma_n; wm.p = mei.p;
    wm.valid = mei.valid;
    if (ns.needs_intersection) return kPhTraceWM;
    return walk_med_rest(S, ds, ns, wm) ? kPhWalk : kPhPost;
}
MH_DEV uint32_t vs_walk(const DScene &S, Pcg &rng, const DirS &ds, NeeState &ns, WMei &wm) {
    uint32_t nph = kPhPost;
    float u = 0.f;
    if (!vs_walk_pre(S, rng, ns, nph, u)) return nph;
    MEI mei;
    sample_interaction(S, ns.medium, ns.ray, u, mei);
    return vs_walk_post(S, ds, ns, wm, mei);
}

// HEAD and WALK lanes in one trip: both end in a medium sample (a grid
// lookup, the trip's latency), so the pending lanes of both take it together
// at one call site instead of one wave trip each.  Per lane the operations
// and draws are vs_head's / vs_walk's.

// the ray of a HEAD / WALK lane's medium sample, as values
MH_DEV RayT vs_medium_ray(const VolState &v, bool head) {
    const RayT rh = v.ray, rw = v.ns.ray;
    RayT r;
    r.o = v3(head ? rh.o.x : rw.o.x, head ? rh.o.y : rw.o.y, head ? rh.o.z : rw.o.z);
    r.d = v3(head ? rh.d.x : rw.d.x, head ? rh.d.y : rw.d.y, head ? rh.d.z : rw.d.z);
    r.maxt = head ? rh.maxt : rw.maxt;
    return r;
}
MH_DEV uint32_t vs_medium_step(const DScene &S, const IntegratorParams &in, Pcg &rng, VolState &v, WMei &wm,
                               uint32_t ph, uint32_t &n_lookups) {
    uint32_t nph = kPhFree;
    float u = 0.f;
    const bool head = ph == kPhHead;
    const bool pend = head ? vs_head_pre(S, in, rng, v, nph, u) : vs_walk_pre(S, rng, v.ns, nph, u);
    if (!pend) return nph;
    // the request as a select of values (a select of the two fields'
    // addresses would pin the state in scratch)
    const uint32_t med = head ? v.medium : v.ns.medium;
    const RayT r = vs_medium_ray(v, head);
    MEI mei;  // the frame only at a real scatter (vs_scatter)
    n_lookups += sample_interaction<false>(S, med, r, u, mei) ? 1u : 0u;
    if (head) {
        v.mei = mei;
        nph = vs_head_post(S, in, rng, v);
    } else {
        nph = vs_walk_post(S, v.ds, v.ns, wm, mei);
    }
    return nph;
}

// TRACE: every lane pending an intersection traces it; then its continuation
MH_DEV uint32_t vs_trace_hit(const DScene &S, const IntegratorParams &in, Pcg &rng, uint32_t ph, VolState &v,
                             WMei &wm, const Hit &h, const RayT &ray, uint32_t &n_closest, uint32_t &n_shadow);
template <bool Pk>
MH_DEV uint32_t vs_trace(const DScene &S, const LdsBvh &B, const IntegratorParams &in, Pcg &rng, uint32_t ph,
                         VolState &v, WMei &wm, uint32_t &n_closest, uint32_t &n_shadow) {
    const bool walk = ph == kPhTraceWM || ph == kPhTraceWS;
    const RayT ray = walk ? v.ns.ray : v.ray;
    Hit h;
    if (Pk) h = packet_batch<false>(S.nodes, S.prims, S.prim_pairs, S.key_sp, B.stack - (threadIdx.x & 63u), B.stride,
                                    ray, true);
    else traverse<false>(B.nodes, B.prims, B.stack, B.stride, ray, h);
    return vs_trace_hit(S, in, rng, ph, v, wm, h, ray, n_closest, n_shadow);
}
// the ray a TRACE lane traces (selected as values, not as one of two fields)
MH_DEV RayT vs_trace_ray(const VolState &v, uint32_t ph) {
    const bool walk = ph == kPhTraceWM || ph == kPhTraceWS;
    const RayT a = v.ns.ray, b = v.ray;
    RayT r;
    r.o = v3(walk ? a.o.x : b.o.x, walk ? a.o.y : b.o.y, walk ? a.o.z : b.o.z);
    r.d = v3(walk ? a.d.x : b.d.x, walk ? a.d.y : b.d.y, walk ? a.d.z : b.d.z);
    r.maxt = walk ? a.maxt : b.maxt;
    return r;
}
// TRACE after the traversal: the hit's interaction, then its continuation
MH_DEV uint32_t vs_trace_si(const DScene &S, const IntegratorParams &in, Pcg &rng, uint32_t ph, VolState &v,
                            WMei &wm, const SI &si, float si_t, uint32_t &n_closest, uint32_t &n_shadow);
MH_DEV uint32_t vs_trace_hit(const DScene &S, const IntegratorParams &in, Pcg &rng, uint32_t ph, VolState &v,
                             WMei &wm, const Hit &h, const RayT &ray, uint32_t &n_closest, uint32_t &n_shadow) {
    SI si;
    float si_t;
    si_from_hit(S, ray, h, si, si_t);
    return vs_trace_si(S, in, rng, ph, v, wm, si, si_t, n_closest, n_shadow);
}
// the continuation of a TRACE lane from its hit's interaction
MH_DEV uint32_t vs_trace_si(const DScene &S, const IntegratorParams &in, Pcg &rng, uint32_t ph, VolState &v,
                            WMei &wm, const SI &si, float si_t, uint32_t &n_closest, uint32_t &n_shadow) {
    const bool walk = ph == kPhTraceWM || ph == kPhTraceWS;
    if (walk) {
        v.ns.si = si;
        v.ns.si_t = si_t;
        ++n_shadow;
        if (ph == kPhTraceWM) return walk_med_rest(S, v.ds, v.ns, wm) ? kPhWalk : kPhPost;
        const float remaining = v.ns.max_dist - v.ns.total_dist;
        return walk_tail(S, v.ns, false, false, true, true, remaining) ? kPhWalk : kPhPost;
    }
    v.si = si;
    v.si_t = si_t;
    ++n_closest;
    if (ph == kPhTraceM) return vs_med_rest(S, in, rng, v);
    return kPhSurf;
}

// ===========================================================================
// prbvolpath's primal (PRBVolpathIntegrator.sample, prbvolpath.py:91-431, mode
// primal) as the same phase machine: prbvol_sample<0>'s loop trip cut at its
// closest-hit queries and at every step of the ratio-tracked NEE walk
// (sample_emitter, :336-431).  The fork's own choices stay as the megakernel
// has them: emitter hits are not added (:216-234 commented out), the NEE ray
// is spawn_ray(ds.d) walked over ds.dist * (1 - ShadowEpsilon) (:357-371),
// the sensor medium is ignored (:123-124), homogeneous media get direct
// transmittance in the walk (:390-394).  Per lane the operations and random
// draws are those of prbvol_sample<0> in its order (bit-identical samples).
//   HEAD     RR, sample_interaction of the current medium
//   TRACE    the closest hit of the loop trip (TraceM: after the medium sample,
//            TraceS: the surface query) or of a walk segment (TraceWS)
//   SCATTER  a real scatter: the emitter sample that starts its walk
//   SURF     a surface hit: albedo, emitter sample
//   WALK     one trip of the transmittance loop up to its intersection
//   POST     the NEE contribution, phase / BSDF sampling
// A null collision (no scatter, no surface) returns to HEAD inside its trip.
// ===========================================================================
struct PvState {
    RayT ray;
    V3 throughput, L;
    SI si;
    float si_t, eta;
    uint32_t medium, depth;
    bool needs_intersection, valid_ray;
    // inside a loop trip
    bool active, active_medium, active_surface, act_scatter, smooth, e_surface, nee;
    uint32_t med;
    MEI mei;
    V3 rho, emitter_val, transmittance;
    DirS ds;
    // the walk (sample_emitter's loop)
    RayT wray;
    SI wsi;
    float wsi_t, total_dist;
    uint32_t wmedium;
    bool w_needs;
};

// The primal's hook points into the trip: no-ops.  The single-pass backward
// (PvBwdMachine below) logs and charges its adjoint terms at the same points.
struct PvNoHook {
    template <class V> MH_DEV void nee_begin(V &, const Pcg &) {}
    template <class V> MH_DEV void medium_log(const DScene &, V &, V3, bool, float, float, float) {}
    template <class V> MH_DEV void walk_step(V &, V3, float) {}
    template <class V>
    MH_DEV void nee_charge(const DScene &, const LdsBvh &, V &, const Pcg &, V3, V3, float, V3, uint32_t &) {}
    template <class V> MH_DEV void surface_log(const DScene &, V &, V3) {}
};

MH_DEV void pv_init(const DScene &S, const IntegratorParams &, Pcg &rng, RayT ray, PvState &v) {
    v.ray = ray;
    v.throughput = v3(1.f, 1.f, 1.f);
    v.L = v3(0.f, 0.f, 0.f);
    v.eta = 1.f;
    v.depth = 0;
    v.si.valid = false;
    v.si_t = 0.f;
    v.medium = MH_INVALID;   // "TODO: support sensors inside media" (prbvolpath.py:123-124)
    v.needs_intersection = true;
    v.valid_ray = false;
    (void)fminf(3.f * rng.next_float(), 2.f);   // RGB channel (scalar majorants: all channels alike)
}

// SURF / SCATTER: the surface block and the emitter sample (:212-270); the
// walk starts here, or the trip goes on to POST without one
template <class V, class Hk>
MH_DEV uint32_t pv_shade(const DScene &S, const IntegratorParams &in, Pcg &rng, V &v, Hk &hk) {
    v.active_surface = v.active_surface && v.si.valid;
    const uint32_t b = v.active_surface ? S.shapes[v.si.shape].bsdf : MH_INVALID;
    v.smooth = b != MH_INVALID && S.bsdf_type[b] == MH_BSDF_DIFFUSE;
    v.rho = v3(0.f, 0.f, 0.f);
    if (v.smooth) v.rho = tex_eval(S, S.bsdf_tex[b], v.si.uvx, v.si.uvy);
    v.e_surface = v.active_surface && v.smooth && v.depth + 1 < in.max_depth;
    const bool sample_emitters = v.med != MH_INVALID && !(S.media[v.med].flags & MH_MEDIUM_NO_EMITTER_SAMPLING);
    const bool e_medium = v.act_scatter && sample_emitters;
    v.nee = v.e_surface || e_medium;
    if (!v.nee) return kPhPost;
    // sample_emitter's head (pvp_sample_emitter: active_medium = e_medium)
    const V3 ref_p = e_medium ? v.mei.p : v.si.p;
    const V3 ref_n = e_medium ? v3(0.f, 0.f, 0.f) : v.si.n;
    hk.nee_begin(v, rng);  // sampler.clone() (prbvolpath.py: the NEE walk's replay)
    const float sx = rng.next_float(), sy = rng.next_float();
    v.emitter_val = scene_sample_emitter_direction(S, ref_p, sx, sy, v.ds);
    v.transmittance = v3(1.f, 1.f, 1.f);
    if (v.ds.pdf == 0.f) {  // emitted = 0
        v.emitter_val = v3(0.f, 0.f, 0.f);
        return kPhPost;
    }
    v.wmedium = v.medium;
    if (!e_medium && is_medium_transition(S, v.si)) v.wmedium = target_medium(S, v.si, v.ds.d);
    v.wray = spawn_ray(ref_p, ref_n, v.ds.d);
    v.total_dist = 0.f;
    v.wsi_t = 0.f;
    v.wsi.valid = false;
    v.w_needs = true;
    return kPhWalk;
}

// the loop trip after its medium block (:206-212), up to the surface query
template <class V, class Hk>
MH_DEV uint32_t pv_mid(const DScene &S, const IntegratorParams &in, V &v, bool act_null, bool escaped,
                       V3 weight, float P, float fw, float mt, Hk &hk) {
    v.active = v.active && v.depth < in.max_depth;
    v.act_scatter = v.act_scatter && v.active;
    if ((S.vol_flags & kVolHandleNull) && act_null) { v.ray.o = v.mei.p; v.si_t = v.si_t - v.mei.t; }
    if (v.act_scatter)
        weight = v3(weight.x * (v.mei.sigma_s.x / P), weight.y * (v.mei.sigma_s.y / P),
                    weight.z * (v.mei.sigma_s.z / P));
    v.throughput = v.throughput * weight;
    if (v.active_medium || escaped) hk.medium_log(S, v, weight, act_null, fw, mt, P);  // (:202-204)
    v.active_surface = v.active_surface || escaped;
    if (v.act_scatter) return kPhScatter;
    if (v.active_surface) return v.needs_intersection ? kPhTraceS : kPhSurf;
    // a null collision (or a scatter cut by max_depth): no surface, no NEE,
    // no sampling -- the loop's tail test (:331)
    v.valid_ray = v.valid_ray || v.act_scatter;
    return (v.active && v.active_medium) ? kPhHead : kPhFree;
}

// the medium block after its (optional) intersection (:165-204)
template <class V, class Hk>
MH_DEV uint32_t pv_med_rest(const DScene &S, const IntegratorParams &in, Pcg &rng, V &v, Hk &hk) {
    MEI &mei = v.mei;
    v.needs_intersection = false;
    if (v.si_t < mei.t) { mei.t = __builtin_huge_valf(); mei.valid = false; }
    const float mt = fminf(mei.t, v.si_t) - mei.mint;
    const float tr = exp_dr((-mt) * mei.maj);
    const float tr_pdf = v.si_t < mei.t ? tr : tr * mei.maj;
    const float fw = tr_pdf > 0.f ? tr / tr_pdf : 0.f;
    V3 weight = v3(fw, fw, fw);
    const bool escaped = !mei.valid;
    v.active_medium = mei.valid;
    bool act_null = false;
    float P = 1.f;
    if (S.vol_flags & kVolHandleNull) {
        P = mei.sigma_t / mei.maj;
        if (v.active_medium) act_null = rng.next_float() >= P;
        v.act_scatter = !act_null && v.active_medium;
        if (act_null) weight = weight * (mei.sigma_n / (1.f - P));
    } else {
        v.act_scatter = v.active_medium;
    }
    if (v.act_scatter) v.depth += 1;
    return pv_mid(S, in, v, act_null, escaped, weight, P, fw, mt, hk);
}

// HEAD: Russian roulette (:142-149) and the medium sample (:157-163), cut at
// the medium sample (as vs_head_pre: true with its draw u when one is
// pending for v.med / v.ray, else the next phase in nph)
template <class V, class Hk>
MH_DEV bool pv_head_pre(const DScene &S, const IntegratorParams &in, Pcg &rng, V &v, Hk &hk, uint32_t &nph, float &u) {
    bool active = nonzero(v.throughput);
    const float q = fminf(hmax(v.throughput) * (v.eta * v.eta), 0.99f);
    const bool perform_rr = v.depth > in.rr_depth;
    if (active) active = rng.next_float() < q || !perform_rr;
    if (perform_rr) v.throughput = v.throughput * rcp(q);
    if (!active) { nph = kPhFree; return false; }
    v.active = true;
    v.active_medium = v.medium != MH_INVALID;
    v.active_surface = !v.active_medium;
    v.act_scatter = false;
    v.nee = false;
    v.med = v.medium;
    MEI &mei = v.mei;
    mei.valid = false;
    mei.t = 0.f;
    mei.maj = 1.f;
    mei.sigma_t = 0.f;
    mei.p = v3(0.f, 0.f, 0.f);
    mei.sigma_s = v3(0.f, 0.f, 0.f);
    if (v.active_medium) { u = rng.next_float(); return true; }
    nph = pv_mid(S, in, v, false, false, v3(1.f, 1.f, 1.f), 1.f, 1.f, 0.f, hk);
    return false;
}
// the rest of HEAD once v.mei holds the medium sample
template <class V, class Hk>
MH_DEV uint32_t pv_head_post(const DScene &S, const IntegratorParams &in, Pcg &rng, V &v, Hk &hk) {
    const DMedium &m = S.media[v.med];
    if (m.type == MH_MEDIUM_HOMOGENEOUS && v.mei.valid) v.ray.maxt = v.mei.t;
    if (v.needs_intersection) return kPhTraceM;
    return pv_med_rest(S, in, rng, v, hk);
}
template <class V, class Hk>
MH_DEV uint32_t pv_head(const DScene &S, const IntegratorParams &in, Pcg &rng, V &v, Hk &hk) {
    uint32_t nph = kPhFree;
    float u = 0.f;
    if (!pv_head_pre(S, in, rng, v, hk, nph, u)) return nph;
    sample_interaction(S, v.med, v.ray, u, v.mei);
    return pv_head_post(S, in, rng, v, hk);
}

// the walk step after its (optional) intersection (pvp_sample_emitter's loop),
// from its medium sample on: mei holds it when the walk is in a medium
// (v.wmedium valid), else the defaults below
MH_DEV void pv_walk_mei_init(MEI &mei) {
    mei.valid = false;
    mei.t = 0.f;
    mei.maj = 1.f;
    mei.p = v3(0.f, 0.f, 0.f);
}
template <class V, class Hk>
MH_DEV uint32_t pv_walk_fin(const DScene &S, V &v, float remaining_dist, Hk &hk, MEI &mei) {
    v.w_needs = false;
    bool act_med = v.wmedium != MH_INVALID, act_surf = !act_med, escaped = false, hom = false;
    float hom_t = 0.f;
    V3 trm = v3(1.f, 1.f, 1.f);
    if (act_med) {
        const DMedium &m = S.media[v.wmedium];
        if (v.wsi_t < mei.t) { mei.t = __builtin_huge_valf(); mei.valid = false; }
        if ((S.vol_flags & kVolNeeHomogeneous) && m.type == MH_MEDIUM_HOMOGENEOUS) {
            mei.t = fminf(remaining_dist, v.wsi_t);
            hom_t = fminf(mei.t, v.wsi_t) - mei.mint;
            const float tr = exp_dr((-hom_t) * mei.maj);
            trm = v3(tr, tr, tr);
            hom = true;
            mei.t = __builtin_huge_valf();
            mei.valid = false;
        }
        escaped = !mei.valid;
        act_med = mei.valid;
        if (act_med) {
            v.wray.o = mei.p;
            v.wsi_t = v.wsi_t - mei.t;
            trm = trm * (mei.sigma_n / mei.maj);
        }
    }
    act_surf = (act_surf || escaped) && v.wsi.valid && !act_med;
    if (act_surf) {
        const uint32_t b = S.shapes[v.wsi.shape].bsdf;
        trm = trm * ((b != MH_INVALID && S.bsdf_type[b] == MH_BSDF_NULL) ? 1.f : 0.f);
    }
    if ((act_med || hom) && (act_med || act_surf)) {  // a gradient step of the walk (:412-414)
        const float tc = trm.x;  // grey: scalar sigma_n / majorant, scalar homogeneous tr
        hk.walk_step(v, mei.p, !(tc > 0.f) ? 0.f : act_med ? (1.f / tc) * (-1.f / mei.maj) : -hom_t);
    }
    v.transmittance = v.transmittance * trm;
    if (act_surf) v.wray = spawn_ray(v.wsi.p, v.wsi.n, v.wray.d);
    v.w_needs = act_surf;
    const bool active = (act_med || act_surf) && nonzero(v.transmittance);
    if (active) v.total_dist += act_med ? mei.t : v.wsi_t;
    if (act_surf && is_medium_transition(S, v.wsi)) v.wmedium = target_medium(S, v.wsi, v.wray.d);
    return active ? kPhWalk : kPhPost;
}
template <class V, class Hk>
MH_DEV uint32_t pv_walk_rest(const DScene &S, Pcg &rng, V &v, float remaining_dist, Hk &hk) {
    MEI mei;
    pv_walk_mei_init(mei);
    if (v.wmedium != MH_INVALID) sample_interaction(S, v.wmedium, v.wray, rng.next_float(), mei);
    return pv_walk_fin(S, v, remaining_dist, hk, mei);
}

MH_DEV float pv_remaining(const PvState &v) { return v.ds.dist * (1.f - kShadowEps) - v.total_dist; }

// WALK: the head of one transmittance-loop trip, cut at its medium sample
// (pending: v.wmedium, v.wray and the draw u)
template <class V, class Hk>
MH_DEV bool pv_walk_pre(const DScene &S, Pcg &rng, V &v, Hk &hk, uint32_t &nph, float &u) {
    const float remaining_dist = pv_remaining(v);
    v.wray.maxt = remaining_dist;
    if (!(remaining_dist > 0.f)) { nph = kPhPost; return false; }
    if (v.w_needs) { nph = kPhTraceWS; return false; }
    if (v.wmedium != MH_INVALID) { u = rng.next_float(); return true; }
    MEI mei;
    pv_walk_mei_init(mei);
    nph = pv_walk_fin(S, v, remaining_dist, hk, mei);
    return false;
}
template <class V, class Hk>
MH_DEV uint32_t pv_walk(const DScene &S, Pcg &rng, V &v, Hk &hk) {
    uint32_t nph = kPhPost;
    float u = 0.f;
    if (!pv_walk_pre(S, rng, v, hk, nph, u)) return nph;
    MEI mei;
    pv_walk_mei_init(mei);
    sample_interaction(S, v.wmedium, v.wray, u, mei);
    nph = pv_walk_fin(S, v, pv_remaining(v), hk, mei);
    return nph;
}

// HEAD and WALK lanes in one trip (vs_medium_step's form for prbvolpath)
template <class V, class Hk>
MH_DEV uint32_t pv_medium_step(const DScene &S, const IntegratorParams &in, Pcg &rng, V &v, Hk &hk, uint32_t ph) {
    uint32_t nph = kPhFree;
    float u = 0.f;
    const bool head = ph == kPhHead;
    const bool pend = head ? pv_head_pre(S, in, rng, v, hk, nph, u) : pv_walk_pre(S, rng, v, hk, nph, u);
    if (!pend) return nph;
    const uint32_t mh = v.med, mw = v.wmedium;
    const RayT rh = v.ray, rw = v.wray;
    RayT r;
    r.o = v3(head ? rh.o.x : rw.o.x, head ? rh.o.y : rw.o.y, head ? rh.o.z : rw.o.z);
    r.d = v3(head ? rh.d.x : rw.d.x, head ? rh.d.y : rw.d.y, head ? rh.d.z : rw.d.z);
    r.maxt = head ? rh.maxt : rw.maxt;
    MEI mei;
    pv_walk_mei_init(mei);
    sample_interaction(S, head ? mh : mw, r, u, mei);
    if (head) {
        v.mei = mei;
        return pv_head_post(S, in, rng, v, hk);
    }
    return pv_walk_fin(S, v, pv_remaining(v), hk, mei);
}

// POST: the emitter sample's contribution (:256-270), phase sampling
// (:274-294), BSDF sampling (:298-331) and the loop's tail test
template <class V, class Hk>
MH_DEV uint32_t pv_post(const DScene &S, const LdsBvh &B, const IntegratorParams &in, Pcg &rng, V &v, Hk &hk,
                        uint32_t &n_shadow) {
    if (v.nee) {
        const V3 emitted = v.emitter_val * v.transmittance;
        V3 nee_w, bv = v3(0.f, 0.f, 0.f);
        float nee_pdf, bp = 0.f;
        const V3 wo_s = to_local(v.si, v.ds.d);
        if (v.e_surface) {
            diffuse_eval_pdf(v.rho, v.si.wi, wo_s, true, bv, bp);
            nee_w = bv;
            nee_pdf = bp;
        } else {
            const float ph = phase_eval(S.media[v.med], mei_to_local(v.mei, v.ds.d));
            nee_w = v3(ph, ph, ph);
            nee_pdf = ph;
        }
        if (v.ds.delta) nee_pdf = 0.f;
        const float mis = mis_weight(v.ds.pdf, nee_pdf);
        const V3 contrib = ((v.throughput * nee_w) * mis) * emitted;
        v.L = v.L + contrib;
        hk.nee_charge(S, B, v, rng, contrib, emitted, mis, wo_s, n_shadow);
    }
    v.valid_ray = v.valid_ray || v.act_scatter;
    bool act_scatter = v.act_scatter;
    if (act_scatter) {
        (void)rng.next_float();
        const float s2x = rng.next_float(), s2y = rng.next_float();
        float ph_pdf;
        const V3 wo = phase_sample(S.media[v.med], s2x, s2y, ph_pdf);
        act_scatter = act_scatter && ph_pdf > 0.f;
        if (act_scatter) {
            v.ray = spawn_ray(v.mei.p, v3(0.f, 0.f, 0.f), mei_to_world(v.mei, wo));
            v.needs_intersection = true;
        }
    }
    if (v.active_surface) {
        (void)rng.next_float();
        const float s2x = rng.next_float(), s2y = rng.next_float();
        V3 bs_wo, bw;
        float bs_pdf;
        if (!v.smooth) {
            bs_wo = -v.si.wi; bs_pdf = 1.f; bw = v3(1.f, 1.f, 1.f);
        } else {
            bs_wo = square_to_cosine_hemisphere(s2x, s2y);
            bs_pdf = kInvPi * bs_wo.z;
            bw = (v.si.wi.z > 0.f && bs_pdf > 0.f) ? v.rho : v3(0.f, 0.f, 0.f);
        }
        v.active_surface = v.active_surface && bs_pdf > 0.f;
        if (v.active_surface) {
            if (v.smooth && v.si.wi.z > 0.f && bs_wo.z > 0.f) hk.surface_log(S, v, bs_wo);  // (:305-312)
            v.throughput = v.throughput * bw;
            v.ray = spawn_ray(v.si.p, v.si.n, to_world(v.si, bs_wo));
            v.needs_intersection = true;
            if (v.smooth) { v.depth += 1; v.valid_ray = true; }
            if (is_medium_transition(S, v.si)) v.medium = target_medium(S, v.si, v.ray.d);
        }
    }
    return (v.active && (v.active_surface || v.active_medium)) ? kPhHead : kPhFree;
}

// the wave-wide TRACE (k_vol_sched): the lane's ray, then its hit's continuation
template <class V>
MH_DEV RayT pv_trace_ray(const V &v, uint32_t ph) {
    const bool ws = ph == kPhTraceWS;
    const RayT a = v.wray, b = v.ray;
    RayT r;
    r.o = v3(ws ? a.o.x : b.o.x, ws ? a.o.y : b.o.y, ws ? a.o.z : b.o.z);
    r.d = v3(ws ? a.d.x : b.d.x, ws ? a.d.y : b.d.y, ws ? a.d.z : b.d.z);
    r.maxt = ws ? a.maxt : b.maxt;
    return r;
}
template <class V, class Hk>
MH_DEV uint32_t pv_trace_hit(const DScene &S, const IntegratorParams &in, Pcg &rng, uint32_t ph, V &v, const Hit &h,
                             const RayT &r, uint32_t &n_closest, uint32_t &n_shadow, Hk &hk) {
    if (ph == kPhTraceWS) {
        si_from_hit(S, r, h, v.wsi, v.wsi_t);
        ++n_shadow;
        return pv_walk_rest(S, rng, v, pv_remaining(v), hk);
    }
    si_from_hit(S, r, h, v.si, v.si_t);
    ++n_closest;
    if (ph == kPhTraceM) return pv_med_rest(S, in, rng, v, hk);
    return kPhSurf;
}
// the same from the hit's interaction
template <class V, class Hk>
MH_DEV uint32_t pv_trace_si(const DScene &S, const IntegratorParams &in, Pcg &rng, uint32_t ph, V &v, const SI &si,
                            float si_t, uint32_t &n_closest, uint32_t &n_shadow, Hk &hk) {
    if (ph == kPhTraceWS) {
        v.wsi = si;
        v.wsi_t = si_t;
        ++n_shadow;
        return pv_walk_rest(S, rng, v, pv_remaining(v), hk);
    }
    v.si = si;
    v.si_t = si_t;
    ++n_closest;
    if (ph == kPhTraceM) return pv_med_rest(S, in, rng, v, hk);
    return kPhSurf;
}
template <bool Pk, class V, class Hk>
MH_DEV uint32_t pv_trace(const DScene &S, const LdsBvh &B, const IntegratorParams &in, Pcg &rng, uint32_t ph,
                         V &v, uint32_t &n_closest, uint32_t &n_shadow, Hk &hk) {
    if (ph == kPhTraceWS) {
        trace_si<Pk>(S, B, v.wray, v.wsi, v.wsi_t);
        ++n_shadow;
        return pv_walk_rest(S, rng, v, pv_remaining(v), hk);
    }
    trace_si<Pk>(S, B, v.ray, v.si, v.si_t);
    ++n_closest;
    if (ph == kPhTraceM) return pv_med_rest(S, in, rng, v, hk);
    return kPhSurf;
}

// The integrators the phase scheduler runs: their state and phase steps.
// Every machine is constructed once per thread from the kernel's backward
// arguments (ignored by the primal machines) and offers the same calls.
#ifndef MH_VS_MERGE
#define MH_VS_MERGE 1
#endif
// prbvolpath's machines keep HEAD and WALK apart: merged (weight 4) the
// config-4 forward measured 24.1 vs 24.1-24.4 ms and the backward 62.9 vs
// 57.6 ms -- its walk steps alternate with their traces, so few walk lanes
// meet a HEAD trip, while the hooks lengthen the divergent halves
#ifndef MH_PV_MERGE
#define MH_PV_MERGE 0
#endif
#ifndef MH_PVB_MERGE
#define MH_PVB_MERGE 0
#endif
struct VolMachine {
    using State = VolState;
    // kMergeMed: HEAD and WALK lanes share a trip (vs_medium_step)
    static constexpr bool kPrb = false, kWritesPos = true, kDeferEnd = false, kMergeMed = MH_VS_MERGE != 0;
    MH_DEV VolMachine(const VsBwdArgs &, const LaneMap &, uint32_t) {}
    MH_DEV void init(const DScene &S, const IntegratorParams &in, Pcg &rng, RayT r, State &v, float, float) {
        volpath_init(S, in, rng, r, v);
    }
    MH_DEV uint32_t head(const DScene &S, const IntegratorParams &in, Pcg &rng, State &v) {
        return vs_head(S, in, rng, v);
    }
    template <bool Pk>
    MH_DEV uint32_t trace(const DScene &S, const LdsBvh &B, const IntegratorParams &in, Pcg &rng,
                          uint32_t ph, State &v, WMei &wm, uint32_t &nc, uint32_t &ns) {
        return vs_trace<Pk>(S, B, in, rng, ph, v, wm, nc, ns);
    }
    MH_DEV uint32_t scatter(const DScene &S, const IntegratorParams &in, Pcg &rng, State &v) {
        return vs_scatter(S, in, rng, v);
    }
    MH_DEV uint32_t surf(const DScene &S, const IntegratorParams &in, Pcg &rng, State &v) {
        return vs_surf(S, in, rng, v);
    }
    MH_DEV uint32_t walk(const DScene &S, Pcg &rng, State &v, WMei &wm) { return vs_walk(S, rng, v.ds, v.ns, wm); }
    MH_DEV uint32_t medium_step(const DScene &S, const IntegratorParams &in, Pcg &rng, State &v, WMei &wm, uint32_t ph,
                                uint32_t &n_lookups) {
        return vs_medium_step(S, in, rng, v, wm, ph, n_lookups);
    }
    MH_DEV RayT trace_ray(const State &v, uint32_t ph) const { return vs_trace_ray(v, ph); }
    MH_DEV uint32_t trace_hit(const DScene &S, const IntegratorParams &in, Pcg &rng, uint32_t ph, State &v, WMei &wm,
                              const Hit &h, const RayT &r, uint32_t &nc, uint32_t &ns) {
        return vs_trace_hit(S, in, rng, ph, v, wm, h, r, nc, ns);
    }
    MH_DEV uint32_t post(const DScene &S, const LdsBvh &, const IntegratorParams &in, Pcg &rng, State &v, uint32_t &) {
        return volpath_post(S, in, rng, v) ? kPhHead : kPhFree;
    }
    MH_DEV void end(const DScene &, const LdsBvh &, const IntegratorParams &, float *out, uint64_t plane,
                    uint32_t pid, const State &v, int alpha, uint32_t &, uint32_t &) {
        vw_write_sample(out, plane, pid, v, alpha);
    }
    MH_DEV void finish() {}
};

struct PvMachine {
    using State = PvState;
    static constexpr bool kPrb = true, kWritesPos = true, kDeferEnd = false, kMergeMed = MH_PV_MERGE != 0;
    PvNoHook h;
    MH_DEV PvMachine(const VsBwdArgs &, const LaneMap &, uint32_t) {}
    MH_DEV void init(const DScene &S, const IntegratorParams &in, Pcg &rng, RayT r, State &v, float, float) {
        pv_init(S, in, rng, r, v);
    }
    MH_DEV uint32_t head(const DScene &S, const IntegratorParams &in, Pcg &rng, State &v) {
        return pv_head(S, in, rng, v, h);
    }
    template <bool Pk>
    MH_DEV uint32_t trace(const DScene &S, const LdsBvh &B, const IntegratorParams &in, Pcg &rng,
                          uint32_t ph, State &v, WMei &, uint32_t &nc, uint32_t &ns) {
        return pv_trace<Pk>(S, B, in, rng, ph, v, nc, ns, h);
    }
    MH_DEV uint32_t scatter(const DScene &S, const IntegratorParams &in, Pcg &rng, State &v) {
        return pv_shade(S, in, rng, v, h);
    }
    MH_DEV uint32_t surf(const DScene &S, const IntegratorParams &in, Pcg &rng, State &v) {
        return pv_shade(S, in, rng, v, h);
    }
    MH_DEV uint32_t walk(const DScene &S, Pcg &rng, State &v, WMei &) { return pv_walk(S, rng, v, h); }
    MH_DEV uint32_t medium_step(const DScene &S, const IntegratorParams &in, Pcg &rng, State &v, WMei &, uint32_t ph,
                                uint32_t &) {
        return pv_medium_step(S, in, rng, v, h, ph);
    }
    MH_DEV RayT trace_ray(const State &v, uint32_t ph) const { return pv_trace_ray(v, ph); }
    MH_DEV uint32_t trace_hit(const DScene &S, const IntegratorParams &in, Pcg &rng, uint32_t ph, State &v, WMei &,
                              const Hit &hh, const RayT &r, uint32_t &nc, uint32_t &ns) {
        return pv_trace_hit(S, in, rng, ph, v, hh, r, nc, ns, h);
    }
    MH_DEV uint32_t post(const DScene &S, const LdsBvh &B, const IntegratorParams &in, Pcg &rng, State &v,
                         uint32_t &ns) {
        return pv_post(S, B, in, rng, v, h, ns);
    }
    MH_DEV void end(const DScene &, const LdsBvh &, const IntegratorParams &, float *out, uint64_t plane,
                    uint32_t pid, const State &v, int alpha, uint32_t &, uint32_t &) {
        out[pid] = v.L.x;
        out[plane + pid] = v.L.y;
        out[2 * plane + pid] = v.L.z;
        if (alpha) out[5 * plane + pid] = v.valid_ray ? 1.f : 0.f;  // aovs[3] (integrator.cpp:1229-1231)
    }
    MH_DEV void finish() {}
};

// ===========================================================================
// prbvolpath's single-pass backward (k_prbvol_backward's Mode 2: primal
// arithmetic, the L-dependent adjoint terms logged per vertex in MainLog and
// charged when the path ends, the NEE walks' gradient steps logged in NeeLog
// and charged once the NEE contribution is known; prbvolpath.py:91-431 with
// common.py:900-983) on the phase scheduler: the primal machine above with
// its hooks filled in.  A path whose MainLog overflows replays its adjoint
// when it ends (Mode 3, the NEE terms already charged); a walk whose NeeLog
// overflows (more than nee_cap steps, or a second medium) is replayed with
// the sampler cloned at its emitter sample (prbvolpath.py:412-414).  Both
// replays run after the scheduler launch from overflow lists (inlined, their
// register demand -- a whole adjoint sample -- would set the scheduler loop's
// allocation: 256 VGPRs with spills instead of 222 without).  Per lane the
// operations and draws are those of the per-sample kernel.
// ===========================================================================
struct PvBwdState : PvState {
    V3 dL;                     // grad_in / W gathered over the sample's footprint (common.py:936-965)
    uint64_t nee_state;        // the PCG32 state at the current emitter sample (sampler.clone())
    uint32_t ml_n, nl_n, nl_med;
    bool ml_over, nl_over;
};

#ifdef MH_EXP_VSCNT
// diagnostic build: PvBwdMachine's POST / END sub-phases (s_memtime cycles per
// wave, summed over the waves; read by mh_exp_vs_sub):
//   [0] POST per-lane code (pv_post)      [1] POST wave loop (post_wave)
//   [2]   its NeeLog entry loads           [3]   its sigma_t scatters
//   [4]   NeeLog entries charged           [5] END per-lane code (end)
//   [6] END wave loop (end_wave)           [7]   its MainLog entry loads
//   [8]   its log-entry charges            [9]   MainLog entries charged
//   [10] post_wave loop steps              [11] end_wave loop steps
//   [12] TRACE trips' packet traversal     [13] TRACE trips' hit continuations (every machine)
__device__ unsigned long long g_vs_sub[16];
#define MH_VS_SUB_DECL uint64_t sub[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#define MH_VS_SUB(k, v) (sub[k] += (uint64_t)(v))
#define MH_VS_T() __builtin_amdgcn_s_memtime()
#define MH_VS_SUB_AT(m, k, v) ((m).sub[k] += (uint64_t)(v))
#else
#define MH_VS_SUB_DECL
#define MH_VS_SUB(k, v) ((void)0)
#define MH_VS_T() 0ull
#endif
struct PvBwdMachine {
    using State = PvBwdState;
    MH_VS_SUB_DECL
    // the end-of-path log application is a phase of its own (kPhEnd): run
    // when a path ends, it would hold the wave for the few lanes that ended
    static constexpr bool kPrb = true, kWritesPos = false, kDeferEnd = true, kMergeMed = MH_PVB_MERGE != 0;
    VsBwdArgs a;
    GradCtx g;
    LaneMap lm;
    // The logs of a lane are contiguous (entry j of thread t: MainLog at
    // float4 (t * main_cap + j) * 4, NeeLog at t * nee_cap + j): the lanes of a
    // scheduler trip sit at different entries, so the per-sample kernel's
    // entry-major layout (lanes writing their j-th entry as one 1-KiB run)
    // would scatter every 64-B entry over four lines here.
    uint32_t seed_value, t;
    // charges deferred to the wave-wide, load-balanced loops that follow the
    // trip's per-lane phase code (post_wave / end_wave): the NEE walk of a
    // POST lane (its NeeLog steps, K, medium) and the MainLog of an ended path
    uint32_t pend_walk = 0, pend_med = 0, pend_main = 0;
    float pend_K = 0.f;
    MH_DEV PvBwdMachine(const VsBwdArgs &a_, const LaneMap &lm_, uint32_t sv)
        : a(a_), g(make_grad_ctx(a_.ga)), lm(lm_), seed_value(sv) {
        t = blockIdx.x * blockDim.x + threadIdx.x;
    }
    MH_DEV uint64_t main_base() const { return (uint64_t)t * a.main_cap * 4; }
    MH_DEV uint64_t nee_base() const { return (uint64_t)t * a.nee_cap; }
    MH_DEV void log_main(State &v, float4 q0, float4 q1, float4 q2, float4 q3) {
        if (v.ml_n >= a.main_cap) { v.ml_over = true; return; }
        float4 *e = a.main_log + main_base() + (uint64_t)4 * v.ml_n;
        e[0] = q0;
        e[1] = q1;
        e[2] = q2;
        e[3] = q3;
        ++v.ml_n;
    }
    // ---- hooks (PvNoHook's points)
    MH_DEV void nee_begin(State &v, const Pcg &rng) {
        v.nee_state = rng.state;
        v.nl_n = 0;
        v.nl_over = false;
    }
    // backward(dL * weight * Lo), Lo = L / max(1e-8, weight) (prbvolpath.py:202-204), logged
    MH_DEV void medium_log(const DScene &S, State &v, V3 weight, bool act_null, float fw, float mt, float P) {
        const DMedium &m = S.media[v.med];
        const bool homog = m.type == MH_MEDIUM_HOMOGENEOUS;
        const float wc[3] = {weight.x, weight.y, weight.z}, dc[3] = {v.dL.x, v.dL.y, v.dL.z};
        const float al[3] = {m.albedo[0], m.albedo[1], m.albedo[2]};
        const float ss[3] = {v.mei.sigma_s.x, v.mei.sigma_s.y, v.mei.sigma_s.z};
        const float dfw = homog ? -mt * fw : 0.f;  // d (tr / tr_pdf) / d sigma_t
        float dwsc[3], dwa = 0.f;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            float dws;
            if (v.act_scatter) {
                dws = dfw * ss[c] / P + fw * al[c] / P;  // sigma_s = sigma_t * albedo
                dwa = fw * v.mei.sigma_t / P;
            } else if (act_null) {
                dws = -fw / (1.f - P);
            } else {
                dws = dfw;
            }
            dwsc[c] = dws;
        }
        log_main(v, make_float4(v.mei.p.x, v.mei.p.y, v.mei.p.z, __uint_as_float((v.act_scatter ? 2u : 0u) | (v.med << 2))),
                 make_float4(v.L.x, v.L.y, v.L.z, 0.f),
                 make_float4(dc[0] / fmaxf(1e-8f, wc[0]), dc[1] / fmaxf(1e-8f, wc[1]), dc[2] / fmaxf(1e-8f, wc[2]), 0.f),
                 make_float4(dwsc[0], dwsc[1], dwsc[2], dwa));
    }
    MH_DEV void walk_step(State &v, V3 p, float coef) {
        if (v.nl_n < a.nee_cap && (v.nl_n == 0 || v.nl_med == v.wmedium)) {
            a.nee_log[nee_base() + v.nl_n] = make_float4(p.x, p.y, p.z, coef);
            v.nl_med = v.wmedium;
            ++v.nl_n;
        } else {
            v.nl_over = true;
        }
    }
    MH_DEV void nee_charge(const DScene &S, const LdsBvh &B, State &v, const Pcg &rng, V3 contrib, V3 emitted,
                           float mis, V3 wo_s, uint32_t &n_shadow) {
        if (!v.nl_over) {  // the logged walk's steps: coef * (dL . adj_emitted), in post_wave
            pend_K = (v.dL.x * contrib.x + v.dL.y * contrib.y) + v.dL.z * contrib.z;
            pend_walk = v.nl_n;
            pend_med = v.nl_med;
        } else {  // the walk is replayed with the cloned sampler after the launch (k_pvb_replay_walks)
            const bool am = !v.e_surface;
            const V3 rp = am ? v.mei.p : v.si.p, rn = am ? v3(0.f, 0.f, 0.f) : v.si.n;
            const uint32_t k = atomicAdd(a.ovf_count + 1, 1u);
            if (k < a.ovf_cap) {
                float4 *r = a.ovf_walks + (uint64_t)kPvbWalkRec * k;
                r[0] = make_float4(rp.x, rp.y, rp.z, __uint_as_float(v.si.shape));
                r[1] = make_float4(rn.x, rn.y, rn.z, __uint_as_float((am ? 1u : 0u) | (v.si.valid ? 2u : 0u)));
                r[2] = make_float4(contrib.x, contrib.y, contrib.z, __uint_as_float(v.medium));
                r[3] = make_float4(v.dL.x, v.dL.y, v.dL.z, 0.f);
                r[4] = make_float4(__uint_as_float((uint32_t)v.nee_state), __uint_as_float((uint32_t)(v.nee_state >> 32)),
                                   __uint_as_float((uint32_t)rng.inc), __uint_as_float((uint32_t)(rng.inc >> 32)));
            } else {
                atomicAdd(a.ovf_count + 2, 1u);
            }
        }
        if (v.e_surface && v.si.wi.z > 0.f && wo_s.z > 0.f) {
            // backward(dL * contrib) through bsdf_val = rho / pi * cos
            const V3 adj = ((((v.dL * emitted) * mis) * v.throughput) * kInvPi) * wo_s.z;
            tex_backward(S, S.bsdf_tex[S.shapes[v.si.shape].bsdf], v.si.uvx, v.si.uvy, adj, g);
        }
    }
    // Lo = bsdf_eval * detach(L / max(1e-8, bsdf_eval)) (prbvolpath.py:305-312), logged
    MH_DEV void surface_log(const DScene &S, State &v, V3 bs_wo) {
        const V3 be = (v.rho * kInvPi) * bs_wo.z;
        log_main(v, make_float4(0.f, 0.f, 0.f, __uint_as_float(1u | (S.bsdf_tex[S.shapes[v.si.shape].bsdf] << 2))),
                 make_float4(v.L.x, v.L.y, v.L.z, v.si.uvx),
                 make_float4(v.dL.x / fmaxf(1e-8f, be.x), v.dL.y / fmaxf(1e-8f, be.y), v.dL.z / fmaxf(1e-8f, be.z), v.si.uvy),
                 make_float4(bs_wo.z, 0.f, 0.f, 0.f));
    }
    // ---- the machine
    MH_DEV void init(const DScene &S, const IntegratorParams &in, Pcg &rng, RayT r, State &v, float sx, float sy) {
        v.dL = gather_dL_wave(S, a.coalesce, a.grad_in, sx, sy);  // grad_in: pre-divided by W (k_grad_over_w)
        pv_init(S, in, rng, r, v);
        v.ml_n = v.nl_n = v.nl_med = 0;
        v.ml_over = v.nl_over = false;
    }
    MH_DEV uint32_t head(const DScene &S, const IntegratorParams &in, Pcg &rng, State &v) {
        return pv_head(S, in, rng, v, *this);
    }
    template <bool Pk>
    MH_DEV uint32_t trace(const DScene &S, const LdsBvh &B, const IntegratorParams &in, Pcg &rng,
                          uint32_t ph, State &v, WMei &, uint32_t &nc, uint32_t &ns) {
        return pv_trace<Pk>(S, B, in, rng, ph, v, nc, ns, *this);
    }
    MH_DEV uint32_t scatter(const DScene &S, const IntegratorParams &in, Pcg &rng, State &v) {
        return pv_shade(S, in, rng, v, *this);
    }
    MH_DEV uint32_t surf(const DScene &S, const IntegratorParams &in, Pcg &rng, State &v) {
        return pv_shade(S, in, rng, v, *this);
    }
    MH_DEV uint32_t walk(const DScene &S, Pcg &rng, State &v, WMei &) { return pv_walk(S, rng, v, *this); }
    MH_DEV uint32_t medium_step(const DScene &S, const IntegratorParams &in, Pcg &rng, State &v, WMei &, uint32_t ph,
                                uint32_t &) {
        return pv_medium_step(S, in, rng, v, *this, ph);
    }
    MH_DEV RayT trace_ray(const State &v, uint32_t ph) const { return pv_trace_ray(v, ph); }
    MH_DEV uint32_t trace_hit(const DScene &S, const IntegratorParams &in, Pcg &rng, uint32_t ph, State &v, WMei &,
                              const Hit &hh, const RayT &r, uint32_t &nc, uint32_t &ns) {
        return pv_trace_hit(S, in, rng, ph, v, hh, r, nc, ns, *this);
    }
    MH_DEV uint32_t post(const DScene &S, const LdsBvh &B, const IntegratorParams &in, Pcg &rng, State &v,
                         uint32_t &ns) {
        return pv_post(S, B, in, rng, v, *this, ns);
    }
    // the path ended with radiance v.L: charge its logged terms, or replay
    MH_DEV void end(const DScene &S, const LdsBvh &B, const IntegratorParams &in, float *, uint64_t, uint32_t pid,
                    State &v, int, uint32_t &nc, uint32_t &ns) {
        if (!v.ml_over) {  // charged by end_wave in this trip
            pend_main = v.ml_n;
            return;
        }
        // the adjoint replayed after the launch (k_pvb_replay_paths)
        const uint32_t k = atomicAdd(a.ovf_count, 1u);
        if (k < a.ovf_cap) {
            a.ovf_paths[2 * (uint64_t)k] = make_float4(v.L.x, v.L.y, v.L.z, __uint_as_float(pid));
            a.ovf_paths[2 * (uint64_t)k + 1] = make_float4(v.dL.x, v.dL.y, v.dL.z, 0.f);
        } else {
            atomicAdd(a.ovf_count + 2, 1u);
        }
    }
    MH_DEV void finish() { flush_small_slots(g, a.ga); }
    // ---- the wave-wide charge loops (every lane of the wave active)
    MH_DEV uint64_t wave_t0() const { return (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); }
    MH_DEV void post_wave(const DScene &S) {
        const uint64_t t0 = wave_t0();
        const uint32_t cnt = pend_walk, med = pend_med;
        const float K = pend_K;
        pend_walk = 0;
        wave_flat(cnt, flat_scratch(), [&](uint32_t o, uint32_t e, bool valid) {
            const float Ko = __shfl(K, (int)o);
            const uint32_t mo = (uint32_t)__shfl((int)med, (int)o);
            const uint64_t ta = MH_VS_T();
            if (valid) {
                const float4 q = a.nee_log[(t0 + o) * a.nee_cap + e];
#ifdef MH_EXP_VSCNT
                asm volatile("" ::"v"(q.x), "v"(q.y), "v"(q.z), "v"(q.w));  // the load's wait here
                MH_VS_SUB(2, MH_VS_T() - ta);
#endif
                const uint64_t tb = MH_VS_T();
                sigma_t_backward(S, mo, v3(q.x, q.y, q.z), q.w * Ko, g);
                MH_VS_SUB(3, MH_VS_T() - tb);
                (void)tb;
            }
            MH_VS_SUB(4, __popcll(__ballot(valid)));
            MH_VS_SUB(10, 1);
            (void)ta;
        });
    }
    MH_DEV void end_wave(const DScene &S, const State &v) {
        const uint64_t t0 = wave_t0();
        const uint32_t cnt = pend_main;
        pend_main = 0;
        wave_flat(cnt, flat_scratch(), [&](uint32_t o, uint32_t e, bool valid) {
            const V3 L = v3(__shfl(v.L.x, (int)o), __shfl(v.L.y, (int)o), __shfl(v.L.z, (int)o));
            const uint64_t ta = MH_VS_T();
            if (valid) {  // MainLog entry e of thread t0 + o: float4 (t * main_cap + e) * 4
                const float4 *q = a.main_log + ((t0 + o) * a.main_cap + e) * 4u;
#ifdef MH_EXP_VSCNT
                const float4 q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
                asm volatile("" ::"v"(q0.x), "v"(q1.x), "v"(q2.x), "v"(q3.x), "v"(q3.w));
                MH_VS_SUB(7, MH_VS_T() - ta);
                const uint64_t tb = MH_VS_T();
                pvp_log_entry(S, q0, q1, q2, q3, L, g);
                MH_VS_SUB(8, MH_VS_T() - tb);
#else
                pvp_log_entry(S, q[0], q[1], q[2], q[3], L, g);
#endif
            }
            MH_VS_SUB(9, __popcll(__ballot(valid)));
            MH_VS_SUB(11, 1);
            (void)ta;
        });
    }
#ifdef MH_EXP_VSCNT
    MH_DEV void sub_flush() {
        if ((threadIdx.x & 63u) == 0)
            for (int k = 0; k < 12; ++k) atomicAdd(&g_vs_sub[k], sub[k]);
    }
#endif
};

#ifndef MH_VS_WAVES
#define MH_VS_WAVES 2
#endif
constexpr uint32_t kVsCtrLookups = 27;  // mh_api.hip kCtrLookups: the density-grid lookups of the launch
// TRACE as one wave-wide packet traversal with sparse-run deferral (packet scenes)
#ifndef MH_VS_DEFER
#define MH_VS_DEFER 1
#endif
__host__ __device__ inline uint32_t vs_defer_bytes(const DScene &S) {
    return MH_VS_DEFER ? 16u + align16(S.n_prims * kPairRecFloats * 4u) + 4u * kDeferScratch : 0u;
}
// phase weights (x16): a phase runs when its pending lanes x weight is the
// largest; heavy phases wait for more lanes
#ifndef MH_VS_W
// free, head, trace, scatter, surf, walk, post, end (swept on config 4: 194 -> 214 Msamples/s;
// trace 12 -> 8 re-swept after the wave-wide TRACE: 32 / 20 / 12 / 8 / 6 / 4 -> 240 / 244 / 246 / 247 / 246 / 242)
#define MH_VS_W 8, 16, 8, 8, 8, 6, 12, 16
#endif
// the weight of the merged HEAD + WALK group (machines with kMergeMed; swept
// on config 4: 16 -> 190, 6 -> 226, 4 -> 233, 3 -> 234 Msamples/s; with the
// wave-wide TRACE at weight 8: 6 -> 237, 4 -> 246, 3 -> 250.5)
#ifndef MH_VS_MERGE_W
#define MH_VS_MERGE_W 3
#endif
// Tab: the shading tables (stage_tables) and the media records staged into
// LDS: every trip reads the medium record (transform, bbox, majorant,
// albedo) and the surface trips walk shape -> bsdf -> texture / emitter
// chains; from global memory each of those is a dependent L2 round trip
// (~20 per trip), from LDS ~100 cycles.
__host__ __device__ inline uint32_t vs_media_bytes(const DScene &S) { return (S.n_media * (uint32_t)sizeof(DMedium) + 15u) & ~15u; }
__host__ __device__ inline uint32_t vs_tab_bytes(const DScene &S) { return ((S.tab_bytes + 15u) & ~15u) + vs_media_bytes(S); }

template <class M, bool InLds, bool Pk, bool Tab>
__global__ void __launch_bounds__(256u, MH_VS_WAVES)
k_vol_sched(DScene S0, IntegratorParams in, LaneMap lm, uint32_t seed_value, uint64_t n, uint64_t plane,
            float *__restrict__ out, unsigned long long *__restrict__ counters, unsigned long long *__restrict__ work,
            int alpha, VsBwdArgs bw) {
    // samples are handed out in batches of 64 from one device counter (work)
    extern __shared__ uint4 lds[];
    DScene S = S0;
    uint32_t tab = 0;
    if (Tab) {
        S = stage_tables(S0, lds);
        const uint32_t mo = (S0.tab_bytes + 15u) & ~15u;
        uint8_t *mb = reinterpret_cast<uint8_t *>(lds) + mo;
        lds_copy(mb, S0.media, S0.n_media * (uint32_t)sizeof(DMedium));
        __syncthreads();
        S.media = reinterpret_cast<const DMedium *>(mb);
        tab = vs_tab_bytes(S0) / 16u;
    }
    LdsBvh B = stage_bvh<InLds>(S0, lds + tab);
    if (Pk && MH_VS_DEFER) {  // pair records + deferral scratch after the stacks (vs_defer_bytes)
        const uint32_t off = (tab * 16u + S0.lds_bytes_bvh + S0.stack_size * blockDim.x * 4u + 15u) & ~15u;
        float *recs = reinterpret_cast<float *>(reinterpret_cast<uint8_t *>(lds) + off);
        stage_pair_records(S0, recs);
        __syncthreads();
        B.recs = recs;
        B.dscr = reinterpret_cast<uint8_t *>(recs) + align16(S0.n_prims * kPairRecFloats * 4u) + (threadIdx.x >> 6) * kDeferScratch;
    }
    constexpr uint32_t W0[kNGroups] = {MH_VS_W};
    uint32_t W[kNGroups];
#pragma unroll
    for (uint32_t k = 0; k < kNGroups; ++k) W[k] = (M::kMergeMed && k == kGHead) ? (uint32_t)MH_VS_MERGE_W : W0[k];
    constexpr uint32_t NG = M::kDeferEnd ? kNGroups : kGEnd;  // groups this machine uses
    const float sw = S.inv_width, sh = S.inv_height;
    uint32_t n_closest = 0, n_shadow = 0, n_lookups = 0;
    M mc(bw, lm, seed_value);
    typename M::State v;
    WMei wm;
    Pcg rng;
    uint32_t pid = 0, ph = kPhFree;
    // XCD-aware work queues.  Workgroups are dispatched round-robin over the
    // 8 XCDs (b % 8), and each XCD has its own 4-MiB L2, while the grid of
    // config 4 is 64 MiB.  Queue x holds the samples of the x-th column band
    // of the chunk's rows (contiguous eighths when the chunk is not whole
    // rows); an XCD serves its own queue first, then the others', so its
    // paths -- and the NEE walks up toward a sun that stays in the band's
    // x-slab -- touch about an eighth of the medium.
    const uint32_t xcd = blockIdx.x & 7u;
    const uint32_t Wd = lm.W;
    const uint64_t S_ = lm.S, npx = n / S_;
    const bool bands = Wd >= 8u && lm.pixel_begin % Wd == 0u && npx % Wd == 0u && npx * S_ == n;
    const uint32_t rows = bands ? (uint32_t)(npx / Wd) : 0u;
    const uint64_t part = (n + 7u) / 8u;
    auto q_size = [&](uint32_t q) -> uint64_t {
        if (bands) return (uint64_t)rows * ((q + 1u) * Wd / 8u - q * Wd / 8u) * S_;
        const uint64_t lo = (uint64_t)q * part;
        return lo >= n ? 0ull : std::min<uint64_t>(part, n - lo);
    };
    auto q_sample = [&](uint32_t q, uint64_t i) -> uint64_t {  // queue-local index -> chunk sample
        if (!bands) return (uint64_t)q * part + i;
        const uint32_t c0 = q * Wd / 8u, bw = (q + 1u) * Wd / 8u - c0;
        const uint64_t j = i / S_, sidx = i - j * S_;
        const uint64_t r = j / bw, c = c0 + (j - r * bw);
        return (r * Wd + c) * S_ + sidx;
    };
    uint32_t cq = 0, tried = 0;  // wave-uniform: queue of the current batch, queues exhausted so far
    uint64_t next = 0, end = 0;  // wave-uniform: the wave's current batch [next, end) of queue cq
    bool drained = false;        // wave-uniform: every queue is exhausted
#ifdef MH_EXP_VSCNT
    unsigned long long d_trips[kNGroups] = {}, d_lanes[kNGroups] = {}, d_ticks[kNGroups] = {};
    unsigned long long d_trace[2] = {0, 0};  // TRACE trips: the packet traversal, the hits' continuations
#endif
    while (true) {
        uint32_t cnt[kNGroups];
        const uint32_t g = (M::kMergeMed && ph == kPhWalk) ? (uint32_t)kGHead : ph_group(ph);
#pragma unroll
        for (uint32_t k = 0; k < NG; ++k) cnt[k] = (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(g == k));
        if (drained && next >= end) cnt[kGFree] = 0;
        uint32_t sel = kNGroups, best = 0;
#pragma unroll
        for (uint32_t k = 0; k < NG; ++k)
            if (cnt[k] * W[k] > best) { best = cnt[k] * W[k]; sel = k; }
        if (sel == kNGroups) break;  // no lane holds a path and the range is done
#ifdef MH_EXP_VSCNT  // diagnostic build: wave trips, lanes and shader cycles per phase (in registers)
#pragma unroll
        for (uint32_t k = 0; k < kNGroups; ++k)
            if (sel == k) { d_trips[k] += 1; d_lanes[k] += cnt[k]; }
        const uint64_t t_phase = __builtin_amdgcn_s_memtime();
#endif
        bool ended = false;
        if (sel == kGFree) {
            while (next >= end && tried < 8u) {  // take the next batch of 64 samples: own queue first
                const uint32_t q = (xcd + tried) & 7u;
                uint64_t b = 0;
                if (vw_lane() == 0) b = atomicAdd(work + 16u * q, 64ull);
                b = __builtin_amdgcn_readfirstlane((uint32_t)b) | ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32);
                const uint64_t qs = q_size(q);
                if (b < qs) {
                    cq = q;
                    next = b;
                    end = std::min<uint64_t>(b + 64u, qs);
                } else {
                    ++tried;
                }
            }
            drained = tried >= 8u;
            const unsigned long long m = __builtin_amdgcn_ballot_w64(ph == kPhFree);
            if (ph == kPhFree) {
                const uint64_t i = next + (uint64_t)__popcll(m & ((1ull << vw_lane()) - 1ull));
                if (i < end) {
                    const uint64_t k = q_sample(cq, i);
                    pid = (uint32_t)k;
                    uint32_t lane, px, py;
                    lane_of(lm, k, lane, px, py);
                    rng.seed(seed_value, lane);
                    const float sx = (float)px + rng.next_float(), sy = (float)py + rng.next_float();
                    const RayT r = camera_ray(S, __builtin_fmaf(sx, sw, -0.f), __builtin_fmaf(sy, sh, -0.f));
                    if (M::kWritesPos) {
                        out[3 * plane + k] = sx;
                        out[4 * plane + k] = sy;
                    }
                    mc.init(S, in, rng, r, v, sx, sy);
                    ph = kPhHead;
                }
            }
            next = std::min<uint64_t>(end, next + (uint64_t)__popcll(m));
        } else if (sel == kGHead) {
            if constexpr (M::kMergeMed) {
                if (g == kGHead) { ph = mc.medium_step(S, in, rng, v, wm, ph, n_lookups); ended = ph == kPhFree; }
            } else if (ph == kPhHead) {
                ph = mc.head(S, in, rng, v);
                ended = ph == kPhFree;
            }
        } else if (sel == kGTrace) {
            if constexpr (Pk && MH_VS_DEFER) {
                // every lane of the wave in the traversal (the deferral hands
                // sparse leaves' (ray, pair) items to all 64 lanes); TRACE lanes
                // carry their rays, the others ride along inactive
                const bool act = g == kGTrace;
                RayT r{v3(0.f, 0.f, 0.f), v3(0.f, 0.f, 1.f), -1.f};
                if (act) r = mc.trace_ray(v, ph);
#ifdef MH_EXP_VSCNT
                const uint64_t tt0 = __builtin_amdgcn_s_memtime();
#endif
                const Hit h = packet_batch<false, true>(S.nodes, S.prims, S.prim_pairs, S.key_sp,
                                                        B.stack - (threadIdx.x & 63u), B.stride, r, act, B.recs, B.dscr);
#ifdef MH_EXP_VSCNT
                asm volatile("" ::"v"(h.t), "v"(h.prim));  // the traversal's results are in
                const uint64_t tt1 = __builtin_amdgcn_s_memtime();
                d_trace[0] += tt1 - tt0;
#endif
                if (act) {
                    ph = mc.trace_hit(S, in, rng, ph, v, wm, h, r, n_closest, n_shadow);
                    ended = ph == kPhFree;
                }
#ifdef MH_EXP_VSCNT
                d_trace[1] += __builtin_amdgcn_s_memtime() - tt1;
#endif
            } else if (g == kGTrace) {
                ph = mc.template trace<Pk>(S, B, in, rng, ph, v, wm, n_closest, n_shadow);
                ended = ph == kPhFree;
            }
        } else if (sel == kGScatter) {
            if (ph == kPhScatter) { ph = mc.scatter(S, in, rng, v); ended = ph == kPhFree; }
        } else if (sel == kGSurf) {
            if (ph == kPhSurf) { ph = mc.surf(S, in, rng, v); ended = ph == kPhFree; }
        } else if (sel == kGWalk) {
            if (ph == kPhWalk) ph = mc.walk(S, rng, v, wm);
        } else if (sel == kGPost) {
#ifdef MH_EXP_VSCNT
            const uint64_t tp0 = __builtin_amdgcn_s_memtime();
#endif
            if (ph == kPhPost) { ph = mc.post(S, B, in, rng, v, n_shadow); ended = ph == kPhFree; }
            if constexpr (M::kDeferEnd) {
#ifdef MH_EXP_VSCNT
                const uint64_t tp1 = __builtin_amdgcn_s_memtime();
                mc.post_wave(S);
                MH_VS_SUB_AT(mc, 0, tp1 - tp0);
                MH_VS_SUB_AT(mc, 1, __builtin_amdgcn_s_memtime() - tp1);
#else
                mc.post_wave(S);
#endif
            }
        } else if (M::kDeferEnd) {
#ifdef MH_EXP_VSCNT
            const uint64_t te0 = __builtin_amdgcn_s_memtime();
#endif
            if (ph == kPhEnd) {
                mc.end(S, B, in, out, plane, pid, v, alpha, n_closest, n_shadow);
                ph = kPhFree;
            }
            if constexpr (M::kDeferEnd) {
#ifdef MH_EXP_VSCNT
                const uint64_t te1 = __builtin_amdgcn_s_memtime();
                mc.end_wave(S, v);
                MH_VS_SUB_AT(mc, 5, te1 - te0);
                MH_VS_SUB_AT(mc, 6, __builtin_amdgcn_s_memtime() - te1);
#else
                mc.end_wave(S, v);
#endif
            }
        }
        if (ended) {
            if (M::kDeferEnd) ph = kPhEnd;
            else mc.end(S, B, in, out, plane, pid, v, alpha, n_closest, n_shadow);
        }
#ifdef MH_EXP_VSCNT
        {
            const uint64_t dt = __builtin_amdgcn_s_memtime() - t_phase;
#pragma unroll
            for (uint32_t k = 0; k < kNGroups; ++k)
                if (sel == k) d_ticks[k] += dt;
        }
#endif
    }
    mc.finish();
#ifdef MH_EXP_VSCNT
    if constexpr (M::kDeferEnd) mc.sub_flush();
#endif
    if (counters) {
        wave_count(&counters[0], n_closest);
        wave_count(&counters[1], n_shadow);
        wave_count(&counters[kVsCtrLookups], n_lookups);
    }
#ifdef MH_EXP_VSCNT
    if (vw_lane() == 0) {
        atomicAdd(&g_vs_sub[12], d_trace[0]);
        atomicAdd(&g_vs_sub[13], d_trace[1]);
    }
    if (vw_lane() == 0 && counters)
        for (uint32_t k = 0; k < kNGroups; ++k) {
            atomicAdd(&counters[2 + k], d_trips[k]);
            atomicAdd(&counters[2 + kNGroups + k], d_lanes[k]);
            atomicAdd(&counters[2 + 2 * kNGroups + k], d_ticks[k]);
        }
#endif
}

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
// volpath execution: phase-scheduled persistent kernel (default) or
// main / walk rounds (MH_VOL_MODE=rounds)
bool vol_sched_mode() {
    const char *e = getenv("MH_VOL_MODE");
    return !(e && !strcmp(e, "rounds"));
}
uint32_t vs_blocks(int cus) {
    uint32_t bpc = MH_VS_WAVES;  // one resident round of 256-lane workgroups (a wave per SIMD each)
    if (const char *e = getenv("MH_VS_BPC")) bpc = std::max(1, atoi(e));
    return (uint32_t)cus * bpc;
}
uint64_t vw_max_chunk() { return 1ull << 23; }
size_t vw_workspace_bytes(uint64_t cap) { return (size_t)2 * kVwPlanes * 16 * cap; }
uint32_t vw_counter_words(uint32_t rounds) { return kVwCtr * (rounds + 1); }
uint32_t vw_rounds(const IntegratorParams &in) { return in.max_depth + 1; }
bool vw_supported(const DScene &S, const IntegratorParams &in) {
    return in.type == MH_INTEGRATOR_VOLPATH && in.max_depth <= 1024 && S.n_media < 255;
}
// the phase scheduler runs volpath and prbvolpath's primal (the rounds mode
// only volpath)
bool vs_supported(const DScene &S, const IntegratorParams &in) {
    return (in.type == MH_INTEGRATOR_VOLPATH || in.type == MH_INTEGRATOR_PRBVOLPATH) && in.max_depth <= 1024 &&
           S.n_media < 255;
}
uint32_t vw_blocks(int cus) {
    uint32_t bpc = 8;
    if (const char *e = getenv("MH_VW_BPC")) bpc = std::max(1, atoi(e));
    return std::max<uint32_t>(kVwSeg, (uint32_t)cus * bpc / kVwSeg * kVwSeg);
}

hipError_t launch_vol_sched(const DScene &S, const IntegratorParams &in, const LaneMap &lm, uint32_t seed_value,
                            uint64_t n, uint64_t plane, float *out, uint32_t grid, unsigned long long *counters,
                            hipStream_t st, int alpha) {
    if (n == 0) return hipSuccess;
    const size_t sh = lds_bytes(S, 256);
    const bool lds = S.lds_bytes_bvh != 0;
    const char *te = getenv("MH_TRAVERSAL");
    const bool pk = S.n_prims > 0 && S.n_prims <= wf_packet_max_prims() && !(te && !strcmp(te, "lane"));
    const bool tab = S.tab_bytes != 0 && !getenv("MH_VS_NOTAB");
#define MH_VS1(Mc, L, P, T)                                                                                   \
    hipLaunchKernelGGL((k_vol_sched<Mc, L, P, T>), dim3(grid), dim3(256), sh + (T ? vs_tab_bytes(S) : 0u) + (P ? vs_defer_bytes(S) : 0u), st, S, \
                       in, lm, seed_value, n, plane, out, counters, work, alpha, VsBwdArgs{})
#define MH_VS(L, P, T)                                                  \
    do {                                                                \
        if (in.type == MH_INTEGRATOR_PRBVOLPATH) MH_VS1(PvMachine, L, P, T); \
        else MH_VS1(VolMachine, L, P, T);                               \
    } while (0)
    unsigned long long *work = counters + 32;  // the 8 queue heads of this launch (128 B apart)
    hipError_t e = hipMemsetAsync(work, 0, 8 * 128, st);
    if (e != hipSuccess) return e;
    if (pk && tab) MH_VS(false, true, true);
    else if (pk) MH_VS(false, true, false);
    else if (lds) MH_VS(true, false, false);
    else MH_VS(false, false, false);
#undef MH_VS
#undef MH_VS1
    return hipGetLastError();
}

#ifdef MH_EXP_VSCNT
extern "C" int mh_exp_vs_sub(unsigned long long *out, int reset) {
    hipMemcpyFromSymbol(out, HIP_SYMBOL(g_vs_sub), sizeof(g_vs_sub));
    if (reset) {
        unsigned long long z[16] = {0};
        hipMemcpyToSymbol(HIP_SYMBOL(g_vs_sub), z, sizeof(z));
    }
    return 0;
}
#endif

// prbvolpath's single-pass backward on the phase scheduler: n samples of the
// lane map, gradients into bw.ga's slot buffers (k_prbvol_backward's Mode 2)
hipError_t launch_vol_sched_bwd(const DScene &S, const IntegratorParams &in, const LaneMap &lm, uint32_t seed_value,
                                uint64_t n, const VsBwdArgs &bw, uint32_t grid, unsigned long long *counters,
                                hipStream_t st) {
    if (n == 0) return hipSuccess;
    if (in.type != MH_INTEGRATOR_PRBVOLPATH || !bw.main_log || !bw.nee_log || !bw.main_cap || !bw.nee_cap)
        return hipErrorInvalidValue;
    const size_t sh = lds_bytes(S, 256);
    const bool lds = S.lds_bytes_bvh != 0;
    const char *te = getenv("MH_TRAVERSAL");
    const bool pk = S.n_prims > 0 && S.n_prims <= wf_packet_max_prims() && !(te && !strcmp(te, "lane"));
    const bool tab = S.tab_bytes != 0 && !getenv("MH_VS_NOTAB");
    unsigned long long *work = counters + 32;  // the 8 queue heads of this launch (128 B apart)
    hipError_t e = hipMemsetAsync(work, 0, 8 * 128, st);
    if (e != hipSuccess) return e;
#define MH_VSB(L, P, T)                                                                                        \
    hipLaunchKernelGGL((k_vol_sched<PvBwdMachine, L, P, T>), dim3(grid), dim3(256), sh + (T ? vs_tab_bytes(S) : 0u) + (P ? vs_defer_bytes(S) : 0u), \
                       st, S, in, lm, seed_value, n, (uint64_t)0, (float *)nullptr, counters, work, 0, bw)
    if (pk && tab) MH_VSB(false, true, true);
    else if (pk) MH_VSB(false, true, false);
    else if (lds) MH_VSB(true, false, false);
    else MH_VSB(false, false, false);
#undef MH_VSB
    return hipGetLastError();
}

// A path whose MainLog overflowed: its adjoint replayed with L = its radiance
// (prbvol_sample Mode 3, the NEE terms already charged), as k_prbvol_backward
// does in place.
template <bool InLds>
__global__ void __launch_bounds__(256)
k_pvb_replay_paths(DScene S, IntegratorParams in, LaneMap lm, uint32_t seed_value, VsBwdArgs bw,
                   unsigned long long *counters) {
    extern __shared__ uint4 lds[];
    LdsBvh B = stage_bvh<InLds>(S, lds);
    GradCtx g = make_grad_ctx(bw.ga);
    uint32_t nc = 0, ns = 0;
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < min(*bw.ovf_count, bw.ovf_cap)) {
        const float4 e = bw.ovf_paths[2 * (uint64_t)k], d = bw.ovf_paths[2 * (uint64_t)k + 1];
        uint32_t lane, px, py;
        lane_of(lm, __float_as_uint(e.w), lane, px, py);
        Pcg r;
        r.seed(seed_value, lane);
        const float sx = (float)px + r.next_float(), sy = (float)py + r.next_float();
        const RayT ray = camera_ray(S, __builtin_fmaf(sx, S.inv_width, -0.f),
                                    __builtin_fmaf(sy, S.inv_height, -0.f));
        prbvol_sample<3>(S, B, in, r, ray, v3(d.x, d.y, d.z), v3(e.x, e.y, e.z), &g, nc, ns);
    }
    flush_small_slots(g, bw.ga);
    if (counters) {
        wave_count(&counters[0], nc);
        wave_count(&counters[1], ns);
    }
}

// An NEE walk whose NeeLog overflowed: replayed with the sampler cloned at its
// emitter sample, back-propagating dL * adj_emitted through every
// tr_multiplier (prbvolpath.py:412-414; pvp_sample_emitter Mode 1).  The walk
// reads of its vertex only the reference point, normal and shape.
template <bool InLds>
__global__ void __launch_bounds__(256)
k_pvb_replay_walks(DScene S, VsBwdArgs bw, unsigned long long *counters) {
    extern __shared__ uint4 lds[];
    LdsBvh B = stage_bvh<InLds>(S, lds);
    GradCtx g = make_grad_ctx(bw.ga);
    uint32_t ns = 0;
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < min(*(bw.ovf_count + 1), bw.ovf_cap)) {
        const float4 *r = bw.ovf_walks + (uint64_t)kPvbWalkRec * k;
        const float4 r0 = r[0], r1 = r[1], r2 = r[2], r3 = r[3], r4 = r[4];
        const uint32_t flags = __float_as_uint(r1.w);
        MEI mei;
        mei.p = v3(r0.x, r0.y, r0.z);
        SI si;
        si.valid = (flags & 2u) != 0;
        si.p = mei.p;
        si.n = v3(r1.x, r1.y, r1.z);
        si.shape = __float_as_uint(r0.w);
        Pcg rng;
        rng.state = (uint64_t)__float_as_uint(r4.x) | ((uint64_t)__float_as_uint(r4.y) << 32);
        rng.inc = (uint64_t)__float_as_uint(r4.z) | ((uint64_t)__float_as_uint(r4.w) << 32);
        DirS ds;
        pvp_sample_emitter<1>(S, B, mei, si, (flags & 1u) != 0, rng, __float_as_uint(r2.w), ds,
                              v3(r2.x, r2.y, r2.z), v3(r3.x, r3.y, r3.z), &g, ns);
    }
    flush_small_slots(g, bw.ga);
    if (counters) wave_count(&counters[1], ns);
}

hipError_t launch_vol_sched_bwd_replays(const DScene &S, const IntegratorParams &in, const LaneMap &lm,
                                        uint32_t seed_value, uint64_t n, const VsBwdArgs &bw,
                                        unsigned long long *counters, hipStream_t st) {
    if (n == 0) return hipSuccess;
    // the lists' lengths stay on the device: every thread beyond them leaves at once
    const size_t sh = lds_bytes(S, 256);
    const uint32_t gp = (bw.ovf_cap + 255) / 256, gw = gp;
    if (S.lds_bytes_bvh) {
        hipLaunchKernelGGL(k_pvb_replay_paths<true>, dim3(gp), dim3(256), sh, st, S, in, lm, seed_value, bw, counters);
        hipLaunchKernelGGL(k_pvb_replay_walks<true>, dim3(gw), dim3(256), sh, st, S, bw, counters);
    } else {
        hipLaunchKernelGGL(k_pvb_replay_paths<false>, dim3(gp), dim3(256), sh, st, S, in, lm, seed_value, bw, counters);
        hipLaunchKernelGGL(k_pvb_replay_walks<false>, dim3(gw), dim3(256), sh, st, S, bw, counters);
    }
    return hipGetLastError();
}

// one chunk of n paths (single pass), all rounds queued on `st` without host
// synchronisation; rounds without work exit at their first instructions
hipError_t launch_volwave(const DScene &S, const IntegratorParams &in, const LaneMap &lm, uint32_t seed_value,
                          uint64_t n, uint64_t plane, float *out, void *ws, uint64_t cap, uint32_t *ctr,
                          uint32_t grid, unsigned long long *counters, hipStream_t st, int alpha) {
    if (n == 0) return hipSuccess;
    if (n > cap || n > 0xffffffffull) return hipErrorInvalidValue;
    const uint32_t rounds = vw_rounds(in);
    hipError_t e = hipMemsetAsync(ctr, 0, sizeof(uint32_t) * vw_counter_words(rounds), st);
    if (e != hipSuccess) return e;
    VwPlanes side[2];
    for (int k = 0; k < 2; ++k) {
        side[k].p = reinterpret_cast<float4 *>(ws) + (size_t)k * kVwPlanes * cap;
        side[k].cap = cap;
    }
    const uint32_t seg_cap = (uint32_t)((n + kVwSeg - 1) / kVwSeg);
    const size_t sh = lds_bytes(S, 256);
    const bool lds = S.lds_bytes_bvh != 0;
    // packet engine for scenes with pair records (MH_TRAVERSAL=lane: per-lane)
    const char *te = getenv("MH_TRAVERSAL");
    const bool pk = S.n_prims > 0 && S.n_prims <= wf_packet_max_prims() && !(te && !strcmp(te, "lane"));
    // main / walk rounds while many paths are live, then one finish launch
    uint32_t wave_rounds = kVwWaveRounds;
    if (const char *e = getenv("MH_VW_ROUNDS")) wave_rounds = (uint32_t)std::max(1, atoi(e));
    for (uint32_t r = 0; r < rounds; ++r) {
        const VwPlanes &c = side[r & 1], &x = side[(r + 1) & 1];
        const uint32_t *cin = ctr + (size_t)kVwCtr * r;
        uint32_t *cout = ctr + (size_t)kVwCtr * (r + 1);
        if (r == wave_rounds) {
#define MH_VW_FIN(L, P) \
    hipLaunchKernelGGL((k_vw_finish<L, P>), dim3(grid), dim3(256), sh, st, S, in, plane, out, c, seg_cap, cin, counters, alpha)
            if (pk) MH_VW_FIN(false, true);
            else if (lds) MH_VW_FIN(true, false);
            else MH_VW_FIN(false, false);
#undef MH_VW_FIN
            break;
        }
#define MH_VW_MAIN(F, L, P)                                                                                   \
    hipLaunchKernelGGL((k_vw_main<F, L, P>), dim3(grid), dim3(256), sh, st, S, in, lm, seed_value, n, plane, out, \
                       c, x, seg_cap, cin, cout, counters, alpha)
#define MH_VW_WALK(L, P) \
    hipLaunchKernelGGL((k_vw_walk<L, P>), dim3(grid), dim3(256), sh, st, S, x, seg_cap, cout, counters)
        if (pk) {
            if (r == 0) MH_VW_MAIN(true, false, true);
            else MH_VW_MAIN(false, false, true);
        } else if (r == 0) {
            if (lds) MH_VW_MAIN(true, true, false); else MH_VW_MAIN(true, false, false);
        } else {
            if (lds) MH_VW_MAIN(false, true, false); else MH_VW_MAIN(false, false, false);
        }
        if (r + 1 == rounds) break;  // depth < max_depth: no walk after the last round
        if (pk) MH_VW_WALK(false, true);
        else if (lds) MH_VW_WALK(true, false);
        else MH_VW_WALK(false, false);
#undef MH_VW_MAIN
#undef MH_VW_WALK
    }
    return hipGetLastError();
}

}  // namespace mh
