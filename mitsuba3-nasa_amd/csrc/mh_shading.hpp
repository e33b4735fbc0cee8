// mh_shading.hpp — per-lane device functions of the hot path shared by the
// megakernels (mh_kernels.hip) and the wavefront kernels (mh_wavefront.hip):
// BVH2 traversal (the OptiX slot), SurfaceInteraction, textures, diffuse
// BSDF, area emitter, perspective camera, and the per-lane path / prb loops.
#pragma once

#include "mh_device.hpp"
#include "mh_internal.hpp"

namespace mh {

// ===========================================================================
// BVH traversal (replaces OptiX; payload = scene_optix.inl:619-657)
// ===========================================================================
struct Hit {
    float t, u, v;
    uint32_t prim, shape;
    uint32_t key;  // scene-order key of the hit primitive (exact-t tie-break)
};

struct RayT {
    V3 o, d;
    float maxt;
};

// Moeller-Trumbore (render/mesh.h:430-453), e1/e2 precomputed bit-identically
MH_DEV bool tri_test_v(V3 v0, V3 e1, V3 e2, const RayT &r, float &t, float &u, float &v) {
    V3 pvec = cross(r.d, e2);
    float inv_det = rcp(dot(e1, pvec));
    V3 tvec = r.o - v0;
    u = dot(tvec, pvec) * inv_det;
    V3 qvec = cross(tvec, e1);
    v = dot(r.d, qvec) * inv_det;
    t = dot(e2, qvec) * inv_det;
    // Non-short-circuit masks: every lane evaluates the whole test, so the
    // compiler emits v_cmp/s_and instead of exec-mask branches.
    return (u >= 0.f) & (u <= 1.f) & (v >= 0.f) & (u + v <= 1.f) & (t >= 0.f) & (t <= r.maxt);
}
MH_DEV bool tri_test(const Prim &p, const RayT &r, float &t, float &u, float &v) {
    return tri_test_v(v3(p.a.x, p.a.y, p.a.z), v3(p.b.x, p.b.y, p.b.z), v3(p.c.x, p.c.y, p.c.z), r, t, u, v);
}

// Rectangle::ray_intersect_preliminary_impl (shapes/rectangle.cpp:446-470)
MH_DEV bool rect_test(const Prim &p, const RayT &r, float &t, float &u, float &v) {
    const float m[12] = {p.a.x, p.a.y, p.a.z, p.a.w, p.b.x, p.b.y, p.b.z, p.b.w,
                         p.c.x, p.c.y, p.c.z, p.c.w};
    V3 o = xf_point(m, r.o), d = xf_vector(m, r.d);
    t = -o.z / d.z;
    V3 local = fma3s(d, t, o);
    u = local.x;
    v = local.y;
    return (t >= 0.f) & (t <= r.maxt) & (__builtin_fabsf(local.x) <= 1.f) &
           (__builtin_fabsf(local.y) <= 1.f);
}

MH_DEV bool prim_test(const Prim &p, const RayT &r, float &t, float &u, float &v) {
    return p.info.z == MH_SHAPE_RECTANGLE ? rect_test(p, r, t, u, v) : tri_test(p, r, t, u, v);
}

// Reciprocal direction for the slab test.  A zero component (axis-aligned
// rays) would give inf * 0 = NaN in `o * inv`; it is replaced by a tiny
// same-signed value, which keeps the (padded, conservative) box test exact
// in outcome.  The primitive tests still use the true direction.
MH_DEV float safe_rcp_dir(float d) {
    const float e = 0x1p-80f;
    return rcp(__builtin_fabsf(d) > e ? d : __builtin_copysignf(e, d));
}
MH_DEV V3 safe_inv_dir(V3 d) { return v3(safe_rcp_dir(d.x), safe_rcp_dir(d.y), safe_rcp_dir(d.z)); }

// Closest-hit update rule.  Exact-t ties (coincident surfaces, e.g. a cube
// standing on the floor) resolve to the lowest (shape, prim) — the scene
// order in which the oracle's brute force (and a scalar scene walk) meets
// them — so the result does not depend on the BVH's visiting order.
MH_DEV bool closer(float tt, const Prim &p, const Hit &hit) {
    return (tt < hit.t) | ((tt == hit.t) & (p.info.w < hit.key));
}

// Slab test for both children; conservative (host pads every box).
MH_DEV void box2(const Node &n, V3 inv, V3 ood, float tmax, bool &h0, bool &h1, float &t0,
                 float &t1) {
    float a0 = __builtin_fmaf(n.lo0.x, inv.x, -ood.x), b0 = __builtin_fmaf(n.hi0.x, inv.x, -ood.x);
    float a1 = __builtin_fmaf(n.lo0.y, inv.y, -ood.y), b1 = __builtin_fmaf(n.hi0.y, inv.y, -ood.y);
    float a2 = __builtin_fmaf(n.lo0.z, inv.z, -ood.z), b2 = __builtin_fmaf(n.hi0.z, inv.z, -ood.z);
    float lo = fmaxf(fmaxf(fminf(a0, b0), fminf(a1, b1)), fmaxf(fminf(a2, b2), 0.f));
    float hi = fminf(fminf(fmaxf(a0, b0), fmaxf(a1, b1)), fminf(fmaxf(a2, b2), tmax));
    h0 = lo <= hi;
    t0 = lo;
    a0 = __builtin_fmaf(n.lo1.x, inv.x, -ood.x); b0 = __builtin_fmaf(n.hi1.x, inv.x, -ood.x);
    a1 = __builtin_fmaf(n.lo1.y, inv.y, -ood.y); b1 = __builtin_fmaf(n.hi1.y, inv.y, -ood.y);
    a2 = __builtin_fmaf(n.lo1.z, inv.z, -ood.z); b2 = __builtin_fmaf(n.hi1.z, inv.z, -ood.z);
    lo = fmaxf(fmaxf(fminf(a0, b0), fminf(a1, b1)), fmaxf(fminf(a2, b2), 0.f));
    hi = fminf(fminf(fmaxf(a0, b0), fmaxf(a1, b1)), fminf(fmaxf(a2, b2), tmax));
    h1 = lo <= hi;
    t1 = lo;
}

// Closest hit (Shadow = false) or any hit (Shadow = true).  `stk` points at
// this lane's column of the LDS stack (entry k at stk[k * stride]).
template <bool Shadow>
MH_DEV bool traverse(const Node *nodes, const Prim *prims, uint32_t *stk, uint32_t stride,
                     const RayT &r, Hit &hit) {
    V3 inv = safe_inv_dir(r.d);
    V3 ood = r.o * inv;
    float best = r.maxt;
    hit.t = __builtin_huge_valf();
    hit.u = hit.v = 0.f;
    hit.prim = MH_INVALID;
    hit.shape = MH_INVALID;
    hit.key = MH_INVALID;
    if (nodes == nullptr) return false;  // scene without primitives
    uint32_t sp = 0;
    uint32_t node = 0;
    // a root that is itself a leaf is encoded as node 0 with lo0.w = first prim
    while (true) {
        const Node n = nodes[node];
        bool h0, h1;
        float t0, t1;
        box2(n, inv, ood, best, h0, h1, t0, t1);
        uint32_t c0 = __float_as_uint(n.lo0.w), n0 = __float_as_uint(n.hi0.w) & kLeafCountMask;
        uint32_t c1 = __float_as_uint(n.lo1.w), n1 = __float_as_uint(n.hi1.w) & kLeafCountMask;
        // leaves are tested immediately
        if (h0 && n0) {
            for (uint32_t i = 0; i < n0; ++i) {
                const Prim p = prims[c0 + i];
                float t, u, v;
                if (prim_test(p, r, t, u, v) && (Shadow || closer(t, p, hit))) {
                    if (Shadow) return true;
                    hit.t = t; hit.u = u; hit.v = v; hit.prim = p.info.y; hit.shape = p.info.x; hit.key = p.info.w;
                    best = t;
                }
            }
            h0 = false;
        }
        if (h1 && n1) {
            for (uint32_t i = 0; i < n1; ++i) {
                const Prim p = prims[c1 + i];
                float t, u, v;
                if (prim_test(p, r, t, u, v) && (Shadow || closer(t, p, hit))) {
                    if (Shadow) return true;
                    hit.t = t; hit.u = u; hit.v = v; hit.prim = p.info.y; hit.shape = p.info.x; hit.key = p.info.w;
                    best = t;
                }
            }
            h1 = false;
        }
        if (h0 && h1) {
            uint32_t near_c = c0, far_c = c1;
            if (t1 < t0) { near_c = c1; far_c = c0; }
            stk[sp * stride] = far_c;
            ++sp;
            node = near_c;
        } else if (h0) {
            node = c0;
        } else if (h1) {
            node = c1;
        } else {
            if (sp == 0) break;
            --sp;
            node = stk[sp * stride];
        }
    }
    return hit.shape != MH_INVALID;
}

// LDS staging of the BVH (nodes then prims) — one copy per workgroup.
struct LdsBvh {
    const Node *nodes;
    const Node4 *nodes4;  // wide BVH (global memory), nullptr when absent
    const QNode4 *qnodes; // quantised wide BVH + compact primitives (global memory), nullptr when absent
    const PrimC *primsc;
    const Prim *prims;
    uint32_t *stack;  // this lane's column
    uint32_t stride;
    // packet engine with sparse-run deferral (k_vol_sched): LDS pair records and
    // this wave's deferral scratch (nullptr: dense packet tests only)
    const float *recs = nullptr;
    uint8_t *dscr = nullptr;
    // the stream engine's stack beyond `scap` LDS entries: this lane's column
    // of the scene's overflow region (DScene::stack_ovf), stride sgstride
    uint32_t scap = 0;
    uint32_t *sglb = nullptr;
    uint32_t sgstride = 0;
    // the LDS column through an LDS-qualified pointer: with the generic one
    // the compiler merged the two branches into one flat access, and a flat
    // pop waits for every outstanding load (vmcnt(0) lgkmcnt(0))
    MH_DEV __attribute__((address_space(3))) uint32_t *lstack() const {
        return (__attribute__((address_space(3))) uint32_t *)stack;
    }
    MH_DEV void push(uint32_t sp, uint32_t v) const {
        if (__builtin_expect(sp >= scap, 0)) {
            sglb[(sp - scap) * sgstride] = v;
            return;
        }
        lstack()[sp * stride] = v;
    }
    // the LDS read is unconditional (index clamped) and the overflow read a
    // wave-uniform branch that waits for it inside, so the common pop waits
    // for its ds_read only, not for the wave's outstanding node loads
    MH_DEV uint32_t pop(uint32_t sp) const {
        uint32_t v = lstack()[min(sp, scap - 1u) * stride];
        if (__builtin_expect(__ballot(sp >= scap) != 0, 0)) {
            uint32_t g = 0;
            if (sp >= scap) g = sglb[(sp - scap) * sgstride];
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) here, so the join needs none
            v = sp >= scap ? g : v;
        }
        return v;
    }
};

// InLds = true: BVH resident in LDS (compile-time choice, so hipcc emits
// ds_read for nodes/prims instead of flat loads); false: HBM/L2 via global.
template <bool InLds>
MH_DEV LdsBvh stage_bvh(const DScene &S, uint4 *lds) {
    LdsBvh b;
    const uint32_t nq = InLds ? S.lds_bytes_bvh / 16u : 0u;
    if (InLds) {
        const uint4 *src_nodes = reinterpret_cast<const uint4 *>(S.nodes);
        const uint4 *src_prims = reinterpret_cast<const uint4 *>(S.prims);
        const uint32_t nq_nodes = S.n_nodes * 4u;
        for (uint32_t i = threadIdx.x; i < nq; i += blockDim.x)
            lds[i] = i < nq_nodes ? src_nodes[i] : src_prims[i - nq_nodes];
        __syncthreads();
        b.nodes = S.n_prims ? reinterpret_cast<const Node *>(lds) : nullptr;
        b.prims = reinterpret_cast<const Prim *>(lds + nq_nodes);
    } else {
        b.nodes = S.n_prims ? S.nodes : nullptr;
        b.prims = S.prims;
    }
    b.nodes4 = InLds ? nullptr : S.nodes4;
    b.qnodes = InLds ? nullptr : S.qnodes;
    b.primsc = InLds ? nullptr : S.primsc;
    b.stack = reinterpret_cast<uint32_t *>(lds + nq) + threadIdx.x;
    b.stride = blockDim.x;
    // the stream engine: S.stream_stack entries in LDS (the launch allocates
    // stream_lds_bytes), the rest in the global overflow region
    const bool ovf = !InLds && S.stack_ovf != nullptr;
    b.scap = ovf ? S.stream_stack : S.stack_size;
    b.sglb = ovf ? S.stack_ovf + (blockIdx.x * blockDim.x + threadIdx.x) : nullptr;
    b.sgstride = S.ovf_threads;
    return b;
}
// dynamic LDS of the stream-engine kernels (k_wf_trace / k_wf_shadow /
// k_trace_*): the BVH when LDS-resident, and stream_stack entries per thread
__host__ __device__ inline size_t stream_lds_bytes(const DScene &S, uint32_t block) {
    return (size_t)S.lds_bytes_bvh + (size_t)(S.lds_bytes_bvh || !S.stack_ovf ? S.stack_size : S.stream_stack) * block * 4u;
}

// ---------------------------------------------------------------------------
// LDS staging of the small shading tables (shapes, BSDFs, textures,
// emitters, mesh vertices / normals / uvs / faces).  A shading lane walks a
// chain of dependent lookups (shape -> bsdf -> texture, shape -> face ->
// vertices, emitter -> shape); from LDS each link costs ~100 cycles instead
// of an L2 round trip.  The returned scene view points into LDS; callers
// instantiate this unconditionally (template) so hipcc emits ds_read.
// Layout and size: tab_layout (host and device agree).
// ---------------------------------------------------------------------------
struct TabLayout {
    uint32_t shapes, bsdf_type, bsdf_tex, textures, emitters, positions, normals, texcoords, faces, total;
};
__host__ __device__ inline TabLayout tab_layout(uint32_t n_shapes, uint32_t n_bsdfs, uint32_t n_textures,
                                                uint32_t n_emitters, uint32_t n_vertices, uint32_t n_faces,
                                                bool normals, bool texcoords) {
    auto al = [](uint32_t x) { return (x + 15u) & ~15u; };
    TabLayout L;
    uint32_t o = 0;
    L.shapes = o; o += al(n_shapes * (uint32_t)sizeof(DShape));
    L.bsdf_type = o; o += al(n_bsdfs * 4u);
    L.bsdf_tex = o; o += al(n_bsdfs * 4u);
    L.textures = o; o += al(n_textures * (uint32_t)sizeof(DTexture));
    L.emitters = o; o += al(n_emitters * (uint32_t)sizeof(DEmitter));
    L.positions = o; o += al(n_vertices * 12u);
    L.normals = o; o += normals ? al(n_vertices * 12u) : 0u;
    L.texcoords = o; o += texcoords ? al(n_vertices * 8u) : 0u;
    L.faces = o; o += al(n_faces * 12u);
    L.total = o;
    return L;
}

MH_DEV void lds_copy(uint8_t *dst, const void *src, uint32_t bytes) {
    const uint32_t *s = reinterpret_cast<const uint32_t *>(src);
    uint32_t *d = reinterpret_cast<uint32_t *>(dst);
    for (uint32_t i = threadIdx.x; i < bytes / 4u; i += blockDim.x) d[i] = s[i];
}

MH_DEV DScene stage_tables(const DScene &S, uint4 *lds) {
    DScene T = S;
    uint8_t *b = reinterpret_cast<uint8_t *>(lds);
    const bool has_n = S.normals != nullptr && S.n_vertices, has_t = S.texcoords != nullptr && S.n_vertices;
    const TabLayout L = tab_layout(S.n_shapes, S.n_bsdfs, S.n_textures, S.n_emitters, S.n_vertices, S.n_faces,
                                   has_n, has_t);
    lds_copy(b + L.shapes, S.shapes, S.n_shapes * (uint32_t)sizeof(DShape));
    lds_copy(b + L.bsdf_type, S.bsdf_type, S.n_bsdfs * 4u);
    lds_copy(b + L.bsdf_tex, S.bsdf_tex, S.n_bsdfs * 4u);
    lds_copy(b + L.textures, S.textures, S.n_textures * (uint32_t)sizeof(DTexture));
    lds_copy(b + L.emitters, S.emitters, S.n_emitters * (uint32_t)sizeof(DEmitter));
    lds_copy(b + L.positions, S.positions, S.n_vertices * 12u);
    if (has_n) lds_copy(b + L.normals, S.normals, S.n_vertices * 12u);
    if (has_t) lds_copy(b + L.texcoords, S.texcoords, S.n_vertices * 8u);
    lds_copy(b + L.faces, S.faces, S.n_faces * 12u);
    __syncthreads();
    T.shapes = reinterpret_cast<const DShape *>(b + L.shapes);
    T.bsdf_type = reinterpret_cast<const uint32_t *>(b + L.bsdf_type);
    T.bsdf_tex = reinterpret_cast<const uint32_t *>(b + L.bsdf_tex);
    T.textures = reinterpret_cast<const DTexture *>(b + L.textures);
    T.emitters = reinterpret_cast<const DEmitter *>(b + L.emitters);
    T.positions = reinterpret_cast<const float *>(b + L.positions);
    // unconditional (a select between LDS and global would force flat loads);
    // compute_si reads them only for shapes that have normals / uvs
    T.normals = reinterpret_cast<const float *>(b + L.normals);
    T.texcoords = reinterpret_cast<const float *>(b + L.texcoords);
    T.faces = reinterpret_cast<const uint32_t *>(b + L.faces);
    return T;
}

// rank of this lane among the lanes set in m below it (v_mbcnt_lo / _hi)
MH_DEV uint32_t lane_rank(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// ---------------------------------------------------------------------------
// Stream traversal engine for the wavefront kernels: while-while traversal
// (inner-node phase until every lane holds a leaf, then a grouped leaf phase)
// with per-lane ray refill from the wave's contiguous item range.  Same hit
// semantics as traverse<>: closest hit with t in [0, maxt], strict-< update.
// Stack entries: inner node index, or kLeafBit | first << 5 | count (count <= 31).
// ---------------------------------------------------------------------------
constexpr uint32_t kLeafBit = 0x80000000u;
constexpr uint32_t kNoNode = 0xffffffffu;  // pop next
constexpr uint32_t kDone = 0xfffffffeu;    // traversal complete

struct TravLane {
    V3 o, d, inv, ood;
    float maxt, best;
    uint32_t node, leaf, nleaf, sp;
    Hit hit;
};

MH_DEV void trav_init(TravLane &t, const RayT &r, bool empty_scene) {
    t.o = r.o;
    t.d = r.d;
    t.maxt = r.maxt;
    t.inv = safe_inv_dir(r.d);
    t.ood = r.o * t.inv;
    t.best = r.maxt;
    t.node = empty_scene ? kDone : 0u;
    t.nleaf = 0;
    t.leaf = 0;
    t.sp = 0;
    t.hit.t = __builtin_huge_valf();
    t.hit.u = t.hit.v = 0.f;
    t.hit.prim = MH_INVALID;
    t.hit.shape = MH_INVALID;
    t.hit.key = MH_INVALID;
}

// Does the lane take part in the next inner step?  It does while it has an
// inner node to visit or a stack to pop.  A lane already holding a postponed
// leaf keeps traversing inner nodes (speculative traversal, Aila & Laine
// 2009) until it meets a second leaf, which it keeps in `node`.
MH_DEV bool trav_wants(const TravLane &t) {
    if (t.node == kDone) return false;
    if (t.node == kNoNode) return t.sp != 0 || t.nleaf == 0;
    return !(t.node & kLeafBit);
}

// a leaf reference is taken into the empty leaf slot; otherwise it stays in
// `node` (processed after the held leaf)
MH_DEV void trav_take(TravLane &t, uint32_t ref) {
    if ((ref & kLeafBit) && t.nleaf == 0) {
        t.leaf = (ref & ~kLeafBit) >> 5;
        t.nleaf = ref & 31u;
        t.node = kNoNode;
    } else {
        t.node = ref;
    }
}

// one inner step: pop if needed, then visit one inner node
MH_DEV void trav_inner_step(TravLane &t, const Node *nodes, const LdsBvh &stk) {
    if (t.node == kNoNode) {
        if (t.sp == 0) { t.node = kDone; return; }  // (only reached without a held leaf)
        --t.sp;
        const uint32_t ref = stk.pop(t.sp);
        trav_take(t, ref);
        if (t.node == kNoNode || (t.node & kLeafBit)) return;
    }
    const Node n = nodes[t.node];
    bool h0, h1;
    float t0, t1;
    box2(n, t.inv, t.ood, t.best, h0, h1, t0, t1);
    const uint32_t c0 = __float_as_uint(n.lo0.w), n0 = __float_as_uint(n.hi0.w) & kLeafCountMask;
    const uint32_t c1 = __float_as_uint(n.lo1.w), n1 = __float_as_uint(n.hi1.w) & kLeafCountMask;
    const uint32_t r0 = n0 ? (kLeafBit | (c0 << 5) | n0) : c0;
    const uint32_t r1 = n1 ? (kLeafBit | (c1 << 5) | n1) : c1;
    if (h0 && h1) {
        const bool swap = t1 < t0;
        stk.push(t.sp, swap ? r0 : r1);
        ++t.sp;
        trav_take(t, swap ? r1 : r0);
    } else if (h0) {
        trav_take(t, r0);
    } else if (h1) {
        trav_take(t, r1);
    } else {
        t.node = kNoNode;
    }
}

// one inner step on the wide BVH: the four child boxes of a Node4 (one
// 128-B record, SoA planes), the hit children sorted near to far, the nearest
// taken and the others pushed far-first (at most 3 pushes per step)
template <bool Shadow>
MH_DEV void trav_inner_step4(TravLane &t, const Node4 *nodes, const LdsBvh &stk) {
    if (t.node == kNoNode) {
        if (t.sp == 0) { t.node = kDone; return; }
        --t.sp;
        const uint32_t ref = stk.pop(t.sp);
        trav_take(t, ref);
        if (t.node == kNoNode || (t.node & kLeafBit)) return;
    }
    const Node4 n = nodes[t.node];
    const float lx[4] = {n.lox.x, n.lox.y, n.lox.z, n.lox.w}, ly[4] = {n.loy.x, n.loy.y, n.loy.z, n.loy.w},
                lz[4] = {n.loz.x, n.loz.y, n.loz.z, n.loz.w}, hx[4] = {n.hix.x, n.hix.y, n.hix.z, n.hix.w},
                hy[4] = {n.hiy.x, n.hiy.y, n.hiy.z, n.hiy.w}, hz[4] = {n.hiz.x, n.hiz.y, n.hiz.z, n.hiz.w};
    const uint32_t rf[4] = {n.ref.x, n.ref.y, n.ref.z, n.ref.w};
    float tc[4];
    uint32_t rc[4];
    uint32_t cnt = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const float a0 = __builtin_fmaf(lx[c], t.inv.x, -t.ood.x), b0 = __builtin_fmaf(hx[c], t.inv.x, -t.ood.x);
        const float a1 = __builtin_fmaf(ly[c], t.inv.y, -t.ood.y), b1 = __builtin_fmaf(hy[c], t.inv.y, -t.ood.y);
        const float a2 = __builtin_fmaf(lz[c], t.inv.z, -t.ood.z), b2 = __builtin_fmaf(hz[c], t.inv.z, -t.ood.z);
        const float lo = fmaxf(fmaxf(fminf(a0, b0), fminf(a1, b1)), fmaxf(fminf(a2, b2), 0.f));
        const float hi = fminf(fminf(fmaxf(a0, b0), fmaxf(a1, b1)), fminf(fmaxf(a2, b2), t.best));
        const bool h = lo <= hi && rf[c] != 0xffffffffu;
        tc[c] = h ? lo : __builtin_huge_valf();
        rc[c] = rf[c];
        cnt += h ? 1u : 0u;
    }
    // sorting network (0,1) (2,3) (0,2) (1,3) (1,2): ascending entry distance
    if (Shadow) {
        // any hit: the visiting order changes only which occluder is found
        // first, not whether one is, so the hit children go as they come --
        // the first is taken, the others pushed (no sort)
        if (cnt == 0) { t.node = kNoNode; return; }
        uint32_t first = kNoNode;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (tc[c] == __builtin_huge_valf()) continue;
            if (first == kNoNode) first = rc[c];
            else { stk.push(t.sp, rc[c]); ++t.sp; }
        }
        trav_take(t, first);
        return;
    }
#define MH_CSWAP(i, j)                                                           \
    {                                                                            \
        const bool sw = tc[j] < tc[i];                                           \
        const float ta = sw ? tc[j] : tc[i], tb = sw ? tc[i] : tc[j];            \
        const uint32_t ra = sw ? rc[j] : rc[i], rb = sw ? rc[i] : rc[j];         \
        tc[i] = ta; tc[j] = tb; rc[i] = ra; rc[j] = rb;                          \
    }
    MH_CSWAP(0, 1) MH_CSWAP(2, 3) MH_CSWAP(0, 2) MH_CSWAP(1, 3) MH_CSWAP(1, 2)
#undef MH_CSWAP
    if (cnt == 0) { t.node = kNoNode; return; }
    if (cnt > 3) { stk.push(t.sp, rc[3]); ++t.sp; }
    if (cnt > 2) { stk.push(t.sp, rc[2]); ++t.sp; }
    if (cnt > 1) { stk.push(t.sp, rc[1]); ++t.sp; }
    trav_take(t, rc[0]);
}

// the same step on the quantised node (QNode4, 64 B = four 16-B loads): each
// child bound decoded by one fma (v_cvt_f32_ubyte of its byte, the node's
// power-of-two scale, the node's origin), then the float slab test of
// trav_inner_step4 on the decoded box
MH_DEV float qscale(uint32_t ebits, uint32_t a) { return __uint_as_float(((ebits >> (8u * a)) & 0xffu) << 23); }
MH_DEV float qbyte(uint32_t w, int c) { return (float)((w >> (8 * c)) & 0xffu); }
template <bool Shadow>
MH_DEV void trav_inner_step_q(TravLane &t, const QNode4 *nodes, const LdsBvh &stk) {
    if (t.node == kNoNode) {
        if (t.sp == 0) { t.node = kDone; return; }
        --t.sp;
        const uint32_t ref = stk.pop(t.sp);
        trav_take(t, ref);
        if (t.node == kNoNode || (t.node & kLeafBit)) return;
    }
    const uint4 *q = reinterpret_cast<const uint4 *>(nodes + t.node);
    const uint4 w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3];
    const float ox = __uint_as_float(w0.x), oy = __uint_as_float(w0.y), oz = __uint_as_float(w0.z);
    const float sx = qscale(w0.w, 0), sy = qscale(w0.w, 1), sz = qscale(w0.w, 2);
    const uint32_t rf[4] = {w3.x, w3.y, w3.z, w3.w};
    float tc[4];
    uint32_t rc[4];
    uint32_t cnt = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const float lx = __builtin_fmaf(qbyte(w1.x, c), sx, ox), hx = __builtin_fmaf(qbyte(w1.w, c), sx, ox);
        const float ly = __builtin_fmaf(qbyte(w1.y, c), sy, oy), hy = __builtin_fmaf(qbyte(w2.x, c), sy, oy);
        const float lz = __builtin_fmaf(qbyte(w1.z, c), sz, oz), hz = __builtin_fmaf(qbyte(w2.y, c), sz, oz);
        const float a0 = __builtin_fmaf(lx, t.inv.x, -t.ood.x), b0 = __builtin_fmaf(hx, t.inv.x, -t.ood.x);
        const float a1 = __builtin_fmaf(ly, t.inv.y, -t.ood.y), b1 = __builtin_fmaf(hy, t.inv.y, -t.ood.y);
        const float a2 = __builtin_fmaf(lz, t.inv.z, -t.ood.z), b2 = __builtin_fmaf(hz, t.inv.z, -t.ood.z);
        const float lo = fmaxf(fmaxf(fminf(a0, b0), fminf(a1, b1)), fmaxf(fminf(a2, b2), 0.f));
        const float hi = fminf(fminf(fmaxf(a0, b0), fmaxf(a1, b1)), fminf(fmaxf(a2, b2), t.best));
        const bool h = lo <= hi && rf[c] != 0xffffffffu;
        tc[c] = h ? lo : __builtin_huge_valf();
        rc[c] = rf[c];
        cnt += h ? 1u : 0u;
    }
    if (Shadow) {
        // any hit: the visiting order changes only which occluder is found
        // first, not whether one is, so the hit children go as they come --
        // the first is taken, the others pushed (no sort)
        if (cnt == 0) { t.node = kNoNode; return; }
        uint32_t first = kNoNode;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (tc[c] == __builtin_huge_valf()) continue;
            if (first == kNoNode) first = rc[c];
            else { stk.push(t.sp, rc[c]); ++t.sp; }
        }
        trav_take(t, first);
        return;
    }
#define MH_CSWAP(i, j)                                                           \
    {                                                                            \
        const bool sw = tc[j] < tc[i];                                           \
        const float ta = sw ? tc[j] : tc[i], tb = sw ? tc[i] : tc[j];            \
        const uint32_t ra = sw ? rc[j] : rc[i], rb = sw ? rc[i] : rc[j];         \
        tc[i] = ta; tc[j] = tb; rc[i] = ra; rc[j] = rb;                          \
    }
    MH_CSWAP(0, 1) MH_CSWAP(2, 3) MH_CSWAP(0, 2) MH_CSWAP(1, 3) MH_CSWAP(1, 2)
#undef MH_CSWAP
    if (cnt == 0) { t.node = kNoNode; return; }
    if (cnt > 3) { stk.push(t.sp, rc[3]); ++t.sp; }
    if (cnt > 2) { stk.push(t.sp, rc[2]); ++t.sp; }
    if (cnt > 1) { stk.push(t.sp, rc[1]); ++t.sp; }
    trav_take(t, rc[0]);
}

template <bool Shadow>
MH_DEV void trav_leaf(TravLane &t, const Prim *prims) {
    RayT r{t.o, t.d, t.maxt};
    for (uint32_t i = 0; i < t.nleaf; ++i) {
        const Prim p = prims[t.leaf + i];
        float tt, u, v;
        if (prim_test(p, r, tt, u, v) && (Shadow || closer(tt, p, t.hit))) {
            t.hit.t = tt; t.hit.u = u; t.hit.v = v; t.hit.prim = p.info.y; t.hit.shape = p.info.x; t.hit.key = p.info.w;
            t.best = tt;
            if (Shadow) { t.node = kDone; t.sp = 0; break; }
        }
    }
    t.nleaf = 0;
    if (t.node != kDone && t.node != kNoNode && (t.node & kLeafBit)) trav_take(t, t.node);
}

// the leaf on compact records (PrimC: three 16-B loads per triangle; a
// rectangle reads its full Prim); the same tests and update rule as trav_leaf
template <bool Shadow>
MH_DEV void trav_leaf_c(TravLane &t, const PrimC *pc, const Prim *prims) {
    RayT r{t.o, t.d, t.maxt};
    for (uint32_t i = 0; i < t.nleaf; ++i) {
        const uint4 *q = reinterpret_cast<const uint4 *>(pc + t.leaf + i);
        const uint4 a = q[0], b = q[1], c = q[2];
        float tt, u, v;
        bool ok;
        if (c.w & kPrimCRect) {
            ok = rect_test(prims[t.leaf + i], r, tt, u, v);
        } else {
            ok = tri_test_v(v3(__uint_as_float(a.x), __uint_as_float(a.y), __uint_as_float(a.z)),
                            v3(__uint_as_float(a.w), __uint_as_float(b.x), __uint_as_float(b.y)),
                            v3(__uint_as_float(b.z), __uint_as_float(b.w), __uint_as_float(c.x)), r, tt, u, v);
        }
        if (ok && (Shadow || (tt < t.hit.t) | ((tt == t.hit.t) & (c.y < t.hit.key)))) {
            t.hit.t = tt; t.hit.u = u; t.hit.v = v; t.hit.prim = c.z; t.hit.shape = c.w & ~kPrimCRect; t.hit.key = c.y;
            t.best = tt;
            if (Shadow) { t.node = kDone; t.sp = 0; break; }
        }
    }
    t.nleaf = 0;
    if (t.node != kDone && t.node != kNoNode && (t.node & kLeafBit)) trav_take(t, t.node);
}

// node formats of the per-lane stream engine
enum { kEngBvh2 = 0, kEngWide = 1, kEngQuant = 2, kEngWideC = 3 };  // WideC: float BVH4 + PrimC
#ifndef MH_SHADOW_UNSORTED
#define MH_SHADOW_UNSORTED 1  // shadow rays skip the near-to-far sort of the wide nodes' children
#endif
constexpr bool kShadowUnsorted = MH_SHADOW_UNSORTED != 0;

// Traces items [r0, r1) of this wave.  load(item) -> RayT, store(item, hit,
// found).  Must be called by all 64 lanes of the wave (uniform r0, r1).
template <bool Shadow, int Eng = kEngBvh2, class Load, class Store>
MH_DEV void trace_stream(const LdsBvh &B, uint32_t r0, uint32_t r1, Load load, Store store) {
    const uint32_t lane = threadIdx.x & 63u;
    const bool empty = B.nodes == nullptr;
    uint32_t fetched = r0 + 64u;  // wave-uniform
    uint32_t item = r0 + lane;
    bool has = item < r1;
    TravLane t;
    if (has) trav_init(t, load(item), empty);
    while (__any(has)) {
        // inner phase: every active lane advances until it holds a leaf or is done
        while (true) {
            const bool inner = has && trav_wants(t);
            const bool ready = !has || t.nleaf != 0 || t.node == kDone;
            if (!__any(inner) || __all(ready)) break;
            if (inner) {
                if (Eng == kEngQuant) trav_inner_step_q<Shadow && kShadowUnsorted>(t, B.qnodes, B);
                else if (Eng == kEngWide || Eng == kEngWideC) trav_inner_step4<Shadow && kShadowUnsorted>(t, B.nodes4, B);
                else trav_inner_step(t, B.nodes, B);
            }
        }
        // grouped leaf phase
        if (has && t.nleaf) {
            // compact 48-B triangle records when the scene carries them (the
            // quantised BVH always; the float BVH4 with MH_PRIMC=1)
            if (Eng == kEngQuant || Eng == kEngWideC) trav_leaf_c<Shadow>(t, B.primsc, B.prims);
            else trav_leaf<Shadow>(t, B.prims);
        }
        if (has && t.node == kNoNode && t.sp == 0 && t.nleaf == 0) t.node = kDone;
        // retire finished lanes and refill them from the wave's range
        const bool fin = has && t.node == kDone && t.nleaf == 0;
        if (fin) store(item, t.hit, t.hit.shape != MH_INVALID);
        const bool need = fin || !has;
        const unsigned long long m = __ballot(need);
        const uint32_t rank = lane_rank(m);
        if (need) {
            const uint32_t cand = fetched + rank;
            has = cand < r1;
            if (has) {
                item = cand;
                trav_init(t, load(item), empty);
            }
        }
        fetched += (uint32_t)__popcll(m);
    }
}

// the stream engine's node format of a scene (host: kernel dispatch)
__host__ __device__ inline int stream_engine(const DScene &S) {
    return S.qnodes ? kEngQuant : S.nodes4 ? (S.primsc ? kEngWideC : kEngWide) : kEngBvh2;
}

// the stream engine on whichever node format the scene carries (quantised
// BVH4, float BVH4, BVH2); B is wave-uniform, so the branch is scalar
template <bool Shadow, class Load, class Store>
MH_DEV void trace_stream_any(const LdsBvh &B, uint32_t r0, uint32_t r1, Load load, Store store) {
    if (B.qnodes) trace_stream<Shadow, kEngQuant>(B, r0, r1, load, store);
    else if (B.nodes4 && B.primsc) trace_stream<Shadow, kEngWideC>(B, r0, r1, load, store);
    else if (B.nodes4) trace_stream<Shadow, kEngWide>(B, r0, r1, load, store);
    else trace_stream<Shadow, kEngBvh2>(B, r0, r1, load, store);
}

// ---------------------------------------------------------------------------
// Wave-coherent ("packet") traversal engine for small BVHs: the 64 lanes of
// a wave walk the BVH together (Wald et al. 2001 ray packets, on the 64-wide
// SIMD).  A child is entered when ANY lane's ray overlaps it; node and
// primitive records are read at wave-uniform addresses (LDS broadcast, no
// bank conflicts), the child indices and the primitive type are
// readfirstlane'd so every branch and the stack are scalar; a primitive is
// tested by the lanes whose ray overlapped its leaf.  No lane diverges, no
// per-lane stack exists.  Same hit semantics as traverse<>: closest hit with
// t in [0, maxt] and strict-< update (only the visiting order differs, which
// matters for exact-t ties alone).  Items [r0, r1) of the wave in batches of 64.
// ---------------------------------------------------------------------------
// Node / primitive records are read through the constant address space at
// wave-uniform indices, so hipcc emits s_load (scalar cache) and the box /
// primitive tests take them as SGPR operands; the visiting decisions are
// ballots (SGPR masks) — the whole control path is scalar.
typedef const __attribute__((address_space(4))) float CFloat;
// wave vote as an SGPR mask: the compiler knows a ballot is wave-uniform, so
// a branch on it stays a scalar branch (no exec-mask structurisation and no
// copies of the values live across it)
MH_DEV bool wave_any(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0; }
template <class T>
MH_DEV T load_uniform(const T *base, uint32_t i) {
    static_assert(sizeof(T) % 4 == 0, "dword records");
    CFloat *p = (CFloat *)(base + i);
    T r;
    float *d = reinterpret_cast<float *>(&r);
#pragma unroll
    for (uint32_t k = 0; k < sizeof(T) / 4; ++k) d[k] = p[k];
    return r;
}

#ifdef MH_EXP_COUNT  // diagnostic build: per-wave event counters of the packet engine
__device__ unsigned long long g_exp_cnt[32];
#define MH_CNT(k) do { if ((threadIdx.x & 63u) == 0) atomicAdd(&g_exp_cnt[(k) + (Shadow ? 8 : 0)], 1ull); } while (0)
// slots 16+: lane sums (k: 0 rect_pair live lanes, 1 tri_pair live lanes, 2 rect accepted, 3 tri accepted)
#define MH_CNTL(k, p) do { const unsigned long long _m = __ballot(p); \
    if ((threadIdx.x & 63u) == 0) atomicAdd(&g_exp_cnt[16 + (k) + (Shadow ? 8 : 0)], (unsigned long long)__popcll(_m)); } while (0)
#else
#define MH_CNT(k) do { } while (0)
#define MH_CNTL(k, p) do { } while (0)
#endif

// Running hit of the packet engine.  t starts at the ray's maxt (every
// accepted t is <= maxt) and key is the scene-order key of the primitive held
// (MH_INVALID: none yet); (shape, prim) are looked up from the key once,
// after the traversal (DScene::key_sp).  Shadow rays only track `occl`, a
// lane mask the compiler keeps in SGPRs (no per-primitive vector selects).
struct PHit {
    float t, u, v;
    uint32_t key;
    bool occl;
};

// closer() on (t, key): strict t, exact-t ties to the lower scene-order key.
// With t starting at maxt this is also the t <= maxt test of the first hit.
template <bool Shadow>
MH_DEV void packet_take(bool ok, float tt, float u, float v, uint32_t key, PHit &h) {
    if (Shadow) {
        h.occl = h.occl | ok;  // any hit occludes
        return;
    }
    const bool take = ok & ((tt < h.t) | ((tt == h.t) & (key < h.key)));
    h.t = take ? tt : h.t;
    h.u = take ? u : h.u;
    h.v = take ? v : h.v;
    h.key = take ? key : h.key;
}

// Two primitives of one type per step: their arithmetic runs on packed f32
// pairs (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32, two IEEE operations per
// lane and instruction, bit-identical to the scalar fmaf/mul/add of
// rect_test / tri_test); the ray's components are broadcast to both halves.
typedef float F2 __attribute__((ext_vector_type(2)));
MH_DEV F2 fma2(F2 a, F2 b, F2 c) { return __builtin_elementwise_fma(a, b, c); }
MH_DEV F2 sp2(float a) { F2 r; r.x = a; r.y = a; return r; }
MH_DEV F2 pair(float a, float b) { F2 r; r.x = a; r.y = b; return r; }
// two rcp() (mh_device.hpp) with the Newton step on packed f32 and one vote
MH_DEV F2 rcp2(F2 x) {
    const F2 y0 = pair(__builtin_amdgcn_rcpf(x.x), __builtin_amdgcn_rcpf(x.y));
    F2 y = fma2(fma2(-x, y0, sp2(1.f)), y0, y0);
    if (rcp_fast_any_bad(x.x) | rcp_fast_any_bad(x.y)) {
        if (!rcp_fast_ok(x.x)) y.x = rcp_slow(x.x);
        if (!rcp_fast_ok(x.y)) y.y = rcp_slow(x.y);
    }
    return y;
}

// field k (dword) of primitive record i, read through the scalar cache at a
// wave-uniform index (no Prim copy in registers / private memory)
MH_DEV float pf(const Prim *P, uint32_t i, uint32_t k) { return ((CFloat *)(P + i))[k]; }
MH_DEV uint32_t pu(const Prim *P, uint32_t i, uint32_t k) { return __float_as_uint(((CFloat *)(P + i))[k]); }
// Pair records of the packet engine (DScene::prim_pairs): the record at
// leaf-ordered position i interleaves the 16 dwords of primitives i and i + 1
// (dword 2k = field k of i, 2k + 1 = field k of i + 1; 128 B), so field k of
// both is one SGPR pair, the direct operand of a v_pk_* instruction (no
// scalar moves to assemble pairs).
MH_DEV F2 pp(const Prim *Q, uint32_t i, uint32_t k) {
    CFloat *p = (CFloat *)(Q + 2u * i) + 2u * k;
    return pair(p[0], p[1]);
}

#ifndef MH_TRI_EARLY
#define MH_TRI_EARLY 1  // wave-level early exit of a triangle pair after u
#endif
#ifndef MH_RECT_EARLY
#define MH_RECT_EARLY 1  // wave-level early exit of a rectangle pair after the plane distance
#endif
// A division-free early exit ahead of the plane distance's two correctly
// rounded divisions: with lz the ray origin's local z and s1 = lz + ldz *
// bound its end's, a lane whose lz and s1 have the same sign, both beyond
// m = 2^-20 (|lz| + |ldz| bound), has no hit: t = -lz / ldz is negative, or
// exceeds bound by more than the division's rounding, so the exact test below
// would reject it as well (the bound is m > 2^-23 (|lz| + |ldz| bound), which
// also covers the rounding of s1).  NaN / inf operands fail the comparisons
// and take the exact test.  Shadow rays inside a closed room never reach the
// walls' planes, so their rectangle tests stop here (round 5).
#ifndef MH_RECT_PRETEST
#define MH_RECT_PRETEST 1
#endif
MH_DEV bool rect_separated(float lz, float ldz, float bound) {
    const float s1 = __builtin_fmaf(ldz, bound, lz);
    // (+ 1e-30: |lz| above it keeps -lz / ldz clear of underflow to -0,
    // which would pass the exact test's t >= 0).  Shadow rays only: a closest
// ray's bound is its best hit so far, infinite until it has one.
    // the margin takes the bound as at least FLT_MIN: |lz| > m >= |ldz| 2^-146
    // keeps |lz / ldz| above 2^-146, so the exact test's quotient cannot
    // underflow to a (passing) -0 when the bound is subnormal
    const float m = __builtin_fmaf(__builtin_fmaf(__builtin_fabsf(ldz), __builtin_fmaxf(bound, 0x1p-126f),
                                                  __builtin_fabsf(lz)), 0x1p-20f, 1e-30f);
    return ((lz > m) & (s1 > m)) | ((lz < -m) & (s1 < -m));
}
template <bool Shadow, bool Pre = true>
MH_DEV void rect_pair(const Prim *Q, uint32_t pos, bool live, const RayT r, PHit &h) {
    MH_CNT(0);
    MH_CNTL(0, live);
    // rows of to_object: x = a, y = b, z = c (shapes/rectangle.cpp:446-470)
    const F2 ox = sp2(r.o.x), oy = sp2(r.o.y), oz = sp2(r.o.z);
    const F2 dx = sp2(r.d.x), dy = sp2(r.d.y), dz = sp2(r.d.z);
    const F2 c0 = pp(Q, pos, 8), c1 = pp(Q, pos, 9), c2 = pp(Q, pos, 10);
    const F2 lz = fma2(c2, oz, fma2(c1, oy, fma2(c0, ox, pp(Q, pos, 11))));
    const F2 ldz = fma2(c2, dz, fma2(c1, dy, c0 * dx));
    const float bound = Shadow ? r.maxt : h.t;
    if (Shadow && Pre && MH_RECT_PRETEST &&
        !wave_any(live & !(rect_separated(lz.x, ldz.x, bound) & rect_separated(lz.y, ldz.y, bound))))
        return;
    const F2 tt = pair(-lz.x / ldz.x, -lz.y / ldz.y);
    bool okA = live & (tt.x >= 0.f) & (tt.x <= bound), okB = live & (tt.y >= 0.f) & (tt.y <= bound);
    if (MH_RECT_EARLY && !wave_any(okA | okB)) return;
    MH_CNT(1);
    const F2 a0 = pp(Q, pos, 0), a1 = pp(Q, pos, 1), a2 = pp(Q, pos, 2);
    const F2 b0 = pp(Q, pos, 4), b1 = pp(Q, pos, 5), b2 = pp(Q, pos, 6);
    const F2 lox = fma2(a2, oz, fma2(a1, oy, fma2(a0, ox, pp(Q, pos, 3))));
    const F2 loy = fma2(b2, oz, fma2(b1, oy, fma2(b0, ox, pp(Q, pos, 7))));
    const F2 ldx = fma2(a2, dz, fma2(a1, dy, a0 * dx));
    const F2 ldy = fma2(b2, dz, fma2(b1, dy, b0 * dx));
    const F2 lx = fma2(ldx, tt, lox), ly = fma2(ldy, tt, loy);
    okA = okA & (__builtin_fabsf(lx.x) <= 1.f) & (__builtin_fabsf(ly.x) <= 1.f);
    okB = okB & (__builtin_fabsf(lx.y) <= 1.f) & (__builtin_fabsf(ly.y) <= 1.f);
    MH_CNTL(2, okA);
    MH_CNTL(2, okB);
    const F2 key = pp(Q, pos, 15);
    packet_take<Shadow>(okA, tt.x, lx.x, ly.x, __float_as_uint(key.x), h);
    packet_take<Shadow>(okB, tt.y, lx.y, ly.y, __float_as_uint(key.y), h);
}

template <bool Shadow>
MH_DEV void tri_pair(const Prim *Q, uint32_t pos, bool live, const RayT r, PHit &h) {
    MH_CNT(2);
    MH_CNTL(1, live);
    // Moeller-Trumbore (render/mesh.h:430-453) on two triangles
    const F2 dx = sp2(r.d.x), dy = sp2(r.d.y), dz = sp2(r.d.z);
    const F2 e1x = pp(Q, pos, 4), e1y = pp(Q, pos, 5), e1z = pp(Q, pos, 6);
    const F2 e2x = pp(Q, pos, 8), e2y = pp(Q, pos, 9), e2z = pp(Q, pos, 10);
    // pvec = cross(d, e2)
    const F2 px = fma2(dy, e2z, -(dz * e2y)), py = fma2(dz, e2x, -(dx * e2z)), pz = fma2(dx, e2y, -(dy * e2x));
    const F2 det = fma2(e1z, pz, fma2(e1y, py, e1x * px));
    // tvec ahead of the reciprocal: its loads are issued before the
    // reciprocal's (rare) slow-path branch splits the block
    const F2 tx = sp2(r.o.x) - pp(Q, pos, 0), ty = sp2(r.o.y) - pp(Q, pos, 1),
             tz = sp2(r.o.z) - pp(Q, pos, 2);
    const F2 inv_det = rcp2(det);
    const F2 u = fma2(tz, pz, fma2(ty, py, tx * px)) * inv_det;
    bool okA = live & (u.x >= 0.f) & (u.x <= 1.f), okB = live & (u.y >= 0.f) & (u.y <= 1.f);
    if (MH_TRI_EARLY && !wave_any(okA | okB)) return;
    MH_CNT(3);
    // qvec = cross(tvec, e1)
    const F2 qx = fma2(ty, e1z, -(tz * e1y)), qy = fma2(tz, e1x, -(tx * e1z)), qz = fma2(tx, e1y, -(ty * e1x));
    const F2 v = fma2(dz, qz, fma2(dy, qy, dx * qx)) * inv_det;
    const F2 tt = fma2(e2z, qz, fma2(e2y, qy, e2x * qx)) * inv_det;
    const F2 uv = u + v;
    okA = okA & (v.x >= 0.f) & (uv.x <= 1.f) & (tt.x >= 0.f) & (tt.x <= r.maxt);
    okB = okB & (v.y >= 0.f) & (uv.y <= 1.f) & (tt.y >= 0.f) & (tt.y <= r.maxt);
    MH_CNTL(3, okA);
    MH_CNTL(3, okB);
    const F2 key = pp(Q, pos, 15);
    packet_take<Shadow>(okA, tt.x, u.x, v.x, __float_as_uint(key.x), h);
    packet_take<Shadow>(okB, tt.y, u.y, v.y, __float_as_uint(key.y), h);
}

template <bool Shadow, bool Pre = true>
MH_DEV void rect_one(const Prim *P, uint32_t pos, bool live, const RayT r, PHit &h) {
    MH_CNT(4);
    const float oz = __builtin_fmaf(pf(P, pos, 10), r.o.z, __builtin_fmaf(pf(P, pos, 9), r.o.y, __builtin_fmaf(pf(P, pos, 8), r.o.x, pf(P, pos, 11))));
    const float dz = __builtin_fmaf(pf(P, pos, 10), r.d.z, __builtin_fmaf(pf(P, pos, 9), r.d.y, pf(P, pos, 8) * r.d.x));
    if (Shadow && Pre && MH_RECT_PRETEST && !wave_any(live & !rect_separated(oz, dz, r.maxt))) return;
    const float tt = -oz / dz;
    bool ok = live & (tt >= 0.f) & (tt <= (Shadow ? r.maxt : h.t));
    if (!wave_any(ok)) return;
    MH_CNT(4);
    // xf_point / xf_vector rows x, y, then fma(d, t, o)
    const float ox = __builtin_fmaf(pf(P, pos, 2), r.o.z, __builtin_fmaf(pf(P, pos, 1), r.o.y, __builtin_fmaf(pf(P, pos, 0), r.o.x, pf(P, pos, 3))));
    const float oy = __builtin_fmaf(pf(P, pos, 6), r.o.z, __builtin_fmaf(pf(P, pos, 5), r.o.y, __builtin_fmaf(pf(P, pos, 4), r.o.x, pf(P, pos, 7))));
    const float dx = __builtin_fmaf(pf(P, pos, 2), r.d.z, __builtin_fmaf(pf(P, pos, 1), r.d.y, pf(P, pos, 0) * r.d.x));
    const float dy = __builtin_fmaf(pf(P, pos, 6), r.d.z, __builtin_fmaf(pf(P, pos, 5), r.d.y, pf(P, pos, 4) * r.d.x));
    const float lx = __builtin_fmaf(dx, tt, ox), ly = __builtin_fmaf(dy, tt, oy);
    ok = ok & (__builtin_fabsf(lx) <= 1.f) & (__builtin_fabsf(ly) <= 1.f);
    packet_take<Shadow>(ok, tt, lx, ly, pu(P, pos, 15), h);
}

template <bool Shadow>
MH_DEV void tri_one(const Prim *P, uint32_t pos, bool live, const RayT r, PHit &h) {
    MH_CNT(5);
    const V3 v0 = v3(pf(P, pos, 0), pf(P, pos, 1), pf(P, pos, 2)), e1 = v3(pf(P, pos, 4), pf(P, pos, 5), pf(P, pos, 6)), e2 = v3(pf(P, pos, 8), pf(P, pos, 9), pf(P, pos, 10));
    const V3 pvec = cross(r.d, e2);
    const float inv_det = rcp(dot(e1, pvec));
    const V3 tvec = r.o - v0;
    const float u = dot(tvec, pvec) * inv_det;
    bool ok = live & (u >= 0.f) & (u <= 1.f);
    if (!wave_any(ok)) return;
    MH_CNT(5);
    const V3 qvec = cross(tvec, e1);
    const float v = dot(r.d, qvec) * inv_det;
    const float tt = dot(e2, qvec) * inv_det;
    ok = ok & (v >= 0.f) & (u + v <= 1.f) & (tt >= 0.f) & (tt <= r.maxt);
    packet_take<Shadow>(ok, tt, u, v, pu(P, pos, 15), h);
}

// One leaf for the lanes whose ray overlapped its box (lane_hit).  The host
// orders every leaf by primitive type (build_bvh), so primitives go in
// same-type pairs with at most one single test per type.  Each test computes
// the quantity that rejects most lanes first (the plane distance of a
// rectangle, u of a triangle) and skips the rest when the wave's ballot is
// empty -- a uniform branch; the values a surviving lane sees are computed
// exactly as in rect_test / tri_test.
template <bool Shadow>
MH_DEV void packet_leaf(const Prim *prims, const Prim *pairs, uint32_t first, uint32_t count, uint32_t nrect, bool lane_hit,
                        const RayT r, PHit &h) {
    // rectangles [0, nrect), then triangles [nrect, count): straight-line
    // loops (one body each) rather than one loop with a per-step type switch
    uint32_t i = 0;
    for (; i + 1u < nrect; i += 2u)
        rect_pair<Shadow>(pairs, first + i, lane_hit & (!Shadow || !h.occl), r, h);
    if (i < nrect) {
        rect_one<Shadow>(prims, first + i, lane_hit & (!Shadow || !h.occl), r, h);
        ++i;
    }
    for (; i + 1u < count; i += 2u)
        tri_pair<Shadow>(pairs, first + i, lane_hit & (!Shadow || !h.occl), r, h);
    if (i < count) tri_one<Shadow>(prims, first + i, lane_hit & (!Shadow || !h.occl), r, h);
}

// ---------------------------------------------------------------------------
// Sparse-leaf compaction (the fused bounce kernels).  A triangle run whose
// leaf box only a few lanes of the wave overlap (the two cubes of the cornell
// box: 16 of 64 closest rays, 7 of 64 shadow rays) wastes most of the packet
// test's lanes.  Such a run is deferred: its overlapping lanes are listed in
// the wave's LDS scratch (ballot + mbcnt compaction), and after the traversal
// the (ray, triangle pair) items of every deferred run are packed densely
// into the 64 lanes: lane j tests item j with per-lane operands (the ray by
// ds_bpermute from its owner lane, the pair record from the LDS copy of the
// pair table).  Results merge into the owner's hit through a 64-bit LDS
// atomic min on (t, scene-order key) -- the lexicographic order of
// packet_take -- and the winner writes its (u, v).  The arithmetic of a test
// is tri_pair's, so hits are bit-identical to the dense packet test.
// ---------------------------------------------------------------------------
#ifndef MH_DEFER_DENSE_MIN
#define MH_DEFER_DENSE_MIN 40  // lanes at or above which a triangle run is tested densely
#endif
constexpr uint32_t kMaxDefer = 2;        // deferred runs per batch (more: tested densely)
constexpr uint32_t kPairRecFloats = 20;  // v0, e1, e2, key of both primitives, interleaved
constexpr uint32_t kDeferScratch = 1536; // per wave: slot u64[64] | uv float2[64] | lists u32[2][64]
// field k of a pair record (mh_api.hip pair records: dword 2k / 2k+1) -> compact slot
MH_DEV void stage_pair_records(const DScene &S, float *dst) {
    const CFloat *src = (CFloat *)S.prim_pairs;
    const uint32_t total = S.n_prims * kPairRecFloats;
    for (uint32_t i = threadIdx.x; i < total; i += blockDim.x) {
        const uint32_t rec = i / kPairRecFloats, w = i - rec * kPairRecFloats, j = w >> 1;
        const uint32_t f = j < 9u ? j + j / 3u : 15u;  // fields 0 1 2 4 5 6 8 9 10 15
        dst[i] = src[rec * 32u + 2u * f + (w & 1u)];
    }
}
__host__ __device__ inline uint32_t align16(uint32_t x) { return (x + 15u) & ~15u; }
// dynamic LDS of the fused bounce kernels: tables | stacks | pair records | scratch
__host__ __device__ inline uint32_t fused_pairs_offset(const DScene &S) {
    return align16(S.tab_bytes + 16u * S.stack_size);
}
__host__ __device__ inline uint32_t fused_scratch_offset(const DScene &S) {
    return fused_pairs_offset(S) + align16(S.n_prims * kPairRecFloats * 4u);
}
__host__ __device__ inline uint32_t fused_lds_bytes(const DScene &S) {
    return fused_scratch_offset(S) + 4u * kDeferScratch;
}

struct Defer {
    const float *recs;   // LDS pair records (nullptr: no deferral)
    uint8_t *scratch;    // this wave's kDeferScratch bytes
    uint32_t n;          // deferred runs so far
    uint32_t first[kMaxDefer], ntri[kMaxDefer], pc[kMaxDefer];
};


// The triangle run [first, first + count) for the lanes `live`: dense packet
// test, or deferred when few lanes overlap the leaf.
template <bool Shadow, bool Def>
MH_DEV void packet_tris(const Prim *prims, const Prim *pairs, uint32_t first, uint32_t count, bool live,
                        const RayT r, PHit &h, Defer &df) {
    if (Def && df.n < kMaxDefer) {
        const unsigned long long m = __builtin_amdgcn_ballot_w64(live);
        const uint32_t pc = (uint32_t)__popcll(m);
        if (pc < MH_DEFER_DENSE_MIN) {
            uint32_t *list = reinterpret_cast<uint32_t *>(df.scratch + 1024) + 64u * df.n;
            if (live) list[lane_rank(m)] = threadIdx.x & 63u;
#pragma unroll
            for (uint32_t k = 0; k < kMaxDefer; ++k)
                if (k == df.n) { df.first[k] = first; df.ntri[k] = count; df.pc[k] = pc; }
            ++df.n;
            return;
        }
    }
    uint32_t i = 0;
    for (; i + 1u < count; i += 2u) tri_pair<Shadow>(pairs, first + i, live, r, h);
    if (i < count) tri_one<Shadow>(prims, first + i, live, r, h);
}

// the deferred items: (ray, pair) of every deferred run, 64 per step
template <bool Shadow>
MH_DEV void run_deferred(const Defer &df, const RayT r, bool act, PHit &h) {
    const uint32_t lane = threadIdx.x & 63u;
    unsigned long long *slot = reinterpret_cast<unsigned long long *>(df.scratch);
    float2 *uv = reinterpret_cast<float2 *>(df.scratch + 512);
    const uint32_t *lists = reinterpret_cast<const uint32_t *>(df.scratch + 1024);
    // the owner's hit so far: (t, key) as one ordered 64-bit key (t >= 0; -0 -> +0)
    if (Shadow) {
        reinterpret_cast<uint32_t *>(slot)[lane] = h.occl ? 1u : 0u;
    } else if (act) {
        slot[lane] = ((unsigned long long)__float_as_uint(h.t + 0.f) << 32) | h.key;
        uv[lane] = make_float2(h.u, h.v);
    }
    __builtin_amdgcn_wave_barrier();
    for (uint32_t k = 0; k < df.n; ++k) {
        uint32_t first = 0, ntri = 0, pc = 1;
#pragma unroll
        for (uint32_t q = 0; q < kMaxDefer; ++q)
            if (q == k) { first = df.first[q]; ntri = df.ntri[q]; pc = df.pc[q]; }
        const uint32_t np = (ntri + 1u) >> 1, total = pc * np;
        const float inv_pc = 1.f / (float)pc;
        for (uint32_t base = 0; base < total; base += 64u) {
            const uint32_t g = base + lane;
            const bool on = g < total;
            const uint32_t p = on ? (uint32_t)(((float)g + 0.5f) * inv_pc) : 0u;  // exact: g < 2^16, pc <= 64
            const uint32_t rank = on ? g - p * pc : 0u;
            const uint32_t owner = lists[64u * k + rank];
            RayT q;
            q.o = v3(__shfl(r.o.x, owner), __shfl(r.o.y, owner), __shfl(r.o.z, owner));
            q.d = v3(__shfl(r.d.x, owner), __shfl(r.d.y, owner), __shfl(r.d.z, owner));
            q.maxt = __shfl(r.maxt, owner);
            const float *rec = df.recs + (first + 2u * p) * kPairRecFloats;
            const float4 a = *reinterpret_cast<const float4 *>(rec), b = *reinterpret_cast<const float4 *>(rec + 4),
                         c = *reinterpret_cast<const float4 *>(rec + 8), d = *reinterpret_cast<const float4 *>(rec + 12),
                         e = *reinterpret_cast<const float4 *>(rec + 16);
            // fields: (v0x v0y v0z e1x e1y e1z e2x e2y e2z key) x (A, B), interleaved
            const F2 v0x = pair(a.x, a.y), v0y = pair(a.z, a.w), v0z = pair(b.x, b.y);
            const F2 e1x = pair(b.z, b.w), e1y = pair(c.x, c.y), e1z = pair(c.z, c.w);
            const F2 e2x = pair(d.x, d.y), e2y = pair(d.z, d.w), e2z = pair(e.x, e.y);
            const bool hasB = 2u * p + 1u < ntri;
            // Moeller-Trumbore (render/mesh.h:430-453): tri_pair's operations
            const F2 dx = sp2(q.d.x), dy = sp2(q.d.y), dz = sp2(q.d.z);
            const F2 px = fma2(dy, e2z, -(dz * e2y)), py = fma2(dz, e2x, -(dx * e2z)), pz = fma2(dx, e2y, -(dy * e2x));
            const F2 det = fma2(e1z, pz, fma2(e1y, py, e1x * px));
            const F2 tx = sp2(q.o.x) - v0x, ty = sp2(q.o.y) - v0y, tz = sp2(q.o.z) - v0z;
            const F2 inv_det = rcp2(det);
            const F2 u = fma2(tz, pz, fma2(ty, py, tx * px)) * inv_det;
            bool okA = on & (u.x >= 0.f) & (u.x <= 1.f), okB = on & hasB & (u.y >= 0.f) & (u.y <= 1.f);
            if (!wave_any(okA | okB)) continue;
            const F2 qx = fma2(ty, e1z, -(tz * e1y)), qy = fma2(tz, e1x, -(tx * e1z)), qz = fma2(tx, e1y, -(ty * e1x));
            const F2 v = fma2(dz, qz, fma2(dy, qy, dx * qx)) * inv_det;
            const F2 tt = fma2(e2z, qz, fma2(e2y, qy, e2x * qx)) * inv_det;
            const F2 uvs = u + v;
            okA = okA & (v.x >= 0.f) & (uvs.x <= 1.f) & (tt.x >= 0.f) & (tt.x <= q.maxt);
            okB = okB & (v.y >= 0.f) & (uvs.y <= 1.f) & (tt.y >= 0.f) & (tt.y <= q.maxt);
            if (Shadow) {
                if (okA | okB) reinterpret_cast<uint32_t *>(slot)[owner] = 1u;
                continue;
            }
            // the better of A and B (packet_take's order), then the merge
            PHit ch;
            ch.t = q.maxt;
            ch.u = ch.v = 0.f;
            ch.key = MH_INVALID;
            ch.occl = false;
            packet_take<false>(okA, tt.x, u.x, v.x, __float_as_uint(e.z), ch);
            packet_take<false>(okB, tt.y, u.y, v.y, __float_as_uint(e.w), ch);
            const bool cand = ch.key != MH_INVALID;
            const unsigned long long key64 = ((unsigned long long)__float_as_uint(ch.t + 0.f) << 32) | ch.key;
            if (cand) __hip_atomic_fetch_min(slot + owner, key64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __builtin_amdgcn_wave_barrier();
            if (cand && slot[owner] == key64) uv[owner] = make_float2(ch.u, ch.v);
            __builtin_amdgcn_wave_barrier();
        }
    }
    __builtin_amdgcn_wave_barrier();
    if (Shadow) {
        h.occl = reinterpret_cast<const uint32_t *>(slot)[lane] != 0u;
    } else if (act) {
        const unsigned long long s = slot[lane];
        const float2 w = uv[lane];
        h.t = __uint_as_float((uint32_t)(s >> 32));
        h.key = (uint32_t)s;
        h.u = w.x;
        h.v = w.y;
    }
    __builtin_amdgcn_wave_barrier();
}

// gnodes / gprims: the BVH in global memory (read via the scalar cache);
// B provides the LDS stack region (one wave-uniform stack per wave).
// One batch: the wave's 64 rays (act: lanes that hold a ray).  ws: the
// wave-uniform stack (entry k at ws[k * stride]).  Def: sparse triangle runs
// are deferred and compacted (dfr: LDS pair records + the wave's scratch).
// Pre: the rectangle tests' division-free early exit (rect_separated; the
// non-generating PRB bounce leaves it out: 2 more VGPRs spill there)
template <bool Shadow, bool Def = false, bool Pre = true>
MH_DEV Hit packet_batch(const Node *gnodes, const Prim *gprims, const Prim *gpairs, const uint2 *key_sp, uint32_t *ws, uint32_t stride,
                        const RayT r, bool act, const float *dfr_recs = nullptr, uint8_t *dfr_scratch = nullptr) {
    const V3 inv = safe_inv_dir(r.d), ood = r.o * inv;
    PHit ph;
    ph.t = r.maxt;
    ph.u = ph.v = 0.f;
    ph.key = MH_INVALID;
    ph.occl = false;
    act = act && gnodes != nullptr;
    Defer df;
    df.recs = dfr_recs;
    df.scratch = dfr_scratch;
    df.n = 0;
    const bool act0 = act;
    uint32_t node = 0, sp = 0;
    auto leaf = [&](uint32_t c, uint32_t cnt, uint32_t nrect, bool hit) {
        // rectangles [0, nrect) densely (nearly every ray overlaps the room),
        // then the triangle run
        uint32_t i = 0;
        for (; i + 1u < nrect; i += 2u) rect_pair<Shadow, Pre>(gpairs, c + i, hit & (!Shadow || !ph.occl), r, ph);
        if (i < nrect) {
            rect_one<Shadow, Pre>(gprims, c + i, hit & (!Shadow || !ph.occl), r, ph);
            ++i;
        }
        if (i < cnt) packet_tris<Shadow, Def>(gprims, gpairs, c + i, cnt - i, hit & (!Shadow || !ph.occl), r, ph, df);
    };
    while (wave_any(act)) {
        const Node n = load_uniform(gnodes, node);
        bool h0, h1;
        float t0, t1;
        MH_CNT(6);
        box2(n, inv, ood, ph.t, h0, h1, t0, t1);
        h0 = h0 && act;
        h1 = h1 && act;
        const uint32_t c0 = __float_as_uint(n.lo0.w), n0 = __float_as_uint(n.hi0.w) & kLeafCountMask;
        const uint32_t c1 = __float_as_uint(n.lo1.w), n1 = __float_as_uint(n.hi1.w) & kLeafCountMask;
        bool any0 = wave_any(h0), any1 = wave_any(h1);
        if (any0 && n0) {
            leaf(c0, n0, __float_as_uint(n.hi0.w) >> kLeafRectShift, h0);
            any0 = false;
        }
        if (any1 && n1) {
            leaf(c1, n1, __float_as_uint(n.hi1.w) >> kLeafRectShift, h1);
            any1 = false;
        }
        if (Shadow) act = act && !ph.occl;
        if (any0 && any1) {
            const unsigned long long both = __ballot(h0 && h1), pref1 = __ballot(h0 && h1 && t1 < t0);
            const bool first1 = 2u * (uint32_t)__popcll(pref1) > (uint32_t)__popcll(both);
            ws[sp * stride] = first1 ? c0 : c1;
            ++sp;
            node = first1 ? c1 : c0;
        } else if (any0) {
            node = c0;
        } else if (any1) {
            node = c1;
        } else {
            if (sp == 0) break;
            --sp;
            node = __builtin_amdgcn_readfirstlane(ws[sp * stride]);
        }
    }
    if (Def && df.n) run_deferred<Shadow>(df, r, act0, ph);
    MH_CNT(7);
    Hit hit;
    hit.key = ph.key;
    hit.prim = MH_INVALID;
    hit.shape = MH_INVALID;
    hit.t = __builtin_huge_valf();
    hit.u = hit.v = 0.f;
    if (Shadow) {
        hit.shape = ph.occl ? 0u : MH_INVALID;  // occluded / not (the shadow consumers' test)
    } else if (ph.key != MH_INVALID) {
        const uint2 sp = key_sp[ph.key];
        hit.shape = sp.x;
        hit.prim = sp.y;
        hit.t = ph.t;
        hit.u = ph.u;
        hit.v = ph.v;
    }
    return hit;
}

template <bool Shadow, class Load, class Store>
MH_DEV void trace_packet(const Node *gnodes, const Prim *gprims, const Prim *gpairs, const uint2 *key_sp, const LdsBvh &B, uint32_t r0,
                         uint32_t r1,
                         Load load, Store store) {
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t *ws = B.stack - lane;  // wave-uniform stack: entry k at ws[k * stride]
    for (uint32_t base = r0; base < r1; base += 64u) {
        const uint32_t item = base + lane;
        const bool has = item < r1;
        RayT r;
        if (has) r = load(item);
        else r = RayT{v3(0, 0, 0), v3(0, 0, 1), -1.f};
        const Hit hit = packet_batch<Shadow>(gnodes, gprims, gpairs, key_sp, ws, B.stride, r, has);
        if (has) store(item, hit, hit.shape != MH_INVALID);
    }
}

// ===========================================================================
// SurfaceInteraction (interaction.h:464-484,731-757; rectangle.cpp:497-567;
// mesh.cpp:1368-1536) — ad-variant branch (p = ray(t) for rectangles)
// ===========================================================================
struct SI {
    bool valid;
    V3 p, n, s, t_, sn;  // geometric p/n; shading frame (s, t_, sn)
    float uvx, uvy;
    V3 wi;               // local
    uint32_t shape;
};

// coordinate_system (core/vector.h:116-136)
MH_DEV void coordinate_system(V3 n, V3 &s, V3 &t) {
    float sign = n.z >= 0.f ? 1.f : -1.f, a = -rcp(sign + n.z), b = n.x * n.y * a;
    s = v3(mulsign(n.x * n.x * a, n.z) + 1.f, mulsign(b, n.z), mulsign_neg(n.x, n.z));
    t = v3(b, __builtin_fmaf(n.y, n.y * a, sign), -n.y);
}

MH_DEV V3 to_local(const SI &si, V3 v) { return v3(dot(v, si.s), dot(v, si.t_), dot(v, si.sn)); }
MH_DEV V3 to_world(const SI &si, V3 v) {
    return fma3s(si.sn, v.z, fma3s(si.t_, v.y, si.s * v.x));
}

MH_DEV V3 vtx(const DScene &S, uint32_t i) { return ld3(S.positions + 3ull * i); }

MH_DEV void compute_si(const DScene &S, const RayT &r, const Hit &h, SI &si) {
    // single-exit form: every field is produced in registers and assigned once
    // (partial early-return initialisation made hipcc spill uv to scratch)
    const bool valid = h.shape != MH_INVALID;
    V3 p = v3(0, 0, 0), n = v3(0, 0, 0), sn = v3(0, 0, 0), dp_du = v3(0, 0, 0);
    float uvx = 0.f, uvy = 0.f;
    if (valid) {
        const DShape &sh = S.shapes[h.shape];
        if (sh.type == MH_SHAPE_RECTANGLE) {
            p = fma3s(r.d, h.t, r.o);
            n = ld3(sh.frame_n);
            sn = n;
            dp_du = ld3(sh.frame_s);
            uvx = __builtin_fmaf(h.u, 0.5f, 0.5f);
            uvy = __builtin_fmaf(h.v, 0.5f, 0.5f);
        } else {
            const uint32_t *fi = S.faces + 3ull * (sh.face_offset + h.prim);
            const uint32_t i0 = sh.vertex_offset + fi[0], i1 = sh.vertex_offset + fi[1],
                           i2 = sh.vertex_offset + fi[2];
            V3 p0 = vtx(S, i0), p1 = vtx(S, i1), p2 = vtx(S, i2);
            float b1 = h.u, b2 = h.v, b0 = 1.f - b1 - b2;
            p = fma3s(p0, b0, fma3s(p1, b1, p2 * b2));
            n = normalize(cross(p1 - p0, p2 - p0));
            uvx = b1;
            uvy = b2;
            V3 dpdv;
            coordinate_system(n, dp_du, dpdv);
            if (sh.has_texcoords) {
                const float *tc = S.texcoords;
                float u0x = tc[2ull * i0], u0y = tc[2ull * i0 + 1], u1x = tc[2ull * i1],
                      u1y = tc[2ull * i1 + 1], u2x = tc[2ull * i2], u2y = tc[2ull * i2 + 1];
                uvx = __builtin_fmaf(u2x, b2, __builtin_fmaf(u1x, b1, u0x * b0));
                uvy = __builtin_fmaf(u2y, b2, __builtin_fmaf(u1y, b1, u0y * b0));
                float d0x = u1x - u0x, d0y = u1y - u0y, d1x = u2x - u0x, d1y = u2y - u0y;
                float det = __builtin_fmaf(d0x, d1y, -(d0y * d1x)), inv_det = rcp(det);
                V3 dp0 = p1 - p0, dp1 = p2 - p0;
                if (det != 0.f)
                    dp_du = v3(__builtin_fmaf(d1y, dp0.x, -(d0y * dp1.x)),
                               __builtin_fmaf(d1y, dp0.y, -(d0y * dp1.y)),
                               __builtin_fmaf(d1y, dp0.z, -(d0y * dp1.z))) * inv_det;
            }
            if (sh.has_normals) {
                V3 n0 = ld3(S.normals + 3ull * i0), n1 = ld3(S.normals + 3ull * i1),
                   n2 = ld3(S.normals + 3ull * i2);
                V3 nn = fma3s(n2, b2, fma3s(n1, b1, n0 * b0));
                sn = nn * rsqrt_(dot(nn, nn));
            } else {
                sn = n;
            }
        }
    }
    // initialize_sh_frame (interaction.h:245-255)
    V3 s = normalize(fma3s(sn, -dot(sn, dp_du), dp_du));
    if (dp_du.x == 0.f && dp_du.y == 0.f && dp_du.z == 0.f) {
        V3 tt;
        coordinate_system(sn, s, tt);
    }
    si.valid = valid;
    si.shape = h.shape;
    si.p = p;
    si.n = n;
    si.sn = sn;
    si.s = s;
    si.t_ = cross(sn, s);
    si.uvx = uvx;
    si.uvy = uvy;
    si.wi = valid ? to_local(si, -r.d) : -r.d;
}

// Interaction::offset_p / spawn_ray / spawn_ray_to (interaction.h:133-162)
MH_DEV V3 offset_p(V3 p, V3 n, V3 d) {
    float mag = (1.f + hmax(v3(__builtin_fabsf(p.x), __builtin_fabsf(p.y), __builtin_fabsf(p.z)))) * kRayEps;
    mag = mulsign(mag, dot(n, d));
    return fma3s(n, mag, p);
}
MH_DEV RayT spawn_ray(V3 p, V3 n, V3 d) { return RayT{offset_p(p, n, d), d, kFloatMax}; }
MH_DEV RayT spawn_ray_to(V3 p, V3 n, V3 target) {
    V3 o = offset_p(p, n, target - p);
    V3 d = target - o;
    float dist = norm(d);
    d = vdiv(d, dist);
    return RayT{o, d, dist * (1.f - kShadowEps)};
}

// ===========================================================================
// Textures, diffuse BSDF, area emitter
// ===========================================================================
MH_DEV int32_t wrap_index(int32_t i, int32_t res, uint32_t mode) {
    if (mode == 2) return i < 0 ? 0 : (i >= res ? res - 1 : i);
    if (mode == 1) {
        int32_t p = 2 * res, m = i % p;
        if (m < 0) m += p;
        return m < res ? m : p - 1 - m;
    }
    int32_t m = i % res;
    if (m < 0) m += res;
    return m;
}

struct Taps {
    uint32_t n;
    uint64_t idx[4];
    float w0x, w1x, w0y, w1y;
};

// bitmap: [drjit] Texture2f::eval_nonaccel at to_uv * uv (textures/bitmap.cpp:696-710)
MH_DEV void bitmap_taps(const DTexture &tx, float uvx, float uvy, Taps &tp) {
    const float *m = tx.to_uv;
    float ux = __builtin_fmaf(m[1], uvy, __builtin_fmaf(m[0], uvx, m[2]));
    float uy = __builtin_fmaf(m[4], uvy, __builtin_fmaf(m[3], uvx, m[5]));
    int32_t W = (int32_t)tx.width, H = (int32_t)tx.height;
    uint32_t C = tx.channels;
    if (tx.filter == 0) {
        int32_t ix = wrap_index((int32_t)floorf(ux * (float)W), W, tx.wrap);
        int32_t iy = wrap_index((int32_t)floorf(uy * (float)H), H, tx.wrap);
        tp.n = 1;
        tp.idx[0] = tx.data_offset + ((uint64_t)iy * W + ix) * C;
        tp.w0x = tp.w0y = 1.f;
        tp.w1x = tp.w1y = 0.f;
        return;
    }
    float fx = __builtin_fmaf(ux, (float)W, -0.5f), fy = __builtin_fmaf(uy, (float)H, -0.5f);
    float flx = floorf(fx), fly = floorf(fy);
    int32_t ix = (int32_t)flx, iy = (int32_t)fly;
    tp.w1x = fx - flx;
    tp.w1y = fy - fly;
    tp.w0x = 1.f - tp.w1x;
    tp.w0y = 1.f - tp.w1y;
    int32_t x0 = wrap_index(ix, W, tx.wrap), x1 = wrap_index(ix + 1, W, tx.wrap);
    int32_t y0 = wrap_index(iy, H, tx.wrap), y1 = wrap_index(iy + 1, H, tx.wrap);
    tp.n = 4;
    tp.idx[0] = tx.data_offset + ((uint64_t)y0 * W + x0) * C;
    tp.idx[1] = tx.data_offset + ((uint64_t)y0 * W + x1) * C;
    tp.idx[2] = tx.data_offset + ((uint64_t)y1 * W + x0) * C;
    tp.idx[3] = tx.data_offset + ((uint64_t)y1 * W + x1) * C;
}

MH_DEV V3 tex_eval(const DScene &S, uint32_t tex, float uvx, float uvy) {
    const DTexture &tx = S.textures[tex];
    if (tx.type == MH_TEX_RGB) return v3(tx.value[0], tx.value[1], tx.value[2]);
    Taps tp;
    bitmap_taps(tx, uvx, uvy, tp);
    float out[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        uint32_t cc = tx.channels == 3 ? (uint32_t)c : 0u;
        if (tp.n == 1) {
            out[c] = S.texels[tp.idx[0] + cc];
        } else {
            float f00 = S.texels[tp.idx[0] + cc], f10 = S.texels[tp.idx[1] + cc],
                  f01 = S.texels[tp.idx[2] + cc], f11 = S.texels[tp.idx[3] + cc];
            out[c] = __builtin_fmaf(tp.w0y, __builtin_fmaf(tp.w0x, f00, tp.w1x * f10),
                                    tp.w1y * __builtin_fmaf(tp.w0x, f01, tp.w1x * f11));
        }
    }
    return v3(out[0], out[1], out[2]);
}

// SmoothDiffuse::eval_pdf (bsdfs/diffuse.cpp:160-180)
MH_DEV void diffuse_eval_pdf(V3 rho, V3 wi, V3 wo, bool active, V3 &val, float &pdf) {
    active = active && wi.z > 0.f && wo.z > 0.f;
    val = active ? (rho * kInvPi) * wo.z : v3(0, 0, 0);
    pdf = active ? kInvPi * wo.z : 0.f;
}

// warp.h:54-90 + warp.h:412-428
MH_DEV V3 square_to_cosine_hemisphere(float sx, float sy) {
    float x = __builtin_fmaf(2.f, sx, -1.f), y = __builtin_fmaf(2.f, sy, -1.f);
    bool is_zero = x == 0.f && y == 0.f, q13 = __builtin_fabsf(x) < __builtin_fabsf(y);
    float r = q13 ? y : x, rp = q13 ? x : y;
    float phi = ((0.25f * kPi) * rp) / r;
    if (q13) phi = (0.5f * kPi) - phi;
    if (is_zero) phi = 0.f;
    float sn, cs;
    sincos_cephes(phi, sn, cs);
    float px = r * cs, py = r * sn;
    float z = __builtin_sqrtf(fmaxf(1.f - __builtin_fmaf(py, py, px * px), 0.f));
    return v3(px, py, z);
}

// mis_weight (integrators/path.cpp:300-305)
MH_DEV float mis_weight(float a, float b) {
    a = a * a;
    b = b * b;
    float w = a / (a + b);
    return isfinite_(w) ? w : 0.f;
}

struct DirS {
    V3 p, n, d;
    float dist, pdf;
    bool delta;
};

// AreaLight::pdf_direction (emitters/area.cpp:170-200), Shape::pdf_direction (shape.cpp:377-388)
MH_DEV float area_pdf_direction(const DScene &S, uint32_t em, const DirS &ds) {
    const DEmitter &e = S.emitters[em];
    if (e.type != MH_EMITTER_AREA) return 0.f;
    float dp = dot(ds.d, ds.n);
    float pdf = S.shapes[e.shape].inv_area, adp = __builtin_fabsf(dp);
    pdf *= (adp != 0.f) ? (ds.dist * ds.dist) / adp : 0.f;
    return dp < 0.f ? pdf : 0.f;
}

// emitter-hit MIS density: DirectionSample3f(scene, si, prev_si) (render/records.h:173-180)
MH_DEV float emitter_hit_pdf(const DScene &S, uint32_t em, const SI &si, V3 prev_p) {
    DirS ds;
    ds.p = si.p;
    ds.n = si.sn;
    V3 rel = si.p - prev_p;
    ds.dist = norm(rel);
    ds.d = si.valid ? vdiv(rel, ds.dist) : -si.wi;
    return area_pdf_direction(S, em, ds) * S.inv_n_emitters;
}

// AreaLight::sample_direction -> Shape::sample_direction -> Rectangle::sample_position
// (area.cpp:118-168, shape.cpp:358-375, rectangle.cpp:166-180)
MH_DEV V3 area_sample_direction(const DScene &S, uint32_t em, V3 ref_p, float sx, float sy,
                                DirS &ds) {
    const DEmitter &e = S.emitters[em];
    const DShape &sh = S.shapes[e.shape];
    ds.p = xf_point(sh.to_world, v3(sx * 2.f - 1.f, sy * 2.f - 1.f, 0.f));
    ds.n = ld3(sh.frame_n);
    ds.pdf = sh.inv_area;
    ds.delta = false;
    ds.d = ds.p - ref_p;
    float dist2 = dot(ds.d, ds.d);
    ds.dist = __builtin_sqrtf(dist2);
    ds.d = vdiv(ds.d, ds.dist);
    float dp = __builtin_fabsf(dot(ds.d, ds.n));
    float x = dist2 / dp;
    ds.pdf *= isfinite_(x) ? x : 0.f;
    bool active = dot(ds.d, ds.n) < 0.f && ds.pdf != 0.f;
    if (!active) return v3(0, 0, 0);
    return vdiv(v3(e.radiance[0], e.radiance[1], e.radiance[2]), ds.pdf);
}

constexpr float kInv4Pi = 0.07957747154594766788f;

// warp::square_to_uniform_sphere (core/warp.h:250-255)
MH_DEV V3 square_to_uniform_sphere(float sx, float sy) {
    float z = __builtin_fmaf(-2.f, sy, 1.f);
    float r = __builtin_sqrtf(fmaxf(__builtin_fmaf(-z, z, 1.f), 0.f));
    float s, c;
    sincos_cephes((2.f * kPi) * sx, s, c);
    return v3(r * c, r * s, z);
}

// Emitter::sample_direction: area (area.cpp:118-168), constant
// (constant.cpp:112-140), directional (directional.cpp:150-175)
MH_DEV V3 emitter_sample_direction(const DScene &S, uint32_t em, V3 ref_p, float sx, float sy, DirS &ds) {
    const DEmitter &e = S.emitters[em];
    if (e.type == MH_EMITTER_AREA) return area_sample_direction(S, em, ref_p, sx, sy, ds);
    if (e.type == MH_EMITTER_CONSTANT) {
        V3 d = square_to_uniform_sphere(sx, sy);
        V3 c = v3(e.center[0], e.center[1], e.center[2]);
        float radius = fmaxf(e.radius, norm(ref_p - c)), dist = 2.f * radius;
        ds.p = fma3s(d, dist, ref_p);
        ds.n = -d;
        ds.pdf = kInv4Pi;
        ds.delta = false;
        ds.d = d;
        ds.dist = dist;
        return vdiv(v3(e.radiance[0], e.radiance[1], e.radiance[2]), ds.pdf);
    }
    // directional: ds.p = p - d * inf (NaN where d has a zero component, as in the reference)
    V3 d = v3(e.direction[0], e.direction[1], e.direction[2]);
    const float dist = __builtin_huge_valf();
    ds.p = ref_p - d * dist;
    ds.n = d;
    ds.pdf = 1.f;
    ds.delta = true;
    ds.d = -d;
    ds.dist = dist;
    return v3(e.radiance[0], e.radiance[1], e.radiance[2]);
}

// Scene::sample_emitter_direction without the visibility test (scene.cpp:299-353)
MH_DEV V3 scene_sample_emitter_direction(const DScene &S, V3 ref_p, float sx, float sy, DirS &ds) {
    ds.p = ds.n = ds.d = v3(0, 0, 0);
    ds.dist = ds.pdf = 0.f;
    ds.delta = false;
    const uint32_t n = S.n_emitters;
    if (n == 0) return v3(0, 0, 0);
    if (n == 1) return emitter_sample_direction(S, 0, ref_p, sx, sy, ds);
    const float nf = S.n_emitters_f, scaled = sx * nf;  // (float)n, converted on the host
    uint32_t idx = (uint32_t)scaled;
    if (idx > n - 1) idx = n - 1;
    V3 spec = emitter_sample_direction(S, idx, ref_p, scaled - (float)idx, sy, ds);
    ds.pdf *= S.inv_n_emitters;  // 1 / nf, divided on the host
    return spec * nf;
}

MH_DEV V3 emitter_eval(const DScene &S, uint32_t em, const SI &si) {
    const DEmitter &e = S.emitters[em];
    V3 L = v3(e.radiance[0], e.radiance[1], e.radiance[2]);
    if (e.type == MH_EMITTER_AREA) return si.wi.z > 0.f ? L : v3(0, 0, 0);
    if (e.type == MH_EMITTER_CONSTANT) return L;
    return v3(0, 0, 0);
}

// Scene::pdf_emitter_direction of DirectionSample3f(scene, si, ref) (scene.cpp:355-366)
MH_DEV float emitter_pdf_direction(const DScene &S, uint32_t em, const SI &si, V3 ref_p) {
    const DEmitter &e = S.emitters[em];
    if (e.type == MH_EMITTER_AREA) return emitter_hit_pdf(S, em, si, ref_p);
    if (e.type == MH_EMITTER_CONSTANT) return S.env_pdf;  // kInv4Pi * inv_n_emitters, multiplied on the host
    return 0.f;
}

// Scene::sample_emitter_direction (scene.cpp:299-353) with the shadow test;
// a sample whose weight is exactly zero traces no shadow ray.
MH_DEV V3 sample_emitter_direction(const DScene &S, const LdsBvh &B, const SI &si, float sx,
                                   float sy, DirS &ds, uint32_t &n_shadow) {
    V3 spec = scene_sample_emitter_direction(S, si.p, sx, sy, ds);
    if (ds.pdf != 0.f && nonzero(spec)) {
        RayT r = spawn_ray_to(si.p, si.n, ds.p);
        Hit h;
        ++n_shadow;
        if (traverse<true>(B.nodes, B.prims, B.stack, B.stride, r, h)) {
            spec = v3(0, 0, 0);
            ds.pdf = 0.f;
        }
    }
    return spec;
}

// PerspectiveCamera::sample_ray_differential (sensors/perspective.cpp:240-281)
MH_DEV RayT camera_ray(const DScene &S, float ax, float ay) {
    const float *m = S.sample_to_camera;
    float r4[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
        r4[i] = __builtin_fmaf(m[4 * i + 2], 0.f,
                               __builtin_fmaf(m[4 * i + 1], ay + 0.f, __builtin_fmaf(m[4 * i + 0], ax + 0.f, m[4 * i + 3])));
    V3 near_p = v3(r4[0] / r4[3], r4[1] / r4[3], r4[2] / r4[3]);
    V3 d = normalize(near_p);
    const float *w = S.cam_to_world;
    RayT r;
    r.o = v3(w[3], w[7], w[11]);
    r.d = v3(__builtin_fmaf(w[2], d.z, __builtin_fmaf(w[1], d.y, w[0] * d.x)),
             __builtin_fmaf(w[6], d.z, __builtin_fmaf(w[5], d.y, w[4] * d.x)),
             __builtin_fmaf(w[10], d.z, __builtin_fmaf(w[9], d.y, w[8] * d.x)));
    float inv_z = rcp(d.z);
    float near_t = S.near_clip * inv_z, far_t = S.far_clip * inv_z;
    r.o = r.o + r.d * near_t;
    r.maxt = far_t - near_t;
    return r;
}

// ===========================================================================
// Lane -> pixel mapping (integrator.cpp:323-340), sample-slab aware
// ===========================================================================


MH_DEV void lane_of(const LaneMap &m, uint64_t k, uint32_t &lane, uint32_t &px, uint32_t &py) {
    // k < 2^32: a wavefront holds at most 2^32 samples (make_layout).  The
    // divisions stay the compiler's: multiply-high forms with host-made
    // multipliers freed the generating kernels' spills but measured 0.3-0.6 %
    // slower on the bench (same box, 2 runs each)
    const uint32_t k32 = (uint32_t)k;
    uint32_t pl, sl;
    if (m.log_S < 32) { pl = k32 >> m.log_S; sl = k32 & ((1u << m.log_S) - 1u); }
    else { pl = k32 / m.S; sl = k32 - pl * m.S; }
    uint32_t pixel = m.pixel_begin + pl;
    lane = pixel * m.spp_pp + (m.s_begin + sl);
    // recompute the reference's own mapping from the lane index
    uint32_t pix2 = m.log_spp < 32 ? (lane >> m.log_spp) : lane / m.spp_pp;
    py = pix2 / m.W;
    px = pix2 - m.W * py;
}

// wave-aggregated counter increment
MH_DEV void wave_count(unsigned long long *ctr, uint32_t v) {
    // sum across the wave with a butterfly, one atomic by the first active lane
    uint32_t s = v;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    if ((threadIdx.x & 63) == (uint32_t)__ffsll(__ballot(1)) - 1u && s)
        atomicAdd(ctr, (unsigned long long)s);
}

// ===========================================================================
// PathIntegrator::sample, JIT semantics (integrators/path.cpp:95-287)
// ===========================================================================
MH_DEV V3 path_sample(const DScene &S, const LdsBvh &B, const IntegratorParams &in, Pcg &rng,
                      RayT ray, uint32_t &n_closest, uint32_t &n_shadow, bool *valid_out = nullptr) {
    if (in.max_depth == 0) return v3(0, 0, 0);
    V3 throughput = v3(1, 1, 1), result = v3(0, 0, 0);
    float eta = 1.f;
    uint32_t depth = 0;
    bool valid_ray = !in.hide_emitters && S.environment != MH_INVALID;
    V3 prev_p = v3(0, 0, 0);
    float prev_bsdf_pdf = 1.f;
    bool prev_bsdf_delta = true;
    bool active = true;
    while (active) {
        Hit h;
        traverse<false>(B.nodes, B.prims, B.stack, B.stride, ray, h);
        ++n_closest;
        SI si;
        compute_si(S, ray, h, si);

        // ---- direct emission (path.cpp:158-174)
        uint32_t em = si.valid ? S.shapes[si.shape].emitter : S.environment;
        if (em != MH_INVALID) {
            float em_pdf = prev_bsdf_delta ? 0.f : emitter_pdf_direction(S, em, si, prev_p);
            float mis_bsdf = mis_weight(prev_bsdf_pdf, em_pdf);
            V3 le = v3(0, 0, 0);
            if (prev_bsdf_pdf > 0.f)
                le = emitter_eval(S, em, si);
            result = fma3(throughput, le * mis_bsdf, result);
        }

        bool active_next = (depth + 1 < in.max_depth) && si.valid;
        uint32_t b = si.valid ? S.shapes[si.shape].bsdf : MH_INVALID;
        bool smooth = b != MH_INVALID && S.bsdf_type[b] == MH_BSDF_DIFFUSE;
        bool active_em = active_next && smooth;

        // ---- emitter sampling (path.cpp:187-208)
        float e0 = rng.next_float(), e1 = rng.next_float();
        DirS ds;
        ds.pdf = 0.f;
        ds.d = v3(0, 0, 0);
        ds.delta = false;
        V3 em_weight = v3(0, 0, 0), wo = v3(0, 0, 0);
        if (active_em) {
            em_weight = sample_emitter_direction(S, B, si, e0, e1, ds, n_shadow);
            active_em = ds.pdf != 0.f;
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

        // ---- emitter sampling contribution (path.cpp:220-230)
        if (active_em) {
            float mis_em = ds.delta ? 1.f : mis_weight(ds.pdf, bsdf_pdf);
            result = fma3(throughput, (bsdf_val * em_weight) * mis_em, result);
        }

        // ---- BSDF sampling + state update (path.cpp:234-262)
        ray = spawn_ray(si.p, si.n, to_world(si, bs_wo));
        throughput = throughput * bsdf_weight;
        eta *= bs_eta;
        valid_ray = valid_ray || si.valid;
        prev_p = si.p;
        prev_bsdf_pdf = bs_pdf;
        prev_bsdf_delta = false;

        // ---- stopping criterion (path.cpp:266-280)
        if (si.valid) depth += 1;
        float tmax = hmax(throughput);
        float rr_prob = fminf(tmax * (eta * eta), 0.95f);
        bool rr_active = depth >= in.rr_depth;
        bool rr_continue = rng.next_float() < rr_prob;
        if (rr_active) throughput = throughput * rcp(rr_prob);
        active = active_next && (!rr_active || rr_continue) && tmax != 0.f;
    }
    if (valid_out) *valid_out = valid_ray;  // alpha (integrator.cpp:1229-1231)
    return valid_ray ? result : v3(0, 0, 0);
}

// ===========================================================================
// PRBIntegrator.sample (python/ad/integrators/prb.py:59-257)
//   primal (Grad == false) or adjoint (Grad == true, L = primal radiance)
// ===========================================================================
struct GradCtx {
    const int32_t *slot_of_tex;   // texture -> param slot or -1
    float *const *bufs;           // per slot gradient buffer
    const uint32_t *is_rgb;       // per slot
    V3 acc0, acc1, acc2, acc3;    // per-lane accumulators of the small slots 0..3 (named, never indexed:
                                  // one runtime-indexed access would put the whole context in scratch)
    const int32_t *sigma_slot;    // prbvolpath: medium -> sigma_t slot or -1 (nullptr: none)
    const int32_t *albedo_slot;   // prbvolpath: medium -> albedo slot or -1 (nullptr: none)
    float *const *corner;         // prbvolpath: slot -> per-cell corner block of a grid (nullptr: atomics into bufs)
    uint32_t fx_mode;             // GradArgs::fx_mode (deterministic grid gradient)
    uint32_t *fx_max;
    double fx_scale;
    long long *fx_i64;            // GradArgs::fx_i64 / fx_f32 (deterministic bitmap texels, replay kernel)
    const float *fx_f32;
    int32_t lds_slot;             // bitmap slot whose texels accumulate in LDS (-1: none)
    float *lds_acc;               // that slot's workgroup accumulator
    uint32_t lds_floats;          // its size (floats; checked under MH_DEBUG)
    // forward mode (render_forward, common.py:696-826): bufs hold the input
    // tangents, and every adjoint sink adds <adj, tangent> to fsum instead of
    // scattering -- with dL = e_c that is the channel-c tangent radiance
    bool fwd;
    float fsum;
    int32_t hot_med, hot_sigma, hot_albedo;  // GradArgs::hot_* (the first medium with a parameter)
    float *hot_buf, *hot_corner;
};

// register accumulator of a small (rgb / scalar) parameter slot
static_assert(kMaxRgbParams == 4, "GradCtx names four small-slot accumulators");
// MH_FLAG_DETERMINISTIC on prbvolpath (GradCtx::fx_mode): the small slots go
// to int64 fixed point like the grid; the words after fx_max hold the
// per-slot scales (doubles at byte 64) and sums (int64 x 3 at byte 192)
// Pass 2 sums each wave's contributions in LDS (ds_add_u64: integer adds are
// exact, so their order does not matter) and adds them to the global words
// once per wave and component at the flush (flush_small_slots), instead of
// three global int64 atomics on one word per contribution.  Every kernel that
// builds a GradCtx does so and flushes it with whole waves.
constexpr uint32_t kFxWaveWords = 3 * kMaxRgbParams, kFxMaxWaves = 16;  // blocks of up to 1024 threads
static __shared__ unsigned long long g_fx_wave[kFxMaxWaves * kFxWaveWords];
// static LDS a kernel holding a GradCtx carries beside its dynamic bytes
// (host budgets subtract it; hipFuncGetAttributes gives the exact figure)
constexpr uint32_t kFxStaticLdsBytes = (uint32_t)sizeof(g_fx_wave);
MH_DEV unsigned long long *fx_wave_sums() { return g_fx_wave + (threadIdx.x >> 6) * kFxWaveWords; }
// Pass 1 keeps the wave's maxima (the grid's, then each small slot's, as the
// bits of non-negative floats) in the same LDS words and flushes them with one
// global atomicMax per wave and word: every lane of every wave maxing one
// global word serialised the pass on that word's L2 channel (config 4: the
// deterministic backward 198 ms against 35 ms).
MH_DEV unsigned int *fx_wave_max() { return reinterpret_cast<unsigned int *>(fx_wave_sums()); }
MH_DEV void acc_add_fx(GradCtx &g, int32_t k, V3 a) {
    if (g.fx_mode == 1) {
        const float m = fmaxf(fabsf(a.x), fmaxf(fabsf(a.y), fabsf(a.z)));
        if (m > 0.f) atomicMax(fx_wave_max() + 1 + k, __float_as_uint(m));
        return;
    }
    const double sc = reinterpret_cast<const double *>(reinterpret_cast<const uint8_t *>(g.fx_max) + 64)[k];
    unsigned long long *w = fx_wave_sums() + 3 * k;
    atomicAdd(w + 0, (unsigned long long)__double2ll_rn((double)a.x * sc));
    atomicAdd(w + 1, (unsigned long long)__double2ll_rn((double)a.y * sc));
    atomicAdd(w + 2, (unsigned long long)__double2ll_rn((double)a.z * sc));
}
// a bitmap texel's charge in fixed point (MH_FLAG_DETERMINISTIC on the replay
// kernel): pass 1 the slot's largest |item| (wave max in LDS, word 1 + k),
// pass 2 round(item * scale_k) added as int64 at the texel's mirror in fx_i64
MH_DEV void bmp_add_fx(const GradCtx &g, int32_t k, const float *dst, float v) {
    if (g.fx_mode == 1) {
        const float a = fabsf(v);
        if (a > 0.f) atomicMax(fx_wave_max() + 1 + k, __float_as_uint(a));
        return;
    }
    const double sc = reinterpret_cast<const double *>(reinterpret_cast<const uint8_t *>(g.fx_max) + 64)[k];
    gatomic_add(reinterpret_cast<unsigned long long *>(g.fx_i64 + (dst - g.fx_f32)),
              (unsigned long long)__double2ll_rn((double)v * sc));
}
MH_DEV void acc_add(GradCtx &g, int32_t k, V3 a) {
    if (g.fx_mode) { acc_add_fx(g, k, a); return; }
    if (k == 0) g.acc0 = g.acc0 + a;
    else if (k == 1) g.acc1 = g.acc1 + a;
    else if (k == 2) g.acc2 = g.acc2 + a;
    else if (k == 3) g.acc3 = g.acc3 + a;
}
MH_DEV V3 acc_get(const GradCtx &g, int32_t k) {
    return k == 0 ? g.acc0 : k == 1 ? g.acc1 : k == 2 ? g.acc2 : k == 3 ? g.acc3 : v3(0.f, 0.f, 0.f);
}

// ---------------------------------------------------------------------------
// Texel gradients of a wave, grouped by address.  The lanes of a coherent wave
// (the samples of one pixel at their camera vertex) add to the same few
// texels, and same-address ds_add_f32 of one instruction serialize lane by
// lane.  The largest group (the first pending lane's address and every lane
// sharing it) is summed across the wave (__ockl_wfred_add_f32, a DPP
// reduction) and added by one lane; the next group follows while groups stay
// large (>= kGroupMin lanes), and the remaining, incoherent lanes add on their
// own.  The whole wave must be active (the DPP reduction reads every lane:
// measured wrong sums from the divergent replay loop), hence `on` masks.
// ---------------------------------------------------------------------------
extern "C" __device__ float __ockl_wfred_add_f32(float);
typedef __attribute__((address_space(3))) float LdsFloat;
// gfx950 runs a no-return ds_add_f32 at ~190 CU cycles per 64-lane
// instruction (~3 per active lane; any address pattern), ds_add_f64 at ~26,
// ds_add_u32 at ~12 (tools/exp_ldsatomic.hip, profiles/r5_lds_atomics.txt):
// an LDS accumulator that takes many adds is kept in double
typedef __attribute__((address_space(3))) double LdsDouble;
#ifndef MH_GROUP_MIN
#define MH_GROUP_MIN 6
#endif
constexpr int kGroupMin = MH_GROUP_MIN, kGroupIters = 4;

template <int C, typename Acc>
MH_DEV void lds_add_grouped(Acc *acc, uint32_t key, bool on, const float (&v)[C]) {
    using T = __typeof__(+*acc);
    const uint32_t me = __lane_id();
    for (int it = 0; it < kGroupIters; ++it) {
        const uint64_t m = __ballot(on);
        if (m == 0) return;
        const uint32_t leader = (uint32_t)__ffsll((unsigned long long)m) - 1u;
        const uint32_t kl = (uint32_t)__builtin_amdgcn_readlane((int)key, (int)leader);
        const bool mine = on && key == kl;
        if (__popcll(__ballot(mine)) < kGroupMin) break;
        float s[C];
#pragma unroll
        for (int c = 0; c < C; ++c) s[c] = __ockl_wfred_add_f32(mine ? v[c] : 0.f);
        if (me == leader) {
#pragma unroll
            for (int c = 0; c < C; ++c)
                __hip_atomic_fetch_add(acc + kl + c, (T)s[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        on = on && !mine;
    }
    if (on) {
#pragma unroll
        for (int c = 0; c < C; ++c)
            __hip_atomic_fetch_add(acc + key + c, (T)v[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}

// tangent of a reflectance texture at uv: tex_eval's taps and operation order
// over the tangent texels of its slot (the bitmap is linear in its data), or
// the slot's rgb tangent; zero when the texture is not differentiated
MH_DEV V3 tex_tangent(const DScene &S, uint32_t tex, float uvx, float uvy, const GradCtx &g) {
    const int32_t k = g.slot_of_tex[tex];
    if (k < 0) return v3(0.f, 0.f, 0.f);
    const float *t = g.bufs[k];
    if (g.is_rgb[k]) return v3(t[0], t[1], t[2]);
    const DTexture &tx = S.textures[tex];
    Taps tp;
    bitmap_taps(tx, uvx, uvy, tp);
    float out[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const uint64_t cc = tx.channels == 3 ? (uint64_t)c : 0u;
        if (tp.n == 1) {
            out[c] = t[tp.idx[0] - tx.data_offset + cc];
        } else {
            const float f00 = t[tp.idx[0] - tx.data_offset + cc], f10 = t[tp.idx[1] - tx.data_offset + cc],
                        f01 = t[tp.idx[2] - tx.data_offset + cc], f11 = t[tp.idx[3] - tx.data_offset + cc];
            out[c] = __builtin_fmaf(tp.w0y, __builtin_fmaf(tp.w0x, f00, tp.w1x * f10),
                                    tp.w1y * __builtin_fmaf(tp.w0x, f01, tp.w1x * f11));
        }
    }
    return v3(out[0], out[1], out[2]);
}

MH_DEV void tex_backward(const DScene &S, uint32_t tex, float uvx, float uvy, V3 adj, GradCtx &g) {
    int32_t k = g.slot_of_tex[tex];
    if (k < 0) return;
    if (g.fwd) {
        const V3 t = tex_tangent(S, tex, uvx, uvy, g);
        g.fsum += (adj.x * t.x + adj.y * t.y) + adj.z * t.z;
        return;
    }
    const DTexture &tx = S.textures[tex];
    if (g.is_rgb[k]) {
        acc_add(g, k, adj);
        return;
    }
    Taps tp;
    bitmap_taps(tx, uvx, uvy, tp);
    // a lane-coherent wave adds to the same few texels: in LDS (ds_add_f32)
    // those same-address adds cost a few cycles, at L2 a round trip each
    const bool in_lds = k == g.lds_slot;
    float *buf = in_lds ? g.lds_acc : g.bufs[k];
    float w[4] = {1.f, 0.f, 0.f, 0.f};
    if (tp.n == 1) { w[0] = 1.f; }
    else { w[0] = tp.w0y * tp.w0x; w[1] = tp.w0y * tp.w1x; w[2] = tp.w1y * tp.w0x; w[3] = tp.w1y * tp.w1x; }
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        if (j >= tp.n) break;
        uint64_t base = tp.idx[j] - tx.data_offset;
        if (in_lds) {  // ds_add_f32 (an LDS-qualified pointer, not a flat atomic)
            MH_GUARD(base + tx.channels <= g.lds_floats, kGuardLds);
            // (not lds_add_grouped: the replay's lanes are divergent here)
            LdsFloat *l = (LdsFloat *)(buf + base);
            if (tx.channels == 3) {
                __hip_atomic_fetch_add(l + 0, adj.x * w[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_fetch_add(l + 1, adj.y * w[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_fetch_add(l + 2, adj.z * w[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            } else {
                __hip_atomic_fetch_add(l, (adj.x + adj.y + adj.z) * w[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            continue;
        }
        if (g.fx_mode) {  // deterministic replay (the host keeps such a slot out of LDS)
            if (tx.channels == 3) {
                bmp_add_fx(g, k, buf + base + 0, adj.x * w[j]);
                bmp_add_fx(g, k, buf + base + 1, adj.y * w[j]);
                bmp_add_fx(g, k, buf + base + 2, adj.z * w[j]);
            } else {
                bmp_add_fx(g, k, buf + base, (adj.x + adj.y + adj.z) * w[j]);
            }
            continue;
        }
        if (tx.channels == 3) {
            gatomic_add(buf + base + 0, adj.x * w[j]);
            gatomic_add(buf + base + 1, adj.y * w[j]);
            gatomic_add(buf + base + 2, adj.z * w[j]);
        } else {
            gatomic_add(buf + base, (adj.x + adj.y + adj.z) * w[j]);
        }
    }
}

template <bool Grad>
MH_DEV V3 prb_sample(const DScene &S, const LdsBvh &B, const IntegratorParams &in, Pcg &rng,
                     RayT ray, V3 dL, V3 L, GradCtx *g, uint32_t &n_closest, uint32_t &n_shadow,
                     bool *valid_out = nullptr) {
    uint32_t depth = 0;
    if (!Grad) L = v3(0, 0, 0);
    V3 beta = v3(1, 1, 1);
    float eta = 1.f;
    bool active = true;
    V3 prev_p = v3(0, 0, 0);
    float prev_bsdf_pdf = 1.f;
    bool prev_bsdf_delta = true;
    while (active) {
        bool active_next = active;
        Hit h;
        traverse<false>(B.nodes, B.prims, B.stack, B.stride, ray, h);
        ++n_closest;
        SI si;
        compute_si(S, ray, h, si);
        uint32_t b = si.valid ? S.shapes[si.shape].bsdf : MH_INVALID;
        bool smooth = b != MH_INVALID && S.bsdf_type[b] == MH_BSDF_DIFFUSE;
        if (in.hide_emitters && depth == 0 && !si.valid) active_next = false;

        // ---- direct emission (prb.py:121-135)
        uint32_t em = si.valid ? S.shapes[si.shape].emitter : S.environment;
        V3 Le = v3(0, 0, 0);
        if (em != MH_INVALID) {
            float em_pdf = prev_bsdf_delta ? 0.f : emitter_pdf_direction(S, em, si, prev_p);
            float mis = mis_weight(prev_bsdf_pdf, em_pdf);
            V3 le = v3(0, 0, 0);
            if (active_next)
                le = emitter_eval(S, em, si);
            Le = (beta * mis) * le;
        }

        // ---- emitter sampling (prb.py:139-163)
        active_next = active_next && (depth + 1 < in.max_depth) && si.valid;
        bool active_em = active_next && smooth;
        float e0 = rng.next_float(), e1 = rng.next_float();
        DirS ds;
        ds.pdf = 0.f;
        ds.d = v3(0, 0, 0);
        ds.delta = false;
        V3 em_weight = v3(0, 0, 0);
        if (active_em) {
            em_weight = sample_emitter_direction(S, B, si, e0, e1, ds, n_shadow);
            active_em = ds.pdf != 0.f;
        }
        V3 rho = v3(0, 0, 0);
        if (smooth) rho = tex_eval(S, S.bsdf_tex[b], si.uvx, si.uvy);
        V3 wo_em = to_local(si, ds.d);
        V3 bsdf_value_em;
        float bsdf_pdf_em;
        diffuse_eval_pdf(rho, si.wi, wo_em, active_em, bsdf_value_em, bsdf_pdf_em);
        float mis_em = ds.delta ? 1.f : mis_weight(ds.pdf, bsdf_pdf_em);
        V3 beta_mis_em = beta * mis_em;
        V3 Lr_dir = active_em ? (beta_mis_em * bsdf_value_em) * em_weight : v3(0, 0, 0);

        // ---- detached BSDF sampling (prb.py:167-170)
        (void)rng.next_float();
        float s2x = rng.next_float(), s2y = rng.next_float();
        V3 bs_wo = v3(0, 0, 0), bsdf_weight = v3(0, 0, 0);
        float bs_pdf = 0.f, bs_eta = 0.f;
        if (smooth && active_next) {
            bs_wo = square_to_cosine_hemisphere(s2x, s2y);
            bs_pdf = kInvPi * bs_wo.z;
            bs_eta = 1.f;
            bsdf_weight = (si.wi.z > 0.f && bs_pdf > 0.f) ? rho : v3(0, 0, 0);
        }

        // ---- state update (prb.py:174-199)
        L = Grad ? (L - Le) - Lr_dir : (L + Le) + Lr_dir;
        ray = spawn_ray(si.p, si.n, to_world(si, bs_wo));
        eta *= bs_eta;
        beta = beta * bsdf_weight;
        prev_p = si.p;
        prev_bsdf_pdf = bs_pdf;
        prev_bsdf_delta = false;
        float beta_max = hmax(beta);
        active_next = active_next && beta_max != 0.f;
        float rr_prob = fminf(beta_max * (eta * eta), 0.95f);
        bool rr_active = depth >= in.rr_depth;
        if (rr_active) beta = beta * rcp(rr_prob);
        bool rr_continue = rng.next_float() < rr_prob;
        active_next = active_next && (!rr_active || rr_continue);

        // ---- differential phase (prb.py:203-248) wrt the diffuse reflectance
        if (Grad && smooth) {
            V3 adj = v3(0, 0, 0);
            if (active_em && si.wi.z > 0.f && wo_em.z > 0.f)
                adj = (((dL * em_weight) * beta_mis_em) * wo_em.z) * kInvPi;
            V3 wo2 = to_local(si, ray.d);
            if (active_next && si.wi.z > 0.f && wo2.z > 0.f) {
                V3 det = bsdf_weight * bs_pdf;
                V3 inv = v3(det.x != 0.f ? rcp(det.x) : 0.f, det.y != 0.f ? rcp(det.y) : 0.f,
                            det.z != 0.f ? rcp(det.z) : 0.f);
                adj = adj + (((dL * L) * inv) * wo2.z) * kInvPi;
            }
            tex_backward(S, S.bsdf_tex[b], si.uvx, si.uvy, adj, *g);
        }

        if (si.valid) depth += 1;
        active = active_next;
    }
    if (valid_out) *valid_out = depth != 0;  // "ray validity flag for alpha blending" (prb.py:253-257)
    return L;
}

// ---------------------------------------------------------------------------
// dL of one sample: the adjoint of ImageBlock::put + develop, i.e. the
// filter-weighted gather of grad_in / W over the sample's footprint
// (common.py:953-965; the W image from common.py:936-947)
// ---------------------------------------------------------------------------
// gw: grad_in / (W == 0 ? 1 : W) per pixel (k_grad_over_w), i.e. the adjoint
// of develop, which Dr.Jit also evaluates once per pixel.
// gw: grad_in / W as one float4 (r, g, b, 0) per pixel (k_grad_over_w), so a
// footprint texel is one 16-B load
MH_DEV V3 gather_dL(const DScene &S, int coalesce, const float *__restrict__ gw, float px, float py) {
    const float4 *__restrict__ g4 = reinterpret_cast<const float4 *>(gw);
    const uint32_t W = S.width, H = S.height;
    float o0 = 0.f, o1 = 0.f, o2 = 0.f;
    if (S.rfilter == MH_RFILTER_BOX) {
        uint32_t ux = (uint32_t)(int32_t)floorf(px), uy = (uint32_t)(int32_t)floorf(py);
        if (ux < W && uy < H) {
            uint64_t p = (uint64_t)uy * W + ux;
            const float4 g = g4[p];
            o0 = g.x; o1 = g.y; o2 = g.z;
        }
        return v3(o0, o1, o2);
    }
    const float radius = S.rfilter_radius;
    if (coalesce) {
        int32_t nn = (int32_t)ceilf(radius - 0.5f), count = 2 * nn + 1;
        if (count > 5) count = 5;  // radius <= 2.5 (host-checked for this path)
        int32_t pix = (int32_t)floorf(px) - nn, piy = (int32_t)floorf(py) - nn;
        float relx = ((float)pix + 0.5f) - px, rely = ((float)piy + 0.5f) - py;
        float wxs[5];
#pragma unroll
        for (int32_t xs = 0; xs < 5; ++xs) wxs[xs] = xs < count ? gaussian_eval(S.filter_coeff, relx + (float)xs) : 0.f;
#pragma unroll
        for (int32_t ys = 0; ys < 5; ++ys) {
            if (ys >= count) break;
            float wy = gaussian_eval(S.filter_coeff, rely + (float)ys);
            uint32_t yy = (uint32_t)(piy + ys);
#pragma unroll
            for (int32_t xs = 0; xs < 5; ++xs) {
                uint32_t xx = (uint32_t)(pix + xs);
                if (xs < count && xx < W && yy < H) {
                    const float4 g = g4[(uint64_t)yy * W + xx];
                    float w = wy * wxs[xs];
                    o0 += g.x * w;
                    o1 += g.y * w;
                    o2 += g.z * w;
                }
            }
        }
    } else {
        float pfx = px - 0.5f, pfy = py - 0.5f;
        int32_t a0x = max((int32_t)ceilf(pfx - radius), 0), a0y = max((int32_t)ceilf(pfy - radius), 0);
        int32_t a1x = min((int32_t)floorf(pfx + radius), (int32_t)W - 1);
        int32_t a1y = min((int32_t)floorf(pfy + radius), (int32_t)H - 1);
        if (!(a0x <= a1x && a0y <= a1y)) return v3(0, 0, 0);
        uint32_t count = (uint32_t)ceilf(2.f * radius);
        float relx = (float)a0x - pfx, rely = (float)a0y - pfy;
        for (uint32_t ys = 0; ys < count; ++ys) {
            float wy = gaussian_eval(S.filter_coeff, rely + (float)ys);
            for (uint32_t xs = 0; xs < count; ++xs) {
                float wx = gaussian_eval(S.filter_coeff, relx + (float)xs);
                int32_t xx = a0x + (int32_t)xs, yy = a0y + (int32_t)ys;
                if (xx <= a1x && yy <= a1y) {
                    const float4 g = g4[(uint64_t)yy * W + xx];
                    float w = wy * wx;
                    o0 += g.x * w;
                    o1 += g.y * w;
                    o2 += g.z * w;
                }
            }
        }
    }
    return v3(o0, o1, o2);
}

// gather_dL for a wave whose active lanes share one footprint -- the usual
// case: the wavefront is pixel-major, so a wave holds 64 samples of one pixel
// at >= 64 spp per slab.  The 25 grad / W texels are then wave-uniform and
// are read once through the scalar cache (s_load into SGPRs, the operands of
// the multiplies) instead of by 25 vector loads per lane, and the 10 filter
// weights run on packed f32.  Per lane the operations and their order are
// gather_dL's, so dL is bit-identical; any other wave (box filter, spp < 4,
// lanes of several pixels) takes gather_dL.
MH_DEV F2 gaussian_eval2(const float *k, F2 x) {
    const F2 X = x * x;  // estrin10(x * x, k), two arguments per instruction
    const F2 c0 = fma2(X, sp2(k[1]), sp2(k[0])), c1 = fma2(X, sp2(k[3]), sp2(k[2])),
             c2 = fma2(X, sp2(k[5]), sp2(k[4])), c3 = fma2(X, sp2(k[7]), sp2(k[6])),
             c4 = fma2(X, sp2(k[9]), sp2(k[8]));
    const F2 X2 = X * X;
    const F2 d0 = fma2(X2, c1, c0), d1 = fma2(X2, c3, c2);
    const F2 X4 = X2 * X2;
    const F2 e0 = fma2(X4, d1, d0);
    const F2 X8 = X4 * X4;
    const F2 r = fma2(X8, c4, e0);
    return pair(fmaxf(r.x, 0.f), fmaxf(r.y, 0.f));
}

MH_DEV V3 gather_dL_wave(const DScene &S, int coalesce, const float *__restrict__ gw, float px, float py) {
    if (!(coalesce && S.rfilter == MH_RFILTER_GAUSSIAN && S.rfilter_radius > 1.5f && S.rfilter_radius <= 2.5f))
        return gather_dL(S, coalesce, gw, px, py);
    const int32_t fx = (int32_t)floorf(px), fy = (int32_t)floorf(py);
    const int32_t ux = __builtin_amdgcn_readfirstlane(fx), uy = __builtin_amdgcn_readfirstlane(fy);
    if (__builtin_amdgcn_ballot_w64(fx != ux || fy != uy) != 0) return gather_dL(S, coalesce, gw, px, py);
    const int32_t pix = ux - 2, piy = uy - 2;  // nn = ceil(radius - 0.5) = 2, count = 5
    const float relx = ((float)pix + 0.5f) - px, rely = ((float)piy + 0.5f) - py;
    const F2 wa = gaussian_eval2(S.filter_coeff, pair(relx + 0.f, relx + 1.f)),
             wb = gaussian_eval2(S.filter_coeff, pair(relx + 2.f, relx + 3.f)),
             wc = gaussian_eval2(S.filter_coeff, pair(relx + 4.f, rely + 0.f)),
             wd = gaussian_eval2(S.filter_coeff, pair(rely + 1.f, rely + 2.f)),
             we = gaussian_eval2(S.filter_coeff, pair(rely + 3.f, rely + 4.f));
    const float wxs[5] = {wa.x, wa.y, wb.x, wb.y, wc.x}, wys[5] = {wc.y, wd.x, wd.y, we.x, we.y};
    const uint32_t W = S.width, H = S.height;
    float o0 = 0.f, o1 = 0.f, o2 = 0.f;
#pragma unroll
    for (int32_t ys = 0; ys < 5; ++ys) {
        const uint32_t yy = (uint32_t)(piy + ys);
        if (yy >= H) continue;  // wave-uniform
        const float wy = wys[ys];
#pragma unroll
        for (int32_t xs = 0; xs < 5; ++xs) {
            const uint32_t xx = (uint32_t)(pix + xs);
            if (xx >= W) continue;
            const CFloat *t = (CFloat *)gw + 4ull * ((uint64_t)yy * W + xx);
            const float w = wy * wxs[xs];
            o0 += t[0] * w;
            o1 += t[1] * w;
            o2 += t[2] * w;
        }
    }
    return v3(o0, o1, o2);
}

// gather_dL_wave with the footprint staged in LDS: lanes 0..24 each load one
// grad / W texel (a vector load) into the wave's LDS scratch, and every lane
// reads the 25 taps back as broadcast ds_read_b128.  The scalar-cache form
// holds the 25 float4 taps in 100 SGPRs, which the fused PRB bounce (already
// at the SGPR limit) spills; here the taps pass through VGPRs one at a time.
// Same taps, weights and summation order: bit-identical dL.
MH_DEV V3 gather_dL_wave_lds(const DScene &S, int coalesce, const float *__restrict__ gw, float px, float py,
                             uint8_t *scratch) {
    if (!(coalesce && S.rfilter == MH_RFILTER_GAUSSIAN && S.rfilter_radius > 1.5f && S.rfilter_radius <= 2.5f))
        return gather_dL(S, coalesce, gw, px, py);
    const int32_t fx = (int32_t)floorf(px), fy = (int32_t)floorf(py);
    const int32_t ux = __builtin_amdgcn_readfirstlane(fx), uy = __builtin_amdgcn_readfirstlane(fy);
    if (__builtin_amdgcn_ballot_w64(fx != ux || fy != uy) != 0) return gather_dL(S, coalesce, gw, px, py);
    const int32_t pix = ux - 2, piy = uy - 2;  // nn = ceil(radius - 0.5) = 2, count = 5
    const uint32_t W = S.width, H = S.height;
    LdsFloat *taps = (LdsFloat *)scratch;  // 25 x (r, g, b, -)
    // the active lanes (a wave's tail may be partial) share the 25 loads
    const uint64_t act = __builtin_amdgcn_ballot_w64(true);
    const uint32_t n_act = (uint32_t)__popcll(act);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u));
    for (uint32_t t = rank; t < 25u; t += n_act) {
        const uint32_t yy = (uint32_t)(piy + (int32_t)(t / 5u)), xx = (uint32_t)(pix + (int32_t)(t % 5u));
        if (yy < H && xx < W) {
            const float4 g = reinterpret_cast<const float4 *>(gw)[(uint64_t)yy * W + xx];
            taps[4 * t + 0] = g.x;
            taps[4 * t + 1] = g.y;
            taps[4 * t + 2] = g.z;
        }
    }
    const float relx = ((float)pix + 0.5f) - px, rely = ((float)piy + 0.5f) - py;
    const F2 wa = gaussian_eval2(S.filter_coeff, pair(relx + 0.f, relx + 1.f)),
             wb = gaussian_eval2(S.filter_coeff, pair(relx + 2.f, relx + 3.f)),
             wc = gaussian_eval2(S.filter_coeff, pair(relx + 4.f, rely + 0.f)),
             wd = gaussian_eval2(S.filter_coeff, pair(rely + 1.f, rely + 2.f)),
             we = gaussian_eval2(S.filter_coeff, pair(rely + 3.f, rely + 4.f));
    const float wxs[5] = {wa.x, wa.y, wb.x, wb.y, wc.x}, wys[5] = {wc.y, wd.x, wd.y, we.x, we.y};
    if (pix >= 0 && piy >= 0 && (uint32_t)pix + 4u < W && (uint32_t)piy + 4u < H) {
        // interior footprint (wave-uniform): a row's 5 taps read back at once
        // (one LDS wait per row, not per tap), the r / g channels on packed
        // pairs; per channel the same products and sums in the same order as
        // the general loop below (bit-identical dL)
        typedef float F4 __attribute__((ext_vector_type(4)));
        typedef __attribute__((address_space(3))) F4 LdsF4;
        const LdsF4 *t4 = (const LdsF4 *)taps;
        F2 o01 = sp2(0.f);
        float o2 = 0.f;
#pragma unroll
        for (int32_t ys = 0; ys < 5; ++ys) {
            F4 t[5];
#pragma unroll
            for (int32_t xs = 0; xs < 5; ++xs) t[xs] = t4[ys * 5 + xs];
            const float wy = wys[ys];
#pragma unroll
            for (int32_t xs = 0; xs < 5; ++xs) {
                const float w = wy * wxs[xs];
                o01 = o01 + pair(t[xs].x, t[xs].y) * sp2(w);
                o2 += t[xs].z * w;
            }
        }
        return v3(o01.x, o01.y, o2);
    }
    float o0 = 0.f, o1 = 0.f, o2 = 0.f;
#pragma unroll
    for (int32_t ys = 0; ys < 5; ++ys) {
        const uint32_t yy = (uint32_t)(piy + ys);
        if (yy >= H) continue;  // wave-uniform
        const float wy = wys[ys];
#pragma unroll
        for (int32_t xs = 0; xs < 5; ++xs) {
            const uint32_t xx = (uint32_t)(pix + xs);
            if (xx >= W) continue;
            const LdsFloat *t = taps + 4 * (ys * 5 + xs);
            const float w = wy * wxs[xs];
            o0 += t[0] * w;
            o1 += t[1] * w;
            o2 += t[2] * w;
        }
    }
    return v3(o0, o1, o2);
}

// ---------------------------------------------------------------------------
// Fused PRB gradient for constant (rgb) reflectance parameters: ONE traversal
// of the path instead of the primal + adjoint replay of
// RBIntegrator.render_backward (common.py:953-974).  The replay revisits the
// same vertices (same RNG stream) with L_{k+1} = L_total - P_k, where
// P_k = sum_{j<=k} e_j is the primal prefix of the radiance contributions
// e_j = Le_j + Lr_dir_j; the indirect term of prb.py:229-240 summed over the
// vertices k of slot s is therefore
//     sum_k dL (L_total - P_k) c_k / pi = sum_j dL e_j A_s(<j) / pi,
// c_k = cos_ind / (rho pdf) and A_s(<j) = sum_{k<j, slot k = s} c_k: every
// radiance contribution is charged, when it is produced, to the c's of the
// earlier vertices.  No suffix is needed, so the same form serves the
// wavefront kernels (contributions produced in k_wf_shade / k_wf_shadow).
// The direct term (prb.py:208-221) needs only dL.  Mathematically identical
// to the replay; differs by fp association only (tests: 1e-3 relative).
// ---------------------------------------------------------------------------
template <int NR>
MH_DEV void charge(float (&acc)[NR][3], const float (&A)[NR][3], uint32_t n_rgb, V3 dLe) {
#pragma unroll
    for (int kk = 0; kk < NR; ++kk)
        if ((uint32_t)kk < n_rgb) {
            acc[kk][0] = __builtin_fmaf(dLe.x, A[kk][0] * kInvPi, acc[kk][0]);
            acc[kk][1] = __builtin_fmaf(dLe.y, A[kk][1] * kInvPi, acc[kk][1]);
            acc[kk][2] = __builtin_fmaf(dLe.z, A[kk][2] * kInvPi, acc[kk][2]);
        }
}

// adjoint factor c_k of a diffuse vertex (prb.py:229-240 with the
// `inv_bsdf_weight * cos` of the local BSDF eval), zero where the replay's
// active mask / cosines vanish
MH_DEV V3 prb_indirect_factor(bool active_next, const SI &si, V3 wo2, V3 bsdf_weight, float bs_pdf) {
    V3 c = v3(0, 0, 0);
    if (active_next && si.wi.z > 0.f && wo2.z > 0.f) {
        V3 det = bsdf_weight * bs_pdf;
        c = v3(det.x != 0.f ? rcp(det.x) : 0.f, det.y != 0.f ? rcp(det.y) : 0.f,
               det.z != 0.f ? rcp(det.z) : 0.f) * wo2.z;
    }
    return c;
}

template <int NR>
MH_DEV void add_slot(float (&arr)[NR][3], int32_t slot, V3 v) {
#pragma unroll
    for (int kk = 0; kk < NR; ++kk)
    {
        const bool m = kk == slot;  // branch-free: keeps arr in registers
        arr[kk][0] += m ? v.x : 0.f;
        arr[kk][1] += m ? v.y : 0.f;
        arr[kk][2] += m ? v.z : 0.f;
    }
}

MH_DEV void prb_fused(const DScene &S, const LdsBvh &B, const IntegratorParams &in, Pcg &rng,
                      RayT ray, V3 dL, uint32_t n_rgb, GradCtx &g, uint32_t &n_closest, uint32_t &n_shadow) {
    uint32_t depth = 0;
    V3 beta = v3(1, 1, 1);
    float eta = 1.f;
    bool active = true;
    V3 prev_p = v3(0, 0, 0);
    float prev_bsdf_pdf = 1.f;
    bool prev_bsdf_delta = true;
    // the small slots' accumulators as a local array for charge / add_slot
    // (indexed only by unrolled constants), written back to g at the end
    float acc[kMaxRgbParams][3];
#pragma unroll
    for (int kk = 0; kk < kMaxRgbParams; ++kk) {
        const V3 a = acc_get(g, kk);
        acc[kk][0] = a.x; acc[kk][1] = a.y; acc[kk][2] = a.z;
    }
    float A[kMaxRgbParams][3];
#pragma unroll
    for (int k = 0; k < kMaxRgbParams; ++k) A[k][0] = A[k][1] = A[k][2] = 0.f;
    while (active) {
        bool active_next = active;
        Hit h;
        traverse<false>(B.nodes, B.prims, B.stack, B.stride, ray, h);
        ++n_closest;
        SI si;
        compute_si(S, ray, h, si);
        uint32_t b = si.valid ? S.shapes[si.shape].bsdf : MH_INVALID;
        bool smooth = b != MH_INVALID && S.bsdf_type[b] == MH_BSDF_DIFFUSE;
        if (in.hide_emitters && depth == 0 && !si.valid) active_next = false;
        uint32_t em = si.valid ? S.shapes[si.shape].emitter : S.environment;
        if (em != MH_INVALID) {
            float em_pdf = prev_bsdf_delta ? 0.f : emitter_pdf_direction(S, em, si, prev_p);
            float mis = mis_weight(prev_bsdf_pdf, em_pdf);
            V3 le = v3(0, 0, 0);
            if (active_next)
                le = emitter_eval(S, em, si);
            charge(acc, A, n_rgb, dL * ((beta * mis) * le));
        }
        active_next = active_next && (depth + 1 < in.max_depth) && si.valid;
        bool active_em = active_next && smooth;
        float e0 = rng.next_float(), e1 = rng.next_float();
        DirS ds;
        ds.pdf = 0.f;
        ds.d = v3(0, 0, 0);
        ds.delta = false;
        V3 em_weight = v3(0, 0, 0);
        if (active_em) {
            em_weight = sample_emitter_direction(S, B, si, e0, e1, ds, n_shadow);
            active_em = ds.pdf != 0.f;
        }
        V3 rho = v3(0, 0, 0);
        if (smooth) rho = tex_eval(S, S.bsdf_tex[b], si.uvx, si.uvy);
        V3 wo_em = to_local(si, ds.d);
        V3 bsdf_value_em;
        float bsdf_pdf_em;
        diffuse_eval_pdf(rho, si.wi, wo_em, active_em, bsdf_value_em, bsdf_pdf_em);
        float mis_em = ds.delta ? 1.f : mis_weight(ds.pdf, bsdf_pdf_em);
        V3 beta_mis_em = beta * mis_em;
        if (active_em) charge(acc, A, n_rgb, dL * ((beta_mis_em * bsdf_value_em) * em_weight));
        (void)rng.next_float();
        float s2x = rng.next_float(), s2y = rng.next_float();
        V3 bs_wo = v3(0, 0, 0), bsdf_weight = v3(0, 0, 0);
        float bs_pdf = 0.f, bs_eta = 0.f;
        if (smooth && active_next) {
            bs_wo = square_to_cosine_hemisphere(s2x, s2y);
            bs_pdf = kInvPi * bs_wo.z;
            bs_eta = 1.f;
            bsdf_weight = (si.wi.z > 0.f && bs_pdf > 0.f) ? rho : v3(0, 0, 0);
        }
        ray = spawn_ray(si.p, si.n, to_world(si, bs_wo));
        eta *= bs_eta;
        beta = beta * bsdf_weight;
        prev_p = si.p;
        prev_bsdf_pdf = bs_pdf;
        prev_bsdf_delta = false;
        float beta_max = hmax(beta);
        active_next = active_next && beta_max != 0.f;
        float rr_prob = fminf(beta_max * (eta * eta), 0.95f);
        bool rr_active = depth >= in.rr_depth;
        if (rr_active) beta = beta * rcp(rr_prob);
        bool rr_continue = rng.next_float() < rr_prob;
        active_next = active_next && (!rr_active || rr_continue);
        if (smooth) {
            const int32_t slot = g.slot_of_tex[S.bsdf_tex[b]];
            if (slot >= 0) {
                if (active_em && si.wi.z > 0.f && wo_em.z > 0.f)
                    add_slot(acc, slot, (((dL * em_weight) * beta_mis_em) * wo_em.z) * kInvPi);
                add_slot(A, slot, prb_indirect_factor(active_next, si, to_local(si, ray.d), bsdf_weight, bs_pdf));
            }
        }
        if (si.valid) depth += 1;
        active = active_next;
    }
    g.acc0 = v3(acc[0][0], acc[0][1], acc[0][2]);
    g.acc1 = v3(acc[1][0], acc[1][1], acc[1][2]);
    g.acc2 = v3(acc[2][0], acc[2][1], acc[2][2]);
    g.acc3 = v3(acc[3][0], acc[3][1], acc[3][2]);
}

// Forward-mode PRB (render_forward, common.py:696-826; prb.py:244-248
// `δL += dr.forward_to(Lo)`) in the single-traversal form of prb_fused.  The
// replay's tangent at vertex k is (D_k + (L_total - P_k) c_k / pi) * t_k with
// t_k = d rho / d pi . delta pi at the vertex (tex_tangent) and D_k the direct
// term's cos-weighted NEE factor; regrouped as in prb_fused, every radiance
// contribution e_j is charged with T(<j) / pi, T = sum_{k<j} c_k t_k.  T is
// one rgb vector whatever the number of parameters (each vertex brings its
// own t_k, bitmap texels included), so a path carries 6 floats.  Returns the
// sample's tangent radiance dL; valid = depth != 0 (prb.py:253-257).
// ---------------------------------------------------------------------------
MH_DEV V3 prb_forward(const DScene &S, const LdsBvh &B, const IntegratorParams &in, Pcg &rng, RayT ray,
                      const GradCtx &g, uint32_t &n_closest, uint32_t &n_shadow, bool *valid_out) {
    uint32_t depth = 0;
    V3 beta = v3(1, 1, 1), T = v3(0, 0, 0), dL = v3(0, 0, 0);
    float eta = 1.f;
    bool active = true;
    V3 prev_p = v3(0, 0, 0);
    float prev_bsdf_pdf = 1.f;
    bool prev_bsdf_delta = true;
    while (active) {
        bool active_next = active;
        Hit h;
        traverse<false>(B.nodes, B.prims, B.stack, B.stride, ray, h);
        ++n_closest;
        SI si;
        compute_si(S, ray, h, si);
        uint32_t b = si.valid ? S.shapes[si.shape].bsdf : MH_INVALID;
        bool smooth = b != MH_INVALID && S.bsdf_type[b] == MH_BSDF_DIFFUSE;
        if (in.hide_emitters && depth == 0 && !si.valid) active_next = false;
        uint32_t em = si.valid ? S.shapes[si.shape].emitter : S.environment;
        if (em != MH_INVALID) {
            float em_pdf = prev_bsdf_delta ? 0.f : emitter_pdf_direction(S, em, si, prev_p);
            float mis = mis_weight(prev_bsdf_pdf, em_pdf);
            V3 le = v3(0, 0, 0);
            if (active_next)
                le = emitter_eval(S, em, si);
            dL = dL + ((beta * mis) * le) * (T * kInvPi);
        }
        active_next = active_next && (depth + 1 < in.max_depth) && si.valid;
        bool active_em = active_next && smooth;
        float e0 = rng.next_float(), e1 = rng.next_float();
        DirS ds;
        ds.pdf = 0.f;
        ds.d = v3(0, 0, 0);
        ds.delta = false;
        V3 em_weight = v3(0, 0, 0);
        if (active_em) {
            em_weight = sample_emitter_direction(S, B, si, e0, e1, ds, n_shadow);
            active_em = ds.pdf != 0.f;
        }
        V3 rho = v3(0, 0, 0);
        if (smooth) rho = tex_eval(S, S.bsdf_tex[b], si.uvx, si.uvy);
        V3 wo_em = to_local(si, ds.d);
        V3 bsdf_value_em;
        float bsdf_pdf_em;
        diffuse_eval_pdf(rho, si.wi, wo_em, active_em, bsdf_value_em, bsdf_pdf_em);
        float mis_em = ds.delta ? 1.f : mis_weight(ds.pdf, bsdf_pdf_em);
        V3 beta_mis_em = beta * mis_em;
        if (active_em) dL = dL + ((beta_mis_em * bsdf_value_em) * em_weight) * (T * kInvPi);
        (void)rng.next_float();
        float s2x = rng.next_float(), s2y = rng.next_float();
        V3 bs_wo = v3(0, 0, 0), bsdf_weight = v3(0, 0, 0);
        float bs_pdf = 0.f, bs_eta = 0.f;
        if (smooth && active_next) {
            bs_wo = square_to_cosine_hemisphere(s2x, s2y);
            bs_pdf = kInvPi * bs_wo.z;
            bs_eta = 1.f;
            bsdf_weight = (si.wi.z > 0.f && bs_pdf > 0.f) ? rho : v3(0, 0, 0);
        }
        ray = spawn_ray(si.p, si.n, to_world(si, bs_wo));
        eta *= bs_eta;
        beta = beta * bsdf_weight;
        prev_p = si.p;
        prev_bsdf_pdf = bs_pdf;
        prev_bsdf_delta = false;
        float beta_max = hmax(beta);
        active_next = active_next && beta_max != 0.f;
        float rr_prob = fminf(beta_max * (eta * eta), 0.95f);
        bool rr_active = depth >= in.rr_depth;
        if (rr_active) beta = beta * rcp(rr_prob);
        bool rr_continue = rng.next_float() < rr_prob;
        active_next = active_next && (!rr_active || rr_continue);
        if (smooth && g.slot_of_tex[S.bsdf_tex[b]] >= 0) {
            const V3 t = tex_tangent(S, S.bsdf_tex[b], si.uvx, si.uvy, g);
            if (active_em && si.wi.z > 0.f && wo_em.z > 0.f)
                dL = dL + (((em_weight * beta_mis_em) * wo_em.z) * kInvPi) * t;
            T = T + prb_indirect_factor(active_next, si, to_local(si, ray.d), bsdf_weight, bs_pdf) * t;
        }
        if (si.valid) depth += 1;
        active = active_next;
    }
    if (valid_out) *valid_out = depth != 0;
    return dL;
}

// ===========================================================================
// volpath (integrators/volpath.cpp:95-450) and its plugins: constant /
// directional emitters, heterogeneous / homogeneous media, grid volume,
// HG / isotropic phase.  Same operation order as the oracle restatement
// (oracle/mh_oracle.c, "volpath" section).
// ===========================================================================
// ---- media -----------------------------------------------------------------
struct MEI {
    bool valid;
    float t, mint;
    V3 p, sigma_s;
    float sigma_n, sigma_t, maj;
    V3 fs, ft, fn;   // Frame3f(ray.d); wi = (0, 0, -1) local
};

// Device layout of a density grid (the host API and gradients keep the
// reference's linear (z, y, x) layout; values are unchanged, so lookups are
// bit-exact either way).
//
// 4 x 4 x 4 bricks of 64 floats (256 B), bricks x-fastest, texels x-fastest
// inside a brick.  (Round 5 measured apron tiles -- every lookup in one
// 128-B line at 3.6x the texels -- as neutral: DESIGN.md section 9.)
__host__ __device__ __forceinline__ uint64_t grid_index(int32_t x, int32_t y, int32_t z, int32_t rx, int32_t ry) {
    const uint32_t nbx = (uint32_t)(rx + 3) >> 2, nby = (uint32_t)(ry + 3) >> 2;
    const uint64_t brick = ((uint64_t)((uint32_t)z >> 2) * nby + ((uint32_t)y >> 2)) * nbx + ((uint32_t)x >> 2);
    return brick * 64u + ((((uint32_t)z & 3u) << 4) | (((uint32_t)y & 3u) << 2) | ((uint32_t)x & 3u));
}
// [drjit] Texture3f::eval_nonaccel, linear, clamp, 1 channel (grid.cpp:545-558),
// in three parts: the tap offsets and weights, the 8 loads, the interpolation
struct GridLookup {
    float w0x, w0y, w0z, w1x, w1y, w1z;
    uint32_t o[8];  // tap (bx, by, bz) at o[bx | by << 1 | bz << 2] in the bricked grid
};
MH_DEV void grid_setup(const DMedium &m, V3 p, GridLookup &L) {
    V3 q = xf_point(m.to_local, p);
    const int32_t rx = (int32_t)m.res[0], ry = (int32_t)m.res[1], rz = (int32_t)m.res[2];
    float px = __builtin_fmaf(q.x, (float)rx, -0.5f), py = __builtin_fmaf(q.y, (float)ry, -0.5f),
          pz = __builtin_fmaf(q.z, (float)rz, -0.5f);
    int32_t ix = (int32_t)floorf(px), iy = (int32_t)floorf(py), iz = (int32_t)floorf(pz);
    L.w1x = px - (float)ix; L.w1y = py - (float)iy; L.w1z = pz - (float)iz;
    L.w0x = 1.f - L.w1x; L.w0y = 1.f - L.w1y; L.w0z = 1.f - L.w1z;
    const int32_t x0 = min(max(ix, 0), rx - 1), x1 = min(max(ix + 1, 0), rx - 1);
    const int32_t y0 = min(max(iy, 0), ry - 1), y1 = min(max(iy + 1, 0), ry - 1);
    const int32_t z0 = min(max(iz, 0), rz - 1), z1 = min(max(iz + 1, 0), rz - 1);
    // grid_index split per axis (brick-major part + texel-in-brick part, the
    // bit fields disjoint), 32-bit (mh_scene_create caps a grid at 2^32 texels)
    const uint32_t nbx = (uint32_t)(rx + 3) >> 2, nby = (uint32_t)(ry + 3) >> 2, sy = nbx * 64u, sz = sy * nby;
    const uint32_t ox0 = ((uint32_t)x0 >> 2) * 64u + ((uint32_t)x0 & 3u), ox1 = ((uint32_t)x1 >> 2) * 64u + ((uint32_t)x1 & 3u);
    const uint32_t oy0 = ((uint32_t)y0 >> 2) * sy + (((uint32_t)y0 & 3u) << 2), oy1 = ((uint32_t)y1 >> 2) * sy + (((uint32_t)y1 & 3u) << 2);
    const uint32_t oz0 = ((uint32_t)z0 >> 2) * sz + (((uint32_t)z0 & 3u) << 4), oz1 = ((uint32_t)z1 >> 2) * sz + (((uint32_t)z1 & 3u) << 4);
    const uint32_t o00 = oy0 + oz0, o10 = oy1 + oz0, o01 = oy0 + oz1, o11 = oy1 + oz1;
    L.o[0] = o00 + ox0; L.o[1] = o00 + ox1; L.o[2] = o10 + ox0; L.o[3] = o10 + ox1;
    L.o[4] = o01 + ox0; L.o[5] = o01 + ox1; L.o[6] = o11 + ox0; L.o[7] = o11 + ox1;
}
MH_DEV float grid_interp(const GridLookup &L, const float (&v)[8]) {
    float f00 = __builtin_fmaf(L.w0x, v[0], L.w1x * v[1]), f01 = __builtin_fmaf(L.w0x, v[4], L.w1x * v[5]),
          f10 = __builtin_fmaf(L.w0x, v[2], L.w1x * v[3]), f11 = __builtin_fmaf(L.w0x, v[6], L.w1x * v[7]);
    float f0 = __builtin_fmaf(L.w0y, f00, L.w1y * f10), f1 = __builtin_fmaf(L.w0y, f01, L.w1y * f11);
    return __builtin_fmaf(L.w0z, f0, L.w1z * f1);
}
MH_DEV float grid_eval(const DScene &S, const DMedium &m, V3 p) {
    GridLookup L;
    grid_setup(m, p, L);
    const float *g = S.grid + m.grid_offset;
    float v[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) v[c] = g[L.o[c]];
    return grid_interp(L, v);
}

// BoundingBox3f::ray_intersect (core/bbox.h:303-327)
MH_DEV bool bbox_ray_intersect(const float *mn, const float *mx, const RayT &r, float &mint, float &maxt) {
    const float o[3] = {r.o.x, r.o.y, r.o.z}, d[3] = {r.d.x, r.d.y, r.d.z};
    bool active = true;
    float t1p[3], t2p[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        active = active && (d[i] != 0.f || (o[i] > mn[i] || o[i] < mx[i]));
        const float rc = rcp(d[i]);
        const float t1 = (mn[i] - o[i]) * rc, t2 = (mx[i] - o[i]) * rc;
        t1p[i] = fminf(t1, t2);
        t2p[i] = fmaxf(t1, t2);
    }
    mint = fmaxf(fmaxf(t1p[0], t1p[1]), t1p[2]);
    maxt = fminf(fminf(t2p[0], t2p[1]), t2p[2]);
    return active && maxt >= mint;
}

// Medium::sample_interaction (medium.cpp:40-86).  Frame = false leaves the
// interaction frame (fs, ft) to the caller (mei_frame), for callers that
// need it only at a real scatter.
// the free-flight part of Medium::sample_interaction: the sampled distance
// and position, and whether it lies inside the medium's segment (valid)
MH_DEV bool free_flight(const DMedium &m, const RayT &ray, float u, float &mint_o, float &t_o, V3 &p_o) {
    float mint, maxt;
    bool active;
    if (m.type == MH_MEDIUM_HOMOGENEOUS) {
        active = true; mint = 0.f; maxt = __builtin_huge_valf();   // homogeneous.cpp:184-187
    } else {
        active = bbox_ray_intersect(m.bbox_min, m.bbox_max, ray, mint, maxt);
    }
    active = active && (isfinite_(mint) || isfinite_(maxt));
    if (!active) { mint = 0.f; maxt = __builtin_huge_valf(); }
    mint = fmaxf(0.f, mint);
    maxt = fminf(ray.maxt, maxt);
    const float sampled_t = mint + (-log_dr(1.f - u) / m.maj);
    mint_o = mint;
    t_o = sampled_t;
    p_o = fma3s(ray.d, sampled_t, ray.o);
    return active && sampled_t <= maxt;
}
// returns whether the sample looked the density grid up (k_vol_sched counts them)
template <bool Frame = true>
MH_DEV bool sample_interaction(const DScene &S, uint32_t med, const RayT &ray, float u, MEI &mei) {
    const DMedium &m = S.media[med];
    mei.fn = ray.d;
    if (Frame) coordinate_system(ray.d, mei.fs, mei.ft);
    float mint, sampled_t;
    V3 p;
    const bool valid = free_flight(m, ray, u, mint, sampled_t, p);
    const float maj = m.maj;
    mei.valid = valid;
    mei.t = valid ? sampled_t : __builtin_huge_valf();
    mei.p = p;
    mei.mint = mint;
    mei.maj = maj;
    float st = 0.f;
    if (valid) st = m.type == MH_MEDIUM_HOMOGENEOUS ? m.sigma_t_const * m.scale : m.scale * grid_eval(S, m, mei.p);
    mei.sigma_t = st;
    mei.sigma_s = valid ? v3(m.albedo[0], m.albedo[1], m.albedo[2]) * st : v3(0, 0, 0);
    mei.sigma_n = m.type == MH_MEDIUM_HOMOGENEOUS ? 0.f : maj - st;
    return valid && m.type != MH_MEDIUM_HOMOGENEOUS;
}
MH_DEV V3 mei_to_local(const MEI &m, V3 v) { return v3(dot(v, m.fs), dot(v, m.ft), dot(v, m.fn)); }
MH_DEV void mei_frame(MEI &m) { coordinate_system(m.fn, m.fs, m.ft); }  // Frame3f(ray.d), as sample_interaction
MH_DEV V3 mei_to_world(const MEI &m, V3 v) { return fma3s(m.fn, v.z, fma3s(m.ft, v.y, m.fs * v.x)); }

// HGPhaseFunction (phase/hg.cpp:66-104), IsotropicPhaseFunction
MH_DEV float eval_hg(float g, float cos_theta) {
    float temp = (1.f + g * g) + (2.f * g) * cos_theta;
    return (kInv4Pi * (1.f - g * g)) / (temp * __builtin_sqrtf(temp));
}
MH_DEV float phase_eval(const DMedium &m, V3 wo) {
    if (m.phase == MH_PHASE_HG) return eval_hg(m.g, dot(wo, v3(0.f, 0.f, -1.f)));
    return kInv4Pi;
}
MH_DEV V3 phase_sample(const DMedium &m, float s2x, float s2y, float &pdf) {
    if (m.phase == MH_PHASE_HG) {
        const float g = m.g;
        float sqr_term = (1.f - g * g) / ((1.f - g) + (2.f * g) * s2x);
        float cos_theta = ((1.f + g * g) - sqr_term * sqr_term) / (2.f * g);
        if (__builtin_fabsf(g) < 5.9604644775390625e-08f) cos_theta = 1.f - 2.f * s2x;
        float sin_theta = __builtin_sqrtf(fmaxf(1.f - cos_theta * cos_theta, 0.f));
        float sp, cp;
        sincos_cephes((2.f * kPi) * s2y, sp, cp);
        pdf = eval_hg(g, -cos_theta);
        return v3(sin_theta * cp, sin_theta * sp, cos_theta);
    }
    pdf = kInv4Pi;
    return square_to_uniform_sphere(s2x, s2y);
}

MH_DEV bool is_medium_transition(const DScene &S, const SI &si) {
    if (!si.valid) return false;
    const DShape &sh = S.shapes[si.shape];
    return sh.interior != sh.exterior;
}
MH_DEV uint32_t target_medium(const DScene &S, const SI &si, V3 d) {
    const DShape &sh = S.shapes[si.shape];
    return dot(d, si.n) > 0.f ? sh.exterior : sh.interior;
}

// Pk: the wave-coherent packet engine (small scenes with pair records; the
// lanes that reach this call trace together, control stays scalar) instead
// of the per-lane traversal; same hits (closest, exact-t ties to the lower key)
// the surface interaction of a closest hit and its distance
MH_DEV void si_from_hit(const DScene &S, const RayT &ray, const Hit &h, SI &si, float &si_t) {
    compute_si(S, ray, h, si);
    si_t = si.valid ? h.t : __builtin_huge_valf();
}
template <bool Pk = false>
MH_DEV void trace_si(const DScene &S, const LdsBvh &B, const RayT &ray, SI &si, float &si_t) {
    Hit h;
    if (Pk) h = packet_batch<false>(S.nodes, S.prims, S.prim_pairs, S.key_sp, B.stack - (threadIdx.x & 63u), B.stride,
                                    ray, true);
    else traverse<false>(B.nodes, B.prims, B.stack, B.stride, ray, h);
    si_from_hit(S, ray, h, si, si_t);
}

// volpath.cpp:333-450: emitter sample + ratio-tracked transmittance, split
// into nee_begin (the emitter sample and the shadow ray) and nee_step (one
// trip of the transmittance loop) so the walk can interleave with the other
// lanes' path steps (volpath_advance).  Same operations in the same order as
// a single call (oracle: vol_sample_emitter).
struct NeeState {
    RayT ray;
    SI si;
    V3 transmittance, emitter_val;
    float max_dist, total_dist, si_t;
    uint32_t medium;
    bool needs_intersection;
};

// returns false when there is nothing to walk (ds.pdf == 0: emitted = 0)
MH_DEV bool nee_begin(const DScene &S, V3 ref_p, V3 ref_n, const SI *si_ref, Pcg &rng, uint32_t medium, DirS &ds,
                      NeeState &ns) {
    ns.transmittance = v3(1, 1, 1);
    const float sx = rng.next_float(), sy = rng.next_float();
    ns.emitter_val = scene_sample_emitter_direction(S, ref_p, sx, sy, ds);
    if (ds.pdf == 0.f) return false;
    ns.ray = spawn_ray_to(ref_p, ref_n, ds.p);
    ns.max_dist = ns.ray.maxt;
    if (si_ref && is_medium_transition(S, *si_ref)) medium = target_medium(S, *si_ref, ns.ray.d);
    ns.medium = medium;
    ns.total_dist = 0.f;
    ns.si.valid = false;
    ns.si_t = 0.f;
    ns.needs_intersection = true;
    return true;
}

MH_DEV V3 nee_result(const NeeState &ns) { return ns.transmittance * ns.emitter_val; }

// one trip of the transmittance loop; false when the loop has ended
template <bool Pk = false>
MH_DEV bool nee_step(const DScene &S, const LdsBvh &B, Pcg &rng, const DirS &ds, NeeState &ns, uint32_t &n_shadow) {
    RayT &ray = ns.ray;
    SI &si = ns.si;
    float &si_t = ns.si_t, &total_dist = ns.total_dist;
    V3 &transmittance = ns.transmittance;
    uint32_t &medium = ns.medium;
    bool &needs_intersection = ns.needs_intersection;
    const float remaining_dist = ns.max_dist - total_dist;
    ray.maxt = remaining_dist;
    if (!(remaining_dist > 0.f)) return false;
    bool escaped_medium = false;
    bool active_medium = medium != MH_INVALID;
    bool active_surface = !active_medium;
    if (active_medium) {
        const DMedium &m = S.media[medium];
        MEI mei;
        sample_interaction(S, medium, ray, rng.next_float(), mei);
        if (m.type == MH_MEDIUM_HOMOGENEOUS && mei.valid) ray.maxt = fminf(mei.t, remaining_dist);
        if (needs_intersection) { trace_si<Pk>(S, B, ray, si, si_t); ++n_shadow; }
        if (si_t < mei.t) { mei.t = __builtin_huge_valf(); mei.valid = false; }
        needs_intersection = needs_intersection && !si.valid;
        const bool spectral = !(m.flags & MH_MEDIUM_NO_SPECTRAL_EXTINCTION);
        if (spectral) {
            const float t = fminf(remaining_dist, fminf(mei.t, si_t)) - mei.mint;
            const float tr = exp_dr((-t) * mei.maj);
            const float pdf = (si_t < mei.t || mei.t > remaining_dist) ? tr : tr * mei.maj;
            transmittance = transmittance * (pdf > 0.f ? tr / pdf : 0.f);
        }
        if (mei.t > remaining_dist && mei.valid) total_dist = ds.dist;
        if (mei.t > remaining_dist) { mei.t = __builtin_huge_valf(); mei.valid = false; }
        escaped_medium = !mei.valid;
        active_medium = mei.valid;
        if (active_medium) {
            total_dist += mei.t;
            ray.o = mei.p;
            si_t = si_t - mei.t;
            transmittance = transmittance * (spectral ? mei.sigma_n : mei.sigma_n / mei.maj);
        }
    }
    const bool intersect = active_surface && needs_intersection;
    if (intersect) { trace_si<Pk>(S, B, ray, si, si_t); ++n_shadow; }
    needs_intersection = needs_intersection && !intersect;
    active_surface = active_surface || escaped_medium;
    if (active_surface) total_dist += si_t;
    active_surface = active_surface && si.valid && !active_medium;
    if (active_surface) {
        const uint32_t b = S.shapes[si.shape].bsdf;
        const float tn = (b != MH_INVALID && S.bsdf_type[b] == MH_BSDF_NULL) ? 1.f : 0.f;
        transmittance = transmittance * tn;
        ray = spawn_ray(si.p, si.n, ray.d);
    }
    ray.maxt = remaining_dist;
    needs_intersection = needs_intersection || active_surface;
    const bool active = (active_medium || active_surface) && nonzero(transmittance);
    if (active_surface && is_medium_transition(S, si)) medium = target_medium(S, si, ray.d);
    return active;
}

// The volpath loop (volpath.cpp:95-450) as a resumable state machine.  One
// trip of `while (loop(active))` is pre -> [NEE walk] -> post:
//   pre   Russian roulette, the medium interaction and, for surface paths,
//         the hit and its emission, up to the emitter sample;
//   NEE   the ratio-tracked shadow walk, one trip per advance;
//   post  the contribution of the emitter sample, phase / BSDF sampling.
// volpath_advance moves a lane by one unit, so in a wave the lanes that walk a
// long shadow ray and the lanes that continue their paths advance together
// instead of the latter idling through the former's loop.
// Per lane the operations and random draws are exactly those of the nested
// loops (oracle: volpath_sample).
enum : uint32_t { kVolPre = 0, kVolNee = 1, kVolPost = 2 };
enum : uint32_t { kNeeNone = 0, kNeeMedium = 1, kNeeSurface = 2 };

struct VolState {
    RayT ray;
    V3 throughput, result, last_p;
    SI si;
    float si_t, last_pdf, eta;
    uint32_t medium, depth;
    bool specular_chain, needs_intersection, valid;
    // between pre and post
    uint32_t mode, nee_kind;
    bool active, active_medium, active_surface, act_scatter;
    MEI mei;
    V3 rho, pend;       // surface albedo; pending contribution factor
    float pend_w;       // medium: MIS weight applied after the emitted radiance
    DirS ds;
    NeeState ns;
};

MH_DEV void volpath_init(const DScene &S, const IntegratorParams &in, Pcg &rng, RayT ray, VolState &v) {
    v.ray = ray;
    v.eta = 1.f;
    v.throughput = v3(1, 1, 1);
    v.result = v3(0, 0, 0);
    v.medium = S.camera_medium;
    v.specular_chain = !in.hide_emitters;
    v.valid = !in.hide_emitters && S.environment != MH_INVALID;  // valid_ray (volpath.cpp:105)
    v.depth = 0;
    (void)fminf(rng.next_float() * 3.f, 2.f);  // RGB channel (scalar majorants: all channels alike)
    v.si.valid = false;
    v.si_t = 0.f;
    v.needs_intersection = true;
    v.last_p = v3(0, 0, 0);
    v.last_pdf = 1.f;
    v.mode = kVolPre;
}

// pre: false when the path ends at the loop head
template <bool Pk = false>
MH_DEV bool volpath_pre(const DScene &S, const LdsBvh &B, const IntegratorParams &in, Pcg &rng, VolState &v,
                        uint32_t &n_closest) {
    RayT &ray = v.ray;
    V3 &throughput = v.throughput, &result = v.result, &last_p = v.last_p;
    SI &si = v.si;
    float &si_t = v.si_t, &last_pdf = v.last_pdf, &eta = v.eta;
    uint32_t &medium = v.medium, &depth = v.depth;
    bool &specular_chain = v.specular_chain, &needs_intersection = v.needs_intersection;
    MEI &mei = v.mei;
    // ---- Russian roulette (volpath.cpp:143-151)
    bool active = nonzero(throughput);
    const float q = fminf(hmax(throughput) * (eta * eta), 0.95f);
    const bool perform_rr = depth > in.rr_depth;
    if (active) active = rng.next_float() < q || !perform_rr;
    if (perform_rr) throughput = throughput * rcp(q);
    active = active && depth < in.max_depth;
    if (!active) return false;

    bool active_medium = medium != MH_INVALID, active_surface = !active_medium;
    bool act_null = false, act_scatter = false, escaped = false, spectral = false;
    mei.valid = false;
    mei.t = __builtin_huge_valf();
    if (active_medium) {
        const DMedium &m = S.media[medium];
        sample_interaction(S, medium, ray, rng.next_float(), mei);
        if (m.type == MH_MEDIUM_HOMOGENEOUS && mei.valid) ray.maxt = mei.t;
        if (needs_intersection) { trace_si<Pk>(S, B, ray, si, si_t); ++n_closest; }
        needs_intersection = needs_intersection && !si.valid;
        if (si_t < mei.t) { mei.t = __builtin_huge_valf(); mei.valid = false; }
        spectral = !(m.flags & MH_MEDIUM_NO_SPECTRAL_EXTINCTION);
        if (spectral) {
            const float t = fminf(mei.t, si_t) - mei.mint;
            const float tr = exp_dr((-t) * mei.maj);
            const float pdf = si_t < mei.t ? tr : tr * mei.maj;
            throughput = throughput * (pdf > 0.f ? tr / pdf : 0.f);
        }
        escaped = !mei.valid;
        active_medium = mei.valid;
        bool null_scatter = false;
        if (active_medium) null_scatter = rng.next_float() >= mei.sigma_t / mei.maj;
        act_null = null_scatter && active_medium;
        act_scatter = !act_null && active_medium;
        if (spectral && act_null) throughput = throughput * ((mei.sigma_n * mei.maj) / mei.sigma_n);
        if (act_scatter) { depth += 1; last_p = mei.p; }
    }
    active = active && depth < in.max_depth;
    act_scatter = act_scatter && active;
    if (act_null) { ray.o = mei.p; si_t = si_t - mei.t; }
    v.nee_kind = kNeeNone;
    bool walk = false;
    if (act_scatter) {
        const DMedium &m = S.media[medium];
        if (spectral) throughput = throughput * vdiv(mei.sigma_s * mei.maj, mei.sigma_t);
        else throughput = throughput * vdiv(mei.sigma_s, mei.sigma_t);
        const bool sample_emitters = !(m.flags & MH_MEDIUM_NO_EMITTER_SAMPLING);
        specular_chain = !sample_emitters;
        v.valid = true;  // valid_ray |= act_medium_scatter (volpath.cpp:223)
        if (sample_emitters) {
            walk = nee_begin(S, mei.p, v3(0, 0, 0), nullptr, rng, medium, v.ds, v.ns);
            const float ph = phase_eval(m, mei_to_local(mei, v.ds.d));
            v.pend = throughput * ph;
            v.pend_w = mis_weight(v.ds.pdf, v.ds.delta ? 0.f : ph);
            v.nee_kind = kNeeMedium;
        }
    }
    // ---- surface interactions (volpath.cpp:254-326), up to the emitter sample
    // (act_scatter paths are not surface paths: only escaped ones join)
    active_surface = active_surface || escaped;
    if (active_surface && needs_intersection) { trace_si<Pk>(S, B, ray, si, si_t); ++n_closest; }
    if (active_surface) {
        const bool count_direct = depth == 0 || specular_chain;
        const uint32_t em = si.valid ? S.shapes[si.shape].emitter : S.environment;
        if (em != MH_INVALID && !(depth == 0 && in.hide_emitters)) {
            float emitter_pdf = 1.f;
            if (!count_direct) emitter_pdf = emitter_pdf_direction(S, em, si, last_p);
            const V3 emitted = emitter_eval(S, em, si);
            result = result + (count_direct ? throughput * emitted
                                            : (throughput * mis_weight(last_pdf, emitter_pdf)) * emitted);
        }
    }
    active_surface = active_surface && si.valid;
    v.rho = v3(0, 0, 0);
    if (active_surface) {
        const uint32_t b = S.shapes[si.shape].bsdf;
        const bool is_null = b == MH_INVALID || S.bsdf_type[b] == MH_BSDF_NULL;
        if (!is_null) v.rho = tex_eval(S, S.bsdf_tex[b], si.uvx, si.uvy);
        if (!is_null && depth + 1 < in.max_depth) {
            walk = nee_begin(S, si.p, si.n, &si, rng, medium, v.ds, v.ns);
            V3 bv;
            float bp;
            diffuse_eval_pdf(v.rho, si.wi, to_local(si, v.ds.d), true, bv, bp);
            const float w = mis_weight(v.ds.pdf, v.ds.delta ? 0.f : bp);
            v.pend = (throughput * bv) * w;
            v.nee_kind = kNeeSurface;
        }
    }
    v.active = active;
    v.active_medium = active_medium;
    v.active_surface = active_surface;
    v.act_scatter = act_scatter;
    if (v.nee_kind != kNeeNone && !walk) {   // ds.pdf == 0: emitted = 0
        v.ns.transmittance = v3(0, 0, 0);
        v.ns.emitter_val = v3(0, 0, 0);
    }
    v.mode = walk ? kVolNee : kVolPost;
    return true;
}

// post: the emitter sample's contribution, then phase / BSDF sampling; false
// when the path has ended
MH_DEV bool volpath_post(const DScene &S, const IntegratorParams &in, Pcg &rng, VolState &v) {
    V3 &throughput = v.throughput, &result = v.result;
    if (v.nee_kind == kNeeMedium) result = result + (v.pend * nee_result(v.ns)) * v.pend_w;
    else if (v.nee_kind == kNeeSurface) result = result + v.pend * nee_result(v.ns);
    bool act_scatter = v.act_scatter;
    const MEI &mei = v.mei;
    if (act_scatter) {
        const DMedium &m = S.media[v.medium];
        (void)rng.next_float();
        const float s2x = rng.next_float(), s2y = rng.next_float();
        float ph_pdf;
        V3 wo = phase_sample(m, s2x, s2y, ph_pdf);
        act_scatter = act_scatter && ph_pdf > 0.f;
        if (act_scatter) {
            v.ray = spawn_ray(mei.p, v3(0, 0, 0), mei_to_world(mei, wo));
            v.needs_intersection = true;
            v.last_pdf = ph_pdf;
        }
    }
    if (v.active_surface) {
        const SI &si = v.si;
        const uint32_t b = S.shapes[si.shape].bsdf;
        const bool is_null = b == MH_INVALID || S.bsdf_type[b] == MH_BSDF_NULL;
        (void)rng.next_float();
        const float s2x = rng.next_float(), s2y = rng.next_float();
        V3 bs_wo, weight;
        float bs_pdf;
        if (is_null) {
            bs_wo = -si.wi; bs_pdf = 1.f; weight = v3(1, 1, 1);
        } else {
            bs_wo = square_to_cosine_hemisphere(s2x, s2y);
            bs_pdf = kInvPi * bs_wo.z;
            weight = (si.wi.z > 0.f && bs_pdf > 0.f) ? v.rho : v3(0, 0, 0);
        }
        throughput = throughput * weight;
        v.ray = spawn_ray(si.p, si.n, to_world(si, bs_wo));
        v.needs_intersection = true;
        if (!is_null) {
            v.depth += 1;
            v.last_p = si.p;
            v.last_pdf = bs_pdf;
            v.specular_chain = false;
            v.valid = true;  // valid_ray |= non_null_bsdf (volpath.cpp:320)
        }
        if (is_medium_transition(S, si)) v.medium = target_medium(S, si, v.ray.d);
    }
    v.mode = kVolPre;
    return v.active && (v.active_surface || v.active_medium);
}

// one unit of progress; false when the path has ended (v.result is final).
// Scheduling (wave vote): lanes in a shadow walk take one step every trip;
// the others run their main work (post of the finished walk, then pre of the
// next loop trip) only once at least MH_VOL_MAIN_PCT % of the wave's live
// lanes wait for it -- the main work is the heavy code, a walk step is
// light, so running both every trip would make the walkers pay for it.
#ifndef MH_VOL_MAIN_PCT
#define MH_VOL_MAIN_PCT 75  // measured best of 25..100 on config 4 (tools/bench_volpath.py)
#endif
template <bool Pk = false>
MH_DEV bool volpath_advance(const DScene &S, const LdsBvh &B, const IntegratorParams &in, Pcg &rng, VolState &v,
                            uint32_t &n_closest, uint32_t &n_shadow) {
    const bool walking = v.mode == kVolNee;
    const uint32_t n_all = (uint32_t)__popcll(__ballot(true)), n_main = (uint32_t)__popcll(__ballot(!walking));
    if (walking) {
        if (!nee_step<Pk>(S, B, rng, v.ds, v.ns, n_shadow)) v.mode = kVolPost;
        return true;
    }
    if (n_main * 100u < n_all * (uint32_t)MH_VOL_MAIN_PCT) return true;
    if (v.mode == kVolPost && !volpath_post(S, in, rng, v)) return false;
    if (!volpath_pre<Pk>(S, B, in, rng, v, n_closest)) return false;
    if (v.mode == kVolPost) return volpath_post(S, in, rng, v);
    return true;
}

MH_DEV V3 volpath_sample(const DScene &S, const LdsBvh &B, const IntegratorParams &in, Pcg &rng,
                         RayT ray, uint32_t &n_closest, uint32_t &n_shadow, bool *valid_out = nullptr) {
    VolState v;
    volpath_init(S, in, rng, ray, v);
    while (volpath_advance(S, B, in, rng, v, n_closest, n_shadow)) {
    }
    if (valid_out) *valid_out = v.valid;
    return v.result;
}

// ===========================================================================
// PRBVolpathIntegrator (python/ad/integrators/prbvolpath.py:91-431)
//   primal (Adj == false) or adjoint replay (Adj == true, L = primal radiance)
//   Same operation order as the oracle restatement (oracle/mh_oracle.c,
//   "PRBVolpathIntegrator" section).
// ===========================================================================
// Grid-gradient scatter into a per-cell corner block (GradArgs::corner): cell
// (ix, iy, iz) of a lookup -- ix = floor(x - 0.5) clamped to [-1, rx - 1],
// which keeps its clamped taps -- owns 8 contiguous floats, one per tap, and
// launch_corner_gather folds them into the (z, y, x) gradient afterwards.
// Float atomics execute at the memory side as one 64-B request per distinct
// segment of a wave-instruction (MI355X_MICROARCH.md, global float atomics):
// 8 atomics per lane into the linear grid put up to 64 rows in every
// instruction.  Here the active lanes stage (cell, 8 values) in wave LDS and
// issue the 8 x n adds transposed -- instruction j takes items j*n .. j*n+n-1
// of the (lane rank, tap) order, the taps of ~n/8 cells, 32 B each.
// Any exec mask (the call sites are divergent loops); kernels of <= 4 waves.
// MH_FLAG_DETERMINISTIC (GradCtx::fx_mode): a pre-pass records the largest
// |item| only; the real pass adds round(item * 2^S) as int64 (the block then
// holds long longs), exact integer sums that no add order changes.
constexpr int kCornerWaves = 4;
MH_DEV void corner_scatter(float *cb, uint32_t cell, const float (&v)[8], const GradCtx &g) {
    if (g.fx_mode == 1) {
        float mx = 0.f;
#pragma unroll
        for (int c = 0; c < 8; ++c) mx = fmaxf(mx, fabsf(v[c]));
        if (mx > 0.f) atomicMax(fx_wave_max(), __float_as_uint(mx));  // non-negative floats order as their bits
        return;
    }
    __shared__ float stage[kCornerWaves * 64 * 9];
    float *sc = stage + (threadIdx.x >> 6) * (64 * 9);
    const uint64_t m = __ballot(1);
    const uint32_t n = (uint32_t)__popcll(m);
    const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    sc[r * 9] = __uint_as_float(cell);
#pragma unroll
    for (int c = 0; c < 8; ++c) sc[r * 9 + 1 + c] = v[c];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
        const uint32_t t = j * n + r, src = t >> 3, c = t & 7u;
        const uint32_t cc = __float_as_uint(sc[src * 9]);
        if (g.fx_mode == 2) {
            const long long q = __double2ll_rn((double)sc[src * 9 + 1 + c] * g.fx_scale);
            gatomic_add(reinterpret_cast<unsigned long long *>(cb) + (size_t)cc * 8 + c, (unsigned long long)q);
        } else {
            gatomic_add(cb + (size_t)cc * 8 + c, sc[src * 9 + 1 + c]);
        }
    }
    __builtin_amdgcn_wave_barrier();
}

// adjoint of sigma_t(p) = scale * Texture3f(grid).eval(p) (heterogeneous.cpp:192)
// or scale * sigma_t (homogeneous.cpp:158); adj = d loss / d sigma_t(p)
// the scatter of one sigma_t adjoint into slot k (buffer buf, corner block
// cb or nullptr)
MH_DEV void sigma_t_backward_at(const DScene &S, uint32_t med, V3 p, float adj, GradCtx &g, int32_t k, float *buf,
                                float *cb) {
    const DMedium &m = S.media[med];
    const float as = adj * m.scale;
    if (m.type == MH_MEDIUM_HOMOGENEOUS) {
        if (g.fwd) g.fsum += as * buf[0];
        else acc_add(g, k, v3(as, 0.f, 0.f));
        return;
    }
    V3 q = xf_point(m.to_local, p);
    const int32_t rx = (int32_t)m.res[0], ry = (int32_t)m.res[1], rz = (int32_t)m.res[2];
    float px = __builtin_fmaf(q.x, (float)rx, -0.5f), py = __builtin_fmaf(q.y, (float)ry, -0.5f),
          pz = __builtin_fmaf(q.z, (float)rz, -0.5f);
    int32_t ix = (int32_t)floorf(px), iy = (int32_t)floorf(py), iz = (int32_t)floorf(pz);
    float w1x = px - (float)ix, w1y = py - (float)iy, w1z = pz - (float)iz;
    float w0x = 1.f - w1x, w0y = 1.f - w1y, w0z = 1.f - w1z;
    const int32_t xs[2] = {min(max(ix, 0), rx - 1), min(max(ix + 1, 0), rx - 1)};
    const int32_t ys[2] = {min(max(iy, 0), ry - 1), min(max(iy + 1, 0), ry - 1)};
    const int32_t zs[2] = {min(max(iz, 0), rz - 1), min(max(iz + 1, 0), rz - 1)};
    if (!g.fwd && cb) {
        float v[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const int bx = c & 1, by = (c >> 1) & 1, bz = c >> 2;
            v[c] = as * (((bz ? w1z : w0z) * (by ? w1y : w0y)) * (bx ? w1x : w0x));
        }
        const uint32_t cx = (uint32_t)(min(max(ix, -1), rx - 1) + 1), cy = (uint32_t)(min(max(iy, -1), ry - 1) + 1),
                       cz = (uint32_t)(min(max(iz, -1), rz - 1) + 1);
        corner_scatter(cb, (cz * (uint32_t)(ry + 1) + cy) * (uint32_t)(rx + 1) + cx, v, g);
        return;
    }
    const uint64_t sy = (uint64_t)rx, sz = (uint64_t)rx * (uint64_t)ry;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const int bx = c & 1, by = (c >> 1) & 1, bz = c >> 2;
        const float w = ((bz ? w1z : w0z) * (by ? w1y : w0y)) * (bx ? w1x : w0x);
        const uint64_t idx = (uint64_t)zs[bz] * sz + (uint64_t)ys[by] * sy + (uint64_t)xs[bx];
        if (g.fwd) {  // tangent of the grid at p: the same taps over the tangent voxels
            g.fsum += (as * w) * buf[idx];
            continue;
        }
        gatomic_add(buf + idx, as * w);
    }
}
// The hot medium (GradArgs::hot_*) takes its slot, buffer and corner block
// from registers, in a branch of its own: a vector load of a slot table entry
// waits (vmcnt, issue order) for every atomic the wave issued before it, so a
// load whose value merged into the scatter made each scatter wait for the
// previous one's atomics to complete.
MH_DEV void sigma_t_backward(const DScene &S, uint32_t med, V3 p, float adj, GradCtx &g) {
    if (!g.sigma_slot) return;
    if ((int32_t)med == g.hot_med) {
        if (g.hot_sigma >= 0) sigma_t_backward_at(S, med, p, adj, g, g.hot_sigma, g.hot_buf, g.hot_corner);
        return;
    }
    const int32_t k = g.sigma_slot[med];
    if (k < 0) return;
    sigma_t_backward_at(S, med, p, adj, g, k, g.bufs[k], g.corner ? g.corner[k] : nullptr);
}

MH_DEV void albedo_backward(uint32_t med, V3 adj, GradCtx &g) {
    if (!g.albedo_slot) return;
    const int32_t k = (int32_t)med == g.hot_med ? g.hot_albedo : g.albedo_slot[med];
    if (k < 0) return;
    if (g.fwd) g.fsum += (adj.x * g.bufs[k][0] + adj.y * g.bufs[k][1]) + adj.z * g.bufs[k][2];
    else acc_add(g, k, adj);
}

// Per-thread log of the gradient steps of one NEE walk (the adjoint pass of
// k_prbvol_backward).  The reference replays the walk with the cloned sampler
// to back-propagate dL * adj_emitted through every tr_multiplier
// (prbvolpath.py:412-414), because adj_emitted (the NEE contribution) is
// known only once the walk has ended.  The transmittance multipliers of a
// grey medium are grey, so a step's gradient is coef * (dL . adj_emitted),
// coef = -1 / (majorant * tr) for a null collision, -hom_t for a homogeneous
// segment: the walk logs (p, coef) and the caller scatters them once
// adj_emitted is known -- one walk instead of two.  Steps beyond `cap`, or in
// a second medium, fall back to the replay.
struct NeeLog {
    float4 *buf;         // [cap][stride]: (p, coef)
    uint32_t stride;     // threads of the launch
    uint32_t cap;        // entries per thread
    uint32_t t;          // this thread
    uint32_t n;          // entries of the current walk
    uint32_t med;        // their medium
    bool overflow;
};

// PRBVolpathIntegrator.sample_emitter (prbvolpath.py:336-431): emitter sample
// + ratio-tracked transmittance; Mode 1 (adjoint): replay with the cloned
// sampler and back-propagate dL * adj_emitted through every tr_multiplier
// (:412-414); Mode 2: the primal walk, logging the gradient steps (NeeLog)
template <int Mode>
MH_DEV V3 pvp_sample_emitter(const DScene &S, const LdsBvh &B, const MEI &mei_ref, const SI &si_ref,
                             bool active_medium, Pcg &rng, uint32_t medium, DirS &ds, V3 adj_emitted, V3 dL,
                             GradCtx *g, uint32_t &n_shadow, NeeLog *nl = nullptr) {
    constexpr bool Adj = Mode == 1;
    if (Mode == 2) { nl->n = 0; nl->overflow = false; }
    const V3 ref_p = active_medium ? mei_ref.p : si_ref.p;
    const V3 ref_n = active_medium ? v3(0.f, 0.f, 0.f) : si_ref.n;
    const float sx = rng.next_float(), sy = rng.next_float();
    const V3 emitter_val = scene_sample_emitter_direction(S, ref_p, sx, sy, ds);
    if (ds.pdf == 0.f) return v3(0.f, 0.f, 0.f);
    if (!active_medium && is_medium_transition(S, si_ref)) medium = target_medium(S, si_ref, ds.d);
    RayT ray = spawn_ray(ref_p, ref_n, ds.d);
    const float k_dist = 1.f - kShadowEps;   // (1.0 - ShadowEpsilon), exact in float
    const bool nee_hom = S.vol_flags & kVolNeeHomogeneous;
    float total_dist = 0.f, si_t = 0.f;
    SI si;
    si.valid = false;
    bool needs_intersection = true, active = true;
    V3 transmittance = v3(1.f, 1.f, 1.f);
    while (active) {
        const float remaining_dist = ds.dist * k_dist - total_dist;
        ray.maxt = remaining_dist;
        if (!(remaining_dist > 0.f)) break;
        if (needs_intersection) { trace_si(S, B, ray, si, si_t); ++n_shadow; }
        needs_intersection = false;
        bool act_med = medium != MH_INVALID, act_surf = !act_med, escaped = false, hom = false;
        float hom_t = 0.f;
        MEI mei;
        mei.valid = false;
        mei.t = 0.f;
        mei.maj = 1.f;
        mei.p = v3(0.f, 0.f, 0.f);
        V3 trm = v3(1.f, 1.f, 1.f);
        if (act_med) {
            const DMedium &m = S.media[medium];
            sample_interaction(S, medium, ray, rng.next_float(), mei);
            if (si_t < mei.t) { mei.t = __builtin_huge_valf(); mei.valid = false; }
            if (nee_hom && m.type == MH_MEDIUM_HOMOGENEOUS) {
                mei.t = fminf(remaining_dist, si_t);
                hom_t = fminf(mei.t, si_t) - mei.mint;
                const float tr = exp_dr((-hom_t) * mei.maj);
                trm = v3(tr, tr, tr);
                hom = true;
                mei.t = __builtin_huge_valf();
                mei.valid = false;
            }
            escaped = !mei.valid;
            act_med = mei.valid;
            if (act_med) {
                ray.o = mei.p;
                si_t = si_t - mei.t;
                trm = trm * (mei.sigma_n / mei.maj);
            }
        }
        act_surf = (act_surf || escaped) && si.valid && !act_med;
        if (act_surf) {
            const uint32_t b = S.shapes[si.shape].bsdf;
            trm = trm * ((b != MH_INVALID && S.bsdf_type[b] == MH_BSDF_NULL) ? 1.f : 0.f);
        }
        if (Adj && (act_med || hom) && (act_med || act_surf)) {
            // backward(tr_multiplier * detach(dL * adj_emitted / tr_multiplier))
            const float tc[3] = {trm.x, trm.y, trm.z}, dc[3] = {dL.x, dL.y, dL.z},
                        ac[3] = {adj_emitted.x, adj_emitted.y, adj_emitted.z};
            float gs = 0.f;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const float up = tc[c] > 0.f ? (dc[c] * ac[c]) / tc[c] : 0.f;
                gs += act_med ? up * (-1.f / mei.maj) : up * (-hom_t * tc[c]);
            }
            sigma_t_backward(S, medium, mei.p, gs, *g);
        }
        if (Mode == 2 && (act_med || hom) && (act_med || act_surf)) {
            const float tc = trm.x;  // grey: scalar sigma_n / majorant, scalar homogeneous tr
            const float coef = !(tc > 0.f) ? 0.f : act_med ? (1.f / tc) * (-1.f / mei.maj) : -hom_t;
            if (nl->n < nl->cap && (nl->n == 0 || nl->med == medium)) {
                nl->buf[(uint64_t)nl->n * nl->stride + nl->t] = make_float4(mei.p.x, mei.p.y, mei.p.z, coef);
                nl->med = medium;
                ++nl->n;
            } else {
                nl->overflow = true;
            }
        }
        transmittance = transmittance * trm;
        if (act_surf) ray = spawn_ray(si.p, si.n, ray.d);
        needs_intersection = act_surf;
        active = (act_med || act_surf) && nonzero(transmittance);
        if (active) total_dist += act_med ? mei.t : si_t;
        if (act_surf && is_medium_transition(S, si)) medium = target_medium(S, si, ray.d);
    }
    return emitter_val * transmittance;
}

// Per-thread log of the L-dependent adjoint terms of one path (single-pass
// prbvolpath backward, Mode 2).  The adjoint replay back-propagates
// dL * weight * (L / weight) at every medium interaction (prbvolpath.py:
// 202-204) and dL * bsdf_eval * (L / bsdf_eval) at every surface vertex
// (:305-312), with L the radiance still to come: L_total minus the
// contributions P collected before that point.  The primal pass logs, per
// such vertex, P and the factors that do not depend on L; once the path ends
// (L_total known) pvp_log_apply charges them.  NEE terms do not depend on L
// and are charged in the pass itself.  One traversal instead of primal +
// adjoint; a path with more than `cap` vertices replays (Mode 3).
// Entry: 4 float4 at ((4 j + q) * stride + t):
//   q0 (p, bits: 1 surface | 2 scatter | index << 2)   q1 (P, uv.x)
//   q2 (dL / max(1e-8, w), uv.y)                       q3 (dws, dwa) or (cos, 0, 0, 0)
struct MainLog {
    float4 *buf;
    uint32_t stride, cap, t, n;
    bool overflow;
    MH_DEV void add(float4 a, float4 b, float4 c, float4 d) {
        if (n >= cap) { overflow = true; return; }
        const uint64_t o = (uint64_t)4 * n * stride + t;
        buf[o] = a;
        buf[o + stride] = b;
        buf[o + 2 * (uint64_t)stride] = c;
        buf[o + 3 * (uint64_t)stride] = d;
        ++n;
    }
};

// Logs are read back in batches before their atomics are issued: on gfx950
// stores and atomics retire through the same in-order vmcnt as loads, so a
// load issued after a gradient scatter waits for the scatter's atomics (~3k
// cycles with every CU issuing); one load per entry then paid that wait
// once per entry, a batch pays it once.
constexpr uint32_t kLogBatchMain = 2, kLogBatchWalk = 8;

// the logged gradient steps of one NEE walk (NeeLog entries (p, coef) at
// e[j * stride]): sigma_t's adjoint coef * K at every step, K = dL . adj_emitted
// Load-balanced wave loop over per-lane item counts (every lane of the wave
// active): lane l owns cnt_l items, the wave takes 64 of them per step, and
// f(owner, e, valid) runs on every lane with its item's owner lane and index
// (valid false past the last item; f shuffles owner data first, then works
// under `valid`).  The divergent per-lane loop it replaces ran max(cnt) steps
// with the lanes that still had items.  scr: 64 words of the wave's LDS.
MH_DEV uint32_t *flat_scratch() {
    __shared__ uint32_t scr[kCornerWaves * 64];
    return scr + (threadIdx.x >> 6) * 64u;
}
template <class F>
MH_DEV void wave_flat(uint32_t cnt, uint32_t *scr, F &&f) {
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t incl = cnt;
#pragma unroll
    for (uint32_t off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(incl, off);
        if (lane >= off) incl += y;
    }
    const uint32_t total = __shfl(incl, 63);
    if (total == 0) return;
    scr[lane] = incl;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (uint32_t base = 0; base < total; base += 64u) {
        const uint32_t item = min(base + lane, total - 1u);
        uint32_t o = 0;  // the first lane whose inclusive count exceeds item
#pragma unroll
        for (uint32_t step = 32; step; step >>= 1)
            if (scr[o + step - 1] <= item) o += step;
        const uint32_t start = o ? scr[o - 1] : 0u;
        f(o, item - start, base + lane < total);
    }
    __builtin_amdgcn_wave_barrier();
}

MH_DEV void charge_walk_log(const DScene &S, const float4 *e, uint32_t stride, uint32_t n, uint32_t med, float K,
                            GradCtx &g) {
    for (uint32_t j0 = 0; j0 < n; j0 += kLogBatchWalk) {
        float4 q[kLogBatchWalk];
#pragma unroll
        for (uint32_t b = 0; b < kLogBatchWalk; ++b)
            if (j0 + b < n) q[b] = e[(uint64_t)(j0 + b) * stride];
#pragma unroll
        for (uint32_t b = 0; b < kLogBatchWalk; ++b)
            if (j0 + b < n) sigma_t_backward(S, med, v3(q[b].x, q[b].y, q[b].z), q[b].w * K, g);
    }
}

// Mode 0: primal; 1: adjoint replay (L = primal radiance); 2: primal + MainLog
// + NEE gradients (single pass); 3: adjoint replay without the NEE gradients
// (the fallback of a Mode-2 path whose log overflowed)
template <int Mode>
MH_DEV V3 prbvol_sample(const DScene &S, const LdsBvh &B, const IntegratorParams &in, Pcg &rng, RayT ray,
                        V3 dL, V3 L, GradCtx *g, uint32_t &n_closest, uint32_t &n_shadow,
                        bool *valid_out = nullptr, NeeLog *nl = nullptr, MainLog *ml = nullptr) {
    constexpr bool Adj = Mode == 1 || Mode == 3;   // adjoint arithmetic, L-dependent terms in place
    constexpr bool Log = Mode == 2;                 // primal arithmetic, L-dependent terms logged
    constexpr bool NeeGrad = Mode == 1 || Mode == 2;
    const bool handle_null = S.vol_flags & kVolHandleNull;
    uint32_t depth = 0;
    if (!Adj) L = v3(0.f, 0.f, 0.f);
    if (Log) { ml->n = 0; ml->overflow = false; }
    V3 throughput = v3(1.f, 1.f, 1.f);
    float eta = 1.f;
    bool active = true, needs_intersection = true;
    SI si;
    si.valid = false;
    float si_t = 0.f;
    uint32_t medium = MH_INVALID;   // "TODO: support sensors inside media" (prbvolpath.py:123-124)
    bool valid_ray = false;         // (prbvolpath.py:128, 274, 327)
    (void)fminf(3.f * rng.next_float(), 2.f);   // RGB channel (scalar majorants: all channels alike)
    while (active) {
        // ---- Russian roulette (:142-149)
        active = active && nonzero(throughput);
        const float q = fminf(hmax(throughput) * (eta * eta), 0.99f);
        const bool perform_rr = depth > in.rr_depth;
        if (active) active = rng.next_float() < q || !perform_rr;
        if (perform_rr) throughput = throughput * rcp(q);
        if (!active) break;

        bool active_medium = medium != MH_INVALID, active_surface = !active_medium;
        bool escaped = false, act_null = false, act_scatter = false;
        float fw = 1.f, P = 1.f, mt = 0.f;
        V3 weight = v3(1.f, 1.f, 1.f);
        MEI mei;
        mei.valid = false;
        mei.t = 0.f;
        mei.maj = 1.f;
        mei.sigma_t = 0.f;
        mei.p = v3(0.f, 0.f, 0.f);
        mei.sigma_s = v3(0.f, 0.f, 0.f);
        const uint32_t med = medium;
        // ---- medium interaction (:157-204)
        if (active_medium) {
            const DMedium &m = S.media[med];
            sample_interaction(S, med, ray, rng.next_float(), mei);
            if (m.type == MH_MEDIUM_HOMOGENEOUS && mei.valid) ray.maxt = mei.t;
            if (needs_intersection) { trace_si(S, B, ray, si, si_t); ++n_closest; }
            needs_intersection = false;
            if (si_t < mei.t) { mei.t = __builtin_huge_valf(); mei.valid = false; }
            // transmittance_eval_pdf (medium.cpp:101-112)
            mt = fminf(mei.t, si_t) - mei.mint;
            const float tr = exp_dr((-mt) * mei.maj);
            const float tr_pdf = si_t < mei.t ? tr : tr * mei.maj;
            fw = tr_pdf > 0.f ? tr / tr_pdf : 0.f;
            weight = v3(fw, fw, fw);
            escaped = !mei.valid;
            active_medium = mei.valid;
            if (handle_null) {
                P = mei.sigma_t / mei.maj;
                if (active_medium) act_null = rng.next_float() >= P;
                act_scatter = !act_null && active_medium;
                if (act_null) weight = weight * (mei.sigma_n / (1.f - P));
            } else {
                act_scatter = active_medium;
            }
            if (act_scatter) depth += 1;
        }
        active = active && depth < in.max_depth;
        act_scatter = act_scatter && active;
        if (handle_null && act_null) { ray.o = mei.p; si_t = si_t - mei.t; }
        if (act_scatter)
            weight = v3(weight.x * (mei.sigma_s.x / P), weight.y * (mei.sigma_s.y / P), weight.z * (mei.sigma_s.z / P));
        throughput = throughput * weight;
        if ((Adj || Log) && (active_medium || escaped)) {
            // backward(dL * weight * Lo), Lo = L / max(1e-8, weight) (:202-204)
            const DMedium &m = S.media[med];
            const bool homog = m.type == MH_MEDIUM_HOMOGENEOUS;
            const float wc[3] = {weight.x, weight.y, weight.z}, Lc[3] = {L.x, L.y, L.z}, dc[3] = {dL.x, dL.y, dL.z};
            const float al[3] = {m.albedo[0], m.albedo[1], m.albedo[2]};
            const float ss[3] = {mei.sigma_s.x, mei.sigma_s.y, mei.sigma_s.z};
            const float dfw = homog ? -mt * fw : 0.f;   // d (tr / tr_pdf) / d sigma_t
            float gs = 0.f, ga[3], dwsc[3], dwa = 0.f;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                float dws;
                if (act_scatter) {
                    dws = dfw * ss[c] / P + fw * al[c] / P;   // sigma_s = sigma_t * albedo
                    dwa = fw * mei.sigma_t / P;
                } else if (act_null) {
                    dws = -fw / (1.f - P);
                } else {
                    dws = dfw;
                }
                dwsc[c] = dws;
                if (Adj) {
                    const float up = dc[c] * (Lc[c] / fmaxf(1e-8f, wc[c]));
                    gs += up * dws;
                    ga[c] = up * dwa;
                }
            }
            if (Adj) {
                sigma_t_backward(S, med, mei.p, gs, *g);
                if (act_scatter) albedo_backward(med, v3(ga[0], ga[1], ga[2]), *g);
            }
            if (Log)
                ml->add(make_float4(mei.p.x, mei.p.y, mei.p.z, __uint_as_float((act_scatter ? 2u : 0u) | (med << 2))),
                        make_float4(L.x, L.y, L.z, 0.f),
                        make_float4(dc[0] / fmaxf(1e-8f, wc[0]), dc[1] / fmaxf(1e-8f, wc[1]),
                                    dc[2] / fmaxf(1e-8f, wc[2]), 0.f),
                        make_float4(dwsc[0], dwsc[1], dwsc[2], dwa));
        }

        // ---- surface interaction (:212-238)
        active_surface = active_surface || escaped;
        if (active_surface && needs_intersection) { trace_si(S, B, ray, si, si_t); ++n_closest; }
        active_surface = active_surface && si.valid;
        const uint32_t b = active_surface ? S.shapes[si.shape].bsdf : MH_INVALID;
        const bool smooth = b != MH_INVALID && S.bsdf_type[b] == MH_BSDF_DIFFUSE;
        V3 rho = v3(0.f, 0.f, 0.f);
        if (smooth) rho = tex_eval(S, S.bsdf_tex[b], si.uvx, si.uvy);

        // ---- emitter sampling (:242-270)
        const bool active_e_surface = active_surface && smooth && depth + 1 < in.max_depth;
        const bool sample_emitters = med != MH_INVALID && !(S.media[med].flags & MH_MEDIUM_NO_EMITTER_SAMPLING);
        const bool active_e_medium = act_scatter && sample_emitters;
        if (active_e_surface || active_e_medium) {
            const Pcg nee_rng = rng;   // sampler.clone()
            DirS ds;
            const bool logged = NeeGrad && nl;
            const V3 emitted = logged ? pvp_sample_emitter<2>(S, B, mei, si, active_e_medium, rng, medium, ds,
                                                              v3(0.f, 0.f, 0.f), v3(0.f, 0.f, 0.f), nullptr, n_shadow, nl)
                                      : pvp_sample_emitter<0>(S, B, mei, si, active_e_medium, rng, medium, ds,
                                                              v3(0.f, 0.f, 0.f), v3(0.f, 0.f, 0.f), nullptr, n_shadow);
            V3 nee_w, bv = v3(0.f, 0.f, 0.f);
            float nee_pdf, bp = 0.f;
            const V3 wo_s = to_local(si, ds.d);
            if (active_e_surface) {
                diffuse_eval_pdf(rho, si.wi, wo_s, true, bv, bp);
                nee_w = bv;
                nee_pdf = bp;
            } else {
                const float ph = phase_eval(S.media[med], mei_to_local(mei, ds.d));
                nee_w = v3(ph, ph, ph);
                nee_pdf = ph;
            }
            if (ds.delta) nee_pdf = 0.f;
            const float mis = mis_weight(ds.pdf, nee_pdf);
            const V3 contrib = ((throughput * nee_w) * mis) * emitted;
            L = Adj ? L + (-contrib) : L + contrib;
            if (NeeGrad) {
                if (logged && !nl->overflow) {  // the logged walk's steps: coef * (dL . adj_emitted)
                    const float K = (dL.x * contrib.x + dL.y * contrib.y) + dL.z * contrib.z;
                    charge_walk_log(S, nl->buf + nl->t, nl->stride, nl->n, nl->med, K, *g);
                } else {
                    Pcg r2 = nee_rng;
                    DirS ds2;
                    pvp_sample_emitter<1>(S, B, mei, si, active_e_medium, r2, medium, ds2, contrib, dL, g, n_shadow);
                }
                if (active_e_surface && si.wi.z > 0.f && wo_s.z > 0.f) {
                    // backward(dL * contrib) through bsdf_val = rho / pi * cos
                    const V3 adj = ((((dL * emitted) * mis) * throughput) * kInvPi) * wo_s.z;
                    tex_backward(S, S.bsdf_tex[b], si.uvx, si.uvy, adj, *g);
                }
            }
        }

        // ---- phase function sampling (:274-294)
        valid_ray = valid_ray || act_scatter;
        if (act_scatter) {
            (void)rng.next_float();
            const float s2x = rng.next_float(), s2y = rng.next_float();
            float ph_pdf;
            const V3 wo = phase_sample(S.media[med], s2x, s2y, ph_pdf);
            act_scatter = act_scatter && ph_pdf > 0.f;
            if (act_scatter) {
                ray = spawn_ray(mei.p, v3(0.f, 0.f, 0.f), mei_to_world(mei, wo));
                needs_intersection = true;
            }
        }

        // ---- BSDF sampling (:298-331)
        if (active_surface) {
            (void)rng.next_float();
            const float s2x = rng.next_float(), s2y = rng.next_float();
            V3 bs_wo, bw;
            float bs_pdf;
            if (!smooth) {
                bs_wo = -si.wi; bs_pdf = 1.f; bw = v3(1.f, 1.f, 1.f);
            } else {
                bs_wo = square_to_cosine_hemisphere(s2x, s2y);
                bs_pdf = kInvPi * bs_wo.z;
                bw = (si.wi.z > 0.f && bs_pdf > 0.f) ? rho : v3(0.f, 0.f, 0.f);
            }
            active_surface = active_surface && bs_pdf > 0.f;
            if (active_surface) {
                if ((Adj || Log) && smooth && si.wi.z > 0.f && bs_wo.z > 0.f) {
                    // Lo = bsdf_eval * detach(L / max(1e-8, bsdf_eval)) (:305-312)
                    const V3 be = (rho * kInvPi) * bs_wo.z;
                    if (Adj) {
                        V3 adj = v3(dL.x * (L.x / fmaxf(1e-8f, be.x)), dL.y * (L.y / fmaxf(1e-8f, be.y)),
                                    dL.z * (L.z / fmaxf(1e-8f, be.z)));
                        adj = (adj * kInvPi) * bs_wo.z;
                        tex_backward(S, S.bsdf_tex[b], si.uvx, si.uvy, adj, *g);
                    }
                    if (Log)
                        ml->add(make_float4(0.f, 0.f, 0.f, __uint_as_float(1u | (S.bsdf_tex[b] << 2))),
                                make_float4(L.x, L.y, L.z, si.uvx),
                                make_float4(dL.x / fmaxf(1e-8f, be.x), dL.y / fmaxf(1e-8f, be.y),
                                            dL.z / fmaxf(1e-8f, be.z), si.uvy),
                                make_float4(bs_wo.z, 0.f, 0.f, 0.f));
                }
                throughput = throughput * bw;
                ray = spawn_ray(si.p, si.n, to_world(si, bs_wo));
                needs_intersection = true;
                if (smooth) { depth += 1; valid_ray = true; }
                if (is_medium_transition(S, si)) medium = target_medium(S, si, ray.d);
            }
        }
        active = active && (active_surface || active_medium);
    }
    if (valid_out) *valid_out = valid_ray;
    return L;
}

// one logged L-dependent term (q0..q3: a MainLog entry) of a path whose
// radiance is now L_total
MH_DEV void pvp_log_entry(const DScene &S, float4 q0, float4 q1, float4 q2, float4 q3, V3 Ltot, GradCtx &g) {
    const uint32_t bits = __float_as_uint(q0.w), idx = bits >> 2;
    const V3 Lsuf = Ltot - v3(q1.x, q1.y, q1.z);  // prbvolpath.py: L - (contributions so far)
    const V3 up = v3(q2.x * Lsuf.x, q2.y * Lsuf.y, q2.z * Lsuf.z);
    if (bits & 1u) {
        const V3 adj = (up * kInvPi) * q3.x;
        tex_backward(S, idx, q1.w, q2.w, adj, g);
    } else {
        const float gs = (up.x * q3.x + up.y * q3.y) + up.z * q3.z;
        sigma_t_backward(S, idx, v3(q0.x, q0.y, q0.z), gs, g);
        if (bits & 2u) albedo_backward(idx, up * q3.w, g);
    }
}

// the logged L-dependent terms of a path whose radiance is now L_total
MH_DEV void pvp_log_apply(const DScene &S, const MainLog &ml, V3 Ltot, GradCtx &g) {
    for (uint32_t j0 = 0; j0 < ml.n; j0 += kLogBatchMain) {
        float4 q[kLogBatchMain][4];
#pragma unroll
        for (uint32_t b = 0; b < kLogBatchMain; ++b) {
            if (j0 + b >= ml.n) break;
            const uint64_t o = (uint64_t)4 * (j0 + b) * ml.stride + ml.t;
#pragma unroll
            for (uint32_t c = 0; c < 4; ++c) q[b][c] = ml.buf[o + c * (uint64_t)ml.stride];
        }
#pragma unroll
        for (uint32_t b = 0; b < kLogBatchMain; ++b) {
            if (j0 + b >= ml.n) break;
            pvp_log_entry(S, q[b][0], q[b][1], q[b][2], q[b][3], Ltot, g);
        }
    }
}


// small (register-accumulated) gradient slots: wave butterfly, then one
// atomic per wave and component
MH_DEV void flush_small_slots(GradCtx &g, const GradArgs &ga) {
    if (g.fx_mode) {
        // a lane's own float sums (prb_fused accumulates in registers, not
        // through acc_add): per lane in a fixed order, so fold them exactly
        for (uint32_t p = 0; p < ga.n_rgb; ++p) {
            const V3 a = acc_get(g, (int32_t)p);
            if (a.x != 0.f || a.y != 0.f || a.z != 0.f) acc_add_fx(g, (int32_t)p, a);
        }
        g.acc0 = g.acc1 = g.acc2 = g.acc3 = v3(0.f, 0.f, 0.f);
    }
    if (g.fx_mode == 1) {  // the wave's maxima (corner_scatter, acc_add_fx, bmp_add_fx) -> fx_max[0 .. kMaxParams]
        __builtin_amdgcn_wave_barrier();
        const uint32_t j = threadIdx.x & 63u;
        if (j <= (uint32_t)kMaxParams) {
            const unsigned int v = fx_wave_max()[j];
            if (v) atomicMax(g.fx_max + j, v);
        }
        return;
    }
    if (g.fx_mode == 2) {  // the wave's exact int64 sums -> the global words (acc_add_fx)
        __builtin_amdgcn_wave_barrier();
        const uint32_t j = threadIdx.x & 63u;
        if (j < 3u * ga.n_rgb) {
            const unsigned long long v = fx_wave_sums()[j];
            unsigned long long *w = reinterpret_cast<unsigned long long *>(reinterpret_cast<uint8_t *>(g.fx_max) + 192);
            if (v) gatomic_add(w + j, v);
        }
        return;
    }
    for (uint32_t p = 0; p < ga.n_rgb; ++p) {
        const int slot = (int)p;
        const V3 a = acc_get(g, slot);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            float v = c == 0 ? a.x : c == 1 ? a.y : a.z;
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
            if ((threadIdx.x & 63) == 0 && v != 0.f) gatomic_add(ga.bufs[slot] + c, v);
        }
    }
}

MH_DEV GradCtx make_grad_ctx(const GradArgs &ga) {
    if (ga.fx_mode) {  // this wave's LDS maxima (pass 1) / sums (pass 2) start at zero
        if ((threadIdx.x & 63u) < kFxWaveWords) fx_wave_sums()[threadIdx.x & 63u] = 0ull;
        __builtin_amdgcn_wave_barrier();
    }
    GradCtx g;
    g.slot_of_tex = ga.slot_of_tex;
    g.bufs = ga.bufs;
    g.is_rgb = ga.is_rgb;
    g.sigma_slot = ga.sigma_slot;
    g.albedo_slot = ga.albedo_slot;
    g.corner = ga.corner;
    g.fx_mode = ga.fx_mode;
    g.fx_max = ga.fx_max;
    g.fx_scale = ga.fx_scale;
    g.fx_i64 = ga.fx_i64;
    g.fx_f32 = ga.fx_f32;
    g.lds_slot = -1;
    g.lds_acc = nullptr;
    g.lds_floats = 0;
    g.fwd = false;
    g.fsum = 0.f;
    g.acc0 = g.acc1 = g.acc2 = g.acc3 = v3(0.f, 0.f, 0.f);
    g.hot_med = ga.hot_med;
    g.hot_sigma = ga.hot_sigma;
    g.hot_albedo = ga.hot_albedo;
    g.hot_buf = ga.hot_buf;
    g.hot_corner = ga.hot_corner;
    return g;
}

}  // namespace mh
