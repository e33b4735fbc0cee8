// mh_bvh.cpp — host BVH2 builder (binned SAH) replacing the OptiX GAS/IAS
// build of the reference (src/render/scene_optix.inl:449-514).
//
// Output layout is the device layout of mh_device.hpp: 64-B nodes holding the
// two child boxes (padded conservatively so the fma slab test can never
// reject a true hit) and 64-B primitive records in leaf order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <stdexcept>

#include "mh_device.hpp"
#include "mh_internal.hpp"

namespace mh {
namespace {

struct Box {
    float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX};
    float hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    void grow(const float *l, const float *h) {
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], l[a]);
            hi[a] = std::max(hi[a], h[a]);
        }
    }
    void grow(const Box &b) { grow(b.lo, b.hi); }
    float area() const {
        float d[3];
        for (int a = 0; a < 3; ++a) d[a] = std::max(hi[a] - lo[a], 0.f);
        return 2.f * (d[0] * d[1] + d[1] * d[2] + d[2] * d[0]);
    }
    bool valid() const { return lo[0] <= hi[0]; }
};

constexpr int kBins = 16;
// leaf limits: the per-lane stream engine packs the count in 3 bits (<= 7)
constexpr uint32_t kMaxDepth = 48;

struct Builder {
    const std::vector<BuildPrim> &p;
    std::vector<uint32_t> idx;
    std::vector<Node> nodes;
    std::vector<uint32_t> order;  // final prim order
    uint32_t max_depth = 0;
    uint32_t kMaxLeaf = 4;
    float trav_cost = 1.0f;  // SAH traversal cost relative to one primitive test

    explicit Builder(const std::vector<BuildPrim> &prims) : p(prims) {
        idx.resize(p.size());
        for (size_t i = 0; i < p.size(); ++i) idx[i] = (uint32_t)i;
    }

    Box bounds(uint32_t b, uint32_t e) const {
        Box bb;
        for (uint32_t i = b; i < e; ++i) bb.grow(p[idx[i]].lo, p[idx[i]].hi);
        return bb;
    }
    float centroid(uint32_t i, int a) const { return 0.5f * (p[idx[i]].lo[a] + p[idx[i]].hi[a]); }

    // split [b, e) -> returns mid (b < mid < e) or e for "make leaf"
    uint32_t split(uint32_t b, uint32_t e, uint32_t depth) {
        const uint32_t n = e - b;
        if (n <= 2) return e;
        Box cb;
        for (uint32_t i = b; i < e; ++i) {
            float c[3] = {centroid(i, 0), centroid(i, 1), centroid(i, 2)};
            cb.grow(c, c);
        }
        Box node_box = bounds(b, e);
        float best_cost = FLT_MAX;
        int best_axis = -1, best_bin = -1;
        for (int a = 0; a < 3; ++a) {
            float ext = cb.hi[a] - cb.lo[a];
            if (!(ext > 0.f)) continue;
            Box bin_box[kBins];
            uint32_t cnt[kBins] = {0};
            for (uint32_t i = b; i < e; ++i) {
                int k = (int)((centroid(i, a) - cb.lo[a]) / ext * kBins);
                k = std::min(std::max(k, 0), kBins - 1);
                cnt[k]++;
                bin_box[k].grow(p[idx[i]].lo, p[idx[i]].hi);
            }
            Box lb[kBins], rb[kBins];
            uint32_t lc[kBins], rc[kBins];
            Box acc;
            uint32_t c = 0;
            for (int k = 0; k < kBins; ++k) {
                acc.grow(bin_box[k]);
                c += cnt[k];
                lb[k] = acc;
                lc[k] = c;
            }
            acc = Box();
            c = 0;
            for (int k = kBins - 1; k >= 0; --k) {
                acc.grow(bin_box[k]);
                c += cnt[k];
                rb[k] = acc;
                rc[k] = c;
            }
            for (int k = 0; k < kBins - 1; ++k) {
                if (lc[k] == 0 || rc[k + 1] == 0) continue;
                float cost = lb[k].area() * lc[k] + rb[k + 1].area() * rc[k + 1];
                if (cost < best_cost) {
                    best_cost = cost;
                    best_axis = a;
                    best_bin = k;
                }
            }
        }
        const bool force = n > kMaxLeaf || depth + 1 >= kMaxDepth;
        if (best_axis < 0) {
            if (n <= kMaxLeaf) return e;
            // degenerate centroids: median split on index
            return b + n / 2;
        }
        const float area = node_box.area();
        if (!force && area > 0.f && trav_cost + best_cost / area >= (float)n) return e;
        const int a = best_axis;
        const float ext = cb.hi[a] - cb.lo[a];
        auto mid_it = std::partition(idx.begin() + b, idx.begin() + e, [&](uint32_t q) {
            float c = 0.5f * (p[q].lo[a] + p[q].hi[a]);
            int k = (int)((c - cb.lo[a]) / ext * kBins);
            k = std::min(std::max(k, 0), kBins - 1);
            return k <= best_bin;
        });
        uint32_t mid = (uint32_t)(mid_it - idx.begin());
        if (mid == b || mid == e) mid = b + n / 2;
        return mid;
    }

    static void pad(Box &b) {
        for (int a = 0; a < 3; ++a) {
            float m = std::max(std::fabs(b.lo[a]), std::fabs(b.hi[a]));
            float e = 1e-5f * (m + (b.hi[a] - b.lo[a])) + 1e-7f;
            b.lo[a] -= e;
            b.hi[a] += e;
        }
    }

    // emit a child reference (leaf or inner) for range [b, e)
    void child(uint32_t b, uint32_t e, uint32_t depth, float4 &lo, float4 &hi) {
        Box bb = bounds(b, e);
        pad(bb);
        lo = make_float4(bb.lo[0], bb.lo[1], bb.lo[2], 0.f);
        hi = make_float4(bb.hi[0], bb.hi[1], bb.hi[2], 0.f);
        uint32_t mid = split(b, e, depth);
        if (mid == e) {  // leaf
            uint32_t first = (uint32_t)order.size();
            for (uint32_t i = b; i < e; ++i) order.push_back(idx[i]);
            uint32_t cnt = e - b;
            memcpy(&lo.w, &first, 4);
            memcpy(&hi.w, &cnt, 4);
            max_depth = std::max(max_depth, depth);
        } else {
            uint32_t ni = inner(b, mid, e, depth);
            uint32_t zero = 0;
            memcpy(&lo.w, &ni, 4);
            memcpy(&hi.w, &zero, 4);
        }
    }

    uint32_t inner(uint32_t b, uint32_t mid, uint32_t e, uint32_t depth) {
        uint32_t ni = (uint32_t)nodes.size();
        nodes.push_back(Node{});
        Node n;
        child(b, mid, depth + 1, n.lo0, n.hi0);
        child(mid, e, depth + 1, n.lo1, n.hi1);
        nodes[ni] = n;
        return ni;
    }
};

}  // namespace

void build_bvh(const std::vector<BuildPrim> &in, BvhOut &out, uint32_t max_leaf, float trav_cost) {
    out = BvhOut();
    if (in.empty()) return;
    Builder bld(in);
    bld.kMaxLeaf = std::max<uint32_t>(2, max_leaf);
    bld.trav_cost = trav_cost;
    const uint32_t n = (uint32_t)in.size();
    if (n == 1) {
        // root with two identical single-prim leaves (the traversal needs an inner root)
        Node r;
        bld.order.push_back(0);
        Box bb = bld.bounds(0, 1);
        Builder::pad(bb);
        uint32_t first = 0, cnt = 1;
        r.lo0 = make_float4(bb.lo[0], bb.lo[1], bb.lo[2], 0.f);
        r.hi0 = make_float4(bb.hi[0], bb.hi[1], bb.hi[2], 0.f);
        memcpy(&r.lo0.w, &first, 4);
        memcpy(&r.hi0.w, &cnt, 4);
        r.lo1 = r.lo0;
        r.hi1 = r.hi0;
        bld.nodes.push_back(r);
        bld.max_depth = 1;
    } else {
        uint32_t mid = bld.split(0, n, 0);
        if (mid == n) mid = n / 2;  // the root is always an inner node
        bld.inner(0, mid, n, 0);
    }
    out.n_nodes = (uint32_t)bld.nodes.size();
    out.n_prims = (uint32_t)bld.order.size();
    out.depth = bld.max_depth;
    out.nodes.resize(sizeof(Node) * out.n_nodes);
    memcpy(out.nodes.data(), bld.nodes.data(), out.nodes.size());
    out.prims.resize(sizeof(Prim) * out.n_prims);
    Prim *dst = reinterpret_cast<Prim *>(out.prims.data());
    for (uint32_t i = 0; i < out.n_prims; ++i) {
        const BuildPrim &bp = in[bld.order[i]];
        Prim q;
        q.a = make_float4(bp.rec[0], bp.rec[1], bp.rec[2], bp.rec[3]);
        q.b = make_float4(bp.rec[4], bp.rec[5], bp.rec[6], bp.rec[7]);
        q.c = make_float4(bp.rec[8], bp.rec[9], bp.rec[10], bp.rec[11]);
        // w: position in scene order (shapes, then faces) = the tie-break key
        q.info = make_uint4(bp.shape, bp.prim, bp.type, bld.order[i]);
        dst[i] = q;
    }
}

}  // namespace mh
