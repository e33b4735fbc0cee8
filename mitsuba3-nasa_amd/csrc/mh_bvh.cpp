// mh_bvh.cpp — host BVH2 builder (binned SAH) replacing the OptiX GAS/IAS
// build of the reference (src/render/scene_optix.inl:449-514).
//
// Output layout is the device layout of mh_device.hpp: 64-B nodes holding the
// two child boxes (padded conservatively so the fma slab test can never
// reject a true hit) and 64-B primitive records in leaf order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <thread>

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

// SAH bins: 16 for the small (packet-engine) scenes, kBinsLarge otherwise --
// 1M / 4M-triangle path 586-592 / 492-500 Msamples/s at 16 bins, 605 / 510 at
// 64, 608-618 / 518-521 at 128 (round 5, same box; build 1.1 -> 1.55 s for 4M)
#ifndef MH_BVH_BINS
#define MH_BVH_BINS 128
#endif
constexpr int kBinsLarge = MH_BVH_BINS, kBinsSmall = 16, kBinsMax = kBinsLarge > kBinsSmall ? kBinsLarge : kBinsSmall;
// leaf limits: the per-lane stream engine packs the count in 3 bits (<= 7)
constexpr uint32_t kMaxDepth = 48;

// Large ranges (the top levels of a big mesh) run each O(n) pass over T
// threads: chunk-local boxes and bins reduced in chunk order (min / max and
// integer counts, so the result does not depend on T), and a stable
// partition through a scratch array.  Below `task_min` primitives a subtree
// is deferred and built by one worker (build_bvh: subtrees in parallel,
// stitched in task order), so the BVH is the same for any thread count.
struct Par {
    uint32_t threads = 1;
    uint32_t min_range = 1u << 16;   // ranges below this run their passes on one thread
    template <class F>
    void chunks(uint32_t b, uint32_t e, F &&f) const {   // f(chunk, cb, ce)
        const uint32_t n = e - b;
        const uint32_t T = (threads > 1 && n >= min_range) ? threads : 1u;
        if (T == 1) { f(0u, b, e); return; }
        std::vector<std::thread> th;
        for (uint32_t t = 0; t < T; ++t)
            th.emplace_back([&, t] { f(t, b + (uint32_t)((uint64_t)n * t / T), b + (uint32_t)((uint64_t)n * (t + 1) / T)); });
        for (auto &x : th) x.join();
    }
    uint32_t nchunks(uint32_t n) const { return (threads > 1 && n >= min_range) ? threads : 1u; }
};

struct Pending { uint32_t node, slot, b, e, depth; };

struct Builder {
    const std::vector<BuildPrim> &p;
    std::vector<uint32_t> &idx;
    std::vector<Node> nodes;
    std::vector<uint32_t> order;  // final prim order
    uint32_t max_depth = 0;
    uint32_t kMaxLeaf = 4;
    int nb = kBinsSmall;     // SAH bins
    float trav_cost = 1.0f;  // SAH traversal cost relative to one primitive test
    Par par;
    uint32_t task_min = 0;            // defer subtrees smaller than this (0: never)
    std::vector<Pending> pending;

    Builder(const std::vector<BuildPrim> &prims, std::vector<uint32_t> &ids) : p(prims), idx(ids) {}

    Box bounds(uint32_t b, uint32_t e) const {
        std::vector<Box> part(par.nchunks(e - b));
        par.chunks(b, e, [&](uint32_t t, uint32_t cb, uint32_t ce) {
            Box bb;
            for (uint32_t i = cb; i < ce; ++i) bb.grow(p[idx[i]].lo, p[idx[i]].hi);
            part[t] = bb;
        });
        Box bb;
        for (const Box &x : part) bb.grow(x);
        return bb;
    }
    float centroid(uint32_t i, int a) const { return 0.5f * (p[idx[i]].lo[a] + p[idx[i]].hi[a]); }

    // split [b, e) -> returns mid (b < mid < e) or e for "make leaf"
    uint32_t split(uint32_t b, uint32_t e, uint32_t depth, const Box &node_box) {
        const uint32_t n = e - b;
        if (n <= 2) return e;
        const uint32_t T = par.nchunks(n);
        std::vector<Box> cparts(T);
        par.chunks(b, e, [&](uint32_t t, uint32_t cb0, uint32_t ce) {
            Box cb;
            for (uint32_t i = cb0; i < ce; ++i) {
                float c[3] = {centroid(i, 0), centroid(i, 1), centroid(i, 2)};
                cb.grow(c, c);
            }
            cparts[t] = cb;
        });
        Box cb;
        for (const Box &x : cparts) cb.grow(x);
        // the three axes' bins in one pass
        struct Bins { Box box[3][kBinsMax]; uint32_t cnt[3][kBinsMax]; };
        std::vector<Bins> bparts(T);
        par.chunks(b, e, [&](uint32_t t, uint32_t c0, uint32_t c1) {
            Bins &B = bparts[t];
            memset(B.cnt, 0, sizeof(B.cnt));
            for (int a = 0; a < 3; ++a)
                for (int k = 0; k < nb; ++k) B.box[a][k] = Box();
            for (uint32_t i = c0; i < c1; ++i) {
                const BuildPrim &q = p[idx[i]];
                for (int a = 0; a < 3; ++a) {
                    const float ext = cb.hi[a] - cb.lo[a];
                    if (!(ext > 0.f)) continue;
                    int k = (int)((0.5f * (q.lo[a] + q.hi[a]) - cb.lo[a]) / ext * nb);
                    k = std::min(std::max(k, 0), nb - 1);
                    B.cnt[a][k]++;
                    B.box[a][k].grow(q.lo, q.hi);
                }
            }
        });
        float best_cost = FLT_MAX;
        int best_axis = -1, best_bin = -1;
        for (int a = 0; a < 3; ++a) {
            float ext = cb.hi[a] - cb.lo[a];
            if (!(ext > 0.f)) continue;
            Box bin_box[kBinsMax];
            uint32_t cnt[kBinsMax] = {0};
            for (uint32_t t = 0; t < T; ++t)
                for (int k = 0; k < nb; ++k) {
                    cnt[k] += bparts[t].cnt[a][k];
                    bin_box[k].grow(bparts[t].box[a][k]);
                }
            Box lb[kBinsMax], rb[kBinsMax];
            uint32_t lc[kBinsMax], rc[kBinsMax];
            Box acc;
            uint32_t c = 0;
            for (int k = 0; k < nb; ++k) {
                acc.grow(bin_box[k]);
                c += cnt[k];
                lb[k] = acc;
                lc[k] = c;
            }
            acc = Box();
            c = 0;
            for (int k = nb - 1; k >= 0; --k) {
                acc.grow(bin_box[k]);
                c += cnt[k];
                rb[k] = acc;
                rc[k] = c;
            }
            for (int k = 0; k < nb - 1; ++k) {
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
        auto left = [&](uint32_t q) {
            float c = 0.5f * (p[q].lo[a] + p[q].hi[a]);
            int k = (int)((c - cb.lo[a]) / ext * nb);
            k = std::min(std::max(k, 0), nb - 1);
            return k <= best_bin;
        };
        uint32_t mid;
        if (T == 1) {
            mid = (uint32_t)(std::stable_partition(idx.begin() + b, idx.begin() + e, left) - idx.begin());
        } else {  // stable partition over T chunks: count, offsets, scatter, copy back
            std::vector<uint32_t> nl(T, 0), tmp(n);
            par.chunks(b, e, [&](uint32_t t, uint32_t c0, uint32_t c1) {
                uint32_t c = 0;
                for (uint32_t i = c0; i < c1; ++i) c += left(idx[i]) ? 1u : 0u;
                nl[t] = c;
            });
            uint32_t total_l = 0;
            std::vector<uint32_t> ol(T), orr(T);
            for (uint32_t t = 0; t < T; ++t) { ol[t] = total_l; total_l += nl[t]; }
            uint32_t acc_r = total_l;
            for (uint32_t t = 0; t < T; ++t) {
                orr[t] = acc_r;
                acc_r += (uint32_t)((uint64_t)n * (t + 1) / T - (uint64_t)n * t / T) - nl[t];
            }
            par.chunks(b, e, [&](uint32_t t, uint32_t c0, uint32_t c1) {
                uint32_t l = ol[t], r = orr[t];
                for (uint32_t i = c0; i < c1; ++i) tmp[left(idx[i]) ? l++ : r++] = idx[i];
            });
            par.chunks(b, e, [&](uint32_t, uint32_t c0, uint32_t c1) {
                std::copy(tmp.begin() + (c0 - b), tmp.begin() + (c1 - b), idx.begin() + c0);
            });
            mid = b + total_l;
        }
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

    // emit a child reference (leaf or inner) for range [b, e) into slot
    // `slot` of node `node` (deferred as a Pending task below task_min)
    void child(uint32_t b, uint32_t e, uint32_t depth, float4 &lo, float4 &hi, uint32_t node = 0, uint32_t slot = 0) {
        Box bb = bounds(b, e);
        const Box raw = bb;
        pad(bb);
        lo = make_float4(bb.lo[0], bb.lo[1], bb.lo[2], 0.f);
        hi = make_float4(bb.hi[0], bb.hi[1], bb.hi[2], 0.f);
        if (task_min && e - b < task_min) {  // built later by a worker (build_bvh stitches it in)
            pending.push_back(Pending{node, slot, b, e, depth});
            return;
        }
        uint32_t mid = split(b, e, depth, raw);
        if (mid == e) {  // leaf
            uint32_t first = (uint32_t)order.size();
            // primitives of one type together (scene order within a type): the
            // packet engine tests same-type pairs on packed f32 (packet_leaf)
            std::stable_sort(idx.begin() + b, idx.begin() + e, [&](uint32_t x, uint32_t y) {
                return p[x].type != p[y].type ? p[x].type < p[y].type : x < y;
            });
            uint32_t nrect = 0;
            for (uint32_t i = b; i < e; ++i) {
                order.push_back(idx[i]);
                nrect += p[idx[i]].type == MH_SHAPE_RECTANGLE ? 1u : 0u;
            }
            uint32_t cnt = (e - b) | nrect << kLeafRectShift;
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
        child(b, mid, depth + 1, n.lo0, n.hi0, ni, 0);
        child(mid, e, depth + 1, n.lo1, n.hi1, ni, 1);
        nodes[ni] = n;
        return ni;
    }
};

// build threads: MH_BVH_THREADS, else the host's cores (at most 32)
uint32_t bvh_threads() {
    if (const char *e = getenv("MH_BVH_THREADS")) return (uint32_t)std::max(1, atoi(e));
    const uint32_t hc = std::thread::hardware_concurrency();
    return std::max(1u, std::min(32u, hc ? hc : 1u));
}

}  // namespace

void build_bvh(const std::vector<BuildPrim> &in, BvhOut &out, uint32_t max_leaf, float trav_cost) {
    out = BvhOut();
    if (in.empty()) return;
    const uint32_t n = (uint32_t)in.size();
    std::vector<uint32_t> ids(n);
    for (uint32_t i = 0; i < n; ++i) ids[i] = i;
    Builder bld(in, ids);
    bld.kMaxLeaf = std::max<uint32_t>(2, max_leaf);
    bld.trav_cost = trav_cost;
    bld.nb = n <= 64 ? kBinsSmall : kBinsLarge;  // the mh_scene_create "small" cut
    const uint32_t T = bvh_threads();
    bld.par.threads = T;
    // subtrees below n / 64 primitives (and at least 4096) go to the workers;
    // the cut does not depend on T, so neither does the node layout
    if (n >= (1u << 15)) bld.task_min = std::max<uint32_t>(4096, n / 64);
    if (n == 1) {
        // root with two identical single-prim leaves (the traversal needs an inner root)
        Node r;
        bld.order.push_back(0);
        Box bb = bld.bounds(0, 1);
        Builder::pad(bb);
        uint32_t first = 0, cnt = 1u | (in[0].type == MH_SHAPE_RECTANGLE ? 1u : 0u) << kLeafRectShift;
        r.lo0 = make_float4(bb.lo[0], bb.lo[1], bb.lo[2], 0.f);
        r.hi0 = make_float4(bb.hi[0], bb.hi[1], bb.hi[2], 0.f);
        memcpy(&r.lo0.w, &first, 4);
        memcpy(&r.hi0.w, &cnt, 4);
        r.lo1 = r.lo0;
        r.hi1 = r.hi0;
        bld.nodes.push_back(r);
        bld.max_depth = 1;
    } else {
        uint32_t mid = bld.split(0, n, 0, bld.bounds(0, n));
        if (mid == n) mid = n / 2;  // the root is always an inner node
        bld.inner(0, mid, n, 0);
    }
    if (!bld.pending.empty()) {
        // deferred subtrees: one sequential builder each, T workers, stitched in task order
        const size_t np = bld.pending.size();
        std::vector<Builder *> sub(np, nullptr);
        std::vector<float4> sub_lo(np), sub_hi(np);   // each subtree's own reference (leaf or local node 0)
        std::atomic<size_t> next{0};
        std::vector<std::thread> th;
        for (uint32_t t = 0; t < std::min<size_t>(T, np); ++t)
            th.emplace_back([&] {
                for (size_t k; (k = next.fetch_add(1)) < np;) {
                    const Pending &pd = bld.pending[k];
                    Builder *sb = new Builder(in, ids);
                    sb->kMaxLeaf = bld.kMaxLeaf;
                    sb->nb = bld.nb;
                    sb->trav_cost = bld.trav_cost;
                    sb->child(pd.b, pd.e, pd.depth, sub_lo[k], sub_hi[k]);
                    sub[k] = sb;
                }
            });
        for (auto &x : th) x.join();
        for (size_t k = 0; k < np; ++k) {
            const Pending &pd = bld.pending[k];
            Builder *sb = sub[k];
            const uint32_t nbase = (uint32_t)bld.nodes.size(), obase = (uint32_t)bld.order.size();
            auto fix = [&](float4 &lo, const float4 &hi) {   // a subtree-local child reference -> global
                uint32_t w, cnt;
                memcpy(&w, &lo.w, 4);
                memcpy(&cnt, &hi.w, 4);
                w = (cnt & kLeafCountMask) ? w + obase : w + nbase;
                memcpy(&lo.w, &w, 4);
            };
            float4 rlo = sub_lo[k];
            fix(rlo, sub_hi[k]);
            Node &parent = bld.nodes[pd.node];
            (pd.slot ? parent.lo1 : parent.lo0).w = rlo.w;
            (pd.slot ? parent.hi1 : parent.hi0).w = sub_hi[k].w;
            for (Node q : sb->nodes) {
                fix(q.lo0, q.hi0);
                fix(q.lo1, q.hi1);
                bld.nodes.push_back(q);
            }
            bld.order.insert(bld.order.end(), sb->order.begin(), sb->order.end());
            bld.max_depth = std::max(bld.max_depth, sb->max_depth);
            delete sb;
        }
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

namespace {
constexpr uint32_t kLeafRef = 0x80000000u, kEmptyRef = 0xffffffffu;  // as mh_shading.hpp kLeafBit

struct Entry {
    float lo[3], hi[3];
    uint32_t inner;   // BVH2 node index, or ~0u for a leaf
    uint32_t first, count;
    float area() const {
        const float d[3] = {hi[0] - lo[0], hi[1] - lo[1], hi[2] - lo[2]};
        return 2.f * (d[0] * d[1] + d[1] * d[2] + d[2] * d[0]);
    }
};

struct Collapser {
    const Node *n2;
    std::vector<Node4> out;
    uint32_t depth = 0;
    void entries_of(uint32_t i, Entry e[2]) const {
        const Node &n = n2[i];
        const float4 *lo[2] = {&n.lo0, &n.lo1}, *hi[2] = {&n.hi0, &n.hi1};
        for (int c = 0; c < 2; ++c) {
            uint32_t w, cnt;
            memcpy(&w, &lo[c]->w, 4);
            memcpy(&cnt, &hi[c]->w, 4);
            cnt &= kLeafCountMask;
            e[c].lo[0] = lo[c]->x; e[c].lo[1] = lo[c]->y; e[c].lo[2] = lo[c]->z;
            e[c].hi[0] = hi[c]->x; e[c].hi[1] = hi[c]->y; e[c].hi[2] = hi[c]->z;
            e[c].inner = cnt ? ~0u : w;
            e[c].first = w;
            e[c].count = cnt;
        }
    }
    uint32_t emit(uint32_t i, uint32_t d) {
        depth = std::max(depth, d);
        Entry e[4];
        int k = 0;
        entries_of(i, e);
        k = 2;
        while (k < 4) {   // open the inner child of largest area
            int best = -1;
            for (int c = 0; c < k; ++c)
                if (e[c].inner != ~0u && (best < 0 || e[c].area() > e[best].area())) best = c;
            if (best < 0) break;
            Entry sub[2];
            entries_of(e[best].inner, sub);
            e[best] = sub[0];
            e[k++] = sub[1];
        }
        const uint32_t me = (uint32_t)out.size();
        out.push_back(Node4{});
        Node4 n;
        float lx[4], ly[4], lz[4], hx[4], hy[4], hz[4];
        uint32_t ref[4];
        for (int c = 0; c < 4; ++c) {
            if (c >= k) {   // empty slot: a box no ray enters
                lx[c] = ly[c] = lz[c] = FLT_MAX;
                hx[c] = hy[c] = hz[c] = -FLT_MAX;
                ref[c] = kEmptyRef;
                continue;
            }
            lx[c] = e[c].lo[0]; ly[c] = e[c].lo[1]; lz[c] = e[c].lo[2];
            hx[c] = e[c].hi[0]; hy[c] = e[c].hi[1]; hz[c] = e[c].hi[2];
            ref[c] = e[c].inner == ~0u ? (kLeafRef | (e[c].first << 5) | e[c].count) : 0u;
        }
        for (int c = 0; c < k; ++c)
            if (e[c].inner != ~0u) ref[c] = emit(e[c].inner, d + 1);
        n.lox = make_float4(lx[0], lx[1], lx[2], lx[3]);
        n.loy = make_float4(ly[0], ly[1], ly[2], ly[3]);
        n.loz = make_float4(lz[0], lz[1], lz[2], lz[3]);
        n.hix = make_float4(hx[0], hx[1], hx[2], hx[3]);
        n.hiy = make_float4(hy[0], hy[1], hy[2], hy[3]);
        n.hiz = make_float4(hz[0], hz[1], hz[2], hz[3]);
        n.ref = make_uint4(ref[0], ref[1], ref[2], ref[3]);
        n.pad = make_uint4(0, 0, 0, 0);
        out[me] = n;
        return me;
    }
};
}  // namespace

void collapse_bvh4(const BvhOut &b2, std::vector<uint8_t> &nodes4, uint32_t &n4, uint32_t &depth4) {
    nodes4.clear();
    n4 = depth4 = 0;
    if (b2.n_nodes == 0) return;
    Collapser c;
    c.n2 = reinterpret_cast<const Node *>(b2.nodes.data());
    c.emit(0, 1);
    n4 = (uint32_t)c.out.size();
    depth4 = c.depth;
    nodes4.resize(sizeof(Node4) * n4);
    memcpy(nodes4.data(), c.out.data(), nodes4.size());
}

// ---------------------------------------------------------------------------
// Quantised wide BVH (round 4).  The stream engine on a large mesh is bound
// by dependent node / primitive fetches from the Infinity Cache, so the bytes
// per fetch and the lines a ray touches are what to cut:
//  - 64-B nodes (QNode4) instead of 128-B Node4: child boxes as 8-bit
//    offsets in a per-node power-of-two grid;
//  - the inner children of a node are stored contiguously, parents before
//    children, depth first over sibling groups, so a node's children (the
//    next fetch) sit in one or two cache lines;
//  - 48-B primitive records (PrimC) instead of 64 B.
// Conservative by construction: every decoded bound fma(q, 2^e, o) computed
// in float, exactly as the device decodes it, is checked against the padded
// float box of the BVH2 and moved outward until it contains it, so the slab
// test enters every child the float boxes would (the hit set of a ray, and
// with the closest-hit rule its result, do not change).
// ---------------------------------------------------------------------------
namespace {
struct QBuild {
    const Node *n2;
    struct CNode { Entry e[4]; int k; uint32_t child[4]; };
    std::vector<CNode> cn;   // collapsed nodes, in creation order
    uint32_t depth = 0;
    uint32_t collapse(uint32_t i, uint32_t d) {
        depth = std::max(depth, d);
        Collapser c;
        c.n2 = n2;
        CNode x;
        c.entries_of(i, x.e);
        int k = 2;
        while (k < 4) {   // open the inner child of largest area (as collapse_bvh4)
            int best = -1;
            for (int j = 0; j < k; ++j)
                if (x.e[j].inner != ~0u && (best < 0 || x.e[j].area() > x.e[best].area())) best = j;
            if (best < 0) break;
            Entry sub[2];
            c.entries_of(x.e[best].inner, sub);
            x.e[best] = sub[0];
            x.e[k++] = sub[1];
        }
        x.k = k;
        const uint32_t me = (uint32_t)cn.size();
        cn.push_back(x);
        for (int j = 0; j < k; ++j) {
            const uint32_t ch = x.e[j].inner != ~0u ? collapse(x.e[j].inner, d + 1) : ~0u;
            cn[me].child[j] = ch;
        }
        return me;
    }
};

// one axis of a node: exponent byte and the 8-bit bounds of its k children
// (lo rounded down, hi up, each checked on the float decode); false if the
// extent cannot be represented (non-finite boxes)
bool quantise_axis(float o, const float *lo, const float *hi, int k, uint32_t &ebyte, uint8_t *qlo, uint8_t *qhi) {
    float ext = 0.f;
    for (int c = 0; c < k; ++c) ext = std::max(ext, hi[c] - o);
    if (!std::isfinite(ext) || !std::isfinite(o)) return false;
    int e = -126;
    if (ext > 0.f) {
        int ex;
        std::frexp((double)ext / 255.0, &ex);   // ext / 255 < 2^ex
        e = std::max(-126, ex);
    }
    for (; e <= 127; ++e) {
        const float s = std::ldexp(1.0f, e);
        bool ok = true;
        for (int c = 0; c < k && ok; ++c) {
            double fl = std::floor(((double)lo[c] - (double)o) / (double)s);
            int ql = (int)std::min(255.0, std::max(0.0, fl));
            while (ql > 0 && std::fmaf((float)ql, s, o) > lo[c]) --ql;
            double ch = std::ceil(((double)hi[c] - (double)o) / (double)s);
            int qh = (int)std::min(256.0, std::max(0.0, ch));
            while (qh <= 255 && std::fmaf((float)qh, s, o) < hi[c]) ++qh;
            if (qh > 255 || std::fmaf((float)ql, s, o) > lo[c]) { ok = false; break; }
            qlo[c] = (uint8_t)ql;
            qhi[c] = (uint8_t)qh;
        }
        if (ok) { ebyte = (uint32_t)(e + 127); return true; }
    }
    return false;
}
}  // namespace

bool build_qbvh4(const BvhOut &b2, std::vector<uint8_t> &qnodes, std::vector<uint8_t> &primsc, uint32_t &n4,
                 uint32_t &depth4) {
    qnodes.clear();
    primsc.clear();
    n4 = depth4 = 0;
    if (b2.n_nodes == 0 || b2.n_prims >= (1u << 26)) return false;
    QBuild qb;
    qb.n2 = reinterpret_cast<const Node *>(b2.nodes.data());
    qb.cn.reserve(b2.n_nodes / 2 + 1);
    qb.collapse(0, 1);
    const uint32_t n = (uint32_t)qb.cn.size();
    // children-contiguous depth-first order: the root, then each node's inner
    // children as one group, then the groups below the first child, ...
    std::vector<uint32_t> pos(n, ~0u);
    pos[0] = 0;
    uint32_t next = 1;
    std::vector<uint32_t> todo{0};   // nodes whose children are not placed yet (a stack: depth first)
    while (!todo.empty()) {
        const uint32_t c = todo.back();
        todo.pop_back();
        const QBuild::CNode &x = qb.cn[c];
        for (int j = 0; j < x.k; ++j)
            if (x.child[j] != ~0u) pos[x.child[j]] = next++;
        for (int j = x.k - 1; j >= 0; --j)
            if (x.child[j] != ~0u) todo.push_back(x.child[j]);
    }
    std::vector<QNode4> out(n);
    for (uint32_t c = 0; c < n; ++c) {
        const QBuild::CNode &x = qb.cn[c];
        QNode4 q;
        memset(&q, 0, sizeof(q));
        float o[3];
        for (int a = 0; a < 3; ++a) {
            o[a] = FLT_MAX;
            for (int j = 0; j < x.k; ++j) o[a] = std::min(o[a], x.e[j].lo[a]);
        }
        uint32_t eb[3];
        uint8_t ql[3][4] = {}, qh[3][4] = {};
        for (int a = 0; a < 3; ++a) {
            float lo[4], hi[4];
            for (int j = 0; j < x.k; ++j) { lo[j] = x.e[j].lo[a]; hi[j] = x.e[j].hi[a]; }
            if (!quantise_axis(o[a], lo, hi, x.k, eb[a], ql[a], qh[a])) return false;
        }
        q.ox = o[0]; q.oy = o[1]; q.oz = o[2];
        q.ebits = eb[0] | eb[1] << 8 | eb[2] << 16;
        uint32_t lo32[3] = {0, 0, 0}, hi32[3] = {0, 0, 0};
        uint32_t ref[4];
        for (int j = 0; j < 4; ++j) {
            if (j >= x.k) { ref[j] = kEmptyRef; continue; }   // empty slot: rejected by its ref
            for (int a = 0; a < 3; ++a) {
                lo32[a] |= (uint32_t)ql[a][j] << (8 * j);
                hi32[a] |= (uint32_t)qh[a][j] << (8 * j);
            }
            const Entry &e = x.e[j];
            ref[j] = e.inner == ~0u ? (kLeafRef | (e.first << 5) | e.count) : pos[x.child[j]];
        }
        q.qlo[0] = lo32[0]; q.qlo[1] = lo32[1]; q.qlo[2] = lo32[2];
        q.qhi_x = hi32[0]; q.qhi_y = hi32[1]; q.qhi_z = hi32[2];
        for (int j = 0; j < 4; ++j) q.ref[j] = ref[j];
        out[pos[c]] = q;
    }
    // compact primitive records, same (leaf) order as Prim
    const Prim *P = reinterpret_cast<const Prim *>(b2.prims.data());
    std::vector<PrimC> pc(b2.n_prims);
    for (uint32_t i = 0; i < b2.n_prims; ++i) {
        PrimC &r = pc[i];
        memset(&r, 0, sizeof(r));
        const Prim &p = P[i];
        r.v0x = p.a.x; r.v0y = p.a.y; r.v0z = p.a.z;
        r.e1x = p.b.x; r.e1y = p.b.y; r.e1z = p.b.z;
        r.e2x = p.c.x; r.e2y = p.c.y; r.e2z = p.c.z;
        r.key = p.info.w;
        r.prim = p.info.y;
        r.shape = p.info.x | (p.info.z == MH_SHAPE_RECTANGLE ? kPrimCRect : 0u);
    }
    n4 = n;
    depth4 = qb.depth;
    qnodes.resize(sizeof(QNode4) * n);
    memcpy(qnodes.data(), out.data(), qnodes.size());
    primsc.resize(sizeof(PrimC) * pc.size());
    memcpy(primsc.data(), pc.data(), primsc.size());
    return true;
}

}  // namespace mh
