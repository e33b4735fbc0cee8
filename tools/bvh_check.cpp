// Host check / timing of the binned-SAH BVH builder (mh_bvh.cpp) on a
// synthetic triangle soup: every primitive in exactly one leaf, every child
// box containing its subtree, and a hash of the node + primitive arrays (the
// same for any MH_BVH_THREADS).  usage: bvh_check <n_tris> [seed]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../mitsuba3-nasa_amd/csrc/mh_device.hpp"
#include "../mitsuba3-nasa_amd/csrc/mh_internal.hpp"

using namespace mh;

static bool inside(const float4 &lo, const float4 &hi, const float *l, const float *h) {
    return lo.x <= l[0] && lo.y <= l[1] && lo.z <= l[2] && hi.x >= h[0] && hi.y >= h[1] && hi.z >= h[2];
}

int main(int argc, char **argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 1000000u;
    std::mt19937 rng(argc > 2 ? atoi(argv[2]) : 1);
    std::uniform_real_distribution<float> U(-1.f, 1.f), S(0.f, 0.01f);
    std::vector<BuildPrim> prims(n);
    for (uint32_t i = 0; i < n; ++i) {
        // clustered: a quarter of the triangles in a small blob (uneven SAH splits)
        const float sc = (i % 4 == 0) ? 0.05f : 1.f;
        float c[3] = {U(rng) * sc, U(rng) * sc, U(rng) * sc};
        BuildPrim &p = prims[i];
        for (int a = 0; a < 3; ++a) {
            const float d = S(rng);
            p.lo[a] = c[a] - d;
            p.hi[a] = c[a] + d;
        }
        for (int k = 0; k < 12; ++k) p.rec[k] = (float)(i * 12 + k);
        p.shape = 0;
        p.prim = i;
        p.type = MH_SHAPE_MESH;
    }
    BvhOut out;
    const auto t0 = std::chrono::steady_clock::now();
    build_bvh(prims, out, 4, 1.0f);
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    const Node *nodes = reinterpret_cast<const Node *>(out.nodes.data());
    const Prim *pr = reinterpret_cast<const Prim *>(out.prims.data());
    std::vector<int> seen(n, 0);
    int bad = 0;
    // walk from the root: each child box must contain every primitive below it
    std::vector<std::pair<uint32_t, int>> stack{{0u, 0}};
    uint64_t leaves = 0;
    std::vector<uint32_t> st{0};
    while (!st.empty()) {
        const uint32_t ni = st.back();
        st.pop_back();
        const Node &nd = nodes[ni];
        const float4 *lo[2] = {&nd.lo0, &nd.lo1}, *hi[2] = {&nd.hi0, &nd.hi1};
        for (int c = 0; c < 2; ++c) {
            uint32_t w, cnt;
            memcpy(&w, &lo[c]->w, 4);
            memcpy(&cnt, &hi[c]->w, 4);
            cnt &= kLeafCountMask;
            if (cnt) {
                ++leaves;
                for (uint32_t j = w; j < w + cnt; ++j) {
                    const uint32_t id = pr[j].info.w;
                    if (id >= n || !inside(*lo[c], *hi[c], prims[id].lo, prims[id].hi)) ++bad;
                    else seen[id]++;
                }
            } else {
                if (w >= out.n_nodes) { ++bad; continue; }
                st.push_back(w);
            }
        }
    }
    for (uint32_t i = 0; i < n; ++i) bad += seen[i] != (n == 1 ? 2 : 1);  // one primitive: two identical leaves
    uint64_t h = 1469598103934665603ull;
    for (uint8_t b : out.nodes) h = (h ^ b) * 1099511628211ull;
    for (uint8_t b : out.prims) h = (h ^ b) * 1099511628211ull;
    printf("{\"n\": %u, \"ms\": %.1f, \"nodes\": %u, \"leaves\": %llu, \"depth\": %u, \"bad\": %d, \"hash\": \"%016llx\"}\n",
           n, ms, out.n_nodes, (unsigned long long)leaves, out.depth, bad, (unsigned long long)h);
    return bad ? 1 : 0;
}
