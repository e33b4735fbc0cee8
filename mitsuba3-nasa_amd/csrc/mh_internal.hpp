// mh_internal.hpp — declarations shared by the host API (mh_api.hip), the BVH
// builder (mh_bvh.cpp) and the kernels (mh_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/mitsuba_hip.h"

namespace mh {

struct DScene;
struct Node;
struct Prim;
struct LaneMap;

using IntegratorParams = mh_integrator;

constexpr int kMaxRgbParams = 4;     // constant-albedo gradient slots (register accumulators)
constexpr int kMaxBitmapParams = 4;  // bitmap gradient slots (global atomics)
constexpr int kMaxParams = kMaxRgbParams + kMaxBitmapParams;

struct GradArgs {
    const int32_t *slot_of_tex;  // device: texture -> slot or -1
    float *const *bufs;          // device: slot -> gradient buffer
    const uint32_t *is_rgb;      // device: slot -> 1 if rgb
    uint32_t n_rgb;              // small (register-accumulated) slots are 0 .. n_rgb-1:
                                 // rgb textures, medium albedo, homogeneous sigma_t
    const int32_t *sigma_slot;   // device: medium -> sigma_t slot or -1 (prbvolpath)
    const int32_t *albedo_slot;  // device: medium -> albedo slot or -1 (prbvolpath)
    int32_t lds_slot = -1;       // bitmap slot accumulated per workgroup in LDS (k_prb_backward replay)
    uint32_t lds_floats = 0;     // its size (floats)
    uint32_t lds_offset = 0;     // byte offset of the accumulator in dynamic LDS (set by the launcher)
    float *const *corner = nullptr;  // device: slot -> per-cell corner block of a grid sigma_t slot or nullptr
                                     // (prbvolpath; gathered into bufs[slot] by launch_corner_gather)
    // MH_FLAG_DETERMINISTIC on the corner blocks: 1 = pre-pass (the largest |item| into fx_max, no
    // scatter), 2 = int64 fixed-point adds of round(item * fx_scale) (order-independent sums)
    uint32_t fx_mode = 0;
    uint32_t *fx_max = nullptr;
    double fx_scale = 0.0;
    // MH_FLAG_DETERMINISTIC on the replay kernel: bitmap texel sums as int64,
    // element i of the slot block (s->tmp_c) at fx_i64[i] (fx_f32 = the block)
    long long *fx_i64 = nullptr;
    const float *fx_f32 = nullptr;
    // the first medium with a parameter, its slots and buffers as values
    // (prbvolpath): the scatter loops of its gradient read them from
    // registers instead of loading sigma_slot / corner / bufs entries, whose
    // vector loads waited (vmcnt) for the loop's outstanding atomics
    int32_t hot_med = -1;      // medium index (-1: none)
    int32_t hot_sigma = -1;    // its sigma_t slot (-1: none)
    int32_t hot_albedo = -1;   // its albedo slot (-1: none)
    float *hot_buf = nullptr;    // bufs[hot_sigma]
    float *hot_corner = nullptr; // corner[hot_sigma] (nullptr: atomics into hot_buf)
};

// ---- BVH builder (host, binned SAH) --------------------------------------
struct BuildPrim {
    float lo[3], hi[3];   // world AABB
    float rec[12];        // Prim a/b/c payload
    uint32_t shape, prim, type;
};
struct BvhOut {
    std::vector<uint8_t> nodes;  // sizeof(Node) * n_nodes
    std::vector<uint8_t> prims;  // sizeof(Prim) * n_prims (reordered)
    uint32_t n_nodes = 0, n_prims = 0, depth = 0;
};
// max_leaf <= 31 (5-bit leaf count of the per-lane stream engine's stack entries)
void build_bvh(const std::vector<BuildPrim> &in, BvhOut &out, uint32_t max_leaf = 4, float trav_cost = 1.0f);
// BVH4 collapsed from a BVH2 (greedy: open the largest-area inner child until
// four children); depth4 = max Node4 nesting
void collapse_bvh4(const BvhOut &b2, std::vector<uint8_t> &nodes4, uint32_t &n4, uint32_t &depth4);
// the same BVH4 quantised (QNode4, children-contiguous order) + compact
// primitive records (PrimC); false when a box cannot be quantised
bool build_qbvh4(const BvhOut &b2, std::vector<uint8_t> &qnodes, std::vector<uint8_t> &primsc, uint32_t &n4,
                 uint32_t &depth4);

// ---- kernel launchers (mh_kernels.hip) -------------------------------------
size_t lds_bytes(const DScene &S, uint32_t block);
hipError_t launch_trace(const DScene &S, bool shadow, uint64_t n, const float *rays, float *t,
                        float *u, float *v, uint32_t *prim, uint32_t *shape, uint32_t *inst, uint32_t *occ,
                        uint32_t grid, hipStream_t st);
hipError_t launch_render(const DScene &S, const IntegratorParams &in, const LaneMap &lm,
                         uint32_t seed_value, uint32_t n_passes, uint64_t n, uint64_t plane,
                         float *out, unsigned long long *counters, hipStream_t st, int alpha = 0);
// splat modes: RGBW film from (L, pos) planes; W image from the RNG jitter;
// alpha channel from (alpha, pos) planes (plane 5)
enum { kSplatFilm = 0, kSplatWeights = 1, kSplatAlpha = 2 };
// invalid: counts samples with a non-finite or negative radiance channel
// (mode 0; ImageBlock::put's warn_invalid / warn_negative test); deterministic:
// the fast path as a fixed-order gather (k_splat_gather) instead of atomics
hipError_t launch_splat(const DScene &S, const LaneMap &lm, int mode, bool fast,
                        uint32_t n_pix, uint32_t n_passes, uint64_t n, uint64_t plane,
                        const float *in, float *film, uint32_t seed_value, int coalesce,
                        hipStream_t st, unsigned long long *invalid, bool deterministic, uint64_t in_floats,
                        uint64_t film_floats, unsigned long long *viol);
hipError_t launch_film_rgbaw(uint64_t n_px, const float *rgbw, const float *a, float *out, hipStream_t st);
size_t wf_workspace_bytes(uint64_t cap);
uint32_t wf_counter_words(uint32_t n_bounces);
uint64_t wf_max_chunk();
hipError_t launch_wavefront(const DScene &S, const IntegratorParams &in, const LaneMap &lm,
                            uint32_t seed_value, uint64_t n, uint64_t plane, float *out, void *ws,
                            uint64_t cap, uint32_t *ctr, uint32_t n_bounces, uint32_t grid,
                            hipEvent_t *trace_ev, hipStream_t st, uint32_t n_passes = 1,
                            uint64_t *carry = nullptr,   // carry: n PCG32 states (n_passes > 1)
                            int alpha = 0);              // alpha: write the validity plane (plane 5)
size_t wf_prb_workspace_bytes(uint64_t cap);
uint32_t wf_grid(uint32_t grid);
uint32_t wf_blocks(int cus, bool shared = false);  // wavefront workgroups for a device of `cus` CUs (shared: another call runs beside)
uint32_t wf_packet_max_prims();  // largest scene (primitives) the packet engine traces
bool wf_fused(const DScene &S);  // launch_wavefront runs the fused bounce kernel  // grid rounded to whole queue segments
// One bitmap parameter on the fused PRB wavefront: the bounce kernel logs a
// record per bitmap vertex, a scatter pass turns the records into texel
// gradients once the chunk's paths have ended (mh_wavefront.hip).
struct WfBitmapArgs {
    void *ws = nullptr;      // wf_bmp_workspace_bytes(cap, n_depth)
    uint32_t n_depth = 0;    // vertex records per path: max_depth - 1
    int32_t slot = -1;       // the first bitmap gradient slot (kMaxRgbParams; -1: none)
    uint32_t tex[kMaxBitmapParams] = {};  // texture of bitmap slot kMaxRgbParams + b
    uint32_t off[kMaxBitmapParams] = {};  // its gradient's float offset in grad
    float *grad = nullptr;   // the bitmap slots' block of gradient buffers (device)
    uint32_t n_floats = 0;   // that block's floats (texels x channels, padded per slot)
    uint32_t lds_max = 0;    // per-workgroup LDS accumulation when n_floats * 4 <= lds_max
    uint32_t wg_lds = 0;     // the device's LDS bytes per workgroup and per CU
    uint32_t cu_lds = 0;
    uint32_t cus = 0;        // the scatter's persistent grid: cus x the accumulators a CU holds
    // MH_FLAG_DETERMINISTIC: int64 sums (n_floats) and the max word of the
    // fixed-point scatter (nullptr: float atomics)
    unsigned long long *fx_acc = nullptr;
    uint32_t *fx_word = nullptr;
    unsigned long long *n_rec = nullptr;  // += the vertex records the scatter reads (mh_stats.aux_items)
};
size_t wf_bmp_workspace_bytes(uint64_t cap, uint32_t n_depth);
hipError_t launch_wavefront_prb(const DScene &S, const IntegratorParams &in, const LaneMap &lm,
                                uint32_t seed_value, uint64_t n, int coalesce, const float *grad_in,
                                const float *weights, const int32_t *slot_of_tex, uint32_t n_rgb,
                                void *ws, void *ws_prb, uint64_t cap, uint32_t *ctr, uint32_t n_bounces,
                                uint32_t grid, float *partial, hipStream_t st,
                                hipEvent_t *span = nullptr,               // span: 2 events around the bounce launches
                                const WfBitmapArgs *bmp = nullptr,       // the bitmap parameters (or none)
                                void *ws_det = nullptr);                 // deterministic rgb gradients (or none)
size_t wf_det_workspace_bytes(uint64_t cap);
// render_forward of `prb` on the fused wavefront (packet-engine scenes): the
// tangent radiance of every path written to the sample planes of launch_render
hipError_t launch_wavefront_fwd(const DScene &S, const IntegratorParams &in, const LaneMap &lm, uint32_t seed_value,
                                uint64_t n, const int32_t *slot_of_tex, float *const *tangents,
                                const uint32_t *is_rgb, float *out, uint64_t plane, int alpha, void *ws,
                                void *ws_prb, uint64_t cap, uint32_t *ctr, uint32_t n_bounces, uint32_t grid,
                                hipStream_t st);
hipError_t launch_wf_grad_reduce(const float *partial, uint32_t grid, uint32_t n_rgb, float *const *bufs,
                                 hipStream_t st);
// max of a float array (gridvolume max for the majorant), as an order-preserving
// uint key in *key (initialised by the launcher)
hipError_t launch_grid_max(const float *data, uint64_t n, uint32_t *key, hipStream_t st);
inline float ordered_key_to_float(uint32_t k) {
    union { uint32_t u; float f; } c;
    c.u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
    return c.f;
}
// linear (z, y, x) grid -> 4^3-brick device layout (grid_index, mh_shading.hpp)
uint64_t grid_bricked_size(const uint32_t res[3]);
void grid_to_bricks(const float *src, const uint32_t res[3], float *dst);
hipError_t launch_grid_to_bricks(const float *src, const uint32_t res[3], float *dst, hipStream_t st);
hipError_t launch_accumulate(float *dst, const float *src, uint64_t n, hipStream_t st);  // dst += src
// grid sigma_t gradient: per-cell corner block (GradArgs::corner) -> (z, y, x) gradient (+=)
uint64_t corner_floats(const uint32_t res[3]);
hipError_t launch_corner_gather(const float *corner, float *grad, const uint32_t res[3], hipStream_t st);
// the int64 fixed-point form (fx_mode 2): grad += (float)(exact integer sum / fx_scale)
hipError_t launch_corner_gather_fx(const long long *corner, float *grad, const uint32_t res[3], double inv_scale,
                                   hipStream_t st);
// deterministic bitmap texels of the replay kernel (GradArgs::fx_i64): grad += (float)(fx / scale)
hipError_t launch_fx_to_float(const long long *fx, float *grad, uint64_t n, double inv_scale, hipStream_t st);
hipError_t launch_grad_over_w(uint64_t n_px, const float *grad_in, const float *w, float *out, hipStream_t st);
#ifdef MH_DEBUG
hipError_t guard_read_wf(unsigned long long *out);  // kGuardCount words each, read and reset
hipError_t guard_read_k(unsigned long long *out);
#endif
hipError_t launch_develop(uint64_t n_px, const float *film, float *rgb, uint32_t fmt, hipStream_t st);
hipError_t launch_prb_backward(const DScene &S, const IntegratorParams &in, const LaneMap &lm,
                               uint32_t seed_value, uint64_t n, int coalesce,
                               const float *grad_in, const float *weights, const GradArgs &ga,
                               bool fused, unsigned long long *counters, hipStream_t st,
                               // prbvolpath: NEE-walk logs ([cap][nee_blocks * 256] float4) on a
                               // persistent grid of nee_blocks pulling work from *head (nullptr: none)
                               float4 *nee_log = nullptr, uint32_t nee_cap = 0, uint32_t nee_blocks = 0,
                               unsigned long long *head = nullptr,
                               // + single pass: per-thread MainLog ([4 main_cap][threads] float4)
                               float4 *main_log = nullptr, uint32_t main_cap = 0);
// render_forward: per-sample tangent radiance (L, pos[, alpha] planes of launch_render); ga.bufs = tangents
hipError_t launch_render_forward(const DScene &S, const IntegratorParams &in, const LaneMap &lm,
                                 uint32_t seed_value, uint64_t n, uint64_t plane, float *out, const GradArgs &ga,
                                 unsigned long long *counters, hipStream_t st, int alpha);
// wavefront volpath (mh_volwave.hip): k_vw_main / k_vw_walk rounds
uint64_t vw_max_chunk();
size_t vw_workspace_bytes(uint64_t cap);
uint32_t vw_counter_words(uint32_t rounds);
uint32_t vw_rounds(const IntegratorParams &in);
bool vw_supported(const DScene &S, const IntegratorParams &in);
bool vs_supported(const DScene &S, const IntegratorParams &in);
uint32_t vw_blocks(int cus);
bool vol_sched_mode();
uint32_t vs_blocks(int cus);
hipError_t launch_vol_sched(const DScene &S, const IntegratorParams &in, const LaneMap &lm, uint32_t seed_value,
                            uint64_t n, uint64_t plane, float *out, uint32_t grid, unsigned long long *counters,
                            hipStream_t st, int alpha);
// prbvolpath's single-pass backward on the phase scheduler (mh_volwave.hip
// PvBwdMachine): the kernel-wide inputs
struct VsBwdArgs {
    const float *grad_in = nullptr;  // grad_in / W, one float4 per pixel (k_grad_over_w)
    int coalesce = 0;
    GradArgs ga{};
    float4 *main_log = nullptr;      // MainLog: [grid threads][main_cap][4] (contiguous per lane)
    float4 *nee_log = nullptr;       // NeeLog: [grid threads][nee_cap]
    uint32_t main_cap = 0, nee_cap = 0;
    // overflow lists, replayed after the scheduler launch: paths whose MainLog
    // overflowed (2 float4: L + pid, dL) and NEE walks whose NeeLog overflowed
    // (kPvbWalkRec float4), at most ovf_cap entries each; ovf_count: [0]
    // paths, [1] walks, [2] entries that found their list full (fails the call)
    float4 *ovf_paths = nullptr;
    float4 *ovf_walks = nullptr;
    uint32_t *ovf_count = nullptr;
    uint32_t ovf_cap = 0;
};
constexpr uint32_t kPvbWalkRec = 5;
hipError_t launch_vol_sched_bwd(const DScene &S, const IntegratorParams &in, const LaneMap &lm, uint32_t seed_value,
                                uint64_t n, const VsBwdArgs &bw, uint32_t grid, unsigned long long *counters,
                                hipStream_t st);
// the replays of bw's overflow lists (after launch_vol_sched_bwd on the same stream)
hipError_t launch_vol_sched_bwd_replays(const DScene &S, const IntegratorParams &in, const LaneMap &lm,
                                        uint32_t seed_value, uint64_t n, const VsBwdArgs &bw,
                                        unsigned long long *counters, hipStream_t st);
hipError_t launch_volwave(const DScene &S, const IntegratorParams &in, const LaneMap &lm, uint32_t seed_value,
                          uint64_t n, uint64_t plane, float *out, void *ws, uint64_t cap, uint32_t *ctr,
                          uint32_t grid, unsigned long long *counters, hipStream_t st, int alpha);

}  // namespace mh

// ---- shared by mh_api.hip and mh_comm.cpp (global namespace, C-ABI side) ----
// sets mh_last_error() of the calling thread and returns `code`
int mh_report_error(int code, const std::string &msg);
// one rank's in-call sum over its communicator (root < 0: all-reduce), stream-ordered on st
int comm_reduce_one(mh_comm *c, int device, float *buf, uint64_t count, hipStream_t st, int root);
// wait for st with a deadline, watching the communicator's async error (aborts it on a failure)
int comm_wait(mh_comm *c, hipStream_t st, const char *api);
// abort after a failed collective call (later collectives on it fail at once)
void comm_abort(mh_comm *c);
// scenes holding the communicator (mh_comm_destroy refuses while > 0)
void comm_attach(mh_comm *c, int delta);
