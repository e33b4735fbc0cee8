// mh_api.hip — C-ABI of the MI355X backend (include/mitsuba_hip.h).
//
// Host orchestration only: scene upload, BVH build, chunked launch of the
// render / splat / develop / PRB kernels on the scene's HIP stream.  There is
// no CPU fallback: every compute entry point requires a HIP device and fails
// with MH_ERR_NO_DEVICE otherwise.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include <rocprofiler-sdk-roctx/roctx.h>

#include "mh_device.hpp"
#include "mh_internal.hpp"
#include "mh_shading.hpp"

// The reference's ProfilerPhase scopes (include/mitsuba/core/profiler.h:20-47,
// ScopedPhase -> ITT / NVTX ranges at :81-110) as roctx ranges around the host
// stages (rocprofv3 --marker-trace shows them beside the kernels).
struct ScopedPhase {
    explicit ScopedPhase(const char *name) { roctxRangePushA(name); }
    ~ScopedPhase() { roctxRangePop(); }
    ScopedPhase(const ScopedPhase &) = delete;
    ScopedPhase &operator=(const ScopedPhase &) = delete;
};

using namespace mh;

namespace {

thread_local std::string g_error;
thread_local bool g_call_issued = false;  // the current entry point has passed its argument checks

int set_error(int code, const std::string &msg) {
    g_error = msg;
    return code;
}

// a wait that failed in comm_wait has already reported why (a collective
// failed, its deadline passed, the communicator was aborted): MH_HIP keeps
// that message instead of replacing it by the HIP code's text
thread_local bool g_keep_error = false;

#define MH_HIP(expr)                                                                        \
    do {                                                                                    \
        hipError_t _e = (expr);                                                             \
        if (_e != hipSuccess) {                                                             \
            if (g_keep_error) {                                                             \
                g_keep_error = false;                                                       \
                return MH_ERR_HIP;                                                          \
            }                                                                               \
            return set_error(MH_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
        }                                                                                   \
    } while (0)

struct DevBuf {
    void *ptr = nullptr;
    size_t bytes = 0;
    hipError_t alloc(size_t n) {
        if (n <= bytes && ptr) return hipSuccess;
        if (ptr) (void)hipFree(ptr);
        ptr = nullptr;
        bytes = 0;
        if (n == 0) return hipSuccess;
        hipError_t e = hipMalloc(&ptr, n);
        if (e == hipSuccess) bytes = n;
        return e;
    }
    void release() {
        if (ptr) (void)hipFree(ptr);
        ptr = nullptr;
        bytes = 0;
    }
    template <typename T> T *as() const { return reinterpret_cast<T *>(ptr); }
};

uint32_t log2_exact(uint32_t v) {
    for (uint32_t k = 0; k < 32; ++k)
        if ((1u << k) == v) return k;
    return 32;
}

template <typename T>
hipError_t upload(DevBuf &b, const T *src, size_t count, hipStream_t st) {
    size_t bytes = sizeof(T) * count;
    if (bytes == 0) bytes = 16;  // keep a valid pointer
    hipError_t e = b.alloc(bytes);
    if (e != hipSuccess) return e;
    if (src && count) return hipMemcpyAsync(b.ptr, src, sizeof(T) * count, hipMemcpyHostToDevice, st);
    return hipMemsetAsync(b.ptr, 0, bytes, st);
}

}  // namespace

int mh_report_error(int code, const std::string &msg) { return set_error(code, msg); }

struct mh_scene {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    DScene S{};
    // device buffers
    DevBuf nodes, nodes4, primsc, stack_ovf, prims, prim_pairs, key_sp, shapes, bsdf_type, bsdf_tex, textures, emitters, positions, normals,
        texcoords, faces, texels, media, grid;
    DevBuf work, film_tmp, film4, alpha_px, counters, grad_meta, tmp_a, tmp_b, tmp_c, tmp_d, tmp_e, weights_tmp;
    std::vector<uint8_t> meta_host;  // the bytes last uploaded to grad_meta (upload_slots)
    DevBuf wf_ws, wf_ctr;  // wavefront state (SoA) and per-chunk/bounce queue counters
    DevBuf wf_ws_prb, wf_partial, gw, wf_carry;  // wavefront PRB: dL / adjoint-factor planes, per-block gradient partials
    DevBuf wf_ws_bmp;  // wavefront PRB with a bitmap parameter: vertex records (WfBmp)
    DevBuf wf_ws_det;  // wavefront PRB, MH_FLAG_DETERMINISTIC: per-path gradient sums (WfDet)
    DevBuf pvp_log;    // prbvolpath backward: per-thread NEE-walk step logs (NeeLog)
    DevBuf pvp_main;   // prbvolpath backward: per-thread path logs of the single pass (MainLog)
    DevBuf pvp_ovf;    // prbvolpath backward on the scheduler: overflow lists + their counters
    DevBuf grid_corner;  // prbvolpath backward: per-cell corner blocks of the grid sigma_t slots
    DevBuf fx_word;      // its deterministic pre-pass: the largest |item| (float bits)
    DevBuf bmp_fx;       // the deterministic bitmap scatter's max word + int64 texel sums
    DevBuf replay_fx;    // the deterministic replay kernel: int64 mirror of the slot block (bitmap texels)
    // multi-GPU: the communicator of MH_FLAG_REDUCE (not owned), and the
    // buffers of the sharded entry points (slab W image, staged peer sums,
    // slab gradients)
    mh_comm *comm = nullptr;
    DevBuf shard_w, shard_tmp, shard_g;
    // host mirrors (parameter updates)
    std::vector<DTexture> h_textures;
    std::vector<mh_medium> h_media;
    std::vector<DMedium> h_dmedia;
    uint32_t n_textures = 0, n_bsdfs = 0, n_shapes = 0, n_media = 0, pixel_format = MH_PIXEL_RGB;
    uint64_t n_texels = 0;
    uint32_t bvh_nodes = 0, bvh_prims = 0, bvh_depth = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    std::vector<hipEvent_t> evpool;  // per-chunk timing events of mh_render
    // two-stream chunk pipeline of the bitmap PRB wavefront (fork_stream): odd
    // chunks run on stream2 with their own workspace
    hipStream_t stream2 = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    DevBuf wf_ws2, wf_ws_prb2, wf_ws_bmp2, wf_partial2, work2, wf_carry2;
    DevBuf stack_ovf2;  // the stream engine's stack overflow columns of stream2's launches
};

extern "C" {

const char *mh_last_error(void) { return g_error.c_str(); }
uint32_t mh_abi_version(void) { return MH_ABI_VERSION; }

int mh_device_count(int *count) {
    if (!count) return set_error(MH_ERR_INVALID_ARGUMENT, "mh_device_count: count is NULL");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    *count = n;
    return MH_OK;
}

static int require_device(int device) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
        return set_error(MH_ERR_NO_DEVICE,
                         "mitsuba_hip: no HIP device available (hip_ad_rgb requires an MI355X; "
                         "there is no CPU fallback)");
    if (device < 0 || device >= n)
        return set_error(MH_ERR_INVALID_ARGUMENT, "mh_scene_create: device index out of bounds");
    return MH_OK;
}


int mh_scene_create(const mh_scene_desc *desc, int device, void *stream, mh_scene **out) {
    ScopedPhase phase_("InitScene");
    if (!desc || !out) return set_error(MH_ERR_INVALID_ARGUMENT, "mh_scene_create: NULL argument");
    if (desc->abi_version != MH_ABI_VERSION)
        return set_error(MH_ERR_INVALID_ARGUMENT, "mh_scene_create: ABI version mismatch");
    int rc = require_device(device);
    if (rc) return rc;
    const mh_sensor &sn = desc->sensor;
    if (sn.width == 0 || sn.height == 0)
        return set_error(MH_ERR_INVALID_ARGUMENT, "mh_scene_create: film size must be positive");
    for (uint32_t i = 0; i < desc->n_emitters; ++i) {
        const mh_emitter &e = desc->emitters[i];
        if (e.type == MH_EMITTER_AREA &&
            (e.shape >= desc->n_shapes || desc->shapes[e.shape].type != MH_SHAPE_RECTANGLE))
            return set_error(MH_ERR_UNSUPPORTED,
                             "mh_scene_create: area emitters are supported on rectangles only");
    }
    MH_HIP(hipSetDevice(device));
    mh_scene *s = new (std::nothrow) mh_scene();
    if (!s) return set_error(MH_ERR_OUT_OF_MEMORY, "mh_scene_create: out of host memory");
    s->device = device;
    if (stream) {
        s->stream = (hipStream_t)stream;
    } else {
        if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess) {
            delete s;
            return set_error(MH_ERR_HIP, "mh_scene_create: hipStreamCreate failed");
        }
        s->own_stream = true;
    }
    hipStream_t st = s->stream;
    auto fail = [&](int code, const std::string &m) {
        mh_scene_destroy(s);
        return set_error(code, m);
    };

    // ---- primitives for the BVH (rectangles + mesh triangles) ----
    std::vector<BuildPrim> bp;
    for (uint32_t si = 0; si < desc->n_shapes; ++si) {
        const mh_shape &sh = desc->shapes[si];
        if (sh.type == MH_SHAPE_RECTANGLE) {
            BuildPrim p{};
            const float *m = sh.to_world;
            for (int a = 0; a < 3; ++a) { p.lo[a] = INFINITY; p.hi[a] = -INFINITY; }
            const float cs[4][2] = {{-1, -1}, {-1, 1}, {1, -1}, {1, 1}};
            for (auto &c : cs) {
                for (int a = 0; a < 3; ++a) {
                    float q = m[4 * a + 0] * c[0] + m[4 * a + 1] * c[1] + m[4 * a + 3];
                    p.lo[a] = std::min(p.lo[a], q);
                    p.hi[a] = std::max(p.hi[a], q);
                }
            }
            memcpy(p.rec, sh.to_object, sizeof(float) * 12);
            p.shape = si;
            p.prim = MH_INVALID;
            p.type = MH_SHAPE_RECTANGLE;
            bp.push_back(p);
        } else if (sh.type == MH_SHAPE_MESH) {
            if ((uint64_t)sh.face_offset + sh.face_count > desc->n_faces ||
                (uint64_t)sh.vertex_offset + sh.vertex_count > desc->n_vertices)
                return fail(MH_ERR_INVALID_ARGUMENT, "mh_scene_create: mesh range out of bounds");
            for (uint32_t f = 0; f < sh.face_count; ++f) {
                const uint32_t *fi = desc->faces + 3ull * (sh.face_offset + f);
                const float *v[3];
                for (int k = 0; k < 3; ++k) {
                    if (fi[k] >= sh.vertex_count)
                        return fail(MH_ERR_INVALID_ARGUMENT, "mh_scene_create: face index out of bounds");
                    v[k] = desc->positions + 3ull * (sh.vertex_offset + fi[k]);
                }
                BuildPrim p{};
                for (int a = 0; a < 3; ++a) {
                    p.lo[a] = std::min(v[0][a], std::min(v[1][a], v[2][a]));
                    p.hi[a] = std::max(v[0][a], std::max(v[1][a], v[2][a]));
                    p.rec[a] = v[0][a];
                    p.rec[4 + a] = v[1][a] - v[0][a];  // e1 (mesh.h:437)
                    p.rec[8 + a] = v[2][a] - v[0][a];  // e2
                }
                p.shape = si;
                p.prim = f;
                p.type = MH_SHAPE_MESH;
                bp.push_back(p);
            }
        } else {
            return fail(MH_ERR_UNSUPPORTED, "mh_scene_create: unknown shape type");
        }
    }
    BvhOut bvh;
    {
        // Leaf size / SAH traversal cost per engine (measured, tools/exp_bvh_leaf.sh):
        // small scenes take the packet engine, where a wave tests every leaf some
        // lane reaches and node visits are the serial part -> few, large leaves
        // (12, C_t = 4); otherwise the per-lane engine (8, C_t = 2).  Leaf counts
        // <= 31 (5-bit field of the stream engine's stack entries); env overrides.
        const bool small = bp.size() <= 64;
        const char *el = getenv("MH_BVH_LEAF"), *ec = getenv("MH_BVH_CT");
        uint32_t max_leaf = el ? (uint32_t)std::max(2, std::min(31, atoi(el))) : (small ? 12u : 8u);
        float ct = ec ? (float)atof(ec) : (small ? 4.0f : 2.0f);
        ScopedPhase accel_("InitAccel");
        build_bvh(bp, bvh, max_leaf, ct);
    }
    s->bvh_nodes = bvh.n_nodes;
    s->bvh_prims = bvh.n_prims;
    s->bvh_depth = bvh.depth;
    // scene-order key -> (shape, prim) of every primitive (the packet engine
    // carries only the key of its running hit)
    std::vector<uint32_t> key_sp(2 * (size_t)bvh.n_prims);
    for (uint32_t i = 0; i < bvh.n_prims; ++i) {
        const Prim &q = reinterpret_cast<const Prim *>(bvh.prims.data())[i];
        key_sp[2 * (size_t)q.info.w] = q.info.x;
        key_sp[2 * (size_t)q.info.w + 1] = q.info.y;
    }
    // pair records of the packet engine: record i interleaves the dwords of
    // leaf-ordered primitives i and i + 1 (the last one with itself); only
    // scenes small enough for that engine (wf_packet_max_prims) get them
    std::vector<uint32_t> pairs(bvh.n_prims <= wf_packet_max_prims() ? 32 * (size_t)bvh.n_prims : 0);
    for (uint32_t i = 0; i < pairs.size() / 32; ++i) {
        const uint32_t *a = reinterpret_cast<const uint32_t *>(bvh.prims.data()) + 16 * (size_t)i;
        const uint32_t *b = reinterpret_cast<const uint32_t *>(bvh.prims.data()) + 16 * (size_t)std::min(i + 1, bvh.n_prims - 1);
        for (int k = 0; k < 16; ++k) {
            pairs[32 * (size_t)i + 2 * k] = a[k];
            pairs[32 * (size_t)i + 2 * k + 1] = b[k];
        }
    }
    if (upload(s->nodes, bvh.nodes.data(), bvh.nodes.size(), st) != hipSuccess ||
        upload(s->prim_pairs, pairs.data(), pairs.size(), st) != hipSuccess ||
        upload(s->prims, bvh.prims.data(), bvh.prims.size(), st) != hipSuccess ||
        upload(s->key_sp, key_sp.data(), key_sp.size(), st) != hipSuccess)
        return fail(MH_ERR_OUT_OF_MEMORY, "mh_scene_create: BVH upload failed");

    // ---- shading-time records ----
    std::vector<DShape> shapes(desc->n_shapes);
    for (uint32_t i = 0; i < desc->n_shapes; ++i) {
        const mh_shape &a = desc->shapes[i];
        DShape &b = shapes[i];
        memset(&b, 0, sizeof(b));
        b.type = a.type; b.bsdf = a.bsdf; b.emitter = a.emitter; b.face_offset = a.face_offset;
        b.vertex_offset = a.vertex_offset; b.has_normals = a.has_normals; b.has_texcoords = a.has_texcoords;
        if (a.bsdf >= desc->n_bsdfs) return fail(MH_ERR_INVALID_ARGUMENT, "mh_scene_create: bsdf index out of bounds");
        memcpy(b.to_world, a.to_world, sizeof(b.to_world));
        memcpy(b.frame_s, a.frame_s, 12);
        memcpy(b.frame_t, a.frame_t, 12);
        memcpy(b.frame_n, a.frame_n, 12);
        b.inv_area = a.inv_area;
        b.interior = a.interior_medium;
        b.exterior = a.exterior_medium;
        if ((b.interior != MH_INVALID && b.interior >= desc->n_media) ||
            (b.exterior != MH_INVALID && b.exterior >= desc->n_media))
            return fail(MH_ERR_INVALID_ARGUMENT, "mh_scene_create: medium index out of bounds");
    }
    // ---- media (heterogeneous.cpp / homogeneous.cpp / grid.cpp) ----
    std::vector<DMedium> meds(desc->n_media);
    for (uint32_t i = 0; i < desc->n_media; ++i) {
        const mh_medium &a = desc->media[i];
        DMedium &b = meds[i];
        memset(&b, 0, sizeof(b));
        b.type = a.type; b.phase = a.phase; b.flags = a.flags;
        b.g = a.g; b.scale = a.scale; b.sigma_t_const = a.sigma_t_const;
        // m_max_density = m_scale * m_sigmat->max() (heterogeneous.cpp:163), in float
        b.maj = a.type == MH_MEDIUM_HOMOGENEOUS ? a.sigma_t_const * a.scale : a.scale * a.max_density;
        memcpy(b.albedo, a.albedo, 12);
        memcpy(b.res, a.grid_res, 12);
        b.grid_offset = 0;   // bricked offset: assigned below
        memcpy(b.to_local, a.grid_to_local, sizeof(b.to_local));
        memcpy(b.bbox_min, a.bbox_min, 12);
        memcpy(b.bbox_max, a.bbox_max, 12);
        if (a.type == MH_MEDIUM_HETEROGENEOUS &&
            (a.grid_res[0] == 0 || a.grid_res[1] == 0 || a.grid_res[2] == 0 ||
             a.grid_offset + (uint64_t)a.grid_res[0] * a.grid_res[1] * a.grid_res[2] > desc->n_grid))
            return fail(MH_ERR_INVALID_ARGUMENT, "mh_scene_create: volume grid out of bounds");
        // grid_eval indexes a grid's bricked texels with 32-bit offsets
        if (a.type == MH_MEDIUM_HETEROGENEOUS && grid_bricked_size(a.grid_res) >= (1ull << 32))
            return fail(MH_ERR_UNSUPPORTED, "mh_scene_create: volume grid above 2^32 texels");
        if (a.phase == MH_PHASE_HG && !(a.g > -1.f && a.g < 1.f))
            return fail(MH_ERR_INVALID_ARGUMENT, "The asymmetry parameter must lie in the interval (-1, 1)!");
    }
    if (desc->sensor.pixel_format > MH_PIXEL_XYZA)
        return fail(MH_ERR_INVALID_ARGUMENT, "mh_scene_create: unknown pixel format");
    s->pixel_format = desc->sensor.pixel_format;
    // density grids in the 4^3-brick device layout (grid_index)
    std::vector<float> bricked;
    for (uint32_t i = 0; i < desc->n_media; ++i) {
        if (desc->media[i].type != MH_MEDIUM_HETEROGENEOUS) continue;
        meds[i].grid_offset = bricked.size();
        bricked.resize(bricked.size() + grid_bricked_size(desc->media[i].grid_res));
        grid_to_bricks(desc->grid_data + desc->media[i].grid_offset, desc->media[i].grid_res,
                       bricked.data() + meds[i].grid_offset);
    }
    s->h_media.assign(desc->media, desc->media + desc->n_media);
    s->h_dmedia = meds;
    s->n_media = desc->n_media;
    if (desc->sensor.medium != MH_INVALID && desc->sensor.medium >= desc->n_media)
        return fail(MH_ERR_INVALID_ARGUMENT, "mh_scene_create: sensor medium index out of bounds");
    std::vector<uint32_t> btype(desc->n_bsdfs), btex(desc->n_bsdfs);
    for (uint32_t i = 0; i < desc->n_bsdfs; ++i) {
        btype[i] = desc->bsdfs[i].type;
        btex[i] = desc->bsdfs[i].reflectance;
        if (btype[i] == MH_BSDF_DIFFUSE && btex[i] >= desc->n_textures)
            return fail(MH_ERR_INVALID_ARGUMENT, "mh_scene_create: texture index out of bounds");
    }
    s->h_textures.resize(desc->n_textures);
    for (uint32_t i = 0; i < desc->n_textures; ++i) {
        const mh_texture &a = desc->textures[i];
        DTexture &b = s->h_textures[i];
        memset(&b, 0, sizeof(b));
        b.type = a.type; b.width = a.width; b.height = a.height; b.channels = a.channels;
        b.data_offset = a.data_offset; b.filter = a.filter; b.wrap = a.wrap;
        memcpy(b.value, a.value, 12);
        memcpy(b.to_uv, a.to_uv, 24);
        if (a.type == MH_TEX_BITMAP &&
            a.data_offset + (uint64_t)a.width * a.height * a.channels > desc->n_texels)
            return fail(MH_ERR_INVALID_ARGUMENT, "mh_scene_create: bitmap data out of bounds");
    }
    std::vector<DEmitter> ems(desc->n_emitters);
    for (uint32_t i = 0; i < desc->n_emitters; ++i) {
        memset(&ems[i], 0, sizeof(DEmitter));
        ems[i].type = desc->emitters[i].type;
        ems[i].shape = desc->emitters[i].shape;
        memcpy(ems[i].radiance, desc->emitters[i].radiance, 12);
        memcpy(ems[i].direction, desc->emitters[i].direction, 12);
        memcpy(ems[i].center, desc->emitters[i].scene_center, 12);
        ems[i].radius = desc->emitters[i].scene_radius;
    }
    s->n_textures = desc->n_textures;
    s->n_bsdfs = desc->n_bsdfs;
    s->n_shapes = desc->n_shapes;
    s->n_texels = desc->n_texels;
    bool ok = upload(s->shapes, shapes.data(), shapes.size(), st) == hipSuccess &&
              upload(s->bsdf_type, btype.data(), btype.size(), st) == hipSuccess &&
              upload(s->bsdf_tex, btex.data(), btex.size(), st) == hipSuccess &&
              upload(s->textures, s->h_textures.data(), s->h_textures.size(), st) == hipSuccess &&
              upload(s->emitters, ems.data(), ems.size(), st) == hipSuccess &&
              upload(s->positions, desc->positions, 3ull * desc->n_vertices, st) == hipSuccess &&
              upload(s->normals, desc->normals, desc->normals ? 3ull * desc->n_vertices : 0, st) == hipSuccess &&
              upload(s->texcoords, desc->texcoords, desc->texcoords ? 2ull * desc->n_vertices : 0, st) == hipSuccess &&
              upload(s->faces, desc->faces, 3ull * desc->n_faces, st) == hipSuccess &&
              upload(s->texels, desc->texels, desc->n_texels, st) == hipSuccess &&
              upload(s->media, meds.data(), meds.size(), st) == hipSuccess &&
              upload(s->grid, bricked.data(), bricked.size(), st) == hipSuccess &&
              s->counters.alloc(256 + 1024) == hipSuccess;  // 32 counters + 8 work heads on own lines
    if (!ok) return fail(MH_ERR_OUT_OF_MEMORY, "mh_scene_create: device upload failed");

    DScene &S = s->S;
    S.nodes = s->nodes.as<Node>();
    S.prims = s->prims.as<Prim>();
    S.key_sp = s->key_sp.as<uint2>();
    S.prim_pairs = s->prim_pairs.as<Prim>();
    S.shapes = s->shapes.as<DShape>();
    S.bsdf_type = s->bsdf_type.as<uint32_t>();
    S.bsdf_tex = s->bsdf_tex.as<uint32_t>();
    S.textures = s->textures.as<DTexture>();
    S.emitters = s->emitters.as<DEmitter>();
    S.positions = s->positions.as<float>();
    S.normals = desc->normals ? s->normals.as<float>() : nullptr;
    S.texcoords = desc->texcoords ? s->texcoords.as<float>() : nullptr;
    S.faces = s->faces.as<uint32_t>();
    S.texels = s->texels.as<float>();
    S.media = s->media.as<DMedium>();
    S.grid = s->grid.as<float>();
    S.n_media = desc->n_media;
    S.camera_medium = desc->sensor.medium;
    S.vol_flags = 0;
    for (uint32_t i = 0; i < desc->n_shapes; ++i)
        for (uint32_t mm : {desc->shapes[i].interior_medium, desc->shapes[i].exterior_medium})
            if (mm != MH_INVALID)
                S.vol_flags |= desc->media[mm].type == MH_MEDIUM_HOMOGENEOUS ? kVolNeeHomogeneous : kVolHandleNull;
    S.n_shapes = desc->n_shapes;
    S.n_bsdfs = desc->n_bsdfs;
    S.n_textures = desc->n_textures;
    S.n_vertices = desc->n_vertices;
    S.n_faces = desc->n_faces;
    {
        const TabLayout TL = tab_layout(S.n_shapes, S.n_bsdfs, S.n_textures, desc->n_emitters, S.n_vertices,
                                        S.n_faces, S.normals != nullptr && S.n_vertices,
                                        S.texcoords != nullptr && S.n_vertices);
        S.tab_bytes = TL.total <= 16384 ? TL.total : 0u;  // staged into LDS by the shade kernels
    }
    S.n_nodes = bvh.n_nodes;
    S.n_prims = bvh.n_prims;
    S.n_emitters = desc->n_emitters;
    S.inv_n_emitters = 1.f / (float)S.n_emitters;  // inf for 0: never read then
    S.n_emitters_f = (float)S.n_emitters;
    S.env_pdf = kInv4Pi * S.inv_n_emitters;
    S.environment = desc->environment;
    S.stack_size = bvh.depth + 2;
    const size_t bvh_bytes = bvh.nodes.size() + bvh.prims.size();
    S.lds_bytes_bvh = bvh_bytes <= 32768 ? (uint32_t)bvh_bytes : 0u;  // stage into LDS when small
    // wide BVH for the stream engine when the BVH lives in global memory
    // (mh_bvh.cpp collapse_bvh4; MH_BVH4=0 keeps BVH2 everywhere)
    S.nodes4 = nullptr;
    S.qnodes = nullptr;
    S.primsc = nullptr;
    {
        // the float BVH4 (round 1); MH_BVH4Q=1: the quantised BVH4 + compact
        // primitives (round 4, measured slower so far: DESIGN.md §3);
        // MH_BVH4=0: BVH2
        const char *e4 = getenv("MH_BVH4"), *eq = getenv("MH_BVH4Q");
        if (S.lds_bytes_bvh == 0 && bvh.n_prims > 64 && !(e4 && !strcmp(e4, "0"))) {
            std::vector<uint8_t> n4, pc;
            uint32_t cnt4 = 0, depth4 = 0;
            const bool quant = (eq && !strcmp(eq, "1")) && build_qbvh4(bvh, n4, pc, cnt4, depth4);
            if (!quant) collapse_bvh4(bvh, n4, cnt4, depth4);
            const uint32_t stack4 = 3u * depth4 + 2u;
            if ((size_t)std::max(S.stack_size, stack4) * 256 * 4 <= 65536 &&
                upload(s->nodes4, n4.data(), n4.size(), st) == hipSuccess &&
                (!quant || upload(s->primsc, pc.data(), pc.size(), st) == hipSuccess)) {
                if (quant) {
                    S.qnodes = reinterpret_cast<const QNode4 *>(s->nodes4.ptr);
                    S.primsc = reinterpret_cast<const PrimC *>(s->primsc.ptr);
                } else {
                    S.nodes4 = reinterpret_cast<const Node4 *>(s->nodes4.ptr);
                    // MH_PRIMC=1: the compact 48-B triangle records with the float BVH4
                    const char *epc = getenv("MH_PRIMC");
                    if (epc && !strcmp(epc, "1")) {
                        std::vector<uint8_t> qn, pc2;
                        uint32_t c2 = 0, d2 = 0;
                        if (build_qbvh4(bvh, qn, pc2, c2, d2) && upload(s->primsc, pc2.data(), pc2.size(), st) == hipSuccess)
                            S.primsc = reinterpret_cast<const PrimC *>(s->primsc.ptr);
                    }
                }
                S.stack_size = std::max(S.stack_size, stack4);
            }
        }
    }
    // The stream engine's stack (round 4): the bound 3 * depth4 + 2 of a
    // wide-BVH traversal (44-50 entries on 1M-4M triangles) put 48 KiB of LDS
    // stack in every 256-thread workgroup and held the trace kernels at 3
    // waves per SIMD; the stacks rays really build stay far shallower
    // (tools/qbvh_stats: at most 14 entries on those meshes).  So the first
    // kStreamStack entries live in LDS and deeper ones in a global overflow
    // region, one column per thread of the largest stream-kernel grid: exact
    // for any depth, and 6 waves per SIMD.  Same box, path 512^2 @ 64 on the
    // 1M / 4M-triangle meshes: 386 / 317 Msamples/s with the full LDS stack,
    // 522 / 434 capped at 12-20 entries (5 waves), 534-538 / 446-451 at 6
    // waves (MH_STREAM_WAVES).  MH_STREAM_STACK overrides the cap.
    S.stream_stack = S.stack_size;
    S.stack_ovf = nullptr;
    S.ovf_threads = 0;
    if (S.lds_bytes_bvh == 0 && (S.nodes4 || S.qnodes)) {
        const char *es = getenv("MH_STREAM_STACK");
        const uint32_t cap = es ? (uint32_t)std::max(4, atoi(es)) : 20u;
        if (cap < S.stack_size) {
            int cus = 256;
            (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
            const uint32_t threads = wf_blocks(cus) * 256u;
            if (upload(s->stack_ovf, (const uint32_t *)nullptr, (size_t)(S.stack_size - cap) * threads, st) == hipSuccess) {
                S.stream_stack = cap;
                S.stack_ovf = s->stack_ovf.as<uint32_t>();
                S.ovf_threads = threads;
            }
        }
    }
    if ((size_t)S.stack_size * 256 * 4 + S.lds_bytes_bvh > 65536)
        return fail(MH_ERR_UNSUPPORTED, "mh_scene_create: BVH too deep for the LDS traversal stack");
    memcpy(S.cam_to_world, sn.to_world, sizeof(S.cam_to_world));
    memcpy(S.sample_to_camera, sn.sample_to_camera, sizeof(S.sample_to_camera));
    S.near_clip = sn.near_clip;
    S.far_clip = sn.far_clip;
    S.width = sn.width;
    S.height = sn.height;
    S.inv_width = 1.f / (float)S.width;
    S.inv_height = 1.f / (float)S.height;
    S.rfilter = sn.rfilter;
    S.rfilter_radius = sn.rfilter_radius;
    memcpy(S.filter_coeff, sn.filter_coeff, sizeof(S.filter_coeff));
    S.sampler_seed = sn.sampler_seed;
    if (hipEventCreate(&s->ev0) != hipSuccess || hipEventCreate(&s->ev1) != hipSuccess)
        return fail(MH_ERR_HIP, "mh_scene_create: hipEventCreate failed");
    if (hipStreamSynchronize(st) != hipSuccess) return fail(MH_ERR_HIP, "mh_scene_create: upload sync failed");
    *out = s;
    return MH_OK;
}

int mh_scene_destroy(mh_scene *s) {
    if (!s) return MH_OK;
    if (s->comm) comm_attach(s->comm, -1);
    (void)hipSetDevice(s->device);
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    for (DevBuf *b : {&s->nodes, &s->nodes4, &s->primsc, &s->stack_ovf, &s->prims, &s->prim_pairs, &s->key_sp, &s->shapes, &s->bsdf_type, &s->bsdf_tex, &s->textures,
                      &s->emitters, &s->positions, &s->normals, &s->texcoords, &s->faces, &s->texels,
                      &s->media, &s->grid, &s->work, &s->film_tmp, &s->film4, &s->alpha_px, &s->counters, &s->grad_meta, &s->tmp_a, &s->tmp_b,
                      &s->tmp_c, &s->tmp_d, &s->tmp_e, &s->weights_tmp, &s->wf_ws, &s->wf_ctr, &s->wf_ws_prb, &s->wf_partial, &s->gw, &s->wf_carry, &s->wf_ws_bmp, &s->wf_ws_det, &s->pvp_log, &s->pvp_main, &s->pvp_ovf, &s->grid_corner, &s->fx_word, &s->bmp_fx,
                      &s->shard_w, &s->shard_tmp, &s->shard_g, &s->replay_fx, &s->wf_ws2, &s->wf_ws_prb2,
                      &s->wf_ws_bmp2, &s->wf_partial2, &s->work2, &s->wf_carry2, &s->stack_ovf2})
        b->release();
    if (s->stream2) {
        (void)hipStreamSynchronize(s->stream2);
        (void)hipStreamDestroy(s->stream2);
    }
    if (s->ev_fork) (void)hipEventDestroy(s->ev_fork);
    if (s->ev_join) (void)hipEventDestroy(s->ev_join);
    for (hipEvent_t e : s->evpool) (void)hipEventDestroy(e);
    if (s->ev0) (void)hipEventDestroy(s->ev0);
    if (s->ev1) (void)hipEventDestroy(s->ev1);
    if (s->own_stream && s->stream) (void)hipStreamDestroy(s->stream);
    delete s;
    return MH_OK;
}

int mh_scene_set_stream(mh_scene *s, void *stream) {
    if (!s) return set_error(MH_ERR_INVALID_ARGUMENT, "mh_scene_set_stream: NULL scene");
    if (s->own_stream && s->stream == (hipStream_t)stream) return MH_OK;
    if (s->own_stream && s->stream) {
        (void)hipStreamSynchronize(s->stream);
        (void)hipStreamDestroy(s->stream);
    }
    s->own_stream = false;
    s->stream = (hipStream_t)stream;
    return MH_OK;
}

int mh_scene_bvh_info(mh_scene *s, uint32_t *n_nodes, uint32_t *n_prims, uint32_t *depth) {
    if (!s) return set_error(MH_ERR_INVALID_ARGUMENT, "mh_scene_bvh_info: NULL scene");
    if (n_nodes) *n_nodes = s->bvh_nodes;
    if (n_prims) *n_prims = s->bvh_prims;
    if (depth) *depth = s->bvh_depth;
    return MH_OK;
}

int mh_scene_update_rgb(mh_scene *s, uint32_t tex, const float value[3]) {
    if (!s || !value) return set_error(MH_ERR_INVALID_ARGUMENT, "mh_scene_update_rgb: NULL argument");
    if (tex >= s->n_textures || s->h_textures[tex].type != MH_TEX_RGB)
        return set_error(MH_ERR_INVALID_ARGUMENT, "mh_scene_update_rgb: not an rgb texture");
    MH_HIP(hipSetDevice(s->device));
    memcpy(s->h_textures[tex].value, value, 12);
    MH_HIP(hipMemcpyAsync(s->textures.as<DTexture>() + tex, &s->h_textures[tex], sizeof(DTexture),
                          hipMemcpyHostToDevice, s->stream));
    MH_HIP(hipStreamSynchronize(s->stream));
    return MH_OK;
}

int mh_scene_update_texture(mh_scene *s, uint32_t tex, const float *data, uint64_t n) {
    if (!s || !data) return set_error(MH_ERR_INVALID_ARGUMENT, "mh_scene_update_texture: NULL argument");
    if (tex >= s->n_textures || s->h_textures[tex].type != MH_TEX_BITMAP)
        return set_error(MH_ERR_INVALID_ARGUMENT, "mh_scene_update_texture: not a bitmap texture");
    const DTexture &t = s->h_textures[tex];
    if (n != (uint64_t)t.width * t.height * t.channels)
        return set_error(MH_ERR_INVALID_ARGUMENT, "mh_scene_update_texture: size mismatch");
    MH_HIP(hipSetDevice(s->device));
    MH_HIP(hipMemcpyAsync(s->texels.as<float>() + t.data_offset, data, n * 4, hipMemcpyHostToDevice,
                          s->stream));
    MH_HIP(hipStreamSynchronize(s->stream));
    return MH_OK;
}

// SceneParameters.update of a medium's differentiable parameters
// (heterogeneous.cpp:169-178 / homogeneous.cpp:150-155): albedo, homogeneous
// sigma_t, heterogeneous sigma_t grid; the majorant is recomputed as
// parameters_changed does (m_max_density = scale * max(grid)).
int mh_scene_update_medium(mh_scene *s, uint32_t medium, const float *albedo, const float *sigma_t,
                           const float *grid, uint64_t n, uint32_t flags) {
    if (!s) return set_error(MH_ERR_INVALID_ARGUMENT, "mh_scene_update_medium: NULL scene");
    if (medium >= s->n_media) return set_error(MH_ERR_INVALID_ARGUMENT, "mh_scene_update_medium: medium index out of bounds");
    MH_HIP(hipSetDevice(s->device));
    mh_medium &a = s->h_media[medium];
    DMedium &b = s->h_dmedia[medium];
    if (albedo) {
        memcpy(a.albedo, albedo, 12);
        memcpy(b.albedo, albedo, 12);
    }
    if (sigma_t) {
        if (a.type != MH_MEDIUM_HOMOGENEOUS)
            return set_error(MH_ERR_INVALID_ARGUMENT, "mh_scene_update_medium: sigma_t value of a heterogeneous medium (use grid)");
        a.sigma_t_const = b.sigma_t_const = *sigma_t;
        b.maj = b.sigma_t_const * b.scale;
    }
    if (grid) {
        if (a.type != MH_MEDIUM_HETEROGENEOUS)
            return set_error(MH_ERR_INVALID_ARGUMENT, "mh_scene_update_medium: grid of a homogeneous medium");
        if (n != (uint64_t)a.grid_res[0] * a.grid_res[1] * a.grid_res[2])
            return set_error(MH_ERR_INVALID_ARGUMENT, "mh_scene_update_medium: size mismatch");
        // linear copy on the device (staging), then the max and the brick scatter
        MH_HIP(s->tmp_e.alloc(n * 4));
        float *lin = s->tmp_e.as<float>();
        MH_HIP(hipMemcpyAsync(lin, grid, n * 4, (flags & MH_FLAG_DEVICE_POINTERS) ? hipMemcpyDeviceToDevice
                                                                                 : hipMemcpyHostToDevice, s->stream));
        MH_HIP(launch_grid_to_bricks(lin, a.grid_res, s->grid.as<float>() + b.grid_offset, s->stream));
        MH_HIP(s->tmp_b.alloc(16));
        MH_HIP(launch_grid_max(lin, n, s->tmp_b.as<uint32_t>(), s->stream));
        uint32_t key = 0;
        MH_HIP(hipMemcpyAsync(&key, s->tmp_b.ptr, 4, hipMemcpyDeviceToHost, s->stream));
        MH_HIP(hipStreamSynchronize(s->stream));
        a.max_density = ordered_key_to_float(key);
        b.maj = b.scale * a.max_density;
    }
    MH_HIP(hipMemcpyAsync(s->media.as<DMedium>() + medium, &b, sizeof(DMedium), hipMemcpyHostToDevice, s->stream));
    MH_HIP(hipStreamSynchronize(s->stream));
    return MH_OK;
}

// ---------------------------------------------------------------------------
// Render
// ---------------------------------------------------------------------------
static bool has_alpha(uint32_t fmt) {
    return fmt == MH_PIXEL_RGBA || fmt == MH_PIXEL_YA || fmt == MH_PIXEL_XYZA;
}
// channels of the developed image (hdrfilm.cpp:349-372: color_ch + alpha)
static uint32_t image_channels(uint32_t fmt) {
    const uint32_t c = (fmt == MH_PIXEL_Y || fmt == MH_PIXEL_YA) ? 1u : 3u;
    return c + (has_alpha(fmt) ? 1u : 0u);
}
struct Layout {
    uint32_t W, H, spp, spp_pp, n_passes, s_begin, s_end;
};

// ad: the Python ADIntegrator's single wavefront (prb / prbvolpath primal,
// W image and render_backward): prepare() accepts up to exactly 2^32 samples
// and raises beyond (common.py:571-578); lane indices [0, 2^32) are uint32.
// Otherwise SamplingIntegrator::render's passes of <= 2^32 - 1 samples.
static int make_layout(const mh_scene *s, uint32_t spp, uint32_t b, uint32_t e, Layout &L, bool ad) {
    L.W = s->S.width;
    L.H = s->S.height;
    L.spp = spp;
    uint64_t wf = (uint64_t)L.W * L.H * spp, lim = 0xffffffffull;
    L.spp_pp = spp;
    L.n_passes = 1;
    if (ad && wf > (1ull << 32))
        return set_error(MH_ERR_INVALID_ARGUMENT,
                         "The total number of Monte Carlo samples required by this rendering task (" +
                             std::to_string(wf) + ") exceeds 2^32 = 4294967296. Please use fewer samples "
                             "per pixel or render using multiple passes.");
    if (!ad && wf > lim) {  // integrator.cpp:281-295
        L.spp_pp = spp / (uint32_t)((wf + lim - 1) / lim);
        L.n_passes = spp / L.spp_pp;
        if (L.spp_pp * L.n_passes != spp)
            return set_error(MH_ERR_INVALID_ARGUMENT,
                             "render(): sample_count should be a multiple of samples_per_wavefront!");
    }
    if (b == 0 && e == 0) e = L.spp_pp;
    if (e > L.spp_pp || b >= e)
        return set_error(MH_ERR_INVALID_ARGUMENT, "render(): invalid sample slab [spp_begin, spp_end)");
    L.s_begin = b;
    L.s_end = e;
    return MH_OK;
}

static LaneMap lane_map(const Layout &L, uint32_t pixel_begin) {
    LaneMap m;
    m.W = L.W;
    m.spp_pp = L.spp_pp;
    m.log_spp = log2_exact(L.spp_pp);
    m.pixel_begin = pixel_begin;
    m.S = L.s_end - L.s_begin;
    m.s_begin = L.s_begin;
    m.log_S = log2_exact(m.S);
    return m;
}

// The scene's 32-word counter block (zeroed per call): [0] closest rays,
// [1] shadow rays, [2..22] k_vol_sched phase statistics (MH_EXP_VSCNT
// builds), [kCtrInvalid] invalid samples, [kCtrPvpHead] the prbvolpath
// backward's work head; bytes 256.. hold k_vol_sched's 8 queue heads
constexpr int kCtrInvalid = 28;
constexpr int kCtrPvpHead = 30;
// [kCtrBounds]: rows of the splat kernels that would have read past their
// input planes (skipped; the call then fails; none in a correct build)
constexpr int kCtrBounds = 29;
// [kCtrLookups]: k_vol_sched's density-grid lookups (mh_stats.grid_lookups)
constexpr int kCtrLookups = 27;
// [kCtrAuxItems]: bitmap vertex records read by the texel scatter (mh_stats.aux_items)
constexpr int kCtrAuxItems = 26;

// launch_splat with its bounds contract: hipErrorInvalidValue from the host
// check becomes a named error instead of a bare HIP code
#define MH_SPLAT(...)                                                                                   \
    do {                                                                                                \
        hipError_t _e = launch_splat(__VA_ARGS__);                                                      \
        if (_e == hipErrorInvalidValue)                                                                 \
            return set_error(MH_ERR_INVALID_ARGUMENT, "splat: sample planes / film smaller than the "   \
                                                      "chunk's layout (bounds contract of launch_splat)"); \
        if (_e != hipSuccess) return set_error(MH_ERR_HIP, std::string("launch_splat: ") + hipGetErrorString(_e)); \
    } while (0)

// the device half of the contract: a non-zero bounds counter fails the call
static int check_bounds_counter(mh_scene *s, const char *api);
// prbvolpath backward grid (MH_VOL_WAVES = 4 waves / SIMD: 4 workgroups per CU)
// and NEE-log entries per thread (16 B each; longer walks replay)
constexpr uint32_t kPvpBlocksPerCu = 4, kPvpNeeCap = 256;
// MainLog entries per thread (64 B each: 4 GiB over the 262,144 threads of a
// 256-CU grid, less when the render has fewer samples than threads); a path
// with more logged vertices replays its adjoint
constexpr uint32_t kPvpMainCap = 256;
// MH_FLAG_DETERMINISTIC or MH_DETERMINISTIC=1: fixed-order splat (k_splat_gather)
static bool deterministic(uint32_t flags) {
    const char *e = getenv("MH_DETERMINISTIC");
    return (flags & MH_FLAG_DETERMINISTIC) || (e && !strcmp(e, "1"));
}

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

static int check_bounds_counter(mh_scene *s, const char *api) {
    unsigned long long v = 0;
    MH_HIP(hipMemcpy(&v, s->counters.as<unsigned long long>() + kCtrBounds, sizeof(v), hipMemcpyDeviceToHost));
    if (v)
        return set_error(MH_ERR_HIP, std::string(api) + ": " + std::to_string(v) +
                                         " splat rows would have read past the sample planes (skipped)");
    return MH_OK;
}

// k_vol_sched's per-phase statistics of the last launch (MH_EXP_VSCNT
// diagnostic builds, MH_VW_DEBUG=1): wave trips, lanes and shader cycles
static int print_vs_phases(mh_scene *s) {
    unsigned long long c[32];
    MH_HIP(hipMemcpy(c, s->counters.ptr, sizeof(c), hipMemcpyDeviceToHost));
    const char *nm[8] = {"free", "head", "trace", "scatter", "surf", "walk", "post", "end"};
    for (int g = 0; g < 8; ++g)  // groups of k_vol_sched (kNGroups = 8): trips, lanes, cycles
        fprintf(stderr, "vs phase %-8s wave trips %llu, lanes %llu (%.1f per trip), cycles %.3e (%.0f per trip)\n",
                nm[g], c[2 + g], c[10 + g], c[2 + g] ? (double)c[10 + g] / c[2 + g] : 0.0, (double)c[18 + g],
                c[2 + g] ? (double)c[18 + g] / c[2 + g] : 0.0);
    return MH_OK;
}

// MH_FLAG_REDUCE / MH_FLAG_REDUCE_ROOT: the call's result summed over the
// scene's communicator (mh_comm.cpp), stream-ordered behind the kernels that
// produced it.  A film honours MH_FLAG_REDUCE_ROOT (a reduce to rank 0); W
// images and gradients are needed on every rank and are always all-reduced.
static bool wants_reduce(uint32_t flags) { return flags & (MH_FLAG_REDUCE | MH_FLAG_REDUCE_ROOT); }

static int check_reduce_flags(const mh_scene *s, uint32_t flags, const char *api, bool accumulating_output) {
    if (!wants_reduce(flags)) return MH_OK;
    if (!s->comm)
        return set_error(MH_ERR_INVALID_ARGUMENT,
                         std::string(api) + ": MH_FLAG_REDUCE needs a communicator (mh_scene_set_comm)");
    if (accumulating_output && (flags & MH_FLAG_ACCUMULATE))
        return set_error(MH_ERR_INVALID_ARGUMENT,
                         std::string(api) + ": MH_FLAG_REDUCE cannot be combined with MH_FLAG_ACCUMULATE "
                                            "(the sum would count the accumulated content once per rank)");
    return MH_OK;
}

static int reduce_result(mh_scene *s, uint32_t flags, float *buf, uint64_t count, hipStream_t st, bool film) {
    if (!wants_reduce(flags)) return MH_OK;
    const int root = (film && (flags & MH_FLAG_REDUCE_ROOT) && !(flags & MH_FLAG_REDUCE)) ? 0 : -1;
    return comm_reduce_one(s->comm, s->device, buf, count, st, root);
}

// The waits of a call whose collectives are in flight: with MH_FLAG_REDUCE a
// deadline-bounded poll that also watches the communicator's async error and
// aborts it on a failure (mh_comm.cpp comm_wait), so a rank whose peer failed
// before issuing its collective returns an error instead of hanging in
// hipStreamSynchronize; otherwise a plain stream sync.
static hipError_t wait_stream(mh_scene *s, uint32_t flags, hipStream_t st) {
    if (wants_reduce(flags) && s->comm) {
        if (comm_wait(s->comm, st, "collective call") == MH_OK) return hipSuccess;
        g_keep_error = true;  // comm_wait's message stands
        return hipErrorLaunchTimeOut;
    }
    return hipStreamSynchronize(st);
}
#define MH_WAIT(s, flags, st)                                                                         \
    do {                                                                                              \
        if (wants_reduce(flags) && (s)->comm) {                                                       \
            if (int _rc = comm_wait((s)->comm, st, __func__)) return _rc;                             \
        } else {                                                                                      \
            MH_HIP(hipStreamSynchronize(st));                                                         \
        }                                                                                             \
    } while (0)

// MH_FLAG_DEVICE_POINTERS | MH_FLAG_NO_SYNC without stats: nothing is read
// back to the host, so the call returns with its work enqueued on the stream
static bool async_call(uint32_t flags, const mh_stats *stats) {
    return (flags & MH_FLAG_DEVICE_POINTERS) && (flags & MH_FLAG_NO_SYNC) && !stats;
}

// Two-stream chunk pipeline of the wavefront (mh_render and
// mh_render_backward): chunk c runs on the scene's stream (c even) or on
// stream2 (c odd), each with its own workspace (and, for the stream engine of
// large meshes, its own stack overflow columns), and the launches take the
// shared-device grid (wf_blocks), so one chunk's late bounces -- a few paths
// each, the chip mostly idle -- and its splat / texel scatter overlap the
// other chunk's launches.  Only where the chunks share nothing but atomically
// updated outputs: the non-deterministic splat / gradient paths; not with MH_FLAG_SHARED_DEVICE
// (the caller already runs another call beside this one).  A single-chunk
// call of at least kTwoStreamMinSamples samples is split into two chunks.
// MH_WF_STREAMS=1 keeps one stream (measurements, the bench's roofline pass).
constexpr uint64_t kTwoStreamMinSamples = 1ull << 19;
static bool chunk_streams_enabled() {
    const char *e = getenv("MH_WF_STREAMS");
    return !(e && !strcmp(e, "1"));
}

// stream2 (created on first use, on the scene's device) waits for the work
// enqueued on st so far
static hipError_t fork_stream(mh_scene *s, hipStream_t st) {
    hipError_t e = hipSuccess;
    if (!s->stream2) e = hipStreamCreateWithFlags(&s->stream2, hipStreamNonBlocking);
    if (e == hipSuccess && !s->ev_fork) e = hipEventCreateWithFlags(&s->ev_fork, hipEventDisableTiming);
    if (e == hipSuccess && !s->ev_join) e = hipEventCreateWithFlags(&s->ev_join, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(s->ev_fork, st);
    if (e == hipSuccess) e = hipStreamWaitEvent(s->stream2, s->ev_fork, 0);
    return e;
}
// st waits for everything enqueued on stream2
static hipError_t join_stream(mh_scene *s, hipStream_t st) {
    hipError_t e = hipEventRecord(s->ev_join, s->stream2);
    if (e == hipSuccess) e = hipStreamWaitEvent(st, s->ev_join, 0);
    return e;
}

static int render_impl(mh_scene *s, const mh_integrator *in, uint32_t seed, uint32_t spp, uint32_t spp_begin,
              uint32_t spp_end, float *film_rgbw, uint32_t flags, mh_stats *stats) {
    ScopedPhase phase_("Render");
    if (!s || !in || !film_rgbw) return set_error(MH_ERR_INVALID_ARGUMENT, "mh_render: NULL argument");
    if (in->type > MH_INTEGRATOR_PRBVOLPATH)
        return set_error(MH_ERR_INVALID_ARGUMENT, "mh_render: unknown integrator");
    if (in->rr_depth == 0)
        return set_error(MH_ERR_INVALID_ARGUMENT, "\"rr_depth\" must be set to a value greater than zero!");
    if (spp == 0) return set_error(MH_ERR_INVALID_ARGUMENT, "mh_render: spp must be > 0");
    if (int rc = check_reduce_flags(s, flags, "mh_render", true)) return rc;
    double t_start = now_ms();
    if (stats) *stats = mh_stats{};
    Layout L;
    const bool ad = in->type == MH_INTEGRATOR_PRB || in->type == MH_INTEGRATOR_PRBVOLPATH;
    int rc = make_layout(s, spp, spp_begin, spp_end, L, ad);
    if (rc) return rc;
    MH_HIP(hipSetDevice(s->device));
    g_call_issued = true;  // past argument validation: a failure from here aborts the communicator
    // test hook of the communicator's failure semantics (tests/test_gpu_comm.py,
    // documented in INTEGRATION.md): a reducing call (MH_FLAG_REDUCE) fails
    // after it was issued.  Calls without a collective never read it.
    if ((flags & MH_FLAG_REDUCE) && getenv("MH_TEST_FAIL_AFTER_ISSUE"))
        return set_error(MH_ERR_HIP, "MH_TEST_FAIL_AFTER_ISSUE: injected failure");
    hipStream_t st = s->stream;
    const uint64_t n_px = (uint64_t)L.W * L.H;
    // film storage: RGBW, or R G B A W for alpha films; the kernels splat into
    // an RGBW film (+ an alpha plane) that an alpha film receives at the end
    const bool alpha = has_alpha(s->pixel_format);
    const size_t film_bytes = n_px * (alpha ? 20 : 16);
    float *film = film_rgbw;
    if (!(flags & MH_FLAG_DEVICE_POINTERS)) {
        MH_HIP(s->film_tmp.alloc(film_bytes));
        film = s->film_tmp.as<float>();
    }
    if (!(flags & MH_FLAG_ACCUMULATE) || !(flags & MH_FLAG_DEVICE_POINTERS)) {
        if (!(flags & MH_FLAG_ACCUMULATE)) MH_HIP(hipMemsetAsync(film, 0, film_bytes, st));
        else MH_HIP(hipMemcpyAsync(film, film_rgbw, film_bytes, hipMemcpyHostToDevice, st));
    }
    float *film4 = film, *film_a = nullptr;
    if (alpha) {
        MH_HIP(s->film4.alloc(n_px * 16));
        MH_HIP(s->alpha_px.alloc(n_px * 4));
        film4 = s->film4.as<float>();
        film_a = s->alpha_px.as<float>();
        MH_HIP(hipMemsetAsync(film4, 0, n_px * 16, st));
        MH_HIP(hipMemsetAsync(film_a, 0, n_px * 4, st));
    }
    MH_HIP(hipMemsetAsync(s->counters.ptr, 0, 256, st));
    const uint32_t S_ = L.s_end - L.s_begin;
    const uint64_t per_pixel = (uint64_t)S_ * L.n_passes;
    // execution mode: wavefront for `path` (bounded depth; several passes only
    // on the fused bounce kernel, which carries each lane's PCG32 state from
    // one pass to the next) unless forced
    bool wavefront = in->type == MH_INTEGRATOR_PATH && in->max_depth <= 64 && (L.n_passes == 1 || wf_fused(s->S));
    // volpath: main / walk rounds (mh_volwave.hip), single pass
    bool volwave = (vol_sched_mode() ? vs_supported(s->S, *in) : vw_supported(s->S, *in)) && L.n_passes == 1;
    const char *env_mode = getenv("MH_MODE");
    if (env_mode && !strcmp(env_mode, "mega")) wavefront = volwave = false;
    if (flags & MH_FLAG_MEGAKERNEL) wavefront = volwave = false;
    if ((flags & MH_FLAG_WAVEFRONT) && !wavefront && !volwave)
        return set_error(MH_ERR_UNSUPPORTED, "mh_render: the wavefront mode supports the 'path' integrator "
                                             "with max_depth <= 64 (several passes: packet-engine scenes) and "
                                             "'volpath' with max_depth <= 1024 (one pass)");
    uint64_t max_samples = volwave ? vw_max_chunk() : 1ull << 25;
    if (wavefront) {
        const char *ec = getenv("MH_WF_CHUNK");
        max_samples = std::min<uint64_t>(wf_max_chunk(), ec ? std::max<uint64_t>(1024, strtoull(ec, nullptr, 10)) : wf_max_chunk());
    }
    uint32_t chunk_px = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(n_px, max_samples / per_pixel));
    // (the unfused stream-engine kernels of large meshes too: stream2's launches
    // get their own stack overflow columns, S2 below)
    const bool two_ok = wavefront && !deterministic(flags) && !(flags & MH_FLAG_SHARED_DEVICE) &&
                        chunk_streams_enabled();
    if (two_ok && chunk_px >= n_px && n_px >= 2 && n_px * per_pixel >= kTwoStreamMinSamples)
        chunk_px = (uint32_t)((n_px + 1) / 2);
    const bool two = two_ok && chunk_px < n_px;
    const uint64_t plane = (uint64_t)chunk_px * per_pixel;
    MH_HIP(s->work.alloc(plane * (alpha ? 6 : 5) * sizeof(float)));
    if (two) MH_HIP(s->work2.alloc(plane * (alpha ? 6 : 5) * sizeof(float)));
    const bool fast_splat = L.spp_pp >= 4 && s->S.rfilter == MH_RFILTER_GAUSSIAN &&
                            s->S.rfilter_radius > 1.5f && s->S.rfilter_radius <= 2.5f;
    const int coalesce = L.spp_pp >= 4;
    const uint32_t seed_value = s->S.sampler_seed + seed;
    const bool determ = deterministic(flags);
    unsigned long long *invalid = s->counters.as<unsigned long long>() + kCtrInvalid;
    unsigned long long *bounds = s->counters.as<unsigned long long>() + kCtrBounds;
    float kernel_ms = 0.f, trace_ms = 0.f;
    const size_t n_chunks = (size_t)((n_px + chunk_px - 1) / chunk_px);
    const uint32_t n_bounces = wavefront ? in->max_depth : 0;
    const size_t ev_per_chunk = 3 + 2 * n_bounces;  // integrator span, bounce spans, splat end
    while (s->evpool.size() < ev_per_chunk * n_chunks) {
        hipEvent_t e;
        MH_HIP(hipEventCreate(&e));
        s->evpool.push_back(e);
    }
    const size_t ctr_words = wavefront ? wf_counter_words(n_bounces) : 0;  // per pass
    const size_t ctr_per_chunk = ctr_words * L.n_passes;
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, s->device);
    if (wavefront) {
        MH_HIP(s->wf_ws.alloc(wf_workspace_bytes(plane)));
        MH_HIP(s->wf_ctr.alloc(std::max<size_t>(16, ctr_per_chunk * n_chunks * 4)));
        if (L.n_passes > 1) MH_HIP(s->wf_carry.alloc((size_t)chunk_px * S_ * 8));
        if (two) {
            MH_HIP(s->wf_ws2.alloc(wf_workspace_bytes(plane)));
            if (L.n_passes > 1) MH_HIP(s->wf_carry2.alloc((size_t)chunk_px * S_ * 8));
        }
    }
    DScene S2 = s->S;  // stream2's scene view: its own stack overflow columns
    if (two && s->S.stack_ovf) {
        MH_HIP(s->stack_ovf2.alloc(s->stack_ovf.bytes));
        S2.stack_ovf = s->stack_ovf2.as<uint32_t>();
    }
    if (two) MH_HIP(fork_stream(s, st));
    if (volwave && !vol_sched_mode()) {
        MH_HIP(s->wf_ws.alloc(vw_workspace_bytes(plane)));
        MH_HIP(s->wf_ctr.alloc((size_t)vw_counter_words(vw_rounds(*in)) * 4));
    }
    size_t chunk = 0;
    for (uint64_t p0 = 0; p0 < n_px; p0 += chunk_px, ++chunk) {
        uint32_t npx = (uint32_t)std::min<uint64_t>(chunk_px, n_px - p0);
        LaneMap lm = lane_map(L, (uint32_t)p0);
        uint64_t n = (uint64_t)npx * S_;
        hipEvent_t *ev = &s->evpool[ev_per_chunk * chunk];
        const bool odd = two && (chunk & 1);
        const hipStream_t cs = odd ? s->stream2 : st;
        DevBuf &work = odd ? s->work2 : s->work;
        MH_HIP(hipEventRecord(ev[0], cs));
        {
        ScopedPhase sample_("SamplingIntegratorSample");
        if (wavefront) {
            MH_HIP(launch_wavefront(odd ? S2 : s->S, *in, lm, seed_value, n, plane, work.as<float>(),
                                    (odd ? s->wf_ws2 : s->wf_ws).ptr, plane,
                                    s->wf_ctr.as<uint32_t>() + ctr_per_chunk * chunk,
                                    n_bounces, wf_blocks(cus, two || (flags & MH_FLAG_SHARED_DEVICE) != 0), ev + 2, cs,
                                    L.n_passes,
                                    L.n_passes > 1 ? (odd ? s->wf_carry2 : s->wf_carry).as<uint64_t>() : nullptr,
                                    alpha));
        } else if (volwave && vol_sched_mode()) {
            MH_HIP(launch_vol_sched(s->S, *in, lm, seed_value, n, plane, s->work.as<float>(), vs_blocks(cus),
                                    s->counters.as<unsigned long long>(), st, alpha));
        } else if (volwave) {
            MH_HIP(launch_volwave(s->S, *in, lm, seed_value, n, plane, s->work.as<float>(), s->wf_ws.ptr, plane,
                                  s->wf_ctr.as<uint32_t>(), vw_blocks(cus), s->counters.as<unsigned long long>(),
                                  st, alpha));
        } else {
            MH_HIP(launch_render(s->S, *in, lm, seed_value, L.n_passes, n, plane, s->work.as<float>(),
                                 s->counters.as<unsigned long long>(), st, alpha));
        }
        }
        MH_HIP(hipEventRecord(ev[1], cs));
        ScopedPhase put_("ImageBlockPut");
        MH_SPLAT(s->S, lm, kSplatFilm, fast_splat, npx, L.n_passes, n, plane, work.as<float>(), film4,
                 seed_value, coalesce, cs, invalid, determ, work.bytes / 4, n_px * 4, bounds);
        if (alpha)
            MH_SPLAT(s->S, lm, kSplatAlpha, fast_splat, npx, L.n_passes, n, plane, work.as<float>(), film_a,
                     seed_value, coalesce, cs, nullptr, determ, work.bytes / 4, n_px, bounds);
        MH_HIP(hipEventRecord(ev[ev_per_chunk - 1], cs));
    }
    if (two) MH_HIP(join_stream(s, st));
    if (alpha) MH_HIP(launch_film_rgbaw(n_px, film4, film_a, film, st));
    if (int rc = reduce_result(s, flags, film, film_bytes / 4, st, true)) return rc;
    if (!(flags & MH_FLAG_DEVICE_POINTERS))
        MH_HIP(hipMemcpyAsync(film_rgbw, film, film_bytes, hipMemcpyDeviceToHost, st));
    // asynchronous call (device film, no stats): return once the work is
    // enqueued on the scene's stream, as a stream-ordered library op does
    if (async_call(flags, stats)) return MH_OK;
    if (!stats && !getenv("MH_VW_DEBUG")) {  // nothing to read back: the call's own sync + the bounds word
        MH_WAIT(s, flags, st);
        return check_bounds_counter(s, "mh_render");
    }
    unsigned long long ctr[2] = {0, 0}, n_invalid = 0, n_lookups = 0;
    std::vector<uint32_t> wctr;
    if (wavefront) {
        wctr.resize(ctr_per_chunk * n_chunks);
        MH_HIP(hipMemcpyAsync(wctr.data(), s->wf_ctr.ptr, wctr.size() * 4, hipMemcpyDeviceToHost, st));
    } else {
        MH_HIP(hipMemcpyAsync(ctr, s->counters.ptr, sizeof(ctr), hipMemcpyDeviceToHost, st));
    }
    unsigned long long iv[2] = {0, 0};  // [kCtrInvalid], [kCtrBounds]
    static_assert(kCtrBounds == kCtrInvalid + 1, "one read-back of both words");
    MH_HIP(hipMemcpyAsync(iv, invalid, sizeof(iv), hipMemcpyDeviceToHost, st));
    if (volwave && vol_sched_mode())
        MH_HIP(hipMemcpyAsync(&n_lookups, s->counters.as<unsigned long long>() + kCtrLookups, 8,
                              hipMemcpyDeviceToHost, st));
    MH_WAIT(s, flags, st);  // the stats counters are read back
    n_invalid = iv[0];
    if (iv[1])
        return set_error(MH_ERR_HIP, "mh_render: " + std::to_string(iv[1]) +
                                         " splat rows would have read past the sample planes (skipped)");
    float splat_ms = 0.f;
    for (size_t c = 0; c < n_chunks; ++c) {
        hipEvent_t *ev = &s->evpool[ev_per_chunk * c];
        float ms = 0.f;
        MH_HIP(hipEventElapsedTime(&ms, ev[0], ev[1]));
        kernel_ms += ms;
        MH_HIP(hipEventElapsedTime(&ms, ev[1], ev[ev_per_chunk - 1]));
        splat_ms += ms;
        // the fused bounce kernels are timed as one span (launch_wavefront_pass)
        const uint32_t pairs = wavefront ? (wf_fused(s->S) || L.n_passes > 1 ? 1u : n_bounces) : 0u;
        for (uint32_t b = 0; b < pairs; ++b) {
            MH_HIP(hipEventElapsedTime(&ms, ev[2 + 2 * b], ev[3 + 2 * b]));
            trace_ms += ms;
        }
    }
    if (wavefront) {
        const size_t per_bounce = ctr_words / (n_bounces + 1), nseg = per_bounce / 32;
        for (size_t c = 0; c < n_chunks; ++c)
            for (uint32_t p = 0; p < L.n_passes; ++p)
                for (uint32_t b = 0; b < n_bounces; ++b)
                    for (size_t sg = 0; sg < nseg; ++sg) {
                        const size_t o = ctr_per_chunk * c + ctr_words * p + per_bounce * b + 32 * sg;
                        ctr[0] += wctr[o + 0];
                        ctr[1] += wctr[o + 1];
                    }
    }
    if (volwave && vol_sched_mode() && getenv("MH_VW_DEBUG"))  // MH_EXP_VSCNT builds: wave trips per phase
        if (int rc2 = print_vs_phases(s)) return rc2;
    if (volwave && !vol_sched_mode() && getenv("MH_VW_DEBUG")) {  // per-round queue sizes (+ MH_EXP_VWCNT builds: trips / steps)
        const uint32_t R = vw_rounds(*in), W = vw_counter_words(R) / (R + 1);
        std::vector<uint32_t> c((size_t)W * (R + 1));
        MH_HIP(hipMemcpy(c.data(), s->wf_ctr.ptr, c.size() * 4, hipMemcpyDeviceToHost));
        for (uint32_t r = 1; r <= R; ++r) {
            unsigned long long q = 0, trips = 0, steps = 0, it_m = 0, it_w = 0;
            for (uint32_t g = 0; g < W / 32; ++g) {
                const uint32_t *w = &c[(size_t)W * r + 32 * g];
                q += w[0];
                trips += w[2] | ((unsigned long long)w[3] << 32);
                steps += w[4] | ((unsigned long long)w[5] << 32);
                it_m += w[6];
                it_w += w[7];
            }
            if (q || trips) fprintf(stderr, "vw round %u: walks %llu, main trips %llu (wave iters %llu), walk steps %llu (wave iters %llu)\n",
                                    r - 1, q, trips, it_m, steps, it_w);
        }
    }
    if (stats) {
        stats->samples = n_px * per_pixel;
        stats->rays_closest = ctr[0];
        stats->rays_shadow = ctr[1];
        stats->bounces = ctr[0];
        stats->ms_total = now_ms() - t_start;
        stats->ms_kernel = kernel_ms;
        // volpath on the phase scheduler: its k_vol_sched launches (one per chunk)
        const bool sched = volwave && vol_sched_mode();
        stats->ms_trace = sched ? kernel_ms : trace_ms;
        stats->n_trace_launches = wavefront ? (uint64_t)n_chunks * n_bounces * L.n_passes : sched ? n_chunks : 0;
        stats->mode = wavefront ? (wf_fused(s->S) ? 2u : 1u) : volwave ? 3u : 0u;
        stats->invalid_samples = (uint32_t)std::min<unsigned long long>(n_invalid, 0xffffffffull);
        stats->grid_lookups = n_lookups;
        stats->aux_items = n_px * per_pixel;
        stats->ms_aux = splat_ms;
        stats->n_aux_launches = n_chunks;
    }
    return MH_OK;
}

int mh_render_samples(mh_scene *s, const mh_integrator *in, uint32_t seed, uint32_t spp,
                      uint32_t spp_begin, uint32_t spp_end, float *out, uint32_t flags) {
    ScopedPhase phase_("Render");
    if (!s || !in || !out) return set_error(MH_ERR_INVALID_ARGUMENT, "mh_render_samples: NULL argument");
    if (in->type > MH_INTEGRATOR_PRBVOLPATH)
        return set_error(MH_ERR_UNSUPPORTED, "mh_render_samples: unsupported integrator");
    if (spp == 0 || in->rr_depth == 0) return set_error(MH_ERR_INVALID_ARGUMENT, "mh_render_samples: bad arguments");
    Layout L;
    const bool ad = in->type == MH_INTEGRATOR_PRB || in->type == MH_INTEGRATOR_PRBVOLPATH;
    int rc = make_layout(s, spp, spp_begin, spp_end, L, ad);
    if (rc) return rc;
    if (L.n_passes != 1) return set_error(MH_ERR_UNSUPPORTED, "mh_render_samples: single pass only");
    MH_HIP(hipSetDevice(s->device));
    hipStream_t st = s->stream;
    const uint64_t n = (uint64_t)L.W * L.H * (L.s_end - L.s_begin);
    const bool alpha = has_alpha(s->pixel_format);
    const size_t out_bytes = n * (alpha ? 24 : 20);
    float *dst = out;
    if (!(flags & MH_FLAG_DEVICE_POINTERS)) {
        MH_HIP(s->tmp_a.alloc(out_bytes));
        dst = s->tmp_a.as<float>();
    }
    MH_HIP(hipMemsetAsync(s->counters.ptr, 0, 256, st));
    LaneMap lm = lane_map(L, 0);
    if ((flags & MH_FLAG_WAVEFRONT) && vs_supported(s->S, *in) && vol_sched_mode()) {
        int cus = 256;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, s->device);
        MH_HIP(launch_vol_sched(s->S, *in, lm, s->S.sampler_seed + seed, n, n, dst, vs_blocks(cus),
                                s->counters.as<unsigned long long>(), st, alpha));
    } else if ((flags & MH_FLAG_WAVEFRONT) && vw_supported(s->S, *in)) {
        int cus = 256;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, s->device);
        MH_HIP(s->wf_ws.alloc(vw_workspace_bytes(n)));
        MH_HIP(s->wf_ctr.alloc((size_t)vw_counter_words(vw_rounds(*in)) * 4));
        MH_HIP(launch_volwave(s->S, *in, lm, s->S.sampler_seed + seed, n, n, dst, s->wf_ws.ptr, n,
                              s->wf_ctr.as<uint32_t>(), vw_blocks(cus), s->counters.as<unsigned long long>(), st,
                              alpha));
    } else if (flags & MH_FLAG_WAVEFRONT) {
        if (in->type != MH_INTEGRATOR_PATH || in->max_depth > 64)
            return set_error(MH_ERR_UNSUPPORTED, "mh_render_samples: wavefront mode needs 'path' (max_depth <= 64) "
                                                 "or 'volpath' (max_depth <= 1024)");
        int cus = 256;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, s->device);
        MH_HIP(s->wf_ws.alloc(wf_workspace_bytes(n)));
        MH_HIP(s->wf_ctr.alloc(std::max<size_t>(16, 4 * (size_t)wf_counter_words(in->max_depth))));
        MH_HIP(launch_wavefront(s->S, *in, lm, s->S.sampler_seed + seed, n, n, dst, s->wf_ws.ptr, n,
                                s->wf_ctr.as<uint32_t>(), in->max_depth, wf_blocks(cus), nullptr, st, 1, nullptr,
                                alpha));
    } else {
        MH_HIP(launch_render(s->S, *in, lm, s->S.sampler_seed + seed, 1, n, n, dst,
                             s->counters.as<unsigned long long>(), st, alpha));
    }
    if (!(flags & MH_FLAG_DEVICE_POINTERS))
        MH_HIP(hipMemcpyAsync(out, dst, out_bytes, hipMemcpyDeviceToHost, st));
    MH_HIP(hipStreamSynchronize(st));
    return MH_OK;
}

int mh_develop(mh_scene *s, const float *film_rgbw, float *image_rgb, uint32_t flags) {
    if (!s || !film_rgbw || !image_rgb) return set_error(MH_ERR_INVALID_ARGUMENT, "mh_develop: NULL argument");
    MH_HIP(hipSetDevice(s->device));
    hipStream_t st = s->stream;
    const uint64_t n_px = (uint64_t)s->S.width * s->S.height;
    const uint32_t fmt = s->pixel_format, ch = image_channels(fmt);
    const size_t film_bytes = n_px * (has_alpha(fmt) ? 20 : 16);
    if (flags & MH_FLAG_DEVICE_POINTERS) {
        MH_HIP(launch_develop(n_px, film_rgbw, image_rgb, fmt, st));
        if (!(flags & MH_FLAG_NO_SYNC)) MH_HIP(hipStreamSynchronize(st));
        return MH_OK;
    }
    MH_HIP(s->tmp_a.alloc(film_bytes));
    MH_HIP(s->tmp_b.alloc(n_px * 4 * ch));
    MH_HIP(hipMemcpyAsync(s->tmp_a.ptr, film_rgbw, film_bytes, hipMemcpyHostToDevice, st));
    MH_HIP(launch_develop(n_px, s->tmp_a.as<float>(), s->tmp_b.as<float>(), fmt, st));
    MH_HIP(hipMemcpyAsync(image_rgb, s->tmp_b.ptr, n_px * 4 * ch, hipMemcpyDeviceToHost, st));
    MH_HIP(hipStreamSynchronize(st));
    return MH_OK;
}

// ---------------------------------------------------------------------------
// PRB backward
// ---------------------------------------------------------------------------
static int prb_weights_impl(mh_scene *s, uint32_t seed, uint32_t spp, uint32_t spp_begin, uint32_t spp_end,
                   float *weights, uint32_t flags) {
    ScopedPhase phase_("ImageBlockPut");
    if (!s || !weights) return set_error(MH_ERR_INVALID_ARGUMENT, "mh_prb_weights: NULL argument");
    if (spp == 0) return set_error(MH_ERR_INVALID_ARGUMENT, "mh_prb_weights: spp must be > 0");
    if (int rc = check_reduce_flags(s, flags, "mh_prb_weights", true)) return rc;
    Layout L;
    int rc = make_layout(s, spp, spp_begin, spp_end, L, true);
    if (rc) return rc;
    MH_HIP(hipSetDevice(s->device));
    g_call_issued = true;  // past argument validation: a failure from here aborts the communicator
    hipStream_t st = s->stream;
    const uint64_t n_px = (uint64_t)L.W * L.H;
    float *w = weights;
    if (!(flags & MH_FLAG_DEVICE_POINTERS)) {
        MH_HIP(s->weights_tmp.alloc(n_px * 4));
        w = s->weights_tmp.as<float>();
    }
    if (!(flags & MH_FLAG_ACCUMULATE)) MH_HIP(hipMemsetAsync(w, 0, n_px * 4, st));
    const bool fast = L.spp_pp >= 4 && s->S.rfilter == MH_RFILTER_GAUSSIAN &&
                      s->S.rfilter_radius > 1.5f && s->S.rfilter_radius <= 2.5f;
    LaneMap lm = lane_map(L, 0);
    const uint32_t S_ = L.s_end - L.s_begin;
    MH_SPLAT(s->S, lm, kSplatWeights, fast, (uint32_t)n_px, 1, n_px * S_, 0, nullptr, w, s->S.sampler_seed + seed,
             L.spp_pp >= 4, st, nullptr, deterministic(flags), 0, n_px, nullptr);
    if (int rc = reduce_result(s, flags, w, n_px, st, false)) return rc;
    if (!(flags & MH_FLAG_DEVICE_POINTERS))
        MH_HIP(hipMemcpyAsync(weights, w, n_px * 4, hipMemcpyDeviceToHost, st));
    if (!async_call(flags, nullptr)) MH_WAIT(s, flags, st);
    return MH_OK;
}

// ---------------------------------------------------------------------------
// Differentiated parameters -> slots: small slots 0..n_rgb-1 (register
// accumulators): rgb textures, medium albedo, homogeneous sigma_t; large
// slots (global atomics / tangent arrays): bitmaps, grids
// ---------------------------------------------------------------------------
struct Slots {
    std::vector<int32_t> slot_of_tex, sigma_slot, albedo_slot;
    std::vector<uint32_t> is_rgb;
    std::vector<size_t> counts;
    std::vector<uint32_t> slot_of_param;
    uint32_t n_rgb = 0, n_bmp = 0, n_medium_params = 0, bmp_tex = 0;
    uint32_t grid_res[kMaxParams][3] = {};  // large sigma_t slots: the grid's resolution (x, y, z)
    std::vector<float *> corner;            // their corner blocks (upload_slots, corners = true)
    bool fx = false;                        // the blocks hold int64 fixed point (deterministic)
    std::vector<uint8_t> meta;  // host image of the meta block (uploaded by upload_slots when it changed)
};

static int build_slots(const mh_scene *s, uint32_t n_params, const uint32_t *param_tex, bool vol, const char *api,
                       const char *method, Slots &P) {
    const std::string a(api), m(method);
    P.slot_of_tex.assign(std::max<uint32_t>(s->n_textures, 1), -1);
    P.sigma_slot.assign(std::max<uint32_t>(s->n_media, 1), -1);
    P.albedo_slot = P.sigma_slot;
    P.is_rgb.assign(kMaxParams, 0);
    P.counts.assign(kMaxParams, 0);
    P.slot_of_param.assign(n_params, 0);
    for (uint32_t k = 0; k < n_params; ++k) {
        const uint32_t kind = param_tex[k] & MH_PARAM_KIND_MASK, idx = param_tex[k] & ~MH_PARAM_KIND_MASK;
        int32_t *owner;
        bool small;
        size_t cnt;
        if (kind == 0) {
            if (idx >= s->n_textures) return set_error(MH_ERR_INVALID_ARGUMENT, a + ": texture index out of bounds");
            const DTexture &tx = s->h_textures[idx];
            owner = &P.slot_of_tex[idx];
            small = tx.type == MH_TEX_RGB;
            cnt = small ? 3 : (size_t)tx.width * tx.height * tx.channels;
        } else if (kind == MH_PARAM_MEDIUM_SIGMA_T || kind == MH_PARAM_MEDIUM_ALBEDO) {
            if (!vol)
                return set_error(MH_ERR_UNSUPPORTED, m + "(): medium parameters require the 'prbvolpath' integrator");
            if (idx >= s->n_media) return set_error(MH_ERR_INVALID_ARGUMENT, a + ": medium index out of bounds");
            const mh_medium &md = s->h_media[idx];
            ++P.n_medium_params;
            if (kind == MH_PARAM_MEDIUM_ALBEDO) {
                owner = &P.albedo_slot[idx]; small = true; cnt = 3;
            } else {
                owner = &P.sigma_slot[idx];
                small = md.type == MH_MEDIUM_HOMOGENEOUS;
                cnt = small ? 1 : (size_t)md.grid_res[0] * md.grid_res[1] * md.grid_res[2];
            }
        } else {
            return set_error(MH_ERR_INVALID_ARGUMENT, a + ": unknown parameter kind");
        }
        if (*owner >= 0) return set_error(MH_ERR_INVALID_ARGUMENT, a + ": duplicate parameter");
        int slot;
        if (small) {
            if (P.n_rgb >= (uint32_t)kMaxRgbParams) return set_error(MH_ERR_UNSUPPORTED, a + ": too many rgb parameters");
            slot = (int)P.n_rgb++;
            P.is_rgb[slot] = 1;
        } else {
            if (P.n_bmp >= (uint32_t)kMaxBitmapParams) return set_error(MH_ERR_UNSUPPORTED, a + ": too many bitmap parameters");
            slot = kMaxRgbParams + (int)P.n_bmp++;
            if (kind == 0) P.bmp_tex = idx;
        }
        P.counts[slot] = cnt;
        if (kind == MH_PARAM_MEDIUM_SIGMA_T && !small)
            for (int a = 0; a < 3; ++a) P.grid_res[slot][a] = s->h_media[idx].grid_res[a];
        *owner = slot;
        P.slot_of_param[k] = (uint32_t)slot;
    }
    return MH_OK;
}

// per-slot device buffers (s->tmp_c, zeroed) and the meta block
// slot_of_tex | is_rgb | bufs | sigma_slot | albedo_slot (s->grad_meta)
// corners: the grid sigma_t slots scatter into per-cell corner blocks
// (s->grid_corner, zeroed; launch_corner_gather after the backward) unless
// MH_GRID_CORNER=0, the block would exceed 16 GiB or cannot be allocated
// fx: MH_FLAG_DETERMINISTIC -- int64 corner blocks (twice the bytes), which
// are then required (no direct-atomic fallback)
static hipError_t upload_slots(mh_scene *s, Slots &P, hipStream_t st, std::vector<float *> &bufs, GradArgs &ga,
                               bool corners = false, bool fx = false) {
    size_t total = 0;
    std::vector<size_t> off(kMaxParams, 0);
    for (int k = 0; k < kMaxParams; ++k) { off[k] = total; total += (P.counts[k] + 3) / 4 * 4; }
    hipError_t e = s->tmp_c.alloc(std::max<size_t>(total, 1) * 4);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(s->tmp_c.ptr, 0, std::max<size_t>(total, 1) * 4, st);
    if (e != hipSuccess) return e;
    bufs.assign(kMaxParams, nullptr);
    for (int k = 0; k < kMaxParams; ++k) bufs[k] = P.counts[k] ? s->tmp_c.as<float>() + off[k] : nullptr;
    P.corner.assign(kMaxParams, nullptr);
    const char *ec = getenv("MH_GRID_CORNER");
    P.fx = false;
    if (corners && (fx || !(ec && !strcmp(ec, "0")))) {
        std::vector<size_t> coff(kMaxParams, 0);
        std::vector<bool> use(kMaxParams, false);
        size_t cfl = 0;
        for (int k = 0; k < kMaxParams; ++k) {
            const uint32_t *r = P.grid_res[k];
            use[k] = r[0] && (uint64_t)(r[0] + 1) * (r[1] + 1) * (r[2] + 1) < (1ull << 32);
            coff[k] = cfl;
            if (use[k]) cfl += corner_floats(r);
        }
        const size_t eb = fx ? 8 : 4;  // bytes per corner value
        if (cfl && cfl * eb <= (32ull << 30) && (fx || cfl * 4 <= (16ull << 30)) &&
            s->grid_corner.alloc(cfl * eb) == hipSuccess) {
            e = hipMemsetAsync(s->grid_corner.ptr, 0, cfl * eb, st);
            if (e != hipSuccess) return e;
            for (int k = 0; k < kMaxParams; ++k)
                if (use[k]) P.corner[k] = reinterpret_cast<float *>(s->grid_corner.as<uint8_t>() + coff[k] * eb);
            P.fx = fx;
        } else {
            (void)hipGetLastError();
        }
    }
    auto al16 = [](size_t x) { return (x + 15) / 16 * 16; };
    const size_t o_slot = 0, o_isrgb = al16(P.slot_of_tex.size() * 4), o_bufs = al16(o_isrgb + kMaxParams * 4),
                 o_sig = al16(o_bufs + kMaxParams * 8), o_alb = al16(o_sig + P.sigma_slot.size() * 4),
                 o_cor = al16(o_alb + P.albedo_slot.size() * 4), meta_bytes = al16(o_cor + kMaxParams * 8);
    std::vector<uint8_t> &meta = P.meta;
    meta.assign(meta_bytes, 0);
    memcpy(meta.data() + o_slot, P.slot_of_tex.data(), P.slot_of_tex.size() * 4);
    memcpy(meta.data() + o_isrgb, P.is_rgb.data(), kMaxParams * 4);
    memcpy(meta.data() + o_bufs, bufs.data(), kMaxParams * 8);
    memcpy(meta.data() + o_sig, P.sigma_slot.data(), P.sigma_slot.size() * 4);
    memcpy(meta.data() + o_alb, P.albedo_slot.data(), P.albedo_slot.size() * 4);
    memcpy(meta.data() + o_cor, P.corner.data(), kMaxParams * 8);
    // uploaded only when it changes (a new parameter set or reallocated slot
    // buffers), then with a stream sync; repeated calls with the same
    // parameters stay asynchronous
    if (!(s->grad_meta.ptr && s->meta_host == meta)) {
        e = s->grad_meta.alloc(meta_bytes);
        if (e != hipSuccess) return e;
        e = hipMemcpyAsync(s->grad_meta.ptr, meta.data(), meta_bytes, hipMemcpyHostToDevice, st);
        if (e != hipSuccess) return e;
        e = hipStreamSynchronize(st);
        if (e != hipSuccess) return e;
        s->meta_host = meta;
    }
    const uint8_t *mb = s->grad_meta.as<uint8_t>();
    ga.slot_of_tex = reinterpret_cast<const int32_t *>(mb + o_slot);
    ga.is_rgb = reinterpret_cast<const uint32_t *>(mb + o_isrgb);
    ga.bufs = reinterpret_cast<float *const *>(mb + o_bufs);
    ga.n_rgb = P.n_rgb;
    ga.sigma_slot = P.n_medium_params ? reinterpret_cast<const int32_t *>(mb + o_sig) : nullptr;
    ga.albedo_slot = P.n_medium_params ? reinterpret_cast<const int32_t *>(mb + o_alb) : nullptr;
    bool any_corner = false;
    for (float *c : P.corner) any_corner = any_corner || c;
    ga.corner = any_corner ? reinterpret_cast<float *const *>(mb + o_cor) : nullptr;
    ga.hot_med = ga.hot_sigma = ga.hot_albedo = -1;
    ga.hot_buf = ga.hot_corner = nullptr;
    for (size_t m = 0; m < P.sigma_slot.size() && P.n_medium_params; ++m) {
        if (P.sigma_slot[m] < 0 && P.albedo_slot[m] < 0) continue;
        ga.hot_med = (int32_t)m;
        ga.hot_sigma = P.sigma_slot[m];
        ga.hot_albedo = P.albedo_slot[m];
        if (ga.hot_sigma >= 0) {
            ga.hot_buf = bufs[ga.hot_sigma];
            ga.hot_corner = P.corner[ga.hot_sigma];
        }
        break;
    }
    return hipSuccess;
}

static int render_backward_impl(mh_scene *s, const mh_integrator *in, uint32_t seed, uint32_t spp,
                       uint32_t spp_begin, uint32_t spp_end, const float *grad_in,
                       const float *weights, uint32_t n_params, const uint32_t *param_tex,
                       float *const *grads, uint32_t flags, mh_stats *stats) {
    ScopedPhase phase_("RenderBackward");
    if (!s || !in || !grad_in || (n_params && (!param_tex || !grads)))
        return set_error(MH_ERR_INVALID_ARGUMENT, "mh_render_backward: NULL argument");
    if (in->type != MH_INTEGRATOR_PRB && in->type != MH_INTEGRATOR_PRBVOLPATH)
        return set_error(MH_ERR_UNSUPPORTED, "render_backward(): requires the 'prb' or 'prbvolpath' integrator");
    const bool vol = in->type == MH_INTEGRATOR_PRBVOLPATH;
    if (in->rr_depth == 0)
        return set_error(MH_ERR_INVALID_ARGUMENT, "\"rr_depth\" must be set to a value greater than zero!");
    if (spp == 0) return set_error(MH_ERR_INVALID_ARGUMENT, "mh_render_backward: spp must be > 0");
    if (int rc = check_reduce_flags(s, flags, "mh_render_backward", false)) return rc;
    double t_start = now_ms();
    if (stats) *stats = mh_stats{};
    Layout L;
    int rc = make_layout(s, spp, spp_begin, spp_end, L, true);
    if (rc) return rc;
    MH_HIP(hipSetDevice(s->device));
    g_call_issued = true;  // past argument validation: a failure from here aborts the communicator
    hipStream_t st = s->stream;
    const uint64_t n_px = (uint64_t)L.W * L.H;
    const bool dev = flags & MH_FLAG_DEVICE_POINTERS;

    // ---- parameter slots ----
    Slots P;
    int rc_slots = build_slots(s, n_params, param_tex, vol, "mh_render_backward", "render_backward", P);
    if (rc_slots) return rc_slots;
    std::vector<float *> bufs;
    GradArgs ga;
    // MH_FLAG_DETERMINISTIC on prbvolpath: the grid gradient and the small
    // slots in int64 fixed point (two passes, see the prbvolpath branch below)
    const bool fx = vol && deterministic(flags);  // also the small slots (acc_add_fx)
    MH_HIP(upload_slots(s, P, st, bufs, ga, vol, fx));
    if (fx)
        for (int k = 0; k < kMaxParams; ++k)
            if (P.grid_res[k][0] && !P.corner[k])
                return set_error(MH_ERR_OUT_OF_MEMORY,
                                 "render_backward(): the deterministic grid gradient's corner block could not be allocated");
    const std::vector<size_t> &counts = P.counts;
    const std::vector<uint32_t> &slot_of_param = P.slot_of_param;
    const uint32_t n_rgb = P.n_rgb, n_bmp = P.n_bmp, bmp_tex = P.bmp_tex;
    // one bitmap parameter of <= 48 KiB: the replay kernel accumulates its
    // texel gradients per workgroup in LDS (k_prb_backward)
    // (MH_PRB_LDS_TEX=0: global atomics, the parity tests' cross-check)
    const char *env_lds = getenv("MH_PRB_LDS_TEX");
    if (n_bmp == 1 && counts[kMaxRgbParams] * 4 <= (48u << 10) && !(env_lds && !strcmp(env_lds, "0"))) {
        ga.lds_slot = kMaxRgbParams;
        ga.lds_floats = (uint32_t)counts[kMaxRgbParams];
    }

    // ---- grad_in / weights on the device ----
    const float *g_in = grad_in;
    if (!dev) {
        MH_HIP(s->tmp_d.alloc(n_px * 12));
        MH_HIP(hipMemcpyAsync(s->tmp_d.ptr, grad_in, n_px * 12, hipMemcpyHostToDevice, st));
        g_in = s->tmp_d.as<float>();
    }
    const float *w = weights;
    if (!weights) {
        MH_HIP(s->weights_tmp.alloc(n_px * 4));
        MH_HIP(hipMemsetAsync(s->weights_tmp.ptr, 0, n_px * 4, st));
        const bool fast = L.spp_pp >= 4 && s->S.rfilter == MH_RFILTER_GAUSSIAN &&
                          s->S.rfilter_radius > 1.5f && s->S.rfilter_radius <= 2.5f;
        // W of every sample of every pixel (common.py:936-947); with
        // MH_FLAG_REDUCE the slab's own samples + an all-reduce, unless each
        // rank is to compute the whole image itself (MH_FLAG_LOCAL_WEIGHTS)
        const bool slab_w = wants_reduce(flags) && !(flags & MH_FLAG_LOCAL_WEIGHTS);
        Layout Lall = L;
        if (!slab_w) {
            Lall.s_begin = 0;
            Lall.s_end = L.spp_pp;
        }
        LaneMap lmw = lane_map(Lall, 0);
        MH_SPLAT(s->S, lmw, kSplatWeights, fast, (uint32_t)n_px, 1, n_px * (Lall.s_end - Lall.s_begin), 0, nullptr,
                 s->weights_tmp.as<float>(), s->S.sampler_seed + seed, L.spp_pp >= 4, st, nullptr,
                 deterministic(flags), 0, n_px, nullptr);
        if (slab_w)
            if (int rc = reduce_result(s, flags, s->weights_tmp.as<float>(), n_px, st, false)) return rc;
        w = s->weights_tmp.as<float>();
    } else if (!dev) {
        MH_HIP(s->tmp_e.alloc(n_px * 4));
        MH_HIP(hipMemcpyAsync(s->tmp_e.ptr, weights, n_px * 4, hipMemcpyHostToDevice, st));
        w = s->tmp_e.as<float>();
    }

    MH_HIP(hipMemsetAsync(s->counters.ptr, 0, 256, st));
    // grad_in / W once per pixel (the adjoint of develop)
    MH_HIP(s->gw.alloc(n_px * 16));  // float4 per pixel (k_grad_over_w)
    MH_HIP(launch_grad_over_w(n_px, g_in, w, s->gw.as<float>(), st));
    g_in = s->gw.as<float>();
    const uint32_t S_ = L.s_end - L.s_begin;
    const uint64_t n = n_px * S_;
    // fused single traversal when every requested parameter is an rgb constant,
    // unless the replay is forced (MH_FLAG_PRB_REPLAY / MH_PRB_REPLAY=1); the
    // fused form runs as wavefront kernels unless MH_FLAG_MEGAKERNEL / MH_MODE=mega
    const char *env_replay = getenv("MH_PRB_REPLAY");
    const char *env_mode = getenv("MH_MODE");
    const bool replay = (flags & MH_FLAG_PRB_REPLAY) || (env_replay && !strcmp(env_replay, "1"));
    const bool mega = (flags & MH_FLAG_MEGAKERNEL) || (env_mode && !strcmp(env_mode, "mega"));
    const bool fused = !vol && n_bmp == 0 && !replay;
    // bitmap parameters: the fused PRB wavefront logs their vertices (with the
    // bitmap's index) and a scatter pass charges the texels (WfBmp,
    // mh_wavefront.hip) -- packet-engine scenes, max_depth <= 32
    // (MH_PRB_BMP_WF=0: the replay megakernel)
    const char *env_bwf = getenv("MH_PRB_BMP_WF");
    const char *env_pvl = getenv("MH_PVP_NEE_LOG");  // 0: prbvolpath replays its NEE walks (no log)
    // (several bitmaps: all with the same channel count, as the scatter's
    // transposed issue assumes)
    bool bmp_same_ch = true;
    {
        uint32_t ch = 0;
        for (uint32_t t = 0; t < (uint32_t)P.slot_of_tex.size(); ++t)
            if (P.slot_of_tex[t] >= kMaxRgbParams) {
                const uint32_t c = s->h_textures[t].channels;
                bmp_same_ch = bmp_same_ch && (ch == 0 || ch == c);
                ch = c;
            }
    }
    const bool bmp_wf = !vol && n_bmp >= 1 && bmp_same_ch && !replay && !mega && wf_fused(s->S) &&
                        in->max_depth >= 1 && in->max_depth <= 32 && !(env_bwf && !strcmp(env_bwf, "0"));
    const bool wavefront = ((fused && in->max_depth <= 64 && !mega) || bmp_wf);
    // MH_FLAG_DETERMINISTIC on the replay kernel (bitmaps the wavefront cannot
    // take, MH_FLAG_PRB_REPLAY, megakernel): the int64 two-pass form of
    // prbvolpath -- small slots through acc_add_fx, bitmap texels through
    // bmp_add_fx into an int64 mirror of the slot block (no LDS accumulator)
    const bool det_replay = deterministic(flags) && !vol && !wavefront;
    const bool fxr = fx || det_replay;
    if (det_replay) {
        size_t total = 0;
        for (int k = 0; k < kMaxParams; ++k) total += (counts[k] + 3) / 4 * 4;
        MH_HIP(s->replay_fx.alloc(std::max<size_t>(total, 1) * 8));
        MH_HIP(hipMemsetAsync(s->replay_fx.ptr, 0, std::max<size_t>(total, 1) * 8, st));
        ga.fx_i64 = s->replay_fx.as<long long>();
        ga.fx_f32 = s->tmp_c.as<float>();
        ga.lds_slot = -1;
    }
    size_t wf_ctr_words = 0, wf_chunks = 0;
    uint32_t *pvb_lost = nullptr;  // prbvolpath on the scheduler: overflow entries that found their list full
    double fx_inv = 1.0;           // deterministic grid gradient: 2^-S of the fixed point
    double fx_small_inv[kMaxParams] = {1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0};  // and of each slot
    // between the two passes of the deterministic grid gradient: the scale
    // from pass 1's largest |item|; pass 1's rgb-slot adds and counters go
    // fx_word: u32 max[0] (grid) and max[1 + k] (small slot k), double
    // scale[k] at byte 64, int64 sums[3 k + c] at byte 192 (acc_add_fx)
    auto fx_exp = [](uint32_t bits) {  // 2^S with |item| * 2^S < 2^31
        float mx;
        memcpy(&mx, &bits, 4);
        int ex = 0;
        if (mx > 0.f && std::isfinite(mx)) (void)std::frexp(mx, &ex);  // mx < 2^ex
        return 31 - ex;
    };
    auto fx_between = [&](GradArgs &gp) -> hipError_t {
        uint32_t mb[1 + kMaxParams] = {};  // words 1 + k: slot k (small slots; bitmaps on the replay)
        hipError_t e = hipMemcpyAsync(mb, s->fx_word.ptr, sizeof(mb), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = wait_stream(s, flags, st);
        if (e != hipSuccess) return e;
        const int S0 = fx_exp(mb[0]);
        fx_inv = std::ldexp(1.0, -S0);
        gp.fx_scale = std::ldexp(1.0, S0);
        double sc[kMaxParams];
        for (int k = 0; k < kMaxParams; ++k) {
            fx_small_inv[k] = std::ldexp(1.0, -fx_exp(mb[1 + k]));
            sc[k] = std::ldexp(1.0, fx_exp(mb[1 + k]));
        }
        e = hipMemcpyAsync(s->fx_word.as<uint8_t>() + 64, sc, sizeof(sc), hipMemcpyHostToDevice, st);
        if (e == hipSuccess) e = hipMemsetAsync(s->fx_word.as<uint8_t>() + 192, 0, 8 * 3 * kMaxRgbParams, st);
        size_t total = 0;
        for (int k = 0; k < kMaxParams; ++k) total += (counts[k] + 3) / 4 * 4;
        if (e == hipSuccess) e = hipMemsetAsync(s->tmp_c.ptr, 0, std::max<size_t>(total, 1) * 4, st);
        if (e == hipSuccess) e = hipMemsetAsync(s->counters.ptr, 0, 256, st);
        return e;
    };
    // after pass 2: the small slots' exact sums into their buffers (which
    // pass 2 left at zero: acc_add_fx bypasses the register accumulators)
    auto fx_small_fold = [&]() -> hipError_t {
        long long w[3 * kMaxRgbParams];
        hipError_t e = hipMemcpyAsync(w, s->fx_word.as<uint8_t>() + 192, sizeof(w), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = wait_stream(s, flags, st);
        for (uint32_t k = 0; e == hipSuccess && k < n_rgb; ++k) {
            float v[3];
            for (int c = 0; c < 3; ++c) v[c] = (float)((double)w[3 * k + c] * fx_small_inv[k]);
            e = hipMemcpyAsync(bufs[k], v, std::min<size_t>(3, (counts[k] + 3) / 4 * 4) * 4, hipMemcpyHostToDevice, st);
            if (e == hipSuccess) e = wait_stream(s, flags, st);
        }
        return e;
    };
    MH_HIP(hipEventRecord(s->ev0, st));
    if (wavefront) {
        int cus = 256;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, s->device);
        const char *ec = getenv("MH_WF_CHUNK");
        uint64_t max_samples = std::min<uint64_t>(
            wf_max_chunk(), ec ? std::max<uint64_t>(1024, strtoull(ec, nullptr, 10)) : wf_max_chunk());
        const uint32_t n_depth = std::max<uint32_t>(1, in->max_depth - 1);
        if (bmp_wf)  // vertex records: 48 B per path and depth; at most 8 GiB of them per chunk
            max_samples = std::min<uint64_t>(max_samples, std::max<uint64_t>(1 << 16, (8ull << 30) / (48ull * n_depth)));
        uint32_t chunk_px = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(n_px, max_samples / S_));
        // two-stream chunk pipeline (fork_stream): float gradients only
        // (per-stream block partials, atomic texel scatter)
        const bool two_ok = !deterministic(flags) && !(flags & MH_FLAG_SHARED_DEVICE) && chunk_streams_enabled();
        if (two_ok && chunk_px >= n_px && n_px >= 2 && n_px * S_ >= kTwoStreamMinSamples)
            chunk_px = (uint32_t)((n_px + 1) / 2);
        const bool two = two_ok && chunk_px < n_px;
        // MH_FLAG_SHARED_DEVICE (another call runs beside this one) or the two
        // chunk streams: the launches take a share of the CUs' slots (wf_blocks)
        const uint32_t grid = wf_grid(wf_blocks(cus, two || (flags & MH_FLAG_SHARED_DEVICE) != 0));
        const uint64_t cap = (uint64_t)chunk_px * S_;
        const size_t n_chunks = (size_t)((n_px + chunk_px - 1) / chunk_px);
        const uint32_t n_bounces = in->max_depth;
        const size_t ctr_per_chunk = wf_counter_words(n_bounces);
        MH_HIP(s->wf_ws.alloc(wf_workspace_bytes(cap)));
        MH_HIP(s->wf_ws_prb.alloc(wf_prb_workspace_bytes(cap)));
        if (two) {
            MH_HIP(s->wf_ws2.alloc(wf_workspace_bytes(cap)));
            MH_HIP(s->wf_ws_prb2.alloc(wf_prb_workspace_bytes(cap)));
        }
        WfBitmapArgs bmp;
        if (bmp_wf) {
            MH_HIP(s->wf_ws_bmp.alloc(wf_bmp_workspace_bytes(cap, n_depth)));
            if (two) MH_HIP(s->wf_ws_bmp2.alloc(wf_bmp_workspace_bytes(cap, n_depth)));
            int max_wg = 64 << 10, per_cu_lds = 160 << 10;
            (void)hipDeviceGetAttribute(&max_wg, hipDeviceAttributeMaxSharedMemoryPerBlock, s->device);
            (void)hipDeviceGetAttribute(&per_cu_lds, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, s->device);
            bmp.ws = s->wf_ws_bmp.ptr;
            bmp.n_depth = n_depth;
            bmp.slot = kMaxRgbParams;
            // every bitmap slot kMaxRgbParams + b: its texture and its offset in
            // the bitmap slots' contiguous block of s->tmp_c (upload_slots)
            size_t boff = 0;
            for (int b = 0; b < kMaxBitmapParams; ++b) {
                bmp.off[b] = (uint32_t)boff;
                boff += (counts[kMaxRgbParams + b] + 3) / 4 * 4;
            }
            for (uint32_t t = 0; t < (uint32_t)P.slot_of_tex.size(); ++t)
                if (P.slot_of_tex[t] >= kMaxRgbParams) bmp.tex[P.slot_of_tex[t] - kMaxRgbParams] = t;
            bmp.grad = bufs[kMaxRgbParams];
            bmp.n_floats = (uint32_t)boff;
            bmp.lds_max = (env_lds && !strcmp(env_lds, "0")) ? 0u : (uint32_t)std::min(max_wg, 64 << 10);
            if (deterministic(flags)) {  // fixed-point texel sums (k_wf_bitmap_scatter<false, Fx>)
                MH_HIP(s->bmp_fx.alloc((size_t)bmp.n_floats * 8 + 256));
                bmp.fx_word = s->bmp_fx.as<uint32_t>();
                bmp.fx_acc = reinterpret_cast<unsigned long long *>(s->bmp_fx.as<uint8_t>() + 256);
            }
            bmp.n_rec = s->counters.as<unsigned long long>() + kCtrAuxItems;
            bmp.wg_lds = (uint32_t)max_wg;
            bmp.cu_lds = (uint32_t)per_cu_lds;
            bmp.cus = (uint32_t)cus;
        }
        // MH_FLAG_DETERMINISTIC: rgb slots summed per path and reduced in a
        // fixed order (WfDet); bitmap texels in int64 fixed point (bmp.fx_acc)
        const bool det_grad = deterministic(flags) && n_rgb > 0;
        if (det_grad) MH_HIP(s->wf_ws_det.alloc(wf_det_workspace_bytes(cap)));
        MH_HIP(s->wf_ctr.alloc(ctr_per_chunk * n_chunks * 4));
        const size_t partial_bytes = (size_t)grid * kMaxRgbParams * 3 * 4;
        MH_HIP(s->wf_partial.alloc(partial_bytes));
        MH_HIP(hipMemsetAsync(s->wf_partial.ptr, 0, partial_bytes, st));
        if (two) {
            MH_HIP(s->wf_partial2.alloc(partial_bytes));
            MH_HIP(hipMemsetAsync(s->wf_partial2.ptr, 0, partial_bytes, st));
        }
        while (s->evpool.size() < 3 * n_chunks) {
            hipEvent_t e;
            MH_HIP(hipEventCreate(&e));
            s->evpool.push_back(e);
        }
        DScene S2 = s->S;  // stream2's scene view: its own stack overflow columns (stream-engine scenes)
        if (two && s->S.stack_ovf) {
            MH_HIP(s->stack_ovf2.alloc(s->stack_ovf.bytes));
            S2.stack_ovf = s->stack_ovf2.as<uint32_t>();
        }
        if (two) MH_HIP(fork_stream(s, st));
        size_t chunk = 0;
        for (uint64_t p0 = 0; p0 < n_px; p0 += chunk_px, ++chunk) {
            const uint32_t npx = (uint32_t)std::min<uint64_t>(chunk_px, n_px - p0);
            // the chunk's stream and buffers (two: odd chunks on stream2)
            const bool odd = two && (chunk & 1);
            WfBitmapArgs bc = bmp;
            if (odd) bc.ws = s->wf_ws_bmp2.ptr;
            MH_HIP(launch_wavefront_prb(odd ? S2 : s->S, *in, lane_map(L, (uint32_t)p0), s->S.sampler_seed + seed,
                                        (uint64_t)npx * S_, L.spp_pp >= 4, g_in, w, ga.slot_of_tex, n_rgb,
                                        (odd ? s->wf_ws2 : s->wf_ws).ptr, (odd ? s->wf_ws_prb2 : s->wf_ws_prb).ptr, cap,
                                        s->wf_ctr.as<uint32_t>() + ctr_per_chunk * chunk, n_bounces, grid,
                                        (odd ? s->wf_partial2 : s->wf_partial).as<float>(), odd ? s->stream2 : st,
                                        &s->evpool[3 * chunk], bmp_wf ? &bc : nullptr,
                                        det_grad ? s->wf_ws_det.ptr : nullptr));
        }
        if (two) MH_HIP(join_stream(s, st));
        MH_HIP(launch_wf_grad_reduce(s->wf_partial.as<float>(), grid, n_rgb, ga.bufs, st));
        if (two) MH_HIP(launch_wf_grad_reduce(s->wf_partial2.as<float>(), grid, n_rgb, ga.bufs, st));
        wf_ctr_words = ctr_per_chunk;
        wf_chunks = n_chunks;
    } else if (vol && !(env_pvl && !strcmp(env_pvl, "0"))) {
        // prbvolpath: persistent grid, one NEE-walk log per thread (NeeLog)
        int cus = 256;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, s->device);
        const char *ecap = getenv("MH_PVP_NEE_CAP");  // tests: small logs exercise the replay fallback
        // single pass (MainLog) unless MH_PVP_SINGLE=0; MH_PVP_MAIN_CAP: entries per thread
        const char *esp = getenv("MH_PVP_SINGLE"), *emc = getenv("MH_PVP_MAIN_CAP");
        uint32_t main_cap = (esp && !strcmp(esp, "0")) ? 0u : emc ? (uint32_t)std::max(1, atoi(emc)) : kPvpMainCap;
        const uint32_t cap = ecap ? (uint32_t)std::max(1, atoi(ecap)) : kPvpNeeCap;
        // the single pass runs on the phase scheduler (k_vol_sched<PvBwdMachine>)
        // unless MH_PVP_SCHED=0 (the per-sample kernel k_prbvol_backward)
        const char *esc = getenv("MH_PVP_SCHED");
        bool sched = main_cap && vs_supported(s->S, *in) && !(esc && !strcmp(esc, "0"));
        // the persistent grid (and with it both per-thread logs): the
        // scheduler's, or k_prbvol_backward's shrunk to the work (a wave takes
        // 64 samples per batch, so more threads than samples would only hold log space)
        const uint32_t blocks = sched ? vs_blocks(cus)
                                      : (uint32_t)std::max<uint64_t>(
                                            1, std::min<uint64_t>((uint64_t)cus * kPvpBlocksPerCu, (n + 255) / 256));
        // a log that cannot be allocated degrades the kernel instead of failing
        // the call: no MainLog -> primal + adjoint replay per sample; no NeeLog
        // either -> one thread per sample with the NEE walks replayed
        bool nee_ok = s->pvp_log.alloc((size_t)blocks * 256 * cap * 16) == hipSuccess;
        if (!nee_ok) { (void)hipGetLastError(); s->pvp_log.release(); }
        if (main_cap && (!nee_ok || s->pvp_main.alloc((size_t)blocks * 256 * main_cap * 64) != hipSuccess)) {
            (void)hipGetLastError();
            s->pvp_main.release();
            main_cap = 0;
        }
        // overflow lists of the scheduler (2 + kPvbWalkRec float4 per entry)
        const uint32_t ovf_cap = (uint32_t)std::min<uint64_t>(n, 1ull << 26);
        sched = sched && main_cap && nee_ok &&
                s->pvp_ovf.alloc((size_t)ovf_cap * (2 + kPvbWalkRec) * 16 + 256) == hipSuccess;
        // MH_FLAG_DETERMINISTIC with a grid: pass 1 finds the largest |item| of
        // the grid scatter (nothing is accumulated that survives), pass 2 adds
        // round(item * 2^S) as int64, S = 31 - ceil(log2 max): |item| <= 2^31, so
        // up to 2^31 items sum without overflow, and the sums are exact
        if (fx) MH_HIP(s->fx_word.alloc(512));
        for (uint32_t pass = fx ? 1u : 0u; pass <= (fx ? 2u : 0u); ++pass) {
        GradArgs gp = ga;
        gp.fx_mode = pass;
        gp.fx_max = fx ? s->fx_word.as<uint32_t>() : nullptr;
        if (pass == 1) MH_HIP(hipMemsetAsync(s->fx_word.ptr, 0, 64, st));
        if (pass == 2) MH_HIP(fx_between(gp));
        if (sched) {
            VsBwdArgs bw;
            bw.grad_in = g_in;
            bw.coalesce = L.spp_pp >= 4;
            bw.ga = gp;
            bw.main_log = s->pvp_main.as<float4>();
            bw.nee_log = s->pvp_log.as<float4>();
            bw.main_cap = main_cap;
            bw.nee_cap = cap;
            bw.ovf_paths = s->pvp_ovf.as<float4>();
            bw.ovf_walks = bw.ovf_paths + (size_t)2 * ovf_cap;
            bw.ovf_count = reinterpret_cast<uint32_t *>(bw.ovf_walks + (size_t)kPvbWalkRec * ovf_cap);
            bw.ovf_cap = ovf_cap;
            MH_HIP(hipMemsetAsync(bw.ovf_count, 0, 16, st));
            pvb_lost = bw.ovf_count + 2;
            const LaneMap lm0 = lane_map(L, 0);
            MH_HIP(launch_vol_sched_bwd(s->S, *in, lm0, s->S.sampler_seed + seed, n, bw, blocks,
                                        s->counters.as<unsigned long long>(), st));
            MH_HIP(launch_vol_sched_bwd_replays(s->S, *in, lm0, s->S.sampler_seed + seed, n, bw,
                                                s->counters.as<unsigned long long>(), st));
            if (getenv("MH_VW_DEBUG")) {
                MH_WAIT(s, flags, st);
                if (int rc2 = print_vs_phases(s)) return rc2;
                uint32_t oc[3];
                MH_HIP(hipMemcpy(oc, bw.ovf_count, sizeof(oc), hipMemcpyDeviceToHost));
                fprintf(stderr, "pvb overflow replays: %u paths, %u walks, %u lost\n", oc[0], oc[1], oc[2]);
            }
        } else {
            MH_HIP(launch_prb_backward(s->S, *in, lane_map(L, 0), s->S.sampler_seed + seed, n, L.spp_pp >= 4,
                                       g_in, w, gp, fused, s->counters.as<unsigned long long>(), st,
                                       nee_ok ? s->pvp_log.as<float4>() : nullptr, cap, blocks,
                                       s->counters.as<unsigned long long>() + kCtrPvpHead,
                                       main_cap ? s->pvp_main.as<float4>() : nullptr, main_cap));
        }
        }  // passes
    } else if (fxr) {  // deterministic: prbvolpath replaying its NEE walks (MH_PVP_NEE_LOG=0), or the prb replay
        MH_HIP(s->fx_word.alloc(512));
        MH_HIP(hipMemsetAsync(s->fx_word.ptr, 0, 64, st));
        GradArgs gp = ga;
        gp.fx_max = s->fx_word.as<uint32_t>();
        for (uint32_t pass = 1; pass <= 2; ++pass) {
            gp.fx_mode = pass;
            if (pass == 2) MH_HIP(fx_between(gp));
            MH_HIP(launch_prb_backward(s->S, *in, lane_map(L, 0), s->S.sampler_seed + seed, n, L.spp_pp >= 4,
                                       g_in, w, gp, fused, s->counters.as<unsigned long long>(), st));
        }
    } else {
        MH_HIP(launch_prb_backward(s->S, *in, lane_map(L, 0), s->S.sampler_seed + seed, n, L.spp_pp >= 4,
                                   g_in, w, ga, fused, s->counters.as<unsigned long long>(), st));
    }
    if (fxr) MH_HIP(fx_small_fold());
    if (det_replay)
        for (int k = kMaxRgbParams; k < kMaxParams; ++k)
            if (counts[k])
                MH_HIP(launch_fx_to_float(s->replay_fx.as<long long>() + (bufs[k] - s->tmp_c.as<float>()), bufs[k],
                                          counts[k], fx_small_inv[k], st));
    for (int k = 0; k < kMaxParams; ++k) {
        if (!P.corner[k]) continue;
        if (P.fx)
            MH_HIP(launch_corner_gather_fx(reinterpret_cast<const long long *>(P.corner[k]), bufs[k], P.grid_res[k],
                                           fx_inv, st));
        else
            MH_HIP(launch_corner_gather(P.corner[k], bufs[k], P.grid_res[k], st));
    }
    MH_HIP(hipEventRecord(s->ev1, st));
    if (wants_reduce(flags)) {  // the slot buffers are one block of s->tmp_c (upload_slots)
        size_t total = 0;
        for (int k = 0; k < kMaxParams; ++k) total += (counts[k] + 3) / 4 * 4;
        if (int rc = reduce_result(s, flags, s->tmp_c.as<float>(), total, st, false)) return rc;
    }
    // accumulate into the caller's gradient buffers
    std::vector<float> host_tmp;
    for (uint32_t k = 0; k < n_params; ++k) {
        uint32_t slot = slot_of_param[k];
        size_t c = counts[slot];
        if (dev) {
            MH_HIP(launch_accumulate(grads[k], bufs[slot], c, st));
        } else {
            host_tmp.resize(c);
            MH_HIP(hipMemcpyAsync(host_tmp.data(), bufs[slot], c * 4, hipMemcpyDeviceToHost, st));
            MH_WAIT(s, flags, st);
            for (size_t i = 0; i < c; ++i) grads[k][i] += host_tmp[i];
        }
    }
    if (async_call(flags, stats)) return MH_OK;  // gradients stay stream-ordered on the device
    auto check_lost = [&]() -> int {  // (after a stream sync) an overflow replay that did not run fails the call
        uint32_t lost = 0;
        if (pvb_lost) MH_HIP(hipMemcpy(&lost, pvb_lost, 4, hipMemcpyDeviceToHost));
        if (lost)
            return set_error(MH_ERR_OUT_OF_MEMORY, "render_backward(): " + std::to_string(lost) +
                                                       " prbvolpath overflow replays did not fit their list "
                                                       "(MH_PVP_SCHED=0 runs the per-sample kernel)");
        return MH_OK;
    };
    if (!stats) {
        MH_WAIT(s, flags, st);
        return check_lost();
    }
    unsigned long long ctr[2] = {0, 0}, n_rec = 0;
    std::vector<uint32_t> wctr(wf_ctr_words * wf_chunks);
    if (wavefront) {
        MH_HIP(hipMemcpyAsync(wctr.data(), s->wf_ctr.ptr, wctr.size() * 4, hipMemcpyDeviceToHost, st));
        MH_HIP(hipMemcpyAsync(&n_rec, s->counters.as<unsigned long long>() + kCtrAuxItems, 8, hipMemcpyDeviceToHost, st));
    } else
        MH_HIP(hipMemcpyAsync(ctr, s->counters.ptr, sizeof(ctr), hipMemcpyDeviceToHost, st));
    MH_WAIT(s, flags, st);
    if (int rc_lost = check_lost()) return rc_lost;
    if (wavefront) {
        const size_t per_bounce = wf_ctr_words / (in->max_depth + 1), nseg = per_bounce / 32;
        for (size_t c = 0; c < wf_chunks; ++c)
            for (uint32_t b = 0; b < in->max_depth; ++b)
                for (size_t sg = 0; sg < nseg; ++sg) {
                    ctr[0] += wctr[wf_ctr_words * c + per_bounce * b + 32 * sg + 0];
                    ctr[1] += wctr[wf_ctr_words * c + per_bounce * b + 32 * sg + 1];
                }
    }
    if (stats) {
        float ms = 0.f, trace_ms = 0.f, scat_ms = 0.f;
        MH_HIP(hipEventElapsedTime(&ms, s->ev0, s->ev1));
        for (size_t c = 0; wavefront && c < wf_chunks; ++c) {
            float t = 0.f;
            MH_HIP(hipEventElapsedTime(&t, s->evpool[3 * c], s->evpool[3 * c + 1]));
            trace_ms += t;
            MH_HIP(hipEventElapsedTime(&t, s->evpool[3 * c + 1], s->evpool[3 * c + 2]));
            scat_ms += t;
        }
        if (bmp_wf) {  // the texel scatter: one launch per chunk
            stats->aux_items = n_rec;
            stats->ms_aux = scat_ms;
            stats->n_aux_launches = wf_chunks;
        }
        // the bounce-kernel span (fused: k_wf_bounce_prb launches only)
        stats->ms_trace = trace_ms;
        stats->n_trace_launches = wavefront ? (uint64_t)wf_chunks * in->max_depth : 0;
        stats->mode = wavefront ? 1u : 0u;
        stats->samples = n;
        stats->rays_closest = ctr[0];
        stats->rays_shadow = ctr[1];
        stats->bounces = ctr[0];
        stats->ms_total = now_ms() - t_start;
        stats->ms_kernel = ms;
    }
    return MH_OK;
}

// ---------------------------------------------------------------------------
// Forward-mode derivative: RBIntegrator.render_forward (common.py:696-826)
// ---------------------------------------------------------------------------
static int render_forward_impl(mh_scene *s, const mh_integrator *in, uint32_t seed, uint32_t spp, uint32_t spp_begin,
                      uint32_t spp_end, uint32_t n_params, const uint32_t *param_tex, const float *const *tangents,
                      float *film_rgbw, uint32_t flags, mh_stats *stats) {
    ScopedPhase phase_("RenderForward");
    if (!s || !in || !film_rgbw || (n_params && (!param_tex || !tangents)))
        return set_error(MH_ERR_INVALID_ARGUMENT, "mh_render_forward: NULL argument");
    if (in->type != MH_INTEGRATOR_PRB && in->type != MH_INTEGRATOR_PRBVOLPATH)
        return set_error(MH_ERR_UNSUPPORTED, "render_forward(): requires the 'prb' or 'prbvolpath' integrator");
    if (in->rr_depth == 0)
        return set_error(MH_ERR_INVALID_ARGUMENT, "\"rr_depth\" must be set to a value greater than zero!");
    if (spp == 0) return set_error(MH_ERR_INVALID_ARGUMENT, "mh_render_forward: spp must be > 0");
    if (int rc = check_reduce_flags(s, flags, "mh_render_forward", true)) return rc;
    const double t_start = now_ms();
    if (stats) *stats = mh_stats{};
    Layout L;
    int rc = make_layout(s, spp, spp_begin, spp_end, L, true);  // prepare(): one wavefront of <= 2^32
    if (rc) return rc;
    MH_HIP(hipSetDevice(s->device));
    g_call_issued = true;  // past argument validation: a failure from here aborts the communicator
    hipStream_t st = s->stream;
    const bool dev = flags & MH_FLAG_DEVICE_POINTERS;
    Slots P;
    rc = build_slots(s, n_params, param_tex, in->type == MH_INTEGRATOR_PRBVOLPATH, "mh_render_forward",
                     "render_forward", P);
    if (rc) return rc;
    std::vector<float *> bufs;
    GradArgs ga;
    MH_HIP(upload_slots(s, P, st, bufs, ga));  // zeroed slot buffers, here the tangents
    for (uint32_t k = 0; k < n_params; ++k) {
        const uint32_t slot = P.slot_of_param[k];
        if (!tangents[k]) return set_error(MH_ERR_INVALID_ARGUMENT, "mh_render_forward: NULL tangent");
        MH_HIP(hipMemcpyAsync(bufs[slot], tangents[k], P.counts[slot] * 4,
                              dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, st));
    }
    // the film: as mh_render (RGBW, or RGBW + an alpha plane gathered into R G B A W)
    const uint64_t n_px = (uint64_t)L.W * L.H;
    const bool alpha = has_alpha(s->pixel_format);
    const size_t film_bytes = n_px * (alpha ? 20 : 16);
    float *film = film_rgbw;
    if (!dev) {
        MH_HIP(s->film_tmp.alloc(film_bytes));
        film = s->film_tmp.as<float>();
    }
    if (!(flags & MH_FLAG_ACCUMULATE)) MH_HIP(hipMemsetAsync(film, 0, film_bytes, st));
    else if (!dev) MH_HIP(hipMemcpyAsync(film, film_rgbw, film_bytes, hipMemcpyHostToDevice, st));
    float *film4 = film, *film_a = nullptr;
    if (alpha) {
        MH_HIP(s->film4.alloc(n_px * 16));
        MH_HIP(s->alpha_px.alloc(n_px * 4));
        film4 = s->film4.as<float>();
        film_a = s->alpha_px.as<float>();
        MH_HIP(hipMemsetAsync(film4, 0, n_px * 16, st));
        MH_HIP(hipMemsetAsync(film_a, 0, n_px * 4, st));
    }
    MH_HIP(hipMemsetAsync(s->counters.ptr, 0, 256, st));
    const uint32_t S_ = L.s_end - L.s_begin;
    const uint32_t chunk_px = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(n_px, wf_max_chunk() / S_));
    const uint64_t plane = (uint64_t)chunk_px * S_;
    MH_HIP(s->work.alloc(plane * (alpha ? 6 : 5) * sizeof(float)));
    // prb on packet-engine scenes: the fused forward-mode wavefront
    // (k_wf_bounce_fwd); prbvolpath, larger scenes or MH_FLAG_MEGAKERNEL /
    // MH_MODE=mega: the per-sample kernel (k_render_forward)
    const char *env_mode = getenv("MH_MODE");
    const bool wavefront = in->type == MH_INTEGRATOR_PRB && wf_fused(s->S) && in->max_depth >= 1 &&
                           in->max_depth <= 64 && !(flags & MH_FLAG_MEGAKERNEL) && !(env_mode && !strcmp(env_mode, "mega"));
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, s->device);
    if (wavefront) {
        MH_HIP(s->wf_ws.alloc(wf_workspace_bytes(plane)));
        MH_HIP(s->wf_ws_prb.alloc(wf_prb_workspace_bytes(plane)));
        MH_HIP(s->wf_ctr.alloc((size_t)wf_counter_words(in->max_depth) * 4));
    }
    const bool fast_splat = L.spp_pp >= 4 && s->S.rfilter == MH_RFILTER_GAUSSIAN && s->S.rfilter_radius > 1.5f &&
                            s->S.rfilter_radius <= 2.5f;
    const int coalesce = L.spp_pp >= 4;  // block.set_coalesce(... and spp >= 4) (common.py:795-796)
    const uint32_t seed_value = s->S.sampler_seed + seed;
    const bool determ = deterministic(flags);
    unsigned long long *bounds = s->counters.as<unsigned long long>() + kCtrBounds;
    MH_HIP(hipEventRecord(s->ev0, st));
    for (uint64_t p0 = 0; p0 < n_px; p0 += chunk_px) {
        const uint32_t npx = (uint32_t)std::min<uint64_t>(chunk_px, n_px - p0);
        const LaneMap lm = lane_map(L, (uint32_t)p0);
        const uint64_t n = (uint64_t)npx * S_;
        if (wavefront)
            MH_HIP(launch_wavefront_fwd(s->S, *in, lm, seed_value, n, ga.slot_of_tex, ga.bufs, ga.is_rgb,
                                        s->work.as<float>(), plane, alpha, s->wf_ws.ptr, s->wf_ws_prb.ptr, plane,
                                        s->wf_ctr.as<uint32_t>(), in->max_depth, wf_grid(wf_blocks(cus)), st));
        else
            MH_HIP(launch_render_forward(s->S, *in, lm, seed_value, n, plane, s->work.as<float>(), ga,
                                         s->counters.as<unsigned long long>(), st, alpha));
        // no sample check here: tangent radiance is legitimately negative
        MH_SPLAT(s->S, lm, kSplatFilm, fast_splat, npx, 1, n, plane, s->work.as<float>(), film4, seed_value,
                 coalesce, st, nullptr, determ, s->work.bytes / 4, n_px * 4, bounds);
        if (alpha)
            MH_SPLAT(s->S, lm, kSplatAlpha, fast_splat, npx, 1, n, plane, s->work.as<float>(), film_a, seed_value,
                     coalesce, st, nullptr, determ, s->work.bytes / 4, n_px, bounds);
    }
    if (alpha) MH_HIP(launch_film_rgbaw(n_px, film4, film_a, film, st));
    MH_HIP(hipEventRecord(s->ev1, st));
    if (int rc2 = reduce_result(s, flags, film, film_bytes / 4, st, true)) return rc2;
    if (!dev) MH_HIP(hipMemcpyAsync(film_rgbw, film, film_bytes, hipMemcpyDeviceToHost, st));
    if (async_call(flags, stats)) return MH_OK;
    if (!stats) {
        MH_WAIT(s, flags, st);
        return check_bounds_counter(s, "mh_render_forward");
    }
    unsigned long long ctr[2] = {0, 0};
    MH_HIP(hipMemcpyAsync(ctr, s->counters.ptr, sizeof(ctr), hipMemcpyDeviceToHost, st));
    MH_WAIT(s, flags, st);
    if (int rc = check_bounds_counter(s, "mh_render_forward")) return rc;
    if (stats) {
        float ms = 0.f;
        MH_HIP(hipEventElapsedTime(&ms, s->ev0, s->ev1));
        stats->samples = n_px * S_;
        stats->rays_closest = ctr[0];
        stats->rays_shadow = ctr[1];
        stats->bounces = ctr[0];
        stats->ms_total = now_ms() - t_start;
        stats->ms_kernel = ms;
        stats->ms_trace = 0.f;
        stats->n_trace_launches = 0;
        stats->mode = wavefront ? 2u : 0u;  // fused wavefront / per-sample kernel
        stats->invalid_samples = 0;  // not counted: a tangent's radiance may be negative
    }
    return MH_OK;
}

// ---------------------------------------------------------------------------
// Ray-query sub-boundary
// ---------------------------------------------------------------------------
static int trace_impl(mh_scene *s, bool shadow, uint64_t n, const float *rays, float *t, float *u,
                      float *v, uint32_t *prim, uint32_t *shape, uint32_t *inst, uint32_t *occ, uint32_t flags,
                      mh_stats *stats) {
    ScopedPhase phase_("RayIntersect");
    if (!s || (n && !rays)) return set_error(MH_ERR_INVALID_ARGUMENT, "mh_trace: NULL argument");
    if (n == 0) return MH_OK;
    double t_start = now_ms();
    if (stats) *stats = mh_stats{};
    MH_HIP(hipSetDevice(s->device));
    hipStream_t st = s->stream;
    const bool dev = flags & MH_FLAG_DEVICE_POINTERS;
    const float *r = rays;
    float *dt = t, *du = u, *dv = v;
    uint32_t *dp = prim, *ds = shape, *di = inst, *doc = occ;
    if (!dev) {
        MH_HIP(s->tmp_a.alloc(n * 28));
        MH_HIP(hipMemcpyAsync(s->tmp_a.ptr, rays, n * 28, hipMemcpyHostToDevice, st));
        r = s->tmp_a.as<float>();
        MH_HIP(s->tmp_b.alloc(n * 24));
        float *base = s->tmp_b.as<float>();
        dt = base; du = base + n; dv = base + 2 * n;
        dp = reinterpret_cast<uint32_t *>(base + 3 * n);
        ds = reinterpret_cast<uint32_t *>(base + 4 * n);
        di = inst ? reinterpret_cast<uint32_t *>(base + 5 * n) : nullptr;
        doc = reinterpret_cast<uint32_t *>(base);
    }
    // persistent grid: 8 workgroups of 256 lanes per CU
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, s->device);
    uint32_t grid = (uint32_t)std::min<uint64_t>((n + 255) / 256, (uint64_t)cus * 8);
    MH_HIP(hipEventRecord(s->ev0, st));
    MH_HIP(launch_trace(s->S, shadow, n, r, dt, du, dv, dp, ds, di, doc, grid, st));
    MH_HIP(hipEventRecord(s->ev1, st));
    if (!dev) {
        if (shadow) {
            MH_HIP(hipMemcpyAsync(occ, doc, n * 4, hipMemcpyDeviceToHost, st));
        } else {
            MH_HIP(hipMemcpyAsync(t, dt, n * 4, hipMemcpyDeviceToHost, st));
            MH_HIP(hipMemcpyAsync(u, du, n * 4, hipMemcpyDeviceToHost, st));
            MH_HIP(hipMemcpyAsync(v, dv, n * 4, hipMemcpyDeviceToHost, st));
            MH_HIP(hipMemcpyAsync(prim, dp, n * 4, hipMemcpyDeviceToHost, st));
            MH_HIP(hipMemcpyAsync(shape, ds, n * 4, hipMemcpyDeviceToHost, st));
            if (inst) MH_HIP(hipMemcpyAsync(inst, di, n * 4, hipMemcpyDeviceToHost, st));
        }
    }
    if (!(flags & MH_FLAG_NO_SYNC) || !dev) MH_HIP(hipStreamSynchronize(st));
    if (stats) {
        MH_HIP(hipEventSynchronize(s->ev1));
        float ms = 0.f;
        MH_HIP(hipEventElapsedTime(&ms, s->ev0, s->ev1));
        stats->samples = 0;
        stats->rays_closest = shadow ? 0 : n;
        stats->rays_shadow = shadow ? n : 0;
        stats->bounces = 0;
        stats->ms_total = now_ms() - t_start;
        stats->ms_kernel = ms;
    }
    return MH_OK;
}

int mh_trace_closest(mh_scene *s, uint64_t n, const float *rays, float *t, float *u, float *v,
                     uint32_t *prim, uint32_t *shape, uint32_t flags, mh_stats *stats) {
    return mh_trace_preliminary(s, n, rays, t, u, v, prim, shape, nullptr, flags, stats);
}

int mh_trace_preliminary(mh_scene *s, uint64_t n, const float *rays, float *t, float *u, float *v,
                         uint32_t *prim, uint32_t *shape, uint32_t *instance, uint32_t flags, mh_stats *stats) {
    if (n && (!t || !u || !v || !prim || !shape))
        return set_error(MH_ERR_INVALID_ARGUMENT, "mh_trace_closest: NULL output");
    return trace_impl(s, false, n, rays, t, u, v, prim, shape, instance, nullptr, flags, stats);
}

int mh_trace_shadow(mh_scene *s, uint64_t n, const float *rays, uint32_t *occluded, uint32_t flags,
                    mh_stats *stats) {
    if (n && !occluded) return set_error(MH_ERR_INVALID_ARGUMENT, "mh_trace_shadow: NULL output");
    return trace_impl(s, true, n, rays, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, occluded, flags,
                      stats);
}

// ===========================================================================
// Multi-GPU (include/mitsuba_hip.h, "Multi-GPU").  The
// reference's splice point is SamplingIntegrator::render
// (src/render/integrator.cpp:276-390): its sample loop is cut into per-device
// slabs of every pixel, whose union is sample-identical to one render.
// ===========================================================================
// The entry points with in-call collectives: a call that fails with
// MH_FLAG_REDUCE aborts the scene's communicator (comm_abort), since it has
// issued only part of the call's collectives and its peers' streams wait on
// the rest: their waits then end in an error (comm_wait), and later
// collectives on this communicator fail at once instead of pairing with a
// peer's different collective.
static int abort_on_failure(mh_scene *s, uint32_t flags, int rc) {
    const bool issued = g_call_issued;  // argument errors (before any work) leave the communicator usable
    g_call_issued = false;
    g_keep_error = false;
#ifdef MH_DEBUG
    // the debug build's device bounds guards (MH_GUARD) fail the call
    // (not for asynchronous calls, whose work is still queued; a call with
    // collectives in flight waits through comm_wait and its deadline, not a
    // device-wide sync.  The guard words are per device: concurrent scenes on
    // one device read each other's counts -- run guard builds one scene at a time)
    if (rc == MH_OK && issued && s && !(flags & MH_FLAG_NO_SYNC)) {
        (void)hipSetDevice(s->device);
        unsigned long long g[2][kGuardCount] = {};
        const bool waited = (wants_reduce(flags) && s->comm) ? comm_wait(s->comm, s->stream, "MH_DEBUG guard read") == MH_OK
                                                             : hipStreamSynchronize(s->stream) == hipSuccess;
        if (!waited) {
            if (!(wants_reduce(flags) && s->comm)) rc = set_error(MH_ERR_HIP, "MH_DEBUG: the stream could not be synchronized");
            else rc = MH_ERR_HIP;  // comm_wait's message stands
        } else if (guard_read_wf(g[0]) != hipSuccess || guard_read_k(g[1]) != hipSuccess)
            rc = set_error(MH_ERR_HIP, "MH_DEBUG: the device guard counters could not be read");
        static const char *what[kGuardCount] = {"queue item beyond its segment", "path id beyond the chunk",
                                                "appended slot beyond its segment", "sample-plane index beyond the plane",
                                                "generated pixel outside the film", "LDS accumulator index beyond its size", "", ""};
        for (int k = 0; rc == MH_OK && k < kGuardCount; ++k)
            if (g[0][k] + g[1][k])
                rc = set_error(MH_ERR_HIP, std::string("MH_DEBUG device guard: ") + what[k] + " (" +
                                               std::to_string(g[0][k] + g[1][k]) + " lanes)");
    }
#endif
    if (rc != MH_OK && issued && s && s->comm && wants_reduce(flags)) {
        const std::string why = g_error;
        comm_abort(s->comm);
        set_error(rc, why + " (the scene's communicator was aborted)");
    }
    return rc;
}

int mh_render(mh_scene *s, const mh_integrator *in, uint32_t seed, uint32_t spp, uint32_t spp_begin,
              uint32_t spp_end, float *film_rgbw, uint32_t flags, mh_stats *stats) {
    g_call_issued = false;
    return abort_on_failure(s, flags, render_impl(s, in, seed, spp, spp_begin, spp_end, film_rgbw, flags, stats));
}

int mh_prb_weights(mh_scene *s, uint32_t seed, uint32_t spp, uint32_t spp_begin, uint32_t spp_end,
                   float *weights, uint32_t flags) {
    g_call_issued = false;
    return abort_on_failure(s, flags, prb_weights_impl(s, seed, spp, spp_begin, spp_end, weights, flags));
}

int mh_render_backward(mh_scene *s, const mh_integrator *in, uint32_t seed, uint32_t spp,
                       uint32_t spp_begin, uint32_t spp_end, const float *grad_in,
                       const float *weights, uint32_t n_params, const uint32_t *param_tex,
                       float *const *grads, uint32_t flags, mh_stats *stats) {
    g_call_issued = false;
    return abort_on_failure(s, flags, render_backward_impl(s, in, seed, spp, spp_begin, spp_end, grad_in, weights,
                                                           n_params, param_tex, grads, flags, stats));
}

int mh_render_forward(mh_scene *s, const mh_integrator *in, uint32_t seed, uint32_t spp, uint32_t spp_begin,
                      uint32_t spp_end, uint32_t n_params, const uint32_t *param_tex, const float *const *tangents,
                      float *film_rgbw, uint32_t flags, mh_stats *stats) {
    g_call_issued = false;
    return abort_on_failure(s, flags, render_forward_impl(s, in, seed, spp, spp_begin, spp_end, n_params, param_tex,
                                                          tangents, film_rgbw, flags, stats));
}

int mh_scene_set_comm(mh_scene *s, mh_comm *comm) {
    if (!s) return set_error(MH_ERR_INVALID_ARGUMENT, "mh_scene_set_comm: NULL scene");
    if (comm) {
        int dev = -1;
        if (int rc = mh_comm_info(comm, nullptr, nullptr, &dev)) return rc;
        if (dev != s->device)
            return set_error(MH_ERR_INVALID_ARGUMENT, "mh_scene_set_comm: the communicator's device is not the scene's");
    }
    if (s->comm) comm_attach(s->comm, -1);
    s->comm = comm;
    if (comm) comm_attach(comm, +1);
    return MH_OK;
}

int mh_scene_synchronize(mh_scene *s) {
    if (!s) return set_error(MH_ERR_INVALID_ARGUMENT, "mh_scene_synchronize: NULL scene");
    MH_HIP(hipSetDevice(s->device));
    MH_HIP(hipStreamSynchronize(s->stream));
    return check_bounds_counter(s, "mh_scene_synchronize");
}

}  // extern "C"

namespace {

// slab i of n: samples [spp*i/n, spp*(i+1)/n) of every pixel
uint32_t slab_edge(uint32_t spp, uint32_t i, uint32_t n) { return (uint32_t)((uint64_t)spp * i / n); }

// fn(i) for every scene, each on a host thread of its own: the devices (and
// streams) then run concurrently although every call synchronises, and an
// in-call collective finds all of its ranks issued.  The first failure wins.
template <class F>
int for_each_scene(uint32_t n, F fn) {
    std::vector<int> rc(n, MH_OK);
    std::vector<std::string> msg(n);
    std::vector<std::thread> th;
    th.reserve(n);
    for (uint32_t i = 0; i < n; ++i)
        th.emplace_back([&, i] {
            rc[i] = fn(i);
            if (rc[i]) msg[i] = g_error;  // the worker thread's own message
        });
    for (auto &t : th) t.join();
    for (uint32_t i = 0; i < n; ++i)
        if (rc[i]) return set_error(rc[i], "scene " + std::to_string(i) + ": " + msg[i]);
    return MH_OK;
}

// argument checks shared by the sharded entry points; *comm = every scene
// has a communicator whose ranks are the scenes' order (else none may have one)
int check_shards(mh_scene *const *sc, uint32_t n, uint32_t spp, const char *api, bool *comm) {
    const std::string a(api);
    if (!sc || n == 0) return set_error(MH_ERR_INVALID_ARGUMENT, a + ": no scenes");
    if (spp < n) return set_error(MH_ERR_INVALID_ARGUMENT, a + ": spp must be >= the number of scenes (one slab each)");
    uint32_t with = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if (!sc[i]) return set_error(MH_ERR_INVALID_ARGUMENT, a + ": NULL scene");
        for (uint32_t j = 0; j < i; ++j)
            if (sc[j] == sc[i]) return set_error(MH_ERR_INVALID_ARGUMENT, a + ": a scene appears twice (one per slab)");
        if (sc[i]->S.width != sc[0]->S.width || sc[i]->S.height != sc[0]->S.height ||
            sc[i]->pixel_format != sc[0]->pixel_format)
            return set_error(MH_ERR_INVALID_ARGUMENT, a + ": the scenes' films differ");
        with += sc[i]->comm ? 1u : 0u;
    }
    if (with != 0 && with != n)
        return set_error(MH_ERR_INVALID_ARGUMENT, a + ": either every scene has a communicator or none has");
    for (uint32_t i = 0; i < with; ++i) {
        int nr = 0, r = 0;
        mh_comm_info(sc[i]->comm, &nr, &r, nullptr);
        if (nr != (int)n || r != (int)i)
            return set_error(MH_ERR_INVALID_ARGUMENT, a + ": scene i's communicator must be rank i of n");
    }
    *comm = with == n;
    return MH_OK;
}

// the sum without a communicator: bufs[i] (count floats on scene i's device)
// are copied onto scene 0's device (peer copies; a plain device copy when the
// scenes share it) and added into bufs[0] in scene order; `all` copies the
// sum back to every bufs[i].  Every stream has drained before and after.
int peer_sum(mh_scene *const *sc, uint32_t n, float *const *bufs, uint64_t count, bool all) {
    mh_scene *s0 = sc[0];
    MH_HIP(hipSetDevice(s0->device));
    MH_HIP(s0->shard_tmp.alloc(count * 4));
    for (uint32_t i = 1; i < n; ++i) {
        MH_HIP(hipMemcpyPeerAsync(s0->shard_tmp.ptr, s0->device, bufs[i], sc[i]->device, count * 4, s0->stream));
        MH_HIP(launch_accumulate(bufs[0], s0->shard_tmp.as<float>(), count, s0->stream));
    }
    if (all)
        for (uint32_t i = 1; i < n; ++i)
            MH_HIP(hipMemcpyPeerAsync(bufs[i], sc[i]->device, bufs[0], s0->device, count * 4, s0->stream));
    MH_HIP(hipStreamSynchronize(s0->stream));
    return MH_OK;
}

}  // namespace

extern "C" {

int mh_render_sharded(mh_scene *const *scenes, uint32_t n, const mh_integrator *in, uint32_t seed, uint32_t spp,
                      float *const *films, uint32_t flags, mh_stats *stats) {
    ScopedPhase phase_("Render");
    bool comm = false;
    if (int rc = check_shards(scenes, n, spp, "mh_render_sharded", &comm)) return rc;
    if (!in || !films) return set_error(MH_ERR_INVALID_ARGUMENT, "mh_render_sharded: NULL argument");
    for (uint32_t i = 0; i < n; ++i)
        if (!films[i]) return set_error(MH_ERR_INVALID_ARGUMENT, "mh_render_sharded: NULL film");
    if (flags & MH_FLAG_ACCUMULATE)
        return set_error(MH_ERR_INVALID_ARGUMENT, "mh_render_sharded: MH_FLAG_ACCUMULATE is not supported (the sum "
                                                  "would count the accumulated film once per scene)");
    const uint32_t pass = (flags & (MH_FLAG_DETERMINISTIC | MH_FLAG_MEGAKERNEL | MH_FLAG_WAVEFRONT)) |
                          MH_FLAG_DEVICE_POINTERS;
    const uint32_t red = comm ? ((flags & MH_FLAG_REDUCE) ? MH_FLAG_REDUCE : MH_FLAG_REDUCE_ROOT) : 0u;
    int rc = for_each_scene(n, [&](uint32_t i) {
        return mh_render(scenes[i], in, seed, spp, slab_edge(spp, i, n), slab_edge(spp, i + 1, n), films[i],
                         pass | red, stats ? &stats[i] : nullptr);
    });
    if (rc || comm) return rc;
    const uint64_t count = (uint64_t)scenes[0]->S.width * scenes[0]->S.height * (has_alpha(scenes[0]->pixel_format) ? 5 : 4);
    return peer_sum(scenes, n, films, count, flags & MH_FLAG_REDUCE);
}

int mh_render_backward_sharded(mh_scene *const *scenes, uint32_t n, const mh_integrator *in, uint32_t seed,
                               uint32_t spp, const float *const *grad_in, uint32_t n_params,
                               const uint32_t *param_tex, float *const *grads, uint32_t flags, mh_stats *stats) {
    ScopedPhase phase_("RenderBackward");
    bool comm = false;
    if (int rc = check_shards(scenes, n, spp, "mh_render_backward_sharded", &comm)) return rc;
    if (!in || !grad_in || (n_params && (!param_tex || !grads)))
        return set_error(MH_ERR_INVALID_ARGUMENT, "mh_render_backward_sharded: NULL argument");
    const uint32_t pass = (flags & (MH_FLAG_DETERMINISTIC | MH_FLAG_MEGAKERNEL | MH_FLAG_PRB_REPLAY)) |
                          MH_FLAG_DEVICE_POINTERS;
    if (comm)  // every rank: slab W + all-reduce, its slab's gradient, all-reduce (mh_render_backward in-call)
        return for_each_scene(n, [&](uint32_t i) {
            return mh_render_backward(scenes[i], in, seed, spp, slab_edge(spp, i, n), slab_edge(spp, i + 1, n),
                                      grad_in[i], nullptr, n_params, param_tex, grads + (size_t)i * n_params,
                                      pass | MH_FLAG_REDUCE | (flags & MH_FLAG_LOCAL_WEIGHTS),
                                      stats ? &stats[i] : nullptr);
        });
    // without communicators: the slab W images summed onto every scene ...
    const uint64_t n_px = (uint64_t)scenes[0]->S.width * scenes[0]->S.height;
    std::vector<float *> wb(n), gb(n);
    for (uint32_t i = 0; i < n; ++i) {
        MH_HIP(hipSetDevice(scenes[i]->device));
        MH_HIP(scenes[i]->shard_w.alloc(n_px * 4));
        wb[i] = scenes[i]->shard_w.as<float>();
    }
    int rc = for_each_scene(n, [&](uint32_t i) {
        return mh_prb_weights(scenes[i], seed, spp, slab_edge(spp, i, n), slab_edge(spp, i + 1, n), wb[i],
                              pass & (MH_FLAG_DEVICE_POINTERS | MH_FLAG_DETERMINISTIC));
    });
    if (rc) return rc;
    if ((rc = peer_sum(scenes, n, wb.data(), n_px, true))) return rc;
    // ... each slab's gradient into zeroed per-scene buffers, summed, then
    // accumulated into the caller's buffers as mh_render_backward does
    Slots P;
    if ((rc = build_slots(scenes[0], n_params, param_tex, in->type == MH_INTEGRATOR_PRBVOLPATH,
                          "mh_render_backward_sharded", "render_backward", P)))
        return rc;
    std::vector<uint64_t> off(n_params + 1, 0);
    for (uint32_t k = 0; k < n_params; ++k) off[k + 1] = off[k] + P.counts[P.slot_of_param[k]];
    const uint64_t total = std::max<uint64_t>(off[n_params], 1);
    for (uint32_t i = 0; i < n; ++i) {
        MH_HIP(hipSetDevice(scenes[i]->device));
        MH_HIP(scenes[i]->shard_g.alloc(total * 4));
        gb[i] = scenes[i]->shard_g.as<float>();
        MH_HIP(hipMemsetAsync(gb[i], 0, total * 4, scenes[i]->stream));
        MH_HIP(hipStreamSynchronize(scenes[i]->stream));
    }
    rc = for_each_scene(n, [&](uint32_t i) {
        std::vector<float *> gp(std::max<uint32_t>(n_params, 1));
        for (uint32_t k = 0; k < n_params; ++k) gp[k] = gb[i] + off[k];
        return mh_render_backward(scenes[i], in, seed, spp, slab_edge(spp, i, n), slab_edge(spp, i + 1, n),
                                  grad_in[i], wb[i], n_params, param_tex, gp.data(), pass, stats ? &stats[i] : nullptr);
    });
    if (rc) return rc;
    if ((rc = peer_sum(scenes, n, gb.data(), total, true))) return rc;
    for (uint32_t i = 0; i < n; ++i) {
        MH_HIP(hipSetDevice(scenes[i]->device));
        for (uint32_t k = 0; k < n_params; ++k) {
            if (!grads[(size_t)i * n_params + k])
                return set_error(MH_ERR_INVALID_ARGUMENT, "mh_render_backward_sharded: NULL gradient buffer");
            MH_HIP(launch_accumulate(grads[(size_t)i * n_params + k], gb[i] + off[k], off[k + 1] - off[k],
                                     scenes[i]->stream));
        }
        MH_HIP(hipStreamSynchronize(scenes[i]->stream));
    }
    return MH_OK;
}

}  // extern "C"
