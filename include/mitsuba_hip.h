/*
 * mitsuba_hip.h — C-ABI of the MI355X-native (gfx950) wavefront backend for the
 * `path` / `volpath` / `prb` integrator loop of ksalesin/mitsuba3-nasa.
 *
 * This is the drop-in boundary.  Plain C types only: no HIP,
 * no torch, no C++ in the signatures.  Every entry point returns an `int`
 * status (MH_OK == 0); on failure `mh_last_error()` returns a thread-local,
 * human-readable message whose text mirrors the reference's `Throw(...)`
 * messages where one exists.  No C++ exception ever crosses this boundary.
 *
 * Reference interfaces each entry point replaces (paths relative to the
 * reference checkout):
 *
 *   mh_scene_create / mh_scene_destroy
 *       Scene::Scene + accel_init_gpu (OptiX GAS/IAS build)
 *       src/render/scene.cpp:22-96, src/render/scene_optix.inl:304-547
 *   mh_scene_update_texture / mh_scene_update_rgb / mh_scene_update_medium
 *       SceneParameters.update -> Scene::parameters_changed
 *       src/python/python/util.py:292-350, src/render/scene.cpp:481-529
 *   mh_render
 *       SamplingIntegrator::render (JIT branch)        src/render/integrator.cpp:276-390
 *       ADIntegrator.render (prb primal)               src/python/python/ad/integrators/common.py:47-111
 *       (the film is left un-developed: RGBW, i.e. `develop=False` + Film storage)
 *   mh_develop
 *       HDRFilm::develop (JIT branch)                  src/films/hdrfilm.cpp:304-405
 *   mh_render_backward
 *       RBIntegrator.render_backward                   src/python/python/ad/integrators/common.py:828-983
 *       (+ PRBIntegrator.sample adjoint mode           src/python/python/ad/integrators/prb.py:59-257)
 *   mh_render_forward
 *       RBIntegrator.render_forward                    src/python/python/ad/integrators/common.py:696-826
 *       (+ PRBIntegrator.sample forward mode           src/python/python/ad/integrators/prb.py:244-248)
 *   mh_trace_closest / mh_trace_shadow
 *       Scene::ray_intersect_preliminary_gpu / ray_test_gpu (the OptiX slot)
 *       src/render/scene_optix.inl:592-721, include/mitsuba/render/optix/common.h:43-58
 *   mh_comm_* / mh_scene_set_comm / mh_render_sharded / mh_render_backward_sharded
 *       no reference counterpart (the reference renders on one device); they
 *       split the sample loop of SamplingIntegrator::render
 *       (src/render/integrator.cpp:276-390) and of render_backward
 *       (common.py:828-983) into per-device slabs, SURVEY.md §8(e)
 *
 * Units / conventions: all matrices are row-major float[16] (4x4) or
 * float[12] (3x4 affine, last row implicitly 0 0 0 1) and equal the
 * reference's `Transform4f::matrix`.  Images are (height, width, channels),
 * channel-fastest, float32.
 */
#ifndef MITSUBA_HIP_H
#define MITSUBA_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MH_ABI_VERSION 2u  /* 2: mh_stats gained grid_lookups, aux_items, ms_aux, n_aux_launches */
#define MH_INVALID 0xffffffffu

/* ----------------------------------------------------------------------- */
/* Status codes                                                             */
/* ----------------------------------------------------------------------- */
enum {
    MH_OK = 0,
    MH_ERR_INVALID_ARGUMENT = 1,
    MH_ERR_HIP = 2,
    MH_ERR_OUT_OF_MEMORY = 3,
    MH_ERR_UNSUPPORTED = 4,
    MH_ERR_NO_DEVICE = 5
};

/* ----------------------------------------------------------------------- */
/* Plugin type tags (names follow the reference plugin names)               */
/* ----------------------------------------------------------------------- */
enum { MH_SHAPE_RECTANGLE = 0, MH_SHAPE_MESH = 1 };           /* rectangle.cpp, mesh.cpp (cube.cpp) */
enum { MH_BSDF_DIFFUSE = 0, MH_BSDF_NULL = 1 };               /* diffuse.cpp, null.cpp */
enum { MH_TEX_RGB = 0, MH_TEX_BITMAP = 1 };                   /* srgb.cpp, bitmap.cpp */
enum { MH_EMITTER_AREA = 0, MH_EMITTER_CONSTANT = 1, MH_EMITTER_DIRECTIONAL = 2 };
enum { MH_RFILTER_BOX = 0, MH_RFILTER_GAUSSIAN = 1 };         /* box.cpp, gaussian.cpp */
/* Bitmap::PixelFormat of hdrfilm's 'pixel_format': rgb / luminance / xyz, and
 * the alpha variants rgba / ya / xyza (films with FilmFlags::Alpha) */
enum { MH_PIXEL_RGB = 0, MH_PIXEL_Y = 1, MH_PIXEL_XYZ = 2, MH_PIXEL_RGBA = 3, MH_PIXEL_YA = 4,
       MH_PIXEL_XYZA = 5 };
enum { MH_MEDIUM_HETEROGENEOUS = 0, MH_MEDIUM_HOMOGENEOUS = 1 };
enum { MH_PHASE_ISOTROPIC = 0, MH_PHASE_HG = 1 };
enum { MH_MEDIUM_NO_EMITTER_SAMPLING = 1u,        /* medium.cpp:29 sample_emitters = false */
       MH_MEDIUM_NO_SPECTRAL_EXTINCTION = 2u };   /* heterogeneous.cpp:161 has_spectral_extinction = false */
enum { MH_INTEGRATOR_PATH = 0, MH_INTEGRATOR_VOLPATH = 1, MH_INTEGRATOR_PRB = 2,
       MH_INTEGRATOR_PRBVOLPATH = 3 };                        /* python/ad/integrators/prbvolpath.py */

/* Differentiable parameter ids of mh_render_backward (param_textures[]):
 * a texture index (kind 0: '<bsdf>.reflectance.value' / '.data'), or a kind
 * tag | medium index.  Medium parameters need MH_INTEGRATOR_PRBVOLPATH.
 *   MH_PARAM_MEDIUM_SIGMA_T | m : '<medium>.sigma_t.data' (heterogeneous grid,
 *                                 res_x*res_y*res_z floats) or '.value'
 *                                 (homogeneous, 1 float)
 *   MH_PARAM_MEDIUM_ALBEDO | m  : '<medium>.albedo.value' (3 floats)        */
#define MH_PARAM_KIND_MASK      0xF0000000u
#define MH_PARAM_MEDIUM_SIGMA_T 0x10000000u
#define MH_PARAM_MEDIUM_ALBEDO  0x20000000u

/* Flags for mh_render / mh_render_backward / mh_trace_*                   */
enum {
    MH_FLAG_DEVICE_POINTERS = 1u << 0,  /* in/out buffers are device pointers on the scene's device */
    MH_FLAG_ACCUMULATE      = 1u << 1,  /* mh_render: add into `film_rgbw` instead of overwriting */
    MH_FLAG_NO_SYNC         = 1u << 2,  /* do not synchronise the stream before returning: with
                                           MH_FLAG_DEVICE_POINTERS and stats == NULL, mh_render /
                                           mh_prb_weights / mh_render_backward / mh_render_forward /
                                           mh_develop return once their work is enqueued */
    MH_FLAG_MEGAKERNEL      = 1u << 3,  /* mh_render: force the per-lane megakernel */
    MH_FLAG_WAVEFRONT       = 1u << 4,  /* mh_render: force the wavefront (trace/shade/shadow) kernels */
    MH_FLAG_PRB_REPLAY      = 1u << 5,  /* mh_render_backward: primal + adjoint replay even for rgb params */
    MH_FLAG_DETERMINISTIC   = 1u << 6,  /* film / W-image splat as a fixed-order gather instead of float
                                           atomics: bit-reproducible films; mh_render_backward on the fused
                                           wavefront: rgb gradients summed per path and reduced in path-id
                                           order, and bitmap texels in int64 fixed point (a max pass sizes
                                           the scale), bit-reproducible; prbvolpath gradients (grid sigma_t
                                           and the small slots) in int64 fixed point (the backward runs
                                           twice), bit-reproducible; the replay kernel and the rgb
                                           megakernel the same way (bitmap texels into an int64 mirror)
                                           (also env MH_DETERMINISTIC=1) */
    /* multi-GPU (the scene has a communicator, mh_scene_set_comm; one host
       thread per rank): the call sums its result over the ranks in-call, on
       the scene's stream -- mh_render / mh_render_forward the film,
       mh_prb_weights the W image, mh_render_backward the W image it computes
       (weights == NULL) and the gradients */
    MH_FLAG_REDUCE          = 1u << 7,  /* all ranks receive the sum */
    MH_FLAG_REDUCE_ROOT     = 1u << 8,  /* films: only rank 0 receives the sum (a reduce, not an all-reduce);
                                           the other ranks' film is left undefined */
    MH_FLAG_LOCAL_WEIGHTS   = 1u << 9,  /* mh_render_backward with weights == NULL and MH_FLAG_REDUCE: every rank
                                           computes the whole W image itself (all spp of every pixel) instead
                                           of its slab's W + an all-reduce */
    MH_FLAG_SHARED_DEVICE   = 1u << 10  /* a performance hint, results unchanged: the caller runs another call on
                                           the same device at the same time (e.g. a forward beside a gradient
                                           pass, on two scene handles and streams), so the wavefront launches
                                           take a share of the CUs' slots and the two calls' launches interleave */
};

/* ----------------------------------------------------------------------- */
/* Flattened scene description (host memory; copied by mh_scene_create)     */
/* ----------------------------------------------------------------------- */
typedef struct mh_shape {
    uint32_t type;              /* MH_SHAPE_* */
    uint32_t bsdf;              /* index into bsdfs[] */
    uint32_t emitter;           /* index into emitters[] or MH_INVALID */
    uint32_t interior_medium;   /* index into media[] or MH_INVALID */
    uint32_t exterior_medium;   /* index into media[] or MH_INVALID */
    uint32_t face_offset;       /* meshes: first face in faces[] */
    uint32_t face_count;        /* meshes: #triangles; rectangles: 1 */
    uint32_t vertex_offset;     /* meshes: first vertex in positions[]/normals[]/texcoords[] */
    uint32_t vertex_count;
    uint32_t has_normals;       /* meshes: per-vertex normals present */
    uint32_t has_texcoords;     /* meshes: per-vertex uvs present */
    uint32_t pad0;
    float to_world[12];         /* rectangles: Transform4f::matrix (3x4) */
    float to_object[12];        /* rectangles: inverse of to_world (3x4) */
    float frame_s[3];           /* rectangles: m_frame (rectangle.cpp:115-126) */
    float frame_t[3];
    float frame_n[3];
    float inv_area;             /* rectangles: m_inv_surface_area */
} mh_shape;

typedef struct mh_texture {
    uint32_t type;              /* MH_TEX_* */
    uint32_t width, height;     /* bitmap resolution */
    uint32_t channels;          /* bitmap: 1 or 3 */
    uint64_t data_offset;       /* bitmap: first float in texels[] (row-major, channel fastest) */
    uint32_t filter;            /* bitmap: 0 nearest, 1 bilinear */
    uint32_t wrap;              /* bitmap: 0 repeat, 1 mirror, 2 clamp */
    float value[3];             /* rgb: SRGBReflectanceSpectrum::m_value */
    float to_uv[6];             /* bitmap: ScalarTransform3f (2x3 row-major) */
    float pad1;
} mh_texture;

typedef struct mh_bsdf {
    uint32_t type;              /* MH_BSDF_* */
    uint32_t reflectance;       /* diffuse: index into textures[] */
} mh_bsdf;

typedef struct mh_emitter {
    uint32_t type;              /* MH_EMITTER_* */
    uint32_t shape;             /* area: index into shapes[] (rectangles only) */
    uint32_t pad0, pad1;
    float radiance[3];          /* area / constant: radiance; directional: irradiance */
    float direction[3];         /* directional: world-space propagation direction (normalised) */
    float scene_center[3];      /* constant / directional: bounding sphere of the scene */
    float scene_radius;
} mh_emitter;

typedef struct mh_medium {
    uint32_t type;              /* MH_MEDIUM_* */
    uint32_t phase;             /* MH_PHASE_* */
    float g;                    /* HG asymmetry */
    float scale;                /* sigma_t scale */
    float albedo[3];            /* constant single-scattering albedo */
    float sigma_t_const;        /* homogeneous: sigma_t (before scale) */
    uint32_t grid_res[3];       /* heterogeneous: sigma_t grid resolution (x, y, z) */
    uint32_t flags;             /* MH_MEDIUM_NO_EMITTER_SAMPLING | MH_MEDIUM_NO_SPECTRAL_EXTINCTION */
    uint64_t grid_offset;       /* heterogeneous: first float in grid_data[] (z-major: x fastest) */
    float grid_to_local[12];    /* world -> grid-local [0,1]^3 (3x4) */
    float bbox_min[3];          /* world-space AABB of the grid */
    float bbox_max[3];
    float max_density;          /* max(grid) — the global majorant is scale * max_density */
    float pad1;
} mh_medium;

typedef struct mh_sensor {
    float to_world[16];         /* PerspectiveCamera m_to_world */
    float sample_to_camera[16]; /* m_sample_to_camera (perspective.cpp:174-184) */
    float near_clip, far_clip;
    uint32_t width, height;     /* film size == crop size (crop_offset = 0) */
    uint32_t rfilter;           /* MH_RFILTER_* */
    float rfilter_radius;       /* gaussian: 4 * stddev */
    float filter_coeff[10];     /* gaussian: scaled Remez coefficients (gaussian.cpp:57-89) */
    uint32_t sample_count;      /* sampler.sample_count */
    uint32_t sampler_seed;      /* sampler base seed ('seed' property, default 0) */
    uint32_t medium;            /* camera medium index or MH_INVALID */
    uint32_t pixel_format;      /* MH_PIXEL_*: hdrfilm 'pixel_format' of mh_develop's output */
} mh_sensor;

typedef struct mh_scene_desc {
    uint32_t abi_version;       /* must be MH_ABI_VERSION */
    uint32_t pad0;
    mh_sensor sensor;
    uint32_t n_shapes, n_bsdfs, n_textures, n_emitters, n_media, n_vertices, n_faces, pad1;
    const mh_shape   *shapes;
    const mh_bsdf    *bsdfs;
    const mh_texture *textures;
    const mh_emitter *emitters;
    const mh_medium  *media;
    const float      *positions;   /* n_vertices * 3 (world space) */
    const float      *normals;     /* n_vertices * 3 or NULL */
    const float      *texcoords;   /* n_vertices * 2 or NULL */
    const uint32_t   *faces;       /* n_faces * 3, shape-local vertex indices */
    const float      *texels;      /* bitmap data */
    uint64_t          n_texels;
    const float      *grid_data;   /* volume grid data */
    uint64_t          n_grid;
    uint32_t          environment; /* index of the environment emitter (constant) or MH_INVALID */
    uint32_t          pad2;
} mh_scene_desc;

typedef struct mh_integrator {
    uint32_t type;              /* MH_INTEGRATOR_* */
    uint32_t max_depth;         /* -1 (infinite) is passed as 0xffffffff */
    uint32_t rr_depth;
    uint32_t hide_emitters;
} mh_integrator;

/* Per-call render statistics (device counters; deterministic at fixed seed) */
typedef struct mh_stats {
    uint64_t samples;           /* W*H*spp processed */
    uint64_t rays_closest;      /* closest-hit traversals */
    uint64_t rays_shadow;       /* shadow (any-hit) traversals */
    uint64_t bounces;           /* active lane-bounces */
    double   ms_total;          /* wall time of the call (host clock, ms) */
    double   ms_kernel;         /* device time of the dominant kernel (hipEvents, ms) */
    double   ms_trace;          /* wavefront: device time of all k_wf_trace (mode 1) / k_wf_bounce (mode 2) launches (ms);
                                   volpath on the phase scheduler (mode 3): its k_vol_sched launches */
    uint64_t n_trace_launches;  /* wavefront: number of those launches */
    uint32_t mode;              /* 0 megakernel, 1 wavefront (trace/shade/shadow), 2 wavefront fused bounce kernel,
                                   3 volpath wavefront (main / walk rounds) */
    uint32_t invalid_samples;   /* samples with a non-finite or negative (< -1e-5) radiance channel: the
                                   test of ImageBlock::put's warn_invalid / warn_negative (imageblock.cpp:180-204) */
    uint64_t grid_lookups;      /* volpath on the phase scheduler: trilinear density-grid lookups (8 taps each,
                                   GridVolume::eval, grid.cpp:321-384); 0 elsewhere */
    uint64_t aux_items;         /* items of the secondary kernel: bitmap vertex records the texel scatter read
                                   (prb with a bitmap parameter), film samples the splat read (mh_render) */
    double   ms_aux;            /* device time (hipEvents) of the secondary kernel's launches: the bitmap texel
                                   scatter (mh_render_backward) or the film splat (mh_render, wavefront modes) */
    uint64_t n_aux_launches;    /* number of those launches (one per chunk).  The fused wavefront runs a
                                   call's chunks on two streams: ms_trace / ms_aux then sum spans that
                                   overlap in time (MH_WF_STREAMS=1: one stream) */
} mh_stats;

typedef struct mh_scene mh_scene;   /* opaque; owns all device buffers */

/* ----------------------------------------------------------------------- */
/* Entry points                                                             */
/* ----------------------------------------------------------------------- */
const char *mh_last_error(void);
uint32_t    mh_abi_version(void);
int         mh_device_count(int *count);

/* Scene lifetime. `device` is a HIP ordinal; `stream` a hipStream_t, or NULL
   to let the scene create (and own) a non-blocking stream.  set_stream(NULL)
   selects the device's default (null) stream. */
int mh_scene_create(const mh_scene_desc *desc, int device, void *stream, mh_scene **out);
int mh_scene_destroy(mh_scene *scene);
int mh_scene_set_stream(mh_scene *scene, void *stream);

/* Parameter updates (traverse()/update() of 'x.reflectance.value' / '.data'). */
int mh_scene_update_rgb(mh_scene *scene, uint32_t texture, const float value[3]);
/*
 * Medium parameters (SceneParameters.update -> HeterogeneousMedium /
 * HomogeneousMedium::parameters_changed, heterogeneous.cpp:176-178):
 *   albedo  : 3 floats (host) or NULL
 *   sigma_t : homogeneous sigma_t value (1 float, host) or NULL
 *   grid    : heterogeneous sigma_t grid (n = res_x*res_y*res_z floats; host,
 *             or device with MH_FLAG_DEVICE_POINTERS) or NULL.  The majorant
 *             is recomputed as scale * max(grid).
 */
int mh_scene_update_medium(mh_scene *scene, uint32_t medium, const float *albedo, const float *sigma_t,
                           const float *grid, uint64_t n, uint32_t flags);
int mh_scene_update_texture(mh_scene *scene, uint32_t texture, const float *data, uint64_t n_floats);

/*
 * Forward render into the un-developed film storage: RGBW (H*W*4 floats), or
 * R G B A W (H*W*5) when the film has an alpha channel (MH_PIXEL_RGBA / YA /
 * XYZA; hdrfilm.cpp:327-330 base_ch = 5).  A sample's alpha is 1 where the
 * integrator reports a valid ray, else 0 (integrator.cpp:1229-1231; path
 * valid_ray, prb depth != 0, volpath / prbvolpath valid_ray), splatted with
 * the sample's filter weights like the colour.
 *   seed      : render seed (Integrator::render `seed`)
 *   spp       : samples per pixel (0 = sensor sample_count)
 *   spp_begin/spp_end : sample-slab [begin, end) of every pixel rendered by this call
 *               (multi-GPU sample-slab sharding); pass 0, 0 for all.
 *   film_rgbw : output (host or device pointer per flags)
 */
int mh_render(mh_scene *scene, const mh_integrator *integrator, uint32_t seed, uint32_t spp,
              uint32_t spp_begin, uint32_t spp_end, float *film_rgbw, uint32_t flags,
              mh_stats *stats);

/*
 * Per-sample outputs of the integrator (the value `sample()` returns per lane,
 * path.cpp:283-286 / prb.py:253-257) and the splat position, for sample-level
 * parity tests.  out = 5 SoA planes of n = W*H*(spp_end-spp_begin) floats:
 * L.r, L.g, L.b, pos.x, pos.y, lane order idx = pixel * S + s, plus a 6th
 * plane (alpha: 1 valid, 0 not) when the film has alpha.  Single pass only.
 */
int mh_render_samples(mh_scene *scene, const mh_integrator *integrator, uint32_t seed,
                      uint32_t spp, uint32_t spp_begin, uint32_t spp_end, float *out,
                      uint32_t flags);

/* film -> developed image (HDRFilm::develop, hdrfilm.cpp:304-405):
 * H*W*3 for MH_PIXEL_RGB (rgb / w) and MH_PIXEL_XYZ (srgb_to_xyz(rgb) / w),
 * H*W*1 for MH_PIXEL_Y (luminance(rgb) / w); the alpha formats append a / w:
 * H*W*4 (RGBA, XYZA), H*W*2 (YA).  w == 0 divides by 1. */
int mh_develop(mh_scene *scene, const float *film_rgbw, float *image_rgb, uint32_t flags);

/*
 * Reverse-mode derivative of render(): accumulates d(loss)/d(param) for each
 * listed parameter into grads[k] (3 floats for MH_TEX_RGB, W*H*C for
 * MH_TEX_BITMAP; medium ids: see MH_PARAM_*).  `grad_in` is d(loss)/d(rgb
 * before the colour conversion of develop), H*W*3: the caller applies the
 * adjoint of luminance / srgb_to_xyz and drops the alpha channel, whose
 * value (a validity mask) carries no derivative.  integrator: MH_INTEGRATOR_PRB (prb.py) or MH_INTEGRATOR_PRBVOLPATH
 * (prbvolpath.py: primal + adjoint replay per lane; grid gradients are
 * scattered with float atomics, so their summation order is not fixed).
 *   weights_rgbw (optional, device flag applies): the per-pixel filter-weight
 *   image W of the backward pass; pass NULL to compute it in-call.  Multi-GPU
 *   callers compute the W image per slab with mh_prb_weights, all-reduce it
 *   and pass it in.
 */
int mh_prb_weights(mh_scene *scene, uint32_t seed, uint32_t spp, uint32_t spp_begin,
                   uint32_t spp_end, float *weights, uint32_t flags);
int mh_render_backward(mh_scene *scene, const mh_integrator *integrator, uint32_t seed,
                       uint32_t spp, uint32_t spp_begin, uint32_t spp_end,
                       const float *grad_in, const float *weights, uint32_t n_params,
                       const uint32_t *param_textures, float *const *grads, uint32_t flags,
                       mh_stats *stats);

/*
 * Forward-mode derivative of render(): RBIntegrator.render_forward
 * (src/python/python/ad/integrators/common.py:696-826).  tangents[k] holds
 * the input tangent of parameter param_textures[k] (same shape and ids as
 * mh_render_backward's grads[k]; host or device per flags).  The sample's
 * tangent radiance dL (prb.py:244-248, `δL += dr.forward_to(Lo)`) is splatted
 * like a primal sample, value = dL, weight 1 and alpha = the ray validity
 * (common.py:799-806), into the film storage of mh_render (RGBW, or R G B A W
 * for alpha films); mh_develop then yields the gradient image, whose alpha
 * channel is the developed coverage, as film.develop() returns it
 * (common.py:808-824).  One AD wavefront of <= 2^32 samples per call
 * (common.py:571-578).  integrator: MH_INTEGRATOR_PRB or MH_INTEGRATOR_PRBVOLPATH.
 */
int mh_render_forward(mh_scene *scene, const mh_integrator *integrator, uint32_t seed,
                      uint32_t spp, uint32_t spp_begin, uint32_t spp_end, uint32_t n_params,
                      const uint32_t *param_textures, const float *const *tangents,
                      float *film_rgbw, uint32_t flags, mh_stats *stats);

/*
 * Ray-query sub-boundary (the OptiX slot).  Rays are SoA: ray[0..6][n] =
 * o.x o.y o.z d.x d.y d.z maxt (mint = 0).  Output = the payload of
 * Scene::ray_intersect_preliminary_gpu (scene_optix.inl:592-657,
 * optix/common.h:43-58, optix_rt.cu:9-17):
 *   t         hit distance; +inf on a miss (the miss program)
 *   u, v      prim_uv; (0, 0) on a miss (the payload's initial value)
 *   prim      prim_index: the face index of a mesh triangle, 0 for a
 *             rectangle (rectangle.cuh:42) and 0 on a miss
 *   shape     shape index; 0xffffffff (null ShapePtr) on a miss
 *   instance  (mh_trace_preliminary only; may be NULL) the instance of the
 *             hit: always 0xffffffff (null) here, since hip_ad_rgb scenes have
 *             no shapegroups / instances (payload_inst_index starts at 0 and
 *             stays null when m_shapegroups is empty, scene_optix.inl:607-608)
 */
int mh_trace_closest(mh_scene *scene, uint64_t n, const float *rays, float *t, float *u,
                     float *v, uint32_t *prim, uint32_t *shape, uint32_t flags, mh_stats *stats);
int mh_trace_preliminary(mh_scene *scene, uint64_t n, const float *rays, float *t, float *u, float *v,
                         uint32_t *prim, uint32_t *shape, uint32_t *instance, uint32_t flags,
                         mh_stats *stats);
int mh_trace_shadow(mh_scene *scene, uint64_t n, const float *rays, uint32_t *occluded,
                    uint32_t flags, mh_stats *stats);

/* BVH introspection (host): #nodes, #primitives, max depth. */
int mh_scene_bvh_info(mh_scene *scene, uint32_t *n_nodes, uint32_t *n_prims, uint32_t *depth);

/* ----------------------------------------------------------------------- */
/* Multi-GPU: sample-slab sharding + RCCL over xGMI        */
/* ----------------------------------------------------------------------- */
/*
 * The reference renders one device per process and has no collective: its
 * splice point is SamplingIntegrator::render (src/render/integrator.cpp:276-390),
 * whose sample loop this layer cuts into per-device slabs [spp*r/N, spp*(r+1)/N)
 * of every pixel.  The global lane index (hence every lane's TEA seed,
 * integrator.cpp:323-340) is the single-device one, so the slabs' union is
 * sample-identical to one render and the only exchanges are sums: the film,
 * the W image of render_backward (common.py:936-947) and the gradients.
 *
 * An mh_comm is one rank of an RCCL communicator, bound to one device.  RCCL
 * (librccl.so.1) is loaded on first use; without it these calls return
 * MH_ERR_UNSUPPORTED and the rest of the library is unaffected.
 *   mh_comm_unique_id   : rank 0 creates the id and ships it to the others
 *                         (any out-of-band channel: MPI, a file, a socket)
 *   mh_comm_create      : one rank per host thread / process (ncclCommInitRank)
 *   mh_comm_create_all  : one host thread drives `ndev` devices (ncclCommInitAll);
 *                         out[i] is the rank on devices[i]
 */
#define MH_COMM_ID_BYTES 128
typedef struct mh_comm mh_comm;
int mh_comm_unique_id(uint8_t id[MH_COMM_ID_BYTES]);
int mh_comm_create(const uint8_t id[MH_COMM_ID_BYTES], int nranks, int rank, int device, mh_comm **out);
int mh_comm_create_all(int ndev, const int *devices, mh_comm **out);
/* Fails (MH_ERR_INVALID_ARGUMENT, nothing destroyed) while a scene still
 * holds the communicator (mh_scene_set_comm): detach it first. */
int mh_comm_destroy(mh_comm *comm);
int mh_comm_info(const mh_comm *comm, int *nranks, int *rank, int *device);
/*
 * Sum `count` floats over the ranks, in place, for `n` ranks driven by the
 * calling thread (n == 1 for one thread per rank; all of them in one RCCL
 * group otherwise).  bufs[i] / streams[i] live on comms[i]'s device (a NULL
 * stream is that device's null stream).  root < 0: all-reduce; root = r:
 * reduce to rank r.  Stream-ordered: returns once enqueued.
 */
int mh_comm_reduce(mh_comm *const *comms, int n, float *const *bufs, uint64_t count, void *const *streams,
                   int root);
/* The scene's communicator for MH_FLAG_REDUCE / MH_FLAG_REDUCE_ROOT (NULL
 * detaches); its device must be the scene's.  The scene holds it until it is
 * detached or the scene is destroyed.
 * Failure handling of the in-call collectives: a call that fails after its
 * argument checks aborts the communicator (ncclCommAbort; later collectives
 * on it fail at once), and a call waits for its collectives with a deadline
 * (MH_COMM_TIMEOUT_S, default 1800 s) while watching the communicator's
 * async error, so a rank whose peer failed returns an error instead of
 * waiting forever.  Create a new communicator after such a failure. */
int mh_scene_set_comm(mh_scene *scene, mh_comm *comm);
/* Wait for the scene's stream (after MH_FLAG_NO_SYNC calls). */
int mh_scene_synchronize(mh_scene *scene);

/*
 * One host thread drives `n` scenes (one per device, or several on one device):
 * scene i renders the sample slab [spp*i/n, spp*(i+1)/n) of every pixel, the
 * slabs run concurrently on the scenes' streams, and the films are summed
 * into films[0] (root) or into every films[i] (MH_FLAG_REDUCE).  The sum goes
 * over the scenes' communicators when every scene has one (one RCCL group),
 * else through device copies onto scene 0's device (peer copies between
 * devices; scenes sharing a device need no peer access).  films[i]: device
 * pointers on scene i's device (MH_FLAG_DEVICE_POINTERS is implied).  stats
 * (optional): n entries.  Returns after every stream has drained.
 */
int mh_render_sharded(mh_scene *const *scenes, uint32_t n, const mh_integrator *integrator, uint32_t seed,
                      uint32_t spp, float *const *films, uint32_t flags, mh_stats *stats);
/*
 * render_backward over the same slabs: every scene computes its slab's W
 * image, the W images are summed to every scene, each scene differentiates
 * its slab with the total W, and the gradients are summed into every
 * grads[i * n_params + k] (device pointers on scene i's device; accumulated
 * into like mh_render_backward).  grad_in[i]: d loss / d image on scene i's
 * device (the same image on every scene).
 */
int mh_render_backward_sharded(mh_scene *const *scenes, uint32_t n, const mh_integrator *integrator,
                               uint32_t seed, uint32_t spp, const float *const *grad_in, uint32_t n_params,
                               const uint32_t *param_textures, float *const *grads, uint32_t flags,
                               mh_stats *stats);

#ifdef __cplusplus
}
#endif
#endif /* MITSUBA_HIP_H */
