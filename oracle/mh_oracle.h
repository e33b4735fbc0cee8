/*
 * mh_oracle.h — CPU restatement of the reference's `path` / `prb` / `volpath`
 * hot path (ksalesin/mitsuba3-nasa, llvm_ad_rgb semantics).
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker and the
 * `cpu_baseline` leg of bench.py.  It is never linked into, loaded by, or
 * called from the product (`mitsuba3-nasa_amd/`).  Only `tests/`,
 * `__graft_entry__.smoke()` and `bench.py`'s cpu_baseline leg may use it.
 *
 * Parity pinning: TEA known answers (src/core/tests/test_random.py:8-27),
 * Gaussian filter value (src/rfilters/tests/test_rfilter.py:14-17), diffuse
 * eval/pdf (src/bsdfs/tests/test_diffuse.py:13-35), rectangle hits
 * (src/shapes/tests/test_rectangle.py:34-60), cube hits
 * (src/shapes/tests/test_cube.py), PRB linearity (src/render/tests/test_ad.py)
 * and the PCG32 reference stream (pcg-basic, pcg32_srandom(42, 54)).  Dr.Jit
 * 0.4.4 internals (PCG32, Cephes sincos, Estrin, Texture2f) are restated from
 * the published algorithms; see DESIGN.md §Oracle.
 */
#ifndef MH_ORACLE_H
#define MH_ORACLE_H

#include <stdint.h>
#include "../include/mitsuba_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* --- known-answer hooks ------------------------------------------------- */
void  oracle_tea32(uint32_t v0, uint32_t v1, int rounds, uint32_t *o0, uint32_t *o1);
float oracle_tea_float32(uint32_t v0, uint32_t v1, int rounds);
double oracle_tea_float64(uint32_t v0, uint32_t v1, int rounds);
/* PCG32 stream: seed(initstate, initseq) then n x next_uint32 */
void  oracle_pcg32_stream(uint64_t initstate, uint64_t initseq, uint32_t n, uint32_t *out);
/* per-lane sampler stream of Mitsuba's PCG32Sampler (sampler.cpp:115-134) */
void  oracle_sampler_floats(uint32_t seed_value, uint32_t lane, uint32_t n, float *out);
float oracle_gaussian_eval(const float coeff[10], float x);
void  oracle_sincos(float x, float *s, float *c);
float oracle_log(float x);
float oracle_exp(float x);
void  oracle_diffuse_eval_pdf(const float wi[3], const float wo[3], const float rho[3],
                              float value[3], float *pdf);
void  oracle_square_to_cosine_hemisphere(const float s[2], float out[3]);

/* --- ray queries (brute force over shapes; SoA rays like mh_trace_*) ---- */
int oracle_trace_closest(const mh_scene_desc *desc, uint64_t n, const float *rays, float *t,
                         float *u, float *v, uint32_t *prim, uint32_t *shape);
int oracle_trace_shadow(const mh_scene_desc *desc, uint64_t n, const float *rays,
                        uint32_t *occluded);

/* --- camera ------------------------------------------------------------- */
int oracle_camera_ray(const mh_scene_desc *desc, const float adjusted_pos[2], float o[3],
                      float d[3], float *maxt);

/* --- rendering ------------------------------------------------------------
 * Per-sample radiance (L, sample_pos, valid) for sample-index range
 * [idx_begin, idx_end) of the wavefront  idx = pixel * spp + s.
 * out_L: 3*(n), out_pos: 2*(n), out_valid: n (may be NULL).              */
int oracle_sample_range(const mh_scene_desc *desc, const mh_integrator *integ, uint32_t seed,
                        uint32_t spp, uint64_t idx_begin, uint64_t idx_end, float *out_L,
                        float *out_pos, uint32_t *out_valid);

/* Full render into an RGBW film (H*W*4, overwritten).  spp_begin/end select
 * a sample slab of every pixel (0,0 = all).  n_threads >= 1.              */
/* density-grid lookups (valid heterogeneous medium samples) of every render
   since the last call with reset = 1 (the check of mh_stats.grid_lookups) */
uint64_t oracle_grid_lookups(int reset);
int oracle_render(const mh_scene_desc *desc, const mh_integrator *integ, uint32_t seed,
                  uint32_t spp, uint32_t spp_begin, uint32_t spp_end, int n_threads,
                  float *film_rgbw);
void oracle_develop(uint32_t w, uint32_t h, const float *film_rgbw, float *rgb);
void oracle_develop_format(uint32_t w, uint32_t h, uint32_t pixel_format, const float *film_rgbw, float *out);

/* PRB: per-pixel filter-weight image W (H*W) of the backward pass. */
int oracle_prb_weights(const mh_scene_desc *desc, uint32_t seed, uint32_t spp,
                       uint32_t spp_begin, uint32_t spp_end, int n_threads, float *weights);
int oracle_prb_weights_rows(const mh_scene_desc *desc, uint32_t seed, uint32_t spp, uint32_t row_lo,
                            uint32_t row_hi, int n_threads, float *weights);
/* PRB render_backward: grads[k] accumulated (double precision internally). */
int oracle_render_backward(const mh_scene_desc *desc, const mh_integrator *integ,
                           uint32_t seed, uint32_t spp, uint32_t spp_begin, uint32_t spp_end,
                           const float *grad_in, const float *weights, uint32_t n_params,
                           const uint32_t *param_textures, float *const *grads, int n_threads);

/* PRB render_forward (common.py:696-826): the film (as oracle_render) of the
   per-sample tangent radiance; tangents[k] has the shape of grads[k] above. */
int oracle_render_forward(const mh_scene_desc *desc, const mh_integrator *integ, uint32_t seed,
                          uint32_t spp, uint32_t spp_begin, uint32_t spp_end, uint32_t n_params,
                          const uint32_t *param_ids, const float *const *tangents, int n_threads,
                          float *film);

const char *oracle_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
