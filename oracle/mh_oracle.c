/*
 * mh_oracle.c — CPU restatement (plain C, scalar, fp32) of the reference's
 * `path` / `prb` hot path with llvm_ad_rgb (JIT) semantics.
 *
 * TEST INFRASTRUCTURE ONLY (see mh_oracle.h).  Every function cites the
 * reference file:line it restates (paths relative to /root/reference).
 * Conventions that make the product bit-comparable:
 *   - compiled with -ffp-contract=off; an explicit fmaf() appears exactly where
 *     the reference (or Dr.Jit) calls dr::fmadd / fmsub / fnmadd;
 *   - Dr.Jit 0.4.4 LLVM-backend lowering: rcp(x) = 1/x, rsqrt(x) = sqrt(1/x),
 *     sqrt/div correctly rounded, sincos/log = Cephes polynomials.
 */
#include "mh_oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* Error reporting                                                          */
/* ------------------------------------------------------------------------ */
static __thread char g_err[512];
const char *oracle_last_error(void) { return g_err; }
static int fail(const char *msg) {
    snprintf(g_err, sizeof(g_err), "%s", msg);
    return 1;
}

/* ------------------------------------------------------------------------ */
/* Dr.Jit scalar primitives (LLVM backend lowering)                         */
/* ------------------------------------------------------------------------ */
#define PI_F      3.14159265358979323846f
#define INV_PI_F  0.31830988618379067154f
#define INV_4PI_F 0.07957747154594766788f
/* include/mitsuba/core/math.h:18-23 with dr::Epsilon<float> = 2^-24 */
#define RAY_EPS    (1500.0f * 5.9604644775390625e-08f)
#define SHADOW_EPS (RAY_EPS * 10.0f)

typedef struct { float x, y, z; } v3;

static inline v3 V3(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 vadd(v3 a, v3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 vsub(v3 a, v3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 vmul(v3 a, v3 b) { return V3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 vscale(v3 a, float s) { return V3(a.x * s, a.y * s, a.z * s); }
static inline v3 vneg(v3 a) { return V3(-a.x, -a.y, -a.z); }
static inline v3 vdivs(v3 a, float s) { return V3(a.x / s, a.y / s, a.z / s); }
/* dr::fmadd(a, b, c) for a vector a, scalar b, vector c */
static inline v3 vfma_s(v3 a, float b, v3 c) {
    return V3(fmaf(a.x, b, c.x), fmaf(a.y, b, c.y), fmaf(a.z, b, c.z));
}
static inline v3 vfma(v3 a, v3 b, v3 c) {
    return V3(fmaf(a.x, b.x, c.x), fmaf(a.y, b.y, c.y), fmaf(a.z, b.z, c.z));
}
/* dr::dot: a.x*b.x, then fmadd chain */
static inline float vdot(v3 a, v3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
/* dr::cross: fmsub(a.y, b.z, a.z * b.y), ... */
static inline v3 vcross(v3 a, v3 b) {
    return V3(fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)),
              fmaf(a.x, b.y, -(a.y * b.x)));
}
static inline float rcpf_(float x) { return 1.0f / x; }
static inline float rsqrtf_(float x) { return sqrtf(1.0f / x); }
static inline v3 vnormalize(v3 v) { return vscale(v, rsqrtf_(vdot(v, v))); }
static inline float vnorm(v3 v) { return sqrtf(vdot(v, v)); }
static inline float vmax(v3 v) { return fmaxf(fmaxf(v.x, v.y), v.z); }
static inline v3 vload(const float *p) { return V3(p[0], p[1], p[2]); }
/* dr::mulsign for differentiable arrays: select(b >= 0, a, -a) */
static inline float mulsign(float a, float b) { return b >= 0.f ? a : -a; }
static inline float mulsign_neg(float a, float b) { return b >= 0.f ? -a : a; }
static inline float signf_(float a) { return a >= 0.f ? 1.f : -1.f; }
static inline int isfinitef_(float x) { return fabsf(x) < INFINITY; }
static inline float safe_sqrtf(float x) { return sqrtf(fmaxf(x, 0.f)); }

static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* Transform4f::operator*(Point) / transform_affine (core/transform.h:104-124),
   matrix m is row-major 3x4 (affine) */
static inline v3 xf_point(const float *m, v3 p) {
    return V3(fmaf(m[2], p.z, fmaf(m[1], p.y, fmaf(m[0], p.x, m[3]))),
              fmaf(m[6], p.z, fmaf(m[5], p.y, fmaf(m[4], p.x, m[7]))),
              fmaf(m[10], p.z, fmaf(m[9], p.y, fmaf(m[8], p.x, m[11]))));
}
/* Transform4f::operator*(Vector) (core/transform.h:132-141) */
static inline v3 xf_vector(const float *m, v3 v) {
    return V3(fmaf(m[2], v.z, fmaf(m[1], v.y, m[0] * v.x)),
              fmaf(m[6], v.z, fmaf(m[5], v.y, m[4] * v.x)),
              fmaf(m[10], v.z, fmaf(m[9], v.y, m[8] * v.x)));
}
/* same with a 4x4 row-major matrix (only the top 3 rows used) */
static inline v3 xf4_vector(const float *m, v3 v) {
    return V3(fmaf(m[2], v.z, fmaf(m[1], v.y, m[0] * v.x)),
              fmaf(m[6], v.z, fmaf(m[5], v.y, m[4] * v.x)),
              fmaf(m[10], v.z, fmaf(m[9], v.y, m[8] * v.x)));
}
/* projective point transform (core/transform.h:118-124) */
static inline v3 xf4_point_proj(const float *m, v3 p) {
    float r[4];
    for (int i = 0; i < 4; ++i)
        r[i] = fmaf(m[4 * i + 2], p.z, fmaf(m[4 * i + 1], p.y, fmaf(m[4 * i + 0], p.x, m[4 * i + 3])));
    return V3(r[0] / r[3], r[1] / r[3], r[2] / r[3]);
}

/* ------------------------------------------------------------------------ */
/* Cephes sincos / log as restated from Dr.Jit 0.4.4 include/drjit/math.h   */
/* ------------------------------------------------------------------------ */
static inline float poly2(float x, float c0, float c1, float c2) {
    float x2 = x * x;
    return fmaf(x2, c2, fmaf(x, c1, c0));
}

void oracle_sincos(float x, float *s_out, float *c_out) {
    float xa = fabsf(x);
    int32_t j = (int32_t)(xa * 1.2732395447351626862f);
    j = (j + 1) & ~1;
    float y = (float)j;
    uint32_t sign_sin = ((uint32_t)j << 29) ^ f2u(x);
    uint32_t sign_cos = (~(uint32_t)(j - 2)) << 29;
    y = xa - y * 0.78515625f - y * 2.4187564849853515625e-4f - y * 3.77489497744594108e-8f;
    float z = y * y;
    if (xa == INFINITY)
        z = u2f(0xffffffffu);
    float s = poly2(z, -1.6666654611e-1f, 8.3321608736e-3f, -1.9515295891e-4f) * z;
    float c = poly2(z, 4.166664568298827e-2f, -1.388731625493765e-3f, 2.443315711809948e-5f) * z;
    s = fmaf(s, y, y);
    c = fmaf(c, z, fmaf(z, -0.5f, 1.0f));
    int polymask = (j & 2) == 0;
    float rs = polymask ? s : c, rc = polymask ? c : s;
    *s_out = u2f(f2u(rs) ^ (sign_sin & 0x80000000u));
    *c_out = u2f(f2u(rc) ^ (sign_cos & 0x80000000u));
}

/* Cephes logf (frexp + rational polynomial), Dr.Jit 0.4.4 math.h `log` */
float oracle_log(float x) {
    if (!(x > 0.f)) {
        if (x == 0.f) return -INFINITY;
        return u2f(0xffffffffu); /* NaN */
    }
    if (x == INFINITY) return INFINITY;
    /* frexp: mantissa in [0.5, 1) */
    uint32_t bits = f2u(x);
    int e;
    float xm;
    if ((bits & 0x7f800000u) == 0) { /* denormal */
        xm = frexpf(x, &e);
    } else {
        e = (int)((bits >> 23) & 0xff) - 126;
        xm = u2f((bits & 0x807fffffu) | 0x3f000000u);
    }
    if (xm < 0.70710678118654752440f) {
        e -= 1;
        xm = xm + xm - 1.0f;
    } else {
        xm = xm - 1.0f;
    }
    float z = xm * xm;
    float y = 7.0376836292e-2f;
    y = fmaf(y, xm, -1.1514610310e-1f);
    y = fmaf(y, xm, 1.1676998740e-1f);
    y = fmaf(y, xm, -1.2420140846e-1f);
    y = fmaf(y, xm, 1.4249322787e-1f);
    y = fmaf(y, xm, -1.6668057665e-1f);
    y = fmaf(y, xm, 2.0000714765e-1f);
    y = fmaf(y, xm, -2.4999993993e-1f);
    y = fmaf(y, xm, 3.3333331174e-1f);
    y = y * xm * z;
    float fe = (float)e;
    y = fmaf(fe, -2.12194440e-4f, y);
    y = fmaf(z, -0.5f, y);
    float r = xm + y;
    r = fmaf(fe, 0.693359375f, r);
    return r;
}

/* ------------------------------------------------------------------------ */
/* TEA + PCG32 (include/mitsuba/core/random.h:77-140, sampler.cpp:115-134)  */
/* ------------------------------------------------------------------------ */
void oracle_tea32(uint32_t v0, uint32_t v1, int rounds, uint32_t *o0, uint32_t *o1) {
    uint32_t sum = 0;
    for (int i = 0; i < rounds; ++i) {
        sum += 0x9e3779b9u;
        v0 += ((v1 << 4) + 0xa341316cu) ^ (v1 + sum) ^ ((v1 >> 5) + 0xc8013ea4u);
        v1 += ((v0 << 4) + 0xad90777du) ^ (v0 + sum) ^ ((v0 >> 5) + 0x7e95761eu);
    }
    *o0 = v0;
    *o1 = v1;
}

float oracle_tea_float32(uint32_t v0, uint32_t v1, int rounds) {
    uint32_t a, b;
    oracle_tea32(v0, v1, rounds, &a, &b);
    return u2f((b >> 9) | 0x3f800000u) - 1.0f;
}

double oracle_tea_float64(uint32_t v0, uint32_t v1, int rounds) {
    uint32_t a, b;
    oracle_tea32(v0, v1, rounds, &a, &b);
    uint64_t v = (uint64_t)a | ((uint64_t)b << 32);
    uint64_t bits = (v >> 12) | 0x3ff0000000000000ull;
    double d;
    memcpy(&d, &bits, 8);
    return d - 1.0;
}

#define PCG32_MULT 0x5851f42d4c957f2dull
typedef struct { uint64_t state, inc; } pcg32;

static inline uint32_t pcg_next(pcg32 *r) {
    uint64_t old = r->state;
    r->state = old * PCG32_MULT + r->inc;
    uint32_t xorshifted = (uint32_t)(((old >> 18u) ^ old) >> 27u);
    uint32_t rot = (uint32_t)(old >> 59u);
    return (xorshifted >> rot) | (xorshifted << ((~rot + 1u) & 31));
}
/* [drjit] PCG32::seed(size, initstate, initseq) */
static inline void pcg_seed(pcg32 *r, uint64_t initstate, uint64_t initseq) {
    r->state = 0;
    r->inc = (initseq << 1) | 1u;
    pcg_next(r);
    r->state += initstate;
    pcg_next(r);
}
static inline float pcg_float(pcg32 *r) {
    return u2f((pcg_next(r) >> 9) | 0x3f800000u) - 1.0f;
}
/* PCG32Sampler::seed (sampler.cpp:115-134): TEA(seed_value, lane) -> seed(v0, v1) */
static inline void sampler_seed(pcg32 *r, uint32_t seed_value, uint32_t lane) {
    uint32_t v0, v1;
    oracle_tea32(seed_value, lane, 4, &v0, &v1);
    pcg_seed(r, v0, v1);
}

void oracle_pcg32_stream(uint64_t initstate, uint64_t initseq, uint32_t n, uint32_t *out) {
    pcg32 r;
    pcg_seed(&r, initstate, initseq);
    for (uint32_t i = 0; i < n; ++i) out[i] = pcg_next(&r);
}

void oracle_sampler_floats(uint32_t seed_value, uint32_t lane, uint32_t n, float *out) {
    pcg32 r;
    sampler_seed(&r, seed_value, lane);
    for (uint32_t i = 0; i < n; ++i) out[i] = pcg_float(&r);
}

/* ------------------------------------------------------------------------ */
/* Reconstruction filter: Gaussian (src/rfilters/gaussian.cpp:94-97)        */
/* [drjit] estrin_impl over 10 coefficients                                 */
/* ------------------------------------------------------------------------ */
static inline float estrin10(float x, const float *k) {
    float c0 = fmaf(x, k[1], k[0]), c1 = fmaf(x, k[3], k[2]), c2 = fmaf(x, k[5], k[4]),
          c3 = fmaf(x, k[7], k[6]), c4 = fmaf(x, k[9], k[8]);
    float x2 = x * x;
    float d0 = fmaf(x2, c1, c0), d1 = fmaf(x2, c3, c2), d2 = c4;
    float x4 = x2 * x2;
    float e0 = fmaf(x4, d1, d0), e1 = d2;
    float x8 = x4 * x4;
    return fmaf(x8, e1, e0);
}

float oracle_gaussian_eval(const float coeff[10], float x) {
    return fmaxf(estrin10(x * x, coeff), 0.f);
}

static inline float rfilter_eval(const mh_sensor *s, float x) {
    if (s->rfilter == MH_RFILTER_GAUSSIAN)
        return oracle_gaussian_eval(s->filter_coeff, x);
    return (fabsf(x) <= 0.5f) ? 1.f : 0.f; /* box.cpp (unused: box takes the fast path) */
}

/* ------------------------------------------------------------------------ */
/* ImageBlock::put (src/render/imageblock.cpp:174-532)                      */
/* values = R G B W (or R G B A W for alpha films, hdrfilm.cpp:327-330);     */
/* `film` is H x W x ch (row range [row0, row0+rows))                        */
/* ------------------------------------------------------------------------ */
typedef struct {
    float *data;
    uint32_t width, height; /* full film size */
    int32_t row0;           /* first row stored in `data` */
    uint32_t rows;          /* number of rows stored */
    uint32_t ch;            /* channels per pixel: 4 (RGBW) or 5 (RGBAW) */
} film_band;

static inline void band_add(film_band *f, uint32_t x, uint32_t y, const float *vals, float w,
                            int nch) {
    (void)nch;
    int32_t r = (int32_t)y - f->row0;
    if (r < 0 || r >= (int32_t)f->rows) return; /* caller sized the band to cover it */
    float *p = f->data + ((size_t)r * f->width + x) * f->ch;
    for (uint32_t k = 0; k < f->ch; ++k) p[k] += vals[k] * w;
}

static void splat(const mh_sensor *s, film_band *f, float px, float py, const float *vals,
                  int coalesce) {
    const uint32_t W = s->width, H = s->height;
    if (s->rfilter == MH_RFILTER_BOX) {
        /* fast special case for the box filter (imageblock.cpp:210-233) */
        int32_t ix = (int32_t)floorf(px), iy = (int32_t)floorf(py);
        uint32_t ux = (uint32_t)ix, uy = (uint32_t)iy;
        if (ux < W && uy < H) band_add(f, ux, uy, vals, 1.0f, 4);
        return;
    }
    const float radius = s->rfilter_radius;
    if (coalesce) {
        /* 2. coalesced, recorded-loop variant (imageblock.cpp:418-531) */
        int32_t n = (int32_t)ceilf(radius - 0.5f);
        int32_t count = 2 * n + 1;
        int32_t pix = (int32_t)floorf(px) - n, piy = (int32_t)floorf(py) - n;
        uint32_t x = (uint32_t)pix, y = (uint32_t)piy;
        float relx = ((float)pix + 0.5f) - px, rely = ((float)piy + 0.5f) - py;
        for (int32_t ys = 0; ys < count; ++ys) {
            float wy = rfilter_eval(s, rely + (float)ys);
            int act1 = (y + (uint32_t)ys) < H;
            for (int32_t xs = 0; xs < count; ++xs) {
                float wx = rfilter_eval(s, relx + (float)xs);
                float w = wx * wy;
                if (act1 && (x + (uint32_t)xs) < W)
                    band_add(f, x + (uint32_t)xs, y + (uint32_t)ys, vals, w, 4);
            }
        }
    } else {
        /* 1.2 non-coalesced, recorded-loop variant (imageblock.cpp:264-409) */
        float pfx = px - 0.5f, pfy = py - 0.5f;
        float p0x = pfx - radius, p0y = pfy - radius, p1x = pfx + radius, p1y = pfy + radius;
        int32_t a0x = (int32_t)ceilf(p0x), a0y = (int32_t)ceilf(p0y);
        int32_t a1x = (int32_t)floorf(p1x), a1y = (int32_t)floorf(p1y);
        if (a0x < 0) a0x = 0;
        if (a0y < 0) a0y = 0;
        if (a1x > (int32_t)W - 1) a1x = (int32_t)W - 1;
        if (a1y > (int32_t)H - 1) a1y = (int32_t)H - 1;
        uint32_t u0x = (uint32_t)a0x, u0y = (uint32_t)a0y, u1x = (uint32_t)a1x, u1y = (uint32_t)a1y;
        if (!(u0x <= u1x && u0y <= u1y)) return;
        uint32_t count = (uint32_t)ceilf(2.f * radius);
        float relx = (float)u0x - pfx, rely = (float)u0y - pfy;
        for (uint32_t ys = 0; ys < count; ++ys) {
            float wy = rfilter_eval(s, rely + (float)ys);
            int act1 = (u0y + ys) <= u1y;
            for (uint32_t xs = 0; xs < count; ++xs) {
                float wx = rfilter_eval(s, relx + (float)xs);
                float w = wx * wy;
                if (act1 && (u0x + xs) <= u1x)
                    band_add(f, u0x + xs, u0y + ys, vals, w, 4);
            }
        }
    }
}

/* HDRFilm::develop (src/films/hdrfilm.cpp:349-405) */
void oracle_develop(uint32_t w, uint32_t h, const float *film, float *rgb) {
    oracle_develop_format(w, h, MH_PIXEL_RGB, film, rgb);
}

/* HDRFilm::develop (hdrfilm.cpp:313-401): luminance / srgb_to_xyz of the
   weighted sums (spectrum.h:396-402, 431-434), then the weight division */
static int fmt_alpha(uint32_t fmt) {
    return fmt == MH_PIXEL_RGBA || fmt == MH_PIXEL_YA || fmt == MH_PIXEL_XYZA;
}

/* alpha films: the film holds R G B A W and the image gets a / w after the
   colour channels (hdrfilm.cpp:327-372: target_ch = color_ch + alpha) */
void oracle_develop_format(uint32_t w, uint32_t h, uint32_t fmt, const float *film, float *out) {
    size_t n = (size_t)w * h;
    const int alpha = fmt_alpha(fmt);
    const uint32_t fch = alpha ? 5 : 4;
    const int to_y = fmt == MH_PIXEL_Y || fmt == MH_PIXEL_YA, to_xyz = fmt == MH_PIXEL_XYZ || fmt == MH_PIXEL_XYZA;
    const uint32_t och = (to_y ? 1 : 3) + (alpha ? 1 : 0);
    for (size_t i = 0; i < n; ++i) {
        const float *v = film + fch * i;
        float W = v[fch - 1];
        float d = (W == 0.f) ? 1.f : W;
        float *o = out + och * i;
        if (to_y) {
            o[0] = ((v[0] * 0.212671f + v[1] * 0.715160f) + v[2] * 0.072169f) / d;
        } else {
            float c[3] = {v[0], v[1], v[2]};
            if (to_xyz) {
                c[0] = fmaf(0.180423f, v[2], fmaf(0.357580f, v[1], 0.412453f * v[0]));
                c[1] = fmaf(0.072169f, v[2], fmaf(0.715160f, v[1], 0.212671f * v[0]));
                c[2] = fmaf(0.950227f, v[2], fmaf(0.119193f, v[1], 0.019334f * v[0]));
            }
            for (int k = 0; k < 3; ++k) o[k] = c[k] / d;
        }
        if (alpha) o[och - 1] = v[3] / d;
    }
}

/* ------------------------------------------------------------------------ */
/* Scene view                                                               */
/* ------------------------------------------------------------------------ */
typedef struct {
    const mh_scene_desc *d;
    float (*bbox)[6]; /* per shape AABB */
} scene_view;

static void shape_bbox(const mh_scene_desc *d, uint32_t i, float *bb) {
    const mh_shape *sh = &d->shapes[i];
    bb[0] = bb[1] = bb[2] = INFINITY;
    bb[3] = bb[4] = bb[5] = -INFINITY;
    if (sh->type == MH_SHAPE_RECTANGLE) {
        static const float cs[4][2] = {{-1, -1}, {-1, 1}, {1, -1}, {1, 1}};
        for (int k = 0; k < 4; ++k) {
            v3 p = xf_point(sh->to_world, V3(cs[k][0], cs[k][1], 0.f));
            float q[3] = {p.x, p.y, p.z};
            for (int a = 0; a < 3; ++a) {
                if (q[a] < bb[a]) bb[a] = q[a];
                if (q[a] > bb[3 + a]) bb[3 + a] = q[a];
            }
        }
    } else {
        for (uint32_t v = 0; v < sh->vertex_count; ++v) {
            const float *q = d->positions + 3 * (size_t)(sh->vertex_offset + v);
            for (int a = 0; a < 3; ++a) {
                if (q[a] < bb[a]) bb[a] = q[a];
                if (q[a] > bb[3 + a]) bb[3 + a] = q[a];
            }
        }
    }
    /* conservative padding: the AABB is only a culling test */
    for (int a = 0; a < 3; ++a) {
        float e = 1e-4f * (fabsf(bb[a]) + fabsf(bb[3 + a]) + 1.f);
        bb[a] -= e;
        bb[3 + a] += e;
    }
}

static int scene_view_init(scene_view *sv, const mh_scene_desc *d) {
    if (!d || d->abi_version != MH_ABI_VERSION) return fail("scene: ABI version mismatch");
    sv->d = d;
    sv->bbox = (float (*)[6])malloc(sizeof(float) * 6 * (d->n_shapes ? d->n_shapes : 1));
    if (!sv->bbox) return fail("out of memory");
    for (uint32_t i = 0; i < d->n_shapes; ++i) shape_bbox(d, i, sv->bbox[i]);
    return 0;
}
static void scene_view_free(scene_view *sv) { free(sv->bbox); }

typedef struct { v3 o, d; float maxt; } ray3;

static inline int bbox_hit(const float *bb, v3 o, v3 d, float maxt) {
    float t0 = 0.f, t1 = maxt;
    float os[3] = {o.x, o.y, o.z}, ds[3] = {d.x, d.y, d.z};
    for (int a = 0; a < 3; ++a) {
        float inv = 1.0f / ds[a];
        float tn = (bb[a] - os[a]) * inv, tf = (bb[3 + a] - os[a]) * inv;
        if (tn > tf) { float tmp = tn; tn = tf; tf = tmp; }
        if (tn != tn) tn = -INFINITY; /* 0 * inf */
        if (tf != tf) tf = INFINITY;
        if (tn > t0) t0 = tn;
        if (tf < t1) t1 = tf;
    }
    return t0 <= t1 * 1.000001f + 1e-6f;
}

/* Rectangle::ray_intersect_preliminary_impl (src/shapes/rectangle.cpp:446-470) */
static inline int rect_intersect(const mh_shape *sh, const ray3 *r, float *t_out, float *u,
                                 float *v) {
    v3 o = xf_point(sh->to_object, r->o);
    v3 d = xf_vector(sh->to_object, r->d);
    float t = -o.z / d.z;
    v3 local = vfma_s(d, t, o); /* Ray::operator() = fmadd(d, t, o) (core/ray.h:61) */
    int hit = t >= 0.f && t <= r->maxt && fabsf(local.x) <= 1.f && fabsf(local.y) <= 1.f;
    *t_out = t;
    *u = local.x;
    *v = local.y;
    return hit;
}

/* Mesh::moeller_trumbore (include/mitsuba/render/mesh.h:430-453) */
static inline int tri_intersect(v3 p0, v3 p1, v3 p2, const ray3 *r, float *t_out, float *uo,
                                float *vo) {
    v3 e1 = vsub(p1, p0), e2 = vsub(p2, p0);
    v3 pvec = vcross(r->d, e2);
    float inv_det = rcpf_(vdot(e1, pvec));
    v3 tvec = vsub(r->o, p0);
    float u = vdot(tvec, pvec) * inv_det;
    int active = u >= 0.f && u <= 1.f;
    v3 qvec = vcross(tvec, e1);
    float v = vdot(r->d, qvec) * inv_det;
    active = active && v >= 0.f && u + v <= 1.f;
    float t = vdot(e2, qvec) * inv_det;
    active = active && t >= 0.f && t <= r->maxt;
    *t_out = t;
    *uo = u;
    *vo = v;
    return active;
}

static inline v3 mesh_vertex(const mh_scene_desc *d, const mh_shape *sh, uint32_t local) {
    return vload(d->positions + 3 * (size_t)(sh->vertex_offset + local));
}

typedef struct {
    float t, u, v;
    uint32_t prim, shape;
} pi_rec;

/* Scene::ray_intersect_preliminary (closest hit; scene.cpp:181-190) */
static void trace_closest(const scene_view *sv, const ray3 *r, pi_rec *pi) {
    const mh_scene_desc *d = sv->d;
    pi->t = INFINITY;
    pi->u = pi->v = 0.f;
    pi->prim = MH_INVALID;
    pi->shape = MH_INVALID;
    ray3 rr = *r;
    for (uint32_t s = 0; s < d->n_shapes; ++s) {
        if (!bbox_hit(sv->bbox[s], r->o, r->d, r->maxt)) continue;
        const mh_shape *sh = &d->shapes[s];
        float t, u, v;
        if (sh->type == MH_SHAPE_RECTANGLE) {
            if (rect_intersect(sh, &rr, &t, &u, &v) && t < pi->t) {
                pi->t = t; pi->u = u; pi->v = v; pi->prim = MH_INVALID; pi->shape = s;
            }
        } else {
            for (uint32_t f = 0; f < sh->face_count; ++f) {
                const uint32_t *fi = d->faces + 3 * (size_t)(sh->face_offset + f);
                if (tri_intersect(mesh_vertex(d, sh, fi[0]), mesh_vertex(d, sh, fi[1]),
                                  mesh_vertex(d, sh, fi[2]), &rr, &t, &u, &v) &&
                    t < pi->t) {
                    pi->t = t; pi->u = u; pi->v = v; pi->prim = f; pi->shape = s;
                }
            }
        }
    }
}

/* Scene::ray_test (any hit; scene.cpp:201-210) */
static int trace_shadow(const scene_view *sv, const ray3 *r) {
    const mh_scene_desc *d = sv->d;
    for (uint32_t s = 0; s < d->n_shapes; ++s) {
        if (!bbox_hit(sv->bbox[s], r->o, r->d, r->maxt)) continue;
        const mh_shape *sh = &d->shapes[s];
        float t, u, v;
        if (sh->type == MH_SHAPE_RECTANGLE) {
            if (rect_intersect(sh, r, &t, &u, &v)) return 1;
        } else {
            for (uint32_t f = 0; f < sh->face_count; ++f) {
                const uint32_t *fi = d->faces + 3 * (size_t)(sh->face_offset + f);
                if (tri_intersect(mesh_vertex(d, sh, fi[0]), mesh_vertex(d, sh, fi[1]),
                                  mesh_vertex(d, sh, fi[2]), r, &t, &u, &v))
                    return 1;
            }
        }
    }
    return 0;
}

int oracle_trace_closest(const mh_scene_desc *desc, uint64_t n, const float *rays, float *t,
                         float *u, float *v, uint32_t *prim, uint32_t *shape) {
    scene_view sv;
    if (scene_view_init(&sv, desc)) return 1;
    for (uint64_t i = 0; i < n; ++i) {
        ray3 r = {V3(rays[i], rays[n + i], rays[2 * n + i]),
                  V3(rays[3 * n + i], rays[4 * n + i], rays[5 * n + i]), rays[6 * n + i]};
        pi_rec pi;
        trace_closest(&sv, &r, &pi);
        /* the OptiX payload: prim_index 0 for rectangles and misses
         * (rectangle.cuh:42, scene_optix.inl:602-606), prim_uv 0 on a miss */
        const int hit = pi.shape != MH_INVALID;
        t[i] = pi.t; u[i] = hit ? pi.u : 0.f; v[i] = hit ? pi.v : 0.f;
        prim[i] = hit && pi.prim != MH_INVALID ? pi.prim : 0u;
        shape[i] = pi.shape;
    }
    scene_view_free(&sv);
    return 0;
}

int oracle_trace_shadow(const mh_scene_desc *desc, uint64_t n, const float *rays,
                        uint32_t *occluded) {
    scene_view sv;
    if (scene_view_init(&sv, desc)) return 1;
    for (uint64_t i = 0; i < n; ++i) {
        ray3 r = {V3(rays[i], rays[n + i], rays[2 * n + i]),
                  V3(rays[3 * n + i], rays[4 * n + i], rays[5 * n + i]), rays[6 * n + i]};
        occluded[i] = (uint32_t)trace_shadow(&sv, &r);
    }
    scene_view_free(&sv);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* SurfaceInteraction                                                       */
/* ------------------------------------------------------------------------ */
typedef struct {
    int valid;
    float t;
    v3 p, n;             /* geometric */
    v3 sh_s, sh_t, sh_n; /* shading frame */
    v3 dp_du;
    float uvx, uvy;
    v3 wi;               /* local */
    uint32_t shape, prim;
} surf_int;

/* coordinate_system (include/mitsuba/core/vector.h:116-136) */
static inline void coordinate_system(v3 n, v3 *s, v3 *t) {
    float sign = signf_(n.z), a = -rcpf_(sign + n.z), b = n.x * n.y * a;
    *s = V3(mulsign(n.x * n.x * a, n.z) + 1.f, mulsign(b, n.z), mulsign_neg(n.x, n.z));
    *t = V3(b, fmaf(n.y, n.y * a, sign), -n.y);
}

static inline v3 to_local(const surf_int *si, v3 v) {
    return V3(vdot(v, si->sh_s), vdot(v, si->sh_t), vdot(v, si->sh_n));
}
/* Frame3f::to_world (include/mitsuba/core/frame.h:40-43) */
static inline v3 to_world(const surf_int *si, v3 v) {
    return vfma_s(si->sh_n, v.z, vfma_s(si->sh_t, v.y, vscale(si->sh_s, v.x)));
}

/* PreliminaryIntersection::compute_surface_interaction (interaction.h:731-757)
   + Rectangle / Mesh::compute_surface_interaction (ad variant branch)
   + finalize_surface_interaction (interaction.h:464-484)                  */
static void compute_si(const mh_scene_desc *d, const ray3 *r, const pi_rec *pi, surf_int *si) {
    memset(si, 0, sizeof(*si));
    si->shape = pi->shape;
    si->prim = pi->prim;
    if (pi->shape == MH_INVALID || !(pi->t != INFINITY)) {
        si->valid = 0;
        si->t = INFINITY;
        si->wi = vneg(r->d); /* world-space -d for invalid lanes */
        return;
    }
    si->valid = 1;
    si->t = pi->t;
    const mh_shape *sh = &d->shapes[pi->shape];
    if (sh->type == MH_SHAPE_RECTANGLE) {
        /* rectangle.cpp:497-567 (IsDiff branch: p = ray(t)) */
        si->p = vfma_s(r->d, pi->t, r->o);
        si->n = vload(sh->frame_n);
        si->sh_n = si->n;
        si->dp_du = vload(sh->frame_s);
        si->uvx = fmaf(pi->u, 0.5f, 0.5f);
        si->uvy = fmaf(pi->v, 0.5f, 0.5f);
    } else {
        /* mesh.cpp:1368-1536 */
        const uint32_t *fi = d->faces + 3 * (size_t)(sh->face_offset + pi->prim);
        v3 p0 = mesh_vertex(d, sh, fi[0]), p1 = mesh_vertex(d, sh, fi[1]),
           p2 = mesh_vertex(d, sh, fi[2]);
        float b1 = pi->u, b2 = pi->v, b0 = 1.f - b1 - b2;
        si->p = vfma_s(p0, b0, vfma_s(p1, b1, vscale(p2, b2)));
        si->n = vnormalize(vcross(vsub(p1, p0), vsub(p2, p0)));
        si->uvx = b1;
        si->uvy = b2;
        v3 dpdv;
        coordinate_system(si->n, &si->dp_du, &dpdv);
        v3 dp0 = vsub(p1, p0), dp1 = vsub(p2, p0);
        if (sh->has_texcoords) {
            const float *tc = d->texcoords;
            size_t o = sh->vertex_offset;
            float u0x = tc[2 * (o + fi[0])], u0y = tc[2 * (o + fi[0]) + 1];
            float u1x = tc[2 * (o + fi[1])], u1y = tc[2 * (o + fi[1]) + 1];
            float u2x = tc[2 * (o + fi[2])], u2y = tc[2 * (o + fi[2]) + 1];
            si->uvx = fmaf(u2x, b2, fmaf(u1x, b1, u0x * b0));
            si->uvy = fmaf(u2y, b2, fmaf(u1y, b1, u0y * b0));
            float d0x = u1x - u0x, d0y = u1y - u0y, d1x = u2x - u0x, d1y = u2y - u0y;
            float det = fmaf(d0x, d1y, -(d0y * d1x)), inv_det = rcpf_(det);
            if (det != 0.f) {
                si->dp_du = vscale(V3(fmaf(d1y, dp0.x, -(d0y * dp1.x)),
                                      fmaf(d1y, dp0.y, -(d0y * dp1.y)),
                                      fmaf(d1y, dp0.z, -(d0y * dp1.z))),
                                   inv_det);
            }
        }
        if (sh->has_normals) {
            const float *nn = d->normals;
            size_t o = sh->vertex_offset;
            v3 n0 = vload(nn + 3 * (o + fi[0])), n1 = vload(nn + 3 * (o + fi[1])),
               n2 = vload(nn + 3 * (o + fi[2]));
            v3 n = vfma_s(n2, b2, vfma_s(n1, b1, vscale(n0, b0)));
            float il = rsqrtf_(vdot(n, n));
            si->sh_n = vscale(n, il);
        } else {
            si->sh_n = si->n;
        }
    }
    /* initialize_sh_frame (interaction.h:245-255) */
    si->sh_s = vnormalize(vfma_s(si->sh_n, -vdot(si->sh_n, si->dp_du), si->dp_du));
    if (si->dp_du.x == 0.f && si->dp_du.y == 0.f && si->dp_du.z == 0.f) {
        v3 tt;
        coordinate_system(si->sh_n, &si->sh_s, &tt);
    }
    si->sh_t = vcross(si->sh_n, si->sh_s);
    si->wi = to_local(si, vneg(r->d));
}

/* Interaction::offset_p (interaction.h:158-162) */
static inline v3 offset_p(v3 p, v3 n, v3 d) {
    float mag = (1.f + vmax(V3(fabsf(p.x), fabsf(p.y), fabsf(p.z)))) * RAY_EPS;
    mag = mulsign(mag, vdot(n, d));
    return vfma_s(n, mag, p);
}
/* Interaction::spawn_ray (interaction.h:133-136) */
static inline ray3 spawn_ray(v3 p, v3 n, v3 d) {
    ray3 r = {offset_p(p, n, d), d, FLT_MAX};
    return r;
}
/* Interaction::spawn_ray_to (interaction.h:138-145) */
static inline ray3 spawn_ray_to(v3 p, v3 n, v3 target) {
    v3 o = offset_p(p, n, vsub(target, p));
    v3 d = vsub(target, o);
    float dist = vnorm(d);
    d = vdivs(d, dist);
    ray3 r = {o, d, dist * (1.f - SHADOW_EPS)};
    return r;
}

/* ------------------------------------------------------------------------ */
/* Textures / BSDF / emitters                                               */
/* ------------------------------------------------------------------------ */
static inline int32_t wrap_index(int32_t i, int32_t res, uint32_t mode) {
    if (mode == 2) return i < 0 ? 0 : (i >= res ? res - 1 : i);   /* clamp */
    if (mode == 1) {                                               /* mirror */
        int32_t p = 2 * res;
        int32_t m = i % p;
        if (m < 0) m += p;
        return m < res ? m : p - 1 - m;
    }
    int32_t m = i % res;                                           /* repeat */
    if (m < 0) m += res;
    return m;
}

/* bitmap texture taps: [drjit] Texture2f::eval_nonaccel (bilinear / nearest)
   at uv' = to_uv.transform_affine(si.uv) (src/textures/bitmap.cpp:696-710)  */
typedef struct {
    int n;             /* 1 (nearest) or 4 (bilinear) */
    uint64_t idx[4];   /* float offset of channel 0: 00, 10, 01, 11 */
    float w0x, w1x, w0y, w1y;
} tex_taps;

static void bitmap_taps(const mh_texture *tx, float uvx, float uvy, tex_taps *tp) {
    const float *m = tx->to_uv;
    float ux = fmaf(m[1], uvy, fmaf(m[0], uvx, m[2]));
    float uy = fmaf(m[4], uvy, fmaf(m[3], uvx, m[5]));
    int32_t W = (int32_t)tx->width, H = (int32_t)tx->height;
    uint32_t C = tx->channels;
    if (tx->filter == 0) {
        int32_t ix = wrap_index((int32_t)floorf(ux * (float)W), W, tx->wrap);
        int32_t iy = wrap_index((int32_t)floorf(uy * (float)H), H, tx->wrap);
        tp->n = 1;
        tp->idx[0] = tx->data_offset + ((uint64_t)iy * W + ix) * C;
        tp->w0x = tp->w0y = 1.f;
        tp->w1x = tp->w1y = 0.f;
        return;
    }
    float fx = fmaf(ux, (float)W, -0.5f), fy = fmaf(uy, (float)H, -0.5f);
    float flx = floorf(fx), fly = floorf(fy);
    int32_t ix = (int32_t)flx, iy = (int32_t)fly;
    tp->w1x = fx - flx;
    tp->w1y = fy - fly;
    tp->w0x = 1.f - tp->w1x;
    tp->w0y = 1.f - tp->w1y;
    int32_t x0 = wrap_index(ix, W, tx->wrap), x1 = wrap_index(ix + 1, W, tx->wrap);
    int32_t y0 = wrap_index(iy, H, tx->wrap), y1 = wrap_index(iy + 1, H, tx->wrap);
    tp->n = 4;
    tp->idx[0] = tx->data_offset + ((uint64_t)y0 * W + x0) * C;
    tp->idx[1] = tx->data_offset + ((uint64_t)y0 * W + x1) * C;
    tp->idx[2] = tx->data_offset + ((uint64_t)y1 * W + x0) * C;
    tp->idx[3] = tx->data_offset + ((uint64_t)y1 * W + x1) * C;
}

static v3 tex_eval(const mh_scene_desc *d, uint32_t tex, float uvx, float uvy) {
    const mh_texture *tx = &d->textures[tex];
    if (tx->type == MH_TEX_RGB) return vload(tx->value);
    tex_taps tp;
    bitmap_taps(tx, uvx, uvy, &tp);
    float out[3];
    for (int c = 0; c < 3; ++c) {
        uint32_t cc = tx->channels == 3 ? (uint32_t)c : 0u;
        if (tp.n == 1) {
            out[c] = d->texels[tp.idx[0] + cc];
        } else {
            float f00 = d->texels[tp.idx[0] + cc], f10 = d->texels[tp.idx[1] + cc],
                  f01 = d->texels[tp.idx[2] + cc], f11 = d->texels[tp.idx[3] + cc];
            out[c] = fmaf(tp.w0y, fmaf(tp.w0x, f00, tp.w1x * f10),
                          tp.w1y * fmaf(tp.w0x, f01, tp.w1x * f11));
        }
    }
    return V3(out[0], out[1], out[2]);
}

/* Gradient sink: d(loss)/d(texture parameter) accumulators (double) */
typedef struct {
    uint32_t n_params;
    const uint32_t *tex;
    double **acc;
    /* forward mode (render_forward, common.py:696-826): tan[k] is the input
       tangent of parameter k, and every sink adds <adj, tangent> to fsum
       instead of scattering adj -- with dL = e_c that is the tangent of
       L_c (prb.py:244-248 `δL += dr.forward_to(Lo)`) */
    const float *const *tan;
    double fsum;
} grad_sink;

/* adjoint of tex_eval: scatter adj (= d loss / d rho) into the texels */
static void tex_backward(const mh_scene_desc *d, uint32_t tex, float uvx, float uvy, v3 adj,
                         grad_sink *g) {
    for (uint32_t k = 0; k < g->n_params; ++k) {
        if (g->tex[k] != tex) continue;
        const mh_texture *tx = &d->textures[tex];
        if (g->tan) {  /* tangent of tex_eval at uv: the same taps over the tangent texels */
            const float *t = g->tan[k];
            if (tx->type == MH_TEX_RGB) {
                g->fsum += (double)adj.x * t[0] + (double)adj.y * t[1] + (double)adj.z * t[2];
                continue;
            }
            tex_taps tp;
            bitmap_taps(tx, uvx, uvy, &tp);
            float av[3] = {adj.x, adj.y, adj.z};
            for (int c = 0; c < 3; ++c) {
                uint32_t cc = tx->channels == 3 ? (uint32_t)c : 0u;
                double tv;
                if (tp.n == 1) {
                    tv = t[tp.idx[0] - tx->data_offset + cc];
                } else {
                    double w[4] = {(double)tp.w0y * tp.w0x, (double)tp.w0y * tp.w1x, (double)tp.w1y * tp.w0x,
                                   (double)tp.w1y * tp.w1x};
                    tv = 0.0;
                    for (int j = 0; j < 4; ++j) tv += w[j] * t[tp.idx[j] - tx->data_offset + cc];
                }
                g->fsum += (double)av[c] * tv;
            }
            continue;
        }
        double *a = g->acc[k];
        if (tx->type == MH_TEX_RGB) {
            a[0] += adj.x; a[1] += adj.y; a[2] += adj.z;
            continue;
        }
        tex_taps tp;
        bitmap_taps(tx, uvx, uvy, &tp);
        float av[3] = {adj.x, adj.y, adj.z};
        float w[4];
        if (tp.n == 1) {
            w[0] = 1.f;
        } else {
            w[0] = tp.w0y * tp.w0x; w[1] = tp.w0y * tp.w1x;
            w[2] = tp.w1y * tp.w0x; w[3] = tp.w1y * tp.w1x;
        }
        for (int j = 0; j < tp.n; ++j) {
            uint64_t base = tp.idx[j] - tx->data_offset;
            if (tx->channels == 3) {
                for (int c = 0; c < 3; ++c) a[base + c] += (double)av[c] * (double)w[j];
            } else {
                a[base] += ((double)av[0] + av[1] + av[2]) * (double)w[j];
            }
        }
    }
}

static inline uint32_t si_bsdf(const mh_scene_desc *d, const surf_int *si) {
    return si->valid ? d->shapes[si->shape].bsdf : MH_INVALID;
}
static inline uint32_t si_emitter(const mh_scene_desc *d, const surf_int *si) {
    return si->valid ? d->shapes[si->shape].emitter : d->environment;
}

/* SmoothDiffuse::eval_pdf (src/bsdfs/diffuse.cpp:160-180) */
static inline void diffuse_eval_pdf(v3 rho, v3 wi, v3 wo, int active, v3 *val, float *pdf) {
    float ci = wi.z, co = wo.z;
    active = active && ci > 0.f && co > 0.f;
    if (active) {
        *val = vscale(vscale(rho, INV_PI_F), co);
        *pdf = INV_PI_F * co;
    } else {
        *val = V3(0, 0, 0);
        *pdf = 0.f;
    }
}

/* warp.h:54-90 square_to_uniform_disk_concentric + warp.h:412-428 */
void oracle_square_to_cosine_hemisphere(const float s[2], float out[3]) {
    float x = fmaf(2.f, s[0], -1.f), y = fmaf(2.f, s[1], -1.f);
    int is_zero = x == 0.f && y == 0.f, q13 = fabsf(x) < fabsf(y);
    float r = q13 ? y : x, rp = q13 ? x : y;
    float phi = ((0.25f * PI_F) * rp) / r;
    if (q13) phi = (0.5f * PI_F) - phi;
    if (is_zero) phi = 0.f;
    float sn, cs;
    oracle_sincos(phi, &sn, &cs);
    float px = r * cs, py = r * sn;
    float z = safe_sqrtf(1.f - fmaf(py, py, px * px));
    out[0] = px; out[1] = py; out[2] = z;
}

typedef struct {
    v3 wo;
    float pdf, eta;
    int sampled_delta, sampled_null;
} bsdf_sample;

/* SmoothDiffuse::sample (diffuse.cpp:101-125): weight = rho, masked */
static inline void diffuse_sample(v3 rho, v3 wi, float s2x, float s2y, int active,
                                  bsdf_sample *bs, v3 *weight) {
    float s[2] = {s2x, s2y}, w[3];
    oracle_square_to_cosine_hemisphere(s, w);
    bs->wo = V3(w[0], w[1], w[2]);
    bs->pdf = INV_PI_F * w[2];
    bs->eta = 1.f;
    bs->sampled_delta = 0;
    bs->sampled_null = 0;
    active = active && wi.z > 0.f;
    *weight = (active && bs->pdf > 0.f) ? rho : V3(0, 0, 0);
}

void oracle_diffuse_eval_pdf(const float wi[3], const float wo[3], const float rho[3],
                             float value[3], float *pdf) {
    v3 v;
    diffuse_eval_pdf(vload(rho), vload(wi), vload(wo), 1, &v, pdf);
    value[0] = v.x; value[1] = v.y; value[2] = v.z;
}

/* mis_weight (path.cpp:300-305, common.py:1817-1825) */
static inline float mis_weight(float a, float b) {
    a = a * a;
    b = b * b;
    float w = a / (a + b);
    return isfinitef_(w) ? w : 0.f;
}

typedef struct {
    v3 p, n, d;
    float dist, pdf;
    int delta;
} dir_sample;

/* AreaLight::pdf_direction (area.cpp:170-200) + Shape::pdf_direction (shape.cpp:377-388) */
static float area_pdf_direction(const mh_scene_desc *d, uint32_t em, const dir_sample *ds) {
    const mh_emitter *e = &d->emitters[em];
    if (e->type != MH_EMITTER_AREA) return 0.f;
    float dp = vdot(ds->d, ds->n);
    int active = dp < 0.f;
    const mh_shape *sh = &d->shapes[e->shape];
    float pdf = sh->inv_area, adp = fabsf(dp);
    pdf *= (adp != 0.f) ? (ds->dist * ds->dist) / adp : 0.f;
    return active ? pdf : 0.f;
}

/* AreaLight::sample_direction (area.cpp:118-168) -> Shape::sample_direction
   (shape.cpp:358-375) -> Rectangle::sample_position (rectangle.cpp:166-180).
   Returns the (masked) spectral weight radiance / pdf.                      */
static v3 area_sample_direction(const mh_scene_desc *d, uint32_t em, v3 ref_p, float sx,
                                float sy, dir_sample *ds) {
    const mh_emitter *e = &d->emitters[em];
    const mh_shape *sh = &d->shapes[e->shape];
    ds->p = xf_point(sh->to_world, V3(sx * 2.f - 1.f, sy * 2.f - 1.f, 0.f));
    ds->n = vload(sh->frame_n);
    ds->pdf = sh->inv_area;
    ds->delta = 0;
    ds->d = vsub(ds->p, ref_p);
    float dist2 = vdot(ds->d, ds->d);
    ds->dist = sqrtf(dist2);
    ds->d = vdivs(ds->d, ds->dist);
    float dp = fabsf(vdot(ds->d, ds->n));
    float x = dist2 / dp;
    ds->pdf *= isfinitef_(x) ? x : 0.f;
    int active = vdot(ds->d, ds->n) < 0.f && ds->pdf != 0.f;
    if (!active) return V3(0, 0, 0);
    return vdivs(vload(e->radiance), ds->pdf);
}

/* defined with the volpath plugins below */
static v3 scene_sample_emitter_direction(const mh_scene_desc *d, v3 ref_p, float sx, float sy,
                                         dir_sample *ds);
static v3 emitter_eval(const mh_scene_desc *d, uint32_t em, const surf_int *si);
static float emitter_pdf_direction(const mh_scene_desc *d, uint32_t em, const surf_int *si, v3 ref_p);

/* Scene::sample_emitter_direction (scene.cpp:299-353), test_visibility =
   true.  A shadow ray whose contribution is exactly zero (back-facing light
   sample) is skipped: it cannot change the result.                        */
static v3 sample_emitter_direction(const scene_view *sv, const surf_int *si, float sx, float sy,
                                   dir_sample *ds, uint64_t *n_shadow) {
    const mh_scene_desc *d = sv->d;
    v3 spec = scene_sample_emitter_direction(d, si->p, sx, sy, ds);
    if (ds->pdf != 0.f && (spec.x != 0.f || spec.y != 0.f || spec.z != 0.f)) {
        ray3 r = spawn_ray_to(si->p, si->n, ds->p);
        if (n_shadow) (*n_shadow)++;
        if (trace_shadow(sv, &r)) {
            spec = V3(0, 0, 0);
            ds->pdf = 0.f;
        }
    }
    return spec;
}

/* ------------------------------------------------------------------------ */
/* Camera: PerspectiveCamera::sample_ray_differential (perspective.cpp:240-281) */
/* ------------------------------------------------------------------------ */
static ray3 camera_ray(const mh_sensor *s, float ax, float ay) {
    v3 near_p = xf4_point_proj(s->sample_to_camera, V3(ax + 0.f, ay + 0.f, 0.f));
    v3 d = vnormalize(near_p);
    ray3 r;
    r.o = V3(s->to_world[3], s->to_world[7], s->to_world[11]);
    r.d = xf4_vector(s->to_world, d);
    float inv_z = rcpf_(d.z);
    float near_t = s->near_clip * inv_z, far_t = s->far_clip * inv_z;
    r.o = vadd(r.o, vscale(r.d, near_t));
    r.maxt = far_t - near_t;
    return r;
}

int oracle_camera_ray(const mh_scene_desc *desc, const float pos[2], float o[3], float d[3],
                      float *maxt) {
    ray3 r = camera_ray(&desc->sensor, pos[0], pos[1]);
    o[0] = r.o.x; o[1] = r.o.y; o[2] = r.o.z;
    d[0] = r.d.x; d[1] = r.d.y; d[2] = r.d.z;
    *maxt = r.maxt;
    return 0;
}

/* Emitter-hit MIS record: DirectionSample3f(scene, si, prev_si) (records.h:173-180) */
static inline float emitter_hit_pdf(const mh_scene_desc *d, uint32_t em, const surf_int *si,
                                    v3 prev_p) {
    dir_sample ds;
    ds.p = si->p;
    ds.n = si->sh_n;
    v3 rel = vsub(si->p, prev_p);
    ds.dist = vnorm(rel);
    ds.d = si->valid ? vdivs(rel, ds.dist) : vneg(si->wi);
    ds.pdf = 0.f;
    ds.delta = 0;
    /* Scene::pdf_emitter_direction (scene.cpp:355-366): uniform pmf */
    return area_pdf_direction(d, em, &ds) * (1.f / (float)d->n_emitters);
}

/* ------------------------------------------------------------------------ */
/* PathIntegrator::sample, JIT semantics (src/integrators/path.cpp:95-287)  */
/* counters: [0] closest rays, [1] shadow rays, [2] lane-bounces            */
/* ------------------------------------------------------------------------ */
/* scalar != 0: the scalar_rgb control flow (config 1): dr::none_or<false>
   breaks the loop before the emitter / BSDF / RR draws when the path cannot
   continue (path.cpp:179-180), and dr::any_or<true> skips the emitter draw
   when emitter sampling is inactive (path.cpp:193-196); in JIT both are
   taken (every lane active at the loop head draws 6 floats) */
static v3 path_sample_mode(const scene_view *sv, const mh_integrator *in, pcg32 *rng, ray3 ray,
                           int *valid_out, uint64_t *counters, int scalar);
static v3 path_sample(const scene_view *sv, const mh_integrator *in, pcg32 *rng, ray3 ray,
                      int *valid_out, uint64_t *counters) {
    return path_sample_mode(sv, in, rng, ray, valid_out, counters, 0);
}
static v3 path_sample_mode(const scene_view *sv, const mh_integrator *in, pcg32 *rng, ray3 ray,
                           int *valid_out, uint64_t *counters, int scalar) {
    const mh_scene_desc *d = sv->d;
    if (in->max_depth == 0) { *valid_out = 0; return V3(0, 0, 0); }
    v3 throughput = V3(1, 1, 1), result = V3(0, 0, 0);
    float eta = 1.f;
    uint32_t depth = 0;
    int valid_ray = !in->hide_emitters && d->environment != MH_INVALID;
    v3 prev_p = V3(0, 0, 0);
    float prev_bsdf_pdf = 1.f;
    int prev_bsdf_delta = 1;
    int active = 1;
    while (active) {
        pi_rec pi;
        trace_closest(sv, &ray, &pi);
        if (counters) { counters[0]++; counters[2]++; }
        surf_int si;
        compute_si(d, &ray, &pi, &si);

        /* ---- direct emission (path.cpp:158-174) ---- */
        uint32_t em = si_emitter(d, &si);
        if (em != MH_INVALID) {
            float em_pdf = prev_bsdf_delta ? 0.f : emitter_pdf_direction(d, em, &si, prev_p);
            float mis_bsdf = mis_weight(prev_bsdf_pdf, em_pdf);
            v3 le = V3(0, 0, 0);
            if (prev_bsdf_pdf > 0.f) le = emitter_eval(d, em, &si);
            result = vfma(throughput, vscale(le, mis_bsdf), result);
        }

        int active_next = (depth + 1 < in->max_depth) && si.valid;
        if (scalar && !active_next) break; /* path.cpp:179-180 (scalar early exit) */
        uint32_t b = si_bsdf(d, &si);
        int smooth = b != MH_INVALID && d->bsdfs[b].type == MH_BSDF_DIFFUSE;
        int active_em = active_next && smooth;

        /* ---- emitter sampling (path.cpp:187-208) ---- */
        float e0 = 0.f, e1 = 0.f;
        if (!scalar || active_em) { e0 = pcg_float(rng); e1 = pcg_float(rng); }
        dir_sample ds;
        memset(&ds, 0, sizeof(ds));
        v3 em_weight = V3(0, 0, 0), wo = V3(0, 0, 0);
        if (active_em) {
            em_weight = sample_emitter_direction(sv, &si, e0, e1, &ds,
                                                 counters ? &counters[1] : NULL);
            active_em = ds.pdf != 0.f;
            wo = to_local(&si, ds.d);
        }

        /* ---- BSDF eval + sample (path.cpp:212-216) ---- */
        float s1 = pcg_float(rng);
        float s2x = pcg_float(rng), s2y = pcg_float(rng);
        (void)s1;
        v3 bsdf_val = V3(0, 0, 0), bsdf_weight = V3(0, 0, 0);
        float bsdf_pdf = 0.f;
        bsdf_sample bs;
        memset(&bs, 0, sizeof(bs));
        if (smooth) {
            v3 rho = tex_eval(d, d->bsdfs[b].reflectance, si.uvx, si.uvy);
            diffuse_eval_pdf(rho, si.wi, wo, 1, &bsdf_val, &bsdf_pdf);
            diffuse_sample(rho, si.wi, s2x, s2y, 1, &bs, &bsdf_weight);
        }

        /* ---- emitter sampling contribution (path.cpp:220-230) ---- */
        if (active_em) {
            float mis_em = ds.delta ? 1.f : mis_weight(ds.pdf, bsdf_pdf);
            result = vfma(throughput, vscale(vmul(bsdf_val, em_weight), mis_em), result);
        }

        /* ---- BSDF sampling, state update (path.cpp:234-262) ---- */
        ray = spawn_ray(si.p, si.n, to_world(&si, bs.wo));
        throughput = vmul(throughput, bsdf_weight);
        eta *= bs.eta;
        valid_ray = valid_ray || (si.valid && !bs.sampled_null);
        prev_p = si.p;
        prev_bsdf_pdf = bs.pdf;
        prev_bsdf_delta = bs.sampled_delta;

        /* ---- stopping criterion (path.cpp:266-280) ---- */
        if (si.valid) depth += 1;
        float tmax = vmax(throughput);
        float rr_prob = fminf(tmax * (eta * eta), 0.95f);
        int rr_active = depth >= in->rr_depth;
        int rr_continue = pcg_float(rng) < rr_prob;
        if (rr_active) throughput = vscale(throughput, rcpf_(rr_prob));
        active = active_next && (!rr_active || rr_continue) && tmax != 0.f;
    }
    *valid_out = valid_ray;
    return valid_ray ? result : V3(0, 0, 0);
}

/* ------------------------------------------------------------------------ */
/* PRBIntegrator.sample (src/python/python/ad/integrators/prb.py:59-257)    */
/* primal: grad == NULL; adjoint: grad != NULL, L_in = primal radiance      */
/* ------------------------------------------------------------------------ */
static v3 prb_sample(const scene_view *sv, const mh_integrator *in, pcg32 *rng, ray3 ray,
                     v3 dL, v3 L_in, grad_sink *grad, int *valid_out) {
    const mh_scene_desc *d = sv->d;
    const int primal = grad == NULL;
    uint32_t depth = 0;
    v3 L = primal ? V3(0, 0, 0) : L_in;
    v3 beta = V3(1, 1, 1);
    float eta = 1.f;
    int active = 1;
    v3 prev_p = V3(0, 0, 0);
    float prev_bsdf_pdf = 1.f;
    int prev_bsdf_delta = 1;
    while (active) {
        int active_next = active;
        pi_rec pi;
        trace_closest(sv, &ray, &pi);
        surf_int si;
        compute_si(d, &ray, &pi, &si);
        uint32_t b = si_bsdf(d, &si);
        int smooth = b != MH_INVALID && d->bsdfs[b].type == MH_BSDF_DIFFUSE;

        if (in->hide_emitters && depth == 0 && !si.valid) active_next = 0;

        /* ---- direct emission (prb.py:121-135) ---- */
        uint32_t em = si_emitter(d, &si);
        v3 Le = V3(0, 0, 0);
        if (em != MH_INVALID) {
            float em_pdf = prev_bsdf_delta ? 0.f : emitter_pdf_direction(d, em, &si, prev_p);
            float mis = mis_weight(prev_bsdf_pdf, em_pdf);
            v3 le = V3(0, 0, 0);
            if (active_next) le = emitter_eval(d, em, &si);
            Le = vmul(vscale(beta, mis), le);
        }

        /* ---- emitter sampling (prb.py:139-163) ---- */
        active_next = active_next && (depth + 1 < in->max_depth) && si.valid;
        int active_em = active_next && smooth;
        float e0 = pcg_float(rng), e1 = pcg_float(rng);
        dir_sample ds;
        memset(&ds, 0, sizeof(ds));
        v3 em_weight = V3(0, 0, 0);
        if (active_em) {
            em_weight = sample_emitter_direction(sv, &si, e0, e1, &ds, NULL);
            active_em = ds.pdf != 0.f;
        }
        v3 rho = V3(0, 0, 0);
        if (smooth) rho = tex_eval(d, d->bsdfs[b].reflectance, si.uvx, si.uvy);
        v3 wo_em = to_local(&si, ds.d);
        v3 bsdf_value_em = V3(0, 0, 0);
        float bsdf_pdf_em = 0.f;
        diffuse_eval_pdf(rho, si.wi, wo_em, active_em, &bsdf_value_em, &bsdf_pdf_em);
        float mis_em = ds.delta ? 1.f : mis_weight(ds.pdf, bsdf_pdf_em);
        v3 beta_mis_em = vscale(beta, mis_em);
        v3 Lr_dir = V3(0, 0, 0);
        if (active_em) Lr_dir = vmul(vmul(beta_mis_em, bsdf_value_em), em_weight);

        /* ---- detached BSDF sampling (prb.py:167-170) ---- */
        float s1 = pcg_float(rng);
        float s2x = pcg_float(rng), s2y = pcg_float(rng);
        (void)s1;
        bsdf_sample bs;
        memset(&bs, 0, sizeof(bs));
        v3 bsdf_weight = V3(0, 0, 0);
        if (smooth && active_next) diffuse_sample(rho, si.wi, s2x, s2y, 1, &bs, &bsdf_weight);

        /* ---- state update (prb.py:174-199) ---- */
        L = primal ? vadd(vadd(L, Le), Lr_dir) : vsub(vsub(L, Le), Lr_dir);
        ray = spawn_ray(si.p, si.n, to_world(&si, bs.wo));
        eta *= bs.eta;
        beta = vmul(beta, bsdf_weight);
        prev_p = si.p;
        prev_bsdf_pdf = bs.pdf;
        prev_bsdf_delta = bs.sampled_delta;
        float beta_max = vmax(beta);
        active_next = active_next && beta_max != 0.f;
        float rr_prob = fminf(beta_max * (eta * eta), 0.95f);
        int rr_active = depth >= in->rr_depth;
        if (rr_active) beta = vscale(beta, rcpf_(rr_prob));
        int rr_continue = pcg_float(rng) < rr_prob;
        active_next = active_next && (!rr_active || rr_continue);

        /* ---- differential phase (prb.py:203-248) wrt the diffuse reflectance:
           Lr_dir = ((beta*mis_em) * (rho/pi*cos_em)) * em_weight
           Lr_ind = L * replace_grad(1, inv_det * (rho/pi*cos_ind))
           adj(rho) = [(dL*em_weight)*(beta*mis_em)*cos_em]/pi
                    + [((dL*L)*inv_det)*cos_ind]/pi                         */
        if (!primal && smooth) {
            v3 adj = V3(0, 0, 0);
            if (active_em && si.wi.z > 0.f && wo_em.z > 0.f)
                adj = vscale(vscale(vmul(vmul(dL, em_weight), beta_mis_em), wo_em.z), INV_PI_F);
            v3 wo2 = to_local(&si, ray.d);
            if (active_next && si.wi.z > 0.f && wo2.z > 0.f) {
                v3 det = vscale(bsdf_weight, bs.pdf);
                v3 inv = V3(det.x != 0.f ? rcpf_(det.x) : 0.f, det.y != 0.f ? rcpf_(det.y) : 0.f,
                            det.z != 0.f ? rcpf_(det.z) : 0.f);
                v3 a2 = vscale(vscale(vmul(vmul(dL, L), inv), wo2.z), INV_PI_F);
                adj = vadd(adj, a2);
            }
            tex_backward(d, d->bsdfs[b].reflectance, si.uvx, si.uvy, adj, grad);
        }

        if (si.valid) depth += 1;
        active = active_next;
    }
    *valid_out = depth != 0;
    return primal ? L : dL;
}

/* ------------------------------------------------------------------------ */
/* Wavefront driver (integrator.cpp:276-390 / common.py:447-525)            */
/* ------------------------------------------------------------------------ */
typedef struct {
    uint32_t W, H, spp, spp_pp, n_passes, log_spp; /* log_spp = 32 if not pow2 */
} wf_layout;

/* ad: ADIntegrator.prepare's single wavefront of <= 2^32 samples
 * (common.py:571-578; prb / prbvolpath primal, W image, render_backward);
 * otherwise SamplingIntegrator::render's passes (integrator.cpp:281-295).
 * Returns nonzero when an ad wavefront exceeds 2^32. */
static int wf_init(const mh_sensor *s, uint32_t spp, wf_layout *L, int ad) {
    L->W = s->width;
    L->H = s->height;
    L->spp = spp;
    uint64_t wf = (uint64_t)L->W * L->H * spp, lim = 0xffffffffull;
    L->spp_pp = spp;
    L->n_passes = 1;
    if (ad && wf > (1ull << 32)) return 1;
    if (!ad && wf > lim) {
        L->spp_pp = spp / (uint32_t)((wf + lim - 1) / lim);
        L->n_passes = spp / L->spp_pp;
    }
    L->log_spp = 32;
    for (uint32_t k = 0; k < 32; ++k)
        if ((1u << k) == L->spp_pp) L->log_spp = k;
    return 0;
}

/* lane -> pixel (integrator.cpp:323-340) */
static inline void lane_pixel(const wf_layout *L, uint32_t lane, uint32_t *px, uint32_t *py) {
    uint32_t pixel = L->log_spp < 32 ? (lane >> L->log_spp) : (lane / L->spp_pp);
    *py = pixel / L->W;
    *px = pixel - L->W * *py;
}

/* ======================================================================== */
/* volpath (src/integrators/volpath.cpp:95-450) and its plugins             */
/* ======================================================================== */

/* Dr.Jit 0.4.4 math.h `exp` (single precision, non-CUDA branch): Cephes
   range reduction e^x = e^g 2^n, Estrin polynomial, ldexp, over/underflow
   masks.  Restated from the published algorithm (parity unpinned).       */
static inline float estrin6(float x, float c0, float c1, float c2, float c3, float c4, float c5) {
    float a0 = fmaf(x, c1, c0), a1 = fmaf(x, c3, c2), a2 = fmaf(x, c5, c4);
    float x2 = x * x;
    float b0 = fmaf(x2, a1, a0), b1 = a2;
    float x4 = x2 * x2;
    return fmaf(x4, b1, b0);
}
float oracle_exp(float x) {
    const int overflow = x > 88.3762626647949f, underflow = x < -88.3762626647949f;
    float n = floorf(fmaf(1.44269504088896340736f, x, 0.5f));
    x = fmaf(-n, 0.693359375f, x);
    x = fmaf(-n, -2.12194440e-4f, x);
    float z = estrin6(x, 5.0000001201e-1f, 1.6666665459e-1f, 4.1665795894e-2f, 8.3334519073e-3f,
                      1.3981999507e-3f, 1.9875691500e-4f);
    z = fmaf(z, x * x, x + 1.0f);
    /* ldexp_finite: multiply by 2^n built from the exponent field */
    int32_t ni = (int32_t)n;
    z = z * u2f((uint32_t)(ni + 127) << 23);
    if (overflow) z = INFINITY;
    if (underflow) z = 0.f;
    return z;
}

/* warp::square_to_uniform_sphere (core/warp.h:250-255) */
static inline v3 square_to_uniform_sphere(float sx, float sy) {
    float z = fmaf(-2.f, sy, 1.f);
    float r = safe_sqrtf(fmaf(-z, z, 1.f));
    float s, c;
    oracle_sincos((2.f * PI_F) * sx, &s, &c);
    return V3(r * c, r * s, z);
}

/* Emitter::sample_direction for the three emitter plugins of the path:
   area (area.cpp:118-168), constant (constant.cpp:112-140),
   directional (directional.cpp:150-175).                                   */
static v3 emitter_sample_direction(const mh_scene_desc *d, uint32_t em, v3 ref_p, float sx,
                                   float sy, dir_sample *ds) {
    const mh_emitter *e = &d->emitters[em];
    if (e->type == MH_EMITTER_AREA) return area_sample_direction(d, em, ref_p, sx, sy, ds);
    if (e->type == MH_EMITTER_CONSTANT) {
        v3 dd = square_to_uniform_sphere(sx, sy);
        v3 c = vload(e->scene_center);
        float radius = fmaxf(e->scene_radius, vnorm(vsub(ref_p, c))), dist = 2.f * radius;
        ds->p = vfma_s(dd, dist, ref_p);
        ds->n = vneg(dd);
        ds->pdf = INV_4PI_F;
        ds->delta = 0;
        ds->d = dd;
        ds->dist = dist;
        return vdivs(vload(e->radiance), ds->pdf);
    }
    /* directional: ds.p = p - d * inf (NaN where d has a zero component) */
    v3 dd = vload(e->direction);
    float dist = INFINITY;
    ds->p = vsub(ref_p, vscale(dd, dist));
    ds->n = dd;
    ds->pdf = 1.f;
    ds->delta = 1;
    ds->d = vneg(dd);
    ds->dist = dist;
    return vload(e->radiance);
}

/* Scene::sample_emitter_direction without the visibility test
   (scene.cpp:299-353): uniform emitter selection when there are several. */
static v3 scene_sample_emitter_direction(const mh_scene_desc *d, v3 ref_p, float sx, float sy,
                                         dir_sample *ds) {
    memset(ds, 0, sizeof(*ds));
    uint32_t n = d->n_emitters;
    if (n == 0) return V3(0, 0, 0);
    if (n == 1) return emitter_sample_direction(d, 0, ref_p, sx, sy, ds);
    float nf = (float)n, scaled = sx * nf;
    uint32_t idx = (uint32_t)scaled;
    if (idx > n - 1) idx = n - 1;
    float sx_re = scaled - (float)idx;
    v3 spec = emitter_sample_direction(d, idx, ref_p, sx_re, sy, ds);
    ds->pdf *= 1.f / nf;
    return vscale(spec, nf);
}

/* Emitter::eval at a surface hit / escaped ray */
static v3 emitter_eval(const mh_scene_desc *d, uint32_t em, const surf_int *si) {
    const mh_emitter *e = &d->emitters[em];
    if (e->type == MH_EMITTER_AREA) return si->wi.z > 0.f ? vload(e->radiance) : V3(0, 0, 0);
    if (e->type == MH_EMITTER_CONSTANT) return vload(e->radiance);
    return V3(0, 0, 0);
}

/* Scene::pdf_emitter_direction (scene.cpp:355-366) of DirectionSample3f(scene, si, ref) */
static float emitter_pdf_direction(const mh_scene_desc *d, uint32_t em, const surf_int *si,
                                   v3 ref_p) {
    const mh_emitter *e = &d->emitters[em];
    float pmf = 1.f / (float)d->n_emitters;
    if (e->type == MH_EMITTER_AREA) return emitter_hit_pdf(d, em, si, ref_p);
    if (e->type == MH_EMITTER_CONSTANT) return INV_4PI_F * pmf;
    return 0.f;
}

/* ---- media: Medium::sample_interaction (medium.cpp:40-86) ---------------- */
typedef struct {
    int valid;
    float t, mint;
    v3 p;
    v3 sigma_s;
    float sigma_n, sigma_t, maj;
    v3 fs, ft, fn; /* sh_frame = Frame3f(ray.d); wi = (0, 0, -1) local */
} med_int;

/* [drjit] Texture3f::eval_nonaccel, linear filter, clamp wrap, 1 channel
   (grid.cpp:545-558; weight form as grid.cpp:502-516)                      */
static float grid_eval(const mh_scene_desc *d, const mh_medium *m, v3 p) {
    v3 q = xf_point(m->grid_to_local, p);
    const int32_t rx = (int32_t)m->grid_res[0], ry = (int32_t)m->grid_res[1], rz = (int32_t)m->grid_res[2];
    float px = fmaf(q.x, (float)rx, -0.5f), py = fmaf(q.y, (float)ry, -0.5f), pz = fmaf(q.z, (float)rz, -0.5f);
    int32_t ix = (int32_t)floorf(px), iy = (int32_t)floorf(py), iz = (int32_t)floorf(pz);
    float w1x = px - (float)ix, w1y = py - (float)iy, w1z = pz - (float)iz;
    float w0x = 1.f - w1x, w0y = 1.f - w1y, w0z = 1.f - w1z;
#define CL(i, r) ((i) < 0 ? 0 : ((i) > (r) - 1 ? (r) - 1 : (i)))
    int32_t x0 = CL(ix, rx), x1 = CL(ix + 1, rx), y0 = CL(iy, ry), y1 = CL(iy + 1, ry),
            z0 = CL(iz, rz), z1 = CL(iz + 1, rz);
#undef CL
    const float *g = d->grid_data + m->grid_offset;
#define V(x, y, z) g[((size_t)(z) * (size_t)ry + (size_t)(y)) * (size_t)rx + (size_t)(x)]
    float v000 = V(x0, y0, z0), v100 = V(x1, y0, z0), v010 = V(x0, y1, z0), v110 = V(x1, y1, z0);
    float v001 = V(x0, y0, z1), v101 = V(x1, y0, z1), v011 = V(x0, y1, z1), v111 = V(x1, y1, z1);
#undef V
    float f00 = fmaf(w0x, v000, w1x * v100), f01 = fmaf(w0x, v001, w1x * v101),
          f10 = fmaf(w0x, v010, w1x * v110), f11 = fmaf(w0x, v011, w1x * v111);
    float f0 = fmaf(w0y, f00, w1y * f10), f1 = fmaf(w0y, f01, w1y * f11);
    return fmaf(w0z, f0, w1z * f1);
}

/* BoundingBox3f::ray_intersect (core/bbox.h:303-327) */
static int bbox_ray_intersect(const float *mn, const float *mx, const ray3 *r, float *mint, float *maxt) {
    float o[3] = {r->o.x, r->o.y, r->o.z}, dd[3] = {r->d.x, r->d.y, r->d.z};
    int active = 1;
    float t1p[3], t2p[3];
    for (int i = 0; i < 3; ++i) {
        active = active && (dd[i] != 0.f || (o[i] > mn[i] || o[i] < mx[i]));
        float rc = 1.f / dd[i];
        float t1 = (mn[i] - o[i]) * rc, t2 = (mx[i] - o[i]) * rc;
        t1p[i] = fminf(t1, t2);
        t2p[i] = fmaxf(t1, t2);
    }
    *mint = fmaxf(fmaxf(t1p[0], t1p[1]), t1p[2]);
    *maxt = fminf(fminf(t2p[0], t2p[1]), t2p[2]);
    return active && *maxt >= *mint;
}

static inline float medium_majorant(const mh_medium *m) {
    if (m->type == MH_MEDIUM_HOMOGENEOUS) return m->sigma_t_const * m->scale;
    return m->scale * m->max_density;
}

/* density-grid lookups since the last oracle_grid_lookups(1): the check of the
   device's mh_stats.grid_lookups (test infrastructure, like the rest of the oracle) */
static uint64_t g_grid_lookups;
uint64_t oracle_grid_lookups(int reset) {
    return reset ? __atomic_exchange_n(&g_grid_lookups, 0, __ATOMIC_RELAXED)
                 : __atomic_load_n(&g_grid_lookups, __ATOMIC_RELAXED);
}

static void sample_interaction(const mh_scene_desc *d, uint32_t med, const ray3 *ray, float u,
                               uint32_t channel, med_int *mei) {
    const mh_medium *m = &d->media[med];
    (void)channel; /* scalar majorant: index_spectrum picks the same value */
    mei->fn = ray->d;
    coordinate_system(ray->d, &mei->fs, &mei->ft);
    float mint, maxt;
    int active;
    if (m->type == MH_MEDIUM_HOMOGENEOUS) {
        active = 1; mint = 0.f; maxt = INFINITY;            /* homogeneous.cpp:184-187 */
    } else {
        active = bbox_ray_intersect(m->bbox_min, m->bbox_max, ray, &mint, &maxt);
    }
    active = active && (isfinitef_(mint) || isfinitef_(maxt));
    if (!active) { mint = 0.f; maxt = INFINITY; }
    mint = fmaxf(0.f, mint);
    maxt = fminf(ray->maxt, maxt);
    float maj = medium_majorant(m);
    float sampled_t = mint + (-oracle_log(1.f - u) / maj);
    int valid = active && sampled_t <= maxt;
    mei->valid = valid;
    mei->t = valid ? sampled_t : INFINITY;
    mei->p = vfma_s(ray->d, sampled_t, ray->o);
    mei->mint = mint;
    mei->maj = maj;
    /* get_scattering_coefficients (heterogeneous.cpp:188-200 / homogeneous.cpp:166-182) */
    float st = 0.f;
    if (valid) st = m->type == MH_MEDIUM_HOMOGENEOUS ? m->sigma_t_const * m->scale
                                                      : m->scale * grid_eval(d, m, mei->p);
    if (valid && m->type != MH_MEDIUM_HOMOGENEOUS) __atomic_fetch_add(&g_grid_lookups, 1, __ATOMIC_RELAXED);
    mei->sigma_t = st;
    mei->sigma_s = vscale(vload(m->albedo), st);
    if (!valid) mei->sigma_s = V3(0, 0, 0);
    mei->sigma_n = m->type == MH_MEDIUM_HOMOGENEOUS ? 0.f : maj - st;
}

static inline v3 mei_to_local(const med_int *m, v3 v) {
    return V3(vdot(v, m->fs), vdot(v, m->ft), vdot(v, m->fn));
}
static inline v3 mei_to_world(const med_int *m, v3 v) {
    return vfma_s(m->fn, v.z, vfma_s(m->ft, v.y, vscale(m->fs, v.x)));
}

/* HGPhaseFunction (phase/hg.cpp:66-104), IsotropicPhaseFunction (isotropic.cpp) */
static inline float eval_hg(float g, float cos_theta) {
    float temp = (1.f + g * g) + (2.f * g) * cos_theta;
    return (INV_4PI_F * (1.f - g * g)) / (temp * sqrtf(temp));
}
static float phase_eval(const mh_medium *m, v3 wo) {
    if (m->phase == MH_PHASE_HG) return eval_hg(m->g, vdot(wo, V3(0.f, 0.f, -1.f)));
    return INV_4PI_F;
}
static v3 phase_sample(const mh_medium *m, float s2x, float s2y, float *pdf) {
    if (m->phase == MH_PHASE_HG) {
        float g = m->g;
        float sqr_term = (1.f - g * g) / ((1.f - g) + (2.f * g) * s2x);
        float cos_theta = ((1.f + g * g) - sqr_term * sqr_term) / (2.f * g);
        if (fabsf(g) < 5.9604644775390625e-08f) cos_theta = 1.f - 2.f * s2x;
        float sin_theta = safe_sqrtf(1.f - cos_theta * cos_theta);
        float sp, cp;
        oracle_sincos((2.f * PI_F) * s2y, &sp, &cp);
        *pdf = eval_hg(g, -cos_theta);
        return V3(sin_theta * cp, sin_theta * sp, cos_theta);
    }
    *pdf = INV_4PI_F;
    return square_to_uniform_sphere(s2x, s2y);
}

static inline int is_medium_transition(const mh_scene_desc *d, const surf_int *si) {
    if (!si->valid) return 0;
    const mh_shape *sh = &d->shapes[si->shape];
    return sh->interior_medium != sh->exterior_medium;
}
/* SurfaceInteraction::target_medium: dot(d, n) > 0 ? exterior : interior */
static inline uint32_t target_medium(const mh_scene_desc *d, const surf_int *si, v3 dir) {
    const mh_shape *sh = &d->shapes[si->shape];
    return vdot(dir, si->n) > 0.f ? sh->exterior_medium : sh->interior_medium;
}

static inline float index_spectrum(v3 s, uint32_t ch) { return ch == 1 ? s.y : (ch == 2 ? s.z : s.x); }

/* volpath.cpp:333-450: emitter sample + ratio-tracked transmittance.
   ref_n = 0 for medium interactions.  si_ref != NULL for surfaces.        */
static v3 vol_sample_emitter(const scene_view *sv, v3 ref_p, v3 ref_n, const surf_int *si_ref,
                             pcg32 *rng, uint32_t medium, uint32_t channel, dir_sample *ds,
                             uint64_t *counters) {
    const mh_scene_desc *d = sv->d;
    v3 transmittance = V3(1, 1, 1);
    float sx = pcg_float(rng), sy = pcg_float(rng);
    v3 emitter_val = scene_sample_emitter_direction(d, ref_p, sx, sy, ds);
    if (ds->pdf == 0.f) return V3(0, 0, 0);
    ray3 ray = spawn_ray_to(ref_p, ref_n, ds->p);
    float max_dist = ray.maxt;
    if (si_ref && is_medium_transition(d, si_ref)) medium = target_medium(d, si_ref, ray.d);
    float total_dist = 0.f;
    surf_int si;
    memset(&si, 0, sizeof(si));
    si.t = 0.f;
    int needs_intersection = 1, active = 1;
    while (active) {
        float remaining_dist = max_dist - total_dist;
        ray.maxt = remaining_dist;
        active = active && remaining_dist > 0.f;
        if (!active) break;
        int escaped_medium = 0;
        int active_medium = medium != MH_INVALID;
        int active_surface = !active_medium;
        med_int mei;
        memset(&mei, 0, sizeof(mei));
        mei.t = INFINITY;
        if (active_medium) {
            const mh_medium *m = &d->media[medium];
            sample_interaction(d, medium, &ray, pcg_float(rng), channel, &mei);
            if (m->type == MH_MEDIUM_HOMOGENEOUS && mei.valid) ray.maxt = fminf(mei.t, remaining_dist);
            if (needs_intersection) {
                pi_rec pi;
                trace_closest(sv, &ray, &pi);
                if (counters) counters[1]++;
                compute_si(d, &ray, &pi, &si);
            }
            if (si.t < mei.t) { mei.t = INFINITY; mei.valid = 0; }
            needs_intersection = needs_intersection && !si.valid;
            /* has_spectral_extinction (heterogeneous.cpp:161, homogeneous.cpp:143) */
            const int spectral = !(m->flags & MH_MEDIUM_NO_SPECTRAL_EXTINCTION);
            if (spectral) {
                float t = fminf(remaining_dist, fminf(mei.t, si.t)) - mei.mint;
                float tr = oracle_exp((-t) * mei.maj);
                float pdf = (si.t < mei.t || mei.t > remaining_dist) ? tr : tr * mei.maj;
                float f = pdf > 0.f ? tr / pdf : 0.f;
                transmittance = vscale(transmittance, f);
            }
            if (mei.t > remaining_dist && mei.valid) total_dist = ds->dist;
            if (mei.t > remaining_dist) { mei.t = INFINITY; mei.valid = 0; }
            escaped_medium = !mei.valid;
            active_medium = mei.valid;
            if (active_medium) {
                total_dist += mei.t;
                ray.o = mei.p;
                si.t = si.t - mei.t;
                if (spectral) transmittance = vscale(transmittance, mei.sigma_n);
                else transmittance = vscale(transmittance, mei.sigma_n / mei.maj);
            }
        }
        int intersect = active_surface && needs_intersection;
        if (intersect) {
            pi_rec pi;
            trace_closest(sv, &ray, &pi);
            if (counters) counters[1]++;
            compute_si(d, &ray, &pi, &si);
        }
        needs_intersection = needs_intersection && !intersect;
        active_surface = active_surface || escaped_medium;
        if (active_surface) total_dist += si.t;
        active_surface = active_surface && si.valid && !active_medium;
        if (active_surface) {
            uint32_t b = si_bsdf(d, &si);
            /* eval_null_transmission: null -> 1, diffuse -> 0 */
            float tn = (b != MH_INVALID && d->bsdfs[b].type == MH_BSDF_NULL) ? 1.f : 0.f;
            transmittance = vscale(transmittance, tn);
            ray = spawn_ray(si.p, si.n, ray.d);
        }
        ray.maxt = remaining_dist;
        needs_intersection = needs_intersection || active_surface;
        active = (active_medium || active_surface) &&
                 (transmittance.x != 0.f || transmittance.y != 0.f || transmittance.z != 0.f);
        if (active_surface && is_medium_transition(d, &si)) medium = target_medium(d, &si, ray.d);
    }
    return vmul(transmittance, emitter_val);
}

static inline float mis_weight_vol(float a, float b) { return mis_weight(a, b); } /* volpath.cpp:463-468 */

static v3 volpath_sample(const scene_view *sv, const mh_integrator *in, pcg32 *rng, ray3 ray,
                         int *valid_out, uint64_t *counters) {
    const mh_scene_desc *d = sv->d;
    int valid_ray = !in->hide_emitters && d->environment != MH_INVALID;
    float eta = 1.f;
    v3 throughput = V3(1, 1, 1), result = V3(0, 0, 0);
    uint32_t medium = d->sensor.medium;
    int specular_chain = !in->hide_emitters;
    uint32_t depth = 0;
    uint32_t channel = (uint32_t)fminf(pcg_float(rng) * 3.f, 2.f);
    surf_int si;
    memset(&si, 0, sizeof(si));
    int needs_intersection = 1;
    v3 last_p = V3(0, 0, 0);
    float last_pdf = 1.f;
    int active = 1;
    for (;;) {
        /* ---- Russian roulette (volpath.cpp:143-151) ---- */
        active = active && (throughput.x != 0.f || throughput.y != 0.f || throughput.z != 0.f);
        float q = fminf(vmax(throughput) * (eta * eta), 0.95f);
        int perform_rr = depth > in->rr_depth;
        if (active) active = pcg_float(rng) < q || !perform_rr;
        if (perform_rr) throughput = vscale(throughput, rcpf_(q));
        active = active && depth < in->max_depth;
        if (!active) break;

        int active_medium = medium != MH_INVALID, active_surface = !active_medium;
        int act_null = 0, act_scatter = 0, escaped = 0, spectral = 0;
        med_int mei;
        memset(&mei, 0, sizeof(mei));
        mei.t = INFINITY;
        if (active_medium) {
            const mh_medium *m = &d->media[medium];
            sample_interaction(d, medium, &ray, pcg_float(rng), channel, &mei);
            if (m->type == MH_MEDIUM_HOMOGENEOUS && mei.valid) ray.maxt = mei.t;
            if (needs_intersection) {
                pi_rec pi;
                trace_closest(sv, &ray, &pi);
                if (counters) counters[0]++;
                compute_si(d, &ray, &pi, &si);
            }
            needs_intersection = needs_intersection && !si.valid;
            if (si.t < mei.t) { mei.t = INFINITY; mei.valid = 0; }
            spectral = !(m->flags & MH_MEDIUM_NO_SPECTRAL_EXTINCTION);
            if (spectral) {
                float t = fminf(mei.t, si.t) - mei.mint;
                float tr = oracle_exp((-t) * mei.maj);
                float pdf = si.t < mei.t ? tr : tr * mei.maj;
                float f = pdf > 0.f ? tr / pdf : 0.f;
                throughput = vscale(throughput, f);
            }
            escaped = !mei.valid;
            active_medium = mei.valid;
            int null_scatter = 0;
            if (active_medium) null_scatter = pcg_float(rng) >= mei.sigma_t / mei.maj;
            act_null = null_scatter && active_medium;
            act_scatter = !act_null && active_medium;
            if (spectral && act_null) throughput = vscale(throughput, (mei.sigma_n * mei.maj) / mei.sigma_n);
            if (act_scatter) { depth += 1; last_p = mei.p; }
        }
        active = active && depth < in->max_depth;
        act_scatter = act_scatter && active;
        if (act_null) { ray.o = mei.p; si.t = si.t - mei.t; }
        if (act_scatter) {
            const mh_medium *m = &d->media[medium];
            v3 ss = mei.sigma_s;
            if (spectral) throughput = vmul(throughput, vdivs(vscale(ss, mei.maj), mei.sigma_t));
            else throughput = vmul(throughput, vdivs(ss, mei.sigma_t));
            int sample_emitters = !(m->flags & MH_MEDIUM_NO_EMITTER_SAMPLING);
            valid_ray = 1;
            specular_chain = !sample_emitters;
            if (sample_emitters) {
                dir_sample ds;
                v3 emitted = vol_sample_emitter(sv, mei.p, V3(0, 0, 0), NULL, rng, medium, channel, &ds, counters);
                v3 wo = mei_to_local(&mei, ds.d);
                float ph = phase_eval(m, wo);
                float w = mis_weight_vol(ds.pdf, ds.delta ? 0.f : ph);
                result = vadd(result, vscale(vmul(vscale(throughput, ph), emitted), w));
            }
            (void)pcg_float(rng);
            float s2x = pcg_float(rng), s2y = pcg_float(rng);
            float ph_pdf;
            v3 wo = phase_sample(m, s2x, s2y, &ph_pdf);
            throughput = vscale(throughput, 1.f);
            act_scatter = act_scatter && ph_pdf > 0.f;
            if (act_scatter) {
                ray = spawn_ray(mei.p, V3(0, 0, 0), mei_to_world(&mei, wo));
                needs_intersection = 1;
                last_pdf = ph_pdf;
                throughput = vscale(throughput, 1.f);
            }
        }

        /* ---- surface interactions (volpath.cpp:254-326) ---- */
        active_surface = active_surface || escaped;
        if (active_surface && needs_intersection) {
            pi_rec pi;
            trace_closest(sv, &ray, &pi);
            if (counters) counters[0]++;
            compute_si(d, &ray, &pi, &si);
        }
        if (active_surface) {
            int count_direct = depth == 0 || specular_chain;
            uint32_t em = si_emitter(d, &si);
            if (em != MH_INVALID && !(depth == 0 && in->hide_emitters)) {
                float emitter_pdf = 1.f;
                if (!count_direct) emitter_pdf = emitter_pdf_direction(d, em, &si, last_p);
                v3 emitted = emitter_eval(d, em, &si);
                v3 contrib = count_direct ? vmul(throughput, emitted)
                                          : vmul(vscale(throughput, mis_weight_vol(last_pdf, emitter_pdf)), emitted);
                result = vadd(result, contrib);
            }
        }
        active_surface = active_surface && si.valid;
        if (active_surface) {
            uint32_t b = si_bsdf(d, &si);
            int is_null = b == MH_INVALID || d->bsdfs[b].type == MH_BSDF_NULL;
            int smooth = !is_null;
            v3 rho = V3(0, 0, 0);
            if (smooth) rho = tex_eval(d, d->bsdfs[b].reflectance, si.uvx, si.uvy);
            if (smooth && depth + 1 < in->max_depth) {
                dir_sample ds;
                v3 emitted = vol_sample_emitter(sv, si.p, si.n, &si, rng, medium, channel, &ds, counters);
                v3 wo = to_local(&si, ds.d);
                v3 bv;
                float bp;
                diffuse_eval_pdf(rho, si.wi, wo, 1, &bv, &bp);
                float w = mis_weight_vol(ds.pdf, ds.delta ? 0.f : bp);
                result = vadd(result, vmul(vscale(vmul(throughput, bv), w), emitted));
            }
            (void)pcg_float(rng);
            float s2x = pcg_float(rng), s2y = pcg_float(rng);
            bsdf_sample bs;
            v3 weight;
            if (is_null) {
                bs.wo = vneg(si.wi); bs.pdf = 1.f; bs.eta = 1.f; bs.sampled_delta = 0; bs.sampled_null = 1;
                weight = V3(1, 1, 1);
            } else {
                diffuse_sample(rho, si.wi, s2x, s2y, 1, &bs, &weight);
            }
            throughput = vmul(throughput, weight);
            eta *= bs.eta;
            ray = spawn_ray(si.p, si.n, to_world(&si, bs.wo));
            needs_intersection = 1;
            if (!bs.sampled_null) {
                depth += 1;
                last_p = si.p;
                last_pdf = bs.pdf;
                valid_ray = 1;
                /* specular_chain |= delta (never for diffuse); &= !smooth */
                specular_chain = 0;
            }
            if (is_medium_transition(d, &si)) medium = target_medium(d, &si, ray.d);
        }
        active = active && (active_surface || active_medium);
    }
    *valid_out = valid_ray;
    return result;
}

/* ------------------------------------------------------------------------ */
/* PRBVolpathIntegrator (src/python/python/ad/integrators/prbvolpath.py)     */
/* primal: grad == NULL; adjoint: grad != NULL with L_in = primal radiance   */
/* ------------------------------------------------------------------------ */
typedef struct { int handle_null, nee_hom; } pvp_flags;

/* prepare_scene (prbvolpath.py:76-89): flags from the media of the shapes;
   use_nee is always True. */
static void pvp_prepare(const mh_scene_desc *d, pvp_flags *f) {
    f->handle_null = 0;
    f->nee_hom = 0;
    for (uint32_t i = 0; i < d->n_shapes; ++i) {
        uint32_t ms[2] = {d->shapes[i].interior_medium, d->shapes[i].exterior_medium};
        for (int k = 0; k < 2; ++k) {
            if (ms[k] == MH_INVALID) continue;
            if (d->media[ms[k]].type == MH_MEDIUM_HOMOGENEOUS) f->nee_hom = 1;
            else f->handle_null = 1;
        }
    }
}

/* adjoint of sigma_t(p) = scale * Texture3f(grid).eval(p) (heterogeneous.cpp:192)
   or scale * sigma_t (homogeneous.cpp:158): adj = d loss / d sigma_t(p) */
static void sigma_t_backward(const mh_scene_desc *d, uint32_t med, v3 p, double adj, grad_sink *g) {
    for (uint32_t k = 0; k < g->n_params; ++k) {
        if (g->tex[k] != (MH_PARAM_MEDIUM_SIGMA_T | med)) continue;
        const mh_medium *m = &d->media[med];
        double *a = g->tan ? NULL : g->acc[k];
        const float *t = g->tan ? g->tan[k] : NULL;
        const double as = adj * (double)m->scale;
        if (m->type == MH_MEDIUM_HOMOGENEOUS) {
            if (t) g->fsum += as * t[0];
            else a[0] += as;
            continue;
        }
        /* grid_eval's taps and weights (Texture3f linear, clamp) */
        v3 q = xf_point(m->grid_to_local, p);
        const int32_t rx = (int32_t)m->grid_res[0], ry = (int32_t)m->grid_res[1], rz = (int32_t)m->grid_res[2];
        float px = fmaf(q.x, (float)rx, -0.5f), py = fmaf(q.y, (float)ry, -0.5f), pz = fmaf(q.z, (float)rz, -0.5f);
        int32_t ix = (int32_t)floorf(px), iy = (int32_t)floorf(py), iz = (int32_t)floorf(pz);
        double w1[3] = {px - (float)ix, py - (float)iy, pz - (float)iz};
        double w0[3] = {1.0 - (float)w1[0], 1.0 - (float)w1[1], 1.0 - (float)w1[2]};
#define CL(i, r) ((i) < 0 ? 0 : ((i) > (r) - 1 ? (r) - 1 : (i)))
        int32_t xs[2] = {CL(ix, rx), CL(ix + 1, rx)}, ys[2] = {CL(iy, ry), CL(iy + 1, ry)},
                zs[2] = {CL(iz, rz), CL(iz + 1, rz)};
#undef CL
        for (int c = 0; c < 8; ++c) {
            const int bx = c & 1, by = (c >> 1) & 1, bz = c >> 2;
            const double w = (bz ? w1[2] : w0[2]) * (by ? w1[1] : w0[1]) * (bx ? w1[0] : w0[0]);
            const size_t vi = ((size_t)zs[bz] * (size_t)ry + (size_t)ys[by]) * (size_t)rx + (size_t)xs[bx];
            if (t) g->fsum += as * w * t[vi];
            else a[vi] += as * w;
        }
    }
}

/* adjoint of the constant albedo (constvolume 'albedo.value') */
static void albedo_backward(uint32_t med, v3 adj, grad_sink *g) {
    for (uint32_t k = 0; k < g->n_params; ++k) {
        if (g->tex[k] != (MH_PARAM_MEDIUM_ALBEDO | med)) continue;
        if (g->tan) {
            g->fsum += (double)adj.x * g->tan[k][0] + (double)adj.y * g->tan[k][1] + (double)adj.z * g->tan[k][2];
            continue;
        }
        g->acc[k][0] += adj.x; g->acc[k][1] += adj.y; g->acc[k][2] += adj.z;
    }
}

/* PRBVolpathIntegrator.sample_emitter (prbvolpath.py:336-431).  primal
   (grad == NULL): transmittance detached.  adjoint: replays the walk with a
   cloned sampler and back-propagates dL * adj_emitted through every
   tr_multiplier (prbvolpath.py:412-414). */
static v3 pvp_sample_emitter(const scene_view *sv, const pvp_flags *f, const med_int *mei_ref,
                             const surf_int *si_ref, int active_medium, pcg32 *rng, uint32_t medium,
                             uint32_t channel, dir_sample *ds, v3 adj_emitted, v3 dL, grad_sink *grad,
                             uint64_t *counters) {
    const mh_scene_desc *d = sv->d;
    /* ref_interaction[active_medium] = mei; [active_surface] = si */
    const v3 ref_p = active_medium ? mei_ref->p : si_ref->p;
    const v3 ref_n = active_medium ? V3(0, 0, 0) : si_ref->n;
    float sx = pcg_float(rng), sy = pcg_float(rng);
    v3 emitter_val = scene_sample_emitter_direction(d, ref_p, sx, sy, ds);
    if (ds->pdf == 0.f) return V3(0, 0, 0);   /* emitter_val[invalid] = 0; loop inactive */
    if (!active_medium && is_medium_transition(d, si_ref)) medium = target_medium(d, si_ref, ds->d);
    ray3 ray = spawn_ray(ref_p, ref_n, ds->d);
    const float k_dist = 1.f - SHADOW_EPS;   /* (1.0 - ShadowEpsilon): exact in float */
    float total_dist = 0.f;
    surf_int si;
    memset(&si, 0, sizeof(si));
    int needs_intersection = 1, active = 1;
    v3 transmittance = V3(1, 1, 1);
    while (active) {
        const float remaining_dist = ds->dist * k_dist - total_dist;
        ray.maxt = remaining_dist;
        active = active && remaining_dist > 0.f;
        if (!active) break;
        if (needs_intersection) {
            pi_rec pi;
            trace_closest(sv, &ray, &pi);
            if (counters) counters[1]++;
            compute_si(d, &ray, &pi, &si);
        }
        needs_intersection = 0;
        int act_med = medium != MH_INVALID, act_surf = !act_med, escaped = 0, hom = 0;
        float hom_t = 0.f;
        med_int mei;
        memset(&mei, 0, sizeof(mei));
        v3 trm = V3(1, 1, 1);
        if (act_med) {
            const mh_medium *m = &d->media[medium];
            sample_interaction(d, medium, &ray, pcg_float(rng), channel, &mei);
            if (si.t < mei.t) { mei.t = INFINITY; mei.valid = 0; }
            if (f->nee_hom && m->type == MH_MEDIUM_HOMOGENEOUS) {
                /* direct transmittance to the next surface / segment end (:390-394) */
                mei.t = fminf(remaining_dist, si.t);
                hom_t = fminf(mei.t, si.t) - mei.mint;
                float tr = oracle_exp((-hom_t) * mei.maj);
                trm = V3(tr, tr, tr);
                hom = 1;
                mei.t = INFINITY;
                mei.valid = 0;
            }
            escaped = !mei.valid;
            act_med = mei.valid;
            if (act_med) {
                ray.o = mei.p;
                si.t = si.t - mei.t;
                trm = vscale(trm, mei.sigma_n / mei.maj);
            }
        }
        act_surf = (act_surf || escaped) && si.valid && !act_med;
        if (act_surf) {
            uint32_t b = si_bsdf(d, &si);
            float bv = (b != MH_INVALID && d->bsdfs[b].type == MH_BSDF_NULL) ? 1.f : 0.f;
            trm = vscale(trm, bv);
        }
        if (grad && (act_med || act_surf)) {
            /* backward(tr_multiplier * detach(dL * adj_emitted / tr_multiplier)) */
            const float tc[3] = {trm.x, trm.y, trm.z};
            const float dc[3] = {dL.x, dL.y, dL.z}, ac[3] = {adj_emitted.x, adj_emitted.y, adj_emitted.z};
            double gs = 0.0;
            for (int c = 0; c < 3; ++c) {
                if (!(tc[c] > 0.f)) continue;
                const double up = (double)((dc[c] * ac[c]) / tc[c]);
                if (act_med) gs += up * (-1.0 / (double)mei.maj);              /* d(sigma_n/maj)/d sigma_t */
                else if (hom) gs += up * (-(double)hom_t * (double)tc[c]);     /* d exp(-t sigma_t) */
            }
            if (act_med || hom) sigma_t_backward(d, medium, mei.p, gs, grad);
        }
        transmittance = vmul(transmittance, trm);
        if (act_surf) ray = spawn_ray(si.p, si.n, ray.d);
        needs_intersection = act_surf;
        active = (act_med || act_surf) &&
                 (transmittance.x != 0.f || transmittance.y != 0.f || transmittance.z != 0.f);
        if (active) total_dist += act_med ? mei.t : si.t;
        if (act_surf && is_medium_transition(d, &si)) medium = target_medium(d, &si, ray.d);
    }
    return vmul(emitter_val, transmittance);
}

static v3 prbvol_sample(const scene_view *sv, const mh_integrator *in, pcg32 *rng, ray3 ray,
                        v3 dL, v3 L_in, grad_sink *grad, int *valid_out, uint64_t *counters) {
    const mh_scene_desc *d = sv->d;
    const int primal = grad == NULL;
    pvp_flags f;
    pvp_prepare(d, &f);
    uint32_t depth = 0;
    v3 L = primal ? V3(0, 0, 0) : L_in;
    v3 throughput = V3(1, 1, 1);
    float eta = 1.f;
    int active = 1, valid_ray = 0, needs_intersection = 1;
    surf_int si;
    memset(&si, 0, sizeof(si));
    uint32_t medium = MH_INVALID;   /* "TODO: support sensors inside media" (:123-124) */
    uint32_t channel = (uint32_t)fminf(3.f * pcg_float(rng), 2.f);
    while (active) {
        /* ---- Russian roulette (:142-149) ---- */
        active = active && (throughput.x != 0.f || throughput.y != 0.f || throughput.z != 0.f);
        const float q = fminf(vmax(throughput) * (eta * eta), 0.99f);
        const int perform_rr = depth > in->rr_depth;
        if (active) active = pcg_float(rng) < q || !perform_rr;
        if (perform_rr) throughput = vscale(throughput, rcpf_(q));
        if (!active) break;

        int active_medium = medium != MH_INVALID, active_surface = !active_medium;
        int escaped = 0, act_null = 0, act_scatter = 0;
        float fw = 1.f, P = 1.f, mt = 0.f;
        v3 weight = V3(1, 1, 1);
        med_int mei;
        memset(&mei, 0, sizeof(mei));
        const mh_medium *m = active_medium ? &d->media[medium] : NULL;
        /* ---- medium interaction (:157-204) ---- */
        if (active_medium) {
            sample_interaction(d, medium, &ray, pcg_float(rng), channel, &mei);
            if (m->type == MH_MEDIUM_HOMOGENEOUS && mei.valid) ray.maxt = mei.t;
            if (needs_intersection) {
                pi_rec pi;
                trace_closest(sv, &ray, &pi);
                if (counters) counters[0]++;
                compute_si(d, &ray, &pi, &si);
            }
            needs_intersection = 0;
            if (si.t < mei.t) { mei.t = INFINITY; mei.valid = 0; }
            /* transmittance_eval_pdf (medium.cpp:101-112) */
            mt = fminf(mei.t, si.t) - mei.mint;
            const float tr = oracle_exp((-mt) * mei.maj);
            const float tr_pdf = si.t < mei.t ? tr : tr * mei.maj;
            fw = tr_pdf > 0.f ? tr / tr_pdf : 0.f;
            weight = V3(fw, fw, fw);
            escaped = !mei.valid;
            active_medium = mei.valid;
            if (f.handle_null) {
                P = mei.sigma_t / mei.maj;
                if (active_medium) act_null = pcg_float(rng) >= P;
                act_scatter = !act_null && active_medium;
                if (act_null) weight = vscale(weight, mei.sigma_n / (1.f - P));
            } else {
                act_scatter = active_medium;
            }
            if (act_scatter) depth += 1;
        }
        active = active && depth < in->max_depth;
        act_scatter = act_scatter && active;
        if (f.handle_null && act_null) { ray.o = mei.p; si.t = si.t - mei.t; }
        if (act_scatter)
            weight = V3(weight.x * (mei.sigma_s.x / P), weight.y * (mei.sigma_s.y / P),
                        weight.z * (mei.sigma_s.z / P));
        throughput = vmul(throughput, weight);
        if (!primal && (active_medium || escaped)) {
            /* backward(dL * weight * Lo), Lo = L / max(1e-8, weight) (:202-204) */
            const int homog = m->type == MH_MEDIUM_HOMOGENEOUS;
            const float wc[3] = {weight.x, weight.y, weight.z}, Lc[3] = {L.x, L.y, L.z},
                        dc[3] = {dL.x, dL.y, dL.z}, al[3] = {m->albedo[0], m->albedo[1], m->albedo[2]},
                        ss[3] = {mei.sigma_s.x, mei.sigma_s.y, mei.sigma_s.z};
            double gs = 0.0, ga[3] = {0, 0, 0};
            for (int c = 0; c < 3; ++c) {
                const double up = (double)dc[c] * (double)(Lc[c] / fmaxf(1e-8f, wc[c]));
                double dws = 0.0, dwa = 0.0;   /* d weight_c / d sigma_t(p), d weight_c / d albedo_c */
                const double dfw = homog ? -(double)mt * (double)fw : 0.0;   /* d (tr/tr_pdf) */
                if (act_scatter) {
                    dws = dfw * (double)ss[c] / P + (double)fw * al[c] / P;   /* sigma_s = sigma_t * albedo */
                    dwa = (double)fw * (double)mei.sigma_t / P;
                } else if (act_null) {
                    dws = (double)fw * (-1.0) / (double)(1.f - P);
                } else {
                    dws = dfw;
                }
                gs += up * dws;
                ga[c] = up * dwa;
            }
            sigma_t_backward(d, medium, mei.p, gs, grad);
            if (act_scatter) albedo_backward(medium, V3((float)ga[0], (float)ga[1], (float)ga[2]), grad);
        }

        /* ---- surface interaction (:212-238) ---- */
        active_surface = active_surface || escaped;
        if (active_surface && needs_intersection) {
            pi_rec pi;
            trace_closest(sv, &ray, &pi);
            if (counters) counters[0]++;
            compute_si(d, &ray, &pi, &si);
        }
        active_surface = active_surface && si.valid;
        uint32_t b = active_surface ? si_bsdf(d, &si) : MH_INVALID;
        const int smooth = b != MH_INVALID && d->bsdfs[b].type == MH_BSDF_DIFFUSE;
        v3 rho = V3(0, 0, 0);
        if (smooth) rho = tex_eval(d, d->bsdfs[b].reflectance, si.uvx, si.uvy);

        /* ---- emitter sampling (:242-270) ---- */
        const int active_e_surface = active_surface && smooth && depth + 1 < in->max_depth;
        const int sample_emitters = m && !(m->flags & MH_MEDIUM_NO_EMITTER_SAMPLING);
        const int active_e_medium = act_scatter && sample_emitters;
        if (active_e_surface || active_e_medium) {
            pcg32 nee_rng = *rng;   /* sampler.clone() */
            dir_sample ds;
            v3 emitted = pvp_sample_emitter(sv, &f, &mei, &si, active_e_medium, rng, medium, channel, &ds,
                                            V3(0, 0, 0), V3(0, 0, 0), NULL, counters);
            v3 nee_w, bv = V3(0, 0, 0);
            float nee_pdf, bp = 0.f;
            v3 wo_s = to_local(&si, ds.d);
            if (active_e_surface) {
                diffuse_eval_pdf(rho, si.wi, wo_s, 1, &bv, &bp);
                nee_w = bv;
                nee_pdf = bp;
            } else {
                float ph = phase_eval(m, mei_to_local(&mei, ds.d));
                nee_w = V3(ph, ph, ph);
                nee_pdf = ph;
            }
            if (ds.delta) nee_pdf = 0.f;
            const float mis = mis_weight(ds.pdf, nee_pdf);
            v3 contrib = vmul(vscale(vmul(throughput, nee_w), mis), emitted);
            L = primal ? vadd(L, contrib) : vadd(L, vneg(contrib));
            if (!primal) {
                dir_sample ds2;
                pvp_sample_emitter(sv, &f, &mei, &si, active_e_medium, &nee_rng, medium, channel, &ds2,
                                   contrib, dL, grad, NULL);
                if (active_e_surface && si.wi.z > 0.f && wo_s.z > 0.f) {
                    /* backward(dL * contrib) through bsdf_val = rho / pi * cos */
                    v3 adj = vscale(vscale(vmul(vscale(vmul(dL, emitted), mis), throughput), INV_PI_F), wo_s.z);
                    tex_backward(d, d->bsdfs[b].reflectance, si.uvx, si.uvy, adj, grad);
                }
            }
        }

        /* ---- phase function sampling (:274-294) ---- */
        valid_ray = valid_ray || act_scatter;
        if (act_scatter) {
            (void)pcg_float(rng);
            const float s2x = pcg_float(rng), s2y = pcg_float(rng);
            float ph_pdf;
            v3 wo = phase_sample(m, s2x, s2y, &ph_pdf);
            act_scatter = act_scatter && ph_pdf > 0.f;
            if (act_scatter) {
                ray = spawn_ray(mei.p, V3(0, 0, 0), mei_to_world(&mei, wo));
                needs_intersection = 1;
            }
        }

        /* ---- BSDF sampling (:298-331) ---- */
        if (active_surface) {
            (void)pcg_float(rng);
            const float s2x = pcg_float(rng), s2y = pcg_float(rng);
            bsdf_sample bs;
            v3 bw;
            if (!smooth) {
                bs.wo = vneg(si.wi); bs.pdf = 1.f; bs.eta = 1.f; bs.sampled_delta = 0; bs.sampled_null = 1;
                bw = V3(1, 1, 1);
            } else {
                diffuse_sample(rho, si.wi, s2x, s2y, 1, &bs, &bw);
            }
            active_surface = active_surface && bs.pdf > 0.f;
            if (active_surface) {
                if (!primal && smooth && si.wi.z > 0.f && bs.wo.z > 0.f) {
                    /* Lo = bsdf_eval * detach(L / max(1e-8, bsdf_eval)) (:305-312) */
                    v3 be = vscale(vscale(rho, INV_PI_F), bs.wo.z);
                    v3 adj = V3(dL.x * (L.x / fmaxf(1e-8f, be.x)), dL.y * (L.y / fmaxf(1e-8f, be.y)),
                                dL.z * (L.z / fmaxf(1e-8f, be.z)));
                    adj = vscale(vscale(adj, INV_PI_F), bs.wo.z);
                    tex_backward(d, d->bsdfs[b].reflectance, si.uvx, si.uvy, adj, grad);
                }
                throughput = vmul(throughput, bw);
                eta *= bs.eta;
                ray = spawn_ray(si.p, si.n, to_world(&si, bs.wo));
                needs_intersection = 1;
                if (!bs.sampled_null) { depth += 1; valid_ray = 1; }
                if (is_medium_transition(d, &si)) medium = target_medium(d, &si, ray.d);
            }
        }
        active = active && (active_surface || active_medium);
    }
    *valid_out = valid_ray;
    return primal ? L : dL;
}

static inline float inv_size(uint32_t n) { return 1.f / (float)n; }

/* one sample of one lane: jitter, camera ray, integrator (render_sample,
   integrator.cpp:1139-1240 / common.py:447-525).  Returns L and sample_pos. */
static v3 lane_sample(const scene_view *sv, const mh_integrator *in, const wf_layout *L,
                      pcg32 *rng, uint32_t lane, float *pos_out, int *valid_out,
                      uint64_t *counters) {
    const mh_sensor *s = &sv->d->sensor;
    uint32_t px, py;
    lane_pixel(L, lane, &px, &py);
    float jx = pcg_float(rng), jy = pcg_float(rng);
    float sx = (float)px + jx, sy = (float)py + jy;
    float ax = fmaf(sx, inv_size(L->W), -0.f), ay = fmaf(sy, inv_size(L->H), -0.f);
    ray3 r = camera_ray(s, ax, ay);
    pos_out[0] = sx;
    pos_out[1] = sy;
    if (in->type == MH_INTEGRATOR_PRB)
        return prb_sample(sv, in, rng, r, V3(0, 0, 0), V3(0, 0, 0), NULL, valid_out);
    if (in->type == MH_INTEGRATOR_VOLPATH)
        return volpath_sample(sv, in, rng, r, valid_out, counters);
    if (in->type == MH_INTEGRATOR_PRBVOLPATH)
        return prbvol_sample(sv, in, rng, r, V3(0, 0, 0), V3(0, 0, 0), NULL, valid_out, counters);
    return path_sample(sv, in, rng, r, valid_out, counters);
}

int oracle_sample_range(const mh_scene_desc *desc, const mh_integrator *integ, uint32_t seed,
                        uint32_t spp, uint64_t idx_begin, uint64_t idx_end, float *out_L,
                        float *out_pos, uint32_t *out_valid) {
    scene_view sv;
    if (scene_view_init(&sv, desc)) return 1;
    if (spp == 0) spp = desc->sensor.sample_count;
    wf_layout L;
    const int ad = integ->type == MH_INTEGRATOR_PRB || integ->type == MH_INTEGRATOR_PRBVOLPATH;
    if (wf_init(&desc->sensor, spp, &L, ad)) { scene_view_free(&sv); return fail("wavefront exceeds 2^32 samples"); }
    if (L.n_passes != 1) { scene_view_free(&sv); return fail("oracle_sample_range: multi-pass not supported"); }
    uint32_t seed_value = desc->sensor.sampler_seed + seed;
    for (uint64_t i = idx_begin; i < idx_end; ++i) {
        pcg32 rng;
        sampler_seed(&rng, seed_value, (uint32_t)i);
        float pos[2];
        int valid;
        v3 l = lane_sample(&sv, integ, &L, &rng, (uint32_t)i, pos, &valid, NULL);
        uint64_t k = i - idx_begin;
        out_L[3 * k] = l.x; out_L[3 * k + 1] = l.y; out_L[3 * k + 2] = l.z;
        if (out_pos) { out_pos[2 * k] = pos[0]; out_pos[2 * k + 1] = pos[1]; }
        if (out_valid) out_valid[k] = (uint32_t)valid;
    }
    scene_view_free(&sv);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* scalar_rgb render (BASELINE config 1, the reference's CPU case):          */
/* SamplingIntegrator::render's non-JIT branch (src/render/integrator.cpp:   */
/* 189-275) and render_block (:1099-1124).  Blocks of block_size^2 pixels in */
/* the order of Spiral::next_block (src/render/spiral.cpp:17-70); block b    */
/* seeds pixel i (Morton order inside the block) with                       */
/*   seed * W * H + b * block_size^2 + i                                     */
/* through PCG32Sampler::seed's scalar branch (sampler.cpp:128-131: PCG32    */
/* initstate = base_seed + seed, initseq = PCG32_DEFAULT_STREAM) and draws   */
/* the pixel's spp samples from that one stream (advance() only resets the   */
/* dimension).  The `path` loop takes the scalar control flow               */
/* (path_sample_mode), and the block splats with the non-coalesced filter    */
/* (coalesce = is_jit = false, hdrfilm.cpp:282-290).  The reference's        */
/* block_size shrinks from 32 until there is a block per thread             */
/* (integrator.cpp:200-211): pass the value its run used.                   */
/* ------------------------------------------------------------------------ */
#define PCG32_DEFAULT_STREAM 0xda3e39cb94b95bdbull

static uint32_t morton_compact1(uint32_t v) { /* bits 0, 2, 4, ... -> 0, 1, 2, ... */
    v &= 0x55555555u;
    v = (v | (v >> 1)) & 0x33333333u;
    v = (v | (v >> 2)) & 0x0f0f0f0fu;
    v = (v | (v >> 4)) & 0x00ff00ffu;
    v = (v | (v >> 8)) & 0x0000ffffu;
    return v;
}

/* block positions (in blocks) of Spiral::next_block for one pass */
static uint32_t spiral_order(uint32_t bw, uint32_t bh, uint32_t *bx, uint32_t *by) {
    const uint32_t count = bw * bh;
    int32_t px = (int32_t)(bw / 2), py = (int32_t)(bh / 2);
    int dir = 0; /* Right, Down, Left, Up */
    uint32_t steps_left = 1, spiral_size = 1;
    for (uint32_t k = 0; k < count; ++k) {
        bx[k] = (uint32_t)px;
        by[k] = (uint32_t)py;
        if (k + 1 == count) break;
        do {
            switch (dir) {
                case 0: ++px; break;
                case 1: ++py; break;
                case 2: --px; break;
                default: --py; break;
            }
            if (--steps_left == 0) {
                dir = (dir + 1) % 4;
                if (dir == 2 || dir == 0) ++spiral_size;
                steps_left = spiral_size;
            }
        } while (px < 0 || py < 0 || px >= (int32_t)bw || py >= (int32_t)bh);
    }
    return count;
}

typedef struct {
    const scene_view *sv;
    const mh_integrator *in;
    uint32_t seed, spp, block_size, n_blocks;
    const uint32_t *bx, *by;
    uint32_t *next;         /* shared block counter */
    pthread_mutex_t *lock;
    float *film;            /* this worker's full RGBW film */
} scalar_job;

static void *scalar_worker(void *arg) {
    scalar_job *j = (scalar_job *)arg;
    const mh_scene_desc *d = j->sv->d;
    const mh_sensor *s = &d->sensor;
    const uint32_t W = s->width, H = s->height, bs = j->block_size, pc = bs * bs;
    film_band band = {j->film, W, H, 0, H, 4};
    for (;;) {
        pthread_mutex_lock(j->lock);
        const uint32_t b = (*j->next)++;
        pthread_mutex_unlock(j->lock);
        if (b >= j->n_blocks) break;
        const uint32_t ox = j->bx[b] * bs, oy = j->by[b] * bs;
        const uint32_t sw = W - ox < bs ? W - ox : bs, sh = H - oy < bs ? H - oy : bs;
        const uint32_t seed_b = j->seed * (W * H) + b * pc; /* integrator.cpp:230, :1103 */
        for (uint32_t i = 0; i < pc; ++i) {
            const uint32_t lx = morton_compact1(i), ly = morton_compact1(i >> 1);
            if (lx >= sw || ly >= sh) continue;
            pcg32 rng;
            pcg_seed(&rng, (uint64_t)(uint32_t)(s->sampler_seed + seed_b + i), PCG32_DEFAULT_STREAM);
            const uint32_t px = ox + lx, py = oy + ly;
            for (uint32_t k = 0; k < j->spp; ++k) {
                const float jx = pcg_float(&rng), jy = pcg_float(&rng);
                const float sx = (float)px + jx, sy = (float)py + jy;
                ray3 r = camera_ray(s, fmaf(sx, inv_size(W), -0.f), fmaf(sy, inv_size(H), -0.f));
                int valid;
                v3 l = path_sample_mode(j->sv, j->in, &rng, r, &valid, NULL, 1);
                const float vals[4] = {l.x, l.y, l.z, 1.f};
                splat(s, &band, sx, sy, vals, 0);
            }
        }
    }
    return NULL;
}

int oracle_render_scalar(const mh_scene_desc *desc, const mh_integrator *integ, uint32_t seed,
                         uint32_t spp, uint32_t block_size, int n_threads, float *film_rgbw) {
    if (integ->type != MH_INTEGRATOR_PATH) return fail("oracle_render_scalar: the 'path' integrator only");
    if (fmt_alpha(desc->sensor.pixel_format)) return fail("oracle_render_scalar: rgb films only");
    if (block_size == 0 || (block_size & (block_size - 1))) return fail("oracle_render_scalar: block_size must be a power of two");
    scene_view sv;
    if (scene_view_init(&sv, desc)) return 1;
    if (spp == 0) spp = desc->sensor.sample_count;
    const uint32_t W = desc->sensor.width, H = desc->sensor.height;
    const uint32_t bw = (W + block_size - 1) / block_size, bh = (H + block_size - 1) / block_size;
    uint32_t *bx = (uint32_t *)malloc(sizeof(uint32_t) * bw * bh), *by = (uint32_t *)malloc(sizeof(uint32_t) * bw * bh);
    const uint32_t nb = spiral_order(bw, bh, bx, by);
    if (n_threads < 1) n_threads = 1;
    float *films = (float *)calloc((size_t)n_threads * W * H * 4, sizeof(float));
    scalar_job *jobs = (scalar_job *)calloc((size_t)n_threads, sizeof(scalar_job));
    pthread_t *th = (pthread_t *)calloc((size_t)n_threads, sizeof(pthread_t));
    pthread_mutex_t lock = PTHREAD_MUTEX_INITIALIZER;
    uint32_t next = 0;
    for (int t = 0; t < n_threads; ++t) {
        scalar_job *j = &jobs[t];
        j->sv = &sv; j->in = integ; j->seed = seed; j->spp = spp; j->block_size = block_size;
        j->n_blocks = nb; j->bx = bx; j->by = by; j->next = &next; j->lock = &lock;
        j->film = films + (size_t)t * W * H * 4;
        pthread_create(&th[t], NULL, scalar_worker, j);
    }
    for (int t = 0; t < n_threads; ++t) pthread_join(th[t], NULL);
    memset(film_rgbw, 0, sizeof(float) * (size_t)W * H * 4);
    for (int t = 0; t < n_threads; ++t)
        for (size_t i = 0; i < (size_t)W * H * 4; ++i) film_rgbw[i] += films[(size_t)t * W * H * 4 + i];
    free(films); free(jobs); free(th); free(bx); free(by);
    scene_view_free(&sv);
    return 0;
}

/* the block order itself, for tests (block positions in units of blocks) */
uint32_t oracle_spiral_order(uint32_t bw, uint32_t bh, uint32_t *bx, uint32_t *by) {
    return spiral_order(bw, bh, bx, by);
}

/* ---- threaded film renderer (row bands, deterministic merge) ---- */
typedef enum { JOB_RENDER = 0, JOB_WEIGHTS = 1, JOB_BACKWARD = 2, JOB_FORWARD = 3 } job_kind;

typedef struct {
    const scene_view *sv;
    const mh_integrator *in;
    const wf_layout *L;
    job_kind kind;
    uint32_t seed_value, spp_begin, spp_end;
    uint32_t row_begin, row_end;
    film_band band;            /* rows [row_begin-2, row_end+2) */
    /* backward */
    const float *grad_in, *weights;
    grad_sink sink;
    int err;
} band_job;

static uint32_t splat_margin(const mh_sensor *s) {
    return s->rfilter == MH_RFILTER_BOX ? 0u : (uint32_t)ceilf(s->rfilter_radius) + 1u;
}

/* δL_i = sum_px grad_in[px] / W'[px] * w_i(px)   (common.py:936-947) */
static v3 gather_dL(const mh_sensor *s, int coalesce, const float *grad_in, const float *weights,
                    float px, float py) {
    const uint32_t W = s->width, H = s->height;
    double acc[3] = {0, 0, 0};
    float out[3] = {0, 0, 0};
    (void)acc;
    if (s->rfilter == MH_RFILTER_BOX) {
        int32_t ix = (int32_t)floorf(px), iy = (int32_t)floorf(py);
        uint32_t ux = (uint32_t)ix, uy = (uint32_t)iy;
        if (ux < W && uy < H) {
            size_t p = (size_t)uy * W + ux;
            float Wp = weights[p] == 0.f ? 1.f : weights[p];
            for (int c = 0; c < 3; ++c) out[c] = grad_in[3 * p + c] / Wp;
        }
        return V3(out[0], out[1], out[2]);
    }
    const float radius = s->rfilter_radius;
    if (coalesce) {
        int32_t n = (int32_t)ceilf(radius - 0.5f), count = 2 * n + 1;
        int32_t pix = (int32_t)floorf(px) - n, piy = (int32_t)floorf(py) - n;
        uint32_t x = (uint32_t)pix, y = (uint32_t)piy;
        float relx = ((float)pix + 0.5f) - px, rely = ((float)piy + 0.5f) - py;
        for (int32_t ys = 0; ys < count; ++ys) {
            float wy = rfilter_eval(s, rely + (float)ys);
            for (int32_t xs = 0; xs < count; ++xs) {
                float wx = rfilter_eval(s, relx + (float)xs);
                uint32_t xx = x + (uint32_t)xs, yy = y + (uint32_t)ys;
                if (xx < W && yy < H) {
                    size_t p = (size_t)yy * W + xx;
                    float Wp = weights[p] == 0.f ? 1.f : weights[p];
                    float w = wy * wx;
                    for (int c = 0; c < 3; ++c) out[c] += (grad_in[3 * p + c] / Wp) * w;
                }
            }
        }
    } else {
        float pfx = px - 0.5f, pfy = py - 0.5f;
        int32_t a0x = (int32_t)ceilf(pfx - radius), a0y = (int32_t)ceilf(pfy - radius);
        int32_t a1x = (int32_t)floorf(pfx + radius), a1y = (int32_t)floorf(pfy + radius);
        if (a0x < 0) a0x = 0;
        if (a0y < 0) a0y = 0;
        if (a1x > (int32_t)W - 1) a1x = (int32_t)W - 1;
        if (a1y > (int32_t)H - 1) a1y = (int32_t)H - 1;
        if (!(a0x <= a1x && a0y <= a1y)) return V3(0, 0, 0);
        uint32_t count = (uint32_t)ceilf(2.f * radius);
        float relx = (float)a0x - pfx, rely = (float)a0y - pfy;
        for (uint32_t ys = 0; ys < count; ++ys) {
            float wy = rfilter_eval(s, rely + (float)ys);
            for (uint32_t xs = 0; xs < count; ++xs) {
                float wx = rfilter_eval(s, relx + (float)xs);
                uint32_t xx = (uint32_t)a0x + xs, yy = (uint32_t)a0y + ys;
                if ((int32_t)xx <= a1x && (int32_t)yy <= a1y) {
                    size_t p = (size_t)yy * W + xx;
                    float Wp = weights[p] == 0.f ? 1.f : weights[p];
                    float w = wy * wx;
                    for (int c = 0; c < 3; ++c) out[c] += (grad_in[3 * p + c] / Wp) * w;
                }
            }
        }
    }
    return V3(out[0], out[1], out[2]);
}

static void *band_worker(void *arg) {
    band_job *j = (band_job *)arg;
    const wf_layout *L = j->L;
    const mh_sensor *s = &j->sv->d->sensor;
    int coalesce = L->spp_pp >= 4;
    for (uint32_t py = j->row_begin; py < j->row_end; ++py) {
        for (uint32_t px = 0; px < L->W; ++px) {
            uint64_t pixel = (uint64_t)py * L->W + px;
            for (uint32_t sidx = j->spp_begin; sidx < j->spp_end; ++sidx) {
                uint32_t lane = (uint32_t)(pixel * L->spp_pp + sidx);
                pcg32 rng;
                sampler_seed(&rng, j->seed_value, lane);
                for (uint32_t pass = 0; pass < L->n_passes; ++pass) {
                    float pos[2];
                    int valid;
                    if (j->kind == JOB_FORWARD) {
                        /* render_forward (common.py:766-806): primal with the
                           cloned sampler, then the forward-mode replay -- here
                           once per colour channel c with dL = e_c through the
                           sinks in forward mode -- splatted as (dL, weight 1,
                           alpha = valid) */
                        float jx = pcg_float(&rng), jy = pcg_float(&rng);
                        float sx = (float)px + jx, sy = (float)py + jy;
                        ray3 r = camera_ray(s, fmaf(sx, inv_size(L->W), -0.f), fmaf(sy, inv_size(L->H), -0.f));
                        const int vol = j->in->type == MH_INTEGRATOR_PRBVOLPATH;
                        pcg32 rng_primal = rng;
                        v3 Lp = vol ? prbvol_sample(j->sv, j->in, &rng_primal, r, V3(0, 0, 0), V3(0, 0, 0), NULL, &valid, NULL)
                                    : prb_sample(j->sv, j->in, &rng_primal, r, V3(0, 0, 0), V3(0, 0, 0), NULL, &valid);
                        float dl[3];
                        for (int c = 0; c < 3; ++c) {
                            pcg32 rc = rng;
                            int v2;
                            v3 e = V3(c == 0 ? 1.f : 0.f, c == 1 ? 1.f : 0.f, c == 2 ? 1.f : 0.f);
                            j->sink.fsum = 0.0;
                            if (vol) prbvol_sample(j->sv, j->in, &rc, r, e, Lp, &j->sink, &v2, NULL);
                            else prb_sample(j->sv, j->in, &rc, r, e, Lp, &j->sink, &v2);
                            dl[c] = (float)j->sink.fsum;
                        }
                        float vals[5] = {dl[0], dl[1], dl[2], 1.f, 1.f};
                        if (j->band.ch == 5) vals[3] = valid ? 1.f : 0.f;
                        splat(s, &j->band, sx, sy, vals, coalesce);
                    } else if (j->kind == JOB_RENDER) {
                        v3 l = lane_sample(j->sv, j->in, L, &rng, lane, pos, &valid, NULL);
                        /* aovs (integrator.cpp:1216-1233): alpha = valid ? 1 : 0 */
                        float vals[5] = {l.x, l.y, l.z, 1.f, 1.f};
                        if (j->band.ch == 5) vals[3] = valid ? 1.f : 0.f;
                        splat(s, &j->band, pos[0], pos[1], vals, coalesce);
                    } else if (j->kind == JOB_WEIGHTS) {
                        float jx = pcg_float(&rng), jy = pcg_float(&rng);
                        float vals[4] = {0.f, 0.f, 0.f, 1.f};
                        splat(s, &j->band, (float)px + jx, (float)py + jy, vals, coalesce);
                    } else {
                        /* render_backward (common.py:900-983) for one sample */
                        float jx = pcg_float(&rng), jy = pcg_float(&rng);
                        float sx = (float)px + jx, sy = (float)py + jy;
                        ray3 r = camera_ray(s, fmaf(sx, inv_size(L->W), -0.f),
                                            fmaf(sy, inv_size(L->H), -0.f));
                        v3 dL = gather_dL(s, coalesce, j->grad_in, j->weights, sx, sy);
                        pcg32 rng_primal = rng; /* sampler.clone() */
                        if (j->in->type == MH_INTEGRATOR_PRBVOLPATH) {
                            v3 Lp = prbvol_sample(j->sv, j->in, &rng_primal, r, V3(0, 0, 0),
                                                  V3(0, 0, 0), NULL, &valid, NULL);
                            prbvol_sample(j->sv, j->in, &rng, r, dL, Lp, &j->sink, &valid, NULL);
                        } else {
                            v3 Lp = prb_sample(j->sv, j->in, &rng_primal, r, V3(0, 0, 0),
                                               V3(0, 0, 0), NULL, &valid);
                            prb_sample(j->sv, j->in, &rng, r, dL, Lp, &j->sink, &valid);
                        }
                    }
                }
            }
        }
    }
    return NULL;
}

/* number of gradient entries of a parameter id (texture index or MH_PARAM_*) */
static size_t param_count(const mh_scene_desc *desc, uint32_t id) {
    const uint32_t kind = id & MH_PARAM_KIND_MASK, idx = id & ~MH_PARAM_KIND_MASK;
    if (kind == MH_PARAM_MEDIUM_ALBEDO) return 3;
    if (kind == MH_PARAM_MEDIUM_SIGMA_T) {
        const mh_medium *m = &desc->media[idx];
        return m->type == MH_MEDIUM_HOMOGENEOUS
                   ? 1 : (size_t)m->grid_res[0] * m->grid_res[1] * m->grid_res[2];
    }
    const mh_texture *tx = &desc->textures[idx];
    return tx->type == MH_TEX_RGB ? 3 : (size_t)tx->width * tx->height * tx->channels;
}

/* rows [row_lo, row_hi) of pixels whose samples are run (0, 0: all rows) */
static int run_bands(const mh_scene_desc *desc, const mh_integrator *in, job_kind kind,
                     uint32_t seed, uint32_t spp, uint32_t spp_begin, uint32_t spp_end,
                     int n_threads, float *film, const float *grad_in, const float *weights,
                     uint32_t n_params, const uint32_t *param_tex, float *const *grads,
                     uint32_t row_lo, uint32_t row_hi, const float *const *tangents) {
    scene_view sv;
    if (scene_view_init(&sv, desc)) return 1;
    const mh_sensor *s = &desc->sensor;
    if (spp == 0) spp = s->sample_count;
    wf_layout L;
    const int ad = kind != JOB_RENDER || in->type == MH_INTEGRATOR_PRB || in->type == MH_INTEGRATOR_PRBVOLPATH;
    if (wf_init(s, spp, &L, ad)) {
        scene_view_free(&sv);
        return fail("The total number of Monte Carlo samples required by this rendering task exceeds 2^32");
    }
    if (spp_end == 0 && spp_begin == 0) spp_end = L.spp_pp;
    if (spp_end > L.spp_pp || spp_begin >= spp_end) { scene_view_free(&sv); return fail("invalid sample slab"); }
    if (row_lo == 0 && row_hi == 0) row_hi = L.H;
    if (row_hi > L.H || row_lo >= row_hi) { scene_view_free(&sv); return fail("invalid row range"); }
    const uint32_t n_rows = row_hi - row_lo;
    if (n_threads < 1) n_threads = 1;
    if ((uint32_t)n_threads > n_rows) n_threads = (int)n_rows;
    uint32_t margin = splat_margin(s);
    band_job *jobs = (band_job *)calloc((size_t)n_threads, sizeof(band_job));
    pthread_t *th = (pthread_t *)calloc((size_t)n_threads, sizeof(pthread_t));
    const uint32_t fch = fmt_alpha(s->pixel_format) ? 5 : 4; /* film channels of JOB_RENDER */
    for (int t = 0; t < n_threads; ++t) {
        band_job *j = &jobs[t];
        j->sv = &sv; j->in = in; j->L = &L; j->kind = kind;
        j->seed_value = s->sampler_seed + seed;
        j->spp_begin = spp_begin; j->spp_end = spp_end;
        j->row_begin = row_lo + (uint32_t)((uint64_t)n_rows * t / n_threads);
        j->row_end = row_lo + (uint32_t)((uint64_t)n_rows * (t + 1) / n_threads);
        j->grad_in = grad_in; j->weights = weights;
        if (kind != JOB_BACKWARD) {
            int32_t r0 = (int32_t)j->row_begin - (int32_t)margin;
            if (r0 < 0) r0 = 0;
            int32_t r1 = (int32_t)j->row_end + (int32_t)margin;
            if (r1 > (int32_t)L.H) r1 = (int32_t)L.H;
            j->band.width = L.W; j->band.height = L.H; j->band.row0 = r0;
            j->band.rows = (uint32_t)(r1 - r0);
            j->band.ch = (kind == JOB_RENDER || kind == JOB_FORWARD) ? fch : 4;
            j->band.data = (float *)calloc((size_t)j->band.rows * L.W * j->band.ch, sizeof(float));
            if (kind == JOB_FORWARD) {
                j->sink.n_params = n_params;
                j->sink.tex = param_tex;
                j->sink.tan = tangents;
            }
        } else {
            j->sink.n_params = n_params;
            j->sink.tex = param_tex;
            j->sink.acc = (double **)calloc(n_params ? n_params : 1, sizeof(double *));
            for (uint32_t k = 0; k < n_params; ++k)
                j->sink.acc[k] = (double *)calloc(param_count(desc, param_tex[k]), sizeof(double));
        }
        pthread_create(&th[t], NULL, band_worker, j);
    }
    for (int t = 0; t < n_threads; ++t) pthread_join(th[t], NULL);
    if (kind == JOB_BACKWARD) {
        for (uint32_t k = 0; k < n_params; ++k) {
            size_t cnt = param_count(desc, param_tex[k]);
            for (size_t c = 0; c < cnt; ++c) {
                double sum = 0.0;
                for (int t = 0; t < n_threads; ++t) sum += jobs[t].sink.acc[k][c];
                grads[k][c] += (float)sum;
            }
        }
        for (int t = 0; t < n_threads; ++t) {
            for (uint32_t k = 0; k < n_params; ++k) free(jobs[t].sink.acc[k]);
            free(jobs[t].sink.acc);
        }
    } else {
        size_t npx = (size_t)L.W * L.H;
        if (kind == JOB_RENDER || kind == JOB_FORWARD) memset(film, 0, npx * fch * sizeof(float));
        else memset(film, 0, npx * sizeof(float));
        for (int t = 0; t < n_threads; ++t) {
            band_job *j = &jobs[t];
            const uint32_t bc = j->band.ch;
            for (uint32_t r = 0; r < j->band.rows; ++r) {
                size_t row = (size_t)(j->band.row0 + (int32_t)r);
                for (uint32_t x = 0; x < L.W; ++x) {
                    const float *src = j->band.data + ((size_t)r * L.W + x) * bc;
                    if (kind == JOB_RENDER || kind == JOB_FORWARD) {
                        float *dst = film + (row * L.W + x) * bc;
                        for (uint32_t c = 0; c < bc; ++c) dst[c] += src[c];
                    } else {
                        film[row * L.W + x] += src[3];
                    }
                }
            }
            free(j->band.data);
        }
    }
    free(jobs);
    free(th);
    scene_view_free(&sv);
    return 0;
}

int oracle_render(const mh_scene_desc *desc, const mh_integrator *integ, uint32_t seed,
                  uint32_t spp, uint32_t spp_begin, uint32_t spp_end, int n_threads,
                  float *film_rgbw) {
    return run_bands(desc, integ, JOB_RENDER, seed, spp, spp_begin, spp_end, n_threads,
                     film_rgbw, NULL, NULL, 0, NULL, NULL, 0, 0, NULL);
}

int oracle_prb_weights(const mh_scene_desc *desc, uint32_t seed, uint32_t spp,
                       uint32_t spp_begin, uint32_t spp_end, int n_threads, float *weights) {
    mh_integrator dummy = {MH_INTEGRATOR_PRB, 1, 1, 0};
    return run_bands(desc, &dummy, JOB_WEIGHTS, seed, spp, spp_begin, spp_end, n_threads,
                     weights, NULL, NULL, 0, NULL, NULL, 0, 0, NULL);
}

/* W image from the samples of pixel rows [row_lo, row_hi) only (test helper
 * for films too large to sweep: rows [row_lo + 2, row_hi - 2) -- and the
 * image border rows inside the range -- equal oracle_prb_weights) */
int oracle_prb_weights_rows(const mh_scene_desc *desc, uint32_t seed, uint32_t spp, uint32_t row_lo,
                            uint32_t row_hi, int n_threads, float *weights) {
    mh_integrator dummy = {MH_INTEGRATOR_PRB, 1, 1, 0};
    return run_bands(desc, &dummy, JOB_WEIGHTS, seed, spp, 0, 0, n_threads, weights, NULL, NULL, 0, NULL,
                     NULL, row_lo, row_hi, NULL);
}

int oracle_render_backward(const mh_scene_desc *desc, const mh_integrator *integ,
                           uint32_t seed, uint32_t spp, uint32_t spp_begin, uint32_t spp_end,
                           const float *grad_in, const float *weights, uint32_t n_params,
                           const uint32_t *param_textures, float *const *grads, int n_threads) {
    if (integ->type != MH_INTEGRATOR_PRB && integ->type != MH_INTEGRATOR_PRBVOLPATH)
        return fail("render_backward: requires the 'prb' or 'prbvolpath' integrator");
    for (uint32_t k = 0; k < n_params; ++k) {
        const uint32_t kind = param_textures[k] & MH_PARAM_KIND_MASK, idx = param_textures[k] & ~MH_PARAM_KIND_MASK;
        if (kind == 0 ? idx >= desc->n_textures
                      : (kind != MH_PARAM_MEDIUM_SIGMA_T && kind != MH_PARAM_MEDIUM_ALBEDO) || idx >= desc->n_media)
            return fail("render_backward: parameter index out of bounds");
        if (kind != 0 && integ->type != MH_INTEGRATOR_PRBVOLPATH)
            return fail("render_backward: medium parameters require the 'prbvolpath' integrator");
    }
    const mh_sensor *s = &desc->sensor;
    float *w_local = NULL;
    if (!weights) {
        w_local = (float *)malloc(sizeof(float) * s->width * s->height);
        if (oracle_prb_weights(desc, seed, spp, 0, 0, n_threads, w_local)) { free(w_local); return 1; }
        weights = w_local;
    }
    int rc = run_bands(desc, integ, JOB_BACKWARD, seed, spp, spp_begin, spp_end, n_threads, NULL,
                       grad_in, weights, n_params, param_textures, grads, 0, 0, NULL);
    free(w_local);
    return rc;
}

int oracle_render_forward(const mh_scene_desc *desc, const mh_integrator *integ, uint32_t seed,
                          uint32_t spp, uint32_t spp_begin, uint32_t spp_end, uint32_t n_params,
                          const uint32_t *param_ids, const float *const *tangents, int n_threads,
                          float *film) {
    if (integ->type != MH_INTEGRATOR_PRB && integ->type != MH_INTEGRATOR_PRBVOLPATH)
        return fail("render_forward(): requires the 'prb' or 'prbvolpath' integrator");
    for (uint32_t k = 0; k < n_params; ++k) {
        const uint32_t kind = param_ids[k] & MH_PARAM_KIND_MASK, idx = param_ids[k] & ~MH_PARAM_KIND_MASK;
        if (kind == 0 ? idx >= desc->n_textures
                      : (kind != MH_PARAM_MEDIUM_SIGMA_T && kind != MH_PARAM_MEDIUM_ALBEDO) || idx >= desc->n_media)
            return fail("render_forward: parameter index out of bounds");
        if (kind != 0 && integ->type != MH_INTEGRATOR_PRBVOLPATH)
            return fail("render_forward(): medium parameters require the 'prbvolpath' integrator");
    }
    return run_bands(desc, integ, JOB_FORWARD, seed, spp, spp_begin, spp_end, n_threads, film, NULL, NULL,
                     n_params, param_ids, NULL, 0, 0, tangents);
}
