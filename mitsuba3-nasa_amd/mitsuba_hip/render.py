"""mi.render / traverse / render_backward on the hip_ad_rgb backend.

Restates src/python/python/util.py:292-350 (traverse / SceneParameters),
util.py:356-408 (_RenderOp) and util.py:512-625 (mi.render) with
``torch.autograd`` standing in for Dr.Jit's AD graph: ``loss.backward()``
drives RBIntegrator.render_backward exactly where ``dr.backward(loss)`` does in
the reference.  Images and gradients live on the scene's HIP device as torch
tensors (torch is plumbing here: device memory + streams).
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Dict, List, Optional

import numpy as np

from . import _abi as A
from .scene import Integrator, Scene


def _torch():
    import torch
    return torch


def sample_tea_32(v0: int, v1: int, rounds: int = 4):
    """core/random.h:77-90"""
    m = 0xFFFFFFFF
    s = 0
    v0 &= m
    v1 &= m
    for _ in range(rounds):
        s = (s + 0x9E3779B9) & m
        v0 = (v0 + ((((v1 << 4) & m) + 0xA341316C) ^ ((v1 + s) & m) ^ ((v1 >> 5) + 0xC8013EA4))) & m
        v1 = (v1 + ((((v0 << 4) & m) + 0xAD90777D) ^ ((v0 + s) & m) ^ ((v0 >> 5) + 0x7E95761E))) & m
    return v0, v1


def _device_index(device) -> int:
    torch = _torch()
    if device is None:
        if not torch.cuda.is_available():
            raise A.MitsubaHipError("mitsuba_hip: no HIP device available (hip_ad_rgb has no CPU fallback)")
        return torch.cuda.current_device()
    return torch.device(device).index or 0


# MH_ASYNC_CALLS=1: the wrappers return once their kernels are enqueued on
# the current stream (torch-op semantics, MH_FLAG_NO_SYNC).  Off by default:
# the bench step measured 36.7 ms with a sync per call and 38.1-40.2 ms
# without, its PRB bounce launches running ~9 % slower back to back
# 
_NO_SYNC = A.FLAG_NO_SYNC if os.environ.get("MH_ASYNC_CALLS") == "1" else 0


def _ptr(t) -> C.c_void_p:
    return C.c_void_p(t.data_ptr())


class SceneParameters:
    """util.py:13-290 (SceneParameters) restricted to the differentiable
    parameters on the hot path: '<bsdf>.reflectance.value' / '.data' and the
    medium parameters '<medium>.sigma_t.data' (grid, shape (z, y, x, 1) as the
    reference's TensorXf), '<medium>.sigma_t.value' (homogeneous) and
    '<medium>.albedo.value'."""

    def __init__(self, scene: Scene, device=None):
        torch = _torch()
        self.scene = scene
        self._device = device
        self._values = {}
        self._kind = {}
        for key, (kind, idx) in scene.params.items():
            if kind == "rgb":
                v = torch.tensor(list(scene.texture(idx).value), dtype=torch.float32)
            elif kind == "bitmap":
                t = scene.texture(idx)
                v = torch.from_numpy(scene.texture_data(idx).reshape(t.height, t.width, t.channels).copy())
            elif kind == "grid":
                m = scene.medium(idx)
                v = torch.from_numpy(scene.grid_data(idx).reshape(m.grid_res[2], m.grid_res[1], m.grid_res[0], 1).copy())
            elif kind == "medium_sigma_t":
                v = torch.tensor([scene.medium(idx).sigma_t_const], dtype=torch.float32)
            elif kind == "medium_albedo":
                v = torch.tensor(list(scene.medium(idx).albedo), dtype=torch.float32)
            else:
                continue
            if device is not None:
                v = v.to(device)
            self._values[key] = v
            self._kind[key] = (kind, idx)
        self._dirty = set()

    def keys(self):
        return self._values.keys()

    def items(self):
        return self._values.items()

    def __contains__(self, k):
        return k in self._values

    def __len__(self):
        return len(self._values)

    def __getitem__(self, k):
        return self._values[k]

    def __setitem__(self, k, v):
        torch = _torch()
        if k not in self._values:
            raise KeyError(k)
        old = self._values[k]
        v = torch.as_tensor(v, dtype=torch.float32, device=old.device)
        if v.shape != old.shape:
            v = v.reshape(old.shape)
        self._values[k] = v
        self._dirty.add(k)

    def texture_of(self, k) -> int:
        return self._kind[k][1]

    def param_id(self, k) -> int:
        """mh_render_backward parameter id (include/mitsuba_hip.h MH_PARAM_*)."""
        kind, idx = self._kind[k]
        if kind in ("grid", "medium_sigma_t"):
            return A.PARAM_MEDIUM_SIGMA_T | idx
        if kind == "medium_albedo":
            return A.PARAM_MEDIUM_ALBEDO | idx
        return idx

    def update(self, values: Optional[Dict] = None):
        """Push modified values into every device copy of the scene."""
        if values:
            for k, v in values.items():
                self[k] = v
        keys = list(self._dirty) if self._dirty else list(self._values.keys())
        L = A.lib() if self.scene._handles else None
        for k in keys:
            kind, idx = self._kind[k]
            arr = self._values[k].detach().float().cpu().contiguous().numpy().reshape(-1)
            if kind == "rgb":
                self.scene.texture(idx).value[:] = [float(x) for x in arr]
                for h in self.scene._handles.values():
                    A.check(L.mh_scene_update_rgb(h, idx, arr.ctypes.data_as(A.PF)))
            elif kind in ("grid", "medium_sigma_t", "medium_albedo"):
                m = self.scene.medium(idx)
                if kind == "grid":
                    self.scene.grid_data(idx)[:] = arr
                    m.max_density = float(arr.max()) if arr.size else 0.0   # parameters_changed
                elif kind == "medium_sigma_t":
                    m.sigma_t_const = float(arr[0])
                else:
                    m.albedo[:] = [float(x) for x in arr]
                p = arr.ctypes.data_as(C.c_void_p)
                for h in self.scene._handles.values():
                    A.check(L.mh_scene_update_medium(h, idx, p if kind == "medium_albedo" else None,
                                                     p if kind == "medium_sigma_t" else None,
                                                     p if kind == "grid" else None, arr.size, 0))
            else:
                dst = self.scene.texture_data(idx)
                dst[:] = arr
                for h in self.scene._handles.values():
                    A.check(L.mh_scene_update_texture(h, idx, arr.ctypes.data_as(A.PF), arr.size))
        self._dirty.clear()
        return [(k, None) for k in keys]

    def __repr__(self):
        return "SceneParameters[\n" + "".join(f"  {k}: {tuple(v.shape)}\n" for k, v in self._values.items()) + "]"


def traverse(scene: Scene, device=None) -> SceneParameters:
    return SceneParameters(scene, device)


# ---------------------------------------------------------------------------
# core entry points (C-ABI wrappers; all buffers stay on the device)
# ---------------------------------------------------------------------------
def render_film(scene: Scene, integrator: Optional[Integrator] = None, seed: int = 0, spp: int = 0,
                spp_begin: int = 0, spp_end: int = 0, device=None, film=None, accumulate=False,
                stats: Optional[A.Stats] = None, mode: str = "auto", deterministic: bool = False,
                shared: bool = False):
    """Integrator::render(develop=False): RGBW film (H, W, 4) on the device.
    mode: 'auto' (wavefront for `path`), 'mega' (per-lane megakernel) or 'wavefront'.
    deterministic: splat as a fixed-order gather (bit-reproducible film) instead
    of float atomics.  stats.invalid_samples counts samples with a non-finite
    or negative channel (ImageBlock::put's warn_invalid / warn_negative test).
    shared: another call runs on the device at the same time
    (MH_FLAG_SHARED_DEVICE, a performance hint; the result is unchanged)."""
    torch = _torch()
    dev = _device_index(device)
    integrator = integrator or scene.integrator()
    spp = spp or scene.sample_count()
    h = scene.handle(dev, torch.cuda.current_stream(dev).cuda_stream)
    if film is None:
        film = torch.empty((scene.height, scene.width, A.film_channels(scene.desc.sensor.pixel_format)),
                           dtype=torch.float32, device=f"cuda:{dev}")
    # stream-ordered like a torch op: the call returns once its kernels are
    # enqueued (a stats request reads counters back, which synchronises)
    flags = A.FLAG_DEVICE_POINTERS | _NO_SYNC | (A.FLAG_ACCUMULATE if accumulate else 0)
    flags |= {"auto": 0, "mega": A.FLAG_MEGAKERNEL, "wavefront": A.FLAG_WAVEFRONT}[mode]
    flags |= A.FLAG_DETERMINISTIC if deterministic else 0
    flags |= A.FLAG_SHARED_DEVICE if shared else 0
    ic = integrator.c()
    A.check(A.lib().mh_render(h, C.byref(ic), seed, spp, spp_begin, spp_end, _ptr(film), flags,
                              C.byref(stats) if stats is not None else None))
    return film


def develop(scene: Scene, film, device=None):
    torch = _torch()
    dev = film.device.index or 0
    h = scene.handle(dev, torch.cuda.current_stream(dev).cuda_stream)
    ch = A.image_channels(scene.desc.sensor.pixel_format)
    out = torch.empty((scene.height, scene.width, ch), dtype=torch.float32, device=film.device)
    A.check(A.lib().mh_develop(h, _ptr(film.contiguous()), _ptr(out), A.FLAG_DEVICE_POINTERS | _NO_SYNC))
    return out


def prb_weights(scene: Scene, seed: int, spp: int, spp_begin=0, spp_end=0, device=None, deterministic=False,
                out=None):
    """The W image of render_backward (common.py:936-947): the filter weight
    sum of samples [spp_begin, spp_end) of every pixel, (H, W) on the device
    (into `out` when given, a contiguous float32 device tensor of H*W)."""
    torch = _torch()
    dev = _device_index(device)
    h = scene.handle(dev, torch.cuda.current_stream(dev).cuda_stream)
    if out is not None:
        if out.dtype != torch.float32 or not out.is_cuda or not out.is_contiguous() or \
                out.numel() != scene.height * scene.width:
            raise A.MitsubaHipError("prb_weights: out must be a contiguous float32 device tensor of H*W")
        w = out
    else:
        w = torch.empty((scene.height, scene.width), dtype=torch.float32, device=f"cuda:{dev}")
    A.check(A.lib().mh_prb_weights(h, seed, spp, spp_begin, spp_end, _ptr(w),
                                   A.FLAG_DEVICE_POINTERS | _NO_SYNC |
                                   (A.FLAG_DETERMINISTIC if deterministic else 0)))
    return w


# srgb_to_xyz (spectrum.h:396-402); row 1 is luminance (spectrum.h:431-434)
_SRGB_TO_XYZ = [[0.412453, 0.357580, 0.180423], [0.212671, 0.715160, 0.072169], [0.019334, 0.119193, 0.950227]]


def _grad_to_rgb(scene: Scene, grad_in):
    """Adjoint of the develop colour conversion: d loss / d (weighted rgb)
    from d loss / d image for luminance / xyz films (the 1/W factor is
    applied by mh_render_backward).  An alpha channel (rgba / ya / xyza) is
    a select of the ray validity mask, which carries no derivative: its
    gradient is dropped."""
    torch = _torch()
    fmt = scene.desc.sensor.pixel_format
    ch = A.image_channels(fmt)
    g = grad_in.reshape(scene.height, scene.width, ch)
    if A.pixel_has_alpha(fmt):
        g = g[..., :ch - 1]
    if fmt in (A.PIXEL_RGB, A.PIXEL_RGBA):
        return g.contiguous()
    M = torch.tensor(_SRGB_TO_XYZ, dtype=torch.float32, device=grad_in.device)
    if fmt in (A.PIXEL_Y, A.PIXEL_YA):
        return g * M[1]
    return g @ M


def render_backward(scene: Scene, params: SceneParameters, grad_in, keys: List[str],
                    integrator: Optional[Integrator] = None, seed: int = 0, spp: int = 0,
                    spp_begin: int = 0, spp_end: int = 0, weights=None,
                    stats: Optional[A.Stats] = None, mode: str = "auto", deterministic: bool = False,
                    shared: bool = False):
    """RBIntegrator.render_backward (ad/integrators/common.py:828-983).
    Returns a list of gradient tensors (one per key, same shape as the param).
    mode: 'auto' (wavefront single-traversal kernels when the keys are rgb
    constants and bitmaps of one channel count -- a bitmap's vertices are
    logged and scattered to its texels once the paths end -- else the
    per-lane primal + adjoint replay), 'mega' (per-lane
    single traversal) or 'replay' (per-lane primal + adjoint replay, the
    reference's own two-pass structure).
    deterministic: bit-reproducible rgb gradients on the fused wavefront (each
    path's sum reduced in a fixed order) and a fixed-order W splat.
    shared: another call runs on the device at the same time
    (MH_FLAG_SHARED_DEVICE, a performance hint; the result is unchanged up to
    float summation order)."""
    torch = _torch()
    integrator = integrator or scene.integrator()
    if integrator.type not in ("prb", "prbvolpath"):
        raise A.MitsubaHipError("render_backward(): requires the 'prb' or 'prbvolpath' integrator")
    spp = spp or scene.sample_count()
    dev = grad_in.device.index or 0
    h = scene.handle(dev, torch.cuda.current_stream(dev).cuda_stream)
    grad_in = _grad_to_rgb(scene, grad_in.to(torch.float32)).contiguous()
    tex = (C.c_uint32 * max(len(keys), 1))(*[params.param_id(k) for k in keys])
    outs = [torch.zeros(params[k].shape, dtype=torch.float32, device=grad_in.device) for k in keys]
    ptrs = (C.c_void_p * max(len(keys), 1))(*[o.data_ptr() for o in outs])
    ic = integrator.c()
    A.check(A.lib().mh_render_backward(
        h, C.byref(ic), seed, spp, spp_begin, spp_end, _ptr(grad_in),
        _ptr(weights) if weights is not None else None, len(keys), tex, ptrs,
        A.FLAG_DEVICE_POINTERS | _NO_SYNC | {"auto": 0, "mega": A.FLAG_MEGAKERNEL, "replay": A.FLAG_PRB_REPLAY}[mode]
        | (A.FLAG_DETERMINISTIC if deterministic else 0) | (A.FLAG_SHARED_DEVICE if shared else 0),
        C.byref(stats) if stats is not None else None))
    return outs


def render_forward(scene: Scene, params: SceneParameters, tangents: Dict[str, object],
                   integrator: Optional[Integrator] = None, seed: int = 0, spp: int = 0,
                   spp_begin: int = 0, spp_end: int = 0, stats: Optional[A.Stats] = None,
                   develop_image: bool = True, deterministic: bool = False):
    """RBIntegrator.render_forward (ad/integrators/common.py:696-826): the
    forward-mode derivative of the rendered image -- the gradient image --
    for the input tangents ``{key: tensor shaped like params[key]}`` (the
    reference reads them from ``dr.set_grad`` on ``params``).  Returns the
    developed (H, W, C) image, or the un-developed film with
    ``develop_image=False`` (slab renders are summed before developing).  As
    film.develop() in the reference, an alpha film's alpha channel holds
    the coverage, not a derivative."""
    torch = _torch()
    integrator = integrator or scene.integrator()
    if integrator.type not in ("prb", "prbvolpath"):
        raise A.MitsubaHipError("render_forward(): requires the 'prb' or 'prbvolpath' integrator")
    spp = spp or scene.sample_count()
    keys = list(tangents.keys())
    dev = _device_index(None)
    for k in keys:
        t = tangents[k]
        if hasattr(t, "device") and t.device.type == "cuda":
            dev = t.device.index or 0
            break
    h = scene.handle(dev, torch.cuda.current_stream(dev).cuda_stream)
    tans = []
    for k in keys:
        t = torch.as_tensor(tangents[k], dtype=torch.float32).to(f"cuda:{dev}").contiguous()
        if tuple(t.shape) != tuple(params[k].shape):
            raise A.MitsubaHipError(f"render_forward(): tangent of '{k}' has shape {tuple(t.shape)}, "
                                    f"expected {tuple(params[k].shape)}")
        tans.append(t)
    ids = (C.c_uint32 * max(len(keys), 1))(*[params.param_id(k) for k in keys])
    ptrs = (C.c_void_p * max(len(keys), 1))(*[t.data_ptr() for t in tans])
    film = torch.empty((scene.height, scene.width, A.film_channels(scene.desc.sensor.pixel_format)),
                       dtype=torch.float32, device=f"cuda:{dev}")
    ic = integrator.c()
    flags = A.FLAG_DEVICE_POINTERS | _NO_SYNC | (A.FLAG_DETERMINISTIC if deterministic else 0)
    A.check(A.lib().mh_render_forward(h, C.byref(ic), seed, spp, spp_begin, spp_end, len(keys), ids, ptrs,
                                      _ptr(film), flags, C.byref(stats) if stats is not None else None))
    return develop(scene, film) if develop_image else film


# ---------------------------------------------------------------------------
# mi.render with torch autograd (util.py:356-408, 512-625)
# ---------------------------------------------------------------------------
def _render_op():
    torch = _torch()

    class _RenderOp(torch.autograd.Function):
        @staticmethod
        def forward(ctx, scene, params, keys, integrator, seeds, spps, *values):
            ctx.scene, ctx.params, ctx.keys, ctx.integrator = scene, params, keys, integrator
            ctx.seeds, ctx.spps = seeds, spps
            ctx.value_devices = [v.device for v in values]
            film = render_film(scene, integrator, seeds[0], spps[0])
            return develop(scene, film)

        @staticmethod
        def backward(ctx, grad_out):
            grads = render_backward(ctx.scene, ctx.params, grad_out, ctx.keys, ctx.integrator,
                                    ctx.seeds[1], ctx.spps[1])
            grads = [g.to(d) for g, d in zip(grads, ctx.value_devices)]
            return (None, None, None, None, None, None, *grads)

        @staticmethod
        def jvp(ctx, *tangents_in):
            # _RenderOp.forward (util.py:386-395): render_forward at the
            # differential seed / spp, driven by torch.autograd.forward_ad
            tans = {k: t for k, t in zip(ctx.keys, tangents_in[6:]) if t is not None}
            return render_forward(ctx.scene, ctx.params, tans, ctx.integrator, ctx.seeds[1], ctx.spps[1])

    return _RenderOp


def _has_tangent(v) -> bool:
    """a forward-mode dual tensor (torch.autograd.forward_ad.make_dual)"""
    import torch.autograd.forward_ad as fwAD
    return fwAD.unpack_dual(v).tangent is not None


def render(scene: Scene, params: Optional[SceneParameters] = None, sensor: int = 0,
           integrator: Optional[Integrator] = None, seed: int = 0, seed_grad: int = 0,
           spp: int = 0, spp_grad: int = 0):
    """mi.render (util.py:512-625): returns an (H, W, 3) torch tensor on the device."""
    if sensor != 0:
        raise A.MitsubaHipError("hip_ad_rgb: only sensor index 0 is supported")
    if params is not None and not isinstance(params, SceneParameters):
        raise A.MitsubaHipError("params should be an instance of mi.SceneParameter!")
    integrator = integrator or scene.integrator()
    if integrator is None:
        raise A.MitsubaHipError("No integrator specified! Add an integrator in the scene "
                                "description or provide an integrator directly as argument.")
    spp = spp or scene.sample_count()
    if spp_grad == 0:
        spp_grad = spp
    if seed_grad == 0:
        seed_grad = sample_tea_32(seed, 1)[0]
    elif seed_grad == seed:
        raise A.MitsubaHipError("The primal and differential seed should be different to ensure "
                                "unbiased gradient computation!")
    keys = [k for k, v in params.items() if v.requires_grad or _has_tangent(v)] if params is not None else []
    if not keys:
        film = render_film(scene, integrator, seed, spp)
        return develop(scene, film)
    values = [params[k] for k in keys]
    return _render_op().apply(scene, params, keys, integrator, (seed, seed_grad), (spp, spp_grad), *values)


def render_1(scene: Scene, params: Optional[SceneParameters] = None, sensor: int = 0,
             integrator: Optional[Integrator] = None, seed: int = 0, seed_grad: int = 0,
             spp: int = 0, spp_grad: int = 0):
    """The fork's radiance-meter loop: every pixel's radiance summed into one
    Spectrum, normalised by 1 / (W H spp).  In an RGB variant (hip_ad_rgb
    mirrors llvm_ad_rgb) the two reference implementations differ:

    - the C++ SamplingIntegrator::render_1 (integrator.cpp:398-411), which
      `path` and `volpath` use, raises;
    - the Python ADIntegrator.render_1 (ad/integrators/common.py:113-196),
      which `prb` and `prbvolpath` inherit, renders the primal and then
      returns Spectrum(0) * nf: its accumulation exists for monochromatic and
      spectral modes only ("Never use render_1() in RGB mode", :180-181).

    The signature and argument checks are mi.render_1's (util.py:627-669):
    (scene, params, sensor, integrator, seed, seed_grad, spp, spp_grad).
    Returns a (3,) float32 tensor on the device for the AD integrators."""
    if params is not None and not isinstance(params, SceneParameters):
        raise A.MitsubaHipError("params should be an instance of mi.SceneParameter!")
    integrator = integrator or scene.integrator()
    if integrator is None:
        raise A.MitsubaHipError("No integrator specified! Add an integrator in the scene "
                                "description or provide an integrator directly as argument.")
    if not isinstance(sensor, int):
        raise A.MitsubaHipError("hip_ad_rgb: the sensor is given by its index (only sensor 0 exists)")
    if sensor != 0:
        raise A.MitsubaHipError("hip_ad_rgb: only sensor index 0 is supported")
    if seed_grad != 0 and seed_grad == seed:
        raise A.MitsubaHipError("The primal and differential seed should be different to ensure "
                                "unbiased gradient computation!")
    if integrator.type not in ("prb", "prbvolpath"):
        raise A.MitsubaHipError("This render loop only supports monochromatic and spectral modes!")
    torch = _torch()
    spp = spp or scene.sample_count()
    film = render_film(scene, integrator, seed, spp)  # the primal pass (common.py:141-153)
    nf = 1.0 / (scene.width * scene.height * spp)
    return torch.zeros(3, dtype=torch.float32, device=film.device) * nf
