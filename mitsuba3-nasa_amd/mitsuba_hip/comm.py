"""Multi-GPU through the C ABI: RCCL communicators and the sharded entry
points of include/mitsuba_hip.h ("Multi-GPU").

This is the torch-free path of the sample-slab split: a host (a C++ plugin,
or this module) owns the communicator and the library sums films, W images
and gradients itself.  `mitsuba_hip.distributed` keeps the torch.distributed
orchestration that bench.py uses; both compute the same slabs.

  Comm.unique_id()                  rank 0 makes the id, ships it to the others
  Comm(uid, nranks, rank, device)   one rank per process / thread
  Comm.create_all([0, 1, ...])      one thread drives every device
  comm.reduce_(tensor, root=-1)     in-place sum over the ranks
  scene_set_comm(scene, comm)       MH_FLAG_REDUCE for the scene's entry points
  render_sharded / render_backward_sharded
                                    one host thread, one slab per scene
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence

from . import _abi as A


class Comm:
    """One rank of an RCCL communicator bound to one device (mh_comm)."""

    def __init__(self, uid: bytes, nranks: int, rank: int, device: int = 0, _handle=None):
        self._h = C.c_void_p()
        if _handle is not None:
            self._h = _handle
        else:
            if len(uid) != A.COMM_ID_BYTES:
                raise A.MitsubaHipError(f"Comm: the unique id has {len(uid)} bytes, expected {A.COMM_ID_BYTES}")
            A.check(A.lib().mh_comm_create(uid, nranks, rank, device, C.byref(self._h)))

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(A.COMM_ID_BYTES)
        A.check(A.lib().mh_comm_unique_id(buf))
        return buf.raw

    @classmethod
    def create_all(cls, devices: Sequence[int]) -> List["Comm"]:
        n = len(devices)
        hs = (C.c_void_p * n)()
        devs = (C.c_int * n)(*devices)
        A.check(A.lib().mh_comm_create_all(n, devs, hs))
        return [cls(b"", 0, 0, _handle=C.c_void_p(hs[i])) for i in range(n)]

    @property
    def handle(self):
        return self._h

    def info(self):
        nr, r, d = C.c_int(), C.c_int(), C.c_int()
        A.check(A.lib().mh_comm_info(self._h, C.byref(nr), C.byref(r), C.byref(d)))
        return nr.value, r.value, d.value

    def reduce_(self, t, root: int = -1, stream=None):
        """Sum a float32 device tensor over the ranks, in place (root < 0:
        all-reduce; else reduce to that rank), ordered on `stream` (default:
        torch's current stream of the tensor's device)."""
        import torch
        if t.dtype != torch.float32 or not t.is_cuda or not t.is_contiguous():
            raise A.MitsubaHipError("Comm.reduce_: needs a contiguous float32 device tensor")
        st = stream if stream is not None else torch.cuda.current_stream(t.device).cuda_stream
        comms = (C.c_void_p * 1)(self._h.value)
        bufs = (C.c_void_p * 1)(t.data_ptr())
        sts = (C.c_void_p * 1)(st)
        A.check(A.lib().mh_comm_reduce(comms, 1, bufs, t.numel(), sts, root))
        return t

    def close(self):
        """Destroy the communicator.  The library refuses while a scene still
        holds it (mh_scene_set_comm); detach it first (scene_set_comm(scene,
        None)) or release the scene."""
        if self._h:
            A.check(A.lib().mh_comm_destroy(self._h))
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def scene_set_comm(scene, comm: Optional[Comm], device: int = 0):
    """Attach `comm` to the scene's handle on `device` (None: detach).  The
    scene keeps a reference to the Comm while it is attached, so the
    communicator cannot be destroyed under it."""
    A.check(A.lib().mh_scene_set_comm(scene.handle(device), comm.handle if comm is not None else None))
    held = scene.__dict__.setdefault("_comms", {})
    if comm is None:
        held.pop(device, None)
    else:
        held[device] = comm


def _devices(scenes, device) -> List[int]:
    """One device per scene: `device` is an int (every scene on it) or a list."""
    if isinstance(device, int):
        return [device] * len(scenes)
    if len(device) != len(scenes):
        raise A.MitsubaHipError("the device list needs one entry per scene")
    return list(device)


def _handles(scenes, devices):
    return (C.c_void_p * len(scenes))(*[s.handle(d).value for s, d in zip(scenes, devices)])


def render_sharded(scenes, integrator, seed: int, spp: int, films, device=0, reduce_all: bool = True,
                   deterministic: bool = False, stats=None):
    """mh_render_sharded: scene i renders the slab [spp*i/n, spp*(i+1)/n) of
    every pixel into films[i] (device tensors on scene i's device; `device`:
    one int for all scenes or one per scene); the films are summed into
    every film (reduce_all) or into films[0] only."""
    n = len(scenes)
    devs = _devices(scenes, device)
    ic = integrator.c()
    fp = (C.c_void_p * n)(*[f.data_ptr() for f in films])
    flags = A.FLAG_DEVICE_POINTERS | (A.FLAG_REDUCE if reduce_all else 0)
    flags |= A.FLAG_DETERMINISTIC if deterministic else 0
    st = (A.Stats * n)() if stats is not None else None
    A.check(A.lib().mh_render_sharded(_handles(scenes, devs), n, C.byref(ic), seed, spp, fp, flags, st))
    if stats is not None:
        stats[:] = list(st)
    return films


def render_backward_sharded(scenes, params, grad_in, keys, integrator, seed: int, spp: int, device=0,
                            local_weights: bool = False):
    """mh_render_backward_sharded: every scene differentiates its slab with
    the summed W image; returns per scene the list of summed gradients, each
    on that scene's device (`device`: one int for all scenes or one per
    scene; grad_in is copied to every scene's device)."""
    import torch
    n = len(scenes)
    devs = _devices(scenes, device)
    ic = integrator.c()
    gi = [grad_in.to(device=f"cuda:{d}", dtype=torch.float32).contiguous() for d in devs]
    gptr = (C.c_void_p * n)(*[g.data_ptr() for g in gi])
    ids = (C.c_uint32 * max(len(keys), 1))(*[params.param_id(k) for k in keys])
    outs = [[torch.zeros(params[k].shape, dtype=torch.float32, device=f"cuda:{d}") for k in keys]
            for d in devs]
    optr = (C.c_void_p * max(n * len(keys), 1))(*[o.data_ptr() for row in outs for o in row])
    flags = A.FLAG_DEVICE_POINTERS | (A.FLAG_LOCAL_WEIGHTS if local_weights else 0)
    A.check(A.lib().mh_render_backward_sharded(_handles(scenes, devs), n, C.byref(ic), seed, spp, gptr,
                                               len(keys), ids, optr, flags, None))
    return outs
