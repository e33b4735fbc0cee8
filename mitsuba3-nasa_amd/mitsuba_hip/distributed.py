"""Multi-GPU orchestration of the hot path.

Sample-slab sharding: with N ranks and `spp` samples per pixel per rank, rank
r renders samples [spp*r, spp*(r+1)) of EVERY pixel of a render at spp*N
samples per pixel.  The global lane index idx = pixel * spp_total + s (and so
the TEA seed of every lane, integrator.cpp:323-340) is the one the single-GPU
render uses, hence the union of the slabs is sample-identical to it.  The
only coupling is additive:

  forward   film (H, W, 4) RGBW                 -> all-reduce(sum) (or reduce to rank 0), develop
  PRB       W image (H, W) of render_backward   -> all-reduce(sum) before the
            dL gather (common.py:936-947), then each rank's gradient slab
            -> all-reduce(sum)

The W image depends only on the gradient seed's pixel jitters, not on the
forward's radiance, so a step can compute it before the forward exchange and
sum film and W in ONE collective (`packed`, the default of bench.py): one
all-reduce of film + W (5 MiB at 512², 80 MiB at 2048²) and one of the
gradients (12 B per rgb parameter) per step.  Unpacked, the film is reduced
(or all-reduced) and W all-reduced separately, or W is computed locally on
every rank (local_weights: no W exchange, N times the W splat).

Overlapped (`overlap`, the default of bench.py since round 6): the forward
and the gradient pass are independent, so they run concurrently on two scene
handles and two streams (PairRunner), after the W image and its
all-reduce; the film and the gradients are summed in one all-reduce after
both (W: 1 MiB, film + gradient: 4 MiB + 12 B at 512²).

One process per GPU; torch.distributed with backend "nccl" (= RCCL over xGMI
on ROCm), or "gloo" for the CPU tests.  No collective sits inside a kernel
loop.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, List, Optional


@dataclass
class Slab:
    spp_total: int
    begin: int
    end: int


def sample_slab(rank: int, world: int, spp_per_rank: int) -> Slab:
    if not (0 <= rank < world) or spp_per_rank <= 0:
        raise ValueError("sample_slab: bad rank / world / spp")
    return Slab(spp_per_rank * world, spp_per_rank * rank, spp_per_rank * (rank + 1))


def _dist():
    import torch.distributed as dist
    return dist if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1 else None


class CollTimer:
    """Times the step's collectives (bench.py at N > 1, so that a scaling
    result can be split into collective cost, imbalance and launch tail):
    per collective its name, its bytes and its duration -- HIP events on the
    current stream around a device tensor's collective (the stream waits for
    the collective before it records the second event), host time around a
    CPU tensor's."""

    def __init__(self):
        self.records = []  # (name, bytes, start, end, device)

    def run(self, name: str, t, fn):
        import time
        import torch
        if t.is_cuda:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            self.records.append((name, t.numel() * t.element_size(), e0, e1, True))
        else:
            t0 = time.perf_counter()
            fn()
            self.records.append((name, t.numel() * t.element_size(), t0, time.perf_counter(), False))

    def summary(self, steps: int) -> dict:
        """{name: {ms_per_step, bytes, calls_per_step}} over the recorded calls; resets."""
        import torch
        if any(r[4] for r in self.records):
            torch.cuda.synchronize()
        out = {}
        for name, nb, a, b, dev in self.records:
            ms = a.elapsed_time(b) if dev else (b - a) * 1e3
            o = out.setdefault(name, {"ms_per_step": 0.0, "bytes": nb, "calls_per_step": 0.0})
            o["ms_per_step"] += ms / max(1, steps)
            o["calls_per_step"] += 1.0 / max(1, steps)
        self.records = []
        return out


_timer: Optional[CollTimer] = None


def set_collective_timer(t: Optional[CollTimer]):
    """Route every collective of this module through t (None: untimed)."""
    global _timer
    _timer = t


def _coll(name: str, t, fn):
    if _timer is not None:
        _timer.run(name, t, fn)
    else:
        fn()


def all_reduce_(t, name: str = "all_reduce"):
    """In-place sum over ranks (no-op on one rank)."""
    d = _dist()
    if d is not None:
        _coll(name, t, lambda: d.all_reduce(t))
    return t


def reduce_to_root_(t, name: str = "reduce"):
    """In-place sum onto rank 0 (no-op on one rank); the other ranks' tensor
    is left undefined, as a reduce leaves it."""
    d = _dist()
    if d is not None:
        if t.is_cuda and d.get_backend() == "gloo":
            # gloo reduces device tensors only by all-reduce; rank 0 gets the same sum
            _coll(name, t, lambda: d.all_reduce(t))
        else:
            _coll(name, t, lambda: d.reduce(t, dst=0))
    return t


@dataclass
class StepOps:
    """The hot-path entry points one step calls (the C-ABI wrappers of
    mitsuba_hip.render on a GPU; the tests substitute the CPU oracle)."""
    render_film: Callable      # (seed, spp_total, begin, end) -> film tensor (H, W, 4)
    develop: Callable          # (film) -> image (H, W, 3)
    prb_weights: Callable      # (seed, spp_total, begin, end) -> W (H, W)
    render_backward: Callable  # (seed, spp_total, begin, end, weights) -> [grad tensors]; weights None:
                               # the W image of every sample computed in-call (local W)
    seed_grad: Callable        # (seed) -> seed of the differential pass (TEA(seed, 1).v0)
    # optional: () -> (buffer, film view, W view), one device buffer holding the
    # film and the W image; render_film / prb_weights then take out= (their
    # output view), so the packed exchange needs no copy.  None: the packed
    # step concatenates the two.
    packed: Optional[Callable] = None
    # optional: (fwd, bwd) -> (fwd(), bwd()) with the two running concurrently
    # (a PairRunner; on a GPU render_film then uses its own scene handle and
    # stream).  None: the overlapped step runs them one after the other.
    concurrent: Optional[Callable] = None
    # render_film / render_backward take shared=True: the overlapped step passes
    # the MH_FLAG_SHARED_DEVICE hint (each call's launches sized for a share
    # of the device)
    shared_hint: bool = False


class PairRunner:
    """Runs `fwd` on a worker thread concurrently with `bwd` on the calling
    thread and returns (fwd(), bwd()).  The C-ABI calls release the GIL, so
    the forward's and the backward's kernels overlap on the device (distinct
    scene handles may be used concurrently, include/mitsuba_hip.h).

    streams = (stream_fwd, stream_bwd) on `device`: each side runs with its
    stream current; both wait for the caller's current stream first, the
    caller's stream waits for both on return, and returned device tensors are
    marked as used on the caller's stream (the caching allocator must not
    reuse them early).  None: host threads only (the CPU tests)."""

    def __init__(self, streams=None, device=None):
        from concurrent.futures import ThreadPoolExecutor
        self.pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="mh-fwd")
        self.streams, self.device = streams, device

    def __call__(self, fwd: Callable, bwd: Callable):
        if self.streams is None:
            fut = self.pool.submit(fwd)
            try:
                b = bwd()
            finally:
                fut.exception()  # joins the forward whatever the backward did
            return fut.result(), b
        import torch
        sa, sb = self.streams
        cur = torch.cuda.current_stream(self.device)
        sa.wait_stream(cur)
        sb.wait_stream(cur)

        def run_fwd():
            torch.cuda.set_device(self.device)  # the current device is per host thread
            with torch.cuda.stream(sa):
                return fwd()

        fut = self.pool.submit(run_fwd)
        try:
            with torch.cuda.stream(sb):
                b = bwd()
        finally:
            fut.exception()  # joins the forward whatever the backward did
        a = fut.result()
        cur.wait_stream(sa)
        cur.wait_stream(sb)
        for t in ([a] if torch.is_tensor(a) else list(a or [])) + ([b] if torch.is_tensor(b) else list(b or [])):
            if torch.is_tensor(t) and t.is_cuda:
                t.record_stream(cur)
        return a, b


def all_reduce_list_(ts: List, name: str = "all_reduce") -> List:
    """Sum a list of tensors over ranks in ONE collective (concatenated when
    there are several); returns the summed tensors (in place for one)."""
    d = _dist()
    if d is None or not ts:
        return ts
    if len(ts) == 1:
        _coll(name, ts[0], lambda: d.all_reduce(ts[0]))
        return ts
    import torch
    flat = torch.cat([t.reshape(-1) for t in ts])
    _coll(name, flat, lambda: d.all_reduce(flat))
    out, o = [], 0
    for t in ts:
        out.append(flat[o:o + t.numel()].view_as(t))
        o += t.numel()
    return out


def fwd_grad_step(ops: StepOps, slab: Slab, seed: int, with_grad: bool = True, local_weights: bool = False,
                  film_to_root: bool = False, packed: bool = False, fwd_slab: Optional[Slab] = None,
                  overlap: bool = False):
    """One benchmark step: forward render of the rank's slab + film
    all-reduce + develop; then (with_grad) PRB render_backward of the slab
    with the globally all-reduced W image and an all-reduced gradient.

    overlap: the forward and the gradient pass are independent (the
    backward's seed is TEA(seed, 1); it needs the W image, not the film), so
    after the W image and its all-reduce they run concurrently
    (ops.concurrent): the forward on one side, render_backward on the other;
    then the film and the gradients are summed in ONE all-reduce (two
    collectives per step: W, film + gradient; one with local_weights).
    film_to_root does not apply.

    packed: the W image of the gradient seed is computed before the forward
    exchange and summed together with the film in one all-reduce (two
    collectives per step: film + W, gradients).
    local_weights: every rank computes the whole W image itself (all
    spp_total samples of every pixel) instead of its slab's W + an
    all-reduce -- one collective fewer for N times the W splat work.
    film_to_root: the film is summed onto rank 0 only (a reduce, not an
    all-reduce); only rank 0's image is then defined.
    fwd_slab: the forward's slab when it differs from the gradient's (a
    multi-pass forward counts its slab in lanes of one pass)."""
    fs = fwd_slab or slab
    if with_grad and overlap:
        sg = ops.seed_grad(seed)
        # W and its all-reduce first, so that no collective runs while the two
        # passes share the device (an RCCL kernel queued behind the forward's
        # launches would hold its peers' kernels spinning); the W splat fills
        # the chip by itself
        w = None if local_weights else all_reduce_(ops.prb_weights(sg, slab.spp_total, slab.begin, slab.end), "W")
        run = ops.concurrent or (lambda f, g: (f(), g()))
        kw = {"shared": True} if (ops.shared_hint and ops.concurrent is not None) else {}
        film, grads = run(lambda: ops.render_film(seed, fs.spp_total, fs.begin, fs.end, **kw),
                          lambda: ops.render_backward(sg, slab.spp_total, slab.begin, slab.end, w, **kw))
        summed = all_reduce_list_([film] + list(grads), "film+gradient")
        return ops.develop(summed[0]), summed[1:]
    if with_grad and packed and not local_weights:
        sg = ops.seed_grad(seed)
        if ops.packed is not None:
            buf, fv, wv = ops.packed()
            film = ops.render_film(seed, fs.spp_total, fs.begin, fs.end, out=fv)
            w = ops.prb_weights(sg, slab.spp_total, slab.begin, slab.end, out=wv)
            all_reduce_(buf, "film+W")  # film + W: one collective
        else:
            film = ops.render_film(seed, fs.spp_total, fs.begin, fs.end)
            w = ops.prb_weights(sg, slab.spp_total, slab.begin, slab.end)
            film, w = all_reduce_list_([film, w], "film+W")
        img = ops.develop(film)
        grads: List = ops.render_backward(sg, slab.spp_total, slab.begin, slab.end, w)
        return img, all_reduce_list_(grads, "gradient")
    film = ops.render_film(seed, fs.spp_total, fs.begin, fs.end)
    film = reduce_to_root_(film, "film") if film_to_root else all_reduce_(film, "film")
    img = ops.develop(film)
    if not with_grad:
        return img, None
    sg = ops.seed_grad(seed)
    w = None if local_weights else all_reduce_(ops.prb_weights(sg, slab.spp_total, slab.begin, slab.end), "W")
    grads = ops.render_backward(sg, slab.spp_total, slab.begin, slab.end, w)
    return img, all_reduce_list_(grads, "gradient")


def max_over_ranks(x: float, device=None) -> float:
    """Max of a host float over ranks (the bench's step time)."""
    d = _dist()
    if d is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64, device=device)
    d.all_reduce(t, op=d.ReduceOp.MAX)
    return float(t.item())


def min_over_ranks(x: float, device=None) -> float:
    """Min of a host float over ranks (the per-rank spread of the step time)."""
    d = _dist()
    if d is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64, device=device)
    d.all_reduce(t, op=d.ReduceOp.MIN)
    return float(t.item())
