#!/usr/bin/env python3
"""Phase split of the fused bounce kernels on the bench step (diagnostic build).

usage: tools/build_variant.sh bph -DMH_EXP_BPHASE
       MH_LIB=gpurun_exp/lib_bph.so python tools/bounce_phases.py [--steps 3]

Runs bench.py's step (path forward + prb backward, cornell_box 512^2 @ 256)
and prints, per kernel family and generating / not, the share of the waves'
s_memtime cycles in each phase of a bounce iteration (64 paths per wave):
state load (or ray generation), closest-hit packet trace, shade, compaction +
state store, shadow packet trace, tail; plus cycles per iteration.  The
instrumented kernels run somewhat slower than the release build; compare
shares within one build."""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mitsuba3-nasa_amd")]

PHASES = ["load/gen", "closest trace", "shade", "store", "shadow trace", "tail"]
SLOTS = 12  # per group: the 6 phases, iterations, prologue, 4 spare
GROUPS = ["k_wf_bounce<Gen>", "k_wf_bounce", "k_wf_bounce_prb<Gen>", "k_wf_bounce_prb"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--res", type=int, default=512)
    ap.add_argument("--spp", type=int, default=256)
    a = ap.parse_args()
    import torch
    import bench
    from mitsuba_hip import _abi
    from mitsuba_hip import distributed as D
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    w = bench.build_step(a.res, a.spp, 8, 0, 1, dev)
    fn = _abi.lib().mh_exp_bphase
    fn.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    buf = (C.c_ulonglong * (4 * SLOTS))()

    def step(i):
        return D.fwd_grad_step(w["ops"], w["slab"], i, with_grad=True, packed=True, fwd_slab=w["fwd_slab"])

    step(1000)
    torch.cuda.synchronize()
    fn(buf, 1)
    for i in range(a.steps):
        step(i)
    torch.cuda.synchronize()
    fn(buf, 1)
    out = {}
    for g, name in enumerate(GROUPS):
        v = [buf[g * SLOTS + k] for k in range(SLOTS)]
        tot = sum(v[:6])
        if not tot:
            continue
        iters = max(1, v[6])
        print(f"{name:24s} iterations {iters:9d}  cycles/iteration {tot / iters:8.0f}  prologue {v[7] / max(1, tot + v[7]):.3f}")
        names, vals = PHASES, v[:6]
        for p, x in zip(names, vals):
            print(f"    {p:15s} {x / tot:6.3f}  {x / iters:8.0f} cycles/iteration")
        out[name] = {"iterations": iters, "cycles_per_iteration": tot / iters,
                     "share": {p: x / tot for p, x in zip(names, vals)}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
