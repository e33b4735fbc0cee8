"""Rank worker of tests/test_gpu_multirank.py, launched by
`python -m torch.distributed.run --nproc-per-node 2 ...`: one bench step
(bench.build_step: the HIP C-ABI path, forward + W all-reduce + PRB
gradient) on this rank's sample slab, every rank on cuda:0 over gloo (the
driver's N-GPU run uses one device per rank over RCCL).  Saves the
all-reduced image and gradient to <out>/r<rank>.npz."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mitsuba3-nasa_amd")]


def main():
    out, res, spp = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    import numpy as np
    import torch
    import torch.distributed as dist
    import bench
    from mitsuba_hip import distributed as D
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    w = bench.build_step(res, spp, 6, rank, world, torch.device("cuda:0"))
    # a warm-up step first, as bench.py runs them: the step's film tensor is
    # reused, each call stream-ordered behind the previous step's develop
    D.fwd_grad_step(w["ops"], w["slab"], seed=3)
    img, grads = D.fwd_grad_step(w["ops"], w["slab"], seed=11)
    # the same step with every rank computing the whole W image itself (no W
    # all-reduce; mh_render_backward's in-call W) and the film summed onto
    # rank 0 only
    img2, grads2 = D.fwd_grad_step(w["ops"], w["slab"], seed=11, local_weights=True, film_to_root=True)
    # bench.py's default: film + W in one packed all-reduce (StepOps.packed views)
    img3, grads3 = D.fwd_grad_step(w["ops"], w["slab"], seed=11, packed=True, fwd_slab=w["fwd_slab"])
    img3, g3 = img3.clone(), grads3[0].clone()
    # bench.py's default since round 6: forward || gradient pass on two scene
    # handles and streams, W all-reduce, film + gradient in one all-reduce
    img4, grads4 = D.fwd_grad_step(w["ops"], w["slab"], seed=11, overlap=True, fwd_slab=w["fwd_slab"])
    torch.cuda.synchronize()
    t = D.max_over_ranks(float(rank) + 0.25, torch.device("cuda:0"))
    np.savez(os.path.join(out, f"r{rank}.npz"), img=img.cpu().numpy(), g=grads[0].cpu().numpy(), t=t,
             begin=w["slab"].begin, end=w["slab"].end, img2=img2.cpu().numpy(), g2=grads2[0].cpu().numpy(),
             img3=img3.cpu().numpy(), g3=g3.cpu().numpy(), img4=img4.cpu().numpy(), g4=grads4[0].cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
