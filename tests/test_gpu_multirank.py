"""The N > 1 path of bench.py on one GPU: 2 ranks (torch.distributed.run,
gloo, both on cuda:0) through the real HIP StepOps (bench.build_step), vs the
single-process HIP result of the same sample set.  Sample-slab sharding
(SURVEY.md §8(e)): rank r renders samples [8 r, 8 r + 8) of a 16-spp render
with unchanged lane indices, so the all-reduced film / W / gradient equal the
one-process run up to float summation order."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_ranks_on_one_gpu_match_single_process(tmp_path):
    import torch
    sys.path[:0] = [ROOT]
    import bench
    from mitsuba_hip import distributed as D
    res, spp = 48, 8
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="2")
    logs = tmp_path / "logs"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", f"--log-dir={logs}", "--redirects=3",
           os.path.join(ROOT, "tests", "dist_hip_worker.py"), str(tmp_path), str(res), str(spp)]
    r = subprocess.run(cmd, env=env, cwd=ROOT, timeout=100, capture_output=True, text=True)
    if r.returncode != 0:
        # every rank's full stdout / stderr (torchrun --redirects 3), kept under
        # gpurun_out/ on the GPU box so a failure's whole log survives the run
        text = []
        for f in sorted(logs.rglob("*.log")):
            text.append(f"=== {f.relative_to(logs)} ===\n" + f.read_text(errors="replace"))
        text.append("=== launcher ===\n" + r.stdout + r.stderr)
        full = "\n".join(text)
        keep = os.environ.get("GRAFT_REPO_ROOT")
        if keep:
            os.makedirs(os.path.join(keep, "gpurun_out"), exist_ok=True)
            with open(os.path.join(keep, "gpurun_out", "multirank_failure.log"), "w") as fh:
                fh.write(full)
        pytest.fail(full[-6000:])
    r0, r1 = (np.load(tmp_path / f"r{i}.npz") for i in range(2))
    assert (int(r0["begin"]), int(r0["end"]), int(r1["begin"]), int(r1["end"])) == (0, 8, 8, 16)
    assert float(r0["t"]) == float(r1["t"]) == 1.25  # max over ranks
    np.testing.assert_array_equal(r0["img"], r1["img"])
    np.testing.assert_array_equal(r0["g"], r1["g"])
    w = bench.build_step(res, 2 * spp, 6, 0, 1, torch.device("cuda:0"))
    img, grads = D.fwd_grad_step(w["ops"], w["slab"], seed=11)
    img, g = img.cpu().numpy(), grads[0].cpu().numpy()
    assert img.mean() > 0 and np.abs(g).min() > 0
    np.testing.assert_allclose(r0["img"], img, rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(r0["g"], g, rtol=1e-4)
    # local W + film to rank 0 (tests/dist_hip_worker.py's second step)
    np.testing.assert_allclose(r0["img2"], img, rtol=1e-5, atol=1e-7)
    np.testing.assert_array_equal(r0["g2"], r1["g2"])
    np.testing.assert_allclose(r0["g2"], g, rtol=1e-4)
    # the packed film + W all-reduce (bench.py's default step)
    for r in (r0, r1):
        np.testing.assert_allclose(r["img3"], img, rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(r["g3"], g, rtol=1e-4)
    # the overlapped step (bench.py's default): forward || gradient pass
    for r in (r0, r1):
        np.testing.assert_allclose(r["img4"], img, rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(r["g4"], g, rtol=1e-4)
    # ... and on one process: the same image and gradient as the serial step
    img5, grads5 = D.fwd_grad_step(w["ops"], w["slab"], seed=11, overlap=True)
    np.testing.assert_allclose(img5.cpu().numpy(), img, rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(grads5[0].cpu().numpy(), g, rtol=1e-4)
