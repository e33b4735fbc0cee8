"""CPU: `bench.py --gpus N` launches N ranks.  The
launcher must build a torch.distributed.run command for exactly N ranks on
127.0.0.1, make no GPU call before it hands over, and a rank under a launcher
must refuse a --gpus that disagrees with WORLD_SIZE."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_launch_command_for_n_ranks():
    argv = ["--gpus", "2", "--backend", "gloo", "--steps", "3"]
    cmd = bench.launch_command(argv, 2, env={})
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=2" in cmd and "--nnodes=1" in cmd and "--master-addr=127.0.0.1" in cmd
    port = [c for c in cmd if c.startswith("--master-port=")]
    assert len(port) == 1 and int(port[0].split("=")[1]) > 0
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == argv  # the ranks see the same arguments


def test_launch_command_keeps_master_port():
    cmd = bench.launch_command(["--gpus", "8"], 8, env={"MASTER_PORT": "29555"})
    assert "--master-port=29555" in cmd and "--nproc-per-node=8" in cmd


@pytest.mark.parametrize("gpus,env", [(None, {}), (1, {}), (2, {"WORLD_SIZE": "2"}), (8, {"WORLD_SIZE": "8"})])
def test_no_launch_for_one_gpu_or_inside_a_rank(gpus, env):
    assert bench.launch_command([], gpus, env=env) is None


def test_rank_checks_gpus_against_world_size():
    a = bench.parse(["--gpus", "4"])
    with pytest.raises(SystemExit):
        bench.world_from(a, env={"WORLD_SIZE": "2", "RANK": "1", "LOCAL_RANK": "1"})
    assert bench.world_from(a, env={"WORLD_SIZE": "4", "RANK": "3", "LOCAL_RANK": "3"}) == (4, 3, 3)
    assert bench.world_from(bench.parse([]), env={"WORLD_SIZE": "2", "RANK": "1", "LOCAL_RANK": "1"}) == (2, 1, 1)
    assert bench.world_from(bench.parse([]), env={}) == (1, 0, 0)


def test_launcher_process_makes_no_gpu_call(tmp_path):
    """Run bench.main() as the launcher with the child replaced by a recorder:
    the parent must exit with the child's code and never initialise HIP."""
    script = tmp_path / "run.py"
    script.write_text(
        "import sys, subprocess, json\n"
        f"sys.path.insert(0, {ROOT!r})\n"
        "import bench\n"
        "seen = {}\n"
        "def call(cmd, env=None):\n"
        "    seen['cmd'] = cmd; seen['addr'] = env.get('MASTER_ADDR'); return 7\n"
        "subprocess.call = call\n"
        "sys.argv = ['bench.py', '--gpus', '2', '--backend', 'gloo']\n"
        "try:\n"
        "    bench.main()\n"
        "except SystemExit as e:\n"
        "    seen['rc'] = e.code\n"
        "import torch\n"
        "seen['cuda_init'] = torch.cuda.is_initialized()\n"
        "print(json.dumps(seen))\n")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, env=env, timeout=300)
    assert out.returncode == 0, out.stderr
    import json
    seen = json.loads(out.stdout.strip().splitlines()[-1])
    assert seen["rc"] == 7 and seen["addr"] == "127.0.0.1" and not seen["cuda_init"]
    assert "--nproc-per-node=2" in seen["cmd"] and seen["cmd"][-4:] == ["--gpus", "2", "--backend", "gloo"]
