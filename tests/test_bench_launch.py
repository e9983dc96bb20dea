"""bench.py --gpus N starts its own N ranks (one process per GPU) when no
launcher did, before any GPU call; under a launcher it checks WORLD_SIZE.
The frame sharding it drives follows frame.rs:232-237 (frames are
independent) and src/main.rs:43-53 (outputs concatenated in frame order)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _dry(n, extra=(), env=None):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--dry-run-launch",
                          *extra], capture_output=True, text=True, env=e, timeout=120)
    return out


@pytest.mark.parametrize("n", [2, 8])
def test_launch_command_for_n_ranks(n):
    out = _dry(n, ["--steps", "3", "--warmup", "1"])
    assert out.returncode == 0, out.stderr
    line = json.loads(out.stdout.strip().splitlines()[-1])
    cmd = line["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == str(n)
    assert cmd[cmd.index("--nnodes") + 1] == "1"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert int(cmd[cmd.index("--master-port") + 1]) > 0
    script = [c for c in cmd if c.endswith("bench.py")]
    assert script and os.path.samefile(script[0], os.path.join(ROOT, "bench.py"))
    rest = cmd[cmd.index(script[0]) + 1:]
    # the children get the same arguments, without the dry-run switch
    assert rest == ["--gpus", str(n), "--steps", "3", "--warmup", "1"]
    assert line["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_one_gpu_runs_in_process():
    sys.path.insert(0, ROOT)
    import bench
    env = os.environ.pop("WORLD_SIZE", None)
    try:
        assert bench.maybe_launch(["--gpus", "1", "--steps", "2"]) is None
        assert bench.maybe_launch([]) is None
    finally:
        if env is not None:
            os.environ["WORLD_SIZE"] = env


def test_under_a_launcher_world_must_match():
    sys.path.insert(0, ROOT)
    import bench
    old = os.environ.get("WORLD_SIZE")
    try:
        os.environ["WORLD_SIZE"] = "8"
        assert bench.maybe_launch(["--gpus", "8"]) is None
        with pytest.raises(AssertionError):
            bench.maybe_launch(["--gpus", "4"])
    finally:
        if old is None:
            os.environ.pop("WORLD_SIZE", None)
        else:
            os.environ["WORLD_SIZE"] = old
