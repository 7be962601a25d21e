"""bench.py's multi-GPU launch contract: `--gpus N > 1`
without a launcher starts N ranks itself under torch.distributed.run (a child
process, before anything touches a GPU); a launcher whose WORLD_SIZE is not
--gpus makes bench.py exit non-zero instead of reporting a 1-rank run as N
GPUs.  CPU only: nothing here renders."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402  (module import: no torch, no GPU)


def test_launcher_command():
    cmd = bench.launcher_command(8, ["--gpus", "8", "--steps", "5"], 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd
    assert cmd[cmd.index("--nproc-per-node") + 1] == "8"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29555"
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "5"]


def test_world_check():
    assert bench.world_check(1, {}) is None
    assert bench.world_check(2, {}) == "launch"
    assert bench.world_check(8, {"WORLD_SIZE": "8"}) is None
    assert bench.world_check(1, {"WORLD_SIZE": "1"}) is None
    assert "WORLD_SIZE 1" in bench.world_check(8, {"WORLD_SIZE": "1"})
    assert "WORLD_SIZE 4" in bench.world_check(1, {"WORLD_SIZE": "4"})
    assert "not an integer" in bench.world_check(2, {"WORLD_SIZE": "x"})


def test_world_size_mismatch_exits_nonzero():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 2
    assert "--gpus 2 but WORLD_SIZE 1" in p.stderr
    assert p.stdout == ""
