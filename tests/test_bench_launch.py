"""bench.py's launch contract (CPU only, nothing touches a GPU): `bench.py --gpus N` without a
launcher starts its N ranks itself under torch.distributed.run (one node, 127.0.0.1), and a rank
count that disagrees with --gpus is an error, never a silent one-GPU run."""
import json
import os
import pathlib
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent


def _run(args, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env)
    return subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, cwd=ROOT, env=e,
                          capture_output=True, text=True, timeout=120)


def test_gpus_n_without_launcher_starts_n_ranks():
    r = _run(["--gpus", "8", "--steps", "3", "--warmup", "2"], SGN_BENCH_LAUNCH_DRY="1")
    assert r.returncode == 0, r.stderr
    cmd = json.loads(r.stdout.strip().splitlines()[-1])
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert int(cmd[cmd.index("--master-port") + 1]) > 0
    i = cmd.index(str(ROOT / "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "3", "--warmup", "2"]


def test_gpus_disagreeing_with_world_size_is_an_error():
    r = _run(["--gpus", "2"], WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2
    assert "--gpus 2 but WORLD_SIZE=1" in r.stderr
    r = _run(["--gpus", "1"], WORLD_SIZE="4", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2
