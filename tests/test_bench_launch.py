"""bench.py's multi-GPU launch contract, CPU side: a WORLD_SIZE that disagrees with --gpus
exits non-zero, and `--gpus N` without a launcher refuses to start N RCCL ranks on fewer GPUs.  The N-rank run
itself is exercised on the GPU box (PCORE_DIST_BACKEND=gloo python bench.py --gpus 2)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, **env):
    e = dict(os.environ, **env)
    e.pop("PCORE_DIST_BACKEND", None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=e,
                          capture_output=True, text=True, timeout=300)


def test_world_size_disagreeing_with_gpus_exits_nonzero():
    r = _bench(["--gpus", "1"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2 and "WORLD_SIZE=2 but --gpus 1" in r.stderr
    r = _bench(["--gpus", "4"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2


def test_gpus_n_without_enough_devices_refuses_rccl_ranks():
    import torch

    if torch.cuda.device_count() >= 2:  # a multi-GPU host would really launch the ranks
        return
    r = _bench(["--gpus", "2", "--steps", "1"])
    assert r.returncode == 2 and "needs 2 GPUs" in r.stderr
