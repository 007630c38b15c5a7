"""The multi-GPU exchange with the product kernels, on the GPU box: world-size-2 gloo ranks (both on cuda:0 --
the pool gives one GPU; RCCL refuses two ranks on one device) each score their contiguous shard of the C2 batch
through pcore_evaluate, fold their keys with pcore_select (index_base = the shard's first global index) and meet in
allreduce_min_keys; the result equals the oracle's selection rule over the single-process costs of the whole
batch."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.multiprocessing as mp  # noqa: E402

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    import torch
    import torch.distributed as dist

    from perception_amd import workloads
    from perception_amd._native import PCORE_KEY_NONE
    from perception_amd.core import decode_keys
    from perception_amd.distributed import allreduce_min_keys, init_from_env, shard_range

    torch.cuda.set_device(0)
    init_from_env("gloo")
    w = workloads.build(poses_per_model=4000)  # the same batch on every rank
    n = int(w.poses.shape[0])
    lo, hi = shard_range(n, rank, world)
    rc, oc, _ = w.core.evaluate(w.poses[lo:hi], w.pose_model[lo:hi], w.pose_label[lo:hi], w.pose_obs_total[lo:hi],
                                stride=w.stride)
    keys = torch.full((w.num_models,), PCORE_KEY_NONE, dtype=torch.int64, device=rc.device)
    w.core.select(rc, oc, w.pose_model[lo:hi], w.num_models, index_base=lo, keys=keys)
    torch.cuda.synchronize()
    allreduce_min_keys(keys)
    q.put((rank, lo, hi, rc.cpu().numpy(), oc.cpu().numpy(), decode_keys(keys)))
    dist.destroy_process_group()


def test_gloo_world2_product_select_equals_oracle_rule():
    import oracle
    from perception_amd import workloads

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rc = np.concatenate([r[3] for r in res])
    oc = np.concatenate([r[4] for r in res])
    assert res[0][1] == 0 and res[0][2] == res[1][1]
    w = workloads.build(poses_per_model=4000)
    full_rc, full_oc, _ = w.core.evaluate(w.poses, w.pose_model, w.pose_label, w.pose_obs_total, stride=w.stride)
    assert np.array_equal(rc.view(np.uint32), full_rc.cpu().numpy().view(np.uint32))
    assert np.array_equal(oc.view(np.uint32), full_oc.cpu().numpy().view(np.uint32))
    ocost, oidx = oracle.select(rc, oc, w.pose_model.cpu().numpy(), w.num_models)
    for _, _, _, _, _, (cost, idx) in res:
        assert np.array_equal(cost, ocost) and np.array_equal(idx, oidx)
    assert int(oidx[0]) == w.gt_index[0]


def test_rccl_one_rank_lane_pattern_keys_equal_no_process_group():
    """the RCCL branch executes on the one-GPU box.  tools/rccl_lane_check.py runs in a fresh
    child process (started with subprocess: no exec, nothing touches the GPU before the process group exists):
    init_process_group("nccl", world 1, device_id cuda:0), then bench.py's lane pattern (two lanes, a ring of int64
    key buffers, all_reduce(MIN, async_op=True) issued from the lane's stream, work.wait() before a buffer is
    refilled).  Every exchanged key buffer equals the keys of the same batch scored with no process group."""
    import json
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, str(root / "tools" / "rccl_lane_check.py"), "--steps", "12", "--poses", "1000"],
                       cwd=root, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert res["backend"] == "nccl" and res["world_size"] == 1
    assert res["keys_equal_no_process_group"] and res["exchanges_checked"] == 12
    assert len(res["keys"]) == 5 and all(k != (2 ** 63 - 1) for k in res["keys"])
