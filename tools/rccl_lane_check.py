#!/usr/bin/env python
"""The argmin exchange over RCCL on one GPU: a one-rank "nccl" process group
(init_process_group with device_id = cuda:0), then bench.py's lane pattern as it is written -- two lanes, each with
its own context, stream, outputs and int64 key buffer; a step fills its lane's keys, runs stage COST with the argmin
folded in (pcore_evaluate_select) on the lane's stream, and issues all_reduce(MIN, async_op=True) from that stream;
the lane's next step first waits on the work (work.wait() under the lane's stream) before it refills the buffer.
Every exchanged key buffer is compared with the keys of the same batch scored without any process group, and the
per-step time is measured with and without the exchange in the loop.  Prints one JSON line.

Run as its own process (nothing may touch the GPU before the process group is set up):
    python tools/rccl_lane_check.py [--steps 12] [--poses 2000]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

C3_NAMES = ["003_cracker_box", "005_tomato_soup_can", "006_mustard_bottle", "010_potted_meat_can", "024_bowl"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--poses", type=int, default=2000, help="candidate poses per object")
    a = ap.parse_args()
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        os.environ.pop(k, None)
    import numpy as np
    import torch
    import torch.distributed as dist

    from perception_amd import distributed as pdist
    from perception_amd import workloads
    from perception_amd._native import PCORE_KEY_NONE

    torch.cuda.set_device(0)
    pdist.init_from_env(backend="nccl", force=True)
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1 and pdist.exchange_active()

    w = workloads.build(names=C3_NAMES, poses_per_model=a.poses)
    n = int(w.poses.shape[0])
    dev = w.poses.device
    # the keys of the batch without any collective (pcore_evaluate + pcore_select on the default stream)
    ref = torch.full((w.num_models,), PCORE_KEY_NONE, dtype=torch.int64, device=dev)
    out0 = tuple(torch.empty(n, dtype=torch.float32, device=dev) for _ in range(3))
    workloads.step(w, out0, ref)
    ref = ref.cpu().numpy()

    L = 2
    lanes = workloads.lanes(w, L)
    outs = [tuple(torch.empty(n, dtype=torch.float32, device=dev) for _ in range(3)) for _ in range(L)]
    keys_ring = [torch.full((w.num_models,), PCORE_KEY_NONE, dtype=torch.int64, device=dev) for _ in range(L)]
    snaps = [torch.empty(w.num_models, dtype=torch.int64, device=dev) for _ in range(a.steps)]

    def run(exchange):
        works = [None] * L
        got = []
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            b = i % L
            core, st = lanes[b]
            if works[b] is not None:
                with torch.cuda.stream(st):
                    works[b].wait()  # orders the lane's stream after its previous exchange
                    snaps[i - L].copy_(keys_ring[b])  # the exchanged keys of step i - L, before the refill
                    got.append(i - L)
            with torch.cuda.stream(st):
                keys_ring[b].fill_(PCORE_KEY_NONE)
                core.evaluate(w.poses, w.pose_model, w.pose_label, w.pose_obs_total, stride=w.stride, out=outs[b],
                              stream=st, select=(keys_ring[b], w.index_base, w.num_models))
                works[b] = pdist.allreduce_min_keys_async(keys_ring[b]) if exchange else None
        for b in range(L):
            i = a.steps - L + b
            core, st = lanes[i % L]
            with torch.cuda.stream(st):
                if works[i % L] is not None:
                    works[i % L].wait()
                snaps[i].copy_(keys_ring[i % L])
                got.append(i)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / a.steps, sorted(got)

    run(True)  # warm-up (RCCL communicator, tile tiers)
    ms_ex, got = run(True)
    ex_keys = [snaps[i].cpu().numpy() for i in got]
    ms_no, _ = run(False)
    ms_ex2, _ = run(True)
    equal = all(np.array_equal(k, ref) for k in ex_keys)
    res = {"backend": dist.get_backend(), "world_size": dist.get_world_size(), "device_id": "cuda:0",
           "steps": a.steps, "poses_per_step": n, "lanes": L, "exchanges_checked": len(ex_keys),
           "keys_equal_no_process_group": bool(equal), "keys": [int(k) for k in ref],
           "ms_per_step_with_exchange": [ms_ex, ms_ex2], "ms_per_step_without_exchange": ms_no,
           "torch": torch.__version__, "nccl_version": ".".join(map(str, torch.cuda.nccl.version()))}
    dist.destroy_process_group()
    print(json.dumps(res), flush=True)
    sys.exit(0 if equal else 1)


if __name__ == "__main__":
    main()
