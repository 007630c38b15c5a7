"""N > 1 path on CPU: world_size-2 gloo ranks each select over their pose shard; one all-reduce(MIN)
of the int64 keys must equal the single-process selection over all poses.  The bench's
pipelined form (two batches' exchanges in flight at once, allreduce_min_keys_async) must give the same."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, rc, oc, pm, K, q, rc2=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist

    import oracle
    from perception_amd.core import decode_keys, encode_key
    from perception_amd.distributed import allreduce_min_keys, allreduce_min_keys_async, init_from_env, shard_range

    init_from_env("gloo")
    lo, hi = shard_range(len(rc), rank, world)

    def local_keys(r):
        cost, idx = oracle.select(r[lo:hi], oc[lo:hi], pm[lo:hi], K, index_base=lo)
        return torch.tensor([encode_key(int(c), int(i)) for c, i in zip(cost, idx)], dtype=torch.int64)

    keys = local_keys(rc)
    allreduce_min_keys(keys)
    # pipelined: both batches' exchanges in flight before either is waited on
    ka, kb = local_keys(rc), local_keys(rc2)
    wa, wb = allreduce_min_keys_async(ka), allreduce_min_keys_async(kb)
    wa.wait()
    wb.wait()
    q.put((rank, decode_keys(keys), decode_keys(ka), decode_keys(kb)))
    dist.destroy_process_group()


def test_gloo_world2_argmin_equals_single_process():
    rng = np.random.default_rng(3)
    n, K = 1001, 3
    rc = rng.integers(0, 40, n).astype(np.float32)
    oc = rng.integers(0, 40, n).astype(np.float32)
    rc[rng.integers(0, n, 30)] = -1.0
    pm = rng.integers(0, K, n).astype(np.int32)
    import oracle

    rc2 = rng.permutation(rc)
    ref_cost, ref_idx = oracle.select(rc, oc, pm, K)
    ref2 = oracle.select(rc2, oc, pm, K)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, rc, oc, pm, K, q, rc2)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, (cost, idx), (ca, ia), (cb, ib) in res:
        assert np.array_equal(cost, ref_cost) and np.array_equal(idx, ref_idx)
        assert np.array_equal(ca, ref_cost) and np.array_equal(ia, ref_idx)
        assert np.array_equal(cb, ref2[0]) and np.array_equal(ib, ref2[1])


def _forced_worker(q):
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        os.environ.pop(k, None)
    import torch
    import torch.distributed as dist

    from perception_amd.distributed import allreduce_min_keys_async, exchange_active, init_from_env

    init_from_env("gloo")  # world 1, not forced: no process group
    before = dist.is_initialized()
    init_from_env("gloo", force=True)
    keys = torch.tensor([5, -3, 2 ** 62], dtype=torch.int64)
    work = allreduce_min_keys_async(keys)
    ok = work is not None
    if ok:
        work.wait()
    q.put((before, dist.is_initialized(), dist.get_world_size(), exchange_active(), ok, keys.tolist()))
    dist.destroy_process_group()


def test_forced_one_rank_process_group_runs_the_exchange():
    """bench.py --force-pg / PCORE_FORCE_PG=1: at world size 1 init_from_env starts a one-rank group only when forced,
    and the exchange then runs (a work handle, keys unchanged by a MIN over one rank)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_forced_worker, args=(q,))
    p.start()
    before, inited, world, active, ok, keys = q.get(timeout=120)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert not before and inited and world == 1 and active and ok
    assert keys == [5, -3, 2 ** 62]
