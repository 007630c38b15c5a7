#!/usr/bin/env python
"""Benchmark of the render-and-compare hot path (BASELINE.json metric, config C2 per GPU).

One step = one pass of the hot path over one batch: render + unproject + 1-NN + score 10k 6-DoF
candidate poses of the 003_cracker_box proxy at 640x480 (stride 8, no ICP) and fold the per-model argmin
keys; with N > 1 GPUs every rank scores its own 10k-pose shard (weak scaling) and the keys meet in one
RCCL all-reduce(MIN).  Inputs are resident in HBM before the timed region.  Two batches are in flight per GPU
(core.PoseLanes: consecutive steps alternate over two contexts on two HIP streams, so one step's drain overlaps
the next step's fill; every step is still one full 10k-pose batch and completes inside the timed region).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--poses P] [--cpu-seconds S]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 --master-port P bench.py --gpus N

Rank 0 prints ONE JSON line (see DESIGN.md "Measurement" for the roofline / cpu_baseline fields;
cpu_reference_path times the reference's own CPU/OMP path, SURVEY.md row a14, on config C1).  The same line
carries "c3": BASELINE.json configs[2] measured in the same run -- 5 objects x 10k candidate poses per GPU,
render + stride cloud + covariances + GICP + re-render + re-score + select per step (the north star's
"rendered + GICP-refined + scored" figure), with its own roofline for the GICP kernel.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_BPS = 8.0e12  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
VALU_SIMDS = 1024      # 256 CUs x 4 SIMDs
VALU_CLOCK_HZ = 2.4e9  # max engine clock; a wave64 VALU instruction issues over 2 cycles (SIMD-32)


def algorithmic_bytes_per_pose(width, height, stride, p_r_mean):
    """B_r + B_c + B_s = 4*W*H*(1 + 1/s) + 24*P_r + 12 (render + score, no GICP)."""
    return 4.0 * width * height * (1.0 + 1.0 / stride) + 24.0 * p_r_mean + 12.0


def cpu_baseline(w, seconds: float):
    """Time the CPU oracle pipeline (same poses, same scene) on a bounded sample."""
    import oracle

    sc = w.scene
    poses = w.poses.cpu().numpy()
    pm = w.pose_model.cpu().numpy()
    tot = w.pose_obs_total.cpu().numpy()
    obs_xyz = w.obs_xyz.cpu().numpy()
    obs_lab = w.obs_label.cpu().numpy()
    order = np.argsort(obs_lab, kind="stable")
    oxyz, olab = obs_xyz[order], obs_lab[order]
    nl = int(olab.max()) + 1 if len(olab) else 0
    ls = np.array([np.searchsorted(olab, L, "left") for L in range(nl)], np.int32)
    le = np.array([np.searchsorted(olab, L, "right") for L in range(nl)], np.int32)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    threads = max(1, min(threads, 64))
    done, t0, batch = 0, time.perf_counter(), max(threads * 4, 32)
    rng = np.random.default_rng(7)
    while time.perf_counter() - t0 < seconds:
        idx = rng.choice(len(poses), size=min(batch, len(poses)), replace=False)
        oracle.evaluate(sc.bank.tris, sc.bank.tris_model_count, poses[idx], pm[idx], pm[idx], sc.width, sc.height,
                        sc.proj, sc.src_depth_cm, sc.mask, 1.0, w.stride, sc.cx, sc.cy, sc.fx, sc.fy, 100.0, oxyz,
                        ls, le, tot[idx], 2, True, 0.01, nthreads=threads)
        done += len(idx)
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "poses/s", "cores": threads, "kind": "port",
            "sample": f"{done} random poses of the same C2 workload through the CPU oracle (full-frame "
                      f"render + stride-8 cloud + brute-force 1-NN + costs), OpenMP over poses, {dt:.1f} s"}


def cpu_reference_path(seconds: float):
    """SURVEY.md 8(a) row a14 on BASELINE.json configs[0] (C1): the reference's own CPU/OMP path --
    render_cpu -> depth2cloud_cpu (stride 1) -> ICP_Point2Plane_cpu against the projective scene -- restated
    in oracle/ref_cpu_path.cpp, over the 128 3-DoF table-top poses of the 003_cracker_box proxy."""
    import oracle
    from perception_amd import workloads

    def render_fn(tris, cnt, p16, pm, W, H, proj):
        return oracle.ref_render_cpu(tris, p16, W, H, proj)

    c1 = workloads.c1_tabletop(render_fn)
    sc = c1.scene
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    threads = max(1, min(threads, 64))
    done, iters, t0 = 0, 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        _, fit, _, its, _ = oracle.ref_cpu_pipeline(sc.bank.tris, c1.poses, sc.width, sc.height, sc.proj, sc.fx,
                                                    sc.fy, sc.cx, sc.cy, c1.src_depth_cm, nthreads=threads)
        done += len(c1.poses)
        iters += int(its.sum())
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "poses/s", "cores": threads, "kind": "port",
            "sample": f"C1: {done // len(c1.poses)} passes over 128 3-DoF poses of the 003_cracker_box proxy at "
                      f"640x480 through render_cpu + depth2cloud_cpu + ICP_Point2Plane_cpu (mean "
                      f"{iters / max(done, 1):.1f} ICP iterations), one pose per OpenMP thread, {dt:.1f} s"}


C3_NAMES = ["003_cracker_box", "005_tomato_soup_can", "006_mustard_bottle", "010_potted_meat_can", "024_bowl"]


def c3_leg(steps: int, warmup: int, local: int, rank: int, world: int, poses_per_model: int = 10000):
    """BASELINE.json configs[2] (C3) on this rank's GPU: 5 objects, poses_per_model candidates each, GICP on.
    One step = pcore_evaluate_icp over the whole batch (render, cloud, covariances, GICP, re-render, re-score)
    + the per-model argmin keys + their all-reduce(MIN).  Timed like the C2 leg (barrier + synchronize on both
    sides, max over ranks); the GICP launches' own time comes from pcore_get_stats (HIP events on the call's
    stream), the time base of the GICP kernel's roofline."""
    import torch
    from perception_amd import distributed as pdist
    from perception_amd import workloads
    from perception_amd._native import ICP_CYCLE_WINDOW, PCORE_KEY_NONE
    from perception_amd.core import decode_keys

    w = workloads.build(names=C3_NAMES, poses_per_model=poses_per_model, device=local, rank=rank)
    n = int(w.poses.shape[0])
    dev = w.poses.device
    # batches in flight (PCORE_BENCH_C3_LANES, A/B): step i runs on lane i % L (its own context, stream, scratch,
    # outputs and key buffer), so one step's GICP tail could overlap the next step's render, clouds and covariances;
    # every step is still one whole 50k-pose batch completing inside the timed region.  Two lanes measured no faster
    # (3.95-3.99 vs 3.98-3.99 M poses/s, profiles/r06m/; 4.34-4.35 vs 4.30-4.35 M at the final build, profiles/r06c3l/),
    # so the C3 leg runs one
    L = max(1, int(os.environ.get("PCORE_BENCH_C3_LANES", "1")))
    lanes = workloads.lanes(w, L)
    outs = [(torch.empty((n, 16), dtype=torch.float32, device=dev), torch.empty(n, dtype=torch.int32, device=dev),
             *(torch.empty(n, dtype=torch.float32, device=dev) for _ in range(3))) for _ in range(L)]
    keys_ring = [torch.full((w.num_models,), PCORE_KEY_NONE, dtype=torch.int64, device=dev) for _ in range(L)]
    works = [None] * L
    pending = [False] * L  # the lane's last call is a timed step whose stats are not read yet
    rec = {"gicp_ms": [], "icp_s": [], "run": [], "exits": []}

    def read_stats(b):
        st = lanes[b][0].stats()  # waits for that call's GICP stage (its events), not for its re-score
        rec["gicp_ms"].append(st["gicp_ms"])
        rec["icp_s"].append(st["icp_runtime"])
        rec["run"].append(st["gicp_iterations_run"])
        rec["exits"].append(st["gicp_cycle_exits"])
        pending[b] = False

    def step(i, record, window):
        b = i % L
        core, st = lanes[b]
        if works[b] is not None:  # the lane's previous exchange completes before its key buffer is rewritten
            with torch.cuda.stream(st):
                works[b].wait()
            works[b] = None
        if pending[b]:  # the lane's previous call's stats, before this call replaces them
            read_stats(b)
        with torch.cuda.stream(st):
            keys_ring[b].fill_(PCORE_KEY_NONE)
            adj, it, rc, oc, df = core.evaluate_icp(w.poses, w.pose_model, w.pose_label, w.pose_obs_total,
                                                    stride=w.stride, out=outs[b], cycle_exit_window=window, stream=st)
            core.select(rc, oc, w.pose_model, w.num_models, index_base=w.index_base, keys=keys_ring[b], stream=st)
            works[b] = pdist.allreduce_min_keys_async(keys_ring[b])
        pending[b] = record

    def timed(window):
        for k in rec:
            rec[k] = []
        for i in range(max(warmup, 1) + L):  # every lane warmed (scratch, target covariances, tile tier)
            step(i, False, window)
        for b in range(L):
            if works[b] is not None:
                works[b].wait()
                works[b] = None
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            step(i, True, window)
        for b in range(L):  # every exchange completes inside the timed region
            if works[b] is not None:
                works[b].wait()
                works[b] = None
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        elapsed = time.perf_counter() - t0
        for b in range(L):  # the last steps' stats (their work is done)
            if pending[b]:
                read_stats(b)
        if world > 1:
            t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            elapsed = float(t.item())
        return elapsed, {k: list(v) for k, v in rec.items()}

    last = (steps - 1) % L  # the lane of the last timed step
    out, keys = outs[last], keys_ring[last]
    # the A/B first: every iteration run out (fast_gicp's loop, cycle_exit_window 0), then the spec's exit -- the
    # measured run -- so out / keys hold the spec's results afterwards
    el_off, rec_off = timed(0)
    its_off = out[1].cpu().numpy()
    elapsed, r = timed(ICP_CYCLE_WINDOW)
    gicp_ms, icp_s = r["gicp_ms"], r["icp_s"]
    its = out[1].cpu().numpy()
    cost, idx = decode_keys(keys)
    g_ms = float(np.mean(gicp_ms)) if gicp_ms else None
    iter_total = int(its.sum())
    iter_run = int(np.mean(r["run"])) if r["run"] else iter_total
    valu_peak = VALU_SIMDS * VALU_CLOCK_HZ / 2.0
    instr_per_iter, cyc_per_iter, sq_note = None, None, "no profiles/sq_counters_gicp.json"
    sq_path = os.path.join(ROOT, "profiles", "sq_counters_gicp.json")
    if os.path.exists(sq_path):
        try:
            from perception_amd.build import gicp_source_digest
            with open(sq_path) as f:
                sq = json.load(f)
            if sq.get("gicp_source_digest") != gicp_source_digest():
                sq_note = "counter profile of other GICP sources (stale): not used"
            else:
                instr_per_iter = float(sq["gicp_kernel"]["derived_valu_instr_per_pose_iteration"])
                cyc_per_iter = sq["gicp_kernel"].get("derived_valu_cycles_per_pose_iteration")
                sq_note = ("profiles/sq_counters_gicp.json (SQ_INSTS_VALU / pose-iterations, counters-only rocprofv3 "
                           "pass of the same GICP sources)")
        except (OSError, ValueError, KeyError) as e:
            sq_note = f"unreadable counter profile: {e}"
    # the executed pose-iterations (the cycle exits' are not run) are the work of the GICP launches
    achieved = instr_per_iter * iter_run / (g_ms * 1e-3) if (instr_per_iter and g_ms) else None
    # the same work priced in SIMD cycles (f64 and transcendental instructions 4 cycles per wave64 instruction,
    # the rest 2) against 1024 SIMDs x 2.4 GHz
    busy = (float(cyc_per_iter) * iter_run / (g_ms * 1e-3) / (VALU_SIMDS * VALU_CLOCK_HZ)
            if (cyc_per_iter and g_ms) else None)
    return {
        "metric": "candidate poses rendered+GICP-refined+scored/sec @640x480 (C3)",
        "value": n * world * steps / elapsed,
        "unit": "poses/s",
        "ms_per_step": elapsed * 1e3 / steps,
        "steps": steps,
        "warmup": max(warmup, 1),
        "config": {"workload": "C3: 5 YCB-proxy objects x 10k 6-DoF candidate poses/GPU, render + GICP (fast_gicp LM, "
                               "k 10, <= 150 iterations) + re-render + score + select, 640x480, stride 8",
                   "poses_per_gpu": n, "objects": C3_NAMES, "parallelism": f"pose-shard x{world}",
                   "batches_in_flight": L},
        "gicp": {"iterations_mean": float(its.mean()), "iterations_p50": float(np.percentile(its, 50)),
                 "iterations_p90": float(np.percentile(its, 90)), "at_max_iterations": int((its >= 150).sum()),
                 "gicp_ms_per_step": g_ms, "icp_stage_ms_per_step": float(np.mean(icp_s)) * 1e3 if icp_s else None,
                 "cycle_exit_window": ICP_CYCLE_WINDOW,
                 "iterations_reported_per_step": iter_total, "iterations_run_per_step": iter_run,
                 "cycle_exits_per_step": int(np.mean(r["exits"])) if r["exits"] else None,
                 "exit_off": {"value": n * world * steps / el_off, "ms_per_step": el_off * 1e3 / steps,
                              "gicp_ms_per_step": float(np.mean(rec_off["gicp_ms"])) if rec_off["gicp_ms"] else None,
                              "iterations_run_per_step": int(np.mean(rec_off["run"])) if rec_off["run"] else None,
                              "iterations_equal": bool(np.array_equal(its, its_off)),
                              "note": "the same steps with cycle_exit_window 0 (every iteration run out, as "
                                      "fast_gicp), timed before the measured run"},
                 "timing": "pcore_get_stats: HIP events on the call's stream around the GICP launches / the "
                           "covariances + GICP launches of every timed step"},
        "roofline": {"bound": "valu", "kernel": "gicp_kernel",
                     "achieved": achieved / 1e9 if achieved else None, "peak": valu_peak / 1e9,
                     "unit": "Gwave-instr/s", "frac": achieved / valu_peak if achieved else None,
                     "traffic": None, "valu_instr_per_pose_iteration": instr_per_iter, "valu_source": sq_note,
                     "frac_cycle_weighted": busy, "valu_cycles_per_pose_iteration": cyc_per_iter,
                     "note": "a serial chain of <= 150 dependent iterations per pose (one wave each): latency-bound "
                             "by design, so the VALU issue fraction is the figure of merit; HBM traffic is a few KB "
                             "per pose-iteration, L2-resident"},
        "argmin": {"best_cost": [int(c) for c in cost], "best_index": [int(i) for i in idx],
                   "gt_index": [int(g) for g in w.gt_index]},
    }


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(gpus: int) -> int:
    """`bench.py --gpus N` run as a single process (no WORLD_SIZE in the environment): start N rank processes
    (one per GPU, torch.distributed.run on 127.0.0.1) with the same arguments and return their exit code.  The
    parent never touches the GPU (torch.cuda.device_count() does not initialise HIP on this image) and never
    re-execs: the ranks are children, and rank 0 prints the JSON line."""
    import subprocess

    import torch

    backend = os.environ.get("PCORE_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if backend == "nccl" and ndev < gpus:
        print(f"bench.py: --gpus {gpus} needs {gpus} GPUs for one RCCL rank per GPU, {ndev} visible "
              f"(PCORE_DIST_BACKEND=gloo rehearses several ranks on one GPU)", file=sys.stderr, flush=True)
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__),
           *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--poses", type=int, default=10000, help="candidate poses per GPU per step")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--ref-cpu-seconds", type=float, default=6.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--c3-steps", type=int, default=3, help="timed C3 (GICP) steps; 0 skips the C3 leg")
    ap.add_argument("--c3-warmup", type=int, default=1)
    ap.add_argument("--force-pg", action="store_true",
                    help="at --gpus 1, start a one-rank process group (RCCL) so every step runs the argmin exchange")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))  # this process only waits for its N rank children
    # (a rank) stdout carries only the JSON line: anything else written to fd 1 (RCCL prints its version banner there when
    # the communicator starts) goes to stderr; the line itself goes to the saved descriptor
    global _JSON_FD
    _JSON_FD = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)
    world = int(env_world or "1")
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}; launch one rank per GPU with matching "
              f"--nproc-per-node and --gpus", file=sys.stderr, flush=True)
        sys.exit(2)

    import torch
    from perception_amd import distributed as pdist
    from perception_amd import workloads
    from perception_amd._native import PCORE_KEY_NONE
    from perception_amd.core import decode_keys

    rank = int(os.environ.get("RANK", "0"))
    # one rank per GPU; the modulo only matters for a several-ranks-per-GPU rehearsal (PCORE_DIST_BACKEND=gloo)
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    pdist.init_from_env(force=True if args.force_pg else None)
    joined = torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1
    if joined != world:
        raise SystemExit(f"bench.py: {joined} ranks joined, WORLD_SIZE={world}")
    # GPUs the ranks run on: one per rank over RCCL; fewer only in a gloo rehearsal (several ranks per GPU)
    devices = min(world, max(torch.cuda.device_count(), 1))
    dev = torch.device("cuda", local)

    w = workloads.build(poses_per_model=args.poses, device=local, rank=rank)
    n = int(w.poses.shape[0])
    # batches in flight: step i runs on lane i % L (its own context, stream, outputs and key buffer)
    L = max(1, int(os.environ.get("PCORE_BENCH_LANES", "2")))
    lanes = workloads.lanes(w, L)
    outs = [tuple(torch.empty(n, dtype=torch.float32, device=dev) for _ in range(3)) for _ in range(L)]
    # one key buffer per lane: step i's all-reduce(MIN) overlaps the next steps' kernels; a buffer is rewritten
    # only after its previous exchange has completed (work.wait() orders the lane's stream after it)
    keys_ring = [torch.full((w.num_models,), PCORE_KEY_NONE, dtype=torch.int64, device=dev) for _ in range(L)]
    works = [None] * L

    # rendered points per pose (for the algorithmic byte count), measured once outside the timed region
    # with one launch over the whole batch, so every fused-kernel launch of this process (and of its
    # rocprofv3 --stats summary) covers the same n poses
    s = w.stride
    hs, ws = (w.scene.height + s - 1) // s, w.scene.width // s
    dbg = torch.empty((n, hs, ws), dtype=torch.int32, device=dev)
    w.core.evaluate(w.poses, w.pose_model, w.pose_label, w.pose_obs_total, stride=s, dbg_zs=dbg)
    p_r_mean = int((dbg > 0).sum().item()) / max(n, 1)
    del dbg
    torch.cuda.synchronize()

    # host timestamps of every timed step (perf_counter, s): step start, around the wait for the lane's previous
    # exchange, around the launch call, after the exchange is issued -- they attribute a slow step to the host wait
    # (the exchange), to the launch call itself, or to the GPU (the HIP-event span) without another run
    host_ts = []

    def run_step(i, ev=None):
        b = i % L
        core, st = lanes[b]
        t0h = time.perf_counter()
        # the lane's previous exchange must have completed before its key buffer is rewritten: with RCCL wait() only
        # orders the lane's stream after the collective; with gloo it blocks the host until the exchange is done
        if works[b] is not None:
            with torch.cuda.stream(st):
                works[b].wait()
        t1h = time.perf_counter()
        with torch.cuda.stream(st):
            keys_ring[b].fill_(PCORE_KEY_NONE)
            if ev is not None:
                ev[0].record(st)
            # stage COST with the per-model argmin folded into the same launch (pcore_evaluate_select)
            core.evaluate(w.poses, w.pose_model, w.pose_label, w.pose_obs_total, stride=s, out=outs[b], stream=st,
                          select=(keys_ring[b], w.index_base, w.num_models))
            if ev is not None:
                ev[1].record(st)
            t2h = time.perf_counter()
            works[b] = pdist.allreduce_min_keys_async(keys_ring[b])
        if ev is not None:
            host_ts.append((t0h, t1h, t2h, time.perf_counter()))

    for i in range(args.warmup + L):  # every lane warmed (tile tier picked from its own first call)
        run_step(i)
    for b in range(L):
        if works[b] is not None:
            works[b].wait()
            works[b] = None
    torch.cuda.synchronize()

    # per-launch duration of the dominant (fused) kernel, by HIP events on the stream it runs on (its lane's)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        run_step(i, ev[i])
    for wk in works:  # every exchange completes inside the timed region
        if wk is not None:
            wk.wait()
    keys = keys_ring[(args.steps - 1) % L]
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    # with L > 1 consecutive launches overlap (one's drain with the next one's fill), so a launch's own span
    # counts time it shares with its neighbours; the GPU time per launch is the union of the launch intervals
    # divided by the launches (= kern_ms when L = 1)
    iv = sorted((ev[0][0].elapsed_time(a), ev[0][0].elapsed_time(b)) for a, b in ev)
    busy, cur_lo, cur_hi = 0.0, iv[0][0], iv[0][1]
    for lo, hi in iv[1:]:
        if lo > cur_hi:
            busy += cur_hi - cur_lo
            cur_lo, cur_hi = lo, hi
        else:
            cur_hi = max(cur_hi, hi)
    busy += cur_hi - cur_lo
    busy_ms = busy / len(iv)

    ht = np.array(host_ts) - t0
    wait_ms = (ht[:, 1] - ht[:, 0]) * 1e3
    launch_ms = (ht[:, 2] - ht[:, 1]) * 1e3
    issue_ms = (ht[:, 3] - ht[:, 2]) * 1e3
    spans = np.array([a.elapsed_time(b) for a, b in ev])
    host_timing = {
        "wait_prev_exchange_ms": {"mean": float(wait_ms.mean()), "max": float(wait_ms.max())},
        "launch_call_ms": {"mean": float(launch_ms.mean()), "max": float(launch_ms.max())},
        "exchange_issue_ms": {"mean": float(issue_ms.mean()), "max": float(issue_ms.max())},
        "launch_span_ms": {"mean": float(spans.mean()), "max": float(spans.max())},
        "slowest_step": int(np.argmax(np.diff(np.append(ht[:, 0], elapsed)))),
        "definition": "per timed step, host perf_counter: wait = works[b].wait() for the lane's previous exchange "
                      "(gloo: host-blocking; RCCL: a stream dependency), launch_call = fill + evaluate call + "
                      "event records, exchange_issue = the async all_reduce call; launch_span = HIP events around "
                      "the stage-COST launch on the lane's stream",
    }

    best_cost, best_idx = decode_keys(keys)
    c3 = None
    if args.c3_steps > 0:
        del lanes, outs, keys_ring, works
        torch.cuda.empty_cache()
        c3 = c3_leg(args.c3_steps, args.c3_warmup, local, rank, world)
    if rank != 0:
        return
    total_poses = n * world * args.steps
    value = total_poses / elapsed
    bpp = algorithmic_bytes_per_pose(w.scene.width, w.scene.height, s, p_r_mean)
    achieved = bpp * n / (busy_ms * 1e-3)
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc_path):
        try:
            with open(pmc_path) as f:
                pmc = json.load(f)
            from perception_amd.build import kernel_source_digest
            if pmc.get("poses_per_launch") == n and pmc.get("kernel_source_digest") == kernel_source_digest():
                traffic = pmc.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None
    # The binding roof ("Kernels and their bounds"): the fused kernel keeps its z-samples in LDS,
    # moves ~770 B of HBM per pose and is bound by vector issue, so roofline.bound is "valu": VALU
    # wave-instructions per pose (SQ_INSTS_VALU of a counters-only pass of the same sources, tools/
    # sq_counters.sh -> profiles/sq_counters.json) x poses per launch / the live launch duration, against
    # 1024 SIMDs x 2.4 GHz / 2 cycles per wave64 instruction (MI355X_MICROARCH.md).  The HBM figures stay
    # beside it: measured traffic against 8 TB/s, and SURVEY.md 8(d)'s algorithmic bytes (a design that
    # materialises every z-buffer) as effective_vs_naive.
    instr_per_pose, sq_note = None, "no profiles/sq_counters.json"
    sq_path = os.path.join(ROOT, "profiles", "sq_counters.json")
    if os.path.exists(sq_path):
        try:
            from perception_amd.build import kernel_source_digest
            with open(sq_path) as f:
                sq = json.load(f)
            if sq.get("fused_cost_poses_per_launch") != n:
                sq_note = "counter profile taken at another batch size"
            elif sq.get("kernel_source_digest") != kernel_source_digest():
                sq_note = "counter profile of other kernel sources (stale): not used"
            else:
                instr_per_pose = float(sq["fused_cost"]["derived_valu_instr_per_pose"])
                sq_note = ("profiles/sq_counters.json (SQ_INSTS_VALU / poses, counters-only rocprofv3 pass of "
                           "the same kernel sources)")
        except (OSError, ValueError, KeyError) as e:
            sq_note = f"unreadable counter profile: {e}"
    kern_s = busy_ms * 1e-3
    valu_peak = VALU_SIMDS * VALU_CLOCK_HZ / 2.0  # wave64 VALU instructions per second
    valu_achieved = instr_per_pose * n / kern_s if instr_per_pose else None
    hbm_meas = traffic / kern_s if traffic else None
    roofline = {
        "bound": "valu",
        "achieved": valu_achieved / 1e9 if valu_achieved else None,
        "peak": valu_peak / 1e9,
        "unit": "Gwave-instr/s",
        "frac": valu_achieved / valu_peak if valu_achieved else None,
        "traffic": traffic,
        "kernel": "fused_cost_kernel (stage COST, one launch per batch)",
        "kernel_ms": busy_ms,
        "timing": {"launch_span_ms": kern_ms, "gpu_ms_per_launch": busy_ms, "launches_in_flight": L,
                   "definition": "HIP events around every stage-COST call on its lane's stream over the timed region: "
                                 "launch_span_ms = mean span of one launch (overlapping its neighbours when "
                                 "launches_in_flight > 1; rocprofv3's average duration); gpu_ms_per_launch = union "
                                 "of the launch intervals / launches, the time base of achieved and frac"},
        "valu_instr_per_pose": instr_per_pose,
        "valu_source": sq_note,
        "hbm": {"measured_GBps": hbm_meas / 1e9 if hbm_meas else None, "peak_GBps": HBM_PEAK_BPS / 1e9,
                "frac": hbm_meas / HBM_PEAK_BPS if hbm_meas else None,
                "bytes_per_pose": traffic / n if traffic else None,
                "source": "profiles/pmc_traffic.json (FETCH_SIZE x2 + WRITE_SIZE, separate --pmc passes)"},
        "effective_vs_naive": {"algorithmic_GBps": achieved / 1e9, "frac_of_hbm_peak": achieved / HBM_PEAK_BPS,
                               "bytes_per_pose": bpp, "p_r_mean": p_r_mean,
                               "definition": "SURVEY.md 8(d) B_r + B_c + B_s (z-buffer materialised in HBM, as "
                                             "the reference does) / kernel time; > 1 means faster than an "
                                             "HBM-bound materialising design could be"},
    }
    line = {
        "metric": "candidate poses rendered+scored/sec @640x480",
        "value": value,
        "unit": "poses/s",
        "n_gpus": joined,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (003_cracker_box proxy mesh, GT-rendered 16-bit depth + 2 mm noise, label mask)",
        "config": {"workload": "C2: 1 YCB mesh (12,288 tris), 10k 6-DoF poses/GPU render+score, 640x480, "
                               "stride 8, no ICP", "poses_per_gpu": n, "width": w.scene.width,
                   "height": w.scene.height, "stride": s, "parallelism": f"pose-shard x{world}",
                   "batches_in_flight": L, "ranks": joined, "devices": devices,
                   "dist_backend": torch.distributed.get_backend() if pdist.exchange_active() else None,
                   "exchange": ("all_reduce(MIN) of the int64 argmin keys per step" if pdist.exchange_active()
                                else "none (one process)")},
        "roofline": roofline,
        "host_timing": host_timing,
        "argmin": {"best_cost": int(best_cost[0]), "best_index": int(best_idx[0]), "gt_index": int(w.gt_index[0])},
    }
    if c3 is not None:
        line["c3"] = c3
    if world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline(w, args.cpu_seconds)
        line["cpu_reference_path"] = cpu_reference_path(args.ref_cpu_seconds)
    os.write(_JSON_FD, (json.dumps(line) + "\n").encode())


_JSON_FD = 1

if __name__ == "__main__":
    main()
