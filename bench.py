#!/usr/bin/env python3
"""Benchmark: DiffusionDrive eval forward (ResNet-34 + LiDAR-BEV backbone, 2 truncated DDIM
steps) on MI355X, scenes/s at batch 64 per GPU (BASELINE.json metric / configs[1], weak scaling
over 1/2/4/8 GPUs with one RCCL all_gather of the predicted trajectories per step).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]

With ``--gpus N > 1`` and no ``$WORLD_SIZE`` the script launches N rank processes itself
(torchrun-style: RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT in their
environment, nothing touches the GPU before that) and exits with the worst rank's code. Under
``python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N`` each rank reads the
launcher's environment; a ``--gpus`` that disagrees with ``$WORLD_SIZE`` is an error.

A step = one forward of B synthetic scenes resident in HBM (+ the all_gather when N > 1). ``--in-flight L``
(default 3) keeps L steps in flight per GPU (diffusiondrive_amd/model.py InFlightPlanner); the timed region
still brackets all K steps completely.
Rank 0 prints ONE JSON line. Besides the contract fields it reports:
  * ``median_ms_per_step``: median step interval from the completion events (HIP events on the lanes' streams,
    end times sorted on the device clock, windows of ``in_flight`` completions: ``completion_intervals``);
    ``median_batch_latency_ms``: median start -> end of one step's forward on its lane (with ``--in-flight N`` > 1,
    N batches share the device, so a batch takes longer while the steps complete faster); ``scenes_resident`` =
    batch x in_flight;
  * ``in_flight_1``: the same workload one batch at a time - the strict "scenes/s at batch 64" figure;
  * ``gather_check``: every rank's slice of the all_gather output equals its own forward (N > 1: the C3 workload,
    shards of one seeded global batch), and shard 0's waypoint L2 against the reference golden;
  * ``fp32_leg``: the same workload on the fp32-MFMA path (N = 1), the conservative headline;
  * ``h2d_included``: the same forward with its inputs copied from pinned host memory every
    step (PCIe-inclusive; never ``value``);
  * ``roofline``: the dominant kernel (the conv / GEMM kernel with the most device time in a
    profiled single-stream replay: conv_x6 for the default f16x3 path), algorithmic FLOP per
    launch / average launch time from HIP events recorded on the kernel's stream; peak = the
    algorithmic fp32 ceiling of the gemm mode (157.3 TFLOP/s fp32 MFMA dense, or 2500 / 3
    TFLOP/s for the 3-product f16 split, MI355X_MICROARCH.md); ``traffic`` = HBM bytes per
    launch from the committed rocprofv3 PMC summary (FETCH x2 + WRITE, separate passes);
  * ``whole_forward``: canonical GFLOP/scene AND the FLOPs the graph executes
    (gathered value_proj, low-res bev_proj: fewer than canonical);
  * ``cpu_baseline``: the golden-pinned CPU oracle (oracle/, PyTorch-CPU fp32) timed on this
    host at the job's CPU share (min of sched affinity, cgroup quota, $OMP_NUM_THREADS) on the
    timed B = 64 batch (3 reps) and a B = 1 sample (rank 0, N = 1 only); its outputs are the
    waypoint-L2 parity check of both GPU legs;
  * ``decoder_cross_attention``: the gathered value_proj launches (the decoder's cross-BEV attention
    contraction) with their live-row TFLOP/s.
``--cpu-plumbing`` (tests only) runs the launcher / gloo all_gather / max-over-ranks / JSON path
on CPU with a stand-in step (zeros; no forward) so the multi-rank plumbing is testable here.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "scenes/s at batch 64, 2 denoise steps, 1/2/4/8 MI355X; waypoint L2 vs ref"
CANONICAL_GFLOP_PER_SCENE_2STEP = 65.27  # SURVEY.md §8d (value_proj once per layer)
FP32_MFMA_PEAK_TFLOPS = 157.3            # MI355X dense fp32 MFMA (= vector) peak
F16_MFMA_PEAK_TFLOPS = 2500.0            # MI355X dense f16 / bf16 MFMA peak (no sparsity)
# measured whole-chip f16 32x32x16 MFMA loop on random operands (clock held ~1.55 GHz under DVFS):
# profiles/archive/round2_h_mfma_shape.txt (tools/micro/mfma_shape.hip) - the rate a real kernel can sustain
F16_MFMA_SUSTAINED_TFLOPS = 1600.0
# peak of ALGORITHMIC FLOPs per gemm mode: f16x3 issues 3 f16 MFMA products per fp32 MAC
ALGO_PEAK = {"fp32": FP32_MFMA_PEAK_TFLOPS, "f16x3": F16_MFMA_PEAK_TFLOPS / 3, "bf16": F16_MFMA_PEAK_TFLOPS}
KERNEL_DESC = {
    "conv_gemm": "conv_gemm (implicit-GEMM conv / GEMM, fp32 MFMA v_mfma_f32_32x32x2_f32)",
    "conv_x3": "conv_x3 (implicit-GEMM conv / GEMM, 3-product fp16 split on v_mfma_f32_32x32x16_f16)",
    "conv_x5": "conv_x5 (implicit-GEMM conv, LDS-DMA staging, 3-product fp16 split on v_mfma_f32_32x32x16_f16)",
    "conv_x6": "conv_x6 (halo-reuse direct 3x3 conv on v_mfma_f32_32x32x16_{f16 x3 | bf16})",
    "basicblock": "basicblock (fused layer-1 BasicBlock: two 3x3 convs, the intermediate in LDS, f16x3 MFMA)",
}
CONV_KERNELS = ("conv_x6", "conv_x5", "conv_x3", "conv_gemm", "basicblock")
OTHER_KERNELS = ("value_proj", "stem_pool", "attn", "layernorm", "softmax", "bilinear", "pool", "mha", "bev_sample",
                 "decoder", "tfdec", "bevproj", "gpt_tail", "misc")
DTYPE = {
    "fp32": "fp32",
    "f16x3": "fp32 via f16x3 (each fp32 operand = hi+lo fp16, products ah*bh+ah*bl+al*bh, fp32 accumulate)",
    "bf16": "bf16 backbone (one bf16 product per MAC, fp32 accumulate; reduced precision), f16x3 after it",
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--batch", type=int, default=64, help="scenes per GPU")
    p.add_argument("--denoise-steps", type=int, default=2)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-threads", default="8", help="extra thread counts of the CPU-oracle baseline beside the job's "
                                                       "CPU share (BASELINE.md: n = 8 and n = all cores; 3 reps each)")
    p.add_argument("--arch", default="resnet34")
    p.add_argument("--gemm", default="f16x3", choices=["fp32", "f16x3", "bf16"],
                   help="conv/linear arithmetic: fp32 MFMA, the fp32-class 3-product fp16 split, or bf16")
    p.add_argument("--no-compare", action="store_true", help="skip the fp32 leg and the H2D-inclusive leg")
    p.add_argument("--in-flight", type=int, default=3,
                   help="batches in flight per GPU (InFlightPlanner lanes: single-stream handles on streams of their "
                        "own); 1 = one forward at a time on a default (two-stream) handle")
    p.add_argument("--lane-streams", type=int, default=1, choices=[1, 2],
                   help="streams of each lane's captured forward when --in-flight > 1")
    p.add_argument("--cpu-plumbing", action="store_true",
                   help="tests only: launcher + gloo all_gather + JSON with a stand-in step (no forward)")
    return p.parse_args()


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int) -> int:
    """Start n rank processes of this script (before any GPU call in this process) and return the
    worst exit code. Rank 0's stdout carries the JSON line."""
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(env_world or "1")
    if world != args.gpus:
        print(f"[bench] --gpus {args.gpus} disagrees with WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.cpu_plumbing:
        return plumbing(args, world, rank)

    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        world = dist.get_world_size()  # the world the RCCL communicator actually formed
    else:
        torch.cuda.set_device(0)
    dev = torch.device(f"cuda:{local}")

    from diffusiondrive_amd.config import TransfuserConfig
    from diffusiondrive_amd.dist import ScenePlanner
    from diffusiondrive_amd.model import InFlightPlanner
    from diffusiondrive_amd.weights import reference_noise, seeded_state_dict, synthetic_inputs

    if args.in_flight < 1:
        print("[bench] --in-flight must be >= 1", file=sys.stderr)
        sys.exit(2)
    cfg = TransfuserConfig(image_architecture=args.arch)
    sd = seeded_state_dict(cfg, 0)
    # args.in_flight lanes (handles with the same weights); lane 0 also serves the profiled replay
    pl = InFlightPlanner(cfg, sd, device=local, lanes=args.in_flight, lane_streams=args.lane_streams)
    pl.set_gemm_mode(args.gemm)
    model = pl.lanes[0]
    B = args.batch
    # this rank's shard of ONE seeded global batch (config C3 at N = 8): scenes of rank r are
    # synthetic_inputs(B, 1234 + r), and the DDIM start noise is drawn once for all B * world scenes
    # (torch.manual_seed(1234); torch.randn(B * world, 20, 8, 2)) and sliced - tests/test_sharding_gpu.py's global
    # batch. Shard 0 is the reference golden's batch (tests/golden/ref_b64_s1234.npz).
    inp = synthetic_inputs(B, 1234 + rank, cfg)
    inp["noise"] = np.ascontiguousarray(reference_noise(B * world, 1234, cfg)[rank * B:(rank + 1) * B])
    keys = ("camera_feature", "lidar_feature", "status_feature")
    feats = {k: torch.from_numpy(inp[k]).to(dev) for k in keys}
    noise = torch.from_numpy(inp["noise"]).to(dev)
    planner = ScenePlanner(lambda f, nz: pl.forward(f, noise=nz, steps=args.denoise_steps)["trajectory"])
    lane_steps = LaneSteps(pl, planner, lambda: torch.cuda.Event(enable_timing=True),
                           lambda: torch.cuda.current_stream(dev))
    marks = lane_steps.marks  # per step: (start, end) HIP events on the stream the step ran on
    lane_step = lane_steps.step

    def step():
        # per-rank shard of the global batch (weak scaling) + one RCCL all_gather of trajectories
        return lane_step(lambda m, s: m.forward(feats, noise=noise, steps=args.denoise_steps, stream=s)["trajectory"])

    def timed(fn, k, lanes=args.in_flight):
        """k steps between barrier + synchronize. Per step: the interval between consecutive step completions
        (HIP events on the lanes' streams, one device clock) and the batch latency (its own start -> end)."""
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        marks.clear()
        e_start = torch.cuda.Event(enable_timing=True)
        e_start.record()
        t0 = time.perf_counter()
        o = None
        for _ in range(k):
            o = fn()
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        el = time.perf_counter() - t0
        return o, el, completion_intervals(e_start, marks, lanes), [e0.elapsed_time(e1) for e0, e1 in marks]

    for _ in range(args.warmup):
        out = step()
    torch.cuda.synchronize()
    out, elapsed, per_step, lat_step = timed(step, args.steps)
    med = float(np.median(per_step))
    lat_med = float(np.median(lat_step))
    if dist is not None:
        t = torch.tensor([elapsed, med, lat_med], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, med, lat_med = float(t[0].item()), float(t[1].item()), float(t[2].item())
    ms_per_step = elapsed / args.steps * 1e3
    scenes_per_s = B * world * args.steps / elapsed
    torch.cuda.synchronize()
    traj_gpu = out[rank * B:(rank + 1) * B].detach().cpu().numpy()
    gather_ok = gather_slices_ok(out, lane_steps.last_local, rank, B, dist, dev)
    gathered = out.detach().cpu().numpy()
    shard0_golden_l2 = golden_l2(gathered, args.arch, B, args.denoise_steps) if B == 64 else None
    num_flags = pl.numerics_flags()
    if num_flags:
        print(f"[bench] WARNING: numerics flags {num_flags:#x} raised (f16x3 overflow): result untrustworthy",
              file=sys.stderr)

    # ---- roofline of the dominant kernel: a profiled single-stream replay of the same workload
    # (HIP events around every launch on the stream it is issued to)
    # (lane 0; a profiled forward runs eagerly on one stream whatever the handle's stream count)
    model.set_profiling(True)
    model.reset_stats()
    prof_steps = max(1, min(args.steps, 5))
    for _ in range(prof_steps):
        model.forward(feats, noise=noise, steps=args.denoise_steps)
    torch.cuda.synchronize()
    conv_stats = {k: model.kernel_stats(k) for k in CONV_KERNELS}
    main_k = max(CONV_KERNELS, key=lambda k: conv_stats[k]["ms"])
    st = conv_stats[main_k]
    other = {k: model.kernel_stats(k) for k in OTHER_KERNELS}
    value_proj = value_proj_record(model, other["value_proj"], prof_steps, B, args)
    other.update({k: v for k, v in conv_stats.items() if k != main_k})
    model.set_profiling(False)
    avg_ms = st["ms"] / max(st["launches"], 1)
    flops_per_launch = st["flops"] / max(st["launches"], 1)
    achieved = flops_per_launch / (avg_ms * 1e-3) / 1e12 if avg_ms > 0 else 0.0
    total_prof_ms = st["ms"] + sum(v["ms"] for v in other.values())
    executed_flops = sum(v["flops"] for v in conv_stats.values()) + other["attn"]["flops"] + other["value_proj"]["flops"]
    executed_gflop_scene = executed_flops / prof_steps / B / 1e9

    fp32_leg = h2d = one_at_a_time = batch1 = None
    if world == 1 and not args.no_compare:
        batch1 = batch1_leg(cfg, sd, feats, noise, args, dev)
        # the fp32-MFMA path on the same workload (the conservative headline)
        other_mode = "fp32" if args.gemm != "fp32" else "f16x3"
        pl.set_gemm_mode(other_mode)
        for _ in range(2 * args.in_flight):
            step()
        n_cmp = max(5, min(args.steps // 2, 30))
        o2, dt, per2, _ = timed(step, n_cmp)
        fp32_leg = {"gemm": other_mode, "value": round(B * n_cmp / dt, 3), "ms_per_step": round(dt / n_cmp * 1e3, 3),
                    "median_ms_per_step": round(float(np.median(per2)), 3), "steps": n_cmp,
                    "in_flight": args.in_flight, "traj": o2.detach().cpu().numpy()}
        pl.set_gemm_mode(args.gemm)
        if args.in_flight > 1:
            # one batch at a time on lane 0 as a default handle (two streams: single-stream graph segments joined by
            # events; the --in-flight 1 configuration), then as a single-stream handle for comparison
            n1 = max(5, min(args.steps // 2, 60))
            one = {}
            for ns in (2, 1):
                model.set_streams(ns)
                for _ in range(3):
                    model.forward(feats, noise=noise, steps=args.denoise_steps)
                _, dt1, _, _ = timed(lambda: model.forward(feats, noise=noise, steps=args.denoise_steps)["trajectory"],
                                     n1, lanes=1)
                one[ns] = (round(B * n1 / dt1, 3), round(dt1 / n1 * 1e3, 3))
            one_at_a_time = {"value": one[2][0], "ms_per_step": one[2][1], "steps": n1,
                             "single_stream": {"value": one[1][0], "ms_per_step": one[1][1]},
                             "note": "in_flight 1: one forward at a time on a default handle (two streams, captured as "
                                     "single-stream graph segments joined by events; its ms_per_step is the batch "
                                     "latency of that mode); single_stream: the same on a one-stream handle"}
            model.set_streams(args.lane_streams)
        # PCIe-inclusive: inputs staged from pinned host memory every step (one device buffer set per lane)
        host = {k: torch.from_numpy(inp[k]).pin_memory() for k in keys}
        host_nz = torch.from_numpy(inp["noise"]).pin_memory()
        dbufs = [({k: torch.empty_like(v, device=dev) for k, v in host.items()}, torch.empty_like(host_nz, device=dev))
                 for _ in range(args.in_flight)]
        h2d_i = [0]

        def step_h2d():
            dbuf, dnz = dbufs[h2d_i[0] % args.in_flight]
            h2d_i[0] += 1

            def body(m, s):
                for k in keys:
                    dbuf[k].copy_(host[k], non_blocking=True)
                dnz.copy_(host_nz, non_blocking=True)
                return m.forward(dbuf, noise=dnz, steps=args.denoise_steps, stream=s)["trajectory"]
            return lane_step(body)

        for _ in range(2 * args.in_flight):
            step_h2d()
        n_h = max(5, min(args.steps // 2, 40))
        _, dt, per3, _ = timed(step_h2d, n_h)
        h2d = {"value": round(B * n_h / dt, 3), "ms_per_step": round(dt / n_h * 1e3, 3),
               "median_ms_per_step": round(float(np.median(per3)), 3), "steps": n_h,
               "bytes_per_step": int(sum(v.numel() * 4 for v in host.values()) + host_nz.numel() * 4),
               "note": "inputs copied host(pinned)->HBM inside every step; not the headline value"}

    # HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC summary (FETCH_SIZE x2 +
    # WRITE_SIZE in separate passes over this same bench command, tools/pmc_traffic.py); the algorithmic
    # bytes per launch come from this run's launch shapes (input map + output + residual + weight image once)
    traffic, pmc_meta = None, {}
    pmc_path = os.path.join(ROOT, "profiles", f"pmc_{main_k}_{args.gemm}.json")
    if os.path.exists(pmc_path):
        try:
            with open(pmc_path) as f:
                pmc_meta = json.load(f)
            traffic = pmc_meta.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None
    algo_bytes = st["bytes"] / max(st["launches"], 1)

    result = {
        "metric": METRIC,
        "value": round(scenes_per_s, 3),
        "unit": "scenes/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "median_ms_per_step": round(med, 3),
        "median_batch_latency_ms": round(lat_med, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": DTYPE[args.gemm],
        "data": "synthetic (seeded camera/LiDAR/status/noise; seeded random weights of the reference architecture)",
        "config": {
            "workload": f"DiffusionDrive eval forward: {args.arch} camera + ResNet-34 LiDAR-BEV backbone, "
                        f"GPT fusion x4, tf decoder, truncated diffusion decoder {args.denoise_steps} DDIM steps x 2 "
                        f"layers, 20 modes; batch {B} scenes per GPU",
            "batch_per_gpu": B,
            "global_batch": B * world,
            "denoise_steps": args.denoise_steps,
            "parallelism": f"dp{world} (scene sharding, RCCL all_gather of trajectories)",
            "graph": True,
            "in_flight": args.in_flight,
            "in_flight_note": "batches in flight per GPU: InFlightPlanner lanes (handles with the same weights, each "
                              "a single-stream captured forward replayed on a stream of its own); consecutive steps "
                              "go to consecutive lanes; every step's forward runs whole inside the timed region. "
                              "1 = one forward at a time on a default (two-stream) handle",
            "gemm": args.gemm,
            "heads": False,
            "heads_note": "the timed forward is the waypoint path (trajectory out); the BEV-semantic and agent "
                          "heads (off that path, 0.33 GFLOP/scene, SURVEY §8a-a10) are not run - parity tests run them",
        },
        "roofline": {
            "kernel": KERNEL_DESC[main_k],
            "bound": "mfma",
            "achieved": round(achieved, 3),
            "peak": round(ALGO_PEAK[args.gemm], 1),
            "unit": "TFLOP/s",
            "frac": round(achieved / ALGO_PEAK[args.gemm], 4),
            "peak_note": {"fp32": "fp32 MFMA 157.3 TF",
                          "f16x3": "algorithmic fp32 FLOP/s ceiling: dense f16 MFMA 2500 TF / 3 products per fp32 MAC",
                          "bf16": "dense bf16 MFMA 2500 TF"}[args.gemm],
            "sustained_peak": round(F16_MFMA_SUSTAINED_TFLOPS / (3.0 if args.gemm == "f16x3" else 1.0), 1)
            if args.gemm != "fp32" else None,
            "frac_of_sustained": round(achieved / (F16_MFMA_SUSTAINED_TFLOPS / (3.0 if args.gemm == "f16x3" else 1.0)), 4)
            if args.gemm != "fp32" else None,
            "sustained_note": "measured f16 32x32x16 MFMA loop on random data, whole chip: 1600 TF "
                              "(profiles/archive/round2_h_mfma_shape.txt); peak/frac stay on the nominal ceiling",
            "traffic": traffic,
            "traffic_source": (f"{os.path.relpath(pmc_path, ROOT)} (measured {pmc_meta.get('measured', '?')}, "
                               f"{pmc_meta.get('source', '?')})") if traffic is not None else None,
            "algorithmic_bytes_per_launch": round(algo_bytes),
            "traffic_over_algorithmic": round(traffic / algo_bytes, 3) if traffic and algo_bytes else None,
            "launches_per_step": st["launches"] // prof_steps,
            "avg_launch_ms": round(avg_ms, 5),
            "gflop_per_launch": round(flops_per_launch / 1e9, 4),
            "share_of_device_time": round(st["ms"] / total_prof_ms, 4) if total_prof_ms else None,
            "conv_kernels": {k: {"launches_per_step": v["launches"] // prof_steps,
                                 "avg_launch_ms": round(v["ms"] / max(v["launches"], 1), 5),
                                 "tflops": round(v["flops"] / (v["ms"] * 1e-3) / 1e12, 2) if v["ms"] else None,
                                 "algorithmic_mb_per_launch": round(v["bytes"] / max(v["launches"], 1) / 1e6, 2),
                                 "share_of_device_time": round(v["ms"] / total_prof_ms, 4) if total_prof_ms else None}
                             for k, v in conv_stats.items() if v["launches"]},
        },
        "device_ms_per_step": {k: round(v["ms"] / prof_steps, 4) for k, v in
                               sorted({main_k: st, **other}.items(), key=lambda kv: -kv[1]["ms"]) if v["launches"]},
        "launches_per_step": {k: v["launches"] // prof_steps for k, v in {main_k: st, **other}.items()
                              if v["launches"]},
        "whole_forward": {
            "canonical_gflop_per_scene": CANONICAL_GFLOP_PER_SCENE_2STEP if args.denoise_steps == 2 else None,
            "canonical_tflops": round(scenes_per_s / world * CANONICAL_GFLOP_PER_SCENE_2STEP / 1e3, 3)
            if args.denoise_steps == 2 else None,
            "executed_gflop_per_scene": round(executed_gflop_scene, 3),
            "executed_tflops": round(scenes_per_s / world * executed_gflop_scene / 1e3, 3),
            "note": "canonical = SURVEY §8d algorithmic work; executed = the GEMM/conv/attention FLOPs the graph "
                    "issues (value_proj only at the sampled taps, bev_proj keyval half at 8x8)",
        },
        "decoder_cross_attention": value_proj,
        "numerics_flags": num_flags,
        "scenes_resident": B * args.in_flight,
        "gather_check": {"gathered_rows": int(gathered.shape[0]), "every_rank_slice_equals_local": gather_ok,
                         "shard0_waypoint_l2_vs_golden": shard0_golden_l2,
                         "note": "each rank's slice of the all_gather output equals its own forward bit for bit "
                                 "(MIN over ranks); shard 0 = scenes 0..63 of the seeded global batch vs the "
                                 "reference golden tests/golden/ref_b64_s1234.npz"},
    }
    if h2d is not None:
        result["h2d_included"] = h2d
    if one_at_a_time is not None:
        result["in_flight_1"] = one_at_a_time
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu, ref = cpu_baseline(args, cfg, sd, inp)
        cpu["waypoint_l2_gpu_vs_oracle"] = waypoint_l2(traj_gpu, ref)
        if fp32_leg is not None:
            fp32_leg["waypoint_l2_vs_oracle"] = waypoint_l2(fp32_leg["traj"], ref)
        result["waypoint_l2_vs_oracle"] = cpu["waypoint_l2_gpu_vs_oracle"]
    if batch1 is not None:
        traj1 = batch1.pop("traj")
        if cpu is not None:
            batch1["waypoint_l2_vs_oracle"] = waypoint_l2(traj1, ref[:1])
        result["batch1"] = batch1
        result["batch1_ms"] = batch1["median_ms"]
    if fp32_leg is not None:
        fp32_leg["waypoint_l2_vs_primary"] = waypoint_l2(fp32_leg.pop("traj"), traj_gpu)
        result["fp32_leg"] = fp32_leg
    if cpu is not None:
        result["cpu_baseline"] = cpu
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def batch1_leg(cfg, sd, feats, noise, args, dev, reps=60):
    """Config C1: the reference's own eval shape (one scene per call: run_pdm_score.py:72-87 ->
    abstract_agent.py:65-86) on a default handle (two streams, f16x3), scene 0 of the timed batch. Each of ``reps``
    graph replays is bracketed by HIP events on the caller's stream and waited for before the next starts (request
    latency, no pipelining across calls): the median and p90 are reported, with the back-to-back rate beside them."""
    from diffusiondrive_amd.model import DiffusionDriveModel
    m = DiffusionDriveModel(cfg, sd, device=dev.index or 0)
    try:
        m.set_gemm_mode(args.gemm)
        f1 = {k: v[:1].contiguous() for k, v in feats.items()}
        n1 = noise[:1].contiguous()
        for _ in range(5):
            m.forward(f1, noise=n1, steps=args.denoise_steps)
        torch.cuda.synchronize()
        lat = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            m.forward(f1, noise=n1, steps=args.denoise_steps)
            e1.record()
            e1.synchronize()
            lat.append(e0.elapsed_time(e1))
        t0 = time.perf_counter()
        for _ in range(reps):
            out = m.forward(f1, noise=n1, steps=args.denoise_steps)["trajectory"]
        torch.cuda.synchronize()
        b2b = (time.perf_counter() - t0) / reps * 1e3
        flags = m.numerics_flags()
        return {"median_ms": round(float(np.median(lat)), 4), "p90_ms": round(float(np.percentile(lat, 90)), 4),
                "min_ms": round(float(np.min(lat)), 4), "replays": reps, "back_to_back_ms": round(b2b, 4),
                "gemm": args.gemm, "streams": m.stream_count(), "numerics_flags": flags,
                "traj": out.detach().cpu().numpy(),
                "note": "config C1: batch 1 on a default handle (scene 0 of the timed batch); per replay HIP events "
                        "on the caller's stream, each replay waited for (request latency); back_to_back_ms = wall "
                        "time per forward over the same number of unsynchronised replays"}
    finally:
        m.close()


def value_proj_record(model, vp, prof_steps, B, args):
    """The decoder's cross-BEV attention contraction (value_proj, blocks.py:68-76,114, evaluated at the grid-sample
    taps: the gathered conv_x3 launches). Its FLOP count in the launch stats covers every row slot (B x 640 per
    launch); the LIVE rows are the distinct tap pixels the dedup counted (taps value_cnt_s*l* of the last profiled
    forward, the same inputs as every profiled forward)."""
    if not vp["launches"]:
        return None
    live = 0
    algo_bytes = []
    for s in range(args.denoise_steps):
        for l in range(2):
            cnt = model.tap(f"value_cnt_s{s}l{l}")[:B].view(torch.int32).cpu().numpy()
            live += int(cnt.sum())
            algo_bytes.append(value_proj_algo_bytes(model.tap(f"value_taps_s{s}l{l}").view(torch.int32).cpu().numpy(),
                                                    cnt, B))
    per_launch_live = live / (2 * args.denoise_steps)
    live_flops = 2.0 * live * 256 * 2304 * prof_steps
    sec = vp["ms"] * 1e-3
    live_tf = live_flops / sec / 1e12
    return {"launches_per_step": vp["launches"] // prof_steps,
            "avg_launch_ms": round(vp["ms"] / vp["launches"], 5),
            "slots_per_launch": B * 640, "live_rows_per_launch": round(per_launch_live, 1),
            "live_tflops": round(live_tf, 2),
            "live_frac_of_f16x3_ceiling": round(live_tf / ALGO_PEAK["f16x3"], 4),
            "live_mfma_equiv_util": round(live_tf * 3 / F16_MFMA_SUSTAINED_TFLOPS, 4),
            "algorithmic_bytes_per_launch": round(float(np.mean(algo_bytes))),
            "note": "live_mfma_equiv_util = live-row f16 MFMA FLOP rate (3 products per MAC) / the measured sustained "
                    "whole-chip f16 MFMA rate; the PMC MFMA-busy of the same launches is in profiles/. "
                    "algorithmic_bytes_per_launch: the distinct map pixels of the live rows' 3x3 neighbourhoods "
                    "(1 KB each) + the live output rows (1 KB each) + the split weight image (2304 x 256 x 4 B), "
                    "averaged over the forward's launches"}


def value_proj_algo_bytes(taps, counts, B, hw=64, C=256):
    """Algorithmic HBM bytes of one gathered value_proj launch: every map pixel some live row's 3x3 neighbourhood
    covers, read once; every live output row written once; the f16x3 weight image (hi + lo fp16) read once. ``taps``
    holds each scene's distinct pixel indices (n * hw * hw + y * hw + x) at [b * cap, b * cap + counts[b])."""
    cap = taps.size // B
    px = np.concatenate([taps[b * cap:b * cap + int(counts[b])] for b in range(B)]).astype(np.int64)
    n, y, x = px // (hw * hw), (px // hw) % hw, px % hw
    cover = set()
    for dy in (-1, 0, 1):
        for dx in (-1, 0, 1):
            yy, xx = y + dy, x + dx
            ok = (yy >= 0) & (yy < hw) & (xx >= 0) & (xx < hw)
            cover.update(((n * hw + yy) * hw + xx)[ok].tolist())
    return (len(cover) + px.size) * C * 4 + 9 * C * C * 4


def completion_intervals(e_start, marks, lanes):
    """Per-step intervals of a timed run from its step-completion events (``marks``: (start, end) HIP events, one
    pair per step, recorded on the stream each step ran on). With several lanes the completions need not arrive in
    issue order, so the end times are read against one start event on the device clock and SORTED; the interval is
    then taken over a window of ``lanes`` consecutive completions ((c[i + L] - c[i]) / L), which is the steady-state
    step time whether the lanes finish evenly staggered or in bursts. One lane: consecutive differences."""
    ends = sorted(e_start.elapsed_time(e1) for _, e1 in marks)
    L = max(1, min(int(lanes), len(ends) - 1))
    if len(ends) < 2:
        return [ends[0]] if ends else [0.0]
    return [(ends[i + L] - ends[i]) / L for i in range(len(ends) - L)]


def golden_l2(traj, arch, batch, steps):
    """Waypoint L2 of the first 64 scenes of ``traj`` against the committed reference golden of that batch
    (tests/golden/ref_b64_s1234.npz: the reference model's own output on seeded weights 0 and bench.py's rank-0 /
    global-batch-shard-0 inputs and noise), or None when the run is not that workload."""
    path = os.path.join(ROOT, "tests", "golden", "ref_b64_s1234.npz")
    if arch != "resnet34" or steps != 2 or len(traj) < 64 or not os.path.exists(path):
        return None
    with np.load(path, allow_pickle=False) as z:
        ref = z["trajectory"]
    return waypoint_l2(np.asarray(traj)[:64], ref)


def waypoint_l2(a, b):
    d = (np.asarray(a, np.float64)[..., :2] - np.asarray(b, np.float64)[..., :2]).reshape(len(a), -1)
    return float(np.sqrt((d ** 2).sum(-1)).max())


def cpu_share():
    """Host threads this job may use: min(sched affinity, the cgroup CPU quota, $OMP_NUM_THREADS) - the GPU box
    shows the whole machine's CPUs to nproc / os.cpu_count() but grants one job a share of them."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = max(1, -(-int(q) // int(per)))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    omp = int(omp) if omp and omp.isdigit() and int(omp) > 0 else None
    share = min(v for v in (aff, quota, omp) if v is not None)
    return share, {"sched_getaffinity": aff, "cgroup_cpu_max": quota, "OMP_NUM_THREADS": omp,
                   "os_cpu_count": os.cpu_count()}


def cpu_baseline(args, cfg, sd, inp):
    """Golden-pinned CPU oracle timed on this host at the job's CPU share (cpu_share): B = 64 (the metric's
    batch, 3 timed reps after an untimed B = 1 and B = 64 warm-up) and B = 1 (3 reps); --cpu-threads adds thread counts.
    Returns (record, oracle trajectories of the B = 64 sample)."""
    from oracle.model import OracleModel
    om = OracleModel(sd, cfg)
    S = inp["status_feature"].shape[0]
    keys = ("camera_feature", "lidar_feature", "status_feature", "noise")
    REPS = 3

    def run(n):
        return om.forward(*(inp[k][:n] for k in keys), steps=args.denoise_steps, heads=False)["trajectory"].numpy()

    share, share_src = cpu_share()
    threads = [share] + [int(t) for t in args.cpu_threads.split(",") if t and int(t) != share]
    grid, ref = {}, None
    for i_t, n_t in enumerate(threads):
        torch.set_num_threads(n_t)
        run(1)  # warm-up
        if i_t == 0:
            ref = run(S)  # warm-up of the batch shape (first-touch allocations); its result is the parity reference
        t0 = time.perf_counter()
        for _ in range(REPS):
            run(1)
        b1 = REPS / (time.perf_counter() - t0)
        reps = REPS
        times = []
        for _ in range(reps):
            t0 = time.perf_counter()
            r = run(S)
            times.append(time.perf_counter() - t0)
            if ref is None:
                ref = r
        bs = S / float(np.median(times))
        grid[f"threads={n_t}"] = {f"B={S}": round(bs, 4), "B=1": round(b1, 4), f"B={S}_reps": reps,
                                  f"B={S}_s_per_rep": [round(t, 3) for t in times]}
    head = share
    cpu_name = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_name = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    rec = {
        "value": grid[f"threads={head}"][f"B={S}"],
        "unit": "scenes/s",
        "cores": head,
        "kind": "port",
        "sample": f"the timed {S}-scene batch x {REPS} reps (median rep; and 1 scene x {REPS} reps) at {head} threads "
                  f"(oracle/model.py, PyTorch-CPU fp32, {cpu_name}; {os.cpu_count()} host CPUs visible, "
                  f"{head} = this job's CPU share: min of the sources in cpu_share)",
        "cpu_share": share_src,
        "grid": grid,
    }
    return rec, ref


class LaneSteps:
    """The timed step of the bench: the next lane of an InFlightPlanner runs ``body(model, stream)`` (the forward),
    then the rank's trajectories are all-gathered (ScenePlanner.gather: one RCCL all_gather_into_tensor) on the same
    lane stream, bracketed by two events recorded there. Every rank issues its collectives in step order whatever
    lane a step takes, and no forward waits for a later collective, so lanes cannot deadlock the ring. The CPU
    plumbing path (gloo, stand-in lanes) runs this same class."""

    def __init__(self, pl, planner, new_event, current_stream):
        self.pl, self.planner = pl, planner
        self.new_event, self.current_stream = new_event, current_stream
        self.marks = []        # per step: (start, end) events on the stream the step ran on
        self.last_local = None  # this rank's own trajectories of the latest step (checked against its gathered slice)
        self.issue = []         # per step: (lane index, the lane's stream) in issue order

    def step(self, body):
        i = self.pl.next_index
        with self.pl.next_lane() as m:
            s = self.current_stream()
            e0, e1 = self.new_event(), self.new_event()
            e0.record(s)
            local = body(m, s)
            o = self.planner.gather(local)
            e1.record(s)
            self.marks.append((e0, e1))
            self.issue.append((i, s))
            self.last_local = local
            return o


def gather_slices_ok(gathered, local, rank, B, dist=None, dev=None):
    """The all_gather output holds every rank's shard in rank order: each rank checks its own slice against the
    trajectories it computed (bit for bit), and the ranks agree on the result (MIN over ranks)."""
    ok = bool(np.array_equal(gathered[rank * B:(rank + 1) * B].detach().cpu().numpy(), local.detach().cpu().numpy()))
    if dist is not None:
        t = torch.tensor([1 if ok else 0], device=dev, dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        ok = bool(t.item())
    return ok


def plumbing(args, world, rank):
    """CPU stand-in for the multi-rank path (tests): gloo process group, bench's own LaneSteps over an InFlightPlanner
    of ``--in-flight`` stand-in lanes (the real round-robin, the real ScenePlanner all_gather per step, the real
    gather check), barrier + max-over-ranks timing, rank-0 JSON. A lane's forward is a stand-in that returns
    rank * 1000 + step for its scenes and records which lane issued which step."""
    import torch.distributed as dist
    from diffusiondrive_amd.dist import ScenePlanner
    from diffusiondrive_amd.model import InFlightPlanner
    if world > 1:
        dist.init_process_group("gloo")
        world = dist.get_world_size()
    B = args.batch

    class _Stream:  # a lane stream: records what was issued on it
        def __init__(self, k):
            self.k, self.log = k, []

        def wait_stream(self, other):
            pass

        def synchronize(self):
            pass

    class _Event:
        def record(self, s):
            s.log.append("event")

    class _Planner(InFlightPlanner):
        cur = [None]

        def _new_stream(self):
            return _Stream(0)  # numbered below

        def _current_stream(self):
            return _Planner.cur[0] or _main

        def _on_stream(self, s):
            import contextlib

            @contextlib.contextmanager
            def ctx():
                prev, _Planner.cur[0] = _Planner.cur[0], s
                try:
                    yield
                finally:
                    _Planner.cur[0] = prev
            return ctx()

    class _Lane:
        device = 0

        def __init__(self):
            self.streams = 2

        def set_streams(self, n):
            self.streams = n

    _main = _Stream(-1)
    lanes_in = [_Lane() for _ in range(args.in_flight)]
    pl = _Planner(models=lanes_in, lane_streams=args.lane_streams)
    for k, st in enumerate(pl.streams):
        if st is not None:
            st.k = k
    planner = ScenePlanner(None)
    lanes = LaneSteps(pl, planner, _Event, pl._current_stream)
    step_no = [0]

    def body(m, s):
        step_no[0] += 1
        s.log.append(("forward", step_no[0]))
        return torch.full((B, 8, 3), float(rank * 1000 + step_no[0]))

    for _ in range(args.warmup):
        lanes.step(body)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = lanes.step(body)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    ranks_seen = sorted({int(v) // 1000 for v in out[:, 0, 0].tolist()})
    # every rank's slice of the last gather came from the same step (collectives issued in step order on all ranks)
    steps_seen = sorted({int(v) % 1000 for v in out[:, 0, 0].tolist()})
    gather_ok = gather_slices_ok(out, lanes.last_local, rank, B, dist if world > 1 else None)
    lane_order = [i for i, _ in lanes.issue]
    lane_streams_ok = all((s is None and len(pl) == 1) or (s is not None and s.k == i) for i, s in lanes.issue)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": round(B * world * args.steps / el, 3), "unit": "scenes/s",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True,
                          "scaling": "weak", "vs_baseline": None, "dtype": "none",
                          "data": "plumbing test: stand-in step, no forward (CPU, gloo)",
                          "config": {"workload": "plumbing", "batch_per_gpu": B, "global_batch": B * world,
                                     "gathered_rows": int(out.shape[0]), "ranks_seen": ranks_seen,
                                     "in_flight": args.in_flight},
                          "lanes": {"issue_order": lane_order, "each_step_on_its_lane_stream": lane_streams_ok,
                                    "last_gather_steps": steps_seen,
                                    "lane_stream_logs": [[e if isinstance(e, str) else list(e) for e in s.log]
                                                         for s in pl.streams if s is not None]},
                          "gather_check": {"gathered_rows": int(out.shape[0]),
                                           "every_rank_slice_equals_local": gather_ok}}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
