#!/usr/bin/env python3
"""Benchmark: DiffusionDrive eval forward (ResNet-34 + LiDAR-BEV backbone, 2 truncated DDIM
steps) on MI355X, scenes/s at batch 64 per GPU (BASELINE.json metric / configs[1], weak scaling
over 1/2/4/8 GPUs with one RCCL all_gather of the predicted trajectories per step).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (N > 1)

A step = one forward of B synthetic scenes resident in HBM (+ the all_gather when N > 1).
Rank 0 prints ONE JSON line. Also reported:
  * roofline: the dominant kernel (the conv / GEMM kernel with the most device time in the
    profiled replay: conv_x6 for the default f16x3 path, conv_gemm for --gemm fp32), algorithmic
    FLOP per launch / average launch time from HIP events recorded on the kernel's stream during a
    profiled replay of the timed workload; peak = the algorithmic fp32 ceiling of the gemm mode
    (157.3 TFLOP/s fp32 MFMA dense, or 2500 / 3 TFLOP/s for the 3-product f16 split,
    MI355X_MICROARCH.md).
  * cpu_baseline: the golden-pinned CPU oracle (oracle/, PyTorch-CPU fp32) timed on this host
    on a bounded sample of the same workload (rank 0, N = 1 only); its outputs double as the
    waypoint-L2 parity check of the GPU result on those scenes.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

CANONICAL_GFLOP_PER_SCENE_2STEP = 65.27  # SURVEY.md §8d (value_proj once per layer)
FP32_MFMA_PEAK_TFLOPS = 157.3            # MI355X dense fp32 MFMA (= vector) peak
F16_MFMA_PEAK_TFLOPS = 2500.0            # MI355X dense f16 MFMA peak (no sparsity)
# peak of ALGORITHMIC fp32 FLOPs per gemm mode: f16x3 issues 3 f16 MFMA products per fp32 MAC
ALGO_PEAK = {"fp32": FP32_MFMA_PEAK_TFLOPS, "f16x3": F16_MFMA_PEAK_TFLOPS / 3}
KERNEL_DESC = {
    "conv_gemm": "conv_gemm (implicit-GEMM conv / GEMM, fp32 MFMA v_mfma_f32_32x32x2_f32)",
    "conv_x3": "conv_x3 (implicit-GEMM conv / GEMM, 3-product fp16 split on v_mfma_f32_32x32x16_f16)",
    "conv_x5": "conv_x5 (implicit-GEMM conv, LDS-DMA staging, 3-product fp16 split on v_mfma_f32_32x32x16_f16)",
    "conv_x6": "conv_x6 (halo-reuse direct 3x3 conv, 3-product fp16 split on v_mfma_f32_32x32x16_f16)",
    "gemm_lat": "gemm_lat (whole-K small GEMM, fp32 MFMA v_mfma_f32_16x16x4_f32)",
}
CONV_KERNELS = ("conv_x6", "conv_x5", "conv_x3", "conv_gemm", "gemm_lat")
DTYPE = {
    "fp32": "fp32",
    "f16x3": "fp32 via f16x3 (each fp32 operand = hi+lo fp16, products ah*bh+ah*bl+al*bh, fp32 accumulate)",
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--batch", type=int, default=64, help="scenes per GPU")
    p.add_argument("--denoise-steps", type=int, default=2)
    p.add_argument("--cpu-sample", type=int, default=64, help="scenes in the CPU-oracle baseline sample")
    p.add_argument("--cpu-reps", type=int, default=3)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--arch", default="resnet34")
    p.add_argument("--gemm", default="f16x3", choices=["fp32", "f16x3"],
                   help="conv/linear arithmetic: fp32 MFMA or the fp32-class 3-product fp16 split")
    p.add_argument("--no-compare", action="store_true", help="skip the fp32-path comparison timing")
    return p.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    else:
        torch.cuda.set_device(0)
    dev = torch.device(f"cuda:{local}")

    from diffusiondrive_amd.config import TransfuserConfig
    from diffusiondrive_amd.model import DiffusionDriveModel
    from diffusiondrive_amd.weights import seeded_state_dict, synthetic_inputs

    cfg = TransfuserConfig(image_architecture=args.arch)
    sd = seeded_state_dict(cfg, 0)
    model = DiffusionDriveModel(cfg, sd, device=local)
    model.set_gemm_mode(args.gemm)
    B = args.batch
    inp = synthetic_inputs(B, 1234 + rank, cfg)
    feats = {k: torch.from_numpy(inp[k]).to(dev) for k in ("camera_feature", "lidar_feature", "status_feature")}
    noise = torch.from_numpy(inp["noise"]).to(dev)
    from diffusiondrive_amd.dist import ScenePlanner
    planner = ScenePlanner(lambda f, nz: model.forward(f, noise=nz, steps=args.denoise_steps)["trajectory"])

    def step():
        # per-rank shard of the global batch (weak scaling) + one RCCL all_gather of trajectories
        return planner.gather(planner.fn(feats, noise))

    for _ in range(args.warmup):
        out = step()
    torch.cuda.synchronize()

    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed / args.steps * 1e3
    scenes_per_s = B * world * args.steps / elapsed
    traj_gpu = out[rank * B:(rank + 1) * B].detach().cpu().numpy()
    num_flags = model.numerics_flags()
    if num_flags:
        print(f"[bench] WARNING: numerics flags {num_flags:#x} raised (f16x3 overflow): result untrustworthy",
              file=sys.stderr)

    # ---- roofline of the dominant kernel: a profiled replay of the same workload (HIP events
    # around every conv_gemm launch on the handle's stream)
    model.set_profiling(True)
    model.reset_stats()
    prof_steps = max(1, min(args.steps, 5))
    for _ in range(prof_steps):
        model.forward(feats, noise=noise, steps=args.denoise_steps)
    torch.cuda.synchronize()
    conv_stats = {k: model.kernel_stats(k) for k in CONV_KERNELS}
    main_k = max(CONV_KERNELS, key=lambda k: conv_stats[k]["ms"])
    st = conv_stats[main_k]
    other = {k: model.kernel_stats(k) for k in ("stem_pool", "attn", "layernorm", "softmax", "bilinear", "pool", "mha", "bev_sample",
                                                 "misc")}
    other.update({k: v for k, v in conv_stats.items() if k != main_k})
    model.set_profiling(False)
    avg_ms = st["ms"] / max(st["launches"], 1)
    flops_per_launch = st["flops"] / max(st["launches"], 1)
    achieved = flops_per_launch / (avg_ms * 1e-3) / 1e12 if avg_ms > 0 else 0.0
    total_prof_ms = st["ms"] + sum(v["ms"] for v in other.values())

    # the other gemm mode on the same workload, for comparison (rank 0 view, N = 1 only)
    compare = None
    if world == 1 and not args.no_compare:
        other_mode = "fp32" if args.gemm == "f16x3" else "f16x3"
        model.set_gemm_mode(other_mode)
        for _ in range(2):
            o2 = step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n_cmp = max(3, args.steps // 2)
        for _ in range(n_cmp):
            o2 = step()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        d = (o2.detach().cpu().numpy()[..., :2].astype(np.float64) - traj_gpu[..., :2]).reshape(B, -1)
        compare = {"gemm": other_mode, "value": round(B * n_cmp / dt, 3), "ms_per_step": round(dt / n_cmp * 1e3, 3),
                   "steps": n_cmp, "waypoint_l2_vs_primary": float(np.sqrt((d ** 2).sum(-1)).max())}
        model.set_gemm_mode(args.gemm)

    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", f"pmc_{main_k}_{args.gemm}.json")
    if os.path.exists(pmc_path):
        try:
            with open(pmc_path) as f:
                traffic = json.load(f).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    result = {
        "metric": "scenes/s at batch 64, 2 denoise steps, 1/2/4/8 MI355X; waypoint L2 vs ref",
        "value": round(scenes_per_s, 3),
        "unit": "scenes/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
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
            "gemm": args.gemm,
        },
        "roofline": {
            "kernel": KERNEL_DESC[main_k],
            "bound": "mfma",
            "achieved": round(achieved, 3),
            "peak": round(ALGO_PEAK[args.gemm], 1),
            "unit": "TFLOP/s",
            "frac": round(achieved / ALGO_PEAK[args.gemm], 4),
            "peak_note": "algorithmic fp32 FLOP/s ceiling: fp32 MFMA 157.3 TF" if args.gemm == "fp32" else
                         "algorithmic fp32 FLOP/s ceiling: dense f16 MFMA 2500 TF / 3 products per fp32 MAC",
            "achieved_vs_fp32_mfma_peak": round(achieved / FP32_MFMA_PEAK_TFLOPS, 4),
            "traffic": traffic,
            "launches_per_step": st["launches"] // prof_steps,
            "avg_launch_ms": round(avg_ms, 5),
            "gflop_per_launch": round(flops_per_launch / 1e9, 4),
            "share_of_device_time": round(st["ms"] / total_prof_ms, 4) if total_prof_ms else None,
            "conv_kernels": {k: {"launches_per_step": v["launches"] // prof_steps,
                                 "avg_launch_ms": round(v["ms"] / max(v["launches"], 1), 5),
                                 "tflops": round(v["flops"] / (v["ms"] * 1e-3) / 1e12, 2) if v["ms"] else None,
                                 "share_of_device_time": round(v["ms"] / total_prof_ms, 4) if total_prof_ms else None}
                             for k, v in conv_stats.items() if v["launches"]},
        },
        "device_ms_per_step": {k: round(v["ms"] / prof_steps, 4) for k, v in
                               sorted({main_k: st, **other}.items(), key=lambda kv: -kv[1]["ms"]) if v["launches"]},
        "whole_forward": {
            "gflop_per_scene": CANONICAL_GFLOP_PER_SCENE_2STEP if args.denoise_steps == 2 else None,
            "tflops": round(scenes_per_s / world * CANONICAL_GFLOP_PER_SCENE_2STEP / 1e3, 3)
            if args.denoise_steps == 2 else None,
        },
    }
    if result["whole_forward"]["tflops"] is not None:
        result["whole_forward"]["frac_of_fp32_peak"] = round(result["whole_forward"]["tflops"] / FP32_MFMA_PEAK_TFLOPS,
                                                             4)

    result["numerics_flags"] = num_flags
    if compare is not None:
        result["compare_gemm_mode"] = compare
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args, cfg, sd, inp, traj_gpu)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def cpu_baseline(args, cfg, sd, inp, traj_gpu):
    """Golden-pinned CPU oracle on a bounded sample (first `cpu_sample` scenes of the batch)."""
    from oracle.model import OracleModel
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    torch.set_num_threads(threads)
    S = min(args.cpu_sample, inp["status_feature"].shape[0])
    om = OracleModel(sd, cfg)
    sl = {k: inp[k][:S] for k in ("camera_feature", "lidar_feature", "status_feature", "noise")}
    om.forward(sl["camera_feature"][:1], sl["lidar_feature"][:1], sl["status_feature"][:1], sl["noise"][:1],
               steps=args.denoise_steps, heads=False)  # warm-up
    t0 = time.perf_counter()
    for _ in range(args.cpu_reps):
        ref = om.forward(sl["camera_feature"], sl["lidar_feature"], sl["status_feature"], sl["noise"],
                         steps=args.denoise_steps, heads=False)["trajectory"].numpy()
    dt = time.perf_counter() - t0
    d = (traj_gpu[:S, :, :2].astype(np.float64) - ref[..., :2].astype(np.float64)).reshape(S, -1)
    l2 = float(np.sqrt((d ** 2).sum(-1)).max())
    cpu_name = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_name = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {
        "value": round(S * args.cpu_reps / dt, 4),
        "unit": "scenes/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{S} scenes x {args.cpu_reps} reps of the same synthetic batch (oracle/model.py, PyTorch-CPU "
                  f"fp32, {threads} threads, {cpu_name})",
        "seconds": round(dt, 2),
        "waypoint_l2_gpu_vs_oracle": l2,
    }


if __name__ == "__main__":
    main()
