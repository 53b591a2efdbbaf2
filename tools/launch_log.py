#!/usr/bin/env python3
"""Per-launch conv_gemm breakdown of one B=64 forward (HIP events on the handle's stream).

    python tools/launch_log.py [--batch 64] [--reps 3] [--out gpurun_out/launches.md]

Runs the bench workload with profiling on and $DDMI_LAUNCH_LOG set, then groups the launches by
shape (M, N, K, kernel size, stride, z-batch) and prints device ms, TFLOP/s and the fraction of the
fp32 MFMA peak per shape class, largest time first. GPU only.
"""
import argparse
import collections
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PEAK = 157.3
PEAK_X3 = 2500.0 / 3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--arch", default="resnet34")
    ap.add_argument("--gemm", default="f16x3")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "launches.md"))
    a = ap.parse_args()
    log = tempfile.NamedTemporaryFile(prefix="ddmi_launch_", suffix=".tsv", delete=False).name
    os.environ["DDMI_LAUNCH_LOG"] = log
    import torch
    from diffusiondrive_amd.config import TransfuserConfig
    from diffusiondrive_amd.model import DiffusionDriveModel
    from diffusiondrive_amd.weights import seeded_state_dict, synthetic_inputs

    cfg = TransfuserConfig(image_architecture=a.arch)
    model = DiffusionDriveModel(cfg, seeded_state_dict(cfg, 0), device=0)
    model.set_gemm_mode(a.gemm)
    inp = synthetic_inputs(a.batch, 1234, cfg)
    feats = {k: torch.from_numpy(inp[k]).cuda() for k in ("camera_feature", "lidar_feature", "status_feature")}
    noise = torch.from_numpy(inp["noise"]).cuda()
    model.forward(feats, noise=noise)
    model.set_profiling(True)
    open(log, "w").close()
    for _ in range(a.reps):
        model.forward(feats, noise=noise)
    torch.cuda.synchronize()
    model.kernel_stats("conv_gemm")  # drains pending events -> log
    model.set_profiling(False)

    groups = collections.OrderedDict()
    other = collections.defaultdict(float)
    total = 0.0
    with open(log) as f:
        for line in f:
            name, detail, flops, ms = line.rstrip("\n").split("\t")[:4]
            ms = float(ms) / a.reps
            total += ms
            if not detail:
                other[name] += ms
                continue
            g = groups.setdefault(f"{name} {detail}", [0, 0.0, 0.0])
            g[0] += 1
            g[1] += float(flops) / a.reps
            g[2] += ms
    rows = sorted(groups.items(), key=lambda kv: -kv[1][2])
    lines = [f"# conv / GEMM launches per forward (B={a.batch}, {a.arch}, gemm={a.gemm}); forward device total {total:.2f} ms", "",
             "| kernel / shape | launches | ms | GFLOP | TFLOP/s | frac fp32 peak | frac f16x3 ceiling | share |", "|---|---|---|---|---|---|---|---|"]
    cg_ms = sum(v[2] for _, v in rows)
    cg_fl = sum(v[1] for _, v in rows)
    for d, (n, fl, ms) in rows:
        n //= a.reps
        tf = fl / (ms * 1e-3) / 1e12 if ms else 0
        lines.append(f"| {d} | {n} | {ms:.3f} | {fl / 1e9:.1f} | {tf:.1f} | {tf / PEAK:.3f} | {tf / PEAK_X3:.3f} | "
                     f"{ms / total:.3f} |")
    lines.append(f"| **GEMM / conv total** | | {cg_ms:.3f} | {cg_fl / 1e9:.1f} | {cg_fl / cg_ms / 1e9:.1f} | "
                 f"{cg_fl / cg_ms / 1e9 / PEAK:.3f} | {cg_fl / cg_ms / 1e9 / PEAK_X3:.3f} | {cg_ms / total:.3f} |")
    by_k = collections.defaultdict(lambda: [0.0, 0.0])
    for d, (n, fl, ms) in rows:
        by_k[d.split()[0]][0] += ms
        by_k[d.split()[0]][1] += fl
    for k, (ms, fl) in sorted(by_k.items(), key=lambda kv: -kv[1][0]):
        lines.append(f"| {k} (all shapes) | | {ms:.3f} | {fl / 1e9:.1f} | {fl / ms / 1e9:.1f} | | | {ms / total:.3f} |")
    for k, v in sorted(other.items(), key=lambda kv: -kv[1]):
        lines.append(f"| {k} | | {v:.3f} | | | | | {v / total:.3f} |")
    txt = "\n".join(lines) + "\n"
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        f.write(txt)
    print(txt)


if __name__ == "__main__":
    main()
