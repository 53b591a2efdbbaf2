#!/usr/bin/env python3
"""Secondary BASELINE.json configs on one MI355X (the headline config C2 is bench.py's line).

    python tools/bench_configs.py [--out profiles/rNN_configs] [--steps 10]

* C1  batch 1 latency (the reference's per-token NAVSIM eval shape), every gemm mode.
* C2  batch 64, ResNet-34, 2 truncated DDIM steps: fp32 / f16x3 / bf16 gemm modes.
* C4  batch 64, ResNet-50 image trunk (nuScenes-style config; LiDAR stays ResNet-34): bf16 (the
      config's dtype) and the fp32-class modes, with the bf16 waypoint deviation from f16x3.
* C6  end to end from raw sensors: GPU feature builder + forward, raw data resident in HBM and
      from host memory (PCIe-inclusive), plus the feature build alone.
* C5  latency curve: truncated DDIM (reference schedule) N = 1..20 steps and vanilla
      (non-truncated, x_T = noise over 1000 train steps) N = 2..20, batch 64, f16x3.
All inputs synthetic and seeded, weights seeded random (no checkpoint download), inputs resident
in HBM, hipGraph replay, device-synchronised wall clock over `steps` forwards after warmup.
"""
import argparse
import subprocess
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def timed(model, feats, noise, steps_ddim, reps, warm=2):
    for _ in range(warm):
        model.forward(feats, noise=noise, steps=steps_ddim)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        model.forward(feats, noise=noise, steps=steps_ddim)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / reps * 1e3
    out = model.forward(feats, noise=noise, steps=steps_ddim, modes=True)
    return ms, {k: v.detach().cpu().numpy() for k, v in out.items()}


def l2(a, b):
    d = (a[..., :2].astype(np.float64) - b[..., :2].astype(np.float64)).reshape(a.shape[0], -1)
    return float(np.sqrt((d ** 2).sum(-1)).max())


def deviation(o, ref):
    """Deviation of one gemm mode's outputs from f16x3's on the same batch: waypoint L2 of the
    selected trajectory (max over scenes), the fraction of scenes selecting the same mode (argmax
    over the 20 cls logits), and the max per-mode waypoint L2 over all 20 modes (no argmax jump)."""
    same = o["poses_cls"].argmax(-1) == ref["poses_cls"].argmax(-1)
    B, Q = o["poses_reg"].shape[:2]
    return {"waypoint_l2_vs_f16x3": l2(o["trajectory"], ref["trajectory"]),
            "mode_agreement_vs_f16x3": float(same.mean()),
            "allmodes_waypoint_l2_vs_f16x3": l2(o["poses_reg"].reshape(B * Q, -1, 3),
                                               ref["poses_reg"].reshape(B * Q, -1, 3))}


def bf16_vs_reference(cfg, sd, inp, out, B):
    """A bf16 row's accuracy against the fp32 CPU oracle on the same batch, beside the reference path's OWN bf16
    (the oracle under torch.autocast(cpu, bfloat16)): selected-trajectory waypoint L2 (max over scenes) and mode
    agreement (argmax of the 20 cls logits equal). No bf16 scenes/s is quoted without these (bf16 is reduced
    precision: near-tied cls logits flip the selected mode)."""
    from oracle.model import OracleModel
    om = OracleModel(sd, cfg)
    args = (inp["camera_feature"], inp["lidar_feature"], inp["status_feature"], inp["noise"])
    ref = {k: v.numpy() for k, v in om.forward(*args, heads=False).items()}
    with torch.autocast("cpu", dtype=torch.bfloat16):
        ac = {k: v.float().numpy() for k, v in om.forward(*args, heads=False).items()}

    def stats(o):
        return l2(o["trajectory"], ref["trajectory"]), float((o["poses_cls"].argmax(-1) == ref["poses_cls"].argmax(-1)).mean())

    sel, agree = stats(out)
    asel, aagree = stats(ac)
    return {"sel_l2_vs_oracle": sel, "agree_vs_oracle": agree, "autocast_sel_l2_vs_oracle": asel,
            "autocast_agree_vs_oracle": aagree, "oracle_batch": B}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "configs"))
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--c1-child", action="store_true",
                    help="child mode: C1 batch-1 latency with --c1-streams streams, one JSON line")
    ap.add_argument("--c1-streams", type=int, default=1, choices=[1, 2], help="child mode's dd_set_streams value")
    a = ap.parse_args()
    from diffusiondrive_amd.config import TransfuserConfig
    from diffusiondrive_amd.model import DiffusionDriveModel
    from diffusiondrive_amd.weights import seeded_state_dict, synthetic_inputs

    res = {"device": torch.cuda.get_device_name(0), "reps": a.steps, "configs": {}}
    dev = torch.device("cuda:0")

    ctx = {}

    def setup(arch, B, seed=1234):
        cfg = TransfuserConfig(image_architecture=arch)
        sd = seeded_state_dict(cfg, 0)
        m = DiffusionDriveModel(cfg, sd, device=0)
        inp = synthetic_inputs(B, seed, cfg)
        ctx.update(cfg=cfg, sd=sd, inp=inp)
        feats = {k: torch.from_numpy(inp[k]).to(dev) for k in ("camera_feature", "lidar_feature", "status_feature")}
        return m, feats, torch.from_numpy(inp["noise"]).to(dev)

    if a.c1_child:  # a fresh process of its own
        m, feats, noise = setup("resnet34", 1)
        m.set_streams(a.c1_streams)
        rows = {}
        for mode in ("f16x3", "bf16", "fp32"):
            m.set_gemm_mode(mode)
            ms, _ = timed(m, feats, noise, 2, 5 * a.steps)
            rows[mode] = {"ms_per_batch": round(ms, 3), "scenes_per_s": round(1 / ms * 1e3, 2)}
        m.close()
        print("C1TWO " + json.dumps(rows), flush=True)
        return

    # ---- C1 / C2 (ResNet-34)
    for B, key in ((1, "C1_batch1_latency"), (64, "C2_batch64")):
        m, feats, noise = setup("resnet34", B)
        rows, outs = {}, {}
        for mode in ("fp32", "f16x3", "bf16"):
            m.set_gemm_mode(mode)
            ms, outs[mode] = timed(m, feats, noise, 2, a.steps if B > 1 else 5 * a.steps)
            rows[mode] = {"ms_per_batch": round(ms, 3), "scenes_per_s": round(B / ms * 1e3, 2),
                          "numerics_flags": m.numerics_flags()}
        rows["bf16"].update(deviation(outs["bf16"], outs["f16x3"]))
        rows["fp32"].update(deviation(outs["fp32"], outs["f16x3"]))
        rows["bf16"].update(bf16_vs_reference(ctx["cfg"], ctx["sd"], ctx["inp"], outs["bf16"], B))
        res["configs"][key] = {"arch": "resnet34", "batch": B, "ddim_steps": 2, "modes": rows}
        print(key, json.dumps(rows), flush=True)
        m.close()

    # ---- C4 (ResNet-50 image trunk)
    m, feats, noise = setup("resnet50", 64)
    rows, outs = {}, {}
    for mode in ("bf16", "f16x3", "fp32"):
        m.set_gemm_mode(mode)
        ms, outs[mode] = timed(m, feats, noise, 2, a.steps)
        rows[mode] = {"ms_per_batch": round(ms, 3), "scenes_per_s": round(64 / ms * 1e3, 2),
                      "numerics_flags": m.numerics_flags()}
    rows["bf16"].update(deviation(outs["bf16"], outs["f16x3"]))
    rows["fp32"].update(deviation(outs["fp32"], outs["f16x3"]))
    rows["bf16"].update(bf16_vs_reference(ctx["cfg"], ctx["sd"], ctx["inp"], outs["bf16"], 64))
    res["configs"]["C4_resnet50_batch64"] = {"arch": "resnet50", "batch": 64, "ddim_steps": 2, "modes": rows,
                                             "gflop_per_scene_note": "SURVEY §8d probe: 162.2 GFLOP/scene"}
    print("C4", json.dumps(rows), flush=True)
    m.close()

    # ---- C5 latency curve (f16x3)
    m, feats, noise = setup("resnet34", 64)
    m.set_gemm_mode("f16x3")
    curve = {"truncated": {}, "vanilla": {}}
    for n in (1, 2, 4, 6, 8, 10, 20):
        ms, _ = timed(m, feats, noise, n, a.steps)
        curve["truncated"][n] = round(ms, 3)
    m.set_schedule("vanilla")
    for n in (2, 5, 10, 20):
        ms, _ = timed(m, feats, noise, n, a.steps)
        curve["vanilla"][n] = round(ms, 3)
    m.set_schedule("truncated")
    res["configs"]["C5_ddim_latency_batch64"] = {"arch": "resnet34", "batch": 64, "gemm": "f16x3",
                                                 "ms_per_batch_by_steps": curve}
    print("C5", json.dumps(curve), flush=True)
    m.close()

    # ---- end to end from raw sensors (GPU feature builder + forward), batch 64, f16x3
    from diffusiondrive_amd import _lib
    from diffusiondrive_amd.features import camera_features, lidar_features
    m, feats, noise = setup("resnet34", 64)
    cfg = m.config
    r = np.random.default_rng(0)
    B, NPTS = 64, 100_000
    imgs = r.integers(0, 256, (B, 3, 1080, 1920, 3), dtype=np.uint8)
    pcs = [np.stack([r.uniform(-40, 40, NPTS), r.uniform(-40, 40, NPTS), r.uniform(-1, 3, NPTS)]).astype(np.float32)
           for _ in range(B)]
    cams_d = torch.from_numpy(imgs).to(dev)
    offs = torch.from_numpy(np.arange(B + 1, dtype=np.int64) * NPTS).to(dev)
    xyz_d = torch.from_numpy(np.concatenate([p.reshape(-1) for p in pcs])).to(dev)
    cam_o = torch.empty((B, 3, 256, 1024), device=dev)
    lid_o = torch.empty((B, 1, 256, 256), device=dev)
    lib = _lib.load()

    def build_resident():
        st = torch.cuda.current_stream().cuda_stream
        _lib.check(lib.dd_build_camera(cams_d.data_ptr(), B, 1080, 1920, cam_o.data_ptr(), 256, 1024, st), lib, op=True)
        _lib.check(lib.dd_build_lidar(xyz_d.data_ptr(), offs.data_ptr(), B, 1, lid_o.data_ptr(), 256, -32.0, 32.0, 4,
                                      100.0, 0.2, 5, NPTS, st), lib, op=True)

    def e2e(resident):
        if resident:
            build_resident()
            f = {"camera_feature": cam_o, "lidar_feature": lid_o, "status_feature": feats["status_feature"]}
        else:
            f = {"camera_feature": camera_features([tuple(imgs[b]) for b in range(B)], cfg, 0),
                 "lidar_feature": lidar_features(pcs, cfg, 0), "status_feature": feats["status_feature"]}
        return m.forward(f, noise=noise)

    e2e_rows = {}
    for name, resident in (("raw_sensors_resident_in_hbm", True), ("raw_sensors_from_host_incl_h2d", False)):
        for _ in range(2):
            e2e(resident)
        torch.cuda.synchronize()
        reps = a.steps if resident else max(2, a.steps // 3)
        t0 = time.perf_counter()
        for _ in range(reps):
            e2e(resident)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / reps * 1e3
        e2e_rows[name] = {"ms_per_batch": round(ms, 3), "scenes_per_s": round(B / ms * 1e3, 2)}
    # the batched runner's pipelining (runner.py _run_batches): batch i+1's host staging while batch i's forward runs
    def host_feats():
        return {"camera_feature": camera_features([tuple(imgs[b]) for b in range(B)], cfg, 0),
                "lidar_feature": lidar_features(pcs, cfg, 0), "status_feature": feats["status_feature"]}

    reps = max(2, a.steps // 3)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    prev = None
    for _ in range(reps):
        f = host_feats()
        if prev is not None:
            prev["trajectory"].cpu()
        prev = m.forward(f, noise=noise)
    prev["trajectory"].cpu()
    ms = (time.perf_counter() - t0) / reps * 1e3
    e2e_rows["raw_sensors_from_host_pipelined"] = {"ms_per_batch": round(ms, 3), "scenes_per_s": round(B / ms * 1e3, 2)}
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        build_resident()
    torch.cuda.synchronize()
    fb = (time.perf_counter() - t0) / a.steps * 1e3
    e2e_rows["feature_build_only_resident"] = {"ms_per_batch": round(fb, 3), "scenes_per_s": round(B / fb * 1e3, 2),
                                               "raw_bytes_per_scene": int(3 * 1080 * 1920 * 3 + 12 * NPTS)}
    res["configs"]["C6_end_to_end_raw_sensors_batch64"] = {"gemm": "f16x3", "points_per_scene": NPTS,
                                                           "rows": e2e_rows}
    print("C6", json.dumps(e2e_rows), flush=True)
    m.close()

    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out + ".json", "w") as f:
        json.dump(res, f, indent=1)
    lines = [f"# Secondary configs ({res['device']}, synthetic seeded inputs/weights, hipGraph replay, "
             f"{a.steps} reps)", "",
             "| config | gemm | ms / batch | scenes/s | waypoint L2 vs f16x3 | mode agreement | all-mode L2 | "
             "bf16: selected L2 vs fp32 oracle (reference bf16 autocast) | bf16: mode agreement vs oracle (autocast) |",
             "|---|---|---|---|---|---|---|---|---|"]
    for key, c in res["configs"].items():
        if "modes" not in c:
            continue
        for mode, r in c["modes"].items():
            g = lambda k: (f"{r[k]:.3g}" if k in r else "-")  # noqa: E731
            lines.append(f"| {key} | {mode} | {r['ms_per_batch']} | {r['scenes_per_s']} | "
                         f"{g('waypoint_l2_vs_f16x3')} | {g('mode_agreement_vs_f16x3')} | "
                         f"{g('allmodes_waypoint_l2_vs_f16x3')} | "
                         f"{g('sel_l2_vs_oracle')} ({g('autocast_sel_l2_vs_oracle')}) | "
                         f"{g('agree_vs_oracle')} ({g('autocast_agree_vs_oracle')}) |")
    lines += ["", "C5 latency (ms per batch of 64, f16x3) by DDIM steps:", "",
              "| schedule | " + " | ".join(f"N={n}" for n in (1, 2, 4, 5, 6, 8, 10, 20)) + " |",
              "|---|" + "---|" * 8]
    for sch, cv in curve.items():
        lines.append(f"| {sch} | " + " | ".join(str(cv.get(n, "-")) for n in (1, 2, 4, 5, 6, 8, 10, 20)) + " |")
    lines += ["", "C6 end to end from raw sensors (3 x 1080x1920 uint8 cameras + 100k LiDAR points per scene), "
                  "batch 64, f16x3:", "", "| path | ms / batch | scenes/s |", "|---|---|---|"]
    for k, v in e2e_rows.items():
        lines.append(f"| {k} | {v['ms_per_batch']} | {v['scenes_per_s']} |")
    # C1 on a single-stream handle (the tables above use the default two-stream handle), in a child process
    r2 = subprocess.run([sys.executable, os.path.abspath(__file__), "--c1-child", "--c1-streams", "1",
                         "--steps", str(a.steps)], capture_output=True, text=True, timeout=600)
    two = [ln for ln in r2.stdout.splitlines() if ln.startswith("C1TWO ")]
    lines += ["", "C1 batch-1 latency on a single-stream handle (dd_set_streams(h, 1); fresh process; the rows above "
              "are the default two-stream handle):", "", "| gemm | ms / batch | scenes/s |", "|---|---|---|"]
    if r2.returncode == 0 and two:
        rows2 = json.loads(two[-1][6:])
        res["configs"]["C1_batch1_latency_single_stream"] = {"arch": "resnet34", "batch": 1, "ddim_steps": 2,
                                                             "streams": 1, "modes": rows2}
        lines += [f"| {k} | {v['ms_per_batch']} | {v['scenes_per_s']} |" for k, v in rows2.items()]
    else:
        lines.append(f"| (child exited {r2.returncode}) | - | - |")
    with open(a.out + ".json", "w") as f:
        json.dump(res, f, indent=1)
    with open(a.out + ".md", "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
