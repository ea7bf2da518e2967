#!/usr/bin/env python
"""Depth Anything V2 throughput on MI355X through the HIP engine.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--encoder vits]

One *step* = one forward of the packed DA-V2 engine over one batch of B
synthetic 518x518 images already resident in HBM (input fp32 NCHW, output
fp32 depth), enqueued on one HIP stream, replayed from the engine's
captured hipGraph.  N > 1: one process per GPU (torch.distributed.run),
each rank an independent replica on its own batch shard -- no collective on
the data path; a gloo barrier brackets the timed region and
the max time over ranks is used.  `value` = images processed by all ranks /
that time (weak scaling: per-GPU batch fixed).

Also measured (rank 0):
  * b1_*: the reference's own methodology (core/bench.py:182-210): batch 1,
    wall clock of one do_inference() = pinned H2D + forward + D2H + sync,
    20 warmup / 100 iterations, with the StageTimer split -- the number to
    hold against the RTX-3080 TensorRT 4.31 ms / 232.11 FPS;
    b1_u8_*: the same with the uint8-NHWC engine (on-device normalisation),
    against the reference's uint8 A/B 294.07 FPS.
  * roofline: the dominant layer class (largest share of forward time), its
    algorithmic FLOP per launch / its average launch time, timed live with
    hipEvents on the engine's stream (the engine profiler), vs the dense
    fp16 MFMA peak (2.5 PF/s, MI355X_MICROARCH.md).
  * cpu_baseline (N == 1 only): the oracle's fp32 CPU forward (a PyTorch
    restatement of upstream DA-V2) on this host's cores, bounded sample.
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MFMA_PEAK_TFLOPS = 2500.0   # dense fp16/bf16 MFMA, MI355X (MI355X_MICROARCH.md chip table)
ENC_LABEL = {"vits": "ViT-S", "vitb": "ViT-B", "vitl": "ViT-L"}
REF_B1_FPS = 232.11         # RTX 3080 TRT fp16, BASELINE.md
REF_B1_U8_FPS = 294.07      # same, uint8-NHWC input engine (reports/uint8_ab/depth_anything_v2.json)


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch", type=int, default=32, help="images per GPU per step")
    p.add_argument("--encoder", default="vits", choices=["vits", "vitb", "vitl"])
    p.add_argument("--size", type=int, default=518)
    p.add_argument("--b1-iters", type=int, default=100)
    p.add_argument("--b1-warmup", type=int, default=20)
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-b1", action="store_true")
    p.add_argument("--profile-iters", type=int, default=3)
    p.add_argument("--layers-json", default="", help="write the per-layer profile here (rank 0)")
    return p.parse_args()


class LayerTimes:
    def __init__(self):
        self.ms = {}

    def report_layer_time(self, name, ms):
        self.ms.setdefault(name, []).append(ms)


def profile_layers(ctx, stream, iters):
    """Per-layer hipEvent timings of the same forward (eager launches)."""
    import torch
    prof = LayerTimes()
    ctx.profiler = prof
    for _ in range(iters):
        ctx.execute_async_v3(stream)
    torch.cuda.synchronize()
    ctx.profiler = None
    return {k: statistics.median(v) for k, v in prof.ms.items()}


# layer class -> kernel symbol substring in rocprofv3 traces (classes whose
# launches map to one kernel template; GEMM classes share gemm_kernel<...>)
CLASS_KERNEL = {"attn": "attn_fwd_kernel"}


def pmc_traffic(cls, cfg, B, size):
    """HBM bytes per launch of the dominant class's kernel from the committed
    PMC profile of this workload (tools/profile_round.sh -> profiles/
    traffic_<enc>_b<B>.json: FETCH_SIZE x2 + WRITE_SIZE, separate passes), or
    None.  Attention is matched by kernel name and grid size."""
    path = os.path.join(ROOT, "profiles", f"traffic_{cfg['encoder']}_b{B}_{size}.json")
    sub = CLASS_KERNEL.get(cls)
    if not sub or not os.path.exists(path):
        return None, None
    with open(path) as f:
        d = json.load(f)
    grid = None
    if cls == "attn":
        grid = ((1370 if size == 518 else (size // 14) ** 2 + 1) + 127) // 128 * B * cfg["num_heads"] * 512
    for r in d["kernels"]:
        if sub in r["kernel"] and (grid is None or r["grid"] == grid):
            return r["hbm_bytes_per_launch"], os.path.relpath(path, ROOT)
    return None, None


def roofline(cfg, B, size, layer_ms):
    from monocular_depth_estimation_trt_amd import flops
    lf = flops.layer_flops(cfg, size, size, B)
    cls_ms, cls_fl, cls_n = {}, {}, {}
    for name, ms in layer_ms.items():
        c = flops.layer_class(name)
        cls_ms[c] = cls_ms.get(c, 0.0) + ms
        cls_fl[c] = cls_fl.get(c, 0.0) + lf.get(name, 0.0)
        cls_n[c] = cls_n.get(c, 0) + 1
    dom = max((c for c in cls_ms if cls_fl.get(c, 0) > 0), key=lambda c: cls_ms[c])
    per_launch_fl = cls_fl[dom] / cls_n[dom]
    avg_ms = cls_ms[dom] / cls_n[dom]
    achieved = per_launch_fl / (avg_ms * 1e-3) / 1e12
    breakdown = {c: {"ms": round(cls_ms[c], 4), "launches": cls_n[c],
                     "tflops": round(cls_fl[c] / (cls_ms[c] * 1e-3) / 1e12, 1) if cls_fl.get(c) else None}
                 for c in sorted(cls_ms, key=lambda c: -cls_ms[c])}
    traffic, src = pmc_traffic(dom, cfg, B, size)
    roof = {"bound": "mfma", "kernel": dom, "achieved": round(achieved, 2), "peak": MFMA_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": round(achieved / MFMA_PEAK_TFLOPS, 4), "traffic": traffic,
            "flop_per_launch": per_launch_fl, "avg_launch_ms": round(avg_ms, 5),
            "launches_per_step": cls_n[dom]}
    if traffic is not None:
        roof["traffic_unit"] = "bytes/launch"
        roof["traffic_source"] = src
    return roof, breakdown


def b1_reference_method(blob, dev, size, warmup, iters, u8=False, prefix="b1_"):
    """Batch-1 wall clock exactly as core/bench.py measures the TRT engine.
    u8: the uint8-NHWC engine (the reference's A/B, reports/uint8_ab/
    depth_anything_v2.json: 294.07 FPS on the 3080), 0.8 MB H2D."""
    from monocular_depth_estimation_trt_amd import common_runtime as cr
    from monocular_depth_estimation_trt_amd import weights
    from monocular_depth_estimation_trt_amd.engine import Engine
    eng = Engine.from_bytes(blob, dev)
    ctx = eng.create_execution_context()
    inputs, outputs, bindings, stream = cr.allocate_buffers(eng, None, profile_idx=0)
    inputs[0].host = (weights.synthetic_images_u8 if u8 else weights.synthetic_images)(1, size, size, first_seed=0)
    timer = cr.StageTimer()
    fn = lambda: cr.do_inference(ctx, eng, bindings, inputs, outputs, stream, timer=timer)  # noqa: E731
    for _ in range(warmup):
        fn()
    samples, stages = [], {k: [] for k in cr.StageTimer.STAGES}
    for _ in range(iters):
        t0 = time.perf_counter()
        fn()
        samples.append((time.perf_counter() - t0) * 1e3)
        for k, v in timer.last.items():
            stages[k].append(v)
    out = outputs[0].host.copy()
    timer.free()
    cr.free_buffers(inputs, outputs, stream)
    ctx.destroy()
    eng.destroy()
    mean = statistics.fmean(samples)
    s = sorted(samples)
    pct = lambda q: s[min(len(s) - 1, max(0, int(np.ceil(q / 100 * len(s))) - 1))]  # noqa: E731
    ref = REF_B1_U8_FPS if u8 else REF_B1_FPS
    res = {"mean_ms": round(mean, 4), "p50_ms": round(pct(50), 4), "p99_ms": round(pct(99), 4),
           "fps": round(1000.0 / mean, 2), "vs_ref_fps": round(1000.0 / mean / ref, 3)}
    for k, v in stages.items():
        res[k] = round(statistics.fmean(v), 4)
    res["out_mean"] = float(out.mean())
    return {prefix + k: v for k, v in res.items()}


def cpu_baseline(cfg, size, seconds):
    import torch
    from oracle import dav2_ref
    from monocular_depth_estimation_trt_amd import weights
    torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)))
    w = dav2_ref.to_torch(weights.synthetic_state_dict(cfg, 1234))
    x = torch.from_numpy(weights.synthetic_images(1, size, size, first_seed=0))
    dav2_ref.forward(w, cfg, x)   # warmup
    n, t0 = 0, time.perf_counter()
    while True:
        dav2_ref.forward(w, cfg, x)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds or n >= 200:
            break
    return {"value": round(n / el, 3), "unit": "images/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"{n} x DA-V2 {cfg['encoder']} {size}x{size} batch-1 fp32 forwards of oracle/dav2_ref.py "
                      f"(torch CPU) after 1 warmup, {el:.1f} s"}


def main():
    a = parse()
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one process per GPU)")
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(local)

    from monocular_depth_estimation_trt_amd import pack, weights
    from monocular_depth_estimation_trt_amd.engine import Engine
    from monocular_depth_estimation_trt_amd.flops import total_flops

    B, S = a.batch, a.size
    cfg = weights.model_config(a.encoder, "metric")
    sd = weights.synthetic_state_dict(cfg, 1234)
    blob = pack.pack_bytes(sd, cfg, S, S)
    eng = Engine.from_bytes(blob, local, profile=((1, 3, S, S), (B, 3, S, S), (B, 3, S, S)))
    ctx = eng.create_execution_context()
    x = torch.from_numpy(weights.synthetic_images(B, S, S, first_seed=rank * B)).cuda()
    y = torch.empty(B, S, S, device="cuda")
    ctx.set_input_shape("input", (B, 3, S, S))
    ctx.set_tensor_address("input", x.data_ptr())
    ctx.set_tensor_address("output", y.data_ptr())
    st = torch.cuda.Stream()
    sh = st.cuda_stream

    from monocular_depth_estimation_trt_amd import replicas
    for _ in range(a.warmup):
        ctx.execute_async_v3(sh)
    torch.cuda.synchronize()
    el = replicas.timed_region(lambda: ctx.execute_async_v3(sh), a.steps, torch.cuda.synchronize,
                               dist.barrier if dist is not None else None)
    el = replicas.max_over_ranks(el)
    out_ok = bool(torch.isfinite(y).all().item())
    value = world * B * a.steps / el
    ms_step = el / a.steps * 1e3

    if rank != 0:
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return

    layer_ms = profile_layers(ctx, sh, a.profile_iters)
    roof, breakdown = roofline(cfg, B, S, layer_ms)
    if a.layers_json:
        with open(a.layers_json, "w") as f:
            json.dump({"batch": B, "layer_ms": layer_ms, "classes": breakdown, "roofline": roof}, f, indent=1)
    gflop = total_flops(cfg, S, S) / 1e9
    model_frac = value / world * gflop * 1e9 / (MFMA_PEAK_TFLOPS * 1e12)
    res_b1 = {} if a.no_b1 else b1_reference_method(blob, local, S, a.b1_warmup, a.b1_iters)
    if not a.no_b1:
        blob_u8 = pack.pack_bytes(sd, cfg, S, S, input_format="uint8_nhwc")
        res_b1.update(b1_reference_method(blob_u8, local, S, a.b1_warmup, a.b1_iters, u8=True, prefix="b1_u8_"))
    ctx.destroy()
    eng.destroy()
    cpu = None
    if world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(cfg, S, a.cpu_seconds)
    for c, v in list(breakdown.items())[:8]:
        log(f"{c:24s} {v['ms']:9.4f} ms  x{v['launches']:3d}  {v['tflops']} TF/s")
    line = {
        "metric": f"depth FPS (images/s) at {S}x{S} fp16, DA-V2 {ENC_LABEL.get(a.encoder, a.encoder)}, MI355X",
        "value": round(value, 2), "unit": "images/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(ms_step, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": round(value / REF_B1_FPS, 3), "dtype": "fp16", "data": "synthetic",
        "config": {"workload": f"Depth Anything V2 {a.encoder} {S}x{S} metric head, forward, batch {B} per GPU, "
                               f"inputs resident in HBM, hipGraph replay",
                   "encoder": a.encoder, "img": [S, S], "batch_per_gpu": B, "global_batch": B * world,
                   "parallelism": f"replica x{world} (batch shards, no collectives)",
                   "weights": "synthetic seeded (seed 1234), fan-in scaled"},
        "model_gflop_per_image": round(gflop, 2),
        "model_mfma_frac": round(model_frac, 4),
        "roofline": roof,
        "cpu_baseline": cpu,
        "output_finite": out_ok,
    }
    line.update(res_b1)
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
