#!/usr/bin/env python
"""Depth Anything V2 throughput on MI355X through the HIP engine.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--encoder vits]
    python bench.py --gpus 8 --encoder vitl --global-batch 8   (BASELINE config 3)
    python bench.py --model depth_pro [--batch 4]     (SURVEY.md 8f row 3, 1536^2)
    python bench.py --model vggt [--batch 8] [--frames 1]   (SURVEY.md 8f row 4, 518^2)

One *step* = one forward of the packed DA-V2 engine over one batch of B
synthetic 518x518 images already resident in HBM (input fp32 NCHW, output
fp32 depth), enqueued on one HIP stream, replayed from the engine's
captured hipGraph.  N > 1: one process per GPU, each rank an independent
replica on its own batch shard -- no collective on the data path (SURVEY.md
8e); a gloo barrier brackets the timed region and the max time over ranks is
used.  Launched either by torch.distributed.run (RANK / WORLD_SIZE set) or
directly: `python bench.py --gpus N` spawns the N rank processes itself
(replicas.spawn_local) before anything touches the GPU.  `value` = images
processed by all ranks / that time.  Default: weak scaling (`--batch` images
per GPU); `--global-batch G` shards G images over the ranks instead (strong
scaling, replicas.shard: config 3 = ViT-L, G = 8).  VGGT counts frames: a
batch item of S frames is S images.

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
    fp16 MFMA peak (2.5 PF/s, MI355X_MICROARCH.md); `traffic` = that class's
    HBM bytes per launch from the committed per-layer PMC profile of this
    workload (tools/profile_round.sh -> profiles/traffic_*.json).
  * vs_baseline: null -- BASELINE.md publishes no number for this metric
    (HBM-resident throughput); the like-for-like ratio is b1_vs_ref_fps
    (batch 1, PCIe-inclusive, the reference's method) and
    throughput_vs_ref_b1 = value / 232.11 says how far batching goes.
  * cpu_baseline (rank 0, after the timed region at every N): the oracle's
    fp32 CPU forward (a PyTorch restatement of upstream DA-V2) on this host's
    cores, bounded sample, in the same run (north_star).
"""

from __future__ import annotations

import argparse
import gc
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MFMA_PEAK_TFLOPS = 2500.0   # dense fp16/bf16 MFMA, MI355X spec (MI355X_MICROARCH.md chip table)
# measured on this chip (tools/mfma_peak.hip: back-to-back MFMAs on random f16
# operands, every CU, clock settled): the sustained rate per MFMA shape --
# attention runs 32x32x16, the GEMMs / convs 16x16x32
MFMA_PEAK_FILE = os.path.join(ROOT, "profiles", "r03_mfma_peak.json")


def measured_peak(kernel_class: str, attn16: bool = False):
    """(TFLOP/s, MFMA shape) the chip sustains for the instruction the class's
    kernel issues, from the committed microbenchmark; (None, None) without it.
    attn16: the attention launch is attn16_fwd_kernel (16x16x32, round 6)."""
    try:
        with open(MFMA_PEAK_FILE) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None
    is_attn = kernel_class.split(".")[-1] in ("attn", "attention", "gattn", "fattn")
    shape = "32x32x16" if is_attn and not attn16 else "16x16x32"
    return d.get(f"mfma_f16_{shape}_tflops"), shape


def attn16_active(cfg, B, size) -> bool:
    """Whether the DA-V2 attention launches run attn16_fwd_kernel: switch
    "attn16" on and the launcher's 8-wave unsplit shape (attention.hip
    launch_attention: B * heads * ceil(T / 256) >= 512)."""
    if cfg.get("family") in ("depth_pro", "vggt"):
        return False
    from monocular_depth_estimation_trt_amd import _lib
    if _lib.get_tuning("attn16") != 1:
        return False
    h, w = size if isinstance(size, tuple) else (size, size)
    T = (h // cfg["patch"]) * (w // cfg["patch"]) + 1
    return B * int(cfg["num_heads"]) * -(-T // 256) >= 512
ENC_LABEL = {"vits": "ViT-S", "vitb": "ViT-B", "vitl": "ViT-L"}
REF_B1_FPS = 232.11         # RTX 3080 TRT fp16, BASELINE.md
REF_B1_FP32_FPS = 88.29     # RTX 3080 TRT fp32 (the reference's default build), reports/tune/fp32_depth_anything_v2.json
REF_B1_U8_FPS = 294.07      # same, uint8-NHWC input engine (reports/uint8_ab/depth_anything_v2.json)
REF_DP_B1_FPS = 4.13        # Depth Pro 1536^2 TRT fp16, RTX 3080 (242.12 ms, BASELINE.md / SURVEY.md 6)
REF_VGGT_B1_FPS = 19.02     # VGGT 518^2 S=1 TRT fp16, RTX 3080 (52.58 ms, BASELINE.md / SURVEY.md 6)


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def parse_size(v: str):
    """'518' -> (518, 518); '392x518' -> (392, 518) (the reference's HxW,
    tools/size_sweep.py / reports/tune/size_depth_anything_v2.json)."""
    h, _, w = str(v).lower().partition("x")
    return int(h), int(w or h)


# the reference's published DA-V2 ViT-S size sweep (RTX 3080, TRT fp16, batch 1,
# mean ms per image incl. copies): reports/tune/size_depth_anything_v2.json
REF_SIZE_MS = {(392, 518): 3.7605, (518, 518): 4.2852, (672, 896): 10.4632}


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--model", default="depth_anything_v2", choices=["depth_anything_v2", "depth_pro", "vggt"])
    p.add_argument("--batch", type=int, default=0,
                   help="batch items per GPU per step (default 48; depth_pro 4; vggt 8)")
    p.add_argument("--global-batch", type=int, default=0,
                   help="shard this many items over the ranks instead (strong scaling; config 3: 8)")
    p.add_argument("--frames", type=int, default=1, help="vggt: frames per batch item (the packed S)")
    p.add_argument("--encoder", default="vits", choices=["vits", "vitb", "vitl"])
    p.add_argument("--precision", default="fp16", choices=["fp16", "fp32"],
                   help="DA-V2 engine precision (get_engine's; fp32 = the exact-fp32 encoder)")
    p.add_argument("--size", type=parse_size, default=(518, 518),
                   help="DA-V2 input H or HxW (the reference's size sweep: 392x518, 518x518, 672x896)")
    p.add_argument("--b1-iters", type=int, default=100)
    p.add_argument("--b1-warmup", type=int, default=20)
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-b1", action="store_true")
    p.add_argument("--no-pcie", action="store_true", help="skip the PCIe-inclusive streamed-batch leg (value_pcie)")
    p.add_argument("--oversubscribe", action="store_true",
                   help="allow more ranks than visible GPUs (a launcher rehearsal: ranks share devices round-robin; "
                        "the line is marked devices_shared and its scaling field is not a scaling measurement)")
    p.add_argument("--profile-iters", type=int, default=3)
    p.add_argument("--layers-json", default="", help="write the per-layer profile here (rank 0)")
    return p.parse_args(argv)


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


def traffic_path(model, encoder, B, size, frames=1):
    h, w = size if isinstance(size, tuple) else (size, size)
    st = f"{h}" if h == w else f"{h}x{w}"
    tag = f"{model}_{encoder}_b{B}_{st}" + (f"_s{frames}" if model == "vggt" else "")
    return os.path.join(ROOT, "profiles", f"traffic_{tag}.json")


def pmc_traffic(layer_names, path):
    """HBM bytes per launch of a layer class from the committed per-layer
    PMC profile (tools/pmc_traffic.py: FETCH_SIZE x2 + WRITE_SIZE per
    dispatch, separate passes, dispatches matched to the engine's layer order),
    averaged over the class's layers; None when no profile covers them."""
    if not os.path.exists(path):
        return None
    with open(path) as f:
        layers = json.load(f).get("layers", {})
    got = [layers[n]["hbm_bytes_per_launch"] for n in layer_names if n in layers]
    if not got or len(got) != len(layer_names):
        return None
    return int(sum(got) / len(got))


def roofline(cfg, B, size, layer_ms, frames=1, traffic_file=""):
    h, w = size if isinstance(size, tuple) else (size, size)
    fam = cfg.get("family")
    if fam == "depth_pro":
        from monocular_depth_estimation_trt_amd import flops_depth_pro as flops
        lf = flops.layer_flops(cfg, B)
    elif fam == "vggt":
        from monocular_depth_estimation_trt_amd import flops_vggt as flops
        lf = flops.layer_flops(cfg, B, frames)
    else:
        from monocular_depth_estimation_trt_amd import flops
        lf = flops.layer_flops(cfg, h, w, B)
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
    traffic = pmc_traffic([n for n in layer_ms if flops.layer_class(n) == dom], traffic_file)
    roof = {"bound": "mfma", "kernel": dom, "achieved": round(achieved, 2), "peak": MFMA_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": round(achieved / MFMA_PEAK_TFLOPS, 4), "traffic": traffic,
            "flop_per_launch": per_launch_fl, "avg_launch_ms": round(avg_ms, 5),
            "launches_per_step": cls_n[dom]}
    mp, shape = measured_peak(dom, attn16_active(cfg, B, size))
    if mp:
        roof.update({"peak_source": "spec (MI355X_MICROARCH.md)", "peak_measured": mp,
                     "peak_measured_mfma": f"v_mfma_f32_{shape}_f16",
                     "peak_measured_source": os.path.relpath(MFMA_PEAK_FILE, ROOT),
                     "frac_of_measured": round(achieved / mp, 4)})
    if traffic is not None:
        roof["traffic_unit"] = "bytes/launch"
        roof["traffic_source"] = os.path.relpath(traffic_file, ROOT)
    return roof, breakdown


def b1_reference_method(blob, dev, images, warmup, iters, ref_fps, prefix="b1_"):
    """Batch-1 wall clock exactly as core/bench.py measures the TRT engine:
    pinned H2D of `images` (one image), enqueue, D2H of every output, sync;
    20 warmup / 100 iterations, StageTimer split.  For the DA-V2 uint8-NHWC
    engine (the reference's A/B, reports/uint8_ab/depth_anything_v2.json:
    294.07 FPS on the 3080) the H2D is 0.8 MB."""
    from monocular_depth_estimation_trt_amd import common_runtime as cr
    from monocular_depth_estimation_trt_amd.engine import Engine
    eng = Engine.from_bytes(blob, dev)
    ctx = eng.create_execution_context()
    inputs, outputs, bindings, stream = cr.allocate_buffers(eng, None, profile_idx=0)
    inputs[0].host = images
    timer = cr.StageTimer()
    fn = lambda: cr.do_inference(ctx, eng, bindings, inputs, outputs, stream, timer=timer)  # noqa: E731
    for _ in range(warmup):
        fn()
    # host-side pauses inside the timed loop: Python's cyclic GC (a gen-2 pass
    # walks every object torch created, milliseconds) -- recorded per sample
    gc_log = []
    t_gc = [0.0]

    def _gc_cb(phase, info):
        if phase == "start":
            t_gc[0] = time.perf_counter()
        else:
            gc_log.append((len(samples), info.get("generation"), (time.perf_counter() - t_gc[0]) * 1e3))

    samples, stages = [], {k: [] for k in cr.StageTimer.STAGES}
    gc.callbacks.append(_gc_cb)
    try:
        for _ in range(iters):
            t0 = time.perf_counter()
            fn()
            samples.append((time.perf_counter() - t0) * 1e3)
            for k, v in timer.last.items():
                stages[k].append(v)
    finally:
        gc.callbacks.remove(_gc_cb)
    out = outputs[0].host.copy()
    timer.free()
    cr.free_buffers(inputs, outputs, stream)
    ctx.destroy()
    eng.destroy()
    mean = statistics.fmean(samples)
    s = sorted(samples)
    pct = lambda q: s[min(len(s) - 1, max(0, int(np.ceil(q / 100 * len(s))) - 1))]  # noqa: E731
    imax = int(np.argmax(samples))
    res = {"mean_ms": round(mean, 4), "p50_ms": round(pct(50), 4), "p99_ms": round(pct(99), 4),
           "max_ms": round(samples[imax], 4), "max_iter": imax,
           "fps": round(1000.0 / mean, 2), "vs_ref_fps": round(1000.0 / mean / ref_fps, 3),
           "max_iter_stages": {k: round(v[imax], 4) for k, v in stages.items() if len(v) > imax},
           "gc_in_loop": [[i, g, round(ms, 3)] for i, g, ms in gc_log]}
    for k, v in stages.items():
        res[k] = round(statistics.fmean(v), 4)
    res["out_mean"] = float(out.mean())
    return {prefix + k: v for k, v in res.items()}


def pcie_streamed_region(wl, ctx, stream, steps, warmup, sync, barrier):
    """The served-batch-stream rate with the copies in (the reference's FPS
    is wall clock over H2D + compute + D2H, core/bench.py:182-210): each step
    copies a batch of B images from pinned host memory, runs the forward and
    copies the depth maps back.  Two streams (the forward's own and one copy
    stream -- GPU_MAX_HW_QUEUES is 4, and streams beyond the hardware queues
    share one and serialise), double-buffered device I/O: while forward(i)
    runs, the copy stream moves batch i+1 in and batch i-1 out.
    Returns (seconds for `steps` steps, bytes in per step, bytes out per step)."""
    import torch
    host_in = torch.from_numpy(wl.images(wl.B, 0)).pin_memory()
    host_out = [{k: torch.empty(t.shape, dtype=t.dtype, pin_memory=True) for k, t in wl.y.items()} for _ in range(2)]
    dev_in = [wl.x, torch.empty_like(wl.x)]
    dev_out = [wl.y, {k: torch.empty_like(t) for k, t in wl.y.items()}]
    s_fwd = stream
    s_cp = torch.cuda.Stream()
    in_ready = [torch.cuda.Event() for _ in range(2)]
    fwd_done = [torch.cuda.Event() for _ in range(2)]
    out_free = [torch.cuda.Event() for _ in range(2)]

    def h2d(i):
        with torch.cuda.stream(s_cp):
            dev_in[i & 1].copy_(host_in, non_blocking=True)
            in_ready[i & 1].record(s_cp)

    def d2h(i):
        with torch.cuda.stream(s_cp):
            for k, t in dev_out[i & 1].items():
                host_out[i & 1][k].copy_(t, non_blocking=True)
            out_free[i & 1].record(s_cp)

    def run(n):
        h2d(0)
        for i in range(n):
            j = i & 1
            s_fwd.wait_event(in_ready[j])
            s_fwd.wait_event(out_free[j])              # D2H(i-2) has read dev_out[j]
            ctx.set_tensor_address(wl.input_name, dev_in[j].data_ptr())
            for k, t in dev_out[j].items():
                ctx.set_tensor_address(k, t.data_ptr())
            ctx.execute_async_v3(s_fwd.cuda_stream)
            fwd_done[j].record(s_fwd)
            if i >= 1:
                s_cp.wait_event(fwd_done[j ^ 1])       # forward(i-1): dev_in / dev_out [j^1] are free / full
            if i + 1 < n:
                h2d(i + 1)
            if i >= 1:
                d2h(i - 1)
        s_cp.wait_event(fwd_done[(n - 1) & 1])
        d2h(n - 1)

    run(max(2, warmup))                            # both slots' graphs captured
    sync()
    if barrier is not None:
        barrier()
    t0 = time.perf_counter()
    run(steps)
    sync()
    el = time.perf_counter() - t0
    # the context goes back to the resident buffers of the main timed region
    ctx.set_tensor_address(wl.input_name, wl.x.data_ptr())
    for k, t in wl.y.items():
        ctx.set_tensor_address(k, t.data_ptr())
    bytes_in = host_in.numel() * host_in.element_size()
    bytes_out = sum(t.numel() * t.element_size() for t in wl.y.values())
    return el, bytes_in, bytes_out


def _timed_cpu(fn, seconds, warmup=True, max_n=200):
    if warmup:
        fn()
    n, t0 = 0, time.perf_counter()
    while True:
        fn()
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds or n >= max_n:
            return n, el


def cpu_baseline(cfg, size, seconds):
    import torch
    h, w = size if isinstance(size, tuple) else (size, size)
    size = h
    torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1)))
    if cfg.get("family") == "depth_pro":
        # one full fp32 forward is ~19 TFLOP: the sample is ONE forward, no warmup
        from oracle import depth_pro_ref
        from monocular_depth_estimation_trt_amd import weights_depth_pro as WD
        w = depth_pro_ref.to_torch(WD.synthetic_state_dict(cfg, 4321))
        x = torch.from_numpy(WD.synthetic_images(1, size, first_seed=0))
        n, el = _timed_cpu(lambda: depth_pro_ref.forward(w, cfg, x), seconds, warmup=False, max_n=1)
        what = f"{n} x Depth Pro {size}x{size} batch-1 fp32 forward of oracle/depth_pro_ref.py (torch CPU), no warmup"
    elif cfg.get("family") == "vggt":
        # ~3.3 TFLOP per frame: the sample is ONE single-frame forward, no warmup
        from oracle import vggt_ref
        from monocular_depth_estimation_trt_amd import weights_vggt as WV
        w = vggt_ref.to_torch(WV.synthetic_state_dict(cfg, 2468))
        x = torch.from_numpy(WV.synthetic_images(1, 1, size, first_seed=0))
        n, el = _timed_cpu(lambda: vggt_ref.forward(w, cfg, x), seconds, warmup=False, max_n=1)
        what = f"{n} x VGGT-1B depth path {size}x{size} S=1 fp32 forward of oracle/vggt_ref.py (torch CPU), no warmup"
    else:
        from oracle import dav2_ref
        from monocular_depth_estimation_trt_amd import weights
        wt = dav2_ref.to_torch(weights.synthetic_state_dict(cfg, 1234))
        x = torch.from_numpy(weights.synthetic_images(1, h, w, first_seed=0))
        n, el = _timed_cpu(lambda: dav2_ref.forward(wt, cfg, x), seconds)
        what = (f"{n} x DA-V2 {cfg['encoder']} {h}x{w} batch-1 fp32 forwards of oracle/dav2_ref.py "
                f"(torch CPU) after 1 warmup")
    return {"value": round(n / el, 3), "unit": "images/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"{what}, {el:.1f} s"}


class Workload:
    """The packed engine, its io tensors and the constants of one bench model."""

    def __init__(self, a, B, first):
        """B items on this rank (0: an idle rank of a strong-scaling run),
        synthetic item seeds from `first` on."""
        import torch
        self.frames = 1
        self.ref_size_ms = None
        self.precision = "fp16"
        self.input_name = "input"
        if a.model == "depth_pro":
            from monocular_depth_estimation_trt_amd import pack_depth_pro as PD
            from monocular_depth_estimation_trt_amd import weights_depth_pro as WD
            from monocular_depth_estimation_trt_amd.flops_depth_pro import total_flops
            self.cfg = WD.depth_pro_config("dinov2l16_384")
            self.S = S = self.cfg["img"]
            self.H = self.W = S
            self.B = B
            self.sd = WD.synthetic_state_dict(self.cfg, 4321)
            self.blob = PD.pack_bytes(self.sd, self.cfg)
            self.images = lambda n, seed: WD.synthetic_images(n, S, first_seed=seed)  # noqa: E731
            self.outs = {"canonical_inverse_depth": (B, 1, S, S), "fov_deg": (B,)}
            self.gflop = total_flops(self.cfg) / 1e9
            self.ref_fps = REF_DP_B1_FPS
            self.label = "Depth Pro"
            self.workload = (f"Depth Pro (3 x DINOv2-L/16 at 384^2, 35-patch pyramid, FOV head) {S}x{S}, forward, "
                             f"{a.per_gpu_desc}, inputs resident in HBM, hipGraph replay")
            self.weights = "synthetic seeded (seed 4321), fan-in scaled"
            self.encoder = "dinov2l16_384"
        elif a.model == "vggt":
            from monocular_depth_estimation_trt_amd import pack_vggt as PV
            from monocular_depth_estimation_trt_amd import weights_vggt as WV
            from monocular_depth_estimation_trt_amd.flops_vggt import total_flops
            self.cfg = WV.vggt_config("vggt_1b")
            self.S = S = self.cfg["img"]
            self.H = self.W = S
            self.B = B
            self.frames = Fr = a.frames
            self.input_name = "images"
            self.sd = WV.synthetic_state_dict(self.cfg, 2468)
            self.blob = PV.pack_bytes(self.sd, self.cfg, Fr)
            self.images = lambda n, seed: WV.synthetic_images(n, Fr, S, first_seed=seed * Fr)  # noqa: E731
            self.outs = {"depth": (B, Fr, S, S, 1)}
            self.gflop = total_flops(self.cfg, 1, Fr) / Fr / 1e9          # per frame
            self.ref_fps = REF_VGGT_B1_FPS
            self.label = "VGGT-1B depth"
            self.workload = (f"VGGT-1B depth path (DINOv2-L/14-reg + 24 frame/global block pairs + DPT) {S}x{S}, "
                             f"S={Fr} frames, forward, {a.per_gpu_desc}, inputs resident in HBM, hipGraph replay")
            self.weights = "synthetic seeded (seed 2468), fan-in scaled"
            self.encoder = "vggt_1b"
        else:
            from monocular_depth_estimation_trt_amd import pack, weights
            from monocular_depth_estimation_trt_amd.flops import total_flops
            self.H, self.W = H, W = a.size
            self.S = S = (H, W) if H != W else H
            self.B = B
            self.cfg = weights.model_config(a.encoder, "metric")
            self.sd = weights.synthetic_state_dict(self.cfg, 1234)
            self.precision = a.precision
            self.blob = pack.pack_bytes(self.sd, self.cfg, H, W, precision=a.precision)
            self.images = lambda n, seed: weights.synthetic_images(n, H, W, first_seed=seed)  # noqa: E731
            self.outs = {"output": (B, H, W)}
            self.gflop = total_flops(self.cfg, H, W) / 1e9
            self.ref_fps = REF_B1_FPS if a.precision == "fp16" else REF_B1_FP32_FPS
            if (H, W) != (518, 518) and a.encoder == "vits" and a.precision == "fp16" and (H, W) in REF_SIZE_MS:
                # the reference's size sweep is the published number at this size
                self.ref_fps = 1000.0 / REF_SIZE_MS[(H, W)]
                self.ref_size_ms = REF_SIZE_MS[(H, W)]
            self.label = f"DA-V2 {ENC_LABEL.get(a.encoder, a.encoder)}"
            self.workload = (f"Depth Anything V2 {a.encoder} {H}x{W} metric head, forward, {a.per_gpu_desc}, "
                             f"inputs resident in HBM, hipGraph replay")
            self.weights = "synthetic seeded (seed 1234), fan-in scaled"
            self.encoder = a.encoder
        if B > 0:
            self.x = torch.from_numpy(self.images(B, first)).cuda()
            self.y = {k: torch.empty(v, device="cuda") for k, v in self.outs.items()}

    def b1_legs(self, a, dev):
        res = b1_reference_method(self.blob, dev, self.images(1, 0), a.b1_warmup, a.b1_iters, self.ref_fps)
        if a.model == "depth_anything_v2" and self.precision == "fp16" and (self.H, self.W) == (518, 518):
            # (the reference's uint8 A/B is an fp16 engine: reports/uint8_ab/depth_anything_v2.json)
            from monocular_depth_estimation_trt_amd import pack, weights
            blob_u8 = pack.pack_bytes(self.sd, self.cfg, self.H, self.W, input_format="uint8_nhwc",
                                      precision=self.precision)
            res.update(b1_reference_method(blob_u8, dev, weights.synthetic_images_u8(1, self.H, self.W, first_seed=0),
                                           a.b1_warmup, a.b1_iters, REF_B1_U8_FPS, prefix="b1_u8_"))
        return res


DEFAULT_BATCH = {"depth_pro": 4, "vggt": 8,
                 # B=48: with three workgroups per CU on the short-K GEMMs the
                 # wave-quantisation tails of every kernel are what a larger
                 # batch amortises -- same-box sweep with this round's kernels
                 # (profiles/r02_v23_batch_sweep_24_48.txt, two passes each):
                 # B=28 4843/4833, B=40 4886/4885, B=48 5015/4998 img/s; past 48
                 # nothing more (r02_v23_batch_sweep_48_96.txt).  Round 1's B=28
                 # (whole rounds of attention workgroups) no longer wins.
                 "depth_anything_v2": 48}


def rank_work(a, world, rank):
    """(items on this rank, first item seed, items per step over all ranks,
    scaling, description) -- weak: --batch per GPU; strong: --global-batch
    sharded contiguously (replicas.shard), an idle rank possible."""
    from monocular_depth_estimation_trt_amd import replicas
    if a.global_batch > 0:
        first, B = replicas.shard(a.global_batch, world, rank)
        return B, first, a.global_batch, "strong", f"global batch {a.global_batch} sharded over {world} GPU(s)"
    B = a.batch or DEFAULT_BATCH[a.model]
    return B, rank * B, world * B, "weak", f"batch {B} per GPU"


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        # self-launch: one child process per GPU, started before this process
        # touches the GPU (it never does); rank 0's JSON line is the output
        from monocular_depth_estimation_trt_amd import replicas
        raise SystemExit(replicas.spawn_local(a.gpus, os.path.abspath(__file__), sys.argv[1:]))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}: launch one process per GPU")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    # one rank per GPU; more ranks than visible GPUs only as an explicit
    # launcher rehearsal (--oversubscribe: ranks share devices round-robin) --
    # device_count() does not initialise HIP
    ndev = max(1, torch.cuda.device_count())
    shared = world > ndev
    if shared and not a.oversubscribe:
        raise SystemExit(f"{world} ranks but {ndev} visible GPU(s): one rank per GPU "
                         f"(--oversubscribe for a launcher rehearsal that shares devices)")
    local = local % ndev
    torch.cuda.set_device(local)

    from monocular_depth_estimation_trt_amd import replicas
    from monocular_depth_estimation_trt_amd.engine import Engine

    B, first, total_items, scaling, a.per_gpu_desc = rank_work(a, world, rank)
    wl = Workload(a, B, first)
    S = wl.S
    ctx = eng = None
    if B > 0:
        shape = tuple(wl.x.shape)
        eng = Engine.from_bytes(wl.blob, local, profile=((1,) + shape[1:], shape, shape))
        ctx = eng.create_execution_context()
        ctx.set_input_shape(wl.input_name, shape)
        ctx.set_tensor_address(wl.input_name, wl.x.data_ptr())
        for k, t in wl.y.items():
            ctx.set_tensor_address(k, t.data_ptr())
    st = torch.cuda.Stream()
    sh = st.cuda_stream
    step = (lambda: ctx.execute_async_v3(sh)) if ctx is not None else (lambda: None)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    el = replicas.timed_region(step, a.steps, torch.cuda.synchronize,
                               dist.barrier if dist is not None else None)
    per_rank = replicas.gather_to_rank0(round(el, 6))
    el = replicas.max_over_ranks(el)
    pcie = None
    if not a.no_pcie:
        if ctx is not None:
            el_p, b_in, b_out = pcie_streamed_region(wl, ctx, st, a.steps, a.warmup, torch.cuda.synchronize,
                                                     dist.barrier if dist is not None else None)
        else:  # an idle rank of a strong-scaling run still joins the barrier
            if dist is not None:
                dist.barrier()
            el_p, b_in, b_out = 0.0, 0, 0
        el_p = replicas.max_over_ranks(el_p)
        pcie = {"value_pcie": round(total_items * wl.frames * a.steps / el_p, 2), "ms_per_step_pcie": round(el_p / a.steps * 1e3, 4),
                "pcie_h2d_mb_per_step": round(b_in / 1e6, 1), "pcie_d2h_mb_per_step": round(b_out / 1e6, 1),
                "pcie_method": "pinned host batch -> H2D -> forward (graph) -> D2H into pinned host; forward stream + "
                               "one copy stream, double-buffered device I/O, H2D(i+1) and D2H(i-1) under forward(i); "
                               "wall clock over K steps bracketed by barrier + device sync, max over ranks"}
    out_ok = all(bool(torch.isfinite(t).all().item()) for t in wl.y.values()) if B > 0 else True
    value = total_items * wl.frames * a.steps / el
    ms_step = el / a.steps * 1e3

    if rank != 0:
        if ctx is not None:
            ctx.destroy()
            eng.destroy()
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return

    layer_ms = profile_layers(ctx, sh, a.profile_iters)
    tfile = traffic_path(a.model, wl.encoder, B, S, wl.frames)
    roof, breakdown = roofline(wl.cfg, B, S, layer_ms, wl.frames, tfile)
    if roof["traffic"] is None:
        log(f"no committed PMC profile covers '{roof['kernel']}' at this workload "
            f"({os.path.relpath(tfile, ROOT)}): roofline.traffic is null -- "
            f"bash tools/profile_round.sh <out> {' '.join(sys.argv[1:])}")
    if a.layers_json:
        with open(a.layers_json, "w") as f:
            json.dump({"batch": B, "frames": wl.frames, "layer_ms": layer_ms, "classes": breakdown, "roofline": roof},
                      f, indent=1)
    # MFMA fraction of the whole job: every GPU's share of the work at the job's rate
    model_frac = value / world * wl.gflop * 1e9 / (MFMA_PEAK_TFLOPS * 1e12)
    ctx.destroy()
    eng.destroy()
    res_b1 = {} if a.no_b1 else wl.b1_legs(a, local)
    if "b1_compute_ms" in res_b1:
        # batch-1 forward (the engine compute of one image, hipEvent-timed inside do_inference)
        res_b1["b1_model_mfma_frac"] = round(wl.gflop * 1e9 / (res_b1["b1_compute_ms"] * 1e-3) /
                                             (MFMA_PEAK_TFLOPS * 1e12), 4)
    cpu = None
    if not a.no_cpu_baseline:
        # N > 1: the other ranks are done and wait at the closing barrier
        cpu = cpu_baseline(wl.cfg, S, a.cpu_seconds)
    for c, v in list(breakdown.items())[:10]:
        log(f"{c:24s} {v['ms']:9.4f} ms  x{v['launches']:3d}  {v['tflops']} TF/s")
    config = {"workload": wl.workload, "encoder": wl.encoder, "img": [wl.H, wl.W], "batch_per_gpu": B,
              "global_batch": total_items, "parallelism": f"replica x{world} (batch shards, no collectives)",
              "weights": wl.weights, "physical_gpus": min(world, ndev)}
    if shared:
        # a rehearsal of the launch path: the ranks shared devices, so neither
        # n_gpus nor the value says anything about multi-GPU scaling
        config["devices_shared"] = True
        scaling = "none (rehearsal: devices shared)"
    if a.model == "vggt":
        config["frames"] = wl.frames
        # oracle/vggt_ref.py: the aggregator (q/k norm, 2-D RoPE, frame/global
        # alternation) is restated from the un-vendored upstream with nothing in
        # the reference to pin it
        config["parity"] = "partially pinned: aggregator parity unpinned"
    line = {
        "metric": f"depth FPS (images/s) at {wl.H}x{wl.W} {wl.precision}, {wl.label}, MI355X",
        "value": round(value, 2), "unit": "images/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(ms_step, 4), "higher_is_better": True, "scaling": scaling,
        "vs_baseline": None, "throughput_vs_ref_b1": round(value / wl.ref_fps, 3),
        "dtype": wl.precision, "data": "synthetic",
        "config": config,
        "rank_seconds": per_rank,
        "model_gflop_per_image": round(wl.gflop, 2),
        "model_mfma_frac": round(model_frac, 4),
        "roofline": roof,
        "cpu_baseline": cpu,
        "output_finite": out_ok,
    }
    if pcie:
        line.update(pcie)
    line.update(res_b1)
    if wl.ref_size_ms:
        line["b1_ref_ms"] = wl.ref_size_ms
        line["b1_ref_source"] = ("reports/tune/size_depth_anything_v2.json (RTX 3080 TRT fp16, batch 1, "
                                 f"{wl.H}x{wl.W})")
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
