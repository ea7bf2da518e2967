"""Two concurrent half-batch forwards vs one full-batch forward (timing probe).

    python tools/two_stream.py [--batch 48] [--steps 40] [--splits 1,2,3]

One engine, one execution context per split, each with its own activation
arena and captured forward graph, launched on its own stream inside the timed
step (fork from / join to the timing stream): the kernels of one split's tail
rounds can run beside the other split's.  Prints img/s per split count.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=48)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--splits", default="1,2,3")
    ap.add_argument("--lib", default="")
    a = ap.parse_args()
    import torch
    from monocular_depth_estimation_trt_amd import _lib, pack, weights
    if a.lib:
        _lib.use_library(a.lib)
    from monocular_depth_estimation_trt_amd.engine import Engine
    B, S = a.batch, 518
    cfg = weights.model_config("vits", "metric")
    sd = weights.synthetic_state_dict(cfg, 1234)
    x = torch.from_numpy(weights.synthetic_images(B, S, S, first_seed=100)).to("cuda:0")
    y = torch.empty(B, S, S, device="cuda:0")
    blob = pack.pack_bytes(sd, cfg, S, S)
    eng = Engine.from_bytes(blob, 0, profile=((1, 3, S, S), (B, 3, S, S), (B, 3, S, S)))
    ref = None
    for ns in [int(v) for v in a.splits.split(",")]:
        if B % ns:
            continue
        b = B // ns
        ctxs, streams = [], []
        for i in range(ns):
            c = eng.create_execution_context()
            c.set_input_shape("input", (b, 3, S, S))
            c.set_tensor_address("input", x[i * b:(i + 1) * b].data_ptr())
            c.set_tensor_address("output", y[i * b:(i + 1) * b].data_ptr())
            ctxs.append(c)
            streams.append(torch.cuda.Stream())
        main_s = torch.cuda.Stream()

        def step():
            ev = torch.cuda.Event()
            ev.record(main_s)
            for c, st in zip(ctxs, streams):
                st.wait_event(ev)
                c.execute_async_v3(st.cuda_stream)
            for st in streams:
                e2 = torch.cuda.Event()
                e2.record(st)
                main_s.wait_event(e2)

        for _ in range(5):
            step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(main_s)
        for _ in range(a.steps):
            step()
        e1.record(main_s)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.steps
        out = y.clone()
        if ref is None:
            ref = out
        same = bool(torch.equal(out, ref))
        print(f"splits {ns} x B={b}: {ms:.3f} ms/step  {B * 1000 / ms:.1f} img/s  output identical to splits 1: {same}",
              flush=True)
        for c in ctxs:
            c.destroy()
    eng.destroy()


if __name__ == "__main__":
    main()
