"""VGGT (depth only) on MI355X -- the counterpart of the reference driver
`models/vggt/onnx2trt.py:main` (:56-148), same sequence:

  images [1, S, 3, 518, 518] in [0, 1] -> get_engine -> create_execution_context
  -> allocate_buffers -> bench.measure(do_inference) (20 warmup / 100
  iterations) -> depth [S, 518, 518] -> crop to the content box
  (onnx2trt.py:131) -> bench.record

    python -m monocular_depth_estimation_trt_amd.models.vggt.run \
        [--source synthetic:vggt:vggt_1b:2468 | model.pt | model.safetensors] [--input x.npy] \
        [--frames S] [--box x1 y1 x2 y2]

`--input` is a float32 [1, S, 3, 518, 518] array already square-padded,
resized and divided by 255 (the reference's cv2 read and cubic resize,
core/preprocess.py, are the caller's side); without it synthetic frames are
used.  `--box` is the content box pre-processing returned (default: the
whole map).
"""

import argparse
import os

import numpy as np

from monocular_depth_estimation_trt_amd import bench, common, spec, weights_vggt
from monocular_depth_estimation_trt_amd.common_runtime import allocate_buffers, do_inference, free_buffers

HERE = os.path.dirname(os.path.abspath(__file__))


def main(argv=None, model="vggt"):
    s = spec.load(model)
    size = spec.size_of(s)[0]
    ap = argparse.ArgumentParser(prog=model)
    ap.add_argument("--source", default="synthetic:vggt:vggt_1b:2468")
    ap.add_argument("--frames", type=int, default=int(s.get("frames", 1)))
    ap.add_argument("--engine", default="")
    ap.add_argument("--input", default="")
    ap.add_argument("--box", type=float, nargs=4, default=None)
    ap.add_argument("--iterations", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--out-dir", default=os.path.join(os.getcwd(), "reports", "bench"))
    a = ap.parse_args(argv)
    x = (np.load(a.input, allow_pickle=False).astype(np.float32) if a.input
         else weights_vggt.synthetic_images(1, a.frames, size, first_seed=0))
    if x.ndim != 5 or x.shape[0] != 1 or x.shape[2:] != (3, size, size):
        raise ValueError(f"[MDET] input must be [1, S, 3, {size}, {size}], got {x.shape}")
    frames = x.shape[1]
    engine_path = a.engine or os.path.join(HERE, "engine", f"vggt_only_depth_{size}x{size}_s{frames}_fp16.mdeng")
    with common.get_engine(a.source, engine_path, "fp16", None, input_hw=(size, size), frames=frames) as engine, \
            engine.create_execution_context() as context:
        inputs, outputs, bindings, stream = allocate_buffers(engine)
        inputs[0].host = x
        outs, samples = bench.measure(
            lambda: do_inference(context, engine=engine, bindings=bindings, inputs=inputs, outputs=outputs,
                                 stream=stream), warmup=a.warmup, iterations=a.iterations)
        depth = outs[0].reshape(frames, size, size).copy()
        bench.record(model, samples, encoder="fixed", warmup=a.warmup, precision="fp16", profile="bench",
                     input_h=size, input_w=size, engine_path=engine_path, outputs={"depth": depth},
                     notes=f"source={a.source}; frames={frames}", model_input=x, out_dir=a.out_dir)
        free_buffers(inputs, outputs, stream)
    if a.box:
        x1, y1, x2, y2 = a.box
        depth = depth[:, int(round(y1)):int(round(y2)), int(round(x1)):int(round(x2))]
    print(f"[MDET] max : {depth.max():0.5f} , min : {depth.min():0.5f}")
    return depth


if __name__ == "__main__":
    main()
