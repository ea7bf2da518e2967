"""Depth Pro on MI355X -- the counterpart of the reference driver
`models/depth_pro/onnx2trt.py:main` (:42-125), same sequence:

  input (normalised to [-1, 1], host-resized to 1536^2 with torch bilinear,
  align_corners=False) -> get_engine -> create_execution_context ->
  allocate_buffers -> bench.measure(do_inference) (20 warmup / 100
  iterations) -> post-process outside the timed loop (focal length from the
  predicted FOV, inverse depth * W / f_px, resize back to the source size,
  depth = 1 / clamp(inv, 1e-4, 1e4)) -> bench.record

    python -m monocular_depth_estimation_trt_amd.models.depth_pro.run \
        [--source synthetic:depth_pro | DepthPro.safetensors] [--input x.npy] [--src-hw H W]

`--input` is a float32 NCHW [1,3,H,W] image already normalised to [-1, 1]
(the reference's cv2 read is unavailable here); it is resized to 1536^2 on the
host like the reference does.  Without it a synthetic 1536^2 image is used.
"""

import argparse
import os

import numpy as np

from monocular_depth_estimation_trt_amd import bench, common, spec, weights_depth_pro
from monocular_depth_estimation_trt_amd.common_runtime import allocate_buffers, do_inference, free_buffers
from monocular_depth_estimation_trt_amd.postprocess import depth_pro_postprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def preprocess(x: np.ndarray, size: int) -> np.ndarray:
    """onnx2trt.py:72-83: bilinear (align_corners=False) resize of the
    normalised image to size x size when it is not already that size."""
    if x.shape[-2:] == (size, size):
        return np.ascontiguousarray(x, dtype=np.float32)
    import torch
    import torch.nn.functional as F
    t = torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32))
    return F.interpolate(t, size=(size, size), mode="bilinear", align_corners=False).numpy()


def main(argv=None, model="depth_pro"):
    s = spec.load(model)
    size = spec.size_of(s)[0]
    ap = argparse.ArgumentParser(prog=model)
    ap.add_argument("--source", default="synthetic:depth_pro:dinov2l16_384:4321")
    ap.add_argument("--engine", default=os.path.join(HERE, "engine", f"depth_pro_{size}x{size}_fp16.mdeng"))
    ap.add_argument("--input", default="")
    ap.add_argument("--src-hw", type=int, nargs=2, default=None,
                    help="source image size for the post-process (default: the input's own size)")
    ap.add_argument("--iterations", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--out-dir", default=os.path.join(os.getcwd(), "reports", "bench"))
    a = ap.parse_args(argv)
    x = (np.load(a.input, allow_pickle=False).astype(np.float32) if a.input
         else weights_depth_pro.synthetic_images(1, size, first_seed=0))
    H, W = x.shape[-2:]
    src_hw = tuple(a.src_hw) if a.src_hw else (H, W)
    x = preprocess(x, size)
    output_shapes = (1, 1, size, size)
    with common.get_engine(a.source, a.engine, "fp16", None, input_hw=(size, size)) as engine, \
            engine.create_execution_context() as context:
        inputs, outputs, bindings, stream = allocate_buffers(engine)
        inputs[0].host = x
        outs, samples = bench.measure(
            lambda: do_inference(context, engine=engine, bindings=bindings, inputs=inputs, outputs=outputs,
                                 stream=stream), warmup=a.warmup, iterations=a.iterations)
        inv = outs[0].reshape(output_shapes).copy()
        fov = outs[1].copy() if len(outs) > 1 else None
        depth, f_px = depth_pro_postprocess(inv, fov, src_hw)
        bench.record(model, samples, encoder="fixed", warmup=a.warmup, precision="fp16", profile="native",
                     input_h=size, input_w=size, engine_path=a.engine, outputs={"depth": depth, "f_px": np.array(f_px)},
                     notes=f"source={a.source}; 1536x1536 is upstream fixed", model_input=x, out_dir=a.out_dir)
        free_buffers(inputs, outputs, stream)
    print(f"[MDET] max : {depth.max()} , min : {depth.min()}")
    print(f"[MDET] predicted Focal length (by Depth Pro) : {f_px:0.2f}")
    return depth, f_px


if __name__ == "__main__":
    main()
