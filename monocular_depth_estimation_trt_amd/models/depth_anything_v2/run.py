"""Depth Anything V2 (and its family) on MI355X -- the counterpart of the
reference drivers `models/depth_anything_v2/onnx2trt.py:main` (:42-127),
`models/depth_anything_ac/onnx2trt.py` and `models/distill_any_depth/
onnx2trt.py` (the same ViT-S DA-V2 graph, relative head), same sequence:

  input -> get_engine -> create_execution_context -> allocate_buffers ->
  bench.measure(do_inference) (20 warmup / 100 iterations) ->
  post-process (bilinear align_corners=True back to the source size, clamp
  [1e-3, 1e3], outside the timed loop) -> bench.record

    python -m monocular_depth_estimation_trt_amd.models.depth_anything_v2.run \
        [--source synthetic:vits:metric | ckpt.pth] [--input x.npy] [--src-hw H W]
        [--input-format float32_nchw | uint8_nhwc] [--host-postprocess]

`--input` is an already-preprocessed float32 NCHW [1,3,518,518] tensor (the
reference's core/preprocess.py needs cv2, absent here), or for
`--input-format uint8_nhwc` the uint8 [1,518,518,3] image the reference's
uint8 engine takes (core/onnx_tools.py:87-219: normalisation on the device);
without it a synthetic image of the spec's input domain is used.  The
post-process runs on the device (postprocess.DevicePostprocess) unless
`--host-postprocess` asks for the reference's torch-CPU version.
"""

import argparse
import os

import numpy as np

from monocular_depth_estimation_trt_amd import bench, common, spec, weights
from monocular_depth_estimation_trt_amd.postprocess import DevicePostprocess
from monocular_depth_estimation_trt_amd.common_runtime import allocate_buffers, do_inference, free_buffers

HERE = os.path.dirname(os.path.abspath(__file__))


def postprocess(depth: np.ndarray, src_hw) -> np.ndarray:
    """onnx2trt.py:111-117: bilinear(align_corners=True) to the source size, clamp."""
    import torch
    import torch.nn.functional as F
    t = torch.from_numpy(np.ascontiguousarray(depth))[:, None]
    t = F.interpolate(t, tuple(src_hw), mode="bilinear", align_corners=True)[0, 0]
    return torch.clamp(t, min=1e-3, max=1e3).numpy()


def main(argv=None, model="depth_anything_v2"):
    s = spec.load(model)
    mc = spec.model_config_of(s)
    input_h, input_w = mc["input_hw"]
    ap = argparse.ArgumentParser(prog=model)
    ap.add_argument("--source", default=f"synthetic:{mc['encoder']}:{mc['depth_type']}:1234")
    ap.add_argument("--engine", default=os.path.join(os.path.dirname(HERE), model, "engine",
                                                     f"{model}_{mc['encoder']}_{input_h}x{input_w}_fp16.mdeng"))
    ap.add_argument("--input", default="")
    ap.add_argument("--src-hw", type=int, nargs=2, default=[2268, 3024])
    ap.add_argument("--iterations", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--out-dir", default=os.path.join(os.getcwd(), "reports", "bench"))
    ap.add_argument("--input-format", choices=("float32_nchw", "uint8_nhwc"), default="float32_nchw")
    ap.add_argument("--host-postprocess", action="store_true")
    a = ap.parse_args(argv)
    u8 = a.input_format == "uint8_nhwc"
    if u8 and a.engine.endswith("_fp16.mdeng"):
        a.engine = a.engine[:-len("_fp16.mdeng")] + "_u8_fp16.mdeng"
    if u8:
        x = (np.load(a.input, allow_pickle=False).astype(np.uint8) if a.input
             else weights.synthetic_images_u8(1, input_h, input_w, first_seed=0))
    else:
        x = (np.load(a.input, allow_pickle=False).astype(np.float32) if a.input
             else weights.synthetic_images(1, input_h, input_w, first_seed=0))
    output_shape = (1, input_h, input_w)
    with common.get_engine(a.source, a.engine, "fp16", None, encoder=mc["encoder"], depth_type=mc["depth_type"],
                           max_depth=mc["max_depth"], input_hw=(input_h, input_w),
                           input_format=a.input_format) as engine, \
            engine.create_execution_context() as context:
        inputs, outputs, bindings, stream = allocate_buffers(engine, output_shape, profile_idx=0)
        inputs[0].host = x
        outs, samples = bench.measure(
            lambda: do_inference(context, engine=engine, bindings=bindings, inputs=inputs, outputs=outputs,
                                 stream=stream), warmup=a.warmup, iterations=a.iterations)
        if mc["postprocess"] == "none":   # distill_any_depth: the 518x518 map as is (its onnx2trt.py:98-100)
            depth = outs[0].reshape(output_shape)[0].copy()
        elif a.host_postprocess:
            depth = postprocess(outs[0].reshape(output_shape), a.src_hw)
        else:  # the engine's output is still in outputs[0].device
            with DevicePostprocess(1, input_h, input_w, *a.src_hw) as pp:
                depth = pp.run(outputs[0].device, stream)[0].copy()
        bench.record(model, samples, warmup=a.warmup, precision="fp16", profile="bench",
                     variant="u8" if u8 else "single",
                     input_h=input_h, input_w=input_w, engine_path=a.engine, outputs={"depth": depth},
                     encoder=mc["encoder"], notes=f"source={a.source}", model_input=x, out_dir=a.out_dir)
        print(f"[MDET] max : {depth.max():0.5f} , min : {depth.min():0.5f}")
        free_buffers(inputs, outputs, stream)
    return depth


if __name__ == "__main__":
    main()
