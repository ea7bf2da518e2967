"""distill_any_depth on MI355X -- the counterpart of the reference's
models/distill_any_depth/onnx2trt.py (no post-process: the 518x518 map, :98-100).  The model is the DA-V2 ViT-S graph with the relative head, so the
DA-V2 driver runs it with this model's spec.json.

    python -m monocular_depth_estimation_trt_amd.models.distill_any_depth.run [DA-V2 driver flags]
"""

from monocular_depth_estimation_trt_amd.models.depth_anything_v2.run import main as _main


def main(argv=None):
    return _main(argv, model="distill_any_depth")


if __name__ == "__main__":
    main()
