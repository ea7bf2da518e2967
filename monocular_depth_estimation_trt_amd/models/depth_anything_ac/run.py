"""depth_anything_ac on MI355X -- the counterpart of the reference's
models/depth_anything_ac/onnx2trt.py (resize to the source size + clamp, :128-130).  The model is the DA-V2 ViT-S graph with the relative head, so the
DA-V2 driver runs it with this model's spec.json.

    python -m monocular_depth_estimation_trt_amd.models.depth_anything_ac.run [DA-V2 driver flags]
"""

from monocular_depth_estimation_trt_amd.models.depth_anything_v2.run import main as _main


def main(argv=None):
    return _main(argv, model="depth_anything_ac")


if __name__ == "__main__":
    main()
