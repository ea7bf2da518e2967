"""Run bench.py against a variant library (timing A/B of a tools/ablate.py or
build_library(defines=...) build in the same gpurun call as the product):

    python tools/bench_lib.py build/var/px_NAME.so [bench.py args ...]
"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    lib = sys.argv[1]
    from monocular_depth_estimation_trt_amd import _lib
    _lib.use_library(lib)
    sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[2:]
    runpy.run_path(os.path.join(ROOT, "bench.py"), run_name="__main__")


if __name__ == "__main__":
    main()
