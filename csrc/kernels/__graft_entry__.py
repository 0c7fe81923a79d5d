"""Driver entry points: build() compiles every native component for gfx950
in-tree; smoke() runs one tiny forward+backward of the flagship model on
cuda:0."""
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def build() -> None:
    os.environ.setdefault("PYTORCH_ROCM_ARCH", "gfx950")
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import build_native

    build_native.build(["core", "kernels"])
    import torch  # noqa: F401  (HIP runtime first)
    import flexflow_train_amd  # noqa: F401
    import flexflow_train_amd._ffcore  # noqa: F401
    import flexflow_train_amd._ffkernels  # noqa: F401


def smoke() -> None:
    from flexflow_train_amd.utils.smoke import run_smoke

    run_smoke()


if __name__ == "__main__":
    build()
    if len(sys.argv) > 1 and sys.argv[1] == "smoke":
        smoke()
