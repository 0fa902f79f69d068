"""MI355X (gfx950) HIP runtime of the YOLOv11 inference path.

`Engine` wraps one yh_handle (include/yolo_hip.h); `nms` is the on-device
non_max_suppression. The drop-in module API lives in `nets.nn` / `utils.util`.
"""
from .variants import VARIANTS, Variant, lookup  # noqa: F401


def __getattr__(name):
    # torch-dependent pieces load lazily so `import yolo_hip` stays cheap
    if name in ("Engine", "nms"):
        from . import engine
        return getattr(engine, name)
    raise AttributeError(name)
