"""Diagnostic: torch HIP init after a raw-ctypes render through a given libmassrt.so (argv[1])."""
import ctypes as C
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
L = C.CDLL(sys.argv[1])
b = C.c_void_p()
assert L.mrt_builder_new(C.c_uint64(1), C.byref(b)) == 0
assert L.mrt_builder_builtin(b, b"cornell", C.c_float(1.0), str(REPO / "tests" / "golden").encode()) == 0
desc = (C.c_uint8 * 4096)()
cam = (C.c_uint8 * 256)()
assert L.mrt_builder_desc(b, desc, cam) == 0
ctx = C.c_void_p()
assert L.mrt_create(0, C.byref(ctx)) == 0
assert L.mrt_upload_scene(ctx, desc) == 0
assert L.mrt_set_camera(ctx, cam) == 0
if len(sys.argv) > 2:
    import numpy as np
    W, H = 64, 48
    args = (C.c_uint32 * 10)(W, H, 0, 2, 1, 0, 50, 0, 1, 0)  # width height spp_begin spp_count seed(lo,hi) max_depth si sc flags
    rgb = np.zeros(W * H * 3, np.float32)
    bo = np.zeros(W * H, np.uint32)
    rc = L.mrt_render(ctx, args, rgb.ctypes.data_as(C.c_void_p), bo.ctypes.data_as(C.c_void_p))
    print("render rc", rc, "sum", float(rgb.sum()))
import torch  # noqa: E402

print(sys.argv[1:], "available:", torch.cuda.is_available(), flush=True)
torch.zeros(4, device="cuda")
print("ok", flush=True)
