"""Diagnostic: does torch's HIP init still work after libmassrt did X?"""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO / "mass-raytrace_amd"))
import massrt  # noqa: E402

step = sys.argv[1]
massrt.lib()
if step in ("single", "multi", "image"):
    b = massrt.Builder(1).builtin("cornell", 1.0, str(REPO / "tests" / "golden"))
    c = massrt.Context(0) if step == "single" else massrt.Context(devices=[0, 0])
    c.upload(b)
    if step == "image":
        im = massrt.Image(c, 64, 48)
        im.render(1, 0, 2)
        print("image passes", im.read()[2])
    else:
        c.render(64, 48, 0, 2)
import torch  # noqa: E402

print(step, "torch.cuda.is_available:", torch.cuda.is_available(), "count:", torch.cuda.device_count(), flush=True)
torch.zeros(4, device="cuda")
print(step, "ok", flush=True)
