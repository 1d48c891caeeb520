"""The C ABI library: loads, exports exactly what include/massrt.h declares,
and fails loudly (no CPU fallback) when no HIP device is present."""
import re

import pytest

import massrt
from conftest import REPO


def header_functions():
    text = (REPO / "include" / "massrt.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mrt_[a-z0-9_]+)\s*\(", text)) - {"mrt_ref"})


def test_header_symbols_exported():
    lib = massrt.lib()
    names = header_functions()
    assert len(names) >= 30
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert sorted(massrt.EXPORTED_SYMBOLS) == names


def test_abi_version():
    assert massrt.lib().mrt_abi_version() == massrt.ABI_VERSION == 9


def test_struct_layouts_match_header(tmp_path):
    """ctypes mirrors == the C compiler's view of massrt.h (size and offsets)."""
    import ctypes as C
    import shutil
    import subprocess
    if not shutil.which("gcc"):
        pytest.skip("gcc missing")
    structs = {"mrt_node": massrt.MrtNode, "mrt_sphere": massrt.MrtSphere, "mrt_triangle": massrt.MrtTriangle,
               "mrt_instance": massrt.MrtInstance, "mrt_model": massrt.MrtModel, "mrt_material": massrt.MrtMaterial,
               "mrt_surface": massrt.MrtSurface, "mrt_texture": massrt.MrtTexture,
               "mrt_background": massrt.MrtBackground, "mrt_scene_desc": massrt.MrtSceneDesc,
               "mrt_camera": massrt.MrtCamera, "mrt_render_args": massrt.MrtRenderArgs, "mrt_hit": massrt.MrtHit,
               "mrt_counters": massrt.MrtCounters, "mrt_kernel_stats": massrt.MrtKernelStats,
               "mrt_tuning": massrt.MrtTuning}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{REPO}/include/massrt.h"', "int main(void){"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0;}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    subprocess.run(["gcc", "-o", str(tmp_path / "layout"), str(src)], check=True)
    out = subprocess.run([str(tmp_path / "layout")], check=True, capture_output=True, text=True).stdout
    for line in out.splitlines():
        key, val = line.rsplit(" ", 1)
        if key.endswith(" size"):
            cname = key[:-5]
            assert C.sizeof(structs[cname]) == int(val), cname
        else:
            cname, f = key.split(".")
            assert getattr(structs[cname], f).offset == int(val), key


def test_library_was_built_from_this_tree():
    """mrt_build_info carries the source hash the Makefile baked in: the
    library the tests (and the GPU box) load is HEAD's code, not a stale build."""
    import src_hash

    assert massrt.build_info() == "src " + src_hash.src_hash()


def test_no_gpu_multi_device_context_fails_loudly():
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(massrt.MassrtError, match="no HIP device"):
        massrt.Context(devices=[0, 0])


def test_no_gpu_fails_loudly():
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(massrt.MassrtError, match="no HIP device"):
        massrt.Context(0)


def test_builder_errors_are_reported():
    b = massrt.Builder(1)
    with pytest.raises(massrt.MassrtError, match="unknown built-in scene"):
        b.builtin("no_such_scene")
    with pytest.raises(massrt.MassrtError, match="empty"):
        b.build_bvh()  # BvhNode::new(vec![]) would recurse forever in the reference
    with pytest.raises(massrt.MassrtError, match="out of range"):
        b.material(massrt.MAT_LAMBERTIAN, surface=7)


def test_transport_choice_and_rccl_fallback():
    """mrt_create_multi's transport choice (frames.hip choose_transport),
    without GPUs: one device "none", repeated devices "peer", distinct devices
    RCCL when librccl opens, and — RCCL pointed at a missing library — the
    peer-copy fallback with the reason in the transport text."""
    import massrt

    assert massrt.debug_transport([0]) == "none"
    assert massrt.debug_transport([0, 0, 0]) == "peer"
    t = massrt.debug_transport([0, 1], rccl_library="librccl_missing_for_test.so")
    assert t.startswith("peer (RCCL unavailable: RCCL (librccl_missing_for_test.so) is not available"), t
    # the real loader: RCCL between distinct devices where librccl opens (it
    # is in this image); elsewhere the peer-copy fallback is the right answer
    import ctypes

    try:
        ctypes.CDLL("librccl.so.1")
        have_rccl = True
    except OSError:
        try:
            ctypes.CDLL("/opt/rocm/lib/librccl.so.1")
            have_rccl = True
        except OSError:
            have_rccl = False
    t8 = massrt.debug_transport([0, 1, 2, 3, 4, 5, 6, 7])
    t2 = massrt.debug_transport([3, 5])  # the hook is reset: the default library again
    if have_rccl:
        assert t8 == "rccl" and t2 == "rccl", (t8, t2)
    else:
        assert t8.startswith("peer (RCCL unavailable") and t2.startswith("peer (RCCL unavailable"), (t8, t2)
