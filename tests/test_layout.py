"""The record-stream layout (layout.h, upload.cpp relayout_blas) on the host,
no GPU: the same rays through the preorder stream (build_host_scene(..., sibling_layout=false)) and
through the default layout (BLAS regions with siblings together, every
successor explicit) find the same closest hits, t bits included, after the
same number of box tests; the early slab decision stays exact
(tools/slab_check.cpp, which restates k_trace's walk on the host)."""
import shutil
import subprocess

import pytest

from conftest import GOLDEN, REPO


@pytest.fixture(scope="module")
def slab_check(tmp_path_factory):
    if not shutil.which("g++"):
        pytest.skip("g++ missing")
    exe = tmp_path_factory.mktemp("slab") / "slab_check"
    lib = REPO / "mass-raytrace_amd" / "massrt"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", str(exe), str(REPO / "tools" / "slab_check.cpp"),
                    f"-L{lib}", "-lmassrt", f"-Wl,-rpath,{lib}"], check=True)
    return exe


@pytest.mark.parametrize("scene", ["cornell", "sphere_grid", "cube_field"])
def test_sibling_layout_walks_like_the_preorder_stream(slab_check, scene):
    r = subprocess.run([str(slab_check), scene, "20000", str(GOLDEN), "layout"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 of 20000 rays differ" in r.stdout, r.stdout


@pytest.mark.slow
def test_sibling_layout_mesh(slab_check, assets_dir):
    r = subprocess.run([str(slab_check), "mesh_ply", "20000", str(assets_dir), "layout"], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0 and " 0 of 20000 rays differ" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("scene", ["cornell", "sphere_grid", "cube_field"])
def test_near_first_walk_finds_the_reference_hits(slab_check, scene):
    """The verified near-first walk (nf_tree.cpp's trees, path.h's steps,
    restated by tools/slab_check.cpp walk_nf): on camera and bounce rays the
    same closest hits as the reference's left-first walk — primitive,
    container, t bits — with fewer box tests; the stack stays within kNfStack."""
    r = subprocess.run([str(slab_check), scene, "30000", str(GOLDEN), "nf"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " nf: 0 of 30000 rays differ" in r.stdout, r.stdout
    boxes = r.stdout.split("box tests ")[1].split(" per ray")[0].split(" vs ")
    assert float(boxes[0]) < float(boxes[1]), r.stdout


@pytest.mark.slow
@pytest.mark.parametrize("scene", ["mesh_ply", "menger_l3"])
def test_near_first_walk_mesh_and_menger(slab_check, assets_dir, scene):
    r = subprocess.run([str(slab_check), scene, "20000", str(assets_dir), "nf"], capture_output=True, text=True,
                       timeout=900)
    assert r.returncode == 0 and " nf: 0 of 20000 rays differ" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("scene", ["cornell", "cube_field", "sphere_grid"])
def test_near_first_grazing_rays(slab_check, scene):
    """The near-first walk's hardest rays (massrt.h MRT_TRAVERSAL_*, DESIGN.md
    §4): nearly parallel to a triangle (10^-8 to 10^-1.5 rad), where
    Moller-Trumbore's computed t can undercut the plane by far more than the
    2^-10 culling margin. The walk's triangle boxes are thickened by 2^-6 of
    the triangle's extent (nf_tree.cpp kTriThick) so such a ray meets the box
    before the plane: no ray of the deterministic sample may differ (before
    the thickening: cornell 24, cube_field 80 of 400k)."""
    r = subprocess.run([str(slab_check), scene, "100000", str(GOLDEN), "graze"], capture_output=True, text=True,
                       timeout=600)
    line = [x for x in r.stdout.splitlines() if " nf: " in x][0]
    assert " nf: 0 of 100000 rays differ" in line, line


@pytest.mark.parametrize("scene", ["sphere_grid"])
def test_near_first_tangent_rays(slab_check, scene):
    """Rays nearly tangent to a sphere from 1-400 radii (the sphere test's
    disc cancels there): the same hits as the reference walk."""
    r = subprocess.run([str(slab_check), scene, "100000", str(GOLDEN), "tangent"], capture_output=True, text=True,
                       timeout=600)
    line = [x for x in r.stdout.splitlines() if " nf: " in x][0]
    assert " nf: 0 of 100000 rays differ" in line, line
