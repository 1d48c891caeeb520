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


def _bound(stdout: str):
    """(checks, worst dist/rho, over) from slab_check's `nf bound:` line."""
    line = [x for x in stdout.splitlines() if " nf bound: " in x][0]
    checks = int(line.split("nf bound: ")[1].split(" accepted")[0])
    worst = float(line.split("worst dist/rho ")[1].split(",")[0])
    over = int(line.split(" over;")[0].rsplit(", ", 1)[1])
    return checks, worst, over, line


@pytest.mark.parametrize("scene", ["cornell", "sphere_grid", "cube_field"])
def test_near_first_walk_finds_the_reference_hits(slab_check, scene):
    """The verified near-first walk (nf_tree.cpp's trees, path.h's steps,
    restated by tools/slab_check.cpp walk_nf): on camera and bounce rays the
    same closest hits as the reference's left-first walk — primitive,
    container, t bits — with fewer record loads; the stack stays within
    kNfStack. Every hit the reference's tests accept lies within the walk's
    rounding margin rho of its box (nf_bound.h)."""
    r = subprocess.run([str(slab_check), scene, "30000", str(GOLDEN), "nf"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " nf: 0 of 30000 rays differ" in r.stdout, r.stdout
    loads = r.stdout.split("record loads ")[1].split(" (x")[0].split(" vs ")
    assert float(loads[0]) < float(loads[1]), r.stdout
    checks, worst, over, line = _bound(r.stdout)
    assert checks > 10000 and over == 0 and worst < 0.25, line


@pytest.mark.slow
@pytest.mark.parametrize("scene", ["mesh_ply", "menger_l3"])
def test_near_first_walk_mesh_and_menger(slab_check, assets_dir, scene):
    r = subprocess.run([str(slab_check), scene, "20000", str(assets_dir), "nf"], capture_output=True, text=True,
                       timeout=900)
    assert r.returncode == 0 and " nf: 0 of 20000 rays differ" in r.stdout, r.stdout + r.stderr
    checks, worst, over, line = _bound(r.stdout)
    assert over == 0 and worst < 0.25, line
    if scene == "mesh_ply":  # normal cones (nf_bound.h nf_cone_rg): the generic term priced per node
        cones = [x for x in r.stdout.splitlines() if " nf cones: " in x][0]
        assert int(cones.split("nf cones: ")[1].split(" of")[0]) > 100_000, cones
        per_ray = float(r.stdout.split(" box tests ")[1].split(" vs")[0])
        assert per_ray < 42.0, r.stdout  # 64.6 with the worst-case |det| >= 1e-6 pricing, 43.7 before wild entries
        # the floor and the two thin light boxes are wild (nf_bound.h NfWild): each is entered only when the
        # ray meets its world box thickened by its own margin, so the walk enters fewer instances than the
        # reference's (3.0 per ray while the nodes above them never culled them)
        _wild_checked(r.stdout, 3)
        entries = float(r.stdout.split("instance entries per ray ")[1].split()[0])
        ref_entries = float(r.stdout.split("reference walk: instance entries per ray ")[1].split()[0])
        assert entries < ref_entries and entries < 1.0, r.stdout


def _wild_checked(stdout: str, n_wild: int):
    """slab_check's wild lines: n_wild wild instances, every accepted hit of one within its own margin of its
    world box (check_hit_wild), and rays that pass them by on that test."""
    assert f", {n_wild} wild instances" in stdout, stdout
    line = [x for x in stdout.splitlines() if " nf wild: " in x][0]
    assert int(line.split("nf wild: ")[1].split(" hits")[0]) > 100, line
    assert float(line.split("worst dist/rho ")[1]) < 0.25, line
    passed = float(stdout.split("nf wild instances passed by per ray ")[1].split()[0].rstrip(";"))
    assert passed > 0.1, stdout


def test_wild_instance_cornell(slab_check):
    """Cornell's thin light (cond |F||G| ~ 1.4e4: a wild instance, nf_tree.cpp wild()): its hits lie within its
    own instance term of its world box, which the walk tests at the wild leaf (path.h nf_wild_enter) instead of
    entering it on every ray; the closest hits stay the reference's."""
    r = subprocess.run([str(slab_check), "cornell", "30000", str(GOLDEN), "nf"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and " nf: 0 of 30000 rays differ" in r.stdout, r.stdout + r.stderr
    _wild_checked(r.stdout, 1)


@pytest.mark.slow
def test_near_first_grazing_rays_mesh_cones(slab_check, assets_dir):
    """The 1M-triangle mesh's generic triangles under the normal-cone bound
    (round 6): rays within 10^-8..10^-1.5 rad of a triangle's plane sit in
    the cone's grazing band, where each node falls back to the worst-case
    |det| >= 1e-6 term; every accepted hit still lies within the (cone-
    narrowed) rho of every NF node above it, and no closest hit differs."""
    r = subprocess.run([str(slab_check), "mesh_ply", "20000", str(assets_dir), "graze"], capture_output=True,
                       text=True, timeout=900)
    line = [x for x in r.stdout.splitlines() if " nf: " in x][0]
    assert " nf: 0 of 20000 rays differ" in line, line
    checks, worst, over, bline = _bound(r.stdout)
    assert checks > 20000 and over == 0 and worst < 0.25, bline
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.parametrize("scene", ["cornell", "cube_field", "sphere_grid"])
def test_near_first_grazing_rays(slab_check, scene):
    """The near-first walk's hardest rays (massrt.h MRT_TRAVERSAL_*, DESIGN.md
    §4): nearly parallel to a triangle (10^-8 to 10^-1.5 rad), where
    Moller-Trumbore's computed t is least accurate. The walk thickens every
    box by its proven bound rho on how far a computed hit can lie outside its
    primitive's box (nf_bound.h): every accepted hit of the sample lies within
    rho of its box, with room to spare (worst dist/rho < 0.25), and no ray's
    closest hit differs."""
    r = subprocess.run([str(slab_check), scene, "100000", str(GOLDEN), "graze"], capture_output=True, text=True,
                       timeout=600)
    line = [x for x in r.stdout.splitlines() if " nf: " in x][0]
    assert " nf: 0 of 100000 rays differ" in line, line
    checks, worst, over, bline = _bound(r.stdout)
    assert checks > 100000 and over == 0 and worst < 0.25, bline
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.parametrize("scene", ["sphere_grid"])
def test_near_first_tangent_rays(slab_check, scene):
    """Rays nearly tangent to a sphere from 1-400 radii (the sphere test's
    disc cancels there): the same hits as the reference walk, and every
    accepted hit within the sphere bound's rho of its box."""
    r = subprocess.run([str(slab_check), scene, "100000", str(GOLDEN), "tangent"], capture_output=True, text=True,
                       timeout=600)
    line = [x for x in r.stdout.splitlines() if " nf: " in x][0]
    assert " nf: 0 of 100000 rays differ" in line, line
    checks, worst, over, bline = _bound(r.stdout)
    assert checks > 100000 and over == 0 and worst < 0.25, bline
