"""bench.py's launch logic and step plan (CPU): `bench.py --gpus N` runs one
process over N devices by default (mode "multi", the library's multi-device
context), starts its own N ranks in mode "ranks" when no launcher did, and
refuses a launcher whose WORLD_SIZE disagrees with --gpus. A step renders
BASELINE's whole 1920x1080x1024 frame for any N (strong scaling; VERDICT r3
next #1), and the bench line's workload label says what was rendered."""
import sys

import pytest

from conftest import REPO

sys.path.insert(0, str(REPO))
import bench  # noqa: E402  (imports no torch at module level)


def test_one_gpu_runs_in_process():
    assert bench.launch_plan(1, {}, ["--gpus", "1"], 29500) is None


def test_multi_mode_runs_in_process():
    assert bench.launch_plan(8, {}, ["--gpus", "8"], 29500) is None
    assert bench.launch_plan(8, {}, ["--gpus", "8"], 29500, "multi") is None


def test_n_gpus_without_launcher_spawns_n_ranks():
    argv = ["--gpus", "4", "--steps", "3", "--dist-backend", "gloo", "--mode", "ranks"]
    cmd = bench.launch_plan(4, {}, argv, 29611, "ranks")
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29611" in cmd
    assert cmd[cmd.index(str(REPO / "bench.py")) + 1:] == argv  # the ranks get the same flags


def test_launcher_ranks_run_in_process():
    assert bench.launch_plan(2, {"WORLD_SIZE": "2", "RANK": "1"}, ["--gpus", "2"], 1) is None


def test_world_size_must_match_gpus():
    with pytest.raises(SystemExit, match="WORLD_SIZE=2 but --gpus 8"):
        bench.launch_plan(8, {"WORLD_SIZE": "2"}, ["--gpus", "8"], 1)


def _args(*argv):
    old = sys.argv
    sys.argv = ["bench.py", *argv]
    try:
        return bench.parse()
    finally:
        sys.argv = old


@pytest.mark.parametrize("n", [1, 2, 4, 8])
def test_step_plan_is_the_config_frame_for_any_n(n):
    a = _args("--gpus", str(n))
    p = bench.step_plan(a, n)
    assert p["spp_per_step"] == 1024
    assert p["samples_per_step"] == 1920 * 1080 * 1024
    assert p["scaling"] == "strong"
    assert p["workload"] == "sphere_grid 1920x1080x1024spp per step, max_depth 50"
    assert bench.device_list(a) == list(range(n))


def test_weak_plan_labels_what_it_renders():
    a = _args("--gpus", "8", "--weak")
    p = bench.step_plan(a, 8)
    assert p["samples_per_step"] == 1920 * 1080 * 1024 * 8 and p["scaling"] == "weak"
    assert "8192spp per step" in p["workload"]


def test_rehearsal_devices():
    assert bench.device_list(_args("--gpus", "2", "--devices", "0,0")) == [0, 0]
    with pytest.raises(SystemExit, match="--devices lists 1"):
        bench.device_list(_args("--gpus", "2", "--devices", "0"))


def test_context_options_from_flags():
    assert bench.context_options(_args("--opt", "queues=1", "--opt", "trace_chunk=256")) == \
        {"queues": 1, "trace_chunk": 256}


def test_env_options_reach_bench_contexts_only(monkeypatch):
    """MASSRT_OPTIONS is read by bench.py (context_options), never by
    massrt.Context itself; --opt overrides it; malformed items name themselves."""
    import massrt

    monkeypatch.setenv("MASSRT_OPTIONS", "traversal=1, queues=2")
    assert bench.context_options(_args("--opt", "queues=1")) == {"traversal": 1, "queues": 1}
    assert massrt.parse_options("a=0x10,b=-1") == {"a": 16, "b": -1}
    for bad in ("queues", "=3", "queues=x"):
        with pytest.raises(ValueError, match="not NAME=INTEGER"):
            massrt.parse_options(bad, "MASSRT_OPTIONS")
    import inspect

    assert "env_options" not in inspect.getsource(massrt.Context.__init__)
