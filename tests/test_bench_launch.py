"""bench.py's launch logic (CPU): `bench.py --gpus N` starts its own N ranks
when no launcher did (the driver passes only --gpus), and refuses
a launcher whose WORLD_SIZE disagrees with --gpus."""
import sys

import pytest

from conftest import REPO

sys.path.insert(0, str(REPO))
import bench  # noqa: E402  (imports no torch at module level)


def test_one_gpu_runs_in_process():
    assert bench.launch_plan(1, {}, ["--gpus", "1"], 29500) is None


def test_n_gpus_without_launcher_spawns_n_ranks():
    argv = ["--gpus", "4", "--steps", "3", "--dist-backend", "gloo"]
    cmd = bench.launch_plan(4, {}, argv, 29611)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29611" in cmd
    assert cmd[cmd.index(str(REPO / "bench.py")) + 1:] == argv  # the ranks get the same flags


def test_launcher_ranks_run_in_process():
    assert bench.launch_plan(2, {"WORLD_SIZE": "2", "RANK": "1"}, ["--gpus", "2"], 1) is None


def test_world_size_must_match_gpus():
    with pytest.raises(SystemExit, match="WORLD_SIZE=2 but --gpus 8"):
        bench.launch_plan(8, {"WORLD_SIZE": "2"}, ["--gpus", "8"], 1)
