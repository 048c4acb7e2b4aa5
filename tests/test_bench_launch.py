"""CPU tests of bench.py's launch decision for `--gpus N` (made before anything touches the GPU): N > 1
without a launcher spawns N ranks (torch.distributed.run) or fails when fewer GPUs are visible -- it
never measures one GPU and reports it as N; under a launcher N must equal WORLD_SIZE and the RCCL path
needs one GPU per rank.  Reference: the multi-worker run, src/bin/mrworker.rs:43-149."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def plan(gpus, env, n_dev, backend="nccl"):
    import bench
    return bench.launch_plan(gpus, backend, env, n_dev)


def test_single_gpu_default():
    assert plan(1, {}, 1) == "single"
    assert plan(1, {}, 0) == "single"           # no device: the library's own error says so later
    assert plan(1, {"WORLD_SIZE": "1"}, 8) == "single"


def test_spawn_when_no_launcher():
    assert plan(8, {}, 8) == "spawn"
    assert plan(2, {}, 8) == "spawn"
    assert plan(2, {}, 1, backend="gloo") == "spawn"   # the gloo rehearsal may share one GPU


@pytest.mark.parametrize("gpus,n_dev", [(2, 1), (8, 4), (4, 0)])
def test_more_gpus_than_visible_is_an_error(gpus, n_dev):
    with pytest.raises(SystemExit, match="visible"):
        plan(gpus, {}, n_dev)


def test_under_a_launcher():
    env = {"WORLD_SIZE": "4", "LOCAL_WORLD_SIZE": "4", "RANK": "1", "LOCAL_RANK": "1"}
    assert plan(4, env, 8) == "rank"
    with pytest.raises(SystemExit, match="WORLD_SIZE"):
        plan(2, env, 8)
    with pytest.raises(SystemExit, match="WORLD_SIZE"):
        plan(2, {"WORLD_SIZE": "1"}, 8)
    with pytest.raises(SystemExit, match="one GPU per rank"):
        plan(4, env, 2)
    assert plan(4, env, 1, backend="gloo") == "rank"
    with pytest.raises(SystemExit):
        plan(0, {}, 1)


def test_cli_exits_nonzero_without_enough_gpus():
    """`python bench.py --gpus 2` on a host with no GPU (this container): exits non-zero at once with the
    reason, instead of running and reporting one device."""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("two GPUs are visible")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--quick"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode != 0 and "visible" in p.stderr, p.stderr[-2000:]
