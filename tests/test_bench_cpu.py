"""bench.py's process-launch contract, checked without a GPU."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_gpus_without_devices_fails_cleanly():
    """`--gpus 2` over RCCL needs two visible GPUs; the launcher says so before any rank starts."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], capture_output=True,
                       text=True, timeout=300, env=dict(os.environ, HIP_VISIBLE_DEVICES=""))
    assert r.returncode == 2 and "needs 2 GPUs" in r.stderr


def test_world_size_must_match_gpus():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"], capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode != 0 and "WORLD_SIZE=2 but --gpus 1" in r.stderr


@pytest.mark.parametrize("args,msg", [(["--shard", "2/2"], "--shard R/N"), (["--shard", "x"], "wants R/N"),
                                      (["--config", "c5", "--graph"], "--graph needs")])
def test_bad_options_fail_before_the_gpu(args, msg):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode != 0 and msg in r.stderr, r.stderr[-2000:]
