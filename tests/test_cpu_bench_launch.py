"""bench.py's N-GPU entry (no GPU needed): --gpus N without a launcher starts torch.distributed.run as
a child and refuses when fewer GPUs are visible; under a launcher the world size must equal --gpus."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "TT_REHEARSE_GLOO")}
    env.update(kw)
    return env


def test_gpus_n_without_gpus_refuses_in_parent():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--no-cpu-baseline"], cwd=ROOT,
                       env=_env(HIP_VISIBLE_DEVICES=""), capture_output=True, text=True, timeout=120)
    assert r.returncode == 2, (r.stdout, r.stderr[-2000:])
    assert "only 0 GPU(s) visible" in r.stderr


def test_world_size_must_match_gpus():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "3", "--no-cpu-baseline"], cwd=ROOT,
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode != 0
    assert "must agree" in r.stderr
