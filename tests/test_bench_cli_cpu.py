"""bench.py's launch checks that run before any GPU call: a launcher whose WORLD_SIZE
differs from --gpus is an error (exit 2), never a silent 1-GPU line."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_world_size_mismatch_exits_nonzero():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "8", "--steps", "1"], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "WORLD_SIZE=2" in r.stderr
    assert '{"metric"' not in r.stdout
