"""bench.py's N > 1 path rehearsed on one GPU: two ranks launched exactly as the driver
launches them (python -m torch.distributed.run --nproc-per-node 2 ... bench.py --gpus 2),
with gloo standing in for RCCL (RCCL refuses two ranks on one device; the code path is the
same: GradReducer buckets streamed out of the backward, row-sparse stack tables, the gated
enc4 schedule, per-bucket Adam, barrier + max-over-ranks timing). fp32 (cfg 2) and the
bf16 mode (cfg 3) at reduced per-GPU batch; rank 0 must print one well-formed JSON line."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("workload", ["cfg2", "cfg3"])
def test_bench_two_ranks_gloo_rehearsal(workload):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    env = dict(os.environ, SAVQA_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
           "--workload", workload, "--batch", "32", "--steps", "2", "--warmup", "1",
           "--no-cpu-baseline", "--no-roofline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 64
    assert d["value"] > 0 and d["ms_per_step"] > 0
    assert d["loss"] == d["loss"] and abs(d["loss"]) < 1e4   # finite
    # the per-rank exchange diagnosis: every rank's own step time, the
    # collectives' summed time, the part that outlasted the backward, and the bytes; the two
    # stack tables go by rows, the rest densely (the whole live range, 457M floats at cfg 2)
    c = d["comm"]
    assert c["bucket_mb"] == 64.0 and c["bwd_schedule"] == "enc4" and c["diag_steps"] == 2
    assert sorted(r["rank"] for r in c["ranks"]) == [0, 1]
    for r in c["ranks"]:
        assert r["ms_per_step"] > 0 and r["allreduce_ms"] > 0 and r["exposed_ms"] >= 0
        assert r["rows_tables"] == 2 and r["rows_MB"] > 0
        assert r["dense_MB"] > 500 and r["collectives"] > 10, r


def test_bench_comm_flags_two_ranks():
    """--bucket-mb / --bwd-gate reach the reducer and the engine (the first real SCALE run
    can sweep them) and are echoed in the line's comm report."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    env = dict(os.environ, SAVQA_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
           "--batch", "16", "--steps", "1", "--warmup", "1", "--no-cpu-baseline",
           "--no-roofline", "--bucket-mb", "256", "--bwd-gate", "concurrent", "--comm-steps", "1"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith('{"metric"')][0])
    c = d["comm"]
    assert c["bucket_mb"] == 256.0 and c["bwd_schedule"] == "concurrent"
    assert c["diag_steps"] == 1 and len(c["ranks"]) == 2


def test_bench_launcherless_form_starts_n_ranks():
    """`python bench.py --gpus 2` with no launcher starts its own two ranks (a
    torch.distributed.run child) and reports the process group's world size, not 1."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    env = dict(os.environ, SAVQA_DIST_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--batch", "16", "--steps", "2",
           "--warmup", "1", "--no-cpu-baseline", "--no-roofline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 32
    assert d["dist"]["world_size"] == 2 and d["dist"]["backend"] == "gloo"
    assert sorted(x["rank"] for x in d["dist"]["ranks"]) == [0, 1]
