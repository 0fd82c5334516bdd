"""bench.py's multi-rank paths, rehearsed on one GPU with the gloo backend.

The driver runs `torch.distributed.run --nproc-per-node N bench.py --gpus N`
over RCCL on an 8-GPU node; here two ranks share the box's one GPU and their
collectives go through gloo on host copies (bench.py --dist-backend gloo), so
the step structure, the timing fields and the JSON line of every workload's
N>1 path run end to end. Values are not performance numbers (two ranks share
one GPU).
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(n, *args, timeout=240):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", "29533", os.path.join(ROOT, "bench.py"),
           "--gpus", str(n), "--dist-backend", "gloo", "--no-cpu-baseline", *args]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]  # rank 0 alone prints
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["none", "all_to_all"])
def test_config2_two_ranks(mode):
    line = run_bench(2, "--steps", "3", "--warmup", "1", "--frames-per-gpu", "2", "--frame-exchange", mode)
    assert line["n_gpus"] == 2 and line["scaling"] == "weak" and line["value"] > 0
    assert line["config"]["frames_per_step"] == 4
    ranks = line["timing"]["per_rank"]
    assert [r["rank"] for r in ranks] == [0, 1] and all(r["kernel_ms"] > 0 for r in ranks)
    if mode == "none":
        assert line["timing"]["collective"] == "none" and "no collective" in line["config"]["parallelism"]
        assert line["roofline"]["bytes_per_launch"] == 2 * 1920 * 1080 * 16
    else:
        assert "all_to_all" in line["timing"]["collective"]
        assert all(r["collective_ms"] > 0 for r in ranks)


@pytest.mark.gpu
def test_config3_two_ranks_gather():
    line = run_bench(2, "--workload", "config3", "--steps", "3", "--warmup", "1")
    assert line["scaling"] == "strong" and line["timing"]["collective"] == "gather to rank 0"
    assert all(r["collective_ms"] > 0 and r["kernel_ms"] > 0 for r in line["timing"]["per_rank"])
    # each rank stores its float3 row blocks: half the frame's rows each
    assert line["roofline"]["bytes_per_launch"] == 3840 * 1080 * 12


@pytest.mark.gpu
def test_config5_two_ranks_all_reduce():
    line = run_bench(2, "--workload", "config5", "--steps", "2", "--warmup", "1")
    assert "all_reduce" in line["timing"]["collective"] and line["value"] > 0
