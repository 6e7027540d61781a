"""The bench contract on the GPU box: the default line, and the N-rank path
(torch.distributed.run, one process per rank, barrier + max over ranks)
rehearsed with two ranks sharing the box's one GPU (MCPT_BENCH_SHARED_GPU=1:
gloo instead of RCCL for the barrier and the max-reduce; the RCCL init path
is the same code with backend "nccl")."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _lines(out):
    return [json.loads(x) for x in out.splitlines() if x.startswith("{")]


def test_bench_two_ranks_rehearsal():
    env = dict(os.environ, MCPT_BENCH_SHARED_GPU="1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
                        "--steps", "4", "--warmup", "1", "--no-cpu"], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _lines(r.stdout)
    assert len(lines) == 1, r.stdout  # rank 0 only
    j = lines[0]
    assert j["n_gpus"] == 2 and j["steps"] == 4 and j["scaling"] == "weak"
    assert j["value"] > 0 and j["config"]["parallelism"] == "row-stripe tiles x2"
    assert j["cpu_baseline"] is None  # rank 0 at N=1 only
    assert j["image_reduce_ms"] is not None and j["image_reduce_ms"] > 0  # the final image reduce ran


def test_bench_c4_strong_two_ranks_rehearsal():
    env = dict(os.environ, MCPT_BENCH_SHARED_GPU="1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
                        "--workload", "C4", "--steps", "2", "--warmup", "1", "--no-cpu"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    j = _lines(r.stdout)[0]
    assert j["scaling"] == "strong" and j["config"]["height_per_gpu"] == 540
    assert j["image_reduce_ms"] is not None
