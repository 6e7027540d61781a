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
    # headline: weak scaling, a 1024x2048 image, a 1024x1024 share per rank
    # (the path partitions: no data-path collective); the strong-scaled leg
    # (the fixed 1024x1024 image striped over the ranks) beside it
    assert j["n_gpus"] == 2 and j["steps"] == 4 and j["scaling"] == "weak"
    assert j["value"] > 0 and j["config"]["parallelism"] == "row-stripe tiles x2"
    assert j["config"]["width"] == 1024 and j["config"]["height"] == 2048
    s = j["strong_scaling"]
    assert s["value"] > 0 and s["image"] == [1024, 1024]
    # the one-GPU time of the same image inside the job, and every rank's share
    assert s["one_gpu_ms"] > 0 and s["speedup_vs_1gpu"] > 0 and s["one_gpu_value"] > 0
    assert len(s["share_ms_per_rank"]) == 2 and all(x > 0 for x in s["share_ms_per_rank"])
    assert s["share_max_over_mean"] >= 1.0
    assert j["cpu_baseline"] is None  # rank 0 at N=1 only
    assert j["image_reduce_ms"] is not None and j["image_reduce_ms"] > 0  # the final image reduce ran
    # the host dump (device-to-host copy of rank 0's image state), timed outside value
    assert j["host_dump"]["bytes"] == 1024 * 2048 * 24 and j["host_dump"]["value_with_dump_per_call"] < j["value"]
    # the strong-scaling answers at the top level (the scaling record's reader):
    # the fixed 1024x1024 image, and C4's 1920x1080 image striped over the ranks
    assert j["strong_speedup_vs_1gpu"] == s["speedup_vs_1gpu"] > 0
    c4 = j["c4_strong_scaling"]
    assert c4["image"] == [1920, 1080] and len(c4["share_ms_per_rank"]) == 2 and c4["one_gpu_ms"] > 0
    assert j["c4_strong_speedup_vs_1gpu"] == c4["speedup_vs_1gpu"] > 0


def test_bench_c4_strong_two_ranks_rehearsal():
    env = dict(os.environ, MCPT_BENCH_SHARED_GPU="1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
                        "--workload", "C4", "--steps", "2", "--warmup", "1", "--no-cpu"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    j = _lines(r.stdout)[0]
    assert j["scaling"] == "strong" and j["config"]["height"] == 1080
    s = j["strong_scaling"]  # the headline's own image: its one-GPU time and shares
    assert s["image"] == [1920, 1080] and s["value"] == j["value"]
    assert s["one_gpu_ms"] > 0 and s["speedup_vs_1gpu"] > 0 and len(s["share_ms_per_rank"]) == 2
    assert j["image_reduce_ms"] is not None
    assert j["strong_speedup_vs_1gpu"] == j["c4_strong_speedup_vs_1gpu"] == s["speedup_vs_1gpu"]


def test_bench_default_line():
    """The driver's own command at N = 1: the contract keys, a roofline whose
    fractions are fractions, and the CPU baseline with its core count."""
    r = subprocess.run([sys.executable, "bench.py", "--steps", "8", "--warmup", "2"], cwd=ROOT, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    j = _lines(r.stdout)[-1]
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in j, k
    assert j["n_gpus"] == 1 and j["steps"] == 8 and j["value"] > 0
    roof = j["roofline"]
    assert roof["bound"] == "hbm" and roof["peak"] == 8000.0
    for k in ("frac", "issue_frac", "valu_lane_utilization"):
        assert roof.get(k) is None or 0.0 <= roof[k] <= 1.0, (k, roof.get(k))
    if "td" in roof:  # the binding unit's busy fraction is a fraction
        assert 0.0 < roof["td"]["frac"] <= 1.0 and roof["binding_unit"] == "td"
    assert roof["lanes_per_node_gather_inst"] > 0 and roof["tests_per_leaf_phase"] > 0
    # the primary-hit cache serves each pixel's first segment of each frame
    assert roof["segments_cache_served"] == 1024 * 1024 * 8
    assert roof["segments_traced"] > 0
    assert j["primary_cache_off"]["value"] > 0
    cpu = j["cpu_baseline"]
    assert cpu["cores"] >= 1 and cpu["threads"] == cpu["cores"] and cpu["cpu_model"] and cpu["value"] > 0
