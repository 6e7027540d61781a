"""The MCPT_DEBUG build of the fused kernel (make -C montecarlopathtracing_amd/csrc
debug -> lib/libmcpt_hip_debug.so): every stack push checked against the
stack's capacity and every node / triangle index against its array.  The
reference traversal keeps an unchecked int stack[64] (objdef.h:247); here the
bound computed at upload is verified at run time on the C1
image, the deep diningroom proxy and the C5 random mesh with both stack
layouts, both search-tree node formats, both modes and both leaf schedules:
zero violations, C1 still equal to the reference kernels' golden image, and
the stack layouts and node formats bit-identical."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEBUG_LIB = os.path.join(ROOT, "montecarlopathtracing_amd", "lib", "libmcpt_hip_debug.so")


@pytest.mark.skipif(not os.path.exists(DEBUG_LIB), reason="debug build missing (__graft_entry__.build makes it)")
def test_debug_build_bounds_checks_clean():
    env = dict(os.environ, MCPT_LIB_OVERRIDE=DEBUG_LIB)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "debug_check.py")], env=env, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert "MCPT_DEBUG" in lines[0]["version"]
    cases = lines[1:]
    assert len(cases) == 24
    for c in cases:
        assert c["violations"] == 0, c
    assert all(c["golden"] for c in cases if c["case"] in ("c1", "c1_quant"))
    # EXACT mode searched the quantized tree where forced (NOPRUNE never does)
    assert {c["quantized"] for c in cases if c["case"].endswith("_quant") and c["mode"] == 0} == {1}
    assert {c["quantized"] for c in cases if not c["case"].endswith("_quant") or c["mode"] == 1} == {0}
    assert {c["stack_window"] for c in cases if c["case"] == "c5_window"} == {1}
    assert {c["stack_window"] for c in cases if c["case"] == "c5_plain"} == {0}
    for mode in (0, 1):
        for sched in (0, 1):
            win = [c for c in cases if c["case"] == "c5_window" and c["mode"] == mode and c["schedule"] == sched]
            plain = [c for c in cases if c["case"] == "c5_plain" and c["mode"] == mode and c["schedule"] == sched]
            assert win[0]["digest"] == plain[0]["digest"]
    for name in ("c1", "dining", "c5_window"):
        assert len({c["digest"] for c in cases if c["case"] == name}) == 1  # modes and schedules agree
    for name in ("c1", "c5_window"):  # node formats agree
        assert {c["digest"] for c in cases if c["case"] == name + "_quant"} == {c["digest"] for c in cases
                                                                               if c["case"] == name}
