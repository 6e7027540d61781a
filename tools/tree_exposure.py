"""How many pixels of C1 / C3 depend on which tree the reference traverses:
the reference kernels over the plain HLBVH and over the GPU-treelet tree
(each also checked bit-exact against the HIP path), the differing pixels
counted (tests/test_gpu_trees.py).  One JSON line per case.

    python tools/tree_exposure.py [C1 C3]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from montecarlopathtracing_amd import render as R  # noqa: E402
from tests.test_gpu_trees import CASES, tree_exposure  # noqa: E402

if __name__ == "__main__":
    rnd = R.Renderer(0)
    for case in sys.argv[1:] or sorted(CASES):
        print(json.dumps(tree_exposure(rnd, case)), flush=True)
