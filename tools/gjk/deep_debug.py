"""Debug helper (GPU box): the GPU GJK test entry vs the oracle on a few deep-overlap pairs."""
import sys
import numpy as np
sys.path.insert(0, "."); sys.path.insert(0, "tests")
from tests.test_gpu_selfcollision import _gpu, _oracle, _pairs  # noqa: E402
p = _pairs(4000, 11)
ids = [6, 10, 37, 38, 42]
g, o = _gpu(p[ids]), _oracle(p[ids])
np.set_printoptions(precision=5, suppress=True, linewidth=150)
print("gpu\n", g)
print("oracle\n", o)
