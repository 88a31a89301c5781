import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "nlos-gaussian-renderer_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")
CASES = ["noocl_g16_s4_r16_d0", "noocl_g64_s8_r32_d3", "netf_g64_s4_r16_d3",
         "noocl_g256_s8_r64_d3", "netf_g32_s8_r64_d1", "noocl_g16_s5_r24_d2",
         "noocl_g32_s4_r16_d4", "netf_g32_s4_r16_d4"]   # SH degree 4: torch preset


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box)")


def load_case(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    d = {k: z[k] for k in z.files}
    if "meta" in d:
        d["meta"] = json.loads(str(d["meta"]))
    return d


@pytest.fixture(params=CASES)
def golden_case(request):
    return load_case(request.param)


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
