"""pytest configuration: `-m gpu` tests need a real MI355X (run them via gpurun);
everything else runs on CPU."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "gym-futbol_amd"), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD GPU (MI355X); run on the GPU box")
    config.addinivalue_line("markers", "slow: long-running CPU test")
