import os
import sys
from pathlib import Path

import pytest

# the tests A/B kernels by toggling S3OD_* dispatch knobs between calls in one process: S3OD_AB=1 makes the library
# re-read its knobs per call (it reads them once otherwise; s3od_amd/csrc/common.hpp S3OD_KNOB)
os.environ.setdefault("S3OD_AB", "1")
# the CHECKER's fp32 torch convolutions (the oracle on cuda) go through MIOpen, whose default find searches and
# compiles candidate kernels per new shape: on a fresh box the oracle's 2048^2 forward took 148 s that way and 2.3 s
# in immediate mode (profiles/r06b_c5_oracle_miopen.txt).  The product path has no MIOpen call.
os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
GOLDEN = REPO / "tests" / "golden"
FIXTURE = REPO / "tests" / "fixture"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through libs3od_hip.so)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def synth_sd_torch():
    import torch
    from s3od_amd.weights import synthetic_state_dict
    return {k: torch.from_numpy(v) for k, v in synthetic_state_dict(0).items()}
