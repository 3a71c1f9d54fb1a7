"""The parity suite against pipeline 2 (cdc_kernels.hip: per-lane sub-span
scan, record links, lane-per-span walk), selected with CHUNKFS_AMD_PIPELINE=2.

Pipeline 2 was written while the GPU pool was unreachable, so it is not the
default and this module only runs when CHUNKFS_AMD_TEST_PIPELINE2=1 (an
explicit, time-limited GPU run), never as part of an unattended `-m gpu`
pass.  It re-runs every test of test_gpu_parity.py with pipeline 2.
"""
import os

import pytest

if os.environ.get("CHUNKFS_AMD_TEST_PIPELINE2") != "1":
    pytest.skip("pipeline 2 parity: set CHUNKFS_AMD_TEST_PIPELINE2=1", allow_module_level=True)

os.environ["CHUNKFS_AMD_PIPELINE"] = "2"
from test_gpu_parity import *  # noqa: E402,F401,F403  (same tests, pipeline 2 handles)
