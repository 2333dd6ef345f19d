"""GPU parity of the 4-wave 256x256 GEMM kernel (gemm_q.hip igemm_q_kernel) through the C ABI: the ping-pong kernel's
linear cases (tests/test_gpu_gemm_pp.py -- same shapes, epilogues, tolerances and fp32 torch references) rerun with
S3OD_GEMM_CFG=6, which routes s3od_linear_fwd / _dgrad / _wgrad to it (the M-tail launches keep their 128x128 /
skinny kernels)."""
import pytest

from tests.test_gpu_gemm_pp import (test_pp_gelu_saved_derivative_pair as test_q_gelu_saved_derivative_pair,  # noqa: F401
                                    test_pp_linear_dgrad_accumulate as test_q_linear_dgrad_accumulate,
                                    test_pp_linear_dgrad_gelu_bwd as test_q_linear_dgrad_gelu_bwd,
                                    test_pp_linear_fwd_gelu as test_q_linear_fwd_gelu,
                                    test_pp_linear_fwd_residual_pre as test_q_linear_fwd_residual_pre,
                                    test_pp_linear_wgrad_split as test_q_linear_wgrad_split,
                                    test_pp_production_rows_65616 as test_q_production_rows_65616)

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _q_config(monkeypatch):
    monkeypatch.setenv("S3OD_GEMM_CFG", "6")       # read per call: tests/conftest.py sets S3OD_AB=1
