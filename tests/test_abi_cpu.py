"""CPU-side checks of the drop-in boundary: the C-ABI library loads (no GPU needed), exports
every symbol include/s3od_hip.h declares, the header is in sync with the sources, and the
product path refuses to run without a GPU (no silent CPU fallback)."""
import ctypes
import subprocess
import sys
from pathlib import Path

import pytest
import torch

REPO = Path(__file__).resolve().parent.parent


def test_header_in_sync(tmp_path):
    from s3od_amd._lib import parse_header, HEADER
    before = HEADER.read_text()
    subprocess.run([sys.executable, str(REPO / "tools" / "gen_header.py")], check=True, capture_output=True)
    assert HEADER.read_text() == before, "include/s3od_hip.h is stale: run tools/gen_header.py"
    decls = parse_header()
    assert len(decls) >= 30


def test_library_exports_every_declared_symbol():
    from s3od_amd._lib import lib, LIB_PATH
    L = lib()
    raw = ctypes.CDLL(str(LIB_PATH))
    for name in L.decls:
        assert hasattr(raw, name), name
    assert L.lib.s3od_abi_version() == 2
    # every declared arg type maps to a ctypes type
    for name, (ret, types) in L.decls.items():
        assert len(L.fns[name][0].argtypes) == len(types)


def test_invalid_argument_reports_error():
    from s3od_amd._lib import lib, HipLibError
    # K not a multiple of 8 is rejected on the host before any launch
    with pytest.raises(HipLibError, match="multiples of 8"):
        lib()("s3od_linear_fwd", 1, 8, 8, 7, 0, 7, 0, None, None, None, 0, None, 8, None, 0, 0, 0, 8, 0, None, 8, 0, 0, 0, 0)


def test_product_path_refuses_cpu():
    from s3od_amd.model import DPTSegmentation
    m = DPTSegmentation(init_seed=None)
    with pytest.raises(RuntimeError, match="GPU"):
        m(torch.zeros(1, 3, 32, 32))


def test_cpu_tensor_rejected():
    from s3od_amd._lib import lib, HipLibError
    with pytest.raises(HipLibError):
        lib()("s3od_rope_table", torch.zeros(4), torch.zeros(4), 1, 1, 1.0, 0)
