"""ctypes binding of libs3od_hip.so, driven by include/s3od_hip.h.

The header is parsed at import time so the Python side binds exactly the declared C ABI.
There is no fallback: if the library is missing or cannot be loaded this raises, and every
op of the product path fails loudly (tier rule: no silent CPU / PyTorch substitute).
"""
from __future__ import annotations

import ctypes
import os
import re
from pathlib import Path

import torch  # noqa: F401  -- must load torch's libamdhip64 first so both share one HIP runtime

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
LIB_PATH = Path(os.environ.get("S3OD_HIP_LIB", PKG / "libs3od_hip.so"))
HEADER = ROOT / "include" / "s3od_hip.h"
if not HEADER.exists():  # installed layout
    HEADER = PKG / "s3od_hip.h"

F32, BF16 = 0, 1
_CT = {
    "int": ctypes.c_int, "long": ctypes.c_long, "float": ctypes.c_float, "double": ctypes.c_double,
    "void*": ctypes.c_void_p, "float*": ctypes.c_void_p, "double*": ctypes.c_void_p, "char*": ctypes.c_char_p,
    "long*": ctypes.c_void_p, "int*": ctypes.c_void_p,
}
_DECL = re.compile(r"^(int|const char\*)\s+(s3od_\w+)\(([^)]*)\);", re.M)


def parse_nrep(path=HEADER):
    """S3OD_NREP: replicas of the accumulation workspaces (their sizes are stated in the header)."""
    return int(re.search(r"#define S3OD_NREP (\d+)", Path(path).read_text()).group(1))


NREP = parse_nrep()


def parse_header(path=HEADER):
    decls = {}
    for ret, name, args in _DECL.findall(Path(path).read_text()):
        types = []
        a = args.strip()
        if a and a != "void":
            for part in a.split(","):
                toks = part.replace("const ", "").replace("*", "* ").split()
                base = toks[0] + ("*" if len(toks) > 1 and toks[1] == "*" else "")
                if "*" in part and not base.endswith("*"):
                    base += "*"
                types.append(base)
        decls[name] = (ret, types)
    return decls


class HipLibError(RuntimeError):
    pass


class _Lib:
    def __init__(self):
        if not LIB_PATH.exists():
            raise HipLibError(f"libs3od_hip.so not found at {LIB_PATH}: run `make` (or __graft_entry__.build())")
        self.lib = ctypes.CDLL(str(LIB_PATH))
        self.decls = parse_header()
        self.fns = {}
        self.timers = {}     # name -> list of (start, end, args, phase) recorded around each call
        self.phase = None    # set by the engine ("encoder" / "decoder" / "prepare") for the bench breakdown
        self.cost = None     # optional fn(name, args) -> (kind, work), evaluated at call time (no tensor kept alive)
        for name, (ret, types) in self.decls.items():
            fn = getattr(self.lib, name)
            fn.argtypes = [_CT[t] for t in types]
            fn.restype = ctypes.c_char_p if ret.startswith("const char") else ctypes.c_int
            self.fns[name] = (fn, types)

    def __call__(self, name, *args):
        fn, types = self.fns[name]
        if len(args) != len(types):
            raise TypeError(f"{name}: expected {len(types)} args, got {len(args)}")
        cargs = []
        for a, t in zip(args, types):
            if t.endswith("*"):
                if a is None:
                    cargs.append(None)
                elif isinstance(a, torch.Tensor):
                    if a.device.type != "cuda":
                        raise HipLibError(f"{name}: tensor argument on {a.device}, expected a GPU tensor")
                    cargs.append(a.data_ptr())
                else:
                    cargs.append(int(a))
            else:
                cargs.append(a)
        tm = None
        if self.timers:
            tm = self.timers.get(name)
            if tm is None and "*" in self.timers:       # time every entry point (bench breakdown pass)
                tm = self.timers.setdefault(name, [])
        if tm is not None:
            # events on the stream the kernel is launched on (the last argument of every entry)
            st = torch.cuda.ExternalStream(cargs[-1]) if types[-1] == "void*" and cargs[-1] else torch.cuda.current_stream()
            e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
            e0.record(st)
            rc = fn(*cargs)
            e1.record(st)
            tm.append((e0, e1, self.cost(name, args) if self.cost else None, self.phase))
        else:
            rc = fn(*cargs)
        if rc != 0:
            raise HipLibError(f"{name} failed (rc={rc}): {self.last_error()}")
        return rc

    def last_error(self):
        return self.lib.s3od_last_error().decode()


_LIB = None


def lib() -> _Lib:
    global _LIB
    if _LIB is None:
        _LIB = _Lib()
    return _LIB


def stream():
    return torch.cuda.current_stream().cuda_stream
