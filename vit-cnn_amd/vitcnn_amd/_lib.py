"""ctypes binding of libvitcnn_hip.so (the C ABI in include/vitcnn.h).

The argument types of every entry point are read from the header itself, so the Python
side can never drift from the C declarations.  There is no fallback: if the library is
missing or a symbol is absent, importing the product path raises.
"""
from __future__ import annotations

import ctypes
import os
import re

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_PKG, "libvitcnn_hip.so")   # the product library: the only one lib() ever loads
_HEADER_CANDIDATES = [
    os.path.join(_PKG, "..", "..", "include", "vitcnn.h"),
    os.path.join(_PKG, "vitcnn.h"),
]

_TYPE_MAP = {
    "unsigned long long": ctypes.c_ulonglong,
    "long long": ctypes.c_longlong,
    "int": ctypes.c_int,
    "long": ctypes.c_long,
    "float": ctypes.c_float,
    "size_t": ctypes.c_size_t,
    "hipStream_t": ctypes.c_void_p,
}


def header_path() -> str:
    for p in _HEADER_CANDIDATES:
        if os.path.exists(p):
            return os.path.abspath(p)
    raise RuntimeError("vitcnn.h not found next to the package (include/vitcnn.h)")


def parse_header(path: str | None = None):
    """{name: [ctypes arg types]} for every `VC_API int vc_*(...)` declaration."""
    text = open(path or header_path()).read()
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    out = {}
    for m in re.finditer(r"VC_API\s+int\s+(vc_\w+)\s*\(([^)]*)\)\s*;", text, flags=re.S):
        name, args = m.group(1), m.group(2)
        types = []
        for a in args.split(","):
            a = " ".join(a.split())
            if not a or a == "void":
                continue
            if "*" in a:
                types.append(ctypes.c_void_p)
                continue
            base = a.rsplit(" ", 1)[0].replace("const ", "").strip()
            if base not in _TYPE_MAP:
                raise RuntimeError(f"vitcnn.h: unsupported argument type '{a}' in {name}")
            types.append(_TYPE_MAP[base])
        out[name] = types
    return out


PROBE_PATH = os.path.join(_PKG, "libvitcnn_probe.so")


class _Lib:
    def __init__(self, path=None):
        path = path or LIB_PATH
        if not os.path.exists(path):
            raise RuntimeError(
                f"HIP extension not built: {path} is missing (run `make -C vit-cnn_amd/csrc` "
                "or __graft_entry__.build()); there is no CPU fallback")
        self.path = path
        self.handle = ctypes.CDLL(path)
        self.sigs = parse_header()
        self.raw = {}
        for name, types in self.sigs.items():
            fn = getattr(self.handle, name)  # AttributeError -> symbol missing: fail loudly
            fn.argtypes = types
            fn.restype = ctypes.c_int
            self.raw[name] = fn
            setattr(self, name, self._size(name, fn) if name.endswith("_floats") else self._checked(name, fn))

    @staticmethod
    def _size(name, fn):
        """`vc_*_floats` entry points are size queries: they return a count, negative on bad arguments"""
        def call(*args):
            n = fn(*args)
            if n < 0:
                raise RuntimeError(f"{name}{args}: invalid shape/argument")
            return n

        call.__name__ = name
        return call

    @staticmethod
    def _checked(name, fn):
        def call(*args):
            rc = fn(*args)
            if rc != 0:
                raise RuntimeError(f"{name} failed with code {rc} "
                                   f"({'invalid shape/argument' if rc == 1 else 'HIP launch error'})")
            return rc

        call.__name__ = name
        return call


_LIB = None


def lib() -> _Lib:
    """the product library, libvitcnn_hip.so next to this file.  No environment variable can point it
    elsewhere: a tool that A/Bs another build calls `use_library_for_tools` first."""
    global _LIB
    if _LIB is None:
        _LIB = _Lib()
    return _LIB


def use_library_for_tools(path: str) -> _Lib:
    """Measurement tools only (tools/knobs.py): bind `lib()` to another build of the same header -- the
    probe library or an A/B build -- before the product path first loads.  Raises if the product library
    is already bound, so a process never mixes two builds."""
    global _LIB
    if _LIB is not None and os.path.abspath(_LIB.path) != os.path.abspath(path):
        raise RuntimeError(f"lib() already bound to {_LIB.path}; cannot switch to {path}")
    if _LIB is None:
        _LIB = _Lib(path)
    return _LIB


_PROBE = None


def probe_lib() -> _Lib:
    """libvitcnn_probe.so (`make -C vit-cnn_amd/csrc probe`): the same sources built with -DVC_PROBE, whose
    measurement knobs read VITCNN_* variables per call (tools/, and tests comparing two
    bit-identical kernel forms in one process).  The product path never loads it."""
    global _PROBE
    if _PROBE is None:
        _PROBE = _Lib(PROBE_PATH)
    return _PROBE
