"""CPU tests of the C-ABI boundary: the library builds for gfx950, loads,
and exports exactly what include/vrpms.h declares (no compute calls)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "vrpms.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(vrpms_[a-z_0-9]+)\s*\(", text)))


@pytest.fixture(scope="module")
def libpath():
    from vrpms_amd.build import build_library
    return build_library()


def test_library_is_gfx950(libpath):
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", libpath],
                         capture_output=True, text=True).stdout
    assert ".hip_fatbin" in out
    blob = open(libpath, "rb").read()
    assert b"gfx950" in blob


def test_exports_every_declared_symbol(libpath):
    import torch  # noqa: F401 -- same load order as the product binding
    lib = ctypes.CDLL(libpath)
    decl = declared_functions()
    assert len(decl) >= 8
    for name in decl:
        assert hasattr(lib, name), f"{name} declared in vrpms.h but not exported"


def test_ctypes_signatures_cover_header():
    from vrpms_amd._lib import SIGNATURES
    assert sorted(SIGNATURES) == declared_functions()


def test_header_compiles_as_c(tmp_path):
    src = tmp_path / "t.c"
    src.write_text('#include "vrpms.h"\nint main(void){return vrpms_version() < 0;}\n')
    res = subprocess.run(["gcc", "-c", "-std=c99", "-Wall", "-Werror", "-I",
                          os.path.join(ROOT, "include"), str(src), "-o", str(tmp_path / "t.o")],
                         capture_output=True, text=True)
    assert res.returncode == 0, res.stderr


def test_version_and_error_paths_without_gpu(libpath):
    import torch  # noqa: F401
    lib = ctypes.CDLL(libpath)
    lib.vrpms_version.restype = ctypes.c_int
    assert lib.vrpms_version() >= 1
    # NULL ctx is rejected before any HIP call
    lib.vrpms_eval.restype = ctypes.c_int
    assert lib.vrpms_eval(None, None, 1, 0, 0, 0, None, None, None, None, None) == -1
    lib.vrpms_last_error.restype = ctypes.c_char_p
    assert b"ctx is NULL" in lib.vrpms_last_error()


def test_product_path_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from vrpms_amd.core import Context
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        Context(0)
