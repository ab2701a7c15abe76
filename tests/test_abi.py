"""CPU-side checks of the drop-in boundary: the C-ABI library loads and exports every function
include/fgi.h declares (no compute calls without a GPU), and the product refuses to run without
its HIP library instead of falling back to anything."""
import ctypes
import os

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "fgi.h")


def test_library_exports_every_header_symbol(pkg):
    lib = pkg.load_library()
    names = pkg.fgi.header_symbols(HEADER)
    assert len(names) >= 30
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, f"missing exports: {missing}"
    # and the ctypes binding declares a signature for each of them
    declared = set(pkg.fgi.SIGNATURES) | {"fgi_last_error"}
    assert set(names) <= declared, set(names) - declared


def test_library_is_gfx950_code_object(pkg):
    import subprocess
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", pkg.LIB_PATH], capture_output=True, text=True)
    blob = open(pkg.LIB_PATH, "rb").read()
    assert b"gfx950" in blob, "libfgi.so carries no gfx950 code object"


def test_version(pkg):
    lib = pkg.load_library()
    a, b = ctypes.c_uint32(), ctypes.c_uint32()
    assert lib.fgi_version(ctypes.byref(a), ctypes.byref(b)) == 0
    assert (a.value, b.value) >= (0, 1)


def test_create_without_gpu_fails_loudly(pkg):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(pkg.FgiError):
        pkg.Graph(16)


def test_missing_library_raises(pkg, tmp_path):
    with pytest.raises(pkg.FgiError):
        pkg.fgi.load_library.__wrapped__ if hasattr(pkg.fgi.load_library, "__wrapped__") else None
        import importlib
        m = importlib.import_module("stl_fusion_amd.fgi")
        saved = m._lib
        try:
            m._lib = None
            m.load_library(str(tmp_path / "libfgi.so"))
        finally:
            m._lib = saved


def test_bad_config_rejected(pkg):
    lib = pkg.load_library()
    cfg = pkg.fgi.Config(0, 0, 16, 0, 0, 0, 1)   # struct_size 0
    h = ctypes.c_void_p()
    assert lib.fgi_create(ctypes.byref(cfg), ctypes.byref(h)) == pkg.fgi.EINVAL


def test_rccl_info_reports_the_bound_library(pkg):
    """fgi_rccl_info names the RCCL the engine's collectives bind to. libfgi does not link librccl: it
    resolves the entry points from /opt/rocm's librccl.so.1 (RTLD_LOCAL), so torch's bundled librccl —
    the same soname, loaded first by any process that imports torch — cannot take its place."""
    import torch  # noqa: F401  (loads torch's librccl into this process first)
    v, path = pkg.fgi.rccl_info()
    assert v >= 22700 and "rccl" in os.path.basename(path)
    assert os.path.realpath(path).startswith(os.path.realpath("/opt/rocm")), path


def test_header_is_plain_c(tmp_path):
    """include/fgi.h is the drop-in boundary: it compiles as strict C99 (no C++ or HIP types), so a cgo,
    JNI, N-API or P/Invoke binding can include or mirror it."""
    import shutil
    import subprocess
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    src = tmp_path / "h.c"
    src.write_text('#include "fgi.h"\nint main(void) { fgi_step s; fgi_batch_stats b; (void)s; (void)b; return 0; }\n')
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
    r = subprocess.run([cc, "-std=c99", "-Wall", "-Wextra", "-pedantic", "-Werror", "-I", inc, "-c", str(src), "-o",
                        str(tmp_path / "h.o")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
