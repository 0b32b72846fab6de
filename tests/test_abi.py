"""The C-ABI library builds, loads, and exports exactly what include/ugpg.h declares
(no compute calls: runs without a GPU)."""
import re
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
HEADER = ROOT / "include" / "ugpg.h"


def declared():
    txt = HEADER.read_text()
    return sorted(set(re.findall(r"\b(ugpg_[a-z0-9_]+)\s*\(", txt)))


def test_library_loads_and_reports_version():
    from ugpg import _C
    assert _C.LIB_PATH.exists(), "build libugpg.so first (python ug-pg-unet_amd/build.py)"
    assert _C.version().startswith("ugpg ")
    assert _C.lib.ugpg_last_error() is not None


def test_library_is_built_from_these_sources():
    """The in-tree library's embedded build id is the content hash of csrc/ + include/ +
    flags (a stale prebuilt .so travels with the tree to the GPU box),
    and the loader refuses a library whose id differs."""
    import importlib.util
    import pytest
    from ugpg import _C
    spec = importlib.util.spec_from_file_location("_b", ROOT / "ug-pg-unet_amd" / "build.py")
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    assert _C.lib.ugpg_build_id().decode() == b.source_id() == b.lib_id(_C.LIB_PATH)
    assert b.source_id().split("-")[0] == b.content_id()

    def fake(ident):
        class Fn:  # a ctypes function stand-in returning `ident`
            def __call__(self):
                return ident.encode()

        class Lib:
            ugpg_build_id = Fn()
        return Lib()

    with pytest.raises(ImportError, match="stale"):
        _C._check_fresh(fake("0" * 32 + "-" + b.source_id().split("-")[1]))
    # the same sources built with another configuration (UGPG_ARCH, defines) are
    # not stale -- only the content part is compared, not this process's environment
    _C._check_fresh(fake(b.content_id() + "-" + "f" * 32))


def test_every_declared_symbol_is_exported_and_bound():
    from ugpg import _C
    names = declared()
    assert len(names) >= 35
    out = subprocess.run(["nm", "-D", "--defined-only", str(_C.LIB_PATH)], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (ugpg_[a-z0-9_]+)", out))
    missing = [n for n in names if n not in exported]
    assert not missing, f"declared but not exported: {missing}"
    unbound = [n for n in names if n not in _C.SIGNATURES]
    assert not unbound, f"declared but not bound in _C.SIGNATURES: {unbound}"
    extra = [n for n in _C.SIGNATURES if n not in names]
    assert not extra, f"bound but not declared: {extra}"


def test_library_is_gfx950_code():
    from ugpg import _C
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", str(_C.LIB_PATH)],
                         capture_output=True, text=True).stdout
    data = _C.LIB_PATH.read_bytes()
    assert b"gfx950" in data


def test_invalid_arguments_fail_loudly_without_gpu():
    """Argument validation runs on the host and reports through ugpg_last_error."""
    from ugpg import _C
    rc = _C.lib.ugpg_pack_conv3x3(None, None, 64, 3, 1, 0, 0, None)
    assert rc == -1
    assert b"pack_conv3x3" in _C.lib.ugpg_last_error()


def test_lazy_bn_dy_wgrad_validation_without_gpu():
    """ugpg_wgrad_t.dy_bn: refused (workspace query 0, an error naming it) outside the
    split-bf16 arithmetic or with a dy beside it; checked before any launch."""
    import ctypes as C
    from ugpg import _C
    p = C.cast(C.c_void_p(0x1000), C.c_void_p)
    lz = _C.BnLazy(p, p, p, p, p, p, p, None, None, None)
    d = _C.WgradDesc()
    d.B, d.H, d.W = 1, 8, 16
    d.src[0] = _C.Src(p, None, None, 64, None)
    d.Cout, d.dw, d.Cin_real, d.math = 64, p, 64, 2  # UGPG_WFMT_BF16
    d.dy_bn = C.pointer(lz)
    assert _C.lib.ugpg_conv3x3_wgrad_workspace(C.byref(d)) == 0
    assert b"dy_bn" in _C.lib.ugpg_last_error()
    d.math = 1  # UGPG_WFMT_X6, but a dy as well
    d.dy = p
    assert _C.lib.ugpg_conv3x3_wgrad_workspace(C.byref(d)) == 0
    d.dy = None
    assert _C.lib.ugpg_conv3x3_wgrad_workspace(C.byref(d)) > 0


def test_ops_refuse_cpu_tensors():
    import pytest
    import torch
    from ugpg import ops
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ops.mean_std(torch.ones(8))


def test_host_side_under_asan_ubsan():
    """the C-ABI's host side (argument validation, error strings, plan and
    workspace arithmetic, communicator bookkeeping) built with AddressSanitizer and
    UndefinedBehaviorSanitizer on the host only (-Xarch_host) and driven with invalid
    arguments through every entry (tests/_abi_sanitized_driver.py), ASan runtime preloaded."""
    import glob
    import importlib.util
    import os
    import sys
    spec = importlib.util.spec_from_file_location("ugpg_build", ROOT / "ug-pg-unet_amd" / "build.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    lib = mod.build_sanitized()
    syms = subprocess.run(["nm", "-D", str(lib)], capture_output=True, text=True, check=True).stdout
    assert "__asan_init" in syms and "__ubsan_handle" in syms, "sanitizers not linked in"
    rt = glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so")
    assert rt, "ASan runtime not found"
    env = dict(os.environ, LD_PRELOAD=rt[0], UGPG_LIB=str(lib),
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([sys.executable, str(ROOT / "tests" / "_abi_sanitized_driver.py")],
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "entries refused invalid arguments" in r.stdout
