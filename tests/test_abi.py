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


def test_ops_refuse_cpu_tensors():
    import pytest
    import torch
    from ugpg import ops
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        ops.mean_std(torch.ones(8))
