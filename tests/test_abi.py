"""The C-ABI library loads and exports every symbol the public header declares; argument
validation paths that need no device behave like the reference's `Plan::try_new` (no GPU)."""
import ctypes
import os
import subprocess

import pytest

from conftest import ROOT


def test_library_exports_header_symbols(engine):
    from tfhe_ntt_amd import _lib

    L = _lib.lib()
    syms = _lib.declared_symbols()
    assert "mi_ntt64_fwd_batch" in syms and "mi_ntt64_plan_create" in syms
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    # and nm agrees that they are real exported (T) text symbols of the .so
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert set(syms) <= exported


def test_library_is_gfx950_code_object(engine):
    from tfhe_ntt_amd import _lib

    out = subprocess.run(["strings", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert "gfx950" in out


@pytest.mark.parametrize("n,p,status", [
    (8, 0xFFFFFFFF00000001, 1),      # N < 16 -> None (prime64.rs:769)
    (48, 0xFFFFFFFF00000001, 1),     # not a power of two
    (0, 0xFFFFFFFF00000001, 1),
    (2048, 1024, 2),                 # not prime (prime64.rs:1988-1990 test_plan_crash_github_11)
    (2048, 2**61 - 1, 3),            # prime without a 4096-th root of unity
])
def test_plan_create_rejects_like_reference(engine, n, p, status):
    from tfhe_ntt_amd import _lib

    h = ctypes.c_void_p()
    st = _lib.lib().mi_ntt64_plan_create(n, p, 0, ctypes.byref(h))
    assert st == status and not h.value
    assert engine.Plan.try_new(n, p) is None
    assert _lib.lib().mi_status_string(st)


def test_null_arguments_are_errors_not_crashes(engine):
    from tfhe_ntt_amd import _lib

    L = _lib.lib()
    assert L.mi_ntt64_plan_create(2048, 0xFFFFFFFF00000001, 0, None) == _lib.MI_ERR_INVALID_ARG
    assert L.mi_ntt64_fwd_batch(None, None, 1, 2048, None) == _lib.MI_ERR_INVALID_ARG
    assert L.mi_ntt64_plan_info(None, None, None, None) == _lib.MI_ERR_INVALID_ARG
    assert L.mi_ntt64_plan_destroy(None) == _lib.MI_OK
    assert b"NULL" in L.mi_last_error_message()


def test_header_compiles_as_c(tmp_path):
    src = tmp_path / "t.c"
    src.write_text('#include "tfhe_ntt_amd.h"\nint main(void){ return (int)sizeof(&mi_ntt64_fwd_batch) == 0; }\n')
    r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), "-c",
                        str(src), "-o", str(tmp_path / "t.o")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


@pytest.mark.gpu
def test_single_hip_runtime_in_process(engine):
    """The engine shares the process's HIP runtime (SONAME libamdhip64.so.7): after torch and the engine have both
    run GPU work, exactly one libamdhip64 is mapped ('two HIP runtimes' — this pins that there is one
    per process, whichever the process loaded first)."""
    import torch
    plan = engine.Plan.try_new(64, 0xFFFFFFFF00000001)
    t = torch.zeros(4 * 64, dtype=torch.int64, device="cuda")
    plan.fwd(t.view(4, 64))
    torch.cuda.synchronize()
    paths = engine._lib.hip_runtimes()
    assert len(paths) == 1, paths


def test_integration_rust_binding_covers_the_header():
    """INTEGRATION.md's Rust extern block is tools/gen_rust_sys.py's output for the current header: every C-ABI
    function is bound, with the translated signature."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    gen = subprocess.run([sys.executable, os.path.join(root, "tools", "gen_rust_sys.py")], capture_output=True,
                         text=True, check=True).stdout.strip()
    assert gen in open(os.path.join(root, "INTEGRATION.md")).read()


def test_integration_rust_binding_declares_every_opaque_type():
    import re
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    hdr = open(os.path.join(root, "include", "tfhe_ntt_amd.h")).read()
    doc = open(os.path.join(root, "INTEGRATION.md")).read()
    opaque = set(re.findall(r"typedef struct (mi_\w+) \1;", hdr))
    assert opaque <= set(re.findall(r"pub struct (mi_\w+)", doc)), opaque - set(re.findall(r"pub struct (mi_\w+)", doc))


def test_library_built_from_this_tree():
    """Build provenance: the loaded library's embedded source hash (tools/source_hash.py, written by the Makefile)
    equals the hash of the sources beside it, so the tests and the bench never run a stale or foreign .so."""
    from tfhe_ntt_amd import _lib
    prov = _lib.build_provenance()
    assert len(prov["so_source_hash"]) == 64
    assert prov["match"] is True, prov
