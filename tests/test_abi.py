"""CPU-only: the C ABI library is built for gfx950, loads, and exports exactly what include/janus_gpu.h
declares.  No compute calls (there is no GPU here)."""
import ctypes
import re
import subprocess
from pathlib import Path

import pytest

import janus_gpu as jg

ROOT = Path(__file__).resolve().parent.parent
HEADER = ROOT / "include" / "janus_gpu.h"


def header_functions():
    src = HEADER.read_text()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*int\s+(jg_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_the_boundary():
    names = header_functions()
    assert len(names) >= 25
    for must in ("jg_open", "jg_pnc_merge_rows", "jg_pnc_values", "jg_pnc_apply_ops", "jg_orset_merge",
                 "jg_orset_contains", "jg_pnc_merge_batch", "jg_orset_union"):
        assert must in names


def test_binding_covers_header():
    assert sorted(jg.EXPORTS) == header_functions()


def test_library_exports_every_symbol():
    lib = ctypes.CDLL(str(jg.LIB_PATH))
    for name in header_functions():
        assert hasattr(lib, name), name
    assert lib.jg_abi_version() == 10  # v10: jg_pnc_apply_ops_encode; v9: jg_pnc_apply_ops_rewind; v8: jg_sha256_batch, jg_update_digests_of; v7: jg_orset_encode_json, jg_orset_apply_ops_ords, jg_pnc_encode_json_before (v6: jg_orset_names_since;
    # v5: jg_apply_stats gains setup_s and loop_s; v4: the RCCL exchange)


def test_library_is_gfx950_only():
    """Every device code object in the offload bundles targets gfx950 (host-side strings of the
    rocPRIM headers may name other architectures; the bundle entries are what loads)."""
    import re
    data = jg.LIB_PATH.read_bytes()
    assert b"__CLANG_OFFLOAD_BUNDLE__" in data
    targets = set(re.findall(rb"amdgcn-amd-amdhsa-[-a-z]*-?(gfx[0-9a-z]+)", data))
    assert targets == {b"gfx950"}, targets


def test_no_device_fails_loudly():
    """Without a GPU, jg_open must return an error code with a message, never fall back."""
    out = subprocess.run(
        ["python", "-c", "import sys; sys.path.insert(0, %r); import janus_gpu as jg\n"
         "try:\n    jg.Context(0)\nexcept jg.JanusError as e:\n    print('ERR', e.code)\nelse:\n    print('OPENED')"
         % str(ROOT / "janus-crdt_amd")],
        capture_output=True, text=True, timeout=120)
    if "OPENED" in out.stdout:
        pytest.skip("a GPU is visible: covered by the gpu tests")
    assert "ERR" in out.stdout, out.stdout + out.stderr


def test_missing_library_raises(tmp_path):
    with pytest.raises(FileNotFoundError):
        jg.load(tmp_path / "nope.so")


def test_integration_binds_every_entry_point():
    # INTEGRATION.md carries the C# [DllImport] declaration a maintainer adds for each ABI function
    text = (ROOT / "INTEGRATION.md").read_text()
    missing = [n for n in header_functions() if f"extern int {n}(" not in text]
    assert not missing, missing
