"""CPU unit test of the host mirror's safe-update tracker (janus-crdt_amd/host/tracker.cpp: the
SafeCRDTManager.safeUpdateTracker map, SafeCRDTManager.cs:33) — ring, overflow table, growth, copies and
concurrent takes against std::unordered_map (janus-crdt_amd/host/test_tracker.cpp).  Plain C++: no GPU."""
import subprocess
from pathlib import Path

PKG = Path(__file__).resolve().parent.parent / "janus-crdt_amd"


def test_safe_update_tracker():
    exe = PKG / "build" / "test_tracker"
    if not exe.exists():  # g++ only (the tracker has no engine calls)
        subprocess.run(["make", "-C", str(PKG), "build/test_tracker"], check=True, capture_output=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "tracker: all passed" in out.stdout
