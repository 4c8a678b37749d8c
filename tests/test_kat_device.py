"""The reference's known-answer tests ON THE DEVICE (janus-crdt_amd/host/kat_device.cpp): every
deterministic scenario of MergeSharp.Tests/PNCounterTests.cs and ORSetTests.cs, each CRDT object a key
of the GPU store, driven through the C ABI by the host mirror (ops -> jg_*_apply_ops, Encode ->
jg_orset_read_sets / jg_pnc_encode_json, ApplySynchronizedUpdate -> the wave path, LookupAll / Contains /
Get -> jg_orset_lookup_all / jg_orset_contains / jg_pnc_values), asserting the reference's literal
values (order-sensitive asserts ORSetTests.cs:113, 144, 327, 343, 346, 473 included) and every shipped
payload byte for byte against the oracle's encoder."""
import subprocess
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

BIN = Path(__file__).resolve().parent.parent / "janus-crdt_amd" / "build" / "kat_device"
SCENARIOS = [
    "PNCounterTests_TestPNCSingle", "PNCounterTests_TestPNCMerge", "PNCounterMsgTests_EncodeDecode",
    "ORSetTests_SingleORSetValueType1", "ORSetTests_SingleORSetReferenceType", "ORSetTests_SingleORSetReferenceType2",
    "ORSetTests_Multiple", "ORSetTests_Multiple2", "ORSetTests_Multiple3", "ORSetTests_Multiple4", "ORSetTests_Multiple5",
    "ORSetTests_Multiple6", "ORSetTests_Same", "ORSetTests_Same2", "ORSetTests_ApplySynchronizedUpdateException",
    "ORSetTests_AddNull", "ORSetTests_RemoveNull", "ORSetTests_RemoveNull2", "ORSetTests_MergeNull", "ORSetTests_MergeNull2",
    "ORSetTests_MergeNull3", "ORSetTests_MergeNull4", "ORSetTests_MergeNull5", "ORSetTests_MergeNull6", "ORSetTests_MergeNull7",
    "ORSetMsgTests_EncodeDecode",
]


def test_reference_known_answers_on_device():
    out = subprocess.run([str(BIN)], capture_output=True, text=True, timeout=110)
    print(out.stdout)
    assert out.returncode == 0, out.stdout + out.stderr
    passed = {line.split()[1] for line in out.stdout.splitlines() if line.startswith("PASS ")}
    missing = [s for s in SCENARIOS if s not in passed]
    assert not missing, missing
