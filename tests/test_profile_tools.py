"""CPU tests of the profiling pipeline's arithmetic: pmc_summary's per-kernel OR-Set loop summary (the bound each
kernel's counters name) and bench.py's decode-bound naming from a committed summary.  Synthetic rocprofv3 CSVs,
no GPU."""
import csv
import importlib.util
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _counters(path, rows):
    path.mkdir(parents=True, exist_ok=True)
    with open(path / "run_counter_collection.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for k, c, v in rows:
            w.writerow({"Kernel_Name": k, "Counter_Name": c, "Counter_Value": v})


def _trace(path, rows):
    path.mkdir(parents=True, exist_ok=True)
    with open(path / "run_kernel_trace.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        t = 0
        for k, ns in rows:
            w.writerow({"Kernel_Name": k, "Start_Timestamp": t, "End_Timestamp": t + ns})
            t += ns + 100


def _fake_orset_profile(d: Path):
    W = 5  # the summary divides by bench_orset's 5 waves
    kernels = {  # name: (ns per wave, FETCH_SIZE KB, WRITE_SIZE KB, VALU, WAIT_ANY, WAVE_CYCLES)
        "void k_ow_strings(Sparse)": (500_000, 3_000_000, 100_000, 1e6, 90, 100),   # 6.4 GB/s... per wave: ~6.3 TB/s random lines
        "void k_ow_group(uint8_t const*)": (400_000, 100_000, 10_000, 3.5e8, 30, 100),  # VALU issue > 50 %
        "void k_cb_count(Sparse)": (60_000, 20_000, 1_000, 1e5, 80, 100),              # parked on memory
    }
    tr, fe, wr, sq = [], [], [], []
    for k, (ns, fkb, wkb, valu, wait, wc) in kernels.items():
        tr += [(k, ns)] * W
        fe.append((k, "FETCH_SIZE", fkb * W))
        wr.append((k, "WRITE_SIZE", wkb * W))
        for c, v in (("SQ_INSTS_VALU", valu * W), ("SQ_WAIT_ANY", wait), ("SQ_WAVE_CYCLES", wc), ("SQ_INSTS_SALU", 1), ("SQ_INSTS_LDS", 1),
                     ("SQ_INSTS_VMEM", 1), ("SQ_WAIT_INST_ANY", 1), ("SQ_BUSY_CYCLES", 1)):
            sq.append((k, c, v))
    _trace(d / "trace_orset_loop", tr)
    _counters(d / "pmc_orset_loop_FETCH_SIZE", fe)
    _counters(d / "pmc_orset_loop_WRITE_SIZE", wr)
    _counters(d / "sq_orset_loop", sq)
    _counters(d / "sq2_orset_loop", [(k, c, 1) for k in kernels for c in ("SQ_ACTIVE_INST_ANY", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_WAIT_INST_LDS")])
    _counters(d / "tcc_orset_loop", [(k, c, 10) for k in kernels for c in ("TCC_ATOMIC_sum", "TCC_HIT_sum", "TCC_MISS_sum", "TCC_EA0_RDREQ_sum")])


def test_orset_loop_summary_names_each_kernels_bound(tmp_path):
    ps = _load("pmc_summary", ROOT / "janus-crdt_amd" / "tools" / "pmc_summary.py")
    _fake_orset_profile(tmp_path)
    out = ps.orset_loop(tmp_path)
    assert set(out) == {"k_ow_strings", "k_ow_group", "k_cb_count"}
    s = out["k_ow_strings"]
    assert abs(s["us_per_wave"] - 500.0) < 1e-6
    # random-line reading: FETCH once + WRITE, per wave, over the kernel's time
    assert abs(s["hbm_GBps_random_lines"] - (3_100_000 * 1024) / 500_000) < 1e-6
    assert abs(s["hbm_GBps"] - (6_100_000 * 1024) / 500_000) < 1e-6
    assert s["bound"] == "hbm"
    assert out["k_ow_group"]["bound"] == "valu"
    assert out["k_cb_count"]["bound"] == "latency"
    assert abs(out["k_cb_count"]["wait_mem_frac"] - 0.8) < 1e-9


def test_bench_names_the_decode_bound_from_the_newest_summary(tmp_path, monkeypatch):
    sys.path.insert(0, str(ROOT))
    import bench
    prof = tmp_path / "profiles"
    prof.mkdir()
    k = {"us_per_wave": 500.0, "bound": "latency", "hbm_GBps": 1.0, "valu_issue_frac": 0.1, "wait_mem_frac": 0.9, "tcc_hit_rate": 0.2,
         "tcc_atomics_per_wave": 5.0}
    (prof / "pmc_r03.json").write_text(json.dumps({"orset_wire": {"kernels": {"k_old": dict(k, bound="hbm")}}}))
    (prof / "pmc_r04.json").write_text(json.dumps({"orset_wire": {"kernels": {"k_ow_strings": k, "k_small": dict(k, us_per_wave=5.0, bound="valu")}}}))
    monkeypatch.setattr(bench, "ROOT", tmp_path)
    roof = {"bound": "pcie", "decode": {"bound": "hbm", "frac": 0.02}}
    bench.name_decode_bound(roof)
    dc = roof["decode_counters"]
    assert dc["dominant_kernel"] == "k_ow_strings" and dc["source"] == "pmc_r04.json"
    assert roof["decode"]["bound"] == "latency" and "k_ow_strings" in roof["decode"]["bound_from"]
    assert abs(dc["kernels_us_per_wave"] - 505.0) < 1e-9
    # no summary: the decode object keeps its own bound, and says nothing about counters
    monkeypatch.setattr(bench, "ROOT", tmp_path / "none")
    roof2 = {"decode": {"bound": "hbm"}}
    bench.name_decode_bound(roof2)
    assert roof2["decode_counters"] is None and roof2["decode"]["bound"] == "hbm"


def test_json_scan_split_separates_steady_and_cold_waves(tmp_path):
    """The json leg's profile holds steady waves (the scan alone: pass A applies the cells) and cold ones (the scan,
    then k_resolve_rows and k_apply_emit); pmc_summary reports the scan's bytes of the steady ones, in dispatch order
    whatever the CSV's row order."""
    ps = _load("pmc_summary", ROOT / "janus-crdt_amd" / "tools" / "pmc_summary.py")
    seq = [("k_reset_status", 0), ("void k_scan<4, 8>(x)", 300), ("k_scan_slow<4>", 0), ("void k_resolve_rows<4>(x)", 240),
           ("void k_apply_emit<4>(x)", 66),
           ("k_reset_status", 0), ("void k_scan<4, 8>(x)", 400), ("k_scan_slow<4>", 0),
           ("k_reset_status", 0), ("void k_scan<4, 8>(x)", 410), ("rocprim::detail::sort", 3),
           ("void k_scan<4, 8>(x)", 290), ("void k_apply_emit<4>(x)", 66)]
    path = tmp_path / "run_counter_collection.csv"
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for i, (k, v) in reversed(list(enumerate(seq))):  # rows out of dispatch order
            w.writerow({"Dispatch_Id": i + 1, "Kernel_Name": k, "Counter_Name": "FETCH_SIZE", "Counter_Value": v})
    out = ps.json_scan_split(path, "FETCH_SIZE")
    assert out["steady"] == [400 * 1024, 410 * 1024]
    assert out["cold"] == [300 * 1024, 290 * 1024]
