"""CPU test of bench.py's driver-parsed line (a 24-KB line left BENCH_r04.json unparsed).  The
canned input is round 4's full bench line (profiles/r04/bench_final_untraced.json): its headline plus every leg
in full, as main() hands them to compact_line.  No GPU."""
import importlib.util
import json
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
REQUIRED = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "dtype", "config", "roofline",
            "cpu_baseline", "higher_is_better", "scaling", "vs_baseline", "data")
LEGS = ("orset", "apply_loop", "apply_loop_orset", "apply_loop_c1", "apply_loop_direct", "update_digests", "json_apply", "exchange")
PRODUCER = {"workload": "producer path ...", "waves": 3, "ops_per_s": 2.5e6, "ms_per_wave": 400.0, "submitted_msgs_per_wave": 999874.0,
            "payload_bytes_per_msg": 366.7, "parity_vs_oracle": True, "roofline": {"bound": "pcie", "achieved": 1.8, "peak": 63.0, "unit": "GB/s",
            "frac": 0.03, "traffic": None, "measured_link": {"GBps": 56.5, "frac": 0.032}}, "cpu_baseline": {"ops_per_s": 256780.9, "cores": 1, "kind": "port"}}


def _bench():
    spec = importlib.util.spec_from_file_location("bench", ROOT / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _canned():
    full = json.loads((ROOT / "profiles" / "r04" / "bench_final_untraced.json").read_text().strip().splitlines()[-1])
    legs = {k: full.pop(k) for k in LEGS if k in full}
    return full, legs


def test_compact_line_fits_and_holds_the_headline():
    b = _bench()
    line, legs = _canned()
    assert len(json.dumps(dict(line, **legs))) > 20_000  # the round-4 shape that broke the parser
    out = b.compact_line(line, legs)
    s = json.dumps(out)
    assert len(s) <= b.LINE_CAP
    assert "\n" not in s
    for k in REQUIRED:
        assert k in out, k
    assert out["config"]["workload"].startswith("PNCounter batch merge (BASELINE configs[1]")
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in out["roofline"], k
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in out["cpu_baseline"], k
    # every leg kept, each with a time and a roofline fraction
    assert set(out["legs"]) == set(LEGS)
    legs = dict(legs, producer_pnc=PRODUCER, producer_orset=PRODUCER)  # round 5's producer-path legs fit too
    out = b.compact_line(line, legs)
    assert len(json.dumps(out)) <= b.LINE_CAP and set(out["legs"]) == set(LEGS) | {"producer_pnc", "producer_orset"}
    assert out["legs"]["producer_pnc"]["ops_per_s"] == 2.5e6 and out["legs"]["producer_pnc"]["parity_vs_oracle"] is True
    for k, leg in out["legs"].items():
        assert "ms_per_step" in leg or "ms_per_wave" in leg, k
    assert out["legs"]["orset"]["roofline"]["bound"] == "hbm"
    assert 0 < out["legs"]["orset"]["roofline"]["frac"] < 1
    assert out["legs"]["apply_loop_direct"]["caller_arena"]["ms_per_wave"] > 0
    assert out["legs"]["apply_loop_orset"]["from_pinned"]["ms_per_wave"] > 0
    # the headline numbers survive rounding to 7 significant digits
    assert abs(out["value"] - line["value"]) / line["value"] < 1e-6


def test_compact_line_drops_legs_past_the_cap():
    b = _bench()
    line, legs = _canned()
    legs = dict(legs)
    for i in range(200):
        legs[f"pad{i}"] = {"ms_per_step": 1.0, "roofline": {"bound": "hbm", "frac": 0.5}}
    out = b.compact_line(line, legs)
    assert len(json.dumps(out)) <= b.LINE_CAP
    assert "orset" in out["legs"]  # legs go from the end


def test_compact_leg_error():
    b = _bench()
    assert b.compact_leg("x", {"error": "E" * 900}) == {"error": "E" * 200}
