"""Summarise a gpu_profile.sh run into profiles/pmc_<round>.json (HBM bytes, instructions and stalls per launch).

gfx950 correction (MI355X_MICROARCH.md, HBM / rocprofv3 section): bytes = 2 * FETCH_SIZE * 1024 +
WRITE_SIZE * 1024 — FETCH_SIZE counts half of a wide coalesced read stream.  FETCH_SIZE and
WRITE_SIZE come from separate --pmc passes of the same command.  OR-Set unions alternate
add-stream / tombstone-stream launches (jg_orset_union), so launches are split by parity.

The OR-Set apply loop (bench_orset --direct, 5 waves of which 2 warm-up) gets a per-kernel breakdown per WAVE
(every launch of the run / 5): HBM bytes (the streaming correction: an upper bound for these random probes,
with TCC_EA0_RDREQ beside it), VALU / SALU / LDS instructions, the share of wave cycles parked on memory
(SQ_WAIT_ANY) and on issue (SQ_WAIT_INST_ANY), LDS bank-conflict cycles, L2 hit rate and atomics — and the bound
each kernel's counters name.

usage: python pmc_summary.py <profile dir> <out json> [<round label>]
"""
import collections
import csv
import json
import re
import statistics
import sys
from pathlib import Path

# bench.py "exchange" at N = 1: 1M rows with keys uniform over 2M -> expected distinct keys
_EXCH_DISTINCT = round(2_000_000 * (1 - (1 - 1 / 2_000_000) ** 1_000_000))
ALGO = {  # algorithmic bytes per launch of the bench.py workloads
    "pnc_merge_dense": 10_000_000 * 64 * 8 * 2 * 3,           # P and N: read local + received, write local
    "orset_union_add": (100_000_000 * 2 + 150_000_000) * 28,  # read both sides, write the union (28 B records)
    "orset_union_rem": (20_000_000 * 2 + 30_000_000) * 28,
    # bench.py "exchange": 1M rows x (4 B key + 2 x 64 x 8 B) per rank
    "exchange_route_scatter": 1_000_000 * 1028 * 2,                 # read every row, write it to its run
    # read every row; read + write each distinct key's A row once (the list head folds its key's rows)
    "exchange_merge_grouped": 1_000_000 * 1028 + _EXCH_DISTINCT * 2 * 1024,
}
ORSET_LOOP_WAVES = 5  # bench_orset --waves 3 + its 2 warm-up waves
# gfx950: 256 CUs x 4 SIMDs, one VALU wave instruction per SIMD every 2 cycles at 2.4 GHz (as bench.py)
VALU_WAVE_INSTS_PER_S = 256 * 4 * 0.5 * 2.4e9


def short(name):
    m = re.search(r"(k_\w+)(<[^>]*>)?", name)
    if m:
        return m.group(0)
    if "rocprim" in name:
        kind = next((k for k in ("merge", "radix", "partition", "transform", "lookback", "scan") if k in name), "other")
        return "rocprim:" + kind
    return name[:40]


def per_kernel(path, counter, key=lambda n: n):
    out = collections.defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == counter:
                out[key(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return out


def json_scan_split(path, counter):
    """k_scan<4, 8> counter values (bytes) of the steady-state waves and of the cold ones, by dispatch order: a cold
    wave's scan is followed by k_resolve_rows / k_apply_emit before the next scan."""
    with open(path) as f:
        rows = sorted((r for r in csv.DictReader(f) if r["Counter_Name"] == counter), key=lambda r: int(r["Dispatch_Id"]))
    out, cur = {"steady": [], "cold": []}, None
    for r in rows + [None]:
        n = r["Kernel_Name"] if r else "k_scan<4, 8>"
        if "k_scan<4, 8>" in n:
            if cur is not None:
                out["cold" if cur[1] else "steady"].append(cur[0])
            cur = [float(r["Counter_Value"]) * 1024, False] if r else None
        elif cur is not None and ("k_resolve_rows" in n or "k_apply_emit" in n):
            cur[1] = True
    return out


def durations(trace_dir):
    """Kernel durations (ns) per short name from a --kernel-trace run."""
    out = collections.defaultdict(list)
    p = trace_dir / "run_kernel_trace.csv"
    if not p.exists():
        return out
    with open(p) as f:
        for r in csv.DictReader(f):
            out[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return out


def orset_loop(d: Path):
    """Per-kernel counters of the OR-Set apply loop, per wave."""
    src = {"fetch": ("pmc_orset_loop_FETCH_SIZE", ["FETCH_SIZE"]), "write": ("pmc_orset_loop_WRITE_SIZE", ["WRITE_SIZE"]),
           "sq": ("sq_orset_loop", ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                    "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES"]),
           "sq2": ("sq2_orset_loop", ["SQ_ACTIVE_INST_ANY", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_WAIT_INST_LDS"]),
           "tcc": ("tcc_orset_loop", ["TCC_ATOMIC_sum", "TCC_HIT_sum", "TCC_MISS_sum", "TCC_EA0_RDREQ_sum"])}
    tot = collections.defaultdict(dict)
    for _, (sub, ctrs) in src.items():
        p = d / sub / "run_counter_collection.csv"
        if not p.exists():
            return None
        for c in ctrs:
            for k, v in per_kernel(p, c, short).items():
                tot[k][c] = sum(v) / ORSET_LOOP_WAVES
    dur = durations(d / "trace_orset_loop")
    out = {}
    for k, c in tot.items():
        if not (k.startswith("k_ow_") or k.startswith("k_cb_") or k.startswith("k_union") or k in ("k_classify", "k_unstage", "k_partition_gallop2<3072>")):
            continue
        ns = sum(dur.get(k, [])) / ORSET_LOOP_WAVES if dur.get(k) else None
        wc = c.get("SQ_WAVE_CYCLES") or 0
        # FETCH_SIZE counts half of a wide streaming read (the 2x correction) but a random 64-byte line fetch
        # once: these kernels probe tables at random, so the bytes lie between the two readings
        hbm = 2 * 1024 * c.get("FETCH_SIZE", 0) + 1024 * c.get("WRITE_SIZE", 0)
        hbm_rand = 1024 * c.get("FETCH_SIZE", 0) + 1024 * c.get("WRITE_SIZE", 0)
        hit, miss = c.get("TCC_HIT_sum", 0), c.get("TCC_MISS_sum", 0)
        e = {"us_per_wave": ns / 1e3 if ns else None,
             "hbm_bytes_per_wave": hbm, "hbm_bytes_per_wave_random_lines": hbm_rand, "tcc_ea_rdreq_per_wave": c.get("TCC_EA0_RDREQ_sum"),
             "hbm_GBps": hbm / ns if ns else None, "hbm_GBps_random_lines": hbm_rand / ns if ns else None,
             "valu_insts_per_wave": c.get("SQ_INSTS_VALU"), "salu_insts_per_wave": c.get("SQ_INSTS_SALU"),
             "lds_insts_per_wave": c.get("SQ_INSTS_LDS"), "vmem_insts_per_wave": c.get("SQ_INSTS_VMEM"),
             "valu_issue_frac": (c.get("SQ_INSTS_VALU", 0) / (ns * 1e-9) / VALU_WAVE_INSTS_PER_S) if ns else None,
             "wait_mem_frac": c.get("SQ_WAIT_ANY", 0) / wc if wc else None,
             "wait_issue_frac": c.get("SQ_WAIT_INST_ANY", 0) / wc if wc else None,
             "active_frac": c.get("SQ_ACTIVE_INST_ANY", 0) / wc if wc else None,
             "lds_conflict_frac": c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"] if c.get("SQ_LDS_IDX_ACTIVE") else None,
             "tcc_hit_rate": hit / (hit + miss) if hit + miss else None, "tcc_atomics_per_wave": c.get("TCC_ATOMIC_sum")}
        # the bound the counters name: the HBM share of peak (on the random-line reading: a random probe fetches
        # its line once), the VALU issue share, or waves parked on memory with neither near its peak (latency:
        # dependent random probes / atomics, the request rate of scattered lines)
        hf = (e["hbm_GBps_random_lines"] or 0) / 8000.0
        vf = e["valu_issue_frac"] or 0
        wm = e["wait_mem_frac"] or 0
        e["bound"] = "hbm" if hf >= 0.5 else "valu" if vf >= 0.5 else "latency" if wm >= 0.5 else "mixed"
        out[k] = e
    return out


def main():
    d, dst = Path(sys.argv[1]), Path(sys.argv[2])
    label = sys.argv[3] if len(sys.argv) > 3 else dst.stem
    fetch = per_kernel(d / "pmc_FETCH_SIZE" / "run_counter_collection.csv", "FETCH_SIZE")
    write = per_kernel(d / "pmc_WRITE_SIZE" / "run_counter_collection.csv", "WRITE_SIZE")
    for extra in ("exch", "json"):
        if (d / f"pmc_{extra}_FETCH_SIZE").exists():
            fetch.update(per_kernel(d / f"pmc_{extra}_FETCH_SIZE" / "run_counter_collection.csv", "FETCH_SIZE"))
            write.update(per_kernel(d / f"pmc_{extra}_WRITE_SIZE" / "run_counter_collection.csv", "WRITE_SIZE"))

    def pick(prefix, parity=None):
        names = [k for k in fetch if prefix in k and "k_scan_slow" not in k]
        if not names:
            return None
        f, w = fetch[names[0]], write.get(names[0], [])
        if parity is not None:
            f, w = f[parity::2], w[parity::2]
        return statistics.median(2 * x * 1024 for x in f) + statistics.median(x * 1024 for x in w)

    res = {"_doc": f"HBM bytes per launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), {label}, MI355X. "
                   "gfx950 correction per MI355X_MICROARCH.md HBM section: bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024. "
                   "Generated by janus-crdt_amd/tools/pmc_summary.py from janus-crdt_amd/tools/gpu_profile.sh output "
                   "(traces, counter passes and the bench line of one gpurun lease)."}
    for key, prefix, parity in [("pnc_merge_dense", "k_merge_dense<8>", None), ("orset_union_add", "k_union<", 0),
                                ("orset_union_rem", "k_union<", 1), ("orset_partition_both", "k_partition_gallop2<", None),
                                ("orset_finish_both", "k_finish2", None), ("exchange_route_scatter", "k_route_scatter<", None),
                                ("exchange_merge_grouped", "k_merge_grouped<8", None), ("exchange_group_link", "k_group_link", None),
                                ("json_scan", "k_scan<4, 8>", None), ("json_apply_emit", "k_apply_emit<4>", None)]:
        v = pick(prefix, parity)
        if v is not None:
            res[key] = v
            if key in ALGO:
                res[key + "_algorithmic"] = ALGO[key]
    # the json leg's steady-state waves (every replica known: pass A applies the cells itself, nothing follows it)
    # apart from its cold ones (first sight of the replicas: k_resolve_rows + k_apply_emit follow the scan)
    if (d / "pmc_json_FETCH_SIZE").exists():
        js = {}
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            js[c] = json_scan_split(d / f"pmc_json_{c}" / "run_counter_collection.csv", c)
        if js["FETCH_SIZE"]["steady"] and js["WRITE_SIZE"]["steady"]:
            f, w = statistics.median(js["FETCH_SIZE"]["steady"]), statistics.median(js["WRITE_SIZE"]["steady"])
            res["json_scan"] = 2 * f + w
            res["json_scan_steady"] = {"fetch_size_bytes": f, "write_size_bytes": w, "streaming_reading": 2 * f + w,
                                       "random_line_reading": f + w, "launches": [len(js["FETCH_SIZE"]["steady"]), len(js["WRITE_SIZE"]["steady"])]}
        if js["FETCH_SIZE"]["cold"] and js["WRITE_SIZE"]["cold"]:
            res["json_scan_cold"] = 2 * statistics.median(js["FETCH_SIZE"]["cold"]) + statistics.median(js["WRITE_SIZE"]["cold"])
            res["json_apply_emit_cold"] = res.pop("json_apply_emit", None)
    # VALU instructions per launch of the json leg's group kernels (SQ_INSTS_VALU, one wave instruction = 64
    # lanes), for the bench's instruction-issue roofline of jg_pnc_merge_wave, with the stall shares beside them
    sq = d / "sq_json" / "run_counter_collection.csv"
    if sq.exists():
        # (the scan's steady-state launches only, as the bytes above; k_apply_emit runs in cold waves alone)
        def counter(path, c, prefix):
            if prefix.startswith("k_scan<"):
                v = json_scan_split(path, c)["steady"]
                return statistics.median(v) / 1024 if v else None
            vals = per_kernel(path, c)
            names = [k for k in vals if prefix in k]
            return statistics.median(vals[names[0]]) if names else None

        for key, prefix in [("json_scan", "k_scan<4, 8>"), ("json_apply_emit_cold", "k_apply_emit<4>")]:
            cs = {}
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES"):
                v = counter(sq, c, prefix)
                if v is not None:
                    cs[c] = v
            sq2 = d / "sq2_json" / "run_counter_collection.csv"
            if sq2.exists():
                for c in ("SQ_ACTIVE_INST_ANY", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE"):
                    v = counter(sq2, c, prefix)
                    if v is not None:
                        cs[c] = v
            if "SQ_INSTS_VALU" in cs:
                res[key + "_valu"] = cs["SQ_INSTS_VALU"]
                wc = cs.get("SQ_WAVE_CYCLES")
                res[key + "_sq"] = {"salu": cs.get("SQ_INSTS_SALU"), "lds": cs.get("SQ_INSTS_LDS"),
                                    "wait_mem_frac": cs["SQ_WAIT_ANY"] / wc if wc and "SQ_WAIT_ANY" in cs else None,
                                    "wait_issue_frac": cs["SQ_WAIT_INST_ANY"] / wc if wc and "SQ_WAIT_INST_ANY" in cs else None,
                                    "active_frac": cs["SQ_ACTIVE_INST_ANY"] / wc if wc and "SQ_ACTIVE_INST_ANY" in cs else None,
                                    "lds_conflict_frac": cs["SQ_LDS_BANK_CONFLICT"] / cs["SQ_LDS_IDX_ACTIVE"]
                                    if cs.get("SQ_LDS_IDX_ACTIVE") else None}
    ol = orset_loop(d)
    if ol:
        res["orset_wire"] = {"_doc": "bench_orset --direct (ORSetWorkload-shaped waves of 200k states, 245 MB), per WAVE: every launch of the "
                                     "5-wave run / 5.  hbm_bytes: the streaming correction (2 x FETCH_SIZE + WRITE_SIZE), an upper bound for "
                                     "random probes, beside the random-line reading (1 x FETCH_SIZE + WRITE_SIZE); bound: hbm if the "
                                     "random-line rate is >= 50 % of 8 TB/s, valu if >= 50 % of the VALU issue rate, latency if "
                                     "waves sit parked on memory (SQ_WAIT_ANY) >= 50 % of their cycles with neither near its peak.",
                             "kernels": ol}
    dst.write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
