#!/usr/bin/env python3
"""bench.py — replica-key merges/sec + achieved HBM GB/s of the MI355X CRDT merge engine.

Headline (BASELINE.json configs[1], C2): PN-Counter batch merge, 10M keys x 64 replicas, int64 P/N,
local store A and received batch B device-resident (synthetic, seeded).  One step = one
jg_pnc_merge_batch over the whole batch = 640M cell merges (P and N).  The OR-Set batch merge (C3:
1M sets, 100M adds + 20M tombstones per side) runs in the same job and is reported under "orset".

Multi-GPU (`torch.distributed.run --nproc-per-node N`): one process per GPU, the keyspace is
hash-sharded; the data path has no collective, torch.distributed only provides the barrier and the
max-over-ranks of the timings.  At N > 1 the PN-Counter workload is BASELINE configs[3] (C4: 200M keys
x 128 replicas over 8 GPUs): by default every rank merges its own 25M x 128 shard (weak scaling,
--scaling weak); --scaling strong splits a fixed 200M-key keyspace over the N ranks (N >= 4: the
819.2 GB of A and B do not fit fewer MI355X).  The OR-Set leg keeps a C3-shaped shard per rank.

Timing: W untimed warmup steps, then K steps bracketed by barrier + device sync on both sides; the
wall time is max over ranks.  The kernel's own average duration comes from HIP events recorded on
the library's stream around the same K launches (`roofline.achieved`).  rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "janus-crdt_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
SEED = 0x4A414E5553
CPU_REPS = 11  # timed passes of every CPU baseline after 3 warm-ups (median of >= 10)

PNC_KEYS, PNC_R, PNC_EB = 10_000_000, 64, 8
PNC_BYTES_PER_CELL = 6 * PNC_EB  # read A.P A.N B.P B.N, write A.P A.N

ORSET_GROUPS, ORSET_E = 10_000_000, 10          # 1M sets x 10 elems
ORSET_ADD, ORSET_ADD_OV, ORSET_REM, ORSET_REM_OV = 10, 5, 2, 1
REC_BYTES = 28  # OR-Set record in HBM: key 8 B + tag 16 B + arrival ordinal 4 B (jg_tagrec.ord)


def shard_keys(total_keys: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous shard of a hash-partitioned keyspace owned by `rank` (weak scaling: every rank
    owns `total_keys` keys of its own, global key = rank * total_keys + local)."""
    return rank * total_keys, total_keys


def dist_env():
    """(world, rank, device).  JANUS_BENCH_DEVICE pins every rank to one device — only for rehearsing
    the N > 1 path on a one-GPU box (with JANUS_BENCH_BACKEND=gloo); the driver never sets it."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("JANUS_BENCH_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    return world, rank, local


class Sync:
    """Barrier + max-over-ranks; plain no-ops at world size 1.  backend "nccl" (RCCL) on the GPU box;
    "gloo" on CPU (tests/test_dist.py)."""

    def __init__(self, world, local, backend="nccl"):
        self.world = world
        self.dist = None
        if world > 1:
            import torch
            import torch.distributed as dist
            if backend == "nccl":
                torch.cuda.set_device(local)
                self.dev = torch.device("cuda", local)
                dist.init_process_group("nccl", device_id=self.dev)
            else:
                self.dev = torch.device("cpu")
                dist.init_process_group(backend)
            self.dist, self.torch = dist, torch

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def broadcast_bytes(self, b: bytes) -> bytes:
        """Rank 0's bytes on every rank (the RCCL unique id of the library's own communicator)."""
        if not self.dist:
            return b
        obj = [b]
        self.dist.broadcast_object_list(obj, src=0)
        return obj[0]

    def max(self, x: float) -> float:
        if not self.dist:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64, device=self.dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum_int(self, x: int) -> int:
        if not self.dist:
            return x
        t = self.torch.tensor([x], dtype=self.torch.int64, device=self.dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return int(t.item())

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


class HipEvents:
    """hipEvent pair on the library's own stream (the stream the kernels are launched on), via ctypes
    on libamdhip64 — torch.cuda.Event only sees torch's streams."""

    def __init__(self, stream: int):
        import ctypes as C
        import janus_gpu as jg
        self.C = C
        # the HIP runtime libjanusgpu is bound to (dlsym through its handle searches its dependencies):
        # a second libamdhip64 instance in the process would not know the library's stream
        self.hip = jg.load()
        self.stream = C.c_void_p(stream)
        self.e = [C.c_void_p(), C.c_void_p()]
        for e in self.e:
            assert self.hip.hipEventCreate(C.byref(e)) == 0

    def record(self, i: int):
        assert self.hip.hipEventRecord(self.e[i], self.stream) == 0

    def elapsed_s(self) -> float:
        C = self.C
        assert self.hip.hipEventSynchronize(self.e[1]) == 0
        ms = C.c_float()
        assert self.hip.hipEventElapsedTime(C.byref(ms), self.e[0], self.e[1]) == 0
        return ms.value / 1e3

    def close(self):
        for e in self.e:
            self.hip.hipEventDestroy(e)


def timed(ctx, sync, fn, steps, warmup, min_warm_s=0.0, info=None):
    """Run fn() warmup+steps times; returns (max-over-ranks wall seconds, event seconds) of the K steps.
    min_warm_s: after the W warmup steps, more untimed steps until about that much warmup time has passed
    (the same count on every rank: fn may hold a collective).  Short HBM-bound steps keep getting faster
    for tens of milliseconds of sustained traffic (the C3 union: 2.07 -> 1.71 ms per add union over its
    first 5 steps, profiles/r03), so a leg of ~2 ms steps is timed once that ramp is over; info["warmup"]
    receives the count actually run."""
    ev = HipEvents(ctx.stream())
    t_w = time.perf_counter()
    for _ in range(warmup):
        fn()
    ctx.fence()
    done = warmup
    if min_warm_s > 0:
        el = time.perf_counter() - t_w
        per = el / max(warmup, 1)
        extra = 0 if el >= min_warm_s or per <= 0 else min(500, int((min_warm_s - el) / per) + 1)
        extra = int(sync.max(float(extra)))
        for _ in range(extra):
            fn()
        ctx.fence()
        done += extra
    if info is not None:
        info["warmup"] = done
    sync.barrier()
    ctx.fence()
    t0 = time.perf_counter()
    ev.record(0)
    for _ in range(steps):
        fn()
    ev.record(1)
    ctx.fence()
    sync.barrier()
    wall = time.perf_counter() - t0
    ev_s = ev.elapsed_s()
    ev.close()
    return sync.max(wall), sync.max(ev_s)


def cpu_info():
    model = platform.processor() or ""
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return model, os.cpu_count()


def load_traffic(kernel: str):
    """HBM bytes per launch from the committed PMC pass (profiles/pmc_*.json, newest round), if any."""
    best = None
    for p in sorted((ROOT / "profiles").glob("pmc_*.json")):
        try:
            d = json.loads(p.read_text())
        except (OSError, ValueError):
            continue
        if kernel in d:
            best = (d[kernel], p.name)
    return best


def _orset_traffic():
    """PMC HBM bytes of one OR-Set step (both union launches), from the committed profile, if any."""
    a, r = load_traffic("orset_union_add"), load_traffic("orset_union_rem")
    return a[0] + r[0] if a and r else None


# Per-GPU PN-Counter shard: C2 (BASELINE configs[1]) at N = 1; "c4" = one GPU's share of configs[3]
# (200M keys x 128 replicas over 8 GPUs = 25M x 128 per GPU, 102.4 GB resident per GPU), the default
# at N > 1.  Strong scaling splits C4_TOTAL_KEYS over the ranks instead.
PNC_SHAPES = {"c2": (PNC_KEYS, PNC_R), "c4": (25_000_000, 128)}
C4_TOTAL_KEYS = 200_000_000
WORKLOAD_NAMES = {
    "c2": "PNCounter batch merge (BASELINE configs[1]: 10M keys x 64 replicas, int64 P/N)",
    "c4": "PNCounter batch merge (BASELINE configs[3] per-GPU shard: 25M keys x 128 replicas, int64 P/N; 200M keys over 8 GPUs)",
    "c4-strong": "PNCounter batch merge (BASELINE configs[3]: 200M keys x 128 replicas, int64 P/N, split over the GPUs)",
}


def pnc_shard(shape: str, scaling: str, rank: int, world: int) -> tuple[int, int, int]:
    """(first global key, keys on this rank, replicas).  weak: every rank owns a full shard of `shape`;
    strong: the C4 keyspace (200M keys) split into `world` contiguous ranges."""
    if scaling == "strong":
        base, extra = divmod(C4_TOTAL_KEYS, world)
        n = base + (1 if rank < extra else 0)
        return rank * base + min(rank, extra), n, PNC_SHAPES["c4"][1]
    keys, R = PNC_SHAPES[shape]
    key0, n = shard_keys(keys, rank, world)
    return key0, n, R


def bench_pnc(jg, ctx, sync, rank, world, steps, warmup, shape="c2", scaling="weak"):
    key0, n_keys, R = pnc_shard(shape, scaling, rank, world)
    store = jg.PNCStore(ctx, n_keys, R, PNC_EB)
    rows = jg.Rows(ctx, n_keys, R, PNC_EB)
    store.synth(SEED + rank)
    rows.synth(SEED + rank, key0=0)  # per-rank seed: every shard holds its own synthetic keys
    wall, ev = timed(ctx, sync, lambda: store.merge_batch(rows, async_=True), steps, warmup)
    store.close()
    rows.close()
    cells = n_keys * R
    keys_total = sync.sum_int(n_keys)
    return {"wall_s": wall, "event_s": ev, "cells_per_rank": cells, "bytes_per_launch": cells * PNC_BYTES_PER_CELL,
            "keys": n_keys, "keys_total": keys_total, "cells_total": keys_total * R, "R": R}


# untimed warmup of the side legs (OR-Set, exchange, JSON, digests): at least this long
SIDE_WARM_S = float(os.environ.get("JANUS_BENCH_SIDE_WARM_S", "0.1"))
ORSET_STRONG_SHARDS = 8  # strong scaling: the C3 shape x 8 shards (80M (set, elem) groups) split over the ranks


def orset_groups(scaling: str, rank: int, world: int) -> int:
    """(set, elem) groups on this rank.  weak: a full C3 shard per rank (1M sets); strong: C3 x 8 shards
    split into `world` parts ("the same for OR-Set with the C3 shape x 8 shards")."""
    if scaling != "strong":
        return ORSET_GROUPS
    total = ORSET_STRONG_SHARDS * ORSET_GROUPS
    base, extra = divmod(total // ORSET_E, world)  # whole sets per rank
    return (base + (1 if rank < extra else 0)) * ORSET_E


def bench_orset(jg, ctx, sync, rank, world, steps, warmup, scaling="weak"):
    groups = orset_groups(scaling, rank, world)
    L = jg.ORSetStore(ctx, 0, 0)
    R = jg.ORSetStore(ctx, 0, 0)
    na, nr = groups * ORSET_ADD, groups * ORSET_REM
    out = jg.ORSetStore(ctx, 2 * na, 2 * nr)
    L.synth(SEED + rank, groups, ORSET_E, ORSET_ADD, 0, ORSET_REM, 0)
    R.synth(SEED + rank, groups, ORSET_E, ORSET_ADD, ORSET_ADD - ORSET_ADD_OV, ORSET_REM, ORSET_REM - ORSET_REM_OV)
    wi = {}
    wall, ev = timed(ctx, sync, lambda: jg.ORSetStore.union(L, R, out, async_=True), steps, max(warmup, 1), SIDE_WARM_S, wi)
    ua, ur = out.size()
    for h in (L, R, out):
        h.close()
    consumed = 2 * (na + nr)
    return {"wall_s": wall, "event_s": ev, "records_per_rank": consumed, "records_total": sync.sum_int(consumed), "groups": groups, "out": [ua, ur],
            "warmup": wi["warmup"],
            "bytes_per_step": consumed * REC_BYTES + (ua + ur) * REC_BYTES}


EXCH_KEYS, EXCH_ROWS = 2_000_000, 1_000_000  # per rank: owned shard, received batch (global keys)


def bench_exchange(jg, ctx, sync, rank, world, local, steps, warmup):
    """Cross-shard exchange: every rank receives a batch of EXCH_ROWS PN-Counter
    rows whose keys are uniform over the WHOLE keyspace (world x EXCH_KEYS) and makes one
    jg_pnc_exchange on the library's own RCCL communicator (csrc/comm.hip): route on its GPU, counts
    all-gather, grouped ncclSend/ncclRecv of the runs over xGMI, merge of what it owns from device memory.
    At world 1 the runs stay on the device (route + copy + merge)."""
    import numpy as np
    if world > 1 and os.environ.get("JANUS_BENCH_BACKEND", "nccl") != "nccl":
        return bench_exchange_staged(jg, ctx, sync, rank, world, local, steps, warmup)
    uid = sync.broadcast_bytes(jg.comm_unique_id() if rank == 0 else b"")
    comm = jg.Comm(ctx, rank, world, uid)
    store = jg.PNCStore(ctx, EXCH_KEYS, PNC_R, PNC_EB)
    rows = jg.Rows(ctx, EXCH_ROWS, PNC_R, PNC_EB)
    try:
        store.synth(SEED + 7 + rank)
        keys = np.random.default_rng(SEED + rank).integers(0, world * EXCH_KEYS, EXCH_ROWS, dtype=np.uint32)
        zeros = np.zeros((EXCH_ROWS, PNC_R), np.int64)
        rows.upload(zeros, zeros, keys)   # the key indices; values synthesised on the device next
        rows.synth(SEED + 11 + rank)
        last = {}
        wall, _ = timed(ctx, sync, lambda: last.update(comm.exchange_pnc(store, rows)), steps, max(warmup, 1), SIDE_WARM_S)
        st = comm.stats()
        phases = {"route_ms": st.route_s * 1e3, "counts_and_runs_ms": st.exchange_s * 1e3, "merge_ms": st.merge_s * 1e3,
                  "link_bytes_sent": int(st.bytes_sent), "link_bytes_received": int(st.bytes_received)}
        # the owner-side merge alone (jg_pnc_merge_batch with key indices: k_group_link + k_merge_grouped +
        # the list heads reset) on a batch of the same shape with keys in this rank's shard
        lkeys = keys % EXCH_KEYS
        rows.upload(zeros, zeros, lkeys)
        rows.synth(SEED + 11 + rank)
        _, ev_m = timed(ctx, sync, lambda: store.merge_batch(rows, async_=True), steps, max(warmup, 1), SIDE_WARM_S)
    finally:
        store.close()
        rows.close()
        comm.close()
    row_bytes = 4 + 2 * PNC_R * PNC_EB
    distinct = int(np.unique(lkeys).size)
    merge_alg = EXCH_ROWS * row_bytes + distinct * 4 * PNC_R * PNC_EB  # every row read; each distinct key's A row (P, N) read + written once
    merge_s = ev_m / steps
    sent = last["sent"].astype(np.int64)
    remote = int(sent.sum() - sent[rank]) if world > 1 else 0
    return {"workload": f"cross-shard exchange: {EXCH_ROWS} received PN-Counter rows per rank (64 replicas, int64, keys "
                        f"uniform over {world} x {EXCH_KEYS} keys): jg_pnc_exchange = route + RCCL send/recv + merge",
            "rows_per_s": world * EXCH_ROWS / (wall / steps), "ms_per_step": wall / steps * 1e3,
            "xgmi_bytes_per_rank": remote * row_bytes, "row_bytes": row_bytes, "last_step": phases,
            "merge": {"kernels": "k_group_link + k_merge_grouped<8,4>", "ms": merge_s * 1e3,
                      "distinct_keys": distinct,
                      "roofline": {"bound": "hbm", "achieved": merge_alg / merge_s / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                   "frac": merge_alg / merge_s / 1e9 / HBM_PEAK_GBS, "algorithmic_bytes": merge_alg,
                                   "pattern_ceiling": {"GBps": GROUPED_CEILING_GBS, "frac": merge_alg / merge_s / 1e9 / GROUPED_CEILING_GBS,
                                                       "source": "profiles/r03/tune_grouped_ceiling.txt",
                                                       "scope": "the same random 1-KB A-row read-modify-write + B-row read per distinct key "
                                                                "with no lists, no link and no merge arithmetic (tools/tune_grouped.hip k_ceiling)"}}},
            "collective": f"library RCCL communicator (jg_comm), world {world}: ncclAllGather of the counts + grouped ncclSend/ncclRecv"}


def bench_exchange_staged(jg, ctx, sync, rank, world, local, steps, warmup):
    """The exchange rehearsed with several ranks on ONE device over gloo (JANUS_BENCH_BACKEND=gloo; RCCL cannot
    put two ranks on one GPU): the library's own jg_pnc_exchange (csrc/comm.hip: route kernels, the exchange
    plan, the owner's merge) on its host transport (jg_comm_init_host), whose all-to-all-v is gloo's
    all_to_all_single over host memory.  Correctness of the shipped path at world > 1 — the time says nothing
    about xGMI."""
    import numpy as np
    import torch
    import torch.distributed as dist

    def a2a(send, sb, rb):  # the caller's all-to-all-v (gloo over host memory)
        out = torch.empty(sum(rb), dtype=torch.uint8)
        inp = torch.frombuffer(bytearray(send), dtype=torch.uint8) if send else torch.empty(0, dtype=torch.uint8)
        dist.all_to_all_single(out, inp, [int(x) for x in rb], [int(x) for x in sb])
        return out.numpy().tobytes()

    comm = jg.Comm(ctx, rank, world, alltoallv=a2a)
    store = jg.PNCStore(ctx, EXCH_KEYS, PNC_R, PNC_EB)
    rows = jg.Rows(ctx, EXCH_ROWS, PNC_R, PNC_EB)
    try:
        store.synth(SEED + 7 + rank)
        keys = np.random.default_rng(SEED + rank).integers(0, world * EXCH_KEYS, EXCH_ROWS, dtype=np.uint32)
        zeros = np.zeros((EXCH_ROWS, PNC_R), np.int64)
        rows.upload(zeros, zeros, keys)
        rows.synth(SEED + 11 + rank)
        last = {}
        wall, _ = timed(ctx, sync, lambda: last.update(comm.exchange_pnc(store, rows)), steps, warmup)
        st = comm.stats()
    finally:
        store.close()
        rows.close()
        comm.close()
    return {"workload": f"cross-shard exchange rehearsal: {world} ranks on one device, the library's exchange on its host transport (gloo)",
            "rows_per_s": world * EXCH_ROWS / (wall / steps), "ms_per_step": wall / steps * 1e3,
            "records_received_last_step": int(st.records_received), "received_per_source": [int(x) for x in last["received"]],
            "collective": "jg_comm_init_host: the caller's all-to-all-v = torch.distributed all_to_all_single over gloo (rehearsal, not xGMI)"}


JSON_MSGS, JSON_KEYS, JSON_R, JSON_EB, JSON_NODES = 1_000_000, 1_000_000, 5, 4, 4  # one C5 wave, device-resident


def json_wave(seed, n=JSON_MSGS, n_keys=JSON_KEYS):
    """C5-shaped PNCounterMsg states (compact System.Text.Json form): message m is the state of key keys[m]
    as one of JSON_NODES nodes knows it, naming 1..JSON_NODES replicas of that key with int32 values.
    Replica Guids per key come from 4096 pools (Guids need only be distinct within a key's row)."""
    import numpy as np
    sys.path.insert(0, str(ROOT / "tests"))
    from jsongen import encode_pnc, random_guids
    rng = np.random.default_rng(seed)
    T, V = 4096, 8
    pools = [random_guids(rng, JSON_NODES) for _ in range(T)]
    var = [[encode_pnc(pools[t][: 1 + (v % JSON_NODES)], list(rng.integers(0, 2**31 - 1, JSON_NODES)),
                       list(rng.integers(0, 2**31 - 1, JSON_NODES))) for v in range(V)] for t in range(T)]
    keys = rng.integers(0, n_keys, n).astype(np.uint32)
    pick = rng.integers(0, V, n)
    msgs = [var[k % T][v] for k, v in zip(keys.tolist(), pick.tolist())]
    lens = np.fromiter((len(x) for x in msgs), np.uint64, n)
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum(lens)
    data = np.frombuffer(b"".join(msgs), np.uint8)
    entries = int(sum(2 * (1 + (v % JSON_NODES)) for v in pick.tolist()))
    return keys, data, off, entries


def bench_json(jg, ctx, sync, rank, steps, warmup):
    """The committed-wave apply from wire bytes (json.hip: k_scan + k_resolve + k_apply) on one C5 wave
    resident in HBM (jg_wave_upload once, jg_pnc_merge_wave per step): steady state (every replica known:
    scan + apply) and a cold wave (every message names replicas its row has not seen: scan + sort +
    resolve + apply).  Algorithmic bytes per message: its payload, offset (8 B) and row index (4 B), per
    entry one int32 cell read + written."""
    keys, data, off, entries = json_wave(SEED + 53 + rank)
    w = jg.Wave(ctx, JSON_MSGS, data.size)
    warm = jg.PNCStore(ctx, JSON_KEYS, JSON_R, JSON_EB)
    try:
        w.upload(keys, data=data, off=off)
        wall, ev = timed(ctx, sync, lambda: warm.merge_wave(w), steps, max(warmup, 1), SIDE_WARM_S)
        cold_ms = []
        for _ in range(2):
            cold = jg.PNCStore(ctx, JSON_KEYS, JSON_R, JSON_EB)
            t0 = time.perf_counter()
            cold.merge_wave(w)
            cold_ms.append((time.perf_counter() - t0) * 1e3)
            cold.close()
    finally:
        warm.close()
        w.close()
    alg = data.size + 12 * JSON_MSGS + 2 * JSON_EB * entries
    kern = ev / steps
    # the parse is instruction-bound, not HBM-bound: VALU wave instructions per wave (PMC SQ_INSTS_VALU of
    # k_scan + k_apply_emit, profiles/pmc_*.json) against the chip's issue rate (one wave instruction per
    # SIMD every 2 cycles: 256 CUs x 4 SIMDs x 0.5 x 2.4 GHz)
    # (with pass A fused, the default, the steady-state wave launches no k_apply_emit: its share is then 0)
    sv, av = load_traffic("json_scan_valu"), load_traffic("json_apply_emit_valu")
    valu = None
    if sv:
        insts, peak = sv[0] + (av[0] if av else 0), VALU_LANE_OPS / 64
        valu = {"bound": "valu", "achieved": insts / kern / 1e12, "peak": peak / 1e12, "unit": "T wave-instructions/s",
                "frac": insts / kern / peak, "valu_insts_per_wave": insts, "source": sv[1],
                "scope": "k_scan (+ k_apply_emit, which a steady-state wave does not launch) VALU instructions over the jg_pnc_merge_wave event time"}
    return {"workload": f"PNCounterMsg wave from wire bytes (C5 shape: {JSON_MSGS} states of {JSON_KEYS} accounts, "
                        f"{JSON_R - 1}-node replicas, int32), resident in HBM, steady state (replicas known)",
            "msgs_per_s": JSON_MSGS / (wall / steps), "ms_per_wave": wall / steps * 1e3, "event_ms": kern * 1e3,
            "payload_bytes": int(data.size), "engine_payload_GBps": data.size / kern / 1e9,
            "cold_wave_ms": min(cold_ms), "json_group": int(os.environ.get("JANUS_JSON_GROUP", "8")),
            "roofline": {"bound": "hbm", "achieved": alg / kern / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": alg / kern / 1e9 / HBM_PEAK_GBS, "algorithmic_bytes_per_wave": alg,
                         "scope": "jg_pnc_merge_wave (k_scan + k_apply, status reads) per step"},
            "roofline_valu": valu}


PCIE_PEAK_GBS = 63.0  # PCIe Gen5 x16 host link, per direction (MI355X_MICROARCH.md)
# One hipMemcpyAsync of 48-MB chunks from page-locked memory, measured on the box: 56.0-56.5 GB/s; split over
# two copy queues, SDMA off (blit kernels) or pulled by a kernel it is no faster (profiles/r03/tune_h2d.txt).
PCIE_MEASURED_GBS = 56.5
# The grouped merge's access pattern alone (random 1-KB A-row read-modify-write + one B-row read per distinct
# key, 787k of 2M keys): 2.42 GB in 0.466 ms on the box (profiles/r03/tune_grouped_ceiling.txt).
GROUPED_CEILING_GBS = 5190.0


def apply_roofline(res):
    """Roofline of an apply-loop leg.  The committed wave's payloads live in host memory (the reference's
    byte[] messages), so every byte the library uploads (payload + per-message uid / identity / type /
    offset) must cross the host link once: the wave is bounded by PCIe, and `frac` is that link's share.
    Beside it: the device share (uploaded bytes / kernel time of the wave, against HBM) and the host
    share (the library's gather into page-locked staging)."""
    if "error" in res or not res.get("uploaded_bytes_per_wave"):
        return None
    up = float(res["uploaded_bytes_per_wave"])
    wave_s = res["ms_per_wave"] / 1e3
    busy_s = res["device_busy_ms_per_wave"] / 1e3
    gather_s = res["gather_ms_per_wave"] / 1e3
    ach = up / wave_s / 1e9
    out = {"bound": "pcie", "achieved": ach, "peak": PCIE_PEAK_GBS, "unit": "GB/s", "frac": ach / PCIE_PEAK_GBS, "traffic": None,
            "bytes_per_wave": up, "ideal_ms_per_wave": up / PCIE_PEAK_GBS / 1e6,
            "measured_link": {"GBps": PCIE_MEASURED_GBS, "frac": ach / PCIE_MEASURED_GBS, "ideal_ms_per_wave": up / PCIE_MEASURED_GBS / 1e6,
                              "source": "profiles/r03/tune_h2d.txt (one hipMemcpyAsync per 48-MB chunk from page-locked memory)"},
            "scope": "bytes the library uploads per wave (payloads + per-message arrays) / wave time",
            "device_share": {"bound": "hbm", "achieved": up / busy_s / 1e9 if busy_s else None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": up / busy_s / 1e9 / HBM_PEAK_GBS if busy_s else None, "busy_ms_per_wave": busy_s * 1e3,
                             "scope": "uploaded bytes / kernel time of the wave (hipEvents around each chunk's kernels and the final phase)"},
            "host_share": {"gather_ms_per_wave": gather_s * 1e3, "gather_GBps": up / gather_s / 1e9 if gather_s else None,
                           "scope": "the library's workers gathering payloads into page-locked staging (overlaps the uploads)"}}
    chunk_s = res.get("chunk_busy_ms_per_wave", 0) / 1e3
    if chunk_s:  # the per-chunk kernels: classify + the payload decode (k_scan / k_ow_group + the OR-Set tables)
        out["decode"] = {"bound": "hbm", "achieved": up / chunk_s / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": up / chunk_s / 1e9 / HBM_PEAK_GBS, "busy_ms_per_wave": chunk_s * 1e3,
                         "scope": "uploaded bytes / kernel time of the per-chunk classify + parse kernels (hipEvents, chunk_busy_s)"}
    return out


def orset_decode_counters():
    """The bound of the OR-Set apply loop's device work, named by its PMC counters: the per-kernel summary of
    bench_orset --direct in the newest profiles/pmc_*.json (janus-crdt_amd/tools/pmc_summary.py: HBM bytes,
    VALU issue share, the share of wave cycles parked on memory, L2 hit rate and atomics per wave).  The
    dominant kernel's bound is the loop's: hbm (>= 50 % of 8 TB/s), valu (>= 50 % of the issue rate), or
    latency (waves parked on memory with neither near its peak)."""
    best = None
    for p in sorted((ROOT / "profiles").glob("pmc_*.json")):
        try:
            d = json.loads(p.read_text())
        except (OSError, ValueError):
            continue
        if "orset_wire" in d:
            best = (d["orset_wire"]["kernels"], p.name)
    if not best:
        return None
    ks = best[0]
    timed_ks = sorted(((k, v) for k, v in ks.items() if v.get("us_per_wave")), key=lambda kv: -kv[1]["us_per_wave"])
    if not timed_ks:
        return None
    top, tv = timed_ks[0]
    keep = ("us_per_wave", "bound", "hbm_GBps", "valu_issue_frac", "wait_mem_frac", "tcc_hit_rate", "tcc_atomics_per_wave")
    return {"bound": tv["bound"], "dominant_kernel": top, "kernels_us_per_wave": sum(v["us_per_wave"] for _, v in timed_ks),
            "kernels": {k: {f: v.get(f) for f in keep} for k, v in timed_ks[:8]}, "source": best[1],
            "scope": "bench_orset --direct per-chunk parse + tables + commit kernels, counters per wave"}


def name_decode_bound(roof):
    """The OR-Set loop's device work is not an HBM stream (random table probes and tag-record inserts): its
    bound comes from the committed counters (orset_decode_counters), and the decode object says so."""
    dc = orset_decode_counters()
    roof["decode_counters"] = dc
    if dc and isinstance(roof.get("decode"), dict):
        roof["decode"]["bound"] = dc["bound"]
        roof["decode"]["bound_from"] = f"PMC counters of the dominant kernel {dc['dominant_kernel']} ({dc['source']})"
        roof["decode"]["frac_note"] = "frac is the uploaded bytes over the decode time against HBM peak, kept for comparison only"


def bench_apply_loop(sync, rank, world, local):
    """C5 committed-batch apply (the banking replay, BankingWorload.cs ops through the
    node batchers, 1M client ops per committed wave) through the C++ host mirror, on every rank.  Every
    rank applies the same committed waves to the accounts it owns (GpuStableStore::ShardOf; other
    uids are skipped like the reference skips unknown uids), so the wave is split N ways with no
    collective: strong scaling over a fixed 1M-account keyspace.  msgs_per_s = wave messages / the
    slowest rank's wave time."""
    import subprocess
    exe = ROOT / "janus-crdt_amd" / "build" / "bench_apply"
    cpu_msgs = "100000" if world == 1 else "0"
    out = subprocess.run([str(exe), "--accounts", "1000000", "--ops", "1000000", "--waves", "3", "--cpu-msgs", cpu_msgs,
                          "--device", str(local), "--rank", str(rank), "--world", str(world)],
                         capture_output=True, text=True, timeout=240)
    ok = out.returncode == 0
    res = json.loads(out.stdout.strip().splitlines()[-1]) if ok else {"error": out.stderr[-500:]}
    worst_ms = sync.max(res["ms_per_wave"] if ok else float("inf"))
    if world > 1 and ok:
        res = {"workload": res["workload"] + f", key-space sharded x{world}", "scaling": "strong",
               "msgs_per_s": res["state_msgs_per_wave"] / (worst_ms / 1e3), "client_ops_per_s": 1_000_000 / (worst_ms / 1e3),
               "ms_per_wave": worst_ms, "rank0_roofline": apply_roofline(res),
               "rank0": {k: res.get(k) for k in ("ms_per_wave", "host_ms_per_wave", "device_busy_ms_per_wave", "device_wait_ms_per_wave",
                                                   "owned_accounts", "applied_msgs_per_wave")}}
    return res


def run_direct(exe_name, args, local, mode="--direct"):
    """One apply-loop bench binary with --direct (the wave laid out in page-locked memory, uploaded in place) or
    --arena (bench_apply: the caller's own copy of the wave into a jg_host_alloc arena, timed)."""
    import subprocess
    mode = [mode] if isinstance(mode, str) else list(mode)
    out = subprocess.run([str(ROOT / "janus-crdt_amd" / "build" / exe_name)] + args + ["--device", str(local)] + mode,
                         capture_output=True, text=True, timeout=240)
    if out.returncode != 0 or not out.stdout.strip():
        return {"error": out.stderr[-500:]}
    res = json.loads(out.stdout.strip().splitlines()[-1])
    res["roofline"] = apply_roofline(res)
    if exe_name == "bench_orset" and res["roofline"]:
        name_decode_bound(res["roofline"])
    return {k: res.get(k) for k in ("ms_per_wave", "msgs_per_s", "caller_flatten_ms_per_wave", "library_ms_per_wave", "setup_ms_per_wave",
                                    "loop_ms_per_wave", "device_wait_ms_per_wave", "device_busy_ms_per_wave", "uploaded_bytes_per_wave",
                                    "roofline")}


def bench_apply_direct(local):
    """The C5 wave of bench_apply_loop as a transport that receives its blocks into page-locked memory
    (jg_host_alloc) would hand it over: the payloads back to back there, laid out outside the timed region
    (that copy is the receive path's), then the same jg_apply_committed, which uploads them in place (the
    library's `direct` path, no gather).  One GPU only: the shard shortcut gathers (it drops other shards'
    states on the host)."""
    import subprocess
    exe = ROOT / "janus-crdt_amd" / "build" / "bench_apply"
    out = subprocess.run([str(exe), "--accounts", "1000000", "--ops", "1000000", "--waves", "3", "--cpu-msgs", "0",
                          "--device", str(local), "--direct"], capture_output=True, text=True, timeout=240)
    if out.returncode != 0:
        return {"error": out.stderr[-500:]}
    res = json.loads(out.stdout.strip().splitlines()[-1])
    res.pop("cpu_baseline", None)  # not run here (--cpu-msgs 0): the gathered leg "apply_loop" carries it
    return res


def bench_apply_orset(sync, rank, world, local):
    """The committed-batch apply loop for OR-Set states (ORSetWorkload-shaped, host/bench_orset.cpp):
    2000 sets, 4 nodes, 200k full-state ORSetMsg payloads per wave, through jg_apply_committed (the payloads
    decoded, element strings interned and the states merged on the device), vs the oracle's decode +
    ORSet.Merge loop."""
    import subprocess
    exe = ROOT / "janus-crdt_amd" / "build" / "bench_orset"
    out = subprocess.run([str(exe), "--sets", "2000", "--msgs", "200000", "--waves", "3", "--cpu-msgs", "20000" if world == 1 else "0",
                          "--device", str(local), "--rank", str(rank), "--world", str(world)],
                         capture_output=True, text=True, timeout=240)
    ok = out.returncode == 0
    res = json.loads(out.stdout.strip().splitlines()[-1]) if ok else {"error": out.stderr[-500:]}
    worst_ms = sync.max(res["ms_per_wave"] if ok else float("inf"))
    if world > 1 and ok:
        res = {"workload": res["workload"] + f", key-space sharded x{world}", "scaling": "strong",
               "msgs_per_s": 200_000 / (worst_ms / 1e3), "ms_per_wave": worst_ms, "rank0_ms_per_wave": res["ms_per_wave"],
               "rank0_roofline": apply_roofline(res)}
    return res


def bench_c1(local):
    """BASELINE configs[0] (C1): the reference's own PN-Counter benchmark shape (benchmark_config_example.json:
    100 objects, opsRatio [0.25, 0.25, 0.5], safeRatio 0.5, 4 servers) as committed waves of 1M client
    ops through the host mirror, the oracle's apply loop timed on the same waves, every key's stable value
    checked against it (host/bench_c1.cpp).  Single process: C1 is the reference's CPU-runnable case."""
    import subprocess
    exe = ROOT / "janus-crdt_amd" / "build" / "bench_c1"
    out = subprocess.run([str(exe), "--device", str(local)], capture_output=True, text=True, timeout=240)
    return json.loads(out.stdout.strip().splitlines()[-1]) if out.stdout.strip() else {"error": out.stderr[-500:]}


def bench_submit(local, workload):
    """The producer path of one node (host/bench_submit.cpp): SafeCRDT.Update
    over a call of client ops (C5 banking ops on 1M accounts, or ORSetWorkload ops on 2000 sets), every shipped
    snapshot encoded on the device, ActualPropagateSyncMsg's batches and their digests — against the oracle's
    SafeCRDT.Update + ActualPropagateSyncMsg + update_digest on a sample, whose batches must equal the GPU's byte for
    byte (parity).  Roofline: the host link — every snapshot byte comes back to the host once and goes out again
    for its UpdateMessage's digest."""
    import subprocess
    args = (["--workload", "pnc", "--keys", "1000000", "--ops", "1000000", "--cpu-ops", "50000", "--waves", "5"] if workload == "pnc" else
            ["--workload", "orset", "--keys", "2000", "--ops", "200000", "--cpu-ops", "20000", "--waves", "5"])
    out = subprocess.run([str(ROOT / "janus-crdt_amd" / "build" / "bench_submit")] + args + ["--device", str(local)],
                         capture_output=True, text=True, timeout=240)
    if not out.stdout.strip():
        return {"error": out.stderr[-500:]}
    res = json.loads(out.stdout.strip().splitlines()[-1])
    if out.returncode != 0:
        res["error"] = f"parity failure: {res.get('parity_failure')}"
        return res
    link = 2.0 * res["submitted_msgs_per_wave"] * res["payload_bytes_per_msg"]
    ach = link / (res["ms_per_wave"] / 1e3) / 1e9
    res["roofline"] = {"bound": "pcie", "achieved": ach, "peak": PCIE_PEAK_GBS, "unit": "GB/s", "frac": ach / PCIE_PEAK_GBS, "traffic": None,
                       "measured_link": {"GBps": PCIE_MEASURED_GBS, "frac": ach / PCIE_MEASURED_GBS},
                       "scope": "snapshot bytes down (encode) + up again (digests) per call / call time"}
    return res


DIGEST_MSGS, DIGEST_PER_UPDATE = 1_000_000, 1000  # one C5-sized wave, clientBatchSize-sized UpdateMessages
DIGEST_PIPE = 8  # waves per pipelined call
# VALU instructions per 64-byte block of the k_sha_msgs loop (compress + window shift, gfx950 ISA count of
# csrc/digest.hip) and the chip's VALU issue rate if every one issued in 2 cycles: 256 CUs x 4
# SIMDs x 32 lanes/clk x 2.4 GHz.  They do not: v_alignbit_b32 (576 per block) and v_add3_u32 (~240) take
# ~4.3 cycles per wave64 instruction, v_bitop3_b32 ~2.5 (tools/valu_rate.hip).  The digest roofline's peak
# is therefore the MEASURED issue ceiling of the same compression code on register-resident blocks at the
# kernel's occupancy: 27.8-28.0 Gblocks/s (profiles/r04/valu_rate.txt; 4 and 5 waves per SIMD agree).
SHA_VALU_PER_BLOCK, VALU_LANE_OPS = 1693, 256 * 4 * 32 * 2.4e9
SHA_CEILING_BLOCKS_PER_S = 27.9e9


def digest_wave(n, seed):
    """n PNCounterMsg-sized payloads (340..375 bytes, ~357 B like the C5 wave's JSON states), back to back."""
    import numpy as np
    rng = np.random.default_rng(seed)
    lens = rng.integers(340, 376, n).astype(np.uint64)
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum(lens)
    data = rng.integers(32, 127, int(off[-1]), dtype=np.uint8)
    return data, off


def bench_digest(jg, ctx, sync, rank, steps, warmup):
    """UpdateMessage.ComputeDigest for one wave resident in HBM: 1M payloads in 1000
    UpdateMessages of 1000 (jg_wave_update_digests: k_sha_msgs + k_sha_updates + 32 KB of digests D2H)."""
    import numpy as np
    data, off = digest_wave(DIGEST_MSGS, SEED + 31 + rank)
    first = np.arange(0, DIGEST_MSGS + 1, DIGEST_PER_UPDATE, dtype=np.uint64)
    data2, off2 = digest_wave(DIGEST_MSGS, SEED + 97 + rank)  # a second, distinct resident wave (pipelined leg)
    w = jg.Wave(ctx, DIGEST_MSGS, data.size)
    w2 = jg.Wave(ctx, DIGEST_MSGS, data2.size)
    try:
        w.upload(np.zeros(DIGEST_MSGS, np.uint32), data=data, off=off)
        w2.upload(np.zeros(DIGEST_MSGS, np.uint32), data=data2, off=off2)
        wall, ev = timed(ctx, sync, lambda: w.update_digests(first), steps, max(warmup, 1), SIDE_WARM_S)
        # the first level alone (k_sha_msgs, digest bytes into device memory: jg_wave_sha256)
        import torch
        dout = torch.empty(DIGEST_MSGS * 32, dtype=torch.uint8, device=torch.device("cuda", ctx.device))
        wall1, ev1 = timed(ctx, sync, lambda: w.sha256_device(dout.data_ptr(), async_=True), steps, max(warmup, 1), SIDE_WARM_S)
        del dout
        # pipelined: DIGEST_PIPE waves in one jg_waves_update_digests call (wave k's chains on the
        # context's second stream beside wave k+1's first level); two distinct resident waves alternate, so
        # wave k+1's first level does not re-read the bytes wave k just streamed through the caches
        pipe = [w, w2] * (DIGEST_PIPE // 2)
        wall_p, ev_p = timed(ctx, sync, lambda: jg.waves_update_digests(pipe, [first] * DIGEST_PIPE), steps, max(warmup, 1), SIDE_WARM_S)
    finally:
        w.close()
        w2.close()
    blocks = int(((off[1:] - off[:-1] + 72) // 64).sum())
    kern, kern1 = ev / steps, ev1 / steps
    chain = int((32 * DIGEST_PER_UPDATE + 72) // 64) if DIGEST_PER_UPDATE <= 32768 else None
    return {"workload": f"UpdateMessage.ComputeDigest: {DIGEST_MSGS} payloads of 340-375 B resident in HBM, "
                        f"{DIGEST_MSGS // DIGEST_PER_UPDATE} UpdateMessages of {DIGEST_PER_UPDATE}",
            "msgs_per_s": DIGEST_MSGS / (wall / steps), "ms_per_wave": wall / steps * 1e3,
            "payload_GBps": data.size / (wall / steps) / 1e9, "event_ms": kern * 1e3, "sha_blocks": blocks,
            "first_level": {"kernel": "k_sha_msgs", "msgs_per_s": DIGEST_MSGS / (wall1 / steps), "event_ms": kern1 * 1e3,
                            "payload_GBps": data.size / kern1 / 1e9},
            "second_level_chain_blocks": chain,
            "pipelined": {"api": "jg_waves_update_digests", "waves_per_call": DIGEST_PIPE,
                          "msgs_per_s": DIGEST_MSGS * DIGEST_PIPE / (wall_p / steps),
                          "ms_per_wave": wall_p / steps / DIGEST_PIPE * 1e3},
            "roofline": {"bound": "valu", "achieved": blocks / kern1 / 1e9, "unit": "Gblocks/s",
                         "peak": SHA_CEILING_BLOCKS_PER_S / 1e9,
                         "frac": blocks / kern1 / SHA_CEILING_BLOCKS_PER_S,
                         "peak_source": "measured issue ceiling of csrc/sha256_device.hpp's compression, no memory traffic "
                                        "(tools/valu_rate.hip, profiles/r04/valu_rate.txt)",
                         "frac_of_2cycle_issue": blocks / kern1 / (VALU_LANE_OPS / SHA_VALU_PER_BLOCK),
                         "scope": "first level (k_sha_msgs, jg_wave_sha256); the full call adds the second level, a "
                                  "serial chain of second_level_chain_blocks SHA-256 blocks per UpdateMessage "
                                  "(one wave's issue latency, DESIGN.md section 4)"}}


def cpu_digest_baseline():
    """The oracle's scalar SHA-256 (port) and hashlib / OpenSSL (the primitive .NET 6's SHA256.HashData calls
    on Linux) over the first 50k payloads of the same wave, 1 thread."""
    import hashlib
    import numpy as np
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_ref as orc
    n = 50_000
    data, off = digest_wave(n, SEED + 31)
    first = np.arange(0, n + 1, DIGEST_PER_UPDATE, dtype=np.uint64)
    t = orc.lib().orc_bench_update_digests(n, off.ctypes.data, data.ctypes.data, first.size - 1, first.ctypes.data, CPU_REPS)
    buf = data.tobytes()
    t0 = time.perf_counter()
    for u in range(first.size - 1):
        toSign = bytearray(32768)
        for j, i in enumerate(range(int(first[u]), int(first[u + 1]))):
            toSign[32 * j:32 * j + 32] = hashlib.sha256(buf[off[i]:off[i + 1]]).digest()
        hashlib.sha256(toSign).digest()
    t_ssl = time.perf_counter() - t0
    return {"msgs_per_s": n / t, "cores": 1, "kind": "port",
            "sample": f"oracle UpdateMessage.ComputeDigest (scalar FIPS 180-4 restatement) over the first {n} payloads, 3 warm-ups, median of {CPU_REPS}",
            "openssl": {"msgs_per_s": n / t_ssl, "cores": 1,
                        "sample": "the same with Python hashlib (OpenSSL SHA-256, SHA extensions where the CPU has them)"}}


def cpu_baseline():
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_ref as orc
    n_keys, reps = 100_000, CPU_REPS
    t = orc.bench_pnc_merge(n_keys, PNC_R, SEED, 1, reps)
    model, ncpu = cpu_info()
    n_sets = 20_000
    t_or = orc.bench_orset_merge(n_sets, ORSET_E, ORSET_ADD, ORSET_ADD_OV, ORSET_REM, ORSET_REM_OV, SEED, 1, CPU_REPS)
    # the same merge split over the host cores this job may use; the box
    # grants 16 CPUs per GPU, os.cpu_count() shows the whole machine
    par = max(1, min(16, ncpu or 1))
    t_par = orc.bench_pnc_merge(4 * n_keys, PNC_R, SEED, par, reps)
    return {
        "value": n_keys * PNC_R / t,
        "unit": "replica-key merges/s",
        "cores": 1,
        "kind": "port",
        "sample": f"PNCounter.Merge over pre-decoded messages, first {n_keys} keys x {PNC_R} replicas of the C2 "
                  f"synthetic workload, int64, dictionary-faithful oracle (oracle/), 3 warm-ups, median of {reps}, 1 thread "
                  f"(the reference's serialized apply task); host: {model}, {ncpu} logical CPUs",
        "orset_records_per_s": n_sets * ORSET_E * 2 * (ORSET_ADD + ORSET_REM) / t_or,
        "parallel": {"value": 4 * n_keys * PNC_R / t_par, "cores": par,
                     "sample": f"the same merge over the first {4 * n_keys} keys, keys split over {par} threads"},
    }


def headline(args, world, res, cpu):
    """The line's headline fields: the C2 PN-Counter step (metric, value, roofline) and the C3 OR-Set step."""
    line = {"metric": "replica-key merges/sec + achieved HBM GB/s (PNCounter & ORSet)", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "higher_is_better": True, "scaling": args.scaling,
            "vs_baseline": None, "data": "synthetic (seeded counter-based generators, DESIGN.md)"}
    if "pnc" in res:
        p = res["pnc"]
        step = p["wall_s"] / args.steps
        kern = p["event_s"] / args.steps
        achieved = p["bytes_per_launch"] / kern / 1e9
        traffic = load_traffic("pnc_merge_dense") if args.pnc_shape == "c2" else None  # PMC pass exists for C2 only
        total_cells = p["cells_total"]
        line.update({
            "value": total_cells / step,
            "unit": "replica-key merges/s",
            "ms_per_step": step * 1e3,
            "dtype": "int64",
            "config": {"workload": WORKLOAD_NAMES["c4-strong" if args.scaling == "strong" else args.pnc_shape],
                       "keys_per_gpu": p["keys"], "total_keys": p["keys_total"], "replicas": p["R"], "elem_bytes": PNC_EB,
                       "parallelism": f"keyspace-sharded x{world}, no data-path collective"},
            "hbm_GBps": total_cells * PNC_BYTES_PER_CELL / step / 1e9,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic[0] if traffic else None,
                         "kernel": "k_merge_dense<8>", "algorithmic_bytes_per_launch": p["bytes_per_launch"],
                         "kernel_ms": kern * 1e3, "traffic_source": traffic[1] if traffic else None},
        })
    if "orset" in res:
        o = res["orset"]
        ost = o["wall_s"] / max(1, args.steps // 2)
        line["orset"] = {
            "workload": ("ORSet batch merge (BASELINE configs[2]: 1M sets, 100M adds + 20M tombstones per side)" if args.scaling != "strong" else
                         f"ORSet batch merge (BASELINE configs[2] shape x {ORSET_STRONG_SHARDS} shards: {ORSET_STRONG_SHARDS}M sets, "
                         f"{ORSET_STRONG_SHARDS * 100}M adds + {ORSET_STRONG_SHARDS * 20}M tombstones per side, split over {world} GPUs)"),
            "scaling": args.scaling, "groups_per_rank": o["groups"],
            "value": o["records_total"] / ost, "unit": "tag records merged/s",
            "ms_per_step": ost * 1e3, "out_records": o["out"], "steps": max(1, args.steps // 2), "warmup": o["warmup"],
            "hbm_GBps": world * o["bytes_per_step"] / ost / 1e9,
            "roofline": {"bound": "hbm", "achieved": o["bytes_per_step"] / (o["event_s"] / max(1, args.steps // 2)) / 1e9,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": o["bytes_per_step"] / (o["event_s"] / max(1, args.steps // 2)) / 1e9 / HBM_PEAK_GBS,
                         "traffic": _orset_traffic(),
                         "frac_24B": o["bytes_per_step"] * 24 / 28 / (o["event_s"] / max(1, args.steps // 2)) / 1e9 / HBM_PEAK_GBS,
                         "scope": "whole step: both streams' boundaries (k_partition_gallop2), the add and tombstone unions (k_union), "
                                  "both finishes (k_finish2); 28-B records (key, tag, "
                                  "arrival ordinal); frac_24B = the same time in SURVEY.md D3's 24-B unit (DESIGN.md section 5)"},
        }
        if "value" not in line:
            line.update({"value": line["orset"]["value"], "unit": "tag records merged/s", "ms_per_step": ost * 1e3,
                         "dtype": "u64+u128 records", "config": {"workload": line["orset"]["workload"]}})
    line["cpu_baseline"] = cpu
    return line


LINE_CAP = 8000  # bytes: the driver keeps an 8-KB stdout tail and parses the last line


def _r(x, nd=4):
    """Round a float to nd significant digits for the compact line (ints and None unchanged)."""
    if isinstance(x, float):
        return float(f"{x:.{nd}g}")
    return x


def _roof(r, keys=("bound", "frac", "achieved", "unit")):
    if not isinstance(r, dict):
        return None
    return {k: _r(r.get(k)) for k in keys if r.get(k) is not None}


def compact_leg(name, leg):
    """One leg reduced to its figures: time per step/wave, throughput, the roofline's bound and frac (full leg on
    stderr).  Apply-loop legs also carry their CPU baseline's rate and the page-locked / caller-arena variants."""
    if not isinstance(leg, dict):
        return None
    if "error" in leg:
        return {"error": str(leg["error"])[:200]}
    out = {}
    for k in ("ms_per_step", "ms_per_wave", "value", "unit", "msgs_per_s", "ops_per_s", "rows_per_s", "client_ops_per_s", "event_ms",
              "cold_wave_ms", "untimed_pack_ms_per_wave", "csharp_caller_ms_per_wave", "ms_per_wave_median", "scaling"):
        if leg.get(k) is not None:
            out[k] = _r(leg[k])
    roof = leg.get("roofline")
    if roof is None and isinstance(leg.get("rank0_roofline"), dict):
        roof = leg["rank0_roofline"]
    if isinstance(roof, dict):
        out["roofline"] = _roof(roof, ("bound", "frac", "achieved", "peak", "unit", "traffic", "frac_24B"))
        ml = roof.get("measured_link")
        if isinstance(ml, dict):
            out["roofline"]["frac_of_measured_link"] = _r(ml.get("frac"))
        dec = roof.get("decode")
        if isinstance(dec, dict):
            out["decode_bound"] = dec.get("bound")
    if isinstance(leg.get("roofline_valu"), dict):
        out["roofline_valu"] = _roof(leg["roofline_valu"])
    cb = leg.get("cpu_baseline")
    if isinstance(cb, dict):
        out["cpu_baseline"] = {k: _r(cb.get(k)) for k in ("msgs_per_s", "ops_per_s", "cores", "kind") if cb.get(k) is not None}
    if "parity_vs_oracle" in leg:
        out["parity_vs_oracle"] = leg["parity_vs_oracle"]
    for sub in ("from_pinned", "caller_arena", "caller_arena_streamed", "pipelined", "first_level", "merge"):
        s = leg.get(sub)
        if isinstance(s, dict):
            c = {k: _r(s[k]) for k in ("ms_per_wave", "ms", "event_ms", "msgs_per_s", "caller_flatten_ms_per_wave") if s.get(k) is not None}
            if isinstance(s.get("roofline"), dict):
                c["frac"] = _r(s["roofline"].get("frac"))
                ml = s["roofline"].get("measured_link")
                if isinstance(ml, dict):
                    c["frac_of_measured_link"] = _r(ml.get("frac"))
            out[sub] = c
    return out


def compact_line(line, legs):
    """The driver-parsed stdout line: the headline (metric, value, roofline with traffic, cpu_baseline) in full and
    one compact object per leg.  Legs are dropped from the end if the line would exceed LINE_CAP."""
    out = dict(line)
    cb = out.get("cpu_baseline")
    if isinstance(cb, dict):
        out["cpu_baseline"] = {k: _r(v) if not isinstance(v, dict) else {kk: _r(vv) for kk, vv in v.items()} for k, v in cb.items()}
    for k in ("value", "ms_per_step", "hbm_GBps"):
        if k in out:
            out[k] = _r(out[k], 7)
    if isinstance(out.get("roofline"), dict):
        out["roofline"] = {k: _r(v, 6) for k, v in out["roofline"].items()}
    out["legs"] = {k: compact_leg(k, v) for k, v in legs.items()}
    out["detail"] = "stderr (full legs, one JSON line)"
    while len(json.dumps(out)) > LINE_CAP and out["legs"]:
        out["legs"].pop(next(reversed(out["legs"])))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=["all", "pnc", "orset", "pnc-orset", "exchange", "digest", "json", "producer"], default="all")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pnc-shape", choices=["auto"] + sorted(PNC_SHAPES), default="auto",
                    help="per-GPU PN-Counter shard: c2 = BASELINE configs[1], c4 = 1/8 of configs[3]; "
                         "auto (default) = c2 on one GPU, c4 on N > 1")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak",
                    help="weak: a fixed shard per GPU; strong: configs[3]'s 200M keys split over N >= 4 GPUs")
    args = ap.parse_args()

    world, rank, local = dist_env()
    if args.pnc_shape == "auto":
        args.pnc_shape = "c2" if world == 1 and args.scaling == "weak" else "c4"
    if args.scaling == "strong" and world < 4:
        sys.exit("--scaling strong needs N >= 4: configs[3]'s 200M keys x 128 replicas (A + B = 819.2 GB) do not fit fewer MI355X")
    if world != args.gpus and world > 1:
        print(f"warning: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
    if world > 1 or args.workload in ("all", "exchange", "digest", "json"):
        # torch (device buffers + RCCL) is loaded before libjanusgpu so both bind ONE HIP runtime
        # instance (torch's libraries also name the runtime by an unversioned soname)
        import torch  # noqa: F401
    sync = Sync(world, local, os.environ.get("JANUS_BENCH_BACKEND", "nccl"))
    import janus_gpu as jg
    ctx = jg.Context(local)

    res = {}
    if args.workload in ("all", "pnc", "pnc-orset"):
        res["pnc"] = bench_pnc(jg, ctx, sync, rank, world, args.steps, args.warmup, args.pnc_shape, args.scaling)
    if args.workload in ("all", "orset", "pnc-orset"):
        res["orset"] = bench_orset(jg, ctx, sync, rank, world, max(1, args.steps // 2), args.warmup, args.scaling)
    if world > 1 and rank == 0 and args.workload in ("all", "exchange") and ("pnc" in res or "orset" in res):
        # the headline (PN-Counter + OR-Set) before the first world > 1 collective of the library's own
        # communicator: whatever the exchange leg does, a line is out; the full line follows at the end
        print(json.dumps(headline(args, world, res, None)), flush=True)
    if args.workload in ("all", "exchange"):
        try:  # a failure here must not cost the headline line
            res["exchange"] = bench_exchange(jg, ctx, sync, rank, world, local, max(1, args.steps // 4), min(args.warmup, 2))
        except Exception as e:  # noqa: BLE001
            res["exchange"] = {"error": repr(e)[:500]}
    if args.workload in ("all", "json"):
        try:
            res["json"] = bench_json(jg, ctx, sync, rank, max(1, args.steps // 2), min(args.warmup, 2))
        except Exception as e:  # noqa: BLE001
            res["json"] = {"error": repr(e)[:500]}
    if args.workload in ("all", "digest"):
        try:
            res["digest"] = bench_digest(jg, ctx, sync, rank, max(1, args.steps // 2), min(args.warmup, 2))
            if rank == 0 and world == 1 and not args.no_cpu_baseline:
                res["digest"]["cpu_baseline"] = cpu_digest_baseline()
        except Exception as e:  # noqa: BLE001
            res["digest"] = {"error": repr(e)[:500]}
    ctx.close()

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline()
    def guarded(fn, *a):  # a leg's failure must not cost the headline line (each leg's collective runs on every
        try:              # rank before anything in it can raise: sync.max takes inf for a failed run)
            return fn(*a)
        except Exception as e:  # noqa: BLE001
            return {"error": repr(e)[:500]}

    apply_loop = guarded(bench_apply_loop, sync, rank, world, local) if args.workload == "all" else None
    apply_orset = guarded(bench_apply_orset, sync, rank, world, local) if args.workload == "all" else None
    apply_c1 = guarded(bench_c1, local) if args.workload == "all" and world == 1 else None
    apply_direct = guarded(bench_apply_direct, local) if args.workload == "all" and world == 1 else None
    producer_pnc = guarded(bench_submit, local, "pnc") if args.workload in ("all", "producer") and world == 1 else None
    producer_orset = guarded(bench_submit, local, "orset") if args.workload in ("all", "producer") and world == 1 else None
    for leg in (apply_loop, apply_orset, apply_c1, apply_direct):
        if leg is not None and "error" not in leg and "scaling" not in leg:
            leg["roofline"] = guarded(apply_roofline, leg)
    if apply_orset is not None and isinstance(apply_orset.get("roofline"), dict):
        guarded(name_decode_bound, apply_orset["roofline"])
    # the same OR-Set and C1 waves from page-locked payloads (one GPU: the shard shortcut gathers)
    if apply_orset is not None and "error" not in apply_orset and world == 1:
        apply_orset["from_pinned"] = guarded(run_direct, "bench_orset", ["--sets", "2000", "--msgs", "200000", "--waves", "3", "--cpu-msgs", "0"], local)
    if apply_c1 is not None and "error" not in apply_c1:
        apply_c1["from_pinned"] = guarded(run_direct, "bench_c1", ["--waves", "3", "--no-cpu"], local)
    # what a C# caller without page-locked receive buffers pays: its own parallel copy of every
    # committed byte[] into a jg_host_alloc arena (plain cached copies, Span.CopyTo), then the in-place upload
    if apply_direct is not None and "error" not in apply_direct:
        apply_direct["caller_arena"] = guarded(run_direct, "bench_apply", ["--accounts", "1000000", "--ops", "1000000", "--waves", "3",
                                                                           "--cpu-msgs", "0"], local, "--arena")
        # the same copy in parts through jg_apply_stream_begin/append/end: part k + 1's copy overlaps part k's upload
        apply_direct["caller_arena_streamed"] = guarded(run_direct, "bench_apply", ["--accounts", "1000000", "--ops", "1000000", "--waves", "3",
                                                                                    "--cpu-msgs", "0"], local, "--arena-stream")
        # the A13 figure a C# caller with pageable byte[]s gets: the streamed arena, whatever the
        # one-shot one measured beside it (the two are within box noise of each other)
        cs = apply_direct.get("caller_arena_streamed")
        if isinstance(cs, dict) and cs.get("ms_per_wave") is not None:
            apply_direct["csharp_caller_ms_per_wave"] = cs["ms_per_wave"]
    sync.close()
    if rank != 0:
        return

    line = headline(args, world, res, cpu)
    legs = {"orset": line.pop("orset", None), "apply_loop": apply_loop, "apply_loop_orset": apply_orset,
            "apply_loop_c1": apply_c1, "apply_loop_direct": apply_direct, "update_digests": res.get("digest"),
            "json_apply": res.get("json"), "exchange": res.get("exchange"), "producer_pnc": producer_pnc, "producer_orset": producer_orset}
    legs = {k: v for k, v in legs.items() if v is not None}
    # every leg in full (per-kernel dicts, nested rooflines, PMC summaries) on stderr and, if asked, in a file;
    # the LAST stdout line is the compact one the driver parses (<= LINE_CAP bytes)
    detail = dict(line, legs=legs)
    print(json.dumps(detail), file=sys.stderr, flush=True)
    if os.environ.get("JANUS_BENCH_DETAIL"):
        Path(os.environ["JANUS_BENCH_DETAIL"]).write_text(json.dumps(detail) + "\n")
    print(json.dumps(compact_line(line, legs)), flush=True)


if __name__ == "__main__":
    main()
