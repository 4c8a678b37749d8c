"""Cross-shard exchange of received CRDT state between the GPUs of one node.

The keyspace is sharded: global key k (PN-Counter row / OR-Set set id) belongs to rank k % world,
where it is local key k // world (csrc/route.hip).  A received batch that lands on a rank that does
not own all of its keys is

  1. routed on its GPU: jg_rows_route / jg_orset_route, a stable partition by owner with the keys
     rewritten to the owner's local ids, into device buffers;
  2. exchanged: one all-to-all of the per-destination counts, then one all-to-all per buffer —
     torch.distributed over RCCL (backend "nccl"), i.e. xGMI peer links between the MI355X GPUs;
  3. merged by the owner straight from the receive buffers: jg_pnc_merge_device /
     jg_orset_merge_device (PNCounter.Merge / ORSet.Merge, MergeSharp/MergeSharp/CRDTs/PNCounters.cs:131-144,
     ORSet.cs:253-283).

torch is plumbing here (device buffers + the collective); every byte is produced and consumed by the
HIP library.  With a non-RCCL group (gloo: several ranks sharing one device in a test) the buffers are
staged through host memory around the same all-to-all.  world = 1 (no group) skips step 2.
"""
from __future__ import annotations

import numpy as np

import janus_gpu as jg


def all_to_all_plan(counts, rank: int, skip_own: bool = False):
    """The layout all_to_all_single gives the runs (what Exchange.runs moves): counts[src, dst, j] records
    source src routes to destination dst in buffer j.  Returns (send_off, send_n, recv_off, recv_n), each
    [world, k]: this rank's send buffer j holds every destination's run in rank order, its receive buffer j
    the sources' runs back to back in rank order.  skip_own: the own run stays out of both (a PN-Counter
    rank merges it from its send buffer).  csrc/comm.hip's jg_exchange_plan must equal this."""
    c = np.asarray(counts, np.uint64)
    world, k = c.shape[0], c.shape[2]
    send_off = np.zeros((world, k), np.uint64)
    send_off[1:] = np.cumsum(c[rank, :-1, :], axis=0)
    send_n = c[rank].copy()
    recv_n = c[:, rank, :].copy()
    if skip_own:
        send_n[rank] = 0
        recv_n[rank] = 0
    recv_off = np.zeros((world, k), np.uint64)
    recv_off[1:] = np.cumsum(recv_n[:-1], axis=0)
    return send_off, send_n, recv_off, recv_n


class Exchange:
    """All-to-all of variable-size runs over a torch.distributed group (RCCL on the GPU box)."""

    def __init__(self, device, group=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.group = torch, dist, group
        self.device = device
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.staged = dist.get_backend(group) != "nccl"

    def counts(self, send_counts) -> np.ndarray:
        """Every rank's per-destination counts -> the counts this rank receives from each source."""
        t = self.torch.as_tensor(np.asarray(send_counts, np.int64))
        if not self.staged:
            t = t.to(self.device)
        r = self.torch.empty_like(t)
        self.dist.all_to_all_single(r, t, group=self.group)
        return r.cpu().numpy().astype(np.uint64)

    def runs(self, send, send_counts, recv_counts):
        """send: tensor whose dim-0 slices are grouped by destination (send_counts); returns the
        concatenation of what every source sent here, in source-rank order."""
        sc = [int(c) for c in send_counts]
        rc = [int(c) for c in recv_counts]
        shape = (sum(rc),) + tuple(send.shape[1:])
        if not self.staged:
            recv = self.torch.empty(shape, dtype=send.dtype, device=send.device)
            self.dist.all_to_all_single(recv, send, rc, sc, group=self.group)
            return recv
        host = self.torch.empty(shape, dtype=send.dtype)
        self.dist.all_to_all_single(host, send.cpu(), rc, sc, group=self.group)
        return host.to(send.device)

    def sync(self):
        self.torch.cuda.synchronize(self.device)


def _empty(torch, shape, dtype, device):
    return torch.empty(shape, dtype=dtype, device=device)


def exchange_pnc(store: jg.PNCStore, rows: jg.Rows, ex: Exchange | None, device) -> dict:
    """Route a received PN-Counter batch (global keys) to its owners and merge what arrives here into
    `store` (this rank's shard, local keys).  Returns per-destination sent / per-source received counts."""
    import torch
    world = ex.world if ex else 1
    dt = torch.int64 if rows.eb == 8 else torch.int32
    n, R = rows.n_rows, rows.R
    k = _empty(torch, (n,), torch.int32, device)
    P = _empty(torch, (n, R), dt, device)
    N = _empty(torch, (n, R), dt, device)
    sent = rows.route(world, k.data_ptr(), P.data_ptr(), N.data_ptr())
    if ex is None:
        got, rk, rP, rN = sent, k, P, N
    else:
        got = ex.counts(sent)
        rk, rP, rN = (ex.runs(x, sent, got) for x in (k, P, N))
        ex.sync()  # the collective's stream -> the library's stream
    store.merge_device(int(got.sum()), rk.data_ptr(), rP.data_ptr(), rN.data_ptr())
    return {"sent": sent, "received": got}


def exchange_orset(store: jg.ORSetStore, received: jg.ORSetStore, ex: Exchange | None, device) -> dict:
    """Route a received OR-Set state (global set ids) to its owners and merge what arrives here into
    `store` (this rank's shard, local set ids)."""
    import torch
    world = ex.world if ex else 1
    na, nr = received.size()
    ak, rk = _empty(torch, (na,), torch.int64, device), _empty(torch, (nr,), torch.int64, device)
    at, rt = _empty(torch, (na, 2), torch.int64, device), _empty(torch, (nr, 2), torch.int64, device)
    ao, ro = _empty(torch, (na,), torch.int32, device), _empty(torch, (nr,), torch.int32, device)
    sa, sr = received.route(world, ak.data_ptr(), at.data_ptr(), ao.data_ptr(), na, rk.data_ptr(), rt.data_ptr(), ro.data_ptr(), nr)
    if ex is None:
        ga, gr = sa, sr
    else:
        ga, gr = ex.counts(sa), ex.counts(sr)
        ak, at, ao = ex.runs(ak, sa, ga), ex.runs(at, sa, ga), ex.runs(ao, sa, ga)
        rk, rt, ro = ex.runs(rk, sr, gr), ex.runs(rt, sr, gr), ex.runs(ro, sr, gr)
        ex.sync()
    store.merge_device(ga, gr, ak.data_ptr(), at.data_ptr(), ao.data_ptr(), rk.data_ptr(), rt.data_ptr(), ro.data_ptr())
    return {"sent": (sa, sr), "received": (ga, gr)}
