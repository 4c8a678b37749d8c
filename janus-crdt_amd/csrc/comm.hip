// comm.hip — the cross-shard exchange inside the library, over RCCL.
//
// The keyspace of a node is sharded over its GPUs, one process per GPU (csrc/route.hip: global key k
// belongs to rank k % world, where it is local key k / world).  A received batch that lands on a rank that
// does not own all of its keys still has to reach PNCounter.Merge (MergeSharp/MergeSharp/CRDTs/
// PNCounters.cs:131-144) / ORSet.Merge (ORSet.cs:253-283) on each key's owner.  One call does it all on the
// context's stream:
//
//   route     the stable partition by owner (k_route_hist / k_route_scan / k_route_scatter) into the
//             communicator's send buffers; per-destination counts to the host
//   counts    ncclAllGather of every rank's count vector (world^2 words): each rank learns what every
//             source sends it and sizes its receive buffers
//   runs      one ncclGroupStart/End holding an ncclSend + ncclRecv per peer and buffer — RCCL over the
//             xGMI peer links; this rank's own run is a device-to-device copy into its place
//   merge     the received runs, in source-rank order, merged from device memory (jg_pnc_merge_device's
//             scatter-max / jg_orset_merge_device's run unions)
//
// The 128-byte ncclUniqueId is created by one rank (jg_comm_unique_id) and handed to the others by the
// caller over whatever channel it already has (the C# node's TCP links, torch.distributed in the bench).
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include "jg_internal.hpp"

#define JG_NCCL(call)                                                                                             \
    do {                                                                                                          \
        ncclResult_t r_ = (call);                                                                                 \
        if (r_ != ncclSuccess) ::jg::fail(JG_EHIP, "%s failed: %s (%s:%d)", #call, ncclGetErrorString(r_), __FILE__, \
                                          __LINE__);                                                              \
    } while (0)

static_assert(sizeof(ncclUniqueId) == 128, "the ABI passes the unique id as 128 bytes");

struct jg_comm {
    jg_ctx* ctx = nullptr;
    ncclComm_t nc = nullptr;
    uint32_t rank = 0, world = 1;
    jg::DevBuf dcounts;                    // [world] mine, then [world x world] gathered
    jg::DevBuf sbuf[6], rbuf[6];           // route output / receive buffers (PN-Counter uses 0..2)
    std::vector<uint64_t> hcounts;
    jg_exchange_stats stats{};
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    ~jg_comm() {
        for (hipEvent_t e : ev)
            if (e) (void)hipEventDestroy(e);
        if (nc) (void)ncclCommDestroy(nc);
    }
};

namespace {

void ensure(jg::DevBuf& b, size_t bytes) {
    if (b.bytes < bytes) b.alloc(bytes + bytes / 4 + 256);
}

// Re-raise the error a nested entry point of this library left in the thread's message.
void check_rc(int rc) {
    if (rc == JG_OK) return;
    char msg[1024];
    jg_last_error(msg, sizeof msg);
    jg::fail(rc, "%s", msg);
}

// Every rank's per-destination counts (k words per destination) -> recv[src * k + j] = what src sends
// this rank; the all-gather runs on the context's stream and the call waits for it.
void gather_counts(jg_comm* c, const uint64_t* send, uint32_t k, std::vector<uint64_t>& recv) {
    jg_ctx* ctx = c->ctx;
    const uint32_t W = c->world;
    ensure(c->dcounts, (size_t)(W + (size_t)W * W) * k * 8);
    auto* mine = c->dcounts.as<uint64_t>();
    auto* all = mine + (size_t)W * k;
    JG_HIP(hipMemcpyAsync(mine, send, (size_t)W * k * 8, hipMemcpyHostToDevice, ctx->stream));
    JG_NCCL(ncclAllGather(mine, all, (size_t)W * k, ncclUint64, c->nc, ctx->stream));
    c->hcounts.resize((size_t)W * W * k);
    JG_HIP(hipMemcpyAsync(c->hcounts.data(), all, c->hcounts.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
    JG_HIP(hipStreamSynchronize(ctx->stream));
    recv.assign((size_t)W * k, 0);
    for (uint32_t src = 0; src < W; ++src)
        for (uint32_t j = 0; j < k; ++j) recv[(size_t)src * k + j] = c->hcounts[((size_t)src * W + c->rank) * k + j];
}

// Buffer b of element size `es` per record: the runs sent (grouped by destination, counts `sc`) and received
// (grouped by source, counts `rc`), exchanged in the caller's open group.  `layout` (default sc) gives the
// send buffer's run sizes when sc leaves a run out (a zero count: not sent, not copied).
void post_runs(jg_comm* c, const char* send, char* recv, size_t es, const uint64_t* sc, const uint64_t* rc, uint32_t stride,
               const uint64_t* layout = nullptr) {
    jg_ctx* ctx = c->ctx;
    if (!layout) layout = sc;
    uint64_t so = 0, ro = 0;
    for (uint32_t p = 0; p < c->world; ++p) {
        const uint64_t ns = sc[(size_t)p * stride], nr = rc[(size_t)p * stride];
        if (p == c->rank) {
            if (ns) JG_HIP(hipMemcpyAsync(recv + ro * es, send + so * es, ns * es, hipMemcpyDeviceToDevice, ctx->stream));
        } else {
            if (ns) JG_NCCL(ncclSend(send + so * es, ns * es, ncclUint8, (int)p, c->nc, ctx->stream));
            if (nr) JG_NCCL(ncclRecv(recv + ro * es, nr * es, ncclUint8, (int)p, c->nc, ctx->stream));
        }
        so += layout[(size_t)p * stride];
        ro += nr;
    }
}

// JANUS_TEST_EXCHANGE_FULL=1: a one-rank communicator takes the whole route / all-gather / run path too
// (tests on a one-GPU box; read per call).
bool full_path() {
    const char* e = std::getenv("JANUS_TEST_EXCHANGE_FULL");
    return e && e[0] == '1';
}

hipEvent_t event(jg_comm* c, int i) {
    if (!c->ev[i]) JG_HIP(hipEventCreate(&c->ev[i]));
    return c->ev[i];
}

float elapsed_ms(jg_comm* c, int a, int b) {
    float ms = 0;
    JG_HIP(hipEventElapsedTime(&ms, c->ev[a], c->ev[b]));
    return ms;
}

}  // namespace

extern "C" {

int jg_comm_unique_id(uint8_t* id) {
    return jg::guard([&] {
        JG_REQUIRE(id, JG_EINVAL, "jg_comm_unique_id: NULL argument");
        ncclUniqueId u;
        JG_NCCL(ncclGetUniqueId(&u));
        std::memcpy(id, &u, sizeof u);
    });
}

int jg_comm_init(jg_ctx* ctx, uint32_t rank, uint32_t world, const uint8_t* id, jg_comm** out) {
    return jg::guard([&] {
        JG_REQUIRE(ctx && id && out, JG_EINVAL, "jg_comm_init: NULL argument");
        JG_REQUIRE(world >= 1 && world <= 64 && rank < world, JG_EINVAL, "jg_comm_init: need rank < world <= 64 (rank %u, world %u)", rank, world);
        auto lk_ = jg::lock(ctx);
        jg::ensure_device(ctx);
        auto c = std::make_unique<jg_comm>();
        c->ctx = ctx;
        c->rank = rank;
        c->world = world;
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof u);
        JG_NCCL(ncclCommInitRank(&c->nc, (int)world, u, (int)rank));
        *out = c.release();
    });
}

int jg_comm_destroy(jg_comm* c) {
    return jg::guard([&] {
        if (!c) return;
        auto lk_ = jg::lock(c->ctx);
        jg::ensure_device(c->ctx);
        JG_HIP(hipStreamSynchronize(c->ctx->stream));
        delete c;
    });
}

int jg_comm_last_stats(jg_comm* c, jg_exchange_stats* out) {
    return jg::guard([&] {
        JG_REQUIRE(c && out, JG_EINVAL, "jg_comm_last_stats: NULL argument");
        auto lk_ = jg::lock(c->ctx);
        *out = c->stats;
    });
}

int jg_pnc_exchange(jg_comm* c, jg_pnc* store, const jg_rows* rows, uint64_t* sent, uint64_t* received) {
    return jg::guard([&] {
        JG_REQUIRE(c && store, JG_EINVAL, "jg_pnc_exchange: NULL argument");
        JG_REQUIRE(store->ctx == c->ctx && (!rows || rows->ctx == c->ctx), JG_EINVAL,
                   "jg_pnc_exchange: the store and the batch must be on the communicator's context");
        JG_REQUIRE(!rows || (store->R == rows->R && store->eb == rows->eb), JG_EINVAL,
                   "jg_pnc_exchange: batch shape (%u x %u B) differs from the store's (%u x %u B)", rows ? rows->R : 0, rows ? rows->eb : 0, store->R,
                   store->eb);
        auto lk_ = jg::lock(c->ctx);
        jg_ctx* ctx = c->ctx;
        jg::ensure_device(ctx);
        const uint32_t W = c->world;
        const uint64_t n = rows ? rows->n_rows : 0, rb = (uint64_t)store->R * store->eb;
        if (W == 1 && !full_path()) {  // every key is this rank's and local key = global key: the batch merges in place
            JG_HIP(hipEventRecord(event(c, 0), ctx->stream));
            if (rows) check_rc(jg_pnc_merge_batch(store, rows, 0));
            JG_HIP(hipEventRecord(event(c, 3), ctx->stream));
            JG_HIP(hipStreamSynchronize(ctx->stream));
            c->stats = jg_exchange_stats{0, 0, elapsed_ms(c, 0, 3) * 1e-3, 0, 0, n};
            if (sent) sent[0] = n;
            if (received) received[0] = n;
            return;
        }
        ensure(c->sbuf[0], n * 4 + 16);
        ensure(c->sbuf[1], n * rb + 16);
        ensure(c->sbuf[2], n * rb + 16);
        JG_HIP(hipEventRecord(event(c, 0), ctx->stream));
        std::vector<uint64_t> sc(W), rc;
        if (rows) check_rc(jg_rows_route(rows, W, sc.data(), c->sbuf[0].p, c->sbuf[1].p, c->sbuf[2].p, n));
        JG_HIP(hipEventRecord(event(c, 1), ctx->stream));
        gather_counts(c, sc.data(), 1, rc);
        // max is order-free: this rank's own run merges straight from the send buffers, the peers' runs
        // land back to back in the receive buffers (rc with the own entry zeroed)
        const uint64_t own = sc[c->rank];
        uint64_t own_at = 0;
        for (uint32_t p = 0; p < c->rank; ++p) own_at += sc[p];
        std::vector<uint64_t> sc2 = sc, rc2 = rc;
        sc2[c->rank] = rc2[c->rank] = 0;
        uint64_t nr = 0;
        for (uint64_t x : rc2) nr += x;
        ensure(c->rbuf[0], nr * 4 + 16);
        ensure(c->rbuf[1], nr * rb + 16);
        ensure(c->rbuf[2], nr * rb + 16);
        JG_NCCL(ncclGroupStart());
        post_runs(c, c->sbuf[0].as<char>(), c->rbuf[0].as<char>(), 4, sc2.data(), rc2.data(), 1, sc.data());
        post_runs(c, c->sbuf[1].as<char>(), c->rbuf[1].as<char>(), rb, sc2.data(), rc2.data(), 1, sc.data());
        post_runs(c, c->sbuf[2].as<char>(), c->rbuf[2].as<char>(), rb, sc2.data(), rc2.data(), 1, sc.data());
        JG_NCCL(ncclGroupEnd());
        JG_HIP(hipEventRecord(event(c, 2), ctx->stream));
        if (own)
            check_rc(jg_pnc_merge_device(store, own, c->sbuf[0].as<char>() + own_at * 4, c->sbuf[1].as<char>() + own_at * rb,
                                         c->sbuf[2].as<char>() + own_at * rb));
        if (nr) check_rc(jg_pnc_merge_device(store, nr, c->rbuf[0].p, c->rbuf[1].p, c->rbuf[2].p));
        nr += own;
        JG_HIP(hipEventRecord(event(c, 3), ctx->stream));
        JG_HIP(hipStreamSynchronize(ctx->stream));
        uint64_t off_rank = 0;
        for (uint32_t p = 0; p < W; ++p) off_rank += p == c->rank ? 0 : sc[p];
        c->stats = jg_exchange_stats{elapsed_ms(c, 0, 1) * 1e-3, elapsed_ms(c, 1, 2) * 1e-3, elapsed_ms(c, 2, 3) * 1e-3, off_rank * (4 + 2 * rb),
                                     (nr - own) * (4 + 2 * rb), nr};
        if (sent) std::copy(sc.begin(), sc.end(), sent);
        if (received) std::copy(rc.begin(), rc.end(), received);
    });
}

int jg_orset_exchange(jg_comm* c, jg_orset* store, jg_orset* received, uint64_t* sent_add, uint64_t* sent_rem, uint64_t* recv_add,
                      uint64_t* recv_rem) {
    return jg::guard([&] {
        JG_REQUIRE(c && store && received, JG_EINVAL, "jg_orset_exchange: NULL argument");
        JG_REQUIRE(store->ctx == c->ctx && received->ctx == c->ctx, JG_EINVAL, "jg_orset_exchange: the stores must be on the communicator's context");
        JG_REQUIRE(store != received, JG_EINVAL, "jg_orset_exchange: the received state cannot be the store itself");
        auto lk_ = jg::lock(c->ctx);
        jg_ctx* ctx = c->ctx;
        jg::ensure_device(ctx);
        const uint32_t W = c->world;
        jg::sync_counts(received);
        const uint64_t na = received->add.n, nrm = received->rem.n;
        if (W == 1 && !full_path()) {  // set id = local id: ORSet.Merge of the received state in place
            JG_HIP(hipEventRecord(event(c, 0), ctx->stream));
            check_rc(jg_orset_merge_store(store, received, 0));
            JG_HIP(hipEventRecord(event(c, 3), ctx->stream));
            JG_HIP(hipStreamSynchronize(ctx->stream));
            c->stats = jg_exchange_stats{0, 0, elapsed_ms(c, 0, 3) * 1e-3, 0, 0, na + nrm};
            if (sent_add) sent_add[0] = na;
            if (sent_rem) sent_rem[0] = nrm;
            if (recv_add) recv_add[0] = na;
            if (recv_rem) recv_rem[0] = nrm;
            return;
        }
        const size_t es[6] = {8, 16, 4, 8, 16, 4};  // key, tag, ord of the add stream, then of the tombstones
        for (int i = 0; i < 6; ++i) ensure(c->sbuf[i], (i < 3 ? na : nrm) * es[i] + 16);
        JG_HIP(hipEventRecord(event(c, 0), ctx->stream));
        std::vector<uint64_t> sa(W), sr(W);
        check_rc(jg_orset_route(received, W, sa.data(), sr.data(), c->sbuf[0].p, c->sbuf[1].p, c->sbuf[2].p, na, c->sbuf[3].p, c->sbuf[4].p,
                                c->sbuf[5].p, nrm));
        JG_HIP(hipEventRecord(event(c, 1), ctx->stream));
        std::vector<uint64_t> sc(2 * (size_t)W), rc;
        for (uint32_t p = 0; p < W; ++p) sc[2 * p] = sa[p], sc[2 * p + 1] = sr[p];
        gather_counts(c, sc.data(), 2, rc);
        std::vector<uint64_t> ra(W), rr(W);
        uint64_t ta = 0, tr = 0;
        for (uint32_t p = 0; p < W; ++p) ra[p] = rc[2 * p], rr[p] = rc[2 * p + 1], ta += ra[p], tr += rr[p];
        for (int i = 0; i < 6; ++i) ensure(c->rbuf[i], (i < 3 ? ta : tr) * es[i] + 16);
        JG_NCCL(ncclGroupStart());
        for (int i = 0; i < 6; ++i)
            post_runs(c, c->sbuf[i].as<char>(), c->rbuf[i].as<char>(), es[i], sc.data() + (i < 3 ? 0 : 1), rc.data() + (i < 3 ? 0 : 1), 2);
        JG_NCCL(ncclGroupEnd());
        JG_HIP(hipEventRecord(event(c, 2), ctx->stream));
        check_rc(jg_orset_merge_device(store, W, ra.data(), rr.data(), c->rbuf[0].p, c->rbuf[1].p, c->rbuf[2].p, c->rbuf[3].p, c->rbuf[4].p,
                                       c->rbuf[5].p));
        JG_HIP(hipEventRecord(event(c, 3), ctx->stream));
        JG_HIP(hipStreamSynchronize(ctx->stream));
        constexpr uint64_t kRec = 28;  // key + tag + ord
        uint64_t out = 0;
        for (uint32_t p = 0; p < W; ++p) out += p == c->rank ? 0 : sa[p] + sr[p];
        c->stats = jg_exchange_stats{elapsed_ms(c, 0, 1) * 1e-3, elapsed_ms(c, 1, 2) * 1e-3, elapsed_ms(c, 2, 3) * 1e-3, out * kRec,
                                     (ta + tr - ra[c->rank] - rr[c->rank]) * kRec, ta + tr};
        if (sent_add) std::copy(sa.begin(), sa.end(), sent_add);
        if (sent_rem) std::copy(sr.begin(), sr.end(), sent_rem);
        if (recv_add) std::copy(ra.begin(), ra.end(), recv_add);
        if (recv_rem) std::copy(rr.begin(), rr.end(), recv_rem);
    });
}

}  // extern "C"
