// comm.hip — the cross-shard exchange inside the library.
//
// The keyspace of a node is sharded over its GPUs, one process per GPU (jg_internal.hpp's owner rule:
// global key k belongs to rank owner_of_key(k) = k % world, where it is local key k / world).  A received
// batch that lands on a rank that does not own all of its keys still has to reach PNCounter.Merge
// (MergeSharp/MergeSharp/CRDTs/PNCounters.cs:131-144) / ORSet.Merge (ORSet.cs:253-283) on each key's
// owner — the routing the reference does by uid lookup on every receiver (safeCRDTsIndexedByuid[u.uid],
// BFT-CRDT/CRDTManagers/SafeCRDTManager.cs:136, fed by ConnectionManager.ReceivedBlock,
// BFT-CRDT/Network/DAGConnectionManager.cs:40-50).  One call does it all on the context's stream:
//
//   route     the stable partition by owner (k_route_hist / k_route_scan / k_route_scatter) into the
//             communicator's send buffers; per-destination counts to the host
//   counts    an all-gather of every rank's count vector (world^2 words): each rank learns what every
//             source sends it
//   plan      jg_exchange_plan (host, pure): every peer's send run and receive slot per buffer
//   runs      one group of send + receive per peer and buffer; this rank's own run by a device copy
//   merge     the received runs, in source-rank order, merged from device memory (jg_pnc_merge_device's
//             grouped fold / jg_orset_merge_device's run unions)
//
// Two transports carry the counts and the runs:
//   RCCL      (jg_comm_init) ncclAllGather + grouped ncclSend / ncclRecv over the xGMI peer links.  The
//             communicator is NON-BLOCKING (ncclConfig_t.blocking = 0): init, every group and every wait
//             for the stream poll ncclCommGetAsyncError against a deadline (JANUS_COMM_TIMEOUT_S, default
//             120 s); past it the communicator is aborted (ncclCommAbort) and the call returns JG_EHIP
//             instead of hanging — a peer that never joins or dies mid-exchange costs a bounded wait.
//   host      (jg_comm_init_host) the caller's all-to-all-v callback over page-locked host memory: the same
//             route / plan / merge code at world > 1 where RCCL cannot run (RCCL refuses two ranks on one
//             GPU), e.g. ranks sharing a device in a test, or a caller that moves shards over its own links.
//
// The 128-byte ncclUniqueId is created by one rank (jg_comm_unique_id) and handed to the others by the
// caller over whatever channel it already has (the C# node's TCP links, torch.distributed in the bench).
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "jg_internal.hpp"

static_assert(sizeof(ncclUniqueId) == 128, "the ABI passes the unique id as 128 bytes");

struct jg_comm {
    jg_ctx* ctx = nullptr;
    ncclComm_t nc = nullptr;               // RCCL transport (nullptr: host transport, or aborted)
    jg_alltoallv_fn host_fn = nullptr;     // host transport
    void* host_user = nullptr;
    bool rccl = false;                     // the RCCL transport (else the host transport)
    bool broken = false;                   // aborted after a timeout / async error: every call fails
    uint32_t rank = 0, world = 1;
    double timeout_s = 120;
    jg::DevBuf dcounts;                    // [world] mine, then [world x world] gathered
    jg::DevBuf sbuf[6], rbuf[6];           // route output / receive buffers (PN-Counter uses 0..2)
    std::vector<uint64_t> hcounts;
    uint8_t* pin = nullptr;                // host transport staging (page-locked)
    size_t pin_cap = 0;
    jg_exchange_stats stats{};
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    ~jg_comm() {
        for (hipEvent_t e : ev)
            if (e) (void)hipEventDestroy(e);
        if (pin) (void)hipHostFree(pin);
    }
};

namespace {

using Clock = std::chrono::steady_clock;

#define JG_NCCL(c, call) nccl_check((c), (call), #call, __LINE__)

bool trace_comm() {
    static const bool t = std::getenv("JANUS_TRACE_COMM") != nullptr;
    return t;
}

// Every abort happens on the calling thread, inside one of the polling loops below (the communicator is
// non-blocking, so no RCCL call of this library ever blocks): the handle is freed exactly once, and nothing
// touches it afterwards (nc = nullptr, broken = true; every entry point checks `broken` first).
void abort_comm(jg_comm* c) {
    if (c->broken) return;
    if (trace_comm()) std::fprintf(stderr, "jg_comm: aborting the communicator\n");
    c->broken = true;
    if (c->nc) (void)ncclCommAbort(c->nc);
    c->nc = nullptr;
    if (trace_comm()) std::fprintf(stderr, "jg_comm: aborted\n");
}

// Poll the communicator until no operation is in progress (non-blocking RCCL), against the deadline.
void nccl_settle(jg_comm* c, const char* what, int line) {
    JG_REQUIRE(c->nc && !c->broken, JG_EHIP, "%s: the communicator was aborted (comm.hip:%d)", what, line);
    const auto end = Clock::now() + std::chrono::duration<double>(c->timeout_s);
    for (;;) {
        ncclResult_t a = ncclSuccess;
        const ncclResult_t q = ncclCommGetAsyncError(c->nc, &a);
        if (q != ncclSuccess) a = q;
        if (a == ncclSuccess) return;
        if (a != ncclInProgress) {
            abort_comm(c);
            jg::fail(JG_EHIP, "%s failed: %s (comm.hip:%d); the communicator was aborted", what, ncclGetErrorString(a), line);
        }
        if (Clock::now() > end) {
            abort_comm(c);
            jg::fail(JG_EHIP, "%s: no progress in %.0f s (a rank missing or stuck, comm.hip:%d); the communicator was aborted", what, c->timeout_s,
                     line);
        }
        std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

void nccl_check(jg_comm* c, ncclResult_t r, const char* what, int line) {
    if (r == ncclSuccess) return;
    if (r == ncclInProgress) return nccl_settle(c, what, line);
    abort_comm(c);
    jg::fail(JG_EHIP, "%s failed: %s (comm.hip:%d); the communicator was aborted", what, ncclGetErrorString(r), line);
}

// The context's stream drained: with RCCL work queued on it, polled against the deadline (a peer that never
// posts its half of a send / receive leaves the RCCL kernel waiting forever; hipStreamSynchronize would too).
void wait_stream(jg_comm* c) {
    jg_ctx* ctx = c->ctx;
    if (!c->rccl) {
        JG_HIP(hipStreamSynchronize(ctx->stream));
        return;
    }
    const auto end = Clock::now() + std::chrono::duration<double>(c->timeout_s);
    for (;;) {
        const hipError_t e = hipStreamQuery(ctx->stream);
        if (e == hipSuccess) return;
        if (e != hipErrorNotReady) JG_HIP(e);
        JG_REQUIRE(!c->broken, JG_EHIP, "exchange: no progress in %.0f s (a rank missing or stuck); the communicator was aborted", c->timeout_s);
        ncclResult_t a = ncclSuccess;
        (void)ncclCommGetAsyncError(c->nc, &a);
        if (a != ncclSuccess && a != ncclInProgress) {
            abort_comm(c);
            jg::fail(JG_EHIP, "exchange: RCCL reported %s; the communicator was aborted", ncclGetErrorString(a));
        }
        if (Clock::now() > end) {
            abort_comm(c);
            jg::fail(JG_EHIP, "exchange: the collective did not finish in %.0f s (a rank missing or stuck); the communicator was aborted",
                     c->timeout_s);
        }
        std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}

void ensure(jg::DevBuf& b, size_t bytes) {
    if (b.bytes < bytes) b.alloc(bytes + bytes / 4 + 256);
}

uint8_t* pinned(jg_comm* c, size_t bytes) {
    if (c->pin_cap < bytes) {
        if (c->pin) JG_HIP(hipHostFree(c->pin));
        c->pin = nullptr;
        c->pin_cap = 0;
        void* p = nullptr;
        JG_HIP(hipHostMalloc(&p, bytes + bytes / 4 + 256, hipHostMallocDefault));
        c->pin = static_cast<uint8_t*>(p);
        c->pin_cap = bytes + bytes / 4 + 256;
    }
    return c->pin;
}

// Re-raise the error a nested entry point of this library left in the thread's message.
void check_rc(int rc) {
    if (rc == JG_OK) return;
    char msg[1024];
    jg_last_error(msg, sizeof msg);
    jg::fail(rc, "%s", msg);
}

void host_xfer(jg_comm* c, const void* send, const uint64_t* sb, void* recv, const uint64_t* rb) {
    const int r = c->host_fn(c->host_user, send, sb, recv, rb);
    JG_REQUIRE(r == 0, JG_EHIP, "exchange: the host transport's all-to-all returned %d", r);
}

// Every rank's per-destination counts (k words per destination) -> all[src][dst][j] (src-major, world^2 k
// words): what every source sends every destination.  The call waits for it.
void gather_counts(jg_comm* c, const uint64_t* send, uint32_t k, std::vector<uint64_t>& all) {
    jg_ctx* ctx = c->ctx;
    const uint32_t W = c->world;
    all.resize((size_t)W * W * k);
    if (c->host_fn) {  // an all-to-all-v carrying this rank's whole vector to every peer
        std::vector<uint64_t> out((size_t)W * W * k), sb(W, (uint64_t)W * k * 8), rb(W, (uint64_t)W * k * 8);
        for (uint32_t p = 0; p < W; ++p) std::memcpy(out.data() + (size_t)p * W * k, send, (size_t)W * k * 8);
        host_xfer(c, out.data(), sb.data(), all.data(), rb.data());
        return;
    }
    ensure(c->dcounts, (size_t)(W + (size_t)W * W) * k * 8);
    auto* mine = c->dcounts.as<uint64_t>();
    auto* dall = mine + (size_t)W * k;
    JG_HIP(hipMemcpyAsync(mine, send, (size_t)W * k * 8, hipMemcpyHostToDevice, ctx->stream));
    JG_NCCL(c, ncclAllGather(mine, dall, (size_t)W * k, ncclUint64, c->nc, ctx->stream));
    c->hcounts.resize(all.size());
    JG_HIP(hipMemcpyAsync(c->hcounts.data(), dall, c->hcounts.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
    wait_stream(c);
    all = c->hcounts;
}

struct Plan {
    std::vector<uint64_t> send_off, send_n, recv_off, recv_n;  // [world x k]: peer p, buffer j at p * k + j
};

Plan plan_of(jg_comm* c, const std::vector<uint64_t>& all, uint32_t k, bool skip_own) {
    Plan pl;
    const uint32_t W = c->world;
    for (auto* v : {&pl.send_off, &pl.send_n, &pl.recv_off, &pl.recv_n}) v->resize((size_t)W * k);
    check_rc(jg_exchange_plan(c->rank, W, k, all.data(), skip_own ? 1 : 0, pl.send_off.data(), pl.send_n.data(), pl.recv_off.data(),
                              pl.recv_n.data()));
    return pl;
}

// Buffer j's runs (element size es): peer p gets send[send_off .. + send_n) and this rank receives
// recv[recv_off .. + recv_n) from it; the own run (p == rank) moves by a device copy.  RCCL: posted into the
// caller's open group.  Host transport: staged through page-locked memory around one all-to-all-v.
void post_runs(jg_comm* c, const Plan& pl, uint32_t k, uint32_t j, const char* send, char* recv, size_t es) {
    jg_ctx* ctx = c->ctx;
    const uint32_t W = c->world;
    for (uint32_t p = 0; p < W; ++p) {
        const size_t x = (size_t)p * k + j;
        if (p == c->rank) {
            JG_REQUIRE(pl.send_n[x] == pl.recv_n[x], JG_EHIP, "exchange plan: own run %llu sent, %llu received", (unsigned long long)pl.send_n[x],
                       (unsigned long long)pl.recv_n[x]);
            if (pl.send_n[x])
                JG_HIP(hipMemcpyAsync(recv + pl.recv_off[x] * es, send + pl.send_off[x] * es, pl.send_n[x] * es, hipMemcpyDeviceToDevice, ctx->stream));
        } else if (c->rccl) {
            if (pl.send_n[x]) JG_NCCL(c, ncclSend(send + pl.send_off[x] * es, pl.send_n[x] * es, ncclUint8, (int)p, c->nc, ctx->stream));
            if (pl.recv_n[x]) JG_NCCL(c, ncclRecv(recv + pl.recv_off[x] * es, pl.recv_n[x] * es, ncclUint8, (int)p, c->nc, ctx->stream));
        }
    }
    if (c->rccl) return;
    // host transport: peers' runs out through page-locked staging, one all-to-all-v, back in
    std::vector<uint64_t> sb(W, 0), rb(W, 0);
    uint64_t ts = 0, tr = 0;
    for (uint32_t p = 0; p < W; ++p)
        if (p != c->rank) sb[p] = pl.send_n[(size_t)p * k + j] * es, rb[p] = pl.recv_n[(size_t)p * k + j] * es, ts += sb[p], tr += rb[p];
    uint8_t* h = pinned(c, ts + tr + 64);
    uint8_t* hs = h;
    uint8_t* hr = h + ((ts + 63) & ~63ull);
    uint64_t o = 0;
    for (uint32_t p = 0; p < W; ++p)
        if (sb[p]) {
            JG_HIP(hipMemcpyAsync(hs + o, send + pl.send_off[(size_t)p * k + j] * es, sb[p], hipMemcpyDeviceToHost, ctx->stream));
            o += sb[p];
        }
    JG_HIP(hipStreamSynchronize(ctx->stream));
    host_xfer(c, hs, sb.data(), hr, rb.data());
    o = 0;
    for (uint32_t p = 0; p < W; ++p)
        if (rb[p]) {
            JG_HIP(hipMemcpyAsync(recv + pl.recv_off[(size_t)p * k + j] * es, hr + o, rb[p], hipMemcpyHostToDevice, ctx->stream));
            o += rb[p];
        }
    JG_HIP(hipStreamSynchronize(ctx->stream));  // the staging is reused by the next buffer
}

void group_start(jg_comm* c) {
    if (c->rccl) JG_NCCL(c, ncclGroupStart());
}
void group_end(jg_comm* c) {
    if (c->rccl) JG_NCCL(c, ncclGroupEnd());
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

double timeout_from_env() {
    const char* e = std::getenv("JANUS_COMM_TIMEOUT_S");
    const double t = e ? std::atof(e) : 120.0;
    return t > 0 ? t : 120.0;
}

jg_comm* usable(jg_comm* c, const char* fn) {
    JG_REQUIRE(c, JG_EINVAL, "%s: NULL communicator", fn);
    JG_REQUIRE(!c->broken, JG_EHIP, "%s: the communicator was aborted by an earlier failure; destroy it and join a new one", fn);
    return c;
}

}  // namespace

extern "C" {

int jg_exchange_plan(uint32_t rank, uint32_t world, uint32_t k, const uint64_t* counts, uint8_t skip_own, uint64_t* send_off, uint64_t* send_n,
                     uint64_t* recv_off, uint64_t* recv_n) {
    return jg::guard([&] {
        JG_REQUIRE(counts && send_off && send_n && recv_off && recv_n, JG_EINVAL, "jg_exchange_plan: NULL argument");
        JG_REQUIRE(world >= 1 && world <= 64 && rank < world && k >= 1, JG_EINVAL, "jg_exchange_plan: need rank < world <= 64, k >= 1");
        const uint32_t W = world;
        auto cnt = [&](uint32_t src, uint32_t dst, uint32_t j) { return counts[((size_t)src * W + dst) * k + j]; };
        for (uint32_t j = 0; j < k; ++j) {
            // send buffer j holds every destination's run, destinations in rank order (the route's stable
            // partition); receive buffer j takes the peers' runs back to back in source-rank order
            uint64_t so = 0, ro = 0;
            for (uint32_t p = 0; p < W; ++p) {
                const size_t x = (size_t)p * k + j;
                const bool own_skipped = skip_own && p == rank;
                send_off[x] = so;
                send_n[x] = own_skipped ? 0 : cnt(rank, p, j);
                recv_off[x] = ro;
                recv_n[x] = own_skipped ? 0 : cnt(p, rank, j);
                so += cnt(rank, p, j);
                ro += recv_n[x];
            }
        }
    });
}

int jg_comm_unique_id(uint8_t* id) {
    return jg::guard([&] {
        JG_REQUIRE(id, JG_EINVAL, "jg_comm_unique_id: NULL argument");
        ncclUniqueId u;
        const ncclResult_t r = ncclGetUniqueId(&u);
        JG_REQUIRE(r == ncclSuccess, JG_EHIP, "ncclGetUniqueId failed: %s", ncclGetErrorString(r));
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
        c->timeout_s = timeout_from_env();
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof u);
        // A non-blocking communicator (blocking = 0): every later call returns ncclInProgress instead of waiting,
        // and this library polls it against the deadline on the calling thread.
        //
        // The rendezvous.  ncclCommInitRankConfig OUTSIDE a group runs the whole init, the bootstrap's wait for every
        // rank included, on the calling thread even for a non-blocking config (RCCL queues it as an async job and,
        // with no group open, runs the job at once).  Round 5 ran it that way on a detached thread; a rank that gave
        // up left that thread inside the bootstrap, and static teardown at exit then faulted under it (rc 139 after
        // the timeout, gpurun_out/comm_dbg.log).  INSIDE ncclGroupStart / ncclGroupEnd the non-blocking
        // config makes ncclGroupEnd hand the job to RCCL's own thread and return ncclInProgress with the handle set.
        // A helper thread issues the group and polls the handle to ready (every RCCL call of the rendezvous on the
        // thread that opened the group, whose thread-local group state RCCL's job may still use); the call waits for
        // it against the deadline.  Past the deadline the helper, no longer stuck in the bootstrap, sees the call give
        // up within a poll, aborts the handle (ncclCommAbort raises the init's abort flag, which the bootstrap's
        // sockets check) and exits, and the call JOINS it: nothing of the rendezvous outlives the call.  Should this
        // RCCL block inside the group calls after all, the helper is left behind (detached) as in round 5, and the
        // call still returns JG_EHIP on time.
        struct Job {
            std::mutex m;
            std::condition_variable cv;
            bool done = false, abandoned = false, exited = false;
            ncclResult_t r = ncclSuccess;
            ncclComm_t nc = nullptr;
        };
        auto job = std::make_shared<Job>();
        const int dev = ctx->device;
        const auto end = Clock::now() + std::chrono::duration_cast<Clock::duration>(std::chrono::duration<double>(c->timeout_s));
        if (trace_comm()) std::fprintf(stderr, "jg_comm: ncclCommInitRankConfig in a group (rank %u of %u, non-blocking)\n", rank, world);
        std::thread helper([job, u, rank, world, dev] {
            (void)hipSetDevice(dev);
            ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
            cfg.blocking = 0;
            ncclComm_t nc = nullptr;
            ncclResult_t r = ncclGroupStart();
            if (r == ncclSuccess) {
                r = ncclCommInitRankConfig(&nc, (int)world, u, (int)rank, &cfg);
                const ncclResult_t e = ncclGroupEnd();
                if (r == ncclSuccess || r == ncclInProgress) r = e;
            }
            while (r == ncclInProgress && nc) {
                {
                    std::lock_guard<std::mutex> g(job->m);
                    if (job->abandoned) break;
                }
                ncclResult_t a = ncclInProgress;
                const ncclResult_t q = ncclCommGetAsyncError(nc, &a);
                r = q != ncclSuccess ? q : a;
                if (r == ncclInProgress) std::this_thread::sleep_for(std::chrono::microseconds(100));
            }
            std::lock_guard<std::mutex> g(job->m);
            if (job->abandoned || r != ncclSuccess) {
                if (nc) (void)ncclCommAbort(nc);
                nc = nullptr;
            }
            if (!job->abandoned) {
                job->r = r;
                job->nc = nc;
                job->done = true;
            }
            job->exited = true;
            job->cv.notify_all();
        });
        bool joined = false;
        {
            std::unique_lock<std::mutex> g(job->m);
            if (!job->cv.wait_until(g, end, [&] { return job->done || job->exited; })) {
                job->abandoned = true;
                if (trace_comm()) std::fprintf(stderr, "jg_comm: rendezvous timed out\n");
                // the helper aborts the handle and exits within a poll, unless RCCL holds it inside the group calls
                joined = job->cv.wait_for(g, std::chrono::seconds(10), [&] { return job->exited; });
                g.unlock();
                if (joined) helper.join();
                else helper.detach();
                if (trace_comm()) std::fprintf(stderr, "jg_comm: rendezvous helper %s\n", joined ? "joined" : "left behind");
                jg::fail(JG_EHIP, "jg_comm_init: not every rank joined in %.0f s (rank %u of %u); JANUS_COMM_TIMEOUT_S sets the wait", c->timeout_s,
                         rank, world);
            }
        }
        helper.join();
        if (trace_comm()) std::fprintf(stderr, "jg_comm: rendezvous settled: %s\n", ncclGetErrorString(job->r));
        JG_REQUIRE(job->r == ncclSuccess && job->nc, JG_EHIP, "ncclCommInitRankConfig failed: %s", ncclGetErrorString(job->r));
        c->nc = job->nc;
        if (trace_comm()) std::fprintf(stderr, "jg_comm: rendezvous complete\n");
        c->rccl = true;
        *out = c.release();
    });
}

int jg_comm_init_host(jg_ctx* ctx, uint32_t rank, uint32_t world, jg_alltoallv_fn fn, void* user, jg_comm** out) {
    return jg::guard([&] {
        JG_REQUIRE(ctx && fn && out, JG_EINVAL, "jg_comm_init_host: NULL argument");
        JG_REQUIRE(world >= 1 && world <= 64 && rank < world, JG_EINVAL, "jg_comm_init_host: need rank < world <= 64 (rank %u, world %u)", rank,
                   world);
        auto lk_ = jg::lock(ctx);
        jg::ensure_device(ctx);
        auto c = std::make_unique<jg_comm>();
        c->ctx = ctx;
        c->rank = rank;
        c->world = world;
        c->host_fn = fn;
        c->host_user = user;
        *out = c.release();
    });
}

int jg_comm_destroy(jg_comm* c) {
    return jg::guard([&] {
        if (!c) return;
        std::unique_ptr<jg_comm> own(c);
        auto lk_ = jg::lock(c->ctx);
        jg::ensure_device(c->ctx);
        if (c->broken || !c->nc) return;  // host transport, or aborted: its queued work was cancelled with it
        wait_stream(c);
        // non-blocking: finalize (flushes the communicator's work) polled to completion, then destroy
        JG_NCCL(c, ncclCommFinalize(c->nc));
        (void)ncclCommDestroy(c->nc);
        c->nc = nullptr;
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
        usable(c, "jg_pnc_exchange");
        JG_REQUIRE(store, JG_EINVAL, "jg_pnc_exchange: NULL argument");
        jg::require_writable(store, "jg_pnc_exchange");
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
        std::vector<uint64_t> sc(W, 0), all;
        if (rows) check_rc(jg_rows_route(rows, W, sc.data(), c->sbuf[0].p, c->sbuf[1].p, c->sbuf[2].p, n));
        JG_HIP(hipEventRecord(event(c, 1), ctx->stream));
        gather_counts(c, sc.data(), 1, all);
        // max is order-free: this rank's own run merges straight from the send buffers (skip_own), the peers'
        // runs land back to back in the receive buffers
        const Plan pl = plan_of(c, all, 1, true);
        const uint64_t own = sc[c->rank], own_at = pl.send_off[c->rank];
        uint64_t nr = 0;
        for (uint32_t p = 0; p < W; ++p) nr += pl.recv_n[p];
        ensure(c->rbuf[0], nr * 4 + 16);
        ensure(c->rbuf[1], nr * rb + 16);
        ensure(c->rbuf[2], nr * rb + 16);
        const size_t es[3] = {4, rb, rb};
        group_start(c);
        for (uint32_t b = 0; b < 3; ++b) post_runs(c, pl, 1, 0, c->sbuf[b].as<char>(), c->rbuf[b].as<char>(), es[b]);
        group_end(c);
        JG_HIP(hipEventRecord(event(c, 2), ctx->stream));
        if (c->rccl) wait_stream(c);  // RCCL: the runs are in before the merges' own host syncs (bounded wait)
        if (own)
            check_rc(jg_pnc_merge_device(store, own, c->sbuf[0].as<char>() + own_at * 4, c->sbuf[1].as<char>() + own_at * rb,
                                         c->sbuf[2].as<char>() + own_at * rb));
        if (nr) check_rc(jg_pnc_merge_device(store, nr, c->rbuf[0].p, c->rbuf[1].p, c->rbuf[2].p));
        JG_HIP(hipEventRecord(event(c, 3), ctx->stream));
        wait_stream(c);
        uint64_t off_rank = 0;
        for (uint32_t p = 0; p < W; ++p) off_rank += pl.send_n[p];
        c->stats = jg_exchange_stats{elapsed_ms(c, 0, 1) * 1e-3, elapsed_ms(c, 1, 2) * 1e-3, elapsed_ms(c, 2, 3) * 1e-3, off_rank * (4 + 2 * rb),
                                     nr * (4 + 2 * rb), nr + own};
        if (sent) std::copy(sc.begin(), sc.end(), sent);
        if (received)
            for (uint32_t p = 0; p < W; ++p) received[p] = all[(size_t)p * W + c->rank];
    });
}

int jg_orset_exchange(jg_comm* c, jg_orset* store, jg_orset* received, uint64_t* sent_add, uint64_t* sent_rem, uint64_t* recv_add,
                      uint64_t* recv_rem) {
    return jg::guard([&] {
        usable(c, "jg_orset_exchange");
        JG_REQUIRE(store && received, JG_EINVAL, "jg_orset_exchange: NULL argument");
        JG_REQUIRE(store->ctx == c->ctx && received->ctx == c->ctx, JG_EINVAL, "jg_orset_exchange: the stores must be on the communicator's context");
        JG_REQUIRE(store != received, JG_EINVAL, "jg_orset_exchange: the received state cannot be the store itself");
        jg::require_writable(store, "jg_orset_exchange");
        jg::require_writable(received, "jg_orset_exchange");
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
        std::vector<uint64_t> sc(2 * (size_t)W), all;
        for (uint32_t p = 0; p < W; ++p) sc[2 * p] = sa[p], sc[2 * p + 1] = sr[p];
        gather_counts(c, sc.data(), 2, all);
        // the union keeps source-rank order (arrival ordinals), so the own run takes its place among the
        // received ones (no skip)
        const Plan pl = plan_of(c, all, 2, false);
        std::vector<uint64_t> ra(W), rr(W);
        uint64_t ta = 0, tr = 0;
        for (uint32_t p = 0; p < W; ++p) ra[p] = pl.recv_n[2 * p], rr[p] = pl.recv_n[2 * p + 1], ta += ra[p], tr += rr[p];
        for (int i = 0; i < 6; ++i) ensure(c->rbuf[i], (i < 3 ? ta : tr) * es[i] + 16);
        group_start(c);
        for (int i = 0; i < 6; ++i) post_runs(c, pl, 2, i < 3 ? 0 : 1, c->sbuf[i].as<char>(), c->rbuf[i].as<char>(), es[i]);
        group_end(c);
        JG_HIP(hipEventRecord(event(c, 2), ctx->stream));
        if (c->rccl) wait_stream(c);  // RCCL: the runs are in before the merge's host reads (bounded wait)
        check_rc(jg_orset_merge_device(store, W, ra.data(), rr.data(), c->rbuf[0].p, c->rbuf[1].p, c->rbuf[2].p, c->rbuf[3].p, c->rbuf[4].p,
                                       c->rbuf[5].p));
        JG_HIP(hipEventRecord(event(c, 3), ctx->stream));
        wait_stream(c);
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
