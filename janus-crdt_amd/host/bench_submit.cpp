// bench_submit.cpp — the producer path of one node.
//
// Every client op goes through SafeCRDT.Update (BFT-CRDT/SafeCRDTs/SafeCRDT.cs:39-62): ApplyOp on the node's
// PROSPECTIVE copy, GetLastSynchronizedUpdate().Encode() of the key's FULL state, tracked when safe, queued in
// the client batcher ActualPropagateSyncMsg (BFT-CRDT/CRDTManagers/SafeCRDTManager.cs:165-198: clientBatchSize
// 1000, safe states kept, non-safe states compacted per uid), and every UpdateMessage the batcher submits gets
// its ComputeDigest (DAGUpdateMessage.cs:25-55).
//   --workload pnc    the banking client ops one node of the C5 replay receives (BankingWorload.cs: deposit
//                     "i" non-safe, transfer "d" safe + "i" non-safe, withdraw "d" safe; every "d" an Increment,
//                     PNCounterCommand.cs:48-50) over `keys` accounts whose prospective copies already hold the
//                     other 3 nodes' replicas (a 4-replica state ≈ 357 B, as the committed waves carry)
//   --workload orset  ORSetWorkload.cs:37-50: Add of a random 5-character string with a fresh Guid tag, Clear once
//                     the set holds 50 elements, over `keys` sets (states up to ≈ 2.5 KB)
// GPU: janus::GpuStableStore::SubmitClientUpdates — one call per wave of `ops` client ops (ApplyOps in chunks,
// snapshots encoded on the device for PN-Counters and by the host writer for OR-Sets, the batcher, digests in
// one device call).  CPU baseline: the oracle's SafeCRDT.Update + ActualPropagateSyncMsg + update_digest per
// submitted UpdateMessage on `cpu_ops` ops after `cpu_warm` untimed ones, one thread (the reference's
// per-request path).  Parity: a second GPU store built from the oracle's own Guids runs the same sample and its
// results, UpdateMessages (order, identities, payload bytes) and digests must equal the oracle's (exit 1).
// Prints one JSON object.
#include <array>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <unordered_map>
#include <vector>

#include "digest.hpp"
#include "host_pool.hpp"
#include "janus_host.hpp"
#include "oracle.hpp"
#include "wire.hpp"

namespace {

double now_s() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
janus::Guid G(const oracle::Guid& g) { return janus::Guid{g.lo, g.hi}; }

struct Op {
    uint32_t k;
    int op;          // PNC 1 Increment; OR-Set 1 Add, 3 Clear
    int64_t amount;  // PNC
    std::string elem;
    bool safe;
    uint64_t origin;
};

const char kChars[] = "abcdefghijklmnorqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789";  // sic (BenchmarkWorload.cs:151)

// One wave of client ops as one node receives them.
std::vector<Op> make_ops(bool pnc, uint64_t keys, uint64_t n, std::mt19937_64& rng, std::vector<uint8_t>& fill) {
    std::vector<Op> ops;
    ops.reserve(n + n / 2);
    while (ops.size() < n) {
        const uint64_t origin = 1 + rng() % 3;  // the node's 3 client threads (12 threads round-robin over 4 servers)
        if (pnc) {
            const uint64_t r = rng() % 4, acct = rng() % keys;  // PickRandomOptionByRatio over [0.25, 0.25, 0.5]
            if (r == 0) continue;                                 // ViewBalance: no state shipped
            if (r == 1) { ops.push_back(Op{(uint32_t)acct, 1, (int64_t)(rng() % 1000), {}, false, origin}); continue; }  // Deposit
            if (rng() % 2 == 0) {                                 // Transfer: "d" safe, then "i" non-safe on the other
                const uint64_t other = rng() % keys;
                const int64_t amt = (int64_t)(rng() % 100);
                ops.push_back(Op{(uint32_t)acct, 1, amt, {}, true, origin});
                ops.push_back(Op{(uint32_t)other, 1, amt, {}, false, origin});
            } else {                                              // Withdraw: "gs", then "d" safe
                ops.push_back(Op{(uint32_t)acct, 1, (int64_t)(rng() % 100), {}, true, origin});
            }
        } else {
            const uint64_t k = rng() % keys;
            if (fill[k] >= 50) {  // ORSetWorkload.cs:37-50: a full set is Cleared (non-safe)
                fill[k] = 0;
                ops.push_back(Op{(uint32_t)k, 3, 0, {}, false, 0});
                continue;
            }
            std::string e(5, ' ');
            for (char& c : e) c = kChars[rng() % (sizeof kChars - 1)];
            ++fill[k];  // a repeated string adds a tag to an existing element: the count is an upper bound
            ops.push_back(Op{(uint32_t)k, 1, 0, std::move(e), rng() % 2 == 0, origin});
        }
    }
    return ops;
}

}  // namespace

int main(int argc, char** argv) {
    bool pnc = true;
    uint64_t keys = 1000000, ops_n = 1000000, cpu_ops = 50000, cpu_warm = UINT64_MAX;
    uint64_t bad_at = UINT64_MAX;  // test: the parity call is first made with op bad_at's method invalid
    int waves = 3, device = 0, batch = 1000;
    for (int i = 1; i < argc; ++i) {
        if (!std::strcmp(argv[i], "--workload") && i + 1 < argc) pnc = std::strcmp(argv[++i], "orset") != 0;
        else if (!std::strcmp(argv[i], "--keys") && i + 1 < argc) keys = std::strtoull(argv[++i], nullptr, 10);
        else if (!std::strcmp(argv[i], "--ops") && i + 1 < argc) ops_n = std::strtoull(argv[++i], nullptr, 10);
        else if (!std::strcmp(argv[i], "--cpu-ops") && i + 1 < argc) cpu_ops = std::strtoull(argv[++i], nullptr, 10);
        else if (!std::strcmp(argv[i], "--cpu-warm") && i + 1 < argc) cpu_warm = std::strtoull(argv[++i], nullptr, 10);
        else if (!std::strcmp(argv[i], "--waves") && i + 1 < argc) waves = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--bad-at") && i + 1 < argc) bad_at = std::strtoull(argv[++i], nullptr, 10);
        else if (!std::strcmp(argv[i], "--device") && i + 1 < argc) device = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--batch") && i + 1 < argc) batch = std::atoi(argv[++i]);
    }
    constexpr int kNodes = 4;
    const uint32_t R = kNodes + 1;
    std::mt19937_64 rng(0x4A414E5553ull + (pnc ? 0 : 1));
    // OR-Set states grow with the ops a set has seen (Clear at 50): the timed sample starts after `cpu_warm` untimed
    // ops (parity covers both), so its states are the size the full-size run's are (25 ops per set by default)
    if (cpu_warm == UINT64_MAX) cpu_warm = pnc ? 0 : 25 * keys;
    if (!cpu_ops) cpu_warm = 0;

    // ---- parity + CPU baseline on the sample: the oracle node and a GPU store built from its Guids ----
    std::vector<uint8_t> fill(keys, 0);
    std::vector<Op> sample;
    bool parity_ok = true;
    std::string parity_why;
    double cpu_s = 0;
    uint64_t cpu_n = 0, cpu_msgs = 0, cpu_bytes = 0;
    if (cpu_ops) {
        std::mt19937_64 srng(0x5EED0000ull + (pnc ? 0 : 1));
        std::vector<uint8_t> sfill(keys, 0);
        sample = make_ops(pnc, keys, cpu_warm + cpu_ops, srng, sfill);
        oracle::SafeCRDTManager node(batch, 77);
        node.nextSeq = 1;
        janus::GpuStableStore gp(device, (uint32_t)(pnc ? keys : 1), R, 4);
        gp.SetNextMessageSeq(1);
        std::vector<oracle::SafeCRDT*> sc(keys, nullptr);
        oracle::GuidGen other(5);
        janus::UpdateMessage warm;  // the other nodes' replicas, merged into the prospective copies first
        for (const Op& o : sample) {
            if (sc[o.k]) continue;
            const oracle::Guid uid = node.gen.next();
            sc[o.k] = &node.CreateSafeCRDT((pnc ? "acct" : "set") + std::to_string(o.k), pnc ? oracle::CrdtType::PNCounter : oracle::CrdtType::ORSet, uid);
            gp.CreateSafeCRDT(G(uid), pnc ? janus::CrdtType::PNCounter : janus::CrdtType::ORSet,
                              pnc ? G(sc[o.k]->pncProspective->pnc.replicaIdx()) : janus::Guid{});
            if (pnc) {
                oracle::PNCounterMsg<int32_t> m;
                janus::Guid g[kNodes];
                int64_t pv[kNodes], nv[kNodes];
                g[0] = G(sc[o.k]->pncProspective->pnc.replicaIdx());
                pv[0] = nv[0] = 0;
                m.pVector[sc[o.k]->pncProspective->pnc.replicaIdx()] = 0;
                m.nVector[sc[o.k]->pncProspective->pnc.replicaIdx()] = 0;
                for (int j = 1; j < kNodes; ++j) {
                    const oracle::Guid x = other.next();
                    const int32_t v = (int32_t)(other.next().lo % 100000);
                    m.pVector[x] = v;
                    m.nVector[x] = 0;
                    g[j] = G(x);
                    pv[j] = v;
                    nv[j] = 0;
                }
                sc[o.k]->pncProspective->pnc.ApplySynchronizedUpdate(m);
                janus::NetworkProtocol np;
                np.uid = G(uid);
                janus::wire::AppendPNCounterMsg(np.message, g, pv, nv, kNodes);
                warm.update.push_back(std::move(np));
            }
        }
        if (!warm.update.empty()) gp.ReceivedBlock({warm});
        // GPU side of the sample (untimed; its time is the full-size run's)
        std::vector<janus::ClientUpdate> ups;
        std::vector<oracle::Guid> tags;
        {
            oracle::GuidGen peek = node.gen;  // the Guid.NewGuid() each Add draws, in op order
            for (const Op& o : sample) {
                janus::ClientUpdate c;
                c.op.uid = G(sc[o.k]->guid);
                c.op.opId = o.op;
                c.op.amount = o.amount;
                if (!pnc && o.op == 1) {
                    c.op.elem = o.elem;
                    c.op.tag = G(peek.next());
                }
                c.isSafe = o.safe;
                c.origin = o.origin;
                ups.push_back(std::move(c));
            }
        }
        janus::SafeUpdateTracker gt(gp.ctx());
        std::vector<janus::UpdateMessage> gsub;
        if (bad_at < ups.size()) {
            // SafeCRDT.Update's wrapper throws on an unknown method (PNCounterWrapper.cs:46, ORSetWrapper.cs): the call
            // must raise with nothing applied and nothing queued, however many of its chunks reached the device first
            std::vector<janus::Guid> all;
            for (uint64_t k = 0; k < keys; ++k)
                if (sc[k] && pnc) all.push_back(G(sc[k]->guid));
            const auto before = gp.EncodePNCStates(all);
            const int saved = ups[bad_at].op.opId;
            ups[bad_at].op.opId = 9;
            bool threw = false;
            try {
                gp.SubmitClientUpdates(ups, batch, gsub, gt);
            } catch (const janus::EngineError&) {
                threw = true;
            }
            ups[bad_at].op.opId = saved;
            if (!threw) parity_ok = false, parity_why = "an invalid method did not raise";
            else if (!gsub.empty() || gt.size() != 0) parity_ok = false, parity_why = "a raising call submitted or tracked messages";
            else if (gp.EncodePNCStates(all) != before) parity_ok = false, parity_why = "a raising call left applied ops in the store";
        }
        const auto gres = gp.SubmitClientUpdates(ups, batch, gsub, gt);
        // the oracle, timed: Update per op (ApplyOp + full-state Encode + the batcher), then ComputeDigest of every
        // UpdateMessage it submitted
        std::vector<uint8_t> ores;
        ores.reserve(sample.size());
        double c0 = now_s();
        size_t u_timed = 0;  // the UpdateMessages submitted from the timed ops on
        for (size_t i = 0; i < sample.size(); ++i) {
            if (i == cpu_warm) c0 = now_s(), u_timed = node.submitted.size();
            const Op& o = sample[i];
            const std::vector<oracle::Arg> a{pnc ? oracle::Arg::I(o.amount) : oracle::Arg::S(o.elem)};
            const auto r = o.op == 3 ? sc[o.k]->Update(3, {}, false, 0) : sc[o.k]->Update(o.op, a, o.safe, o.origin);
            ores.push_back(r.b ? 1 : 0);
        }
        std::vector<std::array<uint8_t, 32>> odig(node.submitted.size());
        for (size_t u = u_timed; u < node.submitted.size(); ++u) {
            std::vector<const uint8_t*> ptr;
            std::vector<uint64_t> len;
            for (const auto& np : node.submitted[u].update) {
                ptr.push_back(reinterpret_cast<const uint8_t*>(np.bytes.data()));
                len.push_back(np.bytes.size());
                cpu_bytes += np.bytes.size();
            }
            oracle::update_digest(ptr.size(), ptr.data(), len.data(), nullptr, odig[u].data());
            cpu_msgs += ptr.size();
        }
        cpu_s = now_s() - c0;
        cpu_n = sample.size() - cpu_warm;
        for (size_t u = 0; u < u_timed; ++u) {  // the warm-up's digests, untimed, for the parity check
            std::vector<const uint8_t*> ptr;
            std::vector<uint64_t> len;
            for (const auto& np : node.submitted[u].update) ptr.push_back(reinterpret_cast<const uint8_t*>(np.bytes.data())), len.push_back(np.bytes.size());
            oracle::update_digest(ptr.size(), ptr.data(), len.data(), nullptr, odig[u].data());
        }
        // parity: results, the submitted UpdateMessages (the oracle batches flushed on size only, like the GPU's
        // call: no 100 ms rule in either), identities, payload bytes and digests
        if (gres != ores) parity_ok = false, parity_why = "op results";  // the warm-up's and the timed ops'
        else if (gsub.size() != node.submitted.size()) parity_ok = false, parity_why = "number of UpdateMessages";
        for (size_t u = 0; parity_ok && u < gsub.size(); ++u) {
            const auto& a = gsub[u].update;
            const auto& b = node.submitted[u].update;
            if (a.size() != b.size()) { parity_ok = false, parity_why = "UpdateMessage size"; break; }
            for (size_t j = 0; j < a.size(); ++j)
                if (!(a[j].uid == G(b[j].uid)) || a[j].seq != b[j].seq || a[j].message != b[j].bytes) {
                    parity_ok = false, parity_why = "message identity / payload bytes";
                    break;
                }
            if (parity_ok && std::memcmp(gsub[u].digest.data(), odig[u].data(), 32) != 0) parity_ok = false, parity_why = "UpdateMessage digest";
        }
    }

    // ---- the full-size GPU run ----
    oracle::GuidGen gen(9);
    janus::GpuStableStore gpu(device, (uint32_t)(pnc ? keys : 1), R, 4);
    std::vector<janus::Guid> uid(keys);
    {
        janus::UpdateMessage warm;
        for (uint64_t k = 0; k < keys; ++k) {
            uid[k] = G(gen.next());
            const janus::Guid own = G(gen.next());
            gpu.CreateSafeCRDT(uid[k], pnc ? janus::CrdtType::PNCounter : janus::CrdtType::ORSet, pnc ? own : janus::Guid{});
            if (pnc) {
                janus::Guid g[kNodes] = {own};
                int64_t pv[kNodes] = {0}, nv[kNodes] = {0};
                for (int j = 1; j < kNodes; ++j) g[j] = G(gen.next()), pv[j] = (int64_t)(gen.next().lo % 100000);
                janus::NetworkProtocol np;
                np.uid = uid[k];
                janus::wire::AppendPNCounterMsg(np.message, g, pv, nv, kNodes);
                warm.update.push_back(std::move(np));
            }
        }
        if (!warm.update.empty()) gpu.ReceivedBlock({warm});
    }
    janus::SafeUpdateTracker tracker(gpu.ctx());
    double gpu_s = 0;
    std::vector<double> wave_ms;
    uint64_t gpu_n = 0, n_msgs = 0, n_um = 0, n_bytes = 0;
    for (int w = 0; w < waves + 1; ++w) {  // wave 0 = warmup
        const auto ops = make_ops(pnc, keys, ops_n, rng, fill);
        std::vector<janus::ClientUpdate> ups;
        ups.reserve(ops.size());
        for (const Op& o : ops) {
            janus::ClientUpdate c;
            c.op.uid = uid[o.k];
            c.op.opId = o.op;
            c.op.amount = o.amount;
            if (!pnc && o.op == 1) {
                c.op.elem = o.elem;
                c.op.tag = G(gen.next());
            }
            c.isSafe = o.safe;
            c.origin = o.origin;
            ups.push_back(std::move(c));
        }
        std::vector<janus::UpdateMessage> sub;
        const double t0 = now_s();
        gpu.SubmitClientUpdates(ups, batch, sub, tracker);
        const double t1 = now_s();
        if (w == 0) continue;
        gpu_s += t1 - t0;
        wave_ms.push_back(1e3 * (t1 - t0));
        gpu_n += ops.size();
        n_um += sub.size();
        for (const auto& um : sub) {
            n_msgs += um.update.size();
            for (const auto& np : um.update) n_bytes += np.message.size();
        }
    }
    const double W = waves;
    std::string wl;
    for (double x : wave_ms) wl += (wl.empty() ? "" : ", ") + std::to_string(x).substr(0, 6);
    std::vector<double> sorted_ms = wave_ms;
    std::sort(sorted_ms.begin(), sorted_ms.end());
    const double med = sorted_ms.empty() ? 0.0 : sorted_ms[sorted_ms.size() / 2];
    std::printf("{\"workload\": \"producer path (SafeCRDT.Update + full-state Encode + ActualPropagateSyncMsg + ComputeDigest) of one node: %s, "
                "%llu keys, clientBatchSize %d, %llu client ops per call\", \"waves\": %d, \"ops_per_s\": %.1f, \"ms_per_wave\": %.3f, \"ms_per_wave_median\": %.3f, \"wave_ms\": [%s], "
                "\"submitted_msgs_per_wave\": %.1f, \"update_messages_per_wave\": %.1f, \"payload_bytes_per_msg\": %.1f, \"host_threads\": %d, "
                "\"parity_vs_oracle\": %s, \"parity_sample_ops\": %llu, \"parity_failure\": \"%s\", "
                "\"cpu_baseline\": {\"ops_per_s\": %.1f, \"msgs_per_s\": %.1f, \"payload_bytes_per_msg\": %.1f, \"cores\": 1, \"kind\": \"port\", "
                "\"sample\": \"oracle SafeCRDT.Update (ApplyOp + GetLastSynchronizedUpdate().Encode()) + ActualPropagateSyncMsg + update_digest "
                "per submitted UpdateMessage over %llu ops after %llu untimed ones\"}}\n",
                pnc ? "C5 banking client ops (deposit / transfer / withdraw as Increments, 4-replica states)"
                    : "ORSetWorkload client ops (Add of random 5-char strings, Clear at 50 elements)",
                (unsigned long long)keys, batch, (unsigned long long)ops_n, waves, gpu_n / gpu_s, 1e3 * gpu_s / W, med, wl.c_str(), n_msgs / W, n_um / W,
                n_msgs ? (double)n_bytes / n_msgs : 0.0, jg::host_threads(), parity_ok ? "true" : "false", (unsigned long long)cpu_n,
                parity_why.c_str(), cpu_s > 0 ? cpu_n / cpu_s : 0.0, cpu_s > 0 ? cpu_msgs / cpu_s : 0.0, cpu_msgs ? (double)cpu_bytes / cpu_msgs : 0.0,
                (unsigned long long)cpu_n, (unsigned long long)cpu_warm);
    return parity_ok ? 0 : 1;
}
