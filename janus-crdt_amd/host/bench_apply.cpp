// bench_apply.cpp — committed-batch apply loop of the banking replay.
//
// Client side, restated from the reference's banking benchmark: BankingBenchmarkRunner.cs:135-163 picks
// an op by opsRatio (benchmark_config_example.json: [0.25 view, 0.25 deposit, 0.5 transfer-or-withdraw])
// and an account (uniform, or N(n/2, n/6) clamped: :208-226); BankingWorload.cs turns each into
//   View      "gp"                                            -> no state shipped          (:30-60)
//   Deposit   "i"  Next(1000), non-safe                      -> 1 state                  (:62-92)
//   Transfer  "d"  Next(100) safe on the account, then "i" non-safe on the other account
//                                                            -> 2 states                 (:94-133)
//   Withdraw  "gs" read, then "d" Next(100) safe             -> 1 state                  (:156-203)
// and every "d" is Update(1, ...) = Increment (PNCounterCommand.cs:48-50): N columns stay 0.
// Node side: each client thread talks to one server (:64-79, threads round-robin over servers); the
// node applies the op to its prospective copy and ships the FULL state (SafeCRDT.cs:39-62: the node's
// own counter plus the other nodes' counters it merged; here every node has seen every other node's
// latest value), and its batcher ActualPropagateSyncMsg (SafeCRDTManager.cs:165-198, clientBatchSize
// 1000, JanusService.cs:29) keeps safe states individually and compacts non-safe ones to the last state
// per account; the 100 ms timer flushes every queue at the end of a wave.  100 UpdateMessages per block
// (DAG.cs:25).  A wave is `ops` client ops (1M: BASELINE configs[4]).
//
// GPU: janus::GpuStableStore::ApplyCommitted = the wave flattened into the jg_commit arrays (the C# caller's
// share) + ONE jg_apply_committed (the library: gather into pinned staging, uid lookup, safe-update tracker,
// decode, replica interning and merge; csrc/node.hip).
// CPU baseline: the oracle's SafeCRDTManager.HandleAfterConsensusUpdates (Decode + Merge per message,
// one thread like the reference's serialized apply task) on the first `cpu_msgs` messages of each wave.
// --parity: the oracle applies EVERY wave in full; after each wave every owned account's stable Get and
// the safe-update completions (origins, in commit order) must equal the oracle's (exit 1 otherwise).
// Prints one JSON object.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <unordered_map>

#include "host_pool.hpp"
#include "janus_host.hpp"
#include "oracle.hpp"
#include "wire.hpp"

namespace {

double now_s() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

}  // namespace

int main(int argc, char** argv) {
    uint64_t accounts = 1000000, ops = 1000000, cpu_msgs = 100000;
    int waves = 3, nodes = 4, device = 0, batch = 1000, threads_per_node = 3;  // 12 client threads (config example)
    uint32_t rank = 0, world = 1;
    bool normal = false, parity = false, direct = false, arena = false, stream = false, stream_cached = false;
    size_t part_msgs = 65536;
    for (int i = 1; i < argc; ++i) {
        if (!std::strcmp(argv[i], "--accounts") && i + 1 < argc) accounts = std::strtoull(argv[++i], nullptr, 10);
        else if (!std::strcmp(argv[i], "--ops") && i + 1 < argc) ops = std::strtoull(argv[++i], nullptr, 10);
        else if (!std::strcmp(argv[i], "--cpu-msgs") && i + 1 < argc) cpu_msgs = std::strtoull(argv[++i], nullptr, 10);
        else if (!std::strcmp(argv[i], "--waves") && i + 1 < argc) waves = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--normal")) normal = true;
        else if (!std::strcmp(argv[i], "--parity")) parity = true;
        else if (!std::strcmp(argv[i], "--direct")) direct = true;  // the wave received into page-locked memory
        else if (!std::strcmp(argv[i], "--arena")) direct = arena = true;  // the caller copies the wave into page-locked memory (timed)
        else if (!std::strcmp(argv[i], "--arena-stream")) stream = true;  // the same copy part by part, overlapped (jg_apply_stream_*)
        else if (!std::strcmp(argv[i], "--arena-stream-cached")) stream = true, stream_cached = true;  // ... with plain cached copies
        else if (!std::strcmp(argv[i], "--part-msgs") && i + 1 < argc) part_msgs = std::strtoull(argv[++i], nullptr, 10);
        else if (!std::strcmp(argv[i], "--device") && i + 1 < argc) device = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--rank") && i + 1 < argc) rank = (uint32_t)std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--world") && i + 1 < argc) world = (uint32_t)std::atoi(argv[++i]);
    }
    const uint32_t R = nodes + 1;  // the stable copy's own replica + one prospective replica per node
    std::mt19937_64 rng(0x4A414E5553ull);
    oracle::GuidGen gen(7);
    auto G = [](const oracle::Guid& g) { return janus::Guid{g.lo, g.hi}; };

    // accounts: key uid, stable replica Guid (column 0), per-node prospective replica Guids
    std::vector<oracle::Guid> uid(accounts), stable(accounts), rep(accounts * nodes);
    for (uint64_t k = 0; k < accounts; ++k) {
        uid[k] = gen.next();
        stable[k] = gen.next();
        for (int n = 0; n < nodes; ++n) rep[k * nodes + n] = gen.next();
    }
    janus::GpuStableStore gpu(device, (uint32_t)accounts, R, 4);
    gpu.SetShard(rank, world);  // non-owned states skipped from the uid alone
    // key-space shard of this rank (every rank sees the whole wave and skips the uids it does not own)
    std::vector<uint8_t> mine(accounts);
    uint64_t owned = 0;
    for (uint64_t k = 0; k < accounts; ++k) {
        mine[k] = janus::GpuStableStore::ShardOf(G(uid[k]), world) == rank;
        if (mine[k]) { gpu.CreateSafeCRDT(G(uid[k]), janus::CrdtType::PNCounter, G(stable[k])); ++owned; }
    }
    const bool run_cpu = parity || cpu_msgs > 0;
    oracle::SafeCRDTManager cpu(batch, 1);
    std::vector<oracle::SafeCRDT*> cref(accounts, nullptr);
    if (run_cpu)
        for (uint64_t k = 0; k < accounts; ++k)
            if (mine[k]) {
                oracle::SafeCRDT& sc = cpu.CreateSafeCRDT("acct" + std::to_string(k), oracle::CrdtType::PNCounter, uid[k]);
                sc.pncStable->pnc = oracle::PNCounter<int32_t>(stable[k]);  // the stable instance's own replica (column 0)
                cref[k] = &sc;
            }

    std::vector<int32_t> P(accounts * nodes, 0), N(accounts * nodes, 0);  // N stays 0: "d" is Increment
    std::normal_distribution<double> nd(accounts / 2.0, accounts / 6.0);
    auto account = [&]() -> uint64_t {  // GetRandomAccount (BankingBenchmarkRunner.cs:208-226)
        if (!normal) return rng() % accounts;
        const double x = std::round(nd(rng));
        return (uint64_t)std::max(0.0, std::min(x, (double)accounts - 1));
    };
    struct Queued { janus::NetworkProtocol np; bool safe; };
    std::vector<std::vector<Queued>> q(nodes);
    janus::SafeUpdateTracker tracker_g(gpu.ctx());       // safe-update tracker: seq -> client origin (GPU node, on the device)
    std::unordered_map<uint64_t, uint64_t> tracker_c;    // the oracle node's
    uint64_t seq = 1;

    double gpu_s = 0, cpu_s = 0, flat_s = 0, gather_s = 0, wait_s = 0, lib_s = 0, busy_s = 0, chunk_s = 0, setup_s = 0, loop_s = 0, pack_s = 0;
    uint64_t gpu_n = 0, cpu_n = 0, payload_timed = 0, up_bytes = 0, up_msgs = 0, applied = 0, n_safe = 0, n_states = 0, n_done = 0;
    std::vector<uint64_t> done_buf;  // the direct legs' completion buffer, reused
    bool ok = true;
    std::string why;
    for (int w = 0; w < waves + 1 && ok; ++w) {  // wave 0 = warmup
        std::vector<janus::UpdateMessage> ums;
        auto flush = [&](int n) {  // ActualPropagateSyncMsg's drain (SafeCRDTManager.cs:170-196)
            std::vector<janus::NetworkProtocol> safe, appeared;
            std::unordered_map<janus::Guid, size_t, janus::GuidHash> pos;
            size_t at = 0;
            for (; at < q[n].size(); ++at) {
                if (!((int)safe.size() < batch)) { ++at; break; }  // dequeued, then dropped (:175)
                Queued& e = q[n][at];
                if (!e.safe) {
                    auto it = pos.find(e.np.uid);
                    if (it == pos.end()) { pos.emplace(e.np.uid, appeared.size()); appeared.push_back(std::move(e.np)); }
                    else appeared[it->second] = std::move(e.np);
                } else {
                    safe.push_back(std::move(e.np));
                }
            }
            q[n].erase(q[n].begin(), q[n].begin() + (long)at);
            for (auto& a : appeared) safe.push_back(std::move(a));
            if (!safe.empty()) ums.push_back(janus::UpdateMessage{std::move(safe)});
        };
        // SafeCRDT.Update on node n: Increment its own column, ship the full state, queue it
        auto update = [&](int n, uint64_t k, int32_t amt, bool safe, uint64_t origin) {
            P[k * nodes + n] += amt;
            janus::NetworkProtocol np;
            np.uid = G(uid[k]);
            np.seq = seq++;
            janus::Guid g[16];
            int64_t pv[16], nv[16];
            for (int j = 0; j < nodes; ++j) { g[j] = G(rep[k * nodes + j]); pv[j] = P[k * nodes + j]; nv[j] = N[k * nodes + j]; }
            janus::wire::AppendPNCounterMsg(np.message, g, pv, nv, nodes);
            if (safe) {  // SafeCRDT.cs:55-56: tracked when safe and the origin is a client
                tracker_g.add(np.seq, origin);
                tracker_c[np.seq] = origin;
                if (w > 0) ++n_safe;
            }
            if (w > 0) ++n_states;
            q[n].push_back(Queued{std::move(np), safe});
            if ((int)q[n].size() >= batch) flush(n);
        };
        for (uint64_t o = 0; o < ops; ++o) {
            const int thread = (int)(rng() % (uint64_t)(nodes * threads_per_node));
            const int n = thread % nodes;                  // client thread i talks to server i mod nodes
            const uint64_t origin = 1 + (uint64_t)thread;  // the client connection notified on completion
            const uint64_t r = rng() % 4;                  // PickRandomOptionByRatio over [0.25, 0.25, 0.5]
            const uint64_t acct = account();
            if (r == 0) continue;                                                        // ViewBalance: "gp"
            if (r == 1) { update(n, acct, (int32_t)(rng() % 1000), false, origin); continue; }  // Deposit: "i"
            if (rng() % 2 == 0) {                                                        // Transfer
                const uint64_t other = account();
                const int32_t amt = (int32_t)(rng() % 100);
                update(n, acct, amt, true, origin);                                      // "d" safe (= Increment)
                update(n, other, amt, false, origin);                                    // then "i" non-safe
            } else {
                update(n, acct, (int32_t)(rng() % 100), true, origin);                   // Withdraw: "gs", then "d" safe
            }
        }
        for (int n = 0; n < nodes; ++n) flush(n);  // the 100 ms timer at the end of the wave
        std::vector<std::vector<janus::UpdateMessage>> wave(1);
        uint64_t wave_msgs = 0, wave_payload = 0;
        for (auto& um : ums) {
            wave_msgs += um.update.size();
            for (const auto& np : um.update) wave_payload += np.message.size();
            if (wave.back().size() == 100) wave.emplace_back();
            wave.back().push_back(std::move(um));
        }
        // the oracle's copy of the wave (all of it for parity, else the first cpu_msgs messages)
        std::vector<std::vector<oracle::UpdateMessage>> cwave;
        if (run_cpu && w > 0) {
            uint64_t left = parity ? UINT64_MAX : cpu_msgs;
            for (const auto& blk : wave) {
                if (!left) break;
                cwave.emplace_back();
                for (const auto& um : blk) {
                    if (!left) break;
                    oracle::UpdateMessage cu;
                    for (const auto& np : um.update) {
                        if (!left) break;
                        oracle::NetworkProtocol cp;
                        cp.uid = oracle::Guid{np.uid.lo, np.uid.hi};
                        cp.seq = np.seq;
                        cp.bytes = np.message;  // decoded by the stable copy's codec (oracle/json.hpp)
                        cu.update.push_back(std::move(cp));
                        --left;
                    }
                    cwave.back().push_back(std::move(cu));
                }
            }
        }
        // --direct: the wave as a transport receiving its blocks into jg_host_alloc memory would hold it (laid
        // out untimed: that copy is the receive path's), applied by the library's in-place upload
        // --arena: a C# caller without page-locked receive buffers copies each committed byte[] into a jg_host_alloc
        // arena itself (parallel Span.CopyTo = plain cached copies), timed as the caller's cost
        const double tp = now_s();
        if (direct) gpu.PackCommitted(wave, !arena);
        const double t0 = arena ? tp : now_s();
        if (direct && w > 0) pack_s += now_s() - tp;
        // (the direct legs hand the library a reused completion buffer, as a C# caller passes its own array)
        std::vector<uint64_t> done;
        size_t k_done = 0;
        const bool into = !stream;  // (the streamed arena keeps its vector form)
        if (direct) k_done = gpu.ApplyPackedInto(&tracker_g, done_buf);
        else if (!stream) k_done = gpu.ApplyCommittedInto(wave, &tracker_g, done_buf);
        else done = gpu.ApplyArenaStreamed(wave, &tracker_g, part_msgs, !stream_cached), k_done = done.size();
        const double t1 = now_s();
        if (w == 0) {
            if (parity) {  // the warmup wave reaches the oracle too (untimed), so states stay in step
                std::vector<std::vector<oracle::UpdateMessage>> all;
                for (const auto& blk : wave) {
                    all.emplace_back();
                    for (const auto& um : blk) {
                        oracle::UpdateMessage cu;
                        for (const auto& np : um.update) {
                            oracle::NetworkProtocol cp;
                            cp.uid = oracle::Guid{np.uid.lo, np.uid.hi};
                            cp.seq = np.seq;
                            cp.bytes = np.message;
                            cu.update.push_back(std::move(cp));
                        }
                        all.back().push_back(std::move(cu));
                    }
                }
                cpu.safeUpdateTracker = tracker_c;
                cpu.notified.clear();
                cpu.HandleAfterConsensusUpdates(all);
                tracker_c = cpu.safeUpdateTracker;
            }
            continue;
        }
        gpu_s += t1 - t0;
        const jg_apply_stats& st = gpu.last_apply_stats();
        flat_s += gpu.last_flatten_s();
        gather_s += st.gather_s;
        wait_s += st.device_wait_s;
        lib_s += st.total_s;
        busy_s += st.device_busy_s;
        chunk_s += st.chunk_busy_s;
        setup_s += st.setup_s;
        loop_s += st.loop_s;
        up_bytes += st.bytes_uploaded;
        up_msgs += st.msgs_uploaded;
        applied += st.msgs_applied;  // counted by the library: states that reached a registered key
        gpu_n += wave_msgs;
        payload_timed += wave_payload;
        n_done += k_done;
        if (!run_cpu) continue;
        cpu.safeUpdateTracker = tracker_c;
        cpu.notified.clear();
        const double c0 = now_s();
        cpu.HandleAfterConsensusUpdates(cwave);
        cpu_s += now_s() - c0;
        tracker_c = cpu.safeUpdateTracker;
        uint64_t cn = 0;
        for (const auto& blk : cwave)
            for (const auto& um : blk) cn += um.update.size();
        cpu_n += cn;
        if (!parity) continue;
        // every owned account's stable Get, and the completions in commit order (unowned uids are
        // skipped on both sides, SafeCRDTManager.cs:136)
        const bool same_done = into ? k_done == cpu.notified.size() && std::equal(cpu.notified.begin(), cpu.notified.end(), done_buf.begin())
                                    : done == cpu.notified;
        if (!same_done) { ok = false; why = "safe-update completions differ"; }
        for (uint64_t k = 0; k < accounts && ok; ++k) {
            if (!mine[k]) continue;
            if (gpu.QueryStablePNC(G(uid[k])) != cref[k]->QueryStable().i) { ok = false; why = "account " + std::to_string(k) + " differs"; }
        }
    }
    if (parity) {
        std::printf("{\"parity\": %s, \"why\": \"%s\", \"waves\": %d, \"msgs_per_wave\": %.1f, \"safe_per_wave\": %.1f, \"completed_per_wave\": %.1f, "
                    "\"owned_accounts\": %llu}\n",
                    ok ? "true" : "false", why.c_str(), waves, (double)gpu_n / waves, (double)n_safe / waves, (double)n_done / waves,
                    (unsigned long long)owned);
        return ok ? 0 : 1;
    }
    const double W = waves;
    if (arena) flat_s = pack_s;  // the caller's copy into the arena is its flatten (inside ms_per_wave)
    // per uploaded message the library moves its payload, 8 B offset, 16 B uid, 8 B identity, 1 B type
    const double pcie_bytes = (double)up_bytes + 33.0 * (double)up_msgs;
    std::printf("{\"workload\": \"C5 banking replay (BankingWorload.cs ops: view/deposit/transfer/withdraw at opsRatio [0.25, 0.25, 0.5], "
                "every d an Increment; %s accounts %llu; %d nodes, clientBatchSize %d with state compaction; committed waves of %llu client ops)\", "
                "\"waves\": %d, \"direct\": %s, \"arena\": %s, \"stream\": %s, \"untimed_pack_ms_per_wave\": %.3f, \"msgs_per_s\": %.1f, \"client_ops_per_s\": %.1f, \"ms_per_wave\": %.3f, \"state_msgs_per_wave\": %.1f, "
                "\"client_states_per_wave\": %.1f, \"safe_states_per_wave\": %.1f, \"completed_per_wave\": %.1f, \"payload_bytes_per_msg\": %.1f, "
                "\"caller_flatten_ms_per_wave\": %.3f, \"library_ms_per_wave\": %.3f, \"gather_ms_per_wave\": %.3f, "
                "\"device_wait_ms_per_wave\": %.3f, \"device_busy_ms_per_wave\": %.3f, \"chunk_busy_ms_per_wave\": %.3f, \"setup_ms_per_wave\": %.3f, \"loop_ms_per_wave\": %.3f, \"host_ms_per_wave\": %.3f, "
                "\"uploaded_msgs_per_wave\": %.1f, \"uploaded_bytes_per_wave\": %.1f, \"pcie_GBps\": %.2f, \"engine_payload_GBps\": %.2f, "
                "\"host_threads\": %d, \"rank\": %u, \"world\": %u, \"owned_accounts\": %llu, \"applied_msgs_per_wave\": %.1f, "
                "\"cpu_baseline\": {\"msgs_per_s\": %.1f, \"sample_msgs_per_wave\": %.1f, \"cores\": 1, \"kind\": \"port\", "
                "\"sample\": \"oracle HandleAfterConsensusUpdates: Decode (System.Text.Json restatement) + PNCounter.Merge per message\"}}\n",
                normal ? "normal" : "uniform", (unsigned long long)accounts, nodes, batch, (unsigned long long)ops, waves, direct ? "true" : "false", (arena || stream) ? "true" : "false", stream ? "true" : "false", arena ? 0.0 : 1e3 * pack_s / W, gpu_n / gpu_s,
                (double)ops * waves / gpu_s, 1e3 * gpu_s / W, (double)gpu_n / W, (double)n_states / W, (double)n_safe / W, (double)n_done / W,
                (double)payload_timed / std::max<uint64_t>(gpu_n, 1), 1e3 * flat_s / W, 1e3 * lib_s / W, 1e3 * gather_s / W, 1e3 * wait_s / W,
                1e3 * busy_s / W, 1e3 * chunk_s / W, 1e3 * setup_s / W, 1e3 * loop_s / W, 1e3 * (flat_s + gather_s) / W, (double)up_msgs / W, pcie_bytes / W, pcie_bytes / lib_s / 1e9,
                (double)up_bytes / std::max(busy_s, 1e-12) / 1e9, jg::host_threads(), rank, world, (unsigned long long)owned,
                (double)applied / W, cpu_s > 0 ? cpu_n / cpu_s : 0.0, (double)cpu_n / W);
    return 0;
}
