// bench_c1.cpp — BASELINE.json configs[0] (C1): the reference's own PN-Counter benchmark shape as
// committed waves through the apply loop, GPU host mirror against the oracle on the same waves.
//
// Client side, restated from BFT-CRDT-Client/WorkloadGenerator/PNCWorkload.cs:32-92 with
// benchmark_config_example.json:1-9 (100 objects, opsRatio [0.25, 0.25, 0.5], safeRatio 0.5, 4 servers):
// keys round-robin from a random start, increments and "decrements" of Next(1, 100) — both reach
// Update(1, ...) = Increment (PNCounterCommand.cs:42-51) — and reads, which ship no state.
// Node side: every update ships the node's full PNCounter state (SafeCRDT.cs:49), and the node's
// batcher ActualPropagateSyncMsg (SafeCRDTManager.cs:165-198, clientBatchSize 1000, JanusService.cs:29)
// keeps safe states individually and compacts the non-safe ones to the last state per key; the
// 100 ms timer flushes every queue at the end of a wave.  100 UpdateMessages per block (DAG.cs:25).
// With 100 hot keys, every key takes thousands of states per wave (SURVEY.md §7 "hot-key contention").
// Prints one JSON object, including an exact check of every key's stable value against the oracle.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <unordered_map>

#include "janus_host.hpp"
#include "oracle.hpp"
#include "wire.hpp"

namespace {
double now_s() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
}  // namespace

int main(int argc, char** argv) {
    bool direct = false;
    uint64_t keys = 100, updates = 1000000;
    int waves = 3, nodes = 4, device = 0, batch = 1000;
    bool cpu = true;
    for (int i = 1; i < argc; ++i) {
        if (!std::strcmp(argv[i], "--keys") && i + 1 < argc) keys = std::strtoull(argv[++i], nullptr, 10);
        else if (!std::strcmp(argv[i], "--ops") && i + 1 < argc) updates = std::strtoull(argv[++i], nullptr, 10);
        else if (!std::strcmp(argv[i], "--waves") && i + 1 < argc) waves = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--device") && i + 1 < argc) device = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--no-cpu")) cpu = false;
        else if (!std::strcmp(argv[i], "--direct")) direct = true;  // the wave received into page-locked memory
    }
    std::mt19937_64 rng(0x4A414E5553ull);
    oracle::GuidGen gen(3);
    auto G = [](const oracle::Guid& g) { return janus::Guid{g.lo, g.hi}; };
    std::vector<oracle::Guid> uid(keys), stable(keys), rep(keys * nodes);
    for (uint64_t k = 0; k < keys; ++k) {
        uid[k] = gen.next();
        stable[k] = gen.next();
        for (int n = 0; n < nodes; ++n) rep[k * nodes + n] = gen.next();
    }
    janus::GpuStableStore gpu(device, (uint32_t)keys, nodes + 1, 4);
    oracle::SafeCRDTManager orc(batch, 1);
    for (uint64_t k = 0; k < keys; ++k) {
        gpu.CreateSafeCRDT(G(uid[k]), janus::CrdtType::PNCounter, G(stable[k]));
        orc.CreateSafeCRDT("key" + std::to_string(k), oracle::CrdtType::PNCounter, uid[k]);
    }
    std::vector<int32_t> P(keys * nodes, 0), N(keys * nodes, 0);
    std::vector<uint64_t> key_loc(nodes);
    for (auto& l : key_loc) l = rng() % keys;
    struct Queued { janus::NetworkProtocol np; bool safe; };
    std::vector<std::vector<Queued>> q(nodes);
    uint64_t seq = 1;

    double gpu_s = 0, cpu_s = 0, up_bytes = 0, busy_s = 0, gather_s = 0, chunk_s = 0, setup_s = 0, loop_s = 0, wait_s = 0, lib_s = 0;
    uint64_t n_msgs = 0, n_updates = 0, n_ops = 0;
    for (int w = 0; w < waves + 1; ++w) {  // wave 0 = warmup
        std::vector<janus::UpdateMessage> ums;
        // ActualPropagateSyncMsg's drain (SafeCRDTManager.cs:170-196)
        auto flush = [&](int n) {
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
        uint64_t wave_updates = 0;
        for (uint64_t o = 0; o < updates; ++o) {
            const int n = (int)(rng() % nodes);
            const uint64_t k = key_loc[n];
            key_loc[n] = (k + 1) % keys;
            const uint64_t r = rng() % 4;            // opsRatio [0.25, 0.25, 0.5]
            const int32_t amt = 1 + (int32_t)(rng() % 99);  // Random.Next(1, 100)
            const bool safe = (rng() & 1) != 0;      // safeRatio 0.5
            if (r >= 2) continue;                    // "gp": a read ships no state
            ++wave_updates;
            P[k * nodes + n] += amt;                 // "i" and "d" are both Increment
            janus::NetworkProtocol np;
            np.uid = G(uid[k]);
            np.seq = seq++;
            janus::Guid g[16];
            int64_t pv[16], nv[16];
            for (int j = 0; j < nodes; ++j) { g[j] = G(rep[k * nodes + j]); pv[j] = P[k * nodes + j]; nv[j] = N[k * nodes + j]; }
            janus::wire::AppendPNCounterMsg(np.message, g, pv, nv, nodes);
            q[n].push_back(Queued{std::move(np), safe});
            if ((int)q[n].size() >= batch) flush(n);
        }
        for (int n = 0; n < nodes; ++n) flush(n);    // the 100 ms timer at the end of the wave
        std::vector<std::vector<janus::UpdateMessage>> wave(1);
        uint64_t wave_msgs = 0;
        for (auto& um : ums) {
            wave_msgs += um.update.size();
            if (wave.back().size() == 100) wave.emplace_back();
            wave.back().push_back(std::move(um));
        }
        std::vector<std::vector<oracle::UpdateMessage>> cwave;
        if (cpu) {
            for (const auto& blk : wave) {
                cwave.emplace_back();
                for (const auto& um : blk) {
                    oracle::UpdateMessage cu;
                    for (const auto& np : um.update) {
                        oracle::NetworkProtocol cp;
                        cp.uid = oracle::Guid{np.uid.lo, np.uid.hi};
                        cp.seq = np.seq;
                        cp.bytes = np.message;
                        cu.update.push_back(std::move(cp));
                    }
                    cwave.back().push_back(std::move(cu));
                }
            }
        }
        if (direct) gpu.PackCommitted(wave);  // untimed: the layout a receive-into-jg_host_alloc transport leaves
        const double t0 = now_s();
        if (direct) gpu.ApplyPacked(nullptr);
        else gpu.ApplyCommitted(wave, nullptr);
        const double t1 = now_s();
        if (cpu) orc.HandleAfterConsensusUpdates(cwave);
        const double t2 = now_s();
        if (w == 0) continue;
        const jg_apply_stats& st = gpu.last_apply_stats();
        up_bytes += (double)st.bytes_uploaded;
        busy_s += st.device_busy_s;
        chunk_s += st.chunk_busy_s;
        setup_s += st.setup_s;
        loop_s += st.loop_s;
        wait_s += st.device_wait_s;
        lib_s += st.total_s;
        gather_s += st.gather_s;
        gpu_s += t1 - t0;
        cpu_s += t2 - t1;
        n_msgs += wave_msgs;
        n_updates += wave_updates;
        n_ops += updates;
    }
    // every key's stable value (PNCounter.Get) against the oracle, exactly
    bool parity = true;
    if (cpu)
        for (uint64_t k = 0; k < keys; ++k)
            parity &= gpu.QueryStablePNC(G(uid[k])) == orc.safeCRDTs.at("key" + std::to_string(k))->QueryStable().i;
    std::printf("{\"workload\": \"C1: PNCWorkload-shaped client ops (%llu keys round-robin, opsRatio [0.25, 0.25, 0.5], safeRatio 0.5, "
                "Next(1,100)), %d nodes, clientBatchSize %d with state compaction, committed waves of %llu client ops\", \"waves\": %d, \"direct\": %s, "
                "\"state_msgs_per_wave\": %.1f, \"client_updates_per_wave\": %.1f, \"msgs_per_s\": %.1f, \"client_ops_per_s\": %.1f, "
                "\"ms_per_wave\": %.3f, \"uploaded_bytes_per_wave\": %.1f, \"device_busy_ms_per_wave\": %.3f, \"chunk_busy_ms_per_wave\": %.3f, \"library_ms_per_wave\": %.3f, \"setup_ms_per_wave\": %.3f, \"loop_ms_per_wave\": %.3f, \"device_wait_ms_per_wave\": %.3f, \"gather_ms_per_wave\": %.3f, "
                "\"parity_vs_oracle\": %s, \"cpu_baseline\": {\"msgs_per_s\": %.1f, \"client_ops_per_s\": %.1f, "
                "\"ms_per_wave\": %.3f, \"cores\": 1, \"kind\": \"port\", \"sample\": \"oracle HandleAfterConsensusUpdates on the same waves\"}}\n",
                (unsigned long long)keys, nodes, batch, (unsigned long long)updates, waves, direct ? "true" : "false", (double)n_msgs / waves, (double)n_updates / waves,
                n_msgs / gpu_s, n_ops / gpu_s, 1e3 * gpu_s / waves, up_bytes / waves, 1e3 * busy_s / waves, 1e3 * chunk_s / waves, 1e3 * lib_s / waves, 1e3 * setup_s / waves, 1e3 * loop_s / waves, 1e3 * wait_s / waves, 1e3 * gather_s / waves, cpu ? (parity ? "true" : "false") : "null", cpu ? n_msgs / cpu_s : 0.0,
                cpu ? n_ops / cpu_s : 0.0, cpu ? 1e3 * cpu_s / waves : 0.0);
    return parity ? 0 : 1;
}
