// bench_apply.cpp — committed-batch apply loop throughput.
//
// Synthetic DAG-committed waves shaped like the reference's banking workload
// (BFT-CRDT-Client/BankingBenchmark.cs/BankingBenchmarkRunner.cs:135-163, BankingWorload.cs): 4 nodes,
// PN-Counter accounts, every client update ships the FULL state of its account as seen by its node
// (SafeCRDT.cs:52), packed clientBatchSize = 1000 states per UpdateMessage (JanusService.cs:29) and
// 100 UpdateMessages per block (DAG.cs:25).  A wave holds `msgs` state messages.
//
// Every state travels as the reference ships it: NetworkProtocol.message = PNCounterMsg JSON
// (SafeCRDT.cs:49, PNCounters.cs:46-49).
// GPU: janus::GpuStableStore::ApplyCommitted (classify + gather the payloads into pinned staging +
// ONE jg_pnc_merge_json: decode, replica interning and merge on the device).  CPU baseline: the
// oracle's SafeCRDTManager.HandleAfterConsensusUpdates (dictionary-faithful restatement of
// SafeCRDTManager.cs:109-160: Decode + Merge per message, one thread like the reference's serialized
// apply task) on the first `cpu_msgs` messages of the same wave.
// Prints one JSON object.
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>

#include "janus_host.hpp"
#include "oracle.hpp"
#include "wire.hpp"

namespace {

double now_s() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

struct Wave {
    std::vector<std::vector<janus::UpdateMessage>> gpu;
    std::vector<std::vector<oracle::UpdateMessage>> cpu;  // first cpu_msgs messages only
    uint64_t n = 0;
};

}  // namespace

int main(int argc, char** argv) {
    uint64_t accounts = 1000000, msgs = 1000000, cpu_msgs = 100000;
    int waves = 5, nodes = 4, device = 0;
    uint32_t rank = 0, world = 1;
    bool normal = false;
    for (int i = 1; i < argc; ++i) {
        if (!std::strcmp(argv[i], "--accounts") && i + 1 < argc) accounts = std::strtoull(argv[++i], nullptr, 10);
        else if (!std::strcmp(argv[i], "--msgs") && i + 1 < argc) msgs = std::strtoull(argv[++i], nullptr, 10);
        else if (!std::strcmp(argv[i], "--cpu-msgs") && i + 1 < argc) cpu_msgs = std::strtoull(argv[++i], nullptr, 10);
        else if (!std::strcmp(argv[i], "--waves") && i + 1 < argc) waves = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--normal")) normal = true;
        else if (!std::strcmp(argv[i], "--device") && i + 1 < argc) device = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--rank") && i + 1 < argc) rank = (uint32_t)std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--world") && i + 1 < argc) world = (uint32_t)std::atoi(argv[++i]);
    }
    const uint32_t R = nodes + 1;  // the stable copy's own replica + one prospective replica per node
    std::mt19937_64 rng(0x4A414E5553ull);
    oracle::GuidGen gen(7);

    // accounts: key uid, per-node prospective replica Guids, stable replica Guid
    std::vector<oracle::Guid> uid(accounts), stable(accounts), rep(accounts * nodes);
    for (uint64_t k = 0; k < accounts; ++k) {
        uid[k] = gen.next();
        stable[k] = gen.next();
        for (int n = 0; n < nodes; ++n) rep[k * nodes + n] = gen.next();
    }
    janus::GpuStableStore gpu(device, (uint32_t)accounts, R, 4);
    auto G = [](const oracle::Guid& g) { return janus::Guid{g.lo, g.hi}; };
    // key-space shard of this rank (every rank sees the whole wave and skips the uids it does not own)
    std::vector<uint8_t> mine(accounts);
    uint64_t owned = 0;
    for (uint64_t k = 0; k < accounts; ++k) {
        mine[k] = janus::GpuStableStore::ShardOf(G(uid[k]), world) == rank;
        if (mine[k]) { gpu.CreateSafeCRDT(G(uid[k]), janus::CrdtType::PNCounter, G(stable[k])); ++owned; }
    }
    uint64_t applied = 0;
    oracle::SafeCRDTManager cpu(1000, 1);
    if (cpu_msgs)
        for (uint64_t k = 0; k < accounts; ++k) cpu.CreateSafeCRDT("acct" + std::to_string(k), oracle::CrdtType::PNCounter, uid[k]);

    // per (account, node) counters: a node's state of an account = its own P/N plus what it merged
    std::vector<int32_t> P(accounts * nodes, 0), N(accounts * nodes, 0);
    std::normal_distribution<double> nd(accounts / 2.0, accounts / 6.0);
    auto pick = [&]() -> uint64_t {
        if (!normal) return rng() % accounts;
        const double x = std::round(nd(rng));
        return (uint64_t)std::max(0.0, std::min(x, (double)accounts - 1));
    };

    double gpu_s = 0, host_s = 0, engine_s = 0, cpu_s = 0, ph[4] = {0, 0, 0, 0};
    uint64_t gpu_n = 0, cpu_n = 0, payload = 0, payload_timed = 0, shard_bytes = 0;
    for (int w = 0; w < waves + 1; ++w) {  // wave 0 = warmup
        Wave wave;
        std::vector<janus::UpdateMessage> block;
        std::vector<oracle::UpdateMessage> cblock;
        janus::UpdateMessage um;
        oracle::UpdateMessage cum;
        for (uint64_t m = 0; m < msgs; ++m) {
            const uint64_t k = pick();
            const int n = (int)(rng() % nodes);
            const uint64_t op = rng() % 4;  // view / deposit / transfer / withdraw (BankingBenchmarkRunner.cs:140-160)
            const int32_t amt = (int32_t)(op == 1 ? rng() % 1000 : rng() % 100);
            if (op == 0) { --m; continue; }           // a read ships no state
            P[k * nodes + n] += amt;                   // "i" and "d" are both Increment (PNCounterCommand.cs:42-51)
            if (rng() % 8 == 0) N[k * nodes + n] += amt / 3;
            janus::NetworkProtocol np;
            np.uid = G(uid[k]);
            np.seq = m;
            {   // the node's full state: every replica it has seen, encoded (GetLastSynchronizedUpdate().Encode())
                janus::Guid g[16];
                int64_t pv[16], nv[16];
                for (int j = 0; j < nodes; ++j) { g[j] = G(rep[k * nodes + j]); pv[j] = P[k * nodes + j]; nv[j] = N[k * nodes + j]; }
                janus::wire::AppendPNCounterMsg(np.message, g, pv, nv, nodes);
            }
            payload += np.message.size();
            if (w > 0 && mine[k]) ++applied;
            if (m < cpu_msgs && w > 0) {
                oracle::NetworkProtocol cp;
                cp.uid = uid[k];
                cp.seq = m;
                cp.bytes = np.message;  // the oracle decodes it in ApplyUpdateStable (oracle/json.hpp)
                cum.update.push_back(std::move(cp));
                if (cum.update.size() == 1000) { cblock.push_back(std::move(cum)); cum = oracle::UpdateMessage(); }
                if (cblock.size() == 100) { wave.cpu.push_back(std::move(cblock)); cblock.clear(); }
            }
            um.update.push_back(std::move(np));
            if (um.update.size() == 1000) { block.push_back(std::move(um)); um = janus::UpdateMessage(); }
            if (block.size() == 100) { wave.gpu.push_back(std::move(block)); block.clear(); }
        }
        if (!um.update.empty()) block.push_back(std::move(um));
        if (!block.empty()) wave.gpu.push_back(std::move(block));
        if (!cum.update.empty()) cblock.push_back(std::move(cum));
        if (!cblock.empty()) wave.cpu.push_back(std::move(cblock));

        const uint64_t wave_payload = payload;
        payload = 0;
        const double t0 = now_s();
        gpu.ApplyCommitted(wave.gpu, nullptr);
        const double t1 = now_s();
        if (w > 0) {
            gpu_s += t1 - t0;
            host_s += gpu.last_apply_host_s();
            engine_s += gpu.last_apply_engine_s();
            for (int q = 0; q < 4; ++q) ph[q] += gpu.last_apply_phases_s()[q];
            gpu_n += msgs;
            payload_timed += wave_payload;
            shard_bytes += gpu.last_apply_pnc_bytes();
            if (!cpu_msgs) continue;
            const double c0 = now_s();
            cpu.HandleAfterConsensusUpdates(wave.cpu);
            cpu_s += now_s() - c0;
            cpu_n += std::min(msgs, cpu_msgs);
        }
    }
    const double bytes = (double)payload_timed;  // JSON payload bytes uploaded and decoded
    std::printf("{\"workload\": \"committed-batch apply (C5 banking-shaped, %s accounts %llu, %d nodes, %llu PNCounterMsg JSON states per wave)\", "
                "\"waves\": %d, \"msgs_per_s\": %.1f, \"ms_per_wave\": %.3f, \"payload_bytes_per_msg\": %.1f, \"host_ms_per_wave\": %.3f, "
                "\"engine_ms_per_wave\": %.3f, \"engine_msgs_per_s\": %.1f, \"engine_payload_GBps\": %.2f, \"host_threads\": %d, \"host_phase_ms\": [%.2f, %.2f, %.2f, %.2f], "
                "\"rank\": %u, \"world\": %u, \"owned_accounts\": %llu, \"applied_msgs_per_wave\": %.1f, "
                "\"cpu_baseline\": {\"msgs_per_s\": %.1f, \"sample_msgs_per_wave\": %llu, \"cores\": 1, \"kind\": \"port\", "
                "\"sample\": \"oracle HandleAfterConsensusUpdates: Decode (System.Text.Json restatement) + PNCounter.Merge per message\"}}\n",
                normal ? "normal" : "uniform", (unsigned long long)accounts, nodes, (unsigned long long)msgs, waves, gpu_n / gpu_s,
                1e3 * gpu_s / waves, bytes / gpu_n, 1e3 * host_s / waves, 1e3 * engine_s / waves, gpu_n / engine_s, shard_bytes / engine_s / 1e9,
                janus::GpuStableStore::host_threads(), 1e3 * ph[0] / waves, 1e3 * ph[1] / waves, 1e3 * ph[2] / waves, 1e3 * ph[3] / waves,
                rank, world, (unsigned long long)owned, (double)applied / waves, cpu_s > 0 ? cpu_n / cpu_s : 0.0,
                (unsigned long long)std::min(msgs, cpu_msgs));
    return 0;
}
