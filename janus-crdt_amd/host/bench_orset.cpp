// bench_orset.cpp — committed-batch apply loop for OR-Set states.
//
// Workload after the reference's OR-Set generator (BFT-CRDT-Client/WorkloadGenerator/ORSetWorkload.cs):
// every update Adds a random 5-character string (GenerateRandomString, BenchmarkWorkload.cs:149-154)
// with a fresh Guid tag (ORSet.cs:134-153); a set holding 50 elements is Cleared instead (non-safe,
// ORSetWorkload.cs:37-50).  4 nodes; each update ships the adding node's FULL state as the reference
// does (NetworkProtocol.message = ORSetMsg JSON, SafeCRDT.cs:49, ORSet.cs:56-69), 1000 states per
// UpdateMessage (JanusService.cs:29), 100 UpdateMessages per block (DAG.cs:25).
// GPU: janus::GpuStableStore::ApplyCommitted (host decode + element interning + ONE jg_orset_merge).
// CPU baseline: the oracle's HandleAfterConsensusUpdates (Decode + ORSet.Merge per message, one
// thread) on the first `cpu_msgs` messages of each wave.  Prints one JSON object.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "host_pool.hpp"
#include "janus_host.hpp"
#include "oracle.hpp"
#include "wire.hpp"

namespace {
double now_s() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
}  // namespace

int main(int argc, char** argv) {
    bool direct = false;
    uint64_t sets = 100000, msgs = 200000, cpu_msgs = 20000;
    int waves = 3, nodes = 4, device = 0;
    uint32_t rank = 0, world = 1;
    for (int i = 1; i < argc; ++i) {
        if (!std::strcmp(argv[i], "--sets") && i + 1 < argc) sets = std::strtoull(argv[++i], nullptr, 10);
        else if (!std::strcmp(argv[i], "--msgs") && i + 1 < argc) msgs = std::strtoull(argv[++i], nullptr, 10);
        else if (!std::strcmp(argv[i], "--cpu-msgs") && i + 1 < argc) cpu_msgs = std::strtoull(argv[++i], nullptr, 10);
        else if (!std::strcmp(argv[i], "--waves") && i + 1 < argc) waves = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--device") && i + 1 < argc) device = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--rank") && i + 1 < argc) rank = (uint32_t)std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--world") && i + 1 < argc) world = (uint32_t)std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--direct")) direct = true;  // the wave received into page-locked memory
    }
    std::mt19937_64 rng(0x4A414E5553ull);
    oracle::GuidGen gen(11);
    auto G = [](const oracle::Guid& g) { return janus::Guid{g.lo, g.hi}; };
    std::vector<oracle::Guid> uid(sets);
    for (auto& u : uid) u = gen.next();
    janus::GpuStableStore gpu(device, 1, 1, 4);
    gpu.SetShard(rank, world);  // non-owned states skipped from the uid alone
    std::vector<uint8_t> mine(sets);
    uint64_t owned = 0;
    for (uint64_t k = 0; k < sets; ++k) {
        mine[k] = janus::GpuStableStore::ShardOf(G(uid[k]), world) == rank;
        if (mine[k]) { gpu.CreateSafeCRDT(G(uid[k]), janus::CrdtType::ORSet); ++owned; }
    }
    oracle::SafeCRDTManager cpu(1000, 1);
    if (cpu_msgs)
        for (uint64_t k = 0; k < sets; ++k) cpu.CreateSafeCRDT("set" + std::to_string(k), oracle::CrdtType::ORSet, uid[k]);

    static const char chars[] = "abcdefghijklmnorqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789";  // sic (BenchmarkWorkload.cs:151)
    // per (set, node): the node's elements since its last Clear, one tag each
    std::vector<janus::ORSetState> st(sets * nodes);
    double gpu_s = 0, cpu_s = 0, flat_s = 0, gather_s = 0, wait_s = 0, lib_s = 0, busy_s = 0, chunk_s = 0, setup_s = 0, loop_s = 0;
    uint64_t up_bytes = 0, up_msgs = 0, applied = 0;
    uint64_t gpu_n = 0, cpu_n = 0, payload = 0, recs = 0;
    const int warm = 2;  // warm-up waves: the staging buffers reach their size, the tables their load
    for (int w = 0; w < waves + warm; ++w) {
        std::vector<std::vector<janus::UpdateMessage>> wave;
        std::vector<std::vector<oracle::UpdateMessage>> cwave;
        std::vector<janus::UpdateMessage> block;
        std::vector<oracle::UpdateMessage> cblock;
        janus::UpdateMessage um;
        oracle::UpdateMessage cum;
        uint64_t wave_payload = 0, wave_recs = 0;
        for (uint64_t m = 0; m < msgs; ++m) {
            const uint64_t k = rng() % sets;
            const int n = (int)(rng() % nodes);
            janus::ORSetState& s = st[k * nodes + n];
            if (s.addSet.size() == 50) {
                s = janus::ORSetState();  // Clear (ORSet.cs:192-198)
            } else {
                std::string e(5, ' ');
                for (char& c : e) c = chars[rng() % (sizeof chars - 1)];
                const oracle::Guid t = gen.next();
                bool found = false;
                for (auto& kv : s.addSet)
                    if (kv.first == e) { kv.second.push_back(G(t)); found = true; break; }
                if (!found) s.addSet.emplace_back(e, std::vector<janus::Guid>{G(t)});
            }
            janus::NetworkProtocol np;
            np.uid = G(uid[k]);
            np.seq = m;
            np.message = janus::wire::EncodeORSetMsg(s);
            wave_payload += np.message.size();
            for (const auto& kv : s.addSet) wave_recs += kv.second.size();
            if (m < cpu_msgs && w >= warm) {
                oracle::NetworkProtocol cp;
                cp.uid = uid[k];
                cp.seq = m;
                cp.bytes = np.message;
                cum.update.push_back(std::move(cp));
                if (cum.update.size() == 1000) { cblock.push_back(std::move(cum)); cum = oracle::UpdateMessage(); }
                if (cblock.size() == 100) { cwave.push_back(std::move(cblock)); cblock.clear(); }
            }
            um.update.push_back(std::move(np));
            if (um.update.size() == 1000) { block.push_back(std::move(um)); um = janus::UpdateMessage(); }
            if (block.size() == 100) { wave.push_back(std::move(block)); block.clear(); }
        }
        if (!um.update.empty()) block.push_back(std::move(um));
        if (!block.empty()) wave.push_back(std::move(block));
        if (!cum.update.empty()) cblock.push_back(std::move(cum));
        if (!cblock.empty()) cwave.push_back(std::move(cblock));

        if (direct) gpu.PackCommitted(wave);  // untimed: the layout a receive-into-jg_host_alloc transport leaves
        const double t0 = now_s();
        if (direct) gpu.ApplyPacked(nullptr);
        else gpu.ApplyCommitted(wave, nullptr);
        const double t1 = now_s();
        if (w < warm) continue;
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
        applied += st.msgs_applied;
        gpu_n += msgs;
        payload += wave_payload;
        recs += wave_recs;
        if (!cpu_msgs) continue;
        const double c0 = now_s();
        cpu.HandleAfterConsensusUpdates(cwave);
        cpu_s += now_s() - c0;
        cpu_n += std::min(msgs, cpu_msgs);
    }
    const double W = waves;
    const double pcie_bytes = (double)up_bytes + 33.0 * (double)up_msgs;
    std::printf("{\"workload\": \"committed-batch apply (OR-Set, ORSetWorkload-shaped: random 5-char adds, Clear at 50, %llu sets, %d nodes, "
                "%llu ORSetMsg JSON states per wave)\", \"waves\": %d, \"direct\": %s, \"msgs_per_s\": %.1f, \"ms_per_wave\": %.3f, \"payload_bytes_per_msg\": %.1f, "
                "\"tag_records_per_msg\": %.2f, \"caller_flatten_ms_per_wave\": %.3f, \"library_ms_per_wave\": %.3f, \"gather_ms_per_wave\": %.3f, "
                "\"device_wait_ms_per_wave\": %.3f, \"device_busy_ms_per_wave\": %.3f, \"chunk_busy_ms_per_wave\": %.3f, \"setup_ms_per_wave\": %.3f, \"loop_ms_per_wave\": %.3f, \"host_ms_per_wave\": %.3f, "
                "\"uploaded_msgs_per_wave\": %.1f, \"uploaded_bytes_per_wave\": %.1f, \"pcie_GBps\": %.2f, \"engine_payload_GBps\": %.2f, "
                "\"host_threads\": %d, \"rank\": %u, \"world\": %u, \"owned_sets\": %llu, \"applied_msgs_per_wave\": %.1f, "
                "\"cpu_baseline\": {\"msgs_per_s\": %.1f, \"sample_msgs_per_wave\": %llu, \"cores\": 1, "
                "\"kind\": \"port\", \"sample\": \"oracle HandleAfterConsensusUpdates: Decode (System.Text.Json restatement) + ORSet.Merge per message\"}}\n",
                (unsigned long long)sets, nodes, (unsigned long long)msgs, waves, direct ? "true" : "false", gpu_n / gpu_s, 1e3 * gpu_s / W, (double)payload / gpu_n,
                (double)recs / gpu_n, 1e3 * flat_s / W, 1e3 * lib_s / W, 1e3 * gather_s / W, 1e3 * wait_s / W, 1e3 * busy_s / W,
                1e3 * chunk_s / W, 1e3 * setup_s / W, 1e3 * loop_s / W, 1e3 * (flat_s + gather_s) / W, (double)up_msgs / W, pcie_bytes / W, pcie_bytes / lib_s / 1e9,
                (double)up_bytes / std::max(busy_s, 1e-12) / 1e9, jg::host_threads(), rank, world, (unsigned long long)owned, (double)applied / W,
                cpu_s > 0 ? cpu_n / cpu_s : 0.0, (unsigned long long)std::min(msgs, cpu_msgs));
    return 0;
}
