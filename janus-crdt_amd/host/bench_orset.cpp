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

#include "janus_host.hpp"
#include "oracle.hpp"
#include "wire.hpp"

namespace {
double now_s() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
}  // namespace

int main(int argc, char** argv) {
    uint64_t sets = 100000, msgs = 200000, cpu_msgs = 20000;
    bool probe = false;
    int waves = 3, nodes = 4, device = 0;
    uint32_t rank = 0, world = 1;
    for (int i = 1; i < argc; ++i) {
        if (!std::strcmp(argv[i], "--sets") && i + 1 < argc) sets = std::strtoull(argv[++i], nullptr, 10);
        else if (!std::strcmp(argv[i], "--msgs") && i + 1 < argc) msgs = std::strtoull(argv[++i], nullptr, 10);
        else if (!std::strcmp(argv[i], "--cpu-msgs") && i + 1 < argc) cpu_msgs = std::strtoull(argv[++i], nullptr, 10);
        else if (!std::strcmp(argv[i], "--probe-copy")) probe = true;
        else if (!std::strcmp(argv[i], "--waves") && i + 1 < argc) waves = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--device") && i + 1 < argc) device = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--rank") && i + 1 < argc) rank = (uint32_t)std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--world") && i + 1 < argc) world = (uint32_t)std::atoi(argv[++i]);
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
    double gpu_s = 0, host_s = 0, engine_s = 0, cpu_s = 0, oph[3] = {0, 0, 0}, hph[4] = {0, 0, 0, 0};
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

        if (probe) {  // host copy rate of this wave's payloads (diagnostic)
            std::vector<const std::string*> ps;
            for (auto& b : wave)
                for (auto& u : b)
                    for (auto& np : u.update) ps.push_back(&np.message);
            std::vector<char> dst(wave_payload + 64);
            jg_ctx* pctx = nullptr;
            void* pinned = nullptr;
            jg_open(device, &pctx);
            jg_host_alloc(pctx, wave_payload + 64, &pinned);
            for (int T : {1, 4, 16, -16}) {
                const double a = now_s();
                std::vector<std::thread> th;
                char* out = T < 0 ? static_cast<char*>(pinned) : dst.data();
                const int TT = T < 0 ? -T : T;
                for (int t = 0; t < TT; ++t)
                    th.emplace_back([&, t, TT, out] {
                        const size_t b = ps.size() * t / TT, e = ps.size() * (t + 1) / TT;
                        size_t o = 0;
                        for (size_t i = 0; i < b; ++i) o += ps[i]->size();
                        for (size_t i = b; i < e; ++i) { std::memcpy(out + o, ps[i]->data(), ps[i]->size()); o += ps[i]->size(); }
                    });
                for (auto& x : th) x.join();
                std::fprintf(stderr, "probe wave %d threads %d%s: %.2f ms (%.1f GB/s)\n", w, TT, T < 0 ? " pinned" : "", 1e3 * (now_s() - a),
                             wave_payload / (now_s() - a) / 1e9);
            }
            jg_host_free(pinned);
            jg_close(pctx);
        }
        const double t0 = now_s();
        gpu.ApplyCommitted(wave, nullptr);
        const double t1 = now_s();
        if (w < warm) continue;
        gpu_s += t1 - t0;
        host_s += gpu.last_apply_host_s();
        engine_s += gpu.last_apply_engine_s();
        for (int q = 0; q < 3; ++q) oph[q] += gpu.last_apply_orset_phases_s()[q];
        for (int q = 0; q < 4; ++q) hph[q] += gpu.last_apply_phases_s()[q];
        gpu_n += msgs;
        payload += wave_payload;
        recs += wave_recs;
        if (!cpu_msgs) continue;
        const double c0 = now_s();
        cpu.HandleAfterConsensusUpdates(cwave);
        cpu_s += now_s() - c0;
        cpu_n += std::min(msgs, cpu_msgs);
    }
    std::printf("{\"workload\": \"committed-batch apply (OR-Set, ORSetWorkload-shaped: random 5-char adds, Clear at 50, %llu sets, %d nodes, "
                "%llu ORSetMsg JSON states per wave)\", \"waves\": %d, \"msgs_per_s\": %.1f, \"ms_per_wave\": %.3f, \"payload_bytes_per_msg\": %.1f, "
                "\"tag_records_per_msg\": %.2f, \"host_ms_per_wave\": %.3f, \"engine_ms_per_wave\": %.3f, "
                "\"orset_ms_per_wave\": {\"validate\": %.3f, \"commit\": %.3f, \"host_names\": %.3f}, \"host_phase_ms\": [%.2f, %.2f, %.2f, %.2f], "
                "\"host_threads\": %d, \"rank\": %u, "
                "\"world\": %u, \"owned_sets\": %llu, \"cpu_baseline\": {\"msgs_per_s\": %.1f, \"sample_msgs_per_wave\": %llu, \"cores\": 1, "
                "\"kind\": \"port\", \"sample\": \"oracle HandleAfterConsensusUpdates: Decode (System.Text.Json restatement) + ORSet.Merge per message\"}}\n",
                (unsigned long long)sets, nodes, (unsigned long long)msgs, waves, gpu_n / gpu_s, 1e3 * gpu_s / waves, (double)payload / gpu_n,
                (double)recs / gpu_n, 1e3 * host_s / waves, 1e3 * engine_s / waves, 1e3 * oph[0] / waves, 1e3 * oph[1] / waves, 1e3 * oph[2] / waves, 1e3 * hph[0] / waves, 1e3 * hph[1] / waves,
                1e3 * hph[2] / waves, 1e3 * hph[3] / waves,
                janus::GpuStableStore::host_threads(), rank, world,
                (unsigned long long)owned, cpu_s > 0 ? cpu_n / cpu_s : 0.0, (unsigned long long)std::min(msgs, cpu_msgs));
    return 0;
}
