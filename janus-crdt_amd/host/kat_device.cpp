// kat_device.cpp — the reference's known-answer tests replayed ON THE DEVICE through the C ABI.
//
// Every deterministic scenario of MergeSharp.Tests/PNCounterTests.cs and ORSetTests.cs (transcribed
// against the oracle in oracle/test_kat.cpp) runs here with each CRDT object as one key of a
// janus::GpuStableStore, i.e. through exactly the calls a C# wrapper makes:
//   ORSet.Add / Remove / Clear, PNCounter.Increment / Decrement -> GpuStableStore::ApplyOps
//                                                                 -> jg_orset_apply_ops / jg_pnc_apply_ops
//   GetLastSynchronizedUpdate().Encode()  -> EncodeORSetStates / EncodePNCStates
//                                            (jg_orset_read_sets / jg_pnc_encode_json)
//   ApplySynchronizedUpdate(Decode(bytes)) -> ReceivedBlock (ReplicationManager.ReceivedUpdateSyncMsg's
//                                            path: jg_orset_wave_* / jg_pnc_wave_*)
//   LookupAll / Contains / Count / Get    -> jg_orset_lookup_all / jg_orset_contains / jg_pnc_values
// and asserts the reference's literal expected values, including its order-sensitive asserts
// (ORSetTests.cs:113, 144, 327, 343, 346, 473: Assert.Equal on enumerations) and the null-element
// cases (:277-448).  The payloads a scenario ships are also checked byte for byte against the oracle's
// encoder run through the same scenario (the reference's System.Text.Json bytes, oracle/json.hpp).
// Exit 0 = every scenario passes; prints "PASS name" / "FAIL name: why".
#include <cstdio>
#include <functional>
#include <optional>
#include <sstream>
#include <string>
#include <vector>

#include "janus_host.hpp"
#include "json.hpp"
#include "oracle.hpp"

namespace {

using E = std::optional<std::string>;
using L = std::vector<E>;
const E NUL = std::nullopt;
E S(const char* s) { return E(std::string(s)); }
E I(int i) { return E(std::to_string(i)); }

struct Failure : std::runtime_error { using std::runtime_error::runtime_error; };
#define CHECK(cond) do { if (!(cond)) throw Failure(std::to_string(__LINE__) + ": CHECK(" #cond ")"); } while (0)

std::string show(const L& l) {
    std::string o = "[";
    for (const E& e : l) o += (o.size() > 1 ? "," : "") + (e ? *e : std::string("null"));
    return o + "]";
}
#define CHECK_LIST(got, ...) do { const L g_ = (got), w_ = L{__VA_ARGS__}; \
    if (g_ != w_) throw Failure(std::to_string(__LINE__) + ": " + show(g_) + " != " + show(w_)); } while (0)
L sorted(L v) { std::sort(v.begin(), v.end()); return v; }

std::vector<std::pair<std::string, std::function<void()>>>& registry() { static std::vector<std::pair<std::string, std::function<void()>>> r; return r; }
struct Reg { Reg(const char* n, std::function<void()> f) { registry().emplace_back(n, std::move(f)); } };
#define TEST(name) static void name(); static Reg reg_##name(#name, name); static void name()

// One device store holds every object of every scenario (each object = one key, never reused).
janus::GpuStableStore* g_store = nullptr;
oracle::GuidGen g_gen(0xD3C1CE);
uint64_t g_uid = 1;

janus::Guid fresh() {
    const oracle::Guid g = g_gen.next();
    return janus::Guid{g.lo, g.hi};
}

// Ship `bytes` (an encoded state) to `uid`: one received block holding one NetworkProtocol.
void deliver(const janus::Guid& uid, const std::string& bytes) {
    janus::UpdateMessage um;
    janus::NetworkProtocol np;
    np.uid = uid;
    np.syncMsgType = janus::NetworkProtocol::CRDTMsg;
    np.message = bytes;
    um.update.push_back(std::move(np));
    g_store->ReceivedBlock({um});
}

// ORSet<string?> on the device, mirrored by an oracle ORSet run through the same ops (the bytes each
// GetLastSynchronizedUpdate ships must be the oracle's, byte for byte).
struct DevORSet {
    janus::Guid uid{g_uid++, 0x0512};
    oracle::ORSet mirror;
    DevORSet() { g_store->CreateSafeCRDT(uid, janus::CrdtType::ORSet); }
    bool op(int id, const E& e) {
        janus::ClientOp o;
        o.uid = uid;
        o.opId = id;
        o.elem = e;
        o.tag = fresh();
        bool want = true;
        if (id == 1) mirror.AddTag(e, oracle::Guid{o.tag.lo, o.tag.hi});
        else if (id == 2) want = mirror.Remove(e);
        else mirror.Clear();
        const bool got = g_store->ApplyOps({o})[0] != 0;
        if (got != want) throw Failure("op result differs from the oracle's");
        return got;
    }
    bool Add(const E& e) { return op(1, e); }
    bool Remove(const E& e) { return op(2, e); }
    void Clear() { op(3, NUL); }
    L LookupAll() const { return g_store->QueryStableLookupAll(uid); }
    bool Contains(const E& e) const { return g_store->QueryStableORSet(uid, e); }
    size_t Count() const { return LookupAll().size(); }
    std::string Msg() const {  // GetLastSynchronizedUpdate().Encode()
        const std::string got = g_store->EncodeORSetStates({uid})[0];
        const std::string want = oracle::json::EncodeORSet(mirror.GetLastSynchronizedUpdate());
        if (got != want) throw Failure("encoded state differs from the reference's bytes:\n  got  " + got + "\n  want " + want);
        return got;
    }
    void Apply(const DevORSet& other) {  // ApplySynchronizedUpdate(other.GetLastSynchronizedUpdate())
        const std::string b = other.Msg();
        deliver(uid, b);
        mirror.ApplySynchronizedUpdate(oracle::json::DecodeORSet(b));
    }
};

struct DevPNC {
    janus::Guid uid{g_uid++, 0x0F1C};
    janus::Guid self = fresh();
    oracle::PNCounter<int32_t> mirror{oracle::Guid{self.lo, self.hi}};
    DevPNC() { g_store->CreateSafeCRDT(uid, janus::CrdtType::PNCounter, self); }
    void op(int id, int32_t v) {
        janus::ClientOp o;
        o.uid = uid;
        o.opId = id;
        o.amount = v;
        g_store->ApplyOps({o});
        if (id == 1) mirror.Increment(v);
        else mirror.Decrement(v);
    }
    void Increment(int32_t v) { op(1, v); }
    void Decrement(int32_t v) { op(2, v); }
    int64_t Get() const { return g_store->QueryStablePNC(uid); }
    std::string Msg() const {
        const std::string got = g_store->EncodePNCStates({uid})[0];
        const std::string want = oracle::json::EncodePNC(mirror.GetLastSynchronizedUpdate());
        if (got != want) throw Failure("encoded state differs from the reference's bytes:\n  got  " + got + "\n  want " + want);
        return got;
    }
    void Apply(const DevPNC& other) {
        const std::string b = other.Msg();
        deliver(uid, b);
        mirror.ApplySynchronizedUpdate(oracle::json::DecodePNC<int32_t>(b));
    }
};

bool overflows(const DevPNC& p) {
    try {
        p.Get();
    } catch (const janus::EngineError& e) {
        return e.code == JG_EOVERFLOW;
    }
    return false;
}

// ===================== MergeSharp.Tests/PNCounterTests.cs ====================================
TEST(PNCounterTests_TestPNCSingle) {  // PNCounterTests.cs:8-19
    DevPNC pnc;
    pnc.Increment(5); pnc.Decrement(8); pnc.Increment(10); pnc.Decrement(3);
    CHECK(pnc.Get() == 4);
}
TEST(PNCounterTests_TestPNCMerge) {  // PNCounterTests.cs:21-38
    DevPNC pnc1, pnc2;
    pnc1.Increment(5); pnc1.Decrement(8); pnc1.Increment(10); pnc1.Decrement(3);
    pnc2.Apply(pnc1);
    CHECK(pnc1.Get() == pnc2.Get());
    CHECK(pnc2.Get() == 4);
}
TEST(PNCounterMsgTests_EncodeDecode) {  // PNCounterTests.cs:46-66
    DevPNC pnc1, pnc2;
    pnc1.Increment(5); pnc1.Decrement(1);
    pnc2.Increment(2); pnc1.Decrement(2);
    pnc1.Apply(pnc2);
    CHECK(pnc1.Get() == 5 - 1 + 2 - 2);
}
TEST(PNCounter_AbsentLocalActsAsZero) {  // PNCounters.cs:131-144: TryGetValue -> 0, then Max(0, v) inserted
    DevPNC a, b;
    b.Increment(-7);  // a negative received entry: max(absent = 0, -7) = 0
    a.Apply(b);
    CHECK(a.Get() == 0);
    a.Msg();  // the inserted 0 column is shipped, as the reference's Dictionary holds it
}
TEST(PNCounter_IncrementWraps) {  // '+=' is unchecked (PNCounters.cs:99)
    DevPNC a;
    a.Increment(INT32_MAX); a.Increment(1);
    CHECK(a.Get() == INT32_MIN);
}
TEST(PNCounter_GetCheckedSumThrows) {  // LINQ Sum is checked (PNCounters.cs:89)
    DevPNC a, b;
    a.Increment(INT32_MAX); b.Increment(1);
    a.Apply(b);
    CHECK(overflows(a));
}
TEST(PNCounter_GetSubtractionWraps) {  // ΣP − ΣN is unchecked
    DevPNC a;
    a.Increment(INT32_MAX); a.Decrement(-1);
    CHECK(a.Get() == INT32_MIN);
}

// ===================== MergeSharp.Tests/ORSetTests.cs ========================================
TEST(ORSetTests_SingleORSetValueType1) {  // ORSetTests.cs:10-40
    DevORSet set;
    set.Add(I(1)); set.Add(I(2));
    CHECK(set.Remove(I(1)));
    CHECK(!set.Remove(I(3)));
    set.Add(I(3));
    CHECK(set.Count() == 2);
    CHECK_LIST(sorted(set.LookupAll()), I(2), I(3));
    set.Clear();
    CHECK(set.Count() == 0);
    CHECK_LIST(set.LookupAll());
    CHECK(!set.Contains(I(1)));
    set.Add(I(1));
    CHECK(set.Contains(I(1)));
    CHECK_LIST(set.LookupAll(), I(1));  // CopyTo(array, 2) -> {0, 0, 1}
    set.Msg();
}
TEST(ORSetTests_SingleORSetReferenceType) {  // ORSetTests.cs:56-81
    DevORSet set;
    set.Add(S("1")); set.Add(S("2"));
    CHECK(set.Remove(S("1")));
    CHECK(!set.Remove(S("3")));
    set.Add(S("3"));
    CHECK(set.Count() == 2);
    CHECK_LIST(sorted(set.LookupAll()), S("2"), S("3"));
    set.Clear();
    CHECK(set.Count() == 0);
    CHECK_LIST(set.LookupAll());
    CHECK(!set.Contains(S("1")));
    set.Add(S("1"));
    CHECK(set.Contains(S("1")));
}
TEST(ORSetTests_SingleORSetReferenceType2) {  // ORSetTests.cs:84-100
    DevORSet set;
    set.Add(S("1")); set.Add(S("1"));
    CHECK(set.Count() == 1);
    CHECK_LIST(set.LookupAll(), S("1"));
    set.Clear();
    set.Add(S(""));
    CHECK(set.Contains(S("")));
}
TEST(ORSetTests_Multiple) {  // ORSetTests.cs:102-129 (order-sensitive at :113)
    DevORSet set1, set2;
    set1.Add(I(1)); set2.Add(I(2));
    set1.Apply(set2);
    CHECK_LIST(set1.LookupAll(), I(1), I(2));
    CHECK(set1.Count() == 2);
    CHECK_LIST(set2.LookupAll(), I(2));
    set2.Apply(set1);
    CHECK(sorted(set1.LookupAll()) == sorted(set2.LookupAll()));
    set1.Remove(I(2));
    CHECK_LIST(set1.LookupAll(), I(1));
    CHECK(set1.Count() == 1);
    set1.Add(I(2));
    set2.Remove(I(2));
    set1.Apply(set2);
    CHECK_LIST(sorted(set1.LookupAll()), I(1), I(2));
    CHECK(set1.Count() == 2);
    set1.Msg();
    set2.Msg();
}
TEST(ORSetTests_Multiple2) {  // ORSetTests.cs:131-147 (order-sensitive at :144)
    DevORSet set1, set2;
    set1.Add(S("a"));
    set2.Add(S("a"));
    set1.Remove(S("a"));
    set1.Apply(set2);
    CHECK_LIST(set1.LookupAll(), S("a"));
    CHECK(set1.Count() == 1);
    CHECK(set2.Count() == 1);
    set1.Msg();
}
TEST(ORSetTests_Multiple3) {  // ORSetTests.cs:149-160
    DevORSet set1, set2;
    for (int i : {1, 2, 3}) set1.Add(I(i));
    for (int i : {1, 2}) set2.Add(I(i));
    set1.Remove(I(1));
    set1.Apply(set2);
    CHECK_LIST(sorted(set1.LookupAll()), I(1), I(2), I(3));
    set1.Msg();
}
TEST(ORSetTests_Multiple4) {  // ORSetTests.cs:163-187
    DevORSet set1, set2;
    set1.Add(I(1));
    set2.Apply(set1);
    CHECK_LIST(set1.LookupAll(), I(1));
    CHECK_LIST(set2.LookupAll(), I(1));
    set1.Add(I(1));
    set2.Remove(I(1));
    CHECK_LIST(set1.LookupAll(), I(1));
    CHECK_LIST(set2.LookupAll());
    set1.Apply(set2);
    set2.Apply(set1);
    CHECK_LIST(set1.LookupAll(), I(1));
    CHECK_LIST(set2.LookupAll(), I(1));
    set1.Msg();
    set2.Msg();
}
TEST(ORSetTests_Multiple5) {  // ORSetTests.cs:189-202
    DevORSet set1, set2, set3;
    for (int i : {1, 2, 3}) set1.Add(I(i));
    for (int i : {1, 2}) set2.Add(I(i));
    for (int i : {1, 2}) set3.Add(I(i));
    set1.Apply(set2);
    set1.Apply(set3);
    set1.Remove(I(1));
    CHECK_LIST(sorted(set1.LookupAll()), I(2), I(3));
    set1.Msg();
}
TEST(ORSetTests_Multiple6) {  // ORSetTests.cs:203-216
    DevORSet set1;
    set1.Add(S("a")); set1.Add(S("a"));
    CHECK_LIST(set1.LookupAll(), S("a"));
    CHECK(set1.Count() == 1);
}
TEST(ORSetTests_Same) {  // ORSetTests.cs:218-237 — Assert.Equal on collections compares enumerations
    DevORSet set1, set2, set3;
    set1.Add(I(1)); set2.Add(I(1)); set3.Add(I(2));
    CHECK(set1.LookupAll() == set2.LookupAll());
    CHECK(!(set1.LookupAll() == set3.LookupAll()));
}
TEST(ORSetTests_Same2) {  // ORSetTests.cs:239-263 — enumeration order is insertion order
    DevORSet set1, set2, set3;
    set1.Add(I(1)); set1.Add(I(2));
    set2.Add(I(2)); set2.Add(I(1));
    set3.Add(I(2));
    CHECK(!(set1.LookupAll() == set2.LookupAll()));  // Assert.NotEqual(set1, set2)
    CHECK_LIST(set1.LookupAll(), I(1), I(2));
    CHECK_LIST(set2.LookupAll(), I(2), I(1));
    CHECK(sorted(set1.LookupAll()) == sorted(set2.LookupAll()));
    CHECK(!(set1.LookupAll() == set3.LookupAll()));
    CHECK(!(sorted(set1.LookupAll()) == sorted(set3.LookupAll())));
}
TEST(ORSetTests_ApplySynchronizedUpdateException) {  // ORSetTests.cs:265-275: a PNCounter state to an OR-Set
    DevORSet set;
    DevPNC pnc;
    pnc.Increment(3);
    bool threw = false;
    try {
        deliver(set.uid, pnc.Msg());
    } catch (const janus::ApplyError& e) {
        threw = e.commit_index == 0;  // the reference throws (NotSupportedException); nothing is applied
    }
    CHECK(threw);
    CHECK_LIST(set.LookupAll());
}
TEST(ORSetTests_AddNull) {  // ORSetTests.cs:277-287
    DevORSet set1;
    set1.Add(NUL);
    CHECK(set1.LookupAll().size() == 1);
    CHECK(set1.Contains(NUL));
    set1.Msg();
}
TEST(ORSetTests_RemoveNull) {  // ORSetTests.cs:289-299
    DevORSet set1;
    set1.Add(NUL); set1.Remove(NUL);
    CHECK_LIST(set1.LookupAll());
}
TEST(ORSetTests_RemoveNull2) {  // ORSetTests.cs:301-312
    DevORSet set1;
    set1.Add(NUL); set1.Add(NUL); set1.Remove(NUL);
    CHECK_LIST(set1.LookupAll());
    set1.Msg();
}
TEST(ORSetTests_MergeNull) {  // ORSetTests.cs:314-328 (order-sensitive at :327)
    DevORSet set1, set2;
    set1.Add(S("hi")); set1.Add(NUL);
    CHECK(!set2.Remove(NUL));
    set1.Apply(set2);
    CHECK_LIST(set1.LookupAll(), S("hi"), NUL);
}
TEST(ORSetTests_MergeNull2) {  // ORSetTests.cs:330-347 (order-sensitive at :343, :346)
    DevORSet set1, set2;
    set1.Add(S("hi")); set1.Add(NUL);
    set2.Add(NUL); set2.Remove(NUL);
    set2.Apply(set1);
    CHECK_LIST(set2.LookupAll(), S("hi"), NUL);
    set1.Apply(set2);
    CHECK_LIST(set1.LookupAll(), S("hi"), NUL);
    set1.Msg();
    set2.Msg();
}
TEST(ORSetTests_MergeNull3) {  // ORSetTests.cs:349-368
    DevORSet set1, set2;
    set1.Add(NUL);
    set1.Apply(set2);
    set2.Apply(set1);
    set1.Add(NUL); set2.Remove(NUL);
    set2.Apply(set1);
    set1.Apply(set2);
    CHECK_LIST(set2.LookupAll(), NUL);
    CHECK_LIST(set1.LookupAll(), NUL);
}
TEST(ORSetTests_MergeNull4) {  // ORSetTests.cs:370-390
    DevORSet set1, set2;
    set1.Add(NUL); set2.Add(NUL);
    set1.Apply(set2);
    set2.Apply(set1);
    set1.Add(NUL); set2.Remove(NUL);
    set2.Apply(set1);
    set1.Apply(set2);
    CHECK_LIST(set2.LookupAll(), NUL);
    CHECK_LIST(set1.LookupAll(), NUL);
    set1.Msg();
}
TEST(ORSetTests_MergeNull5) {  // ORSetTests.cs:392-409
    DevORSet set1, set2;
    set1.Add(NUL); set2.Add(NUL);
    set2.Remove(NUL); set1.Add(NUL);
    set2.Apply(set1);
    set1.Apply(set2);
    CHECK_LIST(set2.LookupAll(), NUL);
    CHECK_LIST(set1.LookupAll(), NUL);
}
TEST(ORSetTests_MergeNull6) {  // ORSetTests.cs:411-429
    DevORSet set1, set2;
    set1.Add(NUL); set2.Add(NUL);
    set2.Remove(NUL); set1.Add(NUL);
    set1.Apply(set2);
    set2.Apply(set1);
    CHECK_LIST(set2.LookupAll(), NUL);
    CHECK_LIST(set1.LookupAll(), NUL);
}
TEST(ORSetTests_MergeNull7) {  // ORSetTests.cs:431-448
    DevORSet set1, set2;
    set1.Add(NUL);
    set2.Apply(set1);
    set2.Remove(NUL); set2.Add(NUL); set2.Remove(NUL);
    set2.Apply(set1);
    CHECK_LIST(set2.LookupAll());
    set2.Msg();
}
TEST(ORSetMsgTests_EncodeDecode) {  // ORSetTests.cs:453-474 (order-sensitive at :473)
    DevORSet set1, set2;
    set1.Add(S("a")); set1.Add(S("b"));
    set2.Add(S("a")); set2.Add(S("b")); set2.Remove(S("b"));
    set1.Apply(set2);
    CHECK_LIST(set1.LookupAll(), S("a"), S("b"));
    set1.Msg();
}
// ORSet.cs:211-226: add-only keys first, then keys whose tag sets differ, each in insertion order.
TEST(ORSet_LookupAllOrderAddOnlyThenBoth) {
    DevORSet s;
    s.Add(S("p")); s.Add(S("q")); s.Add(S("r"));
    s.Remove(S("p"));
    s.Add(S("p"));
    CHECK_LIST(s.LookupAll(), S("q"), S("r"), S("p"));
}
// The wire order of HashSets and Dictionaries (oracle test_kat Json_ORSetEnumerationOrder): shipped
// bytes equal the reference's after ops, removes in an order unlike the adds', merges and a Clear.
TEST(ORSet_EnumerationOrderOnTheWire) {
    DevORSet s, r;
    s.Add(S("b")); s.Add(S("a")); s.Add(S("b")); s.Add(NUL); s.Add(NUL);
    CHECK(s.Remove(S("b")));
    CHECK(s.Remove(S("a")));
    s.Msg();
    r.Add(S("a")); r.Add(S("b"));
    r.Apply(s);
    r.Msg();
    r.Clear();
    r.Add(S("b")); r.Add(S("a"));
    r.Msg();
    r.Apply(s);
    r.Msg();
}

}  // namespace

int main(int argc, char** argv) {
    const char* only = argc > 1 ? argv[1] : nullptr;
    janus::GpuStableStore store(0, 1024, 8, 4);  // the reference width (int) for PN-Counters
    g_store = &store;
    int failed = 0, ran = 0;
    for (const auto& t : registry()) {
        if (only && t.first.find(only) == std::string::npos) continue;
        ++ran;
        try {
            t.second();
            std::printf("PASS %s\n", t.first.c_str());
        } catch (const std::exception& e) {
            ++failed;
            std::printf("FAIL %s: %s\n", t.first.c_str(), e.what());
        }
    }
    std::printf("%d/%d passed\n", ran - failed, ran);
    return failed ? 1 : 0;
}
