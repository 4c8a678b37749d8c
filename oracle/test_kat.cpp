// oracle/test_kat.cpp — TEST INFRASTRUCTURE ONLY.
//
// The reference's known-answer tests, transcribed one-for-one against the oracle.  These pin the
// oracle: the reference has no golden vectors or fixed seeds, so its xunit
// assertions are the only fixed answers.  Each test cites the reference test it restates.
// ORSet<int> tests use the decimal string of the int (ORSet<T> only needs equality/hash on T).
// Run: test_kat [name-substring]; prints "PASS name" / "FAIL name: why"; exit 1 on any failure.
#include <cstdio>
#include <functional>
#include <sstream>

#include "digest.hpp"
#include "json.hpp"
#include "oracle.hpp"

using namespace oracle;

namespace {

struct Failure : std::runtime_error { using std::runtime_error::runtime_error; };

#define CHECK(cond) do { if (!(cond)) { std::ostringstream os_; os_ << __LINE__ << ": CHECK(" #cond ")"; throw Failure(os_.str()); } } while (0)
#define CHECK_EQ(a, b) do { auto a_ = (a); auto b_ = (b); if (!(a_ == b_)) { std::ostringstream os_; os_ << __LINE__ << ": " #a " == " #b " (" << a_ << " vs " << b_ << ")"; throw Failure(os_.str()); } } while (0)
template <class E, class F> void CHECK_THROWS(F f, int line) {
    try { f(); } catch (const E&) { return; }
    throw Failure(std::to_string(line) + ": expected exception");
}

using L = std::vector<Elem>;
Elem S(const char* s) { return Elem(std::string(s)); }
Elem I(int i) { return Elem(std::to_string(i)); }
L sorted(L v) { std::sort(v.begin(), v.end(), [](const Elem& a, const Elem& b) { return std::stoll(*a) < std::stoll(*b); }); return v; }
L sorted_str(L v) { std::sort(v.begin(), v.end()); return v; }
const Elem NUL = std::nullopt;

std::vector<std::pair<std::string, std::function<void()>>>& registry() { static std::vector<std::pair<std::string, std::function<void()>>> r; return r; }
struct Reg { Reg(const char* n, std::function<void()> f) { registry().emplace_back(n, std::move(f)); } };
#define TEST(name) static void name(); static Reg reg_##name(#name, name); static void name()

GuidGen G(0x5EED);

// ===================== MergeSharp.Tests/PNCounterTests.cs ====================================
TEST(PNCounterTests_TestPNCSingle) {  // PNCounterTests.cs:8-19
    PNCounter<int32_t> pnc(G);
    pnc.Increment(5); pnc.Decrement(8); pnc.Increment(10); pnc.Decrement(3);
    CHECK_EQ(pnc.Get(), 4);
}
TEST(PNCounterTests_TestPNCMerge) {  // PNCounterTests.cs:21-38
    PNCounter<int32_t> pnc1(G), pnc2(G);
    pnc1.Increment(5); pnc1.Decrement(8); pnc1.Increment(10); pnc1.Decrement(3);
    pnc2.Merge(pnc1.GetLastSynchronizedUpdate());
    CHECK_EQ(pnc1.Get(), pnc2.Get());
}
TEST(PNCounterMsgTests_EncodeDecode) {  // PNCounterTests.cs:46-66
    PNCounter<int32_t> pnc1(G); pnc1.Increment(5); pnc1.Decrement(1);
    PNCounter<int32_t> pnc2(G); pnc2.Increment(2); pnc1.Decrement(2);
    const std::string encoded = json::EncodePNC(pnc2.GetLastSynchronizedUpdate());  // Encode -> bytes -> Decode
    PNCounterMsg<int32_t> decoded = json::DecodePNC<int32_t>(encoded);
    pnc1.ApplySynchronizedUpdate(decoded);
    CHECK_EQ(pnc1.Get(), 5 - 1 + 2 - 2);
}
// Semantics notes n1-n3, pinned by reading PNCounters.cs:87-144.
TEST(PNCounter_AbsentLocalActsAsZero) {  // Merge: TryGetValue -> 0, then Max(0, v) inserted
    PNCounter<int32_t> a(G), b(G);
    b.Decrement(0); b.mutP()[b.replicaIdx()] = -7;  // a negative received entry
    a.Merge(b.GetLastSynchronizedUpdate());
    int32_t v = 1; CHECK(a.P().TryGetValue(b.replicaIdx(), v)); CHECK_EQ(v, 0);
}
TEST(PNCounter_IncrementWraps) {  // '+=' is unchecked (PNCounters.cs:99)
    PNCounter<int32_t> a(G);
    a.Increment(INT32_MAX); a.Increment(1);
    int32_t v; a.P().TryGetValue(a.replicaIdx(), v); CHECK_EQ(v, INT32_MIN);
}
TEST(PNCounter_GetCheckedSumThrows) {  // LINQ Sum is checked (PNCounters.cs:89)
    PNCounter<int32_t> a(G), b(G);
    a.Increment(INT32_MAX); b.Increment(1);
    a.Merge(b.GetLastSynchronizedUpdate());
    CHECK_THROWS<OverflowException>([&] { a.Get(); }, __LINE__);
}
TEST(PNCounter_GetPrefixOrderMatters) {  // the throw depends on enumeration order of partial sums
    PNCounter<int32_t> a(G);  // {self: 0}
    Guid g1 = G.next(), g2 = G.next();
    a.mutP()[g1] = INT32_MAX; a.mutP()[g2] = -5;  // 0, MAX, MAX-5: fine
    CHECK_EQ(a.Get(), INT32_MAX - 5);
    PNCounter<int32_t> b(G);
    b.mutP()[g2] = 10; b.mutP()[g1] = INT32_MAX - 5;  // 0, 10, MAX+5: throws
    CHECK_THROWS<OverflowException>([&] { b.Get(); }, __LINE__);
}
TEST(PNCounter_GetSubtractionWraps) {  // ΣP − ΣN is unchecked
    PNCounter<int32_t> a(G);
    a.Increment(INT32_MAX); a.Decrement(-1);  // N = -1
    CHECK_EQ(a.Get(), INT32_MIN);
}

// ===================== MergeSharp.Tests/ORSetTests.cs ========================================
TEST(ORSetTests_SingleORSetValueType1) {  // ORSetTests.cs:10-40
    ORSet set;
    set.Add(I(1), G); set.Add(I(2), G);
    CHECK(set.Remove(I(1)));
    CHECK(!set.Remove(I(3)));
    set.Add(I(3), G);
    CHECK_EQ(set.Count(), 2);
    CHECK(sorted(set.LookupAll()) == (L{I(2), I(3)}));
    set.Clear();
    CHECK_EQ(set.Count(), 0);
    CHECK(set.LookupAll().empty());
    CHECK(!set.Contains(I(1)));
    set.Add(I(1), G);
    CHECK(set.Contains(I(1)));
    CHECK(set.LookupAll() == (L{I(1)}));  // CopyTo(array, 2) -> {0, 0, 1}
}
TEST(ORSetTests_SingleORSetReferenceType) {  // ORSetTests.cs:56-81
    ORSet set;
    set.Add(S("1"), G); set.Add(S("2"), G);
    CHECK(set.Remove(S("1")));
    CHECK(!set.Remove(S("3")));
    set.Add(S("3"), G);
    CHECK_EQ(set.Count(), 2);
    CHECK(sorted_str(set.LookupAll()) == (L{S("2"), S("3")}));
    set.Clear();
    CHECK_EQ(set.Count(), 0);
    CHECK(set.LookupAll().empty());
    CHECK(!set.Contains(S("1")));
    set.Add(S("1"), G);
    CHECK(set.Contains(S("1")));
}
TEST(ORSetTests_SingleORSetReferenceType2) {  // ORSetTests.cs:84-100
    ORSet set;
    set.Add(S("1"), G); set.Add(S("1"), G);
    CHECK_EQ(set.Count(), 1);
    CHECK(set.LookupAll() == (L{S("1")}));
    set.Clear();
    set.Add(S(""), G);
    CHECK(set.Contains(S("")));
}
TEST(ORSetTests_Multiple) {  // ORSetTests.cs:102-129 (order-sensitive at :113)
    ORSet set1, set2;
    set1.Add(I(1), G); set2.Add(I(2), G);
    set1.ApplySynchronizedUpdate(set2.GetLastSynchronizedUpdate());
    CHECK(set1.LookupAll() == (L{I(1), I(2)}));
    CHECK_EQ(set1.Count(), 2);
    CHECK(set2.LookupAll() == (L{I(2)}));
    set2.ApplySynchronizedUpdate(set1.GetLastSynchronizedUpdate());
    CHECK(sorted(set1.LookupAll()) == sorted(set2.LookupAll()));
    set1.Remove(I(2));
    CHECK(set1.LookupAll() == (L{I(1)}));
    CHECK_EQ(set1.Count(), 1);
    set1.Add(I(2), G);
    set2.Remove(I(2));
    set1.ApplySynchronizedUpdate(set2.GetLastSynchronizedUpdate());
    CHECK(sorted(set1.LookupAll()) == (L{I(1), I(2)}));
    CHECK_EQ(set1.Count(), 2);
}
TEST(ORSetTests_Multiple2) {  // ORSetTests.cs:131-147
    ORSet set1, set2;
    set1.Add(S("a"), G);
    set2.Add(S("a"), G);
    set1.Remove(S("a"));
    set1.ApplySynchronizedUpdate(set2.GetLastSynchronizedUpdate());
    CHECK(set1.LookupAll() == (L{S("a")}));
    CHECK_EQ(set1.Count(), 1);
    CHECK_EQ(set2.Count(), 1);
}
TEST(ORSetTests_Multiple3) {  // ORSetTests.cs:149-160
    ORSet set1, set2;
    for (int i : {1, 2, 3}) set1.Add(I(i), G);
    for (int i : {1, 2}) set2.Add(I(i), G);
    set1.Remove(I(1));
    set1.ApplySynchronizedUpdate(set2.GetLastSynchronizedUpdate());
    CHECK(sorted(set1.LookupAll()) == (L{I(1), I(2), I(3)}));
}
TEST(ORSetTests_Multiple4) {  // ORSetTests.cs:163-187
    ORSet set1, set2;
    set1.Add(I(1), G);
    set2.ApplySynchronizedUpdate(set1.GetLastSynchronizedUpdate());
    CHECK(set1.LookupAll() == (L{I(1)}));
    CHECK(set2.LookupAll() == (L{I(1)}));
    set1.Add(I(1), G);
    set2.Remove(I(1));
    CHECK(set1.LookupAll() == (L{I(1)}));
    CHECK(set2.LookupAll().empty());
    set1.ApplySynchronizedUpdate(set2.GetLastSynchronizedUpdate());
    set2.ApplySynchronizedUpdate(set1.GetLastSynchronizedUpdate());
    CHECK(set1.LookupAll() == (L{I(1)}));
    CHECK(set2.LookupAll() == (L{I(1)}));
}
TEST(ORSetTests_Multiple5) {  // ORSetTests.cs:189-202
    ORSet set1, set2, set3;
    for (int i : {1, 2, 3}) set1.Add(I(i), G);
    for (int i : {1, 2}) set2.Add(I(i), G);
    for (int i : {1, 2}) set3.Add(I(i), G);
    set1.ApplySynchronizedUpdate(set2.GetLastSynchronizedUpdate());
    set1.ApplySynchronizedUpdate(set3.GetLastSynchronizedUpdate());
    set1.Remove(I(1));
    CHECK(sorted(set1.LookupAll()) == (L{I(2), I(3)}));
}
TEST(ORSetTests_Multiple6) {  // ORSetTests.cs:203-216 (no [Fact] upstream; transcribed anyway)
    ORSet set1;
    set1.Add(S("a"), G); set1.Add(S("a"), G);
    CHECK(set1.LookupAll() == (L{S("a")}));
    CHECK_EQ(set1.Count(), 1);
}
TEST(ORSetTests_Same) {  // ORSetTests.cs:218-237 — Assert.Equal on collections compares enumerations
    ORSet set1, set2, set3;
    set1.Add(I(1), G); set2.Add(I(1), G); set3.Add(I(2), G);
    CHECK(set1.LookupAll() == set2.LookupAll());
    CHECK(!(set1.LookupAll() == set3.LookupAll()));
}
TEST(ORSetTests_Same2) {  // ORSetTests.cs:239-263 — enumeration order is insertion order
    ORSet set1, set2, set3;
    set1.Add(I(1), G); set1.Add(I(2), G);
    set2.Add(I(2), G); set2.Add(I(1), G);
    set3.Add(I(2), G);
    CHECK(!(set1.LookupAll() == set2.LookupAll()));  // Assert.NotEqual(set1, set2)
    CHECK(sorted(set1.LookupAll()) == sorted(set2.LookupAll()));
    CHECK(!(set1.LookupAll() == set3.LookupAll()));
    CHECK(!(sorted(set1.LookupAll()) == sorted(set3.LookupAll())));
}
TEST(ORSetTests_ApplySynchronizedUpdateException) {  // ORSetTests.cs:265-275
    SafeCRDTManager sm;
    SafeCRDT& orset = sm.CreateSafeCRDT("k", CrdtType::ORSet);
    NetworkProtocol np; np.uid = orset.guid; np.message.type = CrdtType::PNCounter;
    CHECK_THROWS<NotSupportedException>([&] { orset.ApplyUpdateStable(np); }, __LINE__);
}
TEST(ORSetTests_AddNull) {  // ORSetTests.cs:277-287
    ORSet set1; set1.Add(NUL, G);
    CHECK_EQ(set1.LookupAll().size(), (size_t)1);
    CHECK(set1.Contains(NUL));
}
TEST(ORSetTests_RemoveNull) {  // ORSetTests.cs:289-299
    ORSet set1; set1.Add(NUL, G); set1.Remove(NUL);
    CHECK(set1.LookupAll().empty());
}
TEST(ORSetTests_RemoveNull2) {  // ORSetTests.cs:301-312
    ORSet set1; set1.Add(NUL, G); set1.Add(NUL, G); set1.Remove(NUL);
    CHECK(set1.LookupAll().empty());
}
TEST(ORSetTests_MergeNull) {  // ORSetTests.cs:314-328 (order-sensitive at :327)
    ORSet set1, set2;
    set1.Add(S("hi"), G); set1.Add(NUL, G);
    CHECK(!set2.Remove(NUL));
    set1.ApplySynchronizedUpdate(set2.GetLastSynchronizedUpdate());
    CHECK(set1.LookupAll() == (L{S("hi"), NUL}));
}
TEST(ORSetTests_MergeNull2) {  // ORSetTests.cs:330-347
    ORSet set1, set2;
    set1.Add(S("hi"), G); set1.Add(NUL, G);
    set2.Add(NUL, G); set2.Remove(NUL);
    set2.ApplySynchronizedUpdate(set1.GetLastSynchronizedUpdate());
    CHECK(set2.LookupAll() == (L{S("hi"), NUL}));
    set1.ApplySynchronizedUpdate(set2.GetLastSynchronizedUpdate());
    CHECK(set1.LookupAll() == (L{S("hi"), NUL}));
}
TEST(ORSetTests_MergeNull3) {  // ORSetTests.cs:349-368
    ORSet set1, set2;
    set1.Add(NUL, G);
    set1.ApplySynchronizedUpdate(set2.GetLastSynchronizedUpdate());
    set2.ApplySynchronizedUpdate(set1.GetLastSynchronizedUpdate());
    set1.Add(NUL, G); set2.Remove(NUL);
    set2.ApplySynchronizedUpdate(set1.GetLastSynchronizedUpdate());
    set1.ApplySynchronizedUpdate(set2.GetLastSynchronizedUpdate());
    CHECK(set2.LookupAll() == (L{NUL}));
    CHECK(set1.LookupAll() == (L{NUL}));
}
TEST(ORSetTests_MergeNull4) {  // ORSetTests.cs:370-390
    ORSet set1, set2;
    set1.Add(NUL, G); set2.Add(NUL, G);
    set1.ApplySynchronizedUpdate(set2.GetLastSynchronizedUpdate());
    set2.ApplySynchronizedUpdate(set1.GetLastSynchronizedUpdate());
    set1.Add(NUL, G); set2.Remove(NUL);
    set2.ApplySynchronizedUpdate(set1.GetLastSynchronizedUpdate());
    set1.ApplySynchronizedUpdate(set2.GetLastSynchronizedUpdate());
    CHECK(set2.LookupAll() == (L{NUL}));
    CHECK(set1.LookupAll() == (L{NUL}));
}
TEST(ORSetTests_MergeNull5) {  // ORSetTests.cs:392-409
    ORSet set1, set2;
    set1.Add(NUL, G); set2.Add(NUL, G);
    set2.Remove(NUL); set1.Add(NUL, G);
    set2.ApplySynchronizedUpdate(set1.GetLastSynchronizedUpdate());
    set1.ApplySynchronizedUpdate(set2.GetLastSynchronizedUpdate());
    CHECK(set2.LookupAll() == (L{NUL}));
    CHECK(set1.LookupAll() == (L{NUL}));
}
TEST(ORSetTests_MergeNull6) {  // ORSetTests.cs:411-429
    ORSet set1, set2;
    set1.Add(NUL, G); set2.Add(NUL, G);
    set2.Remove(NUL); set1.Add(NUL, G);
    set1.ApplySynchronizedUpdate(set2.GetLastSynchronizedUpdate());
    set2.ApplySynchronizedUpdate(set1.GetLastSynchronizedUpdate());
    CHECK(set2.LookupAll() == (L{NUL}));
    CHECK(set1.LookupAll() == (L{NUL}));
}
TEST(ORSetTests_MergeNull7) {  // ORSetTests.cs:431-448
    ORSet set1, set2;
    set1.Add(NUL, G);
    set2.ApplySynchronizedUpdate(set1.GetLastSynchronizedUpdate());
    set2.Remove(NUL); set2.Add(NUL, G); set2.Remove(NUL);
    set2.ApplySynchronizedUpdate(set1.GetLastSynchronizedUpdate());
    CHECK(set2.LookupAll().empty());
}
TEST(ORSetMsgTests_EncodeDecode) {  // ORSetTests.cs:453-474 (order-sensitive at :473)
    ORSet set1, set2;
    set1.Add(S("a"), G); set1.Add(S("b"), G);
    set2.Add(S("a"), G); set2.Add(S("b"), G); set2.Remove(S("b"));
    const std::string encoded = json::EncodeORSet(set2.GetLastSynchronizedUpdate());
    ORSetMsg decoded = json::DecodeORSet(encoded);
    set1.ApplySynchronizedUpdate(decoded);
    CHECK(set1.LookupAll() == (L{S("a"), S("b")}));
}
// Wire codec (oracle/json.hpp): the System.Text.Json shapes and the accepted decode contract.
TEST(Json_PNCShapeAndGuidFormat) {  // PNCounters.cs:46-49, Guid.ToString("D")
    PNCounterMsg<int32_t> m;
    Guid g{0x1122334455667788ull, 0x99AABBCCDDEEFF00ull};  // bytes 88 77 66 55 44 33 22 11 00 FF EE DD CC BB AA 99
    m.pVector[g] = 7; m.nVector[g] = -3;
    CHECK_EQ(json::GuidD(g), std::string("55667788-3344-1122-00ff-eeddccbbaa99"));
    CHECK_EQ(json::EncodePNC(m), std::string("{\"pVector\":{\"55667788-3344-1122-00ff-eeddccbbaa99\":7},\"nVector\":{\"55667788-3344-1122-00ff-eeddccbbaa99\":-3}}"));
    auto d = json::DecodePNC<int32_t>(" {\"nVector\" : {\"55667788-3344-1122-00FF-EEDDCCBBAA99\" : -3 } ,\n\"pVector\":{\"55667788-3344-1122-00ff-eeddccbbaa99\":7}}\r\n");
    int32_t v = 0;
    CHECK(d.pVector.TryGetValue(g, v) && v == 7);
    CHECK(d.nVector.TryGetValue(g, v) && v == -3);
}
TEST(Json_PNCRejects) {
    const char* bad[] = {
        "{\"pVector\":{}}",                                   // nVector missing -> null -> NRE in Merge
        "{\"pVector\":null,\"nVector\":{}}",                // null vector
        "{\"pVector\":{},\"nVector\":{},\"pVector\":null}", // the last occurrence is null
        "{\"x\":[1,],\"pVector\":{},\"nVector\":{}}",      // a skipped member must still be JSON
        "{\"x\":01,\"pVector\":{},\"nVector\":{}}",
        "{\"x\":tru,\"pVector\":{},\"nVector\":{}}",
        "{\"pvector\":{},\"nVector\":{}}",                // case-sensitive: pVector missing
        "{\"pVector\":{\"55667788-3344-1122-00ff-eeddccbbaa99\":01},\"nVector\":{}}",
        "{\"pVector\":{\"55667788-3344-1122-00ff-eeddccbbaa99\":1.0},\"nVector\":{}}",
        "{\"pVector\":{\"55667788-3344-1122-00ff-eeddccbbaa99\":2147483648},\"nVector\":{}}",
        "{\"pVector\":{\"55667788-3344-1122-00ff-eeddccbbaa9\":1},\"nVector\":{}}",
        "{\"pVector\":{},\"nVector\":{}} x",
        "{\"pVector\":{},\"nVector\":{},}",
    };
    for (const char* b : bad) CHECK_THROWS<json::JsonException>([&] { json::DecodePNC<int32_t>(b); }, __LINE__);
    CHECK_EQ(json::DecodePNC<int32_t>("{\"pVector\":{\"55667788-3344-1122-00ff-eeddccbbaa99\":-2147483648},\"nVector\":{}}").pVector.size(), (size_t)1);
    CHECK_EQ(json::DecodePNC<int64_t>("{\"pVector\":{\"55667788-3344-1122-00ff-eeddccbbaa99\":2147483648},\"nVector\":{}}").pVector.size(), (size_t)1);
}
// System.Text.Json's rules past the compact form (oracle/json.hpp, round 6): unknown members skipped, a repeated
// member's last occurrence, a repeated key's last value at its first place, escaped names and Guid keys, MaxDepth.
TEST(Json_STJRules) {
    const std::string A = "55667788-3344-1122-00ff-eeddccbbaa99", B = "00000001-0002-0003-0405-060708090a0b";
    Guid ga, gb;
    CHECK(json::ParseGuidD(A, ga) && json::ParseGuidD(B, gb));
    auto dec = [](const std::string& x) { return json::DecodePNC<int32_t>(x); };
    auto items = [](const OrderedDict<Guid, int32_t, GuidHash>& d) {
        std::vector<std::pair<Guid, int32_t>> v(d.begin(), d.end());
        return v;
    };
    using IV = std::vector<std::pair<Guid, int32_t>>;
    CHECK(items(dec("{\"pVector\":{},\"nVector\":{},\"x\":1}").pVector).empty());
    CHECK(items(dec("{\"pVector\":{\"" + A + "\":1},\"nVector\":{},\"pVector\":{\"" + B + "\":5}}").pVector) == (IV{{gb, 5}}));
    CHECK(items(dec("{\"pVector\":{\"" + A + "\":1,\"" + B + "\":2,\"" + A + "\":3},\"nVector\":{}}").pVector) == (IV{{ga, 3}, {gb, 2}}));
    CHECK(items(dec("{\"pVector\":{\"" + A + "\":1,\"" + json::GuidD(ga).substr(0, 35) + "9\":-4},\"nVector\":{}}").pVector) == (IV{{ga, -4}}));
    CHECK(items(dec("{\"p\\u0056ector\":{\"5566\\u0037788-3344-1122-00FF-eeddccbbaa99\":4},\"nVector\":{}}").pVector) == (IV{{ga, 4}}));
    CHECK(dec("{\"pVector\":null,\"nVector\":{},\"pVector\":{}}").pVector.size() == 0);
    CHECK(dec("{\"z\":{\"a\":[1,-2.5e+3,{\"b\":[]},true,false,null],\"c\":\"\\u00e9\"},\"pVector\":{},\"nVector\":{}}").pVector.size() == 0);
    // MaxDepth 64 counting the message object: a skipped value may open 63 more containers, not 64
    const std::string d63 = std::string(63, '[') + std::string(63, ']'), d64 = std::string(64, '[') + std::string(64, ']');
    CHECK(dec("{\"x\":" + d63 + ",\"pVector\":{},\"nVector\":{}}").nVector.size() == 0);
    CHECK_THROWS<json::JsonException>([&] { dec("{\"x\":" + d64 + ",\"pVector\":{},\"nVector\":{}}"); }, __LINE__);
    // ORSetMsg: an element named twice in one map keeps its first place and its last tag set; `null` only as a last value fails
    const std::string T1 = "\"" + A + "\"", T2 = "\"" + B + "\"";
    const ORSetMsg m = json::DecodeORSet("{\"q\":[],\"addSet\":{\"a\":[" + T1 + "],\"b\":[" + T2 + "],\"a\":null,\"a\":[" + T2 + "," + T2 + "]},"
                                         "\"removeSet\":{},\"nullAddGuid\":null,\"nullRemoveGuid\":[],\"nullAddGuid\":[" + T1 + "]}");
    CHECK_EQ(json::EncodeORSet(m), "{\"addSet\":{\"a\":[" + T2 + "],\"b\":[" + T2 + "]},\"removeSet\":{},\"nullAddGuid\":[" + T1 + "],\"nullRemoveGuid\":[]}");
    CHECK_THROWS<json::JsonException>([&] { json::DecodeORSet("{\"addSet\":{\"a\":[],\"a\":null},\"removeSet\":{},\"nullAddGuid\":[],\"nullRemoveGuid\":[]}"); }, __LINE__);
}
TEST(Json_ORSetEscapesAndRoundTrip) {  // ORSet.cs:56-69; JavaScriptEncoder.Default
    ORSet s;
    s.Add(S("a<b>&\"q\"\\"), G); s.Add(S("caf\xC3\xA9 \xF0\x9F\x98\x80"), G); s.Add(NUL, G); s.Add(S("x"), G); s.Remove(S("x"));
    const std::string e = json::EncodeORSet(s.GetLastSynchronizedUpdate());
    CHECK(e.find("a\\u003Cb\\u003E\\u0026\\u0022q\\u0022\\\\") != std::string::npos);
    CHECK(e.find("caf\\u00E9 \\uD83D\\uDE00") != std::string::npos);
    ORSet t;
    t.ApplySynchronizedUpdate(json::DecodeORSet(e));
    CHECK(t.LookupAll() == s.LookupAll());
    CHECK_THROWS<json::JsonException>([&] { json::DecodeORSet("{\"addSet\":{},\"removeSet\":{},\"nullAddGuid\":[]}"); }, __LINE__);
    CHECK_THROWS<json::JsonException>([&] { json::DecodeORSet("{\"addSet\":{\"\\ud800\":[]},\"removeSet\":{},\"nullAddGuid\":[],\"nullRemoveGuid\":[]}"); }, __LINE__);
}
// HashSet<Guid> / Dictionary enumeration order on the wire (.NET 6 HashSet: entries array, Add appends,
// nothing removes single tags; oracle.hpp GuidSet header).  Tags chosen so that insertion order is
// not their sorted order; removeSet's Dictionary order is first-Remove order, not addSet's.
TEST(Json_ORSetEnumerationOrder) {  // ORSet.cs:134-186, 253-283, 305-308; encoded as SafeCRDT.cs:49 ships it
    const Guid t3{3, 0}, t1{1, 0}, t2{2, 0}, t9{9, 0};
    auto q = [](const Guid& g) { return "\"" + json::GuidD(g) + "\""; };
    ORSet s;
    s.AddTag(S("b"), t3); s.AddTag(S("a"), t1); s.AddTag(S("b"), t2); s.AddTag(NUL, t9); s.AddTag(NUL, t1);
    CHECK(s.Remove(S("b")));  // removeSet["b"] = new HashSet(addSet["b"]): [t3, t2]
    CHECK(s.Remove(S("a")));  // removeSet["a"] appended after "b"
    const std::string e = json::EncodeORSet(s.GetLastSynchronizedUpdate());
    CHECK_EQ(e, "{\"addSet\":{\"b\":[" + q(t3) + "," + q(t2) + "],\"a\":[" + q(t1) + "]},\"removeSet\":{\"b\":[" + q(t3) + "," + q(t2) +
                    "],\"a\":[" + q(t1) + "]},\"nullAddGuid\":[" + q(t9) + "," + q(t1) + "],\"nullRemoveGuid\":[]}");
    // Merge: UnionWith appends the received tags the local set lacks, in the received order; new keys
    // are appended to the Dictionaries in the received Dictionary's order
    ORSet r;
    r.AddTag(S("a"), t9); r.AddTag(S("b"), t2);
    r.ApplySynchronizedUpdate(json::DecodeORSet(e));
    CHECK_EQ(json::EncodeORSet(r.GetLastSynchronizedUpdate()),
             "{\"addSet\":{\"a\":[" + q(t9) + "," + q(t1) + "],\"b\":[" + q(t2) + "," + q(t3) + "]},\"removeSet\":{\"b\":[" + q(t3) + "," +
                 q(t2) + "],\"a\":[" + q(t1) + "]},\"nullAddGuid\":[" + q(t9) + "," + q(t1) + "],\"nullRemoveGuid\":[]}");
    // Clear resets both Dictionaries and their order
    r.Clear();
    r.AddTag(S("b"), t1); r.AddTag(S("a"), t3);
    CHECK_EQ(json::EncodeORSet(r.GetLastSynchronizedUpdate()),
             "{\"addSet\":{\"b\":[" + q(t1) + "],\"a\":[" + q(t3) + "]},\"removeSet\":{},\"nullAddGuid\":[],\"nullRemoveGuid\":[]}");
}
// Semantics note n4 (SetEquals, not "add \ rem non-empty"), pinned by ORSet.cs:216.
TEST(ORSet_SetEqualsNotDifference) {
    ORSet s;
    Guid t1 = G.next(), t2 = G.next();
    s.AddTag(S("x"), t1);
    s.mutRemoveSet()["x"].insert(t1); s.mutRemoveSet()["x"].insert(t2);  // rem ⊋ add
    CHECK(s.Contains(S("x")));  // add \ rem is empty, but the sets differ
}
TEST(ORSet_LookupAllOrderAddOnlyThenBoth) {  // ORSet.cs:211-226
    ORSet s;
    s.Add(S("p"), G); s.Add(S("q"), G); s.Add(S("r"), G);
    s.Remove(S("p"));
    s.Add(S("p"), G);  // p in both with differing sets -> listed after the add-only keys
    CHECK(s.LookupAll() == (L{S("q"), S("r"), S("p")}));
}

// ===================== MergeSharp.Tests/ReplicationManagerTests.cs ============================
// DummyConnectionManager delivers every update's full state synchronously to the peer RM
// (DummyConnectionManager.cs:78-81; ProxyBuilder.cs:66-75 calls HasSideEffect after each op).
struct Rm2 {
    PNCounter<int32_t> a, b;  // the same uid on rm0 and rm1 (each instance has its own Guid)
    Rm2() : a(G), b(G) {}
    void incA(int v) { a.Increment(v); b.ApplySynchronizedUpdate(a.GetLastSynchronizedUpdate()); }
    void incB(int v) { b.Increment(v); a.ApplySynchronizedUpdate(b.GetLastSynchronizedUpdate()); }
    void decA(int v) { a.Decrement(v); b.ApplySynchronizedUpdate(a.GetLastSynchronizedUpdate()); }
};
TEST(ReplicationManagerTests_RepManagerPNCTest) {  // ReplicationManagerTests.cs:53-67
    Rm2 r; r.incA(5); r.decA(8); r.incA(10); r.decA(3);
    CHECK_EQ(r.a.Get(), r.b.Get());
    CHECK_EQ(r.b.Get(), 4);
}
TEST(ReplicationManagerTests_RepManagerPNCTest1) {  // ReplicationManagerTests.cs:70-99
    Rm2 r0, r1, r2, r3;
    uint64_t x = 12345;
    for (int i = 0; i < 5; ++i) {
        for (Rm2* r : {&r0, &r2}) { x = mix64(x); r->incA((int)(x % 100)); }
        for (Rm2* r : {&r1, &r3}) { x = mix64(x); r->incB((int)(x % 100)); }
    }
    for (Rm2* r : {&r0, &r1, &r2, &r3}) CHECK_EQ(r->a.Get(), r->b.Get());
}
TEST(ReplicationManagerTests_LocalConcurrentWrites) {  // ReplicationManagerTests.cs:101-129
    Rm2 r;
    for (int i = 0; i < 10; ++i) { r.incA(1); r.incB(1); }
    CHECK_EQ(r.a.Get(), r.b.Get());
    CHECK_EQ(r.a.Get(), 20);
}

// ===================== Tests/KVStoreTests.cs (convergence invariants) =========================
// 4 nodes; node 0's updates are batched (clientBatchSize = 1, KVStoreTests.cs:64), each batch is
// delivered as a block to every node (prospective merge, ConnectionManager.ReceivedBlock ->
// RM.ReceivedUpdateSyncMsg) and then committed to every node (HandleAfterConsensusUpdates).
struct Cluster4 {
    std::vector<std::unique_ptr<SafeCRDTManager>> nodes;
    explicit Cluster4(int batch = 1) { for (int i = 0; i < 4; ++i) nodes.push_back(std::make_unique<SafeCRDTManager>(batch, 1000 + i)); }
    void create(const std::string& key, CrdtType t) {  // KeySpaceManager.CreateNewKVPair + remote create
        Guid uid = nodes[0]->gen.next();
        for (auto& n : nodes) n->CreateSafeCRDT(key, t, uid);
    }
    SafeCRDT& at(int node, const std::string& key) { return *nodes[node]->safeCRDTs.at(key); }
    void commit_all() {  // deliver every submitted UpdateMessage of every node, in node order
        std::vector<std::vector<UpdateMessage>> wave;
        for (auto& n : nodes) { wave.push_back(n->submitted); n->submitted.clear(); }
        for (auto& recv : nodes)  // prospective merge on block receipt (RM:327-344), other nodes only
            for (size_t src = 0; src < nodes.size(); ++src) {
                if (nodes[src].get() == recv.get()) continue;
                for (const auto& um : wave[src]) for (const auto& np : um.update) {
                    SafeCRDT& sc = *recv->safeCRDTsIndexedByuid.at(np.uid);
                    if (sc.type == CrdtType::PNCounter) sc.pncProspective->pnc.ApplySynchronizedUpdate(np.message.pnc);
                    else sc.orProspective->orset.ApplySynchronizedUpdate(np.message.orset);
                }
            }
        for (auto& n : nodes) n->HandleAfterConsensusUpdates(wave);
    }
};
TEST(KVStoreTests_TestStableConverge) {  // KVStoreTests.cs:225-246
    Cluster4 c; c.create("test", CrdtType::PNCounter);
    c.at(0, "test").Update(1, {Arg::I(5)}, false);
    int64_t p0 = c.at(0, "test").QueryProspective().i;
    c.commit_all();
    for (int n = 0; n < 4; ++n) {
        CHECK_EQ(c.at(n, "test").QueryProspective().i, p0);
        CHECK_EQ(c.at(n, "test").QueryStable().i, p0);
    }
}
TEST(KVStoreTests_TestMultipleConverge) {  // KVStoreTests.cs:248-286
    Cluster4 c;
    for (int i = 0; i < 100; ++i) c.create("test" + std::to_string(i), CrdtType::PNCounter);
    uint64_t x = 99;
    for (int i = 0; i < 100; ++i)
        for (int j = 0; j < 10; ++j) { x = mix64(x); c.at(0, "test" + std::to_string(i)).Update(1, {Arg::I((int)(x % 100))}, false); }
    c.commit_all();
    for (int n = 0; n < 4; ++n)
        for (int i = 0; i < 100; ++i) {
            std::string k = "test" + std::to_string(i);
            CHECK_EQ(c.at(n, k).QueryProspective().i, c.at(0, k).QueryProspective().i);
            CHECK_EQ(c.at(n, k).QueryStable().i, c.at(n, k).QueryProspective().i);
        }
}
TEST(KVStoreTests_TestSafeUpdate) {  // KVStoreTests.cs:288-320
    Cluster4 c; c.create("test", CrdtType::PNCounter);
    SafeCRDT& v0 = c.at(0, "test");
    v0.Update(1, {Arg::I(5)}, false);
    CHECK(v0.QueryProspective().i != v0.QueryStable().i);
    v0.Update(1, {Arg::I(3)}, true, /*origin*/ 1);
    c.commit_all();
    CHECK(c.nodes[0]->notified == std::vector<uint64_t>{1});
    CHECK_EQ(v0.QueryProspective().i, v0.QueryStable().i);
    CHECK_EQ(v0.QueryStable().i, 8);
}
TEST(KVStoreTests_TestMultipleSafeUpdate) {  // KVStoreTests.cs:322-354
    Cluster4 c;
    for (int i = 0; i < 10; ++i) c.create("test" + std::to_string(i), CrdtType::PNCounter);
    uint64_t origin = 1, x = 7;
    for (int n = 0; n < 4; ++n)
        for (int i = 0; i < 10; ++i) {
            x = mix64(x);
            SafeCRDT& v = c.at(n, "test" + std::to_string(i));
            v.Update(1, {Arg::I(1 + (int)(x % 99))}, true, origin);
            c.commit_all();
            CHECK(c.nodes[n]->notified.back() == origin);
            CHECK_EQ(v.QueryProspective().i, v.QueryStable().i);
            ++origin;
        }
}
TEST(KVStore_ORSetConverge) {  // the same invariant (p == s everywhere) on the OR-Set path
    Cluster4 c; c.create("s", CrdtType::ORSet);
    uint64_t x = 3;
    for (int i = 0; i < 200; ++i) {
        x = mix64(x);
        int node = (int)(x % 4), op = (int)((x >> 8) % 3);
        std::string e = std::to_string((x >> 16) % 12);
        c.at(node, "s").Update(op == 2 ? 2 : 1, {Arg::S(e)}, false);
        if (i % 17 == 0) c.commit_all();
    }
    c.commit_all();
    for (int n = 0; n < 4; ++n)
        for (int e = 0; e < 12; ++e) {
            std::vector<Arg> q{Arg::S(std::to_string(e))};
            CHECK_EQ(c.at(n, "s").QueryStable(q).b, c.at(n, "s").QueryProspective(q).b);
            CHECK_EQ(c.at(n, "s").QueryStable(q).b, c.at(0, "s").QueryStable(q).b);
        }
}

// ===================== wrappers / manager (read from the reference source) ====================
TEST(PNCounterWrapper_Dispatch) {  // PNCounterWrapper.cs:33-47
    PNCounterWrapper w(G);
    CHECK(w.Update(1, {Arg::I(7)}).b);
    CHECK(w.Update(2, {Arg::I(2)}).b);
    CHECK_EQ(w.Query().i, 5);
    CHECK_THROWS<InvalidOperationException>([&] { w.Update(3, {Arg::I(1)}); }, __LINE__);
    CHECK_THROWS<InvalidCastException>([&] { w.Update(9, {Arg::S("x")}); }, __LINE__);  // cast before switch
}
TEST(ORSetWrapper_Dispatch) {  // ORSetWrapper.cs:24-46
    ORSetWrapper w;
    CHECK(w.Update(1, {Arg::S("a")}, G).b);
    CHECK(w.Query({Arg::S("a")}).b);
    CHECK(w.Update(2, {Arg::S("a")}, G).b);
    CHECK(!w.Update(2, {Arg::S("a")}, G).b);
    CHECK(!w.Query({Arg::S("a")}).b);
    CHECK(w.Update(3, {}, G).b);
    CHECK_THROWS<InvalidOperationException>([&] { w.Update(4, {Arg::S("a")}, G); }, __LINE__);
}
TEST(SafeCRDTManager_BatcherCompaction) {  // SafeCRDTManager.cs:165-198
    SafeCRDTManager sm(4);
    SafeCRDT& a = sm.CreateSafeCRDT("a", CrdtType::PNCounter);
    SafeCRDT& b = sm.CreateSafeCRDT("b", CrdtType::PNCounter);
    a.Update(1, {Arg::I(1)}, false);
    b.Update(1, {Arg::I(1)}, false);
    a.Update(1, {Arg::I(2)}, true, 42);
    a.Update(1, {Arg::I(4)}, false);  // 4th message: flush
    CHECK_EQ(sm.submitted.size(), (size_t)1);
    const auto& u = sm.submitted[0].update;
    CHECK_EQ(u.size(), (size_t)3);  // safe one individually, then a (last state), b
    CHECK(u[0].seq == 3 && u[1].uid == a.guid && u[1].seq == 4 && u[2].uid == b.guid);
}
TEST(SafeCRDTManager_ApplySkipsCreateAndEmpty) {  // SafeCRDTManager.cs:133-134
    SafeCRDTManager sm;
    SafeCRDT& a = sm.CreateSafeCRDT("a", CrdtType::PNCounter);
    PNCounter<int32_t> src(G); src.Increment(9);
    NetworkProtocol create; create.uid = a.guid; create.syncMsgType = NetworkProtocol::ManagerMsg_Create; create.message.pnc = src.GetLastSynchronizedUpdate();
    NetworkProtocol empty; empty.message.pnc = src.GetLastSynchronizedUpdate();
    NetworkProtocol real; real.uid = a.guid; real.message.pnc = src.GetLastSynchronizedUpdate();
    sm.HandleAfterConsensusUpdates({{UpdateMessage{{create, empty}}}});
    CHECK_EQ(a.QueryStable().i, 0);
    sm.HandleAfterConsensusUpdates({{UpdateMessage{{real}}}});
    CHECK_EQ(a.QueryStable().i, 9);
}

// ---- SHA-256 (FIPS 180-4 / NIST example vectors) and UpdateMessage.ComputeDigest ----------------
std::string hex(const uint8_t* d, size_t n) { static const char* x = "0123456789abcdef"; std::string s; for (size_t i = 0; i < n; ++i) { s += x[d[i] >> 4]; s += x[d[i] & 15]; } return s; }
std::string sha_hex(const std::string& m) { uint8_t o[32]; sha256((const uint8_t*)m.data(), m.size(), o); return hex(o, 32); }
TEST(SHA256_NistVectors) {  // FIPS 180-4 examples (NIST CSRC "SHA256.pdf", SHA2 additional vectors)
    CHECK_EQ(sha_hex(""), std::string("e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"));
    CHECK_EQ(sha_hex("abc"), std::string("ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"));
    CHECK_EQ(sha_hex("abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq"),
             std::string("248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"));
    CHECK_EQ(sha_hex("abcdefghbcdefghicdefghijdefghijkefghijklfghijklmghijklmnhijklmnoijklmnopjklmnopqklmnopqrlmnopqrsmnopqrstnopqrstu"),
             std::string("cf5b16a778af8380036ce59e7b0492370b249b11e8f07a51afac45037afee9d1"));
    CHECK_EQ(sha_hex(std::string(1000000, 'a')), std::string("cdc76e5c9914fb9281a1c7e284d73e67f1809a48a497200e046d39ccc7112cd0"));
}
TEST(ArrayPoolRentLength) {  // .NET 6 TlsOverPerCoreLockedStacksArrayPool buckets (digest.hpp header)
    CHECK_EQ(array_pool_rent_length(0), 0ull);
    CHECK_EQ(array_pool_rent_length(1), 16ull);
    CHECK_EQ(array_pool_rent_length(32), 32ull);
    CHECK_EQ(array_pool_rent_length(96), 128ull);
    CHECK_EQ(array_pool_rent_length(32000), 32768ull);
    CHECK_EQ(array_pool_rent_length(1ull << 20), 1ull << 20);
    CHECK_EQ(array_pool_rent_length((1ull << 20) + 32), (1ull << 20) + 32);
}
TEST(UpdateMessage_ComputeDigest) {  // DAGUpdateMessage.cs:32-55
    // one message: toSign = its 32-byte digest exactly (Rent(32) = 32)
    std::string m = "{\"pVector\":{},\"nVector\":{}}";
    const uint8_t* p = (const uint8_t*)m.data(); uint64_t len = m.size();
    uint8_t d1[32], inner[32], want[32];
    update_digest(1, &p, &len, nullptr, d1);
    sha256(p, len, inner); sha256(inner, 32, want);
    CHECK_EQ(hex(d1, 32), hex(want, 32));
    // three messages, the middle one null: 96 bytes rented as 128, zeros for null and the padding
    const uint8_t* ps[3] = {p, p, p}; uint64_t ls[3] = {len, 0, len}; uint8_t nul[3] = {0, 1, 0};
    uint8_t buf[128] = {0};
    sha256(p, len, buf); sha256(p, len, buf + 64);
    sha256(buf, 128, want);
    update_digest(3, ps, ls, nul, d1);
    CHECK_EQ(hex(d1, 32), hex(want, 32));
    // empty update list: Rent(0) is the empty array
    update_digest(0, nullptr, nullptr, nullptr, d1);
    CHECK_EQ(hex(d1, 32), sha_hex(""));
}

}  // namespace

int main(int argc, char** argv) {
    const char* filt = argc > 1 ? argv[1] : "";
    int fails = 0, runs = 0;
    for (auto& t : registry()) {
        if (*filt && t.first.find(filt) == std::string::npos) continue;
        ++runs;
        try { t.second(); std::printf("PASS %s\n", t.first.c_str()); }
        catch (const std::exception& e) { ++fails; std::printf("FAIL %s: %s\n", t.first.c_str(), e.what()); }
    }
    std::printf("%d/%d passed\n", runs - fails, runs);
    return fails ? 1 : 0;
}
