// oracle/json.hpp — TEST INFRASTRUCTURE ONLY (see oracle.hpp header).
//
// Restatement of the state-message wire codec: PNCounterMsg.Encode/Decode
// (MergeSharp/MergeSharp/CRDTs/PNCounters.cs:38-49) and ORSetMsg<string>.Encode/Decode (ORSet.cs:56-69),
// i.e. System.Text.Json 6.0 JsonSerializer.SerializeToUtf8Bytes / Deserialize with default options
// on those classes (the dependency is pinned at BFT-CRDT/obj/project.assets.json:785).
//
// Encode (what the reference's writer emits, default JsonSerializerOptions):
//   {"pVector":{"<guid>":<int>,...},"nVector":{...}}                              (declaration order)
//   {"addSet":{"<elem>":["<guid>",...],...},"removeSet":{...},"nullAddGuid":[...],"nullRemoveGuid":[...]}
//   Guid keys/values in "D" format, lower-case hex (Guid.ToString()), no whitespace; strings escaped by
//   JavaScriptEncoder.Default (printable ASCII except " & ' + < > ` \ kept; \\ for backslash;
//   \b \t \n \f \r; every other code unit as \uXXXX with upper-case hex).
//
// Decode — the accepted wire contract, identical in this oracle, the host mirror
// (janus-crdt_amd/host/) and the device parsers (janus-crdt_amd/csrc/json.hip, orset_wire.hip), restated from
// System.Text.Json 6.0's documented default behaviour (JsonSerializerOptions defaults; round 6):
//   * JSON whitespace (space, \t, \n, \r) between tokens; the object's properties in any order; property names
//     matched after unescaping, case-sensitively (PropertyNameCaseInsensitive = false);
//   * a property that is not a member is SKIPPED (JsonUnmappedMemberHandling.Skip): its value may be any
//     well-formed JSON value, nested at most MaxDepth = 64 levels counting the message object;
//   * a member given twice: the LAST occurrence wins (each occurrence deserialized and assigned in turn);
//   * PNC vector keys: "D"-form Guid strings (36 characters once unescaped, hex of either case; Guid's
//     property-name converter unescapes); values -?(0|[1-9][0-9]*) within the counter's width (JsonException
//     on overflow / a fraction / an exponent, as Utf8JsonReader.GetInt32 / GetInt64);
//   * a key repeated inside one PNC vector or one ORSet map: Dictionary's indexer set — the LAST value, at the
//     FIRST key's position in enumeration order;
//   * ORSet element keys and Guid strings: full JSON string syntax (escapes, surrogate pairs, UTF-8
//     validated); a Guid repeated inside one tag array is de-duplicated (HashSet<Guid>.Add).
// REJECTED (JsonException here, JG_EINVAL in the engine):
//   * malformed JSON anywhere (skipped values included), a number out of range, a nesting deeper than 64;
//   * a member missing, or whose last occurrence is `null`, or an ORSet element whose last tag set is `null`
//     (the reference's Merge would throw NullReferenceException / ArgumentNullException).
// Parity for the skipped / repeated forms is unpinned: the reference's encoder never emits them and no
// reference fixture holds one; they follow STJ's documented rules so that a node built on this engine applies
// every state a reference node applies.  Where STJ's exact edge is not documented (UTF-8
// validation inside skipped strings, the depth counted at a skipped scalar) the stricter reading is taken.
#pragma once

#include <cstdint>
#include <limits>
#include <stdexcept>
#include <string>
#include <string_view>

#include "oracle.hpp"

namespace oracle::json {

struct JsonException : std::runtime_error { using std::runtime_error::runtime_error; };

// Guid.ToString("D"): bytes b0..b15 (lo = b0..b7, hi = b8..b15, little-endian) print as
// b3b2b1b0-b5b4-b7b6-b8b9-b10b11b12b13b14b15.
inline std::string GuidD(const Guid& g) {
    static const char* hx = "0123456789abcdef";
    uint8_t b[16];
    for (int i = 0; i < 8; ++i) { b[i] = (uint8_t)(g.lo >> (8 * i)); b[8 + i] = (uint8_t)(g.hi >> (8 * i)); }
    static const int order[16] = {3, 2, 1, 0, 5, 4, 7, 6, 8, 9, 10, 11, 12, 13, 14, 15};
    std::string s;
    s.reserve(36);
    for (int i = 0; i < 16; ++i) {
        if (i == 4 || i == 6 || i == 8 || i == 10) s.push_back('-');
        s.push_back(hx[b[order[i]] >> 4]);
        s.push_back(hx[b[order[i]] & 15]);
    }
    return s;
}

inline int hexval(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}

// Utf8Parser 'D' format: exactly 36 chars, dashes at 8/13/18/23, hex digits of either case.
inline bool ParseGuidD(std::string_view s, Guid& g) {
    if (s.size() != 36) return false;
    uint8_t b[16];
    static const int order[16] = {3, 2, 1, 0, 5, 4, 7, 6, 8, 9, 10, 11, 12, 13, 14, 15};
    size_t p = 0;
    for (int i = 0; i < 16; ++i) {
        if (i == 4 || i == 6 || i == 8 || i == 10) {
            if (s[p] != '-') return false;
            ++p;
        }
        const int h = hexval(s[p]), l = hexval(s[p + 1]);
        if (h < 0 || l < 0) return false;
        b[order[i]] = (uint8_t)(h << 4 | l);
        p += 2;
    }
    g.lo = g.hi = 0;
    for (int i = 0; i < 8; ++i) { g.lo |= (uint64_t)b[i] << (8 * i); g.hi |= (uint64_t)b[8 + i] << (8 * i); }
    return true;
}

// JavaScriptEncoder.Default over UTF-8 input (the element strings are valid UTF-8 here).
inline void EscapeTo(std::string& o, std::string_view s) {
    static const char* HX = "0123456789ABCDEF";
    auto u16 = [&](uint32_t u) {
        o += "\\u";
        o.push_back(HX[(u >> 12) & 15]); o.push_back(HX[(u >> 8) & 15]); o.push_back(HX[(u >> 4) & 15]); o.push_back(HX[u & 15]);
    };
    for (size_t i = 0; i < s.size();) {
        const uint8_t c = (uint8_t)s[i];
        if (c < 0x80) {
            ++i;
            switch (c) {
                case '\\': o += "\\\\"; continue;
                case '\b': o += "\\b"; continue;
                case '\t': o += "\\t"; continue;
                case '\n': o += "\\n"; continue;
                case '\f': o += "\\f"; continue;
                case '\r': o += "\\r"; continue;
                default: break;
            }
            if (c < 0x20 || c == 0x7F || c == '"' || c == '&' || c == '\'' || c == '+' || c == '<' || c == '>' || c == '`') u16(c);
            else o.push_back((char)c);
            continue;
        }
        uint32_t cp;
        int len;
        if ((c & 0xE0) == 0xC0) { cp = c & 0x1F; len = 2; }
        else if ((c & 0xF0) == 0xE0) { cp = c & 0x0F; len = 3; }
        else { cp = c & 0x07; len = 4; }
        for (int k = 1; k < len; ++k) cp = cp << 6 | ((uint8_t)s[i + k] & 0x3F);
        i += len;
        if (cp >= 0x10000) {
            cp -= 0x10000;
            u16(0xD800 | (cp >> 10));
            u16(0xDC00 | (cp & 0x3FF));
        } else {
            u16(cp);
        }
    }
}

template <class T> std::string EncodePNC(const PNCounterMsg<T>& m) {  // PNCounters.cs:46-49
    std::string o = "{\"pVector\":{";
    bool first = true;
    for (const auto& kv : m.pVector) {
        if (!first) o.push_back(',');
        first = false;
        o += '"' + GuidD(kv.first) + "\":" + std::to_string(kv.second);
    }
    o += "},\"nVector\":{";
    first = true;
    for (const auto& kv : m.nVector) {
        if (!first) o.push_back(',');
        first = false;
        o += '"' + GuidD(kv.first) + "\":" + std::to_string(kv.second);
    }
    o += "}}";
    return o;
}

inline void EncodeTags(std::string& o, const GuidSet& s) {
    o.push_back('[');
    bool first = true;
    for (const auto& g : s) {
        if (!first) o.push_back(',');
        first = false;
        o += '"' + GuidD(g) + '"';
    }
    o.push_back(']');
}

inline std::string EncodeORSet(const ORSetMsg& m) {  // ORSet.cs:65-69
    std::string o = "{\"addSet\":{";
    for (int which = 0; which < 2; ++which) {
        const auto& d = which ? m.removeSet : m.addSet;
        bool first = true;
        for (const auto& kv : d) {
            if (!first) o.push_back(',');
            first = false;
            o.push_back('"');
            EscapeTo(o, kv.first);
            o += "\":";
            EncodeTags(o, kv.second);
        }
        o += which ? "},\"nullAddGuid\":" : "},\"removeSet\":{";
    }
    EncodeTags(o, m.nullAddGuid);
    o += ",\"nullRemoveGuid\":";
    EncodeTags(o, m.nullRemoveGuid);
    o.push_back('}');
    return o;
}

// ---- decoding ---------------------------------------------------------------------------------
class Reader {
  public:
    explicit Reader(std::string_view s) : s_(s) {}
    [[noreturn]] void fail(const char* what) const {
        throw JsonException(std::string("JsonException: ") + what + " at byte " + std::to_string(p_));
    }
    void ws() { while (p_ < s_.size() && (s_[p_] == ' ' || s_[p_] == '\t' || s_[p_] == '\n' || s_[p_] == '\r')) ++p_; }
    bool peek(char c) { ws(); return p_ < s_.size() && s_[p_] == c; }
    void expect(char c) {
        ws();
        if (p_ >= s_.size() || s_[p_] != c) fail("unexpected token");
        ++p_;
    }
    bool eat(char c) {
        if (peek(c)) { ++p_; return true; }
        return false;
    }
    void end() {
        ws();
        if (p_ != s_.size()) fail("trailing data");
    }
    // A property name / Guid key without escapes (PN-Counter messages): returns the raw bytes.
    std::string_view raw_string() {
        expect('"');
        const size_t b = p_;
        while (p_ < s_.size() && s_[p_] != '"') {
            if (s_[p_] == '\\' || (uint8_t)s_[p_] < 0x20) fail("escaped or control character in a name");
            ++p_;
        }
        if (p_ >= s_.size()) fail("unterminated string");
        return s_.substr(b, p_++ - b);
    }
    // Full JSON string: escapes, surrogate pairs, UTF-8 validation.  Returns UTF-8.
    std::string string() {
        expect('"');
        std::string o;
        for (;;) {
            if (p_ >= s_.size()) fail("unterminated string");
            const uint8_t c = (uint8_t)s_[p_++];
            if (c == '"') return o;
            if (c < 0x20) fail("control character in string");
            if (c == '\\') {
                if (p_ >= s_.size()) fail("bad escape");
                const char e = s_[p_++];
                switch (e) {
                    case '"': o.push_back('"'); break;
                    case '\\': o.push_back('\\'); break;
                    case '/': o.push_back('/'); break;
                    case 'b': o.push_back('\b'); break;
                    case 'f': o.push_back('\f'); break;
                    case 'n': o.push_back('\n'); break;
                    case 'r': o.push_back('\r'); break;
                    case 't': o.push_back('\t'); break;
                    case 'u': {
                        uint32_t u = hex4();
                        if (u >= 0xDC00 && u <= 0xDFFF) fail("lone low surrogate");
                        if (u >= 0xD800 && u <= 0xDBFF) {
                            if (p_ + 1 >= s_.size() || s_[p_] != '\\' || s_[p_ + 1] != 'u') fail("lone high surrogate");
                            p_ += 2;
                            const uint32_t l = hex4();
                            if (l < 0xDC00 || l > 0xDFFF) fail("bad surrogate pair");
                            u = 0x10000 + ((u - 0xD800) << 10) + (l - 0xDC00);
                        }
                        put_utf8(o, u);
                        break;
                    }
                    default: fail("bad escape");
                }
                continue;
            }
            if (c < 0x80) { o.push_back((char)c); continue; }
            // validate one UTF-8 sequence (no overlongs, no surrogates, <= U+10FFFF)
            int len;
            uint32_t cp;
            if (c >= 0xC2 && c <= 0xDF) { len = 2; cp = c & 0x1F; }
            else if (c >= 0xE0 && c <= 0xEF) { len = 3; cp = c & 0x0F; }
            else if (c >= 0xF0 && c <= 0xF4) { len = 4; cp = c & 0x07; }
            else fail("invalid UTF-8");
            if (p_ + len - 1 > s_.size()) fail("invalid UTF-8");
            for (int k = 1; k < len; ++k) {
                const uint8_t cc = (uint8_t)s_[p_ + k - 1];
                if ((cc & 0xC0) != 0x80) fail("invalid UTF-8");
                cp = cp << 6 | (cc & 0x3F);
            }
            if ((len == 3 && (cp < 0x800 || (cp >= 0xD800 && cp <= 0xDFFF))) || (len == 4 && (cp < 0x10000 || cp > 0x10FFFF)))
                fail("invalid UTF-8");
            o.append(s_.substr(p_ - 1, len));
            p_ += len - 1;
        }
    }
    Guid guid_key() {  // "D" Guid key of a PNC vector (Guid's property-name converter unescapes first)
        Guid g;
        if (!ParseGuidD(string(), g)) fail("not a Guid");
        return g;
    }
    Guid guid_value() {  // Guid string inside a tag array (escapes allowed: STJ unescapes values)
        Guid g;
        if (!ParseGuidD(string(), g)) fail("not a Guid");
        return g;
    }
    template <class T> T integer() {
        ws();
        const size_t b = p_;
        bool neg = false;
        if (p_ < s_.size() && s_[p_] == '-') { neg = true; ++p_; }
        if (p_ >= s_.size() || s_[p_] < '0' || s_[p_] > '9') fail("not a number");
        if (s_[p_] == '0' && p_ + 1 < s_.size() && s_[p_ + 1] >= '0' && s_[p_ + 1] <= '9') fail("leading zero");
        unsigned __int128 mag = 0;
        while (p_ < s_.size() && s_[p_] >= '0' && s_[p_] <= '9') {
            mag = mag * 10 + (unsigned)(s_[p_++] - '0');
            if (mag > ((unsigned __int128)1 << 64)) fail("number out of range");
        }
        if (p_ < s_.size() && (s_[p_] == '.' || s_[p_] == 'e' || s_[p_] == 'E')) fail("not an integer");
        const unsigned __int128 lim = neg ? (unsigned __int128)std::numeric_limits<T>::max() + 1 : (unsigned __int128)std::numeric_limits<T>::max();
        if (mag > lim) fail("number out of range");
        (void)b;
        return neg ? (T)(-(__int128)mag) : (T)mag;
    }
    bool null_literal() {
        ws();
        if (s_.substr(p_, 4) == "null") { p_ += 4; return true; }
        return false;
    }
    // One JSON value of an unmapped member, validated and dropped.  `depth` = the containers open around it
    // (the message object = 1); a container that would open level 65 fails (JsonReaderOptions.MaxDepth 64).
    void skip_value(int depth) {
        ws();
        if (p_ >= s_.size()) fail("unexpected end");
        const char c = s_[p_];
        if (c == '{' || c == '[') {
            if (depth + 1 > kMaxDepth) fail("depth past MaxDepth");
            ++p_;
            const char close = c == '{' ? '}' : ']';
            if (eat(close)) return;
            do {
                if (c == '{') {
                    (void)string();
                    expect(':');
                }
                skip_value(depth + 1);
            } while (eat(','));
            expect(close);
            return;
        }
        if (c == '"') { (void)string(); return; }
        if (s_.compare(p_, 4, "true") == 0) { p_ += 4; return; }
        if (s_.compare(p_, 5, "false") == 0) { p_ += 5; return; }
        if (s_.compare(p_, 4, "null") == 0) { p_ += 4; return; }
        // -?(0|[1-9][0-9]*)(.[0-9]+)?([eE][+-]?[0-9]+)?
        if (s_[p_] == '-') ++p_;
        auto digits = [&] {
            const size_t b = p_;
            while (p_ < s_.size() && s_[p_] >= '0' && s_[p_] <= '9') ++p_;
            return p_ - b;
        };
        if (p_ >= s_.size() || s_[p_] < '0' || s_[p_] > '9') fail("not a value");
        if (s_[p_] == '0') ++p_;
        else digits();
        if (p_ < s_.size() && s_[p_] == '.') {
            ++p_;
            if (!digits()) fail("bad number");
        }
        if (p_ < s_.size() && (s_[p_] == 'e' || s_[p_] == 'E')) {
            ++p_;
            if (p_ < s_.size() && (s_[p_] == '+' || s_[p_] == '-')) ++p_;
            if (!digits()) fail("bad number");
        }
        if (p_ < s_.size() && ((s_[p_] >= '0' && s_[p_] <= '9') || s_[p_] == '.' || s_[p_] == 'e' || s_[p_] == 'E' || s_[p_] == '-' || s_[p_] == '+'))
            fail("bad number");
    }
    static constexpr int kMaxDepth = 64;

  private:
    uint32_t hex4() {
        if (p_ + 4 > s_.size()) fail("bad \\u escape");
        uint32_t u = 0;
        for (int k = 0; k < 4; ++k) {
            const int h = hexval(s_[p_++]);
            if (h < 0) fail("bad \\u escape");
            u = u << 4 | (uint32_t)h;
        }
        return u;
    }
    static void put_utf8(std::string& o, uint32_t u) {
        if (u < 0x80) o.push_back((char)u);
        else if (u < 0x800) { o.push_back((char)(0xC0 | u >> 6)); o.push_back((char)(0x80 | (u & 0x3F))); }
        else if (u < 0x10000) {
            o.push_back((char)(0xE0 | u >> 12)); o.push_back((char)(0x80 | ((u >> 6) & 0x3F))); o.push_back((char)(0x80 | (u & 0x3F)));
        } else {
            o.push_back((char)(0xF0 | u >> 18)); o.push_back((char)(0x80 | ((u >> 12) & 0x3F)));
            o.push_back((char)(0x80 | ((u >> 6) & 0x3F))); o.push_back((char)(0x80 | (u & 0x3F)));
        }
    }
    std::string_view s_;
    size_t p_ = 0;
};

template <class T> PNCounterMsg<T> DecodePNC(std::string_view bytes) {  // PNCounters.cs:38-43
    Reader r(bytes);
    PNCounterMsg<T> m;
    bool seen[2] = {false, false}, null_last[2] = {false, false};
    r.expect('{');
    if (!r.peek('}')) {
        do {
            const std::string name = r.string();
            r.expect(':');
            const int which = name == "pVector" ? 0 : name == "nVector" ? 1 : -1;
            if (which < 0) {  // not a member: skipped
                r.skip_value(1);
                continue;
            }
            seen[which] = true;  // a repeat replaces the earlier value (the field is assigned again)
            auto& d = which ? m.nVector : m.pVector;
            d.Clear();
            null_last[which] = r.null_literal();
            if (null_last[which]) continue;
            r.expect('{');
            if (!r.peek('}')) {
                do {
                    const Guid g = r.guid_key();
                    r.expect(':');
                    d[g] = r.integer<T>();  // Dictionary indexer: a repeated key keeps its place, takes the last value
                } while (r.eat(','));
            }
            r.expect('}');
        } while (r.eat(','));
    }
    r.expect('}');
    r.end();
    for (int k = 0; k < 2; ++k)
        if (!seen[k] || null_last[k]) r.fail("missing or null vector (Merge would throw NullReferenceException)");
    return m;
}

inline ORSetMsg DecodeORSet(std::string_view bytes) {  // ORSet.cs:56-63
    Reader r(bytes);
    ORSetMsg m;
    bool seen[4] = {false, false, false, false}, null_last[4] = {false, false, false, false};
    r.expect('{');
    if (!r.peek('}')) {
        do {
            const std::string name = r.string();
            r.expect(':');
            const int which = name == "addSet" ? 0 : name == "removeSet" ? 1 : name == "nullAddGuid" ? 2 : name == "nullRemoveGuid" ? 3 : -1;
            if (which < 0) {  // not a member: skipped
                r.skip_value(1);
                continue;
            }
            seen[which] = true;
            null_last[which] = r.null_literal();
            auto tags = [&](GuidSet& s) {
                r.expect('[');
                if (!r.peek(']')) {
                    do { s.insert(r.guid_value()); } while (r.eat(','));
                }
                r.expect(']');
            };
            if (which < 2) {
                auto& d = which ? m.removeSet : m.addSet;
                d.Clear();
                if (null_last[which]) continue;
                OrderedDict<std::string, bool> nulls;  // elements whose latest tag set is `null`
                r.expect('{');
                if (!r.peek('}')) {
                    do {
                        std::string e = r.string();
                        r.expect(':');
                        GuidSet s;
                        const bool is_null = r.null_literal();
                        if (!is_null) tags(s);
                        d[e] = std::move(s);  // Dictionary indexer: first position, last value
                        nulls[e] = is_null;
                    } while (r.eat(','));
                }
                r.expect('}');
                for (const auto& kv : nulls)
                    if (kv.second) r.fail("null tag set (Merge's UnionWith would throw ArgumentNullException)");
            } else {
                auto& s = which == 2 ? m.nullAddGuid : m.nullRemoveGuid;
                s = GuidSet();
                if (!null_last[which]) tags(s);
            }
        } while (r.eat(','));
    }
    r.expect('}');
    r.end();
    for (int k = 0; k < 4; ++k)
        if (!seen[k] || null_last[k]) r.fail("missing or null member (Merge would throw NullReferenceException)");
    return m;
}

}  // namespace oracle::json
