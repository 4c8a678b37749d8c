// wire.cpp — see wire.hpp.
#include "wire.hpp"

#include <cstring>
#include <unordered_map>
#include <unordered_set>

namespace janus::wire {

namespace {

constexpr char kHex[] = "0123456789abcdef";

inline void put_byte_hex(char* d, uint8_t b) {
    d[0] = kHex[b >> 4];
    d[1] = kHex[b & 15];
}

inline int hex_digit(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    const char l = (char)(c | 0x20);
    return (l >= 'a' && l <= 'f') ? l - 'a' + 10 : -1;
}

[[noreturn]] void reject(const char* why, size_t at) {
    throw EngineError(JG_EINVAL, std::string("JsonException: ") + why + " at byte " + std::to_string(at));
}

// Cursor over one payload; each method consumes one JSON token (with leading whitespace).
struct Scan {
    std::string_view s;
    size_t i = 0;
    void skip_ws() {
        while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i;
    }
    bool at(char c) {
        skip_ws();
        return i < s.size() && s[i] == c;
    }
    void need(char c) {
        if (!at(c)) reject("unexpected token", i);
        ++i;
    }
    bool take(char c) {
        if (!at(c)) return false;
        ++i;
        return true;
    }
    bool take_null() {
        skip_ws();
        if (s.compare(i, 4, "null") == 0) { i += 4; return true; }
        return false;
    }
    uint32_t hex4() {
        if (i + 4 > s.size()) reject("bad \\u escape", i);
        uint32_t u = 0;
        for (int k = 0; k < 4; ++k) {
            const int h = hex_digit(s[i++]);
            if (h < 0) reject("bad \\u escape", i);
            u = u << 4 | (uint32_t)h;
        }
        return u;
    }
    static void utf8(std::string& o, uint32_t u) {
        if (u < 0x80) { o += (char)u; return; }
        if (u < 0x800) { o += (char)(0xC0 | u >> 6); o += (char)(0x80 | (u & 0x3F)); return; }
        if (u < 0x10000) { o += (char)(0xE0 | u >> 12); o += (char)(0x80 | (u >> 6 & 0x3F)); o += (char)(0x80 | (u & 0x3F)); return; }
        o += (char)(0xF0 | u >> 18); o += (char)(0x80 | (u >> 12 & 0x3F)); o += (char)(0x80 | (u >> 6 & 0x3F)); o += (char)(0x80 | (u & 0x3F));
    }
    // JSON string -> UTF-8 (escapes decoded, surrogate pairs joined, raw UTF-8 validated).
    std::string str() {
        need('"');
        {   // fast path: printable ASCII without escapes up to the closing quote (every string the
            // reference's encoder writes for a Guid, and JavaScriptEncoder.Default output of ASCII text)
            size_t j = i;
            while (j < s.size()) {
                const unsigned char c = (unsigned char)s[j];
                if (c == '"' || c == '\\' || c < 0x20 || c >= 0x80) break;
                ++j;
            }
            if (j < s.size() && s[j] == '"') {
                std::string o(s.data() + i, j - i);
                i = j + 1;
                return o;
            }
        }
        std::string o;
        while (true) {
            if (i >= s.size()) reject("unterminated string", i);
            const unsigned char c = (unsigned char)s[i++];
            if (c == '"') return o;
            if (c < 0x20) reject("control character in string", i);
            if (c == '\\') {
                if (i >= s.size()) reject("bad escape", i);
                const char e = s[i++];
                const char* simple = std::strchr("\"\\/bfnrt", e);
                if (e && simple) {
                    static const char out[] = "\"\\/\b\f\n\r\t";
                    o += out[simple - "\"\\/bfnrt"];
                    continue;
                }
                if (e != 'u') reject("bad escape", i);
                uint32_t u = hex4();
                if (u >= 0xDC00 && u <= 0xDFFF) reject("lone low surrogate", i);
                if (u >= 0xD800 && u <= 0xDBFF) {
                    if (i + 2 > s.size() || s[i] != '\\' || s[i + 1] != 'u') reject("lone high surrogate", i);
                    i += 2;
                    const uint32_t lo = hex4();
                    if (lo < 0xDC00 || lo > 0xDFFF) reject("bad surrogate pair", i);
                    u = 0x10000 + ((u - 0xD800) << 10) + (lo - 0xDC00);
                }
                utf8(o, u);
                continue;
            }
            if (c < 0x80) { o += (char)c; continue; }
            int extra;
            uint32_t cp;
            if (c >= 0xC2 && c <= 0xDF) { extra = 1; cp = c & 0x1F; }
            else if (c >= 0xE0 && c <= 0xEF) { extra = 2; cp = c & 0x0F; }
            else if (c >= 0xF0 && c <= 0xF4) { extra = 3; cp = c & 0x07; }
            else reject("invalid UTF-8", i);
            if (i + extra > s.size()) reject("invalid UTF-8", i);
            for (int k = 0; k < extra; ++k) {
                const unsigned char cc = (unsigned char)s[i + k];
                if ((cc & 0xC0) != 0x80) reject("invalid UTF-8", i);
                cp = cp << 6 | (cc & 0x3F);
            }
            const bool bad = (extra == 2 && (cp < 0x800 || (cp >= 0xD800 && cp <= 0xDFFF))) || (extra == 3 && (cp < 0x10000 || cp > 0x10FFFF));
            if (bad) reject("invalid UTF-8", i);
            o.append(s.data() + i - 1, (size_t)extra + 1);
            i += extra;
        }
    }
    // The string as a view into the payload when it has no escapes, else decoded into `scratch`.
    std::string_view str_view(std::string& scratch) {
        skip_ws();
        if (i < s.size() && s[i] == '"') {
            size_t j = i + 1;
            while (j < s.size()) {
                const unsigned char c = (unsigned char)s[j];
                if (c == '"' || c == '\\' || c < 0x20 || c >= 0x80) break;
                ++j;
            }
            if (j < s.size() && s[j] == '"') {
                const std::string_view v = s.substr(i + 1, j - i - 1);
                i = j + 1;
                return v;
            }
        }
        scratch = str();
        return scratch;
    }
    Guid guid() {
        const size_t at = i;
        Guid g;
        skip_ws();
        // fast path: "<36 chars>" parsed in place (no escapes can occur in a valid Guid string)
        if (i + 38 <= s.size() && s[i] == '"' && s[i + 37] == '"' && ParseGuidD(s.substr(i + 1, 36), g)) {
            i += 38;
            return g;
        }
        if (!ParseGuidD(str(), g)) reject("not a Guid", at);
        return g;
    }
    void guids(std::vector<Guid>& out) {
        need('[');
        if (!at(']')) {
            do out.push_back(guid());
            while (take(','));
        }
        need(']');
    }
    // An unmapped member's value, validated and dropped (oracle/json.hpp: MaxDepth 64 counting the message object).
    void skip_value(int depth) {
        skip_ws();
        if (i >= s.size()) reject("unexpected end", i);
        const char c = s[i];
        if (c == '{' || c == '[') {
            if (depth + 1 > 64) reject("depth past MaxDepth", i);
            ++i;
            const char close = c == '{' ? '}' : ']';
            if (take(close)) return;
            do {
                if (c == '{') {
                    (void)str();
                    need(':');
                }
                skip_value(depth + 1);
            } while (take(','));
            need(close);
            return;
        }
        if (c == '"') { (void)str(); return; }
        for (const char* lit : {"true", "false", "null"})
            if (s.compare(i, std::strlen(lit), lit) == 0) { i += std::strlen(lit); return; }
        auto digits = [&] {
            const size_t b = i;
            while (i < s.size() && s[i] >= '0' && s[i] <= '9') ++i;
            return i - b;
        };
        if (s[i] == '-') ++i;
        if (i >= s.size() || s[i] < '0' || s[i] > '9') reject("not a value", i);
        if (s[i] == '0') ++i;
        else digits();
        if (i < s.size() && s[i] == '.') {
            ++i;
            if (!digits()) reject("bad number", i);
        }
        if (i < s.size() && (s[i] == 'e' || s[i] == 'E')) {
            ++i;
            if (i < s.size() && (s[i] == '+' || s[i] == '-')) ++i;
            if (!digits()) reject("bad number", i);
        }
        if (i < s.size() && std::strchr("0123456789.eE+-", s[i])) reject("bad number", i);
    }
};

// JavaScriptEncoder.Default for a UTF-8 element string.
void escape(std::string& o, const std::string& s) {
    static const char HX[] = "0123456789ABCDEF";
    auto unit = [&](uint32_t u) {
        const char e[6] = {'\\', 'u', HX[u >> 12 & 15], HX[u >> 8 & 15], HX[u >> 4 & 15], HX[u & 15]};
        o.append(e, 6);
    };
    size_t i = 0;
    while (i < s.size()) {
        const unsigned char c = (unsigned char)s[i];
        if (c >= 0x80) {
            const int n = c >= 0xF0 ? 4 : c >= 0xE0 ? 3 : 2;
            uint32_t cp = c & (n == 4 ? 0x07 : n == 3 ? 0x0F : 0x1F);
            for (int k = 1; k < n; ++k) cp = cp << 6 | ((unsigned char)s[i + k] & 0x3F);
            i += n;
            if (cp >= 0x10000) {
                unit(0xD800 | (cp - 0x10000) >> 10);
                unit(0xDC00 | ((cp - 0x10000) & 0x3FF));
            } else {
                unit(cp);
            }
            continue;
        }
        ++i;
        if (c == '\\') o += "\\\\";
        else if (c == '\b') o += "\\b";
        else if (c == '\t') o += "\\t";
        else if (c == '\n') o += "\\n";
        else if (c == '\f') o += "\\f";
        else if (c == '\r') o += "\\r";
        else if (c < 0x20 || c == 0x7F || std::strchr("\"&'+<>`", (char)c)) unit(c);
        else o += (char)c;
    }
}

void put_tags(std::string& o, const std::vector<Guid>& v) {
    o += '[';
    for (size_t k = 0; k < v.size(); ++k) {
        if (k) o += ',';
        o += '"';
        AppendGuidD(o, v[k]);
        o += '"';
    }
    o += ']';
}

void put_map(std::string& o, const std::vector<std::pair<std::string, std::vector<Guid>>>& m) {
    o += '{';
    for (size_t k = 0; k < m.size(); ++k) {
        if (k) o += ',';
        o += '"';
        escape(o, m[k].first);
        o += "\":";
        put_tags(o, m[k].second);
    }
    o += '}';
}

}  // namespace

void AppendGuidD(std::string& out, const Guid& g) {
    // text order of the 16 bytes: b3 b2 b1 b0 - b5 b4 - b7 b6 - b8 b9 - b10..b15
    char d[36];
    const uint64_t lo = g.lo, hi = g.hi;
    static const int lo_order[8] = {3, 2, 1, 0, 5, 4, 7, 6};
    int p = 0;
    for (int k = 0; k < 8; ++k) {
        if (k == 4 || k == 6) d[p++] = '-';
        put_byte_hex(d + p, (uint8_t)(lo >> (8 * lo_order[k])));
        p += 2;
    }
    for (int k = 0; k < 8; ++k) {
        if (k == 0 || k == 2) d[p++] = '-';
        put_byte_hex(d + p, (uint8_t)(hi >> (8 * k)));
        p += 2;
    }
    out.append(d, 36);
}

bool ParseGuidD(std::string_view s, Guid& g) {
    if (s.size() != 36 || s[8] != '-' || s[13] != '-' || s[18] != '-' || s[23] != '-') return false;
    // 256-entry nibble table (0xFF = not a hex digit); bytes in text order, then placed
    static const struct Tab {
        uint8_t v[256];
        Tab() {
            for (int c = 0; c < 256; ++c) v[c] = 0xFF;
            for (int c = 0; c < 10; ++c) v['0' + c] = (uint8_t)c;
            for (int c = 0; c < 6; ++c) v['a' + c] = v['A' + c] = (uint8_t)(10 + c);
        }
    } T;
    static const int pos[16] = {0, 2, 4, 6, 9, 11, 14, 16, 19, 21, 24, 26, 28, 30, 32, 34};
    static const int lo_order[8] = {3, 2, 1, 0, 5, 4, 7, 6};
    const unsigned char* p = reinterpret_cast<const unsigned char*>(s.data());
    uint8_t b[16];
    unsigned bad = 0;
    for (int k = 0; k < 16; ++k) {
        const uint8_t a = T.v[p[pos[k]]], c = T.v[p[pos[k] + 1]];
        bad |= (a | c) & 0xF0;
        b[k] = (uint8_t)(a << 4 | (c & 15));
    }
    if (bad) return false;
    uint64_t lo = 0, hi = 0;
    for (int k = 0; k < 8; ++k) lo |= (uint64_t)b[k] << (8 * lo_order[k]);
    for (int k = 0; k < 8; ++k) hi |= (uint64_t)b[8 + k] << (8 * k);
    g.lo = lo;
    g.hi = hi;
    return true;
}

void AppendPNCounterMsg(std::string& out, const Guid* g, const int64_t* p, const int64_t* n, size_t k) {
    char num[24];
    for (int which = 0; which < 2; ++which) {
        out += which ? ",\"nVector\":{" : "{\"pVector\":{";
        const int64_t* v = which ? n : p;
        for (size_t j = 0; j < k; ++j) {
            if (j) out += ',';
            out += '"';
            AppendGuidD(out, g[j]);
            out += "\":";
            const int len = std::snprintf(num, sizeof num, "%lld", (long long)v[j]);
            out.append(num, (size_t)len);
        }
        out += '}';
    }
    out += '}';
}

std::string EncodeORSetMsg(const ORSetState& m) {
    std::string o = "{\"addSet\":";
    put_map(o, m.addSet);
    o += ",\"removeSet\":";
    put_map(o, m.removeSet);
    o += ",\"nullAddGuid\":";
    put_tags(o, m.nullAddGuid);
    o += ",\"nullRemoveGuid\":";
    put_tags(o, m.nullRemoveGuid);
    o += '}';
    return o;
}

ORSetState DecodeORSetMsg(std::string_view bytes) {
    Scan sc{bytes};
    ORSetState m;
    bool seen[4] = {false, false, false, false}, null_last[4] = {false, false, false, false};
    sc.need('{');
    if (!sc.at('}')) {
        do {
            const std::string name = sc.str();
            static const char* names[4] = {"addSet", "removeSet", "nullAddGuid", "nullRemoveGuid"};
            int which = -1;
            for (int k = 0; k < 4; ++k)
                if (name == names[k]) which = k;
            sc.need(':');
            if (which < 0) {  // not a member: skipped (System.Text.Json's default)
                sc.skip_value(1);
                continue;
            }
            seen[which] = true;  // a repeated member: the last occurrence wins
            null_last[which] = sc.take_null();
            if (which >= 2) {
                auto& v = which == 2 ? m.nullAddGuid : m.nullRemoveGuid;
                v.clear();
                if (!null_last[which]) sc.guids(v);
                continue;
            }
            auto& map = which == 0 ? m.addSet : m.removeSet;
            map.clear();
            if (null_last[which]) continue;
            std::unordered_map<std::string, size_t> at;  // element -> its place (Dictionary indexer: first place, last value)
            std::vector<bool> is_null;
            sc.need('{');
            if (!sc.at('}')) {
                do {
                    std::string e = sc.str();
                    sc.need(':');
                    const bool nul = sc.take_null();
                    std::vector<Guid> tags;
                    if (!nul) sc.guids(tags);
                    auto it = at.find(e);
                    if (it == at.end()) {
                        at.emplace(e, map.size());
                        map.emplace_back(std::move(e), std::move(tags));
                        is_null.push_back(nul);
                    } else {
                        map[it->second].second = std::move(tags);
                        is_null[it->second] = nul;
                    }
                } while (sc.take(','));
            }
            sc.need('}');
            for (bool b : is_null)
                if (b) reject("null tag set (Merge's UnionWith would throw)", sc.i);
        } while (sc.take(','));
    }
    sc.need('}');
    sc.skip_ws();
    if (sc.i != bytes.size()) reject("trailing data", sc.i);
    for (int k = 0; k < 4; ++k)
        if (!seen[k] || null_last[k]) reject("missing or null member (Merge would throw NullReferenceException)", sc.i);
    return m;
}

void ScanORSetMsg(std::string_view bytes, ORSetEntryFn fn, void* ctx) {
    // the decoded state in ORSet.Merge's walk (ORSet.cs:255-282): addSet entries, removeSet entries, null tag sets
    const ORSetState m = DecodeORSetMsg(bytes);
    for (const auto& e : m.addSet) fn(ctx, 0, e.first, false, e.second.data(), e.second.size());
    for (const auto& e : m.removeSet) fn(ctx, 1, e.first, false, e.second.data(), e.second.size());
    fn(ctx, 0, std::string_view(), true, m.nullAddGuid.data(), m.nullAddGuid.size());
    fn(ctx, 1, std::string_view(), true, m.nullRemoveGuid.data(), m.nullRemoveGuid.size());
}

}  // namespace janus::wire
