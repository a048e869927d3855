// mt_snapdec.cpp -- native host decoder of SnapshotV1 summaries (include/mt_snapshot.h).
//
// The host half of a cold catch-up (config C5): summary blobs (JSON text) -> mt_seg_rec
// records + text / props arenas for mt_load_snapshots.  Semantics follow the reference
// loader and fluidframework_amd/snapshot.py, its Python restatement:
//   SnapshotLoader.initialize :36-84, loadHeader :120-159, loadBody :161-228,
//   specToSegment :86-118 (MT/snapshotLoader.ts); SnapshotV1.processChunk (MT/snapshotV1.ts:
//   266-277); toLatestVersion / buildHeaderMetadataForLegecyChunk (MT/snapshotChunks.ts:
//   136-188); hasMergeInfo (:72-74).
// Phase 1: `threads` workers take documents dynamically; each parses the document's blobs
// into a flat node array (24-byte nodes in pre-order, strings decoded to UTF-16 units as JS
// holds them, numbers left as lexemes in the source; the buffers are reused, so a worker
// allocates almost nothing) and builds its records with document-local property ids.
// Phase 2 maps local ids to the batch's ids, which numbers keys / values first-seen in
// document order, exactly as wire.Interner does, and places every document in the output;
// mt_snapdec_fetch then concatenates the documents straight into the caller's arrays, in
// parallel (each document's slice is known).
#include <algorithm>
#include <atomic>
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/mt_snapshot.h"

namespace {

constexpr uint32_t NONE = 0xFFFFFFFFu;

// ---------------------------------------------------------------- JSON (RFC 8259)
struct Node {
    enum : uint8_t { NUL, BOOL, NUM, STR, ARR, OBJ };
    uint8_t t = NUL, b = 0;
    uint32_t off = 0, len = 0;   // STR: units in Blob::str; NUM: bytes of the source; ARR/OBJ: -, count
    uint32_t next = 0;           // next sibling (0: none -- the root is never a sibling)
    uint32_t koff = 0, klen = 0; // object member: its key (units in Blob::str)
};
static_assert(sizeof(Node) == 24, "node layout");

struct Blob {
    const char *src = nullptr;
    size_t n = 0;
    std::string path;
    std::vector<Node> nodes;     // pre-order: a container's first child is the next node
    std::vector<char16_t> str;   // decoded string units [0, slen); sized once per blob to an
    uint32_t slen = 0;           // upper bound (a byte never yields more than one unit)

    const char16_t *s(uint32_t off) const { return str.data() + off; }
    uint32_t first(uint32_t i) const { return nodes[i].len ? i + 1 : NONE; }
    static bool eq(const char16_t *u, uint32_t n, const char *k) {
        uint32_t i = 0;
        for (; i < n && k[i]; i++)
            if (u[i] != (char16_t)(unsigned char)k[i]) return false;
        return i == n && !k[i];
    }
    bool is_str(uint32_t i, const char *k) const {
        return i != NONE && nodes[i].t == Node::STR && eq(s(nodes[i].off), nodes[i].len, k);
    }
    // member k of object i (a duplicated member: the last value, as JSON.parse)
    uint32_t get(uint32_t i, const char *k) const {
        if (i == NONE || nodes[i].t != Node::OBJ) return NONE;
        uint32_t r = NONE;
        uint32_t c = first(i);
        for (uint32_t m = 0; m < nodes[i].len; m++, c = nodes[c].next)
            if (eq(s(nodes[c].koff), nodes[c].klen, k)) r = c;
        return r;
    }
    // members of object i named keys[0 .. n) -> out[0 .. n) (NONE if absent; the last of
    // duplicated members, as get)
    void fields(uint32_t i, const char *const *keys, int n, uint32_t *out) const {
        uint32_t c = first(i);
        for (uint32_t m = 0; m < nodes[i].len; m++, c = nodes[c].next)
            for (int k = 0; k < n; k++)
                if (eq(s(nodes[c].koff), nodes[c].klen, keys[k])) {
                    out[k] = c;
                    break;
                }
    }
    bool present(uint32_t i) const { return i != NONE && nodes[i].t != Node::NUL; }
    std::u16string ustr(uint32_t i) const { return std::u16string(s(nodes[i].off), nodes[i].len); }
    bool is_int(uint32_t i) const {
        const char *p = src + nodes[i].off;
        for (uint32_t k = 0; k < nodes[i].len; k++)
            if (p[k] == '.' || p[k] == 'e' || p[k] == 'E') return false;
        return true;
    }
    double num(uint32_t i) const {   // JS Number of the lexeme (locale-independent)
        double x = 0;
        const char *b = src + nodes[i].off, *e = b + nodes[i].len;
        const auto r = std::from_chars(b, e, x);
        if (r.ec == std::errc::result_out_of_range) {
            // JSON.parse / json.loads: overflow is +-Infinity, underflow +-0
            bool big = false;
            for (const char *q = b; q < e; q++)
                if (*q == 'e' || *q == 'E') {
                    big = q + 1 < e && q[1] != '-';
                    break;
                }
            if (!big) {   // no exponent or a positive one: too many digits, i.e. overflow
                bool has_e = false;
                for (const char *q = b; q < e; q++) has_e |= (*q == 'e' || *q == 'E');
                big = !has_e;
            }
            const bool neg = *b == '-';
            x = big ? (neg ? -HUGE_VAL : HUGE_VAL) : (neg ? -0.0 : 0.0);
        }
        return x;
    }
    int64_t as_int(uint32_t i) const {
        if (i == NONE || nodes[i].t != Node::NUM) return 0;
        if (!is_int(i) || nodes[i].len > 18) {   // clamp before the cast (out of range is UB)
            const double x = num(i);
            if (!(x == x)) return 0;
            if (x >= 9.2e18) return INT64_MAX;
            if (x <= -9.2e18) return INT64_MIN;
            return (int64_t)x;
        }
        const char *p = src + nodes[i].off;
        const bool neg = *p == '-';
        int64_t v = 0;
        for (uint32_t k = neg; k < nodes[i].len; k++) v = v * 10 + (p[k] - '0');
        return neg ? -v : v;
    }
    // own members of object i in insertion order: a duplicated key keeps its first position
    // and takes its last value (JSON.parse and json.loads agree)
    void members(uint32_t i, std::vector<uint32_t> &out) const {
        out.clear();
        uint32_t c = first(i);
        for (uint32_t m = 0; m < nodes[i].len; m++, c = nodes[c].next) {
            bool dup = false;
            for (auto &x : out)
                if (nodes[x].klen == nodes[c].klen &&
                    !memcmp(s(nodes[x].koff), s(nodes[c].koff), nodes[c].klen * sizeof(char16_t))) {
                    x = c;
                    dup = true;
                    break;
                }
            if (!dup) out.push_back(c);
        }
    }
};

struct Reader {
    const char *p, *e;
    Blob &B;
    std::string err;

    void ws() {
        while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) p++;
    }
    bool fail(const char *m) {
        if (err.empty()) err = m;
        return false;
    }
    static int hex(char c) {
        if (c >= '0' && c <= '9') return c - '0';
        if (c >= 'a' && c <= 'f') return c - 'a' + 10;
        if (c >= 'A' && c <= 'F') return c - 'A' + 10;
        return -1;
    }
    // a string into B.str (UTF-8 -> UTF-16 units; \u escapes kept as units, lone surrogates too)
    bool str(uint32_t &off, uint32_t &len) {
        if (p >= e || *p != '"') return fail("expected a string");
        p++;
        char16_t *o = B.str.data();   // room for every remaining byte (parse sizes it)
        uint32_t w = B.slen;
        off = w;
        for (;;) {
            {   // ASCII run: 8 bytes at a time up to the first '"', '\\', control or non-ASCII byte
                const char *q = p;
                while (e - q >= 8) {
                    uint64_t x;
                    memcpy(&x, q, 8);
                    const uint64_t hi = 0x8080808080808080ull, one = 0x0101010101010101ull;
                    const uint64_t qt = x ^ (one * 0x22), bs = x ^ (one * 0x5C);
                    const uint64_t stop = (x | ((qt - one) & ~qt) | ((bs - one) & ~bs) | ((x - one * 0x20) & ~x)) & hi;
                    if (stop) {
                        q += __builtin_ctzll(stop) >> 3;
                        goto run_end;
                    }
                    q += 8;
                }
                while (q < e) {
                    const unsigned char c = (unsigned char)*q;
                    if (c < 0x20 || c >= 0x80 || c == '"' || c == '\\') break;
                    q++;
                }
            run_end:
                const size_t k = (size_t)(q - p);
                for (size_t i = 0; i < k; i++) o[w + i] = (char16_t)(unsigned char)p[i];
                w += (uint32_t)k;
                p = q;
            }
            if (p >= e) return fail("unterminated string");
            const unsigned char c = (unsigned char)*p;
            if (c == '"') break;
            if (c == '\\') {
                if (++p >= e) return fail("bad escape");
                const char x = *p++;
                switch (x) {
                    case '"': o[w++] = u'"'; break;
                    case '\\': o[w++] = u'\\'; break;
                    case '/': o[w++] = u'/'; break;
                    case 'b': o[w++] = u'\b'; break;
                    case 'f': o[w++] = u'\f'; break;
                    case 'n': o[w++] = u'\n'; break;
                    case 'r': o[w++] = u'\r'; break;
                    case 't': o[w++] = u'\t'; break;
                    case 'u': {
                        if (e - p < 4) return fail("bad \\u escape");
                        int v = 0;
                        for (int i = 0; i < 4; i++) {
                            const int h = hex(p[i]);
                            if (h < 0) return fail("bad \\u escape");
                            v = v * 16 + h;
                        }
                        p += 4;
                        o[w++] = (char16_t)v;
                        break;
                    }
                    default: return fail("bad escape");
                }
                continue;
            }
            if (c < 0x20) return fail("control character in string");
            // UTF-8 -> UTF-16 as the reference's Buffer.toString("utf8") (fromBase64ToUtf8):
            // each maximal ill-formed subsequence becomes one U+FFFD, and the byte that ends it
            // is read again (WHATWG "UTF-8 decode"; overlong forms, encoded surrogates and code
            // points above U+10FFFF are ill-formed)
            uint32_t cp;
            int n;
            unsigned lo = 0x80, hi = 0xBF;
            if (c >= 0xC2 && c <= 0xDF) { cp = c & 0x1F; n = 1; }
            else if (c >= 0xE0 && c <= 0xEF) { cp = c & 0x0F; n = 2; lo = c == 0xE0 ? 0xA0 : 0x80; hi = c == 0xED ? 0x9F : 0xBF; }
            else if (c >= 0xF0 && c <= 0xF4) { cp = c & 0x07; n = 3; lo = c == 0xF0 ? 0x90 : 0x80; hi = c == 0xF4 ? 0x8F : 0xBF; }
            else { p++; o[w++] = u'\uFFFD'; continue; }
            p++;
            bool ok = true;
            for (int i = 0; i < n; i++) {
                const unsigned x = p < e ? (unsigned char)*p : 0;
                if (p >= e || x < lo || x > hi) { ok = false; break; }
                lo = 0x80, hi = 0xBF;
                cp = (cp << 6) | (x & 0x3F);
                p++;
            }
            if (!ok) { o[w++] = u'\uFFFD'; continue; }
            if (cp >= 0x10000) {   // 4 bytes -> 2 units
                cp -= 0x10000;
                o[w++] = (char16_t)(0xD800 + (cp >> 10));
                o[w++] = (char16_t)(0xDC00 + (cp & 0x3FF));
            } else {
                o[w++] = (char16_t)cp;
            }
        }
        p++;
        B.slen = w;
        len = w - off;
        return true;
    }
    uint32_t node(uint8_t t) {
        B.nodes.emplace_back();
        B.nodes.back().t = t;
        return (uint32_t)B.nodes.size() - 1;
    }
    bool val(uint32_t &out, int depth = 0) {
        if (depth > 512) return fail("nesting too deep");
        ws();
        if (p >= e) return fail("unexpected end");
        const char c = *p;
        if (c == '{' || c == '[') {
            const bool obj = c == '{';
            const uint32_t me = out = node(obj ? Node::OBJ : Node::ARR);
            p++;
            ws();
            if (p < e && *p == (obj ? '}' : ']')) { p++; return true; }
            uint32_t prev = NONE, count = 0;
            for (;;) {
                uint32_t ko = 0, kl = 0, ch;
                if (obj) {
                    ws();
                    if (!str(ko, kl)) return false;
                    ws();
                    if (p >= e || *p != ':') return fail("expected ':'");
                    p++;
                }
                if (!val(ch, depth + 1)) return false;
                B.nodes[ch].koff = ko;
                B.nodes[ch].klen = kl;
                if (prev != NONE) B.nodes[prev].next = ch;
                prev = ch;
                count++;
                ws();
                if (p < e && *p == ',') { p++; continue; }
                if (p < e && *p == (obj ? '}' : ']')) { p++; break; }
                return fail(obj ? "expected ',' or '}'" : "expected ',' or ']'");
            }
            B.nodes[me].len = count;
            return true;
        }
        if (c == '"') {
            uint32_t o, l;
            if (!str(o, l)) return false;
            out = node(Node::STR);
            B.nodes[out].off = o;
            B.nodes[out].len = l;
            return true;
        }
        if (e - p >= 4 && !memcmp(p, "true", 4)) { out = node(Node::BOOL); B.nodes[out].b = 1; p += 4; return true; }
        if (e - p >= 5 && !memcmp(p, "false", 5)) { out = node(Node::BOOL); p += 5; return true; }
        if (e - p >= 4 && !memcmp(p, "null", 4)) { out = node(Node::NUL); p += 4; return true; }
        if (c == '-' || (c >= '0' && c <= '9')) {   // -?(0|[1-9][0-9]*)(.[0-9]+)?([eE][+-]?[0-9]+)?
            const char *s = p;
            auto digits = [&]() {
                const char *q = p;
                while (p < e && *p >= '0' && *p <= '9') p++;
                return p > q;
            };
            if (*p == '-') p++;
            if (p < e && *p == '0') p++;
            else if (!digits()) return fail("bad number");
            if (p < e && *p == '.') {
                p++;
                if (!digits()) return fail("bad number");
            }
            if (p < e && (*p == 'e' || *p == 'E')) {
                p++;
                if (p < e && (*p == '+' || *p == '-')) p++;
                if (!digits()) return fail("bad number");
            }
            out = node(Node::NUM);
            B.nodes[out].off = (uint32_t)(s - B.src);
            B.nodes[out].len = (uint32_t)(p - s);
            return true;
        }
        return fail("unexpected character");
    }
};

bool parse(Blob &b, std::string &err) {
    if (b.n >= 0xFFFFFFFFull) {   // node offsets are 32-bit
        err = "blob larger than 4 GiB";
        return false;
    }
    b.nodes.clear();
    b.nodes.reserve(b.n / 12 + 8);
    b.slen = 0;
    if (b.str.size() < b.n + 1) b.str.resize(b.n + 1);
    Reader r{b.src, b.src + b.n, b, {}};
    uint32_t root;
    if (!r.val(root)) {
        err = r.err;
        return false;
    }
    r.ws();
    if (r.p != r.e) {
        err = "trailing characters";
        return false;
    }
    return true;
}

void utf8(std::string &o, const char16_t *s, size_t n) {
    for (size_t i = 0; i < n; i++) {
        uint32_t c = s[i];
        if (c >= 0xD800 && c < 0xDC00 && i + 1 < n && s[i + 1] >= 0xDC00 && s[i + 1] < 0xE000) {
            c = 0x10000 + ((c - 0xD800) << 10) + (s[i + 1] - 0xDC00);
            i++;
        }
        if (c < 0x80) o.push_back((char)c);
        else if (c < 0x800) { o.push_back((char)(0xC0 | (c >> 6))); o.push_back((char)(0x80 | (c & 0x3F))); }
        else if (c < 0x10000) {
            o.push_back((char)(0xE0 | (c >> 12)));
            o.push_back((char)(0x80 | ((c >> 6) & 0x3F)));
            o.push_back((char)(0x80 | (c & 0x3F)));
        } else {
            o.push_back((char)(0xF0 | (c >> 18)));
            o.push_back((char)(0x80 | ((c >> 12) & 0x3F)));
            o.push_back((char)(0x80 | ((c >> 6) & 0x3F)));
            o.push_back((char)(0x80 | (c & 0x3F)));
        }
    }
}
std::string utf8(const std::u16string &s) {
    std::string o;
    utf8(o, s.data(), s.size());
    return o;
}
void json_str(std::string &o, const char16_t *s, size_t n) {   // JSON text (lone surrogates escaped)
    o.push_back('"');
    for (size_t i = 0; i < n; i++) {
        const char16_t c = s[i];
        const bool pair = c >= 0xD800 && c < 0xDC00 && i + 1 < n && s[i + 1] >= 0xDC00 && s[i + 1] < 0xE000;
        if (c == u'"' || c == u'\\') {
            o.push_back('\\');
            o.push_back((char)c);
        } else if (c < 0x20 || (c >= 0xD800 && c < 0xE000 && !pair)) {
            char b[8];
            snprintf(b, sizeof b, "\\u%04x", (unsigned)c);
            o += b;
        } else if (c < 0x80) {
            o.push_back((char)c);
        } else {
            utf8(o, s + i, pair ? 2 : 1);
            i += pair;
        }
    }
    o.push_back('"');
}

// Canonical JSON of a property value: equal iff wire.canonical_json is equal -- numbers as
// JS Numbers (matchProperties compares with ===), object keys sorted.  json.loads of it
// gives back an equal value.
void canon(std::string &o, const Blob &B, uint32_t i) {
    const Node &v = B.nodes[i];
    switch (v.t) {
        case Node::NUL: o += "null"; break;
        case Node::BOOL: o += v.b ? "true" : "false"; break;
        case Node::NUM:
            if (B.is_int(i) && v.len <= 15) {   // exact in a double: the digits
                if (v.len == 2 && !memcmp(B.src + v.off, "-0", 2)) o += "0";
                else o.append(B.src + v.off, v.len);
            } else {   // JS Number: 1.0, 1e0 and 1 are one value
                const double x = B.num(i);
                if (std::isinf(x)) {   // json.loads reads these back (JSON.parse gave Infinity)
                    o += x > 0 ? "Infinity" : "-Infinity";
                    break;
                }
                char b[400];
                const auto r = std::isfinite(x) && x == std::floor(x) && std::fabs(x) < 1e21
                                   ? std::to_chars(b, b + sizeof b, x == 0 ? 0.0 : x, std::chars_format::fixed, 0)
                                   : std::to_chars(b, b + sizeof b, x);   // shortest round trip
                o.append(b, r.ptr);
            }
            break;
        case Node::STR: json_str(o, B.s(v.off), v.len); break;
        case Node::ARR: {
            o.push_back('[');
            uint32_t c = B.first(i);
            for (uint32_t m = 0; m < v.len; m++, c = B.nodes[c].next) {
                if (m) o.push_back(',');
                canon(o, B, c);
            }
            o.push_back(']');
            break;
        }
        case Node::OBJ: {
            std::vector<uint32_t> m;
            B.members(i, m);
            std::sort(m.begin(), m.end(), [&](uint32_t a, uint32_t b) {
                return std::u16string_view(B.s(B.nodes[a].koff), B.nodes[a].klen) <
                       std::u16string_view(B.s(B.nodes[b].koff), B.nodes[b].klen);
            });
            o.push_back('{');
            for (size_t k = 0; k < m.size(); k++) {
                if (k) o.push_back(',');
                json_str(o, B.s(B.nodes[m[k]].koff), B.nodes[m[k]].klen);
                o.push_back(':');
                canon(o, B, m[k]);
            }
            o.push_back('}');
            break;
        }
    }
}
// JS truthiness of a JSON value (wire.js_falsy)
bool falsy(const Blob &B, uint32_t i) {
    const Node &v = B.nodes[i];
    if (v.t == Node::NUL) return true;
    if (v.t == Node::BOOL) return !v.b;
    if (v.t == Node::STR) return v.len == 0;
    if (v.t == Node::NUM) return B.num(i) == 0.0;
    return false;
}

// toLatestVersion (MT/snapshotChunks.ts:136-167): {segments, segmentCount, headerMetadata}
// with the legacy header's metadata built as buildHeaderMetadataForLegecyChunk (:169-188)
struct Chunk {
    uint32_t segments = NONE;
    int64_t segment_count = 0;
    bool has_meta = false;
    std::vector<std::u16string> ordered;
    uint32_t min_seq = NONE, seq = NONE;
    int64_t total_segments = 0;
};
void meta_of(const Blob &B, uint32_t m, Chunk &out) {
    out.has_meta = true;
    const uint32_t oc = B.get(m, "orderedChunkMetadata");
    if (oc != NONE && B.nodes[oc].t == Node::ARR) {
        uint32_t c = B.first(oc);
        for (uint32_t k = 0; k < B.nodes[oc].len; k++, c = B.nodes[c].next) {
            const uint32_t id = B.get(c, "id");
            if (id != NONE && B.nodes[id].t == Node::STR) out.ordered.push_back(B.ustr(id));
        }
    }
    out.min_seq = B.get(m, "minSequenceNumber");
    out.seq = B.get(m, "sequenceNumber");
    out.total_segments = B.as_int(B.get(m, "totalSegmentCount"));
}
bool latest(const Blob &B, Chunk &out, std::string &err) {
    const uint32_t root = 0, ver = B.get(root, "version");
    if (B.is_str(ver, "1")) {
        out.segments = B.get(root, "segments");
        out.segment_count = B.as_int(B.get(root, "segmentCount"));
        const uint32_t m = B.get(root, "headerMetadata");
        if (B.present(m)) meta_of(B, m, out);
        return true;
    }
    if (B.present(ver)) {
        std::string v;
        if (B.nodes[ver].t == Node::STR) utf8(v, B.s(B.nodes[ver].off), B.nodes[ver].len);
        else if (B.nodes[ver].t == Node::NUM) v.assign(B.src + B.nodes[ver].off, B.nodes[ver].len);
        err = "Unsupported chunk path: " + B.path + " version: " + v;
        return false;
    }
    out.segments = B.get(root, "segmentTexts");
    out.segment_count = B.as_int(B.get(root, "chunkSegmentCount"));
    if (B.path == "header") {
        const uint32_t m = B.get(root, "headerMetadata");
        if (B.present(m)) {
            meta_of(B, m, out);
        } else {
            out.has_meta = true;
            out.ordered.push_back(u"header");
            if (B.as_int(B.get(root, "chunkLengthChars")) < B.as_int(B.get(root, "totalLengthChars")))
                out.ordered.push_back(u"body");
            out.min_seq = B.get(root, "chunkMinSequenceNumber");
            out.seq = B.get(root, "chunkSequenceNumber");
            out.total_segments = B.as_int(B.get(root, "totalSegmentCount"));
        }
    }
    return true;
}

const char *const kSpecKeys[5] = {"json", "seq", "client", "removedSeq", "removedClient"};
const char *const kSegKeys[3] = {"text", "props", "marker"};

// One document's records, property ids local to the document (first-seen order); the merge
// maps them to the batch's ids in document order, which keeps wire.Interner's numbering.
struct DocOut {
    std::vector<mt_seg_rec> segs;     // payload (text) / props: offsets into this document's arenas
    std::vector<uint16_t> text;
    std::vector<uint32_t> props;      // [count, (key, value) x count]: local ids (synthetic: final)
    std::vector<std::u16string> keys; // local key id -> key
    std::vector<std::string> vals;    // local value id -> canonical JSON
    int32_t nh = 0, msn = 0, seq = 0;
    int64_t cu = -1;
    std::string clients, err;
    std::vector<uint32_t> kmap, vmap;   // phase 2: local key / value id -> the batch's
    size_t si = 0, ti = 0, pi = 0;      // phase 2: where the document starts in the output
};

struct Blobs {
    const int64_t *off;
    const char *const *paths;
    const uint32_t *path_len;
    const char *const *json;
    const uint64_t *json_len;
};

// Per-thread scratch: SnapshotLoader.initialize for one document at a time.
struct Worker {
    bool synthetic = false;
    std::vector<Blob> blobs;
    std::unordered_map<std::u16string, uint32_t> key_ids;
    std::unordered_map<std::string, uint32_t> val_ids;
    std::unordered_map<std::u16string, int> shortid;
    std::u16string kbuf;
    std::string cbuf;
    std::vector<uint32_t> mbuf;
    std::vector<std::pair<const Blob *, uint32_t>> specs;
    std::vector<std::string> ordered8;
    std::vector<std::u16string> sid;   // short id k + 1 -> long client id

    uint32_t key(DocOut &o, const Blob &B, uint32_t m) {
        const char16_t *k = B.s(B.nodes[m].koff);
        const uint32_t n = B.nodes[m].klen;
        if (synthetic) {   // "k<n>" -> n (wire.Interner(synthetic=True))
            uint32_t v = 0;
            for (uint32_t i = 1; i < n; i++) v = v * 10 + (uint32_t)(k[i] - u'0');
            return v;
        }
        kbuf.assign(k, n);
        auto it = key_ids.find(kbuf);
        if (it != key_ids.end()) return it->second;
        const uint32_t id = (uint32_t)o.keys.size();
        key_ids.emplace(kbuf, id);
        o.keys.push_back(kbuf);
        return id;
    }
    uint32_t val(DocOut &o, const Blob &B, uint32_t i) {
        if (B.nodes[i].t == Node::NUL) return MT_VAL_NULL;
        if (synthetic) {
            const uint32_t x = (uint32_t)B.as_int(i);
            return x | (x == 0 ? MT_VAL_FALSY_BIT : 0u);
        }
        cbuf.clear();
        canon(cbuf, B, i);
        uint32_t id;
        auto it = val_ids.find(cbuf);
        if (it != val_ids.end()) {
            id = it->second;
        } else {
            id = (uint32_t)o.vals.size();
            val_ids.emplace(cbuf, id);
            o.vals.push_back(cbuf);
        }
        return id | (falsy(B, i) ? MT_VAL_FALSY_BIT : 0u);
    }
    bool bad(DocOut &o, const std::string &m) {
        o.err = m;
        return false;
    }

    bool build(DocOut &o, uint32_t d, const Blobs &in) {
        o.segs.clear();
        o.text.clear();
        o.props.clear();
        o.keys.clear();
        o.vals.clear();
        o.err.clear();
        o.cu = -1;
        key_ids.clear();
        val_ids.clear();
        const int64_t b0 = in.off[d], b1 = in.off[d + 1];
        if (blobs.size() < (size_t)(b1 - b0)) blobs.resize((size_t)(b1 - b0));
        for (int64_t b = b0; b < b1; b++) {   // JSON.parse of every blob (MT/snapshotV1.ts:274)
            Blob &B = blobs[(size_t)(b - b0)];
            B.src = in.json[b];
            B.n = in.json_len[b];
            B.path.assign(in.paths[b], in.path_len[b]);
            std::string e;
            if (!parse(B, e)) return bad(o, "blob " + B.path + ": " + e);
        }
        auto find = [&](const std::string &p) -> const Blob * {
            for (int64_t b = 0; b < b1 - b0; b++)
                if (blobs[(size_t)b].path == p) return &blobs[(size_t)b];
            return nullptr;
        };
        const Blob *H = find("header");
        if (!H) return bad(o, "header blob missing");
        Chunk head;
        std::string e;
        if (!latest(*H, head, e)) return bad(o, e);
        if (!head.has_meta) return bad(o, "header metadata not available");
        ordered8.clear();
        for (const auto &x : head.ordered) ordered8.push_back(utf8(x));
        const int64_t seq = H->as_int(head.seq);
        const int64_t msn = H->present(head.min_seq) ? H->as_int(head.min_seq) : seq;
        specs.clear();
        auto take = [&](const Blob &B, uint32_t arr) {
            if (arr == NONE || B.nodes[arr].t != Node::ARR) return;
            uint32_t c = B.first(arr);
            for (uint32_t k = 0; k < B.nodes[arr].len; k++, c = B.nodes[c].next) specs.emplace_back(&B, c);
        };
        take(*H, head.segments);
        const size_t nh = specs.size();
        if (head.segment_count != head.total_segments) {   // loadBody :170-172
            for (size_t k = 1; k < ordered8.size(); k++) {
                const Blob *C = find(ordered8[k]);
                if (!C) return bad(o, "body blob missing: " + ordered8[k]);
                Chunk ch;
                if (!latest(*C, ch, e)) return bad(o, e);
                take(*C, ch.segments);
            }
        }
        const int64_t nblobs = b1 - b0;   // the legacy catch-up blob (:72-79)
        if (nblobs == (int64_t)ordered8.size() + 1) {
            int n_rest = 0;
            for (int64_t b = b0; b < b1; b++)
                if (std::find(ordered8.begin(), ordered8.end(), blobs[(size_t)(b - b0)].path) == ordered8.end()) {
                    n_rest++;
                    o.cu = b;
                }
            if (n_rest != 1) return bad(o, "There should be only one blob with catch up ops: " + std::to_string(n_rest));
        } else if (nblobs != (int64_t)ordered8.size()) {
            return bad(o, "Unexpected blobs in snapshot");
        }
        // specToSegment :86-118 (+ segmentFromSpec, SEQ/sequenceFactory.ts:31-37)
        shortid.clear();
        sid.clear();
        auto short_of = [&](const Blob &B, uint32_t c) {
            const char16_t *u = B.s(B.nodes[c].off);
            const uint32_t n = B.nodes[c].len;
            if (shortid.empty()) {   // few writers: a linear scan over the first-seen names
                for (size_t k = 0; k < sid.size(); k++)
                    if (sid[k].size() == n && !memcmp(sid[k].data(), u, n * sizeof(char16_t))) return (int)k + 1;
                sid.emplace_back(u, n);
                if (sid.size() > 32)
                    for (size_t k = 0; k < sid.size(); k++) shortid.emplace(sid[k], (int)k + 1);
                return (int)sid.size();
            }
            kbuf.assign(u, n);
            auto it = shortid.find(kbuf);
            if (it != shortid.end()) return it->second;
            const int v = (int)sid.size() + 1;
            sid.emplace_back(kbuf);
            shortid.emplace(kbuf, v);
            return v;
        };
        o.segs.reserve(specs.size());
        for (const auto &sp : specs) {
            const Blob &B = *sp.first;
            const uint32_t spec = sp.second;
            mt_seg_rec r;
            memset(&r, 0, sizeof r);
            r.removed_seq = INT32_MIN;
            r.props = MT_NO_PROPS;
            r.client = -2;
            // one pass over each object's members (the last of duplicated members, as B.get)
            uint32_t sf[5] = {NONE, NONE, NONE, NONE, NONE};   // json, seq, client, removedSeq, removedClient
            if (B.nodes[spec].t == Node::OBJ) B.fields(spec, kSpecKeys, 5, sf);
            const uint32_t jv = sf[0], sq = sf[1], cl = sf[2], rs = sf[3], rc = sf[4];
            const bool mi = jv != NONE;   // hasMergeInfo: `"json" in spec`
            const uint32_t js = mi ? jv : spec;
            uint32_t pr = NONE, tx = NONE, mk = NONE;
            uint32_t jf[3] = {NONE, NONE, NONE};   // text, props, marker
            if (B.nodes[js].t == Node::OBJ) B.fields(js, kSegKeys, 3, jf);
            if (B.nodes[js].t == Node::STR) {
                tx = js;
            } else if ((tx = jf[0]) != NONE) {
                pr = jf[1];
            } else if ((mk = jf[2]) != NONE) {
                r.flags = MT_F_MARKER;
                r.payload = (uint32_t)B.as_int(B.get(mk, "refType"));
                r.len = 1;
                pr = jf[1];
            } else {
                return bad(o, "unsupported segment spec");
            }
            if (tx != NONE) {
                if (B.nodes[tx].t != Node::STR) return bad(o, "segment text is not a string");
                r.payload = (uint32_t)o.text.size();
                o.text.insert(o.text.end(), B.s(B.nodes[tx].off), B.s(B.nodes[tx].off) + B.nodes[tx].len);
                r.len = (int32_t)B.nodes[tx].len;
            }
            if (pr != NONE && B.nodes[pr].t == Node::OBJ) {   // `if (props)`: {} too (Q5)
                r.props = (uint32_t)o.props.size();
                B.members(pr, mbuf);
                o.props.push_back((uint32_t)mbuf.size());
                for (uint32_t kv : mbuf) {
                    o.props.push_back(key(o, B, kv));
                    o.props.push_back(val(o, B, kv));
                }
            }
            if (mi) {
                r.flags |= MT_SEG_MERGE_INFO | (B.present(sq) ? MT_SEG_HAS_SEQ : 0);
                if (B.present(cl)) r.client = (int16_t)short_of(B, cl);
                if (B.present(sq)) r.seq = (int32_t)B.as_int(sq);
                if (B.present(rs)) r.removed_seq = (int32_t)B.as_int(rs);
                if (B.present(rc)) r.removed_client = (int16_t)short_of(B, rc);
            }
            o.segs.push_back(r);
        }
        o.nh = (int32_t)nh;
        o.msn = (int32_t)msn;
        o.seq = (int32_t)seq;
        o.clients = "[";
        for (size_t i = 0; i < sid.size(); i++) {
            if (i) o.clients.push_back(',');
            json_str(o.clients, sid[i].data(), sid[i].size());
        }
        o.clients.push_back(']');
        return true;
    }
};

// ---------------------------------------------------------------- sequenced messages
// ISequencedDocumentMessage JSON (PD/protocol.ts:132-172) carrying IMergeTree ops
// (MT/ops.ts:63-110) -> mt_op_rec records, as fluidframework_amd/wire.py Batch.add_doc /
// _msg / _op encode them (its tests compare the two on the reference's fixtures).
struct OpDocOut {
    std::vector<mt_op_rec> ops;       // payload (text) / props: offsets into this document's arenas
    std::vector<uint16_t> text;
    std::vector<uint32_t> props;      // [count | combine << 16, (key, value) x count]: local ids
    std::vector<std::u16string> keys; // local key id -> key
    std::vector<std::string> vals;    // local value id -> canonical JSON
    std::string clients, err;
    std::vector<uint32_t> kmap, vmap;
    size_t oi = 0, ti = 0, pi = 0;
};

const char *const kMsgKeys[6] = {"clientId", "sequenceNumber", "referenceSequenceNumber", "minimumSequenceNumber",
                                 "type", "contents"};

struct OpWorker {
    bool synthetic = false;
    Blob B;
    std::unordered_map<std::u16string, uint32_t> key_ids, shortid;
    std::unordered_map<std::string, uint32_t> val_ids;
    std::vector<std::u16string> sid;   // short id k + 1 -> long client id (k = 0: the first seen)
    std::u16string kbuf;
    std::string cbuf;
    std::vector<uint32_t> mbuf;

    bool bad(OpDocOut &o, const std::string &m) {
        o.err = m;
        return false;
    }
    // DocEncoder.client: first-seen order from 1 (the observer is 0); a null clientId is an
    // id of its own (a dict key None in the Python encoder)
    int client(uint32_t c) {
        static const char16_t kNull = (char16_t)0xFFFF;   // (not a UTF-16 string)
        const bool str = c != NONE && B.nodes[c].t == Node::STR;
        const char16_t *u = str ? B.s(B.nodes[c].off) : &kNull;
        const uint32_t n = str ? B.nodes[c].len : 1;
        if (sid.size() <= 32) {   // few writers: a linear scan over the first-seen names
            for (size_t k = 0; k < sid.size(); k++)
                if (sid[k].size() == n && !memcmp(sid[k].data(), u, n * sizeof(char16_t))) return (int)k + 1;
            sid.emplace_back(u, n);
            if (sid.size() > 32)
                for (size_t k = 0; k < sid.size(); k++) shortid.emplace(sid[k], (uint32_t)k + 1);
            return (int)sid.size();
        }
        kbuf.assign(u, n);
        auto it = shortid.find(kbuf);
        if (it != shortid.end()) return (int)it->second;
        sid.push_back(kbuf);
        shortid.emplace(kbuf, (uint32_t)sid.size());
        return (int)sid.size();
    }
    uint32_t key(OpDocOut &o, uint32_t m) {
        const char16_t *k = B.s(B.nodes[m].koff);
        const uint32_t n = B.nodes[m].klen;
        if (synthetic) {
            uint32_t v = 0;
            for (uint32_t i = 1; i < n; i++) v = v * 10 + (uint32_t)(k[i] - u'0');
            return v;
        }
        kbuf.assign(k, n);
        auto it = key_ids.find(kbuf);
        if (it != key_ids.end()) return it->second;
        const uint32_t id = (uint32_t)o.keys.size();
        key_ids.emplace(kbuf, id);
        o.keys.push_back(kbuf);
        return id;
    }
    uint32_t val(OpDocOut &o, uint32_t i) {
        if (B.nodes[i].t == Node::NUL) return MT_VAL_NULL;
        if (synthetic) {
            const uint32_t x = (uint32_t)B.as_int(i);
            return x | (x == 0 ? MT_VAL_FALSY_BIT : 0u);
        }
        cbuf.clear();
        canon(cbuf, B, i);
        uint32_t id;
        auto it = val_ids.find(cbuf);
        if (it != val_ids.end()) {
            id = it->second;
        } else {
            id = (uint32_t)o.vals.size();
            val_ids.emplace(cbuf, id);
            o.vals.push_back(cbuf);
        }
        return id | (falsy(B, i) ? MT_VAL_FALSY_BIT : 0u);
    }
    // Batch._props_rec: [count | combine << 16, (key, value) x count], members in insertion order
    bool props_rec(OpDocOut &o, uint32_t pr, uint32_t combine, uint32_t &off) {
        if (pr == NONE || B.nodes[pr].t != Node::OBJ) return bad(o, "props is not an object");
        off = (uint32_t)o.props.size();
        B.members(pr, mbuf);
        o.props.push_back((uint32_t)mbuf.size() | (combine << 16));
        for (uint32_t kv : mbuf) {
            o.props.push_back(key(o, kv));
            o.props.push_back(val(o, kv));
        }
        return true;
    }
    static bool truthy_obj(const Blob &B, uint32_t i) {   // Python truthiness of a JSON value
        if (i == NONE) return false;
        const Node &v = B.nodes[i];
        switch (v.t) {
            case Node::NUL: return false;
            case Node::BOOL: return v.b != 0;
            case Node::NUM: return B.num(i) != 0.0;
            default: return v.len != 0;   // STR: units; ARR / OBJ: members
        }
    }
    // Batch._op for one op (member of a GROUP when `more`)
    bool op(OpDocOut &o, const mt_op_rec &base, uint32_t op, bool more) {
        mt_op_rec r = base;
        r.flags = more ? MT_F_GROUP_MORE : 0;
        if (op == NONE || B.nodes[op].t != Node::OBJ) return bad(o, "op is not an object");
        const int64_t t = B.as_int(B.get(op, "type"));
        if (t == MT_OP_INSERT) {
            const uint32_t seg = B.get(op, "seg");
            const uint32_t p1 = B.get(op, "pos1");
            if (p1 == NONE) return bad(o, "insert without pos1");
            r.kind = MT_OP_INSERT;
            r.pos1 = (int32_t)B.as_int(p1);
            const bool is_obj = seg != NONE && B.nodes[seg].t == Node::OBJ;
            if (!truthy_obj(B, seg) && !is_obj) {   // `if (op.seg)` falsy: seq / msn only
                r.kind = MT_OP_NOOP;
            } else if (B.nodes[seg].t == Node::STR) {
                r.payload = (uint32_t)o.text.size();
                o.text.insert(o.text.end(), B.s(B.nodes[seg].off), B.s(B.nodes[seg].off) + B.nodes[seg].len);
                r.pos2 = (int32_t)B.nodes[seg].len;
            } else if (is_obj && B.get(seg, "text") != NONE) {
                const uint32_t tx = B.get(seg, "text");
                if (B.nodes[tx].t != Node::STR) return bad(o, "insert text is not a string");
                r.payload = (uint32_t)o.text.size();
                o.text.insert(o.text.end(), B.s(B.nodes[tx].off), B.s(B.nodes[tx].off) + B.nodes[tx].len);
                r.pos2 = (int32_t)B.nodes[tx].len;
                const uint32_t pr = B.get(seg, "props");
                if (B.present(pr) && !props_rec(o, pr, MT_COMBINE_NONE, r.props)) return false;
            } else if (is_obj && B.get(seg, "marker") != NONE) {
                r.flags |= MT_F_MARKER;
                const uint32_t mk = B.get(seg, "marker");
                if (B.nodes[mk].t != Node::OBJ) return bad(o, "marker is not an object");
                r.payload = (uint32_t)B.as_int(B.get(mk, "refType"));
                r.pos2 = 1;
                const uint32_t pr = B.get(seg, "props");
                if (B.present(pr) && !props_rec(o, pr, MT_COMBINE_NONE, r.props)) return false;
            } else {
                return bad(o, "unsupported insert segment");
            }
        } else if (t == MT_OP_REMOVE || t == MT_OP_ANNOTATE) {
            r.kind = (uint8_t)t;
            const uint32_t p1 = B.get(op, "pos1"), p2 = B.get(op, "pos2");
            if (p1 == NONE || p2 == NONE) return bad(o, "range op without pos1 / pos2");
            r.pos1 = (int32_t)B.as_int(p1);
            r.pos2 = (int32_t)B.as_int(p2);
            if (t == MT_OP_ANNOTATE) {
                const uint32_t comb = B.get(op, "combiningOp");
                const bool has = truthy_obj(B, comb);
                uint32_t cb = has ? MT_COMBINE_REWRITE : MT_COMBINE_NONE;
                if (has && !B.is_str(B.nodes[comb].t == Node::OBJ ? B.get(comb, "name") : NONE, "rewrite")) {
                    // Batch._combine_rec: a synthetic interner keeps COMBINE_OTHER; otherwise the
                    // transform table needs every value the keys held so far -- wire.Batch builds it
                    if (!synthetic) return bad(o, "combining op: encode with wire.Batch (its transform tables)");
                    cb = MT_COMBINE_OTHER;
                }
                if (!props_rec(o, B.get(op, "props"), cb, r.props)) return false;
            }
        } else {
            return bad(o, "unsupported op type " + std::to_string(t));
        }
        o.ops.push_back(r);
        return true;
    }

    bool build(OpDocOut &o, const char *json, uint64_t len) {
        o.ops.clear();
        o.text.clear();
        o.props.clear();
        o.keys.clear();
        o.vals.clear();
        o.err.clear();
        key_ids.clear();
        val_ids.clear();
        shortid.clear();
        sid.clear();
        B.src = json;
        B.n = (size_t)len;
        std::string e;
        if (!parse(B, e)) return bad(o, e);
        if (B.nodes[0].t != Node::ARR) return bad(o, "messages are not an array");
        uint32_t m = B.first(0);
        o.ops.reserve(B.nodes[0].len);
        for (uint32_t k = 0; k < B.nodes[0].len; k++, m = B.nodes[m].next) {
            if (B.nodes[m].t != Node::OBJ) return bad(o, "message " + std::to_string(k) + " is not an object");
            uint32_t f[6] = {NONE, NONE, NONE, NONE, NONE, NONE};
            B.fields(m, kMsgKeys, 6, f);
            if (f[1] == NONE || f[2] == NONE || f[3] == NONE)
                return bad(o, "message " + std::to_string(k) + " without its sequence numbers");
            mt_op_rec base;
            memset(&base, 0, sizeof base);
            base.seq = (int32_t)B.as_int(f[1]);
            base.ref_seq = (int32_t)B.as_int(f[2]);
            base.min_seq = (int32_t)B.as_int(f[3]);
            base.props = MT_NO_PROPS;
            base.client = (uint16_t)client(f[0]);
            base.kind = MT_OP_NOOP;
            if (f[4] != NONE && !B.is_str(f[4], "op")) {   // a non-op message: seq / msn only
                o.ops.push_back(base);
                continue;
            }
            const uint32_t c = f[5];
            if (c == NONE || B.nodes[c].t != Node::OBJ) return bad(o, "message contents are not an object");
            if (B.as_int(B.get(c, "type")) == 3) {   // GROUP
                const uint32_t arr = B.get(c, "ops");
                if (arr == NONE || B.nodes[arr].t != Node::ARR) return bad(o, "group without ops");
                if (B.nodes[arr].len == 0) {   // applies nothing; applyMsg still updates seq / msn
                    o.ops.push_back(base);
                    continue;
                }
                uint32_t g = B.first(arr);
                for (uint32_t j = 0; j < B.nodes[arr].len; j++, g = B.nodes[g].next)
                    if (!op(o, base, g, j + 1 < B.nodes[arr].len)) return false;
            } else if (!op(o, base, c, false)) {
                return false;
            }
        }
        o.clients = "[";
        for (size_t i = 0; i < sid.size(); i++) {
            if (i) o.clients.push_back(',');
            if (sid[i].size() == 1 && sid[i][0] == (char16_t)0xFFFF) o.clients += "null";
            else json_str(o.clients, sid[i].data(), sid[i].size());
        }
        o.clients.push_back(']');
        return true;
    }
};

}  // namespace

struct mt_snapdec {
    bool synthetic = false;
    std::string err;
    std::unordered_map<std::u16string, uint32_t> key_ids;   // the batch's interning
    std::vector<std::u16string> keys;
    std::unordered_map<std::string, uint32_t> val_ids;
    std::vector<std::string> vals;
    std::vector<DocOut> docs;           // reused between calls
    std::vector<Worker> workers;
    std::vector<OpDocOut> opdocs;       // sequenced-message decoding (mt_opdec_*)
    std::vector<OpWorker> opworkers;
    uint32_t op_n_docs = 0;
    int op_threads = 1;
    size_t nops = 0, optx = 0, oppr = 0;
    uint32_t n_docs = 0;                // of the last successful decode
    int threads = 1;
    size_t ns = 0, ntx = 0, npr = 0;    // its output sizes
};

namespace {
// Runs fn(d) for d in [0, n) on nt threads (dynamic, `grain` documents at a time).
template <class F> void parallel_docs(uint32_t n, int nt, uint32_t grain, F fn) {
    std::atomic<uint32_t> next{0};
    auto work = [&]() {
        for (;;) {
            const uint32_t d0 = next.fetch_add(grain);
            if (d0 >= n) break;
            for (uint32_t d = d0; d < std::min(n, d0 + grain); d++) fn(d);
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; t++) pool.emplace_back(work);
    work();
    for (auto &t : pool) t.join();
}
}  // namespace

extern "C" {

mt_snapdec *mt_snapdec_create(int synthetic) {
    auto *s = new mt_snapdec();
    s->synthetic = synthetic != 0;
    return s;
}
void mt_snapdec_destroy(mt_snapdec *s) { delete s; }
const char *mt_snapdec_error(const mt_snapdec *s) { return s ? s->err.c_str() : "null decoder"; }

int mt_snapdec_decode(mt_snapdec *s, uint32_t n_docs, const int64_t *blob_off, const char *const *paths,
                      const uint32_t *path_len, const char *const *json, const uint64_t *json_len, int threads) {
    if (!s || !blob_off) return -1;
    s->err.clear();
    // offsets: monotonic from 0 (each document's blobs are [blob_off[d], blob_off[d+1]))
    if (blob_off[0] != 0) {
        s->err = "blob_off[0] must be 0";
        return -1;
    }
    for (uint32_t d = 0; d < n_docs; d++)
        if (blob_off[d + 1] < blob_off[d]) {
            s->err = "blob_off must be non-decreasing (document " + std::to_string(d) + ")";
            return -1;
        }
    if (blob_off[n_docs] > 0 && (!paths || !path_len || !json || !json_len)) {
        s->err = "null blob arrays";
        return -1;
    }
    if (s->docs.size() < n_docs) s->docs.resize(n_docs);
    s->n_docs = 0;
    const int nt = std::max(1, std::min({threads, 256, (int)std::max<uint32_t>(n_docs, 1)}));
    if ((int)s->workers.size() < nt) s->workers.resize((size_t)nt);
    const Blobs in{blob_off, paths, path_len, json, json_len};
    // phase 1: documents parsed and specToSegment'ed on nt threads (dynamic, 8 at a time)
    {
        std::atomic<uint32_t> next{0};
        auto work = [&](int t) {
            Worker &w = s->workers[(size_t)t];
            w.synthetic = s->synthetic;
            for (;;) {
                const uint32_t d0 = next.fetch_add(8);
                if (d0 >= n_docs) break;
                for (uint32_t d = d0; d < std::min(n_docs, d0 + 8); d++) {
                    try {
                        w.build(s->docs[d], d, in);
                    } catch (const std::exception &ex) {   // e.g. bad_alloc: the document's error
                        s->docs[d].err = std::string("decode failed: ") + ex.what();
                    }
                }
            }
        };
        std::vector<std::thread> pool;
        for (int t = 1; t < nt; t++) pool.emplace_back(work, t);
        work(0);
        for (auto &t : pool) t.join();
    }
    // phase 2 (sequential, small): the first failing document, each document's place in the
    // output and its local -> batch id maps, numbered first-seen in document order; the
    // concatenation itself runs in parallel straight into the caller's arrays (fetch)
    size_t ns = 0, ntx = 0, npr = 0;
    for (uint32_t d = 0; d < n_docs; d++) {
        DocOut &o = s->docs[d];
        if (!o.err.empty()) {   // the first failing document, as a sequential load would report
            s->err = "document " + std::to_string(d) + ": " + o.err;
            return -1;
        }
        o.si = ns;
        o.ti = ntx;
        o.pi = npr;
        ns += o.segs.size();
        ntx += o.text.size();
        npr += o.props.size();
        if (s->synthetic) continue;
        o.kmap.resize(o.keys.size());
        for (size_t k = 0; k < o.keys.size(); k++) {
            auto it = s->key_ids.find(o.keys[k]);
            if (it == s->key_ids.end()) {
                it = s->key_ids.emplace(o.keys[k], (uint32_t)s->keys.size()).first;
                s->keys.push_back(o.keys[k]);
            }
            o.kmap[k] = it->second;
        }
        o.vmap.resize(o.vals.size());
        for (size_t k = 0; k < o.vals.size(); k++) {
            auto it = s->val_ids.find(o.vals[k]);
            if (it == s->val_ids.end()) {
                it = s->val_ids.emplace(o.vals[k], (uint32_t)s->vals.size()).first;
                s->vals.push_back(o.vals[k]);
            }
            o.vmap[k] = it->second;
        }
    }
    if (ntx > 0xFFFFFFFFull || npr > 0xFFFFFFFFull) {   // mt_seg_rec offsets are 32-bit
        s->err = "decoded text / property arena exceeds 2^32 entries: decode fewer documents per call";
        return -1;
    }
    s->n_docs = n_docs;
    s->threads = nt;
    s->ns = ns;
    s->ntx = ntx;
    s->npr = npr;
    return 0;
}

int mt_snapdec_sizes(const mt_snapdec *s, uint64_t *n_segs, uint64_t *text_len, uint64_t *props_len) {
    if (!s) return -1;
    if (n_segs) *n_segs = s->ns;
    if (text_len) *text_len = s->ntx;
    if (props_len) *props_len = s->npr;
    return 0;
}

int mt_snapdec_fetch(const mt_snapdec *s, int64_t *doc_seg_off, int32_t *n_header, mt_seg_rec *segs, uint16_t *text,
                     uint32_t *props, int32_t *min_seq, int32_t *cur_seq, int64_t *catchup_blob) {
    if (!s) return -1;
    const uint32_t n = s->n_docs;
    // documents back to back, on the decode's threads (64 at a time: a document is ~10 KB)
    parallel_docs(n, s->threads, 64, [&](uint32_t d) {
        const DocOut &o = s->docs[d];
        if (doc_seg_off) doc_seg_off[d] = (int64_t)o.si;
        if (n_header) n_header[d] = o.nh;
        if (min_seq) min_seq[d] = o.msn;
        if (cur_seq) cur_seq[d] = o.seq;
        if (catchup_blob) catchup_blob[d] = o.cu;
        if (segs) {
            mt_seg_rec *dst = segs + o.si;
            for (size_t k = 0; k < o.segs.size(); k++) {
                mt_seg_rec r = o.segs[k];
                if (!(r.flags & MT_F_MARKER)) r.payload += (uint32_t)o.ti;
                if (r.props != MT_NO_PROPS) r.props += (uint32_t)o.pi;
                dst[k] = r;
            }
        }
        if (text && !o.text.empty()) memcpy(text + o.ti, o.text.data(), o.text.size() * sizeof(uint16_t));
        if (props && !o.props.empty()) {
            if (s->synthetic) {
                memcpy(props + o.pi, o.props.data(), o.props.size() * sizeof(uint32_t));
            } else {
                uint32_t *q = props + o.pi;
                for (size_t i = 0; i < o.props.size();) {
                    const uint32_t c = o.props[i++];
                    *q++ = c;
                    for (uint32_t j = 0; j < c; j++, i += 2) {
                        const uint32_t v = o.props[i + 1];
                        *q++ = o.kmap[o.props[i]];
                        *q++ = v == MT_VAL_NULL ? v : (o.vmap[v & ~MT_VAL_FALSY_BIT] | (v & MT_VAL_FALSY_BIT));
                    }
                }
            }
        }
    });
    if (doc_seg_off) doc_seg_off[n] = (int64_t)s->ns;
    return 0;
}

static int64_t copy_out(const std::string &v, char *out, uint64_t cap) {
    if (out) memcpy(out, v.data(), std::min<uint64_t>(cap, v.size()));
    return (int64_t)v.size();
}
int64_t mt_snapdec_key(const mt_snapdec *s, uint32_t i, char *out, uint64_t cap) {
    if (!s || i >= s->keys.size()) return -1;
    return copy_out(utf8(s->keys[i]), out, cap);
}
int64_t mt_snapdec_value(const mt_snapdec *s, uint32_t i, char *out, uint64_t cap) {
    if (!s || i >= s->vals.size()) return -1;
    return copy_out(s->vals[i], out, cap);
}
int64_t mt_snapdec_doc_clients(const mt_snapdec *s, uint32_t d, char *out, uint64_t cap) {
    if (!s || d >= s->n_docs) return -1;
    return copy_out(s->docs[d].clients, out, cap);
}
int64_t mt_snapdec_all_clients(const mt_snapdec *s, char *out, uint64_t cap) {
    if (!s) return -1;
    uint64_t n = 0;
    for (uint32_t d = 0; d < s->n_docs; d++) {
        const std::string &c = s->docs[d].clients;
        if (out && n + c.size() + 1 <= cap) {
            memcpy(out + n, c.data(), c.size());
            out[n + c.size()] = '\n';
        }
        n += c.size() + 1;
    }
    return (int64_t)n;
}
uint32_t mt_snapdec_num_keys(const mt_snapdec *s) { return s ? (uint32_t)s->keys.size() : 0; }

int mt_opdec_decode(mt_snapdec *s, uint32_t n_docs, const char *const *json, const uint64_t *json_len, int threads) {
    if (!s || (n_docs && (!json || !json_len))) return -1;
    s->err.clear();
    if (s->opdocs.size() < n_docs) s->opdocs.resize(n_docs);
    s->op_n_docs = 0;
    const int nt = std::max(1, std::min({threads, 256, (int)std::max<uint32_t>(n_docs, 1)}));
    if ((int)s->opworkers.size() < nt) s->opworkers.resize((size_t)nt);
    {   // phase 1: each document parsed and encoded on its own (dynamic, one at a time)
        std::atomic<uint32_t> next{0};
        auto work = [&](int t) {
            OpWorker &w = s->opworkers[(size_t)t];
            w.synthetic = s->synthetic;
            for (;;) {
                const uint32_t d = next.fetch_add(1);
                if (d >= n_docs) break;
                try {
                    w.build(s->opdocs[d], json[d], json_len[d]);
                } catch (const std::exception &ex) {
                    s->opdocs[d].err = std::string("decode failed: ") + ex.what();
                }
            }
        };
        std::vector<std::thread> pool;
        for (int t = 1; t < nt; t++) pool.emplace_back(work, t);
        work(0);
        for (auto &t : pool) t.join();
    }
    // a failed document fails the call before anything is interned: the decoder's key / value
    // tables (which later calls continue) hold only ids of documents that were returned
    {
        size_t tx = 0, pr = 0;
        for (uint32_t d = 0; d < n_docs; d++) {
            if (!s->opdocs[d].err.empty()) {
                s->err = "document " + std::to_string(d) + ": " + s->opdocs[d].err;
                return -1;
            }
            tx += s->opdocs[d].text.size();
            pr += s->opdocs[d].props.size();
        }
        if (tx > 0xFFFFFFFFull || pr > 0xFFFFFFFFull) {   // mt_op_rec offsets are 32-bit
            s->err = "encoded text / property arena exceeds 2^32 entries: decode fewer documents per call";
            return -1;
        }
    }
    // phase 2: places and the batch's key / value ids, first seen in document order
    size_t no = 0, ntx = 0, npr = 0;
    for (uint32_t d = 0; d < n_docs; d++) {
        OpDocOut &o = s->opdocs[d];
        o.oi = no;
        o.ti = ntx;
        o.pi = npr;
        no += o.ops.size();
        ntx += o.text.size();
        npr += o.props.size();
        if (s->synthetic) continue;
        o.kmap.resize(o.keys.size());
        for (size_t k = 0; k < o.keys.size(); k++) {
            auto it = s->key_ids.find(o.keys[k]);
            if (it == s->key_ids.end()) {
                it = s->key_ids.emplace(o.keys[k], (uint32_t)s->keys.size()).first;
                s->keys.push_back(o.keys[k]);
            }
            o.kmap[k] = it->second;
        }
        o.vmap.resize(o.vals.size());
        for (size_t k = 0; k < o.vals.size(); k++) {
            auto it = s->val_ids.find(o.vals[k]);
            if (it == s->val_ids.end()) {
                it = s->val_ids.emplace(o.vals[k], (uint32_t)s->vals.size()).first;
                s->vals.push_back(o.vals[k]);
            }
            o.vmap[k] = it->second;
        }
    }
    if (ntx > 0xFFFFFFFFull || npr > 0xFFFFFFFFull) {   // mt_op_rec offsets are 32-bit
        s->err = "encoded text / property arena exceeds 2^32 entries: decode fewer documents per call";
        return -1;
    }
    s->op_n_docs = n_docs;
    s->op_threads = nt;
    s->nops = no;
    s->optx = ntx;
    s->oppr = npr;
    return 0;
}

int mt_opdec_sizes(const mt_snapdec *s, uint64_t *n_ops, uint64_t *text_len, uint64_t *props_len) {
    if (!s) return -1;
    if (n_ops) *n_ops = s->nops;
    if (text_len) *text_len = s->optx;
    if (props_len) *props_len = s->oppr;
    return 0;
}

int mt_opdec_fetch(const mt_snapdec *s, int64_t *doc_op_off, mt_op_rec *ops, uint16_t *text, uint32_t *props) {
    if (!s) return -1;
    const uint32_t n = s->op_n_docs;
    parallel_docs(n, s->op_threads, 16, [&](uint32_t d) {
        const OpDocOut &o = s->opdocs[d];
        if (doc_op_off) doc_op_off[d] = (int64_t)o.oi;
        if (ops) {
            mt_op_rec *dst = ops + o.oi;
            for (size_t k = 0; k < o.ops.size(); k++) {
                mt_op_rec r = o.ops[k];
                if (r.kind == MT_OP_INSERT && !(r.flags & MT_F_MARKER)) r.payload += (uint32_t)o.ti;
                if (r.props != MT_NO_PROPS) r.props += (uint32_t)o.pi;
                dst[k] = r;
            }
        }
        if (text && !o.text.empty()) memcpy(text + o.ti, o.text.data(), o.text.size() * sizeof(uint16_t));
        if (props && !o.props.empty()) {
            if (s->synthetic) {
                memcpy(props + o.pi, o.props.data(), o.props.size() * sizeof(uint32_t));
            } else {
                uint32_t *q = props + o.pi;
                for (size_t i = 0; i < o.props.size();) {
                    const uint32_t c = o.props[i++];
                    *q++ = c;
                    for (uint32_t j = 0; j < (c & 0xFFFFu); j++, i += 2) {
                        const uint32_t v = o.props[i + 1];
                        *q++ = o.kmap[o.props[i]];
                        *q++ = v == MT_VAL_NULL ? v : (o.vmap[v & ~MT_VAL_FALSY_BIT] | (v & MT_VAL_FALSY_BIT));
                    }
                }
            }
        }
    });
    if (doc_op_off) doc_op_off[n] = (int64_t)s->nops;
    return 0;
}

int64_t mt_opdec_doc_clients(const mt_snapdec *s, uint32_t d, char *out, uint64_t cap) {
    if (!s || d >= s->op_n_docs) return -1;
    return copy_out(s->opdocs[d].clients, out, cap);
}
uint32_t mt_snapdec_num_values(const mt_snapdec *s) { return s ? (uint32_t)s->vals.size() : 0; }

}  // extern "C"
