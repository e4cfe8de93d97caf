/*
 * kdtn_oracle_json.c — TEST INFRASTRUCTURE ONLY: CPU restatement of the controller's CR
 * ingest, i.e. what the informer does to a Kubernetes `TopologyList` JSON document before
 * Reconcile sees it: decode it into the typed structs of
 * api/v1/topology_types.go:28-56 (TopologySpec/Status), :59-95 (Link), :119-176
 * (LinkProperties), then lay the result out as the engine's epoch tables (kdtn.h).
 *
 * Decoding rules are restated from third-party code that is not under /root/reference:
 *   - sigs.k8s.io/json v0.0.0-20220713155537-f223a00ba0e2 (go.mod:107), the fork of Go's
 *     encoding/json that k8s.io/apimachinery v0.24.5-rc.0 (go.mod:119) uses to decode
 *     API objects (UnmarshalCaseSensitivePreserveInts: exact, case-sensitive key match);
 *   - its scanner (checkValid: the whole document is validated before decoding, nesting
 *     limit 10000), unquote (escapes, \u surrogate pairs, invalid UTF-8 → U+FFFD) and
 *     literalStore (null leaves a value unchanged except that a slice becomes nil;
 *     ints via strconv.ParseInt(s, 10, 64); uint32 via ParseUint + overflow check;
 *     any other JSON type for a typed field → UnmarshalTypeError).
 * The engine's two documented deviations are mirrored so the oracle can check it: a
 * schema field repeated inside one object is KDTN_JSON_DUPKEY (Go: last wins), and
 * fields off the path are skipped without type checks.
 *
 * Table layout (what kdtn_json_ingest leaves in HBM): topologies in items order;
 * desired = spec.links, realised = status.links, records in document order; every string
 * of a schema field is interned into kdict (names, namespaces, src_ip, net_ns, the seven
 * Link key strings) or pdict (the twelve LinkProperties strings) with ids in order of
 * first occurrence in the document, id 0 = "".
 */
#define _GNU_SOURCE
#include "kdtn_oracle.h"

#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- growable buffers */
typedef struct { uint8_t* p; size_t n, cap; } obuf;

static int ob_reserve(obuf* b, size_t add) {
    if (b->n + add <= b->cap) return 0;
    size_t c = b->cap ? b->cap : 256;
    while (c < b->n + add) c *= 2;
    uint8_t* q = (uint8_t*)realloc(b->p, c);
    if (!q) return -1;
    b->p = q;
    b->cap = c;
    return 0;
}
static int ob_put(obuf* b, const void* src, size_t n) {
    if (ob_reserve(b, n)) return -1;
    memcpy(b->p + b->n, src, n);
    b->n += n;
    return 0;
}
static int ob_u32(obuf* b, uint32_t v) { return ob_put(b, &v, 4); }

/* ---------------------------------------------------------------- interner */
typedef struct {
    obuf bytes;          /* arena                        */
    obuf offs;           /* u32 offsets, n + 1           */
    uint32_t* slots;     /* id + 1, 0 = empty            */
    uint32_t cap, n;
} ointern;

static uint64_t ohash(const uint8_t* p, size_t n) {
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; ++i) { h ^= p[i]; h *= 1099511628211ull; }
    return h ^ (h >> 31);
}
static const uint8_t* oi_str(const ointern* t, uint32_t id, uint32_t* len) {
    const uint32_t* o = (const uint32_t*)t->offs.p;
    *len = o[id + 1] - o[id];
    return t->bytes.p + o[id];
}
static int oi_init(ointern* t) {
    memset(t, 0, sizeof(*t));
    t->cap = 1024;
    t->slots = (uint32_t*)calloc(t->cap, 4);
    if (!t->slots || ob_u32(&t->offs, 0) || ob_u32(&t->offs, 0)) return -1;
    t->n = 1;                                        /* id 0 = "" */
    return 0;
}
static int oi_grow(ointern* t) {
    uint32_t cap = t->cap * 2;
    uint32_t* s = (uint32_t*)calloc(cap, 4);
    if (!s) return -1;
    for (uint32_t id = 1; id < t->n; ++id) {
        uint32_t len;
        const uint8_t* p = oi_str(t, id, &len);
        uint32_t h = (uint32_t)ohash(p, len) & (cap - 1);
        while (s[h]) h = (h + 1) & (cap - 1);
        s[h] = id + 1;
    }
    free(t->slots);
    t->slots = s;
    t->cap = cap;
    return 0;
}
/* id of the string (first occurrence assigns the next id); "" is always 0 */
static int64_t oi_intern(ointern* t, const uint8_t* p, size_t len) {
    if (len == 0) return 0;
    if ((t->n + 1) * 2 > t->cap && oi_grow(t)) return -1;
    uint32_t h = (uint32_t)ohash(p, len) & (t->cap - 1);
    for (;;) {
        uint32_t v = t->slots[h];
        if (!v) break;
        uint32_t l2;
        const uint8_t* q = oi_str(t, v - 1, &l2);
        if (l2 == len && memcmp(p, q, len) == 0) return v - 1;
        h = (h + 1) & (t->cap - 1);
    }
    if (ob_put(&t->bytes, p, len) || ob_u32(&t->offs, (uint32_t)t->bytes.n)) return -1;
    t->slots[h] = t->n + 1;
    return t->n++;
}

/* ---------------------------------------------------------------- checkValid */
typedef struct {
    const uint8_t* s;
    size_t n, i;
    int err;             /* kdtn_json_err of the first error */
    size_t err_off;
} ovp;

static int is_ws(uint8_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }
static void skip_ws(ovp* v) { while (v->i < v->n && is_ws(v->s[v->i])) v->i++; }
static int vfail(ovp* v, int code) {
    if (!v->err) { v->err = code; v->err_off = v->i; }
    return -1;
}
static int is_hex(uint8_t c) { return (c >= '0' && c <= '9') || ((c | 32) >= 'a' && (c | 32) <= 'f'); }
static int is_dig(uint8_t c) { return c >= '0' && c <= '9'; }

/* scanner stateInString / stateInStringEsc / stateInStringEscU* (encoding/json/scanner.go) */
static int v_string(ovp* v) {
    v->i++;                                          /* opening quote */
    while (v->i < v->n) {
        uint8_t c = v->s[v->i];
        if (c == '"') { v->i++; return 0; }
        if (c < 0x20) return vfail(v, KDTN_JSON_SYNTAX);
        if (c == '\\') {
            /* the scanner stops at the byte it rejects: the escape byte, or the first non-hex
               digit of \uXXXX (stateInStringEsc / stateInStringEscU*); past the end: EOF */
            if (v->i + 1 >= v->n) { v->i = v->n; return vfail(v, KDTN_JSON_SYNTAX); }
            uint8_t e = v->s[v->i + 1];
            if (e == 'u') {
                for (int k = 0; k < 4; ++k) {
                    if (v->i + 2 + k >= v->n) { v->i = v->n; return vfail(v, KDTN_JSON_SYNTAX); }
                    if (!is_hex(v->s[v->i + 2 + k])) { v->i += 2 + k; return vfail(v, KDTN_JSON_SYNTAX); }
                }
                v->i += 6;
                continue;
            }
            if (!strchr("\"\\/bfnrt", e) || e == 0) { v->i += 1; return vfail(v, KDTN_JSON_SYNTAX); }
            v->i += 2;
            continue;
        }
        v->i++;
    }
    return vfail(v, KDTN_JSON_SYNTAX);              /* unterminated */
}
/* stateNeg / state0 / state1 / stateDot / stateE* */
static int v_number(ovp* v) {
    size_t i = v->i;
    if (i < v->n && v->s[i] == '-') i++;
    if (i >= v->n || !is_dig(v->s[i])) { v->i = i; return vfail(v, KDTN_JSON_SYNTAX); }
    if (v->s[i] == '0') i++;
    else while (i < v->n && is_dig(v->s[i])) i++;
    if (i < v->n && v->s[i] == '.') {
        i++;
        if (i >= v->n || !is_dig(v->s[i])) { v->i = i; return vfail(v, KDTN_JSON_SYNTAX); }
        while (i < v->n && is_dig(v->s[i])) i++;
    }
    if (i < v->n && (v->s[i] == 'e' || v->s[i] == 'E')) {
        i++;
        if (i < v->n && (v->s[i] == '+' || v->s[i] == '-')) i++;
        if (i >= v->n || !is_dig(v->s[i])) { v->i = i; return vfail(v, KDTN_JSON_SYNTAX); }
        while (i < v->n && is_dig(v->s[i])) i++;
    }
    v->i = i;
    return 0;
}
static int v_lit(ovp* v, const char* w) {
    size_t k = strlen(w);
    if (v->n - v->i < k || memcmp(v->s + v->i, w, k) != 0) return vfail(v, KDTN_JSON_SYNTAX);
    v->i += k;
    return 0;
}
/* parseState stack depth = number of open containers; maxNestingDepth = 10000 */
static int v_value(ovp* v, int depth) {
    skip_ws(v);
    if (v->i >= v->n) return vfail(v, KDTN_JSON_SYNTAX);
    uint8_t c = v->s[v->i];
    if (c == '{' || c == '[') {
        if (depth + 1 > 10000) return vfail(v, KDTN_JSON_DEPTH);
        const uint8_t close = c == '{' ? '}' : ']';
        v->i++;
        skip_ws(v);
        if (v->i < v->n && v->s[v->i] == close) { v->i++; return 0; }
        for (;;) {
            if (c == '{') {
                skip_ws(v);
                if (v->i >= v->n || v->s[v->i] != '"') return vfail(v, KDTN_JSON_SYNTAX);
                if (v_string(v)) return -1;
                skip_ws(v);
                if (v->i >= v->n || v->s[v->i] != ':') return vfail(v, KDTN_JSON_SYNTAX);
                v->i++;
            }
            if (v_value(v, depth + 1)) return -1;
            skip_ws(v);
            if (v->i >= v->n) return vfail(v, KDTN_JSON_SYNTAX);
            if (v->s[v->i] == ',') { v->i++; continue; }
            if (v->s[v->i] == close) { v->i++; return 0; }
            return vfail(v, KDTN_JSON_SYNTAX);
        }
    }
    if (c == '"') return v_string(v);
    if (c == '-' || is_dig(c)) return v_number(v);
    if (c == 't') return v_lit(v, "true");
    if (c == 'f') return v_lit(v, "false");
    if (c == 'n') return v_lit(v, "null");
    return vfail(v, KDTN_JSON_SYNTAX);
}

/* ---------------------------------------------------------------- unquote */
static int hex4(const uint8_t* p, const uint8_t* end) {    /* getu4: -1 unless \uXXXX */
    if (end - p < 6 || p[0] != '\\' || p[1] != 'u') return -1;
    int r = 0;
    for (int k = 2; k < 6; ++k) {
        uint8_t c = p[k];
        int d = c <= '9' ? c - '0' : (c | 32) - 'a' + 10;
        if (!is_hex(c)) return -1;
        r = r * 16 + d;
    }
    return r;
}
static size_t put_rune(uint8_t* o, uint32_t r) {             /* utf8.EncodeRune */
    if (r < 0x80) { o[0] = (uint8_t)r; return 1; }
    if (r < 0x800) { o[0] = 0xC0 | (r >> 6); o[1] = 0x80 | (r & 63); return 2; }
    if (r >= 0xD800 && r <= 0xDFFF) r = 0xFFFD;
    if (r < 0x10000) { o[0] = 0xE0 | (r >> 12); o[1] = 0x80 | ((r >> 6) & 63); o[2] = 0x80 | (r & 63); return 3; }
    o[0] = 0xF0 | (r >> 18); o[1] = 0x80 | ((r >> 12) & 63); o[2] = 0x80 | ((r >> 6) & 63); o[3] = 0x80 | (r & 63);
    return 4;
}
/* utf8.DecodeRune: byte length of a valid sequence at p, 0 if invalid (RuneError, 1) */
static size_t utf8_seq(const uint8_t* p, const uint8_t* end) {
    uint8_t c = p[0];
    size_t need;
    uint8_t lo = 0x80, hi = 0xBF;
    if (c >= 0xC2 && c <= 0xDF) need = 1;
    else if (c == 0xE0) { need = 2; lo = 0xA0; }
    else if (c >= 0xE1 && c <= 0xEC) need = 2;
    else if (c == 0xED) { need = 2; hi = 0x9F; }
    else if (c >= 0xEE && c <= 0xEF) need = 2;
    else if (c == 0xF0) { need = 3; lo = 0x90; }
    else if (c >= 0xF1 && c <= 0xF3) need = 3;
    else if (c == 0xF4) { need = 3; hi = 0x8F; }
    else return 0;
    if ((size_t)(end - p) < need + 1) return 0;
    if (p[1] < lo || p[1] > hi) return 0;
    for (size_t k = 2; k <= need; ++k)
        if (p[k] < 0x80 || p[k] > 0xBF) return 0;
    return need + 1;
}
/* decode.go unquoteBytes on a validated string literal at s[i] == '"'; output ≤ 3x input.
 * Returns the index after the closing quote. */
static size_t unquote(const uint8_t* s, size_t i, obuf* out) {
    out->n = 0;
    size_t end = i + 1;
    for (;;) {                                   /* closing quote: skip escapes */
        uint8_t c = s[end];
        if (c == '"') break;
        end += c == '\\' ? 2 : 1;
    }
    ob_reserve(out, (end - i) * 3 + 4);
    uint8_t* o = out->p;
    size_t w = 0, r = i + 1;
    const uint8_t* E = s + end;
    while (r < end) {
        uint8_t c = s[r];
        if (c == '\\') {
            uint8_t e = s[r + 1];
            switch (e) {
            case 'b': o[w++] = '\b'; r += 2; break;
            case 'f': o[w++] = '\f'; r += 2; break;
            case 'n': o[w++] = '\n'; r += 2; break;
            case 'r': o[w++] = '\r'; r += 2; break;
            case 't': o[w++] = '\t'; r += 2; break;
            case 'u': {
                int rr = hex4(s + r, E);
                r += 6;
                if (rr >= 0xD800 && rr < 0xE000) {          /* utf16.IsSurrogate */
                    int r1 = hex4(s + r, E);
                    if (rr < 0xDC00 && r1 >= 0xDC00 && r1 < 0xE000) {   /* utf16.DecodeRune */
                        r += 6;
                        w += put_rune(o + w, (uint32_t)(((rr - 0xD800) << 10) | (r1 - 0xDC00)) + 0x10000);
                        break;
                    }
                    rr = 0xFFFD;
                }
                w += put_rune(o + w, (uint32_t)rr);
                break;
            }
            default: o[w++] = e; r += 2; break;     /* " \ / */
            }
        } else if (c < 0x80) {
            o[w++] = c;
            r++;
        } else {
            size_t k = utf8_seq(s + r, E);
            if (!k) { w += put_rune(o + w, 0xFFFD); r++; }
            else { memcpy(o + w, s + r, k); w += k; r += k; }
        }
    }
    out->n = w;
    return end + 1;
}

/* ---------------------------------------------------------------- typed decode */
enum { SIDE_DES = 0, SIDE_REAL = 1 };
typedef struct {
    ovp v;               /* document + first error */
    obuf tmp;            /* unquote scratch        */
    ointern kd, pd;
    obuf t_ns, t_name, t_src, t_netns, t_flags, t_roff, t_doff;
    obuf key[2][KDTN_NKEY], prop[2][KDTN_NPROP], gap[2], uid[2];
    uint32_t T, n[2];
    int oom;
} odec;

static int dfail(odec* d, int code, size_t at) {
    if (!d->v.err) { d->v.err = code; d->v.err_off = at; }
    return -1;
}
/* skip any validated value */
static size_t skip_value(const uint8_t* s, size_t i) {
    while (is_ws(s[i])) i++;
    uint8_t c = s[i];
    if (c == '"') {
        i++;
        while (s[i] != '"') i += s[i] == '\\' ? 2 : 1;
        return i + 1;
    }
    if (c == '{' || c == '[') {
        int depth = 0;
        for (;;) {
            c = s[i];
            if (c == '"') { i++; while (s[i] != '"') i += s[i] == '\\' ? 2 : 1; i++; continue; }
            if (c == '{' || c == '[') depth++;
            else if (c == '}' || c == ']') { if (--depth == 0) return i + 1; }
            i++;
        }
    }
    while (!is_ws(s[i]) && s[i] != ',' && s[i] != ']' && s[i] != '}') i++;   /* scalar */
    return i;
}
static size_t next_tok(const uint8_t* s, size_t i) { while (is_ws(s[i])) i++; return i; }

typedef int (*field_fn)(odec*, size_t* i, int field, void* ctx);

/* Object members: key → field index via names[]; a repeated schema field is DUPKEY.
 * Calls fn for schema fields, skips others. *i at '{' on entry, after '}' on exit. */
static int d_object(odec* d, size_t* pi, const char* const* names, int nf, field_fn fn, void* ctx) {
    const uint8_t* s = d->v.s;
    size_t i = *pi + 1;
    uint64_t seen = 0;
    i = next_tok(s, i);
    if (s[i] == '}') { *pi = i + 1; return 0; }
    for (;;) {
        i = next_tok(s, i);
        const size_t key_at = i;
        i = unquote(s, i, &d->tmp);
        int f = -1;
        for (int k = 0; k < nf; ++k)
            if (strlen(names[k]) == d->tmp.n && memcmp(names[k], d->tmp.p, d->tmp.n) == 0) { f = k; break; }
        i = next_tok(s, i) + 1;                       /* ':' */
        i = next_tok(s, i);
        if (f >= 0) {
            if (seen >> f & 1) return dfail(d, KDTN_JSON_DUPKEY, key_at);
            seen |= 1ull << f;
            if (fn(d, &i, f, ctx)) return -1;
        } else {
            i = skip_value(s, i);
        }
        i = next_tok(s, i);
        if (s[i] == ',') { i++; continue; }
        *pi = i + 1;                                  /* '}' */
        return 0;
    }
}
static int is_null(const uint8_t* s, size_t i) { return s[i] == 'n'; }

/* string field: null leaves "", a string is unquoted and interned, anything else is a
 * type error. Writes the id into *slot. */
static int d_string(odec* d, size_t* pi, ointern* dict, uint32_t* slot) {
    const uint8_t* s = d->v.s;
    size_t i = *pi;
    if (is_null(s, i)) { *pi = i + 4; return 0; }
    if (s[i] != '"') return dfail(d, KDTN_JSON_TYPE, i);
    *pi = unquote(s, i, &d->tmp);
    int64_t id = oi_intern(dict, d->tmp.p, d->tmp.n);
    if (id < 0) { d->oom = 1; return -1; }
    *slot = (uint32_t)id;
    return 0;
}
/* number literal bounds (validated) */
static size_t num_end(const uint8_t* s, size_t i) {
    while (s[i] == '-' || s[i] == '+' || s[i] == '.' || s[i] == 'e' || s[i] == 'E' || is_dig(s[i])) i++;
    return i;
}
/* strconv.ParseInt(s, 10, 64) on the literal */
static int d_int64(odec* d, size_t* pi, int64_t* out) {
    const uint8_t* s = d->v.s;
    size_t i = *pi;
    if (is_null(s, i)) { *pi = i + 4; return 0; }
    if (!(s[i] == '-' || is_dig(s[i]))) return dfail(d, KDTN_JSON_TYPE, i);
    const size_t e = num_end(s, i);
    size_t k = i;
    int neg = s[k] == '-';
    if (neg) k++;
    uint64_t v = 0;
    for (; k < e; ++k) {
        if (!is_dig(s[k])) return dfail(d, KDTN_JSON_TYPE, i);
        if (v > (UINT64_MAX - 9) / 10) return dfail(d, KDTN_JSON_TYPE, i);
        v = v * 10 + (uint64_t)(s[k] - '0');
        if (v > (1ull << 63)) return dfail(d, KDTN_JSON_TYPE, i);
    }
    if (!neg && v > (uint64_t)INT64_MAX) return dfail(d, KDTN_JSON_TYPE, i);
    *out = neg ? (int64_t)(0 - v) : (int64_t)v;
    *pi = e;
    return 0;
}
/* strconv.ParseUint(s, 10, 64) + reflect OverflowUint for uint32 */
static int d_uint32(odec* d, size_t* pi, uint32_t* out) {
    const uint8_t* s = d->v.s;
    size_t i = *pi;
    if (is_null(s, i)) { *pi = i + 4; return 0; }
    if (!(s[i] == '-' || is_dig(s[i]))) return dfail(d, KDTN_JSON_TYPE, i);
    const size_t e = num_end(s, i);
    uint64_t v = 0;
    for (size_t k = i; k < e; ++k) {
        if (!is_dig(s[k])) return dfail(d, KDTN_JSON_TYPE, i);
        v = v * 10 + (uint64_t)(s[k] - '0');
        if (v > 0xFFFFFFFFull) return dfail(d, KDTN_JSON_TYPE, i);
    }
    *out = (uint32_t)v;
    *pi = e;
    return 0;
}

typedef struct { int side; uint32_t rec; } linkctx;

static uint32_t* col32(obuf* b, uint32_t i) { return (uint32_t*)b->p + i; }

static const char* const PROPS_NAMES[KDTN_NPROP + 1] = {
    "latency", "latency_corr", "jitter", "loss", "loss_corr", "rate", "duplicate",
    "duplicate_corr", "reorder_prob", "reorder_corr", "corrupt_prob", "corrupt_corr", "gap"};
static int f_props(odec* d, size_t* i, int f, void* vctx) {
    linkctx* L = (linkctx*)vctx;
    if (f < KDTN_NPROP) return d_string(d, i, &d->pd, col32(&d->prop[L->side][f], L->rec));
    return d_uint32(d, i, col32(&d->gap[L->side], L->rec));
}
static const char* const LINK_NAMES[KDTN_NKEY + 2] = {"local_intf", "local_ip", "local_mac",
                                                      "peer_intf", "peer_ip", "peer_mac",
                                                      "peer_pod", "uid", "properties"};
static int f_link(odec* d, size_t* i, int f, void* vctx) {
    linkctx* L = (linkctx*)vctx;
    if (f < KDTN_NKEY) return d_string(d, i, &d->kd, col32(&d->key[L->side][f], L->rec));
    if (f == KDTN_NKEY) return d_int64(d, i, (int64_t*)d->uid[L->side].p + L->rec);
    const uint8_t* s = d->v.s;                        /* properties: struct */
    if (is_null(s, *i)) { *i += 4; return 0; }
    if (s[*i] != '{') return dfail(d, KDTN_JSON_TYPE, *i);
    return d_object(d, i, PROPS_NAMES, KDTN_NPROP + 1, f_props, L);
}
static int new_record(odec* d, int side) {
    for (int k = 0; k < KDTN_NKEY; ++k) if (ob_u32(&d->key[side][k], 0)) return -1;
    for (int k = 0; k < KDTN_NPROP; ++k) if (ob_u32(&d->prop[side][k], 0)) return -1;
    int64_t z = 0;
    if (ob_u32(&d->gap[side], 0) || ob_put(&d->uid[side], &z, 8)) return -1;
    d->n[side]++;
    return 0;
}
/* []Link: null → nil (flag stays), array → elements (null element = zero Link) */
static int d_links(odec* d, size_t* pi, int side) {
    const uint8_t* s = d->v.s;
    size_t i = *pi;
    if (is_null(s, i)) { *pi = i + 4; return 0; }
    if (s[i] != '[') return dfail(d, KDTN_JSON_TYPE, i);
    d->t_flags.p[d->T - 1] &= (uint8_t)~(side == SIDE_DES ? KDTN_TOPO_SPEC_NIL : KDTN_TOPO_STATUS_NIL);
    i = next_tok(s, i + 1);
    if (s[i] == ']') { *pi = i + 1; return 0; }
    for (;;) {
        i = next_tok(s, i);
        if (new_record(d, side)) { d->oom = 1; return -1; }
        linkctx L = {side, d->n[side] - 1};
        if (is_null(s, i)) i += 4;
        else if (s[i] == '{') { if (d_object(d, &i, LINK_NAMES, KDTN_NKEY + 2, f_link, &L)) return -1; }
        else return dfail(d, KDTN_JSON_TYPE, i);
        i = next_tok(s, i);
        if (s[i] == ',') { i++; continue; }
        *pi = i + 1;
        return 0;
    }
}
static const char* const META_NAMES[2] = {"name", "namespace"};
static int f_meta(odec* d, size_t* i, int f, void* c) {
    (void)c;
    return d_string(d, i, &d->kd, col32(f ? &d->t_ns : &d->t_name, d->T - 1));
}
static const char* const SPEC_NAMES[1] = {"links"};
static int f_spec(odec* d, size_t* i, int f, void* c) { (void)f; (void)c; return d_links(d, i, SIDE_DES); }
static const char* const STATUS_NAMES[3] = {"links", "src_ip", "net_ns"};
static int f_status(odec* d, size_t* i, int f, void* c) {
    (void)c;
    if (f == 0) return d_links(d, i, SIDE_REAL);
    return d_string(d, i, &d->kd, col32(f == 1 ? &d->t_src : &d->t_netns, d->T - 1));
}
static int d_struct(odec* d, size_t* i, const char* const* names, int nf, field_fn fn) {
    const uint8_t* s = d->v.s;
    if (is_null(s, *i)) { *i += 4; return 0; }
    if (s[*i] != '{') return dfail(d, KDTN_JSON_TYPE, *i);
    return d_object(d, i, names, nf, fn, NULL);
}
static const char* const ITEM_NAMES[3] = {"metadata", "spec", "status"};
static int f_item(odec* d, size_t* i, int f, void* c) {
    (void)c;
    if (f == 0) return d_struct(d, i, META_NAMES, 2, f_meta);
    if (f == 1) return d_struct(d, i, SPEC_NAMES, 1, f_spec);
    return d_struct(d, i, STATUS_NAMES, 3, f_status);
}
static int new_topology(odec* d) {
    uint8_t fl = KDTN_TOPO_SPEC_NIL | KDTN_TOPO_STATUS_NIL;
    if (ob_u32(&d->t_ns, 0) || ob_u32(&d->t_name, 0) || ob_u32(&d->t_src, 0) ||
        ob_u32(&d->t_netns, 0) || ob_put(&d->t_flags, &fl, 1) || ob_u32(&d->t_roff, d->n[SIDE_REAL]) ||
        ob_u32(&d->t_doff, d->n[SIDE_DES]))
        return -1;
    d->T++;
    return 0;
}
static int f_root(odec* d, size_t* pi, int f, void* c) {
    (void)f; (void)c;
    const uint8_t* s = d->v.s;
    size_t i = *pi;
    if (is_null(s, i)) { *pi = i + 4; return 0; }
    if (s[i] != '[') return dfail(d, KDTN_JSON_TYPE, i);
    i = next_tok(s, i + 1);
    if (s[i] == ']') { *pi = i + 1; return 0; }
    for (;;) {
        i = next_tok(s, i);
        if (new_topology(d)) { d->oom = 1; return -1; }
        if (is_null(s, i)) i += 4;
        else if (s[i] == '{') { if (d_object(d, &i, ITEM_NAMES, 3, f_item, NULL)) return -1; }
        else return dfail(d, KDTN_JSON_TYPE, i);
        i = next_tok(s, i);
        if (s[i] == ',') { i++; continue; }
        *pi = i + 1;
        return 0;
    }
}
static const char* const ROOT_NAMES[1] = {"items"};

static uint32_t* take32(obuf* b) { uint32_t* p = (uint32_t*)b->p; b->p = NULL; b->n = b->cap = 0; return p; }

int or_json_ingest(const uint8_t* doc, uint64_t n, or_json_tables* out) {
    memset(out, 0, sizeof(*out));
    odec d;
    memset(&d, 0, sizeof(d));
    d.v.s = doc;
    d.v.n = n;
    /* checkValid: one value, then only whitespace */
    if (v_value(&d.v, 0) == 0) {
        skip_ws(&d.v);
        if (d.v.i != d.v.n) vfail(&d.v, KDTN_JSON_SYNTAX);
    }
    if (d.v.err) {
        out->json_err = d.v.err;
        out->err_offset = d.v.err_off;
        return 0;
    }
    if (oi_init(&d.kd) || oi_init(&d.pd)) return -1;
    /* the document is valid: decode with a NUL-free sentinel-less walk; every helper stays
       inside the validated literal boundaries */
    size_t i = next_tok(doc, 0);
    int rc = 0;
    if (is_null(doc, i)) rc = 0;
    else if (doc[i] != '{') rc = dfail(&d, KDTN_JSON_TYPE, i);
    else rc = d_object(&d, &i, ROOT_NAMES, 1, f_root, NULL);
    if (d.oom) return -1;
    (void)rc;
    out->json_err = d.v.err;
    out->err_offset = d.v.err ? d.v.err_off : 0;
    if (ob_u32(&d.t_roff, d.n[SIDE_REAL]) || ob_u32(&d.t_doff, d.n[SIDE_DES])) return -1;
    out->T = d.T;
    out->N = d.n[SIDE_DES];
    out->M = d.n[SIDE_REAL];
    out->n_kdict = d.kd.n;
    out->n_pdict = d.pd.n;
    out->kd_bytes = d.kd.bytes.p; out->kdict_bytes = d.kd.bytes.n;
    out->kd_offs = take32(&d.kd.offs);
    out->pd_bytes = d.pd.bytes.p; out->pdict_bytes = d.pd.bytes.n;
    out->pd_offs = take32(&d.pd.offs);
    free(d.kd.slots);
    free(d.pd.slots);
    out->ns = take32(&d.t_ns);
    out->name = take32(&d.t_name);
    out->src_ip = take32(&d.t_src);
    out->net_ns = take32(&d.t_netns);
    out->flags = d.t_flags.p;
    out->real_off = take32(&d.t_roff);
    out->des_off = take32(&d.t_doff);
    for (int side = 0; side < 2; ++side) {
        const uint32_t m = d.n[side];
        uint32_t* key = (uint32_t*)malloc((size_t)KDTN_NKEY * m * 4 + 4);
        uint32_t* prop = (uint32_t*)malloc((size_t)KDTN_NPROP * m * 4 + 4);
        if (!key || !prop) return -1;
        for (int k = 0; k < KDTN_NKEY; ++k) {
            if (m) memcpy(key + (size_t)k * m, d.key[side][k].p, (size_t)m * 4);
            free(d.key[side][k].p);
        }
        for (int k = 0; k < KDTN_NPROP; ++k) {
            if (m) memcpy(prop + (size_t)k * m, d.prop[side][k].p, (size_t)m * 4);
            free(d.prop[side][k].p);
        }
        if (side == SIDE_DES) {
            out->des_key = key; out->des_prop = prop;
            out->des_gap = take32(&d.gap[side]); out->des_uid = (int64_t*)d.uid[side].p;
        } else {
            out->real_key = key; out->real_prop = prop;
            out->real_gap = take32(&d.gap[side]); out->real_uid = (int64_t*)d.uid[side].p;
        }
    }
    free(d.tmp.p);
    return 0;
}

void or_json_free(or_json_tables* t) {
    void* ps[] = {t->kd_bytes, t->kd_offs, t->pd_bytes, t->pd_offs, t->ns, t->name, t->src_ip,
                  t->net_ns, t->flags, t->real_off, t->des_off, t->des_key, t->des_prop,
                  t->des_gap, t->des_uid, t->real_key, t->real_prop, t->real_gap, t->real_uid};
    for (size_t k = 0; k < sizeof(ps) / sizeof(ps[0]); ++k) free(ps[k]);
    memset(t, 0, sizeof(*t));
}
