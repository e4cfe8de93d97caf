// kdtn_ingest.hip — CR ingest on the GPU: a Kubernetes TopologyList
// JSON document in HBM → the epoch tables kdtn_epoch_run consumes (interned dictionaries,
// topology table, both AoSoA link stores), following Go's encoding/json as forked by
// sigs.k8s.io/json (see include/kdtn.h kdtn_json_ingest; CPU restatement and parity oracle:
// oracle/kdtn_oracle_json.c).
//
// The document is processed as 64-byte blocks (one lane each, bit k of a block mask =
// byte k) and then as a token stream, bit-parallel in the style of structural indexing:
//   k_js_quotes     backslash / quote / high-bit masks; unescaped quotes (escape runs)
//   [scan]          quote counts → in-string state at every block start (parity)
//   k_js_classify   in-string mask (prefix XOR), structural / string-open / scalar-start
//                   token bits, opens / closes, control bytes
//   [scan x2]       token offsets, nesting depth at every block start
//   k_js_tokens     token stream: {byte offset, pre-depth | kind << 24}
//   k_js_par_*      parent (enclosing container) of every token: per depth level d ≤ 16 the
//                   last open bracket with post-depth d before the token, an element-wise
//                   max-scan over 4096-token tiles; deeper tokens walk back (k_js_deep)
//   k_js_validate   checkValid as local rules on (previous token, token, container kind),
//                   string escapes and number / literal grammar, bracket matching
//   k_js_roles      schema role of every container (items, metadata, spec, links, ...)
//   k_js_elems_*    ordinals of items and links elements (tile counts + scans) → topology
//                   index, record index and the per-topology record offsets
//   k_js_values     every schema field: type check, duplicate check, uid / gap parse, and
//                   string interning into a lock-free open-addressing table (64-bit CAS of
//                   a self-describing key {tag, heap, len, off}); atomicMin keeps each
//                   string's first occurrence
//   k_js_rep_mark / k_js_ids / k_js_dict_copy / k_js_finalize
//                   ids = rank of the first occurrence in document order (bitmap popcount
//                   scan), dictionary arenas in id order, table slots → ids
#include "kdtn_kernels.h"
#include "kdtn_shard.h"

namespace kdtn {

// ---------------------------------------------------------------- byte-class SWAR helpers
KD_INLINE uint32_t mm4(uint32_t z) { return ((z >> 7) * 0x10204080u) >> 28; }   // bits 7,15,23,31 → 4 bits
KD_INLINE uint32_t eqb(uint32_t w, uint32_t c) {                                 // byte == c
    const uint32_t t = w ^ (c * 0x01010101u);
    return ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t) & 0x80808080u;
}
KD_INLINE uint32_t ltb(uint32_t w, uint32_t n) {                                 // byte < n (n ≤ 128)
    return ~(((w & 0x7F7F7F7Fu) + (128u - n) * 0x01010101u) | w) & 0x80808080u;
}
KD_INLINE uint32_t digb(uint32_t w) { return ltb(w, 0x3Au) & ~ltb(w, 0x30u); }  // byte in '0'..'9'
// bit k = byte k of a 32-byte register window is a decimal digit
KD_INLINE uint32_t digit_mask(const uint32_t u[8]) {
    uint32_t D = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) D |= mm4(digb(u[k])) << (4 * k);
    return D;
}
// byte q (< 32, not a compile-time constant) of a register window
KD_INLINE uint32_t win_byte_at(const uint32_t u[8], uint32_t q) {
    const uint32_t i = q >> 2;
    uint32_t w = u[0];
#pragma unroll
    for (int k = 1; k < 8; ++k) w = i == (uint32_t)k ? u[k] : w;
    return (w >> (8 * (q & 3u))) & 0xFFu;
}
// first non-digit byte at or after st (0 or 1) of the window: 32 when the rest is digits
KD_INLINE uint32_t first_non_digit(uint32_t D, uint32_t st) {
    return st + (uint32_t)__builtin_ctzll(~((uint64_t)D >> st));
}
KD_INLINE uint64_t prefix_xor(uint64_t x) {
    x ^= x << 1; x ^= x << 2; x ^= x << 4; x ^= x << 8; x ^= x << 16; x ^= x << 32;
    return x;
}
KD_INLINE void load_block(const uint8_t* doc, uint32_t b, uint32_t w[16]) {
    const uint4* p = reinterpret_cast<const uint4*>(doc + (size_t)b * 64);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint4 v = p[k];
        w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
    }
}
KD_INLINE void js_fail(unsigned long long* err, uint32_t pos, uint32_t code) {
    atomicMin(err, ((unsigned long long)pos << 8) | code);
}
KD_INLINE bool is_struct_byte(uint32_t c) {
    return c == '{' || c == '}' || c == '[' || c == ']' || c == ':' || c == ',';
}

KD_INLINE uint32_t esc_byte(uint32_t x) {          // \b \f \n \r \t; \" \\ \/ stand for themselves
    switch (x) {
    case 'b': return 0x08u;
    case 'f': return 0x0Cu;
    case 'n': return 0x0Au;
    case 'r': return 0x0Du;
    case 't': return 0x09u;
    default: return x;
    }
}
// ---------------------------------------------------------------- k_js_quotes
// Per-workgroup sums of per-block counts (BLOCK blocks of 64 bytes per workgroup): the scans
// run over these group partials only, and the consumer rebuilds a block's offset as its group's
// offset plus a workgroup scan of counts it derives from its own masks (no per-block count or
// offset arrays). Fields of `a` are 16-bit (≤ 64 per block, ≤ 16384 per group).
KD_INLINE void group_sums(uint64_t a, uint64_t d, uint64_t* sh, uint32_t* g, uint32_t ng) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        a += __shfl_xor(a, o, 64);
        d += __shfl_xor(d, o, 64);
    }
    if (lane == 0) { sh[wave] = a; sh[BLOCK / 64 + wave] = d; }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t ta = 0, td = 0;
#pragma unroll
        for (int k = 0; k < BLOCK / 64; ++k) { ta += sh[k]; td += sh[BLOCK / 64 + k]; }
        const uint32_t x = blockIdx.x;
        g[x] = (uint32_t)(ta & 0xFFFFu);                    // tokens
        g[ng + x] = (uint32_t)td;                            // 64 + opens - closes
        g[2 * ng + x] = (uint32_t)((ta >> 16) & 0xFFFFu);    // opens
        g[3 * ng + x] = (uint32_t)((ta >> 32) & 0xFFFFu);    // colons
        g[4 * ng + x] = (uint32_t)(ta >> 48);                // scalars
    }
}

KD_INLINE uint32_t quote_block(const JsDoc& j, uint32_t b, uint64_t* qmask, uint64_t* bsmask, uint64_t* hbmask,
                                uint64_t* escmask);

__global__ void __launch_bounds__(BLOCK) k_js_quotes(JsDoc j, uint64_t* qmask, uint64_t* bsmask,
                                                     uint64_t* hbmask, uint64_t* escmask, uint32_t* gq) {
    __shared__ uint64_t sh[BLOCK / 64];
    const uint32_t b = blockIdx.x * BLOCK + threadIdx.x;
    uint32_t nq = 0;
    if (b < j.nb) nq = quote_block(j, b, qmask, bsmask, hbmask, escmask);
    uint32_t x = nq;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o, 64);
    if ((threadIdx.x & 63u) == 0) sh[threadIdx.x >> 6] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
#pragma unroll
        for (int k = 0; k < BLOCK / 64; ++k) t += sh[k];
        gq[blockIdx.x] = (uint32_t)t;
    }
}

KD_INLINE uint32_t quote_block(const JsDoc& j, uint32_t b, uint64_t* qmask, uint64_t* bsmask, uint64_t* hbmask,
                                uint64_t* escmask) {
    uint32_t w[16];
    load_block(j.doc, b, w);
    uint64_t bs = 0, q = 0, hb = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        bs |= (uint64_t)mm4(eqb(w[k], '\\')) << (4 * k);
        q |= (uint64_t)mm4(eqb(w[k], '"')) << (4 * k);
        hb |= (uint64_t)mm4(w[k] & 0x80808080u) << (4 * k);
    }
    // is byte 0 escaped? an odd run of backslashes ends right before the block
    bool pe = false;
    if (b > 0 && j.doc[(size_t)b * 64 - 1] == '\\') {
        uint64_t i = (uint64_t)b * 64 - 1, run = 0;
        for (;;) {
            if (j.doc[i] != '\\') break;
            ++run;
            if (i == 0) break;
            --i;
        }
        pe = run & 1;
    }
    uint64_t esc = 0;
    if (bs | (uint64_t)pe) {                  // escaped byte = one after an odd backslash run
        bool e = pe;
        for (int k = 0; k < 64; ++k) {
            if (e) { esc |= 1ull << k; e = false; }
            else if ((bs >> k) & 1) e = true;
        }
    }
    const uint64_t quote = q & ~esc;
    qmask[b] = quote;
    bsmask[b] = bs;
    hbmask[b] = hb;
    escmask[b] = esc;                         // k_js_classify checks these bytes (no second run scan)
    return __popcll(quote);
}

// ---------------------------------------------------------------- k_js_classify
KD_INLINE bool is_hexc(uint32_t c) { return (c >= '0' && c <= '9') || ((c | 32) >= 'a' && (c | 32) <= 'f'); }
KD_INLINE void classify_block(const JsDoc& j, uint32_t b, uint64_t quote, bool S, const JsMasks& m,
                              unsigned long long* err, uint64_t* pa, uint64_t* pd);

__global__ void __launch_bounds__(BLOCK) k_js_classify(JsDoc j, const uint64_t* gqoff, JsMasks m, uint32_t ng,
                                                       unsigned long long* err) {
    __shared__ uint64_t sh[2 * (BLOCK / 64)];
    const uint32_t b = blockIdx.x * BLOCK + threadIdx.x;
    const bool valid = b < j.nb;
    const uint64_t quote = valid ? j.qmask[b] : 0;
    uint64_t qt;
    const uint64_t qo = gqoff[blockIdx.x] + block_exclusive(__popcll(quote), sh, &qt);
    uint64_t pa = 0, pd = 0;
    if (valid) classify_block(j, b, quote, qo & 1, m, err, &pa, &pd);
    group_sums(pa, pd, sh, m.gcnt, ng);
}

KD_INLINE void classify_block(const JsDoc& j, uint32_t b, uint64_t quote, bool S, const JsMasks& m,
                              unsigned long long* err, uint64_t* pa, uint64_t* pd) {
    uint32_t w[16];
    load_block(j.doc, b, w);
    uint64_t op = 0, cl = 0, pun = 0, ctl = 0, wsc = 0, colon = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t lw = w[k] | 0x20202020u;            // '[' → '{', ']' → '}'
        const uint32_t o = mm4(eqb(lw, '{')), c = mm4(eqb(lw, '}'));
        op |= (uint64_t)o << (4 * k);
        cl |= (uint64_t)c << (4 * k);
        const uint32_t cn = mm4(eqb(w[k], ':'));
        colon |= (uint64_t)cn << (4 * k);
        pun |= (uint64_t)(cn | mm4(eqb(w[k], ','))) << (4 * k);
        ctl |= (uint64_t)mm4(ltb(w[k], 0x20)) << (4 * k);
        wsc |= (uint64_t)mm4(ltb(w[k], 0x21)) << (4 * k);
    }
    // S: inside a string at byte 0 (odd number of quotes before the block)
    const uint64_t instr = prefix_xor(quote) ^ (S ? ~0ull : 0ull);
    const uint64_t out = ~instr;
    const uint64_t structural = (op | cl | pun) & out;
    const uint64_t str_open = quote & instr;
    const uint64_t scalar = out & ~quote & ~wsc & ~(op | cl | pun);
    bool prev_scalar = false;
    if (b > 0 && !S) {
        const uint32_t c = j.doc[(size_t)b * 64 - 1];
        prev_scalar = !(c <= 0x20 || c == '"' || is_struct_byte(c));
    }
    const uint64_t scalar_start = scalar & ~((scalar << 1) | (uint64_t)prev_scalar);
    const uint64_t tok = structural | str_open | scalar_start;
    // escapes (checkValid's stateInStringEsc*): the byte after an odd backslash run (k_js_quotes'
    // escaped-byte mask) must be one of " \ / b f n r t, or u and four hex digits. Reported where
    // the scanner stops: at the escape byte, or at the first non-hex digit of \uXXXX (an escape
    // cut by the document's end at its length). A backslash outside a string fails the grammar
    // anyway, so the check needs no string state.
    uint64_t escm = j.escmask[b];
    while (escm) {
        const int k = __ffsll((long long)escm) - 1;
        escm &= escm - 1;
        const uint32_t c = (w[k >> 2] >> (8 * (k & 3))) & 0xFFu;
        const unsigned long long p = (unsigned long long)b * 64 + k;
        unsigned long long at = ~0ull;
        if (c == 'u') {                                       // (the document is padded past its end)
            for (int i = 1; i <= 4 && at == ~0ull; ++i)
                if (!is_hexc(j.doc[p + i])) at = p + i;
        } else if (!(c == '"' || c == '\\' || c == '/' || c == 'b' || c == 'f' || c == 'n' || c == 'r' || c == 't')) {
            at = p;
        }
        if (at != ~0ull) js_fail(err, at < j.n ? at : (unsigned long long)j.n, KDTN_JSON_SYNTAX);
    }
    // control bytes: never inside a string; outside only \t \n \r
    if (ctl) {
        uint64_t bad = ctl & instr;
        uint64_t octl = ctl & out;
        while (octl) {
            const int k = __ffsll((long long)octl) - 1;
            octl &= octl - 1;
            const uint32_t c = j.doc[(size_t)b * 64 + k];
            if (c != '\t' && c != '\n' && c != '\r') bad |= 1ull << k;
        }
        if (bad) js_fail(err, b * 64 + (__ffsll((long long)bad) - 1), KDTN_JSON_SYNTAX);
    }
    m.tok[b] = tok;                                        // (with the separators: k_js_tokens tells them apart)
    m.open[b] = op & out;
    m.close[b] = cl & out;
    *pa = (uint64_t)__popcll(tok & ~(pun & out)) | (uint64_t)__popcll(op & out) << 16 |
          (uint64_t)__popcll(colon & out) << 32 | (uint64_t)__popcll(scalar_start) << 48;
    *pd = 64u + __popcll(op & out) - __popcll(cl & out);
}

// ---------------------------------------------------------------- k_js_tokens
KD_INLINE uint32_t kind_of(uint32_t c) {
    switch (c) {
    case '{': return TK_OBJ;
    case '}': return TK_OBJ_END;
    case '[': return TK_ARR;
    case ']': return TK_ARR_END;
    case ':': return TK_COLON;
    case ',': return TK_COMMA;
    case '"': return TK_STR;
    default: return TK_SCALAR;
    }
}

// position of the r-th (0-based) set bit of m (r < popcount(m)): the 32-bit half first, then
// a 32-bit binary search (halves the 64-bit popcount / shift work of a 64-bit search)
KD_INLINE uint32_t select_bit(uint64_t m, uint32_t r) {
    const uint32_t lo = (uint32_t)m, c = __popc(lo);
    const bool up = r >= c;
    uint32_t x = up ? (uint32_t)(m >> 32) : lo;
    r = up ? r - c : r;
    uint32_t pos = up ? 32u : 0u;
#pragma unroll
    for (int w = 16; w >= 1; w >>= 1) {
        const uint32_t cw = __popc(x & ((1u << w) - 1u));
        const bool hi = r >= cw;
        r = hi ? r - cw : r;
        x = hi ? x >> w : x;
        pos += hi ? (uint32_t)w : 0u;
    }
    return pos;
}

KD_INLINE bool is_ws(uint32_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }

// The separators between a token at pos and the previous one, from the bytes before pos: only
// whitespace, ',' and ':' lie between two tokens (every other byte outside a string starts or
// ends a token), so a backward scan needs no string state. Returns SEP_* of the earliest
// separator (SEP_NONE: none) and, in *second, the position of the second separator in document
// order (0xFFFFFFFF: fewer than two). byte(q) reads the document.
template <typename B>
KD_INLINE uint32_t sep_before(uint32_t pos, uint32_t* second, B&& byte) {
    uint32_t q = pos, kind = SEP_NONE, p1 = 0xFFFFFFFFu, p2 = 0xFFFFFFFFu;
    while (q > 0) {
        const uint32_t c = byte(q - 1);
        if (is_ws(c)) { --q; continue; }
        if (c != ':' && c != ',') break;
        p2 = p1;                                           // (found in reverse document order)
        p1 = q - 1;
        kind = c == ':' ? SEP_COLON : SEP_COMMA;
        --q;
    }
    *second = p2;
    return kind;
}

// Token writer. Each lane owns one 64-byte block (its bytes go to LDS, its masks and offsets
// to per-lane LDS slots); the wave's tokens are contiguous in the stream, so the wave writes them
// round by round, lane l taking the wave's token r = round * 64 + l (owner block by binary
// search over the wave's token prefix, bit by select): coalesced 4-byte stores instead of
// every lane walking its own block's tokens into its own region. The ',' and ':' bytes are no
// tokens (m.tok holds them; they are told apart here): a token records the separator before it
// (sep_before), and a member value (a token after a ':') is the C-th entry of vlist, C = the
// number of structural colons before it, less one (the colon it follows is the last of them,
// in this block or an earlier one).
__global__ void __launch_bounds__(BLOCK) k_js_tokens(JsDoc j, JsMasks m, const uint64_t* goff, uint32_t ng,
                                                     JsToks tk, uint32_t* olist, uint8_t* odep, uint32_t* vlist,
                                                     uint32_t* slist, unsigned long long* err) {
    __shared__ uint4 blk[BLOCK * 4];
    __shared__ uint64_t stok[BLOCK], sop[BLOCK], scl[BLOCK], scol[BLOCK], ssc[BLOCK];
    __shared__ int64_t sd0[BLOCK];
    __shared__ uint32_t sex[BLOCK], soo[BLOCK], sco[BLOCK], sso[BLOCK];
    __shared__ uint64_t shs[BLOCK / 64];
    // per wave: bit t of sb = token rank t starts a block; spw = popcounts of sb's earlier words;
    // smap = the lane of the n-th block that has tokens (the owner block of a rank in two steps)
    __shared__ uint64_t sb[BLOCK];
    __shared__ uint32_t spw[BLOCK];
    __shared__ uint8_t smap[BLOCK];
    const uint32_t lane = threadIdx.x & 63u, w0 = threadIdx.x & ~63u;
    sb[threadIdx.x] = 0;
    const uint32_t b = blockIdx.x * BLOCK + threadIdx.x;
    uint64_t tok = 0, pa = 0, pd = 0, colm = 0;
    if (b < j.nb) {
        const uint4* p = reinterpret_cast<const uint4*>(j.doc + (size_t)b * 64);
        uint4 v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = p[q];
        const uint64_t tsep = m.tok[b];                  // tokens and the structural separators
        const uint64_t op = m.open[b], cl = m.close[b];
        sop[threadIdx.x] = op;
        scl[threadIdx.x] = cl;
        uint64_t col = 0, cmm = 0, nsc = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            blk[threadIdx.x * 4 + q] = v[q];
            const uint32_t wd[4] = {v[q].x, v[q].y, v[q].z, v[q].w};
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                const uint32_t x = wd[h], lx = x | 0x20202020u;       // '[' → '{', ']' → '}'
                const uint32_t cn = mm4(eqb(x, ':')), cm = mm4(eqb(x, ','));
                col |= (uint64_t)cn << (4 * (q * 4 + h));
                cmm |= (uint64_t)cm << (4 * (q * 4 + h));
                nsc |= (uint64_t)(cn | cm | mm4(eqb(lx, '{') | eqb(lx, '}') | eqb(x, '"'))) << (4 * (q * 4 + h));
            }
        }
        colm = col & tsep;                               // structural colons
        tok = tsep & ~(col | cmm);                       // the tokens
        scol[threadIdx.x] = colm;
        ssc[threadIdx.x] = tok & ~nsc;                   // scalar token starts (the token's first byte)
        // the block's counts, as k_js_classify summed them per workgroup
        pa = (uint64_t)__popcll(tok) | (uint64_t)__popcll(op) << 16 | (uint64_t)__popcll(colm) << 32 |
             (uint64_t)__popcll(tok & ~nsc) << 48;
        pd = 64u + __popcll(op) - __popcll(cl);
    }
    // the block's offsets: its workgroup's (scanned group partials) + a workgroup scan
    uint64_t ta, td;
    const uint64_t ea = block_exclusive(pa, shs, &ta);
    const uint64_t ed = block_exclusive(pd, shs, &td);
    const uint32_t g = blockIdx.x, G = ng + 1;
    const uint64_t ti = goff[g] + (ea & 0xFFFFu);
    sd0[threadIdx.x] = (int64_t)(goff[G + g] + ed) - 64ll * b;
    soo[threadIdx.x] = (uint32_t)(goff[2 * G + g] + ((ea >> 16) & 0xFFFFu));
    sco[threadIdx.x] = (uint32_t)(goff[3 * G + g] + ((ea >> 32) & 0xFFFFu));
    sso[threadIdx.x] = (uint32_t)(goff[4 * G + g] + (ea >> 48));
    stok[threadIdx.x] = tok;
    const uint32_t cnt = __popcll(tok);
    uint32_t inc = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(inc, d, 64);
        if (lane >= (uint32_t)d) inc += o;
    }
    sex[threadIdx.x] = inc - cnt;
    const uint32_t wtot = __shfl(inc, 63, 64);
    const uint32_t base = (uint32_t)__shfl(ti, 0, 64);  // toff of the wave's first block
    {
        const uint64_t ne = __ballot(cnt != 0);
        if (cnt) {
            const uint32_t first = inc - cnt;              // < 4096: a wave holds 64 blocks
            atomicOr(reinterpret_cast<unsigned long long*>(&sb[w0 + (first >> 6)]), 1ull << (first & 63u));
            smap[w0 + __popcll(ne & ((1ull << lane) - 1ull))] = (uint8_t)lane;
        }
    }
    __syncthreads();
    {
        const uint32_t c = __popcll(sb[threadIdx.x]);
        uint32_t s = c;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = __shfl_up(s, d, 64);
            if (lane >= (uint32_t)d) s += o;
        }
        spw[threadIdx.x] = s - c;
    }
    __syncthreads();
    // document bytes: the workgroup's blocks from LDS, others from global memory
    const uint32_t wg0 = blockIdx.x * BLOCK * 64u;
    const uint8_t* bytes = reinterpret_cast<const uint8_t*>(blk);
    auto byte_at = [&](uint32_t q) -> uint32_t {
        return (q >= wg0 && q - wg0 < BLOCK * 64u && (q >> 6) < j.nb) ? bytes[q - wg0] : j.doc[q];
    };
    for (uint32_t r = lane; r < wtot; r += 64) {
        // owner block of rank r: the blocks starting at or before r (the round's word of sb is
        // one broadcast read), then the lane of that many-th block with tokens
        const uint32_t wd = r >> 6;
        const uint32_t nb = spw[w0 + wd] + (uint32_t)__popcll(sb[w0 + wd] & ((2ull << lane) - 1ull));
        const uint32_t o = w0 + smap[w0 + nb - 1];
        const uint32_t k = select_bit(stok[o], r - sex[o]);
        const uint64_t below = (1ull << k) - 1;
        int64_t d = sd0[o] + __popcll(sop[o] & below) - __popcll(scl[o] & below);
        const uint32_t bb = blockIdx.x * BLOCK + o;
        const uint32_t pos = bb * 64 + k;
        const uint32_t kind = kind_of(reinterpret_cast<const uint8_t*>(blk + o * 4)[k]);
        if (d < 0 || ((kind == TK_OBJ_END || kind == TK_ARR_END) && d < 1)) {
            js_fail(err, pos, KDTN_JSON_SYNTAX);      // a close with nothing open
            d = d < 0 ? 0 : d;
        }
        uint32_t second;
        const uint32_t sep = sep_before(pos, &second, byte_at);
        if (second != 0xFFFFFFFFu) js_fail(err, second, KDTN_JSON_SYNTAX);   // two separators in a row
        const uint32_t idx = base + r;
        if (sep == SEP_COLON) vlist[sco[o] + __popcll(scol[o] & below) - 1] = idx;   // >= 1 colon before it
        if (kind == TK_OBJ || kind == TK_ARR) {
            if (d >= 10000) js_fail(err, pos, KDTN_JSON_DEPTH);
            const uint32_t oi = soo[o] + __popcll(sop[o] & below);
            olist[oi] = idx;
            odep[oi] = (uint8_t)(d > 254 ? 255 : d);             // k_js_roles picks its level by this byte
        } else if (kind == TK_SCALAR) {
            slist[sso[o] + __popcll(ssc[o] & below)] = idx;         // checked by k_js_scalars
        }
        if (d > (int64_t)TK_DEPTH_MASK) d = TK_DEPTH_MASK;
        tk.pos[idx] = pos;
        tk.meta[idx] = (uint32_t)d | (kind << 24) | (sep << 28);
    }
}

// ---------------------------------------------------------------- parents
// Per tile of JS_TILE tokens: lane d (0..JS_PD-1) = 1 + index of the last open bracket whose
// post-depth is d + 1 (pre-depth d), 0 = none; combining is an element-wise max.
KD_INLINE bool tk_open(uint32_t meta) {
    const uint32_t k = (meta >> 24) & 0xFu;
    return k == TK_OBJ || k == TK_ARR;
}

__global__ void __launch_bounds__(BLOCK) k_js_par_agg(const uint32_t* tmeta, uint32_t ntok, uint32_t* tagg) {
    __shared__ uint32_t sh[BLOCK * (JS_PD + 1)];
    uint32_t* row = sh + threadIdx.x * (JS_PD + 1);
#pragma unroll
    for (int d = 0; d < JS_PD; ++d) row[d] = 0;
    // a tile's aggregate is a max, so the tokens are read coalesced (token t0 + q*BLOCK + tid)
    const uint32_t t0 = blockIdx.x * JS_TILE;
    for (int q = 0; q < JS_PER; ++q) {
        const uint32_t i = t0 + q * BLOCK + threadIdx.x;
        if (i >= ntok) break;
        const uint32_t meta = tmeta[i];
        const uint32_t d = meta & TK_DEPTH_MASK;
        if (tk_open(meta) && d < JS_PD) row[d] = i + 1;
    }
    __syncthreads();
    // the max over the 256 rows per lane in two levels (16 parts of 16 rows, then the parts):
    // one thread walking all 256 rows per lane was a serial chain of dependent LDS reads
    __shared__ uint32_t red[BLOCK];
    {
        constexpr int NP = BLOCK / JS_PD, RP = BLOCK / NP;          // 16 parts of 16 rows
        const uint32_t d = threadIdx.x & (JS_PD - 1), part = threadIdx.x / JS_PD;
        uint32_t v = 0;
#pragma unroll
        for (int t = 0; t < RP; ++t) v = max(v, sh[(part * RP + t) * (JS_PD + 1) + d]);
        red[threadIdx.x] = v;
    }
    __syncthreads();
    if (threadIdx.x < JS_PD) {
        uint32_t v = 0;
#pragma unroll
        for (int p = 0; p < BLOCK / JS_PD; ++p) v = max(v, red[p * JS_PD + threadIdx.x]);
        tagg[(size_t)blockIdx.x * JS_PD + threadIdx.x] = v;
    }
}

// groups of BLOCK tiles: per-group max per lane
__global__ void __launch_bounds__(BLOCK) k_js_par_group(const uint32_t* tagg, uint32_t ntiles, uint32_t* gagg) {
    __shared__ uint32_t sh[BLOCK];
    const int lane = threadIdx.x & (JS_PD - 1), part = threadIdx.x / JS_PD;   // 16 parts of 16 tiles
    uint32_t v = 0;
    for (int k = 0; k < BLOCK / (BLOCK / JS_PD); ++k) {
        const uint32_t t = blockIdx.x * BLOCK + part * (BLOCK / (BLOCK / JS_PD)) + k;
        if (t < ntiles) v = max(v, tagg[(size_t)t * JS_PD + lane]);
    }
    sh[threadIdx.x] = v;
    __syncthreads();
    if (threadIdx.x < JS_PD) {
        uint32_t r = 0;
        for (int p = 0; p < BLOCK / JS_PD; ++p) r = max(r, sh[p * JS_PD + threadIdx.x]);
        gagg[(size_t)blockIdx.x * JS_PD + threadIdx.x] = r;
    }
}

// single block: exclusive max-scan over the groups, in place
__global__ void __launch_bounds__(BLOCK) k_js_par_top(uint32_t* gagg, uint32_t ng) {
    __shared__ uint32_t sh[BLOCK];
    const int lane = threadIdx.x & (JS_PD - 1), part = threadIdx.x / JS_PD;
    constexpr int NP = BLOCK / JS_PD;
    const uint32_t per = (ng + NP - 1) / NP;
    const uint32_t g0 = part * per, g1 = min(ng, g0 + per);
    uint32_t v = 0;
    for (uint32_t g = g0; g < g1; ++g) v = max(v, gagg[(size_t)g * JS_PD + lane]);
    sh[threadIdx.x] = v;
    __syncthreads();
    uint32_t run = 0;
    for (int p = 0; p < part; ++p) run = max(run, sh[p * JS_PD + lane]);
    for (uint32_t g = g0; g < g1; ++g) {
        const uint32_t x = gagg[(size_t)g * JS_PD + lane];
        gagg[(size_t)g * JS_PD + lane] = run;
        run = max(run, x);
    }
}

// within each group: exclusive max-scan over its tiles → texcl (in place over tagg)
__global__ void __launch_bounds__(BLOCK) k_js_par_tiles(uint32_t* tagg, uint32_t ntiles, const uint32_t* gagg) {
    __shared__ uint32_t sh[2][BLOCK * JS_PD];
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    uint32_t* cur = sh[0];
    uint32_t* nxt = sh[1];
#pragma unroll
    for (int d = 0; d < JS_PD; ++d) cur[d * BLOCK + threadIdx.x] = t < ntiles ? tagg[(size_t)t * JS_PD + d] : 0u;
    __syncthreads();
    for (int off = 1; off < BLOCK; off <<= 1) {                  // inclusive Hillis-Steele, [lane][thread]
#pragma unroll
        for (int d = 0; d < JS_PD; ++d) {
            uint32_t v = cur[d * BLOCK + threadIdx.x];
            if ((int)threadIdx.x >= off) v = max(v, cur[d * BLOCK + threadIdx.x - off]);
            nxt[d * BLOCK + threadIdx.x] = v;
        }
        __syncthreads();
        uint32_t* tmp = cur; cur = nxt; nxt = tmp;
    }
    if (t < ntiles) {
#pragma unroll
        for (int d = 0; d < JS_PD; ++d) {
            const uint32_t ex = threadIdx.x ? cur[d * BLOCK + threadIdx.x - 1] : 0u;
            tagg[(size_t)t * JS_PD + d] = max(ex, gagg[(size_t)blockIdx.x * JS_PD + d]);
        }
    }
}

// tile-local token l of thread l / JS_PER lives at tpad(l): rows of JS_PER + 1 words, so the
// threads' sequential walks over their JS_PER tokens hit distinct LDS banks
KD_INLINE uint32_t tpad(uint32_t l) { return l + l / JS_PER; }
constexpr int JS_TPAD = JS_TILE + JS_TILE / JS_PER;

// inclusive max-scan over the wave by DPP moves (row shifts 1/2/4/8, then the row broadcasts of
// lanes 15 and 31): VALU data movement instead of six LDS-crossbar permutes per scan; the
// identity 0 fills lanes without a source
KD_INLINE uint32_t wave_incl_max(uint32_t v) {
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));   // row_shr:1
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));   // row_shr:2
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));   // row_shr:4
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));   // row_shr:8
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));   // row_bcast:15
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));   // row_bcast:31
    return v;
}

__global__ void __launch_bounds__(BLOCK) k_js_par_apply(const uint32_t* tmeta, uint32_t ntok, const uint32_t* texcl,
                                                        uint32_t* par, uint32_t* deep) {
    __shared__ uint32_t wt[BLOCK / 64][JS_PD];
    __shared__ uint32_t st[BLOCK * (JS_PD + 1)];
    __shared__ uint32_t tm[JS_TPAD];              // token metas in, parents out
    const uint32_t t0 = blockIdx.x * JS_TILE;
    for (int q = 0; q < JS_PER; ++q) {            // coalesced staging of the tile
        const uint32_t l = q * BLOCK + threadIdx.x;
        tm[tpad(l)] = t0 + l < ntok ? tmeta[t0 + l] : 0u;
    }
    uint32_t* row = st + threadIdx.x * (JS_PD + 1);
#pragma unroll
    for (int d = 0; d < JS_PD; ++d) row[d] = 0;
    __syncthreads();
    const uint32_t base = t0 + threadIdx.x * JS_PER;
    uint32_t* mine = tm + threadIdx.x * (JS_PER + 1);
    for (int k = 0; k < JS_PER; ++k) {
        const uint32_t i = base + k;
        if (i >= ntok) break;
        const uint32_t meta = mine[k];
        const uint32_t d = meta & TK_DEPTH_MASK;
        if (tk_open(meta) && d < JS_PD) row[d] = i + 1;
    }
    // exclusive max-scan of the rows over the workgroup: wave shuffles, then the earlier
    // waves' totals through LDS (no LDS ping-pong buffers, so more workgroups fit per CU)
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint32_t incl[JS_PD];
#pragma unroll
    for (int d = 0; d < JS_PD; ++d) {
        const uint32_t v = wave_incl_max(row[d]);
        incl[d] = v;
        if (lane == 63) wt[wave][d] = v;
    }
    __syncthreads();
#pragma unroll
    for (int d = 0; d < JS_PD; ++d) {
        uint32_t ex = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl[d], 0x138, 0xf, 0xf, false);   // wave_shr:1
        for (uint32_t w = 0; w < wave; ++w) ex = max(ex, wt[w][d]);
        row[d] = max(ex, texcl[(size_t)blockIdx.x * JS_PD + d]);
    }
    bool any_deep = false;
    for (int k = 0; k < JS_PER; ++k) {
        const uint32_t i = base + k;
        if (i >= ntok) break;
        const uint32_t meta = mine[k];
        const uint32_t d = meta & TK_DEPTH_MASK;
        uint32_t p = JS_NONE;
        if (d >= 1 && d <= JS_PD) p = row[d - 1] - 1;          // 0 - 1 = JS_NONE (malformed)
        else if (d > JS_PD) { p = JS_DEEP; any_deep = true; }
        mine[k] = p;
        if (tk_open(meta) && d < JS_PD) row[d] = i + 1;
    }
    if (__ballot(any_deep) && (threadIdx.x & 63u) == 0) atomicOr(deep, 1u);   // k_js_deep has work
    __syncthreads();
    for (int q = 0; q < JS_PER; ++q) {            // coalesced write-out
        const uint32_t l = q * BLOCK + threadIdx.x;
        if (t0 + l < ntok) par[t0 + l] = tm[tpad(l)];
    }
}

// tokens nested deeper than JS_PD: nearest earlier token with a smaller pre-depth. A small
// grid-stride launch that returns at once when k_js_par_apply met no such token (the usual
// document: reading every parent word for nothing cost a 2.4 GB pass)
__global__ void __launch_bounds__(BLOCK) k_js_deep(const uint32_t* tmeta, uint32_t ntok, uint32_t* par, const uint32_t* deep) {
    if (*deep == 0) return;
    for (uint32_t i = blockIdx.x * BLOCK + threadIdx.x; i < ntok; i += gridDim.x * BLOCK) {
        if (par[i] != JS_DEEP) continue;
        const uint32_t d = tmeta[i] & TK_DEPTH_MASK;
        uint32_t k = i;
        while (k > 0) {
            --k;
            if ((tmeta[k] & TK_DEPTH_MASK) < d) break;
        }
        par[i] = k;
    }
}

// ---------------------------------------------------------------- validation
KD_INLINE uint32_t tkind(uint32_t meta) { return (meta >> 24) & 0xFu; }
KD_INLINE uint32_t tsep(uint32_t meta) { return (meta >> 28) & 3u; }
KD_INLINE uint32_t tdepth(uint32_t meta) { return meta & TK_DEPTH_MASK; }
KD_INLINE bool value_start(uint32_t k) { return k == TK_OBJ || k == TK_ARR || k == TK_STR || k == TK_SCALAR; }

// closing quote of the string literal whose opening quote is at pos
KD_INLINE uint32_t str_end(const JsDoc& j, uint32_t pos) {
    uint32_t b = (pos + 1) >> 6;
    uint64_t w = j.qmask[b] & (~0ull << ((pos + 1) & 63));
    while (!w) w = j.qmask[++b];
    return b * 64 + (__ffsll((long long)w) - 1);
}
// any bit of mask[] in byte range [a, e)
KD_INLINE bool any_in(const uint64_t* mask, uint32_t a, uint32_t e) {
    if (a >= e) return false;
    if (e - a <= 64) {                                 // two words, no loop (masks have nb + 1 words)
        const uint32_t b = a >> 6, sh = a & 63u, L = e - a;
        uint64_t w = mask[b] >> sh;
        const uint64_t nx = mask[b + 1];
        w |= sh ? nx << (64 - sh) : 0ull;
        if (L < 64) w &= (1ull << L) - 1;
        return w != 0;
    }
    uint32_t b = a >> 6;
    const uint32_t be = (e - 1) >> 6;
    uint64_t w = mask[b] & (~0ull << (a & 63));
    for (;;) {
        if (b == be) {
            const uint32_t hi = e - b * 64;                        // 1..64
            if (hi < 64) w &= (1ull << hi) - 1;
            return w != 0;
        }
        if (w) return true;
        w = mask[++b];
    }
}
KD_INLINE bool valid_scalar(const JsDoc& j, uint32_t pos) {
    const uint8_t* s = j.doc;
    const uint32_t n = j.n;
    uint32_t i = pos;
    auto term = [&](uint32_t k) {
        if (k >= n) return true;
        const uint32_t c = s[k];
        return c <= 0x20 || c == '"' || is_struct_byte(c);
    };
    const uint32_t c0 = s[i];
    if (c0 == 't') return i + 4 <= n && s[i + 1] == 'r' && s[i + 2] == 'u' && s[i + 3] == 'e' && term(i + 4);
    if (c0 == 'f') return i + 5 <= n && s[i + 1] == 'a' && s[i + 2] == 'l' && s[i + 3] == 's' && s[i + 4] == 'e' && term(i + 5);
    if (c0 == 'n') return i + 4 <= n && s[i + 1] == 'u' && s[i + 2] == 'l' && s[i + 3] == 'l' && term(i + 4);
    if (i < n && s[i] == '-') ++i;
    if (i >= n || !is_digit(s[i])) return false;
    if (s[i] == '0') ++i;
    else while (i < n && is_digit(s[i])) ++i;
    if (i < n && s[i] == '.') {
        ++i;
        if (i >= n || !is_digit(s[i])) return false;
        while (i < n && is_digit(s[i])) ++i;
    }
    if (i < n && (s[i] == 'e' || s[i] == 'E')) {
        ++i;
        if (i < n && (s[i] == '+' || s[i] == '-')) ++i;
        if (i >= n || !is_digit(s[i])) return false;
        while (i < n && is_digit(s[i])) ++i;
    }
    return term(i);
}

// valid_scalar from one window of registers (load_window, below): the literal / number
// grammar as a byte DFA over the 32 bytes at pos. 1 = valid, 0 = invalid, -1 = the window
// holds no decision (a number longer than the window, or the window reaches past the
// document end) and the byte loop above decides.
KD_INLINE void load_window(const uint8_t* doc, uint32_t a, uint32_t u[8]);
KD_INLINE int valid_scalar_window(const JsDoc& j, uint32_t pos) {
    if (pos + 32 > j.n) return -1;
    uint32_t u[8];
    load_window(j.doc, pos, u);
    auto term = [](uint32_t c) { return c <= 0x20 || c == '"' || is_struct_byte(c); };
    const uint32_t c0 = u[0] & 0xFFu, b4 = u[1] & 0xFFu, b5 = (u[1] >> 8) & 0xFFu;
    if (c0 == 't') return u[0] == 0x65757274u && term(b4);            // "true"
    if (c0 == 'f') return u[0] == 0x736c6166u && b4 == 'e' && term(b5); // "fals" "e"
    if (c0 == 'n') return u[0] == 0x6c6c756eu && term(b4);            // "null"
    // Plain integers (the common scalar) from the window's digit mask: an optional '-', digits
    // without a leading zero, a terminator. Every lane of a wave holding one scalar ran the
    // byte DFA below; now only a fraction or an exponent ('.', 'e', 'E' after the digits) does.
    {
        const uint32_t st = c0 == '-' ? 1u : 0u;
        const uint32_t p = first_non_digit(digit_mask(u), st);
        if (p == st) return 0;                                          // no digit: not a number
        if (p >= 32u) return -1;                                        // longer than the window
        const uint32_t c = win_byte_at(u, p);
        if (c != '.' && (c | 32u) != 'e') {
            const bool lead0 = win_byte_at(u, st) == '0' && p > st + 1u;   // "0" then more digits
            return (!lead0 && term(c)) ? 1 : 0;
        }
    }
    // 0 start, 1 after '-', 2 leading 0, 3 integer digits, 4 after '.', 5 fraction digits,
    // 6 after e/E, 7 after the exponent sign, 8 exponent digits
    uint32_t st = 0;
    int res = -1;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
        const uint32_t c = (u[k >> 2] >> (8 * (k & 3))) & 0xFFu;
        if (res >= 0) continue;
        const bool dig = c - '0' < 10u, ee = (c | 32u) == 'e';
        switch (st) {
        case 0: st = c == '-' ? 1u : c == '0' ? 2u : dig ? 3u : 9u; break;
        case 1: st = c == '0' ? 2u : dig ? 3u : 9u; break;
        case 2: st = c == '.' ? 4u : ee ? 6u : 10u; break;
        case 3: st = dig ? 3u : c == '.' ? 4u : ee ? 6u : 10u; break;
        case 4: st = dig ? 5u : 9u; break;
        case 5: st = dig ? 5u : ee ? 6u : 10u; break;
        case 6: st = (c == '+' || c == '-') ? 7u : dig ? 8u : 9u; break;
        case 7: st = dig ? 8u : 9u; break;
        default: st = dig ? 8u : 10u; break;                            // 8
        }
        if (st == 9u) res = 0;                                          // grammar violated
        else if (st == 10u) res = term(c) ? 1 : 0;                      // the number ended at c
    }
    return res;
}

// The string token at pos: its closing quote e and whether a backslash (and, when hb is
// given, a byte >= 0x80) lies in (pos, e). The mask words of the opening block and the next
// one are loaded together, so a string ending within them costs one memory round trip
// (masks have nb + 1 words).
KD_INLINE uint32_t str_end_bs(const JsDoc& j, uint32_t pos, bool* bs, bool* hb = nullptr) {
    const uint32_t a = pos + 1, b = a >> 6, sh = a & 63u;
    const uint64_t q0 = j.qmask[b], q1 = j.qmask[b + 1], s0 = j.bsmask[b], s1 = j.bsmask[b + 1];
    uint64_t h0 = 0, h1 = 0;
    if (hb) { h0 = j.hbmask[b]; h1 = j.hbmask[b + 1]; }
    const uint64_t qa = q0 & (~0ull << sh);
    uint32_t e;
    if (qa) e = b * 64 + (__ffsll((long long)qa) - 1);
    else if (q1) e = (b + 1) * 64 + (__ffsll((long long)q1) - 1);
    else {
        e = str_end(j, pos);
        *bs = any_in(j.bsmask, a, e);
        if (hb) *hb = any_in(j.hbmask, a, e);
        return e;
    }
    // [a, e) lies within words b and b + 1 here (e - b * 64 <= 127)
    const uint32_t eb = e - b * 64;
    const uint64_t m0 = (~0ull << sh) & (eb >= 64 ? ~0ull : ((1ull << eb) - 1));
    const uint64_t m1 = eb > 64 ? ((1ull << (eb - 64)) - 1) : 0ull;
    *bs = ((s0 & m0) | (s1 & m1)) != 0;
    if (hb) *hb = ((h0 & m0) | (h1 & m1)) != 0;
    return e;
}

__global__ void __launch_bounds__(BLOCK) k_js_validate(JsDoc j, JsToks tk, uint32_t ntok, const uint32_t* par,
                                                       uint8_t* ecand, unsigned long long* err) {
    // the block's tokens (with the two before) and parents (with the one before) staged in
    // LDS with coalesced loads: a token's neighbours, and parents inside the block, come from
    // LDS instead of further global loads
    __shared__ uint32_t st[BLOCK + 2];
    __shared__ uint32_t sp[BLOCK + 1];
    const uint32_t b0 = blockIdx.x * BLOCK, i = b0 + threadIdx.x;
    if (i < ntok) {
        st[threadIdx.x + 2] = tk.meta[i];
        sp[threadIdx.x + 1] = par[i];
    }
    if (threadIdx.x < 2) {
        const uint32_t k = b0 + threadIdx.x;                      // token b0 - 2 + threadIdx.x
        st[threadIdx.x] = k >= 2 ? tk.meta[k - 2] : 0u;
        if (threadIdx.x == 1) sp[0] = b0 >= 1 ? par[b0 - 1] : JS_DEEP;
    }
    __syncthreads();
    if (i >= ntok) return;
    auto kind_of = [&](uint32_t q) {                              // tkind(tk.meta[q]), q < JS_DEEP
        return q + 2 >= b0 && q < b0 + BLOCK ? tkind(st[q + 2 - b0]) : tkind(tk.meta[q]);
    };
    const uint32_t t = st[threadIdx.x + 2];
    const uint32_t kind = tkind(t), d = tdepth(t);      // (the offset is read only where needed)
    const uint32_t p = sp[threadIdx.x + 1];
    const uint32_t pkind = p < JS_DEEP ? kind_of(p) : 0xFEu;
    const uint32_t ck = d == 0 ? 0xFFu : pkind;                   // container kind
    const uint32_t sep = tsep(t);                                 // the separator before the token
    const uint32_t pk = i ? tkind(st[threadIdx.x + 1]) : 0xFFu;
    bool ok;
    {
        // element candidate (see k_js_elems_count), from the staged neighbours, with its value's
        // class (1 object, 2 null, 3 anything else): k_js_elems_count then reads one byte per
        // token instead of the token stream, and the element's own token only for an error
        const bool cand = i != 0 && (d == 2 || d == 5) && (sep == SEP_COMMA || (sep == SEP_NONE && pk == TK_ARR)) &&
                          value_start(kind) && p < JS_DEEP && pkind == TK_ARR;
        ecand[i] = (uint8_t)(!cand ? 0u : kind == TK_OBJ ? 1u : (kind == TK_SCALAR && j.doc[tk.pos[i]] == 'n') ? 2u : 3u);
    }
    // The grammar over (previous token, separator, token): the rules the ',' / ':' tokens were
    // checked by are applied to the separator here, and the error lands where checkValid stops —
    // on the separator when it is out of place, else on the token. Admissible kinds are sets
    // (bit k = kind k), selected branch-free.
    bool sep_bad = false;
    {
        // token i - 1 is a member name: a string inside an object after '{' or ','
        const uint32_t tp = i ? st[threadIdx.x + 1] : 0u;
        const uint32_t ps = tsep(tp);
        const uint32_t ppk = i >= 2 ? tkind(st[threadIdx.x]) : 0xFFu;
        const bool key = pk == TK_STR && i >= 1 && p < JS_DEEP && pkind == TK_OBJ &&
                         (ps == SEP_COMMA || (ps == SEP_NONE && i >= 2 && ppk == TK_OBJ));
        constexpr uint32_t VS = 1u << TK_OBJ | 1u << TK_ARR | 1u << TK_STR | 1u << TK_SCALAR;   // a value
        uint32_t allow;
        if (sep != SEP_NONE) {
            // the separator in the predecessor's place: ':' only after a member name, ',' only
            // after a value, never at the top level or before the first token
            const bool after_value = !key && pk != TK_OBJ && pk != TK_ARR;
            sep_bad = i == 0 || d == 0 || (sep == SEP_COLON ? !key : !after_value);
            allow = sep == SEP_COLON ? VS : (ck == TK_OBJ ? 1u << TK_STR : ck == TK_ARR ? VS : 0u);
        } else {
            allow = pk == TK_OBJ ? (1u << TK_STR | 1u << TK_OBJ_END)
                  : pk == TK_ARR ? (VS | 1u << TK_ARR_END)
                  : key ? 0u                                       // a member name needs its ':'
                  : (1u << TK_OBJ_END | 1u << TK_ARR_END);         // after a value: ',' or a close
        }
        ok = (allow >> kind) & 1u;
        ok = ok && !(kind == TK_OBJ_END && ck != TK_OBJ) && !(kind == TK_ARR_END && ck != TK_ARR);
        ok = i == 0 ? (((VS >> kind) & 1u) && d == 0) : (ok && d != 0);   // d == 0: a second top-level value
    }
    if (sep_bad) {                                                // at the run's first separator
        const uint32_t pos = tk.pos[i];
        uint32_t q = pos, at = pos;
        while (q > 0) {
            const uint32_t c = j.doc[q - 1];
            if (is_ws(c)) { --q; continue; }
            if (c != ':' && c != ',') break;
            at = --q;
        }
        js_fail(err, at, KDTN_JSON_SYNTAX);
        return;
    }
    // (a scalar's own grammar is checked by k_js_scalars over the compacted list of scalar
    // tokens: here, one scalar in a wave of 64 tokens made the whole wave run its check)
    // (a string's escapes are checked by k_js_classify, per escaped byte of the block masks)
    if (!ok) js_fail(err, tk.pos[i], KDTN_JSON_SYNTAX);
}

// The end of the document, one thread: separators after the last token are checked as the
// ',' / ':' tokens were (their place after the last token, then a second one); with none, the
// last token must end the top-level value. A document that ends inside a value fails at its
// end, as checkValid's "unexpected end of JSON input" does.
__global__ void k_js_tail(JsDoc j, JsToks tk, uint32_t ntok, const uint32_t* par, unsigned long long* err) {
    if (threadIdx.x != 0 || ntok == 0) return;
    const uint32_t t = tk.meta[ntok - 1];
    const uint32_t kind = tkind(t), d = tdepth(t), pos = tk.pos[ntok - 1];
    uint32_t e = pos + 1;                                     // the last token's end
    if (kind == TK_STR) {
        e = str_end(j, pos) + 1;
    } else if (kind == TK_SCALAR) {
        while (e < j.n) {
            const uint32_t c = j.doc[e];
            if (c <= 0x20 || c == '"' || is_struct_byte(c)) break;
            ++e;
        }
    }
    uint32_t q = e;
    while (q < j.n && is_ws(j.doc[q])) ++q;
    if (q >= j.n) {                                           // the document ends with the token
        const bool ok = (kind == TK_STR || kind == TK_SCALAR) ? d == 0
                                                              : ((kind == TK_OBJ_END || kind == TK_ARR_END) && d == 1);
        if (!ok) js_fail(err, j.n, KDTN_JSON_SYNTAX);
        return;
    }
    const uint32_t c = j.doc[q];                              // a separator: nothing else is left
    const uint32_t p = par[ntok - 1];
    const bool in_obj = p < JS_DEEP && tkind(tk.meta[p]) == TK_OBJ;
    const uint32_t ps = tsep(t);
    const bool key = kind == TK_STR && in_obj &&
                     (ps == SEP_COMMA || (ps == SEP_NONE && ntok >= 2 && tkind(tk.meta[ntok - 2]) == TK_OBJ));
    const int64_t ds = (int64_t)d + ((kind == TK_OBJ || kind == TK_ARR) ? 1 : (kind == TK_OBJ_END || kind == TK_ARR_END) ? -1 : 0);
    const bool ok = ds != 0 && (c == ':' ? key : (!key && kind != TK_OBJ && kind != TK_ARR));
    if (!ok) {
        js_fail(err, q, KDTN_JSON_SYNTAX);
        return;
    }
    uint32_t q2 = q + 1;
    while (q2 < j.n && is_ws(j.doc[q2])) ++q2;
    js_fail(err, q2 < j.n ? q2 : j.n, KDTN_JSON_SYNTAX);
}

// checkValid's literal / number grammar for every scalar token, over the list k_js_tokens
// compacted (full waves of scalars instead of one scalar lane per token wave)
__global__ void __launch_bounds__(BLOCK) k_js_scalars(JsDoc j, const uint32_t* tpos, const uint32_t* slist, uint32_t nscal,
                                                      unsigned long long* err) {
    const uint32_t k = blockIdx.x * BLOCK + threadIdx.x;
    if (k >= nscal || (KDTN_PROFILING && (j.variant & JSV_NO_SCALAR))) return;
    const uint32_t pos = tpos[slist[k]];
    const int w = valid_scalar_window(j, pos);
    if (!(w >= 0 ? w != 0 : valid_scalar(j, pos))) js_fail(err, pos, KDTN_JSON_SYNTAX);
}

// ---------------------------------------------------------------- key matching
// Decodes the member name at string token pos (escapes included) into two little-endian
// words; ok = false when it cannot equal a schema name (names are ASCII, at most 15 bytes).
struct KeyName { uint64_t lo, hi; bool ok; };
// bit k (k < 4): byte k of w is c
KD_INLINE uint32_t eq4(uint32_t w, uint32_t c) { return mm4(eqb(w, c)); }
KD_INLINE KeyName key_name(const JsDoc& j, uint32_t pos, bool fast = true) {
    uint64_t lo = 0, hi = 0;
    uint32_t len = 0;
    // the three aligned words a plain name needs are loaded with the mask words (one round trip)
    const uint64_t* w = reinterpret_cast<const uint64_t*>(j.doc + ((pos + 1) & ~7u));
    const uint64_t w0 = w[0], w1 = w[1], w2 = w[2];
    if (fast) {
        // the name's first 17 bytes from those words: its closing quote and any backslash before
        // it found by SWAR, so a plain name needs no mask words (no escape before the first quote
        // means that quote ends the string; no quote in 17 bytes and no backslash means a name
        // of 17+ bytes, which no schema name is)
        const uint32_t sh = ((pos + 1) & 7u) * 8;
        const uint64_t l = sh ? (w0 >> sh) | (w1 << (64 - sh)) : w0;
        const uint64_t h = sh ? (w1 >> sh) | (w2 << (64 - sh)) : w1;
        const uint32_t b16 = (uint32_t)((sh ? (w2 >> sh) : w2) & 0xFFu);
        const uint32_t x[4] = {(uint32_t)l, (uint32_t)(l >> 32), (uint32_t)h, (uint32_t)(h >> 32)};
        uint32_t Q = (b16 == '"') ? 1u << 16 : 0u, B = (b16 == '\\') ? 1u << 16 : 0u;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            Q |= eq4(x[k], '"') << (4 * k);
            B |= eq4(x[k], '\\') << (4 * k);
        }
        const uint32_t L = Q ? (uint32_t)__builtin_ctz(Q) : 17u;
        if (!(B & ((1u << L) - 1u))) {                        // no escape before the end (or window)
            if (L > 15u) return {0, 0, false};
            uint64_t a = l, b = h;
            if (L < 8) { a &= (1ull << (8 * L)) - 1; b = 0; }
            else b &= L == 8 ? 0ull : (1ull << (8 * (L - 8))) - 1;
            return {a, b, true};
        }
    }
    bool bs;
    const uint32_t e = str_end_bs(j, pos, &bs);
    if (e - pos - 1 > 6 * 16) return {0, 0, false};
    if (e - pos - 1 <= 15 && !bs) {                               // plain name: three aligned words
        const uint32_t a = pos + 1, L = e - a;
        const uint32_t sh = (a & 7u) * 8;
        lo = sh ? (w0 >> sh) | (w1 << (64 - sh)) : w0;
        hi = sh ? (w1 >> sh) | (w2 << (64 - sh)) : w1;
        if (L < 8) { lo &= (1ull << (8 * L)) - 1; hi = 0; }
        else hi &= L == 8 ? 0ull : (1ull << (8 * (L - 8))) - 1;
        return {lo, hi, true};
    }
    for (uint32_t k = pos + 1; k < e; ++k) {
        uint32_t c = j.doc[k];
        if (c == '\\') {
            const uint32_t x = j.doc[k + 1];
            if (x == 'u') {
                uint32_t r = 0;
                for (int q = 2; q < 6; ++q) {
                    const uint32_t h = j.doc[k + q];
                    r = r * 16 + (h <= '9' ? h - '0' : (h | 32) - 'a' + 10);
                }
                if (r >= 0x80) return {0, 0, false};
                c = r;
                k += 5;
            } else {
                c = esc_byte(x);
                k += 1;
            }
        } else if (c >= 0x80) {
            return {0, 0, false};
        }
        if (len >= 15 || c == 0) return {0, 0, false};
        if (len < 8) lo |= (uint64_t)c << (8 * len);
        else hi |= (uint64_t)c << (8 * (len - 8));
        ++len;
    }
    return {lo, hi, true};
}
// index of the decoded name in names[0..n) (distinct), or -1
KD_INLINE int key_match(const KeyName& k, const char (*names)[16], int n) {
    int hit = -1;
    for (int f = 0; f < n; ++f) {
        const uint64_t* nm = reinterpret_cast<const uint64_t*>(names[f]);
        hit = (k.ok && nm[0] == k.lo && nm[1] == k.hi) ? f : hit;
    }
    return hit;
}
KD_INLINE int match_key(const JsDoc& j, uint32_t pos, const char (*names)[16], int n) {
    return key_match(key_name(j, pos), names, n);
}

__constant__ __attribute__((aligned(16))) char kItems[1][16] = {"items"};
__constant__ __attribute__((aligned(16))) char kItem[3][16] = {"metadata", "spec", "status"};
__constant__ __attribute__((aligned(16))) char kMeta[2][16] = {"name", "namespace"};
__constant__ __attribute__((aligned(16))) char kLinks[1][16] = {"links"};
__constant__ __attribute__((aligned(16))) char kStatus[3][16] = {"links", "src_ip", "net_ns"};
__constant__ __attribute__((aligned(16))) char kLink[KDTN_NKEY + 2][16] = {"local_intf", "local_ip", "local_mac", "peer_intf", "peer_ip",
                                              "peer_mac", "peer_pod", "uid", "properties"};
__constant__ __attribute__((aligned(16))) char kProps[KDTN_NPROP + 1][16] = {"latency", "latency_corr", "jitter", "loss", "loss_corr", "rate",
                                                "duplicate", "duplicate_corr", "reorder_prob", "reorder_corr",
                                                "corrupt_prob", "corrupt_corr", "gap"};

// all schema member names, each role's list contiguous (k_js_values): root | item | metadata |
// spec / status (spec uses "links" only) | link | properties
constexpr int KA_ROOT = 0, KA_ITEM = 1, KA_META = 4, KA_LINKS = 6, KA_LINK = 9, KA_PROPS = 18,
              KN_ALL = KA_PROPS + KDTN_NPROP + 1;
__constant__ __attribute__((aligned(16))) char kAll[KN_ALL][16] = {
    "items", "metadata", "spec", "status", "name", "namespace", "links", "src_ip", "net_ns",
    "local_intf", "local_ip", "local_mac", "peer_intf", "peer_ip", "peer_mac", "peer_pod", "uid", "properties",
    "latency", "latency_corr", "jitter", "loss", "loss_corr", "rate", "duplicate", "duplicate_corr",
    "reorder_prob", "reorder_corr", "corrupt_prob", "corrupt_corr", "gap"};
static_assert(KN_ALL == 31, "schema names");
// 7-bit hash of a name's zero-padded 16 bytes, distinct over kAll (multiplier found by search;
// tests/test_ingest_cpu.py checks the property)
KD_INLINE uint32_t name_hash(uint64_t lo, uint64_t hi) {
    return (uint32_t)(((lo ^ (hi * 0x9E3779B97F4A7C15ull)) * 0x1BA1621582283D15ull) >> 57);
}

// ---------------------------------------------------------------- roles
// role of the container c whose enclosing container has role r (c is the child token)
KD_INLINE uint32_t child_role(const JsDoc& j, const JsToks& tk, uint32_t r, uint32_t c) {
    if (r == R_NONE || r == R_META || r >= R_PROPS_S) return R_NONE;
    const uint32_t meta = tk.meta[c];
    const uint32_t kind = tkind(meta);
    const bool member = tsep(meta) == SEP_COLON;
    if (!member) {                                                // array element
        if (kind != TK_OBJ) return R_NONE;
        return r == R_ITEMS ? R_ITEM : r == R_SPEC_LINKS ? R_LINK_S : r == R_STATUS_LINKS ? R_LINK_R : R_NONE;
    }
    const uint32_t kpos = tk.pos[c - 1];
    switch (r) {
    case R_ROOT:
        return (kind == TK_ARR && match_key(j, kpos, kItems, 1) == 0) ? R_ITEMS : R_NONE;
    case R_ITEM: {
        if (kind != TK_OBJ) return R_NONE;
        const int f = match_key(j, kpos, kItem, 3);
        return f == 0 ? R_META : f == 1 ? R_SPEC : f == 2 ? R_STATUS : R_NONE;
    }
    case R_SPEC:
        return (kind == TK_ARR && match_key(j, kpos, kLinks, 1) == 0) ? R_SPEC_LINKS : R_NONE;
    case R_STATUS:
        return (kind == TK_ARR && match_key(j, kpos, kLinks, 1) == 0) ? R_STATUS_LINKS : R_NONE;
    case R_LINK_S:
    case R_LINK_R: {                                  // only "properties" opens a container here
        if (kind != TK_OBJ) return R_NONE;
        const KeyName k = key_name(j, kpos);
        const uint64_t* nm = reinterpret_cast<const uint64_t*>(kLink[KDTN_NKEY + 1]);
        return (k.ok && k.lo == nm[0] && k.hi == nm[1]) ? (r == R_LINK_S ? R_PROPS_S : R_PROPS_R) : R_NONE;
    }
    default:
        return R_NONE;
    }
}

// one nesting level at a time over the open brackets (levels 0, 1, 3, 4, then 6): a container's
// role follows from its parent's (set by an earlier level), its kind and its member name. The
// array elements of levels 2 and 5 are set by k_js_elems_count, which classifies them anyway
// (level 6 runs after it); level 3 therefore derives its parent's role (an items element)
// from the grandparent's. The roles start zeroed (R_NONE) and only the schema's containers
// are written.
__global__ void __launch_bounds__(BLOCK) k_js_roles(JsDoc j, JsToks tk, const uint32_t* olist, uint32_t nopen,
                                                    const uint32_t* par, uint8_t* role, const uint8_t* odep,
                                                    uint32_t level) {
    const uint32_t k = blockIdx.x * BLOCK + threadIdx.x;
    if (k >= nopen || odep[k] != level) return;             // the depth byte k_js_tokens wrote
    const uint32_t i = olist[k];
    uint32_t r;
    if (level == 0) {
        r = tkind(tk.meta[i]) == TK_OBJ ? R_ROOT : R_NONE;
    } else {
        const uint32_t p = par[i];
        uint32_t rp;
        if (level == 3)                                      // p: an items element (an object) or nothing
            rp = (role[par[p]] == R_ITEMS && tkind(tk.meta[p]) == TK_OBJ) ? R_ITEM : R_NONE;
        else
            rp = role[p];
        r = child_role(j, tk, rp, i);
    }
    if (r != R_NONE) role[i] = (uint8_t)r;
}

// ---------------------------------------------------------------- element ordinals
// Element class of token i: 1 + {0 items element, 1 spec.links element, 2 status.links
// element}, or 0. k_js_validate marks the candidates (depth 2 for items elements, 5 for links
// elements; after '[' or ','; a value; parent an array); the parent array's role decides.
__global__ void __launch_bounds__(BLOCK) k_js_elems_count(JsDoc j, JsToks tk, uint32_t ntok, const uint32_t* par,
                                                          uint8_t* role, uint32_t* cnt3, uint8_t* ecls,
                                                          unsigned long long* derr) {
    __shared__ uint32_t sh[3];
    if (threadIdx.x < 3) sh[threadIdx.x] = 0;
    __syncthreads();
    uint32_t c[3] = {0, 0, 0};
    const uint32_t t0 = blockIdx.x * JS_TILE;
    if (t0 + threadIdx.x == 0 && ntok) {                          // the document must be an object or null
        const uint32_t t = tk.meta[0], p0 = tk.pos[0];
        if (!(tkind(t) == TK_OBJ || (tkind(t) == TK_SCALAR && j.doc[p0] == 'n'))) js_fail(derr, p0, KDTN_JSON_TYPE);
    }
    // counts: the thread's 16 candidate bytes (JS_PER == 16) as one coalesced 16-byte load;
    // the buffer is padded to whole tiles, bytes past ntok are ignored
    static_assert(JS_PER == 16, "one uint4 of candidate bytes per thread");
    const uint32_t base = t0 + threadIdx.x * JS_PER;
    uint4* cp = reinterpret_cast<uint4*>(ecls + base);
    uint4 cv = *cp;
    uint32_t w[4] = {cv.x, cv.y, cv.z, cv.w};
    bool changed = false;
    // the candidates' parents, then their roles, each as one batch of loads (in one loop with
    // the role stores below, every candidate waited for the one before it)
    uint32_t rr[JS_PER];
#pragma unroll
    for (int k = 0; k < JS_PER; ++k) {
        const uint32_t vc = (w[k >> 2] >> (8 * (k & 3))) & 0xFFu;
        rr[k] = (vc && base + k < ntok) ? par[base + k] : JS_NONE;
    }
#pragma unroll
    for (int k = 0; k < JS_PER; ++k) rr[k] = rr[k] < JS_DEEP ? (uint32_t)role[rr[k]] : (uint32_t)R_NONE;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if (!w[q]) continue;
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            const uint32_t i = base + q * 4 + h;
            const uint32_t vc = (w[q] >> (8 * h)) & 0xFFu;             // k_js_validate's value class
            if (i >= ntok || !vc) continue;
            changed = true;
            const uint32_t r = rr[q * 4 + h];
            const uint32_t cls = r == R_ITEMS ? 1 : r == R_SPEC_LINKS ? 2 : r == R_STATUS_LINKS ? 3 : 0;
            w[q] = (w[q] & ~(0xFFu << (8 * h))) | (cls << (8 * h));   // the class, for k_js_elems_write
            if (!cls) continue;
            if (vc == 3u) js_fail(derr, tk.pos[i], KDTN_JSON_TYPE);     // neither an object nor null
            if (vc == 1u) role[i] = (uint8_t)(cls == 1 ? R_ITEM : cls == 2 ? R_LINK_S : R_LINK_R);
            c[cls - 1]++;
        }
    }
    if (changed) *cp = make_uint4(w[0], w[1], w[2], w[3]);
#pragma unroll
    for (int q = 0; q < 3; ++q)
        if (c[q]) atomicAdd(&sh[q], c[q]);
    __syncthreads();
    if (threadIdx.x < 3) cnt3[(size_t)threadIdx.x * gridDim.x + blockIdx.x] = sh[threadIdx.x];
}

__global__ void __launch_bounds__(BLOCK) k_js_elems_write(const uint8_t* ecls, uint32_t ntok, const uint64_t* coff3,
                                                          uint32_t ntiles, uint32_t* ord, JsTopoOut to) {
    __shared__ uint64_t sh[BLOCK / 64];
    // the thread's JS_PER classes as one 16-byte load (whole tiles; bytes past ntok ignored)
    const uint32_t base = blockIdx.x * JS_TILE + threadIdx.x * JS_PER;
    const uint4 cv = *reinterpret_cast<const uint4*>(ecls + base);
    const uint32_t w[4] = {cv.x, cv.y, cv.z, cv.w};
    uint32_t c[3] = {0, 0, 0};
    const bool any = (cv.x | cv.y | cv.z | cv.w) != 0;
    if (any) {
#pragma unroll
        for (int k = 0; k < JS_PER; ++k) {
            const uint32_t cls = (w[k >> 2] >> (8 * (k & 3))) & 0xFFu;
            if (cls && base + k < ntok) c[cls - 1]++;
        }
    }
    uint32_t run[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        uint64_t tot;
        run[q] = (uint32_t)(coff3[(size_t)q * (ntiles + 1) + blockIdx.x] + block_exclusive(c[q], sh, &tot));
    }
    if (!any) return;
    for (int k = 0; k < JS_PER; ++k) {
        const uint32_t i = base + k;
        const uint32_t cls = (w[k >> 2] >> (8 * (k & 3))) & 0xFFu;
        if (!cls || i >= ntok) continue;
        const uint32_t o = run[cls - 1]++;
        ord[i] = o;
        if (cls == 1) {                                            // a Topology: its record offsets
            to.des_off[o] = run[1];
            to.real_off[o] = run[2];
        }
    }
}

// ---------------------------------------------------------------- schema values
KD_INLINE uint64_t fnv_step(uint64_t h, uint32_t c) { return (h ^ c) * 1099511628211ull; }

// The 32 document bytes starting at byte a, as 8 words aligned to a: nine aligned dword
// loads issued together (the document has >= 128 bytes of padding), so a short string costs
// one memory round trip instead of one per byte.
constexpr uint32_t WIN = 32;
KD_INLINE void load_window(const uint8_t* doc, uint32_t a, uint32_t u[8]) {
    const uint32_t* p = reinterpret_cast<const uint32_t*>(doc + (a & ~3u));
    uint32_t w[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) w[k] = p[k];
    const uint32_t sh = a & 3u;
#pragma unroll
    for (int k = 0; k < 8; ++k) u[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
}
KD_INLINE uint32_t win_byte(const uint32_t u[8], int k) { return (u[k >> 2] >> (8 * (k & 3))) & 0xFFu; }
// Hash of a string of len (<= WIN) bytes held in a window: one 64-bit FNV-style step per
// 4-byte word (bytes past len masked off, len folded into the seed). Every string of at most
// WIN bytes is hashed this way, from the document or the decode heap alike, and longer
// strings by the byte loop, so equal strings always hash equally. Words past the longest
// string of the wave are skipped (wave-uniform test), the rest predicated without branches.
KD_INLINE uint64_t word_hash(const uint32_t u[8], uint32_t len) {
    uint64_t h = 1469598103934665603ull ^ len;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t lo = 4u * k;
        if (__ballot(lo < len)) {
            const uint32_t m = len >= lo + 4 ? 0xFFFFFFFFu : len <= lo ? 0u : (1u << (8 * (len - lo))) - 1u;
            const uint64_t hn = fnv_step(h, u[k] & m);
            h = lo < len ? hn : h;
        }
    }
    return h;
}
// first len (<= WIN) bytes of two windows equal
KD_INLINE bool window_eq(const uint32_t a[8], const uint32_t b[8], uint32_t len) {
    bool eq = true;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t lo = 4u * k;
        const uint32_t m = len >= lo + 4 ? 0xFFFFFFFFu : len <= lo ? 0u : (1u << (8 * (len - lo))) - 1u;
        eq &= ((a[k] ^ b[k]) & m) == 0;
    }
    return eq;
}

// utf8.DecodeRune length of a valid sequence at s (bounded by e), 0 = invalid
KD_INLINE uint32_t utf8_len(const uint8_t* s, const uint8_t* e) {
    const uint32_t c = s[0];
    uint32_t need, lo = 0x80, hi = 0xBF;
    if (c >= 0xC2 && c <= 0xDF) need = 1;
    else if (c == 0xE0) { need = 2; lo = 0xA0; }
    else if (c >= 0xE1 && c <= 0xEC) need = 2;
    else if (c == 0xED) { need = 2; hi = 0x9F; }
    else if (c >= 0xEE && c <= 0xEF) need = 2;
    else if (c == 0xF0) { need = 3; lo = 0x90; }
    else if (c >= 0xF1 && c <= 0xF3) need = 3;
    else if (c == 0xF4) { need = 3; hi = 0x8F; }
    else return 0;
    if ((uint32_t)(e - s) < need + 1) return 0;
    if (s[1] < lo || s[1] > hi) return 0;
    for (uint32_t k = 2; k <= need; ++k)
        if (s[k] < 0x80 || s[k] > 0xBF) return 0;
    return need + 1;
}
KD_INLINE int hex4(const uint8_t* p, const uint8_t* e) {         // getu4
    if (e - p < 6 || p[0] != '\\' || p[1] != 'u') return -1;
    int r = 0;
    for (int k = 2; k < 6; ++k) {
        const uint32_t h = p[k];
        if (!is_hexc(h)) return -1;
        r = r * 16 + (int)(h <= '9' ? h - '0' : (h | 32) - 'a' + 10);
    }
    return r;
}
KD_INLINE uint32_t rune_len(uint32_t r) { return r < 0x80 ? 1 : r < 0x800 ? 2 : r < 0x10000 ? 3 : 4; }
KD_INLINE uint32_t put_rune(uint8_t* o, uint32_t r) {
    if (r < 0x80) { o[0] = (uint8_t)r; return 1; }
    if (r < 0x800) { o[0] = (uint8_t)(0xC0 | (r >> 6)); o[1] = (uint8_t)(0x80 | (r & 63)); return 2; }
    if (r < 0x10000) {
        o[0] = (uint8_t)(0xE0 | (r >> 12)); o[1] = (uint8_t)(0x80 | ((r >> 6) & 63)); o[2] = (uint8_t)(0x80 | (r & 63));
        return 3;
    }
    o[0] = (uint8_t)(0xF0 | (r >> 18)); o[1] = (uint8_t)(0x80 | ((r >> 12) & 63));
    o[2] = (uint8_t)(0x80 | ((r >> 6) & 63)); o[3] = (uint8_t)(0x80 | (r & 63));
    return 4;
}
// \uXXXX at d[r] (with a following low surrogate when it pairs): the rune, r advanced past it;
// lone or unpaired surrogates become U+FFFD (utf16.DecodeRune, encoding/json unquote)
KD_INLINE uint32_t u_escape(const uint8_t* d, uint32_t& r, uint32_t e) {
    int rr = hex4(d + r, d + e);
    r += 6;
    if (rr >= 0xD800 && rr < 0xE000) {
        const int r1 = hex4(d + r, d + e);
        if (rr < 0xDC00 && r1 >= 0xDC00 && r1 < 0xE000) {
            r += 6;
            return (uint32_t)((((rr - 0xD800) << 10) | (r1 - 0xDC00)) + 0x10000);
        }
        return 0xFFFDu;
    }
    return (uint32_t)rr;
}
// encoding/json unquote of the literal content d[a, e): decoded length (pass 1) and bytes
// (pass 2). Invalid UTF-8 bytes become U+FFFD (3 bytes each).
KD_INLINE uint32_t unquote_len(const uint8_t* d, uint32_t a, uint32_t e) {
    uint32_t w = 0, r = a;
    while (r < e) {
        const uint32_t c = d[r];
        if (c == '\\') {
            if (d[r + 1] == 'u') w += rune_len(u_escape(d, r, e));
            else { w += 1; r += 2; }
        } else if (c < 0x80) {
            w += 1;
            r += 1;
        } else {
            const uint32_t k = utf8_len(d + r, d + e);
            w += k ? k : 3u;
            r += k ? k : 1u;
        }
    }
    return w;
}
KD_INLINE void unquote_write(const uint8_t* d, uint32_t a, uint32_t e, uint8_t* out) {
    uint32_t w = 0, r = a;
    while (r < e) {
        const uint32_t c = d[r];
        if (c == '\\') {
            if (d[r + 1] == 'u') w += put_rune(out + w, u_escape(d, r, e));
            else { out[w++] = (uint8_t)esc_byte(d[r + 1]); r += 2; }
        } else if (c < 0x80) {
            out[w++] = (uint8_t)c;
            r += 1;
        } else {
            const uint32_t k = utf8_len(d + r, d + e);
            if (k) {
                for (uint32_t q = 0; q < k; ++q) out[w + q] = d[r + q];
                w += k;
                r += k;
            } else {
                w += put_rune(out + w, 0xFFFDu);
                r += 1;
            }
        }
    }
}

// intern table key word: [63:57] hash tag | [56] heap | [55:32] length | [31:0] offset
KD_INLINE const uint8_t* key_bytes(const JsIntern& in, uint64_t kw) {
    return ((kw >> 56) & 1 ? in.heap : in.doc) + (uint32_t)kw;
}

// a zero byte among the first len (<= JS_INL) bytes of w: inline bytes not (yet) available
KD_INLINE bool inline_has_zero(const uint32_t w[6], uint32_t len) {
    bool z = false;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const uint32_t lo = 4u * k;
        const uint32_t m = len >= lo + 4 ? 0xFFFFFFFFu : len <= lo ? 0u : (1u << (8 * (len - lo))) - 1u;
        z |= (((w[k] - 0x01010101u) & ~w[k] & 0x80808080u) & (m & 0x80808080u)) != 0;
    }
    return z;
}

// returns the table slot of the string [p, p+len) (len ≥ 1), or JS_NONE on overflow
KD_INLINE uint32_t intern(const JsIntern& in, const JsDict& dt, const uint8_t* p, uint32_t len, uint64_t kw_self,
                          uint64_t h, uint32_t occ, const uint32_t (&pw)[8], bool have_pw) {
    const uint64_t tag = h >> 57;
    const uint64_t kw = (tag << 57) | kw_self;
    bool inl = have_pw && len <= JS_INL;
    if constexpr (KDTN_PROFILING != 0) {
        const uint32_t off = in.variant & (JSV_NO_INLINE | (dt.slots == in.kd.slots ? JSV_NO_INLINE_K : JSV_NO_INLINE_P));
        if (off) inl = false;
    }
    uint32_t s = (uint32_t)h & dt.mask;
    const uint32_t probes = dt.mask < JS_MAX_PROBE ? dt.mask + 1 : JS_MAX_PROBE;   // a run this long: grow the table
    for (uint32_t probe = 0; probe < probes; ++probe) {
        // slots are written once (CAS from 0): a plain load is either that final key or a stale 0,
        // and a stale 0 only sends us to the CAS, which returns the real key. The key word and
        // the inline bytes come from one 32-byte slot (two 16-B loads of one line).
        const uint4 q0 = *reinterpret_cast<const uint4*>(dt.slots + s);
        const uint4 q1 = *reinterpret_cast<const uint4*>(&dt.slots[s].b[2]);
        unsigned long long cur = (KDTN_PROFILING && (in.variant & JSV_COHERENT))
                                     ? __hip_atomic_load(&dt.slots[s].kw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                     : ((unsigned long long)q0.y << 32) | q0.x;
        if (cur == 0) {
            if ((kw >> 56) & 1) __threadfence();       // heap bytes visible before the key
            cur = atomicCAS(&dt.slots[s].kw, 0ull, (unsigned long long)kw);
            if (cur == 0) {
                atomicMin(dt.rep + s, occ);
                dt.keys[s] = kw;
                if (inl && !inline_has_zero(pw, len)) {   // bytes past len stored as they are (ignored)
                    *reinterpret_cast<uint2*>(&dt.slots[s].b[0]) = make_uint2(pw[0], pw[1]);
                    *reinterpret_cast<uint4*>(&dt.slots[s].b[2]) = make_uint4(pw[2], pw[3], pw[4], pw[5]);
                }
                return s;
            }
        }
        if ((cur >> 57) == tag && ((cur >> 32) & 0xFFFFFFu) == len) {
            uint32_t k = 0;
            const uint32_t ib[8] = {q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, 0u, 0u};
            if (inl && !((cur >> 56) & 1) && !inline_has_zero(ib, len)) {
                // the inserter's bytes, final (a string with a zero byte is never stored inline,
                // a word not yet stored reads as zero): they decide equality
                k = window_eq(pw, ib, len) ? len : 0u;
            } else if ((cur >> 56) & 1) {             // heap bytes of another thread: coherent loads
                const uint32_t off = (uint32_t)cur;
                while (k < len) {
                    const uint32_t wd = __hip_atomic_load(reinterpret_cast<const uint32_t*>(in.heap) + ((off + k) >> 2),
                                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (((wd >> (8 * ((off + k) & 3))) & 0xFFu) != p[k]) break;
                    ++k;
                }
            } else if (have_pw && len <= WIN) {       // both in the document: compare windows
                uint32_t qw[8];
                load_window(in.doc, (uint32_t)cur, qw);
                k = window_eq(pw, qw, len) ? len : 0u;
            } else {
                const uint8_t* q = in.doc + (uint32_t)cur;
                while (k < len && q[k] == p[k]) ++k;
            }
            if (k == len) {                           // hot strings: skip the atomic when it cannot lower
                // an occurrence later in the document than the one that inserted the key cannot
                // lower the first occurrence (the inserter's own atomicMin is <= its index, and
                // document offsets grow with token indices): no rep read, no atomic
                const bool later = !((kw_self >> 56) & 1) && !((cur >> 56) & 1) && (uint32_t)kw_self > (uint32_t)cur;
                if (!later && !(KDTN_PROFILING && (in.variant & JSV_NO_REP)) && occ < dt.rep[s])
                    atomicMin(dt.rep + s, occ);
                return s;
            }
        }
        s = (s + 1) & dt.mask;
    }
    atomicOr(in.status, JS_ST_OVERFLOW);
    return JS_NONE;
}

// string value at token i → 1 + table slot (0 = empty string); JS_NONE on overflow
KD_INLINE uint32_t string_slot(const JsDoc& j, const JsIntern& in, const JsDict& dt, uint32_t i, uint32_t pos) {
    const uint32_t a = pos + 1;
    uint32_t pw[8];
    load_window(j.doc, a, pw);
    bool bs = false, hb = false;
    uint32_t e = 0;
    bool found = false;
    if (!(KDTN_PROFILING && (in.variant & JSV_MASKS))) {
        // a string that ends within the window: its closing quote, escapes and high bytes from
        // the window itself (SWAR), no mask words (the first quote with no backslash before it
        // is the end: a quote inside a string is always escaped)
        uint32_t Q = 0, B = 0, H = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            Q |= mm4(eqb(pw[k], '"')) << (4 * k);
            B |= mm4(eqb(pw[k], '\\')) << (4 * k);
            H |= mm4(pw[k] & 0x80808080u) << (4 * k);
        }
        if (Q) {
            const uint32_t L = (uint32_t)__builtin_ctz(Q), below = (1u << L) - 1u;   // L < 32
            if (!(B & below)) {
                e = a + L;
                hb = (H & below) != 0;
                found = true;
            }
        }
    }
    if (!found) e = str_end_bs(j, pos, &bs, &hb);
    if (e == a) return 0;
    if (!bs && !hb) {                                  // plain ASCII: the bytes themselves
        const uint32_t len = e - a;
        if (len > 0xFFFFFFu) { atomicOr(in.status, JS_ST_LONG); return JS_NONE; }
        uint64_t h;
        const bool win = len <= WIN;
        if (win) {
            h = word_hash(pw, len);
        } else {
            h = 1469598103934665603ull;
            for (uint32_t k = a; k < e; ++k) h = fnv_step(h, j.doc[k]);
        }
        h ^= h >> 29;
        const uint32_t s = intern(in, dt, j.doc + a, len, ((uint64_t)len << 32) | a, h, i, pw, win);
        return s == JS_NONE ? JS_NONE : s + 1;
    }
    const uint32_t len = unquote_len(j.doc, a, e);
    if (len == 0) return 0;
    if (len > 0xFFFFFFu) { atomicOr(in.status, JS_ST_LONG); return JS_NONE; }
    const unsigned long long at = atomicAdd(in.heap_used, (unsigned long long)((len + 3) & ~3u));
    if (at + len > in.heap_cap) { atomicOr(in.status, JS_ST_OVERFLOW); return JS_NONE; }
    uint8_t* out = in.heap + at;
    unquote_write(j.doc, a, e, out);
    uint64_t h = 1469598103934665603ull;
    if (len <= WIN) {                                  // the heap has 64 B of slack past heap_cap
        uint32_t hw[8];
        load_window(in.heap, (uint32_t)at, hw);
        h = word_hash(hw, len);
    } else {
        for (uint32_t k = 0; k < len; ++k) h = fnv_step(h, out[k]);
    }
    h ^= h >> 29;
    const uint32_t s = intern(in, dt, out, len, (1ull << 56) | ((uint64_t)len << 32) | (uint32_t)at, h, i, pw, false);
    return s == JS_NONE ? JS_NONE : s + 1;
}

// strconv.ParseInt(s, 10, 64) / ParseUint + uint32 overflow on the scalar at pos
// The scalar's bytes up to its terminator from one window: v = the digits (at most 20) as a
// u64 with overflow beyond 2^64 flagged, nd = their count, neg = a leading '-'; returns false
// when the window holds no terminator (long scalars take the byte loops below).
KD_INLINE bool scalar_window(const JsDoc& j, uint32_t pos, uint64_t* v, uint32_t* nd, bool* neg, bool* bad) {
    uint32_t u[8];
    load_window(j.doc, pos, u);
    *neg = (u[0] & 0xFFu) == '-';
    const uint32_t st = *neg ? 1u : 0u;
    // the digits run from st to the first non-digit p (digit mask: no per-byte loop); p must be
    // a terminator, anything else is a parse error like any non-digit before the terminator
    const uint32_t p = first_non_digit(digit_mask(u), st);
    if (p >= 32u) return false;                                         // no terminator in the window
    const uint32_t c = win_byte_at(u, p);
    bool b = !(c <= 0x20 || c == ',' || c == '}' || c == ']');
    uint32_t w[8];                                                      // digit k at byte k
#pragma unroll
    for (int k = 0; k < 7; ++k) w[k] = st ? __builtin_amdgcn_alignbyte(u[k + 1], u[k], 1) : u[k];
    w[7] = st ? u[7] >> 8 : u[7];
    const uint32_t n = p - st;
    uint64_t x = 0;
#pragma unroll
    for (int k = 0; k < 20; ++k) {
        if (!__ballot(k < (int)n)) break;                               // the wave's longest number
        if (k < (int)n) {
            if (x > (~0ull - 9) / 10) b = true;
            x = x * 10 + (((w[k >> 2] >> (8 * (k & 3))) & 0xFFu) - '0');
        }
    }
    if (n > 20u) b = true;                                              // beyond 2^64 (and the loop)
    *v = x;
    *nd = n;
    *bad = b;
    return true;
}
KD_INLINE bool parse_int64(const JsDoc& j, uint32_t pos, int64_t* out) {
    {
        uint64_t v;
        uint32_t nd;
        bool neg, bad;
        if (scalar_window(j, pos, &v, &nd, &neg, &bad)) {
            if (bad || !nd || v > (1ull << 63) || (!neg && v > 0x7FFFFFFFFFFFFFFFull)) return false;
            *out = neg ? (int64_t)(0ull - v) : (int64_t)v;
            return true;
        }
    }
    uint32_t i = pos;
    const bool neg = j.doc[i] == '-';
    if (neg) ++i;
    uint64_t v = 0;
    uint32_t nd = 0;
    for (; i < j.n; ++i) {
        const uint32_t c = j.doc[i];
        if (c <= 0x20 || c == ',' || c == '}' || c == ']') break;
        if (!is_digit(c)) return false;
        if (v > (~0ull - 9) / 10) return false;
        v = v * 10 + (c - '0');
        if (v > (1ull << 63)) return false;
        ++nd;
    }
    if (!nd || (!neg && v > 0x7FFFFFFFFFFFFFFFull)) return false;
    *out = neg ? (int64_t)(0ull - v) : (int64_t)v;
    return true;
}
KD_INLINE bool parse_uint32(const JsDoc& j, uint32_t pos, uint32_t* out) {
    {
        uint64_t v;
        uint32_t nd;
        bool neg, bad;
        if (scalar_window(j, pos, &v, &nd, &neg, &bad)) {
            if (neg || bad || !nd || v > 0xFFFFFFFFull) return false;
            *out = (uint32_t)v;
            return true;
        }
    }
    uint64_t v = 0;
    uint32_t nd = 0;
    for (uint32_t i = pos; i < j.n; ++i) {
        const uint32_t c = j.doc[i];
        if (c <= 0x20 || c == ',' || c == '}' || c == ']') break;
        if (!is_digit(c)) return false;
        v = v * 10 + (c - '0');
        if (v > 0xFFFFFFFFull) return false;
        ++nd;
    }
    if (!nd) return false;
    *out = (uint32_t)v;
    return true;
}

// a record's word in the row-major staging: the wave decoding a link writes its 88 bytes, where
// column-major tile stores put each 4-byte value in a line of its own, written back partially
// by every XCD whose workgroups touched the tile
KD_INLINE uint32_t* store_word(const JsStore& st, uint32_t rec, int col) {
    return st.base + (size_t)rec * JS_ROW + col;
}

__global__ void __launch_bounds__(BLOCK) k_js_values(JsDoc j, JsToks tk, const uint32_t* vlist, uint32_t nval,
                                                     const uint32_t* par, const uint8_t* role, const uint32_t* ord,
                                                     JsTopoOut to, JsStore des, JsStore real, JsIntern in,
                                                     unsigned long long* derr) {
    // every schema member name in one table, looked up by a perfect hash of its 16 bytes (the
    // per-role name lists it replaces were compared one by one, and a wave of mixed roles ran
    // every role's list)
    __shared__ uint64_t s_nm[KN_ALL][2];
    __shared__ int8_t s_slot[128];
    if (threadIdx.x < 128) s_slot[threadIdx.x] = -1;
    __syncthreads();
    if (threadIdx.x < KN_ALL) {
        const uint64_t* nm = reinterpret_cast<const uint64_t*>(kAll[threadIdx.x]);
        s_nm[threadIdx.x][0] = nm[0];
        s_nm[threadIdx.x][1] = nm[1];
        s_slot[name_hash(nm[0], nm[1])] = (int8_t)threadIdx.x;
    }
    __syncthreads();
    const uint32_t k = blockIdx.x * BLOCK + threadIdx.x;
    if (k >= nval) return;
    const uint32_t i = vlist[k];                       // object member values, document order
    const uint32_t t = tk.meta[i];
    const uint32_t vpos = tk.pos[i], kpos = tk.pos[i - 1];   // the value, the member name before it
    const uint32_t dv = tdepth(t);                     // members of root 1, item 3, meta/spec/status 4,
    // every member value gets its vown word here (JS_NONE: not a schema field), so the array
    // needs no clearing pass
    if (dv != 1 && dv != 3 && dv != 4 && dv != 6 && dv != 7) { in.vown[k] = JS_NONE; return; }   // link 6, props 7
    const uint32_t o = par[i];
    if (o >= JS_DEEP) { in.vown[k] = JS_NONE; return; }
    const uint32_t r = role[o];
    const uint32_t po = par[o];                        // the grandparent, loaded with the role
    const KeyName kn = key_name(j, kpos, !(KDTN_PROFILING && (in.variant & JSV_MASKS)));   // while role[o] is in flight
    if (r == R_NONE || r == R_ITEMS || r == R_SPEC_LINKS || r == R_STATUS_LINKS) { in.vown[k] = JS_NONE; return; }
    const uint32_t kind = tkind(t);
    const bool null = kind == TK_SCALAR && j.doc[vpos] == 'n';
    int f, bit;
    {
        const int g0 = s_slot[name_hash(kn.lo, kn.hi)];
        const int g = (kn.ok && g0 >= 0 && s_nm[g0][0] == kn.lo && s_nm[g0][1] == kn.hi) ? g0 : -1;
        const bool link = r == R_LINK_S || r == R_LINK_R;
        const int lo = r == R_ROOT ? KA_ROOT : r == R_ITEM ? KA_ITEM : r == R_META ? KA_META
                     : (r == R_SPEC || r == R_STATUS) ? KA_LINKS : link ? KA_LINK : KA_PROPS;
        const int hi = r == R_ROOT ? KA_ITEM : r == R_ITEM ? KA_META : r == R_META ? KA_LINKS
                     : r == R_SPEC ? KA_LINKS + 1 : r == R_STATUS ? KA_LINK : link ? KA_PROPS : KN_ALL;
        f = (g >= lo && g < hi) ? g - lo : -1;                  // index in the role's name list
    }
    uint32_t own;                                      // owner slot of (object, field): duplicate check
    uint32_t topo = 0, rec = 0;
    JsStore st{};                                      // by value: a pointer to an argument lives in scratch
    switch (r) {
    case R_ROOT:
        bit = f; own = 0;
        break;
    case R_ITEM:
        topo = ord[o]; bit = f; own = 1 + topo * 9;
        break;
    case R_META:
        topo = ord[po]; bit = 3 + f; own = 1 + topo * 9;
        break;
    case R_SPEC:
        topo = ord[po]; bit = 5 + f; own = 1 + topo * 9;
        break;
    case R_STATUS:
        topo = ord[po]; bit = 6 + f; own = 1 + topo * 9;
        break;
    case R_LINK_S:
    case R_LINK_R:
        st = r == R_LINK_S ? des : real;
        rec = ord[o]; bit = f; own = (r == R_LINK_S ? in.own_des : in.own_real) + rec * 22;
        break;
    default: {                                                    // R_PROPS_S / R_PROPS_R
        st = r == R_PROPS_S ? des : real;
        rec = ord[po]; bit = 9 + f; own = (r == R_PROPS_S ? in.own_des : in.own_real) + rec * 22;
        break;
    }
    }
    if (f < 0) { in.vown[k] = JS_NONE; return; }
    // a plain store of this member's token index; k_js_dups then finds every member whose
    // (object, field) slot another member overwrote (no atomics on the hot path)
    own += bit;
    in.owner[own] = i;
    in.vown[k] = own;
    bool ok = true;
    switch (r) {
    case R_ROOT: ok = null || kind == TK_ARR; break;
    case R_ITEM: ok = null || kind == TK_OBJ; break;
    case R_SPEC:
    case R_STATUS:
        if (r == R_SPEC || f == 0) {                              // links
            ok = null || kind == TK_ARR;
            if (kind == TK_ARR) atomicAnd(to.flags + topo, r == R_SPEC ? ~(uint32_t)KDTN_TOPO_SPEC_NIL : ~(uint32_t)KDTN_TOPO_STATUS_NIL);
            break;
        }
        [[fallthrough]];
    case R_META: {
        if (null) break;
        if (kind != TK_STR) { ok = false; break; }
        const uint32_t v = (KDTN_PROFILING && (in.variant & JSV_NO_INTERN)) ? 1u : string_slot(j, in, in.kd, i, vpos);
        if (v == JS_NONE) return;
        uint32_t* dst = r == R_META ? (f == 0 ? to.name : to.ns) : (f == 1 ? to.src_ip : to.net_ns);
        dst[topo] = v;
        break;
    }
    default: {                                                    // link / properties fields
        const bool props = r == R_PROPS_S || r == R_PROPS_R;
        if (!props && f == KDTN_NKEY + 1) { ok = null || kind == TK_OBJ; break; }   // properties
        if (!props && f == KDTN_NKEY) {                                           // uid
            if (null) break;
            int64_t v;
            ok = kind == TK_SCALAR && parse_int64(j, vpos, &v);
            if (ok) {
                *reinterpret_cast<int64_t*>(store_word(st, rec, COL_UID)) = v;   // 8-B aligned (88-B rows)
            }
            break;
        }
        if (props && f == KDTN_NPROP) {                                           // gap
            if (null) break;
            uint32_t v;
            ok = kind == TK_SCALAR && parse_uint32(j, vpos, &v);
            if (ok) *store_word(st, rec, COL_GAP) = v;
            break;
        }
        if (null) break;
        if (kind != TK_STR) { ok = false; break; }
        const uint32_t v = (KDTN_PROFILING && (in.variant & JSV_NO_INTERN)) ? 1u : string_slot(j, in, props ? in.pd : in.kd, i, vpos);
        if (v == JS_NONE) return;
        *store_word(st, rec, props ? COL_PROP0 + f : COL_KEY0 + f) = v;
        break;
    }
    }
    if (!ok) js_fail(derr, vpos, KDTN_JSON_TYPE);
}

// A schema field repeated in one object: its members stored into the same owner slot and only
// one of them finds itself there. Each other member lowers the slot to its own index, so the
// slot ends at the group's first member (the plain store's winner included), and k_js_dups_report
// then reports every later member at its key — the first repeat in document order is the
// earliest, the position a sequential decoder stops at. `any` gates the report pass.
__global__ void __launch_bounds__(BLOCK) k_js_dups(const uint32_t* vlist, uint32_t nval,
                                                   const uint32_t* vown, uint32_t* owner, uint32_t* any) {
    const uint32_t k = blockIdx.x * BLOCK + threadIdx.x;
    if (k >= nval) return;
    const uint32_t own = vown[k];
    if (own == JS_NONE) return;
    const uint32_t i = vlist[k];
    if (owner[own] != i) {
        atomicMin(owner + own, i);
        if (*any == 0) atomicOr(any, 1u);
    }
}

__global__ void __launch_bounds__(BLOCK) k_js_dups_report(const uint32_t* tpos, const uint32_t* vlist, uint32_t nval,
                                                          const uint32_t* vown, const uint32_t* owner,
                                                          const uint32_t* any, unsigned long long* derr) {
    if (*any == 0) return;
    for (uint32_t k = blockIdx.x * BLOCK + threadIdx.x; k < nval; k += gridDim.x * BLOCK) {
        const uint32_t own = vown[k];
        if (own == JS_NONE) continue;
        const uint32_t i = vlist[k];
        if (owner[own] < i) js_fail(derr, tpos[i - 1], KDTN_JSON_DUPKEY);
    }
}

// ---------------------------------------------------------------- ids in first-occurrence order
__global__ void __launch_bounds__(BLOCK) k_js_rep_mark(JsDict dt, uint32_t* bits) {
    const uint32_t s = blockIdx.x * BLOCK + threadIdx.x;
    if (s > dt.mask || dt.keys[s] == 0) return;
    const uint32_t occ = dt.rep[s];
    atomicOr(bits + (occ >> 5), 1u << (occ & 31));
}

__global__ void __launch_bounds__(BLOCK) k_js_popc(const uint32_t* bits, uint32_t nw, uint32_t* cnt) {
    const uint32_t w = blockIdx.x * BLOCK + threadIdx.x;
    if (w < nw) cnt[w] = __popc(bits[w]);
}

// per slot: id = 1 + rank of its first occurrence; length by id, and the slot of each id
__global__ void __launch_bounds__(BLOCK) k_js_ids(JsDict dt, const uint32_t* bits, const uint64_t* wrank,
                                                  uint32_t* slot_id, uint32_t* len_by_id, uint32_t* slot_of_id) {
    const uint32_t s = blockIdx.x * BLOCK + threadIdx.x;
    if (s > dt.mask) return;
    const unsigned long long kw = dt.keys[s];
    if (kw == 0) return;
    const uint32_t occ = dt.rep[s];
    const uint32_t id = 1u + (uint32_t)wrank[occ >> 5] + __popc(bits[occ >> 5] & ((1u << (occ & 31)) - 1u));
    slot_id[s] = id;
    len_by_id[id] = (uint32_t)(kw >> 32) & 0xFFFFFFu;
    slot_of_id[id] = s;
}

// One thread per id (1 .. n-1), in id order: consecutive threads write consecutive arena
// ranges, and first occurrences in id order sit in document order, so both the reads and the
// writes of a wave stay within a few lines (one thread per hash slot scattered both).
__global__ void __launch_bounds__(BLOCK) k_js_dict_copy(JsDict dt, JsIntern in, const uint32_t* slot_of_id, uint32_t n,
                                                        const uint64_t* off64, uint32_t* offs, uint8_t* arena) {
    const uint32_t id = 1u + blockIdx.x * BLOCK + threadIdx.x;
    if (id >= n) return;
    const unsigned long long kw = dt.keys[slot_of_id[id]];
    const uint32_t len = (uint32_t)(kw >> 32) & 0xFFFFFFu;
    const uint64_t at = off64[id];
    offs[id] = (uint32_t)at;
    if (len <= WIN) {                   // one batch of aligned loads (doc and heap are padded)
        uint32_t u[8];
        load_window((kw >> 56) & 1 ? in.heap : in.doc, (uint32_t)kw, u);
#pragma unroll
        for (uint32_t k = 0; k < WIN; ++k)
            if (k < len) arena[at + k] = (uint8_t)win_byte(u, (int)k);
        return;
    }
    const uint8_t* src = key_bytes(in, kw);
    for (uint32_t k = 0; k < len; ++k) arena[at + k] = src[k];
}

// slot + 1 → id in every id column; topology flags to bytes
// One workgroup per tile: the 64 staged rows (5.5 KB, read with 16-B loads) through LDS into
// the tile's columns (coalesced stores), slot + 1 → id in the id columns (records past n are
// zero rows, so the tail of the last tile is written too).
__global__ void __launch_bounds__(BLOCK) k_js_finalize_links(const uint32_t* rows, uint32_t* tiles,
                                                             const uint32_t* kslot_id, const uint32_t* pslot_id) {
    __shared__ uint4 row4[TILE_WORDS / 4];
    const uint32_t* row = reinterpret_cast<const uint32_t*>(row4);
    const uint4* src = reinterpret_cast<const uint4*>(rows + (size_t)blockIdx.x * TILE_WORDS);
    for (uint32_t k = threadIdx.x; k < TILE_WORDS / 4; k += BLOCK) row4[k] = src[k];
    __syncthreads();
    uint32_t* dst = tiles + (size_t)blockIdx.x * TILE_WORDS;
    for (uint32_t k = threadIdx.x; k < TILE_WORDS; k += BLOCK) {
        const uint32_t col = k / TILE_RECS, lane = k % TILE_RECS;
        uint32_t v;
        if (col < (uint32_t)LINK_COLS32) {
            v = row[lane * JS_ROW + col];
            if (col < (uint32_t)COL_GAP && v) v = (col < (uint32_t)COL_PROP0 ? kslot_id : pslot_id)[v - 1];
        } else {                                    // the i64 uid column: record u / 2, word u % 2
            const uint32_t u = k - LINK_COLS32 * TILE_RECS;
            v = row[(u >> 1) * JS_ROW + LINK_COLS32 + (u & 1u)];
        }
        dst[k] = v;
    }
}

__global__ void __launch_bounds__(BLOCK) k_js_finalize_topos(JsTopoOut to, uint32_t T, const uint32_t* kslot_id,
                                                             uint8_t* flags8) {
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    if (t >= T) return;
    uint32_t* cols[4] = {to.ns, to.name, to.src_ip, to.net_ns};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t v = cols[k][t];
        if (v) cols[k][t] = kslot_id[v - 1];
    }
    flags8[t] = (uint8_t)to.flags[t];
}

// ---------------------------------------------------------------- sharded ingest
// Topology t belongs to this shard when kdtn_topology_shard(namespace, name) says so
// (kdtn_shard.h, the host function itself); kreal / kdes are its record counts when kept.
__global__ void __launch_bounds__(BLOCK) k_shard_mark(DevTopos T, const uint8_t* kd_bytes, const uint32_t* kd_offs,
                                                      uint32_t nshards, uint32_t shard, uint32_t* keep,
                                                      uint32_t* kreal, uint32_t* kdes) {
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    if (t >= T.n) return;
    const uint32_t a = T.ns[t], b = T.name[t];
    const uint32_t a0 = kd_offs[a], a1 = kd_offs[a + 1], b0 = kd_offs[b], b1 = kd_offs[b + 1];
    const bool k = topology_shard(kd_bytes + a0, a1 - a0, kd_bytes + b0, b1 - b0, nshards) == shard;
    keep[t] = k ? 1u : 0u;
    kreal[t] = k ? T.real_off[t + 1] - T.real_off[t] : 0u;
    kdes[t] = k ? T.des_off[t + 1] - T.des_off[t] : 0u;
}

// kept topology t → row tidx[t] of the shard's table (offsets from the kept counts' scans)
__global__ void __launch_bounds__(BLOCK) k_shard_topos(DevTopos T, const uint32_t* keep, const uint64_t* tidx,
                                                       const uint64_t* roff, const uint64_t* noff, DevTopos out,
                                                       uint32_t* doc_index) {
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    if (t > T.n) return;
    if (t == T.n) {                                                 // closing offsets
        const uint32_t n = (uint32_t)tidx[t];
        const_cast<uint32_t*>(out.real_off)[n] = (uint32_t)roff[t];
        const_cast<uint32_t*>(out.des_off)[n] = (uint32_t)noff[t];
        return;
    }
    if (!keep[t]) return;
    const uint32_t r = (uint32_t)tidx[t];
    const_cast<uint32_t*>(out.ns)[r] = T.ns[t];
    const_cast<uint32_t*>(out.name)[r] = T.name[t];
    const_cast<uint32_t*>(out.src_ip)[r] = T.src_ip[t];
    const_cast<uint32_t*>(out.net_ns)[r] = T.net_ns[t];
    const_cast<uint8_t*>(out.flags)[r] = T.flags[t];
    const_cast<uint32_t*>(out.real_off)[r] = (uint32_t)roff[t];
    const_cast<uint32_t*>(out.des_off)[r] = (uint32_t)noff[t];
    doc_index[r] = t;
}

// one thread per record of one side: its topology by binary search over the document's
// offsets (the largest t with off[t] <= j), copied with its 22 words when the topology is kept
__global__ void __launch_bounds__(BLOCK) k_shard_links(DevLinks in, const uint32_t* off, uint32_t nt,
                                                       const uint32_t* keep, const uint64_t* noff,
                                                       uint32_t* out_base) {
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= in.n) return;
    uint32_t lo = 0, hi = nt;                                       // off[lo] <= j < off[hi]
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (off[mid] <= j) lo = mid;
        else hi = mid;
    }
    if (!keep[lo]) return;
    const uint32_t d = (uint32_t)noff[lo] + (j - off[lo]);
    const uint32_t* src = in.base + (size_t)(j >> 6) * TILE_WORDS + (j & 63u);
    uint32_t* dst = out_base + (size_t)(d >> 6) * TILE_WORDS + (d & 63u);
#pragma unroll
    for (int c = 0; c < LINK_COLS32; ++c) dst[c * TILE_RECS] = src[c * TILE_RECS];
    const int64_t* su = reinterpret_cast<const int64_t*>(in.base + (size_t)(j >> 6) * TILE_WORDS + LINK_COLS32 * TILE_RECS);
    int64_t* du = reinterpret_cast<int64_t*>(out_base + (size_t)(d >> 6) * TILE_WORDS + LINK_COLS32 * TILE_RECS);
    du[d & 63u] = su[j & 63u];
}

}  // namespace kdtn
