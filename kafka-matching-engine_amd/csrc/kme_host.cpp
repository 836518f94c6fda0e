// kme_host.cpp -- host-side wire format of the matching path (no device code).
//
//   kme_tape_json        JsonSerializer<Order> (KP:477-495) applied to every forwarded record, in
//                        the order the processor forwards them (KP:97, 272-273, 124), printed as
//                        consumer.js prints MatchOut (consumer.js:19): "<key> <value>\n".
//   kme_order_from_json  JsonDeserializer<Order> (KP:497-521) with Jackson 2.9 defaults: creator
//                        properties action/oid/aid/sid/price/size (KP:462-474), numeric strings and
//                        floats coerced, unknown properties rejected.
//   kme_shard_of         Kafka's default keyed partitioner (murmur2) over decimal(|sid|).
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cmath>
#include <emmintrin.h>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

#include "kme.h"

namespace {

inline char* put_i64(char* p, int64_t v) {
    char tmp[24];
    int n = 0;
    uint64_t u = v < 0 ? (0ull - (uint64_t)v) : (uint64_t)v;
    do { tmp[n++] = (char)('0' + (u % 10)); u /= 10; } while (u);
    if (v < 0) *p++ = '-';
    while (n) *p++ = tmp[--n];
    return p;
}
inline char* put_lit(char* p, const char* s) {
    while (*s) *p++ = *s++;
    return p;
}
// {"action":A,"oid":O,"aid":A,"sid":S,"price":P,"size":Z,"next":N,"prev":V}
inline char* put_order(char* p, int32_t action, int64_t oid, int64_t aid, int64_t sid, int32_t price, int32_t size,
                       bool has_prev, int64_t prev) {
    p = put_lit(p, "{\"action\":"); p = put_i64(p, action);
    p = put_lit(p, ",\"oid\":"); p = put_i64(p, oid);
    p = put_lit(p, ",\"aid\":"); p = put_i64(p, aid);
    p = put_lit(p, ",\"sid\":"); p = put_i64(p, sid);
    p = put_lit(p, ",\"price\":"); p = put_i64(p, price);
    p = put_lit(p, ",\"size\":"); p = put_i64(p, size);
    p = put_lit(p, ",\"next\":null,\"prev\":");
    if (has_prev) p = put_i64(p, prev); else p = put_lit(p, "null");
    *p++ = '}';
    return p;
}

struct Out {
    char* buf;
    size_t cap, len;
    char tmp[320];
    void line(const char* key, char* end_of_tmp_value) {
        (void)key;
        const size_t n = (size_t)(end_of_tmp_value - tmp);
        if (len + n <= cap) std::memcpy(buf + len, tmp, n);
        len += n;
    }
};

}  // namespace

extern "C" {

// The processor's MatchOut rows for records [0, n): IN (KP:97), per trade the maker fill then the
// taker fill (executeTrade, KP:265-274), OUT (KP:124).  Same order and values as kme_tape_json, as
// binary rows the JNI glue hands to Java (one Order per row) instead of text.
// Rows of records [a, b) from w on (the caller checked the capacity).
// One row as three 16-B streaming stores (kme_row's layout: oid, aid | sid, prev | action, price,
// size, kind + has_prev << 8): the rows of an epoch are written once and read once, later, by the
// forward loop, so writing them around the caches saves the line fill each write would start (single
// thread at the drop-in's defaults: ~5.6 GB/s of rows with ordinary stores).
static inline void put_row(kme_row* w, int64_t oid, int64_t aid, int64_t sid, int64_t prev, int32_t action, int32_t price,
                           int32_t size, int kind, int has_prev) {
    __m128i* d = reinterpret_cast<__m128i*>(w);
    _mm_stream_si128(d + 0, _mm_set_epi64x(aid, oid));
    _mm_stream_si128(d + 1, _mm_set_epi64x(prev, sid));
    _mm_stream_si128(d + 2, _mm_set_epi32(kind | has_prev << 8, size, price, action));
}
static void expand_range_nt(const kme_orders* in, uint32_t a, uint32_t b, const kme_epoch_result* r, kme_row* w) {
    for (uint32_t i = a; i < b; ++i) {
        const int32_t act = in->action[i], price = in->price[i];
        const int64_t oid = in->oid[i], aid = in->aid[i], sid = in->sid[i];
        put_row(w++, oid, aid, sid, 0, act, price, in->size[i], 0, 0);                      // IN
        const bool taker_buy = act == KME_BUY;
        for (uint32_t t = r->trade_off[i]; t < r->trade_off[i + 1]; ++t) {
            const kme_trade& tr = r->trades[t];
            put_row(w++, tr.maker_oid, tr.maker_aid, tr.maker_sid, 0, taker_buy ? KME_SOLD : KME_BOUGHT, 0, tr.size, 1, 0);
            put_row(w++, oid, aid, sid, 0, taker_buy ? KME_BOUGHT : KME_SOLD,
                    (int32_t)((uint32_t)price - (uint32_t)tr.maker_price), tr.size, 1, 0);
        }
        const int hp = (r->out_flags[i] & KME_OUT_HAS_PREV) ? 1 : 0;                        // OUT: the mutated order
        put_row(w++, oid, aid, sid, hp ? r->out_prev[i] : 0, r->out_action[i], price, r->out_size[i], 2, hp);
    }
    _mm_sfence();   // (streaming stores are weakly ordered: visible before the range is reported done)
}
static void expand_range(const kme_orders* in, uint32_t a, uint32_t b, const kme_epoch_result* r, kme_row* w) {
    if (((uintptr_t)w & 15) == 0) { expand_range_nt(in, a, b, r, w); return; }
    for (uint32_t i = a; i < b; ++i) {
        const int32_t a = in->action[i], price = in->price[i];
        const int64_t oid = in->oid[i], aid = in->aid[i], sid = in->sid[i];
        kme_row x;
        std::memset(&x, 0, sizeof x);
        x.oid = oid; x.aid = aid; x.sid = sid; x.action = a; x.price = price; x.size = in->size[i]; x.kind = 0;
        *w++ = x;
        const bool taker_buy = a == KME_BUY;
        for (uint32_t t = r->trade_off[i]; t < r->trade_off[i + 1]; ++t) {
            const kme_trade& tr = r->trades[t];
            x.kind = 1; x.prev = 0; x.has_prev = 0;
            x.action = taker_buy ? KME_SOLD : KME_BOUGHT;          // maker fill {oid, aid, sid, 0, size}
            x.oid = tr.maker_oid; x.aid = tr.maker_aid; x.sid = tr.maker_sid; x.price = 0; x.size = tr.size;
            *w++ = x;
            x.action = taker_buy ? KME_BOUGHT : KME_SOLD;          // taker fill {.., price - maker price, size}
            x.oid = oid; x.aid = aid; x.sid = sid;
            x.price = (int32_t)((uint32_t)price - (uint32_t)tr.maker_price);
            *w++ = x;
        }
        x.kind = 2;                                                // OUT: the mutated order
        x.oid = oid; x.aid = aid; x.sid = sid; x.price = price;
        x.action = r->out_action[i]; x.size = r->out_size[i];
        x.has_prev = (r->out_flags[i] & KME_OUT_HAS_PREV) ? 1 : 0;
        x.prev = x.has_prev ? r->out_prev[i] : 0;
        *w++ = x;
    }
}

kme_status kme_expand_rows(const kme_orders* in, uint32_t n, const kme_epoch_result* r, kme_row* rows, size_t cap,
                           size_t* n_rows) {
    if (!in || !r || !n_rows || (cap && !rows)) return KME_E_INVALID;
    const size_t need = 2 * (size_t)n + 2 * (size_t)(r->trade_off[n] - r->trade_off[0]);
    *n_rows = need;
    if (need > cap) return KME_E_CAPACITY;
    expand_range(in, 0, n, r, rows);
    return KME_OK;
}

}  // extern "C"

namespace {
// Workers kme_expand_rows_mt hands its record ranges to: created once (per process, on first use)
// and parked on a condition variable between calls.  Starting threads per call cost ~0.5 ms per
// 65,536-record epoch (the drop-in's default), most of its expand time.  One call at a time uses the
// pool; a concurrent caller (another engine's completion) starts threads of its own as before.
struct ExpandPool {
    std::mutex use;                          // held by the call using the pool
    std::mutex m;                            // everything below; tasks are picked under it
    std::condition_variable wake, done;
    std::vector<std::thread> th;
    uint64_t gen = 0;                        // one generation per call
    uint32_t ntask = 0, next = 0, nleft = 0;
    const kme_orders* in = nullptr;
    const kme_epoch_result* r = nullptr;
    kme_row* rows = nullptr;
    uint32_t n = 0;
    // take the call's tasks until none is left (a task: its record range, read under the lock)
    void drain() {
        for (;;) {
            uint32_t a, b;
            const kme_orders* tin;
            const kme_epoch_result* tr;
            kme_row* tw;
            {
                std::lock_guard<std::mutex> g(m);
                if (next >= ntask) return;
                const uint32_t t = next++;
                a = (uint32_t)((uint64_t)n * t / ntask); b = (uint32_t)((uint64_t)n * (t + 1) / ntask);
                tin = in; tr = r;
                tw = rows + 2 * (size_t)a + 2 * (size_t)(r->trade_off[a] - r->trade_off[0]);
            }
            expand_range(tin, a, b, tr, tw);
            std::lock_guard<std::mutex> g(m);
            if (--nleft == 0) done.notify_all();
        }
    }
    void worker() {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> g(m);
                wake.wait(g, [&] { return gen != seen; });
                seen = gen;
            }
            drain();
        }
    }
    void run(const kme_orders* in_, uint32_t n_, const kme_epoch_result* r_, kme_row* rows_, uint32_t T) {
        while (th.size() + 1 < T) { th.emplace_back([this] { worker(); }); th.back().detach(); }
        {
            std::lock_guard<std::mutex> g(m);
            in = in_; n = n_; r = r_; rows = rows_;
            ntask = T; next = 0; nleft = T;
            ++gen;
        }
        wake.notify_all();
        drain();
        std::unique_lock<std::mutex> g(m);
        done.wait(g, [&] { return nleft == 0; });
        ntask = 0;                           // (a late worker finds nothing to take)
    }
};
ExpandPool& expand_pool() {
    static ExpandPool* p = new ExpandPool;   // (never destroyed: its detached workers outlive static teardown)
    return *p;
}
}  // namespace

extern "C" {

kme_status kme_expand_rows_mt(const kme_orders* in, uint32_t n, const kme_epoch_result* r, kme_row* rows, size_t cap,
                              size_t* n_rows, uint32_t n_threads) {
    if (!in || !r || !n_rows || (cap && !rows)) return KME_E_INVALID;
    const size_t need = 2 * (size_t)n + 2 * (size_t)(r->trade_off[n] - r->trade_off[0]);
    *n_rows = need;
    if (need > cap) return KME_E_CAPACITY;
    uint32_t T = n_threads ? n_threads : std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    // records per thread at least: KME_EXPAND_MIN (A/B runs; default 4,096)
    static const uint32_t min_rec = [] {
        const char* v = std::getenv("KME_EXPAND_MIN");
        return v ? (uint32_t)std::max(1, std::atoi(v)) : 4096u;
    }();
    T = std::min<uint32_t>(std::min<uint32_t>(T, 64), std::max<uint32_t>(1, n / min_rec));
    if (T <= 1) { expand_range(in, 0, n, r, rows); return KME_OK; }
    ExpandPool& pool = expand_pool();
    if (pool.use.try_lock()) {
        pool.run(in, n, r, rows, T);
        pool.use.unlock();
        return KME_OK;
    }
    std::vector<std::thread> th;
    th.reserve(T - 1);
    for (uint32_t t = 0; t < T; ++t) {
        const uint32_t a = (uint32_t)((uint64_t)n * t / T), b = (uint32_t)((uint64_t)n * (t + 1) / T);
        kme_row* w = rows + 2 * (size_t)a + 2 * (size_t)(r->trade_off[a] - r->trade_off[0]);
        if (t + 1 == T) expand_range(in, a, b, r, w);
        else th.emplace_back(expand_range, in, a, b, r, w);
    }
    for (auto& x : th) x.join();
    return KME_OK;
}

kme_status kme_tape_json(const kme_orders* in, uint32_t n, const kme_epoch_result* r, char* buf, size_t cap, size_t* len) {
    if (!in || !r || !len) return KME_E_INVALID;
    Out o{buf, buf ? cap : 0, 0, {}};
    for (uint32_t i = 0; i < n; ++i) {
        const int32_t a = in->action[i];
        // IN: the record as received (next/prev null)
        char* p = put_lit(o.tmp, "IN ");
        p = put_order(p, a, in->oid[i], in->aid[i], in->sid[i], in->price[i], in->size[i], false, 0);
        *p++ = '\n';
        o.line("IN", p);
        const bool taker_buy = a == KME_BUY;
        for (uint32_t t = r->trade_off[i]; t < r->trade_off[i + 1]; ++t) {
            const kme_trade& tr = r->trades[t];
            p = put_lit(o.tmp, "OUT ");
            p = put_order(p, taker_buy ? KME_SOLD : KME_BOUGHT, tr.maker_oid, tr.maker_aid, tr.maker_sid, 0, tr.size, false, 0);
            *p++ = '\n';
            o.line("OUT", p);
            p = put_lit(o.tmp, "OUT ");
            const int32_t dp = (int32_t)((uint32_t)in->price[i] - (uint32_t)tr.maker_price);
            p = put_order(p, taker_buy ? KME_BOUGHT : KME_SOLD, in->oid[i], in->aid[i], in->sid[i], dp, tr.size, false, 0);
            *p++ = '\n';
            o.line("OUT", p);
        }
        p = put_lit(o.tmp, "OUT ");
        p = put_order(p, r->out_action[i], in->oid[i], in->aid[i], in->sid[i], in->price[i], r->out_size[i],
                      (r->out_flags[i] & KME_OUT_HAS_PREV) != 0, r->out_prev[i]);
        *p++ = '\n';
        o.line("OUT", p);
    }
    *len = o.len;
    return KME_OK;
}

// ------------------------------------------------------------------ JSON -> Order
namespace {
struct Parser {
    const char* p;
    const char* e;
    void ws() { while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p; }
    bool lit(char c) { ws(); if (p < e && *p == c) { ++p; return true; } return false; }
    bool word(const char* w) {
        size_t n = std::strlen(w);
        if ((size_t)(e - p) >= n && std::memcmp(p, w, n) == 0) { p += n; return true; }
        return false;
    }
    // string without escapes beyond \" \\ (enough for keys and numeric strings)
    bool str(char* out, size_t cap) {
        ws();
        if (p >= e || *p != '"') return false;
        ++p;
        size_t n = 0;
        while (p < e && *p != '"') {
            char c = *p++;
            if (c == '\\') { if (p >= e) return false; c = *p++; }
            if (n + 1 >= cap) return false;
            out[n++] = c;
        }
        if (p >= e) return false;
        ++p;
        out[n] = 0;
        return true;
    }
};

// Jackson's coercion of a scalar token to a Java long / int (Jackson 2.9 defaults).
// kind: 0 = number token, 1 = string token.  Returns false on a value Jackson would reject.
bool to_integral(const char* s, size_t n, bool is_int, int64_t* out) {
    if (n == 0) return false;
    bool fp = false;
    for (size_t i = 0; i < n; ++i)
        if (s[i] == '.' || s[i] == 'e' || s[i] == 'E') fp = true;
    char buf[64];
    if (n >= sizeof buf) return false;
    std::memcpy(buf, s, n);
    buf[n] = 0;
    if (fp) {  // ACCEPT_FLOAT_AS_INT: truncation toward zero
        char* end = nullptr;
        double d = std::strtod(buf, &end);
        if (end != buf + n || !std::isfinite(d)) return false;
        d = std::trunc(d);
        if (is_int ? (d < -2147483648.0 || d > 2147483647.0) : (d < -9223372036854775808.0 || d >= 9223372036854775808.0))
            return false;
        *out = (int64_t)d;
        return true;
    }
    size_t i = 0;
    bool neg = false;
    if (buf[0] == '-' || buf[0] == '+') { neg = buf[0] == '-'; i = 1; }
    if (i >= n) return false;
    uint64_t acc = 0;
    for (; i < n; ++i) {
        if (buf[i] < '0' || buf[i] > '9') return false;
        const uint64_t d = (uint64_t)(buf[i] - '0');
        if (acc > (UINT64_MAX - d) / 10) return false;
        acc = acc * 10 + d;
    }
    const uint64_t lim = is_int ? (neg ? 2147483648ull : 2147483647ull) : (neg ? 9223372036854775808ull : 9223372036854775807ull);
    if (acc > lim) return false;
    *out = neg ? (int64_t)(0ull - acc) : (int64_t)acc;
    return true;
}
}  // namespace

kme_status kme_order_from_json(const char* json, size_t len, int32_t* action, int64_t* oid, int64_t* aid,
                               int64_t* sid, int32_t* price, int32_t* size) {
    if (!json || !action || !oid || !aid || !sid || !price || !size) return KME_E_INVALID;
    Parser P{json, json + len};
    int64_t v[6] = {0, 0, 0, 0, 0, 0};   // absent creator properties default to 0
    static const char* names[8] = {"action", "oid", "aid", "sid", "price", "size", "next", "prev"};
    static const bool is_int[6] = {true, false, false, false, true, true};
    if (!P.lit('{')) return KME_E_INVALID;
    if (!P.lit('}')) {
        for (;;) {
            char key[32];
            if (!P.str(key, sizeof key)) return KME_E_INVALID;
            if (!P.lit(':')) return KME_E_INVALID;
            int k = -1;
            for (int j = 0; j < 8; ++j) if (std::strcmp(key, names[j]) == 0) k = j;
            if (k < 0) return KME_E_INVALID;              // FAIL_ON_UNKNOWN_PROPERTIES
            P.ws();
            if (P.p >= P.e) return KME_E_INVALID;
            if (P.word("null")) {
                if (k < 6) v[k] = 0;                       // null -> primitive default
            } else if (*P.p == '"') {
                char s[64];
                if (!P.str(s, sizeof s)) return KME_E_INVALID;
                if (k >= 6) return KME_E_DOMAIN;          // linked input orders are not carried
                int64_t x;
                if (!to_integral(s, std::strlen(s), is_int[k], &x)) return KME_E_INVALID;
                v[k] = x;
            } else {
                const char* b = P.p;
                while (P.p < P.e && (std::strchr("+-0123456789.eE", *P.p) != nullptr)) ++P.p;
                if (P.p == b) return KME_E_INVALID;       // true/false/objects/arrays
                if (k >= 6) return KME_E_DOMAIN;
                int64_t x;
                if (!to_integral(b, (size_t)(P.p - b), is_int[k], &x)) return KME_E_INVALID;
                v[k] = x;
            }
            if (P.lit(',')) continue;
            if (P.lit('}')) break;
            return KME_E_INVALID;
        }
    }
    P.ws();
    if (P.p != P.e) return KME_E_INVALID;
    *action = (int32_t)v[0]; *oid = v[1]; *aid = v[2]; *sid = v[3]; *price = (int32_t)v[4]; *size = (int32_t)v[5];
    return KME_OK;
}

// org.apache.kafka.common.utils.Utils.murmur2 + toPositive, over the UTF-8 decimal of |sid|.
uint32_t kme_shard_of(int64_t sid, uint32_t n_shards) {
    if (n_shards == 0) return 0;
    char d[24];
    uint64_t u = sid < 0 ? (0ull - (uint64_t)sid) : (uint64_t)sid;
    int n = 0;
    char tmp[24];
    do { tmp[n++] = (char)('0' + u % 10); u /= 10; } while (u);
    for (int i = 0; i < n; ++i) d[i] = tmp[n - 1 - i];
    const uint32_t m = 0x5bd1e995u;
    const int r = 24;
    uint32_t h = 0x9747b28cu ^ (uint32_t)n;
    const int n4 = n / 4;
    for (int i = 0; i < n4; ++i) {
        const int i4 = i * 4;
        uint32_t k = (uint32_t)(uint8_t)d[i4] | ((uint32_t)(uint8_t)d[i4 + 1] << 8) |
                     ((uint32_t)(uint8_t)d[i4 + 2] << 16) | ((uint32_t)(uint8_t)d[i4 + 3] << 24);
        k *= m; k ^= k >> r; k *= m;
        h *= m; h ^= k;
    }
    switch (n % 4) {
    case 3: h ^= (uint32_t)(uint8_t)d[(n & ~3) + 2] << 16; [[fallthrough]];
    case 2: h ^= (uint32_t)(uint8_t)d[(n & ~3) + 1] << 8; [[fallthrough]];
    case 1: h ^= (uint32_t)(uint8_t)d[n & ~3]; h *= m;
    }
    h ^= h >> 13; h *= m; h ^= h >> 15;
    return (h & 0x7fffffffu) % n_shards;
}

}  // extern "C"

// ------------------------------------------------------------------ the state changelog's chunks
// A checkpoint file cut into chunk_bytes chunks, a content hash each (four multiply-xorshift lanes
// over 8-byte words), read and hashed by up to 16 host threads (pread, no shared file offset).  The
// drop-in puts the chunks whose hash changed since the last commit into its changelogged commit store
// (INTEGRATION.md §3).
namespace {
uint64_t chunk_hash(const unsigned char* p, size_t n) {
    uint64_t a = 0x9e3779b97f4a7c15ull, b = 0xbf58476d1ce4e5b9ull, c = 0x94d049bb133111ebull, d = 0x2545f4914f6cdd1dull;
    size_t k = 0;
    for (; k + 32 <= n; k += 32) {
        uint64_t w[4];
        std::memcpy(w, p + k, 32);
        a = (a ^ w[0]) * 0xff51afd7ed558ccdull; a ^= a >> 29;
        b = (b ^ w[1]) * 0xc4ceb9fe1a85ec53ull; b ^= b >> 31;
        c = (c ^ w[2]) * 0xff51afd7ed558ccdull; c ^= c >> 29;
        d = (d ^ w[3]) * 0xc4ceb9fe1a85ec53ull; d ^= d >> 31;
    }
    for (; k < n; ++k) a = (a ^ p[k]) * 0x100000001b3ull;
    uint64_t h = a ^ (b << 1) ^ (c << 2) ^ (d << 3) ^ (uint64_t)n;
    h ^= h >> 33; h *= 0xff51afd7ed558ccdull; h ^= h >> 33;
    return h;
}
}  // namespace

extern "C" kme_status kme_checkpoint_chunks(const char* path, uint32_t chunk_bytes, uint64_t* hashes, size_t cap,
                                            size_t* n_chunks) {
    if (!path || !n_chunks || chunk_bytes < 4096) return KME_E_INVALID;
    const int fd = ::open(path, O_RDONLY);
    if (fd < 0) return KME_E_INVALID;
    struct stat sb;
    if (::fstat(fd, &sb) != 0) { ::close(fd); return KME_E_INVALID; }
    const uint64_t size = (uint64_t)sb.st_size;
    const size_t n = (size_t)((size + chunk_bytes - 1) / chunk_bytes);
    *n_chunks = n;
    if (n > cap || (n && !hashes)) { ::close(fd); return KME_E_CAPACITY; }
    const uint32_t T = (uint32_t)std::min<size_t>(std::max<size_t>(n, 1), std::min(16u, std::max(1u, std::thread::hardware_concurrency())));
    std::vector<std::thread> th;
    std::vector<int> ok(T, 1);
    for (uint32_t t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            std::vector<unsigned char> buf(chunk_bytes);
            for (size_t k = t; k < n; k += T) {
                const uint64_t at = (uint64_t)k * chunk_bytes;
                const size_t len = (size_t)std::min<uint64_t>(chunk_bytes, size - at);
                size_t got = 0;
                while (got < len) {
                    const ssize_t r = ::pread(fd, buf.data() + got, len - got, (off_t)(at + got));
                    if (r <= 0) { ok[t] = 0; return; }
                    got += (size_t)r;
                }
                hashes[k] = chunk_hash(buf.data(), len);
            }
        });
    for (auto& x : th) x.join();
    ::close(fd);
    for (int v : ok) if (!v) return KME_E_INVALID;
    return KME_OK;
}
