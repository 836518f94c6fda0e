/*
 * kme_oracle.c -- CPU restatement of KProcessor.MatchingEngine.  TEST INFRASTRUCTURE ONLY
 * (see kme_oracle.h).  Every function cites the reference line it follows; "KP" =
 * /root/reference/src/main/java/KProcessor.java.  PARITY UNPINNED (no reference tests exist).
 *
 * Java semantics reproduced exactly:
 *   - int arithmetic wraps at 32 bits, long at 64 bits (all products go through unsigned ops);
 *   - long shifts mask the count with 63 (getBit/setBit/unsetBit, KP:406-416);
 *   - `(sid << 8) | price` sign-extends price (KP:379-381);
 *   - stores are value-semantic: get() returns a copy, put() stores a copy (the Kafka Streams
 *     stores serialise on put and deserialise on get);
 *   - the double-precision bit scans (KP:371-377) become ctz/clz plus the threshold table below.
 */
#include "kme_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- Java arithmetic helpers */
static inline int32_t j_iadd(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
static inline int32_t j_isub(int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); }
static inline int32_t j_imul(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }
static inline int32_t j_ineg(int32_t a) { return (int32_t)(0u - (uint32_t)a); }
static inline int64_t j_ladd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
static inline int64_t j_lsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }
static inline int64_t j_lmul(int64_t a, int64_t b) { return (int64_t)((uint64_t)a * (uint64_t)b); }
static inline int64_t j_lshl(int64_t a, int32_t k) { return (int64_t)((uint64_t)a << (k & 63)); }
static inline int64_t j_lmax(int64_t a, int64_t b) { return a >= b ? a : b; }
static inline int64_t j_lmin(int64_t a, int64_t b) { return a <= b ? a : b; }
static inline int32_t j_imin(int32_t a, int32_t b) { return a <= b ? a : b; }

/* Action codes, KP:65-75. */
enum { ADD_SYMBOL = 0, REMOVE_SYMBOL = 1, BUY = 2, SELL = 3, CANCEL = 4, BOUGHT = 5, SOLD = 6,
       REJECT = 7, CREATE_BALANCE = 100, TRANSFER = 101, PAYOUT = 200 };

/* ---------------------------------------------------------------- log10 bit scans (KP:371-377)
 * getFirstSetBitPos(n) = (int)(log10(n & -n) / log10(2)): for n & -n = 2^k, k <= 62, the quotient
 * truncates to exactly k (checked for all k by tools/gen_log10_table.py); for k = 63 the argument
 * is negative, log10 gives NaN and (int)NaN == 0.
 * getLastSetBitPos(n) = (int)(log10((double)n) / log10(2)): negative n -> NaN -> 0; otherwise
 * h = 63 - clz(n), or h + 1 once n >= T[h] = 2^(h+1) - D[h] (h >= 47).  D[] assumes a correctly
 * rounded log10 (HotSpot's intrinsic is within 1 ulp; values near T[h] are outside the parity
 * domain, DESIGN.md "H5"). */
static const int64_t LOG10_OVERSHOOT_D[16] = { /* h = 47 .. 62 */
    1, 2, 3, 7, 14, 28, 90, 178, 340, 663, 1296, 2527, 4799, 9344, 18175, 35328 };

int32_t ko_first_set_bit_pos(int64_t n) {
    uint64_t low = (uint64_t)n & (0ull - (uint64_t)n);
    if (low == 0) return INT32_MIN;               /* log10(0) = -inf -> (int) = MIN_VALUE */
    if (low == (1ull << 63)) return 0;            /* NaN path */
    return __builtin_ctzll(low);
}

int32_t ko_last_set_bit_pos(int64_t n) {
    if (n < 0) return 0;                          /* NaN path */
    if (n == 0) return INT32_MIN;                 /* -inf */
    int32_t h = 63 - __builtin_clzll((uint64_t)n);
    if (h >= 47 && n >= (int64_t)((2ull << h) - (uint64_t)LOG10_OVERSHOOT_D[h - 47])) h += 1;
    return h;
}

/* ---------------------------------------------------------------- hash map (store stand-in) */
typedef struct { int64_t k0, k1; } hkey;

typedef struct hmap {
    size_t cap, live, used; /* used = live + tombstones */
    uint8_t* st;            /* 0 empty, 1 live, 2 tombstone */
    hkey* keys;
    uint8_t* vals;
    size_t vsz;
} hmap;

static uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
static uint64_t hk_hash(hkey k) { return mix64((uint64_t)k.k0 * 0x9e3779b97f4a7c15ull ^ mix64((uint64_t)k.k1)); }

static void hm_init(hmap* m, size_t vsz) {
    m->cap = 64; m->live = m->used = 0; m->vsz = vsz;
    m->st = (uint8_t*)calloc(m->cap, 1);
    m->keys = (hkey*)malloc(m->cap * sizeof(hkey));
    m->vals = (uint8_t*)malloc(m->cap * vsz);
}
static void hm_free(hmap* m) { free(m->st); free(m->keys); free(m->vals); }

static size_t hm_find(const hmap* m, hkey k) { /* index of live k or SIZE_MAX */
    size_t mask = m->cap - 1, i = hk_hash(k) & mask;
    for (;;) {
        uint8_t s = m->st[i];
        if (s == 0) return SIZE_MAX;
        if (s == 1 && m->keys[i].k0 == k.k0 && m->keys[i].k1 == k.k1) return i;
        i = (i + 1) & mask;
    }
}
static void hm_rehash(hmap* m, size_t ncap) {
    hmap n; n.cap = ncap; n.live = n.used = 0; n.vsz = m->vsz;
    n.st = (uint8_t*)calloc(ncap, 1);
    n.keys = (hkey*)malloc(ncap * sizeof(hkey));
    n.vals = (uint8_t*)malloc(ncap * m->vsz);
    for (size_t i = 0; i < m->cap; ++i) {
        if (m->st[i] != 1) continue;
        size_t j = hk_hash(m->keys[i]) & (ncap - 1);
        while (n.st[j]) j = (j + 1) & (ncap - 1);
        n.st[j] = 1; n.keys[j] = m->keys[i];
        memcpy(n.vals + j * n.vsz, m->vals + i * m->vsz, m->vsz);
        n.live++; n.used++;
    }
    hm_free(m); *m = n;
}
/* get(): copy of the value, or 0 if absent (store get returning null). */
static int hm_get(const hmap* m, hkey k, void* out) {
    size_t i = hm_find(m, k);
    if (i == SIZE_MAX) return 0;
    memcpy(out, m->vals + i * m->vsz, m->vsz);
    return 1;
}
static void hm_put(hmap* m, hkey k, const void* v) {
    size_t i = hm_find(m, k);
    if (i != SIZE_MAX) { memcpy(m->vals + i * m->vsz, v, m->vsz); return; }
    if ((m->used + 1) * 2 > m->cap) hm_rehash(m, (m->live + 1) * 4 > m->cap ? m->cap * 2 : m->cap);
    size_t mask = m->cap - 1; i = hk_hash(k) & mask;
    while (m->st[i] == 1) i = (i + 1) & mask;
    if (m->st[i] == 0) m->used++;
    m->st[i] = 1; m->keys[i] = k; memcpy(m->vals + i * m->vsz, v, m->vsz); m->live++;
}
static void hm_del(hmap* m, hkey k) {
    size_t i = hm_find(m, k);
    if (i == SIZE_MAX) return;
    m->st[i] = 2; m->live--;
}

/* ---------------------------------------------------------------- engine */
typedef struct { int64_t msb, lsb; } uuid_t_; /* java.util.UUID(mostSigBits, leastSigBits) */

typedef struct jorder { /* Order, KP:449-458 */
    int32_t action; int32_t price, size; int32_t has_next, has_prev;
    int64_t oid, aid, sid, next, prev;
} jorder;

struct ko_engine {
    hmap balances;  /* Long -> Long,   KP:30-33 */
    hmap positions; /* UUID -> UUID,   KP:34-37 */
    hmap books;     /* Long -> UUID,   KP:38-41 */
    hmap buckets;   /* Long -> UUID,   KP:42-45 */
    hmap orders;    /* Long -> Order,  KP:46-49 */
    ko_rec* tape; size_t tape_len, tape_cap;
    int keep_tape;
    uint64_t forwarded;
};

static hkey LK(int64_t k) { hkey h = { k, 0 }; return h; }
static hkey UK(uuid_t_ u) { hkey h = { u.msb, u.lsb }; return h; }

ko_engine* ko_create(void) {
    ko_engine* e = (ko_engine*)calloc(1, sizeof(ko_engine));
    hm_init(&e->balances, sizeof(int64_t));
    hm_init(&e->positions, sizeof(uuid_t_));
    hm_init(&e->books, sizeof(uuid_t_));
    hm_init(&e->buckets, sizeof(uuid_t_));
    hm_init(&e->orders, sizeof(jorder));
    e->keep_tape = 1;
    return e;
}
void ko_destroy(ko_engine* e) {
    if (!e) return;
    hm_free(&e->balances); hm_free(&e->positions); hm_free(&e->books);
    hm_free(&e->buckets); hm_free(&e->orders); free(e->tape); free(e);
}
void ko_set_keep_tape(ko_engine* e, int keep) { e->keep_tape = keep; }
uint64_t ko_records_forwarded(const ko_engine* e) { return e->forwarded; }

/* ProcessorContext.forward (KP:97, 124, 272-273): the sink serialises synchronously, so the
 * record is a snapshot of the value at forward time. */
static void forward(ko_engine* e, int key, const jorder* o) {
    e->forwarded++;
    if (!e->keep_tape) return;
    if (e->tape_len == e->tape_cap) {
        e->tape_cap = e->tape_cap ? e->tape_cap * 2 : 4096;
        e->tape = (ko_rec*)realloc(e->tape, e->tape_cap * sizeof(ko_rec));
    }
    ko_rec* r = &e->tape[e->tape_len++];
    r->key = key; r->action = o->action; r->oid = o->oid; r->aid = o->aid; r->sid = o->sid;
    r->price = o->price; r->size = o->size;
    r->next = o->has_next ? o->next : 0; r->prev = o->has_prev ? o->prev : 0;
    r->has_next = o->has_next; r->has_prev = o->has_prev;
}

/* new Order(action, oid, aid, sid, price, size) -- KP:462-474 (next = prev = null). */
static jorder mk_order(int32_t action, int64_t oid, int64_t aid, int64_t sid, int32_t price, int32_t size) {
    jorder o; memset(&o, 0, sizeof o);
    o.action = action; o.oid = oid; o.aid = aid; o.sid = sid; o.price = price; o.size = size;
    return o;
}

/* KP:359-369 */
static int32_t min_price_bucket_pointer(uuid_t_ book) {
    if (book.lsb == 0 && book.msb == 0) return -1;
    if (book.lsb == 0) return j_iadd(ko_first_set_bit_pos(book.msb), 63);
    return ko_first_set_bit_pos(book.lsb);
}
static int32_t max_price_bucket_pointer(uuid_t_ book) {
    if (book.msb == 0 && book.lsb == 0) return -1;
    if (book.msb == 0) return ko_last_set_bit_pos(book.lsb);
    return j_iadd(ko_last_set_bit_pos(book.msb), 63);
}
/* KP:379-416 */
static int64_t bucket_pointer(int64_t sid, int32_t price) { return j_lshl(sid, 8) | (int64_t)price; }
static int get_bit(int64_t n, int32_t k) { return ((n >> (k & 63)) & 1) == 1; }
static int64_t set_bit(int64_t n, int32_t k) { return n | j_lshl(1, k); }
static int64_t unset_bit(int64_t n, int32_t k) { return n & ~j_lshl(1, k); }
static int check_bit(uuid_t_ b, int32_t price) {
    return price < 63 ? get_bit(b.lsb, price) : get_bit(b.msb, j_isub(price, 63));
}
static uuid_t_ with_bit_set(uuid_t_ b, int32_t price) {
    uuid_t_ r = b;
    if (price < 63) r.lsb = set_bit(b.lsb, price); else r.msb = set_bit(b.msb, j_isub(price, 63));
    return r;
}
static uuid_t_ with_bit_unset(uuid_t_ b, int32_t price) {
    uuid_t_ r = b;
    if (price < 63) r.lsb = unset_bit(b.lsb, price); else r.msb = unset_bit(b.msb, j_isub(price, 63));
    return r;
}

/* KP:426-436 */
static int get_position(ko_engine* e, int64_t aid, int64_t sid, uuid_t_* out) {
    uuid_t_ k = { aid, sid };
    return hm_get(&e->positions, UK(k), out);
}
static void set_position_key(ko_engine* e, int64_t aid, int64_t sid, int64_t amount, int64_t avail) {
    uuid_t_ k = { aid, sid }, v = { amount, avail };
    hm_put(&e->positions, UK(k), &v);
}
/* setPosition(UUID position, ...) writes under the VALUE as key (H2, KP:434-436). */
static void set_position_val(ko_engine* e, uuid_t_ position, int64_t amount, int64_t avail) {
    uuid_t_ v = { amount, avail };
    hm_put(&e->positions, UK(position), &v);
}

/* createBalance, KP:131-138 */
static int create_balance(ko_engine* e, const jorder* o) {
    int64_t b;
    if (!hm_get(&e->balances, LK(o->aid), &b)) { b = 0; hm_put(&e->balances, LK(o->aid), &b); return 1; }
    return 0;
}
/* transfer, KP:140-146 */
static int transfer(ko_engine* e, const jorder* o) {
    int64_t b;
    if (!hm_get(&e->balances, LK(o->aid), &b) || b < (int64_t)j_ineg(o->size)) return 0;
    b = j_ladd(b, (int64_t)o->size);
    hm_put(&e->balances, LK(o->aid), &b);
    return 1;
}
/* checkBalance, KP:167-182 */
static int check_balance(ko_engine* e, const jorder* o, int* err) {
    int64_t balance;
    if (!hm_get(&e->balances, LK(o->aid), &balance)) return 0;
    int is_buy = o->action == BUY;
    int32_t size = j_imul(o->size, is_buy ? 1 : -1);
    uuid_t_ pos; int has_pos = get_position(e, o->aid, o->sid, &pos);
    int64_t available = has_pos ? pos.lsb : 0;
    int64_t adj = is_buy ? j_lmax(j_lmin(available, 0), (int64_t)j_ineg(size))
                         : j_lmin(j_lmax(available, 0), (int64_t)j_ineg(size));
    int64_t risk = j_lmul(j_ladd((int64_t)size, adj), (int64_t)(is_buy ? o->price : j_isub(o->price, 100)));
    if (balance < risk) return 0;
    int64_t nb = j_lsub(balance, risk);
    hm_put(&e->balances, LK(o->aid), &nb);
    if (adj != 0) {
        if (!has_pos) { *err = KO_E_NPE_POSITION; return 0; }
        set_position_key(e, o->aid, o->sid, pos.msb, j_lsub(available, adj));
    }
    return 1;
}
/* addSymbol, KP:184-191 */
static int add_symbol(ko_engine* e, int64_t sid) {
    uuid_t_ b;
    if (!hm_get(&e->books, LK(sid), &b)) {
        uuid_t_ z = { 0, 0 };
        hm_put(&e->books, LK(sid), &z);
        hm_put(&e->books, LK(j_lsub(0, sid)), &z);
        return 1;
    }
    return 0;
}
/* removeAllOrders, KP:335-357: returns 0 for a missing book, 1 for an empty one; a non-empty
 * book never leaves the loop (it re-sets, rather than clears, the level bit at KP:344). */
static int remove_all_orders(ko_engine* e, int64_t sid, int* err) {
    uuid_t_ book;
    if (!hm_get(&e->books, LK(sid), &book)) return 0;
    if (min_price_bucket_pointer(book) != -1) { *err = KO_E_HANG; return 1; }
    return 1;
}
/* removeSymbol, KP:193-198 */
static int remove_symbol(ko_engine* e, int64_t sid, int* err) {
    if (remove_all_orders(e, sid, err)) return 0;
    if (*err) return 0;
    if (remove_all_orders(e, j_lsub(0, sid), err)) return 0;
    if (*err) return 0;
    hm_del(&e->books, LK(sid));
    hm_del(&e->books, LK(j_lsub(0, sid)));
    return 1;
}

/* fillOrder, KP:276-287 */
static void fill_order(ko_engine* e, const jorder* o, int* err) {
    int32_t size = j_imul(o->size, o->action == BOUGHT ? 1 : -1);
    uuid_t_ pos;
    if (!get_position(e, o->aid, o->sid, &pos)) {
        set_position_key(e, o->aid, o->sid, (int64_t)size, (int64_t)size);
    } else {
        int64_t np = j_ladd(pos.msb, (int64_t)size);
        if (np == 0) hm_del(&e->positions, UK(pos));
        else set_position_val(e, pos, np, j_ladd(pos.lsb, (int64_t)size));
    }
    int64_t b;
    if (!hm_get(&e->balances, LK(o->aid), &b)) { *err = KO_E_NPE_BALANCE; return; }
    b = j_ladd(b, (int64_t)j_imul(size, o->price));
    hm_put(&e->balances, LK(o->aid), &b);
}
/* executeTrade, KP:265-274 */
static void execute_trade(ko_engine* e, const jorder* taker, const jorder* maker, int32_t trade_size,
                          int taker_is_buy, int* err) {
    jorder nm = mk_order(taker_is_buy ? SOLD : BOUGHT, maker->oid, maker->aid, maker->sid, 0, trade_size);
    jorder nt = mk_order(taker_is_buy ? BOUGHT : SOLD, taker->oid, taker->aid, taker->sid,
                         j_isub(taker->price, maker->price), trade_size);
    fill_order(e, &nm, err); if (*err) return;
    fill_order(e, &nt, err); if (*err) return;
    forward(e, 1, &nm);
    forward(e, 1, &nt);
}
/* tryMatch, KP:225-263 */
static int try_match(ko_engine* e, jorder* taker, int* err) {
    int taker_is_buy = taker->action == BUY;
    int64_t sid = j_lmul(taker->sid, taker_is_buy ? 1 : -1);
    int64_t osid = j_lsub(0, sid);
    int32_t price = taker->price;
    uuid_t_ bitmap;
    if (!hm_get(&e->books, LK(osid), &bitmap)) { *err = KO_E_NPE_BOOK; return 0; }
    int32_t price_bit = taker_is_buy ? min_price_bucket_pointer(bitmap) : max_price_bucket_pointer(bitmap);
    if (price_bit == -1) return 0;
    int64_t bp = bucket_pointer(osid, price_bit);
    uuid_t_ bucket;
    if (!hm_get(&e->buckets, LK(bp), &bucket)) { *err = KO_E_NPE_BUCKET; return 0; }
    int64_t maker_ptr = bucket.msb;
    jorder maker;
    if (!hm_get(&e->orders, LK(maker_ptr), &maker)) { *err = KO_E_NPE_ORDER; return 0; }
    /* KP:237, parsed as ((taker.size > 0 && isBuy) ? maker.price <= price : maker.price >= price) (H3) */
    while ((taker->size > 0 && taker_is_buy) ? maker.price <= price : maker.price >= price) {
        int32_t ts = j_imin(taker->size, maker.size);
        maker.size = j_isub(maker.size, ts);
        taker->size = j_isub(taker->size, ts);
        execute_trade(e, taker, &maker, ts, taker_is_buy, err); if (*err) return 0;
        if (maker.size != 0) break;
        hm_del(&e->orders, LK(maker.oid));
        if (!maker.has_next) {
            hm_del(&e->buckets, LK(bp));
            bitmap = with_bit_unset(bitmap, maker.price);
            hm_put(&e->books, LK(osid), &bitmap);
            price_bit = taker_is_buy ? min_price_bucket_pointer(bitmap) : max_price_bucket_pointer(bitmap);
            if (price_bit == -1) return taker->size == 0;
            bp = bucket_pointer(osid, price_bit);
            if (!hm_get(&e->buckets, LK(bp), &bucket)) { *err = KO_E_NPE_BUCKET; return 0; }
            maker_ptr = bucket.msb;
        } else {
            maker_ptr = maker.next;
        }
        if (!hm_get(&e->orders, LK(maker_ptr), &maker)) { *err = KO_E_NPE_ORDER; return 0; }
    }
    uuid_t_ nb = { maker_ptr, bucket.lsb };
    hm_put(&e->buckets, LK(bp), &nb);
    maker.has_prev = 0; maker.prev = 0;
    hm_put(&e->orders, LK(maker_ptr), &maker);
    return taker->size == 0;
}
/* addOrder, KP:200-223 */
static int add_order(ko_engine* e, jorder* o, int* err) {
    int64_t sid = j_lmul(o->sid, o->action == BUY ? 1 : -1);
    uuid_t_ book;
    if (!hm_get(&e->books, LK(sid), &book)) return 0;
    if (!check_balance(e, o, err)) return 0;
    if (try_match(e, o, err)) return 1;
    if (*err) return 0;
    hm_get(&e->books, LK(sid), &book); /* KP:205 re-read (matters for the sid-0 shared book, H4) */
    int64_t oid = o->oid;
    int32_t price = o->price;
    int64_t bp = bucket_pointer(sid, price);
    if (!check_bit(book, price)) {
        uuid_t_ nbk = { oid, oid };
        hm_put(&e->buckets, LK(bp), &nbk);
        uuid_t_ b2 = with_bit_set(book, price);
        hm_put(&e->books, LK(sid), &b2);
    } else {
        uuid_t_ bucket;
        if (!hm_get(&e->buckets, LK(bp), &bucket)) { *err = KO_E_NPE_BUCKET; return 0; }
        int64_t last_ptr = bucket.lsb;
        jorder curr_last;
        if (!hm_get(&e->orders, LK(last_ptr), &curr_last)) { *err = KO_E_NPE_ORDER; return 0; }
        curr_last.next = oid; curr_last.has_next = 1;
        o->prev = curr_last.oid; o->has_prev = 1;
        hm_put(&e->orders, LK(last_ptr), &curr_last);
        uuid_t_ nbk = { bucket.msb, oid };
        hm_put(&e->buckets, LK(bp), &nbk);
    }
    hm_put(&e->orders, LK(oid), o);
    return 1;
}
/* postRemoveAdjustments, KP:325-333 */
static void post_remove_adjustments(ko_engine* e, const jorder* o, int* err) {
    int is_buy = o->action == BUY;
    int32_t size = j_imul(o->size, is_buy ? 1 : -1);
    uuid_t_ pos; int has_pos = get_position(e, o->aid, o->sid, &pos);
    int64_t blocked = has_pos ? j_lsub(pos.msb, pos.lsb) : 0;
    int64_t adj = is_buy ? j_lmax(j_lmin(blocked, 0), (int64_t)j_ineg(size))
                         : j_lmin(j_lmax(blocked, 0), (int64_t)j_ineg(size));
    int64_t b;
    if (!hm_get(&e->balances, LK(o->aid), &b)) { *err = KO_E_NPE_BALANCE; return; }
    b = j_ladd(b, j_lmul(j_ladd((int64_t)size, adj), (int64_t)(is_buy ? o->price : j_isub(o->price, 100))));
    hm_put(&e->balances, LK(o->aid), &b);
    if (adj != 0) {
        if (!has_pos) { *err = KO_E_NPE_POSITION; return; }
        set_position_val(e, pos, pos.msb, j_ladd(pos.lsb, adj));
    }
}
/* removeOrder, KP:289-323 */
static int remove_order(ko_engine* e, int64_t oid, int64_t aid, int* err) {
    jorder o;
    if (!hm_get(&e->orders, LK(oid), &o) || o.aid != aid) return 0;
    int64_t sid = j_lmul(o.sid, o.action == BUY ? 1 : -1);
    int32_t price = o.price;
    uuid_t_ book;
    if (!hm_get(&e->books, LK(sid), &book)) { *err = KO_E_NPE_BOOK; return 0; }
    int64_t bp = bucket_pointer(sid, price);
    uuid_t_ bucket; int has_bucket = hm_get(&e->buckets, LK(bp), &bucket);
    if (!o.has_prev && !o.has_next) {
        hm_del(&e->buckets, LK(bp));
        uuid_t_ b2 = with_bit_unset(book, price);
        hm_put(&e->books, LK(sid), &b2);
    } else if (!o.has_prev) {
        if (!has_bucket) { *err = KO_E_NPE_BUCKET; return 0; }
        uuid_t_ nb = { o.next, bucket.lsb };
        hm_put(&e->buckets, LK(bp), &nb);
        jorder nn;
        if (!hm_get(&e->orders, LK(o.next), &nn)) { *err = KO_E_NPE_ORDER; return 0; }
        nn.has_prev = 0; nn.prev = 0;
        hm_put(&e->orders, LK(o.next), &nn);
    } else if (!o.has_next) {
        if (!has_bucket) { *err = KO_E_NPE_BUCKET; return 0; }
        uuid_t_ nb = { bucket.msb, o.prev };
        hm_put(&e->buckets, LK(bp), &nb);
        jorder pn;
        if (!hm_get(&e->orders, LK(o.prev), &pn)) { *err = KO_E_NPE_ORDER; return 0; }
        pn.has_next = 0; pn.next = 0;
        hm_put(&e->orders, LK(o.prev), &pn);
    } else {
        jorder pn, nn;
        if (!hm_get(&e->orders, LK(o.prev), &pn)) { *err = KO_E_NPE_ORDER; return 0; }
        if (!hm_get(&e->orders, LK(o.next), &nn)) { *err = KO_E_NPE_ORDER; return 0; }
        pn.next = o.next; pn.has_next = 1;
        nn.prev = o.prev; nn.has_prev = 1;
        hm_put(&e->orders, LK(o.prev), &pn);
        hm_put(&e->orders, LK(o.next), &nn);
    }
    hm_del(&e->orders, LK(oid));
    post_remove_adjustments(e, &o, err);
    return *err ? 0 : 1;
}
/* payout, KP:148-165.  Its result is ignored by process() (KP:113-115).  positions.all() order
 * only matters when a balance is missing, and then the reference dies with an NPE part-way. */
static int payout(ko_engine* e, const jorder* o, int* err) {
    if (!remove_symbol(e, o->sid, err)) return 0;
    size_t n = 0, cap = 64;
    hkey* ks = (hkey*)malloc(cap * sizeof(hkey));
    for (size_t i = 0; i < e->positions.cap; ++i) {
        if (e->positions.st[i] != 1) continue;
        hkey k = e->positions.keys[i];
        if (k.k1 != o->sid) continue;
        if (n == cap) { cap *= 2; ks = (hkey*)realloc(ks, cap * sizeof(hkey)); }
        ks[n++] = k;
    }
    for (size_t i = 0; i < n; ++i) {
        int64_t b;
        if (!hm_get(&e->balances, LK(ks[i].k0), &b)) { *err = KO_E_NPE_BALANCE; free(ks); return 0; }
    }
    for (size_t i = 0; i < n; ++i) {
        int64_t b; uuid_t_ pv;
        hm_get(&e->balances, LK(ks[i].k0), &b);
        hm_get(&e->positions, ks[i], &pv);
        b = j_ladd(b, j_lmul(pv.msb, (int64_t)o->size));
        hm_put(&e->balances, LK(ks[i].k0), &b);
    }
    for (size_t i = 0; i < n; ++i) hm_del(&e->positions, ks[i]);
    free(ks);
    return 1;
}

/* process, KP:96-126 */
static int process(ko_engine* e, jorder* o) {
    int err = 0;
    forward(e, 0, o);
    int result = 0;
    switch (o->action) {
    case ADD_SYMBOL: result = add_symbol(e, o->sid); break;
    case REMOVE_SYMBOL: result = remove_symbol(e, o->sid, &err); break;
    case BUY: case SELL: result = add_order(e, o, &err); break;
    case CANCEL: result = remove_order(e, o->oid, o->aid, &err); break;
    case PAYOUT: (void)payout(e, o, &err); break;
    case CREATE_BALANCE: result = create_balance(e, o); break;
    case TRANSFER: result = transfer(e, o); break;
    default: break; /* source has no default branch (the stale bytecode's store wipe is not followed) */
    }
    if (err) return err;
    if (!result) o->action = REJECT;
    forward(e, 1, o);
    return KO_OK;
}

int ko_process_batch(ko_engine* e, size_t n, const int32_t* action, const int64_t* oid,
                     const int64_t* aid, const int64_t* sid, const int32_t* price,
                     const int32_t* size, size_t* n_done) {
    for (size_t i = 0; i < n; ++i) {
        jorder o = mk_order(action[i], oid[i], aid[i], sid[i], price[i], size[i]);
        int rc = process(e, &o);
        if (rc) { if (n_done) *n_done = i; return rc; }
    }
    if (n_done) *n_done = n;
    return KO_OK;
}

size_t ko_tape_len(const ko_engine* e) { return e->tape_len; }
const ko_rec* ko_tape(const ko_engine* e) { return e->tape; }
void ko_tape_clear(ko_engine* e) { e->tape_len = 0; }
void ko_free(void* p) { free(p); }

/* Jackson ObjectMapper.writeValueAsString(Order): creator properties first, in creator order,
 * then the remaining public fields (KP:451-458, 463-465); Long null -> null. */
size_t ko_order_json(const ko_rec* r, char* buf) {
    char nx[32], pv[32];
    if (r->has_next) snprintf(nx, sizeof nx, "%lld", (long long)r->next); else strcpy(nx, "null");
    if (r->has_prev) snprintf(pv, sizeof pv, "%lld", (long long)r->prev); else strcpy(pv, "null");
    return (size_t)sprintf(buf, "{\"action\":%d,\"oid\":%lld,\"aid\":%lld,\"sid\":%lld,\"price\":%d,"
                                "\"size\":%d,\"next\":%s,\"prev\":%s}",
                           r->action, (long long)r->oid, (long long)r->aid, (long long)r->sid,
                           r->price, r->size, nx, pv);
}

typedef struct { char* p; size_t len, cap; } sbuf;
static void sb_reserve(sbuf* s, size_t extra) {
    if (s->len + extra + 1 > s->cap) {
        while (s->len + extra + 1 > s->cap) s->cap = s->cap ? s->cap * 2 : 1 << 16;
        s->p = (char*)realloc(s->p, s->cap);
    }
}
static void sb_printf_line(sbuf* s, const char* line, size_t n) {
    sb_reserve(s, n + 1);
    memcpy(s->p + s->len, line, n); s->len += n; s->p[s->len++] = '\n'; s->p[s->len] = 0;
}

char* ko_tape_text(const ko_engine* e, size_t* len) {
    sbuf s = { 0, 0, 0 };
    sb_reserve(&s, 0); s.p[0] = 0;
    char line[320];
    for (size_t i = 0; i < e->tape_len; ++i) {
        const ko_rec* r = &e->tape[i];
        size_t k = (size_t)sprintf(line, "%s ", r->key ? "OUT" : "IN");
        k += ko_order_json(r, line + k);
        sb_printf_line(&s, line, k);
    }
    if (len) *len = s.len;
    return s.p;
}

/* ---------------------------------------------------------------- canonical dumps */
typedef struct { int64_t k0, k1; const uint8_t* v; } kv_ref;
static int kv_cmp(const void* a, const void* b) {
    const kv_ref* x = (const kv_ref*)a; const kv_ref* y = (const kv_ref*)b;
    if (x->k0 != y->k0) return x->k0 < y->k0 ? -1 : 1;
    if (x->k1 != y->k1) return x->k1 < y->k1 ? -1 : 1;
    return 0;
}
static kv_ref* sorted_entries(const hmap* m, size_t* n) {
    kv_ref* v = (kv_ref*)malloc((m->live + 1) * sizeof(kv_ref));
    size_t k = 0;
    for (size_t i = 0; i < m->cap; ++i)
        if (m->st[i] == 1) { v[k].k0 = m->keys[i].k0; v[k].k1 = m->keys[i].k1; v[k].v = m->vals + i * m->vsz; k++; }
    qsort(v, k, sizeof(kv_ref), kv_cmp);
    *n = k;
    return v;
}
/* Format shared with the product's snapshot canonicaliser (kme/state.py):
 *   B <key> <msb> <lsb>            Books      (KP:38-41)
 *   K <bucketPtr> <first> <last>   Buckets    (KP:42-45)
 *   O <oid> <action> <aid> <sid> <price> <size> <next|null> <prev|null>   Orders (KP:46-49) */
char* ko_dump_books(const ko_engine* e, size_t* len) {
    sbuf s = { 0, 0, 0 }; sb_reserve(&s, 0); s.p[0] = 0;
    char line[320]; size_t n, k;
    kv_ref* v = sorted_entries(&e->books, &n);
    for (size_t i = 0; i < n; ++i) {
        uuid_t_ u; memcpy(&u, v[i].v, sizeof u);
        k = (size_t)sprintf(line, "B %lld %lld %lld", (long long)v[i].k0, (long long)u.msb, (long long)u.lsb);
        sb_printf_line(&s, line, k);
    }
    free(v);
    v = sorted_entries(&e->buckets, &n);
    for (size_t i = 0; i < n; ++i) {
        uuid_t_ u; memcpy(&u, v[i].v, sizeof u);
        k = (size_t)sprintf(line, "K %lld %lld %lld", (long long)v[i].k0, (long long)u.msb, (long long)u.lsb);
        sb_printf_line(&s, line, k);
    }
    free(v);
    v = sorted_entries(&e->orders, &n);
    for (size_t i = 0; i < n; ++i) {
        jorder o; memcpy(&o, v[i].v, sizeof o);
        char nx[32], pv[32];
        if (o.has_next) sprintf(nx, "%lld", (long long)o.next); else strcpy(nx, "null");
        if (o.has_prev) sprintf(pv, "%lld", (long long)o.prev); else strcpy(pv, "null");
        k = (size_t)sprintf(line, "O %lld %d %lld %lld %d %d %s %s", (long long)o.oid, o.action,
                            (long long)o.aid, (long long)o.sid, o.price, o.size, nx, pv);
        sb_printf_line(&s, line, k);
    }
    free(v);
    if (len) *len = s.len;
    return s.p;
}
/*   A <aid> <balance>                 Balances  (KP:30-33)
 *   P <keyMsb> <keyLsb> <amount> <available>   Positions (KP:34-37) */
char* ko_dump_ledger(const ko_engine* e, size_t* len) {
    sbuf s = { 0, 0, 0 }; sb_reserve(&s, 0); s.p[0] = 0;
    char line[320]; size_t n, k;
    kv_ref* v = sorted_entries(&e->balances, &n);
    for (size_t i = 0; i < n; ++i) {
        int64_t b; memcpy(&b, v[i].v, sizeof b);
        k = (size_t)sprintf(line, "A %lld %lld", (long long)v[i].k0, (long long)b);
        sb_printf_line(&s, line, k);
    }
    free(v);
    v = sorted_entries(&e->positions, &n);
    for (size_t i = 0; i < n; ++i) {
        uuid_t_ u; memcpy(&u, v[i].v, sizeof u);
        k = (size_t)sprintf(line, "P %lld %lld %lld %lld", (long long)v[i].k0, (long long)v[i].k1,
                            (long long)u.msb, (long long)u.lsb);
        sb_printf_line(&s, line, k);
    }
    free(v);
    if (len) *len = s.len;
    return s.p;
}
