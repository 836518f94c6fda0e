/* kme_workload.c -- cancel targets for the synthetic workloads (kme/workloads.py), host only.
 *
 * A cancel/replace trader cancels an order it still has on the book.  Which of an account's orders
 * still rest depends on the matching, so the generator replays the stream through a plain
 * price-time book while it writes it: per (symbol, side, price) a FIFO, BUY matched against the
 * lowest asks up to its price, SELL against the highest bids down to its price, the remainder
 * resting at the tail (KP:200-263 without the ledger and without the H3 / H5 quirks, which never
 * change which orders rest for sizes >= 1 and prices < 127).  A CANCEL row takes the oid of its
 * account's most recent order that is still resting (0 if none: the reference rejects it, KP:290)
 * and removes it from the book.
 *
 * Workload generation only: nothing on the matching path calls it, and the engine and the oracle
 * process whatever stream comes out.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { BUY = 2, SELL = 3, CANCEL = 4, NP = 128 };

typedef struct node { int32_t size, next, prev, acc_prev; int32_t level; uint8_t live; } node;

/* Returns 0, or -1 on bad input / out of memory.  oid[i] of every CANCEL row is overwritten. */
int kme_gen_live_cancels(uint32_t n, const int32_t* action, const int64_t* aid, const int64_t* sid,
                         const int32_t* price, const int32_t* size, int64_t* oid, uint32_t n_accounts,
                         uint32_t max_sid) {
    const size_t n_lev = (size_t)(max_sid + 1) * 2 * NP;
    node* nd = (node*)calloc(n ? n : 1, sizeof(node));
    int32_t* head = (int32_t*)malloc(n_lev * sizeof(int32_t));
    int32_t* tail = (int32_t*)malloc(n_lev * sizeof(int32_t));
    uint64_t* bm = (uint64_t*)calloc((size_t)(max_sid + 1) * 2 * 2, sizeof(uint64_t));   /* [sym][side][2 words] */
    int32_t* top = (int32_t*)malloc((size_t)(n_accounts ? n_accounts : 1) * sizeof(int32_t));
    if (!nd || !head || !tail || !bm || !top) { free(nd); free(head); free(tail); free(bm); free(top); return -1; }
    memset(head, 0xff, n_lev * sizeof(int32_t));
    memset(tail, 0xff, n_lev * sizeof(int32_t));
    memset(top, 0xff, (size_t)(n_accounts ? n_accounts : 1) * sizeof(int32_t));
#define LV(s, side, p) ((((size_t)(s) * 2 + (side)) * NP) + (size_t)(p))
#define BM(s, side) (bm + ((size_t)(s) * 2 + (side)) * 2)
    for (uint32_t i = 0; i < n; ++i) {
        const int32_t a = action[i];
        const int64_t acct = aid[i];
        if (a == CANCEL) {
            int64_t got = 0;
            if (acct >= 0 && (uint64_t)acct < n_accounts) {
                int32_t t = top[acct];
                while (t >= 0 && !nd[t].live) t = nd[t].acc_prev;   /* drop filled / cancelled ones */
                if (t >= 0) {
                    node* v = &nd[t];
                    const size_t L = (size_t)v->level;
                    if (v->prev >= 0) nd[v->prev].next = v->next; else head[L] = v->next;
                    if (v->next >= 0) nd[v->next].prev = v->prev; else tail[L] = v->prev;
                    if (head[L] < 0) {                              /* level empty: clear its bit */
                        const int p = (int)(L % NP), side = (int)((L / NP) % 2);
                        const size_t s = L / NP / 2;
                        BM(s, side)[p >> 6] &= ~(1ull << (p & 63));
                    }
                    v->live = 0;
                    got = oid[t];
                    t = v->acc_prev;
                }
                top[acct] = t;
            }
            oid[i] = got;
            continue;
        }
        if (a != BUY && a != SELL) continue;
        const int64_t s = sid[i] < 0 ? -sid[i] : sid[i];
        const int p = price[i];
        if (s > (int64_t)max_sid || p < 0 || p >= NP || size[i] < 0) continue;   /* not resting anywhere */
        const int side = a == BUY ? 0 : 1, opp = 1 - side;
        int32_t rem = size[i];
        uint64_t* ob = BM(s, opp);
        while (rem > 0) {
            int best;
            if (a == BUY) {                                          /* lowest ask <= p */
                if (ob[0]) best = __builtin_ctzll(ob[0]);
                else if (ob[1]) best = 64 + __builtin_ctzll(ob[1]);
                else break;
                if (best > p) break;
            } else {                                                 /* highest bid >= p */
                if (ob[1]) best = 127 - __builtin_clzll(ob[1]);
                else if (ob[0]) best = 63 - __builtin_clzll(ob[0]);
                else break;
                if (best < p) break;
            }
            const size_t L = LV(s, opp, best);
            while (rem > 0 && head[L] >= 0) {
                node* m = &nd[head[L]];
                const int32_t t = rem < m->size ? rem : m->size;
                rem -= t;
                m->size -= t;
                if (m->size == 0) {
                    m->live = 0;
                    head[L] = m->next;
                    if (head[L] >= 0) nd[head[L]].prev = -1; else tail[L] = -1;
                }
            }
            if (head[L] < 0) ob[best >> 6] &= ~(1ull << (best & 63));
        }
        if (rem > 0 || size[i] == 0) {                               /* rests at the tail of its level */
            const size_t L = LV(s, side, p);
            node* v = &nd[i];
            v->size = rem; v->next = -1; v->prev = tail[L]; v->level = (int32_t)L; v->live = 1;
            if (tail[L] >= 0) nd[tail[L]].next = (int32_t)i; else head[L] = (int32_t)i;
            tail[L] = (int32_t)i;
            BM(s, side)[p >> 6] |= 1ull << (p & 63);
            if (acct >= 0 && (uint64_t)acct < n_accounts) { v->acc_prev = top[acct]; top[acct] = (int32_t)i; }
        }
    }
#undef LV
#undef BM
    free(nd); free(head); free(tail); free(bm); free(top);
    return 0;
}

/* C5: cancel/replace quoting with sweeps, shaped by the same book replay.
 * Every account keeps `quotes` quotes and replaces them in turn: a pair unit of account a is a
 * CANCEL of a's quote in slot j = (its pair count) mod quotes -- the oid of the order that slot holds
 * while it still rests, 0 if the slot is empty or the quote was filled (the reference rejects it,
 * KP:290) -- then the new quote for slot j on side is_sell[u] at a passive price: BUY
 * min(best ask - 1, mid) - d, SELL max(best bid + 1, mid) + d, d = floor(u_price[u] * 10) ticks,
 * clamped to [30, 75].  A sweep unit is a large marketable order (BUY at 75 / SELL at 30) of size
 * min(big_size[u], sweep_frac x the opposite side's quantity within its limit) (at least 1): it clears
 * the best levels and stops inside the book, never resting a remainder that would pin it.  Writes 2 rows per pair and 1 per
 * sweep (new oids from new_oid[], one per unit).  Returns the row count, or -1. */
int64_t kme_gen_cancel_replace(uint32_t n_units, const uint8_t* kind, const int64_t* acct, const int64_t* sym,
                               const uint8_t* is_sell, const double* u_price, const int32_t* quote_size,
                               const int32_t* big_size, const int64_t* new_oid, uint32_t n_accounts, uint32_t max_sid,
                               uint32_t quotes, double sweep_frac, int32_t* action, int64_t* aid, int64_t* sid, int32_t* price,
                               int32_t* size, int64_t* oid) {
    uint64_t rows = 0;
    for (uint32_t u = 0; u < n_units; ++u) rows += kind[u] == 0 ? 2 : 1;
    if (!quotes) quotes = 1;
    node* nd = (node*)calloc(rows ? rows : 1, sizeof(node));
    const size_t n_lev = (size_t)(max_sid + 1) * 2 * NP;
    int32_t* head = (int32_t*)malloc(n_lev * sizeof(int32_t));
    int32_t* tail = (int32_t*)malloc(n_lev * sizeof(int32_t));
    int64_t* qty = (int64_t*)calloc(n_lev, sizeof(int64_t));
    uint64_t* bm = (uint64_t*)calloc((size_t)(max_sid + 1) * 2 * 2, sizeof(uint64_t));
    int32_t* ring = (int32_t*)malloc((size_t)(n_accounts ? n_accounts : 1) * quotes * sizeof(int32_t));
    uint32_t* turn = (uint32_t*)calloc(n_accounts ? n_accounts : 1, sizeof(uint32_t));
    int64_t ret = -1;
    if (!nd || !head || !tail || !qty || !bm || !ring || !turn) goto out;
    memset(head, 0xff, n_lev * sizeof(int32_t));
    memset(tail, 0xff, n_lev * sizeof(int32_t));
    memset(ring, 0xff, (size_t)(n_accounts ? n_accounts : 1) * quotes * sizeof(int32_t));
#define LV(s, side, p) ((((size_t)(s) * 2 + (side)) * NP) + (size_t)(p))
#define BM(s, side) (bm + ((size_t)(s) * 2 + (side)) * 2)
    uint64_t r = 0;
    for (uint32_t u = 0; u < n_units; ++u) {
        const int64_t a = acct[u], s = sym[u];
        if (s < 0 || s > (int64_t)max_sid || a < 0 || (uint64_t)a >= n_accounts) goto out;
        uint64_t* bb = BM(s, 0);
        uint64_t* ab = BM(s, 1);
        const int best_bid = bb[1] ? 127 - __builtin_clzll(bb[1]) : bb[0] ? 63 - __builtin_clzll(bb[0]) : -1;
        const int best_ask = ab[0] ? __builtin_ctzll(ab[0]) : ab[1] ? 64 + __builtin_ctzll(ab[1]) : -1;
        const int sell = is_sell[u] != 0;
        int32_t* slot = NULL;
        int32_t p, z;
        if (kind[u] == 0) {
            /* the cancel: the quote this pair replaces, if it still rests */
            slot = &ring[(size_t)a * quotes + turn[a]++ % quotes];
            int64_t got = 0;
            if (*slot >= 0 && nd[*slot].live) {
                node* v = &nd[*slot];
                const size_t L = (size_t)v->level;
                if (v->prev >= 0) nd[v->prev].next = v->next; else head[L] = v->next;
                if (v->next >= 0) nd[v->next].prev = v->prev; else tail[L] = v->prev;
                qty[L] -= v->size;
                if (head[L] < 0) {
                    const int pp = (int)(L % NP), sd = (int)((L / NP) % 2);
                    BM(L / NP / 2, sd)[pp >> 6] &= ~(1ull << (pp & 63));
                }
                v->live = 0;
                got = oid[*slot];
            }
            *slot = -1;
            action[r] = CANCEL; aid[r] = a; sid[r] = 0; price[r] = 0; size[r] = 0; oid[r] = got;
            ++r;
            /* the replacing quote, at a passive price */
            const int mid = best_bid >= 0 && best_ask >= 0 ? (best_bid + best_ask) / 2
                          : best_ask >= 0 ? best_ask - 1 : best_bid >= 0 ? best_bid + 1 : 52;
            const int d = (int)(u_price[u] * 10.0);
            if (!sell) { int ref = best_ask >= 0 && best_ask - 1 < mid ? best_ask - 1 : mid; p = ref - d; }
            else { int ref = best_bid >= 0 && best_bid + 1 > mid ? best_bid + 1 : mid; p = ref + d; }
            p = p < 30 ? 30 : p > 75 ? 75 : p;
            z = quote_size[u];
        } else {
            /* a sweep: everything it can reach within its limit, at most big_size */
            p = sell ? 30 : 75;
            int64_t depth = 0;
            for (int q = 0; q < NP; ++q)
                if (sell ? q >= p : q <= p) depth += qty[LV(s, sell ? 0 : 1, q)];
            const int64_t reach = (int64_t)(sweep_frac * (double)depth);
            z = big_size[u] < reach ? big_size[u] : (int32_t)(reach > 0 ? reach : 1);
        }
        /* the new order: match, rest the remainder */
        const uint32_t i = (uint32_t)r;
        action[r] = sell ? SELL : BUY; aid[r] = a; sid[r] = s; price[r] = p; size[r] = z; oid[r] = new_oid[u];
        ++r;
        const int side = sell ? 1 : 0, opp = 1 - side;
        uint64_t* ob = BM(s, opp);
        int32_t rem = z;
        while (rem > 0) {
            int best;
            if (!sell) {
                if (ob[0]) best = __builtin_ctzll(ob[0]); else if (ob[1]) best = 64 + __builtin_ctzll(ob[1]); else break;
                if (best > p) break;
            } else {
                if (ob[1]) best = 127 - __builtin_clzll(ob[1]); else if (ob[0]) best = 63 - __builtin_clzll(ob[0]); else break;
                if (best < p) break;
            }
            const size_t L = LV(s, opp, best);
            while (rem > 0 && head[L] >= 0) {
                node* m = &nd[head[L]];
                const int32_t t = rem < m->size ? rem : m->size;
                rem -= t; m->size -= t; qty[L] -= t;
                if (m->size == 0) {
                    m->live = 0;
                    head[L] = m->next;
                    if (head[L] >= 0) nd[head[L]].prev = -1; else tail[L] = -1;
                }
            }
            if (head[L] < 0) ob[best >> 6] &= ~(1ull << (best & 63));
        }
        if (rem > 0) {
            const size_t L = LV(s, side, p);
            node* v = &nd[i];
            v->size = rem; v->next = -1; v->prev = tail[L]; v->level = (int32_t)L; v->live = 1;
            if (tail[L] >= 0) nd[tail[L]].next = (int32_t)i; else head[L] = (int32_t)i;
            tail[L] = (int32_t)i;
            qty[L] += rem;
            BM(s, side)[p >> 6] |= 1ull << (p & 63);
            if (slot) *slot = (int32_t)i;
        }
    }
#undef LV
#undef BM
    ret = (int64_t)r;
out:
    free(nd); free(head); free(tail); free(qty); free(bm); free(ring); free(turn);
    return ret;
}
