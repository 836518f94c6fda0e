// kme_ledger.hip -- FUNDED + KME_FLAG_EXACT_LEDGER (SURVEY §8 row f next-2): the epoch's ledger
// effects applied in parallel, bit-exact with the reference's arrival-order updates.
//
// Reference (KProcessor.java, "KP"): checkBalance KP:167-182, fillOrder KP:276-287 (twice per trade,
// executeTrade KP:265-274), postRemoveAdjustments KP:325-333, createBalance / transfer KP:131-146,
// and the position store's value-keyed writes KP:434-436 (hazard H2).
//
// After the parallel matching every outcome of the epoch is fixed (accept / reject, every trade):
// the funded proof (check_funded, in k_route) guarantees each checkBalance passes.  What remains are the
// ledger's values, and they decompose:
//
//   * Balances: every effect is an addition (checkBalance's -risk, a fill's size * price, a refund,
//     a transfer), so an account's final balance is its start plus the sum of its deltas in any
//     order (Java long wrap-around is a group).  One wavefront per account sums them.
//   * Positions: the entry keyed (aid, sid) -- a "chain" -- is read by the account's checkBalance,
//     fillOrder and postRemoveAdjustments on that symbol, and written back under its own key only by
//     checkBalance (KP:179-180) and the first fill (KP:280).  Every other write goes under the
//     position's VALUE as key (setPosition(UUID, ...) / positions.delete(position), KP:283-284, 332,
//     434-436): a "value write" to the key (amount, available).  One lane applies a chain's ops in
//     arrival order and records its value writes.
//   * A value write whose key is another chain of this epoch, read after the write, couples the two
//     chains: the reference clobbers that real position.  k_ldetect finds them; repair rounds re-run
//     the coupled chains in parallel, each with its incoming value writes merged in arrival order,
//     until a fixed point (k_lr_rounds: link / run / detect).  At C3 (65,536 accounts x 65,536
//     symbols) thousands of position values per epoch are also live keys -- (amount, available) ~
//     (50, 50) is account 50's position on symbol 50.  No fixed point within S.lrounds rounds, or
//     past a capacity, sends the epoch to the serial replay (k_ledger_replay).
//     Value writes to keys no chain of the epoch reads commit last-writer-wins (latest arrival).
//
// Ops are compacted in arrival order, one per (record, chain) -- a BUY/SELL's checkBalance with its
// taker fills (and any maker fill on the same key) is one op on (aid, sid), each other maker fill one
// op on the maker's key, an accepted cancel one op -- and sorted (stable LSD radix, the partition's
// kernels) by aid * 256 + hash8(sid): an account's ops are contiguous and a chain's are in arrival
// order.  Every effect carries its arrival number seq = i + 2 trade_off[i] for record i (its check or
// cancel), + 2k + 1 for trade k's maker fill, + 2k + 2 for its taker fill -- the executeTrade order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "kme.h"
#include "kme_device.h"
#include "kme_jarith.h"
#include "kme_launch.h"

namespace kme {

namespace {

// sort key: aid << S.lhbits | a hash of the sid in lhbits (8) bits
constexpr uint32_t OP_CHECK = 0u, OP_FILL = 1u, OP_CANCEL = 2u;   // LOp::flags & 3 (bit 2: buy / bought)
constexpr uint32_t VW_PUT = 1u, VW_DEL = 2u;
constexpr int32_t VT_NONE = -1, VT_INSERT = -2;     // lvw_tgt: into no chain of the epoch / a winner to create
// a winner to create whose key's first free slot (state 0 or 2) is known: -(3 + 2 slot + (state == 2))
KDEV int32_t vt_insert(int32_t free, uint32_t fst) {
    return free >= 0 && free < (1 << 29) ? -(3 + 2 * free + (fst == 2 ? 1 : 0)) : VT_INSERT;
}

KDEV uint32_t lkey_of(const DevState& S, int64_t aid, int64_t sid) {
    return (uint32_t)aid << S.lhbits | (uint32_t)(mix64((uint64_t)sid ^ 0x632be59bd9b4e019ull) >> (64 - S.lhbits));
}

KDEV unsigned long long* lc(const DevState& S, int k) { return &S.lctr[ci(k)]; }
KDEV void lfallback(const DevState& S) { atomicOr(lc(S, LC_FALLBACK), 1ull); }
KDEV bool lfell(const DevState& S) {
    return __hip_atomic_load(lc(S, LC_FALLBACK), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}
// not this path's epoch: a fault (nothing of it is replayed), or a serial epoch (k_serial kept the ledger)
KDEV bool lskip(const DevState& S) { return failed(S.ctr) || S.ctr[ci(C_FALLBACK)] != 0; }
KDEV uint32_t lops(const DevState& S) { return (uint32_t)S.lctr[ci(LC_OPS)]; }

// ---------------------------------------------------------------- stores (Core's layout, shared)
KDEV uint32_t ld_state(const KG uint32_t* p) { return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT); }
KDEV uint32_t pos_hash(const DevState& S, int64_t k0, int64_t k1) {
    return (uint32_t)mix64((uint64_t)k0 * 0x9e3779b97f4a7c15ull ^ mix64((uint64_t)k1)) & S.pos_mask;
}
// positions.get(UUID(k0, k1)): the slot of a live entry, or -1.  The ledger pass never inserts and
// reads the table in one kernel (updates in place and deletes in k_lcommit, inserts in k_linsert), so
// plain loads see every earlier kernel's writes.  For an absent key also the first free slot (empty or
// tombstone) of its probe sequence and that slot's state then (free = -1: none) -- where its insert
// will go unless another key's takes it first (k_linsert tries it before probing again: one claim
// instead of a probe and a claim).
KDEV int32_t pos_lookup_free(const DevState& S, int64_t k0, int64_t k1, int32_t& free, uint32_t& fst) {
    uint32_t h = pos_hash(S, k0, k1);
    free = -1; fst = 0;
    for (uint32_t p = 0; p <= S.pos_mask; ++p) {
        const uint32_t st = S.pos[h].state;
        if (st != 1 && free < 0) { free = (int32_t)h; fst = st; }
        if (st == 0) return -1;
        if (st == 1 && S.pos[h].k0 == k0 && S.pos[h].k1 == k1) return (int32_t)h;
        h = (h + 1) & S.pos_mask;
    }
    return -1;
}
// positions.put of a key known to be absent (k_linsert: every key inserted by one thread, no reader
// in the kernel): the first free slot (empty or tombstone) of its probe sequence, claimed by CAS --
// first at `hint` (pos_lookup_free's slot, in state hst), then along the probe sequence.
// Returns 1 when it took an empty slot (the table's load grows), 0 for a tombstone, -1: no room.
KDEV int pos_insert(const DevState& S, int64_t k0, int64_t k1, int64_t v0, int64_t v1, int32_t hint = -1, uint32_t hst = 0) {
    if (hint >= 0 && atomicCAS((unsigned int*)&S.pos[hint].state, hst, 1u) == hst) {
        S.pos[hint].k0 = k0; S.pos[hint].k1 = k1; S.pos[hint].v0 = v0; S.pos[hint].v1 = v1;
        return hst == 0 ? 1 : 0;
    }
    uint32_t h = pos_hash(S, k0, k1);
    for (uint32_t p = 0; p <= S.pos_mask; ++p) {
        const uint32_t st = S.pos[h].state;
        if ((st == 0 || st == 2) && atomicCAS((unsigned int*)&S.pos[h].state, st, 1u) == st) {
            S.pos[h].k0 = k0; S.pos[h].k1 = k1; S.pos[h].v0 = v0; S.pos[h].v1 = v1;
            return st == 0 ? 1 : 0;
        }
        h = (h + 1) & S.pos_mask;
    }
    return -1;
}
// the sum of v over the wavefront, added by lane 0 to one of 64 counter lines (k_lbalances folds
// them): a single counter hit once per wavefront serialises the kernel (every lane calls it)
constexpr int LPOSC_LINES = 64;
KDEV void wave_add_spread(const DevState& S, uint32_t v) {
    for (int off = 32; off > 0; off >>= 1) v += (uint32_t)__shfl_xor((int)v, off, 64);
    const uint32_t line = (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) & (LPOSC_LINES - 1);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(&S.lposc[(size_t)line * CTR_STRIDE], (unsigned long long)v);
}
// createBalance's put (KP:134), same protocol (balances are never deleted: no tombstones)
KDEV bool bal_create(const DevState& S, int64_t aid) {
    for (int attempt = 0; attempt < 4096; ++attempt) {
        uint32_t h = (uint32_t)mix64((uint64_t)aid) & S.bal_mask;
        uint32_t p = 0;
        for (; p <= S.bal_mask; ++p) {
            const uint32_t st = ld_state(&S.bal_state[h]);
            if (st == 0) break;
            if (st == 1 && S.bal_key[h] == aid) return true;
            h = (h + 1) & S.bal_mask;
        }
        if (p > S.bal_mask) return false;
        if (atomicCAS((unsigned int*)&S.bal_state[h], 0u, 3u) != 0u) continue;
        S.bal_key[h] = aid;
        S.bal_val[h] = 0;
        __threadfence();
        __hip_atomic_store(&S.bal_state[h], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        atomicAdd(&S.ctr[ci(C_BAL_USED)], 1ull);
        return true;
    }
    return false;
}

// ---------------------------------------------------------------- the effects
struct PState {
    int64_t a, v;      // amount, available (KP:418-424)
    bool present;
};
struct VWrite {        // a value write (H2): key = the position read, and the new value
    int64_t k0, k1, v0, v1;
    uint32_t kind;     // 0 none, VW_PUT, VW_DEL
};

// checkBalance (KP:167-182) of an accepted order: the reservation, and when adj != 0 the position's
// available under its own key (KP:179-180; adj != 0 implies the position exists)
KDEV int64_t eff_check(PState& P, bool is_buy, int32_t size, int32_t price) {
    const int32_t s = jimul(size, is_buy ? 1 : -1);
    const int64_t available = P.present ? P.v : 0;
    const int64_t adj = is_buy ? lmax(lmin(available, 0), (int64_t)jineg(s)) : lmin(lmax(available, 0), (int64_t)jineg(s));
    if (adj != 0) P.v = jlsub(available, adj);
    return jlneg(jlmul(jladd((int64_t)s, adj), (int64_t)(is_buy ? price : jisub(price, 100))));
}
// fillOrder (KP:276-287): absent -> created under (aid, sid); present -> the new value written under
// the old VALUE as key (that key deleted when the amount returns to 0); the entry read stays as is
KDEV int64_t eff_fill(PState& P, bool bought, int32_t fsize, int32_t price, VWrite& w) {
    const int32_t s = jimul(fsize, bought ? 1 : -1);
    w.kind = 0;
    if (!P.present) {
        P.present = true;
        P.a = s;
        P.v = s;
    } else {
        const int64_t np = jladd(P.a, (int64_t)s);
        w.k0 = P.a;
        w.k1 = P.v;
        if (np == 0) {
            w.kind = VW_DEL;
        } else {
            w.kind = VW_PUT;
            w.v0 = np;
            w.v1 = jladd(P.v, (int64_t)s);
        }
    }
    return (int64_t)jimul(s, price);
}
// postRemoveAdjustments (KP:325-333): the refund; adj != 0 writes (amount, available + adj) under the
// position's value as key
KDEV int64_t eff_cancel(PState& P, bool is_buy, int32_t size, int32_t price, VWrite& w) {
    const int32_t s = jimul(size, is_buy ? 1 : -1);
    const int64_t blocked = P.present ? jlsub(P.a, P.v) : 0;
    const int64_t adj = is_buy ? lmax(lmin(blocked, 0), (int64_t)jineg(s)) : lmin(lmax(blocked, 0), (int64_t)jineg(s));
    w.kind = 0;
    if (adj != 0) {
        w.kind = VW_PUT;
        w.k0 = P.a;
        w.k1 = P.v;
        w.v0 = P.a;
        w.v1 = jladd(P.v, adj);
    }
    return jlmul(jladd((int64_t)s, adj), (int64_t)(is_buy ? price : jisub(price, 100)));
}
// a value write to the chain's own key changes the chain itself
KDEV void write_into(PState& P, const VWrite& w) {
    if (w.kind == VW_DEL) {
        P.present = false;
    } else if (w.kind == VW_PUT) {
        P.present = true;
        P.a = w.v0;
        P.v = w.v1;
    }
}

// One op of chain (aid, o.sid): its effect on the position P; returns the balance delta, w = its value write.
KDEV int64_t apply_op(const LOp& o, int64_t aid, PState& P, VWrite& w) {
    const bool buy = (o.flags >> 2) & 1u;
    const uint32_t kind = o.flags & 3u;
    w.kind = 0;
    int64_t d;
    if (kind == OP_CHECK) d = eff_check(P, buy, o.size, o.price);
    else if (kind == OP_FILL) d = eff_fill(P, buy, o.size, o.price, w);
    else d = eff_cancel(P, buy, o.size, o.price, w);
    if (w.kind && w.k0 == aid && w.k1 == (int64_t)o.sid) write_into(P, w);   // into its own key
    return d;
}

// The sorted ops' keys (aid << 8 | hash8(sid)) after the last radix pass (the ops themselves: lsrt).
KDEV const KG uint32_t* skeys(const DevState& S) { return S.lkey[S.lpasses & 1]; }
KDEV uint32_t lower_bound(const KG uint32_t* k, uint32_t lo, uint32_t hi, uint32_t key) {
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (k[mid] < key) lo = mid + 1; else hi = mid;
    }
    return lo;
}
// The chain (head position) of key (k0, k1) among this epoch's ops, or -1.
KDEV int32_t find_chain(const DevState& S, int64_t k0, int64_t k1) {
    if (k0 < 0 || k0 >= S.A) return -1;
    const KG uint32_t* K = skeys(S);
    const uint32_t key = lkey_of(S, k0, k1);
    const uint32_t hi = S.lseg[k0 + 1];
    for (uint32_t p = lower_bound(K, S.lseg[k0], hi, key); p < hi && K[p] == key; ++p)
        if ((int64_t)S.lsrt[p].sid == k1) return (int32_t)p;
    return -1;
}

}  // namespace

// ---------------------------------------------------------------- 1. the ops in arrival order
// One op per effect: an accepted BUY/SELL's checkBalance, each of its trades' maker fill (on the
// maker's key) and taker fill, an accepted cancel's postRemoveAdjustments.
__global__ void __launch_bounds__(256) k_lcount(DevState S, EpochIO io) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    // the epoch's counters start at 0 (was fills before this launch; the per-account deltas are 0
    // already: k_lbalances takes each one it settles)
    if (i < (uint32_t)(LC_N * CTR_STRIDE)) S.lctr[i] = 0;
    if (i < (uint32_t)(LPOSC_LINES * CTR_STRIDE)) S.lposc[i] = 0;
    if (i >= io.n) return;
    uint32_t c = 0;
    if (!lskip(S)) {
        const int32_t a = io.action[i], out = io.out_action[i];
        if ((a == BUY || a == SELL) && out == a) c = 1 + 2 * (io.trade_off[i + 1] - io.trade_off[i]);
        else if (a == CANCEL && out == CANCEL) c = 1;
    }
    S.lcnt[i] = c;
}
// At the scanned offsets, in arrival order: the op (LOp: chain sid and account, arrival number, the
// effect's size / price / side) and its sort key aid * 256 + hash8(sid).  Record i's check / cancel
// has arrival number i + 2 trade_off[i], trade q's maker and taker fills i + 2q + 1 and i + 2q + 2
// (executeTrade's order, KP:265-274).  A wavefront takes 64 records and spreads their ops over its
// lanes: op j of the wavefront's range is lane j mod 64's, which finds its record by a binary search
// over the 64 records' op offsets (shuffles) -- one lane walking its record's trades kept the other 63
// waiting, and each lane stored a run of its own (partial lines); now a wavefront's stores are
// consecutive.
__global__ void __launch_bounds__(256) k_lgen(DevState S, EpochIO io) {
    if (lskip(S)) return;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = (int)(threadIdx.x & 63);
    const uint32_t first = i - (uint32_t)lane;               // the wavefront's first record
    if (first >= io.n) return;                               // (uniform)
    const bool valid = i < io.n;
    int32_t a = -1, out = -1;
    if (valid) { a = io.action[i]; out = io.out_action[i]; }
    const bool bs = (a == BUY || a == SELL) && out == a, cx = a == CANCEL && out == CANCEL;
    uint32_t t0 = 0, c = 0, o = 0;
    int64_t aid = 0, sid = 0;
    int32_t price = 0, size = 0;
    if (valid) {
        t0 = io.trade_off[i];
        o = S.lcnt[i];
        if (bs) {
            c = 1 + 2 * (io.trade_off[i + 1] - t0);
            aid = io.aid[i]; sid = io.sid[i]; price = io.price[i]; size = io.size[i];
        } else if (cx) {
            c = 1;
            aid = io.aid[i];
        }
    }
    const uint32_t nv = io.n - first < 64 ? io.n - first : 64;
    const uint32_t base = (uint32_t)__shfl((int)o, 0);
    const uint32_t end = (uint32_t)__shfl((int)(o + c), (int)nv - 1);
    const uint32_t off = valid ? o - base : 0xFFFFFFFFu;     // non-decreasing over the lanes
    // (every shuffle runs on all 64 lanes: a lane past the range still takes part, its op discarded --
    // a shuffle reads nothing defined from a lane that is not active)
    for (uint32_t j0 = 0; j0 < end - base; j0 += 64) {
        const uint32_t j = j0 + (uint32_t)lane;
        int L = 0;                                           // the last record whose ops start at or before j
#pragma unroll
        for (int step = 32; step > 0; step >>= 1) {
            const uint32_t f = (uint32_t)__shfl((int)off, L + step < 64 ? L + step : 63);
            if (L + step < 64 && f <= j) L += step;
        }
        const uint32_t k = j - (uint32_t)__shfl((int)off, L);
        const uint32_t r = first + (uint32_t)L;
        const int32_t ra = __shfl(a, L);
        const int64_t raid = __shfl(aid, L), rsid = __shfl(sid, L);
        const int32_t rprice = __shfl(price, L), rsize = __shfl(size, L);
        const uint32_t rt0 = (uint32_t)__shfl((int)t0, L);
        if (j >= end - base) continue;
        const uint32_t es0 = r + 2 * rt0;
        int64_t oaid, osid;
        uint32_t es, osize, oprice, flags;
        if (ra == CANCEL) {
            const int4 v = S.vic[r];                         // the removed order: action << 8 | price, size, sid
            oaid = raid;
            osid = (int64_t)(((uint64_t)(uint32_t)v.w << 32) | (uint32_t)v.z);
            es = es0; osize = (uint32_t)v.y; oprice = (uint32_t)(v.x & 0xFF);
            flags = OP_CANCEL | ((v.x >> 8) == BUY ? 1u : 0u) << 2;                                       // KP:325-333
        } else {
            const uint32_t buy = ra == BUY ? 1u : 0u;
            if (k == 0) {
                oaid = raid; osid = rsid; es = es0;
                osize = (uint32_t)rsize; oprice = (uint32_t)rprice;
                flags = OP_CHECK | buy << 2;                                                              // KP:167-182
            } else {
                const uint32_t q = rt0 + (k - 1) / 2;
                const TradeRec tr = io.trades[q];
                osize = (uint32_t)tr.size;
                if (((k - 1) & 1) == 0) {
                    oaid = tr.maid; osid = tr.msid; es = r + 2 * q + 1; oprice = 0;
                    flags = OP_FILL | (buy ^ 1u) << 2;                                                    // KP:266-267
                } else {
                    oaid = raid; osid = rsid; es = r + 2 * q + 2; oprice = (uint32_t)jisub(rprice, tr.mprice);
                    flags = OP_FILL | buy << 2;                                                           // KP:268-269
                }
            }
        }
        // an account outside [0, A) (a maker that rested in a serial epoch, KME_FLAG_SERIAL_FALLBACK) is
        // in the exact Balances only: the serial replay takes the epoch's ledger (the op stays, keyed in
        // range, for the passes that still run before they see the fallback)
        if (oaid < 0 || oaid >= S.A) { lfallback(S); oaid = 0; }
        const uint32_t p = base + j;
        // one 16-B store: sid, arrival number, size, price term | flags << 16 (LOp's layout)
        reinterpret_cast<KG uint4*>(S.lrec)[p] =
            make_uint4((uint32_t)(int32_t)osid, es, osize, (uint32_t)(uint16_t)(int16_t)(int32_t)oprice | flags << 16);
        S.lk0[p] = lkey_of(S, oaid, osid);   // (its value in the sort: p itself, R.val0 = nullptr)
        S.lvw_meta[p] = 0;                    // (per sorted position, and positions cover the same range)
        S.lxmark[p] = 0;
    }
}

// ---------------------------------------------------------------- 2. accounts' ranges of the sorted ops
// (the ops themselves were gathered into sorted order by the sort's last pass: lsrt)
// lseg[a] = the number of sorted ops of accounts below a, for a in [0, A]: thread k (an op, or k = n)
// writes k for the accounts after op k - 1's up to op k's.  A gap longer than LSEG_RUN accounts goes
// to a list that k_lseg_gaps fills a workgroup per gap, and a gap longer than LSEG_HUGE to a second
// list (from the top of lgap) that every workgroup of k_lseg_gaps fills a slice of: one thread walking
// a gap was the serial tail when the ops name a few of many accounts (the last op's thread walked to
// A: 13 ms per epoch at A = 2^20 with 65,536 accounts in use), and so was one workgroup per gap (the
// gap past the last account in use: 0.11 ms of the drop-in's 0.45-ms epoch, round 6).  One counter
// word counts both lists (low / high 32 bits).
constexpr uint32_t LSEG_RUN = 256;
constexpr uint32_t LSEG_HUGE = 1u << 16;
KDEV uint32_t lgap_cap(const DevState& S) { return (uint32_t)S.A / 256 + (uint32_t)S.A / 4096 + 8; }   // (its allocation)
__global__ void __launch_bounds__(256) k_lseg(DevState S) {
    const uint32_t n = lops(S);
    const KG uint32_t* K = skeys(S);
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k <= n; k += gridDim.x * blockDim.x) {
        const int64_t prev = k == 0 ? -1 : (int64_t)(K[k - 1] >> S.lhbits);
        const int64_t cur = k == n ? (int64_t)S.A : (int64_t)(K[k] >> S.lhbits);
        if (cur - prev <= (int64_t)LSEG_RUN) {
            for (int64_t a = prev + 1; a <= cur; ++a) S.lseg[a] = k;
        } else if (cur - prev <= (int64_t)LSEG_HUGE) {
            const uint32_t x = (uint32_t)atomicAdd(lc(S, LC_GAPS), 1ull);   // < (A + 1) / LSEG_RUN + 1
            S.lgap[x] = make_uint4((uint32_t)(prev + 1), (uint32_t)cur, k, 0);
        } else {
            const uint32_t y = (uint32_t)(atomicAdd(lc(S, LC_GAPS), 1ull << 32) >> 32);   // < (A + 1) / LSEG_HUGE + 1
            S.lgap[lgap_cap(S) - 1 - y] = make_uint4((uint32_t)(prev + 1), (uint32_t)cur, k, 0);
        }
    }
}
// (run by k_lchains' blocks past its own, blk of nblk: k_lchains does not read lseg -- k_ldetect's
// find_chain is the first reader -- and a launch of its own was ~5 us of a small epoch)
KDEV void lseg_gaps(const DevState& S, uint32_t blk, uint32_t nblk) {
    const unsigned long long c = __hip_atomic_load(lc(S, LC_GAPS), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t ng = (uint32_t)c, nh = (uint32_t)(c >> 32);
    for (uint32_t y = 0; y < nh; ++y) {   // the huge gaps: a slice of each per workgroup
        const uint4 g = S.lgap[lgap_cap(S) - 1 - y];
        for (uint32_t a = g.x + blk * blockDim.x + threadIdx.x; a <= g.y; a += nblk * blockDim.x) S.lseg[a] = g.z;
    }
    for (uint32_t x = blk; x < ng; x += nblk) {
        const uint4 g = S.lgap[x];
        for (uint32_t a = g.x + threadIdx.x; a <= g.y; a += blockDim.x) S.lseg[a] = g.z;
    }
}

// ---------------------------------------------------------------- 3. chains: one thread per sorted op
// Op p heads a chain when no earlier op of its bucket run has its sid (the sort is stable: a chain's
// ops are in arrival order).  The head's thread applies the chain -- start state the Positions entry
// (aid, sid), its ops in order -- and records it (LChain at the head's position, which is also the
// chain's name); an op's value write is kept at the op's sorted position.  The account's balance
// delta: a segmented sum over the wavefront's lanes (the ops are sorted by account), one atomic per
// account run.
__global__ void __launch_bounds__(256) k_lchains(DevState S, uint32_t nb) {
    if (blockIdx.x >= nb) { lseg_gaps(S, blockIdx.x - nb, gridDim.x - nb); return; }   // (the blocks past nb)
    const uint32_t no = lops(S);
    if (lskip(S) || no == 0) return;
    const KG uint32_t* K = skeys(S);
    const int lane = threadIdx.x & 63;
    for (uint32_t base = blockIdx.x * blockDim.x; base < no; base += nb * blockDim.x) {
        const uint32_t j = base + threadIdx.x;
        int64_t aid = -1, cd = 0;
        bool head = false;
        if (j < no) {
            const uint32_t bj = K[j];
            const int32_t sid = S.lsrt[j].sid;
            aid = bj >> S.lhbits;
            head = true;
            for (uint32_t p = j; p > 0 && K[p - 1] == bj; --p)
                if (S.lsrt[p - 1].sid == sid) { head = false; break; }
            if (head) {
                LChain c;                        // built in registers, stored as four 16-B writes (one line)
                int32_t free;
                uint32_t fst;
                const int32_t slot = pos_lookup_free(S, aid, sid, free, fst);
                PState P;
                P.present = slot >= 0;
                P.a = P.present ? S.pos[slot].v0 : 0;
                P.v = P.present ? S.pos[slot].v1 : 0;
                c.sid = sid; c.aid = (int32_t)aid; c.islot = slot >= 0 ? slot : free;
                c.ipres = P.present ? 1 : 0;
                uint32_t last = 0;
                for (uint32_t p = j; p < no && K[p] == bj; ++p) {
                    const LOp op = S.lsrt[p];
                    if (op.sid != sid) continue;
                    VWrite w;
                    cd = jladd(cd, apply_op(op, aid, P, w));
                    last = op.es;
                    if (w.kind) {
                        S.lvw[p] = make_long4(w.k0, w.k1, w.v0, w.v1);
                        S.lvw_meta[p] = w.kind | (j << 2);
                    }
                }
                c.fpres = P.present ? 1 : 0; c.fa = P.a; c.fv = P.v;
                c.delta = cd; c.last_seq = last; c.late = 0; c.rix = 0; c.dirty = 0;   // (the array persists across epochs)
                c.fst = slot >= 0 ? 0 : (uint8_t)fst; c._p = 0; c._pad = 0;
                const uint4* src = reinterpret_cast<const uint4*>(&c);
                KG uint4* dst = reinterpret_cast<KG uint4*>(&S.lchain[j]);
#pragma unroll
                for (int q = 0; q < (int)(sizeof(LChain) / 16); ++q) dst[q] = src[q];
            }
        }
        if (j < no) S.lhead[j] = head ? 1 : 0;   // (a list would serialise on one counter)
        // segmented inclusive sum of cd over runs of equal aid (wrap-around, order-free)
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)cd, off, 64);
            const uint32_t hi = (uint32_t)__shfl_up((int)(uint32_t)((uint64_t)cd >> 32), off, 64);
            const int64_t oa = (int64_t)(((uint64_t)(uint32_t)__shfl_up((int)(uint32_t)((uint64_t)aid >> 32), off, 64) << 32) |
                                         (uint32_t)__shfl_up((int)(uint32_t)aid, off, 64));
            if (lane >= off && oa == aid) cd = jladd(cd, (int64_t)(((uint64_t)hi << 32) | lo));
        }
        const int64_t next = (int64_t)(((uint64_t)(uint32_t)__shfl_down((int)(uint32_t)((uint64_t)aid >> 32), 1, 64) << 32) |
                                       (uint32_t)__shfl_down((int)(uint32_t)aid, 1, 64));
        if (aid >= 0 && cd != 0 && (lane == 63 || next != aid))
            atomicAdd(reinterpret_cast<KG unsigned long long*>(&S.ldelta[aid]), (unsigned long long)cd);
    }
}

// ---------------------------------------------------------------- 4. couplings between chains
// A value write (op p) into a chain of this epoch that the chain reads afterwards (an earlier
// arrival number than its last effect's).
namespace {
KDEV bool coupling(const DevState& S, uint32_t p, uint32_t meta, int32_t c) {
    return (meta & 3u) && c >= 0 && (uint32_t)c != (meta >> 2) && S.lsrt[p].es < S.lchain[c].last_seq;
}
KDEV void list_coupling(const DevState& S, uint32_t p) {
    if (S.lxmark[p]) return;                     // (one writer per p: no race)
    S.lxmark[p] = 1;
    const unsigned long long x = atomicAdd(lc(S, LC_CROSS), 1ull);
    if (x < S.lx_cap) S.lx[x] = p; else lfallback(S);
}
}  // namespace
__global__ void __launch_bounds__(256) k_ldetect(DevState S) {
    if (lskip(S) || lops(S) == 0) return;
    const uint32_t no = lops(S);
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < no; p += gridDim.x * blockDim.x) {
        const uint32_t meta = S.lvw_meta[p];
        if (!(meta & 3u)) continue;
        const long4 w = S.lvw[p];
        const int32_t c = find_chain(S, w.x, w.y);
        S.lvw_tgt[p] = c;
        if (coupling(S, p, meta, c)) list_coupling(S, p);
    }
}

// ---------------------------------------------------------------- 5. repair rounds
// The coupled chains re-run in parallel, each with the value writes into it merged into its own
// effects in arrival order, until nothing changes (a fixed point: a value write only affects later
// effects, so after round r every effect whose causal chain of couplings is at most r deep is
// final).  Round: (a) link: each chain's incoming couplings threaded into a list, the chain added to
// the run list (which only grows: a chain whose coupling went away re-runs without it); (b) run:
// every chain of the run list re-run from its start state -- new final state, balance delta (the
// difference goes to the account's sum) and value writes, the changed ones listed; (c) detect: the
// changed value writes re-targeted, new couplings listed.  No change = converged.  Not converged in
// S.lrounds rounds, or past a capacity: the epoch goes to the serial replay.
//
// One workgroup runs all rounds (k_lr_rounds: the phases separated by barriers, so an epoch without
// couplings costs one launch; thousands of coupled chains take a few microseconds per round).  Values
// another thread wrote by atomics are read back with atomic loads.
namespace {
KDEV uint32_t lc_get(const DevState& S, int k) {
    return (uint32_t)__hip_atomic_load(lc(S, k), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
KDEV void lr_link(const DevState& S, uint32_t t0, uint32_t nt) {
    const uint32_t nx = min(lc_get(S, LC_CROSS), S.lx_cap);
    for (uint32_t x = t0; x < nx; x += nt) {
        const uint32_t p = S.lx[x];
        const int32_t c = S.lvw_tgt[p];
        if (!coupling(S, p, S.lvw_meta[p], c)) continue;
        S.lxn[x] = atomicExch(&S.lchain[c].rix, x + 1);
        if (atomicExch(&S.lchain[c].dirty, 1u) == 0u) {
            const unsigned long long d = atomicAdd(lc(S, LC_DIRTY), 1ull);
            if (d < S.lr_cap) S.lrun[d] = (uint32_t)c; else lfallback(S);
        }
    }
}
constexpr int LR_IN = 32;   // incoming value writes one chain takes in a round (more: the serial replay)
KDEV void lr_run_chain(const DevState& S, uint32_t head) {
    const uint32_t no = lops(S);
    const KG uint32_t* K = skeys(S);
    KG LChain& c = S.lchain[head];
    // the incoming value writes (ops of other chains), in arrival order
    uint64_t in[LR_IN];                           // arrival number << 32 | op position
    int nin = 0;
    for (uint32_t x = __hip_atomic_load(&c.rix, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); x != 0; x = S.lxn[x - 1]) {
        if (nin == LR_IN) { lfallback(S); return; }
        const uint32_t p = S.lx[x - 1];
        const uint64_t e = (uint64_t)S.lsrt[p].es << 32 | p;
        int k = nin++;
        for (; k > 0 && in[k - 1] > e; --k) in[k] = in[k - 1];
        in[k] = e;
    }
    __hip_atomic_store(&c.rix, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int32_t sid = c.sid;
    const int64_t aid = c.aid;
    PState P{0, 0, c.ipres != 0};                 // the start state: the entry at islot (unchanged until k_lcommit)
    if (P.present) { P.a = S.pos[c.islot].v0; P.v = S.pos[c.islot].v1; }
    int64_t cd = 0;
    int q = 0;
    for (uint32_t p = head; p < no && K[p] == K[head]; ++p) {
        const LOp op = S.lsrt[p];
        if (op.sid != sid) continue;
        for (; q < nin && (uint32_t)(in[q] >> 32) < op.es; ++q) {
            const uint32_t ip = (uint32_t)in[q];
            const long4 x = S.lvw[ip];
            write_into(P, VWrite{x.x, x.y, x.z, x.w, S.lvw_meta[ip] & 3u});
        }
        VWrite w;
        cd = jladd(cd, apply_op(op, aid, P, w));
        const uint32_t om = S.lvw_meta[p];
        const uint32_t nm = w.kind ? (w.kind | head << 2) : 0u;
        bool changed = (om & 3u) != (nm & 3u);
        if (!changed && w.kind) {
            const long4 ow = S.lvw[p];
            changed = ow.x != w.k0 || ow.y != w.k1 || (w.kind == VW_PUT && (ow.z != w.v0 || ow.w != w.v1));
        }
        if (changed) {
            S.lvw[p] = make_long4(w.k0, w.k1, w.v0, w.v1);
            S.lvw_meta[p] = nm;
            const unsigned long long k = atomicAdd(lc(S, LC_CHG), 1ull);
            if (k < S.lc_cap) S.lchg[k] = p; else lfallback(S);
        }
    }
    c.fpres = P.present ? 1 : 0; c.fa = P.a; c.fv = P.v;
    atomicAdd(reinterpret_cast<KG unsigned long long*>(&S.ldelta[c.aid]), (unsigned long long)jlsub(cd, c.delta));
    c.delta = cd;
}
KDEV void lr_detect(const DevState& S, uint32_t t0, uint32_t nt, uint32_t nc) {
    for (uint32_t k = t0; k < nc; k += nt) {
        const uint32_t p = S.lchg[k];
        const uint32_t meta = S.lvw_meta[p];
        int32_t c = VT_NONE;
        if (meta & 3u) {
            const long4 w = S.lvw[p];
            c = find_chain(S, w.x, w.y);
        }
        S.lvw_tgt[p] = c;
        if (coupling(S, p, meta, c)) list_coupling(S, p);
    }
}
}  // namespace
__global__ void __launch_bounds__(1024) k_lr_rounds(DevState S) {
    if (lskip(S) || lops(S) == 0) return;
    const uint32_t t = threadIdx.x, nt = blockDim.x;
    for (uint32_t r = 0; r < S.lrounds; ++r) {
        if (lfell(S)) return;                     // (read after a barrier: the same for every thread)
        if (t == 0) __hip_atomic_store(lc(S, LC_CHG), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        lr_link(S, t, nt);
        __syncthreads();
        const uint32_t nd = min(lc_get(S, LC_DIRTY), S.lr_cap);
        for (uint32_t d = t; d < nd; d += nt) lr_run_chain(S, S.lrun[d]);
        __syncthreads();
        const uint32_t nc = min(lc_get(S, LC_CHG), S.lc_cap);
        if (nc == 0) {                            // converged
            if (t == 0) {
                S.lctr[ci(LC_DONE)] = 1;
                S.lctr[ci(LC_REPAIRED)] = nd;
                S.ctr[ci(C_LREPAIRED)] = nd;
            }
            return;
        }
        lr_detect(S, t, nt, nc);
        __syncthreads();
    }
    if (t == 0) lfallback(S);                     // still changing after the last round: the serial replay
}

// ---------------------------------------------------------------- 6. commit
// Value writes: into a chain of the epoch after its last read -> the chain's final value (latest
// wins, `late`); into a chain it reads later -> already applied; into no chain -> last-writer-wins
// per key through a per-epoch table keyed by a 64-bit hash of the key (the key stored by the writer
// that inserted it, and a second pass checks every writer's key against it: a hash collision of two
// different keys sends the epoch to the serial replay).
namespace {
KDEV uint64_t vkey_hash(int64_t k0, int64_t k1) { return mix64((uint64_t)k0 * 0xc2b2ae3d27d4eb4full ^ mix64((uint64_t)k1 + 1)) | 1ull; }
// The table is not cleared between epochs: an entry's hash word carries the epoch's tag in its low 16
// bits (S.lvk_tag, 1..65535; the host clears the table when the tag wraps) and its max word the tag
// above the arrival number (vk_last), so an entry of an earlier epoch reads as empty and loses every
// atomicMax.
KDEV uint64_t vk_word(const DevState& S, uint64_t h) { return (h & ~0xFFFFull) | (uint64_t)S.lvk_tag; }
KDEV bool vk_live(const DevState& S, unsigned long long cur) { return cur != 0 && (cur & 0xFFFFull) == S.lvk_tag; }
KDEV unsigned long long vk_last(const DevState& S, uint32_t es) {
    return ((unsigned long long)S.lvk_tag << 40) | ((unsigned long long)es + 1);
}
// The slot of key hash h (insert: claimed when absent), or -1.  A position value is a small pair, so
// a few keys take most value writes of an epoch: the probe reads before it claims (no atomic on a
// hot key's line unless the slot is empty).
KDEV int64_t vk_slot(const DevState& S, uint64_t h, bool insert, bool* inserted = nullptr) {
    const uint64_t hx = vk_word(S, h);
    uint64_t p = h & S.lvk_mask;
    for (uint32_t probes = 0; probes < 4096; ++probes) {
        KG unsigned long long* e = reinterpret_cast<KG unsigned long long*>(&S.lvk[p]);
        unsigned long long cur = __hip_atomic_load(e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!vk_live(S, cur)) {
            if (!insert) return -1;
            const unsigned long long prev = atomicCAS(e, cur, (unsigned long long)hx);
            if (prev == cur) {
                if (inserted) *inserted = true;
                return (int64_t)p;
            }
            cur = prev;                                  // another writer's claim of this epoch
            if (!vk_live(S, cur)) continue;              // (cannot happen: only claims change a word; the
                                                         // probe cap bounds the retries regardless)
        }
        if (cur == hx) return (int64_t)p;
        p = (p + 1) & S.lvk_mask;
    }
    return -1;
}
// The latest value write per key: the writers take the seqs from the last down, so the first to
// reach a hot key usually holds the maximum and the others skip the atomic.
KDEV void vk_max(KG unsigned long long* p, unsigned long long v) {
    if (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < v) atomicMax(p, v);
}
}  // namespace
__global__ void __launch_bounds__(256) k_lvw_classify(DevState S) {
    if (lskip(S) || lops(S) == 0 || lfell(S)) return;
    const uint32_t no = lops(S);
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < no; k += gridDim.x * blockDim.x) {
        const uint32_t p = no - 1 - k;           // (top-down: see vk_max)
        const uint32_t meta = S.lvw_meta[p];
        if (!(meta & 3u)) continue;
        const int32_t c = S.lvw_tgt[p];
        const uint32_t es = S.lsrt[p].es;
        if (c >= 0) {
            if ((uint32_t)c != (meta >> 2) && es > S.lchain[c].last_seq)
                vk_max(reinterpret_cast<KG unsigned long long*>(&S.lchain[c].late), (unsigned long long)(es + 1) << 32 | p);
            continue;
        }
        const long4 w = S.lvw[p];
        bool ins = false;
        const int64_t v = vk_slot(S, vkey_hash(w.x, w.y), true, &ins);
        if (v < 0) { lfallback(S); return; }
        if (ins) { S.lvk[v].z = (unsigned long long)w.x; S.lvk[v].w = (unsigned long long)w.y; }   // the key, by its inserter
        vk_max(reinterpret_cast<KG unsigned long long*>(&S.lvk[v]) + 1, vk_last(S, es));
    }
}
// Every writer's key against the one its hash slot holds: two keys with one hash send the epoch to
// the serial replay.
__global__ void __launch_bounds__(256) k_lvw_check(DevState S) {
    if (lskip(S) || lops(S) == 0 || lfell(S)) return;
    const uint32_t no = lops(S);
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < no; p += gridDim.x * blockDim.x) {
        if (!(S.lvw_meta[p] & 3u) || S.lvw_tgt[p] >= 0) continue;
        const long4 w = S.lvw[p];
        const int64_t v = vk_slot(S, vkey_hash(w.x, w.y), false);
        if (v < 0 || (int64_t)S.lvk[v].z != w.x || (int64_t)S.lvk[v].w != w.y) { lfallback(S); return; }
    }
}
// Account records (createBalance / transfer, KP:131-146): outcomes fixed by k_ledger_funded.  (Run by
// k_lcommit's blocks past its own: Balances here, Positions there.)
KDEV void lacct(const DevState& S, const EpochIO& io, uint32_t i) {
    if (i >= io.n || lskip(S) || lfell(S) || S.ctr[ci(C_ACCT_OPS)] == 0) return;
    const int32_t a = io.action[i];
    if (io.out_action[i] != a) return;
    if (a == CREATE_BALANCE) {
        if (!bal_create(S, io.aid[i])) raise_thread(S.ctr, KME_E_CAPACITY, KME_D_CAP_LEDGER, io.n);
    } else if (a == TRANSFER) {
        atomicAdd(reinterpret_cast<KG unsigned long long*>(&S.ldelta[io.aid[i]]), (unsigned long long)(int64_t)io.size[i]);
    }
}
// Updates in place and deletes; a key to create is left to k_linsert (the winning value write's
// lvw_tgt = VT_INSERT, the chain by its state).
namespace {
KDEV bool chain_final(const DevState& S, const KG LChain& c, int64_t& fa, int64_t& fv) {
    bool fp = c.fpres != 0;
    fa = c.fa; fv = c.fv;
    if (c.late) {
        const uint32_t p = (uint32_t)c.late;
        const long4 w = S.lvw[p];
        fp = (S.lvw_meta[p] & 3u) == VW_PUT;
        fa = w.z;
        fv = w.w;
    }
    return fp;
}
}  // namespace
__global__ void __launch_bounds__(256) k_lcommit(DevState S, EpochIO io, uint32_t nb) {
    if (blockIdx.x >= nb) { lacct(S, io, (blockIdx.x - nb) * blockDim.x + threadIdx.x); return; }
    if (lskip(S) || lops(S) == 0 || lfell(S)) return;
    const uint32_t no = lops(S);
    const uint32_t stride = nb * blockDim.x, t0 = blockIdx.x * blockDim.x + threadIdx.x;
    // the winning value write of each key no chain reads
    for (uint32_t p = t0; p < no; p += stride) {
        const uint32_t meta = S.lvw_meta[p];
        if (!(meta & 3u) || S.lvw_tgt[p] >= 0) continue;
        const long4 w = S.lvw[p];
        const int64_t v = vk_slot(S, vkey_hash(w.x, w.y), false);
        if (v < 0 || S.lvk[v].y != vk_last(S, S.lsrt[p].es)) continue;
        int32_t free;
        uint32_t fst;
        const int32_t h = pos_lookup_free(S, w.x, w.y, free, fst);
        if ((meta & 3u) == VW_DEL) {
            if (h >= 0) S.pos[h].state = 2u;
        } else if (h >= 0) {
            S.pos[h].v0 = w.z; S.pos[h].v1 = w.w;
        } else {
            S.lvw_tgt[p] = vt_insert(free, fst);
        }
    }
    // every chain's final entry (its own last state, or a later value write into it)
    for (uint32_t p = t0; p < no; p += stride) {
        if (!S.lhead[p]) continue;
        const KG LChain& c = S.lchain[p];
        if (!c.ipres) continue;
        int64_t fa, fv;
        const bool fp = chain_final(S, c, fa, fv);
        if (fp && fa == S.pos[c.islot].v0 && fv == S.pos[c.islot].v1) continue;
        if (fp) { S.pos[c.islot].v0 = fa; S.pos[c.islot].v1 = fv; }
        else S.pos[c.islot].state = 2u;
    }
}
// The keys to create: chains absent at the epoch's start that end present, and value-write winners
// into absent keys.  Every key is new and inserted by one thread (pos_insert).
__global__ void __launch_bounds__(256) k_linsert(DevState S, EpochIO io) {
    if (lskip(S) || lops(S) == 0 || lfell(S)) return;
    const uint32_t no = lops(S);
    uint32_t grew = 0;
    bool full = false;
    const uint32_t stride = gridDim.x * blockDim.x, t0 = blockIdx.x * blockDim.x + threadIdx.x;
    for (uint32_t p = t0; p < no; p += stride) {
        const int32_t tgt = S.lvw_tgt[p];
        if (!(S.lvw_meta[p] & 3u) || tgt > VT_INSERT) continue;
        const long4 w = S.lvw[p];
        const int32_t hint = tgt == VT_INSERT ? -1 : (-(tgt + 3)) >> 1;
        const int r = pos_insert(S, w.x, w.y, w.z, w.w, hint, (uint32_t)(-(tgt + 3)) & 1u ? 2u : 0u);
        full |= r < 0;
        grew += r > 0;
    }
    for (uint32_t p = t0; p < no; p += stride) {
        if (!S.lhead[p]) continue;
        const KG LChain& c = S.lchain[p];
        if (c.ipres) continue;
        int64_t fa, fv;
        if (!chain_final(S, c, fa, fv)) continue;
        const int r = pos_insert(S, (int64_t)c.aid, c.sid, fa, fv, c.islot, c.fst);
        full |= r < 0;
        grew += r > 0;
    }
    if (full) raise_thread(S.ctr, KME_E_CAPACITY, KME_D_CAP_LEDGER, io.n);
    wave_add_spread(S, grew);
}
// The accounts' balance deltas (k_lchains, the repairs, k_lacct's transfers) onto Balances: one thread
// per account run of the sorted ops and per transfer record -- the accounts the epoch touched, not
// all A of them (2^20 at the drop-in's defaults: a pass over every account's delta, and its clear at
// k_lcount, were ~20 us of its 65,536-record epoch).  Each delta is taken with an exchange, so an
// account reached twice is settled once and every delta is 0 again for the next epoch -- also when
// this epoch's pass fell back or was skipped (then nothing is applied).
// (Balances are not inserted into during k_lbalances -- k_lacct's creates are a launch earlier -- so the
// probe takes plain loads: bal_lookup's acquire loads invalidate the CU's caches per instruction, which
// for one active lane per wavefront made this pass 0.48 ms at C3.)
KDEV int32_t bal_find_settled(const DevState& S, int64_t aid) {
    uint32_t h = (uint32_t)mix64((uint64_t)aid) & S.bal_mask;
    for (uint32_t p = 0; p <= S.bal_mask; ++p) {
        const uint32_t st = S.bal_state[h];
        if (st == 0) return -1;
        if (st == 1 && S.bal_key[h] == aid) return (int32_t)h;
        h = (h + 1) & S.bal_mask;
    }
    return -1;
}
KDEV void settle_delta(const DevState& S, const EpochIO& io, int64_t a, bool apply) {
    const int64_t d = (int64_t)atomicExch(reinterpret_cast<KG unsigned long long*>(&S.ldelta[a]), 0ull);
    if (d == 0 || !apply) return;
    const int32_t h = bal_find_settled(S, a);
    if (h < 0) { raise_thread(S.ctr, KME_E_DOMAIN, KME_D_NPE_BALANCE, io.n); return; }   // (cannot happen)
    S.bal_val[h] = jladd(S.bal_val[h], d);
}
// all = 1 (accounts not many more than the epoch's records, C3): one thread per account instead --
// the touched accounts' run heads are then a sparse lane or two per wavefront.
__global__ void __launch_bounds__(256) k_lbalances(DevState S, EpochIO io, int all) {
    const bool apply = !(lskip(S) || lfell(S));
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, T = gridDim.x * blockDim.x;
    if (t == 0 && apply) {   // the positions k_linsert created (its spread counters), and the tables' load, as Core's inserts check it
        unsigned long long grew = 0;
        for (int k = 0; k < LPOSC_LINES; ++k) grew += S.lposc[(size_t)k * CTR_STRIDE];
        const unsigned long long used = S.ctr[ci(C_POS_USED)] + grew;
        S.ctr[ci(C_POS_USED)] = used;
        if (used * 4 > ((unsigned long long)S.pos_mask + 1) * 3 || S.ctr[ci(C_BAL_USED)] * 2 > (unsigned long long)S.bal_mask + 1)
            raise_thread(S.ctr, KME_E_CAPACITY, KME_D_CAP_LEDGER, io.n);
    }
    if (all) {
        for (int64_t a = t; a < S.A; a += T) {
            const int64_t d = S.ldelta[a];
            if (d == 0) continue;
            S.ldelta[a] = 0;
            if (!apply) continue;
            const int32_t h = bal_find_settled(S, a);
            if (h < 0) { raise_thread(S.ctr, KME_E_DOMAIN, KME_D_NPE_BALANCE, io.n); continue; }   // (cannot happen)
            S.bal_val[h] = jladd(S.bal_val[h], d);
        }
        return;
    }
    const uint32_t no = lops(S);
    const KG uint32_t* K = skeys(S);
    for (uint32_t k = t; k < no; k += T) {
        const uint32_t a = K[k] >> S.lhbits;
        if (k == 0 || (K[k - 1] >> S.lhbits) != a) settle_delta(S, io, (int64_t)a, apply);
    }
    if (S.ctr[ci(C_ACCT_OPS)] == 0) return;
    for (uint32_t i = t; i < io.n; i += T) {
        const int64_t a = io.aid[i];
        if (io.action[i] == TRANSFER && a >= 0 && a < S.A) settle_delta(S, io, a, apply);
    }
}

// ---------------------------------------------------------------- launcher
void launch_ledger_parallel(const DevState& S, const EpochIO& io, uint32_t max_trades, hipStream_t st) {
    const uint32_t n = io.n;
    auto cdiv = [](uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); };
    const uint64_t nops = (uint64_t)n + 2ull * max_trades;    // (ops: at most one per arrival number)
    // (lvw_meta and lxmark of the epoch's ops are cleared by k_lgen: the ops fill [0, count) exactly;
    // the value-key table by its tag, S.lvk_tag; the counters and deltas by k_lcount)
    if (n == 0) {
        (void)hipMemsetAsync(S.lctr, 0, sizeof(unsigned long long) * LC_N * CTR_STRIDE, st);
        (void)hipMemsetAsync(S.lposc, 0, sizeof(unsigned long long) * LPOSC_LINES * CTR_STRIDE, st);
        return;
    }
    static_assert(LC_N * CTR_STRIDE <= 256 && LPOSC_LINES * CTR_STRIDE <= 1024, "k_lcount's first threads clear them");
    hipLaunchKernelGGL(k_lcount, dim3(std::max<uint32_t>(cdiv(n, 256), 4)), dim3(256), 0, st, S, io);
    // offsets (in place) and the op count (LC_OPS, low word)
    launch_excl_scan(S.lcnt, S.lcnt, n, S.lscan, reinterpret_cast<uint32_t*>(S.lctr + ci(LC_OPS)), st, S.ctr);
    hipLaunchKernelGGL(k_lgen, dim3(cdiv(n, 256)), dim3(256), 0, st, S, io);
    RadixIO R{};
    R.key0 = reinterpret_cast<const KG int32_t*>(S.lk0);
    R.val0 = nullptr;
    R.keys0 = S.lkey[0]; R.keys1 = S.lkey[1];
    R.vals0 = S.lval[0]; R.vals1 = S.lval[1];
    R.ghist = S.lghist;
    R.rank = nullptr;
    R.pay_src = reinterpret_cast<const KG uint4*>(S.lrec);   // the ops themselves, into sorted order
    R.pay_dst = reinterpret_cast<KG uint4*>(S.lsrt);
    R.none = 0;
    R.n = (uint32_t)nops;
    R.n_dev = S.lctr + ci(LC_OPS);
    R.passes = S.lpasses;
    R.small = n <= (1u << 17) ? 1 : 0;   // (~2 ops per record: the sort is small though nops is a capacity)
    R.tcnt = R.small ? S.ltcnt : nullptr;   // (allocated for engines whose epochs are all small)
    R.lb = R.small ? S.llb : nullptr;
    R.ctr = S.ctr;
    launch_radix(R, st);
    // The passes over the ops are grid-stride loops sized by nops, a capacity (n + 2 max_trades); a
    // small epoch's ops are ~2n (2^19 + n of capacity at the drop-in's defaults: ~4 of 5 blocks found
    // nothing), so its grids are sized by the records instead.
    const uint64_t gops = R.small ? std::min<uint64_t>(nops, std::max<uint64_t>(2ull * n, 65536)) : nops;
    hipLaunchKernelGGL(k_lseg, dim3(cdiv(gops + 1, 256)), dim3(256), 0, st, S);
    // grid of k_lchains / k_linsert: more blocks (their work per thread is a chain of dependent loads:
    // more threads in flight hide it; 8,192 -> 32,768 blocks: k_lchains 0.52 -> 0.42 ms).
    // KME_LEDGER_GRID: A/B runs.
    static const uint32_t grid_cap = [] {
        const char* v = std::getenv("KME_LEDGER_GRID");
        return v ? (uint32_t)std::max(64, std::atoi(v)) : 32768u;
    }();
    // the grid of the grid-stride passes over the ops (KME_LEDGER_GRID_S: A/B runs)
    static const uint32_t grid_s = [] {
        const char* v = std::getenv("KME_LEDGER_GRID_S");
        return v ? (uint32_t)std::max(64, std::atoi(v)) : 8192u;
    }();
    const uint32_t gs = std::min<uint32_t>(cdiv(gops, 256), grid_s), gl = std::min<uint32_t>(cdiv(gops, 256), grid_cap);
    const uint32_t ngap = std::min<uint32_t>(cdiv((uint64_t)S.A + 1, LSEG_RUN) + 1, 1024);   // (k_lseg's gaps)
    hipLaunchKernelGGL(k_lchains, dim3(gl + ngap), dim3(256), 0, st, S, gl);
    hipLaunchKernelGGL(k_ldetect, dim3(gs), dim3(256), 0, st, S);
    hipLaunchKernelGGL(k_lr_rounds, dim3(1), dim3(1024), 0, st, S);
    hipLaunchKernelGGL(k_lvw_classify, dim3(gs), dim3(256), 0, st, S);
    hipLaunchKernelGGL(k_lvw_check, dim3(gs), dim3(256), 0, st, S);
    hipLaunchKernelGGL(k_lcommit, dim3(gs + cdiv(n, 256)), dim3(256), 0, st, S, io, gs);   // (+ the account records)
    hipLaunchKernelGGL(k_linsert, dim3(gl), dim3(256), 0, st, S, io);
    const int all = (uint64_t)S.A <= 4ull * n ? 1 : 0;
    hipLaunchKernelGGL(k_lbalances, dim3(all ? cdiv((uint32_t)S.A, 256) : std::max(gs, cdiv(n, 256))), dim3(256), 0, st, S, io, all);
}

}  // namespace kme
