// kme_device.h -- device-side data layout of the matching core (HBM-resident stores).
//
// The reference keeps five RocksDB stores (KProcessor.java:30-49).  Here the book stores become
// structure-of-arrays in HBM, sized for the 288 GB of an MI355X:
//
//   GroupState[G]        one per symbol group |sid| (books +sid and -sid, KP:184-191; sid 0 is one
//                        shared book, H4): existence, two 128-bit level bitmaps (the Books values,
//                        KP:38-41), the group's node free list and bump chunk.
//   Level[G][2][128]     one per (book side, price level) = the Buckets store (KP:42-45): FIFO
//                        head/tail node slots, resting quantity, tail oid.
//   Node[P]              order-node pool = the Orders store (KP:46-49), one 64-byte line per order.
//   oid table            open-addressing oid -> node slot, one packed u64 per entry (lazy
//                        deletion: entries are validated against the node, stale ones are dropped
//                        at rebuild).
//   ledger               FUNDED: per-account existence + reservation bound; EXACT: Balances and
//                        Positions as device hash tables (KP:30-37).
#pragma once
#include <stddef.h>
#include <stdint.h>

// Pointer members of the device structs live in the global address space (AS1) for the device
// pass: same 64-bit layout as the host's plain pointers, but every access through them compiles to
// global_load / global_store (not flat_*) even when the struct is read from HBM.
#if defined(__HIP_DEVICE_COMPILE__)
#define KG __attribute__((address_space(1)))
#else
#define KG
#endif

namespace kme {

#if defined(__HIPCC__)
#define KDEV_HOST_INLINE __host__ __device__ inline
#else
#define KDEV_HOST_INLINE inline
#endif

constexpr int NLEV = 128;          // price levels 0..126 (+1 pad)
constexpr int NACT = 11;

enum Action : int32_t {
    ADD_SYMBOL = 0, REMOVE_SYMBOL = 1, BUY = 2, SELL = 3, CANCEL = 4, BOUGHT = 5, SOLD = 6,
    REJECT = 7, CREATE_BALANCE = 100, TRANSFER = 101, PAYOUT = 200
};

struct alignas(32) Level {         // one bucket (KP:379-389)
    int32_t head, tail;            // node slots, -1 = none
    int32_t _pad[2];
    int64_t qty;                   // sum of resting sizes (sweep scan, top of book)
    int64_t tail_oid;              // oid of the tail node (OUT.prev on append, KP:217)
};
static_assert(sizeof(Level) == 32, "Level");

struct alignas(64) Node {          // one resting Order (KP:449-458)
    int64_t oid, aid, sid;         // bytes 0..31: what a maker contributes to a trade, one
    int32_t size, next;            //   s_load_dwordx8 in the matching loop
    int64_t prev_oid;              // oid of the previous node in the level (valid when prev >= 0)
    int32_t prev, group;
    int32_t price, action, live, _pad;   // live = word 14 (free-list blocks use words 0..13)
};
static_assert(sizeof(Node) == 64, "Node");

struct alignas(64) GroupState {
    uint64_t bm0_lsb, bm0_msb;     // book +g  (KP:391-404 layout: lsb = prices 0..62, msb = 63..126)
    uint64_t bm1_lsb, bm1_msb;     // book -g
    int32_t exists, free_head, chunk_next, chunk_end;
    int32_t nneg;                  // resting orders of negative size (only the serial engine rests them)
    int32_t _pad[3];
};
static_assert(sizeof(GroupState) == 64, "GroupState");

struct TradeRec {                  // == kme_trade
    int64_t moid, maid, msid;
    int32_t mprice, size;
};
static_assert(sizeof(TradeRec) == 32, "TradeRec");

struct TradeTmp {                  // unordered trade scratch written by the group wavefronts, two
    int64_t moid, maid;            // 16-B parts (one store each): the maker, then
    int32_t seq;                   //   the taker's input index (-1: a hole k_scatter skips),
    uint32_t ordp;                 //   the trade's ordinal | maker price << 23 | (maker sid < 0) << 30,
    int32_t size, group;           //   the size and the symbol group (the maker's sid is +-group)
};
static_assert(sizeof(TradeTmp) == 32, "TradeTmp");
constexpr uint32_t TT_ORD_BITS = 23;       // a record's trade ordinals (OS_MAX_NTR) fit
constexpr uint32_t FAST_RANK_SHIFT = 20;   // fast segments: ordinal = index | event rank << 20
constexpr int FAST_LVB = 7;                // lvbase words per record: event ranks 1..7 (a sweep over <= 7 levels)
KDEV_HOST_INLINE uint32_t tt_ordp(uint32_t ord, int32_t price, bool sneg) {
    return ord | ((uint32_t)price << TT_ORD_BITS) | (sneg ? 1u << 30 : 0u);
}

// Positions: UUID(aid,sid) -> UUID(amount,available), with the slot's state (0 empty, 1 live, 2
// tombstone) in the same 64-byte line: a probe or an insert touches one line
struct alignas(64) PosEntry {
    int64_t k0, k1, v0, v1;
    uint32_t state;
    uint32_t _pad[7];
};
static_assert(sizeof(PosEntry) == 64, "PosEntry");

// kme_ledger.hip: one position chain of an epoch (the ops on Positions key (aid, sid)), stored at the
// sorted position of its first op (aid -1 there: that op is not a chain's first)
struct alignas(64) LChain {         // one 64-byte line: the head's store is one whole-line write
    int64_t fa, fv;                // after the chain's last effect (fpres)
    int64_t delta;                 // the balance change of its effects
    uint64_t late;                 // (1 + arrival number) << 32 | op position of the latest value write
                                   // into it after its last effect (0: none)
    int32_t sid, aid;
    uint32_t last_seq;             // arrival number of its last effect
    uint32_t dirty;                // in the repair rounds' run list (a value write into it preceded one of its reads)
    uint32_t rix;                  // 1 + the coupling list index of its first incoming value write (this round)
    int32_t islot;                 // the entry's table slot at the start (its value there then: the chain's
                                   // start state, unchanged until k_lcommit); absent (ipres 0): the first
                                   // free slot of its probe sequence (-1: none), fst that slot's state
    uint8_t ipres, fpres, fst, _p;
    uint32_t _pad;
};
static_assert(sizeof(LChain) == 64, "LChain");
// One ledger effect of the epoch (kme_ledger.hip): checkBalance, a fill, or postRemoveAdjustments on
// the position (aid, sid) -- the account is the op's sort key -- with its arrival number.  FUNDED
// sids are symbol groups (|sid| < max_symbols < 2^30) and prices 0..126, so both fit narrow fields.
struct LOp {
    int32_t sid;
    uint32_t es;                   // arrival number
    int32_t size;
    int16_t price;                 // the effect's price term
    uint16_t flags;                // kind (check / fill / cancel) | buy << 2
};
static_assert(sizeof(LOp) == 16 && offsetof(LOp, price) == 12 && offsetof(LOp, flags) == 14, "LOp (k_lgen packs it)");
// the ledger pass's counters (DevState::lctr, one line each)
enum LCtr : int { LC_OPS = 0, LC_DIRTY, LC_CROSS, LC_FALLBACK, LC_REPAIRED, LC_CHG, LC_DONE, LC_GAPS, LC_N = 8 };

// Counters block: one u64 per 128-byte line (ci(k) = word index), so that atomics on different
// counters never contend for one L2 line.
enum Ctr : int {
    C_ERR = 0,         // (index << 16) | (detail << 8) | status; UINT64_MAX = none
    C_TRADES, C_RESTS, C_VISITS, C_CANCEL_OK, C_ORDERS,
    C_TTMP,            // trade scratch records reserved in the overflow region
    C_POOL_BUMP,       // pool slots handed out in chunks
    C_OTAB_USED,       // non-empty oid-table slots
    C_ACCT_OPS,        // FUNDED: account records in the epoch
    C_BAL_USED, C_POS_USED,
    C_FALLBACK,        // FUNDED + KME_FLAG_SERIAL_FALLBACK: nonzero = this epoch runs serially
    C_BUSY,            // FUNDED: groups k_match took this epoch (the host's stream choice for the next)
    C_REBUILD_FAIL,    // oid-table rebuild: entries that found no slot (persistent, zeroed by the rebuild)
    C_LIGHT,           // FUNDED: k_match_lanes wavefronts that had a group this epoch (the next one's launch)
    C_SIZE0,           // persistent: nonzero once a BUY/SELL of size 0 was submitted (a book may then hold
                       // size-0 makers, and k_match's fast segments -- which read a level's emptiness off
                       // its quantity -- stay off)
    C_LREPAIRED,       // exact ledger: position chains the parallel pass replayed for value-key couplings
    C_LSERIAL,         // exact ledger: nonzero = the serial replay applied this epoch's ledger
    C_GLIST,           // FUNDED, list mode: groups k_segments listed for k_match_list (glist)
    C_ODD,             // persistent: nonzero once the serial engine made a book the FUNDED matchers cannot
                       // take (a level above price 100, a negative-size order: GroupState::nneg)
    C_NCTR = 21
};
constexpr int CTR_STRIDE = 16;                 // u64 words per counter line
constexpr int ci(int k) { return k * CTR_STRIDE; }
// Trade scratch shards (k_match -> k_scatter): shard s = group & (TSHARDS - 1) reserves records
// in its own region [s * tshard_cap, (s + 1) * tshard_cap) through its own counter line; a shard
// that runs full spills to the overflow region behind them (counter C_TTMP).
constexpr int TSHARDS = 256;
enum TShardWord : int { TS_USED = 0, TS_RESTS = 1, TS_CANCELS = 2, TS_LIGHT = 3 };


struct DevState {
    int32_t G, mode, A, passes;
    int32_t ledger_replay;            // FUNDED + KME_FLAG_EXACT_LEDGER
    int32_t light_max;                // FUNDED: groups with at most this many records in the epoch
                                      // run in k_match_lanes (one lane each); 0 = none
    int32_t fallback;                 // KME_FLAG_SERIAL_FALLBACK
    int32_t fast;                     // k_match fast segments on (env KME_FAST=0: off, for A/B runs)
    uint32_t pool_cap, otab_mask, credit_div, ttmp_cap;     // ttmp_cap: overflow region records
    uint32_t bal_mask, pos_mask, trades_cap, tshard_cap;
    uint32_t os_base, _pad1;          // osort records (= max_epoch)
    KG GroupState* grp;
    KG Level* lev;
    KG Node* pool;
    KG uint64_t* otab;                // oid -> node slot, packed entries (kme_kernels.hip "oid tables")
    // FUNDED ledger
    KG int64_t* acct_since;
    KG int64_t* acct_lb;
    KG int64_t* acct_need;
    KG int64_t* acct_negx;
    KG int64_t* acct_xfer;
    KG int64_t* acct_demand;          // sum of the epochs' need on this engine (credit re-splitting weights)
    // EXACT ledger
    KG uint32_t* bal_state;
    KG int64_t* bal_key;
    KG int64_t* bal_val;
    KG PosEntry* pos;
    // per-epoch scratch
    KG uint32_t* epos;                // oid-table position of this epoch's BUY/SELL i (k_emap -> k_table)
    KG int32_t* route_grp;
    KG int64_t* cancel_tgt;           // EXACT: cancel target (FUNDED: in the packed record)
    KG int32_t* rest_slot;
    KG uint32_t* lvbase;              // FUNDED: fast segments' per-record trade bases of event ranks 1..FAST_LVB
    KG int4* vic;                     // FUNDED + exact ledger: per accepted cancel, the removed order
                                      // (price | action << 8, size, sid) for postRemoveAdjustments
    KG int4* prec;                    // FUNDED: packed records, 32 B each (k_route -> k_match):
                                      // w0 = action | price << 8 | acct_ok << 16 | (sid < 0) << 17,
                                      // size, oid, aid, cancel target (slot | -(j + 2) | -1), the
                                      // target's level (price | side << 8 | 1 << 9; 0 = unknown)
    KG int4* osort;                   // FUNDED: the OUT echo of the matched records, 16 B each
                                      // (action | has_prev << 8 | n_trades << 9, size, prev) at the
                                      // record's input index; k_unsort spreads it over the SoA results
    KG int32_t* rank;                 // sorted position of input i (last partition pass), when allocated
                                      // (nullptr: nothing reads it)
    KG uint32_t* rkeys[2];
    KG uint32_t* rvals[2];
    KG uint32_t* ghist;
    KG uint32_t* rtcnt;               // small partition sorts: per-tile digit counts of every pass (RadixIO::tcnt)
    KG unsigned long long* rlb;       // and their look-back words (RadixIO::lb)
    KG uint32_t* seg;
    KG uint32_t* gflag;               // per group: 1 = k_match takes it this epoch (then its scanned offset)
    KG uint32_t* glist;               // those groups, in id order (k_match's dense grid); gcount[0] = how many.
                                      // List mode: the groups k_segments found busy, C_GLIST of them, any order
    KG uint32_t* gcount;
    KG TradeTmp* ttmp;                // TSHARDS regions of tshard_cap, then the overflow region
    KG unsigned long long* tsh;       // TSHARDS x CTR_STRIDE words (TShardWord in each line)
    KG unsigned long long* ctr;       // C_NCTR x CTR_STRIDE words
    KG unsigned long long* dbg;     // diagnostic stamps (KME_STAMPS builds), G x 16 words
    // FUNDED + exact ledger, applied in parallel (kme_ledger.hip; lpar = 0: the serial replay)
    int32_t lpar, lpasses, lhbits, _lpad2;
    uint32_t lr_cap, lx_cap, lc_cap, lrounds;
    uint64_t lvk_mask;
    uint32_t lvk_tag, _lpad3;         // this epoch's tag in the value-key table (1..65535: no per-epoch clear)
    KG uint32_t* lcnt;                // per record: its ops, then their offset
    KG uint32_t* lscan;               // scan scratch
    KG uint32_t* lk0;                 // per op (arrival order): sort key aid << 8 | hash8(sid)
    KG uint32_t* lkey[2];
    KG uint32_t* lval[2];
    KG uint32_t* lghist;
    KG uint32_t* ltcnt;               // the op sort's look-back buffers (small epochs; nullptr: none)
    KG unsigned long long* llb;
    KG LOp* lrec;                     // per op, arrival order
    KG LOp* lsrt;                     // per op, sorted order (k_lseg gathers them once)
    KG LChain* lchain;                // per sorted op (written at chain heads only)
    KG uint8_t* lhead;                // per sorted op: 1 = it heads its chain
    KG long4* lvw;                    // per sorted op: its value write (key, value)
    KG uint32_t* lvw_meta;            //   kind | writer chain << 2
    KG int32_t* lvw_tgt;              //   the chain it writes into (-1: none)
    KG uint32_t* lseg;                // per account: its first sorted op
    KG uint4* lgap;                   // k_lseg: account gaps longer than LSEG_RUN (first, last, op position)
    KG int64_t* ldelta;               // per account: the epoch's balance change
    KG ulonglong4* lvk;               // value-key table: hash, 1 + latest arrival, key
    KG uint32_t* lx;                  // couplings: the ops whose value writes go into chains that read later
    KG uint32_t* lxn;                 //   per coupling: 1 + the next one into the same chain (this round)
    KG uint8_t* lxmark;               // per sorted op: listed in lx
    KG uint32_t* lrun;                // the repair rounds' run list (chain heads)
    KG uint32_t* lchg;                // the value writes a repair round changed
    KG unsigned long long* lctr;      // LC_N x CTR_STRIDE words
    KG unsigned long long* lposc;     // 64 x CTR_STRIDE words: positions k_linsert created (k_lbalances folds them)
    // Sparse symbols: the reference takes any long sid (KP:184-191, 201).  Groups G .. G + Gs - 1 of the
    // stores above hold symbols with |sid| >= G, named by gsid (open addressing on |sid|, slot k =
    // group G + k, 0 = free).  Only the serial engine (k_serial) touches them: a FUNDED epoch with a
    // record on one runs serially (KME_FLAG_SERIAL_FALLBACK).
    int32_t Gs;
    int32_t refuse;                   // KME_FLAG_REFUSE_SERIAL: what needs the serial engine is refused
                                      // as an unproven epoch instead (kme_multi's shards)
    KG int64_t* gsid;
};

struct EpochIO {
    const KG int32_t* action;
    const KG int64_t* oid;
    const KG int64_t* aid;
    const KG int64_t* sid;
    const KG int32_t* price;
    const KG int32_t* size;
    KG int32_t* out_action;
    KG int32_t* out_size;
    KG int64_t* out_prev;
    KG uint8_t* out_flags;
    KG uint32_t* n_trades;
    KG uint32_t* trade_off;
    KG TradeRec* trades;
    uint32_t n;
    uint32_t trades_cap;
    int64_t seq_base;
    uint32_t _pad0, _pad;
};

}  // namespace kme
