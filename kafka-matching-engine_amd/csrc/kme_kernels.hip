// kme_kernels.hip -- CDNA4 (gfx950) kernels of the epoch pipeline.
//
// Reference path: KProcessor.MatchingEngine.process -> addOrder / tryMatch / removeOrder
// (/root/reference/src/main/java/KProcessor.java:96-333, "KP").  The reference handles one record
// at a time against RocksDB stores; here one epoch of records is handled per launch sequence:
//
//   FUNDED mode (symbol groups in parallel)
//     k_emap        oid -> input map of the epoch's BUY/SELL; per-account reservation bound
//     k_ledger      account records (CREATE_BALANCE / TRANSFER, KP:131-146) in arrival order
//     k_check       per-account proof that every checkBalance (KP:167-182) passes
//     k_route       symbol group of every record; cancel target (KP:290) via oid table / epoch map
//     k_radix_*     (1) stable LSD radix partition of the epoch by symbol group (arrival order kept)
//     k_match       (2) one wavefront per symbol group: price-time matching (KP:200-263) and
//                   cancels (KP:289-323), touched price levels staged in LDS
//     k_scan_* +    (4) exclusive scan of per-input trade counts (DPP wave scans) and a
//     k_scatter     coalesced scatter of the trades into arrival order
//     k_table       oid table maintenance for the orders that came to rest
//   EXACT mode: k_emap + k_route + k_serial (one wavefront replays the epoch in arrival order with
//   the full ledger, including the value-keyed Positions writes of KP:434-436) + k_table.
//
// Wavefront-uniform code: in the group/serial kernels all 64 lanes run the same scalar program
// (values land in SGPRs); atomics are issued by lane 0 only and broadcast.
#include <hip/hip_runtime.h>

#include <atomic>

#include <algorithm>

#include "kme.h"
#include "kme_device.h"
#include "kme_jarith.h"
#include "kme_launch.h"

namespace kme {



// Diagnostic build only (-DKME_STAMPS): s_memtime stamps accumulated per category in SGPRs and
// written to DevState::dbg at the end of k_match (cdna_hip_programming.md §7 "In-kernel stamps").
// Quote the shares, not the run time, of that build.
#ifdef KME_STAMPS
KDEV unsigned long long stamp() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define KST(x) x
#else
#define KST(x)
#endif
// -DKME_LANE_STAMPS: the same for k_match_lanes, per wavefront step (every lane's step shares the
// wavefront's timeline): drain of the previous step's vector operations, first gather, second
// gather, the record (try_match, rest), the OUT echo; each segment ends with an explicit wait, so
// the build serialises what the product build overlaps (quote shares, not times).
#ifdef KME_LANE_STAMPS
KDEV unsigned long long lstamp() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define LST(...) __VA_ARGS__
#else
#define LST(...)
#endif
// Broadcast lane 0's value with readfirstlane (SGPR result): the compiler then knows it is
// wave-uniform.  (__shfl lowers to ds_bpermute, whose result the divergence analysis treats as
// per-lane; everything computed from it would turn into exec-masked VALU code.)
KDEV unsigned long long bcast64(unsigned long long v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return ((unsigned long long)hi << 32) | lo;
}

// ------------------------------------------------------------------ the book bit scans (KP:359-416)
// getFirstSetBitPos / getLastSetBitPos compute (int)(Math.log10(x) / Math.log10(2)) in double.
// Integer restatement: ctz / clz, the NaN path of a negative argument (-> 0), and the overshoot
// of log10 rounding for h >= 47 (h + 1 once n >= 2^(h+1) - D[h]; D[] from
// tools/gen_log10_table.py under a correctly rounded log10).  No floating point on the device.
// D[h - 47] for h = 47..62, 16 bits each, four per word: register-only (a table in memory put an
// SMEM load and its lgkmcnt wait on every bid-side scan of the matching loop).
constexpr uint64_t kLog10D0 = 0x0007000300020001ull, kLog10D1 = 0x00b2005a001c000eull, kLog10D2 = 0x09df051002970154ull, kLog10D3 = 0x8a0046ff248012bfull;

KDEV int32_t first_set_bit_pos(uint64_t n) {          // KP:371-373, n != 0
    uint64_t low = n & (0ull - n);
    if (low == (1ull << 63)) return 0;
    return (int32_t)__builtin_ctzll(n);
}
KDEV int32_t last_set_bit_pos(uint64_t n) {           // KP:375-377, n != 0
    if ((int64_t)n < 0) return 0;
    int32_t h = 63 - (int32_t)__builtin_clzll(n);
    if (h >= 47) {
        const uint64_t r = (2ull << h) - n;              // n >= 2^(h+1) - D[h]  <=>  r <= D[h]
        if (r <= 35328) {
            const uint32_t k = (uint32_t)(h - 47);
            const uint64_t w = k < 8 ? (k < 4 ? kLog10D0 : kLog10D1) : (k < 12 ? kLog10D2 : kLog10D3);
            if (r <= ((w >> (16 * (k & 3))) & 0xFFFFull)) h += 1;
        }
    }
    return h;
}
KDEV int32_t min_price_ptr(uint64_t lsb, uint64_t msb) {   // KP:359-363
    if (lsb == 0 && msb == 0) return -1;
    if (lsb == 0) return jiadd(first_set_bit_pos(msb), 63);
    return first_set_bit_pos(lsb);
}
KDEV int32_t max_price_ptr(uint64_t lsb, uint64_t msb) {   // KP:365-369
    if (msb == 0 && lsb == 0) return -1;
    if (msb == 0) return last_set_bit_pos(lsb);
    return jiadd(last_set_bit_pos(msb), 63);
}
KDEV bool check_bit(uint64_t lsb, uint64_t msb, int32_t price) {  // KP:391-394, 406-408
    return price < 63 ? ((lsb >> (price & 63)) & 1ull) : ((msb >> (jisub(price, 63) & 63)) & 1ull);
}
KDEV void set_bit(uint64_t& lsb, uint64_t& msb, int32_t price) {   // KP:396-399, 410-412
    if (price < 63) lsb |= 1ull << (price & 63); else msb |= 1ull << (jisub(price, 63) & 63);
}
KDEV void unset_bit(uint64_t& lsb, uint64_t& msb, int32_t price) { // KP:401-404, 414-416
    if (price < 63) lsb &= ~(1ull << (price & 63)); else msb &= ~(1ull << (jisub(price, 63) & 63));
}
// |sid| as a symbol-group index, or -1 when outside [0, G).
KDEV int32_t group_of(int64_t sid, int32_t G) {
    if (sid == INT64_MIN) return -1;
    int64_t a = sid < 0 ? -sid : sid;
    return a < (int64_t)G ? (int32_t)a : -1;
}
// A record only the serial engine takes (a BUY/SELL priced outside 0..100 or of negative size, an
// account id outside [0, A), a sparse symbol, a book holding such an order): with
// KME_FLAG_SERIAL_FALLBACK the epoch runs serially (k_serial, as an unprovable one); with
// KME_FLAG_REFUSE_SERIAL it is refused as unproven -- nothing of it takes effect, KME_E_UNFUNDED at
// index 0 (kme_multi then hands the stream to its consolidated engine).
KDEV bool serial_capable(const DevState& S) { return S.fallback || S.refuse; }
KDEV void need_serial(const DevState& S) {
    if (S.fallback) { if (!S.ctr[ci(C_FALLBACK)]) atomicOr(&S.ctr[ci(C_FALLBACK)], 1ull); }
    else raise_thread(S.ctr, KME_E_UNFUNDED, KME_D_UNPROVEN, 0);
}
// a cancel of an order of this epoch on a symbol the parallel path cannot name (a sparse one): its
// group is resolved by k_serial (route_grp; the target stays in cancel_tgt)
constexpr int32_t GRP_RESOLVE = -3;

// ------------------------------------------------------------------ DPP wavefront scans
// Inclusive scan over 64 lanes: row_shr 1,2,4,8 inside each 16-lane row, then row_bcast:15 and
// row_bcast:31 carry the row totals (gfx9-family DPP controls, available on gfx950).
KDEV uint32_t dpp_shr(uint32_t x, int n) {
    switch (n) {
    case 1: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);
    case 2: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true);
    case 4: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true);
    default: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);
    }
}
KDEV uint32_t wave_incl_scan_u32(uint32_t x) {
    x += dpp_shr(x, 1);
    x += dpp_shr(x, 2);
    x += dpp_shr(x, 4);
    x += dpp_shr(x, 8);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return x;
}
KDEV uint64_t dpp64(uint64_t x, int ctrl_sel) {
    int lo = (int)(uint32_t)x, hi = (int)(uint32_t)(x >> 32);
    int rlo, rhi;
    switch (ctrl_sel) {
    case 1: rlo = __builtin_amdgcn_update_dpp(0, lo, 0x111, 0xf, 0xf, true); rhi = __builtin_amdgcn_update_dpp(0, hi, 0x111, 0xf, 0xf, true); break;
    case 2: rlo = __builtin_amdgcn_update_dpp(0, lo, 0x112, 0xf, 0xf, true); rhi = __builtin_amdgcn_update_dpp(0, hi, 0x112, 0xf, 0xf, true); break;
    case 4: rlo = __builtin_amdgcn_update_dpp(0, lo, 0x114, 0xf, 0xf, true); rhi = __builtin_amdgcn_update_dpp(0, hi, 0x114, 0xf, 0xf, true); break;
    case 8: rlo = __builtin_amdgcn_update_dpp(0, lo, 0x118, 0xf, 0xf, true); rhi = __builtin_amdgcn_update_dpp(0, hi, 0x118, 0xf, 0xf, true); break;
    case 15: rlo = __builtin_amdgcn_update_dpp(0, lo, 0x142, 0xa, 0xf, false); rhi = __builtin_amdgcn_update_dpp(0, hi, 0x142, 0xa, 0xf, false); break;
    default: rlo = __builtin_amdgcn_update_dpp(0, lo, 0x143, 0xc, 0xf, false); rhi = __builtin_amdgcn_update_dpp(0, hi, 0x143, 0xc, 0xf, false); break;
    }
    return ((uint64_t)(uint32_t)rhi << 32) | (uint32_t)rlo;
}
KDEV int64_t wave_incl_scan_i64(int64_t v) {
    uint64_t x = (uint64_t)v;
    x += dpp64(x, 1); x += dpp64(x, 2); x += dpp64(x, 4); x += dpp64(x, 8);
    x += dpp64(x, 15); x += dpp64(x, 31);
    return (int64_t)x;
}

// ------------------------------------------------------------------ oid tables
// Both tables (oid -> resting node slot; oid -> input index of this epoch's BUY/SELL) are linear-
// probing arrays of packed u64 entries ((fingerprint | 1) << 32 | value, 0 = empty): one 8-byte
// word per probe, inserted with one CAS.  The fingerprint is a second hash of the oid; a match is
// confirmed against the oid itself (the node's, or the epoch input's), so a fingerprint collision
// costs a probe, never a wrong answer.  Stale node entries (lazy deletion) fail that check too.
KDEV uint32_t oid_fp(int64_t oid) { return (uint32_t)(mix64((uint64_t)oid ^ 0x9e3779b97f4a7c15ull) >> 32) | 1u; }
KDEV uint64_t hentry(uint32_t fp, uint32_t v) { return ((uint64_t)fp << 32) | v; }

// Entry values: a node slot (< 2^31); OT_PENDING | i for BUY/SELL i of the epoch in flight (k_emap
// inserts every BUY/SELL; the entry becomes the order's rest slot when it rests -- k_unsort, or
// k_table for EXACT / serial epochs, which also mark the others OT_DEAD), so one table answers both
// "an earlier order of this epoch" and "a resting order".  A FUNDED order that did not rest keeps
// its pending entry until the next rebuild; a pending entry is only ever read as "record j of the
// current epoch is a BUY/SELL with this oid", which the reader checks against the epoch's input.
constexpr uint32_t OT_PENDING = 0x80000000u;
constexpr uint32_t OT_DEAD = 0xFFFFFFFFu;

// A resting order's slot (a live node with this oid), or -1.
KDEV int32_t otab_lookup(const DevState& S, int64_t oid) {
    const uint32_t fp = oid_fp(oid);
    uint32_t h = (uint32_t)mix64((uint64_t)oid) & S.otab_mask;
    for (uint32_t probes = 0; probes <= S.otab_mask; ++probes) {
        const uint64_t e = S.otab[h];
        if (e == 0) return -1;
        const uint32_t v = (uint32_t)e;
        if ((uint32_t)(e >> 32) == fp && !(v & OT_PENDING)) {
            if (S.pool[v].live && S.pool[v].oid == oid) return (int32_t)v;
        }
        h = (h + 1) & S.otab_mask;
    }
    return -1;
}
// removeOrder's orders.get(oid) at input i (KP:290): an order of this epoch submitted before i
// (returns -(j + 2)), else a resting order's slot, else -1.  What the caller needs of the target comes
// with the check that finds it, one round trip per probe: a resting order's whole node (nd), an
// order of this epoch's sid and price (jsid, jprice).
KDEV int64_t otab_cancel_target(const DevState& S, const EpochIO& io, int64_t oid, uint32_t i, uint32_t& pos, Node& nd,
                                int64_t& jsid, int32_t& jprice) {
    const uint32_t fp = oid_fp(oid);
    uint32_t h = (uint32_t)mix64((uint64_t)oid) & S.otab_mask;
    for (uint32_t probes = 0; probes <= S.otab_mask; ++probes) {
        const uint64_t e = S.otab[h];
        if (e == 0) return -1;
        const uint32_t v = (uint32_t)e;
        if ((uint32_t)(e >> 32) == fp && v != OT_DEAD) {
            if (v & OT_PENDING) {   // (possibly an earlier epoch's: it counts only as a fact of this one)
                const uint32_t j = v & ~OT_PENDING;
                if (j < i) {
                    const int64_t joid = io.oid[j];
                    const int32_t ja = io.action[j];
                    jsid = io.sid[j];
                    jprice = io.price[j];
                    if (joid == oid && (ja == BUY || ja == SELL)) { pos = h; return -((int64_t)j + 2); }
                }
            } else if (v < S.pool_cap) {
                nd = S.pool[v];
                if (nd.live && nd.oid == oid) return (int64_t)v;
            }
        }
        h = (h + 1) & S.otab_mask;
    }
    return -1;
}
KDEV bool otab_insert(const DevState& S, int64_t oid, int32_t slot) {
    const unsigned long long ent = hentry(oid_fp(oid), (uint32_t)slot);
    uint32_t h = (uint32_t)mix64((uint64_t)oid) & S.otab_mask;
    for (uint32_t probes = 0; probes <= S.otab_mask; ++probes) {
        if (atomicCAS((unsigned long long*)&S.otab[h], 0ull, ent) == 0) return true;
        h = (h + 1) & S.otab_mask;
    }
    return false;
}

// A BUY/SELL's pending entry (k_emap) becomes its rest slot, or OT_DEAD when it did not rest: the
// entry's low word only (the fingerprint stays).  FUNDED: k_unsort stores it from rest_slot.
KDEV void otab_final(decltype(DevState::otab) otab, int32_t h, int32_t slot) {
    if (h >= 0) reinterpret_cast<KG uint32_t*>(otab)[2 * (size_t)h] = slot >= 0 ? (uint32_t)slot : OT_DEAD;
}

// DevState::rest_slot[i] of BUY/SELL i of the epoch: RS_PENDING (k_route) until the order rests,
// then its rest slot; once the matcher has passed i, RS_PENDING means it did not rest (a reader is a
// later record of the same group: arrival order).  The matchers store there
// (a 4-byte store into an array of the epoch's size, which stays in the Infinity Cache) instead of
// into the oid table's random line (a partial-line write to HBM in the middle of the record loop);
// a same-epoch cancel reads its target's final slot there (the matchers take a group's records in
// arrival order), and k_unsort copies the epoch's finals into the oid table in one streaming pass.
constexpr int32_t RS_PENDING = -2;

// ------------------------------------------------------------------ epoch kernels: emap / ledger / route
// Sum of a per-thread count over a 256-thread block (DPP wave scans, then LDS); valid in thread 0.
KDEV uint32_t block_sum_256(uint32_t v, uint32_t* red) {
    const uint32_t w = wave_incl_scan_u32(v);
    if ((threadIdx.x & 63) == 63) red[threadIdx.x >> 6] = w;
    __syncthreads();
    const uint32_t t = red[0] + red[1] + red[2] + red[3];
    __syncthreads();
    return t;
}
// Grid of the streaming epoch kernels: enough 256-thread blocks to fill the chip several times,
// each thread striding over the epoch; counters are summed per block and added once per block
// (a counter hit by one atomic per wavefront serialises the whole kernel on its L2 line).
constexpr uint32_t STREAM_BLOCKS = 2048;

KDEV void write_out(const EpochIO& io, uint32_t i, int32_t action, bool ok, int32_t size, bool has_prev, int64_t prev) {
    io.out_action[i] = ok ? action : (int32_t)REJECT;
    io.out_size[i] = size;
    io.out_prev[i] = has_prev ? prev : 0;
    io.out_flags[i] = has_prev ? (uint8_t)KME_OUT_HAS_PREV : (uint8_t)0;
}

#ifndef KME_DIAG_EMAP_NOCAS
#define KME_DIAG_EMAP_NOCAS 0     // diagnostic builds only: 1 = one oid-table probe per BUY/SELL, 2 = none
#endif
#ifndef KME_DIAG_EMAP_NOPREC
#define KME_DIAG_EMAP_NOPREC 0    // diagnostic builds only: no packed-record stores
#endif
#ifndef KME_DIAG_EMAP_NONEED
#define KME_DIAG_EMAP_NONEED 0    // diagnostic builds only: no per-account need accumulation
#endif
// BUY/SELL oid -> input index of this epoch; duplicate / sentinel oid checks; FUNDED: range domain
// and per-account reservation need (max over adj of checkBalance's risk, KP:172-176).
__global__ void __launch_bounds__(256) k_emap(DevState S, EpochIO io, int funded, EpochIO* io_dev) {
    __shared__ uint32_t red[4];
    const uint32_t t0 = blockIdx.x * blockDim.x + threadIdx.x;
    if (t0 == 0) *io_dev = io;   // the group / serial kernels read the epoch descriptor from HBM
    uint32_t n_orders = 0, n_acct = 0, n_ins = 0;
    for (uint32_t i = t0; i < io.n; i += gridDim.x * blockDim.x) {
        const int32_t a = io.action[i];
        n_orders += (a == BUY || a == SELL || a == CANCEL) ? 1u : 0u;
        if ((a == BUY || a == SELL) && io.size[i] <= 0 && !S.ctr[ci(C_SIZE0)]) atomicOr(&S.ctr[ci(C_SIZE0)], 1ull);
        if (a == BUY || a == SELL) {
            // the order's oid-table entry (pending until k_table); on the way, the duplicate-oid
            // guard: another BUY/SELL of this epoch, or a live resting order, with this oid
            // (KP:221 would overwrite it and corrupt its level's list)
            const int64_t oid = io.oid[i];
            const uint32_t fp = oid_fp(oid);
            const unsigned long long ent = hentry(fp, OT_PENDING | i);
            uint32_t h = (uint32_t)mix64((uint64_t)oid) & S.otab_mask;
            bool placed = false, adopted = false;
            uint32_t pos = OT_DEAD;
            for (uint32_t probes = 0; KME_DIAG_EMAP_NOCAS < 2 && probes <= (KME_DIAG_EMAP_NOCAS ? 0u : S.otab_mask); ++probes) {
                // (after adopting an entry: plain loads, the rest of the probe only looks for duplicates)
                const unsigned long long prev = adopted ? (unsigned long long)S.otab[h] : atomicCAS((unsigned long long*)&S.otab[h], 0ull, ent);
                if (prev == 0) {
                    if (!adopted) { pos = h; placed = true; }
                    break;
                }
                if (prev == ent && !adopted) {
                    // an earlier epoch's pending entry of record i with this fingerprint (an order of
                    // that epoch that did not rest, the same oid again at the same index): it becomes
                    // this order's entry.  A second one further on would be the one k_route's cancel
                    // probe finds after the first -- k_match_lanes then read a never-finalised entry.
                    pos = h; placed = adopted = true;
                    h = (h + 1) & S.otab_mask;
                    continue;
                }
                const uint32_t v = (uint32_t)prev;
                if ((uint32_t)(prev >> 32) == fp && v != OT_DEAD) {
                    if (v & OT_PENDING) {   // (an earlier epoch's entry counts only as a fact of this
                        const uint32_t j = v & ~OT_PENDING;   // one: a BUY/SELL j != i with this oid)
                        if (j != i && j < io.n && io.oid[j] == oid && (io.action[j] == BUY || io.action[j] == SELL)) {
                            // the later of the two is the fault; the earlier one takes effect and
                            // keeps its entry (cancels before the fault must find it), so it goes on
                            // probing past a later one that got there first
                            raise_thread(S.ctr, KME_E_DOMAIN, KME_D_DUP_OID, i > j ? i : j);
                            if (j < i) break;
                        }
                    } else if (S.pool[v].live && S.pool[v].oid == oid) {
                        raise_thread(S.ctr, KME_E_DOMAIN, KME_D_DUP_OID, i);
                        break;
                    }
                }
                h = (h + 1) & S.otab_mask;
            }
            S.epos[i] = pos;
            if (placed && !adopted) ++n_ins;
            if (funded) {
                const int32_t price = io.price[i], size = io.size[i];
                const int64_t aid = io.aid[i];
                const bool aid_in = aid >= 0 && aid < S.A;
                // outside the parallel path's domain: prices 0..100, sizes >= 0 (the proof's risk
                // bound, KP:172-176; the matchers' level staging), dense account and symbol ids
                const bool range_bad = price < 0 || price > 100 || size < 0;
                if (S.fallback && (!aid_in || (S.Gs > 0 && group_of(io.sid[i], S.G) < 0))) need_serial(S);
                if (range_bad) {
                    if (serial_capable(S)) need_serial(S);
                    else raise_thread(S.ctr, KME_E_DOMAIN, KME_D_FUNDED_RANGE, i);
                } else if (aid_in && !KME_DIAG_EMAP_NONEED) {   // the account's reservation need
                    const int64_t risk = (a == BUY) ? (int64_t)size * price : (int64_t)size * (100 - price);
                    atomicAdd((unsigned long long*)&S.acct_need[aid], (unsigned long long)risk);
                }
                // k_route's work for the order, done here while its fields are in registers (the
                // streaming stores overlap this kernel's atomics): symbol group, the packed record
                // with the order's oid-table position, or the books.get == null reject (KP:202-203).
                // acct_ok reads the accounts as they stand before this epoch's account records;
                // k_route redoes it when the epoch has some (C_ACCT_OPS).
                const int64_t sid = io.sid[i];
                const int32_t grp = group_of(sid, S.G);
                S.route_grp[i] = grp;
                if (grp < 0) {
                    write_out(io, i, a, false, size, false, 0);
                } else {
                    const bool acct_ok = aid >= 0 && aid < S.A && S.acct_since[aid] < io.seq_base + (int64_t)i;
                    const int32_t w0 = (a & 0xFF) | ((price & 0xFF) << 8) | ((acct_ok ? 1 : 0) << 16) | ((sid < 0 ? 1 : 0) << 17);
                    KG int4* p = &S.prec[2 * (size_t)i];
                    if (!KME_DIAG_EMAP_NOPREC) {
                        p[0] = make_int4(w0, size, (int32_t)(uint32_t)oid, (int32_t)((uint64_t)oid >> 32));
                        p[1] = make_int4((int32_t)(uint32_t)aid, (int32_t)((uint64_t)aid >> 32), placed ? (int32_t)pos : -1, 0);
                    }
                }
            }
        } else if (funded && (a == CREATE_BALANCE || a == TRANSFER)) {
            ++n_acct;
        }
    }
    const uint32_t no = block_sum_256(n_orders, red);
    const uint32_t na = block_sum_256(n_acct, red);
    const uint32_t ni = block_sum_256(n_ins, red);
    if (threadIdx.x == 0) {
        if (no) atomicAdd(&S.ctr[ci(C_ORDERS)], (unsigned long long)no);
        if (na) atomicAdd(&S.ctr[ci(C_ACCT_OPS)], (unsigned long long)na);
        if (ni) atomicAdd(&S.ctr[ci(C_OTAB_USED)], (unsigned long long)ni);
    }
}

// FUNDED account records in arrival order (one wavefront; skipped when the epoch has none).
// createBalance KP:131-138; transfer KP:140-146 with the balance replaced by the reservation
// bound: a debit is accepted only when it provably passes, otherwise KME_E_UNFUNDED.
__global__ void k_ledger_funded(DevState S, EpochIO io) {
    if (S.ctr[ci(C_ACCT_OPS)] == 0) return;
    const uint32_t lim = err_limit(S.ctr, io.n);
    const int lane = lane_id();
    for (uint32_t base = 0; base < lim; base += 64) {
        const uint32_t i = base + lane;
        const int32_t a = i < lim ? io.action[i] : -1;
        unsigned long long m = __ballot(a == CREATE_BALANCE || a == TRANSFER);
        while (m) {
            const int l = __builtin_ctzll(m);
            m &= m - 1;
            const uint32_t j = base + l;
            const int32_t act = io.action[j];
            const int64_t aid = io.aid[j];
            const int32_t size = io.size[j];
            const int64_t seq = io.seq_base + j;
            bool ok = false;
            if (aid < 0 || aid >= S.A) {
                // (an account outside the dense range lives in the exact Balances only: k_serial)
                if (S.fallback || (S.refuse && act == CREATE_BALANCE)) { need_serial(S); return; }
                if (act == CREATE_BALANCE) { raise_wave(S.ctr, KME_E_CAPACITY, KME_D_CAP_ACCOUNT, j); return; }
            } else if (act == CREATE_BALANCE) {
                if (!(S.acct_since[aid] < seq)) {
                    S.acct_since[aid] = seq;
                    S.acct_lb[aid] = 0;
                    ok = true;
                }
            } else {
                if (S.acct_since[aid] < seq) {
                    const int64_t lbs = S.acct_since[aid] < io.seq_base ? S.acct_lb[aid] : 0;
                    const int64_t cons = lbs - S.acct_need[aid] - S.acct_negx[aid];
                    // transfer rejects when balance < -size as a Java int (KP:142).  With credit_div
                    // shards this shard proves its part of that threshold (ceil of a positive one,
                    // truncation of a negative one) and books floor(credit / d) or ceil(debit / d),
                    // so the shards' bounds never sum above the account's cash.
                    const int64_t d = S.credit_div;
                    const int64_t thr = (int64_t)jineg(size);
                    const int64_t thr_share = thr > 0 ? (thr + d - 1) / d : thr / d;
                    const int64_t share = size >= 0 ? (int64_t)size / d : -((-(int64_t)size + d - 1) / d);
                    if (cons >= thr_share) {
                        ok = true;
                        S.acct_xfer[aid] += share;
                        if (share < 0) S.acct_negx[aid] -= share;
                    } else {
                        if (S.fallback) atomicOr(&S.ctr[ci(C_FALLBACK)], 1ull);   // the epoch runs serially
                        else raise_wave(S.ctr, KME_E_UNFUNDED, KME_D_NONE, j);
                        return;
                    }
                }
            }
            write_out(io, j, act, ok, size, false, 0);
            io.n_trades[j] = 0;
            __builtin_amdgcn_wave_barrier();
        }
    }
}

// FUNDED per-account proof: balance >= lb_start - need - debits >= 0 >= any single risk remaining,
// i.e. every checkBalance (KP:177) of this epoch passes.  Otherwise the epoch runs serially
// (KME_FLAG_SERIAL_FALLBACK) or is refused as a whole: KME_E_UNFUNDED / KME_D_UNPROVEN raised at
// index 0, so that no fault at a later record can replace it (err_code orders by index first) and
// err_limit lets no record of the epoch take effect.  At index 0 itself the code orders by detail,
// and UNPROVEN (18) is the largest: a fault of record 0 (e.g. a duplicate oid) is reported instead.
// That is the reference's outcome -- it throws at record 0 whatever the ledger holds (KP:96) -- and
// either way no record of the epoch takes effect.
// (Run by k_route's blocks past its records: the check is independent of the routing, and a launch of
// its own cost ~4 us of the drop-in's 65,536-record epochs.)
KDEV void check_funded(const DevState& S, const EpochIO& io, int64_t a) {
    if (a >= S.A) return;
    const int64_t need = S.acct_need[a];
    if (need <= 0) return;
    const int64_t lbs = S.acct_since[a] < io.seq_base ? S.acct_lb[a] : 0;
    if (lbs - need - S.acct_negx[a] < 0) {
        if (S.fallback) atomicOr(&S.ctr[ci(C_FALLBACK)], 1ull);   // k_serial takes the epoch
        else raise_thread(S.ctr, KME_E_UNFUNDED, KME_D_UNPROVEN, 0);
    }
}
// The bounds roll forward once the whole proof is in (k_settle_funded, after the epoch's matching:
// nothing between reads the bounds, and the roll-forward was a launch of its own before k_route):
// lb = lb_start - need + transfers.  An epoch none of whose records takes effect (refused by the
// proof, or faulting at its first record) changes no bound, and the accounts its CREATE_BALANCE
// records created (k_ledger_funded, for the acct_ok of the epoch's later orders) are absent again:
// nothing of it took effect, so the caller can resubmit it (KME_E_UNFUNDED is not fatal).
KDEV void commit_funded(const DevState& S, const EpochIO& io, int64_t a) {
    const unsigned long long c = S.ctr[ci(C_ERR)];
    const bool refused = c != ~0ull && (c >> 16) == 0;
    if (refused && S.ctr[ci(C_ACCT_OPS)] != 0) {
        const int64_t since = S.acct_since[a];
        if (since >= io.seq_base && since < io.seq_base + (int64_t)io.n) { S.acct_since[a] = INT64_MAX; S.acct_lb[a] = 0; }
    }
    const int64_t need = S.acct_need[a], negx = S.acct_negx[a], xfer = S.acct_xfer[a];
    if (need == 0 && negx == 0 && xfer == 0) return;
    const int64_t since = S.acct_since[a];
    if (!refused && since < io.seq_base + (int64_t)io.n) {
        S.acct_lb[a] = (since < io.seq_base ? S.acct_lb[a] : 0) - need + xfer;
        S.acct_demand[a] += need;
    }
    S.acct_need[a] = 0; S.acct_negx[a] = 0; S.acct_xfer[a] = 0;
}

// ------------------------------------------------------------------ credit between symbol shards
// With symbols keyed over N engines (credit_shards = N) each engine proves its orders against its
// own share of an account's cash (k_ledger_funded / check_funded), and the funded bound only falls
// inside the proof (refunds are not credited back, KP:269, 286, 331), so a share can run dry while
// the account's other shares still hold most of its cash.  Between epochs the shares are pooled and
// split again: every engine contributes (funded bound, demand so far), all-gathers them
// (kme_credit_rebalance over RCCL, or any caller transport: kme_credit_state / kme_credit_adjust),
// and takes floor(total * w_me / sum w) of the pooled bound, w_k = demand_k + mean demand + 1 (half
// proportional to where the account trades, half equal), the rounding left-over going to shard
// a mod N.  Every engine computes the same split from the same data, the shares sum to exactly the
// pooled bound, so the invariant the proof rests on -- the account's cash is at least the sum of the
// shards' bounds -- holds across the re-split.
// An account absent on a shard (never created there, or created by an epoch only that shard refused,
// commit_funded) reports demand -1: it takes no share, and the rounding left-over goes to a shard
// that holds the account, so no credit leaves the pool.
__global__ void __launch_bounds__(256) k_credit_state(DevState S, int64_t* out) {
    const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (a >= S.A) return;
    const bool present = S.acct_since[a] != INT64_MAX;
    out[a] = present ? S.acct_lb[a] : 0;
    out[S.A + a] = present ? S.acct_demand[a] : -1;
}
// all: n blocks of `stride` words (bound [0, A), demand [A, 2A)), shard-major.
__global__ void __launch_bounds__(256) k_credit_adjust(DevState S, const int64_t* all, uint32_t n, uint32_t me, size_t stride) {
    const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (a >= S.A || S.acct_since[a] == INT64_MAX) return;
    const size_t A = (size_t)S.A;
    unsigned __int128 tot = 0, dsum = 0;
    uint32_t npresent = 0;
    for (uint32_t k = 0; k < n; ++k) {
        const int64_t lb = all[(size_t)k * stride + a], d = all[(size_t)k * stride + A + a];
        if (d < 0) continue;   // absent on shard k
        tot += (unsigned __int128)(lb > 0 ? lb : 0);
        dsum += (unsigned __int128)d;
        ++npresent;
    }
    const unsigned __int128 mean = dsum / npresent;   // (npresent >= 1: this shard holds the account)
    unsigned __int128 wsum = 0;
    for (uint32_t k = 0; k < n; ++k) {
        const int64_t d = all[(size_t)k * stride + A + a];
        if (d >= 0) wsum += (unsigned __int128)d + mean + 1;
    }
    unsigned __int128 mine = 0, given = 0;
    for (uint32_t k = 0; k < n; ++k) {
        const int64_t d = all[(size_t)k * stride + A + a];
        if (d < 0) continue;
        const unsigned __int128 share = tot * ((unsigned __int128)d + mean + 1) / wsum;
        given += share;
        if (k == me) mine = share;
    }
    // the rounding left-over: the first shard holding the account, from a mod n on (cyclic)
    uint32_t first = 0;
    for (uint32_t q = 0; q < n; ++q) {
        const uint32_t k = (uint32_t)((a + q) % n);
        if (all[(size_t)k * stride + A + a] >= 0) { first = k; break; }
    }
    if (first == me) mine += tot - given;
    S.acct_lb[a] = (int64_t)mine;
}

// Symbol group of each record and the node a CANCEL addresses.  The cancel carries no symbol
// (exchange_test.js:101): removeOrder finds it by oid alone (KP:290).  Target = an order of this
// epoch submitted earlier (encoded -(j+2)), else a resting order from the oid table, else none.
__global__ void k_route(DevState S, EpochIO io, int funded) {
    const uint32_t nb = (io.n + blockDim.x - 1) / blockDim.x;
    if (blockIdx.x >= nb) {   // FUNDED: the blocks past the records check the accounts' proof
        check_funded(S, io, (int64_t)(blockIdx.x - nb) * blockDim.x + threadIdx.x);
        return;
    }
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= io.n) return;
    const int32_t a = io.action[i];
    int32_t grp = -1, vlev = 0;
    int64_t tgt = -1;
    uint32_t vpos = 0;
    S.rest_slot[i] = (a == BUY || a == SELL) ? RS_PENDING : -1;
    io.n_trades[i] = 0;
    if (funded && (a == BUY || a == SELL)) {   // routed by k_emap
        if (S.fallback) S.cancel_tgt[i] = -1;
        // with account records in the epoch (k_ledger_funded has applied them) acct_ok is decided
        // again (k_emap read the accounts as they stood before the epoch); was a kernel of its own
        if (S.ctr[ci(C_ACCT_OPS)] != 0 && S.route_grp[i] >= 0) {
            const int64_t aid = io.aid[i];
            const bool acct_ok = aid >= 0 && aid < S.A && S.acct_since[aid] < io.seq_base + (int64_t)i;
            KG int32_t* w0 = reinterpret_cast<KG int32_t*>(&S.prec[2 * (size_t)i]);
            *w0 = (*w0 & ~(1 << 16)) | ((acct_ok ? 1 : 0) << 16);
        }
        return;
    }
    bool direct = false, ok = false, acct_ok = false;
    switch (a) {
    case ADD_SYMBOL:
    case REMOVE_SYMBOL:
    case PAYOUT: {
        grp = group_of(io.sid[i], S.G);
        // a sparse symbol (|sid| >= G) may exist in the serial engine's stores (S.Gs > 0)
        const bool sparse = grp < 0 && S.Gs > 0 && (!funded || S.fallback);
        if (funded && a == PAYOUT && serial_capable(S)) {
            need_serial(S);                                                 // the positions ledger (KP:148-165)
        } else if (grp < 0) {
            if (a == ADD_SYMBOL) {
                if (sparse) { if (funded) need_serial(S); }                 // (EXACT: k_serial names it)
                else if (funded && S.refuse) need_serial(S);
                else raise_thread(S.ctr, KME_E_CAPACITY, KME_D_CAP_SYMBOL, i);
            } else if (a == REMOVE_SYMBOL) {
                if (sparse) { if (funded) need_serial(S); }
                else { direct = true; ok = true; }                          // removeSymbol of an absent symbol
            } else if (funded) {
                raise_thread(S.ctr, KME_E_UNSUPPORTED, KME_D_NONE, i);
            }
        }
        break;
    }
    case BUY:
    case SELL: {
        grp = group_of(io.sid[i], S.G);
        if (grp < 0) { direct = true; ok = false; }                         // books.get == null (KP:202-203)
        if (funded && grp >= 0) {
            const int64_t aid = io.aid[i];
            acct_ok = aid >= 0 && aid < S.A && S.acct_since[aid] < io.seq_base + (int64_t)i;
        }
        break;
    }
    case CANCEL: {
        // the target's level (price | side << 8 | 1 << 9) rides along for k_match_lanes, which then
        // fetches the node and its level in one step (checked against the node there)
        const int64_t oid = io.oid[i];
        uint32_t hpos = 0;
        Node nd;
        int64_t sj = 0;
        int32_t pj = 0;
        const int64_t t = otab_cancel_target(S, io, oid, i, hpos, nd, sj, pj);
        if (t <= -2) vpos = hpos;
        if (t <= -2) {
            const uint32_t j = (uint32_t)(-(t + 2));
            const int32_t gj = group_of(sj, S.G);
            if (gj >= 0) {
                grp = gj; tgt = t;
                const int side = (sj != 0 && ((sj < 0) != (io.action[j] != BUY))) ? 1 : 0;   // book_side
                vlev = (pj & 0xFF) | (side << 8) | (1 << 9);
            } else if (S.Gs > 0 && (!funded || S.fallback)) {
                grp = GRP_RESOLVE; tgt = t;                                 // (order j made the epoch serial)
            }
        } else if (t >= 0) {
            grp = nd.group; tgt = t;
            const int side = (nd.sid != 0 && ((nd.sid < 0) != (nd.action != BUY))) ? 1 : 0;
            vlev = (nd.price & 0xFF) | (side << 8) | (1 << 9);
            if (grp >= S.G) {                                               // an order on a sparse symbol:
                grp = GRP_RESOLVE;                                          // k_serial names its group
                if (funded) need_serial(S);
            }
        }
        if (funded && S.fallback && grp != -1) {
            const int64_t caid = io.aid[i];
            if (caid < 0 || caid >= S.A) need_serial(S);                    // an account of the exact ledger only
        }
        if (grp == -1) { direct = true; ok = false; }                       // orders.get == null (KP:290-291)
        break;
    }
    case CREATE_BALANCE:
    case TRANSFER:
        break;                                                              // k_ledger_funded / k_serial
    default:
        direct = true; ok = false;                                          // no case: REJECT (KP:99-123)
        break;
    }
    S.route_grp[i] = grp;
    if (!funded || S.fallback) S.cancel_tgt[i] = tgt;   // k_serial's cancel target
    if (!funded) return;
    if (direct) write_out(io, i, a, ok, io.size[i], false, 0);
    if (grp >= 0 && grp < S.G) {   // the record as k_match reads it (PRec)
        const int64_t oid = io.oid[i], aid = io.aid[i];
        // word 6: a cancel's target (a same-epoch order j: -(j + 2)); a FUNDED BUY/SELL's packed record
        // is k_emap's, with its own entry's position there.  Word 1 of a cancel of a same-epoch order:
        // that order's oid-table entry position instead of the cancel's size (the OUT echo of a cancel
        // keeps the input's size: k_unsort takes it from the input) -- k_match_lanes reads the entry
        // the order's rest finalised there, k_match reads rest_slot[j]
        const int32_t w0 = (a & 0xFF) | ((io.price[i] & 0xFF) << 8) | ((acct_ok ? 1 : 0) << 16) | ((io.sid[i] < 0 ? 1 : 0) << 17);
        KG int4* p = &S.prec[2 * (size_t)i];
        const int32_t w1 = (a == CANCEL && tgt <= -2) ? (int32_t)vpos : io.size[i];
        p[0] = make_int4(w0, w1, (int32_t)(uint32_t)oid, (int32_t)((uint64_t)oid >> 32));
        p[1] = make_int4((int32_t)(uint32_t)aid, (int32_t)((uint64_t)aid >> 32), (int32_t)tgt, vlev);
    }
}

// ------------------------------------------------------------------ (1) stable radix partition
// LSD radix sort of (group, input index) pairs, RADIX_BITS-bit digits (65,536 symbol groups: two
// passes).  Records without a group sort into bucket G, which nobody processes.  Stability =
// arrival order inside each group.
constexpr int RADIX_DIGITS = 1 << RADIX_BITS;
constexpr int RADIX_PER_T = RADIX_DIGITS / 256;   // digits per thread of a 256-thread block

// c ? b : a for two fields of a kernel argument, as arithmetic: a select between two of its fields was
// folded into a load at a computed offset, which keeps a private copy of the whole argument (136 B
// per lane of scratch, written at every scatter's start and read back on its critical path)
template <typename P>
KDEV P pick(bool c, P a, P b) {
    const uint64_t x = (uint64_t)(uintptr_t)a, y = (uint64_t)(uintptr_t)b;
    return (P)(uintptr_t)(x ^ ((x ^ y) & (0ull - (uint64_t)c)));
}
KDEV uint32_t radix_n(const RadixIO& R) {
    if (!R.n_dev) return R.n;
    const uint32_t d = (uint32_t)*R.n_dev;
    return d < R.n ? d : R.n;
}
// A tile's keys (and values), RJ per thread at base + off + j * stride + lane-offset: every load is
// issued before any is used (no branch between a load and the next one: an index past n reads
// element 0 and is masked afterwards), so a thread has all of them in flight at once -- a load per
// round behind its own wait made both kernels one memory round trip per round.
template <int RJ, bool VALS>
KDEV void radix_load(const RadixIO& R, int pass, int src, uint32_t n, uint32_t first, uint32_t stride, uint32_t* keys,
                     uint32_t* vals) {
    if (n == 0) {
#pragma unroll
        for (int j = 0; j < RJ; ++j) { keys[j] = 0; vals[j] = 0; }
        return;
    }
    // (selects, not an index into the argument's arrays: a dynamic index reads them through a vector
    // load whose wait then lands before every later memory operation)
    const KG uint32_t* kp = pick<const KG uint32_t*>(pass == 0, pick<const KG uint32_t*>(src != 0, R.keys0, R.keys1),
                                                     reinterpret_cast<const KG uint32_t*>(R.key0));
    const KG uint32_t* vp = pick<const KG uint32_t*>(pass == 0, pick<const KG uint32_t*>(src != 0, R.vals0, R.vals1), R.val0);
#pragma unroll
    for (int j = 0; j < RJ; ++j) {
        const uint32_t k = first + j * stride;
        keys[j] = kp[k < n ? k : 0];
    }
    if (VALS && vp) {
#pragma unroll
        for (int j = 0; j < RJ; ++j) {
            const uint32_t k = first + j * stride;
            vals[j] = vp[k < n ? k : 0];
        }
    }
#pragma unroll
    for (int j = 0; j < RJ; ++j) {
        const uint32_t k = first + j * stride;
        // pass 0: the group (int32), records without one into bucket `none`
        if (pass == 0 && (int32_t)keys[j] < 0) keys[j] = R.none;
        if (VALS && !vp) vals[j] = k;
        if (k >= n) { keys[j] = 0; vals[j] = 0; }
    }
}

template <int TILE>
__global__ void __launch_bounds__(256) k_radix_hist(RadixIO R, int pass, int src) {
    __shared__ uint32_t h[RADIX_DIGITS];
    const int t = threadIdx.x;
    for (int q = 0; q < RADIX_PER_T; ++q) h[t + 256 * q] = 0;
    const uint32_t base = blockIdx.x * TILE, n = radix_n(R);
    constexpr int RJ = TILE / 256;
    uint32_t keys[RJ], unused[RJ];
    radix_load<RJ, false>(R, pass, src, n, base + t, 256, keys, unused);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RJ; ++j) {
        if (base + j * 256 + t < n) atomicAdd(&h[(keys[j] >> (RADIX_BITS * pass)) & (RADIX_DIGITS - 1)], 1u);
    }
    __syncthreads();
    for (int q = 0; q < RADIX_PER_T; ++q) R.ghist[(t + 256 * q) * gridDim.x + blockIdx.x] = h[t + 256 * q];
}

// Small sorts: every pass's digit counts of this tile of the unpermuted keys (R.tcnt, pass-major,
// then tile, then digit) -- what radix_lb_offsets sums into the digit totals.
template <int TILE>
__global__ void __launch_bounds__(256) k_radix_tcnt(RadixIO R) {
    __shared__ uint32_t h[RADIX_MAXP][RADIX_DIGITS];
    const int t = threadIdx.x;
    const uint32_t base = blockIdx.x * TILE, n = radix_n(R);
    if (base >= n) return;
    for (int p = 0; p < RADIX_MAXP; ++p)
        for (int q = 0; q < RADIX_PER_T; ++q) h[p][t + 256 * q] = 0;
    constexpr int RJ = TILE / 256;
    uint32_t keys[RJ], unused[RJ];
    radix_load<RJ, false>(R, 0, 0, n, base + t, 256, keys, unused);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RJ; ++j) {
        if (base + j * 256 + t >= n) continue;
        for (int p = 0; p < R.passes; ++p) atomicAdd(&h[p][(keys[j] >> (RADIX_BITS * p)) & (RADIX_DIGITS - 1)], 1u);
    }
    __syncthreads();
    for (int p = 0; p < R.passes; ++p)
        for (int q = 0; q < RADIX_PER_T; ++q)
            R.tcnt[((size_t)p * gridDim.x + blockIdx.x) * RADIX_DIGITS + t + 256 * q] = h[p][t + 256 * q];
}

// One tile's scatter, staged in LDS: the tile is first ordered by digit in LDS (stable), then
// written out in that order, so that each digit's run of the tile leaves in consecutive lanes
// (coalesced stores) instead of one scattered 4-B store per element and array.  Ranking is per
// wavefront: wavefront w owns the tile's w-th quarter (contiguous, so index order = wavefront,
// round, lane) and counts its digits in its own LDS row round by round (match-any over the digit
// bits; the first lane of each digit adds the run), so the only block barriers are the few
// between the counting, the per-digit offsets and the placement.
// Small sorts (launch_radix, R.tcnt): each pass's global digit offsets without the histogram and
// scan launches -- the digit totals from the unpermuted keys' per-tile counts (k_radix_tcnt: a
// permutation does not change them), and the tiles before this one by look-back: each tile publishes
// its digit counts as (count | stamp << 32) words as soon as it has ranked its keys, and reads those of
// every earlier tile (all resident: a small sort is a few dozen tiles, and an earlier tile never
// waits for a later one).  t0 / t1: this tile's counts of digits 2t, 2t + 1; returns their offsets.
KDEV uint32_t block_excl_scan_256(uint32_t v, uint32_t* wsum, uint32_t& total);
constexpr int LB_BATCH = 32;   // (tiles read per round trip)
// The first LB_BATCH tiles' rows of tcnt (thread t's two digits), loaded by the caller before its
// ranking so that their latency overlaps it (the rows are the previous kernel's: nothing to wait for).
KDEV void radix_lb_rows(const RadixIO& R, int pass, uint32_t ntiles, uint2* v) {
    const KG uint32_t* tc = R.tcnt + (size_t)pass * gridDim.x * RADIX_DIGITS;
#pragma unroll
    for (int b = 0; b < LB_BATCH; ++b) {
        const uint32_t q = (uint32_t)b < ntiles ? (uint32_t)b : 0;
        v[b] = *reinterpret_cast<const KG uint2*>(&tc[(size_t)q * RADIX_DIGITS + 2 * threadIdx.x]);
    }
}
KDEV void radix_lb_offsets(const RadixIO& R, int pass, uint32_t stamp, uint32_t ntiles, uint32_t t0, uint32_t t1,
                           uint32_t* wsum, const uint2* first, uint32_t& g0, uint32_t& g1) {
    const int t = threadIdx.x;
    const uint32_t tile = blockIdx.x;
    KG unsigned long long* lb = R.lb;   // per tile 256 words: thread t's two digit counts (12 bits each) | stamp << 32
    const unsigned long long st = (unsigned long long)stamp << 32;
    if (pass > 0)   // (pass 0's tiles are the unpermuted keys': their counts are tcnt's row 0 already)
        __hip_atomic_store(&lb[(size_t)tile * 256 + t], st | (t1 << 16) | t0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // the digits' totals over the sort's tiles, exclusive over the digits (pass 0: and the earlier
    // tiles' counts, from the same rows; the first LB_BATCH rows are the caller's, `first`)
    const KG uint32_t* tc = R.tcnt + (size_t)pass * gridDim.x * RADIX_DIGITS;
    uint32_t T0 = 0, T1 = 0, P0 = 0, P1 = 0;
#pragma unroll
    for (int b = 0; b < LB_BATCH; ++b) {
        if ((uint32_t)b < ntiles) { T0 += first[b].x; T1 += first[b].y; }
        if (pass == 0 && (uint32_t)b < tile) { P0 += first[b].x; P1 += first[b].y; }
    }
    for (uint32_t q0 = LB_BATCH; q0 < ntiles; q0 += LB_BATCH) {
        uint2 v[LB_BATCH];
#pragma unroll
        for (int b = 0; b < LB_BATCH; ++b) {
            const uint32_t q = q0 + b < ntiles ? q0 + b : 0;
            v[b] = *reinterpret_cast<const KG uint2*>(&tc[(size_t)q * RADIX_DIGITS + 2 * t]);
        }
#pragma unroll
        for (int b = 0; b < LB_BATCH; ++b) {
            if (q0 + b < ntiles) { T0 += v[b].x; T1 += v[b].y; }
            if (pass == 0 && q0 + b < tile) { P0 += v[b].x; P1 += v[b].y; }
        }
    }
    uint32_t tot;
    const uint32_t gx = block_excl_scan_256(T0 + T1, wsum, tot);
    // the earlier tiles' counts (their words carry this launch's stamp once written)
    for (uint32_t q0 = 0; pass > 0 && q0 < tile; q0 += LB_BATCH) {
        unsigned long long w[LB_BATCH];
        uint32_t spins = 0;
        for (;;) {
            bool all = true;
#pragma unroll
            for (int b = 0; b < LB_BATCH; ++b) {
                const uint32_t q = q0 + b < tile ? q0 + b : 0;
                w[b] = __hip_atomic_load(&lb[(size_t)q * 256 + t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
#pragma unroll
            for (int b = 0; b < LB_BATCH; ++b) all = all && (q0 + b >= tile || (uint32_t)(w[b] >> 32) == stamp);
            if (all) break;
            if (++spins == (1u << 24)) {   // (cannot happen: an earlier tile never waits for this one)
                printf("kme: radix look-back: tile %u waits for tiles %u.. (stamp %u)\n", tile, q0, stamp);
                if (R.ctr) raise_thread(R.ctr, KME_E_HIP, KME_D_GUARD_LOOKBACK, -1);
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
#pragma unroll
        for (int b = 0; b < LB_BATCH; ++b)
            if (q0 + b < tile) { P0 += (uint32_t)w[b] & 0xFFFFu; P1 += (uint32_t)(w[b] >> 16) & 0xFFFFu; }
    }
    g0 = gx + P0;
    g1 = gx + T0 + P1;
}

template <int TILE, bool LB = false>
__global__ void __launch_bounds__(256) k_radix_scatter(RadixIO R, int pass, int src, uint32_t stamp = 0) {
    static_assert(RADIX_DIGITS == 512, "two digits per thread");
    static_assert(TILE % 256 == 0, "whole rounds");
    static_assert(TILE < 65536, "a tile's digit count fits a look-back word's 16 bits");
    __shared__ uint32_t wh[4][RADIX_DIGITS];     // wavefront w's count of digit d, then its first local slot
    __shared__ uint32_t gdelta[RADIX_DIGITS];    // digit d's global offset minus its local start
    __shared__ uint32_t lkey[TILE], lval[TILE];
    __shared__ uint32_t wsum[4];
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    const uint32_t base = blockIdx.x * TILE, n = radix_n(R);
    if (LB && base >= n) return;   // (a tile past the keys: no later tile waits for it)
    const int dst = src ^ 1;
    const int shift = RADIX_BITS * pass;
    const unsigned long long lt_mask = (1ull << lane) - 1ull;
    constexpr int RJ = TILE / 256;
    constexpr int WCH = TILE / 4;                // elements per wavefront
    uint32_t keys[RJ], vals[RJ], wr[RJ];
    radix_load<RJ, true>(R, pass, src, n, base + w * WCH + lane, 64, keys, vals);
    uint2 rows[LB ? LB_BATCH : 1];
    if constexpr (LB) radix_lb_rows(R, pass, (n + TILE - 1) / TILE, rows);
#pragma unroll
    for (int q = 0; q < RADIX_DIGITS / 64; ++q) wh[w][lane + 64 * q] = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int j = 0; j < RJ; ++j) {
        const bool valid = base + w * WCH + j * 64 + lane < n;
        const uint32_t d = (keys[j] >> shift) & (RADIX_DIGITS - 1);
        unsigned long long peers = __ballot(valid);
        for (int b = 0; b < RADIX_BITS; ++b) {
            const unsigned long long bb = __ballot(valid && ((d >> b) & 1));
            peers &= ((d >> b) & 1) ? bb : ~bb;
        }
        const uint32_t rank = (uint32_t)__popcll(peers & lt_mask);
        const uint32_t old = valid ? wh[w][d] : 0u;
        wr[j] = old + rank;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (valid && rank == 0) wh[w][d] = old + (uint32_t)__popcll(peers);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    __syncthreads();
    {   // digits 2t and 2t + 1: local start (block scan of the tile histogram), each wavefront's first
        // slot, and the global offset (k_radix_hist + scan)
        uint32_t c0[4], c1[4], t0 = 0, t1 = 0;
#pragma unroll
        for (int ww = 0; ww < 4; ++ww) { c0[ww] = wh[ww][2 * t]; c1[ww] = wh[ww][2 * t + 1]; t0 += c0[ww]; t1 += c1[ww]; }
        uint32_t tot;
        const uint32_t ex = block_excl_scan_256(t0 + t1, wsum, tot);
        uint32_t r0 = ex, r1 = ex + t0;
        if constexpr (LB) {
            uint32_t g0, g1;
            radix_lb_offsets(R, pass, stamp, (n + TILE - 1) / TILE, t0, t1, wsum, rows, g0, g1);
            gdelta[2 * t] = g0 - r0;
            gdelta[2 * t + 1] = g1 - r1;
        } else {
            gdelta[2 * t] = R.ghist[(size_t)(2 * t) * gridDim.x + blockIdx.x] - r0;
            gdelta[2 * t + 1] = R.ghist[(size_t)(2 * t + 1) * gridDim.x + blockIdx.x] - r1;
        }
#pragma unroll
        for (int ww = 0; ww < 4; ++ww) { wh[ww][2 * t] = r0; wh[ww][2 * t + 1] = r1; r0 += c0[ww]; r1 += c1[ww]; }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RJ; ++j) {
        if (base + w * WCH + j * 64 + lane < n) {
            const uint32_t pos = wh[w][(keys[j] >> shift) & (RADIX_DIGITS - 1)] + wr[j];
            lkey[pos] = keys[j];
            lval[pos] = vals[j];
        }
    }
    __syncthreads();
    if (base >= n) return;
    const uint32_t cnt = n - base < (uint32_t)TILE ? n - base : (uint32_t)TILE;
    KG uint32_t* okeys = pick(dst != 0, R.keys0, R.keys1);
    KG uint32_t* ovals = pick(dst != 0, R.vals0, R.vals1);
    const bool last = pass == R.passes - 1 && R.rank;
    const bool pay = pass == R.passes - 1 && R.pay_src;
#pragma unroll
    for (int j = 0; j < RJ; ++j) {
        const uint32_t e = j * 256 + t;
        if (e < cnt) {
            const uint32_t key = lkey[e], val = lval[e];
            const uint32_t pos = gdelta[(key >> shift) & (RADIX_DIGITS - 1)] + e;
            okeys[pos] = key;
            ovals[pos] = val;
            if (last) R.rank[val] = (int32_t)pos;
            // a 16-B payload gathered into sorted order, one element at a time: with all of a thread's
            // gathers in flight at once the pass was slower (the exact ledger's op sort: 194 -> 259 us)
            if (pay) R.pay_dst[pos] = R.pay_src[val];
        }
    }
}

// Group segment offsets from the sorted keys: seg[g] = first position with key >= g.
// list_min >= 0: the thread at a group's first record also lists the group when it has more than
// list_min records (its record list_min places on is still the group's) -- k_match_list's work.
__global__ void k_segments(DevState S, EpochIO io, int buf, int list_min) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t n = io.n;
    const uint32_t nseg = (uint32_t)S.G + 2;
    if (n == 0) {
        for (uint32_t g = k; g < nseg; g += gridDim.x * blockDim.x) S.seg[g] = 0;
        return;
    }
    if (k > n) return;
    const uint32_t* keys = buf ? S.rkeys[1] : S.rkeys[0];
    const int64_t prev = k == 0 ? -1 : (int64_t)keys[k - 1];
    const int64_t cur = k == n ? (int64_t)nseg - 1 : (int64_t)keys[k];
    for (int64_t g = prev + 1; g <= cur; ++g) S.seg[g] = k;
    // a group whose book only the serial engine can take (a level above 100, a negative size) makes the
    // epoch serial -- checked once k_serial ever made such a book (C_ODD)
    if (k < n && cur != prev && cur < (int64_t)S.G && S.ctr[ci(C_ODD)] != 0) {
        const GroupState& gs = S.grp[cur];
        if (gs.nneg > 0 || (gs.bm0_msb >> 38) != 0 || (gs.bm1_msb >> 38) != 0) need_serial(S);
    }
    if (list_min >= 0 && k < n && cur != prev && cur < (int64_t)S.G) {
        const uint32_t kl = k + (uint32_t)list_min;
        if (kl < n && (int64_t)keys[kl] == cur) {
            const unsigned long long x = atomicAdd(&S.ctr[ci(C_GLIST)], 1ull);
            S.glist[x] = (uint32_t)cur;
        }
    }
}

// ------------------------------------------------------------------ exclusive scan (DPP)
constexpr int SCAN_ITEMS = 8;
constexpr int SCAN_BLOCK = 256 * SCAN_ITEMS;

KDEV uint32_t block_excl_scan_256(uint32_t v, uint32_t* wsum, uint32_t& total) {
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    const uint32_t inc = wave_incl_scan_u32(v);
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t off = 0;
    for (int k = 0; k < w; ++k) off += wsum[k];
    total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
    return off + inc - v;
}

// Exclusive scan in two launches (reduce, then scan): k_tile_sums writes each 4,096-item tile's
// sum; k_scan_tiles gives every tile its prefix from those sums (at most a few thousand, read by
// every block from L2) and scans the tile in LDS.  Replaces the three-kernel scan (blocks, sums,
// add) and the copy of the total on the epoch path.  (A single-pass decoupled look-back was
// measured slower: with every tile resident at once the inclusive prefixes resolve 64 tiles per
// L2 round trip, ~16 round trips for the 1,024 tiles of a 4M-record epoch.)
constexpr int LB_ITEMS = 16;
constexpr int LB_TILE = 256 * LB_ITEMS;
KDEV uint32_t lb_pad(uint32_t k) { return k + (k >> 5); }
__global__ void __launch_bounds__(256) k_tile_sums(const uint32_t* in, uint32_t L, uint32_t* sums) {
    __shared__ uint32_t wsum[4];
    const uint32_t base = blockIdx.x * LB_TILE;
    uint32_t sum = 0;
#pragma unroll
    for (int j = 0; j < LB_ITEMS; ++j) {
        const uint32_t k = base + j * 256 + threadIdx.x;
        sum += k < L ? in[k] : 0u;
    }
    uint32_t tot;
    (void)block_excl_scan_256(sum, wsum, tot);
    if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}
// LB (small scans, at most LB_MAX_TILES tiles: launch_scan2): one launch -- each tile publishes its sum
// as a (sum | stamp << 32) word in `sums` (then 8-byte words) and thread q reads tile q's, for the tiles
// before this one (all resident; an earlier tile never waits for a later one).
constexpr uint32_t LB_MAX_TILES = 64;
template <bool LB = false>
__global__ void __launch_bounds__(256) k_scan_tiles(const uint32_t* in, uint32_t* out, uint32_t L, const uint32_t* sums,
                                                    uint32_t* total_out, int write_end, uint32_t stamp = 0,
                                                    unsigned long long* ctr = nullptr) {
    __shared__ uint32_t buf[LB_TILE + LB_TILE / 32];
    __shared__ uint32_t wsum[4];
    const int t = threadIdx.x;
    const uint32_t tile = blockIdx.x, base = tile * LB_TILE;
    // every load issued before any is used (clamped indices, masked afterwards): a conditional load
    // per round made each round wait for its own
    uint32_t x[LB_ITEMS];
#pragma unroll
    for (int j = 0; j < LB_ITEMS; ++j) {
        const uint32_t k = base + j * 256 + t;
        x[j] = L ? in[k < L ? k : L - 1] : 0u;
    }
    uint32_t pre = 0;                                  // this thread's share of the tiles before this one
    if constexpr (LB) {
        uint32_t mine = 0;
#pragma unroll
        for (int j = 0; j < LB_ITEMS; ++j) mine += base + j * 256 + t < L ? x[j] : 0u;
        uint32_t tsum;
        (void)block_excl_scan_256(mine, wsum, tsum);
        unsigned long long* w = reinterpret_cast<unsigned long long*>(const_cast<uint32_t*>(sums));
        if (t == 0)
            __hip_atomic_store(&w[tile], (unsigned long long)stamp << 32 | tsum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((uint32_t)t < tile) {
            unsigned long long v = 0;
            for (uint32_t spins = 0;; ++spins) {
                v = __hip_atomic_load(&w[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((uint32_t)(v >> 32) == stamp) break;
                if (spins == (1u << 24)) {   // (cannot happen: an earlier tile never waits for this one)
                    printf("kme: scan look-back: tile %u waits for tile %d (stamp %u)\n", tile, t, stamp);
                    if (ctr) raise_thread(ctr, KME_E_HIP, KME_D_GUARD_LOOKBACK, -1);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            pre = (uint32_t)v;
        }
    }
    for (uint32_t q0 = 0; !LB && q0 < tile; q0 += 8 * 256) {
        uint32_t y[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const uint32_t q = q0 + r * 256 + t;
            y[r] = sums[q < tile ? q : 0];
        }
#pragma unroll
        for (int r = 0; r < 8; ++r) pre += q0 + r * 256 + t < tile ? y[r] : 0u;
    }
#pragma unroll
    for (int j = 0; j < LB_ITEMS; ++j) {
        const uint32_t k = j * 256 + t;
        buf[lb_pad(k)] = base + k < L ? x[j] : 0u;
    }
    uint32_t excl;
    (void)block_excl_scan_256(pre, wsum, excl);        // (its barriers also order the LDS stores above)
    uint32_t v[LB_ITEMS], sum = 0;
#pragma unroll
    for (int j = 0; j < LB_ITEMS; ++j) { v[j] = buf[lb_pad(LB_ITEMS * t + j)]; sum += v[j]; }
    uint32_t tot;
    const uint32_t ex = block_excl_scan_256(sum, wsum, tot);
    if (t == 0 && tile == gridDim.x - 1) {
        if (total_out) *total_out = excl + tot;
        if (write_end) out[L] = excl + tot;
    }
    uint32_t run = excl + ex;
#pragma unroll
    for (int j = 0; j < LB_ITEMS; ++j) { buf[lb_pad(LB_ITEMS * t + j)] = run; run += v[j]; }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < LB_ITEMS; ++j) {
        const uint32_t k = j * 256 + t;
        if (base + k < L) out[base + k] = buf[lb_pad(k)];
    }
}

__global__ void __launch_bounds__(256) k_scan_blocks(const uint32_t* in, uint32_t* out, uint32_t L, uint32_t* bsum) {
    __shared__ uint32_t wsum[4];
    const uint32_t base = blockIdx.x * SCAN_BLOCK;
    uint32_t run = 0;
    for (int j = 0; j < SCAN_ITEMS; ++j) {
        const uint32_t k = base + j * 256 + threadIdx.x;
        const uint32_t v = k < L ? in[k] : 0;
        uint32_t tot;
        const uint32_t ex = block_excl_scan_256(v, wsum, tot);
        if (k < L) out[k] = run + ex;
        run += tot;
    }
    if (threadIdx.x == 0) bsum[blockIdx.x] = run;
}
__global__ void __launch_bounds__(256) k_scan_sums(uint32_t* bsum, uint32_t nb, uint32_t* total_out) {
    __shared__ uint32_t wsum[4];
    uint32_t run = 0;
    for (uint32_t base = 0; base < nb; base += 256) {
        const uint32_t k = base + threadIdx.x;
        const uint32_t v = k < nb ? bsum[k] : 0;
        uint32_t tot;
        const uint32_t ex = block_excl_scan_256(v, wsum, tot);
        if (k < nb) bsum[k] = run + ex;
        run += tot;
    }
    if (threadIdx.x == 0) *total_out = run;
}
__global__ void __launch_bounds__(256) k_scan_add(uint32_t* out, uint32_t L, const uint32_t* bsum) {
    const uint32_t base = blockIdx.x * SCAN_BLOCK;
    const uint32_t off = bsum[blockIdx.x];
    if (off == 0) return;
    for (int j = 0; j < SCAN_ITEMS; ++j) {
        const uint32_t k = base + j * 256 + threadIdx.x;
        if (k < L) out[k] += off;
    }
}

// ------------------------------------------------------------------ record staging helpers
// s_waitcnt vmcnt(0) expcnt(7) lgkmcnt(15): gfx9 encoding (vmcnt bits 3:0 and 15:14)
constexpr int VMCNT0 = 0x0F70;
KDEV int32_t rl32(int32_t v, int j) { return __builtin_amdgcn_readlane(v, j); }
// v_writelane_b32 (the intrinsic has no clang builtin here; bound by name)
extern "C" __device__ int32_t kme_writelane_i32(int32_t v, int32_t lane, int32_t old) __asm("llvm.amdgcn.writelane.i32");
KDEV int64_t rl64(int64_t v, int j) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, j);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), j);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
// One input record as a wavefront consumes it (wave-uniform, SGPR-resident).
struct Rec {
    uint32_t i;
    int32_t action, price, size, acct_ok;
    int64_t oid, aid, sid, tgt;
    int32_t lane;                 // lane of the record in its batch
};
constexpr uint32_t OS_MAX_NTR = 1u << FAST_RANK_SHIFT;   // trades of one record: a plain ordinal in TradeTmp::ordp
static_assert(FAST_RANK_SHIFT + 3 <= TT_ORD_BITS, "a fast segment's ordinal (index | event rank << 20) in TradeTmp::ordp");
static_assert(FAST_LVB <= 7, "a sweep's event ranks 0..FAST_LVB in three bits");
// What process() decided for one record (the OUT echo fields and its trade count).
struct Out {
    int32_t action, size;
    int64_t prev;
    bool has_prev;
    bool rested;                  // the order came to rest (counted per batch, not per record)
    uint32_t ntr;
};

struct Taker {
    int32_t action, price, size, _pad;
    int64_t oid, aid, sid;
};

// EXACT mode (k_serial): the whole epoch in arrival order on one wavefront, every store -- the
// book stores and the Balances / Positions ledger -- exact.  The current symbol group's bitmaps
// and free list are held in registers; levels and nodes are read and written in HBM.
constexpr int FBLK = 13;          // free slots per spilled free-list block (GroupWave::alloc_slot)

struct Core {
    static constexpr bool EXACT = true;
    const DevState& S;
    const EpochIO& io;
    int32_t g;
    int32_t exists;
    uint64_t b0l, b0m, b1l, b1m;      // bitmaps of book +g (side 0) and book -g (side 1)
    int32_t free_head, chunk_next, chunk_end;
    Level* glev;
    uint32_t tnext;                   // running trade count of the epoch
    bool dead;

    KDEV Core(const DevState& s, const EpochIO& e) : S(s), io(e) {
        g = -1; exists = 0; b0l = b0m = b1l = b1m = 0;
        free_head = -1; chunk_next = chunk_end = 0; glev = nullptr;
        tnext = 0; dead = false;
    }
    // A book the FUNDED matchers cannot take (they stage prices 0..100 and assume sizes >= 0): a level
    // above 100 (msb bits 38.., KP:391-404) or an order of negative size (GroupState::nneg counts them,
    // kept here on the rare paths that change one).  k_segments sends an epoch on such a group to this
    // engine; C_ODD (sticky) says one was ever made, so that check runs only from then on.
    KDEV void note_odd() { S.ctr[ci(C_ODD)] = 1; }
    KDEV void nneg_add(int32_t d) {
        S.grp[g].nneg += d;   // (one wavefront: a plain read-modify-write)
        if (d > 0) note_odd();
    }

    KDEV void die(int status, int detail, int64_t idx) { raise_wave(S.ctr, status, detail, idx); dead = true; }

    KDEV void load_group(int32_t gg) {
        g = gg;
        const GroupState& G = S.grp[gg];
        exists = G.exists;
        b0l = G.bm0_lsb; b0m = G.bm0_msb; b1l = G.bm1_lsb; b1m = G.bm1_msb;
        free_head = G.free_head; chunk_next = G.chunk_next; chunk_end = G.chunk_end;
        glev = S.lev + (size_t)gg * 2 * NLEV;
    }
    KDEV void store_group() {
        if (g < 0) return;
        {
            GroupState& G = S.grp[g];
            G.exists = exists;
            G.bm0_lsb = b0l; G.bm0_msb = b0m; G.bm1_lsb = b1l; G.bm1_msb = b1m;
            G.free_head = free_head; G.chunk_next = chunk_next; G.chunk_end = chunk_end;
        }
    }
    // The group of a record's symbol (books +sid / -sid, KP:184-191, 201): |sid| < G is group |sid|; a
    // sparse symbol (|sid| >= G) has the gsid slot its first ADD_SYMBOL took (create), group G + slot;
    // -1 = no group (the books are absent).  Long.MIN_VALUE and |sid| >= 2^55 are refused at ADD_SYMBOL:
    // their bucket pointers (sid << 8) | price alias other books' buckets (KP:379-381).
    KDEV int32_t symbol_group(int64_t sid, bool create, int64_t idx) {
        if (sid == INT64_MIN) { if (create) die(KME_E_DOMAIN, KME_D_SID_RANGE, idx); return -1; }
        const int64_t a = sid < 0 ? -sid : sid;
        if (a < (int64_t)S.G) return (int32_t)a;
        if (S.Gs <= 0) { if (create) die(KME_E_CAPACITY, KME_D_CAP_SYMBOL, idx); return -1; }
        if (create && a >= (1ll << 55)) { die(KME_E_DOMAIN, KME_D_SID_RANGE, idx); return -1; }
        const uint32_t mask = (uint32_t)S.Gs - 1;
        uint32_t h = (uint32_t)mix64((uint64_t)a) & mask;
        for (uint32_t p = 0; p <= mask; ++p) {
            const int64_t k = S.gsid[h];
            if (k == a) return S.G + (int32_t)h;
            if (k == 0) {
                if (!create) return -1;
                S.gsid[h] = a;
                return S.G + (int32_t)h;
            }
            h = (h + 1) & mask;
        }
        if (create) die(KME_E_CAPACITY, KME_D_CAP_SYMBOL, idx);
        return -1;
    }
    KDEV uint64_t bl(int side) const { return side ? b1l : b0l; }
    KDEV uint64_t bm(int side) const { return side ? b1m : b0m; }
    KDEV void set_bm(int side, uint64_t l, uint64_t m) { if (side) { b1l = l; b1m = m; } else { b0l = l; b0m = m; } }

    KDEV Level* lv(int side, int32_t p) {
        return &glev[side * NLEV + p];
    }

    KDEV Node ld_node(int32_t s) const {
        const Node* p = &S.pool[s];
        Node n;
        n.oid = p->oid; n.aid = p->aid; n.sid = p->sid; n.prev_oid = p->prev_oid;
        n.size = p->size; n.next = p->next; n.prev = p->prev; n.group = p->group;
        n.price = p->price; n.action = p->action; n.live = p->live; n._pad = 0;
        return n;
    }

    // Node slots: the group's free list in the block format of the FUNDED matchers (a free slot
    // hosting up to FBLK - 1 more free ids: word 0 = next block, word 1 = count, words 2.. = ids;
    // GroupWave::spill_blocks), so a group's state is valid for every kernel; else a chunk of the
    // pool's bump counter.
    KDEV int32_t alloc_slot(int64_t idx) {
        if (free_head >= 0) {
            const int32_t blk = free_head;
            int32_t* w = reinterpret_cast<int32_t*>(&S.pool[blk]);
            const int32_t cnt = w[1];
            if (cnt > 0) { const int32_t s = w[1 + cnt]; w[1] = cnt - 1; return s; }
            free_head = w[0];
            return blk;
        }
        if (chunk_next >= chunk_end) {
            unsigned long long c = 0;
            if (lane_id() == 0) c = atomicAdd(&S.ctr[ci(C_POOL_BUMP)], (unsigned long long)POOL_CHUNK);
            c = bcast64(c);
            if (c + POOL_CHUNK > S.pool_cap) { die(KME_E_CAPACITY, KME_D_CAP_POOL, idx); return -1; }
            chunk_next = (int32_t)c;
            chunk_end = (int32_t)(c + POOL_CHUNK);
        }
        return chunk_next++;
    }
    KDEV void free_slot(int32_t s) {
        S.pool[s].live = 0;
        if (free_head >= 0) {                               // room in the head block
            int32_t* w = reinterpret_cast<int32_t*>(&S.pool[free_head]);
            const int32_t cnt = w[1];
            if (cnt < FBLK - 1) { w[2 + cnt] = s; w[1] = cnt + 1; return; }
        }
        int32_t* w = reinterpret_cast<int32_t*>(&S.pool[s]);   // s becomes the head block
        w[0] = free_head; w[1] = 0;
        free_head = s;
    }

    // ---------------- exact ledger (EXACT only): device hash tables, one wavefront, plain loads
    KDEV int32_t bal_find(int64_t aid) const {
        uint32_t h = (uint32_t)mix64((uint64_t)aid) & S.bal_mask;
        for (uint32_t p = 0; p <= S.bal_mask; ++p) {
            if (S.bal_state[h] == 0) return -1;
            if (S.bal_key[h] == aid) return (int32_t)h;
            h = (h + 1) & S.bal_mask;
        }
        return -1;
    }
    KDEV void bal_insert(int64_t aid, int64_t v, int64_t idx) {
        uint32_t h = (uint32_t)mix64((uint64_t)aid) & S.bal_mask;
        while (S.bal_state[h] != 0) h = (h + 1) & S.bal_mask;
        S.bal_key[h] = aid; S.bal_val[h] = v; S.bal_state[h] = 1;
        const unsigned long long used = S.ctr[ci(C_BAL_USED)] + 1;
        S.ctr[ci(C_BAL_USED)] = used;
        if (used * 2 > (unsigned long long)S.bal_mask + 1) die(KME_E_CAPACITY, KME_D_CAP_LEDGER, idx);
    }
    KDEV int32_t pos_find(int64_t k0, int64_t k1, int32_t* free_slot_out) const {
        uint32_t h = (uint32_t)mix64((uint64_t)k0 * 0x9e3779b97f4a7c15ull ^ mix64((uint64_t)k1)) & S.pos_mask;
        int32_t first_free = -1;
        for (uint32_t p = 0; p <= S.pos_mask; ++p) {
            const uint32_t st = S.pos[h].state;
            if (st == 0) { if (free_slot_out) *free_slot_out = first_free >= 0 ? first_free : (int32_t)h; return -1; }
            if (st == 1) {
                const PosEntry& e = S.pos[h];
                if (e.k0 == k0 && e.k1 == k1) return (int32_t)h;
            } else if (first_free < 0) {
                first_free = (int32_t)h;
            }
            h = (h + 1) & S.pos_mask;
        }
        if (free_slot_out) *free_slot_out = first_free;
        return -1;
    }
    KDEV bool pos_get(int64_t k0, int64_t k1, int64_t& v0, int64_t& v1) const {
        const int32_t h = pos_find(k0, k1, nullptr);
        if (h < 0) return false;
        v0 = S.pos[h].v0; v1 = S.pos[h].v1;
        return true;
    }
    KDEV void pos_put(int64_t k0, int64_t k1, int64_t v0, int64_t v1, int64_t idx) {
        int32_t fs = -1;
        int32_t h = pos_find(k0, k1, &fs);
        if (h < 0) {
            if (fs < 0) { die(KME_E_CAPACITY, KME_D_CAP_LEDGER, idx); return; }
            h = fs;
            if (S.pos[h].state == 0) {
                const unsigned long long used = S.ctr[ci(C_POS_USED)] + 1;
                S.ctr[ci(C_POS_USED)] = used;
                if (used * 4 > ((unsigned long long)S.pos_mask + 1) * 3) { die(KME_E_CAPACITY, KME_D_CAP_LEDGER, idx); return; }
            }
            S.pos[h].k0 = k0; S.pos[h].k1 = k1; S.pos[h].state = 1;
        }
        S.pos[h].v0 = v0; S.pos[h].v1 = v1;
    }
    KDEV void pos_del(int64_t k0, int64_t k1) {
        const int32_t h = pos_find(k0, k1, nullptr);
        if (h >= 0) S.pos[h].state = 2;
    }

    // createBalance, KP:131-138
    KDEV bool create_balance(int64_t aid, int64_t idx) {
        if (bal_find(aid) < 0) { bal_insert(aid, 0, idx); return !dead; }
        return false;
    }
    // transfer, KP:140-146
    KDEV bool transfer(int64_t aid, int32_t size) {
        const int32_t h = bal_find(aid);
        if (h < 0) return false;
        const int64_t b = S.bal_val[h];
        if (b < (int64_t)jineg(size)) return false;
        S.bal_val[h] = jladd(b, (int64_t)size);
        return true;
    }
    // checkBalance, KP:167-182
    KDEV bool check_balance(const Taker& t, int64_t idx) {
        const int32_t h = bal_find(t.aid);
        if (h < 0) return false;
        const int64_t balance = S.bal_val[h];
        const bool is_buy = t.action == BUY;
        const int32_t size = jimul(t.size, is_buy ? 1 : -1);
        int64_t pa = 0, pv = 0;
        const bool has_pos = pos_get(t.aid, t.sid, pa, pv);
        const int64_t available = has_pos ? pv : 0;
        const int64_t adj = is_buy ? lmax(lmin(available, 0), (int64_t)jineg(size))
                                   : lmin(lmax(available, 0), (int64_t)jineg(size));
        const int64_t risk = jlmul(jladd((int64_t)size, adj), (int64_t)(is_buy ? t.price : jisub(t.price, 100)));
        if (balance < risk) return false;
        S.bal_val[h] = jlsub(balance, risk);
        if (adj != 0) {
            if (!has_pos) { die(KME_E_DOMAIN, KME_D_NPE_POSITION, idx); return false; }
            pos_put(t.aid, t.sid, pa, jlsub(available, adj), idx);
        }
        return true;
    }
    // fillOrder, KP:276-287 (setPosition(UUID,...) writes under the VALUE as key, KP:434-436)
    KDEV void fill_order(int32_t action, int64_t aid, int64_t sid, int32_t price, int32_t fsize, int64_t idx) {
        const int32_t size = jimul(fsize, action == BOUGHT ? 1 : -1);
        int64_t pa, pv;
        if (!pos_get(aid, sid, pa, pv)) {
            pos_put(aid, sid, (int64_t)size, (int64_t)size, idx);
        } else {
            const int64_t np = jladd(pa, (int64_t)size);
            if (np == 0) pos_del(pa, pv);
            else pos_put(pa, pv, np, jladd(pv, (int64_t)size), idx);
        }
        if (dead) return;
        const int32_t h = bal_find(aid);
        if (h < 0) { die(KME_E_DOMAIN, KME_D_NPE_BALANCE, idx); return; }
        S.bal_val[h] = jladd(S.bal_val[h], (int64_t)jimul(size, price));
    }
    // postRemoveAdjustments, KP:325-333
    KDEV void post_remove_adjustments(const Node& o, int64_t idx) {
        const bool is_buy = o.action == BUY;
        const int32_t size = jimul(o.size, is_buy ? 1 : -1);
        int64_t pa = 0, pv = 0;
        const bool has_pos = pos_get(o.aid, o.sid, pa, pv);
        const int64_t blocked = has_pos ? jlsub(pa, pv) : 0;
        const int64_t adj = is_buy ? lmax(lmin(blocked, 0), (int64_t)jineg(size))
                                   : lmin(lmax(blocked, 0), (int64_t)jineg(size));
        const int32_t h = bal_find(o.aid);
        if (h < 0) { die(KME_E_DOMAIN, KME_D_NPE_BALANCE, idx); return; }
        const int64_t delta = jlmul(jladd((int64_t)size, adj), (int64_t)(is_buy ? o.price : jisub(o.price, 100)));
        S.bal_val[h] = jladd(S.bal_val[h], delta);
        if (adj != 0) {
            if (!has_pos) { die(KME_E_DOMAIN, KME_D_NPE_POSITION, idx); return; }
            pos_put(pa, pv, pa, jladd(pv, adj), idx);
        }
    }
    // payout, KP:148-165, after removeSymbol returned true (symbol absent): settles every
    // Positions entry whose key lsb == sid.  All 64 lanes sweep the table.
    KDEV void payout_settle(int64_t sid, int32_t size, int64_t idx) {
        const int lane = lane_id();
        bool bad = false;
        for (uint32_t h = lane; h <= S.pos_mask; h += 64)
            if (S.pos[h].state == 1 && S.pos[h].k1 == sid && bal_find(S.pos[h].k0) < 0) bad = true;
        if (__ballot(bad)) { die(KME_E_DOMAIN, KME_D_NPE_BALANCE, idx); return; }
        for (uint32_t h = lane; h <= S.pos_mask; h += 64) {
            if (S.pos[h].state == 1 && S.pos[h].k1 == sid) {
                const int32_t b = bal_find(S.pos[h].k0);
                atomicAdd((unsigned long long*)&S.bal_val[b], (unsigned long long)jlmul(S.pos[h].v0, (int64_t)size));
            }
        }
        __threadfence();   // the atomics ran at L2: drop this CU's L1 copies before re-reading
        __builtin_amdgcn_wave_barrier();
        for (uint32_t h = lane; h <= S.pos_mask; h += 64)
            if (S.pos[h].state == 1 && S.pos[h].k1 == sid) S.pos[h].state = 2;
        __threadfence();   // other lanes' tombstones become visible to every lane
        __builtin_amdgcn_wave_barrier();
    }

    // ---------------- trades
    // the trades go straight to their arrival-order slots: the epoch runs in one wavefront
    KDEV void emit(uint32_t i, const Node& m, int32_t ts) {
        if (tnext >= io.trades_cap) { die(KME_E_CAPACITY, KME_D_CAP_TRADES, i); return; }
        if (lane_id() == 0) {
            TradeRec& r = io.trades[tnext];
            r.moid = m.oid; r.maid = m.aid; r.msid = m.sid; r.mprice = m.price; r.size = ts;
        }
        tnext++;
    }

    // ---------------- tryMatch, KP:225-263
    // The loop test of KP:237 parses as ((size > 0 && isBuy) ? maker.price <= P : maker.price >= P)
    // (H3).  The level being swept lives in registers and is written back once where the sweep
    // stops; a level swept empty is not written (its bit is cleared, its fields are dead until a
    // rest rewrites them).
    KDEV bool crosses(bool is_buy, int32_t size, int32_t mprice, int32_t P) const {
        return (size > 0 && is_buy) ? mprice <= P : mprice >= P;
    }
    // executeTrade (KP:265-274): the trade record, and in EXACT mode both fillOrder calls.
    KDEV void trade(uint32_t i, uint32_t& ntr, const Node& m, const Taker& t, int32_t ts, bool is_buy) {
        emit(i, m, ts);
        ntr++;
        if (!dead) {
            fill_order(is_buy ? SOLD : BOUGHT, m.aid, m.sid, 0, ts, i);                              // maker fill
            if (!dead) fill_order(is_buy ? BOUGHT : SOLD, t.aid, t.sid, jisub(t.price, m.price), ts, i);  // taker fill
        }
    }
    KDEV bool try_match(uint32_t i, Taker& t, uint32_t& ntr) {
        const bool is_buy = t.action == BUY;
        const int64_t key = jlmul(t.sid, is_buy ? 1 : -1);
        const int os = jlneg(key) < 0 ? 1 : 0;           // opposite book (the same book for sid 0)
        uint64_t lo = bl(os), hi = bm(os);
        int32_t pb = is_buy ? min_price_ptr(lo, hi) : max_price_ptr(lo, hi);
        if (pb == -1) return false;
        if (!check_bit(lo, hi, pb)) { die(KME_E_DOMAIN, KME_D_NPE_BUCKET, i); return false; }
        const int32_t P = t.price;
        if (!crosses(is_buy, t.size, pb, P)) return t.size == 0;
        Level* L = lv(os, pb);
        int32_t ms = L->head;
        int64_t lqty = L->qty;
        if (ms < 0) { die(KME_E_DOMAIN, KME_D_NPE_ORDER, i); return false; }
        Node m = ld_node(ms);
        bool head_moved = false;                             // ms is a later maker of level L
        for (;;) {
            const int32_t ts = imin(t.size, m.size);
            const int32_t msize = jisub(m.size, ts);
            t.size = jisub(t.size, ts);
            lqty -= ts;
            if (msize != 0) {                                // maker stays, partially filled (KP:255-261)
                trade(i, ntr, m, t, ts, is_buy);
                if (dead) return false;
                S.pool[ms].size = msize;
                if ((msize | m.size) < 0) nneg_add((msize < 0 ? 1 : 0) - (m.size < 0 ? 1 : 0));
                if (head_moved) { L->head = ms; S.pool[ms].prev = -1; }
                L->qty = lqty;
                return t.size == 0;
            }
            // maker consumed: orders.delete (KP:243)
            if (m.size < 0) nneg_add(-1);
            int32_t nms;
            bool same_level = m.next >= 0;
            if (same_level) {
                nms = m.next;
                if (!crosses(is_buy, t.size, m.price, P)) {  // stops before the next maker of L
                    trade(i, ntr, m, t, ts, is_buy);
                    if (dead) return false;
                    free_slot(ms);
                    L->head = nms; S.pool[nms].prev = -1;                    L->qty = lqty;
                    return t.size == 0;
                }
            } else {                                         // level exhausted (KP:244-253)
                unset_bit(lo, hi, m.price);
                set_bm(os, lo, hi);
                pb = is_buy ? min_price_ptr(lo, hi) : max_price_ptr(lo, hi);
                const bool go = pb != -1 && check_bit(lo, hi, pb) && crosses(is_buy, t.size, pb, P);
                if (!go) {
                    trade(i, ntr, m, t, ts, is_buy);
                    if (dead) return false;
                    free_slot(ms);
                    if (pb != -1 && !check_bit(lo, hi, pb)) { die(KME_E_DOMAIN, KME_D_NPE_BUCKET, i); return false; }
                    return t.size == 0;
                }
                L = lv(os, pb);
                nms = L->head; lqty = L->qty;
                if (nms < 0) { die(KME_E_DOMAIN, KME_D_NPE_ORDER, i); return false; }
            }
            const Node nm = ld_node(nms);                   // in flight during this trade's stores
            trade(i, ntr, m, t, ts, is_buy);
            if (dead) return false;
            free_slot(ms);
            head_moved = same_level;
            m = nm;
            ms = nms;
        }
    }

    // ---------------- addOrder, KP:200-223 (after the book-exists and balance checks)
    KDEV void rest(uint32_t i, const Taker& t, bool& has_prev, int64_t& prev_oid) {
        const int64_t key = jlmul(t.sid, t.action == BUY ? 1 : -1);
        const int s = key < 0 ? 1 : 0;
        uint64_t lo = bl(s), hi = bm(s);                     // books.get(sid) again (KP:205)
        const int32_t p = t.price;
        if (p < 0 || p > 126) { die(KME_E_DOMAIN, KME_D_PRICE, i); return; }
        const int32_t slot = alloc_slot(i);
        if (dead) return;
        Level* L = lv(s, p);
        int32_t nprev = -1;
        has_prev = false;
        prev_oid = 0;
        if (!check_bit(lo, hi, p)) {                        // new bucket (oid, oid), set bit (KP:209-211)
            L->head = slot; L->tail = slot; L->qty = t.size; L->tail_oid = t.oid;
            set_bit(lo, hi, p);
            set_bm(s, lo, hi);
        } else {                                             // append at the tail (KP:213-219)
            const int32_t tl = L->tail;
            S.pool[tl].next = slot;
            has_prev = true;
            prev_oid = L->tail_oid;
            nprev = tl;
            L->tail = slot; L->tail_oid = t.oid; L->qty += t.size;
        }
        Node* nd = &S.pool[slot];
        nd->oid = t.oid; nd->aid = t.aid; nd->sid = t.sid; nd->prev_oid = prev_oid;
        nd->size = t.size; nd->next = -1; nd->prev = nprev; nd->group = g;
        nd->price = p; nd->action = t.action; nd->live = 1; nd->_pad = 0;
        S.rest_slot[i] = slot;
        if (t.size < 0) nneg_add(1);
        if (p > 100) note_odd();
    }

    // ---------------- removeOrder, KP:289-323
    KDEV bool remove_order(const Rec& r) {
        const uint32_t i = r.i;
        const int64_t tgt = r.tgt;
        int32_t slot = -1;
        if (tgt >= 0) slot = (int32_t)tgt;
        else if (tgt <= -2) slot = S.rest_slot[-(tgt + 2)];
        if (slot < 0) return false;
        const Node o = ld_node(slot);
        if (!o.live || o.oid != r.oid) return false;       // orders.get(oid) == null
        if (o.aid != r.aid) return false;                  // order.aid != aid (KP:291)
        if (!exists) { die(KME_E_DOMAIN, KME_D_NPE_BOOK, i); return false; }
        const int64_t key = jlmul(o.sid, o.action == BUY ? 1 : -1);
        const int s = key < 0 ? 1 : 0;
        Level* L = lv(s, o.price);
        if (o.prev < 0 && o.next < 0) {
            uint64_t lo = bl(s), hi = bm(s);
            unset_bit(lo, hi, o.price);
            set_bm(s, lo, hi);
        } else if (o.prev < 0) {
            L->head = o.next;
            S.pool[o.next].prev = -1;
        } else if (o.next < 0) {
            L->tail = o.prev;
            L->tail_oid = o.prev_oid;
            S.pool[o.prev].next = -1;
        } else {
            S.pool[o.prev].next = o.next;
            S.pool[o.next].prev = o.prev;
            S.pool[o.next].prev_oid = o.prev_oid;
        }
        L->qty -= o.size;
        free_slot(slot);
        if (o.size < 0) nneg_add(-1);
        post_remove_adjustments(o, i);
        return !dead;
    }

    // removeSymbol (KP:193-198) for an existing group: 0 = returns false (empty book), 2 = never
    // returns (removeAllOrders loops, KP:341-353).  Absent symbols return true.
    KDEV int remove_symbol_existing(int64_t sid) const {
        const int s = sid < 0 ? 1 : 0;
        return (bl(s) == 0 && bm(s) == 0) ? 0 : 2;
    }

    // ---------------- one record of this group (MatchingEngine.process, KP:96-126)
    KDEV Out process(const Rec& r) {
        const uint32_t i = r.i;
        const int32_t a = r.action;
        bool ok = false, has_prev = false;
        int64_t prev_oid = 0;
        int32_t out_size = r.size;
        uint32_t ntr = 0;
        Out out;
        out.action = a; out.size = r.size; out.prev = 0; out.has_prev = false; out.rested = false; out.ntr = 0;
        io.trade_off[i] = tnext;
        switch (a) {
        case ADD_SYMBOL:                                    // addSymbol, KP:184-191
            if (!exists) { exists = 1; b0l = b0m = b1l = b1m = 0; ok = true; }
            break;
        case REMOVE_SYMBOL:
        case PAYOUT: {
            if (exists) {
                if (remove_symbol_existing(r.sid) == 2) { die(KME_E_DOMAIN, KME_D_HANG, i); return out; }
                ok = false;                                 // removeAllOrders(sid) returned true
            } else {
                ok = a == REMOVE_SYMBOL;
                if (a == PAYOUT) {
                    payout_settle(r.sid, r.size, i);
                    if (dead) return out;
                }
            }
            if (a == PAYOUT) ok = false;                    // result ignored (KP:113-115)
            break;
        }
        case BUY:
        case SELL: {
            if (!exists) break;                             // books.get(sid) == null
            Taker t;
            t.action = a; t.price = r.price; t.size = r.size; t._pad = 0;
            t.oid = r.oid; t.aid = r.aid; t.sid = r.sid;
            if (!check_balance(t, i)) { if (dead) return out; break; }
            const bool filled = try_match(i, t, ntr);
            if (dead) return out;
            if (!filled) { rest(i, t, has_prev, prev_oid); if (dead) return out; out.rested = true; }
            ok = true;
            out_size = t.size;
            break;
        }
        case CANCEL:
            ok = remove_order(r);
            if (dead) return out;
            break;
        default:
            break;
        }
        out.action = ok ? a : (int32_t)REJECT;
        out.size = out_size;
        out.prev = has_prev ? prev_oid : 0;
        out.has_prev = has_prev;
        out.ntr = ntr;
        return out;
    }

};

// ================================================================== (2)+(3) FUNDED matching
// One 64-lane wavefront owns one symbol group |sid| for the epoch (books +g and -g, KP:184-191;
// sid 0 is one shared book, H4) and runs MatchingEngine.process (KP:96-126) over the group's
// records in arrival order.  The program is wave-uniform: every loaded value that steers control
// flow goes through readfirstlane / readlane into an SGPR, so branches are scalar (s_cbranch on
// SCC), never exec-masked.  Where the book lives:
//   * price levels of both books (Buckets, KP:42-45) in LDS as structure of arrays over prices
//     0..100 (the FUNDED price domain, checked by k_emap): occupied ones are staged in when the
//     group starts and written back when it ends;
//   * the two 128-bit level bitmaps (Books, KP:38-41), free-list heads and counters in SGPRs;
//   * resting orders (Orders, KP:46-49) in the HBM node pool, one 64-byte line each, read only to
//     trade against a maker or to cancel (a cancel's node is prefetched with its batch);
//   * records arrive 64 at a time, one per lane; the OUT fields and the trades collect in lanes
//     and leave in coalesced stores (one per field per batch, one per 64 trades).
constexpr int LVP = 101;          // LDS level entries per book side: prices 0..100
constexpr int FSTK = 128;         // LDS free-slot stack
constexpr int TRD = 32;           // trades staged in LDS between reservations (GroupWave::emit)
constexpr int DIRTY_WORDS = 64;   // 2048-bit filter of node slots written since the batch prefetch
constexpr int FAST_EVCAP = 64;    // events of one fast segment (GroupWave::fast_segment): one lane each

struct GroupLds {
    int2 ht[2 * LVP];             // head / tail node slot of level (side, price)
    int64_t qty[2 * LVP];         // resting quantity (market data; the reference keeps none)
    int64_t toid[2 * LVP];        // oid of the tail node = OUT.prev of an append (KP:213-217)
    int32_t fstack[FSTK];
    uint32_t dirty[DIRTY_WORDS];
    uint64_t bmap[4];             // level bitmaps: book +g (lsb, msb), book -g (lsb, msb)
    int32_t gs[8];                // exists, free-list head block, bump chunk next / end, free-stack top, staged trades
    int4 trd[2 * TRD];            // trade k: (maker oid, maker aid), (price | sid < 0 << 8, size, seq, ord);
                                  // during a fast segment (emptied first): record k's (oid, aid) at trd[k]
    int4 rin[64];                 // fast segment: record k's (input index, PRec w0, rest size, -)
    int4 ev[FAST_EVCAP];          // fast segment: its events in arrival order (GroupWave::fast_segment), then
                                  // their results (trades; has_prev, prev oid)
};

// Two-wavefront k_match (few busy groups: C2, C4, C5): wave 0 runs the batch loop, the fast
// segments' aggregate passes and the serial path; wave 1 runs the segments' level steps and
// epilogues one segment behind, so a busy group costs max(pass, level step) per record instead of
// their sum (GroupWave::fast_segment<true>, GroupWave::run_levels).  They meet at one workgroup
// barrier per segment ("phase"); what wave 1 needs crosses in this block.
constexpr int LFREE = 64;         // node slots wave 1 frees per segment before it chains them as blocks
struct TwoLds {
    // double-buffered by phase parity (the next batch's first segment reuses the record lanes of the
    // segment wave 1 may still have in hand):
    int4 ev[2][FAST_EVCAP];       // a segment's events
    int4 rin[2][64];              // record lane k: (input index, PRec w0, rest size, -)
    int4 rid[2][64];              // record lane k: (oid lo, oid hi, aid lo, aid hi)
    int4 rec[2][64];              // record lane k: the pass's (action | flags << 16, events, rest slot, BUY/SELL)
    uint64_t cb[4];               // levels the segment wave 1 has in hand takes from (the pass's c*)
    int32_t fv[64];               // lane k: the prefetched victim that segment's record k removes
    uint64_t bcb[4];              // ... and the same of the segment wave 1 had in hand when the batch's
    int32_t bfv[64];              //     prefetch ran (its writes may predate the batch's dirty filter)
    uint32_t tb[8], btb[8];       // levels (side * 128 + price) with events in those two segments
    int32_t seg[2][4];            // per buffer: first record, end record, events, command
    int32_t lfree[2][LFREE];      // per buffer: slots wave 1 freed
    int32_t lfcnt[2], lch_head[2], lch_tail[2];   // ... their count, and the one-slot blocks past LFREE
    int32_t lerr;                 // wave 1 faulted (its records' fault is raised; wave 0 stops)
};
enum { TW_NONE = 0, TW_SEG = 1, TW_EXIT = 2 };
// The phase barrier of the two wavefronts: each one's memory operations complete before it (the
// epilogue's rest slots and nodes are read by wave 0's serial path -- through the scalar path, from
// L2 -- and its batch prefetch; wave 0's serial-path nodes by wave 1's next level step).  Both waves
// run on one CU and share its L1, so no cache maintenance is needed.
KDEV void two_barrier() {
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
}

KDEV int32_t U32(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }
// A constant-space view of *p that the compiler cannot hoist: every field read through it is a
// scalar load at the point of use (GroupWave::cold).
template <class T> KDEV const KC T& opaque_const(const T* p) {
    uint64_t v = (uint64_t)(uintptr_t)p;
    asm volatile("" : "+s"(v));
    return *(const KC T*)(uintptr_t)bcast64(v);
}

// A whole 64-byte node into 16 SGPRs through the scalar memory path.  Vector loads and stores share
// one in-order counter (vmcnt), so a vector load of a maker waits for every store the wavefront
// issued before it; a scalar load is counted by lgkmcnt and does not.  glc: the scalar cache is
// bypassed (read from L2), so the line is never stale w.r.t. this wavefront's completed vector
// stores; nodes written since the last vmcnt(0) (the batch dirty filter) take the vector path.
// The wait sits in the same asm block: the compiler does not track this lgkmcnt event.
typedef int32_t v16i __attribute__((ext_vector_type(16)));
typedef int32_t v8i __attribute__((ext_vector_type(8)));
// the first 32 bytes (oid, aid, sid, size, next): a maker
KDEV v8i sload_maker(const KG Node* p) {
    const uint64_t a = bcast64((uint64_t)(uintptr_t)p);
    v8i r;
    asm volatile("s_load_dwordx8 %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "=s"(r) : "s"(a) : "memory");
    return r;
}
KDEV v16i sload_node(const KG Node* p) {
    const uint64_t a = bcast64((uint64_t)(uintptr_t)p);   // an SGPR pair even where the compiler
    v16i r;                                                // would keep the address in VGPRs
    asm volatile("s_load_dwordx16 %0, %1, 0x0 glc\n\ts_waitcnt lgkmcnt(0)" : "=s"(r) : "s"(a) : "memory");
    return r;
}
KDEV int64_t U64(int64_t v) { return (int64_t)bcast64((uint64_t)v); }
KDEV int64_t mk64(int32_t lo, int32_t hi) { return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo); }
KDEV int32_t lo32(int64_t v) { return (int32_t)(uint32_t)(uint64_t)v; }
KDEV int32_t hi32(int64_t v) { return (int32_t)(uint32_t)((uint64_t)v >> 32); }
// Side of book key sid * (BUY ? 1 : -1) (KP:201, 292): 1 when the key is negative.  For the
// records and nodes of a symbol group sid is +-g with g < 2^24, so this is a sign test (no 64-bit
// multiply); sid 0 is the shared book of side 0 (H4).
KDEV int book_side(int64_t sid, bool is_buy) { return (sid != 0 && ((hi32(sid) < 0) != !is_buy)) ? 1 : 0; }

// Overflow path of GroupWave::flush_trades: marks this reservation's share of the shard region
// as holes and reserves n records in the overflow region; ~0 when that is full too.
__device__ __attribute__((noinline)) uint64_t trade_overflow(KG TradeTmp* ttmp, KG unsigned long long* ctr, uint32_t tbase,
                                                             uint32_t tshard_cap, uint32_t ttmp_cap, uint64_t base, uint32_t n) {
    const int lane = lane_id();
    if (base < tshard_cap && (uint64_t)lane < tshard_cap - base && (uint32_t)lane < n) ttmp[tbase + base + lane].seq = -1;
    unsigned long long ob = 0;
    if (lane == 0) ob = atomicAdd(&ctr[ci(C_TTMP)], (unsigned long long)n);
    ob = bcast64(ob);
    if (ob + n > ttmp_cap) return ~(uint64_t)0;
    return (uint64_t)TSHARDS * tshard_cap + ob;
}

// A maker as tryMatch reads it (KP:236-241, 266): oid, aid, sid, size, next.  Lane q of the
// wavefront loads 16-byte piece q of the 64-byte node; readlane picks the fields.
struct Maker {
    int64_t oid, aid;
    int32_t sneg;                 // sid < 0: a maker of group g has sid = +-g (sid 0 for group 0)
    int32_t size, next;
};
// A resting order as removeOrder reads it (KP:290-323), already validated against the cancel.
struct Victim {
    int32_t ok;                   // live, same oid and same aid (KP:290-291)
    int32_t side, price, size, next, prev;
    int32_t sell, sid_neg;        // the order's action (BUY / SELL) and sid sign (sid = +-g)
    int64_t prev_oid;
};

// 64 records staged across the lanes (lane l = record k0 + l of the group's segment), with the
// node of each cancel's target prefetched: one gather per 64 records instead of dependent round
// trips per record.
struct Lanes {
    uint32_t i;
    int32_t w0, size, tgt;        // PRec word 0 (action | price << 8 | acct_ok << 16 | sid < 0 << 17)
    int64_t oid, aid;
    int32_t pf_slot, pf_meta, pf_size, pf_next, pf_prev;   // pf_meta = price | side << 8 | sell << 9 | sid<0 << 10 | ok << 11
                                                           // (pf_slot < 0: rest_slot of this epoch's target)
    int64_t pf_poid;
    int32_t vl;                   // a cancel's target level from k_route (price | side << 8 | 1 << 9), or 0
};

// Diagnostic stamp slots of the -DKME_STAMPS build (cycles unless named n_*), per group.
enum Stamp : int {
    ST_GROUP_IN = 0, ST_BATCH, ST_TRADE_REC, ST_REST_REC, ST_CANCEL_REC, ST_OTHER_REC, ST_GROUP_OUT, ST_KERNEL,
    ST_N_TRADE_REC, ST_N_REST_REC, ST_N_CANCEL_REC, ST_MAKER_WAIT, ST_N_MAKER, ST_VICTIM_WAIT, ST_N_VICTIM, ST_FLUSH,
    ST_REST_ALLOC, ST_REST_LEVEL, ST_REST_NODE, ST_REC_PICK, ST_REC_OUT, ST_TM_PRE, ST_REST_PRE,
    ST_FAST, ST_N_FAST_REC, ST_N_FAST_SEG, ST_FAST_PASS, ST_FAST_DRAIN, ST_FAST_LEVEL, ST_FAST_EPI,
    ST_PASS_REST, ST_N_PASS_REST, ST_PASS_SWEEP, ST_N_PASS_SWEEP, ST_PASS_CANCEL, ST_N_PASS_CANCEL,
    ST_PASS_REJECT, ST_N_PASS_REJECT, ST_PASS_ABSORB, ST_N_PASS_ABSORB,
    ST_N = 40
};

struct GroupWave {
    KG Node* pool;
    KG int32_t* rest_slot;
    const DevState* Sp;           // everything off the per-record path is re-read through cold()
    GroupLds& L;
    const int lane, q;            // q = lane & 3: the node piece this lane loads / stores
    int32_t g;
    uint32_t cur;                 // input index of the record being processed
    bool dead;
    bool seg_retry;               // the last fast segment stopped at a record a new segment may take
    TwoLds* tl = nullptr;         // two-wavefront mode (k_match<true>): the block wave 1 reads
    int kp = 0;                   // wave 0's phase count
    bool lbusy = false;           // wave 1 has a segment to finish
    unsigned long long fastmask = 0;   // records of the batch whose results wave 1 produces
    uint32_t pend_lo = 0, pend_hi = 0; // input indices of the segment wave 1 has in hand
    uint32_t bpend_lo = 1, bpend_hi = 0;   // ... and of the one it had when the batch's prefetch ran
    bool bstale = false;          // that segment existed: the prefetched nodes it wrote are not in the dirty filter
#ifdef KME_STAMPS
    unsigned long long acc[ST_N];
#endif

    KDEV GroupWave(const DevState& S, GroupLds& lds, int32_t gg)
        : pool(S.pool), rest_slot(S.rest_slot), Sp(&S), L(lds),
          lane(lane_id()),
          q(lane_id() & 3), g(gg) {
        cur = 0; dead = false;
        KST(for (int k = 0; k < ST_N; ++k) acc[k] = 0;)
    }

    // Fields used off the per-record path (level and group-state homes, trade scratch, counters,
    // capacities) are not kept in registers across the matching loops: the wavefront's live
    // uniform state already exceeds the SGPR file, and every register such a field pins is one
    // more spill.  cold() hands out the state through an opaque constant-space pointer, so each
    // use is a scalar load (scalar cache) at the point of use, never hoisted.
    KDEV const KC DevState& cold() const { return opaque_const(Sp); }
    KDEV KG Level* lev() const { return cold().lev + (size_t)g * 2 * NLEV; }
    KDEV KG GroupState* gst() const { return cold().grp + g; }
    KDEV KG unsigned long long* ctr() const { return cold().ctr; }
    KDEV KG unsigned long long* tsh() const { return cold().tsh + (size_t)(g & (TSHARDS - 1)) * CTR_STRIDE; }
    KDEV void die(int status, int detail) { raise_wave(ctr(), status, detail, (int64_t)cur); dead = true; }
    // The level bitmaps live in LDS, not in SGPRs: as loop-carried SSA values they cost a copy per
    // bitmap at every join of the record loop, and 8 SGPRs of a file that already spills.
    KDEV uint64_t bl(int side) const { return U64((int64_t)L.bmap[2 * side]); }
    KDEV uint64_t bm(int side) const { return U64((int64_t)L.bmap[2 * side + 1]); }
    KDEV void set_bm(int side, uint64_t l, uint64_t m) { L.bmap[2 * side] = l; L.bmap[2 * side + 1] = m; }
    // so do the group's rarely changing scalars (GroupState words 8..11)
    enum { GS_EXISTS = 0, GS_FREE_HEAD, GS_CHUNK_NEXT, GS_CHUNK_END, GS_FSP, GS_TCNT };
    KDEV int32_t gsv(int k) const { return U32(L.gs[k]); }
    KDEV void set_gs(int k, int32_t v) { L.gs[k] = v; }
    KDEV void sync_lds() {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }

    // ---------------- group state in and out
    KDEV void load_group() {
        const int4 v = reinterpret_cast<const KG int4*>(gst())[q];
        set_bm(0, (uint64_t)mk64(rl32(v.x, 0), rl32(v.y, 0)), (uint64_t)mk64(rl32(v.z, 0), rl32(v.w, 0)));
        set_bm(1, (uint64_t)mk64(rl32(v.x, 1), rl32(v.y, 1)), (uint64_t)mk64(rl32(v.z, 1), rl32(v.w, 1)));
        set_gs(GS_EXISTS, rl32(v.x, 2)); set_gs(GS_FREE_HEAD, rl32(v.y, 2));
        set_gs(GS_CHUNK_NEXT, rl32(v.z, 2)); set_gs(GS_CHUNK_END, rl32(v.w, 2));
        set_gs(GS_FSP, 0); set_gs(GS_TCNT, 0);
        stage_levels(true);
    }
    KDEV void store_group() {
        stage_levels(false);
        const int fsp = gsv(GS_FSP);
        if (fsp > 0) spill_blocks(0, fsp);
        const bool q0 = (q & 1) != 0, q1 = (q & 2) != 0;
        const uint64_t b0l = bl(0), b0m = bm(0), b1l = bl(1), b1m = bm(1);
        const int32_t x = q1 ? gsv(GS_EXISTS) : (q0 ? lo32((int64_t)b1l) : lo32((int64_t)b0l));
        const int32_t y = q1 ? gsv(GS_FREE_HEAD) : (q0 ? hi32((int64_t)b1l) : hi32((int64_t)b0l));
        const int32_t z = q1 ? gsv(GS_CHUNK_NEXT) : (q0 ? lo32((int64_t)b1m) : lo32((int64_t)b0m));
        const int32_t w = q1 ? gsv(GS_CHUNK_END) : (q0 ? hi32((int64_t)b1m) : hi32((int64_t)b0m));
        if (lane < 3) reinterpret_cast<KG int4*>(gst())[lane] = make_int4(x, y, z, w);
    }
    // Occupied levels of both books move between HBM (Level, 32 B) and LDS in one parallel pass:
    // lane l takes prices l and l + 64.  An unoccupied level's fields are dead until a rest
    // rewrites all of them, so only occupied ones move.
    KDEV void stage_levels(bool in) {
#pragma unroll
        for (int side = 0; side < 2; ++side) {
            const uint64_t l = bl(side), m = bm(side);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int p = lane + 64 * h;
                if (p <= 100 && check_bit(l, m, p)) {
                    const int li = side * LVP + p;
                    KG int4* gl = reinterpret_cast<KG int4*>(&lev()[side * NLEV + p]);
                    if (in) {
                        const int4 x0 = gl[0], x1 = gl[1];
                        L.ht[li] = make_int2(x0.x, x0.y);
                        L.qty[li] = mk64(x1.x, x1.y);
                        L.toid[li] = mk64(x1.z, x1.w);
                    } else {
                        const int2 ht = L.ht[li];
                        const int64_t qt = L.qty[li], to = L.toid[li];
                        gl[0] = make_int4(ht.x, ht.y, 0, 0);
                        gl[1] = make_int4(lo32(qt), hi32(qt), lo32(to), hi32(to));
                    }
                }
            }
        }
        sync_lds();
    }

    // ---------------- node slots
    // Free slots: an LDS stack; the group's free slots kept between epochs are a list of BLOCKS,
    // each a free 64-byte slot holding up to FBLK - 1 more free slot ids (word 0 = next block,
    // word 1 = count, words 2.. = ids; word 14 = Node::live stays 0).  One load refills the stack
    // with a whole block.  Last resort: a chunk of the pool's bump counter.
    KDEV int32_t alloc_slot() {
        const int fsp = gsv(GS_FSP);
        if (fsp > 0) { set_gs(GS_FSP, fsp - 1); return U32(L.fstack[fsp - 1]); }
        const int32_t blk = gsv(GS_FREE_HEAD);
        if (blk >= 0) {
            const int32_t w = lane < 2 + FBLK - 1 ? reinterpret_cast<const KG int32_t*>(&pool[blk])[lane] : 0;
            const int32_t nxt = rl32(w, 0), cnt = rl32(w, 1);
            if (lane >= 2 && lane < 2 + cnt) L.fstack[lane - 2] = w;
            sync_lds();
            set_gs(GS_FSP, cnt);
            set_gs(GS_FREE_HEAD, nxt);
            return blk;
        }
        int32_t cn = gsv(GS_CHUNK_NEXT);
        if (cn >= gsv(GS_CHUNK_END)) {
            unsigned long long c = 0;
            KG unsigned long long* bump = &ctr()[ci(C_POOL_BUMP)];   // (no asm inside a lane branch)
            if (lane == 0) c = atomicAdd(bump, (unsigned long long)POOL_CHUNK);
            c = bcast64(c);
            if (c + POOL_CHUNK > cold().pool_cap) { die(KME_E_CAPACITY, KME_D_CAP_POOL); return -1; }
            cn = (int32_t)c;
            set_gs(GS_CHUNK_END, (int32_t)(c + POOL_CHUNK));
        }
        set_gs(GS_CHUNK_NEXT, cn + 1);
        return cn;
    }
    KDEV void free_slot(int32_t s) {
        pool[s].live = 0;
        mark_dirty(s);
        if (gsv(GS_FSP) == FSTK) spill_blocks(FSTK - FBLK, FSTK);
        const int fsp = gsv(GS_FSP);
        L.fstack[fsp] = s;
        set_gs(GS_FSP, fsp + 1);
    }
    // Writes stack entries [b, e) as blocks of FBLK slots (the last slot of each block holds the
    // others' ids), chained onto the group's block list; all lanes in parallel, stores only.
    KDEV void spill_blocks(int b, int e) {
        sync_lds();
        const int n = e - b;
        const int nblk = (n + FBLK - 1) / FBLK;
        const int32_t fh = gsv(GS_FREE_HEAD);
        for (int k = lane; k < nblk * 14; k += 64) {
            const int blk = k / 14, word = k - blk * 14;
            const int base = b + blk * FBLK;
            const int cnt = imin(FBLK, e - base);                // slots in this block incl. itself
            const int32_t host = L.fstack[base + cnt - 1];
            int32_t v;
            if (word == 0) v = blk == 0 ? fh : L.fstack[base - 1];   // previous block's host
            else if (word == 1) v = cnt - 1;
            else v = word - 2 < cnt - 1 ? L.fstack[base + word - 2] : -1;
            reinterpret_cast<KG int32_t*>(&pool[host])[word] = v;
        }
        const int lb = b + (nblk - 1) * FBLK;
        set_gs(GS_FREE_HEAD, U32(L.fstack[lb + imin(FBLK, e - lb) - 1]));
        set_gs(GS_FSP, b);
    }
    // Per-batch filter of node slots written since the batch's cancel-target prefetch (this wave
    // is the only writer of its LDS, so a plain read-modify-write by all lanes is exact).
    KDEV void mark_dirty(int32_t s) {
        const int w = (s >> 5) & (DIRTY_WORDS - 1);
        // (an atomic: in the two-wavefront mode wave 1 may be marking the same word)
        atomicOr(&L.dirty[w], 1u << (s & 31));
    }
    KDEV bool is_dirty(int32_t s) const { return (U32((int32_t)L.dirty[(s >> 5) & (DIRTY_WORDS - 1)]) >> (s & 31)) & 1; }

    KDEV Maker ld_maker(int32_t s) const {
        Maker m;
        if (!is_dirty(s)) {
            const v8i v = sload_maker(&pool[s]);
            m.oid = mk64(v[0], v[1]); m.aid = mk64(v[2], v[3]); m.sneg = v[5] < 0;
            m.size = v[6]; m.next = v[7];
            return m;
        }
        const int4 v = reinterpret_cast<const KG int4*>(&pool[s])[q];
        m.oid = mk64(rl32(v.x, 0), rl32(v.y, 0));
        m.aid = mk64(rl32(v.z, 0), rl32(v.w, 0));
        m.sneg = rl32(v.y, 1) < 0;
        m.size = rl32(v.z, 1);
        m.next = rl32(v.w, 1);
        return m;
    }

    // ---------------- trades: staged in LDS (trade k in L.trd[2k..2k+1]) until TRD are collected
    // (or the group ends), then one coalesced store per lane.  Every lane stores the same values
    // to the same address (no bank conflict, no exec mask); in lanes they would pin 8 VGPRs for the
    // whole kernel, one wavefront per SIMD less.
    KDEV void emit(uint32_t ord, const Maker& m, int32_t mprice, int32_t ts) {
        const int tcnt = gsv(GS_TCNT);
        L.trd[2 * tcnt] = make_int4(lo32(m.oid), hi32(m.oid), lo32(m.aid), hi32(m.aid));
        L.trd[2 * tcnt + 1] = make_int4(mprice | (m.sneg << 8), ts, (int32_t)cur, (int32_t)ord);
        set_gs(GS_TCNT, tcnt + 1);
        if (tcnt + 1 == TRD) flush_trades();
    }
    // Reserves tcnt records in the group's shard region through the shard's own counter line.  When
    // the shard is full, the part of the region that reservation got ([base, cap)) is marked as
    // holes and the batch goes to the overflow region (trade_overflow: out of line, because a
    // second reservation site inline makes the compiler treat the enclosing loops' exits as
    // divergent and demote their wave-uniform state to VGPRs).
    KDEV void flush_trades() {
        const int tcnt = gsv(GS_TCNT);
        if (tcnt == 0) return;
        unsigned long long base = 0;
        // (plain loads here: an opaque cold() on this path makes the compiler treat the exits of
        // the loops around emit() as divergent)
        const uint32_t tshard_cap = Sp->tshard_cap, tbase = (uint32_t)(g & (TSHARDS - 1)) * tshard_cap;
        KG TradeTmp* ttmp = Sp->ttmp;
        KG unsigned long long* used = &Sp->tsh[(size_t)(g & (TSHARDS - 1)) * CTR_STRIDE + TS_USED];
        if (lane == 0) base = atomicAdd(used, (unsigned long long)tcnt);
        base = bcast64(base);
        size_t pos = (size_t)tbase + base;
        if (base + (unsigned long long)tcnt > tshard_cap) {
            pos = (size_t)bcast64(trade_overflow(ttmp, Sp->ctr, tbase, tshard_cap, Sp->ttmp_cap, base, (uint32_t)tcnt));
            if (pos == ~(size_t)0) { die(KME_E_CAPACITY, KME_D_CAP_TRADES); set_gs(GS_TCNT, 0); return; }
        }
        sync_lds();
        if (lane < tcnt) {
            const int4 a = L.trd[2 * lane], b = L.trd[2 * lane + 1];
            KG int4* r = reinterpret_cast<KG int4*>(&ttmp[pos + lane]);
            r[0] = a;
            r[1] = make_int4(b.z, (int32_t)tt_ordp((uint32_t)b.w, b.x & 0xFF, (b.x >> 8) & 1), b.y, g);
        }
        sync_lds();
        set_gs(GS_TCNT, 0);
    }

    // ---------------- tryMatch, KP:225-263 (FUNDED: sizes >= 0, prices 0..100)
    // The loop test of KP:237 parses as ((size > 0 && isBuy) ? maker.price <= P : maker.price >= P)
    // (H3).  A maker's price is the index of its level, so the test needs no node load; the level
    // being swept stays in SGPRs and is written back once where the sweep stops; a level swept
    // empty is not written at all (its bit is cleared).  The next maker's node is requested before
    // the current trade's stores so that its wait does not include them (vmcnt is in order).
    KDEV static bool crosses(bool is_buy, int32_t size, int32_t mprice, int32_t P) {
        return (size > 0 && is_buy) ? mprice <= P : mprice >= P;
    }
    KDEV bool try_match(int32_t P, int32_t& tsize, bool is_buy, int os, uint32_t& ntr) {
        uint64_t lo = bl(os), hi = bm(os);
        int32_t pb = is_buy ? min_price_ptr(lo, hi) : max_price_ptr(lo, hi);
        if (pb == -1) return false;
        if (!check_bit(lo, hi, pb)) { die(KME_E_DOMAIN, KME_D_NPE_BUCKET); return false; }
        if (!crosses(is_buy, tsize, pb, P)) return tsize == 0;
        int li = os * LVP + pb;
        int32_t ms = U32(L.ht[li].x);
        int64_t lqty = U64(L.qty[li]);
        if (ms < 0) { die(KME_E_DOMAIN, KME_D_NPE_ORDER); return false; }
        KST(unsigned long long tw = stamp();)
        Maker m = ld_maker(ms);
        KST(acc[ST_MAKER_WAIT] += stamp() - tw; acc[ST_N_MAKER] += 1;)
        // (3) Sweep scan.  When the best level cannot absorb the taker, lane l takes the l-th level
        // after it in sweep order (ascending asks for a BUY, descending bids for a SELL) and a DPP
        // prefix scan over their resting quantity finds every level the sweep reaches (the
        // quantity before it is at most the taker's size).  Those levels' head makers are fetched
        // now, one lane each, so moving to the next level costs a readlane instead of a dependent
        // load.  Only levels the sweep itself has not touched are prefetched, and nothing writes
        // them before the sweep gets there, so the copies are exact; the loop below still applies
        // KP:237-253 maker by maker.
        const int32_t pb0 = pb;
        uint64_t pfmask = 0;
        int32_t pf_slot = -1, pf_oid0 = 0, pf_oid1 = 0, pf_aid0 = 0, pf_aid1 = 0, pf_sid1 = 0, pf_size = 0,
                pf_next = 0;
        if ((int64_t)tsize > lqty) {
            const int p = is_buy ? pb + 1 + lane : pb - 1 - lane;
            const bool occ = p >= 0 && p <= 100 && check_bit(lo, hi, p) && (is_buy ? p <= P : p >= P);
            const int lp = os * LVP + (occ ? p : 0);
            const int64_t q = occ ? L.qty[lp] : 0;
            const int64_t before = lqty + wave_incl_scan_i64(q) - q;
            const bool reach = occ && before <= (int64_t)tsize;
            pfmask = __ballot(reach);
            // (no branch around the loads: lanes that do not reach a level read the best level's
            // head, a valid node; a divergent branch here would demote the loop state to VGPRs)
            pf_slot = reach ? L.ht[lp].x : ms;
            const KG int4* nd = reinterpret_cast<const KG int4*>(&pool[pf_slot]);
            const int4 c0 = nd[0], c1 = nd[1];
            pf_oid0 = c0.x; pf_oid1 = c0.y; pf_aid0 = c0.z; pf_aid1 = c0.w;
            pf_sid1 = c1.y; pf_size = c1.z; pf_next = c1.w;
        }
        bool head_moved = false;                             // ms is a later maker of level li
        for (;;) {
            const int32_t ts = imin(tsize, m.size);
            const int32_t msize = jisub(m.size, ts);
            tsize = jisub(tsize, ts);
            lqty -= ts;
            if (msize != 0) {                                // maker stays, partially filled (KP:255-261)
                emit(ntr++, m, pb, ts);
                pool[ms].size = msize;
                if (head_moved) { L.ht[li].x = ms; pool[ms].prev = -1; }
                mark_dirty(ms);
                L.qty[li] = lqty;
                return tsize == 0;
            }
            int32_t nms, npb = pb;                           // maker consumed: orders.delete (KP:243)
            const bool same = m.next >= 0;
            if (same) {
                nms = m.next;
                if (!crosses(is_buy, tsize, pb, P)) {        // stops before the next maker of the level
                    emit(ntr++, m, pb, ts);
                    free_slot(ms);
                    L.ht[li].x = nms;
                    pool[nms].prev = -1;
                    mark_dirty(nms);
                    L.qty[li] = lqty;
                    return tsize == 0;
                }
            } else {                                         // level exhausted (KP:244-253)
                unset_bit(lo, hi, pb);
                set_bm(os, lo, hi);
                npb = is_buy ? min_price_ptr(lo, hi) : max_price_ptr(lo, hi);
                const bool go = npb != -1 && check_bit(lo, hi, npb) && crosses(is_buy, tsize, npb, P);
                if (!go) {
                    emit(ntr++, m, pb, ts);
                    free_slot(ms);
                    if (npb != -1 && !check_bit(lo, hi, npb)) die(KME_E_DOMAIN, KME_D_NPE_BUCKET);
                    return tsize == 0;
                }
                li = os * LVP + npb;
                nms = U32(L.ht[li].x);
                lqty = U64(L.qty[li]);
                if (nms < 0) { die(KME_E_DOMAIN, KME_D_NPE_ORDER); return false; }
            }
            KST(tw = stamp();)
            Maker nm;
            const int l = is_buy ? npb - pb0 - 1 : pb0 - 1 - npb;
            if (!same && l >= 0 && l < 64 && ((pfmask >> l) & 1) && rl32(pf_slot, l) == nms) {   // swept level
                nm.oid = mk64(rl32(pf_oid0, l), rl32(pf_oid1, l)); nm.aid = mk64(rl32(pf_aid0, l), rl32(pf_aid1, l));
                nm.sneg = rl32(pf_sid1, l) < 0;
                nm.size = rl32(pf_size, l); nm.next = rl32(pf_next, l);
            } else {
                nm = ld_maker(nms);                          // in flight during this trade's stores
            }
            emit(ntr++, m, pb, ts);
            free_slot(ms);
            KST(acc[ST_MAKER_WAIT] += stamp() - tw; acc[ST_N_MAKER] += 1;)
            head_moved = same;
            m = nm;
            ms = nms;
            pb = npb;
        }
    }

    // ---------------- addOrder, KP:200-223 (after the book-exists and balance checks)
    KDEV void rest(const Rec& r, int32_t tsize, Out& o) {
        KST(unsigned long long ts0 = stamp();)
        const int s = book_side(r.sid, r.action == BUY);
        uint64_t lo = bl(s), hi = bm(s);                     // books.get(sid) again (KP:205)
        const int32_t p = r.price;                           // 0..100 (k_emap)
        const int32_t slot = alloc_slot();
        KST(unsigned long long ts1 = stamp(); acc[ST_REST_ALLOC] += ts1 - ts0;)
        if (dead) return;
        const int li = s * LVP + p;
        int32_t nprev = -1;
        int64_t poid = 0;
        if (!check_bit(lo, hi, p)) {                        // new bucket (oid, oid), set bit (KP:209-211)
            L.ht[li] = make_int2(slot, slot);
            L.qty[li] = (int64_t)tsize;
            L.toid[li] = r.oid;
            set_bit(lo, hi, p);
            set_bm(s, lo, hi);
        } else {                                             // append at the tail (KP:213-219)
            nprev = U32(L.ht[li].y);
            poid = U64(L.toid[li]);
            pool[nprev].next = slot;
            mark_dirty(nprev);
            L.ht[li].y = slot;
            L.toid[li] = r.oid;
            L.qty[li] = U64(L.qty[li]) + tsize;
            o.has_prev = true;
            o.prev = poid;
        }
        KST(unsigned long long ts2 = stamp(); acc[ST_REST_LEVEL] += ts2 - ts1;)
        // the node: lane q < 4 stores 16-byte piece q (Node layout, kme_device.h).  Selected bit
        // by bit: a compare chain on q becomes a switch whose default the compiler marks
        // unreachable, a divergent loop exit that demotes the whole loop's state to VGPRs.
        const bool q0 = (q & 1) != 0, q1 = (q & 2) != 0;
        const int32_t x = q1 ? (q0 ? p : lo32(poid)) : (q0 ? lo32(r.sid) : lo32(r.oid));
        const int32_t y = q1 ? (q0 ? r.action : hi32(poid)) : (q0 ? hi32(r.sid) : hi32(r.oid));
        const int32_t z = q1 ? (q0 ? 1 : nprev) : (q0 ? tsize : lo32(r.aid));
        const int32_t w = q1 ? (q0 ? 0 : g) : (q0 ? -1 : hi32(r.aid));
        if (lane < 4) reinterpret_cast<KG int4*>(&pool[slot])[lane] = make_int4(x, y, z, w);
        mark_dirty(slot);
        rest_slot[r.i] = slot;
        o.rested = true;
        KST(acc[ST_REST_NODE] += stamp() - ts2;)
    }

    // ---------------- removeOrder, KP:289-323
    KDEV Victim ld_victim(int32_t s, int64_t oid, int64_t aid) const {
        Victim o;
        if (!is_dirty(s)) {
            const v16i v = sload_node(&pool[s]);
            const int32_t action = v[13];
            o.ok = v[14] != 0 && mk64(v[0], v[1]) == oid && mk64(v[2], v[3]) == aid;
            o.side = book_side(mk64(v[4], v[5]), action == BUY);
            o.sell = action == SELL; o.sid_neg = v[5] < 0;
            o.price = v[12];
            o.size = v[6]; o.next = v[7]; o.prev = v[10];
            o.prev_oid = mk64(v[8], v[9]);
            return o;
        }
        const int4 v = reinterpret_cast<const KG int4*>(&pool[s])[q];
        const int64_t noid = mk64(rl32(v.x, 0), rl32(v.y, 0)), naid = mk64(rl32(v.z, 0), rl32(v.w, 0));
        const int64_t nsid = mk64(rl32(v.x, 1), rl32(v.y, 1));
        const int32_t action = rl32(v.y, 3);
        o.ok = rl32(v.z, 3) != 0 && noid == oid && naid == aid;
        o.side = book_side(nsid, action == BUY);
        o.sell = action == SELL; o.sid_neg = hi32(nsid) < 0;
        o.price = rl32(v.x, 3);
        o.size = rl32(v.z, 1); o.next = rl32(v.w, 1); o.prev = rl32(v.z, 2);
        o.prev_oid = mk64(rl32(v.x, 2), rl32(v.y, 2));
        return o;
    }
    KDEV bool cancel(const Rec& r, const Lanes& B) {
        int32_t slot = -1;
        if (r.tgt >= 0) slot = (int32_t)r.tgt;
        else if (r.tgt <= -2) slot = U32(rest_slot[-(r.tgt + 2)]);   // (RS_PENDING cannot be: arrival order)
        if (slot < 0) return false;                          // orders.get(oid) == null
        Victim o;
        if (rl32(B.pf_slot, r.lane) == slot && !is_dirty(slot) && !bstale) {   // prefetched with the batch
            const int32_t meta = rl32(B.pf_meta, r.lane);
            o.ok = (meta >> 11) & 1;
            o.price = meta & 0xFF; o.side = (meta >> 8) & 1; o.sell = (meta >> 9) & 1; o.sid_neg = (meta >> 10) & 1;
            o.size = rl32(B.pf_size, r.lane); o.next = rl32(B.pf_next, r.lane); o.prev = rl32(B.pf_prev, r.lane);
            o.prev_oid = rl64(B.pf_poid, r.lane);
        } else {
            KST(const unsigned long long tw = stamp();)
            o = ld_victim(slot, r.oid, r.aid);
            KST(acc[ST_VICTIM_WAIT] += stamp() - tw; acc[ST_N_VICTIM] += 1;)
        }
        if (!o.ok) return false;                             // missing, or order.aid != aid (KP:291)
        if (!gsv(GS_EXISTS)) { die(KME_E_DOMAIN, KME_D_NPE_BOOK); return false; }
        const int li = o.side * LVP + o.price;
        if (o.prev < 0 && o.next < 0) {
            uint64_t lo = bl(o.side), hi = bm(o.side);
            unset_bit(lo, hi, o.price);
            set_bm(o.side, lo, hi);
            // (an empty level's head for the fast segments' level step: in the two-wavefront mode
            // this cancel may run beside wave 1, and no segment start resets the heads then)
            L.ht[li] = make_int2(-1, -1);
        } else if (o.prev < 0) {
            L.ht[li].x = o.next;
            pool[o.next].prev = -1;
            mark_dirty(o.next);
        } else if (o.next < 0) {
            L.ht[li].y = o.prev;
            L.toid[li] = o.prev_oid;
            pool[o.prev].next = -1;
            mark_dirty(o.prev);
        } else {
            pool[o.prev].next = o.next;
            pool[o.next].prev = o.prev;
            pool[o.next].prev_oid = o.prev_oid;
            mark_dirty(o.prev);
            mark_dirty(o.next);
        }
        L.qty[li] = U64(L.qty[li]) - o.size;
        free_slot(slot);
        if (cold().ledger_replay)   // the removed order, for postRemoveAdjustments in k_ledger_replay
            cold().vic[r.i] = make_int4(o.price | ((o.sell ? SELL : BUY) << 8), o.size, o.sid_neg ? -g : g, o.sid_neg ? -1 : 0);
        return !dead;
    }

    // ---------------- fast segments: parallelism inside one book
    // A hot book's records cost ~1.3 us each on the serial path above, mostly issue latency and the
    // dependent loads of one record's chain.  A fast segment takes a run of the batch's records in
    // two steps:
    //   1. the aggregate pass (scalar, one record at a time, no node access): what each record does
    //      to the book's LEVELS -- the level bitmaps (Books, KP:38-41) and each level's resting
    //      quantity -- decides its outcome.  A BUY/SELL sweeps the opposite levels best first
    //      (KP:225-263), taking min(remaining, level quantity) from each while the level crosses;
    //      a level taken whole is unset and the next best one is scanned exactly as KP:244-252 does
    //      (with its H5 bit check); a sweep that ends exactly on an emptied level decides the
    //      zero-size trade against the next level's head (KP:237's loop test with size 0, H3); the
    //      remainder rests at its price (KP:200-223).  A cancel removes its victim's quantity
    //      (KP:289-323): a victim prefetched with the batch, or an order that rested earlier in the
    //      segment.  Each effect on one level is an EVENT (take, zero trade, rest, unlink);
    //   2. the level step (vector): the segment's events grouped by level, one lane per level,
    //      replayed in arrival order -- appends at the tail, takes walking the FIFO from the head
    //      maker by maker as KP:237-261 does (H3 zero-size trades at a level's maker boundary
    //      included), unlinks -- so the touched levels' node work runs side by side.
    // Levels are independent once step 1 fixed every event's level and amount, so the result is the
    // reference's.  A record's trades keep their reference order: the trades of its k-th event
    // carry ordinal (index | k << 20) and the epilogue stores the record's per-event bases
    // (DevState::lvbase) for k_scatter.  The pass stops (the record goes to the serial path) where a
    // record's effect is not decided by levels alone: a sweep over more than FAST_RMAX levels, a
    // price scan that faults (H5), a cancel whose level was already taken from in the segment or
    // whose victim was written since the batch prefetch or decided before the segment, admin
    // actions, a full event buffer; and the fast path is off for group 0 (H4: one shared book) and
    // once a size-0 order was ever submitted (C_SIZE0: a level's emptiness is then not its quantity
    // being 0).
    enum { EK_TAKE = 0, EK_REST = 1, EK_CANCEL = 2, EK_ZERO = 3 };
    static constexpr int FAST_RMAX = FAST_LVB;       // levels one sweep may take from in a segment (its
                                                     // zero trade is event rank FAST_RMAX at most)
    static constexpr int32_t RR_REMOVED = 1 << 24;   // rr flag: rested in the segment, then cancelled in it
    // lane l of the result is v, the others old's (v_cmp + v_cndmask; v scalar)
    // single-lane register writes (v_writelane: one VALU op; l uniform)
    KDEV static int32_t wl(int32_t v, int l, int32_t old) { return kme_writelane_i32(v, l, old); }
    // The pass's level quantities, 32 bits (fast_segment checks the bound at its start): lane p of QA
    // / QC holds level (side 0 / 1, price p) for p < 63 and lane p - 63 of QB / QD the prices above,
    // the bitmap words' split -- read with one readlane, written with two writelanes (side and price
    // uniform; the register the level is not in takes the write in its lane 63, which holds no level:
    // prices 63 and 126+ are QB's / no FUNDED price).  They are locals of fast_segment: a struct behind a reference
    // becomes a dynamically indexed stack array (scratch memory).
#define KME_QGET(s, p) ((s) ? ((p) < 63 ? rl32(QC, (p)) : rl32(QD, (p) - 63)) : ((p) < 63 ? rl32(QA, (p)) : rl32(QB, (p) - 63)))
#define KME_QSET(s, p, v)                                                                              \
    do {                                                                                               \
        const int _p = (p);                                                                            \
        const int32_t _v = (v);                                                                        \
        const int _lo = _p < 63 ? _p : 63, _hi = _p < 63 ? 63 : _p - 63;   /* lane 63: a dummy */     \
        if (s) { QC = wl(_v, _lo, QC); QD = wl(_v, _hi, QD); }                                         \
        else   { QA = wl(_v, _lo, QA); QB = wl(_v, _hi, QB); }                                         \
    } while (0)
    // events of the pass: event e in lane e of Ex, Ev: x = record lane | kind << 6 | rank << 8 | level
    // (side * 128 + price) << 16 | P << 24, v = the amount taken (a take) or the node slot (a rest, an
    // unlink)
#define KME_PUT_EV(e, k, kind, rank, lev, P, v)                                                        \
    do {                                                                                               \
        const int _e = (e);                                                                            \
        Ex = wl((k) | ((kind) << 6) | ((rank) << 8) | ((lev) << 16) | ((P) << 24), _e, Ex);            \
        Ev = wl((v), _e, Ev);                                                                          \
    } while (0)
    enum { PC_TAKE_REST = 0, PC_REJECT = 1, PC_CANCEL_PF = 2, PC_CANCEL_BATCH = 3, PC_SERIAL = 4 };

    // fstack holds at least n slots (n <= 64): free-list blocks, then the bump chunk
    KDEV void fast_refill(int n) {
        int fsp = gsv(GS_FSP);
        while (fsp < n) {
            const int32_t blk = gsv(GS_FREE_HEAD);
            if (blk >= 0) {
                const int32_t w = lane < 2 + FBLK - 1 ? reinterpret_cast<const KG int32_t*>(&pool[blk])[lane] : 0;
                const int32_t nxt = rl32(w, 0), cnt = rl32(w, 1);
                if (lane >= 2 && lane < 2 + cnt) L.fstack[fsp + lane - 2] = w;
                L.fstack[fsp + cnt] = blk;                   // the block's own slot
                fsp += cnt + 1;
                set_gs(GS_FREE_HEAD, nxt);
            } else {
                int32_t cn = gsv(GS_CHUNK_NEXT);
                int32_t ce = gsv(GS_CHUNK_END);
                if (cn >= ce) {
                    unsigned long long c = 0;
                    KG unsigned long long* bump = &ctr()[ci(C_POOL_BUMP)];
                    if (lane == 0) c = atomicAdd(bump, (unsigned long long)POOL_CHUNK);
                    c = bcast64(c);
                    if (c + POOL_CHUNK > cold().pool_cap) { die(KME_E_CAPACITY, KME_D_CAP_POOL); return; }
                    cn = (int32_t)c;
                    ce = (int32_t)(c + POOL_CHUNK);
                    set_gs(GS_CHUNK_END, ce);
                }
                const int k = imin(n - fsp, ce - cn);
                if (lane < k) L.fstack[fsp + lane] = cn + lane;
                fsp += k;
                set_gs(GS_CHUNK_NEXT, cn + k);
            }
            sync_lds();
        }
        set_gs(GS_FSP, fsp);
        sync_lds();
    }

    // per-lane trade scratch (the level step's takes): LANE_TCH slots reserved at a time on the
    // group's shard line, unused ones left as holes (seq = -1) that k_scatter skips
    KDEV void lane_emit(uint32_t& tpos, uint32_t& tlim, uint32_t seq, uint32_t ord, int4 maker, int32_t msneg,
                        int32_t mprice, int32_t ts, int& err) {
        if (err) return;
        if (tpos == tlim) {
            const DevState& S = *Sp;
            const uint32_t tcap = S.tshard_cap, tb = (uint32_t)(g & (TSHARDS - 1)) * tcap;
            KG unsigned long long* used = &S.tsh[(size_t)(g & (TSHARDS - 1)) * CTR_STRIDE + TS_USED];
            const unsigned long long need = __ballot(1);
            const int leader = __ffsll((long long)need) - 1;
            const uint32_t rank = (uint32_t)__popcll(need & ((1ull << lane) - 1));
            unsigned long long base = 0;
            if (lane == leader) base = atomicAdd(used, (unsigned long long)kLaneTradeChunk * __popcll(need));
            base = (unsigned long long)__shfl((long long)base, leader) + (unsigned long long)rank * kLaneTradeChunk;
            if (base + kLaneTradeChunk <= tcap) {
                tpos = tb + (uint32_t)base;
            } else {
                for (unsigned long long q = base; q < tcap; ++q) S.ttmp[tb + q].seq = -1;   // straddles the end
                const unsigned long long ob = atomicAdd(&S.ctr[ci(C_TTMP)], (unsigned long long)kLaneTradeChunk);
                if (ob + kLaneTradeChunk > S.ttmp_cap) {
                    for (unsigned long long q = ob; q < S.ttmp_cap; ++q) S.ttmp[(size_t)TSHARDS * tcap + q].seq = -1;
                    raise_thread(S.ctr, KME_E_CAPACITY, KME_D_CAP_TRADES, (int64_t)seq);
                    err = 1;
                    return;
                }
                tpos = TSHARDS * tcap + (uint32_t)ob;
            }
            tlim = tpos + kLaneTradeChunk;
        }
        KG int4* r = reinterpret_cast<KG int4*>(&Sp->ttmp[tpos++]);
        r[0] = maker;
        r[1] = make_int4((int32_t)seq, (int32_t)tt_ordp(ord, mprice, msneg != 0), ts, g);
    }
    KDEV void lane_dirty(int32_t s) { atomicOr(&L.dirty[(s >> 5) & (DIRTY_WORDS - 1)], 1u << (s & 31)); }
    // a freed node onto the group's free stack (LDS), or, with the stack full, as a one-slot block
    // pushed on the group's free list.  TWO (wave 1): into buffer lb's list for wave 0 to take at the
    // phase's end (wave 0 owns the stack), past LFREE as one-slot blocks on a chain of its own
    template <bool TWO>
    KDEV void lane_free(int32_t s, int lb) {
        pool[s].live = 0;
        lane_dirty(s);
        if constexpr (TWO) {
            const int pos = atomicAdd(&tl->lfcnt[lb], 1);
            if (pos < LFREE) {
                tl->lfree[lb][pos] = s;
            } else {
                const int32_t old = atomicExch(&tl->lch_head[lb], s);
                KG int32_t* w = reinterpret_cast<KG int32_t*>(&pool[s]);
                w[0] = old;
                w[1] = 0;
                if (old < 0) tl->lch_tail[lb] = s;
            }
            return;
        }
        const int pos = atomicAdd(&L.gs[GS_FSP], 1);
        if (pos < FSTK) {
            L.fstack[pos] = s;
        } else {
            const int32_t old = atomicExch(&L.gs[GS_FREE_HEAD], s);
            KG int32_t* w = reinterpret_cast<KG int32_t*>(&pool[s]);
            w[0] = old;
            w[1] = 0;
        }
    }

    // Records [j0, nb) of the batch: returns the first record the segment did not take (== j0: none).
    // Per lane (= record) results go to the batch's OUT registers.
    template <bool TWO>
    KDEV int fast_segment(const Lanes& B, int j0, int nb, int32_t& o_act, int32_t& o_size, int32_t& o_plo,
                          int32_t& o_phi, int32_t& o_ntr, uint32_t& tpos, uint32_t& tlim) {
        const bool inrange = lane >= j0 && lane < nb;
        const int32_t b_act = B.w0 & 0xFF;
        const bool b_bs = b_act == BUY || b_act == SELL;
        const int n_bs = (int)__popcll(__ballot(inrange && b_bs));
        if (gsv(GS_TCNT)) flush_trades();                     // trd is the segment's staging
        fast_refill(n_bs);
        if (dead) return j0;
        const int fsp0 = gsv(GS_FSP);
        const int32_t fslot = lane < n_bs ? L.fstack[fsp0 - 1 - lane] : -1;   // the k-th rest takes lane k's
        uint64_t b0l = bl(0), b0m = bm(0), b1l = bl(1), b1m = bm(1);
        // the level quantities into lanes; levels unoccupied as the segment starts read as empty in
        // the level step
        int64_t qv[4];                                        // QA, QB, QC, QD (see KME_QGET)
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            const int sd = h >> 1, p = (h & 1) ? lane + 63 : lane;
            const bool lv = (h & 1) ? p <= 100 : lane < 63;
            const bool occ = lv && check_bit(sd ? b1l : b0l, sd ? b1m : b0m, p);
            qv[h] = occ ? L.qty[sd * LVP + p] : 0;
            // (two waves: only while wave 1 is idle -- its level step keeps the levels it empties
            // at -1 itself, and only the serial path leaves stale heads behind)
            if (lv && !occ && (!TWO || !lbusy)) L.ht[sd * LVP + p] = make_int2(-1, -1);
        }
        // 32-bit quantities: every level below 2^30 and every order of the segment below 2^23, so 64
        // rests on one level stay below 2^31; otherwise the records take the serial path
        if (__ballot(qv[0] >= (1 << 30) || qv[1] >= (1 << 30) || qv[2] >= (1 << 30) || qv[3] >= (1 << 30) ||
                     (inrange && b_bs && B.size >= (1 << 23))))
            return j0;
        int32_t QA = lo32(qv[0]), QB = lo32(qv[1]), QC = lo32(qv[2]), QD = lo32(qv[3]);
        // each record's class, decided per lane before the serial pass: pk = class | BUY << 4 | P << 8 |
        // action << 16 | victim level << 24 (a prefetched cancel's).  A BUY/SELL with a negative sid
        // (its side is the other book, KP:201) takes the serial path.
        const int exists = gsv(GS_EXISTS);
        const uint32_t bi0 = (uint32_t)rl32((int32_t)B.i, 0);   // the batch's first record
        int32_t pk;
        {
            const int32_t P = (B.w0 >> 8) & 0xFF;
            int cls = PC_SERIAL, vlev = 0;
            if (b_bs) {
                cls = !(exists && ((B.w0 >> 16) & 1)) ? PC_REJECT
                      : (B.size <= 0 || ((B.w0 >> 17) & 1) ? PC_SERIAL : PC_TAKE_REST);
            } else if (b_act == CANCEL) {
                if (B.tgt == -1) {
                    cls = PC_REJECT;                          // orders.get(oid) == null (KP:290)
                } else if (B.pf_slot >= 0) {                  // a victim resting before the batch
                    const bool dirty = (L.dirty[(B.pf_slot >> 5) & (DIRTY_WORDS - 1)] >> (B.pf_slot & 31)) & 1;
                    if (!((B.pf_meta >> 11) & 1)) cls = PC_REJECT;   // gone / another account's (KP:290-291)
                    else cls = dirty || !exists ? PC_SERIAL : PC_CANCEL_PF;   // written since the prefetch /
                    vlev = ((B.pf_meta >> 8) & 1) * 128 + (B.pf_meta & 0xFF);  // KP:294's NPE: serial
                } else {                                      // an order of this epoch not final at the prefetch
                    // (a target before the batch was decided by an earlier batch, and its slot is
                    // still pending: it did not rest, orders.get(oid) == null)
                    const uint32_t ti = (uint32_t)(-(B.tgt + 2));
                    cls = B.pf_meta != RS_PENDING || ti < bi0 ? PC_REJECT : (exists ? PC_CANCEL_BATCH : PC_SERIAL);
                }
            }
            // Two waves: a same-epoch target in the segment wave 1 had in hand when the batch's
            // prefetch ran may have rested with its node and slot half written -- the serial path
            // (after wave 1 is done) reads them again
            if (TWO && b_act == CANCEL && B.tgt <= -2) {
                const uint32_t ti = (uint32_t)(-(B.tgt + 2));
                if (ti >= bpend_lo && ti <= bpend_hi) cls = PC_SERIAL;
            }
            pk = cls | (b_act == BUY ? 16 : 0) | (P << 8) | (b_act << 16) | (vlev << 24);
        }
        // levels taken from in the segment, and lane j: the prefetched victim record j removes (two
        // waves: the pass also checks those of the segment wave 1 has not finished, tl->cb / tl->fv:
        // it may not have written their nodes yet)
        uint64_t c0l = 0, c0m = 0, c1l = 0, c1m = 0;
        int32_t f_vslot = -1;
        int32_t Ex = 0, Ev = 0;
        int nrest = 0, nev = 0;
        int j = j0;
        int32_t oact = 0, osize = 0, flags = 0, rslot = -1, rlev = 0;
        // A BUY (IB) or SELL of sid +g: takes from book side 1 - SIDE, rests on SIDE (KP:201, 292).
        // Returns false where the record goes to the serial path.
        KST(int ksw = 0;)                                    // (stamps: the record swept / took from one level)
        auto take_rest = [&](auto ib_tag) -> bool {
            constexpr bool IB = decltype(ib_tag)::value;
            constexpr int SIDE = IB ? 0 : 1, OS = 1 - SIDE;
            uint64_t& olo = OS ? b1l : b0l;
            uint64_t& ohi = OS ? b1m : b0m;
            uint64_t& slo = SIDE ? b1l : b0l;
            uint64_t& shi = SIDE ? b1m : b0m;
            uint64_t& col = OS ? c1l : c0l;
            uint64_t& coh = OS ? c1m : c0m;
            const int32_t P = (rl32(pk, j) >> 8) & 0xFF;
            int32_t rem = rl32(B.size, j);
            int32_t pb = IB ? min_price_ptr(olo, ohi) : max_price_ptr(olo, ohi);
            if (pb != -1 && !check_bit(olo, ohi, pb)) return false;   // the H5 NPE: the serial path raises it
            if (pb != -1 && crosses(IB, rem, pb, P)) {
                const int32_t q = KME_QGET(OS, pb);
                if (rem < q) {                        // the best level absorbs it (KP:237-261)
                    KST(ksw = 2;)
                    if (nev + 1 > FAST_EVCAP) return false;
                    KME_QSET(OS, pb, q - rem);
                    if (pb < 64) col |= 1ull << pb; else coh |= 1ull << (pb - 64);
                    KME_PUT_EV(nev++, j, EK_TAKE, 0, OS * 128 + pb, P, rem);
                    rem = 0;
                } else {                                       // a sweep, undone if it cannot be taken
                    KST(ksw = 1;)
                    int32_t& ql = OS ? QC : QA;
                    int32_t& qh = OS ? QD : QB;
                    const int32_t sql = ql, sqh = qh, snev = nev;
                    const uint64_t s_lo = olo, s_hi = ohi, s_cl = col, s_ch = coh;
                    int32_t p = pb, nt = 0, zl = -1;
                    bool bad = false;
#pragma nounroll
                    for (;;) {                                 // KP:237-253
                        if (nt == FAST_RMAX || nev + 1 > FAST_EVCAP) { bad = true; break; }
                        const int32_t qq = KME_QGET(OS, p);
                        const int32_t x = qq < rem ? qq : rem;
                        rem -= x;
                        KME_QSET(OS, p, qq - x);
                        if (p < 64) col |= 1ull << p; else coh |= 1ull << (p - 64);
                        KME_PUT_EV(nev++, j, EK_TAKE, nt, OS * 128 + p, P, x);
                        ++nt;
                        if (x < qq) break;                     // stops inside the level
                        unset_bit(olo, ohi, p);                // taken whole (KP:244-252)
                        const int32_t np = IB ? min_price_ptr(olo, ohi) : max_price_ptr(olo, ohi);
                        if (np != -1 && !check_bit(olo, ohi, np)) { bad = true; break; }   // H5
                        if (rem == 0) { if (np != -1 && np >= P) zl = np; break; }        // H3 zero trade
                        if (np == -1 || !crosses(IB, rem, np, P)) break;
                        p = np;
                    }
                    if (bad || nev + (zl >= 0) + (rem > 0) > FAST_EVCAP) {
                        ql = sql; qh = sqh; nev = snev;
                        olo = s_lo; ohi = s_hi; col = s_cl; coh = s_ch;
                        return false;
                    }
                    if (zl >= 0) KME_PUT_EV(nev++, j, EK_ZERO, nt, OS * 128 + zl, P, 0);
                }
            }
            if (rem > 0) {                                     // addOrder (KP:200-223)
                if (nev + 1 > FAST_EVCAP) return false;       // (only when nothing was taken: rem == size)
                const int32_t q = check_bit(slo, shi, P) ? KME_QGET(SIDE, P) : 0;
                KME_QSET(SIDE, P, q + rem);
                set_bit(slo, shi, P);
                rslot = rl32(fslot, nrest);
                ++nrest;
                rlev = SIDE * 128 + P;
                KME_PUT_EV(nev++, j, EK_REST, 0, rlev, P, rslot);
                flags = 2;
            }
            osize = rem;
            return true;
        };
        // (stamps builds: the wait for this wavefront's outstanding vector memory operations, timed
        // apart from the pass)
        KST(const unsigned long long td0 = stamp(); __builtin_amdgcn_s_waitcnt(VMCNT0); acc[ST_FAST_DRAIN] += stamp() - td0;)
        KST(const unsigned long long tp0 = stamp();)
        // ---- 1. the aggregate pass.  Per record: its class and fields by readlane, its events and
        // results by lane selects (results: o_act = action | flags << 16, o_size, o_plo = first event |
        // events << 8 | rest level << 16, o_phi = rest slot; the epilogue replaces the last two).
#pragma nounroll
        for (; j < nb; ++j) {
            KST(const unsigned long long tr0 = stamp(); ksw = 0;)
            const int32_t pj = rl32(pk, j);
            const int cls = pj & 7;
            if (cls == PC_SERIAL) break;
            oact = (pj >> 16) & 0xFF; osize = 0; flags = 0; rslot = -1; rlev = 0;
            const int evb = nev;
            if (cls == PC_TAKE_REST) {
                const bool ok = (pj >> 4) & 1 ? take_rest(std::true_type()) : take_rest(std::false_type());
                if (!ok) break;
            } else if (cls == PC_REJECT) {
                oact = REJECT;                                // (KP:100-104, 290-291)
                osize = rl32(B.size, j);
            } else {                                          // removeOrder (KP:289-323)
                int32_t vlev = -1, vsl = -1, vsz = 0, vrec = -1;
                if (cls == PC_CANCEL_PF) {
                    const int32_t pfs = rl32(B.pf_slot, j);
                    if (__ballot(f_vslot == pfs || (TWO && lbusy && tl->fv[lane] == pfs) || (TWO && bstale && tl->bfv[lane] == pfs))) {
                        oact = REJECT;                        // removed by an earlier cancel of the segment
                    } else {
                        vlev = (pj >> 24) & 0xFF;
                        vsl = pfs;
                        vsz = rl32(B.pf_size, j);
                    }
                } else {                                      // pending: a BUY/SELL of this batch
                    const uint32_t ti = (uint32_t)(-(rl32(B.tgt, j) + 2));
                    const uint64_t hit = __ballot(lane < nb && B.i == ti);
                    if (!hit) break;
                    const int jt = __builtin_ctzll(hit);
                    if (jt < j0 || jt >= j) break;            // decided before the segment: serial
                    const int32_t rx = rl32(o_act, jt);
                    if (!((rx >> 16) & 2) || (rx & RR_REMOVED) || rl64(B.aid, jt) != rl64(B.aid, j)) {
                        oact = REJECT;                        // traded away, removed, another account's
                    } else {
                        vlev = (rl32(o_plo, jt) >> 16) & 0xFF;
                        vsl = rl32(o_phi, jt);
                        vsz = rl32(o_size, jt);
                        vrec = jt;
                    }
                }
                if (vlev >= 0) {
                    if (nev + 1 > FAST_EVCAP) break;
                    const int vs = vlev >> 7, vp = vlev & 127;
                    uint64_t cw = vs ? (vp < 64 ? c1l : c1m) : (vp < 64 ? c0l : c0m);
                    if (TWO && lbusy) cw |= U64((int64_t)tl->cb[vs * 2 + (vp < 64 ? 0 : 1)]);
                    if (TWO && bstale) cw |= U64((int64_t)tl->bcb[vs * 2 + (vp < 64 ? 0 : 1)]);
                    if ((cw >> (vp & 63)) & 1) break;         // its level was taken from: serial
                    const int32_t q = KME_QGET(vs, vp) - vsz;
                    KME_QSET(vs, vp, q);
                    if (q == 0) {
                        if (vs) unset_bit(b1l, b1m, vp); else unset_bit(b0l, b0m, vp);
                    }
                    if (vrec >= 0) o_act = wl(rl32(o_act, vrec) | RR_REMOVED, vrec, o_act);
                    else f_vslot = wl(vsl, j, f_vslot);
                    KME_PUT_EV(nev++, j, EK_CANCEL, 0, vlev, 0, vsl);
                }
            }
            o_act = wl((oact & 0xFFFF) | (flags << 16), j, o_act);
            o_size = wl(osize, j, o_size);
            o_plo = wl(evb | ((nev - evb) << 8) | (rlev << 16), j, o_plo);
            o_phi = wl(rslot, j, o_phi);
            KST(const unsigned long long trd = stamp() - tr0;)
            KST(const bool k_t = cls == PC_TAKE_REST && !ksw; const bool k_s = cls == PC_TAKE_REST && ksw == 1;)
            KST(const bool k_a = cls == PC_TAKE_REST && ksw == 2;)
            KST(acc[ST_PASS_ABSORB] += k_a ? trd : 0; acc[ST_N_PASS_ABSORB] += k_a;)
            KST(const bool k_r = cls == PC_REJECT; const bool k_c = cls != PC_TAKE_REST && !k_r;)
            KST(acc[ST_PASS_REST] += k_t ? trd : 0; acc[ST_N_PASS_REST] += k_t;)
            KST(acc[ST_PASS_SWEEP] += k_s ? trd : 0; acc[ST_N_PASS_SWEEP] += k_s;)
            KST(acc[ST_PASS_CANCEL] += k_c ? trd : 0; acc[ST_N_PASS_CANCEL] += k_c;)
            KST(acc[ST_PASS_REJECT] += k_r ? trd : 0; acc[ST_N_PASS_REJECT] += k_r;)
        }
        const int je = j;
        // where a new segment can go on: a stop at a (nearly) full event buffer, or at a prefetched
        // cancel whose level this segment took from (two waves: only the segment wave 1 has in hand);
        // at any other stop the record is the serial path's and a new segment's set-up would be lost
        seg_retry = false;
        if (je < nb) {
            const int32_t pj = rl32(pk, je);
            if (nev >= FAST_EVCAP - FAST_RMAX - 2) {
                seg_retry = true;
            } else if ((pj & 7) == PC_CANCEL_PF) {
                const int vlev = (pj >> 24) & 0xFF, vs = vlev >> 7, vp = vlev & 127, w = vp < 64 ? 0 : 1;
                const uint64_t own = vs ? (w ? c1m : c1l) : (w ? c0m : c0l);
                if (!TWO) {
                    seg_retry = (own >> (vp & 63)) & 1;
                } else {
                    const uint64_t bw = bstale ? U64((int64_t)tl->bcb[vs * 2 + w]) : 0;
                    const uint64_t tw = lbusy ? U64((int64_t)tl->cb[vs * 2 + w]) : 0;
                    seg_retry = !(((own | bw) >> (vp & 63)) & 1) && ((tw >> (vp & 63)) & 1);
                }
            }
        }
        KST(acc[ST_FAST_PASS] += stamp() - tp0;)
        if (je == j0) return j0;
        set_bm(0, b0l, b0m);
        set_bm(1, b1l, b1m);
        set_gs(GS_FSP, fsp0 - nrest);
        {                                                     // quantities back (occupied levels)
            const int32_t qs[4] = {QA, QB, QC, QD};
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                const int sd = h >> 1, p = (h & 1) ? lane + 63 : lane;
                const bool lv = (h & 1) ? p <= 100 : lane < 63;
                if (lv && check_bit(sd ? b1l : b0l, sd ? b1m : b0m, p)) L.qty[sd * LVP + p] = (int64_t)qs[h];
            }
        }
        if constexpr (TWO) {
            // ---- hand the segment to wave 1 (its level step and epilogue run during the next
            // segment's pass) and end the phase
            if (lane == 0) { tl->cb[0] = c0l; tl->cb[1] = c0m; tl->cb[2] = c1l; tl->cb[3] = c1m; }
            tl->fv[lane] = f_vslot;
            pend_lo = (uint32_t)rl32((int32_t)B.i, j0);
            pend_hi = (uint32_t)rl32((int32_t)B.i, je - 1);
            if (lane < 8) tl->tb[lane] = 0;
            sync_lds();
            if (lane < nev) atomicOr(&tl->tb[(Ex >> 21) & 7], 1u << ((Ex >> 16) & 31));
            const int buf = kp & 1;
            if (lane < nev) tl->ev[buf][lane] = make_int4(Ex, Ev, Ev, 0);
            if (lane >= j0 && lane < je) {
                tl->rin[buf][lane] = make_int4((int32_t)B.i, B.w0, o_size, 0);
                tl->rid[buf][lane] = make_int4(lo32(B.oid), hi32(B.oid), lo32(B.aid), hi32(B.aid));
                tl->rec[buf][lane] = make_int4(o_act, o_plo, o_phi, b_bs ? 1 : 0);
            }
            if (lane == 0) {
                tl->seg[buf][0] = j0; tl->seg[buf][1] = je; tl->seg[buf][2] = nev; tl->seg[buf][3] = TW_SEG;
            }
            fastmask |= (je >= 64 ? ~0ull : (1ull << je) - 1) & ~((1ull << j0) - 1);
            phase_end();
            lbusy = true;
            return je;
        }
        // ---- 2. the level step
        KST(const unsigned long long tl0 = stamp();)
        L.trd[lane] = make_int4(lo32(B.oid), hi32(B.oid), lo32(B.aid), hi32(B.aid));
        L.rin[lane] = make_int4((int32_t)B.i, B.w0, o_size, 0);
        L.ev[lane] = make_int4(Ex, Ev, Ev, 0);
        sync_lds();
        const int err = level_step<false>(L.ev, L.rin, L.trd, nev, tpos, tlim, 0);
        KST(const unsigned long long te0 = stamp(); acc[ST_FAST_LEVEL] += te0 - tl0;)
        {
            const int fsp = U32(L.gs[GS_FSP]);
            if (fsp > FSTK) set_gs(GS_FSP, FSTK);
        }
        // per record: its results, its events' trade bases, its oid-table entry (the rest slot, or
        // dead: KP:221)
        if (lane >= j0 && lane < je) epilogue(L.ev, B.i, b_bs, o_act, o_plo, o_phi, o_ntr);
        sync_lds();
        KST(acc[ST_FAST_EPI] += stamp() - te0;)
        if (__ballot(err != 0)) {
            if (__ballot(err == 2)) { cur = (uint32_t)rl32((int32_t)B.i, j0); die(KME_E_DOMAIN, KME_D_NPE_ORDER); }
            else dead = true;                                 // CAP_TRADES, raised at its record by lane_emit
        }
        return je;
    }

    // A segment's events replayed level by level (one lane per touched level): appends at the tail,
    // takes walking the FIFO from the head maker by maker as KP:237-261 does, unlinks (KP:297-320).
    // ev / rin / rid: the segment's events and its records' (input index, w0, rest size) / (oid, aid)
    // by record lane.  Returns 2 for the reference's NPE (a take finding no maker), 1 when a trade
    // reservation failed (raised at its record), else 0.  TWO: wave 1's call, freed slots to buffer lb.
    template <bool TWO>
    KDEV int level_step(int4* ev, const int4* rin, const int4* rid, int nev, uint32_t& tpos, uint32_t& tlim, int lb) {
        int err = 0;
        const int e = lane;
        const bool ve = e < nev;
        const int lev = ve ? (ev[e].x >> 16) & 0xFF : 0;
        unsigned long long peers = __ballot(ve);              // the segment's events at lane's level
#pragma unroll
        for (int bb = 0; bb < 8; ++bb) {
            const unsigned long long m = __ballot(ve && ((lev >> bb) & 1));
            peers &= ((lev >> bb) & 1) ? m : ~m;
        }
        if (ve && __builtin_ctzll(peers) == lane) {
            const int side = lev >> 7, price = lev & 127, li = side * LVP + price;
            const int2 ht = L.ht[li];
            int32_t head = ht.x, tail = ht.y;
            int64_t toid = L.toid[li];
            unsigned long long m = peers;
            while (m) {
                const int k = __builtin_ctzll(m);
                m &= m - 1;
                const int4 f = ev[k];
                const int kind = (f.x >> 6) & 3, rk = f.x & 63;
                const uint32_t rank = (uint32_t)(f.x >> 8) & 7;
                const int4 ri = rin[rk];                      // the record's (input index, PRec w0, rest size)
                if (kind == EK_TAKE) {                        // tryMatch at one level (KP:237-261)
                    const int32_t P = (f.x >> 24) & 0x7F;
                    int32_t x = f.y, ms = head;
                    uint32_t ntr = 0;
                    bool moved = false;
                    if (ms < 0) err = 2;
                    while (ms >= 0) {
                        const KG int4* nd = reinterpret_cast<const KG int4*>(&pool[ms]);
                        const int4 n0 = nd[0], n1 = nd[1];
                        if (!(x > 0 || price >= P)) break;    // KP:237 with size 0 (H3); x > 0: crosses
                        const int32_t ts = imin(x, n1.z);
                        x -= ts;
                        lane_emit(tpos, tlim, (uint32_t)ri.x, ntr++ | (rank << FAST_RANK_SHIFT), n0, n1.y < 0, price, ts, err);
                        if (n1.z - ts != 0) { pool[ms].size = n1.z - ts; lane_dirty(ms); break; }
                        lane_free<TWO>(ms, lb);               // orders.delete (KP:243)
                        if (n1.w < 0) { if (x != 0) err = 2; ms = -1; break; }   // the level taken whole
                        ms = n1.w;
                        moved = true;
                    }
                    if (ms < 0) { head = -1; tail = -1; }
                    else { if (moved) { pool[ms].prev = -1; lane_dirty(ms); } head = ms; }
                    ev[k].w = (int32_t)ntr;
                } else if (kind == EK_ZERO) {                 // the next level's head, size 0 (KP:237, H3)
                    int32_t n = 0;
                    if (head < 0) {
                        err = 2;
                    } else {
                        const KG int4* nd = reinterpret_cast<const KG int4*>(&pool[head]);
                        const int4 n0 = nd[0], n1 = nd[1];
                        lane_emit(tpos, tlim, (uint32_t)ri.x, rank << FAST_RANK_SHIFT, n0, n1.y < 0, price, 0, err);
                        n = 1;
                    }
                    ev[k].w = n;
                } else if (kind == EK_REST) {                 // addOrder's rest (KP:205-221)
                    const int4 id = rid[rk];
                    const int32_t slot = f.z;
                    int32_t nprev = -1, hp = 0;
                    int64_t poid = 0;
                    if (head < 0) {
                        head = slot;
                    } else {
                        pool[tail].next = slot;
                        lane_dirty(tail);
                        nprev = tail; poid = toid; hp = 1;
                    }
                    tail = slot;
                    toid = mk64(id.x, id.y);
                    const int32_t sidl = ((ri.y >> 17) & 1) ? -g : g;
                    KG int4* nd = reinterpret_cast<KG int4*>(&pool[slot]);
                    nd[0] = id;
                    nd[1] = make_int4(sidl, sidl < 0 ? -1 : 0, ri.z, -1);
                    nd[2] = make_int4(lo32(poid), hi32(poid), nprev, g);
                    nd[3] = make_int4(price, ri.y & 0xFF, 1, 0);
                    lane_dirty(slot);
                    ev[k] = make_int4(f.x, hp, lo32(poid), hi32(poid));
                } else {                                      // removeOrder's unlink (KP:297-320)
                    const int32_t vs = f.z;
                    const KG int4* nd = reinterpret_cast<const KG int4*>(&pool[vs]);
                    const int4 n1 = nd[1], n2 = nd[2], n3 = nd[3];
                    const int32_t next = n1.w, prev = n2.z;
                    const int64_t prev_oid = mk64(n2.x, n2.y);
                    if (prev < 0 && next < 0) {
                        head = -1; tail = -1;
                    } else if (prev < 0) {
                        head = next;
                        pool[next].prev = -1;
                        lane_dirty(next);
                    } else if (next < 0) {
                        tail = prev; toid = prev_oid;
                        pool[prev].next = -1;
                        lane_dirty(prev);
                    } else {
                        pool[prev].next = next;
                        pool[next].prev = prev;
                        pool[next].prev_oid = prev_oid;
                        lane_dirty(prev);
                        lane_dirty(next);
                    }
                    lane_free<TWO>(vs, lb);
                    if (Sp->ledger_replay)                    // the removed order, for postRemoveAdjustments
                        Sp->vic[ri.x] = make_int4(price | ((n3.y == SELL ? SELL : BUY) << 8), n1.z, n1.y < 0 ? -g : g,
                                                  n1.y < 0 ? -1 : 0);
                }
            }
            L.ht[li] = make_int2(head, tail);
            L.toid[li] = toid;
        }
        sync_lds();
        return err;
    }

    // One record's results after the level step (the lane of a record of the segment): trade count,
    // per-event trade bases (lvbase, k_scatter), OUT.prev of an append, its oid-table entry's rest slot.
    KDEV void epilogue(const int4* ev, uint32_t bi, bool bs, int32_t& o_act, int32_t& o_plo, int32_t& o_phi,
                       int32_t& o_ntr) {
        const int eb = o_plo & 0xFF, en = (o_plo >> 8) & 0xFF;
        const int32_t rs = o_phi;
        o_act &= ~RR_REMOVED;
        o_plo = 0; o_phi = 0;
        uint32_t ntr = 0;
        for (int e = eb; e < eb + en; ++e) {
            const int4 f = ev[e];
            const int kind = (f.x >> 6) & 3, rank = (f.x >> 8) & 7;
            if (kind == EK_TAKE || kind == EK_ZERO) {
                if (rank) Sp->lvbase[(size_t)bi * FAST_LVB + rank - 1] = ntr;
                ntr += (uint32_t)f.w;
            } else if (kind == EK_REST && f.y) {
                o_act |= KME_OUT_HAS_PREV << 16;
                o_plo = f.z; o_phi = f.w;
            }
        }
        o_ntr = (int32_t)ntr;
        if (bs && ((o_act >> 16) & 2)) rest_slot[bi] = rs;
    }

    // ---------------- two-wavefront mode (k_match<true>)
    // wave 0: the end of a phase -- the workgroup barrier; then wave 1 has finished the segment of the
    // phase before, whose freed slots go onto the group's free stack / free list here
    KDEV void phase_end() {
        KST(const unsigned long long tw0 = stamp();)
        two_barrier();
        KST(acc[ST_FAST_LEVEL] += stamp() - tw0;)          // (two waves: wave 0's wait for wave 1)
        const int b = (kp + 1) & 1;                           // the buffer wave 1 just finished
        ++kp;
        const int n = imin(U32(tl->lfcnt[b]), LFREE);
        if (n > 0) {
            const int fsp = gsv(GS_FSP), room = imin(n, FSTK - fsp);
            const int32_t s = lane < n ? tl->lfree[b][lane] : -1;
            if (lane < room) L.fstack[fsp + lane] = s;
            if (room < n) {                                   // the rest as one-slot blocks, chained
                const int32_t nx = __shfl(s, lane + 1 < n ? lane + 1 : lane);
                const int32_t old = gsv(GS_FREE_HEAD);
                if (lane >= room && lane < n) {
                    KG int32_t* w = reinterpret_cast<KG int32_t*>(&pool[s]);
                    w[0] = lane + 1 < n ? nx : old;
                    w[1] = 0;
                }
                set_gs(GS_FREE_HEAD, rl32(s, room));
            }
            set_gs(GS_FSP, fsp + room);
        }
        const int32_t ch = U32(tl->lch_head[b]);
        if (ch >= 0) {                                        // wave 1's overflow chain onto the free list
            if (lane == 0) reinterpret_cast<KG int32_t*>(&pool[U32(tl->lch_tail[b])])[0] = gsv(GS_FREE_HEAD);
            set_gs(GS_FREE_HEAD, ch);
        }
        if (lane == 0) { tl->lfcnt[b] = 0; tl->lch_head[b] = -1; tl->lch_tail[b] = -1; }
        if (U32(tl->lerr)) dead = true;                       // (raised by wave 1 at its record)
        sync_lds();
    }
    // wave 0: wave 1 idle (nothing handed over in this phase), before the serial path, the next
    // batch's prefetch and the group's end
    KDEV void drain() {
        if (!lbusy) return;
        if (lane == 0) tl->seg[kp & 1][3] = TW_NONE;
        phase_end();
        lbusy = false;
    }
    // wave 1: every phase, the segment wave 0 handed over in the phase before; returns at TW_EXIT
    KDEV void run_levels(uint32_t& tpos, uint32_t& tlim) {
        for (int k = 0;; ++k) {
            if (k > 0) {
                const int b = (k - 1) & 1;
                if (U32(tl->seg[b][3]) == TW_SEG) {
                    const int j0 = U32(tl->seg[b][0]), je = U32(tl->seg[b][1]), nev = U32(tl->seg[b][2]);
                    const int err = level_step<true>(tl->ev[b], tl->rin[b], tl->rid[b], nev, tpos, tlim, b);
                    // the segment's records: epilogue and OUT echo (wave 0 stores the other records')
                    const bool mine = lane >= j0 && lane < je;
                    int32_t on = 0;
                    if (mine) {
                        const int4 rc = tl->rec[b][lane], ri = tl->rin[b][lane];
                        int32_t oa = rc.x, op = rc.y, oh = rc.z;
                        epilogue(tl->ev[b], (uint32_t)ri.x, rc.w != 0, oa, op, oh, on);
                        Sp->osort[(uint32_t)ri.x] = make_int4((oa & 0xFF) | (((oa >> 16) & KME_OUT_HAS_PREV) << 8) | (on << 9),
                                                              ri.z, op, oh);
                    }
                    // a record with more trades than an ordinal counts (k_match's batch check)
                    const unsigned long long big = __ballot(mine && (uint32_t)on >= OS_MAX_NTR);
                    if (big) raise_wave(ctr(), KME_E_CAPACITY, KME_D_CAP_TRADES, (int64_t)U32(tl->rin[b][__builtin_ctzll(big)].x));
                    if (__ballot(err != 0) && __ballot(err == 2))
                        raise_wave(ctr(), KME_E_DOMAIN, KME_D_NPE_ORDER, (int64_t)U32(tl->rin[b][j0].x));
                    if ((big || __ballot(err != 0)) && lane == 0) tl->lerr = 1;
                }
            }
            two_barrier();
            if (U32(tl->seg[k & 1][3]) == TW_EXIT) break;
        }
        for (uint32_t q = tpos; q < tlim; ++q) Sp->ttmp[q].seq = -1;   // unused trade reservations
    }

    // ---------------- one record (MatchingEngine.process, KP:96-126)
    KDEV Out process(const Rec& r, const Lanes& B) {
        cur = r.i;
        Out o;
        o.action = r.action; o.size = r.size; o.prev = 0; o.has_prev = false; o.rested = false; o.ntr = 0;
        bool ok = false;
        switch (r.action) {
        case ADD_SYMBOL:                                    // addSymbol, KP:184-191
            if (!gsv(GS_EXISTS)) { set_gs(GS_EXISTS, 1); set_bm(0, 0, 0); set_bm(1, 0, 0); ok = true; }
            break;
        case REMOVE_SYMBOL:
        case PAYOUT:
            if (gsv(GS_EXISTS)) {                           // removeSymbol, KP:193-198 / removeAllOrders KP:341-353
                const int s = r.sid < 0 ? 1 : 0;
                if (bl(s) != 0 || bm(s) != 0) { die(KME_E_DOMAIN, KME_D_HANG); return o; }
            } else {
                ok = r.action == REMOVE_SYMBOL;
                if (r.action == PAYOUT) { die(KME_E_UNSUPPORTED, KME_D_NONE); return o; }
            }
            if (r.action == PAYOUT) ok = false;             // result ignored (KP:113-115)
            break;
        case BUY:
        case SELL: {
            if (!gsv(GS_EXISTS) || !r.acct_ok) break;   // books.get(sid) == null / balances.get == null
            const bool is_buy = r.action == BUY;
            const int os = r.sid == 0 ? 0 : 1 - book_side(r.sid, is_buy);   // opposite book (the same for sid 0)
            int32_t tsize = r.size;
            uint32_t ntr = 0;
            KST(unsigned long long tp0 = stamp();)
            const bool filled = try_match(r.price, tsize, is_buy, os, ntr);
            KST(unsigned long long tp1 = stamp(); if (ntr == 0) acc[ST_TM_PRE] += tp1 - tp0;)
            o.ntr = ntr;
            if (dead) return o;
            if (!filled) { rest(r, tsize, o); if (dead) return o; }
            ok = true;
            o.size = tsize;
            break;
        }
        case CANCEL:
            ok = cancel(r, B);
            if (dead) return o;
            break;
        default:
            break;
        }
        o.action = ok ? r.action : (int32_t)REJECT;
        return o;
    }
};

// (2) FUNDED: one wavefront per symbol group, the group's records in arrival order.
// all: k_match_lanes is not launched this epoch (its last launch found no light group), so the
// light groups are k_match's too.
// Four wavefronts per SIMD (<= 128 VGPRs; left to itself the compiler takes 134 and three): same-box
// A/B against three, C2 / C5 / the N = 8 shard shape 1-10% faster.  WAVES = 5 (<= 96 VGPRs, 48 B of
// spills) is the launch for many busy groups and few removes (the shard shapes: N = 8 +2.7% same-box);
// cancel-heavy epochs (C5) lose up to 16% with it and two-wave epochs (C2) gain nothing, so they keep four.
// TWO: two wavefronts per group (TwoLds): wave 0 below, wave 1 GroupWave::run_levels.
// One group's records (the body of k_match's block, and of each of k_match_list's iterations).
template <bool TWO>
KDEV __attribute__((always_inline)) void match_group(const DevState* __restrict__ Sp, const EpochIO* __restrict__ iop, int buf,
                                                     int all, int32_t g, GroupLds& lds, TwoLds* tlsp) {
    const DevState& S = *Sp;
    if (g >= S.G) return;
    const uint32_t b = S.seg[g], e = S.seg[g + 1];
    if (b >= e || (!all && e - b <= (uint32_t)S.light_max)) return;   // empty, or a light group (k_match_lanes)
    if (S.ctr[ci(C_FALLBACK)]) return;
    const uint32_t lim = err_limit(S.ctr, iop->n);          // records from a fault on do not take effect
    if (threadIdx.x == 0 && e - b > (uint32_t)S.light_max) atomicAdd(&S.ctr[ci(C_BUSY)], 1ull);
    KST(const unsigned long long tk0 = stamp();)
    GroupWave w(S, lds, g);
    const int lane = lane_id();
    if constexpr (TWO) {
        TwoLds& tls = *tlsp;
        w.tl = &tls;
        if (threadIdx.x >= 64) {                            // wave 1: the level steps
            uint32_t tpos = 0, tlim = 0;
            w.run_levels(tpos, tlim);
            return;
        }
        if (lane < 2) { tls.lfcnt[lane] = 0; tls.lch_head[lane] = -1; tls.lch_tail[lane] = -1; }
        if (lane == 0) tls.lerr = 0;
    }
    w.load_group();
    KST(w.acc[ST_GROUP_IN] += stamp() - tk0;)
    uint32_t n_rest = 0, n_cancel = 0;
    bool stop = false;
    // fast segments (GroupWave::fast_segment): not for group 0 (one shared book, H4) nor once a
    // size-0 order was ever submitted (C_SIZE0)
    const bool fast = g != 0 && S.fast && !S.ctr[ci(C_SIZE0)];
    uint32_t ftpos = 0, ftlim = 0;                          // this lane's trade scratch (fast segments)
    for (uint32_t k0 = b; k0 < e && !w.dead && !stop; k0 += 64) {
        KST(const unsigned long long tb0 = stamp();)
        const uint32_t k = k0 + lane;
        const bool valid = k < e;
        const KC DevState& C = opaque_const(Sp);
        const KG uint32_t* perm = buf ? C.rvals[1] : C.rvals[0];
        const KG int4* prec = C.prec;
        const KG Node* pool = C.pool;
        Lanes B;
        B.i = valid ? perm[k] : 0;
        if (valid) {   // one 32-byte gather per record (PRec, written by k_route)
            const int4 p0 = prec[2 * (size_t)B.i], p1 = prec[2 * (size_t)B.i + 1];
            B.w0 = p0.x; B.size = p0.y;
            B.oid = mk64(p0.z, p0.w); B.aid = mk64(p1.x, p1.y); B.tgt = p1.z;
            B.vl = (p0.x & 0xFF) == CANCEL ? p1.w : 0;
        } else {
            B.w0 = 0xFF; B.size = 0; B.oid = B.aid = 0; B.tgt = -1; B.vl = 0;
        }
        const int32_t b_action = B.w0 & 0xFF;
        // cancels: the target node, if it came to rest before this batch (an earlier epoch, or an
        // earlier batch of this group), is fetched now; valid unless written since (dirty filter)
        B.pf_slot = -1;
        B.pf_meta = 0; B.pf_size = B.pf_next = B.pf_prev = 0; B.pf_poid = 0;
        if (valid && b_action == CANCEL) {
            if (B.tgt >= 0) {
                B.pf_slot = B.tgt;
            } else if (B.tgt <= -2) {   // final unless the order is in this batch (then still pending:
                                        // pf_meta keeps the raw word, RS_PENDING; -1: did not rest)
                const int32_t v = C.rest_slot[-(B.tgt + 2)];
                if (v < 0) B.pf_meta = v;   // (RS_PENDING also when it did not rest: the pass finds it
                else B.pf_slot = v;         // outside the batch and leaves it to the serial path)
            }
        }
        if (B.pf_slot >= 0) {
            const KG int4* nd = reinterpret_cast<const KG int4*>(&pool[B.pf_slot]);
            const int4 c0 = nd[0], c1 = nd[1], c2 = nd[2], c3 = nd[3];
            const int64_t noid = mk64(c0.x, c0.y), naid = mk64(c0.z, c0.w), nsid = mk64(c1.x, c1.y);
            const bool ok = c3.z != 0 && noid == B.oid && naid == B.aid;
            // (price masked: a slot freed since it was indexed may host a free-list block, whose
            // word 12 is a slot id -- unmasked, its high bits would fake the ok bit)
            B.pf_meta = (c3.x & 0xFF) | (book_side(nsid, c3.y == BUY) << 8) | ((c3.y == SELL ? 1 : 0) << 9) | ((c1.y < 0 ? 1 : 0) << 10) |
                        ((ok ? 1 : 0) << 11);
            B.pf_poid = mk64(c2.x, c2.y);
            B.pf_size = c1.z; B.pf_next = c1.w; B.pf_prev = c2.z;
        }
        lds.dirty[lane] = 0;
        if constexpr (TWO) {   // the segment wave 1 has in hand: its writes may predate the filter
            w.bstale = w.lbusy;
            w.bpend_lo = w.lbusy ? w.pend_lo : 1u;
            w.bpend_hi = w.lbusy ? w.pend_hi : 0u;
            if (w.lbusy) {
                if (lane < 4) w.tl->bcb[lane] = w.tl->cb[lane];
                if (lane < 8) w.tl->btb[lane] = w.tl->tb[lane];
                w.tl->bfv[lane] = w.tl->fv[lane];
            }
        }
        w.sync_lds();
        // The lane registers are read with readlane inside the record loop.  Waiting for them here
        // once keeps the waitcnt pass from placing a vmcnt(0) at the loop header, which would make
        // every record wait for all stores of the record before it (stores share vmcnt on gfx9).
        __builtin_amdgcn_s_waitcnt(VMCNT0);
        // the batch's records before the epoch's first fault (a group's records are in arrival order)
        const int nb = (int)__popcll(__ballot(valid && B.i < lim));
        stop = nb < (int)(e - k0 < 64 ? e - k0 : 64);
        int done = nb;                // records of the batch that took effect (a fault ends the group)
        // per-record OUT fields collect in lane j of these registers; one store per field per batch
        int32_t o_act = 0, o_size = 0, o_plo = 0, o_phi = 0, o_ntr = 0;   // o_act: action | flags << 16
        KST(w.acc[ST_BATCH] += stamp() - tb0;)
#pragma nounroll
        for (int j = 0; j < nb; ++j) {
            if (fast) {
                const int jf0 = j;
                KST(const unsigned long long tf0 = stamp();)
                j = w.fast_segment<TWO>(B, j, nb, o_act, o_size, o_plo, o_phi, o_ntr, ftpos, ftlim);
                KST(w.acc[ST_FAST] += stamp() - tf0; w.acc[ST_N_FAST_REC] += (unsigned long long)(j - jf0); w.acc[ST_N_FAST_SEG] += j > jf0;)
                if (w.dead) { done = j; break; }
                if (j >= nb) break;
                // a segment that took records and stopped where a new segment can go on leaves its
                // next record to one (fast_segment's seg_retry)
                if (j > jf0 && w.seg_retry) { --j; continue; }
            }
            if constexpr (TWO) {
                // the serial path needs every node it reads final: wave 1 finishes its segment first,
                // except for a cancel whose victim's level neither the segment in flight nor the one
                // in flight at the batch's prefetch touches (their levels' lists, heads and nodes are
                // the cancel's alone) and whose same-epoch target is in neither
                bool wait = true;
                if (w.lbusy && (rl32(B.w0, j) & 0xFF) == CANCEL) {
                    const int32_t vl = rl32(B.vl, j), tg = rl32(B.tgt, j);
                    if ((vl >> 9) & 1) {
                        const int lev = ((vl >> 8) & 1) * 128 + (vl & 0xFF);
                        const uint32_t bit = 1u << (lev & 31);
                        wait = (U32((int32_t)w.tl->tb[lev >> 5]) & bit) || (w.bstale && (U32((int32_t)w.tl->btb[lev >> 5]) & bit));
                        if (tg <= -2) {
                            const uint32_t ti = (uint32_t)(-(tg + 2));
                            wait = wait || (ti >= w.pend_lo && ti <= w.pend_hi) || (ti >= w.bpend_lo && ti <= w.bpend_hi);
                        }
                    }
                }
                if (wait) w.drain();
                if (w.dead) { done = j; break; }
            }
            KST(const unsigned long long tr0 = stamp();)
            Rec r;
            r.i = (uint32_t)rl32((int32_t)B.i, j);
            const int32_t w0 = rl32(B.w0, j);
            r.action = w0 & 0xFF;
            r.price = (w0 >> 8) & 0xFF;
            r.acct_ok = (w0 >> 16) & 1;
            r.sid = (w0 >> 17) & 1 ? -(int64_t)g : (int64_t)g;
            r.size = rl32(B.size, j);
            r.oid = rl64(B.oid, j); r.aid = rl64(B.aid, j); r.tgt = (int64_t)rl32(B.tgt, j);
            r.lane = j;
            KST(w.acc[ST_REC_PICK] += stamp() - tr0;)
            const Out o = w.process(r, B);
            if (w.dead) { done = j; break; }   // the faulting record is not answered
#ifdef KME_STAMPS
            {
                const unsigned long long dt = stamp() - tr0;
                // constant indices only: a computed index puts acc[] in scratch memory
                if (r.action == BUY || r.action == SELL) {
                    if (o.ntr) { w.acc[ST_TRADE_REC] += dt; w.acc[ST_N_TRADE_REC] += 1; }
                    else { w.acc[ST_REST_REC] += dt; w.acc[ST_N_REST_REC] += 1; }
                } else if (r.action == CANCEL) { w.acc[ST_CANCEL_REC] += dt; w.acc[ST_N_CANCEL_REC] += 1; }
                else w.acc[ST_OTHER_REC] += dt;
            }
#endif
            const bool me = lane == j;
            o_act = me ? ((o.action & 0xFFFF) | (o.has_prev ? (int32_t)KME_OUT_HAS_PREV << 16 : 0) | (o.rested ? 2 << 16 : 0))
                       : o_act;
            o_size = me ? o.size : o_size;
            o_plo = me ? lo32(o.prev) : o_plo;
            o_phi = me ? hi32(o.prev) : o_phi;
            o_ntr = me ? (int32_t)o.ntr : o_ntr;
            KST(w.acc[ST_REC_OUT] += stamp() - tr0;)
        }
        {   // a record with more trades than an ordinal counts: the fault is that record (the ones before
            // it in the batch are answered)
            // (two waves: wave 1 checks the records of fast segments, GroupWave::run_levels)
            const bool mine = !TWO || !((w.fastmask >> lane) & 1);
            const unsigned long long big = __ballot(lane < done && mine && (uint32_t)o_ntr >= OS_MAX_NTR);
            if (big) {
                done = __builtin_ctzll(big);
                w.cur = (uint32_t)rl32((int32_t)B.i, done);
                w.die(KME_E_CAPACITY, KME_D_CAP_TRADES);
            }
        }
        n_rest += (uint32_t)__popcll(__ballot(lane < done && ((o_act >> 16) & 2)));
        n_cancel += (uint32_t)__popcll(__ballot(lane < done && b_action == CANCEL && (o_act & 0xFFFF) == CANCEL));
        {   // one 16-B record per lane, at the record's input index (k_unsort reads them in order); lanes
            // past the batch's last answered record store to a dump slot behind the array instead of
            // branching: a divergent branch here joins the loop latch, and the uniformity analysis then
            // takes the batch loop's exit (w.dead) as divergent, demoting its state to lane masks
            // (two waves: wave 1 stores those of fast segments)
            const bool mine = !TWO || !((w.fastmask >> lane) & 1);
            const size_t dst = lane < done && mine ? (size_t)B.i : (size_t)opaque_const(Sp).os_base + (size_t)lane;
            opaque_const(Sp).osort[dst] = make_int4((o_act & 0xFF) | (((o_act >> 16) & KME_OUT_HAS_PREV) << 8) | (o_ntr << 9),
                                                    o_size, o_plo, o_phi);
        }
        if constexpr (TWO) {
            w.fastmask = 0;
            if (S.fast & 2) w.drain();                      // (diagnostic: no overlap across batches)
        }
    }
    KST(const unsigned long long to0 = stamp();)
    w.flush_trades();
    if constexpr (TWO) {                                    // wave 1 finishes, then leaves
        w.drain();
        if (lane == 0) w.tl->seg[w.kp & 1][3] = TW_EXIT;
        two_barrier();
    }
    for (uint32_t q = ftpos; q < ftlim; ++q) S.ttmp[q].seq = -1;   // the fast segments' unused reservations
    KST(w.acc[ST_FLUSH] += stamp() - to0;)
    w.store_group();
    KG unsigned long long* tsh = w.tsh();
    if (lane == 0) {
        if (n_rest) atomicAdd(&tsh[TS_RESTS], (unsigned long long)n_rest);
        if (n_cancel) atomicAdd(&tsh[TS_CANCELS], (unsigned long long)n_cancel);
        if (e - b <= (uint32_t)S.light_max) atomicAdd(&tsh[TS_LIGHT], 1ull);   // a light group (all): lanes next epoch
    }
#ifdef KME_STAMPS
    const unsigned long long tk1 = stamp();
    w.acc[ST_GROUP_OUT] += tk1 - to0;
    w.acc[ST_KERNEL] += tk1 - tk0;
    if (lane == 0)
        for (int q = 0; q < ST_N; ++q) S.dbg[(size_t)g * KME_DBG_WORDS + q] += w.acc[q];
#endif
}

template <bool TWO, int WAVES>
__global__ void __launch_bounds__(TWO ? 128 : 64) __attribute__((amdgpu_waves_per_eu(WAVES)))
k_match(const DevState* __restrict__ Sp, const EpochIO* __restrict__ iop,
                                                                      int buf, int all, int dense) {
    __shared__ GroupLds lds;
    const DevState& S = *Sp;
    // dense: block k takes the k-th listed group (the busy ones first in the grid, the rest exit)
    const int32_t g = dense ? (blockIdx.x < S.gcount[0] ? (int32_t)S.glist[blockIdx.x] : S.G) : (int32_t)blockIdx.x;
    if constexpr (TWO) {
        __shared__ TwoLds tls;
        match_group<true>(Sp, iop, buf, all, g, lds, &tls);
    } else {
        match_group<false>(Sp, iop, buf, all, g, lds, nullptr);
    }
}

// List mode: the groups k_segments listed (C_GLIST of them; none at C3), a block per group in turn
// over a grid far smaller than G.
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4)))
k_match_list(const DevState* __restrict__ Sp, const EpochIO* __restrict__ iop, int buf, int all) {
    __shared__ GroupLds lds;
    const DevState& S = *Sp;
    const uint32_t cnt = (uint32_t)S.ctr[ci(C_GLIST)];
    for (uint32_t x = blockIdx.x; x < cnt; x += gridDim.x) {
        match_group<false>(Sp, iop, buf, all, (int32_t)S.glist[x], lds, nullptr);
        __syncthreads();   // (the next group's set-up rewrites the LDS state)
    }
}

// ------------------------------------------------------------------ (2') FUNDED, light groups
// One LANE per symbol group.  With tens of thousands of groups and a few dozen records each
// (C3), the wavefront-per-group program is bound by the CU's single scalar issue port: ~150
// scalar instructions per record, one record at a time per wavefront.  Here 64 groups share one
// wavefront, each lane running its group's records in arrival order with per-lane (vector)
// control flow, the book levels read and written in HBM (no LDS staging), the level bitmaps and
// group scalars in VGPRs.  One vector instruction advances up to 64 groups; the cost is
// divergence (a step runs every path some lane takes) and one dependent HBM round trip per
// level / maker access instead of an LDS access.  Groups with more than DevState::light_max
// records in the epoch stay with k_match (which skips the light ones); both kernels keep the
// same persistent group format (GroupState, Level, Node, free-slot blocks).
constexpr int LFS = 16;           // per-lane free-slot stack in LDS (spills FBLK-slot blocks)
#ifndef KME_DIAG_NO_OUT
#define KME_DIAG_NO_OUT 0       // diagnostic builds only: skip the OUT echo stores of k_match_lanes
#endif
#ifndef KME_DIAG_NO_TRADE
#define KME_DIAG_NO_TRADE 0     // diagnostic builds only: skip the trade-record stores of k_match_lanes
#endif
#ifndef KME_LANE_GROUPS
#define KME_LANE_GROUPS 32
#endif
constexpr int LANE_TCH = kLaneTradeChunk;   // trade scratch slots a lane reserves at a time (sizing: kme_create)
constexpr int LANE_GROUPS = KME_LANE_GROUPS;   // groups per wavefront (the other lanes idle): two
                                  // wavefronts per SIMD at 65,536 groups, so one issues while the other waits
static_assert(LANE_GROUPS >= 1 && LANE_GROUPS <= 64, "k_match_lanes: one group per lane");

// OUT echo (DevState::osort, 16 B per record at its input index): action | has_prev << 8 |
// n_trades << 9, size, prev.
KDEV int4 os_pack(int32_t action, bool has_prev, uint32_t ntr, int32_t size, int64_t prev) {
    return make_int4((action & 0xFF) | (has_prev ? 1 << 8 : 0) | (int32_t)(ntr << 9), size, lo32(prev), hi32(prev));
}


struct GroupLane {
    const DevState& S;
    const EpochIO& io;
    int32_t (*fs)[64];            // fs[k][lane]: free-slot stack entry k of this lane
    KG unsigned long long* tsh;   // this wavefront's trade shard line
    uint32_t tbase;
    int lane;
    int32_t g;
    uint64_t b0l, b0m, b1l, b1m;  // level bitmaps of book +g / book -g
    int32_t exists, free_head, chunk_next, chunk_end, fsp;
    uint32_t cur;
    bool dead;
    size_t tpos, tlim;            // this lane's reserved trade scratch [tpos, tlim) (LANE_TCH at a time)
    uint32_t tspare;              // a spare reservation (shard offset), valid if has_spare: requested
    bool has_spare;               //   with a record's first gather, so running out costs no round trip
    // The last rest's stores, held back until the next record's gathers are issued (flush_rest): a
    // load waits for every older memory operation of the wavefront (vmcnt is in order), so stores
    // issued before the next record's loads would lengthen its first round trip.  The next record's
    // gathers take the values from here where they read what the rest wrote.
    bool pv = false;
    int32_t p_slot = -1, p_nprev = -1;   // the new node; the old tail whose next becomes p_slot (or -1)
    uint32_t p_otpos = 0;                // the oid-table entry that becomes p_slot
    KG Level* p_lev = nullptr;           // the level line, whole
    int4 p_node[4], p_l0, p_l1;
    LST(uint32_t nload = 0;)      // (stamps build) maker loads of the sweep beyond the first

    KDEV GroupLane(const DevState& s, const EpochIO& e, int32_t (*f)[64], int32_t gg)
        : S(s), io(e), fs(f), tsh(s.tsh + (size_t)(blockIdx.x & (TSHARDS - 1)) * CTR_STRIDE),
          tbase((blockIdx.x & (TSHARDS - 1)) * s.tshard_cap), lane(lane_id()), g(gg) {
        b0l = b0m = b1l = b1m = 0;
        exists = 0; free_head = -1; chunk_next = chunk_end = 0; fsp = 0;
        cur = 0; dead = false;
        tpos = tlim = 0;
        tspare = 0; has_spare = false;
    }
    KDEV void die(int status, int detail) { raise_thread(S.ctr, status, detail, (int64_t)cur); dead = true; }
    KDEV uint64_t bl(int side) const { return side ? b1l : b0l; }
    KDEV uint64_t bm(int side) const { return side ? b1m : b0m; }
    KDEV void set_bm(int side, uint64_t l, uint64_t m) { if (side) { b1l = l; b1m = m; } else { b0l = l; b0m = m; } }
    KDEV KG Level* level(int side, int p) const { return &S.lev[((size_t)g * 2 + side) * NLEV + p]; }

    KDEV void load_group() {
        const KG int4* gs = reinterpret_cast<const KG int4*>(&S.grp[g]);
        const int4 a = gs[0], b = gs[1], c = gs[2];
        b0l = (uint64_t)mk64(a.x, a.y); b0m = (uint64_t)mk64(a.z, a.w);
        b1l = (uint64_t)mk64(b.x, b.y); b1m = (uint64_t)mk64(b.z, b.w);
        exists = c.x; free_head = c.y; chunk_next = c.z; chunk_end = c.w;
        if (free_head >= 0) load_block();                   // once per epoch, before the first record
    }
    KDEV void store_group() {
        while (tpos < tlim) mark_hole(tpos++);               // the reservations' unused slots
        if (has_spare)
            for (uint32_t q = tspare; q < tspare + LANE_TCH && q < S.tshard_cap; ++q) mark_hole((size_t)tbase + q);
        while (fsp > 0) spill_block(fsp > FBLK ? fsp - FBLK : 0);
        KG int4* gs = reinterpret_cast<KG int4*>(&S.grp[g]);
        gs[0] = make_int4(lo32((int64_t)b0l), hi32((int64_t)b0l), lo32((int64_t)b0m), hi32((int64_t)b0m));
        gs[1] = make_int4(lo32((int64_t)b1l), hi32((int64_t)b1l), lo32((int64_t)b1m), hi32((int64_t)b1m));
        gs[2] = make_int4(exists, free_head, chunk_next, chunk_end);
    }

    // ---------------- node slots (the block format of GroupWave::spill_blocks)
    // A freed slot's node keeps live = 1 while the slot sits on this lane's stack: most are handed
    // out again within the epoch (a rest rewrites the whole node), so the store of live = 0 -- a
    // partial-line write to a random node -- is made only when the slot leaves the stack unused (in
    // a spilled block, including the ones store_group spills at the end).  Meanwhile a node on the
    // stack is dead to this lane's cancels (in_stack), the only readers of the group's nodes before
    // the group's next epoch.
    // Stack entries [b, fsp) become one block: the last entry hosts the others' ids.
    KDEV void spill_block(int b) {
        const int host = fs[fsp - 1][lane];
        const int cnt = fsp - 1 - b;                        // ids besides the host, <= FBLK - 1
        int32_t w[16];
        w[0] = free_head; w[1] = cnt;
#pragma unroll
        for (int k = 0; k < FBLK - 1; ++k) w[2 + k] = k < cnt ? fs[b + k][lane] : -1;
#pragma unroll
        for (int k = 0; k < FBLK - 1; ++k) if (k < cnt) S.pool[w[2 + k]].live = 0;
        w[14] = 0; w[15] = 0;                               // Node::live = 0
        KG int4* d = reinterpret_cast<KG int4*>(&S.pool[host]);
#pragma unroll
        for (int k = 0; k < 4; ++k) d[k] = make_int4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
        free_head = host;
        fsp = b;
    }
    // the free-list block at free_head onto the (empty) stack: its ids and the block's own slot
    KDEV void load_block() {
        const int32_t blk = free_head;
        const KG int4* d = reinterpret_cast<const KG int4*>(&S.pool[blk]);
        int4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = d[k];
        const int32_t w[16] = {v[0].x, v[0].y, v[0].z, v[0].w, v[1].x, v[1].y, v[1].z, v[1].w,
                               v[2].x, v[2].y, v[2].z, v[2].w, v[3].x, v[3].y, v[3].z, v[3].w};
        const int32_t cnt = w[1];
        fs[0][lane] = blk;
#pragma unroll
        for (int k = 0; k < FBLK - 1; ++k) if (k < cnt) fs[1 + k][lane] = w[2 + k];
        fsp = cnt + 1;
        free_head = w[0];
    }
    KDEV int32_t alloc_slot() {
        if (fsp == 0 && free_head >= 0) load_block();       // (a load in the record's step)
        if (fsp > 0) return fs[--fsp][lane];
        if (chunk_next >= chunk_end) {
            // one bump reservation for every lane of the wavefront that needs a chunk now
            const unsigned long long need = __ballot(1);
            const int leader = __ffsll((long long)need) - 1;
            const uint32_t rank = (uint32_t)__popcll(need & ((1ull << lane) - 1));
            unsigned long long c = 0;
            if (lane == leader) c = atomicAdd(&S.ctr[ci(C_POOL_BUMP)], (unsigned long long)POOL_CHUNK * __popcll(need));
            c = (unsigned long long)__shfl((long long)c, leader) + (unsigned long long)rank * POOL_CHUNK;
            if (c + POOL_CHUNK > S.pool_cap) { die(KME_E_CAPACITY, KME_D_CAP_POOL); return -1; }
            chunk_next = (int32_t)c;
            chunk_end = (int32_t)(c + POOL_CHUNK);
        }
        return chunk_next++;
    }
    KDEV void free_slot(int32_t s) {
        if (fsp == LFS) spill_block(LFS - FBLK);
        fs[fsp++][lane] = s;
    }
    KDEV bool in_stack(int32_t s) const {
        bool hit = false;
        for (int k = 0; k < fsp; ++k) hit |= fs[k][lane] == s;
        return hit;
    }

    // ---------------- trades: one TradeTmp per trade.  Each lane reserves LANE_TCH slots at a time
    // (one atomic per wavefront for the lanes that run out), so most trades need no returning
    // atomic on the record's chain; unused slots are holes (seq = -1) that k_scatter skips.
    KDEV void mark_hole(size_t pos) { S.ttmp[pos].seq = -1; }
    KDEV void refill_trades() {
        const unsigned long long need = __ballot(1);
        const int leader = __ffsll((long long)need) - 1;
        const uint32_t rank = (uint32_t)__popcll(need & ((1ull << lane) - 1));
        unsigned long long base = 0;
        if (lane == leader) base = atomicAdd(&tsh[TS_USED], (unsigned long long)LANE_TCH * __popcll(need));
        base = (unsigned long long)__shfl((long long)base, leader) + (unsigned long long)rank * LANE_TCH;
        if (base + LANE_TCH <= S.tshard_cap) {
            tpos = (size_t)tbase + base;
            tlim = tpos + LANE_TCH;
            return;
        }
        for (unsigned long long q = base; q < S.tshard_cap; ++q) mark_hole((size_t)tbase + q);   // straddles the end
        const unsigned long long ob = atomicAdd(&S.ctr[ci(C_TTMP)], (unsigned long long)LANE_TCH);
        if (ob + LANE_TCH > S.ttmp_cap) {
            for (unsigned long long q = ob; q < S.ttmp_cap; ++q) mark_hole((size_t)TSHARDS * S.tshard_cap + q);
            die(KME_E_CAPACITY, KME_D_CAP_TRADES);
            return;
        }
        tpos = (size_t)TSHARDS * S.tshard_cap + ob;
        tlim = tpos + LANE_TCH;
    }
    // with the record's first gather: a spare reservation for a lane about to run out (one
    // returning atomic per lane, in flight with the gather)
    KDEV void request_spare() {
        if (!has_spare && tlim - tpos <= 2) {
            tspare = (uint32_t)atomicAdd(&tsh[TS_USED], (unsigned long long)LANE_TCH);
            has_spare = true;
        }
    }
    KDEV void emit(uint32_t ord, int64_t moid, int64_t maid, int32_t msneg, int32_t mprice, int32_t ts) {
        if (tpos == tlim) {
            if (has_spare && tspare + LANE_TCH <= S.tshard_cap) {
                tpos = (size_t)tbase + tspare;
                tlim = tpos + LANE_TCH;
                has_spare = false;
            } else {
                refill_trades();
                if (dead) return;
            }
        }
        const size_t pos = tpos++;
        if (KME_DIAG_NO_TRADE) return;
        KG int4* r = reinterpret_cast<KG int4*>(&S.ttmp[pos]);
        r[0] = make_int4(lo32(moid), hi32(moid), lo32(maid), hi32(maid));
        r[1] = make_int4((int32_t)cur, (int32_t)tt_ordp(ord, mprice, msneg != 0), ts, g);
    }

    // ---------------- tryMatch, KP:225-263: the loop of GroupWave::try_match (no sweep scan), from
    // the first maker on (its level and node were fetched by the record's first two gathers)
    KDEV bool try_match(int32_t P, int32_t& tsize, bool is_buy, int os, uint32_t& ntr, int32_t pb, int32_t ms,
                        int64_t lqty, int4 m0, int4 m1) {
        KG Level* lv = level(os, pb);
        bool head_moved = false;
        for (;;) {
            const int32_t msz = m1.z, mnext = m1.w;
            const int32_t ts = imin(tsize, msz);
            const int32_t msize = jisub(msz, ts);
            tsize = jisub(tsize, ts);
            lqty -= ts;
            emit(ntr++, mk64(m0.x, m0.y), mk64(m0.z, m0.w), m1.y < 0, pb, ts);
            if (dead) return false;
            if (msize != 0) {                                // maker stays, partially filled (KP:255-261)
                S.pool[ms].size = msize;
                if (head_moved) { lv->head = ms; S.pool[ms].prev = -1; }
                lv->qty = lqty;
                return tsize == 0;
            }
            free_slot(ms);                                   // maker consumed: orders.delete (KP:243)
            if (mnext >= 0) {
                ms = mnext;
                if (!GroupWave::crosses(is_buy, tsize, pb, P)) {   // stops before the next maker
                    lv->head = ms;
                    S.pool[ms].prev = -1;
                    lv->qty = lqty;
                    return tsize == 0;
                }
                head_moved = true;
            } else {                                         // level exhausted (KP:244-253)
                uint64_t lo = bl(os), hi = bm(os);
                unset_bit(lo, hi, pb);
                set_bm(os, lo, hi);
                const int32_t npb = is_buy ? min_price_ptr(lo, hi) : max_price_ptr(lo, hi);
                const bool go = npb != -1 && check_bit(lo, hi, npb) && GroupWave::crosses(is_buy, tsize, npb, P);
                if (!go) {
                    if (npb != -1 && !check_bit(lo, hi, npb)) die(KME_E_DOMAIN, KME_D_NPE_BUCKET);
                    return tsize == 0;
                }
                pb = npb;
                lv = level(os, pb);
                ms = lv->head;
                lqty = lv->qty;
                if (ms < 0) { die(KME_E_DOMAIN, KME_D_NPE_ORDER); return false; }
                head_moved = false;
            }
            m0 = reinterpret_cast<const KG int4*>(&S.pool[ms])[0];
            m1 = reinterpret_cast<const KG int4*>(&S.pool[ms])[1];
            LST(++nload;)
        }
    }

    // ---------------- addOrder, KP:200-223 (own: the level at the order's price, when prefetched)
    KDEV void rest(const Rec& r, int32_t tsize, Out& o, bool own_pre, int4 l0, int4 l1) {
        const int s = book_side(r.sid, r.action == BUY);
        uint64_t lo = bl(s), hi = bm(s);
        const int32_t p = r.price;
        const int32_t slot = alloc_slot();
        if (dead) return;
        KG Level* lv = level(s, p);
        int32_t nprev = -1;
        int64_t poid = 0;
        if (!check_bit(lo, hi, p)) {                         // new bucket (KP:209-211)
            p_l0 = make_int4(slot, slot, 0, 0);
            p_l1 = make_int4((int32_t)tsize, tsize < 0 ? -1 : 0, lo32(r.oid), hi32(r.oid));
            set_bit(lo, hi, p);
            set_bm(s, lo, hi);
        } else {                                             // append at the tail (KP:213-219)
            if (!own_pre) { l0 = reinterpret_cast<const KG int4*>(lv)[0]; l1 = reinterpret_cast<const KG int4*>(lv)[1]; }
            nprev = l0.y;
            poid = mk64(l1.z, l1.w);
            const int64_t q = mk64(l1.x, l1.y) + tsize;
            p_l0 = make_int4(l0.x, slot, l0.z, l0.w);
            p_l1 = make_int4(lo32(q), hi32(q), lo32(r.oid), hi32(r.oid));
            o.has_prev = true;
            o.prev = poid;
        }
        // its oid-table entry (k_emap's pending one: r.tgt of a BUY/SELL is its position) becomes the
        // rest slot, one 4-B store -- no rest_slot store and no pass in k_unsort (k_match's groups
        // store rest_slot, which k_unsort copies)
        // (consistency check: a BUY/SELL's own entry position from k_emap, never outside the table)
        if (r.tgt > (int64_t)S.otab_mask) {
            printf("kme guard: k_match_lanes rest i=%u tgt=%lld size=%d otab_mask=%u g=%d\n", r.i, (long long)r.tgt, r.size,
                   S.otab_mask, g);
            die(KME_E_CAPACITY, KME_D_GUARD_OTPOS);
            return;
        }
        p_node[0] = make_int4(lo32(r.oid), hi32(r.oid), lo32(r.aid), hi32(r.aid));
        p_node[1] = make_int4(lo32(r.sid), hi32(r.sid), tsize, -1);
        p_node[2] = make_int4(lo32(poid), hi32(poid), nprev, g);
        p_node[3] = make_int4(p, r.action, 1, 0);
        p_slot = slot; p_nprev = nprev; p_otpos = (uint32_t)r.tgt; p_lev = lv;
        pv = true;                                           // (stored by flush_rest)
        o.rested = true;
    }

    KDEV void flush_rest() {
        if (!pv) return;
        pv = false;
        KG int4* lvp = reinterpret_cast<KG int4*>(p_lev);
        lvp[0] = p_l0;
        lvp[1] = p_l1;
        if (p_nprev >= 0) S.pool[p_nprev].next = p_slot;
        KG int4* nd = reinterpret_cast<KG int4*>(&S.pool[p_slot]);
        nd[0] = p_node[0]; nd[1] = p_node[1]; nd[2] = p_node[2]; nd[3] = p_node[3];
        otab_final(S.otab, (int32_t)p_otpos, p_slot);
    }
    // a node the held-back rest wrote, as the next record's gather must see it (all four 16-B pieces)
    KDEV void fwd_node(int32_t s, int4& c0, int4& c1, int4& c2, int4& c3) const {
        if (!pv) return;
        if (s == p_slot) { c0 = p_node[0]; c1 = p_node[1]; c2 = p_node[2]; c3 = p_node[3]; }
        else if (s == p_nprev) c1.w = p_slot;               // the old tail: its next
    }

    // ---------------- removeOrder, KP:289-323 (victim node c0..c3; vl1: its level's qty words when
    // k_route knew the level, vlev = price | side << 8 | 1 << 9)
    KDEV bool cancel(const Rec& r, int32_t slot, int4 c0, int4 c1, int4 c2, int4 c3, int32_t vlev, int4 vl1) {
        if (slot < 0) return false;                          // orders.get(oid) == null
        if (!(c3.z != 0 && mk64(c0.x, c0.y) == r.oid && mk64(c0.z, c0.w) == r.aid)) return false;   // KP:291
        if (in_stack(slot)) return false;                    // freed this epoch (filled or removed)
        if (!exists) { die(KME_E_DOMAIN, KME_D_NPE_BOOK); return false; }
        const int32_t action = c3.y, price = c3.x, size = c1.z, next = c1.w, prev = c2.z;
        const int64_t prev_oid = mk64(c2.x, c2.y);
        const int side = book_side(mk64(c1.x, c1.y), action == BUY);
        KG Level* lv = level(side, price);
        if (prev < 0 && next < 0) {
            uint64_t lo = bl(side), hi = bm(side);
            unset_bit(lo, hi, price);
            set_bm(side, lo, hi);
        } else {
            if (prev < 0) {
                lv->head = next;
                S.pool[next].prev = -1;
            } else if (next < 0) {
                lv->tail = prev;
                lv->tail_oid = prev_oid;
                S.pool[prev].next = -1;
            } else {
                S.pool[prev].next = next;
                S.pool[next].prev = prev;
                S.pool[next].prev_oid = prev_oid;
            }
            const int64_t q = vlev == (price | (side << 8) | (1 << 9)) ? mk64(vl1.x, vl1.y) : lv->qty;
            lv->qty = q - size;
        }
        free_slot(slot);
        if (S.ledger_replay)   // the removed order, for postRemoveAdjustments in k_ledger_replay
            S.vic[r.i] = make_int4(price | ((action == SELL ? SELL : BUY) << 8), size, c1.y < 0 ? -g : g, c1.y < 0 ? -1 : 0);
        return !dead;
    }
};

// The records of the 64 groups run in lock step, one record per lane per step.  A step's loads
// are issued in two gathers shared by every record type (first: the taker's best opposite level,
// a resting order's own level, a cancel's target node or rest slot and its level; second: the
// taker's first maker, a same-epoch cancel's node), so the round trips of a step are ~2 plus the
// makers beyond the first, not the sum of every path's chain.
#ifdef KME_LANES_WAVES   // diagnostic builds: a VGPR cap for k_match_lanes (waves per SIMD)
#define KME_LANES_ATTR __attribute__((amdgpu_waves_per_eu(KME_LANES_WAVES)))
#else
#define KME_LANES_ATTR
#endif
__global__ void __launch_bounds__(64) KME_LANES_ATTR k_match_lanes(const DevState* __restrict__ Sp, const EpochIO* __restrict__ iop, int buf) {
    __shared__ int32_t fs[LFS][64];
    const DevState& S = *Sp;
    const EpochIO& io = *iop;
    if (S.ctr[ci(C_FALLBACK)]) return;
    const uint32_t lim = err_limit(S.ctr, io.n);             // records from a fault on do not take effect
    const int32_t g = (int32_t)(blockIdx.x * LANE_GROUPS + lane_id());
    uint32_t b = 0, e = 0;
    if (lane_id() < LANE_GROUPS && g < S.G) { b = S.seg[g]; e = S.seg[g + 1]; }
    if (e - b > (uint32_t)S.light_max) e = b;                // a heavy group: k_match's
    const bool has_group = __ballot(b < e) != 0;             // (C_LIGHT: the next epoch's launch choice)
    uint32_t n_rest = 0, n_cancel = 0;
    if (b < e) {
        GroupLane w(S, io, fs, g);
        w.load_group();
        const KG uint32_t* perm = buf ? S.rvals[1] : S.rvals[0];
        // records are fetched one step ahead (their input indices two ahead), before the step's
        // stores: a load waits for every older vector memory operation (vmcnt is in order on gfx9)
        uint32_t i_next = perm[b];
        uint32_t i_after = b + 1 < e ? perm[b + 1] : 0;
        int4 n0 = S.prec[2 * (size_t)i_next], n1 = S.prec[2 * (size_t)i_next + 1];
        const int4 z = make_int4(0, 0, 0, 0);
        LST(unsigned long long lacc[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}; unsigned long long lt = lstamp();)
        // the previous record's OUT echo: stored after this record's first gather is issued, so the
        // gather's wait does not include it (vmcnt counts loads and stores in issue order)
        size_t pend_pos = 0;
        int4 pend_a = make_int4(0, 0, 0, 0);
        bool pend = false;
        for (uint32_t k = b; k < e && !w.dead; ++k) {
            if (i_next >= lim) break;                        // arrival order: the rest of the group too
            LST({ const unsigned long long t1 = lstamp(); lacc[0] += t1 - lt; lt = t1; lacc[7] += 1; })
            Rec r;
            r.i = i_next;
            const int4 p0 = n0, p1 = n1;
            if (k + 1 < e) {
                i_next = i_after;
                n0 = S.prec[2 * (size_t)i_next]; n1 = S.prec[2 * (size_t)i_next + 1];
                i_after = k + 2 < e ? perm[k + 2] : 0;
            }
            r.action = p0.x & 0xFF;
            r.price = (p0.x >> 8) & 0xFF;
            r.acct_ok = (p0.x >> 16) & 1;
            r.sid = (p0.x >> 17) & 1 ? -(int64_t)g : (int64_t)g;
            r.size = p0.y;
            r.oid = mk64(p0.z, p0.w); r.aid = mk64(p1.x, p1.y); r.tgt = (int64_t)p1.z;
            r.lane = 0;
            const int32_t vlev = p1.w;
            w.cur = r.i;
            Out o;
            o.action = r.action; o.size = r.size; o.prev = 0; o.has_prev = false; o.rested = false; o.ntr = 0;
            bool ok = false;
            const bool order = (r.action == BUY || r.action == SELL) && w.exists && r.acct_ok;
            const bool cxl = r.action == CANCEL;
            // ---- what the record reads first (MatchingEngine.process, KP:96-126)
            bool is_buy = r.action == BUY, tm = false, filled = false, own_pre = false;
            int os = 0;
            int32_t pb = -1, tsize = r.size;
            if (order) {
                os = r.sid == 0 ? 0 : 1 - book_side(r.sid, is_buy);   // opposite book (the same for sid 0)
                const uint64_t lo = w.bl(os), hi = w.bm(os);
                pb = is_buy ? min_price_ptr(lo, hi) : max_price_ptr(lo, hi);
                if (pb != -1) {
                    if (!check_bit(lo, hi, pb)) w.die(KME_E_DOMAIN, KME_D_NPE_BUCKET);
                    else if (GroupWave::crosses(is_buy, tsize, pb, r.price)) tm = true;
                    else filled = tsize == 0;
                }
                const int s = book_side(r.sid, is_buy);      // the order's own level, unless sid 0 (one
                own_pre = g != 0 && check_bit(w.bl(s), w.bm(s), r.price);   // book: the sweep may change it)
            }
            const KG int4* la = nullptr;                     // a level: the taker's, or the cancel target's
            if (tm) la = reinterpret_cast<const KG int4*>(w.level(os, pb));
            else if (cxl && ((vlev >> 9) & 1)) la = reinterpret_cast<const KG int4*>(w.level((vlev >> 8) & 1, vlev & 0xFF));
            int4 la0 = z, la1 = z, lo0 = z, lo1 = z, c0 = z, c1 = z, c2 = z, c3 = z;
            int32_t vslot = -1;
            // ---- first gather
            if (la) { la0 = la[0]; la1 = la[1]; }
            if (own_pre) {
                const KG int4* lp = reinterpret_cast<const KG int4*>(w.level(book_side(r.sid, is_buy), r.price));
                lo0 = lp[0]; lo1 = lp[1];
            }
            if (cxl) {
                if (r.tgt >= 0) {
                    vslot = (int32_t)r.tgt;
                    const KG int4* nd = reinterpret_cast<const KG int4*>(&S.pool[vslot]);
                    c0 = nd[0]; c1 = nd[1]; c2 = nd[2]; c3 = nd[3];
                    w.fwd_node(vslot, c0, c1, c2, c3);
                } else if (r.tgt <= -2) {   // an order of this epoch (earlier in arrival order, so decided):
                    // the low word of its oid-table entry (position in the size word, k_route) -- its rest
                    // slot, or still pending if it did not rest
                    const uint32_t hv = (uint32_t)r.size;
                    uint32_t v = hv <= S.otab_mask ? reinterpret_cast<const KG uint32_t*>(S.otab)[2 * (size_t)hv] : OT_DEAD;
                    if (w.pv && hv == w.p_otpos) v = (uint32_t)w.p_slot;   // (the held-back rest's entry)
                    vslot = (v & OT_PENDING) ? -1 : (int32_t)v;
                    // (consistency checks: k_route's entry position, the entry's slot)
                    if (hv > S.otab_mask || (vslot >= 0 && (uint32_t)vslot >= S.pool_cap)) {
                        printf("kme guard: k_match_lanes cancel i=%u tgt=%lld pos=%u entry=%u otab_mask=%u pool_cap=%u g=%d\n", r.i,
                               (long long)r.tgt, hv, v, S.otab_mask, S.pool_cap, g);
                        w.die(KME_E_CAPACITY, hv > S.otab_mask ? KME_D_GUARD_OTPOS : KME_D_GUARD_SLOT);
                        vslot = -1;
                    }
                }
            }
            if (w.pv) {                                      // levels the held-back rest wrote
                const KG int4* pl = reinterpret_cast<const KG int4*>(w.p_lev);
                if (la == pl) { la0 = w.p_l0; la1 = w.p_l1; }
                if (own_pre && reinterpret_cast<const KG int4*>(w.level(book_side(r.sid, is_buy), r.price)) == pl) {
                    lo0 = w.p_l0; lo1 = w.p_l1;
                }
            }
            if (order) w.request_spare();
            if (pend && !KME_DIAG_NO_OUT) S.osort[pend_pos] = pend_a;
            pend = false;
            LST({ const unsigned long long t1 = lstamp(); lacc[1] += t1 - lt; lt = t1; })
            // ---- second gather
            int32_t ms = -1;
            int64_t lqty = 0;
            int4 m0 = z, m1 = z;
            if (tm) {
                ms = la0.x;
                lqty = mk64(la1.x, la1.y);
                if (ms < 0) { w.die(KME_E_DOMAIN, KME_D_NPE_ORDER); tm = false; }
                else {
                    const KG int4* nd = reinterpret_cast<const KG int4*>(&S.pool[ms]);
                    m0 = nd[0]; m1 = nd[1];
                    int4 x2 = z, x3 = z;
                    w.fwd_node(ms, m0, m1, x2, x3);
                }
            }
            if (cxl && r.tgt <= -2 && vslot >= 0) {
                const KG int4* nd = reinterpret_cast<const KG int4*>(&S.pool[vslot]);
                c0 = nd[0]; c1 = nd[1]; c2 = nd[2]; c3 = nd[3];
                w.fwd_node(vslot, c0, c1, c2, c3);
            }
            w.flush_rest();                                  // (after both gathers are issued)
            if (w.dead) break;
            LST({ const unsigned long long t1 = lstamp(); lacc[2] += t1 - lt; lt = t1; })
            // ---- the record
            if (order) {
                uint32_t ntr = 0;
                LST(const unsigned long long tq0 = lstamp(); w.nload = 0;)
                if (tm) filled = w.try_match(r.price, tsize, is_buy, os, ntr, pb, ms, lqty, m0, m1);
                LST(const unsigned long long tq1 = lstamp(); lacc[5] += tq1 - tq0;
                    { uint32_t mx = w.nload; for (int off = 32; off > 0; off >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, off));
                      uint32_t sm = w.nload; for (int off = 32; off > 0; off >>= 1) sm += (uint32_t)__shfl_xor((int)sm, off);
                      lacc[8] += mx > 0; lacc[9] += sm; lacc[10] += mx; })
                o.ntr = ntr;
                if (w.dead) break;
                if (!filled) { w.rest(r, tsize, o, own_pre, lo0, lo1); if (w.dead) break; }
                LST(lacc[6] += lstamp() - tq1;)
                ok = true;
                o.size = tsize;
            } else if (cxl) {
                ok = w.cancel(r, vslot, c0, c1, c2, c3, vlev, la1);
                if (w.dead) break;
            } else if (r.action == ADD_SYMBOL) {             // addSymbol, KP:184-191
                if (!w.exists) { w.exists = 1; w.b0l = w.b0m = w.b1l = w.b1m = 0; ok = true; }
            } else if (r.action == REMOVE_SYMBOL || r.action == PAYOUT) {   // KP:193-198 / 341-353
                if (w.exists) {
                    const int s = r.sid < 0 ? 1 : 0;
                    if (w.bl(s) != 0 || w.bm(s) != 0) { w.die(KME_E_DOMAIN, KME_D_HANG); break; }
                } else {
                    ok = r.action == REMOVE_SYMBOL;
                    if (r.action == PAYOUT) { w.die(KME_E_UNSUPPORTED, KME_D_NONE); break; }
                }
                if (r.action == PAYOUT) ok = false;
            }                                                // BUY / SELL without book or balance: REJECT
            o.action = ok ? r.action : (int32_t)REJECT;
            LST({ const unsigned long long t1 = lstamp(); lacc[3] += t1 - lt; lt = t1; })
            {   // the OUT echo (step-major: the wavefront's stores of a step are one run), stored
                // next step
                if (o.ntr >= OS_MAX_NTR) { w.die(KME_E_CAPACITY, KME_D_CAP_TRADES); break; }
                pend_pos = (size_t)r.i;
                pend_a = os_pack(o.action, o.has_prev, o.ntr, o.size, o.has_prev ? o.prev : 0);
                pend = true;
            }
            n_rest += o.rested ? 1u : 0u;
            n_cancel += (cxl && ok) ? 1u : 0u;
            LST({ const unsigned long long t1 = lstamp(); lacc[4] += t1 - lt; lt = t1; })
        }
        w.flush_rest();
        if (pend && !KME_DIAG_NO_OUT) S.osort[pend_pos] = pend_a;
        LST(if (lane_id() == __ffsll((long long)__ballot(1)) - 1) for (int q = 0; q < 12; ++q) atomicAdd(&S.dbg[q], lacc[q]);)
        w.store_group();
    }
    // per-wavefront sums onto the shard line (k_tsh_fold adds the lines up)
    for (int off = 32; off > 0; off >>= 1) {
        n_rest += (uint32_t)__shfl_xor((int)n_rest, off);
        n_cancel += (uint32_t)__shfl_xor((int)n_cancel, off);
    }
    if (lane_id() == 0) {
        KG unsigned long long* tsh = S.tsh + (size_t)(blockIdx.x & (TSHARDS - 1)) * CTR_STRIDE;
        if (n_rest) atomicAdd(&tsh[TS_RESTS], (unsigned long long)n_rest);
        if (n_cancel) atomicAdd(&tsh[TS_CANCELS], (unsigned long long)n_cancel);
        if (has_group) atomicAdd(&tsh[TS_LIGHT], 1ull);
    }
}

// EXACT: one wavefront, the whole epoch in arrival order, every store exact.
__global__ void __launch_bounds__(64) k_serial(const DevState* __restrict__ Sp, const EpochIO* __restrict__ iop, int only_fallback) {
    const DevState& S = *Sp;
    const EpochIO& io = *iop;
    if (only_fallback && !S.ctr[ci(C_FALLBACK)]) return;   // FUNDED epoch whose proof held
    const uint32_t lim = err_limit(S.ctr, io.n);            // records before a fault raised by emap / route
    Core c(S, io);
    const int lane = lane_id();
    uint32_t n_rest = 0, n_cancel = 0;
    for (uint32_t k0 = 0; k0 < lim && !c.dead; k0 += 64) {
        const uint32_t k = k0 + lane;
        const bool valid = k < lim;
        // 64 records staged across the lanes, read with readlane (one gather per 64 records)
        const uint32_t bi = valid ? k : 0;
        const int32_t b_action = valid ? io.action[bi] : -1, b_price = valid ? io.price[bi] : 0;
        const int32_t b_size = valid ? io.size[bi] : 0;
        const int64_t b_oid = valid ? io.oid[bi] : 0, b_aid = valid ? io.aid[bi] : 0, b_sid = valid ? io.sid[bi] : 0;
        const int64_t b_tgt = valid ? S.cancel_tgt[bi] : 0;
        const int32_t bgrp = valid ? S.route_grp[bi] : -1;
        const int nb = (int)(lim - k0 < 64 ? lim - k0 : 64);
#pragma nounroll
        for (int j = 0; j < nb && !c.dead; ++j) {
            Rec r;
            r.i = k0 + (uint32_t)j;
            r.action = rl32(b_action, j); r.price = rl32(b_price, j); r.size = rl32(b_size, j);
            r.acct_ok = 0;
            r.oid = rl64(b_oid, j); r.aid = rl64(b_aid, j); r.sid = rl64(b_sid, j); r.tgt = rl64(b_tgt, j);
            r.lane = j;
            const uint32_t i = r.i;
            const int32_t a = r.action;
            int32_t grp = -1;
            if (a == CANCEL) {
                grp = rl32(bgrp, j);
                if (grp == GRP_RESOLVE) {   // an order on a sparse symbol (k_route): the node's group, or
                    if (r.tgt >= 0) {       // the symbol's of the same-epoch order it names
                        const Node nd = c.ld_node((int32_t)r.tgt);
                        grp = nd.live && nd.oid == r.oid && nd.group >= 0 && nd.group < S.G + S.Gs ? nd.group : -1;
                    } else {
                        grp = c.symbol_group(io.sid[(uint32_t)(-(r.tgt + 2))], false, i);
                    }
                }
            } else if (a == ADD_SYMBOL || a == REMOVE_SYMBOL || a == PAYOUT || a == BUY || a == SELL) {
                grp = c.symbol_group(r.sid, a == ADD_SYMBOL, i);
            }
            if (c.dead) break;
            if (grp >= 0) {
                if (grp != c.g) { c.store_group(); c.load_group(grp); }
                const Out o = c.process(r);
                n_rest += o.rested;
                n_cancel += a == CANCEL && o.action == CANCEL;
                if (!c.dead && lane == 0) {
                    io.out_action[i] = o.action;
                    io.out_size[i] = o.size;
                    io.out_prev[i] = o.prev;
                    io.out_flags[i] = o.has_prev ? (uint8_t)KME_OUT_HAS_PREV : (uint8_t)0;
                }
                continue;
            }
            // records without a symbol group
            io.trade_off[i] = c.tnext;
            bool ok = false;
            switch (a) {
            case CREATE_BALANCE: ok = c.create_balance(r.aid, i); break;
            case TRANSFER: ok = c.transfer(r.aid, r.size); break;
            case ADD_SYMBOL: c.die(KME_E_CAPACITY, KME_D_CAP_SYMBOL, i); break;   // (symbol_group died first)
            case REMOVE_SYMBOL: ok = true; break;           // absent symbol: removeSymbol returns true
            case PAYOUT: c.payout_settle(r.sid, r.size, i); break;
            default: break;                                 // BUY/SELL on absent book, unknown cancel, unknown action
            }
            if (c.dead) break;
            if (lane == 0) write_out(io, i, a, ok, r.size, false, 0);
        }
    }
    c.store_group();
    if (lane_id() == 0) {
        if (!c.dead && lim < io.n) io.trade_off[lim] = c.tnext;   // the trades before a fault raised by emap / route
        io.trade_off[io.n] = c.tnext;
        S.ctr[ci(C_TRADES)] = c.tnext;
        S.ctr[ci(C_RESTS)] = n_rest;
        S.ctr[ci(C_CANCEL_OK)] = n_cancel;
    }
}

// FUNDED, after the epoch's matching: the bounds roll forward (commit_funded), and with
// KME_FLAG_SERIAL_FALLBACK, after an epoch k_serial took, they restart from the exact ledger
// (balance = the tightest lower bound; an account exists from the epoch's end).
KDEV void tsh_fold(const DevState& S);
KDEV void table_final(const DevState& S, const EpochIO& io, uint32_t t0, uint32_t stride);
// nb: the account blocks; the blocks past them (KME_FLAG_SERIAL_FALLBACK engines) finalise the oid-table
// entries of an epoch k_serial took (was k_table, a launch per epoch that mostly found nothing to do)
__global__ void __launch_bounds__(256) k_settle_funded(DevState S, EpochIO io, uint32_t nb) {
    static_assert(TSHARDS == 256, "tsh_fold: one thread per shard line");
    if (blockIdx.x >= nb) {
        if (S.ctr[ci(C_FALLBACK)])
            table_final(S, io, (blockIdx.x - nb) * blockDim.x + threadIdx.x, (gridDim.x - nb) * blockDim.x);
        return;
    }
    if (blockIdx.x == 0) tsh_fold(S);   // the trade shards' counters (was k_tsh_fold, a launch of its own)
    const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (a >= S.A) return;
    commit_funded(S, io, a);
    if (!S.fallback || !S.ctr[ci(C_FALLBACK)] || failed(S.ctr)) return;
    uint32_t h = (uint32_t)mix64((uint64_t)a) & S.bal_mask;   // Core::bal_find
    int64_t bal = 0;
    bool found = false;
    for (uint32_t p = 0; p <= S.bal_mask; ++p) {
        const uint32_t st = S.bal_state[h];
        if (st == 0) break;
        if (st == 1 && S.bal_key[h] == a) { found = true; bal = S.bal_val[h]; break; }
        h = (h + 1) & S.bal_mask;
    }
    const int64_t end = io.seq_base + (int64_t)io.n;
    if (found) {
        if (!(S.acct_since[a] < end)) S.acct_since[a] = end - 1;
        S.acct_lb[a] = bal;
    } else {
        S.acct_since[a] = INT64_MAX;
        S.acct_lb[a] = 0;
    }
    S.acct_need[a] = 0; S.acct_negx[a] = 0; S.acct_xfer[a] = 0;
}

// FUNDED + KME_FLAG_EXACT_LEDGER (row f next-2): the epoch's ledger effects replayed in arrival
// order on one wavefront, after the parallel matching decided every outcome: createBalance /
// transfer (KP:131-146), checkBalance (KP:167-182) for each accepted BUY/SELL, both fillOrder calls
// per trade in executeTrade order (KP:265-287), postRemoveAdjustments (KP:325-333) for each
// accepted cancel -- all on the exact Balances / Positions tables of EXACT mode (Core), so the
// value-keyed position writes (KP:434-436) clobber exactly what the reference clobbers.
KDEV void ledger_replay(const DevState& S, const EpochIO& io) {
    if (failed(S.ctr) || S.ctr[ci(C_FALLBACK)]) return;   // a serial epoch kept the exact ledger itself
    if (S.lpar && S.lctr[ci(LC_FALLBACK)] == 0) return;     // kme_ledger.hip applied it in parallel
    if (lane_id() == 0) S.ctr[ci(C_LSERIAL)] = 1;
    Core c(S, io);
    const int lane = lane_id();
    for (uint32_t k0 = 0; k0 < io.n && !c.dead; k0 += 64) {
        const uint32_t k = k0 + lane;
        const bool valid = k < io.n;
        const uint32_t bi = valid ? k : 0;
        const int32_t b_action = valid ? io.action[bi] : -1, b_out = valid ? io.out_action[bi] : -1;
        const int32_t b_price = valid ? io.price[bi] : 0, b_size = valid ? io.size[bi] : 0;
        const int64_t b_aid = valid ? io.aid[bi] : 0, b_sid = valid ? io.sid[bi] : 0, b_oid = valid ? io.oid[bi] : 0;
        const uint32_t b_t0 = valid ? io.trade_off[bi] : 0, b_t1 = valid ? io.trade_off[bi + 1] : 0;
        const int4 b_vic = (valid && b_action == CANCEL && b_out == CANCEL) ? S.vic[bi] : make_int4(0, 0, 0, 0);
        const int nb = (int)(io.n - k0 < 64 ? io.n - k0 : 64);
#pragma nounroll
        for (int j = 0; j < nb && !c.dead; ++j) {
            const uint32_t i = k0 + (uint32_t)j;
            const int32_t a = rl32(b_action, j), out = rl32(b_out, j);
            const int64_t aid = rl64(b_aid, j);
            if (a == CREATE_BALANCE) {
                c.create_balance(aid, i);
            } else if (a == TRANSFER) {
                c.transfer(aid, rl32(b_size, j));
            } else if ((a == BUY || a == SELL) && out == a) {
                Taker t;
                t.action = a; t.price = rl32(b_price, j); t.size = rl32(b_size, j); t._pad = 0;
                t.oid = rl64(b_oid, j); t.aid = aid; t.sid = rl64(b_sid, j);
                if (!c.check_balance(t, i)) { if (!c.dead) c.die(KME_E_UNFUNDED, KME_D_NONE, i); break; }
                const bool is_buy = a == BUY;
                for (uint32_t q = (uint32_t)rl32((int32_t)b_t0, j); q < (uint32_t)rl32((int32_t)b_t1, j) && !c.dead; ++q) {
                    const TradeRec tr = io.trades[q];
                    const int64_t maid = U64(tr.maid), msid = U64(tr.msid);
                    const int32_t mprice = U32(tr.mprice), ts = U32(tr.size);
                    c.fill_order(is_buy ? SOLD : BOUGHT, maid, msid, 0, ts, i);                       // maker fill
                    if (!c.dead) c.fill_order(is_buy ? BOUGHT : SOLD, aid, t.sid, jisub(t.price, mprice), ts, i);
                }
            } else if (a == CANCEL && out == CANCEL) {
                Node o;
                const int32_t meta = rl32(b_vic.x, j);
                o.price = meta & 0xFF; o.action = meta >> 8; o.size = rl32(b_vic.y, j);
                o.sid = mk64(rl32(b_vic.z, j), rl32(b_vic.w, j)); o.aid = aid;
                c.post_remove_adjustments(o, i);
            }
        }
    }
}
// ctr_out (the epoch slot's pinned host copy of the counters, through its device mapping; set when
// this is the epoch's last launch): the counters block copied there after the replay -- the
// D2H copy that was a launch of its own after every epoch
__global__ void __launch_bounds__(64) k_ledger_replay(const DevState* __restrict__ Sp, const EpochIO* __restrict__ iop,
                                                      unsigned long long* ctr_out) {
    const DevState& S = *Sp;
    ledger_replay(S, *iop);
    if (!ctr_out) return;
    __syncthreads();   // (one wavefront: its own counter writes before the reads)
    for (int k = threadIdx.x; k < C_NCTR * CTR_STRIDE; k += 64)
        ctr_out[k] = __hip_atomic_load(&S.ctr[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------ (3') OUT echo to input order
// The matching kernels leave each record's OUT echo as one packed 16-B record at its input index
// (one random 16-B store in the matching loop instead of five partial-line stores to the C ABI's SoA
// arrays); here it is read in order and spread over those arrays (sequential lines both ways).
// Records without a symbol group were answered by k_route / k_ledger_funded already.
__global__ void __launch_bounds__(256) k_unsort(DevState S, EpochIO io) {
    if (S.ctr[ci(C_FALLBACK)]) return;                   // k_serial answers the epoch
    const uint32_t lim = err_limit(S.ctr, io.n);          // from a fault on: no trades (trade_off stays in bounds)
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < io.n; i += gridDim.x * blockDim.x) {
        const int32_t g = S.route_grp[i];
        // k_table's work for a BUY/SELL k_match rested (rest_slot; k_match_lanes finalises its own
        // orders' entries at the rest): the oid-table entry becomes the rest slot.  The entry of one
        // that did not rest stays pending (OT_PENDING | i): a reader takes a pending entry only where it
        // names a BUY/SELL of the epoch it reads in with this oid, a fact either way
        // (otab_cancel_target, k_emap).
        const int32_t act = io.action[i];
        if ((act == BUY || act == SELL) && g >= 0 && i < lim) {
            const int32_t rs = S.rest_slot[i];
            if (rs >= 0) {
                const uint32_t h = S.epos[i];
                if (h != OT_DEAD) otab_final(S.otab, (int32_t)h, rs);
            }
        }
        if (g < 0) continue;
        if (i >= lim) { io.n_trades[i] = 0; continue; }
        const int4 a = S.osort[i];
        io.out_action[i] = a.x & 0xFF;
        io.out_flags[i] = (uint8_t)((a.x >> 8) & KME_OUT_HAS_PREV);
        io.out_size[i] = act == CANCEL ? io.size[i] : a.y;   // (removeOrder leaves the size, KP:289-333)
        io.out_prev[i] = mk64(a.z, a.w);
        io.n_trades[i] = (uint32_t)a.x >> 9;
    }
}

// ------------------------------------------------------------------ (4) compaction
// Blocks (s, *) with s < TSHARDS move shard s's trades, blocks (TSHARDS, *) the overflow
// region's, each to trades[trade_off[seq] + ord] (arrival order).
constexpr uint32_t SCATTER_SUB = 8;   // blocks per shard region
constexpr int SCATTER_ITEMS = 4;      // trades per thread and round
__global__ void __launch_bounds__(256) k_scatter(DevState S, EpochIO io, const uint32_t* total) {
    const uint32_t s = blockIdx.x;
    if (S.ctr[ci(C_FALLBACK)]) return;
    const uint32_t lim = err_limit(S.ctr, io.n);          // trades of the records that take effect only
    const bool fits = *total <= io.trades_cap;
    if (s == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
        if (!fits) raise_thread(S.ctr, KME_E_CAPACITY, KME_D_CAP_TRADES, -1);
        else S.ctr[ci(C_TRADES)] = *total;
    }
    if (!fits) return;
    size_t base;
    uint32_t cnt;
    if (s < TSHARDS) {
        const unsigned long long used = S.tsh[(size_t)s * CTR_STRIDE + TS_USED];
        base = (size_t)s * S.tshard_cap;
        cnt = (uint32_t)(used < S.tshard_cap ? used : S.tshard_cap);
    } else {
        base = (size_t)TSHARDS * S.tshard_cap;
        const unsigned long long used = S.ctr[ci(C_TTMP)];
        cnt = (uint32_t)(used < S.ttmp_cap ? used : S.ttmp_cap);
    }
    // SCATTER_ITEMS trades per thread and round, every load of the round before its stores (a load
    // after a store would wait for the store too: vmcnt counts both, in order)
    const uint32_t stride = gridDim.y * blockDim.x;
    for (uint32_t k0 = blockIdx.y * blockDim.x + threadIdx.x; k0 < cnt; k0 += SCATTER_ITEMS * stride) {
        TradeTmp r[SCATTER_ITEMS];
        uint32_t off[SCATTER_ITEMS];
#pragma unroll
        for (int q = 0; q < SCATTER_ITEMS; ++q) {
            const uint32_t k = k0 + q * stride;
            r[q].seq = -1;
            if (k < cnt) r[q] = S.ttmp[base + k];
        }
        uint32_t ord[SCATTER_ITEMS];
#pragma unroll
        for (int q = 0; q < SCATTER_ITEMS; ++q) {
            const bool use = r[q].seq >= 0 && (uint32_t)r[q].seq < lim;
            off[q] = use ? io.trade_off[r[q].seq] : 0;
            // a fast segment's trade: index within its record's event | event rank << 20, the event's
            // base in lvbase (GroupWave::fast_segment)
            const uint32_t o = r[q].ordp & ((1u << TT_ORD_BITS) - 1), rk = o >> FAST_RANK_SHIFT;
            ord[q] = (o & ((1u << FAST_RANK_SHIFT) - 1)) +
                     (use && rk ? S.lvbase[(size_t)r[q].seq * FAST_LVB + rk - 1] : 0u);
        }
#pragma unroll
        for (int q = 0; q < SCATTER_ITEMS; ++q)
            if (r[q].seq >= 0 && (uint32_t)r[q].seq < lim) {
                const uint32_t ordp = r[q].ordp;
                TradeRec t;
                t.moid = r[q].moid; t.maid = r[q].maid;
                t.msid = (ordp >> 30) & 1 ? -(int64_t)r[q].group : (int64_t)r[q].group;
                t.mprice = (int32_t)((ordp >> TT_ORD_BITS) & 0x7F);
                t.size = r[q].size;
                io.trades[off[q] + ord[q]] = t;
            }
    }
}
// The shard lines' rest / cancel counts into the counters block; the lines zeroed for the next epoch.
// (Run by k_settle_funded's first block: after k_scatter read TS_USED and after k_serial, whose
// counters of a fallback epoch it leaves as they are -- the parallel kernels left the lines at 0.)
KDEV void tsh_fold(const DevState& S) {
    __shared__ uint32_t red[4];
    KG unsigned long long* line = S.tsh + (size_t)threadIdx.x * CTR_STRIDE;   // TSHARDS == 256 threads
    const unsigned long long rests = line[TS_RESTS], cancels = line[TS_CANCELS], light = line[TS_LIGHT];
    line[TS_USED] = 0; line[TS_RESTS] = 0; line[TS_CANCELS] = 0; line[TS_LIGHT] = 0;
    const uint32_t r = block_sum_256((uint32_t)rests, red), c = block_sum_256((uint32_t)cancels, red);
    const uint32_t l = block_sum_256((uint32_t)light, red);
    if (threadIdx.x == 0) {
        if (r) atomicAdd(&S.ctr[ci(C_RESTS)], (unsigned long long)r);
        if (c) atomicAdd(&S.ctr[ci(C_CANCEL_OK)], (unsigned long long)c);
        if (l) atomicAdd(&S.ctr[ci(C_LIGHT)], (unsigned long long)l);
    }
}

// ------------------------------------------------------------------ oid-table maintenance
// Each BUY/SELL's pending entry (k_emap) becomes its rest slot, or OT_DEAD if it did not rest: one
// plain store at the recorded position, no probe.  An order that rested and left the book later in
// the epoch keeps a stale slot entry, dropped by validation like every lazily deleted one.
KDEV void table_final(const DevState& S, const EpochIO& io, uint32_t t0, uint32_t stride) {
    for (uint32_t i = t0; i < io.n; i += stride) {
        const int32_t a = io.action[i];
        if (a != BUY && a != SELL) continue;
        const uint32_t h = S.epos[i];
        if (h == OT_DEAD) continue;
        const int32_t s = S.rest_slot[i];
        S.otab[h] = hentry(oid_fp(io.oid[i]), s >= 0 ? (uint32_t)s : OT_DEAD);
    }
}
__global__ void __launch_bounds__(256) k_table(DevState S, EpochIO io) {
    table_final(S, io, blockIdx.x * blockDim.x + threadIdx.x, gridDim.x * blockDim.x);
}
// Rebuild: every live node of the pool's used prefix gets an entry.
__global__ void __launch_bounds__(256) k_otab_refill(DevState S, uint32_t nslots) {
    __shared__ uint32_t red[4];
    uint32_t n_ins = 0;
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < nslots; s += gridDim.x * blockDim.x) {
        if (S.pool[s].live) {
            if (otab_insert(S, S.pool[s].oid, (int32_t)s)) ++n_ins;
            else atomicAdd(&S.ctr[ci(C_REBUILD_FAIL)], 1ull);   // (not the per-epoch error word:
                                                                 // an epoch may be in flight)
        }
    }
    const uint32_t tot = block_sum_256(n_ins, red);
    if (threadIdx.x == 0 && tot) atomicAdd(&S.ctr[ci(C_OTAB_USED)], (unsigned long long)tot);
}

// ------------------------------------------------------------------ market data: top of book
KDEV kme_tob tob_of(const DevState& S, int32_t g) {
    const GroupState gs = S.grp[g];
    kme_tob r{-1, -1, 0, 0};
    if (gs.exists) {
        const Level* L = S.lev + (size_t)g * 2 * NLEV;
        // bids: highest occupied level of book +g; asks: lowest of book -g (sid 0: one book)
        const uint64_t bl = gs.bm0_lsb, bh = gs.bm0_msb;
        const uint64_t al = g == 0 ? gs.bm0_lsb : gs.bm1_lsb, ah = g == 0 ? gs.bm0_msb : gs.bm1_msb;
        const int aside = g == 0 ? 0 : 1;
        if (bl | bh) {
            const int p = bh ? 63 + 63 - __builtin_clzll(bh) : 63 - __builtin_clzll(bl);
            r.bid_px = p;
            const int64_t q = L[p].qty;
            r.bid_qty = (int32_t)(q > INT32_MAX ? INT32_MAX : q);
        }
        if (al | ah) {
            const int p = al ? __builtin_ctzll(al) : 63 + __builtin_ctzll(ah);
            r.ask_px = p;
            const int64_t q = L[aside * NLEV + p].qty;
            r.ask_qty = (int32_t)(q > INT32_MAX ? INT32_MAX : q);
        }
    }
    return r;
}
__global__ void k_tob(DevState S, kme_tob* out) {
    const int32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g < S.G) out[g] = tob_of(S, g);
}
// The snapshot of a list of groups (a shard's own symbols): out[k] = top of book of groups[k].
__global__ void k_tob_groups(DevState S, const uint32_t* groups, uint32_t n, uint32_t rows, kme_tob* out) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= rows) return;
    const uint32_t g = k < n ? groups[k] : 0xFFFFFFFFu;   // rows past n: padding (-1 / 0)
    out[k] = g < (uint32_t)S.G ? tob_of(S, (int32_t)g) : kme_tob{-1, -1, 0, 0};
}

__global__ void k_init_state(DevState S) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < (uint32_t)(S.G + S.Gs)) {   // the dense groups and the sparse ones
        GroupState gs;
        __builtin_memset(&gs, 0, sizeof gs);
        gs.free_head = -1;
        S.grp[k] = gs;
    }
    if (k < (uint32_t)S.Gs) S.gsid[k] = 0;
    if (k < (uint32_t)S.A && S.acct_since) S.acct_since[k] = INT64_MAX;
    if (k == 0) S.ctr[ci(C_ERR)] = ~0ull;   // no epoch yet: nothing faulted (a fresh engine can be checkpointed)
}

// Per-epoch counters: error = none, the epoch's statistics = 0 (pool bump and table usage persist).
// One launch instead of four fills.
__global__ void k_epoch_reset(DevState S) {
    const int k = threadIdx.x;
    if (k == C_ERR) S.ctr[ci(k)] = ~0ull;
    else if ((k >= C_TRADES && k <= C_TTMP) || k == C_ACCT_OPS || k == C_FALLBACK || k == C_BUSY || k == C_LIGHT ||
             k == C_LREPAIRED || k == C_LSERIAL || k == C_GLIST)
        S.ctr[ci(k)] = 0ull;
}

// ------------------------------------------------------------------ host epochs: trades to the host
// kme_submit_epoch_host: the epoch's trades, whose count only the device knows (trade_off[n]), copied
// into the caller's registered host buffer through its device mapping (16-B stores, coalesced, each
// lane one half of a 32-B record), on the copy stream beside the next epoch's kernels.
__global__ void __launch_bounds__(256) k_export_trades(const int4* src, const uint32_t* count, uint32_t cap, int4* dst) {
    const uint32_t n = *count < cap ? *count : cap;
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < 2 * n; k += gridDim.x * blockDim.x) dst[k] = src[k];
}

// ------------------------------------------------------------------ launchers
static inline uint32_t cdiv(uint32_t a, uint32_t b) { return (a + b - 1) / b; }

void launch_epoch_reset(const DevState& S, hipStream_t st) {
    hipLaunchKernelGGL(k_epoch_reset, dim3(1), dim3(C_NCTR), 0, st, S);
}
void launch_emap(const DevState& S, const EpochIO& io, bool funded, EpochIO* io_dev, hipStream_t st) {
    const uint32_t nb = std::min<uint32_t>(cdiv(io.n > 0 ? io.n : 1, 256), STREAM_BLOCKS);
    hipLaunchKernelGGL(k_emap, dim3(nb), dim3(256), 0, st, S, io, funded ? 1 : 0, io_dev);
}
void launch_ledger_funded(const DevState& S, const EpochIO& io, hipStream_t st) {
    hipLaunchKernelGGL(k_ledger_funded, dim3(1), dim3(64), 0, st, S, io);
}
void launch_route(const DevState& S, const EpochIO& io, bool funded, hipStream_t st) {
    // FUNDED: the accounts' check of the funded proof in the blocks past the records
    const uint32_t nb = cdiv(io.n, 256) + (funded && io.n > 0 ? cdiv((uint32_t)S.A, 256) : 0);
    if (nb == 0) return;
    hipLaunchKernelGGL(k_route, dim3(nb), dim3(256), 0, st, S, io, funded ? 1 : 0);
}
void launch_scan(const uint32_t* in, uint32_t* out, uint32_t L, uint32_t* bsum, uint32_t* total, hipStream_t st) {
    const uint32_t nb = cdiv(L > 0 ? L : 1, SCAN_BLOCK);
    hipLaunchKernelGGL(k_scan_blocks, dim3(nb), dim3(256), 0, st, in, out, L, bsum);
    hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(256), 0, st, bsum, nb, total);
    hipLaunchKernelGGL(k_scan_add, dim3(nb), dim3(256), 0, st, out, L, bsum);
}
// Exclusive scan of in[0, L) into out (in place allowed): tile sums, then the tiles (sums scratch:
// cdiv(L, LB_TILE) words).
// A look-back launch's stamp: one per launch, any engine or thread, never 0 (look-back words of older
// launches, and zeroed memory, never match)
uint32_t next_stamp() {
    static std::atomic<uint32_t> stamps{1};
    uint32_t s = stamps.fetch_add(1);
    if (s == 0) s = stamps.fetch_add(1);
    return s;
}
static void launch_scan2(const uint32_t* in, uint32_t* out, uint32_t L, uint32_t* sums, uint32_t* total, int write_end,
                         hipStream_t st, unsigned long long* ctr) {
    const uint32_t nb = cdiv(L > 0 ? L : 1, LB_TILE);
    if (nb <= LB_MAX_TILES && ((uintptr_t)sums & 7) == 0) {   // a small scan: one launch (look-back)
        const uint32_t stamp = next_stamp();
        hipLaunchKernelGGL(k_scan_tiles<true>, dim3(nb), dim3(256), 0, st, in, out, L, (const uint32_t*)sums, total, write_end, stamp,
                           ctr);
        return;
    }
    hipLaunchKernelGGL(k_tile_sums, dim3(nb), dim3(256), 0, st, in, L, sums);
    hipLaunchKernelGGL(k_scan_tiles<false>, dim3(nb), dim3(256), 0, st, in, out, L, (const uint32_t*)sums, total, write_end, 0u,
                       ctr);
}
// Stable LSD radix sort of (key, value) pairs, R.passes digit passes; the result is in keys / vals
// [R.passes & 1].
template <int TILE>
static void radix_passes(const RadixIO& R, hipStream_t st) {
    const uint32_t ntiles = cdiv(R.n > 0 ? R.n : 1, TILE);
    int src = 0;
    if (R.tcnt && R.lb && R.passes <= RADIX_MAXP && TILE == RADIX_TILE_SMALL) {
        // a small sort: the per-tile counts of every pass in one launch, then one launch per pass
        // (look-back offsets) instead of three (histogram, two scan kernels) before each scatter
        hipLaunchKernelGGL(k_radix_tcnt<TILE>, dim3(ntiles), dim3(256), 0, st, R);
        for (int pass = 0; pass < R.passes; ++pass) {
            const uint32_t stamp = next_stamp();
            hipLaunchKernelGGL((k_radix_scatter<TILE, true>), dim3(ntiles), dim3(256), 0, st, R, pass, src, stamp);
            src ^= 1;
        }
        return;
    }
    for (int pass = 0; pass < R.passes; ++pass) {
        hipLaunchKernelGGL(k_radix_hist<TILE>, dim3(ntiles), dim3(256), 0, st, R, pass, src);
        // exclusive scan of the digit-major histogram, in place (scratch at the tail of ghist)
        const uint32_t L = RADIX_DIGITS * ntiles;
        launch_scan2(R.ghist, R.ghist, L, R.ghist + L, nullptr, 0, st, R.ctr);
        hipLaunchKernelGGL(k_radix_scatter<TILE>, dim3(ntiles), dim3(256), 0, st, R, pass, src);
        src ^= 1;
    }
}
void launch_radix(const RadixIO& R, hipStream_t st) {
    if (R.small || R.n <= RADIX_SMALL_N) radix_passes<RADIX_TILE_SMALL>(R, st);
    else radix_passes<RADIX_TILE>(R, st);
}
void launch_excl_scan(const uint32_t* in, uint32_t* out, uint32_t L, uint32_t* sums, uint32_t* total, hipStream_t st,
                      unsigned long long* ctr) {
    launch_scan2(in, out, L, sums, total, 0, st, ctr);
}
int launch_partition(const DevState& S, const EpochIO& io, hipStream_t st, int list_min) {
    RadixIO R{};
    R.key0 = S.route_grp;
    R.val0 = nullptr;
    R.keys0 = S.rkeys[0]; R.keys1 = S.rkeys[1];
    R.vals0 = S.rvals[0]; R.vals1 = S.rvals[1];
    R.ghist = S.ghist;
    R.rank = S.rank;
    R.none = (uint32_t)S.G;
    R.n = io.n;
    R.n_dev = nullptr;
    R.passes = S.passes;
    R.tcnt = S.rtcnt;
    R.lb = S.rlb;
    R.ctr = S.ctr;
    launch_radix(R, st);
    const int src = S.passes & 1;
    const uint32_t nthreads = (io.n + 1) > (uint32_t)S.G + 2 ? io.n + 1 : (uint32_t)S.G + 2;
    hipLaunchKernelGGL(k_segments, dim3(cdiv(nthreads, 256)), dim3(256), 0, st, S, io, src, list_min);
    return src;
}
// the groups k_match takes this epoch (non-empty; busy ones unless `all`), listed in id order
__global__ void __launch_bounds__(256) k_glist_flags(DevState S, int all) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= (uint32_t)S.G) return;
    const uint32_t b = S.seg[g], e = S.seg[g + 1];
    S.gflag[g] = (e > b && (all || e - b > (uint32_t)S.light_max)) ? 1u : 0u;
}
__global__ void __launch_bounds__(256) k_glist_scatter(DevState S, const uint32_t* __restrict__ pos) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= (uint32_t)S.G) return;
    const uint32_t b = S.seg[g], e = S.seg[g + 1];
    if (e > b && pos[g + 1] != pos[g]) S.glist[pos[g]] = g;   // (pos: the exclusive scan of the flags, in place)
}
void launch_match(const DevState& S, const DevState* S_dev, const EpochIO* io_dev, int buf, hipStream_t st, int all, int two,
                  int dense, int five) {
    if (dense) {
        const uint32_t G = (uint32_t)S.G;
        hipLaunchKernelGGL(k_glist_flags, dim3(cdiv(G, 256)), dim3(256), 0, st, S, all);
        // exclusive scan of G + 1 flags (the last one 0: pos[G] = the count), in place
        (void)hipMemsetAsync(S.gflag + G, 0, sizeof(uint32_t), st);
        launch_excl_scan(S.gflag, S.gflag, G + 1, S.gcount + 64, S.gcount, st, S.ctr);
        hipLaunchKernelGGL(k_glist_scatter, dim3(cdiv(G, 256)), dim3(256), 0, st, S, (const uint32_t*)S.gflag);
    }
    if (two) hipLaunchKernelGGL((k_match<true, 4>), dim3((uint32_t)S.G), dim3(128), 0, st, S_dev, io_dev, buf, all, dense);
    else if (five) hipLaunchKernelGGL((k_match<false, 5>), dim3((uint32_t)S.G), dim3(64), 0, st, S_dev, io_dev, buf, all, dense);
    else hipLaunchKernelGGL((k_match<false, 4>), dim3((uint32_t)S.G), dim3(64), 0, st, S_dev, io_dev, buf, all, dense);
}
void launch_match_list(const DevState* S_dev, const EpochIO* io_dev, int buf, hipStream_t st, int all, uint32_t blocks) {
    hipLaunchKernelGGL(k_match_list, dim3(blocks), dim3(64), 0, st, S_dev, io_dev, buf, all);
}
void launch_match_lanes(const DevState& S, const DevState* S_dev, const EpochIO* io_dev, int buf, hipStream_t st) {
    hipLaunchKernelGGL(k_match_lanes, dim3(((uint32_t)S.G + LANE_GROUPS - 1) / LANE_GROUPS), dim3(64), 0, st, S_dev, io_dev, buf);
}
void launch_compact(const DevState& S, const EpochIO& io, hipStream_t st) {
    // one thread per record (no counters to sum): a thread striding over several records would
    // wait for its previous record's stores before its next loads (vmcnt counts both, in order)
    if (io.n > 0) hipLaunchKernelGGL(k_unsort, dim3(cdiv(io.n, 256)), dim3(256), 0, st, S, io);
    // trade_off[0..n] = exclusive scan of n_trades; bsum/total scratch in ghist
    uint32_t* total = S.ghist;   // (the partition's histograms are dead by now)
    launch_scan2(io.n_trades, io.trade_off, io.n, S.ghist + 64, total, 1, st, S.ctr);
    hipLaunchKernelGGL(k_scatter, dim3(TSHARDS + 1, SCATTER_SUB), dim3(256), 0, st, S, io, (const uint32_t*)total);
    // (the shard counters are folded by k_settle_funded's first block)
}
void launch_table(const DevState& S, const EpochIO& io, hipStream_t st) {
    if (io.n == 0) return;
    // FUNDED: k_unsort finalised the entries, and after an epoch k_serial took k_settle_funded does
    if (S.mode == KME_MODE_FUNDED) return;
    hipLaunchKernelGGL(k_table, dim3(cdiv(io.n, 256)), dim3(256), 0, st, S, io);   // one thread per record, as k_unsort
}
void launch_ledger_replay(const DevState* S_dev, const EpochIO* io_dev, hipStream_t st, unsigned long long* ctr_out) {
    hipLaunchKernelGGL(k_ledger_replay, dim3(1), dim3(64), 0, st, S_dev, io_dev, ctr_out);
}
void launch_serial(const DevState* S_dev, const EpochIO* io_dev, hipStream_t st, int only_fallback) {
    hipLaunchKernelGGL(k_serial, dim3(1), dim3(64), 0, st, S_dev, io_dev, only_fallback);
}
void launch_settle_funded(const DevState& S, const EpochIO& io, hipStream_t st) {
    const uint32_t nb = std::max<uint32_t>(1, cdiv((uint32_t)S.A, 256));
    const uint32_t nt = S.fallback && io.n > 0 ? cdiv(io.n, 256) : 0;   // (k_table's work, fallback engines)
    hipLaunchKernelGGL(k_settle_funded, dim3(nb + nt), dim3(256), 0, st, S, io, nb);
}
void launch_otab_rebuild(const DevState& S, uint32_t used_slots, hipStream_t st) {
    (void)hipMemsetAsync(S.otab, 0, sizeof(uint64_t) * ((size_t)S.otab_mask + 1), st);
    (void)hipMemsetAsync(&S.ctr[ci(C_OTAB_USED)], 0, sizeof(unsigned long long), st);
    (void)hipMemsetAsync(&S.ctr[ci(C_REBUILD_FAIL)], 0, sizeof(unsigned long long), st);
    const uint32_t n = std::min(used_slots, S.pool_cap);
    hipLaunchKernelGGL(k_otab_refill, dim3(std::min<uint32_t>(cdiv(n > 0 ? n : 1, 256), STREAM_BLOCKS)), dim3(256), 0, st, S, n);
}
void launch_tob(const DevState& S, void* out, hipStream_t st) {
    hipLaunchKernelGGL(k_tob, dim3(cdiv((uint32_t)S.G, 256)), dim3(256), 0, st, S, (kme_tob*)out);
}
void launch_tob_groups(const DevState& S, const uint32_t* groups, uint32_t n, void* out, hipStream_t st, uint32_t rows) {
    if (rows < n) rows = n;
    if (rows == 0) return;
    hipLaunchKernelGGL(k_tob_groups, dim3(cdiv(rows, 256)), dim3(256), 0, st, S, groups, n, rows, (kme_tob*)out);
}
void launch_credit_state(const DevState& S, int64_t* out, hipStream_t st) {
    if (S.A) hipLaunchKernelGGL(k_credit_state, dim3(cdiv((uint32_t)S.A, 256)), dim3(256), 0, st, S, out);
}
void launch_credit_adjust(const DevState& S, const int64_t* all, uint32_t n, uint32_t me, size_t stride, hipStream_t st) {
    if (S.A) hipLaunchKernelGGL(k_credit_adjust, dim3(cdiv((uint32_t)S.A, 256)), dim3(256), 0, st, S, all, n, me, stride);
}
void launch_export_trades(const TradeRec* src, const uint32_t* count, uint32_t cap, TradeRec* dst_mapped, hipStream_t st) {
    hipLaunchKernelGGL(k_export_trades, dim3(128), dim3(256), 0, st, reinterpret_cast<const int4*>(src), count, cap,
                       reinterpret_cast<int4*>(dst_mapped));
}
void launch_init_state(const DevState& S, hipStream_t st) {
    const uint32_t n = (uint32_t)std::max<int64_t>((int64_t)S.G + S.Gs, S.A);
    hipLaunchKernelGGL(k_init_state, dim3(cdiv(n > 0 ? n : 1, 256)), dim3(256), 0, st, S);
}

}  // namespace kme
