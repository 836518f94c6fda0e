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

#include "kme.h"
#include "kme_device.h"
#include "kme_launch.h"

namespace kme {

#define KDEV __device__ __forceinline__

// ------------------------------------------------------------------ Java arithmetic (wraps)
KDEV int32_t jiadd(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
KDEV int32_t jisub(int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); }
KDEV int32_t jimul(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }
KDEV int32_t jineg(int32_t a) { return (int32_t)(0u - (uint32_t)a); }
KDEV int64_t jladd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
KDEV int64_t jlsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }
KDEV int64_t jlmul(int64_t a, int64_t b) { return (int64_t)((uint64_t)a * (uint64_t)b); }
KDEV int64_t jlneg(int64_t a) { return (int64_t)(0ull - (uint64_t)a); }
KDEV int64_t lmax(int64_t a, int64_t b) { return a >= b ? a : b; }
KDEV int64_t lmin(int64_t a, int64_t b) { return a <= b ? a : b; }
KDEV int32_t imin(int32_t a, int32_t b) { return a <= b ? a : b; }

KDEV int lane_id() { return (int)(threadIdx.x & 63); }

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
// Broadcast lane 0's value with readfirstlane (SGPR result): the compiler then knows it is
// wave-uniform.  (__shfl lowers to ds_bpermute, whose result the divergence analysis treats as
// per-lane; everything computed from it would turn into exec-masked VALU code.)
KDEV unsigned long long bcast64(unsigned long long v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return ((unsigned long long)hi << 32) | lo;
}

KDEV uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

KDEV uint64_t err_code(int status, int detail, int64_t idx) {
    uint64_t ix = idx < 0 ? 0xFFFFFFFFFFFFull : (uint64_t)idx;
    return (ix << 16) | ((uint64_t)(detail & 0xFF) << 8) | (uint64_t)(status & 0xFF);
}
KDEV void raise_thread(unsigned long long* ctr, int status, int detail, int64_t idx) {
    atomicMin(&ctr[C_ERR], (unsigned long long)err_code(status, detail, idx));
}
KDEV void raise_wave(unsigned long long* ctr, int status, int detail, int64_t idx) {
    if (lane_id() == 0) atomicMin(&ctr[C_ERR], (unsigned long long)err_code(status, detail, idx));
}
KDEV bool failed(const unsigned long long* ctr) {
    return __hip_atomic_load(&ctr[C_ERR], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != ~0ull;
}

// ------------------------------------------------------------------ the book bit scans (KP:359-416)
// getFirstSetBitPos / getLastSetBitPos compute (int)(Math.log10(x) / Math.log10(2)) in double.
// Integer restatement: ctz / clz, the NaN path of a negative argument (-> 0), and the overshoot
// of log10 rounding for h >= 47 (h + 1 once n >= 2^(h+1) - D[h]; D[] from
// tools/gen_log10_table.py under a correctly rounded log10).  No floating point on the device.
__constant__ int64_t kLog10D[16] = {1, 2, 3, 7, 14, 28, 90, 178, 340, 663, 1296, 2527, 4799, 9344, 18175, 35328};

KDEV int32_t first_set_bit_pos(uint64_t n) {          // KP:371-373, n != 0
    uint64_t low = n & (0ull - n);
    if (low == (1ull << 63)) return 0;
    return (int32_t)__builtin_ctzll(n);
}
KDEV int32_t last_set_bit_pos(uint64_t n) {           // KP:375-377, n != 0
    if ((int64_t)n < 0) return 0;
    int32_t h = 63 - (int32_t)__builtin_clzll(n);
    if (h >= 47 && n >= (2ull << h) - (uint64_t)kLog10D[h - 47]) h += 1;
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
KDEV int32_t otab_lookup(const DevState& S, int64_t oid) {
    const uint64_t key = (uint64_t)oid ^ OID_SALT;
    uint32_t h = (uint32_t)mix64((uint64_t)oid) & S.otab_mask;
    for (uint32_t probes = 0; probes <= S.otab_mask; ++probes) {
        uint64_t k = S.otab_key[h];
        if (k == 0) return -1;
        if (k == key) {
            int32_t s = S.otab_val[h];
            if (s >= 0 && S.pool[s].live && S.pool[s].oid == oid) return s;   // validate (lazy deletion)
        }
        h = (h + 1) & S.otab_mask;
    }
    return -1;
}
KDEV bool otab_insert(const DevState& S, int64_t oid, int32_t slot) {
    const unsigned long long key = (uint64_t)oid ^ OID_SALT;
    uint32_t h = (uint32_t)mix64((uint64_t)oid) & S.otab_mask;
    for (uint32_t probes = 0; probes <= S.otab_mask; ++probes) {
        unsigned long long prev = atomicCAS((unsigned long long*)&S.otab_key[h], 0ull, key);
        if (prev == 0) {
            S.otab_val[h] = slot;
            return true;
        }
        h = (h + 1) & S.otab_mask;
    }
    return false;
}
KDEV int32_t emap_lookup(const DevState& S, const EpochIO& io, int64_t oid) {
    const uint64_t key = (uint64_t)oid ^ OID_SALT;
    uint32_t h = (uint32_t)mix64((uint64_t)oid) & io.emap_mask;
    for (uint32_t probes = 0; probes <= io.emap_mask; ++probes) {
        uint64_t k = S.emap_key[h];
        if (k == 0) return -1;
        if (k == key) return S.emap_val[h];
        h = (h + 1) & io.emap_mask;
    }
    return -1;
}

// ------------------------------------------------------------------ epoch kernels: emap / ledger / route
// BUY/SELL oid -> input index of this epoch; duplicate / sentinel oid checks; FUNDED: range domain
// and per-account reservation need (max over adj of checkBalance's risk, KP:172-176).
__global__ void k_emap(DevState S, EpochIO io, int funded, EpochIO* io_dev) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) *io_dev = io;   // the group / serial kernels read the epoch descriptor from HBM
    bool is_order = false;
    if (i < io.n) {
        const int32_t a = io.action[i];
        is_order = a == BUY || a == SELL || a == CANCEL;
        if (a == BUY || a == SELL) {
            const int64_t oid = io.oid[i];
            if (oid == INT64_MIN) {
                raise_thread(S.ctr, KME_E_DOMAIN, KME_D_SENTINEL_OID, i);
            } else {
                const unsigned long long key = (uint64_t)oid ^ OID_SALT;
                uint32_t h = (uint32_t)mix64((uint64_t)oid) & io.emap_mask;
                for (uint32_t probes = 0; probes <= io.emap_mask; ++probes) {
                    unsigned long long prev = atomicCAS((unsigned long long*)&S.emap_key[h], 0ull, key);
                    if (prev == 0) { S.emap_val[h] = (int32_t)i; break; }
                    if (prev == key) { raise_thread(S.ctr, KME_E_DOMAIN, KME_D_DUP_OID, i); break; }
                    h = (h + 1) & io.emap_mask;
                }
            }
            if (funded) {
                const int32_t price = io.price[i], size = io.size[i];
                if (price < 0 || price > 100 || size < 0) {
                    raise_thread(S.ctr, KME_E_DOMAIN, KME_D_FUNDED_RANGE, i);
                } else {
                    const int64_t aid = io.aid[i];
                    if (aid >= 0 && aid < S.A) {
                        const int64_t risk = (a == BUY) ? (int64_t)size * price : (int64_t)size * (100 - price);
                        atomicAdd((unsigned long long*)&S.acct_need[aid], (unsigned long long)risk);
                    }
                }
            }
        } else if (funded && (a == CREATE_BALANCE || a == TRANSFER)) {
            atomicAdd(&S.ctr[C_ACCT_OPS], 1ull);
        }
    }
    const unsigned long long nb = __ballot(is_order);
    if (lane_id() == 0 && nb) atomicAdd(&S.ctr[C_ORDERS], (unsigned long long)__popcll(nb));
}

KDEV void write_out(const EpochIO& io, uint32_t i, int32_t action, bool ok, int32_t size, bool has_prev, int64_t prev) {
    io.out_action[i] = ok ? action : (int32_t)REJECT;
    io.out_size[i] = size;
    io.out_prev[i] = has_prev ? prev : 0;
    io.out_flags[i] = has_prev ? (uint8_t)KME_OUT_HAS_PREV : (uint8_t)0;
}

// FUNDED account records in arrival order (one wavefront; skipped when the epoch has none).
// createBalance KP:131-138; transfer KP:140-146 with the balance replaced by the reservation
// bound: a debit is accepted only when it provably passes, otherwise KME_E_UNFUNDED.
__global__ void k_ledger_funded(DevState S, EpochIO io) {
    if (S.ctr[C_ACCT_OPS] == 0 || failed(S.ctr)) return;
    const int lane = lane_id();
    for (uint32_t base = 0; base < io.n; base += 64) {
        const uint32_t i = base + lane;
        const int32_t a = i < io.n ? io.action[i] : -1;
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
                        raise_wave(S.ctr, KME_E_UNFUNDED, KME_D_NONE, j);
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
// i.e. every checkBalance (KP:177) of this epoch passes.  Then roll the bound forward.
__global__ void k_check_funded(DevState S, EpochIO io) {
    const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (a >= S.A) return;
    const int64_t need = S.acct_need[a], negx = S.acct_negx[a], xfer = S.acct_xfer[a];
    if (need == 0 && negx == 0 && xfer == 0) return;
    const int64_t since = S.acct_since[a];
    const int64_t lbs = since < io.seq_base ? S.acct_lb[a] : 0;
    if (need > 0 && lbs - need - negx < 0) raise_thread(S.ctr, KME_E_UNFUNDED, KME_D_NONE, -1);
    if (since < io.seq_base + (int64_t)io.n) S.acct_lb[a] = lbs - need + xfer;
    S.acct_need[a] = 0; S.acct_negx[a] = 0; S.acct_xfer[a] = 0;
}

// Symbol group of each record and the node a CANCEL addresses.  The cancel carries no symbol
// (exchange_test.js:101): removeOrder finds it by oid alone (KP:290).  Target = an order of this
// epoch submitted earlier (encoded -(j+2)), else a resting order from the oid table, else none.
__global__ void k_route(DevState S, EpochIO io, int funded) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= io.n) return;
    const int32_t a = io.action[i];
    int32_t grp = -1;
    int64_t tgt = -1;
    S.rest_slot[i] = -1;
    io.n_trades[i] = 0;
    bool direct = false, ok = false;
    switch (a) {
    case ADD_SYMBOL:
    case REMOVE_SYMBOL:
    case PAYOUT: {
        grp = group_of(io.sid[i], S.G);
        if (grp < 0) {
            if (a == ADD_SYMBOL) raise_thread(S.ctr, KME_E_CAPACITY, KME_D_CAP_SYMBOL, i);
            else if (a == REMOVE_SYMBOL) { direct = true; ok = true; }      // removeSymbol of an absent symbol
            else if (funded) raise_thread(S.ctr, KME_E_UNSUPPORTED, KME_D_NONE, i);
        }
        break;
    }
    case BUY:
    case SELL: {
        grp = group_of(io.sid[i], S.G);
        if (grp < 0) { direct = true; ok = false; }                         // books.get == null (KP:202-203)
        if (otab_lookup(S, io.oid[i]) >= 0) raise_thread(S.ctr, KME_E_DOMAIN, KME_D_DUP_OID, i);
        if (funded && grp >= 0) {
            const int64_t aid = io.aid[i];
            S.acct_ok[i] = (aid >= 0 && aid < S.A && S.acct_since[aid] < io.seq_base + (int64_t)i) ? 1 : 0;
        }
        break;
    }
    case CANCEL: {
        const int64_t oid = io.oid[i];
        const int32_t j = emap_lookup(S, io, oid);
        if (j >= 0 && (uint32_t)j < i) {
            const int32_t gj = group_of(io.sid[j], S.G);
            if (gj >= 0) { grp = gj; tgt = -((int64_t)j + 2); }
        } else {
            const int32_t s = otab_lookup(S, oid);
            if (s >= 0) { grp = S.pool[s].group; tgt = s; }
        }
        if (grp < 0) { direct = true; ok = false; }                         // orders.get == null (KP:290-291)
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
    S.cancel_tgt[i] = tgt;
    if (funded && direct) write_out(io, i, a, ok, io.size[i], false, 0);
}

// ------------------------------------------------------------------ (1) stable radix partition
// LSD radix sort of (group, input index) pairs, 8-bit digits.  Records without a group sort into
// bucket G, which nobody processes.  Stability = arrival order inside each group.
__global__ void __launch_bounds__(256) k_radix_hist(DevState S, EpochIO io, int pass, int src) {
    __shared__ uint32_t h[256];
    const int t = threadIdx.x;
    h[t] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * RADIX_TILE;
    for (int j = 0; j < RADIX_TILE / 256; ++j) {
        const uint32_t k = base + j * 256 + t;
        if (k < io.n) {
            uint32_t key;
            if (pass == 0) { int32_t g = S.route_grp[k]; key = g < 0 ? (uint32_t)S.G : (uint32_t)g; }
            else key = (src ? S.rkeys[1] : S.rkeys[0])[k];
            atomicAdd(&h[(key >> (8 * pass)) & 255], 1u);
        }
    }
    __syncthreads();
    S.ghist[t * gridDim.x + blockIdx.x] = h[t];
}

__global__ void __launch_bounds__(256) k_radix_scatter(DevState S, EpochIO io, int pass, int src) {
    __shared__ uint32_t running[256];
    __shared__ uint32_t wcnt[4][256];
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    running[t] = S.ghist[t * gridDim.x + blockIdx.x];
    const uint32_t base = blockIdx.x * RADIX_TILE;
    const int dst = src ^ 1;
    const unsigned long long lt_mask = (1ull << lane) - 1ull;
    for (int j = 0; j < RADIX_TILE / 256; ++j) {
        wcnt[0][t] = 0; wcnt[1][t] = 0; wcnt[2][t] = 0; wcnt[3][t] = 0;
        __syncthreads();
        const uint32_t k = base + j * 256 + t;
        const bool valid = k < io.n;
        uint32_t key = 0, val = 0;
        if (valid) {
            if (pass == 0) { int32_t g = S.route_grp[k]; key = g < 0 ? (uint32_t)S.G : (uint32_t)g; val = k; }
            else { key = (src ? S.rkeys[1] : S.rkeys[0])[k]; val = (src ? S.rvals[1] : S.rvals[0])[k]; }
        }
        const uint32_t d = (key >> (8 * pass)) & 255;
        unsigned long long peers = __ballot(valid);
        for (int b = 0; b < 8; ++b) {
            const unsigned long long bb = __ballot(valid && ((d >> b) & 1));
            peers &= ((d >> b) & 1) ? bb : ~bb;
        }
        const uint32_t rank = (uint32_t)__popcll(peers & lt_mask);
        if (valid && rank == 0) wcnt[w][d] = (uint32_t)__popcll(peers);
        __syncthreads();
        if (valid) {
            uint32_t pos = running[d] + rank;
            for (int ww = 0; ww < w; ++ww) pos += wcnt[ww][d];
            (dst ? S.rkeys[1] : S.rkeys[0])[pos] = key;
            (dst ? S.rvals[1] : S.rvals[0])[pos] = val;
        }
        __syncthreads();
        running[t] += wcnt[0][t] + wcnt[1][t] + wcnt[2][t] + wcnt[3][t];
        __syncthreads();
    }
}

// Group segment offsets from the sorted keys: seg[g] = first position with key >= g.
__global__ void k_segments(DevState S, EpochIO io, int buf) {
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

// ------------------------------------------------------------------ (2) the matching core
// One input record as the group / serial wavefront consumes it (wave-uniform, SGPR-resident).
struct Rec {
    uint32_t i;
    int32_t action, price, size, acct_ok;
    int64_t oid, aid, sid, tgt;
};
// 64 records staged across the lanes of a wavefront: lane l holds record k0 + l.  One gather per
// 64 records replaces two dependent global round trips per record (perm[k], then the fields).
struct Batch {
    uint32_t i;
    int32_t action, price, size, acct_ok;
    int64_t oid, aid, sid, tgt;
};
// s_waitcnt vmcnt(0) expcnt(7) lgkmcnt(15): gfx9 encoding (vmcnt bits 3:0 and 15:14)
constexpr int VMCNT0 = 0x0F70;
KDEV int32_t rl32(int32_t v, int j) { return __builtin_amdgcn_readlane(v, j); }
// lane j of v := x (v_cmp + v_cndmask; x and j are wave-uniform)
KDEV int32_t lane_put(int32_t x, int j, int32_t v) { return lane_id() == j ? x : v; }
KDEV int64_t rl64(int64_t v, int j) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, j);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), j);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
KDEV Batch load_batch(const DevState& S, const EpochIO& io, bool valid, uint32_t i, bool funded) {
    Batch B;
    B.i = i;
    if (valid) {
        B.action = io.action[i]; B.price = io.price[i]; B.size = io.size[i];
        B.oid = io.oid[i]; B.aid = io.aid[i]; B.sid = io.sid[i];
        B.tgt = S.cancel_tgt[i];
        B.acct_ok = funded ? (int32_t)S.acct_ok[i] : 0;
    } else {
        B.action = -1; B.price = B.size = B.acct_ok = 0; B.oid = B.aid = B.sid = B.tgt = 0;
    }
    return B;
}
KDEV Rec pick(const Batch& B, int j) {
    Rec r;
    r.i = (uint32_t)rl32((int32_t)B.i, j);
    r.action = rl32(B.action, j); r.price = rl32(B.price, j); r.size = rl32(B.size, j);
    r.acct_ok = rl32(B.acct_ok, j);
    r.oid = rl64(B.oid, j); r.aid = rl64(B.aid, j); r.sid = rl64(B.sid, j); r.tgt = rl64(B.tgt, j);
    return r;
}

struct Taker {
    int32_t action, price, size, _pad;
    int64_t oid, aid, sid;
};

// What process() decided for one record (the OUT echo fields and its trade count).
struct Out {
    int32_t action, size;
    int64_t prev;
    bool has_prev;
    bool rested;          // the order came to rest (counted per batch, not per record)
    uint32_t ntr;
};

constexpr int FSTACK = 256;       // LDS free-slot stack of a group wavefront
constexpr int DIRTY_WORDS = 64;   // 2048-bit per-batch filter of node slots written in the batch

// Book state of the current symbol group, held in registers (bitmaps, free list) and, for the
// parallel kernel, price levels staged in LDS on first touch and written back at the end.
template <bool EXACT, bool LDS>
struct Core {
    const DevState& S;
    const EpochIO& io;
    Level* cache;                     // LDS [2][NLEV] (LDS == true)
    int32_t g;
    int32_t exists;
    uint64_t b0l, b0m, b1l, b1m;      // bitmaps of book +g (side 0) and book -g (side 1)
    int32_t* fstack;                  // LDS free-slot stack (LDS == true)
    int32_t fsp;
    uint32_t* dirty;                  // LDS per-batch written-slot filter (LDS == true)
    Node* nodepf;                     // LDS cancel-target nodes prefetched with the batch (LDS == true)
    int32_t free_head, chunk_next, chunk_end;
    Level* glev;
    uint32_t tnext, tend;             // FUNDED: trade scratch chunk; EXACT: running trade count
    bool dead;
#ifdef KME_STAMPS
    unsigned long long acc[16];
#endif

    KDEV Core(const DevState& s, const EpochIO& e, Level* c, int32_t* fs, uint32_t* dty, Node* npf)
        : S(s), io(e), cache(c), fstack(fs), dirty(dty), nodepf(npf) {
        g = -1; exists = 0; b0l = b0m = b1l = b1m = 0; fsp = 0;
        free_head = -1; chunk_next = chunk_end = 0; glev = nullptr;
        tnext = tend = 0; dead = false;
        KST(for (int q = 0; q < 16; ++q) acc[q] = 0;)
    }

    KDEV void die(int status, int detail, int64_t idx) { raise_wave(S.ctr, status, detail, idx); dead = true; }

    KDEV void load_group(int32_t gg) {
        g = gg;
        const GroupState& G = S.grp[gg];
        exists = G.exists;
        b0l = G.bm0_lsb; b0m = G.bm0_msb; b1l = G.bm1_lsb; b1m = G.bm1_msb;
        free_head = G.free_head; chunk_next = G.chunk_next; chunk_end = G.chunk_end;
        glev = S.lev + (size_t)gg * 2 * NLEV;
        fsp = 0;
        if (LDS) stage_levels(true);
    }
    // Occupied levels of both books move between HBM and LDS in one parallel pass (lane l takes
    // prices l and l + 64); an unoccupied level's fields are dead until a rest rewrites them all.
    KDEV void stage_levels(bool in) {
        const int lane = lane_id();
#pragma unroll
        for (int side = 0; side < 2; ++side) {
            const uint64_t l = side ? b1l : b0l, m = side ? b1m : b0m;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int p = lane + 64 * h;
                if (p <= 126 && check_bit(l, m, p)) {
                    int4* c = reinterpret_cast<int4*>(&cache[side * NLEV + p]);
                    int4* gl = reinterpret_cast<int4*>(&glev[side * NLEV + p]);
                    if (in) { const int4 x0 = gl[0], x1 = gl[1]; c[0] = x0; c[1] = x1; }
                    else { const int4 x0 = c[0], x1 = c[1]; gl[0] = x0; gl[1] = x1; }
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    KDEV void store_group() {
        if (g < 0) return;
        if (LDS) {
            stage_levels(false);
            flush_free_stack();
        }
        {
            GroupState& G = S.grp[g];
            G.exists = exists;
            G.bm0_lsb = b0l; G.bm0_msb = b0m; G.bm1_lsb = b1l; G.bm1_msb = b1m;
            G.free_head = free_head; G.chunk_next = chunk_next; G.chunk_end = chunk_end;
        }
    }
    KDEV uint64_t bl(int side) const { return side ? b1l : b0l; }
    KDEV uint64_t bm(int side) const { return side ? b1m : b0m; }
    KDEV void set_bm(int side, uint64_t l, uint64_t m) { if (side) { b1l = l; b1m = m; } else { b0l = l; b0m = m; } }

    KDEV Level* lv(int side, int32_t p) {
        return LDS ? &cache[side * NLEV + p] : &glev[side * NLEV + p];
    }

    KDEV Node ld_node(int32_t s) const {
        const Node* p = &S.pool[s];
        Node n;
        n.oid = p->oid; n.aid = p->aid; n.sid = p->sid; n.prev_oid = p->prev_oid;
        n.size = p->size; n.next = p->next; n.prev = p->prev; n.group = p->group;
        n.price = p->price; n.action = p->action; n.live = p->live; n._pad = 0;
        return n;
    }

    // Node slots.  Parallel kernel (LDS): an LDS stack of free slots; the group's free slots kept
    // between epochs are a list of BLOCKS, each a free 64-byte slot holding up to FBLK - 1 more
    // free slot ids (word 0 = next block, word 1 = count, words 2.. = ids; word 14 = Node::live
    // stays 0).  One load refills the stack with a whole block.  Serial kernel: a plain list
    // linked through Node::next.  Last resort: a chunk from the pool's bump counter.
    static constexpr int FBLK = 13;
    KDEV int32_t alloc_slot(int64_t idx) {
        if (LDS) {
            if (fsp > 0) return fstack[--fsp];
            if (free_head >= 0) {
                const int32_t blk = free_head;
                const int lane = lane_id();
                const int32_t w = lane < 2 + FBLK - 1 ? reinterpret_cast<const int32_t*>(&S.pool[blk])[lane] : 0;
                const int32_t nxt = __builtin_amdgcn_readlane(w, 0);
                const int32_t cnt = __builtin_amdgcn_readlane(w, 1);
                if (lane >= 2 && lane < 2 + cnt) fstack[lane - 2] = w;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                fsp = cnt;
                free_head = nxt;
                return blk;
            }
        } else if (free_head >= 0) {
            const int32_t s = free_head;
            free_head = S.pool[s].next;
            return s;
        }
        if (chunk_next >= chunk_end) {
            unsigned long long c = 0;
            if (lane_id() == 0) c = atomicAdd(&S.ctr[C_POOL_BUMP], (unsigned long long)POOL_CHUNK);
            c = bcast64(c);
            if (c + POOL_CHUNK > S.pool_cap) { die(KME_E_CAPACITY, KME_D_CAP_POOL, idx); return -1; }
            chunk_next = (int32_t)c;
            chunk_end = (int32_t)(c + POOL_CHUNK);
        }
        return chunk_next++;
    }
    KDEV void free_slot(int32_t s) {
        S.pool[s].live = 0;
        mark_dirty(s);
        if (LDS) {
            if (fsp == FSTACK) spill_blocks(FSTACK - FBLK, FSTACK);
            fstack[fsp++] = s;
            return;
        }
        S.pool[s].next = free_head;
        free_head = s;
    }
    // Writes stack entries [b, e) as blocks of FBLK slots (the last slot of each block holds the
    // others' ids), chained onto the group's block list; all lanes in parallel, stores only.
    KDEV void spill_blocks(int b, int e) {
        const int n = e - b;
        const int nblk = (n + FBLK - 1) / FBLK;
        for (int k = lane_id(); k < nblk * 14; k += 64) {
            const int blk = k / 14, word = k - blk * 14;
            const int base = b + blk * FBLK;
            const int cnt = imin(FBLK, e - base);                // slots in this block incl. itself
            const int32_t host = fstack[base + cnt - 1];
            int32_t v;
            if (word == 0) v = blk == 0 ? free_head : fstack[base - 1];   // previous block's host
            else if (word == 1) v = cnt - 1;
            else v = word - 2 < cnt - 1 ? fstack[base + word - 2] : -1;
            reinterpret_cast<int32_t*>(&S.pool[host])[word] = v;
        }
        free_head = fstack[b + (nblk - 1) * FBLK + imin(FBLK, e - (b + (nblk - 1) * FBLK)) - 1];
        fsp = b;
    }
    // The LDS stack joins the group's block list when the group is written back.
    KDEV void flush_free_stack() {
        if (!LDS || fsp == 0) return;
        spill_blocks(0, fsp);
    }
    // Per-batch filter of node slots written since the batch's cancel-target prefetch.
    KDEV void mark_dirty(int32_t s) {
        if (!LDS) return;
        if (lane_id() == 0)
            __hip_atomic_fetch_or(&dirty[(s >> 5) & (DIRTY_WORDS - 1)], 1u << (s & 31), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    KDEV bool is_dirty(int32_t s) const {
        return (dirty[(s >> 5) & (DIRTY_WORDS - 1)] >> (s & 31)) & 1u;
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
        const unsigned long long used = S.ctr[C_BAL_USED] + 1;
        S.ctr[C_BAL_USED] = used;
        if (used * 2 > (unsigned long long)S.bal_mask + 1) die(KME_E_CAPACITY, KME_D_CAP_LEDGER, idx);
    }
    KDEV int32_t pos_find(int64_t k0, int64_t k1, int32_t* free_slot_out) const {
        uint32_t h = (uint32_t)mix64((uint64_t)k0 * 0x9e3779b97f4a7c15ull ^ mix64((uint64_t)k1)) & S.pos_mask;
        int32_t first_free = -1;
        for (uint32_t p = 0; p <= S.pos_mask; ++p) {
            const uint32_t st = S.pos_state[h];
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
            if (S.pos_state[h] == 0) {
                const unsigned long long used = S.ctr[C_POS_USED] + 1;
                S.ctr[C_POS_USED] = used;
                if (used * 4 > ((unsigned long long)S.pos_mask + 1) * 3) { die(KME_E_CAPACITY, KME_D_CAP_LEDGER, idx); return; }
            }
            S.pos[h].k0 = k0; S.pos[h].k1 = k1; S.pos_state[h] = 1;
        }
        S.pos[h].v0 = v0; S.pos[h].v1 = v1;
    }
    KDEV void pos_del(int64_t k0, int64_t k1) {
        const int32_t h = pos_find(k0, k1, nullptr);
        if (h >= 0) S.pos_state[h] = 2;
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
            if (S.pos_state[h] == 1 && S.pos[h].k1 == sid && bal_find(S.pos[h].k0) < 0) bad = true;
        if (__ballot(bad)) { die(KME_E_DOMAIN, KME_D_NPE_BALANCE, idx); return; }
        for (uint32_t h = lane; h <= S.pos_mask; h += 64) {
            if (S.pos_state[h] == 1 && S.pos[h].k1 == sid) {
                const int32_t b = bal_find(S.pos[h].k0);
                atomicAdd((unsigned long long*)&S.bal_val[b], (unsigned long long)jlmul(S.pos[h].v0, (int64_t)size));
            }
        }
        __threadfence();   // the atomics ran at L2: drop this CU's L1 copies before re-reading
        __builtin_amdgcn_wave_barrier();
        for (uint32_t h = lane; h <= S.pos_mask; h += 64)
            if (S.pos_state[h] == 1 && S.pos[h].k1 == sid) S.pos_state[h] = 2;
        __threadfence();   // other lanes' tombstones become visible to every lane
        __builtin_amdgcn_wave_barrier();
    }

    // ---------------- trades
    KDEV void emit(uint32_t i, uint32_t ord, const Node& m, int32_t ts) {
        if (EXACT) {
            if (tnext >= io.trades_cap) { die(KME_E_CAPACITY, KME_D_CAP_TRADES, i); return; }
            if (lane_id() == 0) {
                TradeRec& r = io.trades[tnext];
                r.moid = m.oid; r.maid = m.aid; r.msid = m.sid; r.mprice = m.price; r.size = ts;
            }
            tnext++;
        } else {
            if (tnext >= tend) {
                unsigned long long c = 0;
                if (lane_id() == 0) c = atomicAdd(&S.ctr[C_TTMP], (unsigned long long)TRADE_CHUNK);
                c = bcast64(c);
                if (c + TRADE_CHUNK > S.ttmp_cap) { die(KME_E_CAPACITY, KME_D_CAP_TRADES, i); return; }
                tnext = (uint32_t)c;
                tend = (uint32_t)(c + TRADE_CHUNK);
            }
            if (lane_id() == 0) {
                TradeTmp& r = S.ttmp[tnext];
                r.t.moid = m.oid; r.t.maid = m.aid; r.t.msid = m.sid; r.t.mprice = m.price; r.t.size = ts;
                r.seq = (int32_t)i; r.ord = (int32_t)ord;
            }
            tnext++;
        }
    }
    KDEV void close_trade_chunk() {
        if (EXACT) return;
        for (uint32_t k = tnext + lane_id(); k < tend; k += 64) S.ttmp[k].seq = -1;
        tnext = tend;
    }

    // ---------------- tryMatch, KP:225-263
    // The level being swept lives in registers (head, count, qty) and is written back once when
    // the sweep stops inside it; a level swept empty is not written at all (its bit is cleared and
    // an unoccupied level's fields are dead until a rest rewrites them).  A maker's price is the
    // index of its level, so the loop test of KP:237 -- ((size > 0 && isBuy) ? maker.price <= P :
    // maker.price >= P), H3 -- needs no node load, and the next maker's node is requested before
    // the stores of the current trade (vmcnt is in order: a load issued after stores waits for
    // them).
    KDEV bool crosses(bool is_buy, int32_t size, int32_t mprice, int32_t P) const {
        return (size > 0 && is_buy) ? mprice <= P : mprice >= P;
    }
    // executeTrade (KP:265-274): the trade record, and in EXACT mode both fillOrder calls.
    KDEV void trade(uint32_t i, uint32_t& ntr, const Node& m, const Taker& t, int32_t ts, bool is_buy) {
        emit(i, ntr++, m, ts);
        if (EXACT && !dead) {
            fill_order(is_buy ? SOLD : BOUGHT, m.aid, m.sid, 0, ts, i);                              // maker fill
            if (!dead) fill_order(is_buy ? BOUGHT : SOLD, t.aid, t.sid, jisub(t.price, m.price), ts, i);  // taker fill
        }
    }
    KDEV bool try_match(uint32_t i, Taker& t, uint32_t& ntr) {
        KST(unsigned long long tq = stamp();)
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
        int32_t ms = L->head, lcnt = L->count;
        int64_t lqty = L->qty;
        if (ms < 0) { die(KME_E_DOMAIN, KME_D_NPE_ORDER, i); return false; }
        Node m = ld_node(ms);
        bool head_moved = false;                             // ms is a later maker of level L
        KST(acc[10] += stamp() - tq;)
        for (;;) {
            KST(tq = stamp(); acc[14] += 1;)
            const int32_t ts = imin(t.size, m.size);
            const int32_t msize = jisub(m.size, ts);
            t.size = jisub(t.size, ts);
            lqty -= ts;
            if (msize != 0) {                                // maker stays, partially filled (KP:255-261)
                trade(i, ntr, m, t, ts, is_buy);
                if (dead) return false;
                S.pool[ms].size = msize;
                if (head_moved) { L->head = ms; S.pool[ms].prev = -1; }
                mark_dirty(ms);
                L->count = lcnt; L->qty = lqty;
                KST(acc[13] += stamp() - tq;)
                return t.size == 0;
            }
            lcnt -= 1;                                       // maker consumed: orders.delete (KP:243)
            int32_t nms;
            bool same_level = m.next >= 0;
            if (same_level) {
                nms = m.next;
                if (!crosses(is_buy, t.size, m.price, P)) {  // stops before the next maker of L
                    trade(i, ntr, m, t, ts, is_buy);
                    if (dead) return false;
                    free_slot(ms);
                    L->head = nms; S.pool[nms].prev = -1; mark_dirty(nms);
                    L->count = lcnt; L->qty = lqty;
                    KST(acc[13] += stamp() - tq;)
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
                    KST(acc[13] += stamp() - tq;)
                    return t.size == 0;
                }
                L = lv(os, pb);
                nms = L->head; lcnt = L->count; lqty = L->qty;
                if (nms < 0) { die(KME_E_DOMAIN, KME_D_NPE_ORDER, i); return false; }
            }
            const Node nm = ld_node(nms);                   // in flight during this trade's stores
            trade(i, ntr, m, t, ts, is_buy);
            if (dead) return false;
            free_slot(ms);
            head_moved = same_level;
            m = nm;
            ms = nms;
            KST(acc[12] += stamp() - tq;)
        }
    }

    // ---------------- addOrder, KP:200-223 (after the book-exists and balance checks)
    KDEV void rest(uint32_t i, const Taker& t, bool& has_prev, int64_t& prev_oid) {
        const int64_t key = jlmul(t.sid, t.action == BUY ? 1 : -1);
        const int s = key < 0 ? 1 : 0;
        uint64_t lo = bl(s), hi = bm(s);                     // books.get(sid) again (KP:205)
        const int32_t p = t.price;
        if (p < 0 || p > 126) { die(KME_E_DOMAIN, KME_D_PRICE, i); return; }
        KST(const unsigned long long ta = stamp();)
        const int32_t slot = alloc_slot(i);
        KST(acc[15] += stamp() - ta;)
        if (dead) return;
        Level* L = lv(s, p);
        int32_t nprev = -1;
        has_prev = false;
        prev_oid = 0;
        if (!check_bit(lo, hi, p)) {                        // new bucket (oid, oid), set bit (KP:209-211)
            L->head = slot; L->tail = slot; L->count = 1; L->qty = t.size; L->tail_oid = t.oid;
            set_bit(lo, hi, p);
            set_bm(s, lo, hi);
        } else {                                             // append at the tail (KP:213-219)
            const int32_t tl = L->tail;
            S.pool[tl].next = slot;
            mark_dirty(tl);
            has_prev = true;
            prev_oid = L->tail_oid;
            nprev = tl;
            L->tail = slot; L->tail_oid = t.oid; L->count += 1; L->qty += t.size;
        }
        Node* nd = &S.pool[slot];
        nd->oid = t.oid; nd->aid = t.aid; nd->sid = t.sid; nd->prev_oid = prev_oid;
        nd->size = t.size; nd->next = -1; nd->prev = nprev; nd->group = g;
        nd->price = p; nd->action = t.action; nd->live = 1; nd->_pad = 0;
        mark_dirty(slot);
        S.rest_slot[i] = slot;
    }

    // ---------------- removeOrder, KP:289-323
    KDEV bool remove_order(const Rec& r, int j) {
        const uint32_t i = r.i;
        const int64_t tgt = r.tgt;
        int32_t slot = -1;
        if (tgt >= 0) slot = (int32_t)tgt;
        else if (tgt <= -2) slot = S.rest_slot[-(tgt + 2)];
        if (slot < 0) return false;
        // the batch prefetched pre-epoch targets into LDS; valid unless written since
        const Node o = (LDS && j >= 0 && tgt >= 0 && !is_dirty(slot)) ? nodepf[j] : ld_node(slot);
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
            mark_dirty(o.next);
        } else if (o.next < 0) {
            L->tail = o.prev;
            L->tail_oid = o.prev_oid;
            S.pool[o.prev].next = -1;
            mark_dirty(o.prev);
        } else {
            S.pool[o.prev].next = o.next;
            S.pool[o.next].prev = o.prev;
            S.pool[o.next].prev_oid = o.prev_oid;
            mark_dirty(o.prev);
            mark_dirty(o.next);
        }
        L->count -= 1;
        L->qty -= o.size;
        free_slot(slot);
        if (EXACT) post_remove_adjustments(o, i);
        return !dead;
    }

    // removeSymbol (KP:193-198) for an existing group: 0 = returns false (empty book), 2 = never
    // returns (removeAllOrders loops, KP:341-353).  Absent symbols return true.
    KDEV int remove_symbol_existing(int64_t sid) const {
        const int s = sid < 0 ? 1 : 0;
        return (bl(s) == 0 && bm(s) == 0) ? 0 : 2;
    }

    // ---------------- one record of this group (MatchingEngine.process, KP:96-126)
    KDEV Out process(const Rec& r, int j) {
        const uint32_t i = r.i;
        const int32_t a = r.action;
        bool ok = false, has_prev = false;
        int64_t prev_oid = 0;
        int32_t out_size = r.size;
        uint32_t ntr = 0;
        Out out;
        out.action = a; out.size = r.size; out.prev = 0; out.has_prev = false; out.rested = false; out.ntr = 0;
        if (EXACT) io.trade_off[i] = tnext;
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
                    if (EXACT) payout_settle(r.sid, r.size, i);
                    else die(KME_E_UNSUPPORTED, KME_D_NONE, i);
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
            if (EXACT) {
                if (!check_balance(t, i)) { if (dead) return out; break; }
            } else {
                if (!r.acct_ok) break;                      // balances.get(aid) == null
            }
            KST(const unsigned long long t0 = stamp();)
            const bool filled = try_match(i, t, ntr);
            KST(const unsigned long long t1 = stamp(); acc[4] += t1 - t0;)
            if (dead) return out;
            if (!filled) { rest(i, t, has_prev, prev_oid); if (dead) return out; out.rested = true; }
            KST(acc[5] += stamp() - t1;)
            ok = true;
            out_size = t.size;
            break;
        }
        case CANCEL:
            ok = remove_order(r, j);
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

// (2) FUNDED: one wavefront per symbol group, the group's records in arrival order.
__global__ void __launch_bounds__(64) k_match(const DevState* __restrict__ Sp, const EpochIO* __restrict__ iop, int buf) {
    __shared__ Level cache[2 * NLEV];
    __shared__ int32_t fstack[FSTACK];
    __shared__ uint32_t dirty[DIRTY_WORDS];
    __shared__ Node nodepf[64];
    const DevState& S = *Sp;
    const EpochIO& io = *iop;
    const int32_t g = blockIdx.x;
    if (g >= S.G) return;
    const uint32_t b = S.seg[g], e = S.seg[g + 1];
    if (b >= e) return;
    if (failed(S.ctr)) return;
    Core<false, true> c(S, io, cache, fstack, dirty, nodepf);
    c.load_group(g);
    const uint32_t* perm = buf ? S.rvals[1] : S.rvals[0];
    const int lane = lane_id();
    uint32_t n_rest = 0, n_cancel = 0;
    KST(const unsigned long long tk0 = stamp();)
    for (uint32_t k0 = b; k0 < e && !c.dead; k0 += 64) {
        KST(const unsigned long long tb0 = stamp();)
        const uint32_t k = k0 + lane;
        const bool valid = k < e;
        const Batch B = load_batch(S, io, valid, valid ? perm[k] : 0, true);
        // cancels of orders resting since an earlier epoch: fetch the target node with the batch
        dirty[lane] = 0;
        if (valid && B.action == CANCEL && B.tgt >= 0) {
            const int4* src = reinterpret_cast<const int4*>(&S.pool[B.tgt]);
            int4* dst = reinterpret_cast<int4*>(&nodepf[lane]);
            const int4 x0 = src[0], x1 = src[1], x2 = src[2], x3 = src[3];
            dst[0] = x0; dst[1] = x1; dst[2] = x2; dst[3] = x3;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        // The batch registers are read with readlane inside the record loop.  Waiting for them here
        // once keeps the waitcnt pass from placing a vmcnt(0) at the loop header, which would make
        // every record wait for all stores of the record before it (stores share vmcnt on gfx9).
        __builtin_amdgcn_s_waitcnt(VMCNT0);
        const int nb = (int)(e - k0 < 64 ? e - k0 : 64);
        // per-record OUT fields collect in lane j of these registers; one store per field per batch
        int32_t o_act = 0, o_size = 0, o_plo = 0, o_phi = 0, o_flag = 0, o_ntr = 0;
        KST(c.acc[0] += stamp() - tb0;)
#pragma nounroll
        for (int j = 0; j < nb && !c.dead; ++j) {
            KST(const unsigned long long tr0 = stamp();)
            const Rec rr = pick(B, j);
            const Out o = c.process(rr, j);
            KST(const unsigned long long tr1 = stamp();
                const int cat = (rr.action == BUY || rr.action == SELL) ? 1 : (rr.action == CANCEL ? 2 : 3);
                if (cat == 1) { c.acc[1] += tr1 - tr0; c.acc[8] += 1; }
                else if (cat == 2) { c.acc[2] += tr1 - tr0; c.acc[9] += 1; }
                else c.acc[3] += tr1 - tr0;)
            o_act = lane_put(o.action, j, o_act);
            o_size = lane_put(o.size, j, o_size);
            o_plo = lane_put((int32_t)(uint32_t)o.prev, j, o_plo);
            o_phi = lane_put((int32_t)(uint32_t)((uint64_t)o.prev >> 32), j, o_phi);
            o_flag = lane_put((o.has_prev ? (int32_t)KME_OUT_HAS_PREV : 0) | (o.rested ? 2 : 0), j, o_flag);
            o_ntr = lane_put((int32_t)o.ntr, j, o_ntr);
            KST(c.acc[6] += stamp() - tr1;)
        }
        n_rest += (uint32_t)__popcll(__ballot(lane < nb && (o_flag & 2)));
        n_cancel += (uint32_t)__popcll(__ballot(lane < nb && B.action == CANCEL && o_act == CANCEL));
        if (lane < nb && !c.dead) {
            const uint32_t i = B.i;
            io.out_action[i] = o_act;
            io.out_size[i] = o_size;
            io.out_prev[i] = (int64_t)(((uint64_t)(uint32_t)o_phi << 32) | (uint32_t)o_plo);
            io.out_flags[i] = (uint8_t)(o_flag & KME_OUT_HAS_PREV);
            io.n_trades[i] = (uint32_t)o_ntr;
        }
    }
    c.close_trade_chunk();
    c.store_group();
    if (lane == 0) {
        if (n_rest) atomicAdd(&S.ctr[C_RESTS], (unsigned long long)n_rest);
        if (n_cancel) atomicAdd(&S.ctr[C_CANCEL_OK], (unsigned long long)n_cancel);
    }
#ifdef KME_STAMPS
    c.acc[7] = stamp() - tk0;
    if (lane == 0)
        for (int q = 0; q < 16; ++q) S.dbg[(size_t)g * 16 + q] = c.acc[q];
#endif
}

// EXACT: one wavefront, the whole epoch in arrival order, every store exact.
__global__ void __launch_bounds__(64) k_serial(const DevState* __restrict__ Sp, const EpochIO* __restrict__ iop) {
    const DevState& S = *Sp;
    const EpochIO& io = *iop;
    if (failed(S.ctr)) return;
    Core<true, false> c(S, io, nullptr, nullptr, nullptr, nullptr);
    const int lane = lane_id();
    uint32_t n_rest = 0, n_cancel = 0;
    for (uint32_t k0 = 0; k0 < io.n && !c.dead; k0 += 64) {
        const uint32_t k = k0 + lane;
        const bool valid = k < io.n;
        const Batch B = load_batch(S, io, valid, valid ? k : 0, false);
        const int32_t bgrp = valid ? S.route_grp[k] : -1;
        const int nb = (int)(io.n - k0 < 64 ? io.n - k0 : 64);
#pragma nounroll
        for (int j = 0; j < nb && !c.dead; ++j) {
            const Rec r = pick(B, j);
            const uint32_t i = r.i;
            const int32_t a = r.action;
            int32_t grp = -1;
            if (a == CANCEL) grp = rl32(bgrp, j);
            else if (a == ADD_SYMBOL || a == REMOVE_SYMBOL || a == PAYOUT || a == BUY || a == SELL) grp = group_of(r.sid, S.G);
            if (grp >= 0) {
                if (grp != c.g) { c.store_group(); c.load_group(grp); }
                const Out o = c.process(r, -1);
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
            case ADD_SYMBOL: c.die(KME_E_CAPACITY, KME_D_CAP_SYMBOL, i); break;
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
        io.trade_off[io.n] = c.tnext;
        S.ctr[C_TRADES] = c.tnext;
        S.ctr[C_RESTS] = n_rest;
        S.ctr[C_CANCEL_OK] = n_cancel;
    }
}

// ------------------------------------------------------------------ (4) compaction
__global__ void k_scatter(DevState S, EpochIO io, const uint32_t* total) {
    const uint32_t cnt = (uint32_t)S.ctr[C_TTMP];
    if (*total > io.trades_cap) {
        if (blockIdx.x == 0 && threadIdx.x == 0) raise_thread(S.ctr, KME_E_CAPACITY, KME_D_CAP_TRADES, -1);
        return;
    }
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < cnt; k += gridDim.x * blockDim.x) {
        const TradeTmp r = S.ttmp[k];
        if (r.seq < 0) continue;
        io.trades[io.trade_off[r.seq] + (uint32_t)r.ord] = r.t;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) S.ctr[C_TRADES] = *total;
}

// ------------------------------------------------------------------ oid-table maintenance
// Orders that came to rest this epoch and are still live get an oid-table entry.  The used-slot
// counter is bumped once per wavefront (a single hot counter would serialise every insert).
// Oid-table entries for the orders of this epoch that are still resting.
__global__ void k_table(DevState S, EpochIO io) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    bool ins = false;
    if (i < io.n) {
        const int32_t s = S.rest_slot[i];
        if (s >= 0) {
            const int64_t oid = io.oid[i];
            if (S.pool[s].live && S.pool[s].oid == oid) {
                ins = otab_insert(S, oid, s);
                if (!ins) raise_thread(S.ctr, KME_E_CAPACITY, KME_D_CAP_OIDTAB, i);
            }
        }
    }
    const unsigned long long b = __ballot(ins);
    if (lane_id() == 0 && b) atomicAdd(&S.ctr[C_OTAB_USED], (unsigned long long)__popcll(b));
}
__global__ void k_otab_refill(DevState S, uint32_t nslots) {
    const uint32_t stride = gridDim.x * blockDim.x;
    const uint32_t lim = (nslots + stride - 1) / stride * stride;   // whole wavefronts for the ballot
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < lim; s += stride) {
        bool ins = false;
        if (s < nslots && S.pool[s].live) {
            ins = otab_insert(S, S.pool[s].oid, (int32_t)s);
            if (!ins) raise_thread(S.ctr, KME_E_CAPACITY, KME_D_CAP_OIDTAB, -1);
        }
        const unsigned long long b = __ballot(ins);
        if (lane_id() == 0 && b) atomicAdd(&S.ctr[C_OTAB_USED], (unsigned long long)__popcll(b));
    }
}

// ------------------------------------------------------------------ market data: top of book
__global__ void k_tob(DevState S, kme_tob* out) {
    const int32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= S.G) return;
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
    out[g] = r;
}

__global__ void k_init_state(DevState S) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < (uint32_t)S.G) {
        GroupState gs;
        __builtin_memset(&gs, 0, sizeof gs);
        gs.free_head = -1;
        S.grp[k] = gs;
    }
    if (k < (uint32_t)S.A && S.acct_since) S.acct_since[k] = INT64_MAX;
}

// ------------------------------------------------------------------ launchers
static inline uint32_t cdiv(uint32_t a, uint32_t b) { return (a + b - 1) / b; }

void launch_emap(const DevState& S, const EpochIO& io, bool funded, EpochIO* io_dev, hipStream_t st) {
    hipLaunchKernelGGL(k_emap, dim3(cdiv(io.n > 0 ? io.n : 1, 256)), dim3(256), 0, st, S, io, funded ? 1 : 0, io_dev);
}
void launch_ledger_funded(const DevState& S, const EpochIO& io, hipStream_t st) {
    hipLaunchKernelGGL(k_ledger_funded, dim3(1), dim3(64), 0, st, S, io);
}
void launch_check_funded(const DevState& S, const EpochIO& io, hipStream_t st) {
    if (S.A == 0) return;
    hipLaunchKernelGGL(k_check_funded, dim3(cdiv((uint32_t)S.A, 256)), dim3(256), 0, st, S, io);
}
void launch_route(const DevState& S, const EpochIO& io, bool funded, hipStream_t st) {
    if (io.n == 0) return;
    hipLaunchKernelGGL(k_route, dim3(cdiv(io.n, 256)), dim3(256), 0, st, S, io, funded ? 1 : 0);
}
static void launch_scan(const uint32_t* in, uint32_t* out, uint32_t L, uint32_t* bsum, uint32_t* total, hipStream_t st) {
    const uint32_t nb = cdiv(L > 0 ? L : 1, SCAN_BLOCK);
    hipLaunchKernelGGL(k_scan_blocks, dim3(nb), dim3(256), 0, st, in, out, L, bsum);
    hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(256), 0, st, bsum, nb, total);
    hipLaunchKernelGGL(k_scan_add, dim3(nb), dim3(256), 0, st, out, L, bsum);
}
int launch_partition(const DevState& S, const EpochIO& io, hipStream_t st) {
    const uint32_t ntiles = cdiv(io.n > 0 ? io.n : 1, RADIX_TILE);
    int src = 0;
    for (int pass = 0; pass < S.passes; ++pass) {
        hipLaunchKernelGGL(k_radix_hist, dim3(ntiles), dim3(256), 0, st, S, io, pass, src);
        // exclusive scan of the digit-major histogram, in place (scratch at the tail of ghist)
        const uint32_t L = 256 * ntiles;
        uint32_t* bsum = S.ghist + L;
        uint32_t* total = bsum + cdiv(L, SCAN_BLOCK) + 1;
        launch_scan(S.ghist, S.ghist, L, bsum, total, st);
        hipLaunchKernelGGL(k_radix_scatter, dim3(ntiles), dim3(256), 0, st, S, io, pass, src);
        src ^= 1;
    }
    const uint32_t nthreads = (io.n + 1) > (uint32_t)S.G + 2 ? io.n + 1 : (uint32_t)S.G + 2;
    hipLaunchKernelGGL(k_segments, dim3(cdiv(nthreads, 256)), dim3(256), 0, st, S, io, src);
    return src;
}
void launch_match(const DevState& S, const DevState* S_dev, const EpochIO* io_dev, int buf, hipStream_t st) {
    hipLaunchKernelGGL(k_match, dim3((uint32_t)S.G), dim3(64), 0, st, S_dev, io_dev, buf);
}
void launch_compact(const DevState& S, const EpochIO& io, hipStream_t st) {
    // trade_off[0..n] = exclusive scan of n_trades; bsum/total scratch in ghist
    uint32_t* bsum = S.ghist;
    const uint32_t nb = cdiv(io.n > 0 ? io.n : 1, SCAN_BLOCK);
    uint32_t* total = bsum + nb + 1;
    launch_scan(io.n_trades, io.trade_off, io.n, bsum, total, st);
    (void)hipMemcpyAsync(io.trade_off + io.n, total, sizeof(uint32_t), hipMemcpyDeviceToDevice, st);
    hipLaunchKernelGGL(k_scatter, dim3(1024), dim3(256), 0, st, S, io, (const uint32_t*)total);
}
void launch_table(const DevState& S, const EpochIO& io, hipStream_t st) {
    if (io.n == 0) return;
    hipLaunchKernelGGL(k_table, dim3(cdiv(io.n, 256)), dim3(256), 0, st, S, io);
}
void launch_serial(const DevState* S_dev, const EpochIO* io_dev, hipStream_t st) {
    hipLaunchKernelGGL(k_serial, dim3(1), dim3(64), 0, st, S_dev, io_dev);
}
void launch_otab_rebuild(const DevState& S, hipStream_t st) {
    (void)hipMemsetAsync(S.otab_key, 0, sizeof(uint64_t) * ((size_t)S.otab_mask + 1), st);
    (void)hipMemsetAsync(&S.ctr[C_OTAB_USED], 0, sizeof(unsigned long long), st);
    hipLaunchKernelGGL(k_otab_refill, dim3(2048), dim3(256), 0, st, S, S.pool_cap);
}
void launch_tob(const DevState& S, void* out, hipStream_t st) {
    hipLaunchKernelGGL(k_tob, dim3(cdiv((uint32_t)S.G, 256)), dim3(256), 0, st, S, (kme_tob*)out);
}
void launch_init_state(const DevState& S, hipStream_t st) {
    const uint32_t n = (uint32_t)(S.G > S.A ? S.G : S.A);
    hipLaunchKernelGGL(k_init_state, dim3(cdiv(n > 0 ? n : 1, 256)), dim3(256), 0, st, S);
}

}  // namespace kme
