// kme_runtime.cpp -- host runtime behind include/kme.h: HBM allocation of the stores, the epoch
// launch sequence, result retrieval and canonical snapshots.
//
// Reference correspondence (KProcessor.java, "KP"):
//   kme_create            KP:30-49 (store builders) + MatchingEngine.init KP:86-93
//   kme_submit_epoch[_device]  MatchingEngine.process KP:96-126, for a whole epoch of records
//   kme_destroy           MatchingEngine.close KP:129
//   kme_snapshot_*        the contents of Books/Buckets/Orders and Balances/Positions
#include <dlfcn.h>
#include <fcntl.h>
#include <unistd.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "kme.h"
#include "kme_device.h"
#include "kme_launch.h"
#include "kme_internal.h"

using namespace kme;

namespace {

const char* kPhaseNames[] = {"emap", "ledger", "route", "partition", "match", "compact", "table", "serial", "replay"};
enum Phase { PH_EMAP, PH_LEDGER, PH_ROUTE, PH_PART, PH_MATCH, PH_COMPACT, PH_TABLE, PH_SERIAL, PH_REPLAY, PH_N };

uint64_t pow2_at_least(uint64_t x) {
    uint64_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

}  // namespace

namespace kme {
// Tests only: env KME_TEST_FAIL names a failure path to take where the product path cannot otherwise
// be driven into it (an allocation that fails).
bool test_hook_fail(const char* what) {
    const char* v = std::getenv("KME_TEST_FAIL");
    return v && std::strcmp(v, what) == 0;
}
}  // namespace kme

struct kme_engine {
    kme_config cfg{};
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t lane_stream = nullptr;   // k_match_lanes runs here, beside k_match (fork / join events)
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    uint64_t last_busy = 1;              // groups k_match took in the last epoch (C_BUSY)
    // k_match in two-wavefront mode when 1 .. two_max groups were busy in the last epoch (KME_TWO_MAX;
    // 0: never) and fewer than 1 in 8 of its records were cancels that removed an order: the serial
    // path a cancel-heavy stream takes often makes wave 0 wait
    uint64_t two_max = 4096;
    bool dense_grid = true;              // k_match's busy groups first in the grid (KME_DENSE_GRID=0: off, A/B)
    bool match_list = true;              // k_match_list when no group was busy (KME_MATCH_LIST=0: off, A/B)
    uint32_t lvk_next_tag = 1;           // the exact ledger's next value-key table tag (DevState::lvk_tag)
    bool last_cancel_heavy = false;
    uint64_t last_light = 1;             // k_match_lanes wavefronts with a group in the last epoch (C_LIGHT)
    hipStream_t stream = nullptr;
    DevState S{};
    DevState* d_S = nullptr;
    EpochIO* d_io = nullptr;
    // engine-owned epoch buffers
    int32_t *d_action = nullptr, *d_price = nullptr, *d_size = nullptr;
    int64_t *d_oid = nullptr, *d_aid = nullptr, *d_sid = nullptr;
    int32_t *d_out_action = nullptr, *d_out_size = nullptr;
    int64_t* d_out_prev = nullptr;
    uint8_t* d_out_flags = nullptr;
    uint32_t *d_ntrades = nullptr, *d_trade_off = nullptr;
    TradeRec* d_trades = nullptr;
    unsigned long long* h_ctr = nullptr;  // pinned copies of the counters block: one per epoch slot
    unsigned long long* d_hctr = nullptr; // h_ctr's device mapping (k_ledger_replay's copy)
                                          // (two epochs may be in flight), a third for the rebuild
    // device serializer scratch: per-input byte counts, offsets, scan partials, u64 total
    uint32_t *d_ser_len = nullptr, *d_ser_off = nullptr, *d_ser_tmp = nullptr;
    unsigned long long* d_ser_total = nullptr;
    unsigned long long* h_ser_total = nullptr;
    char* h_stage = nullptr;              // pinned bounce buffer of the snapshots' device reads (kStage bytes)
    kme::PinnedRing ring;                 // the checkpoint writer's pinned slots (made at the first checkpoint)
    std::vector<void*> allocs;
    int64_t seq_base = 0;
    // epochs in flight: submitted to the stream, not yet waited for (at most two; slot = submission
    // number & 1; kme_wait takes the oldest)
    int inflight = 0;
    uint32_t sub_count = 0;
    uint32_t fl_n[2] = {};
    int cur_slot = 0;
    hipEvent_t ev_end[2] = {};
    int failed = 0;
    int fail_status = 0, fail_detail = 0;
    int timing = 0;                      // KME_TIMING_* (kme.h)
    hipEvent_t ev[2][PH_N * 2] = {};
    bool ev_used[2][PH_N] = {};
    float phase_ms[KME_MAX_PHASES] = {};
    uint64_t otab_cap = 0;
    // host epochs (kme_submit_epoch_host): two slots of device-side inputs and results, a copy stream
    // each way (allocated at the first host epoch)
    struct HostSlot {
        int32_t *action, *price, *size;
        int64_t *oid, *aid, *sid;
        int32_t *out_action, *out_size;
        int64_t* out_prev;
        uint8_t* out_flags;
        uint32_t* trade_off;
        TradeRec* trades;
    };
    HostSlot hs[2] = {};
    bool hs_ready = false;
    hipStream_t in_stream = nullptr, out_stream = nullptr;
    hipEvent_t ev_in[2] = {};
    // caller host memory registered through this engine (kme_host_register): exact ranges with a
    // count; `owned` = this engine's hipHostRegister made it (another owner's registration of the same
    // pages is used, never undone here)
    struct HostReg { uintptr_t p; size_t bytes; int refs; bool owned; };
    std::vector<HostReg> host_regs;
    bool host_epoch[2] = {};              // the epoch of this slot is a host epoch
    bool host_mapped[2] = {};             // its trades go out through the device mapping (k_export_trades)
    kme_epoch_result host_out[2] = {};    // the caller's result buffers of that epoch
    // exact Balances / Positions (EXACT mode, FUNDED + KME_FLAG_EXACT_LEDGER): rehashed into larger
    // tables between epochs (ledger_reserve), ledger_grows times so far
    bool ledger = false;
    uint32_t ledger_grows = 0;
    unsigned long long* d_maint = nullptr;   // 4 words of maintenance-kernel results
};

#define HIP_TRY(x)                                                                          \
    do {                                                                                    \
        hipError_t _e = (x);                                                                \
        if (_e != hipSuccess) {                                                             \
            std::fprintf(stderr, "kme: HIP error %s at %s:%d\n", hipGetErrorString(_e), __FILE__, __LINE__); \
            return KME_E_HIP;                                                               \
        }                                                                                   \
    } while (0)

template <class T>
static kme_status dalloc(kme_engine* e, T** p, size_t count) {
    size_t bytes = std::max<size_t>(count, 1) * sizeof(T);
    void* q = nullptr;
    HIP_TRY(hipMalloc(&q, bytes));
    e->allocs.push_back(q);
    *p = reinterpret_cast<T*>(q);
    return KME_OK;
}
static void dfree(kme_engine* e, void* p) {
    if (!p) return;
    auto it = std::find(e->allocs.begin(), e->allocs.end(), p);
    if (it != e->allocs.end()) e->allocs.erase(it);
    (void)hipFree(p);
}

// Host <-> device copies of the snapshot, checkpoint and restore paths: stream-ordered, through the
// engine's pinned bounce buffer (kStage bytes, made on first use), never a pageable-host copy on the
// null stream.  Each failure names what was being copied.  (Round 5: a snapshot's pageable read of
// the Balances failed twice with an illegal-address error the plain copy could not attribute.)
constexpr size_t kStage = 8ull << 20;
static bool stage_ready(kme_engine* e) {
    if (e->h_stage) return true;
    if (hipHostMalloc((void**)&e->h_stage, kStage, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        e->h_stage = nullptr;
        return false;
    }
    return true;
}
// src (device) -> dst (host); sink(chunk, bytes) instead of dst when given
template <typename Sink>
static bool staged_read(kme_engine* e, const void* src, size_t bytes, const char* what, Sink&& sink) {
    if (!stage_ready(e)) return false;
    for (size_t off = 0; off < bytes; off += kStage) {
        const size_t c = std::min(kStage, bytes - off);
        hipError_t r = hipMemcpyAsync(e->h_stage, (const char*)src + off, c, hipMemcpyDeviceToHost, e->stream);
        if (r == hipSuccess) r = hipStreamSynchronize(e->stream);
        if (r != hipSuccess) {
            std::fprintf(stderr, "kme: device read of %s (%zu bytes at %p + %zu) failed: %s\n", what, bytes, src, off,
                         hipGetErrorString(r));
            return false;
        }
        if (!sink(e->h_stage, c, off)) return false;
    }
    return true;
}
static bool staged_d2h(kme_engine* e, void* dst, const void* src, size_t bytes, const char* what) {
    return staged_read(e, src, bytes, what, [&](const char* chunk, size_t c, size_t off) {
        std::memcpy((char*)dst + off, chunk, c);
        return true;
    });
}
// Host -> device through the engine's pinned ring when it has one (the checkpoint writer's slots):
// the copy of slot k overlaps the memcpy into slot k + 1, a slot reused once its event completed.
static bool ring_h2d(kme_engine* e, void* dst, const void* src, size_t bytes, const char* what) {
    kme::PinnedRing& R = e->ring;
    bool used[kme::kRingSlots] = {};
    int k = 0;
    hipError_t r = hipSuccess;
    for (size_t off = 0; off < bytes && r == hipSuccess; off += kme::kRingSlot) {
        const size_t c = std::min(kme::kRingSlot, bytes - off);
        if (used[k]) r = hipEventSynchronize(R.ev[k]);
        if (r != hipSuccess) break;
        std::memcpy(R.slot[k], (const char*)src + off, c);
        r = hipMemcpyAsync((char*)dst + off, R.slot[k], c, hipMemcpyHostToDevice, e->stream);
        if (r == hipSuccess) r = hipEventRecord(R.ev[k], e->stream);
        used[k] = true;
        k = (k + 1) % kme::kRingSlots;
    }
    if (r == hipSuccess) r = hipStreamSynchronize(e->stream);   // (the slots are reused by the next call)
    if (r != hipSuccess) {
        (void)hipStreamSynchronize(e->stream);   // (copies still in flight read the slots: drained first)
        (void)hipGetLastError();
        std::fprintf(stderr, "kme: device write of %s (%zu bytes at %p) failed: %s\n", what, bytes, dst, hipGetErrorString(r));
        return false;
    }
    return true;
}
static bool staged_h2d(kme_engine* e, void* dst, const void* src, size_t bytes, const char* what) {
    if (bytes > kStage && e->ring.init(e->device)) return ring_h2d(e, dst, src, bytes, what);
    if (!stage_ready(e)) return false;
    for (size_t off = 0; off < bytes; off += kStage) {
        const size_t c = std::min(kStage, bytes - off);
        std::memcpy(e->h_stage, (const char*)src + off, c);
        hipError_t r = hipMemcpyAsync((char*)dst + off, e->h_stage, c, hipMemcpyHostToDevice, e->stream);
        if (r == hipSuccess) r = hipStreamSynchronize(e->stream);   // (the stage is reused next chunk)
        if (r != hipSuccess) {
            std::fprintf(stderr, "kme: device write of %s (%zu bytes at %p + %zu) failed: %s\n", what, bytes, dst, off,
                         hipGetErrorString(r));
            return false;
        }
    }
    return true;
}
// The snapshots: a device fault pending from earlier work is reported as such before any read.
static kme_status snap_begin(kme_engine* e, const char* what) {
    HIP_TRY(hipSetDevice(e->device));
    const hipError_t q = hipStreamSynchronize(e->stream);
    const hipError_t d = q == hipSuccess ? hipDeviceSynchronize() : q;
    if (d != hipSuccess) {
        std::fprintf(stderr, "kme: %s: a device fault was pending before its reads: %s\n", what, hipGetErrorString(d));
        return KME_E_HIP;
    }
    return stage_ready(e) ? KME_OK : KME_E_HIP;
}
static kme_status snap_read(kme_engine* e, void* dst, const void* src, size_t bytes, const char* what) {
    return staged_d2h(e, dst, src, bytes, what) ? KME_OK : KME_E_HIP;
}

// ------------------------------------------------------------------ ledger table sizes
// The most entries one epoch can add: Balances one per CREATE_BALANCE record (KP:131-138); Positions
// one per ledger effect -- a record's checkBalance / postRemoveAdjustments, both fillOrder calls of
// each trade (KP:167-182, 276-287, 325-333) -- each reads one key and writes at most one new one.
static uint64_t bal_bound(const kme_config& c) { return c.max_epoch; }
static uint64_t pos_bound(const kme_config& c) { return (uint64_t)c.max_epoch + 2ull * c.max_trades; }
// Slots for `live` entries plus `ahead` epochs of worst-case growth at no more than half load.
static uint64_t ledger_slots(uint64_t live, uint64_t bound, uint64_t ahead) {
    return pow2_at_least(std::max<uint64_t>(2 * (live + ahead * bound), 2048));
}

#define ALLOC(ptr, n)                                  \
    do {                                               \
        kme_status _s = dalloc(e, &(ptr), (size_t)(n)); \
        if (_s != KME_OK) { kme_destroy(e); return _s; } \
    } while (0)

// Timing events serialise the stream around them (~10 us each, measured), so KME_TIMING_MATCH
// brackets only the matching kernels.
static bool timed(const kme_engine* e, int ph) {
    return e->timing == KME_TIMING_ALL || (e->timing == KME_TIMING_MATCH && ph == PH_MATCH);
}
static void phase_begin(kme_engine* e, int ph, hipStream_t s = nullptr) {
    if (!timed(e, ph)) return;
    (void)hipEventRecord(e->ev[e->cur_slot][2 * ph], s ? s : e->stream);
    e->ev_used[e->cur_slot][ph] = true;
}
static void phase_end(kme_engine* e, int ph, hipStream_t s = nullptr) {
    if (!timed(e, ph)) return;
    (void)hipEventRecord(e->ev[e->cur_slot][2 * ph + 1], s ? s : e->stream);
}

extern "C" {

const char* kme_strerror(int s) {
    switch (s) {
    case KME_OK: return "ok";
    case KME_E_INVALID: return "invalid argument";
    case KME_E_CAPACITY: return "capacity exceeded";
    case KME_E_DOMAIN: return "input outside the parity domain (reference would throw or hang)";
    case KME_E_UNFUNDED: return "FUNDED mode: order acceptance not provably ledger-independent";
    case KME_E_UNSUPPORTED: return "operation not supported in this mode";
    case KME_E_HIP: return "HIP runtime error";
    case KME_E_FAILED: return "engine failed earlier";
    default: return "unknown";
    }
}
const char* kme_domain_str(int d) {
    static const char* names[] = {"none", "NPE position (KP:179-180/332)", "NPE bucket (KP:234-235/252-253)",
                                  "NPE order (KP:236-237/257)", "NPE balance (KP:157/286/331)",
                                  "removeAllOrders never returns (KP:341-353)", "NPE book (KP:294)",
                                  "resting price outside 0..126", "duplicate live oid", "FUNDED price/size range",
                                  "sentinel oid", "order pool full", "oid table full", "trade buffer full",
                                  "symbol id >= max_symbols", "account id >= max_accounts", "ledger table full",
                                  "epoch larger than max_epoch",
                                  "funded proof failed: the epoch as a whole was refused"};
    if (d < 0 || d >= (int)(sizeof(names) / sizeof(names[0]))) return "unknown";
    return names[d];
}
void kme_free(void* p) { std::free(p); }

kme_status kme_create(const kme_config* cfg, kme_engine** out) {
    if (!cfg || !out) return KME_E_INVALID;
    if (cfg->abi_version != KME_ABI_VERSION) return KME_E_INVALID;
    if (cfg->mode != KME_MODE_EXACT && cfg->mode != KME_MODE_FUNDED) return KME_E_INVALID;
    // sparse symbols (|sid| >= max_symbols, KP:184-191 takes any long): serial engine only, so by default
    // where a serial engine runs (EXACT; FUNDED with the serial fallback)
    uint64_t Gs = 0;
    if (cfg->max_sparse_symbols == KME_SPARSE_NONE) Gs = 0;
    else if (cfg->max_sparse_symbols) Gs = pow2_at_least(cfg->max_sparse_symbols);
    else if (cfg->mode == KME_MODE_EXACT || (cfg->flags & KME_FLAG_SERIAL_FALLBACK)) Gs = 4096;
    if (cfg->max_symbols + Gs > (1ull << 24)) return KME_E_INVALID;
    if (cfg->max_symbols == 0 || cfg->max_symbols > (1u << 24) || cfg->max_epoch == 0 ||
        cfg->max_epoch > (1u << 30) || cfg->max_resting == 0 || cfg->max_resting >= (1ull << 31) ||
        cfg->max_trades == 0)
        return KME_E_INVALID;
    // FUNDED: the oid table (a power of two >= 2 (pool + epoch) entries) stays within 2^30 entries,
    // so an entry's position rides in a packed record's signed 32-bit word (k_route, otab_final)
    if (cfg->mode == KME_MODE_FUNDED && (cfg->max_accounts == 0 || cfg->max_accounts > (1u << 28) ||
                                         cfg->max_resting + (uint64_t)(cfg->max_symbols + 1 + Gs) * POOL_CHUNK +
                                                 cfg->max_epoch > (1ull << 29)))
        return KME_E_INVALID;
    if ((cfg->flags & KME_FLAG_REFUSE_SERIAL) &&
        (cfg->mode != KME_MODE_FUNDED || (cfg->flags & (KME_FLAG_SERIAL_FALLBACK | KME_FLAG_EXACT_LEDGER))))
        return KME_E_INVALID;   // (a shard of kme_multi: refuses what it cannot prove, takes nothing serially)
    if ((cfg->flags & ~(KME_FLAG_EXACT_LEDGER | KME_FLAG_SERIAL_FALLBACK | KME_FLAG_REFUSE_SERIAL)) != 0 ||
        ((cfg->flags & KME_FLAG_EXACT_LEDGER) && cfg->credit_shards > 1) ||   // a shard sees part of the ledger only
        ((cfg->flags & KME_FLAG_SERIAL_FALLBACK) && !(cfg->flags & KME_FLAG_EXACT_LEDGER)))   // needs the exact ledger
        return KME_E_INVALID;
    if (cfg->credit_shards > (1u << 16) || (cfg->mode == KME_MODE_EXACT && cfg->credit_shards > 1))
        return KME_E_INVALID;
    kme_engine* e = new kme_engine();
    e->cfg = *cfg;
    e->device = cfg->device;
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipStreamCreateWithFlags(&e->own_stream, hipStreamNonBlocking));
    HIP_TRY(hipStreamCreateWithFlags(&e->lane_stream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&e->ev_fork, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&e->ev_join, hipEventDisableTiming));
    e->stream = e->own_stream;
    for (auto& evs : e->ev)
        for (auto& ev : evs) HIP_TRY(hipEventCreate(&ev));
    for (auto& ev : e->ev_end) HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));

    const bool funded = cfg->mode == KME_MODE_FUNDED;
    const uint32_t G = cfg->max_symbols;
    const uint32_t E = cfg->max_epoch;
    // node pool: max_resting plus the slots a symbol group can hold back in its bump chunk
    // (k_match takes POOL_CHUNK slots at a time), so that max_resting resting orders always fit
    // (a sparse symbol's group holds back a chunk too)
    const uint64_t P = cfg->max_resting + (funded ? (uint64_t)(G + 1) * POOL_CHUNK : 0) + Gs * POOL_CHUNK;
    DevState& S = e->S;
    S.G = (int32_t)G;
    S.Gs = (int32_t)Gs;
    S.refuse = (cfg->flags & KME_FLAG_REFUSE_SERIAL) ? 1 : 0;
    S.mode = (int32_t)cfg->mode;
    S.A = funded ? (int32_t)cfg->max_accounts : 0;
    {
        int bits = 0;
        while ((1ull << bits) <= (uint64_t)G) ++bits;   // keys 0..G
        S.passes = (bits + RADIX_BITS - 1) / RADIX_BITS;
    }
    S.pool_cap = (uint32_t)P;
    // every BUY/SELL of an epoch takes an entry at k_emap (pending -> its rest slot, or dead, at
    // k_table), so the table holds the live orders and one epoch of new ones at half load
    e->otab_cap = pow2_at_least(std::max<uint64_t>(2 * (P + E), 1024));
    S.otab_mask = (uint32_t)(e->otab_cap - 1);
    S.credit_div = cfg->credit_shards > 1 ? cfg->credit_shards : 1;
    S.trades_cap = cfg->max_trades;
    // trade scratch: TSHARDS shard regions (2x the even share, so only skewed load spills) and an
    // overflow region that alone holds an epoch's worth of trades plus what reservations can waste:
    // k_match_lanes reserves LANE_TCH slots per lane at a time and holds one spare reservation (up
    // to 2 LANE_TCH - 1 unused per light group, at most min(G, E) of them), and a reservation that
    // straddles a shard region's end leaves the straddled part as holes (at most one per shard and
    // matcher)
    // (k_match's fast segments reserve the same way per lane of a busy group: up to 64 partly used
    // reservations per group)
    const uint64_t lane_waste = (uint64_t)(2 * kLaneTradeChunk - 1) * std::min<uint64_t>(G, E) +
                                (uint64_t)64 * (kLaneTradeChunk - 1) * std::min<uint64_t>(G, E);
    const uint64_t ttmp_ov = funded ? (uint64_t)cfg->max_trades + 64 + lane_waste + 64ull * TSHARDS : 1;
    const uint64_t tshard_cap = funded ? std::max<uint64_t>(256, (2 * (uint64_t)cfg->max_trades + TSHARDS - 1) / TSHARDS) : 0;
    const uint64_t ttmp_total = ttmp_ov + (uint64_t)TSHARDS * tshard_cap;
    if (ttmp_total >= (1ull << 32)) { kme_destroy(e); return KME_E_INVALID; }
    S.ttmp_cap = (uint32_t)ttmp_ov;
    S.tshard_cap = (uint32_t)tshard_cap;

    ALLOC(S.grp, G + Gs);
    ALLOC(S.lev, (size_t)(G + Gs) * 2 * NLEV);
    if (Gs) ALLOC(S.gsid, Gs);
    ALLOC(S.pool, P);
    ALLOC(S.otab, e->otab_cap);
    const bool exact_ledger = !funded || (cfg->flags & KME_FLAG_EXACT_LEDGER);
    S.ledger_replay = funded && exact_ledger ? 1 : 0;
    S.fallback = funded && (cfg->flags & KME_FLAG_SERIAL_FALLBACK) ? 1 : 0;
    // FUNDED groups with at most light_max records in an epoch are matched one lane per group
    // (k_match_lanes), the others one wavefront per group (k_match); KME_LIGHT_MAX overrides.
    int32_t lm = cfg->light_max == 0 ? kDefaultLightMax : std::max(0, (int32_t)cfg->light_max);
    if (const char* v = std::getenv("KME_LIGHT_MAX")) lm = std::max(0, std::atoi(v));   // diagnostics
    S.light_max = funded ? lm : 0;
    if (funded) {
        ALLOC(S.acct_since, cfg->max_accounts);
        ALLOC(S.acct_lb, cfg->max_accounts);
        ALLOC(S.acct_need, cfg->max_accounts);
        ALLOC(S.acct_negx, cfg->max_accounts);
        ALLOC(S.acct_xfer, cfg->max_accounts);
        ALLOC(S.acct_demand, cfg->max_accounts);
        if (S.ledger_replay) ALLOC(S.vic, E);
    }
    if (S.ledger_replay) {   // the parallel ledger pass (kme_ledger.hip); KME_LEDGER_SERIAL=1: the serial replay only
        // ops: one per ledger effect (a check / cancel per record, two fills per trade)
        const uint64_t nops = (uint64_t)E + 2ull * cfg->max_trades;
        const char* ls = std::getenv("KME_LEDGER_SERIAL");
        S.lpar = (!ls || !std::atoi(ls)) && cfg->max_accounts <= (1u << 23) && cfg->max_symbols < (1u << 30) &&
                 nops < (1ull << 30) ? 1 : 0;
        if (S.lpar) {
            // sort key aid << hb | hash(sid), hb = 8: a bucket holds ~one chain.  (Measured and not
            // kept: hb = 2 at 65,536 accounts, two radix passes instead of three -- the longer bucket
            // runs cost k_lchains and k_ldetect far more than the pass saves.  KME_LEDGER_HBITS: A/B.)
            // Fewer hash bits where an epoch cannot give an account many ops: with more accounts than
            // ops per epoch (the drop-in's 2^20 accounts, 65,536-record epochs) a bucket holds ~one
            // chain at any hb, so hb shrinks until the key fits one pass fewer (28 -> 27 bits: three
            // passes, not four); at C3 (~113 ops per account) hb stays 8.
            int abits = 0;
            while ((1ull << abits) < (uint64_t)cfg->max_accounts) ++abits;
            const uint64_t per_acct = (nops + cfg->max_accounts - 1) / std::max<uint64_t>(1, cfg->max_accounts);
            int hb_min = 1;
            while (hb_min < 8 && (1ull << (hb_min - 1)) < per_acct) ++hb_min;
            hb_min = std::max(2, hb_min);
            const int passes = (abits + hb_min + RADIX_BITS - 1) / RADIX_BITS;
            int hb = std::min(8, passes * RADIX_BITS - abits);
            if (const char* v = std::getenv("KME_LEDGER_HBITS")) hb = std::max(1, std::min(8, std::atoi(v)));
            S.lhbits = hb;
            S.lpasses = std::max(1, (abits + hb + RADIX_BITS - 1) / RADIX_BITS);
            S.lr_cap = 1u << 18;     // chains re-run by the repair rounds
            S.lx_cap = 1u << 19;     // couplings
            S.lc_cap = 1u << 20;     // value writes changed in one round
            S.lrounds = 8;           // repair rounds before the serial replay (KME_LEDGER_ROUNDS: tests)
            if (const char* v = std::getenv("KME_LEDGER_ROUNDS")) S.lrounds = (uint32_t)std::max(1, std::min(64, std::atoi(v)));
            const uint64_t vk = pow2_at_least(std::min<uint64_t>(2 * nops, 1ull << 22));
            S.lvk_mask = vk - 1;
            const uint64_t lh = (uint64_t)(1 << RADIX_BITS) * ((nops + RADIX_TILE_SMALL - 1) / RADIX_TILE_SMALL);
            ALLOC(S.lcnt, E);
            ALLOC(S.lscan, E / 4096 + 64);
            ALLOC(S.lk0, nops);
            ALLOC(S.lkey[0], nops); ALLOC(S.lkey[1], nops);
            ALLOC(S.lval[0], nops); ALLOC(S.lval[1], nops);
            ALLOC(S.lghist, lh + lh / 4096 + 4096);
            // the op sort of a small epoch (launch_ledger_parallel: R.small) in one launch per pass
            const uint64_t lt = (nops + RADIX_TILE_SMALL - 1) / RADIX_TILE_SMALL;
            if (E <= (1u << 17) && lt <= 1024 && S.lpasses <= RADIX_MAXP) {
                ALLOC(S.ltcnt, (size_t)RADIX_MAXP * lt * (1 << RADIX_BITS));
                ALLOC(S.llb, (size_t)lt * (1 << RADIX_BITS));
            }
            ALLOC(S.lrec, nops); ALLOC(S.lsrt, nops);
            ALLOC(S.lchain, nops); ALLOC(S.lhead, nops);
            ALLOC(S.lvw, nops); ALLOC(S.lvw_meta, nops); ALLOC(S.lvw_tgt, nops);
            ALLOC(S.lseg, (size_t)cfg->max_accounts + 2);
            ALLOC(S.lgap, (size_t)cfg->max_accounts / 256 + (size_t)cfg->max_accounts / 4096 + 8);   // (k_lseg's gaps)
            ALLOC(S.ldelta, cfg->max_accounts);
            HIP_TRY(hipMemsetAsync(S.ldelta, 0, sizeof(int64_t) * cfg->max_accounts, e->stream));   // (then kept 0: k_lbalances)
            ALLOC(S.lvk, vk);
            HIP_TRY(hipMemsetAsync(S.lvk, 0, sizeof(ulonglong4) * vk, e->stream));   // (tags from 1 on)
            ALLOC(S.lx, S.lx_cap); ALLOC(S.lxn, S.lx_cap);
            ALLOC(S.lxmark, nops);
            ALLOC(S.lrun, S.lr_cap);
            ALLOC(S.lchg, S.lc_cap);
            ALLOC(S.lctr, (size_t)LC_N * CTR_STRIDE);
            ALLOC(S.lposc, (size_t)64 * CTR_STRIDE);
        }
    }
    if (exact_ledger) {
        // ledger_capacity: the entries the tables take before their first growth; at least two
        // epochs' worth (one in flight, the next), so that ledger_reserve can always run between them
        e->ledger = true;
        const uint64_t lb = ledger_slots(std::max<uint64_t>(cfg->ledger_capacity, 1024), bal_bound(*cfg), 2);
        const uint64_t lp = ledger_slots(std::max<uint64_t>(cfg->ledger_capacity, 1024), pos_bound(*cfg), 2);
        if (lb > (1ull << 31) || lp > (1ull << 31)) { kme_destroy(e); return KME_E_INVALID; }
        S.bal_mask = (uint32_t)(lb - 1);
        S.pos_mask = (uint32_t)(lp - 1);
        ALLOC(S.bal_state, lb);
        ALLOC(S.bal_key, lb);
        ALLOC(S.bal_val, lb);
        ALLOC(S.pos, lp);
    }
    ALLOC(e->d_maint, 4);
    ALLOC(S.epos, E);
    ALLOC(S.route_grp, E);
    ALLOC(S.cancel_tgt, E);
    ALLOC(S.rest_slot, E);
    if (funded) ALLOC(S.prec, 2 * (size_t)E);
    if (funded) ALLOC(S.lvbase, (size_t)FAST_LVB * E);
    // OUT echo: one 16-B record per input index, stored by the matching kernels where the record
    // arrived (k_unsort then reads it sequentially; no sorted-position map)
    S.os_base = E;
    S.fast = 1;
    if (const char* v = std::getenv("KME_FAST")) S.fast = std::atoi(v) != 0;   // A/B diagnostics
    if (const char* v = std::getenv("KME_TWO_DRAIN")) if (S.fast && std::atoi(v)) S.fast |= 2;   // diagnostics
    if (const char* v = std::getenv("KME_TWO_MAX")) e->two_max = (uint64_t)std::max(0, std::atoi(v));   // A/B diagnostics
    if (const char* v = std::getenv("KME_DENSE_GRID")) e->dense_grid = std::atoi(v) != 0;
    if (const char* v = std::getenv("KME_MATCH_LIST")) e->match_list = std::atoi(v) != 0;
    if (funded) ALLOC(S.osort, (size_t)E + 64);   // + a dump slot per lane (k_match)
    if (funded) {
        ALLOC(S.rkeys[0], E); ALLOC(S.rkeys[1], E);
        ALLOC(S.rvals[0], E); ALLOC(S.rvals[1], E);
        ALLOC(S.ttmp, ttmp_total);
        ALLOC(S.tsh, (size_t)TSHARDS * CTR_STRIDE);
    }
    const uint64_t ntiles = (E + RADIX_TILE_SMALL - 1) / RADIX_TILE_SMALL;
    ALLOC(S.ghist, (size_t)(1 << RADIX_BITS) * ntiles + 2 * (E / 2048 + 16) + 4096);
    {   // the partition's small sorts (at most RADIX_SMALL_N keys): look-back buffers
        const uint64_t st = (std::min<uint64_t>(E, RADIX_SMALL_N) + RADIX_TILE_SMALL - 1) / RADIX_TILE_SMALL;
        ALLOC(S.rtcnt, (size_t)RADIX_MAXP * st * (1 << RADIX_BITS));
        ALLOC(S.rlb, (size_t)st * (1 << RADIX_BITS));
    }
    ALLOC(S.seg, (size_t)G + 2);
    ALLOC(S.gflag, (size_t)G + 1); ALLOC(S.glist, (size_t)G + 1); ALLOC(S.gcount, 64 + (size_t)G / 4096 + 64);
    ALLOC(S.ctr, (size_t)C_NCTR * CTR_STRIDE);
    ALLOC(S.dbg, (size_t)G * KME_DBG_WORDS);
    HIP_TRY(hipMemsetAsync(S.dbg, 0, (size_t)G * KME_DBG_WORDS * sizeof(unsigned long long), e->stream));
    // epoch buffers
    ALLOC(e->d_action, E); ALLOC(e->d_price, E); ALLOC(e->d_size, E);
    ALLOC(e->d_oid, E); ALLOC(e->d_aid, E); ALLOC(e->d_sid, E);
    ALLOC(e->d_out_action, E); ALLOC(e->d_out_size, E); ALLOC(e->d_out_prev, E);
    ALLOC(e->d_out_flags, E); ALLOC(e->d_ntrades, E); ALLOC(e->d_trade_off, (size_t)E + 1);
    ALLOC(e->d_trades, cfg->max_trades);
    ALLOC(e->d_ser_len, E); ALLOC(e->d_ser_off, (size_t)E + 1); ALLOC(e->d_ser_tmp, (size_t)E / 2048 + 64);
    ALLOC(e->d_ser_total, 1);
    ALLOC(e->d_S, 1);
    ALLOC(e->d_io, 1);
    HIP_TRY(hipHostMalloc((void**)&e->h_ser_total, sizeof(unsigned long long), hipHostMallocDefault));
    HIP_TRY(hipHostMalloc((void**)&e->h_ctr, 3 * (size_t)C_NCTR * CTR_STRIDE * sizeof(unsigned long long), hipHostMallocDefault));
    HIP_TRY(hipHostGetDevicePointer((void**)&e->d_hctr, e->h_ctr, 0));

    // initial store contents: every group absent, empty tables
    hipStream_t st = e->stream;
    HIP_TRY(hipMemsetAsync(S.otab, 0, e->otab_cap * sizeof(uint64_t), st));
    HIP_TRY(hipMemsetAsync(S.pool, 0, P * sizeof(Node), st));
    HIP_TRY(hipMemsetAsync(S.ctr, 0, (size_t)C_NCTR * CTR_STRIDE * sizeof(unsigned long long), st));
    if (S.tsh) HIP_TRY(hipMemsetAsync(S.tsh, 0, (size_t)TSHARDS * CTR_STRIDE * sizeof(unsigned long long), st));
    if (funded) {
        HIP_TRY(hipMemsetAsync(S.acct_lb, 0, cfg->max_accounts * sizeof(int64_t), st));
        HIP_TRY(hipMemsetAsync(S.acct_need, 0, cfg->max_accounts * sizeof(int64_t), st));
        HIP_TRY(hipMemsetAsync(S.acct_negx, 0, cfg->max_accounts * sizeof(int64_t), st));
        HIP_TRY(hipMemsetAsync(S.acct_xfer, 0, cfg->max_accounts * sizeof(int64_t), st));
        HIP_TRY(hipMemsetAsync(S.acct_demand, 0, cfg->max_accounts * sizeof(int64_t), st));
    }
    if (exact_ledger) {
        HIP_TRY(hipMemsetAsync(S.bal_state, 0, ((size_t)S.bal_mask + 1) * sizeof(uint32_t), st));
        HIP_TRY(hipMemsetAsync(S.pos, 0, ((size_t)S.pos_mask + 1) * sizeof(PosEntry), st));
    }
    launch_init_state(S, st);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(e->d_S, &e->S, sizeof(DevState), hipMemcpyHostToDevice, st));
    HIP_TRY(hipStreamSynchronize(st));
    *out = e;
    return KME_OK;
}

kme_status kme_destroy(kme_engine* e) {
    if (!e) return KME_E_INVALID;
    (void)hipSetDevice(e->device);
    // every queued copy and kernel of the engine finishes before its memory goes
    if (e->in_stream) (void)hipStreamSynchronize(e->in_stream);
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    if (e->lane_stream) (void)hipStreamSynchronize(e->lane_stream);
    if (e->out_stream) (void)hipStreamSynchronize(e->out_stream);
    for (void* p : e->allocs) (void)hipFree(p);
    if (e->h_ctr) (void)hipHostFree(e->h_ctr);
    if (e->h_ser_total) (void)hipHostFree(e->h_ser_total);
    if (e->h_stage) (void)hipHostFree(e->h_stage);
    e->ring.release();
    for (auto& evs : e->ev)
        for (auto& ev : evs) if (ev) (void)hipEventDestroy(ev);
    for (auto& ev : e->ev_end) if (ev) (void)hipEventDestroy(ev);
    if (e->in_stream) (void)hipStreamSynchronize(e->in_stream);
    if (e->out_stream) (void)hipStreamSynchronize(e->out_stream);
    for (auto& ev : e->ev_in) if (ev) (void)hipEventDestroy(ev);
    if (e->in_stream) (void)hipStreamDestroy(e->in_stream);
    if (e->out_stream) (void)hipStreamDestroy(e->out_stream);
    for (auto& r : e->host_regs)
        if (r.owned) (void)hipHostUnregister((void*)r.p);
    if (e->own_stream) (void)hipStreamDestroy(e->own_stream);
    if (e->lane_stream) (void)hipStreamDestroy(e->lane_stream);
    if (e->ev_fork) (void)hipEventDestroy(e->ev_fork);
    if (e->ev_join) (void)hipEventDestroy(e->ev_join);
    delete e;
    return KME_OK;
}

kme_status kme_set_stream(kme_engine* e, void* s) {
    if (!e) return KME_E_INVALID;
    e->stream = s ? reinterpret_cast<hipStream_t>(s) : e->own_stream;
    return KME_OK;
}

kme_status kme_enable_timing(kme_engine* e, int enable) {
    if (!e) return KME_E_INVALID;
    e->timing = enable == KME_TIMING_MATCH ? KME_TIMING_MATCH : enable != 0 ? KME_TIMING_ALL : 0;
    return KME_OK;
}

static kme_status submit(kme_engine* e, const kme_orders* in, uint32_t n, const kme_epoch_result* out) {
    if (e->failed) return KME_E_FAILED;
    if (n > e->cfg.max_epoch) return KME_E_CAPACITY;
    if (e->inflight == 2) return KME_E_INVALID;   // two epochs in flight: kme_wait the older first
    const int slot = (int)(e->sub_count & 1);
    e->cur_slot = slot;
    const bool funded = e->cfg.mode == KME_MODE_FUNDED;
    DevState& S = e->S;
    hipStream_t st = e->stream;
    EpochIO io{};
    io.action = in->action; io.oid = in->oid; io.aid = in->aid; io.sid = in->sid;
    io.price = in->price; io.size = in->size;
    if (out) {
        io.out_action = out->out_action; io.out_size = out->out_size; io.out_prev = out->out_prev;
        io.out_flags = out->out_flags; io.trade_off = out->trade_off; io.trades = reinterpret_cast<TradeRec*>(out->trades);
        io.trades_cap = out->trades_cap;
    } else {
        io.out_action = e->d_out_action; io.out_size = e->d_out_size; io.out_prev = e->d_out_prev;
        io.out_flags = e->d_out_flags; io.trade_off = e->d_trade_off; io.trades = e->d_trades;
        io.trades_cap = e->cfg.max_trades;
    }
    io.n_trades = e->d_ntrades;
    io.n = n;
    io.seq_base = e->seq_base;
    for (bool& u : e->ev_used[slot]) u = false;

    // per-epoch counters: error = none, stats = 0 (pool bump / table usage persist)
    launch_epoch_reset(S, st);

    phase_begin(e, PH_EMAP);
    launch_emap(S, io, funded, e->d_io, st);
    phase_end(e, PH_EMAP);
    // the funded proof: account records in order, the per-account check and roll-forward (k_emap
    // summed the need).  (Measured and not kept: the need in a kernel of its own on a side stream
    // beside k_route and the partition -- the epoch was 0.08 ms longer: the phases beside it are
    // bound by the same random accesses.)
    if (funded) {
        phase_begin(e, PH_LEDGER);
        launch_ledger_funded(S, io, st);   // (the per-account check runs in k_route's launch)
        phase_end(e, PH_LEDGER);
    }
    phase_begin(e, PH_ROUTE);
    launch_route(S, io, funded, st);
    phase_end(e, PH_ROUTE);
    if (funded) {
        // list mode: with many groups and none busy in the last epoch (C3) k_segments lists the busy
        // ones and k_match_list takes them over a small grid -- a G-block k_match finding nothing
        // costs ~16 us of the epoch
        const bool lanes_next = S.light_max > 0 && e->last_light != 0;
        const bool list = e->match_list && lanes_next && e->last_busy == 0 && S.G >= 4096;
        phase_begin(e, PH_PART);
        const int buf = launch_partition(S, io, st, list ? S.light_max : -1);
        phase_end(e, PH_PART);
        phase_begin(e, PH_MATCH);
        // light groups one lane each, concurrently with k_match's busy ones (a second stream).  When
        // the last epoch had no busy group both go on the engine stream: the fork / join costs
        // ~30 us per epoch (measured), k_match then only finds empty work (~16 us at C3).
        // Likewise, when the last epoch had no light group (every group busy: the N = 8 shard shape,
        // C2, C5), k_match_lanes is not launched and k_match takes any light group itself.
        const bool lanes = lanes_next;
        const bool fork = lanes && e->last_busy != 0;
        if (fork) {
            HIP_TRY(hipEventRecord(e->ev_fork, st));
            HIP_TRY(hipStreamWaitEvent(e->lane_stream, e->ev_fork, 0));
            launch_match_lanes(S, e->d_S, e->d_io, buf, e->lane_stream);
            HIP_TRY(hipEventRecord(e->ev_join, e->lane_stream));
        } else if (lanes) {
            launch_match_lanes(S, e->d_S, e->d_io, buf, st);
        }
        // two wavefronts per busy group when few groups were busy (a group's record chain, not the
        // CU's issue rate, is then the bound) and the stream is not cancel-heavy
        const bool two = S.fast && e->last_busy > 0 && e->last_busy <= e->two_max && !e->last_cancel_heavy;
        // busy groups sparse in the id space (a symbol shard of a larger universe: 8,277 of 65,537
        // ids at the N = 8 shard of C3): k_match's first blocks take them, from a compact list
        const bool dense = e->dense_grid && e->last_busy > 0 && (uint64_t)e->last_busy * 4 < (uint64_t)S.G;
        // five wavefronts per SIMD for many busy groups and few removes (k_match's WAVES)
        const bool five = !two && e->last_busy > e->two_max && !e->last_cancel_heavy;
        if (list) launch_match_list(e->d_S, e->d_io, buf, st, 0, 1024);
        else launch_match(S, e->d_S, e->d_io, buf, st, lanes ? 0 : 1, two ? 1 : 0, dense ? 1 : 0, five ? 1 : 0);
        if (fork) HIP_TRY(hipStreamWaitEvent(st, e->ev_join, 0));
        phase_end(e, PH_MATCH);
        phase_begin(e, PH_COMPACT);
        launch_compact(S, io, st);
        phase_end(e, PH_COMPACT);
        if (S.fallback) {   // an epoch whose funded proof failed: the serial engine takes it
            phase_begin(e, PH_SERIAL);
            launch_serial(e->d_S, e->d_io, st, 1);
            phase_end(e, PH_SERIAL);
        }
        launch_settle_funded(S, io, st);   // the bounds roll forward (or restart after k_serial)
        if (S.ledger_replay) {
            phase_begin(e, PH_REPLAY);
            if (S.lpar) {
                // the value-key table's tag for this epoch; the table is cleared when the tag wraps
                if (e->lvk_next_tag > 0xFFFFu) {
                    HIP_TRY(hipMemsetAsync(S.lvk, 0, sizeof(ulonglong4) * ((size_t)S.lvk_mask + 1), st));
                    e->lvk_next_tag = 1;
                }
                e->S.lvk_tag = e->lvk_next_tag++;
                launch_ledger_parallel(S, io, e->cfg.max_trades, st);
            }
            // (works only when the parallel pass fell back; the epoch's last launch: it also copies
            // the counters to the slot's host copy)
            launch_ledger_replay(e->d_S, e->d_io, st, e->d_hctr + slot * (size_t)C_NCTR * CTR_STRIDE);
            phase_end(e, PH_REPLAY);
        }
    } else {
        phase_begin(e, PH_SERIAL);
        launch_serial(e->d_S, e->d_io, st);
        phase_end(e, PH_SERIAL);
    }
    // k_table stays in line: beside the compaction on lane_stream both random-access phases slowed
    // each other down to the same sum (measured: compact 0.20 -> 0.28 ms, table 0.09 -> 0.16 ms)
    phase_begin(e, PH_TABLE);
    launch_table(S, io, st);
    phase_end(e, PH_TABLE);
    HIP_TRY(hipGetLastError());
    if (!(funded && S.ledger_replay))   // (otherwise k_ledger_replay, the last launch, copied them)
        HIP_TRY(hipMemcpyAsync(e->h_ctr + slot * (size_t)C_NCTR * CTR_STRIDE, S.ctr, (size_t)C_NCTR * CTR_STRIDE * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipEventRecord(e->ev_end[slot], st));
    e->seq_base += n;
    e->fl_n[slot] = n;
    ++e->sub_count;
    ++e->inflight;
    return KME_OK;
}

kme_status kme_submit_epoch_device(kme_engine* e, const kme_orders* in, uint32_t n, const kme_epoch_result* out) {
    if (!e || !in) return KME_E_INVALID;
    HIP_TRY(hipSetDevice(e->device));
    return submit(e, in, n, out);
}

// Online growth of Balances / Positions (the reference's RocksDB stores grow without bound, KP:30-37;
// H2 leaves stale value-keyed positions forever, KP:283-284, 434-436).  Called between epochs with the
// tables' used slots (live entries + tombstones) after the newest completed epoch: when they plus the
// worst case of `ahead` more epochs could pass half load, the stream is drained and the live entries
// are rehashed (kme_maint.hip) into tables sized for them plus two epochs -- at least twice the old
// size when the live entries are what grew, the same size when tombstones filled the old one.
// *changed: the tables were rebuilt (the callers' copies of the used counters are stale).  A failed
// allocation leaves the tables as they are: the device check (KME_D_CAP_LEDGER) then fires only when
// they are really full, i.e. HBM is exhausted.
static kme_status ledger_reserve(kme_engine* e, uint64_t bal_used, uint64_t pos_used, uint64_t ahead, bool* changed) {
    *changed = false;
    DevState& S = e->S;
    const uint64_t bs = (uint64_t)S.bal_mask + 1, ps = (uint64_t)S.pos_mask + 1;
    const uint64_t bb = bal_bound(e->cfg), pb = pos_bound(e->cfg);
    if (2 * (bal_used + ahead * bb) <= bs && 2 * (pos_used + ahead * pb) <= ps) return KME_OK;
    HIP_TRY(hipStreamSynchronize(e->stream));
    unsigned long long live[2];
    launch_ledger_live(S, e->d_maint, e->stream);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(live, e->d_maint, sizeof live, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    auto target = [](uint64_t slots, uint64_t lv, uint64_t used, uint64_t bound) -> uint64_t {
        const uint64_t need = ledger_slots(lv, bound, 2);
        if (need > slots) return std::max(need, 2 * slots);
        return 2 * (used + 2 * bound) > slots ? slots : 0;   // tombstones: same size; 0 = keep the table
    };
    const uint64_t nb = target(bs, live[0], bal_used, bb), np = target(ps, live[1], pos_used, pb);
    if (nb > (1ull << 31) || np > (1ull << 31)) return KME_OK;   // (the tables' masks are 32-bit: full means full)
    DevState N = S;
    bool alloc_ok = true;
    auto tryalloc = [&](void** p, size_t bytes) {
        if (!alloc_ok) return;
        if (hipMalloc(p, bytes) != hipSuccess) { (void)hipGetLastError(); alloc_ok = false; *p = nullptr; }
    };
    if (nb) {
        tryalloc((void**)&N.bal_state, nb * sizeof(uint32_t));
        tryalloc((void**)&N.bal_key, nb * sizeof(int64_t));
        tryalloc((void**)&N.bal_val, nb * sizeof(int64_t));
        N.bal_mask = (uint32_t)(nb - 1);
    }
    if (np) {
        tryalloc((void**)&N.pos, np * sizeof(PosEntry));
        N.pos_mask = (uint32_t)(np - 1);
    }
    auto free_new = [&] {
        if (nb) { (void)hipFree(N.bal_state); (void)hipFree(N.bal_key); (void)hipFree(N.bal_val); }
        if (np) (void)hipFree(N.pos);
    };
    if (!alloc_ok) {   // out of HBM: free what was taken, keep the old tables
        free_new();
        std::fprintf(stderr, "kme: ledger tables cannot grow (HBM): %llu / %llu slots kept\n", (unsigned long long)bs,
                     (unsigned long long)ps);
        return KME_OK;
    }
    // (until the swap below a failure frees the new tables and leaves the old ones in place)
    unsigned long long fail[2] = {0, 0};
    bool rok = (!nb || hipMemsetAsync(N.bal_state, 0, nb * sizeof(uint32_t), e->stream) == hipSuccess) &&
               (!np || hipMemsetAsync(N.pos, 0, np * sizeof(PosEntry), e->stream) == hipSuccess);
    if (rok) launch_ledger_rehash(N, S, e->d_maint + 2, e->stream);
    rok = rok && hipGetLastError() == hipSuccess &&
          hipMemcpyAsync(fail, e->d_maint + 2, sizeof fail, hipMemcpyDeviceToHost, e->stream) == hipSuccess &&
          hipStreamSynchronize(e->stream) == hipSuccess;
    if (!rok) {
        (void)hipGetLastError();
        free_new();
        return KME_E_HIP;
    }
    if (fail[0] || fail[1]) { free_new(); return KME_E_CAPACITY; }   // (cannot happen: the new tables are at most half full)
    for (auto& a : e->allocs) {   // the new tables take the old ones' places in the allocation list
        if (nb && a == (void*)S.bal_state) a = N.bal_state;
        else if (nb && a == (void*)S.bal_key) a = N.bal_key;
        else if (nb && a == (void*)S.bal_val) a = N.bal_val;
        else if (np && a == (void*)S.pos) a = N.pos;
    }
    if (nb) { HIP_TRY(hipFree(S.bal_state)); HIP_TRY(hipFree(S.bal_key)); HIP_TRY(hipFree(S.bal_val)); }
    if (np) HIP_TRY(hipFree(S.pos));
    S = N;
    // used = live after a rehash (no tombstones)
    const unsigned long long bu = nb ? live[0] : bal_used, pu = np ? live[1] : pos_used;
    HIP_TRY(hipMemcpyAsync(&e->S.ctr[ci(C_BAL_USED)], &bu, sizeof bu, hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipMemcpyAsync(&e->S.ctr[ci(C_POS_USED)], &pu, sizeof pu, hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipMemcpyAsync(e->d_S, &e->S, sizeof(DevState), hipMemcpyHostToDevice, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    for (int s = 0; s < 3; ++s) {   // the counter copies of completed epochs not yet waited for
        e->h_ctr[s * (size_t)C_NCTR * CTR_STRIDE + ci(C_BAL_USED)] = bu;
        e->h_ctr[s * (size_t)C_NCTR * CTR_STRIDE + ci(C_POS_USED)] = pu;
    }
    ++e->ledger_grows;
    *changed = true;
    return KME_OK;
}

kme_status kme_wait(kme_engine* e, kme_epoch_status* st) {
    if (!e) return KME_E_INVALID;
    kme_epoch_status s{};
    s.error_index = -1;
    if (e->inflight == 0) {
        s.status = e->failed ? e->fail_status : KME_OK;
        if (st) *st = s;
        return (kme_status)s.status;
    }
    const int slot = (int)((e->sub_count - (uint32_t)e->inflight) & 1);   // the older epoch in flight
    HIP_TRY(hipEventSynchronize(e->ev_end[slot]));
    --e->inflight;
    const uint32_t last_n = e->fl_n[slot];
    bool host_overflow = false;
    if (e->host_epoch[slot]) {   // kme_submit_epoch_host: its results have landed in the caller's buffers
        e->host_epoch[slot] = false;
        const kme_epoch_result& ho = e->host_out[slot];
        const uint32_t nt = ho.trade_off[last_n];
        host_overflow = nt > ho.trades_cap;
        if (!e->host_mapped[slot] && nt && !host_overflow)   // trades buffer not registered: copy them now
            HIP_TRY(hipMemcpy(ho.trades, e->hs[slot].trades, (size_t)nt * sizeof(kme_trade), hipMemcpyDeviceToHost));
    }
    const unsigned long long* c = e->h_ctr + slot * (size_t)C_NCTR * CTR_STRIDE;
    s.n_inputs = last_n;
    s.n_trades = (uint32_t)c[ci(C_TRADES)];
    s.n_orders = c[ci(C_ORDERS)];
    s.n_rests = c[ci(C_RESTS)];
    s.n_maker_visits = c[ci(C_TRADES)];               // every maker visit is one trade (KP:238-242)
    s.n_cancel_ok = c[ci(C_CANCEL_OK)];
    s.serial_fallback = c[ci(C_FALLBACK)] ? 1u : 0u;
    s.ledger_repaired = (uint32_t)c[ci(C_LREPAIRED)];
    s.ledger_serial = c[ci(C_LSERIAL)] ? 1u : 0u;
    s.n_effective = last_n;
    e->last_busy = c[ci(C_BUSY)];
    e->last_light = c[ci(C_LIGHT)];
    e->last_cancel_heavy = c[ci(C_CANCEL_OK)] * 8 > (uint64_t)last_n;
    if (host_overflow && c[ci(C_ERR)] == ~0ull) {
        // (cannot happen: kme_submit_epoch_host takes only trades buffers of max_trades records, and the
        // device never produces more; reported, the engine stays usable)
        s.status = KME_E_CAPACITY; s.detail = KME_D_CAP_TRADES; s.n_effective = 0;
    } else if (c[ci(C_ERR)] != ~0ull) {
        s.status = (int32_t)(c[ci(C_ERR)] & 0xFF);
        s.detail = (int32_t)((c[ci(C_ERR)] >> 8) & 0xFF);
        const uint64_t ix = c[ci(C_ERR)] >> 16;
        // (KME_D_UNPROVEN: the funded proof refused the epoch as a whole, raised at index 0 so that
        // no indexed fault replaces it; reported without an index)
        s.error_index = (ix == 0xFFFFFFFFFFFFull || s.detail == KME_D_UNPROVEN) ? -1 : (int64_t)ix;
        // the records before the fault took effect (their results are valid), none after it
        s.n_effective = s.error_index < 0 ? 0u : (uint32_t)std::min<int64_t>(s.error_index, last_n);
        if (s.detail == KME_D_UNPROVEN) s.n_effective = 0;
        if (s.status == KME_E_UNFUNDED && e->inflight == 0) {
            // not fatal: the refused records changed nothing, so their sequence numbers are
            // handed out again when they are resubmitted
            e->seq_base -= (int64_t)(last_n - s.n_effective);
        } else {
            // (an UNFUNDED epoch with a later one already in flight: that one ran without the refused
            // records, out of the caller's order -- the engine fails)
            e->failed = 1;
            e->fail_status = s.status;
            e->fail_detail = s.detail;
        }
    }
    if (e->timing) {
        for (int p = 0; p < PH_N; ++p) {
            e->phase_ms[p] = 0.f;
            if (e->ev_used[slot][p]) (void)hipEventElapsedTime(&e->phase_ms[p], e->ev[slot][2 * p], e->ev[slot][2 * p + 1]);
        }
    }
    // oid table maintenance: stale (lazily deleted) entries are dropped by a rebuild, early enough
    // that the epoch still in flight and the next one fit (each adds at most max_epoch entries).
    // The rebuild drains the stream first (the in-flight epoch finishes; its counters are already
    // copied) and reports through its own counter, not the per-epoch error word.
    if (!e->failed && (c[ci(C_OTAB_USED)] + (uint64_t)(1 + e->inflight) * e->cfg.max_epoch) * 2 > e->otab_cap) {
        HIP_TRY(hipStreamSynchronize(e->stream));
        // the pool slots to scan: the newest bump (the in-flight epoch's copy, complete after the drain)
        const unsigned long long* latest = e->inflight ? e->h_ctr + (slot ^ 1) * (size_t)C_NCTR * CTR_STRIDE : c;
        launch_otab_rebuild(e->S, (uint32_t)std::min<uint64_t>(latest[ci(C_POOL_BUMP)], e->S.pool_cap), e->stream);
        HIP_TRY(hipGetLastError());
        unsigned long long* rc = e->h_ctr + 2 * (size_t)C_NCTR * CTR_STRIDE;
        HIP_TRY(hipMemcpyAsync(rc, e->S.ctr, (size_t)C_NCTR * CTR_STRIDE * sizeof(unsigned long long), hipMemcpyDeviceToHost, e->stream));
        HIP_TRY(hipStreamSynchronize(e->stream));
        if (rc[ci(C_REBUILD_FAIL)] != 0 || rc[ci(C_OTAB_USED)] * 4 > e->otab_cap * 3) {
            e->failed = 1; e->fail_status = KME_E_CAPACITY; e->fail_detail = KME_D_CAP_OIDTAB;
        }
    }
    // the ledger tables: room for the epochs in flight and the next one (the newest counters known:
    // an epoch still in flight adds at most one epoch's bound on top of these)
    if (!e->failed && e->ledger) {
        bool changed = false;
        const kme_status r = ledger_reserve(e, c[ci(C_BAL_USED)], c[ci(C_POS_USED)], (uint64_t)1 + e->inflight, &changed);
        if (r != KME_OK) { e->failed = 1; e->fail_status = r; e->fail_detail = KME_D_CAP_LEDGER; }
    }
    if (st) *st = s;
    return (kme_status)s.status;
}

kme_status kme_poll(kme_engine* e, int* done) {
    if (!e || !done) return KME_E_INVALID;
    if (e->inflight == 0) { *done = 1; return KME_OK; }
    const int slot = (int)((e->sub_count - (uint32_t)e->inflight) & 1);   // the older epoch in flight
    const hipError_t q = hipEventQuery(e->ev_end[slot]);
    if (q == hipSuccess) { *done = 1; return KME_OK; }
    if (q == hipErrorNotReady) { (void)hipGetLastError(); *done = 0; return KME_OK; }
    return KME_E_HIP;
}

// Registration pins whole pages, so two buffers that share a page cannot be registered and
// unregistered independently: the engine keeps the exact ranges it registered, counts repeats of the
// same range, and refuses a range that shares a page with a different one (KME_E_INVALID; callers
// allocate page-aligned buffers -- the JNI glue allocates the processor's buffers itself).
kme_status kme_host_register(kme_engine* e, void* host, size_t bytes) {
    if (!e || !host || !bytes) return KME_E_INVALID;
    const uintptr_t p = (uintptr_t)host, pg = 4096;
    const uintptr_t lo = p & ~(pg - 1), hi = (p + bytes + pg - 1) & ~(pg - 1);
    for (auto& r : e->host_regs) {
        if (r.p == p && r.bytes == bytes) { ++r.refs; return KME_OK; }
        const uintptr_t rlo = r.p & ~(pg - 1), rhi = (r.p + r.bytes + pg - 1) & ~(pg - 1);
        if (lo < rhi && rlo < hi) return KME_E_INVALID;   // shares a page with another registered range
    }
    HIP_TRY(hipSetDevice(e->device));
    const hipError_t r = hipHostRegister(host, bytes, hipHostRegisterMapped | hipHostRegisterPortable);
    bool owned = true;
    if (r == hipErrorHostMemoryAlreadyRegistered) {   // registered by its owner elsewhere: used, never undone here
        (void)hipGetLastError();
        owned = false;
    } else {
        HIP_TRY(r);
    }
    e->host_regs.push_back({p, bytes, 1, owned});
    return KME_OK;
}

kme_status kme_host_unregister(kme_engine* e, void* host) {
    if (!e || !host) return KME_E_INVALID;
    if (e->inflight) return KME_E_INVALID;
    for (size_t k = 0; k < e->host_regs.size(); ++k) {
        auto& r = e->host_regs[k];
        if (r.p != (uintptr_t)host) continue;
        if (--r.refs > 0) return KME_OK;
        const bool owned = r.owned;
        e->host_regs.erase(e->host_regs.begin() + (long)k);
        if (owned) {
            HIP_TRY(hipSetDevice(e->device));
            HIP_TRY(hipHostUnregister(host));
        }
        return KME_OK;
    }
    return KME_E_INVALID;   // not registered through this engine
}

static kme_status host_slots(kme_engine* e) {
    if (e->hs_ready) return KME_OK;
    HIP_TRY(hipStreamCreateWithFlags(&e->in_stream, hipStreamNonBlocking));
    HIP_TRY(hipStreamCreateWithFlags(&e->out_stream, hipStreamNonBlocking));
    for (auto& ev : e->ev_in) HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    const size_t E = e->cfg.max_epoch;
    for (auto& h : e->hs) {
        kme_status r = KME_OK;
        if ((r = dalloc(e, &h.action, E)) || (r = dalloc(e, &h.price, E)) || (r = dalloc(e, &h.size, E)) ||
            (r = dalloc(e, &h.oid, E)) || (r = dalloc(e, &h.aid, E)) || (r = dalloc(e, &h.sid, E)) ||
            (r = dalloc(e, &h.out_action, E)) || (r = dalloc(e, &h.out_size, E)) || (r = dalloc(e, &h.out_prev, E)) ||
            (r = dalloc(e, &h.out_flags, E)) || (r = dalloc(e, &h.trade_off, E + 1)) ||
            (r = dalloc(e, &h.trades, (size_t)e->cfg.max_trades)))
            return r;
    }
    e->hs_ready = true;
    return KME_OK;
}

kme_status kme_submit_epoch_host(kme_engine* e, const kme_orders* in, uint32_t n, const kme_epoch_result* out) {
    if (!e || !in || !out || !out->out_action || !out->out_size || !out->out_prev || !out->out_flags || !out->trade_off ||
        !out->trades)
        return KME_E_INVALID;
    // the caller's trades buffer must hold an epoch's worth (max_trades): a smaller one could not take
    // the results of an epoch the device has already committed
    if (out->trades_cap < e->cfg.max_trades) return KME_E_INVALID;
    if (e->failed) return KME_E_FAILED;
    if (n > e->cfg.max_epoch) return KME_E_CAPACITY;
    if (e->inflight == 2) return KME_E_INVALID;
    HIP_TRY(hipSetDevice(e->device));
    if (kme_status r = host_slots(e)) return r;
    const int slot = (int)(e->sub_count & 1);   // = submit()'s slot
    const auto& h = e->hs[slot];
    hipStream_t si = e->in_stream, so = e->out_stream;
    // inputs: PCIe while the engine stream still runs the previous epoch's kernels
    if (n) {
        HIP_TRY(hipMemcpyAsync(h.action, in->action, n * sizeof(int32_t), hipMemcpyHostToDevice, si));
        HIP_TRY(hipMemcpyAsync(h.oid, in->oid, n * sizeof(int64_t), hipMemcpyHostToDevice, si));
        HIP_TRY(hipMemcpyAsync(h.aid, in->aid, n * sizeof(int64_t), hipMemcpyHostToDevice, si));
        HIP_TRY(hipMemcpyAsync(h.sid, in->sid, n * sizeof(int64_t), hipMemcpyHostToDevice, si));
        HIP_TRY(hipMemcpyAsync(h.price, in->price, n * sizeof(int32_t), hipMemcpyHostToDevice, si));
        HIP_TRY(hipMemcpyAsync(h.size, in->size, n * sizeof(int32_t), hipMemcpyHostToDevice, si));
    }
    HIP_TRY(hipEventRecord(e->ev_in[slot], si));
    HIP_TRY(hipStreamWaitEvent(e->stream, e->ev_in[slot], 0));
    const kme_orders din{h.action, h.oid, h.aid, h.sid, h.price, h.size};
    const kme_epoch_result dres{h.out_action, h.out_size, h.out_prev, h.out_flags, h.trade_off,
                                reinterpret_cast<kme_trade*>(h.trades), e->cfg.max_trades};
    if (kme_status r = submit(e, &din, n, &dres)) return r;
    // results: behind the kernels (ev_end of this slot), on the other copy stream
    HIP_TRY(hipStreamWaitEvent(so, e->ev_end[slot], 0));
    if (n) {
        HIP_TRY(hipMemcpyAsync(out->out_action, h.out_action, n * sizeof(int32_t), hipMemcpyDeviceToHost, so));
        HIP_TRY(hipMemcpyAsync(out->out_size, h.out_size, n * sizeof(int32_t), hipMemcpyDeviceToHost, so));
        HIP_TRY(hipMemcpyAsync(out->out_prev, h.out_prev, n * sizeof(int64_t), hipMemcpyDeviceToHost, so));
        HIP_TRY(hipMemcpyAsync(out->out_flags, h.out_flags, n * sizeof(uint8_t), hipMemcpyDeviceToHost, so));
    }
    HIP_TRY(hipMemcpyAsync(out->trade_off, h.trade_off, (n + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost, so));
    void* mapped = nullptr;
    e->host_mapped[slot] = out->trades_cap && hipHostGetDevicePointer(&mapped, out->trades, 0) == hipSuccess && mapped;
    if (!e->host_mapped[slot]) (void)hipGetLastError();
    else launch_export_trades(h.trades, h.trade_off + n, out->trades_cap, reinterpret_cast<TradeRec*>(mapped), so);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(e->ev_end[slot], so));   // kme_poll / kme_wait: the results have landed
    e->host_epoch[slot] = true;
    e->host_out[slot] = *out;
    return KME_OK;
}

// ------------------------------------------------------------------ multi-GPU: RCCL
namespace {
// RCCL through dlopen: libkme has no link-time dependency on it.  The copy is chosen explicitly
// (kme_rccl_load: a process that already loaded an RCCL -- torch's -- hands its path, so that one RCCL
// serves both); a kme_comm_* call before that loads the default (env KME_RCCL_LIB, else
// librccl.so.1).  Every RCCL failure is kept as text (kme_rccl_last_error) and printed.
struct Rccl {
    void* h = nullptr;
    std::string path;
    decltype(&ncclGetUniqueId) get_id = nullptr;
    decltype(&ncclCommInitRank) init = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclAllGather) allgather = nullptr;
    decltype(&ncclGetErrorString) err_str = nullptr;
    decltype(&ncclGetLastError) last_err = nullptr;
};
Rccl g_rccl;
std::string g_rccl_error;
kme_status rccl_open(const char* path) {
    Rccl& r = g_rccl;
    const std::string want = path && *path ? path : "librccl.so.1";
    if (r.h) return r.path == want ? KME_OK : KME_E_INVALID;
    void* h = dlopen(want.c_str(), RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
        g_rccl_error = std::string("dlopen ") + want + ": " + dlerror();
        std::fprintf(stderr, "kme: RCCL not available (%s)\n", g_rccl_error.c_str());
        return KME_E_UNSUPPORTED;
    }
    r.get_id = (decltype(r.get_id))dlsym(h, "ncclGetUniqueId");
    r.init = (decltype(r.init))dlsym(h, "ncclCommInitRank");
    r.destroy = (decltype(r.destroy))dlsym(h, "ncclCommDestroy");
    r.allgather = (decltype(r.allgather))dlsym(h, "ncclAllGather");
    r.err_str = (decltype(r.err_str))dlsym(h, "ncclGetErrorString");
    r.last_err = (decltype(r.last_err))dlsym(h, "ncclGetLastError");
    if (!r.get_id || !r.init || !r.destroy || !r.allgather) {
        g_rccl_error = want + ": missing symbols";
        std::fprintf(stderr, "kme: RCCL not available (%s)\n", g_rccl_error.c_str());
        dlclose(h);
        r = Rccl{};
        return KME_E_UNSUPPORTED;
    }
    r.h = h;
    r.path = want;
    return KME_OK;
}
Rccl* rccl() {
    if (!g_rccl.h) {
        const char* env = std::getenv("KME_RCCL_LIB");
        if (rccl_open(env) != KME_OK) return nullptr;
    }
    return &g_rccl;
}
// an RCCL call's result: OK, or KME_E_HIP with the library's own account of it kept and printed
kme_status rccl_check(ncclResult_t res, const char* what, ncclComm_t comm) {
    if (res == ncclSuccess) return KME_OK;
    const Rccl& r = g_rccl;
    g_rccl_error = std::string(what) + ": " + (r.err_str ? r.err_str(res) : "rccl error") + " (ncclResult_t " +
                   std::to_string((int)res) + ")";
    const char* last = r.last_err ? r.last_err(comm) : nullptr;
    if (last && *last) g_rccl_error += std::string("; ") + last;
    std::fprintf(stderr, "kme: %s\n", g_rccl_error.c_str());
    return KME_E_HIP;
}
}  // namespace

struct kme_comm {
    ncclComm_t comm = nullptr;
    uint32_t n = 0, rank = 0;
    int device = 0;
    int64_t* d_credit = nullptr;     // kme_credit_rebalance: n blocks of (bound, demand) x accounts + a status word
    int64_t* h_status = nullptr;     // pinned: the ranks' status words (+ this rank's outgoing one)
    size_t credit_accounts = 0;
};

kme_status kme_rccl_load(const char* path) { return rccl_open(path); }
const char* kme_rccl_last_error(void) { return g_rccl_error.c_str(); }

kme_status kme_comm_unique_id(void* id128) {
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId");
    if (!id128) return KME_E_INVALID;
    Rccl* r = rccl();
    if (!r) return KME_E_UNSUPPORTED;
    ncclUniqueId id;
    if (kme_status s = rccl_check(r->get_id(&id), "ncclGetUniqueId", nullptr)) return s;
    std::memcpy(id128, &id, sizeof id);
    return KME_OK;
}

kme_status kme_comm_init(kme_engine* e, uint32_t n_ranks, uint32_t rank, const void* id128, kme_comm** out) {
    if (!e || !id128 || !out || n_ranks == 0 || rank >= n_ranks) return KME_E_INVALID;
    Rccl* r = rccl();
    if (!r) return KME_E_UNSUPPORTED;
    HIP_TRY(hipSetDevice(e->device));
    ncclUniqueId id;
    std::memcpy(&id, id128, sizeof id);
    kme_comm* c = new kme_comm();
    c->n = n_ranks; c->rank = rank; c->device = e->device;
    if (kme_status s = rccl_check(r->init(&c->comm, (int)n_ranks, id, (int)rank), "ncclCommInitRank", nullptr)) {
        delete c;
        return s;
    }
    *out = c;
    return KME_OK;
}

kme_status kme_comm_destroy(kme_comm* c) {
    if (!c) return KME_E_INVALID;
    Rccl* r = rccl();
    (void)hipSetDevice(c->device);
    if (c->d_credit) (void)hipFree(c->d_credit);
    if (c->h_status) (void)hipHostFree(c->h_status);
    if (r && c->comm) r->destroy(c->comm);
    delete c;
    return KME_OK;
}

kme_status kme_market_data_allgather(kme_engine* e, kme_comm* c, const uint32_t* dev_groups, uint32_t n_groups,
                                     uint32_t rows_per_rank, kme_tob* dev_all) {
    if (!e || !c || !dev_all || n_groups > rows_per_rank || (n_groups && !dev_groups)) return KME_E_INVALID;
    Rccl* r = rccl();
    if (!r) return KME_E_UNSUPPORTED;
    HIP_TRY(hipSetDevice(e->device));
    kme_tob* mine = dev_all + (size_t)c->rank * rows_per_rank;
    launch_tob_groups(e->S, dev_groups, n_groups, mine, e->stream, rows_per_rank);
    HIP_TRY(hipGetLastError());
    if (kme_status s = rccl_check(r->allgather(mine, dev_all, (size_t)rows_per_rank * sizeof(kme_tob), ncclUint8, c->comm, e->stream),
                                  "ncclAllGather (market data)", c->comm))
        return s;
    return KME_OK;
}

kme_status kme_credit_state(kme_engine* e, int64_t* dev_out) {
    if (!e || !dev_out || e->cfg.mode != KME_MODE_FUNDED) return KME_E_INVALID;
    if (e->inflight) return KME_E_INVALID;
    HIP_TRY(hipSetDevice(e->device));
    launch_credit_state(e->S, dev_out, e->stream);
    HIP_TRY(hipGetLastError());
    // complete on return, like kme_credit_adjust: the caller reads dev_out on a stream of its own
    // (a torch stream, a transport's), which nothing orders after the engine stream
    HIP_TRY(hipStreamSynchronize(e->stream));
    return KME_OK;
}

kme_status kme_credit_adjust(kme_engine* e, const int64_t* dev_all, uint32_t n_shards, uint32_t my_shard) {
    if (!e || !dev_all || e->cfg.mode != KME_MODE_FUNDED || n_shards == 0 || my_shard >= n_shards) return KME_E_INVALID;
    if (e->inflight) return KME_E_INVALID;
    if (e->failed) return KME_E_FAILED;
    HIP_TRY(hipSetDevice(e->device));
    launch_credit_adjust(e->S, dev_all, n_shards, my_shard, 2 * (size_t)e->cfg.max_accounts, e->stream);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(e->stream));
    return KME_OK;
}

// A collective: every rank takes part in the all-gather whatever its own state, so no rank waits
// for a peer that returned early.  Each rank's block is (bound, demand) per account plus a status
// word; a rank that cannot re-split (an epoch in flight, a failed engine) sends zeros and its status,
// and when any status is not OK no rank adjusts: that rank returns its own status, the others
// KME_E_INVALID ("skipped on every rank").
kme_status kme_credit_rebalance(kme_engine* e, kme_comm* c) {
    if (!e || !c || e->cfg.mode != KME_MODE_FUNDED) return KME_E_INVALID;
    Rccl* r = rccl();
    if (!r) return KME_E_UNSUPPORTED;   // (a communicator exists only where RCCL loaded: the same on every rank)
    HIP_TRY(hipSetDevice(e->device));
    const size_t A = e->cfg.max_accounts, stride = 2 * A + 1;
    if (!c->d_credit || c->credit_accounts != A) {
        if (c->d_credit) HIP_TRY(hipFree(c->d_credit));
        if (c->h_status) HIP_TRY(hipHostFree(c->h_status));
        c->d_credit = nullptr;
        c->h_status = nullptr;
        HIP_TRY(hipMalloc((void**)&c->d_credit, (size_t)c->n * stride * sizeof(int64_t)));
        HIP_TRY(hipHostMalloc((void**)&c->h_status, ((size_t)c->n + 1) * sizeof(int64_t), hipHostMallocDefault));
        c->credit_accounts = A;
    }
    const int64_t mine_st = e->failed ? KME_E_FAILED : e->inflight ? KME_E_INVALID : KME_OK;
    int64_t* mine = c->d_credit + (size_t)c->rank * stride;
    c->h_status[c->n] = mine_st;
    if (mine_st == KME_OK) launch_credit_state(e->S, mine, e->stream);
    else HIP_TRY(hipMemsetAsync(mine, 0, 2 * A * sizeof(int64_t), e->stream));
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(mine + 2 * A, &c->h_status[c->n], sizeof(int64_t), hipMemcpyHostToDevice, e->stream));
    if (kme_status s = rccl_check(r->allgather(mine, c->d_credit, stride * sizeof(int64_t), ncclUint8, c->comm, e->stream),
                                  "ncclAllGather (credit)", c->comm))
        return s;
    HIP_TRY(hipMemcpy2DAsync(c->h_status, sizeof(int64_t), c->d_credit + 2 * A, stride * sizeof(int64_t), sizeof(int64_t),
                             c->n, hipMemcpyDeviceToHost, e->stream));
    HIP_TRY(hipStreamSynchronize(e->stream));
    bool all_ok = true;
    for (uint32_t k = 0; k < c->n; ++k) all_ok = all_ok && c->h_status[k] == KME_OK;
    if (!all_ok) return mine_st != KME_OK ? (kme_status)mine_st : KME_E_INVALID;
    launch_credit_adjust(e->S, c->d_credit, c->n, c->rank, stride, e->stream);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(e->stream));
    return KME_OK;
}

}  // extern "C"

// ------------------------------------------------------------------ internals for kme_multi (kme_internal.h)
namespace kme {
hipStream_t engine_stream(kme_engine* e) { return e->stream; }
int engine_device(kme_engine* e) { return e->device; }
const kme_config& engine_config(kme_engine* e) { return e->cfg; }
kme_status credit_state_enqueue(kme_engine* e, int64_t* dev_out) {
    HIP_TRY(hipSetDevice(e->device));
    launch_credit_state(e->S, dev_out, e->stream);
    HIP_TRY(hipGetLastError());
    // complete on return, like kme_credit_adjust: the caller reads dev_out on a stream of its own
    // (a torch stream, a transport's), which nothing orders after the engine stream
    HIP_TRY(hipStreamSynchronize(e->stream));
    return KME_OK;
}
kme_status credit_adjust_enqueue(kme_engine* e, const int64_t* dev_all, uint32_t n, uint32_t me, size_t stride) {
    HIP_TRY(hipSetDevice(e->device));
    launch_credit_adjust(e->S, dev_all, n, me, stride, e->stream);
    HIP_TRY(hipGetLastError());
    return KME_OK;
}
kme_status resting_oids(kme_engine* e, std::vector<int64_t>& out) {
    if (e->inflight) return KME_E_INVALID;
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipStreamSynchronize(e->stream));
    unsigned long long ctr[C_NCTR * CTR_STRIDE];
    HIP_TRY(hipMemcpy(ctr, e->S.ctr, sizeof ctr, hipMemcpyDeviceToHost));
    const uint64_t nslots = std::min<uint64_t>(ctr[ci(C_POOL_BUMP)], e->S.pool_cap);
    std::vector<Node> pool(nslots);
    if (nslots) HIP_TRY(hipMemcpy(pool.data(), e->S.pool, nslots * sizeof(Node), hipMemcpyDeviceToHost));
    out.clear();
    for (const Node& nd : pool)
        if (nd.live) out.push_back(nd.oid);
    return KME_OK;
}
}  // namespace kme

extern "C" {
#ifndef KME_SRC_HASH
#define KME_SRC_HASH "unknown"
#endif
const char* kme_build_id(void) { return KME_SRC_HASH; }

// ------------------------------------------------------------------ persistence
// Format 4: header, then the stores in their compact form -- group states (the dense groups, then the
// sparse ones), the FUNDED reservation ledger, the used prefix of the node pool, the set price levels
// (kme_maint.hip), the live Balances and Positions entries, the sparse symbols' ids -- then the
// application record, then the trailer (size of that record and the digest of everything before it;
// kme_internal.h).  The oid table is not stored: a restore rebuilds it from the resting orders (an
// entry of an order that no longer rests is only ever a stale fact), and the ledger
// tables are rebuilt at the size their live entries need.
// Format 3 (ABI 6, no sparse symbols) is still read: the same stores without the sparse groups and
// ids, under a header whose kme_config lacks max_sparse_symbols; they restore as empty.
namespace {
constexpr char kCkptMagic3[8] = {'K', 'M', 'E', 'C', 'K', 'P', 'T', '3'};
constexpr char kCkptMagic4[8] = {'K', 'M', 'E', 'C', 'K', 'P', 'T', '4'};
struct kme_config_v6 {   // kme_config of ABI 6 (format-3 headers)
    uint32_t abi_version, mode, max_symbols, max_accounts, max_epoch, max_trades;
    uint64_t max_resting, ledger_capacity;
    int32_t device;
    uint32_t credit_shards, flags;
    int32_t light_max;
};
static_assert(sizeof(kme_config_v6) == 56, "ABI-6 kme_config");
struct CkptHeader3 {
    char magic[8];
    kme_config_v6 cfg;
    int64_t seq_base;
    uint64_t pool_used, n_levels, bal_live, pos_live, app_bytes;
    uint64_t _reserved[3];
};
struct CkptHeader4 {
    char magic[8];
    kme_config cfg;
    int64_t seq_base;
    uint64_t pool_used, n_levels, bal_live, pos_live, app_bytes;
    uint64_t n_sparse;                 // sparse groups (their GroupStates and ids are in the file)
    uint64_t _reserved[3];
};

}  // namespace
}  // extern "C"

namespace kme {
bool sync_dir_of(const std::string& path) {
    const size_t slash = path.find_last_of('/');
    const std::string dir = slash == std::string::npos ? std::string(".") : (slash == 0 ? std::string("/") : path.substr(0, slash));
    const int fd = open(dir.c_str(), O_RDONLY | O_DIRECTORY);
    if (fd < 0) return false;
    const bool r = fsync(fd) == 0;
    close(fd);
    return r;
}
}  // namespace kme

extern "C" {

kme_status kme_checkpoint_inspect(const char* path, kme_checkpoint_info* out) {
    if (!path || !out) return KME_E_INVALID;
    *out = kme_checkpoint_info{};
    FILE* f = std::fopen(path, "rb");
    if (!f) return KME_E_INVALID;
    kme::CkptTrailer t{};
    bool ok = std::fseek(f, 0, SEEK_END) == 0;
    const long sz = ok ? std::ftell(f) : -1;
    ok = ok && sz >= (long)sizeof t && std::fseek(f, sz - (long)sizeof t, SEEK_SET) == 0 && std::fread(&t, sizeof t, 1, f) == 1 &&
         (std::memcmp(t.magic, kme::kTrailerMagic, sizeof t.magic) == 0 || std::memcmp(t.magic, kme::kTrailerMagic2, sizeof t.magic) == 0);
    std::fclose(f);
    if (!ok) return KME_E_INVALID;
    out->file_bytes = (uint64_t)sz;
    out->app_bytes = t.app_bytes;
    out->digest = t.digest;
    return KME_OK;
}

kme_status kme_checkpoint_app(kme_engine* e, const char* path, const void* app, size_t app_bytes) {
    if (!e || !path || (app_bytes && !app)) return KME_E_INVALID;
    if (e->failed) return KME_E_FAILED;
    if (e->inflight) return KME_E_INVALID;   // between epochs only: kme_wait the submitted epoch first
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipStreamSynchronize(e->stream));
    const DevState& S = e->S;
    unsigned long long ctr[C_NCTR * CTR_STRIDE];
    HIP_TRY(hipMemcpy(ctr, S.ctr, sizeof ctr, hipMemcpyDeviceToHost));
    // the last epoch faulted: its state is not a checkpoint (an epoch refused with KME_E_UNFUNDED
    // changed nothing: the engine's state is the one before it)
    if (ctr[ci(C_ERR)] != ~0ull && (ctr[ci(C_ERR)] & 0xFF) != KME_E_UNFUNDED) return KME_E_FAILED;
    const size_t G = e->cfg.max_symbols, Gs = (size_t)S.Gs, A = e->cfg.max_accounts;
    const bool funded = e->cfg.mode == KME_MODE_FUNDED;
    // (diagnostics: env KME_CKPT_TRACE=1 prints the phases' wall-clock ms on stderr)
    static const bool trace = std::getenv("KME_CKPT_TRACE") && std::atoi(std::getenv("KME_CKPT_TRACE"));
    const auto t_start = std::chrono::steady_clock::now();
    double t_compact = 0, t_stores = 0;
    auto ms_since = [](std::chrono::steady_clock::time_point t) {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
    };
    CkptHeader4 h{};
    std::memcpy(h.magic, kCkptMagic4, sizeof h.magic);
    h.cfg = e->cfg;
    h.seq_base = e->seq_base;
    h.pool_used = std::min<uint64_t>(ctr[ci(C_POOL_BUMP)], S.pool_cap);
    h.app_bytes = app_bytes;
    h.n_sparse = Gs;
    // the compact stores on the device first: the set levels (counted from the group bitmaps) and
    // the live ledger entries (counted by k_ledger_live), into scratch of exactly that size
    std::vector<GroupState> grp(G + Gs);
    if (!staged_d2h(e, grp.data(), S.grp, (G + Gs) * sizeof(GroupState), "groups")) return KME_E_HIP;
    uint64_t nlev = 0;
    for (const GroupState& gs : grp)
        nlev += (uint64_t)(__builtin_popcountll(gs.bm0_lsb) + __builtin_popcountll(gs.bm0_msb) + __builtin_popcountll(gs.bm1_lsb) +
                           __builtin_popcountll(gs.bm1_msb));
    unsigned long long live[2] = {0, 0}, cnt[3] = {0, 0, 0};
    if (e->ledger) {
        launch_ledger_live(S, e->d_maint, e->stream);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(live, e->d_maint, sizeof live, hipMemcpyDeviceToHost, e->stream));
        HIP_TRY(hipStreamSynchronize(e->stream));
    }
    // what went wrong, if anything: scratch allocation (KME_E_CAPACITY), the device (KME_E_HIP), or
    // the file (KME_E_INVALID)
    kme_status why = KME_OK;
    Level* d_lev = nullptr;
    void *d_bal = nullptr, *d_pos = nullptr;
    bool ok = hipMalloc((void**)&d_lev, std::max<uint64_t>(nlev, 1) * sizeof(Level)) == hipSuccess &&
              hipMalloc(&d_bal, std::max<uint64_t>(live[0], 1) * 16) == hipSuccess &&
              hipMalloc(&d_pos, std::max<uint64_t>(live[1], 1) * 32) == hipSuccess;
    if (!ok) why = KME_E_CAPACITY;
    if (ok) {
        launch_ckpt_levels(S, d_lev, e->d_maint, e->stream);
        if (e->ledger) launch_ckpt_ledger(S, d_bal, d_pos, e->d_maint + 1, e->stream);
        ok = hipGetLastError() == hipSuccess &&
             hipMemcpyAsync(cnt, e->d_maint, 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost, e->stream) == hipSuccess &&
             hipStreamSynchronize(e->stream) == hipSuccess;
        if (!e->ledger) cnt[1] = cnt[2] = 0;
        ok = ok && cnt[0] == nlev && cnt[1] == live[0] && cnt[2] == live[1];
        if (!ok) why = KME_E_HIP;
    }
    (void)hipGetLastError();
    t_compact = ms_since(t_start);
    h.n_levels = cnt[0];
    h.bal_live = cnt[1];
    h.pos_live = cnt[2];
    if (ok) {
        // the file in slots: device stores by stream-ordered copies into the engine's pinned ring,
        // hashed and written by host threads while the next slot fills (kme_ckpt.cpp)
        if (!e->ring.init(e->device)) { ok = false; why = KME_E_CAPACITY; }
        kme::CkptWriter w(path, &e->ring, e->stream);
        auto fail_of = [&]() { return std::strcmp(w.error(), "device read") == 0 ? KME_E_HIP : KME_E_INVALID; };
        auto put = [&](const void* dev, size_t n, const char* what) {
            if (ok && !w.write_dev(dev, n)) {
                ok = false;
                why = fail_of();
                std::fprintf(stderr, "kme_checkpoint: %s of %s (%zu bytes) failed\n", w.error(), what, n);
            }
        };
        auto write = [&](const void* p, size_t n) {
            if (ok && !w.write(p, n)) { ok = false; why = fail_of(); }
        };
        write(&h, sizeof h);
        // the stores of fixed size or growing only at their end first (group states, FUNDED accounts,
        // the pool prefix), then the compacted ones: unchanged state keeps its file offsets from one
        // checkpoint to the next, so a changelog of fixed-size chunks carries only what changed
        // 
        write(grp.data(), (G + Gs) * sizeof(GroupState));
        if (funded) {
            put(S.acct_since, A * sizeof(int64_t), "accounts");
            put(S.acct_lb, A * sizeof(int64_t), "accounts");
            put(S.acct_demand, A * sizeof(int64_t), "accounts");
        }
        put(S.pool, h.pool_used * sizeof(Node), "pool");
        put(d_lev, h.n_levels * sizeof(Level), "levels");
        if (e->ledger) {
            put(d_bal, h.bal_live * 16, "Balances");
            put(d_pos, h.pos_live * 32, "Positions");
        }
        if (Gs) put(S.gsid, Gs * sizeof(int64_t), "sparse symbols");
        write(app, app_bytes);
        t_stores = ms_since(t_start);
        if (ok && !w.commit(app_bytes, nullptr)) { ok = false; why = fail_of(); }
    }
    if (trace)
        std::fprintf(stderr, "kme_checkpoint: compaction %.2f ms, stores (D2H, digest, write) %.2f ms, commit (fsync, rename) %.2f ms, "
                             "%llu bytes\n", t_compact, t_stores - t_compact, ms_since(t_start) - t_stores,
                     (unsigned long long)(sizeof h + (G + Gs) * sizeof(GroupState) + h.pool_used * sizeof(Node)));
    (void)hipFree(d_lev);
    if (d_bal) (void)hipFree(d_bal);
    if (d_pos) (void)hipFree(d_pos);
    return ok ? KME_OK : why;
}

kme_status kme_checkpoint(kme_engine* e, const char* path) { return kme_checkpoint_app(e, path, nullptr, 0); }

kme_status kme_restore_app(kme_engine* e, const char* path, void* app, size_t app_cap, size_t* app_bytes) {
    if (!e || !path) return KME_E_INVALID;
    if (e->failed) return KME_E_FAILED;
    if (e->inflight) return KME_E_INVALID;
    if (app_bytes) *app_bytes = 0;
    HIP_TRY(hipSetDevice(e->device));
    kme::CkptReader r(path);
    // the header: format 4, or format 3 (an ABI-6 kme_config, no sparse symbols)
    CkptHeader4 h{};
    char magic[8];
    bool ok = r.read(magic, sizeof magic);
    const bool v3 = ok && std::memcmp(magic, kCkptMagic3, sizeof magic) == 0;
    if (ok && v3) {
        CkptHeader3 h3{};
        std::memcpy(h3.magic, magic, sizeof magic);
        ok = r.read(reinterpret_cast<char*>(&h3) + sizeof magic, sizeof h3 - sizeof magic);
        std::memcpy(h.magic, magic, sizeof magic);
        h.cfg = e->cfg;   // (the fields a format-3 file has are compared below)
        h.cfg.abi_version = e->cfg.abi_version;
        h.cfg.mode = h3.cfg.mode; h.cfg.max_symbols = h3.cfg.max_symbols; h.cfg.max_accounts = h3.cfg.max_accounts;
        h.cfg.max_resting = h3.cfg.max_resting; h.cfg.max_epoch = h3.cfg.max_epoch;
        h.cfg.credit_shards = h3.cfg.credit_shards; h.cfg.flags = h3.cfg.flags;
        ok = ok && h3.cfg.abi_version == 6;
        h.seq_base = h3.seq_base; h.pool_used = h3.pool_used; h.n_levels = h3.n_levels;
        h.bal_live = h3.bal_live; h.pos_live = h3.pos_live; h.app_bytes = h3.app_bytes;
        h.n_sparse = 0;
    } else if (ok) {
        std::memcpy(h.magic, magic, sizeof magic);
        ok = std::memcmp(magic, kCkptMagic4, sizeof magic) == 0 &&
             r.read(reinterpret_cast<char*>(&h) + sizeof magic, sizeof h - sizeof magic) &&
             h.cfg.max_sparse_symbols == e->cfg.max_sparse_symbols && h.n_sparse == (uint64_t)e->S.Gs;
    }
    // the same store geometry (device, stream, timing and the ledger tables' initial size may differ)
    const size_t G = e->cfg.max_symbols, Gs = (size_t)e->S.Gs, A = e->cfg.max_accounts;
    ok = ok && h.cfg.abi_version == e->cfg.abi_version && h.cfg.mode == e->cfg.mode &&
         h.cfg.max_symbols == e->cfg.max_symbols && h.cfg.max_accounts == e->cfg.max_accounts &&
         h.cfg.max_resting == e->cfg.max_resting && h.cfg.max_epoch == e->cfg.max_epoch &&
         h.cfg.credit_shards == e->cfg.credit_shards && h.cfg.flags == e->cfg.flags &&
         h.pool_used <= e->S.pool_cap && h.n_levels <= (uint64_t)(G + h.n_sparse) * 2 * NLEV &&
         h.app_bytes < (1ull << 40) && h.bal_live < (1ull << 31) && h.pos_live < (1ull << 31) &&
         (e->ledger || (h.bal_live == 0 && h.pos_live == 0));
    if (ok && app_bytes) *app_bytes = (size_t)h.app_bytes;
    if (ok && (h.app_bytes > app_cap || (h.app_bytes && !app))) return KME_E_CAPACITY;   // nothing else read
    // the whole file is read and its digest checked before anything reaches the device: a mismatched,
    // truncated or corrupted checkpoint leaves the engine untouched
    const bool funded = e->cfg.mode == KME_MODE_FUNDED;
    std::vector<char> grp, lev, pool, acct, bal, pos, gsid, rec;
    auto take = [&](std::vector<char>& v, uint64_t n) {
        if (!ok) return;
        v.resize(n);
        ok = r.read(v.data(), n);
    };
    take(grp, (G + h.n_sparse) * sizeof(GroupState));
    if (v3) {   // format 3: levels, pool, accounts
        take(lev, h.n_levels * sizeof(Level));
        take(pool, h.pool_used * sizeof(Node));
        if (funded) take(acct, 3 * A * sizeof(int64_t));
    } else {    // format 4: accounts, pool, levels
        if (funded) take(acct, 3 * A * sizeof(int64_t));
        take(pool, h.pool_used * sizeof(Node));
        take(lev, h.n_levels * sizeof(Level));
    }
    take(bal, h.bal_live * 16);
    take(pos, h.pos_live * 32);
    take(gsid, h.n_sparse * sizeof(int64_t));
    take(rec, h.app_bytes);
    kme::CkptTrailer t{};
    ok = ok && r.verify(&t) && t.app_bytes == h.app_bytes;
    if (!ok) {
        if (app_bytes) *app_bytes = 0;
        return KME_E_INVALID;
    }
    // a format-3 file has no sparse groups: they restore empty
    if (h.n_sparse < Gs) {
        grp.resize((G + Gs) * sizeof(GroupState), 0);
        for (size_t g = G + h.n_sparse; g < G + Gs; ++g) reinterpret_cast<GroupState*>(grp.data())[g].free_head = -1;
        gsid.resize(Gs * sizeof(int64_t), 0);
    }
    // the groups whose book only the serial engine takes (C_ODD, k_segments' check)
    uint64_t odd = 0;
    for (size_t g = 0; g < G; ++g) {
        const GroupState& gs = reinterpret_cast<const GroupState*>(grp.data())[g];
        odd += (gs.nneg > 0 || (gs.bm0_msb >> 38) != 0 || (gs.bm1_msb >> 38) != 0) ? 1 : 0;
    }
    // ledger tables large enough for the live entries and two epochs (a fresh engine's may be
    // smaller): every replacement is allocated before any old table is freed, so a failed allocation
    // leaves the engine untouched (KME_E_CAPACITY)
    DevState& S = e->S;
    uint32_t* nbst = nullptr;
    int64_t *nbk = nullptr, *nbv = nullptr;
    PosEntry* npos = nullptr;
    uint64_t nb = 0, np = 0;
    if (e->ledger) {
        nb = ledger_slots(h.bal_live, bal_bound(e->cfg), 2);
        np = ledger_slots(h.pos_live, pos_bound(e->cfg), 2);
        if (nb > (1ull << 31) || np > (1ull << 31)) return KME_E_CAPACITY;
        bool aok = true;
        if (nb > (uint64_t)S.bal_mask + 1)
            aok = hipMalloc((void**)&nbst, nb * 4) == hipSuccess && hipMalloc((void**)&nbk, nb * 8) == hipSuccess &&
                  hipMalloc((void**)&nbv, nb * 8) == hipSuccess;
        if (aok && np > (uint64_t)S.pos_mask + 1) aok = hipMalloc((void**)&npos, np * sizeof(PosEntry)) == hipSuccess;
        if (kme::test_hook_fail("restore_alloc")) aok = false;   // (tests: the failed-allocation path)
        if (!aok) {
            (void)hipGetLastError();
            (void)hipFree(nbst); (void)hipFree(nbk); (void)hipFree(nbv); (void)hipFree(npos);
            return KME_E_CAPACITY;
        }
        if (nbst) {
            dfree(e, S.bal_state); dfree(e, S.bal_key); dfree(e, S.bal_val);
            e->allocs.push_back(nbst); e->allocs.push_back(nbk); e->allocs.push_back(nbv);
            S.bal_state = nbst; S.bal_key = nbk; S.bal_val = nbv;
            S.bal_mask = (uint32_t)(nb - 1);
        }
        if (npos) {
            dfree(e, S.pos);
            e->allocs.push_back(npos);
            S.pos = npos;
            S.pos_mask = (uint32_t)(np - 1);
        }
    }
    // from here on a failure leaves a mix of old and restored state: the engine is dead
    auto dead = [&](kme_status s) {
        e->failed = 1; e->fail_status = s; e->fail_detail = KME_D_NONE;
        return s;
    };
    hipStream_t st = e->stream;
    void *d_lev = nullptr, *d_bal = nullptr, *d_pos = nullptr;
    bool dok = staged_h2d(e, S.grp, grp.data(), grp.size(), "groups") &&
               hipMemsetAsync(S.lev, 0, (G + Gs) * 2 * NLEV * sizeof(Level), st) == hipSuccess &&
               hipMalloc(&d_lev, std::max<size_t>(lev.size(), 16)) == hipSuccess &&
               staged_h2d(e, d_lev, lev.data(), lev.size(), "levels") &&
               (pool.empty() || staged_h2d(e, S.pool, pool.data(), pool.size(), "pool")) &&
               (Gs == 0 || staged_h2d(e, S.gsid, gsid.data(), gsid.size(), "sparse symbols"));
    if (dok) launch_rst_levels(S, (const Level*)d_lev, (uint32_t)h.n_levels, st);
    if (dok && funded) {
        const int64_t* a = reinterpret_cast<const int64_t*>(acct.data());
        dok = staged_h2d(e, S.acct_since, a, A * 8, "accounts") && staged_h2d(e, S.acct_lb, a + A, A * 8, "accounts") &&
              staged_h2d(e, S.acct_demand, a + 2 * A, A * 8, "accounts");
    }
    unsigned long long fail = 0;
    if (dok && e->ledger) {
        dok = hipMemsetAsync(S.bal_state, 0, ((size_t)S.bal_mask + 1) * sizeof(uint32_t), st) == hipSuccess &&
              hipMemsetAsync(S.pos, 0, ((size_t)S.pos_mask + 1) * sizeof(PosEntry), st) == hipSuccess &&
              hipMalloc(&d_bal, std::max<size_t>(bal.size(), 16)) == hipSuccess &&
              hipMalloc(&d_pos, std::max<size_t>(pos.size(), 16)) == hipSuccess &&
              staged_h2d(e, d_bal, bal.data(), bal.size(), "Balances") && staged_h2d(e, d_pos, pos.data(), pos.size(), "Positions");
        if (dok) {
            launch_rst_ledger(S, d_bal, (uint32_t)h.bal_live, d_pos, (uint32_t)h.pos_live, e->d_maint, st);
            dok = hipMemcpyAsync(&fail, e->d_maint, sizeof fail, hipMemcpyDeviceToHost, st) == hipSuccess;
        }
    }
    // the oid table from the resting orders of the used pool prefix
    if (dok) launch_otab_rebuild(S, (uint32_t)h.pool_used, st);
    dok = dok && hipGetLastError() == hipSuccess && hipStreamSynchronize(st) == hipSuccess;
    if (d_lev) (void)hipFree(d_lev);
    if (d_bal) (void)hipFree(d_bal);
    if (d_pos) (void)hipFree(d_pos);
    // the device copy of the engine state (the tables above may have moved) before anything can fail
    // later: a dead engine's kernels never run, a live one's read the state it holds
    if (hipMemcpy(e->d_S, &e->S, sizeof(DevState), hipMemcpyHostToDevice) != hipSuccess) return dead(KME_E_HIP);
    if (!dok) return dead(KME_E_HIP);
    if (fail) return dead(KME_E_CAPACITY);
    unsigned long long ctr[C_NCTR * CTR_STRIDE];
    if (hipMemcpy(ctr, S.ctr, sizeof ctr, hipMemcpyDeviceToHost) != hipSuccess) return dead(KME_E_HIP);
    if (ctr[ci(C_REBUILD_FAIL)] != 0 || ctr[ci(C_OTAB_USED)] * 4 > e->otab_cap * 3) return dead(KME_E_CAPACITY);
    ctr[ci(C_POOL_BUMP)] = h.pool_used;
    ctr[ci(C_BAL_USED)] = h.bal_live;
    ctr[ci(C_POS_USED)] = h.pos_live;
    ctr[ci(C_ODD)] = odd ? 1 : 0;
    ctr[ci(C_ERR)] = ~0ull;
    {   // a restored book may hold size-0 (or negative) makers: then the fast segments stay off (C_SIZE0)
        const Node* nodes = reinterpret_cast<const Node*>(pool.data());
        ctr[ci(C_SIZE0)] = 0;
        for (uint64_t k = 0; k < h.pool_used; ++k)
            if (nodes[k].live && nodes[k].size <= 0) { ctr[ci(C_SIZE0)] = 1; break; }
    }
    if (hipMemcpy(S.ctr, ctr, sizeof ctr, hipMemcpyHostToDevice) != hipSuccess) return dead(KME_E_HIP);
    e->seq_base = h.seq_base;
    if (!rec.empty()) std::memcpy(app, rec.data(), rec.size());
    return KME_OK;
}

kme_status kme_restore(kme_engine* e, const char* path) {
    size_t n = 0;
    kme_status s = kme_restore_app(e, path, nullptr, 0, &n);
    if (s == KME_E_CAPACITY && n) {   // (an application record this caller does not want)
        std::vector<char> sink(n);
        s = kme_restore_app(e, path, sink.data(), sink.size(), &n);
    }
    return s;
}

kme_status kme_ledger_stats(kme_engine* e, kme_ledger_info* out) {
    if (!e || !out) return KME_E_INVALID;
    *out = kme_ledger_info{};
    if (!e->ledger) return KME_E_UNSUPPORTED;
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipStreamSynchronize(e->stream));
    unsigned long long ctr[C_NCTR * CTR_STRIDE];
    HIP_TRY(hipMemcpy(ctr, e->S.ctr, sizeof ctr, hipMemcpyDeviceToHost));
    out->bal_slots = (uint64_t)e->S.bal_mask + 1;
    out->pos_slots = (uint64_t)e->S.pos_mask + 1;
    out->bal_used = ctr[ci(C_BAL_USED)];
    out->pos_used = ctr[ci(C_POS_USED)];
    out->grows = e->ledger_grows;
    return KME_OK;
}

kme_status kme_tape_json_device(kme_engine* e, const kme_orders* in_dev, uint32_t n, const kme_epoch_result* res_dev,
                                void* out_dev, size_t cap, size_t* len) {
    if (!e || !in_dev || !len) return KME_E_INVALID;
    if (n > e->cfg.max_epoch) return KME_E_CAPACITY;
    HIP_TRY(hipSetDevice(e->device));
    kme_epoch_result r{};
    if (res_dev) r = *res_dev; else kme_device_results(e, &r);
    hipStream_t st = e->stream;
    launch_ser_len(*in_dev, r, n, e->d_ser_len, e->d_ser_total, st);
    HIP_TRY(hipMemcpyAsync(e->h_ser_total, e->d_ser_total, sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    const uint64_t total = *e->h_ser_total;
    *len = (size_t)total;
    if (total >= (1ull << 32)) return KME_E_CAPACITY;
    if (total > cap || n == 0) return KME_OK;
    if (!out_dev) return KME_E_INVALID;
    launch_scan(e->d_ser_len, e->d_ser_off, n, e->d_ser_tmp, e->d_ser_off + n, st);
    launch_ser_write(*in_dev, r, n, e->d_ser_off, out_dev, st);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(st));
    return KME_OK;
}

kme_status kme_debug_counters(kme_engine* e, uint64_t* out, size_t n) {
    if (!e || !out) return KME_E_INVALID;
    const size_t cap = (size_t)e->cfg.max_symbols * KME_DBG_WORDS;
    HIP_TRY(hipStreamSynchronize(e->stream));
    HIP_TRY(hipMemcpy(out, e->S.dbg, std::min(n, cap) * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return KME_OK;
}

kme_status kme_device_results(kme_engine* e, kme_epoch_result* r) {
    if (!e || !r) return KME_E_INVALID;
    r->out_action = e->d_out_action; r->out_size = e->d_out_size; r->out_prev = e->d_out_prev;
    r->out_flags = e->d_out_flags; r->trade_off = e->d_trade_off;
    r->trades = reinterpret_cast<kme_trade*>(e->d_trades);
    r->trades_cap = e->cfg.max_trades;
    return KME_OK;
}

kme_status kme_phase_times(kme_engine* e, float* ms, int* n) {
    if (!e || !ms || !n) return KME_E_INVALID;
    for (int p = 0; p < PH_N; ++p) ms[p] = e->phase_ms[p];
    *n = PH_N;
    return KME_OK;
}
const char* kme_phase_name(int i) { return (i >= 0 && i < PH_N) ? kPhaseNames[i] : ""; }

// Host-buffer epoch: copies in, runs, copies out.  FUNDED epochs are split into runs at account
// records so that the reservation proof never has to reason across a CREATE/TRANSFER boundary.
kme_status kme_submit_epoch(kme_engine* e, const kme_orders* in, uint32_t n, kme_epoch_result* out,
                            kme_epoch_status* st) {
    if (e && e->inflight) return KME_E_INVALID;   // device epochs still in flight: kme_wait them first
    if (!e || !in || !out) return KME_E_INVALID;
    HIP_TRY(hipSetDevice(e->device));
    kme_epoch_status total{};
    total.error_index = -1;
    total.n_inputs = n;
    uint32_t a = 0;
    uint32_t tbase = 0;
    out->trade_off[0] = 0;
    const bool funded = e->cfg.mode == KME_MODE_FUNDED;
    auto is_acct = [&](uint32_t i) { return in->action[i] == KME_CREATE_BALANCE || in->action[i] == KME_TRANSFER; };
    while (a < n || (n == 0 && a == 0)) {
        uint32_t b = a;
        if (n > 0) {
            if (funded) {
                const bool kind = is_acct(a);
                while (b < n && is_acct(b) == kind && b - a < e->cfg.max_epoch) ++b;
            } else {
                b = std::min<uint64_t>(n, (uint64_t)a + e->cfg.max_epoch);
            }
        }
        const uint32_t m = b - a;
        hipStream_t s = e->stream;
        if (m > 0) {
            HIP_TRY(hipMemcpyAsync(e->d_action, in->action + a, m * sizeof(int32_t), hipMemcpyHostToDevice, s));
            HIP_TRY(hipMemcpyAsync(e->d_oid, in->oid + a, m * sizeof(int64_t), hipMemcpyHostToDevice, s));
            HIP_TRY(hipMemcpyAsync(e->d_aid, in->aid + a, m * sizeof(int64_t), hipMemcpyHostToDevice, s));
            HIP_TRY(hipMemcpyAsync(e->d_sid, in->sid + a, m * sizeof(int64_t), hipMemcpyHostToDevice, s));
            HIP_TRY(hipMemcpyAsync(e->d_price, in->price + a, m * sizeof(int32_t), hipMemcpyHostToDevice, s));
            HIP_TRY(hipMemcpyAsync(e->d_size, in->size + a, m * sizeof(int32_t), hipMemcpyHostToDevice, s));
        }
        kme_orders din{e->d_action, e->d_oid, e->d_aid, e->d_sid, e->d_price, e->d_size};
        kme_status rc = submit(e, &din, m, nullptr);
        if (rc != KME_OK) return rc;
        kme_epoch_status es{};
        rc = kme_wait(e, &es);
        total.n_trades += es.n_trades;
        total.n_orders += es.n_orders;
        total.n_rests += es.n_rests;
        total.n_maker_visits += es.n_maker_visits;
        total.n_cancel_ok += es.n_cancel_ok;
        total.serial_fallback += es.serial_fallback;   // sub-epochs that ran serially
        total.ledger_repaired += es.ledger_repaired;
        total.ledger_serial += es.ledger_serial;
        if (rc != KME_OK) {
            // the results of the records before the fault (the reference forwarded and committed
            // them, KP:97, 124-125): out arrays, trade offsets and their trades
            const uint32_t k = es.n_effective;
            total.status = es.status;
            total.detail = es.detail;
            total.error_index = es.error_index >= 0 ? es.error_index + a : -1;
            total.n_effective = a + k;
            total.n_trades = tbase;
            if (k > 0) {
                HIP_TRY(hipMemcpyAsync(out->trade_off + a + 1, e->d_trade_off + 1, k * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
                HIP_TRY(hipStreamSynchronize(s));
                const uint32_t kt = out->trade_off[a + k];
                if (tbase + kt <= out->trades_cap) {
                    HIP_TRY(hipMemcpyAsync(out->out_action + a, e->d_out_action, k * sizeof(int32_t), hipMemcpyDeviceToHost, s));
                    HIP_TRY(hipMemcpyAsync(out->out_size + a, e->d_out_size, k * sizeof(int32_t), hipMemcpyDeviceToHost, s));
                    HIP_TRY(hipMemcpyAsync(out->out_prev + a, e->d_out_prev, k * sizeof(int64_t), hipMemcpyDeviceToHost, s));
                    HIP_TRY(hipMemcpyAsync(out->out_flags + a, e->d_out_flags, k * sizeof(uint8_t), hipMemcpyDeviceToHost, s));
                    if (kt) HIP_TRY(hipMemcpyAsync(out->trades + tbase, e->d_trades, (size_t)kt * sizeof(kme_trade), hipMemcpyDeviceToHost, s));
                    HIP_TRY(hipStreamSynchronize(s));
                    for (uint32_t q = a + 1; q <= a + k; ++q) out->trade_off[q] += tbase;
                    total.n_trades = tbase + kt;
                } else {
                    total.n_effective = a;   // (cannot happen: the device epoch fit its own buffer)
                }
            }
            if (st) *st = total;
            return rc;
        }
        if (tbase + es.n_trades > out->trades_cap) {
            total.status = KME_E_CAPACITY;
            total.detail = KME_D_CAP_TRADES;
            if (st) *st = total;
            e->failed = 1; e->fail_status = KME_E_CAPACITY; e->fail_detail = KME_D_CAP_TRADES;
            return KME_E_CAPACITY;
        }
        if (m > 0) {
            HIP_TRY(hipMemcpyAsync(out->out_action + a, e->d_out_action, m * sizeof(int32_t), hipMemcpyDeviceToHost, s));
            HIP_TRY(hipMemcpyAsync(out->out_size + a, e->d_out_size, m * sizeof(int32_t), hipMemcpyDeviceToHost, s));
            HIP_TRY(hipMemcpyAsync(out->out_prev + a, e->d_out_prev, m * sizeof(int64_t), hipMemcpyDeviceToHost, s));
            HIP_TRY(hipMemcpyAsync(out->out_flags + a, e->d_out_flags, m * sizeof(uint8_t), hipMemcpyDeviceToHost, s));
            HIP_TRY(hipMemcpyAsync(out->trade_off + a + 1, e->d_trade_off + 1, m * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
            if (es.n_trades)
                HIP_TRY(hipMemcpyAsync(out->trades + tbase, e->d_trades, (size_t)es.n_trades * sizeof(kme_trade), hipMemcpyDeviceToHost, s));
            HIP_TRY(hipStreamSynchronize(s));
            for (uint32_t k = a + 1; k <= b; ++k) out->trade_off[k] += tbase;
        }
        tbase += es.n_trades;
        a = b;
        if (n == 0) break;
    }
    total.n_trades = tbase;
    total.n_effective = n;
    if (st) *st = total;
    return KME_OK;
}

kme_status kme_top_of_book(kme_engine* e, kme_tob* dev_out) {
    if (!e || !dev_out) return KME_E_INVALID;
    launch_tob(e->S, dev_out, e->stream);
    HIP_TRY(hipGetLastError());
    return KME_OK;
}

kme_status kme_top_of_book_groups(kme_engine* e, const uint32_t* dev_groups, uint32_t n, kme_tob* dev_out) {
    if (!e || (n && (!dev_groups || !dev_out))) return KME_E_INVALID;
    launch_tob_groups(e->S, dev_groups, n, dev_out, e->stream);
    HIP_TRY(hipGetLastError());
    return KME_OK;
}

// ------------------------------------------------------------------ snapshots
static char* dup_string(const std::string& s, size_t* len) {
    char* p = (char*)std::malloc(s.size() + 1);
    std::memcpy(p, s.data(), s.size());
    p[s.size()] = 0;
    if (len) *len = s.size();
    return p;
}

kme_status kme_snapshot_books(kme_engine* e, char** text, size_t* len) {
    if (!e || !text) return KME_E_INVALID;
    if (kme_status r = snap_begin(e, "kme_snapshot_books")) return r;
    const uint32_t G = e->cfg.max_symbols + (uint32_t)e->S.Gs;   // the dense groups, then the sparse ones
    const uint32_t Gd = e->cfg.max_symbols;
    std::vector<GroupState> grp(G);
    std::vector<Level> lev((size_t)G * 2 * NLEV);
    std::vector<int64_t> gsid((size_t)e->S.Gs);
    unsigned long long ctr[C_NCTR * CTR_STRIDE];
    if (kme_status r = snap_read(e, ctr, e->S.ctr, sizeof ctr, "counters")) return r;
    const uint64_t nslots = std::min<uint64_t>(ctr[ci(C_POOL_BUMP)], e->S.pool_cap);
    std::vector<Node> pool(nslots);
    if (kme_status r = snap_read(e, grp.data(), e->S.grp, G * sizeof(GroupState), "groups")) return r;
    if (kme_status r = snap_read(e, lev.data(), e->S.lev, lev.size() * sizeof(Level), "levels")) return r;
    if (nslots)
        if (kme_status r = snap_read(e, pool.data(), e->S.pool, nslots * sizeof(Node), "pool")) return r;
    if (!gsid.empty())
        if (kme_status r = snap_read(e, gsid.data(), e->S.gsid, gsid.size() * sizeof(int64_t), "sparse symbols")) return r;

    struct BookLine { int64_t key, msb, lsb; };
    struct BucketLine { int64_t ptr, first, last; };
    std::vector<BookLine> books;
    std::vector<BucketLine> buckets;
    std::vector<std::string> problems;
    uint64_t listed = 0;
    for (uint32_t g = 0; g < G; ++g) {
        const GroupState& gs = grp[g];
        if (!gs.exists) continue;
        const int64_t asid = g < Gd ? (int64_t)g : gsid[g - Gd];   // |sid| of the group's books
        if (g >= Gd && asid == 0) { problems.push_back("X sparse group without a symbol"); continue; }
        for (int side = 0; side < (g == 0 ? 1 : 2); ++side) {
            const int64_t key = side ? -asid : asid;
            const uint64_t l = side ? gs.bm1_lsb : gs.bm0_lsb, m = side ? gs.bm1_msb : gs.bm0_msb;
            books.push_back({key, (int64_t)m, (int64_t)l});
            for (int p = 0; p <= 126; ++p) {
                const bool set = p < 63 ? ((l >> p) & 1) : ((m >> (p - 63)) & 1);
                if (!set) continue;
                const Level& L = lev[((size_t)g * 2 + side) * NLEV + p];
                if (L.head < 0 || (uint64_t)L.head >= nslots || L.tail < 0 || (uint64_t)L.tail >= nslots) {
                    problems.push_back("X level head/tail out of range");
                    continue;
                }
                buckets.push_back({(int64_t)((uint64_t)key << 8) | p, pool[L.head].oid, pool[L.tail].oid});
                // invariant walk: list links, quantity, tail oid
                int32_t s = L.head, prev = -1, cnt = 0;
                int64_t qty = 0;
                while (s >= 0 && (uint64_t)s < nslots && cnt <= (int32_t)nslots) {
                    const Node& nd = pool[s];
                    if (!nd.live || nd.prev != prev || nd.price != p || nd.group != (int32_t)g) {
                        problems.push_back("X broken list at key " + std::to_string(key) + " price " + std::to_string(p));
                        break;
                    }
                    if (prev >= 0 && nd.prev_oid != pool[prev].oid) problems.push_back("X prev_oid mismatch");
                    qty += nd.size;
                    ++cnt;
                    prev = s;
                    s = nd.next;
                }
                listed += cnt;
                if (prev != L.tail || qty != L.qty || L.tail_oid != pool[L.tail].oid)
                    problems.push_back("X level bookkeeping mismatch at key " + std::to_string(key) + " price " + std::to_string(p));
            }
        }
    }
    std::sort(books.begin(), books.end(), [](const BookLine& a, const BookLine& b) { return a.key < b.key; });
    std::sort(buckets.begin(), buckets.end(), [](const BucketLine& a, const BucketLine& b) { return a.ptr < b.ptr; });
    std::vector<const Node*> live;
    for (uint64_t s = 0; s < nslots; ++s) if (pool[s].live) live.push_back(&pool[s]);
    if (live.size() != listed) problems.push_back("X live nodes not reachable from a level: " + std::to_string(live.size()) + " vs " + std::to_string(listed));
    std::sort(live.begin(), live.end(), [](const Node* a, const Node* b) { return a->oid < b->oid; });
    std::string out;
    out.reserve(64 * (books.size() + buckets.size() + live.size()) + 64);
    char line[256];
    for (auto& b : books) {
        int k = std::snprintf(line, sizeof line, "B %lld %lld %lld\n", (long long)b.key, (long long)b.msb, (long long)b.lsb);
        out.append(line, k);
    }
    for (auto& b : buckets) {
        int k = std::snprintf(line, sizeof line, "K %lld %lld %lld\n", (long long)b.ptr, (long long)b.first, (long long)b.last);
        out.append(line, k);
    }
    for (const Node* nd : live) {
        char nx[32], pv[32];
        if (nd->next >= 0) std::snprintf(nx, sizeof nx, "%lld", (long long)pool[nd->next].oid); else std::strcpy(nx, "null");
        if (nd->prev >= 0) std::snprintf(pv, sizeof pv, "%lld", (long long)nd->prev_oid); else std::strcpy(pv, "null");
        int k = std::snprintf(line, sizeof line, "O %lld %d %lld %lld %d %d %s %s\n", (long long)nd->oid, nd->action,
                              (long long)nd->aid, (long long)nd->sid, nd->price, nd->size, nx, pv);
        out.append(line, k);
    }
    for (auto& p : problems) { out += p; out += '\n'; }
    *text = dup_string(out, len);
    return KME_OK;
}

kme_status kme_snapshot_ledger(kme_engine* e, char** text, size_t* len) {
    if (!e || !text) return KME_E_INVALID;
    if (e->cfg.mode != KME_MODE_EXACT && !e->S.ledger_replay) return KME_E_UNSUPPORTED;
    if (kme_status r = snap_begin(e, "kme_snapshot_ledger")) return r;
    const size_t lb = (size_t)e->S.bal_mask + 1, lp = (size_t)e->S.pos_mask + 1;
    std::vector<uint32_t> bst(lb);
    std::vector<int64_t> bk(lb), bv(lb);
    std::vector<PosEntry> pos(lp);
    if (kme_status r = snap_read(e, bst.data(), e->S.bal_state, lb * 4, "Balances states")) return r;
    if (kme_status r = snap_read(e, bk.data(), e->S.bal_key, lb * 8, "Balances keys")) return r;
    if (kme_status r = snap_read(e, bv.data(), e->S.bal_val, lb * 8, "Balances values")) return r;
    if (kme_status r = snap_read(e, pos.data(), e->S.pos, lp * sizeof(PosEntry), "Positions")) return r;
    std::vector<std::pair<int64_t, int64_t>> bal;
    for (size_t h = 0; h < lb; ++h) if (bst[h] == 1) bal.push_back({bk[h], bv[h]});
    std::sort(bal.begin(), bal.end());
    std::vector<PosEntry> ps;
    for (size_t h = 0; h < lp; ++h) if (pos[h].state == 1) ps.push_back(pos[h]);
    std::sort(ps.begin(), ps.end(), [](const PosEntry& a, const PosEntry& b) { return a.k0 != b.k0 ? a.k0 < b.k0 : a.k1 < b.k1; });
    std::string out;
    char line[256];
    for (auto& b : bal) {
        int k = std::snprintf(line, sizeof line, "A %lld %lld\n", (long long)b.first, (long long)b.second);
        out.append(line, k);
    }
    for (auto& p : ps) {
        int k = std::snprintf(line, sizeof line, "P %lld %lld %lld %lld\n", (long long)p.k0, (long long)p.k1, (long long)p.v0, (long long)p.v1);
        out.append(line, k);
    }
    *text = dup_string(out, len);
    return KME_OK;
}

}  // extern "C"
