// kme_launch.h -- host-side launchers of the epoch kernels (kme_kernels.hip), used by the runtime.
#pragma once
#include <hip/hip_runtime.h>
#include "kme.h"
#include "kme_device.h"

namespace kme {

#ifndef KME_RADIX_TILE
#define KME_RADIX_TILE 8192
#endif
// inputs per partition tile (256 threads x 32): each digit's run of a tile ~16 keys (64 B) at 512
// digits; 4,096 left 32-B runs (same-box A/B: partition 0.128 -> 0.119 ms at C3, 74 KB of LDS)
constexpr int RADIX_TILE = KME_RADIX_TILE;
// small sorts (at most RADIX_SMALL_N keys: the drop-in's 65,536-record epochs) take 2,048-key tiles --
// 32 blocks instead of 8 per pass; buffers sized per tile are sized for these
constexpr int RADIX_TILE_SMALL = 2048;
constexpr uint32_t RADIX_SMALL_N = 1u << 18;
constexpr int RADIX_BITS = 9;        // digit width of the partition passes
constexpr int POOL_CHUNK = 64;       // node slots a group takes from the global bump at a time
constexpr int kDefaultLightMax = 128;  // DevState::light_max default (KME_LIGHT_MAX overrides)
constexpr int kLaneTradeChunk = 8;    // trade scratch slots a k_match_lanes lane reserves at a time
constexpr int kOsLanesMaxLight = 512;  // light_max up to which light groups' OUT echo goes step-major

// A stable LSD radix sort of (key, value) u32 pairs, RADIX_BITS-bit digits (the partition's kernels).
// Pass 0 reads key0 (negative -> `none`) and val0 (nullptr: the element's index); the result is in
// keys / vals [passes & 1].  n_dev: the count on the device (at most n), else n.
struct RadixIO {
    const KG int32_t* key0;
    const KG uint32_t* val0;
    // the ping-pong buffers as four named fields, not arrays: a pass selects them by its parity, and
    // a select between two elements of an array member was folded into a dynamic index into the
    // kernel argument -- which put the whole struct in scratch memory (136 B per lane, stored at
    // every scatter's start and read back on its critical path)
    KG uint32_t* keys0;
    KG uint32_t* keys1;
    KG uint32_t* vals0;
    KG uint32_t* vals1;
    KG uint32_t* ghist;              // RADIX_DIGITS x tiles + the scan's scratch
    KG int32_t* rank;                // the last pass: rank[value] = position (nullptr: none)
    const KG uint4* pay_src;         // the last pass: pay_dst[position] = pay_src[value] (nullptr: none)
    KG uint4* pay_dst;
    uint32_t none;
    uint32_t n;
    const KG unsigned long long* n_dev;
    int passes;
    int small;                       // 2,048-key tiles (a small sort; n may be a capacity far above it)
    // small sorts, one launch per pass (launch_radix): every pass's per-tile digit counts of the
    // unpermuted keys (passes x tiles x digits: the digit totals), and the look-back words (tiles x
    // digits: count | launch stamp << 32).  nullptr: the hist / scan / scatter launches per pass.
    KG uint32_t* tcnt;
    KG unsigned long long* lb;
    KG unsigned long long* ctr;      // the engine's counters: a look-back that never completes is raised there
};
constexpr int RADIX_MAXP = 4;        // passes of a look-back sort (tcnt's rows)
void launch_radix(const RadixIO& R, hipStream_t st);
uint32_t next_stamp();               // a look-back launch's stamp (unique, never 0)
void launch_excl_scan(const uint32_t* in, uint32_t* out, uint32_t L, uint32_t* sums, uint32_t* total, hipStream_t st,
                      unsigned long long* ctr);
// FUNDED + exact ledger: the epoch's ledger effects in parallel (kme_ledger.hip); the serial replay
// (launch_ledger_replay) runs after it and does the work only when this path fell back
void launch_ledger_parallel(const DevState& S, const EpochIO& io, uint32_t max_trades, hipStream_t st);

// FUNDED pipeline
void launch_epoch_reset(const DevState& S, hipStream_t st);   // the per-epoch counters, one launch
void launch_emap(const DevState& S, const EpochIO& io, bool funded, EpochIO* io_dev, hipStream_t st);
void launch_ledger_funded(const DevState& S, const EpochIO& io, hipStream_t st);
void launch_route(const DevState& S, const EpochIO& io, bool funded, hipStream_t st);
// returns the buffer index (0/1) holding the sorted input permutation
// list_min >= 0: k_segments also lists the groups with more than list_min records (glist, C_GLIST)
int launch_partition(const DevState& S, const EpochIO& io, hipStream_t st, int list_min = -1);
// k_match over the listed groups only (a grid of `blocks` looping over the list): for epochs that
// are expected to have few or no busy groups among many (C3: a G-block k_match that finds nothing
// costs ~16 us)
void launch_match_list(const DevState* S_dev, const EpochIO* io_dev, int perm_buf, hipStream_t st, int all, uint32_t blocks);
// two: two wavefronts per group (the pass one segment ahead of the level step; few busy groups)
void launch_match(const DevState& S, const DevState* S_dev, const EpochIO* io_dev, int perm_buf, hipStream_t st, int all, int two, int dense,
                  int five);
// light groups (at most S.light_max records in the epoch), one lane each; independent of k_match
void launch_match_lanes(const DevState& S, const DevState* S_dev, const EpochIO* io_dev, int perm_buf, hipStream_t st);
void launch_compact(const DevState& S, const EpochIO& io, hipStream_t st);
void launch_table(const DevState& S, const EpochIO& io, hipStream_t st);
// EXACT pipeline (emap + route shared)
void launch_serial(const DevState* S_dev, const EpochIO* io_dev, hipStream_t st, int only_fallback = 0);
// FUNDED + KME_FLAG_SERIAL_FALLBACK: funded bounds from the exact ledger after a serial epoch
void launch_settle_funded(const DevState& S, const EpochIO& io, hipStream_t st);
// FUNDED + KME_FLAG_EXACT_LEDGER: the epoch's ledger effects in arrival order (after compaction)
// ctr_out: when the replay is the epoch's last launch, the counters' pinned host copy (device view)
void launch_ledger_replay(const DevState* S_dev, const EpochIO* io_dev, hipStream_t st, unsigned long long* ctr_out = nullptr);
// exclusive scan of L u32 values (DPP wave scans): out[k] = sum(in[0..k)); bsum needs
// L / 2048 + 1 words of scratch, *total receives the sum
void launch_scan(const uint32_t* in, uint32_t* out, uint32_t L, uint32_t* bsum, uint32_t* total, hipStream_t st);
// device serializer (kme_serialize.hip)
void launch_ser_len(const kme_orders& in, const kme_epoch_result& r, uint32_t n, uint32_t* len, unsigned long long* total,
                    hipStream_t st);
void launch_ser_write(const kme_orders& in, const kme_epoch_result& r, uint32_t n, const uint32_t* off, void* out,
                      hipStream_t st);
// maintenance
void launch_otab_rebuild(const DevState& S, uint32_t used_slots, hipStream_t st);   // pool slots [0, used) hold every node
void launch_tob(const DevState& S, void* out, hipStream_t st);
// rows >= n: rows past n are padding (-1 / 0)
void launch_tob_groups(const DevState& S, const uint32_t* groups, uint32_t n, void* out, hipStream_t st, uint32_t rows = 0);
void launch_init_state(const DevState& S, hipStream_t st);
// store maintenance between epochs (kme_maint.hip): live entries of Balances / Positions (out2[0],
// out2[1]); the live entries of O's tables rehashed into N's (fresh, empty) tables where they differ
void launch_ledger_live(const DevState& S, unsigned long long* out2, hipStream_t st);
void launch_ledger_rehash(const DevState& N, const DevState& O, unsigned long long* fail2, hipStream_t st);
// checkpoint format 3: the set levels (index in _pad[0]), live Balances (aid, value) and Positions
// (k0, k1, v0, v1); their restore into an engine whose levels / tables are empty
void launch_ckpt_levels(const DevState& S, Level* out, unsigned long long* cnt, hipStream_t st);
void launch_rst_levels(const DevState& S, const Level* in, uint32_t n, hipStream_t st);
void launch_ckpt_ledger(const DevState& S, void* bal_out, void* pos_out, unsigned long long* cnt2, hipStream_t st);
void launch_rst_ledger(const DevState& S, const void* bal_in, uint32_t nb, const void* pos_in, uint32_t np,
                       unsigned long long* fail, hipStream_t st);
// credit between symbol shards: (funded bound, demand) per account out; the re-split from all shards' pairs
void launch_credit_state(const DevState& S, int64_t* out, hipStream_t st);
// all: n blocks of `stride` int64 words each ([0, A) bound, [A, 2A) demand, -1 = absent on that shard)
void launch_credit_adjust(const DevState& S, const int64_t* all, uint32_t n, uint32_t me, size_t stride, hipStream_t st);
// host epochs (kme_submit_epoch_host): trades[0, min(trade_off[n], cap)) into device-mapped host memory
void launch_export_trades(const TradeRec* src, const uint32_t* count, uint32_t cap, TradeRec* dst_mapped, hipStream_t st);

}  // namespace kme
