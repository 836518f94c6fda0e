// kme_maint.hip -- store maintenance between epochs (never on the epoch path): online growth of the
// exact ledger's Balances / Positions tables, and the compact form of the stores a checkpoint holds.
//
// The reference's Balances and Positions are RocksDB stores that grow without bound (KP:30-37); the
// Positions store keeps every (account, symbol) ever filled and, through the value-keyed writes of
// setPosition(UUID, ...) (KP:283-284, 434-436, hazard H2), stale keys forever.  Here they are
// open-addressing tables in HBM; the runtime (kme_runtime.cpp ledger_reserve) rehashes them into
// larger tables between epochs, before the live entries plus what the next epochs can add could
// pass half load, so the device's capacity check (KME_D_CAP_LEDGER) means "out of HBM", not "the
// initial size was too small".
//
// A checkpoint (kme_runtime.cpp, format 3) keeps only what is live: the price levels whose bit is set
// in their book's bitmap (KP:379-416 -- a level whose bit is clear is never read), the Balances and
// Positions entries in use (no empty slots, no tombstones); the oid table is rebuilt from the resting
// orders on restore.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "kme.h"
#include "kme_device.h"
#include "kme_jarith.h"
#include "kme_launch.h"

namespace kme {

namespace {

// One output slot per lane that wants one: a single atomic per wavefront.
KDEV uint32_t wave_reserve(unsigned long long* cnt, bool want) {
    const unsigned long long m = __ballot(want);
    if (!m) return 0;
    const int lane = lane_id();
    const int leader = __ffsll((long long)m) - 1;
    unsigned long long base = 0;
    if (lane == leader) base = atomicAdd(cnt, (unsigned long long)__popcll(m));
    base = (unsigned long long)__shfl((long long)base, leader);
    return (uint32_t)(base + (unsigned long long)__popcll(m & ((1ull << lane) - 1)));
}

// A key known to be absent from the table (every key of a rehash or a restore is distinct): the first
// empty slot of its probe sequence, claimed by CAS; no reader runs meanwhile.
KDEV bool bal_put_new(const DevState& S, int64_t aid, int64_t val) {
    uint32_t h = (uint32_t)mix64((uint64_t)aid) & S.bal_mask;
    for (uint32_t p = 0; p <= S.bal_mask; ++p) {
        if (S.bal_state[h] == 0 && atomicCAS((unsigned int*)&S.bal_state[h], 0u, 1u) == 0u) {
            S.bal_key[h] = aid;
            S.bal_val[h] = val;
            return true;
        }
        h = (h + 1) & S.bal_mask;
    }
    return false;
}
KDEV bool pos_put_new(const DevState& S, int64_t k0, int64_t k1, int64_t v0, int64_t v1) {
    uint32_t h = (uint32_t)mix64((uint64_t)k0 * 0x9e3779b97f4a7c15ull ^ mix64((uint64_t)k1)) & S.pos_mask;   // = pos_hash
    for (uint32_t p = 0; p <= S.pos_mask; ++p) {
        if (S.pos[h].state == 0 && atomicCAS((unsigned int*)&S.pos[h].state, 0u, 1u) == 0u) {
            KG long4* d = reinterpret_cast<KG long4*>(&S.pos[h]);
            d[0] = make_long4(k0, k1, v0, v1);
            return true;
        }
        h = (h + 1) & S.pos_mask;
    }
    return false;
}

KDEV void block_add(unsigned long long* dst, uint32_t v) {
    for (int off = 32; off > 0; off >>= 1) v += (uint32_t)__shfl_xor((int)v, off);
    if (lane_id() == 0 && v) atomicAdd(dst, (unsigned long long)v);
}

}  // namespace

// Live entries of both tables (out[0] Balances, out[1] Positions).
__global__ void __launch_bounds__(256) k_ledger_live(DevState S, unsigned long long* out) {
    uint32_t nb = 0, np = 0;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t h = blockIdx.x * blockDim.x + threadIdx.x; h <= S.bal_mask; h += stride) nb += S.bal_state[h] == 1u;
    for (uint32_t h = blockIdx.x * blockDim.x + threadIdx.x; h <= S.pos_mask; h += stride) np += S.pos[h].state == 1u;
    block_add(&out[0], nb);
    block_add(&out[1], np);
}
// Rehash: every live entry of the old tables (o*) into the new, empty ones of N.  out[0] counts the
// entries that found no slot (cannot happen: the new tables are at most half full).
__global__ void __launch_bounds__(256) k_bal_rehash(DevState N, const uint32_t* ost, const int64_t* okey,
                                                    const int64_t* oval, uint32_t oslots, unsigned long long* out) {
    uint32_t fail = 0;
    for (uint32_t h = blockIdx.x * blockDim.x + threadIdx.x; h < oslots; h += gridDim.x * blockDim.x)
        if (ost[h] == 1u && !bal_put_new(N, okey[h], oval[h])) ++fail;
    block_add(&out[0], fail);
}
__global__ void __launch_bounds__(256) k_pos_rehash(DevState N, const PosEntry* old, uint32_t oslots, unsigned long long* out) {
    uint32_t fail = 0;
    for (uint32_t h = blockIdx.x * blockDim.x + threadIdx.x; h < oslots; h += gridDim.x * blockDim.x) {
        if (old[h].state != 1u) continue;
        const long4 e = reinterpret_cast<const long4*>(&old[h])[0];
        if (!pos_put_new(N, e.x, e.y, e.z, e.w)) ++fail;
    }
    block_add(&out[0], fail);
}

// ---------------------------------------------------------------- checkpoint compaction / restore
// The levels whose bit is set (one thread per (group, side, price)): the level with its index in
// _pad[0].  Order is irrelevant (restore scatters by index).
__global__ void __launch_bounds__(256) k_ckpt_levels(DevState S, Level* out, unsigned long long* cnt) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t total = (uint64_t)(S.G + S.Gs) * 2 * NLEV;   // dense and sparse groups
    bool set = false;
    uint32_t g = 0, side = 0, p = 0;
    if (t < total) {
        g = (uint32_t)(t / (2 * NLEV)); side = (uint32_t)((t / NLEV) & 1); p = (uint32_t)(t % NLEV);
        const KG uint64_t* bm = reinterpret_cast<const KG uint64_t*>(&S.grp[g]) + 2 * side;   // lsb, msb of book side
        set = p < 127 && (p < 63 ? (bm[0] >> p) & 1ull : (bm[1] >> (p - 63)) & 1ull);
    }
    const uint32_t k = wave_reserve(cnt, set);
    if (set) {
        Level L = S.lev[t];
        L._pad[0] = (int32_t)(uint32_t)t;   // (t < (G + Gs) * 256 <= 2^32)
        L._pad[1] = 0;
        out[k] = L;
    }
}
__global__ void __launch_bounds__(256) k_rst_levels(DevState S, const Level* in, uint32_t n) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    Level L = in[k];
    const uint32_t t = (uint32_t)L._pad[0];
    L._pad[0] = 0;
    S.lev[t] = L;
}
// Balances as (aid, balance) pairs, Positions as (key msb, key lsb, amount, available).
__global__ void __launch_bounds__(256) k_ckpt_bal(DevState S, longlong2* out, unsigned long long* cnt) {
    for (uint32_t base = blockIdx.x * blockDim.x; base <= S.bal_mask; base += gridDim.x * blockDim.x) {
        const uint32_t h = base + threadIdx.x;
        const bool live = h <= S.bal_mask && S.bal_state[h] == 1u;
        const uint32_t k = wave_reserve(cnt, live);
        if (live) out[k] = make_longlong2(S.bal_key[h], S.bal_val[h]);
    }
}
__global__ void __launch_bounds__(256) k_ckpt_pos(DevState S, long4* out, unsigned long long* cnt) {
    for (uint32_t base = blockIdx.x * blockDim.x; base <= S.pos_mask; base += gridDim.x * blockDim.x) {
        const uint32_t h = base + threadIdx.x;
        const bool live = h <= S.pos_mask && S.pos[h].state == 1u;
        const uint32_t k = wave_reserve(cnt, live);
        if (live) out[k] = reinterpret_cast<const KG long4*>(&S.pos[h])[0];
    }
}
__global__ void __launch_bounds__(256) k_rst_bal(DevState S, const longlong2* in, uint32_t n, unsigned long long* fail) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    const bool bad = k < n && !bal_put_new(S, in[k].x, in[k].y);
    block_add(fail, bad ? 1u : 0u);
}
__global__ void __launch_bounds__(256) k_rst_pos(DevState S, const long4* in, uint32_t n, unsigned long long* fail) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    bool bad = false;
    if (k < n) { const long4 e = in[k]; bad = !pos_put_new(S, e.x, e.y, e.z, e.w); }
    block_add(fail, bad ? 1u : 0u);
}

// ---------------------------------------------------------------- launchers
static inline uint32_t mcdiv(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }
constexpr uint32_t MAINT_BLOCKS = 4096;

void launch_ledger_live(const DevState& S, unsigned long long* out2, hipStream_t st) {
    (void)hipMemsetAsync(out2, 0, 2 * sizeof(unsigned long long), st);
    hipLaunchKernelGGL(k_ledger_live, dim3(MAINT_BLOCKS), dim3(256), 0, st, S, out2);
}
void launch_ledger_rehash(const DevState& N, const DevState& O, unsigned long long* fail2, hipStream_t st) {
    (void)hipMemsetAsync(fail2, 0, 2 * sizeof(unsigned long long), st);
    if (N.bal_state != O.bal_state)
        hipLaunchKernelGGL(k_bal_rehash, dim3(std::min<uint32_t>(mcdiv((uint64_t)O.bal_mask + 1, 256), MAINT_BLOCKS)), dim3(256), 0,
                           st, N, O.bal_state, O.bal_key, O.bal_val, O.bal_mask + 1, fail2);
    if (N.pos != O.pos)
        hipLaunchKernelGGL(k_pos_rehash, dim3(std::min<uint32_t>(mcdiv((uint64_t)O.pos_mask + 1, 256), MAINT_BLOCKS)), dim3(256), 0,
                           st, N, O.pos, O.pos_mask + 1, fail2 + 1);
}
void launch_ckpt_levels(const DevState& S, Level* out, unsigned long long* cnt, hipStream_t st) {
    (void)hipMemsetAsync(cnt, 0, sizeof(unsigned long long), st);
    hipLaunchKernelGGL(k_ckpt_levels, dim3(mcdiv((uint64_t)(S.G + S.Gs) * 2 * NLEV, 256)), dim3(256), 0, st, S, out, cnt);
}
void launch_rst_levels(const DevState& S, const Level* in, uint32_t n, hipStream_t st) {
    if (n) hipLaunchKernelGGL(k_rst_levels, dim3(mcdiv(n, 256)), dim3(256), 0, st, S, in, n);
}
void launch_ckpt_ledger(const DevState& S, void* bal_out, void* pos_out, unsigned long long* cnt2, hipStream_t st) {
    (void)hipMemsetAsync(cnt2, 0, 2 * sizeof(unsigned long long), st);
    hipLaunchKernelGGL(k_ckpt_bal, dim3(std::min<uint32_t>(mcdiv((uint64_t)S.bal_mask + 1, 256), MAINT_BLOCKS)), dim3(256), 0, st, S,
                       (longlong2*)bal_out, cnt2);
    hipLaunchKernelGGL(k_ckpt_pos, dim3(std::min<uint32_t>(mcdiv((uint64_t)S.pos_mask + 1, 256), MAINT_BLOCKS)), dim3(256), 0, st, S,
                       (long4*)pos_out, cnt2 + 1);
}
void launch_rst_ledger(const DevState& S, const void* bal_in, uint32_t nb, const void* pos_in, uint32_t np,
                       unsigned long long* fail, hipStream_t st) {
    (void)hipMemsetAsync(fail, 0, sizeof(unsigned long long), st);
    if (nb) hipLaunchKernelGGL(k_rst_bal, dim3(mcdiv(nb, 256)), dim3(256), 0, st, S, (const longlong2*)bal_in, nb, fail);
    if (np) hipLaunchKernelGGL(k_rst_pos, dim3(mcdiv(np, 256)), dim3(256), 0, st, S, (const long4*)pos_in, np, fail);
}

}  // namespace kme
