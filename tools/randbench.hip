// randbench.hip -- random-access ceilings of one MI355X for the access shapes the matching
// pipeline uses: independent random 32-B / 64-B gathers, dependent chains
// (pointer chasing: one outstanding load per lane), random 32-B stores, 4-B partial stores into
// random lines and 8-B CAS, over tables of 0.25-4 GiB.  Prints one JSON line per case.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/randbench tools/randbench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::fprintf(stderr, "%s\n", hipGetErrorString(e_)); std::exit(1); } } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// every lane: `iters` rounds of `k` independent random loads of `bytes` (16, 32 or 64)
template <int BYTES>
__global__ void k_gather(const int4* __restrict__ t, uint64_t nlines, int iters, int k, int4* sink) {
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    int4 acc = make_int4(0, 0, 0, 0);
    uint64_t s = tid * 0x9e3779b97f4a7c15ull;
    for (int it = 0; it < iters; ++it) {
        int4 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (j < k) {
                s = mix(s + j);
                const int4* p = t + (s % nlines) * (BYTES / 16);
                v[j] = p[0];
                if (BYTES >= 32) { int4 w = p[1]; v[j].x ^= w.x; v[j].y ^= w.y; }
                if (BYTES >= 64) { int4 w = p[2], u = p[3]; v[j].z ^= w.z ^ u.x; v[j].w ^= w.w ^ u.y; }
            }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) if (j < k) { acc.x ^= v[j].x; acc.y += v[j].y; acc.z ^= v[j].z; acc.w += v[j].w; }
    }
    if (acc.x == 0x12345678) sink[tid] = acc;
}

// dependent chain: the next address comes from the loaded value
__global__ void k_chase(const uint64_t* __restrict__ t, uint64_t nwords, int iters, uint64_t* sink) {
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t x = mix(tid) % nwords;
    for (int it = 0; it < iters; ++it) x = t[x] % nwords;
    if (x == 0x12345678) sink[tid] = x;
}

__global__ void k_fill_chase(uint64_t* t, uint64_t nwords) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nwords; i += gridDim.x * (uint64_t)blockDim.x)
        t[i] = mix(i ^ 0xabcdefull) % nwords * 16 % nwords;   // stride 16 words: one line per hop
}

template <int BYTES>
__global__ void k_scatter(int4* t, uint64_t nlines, int iters) {
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t s = tid * 0x9e3779b97f4a7c15ull + 7;
    for (int it = 0; it < iters; ++it) {
        s = mix(s);
        int4* p = t + (s % nlines) * (BYTES / 16);
        p[0] = make_int4(it, (int)tid, 1, 2);
        if (BYTES >= 32) p[1] = make_int4(3, 4, 5, 6);
    }
}

__global__ void k_partial(int* t, uint64_t nlines, int iters) {   // one dword into a random 128-B line
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t s = tid * 0x9e3779b97f4a7c15ull + 11;
    for (int it = 0; it < iters; ++it) {
        s = mix(s);
        t[(s % nlines) * 32 + (s >> 60)] = it;
    }
}

__global__ void k_cas(unsigned long long* t, uint64_t nwords, int iters) {
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t s = tid * 0x9e3779b97f4a7c15ull + 13;
    for (int it = 0; it < iters; ++it) {
        s = mix(s);
        atomicCAS(&t[s % nwords], 0ull, s | 1);
    }
}

int main(int argc, char** argv) {
    const size_t max_bytes = (size_t)4 << 30;
    void* buf;
    CK(hipMalloc(&buf, max_bytes));
    CK(hipMemset(buf, 0, max_bytes));
    void* sink;
    CK(hipMalloc(&sink, (size_t)1 << 28));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    auto timeit = [&](auto launch) {
        launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a));
        launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0; CK(hipEventElapsedTime(&ms, a, b));
        return ms;
    };
    const size_t tables[] = {(size_t)256 << 20, (size_t)1 << 30, (size_t)4 << 30};
    for (size_t T : tables) {
        const uint64_t n16 = T / 16;
        for (int waves_per_cu : {4, 8, 16, 32}) {
            const int blocks = 256 * waves_per_cu / 4;   // 256-thread blocks
            for (int k : {1, 4}) {
                const int iters = 64;
                const double acc = (double)blocks * 256 * iters * k;
                float ms;
                ms = timeit([&] { hipLaunchKernelGGL(k_gather<32>, dim3(blocks), dim3(256), 0, 0, (const int4*)buf, n16 / 2, iters, k, (int4*)sink); });
                std::printf("{\"case\":\"gather32\",\"table_mb\":%zu,\"waves_per_cu\":%d,\"indep\":%d,\"G_per_s\":%.2f,\"GB_s\":%.0f}\n", T >> 20, waves_per_cu, k, acc / ms / 1e6, acc * 32 / ms / 1e6);
                ms = timeit([&] { hipLaunchKernelGGL(k_gather<64>, dim3(blocks), dim3(256), 0, 0, (const int4*)buf, n16 / 4, iters, k, (int4*)sink); });
                std::printf("{\"case\":\"gather64\",\"table_mb\":%zu,\"waves_per_cu\":%d,\"indep\":%d,\"G_per_s\":%.2f,\"GB_s\":%.0f}\n", T >> 20, waves_per_cu, k, acc / ms / 1e6, acc * 64 / ms / 1e6);
            }
            {
                const int iters = 64;
                const double acc = (double)blocks * 256 * iters;
                hipLaunchKernelGGL(k_fill_chase, dim3(4096), dim3(256), 0, 0, (uint64_t*)buf, T / 8);
                CK(hipDeviceSynchronize());
                float ms = timeit([&] { hipLaunchKernelGGL(k_chase, dim3(blocks), dim3(256), 0, 0, (const uint64_t*)buf, T / 8, iters, (uint64_t*)sink); });
                std::printf("{\"case\":\"chase\",\"table_mb\":%zu,\"waves_per_cu\":%d,\"G_per_s\":%.2f,\"ns_per_hop\":%.0f}\n", T >> 20, waves_per_cu, acc / ms / 1e6, ms * 1e6 / iters);
                ms = timeit([&] { hipLaunchKernelGGL(k_scatter<32>, dim3(blocks), dim3(256), 0, 0, (int4*)buf, n16 / 2, iters); });
                std::printf("{\"case\":\"store32\",\"table_mb\":%zu,\"waves_per_cu\":%d,\"G_per_s\":%.2f}\n", T >> 20, waves_per_cu, acc / ms / 1e6);
                ms = timeit([&] { hipLaunchKernelGGL(k_partial, dim3(blocks), dim3(256), 0, 0, (int*)buf, T / 128, iters); });
                std::printf("{\"case\":\"store4_partial\",\"table_mb\":%zu,\"waves_per_cu\":%d,\"G_per_s\":%.2f}\n", T >> 20, waves_per_cu, acc / ms / 1e6);
                CK(hipMemset(buf, 0, T));
                ms = timeit([&] { hipLaunchKernelGGL(k_cas, dim3(blocks), dim3(256), 0, 0, (unsigned long long*)buf, T / 8, iters); });
                std::printf("{\"case\":\"cas8\",\"table_mb\":%zu,\"waves_per_cu\":%d,\"G_per_s\":%.2f}\n", T >> 20, waves_per_cu, acc / ms / 1e6);
            }
            std::fflush(stdout);
        }
    }
    return 0;
}
