// randbench2.hip -- random-access costs of the write and atomic shapes the epoch pipeline issues
// (DESIGN.md §5.2, §10): stores of 4 / 16 / 32 / 64 / 128 contiguous bytes into random lines,
// read-modify-write of 32 B, gathers of 16 / 32 / 64 / 128 B, returning 8-B CAS and no-return 8-B
// atomic adds, each over a table of a given size (the MALL is 256 MB; the oid table at C3 is 2 GB).
// One JSON line per case: operations per second and the bytes they name per second.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/randbench2 tools/randbench2.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::fprintf(stderr, "%s\n", hipGetErrorString(e_)); std::exit(1); } } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// every lane: `iters` random stores of BYTES contiguous bytes at a BYTES-aligned (>= 16) slot
template <int BYTES>
__global__ void k_store(int4* t, uint64_t nslots, int iters) {
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t s = tid * 0x9e3779b97f4a7c15ull + 7;
    for (int it = 0; it < iters; ++it) {
        s = mix(s);
        int4* p = t + (s % nslots) * (BYTES / 16);
#pragma unroll
        for (int q = 0; q < BYTES / 16; ++q) p[q] = make_int4(it, (int)tid, q, 2);
    }
}
__global__ void k_store4(int* t, uint64_t nlines, int iters) {   // one dword into a random 64-B line
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t s = tid * 0x9e3779b97f4a7c15ull + 11;
    for (int it = 0; it < iters; ++it) {
        s = mix(s);
        t[(s % nlines) * 16 + (s >> 60)] = it;
    }
}
// k independent random loads of BYTES each per round
template <int BYTES>
__global__ void k_load(const int4* __restrict__ t, uint64_t nslots, int iters, int4* sink) {
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t s = tid * 0x9e3779b97f4a7c15ull;
    int4 acc = make_int4(0, 0, 0, 0);
    for (int it = 0; it < iters; ++it) {
        int4 v[4][BYTES / 16];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            s = mix(s + j);
            const int4* p = t + (s % nslots) * (BYTES / 16);
#pragma unroll
            for (int q = 0; q < BYTES / 16; ++q) v[j][q] = p[q];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int q = 0; q < BYTES / 16; ++q) { acc.x ^= v[j][q].x; acc.y += v[j][q].y; acc.z ^= v[j][q].z; acc.w += v[j][q].w; }
    }
    if (acc.x == 0x12345678) sink[tid] = acc;
}
// read 32 B, store 32 B back (a level update)
__global__ void k_rmw32(int4* t, uint64_t nslots, int iters) {
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t s = tid * 0x9e3779b97f4a7c15ull + 3;
    for (int it = 0; it < iters; ++it) {
        s = mix(s);
        int4* p = t + (s % nslots) * 2;
        int4 a = p[0], b = p[1];
        a.x += 1; b.y ^= it;
        p[0] = a; p[1] = b;
    }
}
__global__ void k_cas(unsigned long long* t, uint64_t nwords, int iters, unsigned long long* sink) {
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t s = tid * 0x9e3779b97f4a7c15ull + 13;
    unsigned long long acc = 0;
    for (int it = 0; it < iters; ++it) {
        s = mix(s);
        acc += atomicCAS(&t[s % nwords], 0ull, s | 1);
    }
    if (acc == 0x12345678) sink[tid] = acc;
}
__global__ void k_add(unsigned long long* t, uint64_t nwords, int iters) {
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t s = tid * 0x9e3779b97f4a7c15ull + 17;
    for (int it = 0; it < iters; ++it) {
        s = mix(s);
        atomicAdd(&t[s % nwords], 1ull);
    }
}

int main() {
    const size_t max_bytes = (size_t)2 << 30;
    void* buf;
    CK(hipMalloc(&buf, max_bytes));
    CK(hipMemset(buf, 0, max_bytes));
    void* sink;
    CK(hipMalloc(&sink, (size_t)1 << 26));
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
    const size_t tables[] = {(size_t)512 << 10, (size_t)64 << 20, (size_t)256 << 20, (size_t)2 << 30};
    const int blocks = 256 * 16 / 4;   // 16 waves per CU
    const int iters = 32;
    const double ops = (double)blocks * 256 * iters;
    auto line = [&](const char* c, size_t T, double n, double bytes_per_op, float ms) {
        std::printf("{\"case\":\"%s\",\"table_mb\":%.1f,\"G_per_s\":%.2f,\"GB_s\":%.0f}\n", c, T / 1048576.0, n / ms / 1e6,
                    n * bytes_per_op / ms / 1e6);
    };
    for (size_t T : tables) {
        float ms;
        ms = timeit([&] { hipLaunchKernelGGL(k_store4, dim3(blocks), dim3(256), 0, 0, (int*)buf, T / 64, iters); });
        line("store4", T, ops, 4, ms);
        ms = timeit([&] { hipLaunchKernelGGL(k_store<16>, dim3(blocks), dim3(256), 0, 0, (int4*)buf, T / 16, iters); });
        line("store16", T, ops, 16, ms);
        ms = timeit([&] { hipLaunchKernelGGL(k_store<32>, dim3(blocks), dim3(256), 0, 0, (int4*)buf, T / 32, iters); });
        line("store32", T, ops, 32, ms);
        ms = timeit([&] { hipLaunchKernelGGL(k_store<64>, dim3(blocks), dim3(256), 0, 0, (int4*)buf, T / 64, iters); });
        line("store64", T, ops, 64, ms);
        ms = timeit([&] { hipLaunchKernelGGL(k_store<128>, dim3(blocks), dim3(256), 0, 0, (int4*)buf, T / 128, iters); });
        line("store128", T, ops, 128, ms);
        ms = timeit([&] { hipLaunchKernelGGL(k_load<16>, dim3(blocks), dim3(256), 0, 0, (const int4*)buf, T / 16, iters, (int4*)sink); });
        line("load16", T, ops * 4, 16, ms);
        ms = timeit([&] { hipLaunchKernelGGL(k_load<32>, dim3(blocks), dim3(256), 0, 0, (const int4*)buf, T / 32, iters, (int4*)sink); });
        line("load32", T, ops * 4, 32, ms);
        ms = timeit([&] { hipLaunchKernelGGL(k_load<64>, dim3(blocks), dim3(256), 0, 0, (const int4*)buf, T / 64, iters, (int4*)sink); });
        line("load64", T, ops * 4, 64, ms);
        ms = timeit([&] { hipLaunchKernelGGL(k_rmw32, dim3(blocks), dim3(256), 0, 0, (int4*)buf, T / 32, iters); });
        line("rmw32", T, ops, 64, ms);
        CK(hipMemset(buf, 0, T));
        ms = timeit([&] { hipLaunchKernelGGL(k_cas, dim3(blocks), dim3(256), 0, 0, (unsigned long long*)buf, T / 8, iters, (unsigned long long*)sink); });
        line("cas8", T, ops, 8, ms);
        ms = timeit([&] { hipLaunchKernelGGL(k_add, dim3(blocks), dim3(256), 0, 0, (unsigned long long*)buf, T / 8, iters); });
        line("add8_noret", T, ops, 8, ms);
        std::fflush(stdout);
    }
    return 0;
}
