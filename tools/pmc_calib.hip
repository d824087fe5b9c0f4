// pmc_calib.hip -- calibration of rocprofv3's memory counters on gfx950 for
// the access shapes k_path has (VERDICT r02 "re-validate the FETCH x2
// correction for 16-B gathers with a microbenchmark whose byte count is known").
//
// Every kernel reads a table whose byte traffic is known by construction and
// writes one word per wave (negligible):
//   k_stream<0>        coalesced 16 B/lane sweep of a 1 GiB table (the guide's
//                      calibrated case: FETCH_SIZE = 1/2 of the bytes)
//   k_gather<16, big>  one random 16-B item per lane from a 2 GiB table, 4 Mi
//                      loads over 16 Mi lines: ~one distinct 128-B line per load
//   k_gather<64, big>  4 lanes read one random 64-B segment
//   k_gather<128, big> 8 lanes read one random 128-B line
//   k_gather<16, small> the same 16-B gathers from a 7 MiB table (the size of
//                      the scene's nodes + triangles: L2 / Infinity-Cache resident)
//   k_scatter<16>      one random 16-B nontemporal store per lane into 2 GiB
//                      (the per-sample colour buffer's access shape)
// The host prints one JSON line with the known byte and line counts per
// kernel, to be divided into the per-dispatch counter values.
//   hipcc --offload-arch=gfx950 -O2 tools/pmc_calib.hip -o tools/_bin/pmc_calib
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
            return 1;                                                             \
        }                                                                         \
    } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t x)
{
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

template <int K>
__global__ void __launch_bounds__(256) k_stream(const uint4* __restrict__ a, uint64_t n, uint32_t* __restrict__ sink)
{
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint4 v = a[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    for (int o = 32; o > 0; o >>= 1) acc ^= (uint32_t)__shfl_xor((int)acc, o);
    if ((threadIdx.x & 63) == 0) sink[(blockIdx.x * 256 + threadIdx.x) >> 6] = acc;
}

// SEG bytes per group of SEG/16 lanes; groups pick random SEG-aligned segments
template <int SEG, int BIG>
__global__ void __launch_bounds__(256) k_gather(const uint4* __restrict__ a, uint64_t nseg, uint64_t loads,
                                                uint32_t seed, uint32_t* __restrict__ sink)
{
    constexpr int G = SEG / 16;  // lanes per segment
    uint32_t acc = 0;
    const uint64_t lanes = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < loads; i += lanes) {
        const uint64_t grp = i / G;
        const uint64_t s = (((uint64_t)hash32((uint32_t)grp ^ seed) << 32) | hash32((uint32_t)(grp >> 32) + 0x9e3779b9u * (uint32_t)grp)) % nseg;
        const uint4 v = a[s * G + (i % G)];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    for (int o = 32; o > 0; o >>= 1) acc ^= (uint32_t)__shfl_xor((int)acc, o);
    if ((threadIdx.x & 63) == 0) sink[(blockIdx.x * 256 + threadIdx.x) >> 6] = acc;
}

template <int K>
__global__ void __launch_bounds__(256) k_scatter(uint4* __restrict__ a, uint64_t nitems, uint64_t stores, uint32_t seed)
{
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    const uint64_t lanes = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < stores; i += lanes) {
        const uint64_t s = (((uint64_t)hash32((uint32_t)i ^ seed) << 32) | hash32((uint32_t)(i >> 32) + 0x85ebca6bu * (uint32_t)i)) % nitems;
        __builtin_nontemporal_store((u4){(uint32_t)i, 1u, 2u, 3u}, reinterpret_cast<u4*>(a + s));
    }
}

int main()
{
    const uint64_t big = 2ull << 30, small = 7ull << 20, stream = 1ull << 30;
    uint4 *A = nullptr, *S = nullptr;
    uint32_t* sink = nullptr;
    CHECK(hipMalloc(&A, big));
    CHECK(hipMalloc(&S, small));
    CHECK(hipMalloc(&sink, 1 << 24));
    CHECK(hipMemset(A, 1, big));
    CHECK(hipMemset(S, 2, small));
    const int grid = 256 * 8;
    const uint64_t loads = 4ull << 20;         // 4 Mi lane-loads per big-table kernel: lines ~distinct
    const uint64_t loads_small = 64ull << 20;  // 64 Mi lane-loads from the resident 7 MiB table
    for (int rep = 0; rep < 3; ++rep) {
        k_stream<0><<<grid, 256>>>(A, stream / 16, sink);
        k_gather<16, 1><<<grid, 256>>>(A, big / 16, loads, 11u + rep, sink);
        k_gather<64, 1><<<grid, 256>>>(A, big / 64, loads, 13u + rep, sink);
        k_gather<128, 1><<<grid, 256>>>(A, big / 128, loads, 17u + rep, sink);
        k_gather<16, 0><<<grid, 256>>>(S, small / 16, loads_small, 19u + rep, sink);
        k_scatter<16><<<grid, 256>>>(A, big / 16, loads, 23u + rep);
        CHECK(hipGetLastError());
        CHECK(hipDeviceSynchronize());
    }
    // known traffic per dispatch: requested bytes; 128-B lines touched (the
    // random gathers from the 2 GiB table touch ~one distinct line per group)
    printf("{\"stream\": {\"bytes\": %llu, \"lines128\": %llu},"
           " \"gather16_big\": {\"bytes\": %llu, \"lines128\": %llu},"
           " \"gather64_big\": {\"bytes\": %llu, \"lines128\": %llu},"
           " \"gather128_big\": {\"bytes\": %llu, \"lines128\": %llu},"
           " \"gather16_small\": {\"bytes\": %llu, \"table_bytes\": %llu},"
           " \"scatter16_nt\": {\"bytes\": %llu, \"stores\": %llu}}\n",
           (unsigned long long)stream, (unsigned long long)(stream / 128),
           (unsigned long long)(loads * 16), (unsigned long long)loads,
           (unsigned long long)(loads * 16), (unsigned long long)(loads / 4),
           (unsigned long long)(loads * 16), (unsigned long long)(loads / 8),
           (unsigned long long)(loads_small * 16), (unsigned long long)small,
           (unsigned long long)(loads * 16), (unsigned long long)loads);
    CHECK(hipFree(A));
    CHECK(hipFree(S));
    CHECK(hipFree(sink));
    return 0;
}
