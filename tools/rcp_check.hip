// Exhaustive check of a short reciprocal tried for the device Moller-Trumbore
// test and normalize (round 6: bit-exact, but no faster -- the IEEE division
// stays; profiles/r06_experiments/rcp_rn.log): for every float x with 2^-24 <= |x| <
// 2^124, r = fma(fma(-x, r0, 1), r0, r0) with r0 = v_rcp_f32(x) against the
// correctly rounded 1.0f / x (the compiler's IEEE division sequence).
// Prints the mismatch count and the first few mismatching inputs.
//   hipcc --offload-arch=gfx950 -O2 -o tools/_bin/rcp_check tools/rcp_check.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

__global__ void k_check(uint32_t per, uint32_t* __restrict__ bad, uint32_t* __restrict__ first)
{
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t lo = tid * per;
    uint32_t n = 0, f = 0xFFFFFFFFu;
    for (uint32_t i = 0; i < per; ++i) {
        const uint32_t bits = (uint32_t)(lo + i);
        const uint32_t e = (bits >> 23) & 255u;
        if (e < 127u - 24u || e >= 127u + 124u) continue;  // 2^-24 <= |x| < 2^124
        const float x = __uint_as_float(bits);
        const float exact = 1.0f / x;
        const float r0 = __builtin_amdgcn_rcpf(x);
        const float r = __builtin_fmaf(__builtin_fmaf(-x, r0, 1.0f), r0, r0);
        if (__float_as_uint(r) != __float_as_uint(exact)) {
            ++n;
            if (f == 0xFFFFFFFFu) f = bits;
        }
    }
    bad[tid] = n;
    first[tid] = f;
}

int main()
{
    const uint32_t threads = 1u << 20, per = (uint32_t)((1ull << 32) / threads);
    uint32_t *bad = nullptr, *first = nullptr;
    if (hipMalloc(&bad, threads * 4) != hipSuccess || hipMalloc(&first, threads * 4) != hipSuccess) return 2;
    k_check<<<threads / 256, 256>>>(per, bad, first);
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    std::vector<uint32_t> b(threads), f(threads);
    (void)hipMemcpy(b.data(), bad, threads * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(f.data(), first, threads * 4, hipMemcpyDeviceToHost);
    uint64_t tot = 0;
    int shown = 0;
    for (uint32_t t = 0; t < threads; ++t) {
        tot += b[t];
        if (b[t] && shown < 8) {
            printf("mismatch at x = %a (0x%08x)\n", (double)__builtin_bit_cast(float, f[t]), f[t]);
            ++shown;
        }
    }
    printf("rcp_rn check: %llu mismatches over 2^-24 <= |x| < 2^124\n", (unsigned long long)tot);
    return tot ? 1 : 0;
}
